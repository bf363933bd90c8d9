// Probe: how fast can the memory system serve the coding kernels' access pattern with no arithmetic in the way?
// K input units and R output units per stripe, one 16-B vector per lane per unit per workgroup (4 KiB chunks, the
// gf_code_vec geometry), output r = XOR of the inputs (rotated by r): the C2 layout (rs-6-3, parity in place in the
// 9-unit stripe) and the C3 layout (rs-10-4 decode: 10 of 14 units read, 4 written to a separate buffer), with
// several block->chunk orders.  Prints one JSON line per case: fraction of 8 TB/s over the algorithmic bytes.
// With argument "r": read-only streaming over 24 GiB in contiguous chunks per workgroup (the CRC kernels' pattern).
//   hipcc --offload-arch=gfx950 -O3 scripts/stream_probe.hip -o scripts/stream_probe && scripts/stream_probe [r]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      std::exit(2);                                                                      \
    }                                                                                    \
  } while (0)

constexpr int kMaxK = 10, kMaxR = 4;
struct Layout {
  const uint8_t *in;
  uint8_t *out;
  int64_t in_ss, out_ss;  // stripe strides
  int in_off[kMaxK], out_off[kMaxR];
  uint32_t in_ext, out_ext;
  uint32_t len, nstripes;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, static_cast<int>(n), 0x00020000);
}

// ORDER 0: chunk-major within a stripe (u = s * cpc + c), XCD-contiguous block order (the product's mapping)
// ORDER 1: the same without the XCD remap
// ORDER 2: stripe-major (u = c * S + s): neighbouring blocks take the same chunk of neighbouring stripes
template <int K, int R, int ORDER, int T = 256>
__global__ __launch_bounds__(T) void stream(const Layout L) {
  const uint32_t cpc = L.len / (T * 16), units = L.nstripes * cpc;
  uint32_t b = blockIdx.x;
  if (ORDER == 0) {
    const uint32_t q = gridDim.x >> 3;
    b = b < (q << 3) ? (b & 7) * q + (b >> 3) : b;
  }
  if (b >= units) return;
  uint32_t s, c;
  if (ORDER == 2) {
    c = b / L.nstripes;
    s = b - c * L.nstripes;
  } else {
    s = b / cpc;
    c = b - s * cpc;
  }
  const auto ri = rsrc(L.in + s * L.in_ss, L.in_ext);
  const auto ro = rsrc(L.out + s * L.out_ss, L.out_ext);
  const uint32_t v = (c * T + threadIdx.x) * 16;
  uint32_t x[K][4];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const auto d = __builtin_amdgcn_raw_buffer_load_b128(ri, v, L.in_off[j], 2);
    x[j][0] = d[0], x[j][1] = d[1], x[j][2] = d[2], x[j][3] = d[3];
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    __attribute__((ext_vector_type(4))) unsigned int o = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int w = 0; w < 4; ++w) o[w] ^= x[(j + r) % K][w];
    __builtin_amdgcn_raw_buffer_store_b128(o, ro, v, L.out_off[r], 2);
  }
}

// read-only streaming (the CRC kernels' side of the memory system): each workgroup reads CH contiguous bytes, U
// 16-B loads per lane in flight, XOR-reduces them and stores nothing (a never-true compare keeps the loads live)
template <int CH, int U>
__global__ __launch_bounds__(256) void read_only(const uint8_t *p, uint64_t n, uint32_t magic, uint32_t *sink) {
  const uint32_t q = gridDim.x >> 3;
  const uint32_t b = blockIdx.x < (q << 3) ? (blockIdx.x & 7) * q + (blockIdx.x >> 3) : blockIdx.x;
  const auto r = rsrc(p + uint64_t(b) * CH, CH);
  uint32_t acc = 0;
  for (int i = 0; i < CH / (256 * 16); i += U) {
    __attribute__((ext_vector_type(4))) unsigned int d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) d[u] = __builtin_amdgcn_raw_buffer_load_b128(r, ((i + u) * 256 + threadIdx.x) * 16, 0, 2);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
  }
  if (acc == magic) sink[threadIdx.x] = acc;
}

template <int CH, int U>
void run_read(const uint8_t *p, uint64_t n, uint32_t *sink) {
  const uint32_t grid = static_cast<uint32_t>(n / CH);
  auto launch = [&]() { hipLaunchKernelGGL((read_only<CH, U>), dim3(grid), dim3(256), 0, 0, p, n, 0x9e3779b9u, sink); };
  for (int i = 0; i < 3; ++i) launch();
  CK(hipGetLastError());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int it = 10;
  CK(hipEventRecord(a));
  for (int i = 0; i < it; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= it;
  const double bytes = double(grid) * CH;
  std::printf("{\"case\": \"read only\", \"chunk\": %d, \"loads_in_flight\": %d, \"ms\": %.3f, \"TB/s\": %.3f, "
              "\"frac_of_8TBps\": %.4f}\n", CH, U, ms, bytes / ms / 1e9, bytes / ms / 1e9 / 8.0);
  std::fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

template <int K, int R, int T = 256>
void run(const char *name, Layout L, int order) {
  const uint32_t units = L.nstripes * (L.len / (T * 16));
  auto launch = [&]() {
    if (order == 0) hipLaunchKernelGGL((stream<K, R, 0, T>), dim3(units), dim3(T), 0, 0, L);
    if (order == 1) hipLaunchKernelGGL((stream<K, R, 1, T>), dim3(units), dim3(T), 0, 0, L);
    if (order == 2) hipLaunchKernelGGL((stream<K, R, 2, T>), dim3(units), dim3(T), 0, 0, L);
  };
  for (int i = 0; i < 3; ++i) launch();
  CK(hipGetLastError());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int it = 10;
  CK(hipEventRecord(a));
  for (int i = 0; i < it; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= it;
  const double bytes = double(K + R) * L.len * L.nstripes;
  std::printf("{\"case\": \"%s\", \"threads\": %d, \"order\": %d, \"k\": %d, \"r\": %d, \"stripes\": %u, \"ms\": %.3f, \"TB/s\": %.3f, "
              "\"frac_of_8TBps\": %.4f}\n",
              name, T, order, K, R, L.nstripes, ms, bytes / ms / 1e9, bytes / ms / 1e9 / 8.0);
  std::fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main(int argc, char **argv) {
  const uint32_t len = 1u << 20;
  if (argc > 1 && argv[1][0] == 'r') {  // read-only cases: a 24 GiB buffer, the CRC leg's volume
    const uint64_t n = uint64_t(24) << 30;
    uint8_t *p;
    uint32_t *sink;
    CK(hipMalloc(&p, n));
    CK(hipMalloc(&sink, 1024));
    CK(hipMemset(p, 1, n));
    run_read<16384, 4>(p, n, sink);
    run_read<65536, 4>(p, n, sink);
    run_read<65536, 8>(p, n, sink);
    run_read<262144, 4>(p, n, sink);
    run_read<262144, 8>(p, n, sink);
    run_read<262144, 16>(p, n, sink);
    CK(hipFree(p));
    CK(hipFree(sink));
    return 0;
  }
  // C2 layout: 2048 stripes of 9 units, parity written in place
  {
    const uint32_t S = 2048;
    uint8_t *buf;
    CK(hipMalloc(&buf, size_t(S) * 9 * len));
    CK(hipMemset(buf, 1, size_t(S) * 9 * len));
    Layout L{};
    L.in = buf, L.out = buf, L.in_ss = L.out_ss = int64_t(9) * len, L.len = len, L.nstripes = S;
    for (int j = 0; j < 6; ++j) L.in_off[j] = j * len;
    for (int r = 0; r < 3; ++r) L.out_off[r] = (6 + r) * len;
    L.in_ext = L.out_ext = 9 * len;
    for (int o = 0; o < 3; ++o) run<6, 3>("c2 layout rs-6-3 in place", L, o);
    for (int o = 0; o < 2; ++o) run<6, 3, 128>("c2 layout rs-6-3 in place", L, o);
    for (int o = 0; o < 2; ++o) run<6, 3, 512>("c2 layout rs-6-3 in place", L, o);
    CK(hipFree(buf));
  }
  // C3 layout: 1024 stripes of 14 units, units {0,2,3,5,6,7,8,9,11,12} read, 4 outputs in their own buffer
  {
    const uint32_t S = 1024;
    uint8_t *in, *out;
    CK(hipMalloc(&in, size_t(S) * 14 * len));
    CK(hipMalloc(&out, size_t(S) * 4 * len));
    CK(hipMemset(in, 1, size_t(S) * 14 * len));
    Layout L{};
    L.in = in, L.out = out, L.in_ss = int64_t(14) * len, L.out_ss = int64_t(4) * len, L.len = len, L.nstripes = S;
    const int rd[10] = {0, 2, 3, 5, 6, 7, 8, 9, 11, 12};
    for (int j = 0; j < 10; ++j) L.in_off[j] = rd[j] * len;
    for (int r = 0; r < 4; ++r) L.out_off[r] = r * len;
    L.in_ext = 14 * len, L.out_ext = 4 * len;
    for (int o = 0; o < 3; ++o) run<10, 4>("c3 layout rs-10-4 decode", L, o);
    for (int o = 0; o < 2; ++o) run<10, 4, 128>("c3 layout rs-10-4 decode", L, o);
    for (int o = 0; o < 2; ++o) run<10, 4, 512>("c3 layout rs-10-4 decode", L, o);
    for (int o = 0; o < 2; ++o) run<10, 4, 1024>("c3 layout rs-10-4 decode", L, o);
    // the same byte volume as 6 in / 3 out on the C3 buffers (is it the unit count or the layout?)
    for (int o = 0; o < 1; ++o) run<6, 3>("c3 buffers, 6 in 3 out", L, o);
    CK(hipFree(in));
    CK(hipFree(out));
  }
  return 0;
}
