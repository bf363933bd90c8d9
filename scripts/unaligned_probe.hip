// Probe for byte-granular cells on the nibble kernel (odd lengths): 16-B raw buffer loads and stores at
// byte offsets that are not multiples of 4 on gfx950 (hipcc itself emits global_load_dwordx4 for align-1 16-B
// accesses on this target, i.e. the amdhsa ABI runs the shader in unaligned access mode), and what a 16-B load
// returns when it crosses the end of its descriptor's range.
//   hipcc --offload-arch=gfx950 -O3 scripts/unaligned_probe.hip -o scripts/unaligned_probe && scripts/unaligned_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                           \
    }                                                                         \
  } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, static_cast<int>(n), 0x00020000);
}

// every thread moves 16 B from src + 16 i + ls to dst + 16 i + ss, grid-stride over `blocks` blocks
__global__ void shift_copy(const uint8_t *src, uint8_t *dst, uint32_t n, int64_t blocks, int ls, int ss) {
  const auto rs = rsrc(src, n), rd = rsrc(dst, n);
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < blocks; i += int64_t(gridDim.x) * blockDim.x) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(i * 16), ls, 2);
    __builtin_amdgcn_raw_buffer_store_b128(v, rd, static_cast<int>(i * 16), ss, 2);
  }
}

// lane l loads 16 B at byte offset base + l from a descriptor of `n` records, writes them to out[16 l ..]
__global__ void edge_load(const uint8_t *src, uint32_t n, int base, uint8_t *out) {
  const auto rs = rsrc(src, n);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(base + threadIdx.x), 0, 2);
  std::memcpy(out + 16 * threadIdx.x, &v, 16);
}

int main() {
  const uint32_t n = 1u << 30;  // 1 GiB per buffer
  uint8_t *src, *dst, *eo;
  CK(hipMalloc(&src, n));
  CK(hipMalloc(&dst, n));
  CK(hipMalloc(&eo, 64 * 16));
  std::vector<uint8_t> h(n), g(n);
  uint64_t x = 0x9e3779b97f4a7c15ull;
  for (uint32_t i = 0; i < n; i += 8) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    std::memcpy(&h[i], &x, 8);
  }
  CK(hipMemcpy(src, h.data(), n, hipMemcpyHostToDevice));
  const int64_t blocks = (n - 32) / 16;
  const int grid = 256 * 8 * 4;
  const int shifts[][2] = {{0, 0}, {1, 0}, {3, 0}, {4, 0}, {7, 0}, {13, 0}, {0, 1}, {0, 7}, {5, 9}, {15, 15}};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  bool all_ok = true;
  for (auto &sh : shifts) {
    const int ls = sh[0], ss = sh[1];
    CK(hipMemset(dst, 0, n));
    hipLaunchKernelGGL(shift_copy, dim3(grid), dim3(256), 0, 0, src, dst, n, blocks, ls, ss);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(g.data(), dst, n, hipMemcpyDeviceToHost));
    const bool ok = std::memcmp(g.data() + ss, h.data() + ls, blocks * 16) == 0;
    all_ok = all_ok && ok;
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(shift_copy, dim3(grid), dim3(256), 0, 0, src, dst, n, blocks, ls, ss);
    const int it = 20;
    CK(hipEventRecord(a));
    for (int r = 0; r < it; ++r)
      hipLaunchKernelGGL(shift_copy, dim3(grid), dim3(256), 0, 0, src, dst, n, blocks, ls, ss);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= it;
    std::printf("{\"probe\": \"shift_copy\", \"load_shift\": %d, \"store_shift\": %d, \"bytes_ok\": %s, \"ms\": %.4f, "
                "\"GBps_read_plus_write\": %.1f}\n",
                ls, ss, ok ? "true" : "false", ms, 2.0 * blocks * 16 / ms / 1e6);
  }
  // a 16-B load that crosses the end of the range: descriptor of 100 records, loads at 80 .. 143
  std::vector<uint8_t> eh(64 * 16);
  hipLaunchKernelGGL(edge_load, dim3(1), dim3(64), 0, 0, src, 100u, 80, eo);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(eh.data(), eo, eh.size(), hipMemcpyDeviceToHost));
  for (int l = 0; l < 24; ++l) {
    const int off = 80 + l;
    int real = 0, zero = 0, other = 0;
    std::printf("{\"probe\": \"edge\", \"records\": 100, \"offset\": %d, \"bytes\": \"", off);
    for (int i = 0; i < 16; ++i) {
      const uint8_t v = eh[16 * l + i], want = h[off + i];
      const bool in = off + i < 100;
      std::printf("%c", v == want && (in || v != 0) ? 'R' : v == 0 ? '0' : '?');
      if (v == want && (in || want != 0)) ++real; else if (v == 0) ++zero; else ++other;
    }
    std::printf("\", \"real\": %d, \"zero\": %d, \"other\": %d}\n", real, zero, other);
  }
  std::printf("{\"probe\": \"done\", \"all_bytes_ok\": %s}\n", all_ok ? "true" : "false");
  return all_ok ? 0 : 1;
}
