// VALU issue-rate microbenchmark for the integer ops the GF/CRC kernels use (gfx950).
// Per op: W waves per SIMD each run ITERS x 8 independent chains of the op; a wave times its loop with
// the core-clock counter (clock64) and the result is cycles per instruction per SIMD = cycles / (n_instr * W).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/valu_rate.hip -o scripts/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHAINS(OPSTR, ...)                                                                \
  _Pragma("unroll") for (int c = 0; c < 8; ++c) asm volatile(OPSTR : "+v"(a[c]) : __VA_ARGS__);

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, long long *cyc, int iters) {
  uint32_t a[8];
  uint32_t b = threadIdx.x * 0x9e3779b9u + 7u, d = b ^ 0x5a5a5a5au;
  float f[8];
  float fb = 1.0001f * (float)(threadIdx.x & 7);
  for (int c = 0; c < 8; ++c) { a[c] = b + c * 0x01010101u; f[c] = (float)c; }
  long long t0 = clock64();
  long long r0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
    if constexpr (OP == 0) { CHAINS("v_xor_b32 %0, %0, %1", "v"(b)) }
    if constexpr (OP == 1) { CHAINS("v_xor_b32_e64 %0, %0, %1", "v"(b)) }
    if constexpr (OP == 2) { CHAINS("v_perm_b32 %0, %0, %1, %2", "v"(b), "v"(d)) }
    if constexpr (OP == 3) { CHAINS("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v"(b), "v"(d)) }
    if constexpr (OP == 4) { CHAINS("v_xor_b32_e64 %0, %1, %0", "s"(0x1234567u)) }
    if constexpr (OP == 5) { CHAINS("v_and_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD", "v"(b)) }
    if constexpr (OP == 6) { CHAINS("v_lshrrev_b32 %0, 3, %0", "v"(b)) }
    if constexpr (OP == 7) { CHAINS("v_alignbit_b32 %0, %0, %1, 7", "v"(b)) }
    if constexpr (OP == 8) { CHAINS("v_bfi_b32 %0, %0, %1, %2", "v"(b), "v"(d)) }
    if constexpr (OP == 9) { CHAINS("v_add_u32 %0, %0, %1", "v"(b)) }
    if constexpr (OP == 10) {
#pragma unroll
      for (int c = 0; c < 8; ++c) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"(fb));
    }
    if constexpr (OP == 11) {
#pragma unroll
      for (int c = 0; c < 8; ++c) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[c]) : "v"(fb));
    }
    if constexpr (OP == 12) { CHAINS("v_and_b32 %0, %0, %1", "v"(b)) }
    if constexpr (OP == 13) { CHAINS("v_lshl_or_b32 %0, %0, 3, %1", "v"(b)) }
    if constexpr (OP == 14) { CHAINS("v_and_or_b32 %0, %0, %1, %2", "v"(b), "v"(d)) }
    if constexpr (OP == 15) { CHAINS("v_perm_b32 %0, %1, %0, %2", "s"(0x03020100u), "v"(d)) }
    if constexpr (OP == 16) { CHAINS("v_bfe_u32 %0, %0, 3, 5", "v"(b)) }
    if constexpr (OP == 17) { CHAINS("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", "v"(b)) }
    if constexpr (OP == 18) { CHAINS("v_pk_add_u16 %0, %0, %1", "v"(b)) }
    if constexpr (OP == 19) { CHAINS("v_xad_u32 %0, %0, %1, %2", "v"(b), "v"(d)) }
    if constexpr (OP == 20) { CHAINS("v_and_b32 %0, 0x7070707, %0", "v"(b)) }
    if constexpr (OP == 21) { CHAINS("v_lshrrev_b16 %0, 8, %0", "v"(b)) }
    if constexpr (OP == 22) { CHAINS("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca", "v"(b), "v"(d)) }
    if constexpr (OP == 23) { CHAINS("v_and_b32 %0, 60, %0", "v"(b)) }
    if constexpr (OP == 24) { CHAINS("v_lshlrev_b32 %0, 2, %0", "v"(b)) }
    if constexpr (OP == 25) { CHAINS("v_or_b32 %0, %0, %1", "v"(b)) }
  }
  long long t1 = clock64();
  long long r1 = wall_clock64();
  uint32_t s = 0;
  for (int c = 0; c < 8; ++c) s ^= a[c] ^ __float_as_uint(f[c]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) { cyc[2 * (blockIdx.x * 4 + threadIdx.x / 64)] = t1 - t0; cyc[2 * (blockIdx.x * 4 + threadIdx.x / 64) + 1] = r1 - r0; }
}

static const char *names[] = {"v_xor_b32", "v_xor_b32_e64", "v_perm_b32", "v_bitop3_b32", "v_xor_b32(sgpr)",
                              "v_and_b32_sdwa", "v_lshrrev_b32", "v_alignbit_b32", "v_bfi_b32", "v_add_u32",
                              "v_fma_f32", "v_add_f32", "v_and_b32", "v_lshl_or_b32", "v_and_or_b32",
                              "v_perm_b32(sgpr)", "v_bfe_u32", "v_mov_b32_dpp", "v_pk_add_u16", "v_xad_u32",
                              "v_and_b32(literal)", "v_lshrrev_b16", "v_bitop3(bfi)", "v_and_b32(inline)", "v_lshlrev_b32", "v_or_b32"};

template <int OP>
static void run(uint32_t *out, long long *cyc, int cus) {
  const int iters = 65536;
  for (int w : {1, 2, 4, 5, 8}) {
    int blocks = cus * w;  // 4 waves per block -> one per SIMD per block
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(blocks * 8);
    hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    double mean = 0, rt = 0; for (size_t q = 0; q < h.size(); q += 2) { mean += h[q]; rt += h[q + 1]; }
    mean /= h.size() / 2; rt /= h.size() / 2;
    int wclk = 0; hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0);  // kHz
    double ghz = mean / (rt / (wclk * 1e3)) / 1e9;
    double ninstr = (double)iters * 8;
    // chip-wide issue rate from wall time: instructions per SIMD per ns
    double per_simd = ninstr * blocks * 4 / (cus * 4.0);
    printf("%-18s W=%d  cyc/instr/wave %.2f  cyc/instr/SIMD %.2f  clk %.2f GHz  wall %.3f ms  -> %.3f G instr/s/SIMD\n", names[OP], w,
           mean / ninstr, mean / ninstr / w, ghz, ms, per_simd / (ms * 1e6));
    hipEventDestroy(e0); hipEventDestroy(e1);
  }
}

template <int... OPS>
static void all(uint32_t *out, long long *cyc, int cus, std::integer_sequence<int, OPS...>) {
  (run<OPS>(out, cyc, cus), ...);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  int cus = p.multiProcessorCount;
  printf("%s CUs %d clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
  uint32_t *out; long long *cyc;
  hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
  hipMalloc(&cyc, (size_t)cus * 8 * 4 * 8 * 2);
  all(out, cyc, cus, std::make_integer_sequence<int, 26>{});
  return 0;
}
