// Read-stream ceiling on gfx950 for the access pattern of the streaming CRC kernel (crc_windows_g26s): each wave
// reads a contiguous run of `run` bytes, 1 KiB per wave-instruction (16 B per lane), with NS-1 instructions in
// flight, and folds the data into one register (XOR, so nothing is optimised away).  Compares global nt loads,
// plain global loads and raw buffer loads, and occupancy, on an 8 GiB buffer.  Tells how far the CRC kernel's
// 75-76 % of 8 TB/s is from what a pure read of the same shape reaches.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/read_bw.hip -o scripts/read_bw
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int NS, int MODE, int WAVES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES, 8))) void read_run(
    const uint8_t *base, int64_t total_steps, int64_t steps_per_wave, uint32_t *out) {
  const int lane = threadIdx.x & 63;
  const int64_t w = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int64_t s0 = w * steps_per_wave;
  if (s0 >= total_steps) return;
  const int64_t s1 = s0 + steps_per_wave < total_steps ? s0 + steps_per_wave : total_steps;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base + s0 * 1024), 0, 0x7fffffff, 0x00020000);
  u32x4 acc = {0, 0, 0, 0};
  u32x4 ring[NS];
  auto ld = [&](int64_t s) -> u32x4 {
    const int64_t sc = s < s1 ? s : s1 - 1;
    if constexpr (MODE == 0) {
      return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base + sc * 1024 + lane * 16));
    } else if constexpr (MODE == 1) {
      return *reinterpret_cast<const u32x4 *>(base + sc * 1024 + lane * 16);
    } else {
      const auto d = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<uint32_t>((sc - s0) * 1024 + lane * 16), 0, 2);
      return u32x4{d[0], d[1], d[2], d[3]};
    }
  };
#pragma unroll
  for (int i = 0; i + 1 < NS; ++i) ring[i] = ld(s0 + i);
  int64_t s = s0;
  for (; s + NS <= s1; s += NS) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      ring[(i + NS - 1) % NS] = ld(s + i + NS - 1);
      acc ^= ring[i];
    }
  }
  for (int i = 0; s < s1; ++s, ++i) acc ^= ld(s);
  const uint32_t v = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (v == 0x12345678u) out[w] = v;  // practically never: keeps the loads live
}

template <int NS, int MODE, int WAVES>
static void run(const char *name, const uint8_t *d, int64_t bytes, int64_t run_bytes, uint32_t *out) {
  const int64_t steps = bytes / 1024, per = run_bytes / 1024;
  const int64_t waves = (steps + per - 1) / per;
  const unsigned grid = static_cast<unsigned>((waves + 3) / 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((read_run<NS, MODE, WAVES>), dim3(grid), dim3(256), 0, 0, d, steps, per, out);
  std::vector<float> ms;
  for (int r = 0; r < 9; ++r) {
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((read_run<NS, MODE, WAVES>), dim3(grid), dim3(256), 0, 0, d, steps, per, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float t;
    hipEventElapsedTime(&t, a, b);
    ms.push_back(t / 5);
  }
  std::sort(ms.begin(), ms.end());
  const double t = ms[ms.size() / 2] * 1e-3;
  std::printf("%-28s run %7lld KiB  %.3f ms  %.2f TB/s  %.1f %% of 8 TB/s\n", name, (long long)(run_bytes >> 10),
              t * 1e3, bytes / t / 1e12, bytes / t / 8e12 * 100);
}



int main() {
  const int64_t bytes = int64_t{8} << 30;
  uint8_t *d;
  uint32_t *out;
  if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
  hipMemset(d, 0x5a, bytes);
  hipDeviceSynchronize();
  for (int64_t rb : {int64_t{64} << 10, int64_t{256} << 10, int64_t{1} << 20}) {
    run<4, 0, 1>("global nt, ring 4", d, bytes, rb, out);
    run<4, 1, 1>("global, ring 4", d, bytes, rb, out);
    run<4, 2, 1>("buffer nt, ring 4", d, bytes, rb, out);
    run<8, 0, 1>("global nt, ring 8", d, bytes, rb, out);
    run<2, 0, 1>("global nt, ring 2", d, bytes, rb, out);
  }
  hipFree(d);
  hipFree(out);
  return 0;
}
