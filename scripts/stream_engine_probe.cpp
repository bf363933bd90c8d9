// Copy rate per HIP stream (round 6: a 3 MiB pinned D2H ran at 17 GB/s on one stream of a process and 50 GB/s on
// another, scripts/percall_probe).  Creates N non-blocking streams, then per stream: H2D of 6 MiB and D2H of 3 MiB
// between a pinned host buffer and device memory, mean over iterations, then both directions at once on two
// consecutive streams.  Run it as is (SDMA engines) and with HSA_ENABLE_SDMA=0 (blit kernels) to compare.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <functional>

static double time_us(int iters, const std::function<void()> &f) {
  f();
  f();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) f();
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 8;
  const size_t hb = 6u << 20, db = 3u << 20;
  uint8_t *h = nullptr, *d = nullptr;
  if (hipHostMalloc(reinterpret_cast<void **>(&h), hb + db, hipHostMallocDefault) != hipSuccess) return 1;
  if (hipMalloc(&d, hb + db) != hipSuccess) return 1;
  // argv[2]: how the streams are made -- 0 hipStreamCreateWithFlags (non-blocking), 1 blocking hipStreamCreate,
  // 2 hipStreamCreateWithPriority at the highest priority, 3 at the lowest
  const int how = argc > 2 ? std::atoi(argv[2]) : 0;
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  hipStream_t st[64];
  for (int i = 0; i < n && i < 64; ++i) {
    if (how == 1) (void)hipStreamCreate(&st[i]);
    else if (how == 2) (void)hipStreamCreateWithPriority(&st[i], hipStreamNonBlocking, prio_hi);
    else if (how == 3) (void)hipStreamCreateWithPriority(&st[i], hipStreamNonBlocking, prio_lo);
    else (void)hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking);
  }
  std::printf("[");
  for (int i = -1; i < n && i < 64; ++i) {
    hipStream_t s = i < 0 ? nullptr : st[i];
    const double h2d = time_us(40, [&] {
      (void)hipMemcpyAsync(d, h, hb, hipMemcpyHostToDevice, s);
      (void)hipStreamSynchronize(s);
    });
    const double d2h = time_us(40, [&] {
      (void)hipMemcpyAsync(h + hb, d + hb, db, hipMemcpyDeviceToHost, s);
      (void)hipStreamSynchronize(s);
    });
    double both = 0;
    if (i >= 0 && i + 1 < n && i + 1 < 64) {
      hipStream_t s2 = st[i + 1];
      both = time_us(40, [&] {
        (void)hipMemcpyAsync(d, h, hb, hipMemcpyHostToDevice, s);
        (void)hipMemcpyAsync(h + hb, d + hb, db, hipMemcpyDeviceToHost, s2);
        (void)hipStreamSynchronize(s);
        (void)hipStreamSynchronize(s2);
      });
    }
    std::printf("%s{\"stream\": %d, \"h2d_6MiB_us\": %.1f, \"d2h_3MiB_us\": %.1f, \"h2d_here_d2h_next_us\": %.1f}\n",
                i < 0 ? "" : ",", i, h2d, d2h, both);
  }
  std::printf("]\n");
  return 0;
}
