// H2D / D2H rates into host memory of each kind libozec and its callers use (round 6: the JNI arena, an
// ozec_host_alloc block, measured D2H at 17 GB/s in scripts/percall_probe while libozec's staging slots ran at link
// rate).  Per kind and size: one H2D and one D2H of `size` bytes on one stream, mean over iterations after two warm-up
// copies.  Kinds: hipHostMalloc; ozec_host_alloc; malloc + hipHostRegister; mmap + MADV_HUGEPAGE + hipHostRegister;
// the same with the pages touched by the CPU first; ozec_host_alloc with the destination rewritten by the CPU between
// copies (what copy_out / copy_in do around every JNI call).
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../include/ozec.h"

static double time_us(int iters, const std::function<void()> &f) {
  f();
  f();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) f();
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
}

int main() {
  const size_t maxb = 8u << 20;
  uint8_t *d = nullptr;
  if (hipMalloc(&d, maxb) != hipSuccess) return 1;
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  struct Kind {
    std::string name;
    uint8_t *p;
    bool touch_between;
  };
  std::vector<Kind> kinds;
  uint8_t *hm = nullptr;
  (void)hipHostMalloc(reinterpret_cast<void **>(&hm), maxb, hipHostMallocDefault);
  kinds.push_back({"hipHostMalloc", hm, false});
  uint8_t *oa = nullptr;
  if (ozec_host_alloc(maxb, reinterpret_cast<void **>(&oa)) != 0) return 2;
  kinds.push_back({"ozec_host_alloc", oa, false});
  uint8_t *ma = static_cast<uint8_t *>(std::aligned_alloc(4096, maxb));
  std::memset(ma, 1, maxb);
  (void)hipHostRegister(ma, maxb, hipHostRegisterPortable);
  kinds.push_back({"malloc+register(touched)", ma, false});
  uint8_t *mm = static_cast<uint8_t *>(mmap(nullptr, maxb, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
  (void)madvise(mm, maxb, MADV_HUGEPAGE);
  (void)hipHostRegister(mm, maxb, hipHostRegisterPortable);
  kinds.push_back({"mmap+THP+register(untouched)", mm, false});
  uint8_t *mt = static_cast<uint8_t *>(mmap(nullptr, maxb, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
  (void)madvise(mt, maxb, MADV_HUGEPAGE);
  std::memset(mt, 1, maxb);
  (void)hipHostRegister(mt, maxb, hipHostRegisterPortable);
  kinds.push_back({"mmap+THP+touch+register", mt, false});
  kinds.push_back({"ozec_host_alloc, CPU rewrite between", oa, true});
  std::vector<uint8_t> src(maxb, 7);
  std::printf("[");
  bool first = true;
  for (const Kind &k : kinds) {
    for (size_t sz : {size_t{192} << 10, size_t{1} << 20, size_t{3} << 20, size_t{6} << 20}) {
      // the CPU's rewrite of the buffer (touch_between) runs before each copy and outside its timing
      auto timed_copy = [&](bool up) {
        double total = 0;
        for (int i = -2; i < 50; ++i) {
          if (k.touch_between) up ? (void)std::memcpy(k.p, src.data(), sz) : (void)std::memcpy(src.data(), k.p, sz);
          const auto t0 = std::chrono::steady_clock::now();
          if (up) (void)hipMemcpyAsync(d, k.p, sz, hipMemcpyHostToDevice, st);
          else (void)hipMemcpyAsync(k.p, d, sz, hipMemcpyDeviceToHost, st);
          (void)hipStreamSynchronize(st);
          if (i >= 0) total += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        }
        return total / 50;
      };
      const double h2d = timed_copy(true);
      const double d2h = timed_copy(false);
      std::printf("%s{\"kind\": \"%s\", \"bytes\": %zu, \"h2d_us\": %.1f, \"h2d_GBps\": %.1f, \"d2h_us\": %.1f, "
                  "\"d2h_GBps\": %.1f}\n", first ? "" : ",", k.name.c_str(), sz, h2d, sz / h2d / 1e3, d2h,
                  sz / d2h / 1e3);
      first = false;
    }
  }
  std::printf("]\n");
  return 0;
}
