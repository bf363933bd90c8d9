// Timeline of one rs-6-3 stripe of 1 MiB cells from pageable memory, the way libozec's zero-copy staged pipeline runs
// it (capi.cpp staged_pipeline, zc branch): per chunk, stage the k input columns into pinned staging (ozec_host_copy),
// launch the coding kernel on the staging in place (zero copy), record an event; unstage chunk c - 1 after its event.
// Rebuilt here step by step with CPU timestamps per phase, to find where a call's ~220 us go beyond the ~142 us the
// kernel needs for the whole stripe over PCIe.  Variants:
//   chunks 1..4; copies by ozec_host_copy (the pool) or memcpy on the calling thread;
//   "sdma": the chunk's inputs go up by hipMemcpyAsync (SDMA) into device memory and the kernel writes the parity
//   straight into pinned staging (zero copy on the write side only).
// Prints one JSON object per variant: mean us per stripe and the mean offset of every phase boundary.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/ozec.h"

using clk = std::chrono::steady_clock;

#define CHECK(x)                                                              \
  do {                                                                        \
    int rc_ = (x);                                                            \
    if (rc_ != 0) {                                                           \
      std::fprintf(stderr, "%s failed: %d %s\n", #x, rc_, ozec_last_error()); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

int main(int argc, char **argv) {
  const size_t cell = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : (1u << 20);
  const int iters = argc > 2 ? std::atoi(argv[2]) : 200;
  const int k = 6, p = 3;
  ozec_coder *enc = nullptr;
  CHECK(ozec_encoder_create(OZEC_CODEC_RS, k, p, &enc));
  std::vector<std::vector<uint8_t>> data(k, std::vector<uint8_t>(cell)), par(p, std::vector<uint8_t>(cell));
  for (int j = 0; j < k; ++j)
    for (size_t i = 0; i < cell; ++i) data[j][i] = static_cast<uint8_t>(i * 131 + j * 7 + (i >> 9));
  uint8_t *stage = nullptr;
  CHECK(ozec_host_alloc((k + p) * cell, reinterpret_cast<void **>(&stage)));
  uint8_t *dstage = nullptr;
  if (hipHostGetDevicePointer(reinterpret_cast<void **>(&dstage), stage, 0) != hipSuccess) return 1;
  uint8_t *dev = nullptr;
  if (hipMalloc(&dev, (k + p) * cell) != hipSuccess) return 1;
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev[8];
  for (auto &e : ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  // reference parity
  {
    const uint8_t *in[16];
    uint8_t *out[16];
    for (int j = 0; j < k; ++j) in[j] = data[j].data();
    for (int r = 0; r < p; ++r) out[r] = par[r].data();
    CHECK(ozec_encode(enc, in, out, cell));
  }
  std::vector<uint8_t> want(p * cell);
  for (int r = 0; r < p; ++r) std::memcpy(want.data() + r * cell, par[r].data(), cell);
  CHECK(ozec_set_tuning("grid", 32));

  std::printf("[");
  bool first = true;
  for (const std::string mode : {"zc-pool", "zc-memcpy", "sdma-pool"}) {
    for (int nch : {1, 2, 3, 4}) {
      const size_t cw = (cell / nch + 4095) / 4096 * 4096;
      const int n = static_cast<int>((cell + cw - 1) / cw);
      const bool pool = mode.find("pool") != std::string::npos, sdma = mode[0] == 's';
      // phase marks per chunk: stage done, launch returned, event waited, unstage done
      std::vector<double> mark(4 * n, 0.0);
      double total = 0;
      auto copy = [&](void **dst, const void **src, size_t *nb, int cnt, int to_staging) {
        if (pool) {
          CHECK(ozec_host_copy(dst, src, nb, cnt, to_staging));
        } else {
          for (int i = 0; i < cnt; ++i) std::memcpy(dst[i], src[i], nb[i]);
        }
      };
      auto once = [&](bool record) {
        const auto t0 = clk::now();
        auto at = [&](int c, int ph) {
          if (record) mark[4 * c + ph] += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
        };
        auto unstage = [&](int c) {
          (void)hipEventSynchronize(ev[c]);
          at(c, 2);
          const size_t off = c * cw, cl = std::min(cw, cell - off);
          void *dst[16];
          const void *src[16];
          size_t nb[16];
          for (int r = 0; r < p; ++r) {
            dst[r] = par[r].data() + off;
            src[r] = stage + (k + r) * cell + off;
            nb[r] = cl;
          }
          copy(dst, src, nb, p, 0);
          at(c, 3);
        };
        for (int c = 0; c < n; ++c) {
          const size_t off = c * cw, cl = std::min(cw, cell - off);
          void *dst[16];
          const void *src[16];
          size_t nb[16];
          for (int j = 0; j < k; ++j) {
            dst[j] = stage + j * cell + off;
            src[j] = data[j].data() + off;
            nb[j] = cl;
          }
          copy(dst, src, nb, k, 1);
          at(c, 0);
          if (sdma) {
            (void)hipMemcpy2DAsync(dev + off, cell, stage + off, cell, cl, k, hipMemcpyHostToDevice, s);
            CHECK(ozec_encode_batch(enc, dev + off, (k + p) * cell, cell, dstage + k * cell + off, (k + p) * cell, cell,
                                    1, cl, s));
          } else {
            CHECK(ozec_encode_batch(enc, dstage + off, (k + p) * cell, cell, dstage + k * cell + off, (k + p) * cell,
                                    cell, 1, cl, s));
          }
          (void)hipEventRecord(ev[c], s);
          at(c, 1);
          if (c > 0) unstage(c - 1);
        }
        unstage(n - 1);
        return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
      };
      once(false);
      once(false);
      for (int i = 0; i < iters; ++i) total += once(true);
      bool ok = true;
      for (int r = 0; r < p; ++r) ok &= std::memcmp(par[r].data(), want.data() + r * cell, cell) == 0;
      std::printf("%s{\"mode\": \"%s\", \"chunks\": %d, \"cell\": %zu, \"us\": %.1f, \"ok\": %d, \"marks_us\": [", first ? "" : ",\n",
                  mode.c_str(), n, cell, total / iters, ok);
      first = false;
      for (int c = 0; c < n; ++c)
        std::printf("%s[%.1f, %.1f, %.1f, %.1f]", c ? ", " : "", mark[4 * c] / iters, mark[4 * c + 1] / iters,
                    mark[4 * c + 2] / iters, mark[4 * c + 3] / iters);
      std::printf("]}");
      std::fflush(stdout);
    }
  }
  std::printf("]\n");
  // the kernel alone on the staging (no copies), and the copies alone
  const auto k0 = clk::now();
  for (int i = 0; i < iters; ++i) {
    CHECK(ozec_encode_batch(enc, dstage, (k + p) * cell, cell, dstage + k * cell, (k + p) * cell, cell, 1, cell, s));
    (void)hipStreamSynchronize(s);
  }
  const double kern = std::chrono::duration<double, std::micro>(clk::now() - k0).count() / iters;
  std::printf("{\"kernel_alone_zc_us\": %.1f}\n", kern);
  (void)hipFree(dev);
  CHECK(ozec_host_free(stage));
  ozec_coder_release(enc);
  ozec_coder_free(enc);
  return 0;
}
