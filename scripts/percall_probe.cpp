// Per-call latency breakdown of one rs-6-3 stripe from host memory (the path an unmodified Ozone
// reaches, one stripe per encodeArrays call, ECKeyOutputStream.java:304).  Times, for cells of CELL bytes:
//   copy_in   : ozec_host_copy of the k data cells, pageable -> pinned arena (what the JNI glue does first)
//   copy_out  : ozec_host_copy of the p parity cells, pinned arena -> pageable
//   enc_pinned: ozec_encode on the arena's cells (DMA in place: H2D, kernel, D2H)
//   enc_pageable[chunk]: ozec_encode on the pageable cells with host_chunk = chunk (libozec's staged pipeline)
//   h2d / d2h / duplex: the raw link: one k-cell H2D, one p-cell D2H, both at once on two streams
// and the sum copy_in + enc_pinned + copy_out (the glue's serial path).  Build: scripts/percall_probe.sh
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "../include/ozec.h"

static double time_us(int iters, const std::function<void()> &f) {
  f();
  f();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) f();
  const auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
}

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
  uint8_t *arena = nullptr;
  CHECK(ozec_host_alloc((k + p) * cell, reinterpret_cast<void **>(&arena)));
  const uint8_t *in_pg[16], *in_pin[16];
  uint8_t *out_pg[16], *out_pin[16];
  void *dst_in[16], *dst_out[16];
  const void *src_in[16], *src_out[16];
  size_t nb[16];
  for (int j = 0; j < k; ++j) {
    in_pg[j] = data[j].data();
    in_pin[j] = arena + j * cell;
    dst_in[j] = arena + j * cell;
    src_in[j] = data[j].data();
    nb[j] = cell;
  }
  for (int r = 0; r < p; ++r) {
    out_pg[r] = par[r].data();
    out_pin[r] = arena + (k + r) * cell;
    dst_out[r] = par[r].data();
    src_out[r] = arena + (k + r) * cell;
  }
  const double cin = time_us(iters, [&] { CHECK(ozec_host_copy(dst_in, src_in, nb, k, 1)); });
  const double cout = time_us(iters, [&] { CHECK(ozec_host_copy(dst_out, src_out, nb, p, 0)); });
  const double epin = time_us(iters, [&] { CHECK(ozec_encode(enc, in_pin, out_pin, cell)); });
  std::printf("{\"cell\": %zu, \"copy_in_us\": %.1f, \"copy_out_us\": %.1f, \"enc_pinned_us\": %.1f, "
              "\"glue_serial_sum_us\": %.1f", cell, cin, cout, epin, cin + epin + cout);
  for (long chunk : {4l << 20, 512l << 10, 256l << 10}) {
    CHECK(ozec_set_tuning("host_chunk", chunk));
    const double e = time_us(iters, [&] { CHECK(ozec_encode(enc, in_pg, out_pg, cell)); });
    std::printf(", \"enc_pageable_chunk%ldK_us\": %.1f", chunk >> 10, e);
  }
  CHECK(ozec_set_tuning("host_chunk", 4 << 20));
  // a lone zero-copy call from pageable cells in 1..4 column chunks (copies of one overlapping the kernel on another),
  // twice over to see the spread
  for (int rep = 0; rep < 2; ++rep)
    for (long z : {1l, 2l, 3l, 4l}) {
      CHECK(ozec_set_tuning("host_zc_chunks", z));
      const double t = time_us(iters, [&] { CHECK(ozec_encode(enc, in_pg, out_pg, cell)); });
      std::printf(", \"enc_pageable_zc_chunks%ld_rep%d_us\": %.1f", z, rep, t);
    }
  CHECK(ozec_set_tuning("host_zc_chunks", 2));
  // the zero-copy grid and coding-kernel variant of the pinned call
  for (long g : {16l, 24l, 32l, 64l, 96l, 128l}) {
    CHECK(ozec_set_tuning("host_zero_copy", g));
    const double t = time_us(iters, [&] { CHECK(ozec_encode(enc, in_pin, out_pin, cell)); });
    std::printf(", \"enc_pinned_zc%ld_us\": %.1f", g, t);
  }
  CHECK(ozec_set_tuning("host_zero_copy", 48));
  for (long v : {1l, 5l, 11l}) {
    CHECK(ozec_set_tuning("gf_variant", v));
    const double t = time_us(iters, [&] { CHECK(ozec_encode(enc, in_pin, out_pin, cell)); });
    std::printf(", \"enc_pinned_gfvar%ld_us\": %.1f", v, t);
  }
  CHECK(ozec_set_tuning("gf_variant", 0));
  // the same two calls with the copy path (host_zero_copy = 0: H2D + kernel + D2H on the slot's stream)
  CHECK(ozec_set_tuning("host_zero_copy", 0));
  const double epin_copy = time_us(iters, [&] { CHECK(ozec_encode(enc, in_pin, out_pin, cell)); });
  const double epg_copy = time_us(iters, [&] { CHECK(ozec_encode(enc, in_pg, out_pg, cell)); });
  CHECK(ozec_set_tuning("host_zero_copy", 48));
  std::printf(", \"enc_pinned_copy_path_us\": %.1f, \"enc_pageable_copy_path_us\": %.1f", epin_copy, epg_copy);
  // the raw link on the arena
  uint8_t *d = nullptr;
  if (hipMalloc(&d, (k + p) * cell) != hipSuccess) return 1;
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  const double h2d = time_us(iters, [&] {
    (void)hipMemcpyAsync(d, arena, k * cell, hipMemcpyHostToDevice, s1);
    (void)hipStreamSynchronize(s1);
  });
  const double d2h = time_us(iters, [&] {
    (void)hipMemcpyAsync(arena + k * cell, d + k * cell, p * cell, hipMemcpyDeviceToHost, s2);
    (void)hipStreamSynchronize(s2);
  });
  const double dup = time_us(iters, [&] {
    (void)hipMemcpyAsync(d, arena, k * cell, hipMemcpyHostToDevice, s1);
    (void)hipMemcpyAsync(arena + k * cell, d + k * cell, p * cell, hipMemcpyDeviceToHost, s2);
    (void)hipStreamSynchronize(s1);
    (void)hipStreamSynchronize(s2);
  });
  const double empty = time_us(iters, [&] { (void)hipStreamSynchronize(s1); });
  // where the arena's pages live, and D2H into its first 3 MiB instead of its parity region
  int gnode = -9, n0 = -9, n6 = -9, n8 = -9;
  (void)ozec_device_numa_node(0, &gnode);
  (void)ozec_host_page_node(arena, &n0);
  (void)ozec_host_page_node(arena + k * cell, &n6);
  (void)ozec_host_page_node(arena + (k + p) * cell - 1, &n8);
  const double d2h_front = time_us(iters, [&] {
    (void)hipMemcpyAsync(arena, d + k * cell, p * cell, hipMemcpyDeviceToHost, s2);
    (void)hipStreamSynchronize(s2);
  });
  const double d2h_again = time_us(iters, [&] {
    (void)hipMemcpyAsync(arena + k * cell, d + k * cell, p * cell, hipMemcpyDeviceToHost, s2);
    (void)hipStreamSynchronize(s2);
  });
  const double d2h_dev0 = time_us(iters, [&] {
    (void)hipMemcpyAsync(arena + k * cell, d, p * cell, hipMemcpyDeviceToHost, s2);
    (void)hipStreamSynchronize(s2);
  });
  const double d2h_s1 = time_us(iters, [&] {
    (void)hipMemcpyAsync(arena + k * cell, d + k * cell, p * cell, hipMemcpyDeviceToHost, s1);
    (void)hipStreamSynchronize(s1);
  });
  std::printf(", \"gpu_node\": %d, \"page_node_0\": %d, \"page_node_parity\": %d, \"page_node_end\": %d, "
              "\"d2h_into_front_us\": %.1f, \"d2h_again_us\": %.1f, \"d2h_from_dev_offset0_us\": %.1f, "
              "\"d2h_on_stream1_us\": %.1f", gnode, n0, n6, n8, d2h_front, d2h_again, d2h_dev0, d2h_s1);
  // zero copy: the coding kernel reads the arena's data cells and writes its parity cells over PCIe itself (the
  // arena is registered, so its pages are mapped for the GPU), one launch and no copy operation
  void *dp = nullptr;
  (void)hipHostGetDevicePointer(&dp, arena, 0);
  std::vector<uint8_t> want(p * cell);
  CHECK(ozec_encode(enc, in_pin, out_pin, cell));  // reference parity through the staged path
  std::memcpy(want.data(), arena + k * cell, p * cell);
  std::memset(arena + k * cell, 0xA5, p * cell);
  uint8_t *dpp = static_cast<uint8_t *>(dp);
  auto zc = [&](hipStream_t s) {
    CHECK(ozec_encode_batch(enc, dpp, (k + p) * cell, cell, dpp + k * cell, (k + p) * cell, cell, 1, cell, s));
    (void)hipStreamSynchronize(s);
  };
  zc(s1);
  const bool zc_ok = std::memcmp(want.data(), arena + k * cell, p * cell) == 0;
  const double zc1 = time_us(iters, [&] { zc(s1); });
  const double zc2 = time_us(iters, [&] { zc(s2); });
  std::printf(", \"dev_ptr_equals_host\": %d, \"zero_copy_ok\": %d, \"zero_copy_encode_us\": %.1f, "
              "\"zero_copy_encode_stream2_us\": %.1f", dp == arena, zc_ok, zc1, zc2);
  for (long g : {8l, 16l, 32l, 64l, 128l, 512l}) {  // grid of the coding kernel (blocks of 256 threads, 4 KiB chunks)
    CHECK(ozec_set_tuning("grid", g));
    const double t = time_us(iters, [&] { zc(s1); });
    std::printf(", \"zero_copy_grid%ld_us\": %.1f", g, t);
  }
  CHECK(ozec_set_tuning("grid", 0));
  for (long v : {1l, 5l}) {  // gf_variant 1: cached loads/stores; 5: two vectors per lane
    CHECK(ozec_set_tuning("gf_variant", v));
    const double t = time_us(iters, [&] { zc(s1); });
    std::printf(", \"zero_copy_gfvar%ld_us\": %.1f", v, t);
  }
  CHECK(ozec_set_tuning("gf_variant", 0));
  std::printf(", \"h2d_us\": %.1f, \"d2h_us\": %.1f, \"h2d_d2h_concurrent_us\": %.1f, \"empty_sync_us\": %.2f}\n", h2d,
              d2h, dup, empty);
  (void)hipFree(d);
  CHECK(ozec_host_free(arena));
  ozec_coder_release(enc);
  ozec_coder_free(enc);
  return 0;
}
