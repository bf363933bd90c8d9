// Launch-side interface of the gfx950 kernels in kernels.hip (host code only sees these declarations).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/ozec.h"

namespace ozec {

// One coding job: rows x k coefficient matrix applied to k input units of every stripe.
//   input j of stripe s  : in  + s * in_stripe_stride  + in_off[j]
//   output r of stripe s : out + s * out_stripe_stride + out_off[r]
// (base may be null with absolute addresses in the offsets; strides may be 0 for a single stripe).
struct CodeArgs {
  const uint8_t *in;
  uint8_t *out;
  int64_t in_stripe_stride;
  int64_t out_stripe_stride;
  int64_t nstripes;
  int64_t len;
  int32_t k;
  int32_t rows;
  int32_t all_ones;  // every coefficient is 1 (XOR codec): pure XOR kernel
  int32_t pad_;
  int64_t in_off[OZEC_MAX_K];
  int64_t out_off[OZEC_MAX_ROWS];
  uint8_t coef[OZEC_MAX_ROWS * OZEC_MAX_K];  // row-major rows x k
};

// Per-window CRC job over equally sized cells: cell c at base + c * cell_stride, `len` bytes each.
struct CrcArgs {
  const uint8_t *base;
  int64_t cell_stride;
  int64_t ncells;
  int64_t len;
  int64_t bpc;
  int64_t nwin;            // ceil(len / bpc)
  uint32_t *out;           // out[c * out_cell_stride + w]
  int64_t out_cell_stride; // in uint32 elements
  const uint32_t *tables;  // device CRC tables for this type (CrcTables layout)
  uint32_t init_full;      // shift(0xFFFFFFFF, bpc bytes)
  uint32_t init_last;      // shift(0xFFFFFFFF, last window bytes)
  int32_t big_endian;
  int32_t raw;             // emit the raw (init 0, no xorout) register instead of getValue()
};

// Fused encode + CRC of every data and parity unit (bpc % 16 == 0, len % 16 == 0, 16-B aligned).
struct EncCrcArgs {
  CodeArgs code;
  CrcArgs crc;  // crc.base unused; crc.out = crcs[s][unit][w] with crc.out_cell_stride = nwin
};

// Device CRC table blob layout (uint32 entries), built on the host (crc_host.cpp):
//   [0, 4096)        slice tables T_0..T_15: T_m[v] = register after byte v then m zero bytes
//   [4096, 5120)     Z_1024: shift by 1024 bytes, 4 x 256 (one table per register byte)
//   [5120, 10240)    Z_32, Z_64, Z_128, Z_256, Z_512 (lane-combine tree levels 1..5; level 0 = T_15..T_12)
constexpr int kCrcSliceOff = 0;
constexpr int kCrcZ1024Off = 4096;
constexpr int kCrcTreeOff = 5120;
constexpr int kCrcTableWords = 10240;

hipError_t launch_code(const CodeArgs &a, hipStream_t stream);
hipError_t launch_crc_windows(const CrcArgs &a, hipStream_t stream);
hipError_t launch_encode_crc(const EncCrcArgs &a, hipStream_t stream);
hipError_t launch_fill_splitmix64(uint8_t *base, int64_t cell_stride, int64_t ncells, int64_t n, uint64_t seed,
                                  uint64_t first_stream, hipStream_t stream);
// true when the fused kernel supports this (k, rows) pair with the given geometry
bool encode_crc_supported(const CodeArgs &a, int64_t bpc);

}  // namespace ozec
