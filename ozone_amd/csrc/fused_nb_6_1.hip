// encode_crc_nb variants of the rs-6-1 shape (fused_nb.hpp): single-unit reconstruction of rs-6-x
#include "fused_nb.hpp"

namespace ozec {
hipError_t launch_nb_6_1(const EncCrcArgs &e, hipStream_t st, int v, bool tail, bool wide) {
  if (wide) return launch_nb_wide_kr<6, 1>(e, st, tail);
  return tail ? launch_nb_tail_kr<6, 1>(e, st, v) : launch_nb_kr<6, 1>(e, st, v);
}
}  // namespace ozec
