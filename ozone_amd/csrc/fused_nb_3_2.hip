// encode_crc_nb variants of the rs-3-2 shape (fused_nb.hpp)
#include "fused_nb.hpp"

namespace ozec {
hipError_t launch_nb_3_2(const EncCrcArgs &e, hipStream_t st, int v, bool tail, bool wide) {
  if (wide) return launch_nb_wide_kr<3, 2>(e, st, tail);
  return tail ? launch_nb_tail_kr<3, 2>(e, st, v) : launch_nb_kr<3, 2>(e, st, v);
}
}  // namespace ozec
