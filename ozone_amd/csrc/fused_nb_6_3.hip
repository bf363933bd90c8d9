// encode_crc_nb variants of the rs-6-3 shape (fused_nb.hpp)
#include "fused_nb.hpp"

namespace ozec {
hipError_t launch_nb_6_3(const EncCrcArgs &e, hipStream_t st, int v, bool tail, bool wide) {
  if (wide) return launch_nb_wide_kr<6, 3>(e, st, tail);
  return tail ? launch_nb_tail_kr<6, 3>(e, st, v) : launch_nb_kr<6, 3>(e, st, v);
}
}  // namespace ozec
