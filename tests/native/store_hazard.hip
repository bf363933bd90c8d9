// Positive / negative controls for tests/isa_scan.py (compiled to a gfx950 code object by the CPU test, never
// launched): a 16-B global store whose data VGPRs a VALU op rewrites at once, and the same with the 2 wait states
// store_data_hold gives.  Registers are named in the asm so the schedule cannot move them apart.
#include <hip/hip_runtime.h>

__global__ void store_then_rewrite(int *p) {
  asm volatile("global_store_dwordx4 v[0:1], v[2:5], off\n\tv_mov_b32 v3, 0" ::: "v0", "v1", "v2", "v3", "v4", "v5",
               "memory");
}

__global__ void store_hold_rewrite(int *p) {
  asm volatile("global_store_dwordx4 v[0:1], v[2:5], off\n\ts_nop 1\n\tv_mov_b32 v3, 0" ::: "v0", "v1", "v2", "v3", "v4",
               "v5", "memory");
}
