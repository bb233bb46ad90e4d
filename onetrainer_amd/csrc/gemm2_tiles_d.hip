// gemm2_kernel instances of tiles 7, 8 (one translation unit per tile family: parallel build).
#include "gemm2_kernel.h"

gemm2_fn gemm2_pick_d(int tile, int am, int bm, bool seg2, bool cs) {
  if (tile == 7) return pick2<128, 160, 8>(am, bm, seg2, cs);
  if (tile == 8) return pick2<256, 160, 8>(am, bm, seg2, cs);
  return nullptr;
}
