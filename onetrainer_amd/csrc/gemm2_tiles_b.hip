// gemm2_kernel instances of tiles 1, 2 (one translation unit per tile family: parallel build).
#include "gemm2_kernel.h"

gemm2_fn gemm2_pick_b(int tile, int am, int bm, bool seg2, bool cs) {
  if (tile == 1) return pick2<256, 128, 8>(am, bm, seg2, cs);
  if (tile == 2) return pick2<128, 256, 8>(am, bm, seg2, cs);
  return nullptr;
}
