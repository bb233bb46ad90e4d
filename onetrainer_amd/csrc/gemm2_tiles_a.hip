// gemm2_kernel instances of tiles 0, 3 (one translation unit per tile family: parallel build).
#include "gemm2_kernel.h"

gemm2_fn gemm2_pick_a(int tile, int am, int bm, bool seg2, bool cs) {
  if (tile == 0) return pick2<256, 256, 8>(am, bm, seg2, cs);
  if (tile == 3 && !seg2) return pick2<256, 256, 4>(am, bm, false, cs);
  return nullptr;
}
