// gemm2_kernel instances of tiles 4, 5, 6 (one translation unit per tile family: parallel build).
#include "gemm2_kernel.h"

gemm2_fn gemm2_pick_c(int tile, int am, int bm, bool seg2, bool cs) {
  if (tile == 4) return pick2<128, 128, 8>(am, bm, seg2, cs);
  if (tile == 5) return pick2<128, 64, 8>(am, bm, seg2, cs);
  if (tile == 6) return pick2<64, 128, 8>(am, bm, seg2, cs);
  return nullptr;
}
