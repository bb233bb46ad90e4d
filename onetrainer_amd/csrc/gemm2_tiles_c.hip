// gemm2_kernel instances of tiles 4, 5, 6, 9, 10 (one translation unit per tile family: parallel build).
#include "gemm2_kernel.h"

gemm2_fn gemm2_pick_c(int tile, int am, int bm, bool seg2, bool cs) {
  if (tile == 4) return pick2<128, 128, 8>(am, bm, seg2, cs);
  if (tile == 5) return pick2<128, 64, 8>(am, bm, seg2, cs);
  if (tile == 6) return pick2<64, 128, 8>(am, bm, seg2, cs);
  // 9 / 10: the same tiles on a 4-deep LDS ring (96 KiB, one workgroup per CU): three K-steps of DMA in flight for
  // the skinny, latency-bound LoRA down-projections and adapter weight gradients (one workgroup per CU anyway)
  if (tile == 9) return pick2<128, 64, 8, 4>(am, bm, seg2, cs);
  if (tile == 10) return pick2<64, 128, 8, 4>(am, bm, seg2, cs);
  return nullptr;
}
