// gemm2h_kernel (half-K DMA units) instances of the 256-wide tiles 0, 1, 2 (one translation unit per family).
#include "gemm2h_kernel.h"

gemm2_fn gemm2h_pick_a(int tile, int am, int bm, bool cs) {
  if (tile == 0) return pick2h<256, 256>(am, bm, cs);
  if (tile == 1) return pick2h<256, 128>(am, bm, cs);
  if (tile == 2) return pick2h<128, 256>(am, bm, cs);
  return nullptr;
}
