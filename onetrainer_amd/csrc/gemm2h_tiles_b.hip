// gemm2h_kernel (half-K DMA units) instances of tiles 4 (128x128), 7 (128x160), 8 (256x160).
#include "gemm2h_kernel.h"

gemm2_fn gemm2h_pick_b(int tile, int am, int bm, bool cs) {
  if (tile == 4) return pick2h<128, 128>(am, bm, cs);
  if (tile == 7) return pick2h<128, 160>(am, bm, cs);
  if (tile == 8) return pick2h<256, 160>(am, bm, cs);
  return nullptr;
}
