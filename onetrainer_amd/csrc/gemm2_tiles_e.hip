// gemm2_kernel instances with a LoRA projection fused into the K loop (LDR = rank per adapter part; forward forms:
// linear and 3x3 conv with K-mode weights, t = x A^T; the linear backward's dgrad with MN-mode weights, u = dY (sB)).  Tiles with 2 waves along N: 256x128 (1), 128x128 (4), 128x160 (7),
// 256x160 (8); 256x256 spills at the 256-VGPR cap with the t accumulators (60-96 bytes of scratch per lane), so its
// plans run the fused form on 128x128 (ops_host.cpp lora_down_fused).  One translation unit: parallel build.
#include "gemm2_kernel.h"

template <int BM, int BN>
static gemm2_fn pick_ld(int am, int bm, int ldr, int parts) {
  if (ldr == 32) {
    if (parts == 1) {
      if (am == OPM_K && bm == OPM_K) return gemm2_kernel<OPM_K, OPM_K, BM, BN, 8, false, 2, false, 32>;
      if (am == OPM_CONV_FWD && bm == OPM_K) return gemm2_kernel<OPM_CONV_FWD, OPM_K, BM, BN, 8, false, 2, false, 32>;
      // the backward's input gradient with u = dY (sB) fused (MN-mode weights)
      if (am == OPM_K && bm == OPM_MN) return gemm2_kernel<OPM_K, OPM_MN, BM, BN, 8, false, 2, false, 32>;
    }
    // ... of a fused q|k|v site: u over three K parts
    if (parts == 3 && am == OPM_K && bm == OPM_MN) return gemm2_kernel<OPM_K, OPM_MN, BM, BN, 8, false, 2, false, 32, 3>;
  }
  return nullptr;
}

gemm2_fn gemm2_pick_ld(int tile, int am, int bm, int ldr, int parts) {
  switch (tile) {
    case 1: return pick_ld<256, 128>(am, bm, ldr, parts);
    case 4: return pick_ld<128, 128>(am, bm, ldr, parts);
    case 7: return pick_ld<128, 160>(am, bm, ldr, parts);
    case 8: return pick_ld<256, 160>(am, bm, ldr, parts);
    default: return nullptr;
  }
}
