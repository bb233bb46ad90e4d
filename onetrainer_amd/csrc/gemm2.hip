// bf16 MFMA GEMM engine v2: launcher (the kernel template is gemm2_kernel.h, its instances are in
// gemm2_tiles_*.hip, one translation unit per tile family so they compile in parallel).
#include "gemm2_kernel.h"

#include <cstdlib>
#include <mutex>
#include <unordered_set>

gemm2_fn gemm2_pick_a(int tile, int am, int bm, bool seg2, bool cs);   // 0, 3   256x256
gemm2_fn gemm2_pick_b(int tile, int am, int bm, bool seg2, bool cs);   // 1, 2   256x128, 128x256
gemm2_fn gemm2_pick_c(int tile, int am, int bm, bool seg2, bool cs);   // 4, 5, 6, 9, 10  128x128, 128x64, 64x128
gemm2_fn gemm2_pick_d(int tile, int am, int bm, bool seg2, bool cs);   // 7, 8   x160
gemm2_fn gemm2_pick_ld(int tile, int am, int bm, int ldr, int parts);   // 1, 4, 7, 8 with a fused LoRA projection

// byte extent an operand's gathers may touch (the DMA descriptor's range)
static long long operand_bytes(int mode, const bf16_t* p, long long ld, int MN, int K, const ConvGeom& g) {
  (void)p;
  if (mode == OPM_K) return ((long long)(MN - 1) * ld + K) * 2;
  if (mode == OPM_MN || mode == OPM_CONV_WT) return ((long long)(K - 1) * ld + MN) * 2;
  return ((long long)g.N * g.SH * g.SW - 1) * g.ld * 2 + (long long)g.SC * 2;
}

// launched by otamd_gemm (gemm.hip) when the v2 tile is selected; returns OTAMD_EUNSUPPORTED
// when the operand extents do not fit the 31-bit DMA offsets (caller falls back to v1)
int gemm2_launch(const GemmArgs& a, int tile, int splits, hipStream_t stream) {
  const long long ab = operand_bytes(a.amode, a.A, a.lda, a.M, a.K, a.ga);
  const long long bb = operand_bytes(a.bmode, a.B, a.ldb, a.N, a.K, a.gb);
  if (ab <= 0 || bb <= 0 || ab >= 0x7fff0000LL || bb >= 0x7fff0000LL) return OTAMD_EUNSUPPORTED;
  gemm2_fn fn = nullptr;
  int BMv = 256, BNv = 256, NWv = 8, NSv = 2;
  const bool seg2 = a.A2 != nullptr;
  const bool cs = a.colsum != nullptr;
  if (cs && (a.amode != OPM_MN || seg2 || a.batch > 1 || (splits > 1 && !a.colsum_slab))) return OTAMD_EUNSUPPORTED;
  unsigned a2b = 0, b2b = 0;
  if (seg2) {
    const long long x = ((long long)(a.M - 1) * a.lda2 + a.K2) * 2;
    const long long y = a.bmode == OPM_K ? ((long long)(a.N - 1) * a.ldb2 + a.K2) * 2 : ((long long)(a.K2 - 1) * a.ldb2 + a.N) * 2;
    if (x <= 0 || y <= 0 || x >= 0x7fff0000LL || y >= 0x7fff0000LL) return OTAMD_EUNSUPPORTED;
    a2b = (unsigned)x;
    b2b = (unsigned)y;
  }
  // OTAMD_SKINNY_NS4=1: tiles 5 / 6 run on the 4-deep ring (tiles 9 / 10) when they have no second K segment
  static const bool skinny4 = [] { const char* e = getenv("OTAMD_SKINNY_NS4"); return e && e[0] == '1'; }();
  if (skinny4 && (tile == 5 || tile == 6) && !seg2) tile += 4;
  if (a.D) {   // LoRA down-projection fused (forward forms; split 1, whole adapter parts per tile: checked here)
    if (seg2 || cs || splits != 1 || a.batch > 1) return OTAMD_EUNSUPPORTED;
    // the dgrad form over several adapter parts along K: K1 = rows per part (gemm.hip validates)
    const int parts = (a.bmode == OPM_MN && a.K1 > 0 && a.K1 < a.K) ? a.K / a.K1 : 1;
    fn = gemm2_pick_ld(tile, a.amode, a.bmode, a.lora_r, parts);
  } else switch (tile) {
    case 0: case 3: fn = gemm2_pick_a(tile, a.amode, a.bmode, seg2, cs); break;
    case 1: case 2: fn = gemm2_pick_b(tile, a.amode, a.bmode, seg2, cs); break;
    case 4: case 5: case 6: case 9: case 10: fn = gemm2_pick_c(tile, a.amode, a.bmode, seg2, cs); break;
    case 7: case 8: fn = gemm2_pick_d(tile, a.amode, a.bmode, seg2, cs); break;
    default: break;
  }
  // tile geometry: (BM, BN, waves, ring depth)
  static const int geo[11][4] = {{256, 256, 8, 2}, {256, 128, 8, 2}, {128, 256, 8, 2}, {256, 256, 4, 2}, {128, 128, 8, 2},
                                 {128, 64, 8, 2},  {64, 128, 8, 2},  {128, 160, 8, 2}, {256, 160, 8, 2}, {128, 64, 8, 4},
                                 {64, 128, 8, 4}};
  if (tile >= 0 && tile < 11) { BMv = geo[tile][0]; BNv = geo[tile][1]; NWv = geo[tile][2]; NSv = geo[tile][3]; }
  if (!fn) return OTAMD_EUNSUPPORTED;
  if (a.D && (a.lora_pw % BNv || a.N % a.lora_pw)) return OTAMD_EUNSUPPORTED;
  const int tiles = ((a.M + BMv - 1) / BMv) * ((a.N + BNv - 1) / BNv);
  const int lds = NSv * (BMv + BNv + (a.D ? a.lora_r : 0)) * 128 + (cs && BMv == 256 ? (NWv * 64 / (BMv / 8)) * BMv * 4 : 0);
  {   // the LDS opt-in once per kernel instance (a per-launch driver call costs host time on every GEMM)
    static std::mutex mu;
    static std::unordered_set<const void*> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.insert((const void*)fn).second)
      hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  }
  hipLaunchKernelGGL(fn, dim3(tiles, a.batch > 1 ? a.batch : 1, splits), dim3(NWv * 64), lds, stream, a, (unsigned)ab,
                     (unsigned)bb, a2b, b2b);
  OTAMD_CHECK_LAUNCH();
  return OTAMD_OK;
}
