// Native host layer of the train step's hot ops: one C++ call per op from the autograd Functions
// (module/functional.py) down to the C-ABI launchers of libotamd.so (include/otamd.h).
//
// Mirrors onetrainer_amd/kernels.py one-for-one (same arguments, same contract checks, ValueError on a
// violated contract, RuntimeError on a launcher status), and is what kernels.py dispatches to: the
// ctypes path builds a GemmArgs struct field by field, keys the measured plan table with a 16-field
// tuple and allocates through torch.empty -- ~10 us of Python per GEMM, ~1,700 GEMMs per SDXL step.
// Here the shape checks read tensor metadata directly, outputs come from at::empty, the plan table is an
// unordered_map, and split-K workspaces are cached per (device, stream) like kernels.workspace.
//
// The reference has no counterpart (it launches every op through diffusers / torch from Python); the ops
// each launcher replaces are cited in include/otamd.h.
#include <torch/extension.h>

#include <array>
#include <map>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <utility>

#define __HIP_PLATFORM_AMD__ 1
#include "otamd.h"

namespace py = pybind11;
using at::Tensor;
using c10::optional;

namespace {

constexpr int kOpmConvWT = 5;

[[noreturn]] void fail(const std::string& m) { throw py::value_error(m); }
inline void req(bool c, const char* m) {
  if (!c) fail(m);
}
void check(int rc, const char* what) {
  static const char* err[] = {"", "invalid arguments (shape/alignment contract)", "kernel launch failed",
                              "unsupported configuration"};
  if (rc != OTAMD_OK) {
    const char* e = (rc >= 1 && rc <= 3) ? err[rc] : "error";
    throw std::runtime_error(std::string(what) + ": " + e + " (status " + std::to_string(rc) + ")");
  }
}
inline hipStream_t S(int64_t s) { return reinterpret_cast<hipStream_t>(s); }
inline void* P(const Tensor& t) { return t.data_ptr(); }
inline void* P(const optional<Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }
inline bool aligned(const Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; }
inline bool is_bf16(const Tensor& t) { return t.scalar_type() == at::kBFloat16; }
inline bool is_f32(const Tensor& t) { return t.scalar_type() == at::kFloat; }

// ---- workspace: one growing buffer per (device, stream), stream-ordered reuse (kernels.workspace) ----
struct WsKey {
  int dev;
  int64_t stream;
  bool operator==(const WsKey& o) const { return dev == o.dev && stream == o.stream; }
};
struct WsHash {
  size_t operator()(const WsKey& k) const { return std::hash<int64_t>()(k.stream) * 31 + k.dev; }
};
// Launchers are thread-compatible (the reference runs the VAE and text encoders in data-loader worker threads,
// DataLoaderMgdsMixin.py:47): the only mutable state is these two caches, each behind its own mutex.  A
// workspace is reused in the order of its own stream, so threads driving different streams never share one.
std::mutex g_ws_mu;
std::unordered_map<WsKey, Tensor, WsHash> g_ws;

void* workspace(int64_t nbytes, const at::Device& dev, int64_t stream) {
  if (nbytes <= 0) return nullptr;
  WsKey k{dev.index(), stream};
  std::lock_guard<std::mutex> lk(g_ws_mu);
  auto it = g_ws.find(k);
  if (it == g_ws.end() || it->second.numel() < nbytes) {
    Tensor t = at::empty({std::max<int64_t>(nbytes, 64LL << 20)}, at::TensorOptions().dtype(at::kByte).device(dev));
    g_ws[k] = t;
    return t.data_ptr();
  }
  return it->second.data_ptr();
}

// ---- measured plan table (kernels._plan_table): 16-field signature -> (tile, splits) ----
using PlanKey = std::array<int64_t, 16>;
struct PlanHash {
  size_t operator()(const PlanKey& k) const {
    size_t h = 1469598103934665603ULL;
    for (int64_t v : k) h = (h ^ (size_t)v) * 1099511628211ULL;
    return h;
  }
};
std::shared_mutex g_plans_mu;   // read per GEMM, written only when a table is loaded
std::unordered_map<PlanKey, std::pair<int, int>, PlanHash> g_plans;

bool lookup_plan(const PlanKey& k, int& tile, int& splits) {
  std::shared_lock<std::shared_mutex> lk(g_plans_mu);
  auto it = g_plans.find(k);
  if (it == g_plans.end()) return false;
  tile = it->second.first;
  splits = it->second.second;
  return true;
}

PlanKey tune_key(const GemmArgs& a) {
  return {a.amode, a.bmode, a.M, a.N, a.K, a.A2 ? a.K1 : 0, a.batch, a.c_f32, a.bias != nullptr, a.rowvec != nullptr,
          a.residual != nullptr, a.accumulate, a.ga.KH, a.ga.stride, a.ga.upsample, a.gb.KH};
}

int64_t ws_bytes(const GemmArgs& a, int s) {
  if (s <= 1) return 0;
  return (int64_t)s * a.M * a.N * 4 + (a.colsum ? (int64_t)s * a.M * 4 : 0);
}

// kernels._gemm with splits == 0 (plan table, else the library's analytic plan) or an explicit split count
void gemm(GemmArgs& a, int splits, const at::Device& dev, int64_t stream) {
  int t = 0, s = 0;
  if (splits == 0 && lookup_plan(tune_key(a), t, s)) {
    const int64_t wb = ws_bytes(a, s);
    check(otamd_gemm_explicit(&a, t, s, workspace(wb, dev, stream), wb, S(stream)), "otamd_gemm_explicit");
    return;
  }
  int s_out = 0;
  const long long wb = otamd_gemm_plan(&a, splits, &s_out);
  req(wb >= 0, "gemm plan");
  check(otamd_gemm(&a, s_out, wb > 0 ? workspace(wb, dev, stream) : nullptr, wb, S(stream)), "otamd_gemm");
}

GemmArgs new_args() {
  GemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.alpha = 1.f;
  a.rows_per_vec = 1;
  return a;
}

int64_t ld_rows(const Tensor& t) {
  req(t.dim() == 2 && t.stride(1) == 1, "2-D row-major tensor with unit inner stride required");
  req(t.stride(0) % 8 == 0 || t.size(0) == 1, "row stride must be a multiple of 8 elements");
  return t.size(0) > 1 ? t.stride(0) : t.size(1);
}

void epilogue(GemmArgs& a, const optional<Tensor>& bias, const optional<Tensor>& rowvec, int64_t rows_per_vec,
              const optional<Tensor>& residual, int64_t M, int64_t N) {
  if (bias) {
    req(is_bf16(*bias) && bias->numel() == N && bias->is_contiguous(), "bias: bf16 [N]");
    a.bias = bias->data_ptr();
  }
  if (rowvec) {
    const Tensor& r = *rowvec;
    req(is_bf16(r) && r.dim() == 2 && r.size(1) == N && r.stride(1) == 1, "rowvec: bf16 [groups, N]");
    req(rows_per_vec > 0 && (M + rows_per_vec - 1) / rows_per_vec <= r.size(0), "rowvec rows");
    a.rowvec = r.data_ptr();
    a.ldv = r.stride(0);
    a.rows_per_vec = (int)rows_per_vec;
  }
  if (residual) {
    const Tensor& r = *residual;
    req(is_bf16(r) && r.dim() == 2 && r.size(0) == M && r.size(1) == N && r.stride(1) == 1, "residual: bf16 [M,N]");
    a.residual = r.data_ptr();
    a.ldr = r.stride(0);
  }
}

Tensor out2d(const optional<Tensor>& out, int64_t M, int64_t N, at::ScalarType dt, const Tensor& like) {
  Tensor o = out ? *out : at::empty({M, N}, like.options().dtype(dt));
  req(o.dim() == 2 && o.size(0) == M && o.size(1) == N && o.stride(1) == 1 && (is_bf16(o) || is_f32(o)),
      "out: [M,N] bf16/f32");
  req(o.stride(0) % 4 == 0 || M == 1, "out row stride must be a multiple of 4");
  return o;
}

// second K segment (LoRA fused into its base GEMM); false when the split point is not 64-aligned
bool seg2(GemmArgs& a, const Tensor& t, const Tensor& b2, int64_t k1, bool b2_mn) {
  const int64_t r = t.size(1);
  if (k1 % 64 || r % 8) return false;
  req(is_bf16(t) && is_bf16(b2) && aligned(t) && aligned(b2), "LoRA operands bf16, aligned");
  req(b2_mn ? b2.size(0) == r : b2.size(1) == r, "LoRA operand shapes");
  a.A2 = t.data_ptr();
  a.lda2 = ld_rows(t);
  a.B2 = b2.data_ptr();
  a.ldb2 = ld_rows(b2);
  a.K1 = (int)k1;
  a.K2 = (int)r;
  a.K = (int)(k1 + r);
  return true;
}

// ---- Linear ----
Tensor linear(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, const optional<Tensor>& residual,
              const optional<Tensor>& rowvec, int64_t rows_per_vec, const optional<Tensor>& out, bool out_f32,
              double alpha, bool accumulate, const optional<Tensor>& lora_t, const optional<Tensor>& lora_b2,
              int64_t stream) {
  req(is_bf16(x) && is_bf16(w) && x.is_cuda(), "linear: bf16 cuda tensors");
  req(x.dim() == 2 && w.dim() == 2, "linear shapes");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  req(K == w.size(1) && K % 8 == 0 && N % 4 == 0, "linear shapes");
  req(aligned(x) && aligned(w), "16-byte aligned operands required");
  Tensor o = out2d(out, M, N, out_f32 ? at::kFloat : at::kBFloat16, x);
  GemmArgs a = new_args();
  a.A = x.data_ptr(); a.lda = ld_rows(x); a.amode = OPM_K;
  a.B = w.data_ptr(); a.ldb = ld_rows(w); a.bmode = OPM_K;
  a.C = o.data_ptr(); a.ldc = M > 1 ? o.stride(0) : N; a.c_f32 = is_f32(o); a.accumulate = accumulate;
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.alpha = (float)alpha;
  epilogue(a, bias, rowvec, rows_per_vec, residual, M, N);
  const bool fused = lora_t && seg2(a, *lora_t, *lora_b2, K, false);
  gemm(a, 0, x.device(), stream);
  if (lora_t && !fused)
    linear(*lora_t, *lora_b2, {}, {}, {}, 0, o, is_f32(o), 1.0, true, {}, {}, stream);
  return o;
}

// ---- LoRA forward with the down-projection fused into the base GEMM (GemmArgs.D) ----
// The plan is the measured one of the two-launch form's base GEMM (its second-segment signature); when that plan is a
// one-split launch on a tile with a fused instance, one launch computes t (into t_out) and y.  Otherwise, or with
// OTAMD_LORA_FUSE=0, the two launches: t = x down^T, then y with t as the second K segment.
std::atomic<bool> g_lora_fuse{[] { const char* e = getenv("OTAMD_LORA_FUSE"); return !(e && e[0] == '0'); }()};
bool lora_fuse_on() { return g_lora_fuse.load(std::memory_order_relaxed); }
void set_lora_fuse(bool on) { g_lora_fuse.store(on); }
std::atomic<long long> g_lora_fused{0}, g_lora_split{0};

// Every tile column of a part recomputes the part's t (BM x r over all of K): r / BN more MFMA work in the base GEMM
// (20-25 %), against the t GEMM's launch, its split-K reduce and two kernel boundaries.  In the C4 step the linear
// forms gain from it and the 3x3 conv forms (K = 2880-11520, the t GEMM a small fraction of the base) lose, so convs
// keep the two launches unless OTAMD_LORA_FUSE_CONV=1 (profiles/r6_lora_fused_ab.txt).
bool lora_fuse_conv() {
  static const bool v = [] { const char* e = getenv("OTAMD_LORA_FUSE_CONV"); return e && e[0] == '1'; }();
  return v;
}

// measured fused-LoRA choices (kernels._lora_plans, lora_plans_mi355x.json): (form, N, K, parts, M class) -> tile,
// or -1 for the two launches; shapes without an entry follow the two-launch form's plan
std::shared_mutex g_lora_plans_mu;
std::map<std::array<int64_t, 5>, int> g_lora_plans;
void set_lora_plans(const std::vector<std::vector<int64_t>>& rows) {
  std::unique_lock<std::shared_mutex> lk(g_lora_plans_mu);
  g_lora_plans.clear();
  for (const auto& r : rows) {
    req(r.size() == 6, "lora plan row: form, N, K, parts, mclass, tile");
    g_lora_plans[{r[0], r[1], r[2], r[3], r[4]}] = (int)r[5];
  }
}
// The entries were measured at M = 4096 / 16384 (one tile per CU or whole waves of them); at the aspect buckets' other
// row counts a tile grid just past a multiple of the 256 CUs runs a second round for a few tiles (4160 rows on
// 128x160 tiles: 264 tiles, ~2x the time), so an entry applies only while the grid fills its rounds >= 85 %.
// An entry for the exact row count (class slot = -M: the aspect buckets' rows, measured) comes first, unchecked.
int lora_plan(int64_t form, int64_t N, int64_t K, int64_t parts, int64_t M) {
  int tile = 0;
  {
    std::shared_lock<std::shared_mutex> lk(g_lora_plans_mu);
    auto ex = g_lora_plans.find({form, N, K, parts, -M});
    if (ex != g_lora_plans.end()) return ex->second;
    auto it = g_lora_plans.find({form, N, K, parts, M >= 8192 ? 1 : 0});
    if (it == g_lora_plans.end()) return 0;
    tile = it->second;
  }
  if (tile <= 0) return tile;
  const int64_t bm = (tile == 1 || tile == 8) ? 256 : 128, bn = (tile == 7 || tile == 8) ? 160 : 128;
  const int64_t tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  const int64_t rounds = (tiles + 255) / 256;
  return tiles * 100 >= rounds * 256 * 85 ? tile : 0;
}

bool lora_down_fused(GemmArgs& a, const Tensor& down2d, const Tensor& up2, const Tensor& t2d, int64_t k1, int64_t r,
                     int64_t pw, int64_t stream) {
  if (!lora_fuse_on() || r != 32 || pw <= 0 || a.N % pw || k1 % 64) return false;
  if (a.amode == OPM_CONV_FWD && !lora_fuse_conv()) return false;
  GemmArgs k = a;   // the two-launch form's base GEMM signature (plan table key)
  if (!seg2(k, t2d, up2, k1, false)) return false;
  int tile = 0, splits = 0;
  const int lp = a.amode == OPM_K ? lora_plan(0, a.N, k1, a.N / pw, a.M) : 0;
  if (lp == -1) return false;
  if (lp > 0) {
    tile = lp;
    splits = 1;
  } else if (!lookup_plan(tune_key(k), tile, splits)) {
    tile = otamd_gemm_plan_tile(&k, 0);
    if (otamd_gemm_plan(&k, 0, &splits) < 0) return false;
  }
  if (splits != 1) return false;
  if (tile == 0) tile = 4;   // no fused 256x256 instance (register cap): the 128x128 tile
  req(is_bf16(down2d) && is_bf16(up2) && is_bf16(t2d) && aligned(down2d) && aligned(up2) && aligned(t2d),
      "LoRA operands bf16, aligned");
  a.D = down2d.data_ptr(); a.ldd = ld_rows(down2d);
  a.B2 = up2.data_ptr(); a.ldb2 = ld_rows(up2);
  a.T = t2d.data_ptr(); a.ldt = ld_rows(t2d);
  a.lora_r = (int)r; a.lora_pw = (int)pw;
  const int rc = otamd_gemm_explicit(&a, tile, 1, nullptr, 0, S(stream));
  if (rc == OTAMD_EUNSUPPORTED) {
    a.D = nullptr; a.B2 = nullptr; a.T = nullptr;
    return false;
  }
  check(rc, "otamd_gemm_explicit (LoRA down fused)");
  return true;
}

Tensor linear_lora(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, const optional<Tensor>& residual,
                   const Tensor& down, const Tensor& up2, const Tensor& t_out, int64_t r, int64_t pw, int64_t stream) {
  req(is_bf16(x) && is_bf16(w) && x.is_cuda() && x.dim() == 2 && w.dim() == 2, "linear_lora: bf16 2-D");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  req(K == w.size(1) && K % 8 == 0 && N % 4 == 0 && aligned(x) && aligned(w), "linear_lora shapes");
  req(down.dim() == 2 && down.size(1) == K && up2.dim() == 2 && up2.size(0) == N && up2.size(1) == down.size(0) &&
      t_out.dim() == 2 && t_out.size(0) == M && t_out.size(1) == down.size(0), "linear_lora: LoRA shapes");
  Tensor o = out2d({}, M, N, at::kBFloat16, x);
  GemmArgs a = new_args();
  a.A = x.data_ptr(); a.lda = ld_rows(x); a.amode = OPM_K;
  a.B = w.data_ptr(); a.ldb = ld_rows(w); a.bmode = OPM_K;
  a.C = o.data_ptr(); a.ldc = M > 1 ? o.stride(0) : N;
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  epilogue(a, bias, {}, 0, residual, M, N);
  if (lora_down_fused(a, down, up2, t_out, K, r, pw, stream)) {
    ++g_lora_fused;
    return o;
  }
  ++g_lora_split;
  linear(x, down, {}, {}, {}, 0, t_out, false, 1.0, false, {}, {}, stream);
  return linear(x, w, bias, residual, {}, 0, o, false, 1.0, false, t_out, up2, stream);
}

Tensor linear_dgrad(const Tensor& dy, const Tensor& w, const optional<Tensor>& out, const optional<Tensor>& residual,
                    bool accumulate, const optional<Tensor>& lora_u, const optional<Tensor>& lora_a2, int64_t stream) {
  req(is_bf16(dy) && is_bf16(w), "linear_dgrad: bf16");
  req(dy.dim() == 2 && w.dim() == 2, "linear_dgrad shapes");
  const int64_t M = dy.size(0), N = dy.size(1), K = w.size(1);
  req(N == w.size(0) && N % 8 == 0 && K % 8 == 0, "linear_dgrad shapes");
  Tensor o = out2d(out, M, K, out ? out->scalar_type() : at::kBFloat16, dy);
  GemmArgs a = new_args();
  a.A = dy.data_ptr(); a.lda = ld_rows(dy); a.amode = OPM_K;
  a.B = w.data_ptr(); a.ldb = ld_rows(w); a.bmode = OPM_MN;
  a.C = o.data_ptr(); a.ldc = M > 1 ? o.stride(0) : K; a.c_f32 = is_f32(o); a.accumulate = accumulate;
  a.M = (int)M; a.N = (int)K; a.K = (int)N;
  epilogue(a, {}, {}, 0, residual, M, K);
  const bool fused = lora_u && seg2(a, *lora_u, *lora_a2, N, true);
  gemm(a, 0, dy.device(), stream);
  if (lora_u && !fused) linear_dgrad(*lora_u, *lora_a2, o, {}, true, {}, {}, stream);
  return o;
}

// ---- LoRA backward input gradient with u = dY (sB) fused into the dgrad GEMM (GemmArgs.D on a B = MN-mode GEMM) ----
// One adapter (a single-module linear site): dX = dY W + u A and u (into u_out, for the down projection's weight
// gradient) in one launch when the two-launch form's dgrad plan is a one-split launch on a tile with a fused instance
// and N (= in features) is a multiple of its width; otherwise (or with OTAMD_LORA_FUSE=0 / OTAMD_LORA_FUSE_DGRAD=0) the
// two launches: u = dY (sB), then dX with u as the second K segment.  Bit-identical either way at one split.
bool lora_fuse_dgrad() {
  static const bool v = [] { const char* e = getenv("OTAMD_LORA_FUSE_DGRAD"); return !(e && e[0] == '0'); }();
  return v;
}
std::atomic<long long> g_lora_dgrad_fused{0}, g_lora_dgrad_split{0};

Tensor linear_dgrad_lora(const Tensor& dy, const Tensor& w, const Tensor& up2, const Tensor& down, const Tensor& upT,
                         const Tensor& downT, const Tensor& u_out, int64_t stream) {
  req(is_bf16(dy) && is_bf16(w) && dy.dim() == 2 && w.dim() == 2, "linear_dgrad_lora: bf16 2-D");
  const int64_t M = dy.size(0), N = dy.size(1), K = w.size(1), r = up2.size(1), r1 = upT.size(0);
  req(N == w.size(0) && N % 8 == 0 && K % 8 == 0 && aligned(dy) && aligned(w), "linear_dgrad_lora shapes");
  req(up2.dim() == 2 && up2.size(0) == N && down.dim() == 2 && down.size(0) == r && down.size(1) == K &&
      upT.dim() == 2 && r1 > 0 && r % r1 == 0 && upT.size(1) == N && downT.dim() == 2 && downT.size(0) == K &&
      downT.size(1) == r && u_out.dim() == 2 && u_out.size(0) == M && u_out.size(1) == r, "linear_dgrad_lora: LoRA shapes");
  const int64_t parts = r / r1;   // adapter parts along the dgrad's K (a fused q|k|v site: 3)
  if (lora_fuse_on() && lora_fuse_dgrad() && r1 == 32 && (parts == 1 || parts == 3) && N % (64 * parts) == 0) {
    Tensor o = out2d({}, M, K, at::kBFloat16, dy);
    GemmArgs a = new_args();
    a.A = dy.data_ptr(); a.lda = ld_rows(dy); a.amode = OPM_K;
    a.B = w.data_ptr(); a.ldb = ld_rows(w); a.bmode = OPM_MN;
    a.C = o.data_ptr(); a.ldc = M > 1 ? o.stride(0) : K;
    a.M = (int)M; a.N = (int)K; a.K = (int)N;
    GemmArgs k = a;   // the two-launch form's dgrad signature (plan table key)
    req(seg2(k, u_out, down, N, true), "linear_dgrad_lora: second segment");
    int tile = 0, splits = 0;
    const int lp = lora_plan(1, K, N, parts, M);
    if (lp > 0) {
      tile = lp;
      splits = 1;
    } else if (lp == 0 && !lookup_plan(tune_key(k), tile, splits)) {
      tile = otamd_gemm_plan_tile(&k, 0);
      if (otamd_gemm_plan(&k, 0, &splits) < 0) splits = 0;
    }
    if (splits == 1) {
      if (tile == 0) tile = 4;   // no fused 256x256 instance (register cap): the 128x128 tile
      req(aligned(upT) && aligned(downT) && aligned(u_out) && is_bf16(upT) && is_bf16(downT) && is_bf16(u_out),
          "LoRA operands bf16, aligned");
      a.D = upT.data_ptr(); a.ldd = ld_rows(upT);
      a.B2 = downT.data_ptr(); a.ldb2 = ld_rows(downT);
      a.T = u_out.data_ptr(); a.ldt = ld_rows(u_out);
      a.lora_r = (int)r1; a.lora_pw = (int)K;
      a.K1 = parts > 1 ? (int)(N / parts) : 0;
      const int rc = otamd_gemm_explicit(&a, tile, 1, nullptr, 0, S(stream));
      if (rc != OTAMD_EUNSUPPORTED) {
        check(rc, "otamd_gemm_explicit (LoRA dgrad fused)");
        ++g_lora_dgrad_fused;
        return o;
      }
    }
  }
  ++g_lora_dgrad_split;
  linear_dgrad(dy, up2, u_out, {}, false, {}, {}, stream);
  return linear_dgrad(dy, w, {}, {}, false, u_out, down, stream);
}

void bias_grad_args(GemmArgs& a, const optional<Tensor>& bg, bool bias_acc, int64_t n) {
  if (bg) {
    req(bg->numel() == n && bg->is_contiguous() && (is_bf16(*bg) || is_f32(*bg)), "bias grad [N]");
    a.colsum = bg->data_ptr();
    a.colsum_f32 = is_f32(*bg);
    a.colsum_acc = bias_acc;
  }
}

Tensor linear_wgrad(const Tensor& dy, const Tensor& x, const optional<Tensor>& out, bool accumulate, int64_t splits,
                    double alpha, const optional<Tensor>& bias_grad, bool bias_acc, int64_t stream) {
  req(is_bf16(dy) && is_bf16(x), "linear_wgrad: bf16");
  req(dy.dim() == 2 && x.dim() == 2, "linear_wgrad shapes");
  const int64_t T = dy.size(0), N = dy.size(1), K = x.size(1);
  req(T == x.size(0) && N % 8 == 0 && K % 8 == 0, "linear_wgrad shapes");
  Tensor o = out2d(out, N, K, out ? out->scalar_type() : at::kBFloat16, dy);
  GemmArgs a = new_args();
  a.A = dy.data_ptr(); a.lda = ld_rows(dy); a.amode = OPM_MN;
  a.B = x.data_ptr(); a.ldb = ld_rows(x); a.bmode = OPM_MN;
  a.C = o.data_ptr(); a.ldc = o.stride(0); a.c_f32 = is_f32(o); a.accumulate = accumulate;
  a.M = (int)N; a.N = (int)K; a.K = (int)T; a.alpha = (float)alpha;
  bias_grad_args(a, bias_grad, bias_acc, N);
  gemm(a, (int)splits, dy.device(), stream);
  return o;
}

// ---- convolutions: NHWC activations, weights [Cout][KH][KW][Cin] ----
ConvGeom geom(int64_t N, int64_t SH, int64_t SW, int64_t SC, int64_t RH, int64_t RW, int64_t KH, int64_t KW,
              int64_t stride, int64_t pad, bool upsample, int64_t ld) {
  ConvGeom g;
  std::memset(&g, 0, sizeof(g));
  g.N = (int)N; g.SH = (int)SH; g.SW = (int)SW; g.SC = (int)SC; g.RH = (int)RH; g.RW = (int)RW;
  g.KH = (int)KH; g.KW = (int)KW; g.stride = (int)stride; g.pad = (int)pad; g.upsample = upsample; g.ld = ld;
  return g;
}

std::pair<int64_t, int64_t> conv_out_hw(int64_t H, int64_t W, int64_t k, int64_t stride, int64_t pad, bool up) {
  if (up) { H *= 2; W *= 2; }
  return {(H + 2 * pad - k) / stride + 1, (W + 2 * pad - k) / stride + 1};
}

struct Nhwc { int64_t N, H, W, C, ld; };
Nhwc nhwc(const Tensor& x) {
  req(x.dim() == 4 && is_bf16(x) && x.stride(3) == 1, "NHWC bf16 activation required");
  Nhwc r{x.size(0), x.size(1), x.size(2), x.size(3), x.stride(2)};
  req(x.stride(2) == x.stride(3) * r.C || x.stride(2) % 8 == 0, "pixel stride");
  req(x.stride(1) == x.stride(2) * r.W && x.stride(0) == x.stride(1) * r.H, "NHWC pixels must be uniformly strided");
  req(r.C % 8 == 0 && x.stride(2) % 8 == 0, "channels and pixel stride must be multiples of 8");
  return r;
}

Tensor conv2d(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, int64_t stride, int64_t pad,
              bool upsample, const optional<Tensor>& residual, const optional<Tensor>& rowvec,
              const optional<Tensor>& out, const optional<Tensor>& lora_t, const optional<Tensor>& lora_b2,
              int64_t out_h, int64_t out_w, int64_t stream) {
  const Nhwc s = nhwc(x);
  req(w.dim() == 4, "conv weight [Cout,KH,KW,Cin]");
  const int64_t Cout = w.size(0), KH = w.size(1), KW = w.size(2);
  req(w.size(3) == s.C && is_bf16(w) && w.is_contiguous() && Cout % 8 == 0, "conv weight [Cout,KH,KW,Cin]");
  req(aligned(x) && aligned(w), "aligned operands");
  auto pq = conv_out_hw(s.H, s.W, KH, stride, pad, upsample);
  int64_t Pp = pq.first, Q = pq.second;
  if (out_h > 0) {
    req(!upsample && out_h <= Pp + 1 && out_w <= Q + 1 && std::min(out_h, out_w) > 0, "conv out_hw");
    Pp = out_h;
    Q = out_w;
  }
  const int64_t M = s.N * Pp * Q;
  Tensor o = out ? *out : at::empty({s.N, Pp, Q, Cout}, x.options());
  req(o.dim() == 4 && o.size(0) == s.N && o.size(1) == Pp && o.size(2) == Q && o.size(3) == Cout && o.is_contiguous(),
      "conv out");
  GemmArgs a = new_args();
  a.A = x.data_ptr(); a.lda = 8; a.amode = OPM_CONV_FWD;
  a.ga = geom(s.N, s.H, s.W, s.C, Pp, Q, KH, KW, stride, pad, upsample, s.ld);
  a.B = w.data_ptr(); a.ldb = KH * KW * s.C; a.bmode = OPM_K;
  a.C = o.data_ptr(); a.ldc = Cout;
  a.M = (int)M; a.N = (int)Cout; a.K = (int)(KH * KW * s.C);
  optional<Tensor> res2;
  if (residual) res2 = residual->reshape({M, Cout});
  epilogue(a, bias, rowvec, rowvec ? Pp * Q : 0, res2, M, Cout);
  optional<Tensor> t2;
  if (lora_t) t2 = lora_t->reshape({M, lora_t->size(-1)});
  const bool fused = lora_t && seg2(a, *t2, *lora_b2, KH * KW * s.C, false);
  gemm(a, 0, x.device(), stream);
  if (lora_t && !fused) linear(*t2, *lora_b2, {}, {}, {}, 0, o.view({M, Cout}), false, 1.0, true, {}, {}, stream);
  return o;
}

// conv forward + LoRA with the down-projection (the base 3x3 geometry, in -> r) fused; t_out [N, P, Q, r]
Tensor conv2d_lora(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, int64_t stride, int64_t pad,
                   bool upsample, const optional<Tensor>& residual, const optional<Tensor>& rowvec, const Tensor& down,
                   const Tensor& up2, const Tensor& t_out, int64_t r, int64_t stream) {
  const Nhwc s = nhwc(x);
  req(w.dim() == 4 && down.dim() == 4, "conv weight [Cout,KH,KW,Cin]");
  const int64_t Cout = w.size(0), KH = w.size(1), KW = w.size(2);
  req(w.size(3) == s.C && is_bf16(w) && w.is_contiguous() && Cout % 8 == 0 && aligned(x) && aligned(w), "conv weight");
  req(down.size(1) == KH && down.size(2) == KW && down.size(3) == s.C && down.is_contiguous() && up2.dim() == 2 &&
      up2.size(0) == Cout && up2.size(1) == down.size(0), "conv2d_lora: LoRA shapes");
  auto pq = conv_out_hw(s.H, s.W, KH, stride, pad, upsample);
  const int64_t Pp = pq.first, Q = pq.second, M = s.N * Pp * Q, Kc = KH * KW * s.C;
  req(t_out.is_contiguous() && t_out.numel() == M * down.size(0), "conv2d_lora: t_out [N, P, Q, r]");
  Tensor o = at::empty({s.N, Pp, Q, Cout}, x.options());
  GemmArgs a = new_args();
  a.A = x.data_ptr(); a.lda = 8; a.amode = OPM_CONV_FWD;
  a.ga = geom(s.N, s.H, s.W, s.C, Pp, Q, KH, KW, stride, pad, upsample, s.ld);
  a.B = w.data_ptr(); a.ldb = Kc; a.bmode = OPM_K;
  a.C = o.data_ptr(); a.ldc = Cout;
  a.M = (int)M; a.N = (int)Cout; a.K = (int)Kc;
  optional<Tensor> res2;
  if (residual) res2 = residual->reshape({M, Cout});
  epilogue(a, bias, rowvec, rowvec ? Pp * Q : 0, res2, M, Cout);
  Tensor t2 = t_out.view({M, down.size(0)});
  if (lora_down_fused(a, down.view({down.size(0), Kc}), up2, t2, Kc, r, Cout, stream)) {
    ++g_lora_fused;
    return o;
  }
  ++g_lora_split;
  conv2d(x, down, {}, stride, pad, upsample, {}, {}, t_out, {}, {}, 0, 0, stream);
  return conv2d(x, w, bias, stride, pad, upsample, residual, rowvec, o, t_out, up2, 0, 0, stream);
}

Tensor conv2d_dgrad(const Tensor& dy, const Tensor& w, int64_t H, int64_t W, int64_t stride, int64_t pad,
                    const optional<Tensor>& out, bool accumulate, int64_t stream) {
  const Nhwc s = nhwc(dy);
  req(w.dim() == 4, "w [Cout,KH,KW,Cin]");
  const int64_t KH = w.size(1), KW = w.size(2), Cin = w.size(3);
  req(w.size(0) == s.C && w.is_contiguous() && Cin % 8 == 0 && s.C % 8 == 0 && aligned(w), "w [Cout,KH,KW,Cin]");
  req(conv_out_hw(H, W, KH, stride, pad, false) == std::make_pair(s.H, s.W), "dgrad geometry");
  Tensor o = out ? *out : at::empty({s.N, H, W, Cin}, dy.options());
  GemmArgs a = new_args();
  a.A = dy.data_ptr(); a.lda = 8; a.amode = OPM_CONV_DGRAD;
  a.ga = geom(s.N, s.H, s.W, s.C, H, W, KH, KW, stride, pad, false, s.ld);
  a.B = w.data_ptr(); a.ldb = Cin; a.bmode = kOpmConvWT;
  a.gb = geom(s.N, s.H, s.W, s.C, H, W, KH, KW, stride, pad, false, Cin);
  a.C = o.data_ptr(); a.ldc = Cin; a.accumulate = accumulate;
  a.M = (int)(s.N * H * W); a.N = (int)Cin; a.K = (int)(KH * KW * s.C);
  gemm(a, 0, dy.device(), stream);
  return o;
}

Tensor conv2d_wgrad(const Tensor& dy, const Tensor& x, int64_t ksize, int64_t stride, int64_t pad, bool upsample,
                    const optional<Tensor>& out, bool accumulate, int64_t splits, const optional<Tensor>& bias_grad,
                    bool bias_acc, int64_t stream) {
  const Nhwc d = nhwc(dy), s = nhwc(x);
  req(d.N == s.N && conv_out_hw(s.H, s.W, ksize, stride, pad, upsample) == std::make_pair(d.H, d.W), "wgrad geometry");
  Tensor o = out ? *out : at::empty({d.C, ksize, ksize, s.C}, dy.options());
  req(o.dim() == 4 && o.size(0) == d.C && o.size(1) == ksize && o.size(2) == ksize && o.size(3) == s.C &&
          o.is_contiguous(), "wgrad out");
  GemmArgs a = new_args();
  a.A = dy.data_ptr(); a.lda = d.ld; a.amode = OPM_MN;
  a.B = x.data_ptr(); a.ldb = 8; a.bmode = OPM_CONV_WGRAD;
  a.gb = geom(s.N, s.H, s.W, s.C, d.H, d.W, ksize, ksize, stride, pad, upsample, s.ld);
  a.C = o.data_ptr(); a.ldc = ksize * ksize * s.C; a.c_f32 = is_f32(o); a.accumulate = accumulate;
  a.M = (int)d.C; a.N = (int)(ksize * ksize * s.C); a.K = (int)(d.N * d.H * d.W);
  bias_grad_args(a, bias_grad, bias_acc, d.C);
  gemm(a, (int)splits, dy.device(), stream);
  return o;
}

// ---- normalization: NHWC / token-major rows ----
struct Rows { int64_t rows, C, ld; };
Rows rows2d(const Tensor& x) {
  req(is_bf16(x) && x.stride(-1) == 1, "bf16 with unit channel stride");
  const int64_t C = x.size(-1);
  const int64_t ld = x.dim() >= 2 ? x.stride(-2) : C;
  int64_t exp = ld;
  for (int64_t d = x.dim() - 2; d >= 0; --d) {
    if (x.size(d) > 1) req(x.stride(d) == exp, "rows must be uniformly strided");
    exp *= x.size(d);
  }
  return {x.numel() / C, C, ld};
}

py::tuple layernorm_fwd(const Tensor& x, const Tensor& gamma, const Tensor& beta, double eps, int64_t stream) {
  const Rows r = rows2d(x);
  Tensor y = at::empty(x.sizes(), x.options());
  const Rows ry = rows2d(y);
  Tensor mean = at::empty({r.rows}, x.options().dtype(at::kFloat));
  Tensor rstd = at::empty({r.rows}, x.options().dtype(at::kFloat));
  check(otamd_layernorm_fwd(P(x), r.ld, P(y), ry.ld, (int)r.rows, (int)r.C, (float)eps, P(gamma), P(beta),
                            (float*)P(mean), (float*)P(rstd), S(stream)), "otamd_layernorm_fwd");
  return py::make_tuple(y, py::make_tuple(mean, rstd));
}

// dx = LayerNorm-backward(dy) + dres; None when the width has no row-group form (kernels.py then runs two passes)
py::object layernorm_bwd_res(const Tensor& x, const Tensor& dy, const Tensor& dres, const Tensor& gamma,
                             const Tensor& mean, const Tensor& rstd, int64_t stream) {
  const Rows r = rows2d(x), rd = rows2d(dy);
  req(dres.sizes() == x.sizes() && is_bf16(dres), "layernorm residual grad: bf16, shape of x");
  const Rows rr = rows2d(dres);
  Tensor dx = at::empty(x.sizes(), x.options());
  const Rows rx = rows2d(dx);
  const int rc = otamd_layernorm_bwd_res(P(x), r.ld, P(dy), rd.ld, P(dres), rr.ld, P(dx), rx.ld, (int)r.rows, (int)r.C,
                                         P(gamma), (const float*)P(mean), (const float*)P(rstd), S(stream));
  if (rc == OTAMD_EUNSUPPORTED) return py::none();
  check(rc, "otamd_layernorm_bwd_res");
  return py::cast(dx);
}

void layernorm_param_grad(const Tensor& x, const Tensor& dy, const Tensor& mean, const Tensor& rstd,
                          const Tensor& dgamma, const Tensor& dbeta, bool param_acc, int64_t stream) {
  const Rows r = rows2d(x), rd = rows2d(dy);
  req(dgamma.scalar_type() == dbeta.scalar_type() && (is_bf16(dgamma) || is_f32(dgamma)),
      "layernorm param grads bf16 / f32");
  void* part = workspace(1024LL * 2 * r.C * 4, x.device(), stream);
  check(otamd_layernorm_param_grad(P(x), r.ld, P(dy), rd.ld, (int)r.rows, (int)r.C, (const float*)P(mean),
                                   (const float*)P(rstd), P(dgamma), P(dbeta), is_f32(dgamma), param_acc, (float*)part,
                                   S(stream)), "otamd_layernorm_param_grad");
}

py::tuple groupnorm_fwd(const Tensor& x, const Tensor& gamma, const Tensor& beta, int64_t groups, double eps,
                        bool silu, int64_t stream) {
  const int64_t N = x.size(0);
  const Rows r = rows2d(x);
  const int64_t HW = x.numel() / (N * r.C);
  Tensor y = at::empty(x.sizes(), x.options());
  const Rows ry = rows2d(y);
  auto f32 = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({N * groups}, f32), rstd = at::empty({N * groups}, f32);
  Tensor a = at::empty({N * r.C}, f32), b = at::empty({N * r.C}, f32);
  void* ws = workspace(4 * otamd_groupnorm_ws_floats((int)N, (int)HW, (int)r.C), x.device(), stream);
  check(otamd_groupnorm_fwd(P(x), r.ld, P(y), ry.ld, (int)N, (int)HW, (int)r.C, (int)groups, (float)eps, P(gamma),
                            P(beta), silu, (float*)P(mean), (float*)P(rstd), (float*)P(a), (float*)P(b), (float*)ws,
                            S(stream)), "otamd_groupnorm_fwd");
  return py::make_tuple(y, py::make_tuple(mean, rstd, a, b));
}

// dx (dgamma / dbeta written in place when given); dres: the input's residual-use gradient, added in the apply pass
Tensor groupnorm_bwd(const Tensor& x, const Tensor& dy, const Tensor& gamma, int64_t groups, bool silu,
                     const Tensor& mean, const Tensor& rstd, const Tensor& ga, const Tensor& gb,
                     const optional<Tensor>& dgamma, const optional<Tensor>& dbeta, bool param_acc,
                     const optional<Tensor>& dres, int64_t stream) {
  const int64_t N = x.size(0);
  const Rows r = rows2d(x), rd = rows2d(dy);
  const int64_t HW = x.numel() / (N * r.C);
  Tensor dx = at::empty(x.sizes(), x.options());
  const Rows rx = rows2d(dx);
  const int pf32 = dgamma && is_f32(*dgamma);
  void* ws = workspace(4 * otamd_groupnorm_ws_floats((int)N, (int)HW, (int)r.C), x.device(), stream);
  if (dres) {
    req(dres->sizes() == x.sizes() && is_bf16(*dres) && aligned(*dres), "groupnorm residual grad: bf16, shape of x, 16-byte aligned");
    const Rows rr = rows2d(*dres);
    check(otamd_groupnorm_bwd_res(P(x), r.ld, P(dy), rd.ld, P(*dres), rr.ld, P(dx), rx.ld, (int)N, (int)HW, (int)r.C,
                                  (int)groups, P(gamma), silu, (const float*)P(mean), (const float*)P(rstd),
                                  (const float*)P(ga), (const float*)P(gb), P(dgamma), P(dbeta), pf32, param_acc,
                                  (float*)ws, S(stream)), "otamd_groupnorm_bwd_res");
  } else {
    check(otamd_groupnorm_bwd(P(x), r.ld, P(dy), rd.ld, P(dx), rx.ld, (int)N, (int)HW, (int)r.C, (int)groups, P(gamma),
                              silu, (const float*)P(mean), (const float*)P(rstd), (const float*)P(ga),
                              (const float*)P(gb), P(dgamma), P(dbeta), pf32, param_acc, (float*)ws, 0, S(stream)),
          "otamd_groupnorm_bwd");
  }
  return dx;
}

// ---- flash attention (head dims <= 128): q [B, Nq, H*D] views, k / v [B, Nk, H*D] ----
std::pair<int64_t, int64_t> attn_view(const Tensor& t, int64_t heads) {
  req(t.dim() == 3 && is_bf16(t) && t.stride(2) == 1, "attention operand [B, N, H*D] bf16");
  req(t.size(2) % heads == 0, "channels must split into heads");
  return {t.stride(1), t.stride(0)};
}

AttnArgs attn_args(const Tensor& q, const Tensor& k, const Tensor& v, int64_t heads, double scale) {
  AttnArgs a;
  std::memset(&a, 0, sizeof(a));
  req(q.dim() == 3 && k.dim() == 3 && v.dim() == 3, "qkv");
  const int64_t B = q.size(0), Nq = q.size(1), Cq = q.size(2), Nk = k.size(1), D = Cq / heads;
  req(k.size(0) == B && v.size(0) == B && v.size(1) == Nk && k.size(2) == Cq && v.size(2) == Cq, "qkv");
  req(D % 8 == 0 && D <= 128, "head dim must be a multiple of 8 and <= 128");
  a.q = P(q); a.k = P(k); a.v = P(v);
  std::tie(a.ldq, a.bsq) = attn_view(q, heads);
  std::tie(a.ldk, a.bsk) = attn_view(k, heads);
  std::tie(a.ldv, a.bsv) = attn_view(v, heads);
  a.B = (int)B; a.H = (int)heads; a.Nq = (int)Nq; a.Nk = (int)Nk; a.Dv = (int)D;
  a.scale = scale > 0 ? (float)scale : (float)(1.0 / std::sqrt((double)D));
  return a;
}

py::tuple attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, int64_t heads, double scale,
                   const optional<Tensor>& out, int64_t stream) {
  AttnArgs a = attn_args(q, k, v, heads, scale);
  Tensor o = out ? *out : at::empty(q.sizes(), q.options());
  Tensor lse = at::empty({a.B, a.H, a.Nq}, q.options().dtype(at::kFloat));
  a.o = P(o);
  a.lse = (float*)P(lse);
  std::tie(a.ldo, a.bso) = attn_view(o, heads);
  check(otamd_attn_fwd(&a, S(stream)), "otamd_attn_fwd");
  return py::make_tuple(o, lse);
}

py::tuple attn_bwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, const Tensor& lse,
                   const Tensor& dout, int64_t heads, double scale, const optional<Tensor>& dq_,
                   const optional<Tensor>& dk_, const optional<Tensor>& dv_, int64_t stream) {
  AttnArgs a = attn_args(q, k, v, heads, scale);
  Tensor dq = dq_ ? *dq_ : at::empty(q.sizes(), q.options());
  Tensor dk = dk_ ? *dk_ : at::empty(k.sizes(), q.options());
  Tensor dv = dv_ ? *dv_ : at::empty(v.sizes(), q.options());
  a.o = P(o); a.lse = (float*)P(lse); a.dout = P(dout);
  std::tie(a.ldo, a.bso) = attn_view(o, heads);
  std::tie(a.lddo, a.bsdo) = attn_view(dout, heads);
  a.dq = P(dq); a.dk = P(dk); a.dv = P(dv);
  std::tie(a.lddq, a.bsdq) = attn_view(dq, heads);
  std::tie(a.lddk, a.bsdk) = attn_view(dk, heads);
  std::tie(a.lddv, a.bsdv) = attn_view(dv, heads);
  const long long nb = otamd_attn_bwd_ws_bytes(&a);
  req(nb > 0, "attention workspace query");
  void* ws = workspace(nb, q.device(), stream);
  check(otamd_attn_bwd(&a, (float*)ws, nb, S(stream)), "otamd_attn_bwd");
  return py::make_tuple(dq, dk, dv);
}

// ---- GEGLU (diffusers GEGLU: hidden * gelu(gate) over the proj output [rows, 2F]) ----
Tensor geglu_fwd(const Tensor& h, int64_t stream) {
  const Rows r = rows2d(h);
  const int64_t F = r.C / 2;
  std::vector<int64_t> sz(h.sizes().begin(), h.sizes().end());
  sz.back() = F;
  Tensor o = at::empty(sz, h.options());
  const Rows ro = rows2d(o);
  check(otamd_geglu_fwd(P(h), r.ld, P(o), ro.ld, (int)r.rows, (int)F, S(stream)), "otamd_geglu_fwd");
  return o;
}

Tensor geglu_bwd(const Tensor& h, const Tensor& dout, int64_t stream) {
  const Rows r = rows2d(h), rd = rows2d(dout);
  Tensor dh = at::empty(h.sizes(), h.options());
  const Rows rh = rows2d(dh);
  check(otamd_geglu_bwd(P(h), r.ld, P(dout), rd.ld, P(dh), rh.ld, (int)r.rows, (int)(r.C / 2), S(stream)),
        "otamd_geglu_bwd");
  return dh;
}

void set_plan_table(const std::vector<std::vector<int64_t>>& rows) {
  std::unordered_map<PlanKey, std::pair<int, int>, PlanHash> table;
  for (const auto& r : rows) {
    req(r.size() == 18, "plan table row: 16 key fields + tile + splits");
    PlanKey k;
    for (int i = 0; i < 16; ++i) k[i] = r[i];
    table[k] = {(int)r[16], (int)r[17]};
  }
  std::unique_lock<std::shared_mutex> lk(g_plans_mu);
  g_plans.swap(table);
}

int64_t plan_table_size() {
  std::shared_lock<std::shared_mutex> lk(g_plans_mu);
  return (int64_t)g_plans.size();
}
void clear_workspaces() {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  g_ws.clear();
}

}  // namespace

PYBIND11_MODULE(_otamd_host, m) {
  m.doc() = "native host layer of onetrainer_amd's hot ops (mirrors onetrainer_amd/kernels.py over libotamd.so)";
  m.def("linear", &linear);
  m.def("linear_dgrad", &linear_dgrad);
  m.def("linear_wgrad", &linear_wgrad);
  m.def("conv2d", &conv2d);
  m.def("linear_lora", &linear_lora);
  m.def("linear_dgrad_lora", &linear_dgrad_lora);
  m.def("set_lora_plans", &set_lora_plans);
  m.def("lora_plan", &lora_plan);   // the lookup alone (tests: the same answers as kernels._lora_plan)
  m.def("lora_dgrad_fused_counts",
        []() { return std::make_pair((long long)g_lora_dgrad_fused, (long long)g_lora_dgrad_split); });
  m.def("conv2d_lora", &conv2d_lora);
  m.def("set_lora_fuse", &set_lora_fuse);
  m.def("lora_fused_counts", []() { return std::make_pair((long long)g_lora_fused, (long long)g_lora_split); });
  m.def("conv2d_dgrad", &conv2d_dgrad);
  m.def("conv2d_wgrad", &conv2d_wgrad);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd_res", &layernorm_bwd_res);
  m.def("layernorm_param_grad", &layernorm_param_grad);
  m.def("groupnorm_fwd", &groupnorm_fwd);
  m.def("groupnorm_bwd", &groupnorm_bwd);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("geglu_fwd", &geglu_fwd);
  m.def("geglu_bwd", &geglu_bwd);
  m.def("set_plan_table", &set_plan_table);
  m.def("plan_table_size", &plan_table_size);
  m.def("clear_workspaces", &clear_workspaces);
  m.def("gemm_args_size", []() { return (int64_t)sizeof(GemmArgs); });
  m.def("attn_args_size", []() { return (int64_t)sizeof(AttnArgs); });
}
