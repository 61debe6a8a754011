// torch.library registration of the llmtrain gfx950 kernels: torch.ops.llmtrain_hip.*
//
// Each op validates device / dtype / contiguity / shape on the host, allocates its outputs with
// the caching allocator and launches on the current HIP stream (so ops compose with RCCL's
// stream-ordered collectives and can be captured in a hipGraph).  Kernels are registered for
// the CUDA dispatch key, which is how PyTorch-ROCm names HIP devices.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <torch/library.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "kernels.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "llmtrain_hip: ", what, " failed: ", hipGetErrorString(e));
}

// fp32 scratch from the caching allocator (stream-ordered reuse; graph-capture safe)
Tensor workspace(const Tensor& like, long floats) {
  return at::empty({floats > 0 ? floats : 1}, like.options().dtype(at::kFloat));
}

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "llmtrain_hip: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), "llmtrain_hip: ", name, " must be contiguous");
}

void check_dtype(const Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.scalar_type() == dt, "llmtrain_hip: ", name, " must be ", dt, ", got ", t.scalar_type());
}

bool is_lowp(const Tensor& t, const char* name) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, "llmtrain_hip: ", name,
              " must be bf16 or f32");
  return t.scalar_type() == at::kBFloat16;
}

// dropout probability + site seed -> kernel arguments (thr = round(p * 2^16); the scale uses the
// quantised keep probability so the mask stays unbiased)
// set_dropout_seed_offset: a device word every dropout kernel launched while it is set adds to its
// site seed (hipGraph-captured steps: the word is restaged per replay; nullptr = off)
const uint32_t* g_seed_add = nullptr;

llmt::DropoutArgs make_dropout(double p, int64_t seed) {
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0, 1)");
  llmt::DropoutArgs d{};
  const uint32_t thr = (uint32_t)std::lround(p * 65536.0);
  if (thr == 0) return d;
  d.seed_add = g_seed_add;
  d.seed = (uint32_t)(seed & 0xffffffffLL);
  d.thr = thr > 65535u ? 65535u : thr;
  d.scale = 65536.0f / (float)(65536u - d.thr);
  return d;
}

// ---- LayerNorm -----------------------------------------------------------------------------
std::tuple<Tensor, Tensor, Tensor, Tensor> add_layernorm_fwd(const Tensor& x, const c10::optional<Tensor>& delta,
                                                             const Tensor& w, const Tensor& b, double eps,
                                                             at::ScalarType out_dtype, double dropout_p,
                                                             int64_t dropout_seed) {
  check_gpu(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "x must be f32 or bf16");
  check_gpu(w, "weight");
  check_gpu(b, "bias");
  check_dtype(w, at::kFloat, "weight");
  check_dtype(b, at::kFloat, "bias");
  TORCH_CHECK(x.dim() == 2, "x must be [M, d]");
  const int64_t M = x.size(0), d = x.size(1);
  TORCH_CHECK(w.numel() == d && b.numel() == d, "weight/bias must have d elements");
  TORCH_CHECK(d % 4 == 0 && d <= 2048, "LayerNorm kernel needs d % 4 == 0 and d <= 2048");
  TORCH_CHECK(out_dtype == at::kBFloat16 || out_dtype == at::kFloat, "out_dtype must be bf16 or f32");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  llmt::LnFwdArgs a{};
  Tensor xs;
  if (delta.has_value()) {
    check_gpu(*delta, "delta");
    TORCH_CHECK(delta->sizes() == x.sizes(), "delta must match x");
    a.delta = delta->data_ptr();
    a.delta_bf16 = is_lowp(*delta, "delta");
    xs = at::empty_like(x);
    a.xs_out = xs.data_ptr();
  } else {
    xs = at::empty({0}, x.options());
  }
  Tensor y = at::empty({M, d}, x.options().dtype(out_dtype));
  Tensor mean = at::empty({M}, x.options().dtype(at::kFloat));
  Tensor rstd = at::empty({M}, x.options().dtype(at::kFloat));
  a.x = x.data_ptr();
  a.x_bf16 = x.scalar_type() == at::kBFloat16;
  a.w = w.data_ptr<float>();
  a.b = b.data_ptr<float>();
  a.y = y.data_ptr();
  a.y_bf16 = out_dtype == at::kBFloat16;
  a.mean = mean.data_ptr<float>();
  a.rstd = rstd.data_ptr<float>();
  a.M = (int)M;
  a.d = (int)d;
  a.eps = (float)eps;
  a.dropout = make_dropout(dropout_p, dropout_seed);
  if (M > 0) check_hip(llmt::launch_add_layernorm_fwd(a, cur_stream()), "add_layernorm_fwd");
  return {xs, y, mean, rstd};
}

std::tuple<Tensor, Tensor, Tensor> layernorm_bwd_impl(const Tensor& dy, const Tensor& xs, const Tensor& mean,
                                                      const Tensor& rstd, const Tensor& w,
                                                      const c10::optional<Tensor>& dresid, Tensor dw, Tensor db,
                                                      const c10::optional<Tensor>& dy_scale, bool want_lowp,
                                                      const c10::optional<Tensor>& dproj, double dropout_p,
                                                      int64_t dropout_seed, bool defer_params, bool grad_lowp) {
  check_gpu(dy, "dy");
  check_gpu(xs, "xs");
  TORCH_CHECK(xs.scalar_type() == at::kFloat || xs.scalar_type() == at::kBFloat16, "xs must be f32 or bf16");
  TORCH_CHECK(dy.sizes() == xs.sizes() && xs.dim() == 2, "dy/xs must be [M, d]");
  const int64_t M = xs.size(0), d = xs.size(1);
  TORCH_CHECK(d % 4 == 0 && d <= 2048, "LayerNorm kernel needs d % 4 == 0 and d <= 2048");
  for (const Tensor* t : {&mean, &rstd}) {
    check_gpu(*t, "mean/rstd");
    check_dtype(*t, at::kFloat, "mean/rstd");
    TORCH_CHECK(t->numel() == M, "mean/rstd must have M elements");
  }
  for (const Tensor* t : {&w, static_cast<const Tensor*>(&dw), static_cast<const Tensor*>(&db)}) {
    check_gpu(*t, "weight/dweight/dbias");
    check_dtype(*t, at::kFloat, "weight/dweight/dbias");
    TORCH_CHECK(t->numel() == d, "weight/dweight/dbias must have d elements");
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(xs.device());
  llmt::LnBwdArgs a{};
  a.dy = dy.data_ptr();
  a.dy_bf16 = is_lowp(dy, "dy");
  a.xs = xs.data_ptr();
  a.xs_bf16 = xs.scalar_type() == at::kBFloat16;
  a.grad_bf16 = grad_lowp;
  TORCH_CHECK(a.dy_bf16 || !(a.xs_bf16 || grad_lowp), "layernorm_bwd: bf16 residual / gradient stream needs bf16 dy");
  TORCH_CHECK(grad_lowp || !a.xs_bf16, "layernorm_bwd: a bf16 residual stream takes a bf16 gradient stream");
  const auto gdt = grad_lowp ? at::kBFloat16 : at::kFloat;
  a.mean = mean.data_ptr<float>();
  a.rstd = rstd.data_ptr<float>();
  a.w = w.data_ptr<float>();
  if (dresid.has_value()) {
    check_gpu(*dresid, "dresid");
    check_dtype(*dresid, gdt, "dresid (the gradient stream's dtype)");
    TORCH_CHECK(dresid->sizes() == xs.sizes(), "dresid must match xs");
    a.dresid = dresid->data_ptr();
  }
  if (dy_scale.has_value()) {
    check_gpu(*dy_scale, "dy_scale");
    check_dtype(*dy_scale, at::kFloat, "dy_scale");
    TORCH_CHECK(dy_scale->numel() == 1, "dy_scale must be a scalar");
    a.dy_scale = dy_scale->data_ptr<float>();
  }
  Tensor dx = at::empty(xs.sizes(), xs.options().dtype(gdt));
  // a bf16 gradient stream without branch dropout IS the bf16 GEMM operand: no second write
  const bool lp_is_dx = want_lowp && grad_lowp && dropout_p <= 0.0;
  Tensor dx_lp = want_lowp ? (lp_is_dx ? dx : at::empty_like(dy)) : at::empty({0}, dy.options());
  a.dx = dx.data_ptr();
  a.dx_lp = want_lowp && !lp_is_dx ? dx_lp.data_ptr() : nullptr;
  a.dw = dw.data_ptr<float>();
  a.db = db.data_ptr<float>();
  if (dproj.has_value()) {
    check_gpu(*dproj, "dproj_bias");
    check_dtype(*dproj, at::kFloat, "dproj_bias");
    TORCH_CHECK(dproj->numel() == d, "dproj_bias must have d elements");
    a.dproj = dproj->data_ptr<float>();
  }
  a.M = (int)M;
  a.d = (int)d;
  a.dropout = make_dropout(dropout_p, dropout_seed);
  a.defer_params = defer_params;
  TORCH_CHECK(!(defer_params && a.dproj != nullptr), "layernorm_bwd: deferred reduce takes no dproj_bias");
  Tensor parts = at::empty({0}, xs.options().dtype(at::kFloat));
  if (M > 0) {
    Tensor ws = workspace(mean, llmt::layernorm_bwd_ws_floats(a));
    a.ws = ws.data_ptr<float>();
    check_hip(llmt::launch_layernorm_bwd(a, cur_stream()), "layernorm_bwd");
    // [2 (dw, db), grid, d] partial rows at the front of the workspace
    if (defer_params) parts = ws.narrow(0, 0, 2L * llmt::layernorm_bwd_grid(a) * d).view({2, -1, d});
  }
  return {dx, dx_lp, parts};
}

std::tuple<Tensor, Tensor> layernorm_bwd(const Tensor& dy, const Tensor& xs, const Tensor& mean, const Tensor& rstd,
                                         const Tensor& w, const c10::optional<Tensor>& dresid, Tensor dw, Tensor db,
                                         const c10::optional<Tensor>& dy_scale, bool want_lowp,
                                         const c10::optional<Tensor>& dproj, double dropout_p, int64_t dropout_seed,
                                         bool grad_lowp) {
  auto r = layernorm_bwd_impl(dy, xs, mean, rstd, w, dresid, dw, db, dy_scale, want_lowp, dproj, dropout_p,
                              dropout_seed, false, grad_lowp);
  return {std::get<0>(r), std::get<1>(r)};
}

// LayerNorm backward that leaves its dgamma / dbeta partial rows to a later batched reduce
// (ln_param_reduce): returns (dx, dx_lowp, parts [2, grid, d])
std::tuple<Tensor, Tensor, Tensor> layernorm_bwd_deferred(const Tensor& dy, const Tensor& xs, const Tensor& mean,
                                                          const Tensor& rstd, const Tensor& w,
                                                          const c10::optional<Tensor>& dresid, Tensor dw, Tensor db,
                                                          const c10::optional<Tensor>& dy_scale, bool want_lowp,
                                                          double dropout_p, int64_t dropout_seed, bool grad_lowp) {
  return layernorm_bwd_impl(dy, xs, mean, rstd, w, dresid, dw, db, dy_scale, want_lowp, c10::nullopt, dropout_p,
                            dropout_seed, true, grad_lowp);
}

// dst[j] += sum over rows of parts[j // 2][j % 2] for every deferred LayerNorm: ONE launch for up to
// two LayerNorms of equal (grid, d) (a block's ln_2 and ln_1), fixed order as in layernorm_bwd
void ln_param_reduce(const std::vector<Tensor>& parts, std::vector<Tensor> dst) {
  TORCH_CHECK(!parts.empty() && parts.size() <= 2 && dst.size() == 2 * parts.size(),
              "ln_param_reduce: 1-2 parts tensors and 2 destinations each");
  const int64_t grid = parts[0].size(1), d = parts[0].size(2);
  const float* p[4];
  float* o[4];
  for (size_t i = 0; i < parts.size(); ++i) {
    TORCH_CHECK(parts[i].dim() == 3 && parts[i].size(0) == 2 && parts[i].size(1) == grid && parts[i].size(2) == d,
                "ln_param_reduce: parts must be [2, grid, d] of one shape");
    for (int j = 0; j < 2; ++j) {
      Tensor& t = dst[2 * i + j];
      check_dtype(t, at::kFloat, "ln_param_reduce dst");
      TORCH_CHECK(t.numel() == d && t.is_contiguous(), "ln_param_reduce: dst must be [d]");
      p[2 * i + j] = parts[i].data_ptr<float>() + (long)j * grid * d;
      o[2 * i + j] = t.data_ptr<float>();
    }
  }
  const int njobs = (int)(2 * parts.size());
  Tensor scratch = workspace(parts[0], (long)njobs * llmt::colsum_scratch_floats((int)grid, d));
  check_hip(llmt::launch_colsum_reduce_multi(p, o, njobs, (int)grid, d, scratch.data_ptr<float>(), cur_stream()),
            "ln_param_reduce");
}

// ---- cross-entropy ---------------------------------------------------------------------------
Tensor cross_entropy_fwd_bwd(Tensor logits, const Tensor& labels, int64_t vocab, const Tensor& row_weight) {
  check_gpu(logits, "logits");
  check_gpu(labels, "labels");
  check_gpu(row_weight, "row_weight");
  check_dtype(labels, at::kLong, "labels");
  check_dtype(row_weight, at::kFloat, "row_weight");
  TORCH_CHECK(logits.dim() == 2, "logits must be [M, Vp]");
  const int64_t M = logits.size(0), Vp = logits.size(1);
  TORCH_CHECK(labels.numel() == M && row_weight.numel() == M, "labels/row_weight must have M elements");
  TORCH_CHECK(vocab > 0 && vocab <= Vp && Vp % 8 == 0 && Vp <= 131072, "need 0 < vocab <= Vp, Vp % 8 == 0");
  at::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  Tensor loss = at::empty({M}, row_weight.options());
  if (M > 0)
    check_hip(llmt::launch_cross_entropy_fwd_bwd(logits.data_ptr(), is_lowp(logits, "logits"),
                                                 labels.data_ptr<int64_t>(), row_weight.data_ptr<float>(),
                                                 loss.data_ptr<float>(), (int)M, (int)Vp, (int)vocab, cur_stream()),
              "cross_entropy_fwd_bwd");
  return loss;
}

// ---- elementwise -----------------------------------------------------------------------------
Tensor gelu_fwd(const Tensor& u) {
  check_gpu(u, "u");
  TORCH_CHECK(u.numel() % 8 == 0, "gelu needs numel % 8 == 0");
  at::hip::HIPGuardMasqueradingAsCUDA guard(u.device());
  Tensor g = at::empty_like(u);
  if (u.numel() > 0)
    check_hip(llmt::launch_gelu_fwd(u.data_ptr(), g.data_ptr(), is_lowp(u, "u"), u.numel(), cur_stream()), "gelu_fwd");
  return g;
}

Tensor scale(const Tensor& x, const Tensor& s) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.numel() % 8 == 0, "scale: contiguous x with numel % 8 == 0");
  TORCH_CHECK(s.is_cuda() && s.numel() == 1, "scale: s must be a 1-element GPU tensor");
  check_dtype(s, at::kFloat, "s");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = at::empty_like(x);
  if (x.numel() > 0)
    check_hip(llmt::launch_scale(x.data_ptr(), y.data_ptr(), s.data_ptr<float>(), is_lowp(x, "x"), x.numel(),
                                 cur_stream()),
              "scale");
  return y;
}

Tensor gelu_bwd(const Tensor& dg, const Tensor& u, const c10::optional<Tensor>& dbias) {
  check_gpu(dg, "dg");
  check_gpu(u, "u");
  TORCH_CHECK(dg.sizes() == u.sizes() && u.dim() == 2, "dg/u must be [M, F]");
  TORCH_CHECK(dg.scalar_type() == u.scalar_type(), "dg/u dtype mismatch");
  const int64_t M = u.size(0), F = u.size(1);
  TORCH_CHECK(F % 8 == 0, "gelu_bwd needs F % 8 == 0");
  float* db = nullptr;
  if (dbias.has_value()) {
    check_gpu(*dbias, "dbias");
    check_dtype(*dbias, at::kFloat, "dbias");
    TORCH_CHECK(dbias->numel() == F, "dbias must have F elements");
    db = dbias->data_ptr<float>();
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(u.device());
  Tensor du = at::empty_like(u);
  if (M > 0) {
    Tensor ws = workspace(u, db != nullptr ? llmt::colwise_ws_floats((int)M, (int)F) : 0);
    check_hip(llmt::launch_gelu_bwd(dg.data_ptr(), u.data_ptr(), du.data_ptr(), db, ws.data_ptr<float>(),
                                    is_lowp(u, "u"), (int)M, (int)F, cur_stream()),
              "gelu_bwd");
  }
  return du;
}

void colsum_accum(const Tensor& dy, Tensor out) {
  check_gpu(dy, "dy");
  check_gpu(out, "out");
  check_dtype(out, at::kFloat, "out");
  TORCH_CHECK(dy.dim() == 2 && out.numel() == dy.size(1), "dy [M, N], out [N]");
  TORCH_CHECK(dy.size(1) % 8 == 0, "colsum needs N % 8 == 0");
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  if (dy.size(0) > 0) {
    Tensor ws = workspace(out, llmt::colwise_ws_floats((int)dy.size(0), (int)dy.size(1)));
    check_hip(llmt::launch_colsum_accum(dy.data_ptr(), is_lowp(dy, "dy"), out.data_ptr<float>(), ws.data_ptr<float>(),
                                        (int)dy.size(0), (int)dy.size(1), cur_stream()),
              "colsum_accum");
  }
}

Tensor embedding_fwd(const Tensor& ids, const Tensor& wte, const Tensor& wpe, double dropout_p, int64_t dropout_seed,
                     bool out_lowp) {
  check_gpu(ids, "ids");
  check_gpu(wte, "wte");
  check_gpu(wpe, "wpe");
  check_dtype(ids, at::kLong, "ids");
  check_dtype(wte, at::kFloat, "wte");
  check_dtype(wpe, at::kFloat, "wpe");
  TORCH_CHECK(ids.dim() == 2, "ids must be [B, T]");
  const int64_t B = ids.size(0), T = ids.size(1), d = wte.size(1);
  TORCH_CHECK(wpe.size(1) == d && wpe.size(0) >= T && d % 4 == 0, "embedding shapes");
  at::hip::HIPGuardMasqueradingAsCUDA guard(ids.device());
  Tensor x = at::empty({B * T, d}, wte.options().dtype(out_lowp ? at::kBFloat16 : at::kFloat));
  if (B * T > 0)
    check_hip(llmt::launch_embedding_fwd(ids.data_ptr<int64_t>(), wte.data_ptr<float>(), wpe.data_ptr<float>(),
                                         x.data_ptr(), out_lowp, (int)B, (int)T, (int)d, (int)wte.size(0),
                                         make_dropout(dropout_p, dropout_seed), cur_stream()),
              "embedding_fwd");
  return x;
}

void embedding_bwd(const Tensor& dx, const Tensor& ids, Tensor dwte, Tensor dwpe, double dropout_p,
                   int64_t dropout_seed) {
  check_gpu(dx, "dx");
  check_gpu(ids, "ids");
  check_gpu(dwte, "dwte");
  check_gpu(dwpe, "dwpe");
  TORCH_CHECK(dx.scalar_type() == at::kFloat || dx.scalar_type() == at::kBFloat16, "dx must be float32 or bfloat16");
  TORCH_CHECK(dx.is_contiguous(), "dx must be contiguous");
  const bool dx_bf16 = dx.scalar_type() == at::kBFloat16;
  check_dtype(ids, at::kLong, "ids");
  check_dtype(dwte, at::kFloat, "dwte");
  check_dtype(dwpe, at::kFloat, "dwpe");
  const int64_t B = ids.size(0), T = ids.size(1), d = dwte.size(1);
  TORCH_CHECK(dx.size(0) == B * T && dx.size(1) == d && dwpe.size(0) >= T && dwpe.size(1) == d, "embedding shapes");
  at::hip::HIPGuardMasqueradingAsCUDA guard(dx.device());
  if (B * T == 0) return;
  const llmt::DropoutArgs dr = make_dropout(dropout_p, dropout_seed);
  check_hip(llmt::launch_embedding_bwd(dx.data_ptr(), dx_bf16, ids.data_ptr<int64_t>(),
                                       llmt::deterministic() ? nullptr : dwte.data_ptr<float>(),
                                       dwpe.data_ptr<float>(), (int)B, (int)T, (int)d, (int)dwte.size(0), dr,
                                       cur_stream()),
            "embedding_bwd");
  if (llmt::deterministic()) {
    // token gradient in a fixed order: stable sort of the token ids (rocPRIM radix sort), then one
    // wave per run of equal tokens sums its dx rows in sorted order (no atomics)
    auto sorted = ids.reshape({-1}).sort(/*stable=*/true, /*dim=*/0, /*descending=*/false);
    const Tensor& sorted_ids = std::get<0>(sorted);
    const Tensor& order = std::get<1>(sorted);
    check_hip(llmt::launch_embedding_bwd_sorted(dx.data_ptr(), dx_bf16, sorted_ids.data_ptr<int64_t>(),
                                                order.data_ptr<int64_t>(), dwte.data_ptr<float>(), (int)(B * T),
                                                (int)d, (int)dwte.size(0), dr, cur_stream()),
              "embedding_bwd_sorted");
  }
}

// ---- attention -------------------------------------------------------------------------------
// head dim from the packed qkv [B*T, 3*H*hd]: a multiple of 8 up to 64 (the kernels' tiles are 64
// wide; smaller heads are zero-filled in LDS/registers) or exactly 128 (two 64-wide halves)
int64_t attn_head_dim(const Tensor& qkv, int64_t B, int64_t T, int64_t H) {
  check_gpu(qkv, "qkv");
  check_dtype(qkv, at::kBFloat16, "qkv");
  TORCH_CHECK(B > 0 && T > 0 && H > 0 && qkv.numel() % (B * T * 3 * H) == 0, "qkv must be [B*T, 3*H*hd]");
  const int64_t hd = qkv.numel() / (B * T * 3 * H);
  TORCH_CHECK((hd % 8 == 0 && hd >= 8 && hd <= 64) || hd == 128,
              "attention kernels need head_dim % 8 == 0 and 8 <= head_dim <= 64, or head_dim == 128, got ", hd);
  return hd;
}

llmt::AttnDims attn_dims(int64_t B, int64_t T, int64_t H, int64_t hd) {
  llmt::AttnDims d{};
  d.B = (int)B;
  d.T = (int)T;
  d.H = (int)H;
  d.hd = (int)hd;
  d.scale = (float)(1.0 / std::sqrt((double)hd));
  return d;
}

std::tuple<Tensor, Tensor> attn_fwd(const Tensor& qkv, int64_t B, int64_t T, int64_t H, double dropout_p,
                                    int64_t dropout_seed, const c10::optional<Tensor>& key_bits) {
  const int64_t hd = attn_head_dim(qkv, B, T, H);
  at::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  llmt::AttnDims dims = attn_dims(B, T, H, hd);
  if (key_bits.has_value()) {
    check_gpu(*key_bits, "key_bits");
    check_dtype(*key_bits, at::kLong, "key_bits");
    TORCH_CHECK(key_bits->numel() == B * ((T + 63) / 64), "key_bits must be [B, ceil(T/64)] int64");
    dims.key_bits = reinterpret_cast<const uint64_t*>(key_bits->data_ptr<int64_t>());
  }
  Tensor out = at::empty({B * T, H * hd}, qkv.options());
  Tensor lse = at::empty({B, H, T}, qkv.options().dtype(at::kFloat));
  check_hip(llmt::launch_attn_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr<float>(), dims,
                                  make_dropout(dropout_p, dropout_seed), cur_stream()),
            "attn_fwd");
  return {out, lse};
}

Tensor attn_bwd(const Tensor& dout, const Tensor& qkv, const Tensor& out, const Tensor& lse, int64_t B, int64_t T,
                int64_t H, double dropout_p, int64_t dropout_seed, const c10::optional<Tensor>& dbias,
                const c10::optional<Tensor>& delta_in, const c10::optional<Tensor>& key_valid) {
  const int64_t hd = attn_head_dim(qkv, B, T, H);
  for (const Tensor* t : {&dout, &out}) {
    check_gpu(*t, "dout/out");
    check_dtype(*t, at::kBFloat16, "dout/out");
    TORCH_CHECK(t->numel() == B * T * H * hd, "dout/out must be [B*T, H*hd]");
  }
  check_gpu(lse, "lse");
  check_dtype(lse, at::kFloat, "lse");
  TORCH_CHECK(lse.numel() == B * H * T, "lse must be [B, H, T]");
  at::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  llmt::AttnDims dims = attn_dims(B, T, H, hd);
  if (key_valid.has_value()) {
    check_gpu(*key_valid, "key_valid");
    TORCH_CHECK(key_valid->scalar_type() == at::kByte || key_valid->scalar_type() == at::kBool,
                "key_valid must be uint8/bool");
    TORCH_CHECK(key_valid->numel() == B * T, "key_valid must be [B, T]");
    dims.key_valid = reinterpret_cast<const uint8_t*>(key_valid->data_ptr());
  }
  Tensor dqkv = at::empty_like(qkv);
  // delta_in: rowsum(dO * O) from the out-proj dX GEMM's epilogue (gemm_fused epilogue 3)
  Tensor delta;
  if (delta_in.has_value()) {
    check_gpu(*delta_in, "delta");
    check_dtype(*delta_in, at::kFloat, "delta");
    TORCH_CHECK(delta_in->numel() == B * H * T && delta_in->is_contiguous(), "delta must be [B, H, T]");
    delta = *delta_in;
  } else {
    delta = at::empty({B, H, T}, lse.options());
  }
  Tensor dq = at::empty({llmt::attn_bwd_workspace_floats((int)B, (int)T, (int)H, (int)hd)}, lse.options());
  Tensor bias_ws = workspace(lse, dbias.has_value() ? llmt::attn_bwd_bias_ws_floats((int)B, (int)T, (int)H, (int)hd) : 0);
  float* db = nullptr;
  if (dbias.has_value()) {
    check_gpu(*dbias, "dbias");
    check_dtype(*dbias, at::kFloat, "dbias");
    TORCH_CHECK(dbias->numel() == 3 * H * hd, "dbias must have 3*H*hd elements");
    db = dbias->data_ptr<float>();
  }
  check_hip(llmt::launch_attn_bwd(dout.data_ptr(), qkv.data_ptr(), out.data_ptr(), lse.data_ptr<float>(),
                                  dqkv.data_ptr(), delta.data_ptr<float>(), dq.data_ptr<float>(), db,
                                  bias_ws.data_ptr<float>(), dims,
                                  make_dropout(dropout_p, dropout_seed), cur_stream(), delta_in.has_value()),
            "attn_bwd");
  return dqkv;
}

// process-wide deterministic mode (run.deterministic): fixed-order split-K / embedding reductions
void set_deterministic(bool on) { llmt::set_deterministic(on); }
void set_dropout_seed_offset(const c10::optional<Tensor>& word) {
  if (!word.has_value()) {
    g_seed_add = nullptr;
    return;
  }
  check_gpu(*word, "dropout seed offset");
  TORCH_CHECK(word->scalar_type() == at::kInt && word->numel() >= 1, "dropout seed offset: int32 device word");
  g_seed_add = reinterpret_cast<const uint32_t*>(word->data_ptr<int32_t>());
}
bool get_deterministic() { return llmt::deterministic(); }

// keep-mask of `n` consecutive elements of one dropout site (tests / debugging)
Tensor dropout_mask(int64_t n, double p, int64_t seed, const Tensor& like) {
  check_gpu(like, "like");
  at::hip::HIPGuardMasqueradingAsCUDA guard(like.device());
  Tensor m = at::empty({n}, like.options().dtype(at::kBool));
  if (n > 0)
    check_hip(llmt::launch_dropout_mask(make_dropout(p, seed), (bool*)m.data_ptr(), n, cur_stream()), "dropout_mask");
  return m;
}

// ---- weight-gradient GEMM --------------------------------------------------------------------
// dst[N, K] (fp32) += dy[M, N]^T x[M, K], and bias[N] += colsum(dy) when given (ping-pong kernel)
void wgrad_gemm_pp(const Tensor& dy, const Tensor& x, Tensor c, const c10::optional<Tensor>& bias, int64_t split,
                   int64_t mode) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && c.is_cuda(), "wgrad_gemm_pp: GPU tensors required");
  check_dtype(dy, at::kBFloat16, "dy");
  check_dtype(x, at::kBFloat16, "x");
  check_dtype(c, at::kFloat, "c");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && c.dim() == 2, "wgrad_gemm_pp: 2D operands");
  TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1 && c.stride(1) == 1, "wgrad_gemm_pp: unit inner stride");
  const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
  TORCH_CHECK(x.size(0) == M && c.size(0) == N && c.size(1) == K, "wgrad_gemm_pp: shape mismatch");
  TORCH_CHECK((uintptr_t)dy.data_ptr() % 16 == 0 && (uintptr_t)x.data_ptr() % 16 == 0,
              "wgrad_gemm_pp: operands must be 16-byte aligned");
  float* bptr = nullptr;
  if (bias.has_value()) {
    check_gpu(*bias, "bias");
    check_dtype(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == N, "wgrad_gemm_pp: bias must have N elements");
    bptr = bias->data_ptr<float>();
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(c.device());
  const long wsf = llmt::wgrad_pp_ws_floats((int)dy.stride(0), (int)x.stride(0), (int)M, (int)N, (int)K, (int)split,
                                            (int)mode, bptr != nullptr);
  Tensor ws = workspace(c, wsf);
  check_hip(llmt::launch_wgrad_pp(dy.data_ptr(), (int)dy.stride(0), x.data_ptr(), (int)x.stride(0),
                                  c.data_ptr<float>(), (int)c.stride(0), (int)M, (int)N, (int)K, (int)split, (int)mode,
                                  wsf > 0 ? ws.data_ptr<float>() : nullptr, bptr, cur_stream()),
            "wgrad_gemm_pp");
}

// the weight-gradient plan for a shape (introspection for tests and bench/wgrad_pp.py; no GPU work)
std::vector<int64_t> wgrad_pp_plan(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, bool bias, int64_t split,
                                   int64_t mode) {
  long out[12] = {0};
  const int n = llmt::wgrad_pp_plan_info((int)lda, (int)ldb, (int)M, (int)N, (int)K, bias, (int)split, (int)mode, out);
  TORCH_CHECK(n == 12, "wgrad_pp_plan: invalid shape");
  return std::vector<int64_t>(out, out + 12);
}

// ---- fused forward / dX GEMM ------------------------------------------------------------------
// out = epi(a @ op(b)): b is [N, K] (weight, forward) or, with b_kn, [K, N] (weight in dX = dy @ W).
// epilogue 0 -> (out, None); 1 -> (u, gelu(u)); 2 -> (du = acc * gelu'(u), None) with dbias += colsum.
// `out_opt` (epilogue 0): write C into this [M, N] bf16 tensor (e.g. a row chunk of a larger output)
// instead of a fresh allocation — no copy of a multi-GB result.
std::tuple<Tensor, c10::optional<Tensor>> gemm_fused(const Tensor& a, const Tensor& b, bool b_kn, int64_t epilogue,
                                                     const c10::optional<Tensor>& bias, const c10::optional<Tensor>& u,
                                                     c10::optional<Tensor> dbias, int64_t seq_len,
                                                     const c10::optional<Tensor>& out_opt) {
  check_gpu(a, "a");
  check_gpu(b, "b");
  check_dtype(a, at::kBFloat16, "a");
  check_dtype(b, at::kBFloat16, "b");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2, "gemm_fused: 2D operands");
  const int64_t M = a.size(0), K = a.size(1);
  const int64_t N = b_kn ? b.size(1) : b.size(0);
  TORCH_CHECK((b_kn ? b.size(0) : b.size(1)) == K, "gemm_fused: inner dimensions differ");
  TORCH_CHECK(K % 64 == 0 && K >= 256 && N % 8 == 0, "gemm_fused: needs K % 64 == 0, K >= 256, N % 8 == 0");
  TORCH_CHECK(epilogue >= 0 && epilogue <= 5, "gemm_fused: epilogue must be 0-5");
  const bool has_u = epilogue == 2 || epilogue == 3 || epilogue == 5;
  const bool gelu_out = epilogue == 1 || epilogue == 4;
  // the kernel's buffer descriptors and tile offsets are 32-bit byte offsets: every operand and
  // output (a [M,K], b, out / u / c2 [M,N]) must stay below 2 GiB, else loads read zeros and
  // stores drop silently — callers split larger GEMMs into row chunks (llmtrain/ops, _gemm_rows)
  TORCH_CHECK(M * std::max(K, N) * 2 < (int64_t(1) << 31) && K * N * 2 < (int64_t(1) << 31),
              "gemm_fused: an operand or output reaches 2 GiB (M=", M, ", K=", K, ", N=", N,
              "); split the rows");
  // 16-byte LDS-DMA / vector stores on every operand, 4-byte DMA of the bias
  TORCH_CHECK((uintptr_t)a.data_ptr() % 16 == 0 && (uintptr_t)b.data_ptr() % 16 == 0,
              "gemm_fused: operands must be 16-byte aligned");
  at::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  llmt::GemmFusedArgs g;
  g.a = a.data_ptr();
  g.lda = (int)K;
  g.b = b.data_ptr();
  g.ldb = (int)b.size(1);
  g.b_kn = b_kn;
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.epilogue = (int)epilogue;
  Tensor out;
  if (out_opt.has_value()) {
    TORCH_CHECK(epilogue == 0, "gemm_fused: out= is for epilogue 0");
    check_gpu(*out_opt, "out");
    check_dtype(*out_opt, at::kBFloat16, "out");
    TORCH_CHECK(out_opt->dim() == 2 && out_opt->size(0) == M && out_opt->size(1) == N && out_opt->is_contiguous(),
                "gemm_fused: out must be a contiguous [M, N] tensor");
    TORCH_CHECK((uintptr_t)out_opt->data_ptr() % 16 == 0, "gemm_fused: out must be 16-byte aligned");
    out = *out_opt;
  } else {
    out = at::empty({M, N}, a.options());
  }
  c10::optional<Tensor> out2;
  g.c = out.data_ptr();
  g.ldc = (int)N;
  if (bias.has_value() && !has_u) {
    check_gpu(*bias, "bias");
    check_dtype(*bias, at::kBFloat16, "bias");
    TORCH_CHECK(bias->numel() == N, "gemm_fused: bias must have N elements");
    TORCH_CHECK((uintptr_t)bias->data_ptr() % 4 == 0, "gemm_fused: bias must be 4-byte aligned");
    g.bias = bias->data_ptr();
  }
  if (gelu_out) {
    out2 = at::empty({M, N}, a.options());
    g.c2 = out2->data_ptr();
  }
  if (epilogue == 3) {
    TORCH_CHECK(seq_len > 0 && M % seq_len == 0 && N % 64 == 0, "gemm_fused: epilogue 3 needs seq_len | M, 64 | N");
    out2 = at::empty({M / seq_len, N / 64, seq_len}, a.options().dtype(at::kFloat));
    g.delta = out2->data_ptr<float>();
    g.T = (int)seq_len;
  }
  if (has_u) {
    TORCH_CHECK(u.has_value(), "gemm_fused: epilogue 2/3 needs u");
    check_gpu(*u, "u");
    check_dtype(*u, at::kBFloat16, "u");
    TORCH_CHECK(u->dim() == 2 && u->size(0) == M && u->size(1) == N, "gemm_fused: u must be [M, N]");
    TORCH_CHECK((uintptr_t)u->data_ptr() % 16 == 0, "gemm_fused: u must be 16-byte aligned");
    g.u = u->data_ptr();
    g.ldu = (int)N;
    if (dbias.has_value()) {
      check_gpu(*dbias, "dbias");
      check_dtype(*dbias, at::kFloat, "dbias");
      TORCH_CHECK(dbias->numel() == N, "gemm_fused: dbias must have N elements");
      g.dbias = dbias->data_ptr<float>();
    }
  }
  Tensor ws = workspace(a, g.dbias != nullptr ? llmt::gemm_fused_ws_floats((int)M, (int)N) : 0);
  g.ws = ws.data_ptr<float>();
  if (M > 0) check_hip(llmt::launch_gemm_fused(g, cur_stream()), "gemm_fused");
  return {out, out2};
}

// ---- optimizer -------------------------------------------------------------------------------
Tensor sumsq(const Tensor& x) {
  check_gpu(x, "x");
  check_dtype(x, at::kFloat, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor partials = at::empty({llmt::kSumsqBlocks}, x.options());
  Tensor out = at::empty({}, x.options());
  check_hip(llmt::launch_sumsq(x.data_ptr<float>(), x.numel(), partials.data_ptr<float>(), out.data_ptr<float>(),
                               cur_stream()),
            "sumsq");
  return out;
}

void adamw_flat(Tensor param, const Tensor& grad, Tensor exp_avg, Tensor exp_avg_sq, const c10::optional<Tensor>& shadow,
                double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                const c10::optional<Tensor>& grad_scale, const c10::optional<Tensor>& dyn,
                const c10::optional<Tensor>& skipped) {
  for (const Tensor* t : {static_cast<const Tensor*>(&param), &grad, static_cast<const Tensor*>(&exp_avg),
                          static_cast<const Tensor*>(&exp_avg_sq)}) {
    check_gpu(*t, "adamw buffer");
    check_dtype(*t, at::kFloat, "adamw buffer");
    TORCH_CHECK(t->numel() == param.numel(), "adamw buffers must have equal numel");
  }
  TORCH_CHECK(step >= 1, "adamw step must be >= 1");
  at::hip::HIPGuardMasqueradingAsCUDA guard(param.device());
  llmt::AdamWArgs a{};
  a.param = param.data_ptr<float>();
  a.grad = grad.data_ptr<float>();
  a.exp_avg = exp_avg.data_ptr<float>();
  a.exp_avg_sq = exp_avg_sq.data_ptr<float>();
  if (shadow.has_value()) {
    check_gpu(*shadow, "shadow");
    TORCH_CHECK(shadow->numel() >= param.numel(), "shadow too small");
    a.shadow = shadow->data_ptr();
    a.shadow_bf16 = is_lowp(*shadow, "shadow");
  }
  if (grad_scale.has_value()) {
    check_gpu(*grad_scale, "grad_scale");
    check_dtype(*grad_scale, at::kFloat, "grad_scale");
    a.grad_scale = grad_scale->data_ptr<float>();
  }
  a.n = param.numel();
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.weight_decay = (float)weight_decay;
  a.bias_correction1 = (float)(1.0 - std::pow(beta1, (double)step));
  a.bias_correction2_sqrt = (float)std::sqrt(1.0 - std::pow(beta2, (double)step));
  if (dyn.has_value()) {
    check_gpu(*dyn, "adamw dyn scalars");
    check_dtype(*dyn, at::kFloat, "adamw dyn scalars");
    TORCH_CHECK(dyn->numel() == 3 && dyn->is_contiguous(), "adamw dyn scalars: 3 contiguous floats");
    a.dyn = dyn->data_ptr<float>();
  }
  if (skipped.has_value()) {
    check_gpu(*skipped, "adamw skipped-step counters");
    check_dtype(*skipped, at::kInt, "adamw skipped-step counters");
    TORCH_CHECK(skipped->numel() == 2 && skipped->is_contiguous(), "adamw skipped-step counters: 2 contiguous int32");
    a.skipped = skipped->data_ptr<int>();
  }
  check_hip(llmt::launch_adamw_flat(a, cur_stream()), "adamw_flat");
}

// [norm, coef] of the gradient clip from the global squared norm (coef NaN when norm is not finite)
Tensor clip_coef(const Tensor& sumsq, double max_norm) {
  check_gpu(sumsq, "sumsq");
  check_dtype(sumsq, at::kFloat, "sumsq");
  TORCH_CHECK(sumsq.numel() == 1, "clip_coef: sumsq must be one float");
  at::hip::HIPGuardMasqueradingAsCUDA guard(sumsq.device());
  Tensor out = at::empty({2}, sumsq.options());
  check_hip(llmt::launch_clip_coef(sumsq.data_ptr<float>(), (float)max_norm, out.data_ptr<float>(), cur_stream()),
            "clip_coef");
  return out;
}

// {decay, step_size, bc2_sqrt} of one AdamW step exactly as adamw_flat forms them (CPU tensor): the
// host stages them into adamw_flat's `dyn` before each hipGraph replay of a captured step
Tensor adamw_stage_scalars(double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step) {
  TORCH_CHECK(step >= 1, "adamw step must be >= 1");
  llmt::AdamWArgs a{};
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.weight_decay = (float)weight_decay;
  a.bias_correction1 = (float)(1.0 - std::pow(beta1, (double)step));
  a.bias_correction2_sqrt = (float)std::sqrt(1.0 - std::pow(beta2, (double)step));
  Tensor out = at::empty({3}, at::TensorOptions().dtype(at::kFloat));
  llmt::adamw_step_scalars(a, out.data_ptr<float>());
  return out;
}

}  // namespace

TORCH_LIBRARY(llmtrain_hip, m) {
  m.def("add_layernorm_fwd(Tensor x, Tensor? delta, Tensor weight, Tensor bias, float eps, ScalarType out_dtype,"
        " float dropout_p=0., int dropout_seed=0) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("layernorm_bwd(Tensor dy, Tensor xs, Tensor mean, Tensor rstd, Tensor weight, Tensor? dresid,"
        " Tensor(a!) dweight, Tensor(b!) dbias, Tensor? dy_scale, bool want_lowp, Tensor(c!)? dproj_bias,"
        " float dropout_p=0., int dropout_seed=0, bool grad_lowp=False) -> (Tensor, Tensor)");
  m.def("layernorm_bwd_deferred(Tensor dy, Tensor xs, Tensor mean, Tensor rstd, Tensor weight, Tensor? dresid,"
        " Tensor(a!) dweight, Tensor(b!) dbias, Tensor? dy_scale, bool want_lowp, float dropout_p=0.,"
        " int dropout_seed=0, bool grad_lowp=False) -> (Tensor, Tensor, Tensor)");
  m.def("ln_param_reduce(Tensor[] parts, Tensor(a!)[] dst) -> ()");
  m.def("cross_entropy_fwd_bwd(Tensor(a!) logits, Tensor labels, int vocab, Tensor row_weight) -> Tensor");
  m.def("gelu_fwd(Tensor u) -> Tensor");
  m.def("scale(Tensor x, Tensor s) -> Tensor");
  m.def("gelu_bwd(Tensor dg, Tensor u, Tensor(a!)? dbias) -> Tensor");
  m.def("colsum_accum(Tensor dy, Tensor(a!) out) -> ()");
  m.def("embedding_fwd(Tensor ids, Tensor wte, Tensor wpe, float dropout_p=0., int dropout_seed=0,"
        " bool out_lowp=False) -> Tensor");
  m.def("embedding_bwd(Tensor dx, Tensor ids, Tensor(a!) dwte, Tensor(b!) dwpe, float dropout_p=0.,"
        " int dropout_seed=0) -> ()");
  m.def("attn_fwd(Tensor qkv, int B, int T, int H, float dropout_p=0., int dropout_seed=0,"
        " Tensor? key_bits=None) -> (Tensor, Tensor)");
  m.def("attn_bwd(Tensor dout, Tensor qkv, Tensor out, Tensor lse, int B, int T, int H, float dropout_p=0.,"
        " int dropout_seed=0, Tensor(a!)? dbias=None, Tensor? delta=None, Tensor? key_valid=None) -> Tensor");
  m.def("dropout_mask(int n, float p, int seed, Tensor like) -> Tensor");
  m.def("set_deterministic(bool on) -> ()", &set_deterministic);  // catch-all: no tensor arguments
  m.def("get_deterministic() -> bool", &get_deterministic);
  m.def("set_dropout_seed_offset(Tensor? word) -> ()", &set_dropout_seed_offset);
  m.def("wgrad_gemm_pp(Tensor dy, Tensor x, Tensor(a!) c, Tensor(b!)? bias=None, int split=0, int mode=-1) -> ()");
  m.def("wgrad_pp_plan(int M, int N, int K, int lda, int ldb, bool bias, int split=0, int mode=-1) -> int[]",
        &wgrad_pp_plan);  // catch-all: no tensor arguments
  m.def("gemm_fused(Tensor a, Tensor b, bool b_kn, int epilogue, Tensor? bias=None, Tensor? u=None,"
        " Tensor(a!)? dbias=None, int seq_len=0, Tensor(b!)? out=None) -> (Tensor, Tensor?)");
  m.def("sumsq(Tensor x) -> Tensor");
  m.def("adamw_flat(Tensor(a!) param, Tensor grad, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, Tensor(d!)? shadow,"
        " float lr, float beta1, float beta2, float eps, float weight_decay, int step, Tensor? grad_scale,"
        " Tensor? dyn=None, Tensor(e!)? skipped=None) -> ()");
  m.def("clip_coef(Tensor sumsq, float max_norm) -> Tensor");
  m.def("adamw_stage_scalars(float lr, float beta1, float beta2, float eps, float weight_decay, int step) -> Tensor",
        &adamw_stage_scalars);
}

TORCH_LIBRARY_IMPL(llmtrain_hip, CUDA, m) {
  m.impl("add_layernorm_fwd", &add_layernorm_fwd);
  m.impl("layernorm_bwd", &layernorm_bwd);
  m.impl("layernorm_bwd_deferred", &layernorm_bwd_deferred);
  m.impl("ln_param_reduce", &ln_param_reduce);
  m.impl("cross_entropy_fwd_bwd", &cross_entropy_fwd_bwd);
  m.impl("gelu_fwd", &gelu_fwd);
  m.impl("scale", &scale);
  m.impl("gelu_bwd", &gelu_bwd);
  m.impl("colsum_accum", &colsum_accum);
  m.impl("embedding_fwd", &embedding_fwd);
  m.impl("embedding_bwd", &embedding_bwd);
  m.impl("attn_fwd", &attn_fwd);
  m.impl("attn_bwd", &attn_bwd);
  m.impl("dropout_mask", &dropout_mask);
  m.impl("wgrad_gemm_pp", &wgrad_gemm_pp);
  m.impl("gemm_fused", &gemm_fused);
  m.impl("sumsq", &sumsq);
  m.impl("adamw_flat", &adamw_flat);
  m.impl("clip_coef", &clip_coef);
}
