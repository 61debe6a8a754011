// Host-side launch API of the llmtrain gfx950 kernels.
//
// The .hip translation units include only the HIP runtime; csrc/bindings.cpp (the only TU that
// sees torch headers) validates tensors and calls these launchers with raw device pointers and
// the current HIP stream.  All launchers are asynchronous and graph-capture safe (no
// allocation, no synchronisation).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llmt {

// ---- LayerNorm --------------------------------------------------------------------------
// Dropout site arguments (see common.h drop_keep): the site seed is already mixed with the step
// seed on the host; thr = round(p * 65536), 0 disables the mask; scale = 1 / keep probability.
struct DropoutArgs {
  uint32_t seed = 0;
  uint32_t thr = 0;
  float scale = 1.f;
  // optional device word added to `seed` at kernel entry: a hipGraph-captured step keeps its
  // captured site seeds and gets fresh masks per replay from the host-staged offset
  const uint32_t* seed_add = nullptr;
};

struct LnFwdArgs {
  const void* x;       // [M, d] residual stream (f32, or bf16 with x_bf16)
  bool x_bf16;
  const void* delta;   // [M, d] optional update added to x (bf16 or f32)
  bool delta_bf16;
  const float* w;
  const float* b;
  void* xs_out;        // [M, d] x + delta, x's dtype (only written when delta != nullptr)
  void* y;             // [M, d] normalised output (bf16 or f32)
  bool y_bf16;
  float* mean;         // [M]
  float* rstd;         // [M]
  int M, d;
  float eps;
  DropoutArgs dropout;  // applied to delta before the add (residual-branch dropout)
};
hipError_t launch_add_layernorm_fwd(const LnFwdArgs& a, hipStream_t stream);

struct LnBwdArgs {
  const void* dy;      // [M, d] (bf16 or f32)
  bool dy_bf16;
  const void* xs;        // [M, d] saved residual (f32, or bf16 with xs_bf16)
  bool xs_bf16;
  const float* mean;
  const float* rstd;
  const float* w;
  const void* dresid;    // optional [M, d] gradient added to dx (the gradient stream's dtype)
  bool grad_bf16;        // residual-gradient stream (dresid, dx) in bf16 instead of f32
  const float* dy_scale; // optional device scalar multiplying dy
  void* dx;              // [M, d]
  void* dx_lp;           // optional [M, d] copy of dx in dy's dtype
  float* dw;             // [d] accumulated
  float* db;             // [d] accumulated
  float* dproj;          // optional [d] accumulated column sum of dx
  int M, d;
  DropoutArgs dropout;   // mask of the branch that fed this stream: applied to dx_lp and dproj
  float* ws;             // layernorm_bwd_ws_floats(*this) floats: partial rows of dw / db / dproj
  bool defer_params;     // leave the dw / db partial rows in ws (layernorm_bwd_grid rows each) for a
                         // later batched reduce (launch_colsum_reduce_multi) instead of reducing now
};
// partial rows per accumulated parameter vector (the backward's grid)
int layernorm_bwd_grid(const LnBwdArgs& a);
// dw, db, dproj are reduced over rows through per-workgroup partial rows in `ws` and a fixed-order
// reduce (no atomics); the workspace size depends on M, d, the dtypes and whether dproj is set
long layernorm_bwd_ws_floats(const LnBwdArgs& a);
hipError_t launch_layernorm_bwd(const LnBwdArgs& a, hipStream_t stream);

// ---- softmax cross-entropy (forward + in-place gradient) --------------------------------
// logits [M, Vp] bf16 (or f32), labels [M] int64, row_weight [M] f32 -> loss [M] f32;
// logits are overwritten with (softmax - onehot) * row_weight (0 beyond column V).
hipError_t launch_cross_entropy_fwd_bwd(void* logits, bool bf16, const int64_t* labels,
                                        const float* row_weight, float* loss, int M, int Vp,
                                        int V, hipStream_t stream);

// ---- elementwise / reductions -----------------------------------------------------------
// y = x * scale[0] (device scalar), fp32 math, bf16 or fp32 storage; n % 8 == 0
hipError_t launch_scale(const void* x, void* y, const float* scale, bool bf16, long long n, hipStream_t stream);
hipError_t launch_gelu_fwd(const void* u, void* g, bool bf16, long long n, hipStream_t stream);
// du = dg * gelu'(u); dbias (optional, [F]) += colsum(du); tensors are [M, F].  The column sums go
// through partial rows in `ws` (colwise_ws_floats(M, F) floats, required with dbias) and a
// fixed-order reduce.
long colwise_ws_floats(int M, int N);
hipError_t launch_gelu_bwd(const void* dg, const void* u, void* du, float* dbias, float* ws, bool bf16,
                           int M, int F, hipStream_t stream);
// out[N] += colsum(dy[M, N]); ws: colwise_ws_floats(M, N) floats
hipError_t launch_colsum_accum(const void* dy, bool bf16, float* out, float* ws, int M, int N,
                               hipStream_t stream);
// x[b*T+t] = wte[ids] + wpe[t]
// x = dropout(wte[ids] + wpe[t]); the backward applies the same mask to dx before the scatter
hipError_t launch_embedding_fwd(const int64_t* ids, const float* wte, const float* wpe, void* x, bool x_bf16,
                                int B, int T, int d, int V, DropoutArgs dropout, hipStream_t stream);
// dx: the residual-stream gradient [B*T, d], fp32 or (dx_bf16) bf16
hipError_t launch_embedding_bwd(const void* dx, bool dx_bf16, const int64_t* ids, float* dwte, float* dwpe,
                                int B, int T, int d, int V, DropoutArgs dropout, hipStream_t stream);
// keep-mask of elements 0..n-1 of one dropout site (tests)
hipError_t launch_dropout_mask(DropoutArgs dropout, bool* out, long long n, hipStream_t stream);

// ---- fixed-order column sums (csrc/reduce.hip) ------------------------------------------
// Producers write one partial row per workgroup, parts[p][c] (p < nparts), with plain
// stores; launch_colsum_reduce adds sum_p parts[p][c] to dst in a fixed order (bitwise
// reproducible, no contended atomics).  `scratch` holds colsum_scratch_floats(nparts, ncols)
// floats (none for nparts <= 256).  dst is a [rows][row_len] view with leading dimension
// dst_ld (row_len <= 0: dst is contiguous, ncols long).
long colsum_scratch_floats(int nparts, long ncols);
hipError_t launch_colsum_reduce(const float* parts, int nparts, long ncols, float* dst, float* scratch,
                                hipStream_t stream, int row_len = 0, long dst_ld = 0);
// njobs (<= 4) reductions of the same nparts x ncols shape in one launch per level; `scratch`
// holds njobs * colsum_scratch_floats(nparts, ncols) floats
hipError_t launch_colsum_reduce_multi(const float* const* parts, float* const* dst, int njobs, int nparts, long ncols,
                                      float* scratch, hipStream_t stream, int row_len = 0, long dst_ld = 0);
// Process-wide deterministic mode (run.deterministic): the weight-gradient GEMM reduces its split-K
// partial tiles in a fixed order instead of with atomics (the other reductions always do).
void set_deterministic(bool on);
bool deterministic();
// dwte[v] += sum of dx[order[j]] over the run of sorted_ids == v (stable sort of the tokens):
// one writer per row, fixed order — the deterministic form of launch_embedding_bwd's scatter.
hipError_t launch_embedding_bwd_sorted(const void* dx, bool dx_bf16, const int64_t* sorted_ids, const int64_t* order,
                                       float* dwte, int M, int d, int V, DropoutArgs dropout, hipStream_t stream);

// ---- optimizer ---------------------------------------------------------------------------
struct AdamWArgs {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  void* shadow;          // optional compute copy (bf16 or f32), first n elements written
  bool shadow_bf16;
  const float* grad_scale;  // optional device scalar
  long long n;
  float lr, beta1, beta2, eps, weight_decay;
  float bias_correction1, bias_correction2_sqrt;
  // optional device [decay, step_size, bc2_sqrt]: per-step scalars staged by the host before a
  // hipGraph replay of the training step (the by-value ones above would be baked into the graph)
  const float* dyn;
  // optional device int32 {total, consecutive} skipped-step counters; a non-finite *grad_scale
  // skips the update (nothing written) and bumps both, an applied step resets the second
  int* skipped;
};
hipError_t launch_adamw_flat(const AdamWArgs& a, hipStream_t stream);
// the three per-step scalars exactly as launch_adamw_flat forms them: {decay, step_size, bc2_sqrt}
void adamw_step_scalars(const AdamWArgs& a, float out[3]);
// out (device scalar) = sum(x^2); `partials` must hold kSumsqBlocks floats
constexpr int kSumsqBlocks = 1024;
hipError_t launch_sumsq(const float* x, long long n, float* partials, float* out,
                        hipStream_t stream);
// out[0] = sqrt(*sumsq) (global gradient norm), out[1] = min(1, max_norm / (out[0] + 1e-6)), NaN
// when the norm is not finite (the AdamW kernels then skip the step)
hipError_t launch_clip_coef(const float* sumsq, float max_norm, float* out, hipStream_t stream);

// Ping-pong weight-gradient GEMM (gemm_wgrad_pp.hip): C[N,K] += dy^T x and, with `bias`,
// bias[N] += colsum(dy).  `ws` holds wgrad_pp_ws_floats(...) floats (split slabs + bias parts).
// mode: -1 auto, 0 slabs + fixed-order reduce, 2 fp32 atomics (ignored in deterministic mode);
// mode + 8 (7, 8, 10): 256 x 256 tiles only, without the K-tail strips / operand swap (A/B timing).
// split: 0 planned; else the 256 x 256 tiles' split + 65536 x the strips' split (0 = planned).
long wgrad_pp_ws_floats(int lda, int ldb, int M, int N, int K, int split, int mode, bool bias);
// the plan launch_wgrad_pp takes: {swap, then per family (256x256, strips): tiles, split, rows per
// chunk, epilogue mode, workgroups; modelled ns}; returns the count written (12) or 0
int wgrad_pp_plan_info(int lda, int ldb, int M, int N, int K, bool bias, int split, int mode, long* out);
hipError_t launch_wgrad_pp(const void* dy, int lda, const void* x, int ldb, float* c, int ldc, int M, int N, int K,
                           int split, int mode, float* ws, float* bias, hipStream_t stream);
// ---- forward / data-gradient GEMM with fused epilogues (bf16 in, fp32 accumulate, bf16 out)
// C[M, N] = epi(A[M, K] . op(B)); B is [N, ldb] (K contiguous, b_kn = false) or [K, ldb]
// (N contiguous, b_kn = true).  epilogue 0: C = acc + bias (bias optional);
// 1: C = acc + bias (pre-activation), c2 = gelu(C); 2: C = acc * gelu'(u), dbias += colsum(C).
// c2 shares C's leading dimension.  K % 64 == 0, K >= 256, N % 8 == 0, leading dimensions % 8 == 0.
struct GemmFusedArgs {
  const void* a = nullptr;
  int lda = 0;
  const void* b = nullptr;
  int ldb = 0;
  bool b_kn = false;
  void* c = nullptr;
  int ldc = 0;
  void* c2 = nullptr;
  const void* bias = nullptr;
  const void* u = nullptr;
  int ldu = 0;
  float* dbias = nullptr;
  float* ws = nullptr;     // with dbias: gemm_fused_ws_floats(M, N) floats of partial column sums
  float* delta = nullptr;  // epilogue 3: per-head row dot products of C and U, [M / T, N / 64, T]
  int T = 0;               // epilogue 3: rows per sequence
  int M = 0, N = 0, K = 0;
  int epilogue = 0;
};
hipError_t launch_gemm_fused(const GemmFusedArgs& args, hipStream_t stream);

inline long gemm_fused_ws_floats(int M, int N) {
  const int nparts = (M + 127) / 128;
  return (long)nparts * N + colsum_scratch_floats(nparts, N);
}

// ---- causal flash attention (head_dim <= 64, multiple of 8) ------------------------------
// Shape + options shared by the forward and backward launchers.  The kernels are specialised for
// head_dim 64 (GPT-2 124M/XL); any other multiple of 8 up to 64 (the reference presets' 32 and
// 48) runs the same kernels with the missing head dims zero-filled in LDS/registers.  The optional
// key-padding mask (reference models/gpt.py:60-64) excludes keys from the softmax; a query row
// whose every causal key is masked gets O = 0 and lse = +inf (P = 0 in the backward).
struct AttnDims {
  int B = 0, T = 0, H = 0;
  int hd = 64;                         // head dim
  float scale = 0.125f;                // softmax scale, 1/sqrt(hd)
  const uint64_t* key_bits = nullptr;  // fwd mask: [B, ceil(T/64)] words, bit j of word w = key 64w+j valid
  const uint8_t* key_valid = nullptr;  // bwd mask: [B, T], nonzero = key valid
};
// qkv [B, T, 3, H, hd] bf16 (the packed projection output), out [B, T, H, hd] bf16,
// lse [B, H, T] f32 (natural-log normaliser).
// `dropout` masks the attention probabilities (element (b, h, q, k) of the site: plane seed
// mix32(seed + (b*H + h) * 0x9E3779B9), index q*T + k); lse stays the undropped normaliser
hipError_t launch_attn_fwd(const void* qkv, void* out, float* lse, const AttnDims& dims, DropoutArgs dropout,
                           hipStream_t stream);
// dqkv [B, T, 3, H, hd] bf16; optional `dbias` [3*H*hd] f32 accumulates the column sums of dqkv
// (the qkv projection's bias gradient); `delta` [B, H, T] f32 and `dq_part`
// (attn_bwd_workspace_floats(B, T, H) floats) scratch
long attn_bwd_workspace_floats(int B, int T, int H, int hd = 64);
// delta_ready: `delta` already holds rowsum(dO * O) (the out-proj dX GEMM's epilogue 3, which
// then also added the V part of `dbias`): the delta pass is skipped
// `bias_ws` (attn_bwd_bias_ws_floats(B, T, H, hd) floats; required with `dbias`) holds the
// partial rows of the bias column sums, reduced in a fixed order (launch_colsum_reduce)
long attn_bwd_bias_ws_floats(int B, int T, int H, int hd);
hipError_t launch_attn_bwd(const void* dout, const void* qkv, const void* out, const float* lse,
                           void* dqkv, float* delta, float* dq_part, float* dbias, float* bias_ws,
                           const AttnDims& dims, DropoutArgs dropout, hipStream_t stream, bool delta_ready = false);

}  // namespace llmt
