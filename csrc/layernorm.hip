// Fused residual-add + LayerNorm forward and LayerNorm backward for gfx950.
//
// Replaces reference call sites models/gpt.py:86 (ln_1), :93 (ln_2), :142 (ln_f) and the
// residual adds at :100/:104-105.  One wave64 owns one row of width d; each lane keeps its
// ceil(d / 256) float4 chunks of the row in registers, so the statistics need no second read
// (mean and variance are two in-register passes).  Memory bound: the kernels move 12 B/elem
// (forward: x f32 + delta bf16 in, x' f32 + y bf16 out) and 16 B/elem (backward).
//
// Backward accumulates dgamma/dbeta (and optionally the column sum of dx, which is the bias
// gradient of the projection whose output was added into this residual stream) with per-lane
// register partials over a grid-stride run of rows, a cross-wave LDS reduction, then one fp32
// atomic per column per workgroup.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace llmt {
namespace {

template <typename T>
__device__ __forceinline__ float4_t load4(const T* p);
template <>
__device__ __forceinline__ float4_t load4<float>(const float* p) {
  return *reinterpret_cast<const float4_t*>(p);
}
template <>
__device__ __forceinline__ float4_t load4<bf16_raw>(const bf16_raw* p) {
  ushort4_t v = *reinterpret_cast<const ushort4_t*>(p);
  return float4_t{bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3])};
}

template <typename T>
__device__ __forceinline__ void store4(T* p, float4_t v);
template <>
__device__ __forceinline__ void store4<float>(float* p, float4_t v) {
  *reinterpret_cast<float4_t*>(p) = v;
}
template <>
__device__ __forceinline__ void store4<bf16_raw>(bf16_raw* p, float4_t v) {
  ushort4_t o;
  o[0] = f2bf(v[0]); o[1] = f2bf(v[1]); o[2] = f2bf(v[2]); o[3] = f2bf(v[3]);
  *reinterpret_cast<ushort4_t*>(p) = o;
}

// the value a bf16 store would keep (round to nearest even), as fp32
__device__ __forceinline__ float4_t round_bf16x4(float4_t v) {
  return float4_t{bf2f(f2bf(v[0])), bf2f(f2bf(v[1])), bf2f(f2bf(v[2])), bf2f(f2bf(v[3]))};
}

constexpr int kLnWaves = 4;  // rows per workgroup in the forward (per resident wave, persistent)

// MAXC = max float4 chunks per lane = ceil(d / 4 / 64); TX = storage type of the residual stream
// (x in, x + delta out): float, or bf16 for the engine's bf16 residual option, in which case the
// sum is rounded to bf16 BEFORE the statistics, so the backward's x-hat of the stored value is the
// forward's exactly (the add and the statistics themselves stay fp32 in registers)
// Rows wider than 768 columns (MAXC > 3, GPT-2 XL's d = 1600) run persistent: each wave loads
// gamma / beta once and strides over rows (M = 32768, d = 1600: 0.087 vs 0.097 ms; at d = 768 the
// one-row-per-wave launch stays ahead, 0.151 vs 0.159 ms; profiles/r6/ln/).
template <int MAXC>
constexpr bool ln_fwd_persistent() { return MAXC > 3; }

template <int MAXC, typename TD, typename TY, typename TX>
__global__ __launch_bounds__(256) void add_ln_fwd_kernel(
    const TX* __restrict__ x, const TD* __restrict__ delta, const float* __restrict__ w,
    const float* __restrict__ b, TX* __restrict__ xs_out, TY* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int M, int d, float eps, DropoutArgs dr) {
  resolve_dropout(dr);
  constexpr bool kPersist = ln_fwd_persistent<MAXC>();
  const int lane = threadIdx.x & 63;
  const int nc = d >> 2;
  float4_t ww[MAXC], bb[MAXC];
  auto load_wb = [&]() {
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int c = lane + j * 64, cc = c < nc ? c : 0;
      ww[j] = load4(w + 4 * cc);
      bb[j] = load4(b + 4 * cc);
    }
  };
  // unconditional loads (lanes past the row end read column 0 and are zeroed): a load under a
  // divergent `if` gets a vmcnt(0) at the branch join, one HBM round trip per 256-column chunk.
  // One-row launches load gamma / beta with the row (on gfx950 vmcnt also counts stores: loading
  // them after the xs stores would wait for those stores to complete).
  auto one_row = [&](long row) {
    const TX* xr = x + row * d;
    float4_t v[MAXC], dv[MAXC];
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int c = lane + j * 64, cc = c < nc ? c : 0;
      v[j] = load4(xr + 4 * cc);
    }
    if (!kPersist) load_wb();
    if (delta != nullptr) {
#pragma unroll
      for (int j = 0; j < MAXC; ++j) {
        const int c = lane + j * 64, cc = c < nc ? c : 0;
        dv[j] = load4(delta + row * d + 4 * cc);
      }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int c = lane + j * 64;
      if (delta != nullptr) {
        if (dr.thr != 0) {  // residual-branch dropout (reference gpt.py resid/mlp_dropout)
          const uint64_t e0 = (uint64_t)row * d + 4 * c;
#pragma unroll
          for (int t = 0; t < 4; ++t) dv[j][t] = drop_keep(dr.seed, dr.thr, e0 + t) ? dv[j][t] * dr.scale : 0.f;
        }
        v[j] += dv[j];
        if (!std::is_same<TX, float>::value) v[j] = round_bf16x4(v[j]);
        if (c < nc) store4(xs_out + row * d + 4 * c, v[j]);
      }
      if (c >= nc) v[j] = float4_t{0.f, 0.f, 0.f, 0.f};
      s += v[j][0] + v[j][1] + v[j][2] + v[j][3];
    }
    const float inv_d = 1.f / (float)d;
    const float mu = wave_sum(s) * inv_d;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int c = lane + j * 64;
      if (c < nc) {
        float4_t t = v[j] - mu;
        q += t[0] * t[0] + t[1] * t[1] + t[2] * t[2] + t[3] * t[3];
      }
    }
    const float rs = rsqrtf(wave_sum(q) * inv_d + eps);
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int c = lane + j * 64;
      const float4_t out = (v[j] - mu) * rs * ww[j] + bb[j];
      if (c < nc) store4(y + row * d + 4 * c, out);
    }
    if (lane == 0) {
      mean_out[row] = mu;
      rstd_out[row] = rs;
    }
  };
  const long row0 = (long)blockIdx.x * kLnWaves + (threadIdx.x >> 6);
  if constexpr (kPersist) {
    load_wb();
    for (long row = row0; row < M; row += (long)gridDim.x * kLnWaves) one_row(row);
  } else {
    if (row0 < M) one_row(row0);
  }
}

constexpr int kBwdWaves = 4;

// plain loads / stores of the residual operands (non-temporal hints measured as noise, git history)
template <typename T>
__device__ __forceinline__ float4_t load4_nt(const T* p) { return load4(p); }
template <typename T>
__device__ __forceinline__ void store4_nt(T* p, float4_t v) { store4(p, v); }

// Lean backward (rows of <= 768 columns; the split-row kernel below takes wider rows), built for
// latency hiding rather than for the fewest instructions:
//  * every load is unconditional (lanes past the row end read column 0 and are zeroed): a load
//    under a divergent `if` gets its own vmcnt(0) at the branch join, which serialised each row
//    into one HBM round trip per 256-column chunk in the earlier prefetching kernel;
//  * ROWS rows per wave per iteration, all their loads issued before the first reduction;
//  * the dproj column partial in this wave's own LDS row instead of registers (12 KB per
//    workgroup; per-wave rows keep the summation order fixed, i.e. deterministic), gamma re-read
//    from L1 at each use.
// The side stream's weight-gradient GEMM (wgrad_kernel<4,4>: 74 VGPRs + 256 AGPRs = 336 of a
// SIMD's 512) leaves 176 registers per SIMD, so what LayerNorm backward has in flight on the CUs
// that GEMM holds is bounded by load-destination registers, not by wave count.
// TX: storage type of the saved residual xs; TG: of the residual-gradient stream (dresid in, dx out):
// float, or bf16 for the engine's bf16 residual / gradient-stream options (row math stays fp32)
template <int MAXC, int ROWS, typename TDY, bool LOWP_OUT, typename TX, typename TG>
__global__ __launch_bounds__(256, ROWS == 1 ? (MAXC <= 3 ? 4 : 2) : 3) void ln_bwd_lean_kernel(
    const TDY* __restrict__ dy, const TX* __restrict__ xs, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ w, const TG* __restrict__ dresid,
    const float* __restrict__ dy_scale, TG* __restrict__ dx, TDY* __restrict__ dx_lp,
    float* __restrict__ dw, float* __restrict__ db, float* __restrict__ dproj, int M, int d, DropoutArgs dr) {
  resolve_dropout(dr);
  extern __shared__ __attribute__((aligned(16))) float smem[];  // [kBwdWaves][d]
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nc = d >> 2;
  const float scale = dy_scale != nullptr ? *dy_scale : 1.f;
  const float inv_d = 1.f / (float)d;
  const bool has_pp = dproj != nullptr;
  const float4_t zero = {0.f, 0.f, 0.f, 0.f};
  float* pp = smem + wid * d;  // this wave's dproj column partial

  float4_t pw[MAXC], pb[MAXC];
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    pw[j] = zero; pb[j] = zero;
    const int c = lane + j * 64;
    if (has_pp && c < nc) store4(pp + 4 * c, zero);
  }

  const long stride = (long)gridDim.x * kBwdWaves;
  for (long row0 = (long)blockIdx.x * kBwdWaves + wid; row0 < M; row0 += ROWS * stride) {
    // gamma through a row-dependent (always zero) offset: keeps the compiler from hoisting the
    // loop-invariant loads into 12 live registers
    const float* wr = w + __builtin_amdgcn_readfirstlane((int)(row0 >> 40));
    long rows[ROWS];
    bool live[ROWS];
    float mu[ROWS], rs[ROWS];
    float4_t g[ROWS][MAXC], xh[ROWS][MAXC], rr[ROWS][MAXC];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      live[r] = row0 + r * stride < M;  // wave-uniform
      rows[r] = live[r] ? row0 + r * stride : row0;
      mu[r] = mean[rows[r]];
      rs[r] = rstd[rows[r]];
#pragma unroll
      for (int j = 0; j < MAXC; ++j) {
        const int c = lane + j * 64, cc = c < nc ? c : 0;
        g[r][j] = load4(dy + rows[r] * d + 4 * cc);
        xh[r][j] = load4_nt(xs + rows[r] * d + 4 * cc);
      }
    }
    if (dresid != nullptr) {
#pragma unroll
      for (int r = 0; r < ROWS; ++r)
#pragma unroll
        for (int j = 0; j < MAXC; ++j) {
          const int c = lane + j * 64, cc = c < nc ? c : 0;
          rr[r][j] = load4_nt(dresid + rows[r] * d + 4 * cc);
        }
    }
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < MAXC; ++j) {
        const int c = lane + j * 64, cc = c < nc ? c : 0;
        const bool ok = live[r] && c < nc;
        g[r][j] = ok ? g[r][j] * scale : zero;
        xh[r][j] = ok ? (xh[r][j] - mu[r]) * rs[r] : zero;
        float4_t gw = g[r][j] * load4(wr + 4 * cc);
        s1 += gw[0] + gw[1] + gw[2] + gw[3];
        float4_t gx = gw * xh[r][j];
        s2 += gx[0] + gx[1] + gx[2] + gx[3];
      }
      const float c1 = wave_sum(s1) * inv_d, c2 = wave_sum(s2) * inv_d;
      const long row = rows[r];
#pragma unroll
      for (int j = 0; j < MAXC; ++j) {
        const int c = lane + j * 64, cc = c < nc ? c : 0;
        float4_t out = (g[r][j] * load4(wr + 4 * cc) - c1 - xh[r][j] * c2) * rs[r];
        if (dresid != nullptr) out += rr[r][j];
        float4_t br = out;
        if (dr.thr != 0) {
          const uint64_t e0 = (uint64_t)row * d + 4 * c;
#pragma unroll
          for (int t = 0; t < 4; ++t) br[t] = drop_keep(dr.seed, dr.thr, e0 + t) ? out[t] * dr.scale : 0.f;
        }
        pw[j] += g[r][j] * xh[r][j];  // zero past the row end and for a dead row
        pb[j] += g[r][j];
        if (live[r] && c < nc) {
          store4_nt(dx + row * d + 4 * c, out);
          if (LOWP_OUT) store4(dx_lp + row * d + 4 * c, br);
          if (has_pp) store4(pp + 4 * c, *reinterpret_cast<const float4_t*>(pp + 4 * c) + br);
        }
      }
    }
  }

  // dproj partials are already in LDS: reduce them first, then dw and db through the same buffer
  const int nacc = has_pp ? 3 : 2;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k >= nacc) break;
    const int which = has_pp ? (k == 0 ? 2 : k - 1) : k;
    if (which != 2) {  // dw / db: stage this wave's register partial (dproj is already there)
      if (k > 0) __syncthreads();  // previous round's readers are done with the buffer
#pragma unroll
      for (int j = 0; j < MAXC; ++j) {
        const int c = lane + j * 64;
        if (c < nc) store4(smem + wid * d + 4 * c, which == 0 ? pw[j] : pb[j]);
      }
    }
    __syncthreads();
    float* dst = which == 0 ? dw : (which == 1 ? db : dproj);
    for (int col = threadIdx.x; col < d; col += blockDim.x) {
      float acc = 0.f;
#pragma unroll
      for (int wv2 = 0; wv2 < kBwdWaves; ++wv2) acc += smem[wv2 * d + col];
      dst[(long)blockIdx.x * d + col] = acc;
    }
  }
}

// Split-row backward for wide rows (GPT-2 XL's d = 1600): a workgroup's 4 waves take 2 rows per
// iteration, each row split into two column halves held by two waves, so a wave keeps half a row
// (MAXC = 7 -> 4 float4 chunks per lane) and the kernel stays at <= 168 VGPRs (written for the
// round-2 side stream's weight-gradient GEMM beside it; since round 6 the wave's half of gamma also
// stays in registers instead of being re-read per row, 164 VGPRs).  The two halves' row sums meet in LDS (one barrier per row
// pair, parity double-buffered); column partials and the per-wave dproj rows are summed over the
// two row slots at the end (fixed order).
template <int MAXC, typename TDY, bool LOWP_OUT, typename TX, typename TG>
__global__ __launch_bounds__(256, 3) void ln_bwd_split_kernel(
    const TDY* __restrict__ dy, const TX* __restrict__ xs, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ w, const TG* __restrict__ dresid,
    const float* __restrict__ dy_scale, TG* __restrict__ dx, TDY* __restrict__ dx_lp,
    float* __restrict__ dw, float* __restrict__ db, float* __restrict__ dproj, int M, int d, DropoutArgs dr) {
  resolve_dropout(dr);
  constexpr int HC = (MAXC + 1) / 2;  // float4 chunks per lane for half a row
  extern __shared__ __attribute__((aligned(16))) float smem[];  // [4][d]: 0-1 staging, 2-3 dproj
  __shared__ float red[2][2][2][2];                              // [parity][slot][half][s1|s2]
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int slot = wid >> 1, half = wid & 1;
  const int nc = d >> 2, nh0 = (nc + 1) >> 1;
  const int cbase = half ? nh0 : 0, nhalf = half ? nc - nh0 : nh0;
  const float scale = dy_scale != nullptr ? *dy_scale : 1.f;
  const float inv_d = 1.f / (float)d;
  const bool has_pp = dproj != nullptr;
  const float4_t zero = {0.f, 0.f, 0.f, 0.f};
  float* pp = smem + (2 + slot) * d;  // this row slot's dproj partial (this wave's half of it)

  float4_t pw[HC], pb[HC];
  float4_t gam[HC];  // this wave's half of gamma, loaded once (XL: 0.113 -> 0.096 ms, profiles/r6/ln/)
#pragma unroll
  for (int j = 0; j < HC; ++j) {
    pw[j] = zero; pb[j] = zero;
    const int cl = lane + j * 64;
    if (has_pp && cl < nhalf) store4(pp + 4 * (cbase + cl), zero);
    gam[j] = load4(w + 4 * (cbase + (cl < nhalf ? cl : 0)));
  }

  int par = 0;
  for (long pr = blockIdx.x; 2 * pr < M; pr += gridDim.x, par ^= 1) {  // uniform over the workgroup
    const long row0 = 2 * pr + slot;
    const bool live = row0 < M;  // wave-uniform
    const long row = live ? row0 : 0;
    const float mu = mean[row], rs = rstd[row];
    float4_t g[HC], xh[HC], rr[HC];
#pragma unroll
    for (int j = 0; j < HC; ++j) {
      const int cl = lane + j * 64, c = cbase + (cl < nhalf ? cl : 0);
      g[j] = load4(dy + row * d + 4 * c);
      xh[j] = load4_nt(xs + row * d + 4 * c);
    }
    if (dresid != nullptr) {
#pragma unroll
      for (int j = 0; j < HC; ++j) {
        const int cl = lane + j * 64, c = cbase + (cl < nhalf ? cl : 0);
        rr[j] = load4_nt(dresid + row * d + 4 * c);
      }
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < HC; ++j) {
      const int cl = lane + j * 64, c = cbase + (cl < nhalf ? cl : 0);
      const bool ok = live && cl < nhalf;
      g[j] = ok ? g[j] * scale : zero;
      xh[j] = ok ? (xh[j] - mu) * rs : zero;
      float4_t gw = g[j] * gam[j];
      s1 += gw[0] + gw[1] + gw[2] + gw[3];
      float4_t gx = gw * xh[j];
      s2 += gx[0] + gx[1] + gx[2] + gx[3];
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
      red[par][slot][half][0] = s1;
      red[par][slot][half][1] = s2;
    }
    __syncthreads();
    const float c1 = (red[par][slot][0][0] + red[par][slot][1][0]) * inv_d;
    const float c2 = (red[par][slot][0][1] + red[par][slot][1][1]) * inv_d;
#pragma unroll
    for (int j = 0; j < HC; ++j) {
      const int cl = lane + j * 64, c = cbase + (cl < nhalf ? cl : 0);
      float4_t out = (g[j] * gam[j] - c1 - xh[j] * c2) * rs;
      if (dresid != nullptr) out += rr[j];
      float4_t br = out;
      if (dr.thr != 0) {
        const uint64_t e0 = (uint64_t)row * d + 4 * c;
#pragma unroll
        for (int t = 0; t < 4; ++t) br[t] = drop_keep(dr.seed, dr.thr, e0 + t) ? out[t] * dr.scale : 0.f;
      }
      pw[j] += g[j] * xh[j];  // zero past the half's end and for a dead row
      pb[j] += g[j];
      if (live && cl < nhalf) {
        store4_nt(dx + row * d + 4 * c, out);
        if (LOWP_OUT) store4(dx_lp + row * d + 4 * c, br);
        if (has_pp) store4(pp + 4 * c, *reinterpret_cast<const float4_t*>(pp + 4 * c) + br);
      }
    }
  }

  // per-workgroup partial rows: dproj (already in LDS rows 2-3), then dw and db staged in rows 0-1
  const int nacc = has_pp ? 3 : 2;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k >= nacc) break;
    const int which = has_pp ? (k == 0 ? 2 : k - 1) : k;
    __syncthreads();  // dproj rows complete / previous round's readers done
    if (which != 2) {
#pragma unroll
      for (int j = 0; j < HC; ++j) {
        const int cl = lane + j * 64;
        if (cl < nhalf) store4(smem + slot * d + 4 * (cbase + cl), which == 0 ? pw[j] : pb[j]);
      }
      __syncthreads();
    }
    const float* src = smem + (which == 2 ? 2 : 0) * d;
    float* dst = which == 0 ? dw : (which == 1 ? db : dproj);
    for (int col = threadIdx.x; col < d; col += blockDim.x)
      dst[(long)blockIdx.x * d + col] = src[col] + src[d + col];
  }
}

template <int MAXC, typename TX>
void launch_fwd_x(const LnFwdArgs& a, hipStream_t st) {
  const long wgs = (a.M + kLnWaves - 1) / kLnWaves;
  dim3 grid((unsigned)(ln_fwd_persistent<MAXC>() ? std::min<long>(wgs, 8L * device_cu_count()) : wgs)), block(256);
#define LN_FWD(TD, TY)                                                                              \
  hipLaunchKernelGGL((add_ln_fwd_kernel<MAXC, TD, TY, TX>), grid, block, 0, st, (const TX*)a.x,     \
                     (const TD*)a.delta, a.w, a.b, (TX*)a.xs_out, (TY*)a.y, a.mean, a.rstd, a.M, a.d, \
                     a.eps, a.dropout)
  if (a.delta_bf16) {
    if (a.y_bf16) LN_FWD(bf16_raw, bf16_raw); else LN_FWD(bf16_raw, float);
  } else {
    if (a.y_bf16) LN_FWD(float, bf16_raw); else LN_FWD(float, float);
  }
#undef LN_FWD
}

template <int MAXC>
void launch_fwd_c(const LnFwdArgs& a, hipStream_t st) {
  if (a.x_bf16) launch_fwd_x<MAXC, bf16_raw>(a, st);
  else launch_fwd_x<MAXC, float>(a, st);
}

// The backward kernel for this row width: the split-row kernel above 768 columns (GPT-2 XL
// same-box +0.7 % over the whole-row lean kernel, profiles/r2/ab_ln_split_xl.txt), else the lean
// kernel with one row per wave per iteration (two measured no better, git history)
template <int MAXC, typename TDY, bool LP, typename TX, typename TG>
const void* bwd_kernel_t() {
  if (MAXC > 3) return (const void*)&ln_bwd_split_kernel<MAXC, TDY, LP, TX, TG>;
  return (const void*)&ln_bwd_lean_kernel<MAXC, 1, TDY, LP, TX, TG>;
}

// residual storage combinations: 0 = fp32 xs / fp32 gradient stream, 1 = fp32 xs / bf16 gradient
// stream, 2 = bf16 xs / bf16 gradient stream (an fp32-dy backward takes only 0)
inline int res_mode(const LnBwdArgs& a) { return a.xs_bf16 ? 2 : (a.grad_bf16 ? 1 : 0); }

template <int MAXC, typename TDY, bool LP>
const void* bwd_kernel_r(int mode) {
  if (mode == 2) return bwd_kernel_t<MAXC, TDY, LP, bf16_raw, bf16_raw>();
  if (mode == 1) return bwd_kernel_t<MAXC, TDY, LP, float, bf16_raw>();
  return bwd_kernel_t<MAXC, TDY, LP, float, float>();
}

template <int MAXC>
const void* bwd_kernel(const LnBwdArgs& a) {
  const int mode = res_mode(a);
  if (a.dy_bf16) return a.dx_lp != nullptr ? bwd_kernel_r<MAXC, bf16_raw, true>(mode) : bwd_kernel_r<MAXC, bf16_raw, false>(mode);
  return a.dx_lp != nullptr ? bwd_kernel_t<MAXC, float, true, float, float>()
                            : bwd_kernel_t<MAXC, float, false, float, float>();
}

template <int MAXC>
int bwd_grid_c(const LnBwdArgs& a) {
  const size_t shm = (size_t)kBwdWaves * a.d * sizeof(float);
  // a whole number of resident waves of workgroups (a partial extra wave would be a pure tail:
  // every workgroup runs the same number of rows)
  static int resident[3][2][2] = {};
  int& per_cu = resident[res_mode(a)][a.dy_bf16 ? 1 : 0][a.dx_lp != nullptr ? 1 : 0];
  if (per_cu == 0) {
    int n = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, bwd_kernel<MAXC>(a), 256, shm);
    // one resident wave of workgroups (mb 32: 1 / 2 / 3 waves 950k / 944k / 936k tok/s, fewer
    // partial rows for the column sums; mb 128 flat: profiles/r2/ab_ln_waves_mb*.txt)
    per_cu = (n > 0 ? n : 4) * device_cu_count();
  }
  const int cap = per_cu;
  return stride_grid((long long)(a.M + kBwdWaves - 1) / kBwdWaves, 1, cap);
}

template <int MAXC>
void launch_bwd_c(const LnBwdArgs& a, hipStream_t st) {
  const size_t shm = (size_t)kBwdWaves * a.d * sizeof(float);
  const int grid = bwd_grid_c<MAXC>(a);
  float* pw = a.ws;
  float* pb = a.ws + (long)grid * a.d;
  float* pp = a.dproj != nullptr ? a.ws + 2L * grid * a.d : nullptr;
  const void* fn = bwd_kernel<MAXC>(a);
  const void* dy = a.dy;
  void* dx_lp = a.dx_lp;
  const void *xs = a.xs, *dresid = a.dresid;
  const float *mean = a.mean, *rstd = a.rstd, *w = a.w, *dy_scale = a.dy_scale;
  void* dx = a.dx;
  int M = a.M, d = a.d;
  DropoutArgs dr = a.dropout;
  void* args[] = {&dy, &xs, &mean, &rstd, &w, &dresid, &dy_scale, &dx, &dx_lp, &pw, &pb, &pp, &M, &d, &dr};
  (void)hipLaunchKernel(fn, dim3(grid), dim3(256), args, shm, st);

  if (a.defer_params) return;  // the caller reduces dw / db later, batched with other LayerNorms
  const int nacc = a.dproj != nullptr ? 3 : 2;
  float* scratch = a.ws + (long)nacc * grid * a.d;
  const float* parts[3] = {pw, pb, pp};
  float* dst[3] = {a.dw, a.db, a.dproj};
  launch_colsum_reduce_multi(parts, dst, nacc, grid, a.d, scratch, st);
}

}  // namespace

#define LN_DISPATCH(FN, ARGS, ST)                      \
  switch ((ARGS.d / 4 + 63) / 64) {                    \
    case 1: FN<1>(ARGS, ST); break;                    \
    case 2: FN<2>(ARGS, ST); break;                    \
    case 3: FN<3>(ARGS, ST); break;                    \
    case 4: FN<4>(ARGS, ST); break;                    \
    case 5: FN<5>(ARGS, ST); break;                    \
    case 6: FN<6>(ARGS, ST); break;                    \
    case 7: FN<7>(ARGS, ST); break;                    \
    case 8: FN<8>(ARGS, ST); break;                    \
    default: return hipErrorInvalidValue;              \
  }

hipError_t launch_add_layernorm_fwd(const LnFwdArgs& a, hipStream_t stream) {
  if (a.d % 4 != 0 || a.M <= 0) return hipErrorInvalidValue;
  LN_DISPATCH(launch_fwd_c, a, stream);
  return hipGetLastError();
}

hipError_t launch_layernorm_bwd(const LnBwdArgs& a, hipStream_t stream) {
  if (a.d % 4 != 0 || a.M <= 0 || a.ws == nullptr) return hipErrorInvalidValue;
  LN_DISPATCH(launch_bwd_c, a, stream);
  return hipGetLastError();
}

namespace {
template <int MAXC>
void grid_c(const LnBwdArgs& a, int& out) { out = bwd_grid_c<MAXC>(a); }
}  // namespace

int layernorm_bwd_grid(const LnBwdArgs& a) {
  if (a.d % 4 != 0 || a.M <= 0) return 0;
  int grid = 0;
  switch ((a.d / 4 + 63) / 64) {
    case 1: grid_c<1>(a, grid); break;
    case 2: grid_c<2>(a, grid); break;
    case 3: grid_c<3>(a, grid); break;
    case 4: grid_c<4>(a, grid); break;
    case 5: grid_c<5>(a, grid); break;
    case 6: grid_c<6>(a, grid); break;
    case 7: grid_c<7>(a, grid); break;
    case 8: grid_c<8>(a, grid); break;
    default: return 0;
  }
  return grid;
}

long layernorm_bwd_ws_floats(const LnBwdArgs& a) {
  if (a.d % 4 != 0 || a.M <= 0) return 0;
  int grid = 0;
  switch ((a.d / 4 + 63) / 64) {
    case 1: grid_c<1>(a, grid); break;
    case 2: grid_c<2>(a, grid); break;
    case 3: grid_c<3>(a, grid); break;
    case 4: grid_c<4>(a, grid); break;
    case 5: grid_c<5>(a, grid); break;
    case 6: grid_c<6>(a, grid); break;
    case 7: grid_c<7>(a, grid); break;
    case 8: grid_c<8>(a, grid); break;
    default: return 0;
  }
  const int nacc = a.dproj != nullptr ? 3 : 2;
  return (long)nacc * grid * a.d + (long)nacc * colsum_scratch_floats(grid, a.d);
}

}  // namespace llmt
