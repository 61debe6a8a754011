// Memory-bound kernels of the fused GPT step (gfx950): exact-erf GELU forward/backward with the
// fc-bias gradient fused in, bias-gradient column sums, token+position embedding forward and
// backward.  Every global access is a 16-byte vector per lane (Guideline 13).
//
// Reference call sites: models/gpt.py:94-95/:102-103 (nn.GELU, exact erf), :176-179 (token and
// position embeddings; gradient of the tied [V, d] table), Linear bias gradients.

#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace llmt {
namespace {

constexpr float kInvSqrt2 = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;

// Exact-erf GELU (nn.GELU() default) with a cheap erf: Abramowitz & Stegun 7.1.26,
// |erf error| < 1.5e-7 absolute — it enters GELU and its derivative only through (1 + erf), far
// below the bf16 rounding of the kernels' outputs — at one v_rcp_f32, one v_exp_f32 and five FMAs
// instead of ocml's erff.  e = exp(-u^2/2) is shared between erf(u/sqrt2) and the pdf term.
struct ErfPdf {
  float erf;  // erf(u / sqrt 2)
  float e;    // exp(-u^2 / 2)
};
__device__ __forceinline__ ErfPdf erf_pdf(float u) {
  constexpr float kLog2e = 1.4426950408889634f;
  const float az = fabsf(u) * kInvSqrt2;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-0.5f * kLog2e * u * u);
  return {copysignf(fmaf(-p * t, e, 1.f), u), e};
}
__device__ __forceinline__ float gelu(float u) { return 0.5f * u * (1.f + erf_pdf(u).erf); }
__device__ __forceinline__ float gelu_grad(float u) {
  const ErfPdf ep = erf_pdf(u);
  return fmaf(0.5f, 1.f + ep.erf, u * kInvSqrt2Pi * ep.e);
}

// 8-wide load/store of either dtype as f32
template <bool BF16>
__device__ __forceinline__ void ld8(const void* base, long i8, float* f) {
  if (BF16) {
    unpack8(reinterpret_cast<const ushort8_t*>(base)[i8], f);
  } else {
    const float4_t* p = reinterpret_cast<const float4_t*>(base) + 2 * i8;
    float4_t a = p[0], b = p[1];
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
    f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
  }
}
template <bool BF16>
__device__ __forceinline__ void st8(void* base, long i8, const float* f) {
  if (BF16) {
    reinterpret_cast<ushort8_t*>(base)[i8] = pack8(f);
  } else {
    float4_t* p = reinterpret_cast<float4_t*>(base) + 2 * i8;
    p[0] = float4_t{f[0], f[1], f[2], f[3]};
    p[1] = float4_t{f[4], f[5], f[6], f[7]};
  }
}

// GELU forward, one tile of 4 x 256 vectors per workgroup (no grid stride): each thread issues its
// four 16-byte loads before the first wait and the grid is large enough that the dispatcher keeps
// every CU full (vs the earlier grid-stride kernel, solo at 131072 x 3072 bf16: 0.335 -> 0.279 ms,
// 4.8 -> 5.8 TB/s, profiles/r2/gelu_tiled_ab.txt)
template <bool BF16>
__global__ __launch_bounds__(256) void gelu_fwd_tiled_kernel(const void* __restrict__ u, void* __restrict__ g,
                                                             long n8) {
  constexpr int kU = 4;
  const long base = (long)blockIdx.x * (256 * kU) + threadIdx.x;
  float f[kU][8];
#pragma unroll
  for (int k = 0; k < kU; ++k) {
    const long i = base + k * 256;
    // unconditional: a load under a divergent if waits alone.  Non-temporal: u is next read in the
    // backward, while g is read by the next GEMM and should keep the cache
    if (BF16) unpack8(__builtin_nontemporal_load(reinterpret_cast<const ushort8_t*>(u) + (i < n8 ? i : 0)), f[k]);
    else ld8<BF16>(u, i < n8 ? i : 0, f[k]);
  }
#pragma unroll
  for (int k = 0; k < kU; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) f[k][e] = gelu(f[k][e]);
  if ((long)(blockIdx.x + 1) * (256 * kU) <= n8) {  // wave-uniform: full tile, stores unguarded
#pragma unroll
    for (int k = 0; k < kU; ++k) st8<BF16>(g, base + k * 256, f[k]);
  } else {
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const long i = base + k * 256;
      if (i < n8) st8<BF16>(g, i, f[k]);
    }
  }
}

// y = x * (*scale) with the scale read from device memory (an autograd upstream gradient: no
// host sync), fp32 math, one rounding: replaces x.float() * s -> .to(bf16) (three passes).
template <bool BF16>
__global__ __launch_bounds__(256) void scale_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                    const float* __restrict__ scale, long n8) {
  const float s = *scale;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float f[8];
    ld8<BF16>(x, i, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] *= s;
    st8<BF16>(y, i, f);
  }
}

// Column-tiled [M, F] pass: a workgroup owns 64 column-vectors (512 columns) and a strip of rows;
// its 4 waves split the strip, keep 8 f32 column partials per lane, reduce through LDS and add
// one f32 atomic per column.  OP 0 = gelu backward (+ optional dbias), OP 1 = column sum only.
template <int OP, bool BF16>
__global__ __launch_bounds__(256) void colwise_kernel(const void* __restrict__ a, const void* __restrict__ u,
                                                      void* __restrict__ out, float* __restrict__ colsum,
                                                      int M, int F8, int rows_per_block) {
  __shared__ float part[4][64 * 8 + 4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int cv = blockIdx.x * 64 + lane;  // column-vector index
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // UNROLL rows per iteration: their loads are all issued before the first use, so each wave keeps
  // UNROLL x (1 or 2) 1-KiB requests in flight instead of one (memory-level parallelism).
  constexpr int UNROLL = 4;
  auto row_op = [&](float* x, const float* uu, long i8) {
    if (OP == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] *= gelu_grad(uu[k]);
      if (BF16) {  // round first so dbias sums exactly what the next GEMM consumes
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = bf2f(f2bf(x[k]));
      }
      st8<BF16>(out, i8, x);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += x[k];
  };
  if (cv < F8) {
    int r = r0 + wid;
    for (; r + 4 * (UNROLL - 1) < r1; r += 4 * UNROLL) {
      float x[UNROLL][8], uu[UNROLL][8];
#pragma unroll
      for (int q = 0; q < UNROLL; ++q) {
        const long i8 = (long)(r + 4 * q) * F8 + cv;
        ld8<BF16>(a, i8, x[q]);
        if (OP == 0) ld8<BF16>(u, i8, uu[q]);
      }
#pragma unroll
      for (int q = 0; q < UNROLL; ++q) row_op(x[q], uu[q], (long)(r + 4 * q) * F8 + cv);
    }
    for (; r < r1; r += 4) {
      float x[8], uu[8];
      const long i8 = (long)r * F8 + cv;
      ld8<BF16>(a, i8, x);
      if (OP == 0) ld8<BF16>(u, i8, uu);
      row_op(x, uu, i8);
    }
  }
  if (colsum == nullptr) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) part[wid][lane * 8 + k] = acc[k];
  __syncthreads();
  // this row block's partial column sums (one row of `colsum` = [gridDim.y][F8 * 8] partials,
  // summed in a fixed order by launch_colsum_reduce: no atomics)
  for (int i = threadIdx.x; i < 64 * 8; i += 256) {
    const int col = blockIdx.x * 512 + i;
    if (col < F8 * 8) colsum[(long)blockIdx.y * F8 * 8 + col] = part[0][i] + part[1][i] + part[2][i] + part[3][i];
  }
}

// one wave per token row; float4 chunks; OUT_BF16: the residual stream starts in bf16 (the engine's
// bf16 residual option), the sum and the dropout scale stay fp32 in registers
template <bool OUT_BF16>
__global__ __launch_bounds__(256) void embedding_fwd_kernel(const int64_t* __restrict__ ids,
                                                            const float* __restrict__ wte,
                                                            const float* __restrict__ wpe,
                                                            void* __restrict__ x, int M, int T,
                                                            int d, int V, DropoutArgs dr) {
  resolve_dropout(dr);
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int lane = threadIdx.x & 63;
  long tok = ids[row];
  LLMT_DASSERT(tok >= 0 && tok < V);              // debug build: report bad token ids
  tok = tok < 0 ? 0 : (tok >= V ? V - 1 : tok);  // release: clamp, never read out of bounds
  const int t = (int)(row % T);
  const float4_t* e = reinterpret_cast<const float4_t*>(wte + tok * (long)d);
  const float4_t* p = reinterpret_cast<const float4_t*>(wpe + (long)t * d);
  for (int c = lane; c < (d >> 2); c += 64) {
    float4_t v = e[c] + p[c];
    if (dr.thr != 0) {  // embedding dropout (reference gpt.py:179 self.drop)
      const uint64_t e0 = (uint64_t)row * d + 4 * c;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = drop_keep(dr.seed, dr.thr, e0 + k) ? v[k] * dr.scale : 0.f;
    }
    if (OUT_BF16) {
      ushort4_t ov;
      ov[0] = f2bf(v[0]); ov[1] = f2bf(v[1]); ov[2] = f2bf(v[2]); ov[3] = f2bf(v[3]);
      reinterpret_cast<ushort4_t*>(static_cast<bf16_raw*>(x) + row * (long)d)[c] = ov;
    } else {
      reinterpret_cast<float4_t*>(static_cast<float*>(x) + row * (long)d)[c] = v;
    }
  }
}

// dwte[ids[row]] += dx[row]: each wave adds one contiguous row (256-B wave segments, the
// full-rate atomic shape on MI355X).  dx is the residual-stream gradient, fp32 or bf16 (read as is:
// no widening pass).
template <typename TX>
__global__ __launch_bounds__(256) void embedding_bwd_tok_kernel(const TX* __restrict__ dx,
                                                                const int64_t* __restrict__ ids,
                                                                float* __restrict__ dwte, int M,
                                                                int d, int V, DropoutArgs dr) {
  resolve_dropout(dr);
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int lane = threadIdx.x & 63;
  const long tok = ids[row];
  LLMT_DASSERT(tok >= 0 && tok < V);
  if (tok < 0 || tok >= V) return;
  const TX* src = dx + row * (long)d;
  float* dst = dwte + tok * (long)d;
  for (int c = lane; c < d; c += 64) {
    float g = to_f32(src[c]);
    if (dr.thr != 0) g = drop_keep(dr.seed, dr.thr, (uint64_t)row * d + c) ? g * dr.scale : 0.f;
    atomicAdd(dst + c, g);
  }
}

// dwpe[t] += sum_b dx[b, t]: one thread per (t, 4-column chunk), no atomics.
template <typename TX>
__global__ __launch_bounds__(256) void embedding_bwd_pos_kernel(const TX* __restrict__ dx,
                                                                float* __restrict__ dwpe, int B,
                                                                int T, int d, DropoutArgs dr) {
  resolve_dropout(dr);
  const int d4 = d >> 2;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)T * d4) return;
  const int t = (int)(idx / d4), c = (int)(idx % d4);
  float4_t acc = {0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < B; ++b) {
    const long row = (long)b * T + t;
    float4_t g = load4_f32(dx + row * d + 4 * c);
    if (dr.thr != 0) {
      const uint64_t e0 = (uint64_t)row * d + 4 * c;
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] = drop_keep(dr.seed, dr.thr, e0 + k) ? g[k] * dr.scale : 0.f;
    }
    acc += g;
  }
  reinterpret_cast<float4_t*>(dwpe + (long)t * d)[c] += acc;
}

__global__ __launch_bounds__(256) void dropout_mask_kernel(DropoutArgs dr, bool* __restrict__ out, long long n) {
  resolve_dropout(dr);
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = dr.thr == 0 || drop_keep(dr.seed, dr.thr, (uint64_t)i);
}

int rows_per_block_for(int M) {
  // ~128 row strips keep the atomic count low while giving 6-13 x 128 workgroups for F=768-3072
  int rpb = (M + 127) / 128;
  return rpb < 4 ? 4 : rpb;
}

}  // namespace

hipError_t launch_gelu_fwd(const void* u, void* g, bool bf16, long long n, hipStream_t stream) {
  if (n % 8 != 0) return hipErrorInvalidValue;
  const long n8 = n / 8;
  // tiled kernel: 0.335 (grid-stride) -> 0.279 ms at 131072 x 3072
  const long blocks = (n8 + 1023) / 1024;
  if (blocks > 0x7fffffffL) return hipErrorInvalidValue;
  if (bf16) hipLaunchKernelGGL(gelu_fwd_tiled_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, u, g, n8);
  else hipLaunchKernelGGL(gelu_fwd_tiled_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, u, g, n8);
  return hipGetLastError();
}

hipError_t launch_scale(const void* x, void* y, const float* scale, bool bf16, long long n, hipStream_t stream) {
  if (n % 8 != 0) return hipErrorInvalidValue;
  const long n8 = n / 8;
  const int grid = stride_grid(n8, 256, 256 * 16);
  if (bf16) hipLaunchKernelGGL(scale_kernel<true>, dim3(grid), dim3(256), 0, stream, x, y, scale, n8);
  else hipLaunchKernelGGL(scale_kernel<false>, dim3(grid), dim3(256), 0, stream, x, y, scale, n8);
  return hipGetLastError();
}

long colwise_ws_floats(int M, int N) {
  const int rpb = rows_per_block_for(M), nparts = (M + rpb - 1) / rpb;
  return (long)nparts * N + colsum_scratch_floats(nparts, N);
}

hipError_t launch_gelu_bwd(const void* dg, const void* u, void* du, float* dbias, float* ws, bool bf16, int M,
                           int F, hipStream_t stream) {
  if (F % 8 != 0 || (dbias != nullptr && ws == nullptr)) return hipErrorInvalidValue;
  const int F8 = F / 8, rpb = rows_per_block_for(M);
  dim3 grid((F8 + 63) / 64, (M + rpb - 1) / rpb);
  float* parts = dbias != nullptr ? ws : nullptr;
  if (bf16)
    hipLaunchKernelGGL((colwise_kernel<0, true>), grid, dim3(256), 0, stream, dg, u, du, parts, M, F8, rpb);
  else
    hipLaunchKernelGGL((colwise_kernel<0, false>), grid, dim3(256), 0, stream, dg, u, du, parts, M, F8, rpb);
  if (dbias != nullptr) return launch_colsum_reduce(parts, (int)grid.y, F, dbias, ws + (long)grid.y * F, stream);
  return hipGetLastError();
}

hipError_t launch_colsum_accum(const void* dy, bool bf16, float* out, float* ws, int M, int N, hipStream_t stream) {
  if (N % 8 != 0 || ws == nullptr) return hipErrorInvalidValue;
  const int N8 = N / 8, rpb = rows_per_block_for(M);
  dim3 grid((N8 + 63) / 64, (M + rpb - 1) / rpb);
  if (bf16)
    hipLaunchKernelGGL((colwise_kernel<1, true>), grid, dim3(256), 0, stream, dy, nullptr, nullptr, ws, M, N8, rpb);
  else
    hipLaunchKernelGGL((colwise_kernel<1, false>), grid, dim3(256), 0, stream, dy, nullptr, nullptr, ws, M, N8, rpb);
  return launch_colsum_reduce(ws, (int)grid.y, N, out, ws + (long)grid.y * N, stream);
}

hipError_t launch_embedding_fwd(const int64_t* ids, const float* wte, const float* wpe, void* x, bool x_bf16, int B,
                                int T, int d, int V, DropoutArgs dropout, hipStream_t stream) {
  if (d % 4 != 0) return hipErrorInvalidValue;
  const int M = B * T;
  if (x_bf16)
    hipLaunchKernelGGL(embedding_fwd_kernel<true>, dim3((M + 3) / 4), dim3(256), 0, stream, ids, wte, wpe, x, M, T, d,
                       V, dropout);
  else
    hipLaunchKernelGGL(embedding_fwd_kernel<false>, dim3((M + 3) / 4), dim3(256), 0, stream, ids, wte, wpe, x, M, T,
                       d, V, dropout);
  return hipGetLastError();
}

hipError_t launch_embedding_bwd(const void* dx, bool dx_bf16, const int64_t* ids, float* dwte, float* dwpe, int B,
                                int T, int d, int V, DropoutArgs dropout, hipStream_t stream) {
  if (d % 4 != 0) return hipErrorInvalidValue;
  const int M = B * T;
  const long work = (long)T * (d / 4);
  auto run = [&](auto* x) {
    using TX = std::remove_const_t<std::remove_pointer_t<decltype(x)>>;
    if (dwte != nullptr)  // nullptr: the caller scatters the token gradient itself (deterministic mode)
      hipLaunchKernelGGL(embedding_bwd_tok_kernel<TX>, dim3((M + 3) / 4), dim3(256), 0, stream, x, ids, dwte, M, d,
                         V, dropout);
    hipLaunchKernelGGL(embedding_bwd_pos_kernel<TX>, dim3((work + 255) / 256), dim3(256), 0, stream, x, dwpe, B, T,
                       d, dropout);
  };
  if (dx_bf16) run(static_cast<const bf16_raw*>(dx));
  else run(static_cast<const float*>(dx));
  return hipGetLastError();
}

hipError_t launch_dropout_mask(DropoutArgs dropout, bool* out, long long n, hipStream_t stream) {
  hipLaunchKernelGGL(dropout_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, dropout, out, n);
  return hipGetLastError();
}

}  // namespace llmt
