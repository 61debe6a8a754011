// Fused AdamW over the flat parameter store + global gradient sum of squares (gfx950).
//
// Replaces reference training/trainer.py:390-394 (clip_grad_norm_ + torch.optim.AdamW.step()).
// One grid-stride pass reads param/grad/exp_avg/exp_avg_sq as float4 and writes param,
// both moments AND the bf16 shadow copy of the weights used by the next forward's GEMMs
// (30 B per parameter, HBM bound).  The gradient-clipping coefficient arrives as a device
// scalar (computed from the sumsq kernel below), so clipping costs no host round trip and
// no extra pass over the gradients.  A non-finite coefficient (clip_coef_kernel below makes it NaN
// when the global gradient norm is NaN/Inf) skips the whole update on device: every workgroup
// returns before its first store, so weights, moments and shadow keep the last good step, and one
// lane bumps the skipped-step counters {total, consecutive} (no poisoned state, no
// host sync).  The update order matches torch.optim.AdamW exactly:
//   p *= 1 - lr*wd;  m += (1-b1)(g-m);  v = b2 v + (1-b2) g^2;
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)

#include "common.h"
#include "kernels.h"

namespace llmt {
namespace {

struct AdamScalars {
  float decay, one_minus_b1, b2, one_minus_b2, step_size, bc2_sqrt, eps;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamScalars& s) {
  p *= s.decay;
  m = fmaf(s.one_minus_b1, g - m, m);
  v = fmaf(s.b2, v, s.one_minus_b2 * g * g);
  const float denom = sqrtf(v) / s.bc2_sqrt + s.eps;
  p -= s.step_size * (m / denom);
}

// Non-finite clip coefficient: the step is skipped by every workgroup (uniform branch).  Block 0's
// first lane keeps the counters: skipped[0] = steps skipped in total, skipped[1] = consecutive
// skips (reset by an applied step).  Plain vector stores from one lane, no atomics.
__device__ __forceinline__ bool adamw_skip(float gs, int* __restrict__ skipped) {
  const bool skip = !isfinite(gs);
  if (skipped != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
    if (skip) {
      skipped[0] += 1;
      skipped[1] += 1;
    } else {
      skipped[1] = 0;
    }
  }
  return skip;
}

template <bool SHADOW_BF16>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ param, const float* __restrict__ grad,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    void* __restrict__ shadow,
                                                    const float* __restrict__ grad_scale, long n,
                                                    AdamScalars s, const float* __restrict__ dyn,
                                                    int* __restrict__ skipped) {
  const float gs = grad_scale != nullptr ? *grad_scale : 1.f;
  if (adamw_skip(gs, skipped)) return;
  if (dyn != nullptr) {  // graph replay: this step's scalars from device memory
    s.decay = dyn[0];
    s.step_size = dyn[1];
    s.bc2_sqrt = dyn[2];
  }
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4_t p = reinterpret_cast<float4_t*>(param)[i];
    float4_t g = reinterpret_cast<const float4_t*>(grad)[i] * gs;
    float4_t mm = reinterpret_cast<float4_t*>(m)[i];
    float4_t vv = reinterpret_cast<float4_t*>(v)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float pk = p[k], mk = mm[k], vk = vv[k];
      adam_elem(pk, g[k], mk, vk, s);
      p[k] = pk; mm[k] = mk; vv[k] = vk;
    }
    reinterpret_cast<float4_t*>(param)[i] = p;
    reinterpret_cast<float4_t*>(m)[i] = mm;
    reinterpret_cast<float4_t*>(v)[i] = vv;
    if (shadow != nullptr) {
      if (SHADOW_BF16) {
        ushort4_t o;
        o[0] = f2bf(p[0]); o[1] = f2bf(p[1]); o[2] = f2bf(p[2]); o[3] = f2bf(p[3]);
        reinterpret_cast<ushort4_t*>(shadow)[i] = o;
      } else {
        reinterpret_cast<float4_t*>(shadow)[i] = p;
      }
    }
  }
  // scalar tail (n % 4 elements)
  for (long i = (n4 << 2) + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float p = param[i], mm = m[i], vv = v[i];
    adam_elem(p, grad[i] * gs, mm, vv, s);
    param[i] = p; m[i] = mm; v[i] = vv;
    if (shadow != nullptr) {
      if (SHADOW_BF16) reinterpret_cast<bf16_raw*>(shadow)[i] = f2bf(p);
      else reinterpret_cast<float*>(shadow)[i] = p;
    }
  }
}

template <bool SHADOW_BF16>
__device__ __forceinline__ void store_shadow(void* shadow, long i, float4_t p) {
  if (SHADOW_BF16) {
    ushort4_t o;
    o[0] = f2bf(p[0]); o[1] = f2bf(p[1]); o[2] = f2bf(p[2]); o[3] = f2bf(p[3]);
    reinterpret_cast<ushort4_t*>(shadow)[i] = o;
  } else {
    reinterpret_cast<float4_t*>(shadow)[i] = p;
  }
}

// Tiled variant (default; the grid-stride kernel takes sizes not a multiple of 4): one tile of
// 2 x 256 float4 groups per workgroup, all eight loads of a thread issued before the first wait,
// no grid stride; the n % 4 tail stays with the grid-stride kernel's scalar loop (launched as a
// second, tiny kernel when present).
template <bool SHADOW_BF16>
__global__ __launch_bounds__(256) void adamw_tiled_kernel(float* __restrict__ param, const float* __restrict__ grad,
                                                          float* __restrict__ m, float* __restrict__ v,
                                                          void* __restrict__ shadow,
                                                          const float* __restrict__ grad_scale, long n4,
                                                          AdamScalars s, const float* __restrict__ dyn,
                                                          int* __restrict__ skipped) {
  constexpr int kU = 2;
  const float gs = grad_scale != nullptr ? *grad_scale : 1.f;
  if (adamw_skip(gs, skipped)) return;
  if (dyn != nullptr) {
    s.decay = dyn[0];
    s.step_size = dyn[1];
    s.bc2_sqrt = dyn[2];
  }
  const long base = (long)blockIdx.x * (256 * kU) + threadIdx.x;
  float4_t p[kU], g[kU], mm[kU], vv[kU];
#pragma unroll
  for (int k = 0; k < kU; ++k) {
    const long i0 = base + k * 256, i = i0 < n4 ? i0 : 0;
    p[k] = reinterpret_cast<const float4_t*>(param)[i];
    g[k] = reinterpret_cast<const float4_t*>(grad)[i];
    mm[k] = reinterpret_cast<const float4_t*>(m)[i];
    vv[k] = reinterpret_cast<const float4_t*>(v)[i];
  }
#pragma unroll
  for (int k = 0; k < kU; ++k) {
    g[k] = g[k] * gs;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pk = p[k][e], mk = mm[k][e], vk = vv[k][e];
      adam_elem(pk, g[k][e], mk, vk, s);
      p[k][e] = pk; mm[k][e] = mk; vv[k][e] = vk;
    }
  }
  // full tiles (all but the last workgroup): branch-free stores, grouped by buffer
  if ((long)(blockIdx.x + 1) * (256 * kU) <= n4) {
#pragma unroll
    for (int k = 0; k < kU; ++k) reinterpret_cast<float4_t*>(param)[base + k * 256] = p[k];
#pragma unroll
    for (int k = 0; k < kU; ++k) reinterpret_cast<float4_t*>(m)[base + k * 256] = mm[k];
#pragma unroll
    for (int k = 0; k < kU; ++k) reinterpret_cast<float4_t*>(v)[base + k * 256] = vv[k];
    if (shadow != nullptr) {
#pragma unroll
      for (int k = 0; k < kU; ++k) store_shadow<SHADOW_BF16>(shadow, base + k * 256, p[k]);
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < kU; ++k) {
    const long i = base + k * 256;
    if (i < n4) {
      reinterpret_cast<float4_t*>(param)[i] = p[k];
      reinterpret_cast<float4_t*>(m)[i] = mm[k];
      reinterpret_cast<float4_t*>(v)[i] = vv[k];
      if (shadow != nullptr) store_shadow<SHADOW_BF16>(shadow, i, p[k]);
    }
  }
}

constexpr int kSumsqThreads = 256;

__global__ __launch_bounds__(kSumsqThreads) void sumsq_partial_kernel(const float* __restrict__ x, long n,
                                                                      float* __restrict__ partials) {
  __shared__ float scratch[kSumsqThreads / 64];
  const long stride = (long)gridDim.x * blockDim.x;
  float acc = 0.f;
  // x may start anywhere (a bucket view of the flat gradient buffer): scalar head up to the first
  // 16-byte boundary, float4 body, scalar tail
  const long head = min(n, (long)((4 - (((unsigned long)x >> 2) & 3)) & 3));
  const long body4 = (n - head) >> 2;
  const float4_t* xb = reinterpret_cast<const float4_t*>(x + head);
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (long i = t0; i < body4; i += stride) {
    float4_t a = xb[i];
    acc += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
  }
  if (t0 < head) acc += x[t0] * x[t0];
  for (long i = head + (body4 << 2) + t0; i < n; i += stride) acc += x[i] * x[i];
  acc = block_sum<kSumsqThreads / 64>(acc, scratch);
  if (threadIdx.x == 0) partials[blockIdx.x] = acc;
}

// fixed-order final reduction: bitwise reproducible across runs
__global__ __launch_bounds__(kSumsqThreads) void sumsq_final_kernel(const float* __restrict__ partials, int n,
                                                                    float* __restrict__ out) {
  __shared__ float scratch[kSumsqThreads / 64];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partials[i];
  acc = block_sum<kSumsqThreads / 64>(acc, scratch);
  if (threadIdx.x == 0) *out = acc;
}

// {norm, coef} of clip_grad_norm_ from the global squared norm: norm = sqrt(sumsq),
// coef = min(1, max_norm / (norm + 1e-6)), and coef = NaN when norm is NaN/Inf (an Inf norm would
// otherwise give coef 0, and 0 * Inf gradients NaN), which makes the AdamW kernels skip the step.
__global__ void clip_coef_kernel(const float* __restrict__ sumsq, float max_norm, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const float norm = sqrtf(*sumsq);
  out[0] = norm;
  out[1] = isfinite(norm) ? fminf(max_norm / (norm + 1e-6f), 1.f) : __builtin_nanf("");
}

}  // namespace

void adamw_step_scalars(const AdamWArgs& a, float out[3]) {
  out[0] = 1.f - a.lr * a.weight_decay;
  out[1] = a.lr / a.bias_correction1;
  out[2] = a.bias_correction2_sqrt;
}

hipError_t launch_adamw_flat(const AdamWArgs& a, hipStream_t stream) {
  if (a.n <= 0) return hipSuccess;
  float per_step[3];
  adamw_step_scalars(a, per_step);
  AdamScalars s;
  s.decay = per_step[0];
  s.one_minus_b1 = 1.f - a.beta1;
  s.b2 = a.beta2;
  s.one_minus_b2 = 1.f - a.beta2;
  s.step_size = per_step[1];
  s.bc2_sqrt = per_step[2];
  s.eps = a.eps;
  // tiled kernel (0.75-0.78 -> 0.60 ms for 124M params); the grid-stride kernel takes sizes that
  // are not a multiple of 4
  const long n4 = (long)(a.n >> 2);
  if (n4 > 0 && (a.n & 3) == 0) {
    const long blocks = (n4 + 511) / 512;
    if (a.shadow_bf16)
      hipLaunchKernelGGL(adamw_tiled_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, a.param, a.grad,
                         a.exp_avg, a.exp_avg_sq, a.shadow, a.grad_scale, n4, s, a.dyn, a.skipped);
    else
      hipLaunchKernelGGL(adamw_tiled_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, a.param, a.grad,
                         a.exp_avg, a.exp_avg_sq, a.shadow, a.grad_scale, n4, s, a.dyn, a.skipped);
    return hipGetLastError();
  }
  const int grid = stride_grid((a.n + 3) / 4, 256, 256 * 8);
  if (a.shadow_bf16)
    hipLaunchKernelGGL(adamw_kernel<true>, dim3(grid), dim3(256), 0, stream, a.param, a.grad, a.exp_avg,
                       a.exp_avg_sq, a.shadow, a.grad_scale, (long)a.n, s, a.dyn, a.skipped);
  else
    hipLaunchKernelGGL(adamw_kernel<false>, dim3(grid), dim3(256), 0, stream, a.param, a.grad, a.exp_avg,
                       a.exp_avg_sq, a.shadow, a.grad_scale, (long)a.n, s, a.dyn, a.skipped);
  return hipGetLastError();
}

hipError_t launch_sumsq(const float* x, long long n, float* partials, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(kSumsqBlocks), dim3(kSumsqThreads), 0, stream, x, (long)n, partials);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(kSumsqThreads), 0, stream, partials, kSumsqBlocks, out);
  return hipGetLastError();
}

hipError_t launch_clip_coef(const float* sumsq, float max_norm, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(64), 0, stream, sumsq, max_norm, out);
  return hipGetLastError();
}

}  // namespace llmt
