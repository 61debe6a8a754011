// Fused softmax-cross-entropy forward + gradient, one pass over the logits (gfx950).
//
// Replaces reference models/gpt.py:256-269 (F.cross_entropy(reduction="none") + masked mean)
// and the autograd backward of that op.  The LM-head logits [M, Vp] (Vp = vocab padded to a
// multiple of 64) are read ONCE into registers — 512 threads per row, each lane holding
// ceil(Vp / 4096) 16-byte vectors — the row's log-sum-exp is reduced in the log2 domain
// (v_exp_f32 is exp2), and the row is overwritten in place with
//     dlogits = (softmax(z) - onehot(label)) * row_weight[row]      (0 for padded columns)
// so the backward never touches the logits as logits again.  At GPT-2 vocab this is one read
// and one write of 100 KB per row, i.e. HBM-bound at ~2 * M * Vp * 2 bytes.

#include "common.h"
#include "kernels.h"

namespace llmt {
namespace {

constexpr int kCeThreads = 512;
constexpr int kCeWaves = kCeThreads / 64;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ float scalar_f(bf16_raw v) { return bf2f(v); }
__device__ __forceinline__ float scalar_f(float v) { return v; }

template <typename T>
struct Vec8;
// The logits are read once and dlogits written once per step (13 GB each at 128K tokens, far past
// every cache): non-temporal vector accesses (-DLLMT_CE_NT=0 drops the hint), and __launch_bounds__
// asks for 3 workgroups (rows) per CU — 80 VGPRs instead of 82, i.e. 3 rows in flight instead of 2.
// Solo at M = 131072: 5.36 -> 4.75 ms, 4.9 -> 5.55 TB/s (profiles/r2/ce_occupancy_nt_ab.txt).
#ifndef LLMT_CE_NT
#define LLMT_CE_NT 1
#endif
template <>
struct Vec8<bf16_raw> {
  ushort8_t v;
  __device__ void load(const bf16_raw* p) {
    if (LLMT_CE_NT) v = __builtin_nontemporal_load(reinterpret_cast<const ushort8_t*>(p));
    else v = *reinterpret_cast<const ushort8_t*>(p);
  }
  __device__ float get(int i) const { return bf2f(v[i]); }
  __device__ void set(int i, float f) { v[i] = f2bf(f); }
  __device__ void store(bf16_raw* p) const {
    if (LLMT_CE_NT) __builtin_nontemporal_store(v, reinterpret_cast<ushort8_t*>(p));
    else *reinterpret_cast<ushort8_t*>(p) = v;
  }
};
template <>
struct Vec8<float> {
  float4_t a, b;
  __device__ void load(const float* p) {
    a = reinterpret_cast<const float4_t*>(p)[0];
    b = reinterpret_cast<const float4_t*>(p)[1];
  }
  __device__ float get(int i) const { return i < 4 ? a[i] : b[i - 4]; }
  __device__ void set(int i, float f) {
    if (i < 4) a[i] = f; else b[i - 4] = f;
  }
  __device__ void store(float* p) const {
    reinterpret_cast<float4_t*>(p)[0] = a;
    reinterpret_cast<float4_t*>(p)[1] = b;
  }
};

// register budget sized for 6 waves per SIMD (3 rows per CU at 80 VGPRs; 2 rows per CU measured
// no better, git history)
template <int MAXV, typename T>
__global__ __launch_bounds__(kCeThreads, 6) void ce_fwd_bwd_kernel(
    T* __restrict__ logits, const int64_t* __restrict__ labels, const float* __restrict__ row_w,
    float* __restrict__ loss, int Vp, int V) {
  __shared__ float scratch[kCeWaves];
  const long row = blockIdx.x;
  T* z = logits + row * (long)Vp;
  const int nvec = Vp >> 3;
  const int64_t label = labels[row];
  LLMT_DASSERT(label < V);  // negative = ignored row; >= V is a data bug
  const bool valid = label >= 0 && label < V;

  // Every vector load of the row is issued before the first wait: the loads are unconditional
  // (vectors past the row end re-read vector 0 and are ignored below) — a load under a divergent
  // `if` gets its own vmcnt(0) at the branch join, which had serialised the row into 13 HBM
  // round trips per thread.  The label logit is read with them (before any write).
  Vec8<T> v[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = threadIdx.x + j * kCeThreads;
    v[j].load(z + 8 * (c < nvec ? c : 0));
  }
  const float t_label = valid ? scalar_f(z[valid ? label : 0]) * kLog2e : 0.f;

  // Only the row's last vector can hold padded columns (Vp - V < 64) and only one vector holds
  // the label: both are handled per vector, so the per-element loops carry no compares.
  const int nfull = V >> 3;  // vectors with 8 real columns
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = threadIdx.x + j * kCeThreads;
    if (c < nvec) {
      if (c < nfull) {
#pragma unroll
        for (int i = 0; i < 8; ++i) m = fmaxf(m, v[j].get(i));
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (8 * c + i < V) m = fmaxf(m, v[j].get(i));
      }
    }
  }
  const float zmax = block_max<kCeWaves>(m, scratch);
  const float tmax = zmax * kLog2e;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = threadIdx.x + j * kCeThreads;
    if (c < nvec) {
      if (c < nfull) {
#pragma unroll
        for (int i = 0; i < 8; ++i) s += __builtin_amdgcn_exp2f(fmaf(v[j].get(i), kLog2e, -tmax));
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (8 * c + i < V) s += __builtin_amdgcn_exp2f(fmaf(v[j].get(i), kLog2e, -tmax));
      }
    }
  }
  const float ssum = block_sum<kCeWaves>(s, scratch);
  const float lse2 = tmax + log2f(ssum);
  const float w = valid ? row_w[row] : 0.f;
  const int label_vec = valid ? (int)(label >> 3) : -1;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = threadIdx.x + j * kCeThreads;
    if (c < nvec) {
      if (c < nfull) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[j].set(i, __builtin_amdgcn_exp2f(fmaf(v[j].get(i), kLog2e, -lse2)) * w);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          v[j].set(i, 8 * c + i < V ? __builtin_amdgcn_exp2f(fmaf(v[j].get(i), kLog2e, -lse2)) * w : 0.f);
      }
      if (c == label_vec) {  // onehot: recompute the label column exactly, then subtract
        const int i = (int)(label & 7);
        v[j].set(i, (__builtin_amdgcn_exp2f(t_label - lse2) - 1.f) * w);  // t_label: read at entry
      }
      v[j].store(z + 8 * c);
    }
  }
  if (threadIdx.x == 0) loss[row] = valid ? (lse2 - t_label) * kLn2 : 0.f;
}

template <typename T>
hipError_t launch_t(T* logits, const int64_t* labels, const float* row_w, float* loss, int M,
                    int Vp, int V, hipStream_t st) {
  const int nvec = Vp / 8;
  const int maxv = (nvec + kCeThreads - 1) / kCeThreads;
  dim3 grid(M), block(kCeThreads);
#define CE_CASE(N)                                                                               \
  case N:                                                                                        \
    hipLaunchKernelGGL((ce_fwd_bwd_kernel<N, T>), grid, block, 0, st, logits, labels, row_w, loss, \
                       Vp, V);                                                                   \
    break;
  switch (maxv) {
    CE_CASE(1) CE_CASE(2) CE_CASE(4) CE_CASE(8) CE_CASE(13) CE_CASE(16) CE_CASE(26) CE_CASE(32)
    default: {
      // round up to the next instantiated size
      if (maxv <= 4) { hipLaunchKernelGGL((ce_fwd_bwd_kernel<4, T>), grid, block, 0, st, logits, labels, row_w, loss, Vp, V); }
      else if (maxv <= 8) { hipLaunchKernelGGL((ce_fwd_bwd_kernel<8, T>), grid, block, 0, st, logits, labels, row_w, loss, Vp, V); }
      else if (maxv <= 13) { hipLaunchKernelGGL((ce_fwd_bwd_kernel<13, T>), grid, block, 0, st, logits, labels, row_w, loss, Vp, V); }
      else if (maxv <= 16) { hipLaunchKernelGGL((ce_fwd_bwd_kernel<16, T>), grid, block, 0, st, logits, labels, row_w, loss, Vp, V); }
      else if (maxv <= 26) { hipLaunchKernelGGL((ce_fwd_bwd_kernel<26, T>), grid, block, 0, st, logits, labels, row_w, loss, Vp, V); }
      else if (maxv <= 32) { hipLaunchKernelGGL((ce_fwd_bwd_kernel<32, T>), grid, block, 0, st, logits, labels, row_w, loss, Vp, V); }
      else return hipErrorInvalidValue;  // Vp > 131072
    }
  }
#undef CE_CASE
  return hipGetLastError();
}

}  // namespace

hipError_t launch_cross_entropy_fwd_bwd(void* logits, bool bf16, const int64_t* labels,
                                        const float* row_weight, float* loss, int M, int Vp,
                                        int V, hipStream_t stream) {
  if (Vp % 8 != 0 || V > Vp || M <= 0) return hipErrorInvalidValue;
  if (bf16) return launch_t((bf16_raw*)logits, labels, row_weight, loss, M, Vp, V, stream);
  return launch_t((float*)logits, labels, row_weight, loss, M, Vp, V, stream);
}

}  // namespace llmt
