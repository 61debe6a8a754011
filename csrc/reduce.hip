// Fixed-order column sums and the deterministic embedding gradient (gfx950).
//
// Every kernel that reduces over rows into a small vector (bias gradients, LayerNorm dgamma /
// dbeta, the attention's qkv-bias gradient, split-K weight-gradient tiles in deterministic mode)
// writes ONE partial row per producing workgroup with plain stores, parts[p][c], and
// launch_colsum_reduce adds sum_p parts[p][c] to dst[c] in a fixed order:
//  * bitwise reproducible (run.deterministic: the reference asserts <= 1e-5 resume parity,
//    tests/test_checkpoint.py:301-320) — float atomics from hundreds of workgroups are not;
//  * and cheaper than contended atomics: the delta / dQ-reduce passes of the attention backward
//    sent 512-2048 atomic adds to each bias address (MI355X_MICROARCH: same-address atomics
//    serialise at the memory side).
// Two levels: groups of G ~ sqrt(nparts) parts -> scratch[g][c] (one thread per column,
// consecutive threads = consecutive columns, i.e. coalesced 256-byte rows), then the groups -> dst.
//
// embedding_bwd_sorted_kernel: dwte[v] += sum of dx rows whose token is v, over the rows in
// (stable) sorted-token order: one wave owns each run of equal tokens, so there is one writer
// per output row and a fixed summation order (the atomic scatter of elementwise.hip is the
// fast default).  Replaces the deterministic index_add of reference gpt.py:176-179's backward.
#include "common.h"
#include "kernels.h"

namespace llmt {
namespace {

constexpr int kOneLevel = 64;  // up to this many parts: one pass straight into dst

// parts summed per first-level thread: ~sqrt(nparts), a multiple of 8, so two levels always do
int group_size(int nparts) {
  int g = 8;
  while ((long)g * g < nparts) g += 8;
  return g;
}

// out[g][c] (+)= sum_{p in group g} parts[p][c]; `accumulate` adds into out (the final level)
__global__ __launch_bounds__(256) void colsum_parts_kernel(const float* __restrict__ parts, int nparts, int group,
                                                           long ncols, float* __restrict__ out, int row_len,
                                                           long out_ld, bool accumulate) {
  const long c = (long)blockIdx.x * 256 + threadIdx.x;
  if (c >= ncols) return;
  const int g = blockIdx.y;
  const int p0 = g * group, p1 = min(nparts, p0 + group);
  float acc = 0.f;
  int p = p0;
  // 8 independent loads in flight per thread, summed in part order
  for (; p + 8 <= p1; p += 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = parts[(long)(p + i) * ncols + c];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += v[i];
  }
  for (; p < p1; ++p) acc += parts[(long)p * ncols + c];
  if (accumulate) {
    // final level: column c of a [rows][row_len] view with leading dimension out_ld
    const long dst = (c / row_len) * out_ld + c % row_len;
    out[dst] += acc;
  } else {
    out[(long)g * ncols + c] = acc;
  }
}

// rows [i0, i1) of the sorted order with equal tokens: the wave at a run's first row sums it
__global__ __launch_bounds__(256) void embedding_bwd_sorted_kernel(const float* __restrict__ dx,
                                                                   const int64_t* __restrict__ sorted_ids,
                                                                   const int64_t* __restrict__ order,
                                                                   float* __restrict__ dwte, int M, int d, int V,
                                                                   DropoutArgs dr) {
  const long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= M) return;
  const int64_t tok = sorted_ids[i];
  if (i > 0 && sorted_ids[i - 1] == tok) return;  // not the first row of its run
  if (tok < 0 || tok >= V) return;
  const int lane = threadIdx.x & 63;
  float* dst = dwte + tok * (long)d;
  for (int c0 = 0; c0 < d; c0 += 64 * 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (long j = i; j < M && sorted_ids[j] == tok; ++j) {
      const long row = order[j];
      const float* src = dx + row * (long)d;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = c0 + lane + 64 * k;
        if (c < d) {
          float g = src[c];
          if (dr.thr != 0) g = drop_keep(dr.seed, dr.thr, (uint64_t)row * d + c) ? g * dr.scale : 0.f;
          acc[k] += g;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = c0 + lane + 64 * k;
      if (c < d) dst[c] += acc[k];
    }
  }
}

bool g_deterministic = false;

}  // namespace

void set_deterministic(bool on) { g_deterministic = on; }
bool deterministic() { return g_deterministic; }

long colsum_scratch_floats(int nparts, long ncols) {
  if (nparts <= kOneLevel) return 0;
  const int g = group_size(nparts);
  return (long)((nparts + g - 1) / g) * ncols;
}

hipError_t launch_colsum_reduce(const float* parts, int nparts, long ncols, float* dst, float* scratch,
                                hipStream_t stream, int row_len, long dst_ld) {
  if (nparts <= 0 || ncols <= 0) return hipSuccess;
  if (row_len <= 0) {
    row_len = (int)ncols;
    dst_ld = ncols;
  }
  const dim3 block(256);
  const unsigned gx = (unsigned)((ncols + 255) / 256);
  if (nparts <= kOneLevel) {
    hipLaunchKernelGGL(colsum_parts_kernel, dim3(gx, 1), block, 0, stream, parts, nparts, nparts, ncols, dst, row_len,
                       dst_ld, true);
    return hipGetLastError();
  }
  if (scratch == nullptr) return hipErrorInvalidValue;
  const int g = group_size(nparts), groups = (nparts + g - 1) / g;
  hipLaunchKernelGGL(colsum_parts_kernel, dim3(gx, groups), block, 0, stream, parts, nparts, g, ncols, scratch, row_len,
                     dst_ld, false);
  hipLaunchKernelGGL(colsum_parts_kernel, dim3(gx, 1), block, 0, stream, (const float*)scratch, groups, groups, ncols,
                     dst, row_len, dst_ld, true);
  return hipGetLastError();
}

hipError_t launch_embedding_bwd_sorted(const float* dx, const int64_t* sorted_ids, const int64_t* order, float* dwte,
                                       int M, int d, int V, DropoutArgs dropout, hipStream_t stream) {
  if (M <= 0) return hipSuccess;
  hipLaunchKernelGGL(embedding_bwd_sorted_kernel, dim3((M + 3) / 4), dim3(256), 0, stream, dx, sorted_ids, order, dwte,
                     M, d, V, dropout);
  return hipGetLastError();
}

}  // namespace llmt
