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
// Workgroup = 64 columns (one per lane: coalesced 256-byte rows) x 16 waves, each wave summing a
// contiguous sixteenth of the parts in order, the sixteenths added in wave order.  Up to 2048
// parts: one pass into dst; above: groups of 128 parts -> scratch[g][c], then the groups -> dst
// (two launches).  The launches are latency-bound (12-48 workgroups, one per 64 columns) and a
// launch costs ~4 us by itself, so a lane issues a whole round of 16 loads before the first add
// and the one-pass range covers every reduce of the GPT-2 124M step (LayerNorm backward's ~1,024
// partial rows, the GEMM epilogues' M / 128, the attention's per-row-tile rows): <= 4 dependent
// load rounds in ONE launch (was 4 waves x 8 loads: two launches of up to 8 rounds above 256
// parts; 9.4 us per reduce at micro-batch 32, ~100 reduces per step).  Several same-shape reductions share one launch
// (launch_colsum_reduce_multi: LayerNorm backward's 2-3 column sums).
//
// embedding_bwd_sorted_kernel: dwte[v] += sum of dx rows whose token is v, over the rows in
// (stable) sorted-token order: one wave owns each run of equal tokens, so there is one writer
// per output row and a fixed summation order (the atomic scatter of elementwise.hip is the
// fast default).  Replaces the deterministic index_add of reference gpt.py:176-179's backward.
#include "common.h"
#include "kernels.h"

namespace llmt {
namespace {

constexpr int kStrip = 64;      // columns per workgroup: one per lane, 256-byte coalesced rows
constexpr int kWaves = 16;      // waves per workgroup, each summing a contiguous sixteenth of the parts
constexpr int kOneLevel = 2048; // up to this many parts: one pass straight into dst
constexpr int kGroup = 128;     // parts per first-level group above that (8 per wave)
constexpr int kInFlight = 16;   // loads a lane issues before it adds

// One job = one (parts, dst, scratch) triple; up to kMaxJobs jobs of the same shape share a
// launch (blockIdx.z), e.g. LayerNorm backward's dgamma / dbeta / projection-bias rows.
constexpr int kMaxJobs = 4;
struct Jobs {
  const float* parts[kMaxJobs];
  float* dst[kMaxJobs];
};

// out[g][c] (+)= sum_{p in group g} parts[p][c].  Wave w of the workgroup sums its sixteenth of
// the group's parts in order (kInFlight loads in flight per lane), they are added in wave order
// through LDS: a fixed association for a given (nparts, group), hence bitwise reproducible.
// `accumulate` (final level) adds into column c of a [rows][row_len] view with leading dimension
// out_ld; otherwise the group's sum is stored to out[g][c].
__global__ __launch_bounds__(64 * kWaves) void colsum_parts_kernel(Jobs jobs, int nparts, int group, long ncols,
                                                           int row_len, long out_ld, bool accumulate) {
  __shared__ float red[kWaves][kStrip];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long c = (long)blockIdx.x * kStrip + lane;
  const int g = blockIdx.y;
  const float* parts = jobs.parts[blockIdx.z];
  const int p0 = g * group, p1 = min(nparts, p0 + group);
  const int per = (p1 - p0 + kWaves - 1) / kWaves;
  const int w0 = min(p1, p0 + wave * per), w1 = min(p1, w0 + per);
  float acc = 0.f;
  if (c < ncols) {
    int p = w0;
    for (; p + kInFlight <= w1; p += kInFlight) {
      float v[kInFlight];
#pragma unroll
      for (int i = 0; i < kInFlight; ++i) v[i] = parts[(long)(p + i) * ncols + c];
#pragma unroll
      for (int i = 0; i < kInFlight; ++i) acc += v[i];
    }
    if (p < w1) {  // the remainder as one more round (adding 0.f past w1 leaves acc unchanged)
      float v[kInFlight];
#pragma unroll
      for (int i = 0; i < kInFlight; ++i) v[i] = p + i < w1 ? parts[(long)(p + i) * ncols + c] : 0.f;
#pragma unroll
      for (int i = 0; i < kInFlight; ++i) acc += v[i];
    }
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave != 0 || c >= ncols) return;
  float sum = red[0][lane];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) sum += red[w][lane];
  float* out = jobs.dst[blockIdx.z];
  if (accumulate) {
    out[(c / row_len) * out_ld + c % row_len] += sum;
  } else {
    out[(long)g * ncols + c] = sum;
  }
}

int num_groups(int nparts) { return nparts <= kOneLevel ? 1 : (nparts + kGroup - 1) / kGroup; }

// rows [i0, i1) of the sorted order with equal tokens: the wave at a run's first row sums it
template <typename TX>
__global__ __launch_bounds__(256) void embedding_bwd_sorted_kernel(const TX* __restrict__ dx,
                                                                   const int64_t* __restrict__ sorted_ids,
                                                                   const int64_t* __restrict__ order,
                                                                   float* __restrict__ dwte, int M, int d, int V,
                                                                   DropoutArgs dr) {
  resolve_dropout(dr);
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
      const TX* src = dx + row * (long)d;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = c0 + lane + 64 * k;
        if (c < d) {
          float g = to_f32(src[c]);
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
  return nparts <= kOneLevel ? 0 : (long)num_groups(nparts) * ncols;
}

hipError_t launch_colsum_reduce_multi(const float* const* parts, float* const* dst, int njobs, int nparts, long ncols,
                                      float* scratch, hipStream_t stream, int row_len, long dst_ld) {
  if (nparts <= 0 || ncols <= 0 || njobs <= 0) return hipSuccess;
  if (njobs > kMaxJobs) return hipErrorInvalidValue;
  if (row_len <= 0) {
    row_len = (int)ncols;
    dst_ld = ncols;
  }
  const dim3 block(64 * kWaves);
  const unsigned gx = (unsigned)((ncols + kStrip - 1) / kStrip);
  Jobs final_jobs{}, first{};
  const int groups = num_groups(nparts);
  for (int j = 0; j < njobs; ++j) {
    final_jobs.dst[j] = dst[j];
    if (groups == 1) {
      final_jobs.parts[j] = parts[j];
    } else {
      first.parts[j] = parts[j];
      first.dst[j] = scratch + (long)j * groups * ncols;
      final_jobs.parts[j] = first.dst[j];
    }
  }
  if (groups > 1) {
    if (scratch == nullptr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(colsum_parts_kernel, dim3(gx, groups, njobs), block, 0, stream, first, nparts, kGroup, ncols,
                       row_len, dst_ld, false);
  }
  const int n2 = groups == 1 ? nparts : groups;
  hipLaunchKernelGGL(colsum_parts_kernel, dim3(gx, 1, njobs), block, 0, stream, final_jobs, n2, n2, ncols, row_len,
                     dst_ld, true);
  return hipGetLastError();
}

hipError_t launch_colsum_reduce(const float* parts, int nparts, long ncols, float* dst, float* scratch,
                                hipStream_t stream, int row_len, long dst_ld) {
  return launch_colsum_reduce_multi(&parts, &dst, 1, nparts, ncols, scratch, stream, row_len, dst_ld);
}

hipError_t launch_embedding_bwd_sorted(const void* dx, bool dx_bf16, const int64_t* sorted_ids, const int64_t* order,
                                       float* dwte, int M, int d, int V, DropoutArgs dropout, hipStream_t stream) {
  if (M <= 0) return hipSuccess;
  if (dx_bf16)
    hipLaunchKernelGGL(embedding_bwd_sorted_kernel<bf16_raw>, dim3((M + 3) / 4), dim3(256), 0, stream,
                       static_cast<const bf16_raw*>(dx), sorted_ids, order, dwte, M, d, V, dropout);
  else
    hipLaunchKernelGGL(embedding_bwd_sorted_kernel<float>, dim3((M + 3) / 4), dim3(256), 0, stream,
                       static_cast<const float*>(dx), sorted_ids, order, dwte, M, d, V, dropout);
  return hipGetLastError();
}

}  // namespace llmt
