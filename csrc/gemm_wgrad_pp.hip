// Weight-gradient GEMM, ping-pong schedule (gfx950):  C[N, K] (f32) += A^T B
//   A = dY [M, N] bf16 row-major (lda), B = X [M, K] bf16 row-major (ldb), reduction over M.
//
// The round-3 kernels (deleted in round 5) ran one wave per SIMD: each wave issues its own LDS-DMA
// fill, its transposed fragment reads and then its MFMAs, so the matrix pipe idles whenever the
// wave waits (45 % MFMA-busy, profiles/r2/pmc_wgrad_qkv_plain.txt); the software-pipelined variant
// fixes that but needs all 512 registers.  Here each SIMD hosts TWO waves of one 512-thread
// workgroup that take turns (MI355X_MICROARCH "Two waves per SIMD"; the 256x256 8-wave GEMM
// template of the CDNA playbook): waves 0-3 ("X") and 4-7 ("Y", one barrier behind) alternate
//
//     X: [LOAD p  ] | [MFMA p  ] | [LOAD p+1] | [MFMA p+1] ...
//     Y: [MFMA p-1] | [LOAD p  ] | [MFMA p  ] | [LOAD p+1] ...
//
// so one wave's 32 MFMAs cover its partner's fragment reads, LDS-DMA issue and waits, and the
// pipe stays busy with ~200 registers per wave.  Per wave: a 128 (n) x 64 (k) output = 8 x 4
// v_mfma_f32_16x16x32_bf16 accumulators (128 AGPRs).  The 16x16x32 shape is chosen over 32x32x16
// at equal LDS traffic because the chip holds a higher clock on it (MI355X_MICROARCH, DVFS item 7).
//
// Stages of 32 reduction rows (one MFMA k-step) stream through a 2-slot LDS ring (2 x 32 KiB):
//  * register-staged fills (4 x 16 bytes per lane and stage); the buffer descriptor of a stage ends
//    at the workgroup's row chunk, so rows past it read as zero;
//  * LOAD(p) reads stage p's fragments, writes stage p+1 (loaded two phases earlier) into the other
//    slot and loads stage p+3, then waits for its own LDS operations (lgkmcnt(0)) BEFORE the
//    barrier: every wave finished reading stage p-1 (the other slot) at the barrier that precedes
//    any LOAD(p), and stage p+1 has landed everywhere before any wave reads it;
//  * both operands have the reduction index running down their rows, so fragments are read with
//    ds_read_b64_tr_b16 (two per fragment: k rows 8g..8g+3 and 8g+4..8g+7); the 32-byte column
//    segments of each 512-byte LDS row are XOR-swizzled by f(row) = (row & 3) | ((row >> 3) & 1) << 2,
//    which puts the 8 rows one 32-lane half reads on 8 distinct 32-byte bank groups (conflict-free);
//    the swizzle is applied to the per-lane DMA source address because LDS-DMA writes lane-linear.
//
// Epilogues (MODE): 0 = plain 16-byte stores of the tile into its own fp32 slab; a second pass
// (wgrad_finish_kernel) adds the split slabs to C in chunk order — deterministic, and cheaper
// than fp32 atomics at ~1.3 TB/s for these 64-256 MB of partials.  1 = C += acc read-modify-write
// (split == 1: each element has one owner, no atomics).  2 = fp32 atomics (huge outputs whose
// slabs would not pay, fast mode only).
//
// Column sums of A (bias gradients, db = dY^T 1) ride along when `bias_slab` is set: the
// workgroups of tile column 0 add one v_mfma_f32_16x16x32_bf16 per wave and stage against a ones
// operand (the wave's first two A fragments; the 4 waves of a row sweep rotate their fragment
// order so they cover 8 distinct fragments), replacing the separate column-sum launches.
//
// Replaces the autograd weight (and bias) gradients of every nn.Linear of the reference
// (models/gpt.py:27-29, 94-96, 184 via loss.backward() at training/trainer.py:386-387).
#include <algorithm>

#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

namespace llmt {
namespace wpp {

using namespace gemm;

constexpr int kThreads = 512;  // 8 waves, 2 per SIMD
constexpr int BR = 32;         // reduction rows per stage
constexpr int TW = 256;        // tile edge
constexpr int ROWB = TW * 2;   // LDS bytes per image row
constexpr int IMG = BR * ROWB; // 16 KiB per operand per stage
constexpr int SLOT = 2 * IMG;  // 32 KiB
constexpr int FA = 8, FB = 4;  // 16-wide fragments per wave: 128 (n) x 64 (k)
constexpr int NACC = FA * FB;
constexpr int SLAB_FLOATS = TW * TW;  // one tile's partial

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int swz_f(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }

__device__ __forceinline__ bf16x8 tr_read(unsigned addr) {
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(unsigned long)addr);
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(unsigned long)(addr + 4 * ROWB));
  const short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

// Buffer descriptor from provably wave-uniform inputs (readfirstlane of the base halves and the
// record count): otherwise hipcc wraps every buffer load in a waterfall loop (playbook T20), which
// also serialises them and drains vmcnt before each use.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int bytes) {
  const unsigned long a = (unsigned long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long)hi << 32) | lo), (short)0, n, 0x00020000);
}

// Fills are register-staged: in LOAD(st) each wave writes stage st+1 (loaded two phases earlier)
// into its ring slot with 16-byte lane-linear ds_write_b128 and loads stage st+3 into the freed
// registers (two register sets, stage parity).  A slot is free one phase after its last read, so two
// 32 KiB slots suffice, and half the LDS is left for other kernels' workgroups on the CU.  (Measured
// against LDS-DMA fills through a 4-slot ring: +2-4 % op level, +0.5 % in the step; the LDS-DMA op
// costs its wave ~60-185 issue cycles inside a phase that also reads fragments, docs/round4.md.)
template <int MODE>
__global__ __launch_bounds__(kThreads, 2) void wgrad_pp_kernel(
    const bf16_raw* __restrict__ A, int lda, const bf16_raw* __restrict__ B, int ldb, float* __restrict__ C,
    int ldc, int M, int N, int K, int tiles, int tiles_k, int m_chunk, int split, int nwg, float* __restrict__ slab,
    float* __restrict__ bias_slab) {
  constexpr int NS = 2;  // ring slots
  __shared__ __attribute__((aligned(16))) bf16_raw smem[NS * SLOT / 2];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave >> 2, wk = wave & 3;  // wn: 0 = X (leads), 1 = Y (one barrier behind)

  const int w = xcd_remap(blockIdx.x, nwg);  // the workgroups of one row chunk share an XCD
  const int chunk = w / tiles, tile = w - chunk * tiles;
  const int tile_n = tile / tiles_k, tile_k = tile - tile_n * tiles_k;
  const int n0 = tile_n * TW, k0 = tile_k * TW;
  const int m_begin = chunk * m_chunk;
  const int rows = min(M - m_begin, m_chunk);
  if (rows <= 0) return;  // whole workgroup, uniform
  const int nst = (rows + BR - 1) / BR;
  const bool want_bias = bias_slab != nullptr && tile_k == 0;

  // fills: this wave copies image rows 4*wave .. 4*wave+3 of A and of B (two 1-KiB pieces each);
  // lane l lands at LDS chunk (l & 31) of row 2*j + (l >> 5) and holds the source chunk whose
  // 32-byte segment is that one XOR f(row)
  int voa[2], vob[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 4 * wave + 2 * j + (lane >> 5);
    const int c = lane & 31;
    const int csrc = ((((c >> 1) ^ swz_f(row))) << 1) | (c & 1);
    voa[j] = (row * lda + n0 + 8 * csrc) * 2;
    vob[j] = (row * ldb + k0 + 8 * csrc) * 2;
  }
  const unsigned lds = (unsigned)(unsigned long)(lds_void*)smem;

  // fragment read addresses (bytes within a slot): lane (g, q, p) reads rows 8g + q (+4) at the
  // 32-byte segment (logical ^ f), bytes 8p..8p+7; A fragments are taken in an order rotated by
  // 2*wk so the bias sweep below covers distinct fragments with compile-time register indices
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int fl = q | ((g & 1) << 2);
  const unsigned rowb = (unsigned)((8 * g + q) * ROWB + 8 * p);
  unsigned ao[FA], bo[FB];
#pragma unroll
  for (int i = 0; i < FA; ++i) ao[i] = rowb + ((8 * wn + (((i + 2 * wk) & 7) ^ fl)) << 5);
#pragma unroll
  for (int j = 0; j < FB; ++j) bo[j] = IMG + rowb + (((4 * wk + j) ^ fl) << 5);

  f32x4v acc[FA][FB];
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) acc[i][j] = 0.f;
  f32x4v bacc[2] = {0.f, 0.f};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, (short8v){0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80});

  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
  u32x4 R0[4], R1[4];  // staged stage parity
  // (unconditional: a stage past the chunk has a zero-record descriptor and loads zeros — a
  // conditional load made hipcc drain every outstanding load before each LDS write)
  auto load_stage = [&](int st, u32x4 (&R)[4]) {
    const int r0 = st * BR, nr = max(0, min(BR, rows - r0));
    const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(A + (long)(m_begin + r0) * lda, nr * lda * 2);
    const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(B + (long)(m_begin + r0) * ldb, nr * ldb * 2);
    R[0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, voa[0], 0, 0));
    R[1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, voa[1], 0, 0));
    R[2] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rb, vob[0], 0, 0));
    R[3] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rb, vob[1], 0, 0));
  };
  auto write_stage = [&](int slot, const u32x4 (&R)[4]) {
    const unsigned a = lds + slot * SLOT + wave * 2048 + 16 * lane;
    *(lds_u32x4*)(size_t)a = R[0];
    *(lds_u32x4*)(size_t)(a + 1024) = R[1];
    *(lds_u32x4*)(size_t)(a + IMG) = R[2];
    *(lds_u32x4*)(size_t)(a + IMG + 1024) = R[3];
  };

  // prologue: stage 0 landed everywhere, stages 1 and 2 loading; Y then falls one barrier behind
  load_stage(0, R0);
  load_stage(1, R1);
  write_stage(0, R0);
  load_stage(2, R0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (wn == 1) barrier();

  // R: the register set of stage st+1 (= that of st+3)
  auto phase = [&](int st, int slot, u32x4 (&R)[4]) {
    // ---- LOAD(st): fragments of stage st, stage st+1 into the other slot, stage st+3 loading
    const unsigned sb = lds + slot * SLOT;
    bf16x8 af[FA], bfr[FB];
#pragma unroll
    for (int i = 0; i < FA; ++i) af[i] = tr_read(sb + ao[i]);
#pragma unroll
    for (int j = 0; j < FB; ++j) bfr[j] = tr_read(sb + bo[j]);
    // both unconditional (a slot past the last stage is never read)
    write_stage(slot ^ 1, R);
    load_stage(st + 3, R);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // ---- MFMA(st)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FA; ++i)
#pragma unroll
      for (int j = 0; j < FB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (want_bias) {
      bacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], ones, bacc[0], 0, 0, 0);
      bacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], ones, bacc[1], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    barrier();
  };
  // pairs of phases with no per-phase condition (a conditional phase made hipcc assume the loads
  // of a skipped phase were never issued and drain vmcnt early); an odd last stage is padded with a
  // stage of zeros (zero-record loads, MFMAs on zeros)
  for (int s0 = 0; s0 < nst; s0 += 2) {
    phase(s0, 0, R1);
    phase(s0 + 1, 1, R0);
  }
  if (wn == 0) barrier();  // X matches Y's extra barrier

  // ---- epilogue.  Accumulator (i, j) register r of lane l: n = n0 + 128 wn + 16 ((i + 2wk) & 7)
  // + 4 (l >> 4) + r, k = k0 + 64 wk + 16 j + (l & 15)
  if (want_bias) {
    // bacc[t][r] = column sums of logical fragment 2wk + t, rows 4g + r; identical in all 16 lanes
    // of a group (every column of the ones product), so lane (g, c) keeps row 4g + (c & 3)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int r = lane & 3;
      const float v = r == 0 ? bacc[t][0] : r == 1 ? bacc[t][1] : r == 2 ? bacc[t][2] : bacc[t][3];
      const int n = n0 + 128 * wn + 16 * (2 * wk + t) + 4 * g + r;
      // atomic epilogue (fast mode): straight into the bias vector; otherwise this chunk's row
      if ((lane & 15) < 4 && n < N) {
        if (MODE == 2) atomicAdd(bias_slab + n, v);
        else bias_slab[(long)chunk * N + n] = v;
      }
    }
  }
  if (MODE == 0) {
    float* s = slab + ((long)(tile * split + chunk) * 8 + wave) * (NACC * 64 * 4);
#pragma unroll
    for (int i = 0; i < FA; ++i)
#pragma unroll
      for (int j = 0; j < FB; ++j) *(f32x4v*)(s + ((i * FB + j) * 64 + lane) * 4) = acc[i][j];
  } else {
    const int kc = k0 + 64 * wk + (lane & 15);
#pragma unroll
    for (int i = 0; i < FA; ++i) {
      const int nb = n0 + 128 * wn + 16 * ((i + 2 * wk) & 7) + 4 * g;
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        const int k = kc + 16 * j;
        if (k >= K) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nb + r;
          if (n >= N) continue;
          float* dst = C + (long)n * ldc + k;
          if (MODE == 1) *dst += acc[i][j][r];
          else atomicAdd(dst, acc[i][j][r]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// One finishing launch per GEMM: threads [0, total) add the split slabs of each tile to C in chunk
// order (bitwise reproducible; one thread per (tile, wave, accumulator, lane): a 16-byte load per
// slab, 4 output rows), threads [total, total + nbias) add the bias partial rows in chunk order.
__global__ __launch_bounds__(256) void wgrad_finish_kernel(const float* __restrict__ slab, int split,
                                                          float* __restrict__ C, int ldc, int N, int K, int tiles_k,
                                                          long total, const float* __restrict__ bias_parts,
                                                          float* __restrict__ bias, int nbias) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= total) {
    const int n = (int)(t - total);
    if (n >= nbias) return;
    float s = bias_parts[n];
    for (int c = 1; c < split; ++c) s += bias_parts[(long)c * N + n];
    bias[n] += s;
    return;
  }
  const int lane = (int)(t & 63);
  const long u = t >> 6;               // (tile, wave, acc)
  const int a = (int)(u % NACC);
  const long v = u / NACC;             // (tile, wave)
  const int wave = (int)(v & 7);
  const long tile = v >> 3;
  const int i = a / FB, j = a - i * FB;
  const int wn = wave >> 2, wk = wave & 3;
  const int tile_n = (int)(tile / tiles_k), tile_k = (int)(tile - (long)tile_n * tiles_k);
  const int k = tile_k * TW + 64 * wk + 16 * j + (lane & 15);
  const int nb = tile_n * TW + 128 * wn + 16 * ((i + 2 * wk) & 7) + 4 * (lane >> 4);
  const float* src = slab + (tile * split * 8 + wave) * (long)(NACC * 64 * 4) + (a * 64 + lane) * 4;
  f32x4v sum = *(const f32x4v*)src;
  for (int s = 1; s < split; ++s) sum += *(const f32x4v*)(src + (long)s * SLAB_FLOATS);
  if (k >= K) return;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (nb + r < N) C[(long)(nb + r) * ldc + k] += sum[r];
}

}  // namespace wpp

namespace {
struct PPPlan {
  int split = 1, m_chunk = 0, tiles = 0, tiles_k = 0, mode = 0;
  bool slabs = false;  // partial tiles go to slabs + the finishing launch
  double cost = 1e30;
};

// rounds of 256-CU workgroup waves x per-workgroup MFMA time, plus the partial-sum traffic of the
// epilogue (slabs: stored and re-read at ~5 TB/s; atomics ~1.3 TB/s)
PPPlan plan_pp(int M, int N, int K, int split_req, int mode_req, int ncu, int min_split) {
  PPPlan p;
  const int tiles_n = (N + wpp::TW - 1) / wpp::TW;
  p.tiles_k = (K + wpp::TW - 1) / wpp::TW;
  p.tiles = tiles_n * p.tiles_k;
  const double rate_cu = 1.25e15 / ncu;
  const int max_split = (M + wpp::BR - 1) / wpp::BR;
  auto eval = [&](int s) {
    int chunk = (M + s - 1) / s;
    chunk = (chunk + wpp::BR - 1) / wpp::BR * wpp::BR;
    const int ss = (M + chunk - 1) / chunk;
    const long long nwg = (long long)p.tiles * ss;
    const long long rounds = (nwg + ncu - 1) / ncu;
    const double t_wg = 2.0 * chunk * wpp::TW * wpp::TW / rate_cu;
    int mode = ss == 1 ? 1 : 0;
    double t_epi = ss == 1 ? 0.0 : (double)nwg * wpp::SLAB_FLOATS * 8.0 / 5e12;
    const double t_atomic = ss == 1 ? 0.0 : (double)nwg * wpp::SLAB_FLOATS * 4.0 / 1.3e12;
    if (mode_req == 2 || (mode_req < 0 && ss > 1 && t_atomic < t_epi)) {
      mode = 2;
      t_epi = t_atomic;
    }
    if (mode_req == 0 && ss > 1) {
      mode = 0;
      t_epi = (double)nwg * wpp::SLAB_FLOATS * 8.0 / 5e12;
    }
    const double cost = rounds * t_wg + t_epi;
    if (cost < p.cost) {
      p.cost = cost;
      p.split = ss;
      p.m_chunk = chunk;
      p.mode = mode;
    }
  };
  if (split_req > 0) {
    eval(std::max(std::min(split_req, max_split), min_split));
  } else {
    for (int s = min_split; s <= std::max(min_split, std::min(max_split, 4 * ncu)); ++s) eval(s);
  }
  return p;
}

hipError_t plan_wgrad_pp(int lda, int ldb, int M, int N, int K, int split, int mode, bool det, PPPlan& p) {
  if (lda % 8 || ldb % 8 || K % 8 || lda < N) return hipErrorInvalidValue;
  // one stage of either operand must stay below the 32-bit buffer range
  if ((long long)wpp::BR * std::max(lda, ldb) * 2 >= (1LL << 31)) return hipErrorInvalidValue;
  // deterministic runs never use atomics
  p = plan_pp(M, N, K, split, det ? 0 : mode, device_cu_count(), 1);
  p.slabs = p.mode == 0 && p.split > 1;
  return hipSuccess;
}
}  // namespace

long wgrad_pp_ws_floats(int lda, int ldb, int M, int N, int K, int split, int mode, bool bias) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  PPPlan p;
  if (plan_wgrad_pp(lda, ldb, M, N, K, split, mode, deterministic(), p) != hipSuccess) return 0;
  long f = p.slabs ? (long)p.tiles * p.split * wpp::SLAB_FLOATS : 0;
  if (bias && !(p.mode == 2 && p.split > 1)) f += (long)p.split * N;
  return f;
}

hipError_t launch_wgrad_pp(const void* dy, int lda, const void* x, int ldb, float* c, int ldc, int M, int N, int K,
                           int split, int mode, float* ws, float* bias, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  PPPlan p;
  const hipError_t e = plan_wgrad_pp(lda, ldb, M, N, K, split, mode, deterministic(), p);
  if (e != hipSuccess) return e;
  const int nwg = p.tiles * p.split;
  const bool slabs = p.slabs;
  const bool atomic = !slabs && p.split > 1;  // mode 2: partials and bias sums added with fp32 atomics
  float* slab = slabs ? ws : nullptr;
  float* bias_parts =
      bias == nullptr ? nullptr : atomic ? bias : ws + (slabs ? (long)p.tiles * p.split * wpp::SLAB_FLOATS : 0);
  if ((slabs || (bias != nullptr && !atomic)) && ws == nullptr) return hipErrorInvalidValue;
  const int m = slabs ? 0 : (p.split == 1 ? 1 : 2);
#define LLMT_WPP_LAUNCH(MD)                                                                                    \
  hipLaunchKernelGGL(wpp::wgrad_pp_kernel<MD>, dim3(nwg), dim3(wpp::kThreads), 0, stream, (const bf16_raw*)dy, lda,  \
                     (const bf16_raw*)x, ldb, c, ldc, M, N, K, p.tiles, p.tiles_k, p.m_chunk, p.split, nwg, slab,      \
                     bias_parts)
  if (m == 0) LLMT_WPP_LAUNCH(0);
  else if (m == 1) LLMT_WPP_LAUNCH(1);
  else LLMT_WPP_LAUNCH(2);
#undef LLMT_WPP_LAUNCH
  const long total = slabs ? (long)p.tiles * wpp::SLAB_FLOATS / 4 : 0;
  const int nbias = bias != nullptr && !atomic ? N : 0;
  if (total + nbias > 0)
    hipLaunchKernelGGL(wpp::wgrad_finish_kernel, dim3((unsigned)((total + nbias + 255) / 256)), dim3(256), 0, stream,
                       slab, p.split, c, ldc, N, K, p.tiles_k, total, bias_parts, bias, nbias);
  return hipGetLastError();
}

}  // namespace llmt
