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
// Shapes whose reduction-free dimensions are not multiples of 256 (GPT-2 XL: d = 1600 = 6 x 256 +
// 64) would waste a quarter-full tile column on every row of tiles (12 % of the XL weight-gradient
// MFMA work).  Instead:
//  * K tail (K % 256 in {64, 128, 192}): the last K % 256 columns are covered by "strip" tiles of
//    512 (n) x 64 (k) — every wave a 64 x 64 block (4 x 4 accumulators), the X operand's image only
//    64 columns wide (128-byte rows, their own swizzle) — launched in the same grid after the
//    256 x 256 tiles, so they fill the last round of workgroups;
//  * N tail only (N % 256 != 0, K % 256 == 0, e.g. the MLP projection [1600, 6400]): the launcher
//    swaps the operands (C^T = X^T dY) so the tail lands on the strip side, the epilogue / finishing
//    pass write the transposed tile, and the bias column sums of dY run as a separate column-sum
//    pass.
// The planner (plan_pp) takes the tail tiling only where its model gives a >= 10 % margin over the
// square tiling.  GPT-2 XL at M = 32768 (same box, profiles/r6/wgrad_xl/): qkv 0.46-0.51 vs
// 0.56-0.57 ms, fc 0.62-0.65 vs 0.68-0.69, proj (swapped) 0.63 vs 0.74; 1600 x 1600 stays square.
// Replaces the autograd weight (and bias) gradients of every nn.Linear of the reference
// (models/gpt.py:27-29, 94-96, 184 via loss.backward() at training/trainer.py:386-387).
#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

namespace llmt {
namespace wpp {

using namespace gemm;

constexpr int kThreads = 512;  // 8 waves, 2 per SIMD
constexpr int BR = 32;         // reduction rows per stage
constexpr int TW = 256;        // main tile edge
constexpr int SN = 512;        // strip tile: SN (n) x SK (k)
constexpr int SK = 64;

// Tile geometry.  Main: waves 0-7 = (wn, wk) = (wave >> 2, wave & 3), a 128 (n) x 64 (k) block
// each.  Strip: wave w owns n columns 64w..64w+63 and all 64 k columns.
template <bool STRIP>
struct Geo {
  static constexpr int TA = STRIP ? SN : TW;    // n columns of the tile (dY image width)
  static constexpr int TB = STRIP ? SK : TW;    // k columns (X image width)
  static constexpr int ROWA = 2 * TA, ROWB = 2 * TB;
  static constexpr int IMGA = BR * ROWA, IMGB = BR * ROWB;
  static constexpr int SLOT = IMGA + IMGB;      // 32 KiB / 36 KiB
  static constexpr int FA = STRIP ? 4 : 8, FB = 4;  // 16-wide fragments per wave
  static constexpr int NACC = FA * FB;
  static constexpr int SLAB = TA * TB;          // floats of one tile's partial
  static constexpr int OPSA = 4 * ROWA / 1024;  // 16-byte-per-lane fill ops per wave (its 4 image rows)
  static constexpr int OPSB = (4 * ROWB + 1023) / 1024;
  static constexpr int NOPS = OPSA + OPSB;
};
constexpr int kSmemBytes = 2 * Geo<true>::SLOT;
#ifndef LLMT_WPP_L2_PROBE
#define LLMT_WPP_L2_PROBE 0  // 1: variant build whose operand loads stay L2-resident (timing probe)
#endif  // 72 KiB: two ring slots of the larger geometry

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

// 32-byte segment swizzle of an image row.  Rows of >= 256 bytes (a multiple of the 64 banks):
// f(row) = (row & 3) | ((row >> 3) & 1) << 2 puts the 8 rows one 32-lane half of a transposed
// fragment read touches (rows r..r+3, r+8..r+11) on 8 distinct 32-byte bank groups.  128-byte rows
// (the strip's X image, 4 segments) already alternate bank halves with row parity, so the XOR takes
// bits 1 and 3 of the row instead: (row parity, segment ^ h(row)) is distinct over those 8 rows.
template <int ROWBYTES>
__device__ __forceinline__ int swz(int row) {
  if constexpr (ROWBYTES >= 256) return (row & 3) | (((row >> 3) & 1) << 2);
  else return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
}

template <int ROWBYTES>
__device__ __forceinline__ bf16x8 tr_read(unsigned addr) {
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(unsigned long)addr);
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(unsigned long)(addr + 4 * ROWBYTES));
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

// One tile family of a launch: [0] the 256 x 256 tiles over k < k_end, [1] the 512 x 64 strips.
struct Seg {
  int tiles = 0, tiles_k = 0;  // tile = tile_n * tiles_k + tile_k
  int k_base = 0;              // first k column of the family
  int m_chunk = 0, split = 1;  // reduction rows per workgroup, chunks
  int nwg = 0;                 // tiles * split
  int mode = 0;                // 0 slab partials, 1 C += acc (one owner), 2 fp32 atomics
  float* slab = nullptr;
};
struct Args {
  const bf16_raw* A;  // dY (or X when the launcher swapped the operands)
  const bf16_raw* B;
  float* C;
  float* bias_slab;
  int lda, ldb, ldc, M, N, K;
  int trans;  // output element (n, k) lives at C[k * ldc + n]
  Seg seg[2];
};

// The wave's n-fragment i -> 16-column group within the tile.  Main tiles take their 8 fragments in
// an order rotated by 2 * wk so the bias sweep covers distinct fragments with compile-time indices.
template <bool STRIP>
__device__ __forceinline__ int frag_n(int i, int wn, int wk) {
  return STRIP ? 4 * wn + i : 8 * wn + ((i + 2 * wk) & 7);
}

// Fills are register-staged: in LOAD(st) each wave writes stage st+1 (loaded two phases earlier)
// into its ring slot with 16-byte lane-linear ds_write_b128 and loads stage st+3 into the freed
// registers (two register sets, stage parity).  A slot is free one phase after its last read, so two
// slots suffice, and over half the LDS is left for other kernels' workgroups on the CU.  (Measured
// against LDS-DMA fills through a 4-slot ring: +2-4 % op level, +0.5 % in the step, docs/round4.md.)
template <bool STRIP>
__device__ __forceinline__ void tile_body(const Args& p, const Seg& sg, int w, unsigned lds) {
  using G = Geo<STRIP>;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave >> 2;  // 0 = X (leads), 1 = Y (one barrier behind)
  const int wn = STRIP ? wave : wave >> 2, wk = STRIP ? 0 : wave & 3;

  const int chunk = w / sg.tiles, tile = w - chunk * sg.tiles;
  const int tile_n = tile / sg.tiles_k, tile_k = tile - tile_n * sg.tiles_k;
  const int n0 = tile_n * G::TA, k0 = sg.k_base + tile_k * G::TB;
  const int m_begin = chunk * sg.m_chunk;
  const int rows = min(p.M - m_begin, sg.m_chunk);
  if (rows <= 0) return;  // whole workgroup, uniform
  const int nst = (rows + BR - 1) / BR;
  const bool want_bias = !STRIP && p.bias_slab != nullptr && tile_k == 0;

  // fills: this wave copies image rows 4*wave .. 4*wave+3 of each operand; op j, lane l moves
  // 16-byte chunk e = 64 j + l of those rows (lane-linear in LDS) and holds the source chunk whose
  // 32-byte segment is that one XOR swz(row).  The strip's X rows (4 x 128 B) take 32 lanes: lanes
  // 32-63 repeat lanes 0-31 (same data to the same address).
  int voff[G::NOPS];
  unsigned loff[G::NOPS];
#pragma unroll
  for (int j = 0; j < G::NOPS; ++j) {
    const bool isa = j < G::OPSA;
    const int rb = isa ? G::ROWA : G::ROWB, lpr = rb / 16;
    const int e = ((isa ? j : j - G::OPSA) * 64 + lane) % (4 * lpr);
    const int row = 4 * wave + e / lpr, c = e % lpr;
    const int sw = isa ? swz<G::ROWA>(row) : swz<G::ROWB>(row);
    const int csrc = (((c >> 1) ^ sw) << 1) | (c & 1);
    voff[j] = isa ? (row * p.lda + n0 + 8 * csrc) * 2 : (row * p.ldb + k0 + 8 * csrc) * 2;
    loff[j] = (isa ? 0u : (unsigned)G::IMGA) + (unsigned)(row * rb + 16 * c);
  }

  // fragment read addresses (bytes within a slot): lane (g, q, pp) reads rows 8g + q (+4) at the
  // 32-byte segment (logical ^ swz), bytes 8pp..8pp+7
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int fla = swz<G::ROWA>(8 * g + q), flb = swz<G::ROWB>(8 * g + q);
  const unsigned rowa = (unsigned)((8 * g + q) * G::ROWA + 8 * pp);
  const unsigned rowb = (unsigned)(G::IMGA + (8 * g + q) * G::ROWB + 8 * pp);
  unsigned ao[G::FA], bo[G::FB];
#pragma unroll
  for (int i = 0; i < G::FA; ++i) ao[i] = rowa + ((frag_n<STRIP>(i, wn, wk) ^ fla) << 5);
#pragma unroll
  for (int j = 0; j < G::FB; ++j) bo[j] = rowb + (((STRIP ? j : 4 * wk + j) ^ flb) << 5);

  f32x4v acc[G::FA][G::FB];
#pragma unroll
  for (int i = 0; i < G::FA; ++i)
#pragma unroll
    for (int j = 0; j < G::FB; ++j) acc[i][j] = 0.f;
  f32x4v bacc[2] = {0.f, 0.f};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, (short8v){0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80});

  u32x4 R0[G::NOPS], R1[G::NOPS];  // staged stage parity
  // (unconditional: a stage past the chunk has a zero-record descriptor and loads zeros — a
  // conditional load made hipcc drain every outstanding load before each LDS write)
  auto load_stage = [&](int st, u32x4 (&R)[G::NOPS]) {
#if LLMT_WPP_L2_PROBE
    // timing probe: the chunk's first two stages again (L2-hot, wrong results)
    const int r0 = (st & 1) * BR, nr = max(0, min(BR, rows - r0));
#else
    const int r0 = st * BR, nr = max(0, min(BR, rows - r0));
#endif
    const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(p.A + (long)(m_begin + r0) * p.lda, nr * p.lda * 2);
    const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(p.B + (long)(m_begin + r0) * p.ldb, nr * p.ldb * 2);
#pragma unroll
    for (int j = 0; j < G::NOPS; ++j)
      R[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(j < G::OPSA ? ra : rb, voff[j], 0, 0));
  };
  auto write_stage = [&](int slot, const u32x4 (&R)[G::NOPS]) {
#pragma unroll
    for (int j = 0; j < G::NOPS; ++j) *(lds_u32x4*)(size_t)(lds + slot * G::SLOT + loff[j]) = R[j];
  };

  // prologue: stage 0 landed everywhere, stages 1 and 2 loading; Y then falls one barrier behind
  load_stage(0, R0);
  load_stage(1, R1);
  write_stage(0, R0);
  load_stage(2, R0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (grp == 1) barrier();

  // R: the register set of stage st+1 (= that of st+3)
  auto phase = [&](int st, int slot, u32x4 (&R)[G::NOPS]) {
    // ---- LOAD(st): fragments of stage st, stage st+1 into the other slot, stage st+3 loading
    const unsigned sb = lds + slot * G::SLOT;
    bf16x8 af[G::FA], bfr[G::FB];
#pragma unroll
    for (int i = 0; i < G::FA; ++i) af[i] = tr_read<G::ROWA>(sb + ao[i]);
#pragma unroll
    for (int j = 0; j < G::FB; ++j) bfr[j] = tr_read<G::ROWB>(sb + bo[j]);
    // both unconditional (a slot past the last stage is never read)
    write_stage(slot ^ 1, R);
    load_stage(st + 3, R);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // ---- MFMA(st)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < G::FA; ++i)
#pragma unroll
      for (int j = 0; j < G::FB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (!STRIP && want_bias) {
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
  if (grp == 0) barrier();  // X matches Y's extra barrier

  // ---- epilogue.  Accumulator (i, j) register r of lane l: n = n0 + 16 frag_n(i) + 4 (l >> 4) + r,
  // k = k0 + 64 wk + 16 j + (l & 15)
  if (!STRIP && want_bias) {
    // bacc[t][r] = column sums of logical fragment 2wk + t, rows 4g + r; identical in all 16 lanes
    // of a group (every column of the ones product), so lane (g, c) keeps row 4g + (c & 3)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int r = lane & 3;
      const float v = r == 0 ? bacc[t][0] : r == 1 ? bacc[t][1] : r == 2 ? bacc[t][2] : bacc[t][3];
      const int n = n0 + 128 * wn + 16 * (2 * wk + t) + 4 * g + r;
      // atomic epilogue (fast mode): straight into the bias vector; otherwise this chunk's row
      if ((lane & 15) < 4 && n < p.N) {
        if (sg.mode == 2) atomicAdd(p.bias_slab + n, v);
        else p.bias_slab[(long)chunk * p.N + n] = v;
      }
    }
  }
  if (sg.mode == 0) {
    float* s = sg.slab + ((long)(tile * sg.split + chunk) * 8 + wave) * (G::NACC * 64 * 4);
#pragma unroll
    for (int i = 0; i < G::FA; ++i)
#pragma unroll
      for (int j = 0; j < G::FB; ++j) *(f32x4v*)(s + ((i * G::FB + j) * 64 + lane) * 4) = acc[i][j];
  } else {
    const int kc = k0 + 64 * wk + (lane & 15);
#pragma unroll
    for (int i = 0; i < G::FA; ++i) {
      const int nb = n0 + 16 * frag_n<STRIP>(i, wn, wk) + 4 * g;
#pragma unroll
      for (int j = 0; j < G::FB; ++j) {
        const int k = kc + 16 * j;
        if (k >= p.K) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nb + r;
          if (n >= p.N) continue;
          float* dst = p.trans ? p.C + (long)k * p.ldc + n : p.C + (long)n * p.ldc + k;
          if (sg.mode == 1) *dst += acc[i][j][r];
          else atomicAdd(dst, acc[i][j][r]);
        }
      }
    }
  }
}

// 256 x 256 tiles first (blockIdx order is dispatch order), then the strips, so the strips fill the
// last round of workgroups; each family is XCD-remapped on its own (the workgroups of one row chunk
// share an XCD)
__global__ __launch_bounds__(kThreads, 2) void wgrad_pp_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) bf16_raw smem[kSmemBytes / 2];
  const unsigned lds = (unsigned)(unsigned long)(lds_void*)smem;
  const int b = blockIdx.x;
  if (b < p.seg[0].nwg) tile_body<false>(p, p.seg[0], xcd_remap(b, p.seg[0].nwg), lds);
  else tile_body<true>(p, p.seg[1], xcd_remap(b - p.seg[0].nwg, p.seg[1].nwg), lds);
}

// ---------------------------------------------------------------------------------------------
// One finishing launch per GEMM: one thread per (family, tile, wave, accumulator, lane) adds the
// split slabs of that 16-byte piece in chunk order (bitwise reproducible) into C; the threads past
// them add the bias partial rows in chunk order.
struct Finish {
  const float* slab[2];
  int split[2], tiles_k[2], k_base[2];
  long total[2];
  float* C;
  int ldc, N, K, trans, vec;  // vec: 16-byte read-modify-write of transposed rows is aligned
  const float* bias_parts;
  float* bias;
  int nbias, bias_split;
};

template <bool STRIP>
__device__ __forceinline__ void finish_piece(const Finish& f, long t) {
  using G = Geo<STRIP>;
  const int fam = STRIP ? 1 : 0;
  const int lane = (int)(t & 63);
  const long u = t >> 6;  // (tile, wave, acc)
  const int a = (int)(u % G::NACC);
  const long v = u / G::NACC;  // (tile, wave)
  const int wave = (int)(v & 7);
  const long tile = v >> 3;
  const int i = a / G::FB, j = a - i * G::FB;
  const int wn = STRIP ? wave : wave >> 2, wk = STRIP ? 0 : wave & 3;
  const int tile_n = (int)(tile / f.tiles_k[fam]), tile_k = (int)(tile - (long)tile_n * f.tiles_k[fam]);
  const int k = f.k_base[fam] + tile_k * G::TB + 64 * wk + 16 * j + (lane & 15);
  const int nb = tile_n * G::TA + 16 * frag_n<STRIP>(i, wn, wk) + 4 * (lane >> 4);
  const int split = f.split[fam];
  const float* src = f.slab[fam] + (tile * split * 8 + wave) * (long)(G::NACC * 64 * 4) + (a * 64 + lane) * 4;
  f32x4v sum = *(const f32x4v*)src;
  for (int s = 1; s < split; ++s) sum += *(const f32x4v*)(src + (long)s * G::SLAB);
  if (k >= f.K) return;
  if (f.trans) {
    float* dst = f.C + (long)k * f.ldc + nb;  // 4 consecutive floats
    if (f.vec && nb + 3 < f.N) {
      *(f32x4v*)dst += sum;
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (nb + r < f.N) dst[r] += sum[r];
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (nb + r < f.N) f.C[(long)(nb + r) * f.ldc + k] += sum[r];
}

__global__ __launch_bounds__(256) void wgrad_finish_kernel(Finish f) {
  long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t < f.total[0]) return finish_piece<false>(f, t);
  t -= f.total[0];
  if (t < f.total[1]) return finish_piece<true>(f, t);
  const int n = (int)(t - f.total[1]);
  if (n >= f.nbias) return;
  float s = f.bias_parts[n];
  for (int c = 1; c < f.bias_split; ++c) s += f.bias_parts[(long)c * f.N + n];
  f.bias[n] += s;
}

}  // namespace wpp

namespace {
struct SegPlan {
  int tiles = 0, tiles_k = 0, k_base = 0, split = 0, m_chunk = 0, mode = 0;
  int nwg() const { return tiles * split; }
  bool slabs() const { return mode == 0 && split > 1; }
};
struct PPPlan {
  SegPlan seg[2];
  bool swap = false;  // operands swapped, output transposed, bias by a separate column-sum pass
  double cost = 1e30;
};

constexpr double kTailMargin = 0.9;   // modelled cost ratio below which the tail tiling is taken
constexpr double kStripCost = 1.7;  // strip time per FLOP relative to the 256 x 256 tile (LDS-write-bound, measured)

// Finishing time of n1 workgroups of length d1 followed (in dispatch order) by n2 of length d2 on
// ncu CUs, as rounds of ncu workgroups each lasting its longest member.  Measured at GPT-2 XL
// (profiles/r6/wgrad_xl/sweep_*.jsonl): workgroups past the first ncu start only about when the
// first round's long workgroups end, not when its short ones do (qkv, 228 tiles + 20 strips:
// 0.45-0.48 ms; + 40 strips of half the length: 0.59 ms), so list scheduling is the wrong model.
double makespan(long n1, double d1, long n2, double d2, int ncu) {
  double t = 0.0;
  for (long r0 = 0; r0 < n1 + n2; r0 += ncu) {
    const long r1 = std::min(n1 + n2, r0 + ncu);  // this round: [r0, r1)
    t += r0 < n1 ? d1 : 0.0;
    if (r0 >= n1 || r1 > n1) t += r0 < n1 ? std::max(0.0, d2 - d1) : d2;
  }
  return t;
}

// rounds of 256-CU workgroup waves x per-workgroup MFMA time, plus the partial-sum traffic of the
// epilogue (slabs: stored and re-read at ~5 TB/s; atomics ~1.3 TB/s)
PPPlan plan_pp(int M, int N, int K, int split_req, int mode_req, int ncu, bool tails) {
  PPPlan p;
  const double rate_cu = 1.25e15 / ncu;
  const int max_split = (M + wpp::BR - 1) / wpp::BR;
  // strips for a K tail of 64-192 columns behind at least one full 256-column tile
  const int tail = K % wpp::TW;
  const bool strips = tails && K > wpp::TW && tail != 0 && tail % wpp::SK == 0;
  const int k_main = strips ? K - tail : K;
  SegPlan& m = p.seg[0];
  SegPlan& s = p.seg[1];
  m.tiles_k = (k_main + wpp::TW - 1) / wpp::TW;
  m.tiles = (N + wpp::TW - 1) / wpp::TW * m.tiles_k;
  if (strips) {
    s.tiles_k = tail / wpp::SK;
    s.k_base = k_main;
    s.tiles = (N + wpp::SN - 1) / wpp::SN * s.tiles_k;
  }
  auto chunk_of = [&](int sp, int& ss) {
    int chunk = (M + sp - 1) / sp;
    chunk = (chunk + wpp::BR - 1) / wpp::BR * wpp::BR;
    ss = (M + chunk - 1) / chunk;
    return chunk;
  };
  // epilogue mode and partial-sum traffic of one family
  auto epi = [&](long nwg, int ss, int slab_floats, int& mode) {
    if (ss == 1) {
      mode = 1;
      return 0.0;
    }
    const double t_slab = (double)nwg * slab_floats * 8.0 / 5e12;
    const double t_atomic = (double)nwg * slab_floats * 4.0 / 1.3e12;
    mode = 0;
    if (mode_req == 2 || (mode_req < 0 && t_atomic < t_slab)) {
      mode = 2;
      return t_atomic;
    }
    return t_slab;
  };
  auto eval = [&](int sm, int sst) {
    int ssm = 0, sss = 0;
    const int cm = chunk_of(sm, ssm);
    const long n1 = (long)m.tiles * ssm;
    const double d1 = 2.0 * cm * wpp::TW * wpp::TW / rate_cu;
    int mode_m = 0, mode_s = 0, cs = 0;
    double t = epi(n1, ssm, wpp::TW * wpp::TW, mode_m);
    long n2 = 0;
    double d2 = 0.0;
    if (strips) {
      cs = chunk_of(sst, sss);
      n2 = (long)s.tiles * sss;
      d2 = kStripCost * 2.0 * cs * wpp::SN * wpp::SK / rate_cu;
      t += epi(n2, sss, wpp::SN * wpp::SK, mode_s);
    }
    t += strips ? makespan(n1, d1, n2, d2, ncu) : (double)((n1 + ncu - 1) / ncu) * d1;
    if (t < p.cost) {
      p.cost = t;
      m.split = ssm;
      m.m_chunk = cm;
      m.mode = mode_m;
      if (strips) {
        s.split = sss;
        s.m_chunk = cs;
        s.mode = mode_s;
      }
    }
  };
  // split_req = main split + 65536 * strip split (0: searched)
  const int req_m = split_req & 0xffff, req_s = split_req >> 16;
  const int lo_m = req_m > 0 ? std::min(req_m, max_split) : 1;
  const int hi_m = req_m > 0 ? lo_m : strips ? std::min(max_split, 64) : std::max(1, std::min(max_split, 4 * ncu));
  const int lo_s = req_s > 0 ? std::min(req_s, max_split) : 1;
  const int hi_s = req_s > 0 ? lo_s : std::min(max_split, 64);
  for (int sm = lo_m; sm <= hi_m; ++sm) {
    if (!strips) {
      eval(sm, 0);
      continue;
    }
    for (int sst = lo_s; sst <= hi_s; ++sst) eval(sm, sst);
  }
  return p;
}

// plans are cached per shape (the strip search simulates the dispatch: ~10 ms per new shape)
// mode: -1 auto, 0 slabs, 2 atomics; +8 (7, 8, 10): 256 x 256 tiles only (no strips, no swap: the
// rounds-1-5 tiling, kept for A/B timing in bench/wgrad_pp.py)
hipError_t plan_wgrad_pp(int lda, int ldb, int M, int N, int K, bool bias, int split, int mode, bool det, PPPlan& p) {
  const bool tails = mode < 7;
  if (!tails) mode -= 8;
  if (lda % 8 || ldb % 8 || K % 8 || lda < N) return hipErrorInvalidValue;
  // one stage of either operand must stay below the 32-bit buffer range
  if ((long long)wpp::BR * std::max(lda, ldb) * 2 >= (1LL << 31)) return hipErrorInvalidValue;
  // N tail with a whole K: swap the operands so the tail becomes the strips' K tail (the bias
  // column-sum pass of the swapped case reads a dense dY)
  const bool swap = tails && N % wpp::TW != 0 && N % wpp::SK == 0 && N > wpp::TW && K % wpp::TW == 0 && (!bias || lda == N);
  const int mode_req = det ? 0 : mode;  // deterministic runs never use atomics
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int, int, int, bool>, PPPlan> cache;
  const auto key = std::make_tuple(M, swap ? K : N, swap ? N : K, split, mode_req, (int)swap, tails);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it == cache.end()) {
    // the tail tiling only where the model gives it a clear margin: at 1600 x 1600 (modelled -2 %)
    // it measured +8 % (0.203 vs 0.189 ms, profiles/r6/wgrad_xl/)
    const int ncu = device_cu_count();
    PPPlan np = plan_pp(M, N, K, split, mode_req, ncu, false);
    if (tails) {
      PPPlan tp = plan_pp(M, swap ? K : N, swap ? N : K, split, mode_req, ncu, true);
      tp.swap = swap;
      if (tp.seg[1].tiles > 0 && tp.cost < kTailMargin * np.cost) np = tp;
    }
    it = cache.emplace(key, np).first;
  }
  p = it->second;
  return hipSuccess;
}

long slab_floats(const SegPlan& s, int slab) { return s.slabs() ? (long)s.tiles * s.split * slab : 0; }

// workspace: [main slabs][strip slabs][bias partial rows | column-sum workspace of the swapped case]
long ws_layout(const PPPlan& p, int M, int N, bool bias, long& off_strip, long& off_bias) {
  off_strip = slab_floats(p.seg[0], wpp::TW * wpp::TW);
  off_bias = off_strip + slab_floats(p.seg[1], wpp::SN * wpp::SK);
  long f = off_bias;
  if (bias) {
    if (p.swap) f += colwise_ws_floats(M, N);
    else if (p.seg[0].mode != 2) f += (long)p.seg[0].split * N;
  }
  return f;
}
}  // namespace

int wgrad_pp_plan_info(int lda, int ldb, int M, int N, int K, bool bias, int split, int mode, long* out) {
  PPPlan p;
  if (plan_wgrad_pp(lda, ldb, M, N, K, bias, split, mode, deterministic(), p) != hipSuccess) return 0;
  out[0] = p.swap;
  for (int f = 0; f < 2; ++f) {
    out[1 + 5 * f] = p.seg[f].tiles;
    out[2 + 5 * f] = p.seg[f].split;
    out[3 + 5 * f] = p.seg[f].m_chunk;
    out[4 + 5 * f] = p.seg[f].mode;
    out[5 + 5 * f] = p.seg[f].nwg();
  }
  out[11] = (long)(p.cost * 1e9);  // modelled ns
  return 12;
}

long wgrad_pp_ws_floats(int lda, int ldb, int M, int N, int K, int split, int mode, bool bias) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  PPPlan p;
  if (plan_wgrad_pp(lda, ldb, M, N, K, bias, split, mode, deterministic(), p) != hipSuccess) return 0;
  long o1, o2;
  return ws_layout(p, M, N, bias, o1, o2);
}

hipError_t launch_wgrad_pp(const void* dy, int lda, const void* x, int ldb, float* c, int ldc, int M, int N, int K,
                           int split, int mode, float* ws, float* bias, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  PPPlan p;
  const hipError_t e = plan_wgrad_pp(lda, ldb, M, N, K, bias != nullptr, split, mode, deterministic(), p);
  if (e != hipSuccess) return e;
  long off_strip = 0, off_bias = 0;
  const long need = ws_layout(p, M, N, bias != nullptr, off_strip, off_bias);
  if (need > 0 && ws == nullptr) return hipErrorInvalidValue;

  wpp::Args a;
  a.A = (const bf16_raw*)(p.swap ? x : dy);
  a.B = (const bf16_raw*)(p.swap ? dy : x);
  a.lda = p.swap ? ldb : lda;
  a.ldb = p.swap ? lda : ldb;
  a.C = c;
  a.ldc = ldc;
  a.M = M;
  a.N = p.swap ? K : N;
  a.K = p.swap ? N : K;
  a.trans = p.swap ? 1 : 0;
  const bool atomic_bias = !p.swap && p.seg[0].mode == 2;  // split > 1 with fp32 atomics
  a.bias_slab = (bias == nullptr || p.swap) ? nullptr : atomic_bias ? bias : ws + off_bias;
  for (int f = 0; f < 2; ++f) {
    const SegPlan& s = p.seg[f];
    wpp::Seg& d = a.seg[f];
    d.tiles = s.tiles;
    d.tiles_k = std::max(1, s.tiles_k);
    d.k_base = s.k_base;
    d.m_chunk = s.m_chunk;
    d.split = std::max(1, s.split);
    d.nwg = s.nwg();
    d.mode = s.mode;
    d.slab = s.slabs() ? ws + (f == 0 ? 0 : off_strip) : nullptr;
  }
  const int nwg = a.seg[0].nwg + a.seg[1].nwg;
  hipLaunchKernelGGL(wpp::wgrad_pp_kernel, dim3(nwg), dim3(wpp::kThreads), 0, stream, a);

  wpp::Finish f;
  for (int i = 0; i < 2; ++i) {
    const SegPlan& s = p.seg[i];
    f.slab[i] = a.seg[i].slab;
    f.split[i] = a.seg[i].split;
    f.tiles_k[i] = a.seg[i].tiles_k;
    f.k_base[i] = s.k_base;
    f.total[i] = s.slabs() ? (long)s.tiles * (i == 0 ? wpp::TW * wpp::TW : wpp::SN * wpp::SK) / 4 : 0;
  }
  f.C = c;
  f.ldc = ldc;
  f.N = a.N;
  f.K = a.K;
  f.trans = a.trans;
  f.vec = (uintptr_t)c % 16 == 0 && ldc % 4 == 0;
  f.bias_parts = a.bias_slab;
  f.bias = bias;
  f.nbias = bias != nullptr && !p.swap && !atomic_bias ? N : 0;
  f.bias_split = p.seg[0].split;
  const long total = f.total[0] + f.total[1] + f.nbias;
  if (total > 0)
    hipLaunchKernelGGL(wpp::wgrad_finish_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, f);
  if (bias != nullptr && p.swap) {
    const hipError_t ce = launch_colsum_accum(dy, true, bias, ws + off_bias, M, N, stream);
    if (ce != hipSuccess) return ce;
  }
  return hipGetLastError();
}

}  // namespace llmt
