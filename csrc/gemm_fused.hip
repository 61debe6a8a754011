// Forward / data-gradient GEMM with fused epilogues for gfx950:
//   C[M, N] (bf16) = epilogue( A[M, K] · op(B) )
//   A  bf16 row-major [M, lda], K contiguous (activations);
//   B  bf16 either [N, ldb] K contiguous ("NT": nn.Linear weight, forward y = x W^T) or
//      [K, ldb] N contiguous ("NN": the same weight in the data-gradient dX = dY W).
// Epilogues (EPI):
//   0  C = bf16(acc + bias)                      (bias optional)
//   1  U = bf16(acc + bias), C2 = bf16(gelu(U))  (fc forward: pre-activation kept for backward)
//   2  C = bf16(acc * gelu'(U)), dbias += colsum(C)   (proj dX: GELU backward + fc bias grad)
//   3  C = bf16(acc), delta[b, h, t] = sum_d C[m, 64h + d] * U[m, 64h + d], dbias += colsum(C)
//   4  u = bf16(acc + bias), C = bf16(gelu'(u)), C2 = bf16(gelu(u))  (fc forward keeping the GELU
//      derivative instead of the pre-activation: the backward's epilogue 5 then skips the erf math)
//   5  C = bf16(acc * U), dbias += colsum(C)  (U = the stored gelu'(u): proj dX + GELU backward)
//      (attention out-proj dX = dO; U = the attention output O: the flash-attention backward's
//      row constant and, without dropout, the V part of the qkv bias gradient — each wave's 64
//      output columns are exactly one head, so the per-head dot product never leaves the wave)
//
// Why: in the GPT MLP (reference models/gpt.py:94-105, nn.Linear -> nn.GELU -> nn.Linear) the
// library GEMM writes the pre-activation, a separate pass reads it and writes gelu(u), and in the
// backward a third pass reads dg and u to form du and its column sums — 3 x 400 MB of extra HBM
// traffic per layer at GPT-2 124M / 64K tokens.  Here those passes ride in the GEMM epilogue.
//
// Structure (MI355X playbook: LDS-DMA ring, counted vmcnt + raw barrier, XCD-aware persistent
// tiles; shared building blocks in gemm_common.h; measured history in docs/performance.md):
//  * 256x256 output tiles, 8 waves = two per SIMD: waves 0-3 own the upper 128 rows, waves 4-7
//    the lower; each wave a 128x64 tile of 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators (128 fp32
//    per lane), so one wave's LDS reads / waits overlap the other wave's MFMAs on the SIMD;
//  * PERSISTENT: min(#tiles, #CUs) workgroups; each XCD owns a contiguous range of tiles (raster
//    in bands of kBand n-tiles, m-major inside a band) and its workgroups stride through it.  The
//    64-deep K stages of ALL of a workgroup's tiles form one stream through a 2-slot LDS ring
//    (128 KiB: stage g+1 lands while stage g computes), so the next tile's first stage loads
//    while this tile's epilogue runs;
//  * A image [256 m][64 k] and NT B image [256 n][64 k]: 128-byte rows (each 1-KiB LDS-DMA op
//    moves 8 whole cache lines), 16-byte chunks XOR (row & 7) so every ds_read_b128 lane group of
//    a 16x16x32 fragment read hits 16 distinct bank slots.  NN B image [64 k][256 n] with
//    the swz_nn swizzle, read transposed (ds_read_b64_tr_b16);
//  * fragment reads are issued one MFMA sub-group (16 MFMAs) ahead; one wait + barrier per stage,
//    placed before the last sub-group so the next stage's first fragments load under it;
//  * MFMA srcA = B fragment, srcB = A fragment, so a lane's accumulator column is one output ROW
//    and its registers run along N in groups of 4 — the epilogue stages each 16x64 piece through
//    a per-wave XOR-swizzled fp32 LDS image (no cross-wave sync) and writes 16-byte stores, 8
//    whole 128-byte row segments per wave instruction, with buffer stores (out-of-range lanes get
//    an offset past the descriptor, so the store count is branch-free and known: the counted
//    waits after an epilogue rely on it); the tile's bias rides with its last K stage by LDS-DMA.

#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

namespace llmt {
namespace fgemm {

using namespace gemm;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int BM = 256, BN = 256, BK = 64, NSLOT = 2;
constexpr int kWaves = 8, kThreads = 64 * kWaves;  // two waves per SIMD
constexpr int kAElems = BM * BK;                // [256][64]: 128-byte rows = whole cache lines
constexpr int kBElems = BN * BK;                // [256][64] or [64][256]
constexpr int kSlotElems = kAElems + kBElems;   // 64 KiB
constexpr int kDmaA = kAElems * 2 / 1024 / kWaves;  // 1-KiB DMA ops per wave per stage (4)
constexpr int kDmaB = kBElems * 2 / 1024 / kWaves;  // (4)
constexpr int P = kDmaA + kDmaB;                // 8
constexpr int kEpiFloats = 16 * 64;             // per-wave fp32 staging image [16][64] (4 KiB)
constexpr int kSmemElems = NSLOT * kSlotElems + kWaves * kEpiFloats * 2;  // 160 KiB
constexpr int kOob = 0x7ffffff0;                // buffer offset past any descriptor: dropped / 0
constexpr int kBand = 4;                        // n-tiles per raster band (see tile_origin)
constexpr int kWideM = 256;                     // from this many m-tiles on, one band spans all of N
#ifndef LLMT_FGEMM_EPI_PROBE
#define LLMT_FGEMM_EPI_PROBE 0  // 1: variant build without epilogues (timing probe, wrong results)
#endif

constexpr float kInvSqrt2 = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;

// exact-erf GELU and derivative (same A&S 7.1.26 erf as elementwise.hip, |err| < 1.5e-7)
struct ErfPdf {
  float erf, e;
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

// VMEM ops each epilogue issues unconditionally (a lower bound is what the counted waits need)
template <int EPI>
struct EpiOps {
  static constexpr int value = EPI == 0 ? 16 : (EPI == 3 ? 48 : 32);  // 4 as 1, 5 as 2
};

// one 256-byte LDS-DMA op (4 bytes per lane), M0 saved/restored like dma16
__device__ __forceinline__ void dma4(unsigned lds_dst, int voff, __amdgpu_buffer_rsrc_t rsrc, int soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %[keep], m0\n\t"
      "s_nop 4\n\t"
      "s_mov_b32 m0, %[dst]\n\t"
      "s_nop 0\n\t"
      "buffer_load_dword %[v], %[r], %[so] offen lds\n\t"
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [dst] "s"(lds_dst), [v] "v"(voff), [r] "s"(rsrc), [so] "s"(soff)
      : "memory");
}

// One stage of this wave's LDS-DMA: 4 A ops (1 KiB each, consecutive LDS KiB from dst_a) and 4 B
// ops (from dst_b), one M0 save/restore per stage instead of per op.
__device__ __forceinline__ void dma_stage(unsigned dst_a, unsigned dst_b, const int (&va)[4], const int (&vb)[4],
                                          __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int soa, int sob) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %[keep], m0\n\t"
      "s_mov_b32 m0, %[da]\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[a0], %[ra], %[soa] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[a1], %[ra], %[soa] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[a2], %[ra], %[soa] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[a3], %[ra], %[soa] offen lds\n\t"
      "s_mov_b32 m0, %[db]\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[b0], %[rb], %[sob] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[b1], %[rb], %[sob] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[b2], %[rb], %[sob] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[b3], %[rb], %[sob] offen lds\n\t"
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [da] "s"(dst_a), [db] "s"(dst_b), [a0] "v"(va[0]), [a1] "v"(va[1]), [a2] "v"(va[2]), [a3] "v"(va[3]),
        [b0] "v"(vb[0]), [b1] "v"(vb[1]), [b2] "v"(vb[2]), [b3] "v"(vb[3]), [ra] "s"(ra), [rb] "s"(rb),
        [soa] "s"(soa), [sob] "s"(sob)
      // s_add_u32 writes SCC: left undeclared, the compiler may branch on a flag it set before the
      // asm (a BK = 32 variant of this kernel did exactly that and re-loaded stage 0; round5 §13)
      : "memory", "scc");
}

// Wait for the newest issued stage (nothing was issued after it but, when `post`, an epilogue's
// >= S VMEM ops; in-order VM counter), retire this wave's LDS reads, then the workgroup barrier:
// afterwards the stage is visible to every wave and the other ring slot is free to refill.
template <int S>
__device__ __forceinline__ void wait_ring(bool post) {
  constexpr int cs = S > 63 ? 63 : S;
  if (post) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(cs) : "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ bf16x8 lds_b128(const bf16_raw* p) { return *reinterpret_cast<const bf16x8*>(p); }

// NN B image [64 k][256 n]: 16-byte chunk c of row r sits at chunk c ^ swz_nn(r).  The wgrad
// swizzle 4 * (r & 3) alone leaves a 16x16x32 transposed fragment read 2-way conflicted: its lane
// group {0-31} covers rows r0..r0+3 and r0+8..r0+11 (two chunks each) and rows 8 apart repeat the
// same (r & 3) — 19 % of the kernel's LDS cycles were bank-conflict cycles at M = 131072
// (profiles/r2/pmc_fgemm_dx_gelu_nn.txt).  Bit 3 of the row flips bit 1 of the chunk, so the 16
// (row, chunk) pairs of every lane group land on 16 distinct 4-bank groups.
__device__ __forceinline__ int swz_nn(int row) { return ((row & 3) << 2) ^ (((row >> 3) & 1) << 1); }
template <int W>
__device__ __forceinline__ int nn_off(int row, int col) {
  return row * W + (((col >> 3) ^ swz_nn(row)) << 3) + (col & 7);
}

// 16x16x32 operand from a [k rows][W cols] image with k running down the rows: lane l -> column
// col0 + (l & 15), elements j = 0..7 -> rows row0 + 8*(l >> 4) + j (two ds_read_b64_tr_b16: in
// each 16-lane group lane 4q+p addresses row r+q, columns 4p..4p+3)
template <int W>
__device__ __forceinline__ bf16x8 tr_frag16(const bf16_raw* tile, int row0, int col0, int lane) {
  const int i = lane & 15;
  const int row = row0 + 8 * (lane >> 4) + (i >> 2);
  const int col = col0 + 4 * (i & 3);
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(tile + nn_off<W>(row, col)));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(tile + nn_off<W>(row + 4, col)));
  const short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// element offset of (row, 16-byte chunk c) in a [rows][64] image (128-byte rows) with the chunk
// XOR-swizzled by G(row) = row & 7.  A 16x16x32 fragment read (ds_read_b128) puts rows r0..r0+15
// on lanes 0-15 (chunk c) and again on lanes 16-31 (chunk c+1); each hardware lane group of 16
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) then covers all 16 bank slots exactly once.
__device__ __forceinline__ int swz_g(int row) { return row & 7; }
__device__ __forceinline__ int k64_off(int row, int c) { return row * 64 + 8 * (c ^ swz_g(row)); }

struct Args {
  const bf16_raw* A;
  const bf16_raw* B;
  bf16_raw* C;
  bf16_raw* C2;          // EPI 1: gelu output
  const bf16_raw* bias;  // EPI 0/1 (optional for 0)
  const bf16_raw* U;     // EPI 2: pre-activation; EPI 3: attention output O
  float* dbias;          // EPI 2/3: column sums (optional) -> partial rows [ceil(M / 128)][N] (see below)
  float* delta;          // EPI 3: [M / T, N / 64, T] per-head row dot products
  int T;                 // EPI 3: rows per sequence
  int lda, ldb, ldc, ldu;
  int M, N, K;
  int tiles_m, tiles_n, ntiles, nwg;
  int band;  // n-tiles per raster band (tile_origin)
  // non-temporal epilogue I/O (C / C2 stores, U loads): from kWideM m-tiles on the 0.2-1.6 GB of
  // output streams past every cache and, left temporal, evicts the weight and the activation strip
  // the tile order keeps in L2 / the Infinity Cache.  M = 131072: qkv fwd 0.517 -> 0.419 ms, fc fwd
  // 0.630 -> 0.533, fc fwd + GELU 0.851 -> 0.725, proj dX 0.622 -> 0.539, dX + dGELU 0.829 ->
  // 0.771; at M = 32768 mixed (qkv fwd 0.120 -> 0.133), so the rule is tied to the tile order's
  // (profiles/r3/nt/)
  int nt;
};

template <bool NN, int EPI>
__global__ __launch_bounds__(kThreads, 1) void gemm_fused_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) bf16_raw smem[kSmemElems];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // two wave groups (waves 0-3 / 4-7: one wave of each per SIMD) own the upper / lower 128 rows
  // of the tile; wave wq of a group owns 64 columns -> a 128x64 wave tile (4 x 2 MFMA tiles)
  const int wm = wave >> 2, wn = wave & 3;

  // ---- this workgroup's tiles: XCD-contiguous range, strided by the XCD's workgroup count
  const int L = blockIdx.x, xcd = L & 7, jx = L >> 3;
  const int wgx = (p.nwg - xcd + 7) >> 3;
  const int q = p.ntiles >> 3, r = p.ntiles & 7;
  const int cnt = q + (xcd < r ? 1 : 0);
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int my_tiles = jx < cnt ? (cnt - jx + wgx - 1) / wgx : 0;
  if (my_tiles == 0) return;
  const int nst = p.K / BK;
  const int total = my_tiles * nst;

  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.M * p.lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.B, (short)0, (NN ? p.K : p.N) * p.ldb * 2, 0x00020000);

  // per-lane DMA source offsets (bytes, relative to the stage's scalar offset)
  int va[kDmaA], vb[kDmaB];
#pragma unroll
  for (int j = 0; j < kDmaA; ++j) {  // A image: 8 rows of 128 B per op
    const int row = (wave * kDmaA + j) * 8 + (lane >> 3);
    va[j] = (row * p.lda + 8 * ((lane & 7) ^ swz_g(row))) * 2;
  }
#pragma unroll
  for (int j = 0; j < kDmaB; ++j) {
    if (NN) {  // [64 k][256 n]: 2 rows of 512 B per op, swz_nn swizzle
      const int row = (wave * kDmaB + j) * 2 + (lane >> 5);
      const int c = (lane & 31) ^ swz_nn(row);
      vb[j] = (row * p.ldb + 8 * c) * 2;
    } else {
      const int row = (wave * kDmaB + j) * 8 + (lane >> 3);
      vb[j] = (row * p.ldb + 8 * ((lane & 7) ^ swz_g(row))) * 2;
    }
  }
  const unsigned lds_base = (unsigned)(unsigned long)(lds_void*)smem;

  float* epi = reinterpret_cast<float*>(smem + NSLOT * kSlotElems) + wave * kEpiFloats;
  const unsigned epi_lds = (unsigned)(unsigned long)(lds_void*)epi;
  constexpr bool kHasU = EPI == 2 || EPI == 3 || EPI == 5;  // an [M, N] bf16 operand read per row segment
  constexpr bool kGelu = EPI == 1 || EPI == 4;              // second output C2 = gelu(u)
  const bool kBiasDma = !kHasU && p.bias != nullptr;
  const __amdgpu_buffer_rsrc_t rbias = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(kBiasDma ? p.bias : p.A), (short)0, kBiasDma ? p.N * 2 : 0, 0x00020000);

  // issue cursor (stage stream over this workgroup's tiles)
  int is_s = 0, is_t = 0, is_m0 = 0, is_n0 = 0;
  // Tile order: N is cut into bands of p.band tiles and the tiles run band-major, m-major inside
  // a band.  With kBand = 4 the ~32 workgroups an XCD runs together cover ~8 m-tiles x 4 n-tiles:
  // the band's weight rows (4 x 256 x K bf16, 1.5 MiB at K = 768) stay in that XCD's 4 MiB L2
  // across rounds while activation strips stream through.  From kWideM m-tiles on (M >= 64K
  // rows: activations of 100-800 MB) one band spans all of N instead, so each activation strip is
  // fetched from HBM once and reused by every n-tile while the whole weight (<= 4.7 MB) stays in
  // L2 / the Infinity Cache: at M = 131072 qkv fwd 0.527 -> 0.463 ms, fc fwd 0.665 -> 0.622, MLP
  // projection dX + GELU backward 0.825 -> 0.799 (profiles/r3/band/); at M = 32768 no difference.
  auto tile_origin = [&](int t, int& m0, int& n0) {
    const int w = base + jx + t * wgx;
    const int band = p.band;
    const int full = p.tiles_n / band, per_band = p.tiles_m * band;
    int mt, nt;
    if (w < full * per_band) {
      const int b = w / per_band, r = w - b * per_band;
      mt = r / band;
      nt = b * band + (r - mt * band);
    } else {
      const int wl = p.tiles_n - full * band, r = w - full * per_band;
      mt = r / wl;
      nt = full * band + (r - mt * wl);
    }
    LLMT_DASSERT(mt < p.tiles_m && nt < p.tiles_n);
    m0 = mt * BM;
    n0 = nt * BN;
  };
  tile_origin(0, is_m0, is_n0);
  auto issue = [&](int g) {
    const unsigned slot = lds_base + (unsigned)((g % NSLOT) * kSlotElems * 2);
    const int kk = is_s * BK;
    const int soa = (is_m0 * p.lda + kk) * 2;
    const int sob = NN ? (kk * p.ldb + is_n0) * 2 : (is_n0 * p.ldb + kk) * 2;
    dma_stage(slot + wave * kDmaA * 1024, slot + kAElems * 2 + wave * kDmaB * 1024, va, vb, ra, rb, soa, sob);
    if (kBiasDma && is_s == nst - 1) {
      // the tile's bias (this wave's 128 columns, bf16) rides with its last K stage into the head
      // of the wave's epilogue staging image: landed by that stage's wait, read before staging
      dma4(epi_lds, lane * 4, rbias, (is_n0 + wn * 64) * 2);
    }
    if (++is_s == nst) {
      is_s = 0;
      if (++is_t < my_tiles) tile_origin(is_t, is_m0, is_n0);
    }
  };

  const __amdgpu_buffer_rsrc_t rc =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.C, (short)0, p.M * p.ldc * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rc2 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(kGelu ? p.C2 : p.C), (short)0, p.M * p.ldc * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(kHasU ? p.U : p.C), (short)0, p.M * (kHasU ? p.ldu : p.ldc) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rdel = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(EPI == 3 ? p.delta : (float*)p.C), (short)0, EPI == 3 ? p.M * (p.N / 64) * 4 : 0, 0x00020000);

  // output stores / U loads with the non-temporal hint at large M (see Args::nt)
  auto st16 = [&](u32x4 v, __amdgpu_buffer_rsrc_t rs, int off) {
    if (p.nt) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 2);
    else __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
  };

  // Software pipeline over the stage stream (2-slot ring of 64-deep stages; stage g+1 lands while
  // stage g computes).  Iteration g runs its four k16 MFMA groups with every fragment read issued
  // one group ahead; before the last group: wait stage g+1 + retire reads + barrier, DMA stage g+2
  // into the slot stage g vacated, read the first fragments of stage g+1.
  // 16x16x32 MFMAs (at equal cycles per FLOP they hold a higher clock than 32x32x16 on random
  // data).  A stage (64 k) = 2 k32 steps x 2 halves of the wave's 8 m-fragments = 4 sub-groups of
  // 16 MFMAs; A fragments double-buffered per sub-group, B fragments per k32 step.
  auto read_a = [&](int g, int s2, int mh, bf16x8 (&af)[4]) {
    const bf16_raw* aimg = smem + (g % NSLOT) * kSlotElems;
    const int c = 4 * s2 + (lane >> 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = lds_b128(aimg + k64_off(wm * 128 + 64 * mh + 16 * i + (lane & 15), c));
  };
  auto read_b = [&](int g, int s2, bf16x8 (&bfr)[4]) {
    const bf16_raw* bimg = smem + (g % NSLOT) * kSlotElems + kAElems;
    const int c = 4 * s2 + (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (NN) bfr[j] = tr_frag16<BN>(bimg, 32 * s2, wn * 64 + 16 * j, lane);
      else bfr[j] = lds_b128(bimg + k64_off(wn * 64 + 16 * j + (lane & 15), c));
    }
  };
  auto mfma_group = [&](f32x4 (&acc)[4][8], int mh, const bf16x8 (&af)[4], const bf16x8 (&bfr)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[j][4 * mh + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[j][4 * mh + i], 0, 0, 0);
  };

  issue(0);
  if (total > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(P) : "memory");  // stage 0 (stage 1 flies)
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  bf16x8 a0[4], a1[4], b0[4], b1[4];
  read_a(0, 0, 0, a0);
  read_b(0, 0, b0);

  int g = 0;  // global stage index of the stream
  for (int t = 0; t < my_tiles; ++t) {
    f32x4 acc[4][8];  // [n-fragment j][m-fragment i], 16x16 each
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = 0.f;

    for (int s = 0; s < nst; ++s, ++g) {
      read_a(g, 0, 1, a1);
      mfma_group(acc, 0, a0, b0);
      read_a(g, 1, 0, a0);
      read_b(g, 1, b1);
      mfma_group(acc, 1, a1, b0);
      read_a(g, 1, 1, a1);
      mfma_group(acc, 0, a0, b1);
      if (g + 1 < total) {
        // stage g+1 was issued last, in iteration g-1; an epilogue after it iff g starts a tile
        wait_ring<EpiOps<EPI>::value>(!LLMT_FGEMM_EPI_PROBE && t > 0 && s == 0);
        if (g + 2 < total) issue(g + 2);
        read_a(g + 1, 0, 0, a0);
        read_b(g + 1, 0, b0);
      }
      mfma_group(acc, 1, a1, b1);
    }

#if LLMT_FGEMM_EPI_PROBE
    // timing probe (variant builds only, wrong results): no epilogue — every accumulator feeds one
    // sum whose store never happens, so the MFMAs stay; measures the main loop alone
    // (profiles/r6/fgemm/probe_*.jsonl, docs/round6.md section 6)
    {
      float sink = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) sink += acc[j][i][0] + acc[j][i][1] + acc[j][i][2] + acc[j][i][3];
      if (sink == 1.2345e38f) p.C[lane] = 0;
      continue;
    }
#endif
    // ---------------- epilogue of tile t ----------------
    // per 16-row m-fragment: its four 16x16 accumulator tiles -> [16 m][64 n] fp32 LDS image
    // (16-byte chunks XOR (row & 15)) -> 8 lanes per row read 8 columns each -> one 16-byte store
    // per lane, a wave instruction writing 8 whole 128-byte row segments
    int m0, n0;
    tile_origin(t, m0, n0);
    const int mw = m0 + wm * 128, nw = n0 + wn * 64;
    const int q = lane & 7;  // this lane's 8-column group of the wave's 64 columns
    const int n = nw + 8 * q;
    float bias_f[8];
    float csum[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bias_f[k] = 0.f;
      csum[k] = 0.f;
    }
    if (kBiasDma) {
      const ushort8_t bv = *reinterpret_cast<const ushort8_t*>(reinterpret_cast<const bf16_raw*>(epi) + 8 * q);
#pragma unroll
      for (int k = 0; k < 8; ++k) bias_f[k] = bf2f(bv[k]);
    }
    // EPI 2 / 3 read a bf16 operand (U = the GELU pre-activation / the attention output) per row
    // segment: those loads run one m-fragment ahead, so a tile's epilogue pays one memory round
    // trip instead of eight (each m-fragment used to load and wait on its own)
    u32x4 uraw[2][2];
    auto load_u = [&](int mf, u32x4(&dst)[2]) {
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int m = mw + 16 * mf + 8 * it + (lane >> 3);
        const int uoff = (m < p.M && n < p.N) ? (m * p.ldu + n) * 2 : kOob;
        dst[it] = p.nt ? __builtin_amdgcn_raw_buffer_load_b128(ru, uoff, 0, 2)
                        : __builtin_amdgcn_raw_buffer_load_b128(ru, uoff, 0, 0);
      }
    };
    if (kHasU) load_u(0, uraw[0]);
#pragma unroll
    for (int mf = 0; mf < 8; ++mf) {
      __builtin_amdgcn_sched_barrier(0);
      if (kHasU && mf + 1 < 8) load_u(mf + 1, uraw[(mf + 1) & 1]);
      {
        const int row = lane & 15;
#pragma unroll
        for (int nf = 0; nf < 4; ++nf) {
          const int ch = 4 * nf + (lane >> 4);
          const f32x4& v = acc[nf][mf];
          *reinterpret_cast<float4_t*>(epi + row * 64 + 4 * (ch ^ row)) = float4_t{v[0], v[1], v[2], v[3]};
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // wave-local: LDS executes a wave's ops in order
      float vals[2][8];
      int off[2];
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int R = 8 * it + (lane >> 3);
        const float4_t lo = *reinterpret_cast<const float4_t*>(epi + R * 64 + 4 * ((2 * q) ^ R));
        const float4_t hi = *reinterpret_cast<const float4_t*>(epi + R * 64 + 4 * ((2 * q + 1) ^ R));
        vals[it][0] = lo[0]; vals[it][1] = lo[1]; vals[it][2] = lo[2]; vals[it][3] = lo[3];
        vals[it][4] = hi[0]; vals[it][5] = hi[1]; vals[it][6] = hi[2]; vals[it][7] = hi[3];
        const int m = mw + 16 * mf + R;
        off[it] = (m < p.M && n < p.N) ? (m * p.ldc + n) * 2 : kOob;
      }
      asm volatile("" ::: "memory");
      if (EPI == 3) {
        const u32x4(&oraw)[2] = uraw[mf & 1];
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          __builtin_amdgcn_sched_barrier(0);
          const ushort8_t ov = __builtin_bit_cast(ushort8_t, oraw[it]);
          float o[8];
          float dot = 0.f;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            o[k] = bf2f(f2bf(vals[it][k]));  // the bf16 dO the attention backward reads
            dot = fmaf(o[k], bf2f(ov[k]), dot);
            csum[k] += o[k];
          }
          st16(__builtin_bit_cast(u32x4, pack8(o)), rc, off[it]);
          // the 8 lanes of one row segment (lane & 7) hold the head's 64 columns
          dot += __shfl_xor(dot, 1, 64);
          dot += __shfl_xor(dot, 2, 64);
          dot += __shfl_xor(dot, 4, 64);
          const int m = mw + 16 * mf + 8 * it + (lane >> 3);
          int doff = kOob;
          if (q == 0 && m < p.M && nw < p.N) {
            const int bb = m / p.T, t = m - bb * p.T;
            doff = ((bb * (p.N >> 6) + (nw >> 6)) * p.T + t) * 4;
          }
          // unconditional (dropped past the descriptor): the counted waits see a fixed op count
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dot), rdel, doff, 0, 0);
          asm volatile("" : "+v"(csum[0]), "+v"(csum[1]), "+v"(csum[2]), "+v"(csum[3]), "+v"(csum[4]),
                       "+v"(csum[5]), "+v"(csum[6]), "+v"(csum[7]));
        }
      } else if (EPI == 2 || EPI == 5) {
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          __builtin_amdgcn_sched_barrier(0);  // one row segment at a time: bounded VGPR pressure
          const ushort8_t uv = __builtin_bit_cast(ushort8_t, uraw[mf & 1][it]);
          float o[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            o[k] = EPI == 5 ? bf2f(f2bf(vals[it][k] * bf2f(uv[k]))) : bf2f(f2bf(vals[it][k] * gelu_grad(bf2f(uv[k]))));
            csum[k] += o[k];
          }
          st16(__builtin_bit_cast(u32x4, pack8(o)), rc, off[it]);
          // pin the running sums here: left alone, hipcc sinks the adds to the end of the epilogue
          // and keeps every product live (spills)
          asm volatile("" : "+v"(csum[0]), "+v"(csum[1]), "+v"(csum[2]), "+v"(csum[3]), "+v"(csum[4]),
                       "+v"(csum[5]), "+v"(csum[6]), "+v"(csum[7]));
        }
      } else {
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          float o[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = vals[it][k] + bias_f[k];
          const ushort8_t ov = pack8(o);
          if (EPI == 4) {  // gelu'(u) and gelu(u) of the bf16 pre-activation, one erf evaluation
            float gd[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float uu = bf2f(ov[k]);
              const ErfPdf ep = erf_pdf(uu);
              gd[k] = fmaf(0.5f, 1.f + ep.erf, uu * kInvSqrt2Pi * ep.e);
              o[k] = 0.5f * uu * (1.f + ep.erf);
            }
            st16(__builtin_bit_cast(u32x4, pack8(gd)), rc, off[it]);
            st16(__builtin_bit_cast(u32x4, pack8(o)), rc2, off[it]);
          } else {
            st16(__builtin_bit_cast(u32x4, ov), rc, off[it]);
            if (EPI == 1) {
#pragma unroll
              for (int k = 0; k < 8; ++k) o[k] = gelu(bf2f(ov[k]));
              st16(__builtin_bit_cast(u32x4, pack8(o)), rc2, off[it]);
            }
          }
        }
      }
    }
    if (kHasU && p.dbias != nullptr) {  // column sums over the wave's 128 rows: lanes sharing q
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = csum[k];
        v += __shfl_xor(v, 8, 64);
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        csum[k] = v;
      }
      // this wave's 128-row block owns partial row mw / 128 of the column sums (plain stores; the
      // launcher's fixed-order reduce adds the rows to the bias gradient: no atomics).  Only
      // ceil(M / 128) rows exist: a wave whose block lies wholly past M (the lower half of the
      // last 256-row tile when M % 256 <= 128) has nothing to store
      if (lane < 8 && n < p.N && mw < p.M) {
        float* dst = p.dbias + (long)(mw / 128) * p.N + n;
        *reinterpret_cast<float4_t*>(dst) = float4_t{csum[0], csum[1], csum[2], csum[3]};
        *reinterpret_cast<float4_t*>(dst + 4) = float4_t{csum[4], csum[5], csum[6], csum[7]};
      }
    }
  }
}

template <bool NN, int EPI>
void launch_one(const Args& a, hipStream_t stream) {
  hipLaunchKernelGGL((gemm_fused_kernel<NN, EPI>), dim3(a.nwg), dim3(kThreads), 0, stream, a);
}

}  // namespace fgemm

hipError_t launch_gemm_fused(const GemmFusedArgs& g, hipStream_t stream) {
  using namespace fgemm;
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  if (g.K < 4 * BK || g.K % BK || g.N % 8 || g.lda % 8 || g.ldb % 8 || g.ldc % 8) return hipErrorInvalidValue;
  if (g.epilogue < 0 || g.epilogue > 5) return hipErrorInvalidValue;
  const bool has_u = g.epilogue == 2 || g.epilogue == 3 || g.epilogue == 5;
  if ((g.epilogue == 1 || g.epilogue == 4) && g.c2 == nullptr) return hipErrorInvalidValue;
  if (has_u && (g.u == nullptr || g.ldu % 8)) return hipErrorInvalidValue;
  if (g.epilogue == 3 && (g.delta == nullptr || g.T <= 0 || g.M % g.T || g.N % 64 ||
                          (long long)g.M * (g.N / 64) * 4 >= (1LL << 31) - 64))
    return hipErrorInvalidValue;
  // 32-bit signed buffer offsets over every operand
  const long long lim = (1LL << 31) - 64;
  if ((long long)g.M * g.lda * 2 >= lim || (long long)g.M * g.ldc * 2 >= lim ||
      (long long)(g.b_kn ? g.K : g.N) * g.ldb * 2 >= lim || (long long)g.M * g.ldu * 2 >= lim)
    return hipErrorInvalidValue;
  Args a;
  a.A = (const bf16_raw*)g.a;
  a.B = (const bf16_raw*)g.b;
  a.C = (bf16_raw*)g.c;
  a.C2 = (bf16_raw*)g.c2;
  a.bias = (const bf16_raw*)g.bias;
  a.U = (const bf16_raw*)g.u;
  const int nparts = (g.M + 127) / 128;
  if (g.dbias != nullptr && g.ws == nullptr) return hipErrorInvalidValue;
  a.dbias = g.dbias != nullptr ? g.ws : nullptr;
  a.delta = g.delta;
  a.T = g.T;
  a.lda = g.lda;
  a.ldb = g.ldb;
  a.ldc = g.ldc;
  a.ldu = g.ldu;
  a.M = g.M;
  a.N = g.N;
  a.K = g.K;
  a.tiles_n = (g.N + BN - 1) / BN;
  a.tiles_m = (g.M + BM - 1) / BM;
  a.ntiles = a.tiles_m * a.tiles_n;
  const int ncu = gemm::cu_count();
  a.nwg = a.ntiles < ncu ? a.ntiles : ncu;  // persistent: one workgroup per CU
  // at large M one band spans all of N: see tile_origin
  a.band = a.tiles_m >= kWideM || kBand >= a.tiles_n ? a.tiles_n : kBand;
  a.nt = a.tiles_m >= kWideM ? 1 : 0;
  switch (g.epilogue * 2 + (g.b_kn ? 1 : 0)) {
    case 0: launch_one<false, 0>(a, stream); break;
    case 1: launch_one<true, 0>(a, stream); break;
    case 2: launch_one<false, 1>(a, stream); break;
    case 3: launch_one<true, 1>(a, stream); break;
    case 4: launch_one<false, 2>(a, stream); break;
    case 5: launch_one<true, 2>(a, stream); break;
    case 6: launch_one<false, 3>(a, stream); break;
    case 7: launch_one<true, 3>(a, stream); break;
    case 8: launch_one<false, 4>(a, stream); break;
    case 9: launch_one<true, 4>(a, stream); break;
    case 10: launch_one<false, 5>(a, stream); break;
    default: launch_one<true, 5>(a, stream); break;
  }
  if (g.dbias != nullptr) return launch_colsum_reduce(g.ws, nparts, g.N, g.dbias, g.ws + (long)nparts * g.N, stream);
  return hipGetLastError();
}

}  // namespace llmt
