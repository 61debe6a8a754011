// Weight-gradient GEMM for gfx950:  C[N, K] (f32, accumulated in place) += A^T B
//   A = dY [M, N] bf16 row-major (lda), B = X [M, K] bf16 row-major (ldb), reduction over M.
//
// Why a hand-written kernel: in a GPT step every weight gradient is a "tall-skinny" reduction
// (M = batch*seq = 32-64K tokens deep, output only 768..3072 wide).  hipBLASLt picks 256x256
// macro-tiles without split-K for these, i.e. 9..48 workgroups for 256 CUs, and measures
// 180-520 TFLOP/s on MI355X (bench/micro.py).  Here the M reduction is split across
// workgroups (split-K) so every launch fills the chip, and the partial tiles are summed with
// no-return f32 atomics straight into the flat fp32 gradient buffer — the beta=1 accumulation
// the training step needs anyway (no "grad += tmp" pass).  This replaces the reference's
// autograd weight gradients of every nn.Linear (models/gpt.py:27-29, 94-96 via loss.backward()
// at training/trainer.py:386-387).
//
// Two tile configurations share one kernel body (template <TN, TK>: 32x32 MFMA tiles per wave):
//  * <4,4>: 256x256 output tile, 4 waves (2x2) of 128x128 = 4x4 v_mfma_f32_32x32x16_bf16
//    accumulators (256 fp32 per lane, AGPR-resident), ONE workgroup per CU.  Per 32-row stage a
//    wave issues 32 MFMAs (1024 cycles/SIMD) against 32 transposed 8-byte LDS reads plus a
//    32 KiB DMA fill per CU — LDS busy ~50% of the MFMA time (MI355X_MICROARCH §LDS), which is
//    what the 64x64-per-wave <2,2> tile (LDS-bound, ~100%) could not reach;
//  * <2,2>: 128x128 tile, 2 workgroups per CU — kept for small outputs where the 256-wide tile
//    would need too many split-K atomics per useful FLOP.
// The launcher prices both (MFMA time per round of workgroups + atomic bytes at the measured
// ~1.3 TB/s chip-wide atomic rate) and picks the cheaper split/tile.
//
// Common structure (MI355X playbook: LDS-DMA staging, counted vmcnt, raw barriers, XCD remap):
//  * operands stream through a 4-slot LDS ring of 32-row stages filled by
//    `buffer_load_dwordx4 ... lds` (no VGPR staging, 3 stages in flight); the buffer
//    descriptor's record count ends at the workgroup's M chunk, so rows past the chunk (and past
//    the array) read as zero with no branches;
//  * waits are counted (`s_waitcnt vmcnt(2P|P|0)` = "this stage landed, the next two may still
//    be in flight", P = DMA ops per stage) followed by a raw s_barrier, never __syncthreads()
//    (whose vmcnt(0) would drain the whole ring every stage);
//  * both operands have the reduction index running DOWN their rows, so both are read with the
//    transposing ds_read_b64_tr_b16; the 16-byte chunks of each LDS row are XOR-swizzled by
//    4*(row & 3) (applied to the per-lane SOURCE address because the LDS-DMA destination is
//    lane-linear), which puts the 4 rows of each transposed read on distinct 64-byte bank groups;
//  * work items are remapped so the workgroups of one M chunk run on one XCD and share its L2;
//  * epilogue: one f32 atomic per accumulator register and lane — lanes 0-31 / 32-63 each add a
//    contiguous 128-byte row segment, the full-rate atomic shape;
//  * deterministic mode (run.deterministic): the same stores go to this M chunk's own partial
//    slab [chunk][N][K] instead, and launch_colsum_reduce adds the slabs to C in chunk order —
//    bitwise reproducible at the cost of one extra pass over split x N x K floats.
#include <cstdlib>

#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

namespace llmt {
namespace wgrad {

using namespace gemm;

constexpr int BM = 32, NSLOT = 4;
constexpr int kThreads = 256;

template <int TN, int TK>
struct Cfg {
  static constexpr int BN = 64 * TN, BK = 64 * TK;          // workgroup tile (2x2 waves)
  static constexpr int WA = BN, WB = BK;                     // LDS row widths (elements)
  static constexpr int kAElems = BM * WA, kBElems = BM * WB;
  static constexpr int kSlotElems = kAElems + kBElems;
  static constexpr int kDmaA = kAElems * 2 / 1024 / 4;      // 1-KiB DMA ops per wave per stage
  static constexpr int kDmaB = kBElems * 2 / 1024 / 4;
  static constexpr int kDmaPerStage = kDmaA + kDmaB;
  static constexpr int kMinBlocks = (TN * TK >= 16) ? 1 : 2;
};

template <int TN, int TK>
__global__ __launch_bounds__(kThreads, (Cfg<TN, TK>::kMinBlocks)) void wgrad_kernel(
    const bf16_raw* __restrict__ A, int lda, const bf16_raw* __restrict__ B, int ldb, float* __restrict__ C,
    int ldc, int M, int N, int K, int tiles, int tiles_k, int m_chunk, int nwg, float* __restrict__ slabs) {
  using G = Cfg<TN, TK>;
  __shared__ __attribute__((aligned(16))) bf16_raw smem[NSLOT * G::kSlotElems];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // XCD-aware bijective remap: the 1/8 of the grid dispatched to one XCD gets contiguous work
  const int w = xcd_remap(blockIdx.x, nwg);
  const int chunk = w / tiles, tile = w - chunk * tiles;
  const int tile_n = tile / tiles_k, tile_k = tile - tile_n * tiles_k;
  const int n0 = tile_n * G::BN, k0 = tile_k * G::BK;
  LLMT_DASSERT(n0 < N && k0 < K);
  const int m_begin = chunk * m_chunk;
  const int rows = min(M - m_begin, m_chunk);
  if (rows <= 0) return;
  const int nst = (rows + BM - 1) / BM;

  // buffer descriptors over exactly this chunk's rows: anything past them reads as 0
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A + (long)m_begin * lda), (short)0, rows * lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(B + (long)m_begin * ldb), (short)0, rows * ldb * 2, 0x00020000);

  // DMA op j of this wave covers rows (wave*ops + j) * (512 / W) .. of its operand; lane l
  // lands at LDS chunk (l % (W/8)) of row l / (W/8), holding source chunk (that ^ swizzle)
  constexpr int cpa = G::WA / 8, cpb = G::WB / 8;  // 16-byte chunks per row
  int va[G::kDmaA], vb[G::kDmaB];
#pragma unroll
  for (int j = 0; j < G::kDmaA; ++j) {
    const int row = (wave * G::kDmaA + j) * (1024 / (2 * G::WA)) + lane / cpa;
    const int c = (lane % cpa) ^ ((row & 3) << 2);
    va[j] = (row * lda + n0 + 8 * c) * 2;
  }
#pragma unroll
  for (int j = 0; j < G::kDmaB; ++j) {
    const int row = (wave * G::kDmaB + j) * (1024 / (2 * G::WB)) + lane / cpb;
    const int c = (lane % cpb) ^ ((row & 3) << 2);
    vb[j] = (row * ldb + k0 + 8 * c) * 2;
  }
  const unsigned lds_base = (unsigned)(unsigned long)(lds_void*)smem;
  auto issue = [&](int s) {
    const unsigned slot = lds_base + (unsigned)((s % NSLOT) * G::kSlotElems * 2);
    const int soa = s * BM * lda * 2, sob = s * BM * ldb * 2;
#pragma unroll
    for (int j = 0; j < G::kDmaA; ++j) dma16(slot + (wave * G::kDmaA + j) * 1024, va[j], ra, soa);
#pragma unroll
    for (int j = 0; j < G::kDmaB; ++j) dma16(slot + G::kAElems * 2 + (wave * G::kDmaB + j) * 1024, vb[j], rb, sob);
  };

  const int wn = wave >> 1, wk = wave & 1;
  f32x16 acc[TN][TK];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) acc[i][j] = 0.f;

#pragma unroll
  for (int s = 0; s < NSLOT - 1; ++s)
    if (s < nst) issue(s);

  for (int s = 0; s < nst; ++s) {
    wait_stage_and_barrier<G::kDmaPerStage>(min(nst - 1 - s, NSLOT - 2));  // stage s landed; slot s-1 free
    if (s + NSLOT - 1 < nst) issue(s + NSLOT - 1);
    const bf16_raw* a = smem + (s % NSLOT) * G::kSlotElems;
    const bf16_raw* b = a + G::kAElems;
#pragma unroll
    for (int ks = 0; ks < BM / 16; ++ks) {
      bf16x8 af[TN], bfv[TK];
#pragma unroll
      for (int i = 0; i < TN; ++i) af[i] = tr_frag<G::WA>(a, 16 * ks, wn * 32 * TN + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < TK; ++j) bfv[j] = tr_frag<G::WB>(b, 16 * ks, wk * 32 * TK + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: C[n][k] += acc (rows n in registers, column k on the lane)
  const int half = lane >> 5, col = lane & 31;
#pragma unroll
  for (int i = 0; i < TN; ++i) {
#pragma unroll
    for (int j = 0; j < TK; ++j) {
      const int k = k0 + wk * 32 * TK + 32 * j + col;
      if (k >= K) continue;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int n = n0 + wn * 32 * TN + 32 * i + (rr & 3) + 8 * (rr >> 2) + 4 * half;
        if (n >= N) continue;
        if (slabs != nullptr) slabs[((long)chunk * N + n) * K + k] = acc[i][j][rr];
        else atomicAdd(C + (long)n * ldc + k, acc[i][j][rr]);
      }
    }
  }
}

// The 256x256 tile as a software pipeline, for GEMMs that own the chip (launch_wgrad_gemm's
// `pipe`; the LM head's weight gradient on the main stream).  It needs all 512 registers per lane,
// so no other kernel's wave fits on its SIMDs — on the side stream that starved the main stream's
// small kernels (a column sum queued ~490 us behind it) and cancelled the gain; the side stream
// keeps the kernel above.  Counter passes on the kernel above (qkv at M = 131072, profiles/r2/) put the
// MFMA pipe at 45 % busy: per 32-row stage a wave first issued its 8 LDS-DMA ops (each an asm
// statement with a memory clobber, so no LDS read could move above them), then 20 fragment reads,
// then waited lgkmcnt(0) before its first MFMA — ~1960 cycles per stage for 1024 of MFMA.
// Here, per stage s:
//   top:   s_waitcnt vmcnt(P) lgkmcnt(0) + barrier   (stage s+1 landed everywhere; this wave's
//          reads of stage s, issued one stage earlier, are in registers)
//   body:  8 groups of { 4 fragment reads of stage s+1 ; 4 MFMAs on stage s's registers ;
//          1 LDS-DMA op of stage s+3 }, each group pinned in place by a sched_barrier
// so the DMA issue and the next stage's LDS reads hide under the MFMAs and no read latency is
// exposed.  Fragments are double-buffered in registers (64 + 64 VGPRs beside the 256 AGPR
// accumulators); the stage loop is unrolled by two so the buffers swap by renaming.  DMAs past the
// last stage re-read the last stage into a slot nobody reads again, keeping every wait uniform.
namespace {
constexpr int PT = 4;  // 32x32 tiles per wave edge (4 waves of 128x128 = a 256x256 tile)
constexpr int PW = 64 * PT;
constexpr int PA = BM * PW;               // elements per operand image per stage
constexpr int PSLOT = 2 * PA;
constexpr int PDMA = PA * 2 / 1024 / 4;   // 1-KiB DMA ops per wave per operand per stage (4)
}  // namespace

// PNS ring slots of 32 KiB: 4 (128 KiB, two stages in flight behind the one being read) or 5 (all
// 160 KiB of LDS, three in flight)
template <int PNS>
__global__ __launch_bounds__(kThreads, 1) void wgrad_pipe_kernel(
    const bf16_raw* __restrict__ A, int lda, const bf16_raw* __restrict__ B, int ldb, float* __restrict__ C,
    int ldc, int M, int N, int K, int tiles, int tiles_k, int m_chunk, int nwg, float* __restrict__ slabs,
    int stage_mask) {
  __shared__ __attribute__((aligned(16))) bf16_raw smem[PNS * PSLOT];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int w = xcd_remap(blockIdx.x, nwg);
  const int chunk = w / tiles, tile = w - chunk * tiles;
  const int tile_n = tile / tiles_k, tile_k = tile - tile_n * tiles_k;
  const int n0 = tile_n * PW, k0 = tile_k * PW;
  LLMT_DASSERT(n0 < N && k0 < K);
  const int m_begin = chunk * m_chunk;
  const int rows = min(M - m_begin, m_chunk);
  if (rows <= 0) return;
  const int nst = (rows + BM - 1) / BM;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A + (long)m_begin * lda), (short)0, rows * lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(B + (long)m_begin * ldb), (short)0, rows * ldb * 2, 0x00020000);
  constexpr int cp = PW / 8;  // 16-byte chunks per LDS row
  int va[PDMA], vb[PDMA];
#pragma unroll
  for (int j = 0; j < PDMA; ++j) {
    const int row = (wave * PDMA + j) * (1024 / (2 * PW)) + lane / cp;
    const int c = (lane % cp) ^ ((row & 3) << 2);
    va[j] = (row * lda + n0 + 8 * c) * 2;
    vb[j] = (row * ldb + k0 + 8 * c) * 2;
  }
  const unsigned lds_base = (unsigned)(unsigned long)(lds_void*)smem;
  // DMA op j (0..7: A ops then B ops) of stage `st` into ring slot `slot`
  auto dma = [&](int j, int st, int slot) {
    const unsigned dst = lds_base + (unsigned)(slot * PSLOT * 2);
    if (j < PDMA) dma16(dst + (wave * PDMA + j) * 1024, va[j], ra, st * BM * lda * 2);
    else dma16(dst + PA * 2 + (wave * PDMA + j - PDMA) * 1024, vb[j - PDMA], rb, st * BM * ldb * 2);
  };

  const int wn = wave >> 1, wk = wave & 1;
  f32x16 acc[PT][PT];
#pragma unroll
  for (int i = 0; i < PT; ++i)
#pragma unroll
    for (int j = 0; j < PT; ++j) acc[i][j] = 0.f;

  // fragment f of a stage (0..15): k-step f / 8, operand (f % 8) / 4 (A, B), tile f % 4
  auto read = [&](bf16x8 (&fr)[16], int slot, int f) {
    const bf16_raw* img = smem + slot * PSLOT + ((f & 4) ? PA : 0);
    const int col0 = ((f & 4) ? wk : wn) * 32 * PT + 32 * (f & 3);
    fr[f] = tr_frag<PW>(img, 16 * (f >> 3), col0, lane);
  };

  // prologue: stages 0..PNS-2 in flight, stage 0 landed, its fragments read
#pragma unroll
  for (int s = 0; s < PNS - 1; ++s)
#pragma unroll
    for (int j = 0; j < 2 * PDMA; ++j) dma(j, min(s, nst - 1), s);
  bf16x8 f0[16], f1[16];
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * PDMA * (PNS - 2)) : "memory");
#pragma unroll
  for (int f = 0; f < 16; ++f) read(f0, 0, f);

  // one stage: MFMAs on `cur` (stage s), reads of stage s+1 into `nxt`, DMAs of stage s+PNS-1
  auto stage = [&](int s, bf16x8 (&cur)[16], bf16x8 (&nxt)[16]) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): cur is in registers
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * PDMA * (PNS - 3)) : "memory");
    const int rs = (s + 1) % PNS, ds = (s + PNS - 1) % PNS, dst_stage = min(s + PNS - 1, nst - 1) & stage_mask;
#pragma unroll
    for (int g = 0; g < 8; ++g) {  // g = k-step * 4 + A tile i
      read(nxt, rs, 2 * g);
      read(nxt, rs, 2 * g + 1);
      const int ks = g >> 2, i = g & 3;
#pragma unroll
      for (int j = 0; j < PT; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[8 * ks + i], cur[8 * ks + 4 + j], acc[i][j], 0, 0, 0);
      dma(g, dst_stage, ds);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  int s = 0;
  for (; s + 1 < nst; s += 2) {
    stage(s, f0, f1);
    stage(s + 1, f1, f0);
  }
  if (s < nst) stage(s, f0, f1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup ends

  const int half = lane >> 5, col = lane & 31;
#pragma unroll
  for (int i = 0; i < PT; ++i) {
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int k = k0 + wk * 32 * PT + 32 * j + col;
      if (k >= K) continue;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int n = n0 + wn * 32 * PT + 32 * i + (rr & 3) + 8 * (rr >> 2) + 4 * half;
        if (n >= N) continue;
        if (slabs != nullptr) slabs[((long)chunk * N + n) * K + k] = acc[i][j][rr];
        else atomicAdd(C + (long)n * ldc + k, acc[i][j][rr]);
      }
    }
  }
}

struct Plan {
  int tile = 0, split = 1, m_chunk = 0, tiles = 0, tiles_k = 0;
  double cost = 1e30;
};

// Modelled time of one configuration: rounds of workgroups x per-workgroup MFMA time at the
// tile's measured efficiency, plus the split-K atomic traffic at the chip-wide atomic rate.
Plan plan_for(int tile, int M, int N, int K, int split_req, int ncu, int min_split, bool det) {
  Plan p;
  p.tile = tile;
  const int bn = tile, bk = tile;
  const int tiles_n = (N + bn - 1) / bn;
  p.tiles_k = (K + bk - 1) / bk;
  p.tiles = tiles_n * p.tiles_k;
  const int slots = ncu * (tile == 256 ? 1 : 2);
  // per resident workgroup; chip rates measured at M = 65536 (bench/micro.py wgrad): <4,4> 0.9-1.0 PF
  // on 768..3072-wide outputs, <2,2> 0.76-0.87 PF solo — but inside the step (side stream, sharing
  // the chip) the 128 tile's half arithmetic intensity costs more: modelled at 0.6 PF, GPT-2 XL
  // forced to 256 tiles measured +2.7 % (profiles/r2/ab_xl_wgrad_tile.txt) where 0.85 picked 128
  const double rate_cu = (tile == 256 ? 1.0e15 : 0.6e15) / ncu * (tile == 256 ? 1.0 : 0.5);
  const int max_split = (M + BM - 1) / BM;
  auto eval = [&](int s, Plan& out) {
    int chunk = (M + s - 1) / s;
    chunk = (chunk + BM - 1) / BM * BM;
    const int ss = (M + chunk - 1) / chunk;
    const long long nwg = (long long)p.tiles * ss;
    const long long rounds = (nwg + slots - 1) / slots;
    const double t_wg = 2.0 * chunk * bn * bk / rate_cu;
    // atomics at ~1.3 TB/s chip-wide; deterministic slabs: stored once and read once at ~5 TB/s
    const double t_atomic = det ? (double)nwg * bn * bk * 8.0 / 5e12 : (double)nwg * bn * bk * 4.0 / 1.3e12;
    const double cost = rounds * t_wg + t_atomic;
    if (cost < out.cost) {
      out.cost = cost;
      out.split = ss;
      out.m_chunk = chunk;
    }
  };
  if (split_req > 0) {
    const int s = split_req > min_split ? split_req : min_split;
    eval(s < max_split ? s : max_split, p);
  } else {
    const int hi = max_split < 4 * slots ? max_split : 4 * slots;
    for (int s = min_split; s <= (hi > min_split ? hi : min_split); ++s) eval(s, p);
  }
  return p;
}

}  // namespace wgrad

namespace {
// the launcher's plan (split, tile): shared by the launch and the deterministic workspace query
hipError_t plan_wgrad(int lda, int ldb, int M, int N, int K, int split, int tile, wgrad::Plan& p) {
  if (lda % 8 || ldb % 8 || K % 8 || lda < N) return hipErrorInvalidValue;
  const int ncu = gemm::cu_count();
  // 32-bit buffer offsets: one M chunk of either operand must stay below 2 GiB (wide rows such
  // as the LM head's 50304-column logits force a minimum split)
  const long long row_bytes = 2LL * (lda > ldb ? lda : ldb);
  const int min_split =
      (int)(((long long)M * row_bytes + (1LL << 31) - 1 - 4096) / ((1LL << 31) - 4096 - row_bytes * 32));
  const int ms = min_split > 0 ? min_split : 1;
  const bool det = deterministic();
  if (tile == 128 || tile == 256) {
    p = wgrad::plan_for(tile, M, N, K, split, ncu, ms, det);
  } else {
    const wgrad::Plan a = wgrad::plan_for(256, M, N, K, split, ncu, ms, det);
    const wgrad::Plan b = wgrad::plan_for(128, M, N, K, split, ncu, ms, det);
    p = a.cost <= b.cost ? a : b;
  }
  // 32-bit buffer offsets: one chunk of either operand must stay below 2 GiB
  if ((long long)p.m_chunk * (lda > ldb ? lda : ldb) * 2 >= (1LL << 31)) return hipErrorInvalidValue;
  return hipSuccess;
}
}  // namespace

long wgrad_gemm_det_ws_floats(int lda, int ldb, int M, int N, int K, int split, int tile) {
  if (M <= 0 || N <= 0 || K <= 0 || !deterministic()) return 0;
  wgrad::Plan p;
  if (plan_wgrad(lda, ldb, M, N, K, split, tile, p) != hipSuccess) return 0;
  return (long)p.split * N * K + colsum_scratch_floats(p.split, (long)N * K);
}

hipError_t launch_wgrad_gemm(const void* dy, int lda, const void* x, int ldb, float* c, int ldc, int M, int N,
                             int K, int split, int tile, hipStream_t stream, float* det_ws, int pipe_req) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  // N needs no alignment: tiles past N read the next rows' data (or zeros past the chunk) into
  // accumulators whose stores the epilogue masks with n < N (the LM head's N = 50257)
  wgrad::Plan p;
  const hipError_t e = plan_wgrad(lda, ldb, M, N, K, split, tile, p);
  if (e != hipSuccess) return e;
  const bool det = deterministic();
  if (det && det_ws == nullptr) return hipErrorInvalidValue;
  float* slabs = det ? det_ws : nullptr;
  const int nwg = p.tiles * p.split;
  // the caller picks the software-pipelined 256 tile (pipe_req > 0) for GEMMs that own the chip
  const int pipe = pipe_req > 0 ? pipe_req : 0;
  const int stage_mask = -1;  // (0 = every stage re-reads stage 0: a timing skeleton, never shipped)
  if (p.tile == 256 && pipe != 0) {
    hipLaunchKernelGGL(wgrad::wgrad_pipe_kernel<4>, dim3(nwg), dim3(wgrad::kThreads), 0, stream, (const bf16_raw*)dy,
                       lda, (const bf16_raw*)x, ldb, c, ldc, M, N, K, p.tiles, p.tiles_k, p.m_chunk, nwg, slabs, stage_mask);
  } else if (p.tile == 256) {
    hipLaunchKernelGGL((wgrad::wgrad_kernel<4, 4>), dim3(nwg), dim3(wgrad::kThreads), 0, stream,
                       (const bf16_raw*)dy, lda, (const bf16_raw*)x, ldb, c, ldc, M, N, K, p.tiles, p.tiles_k,
                       p.m_chunk, nwg, slabs);
  } else {
    hipLaunchKernelGGL((wgrad::wgrad_kernel<2, 2>), dim3(nwg), dim3(wgrad::kThreads), 0, stream,
                       (const bf16_raw*)dy, lda, (const bf16_raw*)x, ldb, c, ldc, M, N, K, p.tiles, p.tiles_k,
                       p.m_chunk, nwg, slabs);
  }
  if (det)  // slabs of chunks that had no rows (split > M / BM) were never written: only p.split exist
    return launch_colsum_reduce(slabs, p.split, (long)N * K, c, slabs + (long)p.split * N * K, stream, K, ldc);
  return hipGetLastError();
}

}  // namespace llmt
