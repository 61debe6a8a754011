// Causal flash-attention forward, head_dim <= 64, bf16 in / bf16 out, for gfx950 (MI355X).
//
// Replaces reference models/gpt.py:49-71 (qkv split, Q K^T / sqrt(hd), causal masked_fill,
// softmax, P V), which materialises [B, H, T, T] fp32 scores; here nothing of size T^2 ever
// reaches memory and the kernel reads Q/K/V straight out of the packed projection output
// qkv[B, T, 3, H, 64] (no transpose/contiguous copies) and writes out[B, T, H, 64], i.e. the
// exact operand layout of the following out_proj GEMM.
//
// Structure (CDNA4 idioms from the MI355X playbook):
//  * workgroup = 4 wave64s = a 128-row query block; each wave owns 32 query rows and keeps its
//    Q fragments in registers for the whole key sweep;
//  * "swapped" S^T = K Q^T with v_mfma_f32_32x32x16_bf16: the query index lands on the MFMA
//    lane, so the online-softmax row max / row sum are lane-local (one xor-32 shuffle joins the
//    two lane halves) and the running O^T accumulator is rescaled without any cross-lane move;
//  * the S^T accumulator is converted to bf16 in registers and used directly as the B operand
//    of O^T += V^T P^T (no LDS round trip for P); V^T fragments come from LDS through the gfx950
//    transposing read ds_read_b64_tr_b16;
//  * K/V tiles of 64 keys stream into a 4-slot LDS ring by LDS-DMA three tiles ahead (no VGPR
//    staging), one counted-vmcnt wait + barrier per tile;
//  * software pipelined: the next tile's eight Q K^T MFMAs are interleaved into this tile's
//    mask / max / exp VALU stream, so the matrix pipe runs under the softmax;
//  * one XOR swizzle of the 16-byte chunks of each 128-byte LDS row makes both the row reads
//    (ds_read_b128, K as the A operand) and the transposed reads (V) bank-conflict free;
//  * softmax in the exp2 domain (v_exp_f32), scale folded into one multiply;
//  * heaviest (last) query blocks are dispatched first to shorten the causal tail;
//  * SMALLHD: head dims below 64 (multiples of 8: the reference presets' 32 and 48) run the same
//    64-wide tiles with the missing dims zero-filled at load time and never stored;
//  * KMASK: key-padding mask (reference gpt.py:60-64) from one 64-bit word per 64-key tile (a
//    scalar load: the tile's keys are wave-uniform); padded keys score -inf like future keys.  A
//    row whose keys so far are ALL masked keeps m = -inf: its exponent offset is taken as 0 then
//    (P = exp2(-inf) = 0, no inf - inf), and the first real key rescales with alpha = 0; rows that
//    never saw a real key are written as O = 0, lse = +inf.
#include <type_traits>

#include "attention_common.h"
#include "gemm_common.h"

namespace llmt {
namespace attn {

#ifdef LLMT_ATTN_PROBE
// Timing probe (bench/native/attn_fwd_timer.cpp builds this file with -DLLMT_ATTN_PROBE): lane 0 of
// each wave of the (b, h) = 0 workgroups stores s_memtime stamps [qb][wave][event]: 0 entry, 1 after
// the prologue, 2 + 2 it after step it's compute, 3 + 2 it after its barrier, 63 exit.
__device__ unsigned long long* g_attn_probe = nullptr;  // null: no stamps
// Every workgroup's wave 0 also stores its entry / exit stamps (events 0 / 63) to
// g_attn_probe[nqb * kFwdWaves * 64 + 4 * (bh * nqb + qb) + {0, 1}] (s_memtime) and
// + {2, 3} (s_memrealtime: 100 MHz, one clock for the whole chip).
#define ATTN_PROBE(ev)                                                                                   \
  do {                                                                                                   \
    if (g_attn_probe != nullptr && (threadIdx.x & 63) == 0) {                                            \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                        \
      if (blockIdx.x == 0 && (ev) < 64)                                                                  \
        g_attn_probe[((long)(nqb - 1 - (int)blockIdx.y) * kFwdWaves + (threadIdx.x >> 6)) * 64 + (ev)] = t_; \
      if (threadIdx.x == 0 && ((ev) == 0 || (ev) == 63)) {                                               \
        unsigned long long* g_ = g_attn_probe + (long)nqb * kFwdWaves * 64 + 4 * ((long)blockIdx.x * nqb + nqb - 1 - blockIdx.y); \
        g_[(ev) == 63] = t_;                                                                             \
        g_[2 + ((ev) == 63)] = __builtin_amdgcn_s_memrealtime();                                         \
      }                                                                                                  \
    }                                                                                                    \
  } while (0)
#else
#define ATTN_PROBE(ev) \
  do {                 \
  } while (0)
#endif

constexpr int kFwdWaves = 4;
constexpr int kQBlk = 32 * kFwdWaves;  // 128 query rows per workgroup
constexpr int kKBlk = 64;              // keys per LDS tile
constexpr int kRing = 4;               // K/V tiles resident in LDS (2 computing + 2 in flight)

// lane-half exchange (x[l ^ 32]) as one VALU op (v_permlane32_swap) instead of a ds_bpermute
__device__ __forceinline__ float half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <bool DROPOUT, bool KMASK, bool SMALLHD>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(const bf16_raw* __restrict__ qkv,
                                                          bf16_raw* __restrict__ out,
                                                          float* __restrict__ lse, int T, int H,
                                                          int nqb, DropoutArgs dr, int hd_arg, float c_arg,
                                                          const uint64_t* __restrict__ key_bits) {
  // ring of four K/V tiles: tile it (P V), tile it+1 (Q K^T of the next step, software pipelined
  // under this step's softmax) and tiles it+2, it+3 (LDS-DMA in flight) -- 64 KiB, two
  // workgroups per CU
  __shared__ __attribute__((aligned(16))) bf16_raw smem[kRing][2][kKBlk * kHD];  // [slot][K|V][tile]
  const int lane = threadIdx.x & 63;
  // readfirstlane makes the wave index (and every tile/mask decision derived from it) provably
  // wave-uniform, so hipcc emits scalar branches instead of per-lane exec-mask control flow
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = lane >> 5, col = lane & 31;
  // grid (B*H, nqb), x fastest: dispatch runs through ALL (b, h) of the heaviest (last) query
  // block first, so the grid ends on the lightest blocks instead of a tail of heavy ones (with
  // (b, h) outermost the last-dispatched heavy blocks left ~40% of the workgroup slots idle at the
  // end: 315 of 512 resident on average, bench/native/attn_fwd_timer probe).  All blocks of one
  // (b, h) land on the same XCD (B*H is a multiple of 8 at the model shapes), sharing K/V in L2.
  const int qb = nqb - 1 - (int)blockIdx.y;
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh - b * H;
  const int hd = SMALLHD ? hd_arg : kHD;  // head dim in memory; tiles stay 64 wide
  const long row_stride = 3L * H * hd;   // elements between consecutive tokens in qkv
  const bf16_raw* base = qkv + (long)b * T * row_stride + (long)h * hd;
  // attention-probability dropout: plane seed per (b, h), element index q*T + key
  const uint32_t pseed = DROPOUT ? mix32(dr.seed + (uint32_t)bh * 0x9E3779B9u) : 0u;

  const int q0w = qb * kQBlk + wave * 32;   // first query row of this wave
  const int q = q0w + col;                   // this lane's query row
  const int q_hi = min(q0w + 31, T - 1);     // last valid query row of the wave

  bf16x8 qf[4];  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q][16kk + 8*half + 0..7]
  const int kv_end = min(T, qb * kQBlk + kQBlk);
  const int ntiles = (kv_end + kKBlk - 1) / kKBlk;  // tiles the workgroup stages
  // tiles this wave computes: its rows see keys up to q_hi (wave-uniform, always >= 1)
  const int wave_tiles = __builtin_amdgcn_readfirstlane(min(ntiles, q_hi / kKBlk + 1));

  // K/V tiles stream straight into the LDS ring by LDS-DMA (buffer_load_dwordx4 ... lds, no VGPR
  // staging): a tile is 16 one-KiB DMA ops (8 rows x 8 chunks each), 4 per wave.  The DMA
  // destination is lane-linear, so the chunk swizzle is applied to the SOURCE: lane l of op j
  // lands at row 8j + l/8, slot l%8 and loads chunk (l%8) ^ g(row).  Buffer loads are bounded at
  // row T of this (b, h) (keys past the sequence land as zeros); chunks past a small head dim use
  // an out-of-record offset (zeros, never a read past the end of the qkv allocation).
  // One buffer resource per tile (scalar work): based at the tile's first key, bounded at the
  // sequence end, so the per-lane offsets below stay loop-invariant.
  const long record = (((long)T - 1) * row_stride + 3 * hd * H) * 2;  // bytes of this (b, h)'s qkv
  const long tile_bytes = (long)kKBlk * row_stride * 2;
  int voff[4];  // per op: byte offset inside a tile (an out-of-record offset for dead chunks)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int op = wave * 4 + j;            // 0..15: ops 0..7 = K rows 8op.., 8..15 = V
    const int row = 8 * (op & 7) + (lane >> 3);
    const int ch = swz(row, lane & 7);  // the chunk LDS slot lane%8 of this row holds
    const bool live = !SMALLHD || ch * 8 < hd;
    voff[j] = live ? (int)(((long)row * row_stride + ch * 8 + hd * H * (1 + (op >> 3))) * 2) : kOobOff;
  }
  const unsigned lds_base = (unsigned)(unsigned long)(gemm::lds_void*)&smem[0][0][0];
  auto dma_tile = [&](int tile, int slot) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)base + tile * tile_bytes), (short)0, (int)max(0L, record - tile * tile_bytes), 0x00020000);
    const unsigned slot_base = lds_base + (unsigned)(slot * 2 * kKBlk * kHD * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int op = wave * 4 + j;
      const unsigned dst = slot_base + (unsigned)((op >> 3) * kKBlk * kHD * 2 + (op & 7) * 1024);
      gemm::dma16(dst, voff[j], r, 0);
    }
  };
  // end of a step: the next tile to compute has landed (the newest tile's 4 ops may still fly)
  auto land_and_barrier = [&](bool newest_in_flight) {
    if (newest_in_flight) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  };

  f32x16 o[2];
  o[0] = 0.f;
  o[1] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const float c = SMALLHD ? c_arg : 0.125f * 1.4426950408889634f;  // softmax scale * log2(e)
  const int nkw = (T + kKBlk - 1) / kKBlk;  // key-mask words per sequence

  // K fragments of a tile (A operand of S^T = K Q^T), all eight read before the first MFMA
  auto read_k = [&](bf16x8(&kf)[8], int slot) {
    const bf16_raw* Kt = smem[slot][0];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) kf[4 * kt + kk] = lds_row_read(Kt, kt * 32 + col, 2 * kk + half);
  };
  // one MFMA of the next tile's S, fenced so the scheduler keeps it where it is placed in the
  // VALU stream (otherwise it clusters the MFMAs and the softmax serialises behind them)
  auto qk_mfma = [&](f32x16(&s)[2], const bf16x8(&kf)[8], int i) {
    const int kt = i >> 2, kk = i & 3;
    __builtin_amdgcn_sched_barrier(0);
    s[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[i], qf[kk], kk == 0 ? f32x16{} : s[kt], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // One pipelined step: S of tile it (in s_cur, computed during the previous step) -> masks, online
  // softmax, P V; the eight MFMAs of the NEXT tile's S (into s_nxt) are interleaved with this
  // step's VALU work, so the matrix pipe runs under the exp/max/sum of the softmax.
  // NEXT (compile-time): whether this wave also computes the next tile's S.  The three shapes of a
  // step -- current + next, current only (the wave's last tile), none (the wave is done but the
  // workgroup still stages tiles) -- are separate straight-line bodies selected by one
  // wave-uniform branch, so nothing inside the interleaved MFMA/VALU stream is conditional.
  // slot: tile it's ring slot (== it % kRing, a literal at every call site)
  auto compute = [&](auto NEXT, int it, int slot, f32x16(&s_cur)[2], f32x16(&s_nxt)[2]) __attribute__((always_inline)) {
    constexpr bool next = decltype(NEXT)::value;
    bf16x8 kf[8];
    if (next) {
      read_k(kf, (slot + 1) % kRing);  // issued first: ~50-cycle LDS latency hidden by the masks / max
      __builtin_amdgcn_sched_barrier(0);
    }
    {
      const int kbase = it * kKBlk;
      f32x16(&s)[2] = s_cur;
      if (next) qk_mfma(s_nxt, kf, 0);
      if (KMASK) {  // key padding: one word for the tile's 64 keys (wave-uniform scalar load)
        const uint64_t mw = key_bits[(long)b * nkw + it];
        if (mw != ~0ull) {
          const uint64_t ml = mw >> (4 * half);  // register r of this lane half is key bit (r&3)+8(r>>2)+32kt
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              s[kt][r] = ((ml >> ((r & 3) + 8 * (r >> 2) + 32 * kt)) & 1ull) ? s[kt][r] : -INFINITY;
        }
      }
      // causal / sequence-end mask (diagonal tiles only), on RAW scores: the softmax scale is
      // folded into the exponent below (one FMA per score instead of mul + sub)
      const bool need_mask = (kbase + kKBlk - 1 > q0w) || (kbase + kKBlk > T);  // wave-uniform
      if (need_mask) {
        // key offset within the tile, (r&3) + 8(r>>2) + 4*half + 32*kt, must be <= lim
        const int lim = min(q, T - 1) - kbase - 4 * half;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            s[kt][r] = ((r & 3) + 8 * (r >> 2) + 32 * kt > lim) ? -INFINITY : s[kt][r];
      }
      if (next) qk_mfma(s_nxt, kf, 1);
      float tmax = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, s[kt][r]);
      tmax = half_max(tmax);
      if (next) qk_mfma(s_nxt, kf, 2);
      // lazy rescale: keep a stale running max while no row's max grew by more than 2^8 in
      // probability (P <= 256 is exact enough in fp32 and bf16; l and O use the same stale max,
      // so the result is unchanged).  The O/l rescale (16 packed muls + one exp per lane) then
      // runs only on the few tiles where some row of the wave jumps, wave-uniformly.  The first
      // tile always rescales (m_run = -inf), and tile 0 gives every row a finite max.
      if (__builtin_amdgcn_ballot_w64((tmax - m_run) * c > 8.f) != 0) {
        const float m_new = fmaxf(m_run, tmax);  // raw-score units
        // (KMASK: a lane still without any real key has m_new = -inf; -inf - -inf would be NaN)
        const float alpha = (KMASK && m_new == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f((m_run - m_new) * c);
        l_run *= alpha;
        o[0] *= alpha;
        o[1] *= alpha;
        m_run = m_new;
      }
      // an all-masked row so far (KMASK only) has m = -inf: offset 0 gives P = 0, not NaN
      const float mc = (KMASK && m_run == -INFINITY) ? 0.f : m_run * c;
      float psum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[kt][r], c, -mc));  // v_exp_f32, no denorm fixup
          s[kt][r] = p;
          psum += p;
          // the next tile's remaining S MFMAs, one per 6 exponentials (flat score 5, 11, ..., 29)
          if (next && (16 * kt + r) % 6 == 5) qk_mfma(s_nxt, kf, 3 + (16 * kt + r) / 6);
        }
      }
      psum = half_sum(psum);
      if (DROPOUT) {  // the normaliser sums the undropped P; P V uses the masked, rescaled P
        const uint32_t e_q = (uint32_t)q * (uint32_t)T + (uint32_t)(kbase + 4 * half);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint32_t e = e_q + (uint32_t)(kt * 32 + (r & 3) + 8 * (r >> 2));
            s[kt][r] = drop_keep(pseed, dr.thr, e) ? s[kt][r] * dr.scale : 0.f;
          }
      }
      l_run += psum;
      // O^T += V^T P^T: P^T (the S^T accumulator) is the B operand straight from registers
      const bf16_raw* Vt = smem[slot][1];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int st2 = 0; st2 < 2; ++st2) {
          const bf16x8 pb = pack_acc8(s[kt], st2);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const bf16x8 va = lds_tr_read_operand(Vt, kt * 32 + 16 * st2 + 4 * half, dt * 32, lane);
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb, o[dt], 0, 0, 0);
          }
        }
      }
    }
  };
  // one tile step of the workgroup: stage tile it+3 into the slot tile it-1 left (its P V finished
  // before the last barrier), compute tile it, then make tile it+2 visible to every wave.  Every
  // wave runs exactly ntiles steps (ntiles barriers), computing or not.
  auto step = [&](auto NEXT, int it, int slot, f32x16(&s_cur)[2], f32x16(&s_nxt)[2]) __attribute__((always_inline)) {
    if (it + 3 < ntiles) dma_tile(it + 3, (slot + 3) % kRing);
    compute(NEXT, it, slot, s_cur, s_nxt);
    ATTN_PROBE(2 + 2 * it);
    land_and_barrier(it + 3 < ntiles);
    ATTN_PROBE(3 + 2 * it);
  };
  const std::true_type nxt;
  const std::false_type last;

  ATTN_PROBE(0);
  // prologue: tiles 0..2 and Q in flight together (one memory round trip, not two); tiles 0 and 1
  // landed -> S of tile 0.  The Q loads are the compiler's own, issued after the DMA ops, so its
  // wait before the first use of qf (vmcnt(0)) also covers the DMAs it cannot see.
  dma_tile(0, 0);
  dma_tile(1, 1);  // past the sequence end / the causal range: zeros, harmless, keeps the count fixed
  dma_tile(2, 2);
  {
    // branch-free buffer loads (rows past T / chunks past hd read as zeros), so every wave issues
    // exactly 4 of them after its 12 DMA ops: vmcnt(4) below then means tiles 0..2 have landed
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)record, 0x00020000);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const bool live = q < T && (!SMALLHD || 16 * kk + 8 * half < hd);
      const int off = live ? (int)(((long)q * row_stride + 16 * kk + 8 * half) * 2) : kOobOff;
      qf[kk] = __builtin_bit_cast(bf16x8, buf_load16(rq, off));
    }
  }
  land_and_barrier(true);
  f32x16 sA[2], sB[2];
  {
    bf16x8 kf[8];
    read_k(kf, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) qk_mfma(sA, kf, i);
  }
  ATTN_PROBE(1);
  // Steady state unrolled by the ring depth with no per-step branches: every LDS slot index is a
  // compile-time constant (K / V^T fragment reads = a few per-lane base registers + immediate
  // offsets) and the S accumulators alternate statically (conditional steps made the register
  // allocator keep copies of them, and spill).
  int it = 0;
  for (; it + kRing < wave_tiles; it += kRing) {
    step(nxt, it, 0, sA, sB);
    step(nxt, it + 1, 1, sB, sA);
    step(nxt, it + 2, 2, sA, sB);
    step(nxt, it + 3, 3, sB, sA);
  }
  // the wave's last 1..4 tiles (it % kRing == 0 here), the last one without a next S
  switch (wave_tiles - it) {
    case 1:
      step(last, it, 0, sA, sB);
      break;
    case 2:
      step(nxt, it, 0, sA, sB);
      step(last, it + 1, 1, sB, sA);
      break;
    case 3:
      step(nxt, it, 0, sA, sB);
      step(nxt, it + 1, 1, sB, sA);
      step(last, it + 2, 2, sA, sB);
      break;
    default:
      step(nxt, it, 0, sA, sB);
      step(nxt, it + 1, 1, sB, sA);
      step(nxt, it + 2, 2, sA, sB);
      step(last, it + 3, 3, sB, sA);
      break;
  }
  // tiles the workgroup still stages past this wave's diagonal: barriers only (no DMA is left to
  // issue: tile wave_tiles+3 >= ntiles)
  for (it = wave_tiles; it < ntiles; ++it) land_and_barrier(false);

  if (q < T) {
    // a row that never saw an unpadded key: O = 0 and lse = +inf (P = 0 in the backward)
    const bool dead = KMASK && m_run == -INFINITY;
    const float inv_l = dead ? 0.f : 1.f / l_run;
    bf16_raw* dst = out + ((long)b * T + q) * H * hd + (long)h * hd;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        ushort4_t v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = f2bf(o[dt][4 * g + i] * inv_l);
        const int d = dt * 32 + 8 * g + 4 * half;
        if (!SMALLHD || d < hd) *reinterpret_cast<ushort4_t*>(dst + d) = v;
      }
    }
    if (half == 0)
      lse[((long)b * H + h) * T + q] = dead ? INFINITY : (m_run * c + log2f(l_run)) * 0.6931471805599453f;
  }
  ATTN_PROBE(63);
}

}  // namespace attn

#ifdef LLMT_ATTN_PROBE
void attn_probe_set(unsigned long long* buf) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(attn::g_attn_probe), &buf, sizeof(buf));
}
#endif

template <bool DROPOUT, bool KMASK, bool SMALLHD>
static void launch_fwd_variant(dim3 grid, hipStream_t stream, const bf16_raw* qkv, bf16_raw* out, float* lse,
                               const AttnDims& d, int nqb, DropoutArgs dr) {
  hipLaunchKernelGGL((attn::attn_fwd_kernel<DROPOUT, KMASK, SMALLHD>), grid, dim3(256), 0, stream, qkv, out, lse, d.T,
                     d.H, nqb, dr, d.hd, d.scale * 1.4426950408889634f, d.key_bits);
}

hipError_t launch_attn_fwd(const void* qkv, void* out, float* lse, const AttnDims& d, DropoutArgs dropout,
                           hipStream_t stream) {
  if (d.B <= 0 || d.T <= 0 || d.H <= 0 || d.T > 65535 || d.hd <= 0 || d.hd > attn::kHD || d.hd % 8 != 0)
    return hipErrorInvalidValue;
  const int nqb = (d.T + attn::kQBlk - 1) / attn::kQBlk;
  dim3 grid(d.B * d.H, nqb);
  const bool drop = dropout.thr != 0, km = d.key_bits != nullptr, small = d.hd != attn::kHD;
  const int variant = (drop ? 4 : 0) | (km ? 2 : 0) | (small ? 1 : 0);
  auto q = (const bf16_raw*)qkv;
  auto o = (bf16_raw*)out;
  switch (variant) {
    case 0: launch_fwd_variant<false, false, false>(grid, stream, q, o, lse, d, nqb, dropout); break;
    case 1: launch_fwd_variant<false, false, true>(grid, stream, q, o, lse, d, nqb, dropout); break;
    case 2: launch_fwd_variant<false, true, false>(grid, stream, q, o, lse, d, nqb, dropout); break;
    case 3: launch_fwd_variant<false, true, true>(grid, stream, q, o, lse, d, nqb, dropout); break;
    case 4: launch_fwd_variant<true, false, false>(grid, stream, q, o, lse, d, nqb, dropout); break;
    case 5: launch_fwd_variant<true, false, true>(grid, stream, q, o, lse, d, nqb, dropout); break;
    case 6: launch_fwd_variant<true, true, false>(grid, stream, q, o, lse, d, nqb, dropout); break;
    default: launch_fwd_variant<true, true, true>(grid, stream, q, o, lse, d, nqb, dropout); break;
  }
  return hipGetLastError();
}

}  // namespace llmt
