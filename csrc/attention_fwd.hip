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
//  * K/V tiles of 64 keys are double-buffered in LDS and filled by LDS-DMA (buffer_load ... lds;
//    each lane's source chunk chosen so the image lands swizzled), one tile ahead, one barrier per
//    tile.  Without staging registers the kernel fits 128 VGPRs, i.e. FOUR workgroups (16 waves)
//    per CU instead of three: 0.391-0.393 vs 0.406-0.410 ms at GPT-2 124M micro-batch 128,
//    0.216 vs 0.223-0.231 at XL (profiles/r6/attn/fwd_lds_dma_4wg_ab.txt).  hd = 128 (NH = 2) keeps
//    register staging two tiles ahead;
//  * one XOR swizzle of the 16-byte chunks of each 128-byte LDS row makes both the row reads
//    (ds_read_b128, K as the A operand) and the transposed reads (V) bank-conflict free;
//  * softmax in the exp2 domain (v_exp_f32), scale folded into one multiply;
//  * heaviest (last) query blocks of ALL (b, h) are dispatched first to shorten the causal tail;
//  * measured alternatives: K/V by LDS-DMA into a 4-slot ring with the next tile's Q K^T MFMAs
//    interleaved into this tile's softmax (commit f15d290) ran 2-7% SLOWER than register staging,
//    and so did a cross-tile pipeline (softmax of tile j beside the S MFMAs of tile j + 1, 8-13%,
//    docs/round6.md section 18): the loop is bound by VALU issue (~130 VALU per 16 MFMA per
//    wave-tile), and what pays is more resident waves, not intra-wave pipelining;
//  * SMALLHD: head dims below 64 (multiples of 8: the reference presets' 32 and 48) run the same
//    64-wide tiles with the missing dims zero-filled at load time and never stored;
//  * KMASK: key-padding mask (reference gpt.py:60-64) from one 64-bit word per 64-key tile (a
//    scalar load: the tile's keys are wave-uniform); padded keys score -inf like future keys.  A
//    row whose keys so far are ALL masked keeps m = -inf: its exponent offset is taken as 0 then
//    (P = exp2(-inf) = 0, no inf - inf), and the first real key rescales with alpha = 0; rows that
//    never saw a real key are written as O = 0, lse = +inf.

#include "attention_common.h"

namespace llmt {
namespace attn {

#ifdef LLMT_ATTN_PROBE
// Timing probe (bench/native/attn_fwd_timer.cpp builds this file with -DLLMT_ATTN_PROBE): lane 0 of
// each wave of the (b, h) = 0 workgroups stores s_memtime stamps [qb][wave][event]: 0 entry, 1 after
// the prologue, 2 + 2 it after tile it's compute, 3 + 2 it after its barrier, 63 exit.  Every
// workgroup's wave 0 also stores its entry / exit stamps (events 0 / 63) to
// g_attn_probe[nqb * kFwdWaves * 64 + 4 * (bh * nqb + qb) + {0, 1}] (s_memtime) and + {2, 3}
// (s_memrealtime: 100 MHz, one clock for the whole chip).
__device__ unsigned long long* g_attn_probe = nullptr;  // null: no stamps
#define ATTN_PROBE(ev)                                                                                   \
  do {                                                                                                   \
    if (g_attn_probe != nullptr && (threadIdx.x & 63) == 0) {                                            \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                        \
      if (bh == 0 && (ev) < 64)                                                                          \
        g_attn_probe[((long)qb * kFwdWaves + (threadIdx.x >> 6)) * 64 + (ev)] = t_;                      \
      if (threadIdx.x == 0 && ((ev) == 0 || (ev) == 63)) {                                               \
        unsigned long long* g_ = g_attn_probe + (long)nqb * kFwdWaves * 64 + 4 * ((long)bh * nqb + qb);  \
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

// one tile's K and V rows of this wave (2 + 2 one-KiB LDS-DMA ops), M0 saved / restored
__device__ __forceinline__ void dma_kv(unsigned lds_k, unsigned lds_v, int v0, int v1, __amdgpu_buffer_rsrc_t r,
                                       int sk, int sv) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %[keep], m0\n\t"
      "s_mov_b32 m0, %[dk]\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[v0], %[r], %[sk] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[v1], %[r], %[sk] offen lds\n\t"
      "s_mov_b32 m0, %[dv]\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[v0], %[r], %[sv] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[v1], %[r], %[sv] offen lds\n\t"
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [dk] "s"(lds_k), [dv] "s"(lds_v), [v0] "v"(v0), [v1] "v"(v1), [r] "s"(r), [sk] "s"(sk), [sv] "s"(sv)
      : "memory", "scc");
}

// NH: 64-wide halves of the head dim (1: hd <= 64; 2: hd = 128, every [64][128] K/V tile kept as two
// [64][64] LDS images so the swizzle and fragment readers stay the 64-wide ones)
template <bool DROPOUT, bool KMASK, bool SMALLHD, int NH = 1>
__global__ __launch_bounds__(256, NH == 1 ? 4 : 2) void attn_fwd_kernel(const bf16_raw* __restrict__ qkv,
                                                          bf16_raw* __restrict__ out,
                                                          float* __restrict__ lse, int T, int H,
                                                          int nqb, DropoutArgs dr, int hd_arg, float c_arg,
                                                          const uint64_t* __restrict__ key_bits) {
  resolve_dropout(dr);
  __shared__ __attribute__((aligned(16))) bf16_raw smem[2][2][NH][kKBlk * kHD];  // [buf][K|V][half][tile]
  const int lane = threadIdx.x & 63;
  // readfirstlane makes the wave index (and every tile/mask decision derived from it) provably
  // wave-uniform, so hipcc emits scalar branches instead of per-lane exec-mask control flow
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = lane >> 5, col = lane & 31;
  // grid (B*H, nqb): chunked heaviest-first dispatch (attention_common.h chunked_dispatch); the
  // last query block is the heaviest.  (With (b, h) outermost the last-dispatched heavy blocks left
  // ~40% of the workgroup slots idle at the end: 315 of 512 resident on average,
  // bench/native/attn_fwd_timer probe.)
  int bh, qrank;
  chunked_dispatch(bh, qrank);
  const int qb = nqb - 1 - qrank;
  const int b = bh / H, h = bh - b * H;
  const int hd = SMALLHD ? hd_arg : kHD * NH;  // head dim in memory; tiles stay 64 wide
  const long row_stride = 3L * H * hd;   // elements between consecutive tokens in qkv
  const bf16_raw* base = qkv + (long)b * T * row_stride + (long)h * hd;
  // attention-probability dropout: plane seed per (b, h), element index q*T + key
  const uint32_t pseed = DROPOUT ? mix32(dr.seed + (uint32_t)bh * 0x9E3779B9u) : 0u;

  const int q0w = qb * kQBlk + wave * 32;   // first query row of this wave
  const int q = q0w + col;                   // this lane's query row
  const int q_hi = min(q0w + 31, T - 1);     // last valid query row of the wave

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q][16kk + 8*half + 0..7]
  bf16x8 qf[4 * NH];
#pragma unroll
  for (int kk = 0; kk < 4 * NH; ++kk) {
    ushort8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (q < T && (!SMALLHD || 16 * kk + 8 * half < hd))
      v = *reinterpret_cast<const ushort8_t*>(base + (long)q * row_stride + 16 * kk + 8 * half);
    qf[kk] = __builtin_bit_cast(bf16x8, v);
  }
  if (NH == 1) {
    // retire the Q loads here: the compiler counts only its own VMEM ops, so a first use of qf inside
    // the tile loop would get a counted wait there that also drains the in-flight K/V LDS-DMA
#pragma unroll
    for (int kk = 0; kk < 4 * NH; ++kk) asm volatile("" : "+v"(qf[kk]));
  }

  const int kv_end = min(T, qb * kQBlk + kQBlk);
  const int ntiles = (kv_end + kKBlk - 1) / kKBlk;

  // register staging of K/V tiles TWO tiles ahead (two stage sets): a tile's global loads get two
  // iterations of compute to land instead of one.  Buffer loads bounded at row T of this (b, h):
  // keys past the sequence read as zeros without branches.
  const __amdgpu_buffer_rsrc_t rkv = __builtin_amdgcn_make_buffer_rsrc(
      (void*)base, (short)0, (int)(((long)T - 1) * row_stride + 3 * hd * H) * 2, 0x00020000);
  constexpr int kCh = 2 * NH;  // 16-byte chunks per thread per K (and per V) tile
  ushort8_t st0[2 * kCh], st1[2 * kCh];
  auto load_tile = [&](ushort8_t(&st)[2 * kCh], int tile) {
#pragma unroll
    for (int i = 0; i < kCh; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int r = c / (8 * NH), ch = c % (8 * NH);
      // chunks past a small head dim are never read: an offset past the descriptor's record
      // count loads zeros (reading them would run past the last head of the last token, i.e.
      // past the end of the qkv allocation, by (64 - hd) * 2 bytes)
      const bool live = !SMALLHD || ch * 8 < hd;
      const int off = live ? (int)(((long)(tile * kKBlk + r) * row_stride + ch * 8 + hd * H) * 2) : kOobOff;
      const int off_v = live ? off + hd * H * 2 : kOobOff;
      st[i] = __builtin_bit_cast(ushort8_t, __builtin_amdgcn_raw_buffer_load_b128(rkv, off, 0, 0));
      st[kCh + i] = __builtin_bit_cast(ushort8_t, __builtin_amdgcn_raw_buffer_load_b128(rkv, off_v, 0, 0));
    }
  };
  auto store_tile = [&](const ushort8_t(&st)[2 * kCh], int buf) {
#pragma unroll
    for (int i = 0; i < kCh; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int r = c / (8 * NH), ch = c % (8 * NH);
      const int off = tile_chunk_off(r, ch & 7);
      *reinterpret_cast<ushort8_t*>(&smem[buf][0][ch >> 3][off]) = st[i];
      *reinterpret_cast<ushort8_t*>(&smem[buf][1][ch >> 3][off]) = st[kCh + i];
    }
  };

  f32x16 o[2 * NH];
#pragma unroll
  for (int dt = 0; dt < 2 * NH; ++dt) o[dt] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const float c = (SMALLHD || NH != 1) ? c_arg : 0.125f * 1.4426950408889634f;  // softmax scale * log2(e)
  const int nkw = (T + kKBlk - 1) / kKBlk;  // key-mask words per sequence

  ATTN_PROBE(0);
  constexpr bool kDma = NH == 1;  // K/V by LDS-DMA (hd <= 64); register staging for hd = 128
  // LDS-DMA fills (kDma): op i of wave w fills rows 8 (2w + i) .. + 7 of the K (V) image, lane l
  // the 16-byte chunk (l & 7) of row 8 (2w + i) + (l >> 3), i.e. logical chunk (l & 7) ^ g(row)
  int voff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 8 * (2 * (threadIdx.x >> 6) + i) + (lane >> 3);
    const int ch = swz(row, lane & 7);
    voff[i] = (!SMALLHD || ch * 8 < hd) ? (int)((row * row_stride + ch * 8 + hd * H) * 2) : kOobOff;
  }
  auto issue = [&](int tile, int buf) {
    const unsigned dst = (unsigned)(unsigned long)(lds_void*)&smem[buf][0][0][0] + (unsigned)(wave * 2048);
    const int sk = (int)((long)tile * kKBlk * row_stride * 2);
    dma_kv(dst, dst + kKBlk * kHD * NH * 2, voff[0], voff[1], rkv, sk, sk + hd * H * 2);
  };
  if (kDma) {
    issue(0, 0);
    if (ntiles > 1) issue(1, 1);
    if (ntiles > 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  } else {
    load_tile(st0, 0);
    store_tile(st0, 0);
    __syncthreads();
    if (ntiles > 1) load_tile(st1, 1);
    if (ntiles > 2) load_tile(st0, 2);
  }
  ATTN_PROBE(1);

  // iteration `it` computes from LDS buffer it&1, then stages tile it+1 (held in stage set
  // (it+1)&1 since two iterations ago) into the other buffer and refills that set with tile it+3
  auto tile_step = [&](int it, ushort8_t(&st_next)[2 * kCh]) __attribute__((always_inline)) {
    const int cur = it & 1;
    const bool more = it + 1 < ntiles;
    const int kbase = it * kKBlk;
    if (kbase <= q_hi) {
      f32x16 s[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = 0.f;
#pragma unroll
        for (int kk = 0; kk < 4 * NH; ++kk) {
          const bf16x8 a = lds_row_read(smem[cur][0][kk >> 2], kt * 32 + col, 2 * (kk & 3) + half);
          s[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[kk], s[kt], 0, 0, 0);
        }
      }
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
      // causal / sequence-end mask (diagonal tiles only) and the tile max, on RAW scores: the
      // softmax scale is folded into the exponent below (one FMA per score instead of mul + sub)
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
      float tmax = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, s[kt][r]);
      tmax = halves_max(tmax);
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
#pragma unroll
        for (int dt = 0; dt < 2 * NH; ++dt) o[dt] *= alpha;
        m_run = m_new;
      }
      // an all-masked row so far (KMASK only) has m = -inf: offset 0 gives P = 0, not NaN
      const float mc = (KMASK && m_run == -INFINITY) ? 0.f : m_run * c;
      // exponent arguments and the row sum in packed fp32 (v_pk_fma_f32 / v_pk_add_f32: half the
      // VALU issue of the scalar forms; the loop is VALU-issue bound).  The sum stays per lane half
      // (this lane's 32 keys of the tile): l_run is joined across the halves once, after the sweep.
      const f32x2 cc = {c, c}, nmc = {-mc, -mc};
      f32x2 ps = {0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const f32x2 x = {s[kt][r], s[kt][r + 1]};
          const f32x2 y = __builtin_elementwise_fma(x, cc, nmc);
          const f32x2 p = {__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};  // v_exp_f32
          s[kt][r] = p[0];
          s[kt][r + 1] = p[1];
          ps += p;
        }
      }
      const float psum = ps[0] + ps[1];
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
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pb = pack_acc8(s[kt], st);
#pragma unroll
          for (int dt = 0; dt < 2 * NH; ++dt) {
            const bf16x8 va = lds_tr_read_operand(smem[cur][1][dt >> 1], kt * 32 + 16 * st + 4 * half, (dt & 1) * 32, lane);
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb, o[dt], 0, 0, 0);
          }
        }
      }
    }
    ATTN_PROBE(2 + 2 * it);
    if (kDma) {  // tile it + 1 landed; every wave is past tile it's buffer: refill it with it + 2
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      ATTN_PROBE(3 + 2 * it);
      if (it + 2 < ntiles) issue(it + 2, cur);
    } else {
      if (more) store_tile(st_next, cur ^ 1);
      __syncthreads();
      ATTN_PROBE(3 + 2 * it);
      if (it + 3 < ntiles) load_tile(st_next, it + 3);
    }
  };
  for (int it = 0; it < ntiles; it += 2) {
    tile_step(it, st1);
    if (it + 1 < ntiles) tile_step(it + 1, st0);
  }

  l_run = halves_sum(l_run);  // both key halves of the row (every rescale hit both alike)
  if (q < T) {
    // a row that never saw an unpadded key: O = 0 and lse = +inf (P = 0 in the backward)
    const bool dead = KMASK && m_run == -INFINITY;
    const float inv_l = dead ? 0.f : 1.f / l_run;
    bf16_raw* dst = out + ((long)b * T + q) * H * hd + (long)h * hd;
#pragma unroll
    for (int dt = 0; dt < 2 * NH; ++dt) {
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

template <bool DROPOUT, bool KMASK, bool SMALLHD, int NH = 1>
static void launch_fwd_variant(dim3 grid, hipStream_t stream, const bf16_raw* qkv, bf16_raw* out, float* lse,
                               const AttnDims& d, int nqb, DropoutArgs dr) {
  hipLaunchKernelGGL((attn::attn_fwd_kernel<DROPOUT, KMASK, SMALLHD, NH>), grid, dim3(256), 0, stream, qkv, out, lse,
                     d.T, d.H, nqb, dr, d.hd, d.scale * 1.4426950408889634f, d.key_bits);
}

hipError_t launch_attn_fwd(const void* qkv, void* out, float* lse, const AttnDims& d, DropoutArgs dropout,
                           hipStream_t stream) {
  const bool hd128 = d.hd == 2 * attn::kHD;
  if (d.B <= 0 || d.T <= 0 || d.H <= 0 || d.T > 65535 || d.hd <= 0 || (d.hd > attn::kHD && !hd128) || d.hd % 8 != 0)
    return hipErrorInvalidValue;
  const int nqb = (d.T + attn::kQBlk - 1) / attn::kQBlk;
  dim3 grid(d.B * d.H, nqb);
  const bool drop = dropout.thr != 0, km = d.key_bits != nullptr, small = d.hd < attn::kHD;
  const int variant = (drop ? 4 : 0) | (km ? 2 : 0) | (small ? 1 : 0);
  auto q = (const bf16_raw*)qkv;
  auto o = (bf16_raw*)out;
  if (hd128) {
    switch (variant) {
      case 0: launch_fwd_variant<false, false, false, 2>(grid, stream, q, o, lse, d, nqb, dropout); break;
      case 2: launch_fwd_variant<false, true, false, 2>(grid, stream, q, o, lse, d, nqb, dropout); break;
      case 4: launch_fwd_variant<true, false, false, 2>(grid, stream, q, o, lse, d, nqb, dropout); break;
      default: launch_fwd_variant<true, true, false, 2>(grid, stream, q, o, lse, d, nqb, dropout); break;
    }
    return hipGetLastError();
  }
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
