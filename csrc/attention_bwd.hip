// Causal flash-attention backward, head_dim <= 64, for gfx950 (MI355X).
//
// Replaces the autograd backward of reference models/gpt.py:56-69 (softmax + two batched
// matmuls over materialised [B, H, T, T] tensors).  P is recomputed from Q, K and the forward's
// log-sum-exp; nothing of size T^2 touches memory.
//
// Structure (after the MI355X playbook's attention-backward recipe):
//  * workgroup = 8 wave64s = one 256-key block of one (batch, head); wave w owns keys
//    32w..32w+31 with the KEY ON THE MFMA LANE: its K and V fragments stay in registers and its
//    dK^T / dV^T accumulators (2 x 32x32 f32 tiles each) live in registers for the whole sweep
//    over query tiles, so dK and dV need no cross-workgroup reduction;
//  * per 32-row query sub-tile: S = Q K^T and dP = dO V^T from zero accumulators, then
//    P = exp2(fma(S, scale*log2e, -lse*log2e)) and dP - delta, the row constants read from LDS
//    after the MFMA chains; dS = P o (dP - delta);
//  * P and dS are already the B operands of dV^T += dO^T P and dK^T += Q^T dS (accumulator used
//    as the next MFMA's operand); dO^T and Q^T fragments come from ds_read_b64_tr_b16 on the
//    same LDS images that serve the row reads (one swizzle, conflict free both ways);
//  * dS crosses LDS once (as a [key][q] image written 8 bytes per lane) and dQ = dS K is formed
//    with 16x16x32 MFMAs over the block's 256 keys (K^T LDS image, one ds_read_b128 per B
//    operand);
//  * work split: when B*H fills the CUs evenly (GPT-2 124M at micro-batch 128: 1,536 pairs on 256
//    CUs), ONE workgroup per (batch, head) sweeps its key blocks in order and keeps dQ in fp32 in
//    a private buffer — each query tile's partial is read at the top of the tile (latency under
//    phase A) and the rows of the current key block's own 256-row band, which no later block
//    touches, leave as bf16 straight into dqkv: no reduce pass, no bf16 partials, every
//    workgroup the same causal work (no tail).  Otherwise (small B*H, or dropout) one workgroup
//    per (batch, head, key block), heaviest first, each storing its dQ contribution to its own
//    bf16 partial plane, and a reduce pass sums the <= T/256 planes per row into dqkv;
//  * Q/dO tiles by LDS-DMA two tiles ahead into a 3-buffer ring (the register-staged version
//    exposed one global round trip per 64-row tile), row constants one tile ahead in registers;
//    branch-free buffer loads (rows past T read as zero), double-buffered dS images, one barrier
//    per query tile;
//  * measured LDS bank conflicts (rocprofv3 PMC, profiles/r2/pmc_attention_b32_after.txt): 8.9 %
//    of LDS-active cycles at B=32 (the forward: 0).  The Q/dO row and transposed reads are
//    conflict free by construction; the remainder is not attributed per access site (candidates:
//    the 2-byte K^T image stores of the prologue and the 8-byte dS^T image stores);
//  * SMALLHD (head dims < 64, multiples of 8) zero-fills the missing dims at load time; KMASK
//    (key padding) zeroes P of this lane's key when it is padded — one per-lane flag, because the
//    key sits on the MFMA lane here (rows the forward marked dead have lse = +inf, so P = 0).


#include "attention_common.h"

namespace llmt {
namespace attn {

constexpr int kBwdWaves = 8;

#ifdef LLMT_ATTN_PROBE
// Timing probe (bench/native/attn_bwd_timer.cpp with -DLLMT_ATTN_PROBE): lane 0 of each wave of the
// (b, h) = 0 workgroups stores s_memtime stamps [kb][wave][event]: 0 entry, 1 after the prologue,
// then per query tile it: 2 + 3 it after phase A, 3 + 3 it after the staging store + barrier,
// 4 + 3 it after the dQ phase; 63 exit.  Every workgroup's wave 0 stores entry / exit as
// s_memtime and s_memrealtime at g_attn_bwd_probe[nkb * kBwdWaves * 64 + 4 * (bh * nkb + kb)].
__device__ unsigned long long* g_attn_bwd_probe = nullptr;
#define BWD_PROBE(ev)                                                                                    \
  do {                                                                                                   \
    if (g_attn_bwd_probe != nullptr && (threadIdx.x & 63) == 0) {                                        \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                        \
      if (bh == 0 && (ev) < 64) g_attn_bwd_probe[((long)kb * kBwdWaves + wave) * 64 + (ev)] = t_;         \
      if (threadIdx.x == 0 && ((ev) == 0 || (ev) == 63)) {                                               \
        unsigned long long* g_ = g_attn_bwd_probe + (long)nkb * kBwdWaves * 64 + 4 * ((long)bh * nkb + kb); \
        g_[(ev) == 63] = t_;                                                                             \
        g_[2 + ((ev) == 63)] = __builtin_amdgcn_s_memrealtime();                                         \
      }                                                                                                  \
    }                                                                                                    \
  } while (0)
#else
#define BWD_PROBE(ev) \
  do {                \
  } while (0)
#endif
constexpr int kKvBlk = 32 * kBwdWaves;  // 256 keys per workgroup
constexpr int kQTile = 64;  // query rows per sweep step (two 32-row MFMA tiles)

// delta[b, h, t] = sum_d dO[b, t, h, d] * O[b, t, h, d]; a workgroup owns kDeltaRows consecutive t
// of one (b, h) in kDeltaRows / 32 unrolled sweeps of 32 rows (8 lanes per row, every sweep's
// loads issued up front).  With `vparts` it also forms the column sums of dO per head: without
// dropout every valid row of P sums to 1, so sum_key dV[key, d] = sum_q dO[q, d] — the V part of
// the qkv-bias gradient costs one LDS reduction here instead of a pass over dqkv.  Each
// workgroup stores its hd partial sums to vparts[b * gridDim.x + blockIdx.x][h * hd + d] (no
// atomics: 512+ workgroups per head would serialise on the same 64 addresses);
// launch_colsum_reduce sums them in a fixed order.
// NH = 64-wide halves of the head dim (2: hd = 128): 8 * NH lanes per row, 32 / NH rows per sweep.
constexpr int kDeltaRows = 256;
template <bool SMALLHD, int NH = 1>
__global__ __launch_bounds__(256) void attn_delta_kernel(const bf16_raw* __restrict__ dout,
                                                         const bf16_raw* __restrict__ out,
                                                         float* __restrict__ delta, float* __restrict__ vparts,
                                                         int T, int H, int hd_arg) {
  constexpr int kLpr = 8 * NH, kRps = 256 / kLpr;  // lanes per row, rows per sweep
  const int hd = SMALLHD ? hd_arg : kHD * NH;
  __shared__ float red[4][kHD * NH];
  const int bh = blockIdx.y;
  const int b = bh / H, h = bh - b * H;
  const int rl = threadIdx.x / kLpr, sub = threadIdx.x % kLpr;
  constexpr int kSweeps = kDeltaRows / kRps;
  ushort8_t dv[kSweeps], ov[kSweeps];
#pragma unroll
  for (int it = 0; it < kSweeps; ++it) {
    const int t = blockIdx.x * kDeltaRows + kRps * it + rl;
    dv[it] = ushort8_t{0, 0, 0, 0, 0, 0, 0, 0};
    ov[it] = dv[it];
    if (t < T && 8 * sub < hd) {
      const long row = ((long)b * T + t) * H + h;
      dv[it] = *reinterpret_cast<const ushort8_t*>(dout + row * hd + 8 * sub);
      ov[it] = *reinterpret_cast<const ushort8_t*>(out + row * hd + 8 * sub);
    }
  }
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < kSweeps; ++it) {
    float a[8], o[8];
    unpack8(dv[it], a);
    unpack8(ov[it], o);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc += a[i] * o[i];
      csum[i] += a[i];  // rows past T loaded as zeros
    }
#pragma unroll
    for (int off = 1; off < kLpr; off <<= 1) acc += __shfl_xor(acc, off, 64);
    const int t = blockIdx.x * kDeltaRows + kRps * it + rl;
    if (t < T && sub == 0) delta[(long)bh * T + t] = acc;
  }
  if (vparts == nullptr) return;  // uniform: kernel argument
  // column sums: over the wave's rows with shuffles (lanes sharing `sub`), then the 4 waves
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int off = kLpr; off < 64; off <<= 1) csum[i] += __shfl_xor(csum[i], off, 64);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < kLpr) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[wv][8 * sub + i] = csum[i];
  }
  __syncthreads();
  if (threadIdx.x < hd) {
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    vparts[((long)b * gridDim.x + blockIdx.x) * (H * hd) + h * hd + threadIdx.x] = s;
  }
}

// dqkv[b, t, 0, h, :] = bf16(sum over key blocks kb <= t / 256 of dq_part[kb][b, h, t, :]) with
// bf16 partial planes summed in fp32:
// the main kernel stores each key block's dQ contribution with plain stores (no memset, no
// atomics); rows only ever read the partials their causal key blocks wrote.  A workgroup owns
// kDqRows rows t of one (b, h) inside one 256-key block, so all its rows sum the same number of
// planes; row tiles are dispatched last-first (most planes first) and the Q part of the qkv-bias
// gradient (column sums of dQ) leaves the workgroup as one partial row,
// qparts[b * gridDim.y + tile][h * hd + d] (fixed-order reduce afterwards, no atomics).
constexpr int kDqRows = 64;
template <bool SMALLHD, int NH = 1>
__global__ __launch_bounds__(256) void attn_dq_reduce_kernel(const bf16_raw* __restrict__ part, bf16_raw* __restrict__ dqkv,
                                                             float* __restrict__ qparts, int T, int H, int hd_arg,
                                                             int nkb, long plane, int kvblk) {
  constexpr int kLpr = 8 * NH, kRps = 256 / kLpr, kW = kHD * NH;  // lanes per row, rows per sweep, width
  const int hd = SMALLHD ? hd_arg : kW;
  __shared__ float red[4][kW];
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh - b * H;
  const int rl = threadIdx.x / kLpr, c = threadIdx.x % kLpr;
  const int tile = (int)(gridDim.y - 1 - blockIdx.y);  // heavy (late) rows first
  const int t0 = tile * kDqRows + rl;  // this thread's rows: t0 + kRps * it
  const int last = min(tile * kDqRows / kvblk, nkb - 1);
  constexpr int kSweeps = kDqRows / kRps;
  // key-block planes outermost: each plane step issues all 8 loads of the thread's 8 rows at
  // once (rows past T re-read row T - 1, which every plane up to `last` holds; result unused)
  float f[kSweeps][8];
#pragma unroll
  for (int it = 0; it < kSweeps; ++it)
#pragma unroll
    for (int j = 0; j < 8; ++j) f[it][j] = 0.f;
  for (int kb = 0; kb <= last; ++kb) {
#pragma unroll
    for (int it = 0; it < kSweeps; ++it) {
      const int t = min(t0 + kRps * it, T - 1);
      float x[8];
      unpack8(*reinterpret_cast<const ushort8_t*>(part + kb * plane + ((long)bh * T + t) * kW + 8 * c), x);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[it][j] += x[j];
    }
  }
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < kSweeps; ++it) {
    const int t = t0 + kRps * it;
    if (t < T && 8 * c < hd) {  // the partial planes are kW wide; dims >= hd are zero
      *reinterpret_cast<ushort8_t*>(dqkv + ((long)b * T + t) * 3L * H * hd + (long)h * hd + 8 * c) = pack8(f[it]);
#pragma unroll
      for (int j = 0; j < 8; ++j) csum[j] += f[it][j];
    }
  }
  if (qparts == nullptr) return;  // uniform: kernel argument
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int off = kLpr; off < 64; off <<= 1) csum[j] += __shfl_xor(csum[j], off, 64);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < kLpr) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wv][8 * c + j] = csum[j];
  }
  __syncthreads();
  if (threadIdx.x < hd) {
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    qparts[((long)b * gridDim.y + tile) * (H * hd) + h * hd + threadIdx.x] = s;
  }
}

// x of lane l ^ 1 (DPP quad_perm [1,0,3,2]: one VALU op, no LDS round trip)
__device__ __forceinline__ float swap_pair(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));
}

// K^T image [64 d][256 keys]: 512-byte rows, 16-byte chunk index XOR-swizzled by (d & 15) so the
// 16 rows a ds_read_b128 lane group touches land on 16 distinct chunks (all 64 banks)
__device__ __forceinline__ int kt_off(int d, int key) { return d * kKvBlk + ((((key >> 3) ^ (d & 15))) << 3) + (key & 7); }

template <bool DROPOUT, bool KMASK, bool SMALLHD, bool SPLIT>
__global__ __launch_bounds__(512, 1) void attn_bwd_kernel(const bf16_raw* __restrict__ qkv,
                                                          const bf16_raw* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ delta,
                                                          bf16_raw* __restrict__ dqkv,
                                                          float* __restrict__ dq_acc, float* __restrict__ vparts,
                                                          float* __restrict__ qparts,
                                                          int T, int H, int nkb, DropoutArgs dr, int hd_arg,
                                                          float scale_arg, const uint8_t* __restrict__ key_valid) {
  resolve_dropout(dr);
  __shared__ __attribute__((aligned(16))) bf16_raw kt_lds[kHD * kKvBlk];             // K^T, 32 KB
  __shared__ __attribute__((aligned(16))) bf16_raw qd_lds[3][2][kQTile * kHD];      // [buf][Q|dO] 48 KB
  __shared__ __attribute__((aligned(16))) bf16_raw ds_lds[2][kKvBlk * kQTile];      // [buf][key][q] 64 KB
  __shared__ __attribute__((aligned(16))) float rowc_lds[2][2 * kQTile];            // lse*log2e | delta
  __shared__ float bias_red[kBwdWaves][kHD];                                       // V (dropout) / Q bias

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = lane >> 5, col = lane & 31;
  // Two work splits (template SPLIT: separate code, so the split grid keeps the leaner register
  // allocation of a body without the fp32 accumulation):
  //  * grid (B*H): one workgroup per (b, h) sweeps its key blocks in order and accumulates dQ in
  //    fp32 in a private buffer (no reduce pass; every workgroup the same causal work, so no tail
  //    as long as B*H fills the CUs evenly);
  //  * grid (B*H, nkb) ("split", for B*H that would leave CUs idle): one workgroup per (b, h, key
  //    block), heaviest first (attention_common.h chunked_dispatch), each key block's dQ into its
  //    own bf16 partial plane, summed by attn_dq_reduce_kernel.
  constexpr bool split = SPLIT;
  int bh, kb_first;
  if (split) {
    chunked_dispatch(bh, kb_first);
  } else {
    bh = blockIdx.x;
    kb_first = 0;
  }
  const int kb_end = split ? kb_first + 1 : nkb;
  const int b = bh / H, h = bh - b * H;
  const int hd = SMALLHD ? hd_arg : kHD;  // head dim in memory; tiles and fragments stay 64 wide
  const long row_stride = 3L * H * hd;
  const bf16_raw* base = qkv + (long)b * T * row_stride + (long)h * hd;
  const bf16_raw* dobase = dout + (long)b * T * H * hd + (long)h * hd;  // [B, T, H, hd]
  const long out_stride = (long)H * hd;
  const float* lse_bh = lse + ((long)b * H + h) * T;
  const float* delta_bh = delta + ((long)b * H + h) * T;
  // descriptors bounded at row T of this (b, h): rows past the sequence load as zeros
  const __amdgpu_buffer_rsrc_t r_q = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0,
                                                                        (int)((T - 1) * row_stride + hd) * 2, 0x00020000);
  // K/V of the block's keys: bounded past row T - 1's V section (a descriptor ending at row T - 1's
  // Q section would read the last key's K and V as zeros)
  const __amdgpu_buffer_rsrc_t r_kv = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0,
                                                                         (int)((T - 1) * row_stride + 3 * hd * H) * 2,
                                                                         0x00020000);
  const __amdgpu_buffer_rsrc_t r_do = __builtin_amdgcn_make_buffer_rsrc((void*)dobase, (short)0,
                                                                         (int)((T - 1) * out_stride + hd) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t r_lse = __builtin_amdgcn_make_buffer_rsrc((void*)lse_bh, (short)0, T * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t r_del = __builtin_amdgcn_make_buffer_rsrc((void*)delta_bh, (short)0, T * 4, 0x00020000);
  const uint32_t pseed = DROPOUT ? mix32(dr.seed + (uint32_t)bh * 0x9E3779B9u) : 0u;  // see attn fwd
  const float scale = SMALLHD ? scale_arg : 0.125f;
  const float c = scale * 1.4426950408889634f;
  const int ntq = (T + kQTile - 1) / kQTile;
  const int qt_dq = wave & 3;   // dQ output rows 16*qt_dq .. of the 64-row tile
  const int dp_dq = wave >> 2;  // dQ output cols 32*dp_dq .. (two 16-wide tiles)
  // column sums of this lane's final dQ (columns 32 dp + (lane & 15) and + 16): the Q part of the
  // qkv-bias gradient
  float qsum0 = 0.f, qsum1 = 0.f;

  for (int kb = kb_first; kb < kb_end; ++kb) {
  if (kb > kb_first) __syncthreads();  // the previous key block's K^T image / LDS rings are retired
  const int kblk0 = kb * kKvBlk;
  const int kw0 = kblk0 + 32 * wave;  // first key of this wave
  const int key = kw0 + col;          // this lane's key

  // key padding: this lane's key (on the MFMA lane) is excluded from P when padded
  const bool kvalid = !KMASK || (key < T && key_valid[(long)b * T + key] != 0);

  // K and V fragments of this lane's key: B operands of S = Q K^T and dP = dO V^T
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    // fragments past a small head dim load zeros through an out-of-record offset (a real read of
    // the last key's last head would run past the end of the qkv allocation)
    const bool live = !SMALLHD || 16 * kk + 8 * half < hd;
    const int off = (int)(key * row_stride + 16 * kk + 8 * half) * 2;
    kf[kk] = __builtin_bit_cast(bf16x8, buf_load16(r_kv, live ? off + hd * H * 2 : kOobOff));
    vf[kk] = __builtin_bit_cast(bf16x8, buf_load16(r_kv, live ? off + 2 * hd * H * 2 : kOobOff));
  }
  // K^T image for dQ = dS K (B operand read 8 keys at a time); written from the K fragments
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const ushort8_t kv = __builtin_bit_cast(ushort8_t, kf[kk]);
#pragma unroll
    for (int j = 0; j < 8; ++j) kt_lds[kt_off(16 * kk + 8 * half + j, 32 * wave + col)] = kv[j];
  }

  // Q/dO tiles arrive by LDS-DMA two tiles ahead into a 3-buffer ring (no register staging, ~32 KB
  // in flight per CU instead of 16: the register-staged version exposed one global round trip per
  // tile).  Wave w moves rows 8w..8w+7 of the Q and of the dO tile, one 1-KiB op each: lane l lands
  // at LDS byte 16 l of the op, i.e. row 8w + (l >> 3), swizzled slot l & 7, so it loads the source
  // chunk swz(row, slot) (the swizzle is an involution); head dims past a small hd and rows past T
  // load as zeros.
  const int dma_row = 8 * wave + (lane >> 3);
  const int dma_ch = swz(dma_row, lane & 7);
  const bool dma_live = !SMALLHD || dma_ch * 8 < hd;
  auto dma_tile = [&](int q0, int buf) {
    const int qrow = q0 + dma_row;
    const int oq = dma_live ? (int)(qrow * row_stride + dma_ch * 8) * 2 : kOobOff;
    const int od = dma_live ? (int)(qrow * out_stride + dma_ch * 8) * 2 : kOobOff;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r_q, (lds_void*)&qd_lds[buf][0][8 * wave * kHD], 16, oq, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r_do, (lds_void*)&qd_lds[buf][1][8 * wave * kHD], 16, od, 0, 0, 0);
  };
  // row constants of a tile (lse: wave 0, delta: wave 1) through one register each, one tile ahead;
  // a wave-uniform choice of descriptor (a per-lane select made hipcc emit a readfirstlane
  // waterfall loop around the load)
  float stc = 0.f;
  auto load_rowc = [&](int q0) {
    if (wave < 2) {
      const int qq = q0 + (threadIdx.x & (kQTile - 1));
      stc = wave == 0 ? buf_load_f32(r_lse, qq * 4) : buf_load_f32(r_del, qq * 4);
    }
  };
  auto store_rowc = [&](int buf) {
    if (threadIdx.x < 2 * kQTile) rowc_lds[buf][threadIdx.x] = threadIdx.x < kQTile ? stc * 1.4426950408889634f : stc;
  };

  f32x16 dk[2], dv[2];
  dk[0] = 0.f; dk[1] = 0.f; dv[0] = 0.f; dv[1] = 0.f;

  // ---- phase A of one 32-row query sub-tile: S, P, dP, dS, dV^T, dK^T, dS^T image ----------
  // full: the whole 64-row tile lies below the diagonal of every key of the block and inside the
  // sequence — no activity test, no mask (one body: two specialisations would each hoist their own
  // loop invariants and overflow the 256-VGPR budget).
  auto phase_a = [&](bool full, int q0, const bf16_raw* q_lds, const bf16_raw* do_lds, const float* rowc,
                     bf16_raw* dsimg) {
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qb0 = q0 + 32 * qs;
      const bool active = full || (kw0 <= qb0 + 31 && kw0 < T && qb0 < T);  // wave-uniform
      bf16x8 sbs[2];  // dS packed to bf16: the dK^T operand and, as is, the dS^T image
      if (active) {
        f32x16 p, dp, ds;
        p = 0.f;
        dp = 0.f;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const bf16x8 qa = lds_row_read(q_lds, 32 * qs + col, 2 * kk + half);
          p = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[kk], p, 0, 0, 0);
          const bf16x8 da = lds_row_read(do_lds, 32 * qs + col, 2 * kk + half);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[kk], dp, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);  // row constants are read after the chains (VGPR budget)
        float ddv[16];  // delta per row, kept only by the dropout variant
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const f32x4 l2 = *reinterpret_cast<const f32x4*>(&rowc[32 * qs + 8 * rr + 4 * half]);
          const f32x4 dd = *reinterpret_cast<const f32x4*>(&rowc[kQTile + 32 * qs + 8 * rr + 4 * half]);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            p[4 * rr + i] = __builtin_amdgcn_exp2f(fmaf(p[4 * rr + i], c, -l2[i]));
            if (DROPOUT) ddv[4 * rr + i] = dd[i];
            else dp[4 * rr + i] -= dd[i];
          }
        }
        if (KMASK && !kvalid) {
#pragma unroll
          for (int r = 0; r < 16; ++r) p[r] = 0.f;
        }
        if (!full && ((kw0 + 31 > qb0) || (kw0 + 32 > T) || (qb0 + 32 > T))) {
          // causal / sequence-end mask: element r is query qb0 + 4*half + (r&3) + 8(r>>2),
          // valid iff key <= query < T (branch-free selects)
          const int lo = key - qb0 - 4 * half, hi = T - 1 - qb0 - 4 * half;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int roff = (r & 3) + 8 * (r >> 2);
            p[r] = (roff < lo || roff > hi) ? 0.f : p[r];
          }
        }
        if (DROPOUT) {
          // dP above is the gradient of the DROPPED probabilities: undo the mask for dS, and feed
          // dV the dropped P (element (q, key) of the plane: q*T + key, as in the forward)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint32_t qq = (uint32_t)(qb0 + 4 * half + (r & 3) + 8 * (r >> 2));
            const bool kp = drop_keep(pseed, dr.thr, qq * (uint32_t)T + (uint32_t)key);
            ds[r] = p[r] * ((kp ? dp[r] * dr.scale : 0.f) - ddv[r]);
            p[r] = kp ? p[r] * dr.scale : 0.f;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) ds[r] = p[r] * dp[r];
        }
        // dV^T += dO^T P ; dK^T += Q^T dS  (P, dS used in place as B operands)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pb = pack_acc8(p, st);
          sbs[st] = pack_acc8(ds, st);
          const bf16x8 sb = sbs[st];
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const bf16x8 doa = lds_tr_read_operand(do_lds, 32 * qs + 16 * st + 4 * half, dt * 32, lane);
            dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(doa, pb, dv[dt], 0, 0, 0);
            const bf16x8 qa = lds_tr_read_operand(q_lds, 32 * qs + 16 * st + 4 * half, dt * 32, lane);
            dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, sb, dk[dt], 0, 0, 0);
          }
        }
      } else {
        const bf16x8 z = {};
        sbs[0] = z;
        sbs[1] = z;
      }
      // dS^T image [key][q]: this lane's key, q rows 32 qs + 8g + 4h .. +3 (one 8-byte write each)
      const int kl = 32 * wave + col;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const ushort8_t u = __builtin_bit_cast(ushort8_t, sbs[g >> 1]);  // rows 8(g>>1) .. +7
        const int o = 4 * (g & 1);
        const ushort4_t v = {u[o], u[o + 1], u[o + 2], u[o + 3]};
        *reinterpret_cast<ushort4_t*>(&dsimg[tile_elem_off(kl, 32 * qs + 8 * g + 4 * half)]) = v;
      }
      // keep the two sub-tiles' live ranges apart: overlapping them exceeds the 256-VGPR budget
      // of two waves per SIMD (spills)
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  BWD_PROBE(0);
  const int ntiles = (T - kblk0 + kQTile - 1) / kQTile;
  load_rowc(kblk0);
  dma_tile(kblk0, 0);
  if (ntiles > 1) dma_tile(kblk0 + kQTile, 1);
  store_rowc(0);
  // tile 0 landed (this wave's ops; the barrier covers the others'): tile 1's two ops may fly
  if (ntiles > 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  BWD_PROBE(1);

  int it = 0, cur3 = 0;
  for (int q0 = kblk0; q0 < T; q0 += kQTile, ++it) {
    const int cur = it & 1;
    const bool more = it + 1 < ntiles, more2 = it + 2 < ntiles;
    // the next tile's row constants, then the DMA of the tile after it (program order matters: the
    // constants' own wait must not cover those two ops)
    if (more) load_rowc(q0 + kQTile);
    // this lane's fp32 dQ partial of the tile from the earlier key blocks (workgroup-private buffer
    // in MFMA-fragment order: 32 contiguous bytes per lane), read now, used after phase A
    float* accp = dq_acc + ((((long)bh * ntq + q0 / kQTile) * kBwdWaves + wave) * 64 + lane) * 8;
    f32x4 prev0 = {0.f, 0.f, 0.f, 0.f}, prev1 = prev0;
    if (!split && kb > 0) {
      prev0 = *reinterpret_cast<const f32x4*>(accp);
      prev1 = *reinterpret_cast<const f32x4*>(accp + 4);
    }
    const int nxt3 = cur3 == 2 ? 0 : cur3 + 1, nxt3b = nxt3 == 2 ? 0 : nxt3 + 1;
    if (more2) dma_tile(q0 + 2 * kQTile, nxt3b);
    const bf16_raw* q_lds = qd_lds[cur3][0];
    const bf16_raw* do_lds = qd_lds[cur3][1];
    bf16_raw* dsimg = ds_lds[cur];
    phase_a(q0 >= kblk0 + kKvBlk && q0 + kQTile <= T, q0, q_lds, do_lds, rowc_lds[cur], dsimg);
    BWD_PROBE(2 + 3 * it);
    if (more) store_rowc(cur ^ 1);
    // one barrier per tile: tile it+1's Q/dO landed (only tile it+2's two ops may still fly; the
    // buffer they fill was last read by phase A of tile it-1, before the previous barrier), the
    // dS image is double-buffered, so the only hand-off is "phase A of this tile done by every wave"
    if (more2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    BWD_PROBE(3 + 3 * it);
    cur3 = nxt3;

    // ---- dQ[q0 + 16 qt .., 32 dp + (0..31)] += dS K over the block's 256 keys (16x16x32) ----
    {
      const int i = lane & 15, g = lane >> 4;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      typedef short short8v __attribute__((ext_vector_type(8)));
      // software pipeline: the operands of step ks + 3 are read while step ks's MFMAs run (12 LDS
      // reads in flight, inside lgkmcnt's 15).  The compiler's own schedule read one pair ahead
      // and waited on LDS latency before every MFMA (~2.2k cycles for 256 cycles of MFMA);
      // hoisting all 8 steps' reads spilled (address registers: the K^T swizzle makes every step's
      // offset distinct).
      constexpr int kSteps = kKvBlk / 32, kAhead = 3;
      bf16x8 av[kSteps], b0[kSteps], b1[kSteps];
      auto read_step = [&](int ks) {
        const int krow = 32 * ks + 8 * g + (i >> 2);
        const int qcol = 16 * qt_dq + 4 * (i & 3);
        const short4v a_lo = tr_read(dsimg, krow, qcol);
        const short4v a_hi = tr_read(dsimg, krow + 4, qcol);
        const short8v a8 = {a_lo[0], a_lo[1], a_lo[2], a_lo[3], a_hi[0], a_hi[1], a_hi[2], a_hi[3]};
        av[ks] = __builtin_bit_cast(bf16x8, a8);
        const int kc = 32 * ks + 8 * g;  // first of this lane's 8 keys
        b0[ks] = *reinterpret_cast<const bf16x8*>(&kt_lds[kt_off(32 * dp_dq + i, kc)]);
        b1[ks] = *reinterpret_cast<const bf16x8*>(&kt_lds[kt_off(32 * dp_dq + 16 + i, kc)]);
      };
#pragma unroll
      for (int ks = 0; ks < kAhead; ++ks) read_step(ks);
#pragma unroll
      for (int ks = 0; ks < kSteps; ++ks) {
        __builtin_amdgcn_sched_barrier(0);
        if (ks + kAhead < kSteps) read_step(ks + kAhead);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[ks], b0[ks], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[ks], b1[ks], acc1, 0, 0, 0);
      }
      // dQ accumulates in fp32 across the key blocks: rows below this key block (every earlier block
      // contributed) add the partial read at the top of the tile; rows of the block's own 256-row
      // band get no later contribution, so they leave as bf16 straight into dqkv (scaled), all other
      // rows go back to the private buffer.  Rows past T and dims past hd are zero (zero Q rows /
      // masked P; zero K^T dims).
      acc0 += prev0;
      acc1 += prev1;
      // lanes i and i^1 swap half their rows so each lane stores whole dwords (two adjacent
      // columns): even lanes rows 0,1, odd rows 2,3
      const int p = i & 1;
      if (split) {  // this key block's bf16 partial plane [kb][b, h, t, 64]
        bf16_raw* plane = reinterpret_cast<bf16_raw*>(dq_acc) + ((long)kb * gridDim.x + bh) * T * kHD;
        const int dcol = 32 * dp_dq + (i & ~1);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int r = p ? 2 + j : j;
          const int qq = q0 + 16 * qt_dq + 4 * g + r;
          const float s0 = swap_pair(p ? acc0[j] : acc0[2 + j]);
          const float s1 = swap_pair(p ? acc1[j] : acc1[2 + j]);
          const float o0 = p ? acc0[2 + j] : acc0[j], o1 = p ? acc1[2 + j] : acc1[j];
          const uint32_t w0 = (uint32_t)f2bf((p ? s0 : o0) * scale) | ((uint32_t)f2bf((p ? o0 : s0) * scale) << 16);
          const uint32_t w1 = (uint32_t)f2bf((p ? s1 : o1) * scale) | ((uint32_t)f2bf((p ? o1 : s1) * scale) << 16);
          if (qq < T) {
            bf16_raw* dst = plane + (long)qq * kHD + dcol;
            *reinterpret_cast<uint32_t*>(dst) = w0;
            *reinterpret_cast<uint32_t*>(dst + 16) = w1;
          }
        }
      } else if (q0 >= kblk0 + kKvBlk) {
        *reinterpret_cast<f32x4*>(accp) = acc0;
        *reinterpret_cast<f32x4*>(accp + 4) = acc1;
      } else {
        const int dcol = 32 * dp_dq + (i & ~1);  // even column of this lane's pair
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int r = p ? 2 + j : j;  // the row this lane stores
          const int qq = q0 + 16 * qt_dq + 4 * g + r;
          const float s0 = swap_pair(p ? acc0[j] : acc0[2 + j]);
          const float s1 = swap_pair(p ? acc1[j] : acc1[2 + j]);
          const float o0 = p ? acc0[2 + j] : acc0[j], o1 = p ? acc1[2 + j] : acc1[j];
          const uint32_t w0 = (uint32_t)f2bf((p ? s0 : o0) * scale) | ((uint32_t)f2bf((p ? o0 : s0) * scale) << 16);
          const uint32_t w1 = (uint32_t)f2bf((p ? s1 : o1) * scale) | ((uint32_t)f2bf((p ? o1 : s1) * scale) << 16);
          if (qq < T) {
            bf16_raw* dst = dqkv + ((long)b * T + qq) * row_stride + (long)h * hd + dcol;
            if (!SMALLHD || dcol < hd) *reinterpret_cast<uint32_t*>(dst) = w0;
            if (!SMALLHD || dcol + 16 < hd) *reinterpret_cast<uint32_t*>(dst + 16) = w1;
          }
        }
        qsum0 += (acc0[0] + acc0[1] + acc0[2] + acc0[3]) * scale;
        qsum1 += (acc1[0] + acc1[1] + acc1[2] + acc1[3]) * scale;
      }
    }
    BWD_PROBE(4 + 3 * it);
  }

  // ---- dK = scale * dK^T, dV = dV^T  -> dqkv[b, key, 1|2, h, :] ------------------------------
  if (key < T) {
    bf16_raw* dst = dqkv + ((long)b * T + key) * row_stride + (long)h * hd;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        ushort4_t kv, vv;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          kv[i] = f2bf(dk[dt][4 * g + i] * scale);
          vv[i] = f2bf(dv[dt][4 * g + i]);
        }
        const int d = dt * 32 + 8 * g + 4 * half;
        if (!SMALLHD || d < hd) {
          *reinterpret_cast<ushort4_t*>(dst + hd * H + d) = kv;
          *reinterpret_cast<ushort4_t*>(dst + 2 * hd * H + d) = vv;
        }
      }
    }
  }
  // qkv-bias gradient, K and V parts.  K: exactly zero — adding b_k shifts every score of a query
  // row by q.b_k, which softmax ignores — so nothing is accumulated.  V without dropout: the
  // delta kernel's column sums of dO.  V with dropout (rows of the dropped P no longer sum to 1):
  // sum this block's 256 keys of dV^T — over the 32 lanes of each half, then over the 8 waves —
  // into this block's partial row vparts[b * nkb + kb][h * hd + d].
  BWD_PROBE(63);
  if (DROPOUT && vparts != nullptr) {
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float vv = dv[dt][r];
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) vv += __shfl_xor(vv, off, 64);
        if (col == 0) bias_red[wave][dt * 32 + 8 * (r >> 2) + 4 * half + (r & 3)] = vv;
      }
    }
    __syncthreads();
    if (threadIdx.x < hd) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < kBwdWaves; ++w) acc += bias_red[w][threadIdx.x];
      vparts[((long)b * nkb + kb) * (H * hd) + h * hd + threadIdx.x] = acc;
    }
  }
  }  // key blocks

  // Q part of the qkv-bias gradient: this (b, h)'s column sums of dQ, one partial row
  // qparts[b][h * hd + d] (lanes of one column, then the four waves of one column half, fixed order)
  if (split || qparts == nullptr) return;  // uniform (the split grid's Q part comes from the reduce)
  qsum0 += __shfl_xor(qsum0, 16, 64);
  qsum0 += __shfl_xor(qsum0, 32, 64);
  qsum1 += __shfl_xor(qsum1, 16, 64);
  qsum1 += __shfl_xor(qsum1, 32, 64);
  __syncthreads();  // bias_red's V use is over
  if (lane < 16) {
    bias_red[wave][32 * dp_dq + lane] = qsum0;
    bias_red[wave][32 * dp_dq + 16 + lane] = qsum1;
  }
  __syncthreads();
  if (threadIdx.x < hd) {
    const int dp = threadIdx.x >> 5;
    float acc = 0.f;
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) acc += bias_red[qt + 4 * dp][threadIdx.x];
    qparts[(long)b * (H * hd) + h * hd + threadIdx.x] = acc;
  }
}

// ---------------------------------------------------------------------------------------------
// Head dim 128: 4 waves (one per SIMD, 512 registers per lane) x 32 keys = a 128-key block.  The
// 8-wave kernel's per-wave state doubles at hd = 128 (dK^T / dV^T 128 registers, K/V fragments 64)
// and no longer fits two waves per SIMD; here each wave keeps dK^T / dV^T of its 32 keys over the
// full 128 dims, its K/V fragments, and the B operand of dQ = dS K for its 32 dQ columns over the
// block's 128 keys (read once from a K^T image).  Q/dO tiles are [64][128], kept as two [64][64]
// swizzled LDS images each; dS^T crosses LDS as in the other kernels.  Same contract, masks,
// dropout; dQ partial planes are 128 wide, one per 128-key block.
constexpr int kKv128 = 128;
__device__ __forceinline__ int kt128_off(int d, int key) {
  return d * kKv128 + ((((key >> 3) ^ (d & 15))) << 3) + (key & 7);
}

template <bool DROPOUT, bool KMASK>
__global__ __launch_bounds__(256, 1) void attn_bwd128_kernel(const bf16_raw* __restrict__ qkv,
                                                             const bf16_raw* __restrict__ dout,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ delta,
                                                             bf16_raw* __restrict__ dqkv,
                                                             float* __restrict__ dq_part, float* __restrict__ vparts,
                                                             int T, int H, int nkb, DropoutArgs dr,
                                                             const uint8_t* __restrict__ key_valid) {
  resolve_dropout(dr);
  constexpr int hd = 2 * kHD;
  __shared__ __attribute__((aligned(16))) bf16_raw qd_lds[2][2][2][kQTile * kHD];  // [buf][Q|dO][half] 64 KB
  __shared__ __attribute__((aligned(16))) bf16_raw ds_lds[2][kKv128 * kQTile];     // [buf][key][q] 32 KB
  __shared__ __attribute__((aligned(16))) float rowc_lds[2][2 * kQTile];
  __shared__ float bias_red[4][hd];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = lane >> 5, col = lane & 31;
  int bh, kb;
  chunked_dispatch(bh, kb);
  const int b = bh / H, h = bh - b * H;
  const long row_stride = 3L * H * hd;
  const bf16_raw* base = qkv + (long)b * T * row_stride + (long)h * hd;
  const bf16_raw* dobase = dout + (long)b * T * H * hd + (long)h * hd;
  const long out_stride = (long)H * hd;
  const float* lse_bh = lse + ((long)b * H + h) * T;
  const float* delta_bh = delta + ((long)b * H + h) * T;
  const __amdgpu_buffer_rsrc_t r_q = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0,
                                                                        (int)((T - 1) * row_stride + hd) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t r_kv = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0,
                                                                         (int)((T - 1) * row_stride + 3 * hd * H) * 2,
                                                                         0x00020000);
  const __amdgpu_buffer_rsrc_t r_do = __builtin_amdgcn_make_buffer_rsrc((void*)dobase, (short)0,
                                                                         (int)((T - 1) * out_stride + hd) * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t r_lse = __builtin_amdgcn_make_buffer_rsrc((void*)lse_bh, (short)0, T * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t r_del = __builtin_amdgcn_make_buffer_rsrc((void*)delta_bh, (short)0, T * 4, 0x00020000);

  const uint32_t pseed = DROPOUT ? mix32(dr.seed + (uint32_t)bh * 0x9E3779B9u) : 0u;
  const int kblk0 = kb * kKv128;
  const int kw0 = kblk0 + 32 * wave;
  const int key = kw0 + col;
  constexpr float scale = 0.08838834764831845f;  // 1 / sqrt(128)
  const float c = scale * 1.4426950408889634f;
  const bool kvalid = !KMASK || (key < T && key_valid[(long)b * T + key] != 0);

  bf16x8 kf[8], vf[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int off = (int)(key * row_stride + 16 * kk + 8 * half) * 2;
    kf[kk] = __builtin_bit_cast(bf16x8, buf_load16(r_kv, off + hd * H * 2));
    vf[kk] = __builtin_bit_cast(bf16x8, buf_load16(r_kv, off + 2 * hd * H * 2));
  }
  // dQ B operand (16x16x32, k = key, n = d): lane l holds K[32 ks + 8 (l >> 4) + 0..7][32 w + 16 dn + (l & 15)],
  // read once through a K^T image [128 d][128 keys] laid over both dS buffers
  bf16x8 kq[kKv128 / 32][2];
  {
    bf16_raw* kt_img = ds_lds[0];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const ushort8_t kv = __builtin_bit_cast(ushort8_t, kf[kk]);
#pragma unroll
      for (int e = 0; e < 8; ++e) kt_img[kt128_off(16 * kk + 8 * half + e, 32 * wave + col)] = kv[e];
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < kKv128 / 32; ++ks)
#pragma unroll
      for (int dn = 0; dn < 2; ++dn)
        kq[ks][dn] = *reinterpret_cast<const bf16x8*>(&kt_img[kt128_off(32 * wave + 16 * dn + (lane & 15), 32 * ks + 8 * (lane >> 4))]);
    __syncthreads();  // every wave's reads of the image are done before the first dS write
  }

  // register staging of one 64-row Q/dO tile (+ row constants): 4 Q + 4 dO chunks per thread
  ushort8_t stg[8];
  float stc = 0.f;
  auto load_tile = [&](int q0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int cidx = threadIdx.x + 256 * (i & 3);
      const int r = cidx >> 4, ch = cidx & 15;
      const int qrow = q0 + r;
      stg[i] = i < 4 ? buf_load16(r_q, (int)(qrow * row_stride + ch * 8) * 2)
                     : buf_load16(r_do, (int)(qrow * out_stride + ch * 8) * 2);
    }
    if (wave < 2) {  // wave 0: lse, wave 1: delta (wave-uniform descriptor choice)
      const int qq = q0 + (threadIdx.x & (kQTile - 1));
      stc = wave == 0 ? buf_load_f32(r_lse, qq * 4) : buf_load_f32(r_del, qq * 4);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int cidx = threadIdx.x + 256 * (i & 3);
      const int r = cidx >> 4, ch = cidx & 15;
      *reinterpret_cast<ushort8_t*>(&qd_lds[buf][i >> 2][ch >> 3][tile_chunk_off(r, ch & 7)]) = stg[i];
    }
    if (threadIdx.x < 2 * kQTile) rowc_lds[buf][threadIdx.x] = threadIdx.x < kQTile ? stc * 1.4426950408889634f : stc;
  };

  f32x16 dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    dk[dt] = 0.f;
    dv[dt] = 0.f;
  }

  auto phase_a = [&](bool full, int q0, int buf, bf16_raw* dsimg) {
    const float* rowc = rowc_lds[buf];
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qb0 = q0 + 32 * qs;
      const bool active = full || (kw0 <= qb0 + 31 && kw0 < T && qb0 < T);
      f32x16 ds;
      if (active) {
        f32x16 p = 0.f, dp = 0.f;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const bf16x8 qa = lds_row_read(qd_lds[buf][0][kk >> 2], 32 * qs + col, 2 * (kk & 3) + half);
          const bf16x8 da = lds_row_read(qd_lds[buf][1][kk >> 2], 32 * qs + col, 2 * (kk & 3) + half);
          p = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[kk], p, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[kk], dp, 0, 0, 0);
        }
        float ddv[16];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const f32x4 l2 = *reinterpret_cast<const f32x4*>(&rowc[32 * qs + 8 * rr + 4 * half]);
          const f32x4 dd = *reinterpret_cast<const f32x4*>(&rowc[kQTile + 32 * qs + 8 * rr + 4 * half]);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            p[4 * rr + i] = __builtin_amdgcn_exp2f(fmaf(p[4 * rr + i], c, -l2[i]));
            if (DROPOUT) ddv[4 * rr + i] = dd[i];
            else dp[4 * rr + i] -= dd[i];
          }
        }
        if (KMASK && !kvalid) p = 0.f;
        if (!full && ((kw0 + 31 > qb0) || (kw0 + 32 > T) || (qb0 + 32 > T))) {
          const int lo = key - qb0 - 4 * half, hi = T - 1 - qb0 - 4 * half;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int roff = (r & 3) + 8 * (r >> 2);
            p[r] = (roff < lo || roff > hi) ? 0.f : p[r];
          }
        }
        if (DROPOUT) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint32_t qq = (uint32_t)(qb0 + 4 * half + (r & 3) + 8 * (r >> 2));
            const bool kp = drop_keep(pseed, dr.thr, qq * (uint32_t)T + (uint32_t)key);
            ds[r] = p[r] * ((kp ? dp[r] * dr.scale : 0.f) - ddv[r]);
            p[r] = kp ? p[r] * dr.scale : 0.f;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) ds[r] = p[r] * dp[r];
        }
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pb = pack_acc8(p, st);
          const bf16x8 sb = pack_acc8(ds, st);
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const int rb = 32 * qs + 16 * st + 4 * half;
            const bf16x8 doa = lds_tr_read_operand(qd_lds[buf][1][dt >> 1], rb, (dt & 1) * 32, lane);
            dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(doa, pb, dv[dt], 0, 0, 0);
            const bf16x8 qa = lds_tr_read_operand(qd_lds[buf][0][dt >> 1], rb, (dt & 1) * 32, lane);
            dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, sb, dk[dt], 0, 0, 0);
          }
        }
      } else {
        ds = 0.f;
      }
      const int kl = 32 * wave + col;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        ushort4_t v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = f2bf(ds[4 * g + i]);
        *reinterpret_cast<ushort4_t*>(&dsimg[tile_elem_off(kl, 32 * qs + 8 * g + 4 * half)]) = v;
      }
    }
  };

  load_tile(kblk0);
  store_tile(0);
  __syncthreads();

  int it = 0;
  for (int q0 = kblk0; q0 < T; q0 += kQTile, ++it) {
    const int cur = it & 1;
    const bool more = q0 + kQTile < T;
    if (more) load_tile(q0 + kQTile);
    phase_a(q0 >= kblk0 + kKv128 && q0 + kQTile <= T, q0, cur, ds_lds[cur]);
    if (more) store_tile(cur ^ 1);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

    // ---- dQ[q0 + 16 qt + .., 32 w + 16 dn + ..] = dS K over the block's 128 keys (16x16x32) ----
    {
      const int i = lane & 15, g = lane >> 4;
      const bf16_raw* dsimg = ds_lds[cur];
      f32x4 acc[4][2];
#pragma unroll
      for (int qt = 0; qt < 4; ++qt)
#pragma unroll
        for (int dn = 0; dn < 2; ++dn) acc[qt][dn] = f32x4{0.f, 0.f, 0.f, 0.f};
      typedef short short8v __attribute__((ext_vector_type(8)));
#pragma unroll
      for (int ks = 0; ks < kKv128 / 32; ++ks) {
        const int krow = 32 * ks + 8 * g + (i >> 2);
#pragma unroll
        for (int qt = 0; qt < 4; ++qt) {
          const int qcol = 16 * qt + 4 * (i & 3);
          const short4v lo = tr_read(dsimg, krow, qcol);
          const short4v hi = tr_read(dsimg, krow + 4, qcol);
          const short8v a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          const bf16x8 a = __builtin_bit_cast(bf16x8, a8);
#pragma unroll
          for (int dn = 0; dn < 2; ++dn)
            acc[qt][dn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, kq[ks][dn], acc[qt][dn], 0, 0, 0);
        }
      }
      const int p = i & 1;
      bf16_raw* plane = reinterpret_cast<bf16_raw*>(dq_part) + ((long)kb * gridDim.x + bh) * T * hd;
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int r = p ? 2 + jj : jj;
          const int qq = q0 + 16 * qt + 4 * g + r;
#pragma unroll
          for (int dn = 0; dn < 2; ++dn) {
            const float sw = swap_pair(p ? acc[qt][dn][jj] : acc[qt][dn][2 + jj]);
            const float own = p ? acc[qt][dn][2 + jj] : acc[qt][dn][jj];
            const uint32_t w = (uint32_t)f2bf((p ? sw : own) * scale) | ((uint32_t)f2bf((p ? own : sw) * scale) << 16);
            if (qq < T) *reinterpret_cast<uint32_t*>(plane + (long)qq * hd + 32 * wave + 16 * dn + (i & ~1)) = w;
          }
        }
      }
    }
  }

  if (key < T) {
    bf16_raw* dst = dqkv + ((long)b * T + key) * row_stride + (long)h * hd;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        ushort4_t kv, vv;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          kv[i] = f2bf(dk[dt][4 * g + i] * scale);
          vv[i] = f2bf(dv[dt][4 * g + i]);
        }
        const int d = dt * 32 + 8 * g + 4 * half;
        *reinterpret_cast<ushort4_t*>(dst + hd * H + d) = kv;
        *reinterpret_cast<ushort4_t*>(dst + 2 * hd * H + d) = vv;
      }
    }
  }
  if (!DROPOUT || vparts == nullptr) return;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float vv = dv[dt][r];
#pragma unroll
      for (int off = 1; off < 32; off <<= 1) vv += __shfl_xor(vv, off, 64);
      if (col == 0) bias_red[wave][dt * 32 + 8 * (r >> 2) + 4 * half + (r & 3)] = vv;
    }
  }
  __syncthreads();
  if (threadIdx.x < hd) {
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) acc += bias_red[w][threadIdx.x];
    vparts[((long)b * nkb + kb) * (H * hd) + h * hd + threadIdx.x] = acc;
  }
}

}  // namespace attn

namespace {
// key-block size of the backward: 256 (8-wave kernel) for hd <= 64, 128 for hd = 128
int bwd_kvblk(int hd) { return hd == 2 * attn::kHD ? attn::kKv128 : attn::kKvBlk; }
int bwd_plane_width(int hd) { return hd == 2 * attn::kHD ? 2 * attn::kHD : attn::kHD; }
}  // namespace

long attn_bwd_workspace_floats(int B, int T, int H, int hd) {
  if (hd == 2 * attn::kHD) {  // bf16 partial planes, one per 128-key block
    const long nkb = (T + bwd_kvblk(hd) - 1) / bwd_kvblk(hd);
    return (nkb * B * H * (long)T * bwd_plane_width(hd) + 1) / 2;
  }
  // the 8-wave kernel: fp32 dQ accumulator (one [64 rows][64] tile per query tile per (b, h)) or,
  // split, bf16 partial planes (one per 256-key block)
  const long ntq = (T + attn::kQTile - 1) / attn::kQTile;
  const long acc = (long)B * H * ntq * attn::kQTile * attn::kHD;
  const long nkb = (T + attn::kKvBlk - 1) / attn::kKvBlk;
  const long planes = (nkb * B * H * (long)T * attn::kHD + 1) / 2;
  return acc > planes ? acc : planes;
}

namespace {
// partial rows of the qkv-bias column sums: V (delta kernel or, with dropout, the main kernel)
// and Q (dQ reduce), then the fixed-order reduce's scratch
struct BiasParts {
  int nv, nq;
  long cols;
};
BiasParts bias_parts(int B, int T, int H, int hd) {
  const int nkb = (T + bwd_kvblk(hd) - 1) / bwd_kvblk(hd);
  const int nv1 = B * ((T + attn::kDeltaRows - 1) / attn::kDeltaRows), nv2 = B * nkb;
  return {nv1 > nv2 ? nv1 : nv2, B * ((T + attn::kDqRows - 1) / attn::kDqRows), (long)H * hd};
}
}  // namespace

long attn_bwd_bias_ws_floats(int B, int T, int H, int hd) {
  const BiasParts p = bias_parts(B, T, H, hd);
  const long sv = colsum_scratch_floats(p.nv, p.cols), sq = colsum_scratch_floats(p.nq, p.cols);
  return (long)(p.nv + p.nq) * p.cols + (sv > sq ? sv : sq);
}

#ifdef LLMT_ATTN_PROBE
void attn_bwd_probe_set(unsigned long long* buf) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(attn::g_attn_bwd_probe), &buf, sizeof(buf));
}
#endif

template <bool DROPOUT, bool KMASK, bool SMALLHD>
static void launch_bwd_variant(dim3 grid, hipStream_t stream, const bf16_raw* qkv, const bf16_raw* dout,
                               const float* lse, const float* delta, bf16_raw* dqkv,
                               float* dq_acc, float* vparts, float* qparts, const AttnDims& d, int nkb,
                               DropoutArgs dr) {
  if (grid.y > 1)
    hipLaunchKernelGGL((attn::attn_bwd_kernel<DROPOUT, KMASK, SMALLHD, true>), grid, dim3(512), 0, stream, qkv, dout,
                       lse, delta, dqkv, dq_acc, vparts, qparts, d.T, d.H, nkb, dr, d.hd, d.scale, d.key_valid);
  else
    hipLaunchKernelGGL((attn::attn_bwd_kernel<DROPOUT, KMASK, SMALLHD, false>), grid, dim3(512), 0, stream, qkv, dout,
                       lse, delta, dqkv, dq_acc, vparts, qparts, d.T, d.H, nkb, dr, d.hd, d.scale, d.key_valid);
}

hipError_t launch_attn_bwd(const void* dout, const void* qkv, const void* out, const float* lse, void* dqkv,
                           float* delta, float* dq_part, float* dbias, float* bias_ws, const AttnDims& d,
                           DropoutArgs dropout, hipStream_t stream, bool delta_ready) {
  const int B = d.B, T = d.T, H = d.H, hd = d.hd;
  const bool hd128 = hd == 2 * attn::kHD;
  if (B <= 0 || T <= 0 || H <= 0 || T > 65535 || hd <= 0 || (hd > attn::kHD && !hd128) || hd % 8 != 0)
    return hipErrorInvalidValue;
  if (dbias != nullptr && bias_ws == nullptr) return hipErrorInvalidValue;
  const long rows = (long)B * T * H;
  const BiasParts bp = bias_parts(B, T, H, hd);
  float* vparts = dbias != nullptr ? bias_ws : nullptr;
  float* qparts = dbias != nullptr ? bias_ws + (long)bp.nv * bp.cols : nullptr;
  float* scratch = dbias != nullptr ? bias_ws + (long)(bp.nv + bp.nq) * bp.cols : nullptr;
  const bool v_from_delta = !delta_ready && dropout.thr == 0 && dbias != nullptr;
  const dim3 dgrid((T + attn::kDeltaRows - 1) / attn::kDeltaRows, B * H);
  const bool small = hd < attn::kHD;
  if (!delta_ready) {
    auto dk = hd128 ? attn::attn_delta_kernel<false, 2>
                    : (small ? attn::attn_delta_kernel<true> : attn::attn_delta_kernel<false>);
    hipLaunchKernelGGL(dk, dgrid, dim3(256), 0, stream, (const bf16_raw*)dout, (const bf16_raw*)out, delta,
                       v_from_delta ? vparts : nullptr, T, H, hd);
  }
  const int kvblk = bwd_kvblk(hd);
  const int nkb = (T + kvblk - 1) / kvblk;
  const bool drop = dropout.thr != 0, km = d.key_valid != nullptr;
  const int variant = (drop ? 4 : 0) | (km ? 2 : 0) | (small ? 1 : 0);
  auto q = (const bf16_raw*)qkv;
  auto g = (const bf16_raw*)dout;
  auto dq = (bf16_raw*)dqkv;
  // the main kernel forms the V-bias partials with dropout (per key block)
  float* vp = drop ? vparts : nullptr;
  int nq_rows = bp.nq;  // partial rows of the Q-bias column sums
  if (hd128) {
    auto k = drop ? (km ? attn::attn_bwd128_kernel<true, true> : attn::attn_bwd128_kernel<true, false>)
                  : (km ? attn::attn_bwd128_kernel<false, true> : attn::attn_bwd128_kernel<false, false>);
    hipLaunchKernelGGL(k, dim3(B * H, nkb), dim3(256), 0, stream, q, g, lse, delta, dq, dq_part, vp, T, H, nkb,
                       dropout, d.key_valid);
    // dQ: sum of the key blocks' bf16 partial planes (+ the Q-bias partial rows)
    hipLaunchKernelGGL((attn::attn_dq_reduce_kernel<false, 2>), dim3(B * H, (T + attn::kDqRows - 1) / attn::kDqRows),
                       dim3(256), 0, stream, (const bf16_raw*)dq_part, dq, qparts, T, H, hd, nkb,
                       rows * (long)bwd_plane_width(hd), kvblk);
  } else {
  // one workgroup per (b, h) over its key blocks (fp32 dQ inside, no reduce pass) when B*H fills
  // the CUs evenly (>= 85 % of the slots of its last round) and there is no dropout (the dropout
  // body spills in that form); else one per (b, h, key block).  Same box, B = 128 / 32, H = 12
  // (1,536 / 384 pairs): 0.98 vs 1.11 ms per-(b, h), 0.34 vs 0.31 ms split.
  const int ncu = device_cu_count(), pairs = B * H;
  const bool split = nkb > 1 && (drop || (long)pairs * 100 < 85L * ncu * ((pairs + ncu - 1) / ncu));
  const dim3 grid(pairs, split ? nkb : 1);
  switch (variant) {
    case 0: launch_bwd_variant<false, false, false>(grid, stream, q, g, lse, delta, dq, dq_part, vp, qparts, d, nkb, dropout); break;
    case 1: launch_bwd_variant<false, false, true>(grid, stream, q, g, lse, delta, dq, dq_part, vp, qparts, d, nkb, dropout); break;
    case 2: launch_bwd_variant<false, true, false>(grid, stream, q, g, lse, delta, dq, dq_part, vp, qparts, d, nkb, dropout); break;
    case 3: launch_bwd_variant<false, true, true>(grid, stream, q, g, lse, delta, dq, dq_part, vp, qparts, d, nkb, dropout); break;
    case 4: launch_bwd_variant<true, false, false>(grid, stream, q, g, lse, delta, dq, dq_part, vp, qparts, d, nkb, dropout); break;
    case 5: launch_bwd_variant<true, false, true>(grid, stream, q, g, lse, delta, dq, dq_part, vp, qparts, d, nkb, dropout); break;
    case 6: launch_bwd_variant<true, true, false>(grid, stream, q, g, lse, delta, dq, dq_part, vp, qparts, d, nkb, dropout); break;
    default: launch_bwd_variant<true, true, true>(grid, stream, q, g, lse, delta, dq, dq_part, vp, qparts, d, nkb, dropout); break;
  }
  if (split) {
    auto rk = small ? attn::attn_dq_reduce_kernel<true> : attn::attn_dq_reduce_kernel<false>;
    hipLaunchKernelGGL(rk, dim3(pairs, (T + attn::kDqRows - 1) / attn::kDqRows), dim3(256), 0, stream,
                       (const bf16_raw*)dq_part, dq, qparts, T, H, hd, nkb, rows * (long)attn::kHD, kvblk);
  }
  nq_rows = split ? bp.nq : B;
  }
  if (dbias != nullptr) {
    // fixed-order sums of the partial rows: Q part (a row per (b, row tile) from the hd-128 dQ
    // reduce, a row per b from the 8-wave kernel), then (unless the out-proj GEMM's epilogue
    // already added it) the V part; the K part of the qkv-bias gradient is exactly zero
    hipError_t e = launch_colsum_reduce(qparts, nq_rows, bp.cols, dbias, scratch, stream);
    if (e != hipSuccess) return e;
    const int nv = drop ? B * nkb : (v_from_delta ? (int)dgrid.x * B : 0);
    if (nv > 0) {
      e = launch_colsum_reduce(vparts, nv, bp.cols, dbias + 2L * H * hd, scratch, stream);
      if (e != hipSuccess) return e;
    }
  }
  return hipGetLastError();
}

}  // namespace llmt
