// Causal flash-attention backward, head_dim 64, for gfx950 (MI355X).
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
//  * per 32-row query tile: S = Q K^T and dP = dO V^T with the accumulators PRE-LOADED with the
//    row constants (-LSE/scale and -delta) so exp2(c*S) is P directly and dP - delta comes out
//    of the MFMA chain; dS = P o (dP - delta);
//  * P and dS are already the B operands of dV^T += dO^T P and dK^T += Q^T dS (accumulator used
//    as the next MFMA's operand); dO^T and Q^T fragments come from ds_read_b64_tr_b16 on the
//    same LDS images that serve the row reads (one swizzle, conflict free both ways);
//  * dS crosses LDS once (as a [key][q] image written 8 bytes per lane) and dQ = dS K is formed
//    with 16x16x32 MFMAs over the block's 256 keys, then added to an f32 dQ buffer with
//    no-return float atomics (dQ bytes / 1.3 TB/s is the floor of this design; a 256-key block
//    halves it vs 128).  A tiny epilogue kernel converts dQ to bf16 into the packed dqkv.
#include <cstdlib>
#include <cstring>

#include "attention_common.h"

namespace llmt {
namespace attn {

constexpr int kBwdWaves = 8;
constexpr int kKvBlk = 32 * kBwdWaves;  // 256 keys per workgroup
constexpr int kQTile = 64;  // query rows per sweep step (two 32-row MFMA tiles)

// delta[b, h, t] = sum_d dO[b, t, h, d] * O[b, t, h, d]; 8 lanes per row
__global__ __launch_bounds__(256) void attn_delta_kernel(const bf16_raw* __restrict__ dout,
                                                         const bf16_raw* __restrict__ out,
                                                         float* __restrict__ delta, int T, int H, long rows) {
  const long row = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 3;  // row = (b*T + t)*H + h
  const int sub = threadIdx.x & 7;
  float acc = 0.f;
  if (row < rows) {
    float a[8], o[8];
    unpack8(*reinterpret_cast<const ushort8_t*>(dout + row * kHD + 8 * sub), a);
    unpack8(*reinterpret_cast<const ushort8_t*>(out + row * kHD + 8 * sub), o);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i] * o[i];
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (row < rows && sub == 0) {
    const long bt = row / H;
    const int h = (int)(row - bt * H);
    const long b = bt / T, t = bt - b * T;
    delta[(b * H + h) * T + t] = acc;
  }
}

// dqkv[b, t, 0, h, :] = bf16(dq_accum[b, t, h, :])
__global__ __launch_bounds__(256) void attn_dq_store_kernel(const float* __restrict__ dq, bf16_raw* __restrict__ dqkv,
                                                            int H, long n8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one 8-element chunk
  if (i >= n8) return;
  const long row = i >> 3;  // (b*T + t)*H + h
  const int c = (int)(i & 7);
  const long bt = row / H;
  const int h = (int)(row - bt * H);
  const float4_t* src = reinterpret_cast<const float4_t*>(dq + row * kHD + 8 * c);
  const float4_t a = src[0], b2 = src[1];
  const float f[8] = {a[0], a[1], a[2], a[3], b2[0], b2[1], b2[2], b2[3]};
  *reinterpret_cast<ushort8_t*>(dqkv + (bt * 3 * H + h) * kHD + 8 * c) = pack8(f);
}

template <bool DQ_ATOMICS>
__global__ __launch_bounds__(512, 1) void attn_bwd_kernel(const bf16_raw* __restrict__ qkv,
                                                          const bf16_raw* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ delta,
                                                          bf16_raw* __restrict__ dqkv,
                                                          float* __restrict__ dq_accum, int T, int H) {
  __shared__ __attribute__((aligned(16))) bf16_raw k_lds[kKvBlk * kHD];          // 32 KB
  __shared__ __attribute__((aligned(16))) bf16_raw qd_lds[2][2][kQTile * kHD];   // [buf][Q|dO] 32 KB
  __shared__ __attribute__((aligned(16))) bf16_raw ds_lds[kKvBlk * kQTile];      // [key][q] 32 KB
  __shared__ __attribute__((aligned(16))) float rowc_lds[2][2 * kQTile];         // -lse/scale | -delta

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably wave-uniform
  const int half = lane >> 5, col = lane & 31;
  const int kb = blockIdx.x;
  const int bh = blockIdx.y;
  const int b = bh / H, h = bh - b * H;
  const long row_stride = 3L * H * kHD;
  const bf16_raw* base = qkv + (long)b * T * row_stride + (long)h * kHD;
  const bf16_raw* dobase = dout + (long)b * T * H * kHD + (long)h * kHD;  // [B, T, H, 64]
  const long out_stride = (long)H * kHD;
  const float* lse_bh = lse + ((long)b * H + h) * T;
  const float* delta_bh = delta + ((long)b * H + h) * T;

  const int kblk0 = kb * kKvBlk;
  const int kw0 = kblk0 + 32 * wave;  // first key of this wave
  const int key = kw0 + col;          // this lane's key

  constexpr float scale = 0.125f;
  constexpr float c = scale * 1.4426950408889634f;

  // K and V fragments of this lane's key: B operands of S = Q K^T and dP = dO V^T
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    ushort8_t kz = {0, 0, 0, 0, 0, 0, 0, 0}, vz = kz;
    if (key < T) {
      const bf16_raw* src = base + (long)key * row_stride + 16 * kk + 8 * half;
      kz = *reinterpret_cast<const ushort8_t*>(src + kHD * H);
      vz = *reinterpret_cast<const ushort8_t*>(src + 2 * kHD * H);
    }
    kf[kk] = __builtin_bit_cast(bf16x8, kz);
    vf[kk] = __builtin_bit_cast(bf16x8, vz);
  }
  // whole 256-key K block into LDS (B operand of dQ = dS K through transposed reads)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cidx = threadIdx.x + 512 * i;
    const int r = cidx >> 3, ch = cidx & 7;
    ushort8_t kz = {0, 0, 0, 0, 0, 0, 0, 0};
    if (kblk0 + r < T) kz = *reinterpret_cast<const ushort8_t*>(base + (long)(kblk0 + r) * row_stride + kHD * H + ch * 8);
    *reinterpret_cast<ushort8_t*>(&k_lds[tile_chunk_off(r, ch)]) = kz;
  }

  // register staging of one 64-row Q/dO tile (+ its row constants): 2 chunks per thread
  ushort8_t stg[2];
  float stc = 0.f;
  auto load_tile = [&](int q0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cidx = threadIdx.x + 512 * i;
      const int which = cidx >> 9, r = (cidx >> 3) & 63, ch = cidx & 7;
      const int qrow = q0 + r;
      ushort8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (qrow < T)
        v = which == 0 ? *reinterpret_cast<const ushort8_t*>(base + (long)qrow * row_stride + ch * 8)
                       : *reinterpret_cast<const ushort8_t*>(dobase + (long)qrow * out_stride + ch * 8);
      stg[i] = v;
    }
    if (threadIdx.x < 2 * kQTile) {
      const int qq = q0 + (threadIdx.x & (kQTile - 1));
      stc = 0.f;
      if (qq < T) stc = threadIdx.x < kQTile ? -lse_bh[qq] / scale : -delta_bh[qq];
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cidx = threadIdx.x + 512 * i;
      const int which = cidx >> 9, r = (cidx >> 3) & 63, ch = cidx & 7;
      *reinterpret_cast<ushort8_t*>(&qd_lds[buf][which][tile_chunk_off(r, ch)]) = stg[i];
    }
    if (threadIdx.x < 2 * kQTile) rowc_lds[buf][threadIdx.x] = stc;
  };

  f32x16 dk[2], dv[2];
  dk[0] = 0.f; dk[1] = 0.f; dv[0] = 0.f; dv[1] = 0.f;

  const int qt_dq = wave & 3;   // dQ output rows 16*qt_dq .. of the 64-row tile
  const int dp_dq = wave >> 2;  // dQ output cols 32*dp_dq .. (two 16-wide tiles)

  load_tile(kblk0);
  store_tile(0);
  __syncthreads();

  int it = 0;
  for (int q0 = kblk0; q0 < T; q0 += kQTile, ++it) {
    const int cur = it & 1;
    const bool more = q0 + kQTile < T;
    if (more) load_tile(q0 + kQTile);  // latency hidden under this tile's MFMAs
    const bf16_raw* q_lds = qd_lds[cur][0];
    const bf16_raw* do_lds = qd_lds[cur][1];
    const float* rowc = rowc_lds[cur];

#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qb0 = q0 + 32 * qs;
      const bool active = kw0 <= qb0 + 31 && kw0 < T && qb0 < T;  // wave-uniform
      f32x16 p, ds;
      if (active) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const f32x4 lc = *reinterpret_cast<const f32x4*>(&rowc[32 * qs + 8 * rr + 4 * half]);
          const f32x4 dc = *reinterpret_cast<const f32x4*>(&rowc[kQTile + 32 * qs + 8 * rr + 4 * half]);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            p[4 * rr + i] = lc[i];
            ds[4 * rr + i] = dc[i];
          }
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const bf16x8 qa = lds_row_read(q_lds, 32 * qs + col, 2 * kk + half);
          p = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[kk], p, 0, 0, 0);
          const bf16x8 da = lds_row_read(do_lds, 32 * qs + col, 2 * kk + half);
          ds = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[kk], ds, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) p[r] = __builtin_amdgcn_exp2f(p[r] * c);
        // causal / sequence-end mask, diagonal and tail tiles only (wave-uniform branch): element
        // r is query qb0 + 4*half + (r&3) + 8(r>>2), valid iff key <= query < T (branch-free)
        if ((kw0 + 31 > qb0) || (kw0 + 32 > T) || (qb0 + 32 > T)) {
          const int lo = key - qb0 - 4 * half, hi = T - 1 - qb0 - 4 * half;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int roff = (r & 3) + 8 * (r >> 2);
            p[r] = (roff < lo || roff > hi) ? 0.f : p[r];
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) ds[r] = p[r] * ds[r];
        // dV^T += dO^T P ; dK^T += Q^T dS  (P, dS used in place as B operands)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pb = pack_acc8(p, st);
          const bf16x8 sb = pack_acc8(ds, st);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const bf16x8 doa = lds_tr_read_operand(do_lds, 32 * qs + 16 * st + 4 * half, dt * 32, lane);
            dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(doa, pb, dv[dt], 0, 0, 0);
            const bf16x8 qa = lds_tr_read_operand(q_lds, 32 * qs + 16 * st + 4 * half, dt * 32, lane);
            dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, sb, dk[dt], 0, 0, 0);
          }
        }
      } else {
        ds = 0.f;
      }
      // dS^T image [key][q]: this lane's key, q rows 32 qs + 8g + 4h .. +3 (one 8-byte write each)
      const int kl = 32 * wave + col;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        ushort4_t v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = f2bf(ds[4 * g + i]);
        *reinterpret_cast<ushort4_t*>(&ds_lds[tile_elem_off(kl, 32 * qs + 8 * g + 4 * half)]) = v;
      }
    }
    __syncthreads();

    // ---- dQ[q0 + 16 qt .., 32 dp + (0..31)] += dS K over the block's 256 keys (16x16x32) ----
    {
      const int i = lane & 15, g = lane >> 4;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      typedef short short8v __attribute__((ext_vector_type(8)));
#pragma unroll
      for (int ks = 0; ks < kKvBlk / 32; ++ks) {
        const int krow = 32 * ks + 8 * g + (i >> 2);
        const int qcol = 16 * qt_dq + 4 * (i & 3);
        const short4v a_lo = tr_read(ds_lds, krow, qcol);
        const short4v a_hi = tr_read(ds_lds, krow + 4, qcol);
        const short8v av = {a_lo[0], a_lo[1], a_lo[2], a_lo[3], a_hi[0], a_hi[1], a_hi[2], a_hi[3]};
        const int dcol = 32 * dp_dq + 4 * (i & 3);
        const short4v b0l = tr_read(k_lds, krow, dcol), b0h = tr_read(k_lds, krow + 4, dcol);
        const short4v b1l = tr_read(k_lds, krow, dcol + 16), b1h = tr_read(k_lds, krow + 4, dcol + 16);
        const short8v b0 = {b0l[0], b0l[1], b0l[2], b0l[3], b0h[0], b0h[1], b0h[2], b0h[3]};
        const short8v b1 = {b1l[0], b1l[1], b1l[2], b1l[3], b1h[0], b1h[1], b1h[2], b1h[3]};
        const bf16x8 a = __builtin_bit_cast(bf16x8, av);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, b0), acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, b1), acc1, 0, 0, 0);
      }
      const int d0 = 32 * dp_dq + i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = q0 + 16 * qt_dq + 4 * g + r;
        if (qq < T) {
          float* dst = &dq_accum[(((long)b * T + qq) * H + h) * kHD + d0];
          if (DQ_ATOMICS) {
            atomicAdd(dst, acc0[r] * scale);
            atomicAdd(dst + 16, acc1[r] * scale);
          } else {  // timing experiment only (LLMT_EXPERIMENT=attn_no_dq): wrong dQ
            asm volatile("" ::"v"(acc0[r]), "v"(acc1[r]));
          }
        }
      }
    }
    if (more) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- dK = scale * dK^T, dV = dV^T  -> dqkv[b, key, 1|2, h, :] ------------------------------
  if (key < T) {
    bf16_raw* dst = dqkv + ((long)b * T + key) * row_stride + (long)h * kHD;
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
        *reinterpret_cast<ushort4_t*>(dst + kHD * H + d) = kv;
        *reinterpret_cast<ushort4_t*>(dst + 2 * kHD * H + d) = vv;
      }
    }
  }
}

}  // namespace attn

hipError_t launch_attn_bwd(const void* dout, const void* qkv, const void* out, const float* lse, void* dqkv,
                           float* delta, float* dq_accum, int B, int T, int H, hipStream_t stream) {
  if (B <= 0 || T <= 0 || H <= 0) return hipErrorInvalidValue;
  const long rows = (long)B * T * H;
  hipError_t e = hipMemsetAsync(dq_accum, 0, rows * attn::kHD * sizeof(float), stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(attn::attn_delta_kernel, dim3((rows * 8 + 255) / 256), dim3(256), 0, stream,
                     (const bf16_raw*)dout, (const bf16_raw*)out, delta, T, H, rows);
  const int nkb = (T + attn::kKvBlk - 1) / attn::kKvBlk;
  static const bool no_dq = [] {
    const char* e = getenv("LLMT_EXPERIMENT");
    return e != nullptr && strcmp(e, "attn_no_dq") == 0;
  }();
  auto kern = no_dq ? attn::attn_bwd_kernel<false> : attn::attn_bwd_kernel<true>;
  hipLaunchKernelGGL(kern, dim3(nkb, B * H), dim3(512), 0, stream, (const bf16_raw*)qkv,
                     (const bf16_raw*)dout, lse, delta, (bf16_raw*)dqkv, dq_accum, T, H);
  const long n8 = rows * attn::kHD / 8;
  hipLaunchKernelGGL(attn::attn_dq_store_kernel, dim3((n8 + 255) / 256), dim3(256), 0, stream, dq_accum,
                     (bf16_raw*)dqkv, H, n8);
  return hipGetLastError();
}

}  // namespace llmt
