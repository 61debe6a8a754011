// Forward GEMM, ping-pong schedule (gfx950):  C[M, N] (bf16) = X[M, K] W[N, K]^T (+ bias) (+ GELU)
//
// The nn.Linear forward of every GPT block (reference models/gpt.py:27-29, 94-96: qkv / out /
// fc / proj), as the weight-gradient kernel's schedule (gemm_wgrad_pp.hip) applied to the
// "both operands K-contiguous" layout:
//
//  * 512-thread workgroups, 2 waves per SIMD, one 256 x 256 output tile per workgroup; waves 0-3
//    ("X") and 4-7 ("Y", one barrier behind) alternate a LOAD segment (fragment reads) and an MFMA
//    segment (32 x v_mfma_f32_16x16x32_bf16, 128 (n) x 64 (m) per wave), so one wave's MFMAs cover
//    its partner's LDS work;
//  * the MFMA computes D = W X^T (n on the accumulator rows): a lane's 4 accumulator registers are
//    4 consecutive n of one m, i.e. 8 contiguous bytes of a row of C — stored straight from
//    registers, no LDS round trip;
//  * stages of 32 k: both images are [256 rows][32 k] (64-byte rows), fragments are single
//    ds_read_b128 (12 per wave and stage vs 24 transposed half-reads in the weight gradient); the
//    16-byte chunk of a row is XOR-swizzled by (row >> 2) & 3, which puts the 16 rows a 16-lane
//    group reads on 16 distinct 16-byte bank slots;
//  * fills are register-staged (4 x 16-byte buffer loads per thread and stage, ds_write_b128 at
//    the swizzled address) through a 2-slot ring (64 KiB); FILL 1 issues them in the LOAD segment,
//    FILL 3 inside the wave's own MFMA segment with the weight-gradient kernel's asymmetric X / Y
//    stage schedule (X writes stage st+1, Y stage st+2; see gemm_wgrad_pp.hip);
//  * tiles are enumerated n-fastest and remapped per XCD, so the workgroups that share one X row
//    band run on one XCD and read it from HBM once; the weights (<= 5 MB) stay L2-resident.
//
// KN (data gradient dX = dY W of nn.Linear, W [K_red][N] row-major): the W operand has the reduction
// index down its rows, so its image is the weight-gradient kernel's [32][256] layout (512-byte rows,
// 32-byte segments XOR-swizzled by f(row)) read with ds_read_b64_tr_b16; dY stays a [256][32] image.
//
// Epilogues (EPI): 0 = bf16(acc + bias); 1 = u = bf16(acc + bias) and bf16(gelu(u)) (fc forward,
// the pre-activation is kept for the backward); 2 = bf16(acc * gelu'(u)) with u read from C2's
// place (proj dX fused with the GELU backward); 3 = bf16(acc) and delta[b, h, t] = sum_d dO * O
// over each 64-wide head with O read from C2's place (out-proj dX fused with the attention
// backward's row constants).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

namespace llmt {
namespace gpp {

using namespace gemm;

constexpr int kThreads = 512;
constexpr int BR = 32;            // k per stage
constexpr int TW = 256;           // tile edge
constexpr int ROWB = BR * 2;      // 64 bytes per image row
constexpr int IMG = TW * ROWB;    // 16 KiB per operand per stage
constexpr int SLOT = 2 * IMG;     // 32 KiB: [W image | X image]
constexpr int NS = 2;             // ring slots
constexpr int FA = 8, FB = 4;     // fragments per wave: 8 x 16 n (W), 4 x 16 m (X)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr float kInvSqrt2 = 0.70710678118654752f;

// exact-erf GELU (A&S 7.1.26 erf, |err| < 1.5e-7; the same as elementwise.hip / gemm_fused.hip)
__device__ __forceinline__ float gelu_erf(float u) {
  constexpr float kLog2e = 1.4426950408889634f;
  const float az = fabsf(u) * kInvSqrt2;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-0.5f * kLog2e * u * u);
  const float erf = copysignf(fmaf(-p * t, e, 1.f), u);
  return 0.5f * u * (1.f + erf);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int bytes) {
  const unsigned long a = (unsigned long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long)hi << 32) | lo), (short)0, n, 0x00020000);
}

__device__ __forceinline__ float gelu_erf_grad(float u) {
  constexpr float kLog2e = 1.4426950408889634f, kInvSqrt2Pi = 0.39894228040143268f;
  const float az = fabsf(u) * kInvSqrt2;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-0.5f * kLog2e * u * u);
  const float erf = copysignf(fmaf(-p * t, e, 1.f), u);
  return fmaf(0.5f, 1.f + erf, u * kInvSqrt2Pi * e);
}

// KN W image: 32-byte segment swizzle of the weight-gradient kernel (8 rows one 32-lane half reads
// with ds_read_b64_tr_b16 land on 8 distinct bank groups)
constexpr int KROWB = TW * 2;  // 512-byte rows
__device__ __forceinline__ int swz_f(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }
__device__ __forceinline__ bf16x8 tr_read(unsigned addr) {
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(unsigned long)addr);
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(unsigned long)(addr + 4 * KROWB));
  const short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int EPI, int FILL, bool KN>
__global__ __launch_bounds__(kThreads, 2) void gemm_pp_kernel(const bf16_raw* __restrict__ X, int ldx,
                                                             const bf16_raw* __restrict__ W, int ldw,
                                                             const bf16_raw* __restrict__ bias,
                                                             bf16_raw* __restrict__ C, bf16_raw* __restrict__ C2,
                                                             int ldc, int M, int N, int K, int tiles_n, int nwg,
                                                             float* __restrict__ delta, int T) {
  __shared__ __attribute__((aligned(16))) bf16_raw smem[NS * SLOT / 2];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave >> 2, wk = wave & 3;  // wn: 0 = X (leads), 1 = Y; wk: 64-row m slice

  const int w = xcd_remap(blockIdx.x, nwg);
  const int tile_m = w / tiles_n, tile_n = w - tile_m * tiles_n;
  const int m0 = tile_m * TW, n0 = tile_n * TW;
  const int nst = K / BR;  // K % 32 == 0 (host check)

  // tile descriptors: rows past M / N read as zeros (KN: the W block starts at column n0; a row's
  // columns past N read the next row — their outputs are never stored — and the last rows' reads
  // past the matrix end read zeros)
  const __amdgpu_buffer_rsrc_t rw = KN ? uniform_rsrc(W + n0, (K * ldw - n0) * 2)
                                       : uniform_rsrc(W + (long)n0 * ldw, min(TW, N - n0) * ldw * 2);
  const __amdgpu_buffer_rsrc_t rx = uniform_rsrc(X + (long)m0 * ldx, min(TW, M - m0) * ldx * 2);

  // fill: thread t moves chunks c = t and t + 512 of each image (row c >> 2, 16-byte chunk c & 3)
  const int frow = threadIdx.x >> 2, fq = threadIdx.x & 3;
  int vw[2], vx[2];
  unsigned wdst[2];
  unsigned xdst[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = frow + 128 * h;
    vx[h] = (row * ldx + 8 * fq) * 2;
    xdst[h] = (unsigned)(row * ROWB + 16 * (fq ^ ((row >> 2) & 3)));
    if (KN) {  // W image [32][256]: chunk c = t + 512 h is row c >> 5, 16-byte chunk c & 31
      const int c = threadIdx.x + 512 * h, kr = c >> 5, ch = c & 31;
      vw[h] = (kr * ldw + 8 * ch) * 2;
      wdst[h] = (unsigned)(kr * KROWB + ((((ch >> 1) ^ swz_f(kr))) << 5) + 16 * (ch & 1));
    } else {
      vw[h] = (row * ldw + 8 * fq) * 2;
      wdst[h] = xdst[h];
    }
  }
  const int wstage = KN ? BR * ldw * 2 : ROWB;  // bytes per stage along the W operand
  const unsigned lds = (unsigned)(unsigned long)(lds_void*)smem;

  u32x4 R0[4], R1[4];
  // R[0], R[1]: W rows frow, frow + 128; R[2], R[3]: X rows.  Unconditional: the stages past the
  // last that the schedule loads (and writes to slots nobody reads again) re-load the last stage
  auto load_stage = [&](int st, u32x4 (&R)[4]) {
    const int ko = min(st, nst - 1) * ROWB, kw = min(st, nst - 1) * wstage;
    R[0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, vw[0] + kw, 0, 0));
    R[1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, vw[1] + kw, 0, 0));
    R[2] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, vx[0] + ko, 0, 0));
    R[3] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, vx[1] + ko, 0, 0));
  };
  auto write_part = [&](int slot, const u32x4 (&R)[4], int part) {  // part 0: W chunks, 1: X chunks
    const unsigned a = lds + slot * SLOT + part * IMG;
    *(lds_u32x4*)(size_t)(a + (part == 0 ? wdst[0] : xdst[0])) = R[2 * part];
    *(lds_u32x4*)(size_t)(a + (part == 0 ? wdst[1] : xdst[1])) = R[2 * part + 1];
  };
  auto write_stage = [&](int slot, const u32x4 (&R)[4]) {
    write_part(slot, R, 0);
    write_part(slot, R, 1);
  };

  // fragment read offsets: lane (c16 = l & 15, kc = l >> 4) reads row base + c16 at chunk kc ^ f,
  // f = (c16 >> 2) & 3 (row bases are multiples of 16)
  const int c16 = lane & 15, kc = lane >> 4;
  const unsigned rd = (unsigned)(c16 * ROWB + 16 * (kc ^ (c16 >> 2)));
  const unsigned wrd = rd + (unsigned)(128 * wn) * ROWB;             // + i * 16 rows
  // KN: lane (g, q, p) reads rows 8g + q (+4) of the W image at segment (8 wn + i) ^ f, bytes 8p..
  const int tg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int tfl = tq | ((tg & 1) << 2);
  unsigned kao[FA];
#pragma unroll
  for (int i = 0; i < FA; ++i) kao[i] = (unsigned)((8 * tg + tq) * KROWB + 8 * tp + ((8 * wn + (i ^ tfl)) << 5));
  const unsigned xrd = IMG + rd + (unsigned)(64 * wk) * ROWB;         // + j * 16 rows

  f32x4v acc[FA][FB];
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) acc[i][j] = 0.f;

  // prologue (as gemm_wgrad_pp.hip): FILL 1 — stage 0 written, stages 1 and 2 loading; FILL 3 —
  // X keeps stage s in set s & 1, Y in set (s + 1) & 1; X writes stage 0 (and 1), Y stages 0, 1
  if (FILL == 3) {
    load_stage(wn, R0);
    load_stage(1 - wn, R1);
    write_stage(wn, R0);
    write_stage(1 - wn, R1);
    load_stage(1 + wn, R1);
    load_stage(2 + wn, R0);
  } else {
    load_stage(0, R0);
    load_stage(1, R1);
    write_stage(0, R0);
    load_stage(2, R0);
  }
  lds_barrier();
  if (wn == 1) barrier();

  auto phase = [&](int st, int slot, u32x4 (&R)[4]) {
    const unsigned sb = lds + slot * SLOT;
    bf16x8 af[FA], bfr[FB];
#pragma unroll
    for (int i = 0; i < FA; ++i)
      af[i] = KN ? tr_read(sb + kao[i]) : *(const __attribute__((address_space(3))) bf16x8*)(size_t)(sb + wrd + i * 16 * ROWB);
#pragma unroll
    for (int j = 0; j < FB; ++j) bfr[j] = *(const __attribute__((address_space(3))) bf16x8*)(size_t)(sb + xrd + j * 16 * ROWB);
    if (FILL == 1) {
      write_stage(slot + 1 == NS ? 0 : slot + 1, R);
      load_stage(st + 3, R);
    }
    lds_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FA; ++i) {
#pragma unroll
      for (int j = 0; j < FB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (FILL == 3 && i < 4) {
        __builtin_amdgcn_sched_barrier(0);
        if (i < 2) {
          write_part((st + 1 - wn) & 1, R, i);
        } else {
          const int ko = min(st + 3 + wn, nst - 1) * ROWB, kw = min(st + 3 + wn, nst - 1) * wstage;
          if (i == 2) {
            R[0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, vw[0] + kw, 0, 0));
            R[1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, vw[1] + kw, 0, 0));
          } else {
            R[2] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, vx[0] + ko, 0, 0));
            R[3] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, vx[1] + ko, 0, 0));
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (FILL == 3) lds_barrier();
    else barrier();
  };
  // pairs of unconditional phases (K % 64 == 0: an even stage count)
  for (int s0 = 0; s0 < nst; s0 += 2) {
    phase(s0, 0, R1);
    phase(s0 + 1, 1, R0);
  }
  if (wn == 0) barrier();

  // ---- epilogue: acc[i][j] register r = D[n][m], n = n0 + 128 wn + 16 i + 4 (l >> 4) + r,
  // m = m0 + 64 wk + 16 j + (l & 15): 8 contiguous bytes of row m of C
  const int g = lane >> 4;
  const int nb = n0 + 128 * wn + 4 * g;
  const int mrow = m0 + 64 * wk + c16;
  float bv[FA][4];
#pragma unroll
  for (int i = 0; i < FA; ++i) {
    const int n = nb + 16 * i;
    if (EPI != 2 && bias != nullptr && n < N) {
      const u32x2 b2 = *(const u32x2*)(bias + n);
      bv[i][0] = __uint_as_float(b2[0] << 16);
      bv[i][1] = __uint_as_float(b2[0] & 0xffff0000u);
      bv[i][2] = __uint_as_float(b2[1] << 16);
      bv[i][3] = __uint_as_float(b2[1] & 0xffff0000u);
    } else {
      bv[i][0] = bv[i][1] = bv[i][2] = bv[i][3] = 0.f;
    }
  }
  const __amdgpu_buffer_rsrc_t rc = uniform_rsrc(C + (long)m0 * ldc, min(TW, M - m0) * ldc * 2);
  const __amdgpu_buffer_rsrc_t rc2 =
      uniform_rsrc((EPI >= 1 ? C2 : C) + (long)m0 * ldc, min(TW, M - m0) * ldc * 2);
#pragma unroll
  for (int j = 0; j < FB; ++j) {
    const int mo = (mrow + 16 * j - m0) * ldc * 2;
    float dot[2] = {0.f, 0.f};  // EPI 3: this lane's part of the row dot of each of the wave's 2 heads
#pragma unroll
    for (int i = 0; i < FA; ++i) {
      const int n = nb + 16 * i;
      if (n >= N) continue;
      float v[4];
      if (EPI == 2) {  // du = acc * gelu'(u), u from C2's place (same layout as C)
        const u32x2 uu = __builtin_amdgcn_raw_buffer_load_b64(rc2, mo + n * 2, 0, 0);
        const float uf[4] = {__uint_as_float(uu[0] << 16), __uint_as_float(uu[0] & 0xffff0000u),
                             __uint_as_float(uu[1] << 16), __uint_as_float(uu[1] & 0xffff0000u)};
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * gelu_erf_grad(uf[r]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bv[i][r];
      }
      const bf16_raw u0 = f2bf(v[0]), u1 = f2bf(v[1]), u2 = f2bf(v[2]), u3 = f2bf(v[3]);
      const u32x2 pu = {(unsigned)u0 | ((unsigned)u1 << 16), (unsigned)u2 | ((unsigned)u3 << 16)};
      __builtin_amdgcn_raw_buffer_store_b64(pu, rc, mo + n * 2, 0, 0);
      if (EPI == 3) {  // delta: the bf16 dO the attention backward reads, times O (from C2's place)
        const u32x2 oo = __builtin_amdgcn_raw_buffer_load_b64(rc2, mo + n * 2, 0, 0);
        dot[i >> 2] = fmaf(bf2f(u0), __uint_as_float(oo[0] << 16), dot[i >> 2]);
        dot[i >> 2] = fmaf(bf2f(u1), __uint_as_float(oo[0] & 0xffff0000u), dot[i >> 2]);
        dot[i >> 2] = fmaf(bf2f(u2), __uint_as_float(oo[1] << 16), dot[i >> 2]);
        dot[i >> 2] = fmaf(bf2f(u3), __uint_as_float(oo[1] & 0xffff0000u), dot[i >> 2]);
      }
      if (EPI == 1) {
        const float g0 = gelu_erf(bf2f(u0)), g1 = gelu_erf(bf2f(u1)), g2 = gelu_erf(bf2f(u2)), g3 = gelu_erf(bf2f(u3));
        const u32x2 pg = {(unsigned)f2bf(g0) | ((unsigned)f2bf(g1) << 16), (unsigned)f2bf(g2) | ((unsigned)f2bf(g3) << 16)};
        __builtin_amdgcn_raw_buffer_store_b64(pg, rc2, mo + n * 2, 0, 0);
      }
    }
    if (EPI == 3) {  // the 4 lanes g = 0..3 of a row hold its 64 head columns (N % 64 == 0)
      const int m = mrow + 16 * j;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        float d = dot[hh];
        d += __shfl_xor(d, 16, 64);
        d += __shfl_xor(d, 32, 64);
        const int head = (n0 + 128 * wn + 64 * hh) >> 6;
        if (g == 0 && m < M && 64 * head < N) {
          const int bb = m / T, t = m - bb * T;
          delta[((long)bb * (N >> 6) + head) * T + t] = d;
        }
      }
    }
  }
}

}  // namespace gpp

bool gemm_pp_supported(int M, int N, int K, int ldx, int ldw, int ldc, bool kn) {
  return M > 0 && N > 0 && K >= 64 && K % 64 == 0 && N % 8 == 0 && ldx % 8 == 0 && ldw % 8 == 0 && ldc % 8 == 0 &&
         (long long)gpp::TW * std::max(std::max(ldx, kn ? 0 : ldw), ldc) * 2 < (1LL << 31) &&
         (!kn || ((long long)K * ldw * 2 < (1LL << 31) && ldw >= N));
}

hipError_t launch_gemm_pp(const void* x, int ldx, const void* w, int ldw, const void* bias, void* c, void* c2, int ldc,
                          int M, int N, int K, int epi, bool kn, float* delta, int T, hipStream_t stream) {
  if (!gemm_pp_supported(M, N, K, ldx, ldw, ldc, kn) || (epi >= 1 && c2 == nullptr) || epi < 0 || epi > 3)
    return hipErrorInvalidValue;
  if (epi == 3 && (delta == nullptr || T <= 0 || M % T != 0 || N % 64 != 0)) return hipErrorInvalidValue;
  const int tiles_m = (M + gpp::TW - 1) / gpp::TW, tiles_n = (N + gpp::TW - 1) / gpp::TW;
  const int nwg = tiles_m * tiles_n;
  // fill placement (A/B knob LLMT_GPP_FILL=3: fills inside the MFMA segment; 1 measured equal or
  // faster on 8 of the 9 shapes, profiles/r4/gemm_pp/op_times_vs_hipblaslt.txt)
  static const int fill = [] {
    const char* e = std::getenv("LLMT_GPP_FILL");
    return e != nullptr && std::atoi(e) == 3 ? 3 : 1;
  }();
#define LLMT_GPP_LAUNCH(E, F, KN)                                                                                 \
  hipLaunchKernelGGL((gpp::gemm_pp_kernel<E, F, KN>), dim3(nwg), dim3(gpp::kThreads), 0, stream,                   \
                     (const bf16_raw*)x, ldx, (const bf16_raw*)w, ldw, (const bf16_raw*)bias, (bf16_raw*)c,          \
                     (bf16_raw*)c2, ldc, M, N, K, tiles_n, nwg, delta, T)
#define LLMT_GPP_FILLS(E, KN)            \
  if (fill == 1) LLMT_GPP_LAUNCH(E, 1, KN); \
  else LLMT_GPP_LAUNCH(E, 3, KN);
  if (!kn) {
    if (epi == 0) { LLMT_GPP_FILLS(0, false) }
    else if (epi == 1) { LLMT_GPP_FILLS(1, false) }
    else return hipErrorInvalidValue;
  } else {
    if (epi == 0) { LLMT_GPP_FILLS(0, true) }
    else if (epi == 2) { LLMT_GPP_FILLS(2, true) }
    else if (epi == 3) { LLMT_GPP_FILLS(3, true) }
    else return hipErrorInvalidValue;
  }
#undef LLMT_GPP_FILLS
#undef LLMT_GPP_LAUNCH
  return hipGetLastError();
}

}  // namespace llmt
