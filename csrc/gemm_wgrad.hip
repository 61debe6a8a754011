// Weight-gradient GEMM for gfx950:  C[N, K] (f32, accumulated in place) += A^T B
//   A = dY [M, N] bf16 row-major (lda), B = X [M, K] bf16 row-major (ldb), reduction over M.
//
// Why a hand-written kernel: in a GPT step every weight gradient is a "tall-skinny" reduction
// (M = batch*seq = 32768 tokens deep, output only 768..3072 wide).  hipBLASLt picks 256x256
// macro-tiles without split-K for these, i.e. 9..48 workgroups for 256 CUs, and measures
// 210-520 TFLOP/s on MI355X (bench/micro.py).  Here the M reduction is split across
// workgroups (split-K) so every launch fills the chip, and the partial tiles are summed with
// no-return f32 atomics straight into the flat fp32 gradient buffer — the beta=1 accumulation
// the training step needs anyway (no "grad += tmp" pass).
//
// Structure (MI355X playbook: LDS-DMA staging, counted vmcnt, raw barriers, XCD remap):
//  * 128(n) x 128(k) output tile per 4-wave workgroup, each wave 64x64 = 2x2
//    v_mfma_f32_32x32x16_bf16 accumulators;
//  * operands stream through a 4-slot LDS ring of 32-row stages filled by
//    `buffer_load_dwordx4 ... lds` (no VGPR staging, 3 stages in flight); the buffer
//    descriptor's record count ends at the workgroup's M chunk, so rows past the chunk (and past
//    the array) read as zero with no branches;
//  * waits are counted (`s_waitcnt vmcnt(8|4|0)` = "this stage landed, the next two may still be
//    in flight") followed by a raw s_barrier, never __syncthreads() (whose vmcnt(0) would drain
//    the whole ring every stage);
//  * both operands have the reduction index running DOWN their rows, so both are read with the
//    transposing ds_read_b64_tr_b16; each 256-byte LDS row is XOR-swizzled by 4*(row & 3) chunks
//    (the swizzle is applied to the per-lane SOURCE address because the LDS-DMA destination is
//    lane-linear), which makes every transposed read bank-conflict free;
//  * work items are remapped so the workgroups of one M chunk run on one XCD and share its L2;
//  * epilogue: one f32 atomic per accumulator register and lane — lanes 0-31 / 32-63 each add a
//    contiguous 128-byte row segment, the full-rate atomic shape.
#include "common.h"
#include "kernels.h"

namespace llmt {
namespace wgrad {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) short4v lds_short4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BN = 128, BK = 128, BM = 32, NSLOT = 4;
constexpr int kThreads = 256;
constexpr int kOperandElems = BM * 128;           // one operand of one stage: 32 rows x 128 cols
constexpr int kSlotElems = 2 * kOperandElems;     // A + B

__device__ __forceinline__ int swz_off(int row, int col) {  // element offset in a [rows][128] image
  return row * 128 + ((((col >> 3) ^ ((row & 3) << 2))) << 3) + (col & 7);
}

// 32x32x16 operand with k running down the rows: lane l -> column col0 + (l & 31),
// elements j = 0..7 -> rows row0 + 8*(l >> 5) + j
__device__ __forceinline__ bf16x8 tr_frag(const bf16_raw* tile, int row0, int col0, int lane) {
  const int i = lane & 15;
  const int row = row0 + 8 * (lane >> 5) + (i >> 2);
  const int col = col0 + 16 * ((lane >> 4) & 1) + 4 * (i & 3);
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(tile + swz_off(row, col)));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(tile + swz_off(row + 4, col)));
  const short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// "stage s landed for this wave" (n later stages, 4 DMA ops each, may stay in flight) followed
// by the workgroup barrier, in ONE asm statement with a memory clobber so no LDS read can be
// scheduled between the wait and the barrier.
__device__ __forceinline__ void wait_stage_and_barrier(int n) {
  if (n >= 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
}

__global__ __launch_bounds__(kThreads, 2) void wgrad_kernel(const bf16_raw* __restrict__ A, int lda,
                                                            const bf16_raw* __restrict__ B, int ldb,
                                                            float* __restrict__ C, int ldc, int M, int N, int K,
                                                            int tiles, int tiles_k, int m_chunk, int nwg) {
  __shared__ __attribute__((aligned(16))) bf16_raw smem[NSLOT * kSlotElems];  // 64 KB ring
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // XCD-aware bijective remap: the 1/8 of the grid dispatched to one XCD gets contiguous work
  const int L = blockIdx.x, q = nwg >> 3, r = nwg & 7, xcd = L & 7;
  const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
  const int chunk = w / tiles, tile = w - chunk * tiles;
  const int tile_n = tile / tiles_k, tile_k = tile - tile_n * tiles_k;
  const int n0 = tile_n * BN, k0 = tile_k * BK;
  const int m_begin = chunk * m_chunk;
  const int rows = min(M - m_begin, m_chunk);
  if (rows <= 0) return;
  const int nst = (rows + BM - 1) / BM;

  // buffer descriptors over exactly this chunk's rows: anything past them reads as 0
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A + (long)m_begin * lda), (short)0, rows * lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(B + (long)m_begin * ldb), (short)0, rows * ldb * 2, 0x00020000);

  // this wave fills rows 8w..8w+7 of each operand in every stage: two 1-KiB DMA pieces each
  int va[2], vb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * wave + 4 * j + (lane >> 4);
    const int c = (lane & 15) ^ ((row & 3) << 2);  // inverse swizzle on the source address
    va[j] = (row * lda + n0 + 8 * c) * 2;
    vb[j] = (row * ldb + k0 + 8 * c) * 2;
  }
  // LDS-DMA issue in inline asm: hipcc does not track asm memory ops, so it cannot insert its
  // conservative "vmcnt(0) before every LDS read" — the counted waits below are the only ones.
  // M0 (the DMA destination base) is saved/restored inside the one statement that uses it.
  const unsigned lds_base = (unsigned)(unsigned long)(lds_void*)smem;
  auto issue = [&](int s) {
    const unsigned slot = lds_base + (unsigned)((s % NSLOT) * kSlotElems * 2);
    const unsigned la0 = slot + (8 * wave) * 256, la1 = la0 + 4 * 256;
    const unsigned lb0 = la0 + kOperandElems * 2, lb1 = lb0 + 4 * 256;
    const int soa = s * BM * lda * 2, sob = s * BM * ldb * 2;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %[keep], m0\n\t"
        "s_nop 4\n\t"
        "s_mov_b32 m0, %[la0]\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %[va0], %[ra], %[soa] offen lds\n\t"
        "s_mov_b32 m0, %[la1]\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %[va1], %[ra], %[soa] offen lds\n\t"
        "s_mov_b32 m0, %[lb0]\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %[vb0], %[rb], %[sob] offen lds\n\t"
        "s_mov_b32 m0, %[lb1]\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %[vb1], %[rb], %[sob] offen lds\n\t"
        "s_mov_b32 m0, %[keep]"
        : [keep] "=&s"(keep)
        : [la0] "s"(la0), [la1] "s"(la1), [lb0] "s"(lb0), [lb1] "s"(lb1), [va0] "v"(va[0]), [va1] "v"(va[1]),
          [vb0] "v"(vb[0]), [vb1] "v"(vb[1]), [ra] "s"(ra), [rb] "s"(rb), [soa] "s"(soa), [sob] "s"(sob)
        : "memory");
  };

  const int wn = wave >> 1, wk = wave & 1;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = 0.f;

#pragma unroll
  for (int s = 0; s < NSLOT - 1; ++s)
    if (s < nst) issue(s);

  for (int s = 0; s < nst; ++s) {
    wait_stage_and_barrier(min(nst - 1 - s, NSLOT - 2));  // stage s landed; slot s-1 free again
    if (s + NSLOT - 1 < nst) issue(s + NSLOT - 1);
    const bf16_raw* a = smem + (s % NSLOT) * kSlotElems;
    const bf16_raw* b = a + kOperandElems;
#pragma unroll
    for (int ks = 0; ks < BM / 16; ++ks) {
      bf16x8 af[2], bfv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = tr_frag(a, 16 * ks, wn * 64 + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfv[j] = tr_frag(b, 16 * ks, wk * 64 + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: C[n][k] += acc (rows n in registers, column k on the lane)
  const int half = lane >> 5, col = lane & 31;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = k0 + wk * 64 + 32 * j + col;
      if (k >= K) continue;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int n = n0 + wn * 64 + 32 * i + (rr & 3) + 8 * (rr >> 2) + 4 * half;
        if (n < N) atomicAdd(C + (long)n * ldc + k, acc[i][j][rr]);
      }
    }
  }
}

}  // namespace wgrad

hipError_t launch_wgrad_gemm(const void* dy, int lda, const void* x, int ldb, float* c, int ldc, int M, int N,
                             int K, int split, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  if (lda % 8 || ldb % 8 || N % 8 || K % 8) return hipErrorInvalidValue;
  const int tiles_n = (N + wgrad::BN - 1) / wgrad::BN, tiles_k = (K + wgrad::BK - 1) / wgrad::BK;
  const int tiles = tiles_n * tiles_k;
  const int max_split = (M + wgrad::BM - 1) / wgrad::BM;
  if (split <= 0) split = (512 + tiles - 1) / tiles;  // ~2 workgroups per CU
  split = split < 1 ? 1 : (split > max_split ? max_split : split);
  int m_chunk = (M + split - 1) / split;
  m_chunk = (m_chunk + wgrad::BM - 1) / wgrad::BM * wgrad::BM;
  split = (M + m_chunk - 1) / m_chunk;
  // 32-bit buffer offsets: one chunk of either operand must stay below 2 GiB
  if ((long long)m_chunk * (lda > ldb ? lda : ldb) * 2 >= (1LL << 31)) return hipErrorInvalidValue;
  const int nwg = tiles * split;
  hipLaunchKernelGGL(wgrad::wgrad_kernel, dim3(nwg), dim3(wgrad::kThreads), 0, stream, (const bf16_raw*)dy, lda,
                     (const bf16_raw*)x, ldb, c, ldc, M, N, K, tiles, tiles_k, m_chunk, nwg);
  return hipGetLastError();
}

}  // namespace llmt
