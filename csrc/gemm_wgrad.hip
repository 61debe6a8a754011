// Weight-gradient GEMM for gfx950:  C[N, K] (f32, accumulated in place) += A^T B
//   A = dY [M, N] bf16 row-major (lda), B = X [M, K] bf16 row-major (ldb), reduction over M.
//
// Why a hand-written kernel: in a GPT step every weight gradient is a "tall-skinny" reduction
// (M = batch*seq = 32768 tokens deep, output only 768..3072 wide).  hipBLASLt picks 256x256
// macro-tiles without split-K for these, i.e. 9..48 workgroups for 256 CUs, and measures
// 210-520 TFLOP/s on MI355X (bench/micro.py).  Here the M reduction is split across
// workgroups (split-K) so every launch fills the chip, and the partial tiles are summed with
// no-return f32 atomics straight into the flat fp32 gradient buffer — which is exactly the
// beta=1 accumulation the training step needs anyway (no extra "grad += tmp" pass).
//
// Tile: 128(n) x 128(k) per 4-wave workgroup, each wave 64x64 = 2x2 v_mfma_f32_32x32x16_bf16;
// 64-deep M stages double-buffered in LDS with register staging (global loads for stage s+1
// are issued before the MFMAs of stage s and written after them: one barrier per stage).
// Both operands have the reduction index running DOWN their rows, so both are read with the
// gfx950 transposing LDS read ds_read_b64_tr_b16 from row-major tile images whose 16-byte
// chunks are XOR-swizzled by 4*(row & 3) (the four rows one transposed read touches land in
// four different 64-byte quarters of the 256-byte bank row: conflict free).  Epilogue atomics
// are issued per accumulator register: lanes 0-31 and 32-63 each add one 128-byte row
// segment, the full-rate atomic shape.
#include "common.h"
#include "kernels.h"

namespace llmt {
namespace wgrad {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) short4v lds_short4;

constexpr int BN = 128, BK = 128, BM = 64;
constexpr int kThreads = 256;
constexpr int kTileElems = BM * 128;  // one operand stage: 64 rows x 128 columns

__device__ __forceinline__ int swz_off(int row, int col) {  // element offset in a [64][128] image
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

__global__ __launch_bounds__(kThreads, 2) void wgrad_kernel(const bf16_raw* __restrict__ A, int lda,
                                                            const bf16_raw* __restrict__ B, int ldb,
                                                            float* __restrict__ C, int ldc, int M, int N, int K,
                                                            int tiles_k, int m_chunk) {
  __shared__ __attribute__((aligned(16))) bf16_raw smem[2 * 2 * kTileElems];  // [buf][A|B][64][128]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile_n = blockIdx.x / tiles_k, tile_k = blockIdx.x - tile_n * tiles_k;
  const int n0 = tile_n * BN, k0 = tile_k * BK;
  const int m_begin = blockIdx.y * m_chunk;
  const int m_end = min(M, m_begin + m_chunk);
  if (m_begin >= m_end) return;
  const int nstages = (m_end - m_begin + BM - 1) / BM;

  // staging: each operand stage is 64 rows x 16 chunks = 1024 chunks, 4 per thread
  ushort8_t stA[4], stB[4];
  auto load_stage = [&](int s) {
    const int mbase = m_begin + s * BM;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = threadIdx.x + kThreads * i;
      const int r = c >> 4, ch = c & 15;
      const int m = mbase + r;
      const int na = n0 + ch * 8, kb = k0 + ch * 8;
      ushort8_t za = {0, 0, 0, 0, 0, 0, 0, 0}, zb = za;
      if (m < m_end) {
        if (na < N) za = *reinterpret_cast<const ushort8_t*>(A + (long)m * lda + na);
        if (kb < K) zb = *reinterpret_cast<const ushort8_t*>(B + (long)m * ldb + kb);
      }
      stA[i] = za;
      stB[i] = zb;
    }
  };
  auto store_stage = [&](int buf) {
    bf16_raw* a = smem + buf * 2 * kTileElems;
    bf16_raw* b = a + kTileElems;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = threadIdx.x + kThreads * i;
      const int r = c >> 4, ch = c & 15;
      const int off = r * 128 + ((ch ^ ((r & 3) << 2)) << 3);
      *reinterpret_cast<ushort8_t*>(a + off) = stA[i];
      *reinterpret_cast<ushort8_t*>(b + off) = stB[i];
    }
  };

  const int wn = wave >> 1, wk = wave & 1;  // 2x2 waves, 64x64 each
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = 0.f;

  load_stage(0);
  store_stage(0);
  __syncthreads();
  for (int s = 0; s < nstages; ++s) {
    const int cur = s & 1;
    const bool more = s + 1 < nstages;
    if (more) load_stage(s + 1);
    const bf16_raw* a = smem + cur * 2 * kTileElems;
    const bf16_raw* b = a + kTileElems;
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
    if (more) store_stage(cur ^ 1);
    __syncthreads();
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
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (n < N) atomicAdd(C + (long)n * ldc + k, acc[i][j][r]);
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
  if (split <= 0) {
    split = (512 + tiles - 1) / tiles;  // ~2 workgroups per CU
    const int max_split = (M + wgrad::BM - 1) / wgrad::BM;
    split = split < 1 ? 1 : (split > max_split ? max_split : split);
  }
  int m_chunk = (M + split - 1) / split;
  m_chunk = (m_chunk + wgrad::BM - 1) / wgrad::BM * wgrad::BM;
  split = (M + m_chunk - 1) / m_chunk;
  dim3 grid(tiles, split);
  hipLaunchKernelGGL(wgrad::wgrad_kernel, grid, dim3(wgrad::kThreads), 0, stream, (const bf16_raw*)dy, lda,
                     (const bf16_raw*)x, ldb, c, ldc, M, N, K, tiles_k, m_chunk);
  return hipGetLastError();
}

}  // namespace llmt
