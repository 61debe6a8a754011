// Shared pieces of the gfx950 flash-attention kernels (head_dim 64).
#pragma once

#include "common.h"
#include "kernels.h"

namespace llmt {
namespace attn {

constexpr int kHD = 64;  // head dim: one 128-byte bf16 row per key/query
// a buffer-load byte offset past every descriptor's record count (records stay < 2 GiB - 64):
// the load returns zeros without touching memory
constexpr int kOobOff = 0x7ffffff0;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4;
typedef __attribute__((address_space(3))) void lds_void;

// Dispatch order of a (B*H) x nblk attention grid (x fastest): (b, h) pairs in chunks of
// kDispatchChunk; inside a chunk every pair's heaviest block first, then the next-heaviest, ...
// Heaviest-first keeps the causal tail short (a grid that ends on heavy blocks left ~40% of the
// slots idle); the chunk keeps all blocks of a pair close in time, so its K/V (forward) or Q/dO
// (backward) are re-read from L2 / Infinity Cache instead of HBM once the whole qkv no longer fits
// there (B=128: 604 MB).  With chunk and pair counts multiples of 8, every block of a pair runs on
// one XCD.  Returns (pair, heaviness rank 0 = heaviest).
constexpr int kDispatchChunk = 64;
__device__ __forceinline__ void chunked_dispatch(int& pair, int& rank) {
  const int npairs = gridDim.x, nblk = gridDim.y;
  const long L = blockIdx.x + (long)gridDim.x * blockIdx.y;
  const long per_chunk = (long)kDispatchChunk * nblk;
  const int chunk = (int)(L / per_chunk);
  const int c0 = chunk * kDispatchChunk;
  const int cn = min(kDispatchChunk, npairs - c0);
  const int r = (int)(L - chunk * per_chunk);
  rank = r / cn;
  pair = c0 + (r - rank * cn);
}

// LDS image of a [rows][64] bf16 tile: 128-byte rows of eight 16-byte chunks, chunk index
// XOR-swizzled by g((row >> 1) & 7) with g(k) = ((k & 1) << 2) | (k >> 1).
//  * row reads (ds_read_b128; 16 lanes = 16 distinct rows mod 16, one chunk): slot
//    (row & 1) * 8 + (ch ^ g) is a bijection over those rows -> conflict free;
//  * transposed reads (ds_read_b64_tr_b16; rows r0..r0+3, r0 % 4 == 0, four aligned chunks):
//    g(2m) ^ g(2m + 1) == 4 moves rows r0+2/r0+3 to the other half of the 256-byte bank row
//    -> conflict free.
__device__ __forceinline__ int swz(int row, int ch) {
  const int k = (row >> 1) & 7;
  return ch ^ (((k & 1) << 2) | (k >> 1));
}
__device__ __forceinline__ int tile_chunk_off(int row, int ch) { return row * kHD + (swz(row, ch) << 3); }
__device__ __forceinline__ int tile_elem_off(int row, int col) {
  return row * kHD + (swz(row, col >> 3) << 3) + (col & 7);
}

// raw 16-byte / 4-byte buffer loads: offsets past the descriptor's record count read as zero
__device__ __forceinline__ ushort8_t buf_load16(__amdgpu_buffer_rsrc_t r, int byte_off) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
  return __builtin_bit_cast(ushort8_t, v);
}
__device__ __forceinline__ float buf_load_f32(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}

// 8 contiguous bf16 of one row (an MFMA A/B fragment with k along the row)
__device__ __forceinline__ bf16x8 lds_row_read(const bf16_raw* tile, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(tile + tile_chunk_off(row, ch));
}

__device__ __forceinline__ short4v tr_read(const bf16_raw* tile, int row, int col) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(tile + tile_elem_off(row, col)));
}

// 32x32x16 MFMA operand whose k index runs DOWN the tile's rows (e.g. V^T with k = key):
// lane l gets column (dcol_base + (l & 31)) and rows row_base + {0..3} (elements 0..3) and
// row_base + 8 + {0..3} (elements 4..7) — the k order of an accumulator used as the other
// operand ("element j of lane half h is row 16s + 8(j>>2) + 4h + (j&3)"); callers fold the
// 16s + 4h part into row_base.
__device__ __forceinline__ bf16x8 lds_tr_read_operand(const bf16_raw* tile, int row_base, int dcol_base, int lane) {
  const int i = lane & 15;
  const int col = dcol_base + 16 * ((lane >> 4) & 1) + 4 * (i & 3);
  const short4v lo = tr_read(tile, row_base + (i >> 2), col);
  const short4v hi = tr_read(tile, row_base + 8 + (i >> 2), col);
  typedef short short8v __attribute__((ext_vector_type(8)));
  const short8v all = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, all);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Join the two 32-lane halves of a wave (the two key halves of a swapped-S^T row): one
// v_permlane32_swap (gfx950) instead of the ds_bpermute + address arithmetic + lgkmcnt(0) wait that
// __shfl_xor(x, 32) compiles to.  With x in both operands the swap leaves {x[l], x[l ^ 32]} in every
// lane l (in some order), so max / sum of the pair is the reduction over both halves.
__device__ __forceinline__ float halves_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halves_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// row (within a 32x32 accumulator tile) held in register r by lane half `half`
__device__ __forceinline__ int acc_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// registers 8*st .. 8*st+7 of an accumulator -> bf16 fragment for k-step st
__device__ __forceinline__ bf16x8 pack_acc8(const f32x16& acc, int st) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = static_cast<__bf16>(acc[8 * st + j]);
  return v;
}

}  // namespace attn
}  // namespace llmt
