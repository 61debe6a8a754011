// Building blocks shared by the gfx950 MFMA GEMM kernels (gemm_wgrad_pp.hip, gemm_fused.hip):
// LDS-DMA staging (`buffer_load_dwordx4 ... lds`), counted vmcnt + raw barrier stage waits,
// XOR-swizzled LDS images and the fragment readers for v_mfma_f32_32x32x16_bf16.
#pragma once

#include "common.h"

namespace llmt {
namespace gemm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4;
typedef __attribute__((address_space(3))) void lds_void;

// Element offset in a [rows][W] bf16 LDS image whose 16-byte chunks are XOR-swizzled by
// 4*(row & 3): the 4 rows of one transposed read then land on distinct 64-byte bank groups.
template <int W>
__device__ __forceinline__ int swz_off(int row, int col) {
  return row * W + ((((col >> 3) ^ ((row & 3) << 2))) << 3) + (col & 7);
}

// 32x32x16 operand read from a [k rows][W cols] image with k running DOWN the rows
// (ds_read_b64_tr_b16): lane l -> column col0 + (l & 31), elements j = 0..7 -> rows
// row0 + 8*(l >> 5) + j.
template <int W>
__device__ __forceinline__ bf16x8 tr_frag(const bf16_raw* tile, int row0, int col0, int lane) {
  const int i = lane & 15;
  const int row = row0 + 8 * (lane >> 5) + (i >> 2);
  const int col = col0 + 16 * ((lane >> 4) & 1) + 4 * (i & 3);
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(tile + swz_off<W>(row, col)));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(tile + swz_off<W>(row + 4, col)));
  const short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// "stage s landed for this wave" (n later stages, P DMA ops each, may stay in flight) followed
// by the workgroup barrier, in ONE asm statement with a memory clobber so no LDS read can be
// scheduled between the wait and the barrier.
template <int P>
__device__ __forceinline__ void wait_stage_and_barrier(int n) {
  if (n >= 2) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * P) : "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(P) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
}

// one 1-KiB LDS-DMA op: M0 (the LDS destination base) is saved/restored inside the statement
__device__ __forceinline__ void dma16(unsigned lds_dst, int voff, __amdgpu_buffer_rsrc_t rsrc, int soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %[keep], m0\n\t"
      "s_nop 4\n\t"
      "s_mov_b32 m0, %[dst]\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[v], %[r], %[so] offen lds\n\t"
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [dst] "s"(lds_dst), [v] "v"(voff), [r] "s"(rsrc), [so] "s"(soff)
      : "memory");
}

// Bijective XCD-aware remap of a workgroup id: the 1/8 of the grid the dispatcher sends to one
// XCD (ids with equal L & 7) gets a contiguous range of work ids, so they share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int L, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = L & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
}

inline int cu_count() { return device_cu_count(); }

}  // namespace gemm
}  // namespace llmt
