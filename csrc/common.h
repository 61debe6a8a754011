// Shared device helpers for the llmtrain gfx950 (MI355X, CDNA4) kernels.
//
// Conventions: wave64 everywhere (CDNA wavefront = 64 lanes), bf16 held as raw 16-bit values
// in vector registers and converted with clang's native __bf16 type (hipcc emits
// v_cvt_pk_bf16_f32 for the f32->bf16 direction, round-to-nearest-even, NaN preserving), global
// memory moved in 16-byte vectors (Guideline 13: bf16 must never be loaded scalar).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"  // DropoutArgs

// Device-side bounds checks of the debug build (`python -m llmtrain.ops.build --debug`,
// -DLLMT_DEBUG=1): a failing check aborts the kernel with file/line instead of silently reading
// or writing out of bounds.  Compiled out of the release build.
#if defined(LLMT_DEBUG) && LLMT_DEBUG
#include <cassert>
#define LLMT_DASSERT(cond) assert(cond)
#else
#define LLMT_DASSERT(cond) ((void)0)
#endif

namespace llmt {

constexpr int kWave = 64;

typedef unsigned short bf16_raw;
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef float float2_t __attribute__((ext_vector_type(2)));
typedef unsigned short ushort8_t __attribute__((ext_vector_type(8)));
typedef unsigned short ushort4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

// compute units of the current device (queried once per process; every MI355X has 256) that grid
// sizing (persistent kernels, one-round plans) counts on
inline int device_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

__device__ __forceinline__ float bf2f(bf16_raw v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_raw f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(bf16_raw, b);
}

// one element / four consecutive elements of an fp32 or bf16 stream, as fp32
__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16_raw v) { return bf2f(v); }
__device__ __forceinline__ float4_t load4_f32(const float* p) { return *reinterpret_cast<const float4_t*>(p); }
__device__ __forceinline__ float4_t load4_f32(const bf16_raw* p) {
  const ushort4_t v = *reinterpret_cast<const ushort4_t*>(p);
  return float4_t{bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3])};
}

// 8 x bf16 <-> 8 x f32
__device__ __forceinline__ void unpack8(const ushort8_t v, float* f) {
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf2f(v[i]);
}
__device__ __forceinline__ ushort8_t pack8(const float* f) {
  ushort8_t v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = f2bf(f[i]);
  return v;
}

// ---- dropout masks ----------------------------------------------------------------------
// Counter-based, so the backward regenerates the forward's mask instead of storing it.  Element e
// of a site keeps iff its 16-bit uniform, half of h = mix32((e >> 1) ^ seed ^ hi * 0x85ebca6b)
// (low half for even e, high half for odd e), is >= thr = round(p * 65536).  `seed` is already
// mixed with the step seed and the site id on the host.  Bit-identical to
// llmtrain/ops/reference.py (dropout_keep), which the CPU engine and the tests use.
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {  // "lowbias32" finaliser
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t drop_hash(uint32_t seed, uint64_t pair) {
  return mix32((uint32_t)pair ^ seed ^ (uint32_t)(pair >> 32) * 0x85ebca6bu);
}

// per-step seed offset of a graph-replayed step (DropoutArgs::seed_add), applied once at kernel entry
__device__ __forceinline__ void resolve_dropout(DropoutArgs& d) {
  if (d.seed_add != nullptr) d.seed += *d.seed_add;
}

__device__ __forceinline__ bool drop_keep(uint32_t seed, uint32_t thr, uint64_t e) {
  const uint32_t h = drop_hash(seed, e >> 1);
  return ((e & 1) ? (h >> 16) : (h & 0xffffu)) >= thr;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// Block-wide sum for blockDim.x = 64 * NWAVES; `scratch` must hold NWAVES floats.
template <int NWAVES>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int w = 0; w < NWAVES; ++w) r += scratch[w];
  return r;
}

template <int NWAVES>
__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int w = 0; w < NWAVES; ++w) r = fmaxf(r, scratch[w]);
  return r;
}

// Number of workgroups for a grid-stride memory-bound kernel: enough to fill 256 CUs several
// times over without launching millions of tiny blocks (Guideline 11).
inline int stride_grid(long long work_items, int per_block, int cap = 256 * 8) {
  long long g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace llmt
