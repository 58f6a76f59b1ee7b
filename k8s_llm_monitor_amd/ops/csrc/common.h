// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of k8s-llm-monitor-amd.
//
// Everything here is written for 64-lane wavefronts and the gfx950 MFMA/LDS model:
//  * bf16 is carried as raw 16-bit patterns and widened with a shift (one VALU op),
//    narrowed with the hardware v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN-safe).
//  * global traffic is issued as 16-byte (dwordx4) or 8-byte vectors, never scalar bf16.
//  * reductions are wave64 butterflies followed by one LDS exchange per workgroup.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace k8sllm {

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

// low half of a dword holds the first element (little endian)
__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// unpack 8 bf16 held in a uint4 into floats
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = lo_bf(v.x); f[1] = hi_bf(v.x);
  f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
  f[4] = lo_bf(v.z); f[5] = hi_bf(v.z);
  f[6] = lo_bf(v.w); f[7] = hi_bf(v.w);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2(f[0], f[1]);
  v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]);
  v.w = pack2(f[6], f[7]);
  return v;
}

// Element (row, col) of an activation matrix: row-major [rows][stride] when stride > 0, or the
// fragment-packed [ceil(rows/16)][K/32][64][8] layout of gemm_skinny's A operand when
// stride == -(K/32) (lane = 16 * ((col / 8) % 4) + row % 16; 8 consecutive cols are contiguous).
__device__ __forceinline__ long act_index(int row, int col, long stride) {
  if (stride > 0) return (long)row * stride + col;
  return (((long)(row >> 4) * (-stride) + (col >> 5)) * 64 + ((col >> 3) & 3) * 16 + (row & 15)) * 8 + (col & 7);
}

// V-cache token order inside each 16-token block (v_cache [NB][Hkv][D][BS], a dim's 16 tokens
// in 32 contiguous bytes): token t sits at position v_perm(t), an involution that swaps bits 2
// and 3 - tokens 0-3, 8-11 fill the first 16-byte chunk of a dim row, 4-7, 12-15 the second.  That
// is exactly the k order of a v_mfma_f32_32x32x16_bf16 operand that sums over the row index of a
// 32x32 accumulator (lane half h, element j <-> row 8(j>>2) + 4h + (j&3); cdna_hip_programming.md
// §3): flash prefill's PV A-fragment is one ds_read_b128 of a cache block staged verbatim by
// LDS-DMA.  Paged decode reads 4-token groups, which v_perm keeps contiguous.
__device__ __forceinline__ int v_perm(int t) { return (t & ~12) | ((t & 4) << 1) | ((t & 8) >> 1); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Workgroup sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

}  // namespace k8sllm
