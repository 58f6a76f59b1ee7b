// Split-K paged decode attention with GQA on gfx950 MFMA.
//
// One query token per sequence; the G = Hq/Hkv query heads that share a KV head are the
// 16 columns (G <= 16 used) of a v_mfma_f32_16x16x32_bf16 tile, so one K/V read serves the
// whole GQA group:
//   scores  S[t][h]   = K[t][:] . Q[h][:]          A = K   (16 tokens x 32 dims per MFMA)
//   output  O^T[d][h] = sum_t V^T[d][t] P^T[t][h]  A = V^T (16 dims  x 32 tokens per MFMA)
// The KV-cache layouts of rope_cache.hip make every A-operand load of a wave contiguous:
// K loads are 1 KiB per wave-instruction, V loads 512 B.  P never leaves registers: the
// score accumulator of two 16-token blocks is, element for element, the B operand of the
// PV product (token order inside the k-step is permuted identically on both operands).
//
// Grid = (partitions of 256 tokens, Hkv, batch); 4 waves x 64 tokens per workgroup.  Each
// workgroup writes an un-normalised partial (max, sum, O) that paged_decode_reduce merges.
// Everything is static-shaped so the decode step can be captured in a hipGraph: the
// partition count comes from the engine's max_model_len and idle partitions exit at once.
#include "common.h"

namespace k8sllm {

constexpr int kBS = 16;   // tokens per KV-cache block
constexpr int kPT = 256;  // tokens per partition (workgroup)

__device__ __forceinline__ bf16x8 zero_bf16x8() { return __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0)); }

template <int D, int G>
__global__ __launch_bounds__(256) void paged_decode_kernel(float* __restrict__ part_out,  // [B][Hq][NP][D]
                                                           float* __restrict__ part_ml,   // [B][Hq][NP][2]
                                                           const bf16_t* __restrict__ q, long q_stride,
                                                           const bf16_t* __restrict__ k_cache,
                                                           const bf16_t* __restrict__ v_cache,
                                                           const int* __restrict__ block_tables, int bt_stride,
                                                           const int* __restrict__ seq_lens, int Hq, int Hkv, int NP,
                                                           float scale_log2) {
  constexpr int KS = D / 32;  // QK k-steps
  constexpr int DT = D / 16;  // PV output tiles (16 dims each)
  __shared__ float s_max[4][16];
  __shared__ float s_sum[4][16];
  __shared__ float s_o[4][G][D];

  const int part = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int seq_len = seq_lens[b];
  const int tok0 = part * kPT;
  if (tok0 >= seq_len) return;  // uniform over the workgroup: no barrier is skipped unevenly
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = lane & 15, kg = lane >> 4;
  const int wtok0 = tok0 + wave * 64;
  const int* bt = block_tables + (long)b * bt_stride;

  bf16x8 qf[KS];
  if (col < G) {
    const bf16_t* qp = q + (long)b * q_stride + (long)(kvh * G + col) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qp + 32 * s + 8 * kg);
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = zero_bf16x8();
  }

  int phys[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) phys[i] = (wtok0 + 16 * i < seq_len) ? bt[(wtok0 >> 4) + i] : -1;

  const long head_block = (long)D * kBS;  // elements of one (block, head) tile
  f32x4 sacc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (phys[i] >= 0) {
      const bf16_t* kb = k_cache + ((long)phys[i] * Hkv + kvh) * head_block;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(kb + ((4 * s + kg) * kBS + col) * 8);
        sacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[s], sacc[i], 0, 0, 0);
      }
    }
  }

  // scale + mask; sacc[i][r] = S[token 4*kg + r of block i][head col]
  float mx = -1e30f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = wtok0 + 16 * i + 4 * kg + r;
      const float v = (t < seq_len) ? sacc[i][r] * scale_log2 : -1e30f;
      sacc[i][r] = v;
      mx = fmaxf(mx, v);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  if (lane < 16) s_max[wave][lane] = mx;
  __syncthreads();
  const float M = fmaxf(fmaxf(s_max[0][col], s_max[1][col]), fmaxf(s_max[2][col], s_max[3][col]));

  float ls = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = exp2f(sacc[i][r] - M);
      sacc[i][r] = p;
      ls += p;
    }
  ls += __shfl_xor(ls, 16, 64);
  ls += __shfl_xor(ls, 32, 64);
  if (lane < 16) s_sum[wave][lane] = ls;

  f32x4 oacc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) oacc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (phys[2 * s] < 0) continue;  // wave-uniform
    bf16x8 pb;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pb[j] = (__bf16)sacc[2 * s][j];
      pb[4 + j] = (__bf16)sacc[2 * s + 1][j];
    }
    const bf16_t* va = v_cache + ((long)phys[2 * s] * Hkv + kvh) * head_block + 4 * kg;
    const bool has_b = phys[2 * s + 1] >= 0;
    const bf16_t* vb = v_cache + ((long)(has_b ? phys[2 * s + 1] : 0) * Hkv + kvh) * head_block + 4 * kg;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int d = 16 * dt + col;
      const uint2 lo = *reinterpret_cast<const uint2*>(va + d * kBS);
      const uint2 hi = has_b ? *reinterpret_cast<const uint2*>(vb + d * kBS) : make_uint2(0, 0);
      const bf16x8 a = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      oacc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb, oacc[dt], 0, 0, 0);
    }
  }
  // oacc[dt][r] = O^T[d = 16*dt + 4*kg + r][head col]
  if (col < G) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_o[wave][col][16 * dt + 4 * kg + r] = oacc[dt][r];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += 256) {
    const int h = i / D, d = i - h * D;
    const float o = s_o[0][h][d] + s_o[1][h][d] + s_o[2][h][d] + s_o[3][h][d];
    const long ph = ((long)b * Hq + kvh * G + h) * NP + part;
    part_out[ph * D + d] = o;
    if (d == 0) {
      part_ml[ph * 2] = fmaxf(fmaxf(s_max[0][h], s_max[1][h]), fmaxf(s_max[2][h], s_max[3][h]));
      part_ml[ph * 2 + 1] = s_sum[0][h] + s_sum[1][h] + s_sum[2][h] + s_sum[3][h];
    }
  }
}

template <int D>
__global__ __launch_bounds__(D) void paged_decode_reduce_kernel(bf16_t* __restrict__ out, long out_stride,
                                                                const float* __restrict__ part_out,
                                                                const float* __restrict__ part_ml,
                                                                const int* __restrict__ seq_lens, int Hq, int NP) {
  const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int seq_len = seq_lens[b];
  const int n = (seq_len + kPT - 1) / kPT;
  bf16_t* o = out + (long)b * out_stride + (long)h * D + d;
  if (n <= 0) {
    *o = 0;
    return;
  }
  const long ph = ((long)b * Hq + h) * NP;
  float M = -1e30f;
  for (int p = 0; p < n; ++p) M = fmaxf(M, part_ml[(ph + p) * 2]);
  float acc = 0.f, L = 0.f;
  for (int p = 0; p < n; ++p) {
    const float w = exp2f(part_ml[(ph + p) * 2] - M);
    L += w * part_ml[(ph + p) * 2 + 1];
    acc += w * part_out[(ph + p) * D + d];
  }
  *o = f2bf(acc / L);
}

}  // namespace k8sllm

using namespace k8sllm;

extern "C" int k8sllm_paged_decode(void* out, long out_stride, float* part_out, float* part_ml, const void* q,
                                   long q_stride, const void* k_cache, const void* v_cache, const int* block_tables,
                                   int bt_stride, const int* seq_lens, int B, int Hq, int Hkv, int D, int NP,
                                   float scale, hipStream_t s) {
  if (B <= 0) return 0;
  const int G = Hq / Hkv;
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid(NP, Hkv, B), blk(256);
#define K8S_DEC(DD, GG)                                                                                         \
  hipLaunchKernelGGL((paged_decode_kernel<DD, GG>), grid, blk, 0, s, part_out, part_ml, (const bf16_t*)q,       \
                     q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, seq_lens, \
                     Hq, Hkv, NP, sl2)
  if (D == 128) {
    switch (G) {
      case 1: K8S_DEC(128, 1); break;
      case 2: K8S_DEC(128, 2); break;
      case 4: K8S_DEC(128, 4); break;
      case 8: K8S_DEC(128, 8); break;
      case 16: K8S_DEC(128, 16); break;
      default: return -1;
    }
    hipLaunchKernelGGL((paged_decode_reduce_kernel<128>), dim3(Hq, B), dim3(128), 0, s, (bf16_t*)out, out_stride,
                       part_out, part_ml, seq_lens, Hq, NP);
  } else if (D == 64) {
    switch (G) {
      case 1: K8S_DEC(64, 1); break;
      case 2: K8S_DEC(64, 2); break;
      case 4: K8S_DEC(64, 4); break;
      case 8: K8S_DEC(64, 8); break;
      default: return -1;
    }
    hipLaunchKernelGGL((paged_decode_reduce_kernel<64>), dim3(Hq, B), dim3(64), 0, s, (bf16_t*)out, out_stride,
                       part_out, part_ml, seq_lens, Hq, NP);
  } else {
    return -1;
  }
#undef K8S_DEC
  return (int)hipGetLastError();
}
