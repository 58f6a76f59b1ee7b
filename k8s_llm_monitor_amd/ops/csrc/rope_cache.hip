// Rotary embedding (neox half-split pairs i, i+D/2) applied in place to the q and k
// sections of the fused QKV GEMM output, fused with the paged KV-cache write.
// SURVEY.md §2.12 K-2.
//
// KV-cache layouts (chosen for the decode kernel's MFMA operand loads, see paged_decode.hip):
//   key_cache   [num_blocks][Hkv][D/8][BS][8]   -> one 16-dim "piece" of all BS tokens is
//                                                   contiguous: a wave loads 1 KiB per instr.
//   value_cache [num_blocks][Hkv][D][BS]        -> V^T per block: 8 tokens of one dim are
//                                                   contiguous (MFMA A-operand of O^T = V^T P^T).
#include "common.h"

namespace k8sllm {

// Sum of the split-K slabs of the qkv projection (gemm_skinny EPI_SLAB) for N consecutive columns.
template <int N>
__device__ __forceinline__ void slab_sum(const float* __restrict__ p, long slab_stride, int S, float* out) {
#pragma unroll
  for (int j = 0; j < N; ++j) out[j] = 0.f;
#pragma unroll 4
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int j = 0; j < N; j += 4) {
      const float4 v = *reinterpret_cast<const float4*>(p + s * slab_stride + j);
      out[j] += v.x; out[j + 1] += v.y; out[j + 2] += v.z; out[j + 3] += v.w;
    }
  }
}

// grid = (T, ceil(items / 128)), 128 threads, one work item per thread.  Items: (Hq + Hkv) heads
// x D/8 "quads" of rotary pairs (each rotates 4 pairs = 8 B of the lower half and 8 B of the upper
// half), then Hkv heads x D/8 value chunks of 8 dims (16 B) that are only copied into the cache.
// SLAB: the qkv values are the sum of S fp32 split-K slabs partial[s][t][col] (the decode qkv
// projection's launch-boundary reduce); the reduced, rotated q/k are written back to the bf16 qkv
// row (the attention reads q from there).
template <int D, bool SLAB>
__global__ __launch_bounds__(128) void rope_cache_kernel(bf16_t* __restrict__ qkv, long qkv_stride,
                                                         const int* __restrict__ positions,
                                                         const float* __restrict__ cos_sin,  // [max_pos][D]: cos | sin
                                                         bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
                                                         const int* __restrict__ slot_mapping, int Hq, int Hkv,
                                                         int block_size, int apply_rope, const float* __restrict__ partial,
                                                         int S, int T) {
  constexpr int HALF = D / 2;
  constexpr int QPH = D / 8;  // items per head
  const int t = blockIdx.x;
  const int n_rope = (Hq + Hkv) * QPH;
  const int n_total = n_rope + Hkv * QPH;
  const int w = blockIdx.y * 128 + threadIdx.x;
  if (w >= n_total) return;
  const int slot = slot_mapping ? slot_mapping[t] : -1;
  const int blk = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? slot - blk * block_size : 0;
  bf16_t* row = qkv + (long)t * qkv_stride;
  const int ncols = (Hq + 2 * Hkv) * D;
  const float* prow = SLAB ? partial + (long)t * ncols : nullptr;
  const long slab_stride = (long)T * ncols;
  if (w < n_rope) {
    const int head = w / QPH;
    const int p = (w - head * QPH) * 4;  // first of 4 pairs, p in [0, HALF)
    bf16_t* hp = row + head * D;
    float x1[4], x2[4];
    if constexpr (SLAB) {
      slab_sum<4>(prow + head * D + p, slab_stride, S, x1);
      slab_sum<4>(prow + head * D + HALF + p, slab_stride, S, x2);
    } else {
      const uint2 a = *reinterpret_cast<const uint2*>(hp + p);
      const uint2 b = *reinterpret_cast<const uint2*>(hp + HALF + p);
      x1[0] = lo_bf(a.x); x1[1] = hi_bf(a.x); x1[2] = lo_bf(a.y); x1[3] = hi_bf(a.y);
      x2[0] = lo_bf(b.x); x2[1] = hi_bf(b.x); x2[2] = lo_bf(b.y); x2[3] = hi_bf(b.y);
    }
    if constexpr (SLAB) {  // round to bf16 first, as an unfused GEMM output would be
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x1[j] = bf2f(f2bf(x1[j]));
        x2[j] = bf2f(f2bf(x2[j]));
      }
    }
    if (apply_rope) {
      const float* cs = cos_sin + (long)positions[t] * D;
      const float4 c = *reinterpret_cast<const float4*>(cs + p);
      const float4 s = *reinterpret_cast<const float4*>(cs + HALF + p);
      const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float o1 = x1[j] * cc[j] - x2[j] * ss[j];
        const float o2 = x2[j] * cc[j] + x1[j] * ss[j];
        x1[j] = o1;
        x2[j] = o2;
      }
    }
    uint2 a, b;
    a.x = pack2(x1[0], x1[1]);
    a.y = pack2(x1[2], x1[3]);
    b.x = pack2(x2[0], x2[1]);
    b.y = pack2(x2[2], x2[3]);
    *reinterpret_cast<uint2*>(hp + p) = a;
    *reinterpret_cast<uint2*>(hp + HALF + p) = b;
    if (head >= Hq && slot >= 0) {
      const int kh = head - Hq;
      bf16_t* kb = k_cache + ((long)blk * Hkv + kh) * (D * block_size);
      // dims p..p+3 live in piece p/8 at inner offset p%8 (4-aligned)
      *reinterpret_cast<uint2*>(kb + ((p >> 3) * block_size + off) * 8 + (p & 7)) = a;
      const int p2 = HALF + p;
      *reinterpret_cast<uint2*>(kb + ((p2 >> 3) * block_size + off) * 8 + (p2 & 7)) = b;
    }
  } else if (slot >= 0) {
    const int i = w - n_rope;
    const int vh = i / QPH;
    const int c = (i - vh * QPH) * 8;
    uint32_t wv[4];
    if constexpr (SLAB) {
      float f[8];
      slab_sum<8>(prow + (Hq + Hkv + vh) * D + c, slab_stride, S, f);
      const uint4 v = pack8(f);
      wv[0] = v.x; wv[1] = v.y; wv[2] = v.z; wv[3] = v.w;
    } else {
      const uint4 v = *reinterpret_cast<const uint4*>(row + (Hq + Hkv + vh) * D + c);
      wv[0] = v.x; wv[1] = v.y; wv[2] = v.z; wv[3] = v.w;
    }
    bf16_t* vb = v_cache + ((long)blk * Hkv + vh) * (D * block_size) + v_perm(off);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      vb[(long)(c + 2 * j) * block_size] = (bf16_t)(wv[j] & 0xffff);
      vb[(long)(c + 2 * j + 1) * block_size] = (bf16_t)(wv[j] >> 16);
    }
  }
}

// Prefill KV-cache write (the non-SLAB path; rope_cache_kernel then only rotates q / k in place).
// A token-per-workgroup write scatters V badly: the V^T cache rows ([D][BS] per block) take one
// token's 128 dims as 128 two-byte stores 32 B apart, and the measured prefill chunk spent 2/3 of
// rope_and_cache there (tools/bench_rope_cache.py: 174 us with the cache write vs 57 us rope only,
// 16k tokens).  Here one workgroup owns the cache-block RUNS that start in its 16-token window (a run
// = consecutive tokens whose slots are consecutive inside one block: a sequence's new tokens,
// split at block boundaries), so it holds a whole block row of V at once: K goes out as 16-byte
// pieces, V as one 16-byte store per (dim, 8 tokens) when the run covers them (every interior
// block), two-byte stores only at a run's ragged ends.  grid = (ceil(T / 16), Hkv), 256 threads.
template <int D>
__global__ __launch_bounds__(256) void kv_cache_write_kernel(const bf16_t* __restrict__ qkv, long qkv_stride,
                                                             const int* __restrict__ slot_mapping,
                                                             bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
                                                             int Hq, int Hkv, int T) {
  constexpr int BS = 16;
  __shared__ int s_slot[33];  // slots of tokens t0 - 1 .. t0 + 31
  const int t0 = blockIdx.x * 16, h = blockIdx.y, tid = threadIdx.x;
  if (tid < 33) {
    const int t = t0 - 1 + tid;
    s_slot[tid] = (t >= 0 && t < T) ? slot_mapping[t] : -1;
  }
  __syncthreads();
  const long koff = (long)(Hq + h) * D, voff = (long)(Hq + Hkv + h) * D;
  for (int i = 0; i < 16 && t0 + i < T; ++i) {  // uniform: every thread reads the same LDS slots
    const int sl = s_slot[i + 1];
    if (sl < 0) continue;
    if (sl % BS != 0 && s_slot[i] == sl - 1) continue;  // not a run start: an earlier window owns it
    const int off0 = sl % BS;
    int len = 1;
    while (len < BS - off0 && i + 1 + len < 33 && s_slot[i + 1 + len] == sl + len) ++len;
    const long blk = sl / BS;
    const int ts = t0 + i;
    bf16_t* kb = k_cache + (blk * Hkv + h) * (long)(D * BS);  // [D/8][BS][8]
    for (int e = tid; e < (D / 8) * BS; e += 256) {
      const int c = e / BS, j = e % BS;
      if (j < len) {  // the cache is next read by a later step: non-temporal stores
        typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(*reinterpret_cast<const u32x4_t*>(qkv + (long)(ts + j) * qkv_stride + koff + c * 8),
                                    reinterpret_cast<u32x4_t*>(kb + ((long)c * BS + off0 + j) * 8));
      }
    }
    bf16_t* vb = v_cache + (blk * Hkv + h) * (long)(D * BS);  // [D][BS], tokens in v_perm order
    for (int e = tid; e < D * 2; e += 256) {
      const int d = e >> 1, o0 = (e & 1) * 8;  // block positions o0 .. o0 + 7 of dim d
      bf16_t v[8];
      int have = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int j = v_perm(o0 + q) - off0;  // token of this position, relative to the run
        const bool in = j >= 0 && j < len;
        have += in;
        v[q] = in ? qkv[(long)(ts + j) * qkv_stride + voff + d] : (bf16_t)0;
      }
      if (have == 0) continue;
      bf16_t* dst = vb + (long)d * BS + o0;
      if (have == 8) {
        typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
        u32x4_t w;
        w.x = (uint32_t)v[0] | ((uint32_t)v[1] << 16);
        w.y = (uint32_t)v[2] | ((uint32_t)v[3] << 16);
        w.z = (uint32_t)v[4] | ((uint32_t)v[5] << 16);
        w.w = (uint32_t)v[6] | ((uint32_t)v[7] << 16);
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(dst));
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int j = v_perm(o0 + q) - off0;
          if (j >= 0 && j < len) dst[q] = v[q];
        }
      }
    }
  }
}

}  // namespace k8sllm

using namespace k8sllm;

extern "C" int k8sllm_rope_cache(void* qkv, long qkv_stride, const int* positions, const float* cos_sin, void* k_cache,
                                 void* v_cache, const int* slot_mapping, long T, int Hq, int Hkv, int D,
                                 int block_size, int apply_rope, const float* partial, int S, hipStream_t s) {
  if (T <= 0) return 0;
  if (D != 128 && D != 64) return -1;
  // prefill (no slabs, 16-token blocks): rotate in place, then write the cache block-run-wise
  const bool runs = partial == nullptr && slot_mapping != nullptr && block_size == 16;
  const int* rope_slots = runs ? nullptr : slot_mapping;
  const int items = (Hq + (runs ? 1 : 2) * Hkv) * (D / 8);
  dim3 grid((unsigned)T, (items + 127) / 128);
  // nothing to rotate (q / k rotated by the qkv GEMM epilogue, or a model without RoPE) and the
  // cache written run-wise below: the in-place pass would only copy q / k onto themselves
  const bool skip_rope = runs && !apply_rope;
#define K8S_ROPE(DV, SL)                                                                                       \
  hipLaunchKernelGGL((rope_cache_kernel<DV, SL>), grid, dim3(128), 0, s, (bf16_t*)qkv, qkv_stride, positions,  \
                     cos_sin, (bf16_t*)k_cache, (bf16_t*)v_cache, rope_slots, Hq, Hkv, block_size, apply_rope,   \
                     partial, S, (int)T)
  if (skip_rope) {
  } else if (D == 128) {
    if (partial) K8S_ROPE(128, true); else K8S_ROPE(128, false);
  } else if (D == 64) {
    if (partial) K8S_ROPE(64, true); else K8S_ROPE(64, false);
  } else {
    return -1;
  }
#undef K8S_ROPE
  if (runs) {
    dim3 g2((unsigned)((T + 15) / 16), Hkv);
    if (D == 128)
      hipLaunchKernelGGL((kv_cache_write_kernel<128>), g2, dim3(256), 0, s, (const bf16_t*)qkv, qkv_stride,
                         slot_mapping, (bf16_t*)k_cache, (bf16_t*)v_cache, Hq, Hkv, (int)T);
    else
      hipLaunchKernelGGL((kv_cache_write_kernel<64>), g2, dim3(256), 0, s, (const bf16_t*)qkv, qkv_stride,
                         slot_mapping, (bf16_t*)k_cache, (bf16_t*)v_cache, Hq, Hkv, (int)T);
  }
  return (int)hipGetLastError();
}
