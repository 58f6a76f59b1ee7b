// Token sampler over logits[B][V].
//   temperature <= 0        -> greedy argmax (first index on ties, like torch.argmax)
//   temperature  > 0        -> Gumbel-max over logits/T  (exact sample from softmax(logits/T))
//   top_k > 0 / top_p < 1   -> the kept set {x >= thr} is found by bisection on the threshold
//                              (count for top-k, probability mass for top-p); no sort needed.
// Randomness is a counter hash of (seed, offset, row, index); `rng` lives in device memory so a
// hipGraph-captured decode step draws fresh numbers on every replay (the engine bumps offset).
//
// Decomposition: a decode batch has only B <= 64 rows, and Gumbel-max over a 128K vocabulary is
// VALU-bound (hash + two logs per element), so one workgroup per row used 64 of 256 CUs and took
// 125 us at B = 64.  Rows are split into P parts: grid (B, P) of 1024-thread workgroups each
// produce a partial (value, index) argmax, and a one-wave kernel picks the winner per row.  Rows
// with top-k / top-p need a row-wide threshold; part 0 of such a row runs the whole-row bisection
// path and its answer is taken as is.  The per-element hash is 32-bit (two murmur3 finalisers of
// a per-row 64-bit key) - 64-bit multiplies are multi-instruction sequences on CDNA.
#include <type_traits>

#include "common.h"
#include <stdlib.h>

namespace k8sllm {

constexpr int kST = 1024;

template <typename T>
__device__ __forceinline__ float ld(const T* p, long i);
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, long i) { return bf2f(p[i]); }
template <>
__device__ __forceinline__ float ld<float>(const float* p, long i) { return p[i]; }

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint64_t row_key(const int64_t* rng, int row) {
  const uint64_t seed = rng ? (uint64_t)rng[0] : 0ull;
  const uint64_t off = rng ? (uint64_t)rng[1] : 0ull;
  return mix64(seed ^ mix64(off * 0x100000001b3ull + (uint64_t)row * 0x9e3779b97ull));
}

// Standard Gumbel noise -log(-log(u)).  u is drawn as 1 - w with w = (23-bit hash + 0.5) / 2^23,
// so w lies in [2^-24, 1 - 2^-24] and -log(u) = -log(1 - w) is taken by its series for small w:
// accurate and > 0 as u -> 1.
// (The earlier 24-bit u = (h + 0.5) / 2^24 rounded to exactly 1.0f for the top hash value, and the
// fast log of 1 is 0: a +inf noise that made an arbitrary token win - about once per two 64-row
// steps of a 128K vocabulary.)  Range: [-log(16.64), 16.64] = [-2.81, 16.64].
__device__ __forceinline__ float gumbel(uint64_t key, int i) {
  const uint32_t h = fmix32(fmix32((uint32_t)i * 0x9e3779b9u ^ (uint32_t)key) + (uint32_t)(key >> 32));
  const float w = ((float)(h >> 9) + 0.5f) * (1.0f / 8388608.0f);
  // -log(1 - w): the series w + w^2 / 2 below 2^-10 (relative error < 4e-7), the fast log above
  const float e = w < 0x1p-10f ? __builtin_fmaf(0.5f * w, w, w) : -__logf(1.f - w);
  return -__logf(e);
}

struct ArgMax {
  float v;
  int i;
};

__device__ __forceinline__ ArgMax better(ArgMax a, ArgMax b) {
  return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}

__device__ __forceinline__ ArgMax block_argmax(ArgMax a, float* sv, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = better(a, b);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[w] = a.v;
    si[w] = a.i;
  }
  __syncthreads();
  ArgMax r{sv[0], si[0]};
#pragma unroll
  for (int k = 1; k < kST / 64; ++k) r = better(r, ArgMax{sv[k], si[k]});
  __syncthreads();
  return r;
}

// Whole-row path for rows with top-k / top-p (one workgroup); returns the token on every thread.
template <typename T>
__device__ int sample_row_filtered(const T* __restrict__ x, int V, float temp, int k, float p, uint64_t key,
                                   float* sv, int* si) {
  const int tid = threadIdx.x;
  const float itemp = 1.f / temp;
  float mx = -INFINITY, mn = INFINITY;
  for (int i = tid; i < V; i += kST) {
    const float v = ld<T>(x, i) * itemp;
    mx = fmaxf(mx, v);
    mn = fminf(mn, v);
  }
  mx = block_max<kST>(mx, sv);
  mn = -block_max<kST>(-mn, sv);
  float thr = -INFINITY;
  if (k > 0 && k < V) {
    float lo = mn, hi = mx;  // invariant: count(x >= lo) >= k
    for (int it = 0; it < 26; ++it) {
      const float mid = 0.5f * (lo + hi);
      float c = 0.f;
      for (int i = tid; i < V; i += kST) c += (ld<T>(x, i) * itemp >= mid) ? 1.f : 0.f;
      c = block_sum<kST>(c, sv);
      if (c >= (float)k) lo = mid; else hi = mid;
    }
    thr = lo;
  }
  if (p < 1.f) {
    float z = 0.f;
    for (int i = tid; i < V; i += kST) z += __expf(ld<T>(x, i) * itemp - mx);
    z = block_sum<kST>(z, sv);
    const float target = p * z;
    float lo = fmaxf(mn, mx - 80.f), hi = mx;  // invariant: mass(x >= lo) >= target
    for (int it = 0; it < 26; ++it) {
      const float mid = 0.5f * (lo + hi);
      float s = 0.f;
      for (int i = tid; i < V; i += kST) {
        const float v = ld<T>(x, i) * itemp;
        s += (v >= mid) ? __expf(v - mx) : 0.f;
      }
      s = block_sum<kST>(s, sv);
      if (s >= target) lo = mid; else hi = mid;
    }
    thr = fmaxf(thr, lo);
  }
  ArgMax a{-INFINITY, 0x7fffffff};
  for (int i = tid; i < V; i += kST) {
    const float v = ld<T>(x, i) * itemp;
    if (v >= thr) a = better(a, ArgMax{v + gumbel(key, i), i});
  }
  return block_argmax(a, sv, si).i;
}

__device__ __forceinline__ bool row_filtered(int V, float temp, int k, float p) {
  return temp > 0.f && ((k > 0 && k < V) || p < 1.f);
}

// grid (B, P): partial argmax of part `blockIdx.y` of row `blockIdx.x` -> pv/pi[row * P + part]
template <typename T>
__global__ __launch_bounds__(kST) void sample_partial_kernel(float* __restrict__ pv, int* __restrict__ pi,
                                                             const T* __restrict__ logits, long stride, int V, int P,
                                                             const float* __restrict__ temps,
                                                             const int* __restrict__ top_k,
                                                             const float* __restrict__ top_p,
                                                             const int64_t* __restrict__ rng) {
  __shared__ float sv[kST / 64];
  __shared__ int si[kST / 64];
  const int row = blockIdx.x, part = blockIdx.y, tid = threadIdx.x;
  const T* x = logits + (long)row * stride;
  const float temp = temps ? temps[row] : 0.f;
  const int k = top_k ? top_k[row] : 0;
  const float p = top_p ? top_p[row] : 1.f;
  if (row_filtered(V, temp, k, p)) {
    if (part != 0) return;
    const int tok = sample_row_filtered<T>(x, V, temp, k, p, row_key(rng, row), sv, si);
    if (tid == 0) pi[row * P] = tok;
    return;
  }
  // parts start on 8-element boundaries so that bf16 rows with an 8-aligned stride are read 16 B
  // per lane (one load per 8 logits instead of eight dependent 2-byte loads)
  const int chunk = ((V + P - 1) / P + 7) & ~7;
  const int lo = min(V, part * chunk), hi = min(V, lo + chunk);
  const bool vec = std::is_same<T, bf16_t>::value && (stride & 7) == 0;
  const int hv = vec ? lo + ((hi - lo) & ~7) : lo;  // [lo, hv) in 8-element vectors, [hv, hi) scalar
  ArgMax a{-INFINITY, 0x7fffffff};
  const bool greedy = !(temp > 0.f);
  const float itemp = greedy ? 1.f : 1.f / temp;
  const uint64_t key = greedy ? 0ull : row_key(rng, row);
  if constexpr (std::is_same<T, bf16_t>::value) {
    for (int i = lo + tid * 8; i < hv; i += kST * 8) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(x + i), v);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        a = better(a, ArgMax{greedy ? v[j] : v[j] * itemp + gumbel(key, i + j), i + j});
    }
  }
  for (int i = hv + tid; i < hi; i += kST)
    a = better(a, ArgMax{greedy ? ld<T>(x, i) : ld<T>(x, i) * itemp + gumbel(key, i), i});
  a = block_argmax(a, sv, si);
  if (tid == 0) {
    pv[row * P + part] = a.v;
    pi[row * P + part] = a.i;
  }
}

// one thread per row: the best of the P partials (or part 0's answer for a filtered row)
__global__ __launch_bounds__(64) void sample_final_kernel(int* __restrict__ out, const float* __restrict__ pv,
                                                          const int* __restrict__ pi, int B, int V, int P,
                                                          const float* __restrict__ temps,
                                                          const int* __restrict__ top_k,
                                                          const float* __restrict__ top_p,
                                                          int64_t* __restrict__ rng_advance) {
  const int row = blockIdx.x * 64 + threadIdx.x;
  // the partial kernel has drawn this step's numbers: advance the counter for the next step here
  // (one lane, a vector store) instead of a separate `rng[1] += 1` launch after every sample
  if (rng_advance != nullptr && row == 0) rng_advance[1] = rng_advance[1] + 1;
  if (row >= B) return;
  const float temp = temps ? temps[row] : 0.f;
  const int k = top_k ? top_k[row] : 0;
  const float p = top_p ? top_p[row] : 1.f;
  if (row_filtered(V, temp, k, p)) {
    out[row] = pi[row * P];
    return;
  }
  ArgMax a{pv[row * P], pi[row * P]};
  for (int j = 1; j < P; ++j) a = better(a, ArgMax{pv[row * P + j], pi[row * P + j]});
  out[row] = a.i;
}

}  // namespace k8sllm

using namespace k8sllm;

extern "C" int k8sllm_sample_parts(long B, int V) {
  // ~2 workgroups per CU in total, at least 8K vocabulary entries per part
  long p = (512 + B - 1) / B;
  p = p < 1 ? 1 : p;
  const long pmax = V / 8192 > 1 ? V / 8192 : 1;
  return (int)(p < pmax ? p : pmax);
}

// pv/pi: workspace of at least B * k8sllm_sample_parts(B, V) entries
extern "C" int k8sllm_sample(int* out, const void* logits, int is_fp32, long B, long stride, int V,
                             const float* temps, const int* top_k, const float* top_p, const int64_t* rng,
                             float* pv, int* pi, int advance, hipStream_t s) {
  if (B <= 0) return 0;
  const int P = k8sllm_sample_parts(B, V);
  dim3 grid((unsigned)B, P);
  if (is_fp32)
    hipLaunchKernelGGL((sample_partial_kernel<float>), grid, dim3(kST), 0, s, pv, pi, (const float*)logits, stride,
                       V, P, temps, top_k, top_p, rng);
  else
    hipLaunchKernelGGL((sample_partial_kernel<bf16_t>), grid, dim3(kST), 0, s, pv, pi, (const bf16_t*)logits,
                       stride, V, P, temps, top_k, top_p, rng);
  hipLaunchKernelGGL(sample_final_kernel, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, s, out, pv, pi, (int)B, V, P,
                     temps, top_k, top_p, advance && rng ? const_cast<int64_t*>(rng) : nullptr);
  return (int)hipGetLastError();
}
