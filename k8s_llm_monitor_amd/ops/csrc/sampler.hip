// Token sampler over logits[B][V]: one 1024-thread workgroup per row.
//   temperature <= 0        -> greedy argmax (first index on ties, like torch.argmax)
//   temperature  > 0        -> Gumbel-max over logits/T  (exact sample from softmax(logits/T))
//   top_k > 0 / top_p < 1   -> the kept set {x >= thr} is found by bisection on the threshold
//                              (count for top-k, probability mass for top-p); no sort needed.
// Randomness is a counter hash of (seed, offset, row, index); `rng` lives in device memory so a
// hipGraph-captured decode step draws fresh numbers on every replay (the engine bumps offset).
#include "common.h"

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

__device__ __forceinline__ float gumbel(uint64_t seed, uint64_t off, int row, int i) {
  const uint64_t h = mix64(seed ^ mix64(off * 0x100000001b3ull + (uint64_t)row * 0x9e3779b97ull + (uint64_t)i));
  const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
  return -__logf(-__logf(u));
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

template <typename T>
__global__ __launch_bounds__(kST) void sample_kernel(int* __restrict__ out, const T* __restrict__ logits, long stride,
                                                     int V, const float* __restrict__ temps,
                                                     const int* __restrict__ top_k, const float* __restrict__ top_p,
                                                     const int64_t* __restrict__ rng) {
  __shared__ float sv[kST / 64];
  __shared__ int si[kST / 64];
  const int row = blockIdx.x;
  const T* x = logits + (long)row * stride;
  const float temp = temps ? temps[row] : 0.f;
  const int tid = threadIdx.x;

  if (!(temp > 0.f)) {
    ArgMax a{-INFINITY, 0x7fffffff};
    for (int i = tid; i < V; i += kST) a = better(a, ArgMax{ld<T>(x, i), i});
    a = block_argmax(a, sv, si);
    if (tid == 0) out[row] = a.i;
    return;
  }

  const float itemp = 1.f / temp;
  const int k = top_k ? top_k[row] : 0;
  const float p = top_p ? top_p[row] : 1.f;
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
  const uint64_t seed = rng ? (uint64_t)rng[0] : 0ull;
  const uint64_t off = rng ? (uint64_t)rng[1] : 0ull;
  ArgMax a{-INFINITY, 0x7fffffff};
  for (int i = tid; i < V; i += kST) {
    const float v = ld<T>(x, i) * itemp;
    if (v >= thr) a = better(a, ArgMax{v + gumbel(seed, off, row, i), i});
  }
  a = block_argmax(a, sv, si);
  if (tid == 0) out[row] = a.i;
}

}  // namespace k8sllm

using namespace k8sllm;

extern "C" int k8sllm_sample(int* out, const void* logits, int is_fp32, long B, long stride, int V,
                             const float* temps, const int* top_k, const float* top_p, const int64_t* rng,
                             hipStream_t s) {
  if (B <= 0) return 0;
  if (is_fp32)
    hipLaunchKernelGGL((sample_kernel<float>), dim3(B), dim3(kST), 0, s, out, (const float*)logits, stride, V, temps,
                       top_k, top_p, rng);
  else
    hipLaunchKernelGGL((sample_kernel<bf16_t>), dim3(B), dim3(kST), 0, s, out, (const bf16_t*)logits, stride, V,
                       temps, top_k, top_p, rng);
  return (int)hipGetLastError();
}
