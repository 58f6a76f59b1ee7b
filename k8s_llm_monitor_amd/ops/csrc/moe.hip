// Mixture-of-experts plumbing for the Mixtral family:
//   moe_route   softmax over E router logits, top-K, optional renormalisation (one lane per token)
//   moe_align   deterministic counting sort of the T*K (token, slot) pairs by expert, producing
//               expert_offsets[E+1], sorted_idx (position -> flat pair) and inv_idx (pair -> position)
//   gather_rows out[j] = x[idx[j] / div]          (token rows into expert-sorted order)
//   moe_combine out[t] = sum_k w[t][k] * y[inv_idx[t*K + k]]   (fp32 accumulate)
#include "common.h"

namespace k8sllm {

__global__ __launch_bounds__(256) void moe_route_kernel(const float* __restrict__ logits, long T, int E, int K,
                                                        int renorm, int* __restrict__ ids, float* __restrict__ w) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  const float* x = logits + t * E;
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) mx = fmaxf(mx, x[e]);
  float z = 0.f;
  for (int e = 0; e < E; ++e) z += __expf(x[e] - mx);
  uint64_t taken = 0ull;
  float sel = 0.f;
  for (int k = 0; k < K; ++k) {
    int best = -1;
    float bv = -INFINITY;
    for (int e = 0; e < E; ++e)
      if (!((taken >> e) & 1ull) && x[e] > bv) {
        bv = x[e];
        best = e;
      }
    taken |= 1ull << best;
    const float p = __expf(bv - mx) / z;
    ids[t * K + k] = best;
    w[t * K + k] = p;
    sel += p;
  }
  if (renorm)
    for (int k = 0; k < K; ++k) w[t * K + k] /= sel;
}

// MoE decode router in one launch (one workgroup per row): logits = bf16(x . W_router^T) (as the
// library GEMM's bf16 output would be), softmax top-k (+ renormalisation) as moe_route_kernel, and
// the dense per-expert weight row wd[t][e] (0 for an expert the row did not choose) that the grouped
// expert kernels scale their slabs by.  Replaces GEMM + fp32 cast + route + zeros + scatter.
template <int EMAX>
__global__ __launch_bounds__(256) void moe_router_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wr,
                                                         int d, int E, int K, int renorm, int* __restrict__ ids,
                                                         float* __restrict__ w, float* __restrict__ wd) {
  __shared__ float red[4][EMAX];
  const int t = blockIdx.x, tid = threadIdx.x;
  float acc[EMAX];
#pragma unroll
  for (int e = 0; e < EMAX; ++e) acc[e] = 0.f;
  const bf16_t* xr = x + (long)t * d;
  for (int c = tid * 8; c < d; c += 256 * 8) {
    float xv[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c), xv);
#pragma unroll
    for (int e = 0; e < EMAX; ++e) {
      if (e < E) {
        float wv[8];
        unpack8(*reinterpret_cast<const uint4*>(wr + (long)e * d + c), wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[e] = __builtin_fmaf(xv[j], wv[j], acc[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EMAX; ++e) {
    const float v = wave_sum(acc[e]);
    if ((tid & 63) == 0) red[tid >> 6][e] = v;
  }
  __syncthreads();
  if (tid != 0) return;
  float lg[EMAX];
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) {
    lg[e] = bf2f(f2bf((red[0][e] + red[1][e]) + (red[2][e] + red[3][e])));
    mx = fmaxf(mx, lg[e]);
  }
  float z = 0.f;
  for (int e = 0; e < E; ++e) z += __expf(lg[e] - mx);
  uint32_t taken = 0u;
  float sel = 0.f, pk[EMAX];
  int bk[EMAX];
  for (int k = 0; k < K; ++k) {
    int best = -1;
    float bv = -INFINITY;
    for (int e = 0; e < E; ++e)
      if (!((taken >> e) & 1u) && lg[e] > bv) {
        bv = lg[e];
        best = e;
      }
    if (best < 0) {  // NaN logits: no comparison holds - take the first untaken expert (a valid id)
      for (best = 0; (taken >> best) & 1u; ++best) {
      }
      bv = lg[best];
    }
    taken |= 1u << best;
    pk[k] = __expf(bv - mx) / z;
    bk[k] = best;
    sel += pk[k];
  }
  for (int e = 0; e < E; ++e) wd[(long)t * E + e] = 0.f;
  for (int k = 0; k < K; ++k) {
    const float p = renorm ? pk[k] / sel : pk[k];
    ids[(long)t * K + k] = bk[k];
    w[(long)t * K + k] = p;
    wd[(long)t * E + bk[k]] = p;
  }
}

constexpr int kAT = 1024;
constexpr int kMaxE = 16;

// exclusive scan of one value per thread over the 1024-thread workgroup
__device__ __forceinline__ int block_exscan(int v, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int pre = 0;
  total = 0;
#pragma unroll
  for (int i = 0; i < kAT / 64; ++i) {
    const int s = wsum[i];
    if (i < w) pre += s;
    total += s;
  }
  __syncthreads();
  return pre + x - v;
}

__global__ __launch_bounds__(kAT) void moe_align_kernel(const int* __restrict__ ids, long n, int E,
                                                        int* __restrict__ offsets, int* __restrict__ sorted_idx,
                                                        int* __restrict__ inv_idx) {
  __shared__ int cnt[kMaxE][kAT];
  __shared__ int wsum[kAT / 64];
  const int t = threadIdx.x;
  const long C = (n + kAT - 1) / kAT;
  const long b0 = t * C, b1 = min(n, b0 + C);
  for (int e = 0; e < E; ++e) cnt[e][t] = 0;
  for (long i = b0; i < b1; ++i) cnt[ids[i]][t] += 1;
  __syncthreads();
  int base = 0;
  for (int e = 0; e < E; ++e) {
    int tot;
    const int ex = block_exscan(cnt[e][t], wsum, tot);
    if (t == 0) offsets[e] = base;
    cnt[e][t] = base + ex;  // start position of this thread's items of expert e
    base += tot;
  }
  if (t == 0) offsets[E] = base;
  for (long i = b0; i < b1; ++i) {
    const int e = ids[i];
    const int pos = cnt[e][t]++;
    sorted_idx[pos] = (int)i;
    inv_idx[i] = pos;
  }
}

__global__ __launch_bounds__(256) void gather_rows_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                                                          const int* __restrict__ idx, int d, int div) {
  const long j = blockIdx.x;
  const long src = idx[j] / div;
  const uint4* s = reinterpret_cast<const uint4*>(x + src * d);
  uint4* o = reinterpret_cast<uint4*>(out + j * d);
  for (int i = threadIdx.x; i < (d >> 3); i += 256) o[i] = s[i];
}

__global__ __launch_bounds__(256) void moe_combine_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ y,
                                                          const int* __restrict__ inv_idx,
                                                          const float* __restrict__ w, int K, int d) {
  const long t = blockIdx.x;
  for (int c = threadIdx.x * 8; c < d; c += 256 * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      const float wk = w[t * K + k];
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(y + (long)inv_idx[t * K + k] * d + c), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += wk * v[j];
    }
    *reinterpret_cast<uint4*>(out + t * d + c) = pack8(acc);
  }
}

}  // namespace k8sllm

using namespace k8sllm;

extern "C" {

int k8sllm_moe_route(const void* logits, long T, int E, int K, int renorm, int* topk_ids, float* topk_w,
                     hipStream_t s) {
  if (T <= 0) return 0;
  if (E > 64 || K > E) return -1;
  hipLaunchKernelGGL(moe_route_kernel, dim3((T + 255) / 256), dim3(256), 0, s, (const float*)logits, T, E, K, renorm,
                     topk_ids, topk_w);
  return (int)hipGetLastError();
}

int k8sllm_moe_router(const void* x, const void* wr, long T, int d, int E, int K, int renorm, int* ids, float* w,
                      float* wd, hipStream_t s) {
  if (T <= 0) return 0;
  if (E > 16 || K > E || d % 8 != 0) return -1;
  if (E <= 8)
    hipLaunchKernelGGL(moe_router_kernel<8>, dim3(T), dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)wr, d, E, K,
                       renorm, ids, w, wd);
  else
    hipLaunchKernelGGL(moe_router_kernel<16>, dim3(T), dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)wr, d, E, K,
                       renorm, ids, w, wd);
  return (int)hipGetLastError();
}

int k8sllm_moe_align(const int* topk_ids, long n, int E, int* expert_offsets, int* sorted_idx, int* inv_idx,
                     hipStream_t s) {
  if (E > kMaxE) return -1;
  hipLaunchKernelGGL(moe_align_kernel, dim3(1), dim3(kAT), 0, s, topk_ids, n, E, expert_offsets, sorted_idx, inv_idx);
  return (int)hipGetLastError();
}

int k8sllm_gather_rows(void* out, const void* x, const int* idx, long n, int d, int div, hipStream_t s) {
  if (n <= 0) return 0;
  if (d % 8 != 0) return -1;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(n), dim3(256), 0, s, (bf16_t*)out, (const bf16_t*)x, idx, d, div);
  return (int)hipGetLastError();
}

int k8sllm_moe_combine(void* out, const void* expert_out, const int* inv_idx, const float* topk_w, long T, int K,
                       int d, hipStream_t s) {
  if (T <= 0) return 0;
  if (d % 8 != 0) return -1;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, s, (bf16_t*)out, (const bf16_t*)expert_out, inv_idx,
                     topk_w, K, d);
  return (int)hipGetLastError();
}

}  // extern "C"
