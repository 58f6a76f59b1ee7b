// RMSNorm (optionally fused with the residual add), LayerNorm, SwiGLU and GELU(tanh)
// for gfx950.  All memory-bound: 16-byte vector loads, one workgroup per row for the
// norms (the row stays in registers between the reduction and the scale pass) and a
// grid-stride elementwise loop for the activations.
//
// Replaces the reference's *intended* remote-LLM path;
// the reference itself has no device code.
#include "common.h"

namespace k8sllm {

// out = rmsnorm(x [+ residual]) * w.  When ADD, residual <- bf16(x + residual) and the
// normalised value is computed from that rounded sum (matches HF's bf16 residual stream).
template <int NC, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                                                      bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
                                                      int d, float eps, long x_stride, long out_stride) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  const bf16_t* xr = x + (long)row * x_stride;
  bf16_t* rr = ADD ? residual + (long)row * d : nullptr;
  float v[NC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < d) {
      typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
      if (ADD) {
        // fused residual add (the prefill path): x (a projection output) and the old residual are
        // read once, and the new residual is not read again before the next layer half - all three
        // streams non-temporal; only the normalised output (the next GEMM's input) stays cached
        const u32x4_t a = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(xr + idx));
        const u32x4_t b = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(rr + idx));
        float r[8];
        unpack8(make_uint4(a.x, a.y, a.z, a.w), v[c]);
        unpack8(make_uint4(b.x, b.y, b.z, b.w), r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = bf2f(f2bf(v[c][j] + r[j]));
        const uint4 q = pack8(v[c]);
        __builtin_nontemporal_store(u32x4_t{q.x, q.y, q.z, q.w}, reinterpret_cast<u32x4_t*>(rr + idx));
      } else {
        unpack8(*reinterpret_cast<const uint4*>(xr + idx), v[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
    }
  }
  ss = block_sum<256>(ss, red);
  const float inv = rsqrtf(ss / (float)d + eps);
  bf16_t* orow = out + (long)row * out_stride;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < d) {
      float wf[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(w + idx), wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[c][j] * inv * wf[j];
      *reinterpret_cast<uint4*>(orow + idx) = pack8(o);
    }
  }
}

// LayerNorm with bias (GPT-2 family).  Two-moment reduction in one pass over registers.
template <int NC>
__global__ __launch_bounds__(256) void layernorm_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                                                        const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                        int d, float eps) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  const bf16_t* xr = x + (long)row * d;
  float v[NC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < d) {
      unpack8(*reinterpret_cast<const uint4*>(xr + idx), v[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    }
  }
  const float mean = block_sum<256>(s, red) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < d) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = v[c][j] - mean;
        q += t * t;
      }
    }
  }
  const float inv = rsqrtf(block_sum<256>(q, red) / (float)d + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < d) {
      float wf[8], bf[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(w + idx), wf);
      unpack8(*reinterpret_cast<const uint4*>(b + idx), bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * inv * wf[j] + bf[j];
      *reinterpret_cast<uint4*>(out + (long)row * d + idx) = pack8(o);
    }
  }
}

// SwiGLU: x = [gate | up] per row (width 2F), out = silu(gate) * up (width F).
// IL: gate/up interleaved per 128 columns as [64 gate | 64 up] (the single resident w13 layout,
// ops.interleave_gate_up, shared with the decode skinny SwiGLU epilogue); else [F gate | F up].
template <bool IL>
__global__ __launch_bounds__(256) void silu_mul_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                                                       long rows, int F) {
  // grid (ceil(F/8 / 256), min(rows, 65535)): 2-D indexing, no 64-bit division per element
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= F) return;
  for (long r = blockIdx.y; r < rows; r += gridDim.y) {
    const bf16_t* xr = x + r * 2 * F;
    float g[8], u[8], o[8];
    // the gate_up activations are read exactly once: non-temporal loads
    typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
    const int gc = IL ? ((c >> 6) << 7) + (c & 63) : c;
    const int uc = IL ? gc + 64 : F + c;
    const u32x4_t ga = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(xr + gc));
    const u32x4_t ua = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(xr + uc));
    unpack8(make_uint4(ga.x, ga.y, ga.z, ga.w), g);
    unpack8(make_uint4(ua.x, ua.y, ua.z, ua.w), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] / (1.f + __expf(-g[j])) * u[j];
    *reinterpret_cast<uint4*>(out + r * F + c) = pack8(o);
  }
}

// GELU, tanh approximation (GPT-2 "gelu_new"), elementwise over n elements (n % 8 == 0).
__global__ __launch_bounds__(256) void gelu_tanh_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                                                        long n) {
  const long nv = n >> 3;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    float a[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(x + i * 8), a);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = a[j];
      const float u = 0.7978845608028654f * (t + 0.044715f * t * t * t);
      o[j] = 0.5f * t * (1.f + tanhf(u));
    }
    *reinterpret_cast<uint4*>(out + i * 8) = pack8(o);
  }
}

// Vocab-parallel embedding gather: out[t] = W[ids[t] - vocab_start] when the id falls in
// this shard's [vocab_start, vocab_start + rows), else zeros (summed by the TP all-reduce).
__global__ __launch_bounds__(256) void embedding_kernel(bf16_t* __restrict__ out, const int* __restrict__ ids,
                                                        const bf16_t* __restrict__ weight, int d, int vocab_start,
                                                        int rows) {
  const int t = blockIdx.x;
  const int id = ids[t] - vocab_start;
  const bool in = id >= 0 && id < rows;
  const uint4* src = reinterpret_cast<const uint4*>(weight + (long)(in ? id : 0) * d);
  uint4* dst = reinterpret_cast<uint4*>(out + (long)t * d);
  for (int i = threadIdx.x; i < (d >> 3); i += 256) dst[i] = in ? src[i] : make_uint4(0, 0, 0, 0);
}

// Pipelined decode input ids: row i feeds prev[src[i]] (the token the previous, possibly still
// running, step sampled in row src[i]) when src[i] >= 0, else the host-provided ids[i].  One launch
// in the decode graph instead of torch's clamp / cast / index_select / compare / where chain.
__global__ __launch_bounds__(64) void resolve_ids_kernel(int* __restrict__ out, const int* __restrict__ ids,
                                                         const int* __restrict__ src, const int* __restrict__ prev,
                                                         int n) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const int r = src[i];
  out[i] = r >= 0 ? prev[r] : ids[i];
}

}  // namespace k8sllm

using namespace k8sllm;

static inline int grid_for(long work) {
  long g = (work + 255) / 256;
  if (g > 2048) g = 2048;  // 256 CUs x 8 resident blocks; grid-stride the rest
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" {

int k8sllm_rmsnorm(void* out, const void* x, void* residual, const void* w, long rows, int d, float eps,
                   long x_stride, long out_stride, hipStream_t s) {
  if (d % 8 != 0 || d > 256 * 8 * 8) return -1;
  const int nc = (d + 2047) / 2048;
  dim3 g(rows), b(256);
#define K8S_RMS(NC)                                                                                              \
  if (residual)                                                                                                  \
    hipLaunchKernelGGL((rmsnorm_kernel<NC, true>), g, b, 0, s, (bf16_t*)out, (const bf16_t*)x, (bf16_t*)residual, \
                       (const bf16_t*)w, d, eps, x_stride, out_stride);                                          \
  else                                                                                                           \
    hipLaunchKernelGGL((rmsnorm_kernel<NC, false>), g, b, 0, s, (bf16_t*)out, (const bf16_t*)x, nullptr,         \
                       (const bf16_t*)w, d, eps, x_stride, out_stride);
  if (nc <= 1) { K8S_RMS(1) }
  else if (nc <= 2) { K8S_RMS(2) }
  else if (nc <= 4) { K8S_RMS(4) }
  else { K8S_RMS(8) }
#undef K8S_RMS
  return (int)hipGetLastError();
}

int k8sllm_layernorm(void* out, const void* x, const void* w, const void* b, long rows, int d, float eps,
                     hipStream_t s) {
  if (d % 8 != 0 || d > 256 * 8 * 4) return -1;
  const int nc = (d + 2047) / 2048;
  if (nc <= 1)
    hipLaunchKernelGGL((layernorm_kernel<1>), dim3(rows), dim3(256), 0, s, (bf16_t*)out, (const bf16_t*)x,
                       (const bf16_t*)w, (const bf16_t*)b, d, eps);
  else if (nc <= 2)
    hipLaunchKernelGGL((layernorm_kernel<2>), dim3(rows), dim3(256), 0, s, (bf16_t*)out, (const bf16_t*)x,
                       (const bf16_t*)w, (const bf16_t*)b, d, eps);
  else
    hipLaunchKernelGGL((layernorm_kernel<4>), dim3(rows), dim3(256), 0, s, (bf16_t*)out, (const bf16_t*)x,
                       (const bf16_t*)w, (const bf16_t*)b, d, eps);
  return (int)hipGetLastError();
}

int k8sllm_silu_mul(void* out, const void* x, long rows, int F, int interleaved, hipStream_t s) {
  if (F % 8 != 0 || (interleaved && F % 64 != 0)) return -1;
  if (rows <= 0) return 0;
  const dim3 grid((F / 8 + 255) / 256, (unsigned)(rows < 65535 ? rows : 65535));
  if (interleaved)
    hipLaunchKernelGGL(silu_mul_kernel<true>, grid, dim3(256), 0, s, (bf16_t*)out, (const bf16_t*)x, rows, F);
  else
    hipLaunchKernelGGL(silu_mul_kernel<false>, grid, dim3(256), 0, s, (bf16_t*)out, (const bf16_t*)x, rows, F);
  return (int)hipGetLastError();
}

int k8sllm_gelu_tanh(void* out, const void* x, long n, hipStream_t s) {
  if (n % 8 != 0) return -1;
  hipLaunchKernelGGL(gelu_tanh_kernel, dim3(grid_for(n / 8)), dim3(256), 0, s, (bf16_t*)out, (const bf16_t*)x, n);
  return (int)hipGetLastError();
}

int k8sllm_embedding(void* out, const int* ids, const void* weight, long T, int d, int vocab_start, int rows,
                     hipStream_t s) {
  if (d % 8 != 0) return -1;
  hipLaunchKernelGGL(embedding_kernel, dim3(T), dim3(256), 0, s, (bf16_t*)out, ids, (const bf16_t*)weight, d,
                     vocab_start, rows);
  return (int)hipGetLastError();
}

int k8sllm_resolve_ids(int* out, const int* ids, const int* src, const int* prev, int n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(resolve_ids_kernel, dim3((n + 63) / 64), dim3(64), 0, s, out, ids, src, prev, n);
  return (int)hipGetLastError();
}

}  // extern "C"
