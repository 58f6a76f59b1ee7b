// Sustained MFMA ceiling on this MI355X: every CU runs 4 waves (one per SIMD) issuing back-to-back
// v_mfma_f32_16x16x32_bf16 on 64 independent accumulators (the prefill GEMM's per-wave shape), no
// memory traffic.  Prints achieved PF/s and the implied shader clock - the roof the GEMM kernels
// (ops/csrc/gemm_tile.hip) are compared against, since the spec peak assumes 2.4 GHz.
//
//   hipcc --offload-arch=gfx950 -O3 -o bin/mfma_peak tools/mfma_peak.hip && bin/mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// the same 256 accumulator registers as 16 tiles of v_mfma_f32_32x32x16_bf16 (4 x 4 per wave)
__global__ __launch_bounds__(256, 1) void mfma32_loop(float* out, int iters) {
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};
  bf16x8 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = bf16x8{} + (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = bf16x8{} + (__bf16)(0.002f * (threadIdx.x - i));
  }
  long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);  // issue order as written (no accumulator rotation)
      }
  }
  long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (float)(t1 - t0);
}

__global__ __launch_bounds__(256, 1) void mfma_loop(float* out, int iters) {
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = bf16x8{} + (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = bf16x8{} + (__bf16)(0.002f * (threadIdx.x - i));
  }
  long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
  }
  long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (float)(t1 - t0);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = cus * 4, iters = 4000;  // 4 rounds of one workgroup per CU
  float* d;
  hipMalloc(&d, (size_t)grid * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // kind 0: 16x16x32 on every CU (4 waves), 1: 32x32x16 on every CU, 2: 16x16x32 with ONE wave
  // per CU (no SIMD neighbours busy), 3: 32x32x16 with one wave per CU
  for (int kind = 0; kind < 4; ++kind) {
    const int threads = kind >= 2 ? 64 : 256;
    auto launch = [&](int it) {
      if (kind & 1) mfma32_loop<<<grid, threads>>>(d, it * 2);  // same flops: 16 x 32x32x16 = half an iteration of 64 x 16x16x32
      else mfma_loop<<<grid, threads>>>(d, it);
    };
    launch(100);
    hipDeviceSynchronize();
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      launch(iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      float cyc = 0.f;
      hipMemcpy(&cyc, d, 4, hipMemcpyDeviceToHost);
      const double flops = (double)grid * (threads / 64) * iters * 64 * 16.0 * 16 * 32 * 2;
      const double wg_ms = ms / 4.0;
      printf("{\"kind\": %d, \"mfma\": \"%s\", \"waves_per_cu\": %d, \"rep\": %d, \"ms\": %.3f, \"PFps\": %.3f, "
             "\"cyc_per_16x16x32_equiv\": %.2f, \"implied_GHz\": %.3f}\n",
             kind, (kind & 1) ? "32x32x16" : "16x16x32", threads / 64, rep, ms, flops / (ms * 1e-3) / 1e15,
             cyc / (iters * 64.0), cyc / (wg_ms * 1e-3) / 1e9);
    }
  }
  hipFree(d);
  return 0;
}
