// HBM streaming microbenchmark for the decode GEMM access patterns on MI355X.
// Reads a [N=4096, K] bf16 weight (rotating over > 256 MiB of copies so the MALL cannot serve
// it) with different per-lane address patterns and reports TB/s:
//   flat      - grid-stride, each lane 16 B, a wave reads 1 KiB contiguous
//   frag      - MFMA B-fragment order: 16 rows x 4 lanes x 16 B per instruction; the WG's waves
//               interleave k-steps (what gemm_skinny v1 does)
//   fragperm  - fragment order with a k permutation: lane (r, q) reads U consecutive 16 B
//               pieces, so each row's 4 lanes cover U*64 B contiguous per wave
//   rows      - a wave reads 4 rows x 256 B per instruction (LDS-staged GEMM order)
// Build: hipcc --offload-arch=gfx950 -O3 tools/membw.hip -o /tmp/membw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef unsigned short bf16;

__global__ __launch_bounds__(256) void flat(const uint4* __restrict__ w, long n16, float* out) {
  uint32_t acc = 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256) {
    uint4 v = w[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) out[0] = 1.f;
}

// grid (N/64, S): 64 columns x K/S; U k-steps of 32 in flight per wave
template <int U>
__global__ __launch_bounds__(256) void frag(const bf16* __restrict__ W, int K, int kchunk, float* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r16 = lane & 15, kq = lane >> 4;
  const int n0 = blockIdx.x * 64, kbeg = blockIdx.y * kchunk, nsteps = kchunk / 32;
  uint32_t acc = 0;
  for (int i0 = wave; i0 < nsteps; i0 += 4 * U) {
    uint4 b[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = kbeg + 32 * min(i0 + 4 * u, nsteps - 1) + 8 * kq;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) b[u][nt] = *reinterpret_cast<const uint4*>(W + (long)(n0 + nt * 16 + r16) * K + k);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc ^= b[u][nt].x ^ b[u][nt].w;
  }
  if (acc == 0x12345678) out[0] = 1.f;
}

// each wave owns a contiguous K range of the WG chunk; lane (r,q) reads U pieces at q*U*16B + u*16B
template <int U>
__global__ __launch_bounds__(256) void fragperm(const bf16* __restrict__ W, int K, int kchunk, float* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r16 = lane & 15, kq = lane >> 4;
  const int n0 = blockIdx.x * 64, kbeg = blockIdx.y * kchunk;
  const int span = 32 * U;  // k per wave round
  uint32_t acc = 0;
  for (int k0 = kbeg + wave * span; k0 < kbeg + kchunk; k0 += 4 * span) {
    uint4 b[U][4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int u = 0; u < U; ++u)
        b[u][nt] = *reinterpret_cast<const uint4*>(W + (long)(n0 + nt * 16 + r16) * K + k0 + kq * 8 * U + 8 * u);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc ^= b[u][nt].x ^ b[u][nt].w;
  }
  if (acc == 0x12345678) out[0] = 1.f;
}

// a wave instruction reads 4 rows x 256 B; WG covers 64 rows x kchunk
template <int U>
__global__ __launch_bounds__(256) void rows(const bf16* __restrict__ W, int K, int kchunk, float* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = blockIdx.x * 64, kbeg = blockIdx.y * kchunk;
  uint32_t acc = 0;
  // wave w handles rows n0 + 16w .. +16; per instruction 4 rows (lane>>4) x 16 lanes x 16 B (128 k)
  for (int k0 = kbeg; k0 < kbeg + kchunk; k0 += 128 * U) {
    uint4 b[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = n0 + wave * 16 + j * 4 + (lane >> 4);
        const int k = min(k0 + u * 128, kbeg + kchunk - 128) + (lane & 15) * 8;
        b[u][j] = *reinterpret_cast<const uint4*>(W + (long)row * K + k);
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc ^= b[u][j].x ^ b[u][j].w;
  }
  if (acc == 0x12345678) out[0] = 1.f;
}

int main() {
  const int N = 4096;
  const int Ks[2] = {4096, 14336};
  float* out;
  CK(hipMalloc(&out, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int K : Ks) {
    const size_t bytes = (size_t)N * K * 2;
    const int ncopy = (int)((640ull << 20) / bytes) + 1;
    std::vector<bf16*> ws(ncopy);
    for (auto& p : ws) {
      CK(hipMalloc(&p, bytes));
      CK(hipMemset(p, 1, bytes));
    }
    auto run = [&](const char* name, int S, auto launch) {
      for (int i = 0; i < 3; ++i) launch(ws[i % ncopy]);
      hipDeviceSynchronize();
      const int iters = 60;
      hipEventRecord(a);
      for (int i = 0; i < iters; ++i) launch(ws[i % ncopy]);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double us = ms * 1e3 / iters;
      printf("K=%5d %-14s S=%2d  %7.2f us  %5.2f TB/s\n", K, name, S, us, bytes / us / 1e6);
    };
    for (int grid : {256, 512, 1024, 2048}) {
      char nm[32];
      snprintf(nm, sizeof nm, "flat g%d", grid);
      run(nm, 0, [&](bf16* w) { hipLaunchKernelGGL(flat, dim3(grid), dim3(256), 0, 0, (const uint4*)w, (long)(bytes / 16), out); });
    }
    for (int S : {1, 2, 4, 8, 16}) {
      const int kc = K / S;
      if (kc % 512) continue;
      run("frag U4", S, [&](bf16* w) { hipLaunchKernelGGL(frag<4>, dim3(N / 64, S), dim3(256), 0, 0, w, K, kc, out); });
      run("frag U8", S, [&](bf16* w) { hipLaunchKernelGGL(frag<8>, dim3(N / 64, S), dim3(256), 0, 0, w, K, kc, out); });
      run("fragperm U4", S, [&](bf16* w) { hipLaunchKernelGGL(fragperm<4>, dim3(N / 64, S), dim3(256), 0, 0, w, K, kc, out); });
      run("fragperm U8", S, [&](bf16* w) { hipLaunchKernelGGL(fragperm<8>, dim3(N / 64, S), dim3(256), 0, 0, w, K, kc, out); });
      run("rows U2", S, [&](bf16* w) { hipLaunchKernelGGL(rows<2>, dim3(N / 64, S), dim3(256), 0, 0, w, K, kc, out); });
      run("rows U4", S, [&](bf16* w) { hipLaunchKernelGGL(rows<4>, dim3(N / 64, S), dim3(256), 0, 0, w, K, kc, out); });
    }
    for (auto p : ws) CK(hipFree(p));
  }
  return 0;
}
