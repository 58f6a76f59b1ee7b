// Grouped expert GEMM for MoE prefill, ONE launch over every local expert,
// driven by the device-side expert offsets of moe_align - no host synchronisation, so a MoE layer
// needs no `.tolist()` and a prefill step stays capturable.
//
//   Y[o_e + i][n] = sum_k X[o_e + i][k] * W[e][n][k]      i < M_e = o_{e+1} - o_e
//
// X: expert-sorted token rows [rows][K] (gather_rows), W: [E][N][K] row-major (the resident expert
// weights: the same tensors the decode skinny kernels read), both K-contiguous, so both MFMA
// operands are "row" fragments.  EPI_SWIGLU: W is gate/up-interleaved per 128 rows ([64 gate |
// 64 up], ops.interleave_gate_up) and the epilogue writes silu(gate) * up [rows][N / 2] directly.
//
// Tiling: workgroup = 128 rows x 128 columns, 4 waves, wave w owns rows 32w .. 32w + 31 across all
// 128 columns (4 accumulators of v_mfma_f32_32x32x16_bf16) - a SwiGLU tile's gate (columns 0-63)
// and up (64-127) values of a row then sit in the same lane and register.  K in 64-deep stages:
// A 128 x 128 B and B 128 x 128 B staged by global_load_lds_dwordx4 (8 rows x 128 B, whole lines,
// per instruction; 8 pieces per wave per stage) into a two-slot ring, one barrier per stage; the
// 16-B chunk c of LDS row r holds global chunk c ^ ((r >> 1) & 7), which makes the 16 lanes of a
// ds_read_b128 group hit 16 distinct bank quads (cdna_hip_programming.md T2, swizzle applied to
// the DMA source address, rule 21).
//
// Grid: (N / 128, mtiles_max) with mtiles_max = ceil(rows / 128) + E, an upper bound on
// sum_e ceil(M_e / 128) known on the host; each workgroup finds its (expert, m-tile) from the
// offsets (a scan over E <= 64 counts) and returns if it has none.
#include "common.h"

namespace k8sllm {

namespace {
typedef __attribute__((address_space(3))) void lds_void_g;
typedef __attribute__((address_space(1))) void gbl_void_g;

template <int N>
__device__ __forceinline__ void wait_vm_g() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
}  // namespace

enum { MOE_EPI_BF16 = 0, MOE_EPI_SWIGLU = 1 };

template <int EPI>
__global__ __launch_bounds__(256, 2) void moe_grouped_gemm_kernel(const bf16_t* __restrict__ X,
                                                                  const bf16_t* __restrict__ W,
                                                                  bf16_t* __restrict__ Y,
                                                                  const int* __restrict__ offsets, int E, int N,
                                                                  int K, long w_es) {
  constexpr int BM = 128, BN = 128, STAGE = (BM + BN) * 128;  // 32 KiB
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;

  // (expert, m-tile) of this workgroup from the device offsets
  int e = -1, row0 = 0, mrows = 0;
  {
    int acc = 0;
    const int mt = blockIdx.y;
    for (int x = 0; x < E; ++x) {
      const int o0 = offsets[x], o1 = offsets[x + 1];
      const int tiles = (o1 - o0 + BM - 1) / BM;
      if (e < 0 && mt < acc + tiles) {
        e = x;
        row0 = o0 + (mt - acc) * BM;
        mrows = min(BM, o1 - row0);
      }
      acc += tiles;
    }
  }
  if (e < 0) return;  // uniform: past the last expert's tiles
  const int n0 = blockIdx.x * BN;
  const bf16_t* Wt = W + (long)e * w_es;

  // DMA sources: piece j (0..31) of a stage = LDS rows 8j .. 8j + 7; pieces 0-15 A, 16-31 B;
  // wave w issues pieces 8w .. 8w + 7
  const bf16_t* src[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int j = wave * 8 + i;
    const int rl = (j & 15) * 8 + (lane >> 3);  // row within the A or B tile
    const int c = (lane & 7) ^ ((rl >> 1) & 7);
    if (j < 16) {
      const int r = row0 + min(rl, mrows - 1);  // rows past the expert's last: clamped, discarded
      src[i] = X + (long)r * K + c * 8;
    } else {
      src[i] = Wt + (long)(n0 + rl) * K + c * 8;
    }
  }
  auto issue = [&](int kt, int slot) {
    char* st = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void_g*)(src[i] + kt * 64), (lds_void_g*)(st + (wave * 8 + i) * 1024),
                                       16, 0, 0);
  };

  f32x16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  const int r32 = lane & 31, hh = lane >> 5;
  const int arow = wave * 32 + r32;
  const int nk = K / 64;
  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    wait_vm_g<0>();                 // this wave's pieces of stage kt landed
    __builtin_amdgcn_s_barrier();   // everyone's did; everyone is done reading stage kt - 1
    if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);
    const char* st = smem + (kt & 1) * STAGE;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = 2 * ks + hh;  // 16-B chunk of the 128-B row: k = 16 ks + 8 hh
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(st + arow * 128 + ((c ^ ((arow >> 1) & 7)) << 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int br = 32 * j + r32;
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(st + BM * 128 + br * 128 + ((c ^ ((br >> 1) & 7)) << 4));
        // acc[j][reg]: row (reg & 3) + 8 (reg >> 2) + 4 hh of the wave's 32, column 32 j + r32
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc[j], 0, 0, 0);
      }
    }
  }

  // epilogue.  acc[j] = (W X^T)[n = 32 j + (reg-row)][row = r32]: the MFMA above took B (weights)
  // as the A operand, so the accumulator's row index runs over columns n and its column (lane)
  // over the token rows - each lane owns one token row and 64 of the tile's columns.
  const int row = wave * 32 + r32;
  if (row >= mrows) return;
  bf16_t* yr;
  if constexpr (EPI == MOE_EPI_SWIGLU) {
    // gate columns 32 j (j = 0, 1) pair with up columns 64 + 32 j (j + 2), same register index
    yr = Y + (long)(row0 + row) * (N >> 1) + (n0 >> 1);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float o[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int reg = q * 4 + t;
          const float g = bf2f(f2bf(acc[j][reg])), u = bf2f(f2bf(acc[j + 2][reg]));
          o[t] = g * u / (1.f + __expf(-g));
        }
        // registers 4q .. 4q + 3 = columns 32 j + 8 q + 4 hh + 0..3: one 8-byte store
        *reinterpret_cast<uint2*>(yr + 32 * j + 8 * q + 4 * hh) = uint2{pack2(o[0], o[1]), pack2(o[2], o[3])};
      }
  } else {
    yr = Y + (long)(row0 + row) * N + n0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<uint2*>(yr + 32 * j + 8 * q + 4 * hh) =
            uint2{pack2(acc[j][4 * q], acc[j][4 * q + 1]), pack2(acc[j][4 * q + 2], acc[j][4 * q + 3])};
  }
}

}  // namespace k8sllm

using namespace k8sllm;

// rows: total expert-sorted rows (the grid bound); epi 0: Y [rows][N]; 1: SwiGLU Y [rows][N / 2].
extern "C" int k8sllm_moe_grouped_gemm(const void* X, const void* W, void* Y, const int* offsets, int E, long rows,
                                       int N, int K, long w_es, int epi, hipStream_t s) {
  if (rows <= 0) return 0;
  if (N % 128 != 0 || K % 64 != 0 || E < 1 || E > 256) return -1;
  const long mt = (rows + 127) / 128 + E;
  if (mt > 65535) return -2;
  dim3 grid(N / 128, (unsigned)mt), blk(256);
  if (epi == MOE_EPI_SWIGLU)
    hipLaunchKernelGGL((moe_grouped_gemm_kernel<MOE_EPI_SWIGLU>), grid, blk, 0, s, (const bf16_t*)X,
                       (const bf16_t*)W, (bf16_t*)Y, offsets, E, N, K, w_es);
  else
    hipLaunchKernelGGL((moe_grouped_gemm_kernel<MOE_EPI_BF16>), grid, blk, 0, s, (const bf16_t*)X, (const bf16_t*)W,
                       (bf16_t*)Y, offsets, E, N, K, w_es);
  return (int)hipGetLastError();
}
