// Decode-time "skinny" GEMM on gfx950 MFMA: Y[M, N] = A[M, K] . W[N, K]^T for M <= 64 rows (the
// decode batch), bf16 in, fp32 accumulate.  Serves the decode projections gemm_decode.hip has no
// launch configuration for (MoE experts as grouped launches, odd shapes) and models built without
// CausalLM.ONE_LAYOUT; dense Llama decode runs on gemm_decode.hip over the one packed weight copy,
// which the prefill tile GEMM (gemm_tile.hip) reads as well.
//
// Weight layout - "fragment-packed" [N/16][K/32][64 lanes][8] bf16 (pack_weight_for_skinny in
// ops/__init__.py): the 16x32 B fragment of v_mfma_f32_16x16x32_bf16 for n-tile j, k-step s is one
// contiguous 1 KiB block in lane order, so every weight load instruction of a wave reads 1 KiB
// contiguous straight into MFMA operand registers.  Measured on MI355X (tools/membw.hip): reading
// a row-major [N][K] weight in MFMA-fragment order (16 rows x 64 B per instruction) streams at
// 1.1-3.9 TB/s; whole-line orders reach 4.7-5.7 TB/s - the packed layout gets the latter with no
// LDS round trip.  Weights are read once per step (14 GB for Llama-3-8B), so loads are
// non-temporal (MI355X_MICROARCH.md "nt-weights"; measured 2-10 % faster than default-policy
// loads here, tools/bench_skinny.py).
//
// Decomposition: workgroup = 4 waves, NT n-tiles (16 NT output columns) x one K slice; grid =
// (N / (16 NT), slices).  The waves take interleaved groups of U consecutive k-steps of the slice
// and combine through LDS at the end.  Epilogues:
//   SLAB   - fp32 split-K partials partial[slice][m][n], summed by the NEXT kernel
//            (reduce_add_rmsnorm below, or rope_and_cache for qkv): the launch-boundary reduce of
//            cdna_hip_programming.md §5 "Projection GEMM at M = 256" item 2 - no in-launch fences
//   BF16   - one slice: Y = bf16(acc)
//   SWIGLU - one slice, NT = 4, weight rows interleaved per 64-column tile as [32 gate | 32 up]:
//            Y[m, f] = silu(gate) * up - the gate_up projection writes the MLP activation directly
//            (no silu_mul pass, and the down projection reads F, not 2F, columns)
//   SWIGLU_PACKED - the same, written fragment-packed ([ceil(M/16)][F/32][64][8]) as the down
//            projection's A operand
// A (activations) is row-major or fragment-packed like W; the packed form turns the A loads into
// whole-line reads too (at M = 64 the A bytes per workgroup equal the W bytes).
#include <cstdlib>

#include "common.h"
#include <type_traits>

namespace k8sllm {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

enum { EPI_SLAB = 0, EPI_BF16 = 1, EPI_SWIGLU = 2, EPI_SWIGLU_PACKED = 3 };

// Grouped (MoE expert) launches: grid.z = experts; expert x reads weights Wp + x * w_es, activations
// A + x * a_es (0: every expert reads the same A), writes Y + x * y_es / slabs [x * S + s], and
// (row_w) scales output row m by row_w[m * row_w_ld + x] - the routing weight, 0 for experts the
// token did not select.  The down projection's slabs over (expert, split) are then summed by the
// same residual-add kernels as a dense layer's split-K slabs.
struct SkinnyGroup {
  long w_es, a_es, y_es;
  const float* row_w;
  int row_w_ld;
};

// n-tile read for the workgroup's nt-th tile.  SwiGLU weights are interleaved per 128 rows as
// [64 gate | 64 up] (interleave_gate_up): a 4-tile workgroup takes two gate tiles and the two
// matching up tiles, so every output column has its gate and up value in the same workgroup.
template <int EPI, int NT>
__device__ __forceinline__ int swiglu_tile(int ntile0, int nt) {
  if constexpr (EPI == 2 || EPI == 3) {
    const int bx = ntile0 / NT;
    return (bx >> 1) * 8 + (bx & 1) * 2 + (nt & 1) + (nt >> 1) * 4;
  } else {
    return ntile0 + nt;
  }
}

// Loads of one wave group: U consecutive k-steps, NT weight and MT activation fragments each.
template <int U, int MT, int NT>
struct SkinnyBatch {
  u32x4 b[U][NT];
  bf16x8 a[U][MT];
};

// Cross-wave combine of the per-wave accumulators and the epilogue (shared by the packed and the
// row-major kernels), one m-tile per round.  red: [WAVES][NT][64][4] floats.  s_inv: the A rows'
// 1/rms (deferred RMSNorm) or nullptr.  C/D layout of the 16x16 tile: col = lane & 15, rows
// (lane >> 4) * 4 + r.
template <int MT, int NT, int EPI, int WAVES>
__device__ __forceinline__ void skinny_epilogue(const f32x4 (&acc)[MT][NT], float* red, const float* s_inv,
                                                float* __restrict__ partial, bf16_t* __restrict__ Y, long ldy, int M,
                                                int N, int ntile0, int s, int ex, const SkinnyGroup& grp) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  auto R = [&](int w, int nt, int l) -> f32x4* {
    return reinterpret_cast<f32x4*>(red + ((w * NT + nt) * 64 + l) * 4);
  };
  constexpr int NOUT = EPI == EPI_SWIGLU || EPI == EPI_SWIGLU_PACKED ? NT / 2 : NT;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    if (mt > 0) __syncthreads();  // previous round's reads done
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) *R(wave, nt, lane) = acc[mt][nt];
    __syncthreads();
    for (int idx = threadIdx.x; idx < NOUT * 64; idx += 64 * WAVES) {
      const int nt = idx >> 6, l = idx & 63;
      f32x4 v = *R(0, nt, l);
#pragma unroll
      for (int w = 1; w < WAVES; ++w) v += *R(w, nt, l);
      // deferred RMSNorm of the A rows (add_norm_partial): A held x * w, the row's 1/rms
      // (s_inv, computed at kernel start) is applied here - linear, so exact for split-K slabs too
      f32x4 rs = f32x4{1.f, 1.f, 1.f, 1.f};
      if (s_inv != nullptr) {
#pragma unroll
        for (int r = 0; r < 4; ++r) rs[r] = s_inv[mt * 16 + (l >> 4) * 4 + r];
      }
      v *= rs;
      if constexpr (EPI == EPI_SWIGLU || EPI == EPI_SWIGLU_PACKED) {
        f32x4 u = *R(0, nt + NT / 2, l);
#pragma unroll
        for (int w = 1; w < WAVES; ++w) u += *R(w, nt + NT / 2, l);
        u *= rs;
        // gate n-tiles 8q + 2h + {0,1} pair with up n-tiles 8q + 4 + 2h + {0,1} (swiglu_tile)
        const int f = (blockIdx.x >> 1) * 64 + (blockIdx.x & 1) * 32 + nt * 16 + (l & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = mt * 16 + (l >> 4) * 4 + r;
          // the gate and up values are rounded to bf16 first, as the unfused GEMM -> silu_mul does
          const float g = bf2f(f2bf(v[r]));
          const float uu = bf2f(f2bf(u[r]));
          const bf16_t o = f2bf(g * uu / (1.f + __expf(-g)));
          if constexpr (EPI == EPI_SWIGLU_PACKED) {
            // fragment-packed activation for the down projection's A operand: [MT][F/32][64][8]
            const int F = N >> 1;
            Y[(((long)mt * (F >> 5) + (f >> 5)) * 64 + ((f >> 3) & 3) * 16 + (row & 15)) * 8 + (f & 7)] = o;
          } else if (row < M) {
            Y[(long)row * ldy + f] = o;
          }
        }
      } else {  // SLAB / BF16
        const int col = swiglu_tile<EPI, NT>(ntile0, nt) * 16 + (l & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = mt * 16 + (l >> 4) * 4 + r;
          if (row < M) {
            const float o = grp.row_w != nullptr ? v[r] * grp.row_w[(long)row * grp.row_w_ld + ex] : v[r];
            if constexpr (EPI == EPI_BF16)
              Y[(long)row * ldy + col] = f2bf(o);
            else
              partial[((long)(ex * gridDim.y + s) * M + row) * N + col] = o;
          }
        }
      }
    }
  }
}

template <int MT, int NT, int EPI, bool APK, int WAVES>
__global__ __launch_bounds__(64 * WAVES, 2) void gemm_skinny_kernel(const bf16_t* __restrict__ A, long lda,
                                                          const bf16_t* __restrict__ Wp, float* __restrict__ partial,
                                                          bf16_t* __restrict__ Y, long ldy, int M, int N, int K,
                                                          int kchunk, const float* __restrict__ rn_ss, int rn_nc,
                                                          float rn_inv_d, float rn_eps, SkinnyGroup grp) {
  // U k-steps per wave group; two groups in flight per wave (register double buffer)
  constexpr int U = MT <= 2 ? 4 : 2;
  __shared__ __attribute__((aligned(16))) float red[WAVES][NT][64][4];  // one m-tile at a time: 16 KiB per 4 waves
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ntile0 = blockIdx.x * NT;
  const int s = blockIdx.y;
  const int ex = blockIdx.z;  // expert of a grouped launch (0 otherwise)
  Wp += ex * grp.w_es;
  A += ex * grp.a_es;
  if (Y != nullptr) Y += ex * grp.y_es;
  const int kbeg = s * kchunk;
  const int nsteps = (min(K, kbeg + kchunk) - kbeg) >> 5;  // host guarantees 32 | K and 32 | kchunk
  const int ksteps = K >> 5;

  const u32x4* wp[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    wp[nt] = reinterpret_cast<const u32x4*>(Wp) + ((long)swiglu_tile<EPI, NT>(ntile0, nt) * ksteps + (kbeg >> 5)) * 64 +
             lane;
  // A: row-major [M][lda] (fragment-shaped loads, padding rows clamped) or, APK, fragment-packed
  // like W ([ceil(M/16)][K/32][64][8], padding rows present) so A loads are 1 KiB contiguous too
  const bf16_t* ap[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    if constexpr (APK)
      ap[mt] = A + (((long)mt * ksteps + (kbeg >> 5)) * 64 + lane) * 8;
    else
      ap[mt] = A + (long)min(mt * 16 + (lane & 15), M - 1) * lda + kbeg + 8 * (lane >> 4);
  }
  constexpr int ASTEP = APK ? 512 : 32;  // bf16 elements between consecutive k-steps

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // deferred RMSNorm: 1/rms of each A row from its partial sums of squares, once per workgroup
  // (its loads overlap the first weight loads; read back in the epilogue after the barriers)
  // (4 threads per row: the producer may leave up to 128 partial sums per row)
  __shared__ float s_inv[MT * 16];
  if (rn_ss != nullptr && threadIdx.x < MT * 64) {  // whole waves: MT * 64 threads
    const int rl = threadIdx.x >> 2, part = threadIdx.x & 3;
    const int row = min(rl, M - 1);
    float ss = 0.f;
    for (int c = part; c < rn_nc; c += 4) ss += rn_ss[row * rn_nc + c];
    ss += __shfl_xor(ss, 1, kWave);
    ss += __shfl_xor(ss, 2, kWave);
    if (part == 0) s_inv[rl] = rsqrtf(ss * rn_inv_d + rn_eps);
  }

  auto load = [&](SkinnyBatch<U, MT, NT>& bt, int i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int st = min(i0 + u, nsteps - 1);  // tail steps re-read a valid step; their MFMAs are skipped
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bt.b[u][nt] = __builtin_nontemporal_load(wp[nt] + st * 64);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) bt.a[u][mt] = *reinterpret_cast<const bf16x8*>(ap[mt] + st * ASTEP);
    }
  };
  auto compute = [&](const SkinnyBatch<U, MT, NT>& bt, int i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i0 + u < nsteps) {  // wave-uniform
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bt.a[u][mt], __builtin_bit_cast(bf16x8, bt.b[u][nt]),
                                                                   acc[mt][nt], 0, 0, 0);
      }
    }
  };

  // software pipeline: the next group's loads are issued before this group's MFMAs, so every
  // wave keeps two groups of weight lines in flight instead of stalling once per group
  constexpr int STRIDE = WAVES * U;
  int i0 = wave * U;
  if (i0 < nsteps) {
    SkinnyBatch<U, MT, NT> b0, b1;
    load(b0, i0);
    while (true) {
      const int i1 = i0 + STRIDE;
      if (i1 < nsteps) load(b1, i1);
      __builtin_amdgcn_sched_barrier(0);
      compute(b0, i0);
      if (i1 >= nsteps) break;
      const int i2 = i1 + STRIDE;
      if (i2 < nsteps) load(b0, i2);
      __builtin_amdgcn_sched_barrier(0);
      compute(b1, i1);
      if (i2 >= nsteps) break;
      i0 = i2;
    }
  }

  skinny_epilogue<MT, NT, EPI, WAVES>(acc, &red[0][0][0][0], rn_ss != nullptr ? s_inv : nullptr, partial, Y, ldy, M,
                                      N, ntile0, s, ex, grp);
}

// Row-major weights, LDS-DMA staged: the SAME decomposition, epilogues and fragment-packed A as
// gemm_skinny_kernel, but W is the plain row-major [N][K] tensor (MoE experts, and dense models
// built without CausalLM.ONE_LAYOUT, whose prefill GEMMs read the same tensor).
//
// Why LDS: an MFMA B fragment (16 rows x 32 k) read straight from a row-major W touches 16 rows x
// 64 B per wave-instruction; whole-line orders stream 1.5-4x faster (tools/membw.hip).  Here each
// wave streams its own rows in whole 128-B lines with global_load_lds_dwordx4 (8 rows x 128 B per
// instruction, non-temporal: weights are read once per step) into a private two-slot LDS ring,
// and reads the fragments back with conflict-free ds_read_b128: the 16-B chunk c of LDS row r
// holds global chunk c ^ ((r >> 1) & 7), so the 16 rows of one fragment read hit 16 distinct
// bank quads (cdna_hip_programming.md T2; the swizzle sits on the per-lane SOURCE address because
// the DMA writes lane-linear, rule 21).  The fragment-packed A operand is staged the same way
// (1 KiB contiguous per m-tile and k-step, read lane-linear).  Every load of the main loop is an
// LDS-DMA, so the waits are explicit counted vmcnt (hipcc drains to vmcnt(0) beside a mix of
// DMA and register loads, §5 "Projection GEMM" item 4(b)); no barrier - each wave reads only
// what it loaded itself.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

// Row-oriented combine + epilogue of the row-major kernel, all m-tiles in one round: every wave
// parks its accumulators as rows of a padded [WAVES][MT*16][NT*16 + 4] fp32 image (conflict-free
// ds_write_b32: the 4-float pad moves each 4-row lane group to its own 16 banks), one barrier,
// then each thread sums 4 consecutive columns of one row over the waves (ds_read_b128, one
// 256-B row per 16 lanes) and stores them whole: 16-B slab stores (a 64-column tile row = one
// 256-B segment) and 8-B bf16 stores.  The ablation that motivated it (tools/abl_skinny_rm.py,
// profiles/r02/skinny_rm_ablation.jsonl): at M = 64 the per-m-tile rounds with 4-byte slab
// stores cost 2-3.5 us per projection.
template <int MT, int NT, int EPI, int WAVES>
__device__ __forceinline__ void skinny_epilogue_rows(const f32x4 (&acc)[MT][NT], float* red, const float* s_inv,
                                                     float* __restrict__ partial, bf16_t* __restrict__ Y, long ldy,
                                                     int M, int N, int ntile0, int s, int ex, const SkinnyGroup& grp) {
  constexpr int LD = NT * 16 + 4, ROWS = MT * 16, NTH = 64 * WAVES;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(wave * ROWS + mt * 16 + (lane >> 4) * 4 + r) * LD + nt * 16 + (lane & 15)] = acc[mt][nt][r];
  __syncthreads();
  auto sum4 = [&](int row, int c) {
    f32x4 v = *reinterpret_cast<const f32x4*>(red + row * LD + c);
#pragma unroll
    for (int w = 1; w < WAVES; ++w) v += *reinterpret_cast<const f32x4*>(red + (w * ROWS + row) * LD + c);
    return v;
  };
  if constexpr (EPI == EPI_SWIGLU || EPI == EPI_SWIGLU_PACKED) {
    // gate n-tiles (nt 0, 1) pair with up n-tiles (nt 2, 3): column j of the gate half with 32 + j
    for (int it = threadIdx.x; it < ROWS * 8; it += NTH) {
      const int row = it >> 3, j = (it & 7) * 4;
      const float rs = s_inv != nullptr ? s_inv[row] : 1.f;
      const f32x4 g4 = sum4(row, j) * rs, u4 = sum4(row, 32 + j) * rs;
      float o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // the gate and up values are rounded to bf16 first, as the unfused GEMM -> silu_mul does
        const float g = bf2f(f2bf(g4[q])), uu = bf2f(f2bf(u4[q]));
        o[q] = g * uu / (1.f + __expf(-g));
      }
      const int f = (blockIdx.x >> 1) * 64 + (blockIdx.x & 1) * 32 + j;
      if constexpr (EPI == EPI_SWIGLU_PACKED) {  // 4 consecutive f: contiguous in the packed layout
        const int F = N >> 1;
        *reinterpret_cast<uint2*>(Y + (((long)(row >> 4) * (F >> 5) + (f >> 5)) * 64 + ((f >> 3) & 3) * 16 +
                                       (row & 15)) * 8 + (f & 7)) = uint2{pack2(o[0], o[1]), pack2(o[2], o[3])};
      } else if (row < M) {
#pragma unroll
        for (int q = 0; q < 4; ++q) Y[(long)row * ldy + f + q] = f2bf(o[q]);
      }
    }
  } else {
    for (int it = threadIdx.x; it < ROWS * NT * 4; it += NTH) {
      const int row = it / (NT * 4), c = (it % (NT * 4)) * 4;
      if (row >= M) continue;
      f32x4 v = sum4(row, c);
      if (s_inv != nullptr) v *= s_inv[row];
      if (grp.row_w != nullptr) v *= grp.row_w[(long)row * grp.row_w_ld + ex];
      const int col = swiglu_tile<EPI, NT>(ntile0, c >> 4) * 16 + (c & 15);
      if constexpr (EPI == EPI_BF16) {
#pragma unroll
        for (int q = 0; q < 4; ++q) Y[(long)row * ldy + col + q] = f2bf(v[q]);
      } else {
        *reinterpret_cast<f32x4*>(partial + ((long)(ex * gridDim.y + s) * M + row) * N + col) = v;
      }
    }
  }
}

template <int MT, int NT, int EPI, int WAVES>
struct SkinnyRmGeom {
  static constexpr int U = 2;                        // k-steps per stage: 64 k = one 128-B line per row
  static constexpr int WB = NT * 16 * 128;           // W bytes per stage
  static constexpr int AB = MT * U * 1024;           // A bytes per stage
  static constexpr int SB = WB + AB;
  static constexpr int RING = 2 * SB;                // per wave
  static constexpr int LDR = NT * 16 + 4;            // combine row pitch (floats): conflict-free
  static constexpr int RED = WAVES * MT * 16 * LDR * 4;  // cross-wave combine (aliases the rings)
  static constexpr int EPI_LDS = RED + MT * 16 * 4;  // + s_inv, written after the main loop
  static constexpr int LDS = WAVES * RING > EPI_LDS ? WAVES * RING : EPI_LDS;
  static constexpr int NLOAD = NT * 2 + MT * U;      // DMA instructions per stage
};

template <int MT, int NT, int EPI, int WAVES>
__global__ __launch_bounds__(64 * WAVES, 1) void gemm_skinny_rm_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ W, long ldw, float* __restrict__ partial,
    bf16_t* __restrict__ Y, long ldy, int M, int N, int K, int kchunk, const float* __restrict__ rn_ss, int rn_nc,
    float rn_inv_d, float rn_eps, SkinnyGroup grp) {
  using G = SkinnyRmGeom<MT, NT, EPI, WAVES>;
  constexpr int U = G::U;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  float* s_inv = reinterpret_cast<float*>(smem + G::RED);  // aliases a ring: written after the loop
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ntile0 = blockIdx.x * NT;
  const int s = blockIdx.y;
  const int ex = blockIdx.z;
  W += ex * grp.w_es;
  A += ex * grp.a_es;
  if (Y != nullptr) Y += ex * grp.y_es;
  const int kbeg = s * kchunk;
  const int nsteps = (min(K, kbeg + kchunk) - kbeg) >> 5;  // host: 64 | K and 64 | kchunk
  const int ksteps = K >> 5;
  const int ngroups = nsteps / U;

  // deferred RMSNorm: partial sums of squares of the A rows (4 threads per row, so a 2-wave
  // workgroup covers 32 rows per pass and holds two), loaded before the first DMA (its waits then
  // drain nothing of the ring) and held in registers through the main loop
  constexpr int SSP = (MT * 64 + 64 * WAVES - 1) / (64 * WAVES);
  float ss[SSP];
#pragma unroll
  for (int p = 0; p < SSP; ++p) {
    ss[p] = 0.f;
    const int t = threadIdx.x + p * 64 * WAVES;  // wave-uniform bound: MT * 64 is whole waves
    if (rn_ss != nullptr && t < MT * 64) {
      const int row = min(t >> 2, M - 1);
      for (int c = t & 3; c < rn_nc; c += 4) ss[p] += rn_ss[row * rn_nc + c];
    }
  }

  // per-lane DMA sources at k-step 0 of the slice: W instruction j covers LDS rows 8j..8j+7
  const bf16_t* wsrc[NT * 2];
#pragma unroll
  for (int j = 0; j < NT * 2; ++j) {
    const int rl = 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ ((rl >> 1) & 7);
    const long grow = (long)swiglu_tile<EPI, NT>(ntile0, rl >> 4) * 16 + (rl & 15);
    wsrc[j] = W + grow * ldw + kbeg + c * 8;
  }
  const bf16_t* asrc = A + ((long)(kbeg >> 5) * 64 + lane) * 8;
  char* ring = smem + wave * G::RING;

  auto issue = [&](int slot, int g) {
    const int k0 = g * U;  // k-step within the slice
    char* st = ring + slot * G::SB;
#pragma unroll
    for (int j = 0; j < NT * 2; ++j)
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(wsrc[j] + k0 * 32), (lds_void_t*)(st + j * 1024), 16, 0, 2);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int u = 0; u < U; ++u)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(asrc + ((long)mt * ksteps + k0 + u) * 512),
                                         (lds_void_t*)(st + G::WB + (mt * U + u) * 1024), 16, 0, 0);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (bytes within a stage)
  int woff[NT][U];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rl = nt * 16 + (lane & 15);
      woff[nt][u] = rl * 128 + (((u * 4 + (lane >> 4)) ^ ((rl >> 1) & 7)) << 4);
    }

  // groups g = wave, wave + WAVES, ... ; two stages in flight per wave
  const int nmy = wave < ngroups ? (ngroups - wave + WAVES - 1) / WAVES : 0;
  if (nmy > 0) issue(0, wave);
  if (nmy > 1) issue(1, wave + WAVES);
  // one stage: wait for it, read its fragments (the slot is then free), MFMAs.  In the main loop
  // the next-but-one stage's DMA pieces are interleaved with the MFMAs (each piece's issue cost
  // overlaps the MFMA pipeline instead of preceding all of it); the last two stages issue nothing.
  // Two loops with branch-free bodies keep the accumulators in AGPRs across iterations.
  auto body = [&](int i, auto refill) {
    const int slot = i & 1;
    if (i + 1 < nmy)
      wait_vmcnt<G::NLOAD>();  // stage i landed, stage i + 1 may still fly
    else
      wait_vmcnt<0>();
    const char* st = ring + slot * G::SB;
    bf16x8 bw[U][NT], ba[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bw[u][nt] = *reinterpret_cast<const bf16x8*>(st + woff[nt][u]);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        ba[u][mt] = *reinterpret_cast<const bf16x8*>(st + G::WB + (mt * U + u) * 1024 + lane * 16);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // fragments in registers: the slot is free
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (decltype(refill)::value) issue(slot, wave + (i + 2) * WAVES);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ba[u][mt], bw[u][nt], acc[mt][nt], 0, 0, 0);
    if constexpr (decltype(refill)::value) {
      constexpr int PER = (U * MT * NT + G::NLOAD - 1) / G::NLOAD;
#pragma unroll
      for (int k = 0; k < G::NLOAD; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);    // one VMEM read (LDS-DMA piece)
        __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);  // then PER MFMAs
      }
    }
  };
  int i = 0;
  for (; i + 2 < nmy; ++i) body(i, std::true_type{});
  for (; i < nmy; ++i) body(i, std::false_type{});
  __syncthreads();  // every wave is done with its ring before the combine buffer aliases it
#pragma unroll
  for (int p = 0; p < SSP; ++p) {
    const int t = threadIdx.x + p * 64 * WAVES;
    if (rn_ss != nullptr && t < MT * 64) {  // published by the epilogue's first barrier
      float v = ss[p];
      v += __shfl_xor(v, 1, kWave);
      v += __shfl_xor(v, 2, kWave);
      if ((t & 3) == 0) s_inv[t >> 2] = rsqrtf(v * rn_inv_d + rn_eps);
    }
  }
  skinny_epilogue_rows<MT, NT, EPI, WAVES>(acc, reinterpret_cast<float*>(smem), rn_ss != nullptr ? s_inv : nullptr,
                                           partial, Y, ldy, M, N, ntile0, s, ex, grp);
}

// residual[m] <- bf16(residual[m] + sum_s partial[s][m]); out[m] <- rmsnorm(residual[m]) * w
// One workgroup per row, 256 threads x 8 columns per chunk (d <= 2048 * NC).  S = 0 is a plain
// RMSNorm of the residual.  out_stride < 0: out is written fragment-packed (act_index) as the next
// skinny GEMM's A operand.  out2 (optional): a second, fragment-packed copy (the MoE decode: the
// router reads the row-major form, the expert GEMMs the packed one - no separate pack pass).
template <int NC>
__global__ __launch_bounds__(256) void reduce_add_rmsnorm_kernel(bf16_t* __restrict__ out,
                                                                 bf16_t* __restrict__ residual,
                                                                 const float* __restrict__ partial, int S, int M,
                                                                 const bf16_t* __restrict__ w, int d, float eps,
                                                                 long out_stride, bf16_t* __restrict__ out2) {
  __shared__ float sred[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  bf16_t* rr = residual + (long)row * d;
  float v[NC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < d) {
      float acc[8];
      unpack8(*reinterpret_cast<const uint4*>(rr + idx), acc);
#pragma unroll 4
      for (int s = 0; s < S; ++s) {
        const float* p = partial + ((long)s * M + row) * d + idx;
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(p + 4);
        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
        acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
      }
      const uint4 q = pack8(acc);  // the residual stream is bf16 (HF semantics): round, then norm
      *reinterpret_cast<uint4*>(rr + idx) = q;
      unpack8(q, v[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
    }
  }
  const float inv = rsqrtf(block_sum<256>(ss, sred) / (float)d + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < d) {
      float wf[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(w + idx), wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[c][j] * inv * wf[j];
      const uint4 q = pack8(o);
      *reinterpret_cast<uint4*>(out + act_index(row, idx, out_stride)) = q;
      if (out2 != nullptr) *reinterpret_cast<uint4*>(out2 + act_index(row, idx, -(long)(d >> 5))) = q;
    }
  }
}

// Residual update with a deferred RMSNorm, fully parallel (grid (M, d/512), one wave per 512
// columns): residual <- bf16(residual + sum_s partial[s]); out <- bf16(residual * w) (packed via
// act_index); ss_part[m][chunk] <- sum of residual^2 over the chunk.  The consumer skinny GEMM
// applies 1/rms per row (rn_ss).  Replaces a one-workgroup-per-row norm pass, which is latency-
// bound at decode batch sizes (64 workgroups on 256 CUs).
// SC > 0: the slab count as a compile-time constant, so the residual, weight and every slab load
// are issued before the first wait (one memory round trip; with a runtime count hipcc waited for
// the residual before the slab loop and loaded the weight after the residual store: three).
template <int SC>
__global__ __launch_bounds__(64) void add_norm_partial_kernel(bf16_t* __restrict__ out, long out_stride,
                                                              bf16_t* __restrict__ residual,
                                                              const float* __restrict__ partial, int S, int M,
                                                              const bf16_t* __restrict__ w, int d,
                                                              float* __restrict__ ss_part) {
  const int row = blockIdx.x, chunk = blockIdx.y;
  const int col = chunk * 512 + threadIdx.x * 8;
  bf16_t* rr = residual + (long)row * d + col;
  const uint4 rv = *reinterpret_cast<const uint4*>(rr);
  const uint4 wv = *reinterpret_cast<const uint4*>(w + col);
  float acc[8];
  if constexpr (SC > 0) {
    f32x4 pa[SC], pb[SC];
#pragma unroll
    for (int s = 0; s < SC; ++s) {  // the slabs are read exactly once: non-temporal
      const float* p = partial + ((long)s * M + row) * d + col;
      pa[s] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
      pb[s] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 4));
    }
    unpack8(rv, acc);
#pragma unroll
    for (int s = 0; s < SC; ++s) {
      acc[0] += pa[s].x; acc[1] += pa[s].y; acc[2] += pa[s].z; acc[3] += pa[s].w;
      acc[4] += pb[s].x; acc[5] += pb[s].y; acc[6] += pb[s].z; acc[7] += pb[s].w;
    }
  } else {
    unpack8(rv, acc);
#pragma unroll 4
    for (int s = 0; s < S; ++s) {
      const float* p = partial + ((long)s * M + row) * d + col;
      const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
      const f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 4));
      acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
      acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
    }
  }
  const uint4 q = pack8(acc);
  float v[8], wf[8], o[8];
  unpack8(q, v);
  unpack8(wv, wf);
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ss += v[j] * v[j];
    o[j] = v[j] * wf[j];
  }
  // the normed output first: its weight operand is then waited for before any store is in flight
  *reinterpret_cast<uint4*>(out + act_index(row, col, out_stride)) = pack8(o);
  if (S > 0) *reinterpret_cast<uint4*>(rr) = q;
  ss = wave_sum(ss);
  if (threadIdx.x == 0) ss_part[row * (d / 512) + chunk] = ss;
}

// The decode step's front end in one launch (grid (M, d/512), one wave per 512 columns): the row's
// input id - prev[src[row]] when src[row] >= 0 (the token the previous, possibly still running,
// step sampled: pipelined decode), else ids[row] - its embedding row -> residual, and the first
// layer's deferred RMSNorm operands as add_norm_partial writes them (residual * w, packed via
// act_index; per-512-column sums of squares).  Replaces resolve_ids + embedding + add_norm_partial.
__global__ __launch_bounds__(64) void embed_norm_partial_kernel(bf16_t* __restrict__ out, long out_stride,
                                                                bf16_t* __restrict__ residual,
                                                                const int* __restrict__ ids,
                                                                const int* __restrict__ src,
                                                                const int* __restrict__ prev,
                                                                const bf16_t* __restrict__ emb, int vocab,
                                                                const bf16_t* __restrict__ w, int d,
                                                                float* __restrict__ ss_part) {
  const int row = blockIdx.x, chunk = blockIdx.y;
  const int col = chunk * 512 + threadIdx.x * 8;
  int id = ids[row];
  if (src != nullptr) {
    const int r = src[row];
    if (r >= 0) id = prev[r];
  }
  const bool in = id >= 0 && id < vocab;
  const uint4 ev = in ? *reinterpret_cast<const uint4*>(emb + (long)id * d + col) : make_uint4(0, 0, 0, 0);
  const uint4 wv = *reinterpret_cast<const uint4*>(w + col);
  *reinterpret_cast<uint4*>(residual + (long)row * d + col) = ev;
  float v[8], wf[8], o[8];
  unpack8(ev, v);
  unpack8(wv, wf);
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ss += v[j] * v[j];
    o[j] = v[j] * wf[j];
  }
  *reinterpret_cast<uint4*>(out + act_index(row, col, out_stride)) = pack8(o);
  ss = wave_sum(ss);
  if (threadIdx.x == 0) ss_part[row * (d / 512) + chunk] = ss;
}

// out[i] = bf16(sum_s partial[s][i]) over n elements (n % 8 == 0): the TP>1 decode tails sum
// the split-K slabs before the RCCL all-reduce.
__global__ __launch_bounds__(256) void reduce_slabs_kernel(bf16_t* __restrict__ out,
                                                           const float* __restrict__ partial, int S, long n) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= n) return;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    const float4 a = *reinterpret_cast<const float4*>(partial + s * n + i);
    const float4 b = *reinterpret_cast<const float4*>(partial + s * n + i + 4);
    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
    acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
  }
  *reinterpret_cast<uint4*>(out + i) = pack8(acc);
}

}  // namespace k8sllm

using namespace k8sllm;

extern "C" int k8sllm_add_norm_partial(void* out, long out_stride, void* residual, const float* partial, int S,
                                       int M, const void* w, int d, float* ss_part, hipStream_t s) {
  if (M <= 0) return 0;
  if (d % 512 != 0) return -1;
  const dim3 grid(M, d / 512), blk(64);
#define K8S_ANP(SCV)                                                                                         \
  hipLaunchKernelGGL((add_norm_partial_kernel<SCV>), grid, blk, 0, s, (bf16_t*)out, out_stride, (bf16_t*)residual, \
                     partial, S, M, (const bf16_t*)w, d, ss_part)
  switch (S) {
    case 1: K8S_ANP(1); break;
    case 2: K8S_ANP(2); break;
    case 3: K8S_ANP(3); break;
    case 4: K8S_ANP(4); break;
    case 8: K8S_ANP(8); break;
    default: K8S_ANP(0); break;
  }
#undef K8S_ANP
  return (int)hipGetLastError();
}

extern "C" int k8sllm_embed_norm_partial(void* out, long out_stride, void* residual, const int* ids, const int* src,
                                         const int* prev, const void* emb, int vocab, const void* w, int M, int d,
                                         float* ss_part, hipStream_t s) {
  if (M <= 0) return 0;
  if (d % 512 != 0) return -1;
  hipLaunchKernelGGL(embed_norm_partial_kernel, dim3(M, d / 512), dim3(64), 0, s, (bf16_t*)out, out_stride,
                     (bf16_t*)residual, ids, src, prev, (const bf16_t*)emb, vocab, (const bf16_t*)w, d, ss_part);
  return (int)hipGetLastError();
}

extern "C" int k8sllm_reduce_slabs(void* out, const float* partial, int S, long n, hipStream_t s) {
  if (n <= 0) return 0;
  if (n % 8 != 0 || S < 1) return -1;
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3((unsigned)((n / 8 + 255) / 256)), dim3(256), 0, s, (bf16_t*)out,
                     partial, S, n);
  return (int)hipGetLastError();
}

// kchunk: K split into `S` slices rounded up to whole wave groups (128 k) where that keeps the
// slice count, else to whole k-steps.
// `gran`: the smallest slice granule (32: one k-step; 64 for the row-major kernel's 64-deep stages).
static int skinny_kchunk(int K, int S, int gran = 32) {
  int kc = (K + S - 1) / S;
  const int kc128 = (kc + 127) / 128 * 128;
  if ((K + kc128 - 1) / kc128 == S) return kc128;
  return (kc + gran - 1) / gran * gran;
}

extern "C" int k8sllm_gemm_skinny_slabs(int K, int S) {
  const int kc = skinny_kchunk(K, S);
  return (K + kc - 1) / kc;
}

// epi: 0 slab, 1 bf16, 2 swiglu; nt_tiles: 2 or 4 n-tiles per workgroup; a_packed: A in the
// fragment-packed layout (lda ignored)
// splits <= 0: automatic split-K - the largest power of two that keeps the grid within one
// workgroup per CU, K slices >= 512 deep and whole 256-deep rounds of the 4 waves (uneven rounds
// leave waves idle at the tail).  Measured at M = 64 (tools/bench_skinny_waves.py,
// profiles/r01_s3_skinny_waves.jsonl): qkv S 2 14.9 us vs S 3 18.1 us; o / down S 4 beat 2, 3, 6
// and 8.  (A 128-column variant for 32 < M <= 64 measured 10-25 % slower and was removed.)
extern "C" int k8sllm_gemm_skinny_auto_splits(int M, int N, int K) {
  const int tiles = N / 64;
  int sp = 1;
  while (sp < 16 && (long)tiles * sp * 2 <= 256 && K / (sp * 2) >= 512 && K % (sp * 2 * 256) == 0) sp *= 2;
  return sp;
}

template <int MT, int NT, int EPI, int WAVES, typename... Args>
static void launch_rm(dim3 grid, dim3 blk, hipStream_t s, Args... args) {
  hipLaunchKernelGGL((gemm_skinny_rm_kernel<MT, NT, EPI, WAVES>), grid, blk, 0, s, args...);
}

// rn_ss (optional): per-row partial sums of squares [M][rn_nc] of the un-normalised A rows
// (add_norm_partial); outputs are scaled by rsqrt(sum / rn_d + eps) - the deferred RMSNorm.
static int skinny_launch(const void* A, long lda, const void* Wp, float* partial, void* Y, long ldy, int M, int N,
                         int K, int S, int epi, int nt_tiles, int a_packed, const float* rn_ss, int rn_nc, int rn_d,
                         float rn_eps, int waves, int experts, long w_es, long a_es, long y_es,
                         const float* row_w, int row_w_ld, int w_rm, hipStream_t s);

extern "C" int k8sllm_gemm_skinny(const void* A, long lda, const void* Wp, float* partial, void* Y, long ldy, int M,
                                  int N, int K, int S, int epi, int nt_tiles, int a_packed, const float* rn_ss,
                                  int rn_nc, int rn_d, float rn_eps, int waves, int experts, long w_es,
                                  long a_es, long y_es, const float* row_w, int row_w_ld, int w_rm, hipStream_t s) {
  return skinny_launch(A, lda, Wp, partial, Y, ldy, M, N, K, S, epi, nt_tiles, a_packed, rn_ss, rn_nc, rn_d, rn_eps,
                       waves, experts, w_es, a_es, y_es, row_w, row_w_ld, w_rm, s);
}

static int skinny_launch(const void* A, long lda, const void* Wp, float* partial, void* Y, long ldy, int M, int N,
                         int K, int S, int epi, int nt_tiles, int a_packed, const float* rn_ss, int rn_nc, int rn_d,
                         float rn_eps, int waves, int experts, long w_es, long a_es, long y_es,
                         const float* row_w, int row_w_ld, int w_rm, hipStream_t s) {
  if (M <= 0) return 0;
  if (experts < 1) return -5;
  const SkinnyGroup grp{w_es, a_es, y_es, row_w, row_w_ld};
  // 65..128 rows: grouped (expert) launches over row-major weights only - the EP all-to-all
  // decode's received rows (P x cap x top-k), so every local expert's weights stream ONCE per step
  // instead of once per 64-row chunk (2-wave workgroups: 8 m-tiles of A per stage)
  if (M > 64) {
    if (M > 128 || !w_rm || experts < 2 || !a_packed || K % 64 != 0 || N % 64 != 0 ||
        (epi != EPI_SLAB && epi != EPI_SWIGLU_PACKED))
      return -1;
    if (S <= 0) S = 1;
    const int kc8 = skinny_kchunk(K, S, 64);
    const int slabs8 = (K + kc8 - 1) / kc8;
    if (epi != EPI_SLAB && slabs8 != 1) return -3;
    const float inv_d8 = rn_d > 0 ? 1.f / (float)rn_d : 0.f;
    dim3 grid8(N / 64, slabs8, experts), blk8(128);
#define K8S_RM8(MTV, EPV)                                                                                                launch_rm<MTV, 4, EPV, 2>(grid8, blk8, s, (const bf16_t*)A, (const bf16_t*)Wp, (long)K, partial, (bf16_t*)Y, ldy,                               M, N, K, kc8, rn_ss, rn_nc, inv_d8, rn_eps, grp)
#define K8S_RM8_M(EPV)                  \
  switch ((M + 15) / 16) {              \
    case 5: K8S_RM8(5, EPV); break;     \
    case 6: K8S_RM8(6, EPV); break;     \
    case 7: K8S_RM8(7, EPV); break;     \
    default: K8S_RM8(8, EPV); break;    \
  }
    if (epi == EPI_SLAB) {
      K8S_RM8_M(EPI_SLAB)
    } else {
      K8S_RM8_M(EPI_SWIGLU_PACKED)
    }
#undef K8S_RM8_M
#undef K8S_RM8
    return (int)hipGetLastError();
  }
  if (K % 32 != 0 || (nt_tiles != 2 && nt_tiles != 4) || N % (16 * nt_tiles) != 0) return -1;
  if (S <= 0) S = epi == EPI_SLAB ? k8sllm_gemm_skinny_auto_splits(M, N, K) : 1;
  const int kc = skinny_kchunk(K, S, w_rm ? 64 : 32);
  if (w_rm) {
    if (!a_packed || K % 64 != 0 || N % 64 != 0) return -9;  // row-major W: packed A, 64-deep stages, NT = 4
    const int slabs_rm = (K + kc - 1) / kc;
    if (epi != EPI_SLAB && slabs_rm != 1) return -3;
    const float inv_d_rm = rn_d > 0 ? 1.f / (float)rn_d : 0.f;
    const int MT = (M + 15) / 16;
    // 4 waves per workgroup unless the grid then needs more than one round of workgroups: each
    // wave's ring holds two 16-KiB stages at M = 64, so LDS caps residency (4 waves: 1 workgroup
    // per CU at MT 2-4); 2-wave workgroups keep e.g. gate_up's 448 tiles co-resident.
    // waves = 2 or 4 forces one.
    static const int lds4[5] = {0, SkinnyRmGeom<1, 4, 0, 4>::LDS, SkinnyRmGeom<2, 4, 0, 4>::LDS,
                                SkinnyRmGeom<3, 4, 0, 4>::LDS, SkinnyRmGeom<4, 4, 0, 4>::LDS};
    // split-K slab projections whose 64-column grid leaves CUs idle (qkv: 96 tiles x 2 slices =
    // 192 workgroups) use 48-column tiles when that fills the chip (128 x 2 = 256).
    const bool nt3_ok = epi == EPI_SLAB && N % 48 == 0;
    const bool nt3 = nt3_ok && (long)(N / 64) * slabs_rm * experts < 224 && (long)(N / 48) * slabs_rm * experts <= 256;
    if (nt3) {
      dim3 grid3(N / 48, slabs_rm, experts), blk3(256);
#define K8S_RM3(MTV)                                                                                              \
  launch_rm<MTV, 3, EPI_SLAB, 4>(grid3, blk3, s, (const bf16_t*)A,            \
                     (const bf16_t*)Wp, (long)K, partial, (bf16_t*)Y, ldy, M, N, K, kc, rn_ss, rn_nc, inv_d_rm, rn_eps, \
                     grp)
      switch (MT) {
        case 1: K8S_RM3(1); break;
        case 2: K8S_RM3(2); break;
        case 3: K8S_RM3(3); break;
        default: K8S_RM3(4); break;
      }
#undef K8S_RM3
      return (int)hipGetLastError();
    }
    const long nwg = (long)(N / 64) * slabs_rm * experts;
    int rw = waves == 2 || waves == 4 ? waves : 4;
    if (waves != 2 && waves != 4 && nwg > 256L * (163840 / lds4[MT])) rw = 2;
    dim3 grid(N / 64, slabs_rm, experts), blk(64 * rw);
#define K8S_RM(MTV, EPV)                                                                                             \
  if (rw == 4)                                                                                                       \
    launch_rm<MTV, 4, EPV, 4>(grid, blk, s, (const bf16_t*)A, (const bf16_t*)Wp, \
                       (long)K, partial, (bf16_t*)Y, ldy, M, N, K, kc, rn_ss, rn_nc, inv_d_rm, rn_eps, grp);         \
  else                                                                                                               \
    launch_rm<MTV, 4, EPV, 2>(grid, blk, s, (const bf16_t*)A, (const bf16_t*)Wp, \
                       (long)K, partial, (bf16_t*)Y, ldy, M, N, K, kc, rn_ss, rn_nc, inv_d_rm, rn_eps, grp)
#define K8S_RM_M(EPV)                  \
  switch (MT) {                        \
    case 1: K8S_RM(1, EPV); break;     \
    case 2: K8S_RM(2, EPV); break;     \
    case 3: K8S_RM(3, EPV); break;     \
    default: K8S_RM(4, EPV); break;    \
  }
    switch (epi) {
      case EPI_SLAB: K8S_RM_M(EPI_SLAB) break;
      case EPI_BF16: K8S_RM_M(EPI_BF16) break;
      case EPI_SWIGLU: K8S_RM_M(EPI_SWIGLU) break;
      default: K8S_RM_M(EPI_SWIGLU_PACKED) break;
    }
#undef K8S_RM_M
#undef K8S_RM
    return (int)hipGetLastError();
  }
  const int slabs = (K + kc - 1) / kc;
  if (epi != EPI_SLAB && slabs != 1) return -3;
  if ((epi == EPI_SWIGLU || epi == EPI_SWIGLU_PACKED) && nt_tiles != 4) return -4;
  const float inv_d = rn_d > 0 ? 1.f / (float)rn_d : 0.f;
  // 8-wave workgroups: twice the weight lines in flight per CU for the same K slice.  waves <= 0
  // (auto): 8 for the split-K slab projections (o 11.1 vs 11.8 us, down 24.3 vs 25.9 at M = 64),
  // 4 for the single-slice SwiGLU / bf16 epilogues (gate_up 47.5 vs 50.5 us).
  const int nwaves = waves == 8 || (waves <= 0 && epi == EPI_SLAB) ? 8 : 4;
  dim3 grid(N / (16 * nt_tiles), slabs, experts), blk(64 * nwaves);
  const int MT = (M + 15) / 16;
#define K8S_SK(MTV, NTV, EPV, APKV, WV)                                                                        \
  hipLaunchKernelGGL((gemm_skinny_kernel<MTV, NTV, EPV, APKV, WV>), grid, blk, 0, s, (const bf16_t*)A, lda,   \
                     (const bf16_t*)Wp, partial, (bf16_t*)Y, ldy, M, N, K, kc, rn_ss, rn_nc, inv_d, rn_eps, grp)
#define K8S_SK_W(MTV, NTV, EPV, NTLV)                                       \
  if (nwaves == 8) { K8S_SK(MTV, NTV, EPV, NTLV, 8); }                      \
  else { K8S_SK(MTV, NTV, EPV, NTLV, 4); }
#define K8S_SK_M(NTV, EPV, NTLV)                   \
  switch (MT) {                                    \
    case 1: K8S_SK_W(1, NTV, EPV, NTLV); break;     \
    case 2: K8S_SK_W(2, NTV, EPV, NTLV); break;     \
    case 3: K8S_SK_W(3, NTV, EPV, NTLV); break;     \
    default: K8S_SK_W(4, NTV, EPV, NTLV); break;    \
  }
#define K8S_SK_NTL(NTV, EPV)  \
  if (a_packed) {             \
    K8S_SK_M(NTV, EPV, true)  \
  } else {                    \
    K8S_SK_M(NTV, EPV, false) \
  }
  if (epi == EPI_SWIGLU) {
    K8S_SK_NTL(4, EPI_SWIGLU)
  } else if (epi == EPI_SWIGLU_PACKED) {
    K8S_SK_NTL(4, EPI_SWIGLU_PACKED)
  } else if (epi == EPI_BF16) {
    if (nt_tiles == 4) { K8S_SK_NTL(4, EPI_BF16) } else { K8S_SK_NTL(2, EPI_BF16) }
  } else {
    if (nt_tiles == 4) { K8S_SK_NTL(4, EPI_SLAB) } else { K8S_SK_NTL(2, EPI_SLAB) }
  }
#undef K8S_SK_NTL
#undef K8S_SK_M
#undef K8S_SK_W
#undef K8S_SK
  return (int)hipGetLastError();
}

extern "C" int k8sllm_reduce_add_rmsnorm(void* out, void* residual, const float* partial, int S, int M,
                                         const void* w, int d, float eps, long out_stride, void* out2,
                                         hipStream_t s) {
  if (M <= 0) return 0;
  if (d % 8 != 0 || d > 256 * 8 * 4) return -1;
  const int nc = (d + 2047) / 2048;
#define K8S_RAR(NC)                                                                                           \
  hipLaunchKernelGGL((reduce_add_rmsnorm_kernel<NC>), dim3(M), dim3(256), 0, s, (bf16_t*)out,                 \
                     (bf16_t*)residual, partial, S, M, (const bf16_t*)w, d, eps, out_stride, (bf16_t*)out2)
  if (nc <= 1) K8S_RAR(1);
  else if (nc <= 2) K8S_RAR(2);
  else K8S_RAR(4);
#undef K8S_RAR
  return (int)hipGetLastError();
}
