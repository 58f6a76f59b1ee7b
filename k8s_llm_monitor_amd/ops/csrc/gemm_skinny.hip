// Decode-time "skinny" GEMM on gfx950 MFMA: Y[M, N] = A[M, K] . W[N, K]^T for M <= 64 rows (the
// decode batch), bf16 in, fp32 accumulate.  Every decode projection of a dense Llama layer runs
// here (qkv, o, gate_up, down); prefill keeps hipBLASLt on the row-major copy of the weights.
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
#include "common.h"

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

template <int MT, int NT, int EPI, bool APK, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void gemm_skinny_kernel(const bf16_t* __restrict__ A, long lda,
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
  __shared__ float s_inv[MT * 16];
  if (rn_ss != nullptr && threadIdx.x < MT * 16) {
    const int row = min((int)threadIdx.x, M - 1);
    float ss = 0.f;
    for (int c = 0; c < rn_nc; ++c) ss += rn_ss[row * rn_nc + c];
    s_inv[threadIdx.x] = rsqrtf(ss * rn_inv_d + rn_eps);
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

  // cross-wave combine, one m-tile per round (keeps LDS at 16 KiB so occupancy is VGPR-bound).
  // C/D layout of the 16x16 tile: col = lane & 15, rows (lane >> 4) * 4 + r
  constexpr int NOUT = EPI == EPI_SWIGLU || EPI == EPI_SWIGLU_PACKED ? NT / 2 : NT;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    if (mt > 0) __syncthreads();  // previous round's reads done
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) *reinterpret_cast<f32x4*>(&red[wave][nt][lane][0]) = acc[mt][nt];
    __syncthreads();
    for (int idx = threadIdx.x; idx < NOUT * 64; idx += 64 * WAVES) {
      const int nt = idx >> 6, l = idx & 63;
      f32x4 v = *reinterpret_cast<const f32x4*>(&red[0][nt][l][0]);
#pragma unroll
      for (int w = 1; w < WAVES; ++w) v += *reinterpret_cast<const f32x4*>(&red[w][nt][l][0]);
      // deferred RMSNorm of the A rows (add_norm_partial): A held x * w, the row's 1/rms
      // (s_inv, computed at kernel start) is applied here - linear, so exact for split-K slabs too
      f32x4 rs = f32x4{1.f, 1.f, 1.f, 1.f};
      if (rn_ss != nullptr) {
#pragma unroll
        for (int r = 0; r < 4; ++r) rs[r] = s_inv[mt * 16 + (l >> 4) * 4 + r];
      }
      v *= rs;
      if constexpr (EPI == EPI_SWIGLU || EPI == EPI_SWIGLU_PACKED) {
        f32x4 u = *reinterpret_cast<const f32x4*>(&red[0][nt + NT / 2][l][0]);
#pragma unroll
        for (int w = 1; w < WAVES; ++w) u += *reinterpret_cast<const f32x4*>(&red[w][nt + NT / 2][l][0]);
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
      } else {
        const int col = (ntile0 + nt) * 16 + (l & 15);
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

// residual[m] <- bf16(residual[m] + sum_s partial[s][m]); out[m] <- rmsnorm(residual[m]) * w
// One workgroup per row, 256 threads x 8 columns per chunk (d <= 2048 * NC).  S = 0 is a plain
// RMSNorm of the residual.  out_stride < 0: out is written fragment-packed (act_index) as the next
// skinny GEMM's A operand.
template <int NC>
__global__ __launch_bounds__(256) void reduce_add_rmsnorm_kernel(bf16_t* __restrict__ out,
                                                                 bf16_t* __restrict__ residual,
                                                                 const float* __restrict__ partial, int S, int M,
                                                                 const bf16_t* __restrict__ w, int d, float eps,
                                                                 long out_stride) {
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
      *reinterpret_cast<uint4*>(out + act_index(row, idx, out_stride)) = pack8(o);
    }
  }
}

// Wide variant for 32 < M <= 64 (A fragment-packed): the 4 waves own the 4 m-tiles, a workgroup
// covers 128 output columns (8 n-tiles) of one K slice, and the weight tile is staged through LDS
// once and shared by the waves.  Compared with the narrow kernel (waves split K, 64 columns), the
// activation bytes read per weight byte halve (64 rows / 128 columns), every A fragment is read by
// exactly one wave, and the epilogue needs no cross-wave reduction.  Register-staged double
// buffer: group g+1's weight and activation loads are in flight while group g is multiplied.
// Measured on MI355X (tools/bench_skinny.py, M 33-64, Llama-3-8B shapes): 10-25 % SLOWER than the
// narrow kernel - one 16 KiB group in flight per workgroup plus a barrier per group cost more than
// the halved activation traffic saves - so it is opt-in (K8SLLM_SKINNY_WIDE=1), kept as the
// starting point for an LDS-DMA ring version.
template <int EPI>
__global__ __launch_bounds__(256) void gemm_skinny_wide_kernel(const bf16_t* __restrict__ A,
                                                               const bf16_t* __restrict__ Wp,
                                                               float* __restrict__ partial, bf16_t* __restrict__ Y,
                                                               long ldy, int M, int N, int K, int kchunk,
                                                               const float* __restrict__ rn_ss, int rn_nc,
                                                               float rn_inv_d, float rn_eps) {
  constexpr int NT = 8, U = 2;
  constexpr int WPW = U * NT / 4;  // 1 KiB weight blocks staged per wave per group
  __shared__ __attribute__((aligned(16))) u32x4 sW[2][U * NT][64];
  __shared__ float s_inv[64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile0 = blockIdx.x * NT;
  const int s = blockIdx.y;
  const int kbeg = s * kchunk;
  const int nsteps = (min(K, kbeg + kchunk) - kbeg) >> 5;
  const int ksteps = K >> 5;
  const int MT = (M + 15) >> 4;
  const bool active = wave < MT;

  if (rn_ss != nullptr && threadIdx.x < 64) {
    const int row = min((int)threadIdx.x, M - 1);
    float ss = 0.f;
    for (int c = 0; c < rn_nc; ++c) ss += rn_ss[row * rn_nc + c];
    s_inv[threadIdx.x] = rsqrtf(ss * rn_inv_d + rn_eps);
  }

  const u32x4* wbase = reinterpret_cast<const u32x4*>(Wp) + (long)(kbeg >> 5) * 64 + lane;
  const bf16x8* abase = reinterpret_cast<const bf16x8*>(A) + ((long)min(wave, MT - 1) * ksteps + (kbeg >> 5)) * 64 +
                        lane;
  auto load_w = [&](u32x4* r, int g) {
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int idx = wave * WPW + j, u = idx / NT, nt = idx % NT;
      const int st = min(g * U + u, nsteps - 1);
      r[j] = __builtin_nontemporal_load(wbase + ((long)(tile0 + nt) * ksteps + st) * 64);
    }
  };
  auto load_a = [&](bf16x8* r, int g) {
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = abase[(long)min(g * U + u, nsteps - 1) * 64];
  };

  f32x4 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ngroups = (nsteps + U - 1) / U;
  u32x4 wr[WPW];
  bf16x8 ar[U], ac[U];
  load_w(wr, 0);
  load_a(ar, 0);
  for (int g = 0; g < ngroups; ++g) {
    const int buf = g & 1;
#pragma unroll
    for (int j = 0; j < WPW; ++j) sW[buf][wave * WPW + j][lane] = wr[j];
#pragma unroll
    for (int u = 0; u < U; ++u) ac[u] = ar[u];
    if (g + 1 < ngroups) {
      load_w(wr, g + 1);
      load_a(ar, g + 1);
    }
    __syncthreads();  // group g staged by every wave (and group g-1's reads of this buffer done)
    if (active) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (g * U + u < nsteps) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ac[u], __builtin_bit_cast(bf16x8, sW[buf][u * NT + nt][lane]),
                                                              acc[nt], 0, 0, 0);
        }
      }
    }
  }
  if (!active) return;
  f32x4 rs = f32x4{1.f, 1.f, 1.f, 1.f};
  if (rn_ss != nullptr) {
#pragma unroll
    for (int r = 0; r < 4; ++r) rs[r] = s_inv[wave * 16 + (lane >> 4) * 4 + r];
  }
  if constexpr (EPI == EPI_SWIGLU || EPI == EPI_SWIGLU_PACKED) {
#pragma unroll
    for (int nt = 0; nt < NT / 2; ++nt) {
      const f32x4 gv = acc[nt] * rs, uv = acc[nt + NT / 2] * rs;
      const int f = blockIdx.x * 64 + nt * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wave * 16 + (lane >> 4) * 4 + r;
        const float g = bf2f(f2bf(gv[r]));
        const float uu = bf2f(f2bf(uv[r]));
        const bf16_t o = f2bf(g * uu / (1.f + __expf(-g)));
        if constexpr (EPI == EPI_SWIGLU_PACKED) {
          const int F = N >> 1;
          Y[(((long)wave * (F >> 5) + (f >> 5)) * 64 + ((f >> 3) & 3) * 16 + (row & 15)) * 8 + (f & 7)] = o;
        } else if (row < M) {
          Y[(long)row * ldy + f] = o;
        }
      }
    }
  } else {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const f32x4 v = acc[nt] * rs;
      const int col = (tile0 + nt) * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wave * 16 + (lane >> 4) * 4 + r;
        if (row < M) {
          if constexpr (EPI == EPI_BF16)
            Y[(long)row * ldy + col] = f2bf(v[r]);
          else
            partial[((long)s * M + row) * N + col] = v[r];
        }
      }
    }
  }
}

// Residual update with a deferred RMSNorm, fully parallel (grid (M, d/512), one wave per 512
// columns): residual <- bf16(residual + sum_s partial[s]); out <- bf16(residual * w) (packed via
// act_index); ss_part[m][chunk] <- sum of residual^2 over the chunk.  The consumer skinny GEMM
// applies 1/rms per row (rn_ss).  Replaces a one-workgroup-per-row norm pass, which is latency-
// bound at decode batch sizes (64 workgroups on 256 CUs).
__global__ __launch_bounds__(64) void add_norm_partial_kernel(bf16_t* __restrict__ out, long out_stride,
                                                              bf16_t* __restrict__ residual,
                                                              const float* __restrict__ partial, int S, int M,
                                                              const bf16_t* __restrict__ w, int d,
                                                              float* __restrict__ ss_part) {
  const int row = blockIdx.x, chunk = blockIdx.y;
  const int col = chunk * 512 + threadIdx.x * 8;
  bf16_t* rr = residual + (long)row * d + col;
  float acc[8];
  unpack8(*reinterpret_cast<const uint4*>(rr), acc);
#pragma unroll 4
  for (int s = 0; s < S; ++s) {
    const float* p = partial + ((long)s * M + row) * d + col;
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
    acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
  }
  const uint4 q = pack8(acc);
  if (S > 0) *reinterpret_cast<uint4*>(rr) = q;
  float v[8], wf[8], o[8];
  unpack8(q, v);
  unpack8(*reinterpret_cast<const uint4*>(w + col), wf);
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
  hipLaunchKernelGGL(add_norm_partial_kernel, dim3(M, d / 512), dim3(64), 0, s, (bf16_t*)out, out_stride,
                     (bf16_t*)residual, partial, S, M, (const bf16_t*)w, d, ss_part);
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
static int skinny_kchunk(int K, int S) {
  int kc = (K + S - 1) / S;
  const int kc128 = (kc + 127) / 128 * 128;
  if ((K + kc128 - 1) / kc128 == S) return kc128;
  return (kc + 31) / 32 * 32;
}

extern "C" int k8sllm_gemm_skinny_slabs(int K, int S) {
  const int kc = skinny_kchunk(K, S);
  return (K + kc - 1) / kc;
}

// epi: 0 slab, 1 bf16, 2 swiglu; nt_tiles: 2 or 4 n-tiles per workgroup; a_packed: A in the
// fragment-packed layout (lda ignored)
// Kernel choice: the wide kernel for fragment-packed A with 32 < M <= 64 and N % 128 == 0
// (unless disabled), else the narrow one.  splits <= 0: automatic split-K - the largest power of
// two that keeps the grid within one workgroup per CU, K slices >= 512 deep and whole 256-deep
// rounds of the 4 waves (uneven rounds leave waves idle at the tail).  Measured at M = 64
// (tools/bench_skinny_waves.py, profiles/r01_s3_skinny_waves.jsonl): qkv S 2 14.9 us vs S 3
// 18.1 us; o / down S 4 beat 2, 3, 6 and 8.
static bool skinny_use_wide(int M, int N, int a_packed, int wide) {
  return wide && a_packed && M > 32 && N % 128 == 0;
}

extern "C" int k8sllm_gemm_skinny_auto_splits(int M, int N, int K, int a_packed, int wide) {
  const int tiles = N / (skinny_use_wide(M, N, a_packed, wide) ? 128 : 64);
  int sp = 1;
  while (sp < 16 && (long)tiles * sp * 2 <= 256 && K / (sp * 2) >= 512 && K % (sp * 2 * 256) == 0) sp *= 2;
  return sp;
}

// rn_ss (optional): per-row partial sums of squares [M][rn_nc] of the un-normalised A rows
// (add_norm_partial); outputs are scaled by rsqrt(sum / rn_d + eps) - the deferred RMSNorm.
extern "C" int k8sllm_gemm_skinny(const void* A, long lda, const void* Wp, float* partial, void* Y, long ldy, int M,
                                  int N, int K, int S, int epi, int nt_tiles, int a_packed, const float* rn_ss,
                                  int rn_nc, int rn_d, float rn_eps, int wide, int waves, int experts, long w_es,
                                  long a_es, long y_es, const float* row_w, int row_w_ld, hipStream_t s) {
  if (M <= 0) return 0;
  if (experts < 1) return -5;
  if (experts > 1) wide = 0;  // grouped launches use the narrow kernel
  const SkinnyGroup grp{w_es, a_es, y_es, row_w, row_w_ld};
  if (M > 64 || K % 32 != 0 || (nt_tiles != 2 && nt_tiles != 4) || N % (16 * nt_tiles) != 0) return -1;
  if (S <= 0) S = epi == EPI_SLAB ? k8sllm_gemm_skinny_auto_splits(M, N, K, a_packed, wide) : 1;
  const int kc = skinny_kchunk(K, S);
  const int slabs = (K + kc - 1) / kc;
  if (epi != EPI_SLAB && slabs != 1) return -3;
  if ((epi == EPI_SWIGLU || epi == EPI_SWIGLU_PACKED) && nt_tiles != 4) return -4;
  const float inv_d = rn_d > 0 ? 1.f / (float)rn_d : 0.f;
  if (skinny_use_wide(M, N, a_packed, wide)) {
    dim3 grid(N / 128, slabs), blk(256);
#define K8S_WIDE(EPV)                                                                                      \
  hipLaunchKernelGGL((gemm_skinny_wide_kernel<EPV>), grid, blk, 0, s, (const bf16_t*)A, (const bf16_t*)Wp, \
                     partial, (bf16_t*)Y, ldy, M, N, K, kc, rn_ss, rn_nc, inv_d, rn_eps)
    switch (epi) {
      case EPI_SLAB: K8S_WIDE(EPI_SLAB); break;
      case EPI_BF16: K8S_WIDE(EPI_BF16); break;
      case EPI_SWIGLU: K8S_WIDE(EPI_SWIGLU); break;
      default: K8S_WIDE(EPI_SWIGLU_PACKED); break;
    }
#undef K8S_WIDE
    return (int)hipGetLastError();
  }
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
                                         const void* w, int d, float eps, long out_stride, hipStream_t s) {
  if (M <= 0) return 0;
  if (d % 8 != 0 || d > 256 * 8 * 4) return -1;
  const int nc = (d + 2047) / 2048;
#define K8S_RAR(NC)                                                                                           \
  hipLaunchKernelGGL((reduce_add_rmsnorm_kernel<NC>), dim3(M), dim3(256), 0, s, (bf16_t*)out,                 \
                     (bf16_t*)residual, partial, S, M, (const bf16_t*)w, d, eps, out_stride)
  if (nc <= 1) K8S_RAR(1);
  else if (nc <= 2) K8S_RAR(2);
  else K8S_RAR(4);
#undef K8S_RAR
  return (int)hipGetLastError();
}
