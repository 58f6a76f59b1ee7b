// Decode-time GEMM, second design ("W stream, shared A"): Y[M, N] = A[M, K] . W[N, K]^T for
// M <= 64 rows, bf16 in, fp32 accumulate, gfx950 v_mfma_f32_16x16x32_bf16.
//
// Why a second kernel.  gemm_skinny_rm_kernel (gemm_skinny.hip) stages BOTH operands by LDS-DMA,
// and at M = 64 every 64-column workgroup re-reads all 64 A rows - as many bytes as its weight
// slab.  The round-2 PMC reading (profiles/r02/README.md "Why the row-major skinny GEMM loses
// weight bandwidth") put the vector-memory path at 84-88 % busy moving ~16 B/cycle/CU of W + A,
// half of it A, and the decode GEMMs at 3.4-4.8 TB/s against 5.9-6.2 at M = 1.  Here:
//   * W is a decode-only fragment-packed copy [N/16][K/32][64][8] (pack_skinny): every wave
//     instruction is 1 KiB contiguous straight into MFMA operand registers (global_load_dwordx4,
//     non-temporal: read once per step), no LDS round trip, and each wave keeps DEPTH k-steps of
//     its weight stream in flight in a register ring;
//   * A (fragment-packed activations) is loaded ONCE per workgroup per K chunk into LDS (register
//     staged: global_load -> ds_write_b128, a 2-slot ring, one barrier per chunk) and read by
//     every wave - the waves split the workgroup's COLUMNS, not K, so A bytes per weight byte are
//     MT / (n-tiles per workgroup) instead of MT / 4;
//   * the grid is sized to the chip: n-tiles per workgroup x split-K chosen so the workgroup count
//     is ~256 (one per CU, every CU the same weight bytes; e.g. gate_up: 1792 n-tiles / 7 = 256);
//   * no cross-wave combine: each wave owns whole-K sums of its columns.
// Epilogues: SLAB (fp32 split-K partials [S][M][N] for the next kernel's reduce, as the skinny
// kernels), BF16 (the LM head), SWIGLU8 (gate_up with the weight rows interleaved per 16-row
// n-tile as [8 gate | 8 up]: the pair sits in lanes l and l ^ 8 of the same accumulator, so the
// epilogue is one lane swap; output fragment-packed as the down projection's A operand).
#include <type_traits>

#include "common.h"

namespace k8sllm {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

enum { DEC_SLAB = 0, DEC_BF16 = 1, DEC_SWIGLU8 = 2 };

constexpr int kDecCH = 8;  // k-steps (32 deep) per A chunk

template <int MT, int WAVES>
struct DecGeom {
  static constexpr int SLOT = kDecCH * MT * 1024;                   // bytes of one A chunk
  static constexpr int PIECES = kDecCH * MT * 64;                   // 16-B pieces per chunk
  static constexpr int NLD = (PIECES + 64 * WAVES - 1) / (64 * WAVES);  // staging loads per thread
};

template <int MT, int NTW, int WAVES, int EPI, int DEPTH>
__global__ __launch_bounds__(64 * WAVES, 1) void gemm_dec_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ W, float* __restrict__ partial,
    bf16_t* __restrict__ Y, long ldy, int M, int N, int K, int kchunk, const float* __restrict__ rn_ss, int rn_nc,
    float rn_inv_d, float rn_eps) {
  using G = DecGeom<MT, WAVES>;
  constexpr int ITER = DEPTH > kDecCH ? DEPTH : kDecCH;  // k-steps per unrolled main-loop iteration
  __shared__ __attribute__((aligned(16))) char sA[2 * G::SLOT];
  __shared__ float s_inv[MT * 16];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ksteps = K >> 5;
  const int kb = blockIdx.y * (kchunk >> 5);  // first k-step of this workgroup's K slice
  const int nsteps = kchunk >> 5;             // host: kchunk | K, (kchunk / 32) % ITER == 0
  const int niter = nsteps / ITER;
  const int tile0 = (blockIdx.x * WAVES + wave) * NTW;  // this wave's first n-tile

  // ---- A chunks: register-staged, 2 LDS slots
  u32x4 stg[G::NLD];
  auto stage_load = [&](int c) {
#pragma unroll
    for (int i = 0; i < G::NLD; ++i) {
      // threads past the chunk (waves that do not divide it) repeat its last piece: every load
      // unconditional, so the counted vmcnt waits stay exact
      const int p = min(threadIdx.x + i * 64 * WAVES, G::PIECES - 1);
      {
        const int mt = p / (kDecCH * 64), j = (p >> 6) % kDecCH, ln = p & 63;
        stg[i] = *reinterpret_cast<const u32x4*>(A + (((long)mt * ksteps + kb + c * kDecCH + j) * 64 + ln) * 8);
      }
    }
  };
  auto stage_store = [&](int c) {
    char* slot = sA + (c & 1) * G::SLOT;
#pragma unroll
    for (int i = 0; i < G::NLD; ++i) {
      const int p = min(threadIdx.x + i * 64 * WAVES, G::PIECES - 1);
      *reinterpret_cast<u32x4*>(slot + p * 16) = stg[i];
    }
  };

  // chunk 0's staging loads go out BEFORE the weight ring's first loads: at the loop head the
  // staging registers are then the oldest loads in flight on both entry paths (prologue and back
  // edge), so the counted vmcnt there leaves the weight ring in flight (with the staging loads
  // last, the merged wait drained the ring at every chunk boundary).
  stage_load(0);
  // ---- weight stream: DEPTH k-steps x NTW fragments in flight per wave
  const u32x4* wp[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
    wp[t] = reinterpret_cast<const u32x4*>(W) + ((long)min(tile0 + t, (N >> 4) - 1) * ksteps + kb) * 64 + lane;
  u32x4 wr[DEPTH][NTW];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
#pragma unroll
    for (int t = 0; t < NTW; ++t) wr[d][t] = __builtin_nontemporal_load(wp[t] + d * 64);

  // ---- deferred RMSNorm: 1/rms of each A row from its partial sums of squares
  if (rn_ss != nullptr && threadIdx.x < MT * 64) {
    const int rl = threadIdx.x >> 2, part = threadIdx.x & 3;
    const int row = min(rl, M - 1);
    float ss = 0.f;
    for (int c = part; c < rn_nc; c += 4) ss += rn_ss[row * rn_nc + c];
    ss += __shfl_xor(ss, 1, kWave);
    ss += __shfl_xor(ss, 2, kWave);
    if (part == 0) s_inv[rl] = rsqrtf(ss * rn_inv_d + rn_eps);
  }

  f32x4 acc[MT][NTW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = nsteps / kDecCH;
  auto read_a = [&](bf16x8 (&af)[MT], int ks) {
    const char* slot = sA + ((ks / kDecCH) & 1) * G::SLOT + (ks % kDecCH) * 1024 + lane * 16;
#pragma unroll
    for (int m = 0; m < MT; ++m) af[m] = *reinterpret_cast<const bf16x8*>(slot + m * kDecCH * 1024);
  };
  // One unrolled iteration = ITER k-steps (a whole number of A chunks and of W ring turns).
  // Program order is pinned per k-step (sched_barrier): vmcnt retires in issue order, so a weight
  // load the scheduler sinks below the next chunk's staging loads would be drained at the next
  // chunk boundary and the ring would hold nothing across it.  Per k-step: the next step's A
  // fragments are read from LDS (one step of LDS latency hidden), the MFMAs consume ring slot
  // j % DEPTH, and the slot is refilled with k-step ks + DEPTH.  LAST: the final iteration issues
  // no weight loads past the slice.
  bf16x8 af[MT], an[MT];
  auto iteration = [&](int it, auto last) {
    constexpr bool LAST = decltype(last)::value;
#pragma unroll
    for (int j = 0; j < ITER; ++j) {
      const int ks = it * ITER + j;
      if (j % kDecCH == 0) {  // chunk boundary: publish chunk c, start loading chunk c + 1
        const int c = ks / kDecCH;
        stage_store(c);
        __syncthreads();
        if (c + 1 < nchunks) stage_load(c + 1);
        read_a(af, ks);
        __builtin_amdgcn_sched_barrier(0);
      } else {
#pragma unroll
        for (int m = 0; m < MT; ++m) af[m] = an[m];
      }
      if ((j + 1) % kDecCH != 0) read_a(an, ks + 1);
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, wr[j % DEPTH][t]);
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], b, acc[m][t], 0, 0, 0);
      }
      if (!LAST || j + DEPTH < ITER) {
#pragma unroll
        for (int t = 0; t < NTW; ++t) wr[j % DEPTH][t] = __builtin_nontemporal_load(wp[t] + (ks + DEPTH) * 64);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  int it = 0;
  for (; it + 1 < niter; ++it) iteration(it, std::false_type{});
  iteration(it, std::true_type{});

  // ---- epilogue.  C layout of a 16x16 tile: col = lane & 15, rows (lane >> 4) * 4 + r.
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    float rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) rs[r] = rn_ss != nullptr ? s_inv[m * 16 + (lane >> 4) * 4 + r] : 1.f;
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      const int tile = tile0 + t;
      if (tile >= (N >> 4)) continue;  // the last workgroup of a grid that does not divide N
      if constexpr (EPI == DEC_SWIGLU8) {
        // n-tile rows [8 gate | 8 up] of features 8 tile .. 8 tile + 7: lane l (l & 8 == 0) holds
        // the gate of feature 8 tile + (l & 7), lane l ^ 8 the matching up
        const int F = N >> 1;
        const int f = tile * 8 + (lane & 7);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[m][t][r] * rs[r];
          const float o = __shfl_xor(v, 8, kWave);
          const int row = m * 16 + (lane >> 4) * 4 + r;
          if ((lane & 8) == 0) {
            // gate and up rounded to bf16 first, as the unfused GEMM -> silu_mul does
            const float g = bf2f(f2bf(v)), u = bf2f(f2bf(o));
            Y[(((long)(row >> 4) * (F >> 5) + (f >> 5)) * 64 + ((f >> 3) & 3) * 16 + (row & 15)) * 8 + (f & 7)] =
                f2bf(g * u / (1.f + __expf(-g)));
          }
        }
      } else {
        const int col = tile * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m * 16 + (lane >> 4) * 4 + r;
          if (row < M) {
            const float v = acc[m][t][r] * rs[r];
            if constexpr (EPI == DEC_BF16)
              Y[(long)row * ldy + col] = f2bf(v);
            else
              partial[((long)blockIdx.y * M + row) * N + col] = v;
          }
        }
      }
    }
  }
}

}  // namespace k8sllm

using namespace k8sllm;

// Weight layout for DEC_SWIGLU8: fragment-packed over rows interleaved per 16-row n-tile as
// [8 gate | 8 up] (ops.interleave_gate_up8).  ntw x waves n-tiles per workgroup; grid
// (ceil((N / 16) / (ntw * waves)), splits) - the last workgroup may hold fewer n-tiles.  depth: weight k-steps in flight per wave.
// Returns 0, or a negative code when the shape / configuration is not supported (the caller then
// uses gemm_skinny).
extern "C" int k8sllm_gemm_dec(const void* A, const void* Wp, float* partial, void* Y, long ldy, int M, int N, int K,
                               int splits, int epi, int ntw, int waves, int depth, const float* rn_ss, int rn_nc,
                               int rn_d, float rn_eps, hipStream_t s) {
  if (M <= 0) return 0;
  if (M > 64 || N % 16 || K % 32 || splits < 1 || K % splits) return -1;
  const int ntiles = N / 16, nwg_tiles = ntw * waves;
  const int kchunk = K / splits;
  const int iter = depth > kDecCH ? depth : kDecCH;
  if (kchunk % 32 || kchunk < 32 * iter || (kchunk / 32) % iter) return -3;
  if (epi != DEC_SLAB && splits != 1) return -4;
  const float inv_d = rn_d > 0 ? 1.f / (float)rn_d : 0.f;
  const int MT = (M + 15) / 16;
  const dim3 grid((ntiles + nwg_tiles - 1) / nwg_tiles, splits), blk(64 * waves);
  int rc = -5;
#define K8S_DEC(MTV, NTWV, WV, EPV, DV)                                                                              \
  hipLaunchKernelGGL((gemm_dec_kernel<MTV, NTWV, WV, EPV, DV>), grid, blk, 0, s, (const bf16_t*)A, (const bf16_t*)Wp, \
                     partial, (bf16_t*)Y, ldy, M, N, K, kchunk, rn_ss, rn_nc, inv_d, rn_eps);                        \
  rc = 0
#define K8S_DEC_M(NTWV, WV, EPV, DV) \
  switch (MT) {                      \
    case 1: K8S_DEC(1, NTWV, WV, EPV, DV); break; \
    case 2: K8S_DEC(2, NTWV, WV, EPV, DV); break; \
    case 3: K8S_DEC(3, NTWV, WV, EPV, DV); break; \
    default: K8S_DEC(4, NTWV, WV, EPV, DV); break; \
  }
  // configurations (ntw, waves, depth) per epilogue: the ones the launcher's table picks plus
  // the sweep neighbours of tools/bench_decode_gemm.py
  if (epi == DEC_SLAB) {
    if (ntw == 1 && waves == 4 && depth == 16) { K8S_DEC_M(1, 4, DEC_SLAB, 16) }
    else if (ntw == 1 && waves == 8 && depth == 8) { K8S_DEC_M(1, 8, DEC_SLAB, 8) }
    else if (ntw == 2 && waves == 4 && depth == 8) { K8S_DEC_M(2, 4, DEC_SLAB, 8) }
    else if (ntw == 2 && waves == 8 && depth == 8) { K8S_DEC_M(2, 8, DEC_SLAB, 8) }
    else if (ntw == 3 && waves == 4 && depth == 8) { K8S_DEC_M(3, 4, DEC_SLAB, 8) }
    else if (ntw == 4 && waves == 4 && depth == 4) { K8S_DEC_M(4, 4, DEC_SLAB, 4) }
    else if (ntw == 4 && waves == 4 && depth == 8) { K8S_DEC_M(4, 4, DEC_SLAB, 8) }
    else if (ntw == 3 && waves == 8 && depth == 8) { K8S_DEC_M(3, 8, DEC_SLAB, 8) }
    else if (ntw == 1 && waves == 4 && depth == 8) { K8S_DEC_M(1, 4, DEC_SLAB, 8) }
    // qkv at 4 splits: 384 n-tiles / 6 per workgroup = 64 column groups x 4 = 256 workgroups
    else if (ntw == 1 && waves == 6 && depth == 8) { K8S_DEC_M(1, 6, DEC_SLAB, 8) }
    else if (ntw == 2 && waves == 3 && depth == 8) { K8S_DEC_M(2, 3, DEC_SLAB, 8) }
  } else if (epi == DEC_SWIGLU8) {
    if (ntw == 1 && waves == 7 && depth == 16) { K8S_DEC_M(1, 7, DEC_SWIGLU8, 16) }
    else if (ntw == 1 && waves == 8 && depth == 16) { K8S_DEC_M(1, 8, DEC_SWIGLU8, 16) }
    else if (ntw == 2 && waves == 4 && depth == 8) { K8S_DEC_M(2, 4, DEC_SWIGLU8, 8) }
    else if (ntw == 1 && waves == 7 && depth == 8) { K8S_DEC_M(1, 7, DEC_SWIGLU8, 8) }
  } else if (epi == DEC_BF16) {
    if (ntw == 4 && waves == 8 && depth == 4) { K8S_DEC_M(4, 8, DEC_BF16, 4) }
    else if (ntw == 2 && waves == 8 && depth == 8) { K8S_DEC_M(2, 8, DEC_BF16, 8) }
    else if (ntw == 4 && waves == 4 && depth == 8) { K8S_DEC_M(4, 4, DEC_BF16, 8) }
    else if (ntw == 3 && waves == 8 && depth == 8) { K8S_DEC_M(3, 8, DEC_BF16, 8) }
  }
#undef K8S_DEC_M
#undef K8S_DEC
  if (rc) return rc;
  return (int)hipGetLastError();
}
