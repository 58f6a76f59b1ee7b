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

// Grouped launches (MoE experts, grid.z = local expert e): A, W and the SWIGLU8 output advance by
// a per-expert stride; SLAB partials land in slab e * S + split, scaled by the routing weight
// rw[row * rw_ld + e] (0 where the row did not pick the expert), so the residual-add kernel's slab
// sum IS the expert combine.  Dense launches: all strides 0, rw null, grid.z 1.
struct DecGroup {
  long a_es, w_es, y_es;  // elements between experts' A / W / SWIGLU8 outputs
  const float* rw;        // [M][rw_ld] routing weights (SLAB epilogue) or null
  int rw_ld;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dec_rsrc(const void* base, long bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)min(bytes, 0x7fffffffL));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}
constexpr int kRnMax = 4;   // narrow deferred-norm rows: up to 16 partials (4 per thread)
constexpr int kRnWide = 16;  // wide rows: up to 256 partials (16 x 16 B per thread)

constexpr int kDecCH = 8;  // k-steps (32 deep) per A chunk

template <int MT, int WAVES>
struct DecGeom {
  static constexpr int SLOT = kDecCH * MT * 1024;                   // bytes of one A chunk
  static constexpr int PIECES = kDecCH * MT * 64;                   // 16-B pieces per chunk
  static constexpr int NLD = (PIECES + 64 * WAVES - 1) / (64 * WAVES);  // staging loads per thread
};

template <int MT, int NTW, int WAVES, int EPI, int DEPTH, bool RNW = false>
__global__ __launch_bounds__(64 * WAVES, 1) void gemm_dec_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ W, float* __restrict__ partial,
    bf16_t* __restrict__ Y, long ldy, int M, int N, int K, int kchunk, const float* __restrict__ rn_ss, int rn_nc,
    float rn_inv_d, float rn_eps, DecGroup grp) {
  using G = DecGeom<MT, WAVES>;
  const int ex = blockIdx.z;  // expert of a grouped launch (0 otherwise)
  A += ex * grp.a_es;
  W += ex * grp.w_es;
  if constexpr (EPI == DEC_SWIGLU8) Y += ex * grp.y_es;
  constexpr int ITER = DEPTH > kDecCH ? DEPTH : kDecCH;  // k-steps per unrolled main-loop iteration
  __shared__ __attribute__((aligned(16))) char sA[2 * G::SLOT];
  __shared__ float s_inv[MT * 16];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ksteps = K >> 5;
  const int kb = blockIdx.y * (kchunk >> 5);  // first k-step of this workgroup's K slice
  const int nsteps = kchunk >> 5;             // host: kchunk | K, (kchunk / 32) % ITER == 0
  const int niter = nsteps / ITER;
  const int tile0 = (blockIdx.x * WAVES + wave) * NTW;  // this wave's first n-tile

  // ---- weight stream: DEPTH k-steps x NTW fragments in flight per wave, filled after chunk 0's
  // staging loads (below)
  const u32x4* wp[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
    wp[t] = reinterpret_cast<const u32x4*>(W) + ((long)min(tile0 + t, (N >> 4) - 1) * ksteps + kb) * 64 + lane;
  u32x4 wr[DEPTH][NTW];
  auto ring_fill = [&]() {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int t = 0; t < NTW; ++t) wr[d][t] = __builtin_nontemporal_load(wp[t] + d * 64);
  };

  // ---- the A rows' partial sums of squares (deferred RMSNorm), 4 threads per row, loaded first so
  // their wait below is a counted one.  Narrow rows (<= 16 partials:
  // add_norm_partial's per-512-column sums) one float per load; wide rows (16 | partials <= 256:
  // gemm_dec_rc_kernel's per-16-column sums) 16-byte loads, each thread a quarter of the row.
  // (RNW: the wide form, a compile-time choice - the host picks the instantiation by rn_nc)
  float rnv[kRnMax];  // no initial value: read only under the same condition (no join wait)
  f32x4 rnw[RNW ? kRnWide : 1];
  const bool rn_narrow = !RNW && rn_nc <= 4 * kRnMax, rn_wide = RNW && rn_nc % 16 == 0 && rn_nc <= 16 * kRnWide;
  if (rn_ss != nullptr && threadIdx.x < MT * 64 && (rn_narrow || rn_wide)) {
    const int row = min((int)(threadIdx.x >> 2), M - 1), part = threadIdx.x & 3;
    const __amdgpu_buffer_rsrc_t ss_rs = dec_rsrc(rn_ss, (long)M * rn_nc * 4);
    if constexpr (!RNW) {
#pragma unroll
      for (int j = 0; j < kRnMax; ++j) {
        const uint32_t off = (uint32_t)((row * rn_nc + min(part + 4 * j, rn_nc - 1)) * 4);
        rnv[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ss_rs, off, 0, 0));
      }
    } else {
      const int q = rn_nc >> 2;  // this thread's quarter: floats part*q .. part*q + q - 1
#pragma unroll
      for (int j = 0; j < (RNW ? kRnWide : 1); ++j) {
        const uint32_t off = (uint32_t)((row * rn_nc + part * q + min(4 * j, q - 4)) * 4);
        rnw[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ss_rs, off, 0, 0));
      }
    }
  }

  // ---- A chunks: register-staged, 2 LDS slots
  u32x4 stg[G::NLD];
  auto stage_load = [&](int c) {
#pragma unroll
    for (int i = 0; i < G::NLD; ++i) {
      // threads past the chunk (waves that do not divide it) repeat its last piece: every load
      // unconditional, so the counted vmcnt waits stay exact
      const int p = min((int)threadIdx.x + i * 64 * WAVES, G::PIECES - 1);
      const int mt = p / (kDecCH * 64), j = (p >> 6) % kDecCH, ln = p & 63;
      const long e = (((long)mt * ksteps + kb + c * kDecCH + j) * 64 + ln) * 8;
      stg[i] = *reinterpret_cast<const u32x4*>(A + e);
    }
  };
  auto stage_store = [&](int c) {
    char* slot = sA + (c & 1) * G::SLOT;
#pragma unroll
    for (int i = 0; i < G::NLD; ++i) {
      const int p = min((int)threadIdx.x + i * 64 * WAVES, G::PIECES - 1);
      *reinterpret_cast<u32x4*>(slot + p * 16) = stg[i];
    }
  };

  // chunk 0's staging loads go out BEFORE the weight ring's first loads: at the loop head the
  // staging registers are then the oldest loads in flight on both entry paths (prologue and back
  // edge), so the counted vmcnt there leaves the weight ring in flight (with the staging loads
  // last, the merged wait drained the ring at every chunk boundary).
  stage_load(0);
  ring_fill();

  // ---- deferred RMSNorm: 1/rms of each A row from its partial sums of squares (loads issued
  // above, ahead of the A staging and the weight ring, so this wait leaves both in flight)
  if (rn_ss != nullptr && threadIdx.x < MT * 64) {
    const int rl = threadIdx.x >> 2, part = threadIdx.x & 3;
    float ss = 0.f;
    if (rn_narrow) {
#pragma unroll
      for (int j = 0; j < kRnMax; ++j) {
        asm volatile("" : "+v"(rnv[j]));  // keeps the first use (and its wait) here, past the ring issue
        ss += part + 4 * j < rn_nc ? rnv[j] : 0.f;
      }
    } else if (rn_wide) {
      const int q = rn_nc >> 2;
#pragma unroll
      for (int j = 0; j < (RNW ? kRnWide : 1); ++j) {
        asm volatile("" : "+v"(rnw[j][0]), "+v"(rnw[j][1]), "+v"(rnw[j][2]), "+v"(rnw[j][3]));
        if (4 * j < q) ss += (rnw[j][0] + rnw[j][1]) + (rnw[j][2] + rnw[j][3]);
      }
    } else {  // other widths: a plain loop (no decode GEMM today)
      const int row = min(rl, M - 1);
      for (int c = part; c < rn_nc; c += 4) ss += rn_ss[row * rn_nc + c];
    }
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
              partial[((long)(ex * gridDim.y + blockIdx.y) * M + row) * N + col] =
                  grp.rw != nullptr ? v * grp.rw[(long)row * grp.rw_ld + ex] : v;
          }
        }
      }
    }
  }
}


// Row-complete decode GEMM for a row-parallel projection feeding a residual add (the o projection
// of a TP=1 decode step): NO split-K slabs.  Each workgroup owns one 16-column n-tile for all M
// rows and the whole K; its 8 waves split K (one eighth each, the slices the split-K kernel's 8
// slabs had), stream their weight fragments AND their activation fragments straight into a
// register ring (the activations are L2-resident: every workgroup reads all of them), and reduce
// through LDS in slice order.  The epilogue then does what add_norm_partial_kernel did as its own
// launch over 8 MB of fp32 slabs:
//   resid <- bf16(resid + y)  (y summed slice by slice, in the slab kernel's order: bit-identical),
//   xw    <- bf16(resid * w)  fragment-packed as the next GEMM's A operand,
//   ss[row][tile] <- sum over the tile's 16 columns of resid^2 (the consumer's deferred RMSNorm
//                    sums N/16 partials per row).
// One launch and 16 MB of slab traffic fewer per layer; the price is the activation re-read from
// L2 (M x K bf16 per workgroup).
template <int MT, int DEPTH, int NKS>
__global__ __launch_bounds__(512, 1) void gemm_dec_rc_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                             bf16_t* __restrict__ resid, const bf16_t* __restrict__ nw,
                                                             bf16_t* __restrict__ xw, float* __restrict__ ss_out,
                                                             int M, int N, int K) {
  constexpr int WAVES = 8;
  static_assert(NKS % DEPTH == 0, "the ring consumes whole DEPTH groups of k-steps");
  __shared__ __attribute__((aligned(16))) f32x4 red[WAVES][MT][64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int tile = blockIdx.x;
  const int ksteps = K >> 5;  // host: ksteps == 8 NKS
  constexpr int nks = NKS;     // k-steps per wave: compile-time, so every ring wait is a counted one
  const int kb = wave * nks;
  const u32x4* wp = reinterpret_cast<const u32x4*>(W) + ((long)tile * ksteps + kb) * 64 + lane;
  const u32x4* ap[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) ap[m] = reinterpret_cast<const u32x4*>(A) + ((long)m * ksteps + kb) * 64 + lane;
  u32x4 rw[DEPTH], ra[DEPTH][MT];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    rw[d] = __builtin_nontemporal_load(wp + d * 64);
#pragma unroll
    for (int m = 0; m < MT; ++m) ra[d][m] = ap[m][d * 64];
  }
  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k0 = 0; k0 < nks; k0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const bf16x8 b = __builtin_bit_cast(bf16x8, rw[d]);
#pragma unroll
      for (int m = 0; m < MT; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ra[d][m]), b, acc[m], 0, 0, 0);
      const int kn = k0 + d + DEPTH;
      if (kn < nks) {  // compile-time
        rw[d] = __builtin_nontemporal_load(wp + kn * 64);
#pragma unroll
        for (int m = 0; m < MT; ++m) ra[d][m] = ap[m][kn * 64];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) red[wave][m][lane] = acc[m];
  __syncthreads();
  if (wave >= MT) return;
  // wave m: m-tile m.  C layout: col = lane & 15, rows (lane >> 4) * 4 + r
  const int m = wave;
  const int col = tile * 16 + (lane & 15);
  const float wcol = bf2f(nw[col]);
  float ssr[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = m * 16 + (lane >> 4) * 4 + r;
    const int rowc = min(row, M - 1);
    float h = bf2f(resid[(long)rowc * N + col]);
#pragma unroll
    for (int w = 0; w < WAVES; ++w) h += red[w][m][lane][r];  // slice order = the slab kernel's
    const bf16_t hb = f2bf(h);
    const float hv = bf2f(hb);
    ssr[r] = hv * hv;
    if (row < M) {
      resid[(long)row * N + col] = hb;
      xw[act_index(row, col, -(long)(N >> 5))] = f2bf(hv * wcol);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = ssr[r];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, kWave);  // the 16 columns of the row
    const int row = m * 16 + (lane >> 4) * 4 + r;
    if ((lane & 15) == 0 && row < M) ss_out[(long)row * (N >> 4) + tile] = v;
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
                               int rn_d, float rn_eps, int experts, long a_es, long w_es,
                               long y_es, const float* rw, int rw_ld, hipStream_t s) {
  if (M <= 0) return 0;
  if (experts < 1 || (rw != nullptr && epi != DEC_SLAB)) return -1;
  if (M > 64 || N % 16 || K % 32 || splits < 1 || K % splits) return -1;
  const int ntiles = N / 16, nwg_tiles = ntw * waves;
  const int kchunk = K / splits;
  const int iter = depth > kDecCH ? depth : kDecCH;
  if (kchunk % 32 || kchunk < 32 * iter || (kchunk / 32) % iter) return -3;
  if (epi != DEC_SLAB && splits != 1) return -4;
  const float inv_d = rn_d > 0 ? 1.f / (float)rn_d : 0.f;
  const int MT = (M + 15) / 16;
  const dim3 grid((ntiles + nwg_tiles - 1) / nwg_tiles, splits, experts), blk(64 * waves);
  const DecGroup dg{a_es, w_es, y_es, rw, rw_ld};
  int rc = -5;
  const bool rnw = rn_ss != nullptr && rn_nc > 4 * kRnMax;  // the wide deferred-norm form (gemm_dec_rc sums)
  if (rnw && (rn_nc % 16 || rn_nc > 16 * kRnWide)) return -1;
#define K8S_DEC_W(MTV, NTWV, WV, EPV, DV, RW)                                                                       \
  hipLaunchKernelGGL((gemm_dec_kernel<MTV, NTWV, WV, EPV, DV, RW>), grid, blk, 0, s, (const bf16_t*)A,               \
                     (const bf16_t*)Wp, partial, (bf16_t*)Y, ldy, M, N, K, kchunk, rn_ss, rn_nc, inv_d, rn_eps, dg);     \
  rc = 0
#define K8S_DEC(MTV, NTWV, WV, EPV, DV) K8S_DEC_W(MTV, NTWV, WV, EPV, DV, false)
#define K8S_DEC_M(NTWV, WV, EPV, DV) \
  switch (MT) {                      \
    case 1: K8S_DEC(1, NTWV, WV, EPV, DV); break; \
    case 2: K8S_DEC(2, NTWV, WV, EPV, DV); break; \
    case 3: K8S_DEC(3, NTWV, WV, EPV, DV); break; \
    default: K8S_DEC(4, NTWV, WV, EPV, DV); break; \
  }
  if (rnw) {  // consumers of gemm_dec_rc's per-16-column partials: gate_up behind the row-complete o
#define K8S_DEC_MW(NTWV, WV, EPV, DV) \
  switch (MT) {                       \
    case 1: K8S_DEC_W(1, NTWV, WV, EPV, DV, true); break; \
    case 2: K8S_DEC_W(2, NTWV, WV, EPV, DV, true); break; \
    case 3: K8S_DEC_W(3, NTWV, WV, EPV, DV, true); break; \
    default: K8S_DEC_W(4, NTWV, WV, EPV, DV, true); break; \
  }
    if (epi == DEC_SWIGLU8 && ntw == 1 && waves == 7 && depth == 8) { K8S_DEC_MW(1, 7, DEC_SWIGLU8, 8) }
    else if (epi == DEC_SWIGLU8 && ntw == 1 && waves == 7 && depth == 16) { K8S_DEC_MW(1, 7, DEC_SWIGLU8, 16) }
#undef K8S_DEC_MW
    if (rc) return rc;
    return (int)hipGetLastError();
  }
  // configurations (ntw, waves, depth) per epilogue: exactly the ones ops.dec_config can pick - every
  // Llama-3-8B / 70B / Mixtral projection and LM head at TP 1..8 lands on one of them
  if (epi == DEC_SLAB) {
    if (ntw == 1 && waves == 8 && depth == 8) { K8S_DEC_M(1, 8, DEC_SLAB, 8) }         // o, down; TP 2-8 shapes
    else if (ntw == 1 && waves == 6 && depth == 8) { K8S_DEC_M(1, 6, DEC_SLAB, 8) }    // qkv: 64 groups x 4 splits
    else if (ntw == 1 && waves == 4 && depth == 8) { K8S_DEC_M(1, 4, DEC_SLAB, 8) }    // narrow TP shards
    else if (ntw == 1 && waves == 4 && depth == 16) { K8S_DEC_M(1, 4, DEC_SLAB, 16) }  // 70B TP=8 qkv
  } else if (epi == DEC_SWIGLU8) {
    if (ntw == 1 && waves == 7 && depth == 8) { K8S_DEC_M(1, 7, DEC_SWIGLU8, 8) }      // gate_up
    else if (ntw == 1 && waves == 7 && depth == 16) { K8S_DEC_M(1, 7, DEC_SWIGLU8, 16) }
    else if (ntw == 1 && waves == 8 && depth == 16) { K8S_DEC_M(1, 8, DEC_SWIGLU8, 16) }  // 70B TP=1 gate_up
  } else if (epi == DEC_BF16) {
    if (ntw == 4 && waves == 8 && depth == 4) { K8S_DEC_M(4, 8, DEC_BF16, 4) }         // LM head, TP=1
    else if (ntw == 2 && waves == 8 && depth == 8) { K8S_DEC_M(2, 8, DEC_BF16, 8) }    // vocab shards, TP 2-8
    else if (ntw == 3 && waves == 8 && depth == 8) { K8S_DEC_M(3, 8, DEC_BF16, 8) }
    else if (ntw == 1 && waves == 8 && depth == 8) { K8S_DEC_M(1, 8, DEC_BF16, 8) }    // Mixtral's 32000-row head
  }
#undef K8S_DEC_M
#undef K8S_DEC
#undef K8S_DEC_W
  if (rc) return rc;
  return (int)hipGetLastError();
}


// Row-complete decode GEMM (gemm_dec_rc_kernel): A packed [ceil(M/16)][K/32][64][8], Wp packed
// [N/16][K/32][64][8]; resid [M][N] bf16 updated in place; xw packed [ceil(M/16)][N/32][64][8];
// ss [M][N/16] fp32.  Returns -1 for a shape the kernel does not tile.
extern "C" int k8sllm_gemm_dec_rc(const void* A, const void* Wp, void* resid, const void* nw, void* xw, float* ss,
                                  int M, int N, int K, hipStream_t s) {
  if (M <= 0) return 0;
  if (M > 64 || N % 32 || K % 32 || (K / 32) % 8) return -1;
  const int nks = K / 32 / 8;
  const int MT = (M + 15) / 16;
  const dim3 grid(N / 16), blk(512);
#define K8S_RC(MTV, DV, NK)                                                                                        \
  hipLaunchKernelGGL((gemm_dec_rc_kernel<MTV, DV, NK>), grid, blk, 0, s, (const bf16_t*)A, (const bf16_t*)Wp,    \
                     (bf16_t*)resid, (const bf16_t*)nw, (bf16_t*)xw, ss, M, N, K)
  if (nks == 16) {  // K = 4096: the o projection of Llama-3-8B / Mixtral at TP=1
    switch (MT) {
      case 1: K8S_RC(1, 8, 16); break;
      case 2: K8S_RC(2, 8, 16); break;
      case 3: K8S_RC(3, 8, 16); break;
      default: K8S_RC(4, 8, 16); break;
    }
  } else {  // (K = 14336, the down projection row-complete: bit-identical but 0.2-4.5 % slower per
            // decode step at 4-32 rows, profiles/r05/rc_down_*_ab.jsonl - removed)
    return -1;
  }
#undef K8S_RC
  return (int)hipGetLastError();
}
