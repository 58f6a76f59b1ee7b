// 256 x 256 MFMA GEMM for prefill-sized projections, dense or grouped
// over experts, with the SwiGLU activation fused into the epilogue.
//
//   Y[r][n] = sum_k X[r][k] * W[n][k]        (both operands K-contiguous: X [rows][K], W [N][K])
//
// Dense:   one weight, rows 0 .. M-1.
// Grouped: W [E][N][K]; expert e owns rows offsets[e] .. offsets[e+1]-1 of the expert-sorted X
//          (moe_align); each workgroup finds its (expert, m-tile) from the device offsets, so a
//          MoE layer needs no host synchronisation.
// EPI_SWIGLU: W is gate/up-interleaved per 128 rows ([64 gate | 64 up], ops.interleave_gate_up),
//          Y = silu(gate) * up [rows][N / 2] - the separate silu_mul pass over the [rows][N]
//          intermediate disappears.
//
// Structure (cdna_hip_programming.md §5, "The 256² 8-phase template"; own schedule):
//  * workgroup = 8 waves, 256 x 256 output, K in 64-deep tiles.  LDS: two buffers x (A 256 x 128 B
//    + B 256 x 128 B) = 128 KiB, ONE __shared__ array (a second one makes hipcc drain vmcnt).
//  * every tile is split into four half-tiles A0 A1 B0 B1 (128 rows x 128 B = 16 KiB, two
//    global_load_lds_dwordx4 per thread); the tile's output is computed as four 128 x 128
//    quadrants (qm, qn) in the order (0,0) (0,1) (1,1) (1,0), one per phase.  Per quadrant a wave
//    owns 64 rows x 32 columns (16 v_mfma_f32_16x16x32_bf16: 4 m-fragments x 2 n-fragments x 2
//    k-steps); its two n-fragments sit 64 columns apart, so a SwiGLU tile's gate and up values of
//    one output element are in the same lane and register index.
//  * operand fragments live in four register sets xa0 xa1 (X, quadrant row halves) and wf0 wf1
//    (W, column halves); the quadrant order alternates with the tile's parity so each phase's
//    ds_reads fill a set only a LATER phase uses - no fragment read is waited for synchronously.
//  * one half-tile DMA refill per phase, issued as single pieces between the MFMA k-steps, one
//    raw s_barrier per two phases (32 MFMAs per wave) preceded by `s_waitcnt vmcnt(8)`: 4 younger
//    half-tiles stay in flight across it - never __syncthreads() while a DMA is pending.
//  * LDS rows are 128 B; chunk c of row r is stored at c ^ ((r >> 1) & 7) (swizzle applied to the
//    DMA source address, the LDS side stays lane-linear), so every ds_read_b128 16-lane group hits
//    16 distinct bank quads.
//  * XCD-aware tile order: workgroup ids are remapped so each XCD runs a contiguous range of
//    logical tiles, ordered in groups of 8 m-tiles (neighbours share A or B through that XCD's L2).
#include <type_traits>

#include "common.h"

namespace k8sllm {

namespace {
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
}  // namespace

enum { TILE_EPI_BF16 = 0, TILE_EPI_SWIGLU = 1 };

template <int EPI, bool GROUPED>
__global__ __launch_bounds__(512, 1) void gemm_tile256_kernel(const bf16_t* __restrict__ X,
                                                              const bf16_t* __restrict__ W, bf16_t* __restrict__ Y,
                                                              const int* __restrict__ offsets, int E, int M, int N,
                                                              int K, long w_es, int n_mt, int n_nt) {
  constexpr int BUF = 65536, BOFF = 32768, HALF = 16384;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // ---- logical tile of this workgroup: XCD remap (bijective) then groups of 8 m-tiles ----
  const int nwg = n_mt * n_nt;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = 8;
  const int grp = lid / (GM * n_nt), first_m = grp * GM;
  const int gsz = min(n_mt - first_m, GM);
  const int in_g = lid - grp * GM * n_nt;
  const int mt = first_m + in_g % gsz, nt = in_g / gsz;

  int row0, mrows;
  const bf16_t* Wt = W;
  if constexpr (GROUPED) {
    int e = -1, acc_t = 0;
    row0 = 0;
    mrows = 0;
    for (int x = 0; x < E; ++x) {
      const int o0 = offsets[x], o1 = offsets[x + 1];
      const int tiles = (o1 - o0 + 255) >> 8;
      if (e < 0 && mt < acc_t + tiles) {
        e = x;
        row0 = o0 + (mt - acc_t) * 256;
        mrows = min(256, o1 - row0);
      }
      acc_t += tiles;
    }
    if (e < 0) return;  // uniform: past the last expert's tiles
    Wt = W + (long)e * w_es;
  } else {
    row0 = mt * 256;
    mrows = min(256, M - row0);
  }
  const int n0 = nt * 256;

  // ---- DMA sources: half h (0 A0, 1 A1, 2 B0, 3 B1), piece j (0, 1) -> LDS rows of the half
  // (j * 8 + wave) * 8 .. + 7; lane -> row + (lane >> 3), 16-B slot lane & 7 ----
  uint32_t soff[4][2];
  const char* xb = reinterpret_cast<const char*>(X);
  const char* wb_ = reinterpret_cast<const char*>(Wt);
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int rl = (h & 1) * 128 + (j * 8 + wave) * 8 + (lane >> 3);  // row within the A or B tile
      const int c = (lane & 7) ^ ((rl >> 1) & 7);
      if (h < 2) {
        const int r = row0 + min(rl, mrows - 1);  // rows past the end: clamped, never stored
        soff[h][j] = (uint32_t)(((long)r * K + c * 8) * 2 - (long)row0 * K * 2);
      } else {
        soff[h][j] = (uint32_t)(((long)(n0 + rl) * K + c * 8) * 2);
      }
    }
  const char* xbase = xb + (long)row0 * K * 2;
  const int nk = K >> 6;

  // issue half-tile h of K-tile kt into buffer kt & 1
  auto issue = [&](int h, int kt) {
    char* dst = smem + (kt & 1) * BUF + (h >> 1) * BOFF + (h & 1) * HALF;
    const char* base = (h < 2 ? xbase : wb_) + kt * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + soff[h][j]), (lds_void_t*)(dst + (j * 8 + wave) * 1024),
                                       16, 0, 0);
  };

  // fragment reads: lane row = lane & 15, 16-B chunk 4 ks + (lane >> 4), swizzle (lane >> 1) & 7
  const int swz = (lane >> 1) & 7;
  const int rd_row = (lane & 15) * 128;
  int chk[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) chk[ks] = ((4 * ks + (lane >> 4)) ^ swz) << 4;
  // X set qm: rows qm*128 + wm*64 + i*16 ; W set qn: rows qn*128 + jj*64 + wn*16
  auto read_x = [&](bf16x8 (&f)[4][2], int kt, int qm) {
    const char* b = smem + (kt & 1) * BUF + (qm * 128 + wm * 64) * 128 + rd_row;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) f[i][ks] = *reinterpret_cast<const bf16x8*>(b + i * 2048 + chk[ks]);
  };
  auto read_w = [&](bf16x8 (&f)[2][2], int kt, int qn) {
    const char* b = smem + (kt & 1) * BUF + BOFF + (qn * 128 + wn * 16) * 128 + rd_row;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) f[jj][ks] = *reinterpret_cast<const bf16x8*>(b + jj * 8192 + chk[ks]);
  };

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[a][b][i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one k-step (8 MFMAs) of quadrant (qm, qn)
  auto mma = [&](int qm, int qn, const bf16x8 (&xa)[4][2], const bf16x8 (&wf)[2][2], int ks) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[qm][qn][i][jj] = mfma16(wf[jj][ks], xa[i][ks], acc[qm][qn][i][jj]);
    __builtin_amdgcn_s_setprio(0);
  };
  // one DMA piece (1 KiB per wave) between MFMA k-steps: the texture path streams the next tiles
  // while the matrix cores run, instead of every wave queueing 4 DMAs at once at a barrier
  auto piece = [&](bool on, int h, int kt, int j) {
    __builtin_amdgcn_sched_barrier(0);
    if (on) {
      char* dst = smem + (kt & 1) * BUF + (h >> 1) * BOFF + (h & 1) * HALF;
      const char* base = (h < 2 ? xbase : wb_) + kt * 128;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + soff[h][j]), (lds_void_t*)(dst + (j * 8 + wave) * 1024),
                                       16, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  bf16x8 xa0[4][2], xa1[4][2], wf0[2][2], wf1[2][2];

  // ---- quadrant order alternates with the tile's parity P so that no fragment set is read
  // synchronously: P = 0: (0,0) (0,1) (1,1) (1,0); P = 1: (0,1) (0,0) (1,0) (1,1).  The last
  // quadrant of a tile and the first of the next differ in both coordinates, so both sets the
  // next tile starts with are free one phase early.  Fragment reads (one phase ahead of use):
  //   ph1: W half 1-P of tile t     ph2: X half 1 of t     ph3: X half 0 of t+1
  //   ph4: W half 1-P of t+1 (= the first W half of tile t+1, whose parity is 1-P)
  // Barriers: one per two phases (S1 = ph1+ph2, S2 = ph3+ph4; 32 MFMAs per wave between
  // barriers).  S1(t) reads W_(1-P)(t), A1(t); S2(t) reads A0(t+1), W_(1-P)(t+1).  A region is
  // refilled for tile t+2 in the half-phase after the barrier that retires its read:
  //   S1(t) issues A0(t+2), W_P(t+2)        S2(t) issues W_(1-P)(t+2), A1(t+2)
  // which is 3 half-phases before tile t+2 reads it; each half-phase ends with lgkmcnt(0),
  // vmcnt(8) (4 younger half-tiles in flight) and one raw s_barrier. ----

  // prologue: tile 0 (parity 0) is preceded by the reads of A0(0) and W0(0) ("S2(-1)");
  // halves in issue order: A0(0) B0(0) B1(0) A1(0) | A0(1) B1(1) B0(1) A1(1)
  issue(0, 0);
  issue(2, 0);
  issue(3, 0);
  issue(1, 0);
  if (nk > 1) {
    issue(0, 1);
    issue(3, 1);
    issue(2, 1);
    issue(1, 1);
    vm_wait<12>();  // A0(0), B0(0) landed
  } else {
    vm_wait<0>();
  }
  __builtin_amdgcn_s_barrier();
  read_x(xa0, 0, 0);
  read_w(wf0, 0, 0);
  lgkm_wait0();
  if (nk > 1) vm_wait<8>(); else vm_wait<0>();  // B1(0), A1(0) landed
  __builtin_amdgcn_s_barrier();

  auto tile = [&](int t, auto par) {
    constexpr int P = decltype(par)::value;
    const bool full = t + 2 < nk;  // every DMA counted by this tile's waits is real
    auto end_half = [&]() {
      lgkm_wait0();
      if (full) vm_wait<8>(); else vm_wait<0>();
      __builtin_amdgcn_s_barrier();
    };
    // S1: phase 1 + phase 2 (DMA: A0(t+2), W_P(t+2), one piece per MFMA k-step)
    const bool ld = t + 2 < nk;
    if constexpr (P == 0) read_w(wf1, t, 1); else read_w(wf0, t, 0);
    if constexpr (P == 0) {
      mma(0, 0, xa0, wf0, 0); piece(ld, 0, t + 2, 0); mma(0, 0, xa0, wf0, 1); piece(ld, 0, t + 2, 1);
    } else {
      mma(0, 1, xa0, wf1, 0); piece(ld, 0, t + 2, 0); mma(0, 1, xa0, wf1, 1); piece(ld, 0, t + 2, 1);
    }
    read_x(xa1, t, 1);
    if constexpr (P == 0) {
      mma(0, 1, xa0, wf1, 0); piece(ld, 2 + P, t + 2, 0); mma(0, 1, xa0, wf1, 1); piece(ld, 2 + P, t + 2, 1);
    } else {
      mma(0, 0, xa0, wf0, 0); piece(ld, 2 + P, t + 2, 0); mma(0, 0, xa0, wf0, 1); piece(ld, 2 + P, t + 2, 1);
    }
    end_half();
    // S2: phase 3 + phase 4 (DMA: W_(1-P)(t+2), A1(t+2))
    if (t + 1 < nk) read_x(xa0, t + 1, 0);
    if constexpr (P == 0) {
      mma(1, 1, xa1, wf1, 0); piece(ld, 3 - P, t + 2, 0); mma(1, 1, xa1, wf1, 1); piece(ld, 3 - P, t + 2, 1);
    } else {
      mma(1, 0, xa1, wf0, 0); piece(ld, 3 - P, t + 2, 0); mma(1, 0, xa1, wf0, 1); piece(ld, 3 - P, t + 2, 1);
    }
    if (t + 1 < nk) {
      if constexpr (P == 0) read_w(wf1, t + 1, 1); else read_w(wf0, t + 1, 0);
    }
    if constexpr (P == 0) {
      mma(1, 0, xa1, wf0, 0); piece(ld, 1, t + 2, 0); mma(1, 0, xa1, wf0, 1); piece(ld, 1, t + 2, 1);
    } else {
      mma(1, 1, xa1, wf1, 0); piece(ld, 1, t + 2, 0); mma(1, 1, xa1, wf1, 1); piece(ld, 1, t + 2, 1);
    }
    end_half();
  };
  for (int t = 0; t < nk; t += 2) {
    tile(t, std::integral_constant<int, 0>{});
    if (t + 1 < nk) tile(t + 1, std::integral_constant<int, 1>{});
  }

  // ---- epilogue: acc[qm][qn][i][jj][r] = Y[m][n] with m = qm*128 + wm*64 + i*16 + (lane & 15),
  // n = qn*128 + jj*64 + wn*16 + 4 (lane >> 4) + r (the MFMA took W as its A operand) ----
  const int ml = lane & 15, nq = 4 * (lane >> 4);
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = qm * 128 + wm * 64 + i * 16 + ml;
      if (m >= mrows) continue;
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
        if constexpr (EPI == TILE_EPI_SWIGLU) {
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float g = bf2f(f2bf(acc[qm][qn][i][0][r])), u = bf2f(f2bf(acc[qm][qn][i][1][r]));
            o[r] = g * u / (1.f + __expf(-g));
          }
          bf16_t* yp = Y + (long)(row0 + m) * (N >> 1) + ((n0 + qn * 128) >> 1) + wn * 16 + nq;
          *reinterpret_cast<uint2*>(yp) = uint2{pack2(o[0], o[1]), pack2(o[2], o[3])};
        } else {
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const f32x4 v = acc[qm][qn][i][jj];
            bf16_t* yp = Y + (long)(row0 + m) * N + n0 + qn * 128 + jj * 64 + wn * 16 + nq;
            *reinterpret_cast<uint2*>(yp) = uint2{pack2(v[0], v[1]), pack2(v[2], v[3])};
          }
        }
      }
    }
}

// ------------------------------------------------------------------------------------------------
// 4-wave variant: the same 256 x 256 output tile, but each wave owns a 128 x 128 quarter (64
// accumulators of v_mfma_f32_16x16x32_bf16 = 256 f32 per lane in AGPRs, one wave per SIMD).  Per
// 32-deep k sub-step a wave reads 16 ds_read_b128 for 64 MFMAs (0.25 per MFMA; the 8-wave kernel
// above needs 0.375).
//
//  * K in 64-deep tiles with 128-B LDS rows, so every DMA row segment is one whole 128-B line
//    (a 32-deep / 64-B-row build of this kernel issued twice the L2 requests, and its TA spent a
//    third of the kernel stalled on the cache: profiles/r03/gemm_pmc_qkv.jsonl).
//  * LDS = a ring of five 32 KiB half-slots (160 KiB, one __shared__ array); half-tile h (A_t = 2t,
//    B_t = 2t + 1) lives in slot h % 5.  A_{t+2} is DMA'd during sub-step (t, 0) and B_{t+2} during
//    (t, 1), each into the slot its predecessor h - 5 left once its last fragments were read, so A
//    has 3 and B 2 sub-steps (~2-3k cycles) to land.
//  * fragments of the next sub-step are read (16 ds_read_b128) in between the current one's MFMAs
//    into the second register set: (t, 1) during (t, 0), (t + 1, 0) during (t, 1).  ONE raw
//    s_barrier per tile, before (t, 1): lgkmcnt(0) and vmcnt(8) (tile t + 1 has landed, A_{t+2}
//    stays in flight) - never vmcnt(0) in the loop.
//  * 128-B LDS rows: logical 16-B chunk c of row r sits at physical chunk c ^ ((r >> 1) & 7)
//    (applied to the DMA source address; the LDS side is lane-linear), so each 16-lane group of a
//    fragment ds_read_b128 (rows 0-15 of a block) hits 16 distinct bank quads.
//  * the DMA is buffer_load_dwordx4 ... lds against SGPR buffer descriptors of this tile's rows:
//    lane offsets are per-lane constants, the k offset goes in soffset (no 64-bit address math).
template <int N>
__device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// CPX / CPW: cache-policy bits of the X / W DMA loads (17 = sc0 sc1: bypass the CU's L1).
// SCH: 0 = one barrier per k-tile, A_{t+2} DMA'd during (t, 0) and B_{t+2} during (t, 1);
//      1 = two barriers per k-tile: the mid-(t, 0) barrier (every wave has tile t's k-half-1
//      fragments in registers) frees BOTH of tile t's half-slots, so B_{t+2} and A_{t+3} are
//      DMA'd from there on - every piece gets >= ~120 MFMAs to land instead of ~64.
// SWZ: 1 = XOR-swizzled 16-B chunks (permuted DMA source, conflict-free reads); 0 = linear rows
// (sequential DMA source, bank-conflicted fragment reads) - diagnosis.
// WST (SCH = 1): wave w issues its DMA pieces w MFMAs later than wave 0, so the four waves' pieces
// reach the texture-address unit one MFMA (16 cycles) apart instead of together.
// STG (SCH = 0): 1 = register-staged refill instead of LDS-DMA: each piece is a buffer_load_dwordx4
// into VGPRs issued one k-tile ahead and a ds_write_b128 of the previous one (an LDS-DMA piece
// holds its wave's issue for ~60-185 cycles among MFMAs; a VGPR load and an LDS store ride the
// MFMA shadow like the fragment reads).
template <int EPI, bool GROUPED, int ABL = 0, int CPX = 0, int CPW = 0, int SCH = 0, int SWZ = 1, int WST = 0,
          int STG = 0, int LGK = 0>  // ABL (diagnosis): 1 no MFMA, 2 no in-loop DMA
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                         bf16_t* __restrict__ Y, const int* __restrict__ offsets,
                                                         int E, int M, int N, int K, long w_es, int n_mt, int n_nt) {
  constexpr int HS = 32768;  // one half-slot: 256 rows x 128 B
  __shared__ __attribute__((aligned(16))) char smem[5 * HS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // ---- logical tile: bijective XCD remap, then groups of 8 m-tiles ----
  const int nwg = n_mt * n_nt;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = 8;
  const int grp = lid / (GM * n_nt), first_m = grp * GM;
  const int gsz = min(n_mt - first_m, GM);
  const int in_g = lid - grp * GM * n_nt;
  const int mt = first_m + in_g % gsz, nt = in_g / gsz;

  int row0, mrows;
  const bf16_t* Wt = W;
  if constexpr (GROUPED) {
    int e = -1, acc_t = 0;
    row0 = 0;
    mrows = 0;
    for (int x = 0; x < E; ++x) {
      const int o0 = offsets[x], o1 = offsets[x + 1];
      const int tiles = (o1 - o0 + 255) >> 8;
      if (e < 0 && mt < acc_t + tiles) {
        e = x;
        row0 = o0 + (mt - acc_t) * 256;
        mrows = min(256, o1 - row0);
      }
      acc_t += tiles;
    }
    if (e < 0) return;  // uniform: past the last expert's tiles
    Wt = W + (long)e * w_es;
  } else {
    row0 = mt * 256;
    mrows = min(256, M - row0);
  }
  const int n0 = nt * 256;
  const int nrows = min(256, N - n0);

  // ---- DMA of one half-tile (256 rows x 128 B = 32 pieces of 1 KiB): piece p (0..7) of this
  // wave covers rows (p * 4 + wave) * 8 .. + 7; lane -> row + (lane >> 3), physical chunk lane & 7 ----
  uint32_t soff[2][8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int rl = (p * 4 + wave) * 8 + (lane >> 3);
    const int cl = SWZ ? (lane & 7) ^ ((rl >> 1) & 7) : (lane & 7);
    soff[0][p] = (uint32_t)(((long)min(rl, mrows - 1) * K + cl * 8) * 2);  // rows past the end: clamped, never stored
    soff[1][p] = (uint32_t)(((long)min(rl, nrows - 1) * K + cl * 8) * 2);
  }
  // buffer descriptors over this tile's X rows / W rows, built from wave-uniform values only so
  // hipcc keeps them in SGPRs (no waterfall loops, cdna_hip_programming.md T20)
  auto rsrc = [](const void* base, long bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t xr = rsrc(reinterpret_cast<const char*>(X) + (long)row0 * K * 2, (long)mrows * K * 2);
  const __amdgpu_buffer_rsrc_t wr = rsrc(reinterpret_cast<const char*>(Wt) + (long)n0 * K * 2, (long)nrows * K * 2);
  const int nk = K >> 6;

  // piece p of half-tile (operand o, k-tile kt) into half-slot `slot`; k-tiles past the end re-read
  // the last one (identical bytes into a slot no live fragment read uses), so every sub-step
  // issues the same count and the vmcnt arithmetic never changes
  auto piece = [&](int o, int p, int kt, int slot) {
    char* dst = smem + slot * HS + (p * 4 + wave) * 1024;
    if (o)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void_t*)dst, 16, soff[1][p], min(kt, nk - 1) * 128, 0, CPW);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void_t*)dst, 16, soff[0][p], min(kt, nk - 1) * 128, 0, CPX);
  };
  auto issue_half = [&](int o, int kt) {
#pragma unroll
    for (int p = 0; p < 8; ++p) piece(o, p, kt, (2 * kt + o) % 5);
  };
  // register staging (STG): piece p of half-tile (o, kt) into st[o][p]; written lane-linear into
  // the same LDS bytes the DMA piece would fill
  typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));
  u32x4s st[2][8];
  auto st_load = [&](int o, int p, int kt) {
    if (o)
      st[o][p] = __builtin_amdgcn_raw_buffer_load_b128(wr, soff[1][p], min(kt, nk - 1) * 128, CPW);
    else
      st[o][p] = __builtin_amdgcn_raw_buffer_load_b128(xr, soff[0][p], min(kt, nk - 1) * 128, CPX);
  };
  auto st_write = [&](int o, int p, int slot) {
    *reinterpret_cast<u32x4s*>(smem + slot * HS + (p * 4 + wave) * 1024 + lane * 16) = st[o][p];
  };

  // fragment read: lane row lane & 15 of a 16-row block, 16-B chunk 4 ks + (lane >> 4)
  int rd[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
    rd[ks] = (lane & 15) * 128 + (((4 * ks + (lane >> 4)) ^ (SWZ ? ((lane >> 1) & 7) : 0)) << 4);
  auto frag = [&](int slot, int ks, int o, int blk) -> bf16x8 {
    const char* b = smem + slot * HS + ((o ? wn : wm) * 8 + blk) * 2048 + rd[ks];
    return *reinterpret_cast<const bf16x8*>(b);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // One 32-deep sub-step: 64 MFMAs from (ca, cb), each carrying at most one other instruction in
  // its shadow (explicit order: a sched_barrier after every MFMA).  The 8 DMA pieces of the
  // sub-step ride MFMAs 4, 12, ..., 60 - evenly spread: an LDS-DMA instruction holds its wave's
  // issue for tens of cycles (MI355X_MICROARCH.md, LDS-DMA piece issue cost), and bunched pieces
  // starve the matrix pipe (measured: all 16 pieces of a k-tile in one sub-step, 8-13 % slower;
  // 8 in a row at the sub-step start, 3-4 % slower than spread).  The 16 fragment reads of the
  // next sub-step ride the other MFMAs from the first on (W blocks first: the next sub-step's first
  // row block needs all eight), done by MFMA 17.
  auto sub = [&](bf16x8 (&ca)[8], bf16x8 (&cb)[8], bf16x8 (&na)[8], bf16x8 (&nb)[8], int sa, int sb, int nks,
                 int o, int kt, int ds) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int n = g * 8 + j;
        if constexpr (ABL == 1) {
          asm volatile("" ::"v"(cb[j]), "v"(ca[g]));  // keep the fragment reads alive
        } else {
          acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[j], ca[g], acc[g][j], 0, 0, 0);
        }
        const int q = n - (n > 4) - (n > 12);  // read index: skips the DMA slots 4 and 12
        if (j == 4) {
          if constexpr (STG) {
            st_write(o, g, ds);   // half-tile (o, kt) piece g, loaded one k-tile ago
            st_load(o, g, kt + 1);
          } else if constexpr (ABL != 2) {
            piece(o, g, kt, ds);
          }
        } else if (q < 8) {
          nb[q] = frag(sb, nks, 1, q);
        } else if (q < 16) {
          na[q - 8] = frag(sa, nks, 0, q - 8);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  if constexpr (SCH == 1) {
    // piece i (0..15) of iteration t: B_{t+2} pieces 0..7 into A_t's half-slot, then A_{t+3}
    // pieces 0..7 into B_t's (both free once the mid-(t, 0) barrier has passed)
    auto piece16 = [&](int i, int t) {
      if (i < 8)
        piece(1, i, t + 2, (2 * t) % 5);
      else
        piece(0, i - 8, t + 3, (2 * t + 1) % 5);
    };
    // PH 0 = (t, 0): fragment reads of k-half 1 of tile t on MFMAs 0-15, lgkmcnt(0) + barrier after
    // MFMA 19, pieces 0-6 on MFMAs 22, 28, ..., 58.  PH 1 = (t, 1): reads of k-half 0 of tile t+1
    // on MFMAs 0-15, pieces 7-15 on MFMAs 19, 24, ..., 59.
    auto sub1 = [&](auto ph, auto wo, bf16x8 (&ca)[8], bf16x8 (&cb)[8], bf16x8 (&na)[8], bf16x8 (&nb)[8], int sa,
                    int sb, int nks, int t) {
      constexpr int PH = decltype(ph)::value, WO = decltype(wo)::value;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int n = g * 8 + j;
          if constexpr (ABL == 1) {
            asm volatile("" ::"v"(cb[j]), "v"(ca[g]));
          } else {
            acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[j], ca[g], acc[g][j], 0, 0, 0);
          }
          if (n < 8) {
            nb[n] = frag(sb, nks, 1, n);
          } else if (n < 16) {
            na[n - 8] = frag(sa, nks, 0, n - 8);
          } else if (PH == 0 && n == 19) {
            lgkm_wait0();
            __builtin_amdgcn_s_barrier();
          } else if (PH == 0 && n >= 22 + WO && (n - 22 - WO) % 6 == 0 && (n - 22 - WO) / 6 < 7) {
            if constexpr (ABL != 2) piece16((n - 22 - WO) / 6, t);
          } else if (PH == 1 && n >= 19 + WO && (n - 19 - WO) % 5 == 0 && (n - 19 - WO) / 5 < 9) {
            if constexpr (ABL != 2) piece16(7 + (n - 19 - WO) / 5, t);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    // prologue: A_0 B_0 A_1 B_1 A_2 in flight (all five half-slots); tile 0 landed -> its k-half 0
    issue_half(0, 0);
    issue_half(1, 0);
    issue_half(0, 1);
    issue_half(1, 1);
    issue_half(0, 2);
    vm_wait_n<24>();
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      fa0[g] = frag(0, 0, 0, g);
      fb0[g] = frag(1, 0, 1, g);
    }
    auto kloop = [&](auto wo) {
      for (int t = 0; t < nk; ++t) {
        // the previous sub-step's reads landed long ago; saying so keeps hipcc from waiting for the
        // first read of this one before the first MFMA
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) as a real instruction the waitcnt pass sees
        sub1(std::integral_constant<int, 0>{}, wo, fa0, fb0, fa1, fb1, (2 * t) % 5, (2 * t + 1) % 5, 1, t);
        vm_wait_n<15>();  // B_{t+1} landed (younger: A_{t+2}'s 8 pieces and this tile's first 7)
        __builtin_amdgcn_s_barrier();
        sub1(std::integral_constant<int, 1>{}, wo, fa1, fb1, fa0, fb0, (2 * t + 2) % 5, (2 * t + 3) % 5, 0, t);
      }
    };
    if constexpr (WST) {
      if (wave == 0) kloop(std::integral_constant<int, 0>{});
      else if (wave == 1) kloop(std::integral_constant<int, 1>{});
      else if (wave == 2) kloop(std::integral_constant<int, 2>{});
      else kloop(std::integral_constant<int, 3>{});
    } else {
      kloop(std::integral_constant<int, 0>{});
    }
    vm_wait_n<0>();
  } else {
  // prologue: A_0 B_0 A_1 B_1 in flight; tile 0 landed -> read its first k-half
  issue_half(0, 0);
  issue_half(1, 0);
  issue_half(0, 1);
  issue_half(1, 1);
  if constexpr (STG) {
    // A_2, B_2 into the staging registers; they are written to LDS during (0, 0) / (0, 1)
#pragma unroll
    for (int p = 0; p < 8; ++p) st_load(0, p, 2);
#pragma unroll
    for (int p = 0; p < 8; ++p) st_load(1, p, 2);
    vm_wait_n<32>();  // tile 0 landed (tile 1 and the 16 staged loads younger)
  } else {
    vm_wait_n<16>();
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    fa0[g] = frag(0, 0, 0, g);
    fb0[g] = frag(1, 0, 1, g);
  }

  for (int t = 0; t < nk; ++t) {
    const int sa = (2 * t) % 5, sb = (2 * t + 1) % 5;            // tile t's half-slots
    const int sa1 = (2 * t + 2) % 5, sb1 = (2 * t + 3) % 5;      // tile t+1's
    // the previous sub-step's fragment reads landed long ago; an explicit lgkmcnt(0) here keeps
    // hipcc from merging that wait with the first read of this sub-step (a full LDS latency before
    // the first MFMA of every k-tile)
    if constexpr (LGK) __builtin_amdgcn_s_waitcnt(0xc07f);
    // (t, 0): MFMAs on k-half 0; read k-half 1 of tile t; DMA A_{t+2}
    sub(fa0, fb0, fa1, fb1, sa, sb, 1, 0, t + 2, (2 * t + 4) % 5);
    lgkm_wait0();
    if constexpr (STG)
      vm_wait_n<24>();  // t = 0: B_1 (DMA) landed - younger: B_2, A_2... staged loads (<= 24); later a no-op
    else
      vm_wait_n<8>();  // B_{t+1} landed (only A_{t+2} younger)
    __builtin_amdgcn_s_barrier();
    // (t, 1): MFMAs on k-half 1; read k-half 0 of tile t+1 (garbage past the end, never used); DMA B_{t+2}
    sub(fa1, fb1, fa0, fb0, sa1, sb1, 0, 1, t + 2, (2 * t + 5) % 5);
  }
  vm_wait_n<0>();
  }

  // ---- epilogue: acc[i][j][r] = Y[m][n], m = wm*128 + i*16 + (lane & 15),
  // n = wn*128 + j*16 + 4 (lane >> 4) + r.  Staged through LDS (the ring is idle now): each wave
  // writes its quarter as bf16 rows (8-B ds_write per 4 columns), then reads back whole rows and
  // stores 16 B per lane, 256 contiguous bytes per row - half the store instructions of writing
  // the accumulator layout directly, which is what bounds a store tail (T21). ----
  lgkm_wait0();
  __builtin_amdgcn_s_barrier();  // every wave is done with the ring (its last DMAs retired above)
  constexpr int OUTW = EPI == TILE_EPI_SWIGLU ? 64 : 128;  // output columns of this wave's quarter
  constexpr int RS = OUTW * 2 + 16;                        // LDS row stride (16-B pad: 2-way writes)
  char* stage = smem + wave * (128 * RS);
  const int ml = lane & 15, nq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    __builtin_amdgcn_sched_barrier(0);  // one row block's accumulators at a time (no hoisted AGPR reads)
    char* srow = stage + (i * 16 + ml) * RS + nq * 2;
    if constexpr (EPI == TILE_EPI_SWIGLU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gt = bf2f(f2bf(acc[i][j][r])), up = bf2f(f2bf(acc[i][j + 4][r]));
          o[r] = gt * up / (1.f + __expf(-gt));
        }
        *reinterpret_cast<uint2*>(srow + j * 32) = uint2{pack2(o[0], o[1]), pack2(o[2], o[3])};
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f32x4 v = acc[i][j];
        *reinterpret_cast<uint2*>(srow + j * 32) = uint2{pack2(v[0], v[1]), pack2(v[2], v[3])};
      }
    }
  }
  lgkm_wait0();
  constexpr int CPR = OUTW / 8;  // 16-B chunks per row
  constexpr int RPI = 64 / CPR;  // rows per wave instruction
  const int ldy = EPI == TILE_EPI_SWIGLU ? (N >> 1) : N;
  const int col0 = EPI == TILE_EPI_SWIGLU ? ((n0 + wn * 128) >> 1) : n0 + wn * 128;
  const int ncols = EPI == TILE_EPI_SWIGLU ? (nrows >> 1) - wn * 64 : nrows - wn * 128;
  const int rr = lane / CPR, cc = lane % CPR;
  // branch-free masked stores: a buffer descriptor over this m-tile's rows drops every store past
  // row mrows (out of range), and a lane whose columns are past N gets an out-of-range offset
  const __amdgpu_buffer_rsrc_t yr = rsrc(Y + (long)row0 * ldy, (long)mrows * ldy * 2);
  const uint32_t yo = cc * 8 < ncols ? (uint32_t)(((wm * 128 + rr) * ldy + col0 + cc * 8) * 2) : 0x80000000u;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int b = 0; b < 128 / RPI; b += 8) {  // 8 row groups per batch: reads issued back to back
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const u32x4*>(stage + ((b + u) * RPI + rr) * RS + cc * 16);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      __builtin_amdgcn_raw_buffer_store_b128(v[u], yr, yo + (uint32_t)((b + u) * RPI * ldy * 2), 0, 0);
  }
}

// ------------------------------------------------------------------------------------------------
// Persistent form of the 4-wave kernel (the prefill default): one workgroup per CU loops over its
// XCD's tiles, and the LDS-DMA ring runs on ACROSS tiles - the first two k-tiles of the next tile
// are fetched during the last two k-tiles of the current one, exactly like any other k-tile - so
// a tile starts with its data already in LDS.  In the one-launch-per-tile form every CU issued
// its 128 KiB prologue and its 128 KiB of output in the same instant (all tiles of a round start
// and end together): ~14 us of fixed cost per tile round, 15 % of a 4096-deep projection
// (profiles/r03, fixed cost vs k-tiles fit).  Rows past M and k beyond the operand rows read as
// zeros through the buffer descriptors' range checks (no clamping, so the lane's DMA offset is
// one constant), and the epilogue stores straight from the accumulators through a descriptor
// over the tile's rows (rows past M are dropped by the range check).
template <int EPI, bool GROUPED>
__global__ __launch_bounds__(256, 1) void gemm_w4p_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                          bf16_t* __restrict__ Y, const int* __restrict__ offsets,
                                                          int E, int M, int N, int K, long w_es, int n_mt, int n_nt) {
  constexpr int HS = 32768;
  __shared__ __attribute__((aligned(16))) char smem[5 * HS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nk = K >> 6;

  // ---- this workgroup's tiles: XCD x owns a contiguous chunk of the logical tile order (split
  // bijectively over the 8 XCDs); its `per` workgroups take every per-th tile of the chunk ----
  const int nwg = n_mt * n_nt;
  const int xcd = blockIdx.x & 7, per = gridDim.x >> 3, sl = blockIdx.x >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int lo = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int cnt = q8 + (xcd < r8 ? 1 : 0);

  auto rsrc = [](const void* base, long bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const uint32_t lo_ = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo_), 0, nb, 0x00020000);
  };
  struct Tile {
    int idx, row0, mrows, n0, nrows;
    __amdgpu_buffer_rsrc_t xr, wr;
  };
  constexpr int GM = 8;
  // the first valid tile at chunk index >= idx (idx >= cnt: none)
  auto find = [&](int idx) -> Tile {
    Tile tl;
    for (; idx < cnt; idx += per) {
      const int lid = lo + idx;
      const int grp = lid / (GM * n_nt), first_m = grp * GM;
      const int gsz = min(n_mt - first_m, GM);
      const int in_g = lid - grp * GM * n_nt;
      const int mt = first_m + in_g % gsz, nt = in_g / gsz;
      int row0 = mt * 256, mrows = M - row0;
      const bf16_t* Wt = W;
      if constexpr (GROUPED) {
        int e = -1, acc_t = 0;
        for (int x = 0; x < E; ++x) {
          const int o0 = offsets[x], o1 = offsets[x + 1];
          const int tiles = (o1 - o0 + 255) >> 8;
          if (e < 0 && mt < acc_t + tiles) {
            e = x;
            row0 = o0 + (mt - acc_t) * 256;
            mrows = o1 - row0;
          }
          acc_t += tiles;
        }
        if (e < 0) continue;  // past the last expert's tiles
        Wt = W + (long)e * w_es;
      }
      tl.idx = idx;
      tl.row0 = row0;
      tl.mrows = min(256, mrows);
      tl.n0 = nt * 256;
      tl.nrows = min(256, N - tl.n0);
      tl.xr = rsrc(X + (long)row0 * K, (long)tl.mrows * K * 2);
      tl.wr = rsrc(Wt + (long)tl.n0 * K, (long)tl.nrows * K * 2);
      return tl;
    }
    tl.idx = cnt;
    return tl;
  };

  Tile cur = find(sl);
  if (cur.idx >= cnt) return;  // uniform: nothing for this workgroup
  Tile nxt = find(cur.idx + per);

  // ---- DMA: piece p of a half-tile = rows (p * 4 + wave) * 8 + (lane >> 3); the lane's offset
  // (row, swizzled 16-B chunk) is one constant, p and k go to soffset ----
  const int rl0 = wave * 8 + (lane >> 3);
  const uint32_t vo = (uint32_t)(((long)rl0 * K + (((lane & 7) ^ ((rl0 >> 1) & 7)) * 8)) * 2);
  // global k-tile stream position of the next DMA: half-tiles h = 2 * gk + o live in slot h % 5
  auto piece = [&](const __amdgpu_buffer_rsrc_t& r, int p, int kt, int slot) {
    char* dst = smem + slot * HS + (p * 4 + wave) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)dst, 16, vo, kt * 128 + p * 64 * K, 0, 0);
  };

  int rd[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) rd[ks] = (lane & 15) * 128 + (((4 * ks + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4);
  auto frag = [&](int slot, int ks, int o, int blk) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(smem + slot * HS + ((o ? wn : wm) * 8 + blk) * 2048 + rd[ks]);
  };

  f32x4 acc[8][8];
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // one 32-deep sub-step (see gemm_w4_kernel); FIRST: the tile's first sub-step (C = 0)
  auto sub = [&](bf16x8 (&ca)[8], bf16x8 (&cb)[8], bf16x8 (&na)[8], bf16x8 (&nb)[8], int sa, int sb, int nks,
                 const __amdgpu_buffer_rsrc_t& dr, int kt, int ds, auto first) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (decltype(first)::value)
          acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[j], ca[g], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        else
          acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[j], ca[g], acc[g][j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 3 * g; q < 3 * g + 3 && q < 16; ++q) {
        if (q < 8) nb[q] = frag(sb, nks, 1, q);
        else na[q - 8] = frag(sa, nks, 0, q - 8);
      }
      piece(dr, g, kt, ds);
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue (first tile only): k-tiles 0 and 1 (of the next tile when nk == ... nk >= 2 here)
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int p = 0; p < 8; ++p) piece((h & 1) ? cur.wr : cur.xr, p, h >> 1, h);
  vm_wait_n<16>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    fa0[g] = frag(0, 0, 0, g);
    fb0[g] = frag(1, 0, 1, g);
  }

  int h0 = 0;  // (2 * global k-tile) % 5 of the current k-tile
  const int ldy = EPI == TILE_EPI_SWIGLU ? (N >> 1) : N;
  const int ml = lane & 15, nq = 4 * (lane >> 4);
  while (true) {
    for (int t = 0; t < nk; ++t) {
      const int sa = h0, sb = h0 + 1 == 5 ? 0 : h0 + 1;
      const int sa1 = h0 + 2 >= 5 ? h0 - 3 : h0 + 2, sb1 = h0 + 3 >= 5 ? h0 - 2 : h0 + 3;
      const int da = h0 + 4 >= 5 ? h0 - 1 : h0 + 4, db = h0;  // A/B half-slots of k-tile t + 2
      // the k-tile two ahead: of this tile, or the next one's (a dummy re-read after the last tile)
      const bool in_cur = t + 2 < nk || nxt.idx >= cnt;
      const __amdgpu_buffer_rsrc_t ax = in_cur ? cur.xr : nxt.xr, aw = in_cur ? cur.wr : nxt.wr;
      const int k2 = t + 2 < nk ? t + 2 : (nxt.idx >= cnt ? nk - 1 : t + 2 - nk);
      if (t == 0)
        sub(fa0, fb0, fa1, fb1, sa, sb, 1, ax, k2, da, std::true_type{});
      else
        sub(fa0, fb0, fa1, fb1, sa, sb, 1, ax, k2, da, std::false_type{});
      lgkm_wait0();
      vm_wait_n<8>();
      __builtin_amdgcn_s_barrier();
      sub(fa1, fb1, fa0, fb0, sa1, sb1, 0, aw, k2, db, std::false_type{});
      h0 = sa1;
    }
    // ---- epilogue of `cur`: acc[i][j][r] = Y[m][n], m = wm*128 + i*16 + (lane & 15),
    // n = wn*128 + j*16 + 4 (lane >> 4) + r; 8-B stores through a descriptor over the tile's rows ----
    {
      const __amdgpu_buffer_rsrc_t yr = rsrc(Y + (long)cur.row0 * ldy, (long)cur.mrows * ldy * 2);
      const int col0 = EPI == TILE_EPI_SWIGLU ? ((cur.n0 + wn * 128) >> 1) : cur.n0 + wn * 128;
      const int ncols = EPI == TILE_EPI_SWIGLU ? (cur.nrows >> 1) - wn * 64 : cur.nrows - wn * 128;
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t ro = (uint32_t)((wm * 128 + i * 16 + ml) * ldy * 2);
        if constexpr (EPI == TILE_EPI_SWIGLU) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float gt = bf2f(f2bf(acc[i][j][r])), up = bf2f(f2bf(acc[i][j + 4][r]));
              o[r] = gt * up / (1.f + __expf(-gt));
            }
            const int c = j * 16 + nq;
            const uint32_t off = c < ncols ? ro + (uint32_t)((col0 + c) * 2) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{pack2(o[0], o[1]), pack2(o[2], o[3])}, yr, off, 0, 0);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const f32x4 v = acc[i][j];
            const int c = j * 16 + nq;
            const uint32_t off = c < ncols ? ro + (uint32_t)((col0 + c) * 2) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])}, yr, off, 0, 0);
          }
        }
      }
    }
    if (nxt.idx >= cnt) break;
    cur = nxt;
    nxt = find(cur.idx + per);
  }
  vm_wait_n<0>();
}

}  // namespace k8sllm

using namespace k8sllm;

// Dense (offsets == nullptr): Y [M][N] (SwiGLU: [M][N / 2]) = X [M][K] . W[N][K]^T.
// Grouped: W [E][N][K] with expert stride w_es elements; M = total expert-sorted rows (the grid
// bound: ceil(M / 256) + E m-tiles); expert e's rows are offsets[e] .. offsets[e + 1] - 1.
// algo 0: 4-wave 128 x 128 wave tiles (gemm_w4_kernel, N % 16 == 0, K % 64 == 0; SwiGLU N % 256);
// algo 2: its persistent form (gemm_w4p_kernel, K >= 128; same shape rules);
// algo 1: 8-wave 128 x 64 wave tiles (gemm_tile256_kernel, N % 256 == 0, K % 64 == 0).
extern "C" int k8sllm_gemm_tile(const void* X, const void* W, void* Y, int M, int N, int K, const int* offsets, int E,
                                long w_es, int epi, int algo, hipStream_t s) {
  if (M <= 0) return 0;
  const bool grouped = offsets != nullptr;
  if (grouped && (E < 1 || E > 256)) return -1;
  if ((algo >= 0 && algo <= 5 && algo != 1) || (algo >= 40 && algo <= 45)) {
    if (N % 16 != 0 || K % 64 != 0 || K < 64 || (epi == TILE_EPI_SWIGLU && N % 256 != 0)) return -1;
  } else if (N % 256 != 0 || K % 64 != 0 || K < 64) {
    return -1;
  }
  // 32-bit DMA offsets (X: relative to the tile's first row; W: within one expert / n-tile)
  if ((long)N * K * 2 >= (1L << 31) || 256L * K * 2 >= (1L << 31)) return -3;
  const int n_mt = (M + 255) / 256 + (grouped ? E : 0), n_nt = (N + 255) / 256;
  const long nwg = (long)n_mt * n_nt;
  if (nwg > (1L << 30)) return -2;
  dim3 grid((unsigned)nwg);
#define K8_TILE_LAUNCH(KER_, NT_, EPI_, G_)                                                                         \
  hipLaunchKernelGGL((KER_<EPI_, G_>), grid, dim3(NT_), 0, s, (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y,     \
                     offsets, E, M, N, K, w_es, n_mt, n_nt)
#define K8_TILE_EPI(KER_, NT_)                                                                                     \
  if (grouped) {                                                                                                   \
    if (epi == TILE_EPI_SWIGLU) K8_TILE_LAUNCH(KER_, NT_, TILE_EPI_SWIGLU, true);                                  \
    else K8_TILE_LAUNCH(KER_, NT_, TILE_EPI_BF16, true);                                                          \
  } else {                                                                                                         \
    if (epi == TILE_EPI_SWIGLU) K8_TILE_LAUNCH(KER_, NT_, TILE_EPI_SWIGLU, false);                                 \
    else K8_TILE_LAUNCH(KER_, NT_, TILE_EPI_BF16, false);                                                         \
  }
  if (algo == 2 && K >= 128) {  // persistent: one workgroup per CU (multiple of 8: whole XCDs)
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    grid = dim3((unsigned)max(8, min((long)(cus & ~7), (nwg + 7) & ~7L)));
    K8_TILE_EPI(gemm_w4p_kernel, 256)
  } else if (algo == 0 || algo == 2) {
    K8_TILE_EPI(gemm_w4_kernel, 256)
  } else if (algo == 4 || algo == 5) {  // explicit loop-top lgkmcnt(0) (LGK = 1); 5: + no in-loop DMA (diagnosis)
    if (algo == 5) {
      if (grouped || epi != TILE_EPI_BF16) return -1;
      hipLaunchKernelGGL((gemm_w4_kernel<TILE_EPI_BF16, false, 2, 0, 0, 0, 1, 0, 0, 1>), grid, dim3(256), 0, s,
                         (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt);
    } else {
#define K8_LGK(EPI_, G_)                                                                                             \
  hipLaunchKernelGGL((gemm_w4_kernel<EPI_, G_, 0, 0, 0, 0, 1, 0, 0, 1>), grid, dim3(256), 0, s, (const bf16_t*)X,    \
                     (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt)
      if (grouped) {
        if (epi == TILE_EPI_SWIGLU) K8_LGK(TILE_EPI_SWIGLU, true); else K8_LGK(TILE_EPI_BF16, true);
      } else {
        if (epi == TILE_EPI_SWIGLU) K8_LGK(TILE_EPI_SWIGLU, false); else K8_LGK(TILE_EPI_BF16, false);
      }
#undef K8_LGK
    }
  } else if (algo == 3) {  // register-staged refill (STG = 1)
#define K8_STG(EPI_, G_)                                                                                             \
  hipLaunchKernelGGL((gemm_w4_kernel<EPI_, G_, 0, 0, 0, 0, 1, 0, 1>), grid, dim3(256), 0, s, (const bf16_t*)X,       \
                     (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt)
    if (grouped) {
      if (epi == TILE_EPI_SWIGLU) K8_STG(TILE_EPI_SWIGLU, true); else K8_STG(TILE_EPI_BF16, true);
    } else {
      if (epi == TILE_EPI_SWIGLU) K8_STG(TILE_EPI_SWIGLU, false); else K8_STG(TILE_EPI_BF16, false);
    }
#undef K8_STG
  } else if (algo == 40 || algo == 41) {  // two-barrier schedule of the 4-wave kernel (SCH = 1); 41: no swizzle
    if (grouped) return -1;
#define K8_SCH(SW_)                                                                                                  \
  if (epi == TILE_EPI_SWIGLU)                                                                                        \
    hipLaunchKernelGGL((gemm_w4_kernel<TILE_EPI_SWIGLU, false, 0, 0, 0, 1, SW_>), grid, dim3(256), 0, s,              \
                       (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt);        \
  else                                                                                                               \
    hipLaunchKernelGGL((gemm_w4_kernel<TILE_EPI_BF16, false, 0, 0, 0, 1, SW_>), grid, dim3(256), 0, s,                \
                       (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt)
    if (algo == 40) { K8_SCH(1); } else { K8_SCH(0); }
#undef K8_SCH
  } else if (algo >= 42 && algo <= 44) {  // SCH = 1 with sc1 (device-scope: L1 bypass) DMA loads
    if (grouped) return -1;
#define K8_SC1(CX, CW)                                                                                               \
  if (epi == TILE_EPI_SWIGLU)                                                                                        \
    hipLaunchKernelGGL((gemm_w4_kernel<TILE_EPI_SWIGLU, false, 0, CX, CW, 1, 1>), grid, dim3(256), 0, s,             \
                       (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt);        \
  else                                                                                                               \
    hipLaunchKernelGGL((gemm_w4_kernel<TILE_EPI_BF16, false, 0, CX, CW, 1, 1>), grid, dim3(256), 0, s,               \
                       (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt)
    if (algo == 42) { K8_SC1(16, 16); } else if (algo == 43) { K8_SC1(16, 0); } else { K8_SC1(0, 16); }
#undef K8_SC1
  } else if (algo == 45) {  // SCH = 1 with per-wave staggered DMA issue (WST)
    if (grouped) return -1;
    if (epi == TILE_EPI_SWIGLU)
      hipLaunchKernelGGL((gemm_w4_kernel<TILE_EPI_SWIGLU, false, 0, 0, 0, 1, 1, 1>), grid, dim3(256), 0, s,
                         (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt);
    else
      hipLaunchKernelGGL((gemm_w4_kernel<TILE_EPI_BF16, false, 0, 0, 0, 1, 1, 1>), grid, dim3(256), 0, s,
                         (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt);
  } else if (algo >= 20 && algo <= 23) {  // cache-policy variants of the 4-wave kernel (dense, bf16 out)
    if (grouped || epi != TILE_EPI_BF16) return -1;
#define K8_CP(CX, CW)                                                                                             \
  hipLaunchKernelGGL((gemm_w4_kernel<TILE_EPI_BF16, false, 0, CX, CW>), grid, dim3(256), 0, s, (const bf16_t*)X, \
                     (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt)
    if (algo == 20) K8_CP(17, 0);
    else if (algo == 21) K8_CP(0, 17);
    else if (algo == 22) K8_CP(17, 17);
    else K8_CP(2, 2);
#undef K8_CP
  } else if (algo == 10 || algo == 11) {  // diagnosis builds of the 4-wave kernel (dense, bf16 out)
    if (grouped || epi != TILE_EPI_BF16) return -1;
    if (algo == 10)
      hipLaunchKernelGGL((gemm_w4_kernel<TILE_EPI_BF16, false, 1>), grid, dim3(256), 0, s, (const bf16_t*)X,
                         (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt);
    else
      hipLaunchKernelGGL((gemm_w4_kernel<TILE_EPI_BF16, false, 2>), grid, dim3(256), 0, s, (const bf16_t*)X,
                         (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt);
  } else {
    K8_TILE_EPI(gemm_tile256_kernel, 512)
  }
#undef K8_TILE_EPI
#undef K8_TILE_LAUNCH
  return (int)hipGetLastError();
}
