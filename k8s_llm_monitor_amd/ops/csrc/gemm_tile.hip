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
// EPI_ROPE / EPI_RESID / RS: the qkv projection's rotary embedding, the o / down residual add +
//          next-RMSNorm operands, and the consumers' deferred 1/rms row scale (see TileEpi below).
//
// Structure: 4 waves (one per SIMD), each owning a 128 x 128 quarter of the tile as 64 accumulators
// of v_mfma_f32_16x16x32_bf16 (256 f32 per lane in AGPRs).  Per 32-deep k sub-step a wave reads 16
// ds_read_b128 for 64 MFMAs.
//  * K in 64-deep tiles with 128-B LDS rows, so every DMA row segment is one whole 128-B line.
//  * LDS = a ring of five 32 KiB half-slots (160 KiB, one __shared__ array); half-tile h (A_t = 2t,
//    B_t = 2t + 1) lives in slot h % 5, refilled by LDS-DMA (buffer_load_dwordx4 ... lds against
//    SGPR buffer descriptors of the tile's rows: lane offsets are per-lane constants, the k offset
//    goes in soffset).
//  * fragments of the next sub-step are read in between the current one's MFMAs into the second
//    register set: (t, 1) during (t, 0), (t + 1, 0) during (t, 1).
//  * 128-B LDS rows: logical 16-B chunk c of row r sits at physical chunk c ^ ((r >> 1) & 7)
//    (applied to the DMA source address; the LDS side is lane-linear), so each 16-lane group of a
//    fragment ds_read_b128 (rows 0-15 of a block) hits 16 distinct bank quads.
//  * XCD-aware tile order: workgroup ids are remapped so each XCD runs a contiguous range of
//    logical tiles, ordered in groups of 8 m-tiles (neighbours share A or B through that XCD's L2).
//
// Two refill schedules (SCH):
//  0: one barrier per k-tile, before (t, 1); A_{t+2} DMA'd during (t, 0), B_{t+2} during (t, 1),
//     pieces spread one per 8 MFMAs.
//  1: two barriers per k-tile: the mid-(t, 0) barrier (every wave holds tile t's k-half-1
//     fragments in registers) frees BOTH of tile t's half-slots, so B_{t+2} and A_{t+3} are DMA'd
//     from there on and every piece gets >= ~120 MFMAs to land.  2-6 % faster than SCH 0 on the
//     Llama-3-8B prefill shapes (profiles/r03/gemm_schedules.jsonl).  Its ring addressing is
//     scalar: the tile's five half-slot offsets advance in SGPRs (one conditional subtract) and each
//     sub-step forms one A and one B fragment base VGPR (block reads = base + immediate).  With
//     `(2t + i) % 5` written inline hipcc emitted ~25 mul-hi / per-read address instructions in
//     front of every k-tile's first MFMA; removing them made the kernel 4-5 % faster on every
//     shape (profiles/r03/gemm_ring_addressing.jsonl).
// Measured against hipBLASLt's own gfx950 256x256x64 kernel (profiles/r06/README.md): the same
// instruction mix per k-tile (128 MFMA, 32 ds_read_b128, 16 LDS-DMA pieces); ported its schedule
// (two whole-k-tile buffers, three barriers per k-tile, reads one per two MFMAs, its operand
// order) and four other row swizzles - all within +-1 % of this kernel, bit-identical, removed;
// the 5-7 % gap to it is per-tile and independent of the tile-wave count (1, 4, 16).
// Measured and removed (profiles/r03, r05): an 8-wave 128 x 64-per-wave kernel (0.375 reads per MFMA;
// the round-5 ping-pong form of it, bit-identical, 5-6 % slower), non-temporal residual-epilogue
// stores (-1.9 % on o in isolation, below what an end-to-end A/B resolves),
// a persistent form (spilled), register-staged refill (8-10 % slower: ds_write_b128 costs more
// than the DMA issue), the same tile on v_mfma_f32_32x32x16_bf16 (1-5 % slower), unswizzled rows
// (bank conflicts, 10-15 % slower), L1-bypass / nt cache policies and staggered per-wave issue
// (within 1 %).
#include <type_traits>

#include "common.h"
#include "tile_epi.h"

namespace k8sllm {

namespace {
typedef __attribute__((address_space(3))) void lds_void_t;

template <int N>
__device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
}  // namespace

template <int EPI, bool GROUPED, int SCH, bool RS = false>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                         bf16_t* __restrict__ Y, const int* __restrict__ offsets,
                                                         int E, int M, int N, int K, long w_es, int n_mt, int n_nt,
                                                         TileEpi ep, int wpk) {
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
    const int cl = (lane & 7) ^ ((rl >> 1) & 7);
    soff[0][p] = (uint32_t)(((long)min(rl, mrows - 1) * K + cl * 8) * 2);  // rows past the end: clamped, never stored
    soff[1][p] = (uint32_t)(((long)min(rl, nrows - 1) * K + cl * 8) * 2);
    if (wpk) {  // W fragment-packed [N/16][K/32][64][8]: piece = one contiguous 1-KiB block (n-tile, k-step)
      const int blk = p * 4 + wave, j = min(blk >> 1, (nrows >> 4) - 1);
      soff[1][p] = (uint32_t)(((long)j * (K >> 5) + (blk & 1)) * 1024 + lane * 16);
    }
  }
  const int kstrB = wpk ? 2048 : 128;  // bytes of W per k-tile step, in the piece's soffset
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
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void_t*)dst, 16, soff[1][p], min(kt, nk - 1) * kstrB, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void_t*)dst, 16, soff[0][p], min(kt, nk - 1) * 128, 0, 0);
  };
  auto issue_half = [&](int o, int kt) {
#pragma unroll
    for (int p = 0; p < 8; ++p) piece(o, p, kt, (2 * kt + o) % 5);
  };

  // fragment read: lane row lane & 15 of a 16-row block, 16-B chunk 4 ks + (lane >> 4)
  int rd[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) rd[ks] = (lane & 15) * 128 + (((4 * ks + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4);
  // packed W: the LDS image is the blocks verbatim, block (n-tile, k-step) at (2 n-tile + k-step) KiB:
  // every fragment read is lane-linear (conflict-free without a swizzle)
  int rdB[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) rdB[ks] = wpk ? ks * 1024 + lane * 16 : rd[ks];
  auto frag = [&](int slot, int ks, int o, int blk) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(smem + slot * HS + ((o ? wn : wm) * 8 + blk) * 2048 + (o ? rdB[ks] : rd[ks]));
  };

  float rs_inv = 1.f;  // RS: 1 / rms of this thread's row (threadIdx.x of the tile)
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  // RESID: this lane's first 16 residual chunks (rows rr + 4b of the wave's 128, 16 B at column
  // chunk cc), issued during the last k-tile's second half so they land behind its MFMAs
  u32x4 resq[EPI == TILE_EPI_RESID ? 16 : 1];

  if constexpr (SCH == 1) {
    // Ring addressing: the half-slot byte offsets of the current tile live in SGPRs and rotate
    // by one conditional subtract per tile, and each sub-step forms ONE A and ONE B fragment base
    // VGPR (every block read is that base + an immediate).
    const uint32_t fbA0 = (uint32_t)(rd[0] + wm * 16384), fbA1 = (uint32_t)(rd[1] + wm * 16384);
    const uint32_t fbB0 = (uint32_t)(rdB[0] + wn * 16384), fbB1 = (uint32_t)(rdB[1] + wn * 16384);
    auto rd16 = [&](uint32_t base, int blk) -> bf16x8 {
      return *reinterpret_cast<const bf16x8*>(smem + base + blk * 2048);
    };
    auto pc = [&](int o, int p, int kt, uint32_t slot_bytes) {
      char* dst = smem + slot_bytes + (p * 4 + wave) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(o ? wr : xr, (lds_void_t*)dst, 16, soff[o][p], min(kt, nk - 1) * (o ? kstrB : 128),
                                               0, 0);
    };
    // PM (the ring tail, peeled): 0 = B_{t+2} and A_{t+3} refills; 1 = B_{t+2} only (A_{t+3} is
    // past the end); 2 = no refill; 3 = no refill and, in (t, 1), no reads of tile t+1 (there is
    // none).  The tail issues no dummy pieces (a re-read of the last k-tile kept the counts fixed:
    // 40 of every tile's 1064 pieces per wave, ~4 % of the DMA issue at K = 4096).
    auto sub = [&](auto ph, auto pm, bf16x8 (&ca)[8], bf16x8 (&cb)[8], bf16x8 (&na)[8], bf16x8 (&nb)[8],
                   uint32_t sa, uint32_t sb, uint32_t da, uint32_t db, int t) {
      constexpr int PH = decltype(ph)::value, PM = decltype(pm)::value;
      constexpr bool READS = !(PH == 1 && PM == 3);
      // sa / sb: half-slot bytes of the fragments read here; da / db: B_{t+2}'s / A_{t+3}'s targets
      const uint32_t ba = sa + (PH == 0 ? fbA1 : fbA0), bb = sb + (PH == 0 ? fbB1 : fbB0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int n = g * 8 + j;
          acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[j], ca[g], acc[g][j], 0, 0, 0);
          if (n < 8) {
            if constexpr (READS) nb[n] = rd16(bb, n);
          } else if (n < 16) {
            if constexpr (READS) na[n - 8] = rd16(ba, n - 8);
          } else if (PH == 0 && PM <= 1 && n == 19) {  // frees tile t's half-slots for the refills
            lgkm_wait0();
            __builtin_amdgcn_s_barrier();
          } else if (PH == 0 && PM <= 1 && n >= 22 && (n - 22) % 6 == 0 && (n - 22) / 6 < 7) {
            pc(1, (n - 22) / 6, t + 2, da);
          } else if (PH == 1 && PM <= 1 && n >= 19 && (n - 19) % 5 == 0 && (n - 19) / 5 < 9) {
            const int i = 7 + (n - 19) / 5;
            if (i < 8)
              pc(1, i, t + 2, da);
            else if (PM == 0)
              pc(0, i - 8, t + 3, db);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    // RS: this thread's row partials (row row0 + tid, clamped), loaded ahead of the prologue DMAs
    // so their wait is the prologue's own (a fixed 16 loads: up to 64 partials, extra ones masked)
    f32x4 rsq[RS ? 16 : 1];
    if constexpr (RS) {
      const float* rp = ep.rs_part + (long)(row0 + min((int)threadIdx.x, mrows - 1)) * ep.rs_np;
#pragma unroll
      for (int j = 0; j < 16; ++j) rsq[j] = *reinterpret_cast<const f32x4*>(rp + min(4 * j, ep.rs_np - 4));
    }
    issue_half(0, 0);
    issue_half(1, 0);
    issue_half(0, 1);
    issue_half(1, 1);
    issue_half(0, 2);
    vm_wait_n<24>();
    __builtin_amdgcn_s_barrier();
    if constexpr (RS) {
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (4 * j < ep.rs_np) sum += (rsq[j][0] + rsq[j][1]) + (rsq[j][2] + rsq[j][3]);
      rs_inv = rsqrtf(sum / (float)K + ep.rs_eps);
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      fa0[g] = frag(0, 0, 0, g);
      fb0[g] = frag(1, 0, 1, g);
    }
    // half-slot bytes of tile t: S0 = (2t % 5) HS (A_t), S1 = ((2t + 1) % 5) HS (B_t), S2 / S3 =
    // tile t+1's.  Tile t+1: S0' = S2, S1' = S3, S2' = ((2t + 4) % 5) HS, S3' = S0.
    uint32_t S0 = 0, S1 = HS, S2 = 2 * HS, S3 = 3 * HS;
    auto rotate = [&]() {
      const uint32_t s4 = S0 == 0 ? 4 * HS : S0 - HS, s0 = S0;
      S0 = S2;
      S1 = S3;
      S2 = s4;
      S3 = s0;
    };
    // vmcnt at the mid-tile wait: B_{t+1} must have landed; younger are A_{t+2} (8) + B_{t+2}'s
    // first 7 pieces (15) in the steady state and at t = nk - 3, nothing from t = nk - 2 on
    for (int t = 0; t < nk - 3; ++t) {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the previous sub-step's reads, explicitly
      sub(P0{}, P0{}, fa0, fb0, fa1, fb1, S0, S1, S0, S1, t);
      vm_wait_n<15>();
      __builtin_amdgcn_s_barrier();
      sub(P1{}, P0{}, fa1, fb1, fa0, fb0, S2, S3, S0, S1, t);
      rotate();
    }
    {  // t = nk - 3 (host: nk >= 3): B_{nk-1} is the last refill
      const int t = nk - 3;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      sub(P0{}, P1{}, fa0, fb0, fa1, fb1, S0, S1, S0, S1, t);
      vm_wait_n<15>();
      __builtin_amdgcn_s_barrier();
      sub(P1{}, P1{}, fa1, fb1, fa0, fb0, S2, S3, S0, S1, t);
      rotate();
    }
    {  // t = nk - 2: every piece issued so far must land (B_{nk-1} is read in (t, 1))
      const int t = nk - 2;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      sub(P0{}, P2{}, fa0, fb0, fa1, fb1, S0, S1, S0, S1, t);
      vm_wait_n<0>();
      __builtin_amdgcn_s_barrier();
      sub(P1{}, P2{}, fa1, fb1, fa0, fb0, S2, S3, S0, S1, t);
      rotate();
    }
    {  // t = nk - 1: the last k-tile; (t, 1) reads nothing - RESID issues its residual loads here
      const int t = nk - 1;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      sub(P0{}, P3{}, fa0, fb0, fa1, fb1, S0, S1, S0, S1, t);
      if constexpr (EPI == TILE_EPI_RESID) {
        const __amdgpu_buffer_rsrc_t rres = rsrc(ep.resid + (long)row0 * N, (long)mrows * N * 2);
        const uint32_t ro = (uint32_t)(((wm * 128 + (lane >> 4)) * N + n0 + wn * 128 + (lane & 15) * 8) * 2);
#pragma unroll
        for (int b = 0; b < 16; ++b)
          resq[b] = __builtin_amdgcn_raw_buffer_load_b128(rres, ro + (uint32_t)(4 * b * N * 2), 0, 0);
      }
      sub(P1{}, P3{}, fa1, fb1, fa0, fb0, S2, S3, S0, S1, t);
    }
  } else {
    // One 32-deep sub-step: 64 MFMAs from (ca, cb), each carrying at most one other instruction in
    // its shadow.  The 8 DMA pieces of the sub-step ride MFMAs 4, 12, ..., 60 - evenly spread: an
    // LDS-DMA instruction holds its wave's issue for tens of cycles (MI355X_MICROARCH.md, LDS-DMA
    // piece issue cost), and bunched pieces starve the matrix pipe (all 16 pieces of a k-tile in
    // one sub-step: 8-13 % slower).  The 16 fragment reads of the next sub-step ride the other
    // MFMAs from the first on (W blocks first), done by MFMA 17.
    auto sub = [&](bf16x8 (&ca)[8], bf16x8 (&cb)[8], bf16x8 (&na)[8], bf16x8 (&nb)[8], int sa, int sb, int nks,
                   int o, int kt, int ds) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int n = g * 8 + j;
          acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[j], ca[g], acc[g][j], 0, 0, 0);
          const int q = n - (n > 4) - (n > 12);  // read index: skips the DMA slots 4 and 12
          if (j == 4) {
            piece(o, g, kt, ds);
          } else if (q < 8) {
            nb[q] = frag(sb, nks, 1, q);
          } else if (q < 16) {
            na[q - 8] = frag(sa, nks, 0, q - 8);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    // prologue: A_0 B_0 A_1 B_1 in flight; tile 0 landed -> read its first k-half
    issue_half(0, 0);
    issue_half(1, 0);
    issue_half(0, 1);
    issue_half(1, 1);
    vm_wait_n<16>();
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      fa0[g] = frag(0, 0, 0, g);
      fb0[g] = frag(1, 0, 1, g);
    }
    for (int t = 0; t < nk; ++t) {
      const int sa = (2 * t) % 5, sb = (2 * t + 1) % 5;        // tile t's half-slots
      const int sa1 = (2 * t + 2) % 5, sb1 = (2 * t + 3) % 5;  // tile t+1's
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): see SCH 1
      // (t, 0): MFMAs on k-half 0; read k-half 1 of tile t; DMA A_{t+2}
      sub(fa0, fb0, fa1, fb1, sa, sb, 1, 0, t + 2, (2 * t + 4) % 5);
      lgkm_wait0();
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
  constexpr bool SWG = EPI == TILE_EPI_SWIGLU || EPI == TILE_EPI_SWIGLU8;
  constexpr int OUTW = SWG ? 64 : 128;  // output columns of this wave's quarter
  constexpr int RS_ = OUTW * 2 + 16;                       // LDS row stride (16-B pad: 2-way writes)
  char* stage = smem + wave * (128 * RS_);
  const int ml = lane & 15, nq = 4 * (lane >> 4);
  const int rr = lane >> 4, cc = lane & 15;
  uint4 nwv{};
  if constexpr (EPI == TILE_EPI_RESID) nwv = *reinterpret_cast<const uint4*>(ep.norm_w + n0 + wn * 128 + cc * 8);
  // RS: each thread's row scale through LDS (after the staging area) to the lanes holding the row
  float sc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sc[i] = 1.f;
  if constexpr (RS) {
    float* inv_s = reinterpret_cast<float*>(smem + 4 * 128 * (128 * 2 + 16));
    inv_s[threadIdx.x] = rs_inv;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) sc[i] = inv_s[wm * 128 + i * 16 + ml];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    __builtin_amdgcn_sched_barrier(0);  // one row block's accumulators at a time (no hoisted AGPR reads)
    char* srow = stage + (i * 16 + ml) * RS_ + nq * 2;
    if constexpr (EPI == TILE_EPI_SWIGLU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gt = bf2f(f2bf(acc[i][j][r] * sc[i])), up = bf2f(f2bf(acc[i][j + 4][r] * sc[i]));
          o[r] = gt * up / (1.f + __expf(-gt));
        }
        *reinterpret_cast<uint2*>(srow + j * 32) = uint2{pack2(o[0], o[1]), pack2(o[2], o[3])};
      }
    } else if constexpr (EPI == TILE_EPI_SWIGLU8) {
      // [8 gate | 8 up] per 16-column n-tile j: gate column 4 q + r (q = 0, 1: lanes 0-31) pairs
      // with up column 8 + 4 q + r in lane + 32.  One v_permlane32_swap per register puts (gate,
      // up) in both lane halves; lanes 0-31 finish r = 0, 1 and lanes 32-63 r = 2, 3 of feature
      // 8 j + 4 q + r (4 bytes each).
      const int hi = lane >> 5, qq = (lane >> 4) & 1;
      char* srow8 = stage + (i * 16 + ml) * RS_ + (8 * qq + 4 * hi);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float g[4], u[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t v = __float_as_uint(acc[i][j][r] * sc[i]);
          const auto pr = __builtin_amdgcn_permlane32_swap(v, v, false, false);
          g[r] = __uint_as_float(pr[0]);
          u[r] = __uint_as_float(pr[1]);
        }
        float o[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const float gt = bf2f(f2bf(hi ? g[2 + k] : g[k])), up = bf2f(f2bf(hi ? u[2 + k] : u[k]));
          o[k] = gt * up / (1.f + __expf(-gt));
        }
        *reinterpret_cast<uint32_t*>(srow8 + j * 16) = pack2(o[0], o[1]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f32x4 v = acc[i][j] * sc[i];
        *reinterpret_cast<uint2*>(srow + j * 32) = uint2{pack2(v[0], v[1]), pack2(v[2], v[3])};
      }
    }
  }
  lgkm_wait0();
  if constexpr (EPI == TILE_EPI_RESID) {
    // lane (rr, cc): row rr + 4b, columns cc*8 .. +7 of the wave's quarter; N % 128 == 0 (host)
    const __amdgpu_buffer_rsrc_t rres = rsrc(ep.resid + (long)row0 * N, (long)mrows * N * 2);
    const __amdgpu_buffer_rsrc_t rhw = rsrc(ep.hw + (long)row0 * N, (long)mrows * N * 2);
    const uint32_t ro = (uint32_t)(((wm * 128 + rr) * N + n0 + wn * 128 + cc * 8) * 2);
    float wf[8];
    unpack8(nwv, wf);
    const int ss_np = N >> 7, ssc = (n0 + wn * 128) >> 7;
#pragma unroll
    for (int b = 0; b < 32; ++b) {
      const int r = rr + 4 * b;
      const uint4 yv = *reinterpret_cast<const uint4*>(stage + r * RS_ + cc * 16);
      float y[8], rv[8], h[8], hw[8];
      unpack8(yv, y);
      const u32x4 rb = resq[b & 15];
      if (b < 16) resq[b] = __builtin_amdgcn_raw_buffer_load_b128(rres, ro + (uint32_t)(4 * (b + 16) * N * 2), 0, 0);
      unpack8(uint4{rb[0], rb[1], rb[2], rb[3]}, rv);
      float ss = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        h[e] = bf2f(f2bf(y[e] + rv[e]));
        ss += h[e] * h[e];
        hw[e] = h[e] * wf[e];
      }
      const uint4 hq = pack8(h), wq = pack8(hw);
      const uint32_t off = ro + (uint32_t)(4 * b * N * 2);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{hq.x, hq.y, hq.z, hq.w}, rres, off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{wq.x, wq.y, wq.z, wq.w}, rhw, off, 0, 0);
      ss = row16_sum(ss);
      const int grow = wm * 128 + r;
      if (cc == 0 && grow < mrows) ep.ss_out[(long)(row0 + grow) * ss_np + ssc] = ss;
    }
    return;
  }
  if constexpr (EPI == TILE_EPI_ROPE) {
    const int head = (n0 + wn * 128) >> 7;
    if (head < ep.rope_heads && nrows - wn * 128 >= 128) {
      // one lane per (row, chunk pair c, c + 8): 8 rows per pass, 16 passes over the quarter's rows
      const int c = lane & 7, rsub = lane >> 3;
      bf16_t* ybase = Y + (long)row0 * N + n0 + wn * 128;
#pragma unroll 4
      for (int pass = 0; pass < 16; ++pass) {
        const int r = pass * 8 + rsub, grow = wm * 128 + r;
        if (grow >= mrows) continue;
        const uint4 a = *reinterpret_cast<const uint4*>(stage + r * RS_ + c * 16);
        const uint4 b = *reinterpret_cast<const uint4*>(stage + r * RS_ + (c + 8) * 16);
        const float* cs = ep.cos_sin + (long)ep.positions[row0 + grow] * 128;
        const float4 c0 = *reinterpret_cast<const float4*>(cs + c * 8), c1 = *reinterpret_cast<const float4*>(cs + c * 8 + 4);
        const float4 s0 = *reinterpret_cast<const float4*>(cs + 64 + c * 8),
                     s1 = *reinterpret_cast<const float4*>(cs + 64 + c * 8 + 4);
        const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        float x1[8], x2[8], o1[8], o2[8];
        unpack8(a, x1);
        unpack8(b, x2);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o1[j] = x1[j] * cc[j] - x2[j] * ss[j];
          o2[j] = x2[j] * cc[j] + x1[j] * ss[j];
        }
        bf16_t* yr = ybase + (long)grow * N;
        *reinterpret_cast<uint4*>(yr + c * 8) = pack8(o1);
        *reinterpret_cast<uint4*>(yr + 64 + c * 8) = pack8(o2);
      }
      return;
    }
  }
  constexpr int CPR = OUTW / 8;  // 16-B chunks per row
  constexpr int RPI = 64 / CPR;  // rows per wave instruction
  const int ldy = SWG ? (N >> 1) : N;
  const int col0 = SWG ? ((n0 + wn * 128) >> 1) : n0 + wn * 128;
  const int ncols = SWG ? (nrows >> 1) - wn * 64 : nrows - wn * 128;
  const int rr2 = lane / CPR, cc2 = lane % CPR;
  // branch-free masked stores: a buffer descriptor over this m-tile's rows drops every store past
  // row mrows (out of range), and a lane whose columns are past N gets an out-of-range offset
  const __amdgpu_buffer_rsrc_t yr = rsrc(Y + (long)row0 * ldy, (long)mrows * ldy * 2);
  const uint32_t yo = cc2 * 8 < ncols ? (uint32_t)(((wm * 128 + rr2) * ldy + col0 + cc2 * 8) * 2) : 0x80000000u;
#pragma unroll
  for (int b = 0; b < 128 / RPI; b += 8) {  // 8 row groups per batch: reads issued back to back
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const u32x4*>(stage + ((b + u) * RPI + rr2) * RS_ + cc2 * 16);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      __builtin_amdgcn_raw_buffer_store_b128(v[u], yr, yo + (uint32_t)((b + u) * RPI * ldy * 2), 0, 0);
  }
}

}  // namespace k8sllm

using namespace k8sllm;

// Dense (offsets == nullptr): Y [M][N] (SwiGLU: [M][N / 2]) = X [M][K] . W[N][K]^T.
// Grouped: W [E][N][K] with expert stride w_es elements; M = total expert-sorted rows (the grid
// bound: ceil(M / 256) + E m-tiles); expert e's rows are offsets[e] .. offsets[e + 1] - 1.
// Shapes: N % 16 == 0 (SwiGLU: N % 256 == 0), K % 64 == 0.  algo: the refill schedule (0 or 1).
// wpk: W is fragment-packed ([E][N/16][K/32][64][8], ops.pack_skinny - the decode GEMMs' layout)
// instead of row-major: every W DMA piece is one contiguous 1-KiB block, read lane-linear from LDS.
extern "C" int k8sllm_gemm_tile(const void* X, const void* W, void* Y, int M, int N, int K, const int* offsets, int E,
                                long w_es, int epi, int algo, const int* rope_pos, const float* rope_cs,
                                int rope_heads, const float* rs_part, int rs_np, float rs_eps, void* resid, void* hw,
                                const void* norm_w, float* ss_out, int wpk, hipStream_t s) {
  if (M <= 0) return 0;
  const bool grouped = offsets != nullptr;
  const bool rs = rs_part != nullptr;
  if (grouped && (E < 1 || E > 256)) return -1;
  if (algo < 0 || algo > 1) return -1;
  if (algo == 1 && K < 192) {  // schedule 1's peeled ring tail needs three k-tiles
    if (epi == TILE_EPI_RESID || rs_part != nullptr) return -1;
    algo = 0;
  }
  const bool swg = epi == TILE_EPI_SWIGLU || epi == TILE_EPI_SWIGLU8;
  if (N % 16 != 0 || K % 64 != 0 || K < 64 || (swg && N % 256 != 0) || epi < 0 || epi > 4) return -1;
  if (epi == TILE_EPI_ROPE && (grouped || N % 128 != 0 || rope_pos == nullptr || rope_cs == nullptr)) return -1;
  if (epi == TILE_EPI_RESID && (grouped || rs || N % 128 != 0 || resid == nullptr || hw == nullptr ||
                                norm_w == nullptr || ss_out == nullptr || algo != 1))
    return -1;
  // row scale: the fused consumers only (qkv + RoPE, gate_up + SwiGLU), schedule 1
  if (rs && (grouped || algo != 1 || rs_np < 4 || rs_np > 64 || rs_np % 4 != 0 ||
             (epi != TILE_EPI_ROPE && !swg)))
    return -1;
  const TileEpi ep{rope_pos, rope_cs, rope_heads, rs_part, rs_np, rs_eps, (bf16_t*)resid, (bf16_t*)hw,
                   (const bf16_t*)norm_w, ss_out};
  // 32-bit DMA offsets (X: relative to the tile's first row; W: within one expert / n-tile)
  if ((long)N * K * 2 >= (1L << 31) || 256L * K * 2 >= (1L << 31)) return -3;
  if (epi == TILE_EPI_RESID && 256L * N * 2 >= (1L << 31)) return -3;
  const int n_mt = (M + 255) / 256 + (grouped ? E : 0), n_nt = (N + 255) / 256;
  const long nwg = (long)n_mt * n_nt;
  if (nwg > (1L << 30)) return -2;
  const dim3 grid((unsigned)nwg);
#define K8_TILE_LAUNCH(EPI_, G_, SCH_, RS_)                                                                          \
  hipLaunchKernelGGL((gemm_w4_kernel<EPI_, G_, SCH_, RS_>), grid, dim3(256), 0, s, (const bf16_t*)X,                \
                     (const bf16_t*)W, (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt, ep, wpk)
#define K8_TILE_SCH(SCH_)                                                                                            \
  if (grouped) {                                                                                                     \
    if (epi == TILE_EPI_SWIGLU) K8_TILE_LAUNCH(TILE_EPI_SWIGLU, true, SCH_, false);                                  \
    else if (epi == TILE_EPI_SWIGLU8) K8_TILE_LAUNCH(TILE_EPI_SWIGLU8, true, SCH_, false);                           \
    else K8_TILE_LAUNCH(TILE_EPI_BF16, true, SCH_, false);                                                           \
  } else {                                                                                                           \
    if (epi == TILE_EPI_SWIGLU) K8_TILE_LAUNCH(TILE_EPI_SWIGLU, false, SCH_, false);                                 \
    else if (epi == TILE_EPI_SWIGLU8) K8_TILE_LAUNCH(TILE_EPI_SWIGLU8, false, SCH_, false);                          \
    else if (epi == TILE_EPI_ROPE) K8_TILE_LAUNCH(TILE_EPI_ROPE, false, SCH_, false);                                \
    else K8_TILE_LAUNCH(TILE_EPI_BF16, false, SCH_, false);                                                          \
  }
  if (epi == TILE_EPI_RESID) {
    K8_TILE_LAUNCH(TILE_EPI_RESID, false, 1, false);
  } else if (rs) {
    if (epi == TILE_EPI_SWIGLU) K8_TILE_LAUNCH(TILE_EPI_SWIGLU, false, 1, true);
    else if (epi == TILE_EPI_SWIGLU8) K8_TILE_LAUNCH(TILE_EPI_SWIGLU8, false, 1, true);
    else K8_TILE_LAUNCH(TILE_EPI_ROPE, false, 1, true);
  } else if (algo == 1) {
    K8_TILE_SCH(1)
  } else {
    K8_TILE_SCH(0)
  }
#undef K8_TILE_SCH
#undef K8_TILE_LAUNCH
  return (int)hipGetLastError();
}
