// 256 x 256 prefill GEMM, 8-wave PING-PONG schedule (gfx950): the same tile, operand layout, XCD
// remap, LDS swizzle and fused epilogues as gemm_tile.hip's 4-wave kernel, with its matrix pipe
// kept busy by a different division of labour.
//
// Why.  The 4-wave kernel (one 128 x 128 wave per SIMD) issues its own LDS-DMA refill pieces
// between its MFMAs; an LDS-DMA instruction holds the issuing wave for tens to ~185 cycles
// (MI355X_MICROARCH.md per-instruction constants), and with one wave per SIMD nothing else feeds
// the matrix pipe meanwhile: 1.47 us per 64-deep k-tile with the in-loop DMA against 1.19-1.28
// without it (profiles/r03/README.md), PMC MFMA busy 74.8 % (profiles/r04).
//
// Here every SIMD hosts two waves, one from each half of the workgroup:
//   group 0 (waves 0-3) computes tile rows 0-127, group 1 (waves 4-7) rows 128-255; wave w4 of a
//   group owns columns 64 w4 .. 64 w4 + 63 (8 x 4 accumulators of v_mfma_f32_16x16x32_bf16 =
//   128 AGPRs, so two waves fit one SIMD's register file);
//   the groups alternate roles every segment, separated by s_barrier:
//       segment 2t:     group 0 runs k-tile t's 64 MFMAs | group 1 reads its fragments of tile t
//                                                          and issues refill DMA
//       segment 2t + 1: group 1 runs k-tile t's MFMAs    | group 0 reads tile t + 1, issues DMA
//   (MI355X_MICROARCH.md "Two waves per SIMD": one wave in a matrix segment beside its partner in
//   a load segment).  A computing wave's segment is MFMAs only; all DMA issue, fragment reads and
//   waits sit in the partner's segment.
//
// LDS: ten 16 KiB units (128 rows x 128 B, the 4-wave kernel's row format and XOR swizzle); k-tile
// t occupies units (4t + j) % 10, j = 0 A rows 0-127, 1 / 2 W rows 0-127 / 128-255, 3 A rows
// 128-255.  Refills of tile t + 2: A-top and W-low by group 1 in segment 2t, W-high and A-bottom by
// group 0 in segment 2t + 1 (8 pieces of 1 KiB per wave each time) - each into a unit whose last
// reader finished at least one barrier earlier; every issuing wave retires its pieces with a
// counted vmcnt before the barrier that precedes their first read (group 1 at the end of its next
// load segment, group 0 at the end of its next compute segment).
//
// Epilogue: the accumulators (row-scaled for RS) are staged as a bf16 256 x 256 tile in the idle
// ring, then all 512 threads run the epilogue over LDS rows: plain bf16 rows, SwiGLU pairs, RoPE
// pairs or the residual-add / next-norm operands - bit-identical to the 4-wave kernel's epilogues
// (each applies the same operations to the same bf16-rounded products).
#include <type_traits>

#include "common.h"
#include "tile_epi.h"

namespace k8sllm {

namespace {
typedef __attribute__((address_space(3))) void lds_void_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void pp_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void pp_lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
}  // namespace

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pp_rsrc(const void* base, long bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}

template <int EPI, bool GROUPED, bool RS, int SCH>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                         bf16_t* __restrict__ Y, const int* __restrict__ offsets, int E,
                                                         int M, int N, int K, long w_es, int n_mt, int n_nt,
                                                         TileEpi ep) {
  constexpr int U = 16384;  // one LDS unit: 128 rows x 128 B
  __shared__ __attribute__((aligned(16))) char smem[10 * U];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wave >> 2, w4 = wave & 3;

  // ---- logical tile: bijective XCD remap, then groups of 8 m-tiles (as gemm_w4_kernel) ----
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
  const int nk = K >> 6;

  const __amdgpu_buffer_rsrc_t xr = pp_rsrc(reinterpret_cast<const char*>(X) + (long)row0 * K * 2, (long)mrows * K * 2);
  const __amdgpu_buffer_rsrc_t wr = pp_rsrc(reinterpret_cast<const char*>(Wt) + (long)n0 * K * 2, (long)nrows * K * 2);

  // ---- this wave's refill pieces: group 1 fills units j = 0 (A rows 0-127) and 1 (W rows 0-127),
  // group 0 units j = 2 (W rows 128-255) and 3 (A rows 128-255).  Piece p (0..3) of a unit: rows
  // (4p + w4) * 8 .. + 7 of the unit; lane -> row + (lane >> 3), physical 16-B chunk lane & 7
  // (logical chunk c of row r sits at c ^ ((r >> 1) & 7): the swizzle is applied to the source) ----
  // piece p's source offsets are recomputed per refill (a few VALU) rather than held in 8 VGPRs
  // (written inline: a lambda called from the refill lambda breaks hipcc's host-side stubs)
  const int lim0 = (g ? mrows : nrows) - 1, lim1 = (g ? nrows : mrows) - 1;  // g1: A, W; g0: W, A
  const int rbase = g ? 0 : 128;
  const __amdgpu_buffer_rsrc_t rs0 = g ? xr : wr, rs1 = g ? wr : xr;
  const int j0 = g ? 0 : 2;  // unit index (within a k-tile) of this wave's first refill unit
  auto unit = [](int t, int j) -> uint32_t { return (uint32_t)(((4 * t + j) % 10) * U); };
  // SCH 1: group 1 refills units 0-2 of tile t + 2 in segment 2t (12 pieces per wave), group 0 only
  // unit 3 in segment 2t + 1 (4 pieces), so every piece is read no earlier than two segments after
  // its issue (SCH 0: group 0's W-high pieces are read one segment after theirs)
  const int lim2 = nrows - 1;  // SCH 1, group 1's third unit: W rows 128-255
  // the 8 refill pieces of k-tile kt by this wave (k-tiles past the end are never requested)
  auto refill = [&](int kt) {
    if constexpr (SCH == 1) {
      if (g == 0) {  // unit 3: A rows 128-255
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int rl = (p * 4 + w4) * 8 + (lane >> 3);
          const int cl = (lane & 7) ^ ((rl >> 1) & 7);
          const uint32_t so = (uint32_t)(((long)min(128 + rl, mrows - 1) * K + cl * 8) * 2);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void_t*)(smem + unit(kt, 3) + (p * 4 + w4) * 1024), 16, so,
                                                   kt * 128, 0, 0);
        }
        return;
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {  // group 1's third unit (2): W rows 128-255
        const int rl = (p * 4 + w4) * 8 + (lane >> 3);
        const int cl = (lane & 7) ^ ((rl >> 1) & 7);
        const uint32_t so = (uint32_t)(((long)min(128 + rl, lim2) * K + cl * 8) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void_t*)(smem + unit(kt, 2) + (p * 4 + w4) * 1024), 16, so,
                                                 kt * 128, 0, 0);
      }
    }
    const uint32_t u0 = unit(kt, j0), u1 = unit(kt, j0 + 1);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int rl = (p * 4 + w4) * 8 + (lane >> 3);
      const int cl = (lane & 7) ^ ((rl >> 1) & 7);
      const uint32_t so = (uint32_t)(((long)min(rbase + rl, lim0) * K + cl * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs0, (lds_void_t*)(smem + u0 + (p * 4 + w4) * 1024), 16, so,
                                               kt * 128, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int rl = (p * 4 + w4) * 8 + (lane >> 3);
      const int cl = (lane & 7) ^ ((rl >> 1) & 7);
      const uint32_t so = (uint32_t)(((long)min(rbase + rl, lim1) * K + cl * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs1, (lds_void_t*)(smem + u1 + (p * 4 + w4) * 1024), 16, so,
                                               kt * 128, 0, 0);
    }
  };

  // fragment read: lane row lane & 15 of a 16-row block, 16-B chunk 4 ks + (lane >> 4)
  int rd[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) rd[ks] = (lane & 15) * 128 + (((4 * ks + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4);
  const int ja = g ? 3 : 0, jb = 1 + (w4 >> 1);  // units of this wave's A rows and W columns
  const int bb = (w4 & 1) * 4;                   // first 16-row W block of this wave in its unit
  bf16x8 fa[2][8], fb[2][4];
  auto load_frags = [&](int t) {
    const char* pa = smem + unit(t, ja);
    const char* pb = smem + unit(t, jb) + bb * 2048;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[ks][j] = *reinterpret_cast<const bf16x8*>(pb + j * 2048 + rd[ks]);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[ks][i] = *reinterpret_cast<const bf16x8*>(pa + i * 2048 + rd[ks]);
    }
  };
  f32x4 acc[8][4];  // zeroed after the prologue (the row-scale partials' registers are free by then)
  auto compute = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ks][j], fa[ks][i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // RS: this thread's row scale (row row0 + threadIdx.x for threads 0..255), loaded ahead of the
  // prologue DMA so its wait is the prologue's own
  float rs_inv = 1.f;
  f32x4 rsq[RS ? 16 : 1];
  if constexpr (RS) {
    const float* rp = ep.rs_part + (long)(row0 + min((int)(threadIdx.x & 255), mrows - 1)) * ep.rs_np;
#pragma unroll
    for (int j = 0; j < 16; ++j) rsq[j] = *reinterpret_cast<const f32x4*>(rp + min(4 * j, ep.rs_np - 4));
  }

  // ---- prologue: k-tiles 0 and 1 (each wave its two units of each), then group 0 reads tile 0 ----
  refill(0);
  if (nk > 1) refill(1);
  if constexpr (RS) {  // the partials are the oldest loads: their wait leaves the DMA pieces in flight
    if (SCH == 1 && g == 0)
      pp_vm_wait<8>();
    else if (SCH == 1)
      pp_vm_wait<24>();
    else
      pp_vm_wait<16>();
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      asm volatile("" : "+v"(rsq[j][0]), "+v"(rsq[j][1]), "+v"(rsq[j][2]), "+v"(rsq[j][3]));
      if (4 * j < ep.rs_np) sum += (rsq[j][0] + rsq[j][1]) + (rsq[j][2] + rsq[j][3]);
    }
    rs_inv = rsqrtf(sum / (float)K + ep.rs_eps);
  }
  pp_vm_wait<0>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // ---- main loop: two segments per k-tile; each group runs its own straight-line loop (the
  // same barrier count), so a fragment set lives from its load segment to its compute segment ----
  if (g == 0) {
    load_frags(0);  // segment -1 (group 1 idle)
    pp_lgkm_wait0();
    __builtin_amdgcn_s_barrier();
    for (int t = 0; t < nk; ++t) {
      compute();  // segment 2t
      if constexpr (SCH == 0)
        pp_vm_wait<0>();  // this wave's refill of tile t + 1 (segment 2t - 1): read from segment 2t + 1 on
      __builtin_amdgcn_s_barrier();
      if (t + 1 < nk) {  // segment 2t + 1: tile t + 1's fragments; refill tile t + 2's W-high / A-bottom
        load_frags(t + 1);
        if (t + 2 < nk) {
          refill(t + 2);
          pp_lgkm_wait0();
          if constexpr (SCH == 1) pp_vm_wait<4>();  // A-bottom of tile t + 1 (segment 2t - 1) landed
        } else {
          pp_lgkm_wait0();
          if constexpr (SCH == 1) pp_vm_wait<0>();
        }
      }
      __builtin_amdgcn_s_barrier();
    }
  } else {
    __builtin_amdgcn_s_barrier();
    for (int t = 0; t < nk; ++t) {
      load_frags(t);  // segment 2t: tile t's fragments; refill tile t + 2's A-top / W-low
      if (t + 2 < nk) {
        refill(t + 2);
        pp_lgkm_wait0();
        if constexpr (SCH == 1)
          pp_vm_wait<12>();
        else
          pp_vm_wait<8>();  // this wave's refill of tile t + 1 (segment 2t - 2) landed; t + 2's in flight
      } else {
        pp_lgkm_wait0();
        pp_vm_wait<0>();
      }
      __builtin_amdgcn_s_barrier();
      compute();  // segment 2t + 1
      __builtin_amdgcn_s_barrier();
    }
  }
  pp_vm_wait<0>();

  // ---- epilogue: stage the tile as bf16 rows (row-scaled for RS), then run it from LDS ----
  constexpr int RSB = 256 * 2 + 16;  // LDS row stride of the staged tile (16-B pad)
  float sc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sc[i] = 1.f;
  if constexpr (RS) {
    float* inv_s = reinterpret_cast<float*>(smem + 256 * RSB);
    if (threadIdx.x < 256) inv_s[threadIdx.x] = rs_inv;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) sc[i] = inv_s[g * 128 + i * 16 + (lane & 15)];
  }
  {
    const int ml = lane & 15, nq = 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_barrier(0);  // one row block's accumulators at a time
      char* srow = smem + (g * 128 + i * 16 + ml) * RSB + (w4 * 64 + nq) * 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = acc[i][j] * sc[i];
        *reinterpret_cast<uint2*>(srow + j * 32) = uint2{pack2(v[0], v[1]), pack2(v[2], v[3])};
      }
    }
  }
  __syncthreads();
  const int tid = threadIdx.x;

  if constexpr (EPI == TILE_EPI_RESID) {
    // thread: row tid / 32 + 16 pass, 8 columns (tid & 31) * 8; the 16 threads of one 128-column
    // group are 16 aligned consecutive lanes (row16_sum)
    const __amdgpu_buffer_rsrc_t rres = pp_rsrc(ep.resid + (long)row0 * N, (long)mrows * N * 2);
    const __amdgpu_buffer_rsrc_t rhw = pp_rsrc(ep.hw + (long)row0 * N, (long)mrows * N * 2);
    const int c = tid & 31, r0 = tid >> 5;
    float wf[8];
    unpack8(*reinterpret_cast<const uint4*>(ep.norm_w + n0 + c * 8), wf);
    const int ss_np = N >> 7, ssc = (n0 >> 7) + (c >> 4);
    u32x4 rq[16];
#pragma unroll
    for (int pass = 0; pass < 16; ++pass) {
      const uint32_t off = (uint32_t)((((r0 + 16 * pass) * N) + n0 + c * 8) * 2);
      rq[pass] = __builtin_amdgcn_raw_buffer_load_b128(rres, off, 0, 0);
    }
#pragma unroll
    for (int pass = 0; pass < 16; ++pass) {
      const int r = r0 + 16 * pass;
      const uint4 yv = *reinterpret_cast<const uint4*>(smem + r * RSB + c * 16);
      float y[8], rv[8], h[8], hw[8];
      unpack8(yv, y);
      unpack8(uint4{rq[pass][0], rq[pass][1], rq[pass][2], rq[pass][3]}, rv);
      float ss = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        h[e] = bf2f(f2bf(y[e] + rv[e]));
        ss += h[e] * h[e];
        hw[e] = h[e] * wf[e];
      }
      const uint4 hq = pack8(h), wq = pack8(hw);
      const uint32_t off = (uint32_t)(((r * N) + n0 + c * 8) * 2);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{hq.x, hq.y, hq.z, hq.w}, rres, off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{wq.x, wq.y, wq.z, wq.w}, rhw, off, 0, 0);
      ss = row16_sum(ss);
      if ((c & 15) == 0 && r < mrows) ep.ss_out[(long)(row0 + r) * ss_np + ssc] = ss;
    }
    return;
  } else if constexpr (EPI == TILE_EPI_SWIGLU) {
    // output row: 128 features = 2 groups of [64 gate | 64 up] staged columns; thread: row tid / 16
    // + 32 pass, features (tid & 15) * 8 .. + 7
    const int ldy = N >> 1;
    const int c = tid & 15, r0 = tid >> 4, gg = c >> 3, cc = c & 7;
    const __amdgpu_buffer_rsrc_t yr = pp_rsrc(Y + (long)row0 * ldy, (long)mrows * ldy * 2);
    const int col = (n0 >> 1) + gg * 64 + cc * 8;
    const uint32_t yo = gg * 128 < nrows ? (uint32_t)((r0 * ldy + col) * 2) : 0x80000000u;
#pragma unroll
    for (int pass = 0; pass < 8; ++pass) {
      const int r = r0 + 32 * pass;
      const char* srow = smem + r * RSB + gg * 256;
      float gt[8], up[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(srow + cc * 16), gt);
      unpack8(*reinterpret_cast<const uint4*>(srow + 128 + cc * 16), up);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = gt[e] * up[e] / (1.f + __expf(-gt[e]));
      const uint4 q = pack8(o);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{q.x, q.y, q.z, q.w}, yr, yo + (uint32_t)(32 * pass * ldy * 2), 0, 0);
    }
  } else if constexpr (EPI == TILE_EPI_ROPE) {
    // heads of 128 columns: thread: row tid / 16 + 32 pass, head hh = (tid & 15) >> 3, pair chunk
    // cc = tid & 7 (elements cc*8 .. +7 and 64 + cc*8 .. +7 of the head)
    const int c = tid & 15, r0 = tid >> 4, hh = c >> 3, cc = c & 7;
    const int head = (n0 >> 7) + hh;
    const bool rot = head < ep.rope_heads && nrows >= (hh + 1) * 128;
    const __amdgpu_buffer_rsrc_t yr = pp_rsrc(Y + (long)row0 * N, (long)mrows * N * 2);
    const bool colok = hh * 128 < nrows;
#pragma unroll 2
    for (int pass = 0; pass < 8; ++pass) {
      const int r = r0 + 32 * pass;
      const char* srow = smem + r * RSB + hh * 256;
      const uint4 a = *reinterpret_cast<const uint4*>(srow + cc * 16);
      const uint4 b = *reinterpret_cast<const uint4*>(srow + 128 + cc * 16);
      uint4 oa = a, ob = b;
      if (rot && r < mrows) {
        const float* cs = ep.cos_sin + (long)ep.positions[row0 + r] * 128;
        const float4 c0 = *reinterpret_cast<const float4*>(cs + cc * 8), c1 = *reinterpret_cast<const float4*>(cs + cc * 8 + 4);
        const float4 s0 = *reinterpret_cast<const float4*>(cs + 64 + cc * 8),
                     s1 = *reinterpret_cast<const float4*>(cs + 64 + cc * 8 + 4);
        const float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        float x1[8], x2[8], o1[8], o2[8];
        unpack8(a, x1);
        unpack8(b, x2);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o1[j] = x1[j] * cv[j] - x2[j] * sv[j];
          o2[j] = x2[j] * cv[j] + x1[j] * sv[j];
        }
        oa = pack8(o1);
        ob = pack8(o2);
      }
      const uint32_t base = colok ? (uint32_t)((r * N + n0 + hh * 128) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{oa.x, oa.y, oa.z, oa.w}, yr, base + cc * 16, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{ob.x, ob.y, ob.z, ob.w}, yr, base + 128 + cc * 16, 0, 0);
    }
  } else {
    // plain bf16 rows: thread: row tid / 32 + 16 pass, columns (tid & 31) * 8 .. + 7
    const int c = tid & 31, r0 = tid >> 5;
    const __amdgpu_buffer_rsrc_t yr = pp_rsrc(Y + (long)row0 * N, (long)mrows * N * 2);
    const uint32_t yo = c * 8 < nrows ? (uint32_t)((r0 * N + n0 + c * 8) * 2) : 0x80000000u;
#pragma unroll
    for (int b = 0; b < 16; b += 8) {
      u32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const u32x4*>(smem + (r0 + 16 * (b + u)) * RSB + c * 16);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(v[u], yr, yo + (uint32_t)(16 * (b + u) * N * 2), 0, 0);
    }
  }
}

}  // namespace k8sllm

using namespace k8sllm;

// Same contract as k8sllm_gemm_tile (gemm_tile.hip), 8-wave ping-pong schedule; called by it for
// algo 2.  Shapes: N % 16 == 0 (SwiGLU: N % 256 == 0), K % 64 == 0, K >= 128.
static int pp_sched = 1;  // refill schedule (SCH): k8sllm_gemm_pp_sched

extern "C" void k8sllm_gemm_pp_sched(int sch) { pp_sched = sch; }

extern "C" int k8sllm_gemm_pp(const void* X, const void* W, void* Y, int M, int N, int K, const int* offsets, int E,
                              long w_es, int epi, const int* rope_pos, const float* rope_cs, int rope_heads,
                              const float* rs_part, int rs_np, float rs_eps, void* resid, void* hw, const void* norm_w,
                              float* ss_out, hipStream_t s) {
  if (M <= 0) return 0;
  const bool grouped = offsets != nullptr;
  const bool rs = rs_part != nullptr;
  if (grouped && (E < 1 || E > 256)) return -1;
  if (N % 16 != 0 || K % 64 != 0 || K < 128 || (epi == TILE_EPI_SWIGLU && N % 256 != 0)) return -1;
  if (epi == TILE_EPI_ROPE && (grouped || N % 128 != 0 || rope_pos == nullptr || rope_cs == nullptr)) return -1;
  if (epi == TILE_EPI_RESID && (grouped || rs || N % 256 != 0 || resid == nullptr || hw == nullptr ||
                                norm_w == nullptr || ss_out == nullptr))
    return -1;
  if (rs && (grouped || rs_np < 4 || rs_np > 64 || rs_np % 4 != 0 || (epi != TILE_EPI_ROPE && epi != TILE_EPI_SWIGLU)))
    return -1;
  const TileEpi ep{rope_pos, rope_cs, rope_heads, rs_part, rs_np, rs_eps, (bf16_t*)resid, (bf16_t*)hw,
                   (const bf16_t*)norm_w, ss_out, 0};
  if ((long)N * K * 2 >= (1L << 31) || 256L * K * 2 >= (1L << 31)) return -3;
  if (epi == TILE_EPI_RESID && 256L * N * 2 >= (1L << 31)) return -3;
  const int n_mt = (M + 255) / 256 + (grouped ? E : 0), n_nt = (N + 255) / 256;
  const long nwg = (long)n_mt * n_nt;
  if (nwg > (1L << 30)) return -2;
  const dim3 grid((unsigned)nwg);
#define K8_PP1(EPI_, G_, RS_, SCH_)                                                                                  \
  hipLaunchKernelGGL((gemm_pp_kernel<EPI_, G_, RS_, SCH_>), grid, dim3(512), 0, s, (const bf16_t*)X, (const bf16_t*)W, \
                     (bf16_t*)Y, offsets, E, M, N, K, w_es, n_mt, n_nt, ep)
#define K8_PP(EPI_, G_, RS_) \
  if (pp_sched == 1) K8_PP1(EPI_, G_, RS_, 1); else K8_PP1(EPI_, G_, RS_, 0)
  if (grouped) {
    if (epi == TILE_EPI_SWIGLU) K8_PP(TILE_EPI_SWIGLU, true, false);
    else K8_PP(TILE_EPI_BF16, true, false);
  } else if (epi == TILE_EPI_RESID) {
    K8_PP(TILE_EPI_RESID, false, false);
  } else if (rs) {
    if (epi == TILE_EPI_SWIGLU) K8_PP(TILE_EPI_SWIGLU, false, true);
    else K8_PP(TILE_EPI_ROPE, false, true);
  } else if (epi == TILE_EPI_SWIGLU) {
    K8_PP(TILE_EPI_SWIGLU, false, false);
  } else if (epi == TILE_EPI_ROPE) {
    K8_PP(TILE_EPI_ROPE, false, false);
  } else {
    K8_PP(TILE_EPI_BF16, false, false);
  }
#undef K8_PP
#undef K8_PP1
  return (int)hipGetLastError();
}
