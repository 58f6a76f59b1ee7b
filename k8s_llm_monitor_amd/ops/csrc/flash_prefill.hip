// Causal varlen flash-attention forward (prefill) with GQA on gfx950.
//
// Workgroup = 4 waves = 128 query rows of one query head; each wave owns 32 rows.
// K/V tiles of 64 keys are staged through LDS (XOR-swizzled so that both the row reads of K
// and the transposed reads of V are bank-conflict free).  All products use
// v_mfma_f32_32x32x16_bf16 in the "swapped" orientation (cdna_hip_programming.md §3):
//   S^T[kv][q] = K[kv][:] . Q[q][:]        A = K (ds_read_b128),   B = Q^T (registers)
//   O^T[d][q] += V^T[d][kv] . P^T[kv][q]    A = V^T (ds_read_b64_tr_b16), B = S^T accumulator
// With the query on the MFMA column (= lane), the online-softmax statistics (m, l) and the
// rescale of O are lane-local: no cross-lane traffic except one xor-32 per reduction.
// The score accumulator is converted to bf16 and consumed as the PV B operand in place.
//
// PAGED variant (prefix caching / chunked prefill): the queries are the NEW tokens of each
// sequence (rows of the qkv buffer), but keys and values come from the paged KV cache (which
// rope_and_cache has already extended with the new tokens), covering positions [0, ctx_start +
// new): the cached prefix is attended without being recomputed.  Only the tile staging and the
// causal offsets differ: keys of the new tokens stage from the qkv rows exactly as in the plain
// kernel; only cached keys (position < ctx_start) are read from the paged cache.
#include "common.h"
#include <stdlib.h>

namespace k8sllm {

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt_fp() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// x combined with its lane ^ 32 partner by one v_permlane32_swap (VALU, no LDS round trip; a
// __shfl_xor(x, 32) is a ds_bpermute): the swap leaves (own, partner) in lanes 0-31 and
// (partner, own) in lanes 32-63, so an order-free op of the pair is the same on every lane.
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <int D, bool PAGED>
__global__ __launch_bounds__(256, 2) void flash_prefill_kernel(bf16_t* __restrict__ out, long out_stride,
                                                               const bf16_t* __restrict__ qkv, long qkv_stride,
                                                               const int* __restrict__ cu_seqlens,
                                                               const int* __restrict__ qb_seq,
                                                               const int* __restrict__ qb_start, int Hq, int Hkv,
                                                               float scale_log2, const int* __restrict__ ctx_start,
                                                               const bf16_t* __restrict__ k_cache,
                                                               const bf16_t* __restrict__ v_cache,
                                                               const int* __restrict__ block_tables, int bt_stride) {
  static_assert(D == 128, "prefill kernel is specialised for head_dim 128");
  constexpr int KS = D / 16;  // 8 k-steps over the head dim
  constexpr int DT = D / 32;  // 4 output tiles of 32 dims
  constexpr int CH = D / 8;   // 16-byte chunks per row (16)
  __shared__ __attribute__((aligned(16))) bf16_t Ks[64 * D];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[64 * D];

  // grid (Hq, q-blocks): the host orders q-blocks heaviest first (most keys), and x = head runs
  // fastest so the whole grid drains heavy-first.  Blocks x and x + 8 share an XCD (round-robin
  // dispatch), so heads are remapped to give each XCD a contiguous head range - the query heads
  // of one GQA group then share their K/V tiles through that XCD's L2.
  const int qb = blockIdx.y;
  const int hq = (Hq & 7) == 0 ? (blockIdx.x & 7) * (Hq >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int G = Hq / Hkv;
  const int kvh = hq / G;
  const int seq = qb_seq[qb];
  const int qs = qb_start[qb];
  const int s0 = cu_seqlens[seq];
  const int L = cu_seqlens[seq + 1] - s0;  // query rows (new tokens)
  const int cst = PAGED ? ctx_start[seq] : 0;  // absolute position of query row 0
  const int LK = cst + L;                      // keys: positions [0, LK)
  const int* bt = PAGED ? block_tables + (long)seq * bt_stride : nullptr;
  const int tid = threadIdx.x, lane = tid & 63;
  // wave-uniform (SGPR): the causal tile skip and the diagonal-mask test become scalar branches
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int myq = qs + wave * 32 + r32;
  const bf16_t* base = qkv + (long)s0 * qkv_stride;
  const int koff = (Hq + kvh) * D, voff = (Hq + Hkv + kvh) * D;

  bf16x8 qf[KS];
  if (myq < L) {
    const bf16_t* qp = base + (long)myq * qkv_stride + hq * D + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
  } else {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
  }

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m = -1e30f, l = 0.f;

  const int wave_q0 = cst + qs + wave * 32;  // absolute position of the wave's first query
  const int kv_end = min(LK, cst + qs + 128);
  // per-lane constants of the transposed V read (see header): group g = lane>>4
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
  const int vcol_base = 16 * ((lane >> 4) & 1) + 4 * p4;

  // K/V tile staging, software-pipelined (cdna_hip_programming.md T14, issue-early / write-late):
  // tile t+1's global loads are issued into registers right after tile t is staged, so they are in
  // flight during tile t's MFMAs, and land in LDS at the top of the next iteration.
  uint4 kreg[4], vreg[4];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      const int r = c / CH, ch = c % CH;
      const int kr = k0 + r;
      uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if constexpr (!PAGED) {
        if (kr < L) {
          kv = *reinterpret_cast<const uint4*>(base + (long)kr * qkv_stride + koff + ch * 8);
          vv = *reinterpret_cast<const uint4*>(base + (long)kr * qkv_stride + voff + ch * 8);
        }
      } else {
        // keys of the new tokens come from this step's qkv rows (16-byte loads, as above); only
        // the cached prefix [0, cst) is read from the paged cache: K as 16-byte [D/8][16][8]
        // pieces, V (d-major [D][16] per block) gathered 8 dims x 2 bytes
        if (kr >= cst && kr < LK) {
          const bf16_t* row = base + (long)(kr - cst) * qkv_stride;
          kv = *reinterpret_cast<const uint4*>(row + koff + ch * 8);
          vv = *reinterpret_cast<const uint4*>(row + voff + ch * 8);
        } else if (kr < cst) {
          const long blk = bt[kr >> 4];
          kv = *reinterpret_cast<const uint4*>(k_cache + (((blk * Hkv + kvh) * CH + ch) * 16 + (kr & 15)) * 8);
          const bf16_t* vp = v_cache + ((blk * Hkv + kvh) * D + ch * 8) * 16 + v_perm(kr & 15);
          uint32_t w[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) w[j] = (uint32_t)vp[(2 * j) * 16] | ((uint32_t)vp[(2 * j + 1) * 16] << 16);
          vv = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
      kreg[i] = kv;
      vreg[i] = vv;
    }
  };
  fetch(0);
  for (int k0 = 0; k0 < kv_end; k0 += 64) {
    __syncthreads();  // every wave is done reading the previous tile
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      const int r = c / CH, ch = c % CH;
      *reinterpret_cast<uint4*>(Ks + (r * CH + (ch ^ (r & 15))) * 8) = kreg[i];
      *reinterpret_cast<uint4*>(Vs + (r * CH + (ch ^ ((r & 3) << 2))) * 8) = vreg[i];
    }
    __syncthreads();
    if (k0 + 64 < kv_end) fetch(k0 + 64);
    if (k0 > wave_q0 + 31) continue;  // every key of this tile is in the future of every row of this wave

    // the two 32-key halves are independent accumulation chains: interleave them (k-step outer)
    // so consecutive MFMAs never wait on each other's result
    f32x16 sacc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[i][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int ch = 2 * ks + hh;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int kr = 32 * i + r32;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(Ks + (kr * CH + (ch ^ (kr & 15))) * 8);
        sacc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], sacc[i], 0, 0, 0);
      }
    }

    // scores stay unscaled: the running max is kept in the log2 domain and the scale is folded
    // into the exponent (one v_fma per score instead of a v_mul + v_sub); exponentials are the raw
    // v_exp_f32 (arguments are <= 0, flushing tiny results to 0 is what a softmax wants) instead of
    // exp2f's denormal-range wrapper (cmp + 2 cndmask + ldexp around every v_exp)
    const bool need_mask = (k0 + 63 > wave_q0) || (k0 + 64 > LK);
    if (need_mask) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kv = k0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (kv > cst + myq || kv >= LK) sacc[i][r] = -1e30f;
        }
    }
    float mx = sacc[0][0];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[i][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(m, mx * scale_log2);
    const float alpha = __builtin_amdgcn_exp2f(m - mnew);
    float rs = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[i][r], scale_log2, -mnew));
        sacc[i][r] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    const bool grew = __builtin_amdgcn_ballot_w64(mnew > m) != 0;  // lazy rescale: O only when a max moved
    m = mnew;
    if (grew) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
    }

#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[j] = (__bf16)sacc[i][8 * s + j];
        const int row0 = 32 * i + 16 * s + 4 * hh + q4;  // + 8*jj
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int colv = 32 * dt + vcol_base;
          const int ch = colv >> 3, half = (colv >> 2) & 1;
          s16x4 t[2];
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int row = row0 + 8 * jj;
            const bf16_t* addr = Vs + (row * CH + (ch ^ ((row & 3) << 2))) * 8 + half * 4;
            t[jj] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(addr));
          }
          const bf16x8 a = __builtin_bit_cast(
              bf16x8, make_uint4(__builtin_bit_cast(uint2, t[0]).x, __builtin_bit_cast(uint2, t[0]).y,
                                 __builtin_bit_cast(uint2, t[1]).x, __builtin_bit_cast(uint2, t[1]).y));
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pb, o[dt], 0, 0, 0);
        }
      }
  }

  if (myq < L) {
    const float inv = 1.f / l;
    bf16_t* op = out + (long)(s0 + myq) * out_stride + (long)hq * D + 4 * hh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint2 v;
        v.x = pack2(o[dt][4 * k] * inv, o[dt][4 * k + 1] * inv);
        v.y = pack2(o[dt][4 * k + 2] * inv, o[dt][4 * k + 3] * inv);
        *reinterpret_cast<uint2*>(op + 32 * dt + 8 * k) = v;
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Paged prefill v2: every key / value tile is staged VERBATIM from the paged cache by LDS-DMA
// (rope_and_cache has already written the new tokens), shared by all G query heads of a kv head.
//
//  * workgroup = one kv head x QR = 256 / G query rows x all G heads: 8 waves, each 32 rows of
//    one head (G = 4: 64 rows; grid z splits the host's 128-row q-blocks).  One 64-key tile
//    (4 cache blocks: K 16 KiB + V 16 KiB) feeds 8 waves instead of 4: half the staging per MFMA
//    of the v1 kernel (one head per workgroup), and no staging registers: 4 global_load_lds_dwordx4
//    per wave per tile.
//  * four-slot LDS ring (128 KiB), ONE barrier per tile, two tiles in flight across it (counted
//    vmcnt; cdna_hip_programming.md §5 "Pipelining across barriers": raw s_barrier, never
//    __syncthreads with a DMA in flight); see the pipeline comment at the main loop.
//  * fragments: K as cached ([piece of 8 dims][16 tokens][8]) is read lane-linear per 16 tokens -
//    conflict-free ds_read_b128; V as cached ([dim][16 tokens], v_perm token order, common.h) gives
//    the PV A-operand of a 32x32x16 MFMA in one ds_read_b128 per lane, the dim row's two 16-B
//    chunks XOR-swapped by bit 3 of the dim (applied to the DMA source address) so the 16 lanes of
//    a read group hit 16 distinct bank quads.  v1 gathered the cached V with 2-byte loads.
//  * products as v1: S^T = K Q^T (A = K, B = Q^T from registers), O^T += V^T P^T (B = the score
//    accumulator converted in place), online softmax lane-local (query = lane).
//  * heads are remapped nowhere: blockIdx.x = kv head, so all workgroups of one kv head share an
//    XCD (dispatch round-robin over 8 XCDs) and its L2 serves the head's K/V to every q-block.
template <int G>
__global__ __launch_bounds__(512, 2) void flash_prefill_paged_v2_kernel(
    bf16_t* __restrict__ out, long out_stride, const bf16_t* __restrict__ qkv, long qkv_stride,
    const int* __restrict__ cu_seqlens, const int* __restrict__ qb_seq, const int* __restrict__ qb_start, int Hq,
    int Hkv, float scale_log2, const int* __restrict__ ctx_start, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride) {
  constexpr int D = 128, KS = D / 16, DT = D / 32;
  constexpr int WPH = 8 / G;      // waves per head
  constexpr int QR = 32 * WPH;    // query rows per workgroup
  constexpr int Z = 128 / QR;     // workgroups per 128-row q-block
  constexpr int TILE = 32768;     // K (16 KiB) + V (16 KiB) of 64 keys
  constexpr int NBUF = 4;
  constexpr int MAXB = 2048;      // block ids per sequence staged in LDS (32k tokens)
  __shared__ __attribute__((aligned(16))) char fp2_smem[NBUF * TILE + MAXB * 4];  // ring + block ids
  int* s_blk = reinterpret_cast<int*>(fp2_smem + NBUF * TILE);

  // grid (Hkv, q-blocks x Z): the Z workgroups of one q-block are dispatched back to back, on one
  // XCD (x = kv head), so they share the block's K/V tiles in L2
  const int kvh = blockIdx.x, qb = blockIdx.y / Z;
  const int seq = qb_seq[qb];
  const int qs = qb_start[qb] + (blockIdx.y % Z) * QR;  // first query row (new-token index) of the workgroup
  const int s0 = cu_seqlens[seq];
  const int L = cu_seqlens[seq + 1] - s0;
  if (qs >= L) return;  // uniform: the last q-block's upper part
  const int cst = ctx_start[seq];
  const int LK = cst + L;
  const int nblk = (LK + 15) / 16;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave / WPH, sub = wave % WPH;
  const int hq = kvh * G + g;
  const int r32 = lane & 31, hh = lane >> 5;
  const int myq = qs + sub * 32 + r32;
  const int wave_q0 = cst + qs + sub * 32;  // absolute position of the wave's first query
  const int kv_end = min(LK, cst + qs + QR);
  const int ntiles = (kv_end + 63) >> 6;

  // the sequence's block ids (the tiles' DMA sources) and this wave's q fragments, loaded with
  // plain loads and retired before the first DMA: no register load is outstanding beside one
  const int* bt = block_tables + (long)seq * bt_stride;
  for (int i = tid; i < ntiles * 4; i += 512) s_blk[i] = i < nblk ? bt[i] : bt[0];
  bf16x8 qf[KS];
  {
    const int qrow = min(myq, L - 1);
    const bf16_t* qp = qkv + (long)(s0 + qrow) * qkv_stride + hq * D + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
  }
  // consume q here, so the compiler's own wait for these loads sits before the loop; otherwise
  // hipcc re-waits vmcnt(0) at the first MFMA of EVERY tile, draining the DMAs in flight
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(qf[ks]));
  __syncthreads();

  // 32 x 1 KiB DMA pieces per tile: wave w issues pieces 4w .. 4w + 3 (waves 0-3 K, 4-7 V)
  const int kind = wave >> 2, bsel = wave & 3;
  const bf16_t* cache = kind ? v_cache : k_cache;
  int src_chunk[4];
#pragma unroll
  for (int part = 0; part < 4; ++part) {
    const int c = part * 64 + lane;  // 16-B chunk of the 4 KiB block image, in LDS order
    src_chunk[part] = kind ? (((c >> 1) << 1) | ((c & 1) ^ ((c >> 4) & 1))) : c;  // V: dim = c >> 1
  }
  auto issue = [&](int t, int buf) {
    const long phys = s_blk[t * 4 + bsel];
    const bf16_t* base = cache + (phys * Hkv + kvh) * (D * 16);
    char* dst = fp2_smem + buf * TILE + kind * 16384 + bsel * 4096;
#pragma unroll
    for (int part = 0; part < 4; ++part)
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + src_chunk[part] * 8), (lds_void_t*)(dst + part * 1024),
                                       16, 0, 0);
  };

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m = -1e30f, l = 0.f;

  // QK of one tile: S^T[64 keys][32 queries] as two 32-key accumulators
  auto qk = [&](int t, f32x16 (&sa)[2]) {
    const char* kt = fp2_smem + (t % NBUF) * TILE;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) sa[i][r] = 0.f;
    // all 16 K fragments of the tile are read first (64 VGPRs), then the 16 MFMAs consume them:
    // one LDS round trip per tile instead of one per MFMA pair (287 vs 301 us at 10 x 1609)
    bf16x8 kfr[KS][2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        // key 32 i + r32: block 2 i + (r32 >> 4), token r32 & 15; dims 16 ks + 8 hh = piece 2 ks + hh
        kfr[ks][i] = *reinterpret_cast<const bf16x8*>(kt + (2 * i + (r32 >> 4)) * 4096 +
                                                      ((2 * ks + hh) * 16 + (r32 & 15)) * 16);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i) sa[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfr[ks][i], qf[ks], sa[i], 0, 0, 0);
  };
  // causal / end-of-sequence mask of one tile's scores: only the diagonal tile and the
  // sequence's last tile - a uniform scalar branch, kept OUT of the compute block below
  auto mask = [&](int t, f32x16 (&sa)[2]) {
    const int k0 = t * 64;
    if (__builtin_amdgcn_readfirstlane((k0 + 63 > wave_q0) || (k0 + 64 > LK))) {
      // last visible key, relative to this lane's first score row; one compare + select per score
      // (a branchy form made hipcc build cumulative scalar masks: a 30-deep dependent SALU chain)
      const float lim = (float)(min(cst + myq, LK - 1) - k0 - 4 * hh);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sa[i][r] = (float)(32 * i + (r & 3) + 8 * (r >> 2)) > lim ? -1e30f : sa[i][r];
    }
  };
  // online softmax of one tile's scores (in place -> probabilities), then O += V^T P^T
  auto softmax_pv = [&](int t, f32x16 (&sa)[2]) {
    // the tile's 16 V fragments are read before the softmax VALU work, which hides their latency
    const char* vt = fp2_smem + (t % NBUF) * TILE + 16384;
    bf16x8 vfr[2][2][DT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int d = 32 * dt + r32;
          vfr[i][s][dt] = *reinterpret_cast<const bf16x8*>(vt + (2 * i + s) * 4096 + (d * 2 + (hh ^ ((d >> 3) & 1))) * 16);
        }
    __builtin_amdgcn_sched_barrier(0);
    // row max and row sum as four independent chains each (a single 32-long dependent chain is
    // latency-bound), combined across the lane halves by v_permlane32_swap
    float mq[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) mq[c] = fmaxf(sa[c >> 1][8 * (c & 1)], sa[c >> 1][8 * (c & 1) + 1]);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 2; r < 8; ++r) mq[c] = fmaxf(mq[c], sa[c >> 1][8 * (c & 1) + r]);
    const float mx = xor32_max(fmaxf(fmaxf(mq[0], mq[1]), fmaxf(mq[2], mq[3])));
    // Lazy max with headroom: the reference max m moves only when the tile's max exceeds it by
    // more than 2^8 in probability (then to the exact max), so probabilities stay <= 256 - exact in
    // fp32 and in their bf16 rounding - and O is rescaled only on such a jump, which after a row's
    // first tiles is rare.  The rescale comes BEFORE the probabilities, so each 16-key group's
    // exponentials -> bf16 -> 4 PV MFMAs can run back to back: the MFMAs of one group execute
    // while the VALU computes the next group's exponentials.
    const float mt = mx * scale_log2;
    const float mnew = mt > m + 8.f ? mt : m;
    const float alpha = __builtin_amdgcn_exp2f(m - mnew);
    if (__builtin_amdgcn_ballot_w64(mnew != m) != 0) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
    }
    m = mnew;
    float rq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sa[i][8 * s + j], scale_log2, -mnew));
          rq[2 * i + s] += p;
          pb[j] = (__bf16)p;
        }
        // block 2 i + s: keys 32 i + 16 s ..
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr[i][s][dt], pb, o[dt], 0, 0, 0);
      }
    l = l * alpha + xor32_sum((rq[0] + rq[1]) + (rq[2] + rq[3]));
  };

  // Main loop: ONE barrier per tile; tiles t + 1 and t + 2 are in flight while tile t is
  // computed (4-slot ring).  At tile t's barrier every wave has finished tile t - 1, whose slot
  // (t + 3) % 4 is refilled right after it.  (A software-pipelined variant that put tile t + 1's
  // QK beside tile t's softmax measured no faster and spilled once the two phases shared a
  // basic block.  Round 6: a staggered form - the two waves of a SIMD half a tile apart, one's
  // softmax under the other's MFMAs: PV(t-1) + QK(t) then softmax(t) vs softmax(t-1) then
  // PV(t-1) + QK(t), K in two 8-fragment halves, 196 VGPRs - was bit-identical and 3-8 % SLOWER at
  // 10 x 1609, 64 x 1609 and 2 x 8192, Hq 32 and 64: profiles/r06/flash_stagger_ab.jsonl.  A
  // persistent form - one workgroup per CU walking these work items, the next item's first three
  // tiles DMA'd under the current item's last three - was bit-identical and 0-14 % SLOWER: the
  // static item assignment loses more to imbalance than the hardware dispatcher's per-workgroup
  // overhead costs; profiles/r06/flash_persistent_v3_ab.jsonl.  A 4-wave form with two 32-row
  // units per wave (one wave per SIMD; each LDS fragment feeds twice the MFMAs), plain or with
  // the units' MFMA / softmax interleaved by sched_group_barrier, was bit-identical and 15-22 %
  // SLOWER: the softmax VALU needs the second wave per SIMD to hide behind;
  // profiles/r06/flash_v4_two_unit_ab.jsonl.)  The wave computes only its first nt_w tiles (later ones are in the future of
  // all its rows) but joins every barrier and issues its DMA pieces for every tile.
  const int nt_w = min(ntiles, (wave_q0 + 31) / 64 + 1);
  // (No static priority for the second-dispatched half: with each 16-key group's exponentials
  // interleaved with the PV MFMAs it measured 1-2 % slower at 10 x 1609 and equal at 4k-16k,
  // profiles/r04/flash_no_setprio_ab.jsonl.)
  issue(0, 0);
  if (ntiles > 1) issue(1, 1);
  if (ntiles > 2) issue(2, 2);
  for (int t = 0; t < ntiles; ++t) {
    if (t + 2 < ntiles)
      wait_vmcnt_fp<8>();  // this wave's pieces of tile t landed; t + 1, t + 2 may still fly
    else if (t + 1 < ntiles)
      wait_vmcnt_fp<4>();
    else
      wait_vmcnt_fp<0>();
    __builtin_amdgcn_s_barrier();  // every wave's pieces of tile t landed; tile t - 1 reads done
    if (t + 3 < ntiles) issue(t + 3, (t + 3) % NBUF);
    if (t >= nt_w) continue;
    f32x16 sa[2];
    qk(t, sa);
    mask(t, sa);
    softmax_pv(t, sa);
  }

  if (myq < L) {
    const float inv = 1.f / l;
    bf16_t* op = out + (long)(s0 + myq) * out_stride + (long)hq * D + 4 * hh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint2 v;
        v.x = pack2(o[dt][4 * k] * inv, o[dt][4 * k + 1] * inv);
        v.y = pack2(o[dt][4 * k + 2] * inv, o[dt][4 * k + 3] * inv);
        *reinterpret_cast<uint2*>(op + 32 * dt + 8 * k) = v;
      }
  }
}

}  // namespace k8sllm

using namespace k8sllm;

extern "C" int k8sllm_flash_prefill(void* out, long out_stride, const void* qkv, long qkv_stride,
                                    const int* cu_seqlens, const int* qb_seq, const int* qb_start, int n_qblocks,
                                    int Hq, int Hkv, int D, float scale, const int* ctx_start, const void* k_cache,
                                    const void* v_cache, const int* block_tables, int bt_stride, hipStream_t s) {
  if (n_qblocks <= 0) return 0;
  if (D != 128 || Hq % Hkv != 0) return -1;
  const float sl2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  // bt_stride = the block-table width = most blocks a sequence can hold: <= 2048 - 3 fit the LDS copy
  if (ctx_start != nullptr && (G == 2 || G == 4 || G == 8) && bt_stride <= 2045) {
    // v2: q-blocks of 128 rows split into 128 / QR workgroups (QR = 256 / G rows each), adjacent in y
    const int z = 128 / (256 / G);
#define K8S_FP2(GG)                                                                                                 \
  hipLaunchKernelGGL((flash_prefill_paged_v2_kernel<GG>), dim3(Hkv, n_qblocks * z), dim3(512), 0, s, (bf16_t*)out,  \
                     out_stride, (const bf16_t*)qkv, qkv_stride, cu_seqlens, qb_seq, qb_start, Hq, Hkv, sl2,       \
                     ctx_start, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride)
    switch (G) {
      case 2: K8S_FP2(2); break;
      case 4: K8S_FP2(4); break;
      default: K8S_FP2(8); break;
    }
#undef K8S_FP2
    return (int)hipGetLastError();
  }
  if (ctx_start != nullptr) {
    hipLaunchKernelGGL((flash_prefill_kernel<128, true>), dim3(Hq, n_qblocks), dim3(256), 0, s, (bf16_t*)out,
                       out_stride, (const bf16_t*)qkv, qkv_stride, cu_seqlens, qb_seq, qb_start, Hq, Hkv, sl2,
                       ctx_start, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride);
  } else {
    hipLaunchKernelGGL((flash_prefill_kernel<128, false>), dim3(Hq, n_qblocks), dim3(256), 0, s, (bf16_t*)out,
                       out_stride, (const bf16_t*)qkv, qkv_stride, cu_seqlens, qb_seq, qb_start, Hq, Hkv, sl2,
                       nullptr, nullptr, nullptr, nullptr, 0);
  }
  return (int)hipGetLastError();
}
