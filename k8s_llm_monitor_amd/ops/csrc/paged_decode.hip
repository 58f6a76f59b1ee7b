// Split-K paged decode attention with GQA on gfx950 MFMA.
//
// One query token per sequence; the G = Hq/Hkv query heads that share a KV head are the
// 16 columns (G <= 16 used) of a v_mfma_f32_16x16x32_bf16 tile, so one K/V read serves the
// whole GQA group:
//   scores  S[t][h]   = K[t][:] . Q[h][:]          A = K   (16 tokens x 32 dims per MFMA)
//   output  O^T[d][h] = sum_t V^T[d][t] P^T[t][h]  A = V^T (16 dims  x 32 tokens per MFMA)
// The KV-cache layouts of rope_cache.hip make every A-operand load a 16-byte piece: K and V
// loads are 1 KiB per wave-instruction (V by the token order described at `issue`).  P never
// leaves registers: the
// score accumulator of two 16-token blocks is, element for element, the B operand of the
// PV product (token order inside the k-step is permuted identically on both operands).
//
// Work decomposition (measured on MI355X, tools/bench_decode.py):
//  * grid = (S splits, Hkv, batch) with S chosen per batch size by the host so that the grid is
//    ~1-4 workgroups per CU - NOT one workgroup per fixed 256-token partition: an empty
//    workgroup still holds its CU slot for a global-load round trip, and a grid sized for
//    max_model_len spent 130 us per layer launching empty workgroups at batch 64.
//  * each workgroup walks its chunks of 256 tokens (4 waves x 64) with an online softmax per
//    wave; per chunk every wave issues ALL of its K (16 x dwordx4) and V (32 x dwordx2) loads
//    before the first MFMA (block ids past the sequence end are clamped to a valid block and
//    masked), i.e. 32 KiB in flight per wave.
//  * if a sequence's chunks fit one split, that workgroup writes the normalised output;
//    otherwise each split writes (max, sum, O) partials that are merged either by the LAST
//    arriving split of the (sequence, kv head) inside this launch (MERGE: partials stored
//    write-through, one agent-scope counter per (sequence, kv head) - the hand-off protocol of the
//    decode GEMM's grid seam, no L2 write-back) or by paged_decode_reduce_kernel in a second
//    launch.  (An earlier in-kernel merge with agent release/acquire FENCES measured 2.3x slower at
//    batch 64 x 1.8k context: every workgroup paid an L2 write-back.)
// Everything is static-shaped so the decode step can be captured in a hipGraph.
#include "common.h"
#include <stdlib.h>

namespace k8sllm {

constexpr int kBS = 16;   // tokens per KV-cache block
constexpr int kPdSC1 = 16;  // buffer-op aux bits: sc1 (write-through stores / L2-coherent loads)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pd_rsrc(const void* base, long bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)min(bytes, 0x7fffffffL));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}

// kch: tokens per chunk (4 waves x TW tokens)
__device__ __forceinline__ void split_range(int seq_len, int S, int split, int kch, int* c0, int* c1, int* nvalid) {
  const int nch = (seq_len + kch - 1) / kch;
  const int per = (nch + S - 1) / S;
  *c0 = split * per;
  *c1 = min(nch, *c0 + per);
  *nvalid = (nch + per - 1) / per;
}

// FQ (fused q/k/v, decode at TP>=1 behind the skinny qkv GEMM, D = 128): the kernel also does
// what rope_and_cache did between the two launches - the new token's q / k / v are the sum of the
// qkv projection's fp32 split-K slabs, rounded to bf16, q and k rotated (neox pairs) - so one
// launch per layer disappears.  The new token is not read back from the cache: every split
// attends to the cached tokens [0, seq_len - 1) and the split owning the last chunk folds the new
// token into its online softmax from registers (and writes its k / v to the cache for the next
// steps), so no workgroup waits for another's cache write.
struct DecodeFuse {
  const float* slabs;  // [nslabs][B][(Hq + 2 Hkv) * D] fp32
  int nslabs;
  const int* positions;    // [B]
  const float* cos_sin;    // [max_pos][D]: cos | sin
  const int* slot_mapping;  // [B], -1 = no cache write
  bf16_t* k_cache;
  bf16_t* v_cache;
};

// TW: tokens per wave per chunk.  TW = 32: two chunk buffers per wave (double-buffered loads,
// ~240 VGPRs: 2 waves per SIMD) for grids that fill the chip (batch 64: 512 workgroups);
// TW = 64: one buffer of 64 tokens (~120 VGPRs: up to 4 workgroups per CU) for small, split
// grids, where residency, not the per-wave pipeline, hides the memory latency.
template <int D, int G, bool FQ, int TW, bool MERGE = false>
__global__ __launch_bounds__(256, TW == 32 ? 2 : 1) void paged_decode_kernel(bf16_t* __restrict__ out, long out_stride,
                                                           float* __restrict__ part_out,  // [B][Hq][S][D]
                                                           float* __restrict__ part_ml,   // [B][Hq][S][2]
                                                           const bf16_t* __restrict__ q, long q_stride,
                                                           const bf16_t* __restrict__ k_cache,
                                                           const bf16_t* __restrict__ v_cache,
                                                           const int* __restrict__ block_tables, int bt_stride,
                                                           const int* __restrict__ seq_lens, int Hq, int Hkv, int S,
                                                           float scale_log2, DecodeFuse fz,
                                                           int* __restrict__ merge_ctr) {  // MERGE: [B][Hkv], zero between launches
  constexpr int KS = D / 32;  // QK k-steps
  constexpr int DT = D / 16;  // PV output tiles (16 dims each)
  __shared__ float s_max[4][16];
  __shared__ float s_sum[4][16];
  __shared__ float s_o[4][G][D];
  __shared__ __attribute__((aligned(16))) bf16_t s_q[FQ ? G : 1][D];  // FQ: rotated q of the group's heads
  __shared__ __attribute__((aligned(16))) bf16_t s_kv[FQ ? 2 : 1][D];  // FQ: the new token's rotated k, v

  const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int seq_len = seq_lens[b];
  if (seq_len <= 0) {  // padding row (graph bucket slack): define the output as zeros
    if (split == 0)
      for (int i = threadIdx.x; i < G * D; i += 256) out[act_index(b, kvh * G * D + i, out_stride)] = 0;
    return;
  }
  int c0, c1, nvalid;
  constexpr int kTW = TW, kCH = 4 * TW;
  constexpr int kNI = kTW / 16;  // 16-token K tiles (QK MFMAs) per wave and chunk
  constexpr int kNS = kTW / 32;  // 32-token PV k-steps per wave and chunk
  constexpr bool DB = TW == 32;  // double-buffered chunk loads
  split_range(seq_len, S, split, kCH, &c0, &c1, &nvalid);
  if (c0 >= c1) return;  // uniform over the workgroup
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = lane & 15, kg = lane >> 4;
  const int* bt = block_tables + (long)b * bt_stride;
  const long head_block = (long)D * kBS;  // elements of one (block, head) tile
  const int nblk = (seq_len + kBS - 1) / kBS;
  const int first_blk = bt[0];
  // FQ: the cache holds tokens [0, seq_len - 1); the new token is folded in from registers
  const int n_cached = FQ ? seq_len - 1 : seq_len;
  const bool owns_new = FQ && c1 == (seq_len + kCH - 1) / kCH;

  // ---- every K and V load of a wave's kTW tokens of chunk c, issued up front (16 KiB per wave),
  // two chunk buffers per wave: chunk c + 1's loads fly while chunk c is multiplied (and the first
  // two chunks' loads fly through the FQ prologue), so a wave never sits out a memory round trip
  // between chunks.  (The single-buffered 64-token form measured 82 us per layer in the engine at
  // batch 64, ctx ~1.7k, against 75 us in isolation: the prologue and each chunk's round trip
  // were exposed.)
  // Token order inside each 32-token PV step s (tiles 2s, 2s + 1): QK tile 2s + j, row c holds
  // token 16 (c >> 3) + 8 j + 4 ((c >> 2) & 1) + (c & 3) of the step, so the score lanes of k-group
  // kg hold tokens 16 (kg >> 1) + 4 (kg & 1) + {0..3, 8..11} - in the V cache's v_perm order
  // (common.h) exactly positions 8 (kg & 1) .. + 7 of block 2s + (kg >> 1): ONE 16-byte load per
  // lane, dim tile and step (was two 8-byte loads from two blocks: half the V load instructions).
  typedef bf16x8 KF[kNI][KS];
  typedef bf16x8 VF[kNS][DT];
  auto issue = [&](KF& kf, VF& vf, int c) {
    const int wtok0 = c * kCH + wave * kTW;
    int phys[kNI];  // the wave's kNI blocks (16 tokens each)
#pragma unroll
    for (int i = 0; i < kNI; ++i) {
      const int bi = (wtok0 >> 4) + i;
      phys[i] = bi < nblk ? bt[bi] : first_blk;
    }
#pragma unroll
    for (int i = 0; i < kNI; ++i) {
      const int sp = i >> 1, j = i & 1;  // PV step, tile within it
      const int blk = phys[2 * sp + (col >> 3)];
      const int tok = 8 * j + 4 * ((col >> 2) & 1) + (col & 3);
      const bf16_t* kb = k_cache + ((long)blk * Hkv + kvh) * head_block + (kg * kBS + tok) * 8;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        kf[i][s] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(kb + s * 4 * kBS * 8));
    }
#pragma unroll
    for (int s = 0; s < kNS; ++s) {
      const bf16_t* vb = v_cache + ((long)phys[2 * s + (kg >> 1)] * Hkv + kvh) * head_block + col * kBS + 8 * (kg & 1);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        vf[s][dt] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(vb + 16 * dt * kBS));
    }
  };
  KF kf0, kf1;
  VF vf0, vf1;
  // the first chunks' K/V loads fly while q is loaded (FQ: reduced from the slabs and rotated)
  issue(kf0, vf0, c0);
  if constexpr (DB) {
    if (c0 + 1 < c1) issue(kf1, vf1, c0 + 1);
  }

  bf16x8 qf[KS];
  if constexpr (FQ) {
    // q (G heads) + the new k (rotated) + v of kv head kvh from the qkv slabs: (G + 1) * D/2
    // rotary pairs and D/2 value pairs
    const int ncols = (Hq + 2 * Hkv) * D;
    const long slab = (long)gridDim.z * ncols;
    const float* row = fz.slabs + (long)b * ncols;
    const float* cs = fz.cos_sin + (long)fz.positions[b] * D;
    constexpr int HALF = D / 2;
    // 4 rotary pairs per item: 16-byte (non-temporal: read once) slab loads, one round for G <= 8
    constexpr int QP = HALF / 4;
    for (int it = threadIdx.x; it < (G + 2) * QP; it += 256) {
      const int h = it / QP, p = (it - h * QP) * 4;  // h < G: q head kvh*G+h; h == G: k; h == G+1: v
      const int c = h < G ? (kvh * G + h) * D : (h == G ? (Hq + kvh) * D : (Hq + Hkv + kvh) * D);
      f32x4 x1 = {0.f, 0.f, 0.f, 0.f}, x2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int z = 0; z < fz.nslabs; ++z) {
        x1 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row + z * slab + c + p));
        x2 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row + z * slab + c + HALF + p));
      }
      bf16_t* dst = h < G ? s_q[h] : s_kv[h - G];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a = bf2f(f2bf(x1[j]));  // rounded as the unfused GEMM output -> rope_cache path is
        float e = bf2f(f2bf(x2[j]));
        if (h <= G) {
          const float cc = cs[p + j], sn = cs[HALF + p + j];
          const float o1 = a * cc - e * sn, o2 = e * cc + a * sn;
          a = o1;
          e = o2;
        }
        dst[p + j] = f2bf(a);
        dst[HALF + p + j] = f2bf(e);
      }
    }
    __syncthreads();
    const int hc = col < G ? col : 0;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(&s_q[hc][32 * s + 8 * kg]);
    const int slot = fz.slot_mapping != nullptr ? fz.slot_mapping[b] : -1;
    if (owns_new && slot >= 0 && threadIdx.x < D) {  // the new token's k / v for the next steps
      const int blk = slot / kBS, off = slot - blk * kBS, d = threadIdx.x;
      fz.k_cache[(((long)blk * Hkv + kvh) * (D / 8) + (d >> 3)) * (kBS * 8) + off * 8 + (d & 7)] = s_kv[0][d];
      fz.v_cache[(((long)blk * Hkv + kvh) * D + d) * kBS + v_perm(off)] = s_kv[1][d];
    }
  } else {
    const int hc = col < G ? col : 0;
    const bf16_t* qp = q + (long)b * q_stride + (long)(kvh * G + hc) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qp + 32 * s + 8 * kg);
  }

  float m = -1e30f, l = 0.f;  // running max / sum of this wave, for head `col`
  f32x4 oacc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) oacc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const KF& kf, const VF& vf, int c) {
    const int wtok0 = c * kCH + wave * kTW;

    // ---- scores, online softmax (per lane: head `col`)
    f32x4 sacc[kNI];
#pragma unroll
    for (int i = 0; i < kNI; ++i) {
      sacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
        sacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[i][s], qf[s], sacc[i], 0, 0, 0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < kNI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = wtok0 + 32 * (i >> 1) + 16 * (kg >> 1) + 8 * (i & 1) + 4 * (kg & 1) + r;
        const float v = (t < n_cached) ? sacc[i][r] * scale_log2 : -INFINITY;
        sacc[i][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(m, mx);
    const float alpha = exp2f(m - mnew);
    float ls = 0.f;
#pragma unroll
    for (int i = 0; i < kNI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(sacc[i][r] - mnew);
        sacc[i][r] = p;
        ls += p;
      }
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    l = l * alpha + ls;
    m = mnew;
    // ---- P V  (oacc rows are dims, columns are heads: the rescale is per column = per lane)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) oacc[dt] *= alpha;
#pragma unroll
    for (int s = 0; s < kNS; ++s) {
      bf16x8 pb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (__bf16)sacc[2 * s][j];
        pb[4 + j] = (__bf16)sacc[2 * s + 1][j];
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) oacc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[s][dt], pb, oacc[dt], 0, 0, 0);
    }
  };
  if constexpr (DB) {
    for (int c = c0; c < c1; c += 2) {
      compute(kf0, vf0, c);
      if (c + 2 < c1) issue(kf0, vf0, c + 2);
      __builtin_amdgcn_sched_barrier(0);  // chunk c + 2's loads go out before chunk c + 1's MFMAs
      if (c + 1 >= c1) break;
      compute(kf1, vf1, c + 1);
      if (c + 3 < c1) issue(kf1, vf1, c + 3);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    for (int c = c0; c < c1; ++c) {
      if (c != c0) issue(kf0, vf0, c);  // chunk c0's loads were issued before the q prologue
      __builtin_amdgcn_sched_barrier(0);  // keep every load above: none may wait behind an MFMA
      compute(kf0, vf0, c);
    }
  }

  if constexpr (FQ) {
    // the new token, folded into wave 0's online softmax: score per head from the LDS copies (the
    // 4 lanes of a head column each take 32 dims), then the usual rescale + p * v_new update
    if (owns_new && wave == 0) {
      const int hc = col < G ? col : 0;
      float sc = 0.f;
#pragma unroll 8
      for (int j = 0; j < D / 4; ++j) {
        const int d = kg * (D / 4) + j;
        sc += bf2f(s_q[hc][d]) * bf2f(s_kv[0][d]);
      }
      sc += __shfl_xor(sc, 16, 64);
      sc += __shfl_xor(sc, 32, 64);
      sc *= scale_log2;
      const float mnew = fmaxf(m, sc);
      const float alpha = exp2f(m - mnew);
      const float pn = bf2f(f2bf(exp2f(sc - mnew)));  // P enters the PV product as bf16
      l = l * alpha + pn;
      m = mnew;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) oacc[dt][r] = oacc[dt][r] * alpha + pn * bf2f(s_kv[1][16 * dt + 4 * kg + r]);
    }
  }

  // ---- combine the 4 waves: oacc[dt][r] = O^T[d = 16*dt + 4*kg + r][head col]
  if (lane < 16) {
    s_max[wave][lane] = m;
    s_sum[wave][lane] = l;
  }
  if (col < G) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_o[wave][col][16 * dt + 4 * kg + r] = oacc[dt][r];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += 256) {
    const int h = i / D, d = i - h * D;
    const float M = fmaxf(fmaxf(s_max[0][h], s_max[1][h]), fmaxf(s_max[2][h], s_max[3][h]));
    const float w0 = exp2f(s_max[0][h] - M), w1 = exp2f(s_max[1][h] - M);
    const float w2 = exp2f(s_max[2][h] - M), w3 = exp2f(s_max[3][h] - M);
    const float o = w0 * s_o[0][h][d] + w1 * s_o[1][h][d] + w2 * s_o[2][h][d] + w3 * s_o[3][h][d];
    const float L = w0 * s_sum[0][h] + w1 * s_sum[1][h] + w2 * s_sum[2][h] + w3 * s_sum[3][h];
    if (nvalid == 1) {
      out[act_index(b, (kvh * G + h) * D + d, out_stride)] = f2bf(o / L);
    } else {
      const long ph = ((long)b * Hq + kvh * G + h) * S + split;
      if constexpr (MERGE) {  // write-through: read by another workgroup of this launch
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), pd_rsrc(part_out, 0x7fffffffL),
                                              (uint32_t)((ph * D + d) * 4), 0, kPdSC1);
        if (d == 0) {
          const __amdgpu_buffer_rsrc_t ml = pd_rsrc(part_ml, 0x7fffffffL);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(M), ml, (uint32_t)(ph * 8), 0, kPdSC1);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(L), ml, (uint32_t)(ph * 8 + 4), 0, kPdSC1);
        }
      } else {
        part_out[ph * D + d] = o;
        if (d == 0) {
          part_ml[ph * 2] = M;
          part_ml[ph * 2 + 1] = L;
        }
      }
    }
  }
  if constexpr (MERGE) {
    if (nvalid == 1) return;  // uniform
    // hand-off (the grid seam's protocol, gemm_decode.hip DecNorm): every wave drains its
    // write-through stores, a barrier, ONE lane takes a ticket on the (sequence, kv head) counter;
    // the split holding the last ticket resets the counter for the next launch and merges every
    // split's partials with L2-coherent (sc1) loads
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (threadIdx.x == 0) {
      int* c = merge_ctr + (long)b * gridDim.y + kvh;
      const int t = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == nvalid - 1;
      if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    const __amdgpu_buffer_rsrc_t po_rs = pd_rsrc(part_out, 0x7fffffffL), ml_rs = pd_rsrc(part_ml, 0x7fffffffL);
    float* s_w = &s_o[0][0][0];  // [G][64] split weights (s_o is free now)
    for (int h = wave; h < G; h += 4) {
      const long ph = ((long)b * Hq + kvh * G + h) * S;
      float mp = -1e30f, lp = 0.f;
      if (lane < nvalid) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b64(ml_rs, (uint32_t)((ph + lane) * 8), 0, kPdSC1);
        mp = __uint_as_float(x[0]);
        lp = __uint_as_float(x[1]);
      }
      const float mm = wave_max(mp);
      const float w = lane < nvalid ? exp2f(mp - mm) : 0.f;
      const float lw = wave_sum(w * lp);
      s_w[h * 64 + lane] = w / lw;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G * D; i += 256) {
      const int h = i / D, d = i - h * D;
      const long base = (((long)b * Hq + kvh * G + h) * S * D + d) * 4;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
      int p = 0;
      for (; p + 4 <= nvalid; p += 4) {  // the reduce kernel's summation order: bit-identical
        a0 += s_w[h * 64 + p] * __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(po_rs, (uint32_t)(base + (long)p * D * 4), 0, kPdSC1));
        a1 += s_w[h * 64 + p + 1] * __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(po_rs, (uint32_t)(base + (long)(p + 1) * D * 4), 0, kPdSC1));
        a2 += s_w[h * 64 + p + 2] * __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(po_rs, (uint32_t)(base + (long)(p + 2) * D * 4), 0, kPdSC1));
        a3 += s_w[h * 64 + p + 3] * __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(po_rs, (uint32_t)(base + (long)(p + 3) * D * 4), 0, kPdSC1));
      }
      for (; p < nvalid; ++p)
        a0 += s_w[h * 64 + p] * __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(po_rs, (uint32_t)(base + (long)p * D * 4), 0, kPdSC1));
      out[act_index(b, (kvh * G + h) * D + d, out_stride)] = f2bf((a0 + a1) + (a2 + a3));
    }
  }
}

// Second launch: merge the split partials.  One workgroup per (kv head, sequence); the (m, l)
// of all splits are read in one parallel step, then every thread sums its (head, dim) items with
// independent loads.  Sequences whose chunks fit one split were finished by the main kernel.
template <int D, int G>
__global__ __launch_bounds__(256) void paged_decode_reduce_kernel(bf16_t* __restrict__ out, long out_stride,
                                                                  const float* __restrict__ part_out,
                                                                  const float* __restrict__ part_ml,
                                                                  const int* __restrict__ seq_lens, int Hq, int S,
                                                                  int kch) {
  __shared__ float s_w[G][64];
  const int kvh = blockIdx.x, b = blockIdx.y;
  const int seq_len = seq_lens[b];
  if (seq_len <= 0) return;
  int c0, c1, nvalid;
  split_range(seq_len, S, 0, kch, &c0, &c1, &nvalid);
  if (nvalid <= 1) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int h = wave; h < G; h += 4) {
    const long ph = ((long)b * Hq + kvh * G + h) * S;
    const float mp = lane < nvalid ? part_ml[(ph + lane) * 2] : -1e30f;
    const float lp = lane < nvalid ? part_ml[(ph + lane) * 2 + 1] : 0.f;
    const float mm = wave_max(mp);
    const float w = lane < nvalid ? exp2f(mp - mm) : 0.f;
    const float lw = wave_sum(w * lp);
    s_w[h][lane] = w / lw;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += 256) {
    const int h = i / D, d = i - h * D;
    const float* po = part_out + ((long)b * Hq + kvh * G + h) * S * D + d;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int p = 0;
    for (; p + 4 <= nvalid; p += 4) {
      a0 += s_w[h][p] * po[(long)p * D];
      a1 += s_w[h][p + 1] * po[(long)(p + 1) * D];
      a2 += s_w[h][p + 2] * po[(long)(p + 2) * D];
      a3 += s_w[h][p + 3] * po[(long)(p + 3) * D];
    }
    for (; p < nvalid; ++p) a0 += s_w[h][p] * po[(long)p * D];
    out[act_index(b, (kvh * G + h) * D + d, out_stride)] = f2bf((a0 + a1) + (a2 + a3));
  }
}

}  // namespace k8sllm

using namespace k8sllm;

// S = number of splits per (sequence, kv head); part buffers hold [B][Hq][S][D].
// out_stride < 0: write the output fragment-packed for gemm_skinny (common.h act_index).
// slabs != nullptr: the fused q/k/v form (D = 128; see DecodeFuse) - q is ignored, the new token's
// q / k / v come from the qkv projection's nslabs fp32 slabs [nslabs][B][(Hq + 2 Hkv) * D], are
// rotated at `positions` and k / v written to the cache at `slot_mapping` (nullptr: no write).
extern "C" int k8sllm_paged_decode_fused(void* out, long out_stride, float* part_out, float* part_ml,
                                         const float* slabs, int nslabs, const int* positions, const float* cos_sin,
                                         const int* slot_mapping, void* k_cache, void* v_cache,
                                         const int* block_tables, int bt_stride, const int* seq_lens, int B, int Hq,
                                         int Hkv, int D, int S, float scale, int* merge_ctr, hipStream_t s);

// Tokens per wave per chunk: the double-buffered 32-token form once the grid fills the chip
// (>= 384 workgroups, e.g. batch 64 x 8 kv heads), else the single-buffered 64-token form (small
// batches, split grids: higher residency).
static int g_tw_force = 0;  // tools/bench_decode_step.py: 32 / 64 forces one form (0: by grid size)
extern "C" void k8sllm_decode_tw_force(int tw) { g_tw_force = tw; }

static int decode_tw(int S, int Hkv, int B) {
  if (g_tw_force == 32 || g_tw_force == 64) return g_tw_force;
  return (long)S * Hkv * B >= 384 ? 32 : 64;
}

extern "C" int k8sllm_paged_decode(void* out, long out_stride, float* part_out, float* part_ml, const void* q,
                                   long q_stride, const void* k_cache, const void* v_cache, const int* block_tables,
                                   int bt_stride, const int* seq_lens, int B, int Hq, int Hkv, int D, int S,
                                   float scale, hipStream_t s) {
  if (B <= 0) return 0;
  if (S < 1 || S > 64) return -2;
  const int G = Hq / Hkv;
  const float sl2 = scale * 1.4426950408889634f;
  const DecodeFuse fz{};
  const int tw = decode_tw(S, Hkv, B);
  dim3 grid(S, Hkv, B), blk(256);
#define K8S_DEC_T(DD, GG, TWV)                                                                                       \
  hipLaunchKernelGGL((paged_decode_kernel<DD, GG, false, TWV>), grid, blk, 0, s, (bf16_t*)out, out_stride, part_out, \
                     part_ml, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache,            \
                     block_tables, bt_stride, seq_lens, Hq, Hkv, S, sl2, fz, nullptr)
#define K8S_DEC(DD, GG)                                                                                              \
  if (tw == 32) K8S_DEC_T(DD, GG, 32); else K8S_DEC_T(DD, GG, 64);                                                  \
  if (S > 1)                                                                                                         \
    hipLaunchKernelGGL((paged_decode_reduce_kernel<DD, GG>), dim3(Hkv, B), blk, 0, s, (bf16_t*)out, out_stride,      \
                       part_out, part_ml, seq_lens, Hq, S, 4 * tw);
  if (D == 128) {
    switch (G) {
      case 1: K8S_DEC(128, 1); break;
      case 2: K8S_DEC(128, 2); break;
      case 4: K8S_DEC(128, 4); break;
      case 8: K8S_DEC(128, 8); break;
      case 16: K8S_DEC(128, 16); break;
      default: return -1;
    }
  } else if (D == 64) {
    switch (G) {
      case 1: K8S_DEC(64, 1); break;
      case 2: K8S_DEC(64, 2); break;
      case 4: K8S_DEC(64, 4); break;
      case 8: K8S_DEC(64, 8); break;
      default: return -1;
    }
  } else {
    return -1;
  }
#undef K8S_DEC
#undef K8S_DEC_T
  return (int)hipGetLastError();
}

extern "C" int k8sllm_paged_decode_fused(void* out, long out_stride, float* part_out, float* part_ml,
                                         const float* slabs, int nslabs, const int* positions, const float* cos_sin,
                                         const int* slot_mapping, void* k_cache, void* v_cache,
                                         const int* block_tables, int bt_stride, const int* seq_lens, int B, int Hq,
                                         int Hkv, int D, int S, float scale, int* merge_ctr, hipStream_t s) {
  if (B <= 0) return 0;
  if (S < 1 || S > 64) return -2;
  if (D != 128 || slabs == nullptr || nslabs < 1 || positions == nullptr || cos_sin == nullptr) return -3;
  const int G = Hq / Hkv;
  const float sl2 = scale * 1.4426950408889634f;
  const DecodeFuse fz{slabs, nslabs, positions, cos_sin, slot_mapping, (bf16_t*)k_cache, (bf16_t*)v_cache};
  const int tw = decode_tw(S, Hkv, B);
  // merge_ctr (B x Hkv ints, zero): split partials merged in-launch by the last arriving split
  const bool merge = merge_ctr != nullptr && S > 1;
  dim3 grid(S, Hkv, B), blk(256);
#define K8S_DECF_T(GG, TWV, MG)                                                                                      \
  hipLaunchKernelGGL((paged_decode_kernel<128, GG, true, TWV, MG>), grid, blk, 0, s, (bf16_t*)out, out_stride,       \
                     part_out, part_ml, nullptr, 0, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables,    \
                     bt_stride, seq_lens, Hq, Hkv, S, sl2, fz, merge_ctr)
#define K8S_DECF(GG)                                                                                                 \
  if (merge) {                                                                                                       \
    if (tw == 32) K8S_DECF_T(GG, 32, true); else K8S_DECF_T(GG, 64, true);                                          \
  } else {                                                                                                           \
    if (tw == 32) K8S_DECF_T(GG, 32, false); else K8S_DECF_T(GG, 64, false);                                        \
    if (S > 1)                                                                                                       \
      hipLaunchKernelGGL((paged_decode_reduce_kernel<128, GG>), dim3(Hkv, B), blk, 0, s, (bf16_t*)out, out_stride,   \
                         part_out, part_ml, seq_lens, Hq, S, 4 * tw);                                                \
  }
  switch (G) {
    case 1: K8S_DECF(1); break;
    case 2: K8S_DECF(2); break;
    case 4: K8S_DECF(4); break;
    case 8: K8S_DECF(8); break;
    default: return -1;
  }
#undef K8S_DECF
#undef K8S_DECF_T
  return (int)hipGetLastError();
}
