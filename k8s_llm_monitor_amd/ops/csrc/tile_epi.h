// Fused epilogues of the prefill tile GEMM (gemm_tile.hip): epilogue kinds, their operands, and a
// 16-lane row reduction.
#pragma once
#include "common.h"

namespace k8sllm {

enum { TILE_EPI_BF16 = 0, TILE_EPI_SWIGLU = 1, TILE_EPI_ROPE = 2, TILE_EPI_RESID = 3, TILE_EPI_SWIGLU8 = 4 };

// Fused epilogues of the dense prefill projections.
//
// TILE_EPI_SWIGLU / TILE_EPI_SWIGLU8: silu(gate) * up of a gate/up-interleaved weight, [64 gate |
// 64 up] per 128 rows (interleave_gate_up) or [8 gate | 8 up] per 16 rows (interleave_gate_up8:
// the decode GEMMs' packed copy, so prefill and decode share ONE weight).
//
// TILE_EPI_ROPE (the qkv projection): the output columns are heads of 128; a wave's 128-column
// quarter is exactly one head, and for q / k heads (head < rope_heads) the rotary embedding (neox
// pairs i, i + 64) is applied to the staged bf16 rows before they are stored - rope_cache's
// separate read-rotate-write pass over q / k disappears.
//
// TILE_EPI_RESID (o / down, the residual producers): resid <- bf16(resid + bf16(y)) in place,
// hw <- bf16(resid * norm_w) (the next RMSNorm's weighted input, NOT yet divided by the row's rms)
// and ss_out[row][c] <- sum of resid^2 over the 128 columns c*128 .. c*128+127 - the fused
// residual-add RMSNorm pass between two projections becomes part of the producer's epilogue.
//
// RS (row scale, the consumers qkv / gate_up that read hw): every output row is multiplied by
// rsqrt(sum_c rs_part[row][c] / K + rs_eps) before its epilogue - the deferred half of the RMSNorm
// (a row scale commutes with the projection; SwiGLU and RoPE see the normalised values).
struct TileEpi {
  const int* positions;  // ROPE: [M] absolute position of each row
  const float* cos_sin;  // ROPE: [max_pos][128]: cos (64) | sin (64)
  int rope_heads;        // ROPE: Hq + Hkv: heads 0 .. rope_heads - 1 are rotated
  const float* rs_part;  // RS: [M][rs_np] partial sums of squares of the A rows
  int rs_np;             // RS: partials per row (K / 128, <= 64)
  float rs_eps;
  bf16_t* resid;         // RESID: [M][N] residual stream, updated in place
  bf16_t* hw;            // RESID: [M][N] resid * norm_w
  const bf16_t* norm_w;  // RESID: [N] the next RMSNorm's weight
  float* ss_out;         // RESID: [M][N / 128]
};

// sum over the 16 lanes of a DPP row (lanes 16r .. 16r + 15), the total in every lane
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false));  // row_ror:2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));  // row_ror:1
  return v;
}

}  // namespace k8sllm
