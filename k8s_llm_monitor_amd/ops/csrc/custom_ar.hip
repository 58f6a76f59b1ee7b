// IPC all-reduce / all-gather over mapped peer buffers for latency-bound tensor-parallel decode
// messages ("a custom one-shot all-reduce: IPC-mapped peer buffers via
// hipIpcGetMemHandle, then each GPU reads all 7 peers over the 7 links simultaneously and reduces
// locally; hipGraph-capturable, with RCCL as fallback").
//
// An 8-GPU MI355X node is a full xGMI mesh (7 links per GPU).  A ring all-reduce of a decode-sized
// message (64 rows x 8192 x bf16 = 1 MiB for Llama-3-70B at TP=8) pays 2(W-1) latency-bound hops
// on ONE link per direction; one-shot pays one hop and pulls from all 7 peers at once.  Above
// ~0.5 MiB the one-shot form pulls (W-1) x n bytes per rank; the TWO-SHOT form (reduce-scatter,
// then all-gather, inside one launch) pulls 2 (W-1) / W x n - 1.75 n at W = 8 instead of 7 n -
// for one more flag round.
//
// Per call (epoch e = 1 + the number of calls this rank has completed; ONE counter per rank in the
// signal block, advanced on the device by the call's last workgroup, so hipGraph replays advance it
// and every workgroup of a call uses the same buffer half whatever the call's size):
//   1. workgroup b writes its slice of the message into this rank's registered staging buffer
//      (half e & 1 of a double buffer) - a copy of the input, or (fused tail) the projection's
//      split-K partial sum computed straight into it, so that path has no staging copy at all;
//   2. lane 0: system-scope release (writes the XCD L2 back) -> flag[rank][b] = e in EVERY rank's
//      signal block (remote stores over xGMI);
//   3. lanes r < W poll flag[r][b] >= e in this rank's signal block (bounded spin: a peer that never
//      arrives sets `err` and the kernel still exits - it can never hang the GPU);
//   4. system-scope acquire, then the result from the peers' staged slices (plain 16-byte loads):
//      ALL-REDUCE: out[slice] = sum over ranks in RANK ORDER (bit-identical on every rank, as the
//      replicated TP forward requires); ALL-GATHER: out[r * n + slice] = rank r's slice;
//      TWO-SHOT: rank r reduces part r of the slice IN PLACE in its own staging buffer, flags a
//      second round (flag2), and every rank then copies part r from rank r;
//      FUSED TAIL (one workgroup per row): residual += the reduced row, RMSNorm, and the next
//      projection's input written in its final layout - the row-parallel o / down tail of a TP
//      decode layer in ONE launch instead of reduce_slabs + all-reduce + add-norm + pack.
//   5. the last workgroup to finish (done counter) publishes epoch = e.
// Buffer-reuse safety: a rank writes half e & 1 only after completing call e - 1, which required a
// flag of call e - 1 from every peer, i.e. every peer had started call e - 1 and therefore finished
// reading half e & 1 in call e - 2 (both rounds of a two-shot call e - 2 included).  With a per-call
// epoch this holds for any sequence of message sizes and call kinds.
// Signal blocks live in uncached device memory (hipDeviceMallocUncached); data buffers are plain
// hipMalloc memory ordered by the release/acquire pairs.
//
// Memory-ordering argument (car_exchange; the HSA / AMDGPU memory model as it applies to gfx950,
// where each XCD has its own L2 that is NOT coherent with the other XCDs' L2s or with a peer GPU for
// coarse-grained hipMalloc memory):
//  (a) producer side.  Every thread's staging stores are complete at its L2 before the barrier
//      (`s_waitcnt vmcnt(0)` per thread, then __syncthreads: the barrier orders them before lane 0's
//      next instruction).  Lane 0's system-scope RELEASE fence then writes back the dirty lines of
//      this XCD's L2 - the whole cache, so the other threads' completed stores are included - and
//      waits for the write-back before any later store issues.  The flag stores that follow are
//      therefore ordered after the data at system scope (release fence + relaxed store = a
//      release store), wherever the data lives (our staging buffer: a peer reads it over xGMI
//      from our HBM).
//  (b) flag transport.  Flags live in the READER's signal block, uncached memory: the remote
//      store goes straight to the reader's HBM and the reader's relaxed system-scope polls bypass
//      every cache, so a poll cannot be satisfied from a stale line and observes the store once it
//      lands.  Flags only grow (epochs), compared wrap-safe as `(int)(flag - e) >= 0`.
//  (c) consumer side.  Lanes r < W each observe flag[r][b] >= e, then __syncthreads, then lane 0
//      issues a system-scope ACQUIRE fence, which invalidates this CU's L1 and the non-coherent
//      lines of this XCD's L2; a second __syncthreads orders every thread's subsequent loads of
//      the peers' staged data after that invalidation, so they are served from memory written
//      under (a) - the acquire synchronizes-with each peer's release through the flag it read.
//      All threads of a workgroup share one CU, so the one L1 invalidation covers them.
//  (d) two-shot.  Round 2 repeats (a)-(c) over flag2 for the part each rank reduced IN PLACE in
//      its own staging buffer; that reduction reads peers' data (after the round-1 acquire) and
//      writes only the own buffer (before the round-2 release).
//  (e) reuse / epochs.  Half e & 1 of the double buffer is rewritten only in call e + 2; the
//      argument above ("Buffer-reuse safety") shows every peer has finished reading it by then.
//      `epoch` / `done` are agent-scope counters touched only by this rank's own kernels, ordered
//      between launches by stream order (a kernel boundary is a full agent-scope release/acquire),
//      and within a call only the last-arriving workgroup (fetch_add on `done`) publishes it.
//  (f) liveness.  Every spin is bounded (spin_limit); a missing peer sets `err` (checked on the host
//      after the step) and the kernel still completes, so a failed peer cannot hang the GPU.
// Exercised before the engine may use the IPC path: custom_ar.self_test runs every mode against
// exact integer references (tests/test_custom_ar.py at W = 2 / 4 / 8 on one GPU, where the same
// fences order the ranks' accesses across XCDs of that GPU).  Over xGMI between GPUs the protocol
// has NOT been measured: no multi-GPU node was available to this work.
#include <hip/hip_runtime.h>
#include <string.h>

#include "common.h"

namespace k8sllm {

constexpr int CAR_MAX_RANKS = 8;
constexpr int CAR_MAX_WG = 256;

struct CarSignal {
  uint32_t flag[CAR_MAX_RANKS][CAR_MAX_WG];   // flag[src][b]: epoch of src's latest staged slice b
  uint32_t flag2[CAR_MAX_RANKS][CAR_MAX_WG];  // two-shot: epoch of src's reduced part of slice b
  uint32_t epoch;                             // calls completed by this rank
  uint32_t done;                              // workgroups of the current call that have finished
  uint32_t err;                               // set when a peer did not arrive within the spin bound
};

struct CarPeers {
  bf16_t* buf[CAR_MAX_RANKS];      // every rank's staging buffer (2 x max_elems bf16), mapped here
  CarSignal* sig[CAR_MAX_RANKS];   // every rank's signal block, mapped here
};

// this call's epoch (1 + calls completed), read once per workgroup
__device__ __forceinline__ uint32_t car_epoch(CarSignal* my) {
  __shared__ uint32_t s_e;
  if (threadIdx.x == 0) s_e = __hip_atomic_load(&my->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  return s_e;
}

// Publish this workgroup's slice b (every thread's stores issued) and wait for every peer's slice
// b of this call: flags[src][b] in the signal blocks (flag or flag2 round).
template <bool ROUND2>
__device__ __forceinline__ void car_exchange(const CarPeers& p, int rank, int world, int b, uint32_t e,
                                             long spin_limit) {
  CarSignal* my = p.sig[rank];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the staged slice reaches memory
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int r = 0; r < world; ++r) {
      uint32_t* f = ROUND2 ? &p.sig[r]->flag2[rank][b] : &p.sig[r]->flag[rank][b];
      __hip_atomic_store(f, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if ((int)threadIdx.x < world) {
    uint32_t* f = ROUND2 ? &my->flag2[threadIdx.x][b] : &my->flag[threadIdx.x][b];
    long it = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (++it > spin_limit) {
        __hip_atomic_store(&my->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // peers' slices are visible to this CU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// the call's last workgroup to finish publishes the epoch for the next call on this stream
__device__ __forceinline__ void car_finish(CarSignal* my, uint32_t e) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t d = __hip_atomic_fetch_add(&my->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d + 1 == gridDim.x) {
      __hip_atomic_store(&my->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&my->epoch, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ void sum_ranks8(const CarPeers& p, int world, long half, long v, float* acc) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int r = 0; r < world; ++r) {  // fixed rank order: identical sums on every rank
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(p.buf[r] + half)[v], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += f[j];
  }
}

// MODE 0: one-shot all-reduce, 1: one-shot all-gather, 2: two-shot all-reduce, 3: all-to-all.
// n: elements of THIS rank's input (the all-gather output holds world * n; the all-to-all input
// and output are [world][n / world]: out[p] = peer p's in[rank]).
template <int MODE>
__global__ __launch_bounds__(256) void car_kernel(const bf16_t* in, bf16_t* out,  // may alias (reduce)
                                                  long n, long max_elems, int rank, int world, CarPeers p,
                                                  long spin_limit) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  CarSignal* my = p.sig[rank];
  const uint32_t e = car_epoch(my);
  const long half = (long)(e & 1) * max_elems;
  const long nv = n >> 3;  // 16-byte vectors
  const long per = (nv + nb - 1) / nb;
  const long v0 = (long)b * per, v1 = min(nv, v0 + per);

  uint4* mine = reinterpret_cast<uint4*>(p.buf[rank] + half);
  const uint4* src = reinterpret_cast<const uint4*>(in);
  uint4* dst = reinterpret_cast<uint4*>(out);
  if constexpr (MODE == 3) {
    // workgroup b owns vectors [a0, a1) of EVERY destination's block, so the peer's workgroup b
    // staged exactly the part of block `rank` this workgroup reads back (flag[peer][b])
    const long mv = nv / world, pm = (mv + nb - 1) / nb;
    const long a0 = (long)b * pm, a1 = min(mv, a0 + pm);
    for (int q = 0; q < world; ++q)
      for (long v = a0 + tid; v < a1; v += 256) mine[q * mv + v] = src[q * mv + v];
    car_exchange<false>(p, rank, world, b, e, spin_limit);
    for (int r = 0; r < world; ++r) {
      const uint4* peer = reinterpret_cast<const uint4*>(p.buf[r] + half);
      for (long v = a0 + tid; v < a1; v += 256) dst[r * mv + v] = peer[(long)rank * mv + v];
    }
    car_finish(my, e);
    return;
  }
  for (long v = v0 + tid; v < v1; v += 256) mine[v] = src[v];
  car_exchange<false>(p, rank, world, b, e, spin_limit);
  if constexpr (MODE == 1) {
    for (int r = 0; r < world; ++r) {
      const uint4* peer = reinterpret_cast<const uint4*>(p.buf[r] + half);
      for (long v = v0 + tid; v < v1; v += 256) dst[(long)r * nv + v] = peer[v];
    }
  } else if constexpr (MODE == 0) {
    for (long v = v0 + tid; v < v1; v += 256) {
      float acc[8];
      sum_ranks8(p, world, half, v, acc);
      dst[v] = pack8(acc);
    }
  } else {
    // part r of slice b = vectors [v0 + r * pp, v0 + (r + 1) * pp): reduced by rank r in place
    const long pp = (v1 - v0 + world - 1) / world;
    const long a0 = v0 + rank * pp, a1 = min(v1, a0 + pp);
    for (long v = a0 + tid; v < a1; v += 256) {
      float acc[8];
      sum_ranks8(p, world, half, v, acc);
      mine[v] = pack8(acc);
    }
    car_exchange<true>(p, rank, world, b, e, spin_limit);
    for (int r = 0; r < world; ++r) {
      const uint4* peer = reinterpret_cast<const uint4*>(p.buf[r] + half);
      const long r0 = v0 + r * pp, r1 = min(v1, r0 + pp);
      for (long v = r0 + tid; v < r1; v += 256) dst[v] = peer[v];
    }
  }
  car_finish(my, e);
}

// Fused row-parallel tail of a TP decode layer, one workgroup per row m of an [M, d] message:
//   partial = bf16(sum over the ns fp32 split-K slabs of THIS rank's projection)  -> staging
//   y = bf16(sum over ranks, rank order); residual = bf16(residual + y) (written back)
//   out = bf16(residual * rsqrt(mean(residual^2) + eps) * w), row-major (ldo) or, when PACKED,
//         in the fragment-packed A layout of the next skinny GEMM (act_index)
// - exactly the arithmetic of reduce_slabs -> all-reduce -> fused_add_rms_norm -> pack_activation.
// TS (two-shot): rank r sums only its 1/world of the row's columns over the ranks (rank order, fp32,
// rounded to bf16 in place in its staging row) and every rank then gathers the other ranks' reduced
// parts - 2 (W - 1) / W of a row crosses the links per rank instead of W - 1 rows: at TP=8 decode
// (64 x 8192 bf16 per tail) 1.75 MiB inbound per rank instead of 7.  Same sums in the same order:
// bit-identical to the one-shot form.
template <int NC, bool PACKED, bool TS = false>
__global__ __launch_bounds__(256) void car_fused_tail_kernel(const float* __restrict__ slabs, int ns, long slab_stride,
                                                             bf16_t* __restrict__ residual,
                                                             const bf16_t* __restrict__ w, bf16_t* __restrict__ out,
                                                             long ldo, int d, float eps, long max_elems, int rank,
                                                             int world, CarPeers p, long spin_limit) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  CarSignal* my = p.sig[rank];
  const uint32_t e = car_epoch(my);
  const long half = (long)(e & 1) * max_elems;
  const long row = (long)m * d;
  bf16_t* mine = p.buf[rank] + half + row;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < d) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int sl = 0; sl < ns; ++sl) {
        const float4* q = reinterpret_cast<const float4*>(slabs + sl * slab_stride + row + idx);
        const float4 a = q[0], b2 = q[1];
        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
        acc[4] += b2.x; acc[5] += b2.y; acc[6] += b2.z; acc[7] += b2.w;
      }
      *reinterpret_cast<uint4*>(mine + idx) = pack8(acc);
    }
  }
  car_exchange<false>(p, rank, world, m, e, spin_limit);
  const int cs = d / world;  // TS: columns per rank's part (host: d % (8 * world) == 0)
  if constexpr (TS) {
    // reduce-scatter: this rank's part [rank * cs, (rank + 1) * cs) of the row, in place
    for (int i = tid * 8; i < cs; i += 256 * 8) {
      const int idx = rank * cs + i;
      float acc[8];
      sum_ranks8(p, world, half, (row + idx) >> 3, acc);
      *reinterpret_cast<uint4*>(mine + idx) = pack8(acc);
    }
    car_exchange<true>(p, rank, world, m, e, spin_limit);
  }
  float v[NC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < d) {
      float acc[8], r[8];
      if constexpr (TS)  // all-gather: the owner's reduced (bf16) part
        unpack8(*reinterpret_cast<const uint4*>(p.buf[idx / cs] + half + row + idx), acc);
      else
        sum_ranks8(p, world, half, (row + idx) >> 3, acc);
      unpack8(*reinterpret_cast<const uint4*>(residual + row + idx), r);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[c][j] = bf2f(f2bf(bf2f(f2bf(acc[j])) + r[j]));
        ss += v[c][j] * v[c][j];
      }
      *reinterpret_cast<uint4*>(residual + row + idx) = pack8(v[c]);
    }
  }
  ss = block_sum<256>(ss, red);
  const float inv = rsqrtf(ss / (float)d + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < d) {
      float wf[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(w + idx), wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[c][j] * inv * wf[j];
      const long oi = PACKED ? act_index(m, idx, -(long)(d >> 5)) : (long)m * ldo + idx;
      *reinterpret_cast<uint4*>(out + oi) = pack8(o);
    }
  }
  car_finish(my, e);
}

struct CarState {
  int rank = 0, world = 0, device = 0;
  long max_elems = 0;
  bf16_t* buf = nullptr;
  CarSignal* sig = nullptr;
  CarPeers peers{};
  bool opened[CAR_MAX_RANKS] = {};
};

}  // namespace k8sllm

using namespace k8sllm;

// Allocates this rank's staging buffer and signal block; writes their two IPC handles
// (2 x HIP_IPC_HANDLE_SIZE bytes) to `handles`.  Returns the state or nullptr (rc in *err).
extern "C" void* k8sllm_car_create(int rank, int world, long max_elems, void* handles, int* err) {
  *err = 0;
  if (world < 1 || world > CAR_MAX_RANKS || rank < 0 || rank >= world || max_elems <= 0 || max_elems % 8) {
    *err = -1;
    return nullptr;
  }
  auto* st = new CarState();
  st->rank = rank;
  st->world = world;
  st->max_elems = max_elems;
  (void)hipGetDevice(&st->device);
  hipError_t e = hipMalloc((void**)&st->buf, 2 * max_elems * sizeof(bf16_t));
  if (e == hipSuccess) e = hipExtMallocWithFlags((void**)&st->sig, sizeof(CarSignal), hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(st->sig, 0, sizeof(CarSignal));
  hipIpcMemHandle_t hb, hs;
  if (e == hipSuccess) e = hipIpcGetMemHandle(&hb, st->buf);
  if (e == hipSuccess) e = hipIpcGetMemHandle(&hs, st->sig);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    *err = (int)e;
    if (st->buf) (void)hipFree(st->buf);
    if (st->sig) (void)hipFree(st->sig);
    delete st;
    return nullptr;
  }
  memcpy(handles, &hb, sizeof(hb));
  memcpy((char*)handles + sizeof(hb), &hs, sizeof(hs));
  st->peers.buf[rank] = st->buf;
  st->peers.sig[rank] = st->sig;
  return st;
}

extern "C" int k8sllm_car_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// all_handles: world x (buffer handle, signal handle), rank order (from an all-gather).
extern "C" int k8sllm_car_open(void* state, const void* all_handles) {
  auto* st = (CarState*)state;
  const size_t hsz = sizeof(hipIpcMemHandle_t);
  for (int r = 0; r < st->world; ++r) {
    if (r == st->rank) continue;
    hipIpcMemHandle_t hb, hs;
    memcpy(&hb, (const char*)all_handles + (2 * r) * hsz, hsz);
    memcpy(&hs, (const char*)all_handles + (2 * r + 1) * hsz, hsz);
    void *pb = nullptr, *ps = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&pb, hb, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    e = hipIpcOpenMemHandle(&ps, hs, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      (void)hipIpcCloseMemHandle(pb);
      return (int)e;
    }
    st->peers.buf[r] = (bf16_t*)pb;
    st->peers.sig[r] = (CarSignal*)ps;
    st->opened[r] = true;
  }
  return 0;
}

static int car_check(CarState* st, long n) {
  if (n % 8 || n > st->max_elems) return -1;
  for (int r = 0; r < st->world; ++r)
    if (st->peers.buf[r] == nullptr) return -2;  // not opened
  return 0;
}

// workgroups for an n-element message: one per 2048 elements (8 per thread), at most CAR_GRID_CAP.
// The cap keeps a call off most of the chip: a workgroup spinning on a peer's flag holds its CU's
// wave slots, and a full-register GEMM workgroup (256 accumulators per wave: a whole SIMD register
// file) cannot be placed beside it - with every CU holding one, the next GEMM of this rank (or,
// ranks sharing a GPU, of the peer the spin waits for) could not start at all.  64 workgroups
// leave >= 3/4 of the CUs to compute (the overlapped TP prefill runs its all-reduces on the comm
// stream beside the other micro-batch's GEMMs) and still keep ~1 MiB of loads in flight.
constexpr int CAR_GRID_CAP = 64;
static int car_grid(long n) {
  const long nb = (n / 8 + 255) / 256;
  return (int)(nb < 1 ? 1 : (nb > CAR_GRID_CAP ? CAR_GRID_CAP : nb));
}

// out = sum over ranks of in (n bf16, n % 8 == 0, n <= max_elems); in may alias out.
// algo: 0 one-shot, 1 two-shot, -1 auto (two-shot from 512 KiB at W > 2)
extern "C" int k8sllm_car_all_reduce(void* state, const void* in, void* out, long n, long spin_limit, int algo,
                                     hipStream_t s) {
  auto* st = (CarState*)state;
  if (n <= 0) return 0;
  if (int rc = car_check(st, n)) return rc;
  if (algo < 0) algo = (st->world > 2 && n * 2 >= (512L << 10)) ? 1 : 0;
  const int nb = car_grid(n);
  if (algo == 1)
    hipLaunchKernelGGL(car_kernel<2>, dim3(nb), dim3(256), 0, s, (const bf16_t*)in, (bf16_t*)out, n, st->max_elems,
                       st->rank, st->world, st->peers, spin_limit);
  else
    hipLaunchKernelGGL(car_kernel<0>, dim3(nb), dim3(256), 0, s, (const bf16_t*)in, (bf16_t*)out, n, st->max_elems,
                       st->rank, st->world, st->peers, spin_limit);
  return (int)hipGetLastError();
}

// out[world * n] = every rank's in[n] in rank order (n bf16, n % 8 == 0, n <= max_elems); out must
// not alias in.  Same one-shot protocol and epoch as the all-reduce (they may be interleaved).
extern "C" int k8sllm_car_all_gather(void* state, const void* in, void* out, long n, long spin_limit,
                                     hipStream_t s) {
  auto* st = (CarState*)state;
  if (n <= 0) return 0;
  if (int rc = car_check(st, n)) return rc;
  hipLaunchKernelGGL(car_kernel<1>, dim3(car_grid(n)), dim3(256), 0, s, (const bf16_t*)in, (bf16_t*)out, n,
                     st->max_elems, st->rank, st->world, st->peers, spin_limit);
  return (int)hipGetLastError();
}

// out[world][m] = (peer p's in[rank]) for p in rank order; in [world][m] (m = n / world bf16,
// m % 8 == 0, n <= max_elems); out must not alias in.  Static shapes: hipGraph-capturable (the EP
// decode dispatch / combine of fixed per-pair capacity).
extern "C" int k8sllm_car_all_to_all(void* state, const void* in, void* out, long n, long spin_limit,
                                     hipStream_t s) {
  auto* st = (CarState*)state;
  if (n <= 0) return 0;
  if (n % ((long)st->world * 8)) return -1;
  if (int rc = car_check(st, n)) return rc;
  hipLaunchKernelGGL(car_kernel<3>, dim3(car_grid(n / st->world)), dim3(256), 0, s, (const bf16_t*)in,
                     (bf16_t*)out, n, st->max_elems, st->rank, st->world, st->peers, spin_limit);
  return (int)hipGetLastError();
}

// Fused TP row-parallel tail (see car_fused_tail_kernel): slabs [ns][M][d] fp32 (slab_stride
// elements apart), residual [M][d] bf16 updated in place, w [d], out [M][ldo] row-major or
// fragment-packed (packed != 0; ldo ignored).  M <= CAR_MAX_WG, d % 8 == 0, d <= 8192.
// algo: 0 one-shot, 1 two-shot (needs d % (8 world) == 0), -1 auto: two-shot from 512 KiB at
// world > 2 (the plain all-reduce's rule).
extern "C" int k8sllm_car_fused_tail(void* state, const float* slabs, int ns, long slab_stride, void* residual,
                                     const void* w, void* out, long ldo, int M, int d, float eps, int packed,
                                     long spin_limit, int algo, hipStream_t s) {
  auto* st = (CarState*)state;
  if (M <= 0) return 0;
  if (M > CAR_MAX_WG || d % 8 || d > 8192 || ns < 1 || (packed && d % 32)) return -1;
  if (int rc = car_check(st, (long)M * d)) return rc;
  const bool ts_ok = d % (8 * st->world) == 0;
  if (algo == 1 && !ts_ok) return -1;
  const bool ts = algo == 1 || (algo < 0 && ts_ok && st->world > 2 && (long)M * d * 2 >= (512L << 10));
  const int nc = (d + 2047) / 2048;
#define K8_TAIL(NC_, PK_, TS_)                                                                                     \
  hipLaunchKernelGGL((car_fused_tail_kernel<NC_, PK_, TS_>), dim3(M), dim3(256), 0, s, slabs, ns, slab_stride,   \
                     (bf16_t*)residual, (const bf16_t*)w, (bf16_t*)out, ldo, d, eps, st->max_elems, st->rank,    \
                     st->world, st->peers, spin_limit)
  if (ts) {
    if (packed) {
      if (nc <= 2) K8_TAIL(2, true, true); else K8_TAIL(4, true, true);
    } else {
      if (nc <= 2) K8_TAIL(2, false, true); else K8_TAIL(4, false, true);
    }
  } else if (packed) {
    if (nc <= 2) K8_TAIL(2, true, false); else K8_TAIL(4, true, false);
  } else {
    if (nc <= 2) K8_TAIL(2, false, false); else K8_TAIL(4, false, false);
  }
#undef K8_TAIL
  return (int)hipGetLastError();
}

// Enqueue a copy of the error flag to host memory (pinned) on stream s: checked after the step's
// readback instead of a synchronous hipMemcpy per step.
extern "C" int k8sllm_car_error_async(void* state, void* host_dst, hipStream_t s) {
  auto* st = (CarState*)state;
  return (int)hipMemcpyAsync(host_dst, &st->sig->err, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
}

// 1 if a call gave up waiting for a peer (its output is then invalid), else 0; <0 on error.
extern "C" int k8sllm_car_error(void* state) {
  auto* st = (CarState*)state;
  uint32_t v = 0;
  if (hipMemcpy(&v, &st->sig->err, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)v;
}

extern "C" void k8sllm_car_destroy(void* state) {
  auto* st = (CarState*)state;
  if (st == nullptr) return;
  (void)hipDeviceSynchronize();
  for (int r = 0; r < st->world; ++r) {
    if (!st->opened[r]) continue;
    (void)hipIpcCloseMemHandle(st->peers.buf[r]);
    (void)hipIpcCloseMemHandle(st->peers.sig[r]);
  }
  (void)hipFree(st->buf);
  (void)hipFree(st->sig);
  delete st;
}
