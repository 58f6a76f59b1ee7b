// One-shot all-reduce over IPC-mapped peer buffers for latency-bound tensor-parallel decode
// messages ("a custom one-shot all-reduce: IPC-mapped peer buffers via
// hipIpcGetMemHandle, then each GPU reads all 7 peers over the 7 links simultaneously and reduces
// locally; hipGraph-capturable, with RCCL as fallback").
//
// An 8-GPU MI355X node is a full xGMI mesh (7 links per GPU).  A ring all-reduce of a decode-sized
// message (64 rows x 8192 x bf16 = 1 MiB for Llama-3-70B at TP=8) pays 2(W-1) latency-bound hops
// on ONE link per direction; one-shot pays one hop and pulls from all 7 peers at once.
//
// Per call (epoch e = 1 + the number of calls this rank has completed; ONE counter per rank in the
// signal block, advanced on the device by the call's last workgroup, so hipGraph replays advance it
// and every workgroup of a call uses the same buffer half whatever the call's size):
//   1. workgroup b copies its slice of the input into this rank's registered staging buffer
//      (half e & 1 of a double buffer);
//   2. lane 0: system-scope release (writes the XCD L2 back) -> flag[rank][b] = e in EVERY rank's
//      signal block (remote stores over xGMI);
//   3. lanes r < W poll flag[r][b] >= e in this rank's signal block (bounded spin: a peer that never
//      arrives sets `err` and the kernel still exits - it can never hang the GPU);
//   4. system-scope acquire, then the result from the peers' staged slices (plain 16-byte loads):
//      ALL-REDUCE: out[slice] = sum over ranks in RANK ORDER (bit-identical on every rank, as the
//      replicated TP forward requires); ALL-GATHER: out[r * n + slice] = rank r's slice.
//   5. the last workgroup to finish (done counter) publishes epoch = e.
// Buffer-reuse safety: a rank writes half e & 1 only after completing call e - 1, which required a
// flag of call e - 1 from every peer, i.e. every peer had started call e - 1 and therefore finished
// reading half e & 1 in call e - 2.  With a per-call epoch this holds for any sequence of message
// sizes (per-slot epochs, the previous design, broke it when consecutive calls differed in size).
// Signal blocks live in uncached device memory (hipDeviceMallocUncached); data buffers are plain
// hipMalloc memory ordered by the release/acquire pair.
#include <hip/hip_runtime.h>
#include <string.h>

#include "common.h"

namespace k8sllm {

constexpr int CAR_MAX_RANKS = 8;
constexpr int CAR_MAX_WG = 64;

struct CarSignal {
  uint32_t flag[CAR_MAX_RANKS][CAR_MAX_WG];  // flag[src][b]: epoch of src's latest staged slice b
  uint32_t epoch;                            // calls completed by this rank
  uint32_t done;                             // workgroups of the current call that have finished
  uint32_t err;                              // set when a peer did not arrive within the spin bound
};

struct CarPeers {
  bf16_t* buf[CAR_MAX_RANKS];      // every rank's staging buffer (2 x max_elems bf16), mapped here
  CarSignal* sig[CAR_MAX_RANKS];   // every rank's signal block, mapped here
};

// n: elements of THIS rank's input (the all-gather output holds world * n).
template <bool GATHER>
__global__ __launch_bounds__(256) void car_oneshot_kernel(const bf16_t* in, bf16_t* out,  // may alias (reduce)
                                                          long n, long max_elems, int rank, int world, CarPeers p,
                                                          long spin_limit) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  CarSignal* my = p.sig[rank];
  __shared__ uint32_t s_e;
  if (tid == 0) s_e = __hip_atomic_load(&my->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const uint32_t e = s_e;
  const long half = (long)(e & 1) * max_elems;
  const long nv = n >> 3;  // 16-byte vectors
  const long per = (nv + nb - 1) / nb;
  const long v0 = (long)b * per, v1 = min(nv, v0 + per);

  uint4* mine = reinterpret_cast<uint4*>(p.buf[rank] + half);
  const uint4* src = reinterpret_cast<const uint4*>(in);
  for (long v = v0 + tid; v < v1; v += 256) mine[v] = src[v];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the staged slice reaches memory
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int r = 0; r < world; ++r)
      __hip_atomic_store(&p.sig[r]->flag[rank][b], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < world) {
    long it = 0;
    while ((int)(__hip_atomic_load(&my->flag[tid][b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (++it > spin_limit) {
        __hip_atomic_store(&my->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // peers' slices are visible to this CU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  uint4* dst = reinterpret_cast<uint4*>(out);
  if constexpr (GATHER) {
    for (int r = 0; r < world; ++r) {
      const uint4* peer = reinterpret_cast<const uint4*>(p.buf[r] + half);
      for (long v = v0 + tid; v < v1; v += 256) dst[(long)r * nv + v] = peer[v];
    }
  } else {
    for (long v = v0 + tid; v < v1; v += 256) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < world; ++r) {  // fixed rank order: identical sums on every rank
        float f[8];
        unpack8(reinterpret_cast<const uint4*>(p.buf[r] + half)[v], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      }
      dst[v] = pack8(acc);
    }
  }
  __syncthreads();
  if (tid == 0) {  // the call's last workgroup publishes the epoch for the next call on this stream
    const uint32_t d = __hip_atomic_fetch_add(&my->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d + 1 == (uint32_t)nb) {
      __hip_atomic_store(&my->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&my->epoch, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
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

// out = sum over ranks of in (n bf16, n % 8 == 0, n <= max_elems); in may alias out.
extern "C" int k8sllm_car_all_reduce(void* state, const void* in, void* out, long n, long spin_limit,
                                     hipStream_t s) {
  auto* st = (CarState*)state;
  if (n <= 0) return 0;
  if (n % 8 || n > st->max_elems) return -1;
  for (int r = 0; r < st->world; ++r)
    if (st->peers.buf[r] == nullptr) return -2;  // not opened
  const long nv = n / 8;
  int nb = (int)((nv + 255) / 256);
  nb = nb < 1 ? 1 : (nb > CAR_MAX_WG ? CAR_MAX_WG : nb);
  hipLaunchKernelGGL(car_oneshot_kernel<false>, dim3(nb), dim3(256), 0, s, (const bf16_t*)in, (bf16_t*)out, n,
                     st->max_elems, st->rank, st->world, st->peers, spin_limit);
  return (int)hipGetLastError();
}

// out[world * n] = every rank's in[n] in rank order (n bf16, n % 8 == 0, n <= max_elems); out must
// not alias in.  Same one-shot protocol and epoch as the all-reduce (they may be interleaved).
extern "C" int k8sllm_car_all_gather(void* state, const void* in, void* out, long n, long spin_limit,
                                     hipStream_t s) {
  auto* st = (CarState*)state;
  if (n <= 0) return 0;
  if (n % 8 || n > st->max_elems) return -1;
  for (int r = 0; r < st->world; ++r)
    if (st->peers.buf[r] == nullptr) return -2;
  const long nv = n / 8;
  int nb = (int)((nv + 255) / 256);
  nb = nb < 1 ? 1 : (nb > CAR_MAX_WG ? CAR_MAX_WG : nb);
  hipLaunchKernelGGL(car_oneshot_kernel<true>, dim3(nb), dim3(256), 0, s, (const bf16_t*)in, (bf16_t*)out, n,
                     st->max_elems, st->rank, st->world, st->peers, spin_limit);
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
