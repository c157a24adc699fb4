// One-shot peer-to-peer all-reduce for tensor-parallel decode.
//
// TP=8 decode issues 2 all-reduces per layer of [batch, hidden] bf16 - small
// messages for which a ring (2(N-1) latency-bound steps, per-link bound on the
// point-to-point xGMI mesh) is the wrong shape.  Here every rank copies its
// input into its own IPC-shared staging buffer, raises a flag in every peer,
// and once all peers' flags are up reads the N staging buffers over xGMI
// (all 7 links busy at once) and sums them in a fixed rank order - so every
// rank produces bit-identical output, which the TP lockstep engines rely on.
//
// Two-shot variant (large messages, e.g. 70B TP=8 decode at batch 256 =
// 4 MiB per all-reduce): reduce-scatter then all-gather over the same staging
// - rank r sums sub-chunk r of every block (fixed rank order) into its result
// area, raises a second flag, and every rank gathers the N reduced sub-chunks.
// Each rank then reads 2(N-1)/N of the message over xGMI instead of N-1 times
// it: 4x less ingress at N = 8, bit-identical results (each element is still
// summed once, in rank order).
//
// Memory: one uncached (fine-grained) device allocation per rank, mapped
// into the peers with hipIpcOpenMemHandle:
//   [0, 2 KiB)        flags[block][src_rank]   written remotely by peers
//   [2 KiB, 2.25 KiB) per-block epoch counters (local)
//   [2.25 KiB, +4)    error word (a flag wait that timed out)
//   [4 KiB, 6 KiB)    phase-2 flags[block][src_rank] (two-shot)
//   [8 KiB, ...)      input staging, then two-shot result staging, each
//                     double-buffered by epoch parity
// Synchronisation is per block: block b of every rank owns the same chunk of
// the message, so block b only waits for block b of the peers (no grid-wide
// barrier, no deadlock whatever the residency).  Epochs grow monotonically,
// so flags never need resetting and the kernel is hipGraph-replayable.  The
// double buffer makes a second barrier unnecessary: a rank can reuse a
// staging half only two calls later, after every peer has raised a flag for
// the intermediate call, i.e. after it finished reading the half.
//
// Every flag wait has a wall-clock bound (s_memrealtime, 100 MHz): a missing
// peer sets the error word and the kernel drains instead of hanging the GPU.
#include "common.h"
#include "launchers.h"

namespace drtc {

constexpr int kArMaxBlocks = 64;
constexpr int kArMaxRanks = 8;
constexpr int64_t kArHeader = 8192;
constexpr int64_t kArFlags2 = 4096;
constexpr uint64_t kArTimeoutTicks = 200000000ull;  // 2 s at 100 MHz

// Publish `epoch` into every peer's flag slot [b][rank] and wait until every
// peer has published it into ours (thread q < world handles peer q).
DRTC_DEVICE void ar_exchange(const ArPeers& P, int64_t flag_off, int* my_flags, int* err, int b,
                             int rank, int world, int epoch) {
  const int tid = threadIdx.x;
  if (tid < world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* peer_flags = reinterpret_cast<int*>(P.base[tid] + flag_off);
    __hip_atomic_store(peer_flags + b * kArMaxRanks + rank, epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(my_flags + b * kArMaxRanks + tid, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kArTimeoutTicks) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

__global__ __launch_bounds__(512) void custom_allreduce_2shot_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ in, ArPeers P, int rank, int world,
    int64_t n8, int64_t stage_elems) {
  __shared__ int s_epoch;
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  char* mine = P.base[rank];
  int* ctr = reinterpret_cast<int*>(mine + 2048);
  int* err = reinterpret_cast<int*>(mine + 2048 + 256);
  if (tid == 0) {
    const int e = ctr[b] + 1;
    ctr[b] = e;
    s_epoch = e;
  }
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t in_off = kArHeader + (int64_t)(epoch & 1) * stage_elems * 2;
  const int64_t res_off = kArHeader + (int64_t)(2 + (epoch & 1)) * stage_elems * 2;
  const int64_t per = (n8 + nb - 1) / nb;
  const int64_t c0 = (int64_t)b * per;
  const int64_t c1 = c0 + per < n8 ? c0 + per : n8;
  const int64_t sub = (c1 - c0 + world - 1) / world;  // sub-chunk reduced by each rank

  bf16x8* my_stage = reinterpret_cast<bf16x8*>(mine + in_off);
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  for (int64_t i = c0 + tid; i < c1; i += blockDim.x) my_stage[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ar_exchange(P, 0, reinterpret_cast<int*>(mine), err, b, rank, world, epoch);
  // reduce-scatter: my sub-chunk of this block, summed over ranks in order
  const int64_t r0 = c0 + rank * sub;
  const int64_t r1 = r0 + sub < c1 ? r0 + sub : c1;
  bf16x8* my_res = reinterpret_cast<bf16x8*>(mine + res_off);
  for (int64_t i = r0 + tid; i < r1; i += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < world; ++q) {
      const bf16x8 v = reinterpret_cast<const bf16x8*>(P.base[q] + in_off)[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    my_res[i] = o;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ar_exchange(P, kArFlags2, reinterpret_cast<int*>(mine + kArFlags2), err, b, rank, world, epoch);
  // all-gather: sub-chunk q of this block from rank q's result area
  bf16x8* dst = reinterpret_cast<bf16x8*>(out);
  for (int64_t i = c0 + tid; i < c1; i += blockDim.x) {
    const int q = (int)((i - c0) / sub);
    dst[i] = reinterpret_cast<const bf16x8*>(P.base[q] + res_off)[i];
  }
}

__global__ __launch_bounds__(512) void custom_allreduce_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ in, ArPeers P, int rank, int world,
    int64_t n8, int64_t stage_elems) {
  __shared__ int s_epoch;
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  char* mine = P.base[rank];
  int* flags = reinterpret_cast<int*>(mine);
  int* ctr = reinterpret_cast<int*>(mine + 2048);
  int* err = reinterpret_cast<int*>(mine + 2048 + 256);
  if (tid == 0) {
    const int e = ctr[b] + 1;
    ctr[b] = e;
    s_epoch = e;
  }
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t buf_off = kArHeader + (int64_t)(epoch & 1) * stage_elems * 2;
  const int64_t per = (n8 + nb - 1) / nb;
  const int64_t c0 = (int64_t)b * per;
  const int64_t c1 = c0 + per < n8 ? c0 + per : n8;

  bf16x8* my_stage = reinterpret_cast<bf16x8*>(mine + buf_off);
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  for (int64_t i = c0 + tid; i < c1; i += blockDim.x) my_stage[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < world) {
    // publish my chunk to peer `tid`, then wait for peer `tid`'s chunk
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* peer_flags = reinterpret_cast<int*>(P.base[tid]);
    __hip_atomic_store(peer_flags + b * kArMaxRanks + rank, epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flags + b * kArMaxRanks + tid, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kArTimeoutTicks) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  bf16x8* dst = reinterpret_cast<bf16x8*>(out);
  for (int64_t i = c0 + tid; i < c1; i += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < world; ++q) {  // fixed order: identical bits on every rank
      const bf16x8 v = reinterpret_cast<const bf16x8*>(P.base[q] + buf_off)[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    dst[i] = o;
  }
}

// header + input staging and result staging, each 2 parities x stage_elems bf16
int64_t custom_ar_buffer_bytes(int64_t stage_elems) { return kArHeader + 8 * stage_elems; }

int launch_custom_allreduce(void* out, const void* in, int64_t n, const ArPeers& peers, int rank,
                            int world, int64_t stage_elems, int two_shot, hipStream_t st) {
  if (n == 0) return 0;
  if (world < 1 || world > kArMaxRanks || rank < 0 || rank >= world || n % 8 != 0 ||
      n > stage_elems)
    return -1;
  const int64_t n8 = n / 8;
  int64_t nb = (n8 + 1023) / 1024;  // >= 2 vectors per thread
  nb = nb < 1 ? 1 : (nb > kArMaxBlocks ? kArMaxBlocks : nb);
  if (two_shot)
    hipLaunchKernelGGL(custom_allreduce_2shot_kernel, dim3((int)nb), dim3(512), 0, st,
                       (bf16_t*)out, (const bf16_t*)in, peers, rank, world, n8, stage_elems);
  else
    hipLaunchKernelGGL(custom_allreduce_kernel, dim3((int)nb), dim3(512), 0, st, (bf16_t*)out,
                       (const bf16_t*)in, peers, rank, world, n8, stage_elems);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------ host helpers
int ar_alloc(void** p, int64_t bytes) {
  hipError_t e = hipExtMallocWithFlags(p, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*p, 0, (size_t)bytes);
}

int ar_free(void* p) { return (int)hipFree(p); }

int ar_ipc_get(void* p, char* handle) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  *reinterpret_cast<hipIpcMemHandle_t*>(handle) = h;
  return 0;
}

int ar_ipc_open(const char* handle, void** p) {
  const hipIpcMemHandle_t h = *reinterpret_cast<const hipIpcMemHandle_t*>(handle);
  return (int)hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess);
}

int ar_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

int ar_error(void* base) {
  int v = 0;
  hipError_t e = hipMemcpy(&v, (char*)base + 2048 + 256, 4, hipMemcpyDeviceToHost);
  return e != hipSuccess ? -(int)e : v;
}

}  // namespace drtc
