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
//   [0, 4 KiB)        flags[block][src_rank] (u64 epochs) written remotely by peers
//   [4 KiB, 8 KiB)    phase-2 flags[block][src_rank] (two-shot)
//   [8 KiB, +512)     per-block epoch counters (u64, local)
//   [8.5 KiB, +4)     error word (a flag wait that timed out)
//   [16 KiB, ...)     input staging, then two-shot result staging, each
//                     double-buffered by epoch parity
// Synchronisation is per block: the message is cut into FIXED chunks of
// `chunk` vectors (stage_elems / 64 blocks, the same for every call of a
// communicator), block b always owns chunk b, and block b only waits for
// block b of the peers (no grid-wide barrier, no deadlock whatever the
// residency).  Because chunk b's staging range never depends on the message
// size, the double buffer needs no second barrier even across calls of
// different sizes: block b reuses a staging half only two of ITS calls later,
// after every peer's block b has raised a flag for the intermediate call,
// i.e. after it finished reading the half.  Epochs are 64-bit and grow
// monotonically (no wrap in any realistic uptime: 2^64 calls), so flags never
// need resetting and the kernel is hipGraph-replayable.
//
// Every flag wait has a wall-clock bound (s_memrealtime, 100 MHz): a missing
// peer sets the error word and the kernel drains instead of hanging the GPU;
// the TP engine checks the word at every step boundary and fails the group
// (parallel/tp_engine.py).
#include "common.h"
#include "launchers.h"

namespace drtc {

constexpr int kArMaxBlocks = 64;
constexpr int kArMaxRanks = 8;
constexpr int64_t kArHeader = 16384;
constexpr int64_t kArFlags2 = 4096;
constexpr int64_t kArCounters = 8192;
constexpr int64_t kArError = 8192 + 512;
constexpr uint64_t kArTimeoutTicks = 200000000ull;  // 2 s at 100 MHz

// Publish `epoch` into every peer's flag slot [b][rank] and wait until every
// peer has published it into ours (thread q < world handles peer q).
DRTC_DEVICE void ar_exchange(const ArPeers& P, int64_t flag_off, uint64_t* my_flags, int* err,
                             int b, int rank, int world, uint64_t epoch) {
  const int tid = threadIdx.x;
  if (tid < world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint64_t* peer_flags = reinterpret_cast<uint64_t*>(P.base[tid] + flag_off);
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
    int64_t n8, int64_t stage_elems, int64_t chunk) {
  __shared__ uint64_t s_epoch;
  const int b = blockIdx.x, tid = threadIdx.x;
  char* mine = P.base[rank];
  uint64_t* ctr = reinterpret_cast<uint64_t*>(mine + kArCounters);
  int* err = reinterpret_cast<int*>(mine + kArError);
  if (tid == 0) {
    const uint64_t e = ctr[b] + 1;
    ctr[b] = e;
    s_epoch = e;
  }
  __syncthreads();
  const uint64_t epoch = s_epoch;
  const int64_t in_off = kArHeader + (int64_t)(epoch & 1) * stage_elems * 2;
  const int64_t res_off = kArHeader + (int64_t)(2 + (epoch & 1)) * stage_elems * 2;
  const int64_t c0 = (int64_t)b * chunk;  // fixed per block, whatever the message size
  const int64_t c1 = c0 + chunk < n8 ? c0 + chunk : n8;
  const int64_t sub = (c1 - c0 + world - 1) / world;  // sub-chunk reduced by each rank

  bf16x8* my_stage = reinterpret_cast<bf16x8*>(mine + in_off);
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  for (int64_t i = c0 + tid; i < c1; i += blockDim.x) my_stage[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ar_exchange(P, 0, reinterpret_cast<uint64_t*>(mine), err, b, rank, world, epoch);
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
  ar_exchange(P, kArFlags2, reinterpret_cast<uint64_t*>(mine + kArFlags2), err, b, rank, world,
              epoch);
  // all-gather: sub-chunk q of this block from rank q's result area
  bf16x8* dst = reinterpret_cast<bf16x8*>(out);
  for (int64_t i = c0 + tid; i < c1; i += blockDim.x) {
    const int q = (int)((i - c0) / sub);
    dst[i] = reinterpret_cast<const bf16x8*>(P.base[q] + res_off)[i];
  }
}

__global__ __launch_bounds__(512) void custom_allreduce_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ in, ArPeers P, int rank, int world,
    int64_t n8, int64_t stage_elems, int64_t chunk) {
  __shared__ uint64_t s_epoch;
  const int b = blockIdx.x, tid = threadIdx.x;
  char* mine = P.base[rank];
  uint64_t* flags = reinterpret_cast<uint64_t*>(mine);
  uint64_t* ctr = reinterpret_cast<uint64_t*>(mine + kArCounters);
  int* err = reinterpret_cast<int*>(mine + kArError);
  if (tid == 0) {
    const uint64_t e = ctr[b] + 1;
    ctr[b] = e;
    s_epoch = e;
  }
  __syncthreads();
  const uint64_t epoch = s_epoch;
  const int64_t buf_off = kArHeader + (int64_t)(epoch & 1) * stage_elems * 2;
  const int64_t c0 = (int64_t)b * chunk;  // fixed per block, whatever the message size
  const int64_t c1 = c0 + chunk < n8 ? c0 + chunk : n8;

  const int64_t s0 = (int64_t)b * chunk - c0;  // staging index = element index + s0
  bf16x8* my_stage = reinterpret_cast<bf16x8*>(mine + buf_off) + s0;
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  for (int64_t i = c0 + tid; i < c1; i += blockDim.x) my_stage[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < world) {
    // publish my chunk to peer `tid`, then wait for peer `tid`'s chunk
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint64_t* peer_flags = reinterpret_cast<uint64_t*>(P.base[tid]);
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

// One-shot all-reduce fused with the residual add and RMSNorm of a TP decode
// sublayer: h = residual + sum_q partial_q (fixed rank order, rounded to bf16 once
// as the all-reduce alone would), residual <- h, normed = rmsnorm(h) * w (Gemma:
// * (1 + w)).  Block b owns whole rows [b R, (b+1) R), R = floor(chunk / (H / 8)), and
// stages them at the START of its own fixed chunk [b chunk, (b+1) chunk) of the staging
// buffer (not at row * H / 8, which crosses into block b-1's chunk whenever chunk is not a
// multiple of H / 8, e.g. H = 5120), so the epoch/parity protocol is the one of the plain
// kernels (they may be interleaved on one communicator).  Every rank
// reduces the same bytes in the same order: bit-identical outputs on all ranks.
__global__ __launch_bounds__(512) void custom_ar_rmsnorm_kernel(
    bf16_t* __restrict__ normed, bf16_t* __restrict__ residual, const bf16_t* __restrict__ in,
    const bf16_t* __restrict__ w, ArPeers P, int rank, int world, int rows, int H, float eps,
    int gemma, int64_t stage_elems, int rows_per_block, int64_t chunk) {
  __shared__ uint64_t s_epoch;
  __shared__ float s_red[16];
  const int b = blockIdx.x, tid = threadIdx.x;
  char* mine = P.base[rank];
  uint64_t* flags = reinterpret_cast<uint64_t*>(mine);
  uint64_t* ctr = reinterpret_cast<uint64_t*>(mine + kArCounters);
  int* err = reinterpret_cast<int*>(mine + kArError);
  if (tid == 0) {
    const uint64_t e = ctr[b] + 1;
    ctr[b] = e;
    s_epoch = e;
  }
  __syncthreads();
  const uint64_t epoch = s_epoch;
  const int64_t buf_off = kArHeader + (int64_t)(epoch & 1) * stage_elems * 2;
  const int hv = H / 8;  // vectors per row
  const int r0 = b * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  const int64_t c0 = (int64_t)r0 * hv, c1 = (int64_t)r1 * hv;
  const int64_t s0 = (int64_t)b * chunk - c0;  // staging index = element index + s0
  bf16x8* my_stage = reinterpret_cast<bf16x8*>(mine + buf_off) + s0;
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  for (int64_t i = c0 + tid; i < c1; i += blockDim.x) my_stage[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ar_exchange(P, 0, flags, err, b, rank, world, epoch);
  const bf16x8* wv = reinterpret_cast<const bf16x8*>(w);
  bf16x8* res = reinterpret_cast<bf16x8*>(residual);
  bf16x8* outv = reinterpret_cast<bf16x8*>(normed);
  const int lane = tid & 63, wid = tid >> 6;
  for (int row = r0; row < r1; ++row) {
    float ss = 0.f;
    for (int j = tid; j < hv; j += blockDim.x) {
      const int64_t i = (int64_t)row * hv + j;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int q = 0; q < world; ++q) {
        const bf16x8 v = reinterpret_cast<const bf16x8*>(P.base[q] + buf_off)[i + s0];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += bf2f(v[e]);
      }
      const bf16x8 rv = res[i];
      bf16x8 hsum;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float o = bf2f(f2bf(acc[e]));  // the all-reduce result, rounded once
        hsum[e] = f2bf(o + bf2f(rv[e]));
        const float hf = bf2f(hsum[e]);
        ss += hf * hf;
      }
      res[i] = hsum;
    }
    ss = wave_sum(ss);
    if (lane == 0) s_red[wid] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) tot += s_red[k];
    const float rstd = rsqrtf(tot / (float)H + eps);
    for (int j = tid; j < hv; j += blockDim.x) {
      const int64_t i = (int64_t)row * hv + j;
      const bf16x8 hsum = res[i];  // this thread wrote it above
      const bf16x8 ww = wv[j];
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        o[e] = f2bf(bf2f(hsum[e]) * rstd * (bf2f(ww[e]) + (gemma ? 1.f : 0.f)));
      outv[i] = o;
    }
    __syncthreads();  // s_red reuse
  }
}

int launch_custom_ar_rmsnorm(void* normed, void* residual, const void* in, const void* w,
                             int rows, int H, float eps, int gemma, const ArPeers& peers,
                             int rank, int world, int64_t stage_elems, hipStream_t st) {
  if (rows == 0) return 0;
  if (world < 1 || world > kArMaxRanks || rank < 0 || rank >= world || H % 8 != 0 || H > 16384 ||
      (int64_t)rows * H > stage_elems)
    return -1;
  const int64_t chunk = (stage_elems / 8 + kArMaxBlocks - 1) / kArMaxBlocks;  // vectors
  const int rpb = (int)(chunk / (H / 8));
  if (rpb < 1) return -1;  // a row does not fit one block's fixed chunk
  const int nb = (rows + rpb - 1) / rpb;
  if (nb > kArMaxBlocks) return -1;
  hipLaunchKernelGGL(custom_ar_rmsnorm_kernel, dim3(nb), dim3(512), 0, st, (bf16_t*)normed,
                     (bf16_t*)residual, (const bf16_t*)in, (const bf16_t*)w, peers, rank, world,
                     rows, H, eps, gemma, stage_elems, rpb, chunk);
  return (int)hipGetLastError();
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
  // fixed partition of the staging area: chunk b always belongs to block b
  const int64_t chunk = (stage_elems / 8 + kArMaxBlocks - 1) / kArMaxBlocks;
  const int64_t nb = (n8 + chunk - 1) / chunk;
  if (two_shot)
    hipLaunchKernelGGL(custom_allreduce_2shot_kernel, dim3((int)nb), dim3(512), 0, st,
                       (bf16_t*)out, (const bf16_t*)in, peers, rank, world, n8, stage_elems, chunk);
  else
    hipLaunchKernelGGL(custom_allreduce_kernel, dim3((int)nb), dim3(512), 0, st, (bf16_t*)out,
                       (const bf16_t*)in, peers, rank, world, n8, stage_elems, chunk);
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
  hipError_t e = hipMemcpy(&v, (char*)base + kArError, 4, hipMemcpyDeviceToHost);
  return e != hipSuccess ? -(int)e : v;
}

// Test hook: start every local epoch counter and flag at `epoch` (all ranks
// must call it with the same value, with no all-reduce in flight).
int ar_set_epoch(void* base, uint64_t epoch) {
  uint64_t h[kArMaxBlocks * kArMaxRanks];
  for (auto& v : h) v = epoch;
  hipError_t e = hipMemcpy(base, h, sizeof(h), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy((char*)base + kArFlags2, h, sizeof(h), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy((char*)base + kArCounters, h, 8 * kArMaxBlocks, hipMemcpyHostToDevice);
  return (int)e;
}

}  // namespace drtc
