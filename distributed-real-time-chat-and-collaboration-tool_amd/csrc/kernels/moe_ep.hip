// Expert-parallel dispatch / combine for the MoE all-to-all (ref call site
// replaced: llm_server/llm_server.py:403, the hosted context-suggestion model).
//
// A rank holds T tokens routed to k experts each (P = T k pairs) and ships every pair to the
// rank that owns its expert.  The send buffer has a STATIC capacity of C rows per destination
// (C = ceil(cf T k / world), cf the capacity factor), so the all-to-alls have fixed, equal
// splits (hipGraph-capturable, no host sync) and move 2 cf T k H elements per rank instead of
// the worst case 2 world T k H.  Three kernels:
//
//   ep_plan     one workgroup: owner rank and slot of every pair (slot = rank of the pair
//               among the pairs with the same owner, in (token, pick) order: deterministic),
//               dst_row[p] = owner C + slot (-1 when slot >= C: dropped), the inverse map
//               send_pair[row] and the expert id of every send row (-1 = padding), and the
//               number of dropped pairs added to an overflow counter (the caller re-runs the
//               step with the worst-case capacity when it is nonzero);
//   ep_gather   send_x[row] = x[send_pair[row] / k] (padding rows are not written);
//   ep_combine  out[t] = sum_j w[t, j] back[dst_row[t k + j]] in fp32, fixed order j
//               (dropped pairs contribute nothing: the overflow counter flags the step).
#include "common.h"
#include "launchers.h"

namespace drtc {
namespace {

constexpr int kPlanThreads = 1024;
constexpr int kEpMaxWorld = 8;

// block-wide exclusive scan of one int per thread (1024 threads = 16 waves)
DRTC_DEVICE int block_excl_scan(int v, int* s_wave, int& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) s_wave[wid] = incl;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kPlanThreads / 64; ++w) {
    const int x = s_wave[w];
    base += (w < wid) ? x : 0;
    tot += x;
  }
  __syncthreads();  // s_wave reuse by the next scan
  total = tot;
  return base + incl - v;
}

__global__ __launch_bounds__(kPlanThreads) void ep_plan_kernel(
    const int* __restrict__ topi, int P, int e_local, int world, int cap,
    int* __restrict__ dst_row, int* __restrict__ send_pair, int* __restrict__ send_e,
    int* __restrict__ overflow) {
  __shared__ int s_wave[kPlanThreads / 64];
  __shared__ int s_total[kEpMaxWorld];
  const int t = threadIdx.x;
  const int per = (P + kPlanThreads - 1) / kPlanThreads;
  const int p0 = min(P, t * per), p1 = min(P, p0 + per);
  int cnt[kEpMaxWorld];
#pragma unroll
  for (int d = 0; d < kEpMaxWorld; ++d) cnt[d] = 0;
  for (int p = p0; p < p1; ++p) {
    const int d = topi[p] / e_local;
#pragma unroll
    for (int q = 0; q < kEpMaxWorld; ++q) cnt[q] += (q == d);
  }
  int base[kEpMaxWorld];
#pragma unroll
  for (int d = 0; d < kEpMaxWorld; ++d) {
    if (d < world) {
      int tot;
      base[d] = block_excl_scan(cnt[d], s_wave, tot);
      if (t == 0) s_total[d] = tot;
    } else {
      base[d] = 0;
    }
  }
  __syncthreads();
  for (int p = p0; p < p1; ++p) {
    const int e = topi[p];
    const int d = e / e_local;
    int slot = 0;
#pragma unroll
    for (int q = 0; q < kEpMaxWorld; ++q)
      if (q == d) slot = base[q]++;
    if (slot < cap) {
      const int r = d * cap + slot;
      dst_row[p] = r;
      send_pair[r] = p;
      send_e[r] = e;
    } else {
      dst_row[p] = -1;
    }
  }
  // padding rows of every destination
  for (int r = t; r < world * cap; r += kPlanThreads) {
    const int d = r / cap, s = r - d * cap;
    if (s >= s_total[d]) {
      send_pair[r] = -1;
      send_e[r] = -1;
    }
  }
  if (t == 0 && overflow != nullptr) {
    int dropped = 0;
    for (int d = 0; d < world; ++d) dropped += max(0, s_total[d] - cap);
    if (dropped) atomicAdd(overflow, dropped);
  }
}

__global__ __launch_bounds__(256) void ep_gather_kernel(
    bf16_t* __restrict__ send_x, const bf16_t* __restrict__ x, const int* __restrict__ send_pair,
    int k, int H, int ldx) {
  const int r = blockIdx.x;
  const int p = send_pair[r];
  if (p < 0) return;
  const bf16x8* src = reinterpret_cast<const bf16x8*>(x + (int64_t)(p / k) * ldx);
  bf16x8* dst = reinterpret_cast<bf16x8*>(send_x + (int64_t)r * H);
  for (int i = threadIdx.x; i < H / 8; i += blockDim.x) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void ep_combine_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ back, const int* __restrict__ dst_row,
    const float* __restrict__ w, int k, int H) {
  const int t = blockIdx.x;
  for (int i = threadIdx.x; i < H / 8; i += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {  // fixed order: identical bits wherever it runs
      const int r = dst_row[t * k + j];
      if (r < 0) continue;
      const float wj = w[t * k + j];
      const bf16x8 v = reinterpret_cast<const bf16x8*>(back + (int64_t)r * H)[i];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += wj * bf2f(v[e]);
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    reinterpret_cast<bf16x8*>(out + (int64_t)t * H)[i] = o;
  }
}

}  // namespace

int launch_ep_plan(const int* topi, int P, int e_local, int world, int cap, int* dst_row,
                   int* send_pair, int* send_e, int* overflow, hipStream_t st) {
  if (P < 0 || e_local < 1 || world < 1 || world > kEpMaxWorld || cap < 1) return -1;
  if (P > 64 * kPlanThreads) return -1;  // one workgroup, <= 64 pairs per thread
  hipLaunchKernelGGL(ep_plan_kernel, dim3(1), dim3(kPlanThreads), 0, st, topi, P, e_local, world,
                     cap, dst_row, send_pair, send_e, overflow);
  return (int)hipGetLastError();
}

int launch_ep_gather(void* send_x, const void* x, const int* send_pair, int rows, int k, int H,
                     int ldx, hipStream_t st) {
  if (rows == 0) return 0;
  if (rows < 0 || k < 1 || H % 8 || ldx % 8 || (uintptr_t)x % 16 || (uintptr_t)send_x % 16)
    return -1;
  hipLaunchKernelGGL(ep_gather_kernel, dim3(rows), dim3(256), 0, st, (bf16_t*)send_x,
                     (const bf16_t*)x, send_pair, k, H, ldx);
  return (int)hipGetLastError();
}

int launch_ep_combine(void* out, const void* back, const int* dst_row, const float* w, int T,
                      int k, int H, hipStream_t st) {
  if (T == 0) return 0;
  if (T < 0 || k < 1 || H % 8 || (uintptr_t)back % 16 || (uintptr_t)out % 16) return -1;
  hipLaunchKernelGGL(ep_combine_kernel, dim3(T), dim3(256), 0, st, (bf16_t*)out,
                     (const bf16_t*)back, dst_row, w, k, H);
  return (int)hipGetLastError();
}

}  // namespace drtc
