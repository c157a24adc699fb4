// Fused token sampler (gfx950): one 1024-thread workgroup (16 waves) per row.
//
//  * temperature <= 0 : greedy argmax (ties -> lowest index).
//  * otherwise        : exact top-k by a 16-bit radix select on the bf16 keys
//                       (two 8-bit passes, wave-private LDS histograms so the
//                       16 waves never contend on one bin) -> the <= 1024
//                       candidates are gathered into LDS, bitonic-sorted
//                       (only up to the next power of two of their count),
//                       softmax'd with the temperature, cut at top-p on the
//                       inclusive prefix sum, and drawn by inverse CDF.
// Rows are streamed with 16-byte loads (8 bf16 per lane) when the row is
// 16-B aligned.  The random draw is a counter-based hash of
// (seed, step, row); `step` lives in device memory so the kernel replays
// inside a hipGraph (the host advances it with a captured increment).
#include "common.h"
#include "launchers.h"

namespace drtc {

constexpr int kSampThreads = 1024;
constexpr int kSampWaves = kSampThreads / 64;
constexpr int kCand = 1024;

DRTC_DEVICE unsigned ord16(unsigned short b) {
  // bf16 bit pattern -> unsigned key ordered like the float value
  return (b & 0x8000u) ? (unsigned)(~b & 0xFFFFu) : (unsigned)(b | 0x8000u);
}
DRTC_DEVICE float bits2f(unsigned short b) { return __uint_as_float((unsigned)b << 16); }

DRTC_DEVICE uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

// Visit every element of the row: f(index, raw bf16 bits).
template <class F>
DRTC_DEVICE void for_row(const unsigned short* lr, int V, bool vec, F&& f) {
  const int tid = threadIdx.x;
  if (vec) {
    const int nv = V >> 3;
    for (int v = tid; v < nv; v += kSampThreads) {
      const u16x8 x = *reinterpret_cast<const u16x8*>(lr + 8 * v);
#pragma unroll
      for (int j = 0; j < 8; ++j) f(8 * v + j, x[j]);
    }
    for (int i = (nv << 3) + tid; i < V; i += kSampThreads) f(i, lr[i]);
  } else {
    for (int i = tid; i < V; i += kSampThreads) f(i, lr[i]);
  }
}

__global__ __launch_bounds__(kSampThreads) void sample_kernel(
    int* __restrict__ out_tokens, const bf16_t* __restrict__ logits, int V,
    int ld, const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, uint64_t seed,
    const int64_t* __restrict__ step) {
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const unsigned short* lr = (const unsigned short*)(logits + (int64_t)row * ld);
  const bool vec = ((reinterpret_cast<uintptr_t>(lr) & 15) == 0);
  const float temp = temperature ? temperature[row] : 0.f;

  __shared__ float s_val[kCand];
  __shared__ int s_idx[kCand];
  __shared__ unsigned s_hist[kSampWaves][256];
  __shared__ int s_misc[4];

  if (temp <= 0.f) {  // ---------------------------------- greedy argmax
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for_row(lr, V, vec, [&](int i, unsigned short b) {
      const float v = bits2f(b);
      if (v > best || (v == best && i < bi)) { best = v; bi = i; }
    });
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (lane == 0) { s_val[wid] = best; s_idx[wid] = bi; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < kSampWaves; ++w)
        if (s_val[w] > best || (s_val[w] == best && s_idx[w] < bi)) { best = s_val[w]; bi = s_idx[w]; }
      out_tokens[row] = bi;
    }
    return;
  }

  // ------------------------------------------------ top-k radix select
  int k = (top_k && top_k[row] > 0) ? top_k[row] : kCand;
  if (k > kCand) k = kCand;
  if (k > V) k = V;
  unsigned prefix = 0, mask = 0;
  int remaining = k;
  for (int pass = 8; pass >= 0; pass -= 8) {
    for (int i = tid; i < kSampWaves * 256; i += kSampThreads) (&s_hist[0][0])[i] = 0;
    __syncthreads();
    unsigned* h = s_hist[wid];
    for_row(lr, V, vec, [&](int, unsigned short b) {
      const unsigned key = ord16(b);
      if ((key & mask) == prefix) atomicAdd(&h[(key >> pass) & 255u], 1u);
    });
    __syncthreads();
    if (tid < 256) {
      unsigned s = 0;
#pragma unroll
      for (int w = 0; w < kSampWaves; ++w) s += s_hist[w][tid];
      s_hist[0][tid] = s;
    }
    __syncthreads();
    if (tid == 0) {
      int cum = 0, d = 255;
      for (; d > 0; --d) {
        if (cum + (int)s_hist[0][d] >= remaining) break;
        cum += s_hist[0][d];
      }
      s_misc[0] = d;
      s_misc[1] = remaining - cum;
    }
    __syncthreads();
    prefix |= (unsigned)s_misc[0] << pass;
    mask |= 255u << pass;
    remaining = s_misc[1];
    __syncthreads();
  }
  const unsigned thr = prefix;  // key of the k-th largest logit

  // ------------------------------------------------ gather candidates
  if (tid == 0) s_misc[2] = 0;
  s_val[tid] = -INFINITY;
  s_idx[tid] = 0x7fffffff;
  __syncthreads();
  for_row(lr, V, vec, [&](int i, unsigned short b) {
    if (ord16(b) >= thr) {
      const int slot = atomicAdd(&s_misc[2], 1);
      if (slot < kCand) { s_val[slot] = bits2f(b); s_idx[slot] = i; }
    }
  });
  __syncthreads();
  int n = s_misc[2];
  if (n > kCand) n = kCand;
  int np2 = 1;
  while (np2 < n) np2 <<= 1;

  // ------------------------------------------------ bitonic sort (desc)
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int j = tid ^ stride;
      if (tid < np2 && j > tid) {
        const bool desc = ((tid & size) == 0);
        const float a = s_val[tid], b = s_val[j];
        const int ia = s_idx[tid], ib = s_idx[j];
        const bool a_first = (a > b) || (a == b && ia < ib);
        if (desc != a_first) {
          s_val[tid] = b; s_val[j] = a;
          s_idx[tid] = ib; s_idx[j] = ia;
        }
      }
      __syncthreads();
    }
  }

  // ------------------------------------------------ softmax + top-p + draw
  const float top = s_val[0];
  const float inv_t = 1.f / temp;
  const float pv = (tid < n) ? __expf((s_val[tid] - top) * inv_t) : 0.f;
  __syncthreads();
  s_val[tid] = pv;
  __syncthreads();
  for (int off = 1; off < np2; off <<= 1) {  // inclusive Hillis-Steele scan
    const float add = (tid >= off && tid < np2) ? s_val[tid - off] : 0.f;
    __syncthreads();
    s_val[tid] += add;
    __syncthreads();
  }
  const float total = s_val[n - 1];
  const float pp = (top_p && top_p[row] > 0.f && top_p[row] < 1.f) ? top_p[row] : 1.f;
  if (tid == 0) s_misc[3] = n - 1;
  __syncthreads();
  {
    const float need = pp * total;
    const bool hit = tid < n && s_val[tid] >= need && (tid == 0 || s_val[tid - 1] < need);
    if (hit) s_misc[3] = tid;
  }
  __syncthreads();
  const int cut = s_misc[3];
  const uint64_t st = step ? (uint64_t)step[0] : 0ull;
  const uint64_t hsh = mix64(seed ^ mix64(st * 0x9E3779B97F4A7C15ULL + (uint64_t)row));
  const float u = (float)((hsh >> 40) + 0.5) * (1.0f / 16777216.0f);
  const float target = u * s_val[cut];
  if (tid <= cut) {
    const float lo = (tid == 0) ? 0.f : s_val[tid - 1];
    if (target >= lo && (target < s_val[tid] || tid == cut)) out_tokens[row] = s_idx[tid];
  }
}

int launch_sample(int* out_tokens, const void* logits, int B, int V, int ld,
                  const float* temperature, const int* top_k, const float* top_p,
                  uint64_t seed, const int64_t* step, hipStream_t st) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(sample_kernel, dim3(B), dim3(kSampThreads), 0, st, out_tokens,
                     (const bf16_t*)logits, V, ld, temperature, top_k, top_p,
                     seed, step);
  return (int)hipGetLastError();
}

}  // namespace drtc
