// Fused token sampler (gfx950): one 1024-thread workgroup (16 waves) per row.
//
//  * temperature <= 0 : greedy argmax (ties -> lowest index), one row pass.
//  * 0 < top_k <= 1024: exact top-k, then temperature softmax + top-p over the
//    k candidates.  Selection without a histogram in the common case: every
//    thread keeps the max key of the elements it streams; the k-th largest of
//    those 1024 thread maxima is a lower bound tau0 on the k-th largest logit
//    (the top-k thread maxima are k distinct elements >= tau0), so gathering
//    `key >= tau0` yields all top-k plus a few extra (~k + O(1) on real logit
//    rows), and such an element can only sit in a thread whose own max is
//    >= tau0: only those ~k threads re-read their own elements to gather.
//    One row pass.  If ties push the gather past 1024 slots, the row falls
//    back to a 16-bit radix select (two histogram passes) and a ballot-
//    compacted full gather.
//    Candidates are bitonic-sorted; all tokens tied with the k-th value stay.
//  * top_k == 0       : temperature sampling with EXACT top-p over the whole
//    vocabulary (no candidate cap).  With p_i ~ exp(x_i / T) and
//    P = top_p * sum(p), token i is in the nucleus iff the mass of tokens
//    strictly more probable than i is < P (ties are in or out together).
//    Pivot rejection: draw j from the tokens above a pivot L (inverse CDF:
//    per-thread masses, block scan, the owning thread re-walks its own
//    elements), then one row pass computes mass(key > key_j); accept if < P,
//    else every token up to key_j is outside and L = key_j.  The same pass
//    evaluates a bisection key between L and a known-inside bound H, so the
//    pivot range halves every pass: <= ~17 passes worst case, 1-2 on real
//    distributions.  Accepted draws follow p restricted to the nucleus
//    exactly (the eligible set always contains the nucleus).
// Rows are streamed with 16-byte loads (8 bf16 per lane) when 16-B aligned.
// The random draws are counter-based hashes of (seed, step, row, round);
// `step` lives in device memory so the kernel replays inside a hipGraph.
// Keys: bf16 bit patterns mapped to unsigned 16-bit keys ordered like the
// float values, so comparisons on keys are exact comparisons on logits.
#include "common.h"
#include "launchers.h"

namespace drtc {

constexpr int kSampThreads = 1024;
constexpr int kSampWaves = kSampThreads / 64;
constexpr int kCand = 1024;
constexpr int kMaxRounds = 40;

DRTC_DEVICE unsigned ord16(unsigned short b) {
  return (b & 0x8000u) ? (unsigned)(~b & 0xFFFFu) : (unsigned)(b | 0x8000u);
}
DRTC_DEVICE float bits2f(unsigned short b) { return __uint_as_float((unsigned)b << 16); }

DRTC_DEVICE uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}
// uniform in (0, 1) for draw `round` of (seed, step, row)
DRTC_DEVICE float uniform(uint64_t seed, uint64_t st, int row, int round) {
  const uint64_t h = mix64(seed ^ mix64(st * 0x9E3779B97F4A7C15ULL + (uint64_t)row) +
                           (uint64_t)round * 0xD1B54A32D192ED03ULL);
  return (float)((h >> 40) + 0.5) * (1.0f / 16777216.0f);
}

// Visit this thread's elements of the row, in a fixed order: f(index, raw bf16).
// kUnroll 16-byte loads are issued before any is consumed (a lane streams
// ~16 vectors of a 128k row: one load in flight would leave the pass
// latency-bound at about half the HBM rate).
constexpr int kUnroll = 4;  // default U (one workgroup per CU)
template <int U, class F>
DRTC_DEVICE void for_row(const unsigned short* lr, int V, bool vec, F&& f) {
  const int tid = threadIdx.x;
  if (vec) {
    const int nv = V >> 3;
    for (int v = tid; v < nv; v += U * kSampThreads) {
      u16x8 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (v + u * kSampThreads < nv)
          x[u] = *reinterpret_cast<const u16x8*>(lr + 8 * (v + u * kSampThreads));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (v + u * kSampThreads < nv) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f(8 * (v + u * kSampThreads) + j, x[u][j]);
        }
      }
    }
    for (int i = (nv << 3) + tid; i < V; i += kSampThreads) f(i, lr[i]);
  } else {
    for (int i = tid; i < V; i += kSampThreads) f(i, lr[i]);
  }
}

DRTC_DEVICE float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
DRTC_DEVICE float wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, 64));
  return x;
}

struct SampShared {
  float val[kCand];
  int idx[kCand];
  unsigned hist[kSampWaves][256];
  float wred[4][kSampWaves];
  int misc[8];
};

// Sum over the block of two values (fixed order: deterministic).
DRTC_DEVICE void block_sum2(SampShared& s, float a, float b, float& ra, float& rb) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) { s.wred[0][wid] = a; s.wred[1][wid] = b; }
  __syncthreads();
  float x = 0.f, y = 0.f;
#pragma unroll
  for (int w = 0; w < kSampWaves; ++w) { x += s.wred[0][w]; y += s.wred[1][w]; }
  __syncthreads();
  ra = x; rb = y;
}

// Exclusive block scan of v (thread order); also returns the block total and
// the highest thread index with v > 0 (-1 if none).
DRTC_DEVICE float block_excl_scan(SampShared& s, float v, float& total, int& last_pos) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  const uint64_t pos = __ballot(v > 0.f);
  if (lane == 63) {
    s.wred[2][wid] = x;
    s.wred[3][wid] = pos ? __int_as_float(wid * 64 + 63 - __clzll(pos)) : __int_as_float(-1);
  }
  __syncthreads();
  float off = 0.f, tot = 0.f;
  int lp = -1;
#pragma unroll
  for (int w = 0; w < kSampWaves; ++w) {
    const float t = s.wred[2][w];
    if (w < wid) off += t;
    tot += t;
    lp = max(lp, __float_as_int(s.wred[3][w]));
  }
  __syncthreads();
  total = tot;
  last_pos = lp;
  return off + x - v;
}

// Among 256 bins (hist[d], d = 0..255), walking from the top bin down, the bin
// where the running count reaches `remaining`: returns it in misc[0] and the
// count still needed inside it in misc[1].  Threads 0..255 take part.
DRTC_DEVICE void select_bin(SampShared& s, const unsigned* hist, int remaining) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int c = 0, x = 0;
  if (tid < 256) {
    c = (int)hist[255 - tid];
    x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) s.misc[4 + wid] = x;  // misc[4..7]: 4 wave totals
  }
  __syncthreads();
  if (tid < 256) {
    int off = 0;
    for (int w = 0; w < wid; ++w) off += s.misc[4 + w];
    const int incl = off + x, excl = incl - c;
    if (incl >= remaining && excl < remaining) { s.misc[0] = 255 - tid; s.misc[1] = remaining - excl; }
    if (tid == 255 && incl < remaining) { s.misc[0] = 0; s.misc[1] = remaining - excl; }
  }
  __syncthreads();
}

// Exact key of the k-th largest element by a 16-bit radix select (two
// histogram passes over the row; per-wave histograms).
template <int U>
DRTC_DEVICE unsigned radix_kth(SampShared& s, const unsigned short* lr, int V, bool vec, int k) {
  const int tid = threadIdx.x, wid = tid >> 6;
  unsigned prefix = 0, mask = 0;
  int remaining = k;
  for (int pass = 8; pass >= 0; pass -= 8) {
    for (int i = tid; i < kSampWaves * 256; i += kSampThreads) (&s.hist[0][0])[i] = 0;
    __syncthreads();
    unsigned* h = s.hist[wid];
    for_row<U>(lr, V, vec, [&](int, unsigned short b) {
      const unsigned key = ord16(b);
      if ((key & mask) == prefix) atomicAdd(&h[(key >> pass) & 255u], 1u);
    });
    __syncthreads();
    if (tid < 256) {
      unsigned t = 0;
#pragma unroll
      for (int w = 1; w < kSampWaves; ++w) t += s.hist[w][tid];
      s.hist[0][tid] += t;
    }
    __syncthreads();
    select_bin(s, s.hist[0], remaining);
    prefix |= (unsigned)s.misc[0] << pass;
    mask |= 255u << pass;
    remaining = s.misc[1];
    __syncthreads();
  }
  return prefix;
}

// Gather every element with key >= thr into s.val / s.idx (ballot-compacted);
// returns the number found (may exceed kCand: only the first kCand are kept).
template <int U>
DRTC_DEVICE int gather_ge(SampShared& s, const unsigned short* lr, int V, bool vec, unsigned thr) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid == 0) s.misc[2] = 0;
  s.val[tid] = -INFINITY;
  s.idx[tid] = 0x7fffffff;
  __syncthreads();
  auto put = [&](bool pred, int i, unsigned short b) {
    const uint64_t m = __ballot(pred);
    if (m == 0) return;
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(&s.misc[2], __popcll(m));
    base = __shfl(base, leader, 64);
    if (pred) {
      const int slot = base + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      if (slot < kCand) { s.val[slot] = bits2f(b); s.idx[slot] = i; }
    }
  };
  // wave-uniform trip counts (the ballots need every lane): pad to whole waves
  const int w0 = tid & ~63;
  if (vec) {
    const int nv = V >> 3;
    for (int v0 = w0; v0 < nv; v0 += U * kSampThreads) {
      u16x8 x[U];
      bool any[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int v = v0 + u * kSampThreads + lane;
        x[u] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (v < nv) x[u] = *reinterpret_cast<const u16x8*>(lr + 8 * v);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int v = v0 + u * kSampThreads + lane;
        any[u] = false;
        if (v < nv) {
#pragma unroll
          for (int j = 0; j < 8; ++j) any[u] |= ord16(x[u][j]) >= thr;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (__ballot(any[u]) == 0) continue;  // wave-uniform
        const int v = v0 + u * kSampThreads + lane;
#pragma unroll
        for (int j = 0; j < 8; ++j) put(v < nv && ord16(x[u][j]) >= thr, 8 * v + j, x[u][j]);
      }
    }
    for (int i0 = (nv << 3) + w0; i0 < V; i0 += kSampThreads) {
      const int i = i0 + lane;
      const unsigned short b = i < V ? lr[i] : (unsigned short)0;
      put(i < V && ord16(b) >= thr, i, b);
    }
  } else {
    for (int i0 = w0; i0 < V; i0 += kSampThreads) {
      const int i = i0 + lane;
      const unsigned short b = i < V ? lr[i] : (unsigned short)0;
      put(i < V && ord16(b) >= thr, i, b);
    }
  }
  __syncthreads();
  return s.misc[2];
}

template <int U>
DRTC_DEVICE void sample_topk(SampShared& s, int* out_tokens, const unsigned short* lr, int V,
                             bool vec, int row, float temp, int k, float pp, uint64_t seed,
                             uint64_t st) {
  const int tid = threadIdx.x;
  // ---- pass 1: per-thread max key; tau0 = k-th largest of the thread maxima
  unsigned tm = 0;
  for_row<U>(lr, V, vec, [&](int, unsigned short b) { tm = max(tm, ord16(b)); });
  unsigned* h = &s.hist[0][0];
  h[tid] = tm;  // hist doubles as a 1024-key buffer here
  __syncthreads();
  // radix select over the 1024 thread maxima (LDS only)
  unsigned prefix = 0, mask = 0;
  int remaining = k;
  for (int pass = 8; pass >= 0; pass -= 8) {
    unsigned* bins = &s.hist[4][0];  // bins after the 1024-key buffer (hist[0..3])
    if (tid < 256) bins[tid] = 0;
    __syncthreads();
    const unsigned key = h[tid];
    if ((key & mask) == prefix) atomicAdd(&bins[(key >> pass) & 255u], 1u);
    __syncthreads();
    select_bin(s, bins, remaining);
    prefix |= (unsigned)s.misc[0] << pass;
    mask |= 255u << pass;
    remaining = s.misc[1];
    __syncthreads();
  }
  // ---- gather key >= tau0 (>= k elements by construction).  Such an element
  // can only sit in a thread whose own max is >= tau0, so only those threads
  // (about k of the 1024) re-read their own elements: no second row pass.
  if (tid == 0) s.misc[2] = 0;
  s.val[tid] = -INFINITY;
  s.idx[tid] = 0x7fffffff;
  __syncthreads();
  if (tm >= prefix) {
    for_row<U>(lr, V, vec, [&](int i, unsigned short b) {
      if (ord16(b) >= prefix) {
        const int slot = atomicAdd(&s.misc[2], 1);
        if (slot < kCand) { s.val[slot] = bits2f(b); s.idx[slot] = i; }
      }
    });
  }
  __syncthreads();
  int n = s.misc[2];
  if (n > kCand) {  // heavy ties: exact k-th key by radix select, gather again
    const unsigned thr = radix_kth<U>(s, lr, V, vec, k);
    n = min(gather_ge<U>(s, lr, V, vec, thr), kCand);
  }
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  // ---- bitonic sort, descending (ties -> lower index first)
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int j = tid ^ stride;
      if (tid < np2 && j > tid) {
        const bool desc = ((tid & size) == 0);
        const float a = s.val[tid], b = s.val[j];
        const int ia = s.idx[tid], ib = s.idx[j];
        const bool a_first = (a > b) || (a == b && ia < ib);
        if (desc != a_first) {
          s.val[tid] = b; s.val[j] = a;
          s.idx[tid] = ib; s.idx[j] = ia;
        }
      }
      __syncthreads();
    }
  }
  // keep exactly the elements >= the k-th value (ties with it included)
  const float kth = s.val[min(k, n) - 1];
  {
    const bool edge = tid < n && s.val[tid] >= kth && (tid + 1 == n || s.val[tid + 1] < kth);
    if (edge) s.misc[3] = tid + 1;
  }
  __syncthreads();
  n = s.misc[3];
  np2 = 1;
  while (np2 < n) np2 <<= 1;
  // ---- softmax + top-p + draw over the n candidates
  const float top = s.val[0];
  const float inv_t = 1.f / temp;
  const float pv = (tid < n) ? __expf((s.val[tid] - top) * inv_t) : 0.f;
  __syncthreads();
  s.val[tid] = pv;
  __syncthreads();
  for (int off = 1; off < np2; off <<= 1) {  // inclusive Hillis-Steele scan
    const float add = (tid >= off && tid < np2) ? s.val[tid - off] : 0.f;
    __syncthreads();
    s.val[tid] += add;
    __syncthreads();
  }
  const float total = s.val[n - 1];
  if (tid == 0) s.misc[3] = n - 1;
  __syncthreads();
  {
    const float need = pp * total;
    const bool hit = tid < n && s.val[tid] >= need && (tid == 0 || s.val[tid - 1] < need);
    if (hit) s.misc[3] = tid;
  }
  __syncthreads();
  const int cut = s.misc[3];
  const float target = uniform(seed, st, row, 0) * s.val[cut];
  if (tid <= cut) {
    const float lo = (tid == 0) ? 0.f : s.val[tid - 1];
    if (target >= lo && (target < s.val[tid] || tid == cut)) out_tokens[row] = s.idx[tid];
  }
}

template <int U>
DRTC_DEVICE void sample_topp_full(SampShared& s, int* out_tokens, const unsigned short* lr, int V,
                                  bool vec, int row, float temp, float pp, uint64_t seed,
                                  uint64_t st) {
  const int tid = threadIdx.x;
  const float inv_t = 1.f / temp;
  // ---- pass 1: row max and per-thread softmax mass (online, 8 at a time)
  float m_t = -INFINITY, s_t = 0.f;
  for_row<U>(lr, V, vec, [&](int, unsigned short b) {
    const float x = bits2f(b);
    if (!(x > -INFINITY)) return;  // -inf (masked) or NaN: zero mass
    if (x > m_t) {
      s_t = s_t * __expf((m_t - x) * inv_t) + 1.f;
      m_t = x;
    } else {
      s_t += __expf((x - m_t) * inv_t);
    }
  });
  const int lane = tid & 63, wid = tid >> 6;
  float wm = wave_max(m_t);
  if (lane == 0) s.wred[0][wid] = wm;
  __syncthreads();
  float m = -INFINITY;
#pragma unroll
  for (int w = 0; w < kSampWaves; ++w) m = fmaxf(m, s.wred[0][w]);
  __syncthreads();
  float e = (s_t > 0.f) ? s_t * __expf((m_t - m) * inv_t) : 0.f;  // eligible mass, this thread
  float Z, dummy;
  block_sum2(s, e, 0.f, Z, dummy);
  const float P = pp * Z;
  unsigned L = 0;                                     // eligible: key > L (0 = every finite key)
  unsigned H = ord16(__float_as_uint(m) >> 16);       // keys >= H are inside the nucleus
  bool l_open = true;                                 // L not yet set: everything eligible
  for (int round = 0; round < kMaxRounds; ++round) {
    // ---- draw j from the eligible set
    float E;
    int last_pos;
    if (tid == 0) s.misc[0] = -1;
    const float excl = block_excl_scan(s, e, E, last_pos);  // (barriers inside)
    const float target = uniform(seed, st, row, round) * E;
    // the owning thread re-walks its own elements in the pass order
    auto walk = [&](float tgt) {
      float acc = excl;
      int pick = -1, last = -1;
      unsigned pk = 0, lk = 0;
      for_row<U>(lr, V, vec, [&](int i, unsigned short b) {
        const unsigned key = ord16(b);
        const float x = bits2f(b);
        if (pick < 0 && (l_open || key > L) && x > -INFINITY) {
          acc += __expf((x - m) * inv_t);
          last = i; lk = key;
          if (acc > tgt) { pick = i; pk = key; }
        }
      });
      if (pick < 0) { pick = last; pk = lk; }
      s.misc[0] = pick;
      s.misc[1] = (int)pk;
    };
    if (e > 0.f && target >= excl && target < excl + e) walk(target);
    __syncthreads();
    if (s.misc[0] < 0 && tid == last_pos) walk(INFINITY);  // rounding at the scan edges
    __syncthreads();
    const int j = s.misc[0];
    const unsigned kj = (unsigned)s.misc[1];
    __syncthreads();
    if (pp >= 1.f || kj >= H || round == kMaxRounds - 1) {
      if (tid == 0) out_tokens[row] = j;
      return;
    }
    // ---- verify: mass above key_j, plus the bisection key between L and H
    const unsigned lo = l_open ? 0u : L;
    const unsigned t = lo + ((H - lo) >> 1);
    const bool bis = t > lo && t < H && t != kj;
    float a_t = 0.f, f_t = 0.f;
    for_row<U>(lr, V, vec, [&](int, unsigned short b) {
      const unsigned key = ord16(b);
      const float w = __expf((bits2f(b) - m) * inv_t);
      a_t += key > kj ? w : 0.f;
      f_t += key > t ? w : 0.f;
    });
    float A, F;
    block_sum2(s, a_t, f_t, A, F);
    if (A < P) {  // token j is inside the nucleus
      if (tid == 0) out_tokens[row] = j;
      return;
    }
    // key_j and everything below it is outside
    L = kj; l_open = false; e = a_t;
    if (bis) {
      if (F >= P) {
        if (t > L) { L = t; e = f_t; }
      } else {
        H = min(H, t);
      }
    }
  }
}

// OCC = 1: one 1024-thread workgroup per CU (91 VGPRs, 4-deep load unroll); OCC = 2: two
// (<= 64 VGPRs, 2-deep unroll), so one row's selection tail (scans, block reductions,
// barriers) overlaps another row's stream on the same CU.
template <int OCC>
__global__ __launch_bounds__(kSampThreads, 4 * OCC) void sample_kernel(
    int* __restrict__ out_tokens, const bf16_t* __restrict__ logits, int V,
    int ld, const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, uint64_t seed,
    const int64_t* __restrict__ step) {
  constexpr int U = OCC == 1 ? kUnroll : 2;
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const unsigned short* lr = (const unsigned short*)(logits + (int64_t)row * ld);
  const bool vec = ((reinterpret_cast<uintptr_t>(lr) & 15) == 0);
  const float temp = temperature ? temperature[row] : 0.f;
  __shared__ SampShared s;

  if (temp <= 0.f) {  // ---------------------------------- greedy argmax
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for_row<U>(lr, V, vec, [&](int i, unsigned short b) {
      const float v = bits2f(b);
      if (v > best || (v == best && i < bi)) { best = v; bi = i; }
    });
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (lane == 0) { s.val[wid] = best; s.idx[wid] = bi; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < kSampWaves; ++w)
        if (s.val[w] > best || (s.val[w] == best && s.idx[w] < bi)) { best = s.val[w]; bi = s.idx[w]; }
      out_tokens[row] = bi;
    }
    return;
  }
  const uint64_t st = step ? (uint64_t)step[0] : 0ull;
  const float pp = (top_p && top_p[row] > 0.f && top_p[row] < 1.f) ? top_p[row] : 1.f;
  int k = top_k ? top_k[row] : 0;
  if (k >= V) k = 0;
  if (k > 0) {
    sample_topk<U>(s, out_tokens, lr, V, vec, row, temp, min(k, kCand), pp, seed, st);
  } else {
    sample_topp_full<U>(s, out_tokens, lr, V, vec, row, temp, pp, seed, st);
  }
}

int launch_sample(int* out_tokens, const void* logits, int B, int V, int ld,
                  const float* temperature, const int* top_k, const float* top_p,
                  uint64_t seed, const int64_t* step, hipStream_t st) {
  if (B == 0) return 0;
  // two workgroups per CU by default: B = 1024, V = 128k, top-k 64 / top-p 0.95 in 76.5 vs
  // 106.0 us, greedy 44.8 vs 58.1, full-vocabulary top-p 179 vs 237 (profiles/r3v);
  // DRTC_SAMPLER_OCC=1 restores one per CU
  static const int occ = [] {
    const char* e = getenv("DRTC_SAMPLER_OCC");
    return e && e[0] == '1' ? 1 : 2;
  }();
  if (occ == 2)
    hipLaunchKernelGGL(sample_kernel<2>, dim3(B), dim3(kSampThreads), 0, st, out_tokens,
                       (const bf16_t*)logits, V, ld, temperature, top_k, top_p, seed, step);
  else
    hipLaunchKernelGGL(sample_kernel<1>, dim3(B), dim3(kSampThreads), 0, st, out_tokens,
                       (const bf16_t*)logits, V, ld, temperature, top_k, top_p, seed, step);
  return (int)hipGetLastError();
}

}  // namespace drtc
