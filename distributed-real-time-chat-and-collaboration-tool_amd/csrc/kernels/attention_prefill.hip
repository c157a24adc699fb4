// Varlen causal flash-attention forward on MFMA (gfx950), GQA/MQA-aware.
//
// Inputs are read straight out of the fused QKV GEMM output (after the
// in-place RoPE kernel), so no Q/K/V copies are made: sequence s occupies
// rows cu_seqlens[s] .. cu_seqlens[s+1] of the packed [T, qkv_stride] buffer.
//
// Work decomposition: grid = (n_q_tiles, Hq / GH); a workgroup owns a
// 64-row query tile of GH query heads sharing one KV head (details below).
// Measured on MI355X (scripts/prefill_attn_bench.py, vs the previous
// one-head-per-workgroup kernel with synchronous staging and a scattered
// V^T LDS image): Llama-3-8B smart-reply batch (1024 x ~148 tokens)
// 1.67 -> 1.13 ms, summarize batch (512 x ~432) 3.62 -> 2.09 ms,
// 16 x 4096 tokens 7.0 -> 3.3 ms (708 TFLOP/s), Gemma-2B 1.12 -> 0.61 ms.
//
// MFMA formulation (16x16x32 bf16): the scores are computed transposed,
//   S^T[key, q] = K[key, :] . Q[q, :]   (A = K from LDS, B = Q^T in registers)
// so that the accumulator tiles of two 16-key halves become the P^T
// B-operand of O^T[d, q] += V^T[d, key] . P^T[key, q] without any lane
// movement (same token permutation trick as the decode kernel).  The online
// softmax per query column needs only two cross-lane xor-shuffles.
#include "common.h"
#include "launchers.h"

namespace drtc {

constexpr int kQT = 64;   // query rows per workgroup
constexpr int kKT = 64;   // keys per LDS tile

// One workgroup = one 64-row query tile x GH query heads that share a KV head
// (4 waves per head, 16 rows per wave): each K/V tile is fetched from HBM and
// staged in LDS ONCE for the GH heads instead of once per head.  Staging is
// split issue-early / write-late (the next tile's global loads are in flight
// during this tile's MFMAs; double-buffered LDS, one barrier per tile).  V is
// staged row-major exactly as loaded (16-B ds_write) and read as the P.V
// A-operand with ds_read_b64_tr_b16 (CDNA4 hardware transpose: lanes 4q+p of a
// 16-lane group address row q / columns 4p..4p+3, lane i receives column i).
// Row paddings: K rows D+8 (conflict-free ds_read_b128), V rows D+16 (the 8
// rows of one tr-read half land on distinct bank octets).
template <int D, int GH>
struct PrefillLds {
  static constexpr int KROW = D + 8;
  static constexpr int VROW = D + 16;
  static constexpr int K_ELEMS = kKT * KROW;
  static constexpr int V_ELEMS = kKT * VROW;
  static constexpr int BUF = K_ELEMS + V_ELEMS;  // one stage
  static constexpr size_t BYTES = (size_t)2 * BUF * 2;
};

typedef short s16x4 __attribute__((ext_vector_type(4)));

DRTC_DEVICE bf16x4 lds_read_tr16(const bf16_t* p) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

template <int D, int GH>
__global__ __launch_bounds__(256 * GH) void prefill_attn_kernel(
    bf16_t* __restrict__ out, int out_stride, const bf16_t* __restrict__ qkv,
    int qkv_stride, int Hq, int Hkv, const int* __restrict__ cu_seqlens,
    const int* __restrict__ tile_seq, const int* __restrict__ tile_q0,
    float scale_log2e, int causal) {
  using L = PrefillLds<D, GH>;
  constexpr int NTHR = 256 * GH;
  constexpr int KS = D / 32;
  constexpr int NT = D / 16;
  constexpr int VPR = D / 8;                 // 16-B vectors per K/V row
  constexpr int NV = kKT * VPR / NTHR;       // vectors per thread per operand
  static_assert(NV >= 1 && (kKT * VPR) % NTHR == 0, "staging split");
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];

  const int tile = blockIdx.x;
  const int G = Hq / Hkv;
  const int groups = G / GH;
  const int hk = blockIdx.y / groups;
  const int hq0 = hk * G + (blockIdx.y - hk * groups) * GH;
  const int w = wave_id_uniform();
  const int hq = hq0 + (w >> 2);
  const int seq = tile_seq[tile];
  const int q0 = tile_q0[tile];
  const int s_begin = cu_seqlens[seq];
  const int seqlen = cu_seqlens[seq + 1] - s_begin;
  const int lane = threadIdx.x & 63;
  const int col = lane & 15, g = lane >> 4;
  const int qrow = q0 + 16 * (w & 3) + col;
  const int k_off = (Hq + hk) * D;
  const int v_off = (Hq + Hkv + hk) * D;
  const int kv_end = causal ? min(seqlen, q0 + kQT) : seqlen;
  const int ntiles = (kv_end + kKT - 1) / kKT;

  bf16x8 kr[NV], vr[NV];
  auto issue = [&](int k0) {
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      const int v = threadIdx.x + n * NTHR;
      const int key = v / VPR;
      const int c = (v - key * VPR) * 8;
      if (k0 + key < seqlen) {
        const bf16_t* rp = qkv + (int64_t)(s_begin + k0 + key) * qkv_stride;
        kr[n] = load_bf16x8(rp + k_off + c);
        vr[n] = load_bf16x8(rp + v_off + c);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { kr[n][j] = f2bf(0.f); vr[n][j] = f2bf(0.f); }
      }
    }
  };
  auto commit = [&](bf16_t* kb) {
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      const int v = threadIdx.x + n * NTHR;
      const int key = v / VPR;
      const int c = (v - key * VPR) * 8;
      store_bf16x8(kb + key * L::KROW + c, kr[n]);
      store_bf16x8(kb + L::K_ELEMS + key * L::VROW + c, vr[n]);
    }
  };

  issue(0);
  bf16x8 qf[KS];
  {
    const bf16_t* qp = qkv + (int64_t)(s_begin + qrow) * qkv_stride + hq * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (qrow < seqlen) qf[s] = load_bf16x8(qp + 32 * s + 8 * g);
      else for (int j = 0; j < 8; ++j) qf[s][j] = f2bf(0.f);
    }
  }
  f32x4 o[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) o[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = kNegBig, lsum = 0.f;
  // tr-read lane address within a 16-lane group: row q = (lane&15)>>2, cols 4p
  const int tr_off = ((col >> 2) + 4 * g) * L::VROW + 4 * (col & 3);

  for (int kt = 0; kt < ntiles; ++kt) {
    bf16_t* kb = lds + (kt & 1) * L::BUF;
    const bf16_t* vb = kb + L::K_ELEMS;
    commit(kb);
    __syncthreads();
    if (kt + 1 < ntiles) issue((kt + 1) * kKT);
    const int k0 = kt * kKT;

    f32x4 sc[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      sc[st] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8 a = load_bf16x8(kb + (16 * st + col) * L::KROW + 32 * s + 8 * g);
        sc[st] = mfma16(a, qf[s], sc[st]);
      }
    }
    float bmax = kNegBig;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 16 * st + 4 * g + r;
        const bool ok = key < seqlen && (!causal || key <= qrow);
        sc[st][r] = ok ? sc[st][r] * scale_log2e : kNegBig;
        bmax = fmaxf(bmax, sc[st][r]);
      }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
    const float m_new = fmaxf(m, bmax);
    const float alpha = fast_exp2(m - m_new);
    m = m_new;
    bf16x8 pf[2];
    float psum = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pa = fast_exp2(sc[2 * ks][r] - m_new);
        const float pb = fast_exp2(sc[2 * ks + 1][r] - m_new);
        psum += pa + pb;
        pf[ks][r] = f2bf(pa);
        pf[ks][4 + r] = f2bf(pb);
      }
    lsum = lsum * alpha + psum;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      o[i] *= alpha;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x4 lo = lds_read_tr16(vb + tr_off + 32 * ks * L::VROW + 16 * i);
        const bf16x4 hi = lds_read_tr16(vb + tr_off + (32 * ks + 16) * L::VROW + 16 * i);
        bf16x8 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) { a[j] = lo[j]; a[4 + j] = hi[j]; }
        o[i] = mfma16(a, pf[ks], o[i]);
      }
    }
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (qrow < seqlen) {
    const float inv = 1.f / lsum;
    bf16_t* op = out + (int64_t)(s_begin + qrow) * out_stride + hq * D + 4 * g;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      bf16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(o[i][r] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * i) = v;
    }
  }
}

// Persistent variant: resident workgroups loop over the work items (query
// tile, head group), tile-major in the longest-first order of prefill_tiles,
// one item per round of gridDim.x items in snake order.  Chat
// prompts give ~24k items of 1-3 K/V tiles each: with one 1024-thread
// workgroup resident per CU, the non-persistent kernel spends most of its
// time launching and draining workgroups (r1j PMC: waves alive ~20 % of the
// kernel).  Here the waves stay resident; the next item's first K/V tile and
// its Q fragments are loaded while the current item's last tile is computed,
// and the LDS double buffer keeps alternating across items (the barrier of
// each step orders the reuse exactly as inside one item).  Per-tile math is
// identical to prefill_attn_kernel.
template <int D, int GH>
__global__ __launch_bounds__(256 * GH) void prefill_attn_persist_kernel(
    bf16_t* __restrict__ out, int out_stride, const bf16_t* __restrict__ qkv,
    int qkv_stride, int Hq, int Hkv, const int* __restrict__ cu_seqlens,
    const int* __restrict__ tile_seq, const int* __restrict__ tile_q0, int n_tiles,
    float scale_log2e, int causal) {
  using L = PrefillLds<D, GH>;
  constexpr int NTHR = 256 * GH;
  constexpr int KS = D / 32;
  constexpr int NT = D / 16;
  constexpr int VPR = D / 8;
  constexpr int NV = kKT * VPR / NTHR;
  static_assert(NV >= 1 && (kKT * VPR) % NTHR == 0, "staging split");
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];

  const int G = Hq / Hkv;
  const int groups = G / GH;
  const int n_hg = Hq / GH;
  const int n_work = n_tiles * n_hg;
  const int w = wave_id_uniform();
  const int lane = threadIdx.x & 63;
  const int col = lane & 15, g = lane >> 4;

  struct Item {
    int item, s_begin, seqlen, q0, hq, hk, ntiles;
  };
  auto info = [&](int item) -> Item {
    const int tile = item / n_hg;
    const int hg = item - tile * n_hg;
    const int hk = hg / groups;
    const int hq = hk * G + (hg - hk * groups) * GH + (w >> 2);
    const int seq = tile_seq[tile];
    const int q0 = tile_q0[tile];
    const int s_begin = cu_seqlens[seq];
    const int seqlen = cu_seqlens[seq + 1] - s_begin;
    const int kv_end = causal ? min(seqlen, q0 + kQT) : seqlen;
    return Item{item, s_begin, seqlen, q0, hq, hk, (kv_end + kKT - 1) / kKT};
  };
  bf16x8 kr[NV], vr[NV];
  auto issue = [&](const Item& it, int k0) {
    const int k_off = (Hq + it.hk) * D;
    const int v_off = (Hq + Hkv + it.hk) * D;
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      const int v = threadIdx.x + n * NTHR;
      const int key = v / VPR;
      const int c = (v - key * VPR) * 8;
      if (k0 + key < it.seqlen) {
        const bf16_t* rp = qkv + (int64_t)(it.s_begin + k0 + key) * qkv_stride;
        kr[n] = load_bf16x8(rp + k_off + c);
        vr[n] = load_bf16x8(rp + v_off + c);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { kr[n][j] = f2bf(0.f); vr[n][j] = f2bf(0.f); }
      }
    }
  };
  auto commit = [&](bf16_t* kb) {
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      const int v = threadIdx.x + n * NTHR;
      const int key = v / VPR;
      const int c = (v - key * VPR) * 8;
      store_bf16x8(kb + key * L::KROW + c, kr[n]);
      store_bf16x8(kb + L::K_ELEMS + key * L::VROW + c, vr[n]);
    }
  };
  auto load_q = [&](bf16x8* qf, const Item& it) {
    const int qrow = it.q0 + 16 * (w & 3) + col;
    const bf16_t* qp = qkv + (int64_t)(it.s_begin + qrow) * qkv_stride + it.hq * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (qrow < it.seqlen) qf[s] = load_bf16x8(qp + 32 * s + 8 * g);
      else for (int j = 0; j < 8; ++j) qf[s][j] = f2bf(0.f);
    }
  };
  const int tr_off = ((col >> 2) + 4 * g) * L::VROW + 4 * (col & 3);

  // Items are sorted longest-first; a workgroup takes one item per round of
  // gridDim.x items, in snake order (round r even: slot blockIdx.x, odd: the
  // mirrored slot), so every workgroup gets a balanced mix of long and short
  // items instead of the longest of every round.
  const int nwg = gridDim.x;
  auto item_of = [&](int round) -> int {
    const int slot = (round & 1) ? nwg - 1 - (int)blockIdx.x : (int)blockIdx.x;
    return round * nwg + slot;
  };
  int round = 0;
  if (item_of(0) >= n_work) return;
  Item cur = info(item_of(0));
  issue(cur, 0);
  bf16x8 qf[KS], qn[KS];
  load_q(qf, cur);
  int buf = 0;
  while (true) {
    const int qrow = cur.q0 + 16 * (w & 3) + col;
    f32x4 o[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) o[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float m = kNegBig, lsum = 0.f;
    const int nxt_item = item_of(round + 1);
    const bool have_next = nxt_item < n_work;
    Item nxt = cur;
    for (int kt = 0; kt < cur.ntiles; ++kt) {
      bf16_t* kb = lds + buf * L::BUF;
      const bf16_t* vb = kb + L::K_ELEMS;
      buf ^= 1;
      commit(kb);
      __syncthreads();
      if (kt + 1 < cur.ntiles) {
        issue(cur, (kt + 1) * kKT);
      } else if (have_next) {
        nxt = info(nxt_item);
        issue(nxt, 0);
        load_q(qn, nxt);
      }
      const int k0 = kt * kKT;
      f32x4 sc[4];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        sc[st] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          bf16x8 a = load_bf16x8(kb + (16 * st + col) * L::KROW + 32 * s + 8 * g);
          sc[st] = mfma16(a, qf[s], sc[st]);
        }
      }
      float bmax = kNegBig;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 16 * st + 4 * g + r;
          const bool ok = key < cur.seqlen && (!causal || key <= qrow);
          sc[st][r] = ok ? sc[st][r] * scale_log2e : kNegBig;
          bmax = fmaxf(bmax, sc[st][r]);
        }
      bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
      bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
      const float m_new = fmaxf(m, bmax);
      const float alpha = fast_exp2(m - m_new);
      m = m_new;
      bf16x8 pf[2];
      float psum = 0.f;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pa = fast_exp2(sc[2 * ks][r] - m_new);
          const float pb = fast_exp2(sc[2 * ks + 1][r] - m_new);
          psum += pa + pb;
          pf[ks][r] = f2bf(pa);
          pf[ks][4 + r] = f2bf(pb);
        }
      lsum = lsum * alpha + psum;
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        o[i] *= alpha;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x4 lo = lds_read_tr16(vb + tr_off + 32 * ks * L::VROW + 16 * i);
          const bf16x4 hi = lds_read_tr16(vb + tr_off + (32 * ks + 16) * L::VROW + 16 * i);
          bf16x8 a;
#pragma unroll
          for (int j = 0; j < 4; ++j) { a[j] = lo[j]; a[4 + j] = hi[j]; }
          o[i] = mfma16(a, pf[ks], o[i]);
        }
      }
    }
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    if (qrow < cur.seqlen) {
      const float inv = 1.f / lsum;
      bf16_t* op = out + (int64_t)(cur.s_begin + qrow) * out_stride + cur.hq * D + 4 * g;
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = f2bf(o[i][r] * inv);
        *reinterpret_cast<bf16x4*>(op + 16 * i) = v;
      }
    }
    if (!have_next) break;
    cur = nxt;
    ++round;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = qn[s];
  }
}

static int prefill_persist_grid(int n_work) {
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cu <= 0)
      n_cu = 256;
  }
  return std::max(1, std::min(n_work, n_cu));
}

template <int D, int GH>
static void launch_tile(dim3 grid, hipStream_t st, bf16_t* out, int out_stride, const bf16_t* qkv,
                      int qkv_stride, int Hq, int Hkv, const int* cu, const int* ts,
                      const int* tq, float sl2, int causal, int persist) {
  constexpr size_t lds_bytes = PrefillLds<D, GH>::BYTES;
  if (persist) {
    // resident workgroups per CU for this instantiation (VGPRs / LDS / waves)
    static int per_cu = 0;
    if (per_cu == 0) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
              &per_cu, prefill_attn_persist_kernel<D, GH>, 256 * GH, lds_bytes) != hipSuccess ||
          per_cu <= 0)
        per_cu = 1;
    }
    const int n_work = (int)(grid.x * grid.y);
    const int n_wg = std::min(n_work, prefill_persist_grid(n_work * per_cu) * per_cu);
    prefill_attn_persist_kernel<D, GH><<<dim3(std::max(1, n_wg)), dim3(256 * GH),
                                          lds_bytes, st>>>(
        out, out_stride, qkv, qkv_stride, Hq, Hkv, cu, ts, tq, (int)grid.x, sl2, causal);
    return;
  }
  prefill_attn_kernel<D, GH><<<grid, dim3(256 * GH), lds_bytes, st>>>(
      out, out_stride, qkv, qkv_stride, Hq, Hkv, cu, ts, tq, sl2, causal);
}


template <int D>
static int launch_gh(int GH, int ntiles, int Hq, int Hkv, hipStream_t st, bf16_t* out,
                        int out_stride, const bf16_t* qkv, int qkv_stride, const int* cu,
                        const int* ts, const int* tq, float sl2, int causal, int persist) {
  dim3 grid(ntiles, Hq / GH);
  switch (GH) {
    case 1: launch_tile<D, 1>(grid, st, out, out_stride, qkv, qkv_stride, Hq, Hkv, cu, ts, tq, sl2, causal, persist); break;
    case 2: launch_tile<D, 2>(grid, st, out, out_stride, qkv, qkv_stride, Hq, Hkv, cu, ts, tq, sl2, causal, persist); break;
    case 4:
      if constexpr (D == 128) {
        launch_tile<D, 4>(grid, st, out, out_stride, qkv, qkv_stride, Hq, Hkv, cu, ts, tq, sl2, causal, persist);
        break;
      }
      return -1;
    default: return -1;
  }
  return 0;
}

int launch_prefill_attn(void* out, int out_stride, const void* qkv,
                        int qkv_stride, int Hq, int Hkv, int D,
                        const int* cu_seqlens, const int* tile_seq,
                        const int* tile_q0, int ntiles, float scale, int causal,
                        int persist, hipStream_t st) {
  if (ntiles == 0) return 0;
  if (Hkv <= 0 || Hq % Hkv != 0) return -1;
  const float sl2 = scale * kLog2e;
  const int G = Hq / Hkv;
  // heads per workgroup: 4 for D=128 (1024 threads), 2 for D=64 (one
  // 16-B K and V vector per thread) and D=256 (VGPR budget)
  const int gh_max = D == 128 ? 4 : 2;
  const int GH = gh_max <= G ? gh_max : (G >= 2 ? 2 : 1);
  if (G % GH != 0) return -1;
  const bf16_t* q = (const bf16_t*)qkv;
  bf16_t* o = (bf16_t*)out;
  int rc;
  switch (D) {
    case 64: rc = launch_gh<64>(GH, ntiles, Hq, Hkv, st, o, out_stride, q, qkv_stride, cu_seqlens, tile_seq, tile_q0, sl2, causal, persist); break;
    case 128: rc = launch_gh<128>(GH, ntiles, Hq, Hkv, st, o, out_stride, q, qkv_stride, cu_seqlens, tile_seq, tile_q0, sl2, causal, persist); break;
    case 256: rc = launch_gh<256>(GH, ntiles, Hq, Hkv, st, o, out_stride, q, qkv_stride, cu_seqlens, tile_seq, tile_q0, sl2, causal, persist); break;
    default: return -1;
  }
  if (rc) return rc;
  return (int)hipGetLastError();
}

template <int D, int GH>
static int set_lds() {
  int e = (int)hipFuncSetAttribute((const void*)prefill_attn_kernel<D, GH>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)PrefillLds<D, GH>::BYTES);
  if (!e)
    e = (int)hipFuncSetAttribute((const void*)prefill_attn_persist_kernel<D, GH>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)PrefillLds<D, GH>::BYTES);
  return e;
}

int configure_prefill() {
  int e = set_lds<64, 1>();
  if (!e) e = set_lds<64, 2>();
  if (!e) e = set_lds<128, 1>();
  if (!e) e = set_lds<128, 2>();
  if (!e) e = set_lds<128, 4>();
  if (!e) e = set_lds<256, 1>();
  if (!e) e = set_lds<256, 2>();
  return e;
}

}  // namespace drtc
