// Paged decode attention on MFMA (gfx950): one query token per sequence
// against a paged KV cache, GQA/MQA-aware.
//
// Work decomposition
//   grid = (B * Hkv, max_partitions); one 256-thread workgroup (4 waves) per
//   (sequence, kv head, context partition).  All G = Hq/Hkv query heads that
//   share a kv head are processed together, so every K/V byte is read from
//   HBM once per step.  Waves take the partition's 32-token cache blocks
//   round-robin, keep an online softmax each, and merge through LDS; when a
//   sequence spans several partitions the fp32 partials are merged
//   (flash-decoding split-K) by the last partition workgroup to finish
//   (agent-scope counter per (sequence, kv head)), or by
//   `decode_reduce_kernel` when no counter buffer is given.
//
// MFMA formulation (16x16x32 bf16, operand maps in common.h)
//   S^T[tok, head] = K[tok, :] . Q[head, :]    A = K rows (16-B loads straight
//                                             from the token-major K block),
//                                             B = Q^T (registers, whole step)
//   O^T[d, head]  += V^T[d, tok] . P^T[tok, head]
//   The S^T accumulators of the two 16-token halves of a block are fed back
//   as the P^T B-operand with NO lane movement: lane l (g = l>>4) holds tokens
//   {4g..4g+3} and {16+4g..16+4g+3}; the V^T A-operand is loaded with the
//   same token permutation from the V block, stored as 8 groups of 4 tokens,
//   dim-major inside a group (two 8-B loads, 128-B coalesced per d-tile).
//   Columns are query heads: G <= 16 (Llama-3 4, 70B 8, Gemma-2B 8).
#include "common.h"
#include "launchers.h"

typedef __attribute__((address_space(3))) void* ad_lds_ptr;

namespace {
// s_waitcnt vmcnt(0): every vector-memory load of this wave has landed.  Used right after the
// first K/V block of a register double-buffered block loop is issued (see the persistent
// kernel): without it the waitcnt pass merges the loop's entry edge (that block still in
// flight) with the iterations that issue no next-block loads and guards the block's first
// QK MFMA with vmcnt(0) / a small vmcnt(n) on EVERY iteration - which waits for the next
// block's loads as well, so no block ever streams while another is computed.
__device__ __forceinline__ void vm_wait_all() {
  __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
}
}  // namespace

namespace drtc {

constexpr int kBS = 32;  // tokens per KV-cache block (fixed by the layout)

template <int D>
struct KVRegs {
  bf16x8 k0[D / 32], k1[D / 32];  // tokens 0..15 / 16..31 of the block
  bf16x4 vlo[D / 16], vhi[D / 16];
};

template <int D>
DRTC_DEVICE void load_kv_block(KVRegs<D>& r, const bf16_t* kb, const bf16_t* vb,
                               int lane) {
  const int t = lane & 15, g = lane >> 4;
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    r.k0[s] = load_bf16x8(kb + t * D + 32 * s + 8 * g);
    r.k1[s] = load_bf16x8(kb + (16 + t) * D + 32 * s + 8 * g);
  }
  // V block = 8 groups of 4 tokens, each group dim-major [D][4] (kv_cache.py):
  // tokens 4g..4g+3 of row d are 8 contiguous bytes, and the 16 rows of one
  // d-tile are 128 contiguous bytes.
#pragma unroll
  for (int i = 0; i < D / 16; ++i) {
    r.vlo[i] = load_bf16x4(vb + g * (4 * D) + (16 * i + t) * 4);
    r.vhi[i] = load_bf16x4(vb + (4 + g) * (4 * D) + (16 * i + t) * 4);
  }
}

template <int D>
__global__ __launch_bounds__(256, D >= 256 ? 1 : 2) void paged_decode_kernel(
    bf16_t* __restrict__ out, float* __restrict__ part_o,
    float* __restrict__ part_ml, int* __restrict__ counters, const bf16_t* __restrict__ q,
    int q_stride, const bf16_t* __restrict__ k_cache, const bf16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ context_lens, int Hq, int Hkv, float scale_log2e,
    int max_parts, int blocks_per_part) {
  constexpr int NT = D / 16;  // output d-tiles
  constexpr int KS = D / 32;  // k-steps of the QK product
  const int b = blockIdx.x / Hkv;
  const int h = blockIdx.x - b * Hkv;
  const int p = blockIdx.y;
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63;
  const int w = wave_id_uniform();
  const int col = lane & 15, g = lane >> 4;
  const int blk_begin = p * blocks_per_part;
  // Issue every load that does not depend on the context length first: the
  // block-table entries of this wave's first two blocks (clamped into the
  // row: speculative, used only if the blocks exist) and Q.  The critical
  // path becomes max(ctx, table) -> K/V instead of ctx -> table -> K/V.
  const int* bt = block_tables + (int64_t)b * bt_stride;
  const int ph_a = bt[min(blk_begin + w, bt_stride - 1)];
  const int ph_b = bt[min(blk_begin + w + 4, bt_stride - 1)];
  bf16x8 qf[KS];  // Q^T B-operand fragments (zero for padding columns col >= G)
  const bf16_t* qrow = q + (int64_t)b * q_stride + (int64_t)(h * G + col) * D;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (col < G) qf[s] = load_bf16x8(qrow + 32 * s + 8 * g);
    else for (int j = 0; j < 8; ++j) qf[s][j] = f2bf(0.f);
  }
  const int ctx = context_lens[b];
  const int nblk = (ctx + kBS - 1) / kBS;
  const int nparts = (nblk + blocks_per_part - 1) / blocks_per_part;

  if (ctx <= 0) {  // padded batch slot: deterministic zeros, no cache reads
    if (p == 0)
      for (int i = threadIdx.x; i < G * D; i += 256)
        out[(int64_t)b * Hq * D + (int64_t)h * G * D + i] = f2bf(0.f);
    return;
  }
  if (p >= nparts) return;

  const int blk_end = min(nblk, blk_begin + blocks_per_part);

  f32x4 o[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) o[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = kNegBig, lsum = 0.f;

  const int64_t blk_elems = (int64_t)kBS * D;
  KVRegs<D> cur, nxt;
  int blk = blk_begin + w;
  int ph_next = ph_b;  // table entry of block blk + 4, loaded one step ahead
  if (blk < blk_end) {
    const int64_t phys = ph_a;
    load_kv_block<D>(cur, k_cache + (phys * Hkv + h) * blk_elems,
                     v_cache + (phys * Hkv + h) * blk_elems, lane);
  }
  vm_wait_all();  // the first block lands before the loop (vm_wait_all)
  for (; blk < blk_end; blk += 4) {
    const int nb = blk + 4;
    if (nb < blk_end) {  // register double-buffer: next block in flight
      const int64_t phys = ph_next;
      load_kv_block<D>(nxt, k_cache + (phys * Hkv + h) * blk_elems,
                       v_cache + (phys * Hkv + h) * blk_elems, lane);
      ph_next = bt[min(nb + 4, bt_stride - 1)];
    }
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      s0 = mfma16(cur.k0[s], qf[s], s0);
      s1 = mfma16(cur.k1[s], qf[s], s1);
    }
    const int tok0 = blk * kBS + 4 * g;
    float bmax = kNegBig;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s0[r] = (tok0 + r < ctx) ? s0[r] * scale_log2e : kNegBig;
      s1[r] = (tok0 + 16 + r < ctx) ? s1[r] * scale_log2e : kNegBig;
      bmax = fmaxf(bmax, fmaxf(s0[r], s1[r]));
    }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
    const float m_new = fmaxf(m, bmax);
    const float alpha = fast_exp2(m - m_new);
    m = m_new;
    bf16x8 pf;
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p0 = fast_exp2(s0[r] - m_new);
      const float p1 = fast_exp2(s1[r] - m_new);
      psum += p0 + p1;
      pf[r] = f2bf(p0);
      pf[4 + r] = f2bf(p1);
    }
    lsum = lsum * alpha + psum;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      o[i] *= alpha;
      bf16x8 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = cur.vlo[i][j];
        a[4 + j] = cur.vhi[i][j];
      }
      o[i] = mfma16(a, pf, o[i]);
    }
    if (nb < blk_end) cur = nxt;
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);

  // ---- merge the 4 waves through LDS
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sm_m = smem;              // [4][16]
  float* sm_l = smem + 64;         // [4][16]
  float* sm_o = smem + 128;        // [4][D][16]
  if (lane < 16) {
    sm_m[w * 16 + lane] = m;
    sm_l[w * 16 + lane] = lsum;
  }
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      sm_o[(w * D + 16 * i + 4 * g + r) * 16 + col] = o[i][r];
  __syncthreads();

  const bool single = (nparts == 1);
  for (int item = threadIdx.x; item < G * D; item += 256) {
    const int hh = item / D;
    const int d = item - hh * D;
    float M = kNegBig;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, sm_m[ww * 16 + hh]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float f = fast_exp2(sm_m[ww * 16 + hh] - M);
      L += sm_l[ww * 16 + hh] * f;
      O += sm_o[(ww * D + d) * 16 + hh] * f;
    }
    const int hq = h * G + hh;
    if (single) {
      out[((int64_t)b * Hq + hq) * D + d] = f2bf(O / L);
    } else {
      const int64_t pi = ((int64_t)b * Hq + hq) * max_parts + p;
      part_o[pi * D + d] = O;
      if (d == 0) {
        part_ml[pi * 2 + 0] = M;
        part_ml[pi * 2 + 1] = L;
      }
    }
  }
  if (single || counters == nullptr) return;
  // Split-K merge without a second launch: the last partition of this
  // (sequence, kv head) to finish - counted with an agent-scope atomic after
  // a release fence over the partial stores - merges all partitions in fixed
  // order (deterministic) and re-arms the counter for the next launch.
  __shared__ int is_last;
  __shared__ float mh[16], ilh[16];
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(counters + blockIdx.x, 1, __ATOMIC_ACQ_REL,
                                            __HIP_MEMORY_SCOPE_AGENT);
    is_last = (prev == nparts - 1);
    if (is_last) __hip_atomic_store(counters + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!is_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (threadIdx.x < G) {
    const float* ml = part_ml + ((int64_t)b * Hq + h * G + threadIdx.x) * max_parts * 2;
    float M = kNegBig;
    for (int pp = 0; pp < nparts; ++pp) M = fmaxf(M, ml[2 * pp]);
    float L = 0.f;
    for (int pp = 0; pp < nparts; ++pp) L += ml[2 * pp + 1] * fast_exp2(ml[2 * pp] - M);
    mh[threadIdx.x] = M;
    ilh[threadIdx.x] = 1.f / L;
  }
  __syncthreads();
  for (int item = threadIdx.x; item < G * D; item += 256) {
    const int hh = item / D;
    const int d = item - hh * D;
    const int64_t bh = (int64_t)b * Hq + h * G + hh;
    const float* ml = part_ml + bh * max_parts * 2;
    const float M = mh[hh];
    float O = 0.f;
    for (int pp = 0; pp < nparts; ++pp)
      O += part_o[(bh * max_parts + pp) * D + d] * fast_exp2(ml[2 * pp] - M);
    out[bh * D + d] = f2bf(O * ilh[hh]);
  }
}

// Variant 2: one WAVE per (sequence, kv head, partition) work item, four
// independent items per workgroup, no cross-wave merge (no LDS, no barrier).
// Short chat contexts (~6 cache blocks) make variant 1's per-workgroup fixed
// costs - the 4-way LDS merge and the barrier that waits for the slowest
// wave - a large share of each workgroup's life; here every wave streams its
// item's blocks back to back (register double buffer), with the partition's
// block-table slice preloaded into one VGPR (lane j = block j, readlane per
// block) so the K/V loads of block j+1 never wait on a block-table load.
template <int D>
__global__ __launch_bounds__(256, D >= 256 ? 1 : 2) void paged_decode_wave_kernel(
    bf16_t* __restrict__ out, float* __restrict__ part_o,
    float* __restrict__ part_ml, const bf16_t* __restrict__ q, int q_stride,
    const bf16_t* __restrict__ k_cache, const bf16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ context_lens, int B, int Hq, int Hkv, float scale_log2e,
    int max_parts, int blocks_per_part) {
  constexpr int NT = D / 16;
  constexpr int KS = D / 32;
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + wave_id_uniform();
  const int BH = B * Hkv;
  if (item >= BH * max_parts) return;
  const int p = item / BH;  // partition slowest: idle items cluster in late workgroups
  const int bh = item - p * BH;
  const int b = bh / Hkv;
  const int h = bh - b * Hkv;
  const int G = Hq / Hkv;
  const int col = lane & 15, g = lane >> 4;
  const int ctx = context_lens[b];
  if (ctx <= 0) {  // padded batch slot: deterministic zeros, no cache reads
    if (p == 0) {
      bf16x8 z;
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] = f2bf(0.f);
      for (int i = lane; i < G * D / 8; i += 64)
        store_bf16x8(out + ((int64_t)b * Hq + h * G) * D + 8 * i, z);
    }
    return;
  }
  const int nblk = (ctx + kBS - 1) / kBS;
  const int nparts = (nblk + blocks_per_part - 1) / blocks_per_part;
  if (p >= nparts) return;
  const int blk_begin = p * blocks_per_part;
  const int blk_end = min(nblk, blk_begin + blocks_per_part);

  bf16x8 qf[KS];
  const bf16_t* qrow = q + (int64_t)b * q_stride + (int64_t)(h * G + col) * D;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (col < G) qf[s] = load_bf16x8(qrow + 32 * s + 8 * g);
    else for (int j = 0; j < 8; ++j) qf[s][j] = f2bf(0.f);
  }
  const int* bt = block_tables + (int64_t)b * bt_stride;
  int chunk = blk_begin;  // block-table slice [chunk, chunk + 64) held in bt_reg
  int bt_reg = (chunk + lane < blk_end) ? bt[chunk + lane] : 0;
  auto phys_of = [&](int j) -> int64_t {
    if (j - chunk >= 64) {
      chunk += 64;
      bt_reg = (chunk + lane < blk_end) ? bt[chunk + lane] : 0;
    }
    return (int64_t)__builtin_amdgcn_readlane(bt_reg, j - chunk);
  };

  f32x4 o[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) o[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = kNegBig, lsum = 0.f;
  const int64_t blk_elems = (int64_t)kBS * D;
  KVRegs<D> cur, nxt;
  {
    const int64_t ph = phys_of(blk_begin);
    load_kv_block<D>(cur, k_cache + (ph * Hkv + h) * blk_elems,
                     v_cache + (ph * Hkv + h) * blk_elems, lane);
  }
  vm_wait_all();  // the first block lands before the loop (vm_wait_all)
  for (int blk = blk_begin; blk < blk_end; ++blk) {
    const bool more = blk + 1 < blk_end;
    if (more) {
      const int64_t ph = phys_of(blk + 1);
      load_kv_block<D>(nxt, k_cache + (ph * Hkv + h) * blk_elems,
                       v_cache + (ph * Hkv + h) * blk_elems, lane);
    }
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      s0 = mfma16(cur.k0[s], qf[s], s0);
      s1 = mfma16(cur.k1[s], qf[s], s1);
    }
    const int tok0 = blk * kBS + 4 * g;
    float bmax = kNegBig;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s0[r] = (tok0 + r < ctx) ? s0[r] * scale_log2e : kNegBig;
      s1[r] = (tok0 + 16 + r < ctx) ? s1[r] * scale_log2e : kNegBig;
      bmax = fmaxf(bmax, fmaxf(s0[r], s1[r]));
    }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
    const float m_new = fmaxf(m, bmax);
    const float alpha = fast_exp2(m - m_new);
    m = m_new;
    bf16x8 pf;
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p0 = fast_exp2(s0[r] - m_new);
      const float p1 = fast_exp2(s1[r] - m_new);
      psum += p0 + p1;
      pf[r] = f2bf(p0);
      pf[4 + r] = f2bf(p1);
    }
    lsum = lsum * alpha + psum;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      o[i] *= alpha;
      bf16x8 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = cur.vlo[i][j];
        a[4 + j] = cur.vhi[i][j];
      }
      o[i] = mfma16(a, pf, o[i]);
    }
    if (more) cur = nxt;
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (col >= G) return;
  const int hq = h * G + col;
  if (nparts == 1) {
    const float inv = 1.f / lsum;
    bf16_t* orow = out + ((int64_t)b * Hq + hq) * D + 4 * g;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      bf16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(o[i][r] * inv);
      *reinterpret_cast<bf16x4*>(orow + 16 * i) = v;
    }
  } else {
    const int64_t pi = ((int64_t)b * Hq + hq) * max_parts + p;
    float* po = part_o + pi * D + 4 * g;
#pragma unroll
    for (int i = 0; i < NT; ++i) *reinterpret_cast<f32x4*>(po + 16 * i) = o[i];
    if (g == 0) {
      part_ml[pi * 2 + 0] = m;
      part_ml[pi * 2 + 1] = lsum;
    }
  }
}

// Block loads that skip the tokens of a partial last block (nvalid < 32):
// a K row (256 B at D = 128) or a 4-token V group is not fetched when all of
// its tokens are past the context; the registers are zeroed instead (their
// probabilities are exactly 0, zeros keep 0 * V finite).
template <int D>
DRTC_DEVICE void load_kv_block_n(KVRegs<D>& r, const bf16_t* kb, const bf16_t* vb, int lane,
                                 int nvalid) {
  if (nvalid >= kBS) {
    load_kv_block<D>(r, kb, vb, lane);
    return;
  }
  const int t = lane & 15, g = lane >> 4;
  bf16x8 z8;
  bf16x4 z4;
#pragma unroll
  for (int j = 0; j < 8; ++j) z8[j] = f2bf(0.f);
#pragma unroll
  for (int j = 0; j < 4; ++j) z4[j] = f2bf(0.f);
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    r.k0[s] = z8;
    r.k1[s] = z8;
  }
#pragma unroll
  for (int i = 0; i < D / 16; ++i) {
    r.vlo[i] = z4;
    r.vhi[i] = z4;
  }
  if (t < nvalid) {
#pragma unroll
    for (int s = 0; s < D / 32; ++s) r.k0[s] = load_bf16x8(kb + t * D + 32 * s + 8 * g);
  }
  if (16 + t < nvalid) {
#pragma unroll
    for (int s = 0; s < D / 32; ++s) r.k1[s] = load_bf16x8(kb + (16 + t) * D + 32 * s + 8 * g);
  }
  if (4 * g < nvalid) {
#pragma unroll
    for (int i = 0; i < D / 16; ++i) r.vlo[i] = load_bf16x4(vb + g * (4 * D) + (16 * i + t) * 4);
  }
  if (16 + 4 * g < nvalid) {
#pragma unroll
    for (int i = 0; i < D / 16; ++i)
      r.vhi[i] = load_bf16x4(vb + (4 + g) * (4 * D) + (16 * i + t) * 4);
  }
}

// Variant 3: persistent waves.  The grid holds ~2 workgroups per CU; wave w
// of the grid takes work items w, w + W, w + 2W, ... (item = (partition,
// sequence, kv head), partition slowest) and streams their cache blocks back
// to back through one register double buffer: the NEXT item's Q and
// block-table row are loaded when the current item starts, and its first K/V
// block is issued while the current item's last block is computed, so a
// wave never pays the ctx -> table -> K/V load chain between items (variant 2
// pays it once per ~6-block chat context).  Tokens past the context in a
// partial last block are not fetched (load_kv_block_n).  Math per block is
// variant 2's; per-item outputs / partials likewise.
// Fused RoPE + KV write (ROPE = true; engine decode steps): q / k / v of the step's token
// come unrotated straight from the QKV GEMM output (q = its row base, k / v at +Hq*D /
// +(Hq+Hkv)*D), replacing the rope_kv launch of every layer:
//   * each item rotates its G query heads in registers when it starts (NeoX halves: dims
//     32s + 8g + j and D/2 + 32s + 8g + j sit in the same lane, fragments s and s + KS/2);
//   * the cache holds tokens [0, ctx - 1); the step's token (position ctx - 1, its cache row
//     not yet written) is masked out of the block loop (its probability forced to 0, its
//     row not fetched); the item of the LAST partition opens its online softmax with it
//     from registers instead: k rotated the same way, q.k reduced over the 4 lane groups,
//     m = that score, p = 1, o = its v row;
//   * that item also writes the rotated k row and the v row into the paged cache (slot from
//     `slots`) for the next steps - the same bytes rope_kv_kernel_v2 writes.
struct DecodeRope {
  const int* positions;
  const int64_t* slots;
  const float* cos_sin;   // [max_pos][D]: cos | sin
  bf16_t* k_cache;        // the caches the kernel reads (written for the step's token)
  bf16_t* v_cache;
};

// rotate the lane's fragments f[0..KS) of one head (position pos), rounding as rope_kv
template <int D>
DRTC_DEVICE void rope_frags(bf16x8* f, const float* __restrict__ cos_sin, int pos, int g) {
  constexpr int KS = D / 32;
  const float* cs = cos_sin + (int64_t)pos * D + 8 * g;
#pragma unroll
  for (int s = 0; s < KS / 2; ++s) {
    const f32x4 ca = *reinterpret_cast<const f32x4*>(cs + 32 * s);
    const f32x4 cb = *reinterpret_cast<const f32x4*>(cs + 32 * s + 4);
    const f32x4 sa = *reinterpret_cast<const f32x4*>(cs + D / 2 + 32 * s);
    const f32x4 sb = *reinterpret_cast<const f32x4*>(cs + D / 2 + 32 * s + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = j < 4 ? ca[j] : cb[j - 4];
      const float sn = j < 4 ? sa[j] : sb[j - 4];
      const float a = bf2f(f[s][j]), b = bf2f(f[s + KS / 2][j]);
      f[s][j] = f2bf(a * c - b * sn);
      f[s + KS / 2][j] = f2bf(b * c + a * sn);
    }
    // one fragment pair's cos / sin (16 VGPRs) live at a time: this runs beside a whole
    // prefetched K/V block in the persistent kernel, at its register ceiling
    __builtin_amdgcn_sched_barrier(0);
  }
}

// One LDS-DMA wave-instruction of one dword per lane: 256 contiguous bytes land at the LDS byte
// address `dst` (M0 saved and restored).  Counts in vmcnt like any vector load.
DRTC_DEVICE void dma_dword_lds(unsigned dst, unsigned voff, __amdgpu_buffer_rsrc_t rsrc) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dword %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(dst), "v"(voff), "s"(rsrc), "s"(0u)
               : "memory");
}

// rope_frags with the position's cos | sin row read from LDS (the staged row of the item)
template <int D>
DRTC_DEVICE void rope_frags_lds(bf16x8* f, const float* cs_row, int g) {
  constexpr int KS = D / 32;
  const float* cs = cs_row + 8 * g;
#pragma unroll
  for (int s = 0; s < KS / 2; ++s) {
    const f32x4 ca = *reinterpret_cast<const f32x4*>(cs + 32 * s);
    const f32x4 cb = *reinterpret_cast<const f32x4*>(cs + 32 * s + 4);
    const f32x4 sa = *reinterpret_cast<const f32x4*>(cs + D / 2 + 32 * s);
    const f32x4 sb = *reinterpret_cast<const f32x4*>(cs + D / 2 + 32 * s + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = j < 4 ? ca[j] : cb[j - 4];
      const float sn = j < 4 ? sa[j] : sb[j - 4];
      const float a = bf2f(f[s][j]), b = bf2f(f[s + KS / 2][j]);
      f[s][j] = f2bf(a * c - b * sn);
      f[s + KS / 2][j] = f2bf(b * c + a * sn);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int D, bool ROPE>
__global__ __launch_bounds__(256, D >= 256 ? 1 : 2) void paged_decode_persist_kernel(
    bf16_t* __restrict__ out, float* __restrict__ part_o,
    float* __restrict__ part_ml, const bf16_t* __restrict__ q, int q_stride,
    const bf16_t* __restrict__ k_cache, const bf16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ context_lens, int B, int Hq, int Hkv, float scale_log2e,
    int max_parts, int blocks_per_part, DecodeRope rope) {
  constexpr int NT = D / 16;
  constexpr int KS = D / 32;
  const int lane = threadIdx.x & 63;
  const int W = gridDim.x * 4;
  const int BH = B * Hkv;
  const int n_items = BH * max_parts;
  const int G = Hq / Hkv;
  const int col = lane & 15, g = lane >> 4;
  const int64_t blk_elems = (int64_t)kBS * D;

  struct Item {
    int it, b, h, ctx, begin, end, nparts, pos;  // pos: the step token's position (ROPE)
    int64_t slot;                                // its KV-cache slot (ROPE)
    int p;                                       // its partition
  };
  // Wave w takes logical items w, w + W, w + 2W, ... (W = the grid's waves).  Every odd full
  // round is mirrored (logical item k W + j is work item k W + W - 1 - j): with the engine's
  // slots ordered by context length (LLMEngine._sort_slots) a wave then takes one long and
  // one short sequence per pair of rounds, so the slowest wave carries ~2-6 % more blocks
  // than the mean instead of ~10-12 % (chat contexts of 4-8 blocks, 4 items per wave).
  auto phys = [&](int it) -> int {
    const int k = it / W, j = it - k * W;
    return ((k & 1) && (k + 1) * W <= n_items) ? k * W + (W - 1 - j) : it;
  };
  // first item >= it (stride W) with work; padded sequences get their zeros
  auto next_item = [&](int it) -> Item {
    for (; it < n_items; it += W) {
      const int ip = phys(it);
      const int p = ip / BH, bh = ip - p * BH;
      const int b = bh / Hkv, h = bh - b * Hkv;
      // the sequence's three words in one round trip (issued together, then used)
      const int ctx_l = context_lens[b];
      const int pos_l = ROPE ? rope.positions[b] : 0;
      const int64_t slot_l = ROPE ? rope.slots[b] : 0;
      const int ctx = __builtin_amdgcn_readfirstlane(ctx_l);
      if (ctx <= 0) {
        if (p == 0) {
          bf16x8 z;
#pragma unroll
          for (int j = 0; j < 8; ++j) z[j] = f2bf(0.f);
          for (int i = lane; i < G * D / 8; i += 64)
            store_bf16x8(out + ((int64_t)b * Hq + h * G) * D + 8 * i, z);
        }
        continue;
      }
      const int nblk = (ctx + kBS - 1) / kBS;
      const int nparts = (nblk + blocks_per_part - 1) / blocks_per_part;
      if (p >= nparts) continue;
      const int begin = p * blocks_per_part;
      // ROPE: the position and slot are read here, one item ahead of their use
      const int pos = ROPE ? __builtin_amdgcn_readfirstlane(pos_l) : 0;
      const int64_t slot = ROPE ? (int64_t)__builtin_amdgcn_readfirstlane((int)slot_l) |
                                      ((int64_t)__builtin_amdgcn_readfirstlane(
                                           (int)(slot_l >> 32)) << 32)
                                : 0;
      return Item{it, b, h, ctx, begin, min(nblk, begin + blocks_per_part), nparts, pos, slot,
                  p};
    }
    return Item{n_items, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  };
  // ROPE, D = 128 (STAGE): the step token's k and v rows (256 B each, QKV GEMM output) and its
  // cos | sin row (512 B) are staged into this wave's 1 KiB LDS slot by LDS-DMA when the item
  // is chosen - one item ahead, beside the current item's block stream, holding no registers -
  // so starting an item (q rotation, the step token's score, v row and cache write) reads LDS
  // instead of waiting on three memory round trips.  Slot: [0, 256) k row, [256, 512) v row,
  // [512, 1024) cos | sin.
  constexpr bool STAGE = ROPE && D == 128;
  __shared__ __attribute__((aligned(16))) char rope_lds[STAGE ? 4 * 1024 : 16];
  char* const slot_lds = rope_lds + (STAGE ? 1024 * wave_id_uniform() : 0);
  const unsigned slot_dst =
      __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(ad_lds_ptr)slot_lds);
  const __amdgpu_buffer_rsrc_t rsrc_q =
      __builtin_amdgcn_make_buffer_rsrc((void*)q, (short)0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsrc_cs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)rope.cos_sin, (short)0, 0x7FFFFFFF, 0x00020000);
  auto stage_rope = [&](const Item& X) {
    if constexpr (STAGE) {
      const unsigned row = (unsigned)X.b * (unsigned)q_stride * 2u + (unsigned)lane * 4u;
      dma_dword_lds(slot_dst, row + (unsigned)((Hq + X.h) * D) * 2u, rsrc_q);
      dma_dword_lds(slot_dst + 256, row + (unsigned)((Hq + Hkv + X.h) * D) * 2u, rsrc_q);
      const unsigned cs = (unsigned)X.pos * (unsigned)(D * 4) + (unsigned)lane * 4u;
      dma_dword_lds(slot_dst + 512, cs, rsrc_cs);
      dma_dword_lds(slot_dst + 768, cs + 256u, rsrc_cs);
    }
  };
  auto load_q = [&](bf16x8* qf, const Item& A) {
    const bf16_t* qrow = q + (int64_t)A.b * q_stride + (int64_t)(A.h * G + col) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (col < G) qf[s] = load_bf16x8(qrow + 32 * s + 8 * g);
      else for (int j = 0; j < 8; ++j) qf[s][j] = f2bf(0.f);
    }
  };
  auto load_bt = [&](const Item& A, int chunk) -> int {
    const int* bt = block_tables + (int64_t)A.b * bt_stride;
    return (chunk + lane < A.end) ? bt[chunk + lane] : 0;
  };
  // tokens read from the cache: all of the context, or (ROPE) all but the step's own token
  auto cached = [&](const Item& A) { return ROPE ? A.ctx - 1 : A.ctx; };
  auto load_blk = [&](KVRegs<D>& r, const Item& A, int64_t phys, int blk) {
    load_kv_block_n<D>(r, k_cache + (phys * Hkv + A.h) * blk_elems,
                       v_cache + (phys * Hkv + A.h) * blk_elems, lane, cached(A) - blk * kBS);
  };
  auto rope_q = [&](bf16x8* qf, const Item& A) {
    if constexpr (STAGE)
      rope_frags_lds<D>(qf, reinterpret_cast<const float*>(slot_lds + 512), g);
    else if constexpr (ROPE)
      rope_frags<D>(qf, rope.cos_sin, A.pos, g);
  };

  Item A = next_item(blockIdx.x * 4 + wave_id_uniform());
  if (A.it >= n_items) return;
  bf16x8 qf[KS], qn[KS];
  stage_rope(A);
  load_q(qf, A);
  int chunk = A.begin;  // block-table slice [chunk, chunk + 64) of item A in bt_reg
  int bt_reg = load_bt(A, chunk);
  KVRegs<D> cur, nxt;
  load_blk(cur, A, __builtin_amdgcn_readlane(bt_reg, 0), A.begin);
  if constexpr (STAGE) vm_wait_all();  // the first item's staged rows
  rope_q(qf, A);
  // the first block lands before the loop (vm_wait_all: here the merge left a vmcnt(5..2)
  // in front of every block's QK MFMAs, i.e. a wait for 19 of the 24 next-block loads just
  // issued; removing it: kernel -1 %, decode pass -0.2 %, profiles/r6c)
  vm_wait_all();
  while (true) {
    f32x4 o[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) o[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float m = kNegBig, lsum = 0.f;
    if constexpr (ROPE) {
      if (A.p == A.nparts - 1) {
        // the partition holding the step's token: it opens the online softmax (m = its
        // score, p = 1 counted once in lane group 0, o = its v row), before the next
        // item's loads are issued (fewest live registers)
        const bf16_t* kn = STAGE ? reinterpret_cast<const bf16_t*>(slot_lds)
                                 : q + (int64_t)A.b * q_stride + (int64_t)(Hq + A.h) * D;
        const bf16_t* vn = STAGE ? reinterpret_cast<const bf16_t*>(slot_lds + 256)
                                 : kn + (int64_t)Hkv * D;
        bf16x8 kf[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) kf[s] = load_bf16x8(kn + 32 * s + 8 * g);
        if constexpr (STAGE)
          rope_frags_lds<D>(kf, reinterpret_cast<const float*>(slot_lds + 512), g);
        else
          rope_frags<D>(kf, rope.cos_sin, A.pos, g);
        float dot = 0.f;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) dot += bf2f(qf[s][j]) * bf2f(kf[s][j]);
        dot += __shfl_xor(dot, 16, 64);
        dot += __shfl_xor(dot, 32, 64);
        m = dot * scale_log2e;
        lsum = g == 0 ? 1.f : 0.f;
        const int64_t slot = A.slot;
        const bool writer = col == 0 && slot >= 0;  // lanes 0 / 16 / 32 / 48
        const int64_t cblk = slot / kBS, off = slot - cblk * kBS;
        if (writer) {
          bf16_t* kd = rope.k_cache + ((cblk * Hkv + A.h) * kBS + off) * D + 8 * g;
#pragma unroll
          for (int s = 0; s < KS; ++s) store_bf16x8(kd + 32 * s, kf[s]);
        }
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          const bf16x4 v = load_bf16x4(vn + 16 * i + 4 * g);
#pragma unroll
          for (int r = 0; r < 4; ++r) o[i][r] = bf2f(v[r]);  // p = 1 (exact in bf16) times v
        }
        if (slot >= 0) {  // V block [8 groups of 4 tokens][D][4]: one dim per lane per store
          bf16_t* vd = rope.v_cache + (cblk * Hkv + A.h) * blk_elems + (off >> 2) * (4 * D) +
                       (off & 3);
#pragma unroll
          for (int d = lane; d < D; d += 64) vd[d * 4] = vn[d];
        }
      }
    }
    const Item Bn = next_item(A.it + W);
    const bool have_next = Bn.it < n_items;
    int bt_n = 0;
    if (have_next) {
      if constexpr (STAGE) {
        // this item's slot reads (q rotation, step token) have returned before the DMA
        // that overwrites the slot is issued
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        stage_rope(Bn);
      }
      load_q(qn, Bn);
      bt_n = load_bt(Bn, Bn.begin);
    }
    for (int blk = A.begin; blk < A.end; ++blk) {
      const bool more = blk + 1 < A.end;
      if (more) {
        if (blk + 1 - chunk >= 64) {
          chunk += 64;
          bt_reg = load_bt(A, chunk);
        }
        load_blk(nxt, A, __builtin_amdgcn_readlane(bt_reg, blk + 1 - chunk), blk + 1);
      } else if (have_next) {
        load_blk(nxt, Bn, __builtin_amdgcn_readlane(bt_n, 0), Bn.begin);
      }
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        s0 = mfma16(cur.k0[s], qf[s], s0);
        s1 = mfma16(cur.k1[s], qf[s], s1);
      }
      const int tok0 = blk * kBS + 4 * g;
      const int nc = cached(A);
      float bmax = kNegBig;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s0[r] = (tok0 + r < nc) ? s0[r] * scale_log2e : kNegBig;
        s1[r] = (tok0 + 16 + r < nc) ? s1[r] * scale_log2e : kNegBig;
        bmax = fmaxf(bmax, fmaxf(s0[r], s1[r]));
      }
      bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
      bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
      const float m_new = fmaxf(m, bmax);
      const float alpha = fast_exp2(m - m_new);
      m = m_new;
      bf16x8 pf;
      float psum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p0 = fast_exp2(s0[r] - m_new);
        float p1 = fast_exp2(s1[r] - m_new);
        if constexpr (ROPE) {  // a block may hold no cached token at all (m_new = kNegBig)
          p0 = (tok0 + r < nc) ? p0 : 0.f;
          p1 = (tok0 + 16 + r < nc) ? p1 : 0.f;
        }
        psum += p0 + p1;
        pf[r] = f2bf(p0);
        pf[4 + r] = f2bf(p1);
      }
      lsum = lsum * alpha + psum;
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        o[i] *= alpha;
        bf16x8 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = cur.vlo[i][j];
          a[4 + j] = cur.vhi[i][j];
        }
        o[i] = mfma16(a, pf, o[i]);
      }
      if (more || have_next) cur = nxt;
    }
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    if (col < G) {
      const int hq = A.h * G + col;
      const int p = A.p;
      if (A.nparts == 1) {
        const float inv = 1.f / lsum;
        bf16_t* orow = out + ((int64_t)A.b * Hq + hq) * D + 4 * g;
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = f2bf(o[i][r] * inv);
          *reinterpret_cast<bf16x4*>(orow + 16 * i) = v;
        }
      } else {
        const int64_t pi = ((int64_t)A.b * Hq + hq) * max_parts + p;
        float* po = part_o + pi * D + 4 * g;
#pragma unroll
        for (int i = 0; i < NT; ++i) *reinterpret_cast<f32x4*>(po + 16 * i) = o[i];
        if (g == 0) {
          part_ml[pi * 2 + 0] = m;
          part_ml[pi * 2 + 1] = lsum;
        }
      }
    }
    if (!have_next) break;
    A = Bn;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = qn[s];
    rope_q(qf, A);
    chunk = A.begin;
    bt_reg = bt_n;
  }
}

// Merge the per-partition partials of sequences that span > 1 partition.
__global__ __launch_bounds__(256) void decode_reduce_kernel(
    bf16_t* __restrict__ out, const float* __restrict__ part_o,
    const float* __restrict__ part_ml, const int* __restrict__ context_lens,
    int Hq, int D, int max_parts, int blocks_per_part) {
  const int bh = blockIdx.x;  // b * Hq + hq
  const int b = bh / Hq;
  const int ctx = context_lens[b];
  const int nblk = (ctx + kBS - 1) / kBS;
  const int nparts = (nblk + blocks_per_part - 1) / blocks_per_part;
  if (nparts <= 1) return;
  const float* ml = part_ml + (int64_t)bh * max_parts * 2;
  float M = kNegBig;
  for (int p = 0; p < nparts; ++p) M = fmaxf(M, ml[2 * p]);
  float L = 0.f;
  for (int p = 0; p < nparts; ++p) L += ml[2 * p + 1] * fast_exp2(ml[2 * p] - M);
  const float invL = 1.f / L;
  for (int d = threadIdx.x; d < D; d += 256) {
    float O = 0.f;
    for (int p = 0; p < nparts; ++p)
      O += part_o[((int64_t)bh * max_parts + p) * D + d] * fast_exp2(ml[2 * p] - M);
    out[(int64_t)bh * D + d] = f2bf(O * invL);
  }
}

int launch_paged_decode(void* out, float* part_o, float* part_ml, int* counters, const void* q,
                        int q_stride, const void* k_cache, const void* v_cache,
                        const int* block_tables, int bt_stride,
                        const int* context_lens, int B, int Hq, int Hkv, int D,
                        float scale, int max_parts, int blocks_per_part, int variant,
                        hipStream_t st) {
  if (B == 0) return 0;
  if (Hkv <= 0 || Hq % Hkv != 0 || Hq / Hkv > 16) return -1;
  if (max_parts > 1 && (!part_o || !part_ml)) return -2;
  const float sl2 = scale * kLog2e;
  if (variant == 3) {
    static int n_cu = 0;
    if (n_cu == 0) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          n_cu <= 0)
        n_cu = 256;
    }
    // two K/V blocks + two Q fragments per wave: at D = 256 that is ~400 VGPRs,
    // so one workgroup per CU (one wave per SIMD) instead of two
    const int items = B * Hkv * max_parts;
    const int per_cu = D >= 256 ? 1 : 2;
    const dim3 pgrid(std::max(1, std::min((items + 3) / 4, per_cu * n_cu))), pblock(256);
    const DecodeRope nr{};
    switch (D) {
      case 64:
        hipLaunchKernelGGL((paged_decode_persist_kernel<64, false>), pgrid, pblock, 0, st, (bf16_t*)out, part_o, part_ml, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, B, Hq, Hkv, sl2, max_parts, blocks_per_part, nr);
        break;
      case 128:
        hipLaunchKernelGGL((paged_decode_persist_kernel<128, false>), pgrid, pblock, 0, st, (bf16_t*)out, part_o, part_ml, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, B, Hq, Hkv, sl2, max_parts, blocks_per_part, nr);
        break;
      case 256:
        hipLaunchKernelGGL((paged_decode_persist_kernel<256, false>), pgrid, pblock, 0, st, (bf16_t*)out, part_o, part_ml, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, B, Hq, Hkv, sl2, max_parts, blocks_per_part, nr);
        break;
      default:
        return -1;
    }
    if (max_parts > 1)
      hipLaunchKernelGGL(decode_reduce_kernel, dim3(B * Hq), dim3(256), 0, st,
                         (bf16_t*)out, (const float*)part_o, (const float*)part_ml,
                         context_lens, Hq, D, max_parts, blocks_per_part);
    return (int)hipGetLastError();
  }
  if (variant == 2) {
    const dim3 wgrid((B * Hkv * max_parts + 3) / 4), wblock(256);
    switch (D) {
      case 64:
        hipLaunchKernelGGL(paged_decode_wave_kernel<64>, wgrid, wblock, 0, st, (bf16_t*)out, part_o, part_ml, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, B, Hq, Hkv, sl2, max_parts, blocks_per_part);
        break;
      case 128:
        hipLaunchKernelGGL(paged_decode_wave_kernel<128>, wgrid, wblock, 0, st, (bf16_t*)out, part_o, part_ml, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, B, Hq, Hkv, sl2, max_parts, blocks_per_part);
        break;
      case 256:
        hipLaunchKernelGGL(paged_decode_wave_kernel<256>, wgrid, wblock, 0, st, (bf16_t*)out, part_o, part_ml, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, B, Hq, Hkv, sl2, max_parts, blocks_per_part);
        break;
      default:
        return -1;
    }
    if (max_parts > 1)
      hipLaunchKernelGGL(decode_reduce_kernel, dim3(B * Hq), dim3(256), 0, st,
                         (bf16_t*)out, (const float*)part_o, (const float*)part_ml,
                         context_lens, Hq, D, max_parts, blocks_per_part);
    return (int)hipGetLastError();
  }
  if (variant != 1) return -3;
  dim3 grid(B * Hkv, max_parts), block(256);
  const size_t lds = (128 + 4 * (size_t)D * 16) * sizeof(float);
  switch (D) {
    case 64:
      hipLaunchKernelGGL(paged_decode_kernel<64>, grid, block, lds, st, (bf16_t*)out, part_o, part_ml, counters, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, Hq, Hkv, sl2, max_parts, blocks_per_part);
      break;
    case 128:
      hipLaunchKernelGGL(paged_decode_kernel<128>, grid, block, lds, st, (bf16_t*)out, part_o, part_ml, counters, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, Hq, Hkv, sl2, max_parts, blocks_per_part);
      break;
    case 256:
      hipLaunchKernelGGL(paged_decode_kernel<256>, grid, block, lds, st, (bf16_t*)out, part_o, part_ml, counters, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, Hq, Hkv, sl2, max_parts, blocks_per_part);
      break;
    default:
      return -1;
  }
  if (max_parts > 1 && counters == nullptr)
    hipLaunchKernelGGL(decode_reduce_kernel, dim3(B * Hq), dim3(256), 0, st,
                       (bf16_t*)out, (const float*)part_o, (const float*)part_ml,
                       context_lens, Hq, D, max_parts, blocks_per_part);
  return (int)hipGetLastError();
}

// Persistent decode attention with the step's RoPE + KV write fused (DecodeRope above).
// q = row 0 of the QKV GEMM output [B][q_stride] (q | k | v heads, unrotated); D <= 128
// (the persistent form at D = 256 spills; the caller runs rope_kv + the plain form there).
int launch_paged_decode_rope(void* out, float* part_o, float* part_ml, const void* q,
                             int q_stride, void* k_cache, void* v_cache,
                             const int* block_tables, int bt_stride, const int* context_lens,
                             int B, int Hq, int Hkv, int D, float scale, int max_parts,
                             int blocks_per_part, const int* positions, const int64_t* slots,
                             const float* cos_sin, int max_wgs, hipStream_t st) {
  if (B == 0) return 0;
  if (Hkv <= 0 || Hq % Hkv != 0 || Hq / Hkv > 16 || D > 128) return -1;
  if (!positions || !slots || !cos_sin || q_stride < (Hq + 2 * Hkv) * D) return -1;
  if (max_parts > 1 && (!part_o || !part_ml)) return -2;
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cu <= 0)
      n_cu = 256;
  }
  const float sl2 = scale * kLog2e;
  const int items = B * Hkv * max_parts;
  // max_wgs > 0 caps the persistent grid (the kernel strides over its items by the grid's
  // wave count, so any grid size covers every item): attention on part of the chip
  int wgs = std::min((items + 3) / 4, 2 * n_cu);
  if (max_wgs > 0) wgs = std::min(wgs, max_wgs);
  const dim3 pgrid(std::max(1, wgs)), pblock(256);
  const DecodeRope r{positions, slots, cos_sin, (bf16_t*)k_cache, (bf16_t*)v_cache};
  switch (D) {
    case 64:
      hipLaunchKernelGGL((paged_decode_persist_kernel<64, true>), pgrid, pblock, 0, st, (bf16_t*)out, part_o, part_ml, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, B, Hq, Hkv, sl2, max_parts, blocks_per_part, r);
      break;
    case 128:
      hipLaunchKernelGGL((paged_decode_persist_kernel<128, true>), pgrid, pblock, 0, st, (bf16_t*)out, part_o, part_ml, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, bt_stride, context_lens, B, Hq, Hkv, sl2, max_parts, blocks_per_part, r);
      break;
    default:
      return -1;
  }
  if (max_parts > 1)
    hipLaunchKernelGGL(decode_reduce_kernel, dim3(B * Hq), dim3(256), 0, st,
                       (bf16_t*)out, (const float*)part_o, (const float*)part_ml,
                       context_lens, Hq, D, max_parts, blocks_per_part);
  return (int)hipGetLastError();
}

int configure_decode() {
  const int lds = (128 + 4 * 256 * 16) * sizeof(float);
  return (int)hipFuncSetAttribute((const void*)paged_decode_kernel<256>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

}  // namespace drtc
