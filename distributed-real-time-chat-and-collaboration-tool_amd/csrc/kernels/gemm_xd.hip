// XCD-partitioned decode GEMM for gfx950 (MI355X):  c[M, N] = epi( a[M, K] . b[N, K]^T )
//
// The full-batch decode projections (M = 512..1024 rows of activations, N x K weights: Llama-3-8B
// qkv / o / down) have too few 256 x 256 tiles to fill 256 CUs (o: 4 x 16 = 64), and every CU
// ingests operands at a bounded rate (~54 GB/s per CU measured on these tiles,
// profiles/r4g, r4h: the same for 3 and 4 K tiles in flight), so the time of a decode GEMM is
// set by the operand bytes each CU must read: (rows + columns of its tile) x K x 2.  This
// kernel picks the tile per shape:
//
//   * 128 MT x 32 NF output tiles (MT 1 / 2, NF 2 / 4 / 6 / 8), K split over splitk = 1..8 slices
//     (whole K tiles, as even as they divide), one workgroup per (tile, slice) and per CU
//     (o / down at M = 1024: 8 x 32 tiles of 128 x 128, or 4 x 32 x 2 slices of 256 x 128;
//     qkv N = 6144: 8 x 32 of 128 x 192; Llama-3-70B at M = 256: 256 x 128 x 3-4 slices;
//     gated gate_up at M = 512-1024: 256 x 256).  Per shape the tuning table picks the form
//     (scripts/tune_xd.py, ops/gemm.py route / glu_form).
//   * Tile order partitioned by XCD (workgroup b runs on XCD b % 8 under round-robin dispatch -
//     used for speed only, the map below is a bijection of blockIdx): XCD x owns one K slice of
//     a contiguous range of the column-major tile order, i.e. a contiguous set of weight column
//     panels and ALL row tiles of each.  Every weight byte is fetched from HBM into ONE XCD's
//     L2, and the workgroups that share a panel stream it through that L2 in K-lockstep (the
//     activations, 1-8 MB, are read by every XCD from the Infinity Cache).
//   * 4 waves, one per SIMD, 64 MT x 16 NF outputs per wave (4 MT x NF MFMA 16x16x32 tiles);
//     the 16x16x32 form, not 32x32x16: same LDS bytes per FLOP at a given wave tile, and the
//     bf16 16x16x32 loop holds a 12-15 % higher clock on random data (MI355X_MICROARCH.md,
//     DVFS give-back item 7).
//   * LDS: S stages x [A 128 MT rows | B 32 NF rows] x 128 B (one 64-deep K tile), filled by
//     LDS-DMA (buffer_load_dwordx4 ... lds, 8 rows per wave-instruction), chunk c of row r
//     stored at c ^ ((r >> 1) & 7): conflict-free ds_read_b128 of the MFMA fragments (the same
//     involution on the DMA source address and on the read address).  S - 1 K tiles in flight.
//   * Per K tile a fixed order pinned with sched_barrier: half 0 MFMAs | ds_read of half 1;
//     [vmcnt: own DMA of tile t + 1 landed, lgkmcnt(0), ONE barrier: everyone's tile t + 1
//     landed and every read of stage t done]; half 1 MFMAs | LDS-DMA of tile t + S into stage
//     t + ds_read of tile t + 1 half 0.  The first K tile accumulates onto a zero C operand.
//   * Split-K with a ticket-first combine: each slice draws a ticket when its K loop ends;
//     tickets 0 .. splitk - 2 write their fp32 tile to their slice's slab slot (write-through
//     sc1 stores, drained, barrier) and count themselves ready; the last ticket (resident, and
//     waiting only for slices that already hold a ticket: no wait on an unscheduled
//     workgroup) polls the ready count (bounded), sums the slices in slice order (its own
//     accumulators at its own position: bitwise deterministic whatever the arrival order;
//     sc1 loads) inside its epilogue and re-arms both counters.  cdna_hip_programming.md §6
//     G16 hand-off recipe.
//   * Epilogue through LDS (the wave's tile as bf16, then 16-B row-contiguous global stores):
//     store, + residual (may alias c), or SiLU / tanh-GELU gating of a [gate; up] weight:
//     each wave's B rows hold the gate rows (fragments j < NF / 2) and the up rows (j >= NF /
//     2) of the SAME 8 NF output columns, so the gate value meets its up value in a lane.
#include "common.h"
#include "launchers.h"

#include <cstdlib>
#include <utility>

namespace drtc {
namespace {

typedef __attribute__((address_space(3))) void* xd_lds_ptr;

constexpr int kXdThreads = 256;
enum { XD_STORE = 0, XD_RESIDUAL = 1, XD_SILU = 2, XD_GELU = 3 };
template <int EPI>
DRTC_DEVICE constexpr bool xd_glu() { return EPI == XD_SILU || EPI == XD_GELU; }

template <int MT_, int NF_, int S_, bool SPLIT_, bool NT_ = false>
struct XdCfg {
  static constexpr int MT = MT_, NF = NF_, S = S_;
  static constexpr bool SPLIT = SPLIT_;            // split-K combine compiled in
  static constexpr bool NT = NT_;                  // weight (B) LDS-DMA non-temporal
  static constexpr int TM = 128 * MT;              // tile rows
  static constexpr int TN = 32 * NF;               // tile columns
  static constexpr int FA = 4 * MT;                // A fragments per wave (16 rows each)
  static constexpr int H = FA * NF;                // MFMAs per 32-deep K half (per wave)
  static constexpr int DA = 4 * MT, DB = NF, D = DA + DB;  // LDS-DMA per wave per K tile
  static constexpr int NR = FA + NF;               // fragment reads per wave per K half
  static constexpr int BOFF = TM * 128;            // B region within a stage
  static constexpr int STAGE = BOFF + TN * 128;
  static constexpr int LDS = S * STAGE;            // the K-tile ring
  static constexpr int PITCH = 32 * NF + 16;       // epilogue bytes per wave-tile row (padded)
  static constexpr int IMAGE = 4 * 64 * MT * PITCH;  // the epilogue's bf16 tile image
  static constexpr int ALLOC = LDS > IMAGE ? LDS : IMAGE;
  static_assert(ALLOC <= 160 * 1024, "LDS exceeds the CU's 160 KiB");
  static_assert(NR < H, "half-0 fragment reads must fit the half");
};

struct XdParams {
  bf16_t* c;
  const bf16_t* a;
  const bf16_t* b;
  const bf16_t* r;
  float* slab;
  int* counters;
  int M, N, K;  // N = columns of c (gated: N = up_off, b has 2 N rows)
  int lda, ldb, ldc, ldr;
  int tiles_m, tiles_n, per_xcd;
  int splitk, up_off;
  int slab_bytes;  // the split-K slab descriptor's range
  int* err;        // split-K fault word: a fixed slot of the workspace (the last counter),
                   // outside every launch's ticket range; read and cleared by the host
  int spin_limit;  // bound of the last ticket's ready poll (< 0: test hook, always fault)
  // grouped (mixture-of-experts) mode, kernel template G: row tile tm of the launch is entry tm
  // of a device tile table - rows [g_row0[tm], + g_rows[tm]) of A and C, weights of expert
  // g_expert[tm] (b + expert * g_bstride); A rows gathered through g_aidx (token of each
  // (token, expert) pair) when given; entries at or past *g_ntiles are empty
  const int* g_row0;
  const int* g_rows;
  const int* g_expert;
  const int* g_ntiles;
  const int* g_aidx;
  int64_t g_bstride;
};

template <class C>
struct XdDma {
  __amdgpu_buffer_rsrc_t ra, rb;
  unsigned va[C::DA];
  unsigned vb[C::DB];
  unsigned lds_a, lds_b;  // LDS byte address of this wave's first DMA block in stage 0
};

// Fragment read offsets within a stage (bytes): row 64 MT wm + l16 (A) / 16 NF wn + l16 (B),
// 16-B chunk 4 h + g stored at chunk ^ ((row >> 1) & 7); + 2048 per 16-row fragment.
struct XdFrag {
  int ra0, ra1, rb0, rb1;
};

DRTC_DEVICE void xd_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int N>
DRTC_DEVICE void xd_vmcnt() {
  constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
  __builtin_amdgcn_s_waitcnt(imm);
}
DRTC_DEVICE void xd_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
DRTC_DEVICE bf16x8 xd_rd(const char* lds, int off) {
  return *reinterpret_cast<const bf16x8*>(lds + off);
}

// One LDS-DMA wave-instruction outside the main loop: M0 saved and restored.  NT: the
// non-temporal policy (a weight byte that one CU reads once, MI355X_MICROARCH.md nt-weights).
template <bool NT = false>
DRTC_DEVICE void xd_dma(unsigned dst, unsigned voff, __amdgpu_buffer_rsrc_t rsrc, unsigned soff) {
  unsigned keep;
  if constexpr (NT)
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "s"(dst), "v"(voff), "s"(rsrc), "s"(soff)
        : "memory");
  else
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "s"(dst), "v"(voff), "s"(rsrc), "s"(soff)
        : "memory");
}

// Fragment r of a K half in consumption order (A row block 0, every B column block, then the
// other A row blocks): the half's reads are issued in this order.
template <class C, int R>
DRTC_DEVICE void xd_read(bf16x8 (&fa)[C::FA], bf16x8 (&fb)[C::NF], const char* lds, int base,
                         int ra, int rb) {
  if constexpr (R == 0)
    fa[0] = xd_rd(lds, base + ra);
  else if constexpr (R <= C::NF)
    fb[R - 1] = xd_rd(lds, base + rb + 2048 * (R - 1));
  else
    fa[R - C::NF] = xd_rd(lds, base + ra + 2048 * (R - C::NF));
}

template <class C, int R0, int R1>
DRTC_DEVICE void xd_reads(bf16x8 (&fa)[C::FA], bf16x8 (&fb)[C::NF], const char* lds, int base,
                          int ra, int rb) {
  if constexpr (R0 < R1) {
    xd_read<C, R0>(fa, fb, lds, base, ra, rb);
    xd_reads<C, R0 + 1, R1>(fa, fb, lds, base, ra, rb);
  }
}

// LDS-DMA s (0 .. D - 1) of the main loop: the A group then the B group.  M0 (the LDS
// destination) is set at the first DMA of each group and advanced by 1 KiB after each; K
// advances through the scalar offset (nothing else in this kernel uses M0).
template <class C, int Sd>
DRTC_DEVICE void xd_dma_step(const XdDma<C>& d, int cur, unsigned kb) {
  if constexpr (Sd < C::DA) {
    if constexpr (Sd == 0)
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(d.lds_a + cur) : "memory");
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
                 : : "v"(d.va[Sd]), "s"(d.ra), "s"(kb) : "memory");
    if constexpr (Sd + 1 < C::DA) asm volatile("s_add_u32 m0, m0, 0x400" ::: "memory");
  } else {
    if constexpr (Sd == C::DA)
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(d.lds_b + cur) : "memory");
    if constexpr (C::NT)
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen nt lds"
                   : : "v"(d.vb[Sd - C::DA]), "s"(d.rb), "s"(kb) : "memory");
    else
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
                   : : "v"(d.vb[Sd - C::DA]), "s"(d.rb), "s"(kb) : "memory");
    if constexpr (Sd + 1 < C::D) asm volatile("s_add_u32 m0, m0, 0x400" ::: "memory");
  }
}

template <class C, int S0, int S1>
DRTC_DEVICE void xd_dmas(const XdDma<C>& d, int cur, unsigned kb) {
  if constexpr (S0 < S1) {
    xd_dma_step<C, S0>(d, cur, kb);
    xd_dmas<C, S0 + 1, S1>(d, cur, kb);
  }
}

// Step Q of a K tile (0 .. 2 H - 1): MFMA Q, then the memory work scheduled behind it.  All
// conditions are compile-time constants; sched_barrier(0) pins the emitted order.
template <class C, bool DMA, bool NEXT, int WT, bool Z, int Q>
DRTC_DEVICE void xd_step(f32x4 (&acc)[C::FA][C::NF], bf16x8 (&fa0)[C::FA], bf16x8 (&fb0)[C::NF],
                         bf16x8 (&fa1)[C::FA], bf16x8 (&fb1)[C::NF], const char* lds, int cur,
                         int nxt, unsigned kb, const XdFrag& f, const XdDma<C>& d) {
  constexpr int H = C::H, NF = C::NF;
  constexpr int h = Q / H, rem = Q % H, i = rem / NF, j = rem % NF;
  if constexpr (h == 0 && Z)  // first K tile: accumulate onto 0 (no zeroed AGPRs to coalesce)
    acc[i][j] = mfma16(fa0[i], fb0[j], (f32x4){0.f, 0.f, 0.f, 0.f});
  else if constexpr (h == 0)
    acc[i][j] = mfma16(fa0[i], fb0[j], acc[i][j]);
  else
    acc[i][j] = mfma16(fa1[i], fb1[j], acc[i][j]);
  // ---- half 0: fragments of this tile's half 1 (one per MFMA from step 1)
  if constexpr (h == 0 && Q >= 1 && Q <= C::NR)
    xd_read<C, Q - 1>(fa1, fb1, lds, cur, f.ra1, f.rb1);
  // ---- boundary: tile t + 1 landed for every wave; every read of this stage is done
  if constexpr (NEXT && Q == H - 1) {
    xd_vmcnt<WT * C::D>();  // WT younger K tiles of this wave may still be in flight
    xd_lgkm0();
    xd_barrier();
  }
  // ---- half 1: DMA of tile t + S into this stage, spread over the half; the next tile's
  // half-0 fragments in between
  if constexpr (DMA && h == 1)
    xd_dmas<C, (rem * C::D + H - 1) / H, ((rem + 1) * C::D + H - 1) / H>(d, cur, kb);
  if constexpr (NEXT && h == 1)
    xd_reads<C, (rem * C::NR + H - 1) / H, ((rem + 1) * C::NR + H - 1) / H>(fa0, fb0, lds, nxt,
                                                                           f.ra0, f.rb0);
  __builtin_amdgcn_sched_barrier(0);
}

template <class C, bool DMA, bool NEXT, int WT, bool Z, int... Qs>
DRTC_DEVICE void xd_steps(std::integer_sequence<int, Qs...>, f32x4 (&acc)[C::FA][C::NF],
                          bf16x8 (&fa0)[C::FA], bf16x8 (&fb0)[C::NF], bf16x8 (&fa1)[C::FA],
                          bf16x8 (&fb1)[C::NF], const char* lds, int cur, int nxt, unsigned kb,
                          const XdFrag& f, const XdDma<C>& d) {
  (xd_step<C, DMA, NEXT, WT, Z, Qs>(acc, fa0, fb0, fa1, fb1, lds, cur, nxt, kb, f, d), ...);
}

template <class C, bool DMA, bool NEXT, int WT, bool Z = false>
DRTC_DEVICE void xd_tile(f32x4 (&acc)[C::FA][C::NF], bf16x8 (&fa0)[C::FA], bf16x8 (&fb0)[C::NF],
                         bf16x8 (&fa1)[C::FA], bf16x8 (&fb1)[C::NF], const char* lds, int cur,
                         int nxt, unsigned kb, const XdFrag& f, const XdDma<C>& d) {
  xd_steps<C, DMA, NEXT, WT, Z>(std::make_integer_sequence<int, 2 * C::H>{}, acc, fa0, fb0, fa1,
                                fb1, lds, cur, nxt, kb, f, d);
}

// The last S tiles: nothing more to load; WT = S - 2, ..., 0 younger tiles still in flight.
template <class C, int WT>
DRTC_DEVICE void xd_tail(f32x4 (&acc)[C::FA][C::NF], bf16x8 (&fa0)[C::FA], bf16x8 (&fb0)[C::NF],
                         bf16x8 (&fa1)[C::FA], bf16x8 (&fb1)[C::NF], const char* lds, int cur,
                         const XdFrag& f, const XdDma<C>& d) {
  if constexpr (WT < 0) {
    xd_tile<C, false, false, 0>(acc, fa0, fb0, fa1, fb1, lds, cur, cur, 0u, f, d);
  } else {
    const int nxt = cur + C::STAGE == C::LDS ? 0 : cur + C::STAGE;
    xd_tile<C, false, true, WT>(acc, fa0, fb0, fa1, fb1, lds, cur, nxt, 0u, f, d);
    xd_tail<C, WT - 1>(acc, fa0, fb0, fa1, fb1, lds, nxt, f, d);
  }
}

// Split-K, ticket-first combine (see the file comment).  Counters of tile t: [2 t] ticket,
// [2 t + 1] ready count; the error word p.err is a fixed slot outside every ticket range (a
// partial that never arrived).  The slab holds one partial slot per slice and tile.  Returns
// 0 for a slice that published its partial (it is done), 1 for the last ticket, which sums
// the slices inside the epilogue (xd_sum_frags: groups of fragments, in place) and
// re-arms the counters, 2 for a last ticket whose poll timed out: it records the fault and
// does NOT re-arm (the host reads the word, zeroes the counters and raises).
template <class C>
constexpr int xd_tile_bytes() { return C::FA * C::NF * kXdThreads * 16; }
constexpr int kXdSc1 = 16;  // cache-policy bits of the buffer op: sc1 (write-through)

// A work item's place in its tile's combine: n slices (K ranges of the tile, in K order), this
// one at position c; position s publishes into slab slot base + s (tile * n + s), of
// xd_tile_bytes each.
struct XdPart {
  int n, c, base;
};
template <class C>
DRTC_DEVICE unsigned xd_slot_off(const XdPart& q, int s) {
  return (unsigned)(q.base + s) * (unsigned)xd_tile_bytes<C>();
}

DRTC_DEVICE __amdgpu_buffer_rsrc_t xd_slab(const XdParams& p) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p.slab, (short)0, p.slab_bytes, 0x00020000);
}

template <class C>
DRTC_DEVICE int xd_combine(const XdParams& p, f32x4 (&acc)[C::FA][C::NF], int tile,
                           const XdPart& q, char* lds) {
  const __amdgpu_buffer_rsrc_t slab = xd_slab(p);
  int* ticket = p.counters + 2 * tile;
  int* ready = ticket + 1;
  int* flag = reinterpret_cast<int*>(lds);
  const int tid = threadIdx.x;
  __syncthreads();  // every wave is done with the stages (flag lives in LDS)
  if (tid == 0)
    *flag = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int t = *flag;
  if (t < q.n - 1) {
    // publish the partial in this position's slot, fragment order (16 B per lane, coalesced),
    // then count it ready
    const unsigned base = xd_slot_off<C>(q, q.c);
#pragma unroll
    for (int i = 0; i < C::FA; ++i)
#pragma unroll
      for (int j = 0; j < C::NF; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), slab,
                                               base + ((i * C::NF + j) * kXdThreads + tid) * 16,
                                               0, kXdSc1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  // the last ticket: every other contributor holds a ticket (resident, past its K loop)
  __syncthreads();  // every wave has read the ticket before the flag word is reused
  if (tid == 0) {
    int spins = 0, fault = 0;
    while (p.spin_limit < 0 ||
           __hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < q.n - 1) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > p.spin_limit) {  // never hang the GPU: record the fault, keep the counters
        __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fault = 1;
        break;
      }
    }
    *flag = fault;
  }
  __syncthreads();
  return *flag ? 2 : 1;
}

// Split-K: the NJ fragments (i, col(jj)) of the tile summed over the slices in slice order
// (this workgroup's accumulators at its own position: bitwise deterministic whatever the
// arrival order) into out[].  Every load of a group of QG slice positions is issued before the
// first is used, so the combine pays one memory latency per fragment group and slice group
// instead of one per fragment and slice (the per-fragment form cost 66 us of an 88 us 2x8
// split-4 GEMM, profiles/r5t).  A position past n, and this item's own, reads outside
// the slab descriptor's range: 0, no memory access.
template <class C, int NJ, int QG, bool GLU>
DRTC_DEVICE void xd_sum_frags(const XdParams& p, const __amdgpu_buffer_rsrc_t& slab, int i,
                              int j0, const XdPart& pq, const f32x4 (&acc)[C::FA][C::NF],
                              f32x4 (&out)[NJ]) {
  constexpr int NF = C::NF;
  // fragment column of group member jj: plain j0 + jj; gated: the gate columns j0 + jj, then
  // the up columns of the same outputs
  auto col = [&](int jj) {
    return GLU ? (jj < NJ / 2 ? j0 + jj : NF / 2 + j0 + jj - NJ / 2) : j0 + jj;
  };
  const unsigned tid = threadIdx.x;
  const unsigned oob = (unsigned)p.slab_bytes;
#pragma unroll
  for (int s0 = 0; s0 < 8; s0 += QG) {  // n <= 8; whole groups past n are skipped
    if (s0 >= pq.n) continue;
    f32x4 v[QG][NJ];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
      const int s = s0 + q;
      const unsigned base = (s == pq.c || s >= pq.n) ? oob : xd_slot_off<C>(pq, s);
#pragma unroll
      for (int jj = 0; jj < NJ; ++jj)
        v[q][jj] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       slab, base + ((i * NF + col(jj)) * kXdThreads + tid) * 16u, 0, kXdSc1));
    }
    // positions past n loaded 0: adding them is exact
#pragma unroll
    for (int q = 0; q < QG; ++q) {
      const int s = s0 + q;
#pragma unroll
      for (int jj = 0; jj < NJ; ++jj) {
        const f32x4 x = s == pq.c ? acc[i][col(jj)] : v[q][jj];
        out[jj] = s == 0 ? x : out[jj] + x;
      }
    }
  }
}
template <class C, int EPI, bool G = false>
__global__ __launch_bounds__(kXdThreads, 1) void gemm_xd_kernel(XdParams p) {
  constexpr int MT = C::MT, NF = C::NF, FA = C::FA;
  extern __shared__ __attribute__((aligned(16))) char xd_lds[];
  // ---- work item: XCD label x = b % 8 takes the items [x per_xcd, (x + 1) per_xcd) of the
  // slice-major, column-major order (item = slice * tiles + tile; all row tiles of a weight
  // panel consecutive): an XCD streams one K slice of a contiguous block of column panels
  const int b = blockIdx.x;
  const int ntiles = p.tiles_m * p.tiles_n;
  const int item = (b & 7) * p.per_xcd + (b >> 3);
  if (item >= ntiles * p.splitk) return;
  const int slice = item / ntiles, tile = item - slice * ntiles;
  const int nkt = p.K >> 6;  // slice s: K tiles [s nkt / splitk, (s + 1) nkt / splitk)
  const int kt0 = slice * nkt / p.splitk;
  const int nk = (slice + 1) * nkt / p.splitk - kt0;
  const XdPart q{p.splitk, slice, tile * p.splitk};
  const int tn = tile / p.tiles_m, tm = tile - tn * p.tiles_m;
  constexpr int TNO = xd_glu<EPI>() ? C::TN / 2 : C::TN;  // output columns per tile
  const int n0 = TNO * tn;
  int m0, rows_a;  // first row of the tile in A / C, valid rows
  const bf16_t* bmat = p.b;
  if constexpr (G) {
    if (tm >= p.g_ntiles[0]) return;  // an empty entry of the tile table
    m0 = p.g_row0[tm];
    rows_a = p.g_rows[tm];
    bmat += (int64_t)p.g_expert[tm] * p.g_bstride;
  } else {
    m0 = C::TM * tm;
    rows_a = min(C::TM, p.M - m0);
  }

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wv >> 1, wn = wv & 1, l16 = lane & 15, g = lane >> 4;
  const int64_t k0 = (int64_t)kt0 * 64;

  // ---- DMA plan: instruction i of wave wv fills stage rows 32 MT wv + 8 i + (lane >> 3)
  // (A) / 8 NF wv + 8 i + (lane >> 3) (B), lane's LDS chunk lane & 7 <- source chunk ^
  // swizzle.  A rows past M read row M - 1 (valid bytes, never stored).
  XdDma<C> d;
  const unsigned lds0 = (unsigned)(uintptr_t)(xd_lds_ptr)xd_lds;
  {
    const bool gather = G && p.g_aidx != nullptr;
    const char* abase =
        reinterpret_cast<const char*>(p.a + (gather ? 0 : (int64_t)m0 * p.lda) + k0);
    const char* bbase = reinterpret_cast<const char*>(bmat + (int64_t)n0 * p.ldb + k0);
    d.ra = __builtin_amdgcn_make_buffer_rsrc((void*)abase, (short)0, 0x7FFFFFFF, 0x00020000);
    d.rb = __builtin_amdgcn_make_buffer_rsrc((void*)bbase, (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
    for (int i = 0; i < C::DA; ++i) {
      const int R = 32 * MT * wv + 8 * i + (lane >> 3);
      const int c = (lane & 7) ^ ((R >> 1) & 7);
      const int row = min(R, rows_a - 1);
      const int src = gather ? p.g_aidx[m0 + row] : row;  // A row (a token, grouped mode)
      d.va[i] = (unsigned)(src * p.lda * 2 + c * 16);
    }
#pragma unroll
    for (int i = 0; i < C::DB; ++i) {
      const int R = 8 * NF * wv + 8 * i + (lane >> 3);
      const int c = (lane & 7) ^ ((R >> 1) & 7);
      int src = R;  // weight row (relative to n0) of stage row R
      if constexpr (xd_glu<EPI>()) {
        // wave half w = R / 16 NF, fragment jb = (R % 16 NF) / 16: gate rows of output
        // columns w 8 NF + (jb % (NF / 2)) 16 + (R % 16), then the up rows of the same columns
        const int w = R / (16 * NF), jb = (R % (16 * NF)) / 16;
        const int col = w * 8 * NF + (jb % (NF / 2)) * 16 + (R & 15);
        src = jb < NF / 2 ? col : p.up_off + col;
      }
      d.vb[i] = (unsigned)(src * p.ldb * 2 + c * 16);
    }
    d.lds_a = __builtin_amdgcn_readfirstlane(lds0 + 32 * MT * wv * 128);
    d.lds_b = __builtin_amdgcn_readfirstlane(lds0 + C::BOFF + 8 * NF * wv * 128);
  }
  XdFrag f;
  {
    const int fx = (l16 >> 1) & 7;
    f.ra0 = (64 * MT * wm + l16) * 128 + ((0 + g) ^ fx) * 16;
    f.ra1 = (64 * MT * wm + l16) * 128 + ((4 + g) ^ fx) * 16;
    f.rb0 = C::BOFF + (16 * NF * wn + l16) * 128 + ((0 + g) ^ fx) * 16;
    f.rb1 = C::BOFF + (16 * NF * wn + l16) * 128 + ((4 + g) ^ fx) * 16;
  }
  const char* lds = xd_lds;

  f32x4 acc[FA][NF];  // written first by the K tile 0 MFMAs (onto a zero C operand)

  // ---- prologue: K tiles 0 .. S-1 into the S stages (the launcher guarantees nk > S)
#pragma unroll
  for (int u = 0; u < C::S; ++u) {
#pragma unroll
    for (int i = 0; i < C::DA; ++i)
      xd_dma(d.lds_a + u * C::STAGE + 1024 * i, d.va[i], d.ra, (unsigned)u * 128u);
#pragma unroll
    for (int i = 0; i < C::DB; ++i)
      xd_dma<C::NT>(d.lds_b + u * C::STAGE + 1024 * i, d.vb[i], d.rb, (unsigned)u * 128u);
  }
  xd_vmcnt<(C::S - 1) * C::D>();
  xd_barrier();
  bf16x8 fa0[FA], fb0[NF], fa1[FA], fb1[NF];
  xd_reads<C, 0, C::NR>(fa0, fb0, lds, 0, f.ra0, f.rb0);

  // ---- main loop: tile t in stage cur; its half 1 DMAs tile t + S into the same stage
  xd_tile<C, true, true, C::S - 2, true>(acc, fa0, fb0, fa1, fb1, lds, 0, C::STAGE % C::LDS,
                                         (unsigned)C::S * 128u, f, d);
  int cur = C::STAGE % C::LDS;
  for (int t = 1; t + C::S < nk; ++t) {
    const int nxt = cur + C::STAGE == C::LDS ? 0 : cur + C::STAGE;
    xd_tile<C, true, true, C::S - 2>(acc, fa0, fb0, fa1, fb1, lds, cur, nxt,
                                     (unsigned)(t + C::S) * 128u, f, d);
    cur = nxt;
  }
  xd_tail<C, C::S - 2>(acc, fa0, fb0, fa1, fb1, lds, cur, f, d);
  xd_vmcnt<0>();

  bool part = false;   // split-K: this workgroup adds the other slices' partials
  bool rearm = false;  // ... and re-arms the tile's counters (not after a fault)
  if constexpr (C::SPLIT) {
    const int st = xd_combine<C>(p, acc, tile, q, xd_lds);
    if (st == 0) return;
    part = true;
    rearm = st == 1;
  }

  // ---- epilogue: the wave's tile as bf16 into LDS, then 16-B global stores of whole row
  // segments (acc[i][j][r] = C[64 MT wm + 16 i + 4 g + r][16 NF wn + 16 j + l16]; gated:
  // output column 8 NF wn + 16 j + l16 = act(acc[i][j]) * acc[i][j + NF / 2], j < NF / 2)
  __syncthreads();  // every wave is done reading the stages
  constexpr int OC = xd_glu<EPI>() ? 8 * NF : 16 * NF;  // output columns per wave
  constexpr int PITCH = 2 * OC + 16;
  char* ep = xd_lds + wv * 64 * MT * PITCH;
  const __amdgpu_buffer_rsrc_t slab = xd_slab(p);
  // split-K combine groups (the sums are consumed here, the accumulators stay in place): a
  // row block's fragments x 4 slice positions in flight, NF 6 / 8 one position at a time
  // (more spills: those kernels hold 192 / 256 accumulator registers)
  constexpr int QG = NF >= 6 ? 1 : 4;
  constexpr int NP = NF >= 8 ? 4 : NF / 2;  // gated: column pairs per group
  constexpr int JB = NF >= 8 ? 8 : NF;      // plain: fragments per group
  static_assert(NF % JB == 0 && (NF / 2) % NP == 0, "combine groups tile the fragments");
#pragma unroll
  for (int i = 0; i < FA; ++i) {
    if constexpr (xd_glu<EPI>()) {
#pragma unroll
      for (int jp0 = 0; jp0 < NF / 2; jp0 += NP) {
        f32x4 v[2 * NP];
#pragma unroll
        for (int jj = 0; jj < NP; ++jj) {
          v[jj] = acc[i][jp0 + jj];
          v[NP + jj] = acc[i][NF / 2 + jp0 + jj];
        }
        if constexpr (C::SPLIT) {
          if (part) xd_sum_frags<C, 2 * NP, QG, true>(p, slab, i, jp0, q, acc, v);
        }
#pragma unroll
        for (int jj = 0; jj < NP; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            *reinterpret_cast<bf16_t*>(ep + (16 * i + 4 * g + r) * PITCH +
                                       (16 * (jp0 + jj) + l16) * 2) =
                f2bf(act_value<EPI == XD_SILU ? 0 : 1>(v[jj][r]) * v[NP + jj][r]);
      }
    } else {
#pragma unroll
      for (int j0 = 0; j0 < NF; j0 += JB) {
        f32x4 v[JB];
#pragma unroll
        for (int jj = 0; jj < JB; ++jj) v[jj] = acc[i][j0 + jj];
        if constexpr (C::SPLIT) {
          if (part) xd_sum_frags<C, JB, QG, false>(p, slab, i, j0, q, acc, v);
        }
#pragma unroll
        for (int jj = 0; jj < JB; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            *reinterpret_cast<bf16_t*>(ep + (16 * i + 4 * g + r) * PITCH +
                                       (16 * (j0 + jj) + l16) * 2) = f2bf(v[jj][r]);
      }
    }
  }
  if (C::SPLIT && rearm && threadIdx.x == 0) {
    // re-arm (the next launch on this stream starts after this one ends)
    __hip_atomic_store(p.counters + 2 * tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p.counters + 2 * tile + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  constexpr int CPR = OC / 8;  // 16-B chunks per wave-tile row
#pragma unroll
  for (int s = 0; s < CPR * MT; ++s) {
    const int q = lane + 64 * s;
    const int row = q / CPR, ch = q - row * CPR;
    if (64 * MT * wm + row >= rows_a) continue;
    const int m = m0 + 64 * MT * wm + row;
    const int n = n0 + OC * wn + 8 * ch;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(ep + row * PITCH + ch * 16);
    if constexpr (EPI == XD_RESIDUAL) {
      const bf16x8 rv = *reinterpret_cast<const bf16x8*>(p.r + (int64_t)m * p.ldr + n);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(rv[e]));
    }
    *reinterpret_cast<bf16x8*>(p.c + (int64_t)m * p.ldc + n) = v;
  }
}

template <class C, int EPI, bool G = false>
int xd_launch_e(const XdParams& p, hipStream_t st) {
  hipLaunchKernelGGL((gemm_xd_kernel<C, EPI, G>), dim3(8 * p.per_xcd), dim3(kXdThreads),
                     (C::ALLOC), st, p);
  return (int)hipGetLastError();
}

template <class C>
int xd_launch(const XdParams& p, int epi, hipStream_t st) {
  switch (epi) {
    case XD_STORE: return xd_launch_e<C, XD_STORE>(p, st);
    case XD_RESIDUAL: return xd_launch_e<C, XD_RESIDUAL>(p, st);
    case XD_SILU: return xd_launch_e<C, XD_SILU>(p, st);
    default: return xd_launch_e<C, XD_GELU>(p, st);
  }
}

// grouped mode: store (expert down projection) and the gated epilogues (expert gate_up)
template <class C>
int xd_launch_g(const XdParams& p, int epi, hipStream_t st) {
  switch (epi) {
    case XD_STORE: return xd_launch_e<C, XD_STORE, true>(p, st);
    case XD_SILU: return xd_launch_e<C, XD_SILU, true>(p, st);
    case XD_GELU: return xd_launch_e<C, XD_GELU, true>(p, st);
    default: return -1;
  }
}

template <class C>
int xd_cfg() {
  int e = 0;
  for (const void* f : {(const void*)gemm_xd_kernel<C, XD_STORE>,
                        (const void*)gemm_xd_kernel<C, XD_RESIDUAL>,
                        (const void*)gemm_xd_kernel<C, XD_SILU>,
                        (const void*)gemm_xd_kernel<C, XD_GELU>})
    e |= (int)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, C::ALLOC);
  return e;
}
template <class C>
int xd_cfg_g() {
  int e = 0;
  for (const void* f : {(const void*)gemm_xd_kernel<C, XD_STORE, true>,
                        (const void*)gemm_xd_kernel<C, XD_SILU, true>,
                        (const void*)gemm_xd_kernel<C, XD_GELU, true>})
    e |= (int)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, C::ALLOC);
  return e;
}

// Forms built (mt, nf) -> ring depth: 128-row tiles nf 2 / 4 / 6 (4 / 4 / 3 stages), 256-row
// tiles nf 4 / 6 / 8 (3 / 2 / 2 stages); each with and without the split-K combine.
// The 128 x 128 .. 256 x 256 tiles also with non-temporal weight loads (decode batches of one
// row tile, where each weight byte enters one CU once).
template <bool SP, bool NT = false>
using Xd1x2 = XdCfg<1, 2, 4, SP, NT>;
template <bool SP, bool NT = false>
using Xd1x4 = XdCfg<1, 4, 4, SP, NT>;
template <bool SP, bool NT = false>
using Xd1x6 = XdCfg<1, 6, 3, SP, NT>;
template <bool SP, bool NT = false>
using Xd2x4 = XdCfg<2, 4, 3, SP, NT>;
template <bool SP, bool NT = false>
using Xd2x6 = XdCfg<2, 6, 2, SP, NT>;
template <bool SP, bool NT = false>
using Xd2x8 = XdCfg<2, 8, 2, SP, NT>;

int xd_stages(int mt, int nf) {
  if (mt == 1) return nf == 6 ? 3 : (nf == 2 || nf == 4 ? 4 : 0);
  if (mt == 2) return nf == 4 ? 3 : (nf == 6 || nf == 8 ? 2 : 0);
  return 0;
}

template <bool SP>
int xd_dispatch(const XdParams& p, int mt, int nf, bool nt, int epi, hipStream_t st) {
  if (nt) {
    switch (mt * 10 + nf) {
      case 14: return xd_launch<Xd1x4<SP, true>>(p, epi, st);
      case 16: return xd_launch<Xd1x6<SP, true>>(p, epi, st);
      case 24: return xd_launch<Xd2x4<SP, true>>(p, epi, st);
      case 26: return xd_launch<Xd2x6<SP, true>>(p, epi, st);
      case 28: return xd_launch<Xd2x8<SP, true>>(p, epi, st);
      default: return -1;
    }
  }
  switch (mt * 10 + nf) {
    case 12: return xd_launch<Xd1x2<SP>>(p, epi, st);
    case 14: return xd_launch<Xd1x4<SP>>(p, epi, st);
    case 16: return xd_launch<Xd1x6<SP>>(p, epi, st);
    case 24: return xd_launch<Xd2x4<SP>>(p, epi, st);
    case 26: return xd_launch<Xd2x6<SP>>(p, epi, st);
    case 28: return xd_launch<Xd2x8<SP>>(p, epi, st);
    default: return -1;
  }
}

// grouped (MoE) mode: the 128 x 128, 256 x 128 and 256 x 256 tiles
template <bool SP>
int xd_dispatch_g(const XdParams& p, int mt, int nf, bool nt, int epi, hipStream_t st) {
  switch (mt * 10 + nf + (nt ? 100 : 0)) {
    case 14: return xd_launch_g<Xd1x4<SP>>(p, epi, st);
    case 24: return xd_launch_g<Xd2x4<SP>>(p, epi, st);
    case 28: return xd_launch_g<Xd2x8<SP>>(p, epi, st);
    case 114: return xd_launch_g<Xd1x4<SP, true>>(p, epi, st);
    case 124: return xd_launch_g<Xd2x4<SP, true>>(p, epi, st);
    case 128: return xd_launch_g<Xd2x8<SP, true>>(p, epi, st);
    default: return -1;
  }
}

int g_spin_limit = 1 << 24;

}  // namespace

int splitk_spin_limit() { return g_spin_limit; }
void set_splitk_spin_limit(int limit) { g_spin_limit = limit; }

int64_t gemm_xd_workspace_bytes(int M, int N, int mt, int nf, int splitk, int glu) {
  if (splitk < 2 || mt < 1 || nf < 1) return 0;
  const int tno = glu ? 16 * nf : 32 * nf;
  const int64_t tiles = (int64_t)((M + 128 * mt - 1) / (128 * mt)) * (N / tno);
  return tiles * splitk * (128 * mt) * (32 * nf) * 4;
}

int launch_gemm_xd(void* c, const void* a, const void* b, const void* r, int M, int N, int K,
                   int lda, int ldb, int ldc, int ldr, int epi, int mt, int nf, int splitk,
                   void* slab, int64_t slab_bytes, int* counters, int n_counters,
                   hipStream_t st) {
  const bool nt = (mt & 16) != 0;  // mt bit 4: non-temporal weight loads
  mt &= 15;
  if (epi < XD_STORE || epi > XD_GELU) return -1;
  const bool glu = epi == XD_SILU || epi == XD_GELU;
  const int stages = xd_stages(mt, nf);
  if (stages == 0 || splitk < 1 || splitk > 8 || (glu && nf % 2)) return -1;
  if (lda % 8 || ldb % 8 || ldc % 8) return -1;
  if ((uintptr_t)a % 16 || (uintptr_t)b % 16 || (uintptr_t)c % 16) return -1;
  if (epi == XD_RESIDUAL && (r == nullptr || ldr % 8 || (uintptr_t)r % 16)) return -1;
  const int tm_rows = 128 * mt, tno = glu ? 16 * nf : 32 * nf;
  // shape contract: whole column tiles, every slice more K tiles than the ring holds (the
  // first K tile is peeled), 32-bit buffer offsets from the tile bases
  if (M <= 0 || N <= 0 || N % tno || K % 64 || K / 64 / splitk <= stages) return -1;
  if ((int64_t)tm_rows * lda * 2 >= (1ll << 31) ||
      (int64_t)(glu ? N + tno : 32 * nf) * ldb * 2 >= (1ll << 31))
    return -1;
  XdParams p{};
  p.c = (bf16_t*)c;
  p.a = (const bf16_t*)a;
  p.b = (const bf16_t*)b;
  p.r = (const bf16_t*)r;
  p.M = M; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldr = ldr;
  p.tiles_m = (M + tm_rows - 1) / tm_rows;
  p.tiles_n = N / tno;
  p.splitk = splitk;
  p.up_off = glu ? N : 0;
  const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
  if (tiles * splitk * 8 >= (1ll << 31)) return -1;
  p.per_xcd = (int)((tiles * splitk + 7) / 8);
  const int64_t need = gemm_xd_workspace_bytes(M, N, mt, nf, splitk, glu);
  if (splitk > 1) {
    // tile counters [0, 2 tiles) and the error word at the workspace's last slot
    if (slab == nullptr || counters == nullptr || n_counters < 2 * tiles + 2 ||
        slab_bytes < need || need >= (1ll << 31))
      return -2;
    p.slab = (float*)slab;
    // DRTC_XD_SLAB_TIMING=1: a timing-only build of the combine's memory traffic - a zero-range
    // slab descriptor drops every partial load and store while the ticket protocol, the
    // instruction stream and the waits stay (cdna_hip_programming.md pricing recipe); WRONG
    // results, probes only
    static const bool slab_timing = std::getenv("DRTC_XD_SLAB_TIMING") != nullptr;
    p.slab_bytes = slab_timing ? 0 : (int)need;
    p.counters = counters;
    p.err = counters + n_counters - 1;
    p.spin_limit = splitk_spin_limit();
    return xd_dispatch<true>(p, mt, nf, nt, epi, st);
  }
  return xd_dispatch<false>(p, mt, nf, nt, epi, st);
}

int launch_gemm_xd_grouped(void* c, const void* a, const void* b, int a_rows, int N, int K,
                           int lda, int ldb, int ldc, int epi, int mt, int nf, int splitk,
                           int max_tiles, const int* tile_row0, const int* tile_rows,
                           const int* tile_expert, const int* n_tiles, const int* a_index,
                           int64_t b_stride, void* slab, int64_t slab_bytes, int* counters,
                           int n_counters, hipStream_t st) {
  const bool nt = (mt & 16) != 0;
  mt &= 15;
  if (epi != XD_STORE && epi != XD_SILU && epi != XD_GELU) return -1;
  const bool glu = epi != XD_STORE;
  const int stages = xd_stages(mt, nf);
  if (stages == 0 || splitk < 1 || splitk > 8 || (glu && nf % 2)) return -1;
  if (lda % 8 || ldb % 8 || ldc % 8 || max_tiles < 1 || a_rows < 1) return -1;
  if ((uintptr_t)a % 16 || (uintptr_t)b % 16 || (uintptr_t)c % 16) return -1;
  if (tile_row0 == nullptr || tile_rows == nullptr || tile_expert == nullptr || n_tiles == nullptr)
    return -1;
  const int tm_rows = 128 * mt, tno = glu ? 16 * nf : 32 * nf;
  if (N <= 0 || N % tno || K % 64 || K / 64 / splitk <= stages) return -1;
  // 32-bit buffer offsets: a gathered A row anywhere in A, a tile's rows of contiguous A, the
  // weight rows of one expert
  if ((int64_t)(a_index ? a_rows : tm_rows) * lda * 2 >= (1ll << 31) ||
      (int64_t)(glu ? N + tno : 32 * nf) * ldb * 2 >= (1ll << 31))
    return -1;
  XdParams p{};
  p.c = (bf16_t*)c;
  p.a = (const bf16_t*)a;
  p.b = (const bf16_t*)b;
  p.M = max_tiles * tm_rows; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.tiles_m = max_tiles;
  p.tiles_n = N / tno;
  p.splitk = splitk;
  p.up_off = glu ? N : 0;
  p.g_row0 = tile_row0;
  p.g_rows = tile_rows;
  p.g_expert = tile_expert;
  p.g_ntiles = n_tiles;
  p.g_aidx = a_index;
  p.g_bstride = b_stride;
  const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
  if (tiles * splitk * 8 >= (1ll << 31)) return -1;
  p.per_xcd = (int)((tiles * splitk + 7) / 8);
  if (splitk > 1) {
    const int64_t need = tiles * splitk * tm_rows * (32 * nf) * 4;
    if (slab == nullptr || counters == nullptr || n_counters < 2 * tiles + 2 ||
        slab_bytes < need || need >= (1ll << 31))
      return -2;
    p.slab = (float*)slab;
    p.slab_bytes = (int)need;
    p.counters = counters;
    p.err = counters + n_counters - 1;
    p.spin_limit = splitk_spin_limit();
    return xd_dispatch_g<true>(p, mt, nf, nt, epi, st);
  }
  return xd_dispatch_g<false>(p, mt, nf, nt, epi, st);
}

int configure_gemm_xd() {
  const int g = xd_cfg_g<Xd1x4<false>>() | xd_cfg_g<Xd2x4<false>>() | xd_cfg_g<Xd2x8<false>>() |
                xd_cfg_g<Xd1x4<true>>() | xd_cfg_g<Xd2x4<true>>() | xd_cfg_g<Xd2x8<true>>() |
                xd_cfg_g<Xd1x4<false, true>>() | xd_cfg_g<Xd2x4<false, true>>() |
                xd_cfg_g<Xd2x8<false, true>>() | xd_cfg_g<Xd1x4<true, true>>() |
                xd_cfg_g<Xd2x4<true, true>>() | xd_cfg_g<Xd2x8<true, true>>();
  if (g) return g;
  return xd_cfg<Xd1x2<false>>() | xd_cfg<Xd1x4<false>>() | xd_cfg<Xd1x6<false>>() |
         xd_cfg<Xd2x4<false>>() | xd_cfg<Xd2x6<false>>() | xd_cfg<Xd1x2<true>>() |
         xd_cfg<Xd1x4<true>>() | xd_cfg<Xd1x6<true>>() | xd_cfg<Xd2x4<true>>() |
         xd_cfg<Xd2x6<true>>() | xd_cfg<Xd2x8<false>>() | xd_cfg<Xd2x8<true>>() |
         xd_cfg<Xd1x4<false, true>>() | xd_cfg<Xd1x6<false, true>>() |
         xd_cfg<Xd2x4<false, true>>() | xd_cfg<Xd2x6<false, true>>() |
         xd_cfg<Xd2x8<false, true>>() | xd_cfg<Xd1x4<true, true>>() |
         xd_cfg<Xd1x6<true, true>>() | xd_cfg<Xd2x4<true, true>>() |
         xd_cfg<Xd2x6<true, true>>() | xd_cfg<Xd2x8<true, true>>();
}

}  // namespace drtc
