// Hand-scheduled 4-wave CDNA4 (gfx950) bf16 GEMM for the projection layers:
//
//   C[M, N] = epi( A[M, K] . B[N, K]^T )      (A activations, B weights, both K-contiguous)
//
// epilogues: store / + residual (may alias C) / SiLU- or GELU-gated [gate; up].
// This is the GEMM of the engine's prefill and full-batch decode passes (replacing the model
// hop of ref llm_server/llm_server.py:231 / :287 with on-node compute).
//
// Why this layout: 8-wave forms (2 waves per SIMD, 128 x 64 per wave; round 2, removed in
// round 4) reached 0.76-0.81x of hipBLASLt on the Llama shapes (profiles/r2a_hand_gemm.md):
// parked at barriers (SQ_WAIT_ANY 9x the library's) and issuing 1.5x the LDS reads per
// MFMA.  This kernel uses the layout that reads the least LDS per FLOP - one wave per SIMD,
// 128 x 128 outputs per wave (64 MFMA 16x16x32 tiles = 256 accumulator registers, the AGPR
// half of the unified file) - and hides every latency INSIDE the wave with an explicit
// instruction schedule instead of a partner wave:
//
//   * LDS: 2 stages x [A 256 rows | B 256 rows] x 128 B (one 64-deep K tile) = 129 KiB, filled
//     by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB = 8 rows per wave-instruction).  A: the
//     16-B chunk of row r stored at chunk ^ ((r >> 1) & 7) - conflict-free ds_read_b128 for
//     the MFMA lane groups (the XOR is applied to the per-lane DMA SOURCE address and to the
//     read address - the two sides of one involution).  B: 1040-B blocks of 8 rows (16 B of
//     padding), read 8 rows apart (fragment j, lane row l -> B row 8 l + j).
//   * Registers: the fragments of a whole K tile (both 32-deep halves, A and B: 128 VGPRs),
//     so a stage is released as soon as its reads are in registers - the DMA of tile t + 2
//     goes into the stage of tile t while tile t's MFMAs still run (two tiles in flight).
//   * Per K tile (128 MFMAs) a fixed order, pinned with sched_barrier:
//       MFMA   0- 21  half 0 | ds_read of B half 1 (tile t)
//       [lgkmcnt(0), barrier 1: B region of stage t free]
//       MFMA  22- 57  half 0 | ds_read of A half 1 (tile t) + 8 DMA of B (tile t+2), one per 4 MFMA
//       [lgkmcnt(0), barrier 2: A region free]
//       MFMA  58-103  half 0/1 | 8 DMA of A (tile t+2)
//       [vmcnt(16): own DMA of tile t+1 landed; barrier 3: everyone's]
//       MFMA 104-127  half 1 | 16 ds_read of half 0 of tile t+1
//     Three barriers per K tile, each in the middle of an MFMA stream.
//   * B fragment j, lane row l reads B row 8 l + j, so a lane's accumulators over the 8 B
//     fragments are 8 consecutive output columns: the epilogue stores 16 B per lane (4 rows x
//     256 contiguous bytes per instruction), and a gated tile pairs gate fragment j with up
//     fragment j + 4 of the same columns in a lane.  Every DMA instruction still reads 8
//     consecutive weight rows (a first form that permuted the rows in the DMA read 8 rows
//     64 KiB apart per instruction and ran 1.5-2.5x slower wherever B streams from HBM).
//   * XCD-aware, row-grouped tile order; split-K with an fp32 slab and an in-launch combine
//     by the last arriving slice (agent-scope release / acquire ticket) for short-M shapes.
#include "common.h"
#include "launchers.h"

#include <utility>

namespace drtc {
int w4_num_cus();
namespace {

typedef __attribute__((address_space(3))) void* w4_lds_ptr;

constexpr int kW4Threads = 256;
// Stage: A 256 rows x 128 B (XOR-swizzled chunks) | B 32 blocks of 8 rows x 128 B, each block
// followed by 16 B of padding (1040-B blocks: B rows are read 8 apart, the padding spreads
// them over the banks while every DMA instruction still loads 8 CONSECUTIVE weight rows).
constexpr int kW4BOff = 32768;                 // B region within a stage
constexpr int kW4BBlk = 1040;                  // bytes per 8-row B block
constexpr int kW4Stage = kW4BOff + 32 * kW4BBlk;  // 66048
constexpr int kW4Lds = 2 * kW4Stage;

enum { W4_STORE = 0, W4_RESIDUAL = 1, W4_SILU = 2, W4_GELU = 3 };

struct W4Params {
  bf16_t* c;
  const bf16_t* a;
  const bf16_t* b;
  const bf16_t* r;
  float* slab;
  int* counters;
  int M, N, K;  // N = columns of C
  int lda, ldb, ldc, ldr;
  int tiles_m, tiles_n, splitk, kt_split;
  int up_off;
  int group_m;
  int xk;  // K-slice-by-XCD tile order (split-K forms; see gemm_w4_kernel)
  int krot;  // V & 16: distinct K start offsets over the 8 XCD labels (8: one per XCD)
  int* err;        // split-K fault word: the workspace's last counter, outside every ticket
                   // range; read and cleared by the host
  int spin_limit;  // bound of the parallel combine's arrival poll (< 0: test hook, always fault)
  // V & 64, grouped form (persistent only): n_grp row groups of A / C, group g = rows
  // [grp[g], grp[g + 1]) (device array, written by the producing kernel: no host sync), each
  // multiplied by its own B at b + g * b_grp.  tiles_m is unused (the tile count is derived on
  // the device); M bounds the rows the launcher sized the grid for.
  // ksplit > 1: every group's K is cut into ksplit slices (kt_split K tiles each), slice s
  // written to c + s * c_split (bf16 partial products, summed by the consumer)
  const int* grp;
  int n_grp;
  int64_t b_grp;
  int ksplit;
  int64_t c_split;
};

// Position of one output tile: row tile tm, column tile tn; grouped form: rows [row0,
// min(row0 + 256, mend)) and operand B b (the plain forms read 256 tm, M and p.b instead, so
// their code is the same as before the grouped form existed: no spill of the 256 + 256
// register budget).
struct W4Pos {
  int tm, tn;
  int row0, mend;
  const bf16_t* b;
  int koff;  // grouped split-K: K element offset of the slice
  bf16_t* c;  // grouped split-K: the slice's output
};
template <int V>
DRTC_DEVICE int w4_row0(const W4Pos& q) {
  if constexpr ((V & 64) != 0) return q.row0; else return 256 * q.tm;
}
template <int V>
DRTC_DEVICE int w4_mend(const W4Params& p, const W4Pos& q) {
  if constexpr ((V & 64) != 0) return q.mend; else return p.M;
}
template <int V>
DRTC_DEVICE const bf16_t* w4_bop(const W4Params& p, const W4Pos& q) {
  if constexpr ((V & 64) != 0) return q.b; else return p.b;
}
template <int V>
DRTC_DEVICE int w4_koff(const W4Pos& q) {
  if constexpr ((V & 64) != 0) return q.koff; else return 0;
}
template <int V>
DRTC_DEVICE bf16_t* w4_cop(const W4Params& p, const W4Pos& q) {
  if constexpr ((V & 64) != 0) return q.c; else return p.c;
}

template <int EPI>
DRTC_DEVICE constexpr bool w4_glu() { return EPI == W4_SILU || EPI == W4_GELU; }
template <int EPI>
DRTC_DEVICE constexpr bool w4_res() { return EPI == W4_RESIDUAL; }
template <int EPI>
DRTC_DEVICE constexpr int w4_act() { return EPI == W4_SILU ? 0 : 1; }

// One LDS-DMA wave-instruction: 64 lanes x 16 B from rsrc + voff + soff into LDS bytes
// [dst, dst + 1024).  Inline asm (hipcc would pin vmcnt / lgkmcnt waits around a builtin
// form it cannot order against the ds_reads); M0 is written and restored in the statement.
// One LDS-DMA wave-instruction outside the main loop (prologue): M0 saved and restored.
DRTC_DEVICE void w4_dma(unsigned dst, unsigned voff, __amdgpu_buffer_rsrc_t rsrc, unsigned soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(dst), "v"(voff), "s"(rsrc), "s"(soff)
      : "memory");
}

template <int N>
DRTC_DEVICE void w4_vmcnt() {
  constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
  __builtin_amdgcn_s_waitcnt(imm);
}
DRTC_DEVICE void w4_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
DRTC_DEVICE void w4_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

DRTC_DEVICE bf16x8 w4_rd(const char* lds, int off) {
  return *reinterpret_cast<const bf16x8*>(lds + off);
}

// Per-wave DMA plan: A rows of instruction i are 32 i + 8 wv + (lane >> 3) of the tile
// (rows past M lie outside the descriptor range: read as 0, never stored), B rows 32 i / 16 i
// (gated) apart (one VGPR offset + scalar steps).
struct W4Dma {
  __amdgpu_buffer_rsrc_t ra, rb;
  unsigned va[8];
  unsigned vb;
  unsigned sb[8];     // byte offset of B instruction s (beyond the per-lane row)
  unsigned lds_a, lds_b;  // LDS byte address of this wave's first block in stage 0
  const char* abase;      // operand bases (lean form: descriptors rebuilt per tile)
  const char* bbase;
  unsigned na;            // bytes of this tile's valid A rows from abase: DMA rows past M
                          // are out of the descriptor's range (read as 0, never stored)
};

// Per-tile state handed to every step of the unrolled schedule.
struct W4Tile {
  const char* lds;
  int cur, nxt;        // byte offsets of this tile's stage and the next tile's
  int ra0, ra1, rb0, rb1;
  unsigned kb;         // K byte offset of tile t + 2 (its DMA goes into stage `cur`)
  __amdgpu_buffer_rsrc_t rak, rbk;  // lean form: descriptors based at K byte kb
  bool seam;           // persistent step 0 after a full tile's epilogue (its 32 stores are
                       // younger than the DMA this step waits for)
};

// Step Q (0..127) of a K tile: MFMA Q, then the memory work scheduled behind it.  Every
// condition is a compile-time constant (the tile is a fold over Q), so the emitted stream is
// straight-line, and sched_barrier(0) pins it in this order.
//
// Main-loop DMA issue: M0 (the LDS destination) is set once per operand group, one MFMA ahead
// of the group's first DMA, and advanced by 4 KiB right after each DMA; K advances through
// the buffer base (descriptor rebuilt once per tile) so the scalar offsets are loop-invariant:
// one SALU per DMA (nothing else in this kernel uses M0).
//
// Schedule variants (mfma_gemm variant 7 + V):
//   V & 2  plain (temporal) epilogue stores instead of non-temporal ones
//   V & 8  persistent form (see gemm_w4_kernel); V & 16 its per-XCD K rotation
//   V & 32 the next tile's half-0 fragments read one per 4 MFMAs over half 1 (barrier 3 at
//          MFMA 63) instead of one per MFMA at 104-119: the burst ran the LDS array at its
//          256 B/clk limit beside the landing LDS-DMA (PMC: +72 % SQ_WAIT_INST_LDS against
//          hipBLASLt's kernel of the same tile, profiles/r4j)
template <int V, bool DMA, bool NEXT, bool Z, int Q>
DRTC_DEVICE void w4_step(f32x4 (&acc)[8][8], bf16x8 (&fa0)[8], bf16x8 (&fb0)[8],
                         bf16x8 (&fa1)[8], bf16x8 (&fb1)[8], const W4Tile& T, const W4Dma& d) {
  constexpr int i = (Q >> 3) & 7, j = Q & 7;
  if constexpr (Q < 64 && Z)  // first K tile of a persistent tile: accumulate onto 0
    acc[i][j] = mfma16(fa0[i], fb0[j], (f32x4){0.f, 0.f, 0.f, 0.f});
  else if constexpr (Q < 64)
    acc[i][j] = mfma16(fa0[i], fb0[j], acc[i][j]);
  else
    acc[i][j] = mfma16(fa1[i], fb1[j], acc[i][j]);
  // ---- half 1 of this tile: B fragments (one read per 2 MFMA), then A
  if constexpr (Q < 16 && (Q & 1) == 0) fb1[Q >> 1] = w4_rd(T.lds, T.cur + T.rb1 + 128 * (Q >> 1));
  if constexpr (Q == 21) {
    w4_lgkm0();
    w4_barrier();  // every wave's B reads of this stage are done
  }
  if constexpr (Q >= 22 && Q < 38 && ((Q - 22) & 3) < 2) {
    constexpr int a = ((Q - 22) >> 2) * 2 + ((Q - 22) & 1);
    fa1[a] = w4_rd(T.lds, T.cur + T.ra1 + 2048 * a);
  }
  if constexpr (Q == 57) {
    w4_lgkm0();
    w4_barrier();  // every wave's A reads of this stage are done
  }
  // ---- DMA of tile t + 2 into this stage: B group, then A group, one per 4 MFMA
  constexpr int qb = 24, qa = 60;
  if constexpr (DMA && Q == qb - 1)
    asm volatile("s_mov_b32 m0, %0" : : "s"(d.lds_b + T.cur) : "memory");
  if constexpr (DMA && Q >= qb && Q <= qb + 28 && ((Q - qb) & 3) == 0) {
    constexpr int s = (Q - qb) >> 2;
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
                 : : "v"(d.vb), "s"(T.rbk), "s"(d.sb[s]) : "memory");
    if constexpr (s < 7) asm volatile("s_add_u32 m0, m0, 0x1040" ::: "memory");  // 4 blocks
  }
  if constexpr (DMA && Q == qa - 1)
    asm volatile("s_mov_b32 m0, %0" : : "s"(d.lds_a + T.cur) : "memory");
  if constexpr (DMA && Q >= qa && Q <= qa + 28 && ((Q - qa) & 3) == 0) {
    constexpr int s = (Q - qa) >> 2;
    asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds"
                 : : "v"(d.va[s]), "s"(T.rak) : "memory");
    if constexpr (s < 7) asm volatile("s_add_u32 m0, m0, 0x1000" ::: "memory");
  }
  // ---- tile t + 1: its DMA (issued during tile t - 1) landed for every wave, then its
  // half-0 fragments: fa0[0], fb0[0..7], fa0[1..7]
  constexpr bool kSpread = (V & 32) != 0;
  constexpr int qn = kSpread ? 63 : 103;
  // this step's own DMAs (tile t + 2) issued before qn: B 8 + A (1 at qn 63, 8 at 103)
  constexpr int kYoung = kSpread ? 9 : 16;
  if constexpr (NEXT && Q == qn) {
    if constexpr (DMA && Z) {
      // first K step of a persistent tile: the previous tile's epilogue stores sit between
      // the DMA of K step 1 (needed now) and this step's DMA - do not wait for them
      if (T.seam)
        w4_vmcnt<32 + kYoung>();
      else
        w4_vmcnt<kYoung>();
    } else if constexpr (DMA) {
      w4_vmcnt<kYoung>();
    } else {
      w4_vmcnt<0>();
    }
    w4_barrier();
  }
  if constexpr (NEXT && kSpread && Q > qn && ((Q - qn - 1) & 3) == 0 && (Q - qn - 1) / 4 < 16) {
    constexpr int r = (Q - qn - 1) / 4;
    if constexpr (r == 0)
      fa0[0] = w4_rd(T.lds, T.nxt + T.ra0);
    else if constexpr (r <= 8)
      fb0[r - 1] = w4_rd(T.lds, T.nxt + T.rb0 + 128 * (r - 1));
    else
      fa0[r - 8] = w4_rd(T.lds, T.nxt + T.ra0 + 2048 * (r - 8));
  }
  if constexpr (NEXT && !kSpread && Q > qn && Q <= qn + 16) {
    constexpr int r = Q - qn - 1;
    if constexpr (r == 0)
      fa0[0] = w4_rd(T.lds, T.nxt + T.ra0);
    else if constexpr (r <= 8)
      fb0[r - 1] = w4_rd(T.lds, T.nxt + T.rb0 + 128 * (r - 1));
    else
      fa0[r - 8] = w4_rd(T.lds, T.nxt + T.ra0 + 2048 * (r - 8));
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int V, bool DMA, bool NEXT, bool Z, int... Qs>
DRTC_DEVICE void w4_steps(std::integer_sequence<int, Qs...>, f32x4 (&acc)[8][8],
                          bf16x8 (&fa0)[8], bf16x8 (&fb0)[8], bf16x8 (&fa1)[8],
                          bf16x8 (&fb1)[8], const W4Tile& T, const W4Dma& d) {
  (w4_step<V, DMA, NEXT, Z, Qs>(acc, fa0, fb0, fa1, fb1, T, d), ...);
}

template <int V, bool DMA, bool NEXT, bool Z = false>
DRTC_DEVICE void w4_tile(f32x4 (&acc)[8][8], bf16x8 (&fa0)[8], bf16x8 (&fb0)[8],
                         bf16x8 (&fa1)[8], bf16x8 (&fb1)[8], const char* lds, int cur, int ra0,
                         int ra1, int rb0, int rb1, const W4Dma& d, int t2, bool seam = false) {
  W4Tile T{lds, cur, kW4Stage - cur, ra0, ra1, rb0, rb1, (unsigned)t2 * 128u};
  T.seam = seam;
  T.rak = __builtin_amdgcn_make_buffer_rsrc((void*)(d.abase + T.kb), (short)0, (int)(d.na - T.kb),
                                            0x00020000);
  T.rbk = __builtin_amdgcn_make_buffer_rsrc((void*)(d.bbase + T.kb), (short)0, 0x7FFFFFFF,
                                            0x00020000);
  w4_steps<V, DMA, NEXT, Z>(std::make_integer_sequence<int, 128>{}, acc, fa0, fb0, fa1, fb1, T, d);
}

// acc[i][j][r] = C[row 128 wm + 16 i + 4 g + r][column of B fragment j, row l16]: lane l16
// holds columns 8 l16 + j (j = 0..7) of its 4 rows -> one 16-B store per (i, r); a store
// instruction writes 4 rows x 256 contiguous bytes.
// Epilogue stores are non-temporal (measured +2-3 % on the 16k-row shapes: the output does
// not displace the operands' lines in the L2 on its way out).
template <int V>
DRTC_DEVICE void w4_st16(bf16_t* p, bf16x8 v) {
  if constexpr (V & 2)
    *reinterpret_cast<bf16x8*>(p) = v;
  else
    __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p));
}
template <int V>
DRTC_DEVICE void w4_st8(bf16_t* p, bf16x4 v) {
  if constexpr (V & 2)
    *reinterpret_cast<bf16x4*>(p) = v;
  else
    __builtin_nontemporal_store(v, reinterpret_cast<bf16x4*>(p));
}

template <int EPI, int V>
DRTC_DEVICE void w4_epilogue(const W4Params& p, bf16_t* cbase, f32x4 (&acc)[8][8], int row0,
                             int mend, int tn, int wm, int wn, int l16, int g, int slice) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = row0 + 128 * wm + 16 * i + 4 * g + r;
      if (m >= mend) continue;
      bf16_t* crow = cbase + (int64_t)m * p.ldc;
      if constexpr (w4_glu<EPI>()) {
        const int n = 128 * tn + 64 * wn + 4 * l16;
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = f2bf(act_value<w4_act<EPI>()>(acc[i][j][r]) * acc[i][j + 4][r]);
        w4_st8<V>(crow + n, o);
      } else if constexpr (!w4_res<EPI>()) {
        const int n = 256 * tn + 128 * wn + 8 * l16;
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[i][j][r]);
        w4_st16<V>(crow + n, o);
      }
    }
  }
  if constexpr (w4_res<EPI>()) {
    // every residual row is loaded before the first store: R may alias C (in-place add into
    // the residual stream), so a load placed after a store could not be hoisted above it and
    // each (load, add, store) would pay a full memory round trip
    const int n = 256 * tn + 128 * wn + 8 * l16;
    bf16x8 rv[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = min(row0 + 128 * wm + 16 * i + 4 * g + r, mend - 1);
        rv[i][r] = *reinterpret_cast<const bf16x8*>(p.r + (int64_t)m * p.ldr + n);
      }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = row0 + 128 * wm + 16 * i + 4 * g + r;
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[i][j][r] + bf2f(rv[i][r][j]));
        if (m >= mend) continue;
        w4_st16<V>(cbase + (int64_t)m * p.ldc + n, o);
      }
  }
}

// Split-K: publish this slice's fp32 partial tile, draw a ticket; the last arriver adds every
// other slice's partials.  The slabs are written through (sc1 stores: no L2 write-back fence,
// cdna_hip_programming.md §5 'Projection GEMM at M = 256' item 2 and the MI355X hand-off
// table's counter row): every storing wave waits for its stores, a workgroup barrier, then
// ONE lane's agent-scope atomic add; the workgroup whose add returns splitk - 1 reads the
// other slabs with sc1 loads only (its other waves after the LDS flag + barrier).
DRTC_DEVICE bool w4_splitk(const W4Params& p, f32x4 (&acc)[8][8], int tile, int slice,
                           char* lds) {
  constexpr int kSc1 = 16;  // cache-policy bits of the buffer op: sc1
  const int tid = threadIdx.x;
  const int per_slice = 64 * kW4Threads * 16;  // bytes (256 KiB)
  const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(reinterpret_cast<char*>(p.slab) + (int64_t)tile * p.splitk * per_slice), (short)0,
      p.splitk * per_slice, 0x00020000);
  const int mine = slice * per_slice + tid * 16;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), slab,
                                             mine + (i * 8 + j) * kW4Threads * 16, 0, kSc1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(lds);
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == p.splitk - 1);
    if (last) __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return false;
  for (int s = 0; s < p.splitk; ++s) {
    if (s == slice) continue;
    const int src = s * per_slice + tid * 16;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] += __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(slab, src + (i * 8 + j) * kW4Threads * 16,
                                                         0, kSc1));
  }
  return true;
}

// Split-K, parallel combine (pcomb; every workgroup of the grid resident at once - the
// launcher checks grid <= CUs, one workgroup per CU by its LDS): each slice writes its fp32
// partial tile ROW-MAJOR [256][256] to its slab with write-through (sc1) stores, every
// storing wave drains (vmcnt(0)), a workgroup barrier, then ONE lane's agent-scope add to the
// tile's arrival counter and a bounded sc1 poll until all splitk slices arrived (the
// MI355X hand-off table's counter row: sc1 stores + drained waves + agent atomic, sc1 loads).
// Then slice s finishes rows [s 256/splitk, (s+1) 256/splitk) of the tile: 8 consecutive
// columns per thread, summed over the slabs in slice order (deterministic), and the epilogue
// (store / residual / gated activation).  The last slice to leave re-arms both counters.
// Per workgroup 256 KiB written and (splitk x 256/splitk rows) = 256 KiB read, in parallel
// on every CU - instead of one last arriver reading (splitk - 1) x 256 KiB alone.
template <int EPI, int V>
DRTC_DEVICE void w4_splitk_par(const W4Params& p, f32x4 (&acc)[8][8], int tile, int slice,
                               int tm, int tn, int wm, int wn, int l16, int g) {
  constexpr int kSc1 = 16;
  constexpr int kSlab = 256 * 256 * 4;  // one slice's row-major fp32 tile
  const int sk = p.splitk;
  const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(reinterpret_cast<char*>(p.slab) + (int64_t)tile * sk * kSlab), (short)0,
      sk * kSlab, 0x00020000);
  // my partial: row 128 wm + 16 i + 4 g + r, columns 128 wn + 8 l16 + j (j = 0..7)
  const int mine = slice * kSlab;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 128 * wm + 16 * i + 4 * g + r;
      const int off = mine + (row * 256 + 128 * wn + 8 * l16) * 4;
      f32x4 lo, hi;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lo[j] = acc[i][j][r];
        hi[j] = acc[i][j + 4][r];
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo), slab, off, 0, kSc1);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi), slab, off + 16, 0,
                                             kSc1);
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* arrive = p.counters + 2 * tile;
  int* depart = arrive + 1;
  __shared__ int faulted;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0, fault = 0;
    while (p.spin_limit < 0 ||
           __hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < sk) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > p.spin_limit) {  // a slice never arrived: give up (never hang the GPU)
        __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fault = 1;
        break;
      }
    }
    faulted = fault;
  }
  __syncthreads();
  const bool rearm = !faulted;  // after a fault the counters stay as they are (host resets)
  // my row band: thread t takes column chunk t & 31 (8 columns) of rows band0 + t / 32 + 8 k
  const int band = 256 / sk, band0 = slice * band;
  const int t = threadIdx.x, cc = t & 31;
#pragma unroll 1
  for (int rr = t >> 5; rr < band; rr += 8) {
    const int row = band0 + rr;
    f32x4 lo = (f32x4){0.f, 0.f, 0.f, 0.f}, hi = lo;
#pragma unroll 1
    for (int s2 = 0; s2 < sk; ++s2) {
      const int off = s2 * kSlab + (row * 256 + 8 * cc) * 4;
      lo += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(slab, off, 0, kSc1));
      hi += __builtin_bit_cast(f32x4,
                               __builtin_amdgcn_raw_buffer_load_b128(slab, off + 16, 0, kSc1));
    }
    const int m = 256 * tm + row;
    if (m >= p.M) continue;
    if constexpr (w4_glu<EPI>()) {
      // slab columns [8 c, 8 c + 8) of wave column half h = c / 16, lane l = c % 16: gate
      // columns 64 h + 4 l + (0..3), then the matching up columns
      const int n = 128 * tn + 64 * (cc >> 4) + 4 * (cc & 15);
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bf(act_value<w4_act<EPI>()>(lo[j]) * hi[j]);
      w4_st8<V>(p.c + (int64_t)m * p.ldc + n, o);
    } else {
      const int n = 256 * tn + 8 * cc;
      bf16x8 o;
      if constexpr (w4_res<EPI>()) {
        const bf16x8 rv = *reinterpret_cast<const bf16x8*>(p.r + (int64_t)m * p.ldr + n);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f2bf(lo[j] + bf2f(rv[j]));
          o[j + 4] = f2bf(hi[j] + bf2f(rv[j + 4]));
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f2bf(lo[j]);
          o[j + 4] = f2bf(hi[j]);
        }
      }
      w4_st16<V>(p.c + (int64_t)m * p.ldc + n, o);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && rearm) {
    const int d = __hip_atomic_fetch_add(depart, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == sk - 1) {  // every slice of the tile has read the slabs: re-arm
      __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(depart, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Tile coordinates of tile-order index tt within a tiles_m x tiles_n grid (row-grouped:
// group_m row tiles sweep the columns).
DRTC_DEVICE void w4_tile_mn(int tiles_m, int tiles_n, int group_m, int tt, int& tm, int& tn) {
  const int gsize = group_m * tiles_n;
  const int first_m = (tt / gsize) * group_m;
  const int gm = min(tiles_m - first_m, group_m);
  tm = first_m + (tt % gsize) % gm;
  tn = (tt % gsize) / gm;
}
DRTC_DEVICE void w4_tile_of(const W4Params& p, int tt, int& tm, int& tn) {
  w4_tile_mn(p.tiles_m, p.tiles_n, p.group_m, tt, tm, tn);
}

// Rows [r0, r1) of group e, clamped to [0, M] and to the previous group's end (prev, carried
// by the caller's walk over the groups): offsets written by another kernel can never make the
// launch touch rows outside the operands it was sized for, nor two groups write one row.
DRTC_DEVICE void w4_grp_rows(const W4Params& p, int e, int& prev, int& r0, int& r1) {
  r0 = max(min(max(p.grp[e], 0), p.M), prev);
  r1 = max(min(p.grp[e + 1], p.M), r0);
  prev = r1;
}

// Tiles of the launch: tiles_m x tiles_n, or (grouped) the sum over the row groups.
template <int V>
DRTC_DEVICE int w4_ntiles(const W4Params& p) {
  if constexpr ((V & 64) != 0) {
    int n = 0, prev = 0;
    for (int e = 0; e < p.n_grp; ++e) {
      int r0, r1;
      w4_grp_rows(p, e, prev, r0, r1);
      n += (r1 - r0 + 255) >> 8;
    }
    return n * p.tiles_n * p.ksplit;
  } else {
    return p.tiles_m * p.tiles_n;
  }
}

// Position of tile-order index tt (grouped: the groups' tiles one after another, each group
// in the row-grouped order of its own row tiles).
template <int V>
DRTC_DEVICE W4Pos w4_pos_of(const W4Params& p, int tt) {
  W4Pos q;
  if constexpr ((V & 64) != 0) {
    int base = 0, prev = 0;
    for (int e = 0; e < p.n_grp; ++e) {
      int r0, r1;
      w4_grp_rows(p, e, prev, r0, r1);
      const int tme = (r1 - r0 + 255) >> 8, ns = tme * p.tiles_n, nt = ns * p.ksplit;
      if (tt < base + nt) {
        const int s = (tt - base) / ns;  // K slice
        w4_tile_mn(tme, p.tiles_n, p.group_m, tt - base - s * ns, q.tm, q.tn);
        q.row0 = r0 + 256 * q.tm;
        q.mend = r1;
        q.b = p.b + (int64_t)e * p.b_grp;
        q.koff = s * p.kt_split * 64;
        q.c = p.c + (int64_t)s * p.c_split;
        return q;
      }
      base += nt;
    }
    q.tm = 0; q.tn = 0; q.row0 = 0; q.mend = 0; q.b = p.b;  // unreachable (tt < w4_ntiles)
    q.koff = 0; q.c = p.c;
    return q;
  } else {
    w4_tile_of(p, tt, q.tm, q.tn);
    return q;
  }
}

// DMA plan of tile (tm, tn) for this wave (operand bases, per-lane source offsets).
template <int EPI, int V>
DRTC_DEVICE void w4_plan(W4Dma& d, const W4Params& p, const W4Pos& q, int wv, int lane,
                         int k_base0, unsigned lds0) {
  const int k_base = k_base0 + w4_koff<V>(q);
  const int r8 = lane >> 3;
  const int tn = q.tn;
  const int chunk = (lane & 7) ^ ((4 * wv + (lane >> 4)) & 7);  // logical chunk of this lane
  const int row0 = w4_row0<V>(q);
  const int rows_a = min(256, w4_mend<V>(p, q) - row0);
  const bf16_t* abase = p.a + (int64_t)row0 * p.lda + k_base;
  d.na = (unsigned)(rows_a * p.lda * 2 - k_base * 2);
  d.ra = __builtin_amdgcn_make_buffer_rsrc((void*)abase, (short)0, (int)d.na, 0x00020000);
  // tile-independent lane offsets: rows past the tile's valid rows fall outside `na`
#pragma unroll
  for (int s = 0; s < 8; ++s)
    d.va[s] = (unsigned)((32 * s + 8 * wv + r8) * p.lda * 2 + chunk * 16);
  // B: fragment j of wave column half h reads LDS rows 128 h + 8 l + j (l = lane & 15),
  // so lane l16 of the MFMA output holds the 8 CONSECUTIVE columns 8 l16 .. 8 l16 + 7 over
  // j = 0..7 (16-B epilogue stores).  Plain tiles keep tile row = LDS row.  Gated tiles:
  // 64 output columns per half, LDS row 128 h + 8 l + j holds the gate row (j < 4) or the
  // up row (j >= 4) of column 64 h + 4 l + (j & 3): each DMA instruction (8 LDS rows) loads
  // 4 consecutive gate rows and the 4 matching up rows.  DMA instruction s of wave wv fills
  // LDS rows 32 s + 8 wv + r8: h = s >> 2, l = 4 (s & 3) + wv, j = r8.
  const bf16_t* bbase;
  int brow;
  if constexpr (w4_glu<EPI>()) {
    bbase = w4_bop<V>(p, q) + (int64_t)(128 * tn) * p.ldb + k_base;
    brow = 4 * wv + (r8 & 3) + (r8 >= 4 ? p.up_off : 0);
#pragma unroll
    for (int s = 0; s < 8; ++s)
      d.sb[s] = (unsigned)((64 * (s >> 2) + 16 * (s & 3)) * p.ldb * 2);
  } else {
    bbase = w4_bop<V>(p, q) + (int64_t)(256 * tn) * p.ldb + k_base;
    brow = 8 * wv + r8;
#pragma unroll
    for (int s = 0; s < 8; ++s) d.sb[s] = (unsigned)(32 * s * p.ldb * 2);
  }
  d.rb = __builtin_amdgcn_make_buffer_rsrc((void*)bbase, (short)0, 0x7FFFFFFF, 0x00020000);
  d.abase = reinterpret_cast<const char*>(abase);
  d.bbase = reinterpret_cast<const char*>(bbase);
  d.vb = (unsigned)(brow * p.ldb * 2 + (lane & 7) * 16);  // B: chunks in natural order
  d.lds_a = __builtin_amdgcn_readfirstlane(lds0 + 8 * wv * 128);
  d.lds_b = __builtin_amdgcn_readfirstlane(lds0 + kW4BOff + wv * kW4BBlk);
}

// Select of two DMA plans on a wave-uniform condition: only the operand bases and the valid-A
// extent depend on the tile (lane offsets, B row steps and LDS bases do not; the prologue-only
// descriptors are not used by the main loop), so the pick is scalar.
DRTC_DEVICE W4Dma w4_pick(bool first, const W4Dma& x, const W4Dma& y) {
  W4Dma r = x;
  r.abase = first ? x.abase : y.abase;
  r.bbase = first ? x.bbase : y.bbase;
  r.na = first ? x.na : y.na;
  return r;
}

// V & 8: persistent form (split-K 1 only).  min(tiles, CUs) workgroups walk the tile order
// (tile tt, tt + grid, ...), and the last two K steps of a tile DMA the NEXT tile's first two
// K tiles into the ring (and the last one reads its first fragments), so a tile seam costs the
// epilogue only: no workgroup launch, no prologue latency, no drain of the DMA ring.
template <int EPI, int V>
__global__ __launch_bounds__(kW4Threads, 1) void gemm_w4_kernel(W4Params p) {
  extern __shared__ __attribute__((aligned(16))) char w4_lds[];
  constexpr bool kPers = (V & 8) != 0;
  // ---- tile assignment: XCD remap (bijective), split-K slice fastest, grouped rows
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, qq = nwg >> 3, rmd = nwg & 7;
  const int wgid = (xcd < rmd ? xcd * (qq + 1) : rmd * (qq + 1) + (xcd - rmd) * qq) + (orig >> 3);
  int slice = kPers ? 0 : wgid % p.splitk;
  int tt = kPers ? wgid : wgid / p.splitk;
  if (!kPers && p.xk) {
    // K-slice-by-XCD order (split-K decode shapes): the 8 block labels b % 8 (one XCD each
    // under round-robin dispatch - speed only, the map is a bijection of blockIdx) split into
    // splitk slices x (8 / splitk) tile subsets, so an XCD's 32 workgroups stream ONE K slice
    // of a compact block of tiles: its L2 holds a quarter of the operand panels the
    // tile-major order needs.  Host contract: splitk | 8, nwg % 8 == 0, ntiles % (8/splitk) == 0.
    const int per = nwg >> 3;
    slice = xcd % p.splitk;
    tt = (xcd / p.splitk) * per + (orig >> 3);
  }
  const int ntiles = w4_ntiles<V>(p);
  if constexpr ((V & 64) != 0) {
    // grouped: the grid is sized for the most tiles the rows can make (whole workgroups leave
    // before any DMA when the groups' actual tiles are fewer)
    if (tt >= ntiles) return;
  }
  W4Pos q = w4_pos_of<V>(p, tt);
  const int tm = q.tm, tn = q.tn;

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wv >> 1, wn = wv & 1, l16 = lane & 15, g = lane >> 4;
  const int k_base = slice * p.kt_split * 64;
  const int nk = p.kt_split;

  // ---- DMA plan
  W4Dma d;
  const unsigned lds0 = (unsigned)(uintptr_t)(w4_lds_ptr)w4_lds;
  w4_plan<EPI, V>(d, p, q, wv, lane, k_base, lds0);
  // fragment read offsets (bytes within a stage): row 128 w + l16 (+ 16 per fragment), the
  // 16-B chunk 4 h + g stored at chunk ^ ((row >> 1) & 7)
  const int fx = (l16 >> 1) & 7;
  const int ra0 = (128 * wm + l16) * 128 + ((0 + g) ^ fx) * 16;
  const int ra1 = (128 * wm + l16) * 128 + ((4 + g) ^ fx) * 16;
  // B: block 16 wn + l16 of the padded image, row j in it (+128 j), chunk 4 h + g
  const int rb0 = kW4BOff + (16 * wn + l16) * kW4BBlk + g * 16;
  const int rb1 = rb0 + 64;
  const char* lds = w4_lds;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // K tiles may run in a rotated order kst, kst + 1, ... (mod nk).  V & 16 (persistent form):
  // each XCD label b % 8 starts at its own eighth of K, so the eight XCDs reach their tile
  // seams (the epilogue's store burst, 4 MiB per XCD) at different times while the 32
  // workgroups of one XCD still stream the same K tile through its L2 in lockstep.
  // (p.krot < 8 gives XCD labels b % 8 in groups of 8 / krot one offset: w4_set_krot)
  const int kst = (V & 16) ? ((((orig & 7) * p.krot) >> 3) * nk) / p.krot : 0;
  const unsigned k0b = (unsigned)kst * 128u, k1b = (unsigned)(kst + 1 < nk ? kst + 1 : 0) * 128u;
  // ---- prologue: tiles 0 and 1 into stages 0 and 1
#pragma unroll
  for (int s = 0; s < 8; ++s) w4_dma(d.lds_b + 4 * kW4BBlk * s, d.vb, d.rb, k0b + d.sb[s]);
#pragma unroll
  for (int s = 0; s < 8; ++s) w4_dma(d.lds_a + 4096 * s, d.va[s], d.ra, k0b);
  if (nk > 1) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
      w4_dma(d.lds_b + kW4Stage + 4 * kW4BBlk * s, d.vb, d.rb, k1b + d.sb[s]);
#pragma unroll
    for (int s = 0; s < 8; ++s) w4_dma(d.lds_a + kW4Stage + 4096 * s, d.va[s], d.ra, k1b);
    w4_vmcnt<16>();
  } else {
    w4_vmcnt<0>();
  }
  w4_barrier();
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  fa0[0] = w4_rd(lds, ra0);
#pragma unroll
  for (int j = 0; j < 8; ++j) fb0[j] = w4_rd(lds, rb0 + 128 * j);
#pragma unroll
  for (int i = 1; i < 8; ++i) fa0[i] = w4_rd(lds, ra0 + 2048 * i);

  if constexpr (kPers) {
    // the persistent seam needs two K tiles per tile (the next tile's pair is staged by
    // this tile's last two steps); the launcher guarantees nk >= 2
    int par = 0;  // stage parity of this tile's K step 0 (flips after an odd nk)
    // exactly 32 store instructions per wave in a full tile's epilogue (one per row fragment
    // i and row r; STORE / RESIDUAL 16 B, GLU 8 B): checked in the disassembly
    constexpr bool kSeamOk = EPI == W4_STORE || EPI == W4_RESIDUAL || EPI == W4_SILU || EPI == W4_GELU;
    bool seam = false;
    for (;;) {
      const int tnext = tt + nwg;
      const bool more = tnext < ntiles;
      W4Pos q2 = q;
      if (more) q2 = w4_pos_of<V>(p, tnext);
      W4Dma dn;
      w4_plan<EPI, V>(dn, p, q2, wv, lane, 0, lds0);
      // K step t + 2 of this tile, or step t + 2 - nk of the next one; the very last tile
      // re-stages its final K tile (valid bytes, never read) as the plain form does.  Step 0
      // starts the accumulators from 0 (MFMA with a zero C operand: no separate zeroing of the
      // 256 AGPRs, which hipcc would hoist above the previous tile's epilogue and spill).
      {
        int t2 = 2 < nk ? 2 : (more ? 2 - nk : nk - 1);
        t2 += kst;
        t2 -= t2 >= nk ? nk : 0;
        const W4Dma dd = w4_pick(2 < nk || !more, d, dn);
        w4_tile<V, true, true, true>(acc, fa0, fb0, fa1, fb1, lds, (par & 1) * kW4Stage, ra0, ra1,
                                     rb0, rb1, dd, t2, seam);
      }
      for (int t = 1; t < nk; ++t) {
        const bool own = t + 2 < nk;
        int t2 = own ? t + 2 : (more ? t + 2 - nk : nk - 1);
        t2 += kst;
        t2 -= t2 >= nk ? nk : 0;
        const W4Dma dd = w4_pick(own || !more, d, dn);
        w4_tile<V, true, true>(acc, fa0, fb0, fa1, fb1, lds, ((t + par) & 1) * kW4Stage, ra0, ra1,
                               rb0, rb1, dd, t2);
      }
      // one epilogue call site (two would make hipcc copy all 256 accumulators out of the
      // AGPRs ahead of the branch between them, and spill)
      if (!more) w4_vmcnt<0>();  // no LDS-DMA may still be landing when the workgroup leaves
      // the lane index re-derived here (opaque to hipcc): kept live across the K loop it is
      // spilled, and its reload's vmcnt(0) would wait for the next tile's DMA
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      w4_epilogue<EPI, V>(p, w4_cop<V>(p, q), acc, w4_row0<V>(q), w4_mend<V>(p, q), q.tn, wm, wn,
                          ln & 15, ln >> 4, 0);
      if (!more) break;
      seam = kSeamOk && w4_row0<V>(q) + 256 <= w4_mend<V>(p, q);
      par ^= nk & 1;
      tt = tnext;
      q = q2;
      d = dn;
    }
    return;
  }

  // One loop body for every tile (a single straight-line schedule keeps the 256 accumulators
  // in place in the AGPRs): the last two tiles re-stage the final tile (kb clamped: valid
  // bytes, never read) and the last one reads stale fragments it never uses.
  for (int t = 0; t < nk; ++t) {
    int t2 = min(t + 2, nk - 1) + kst;
    t2 -= t2 >= nk ? nk : 0;
    w4_tile<V, true, true>(acc, fa0, fb0, fa1, fb1, lds, (t & 1) * kW4Stage, ra0, ra1, rb0, rb1, d,
                           t2);
  }
  w4_vmcnt<0>();  // no LDS-DMA may still be landing when the workgroup leaves

  if constexpr ((V & 4) != 0) {  // the launcher guarantees splitk > 1: one epilogue site
    w4_splitk_par<EPI, V>(p, acc, tm * p.tiles_n + tn, slice, tm, tn, wm, wn, l16, g);
    return;
  } else if (p.splitk > 1) {
    __syncthreads();
    if (!w4_splitk(p, acc, tm * p.tiles_n + tn, slice, w4_lds)) return;
  }
  w4_epilogue<EPI, V>(p, p.c, acc, 256 * tm, p.M, tn, wm, wn, l16, g, slice);
}

template <int EPI, int V>
int w4_launch_v(const W4Params& p, hipStream_t st) {
  int nwg = p.tiles_m * p.tiles_n * p.splitk;
  if constexpr ((V & 8) != 0) nwg = min(nwg, w4_num_cus());
  if constexpr ((V & 16) != 0) nwg -= nwg & 7;  // whole XCD rounds (>= 8: launcher contract)
  hipLaunchKernelGGL((gemm_w4_kernel<EPI, V>), dim3(nwg), dim3(kW4Threads), kW4Lds, st, p);
  return (int)hipGetLastError();
}

// schedule variants built: 0 per-tile (split-K capable: last-arriver combine), 2 the same
// with temporal stores, 4 / 6 per-tile with the parallel split-K combine, 8 persistent, 24
// persistent with the per-XCD K rotation
template <int EPI>
int w4_launch(const W4Params& p, int v, hipStream_t st) {
  switch (v) {
    case 0: return w4_launch_v<EPI, 0>(p, st);
    case 2: return w4_launch_v<EPI, 2>(p, st);
    case 4: return w4_launch_v<EPI, 4>(p, st);
    case 6: return w4_launch_v<EPI, 6>(p, st);
    case 8: return w4_launch_v<EPI, 8>(p, st);
    case 24: return w4_launch_v<EPI, 24>(p, st);
    case 40: return w4_launch_v<EPI, 40>(p, st);
    case 56: return w4_launch_v<EPI, 56>(p, st);
    default: return -1;
  }
}

// grouped persistent form (V & 64 on schedule 40: spread fragment reads, NO per-XCD K
// rotation): store and gated epilogues.  The routing kernel places a pair's row within its
// expert's group by an atomic ticket, so a row's tile - and with the rotation its workgroup's
// K start - would vary run to run; without it every tile sums K in the same order and the
// layer is deterministic.
// (w4_set_grouped_rot(1): schedule 56 + 64, with the rotation - an A/B arm, not deterministic)
static int g_w4_grouped_rot = 0;
template <int EPI>
int w4_launch_grouped(const W4Params& p, int nwg, hipStream_t st) {
  if (g_w4_grouped_rot)
    hipLaunchKernelGGL((gemm_w4_kernel<EPI, 120>), dim3(nwg), dim3(kW4Threads), kW4Lds, st, p);
  else
    hipLaunchKernelGGL((gemm_w4_kernel<EPI, 104>), dim3(nwg), dim3(kW4Threads), kW4Lds, st, p);
  return (int)hipGetLastError();
}

template <int EPI, int V>
int w4_cfg_one() {
  return (int)hipFuncSetAttribute((const void*)gemm_w4_kernel<EPI, V>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kW4Lds);
}
template <int EPI>
int w4_cfg() {
  return w4_cfg_one<EPI, 0>() | w4_cfg_one<EPI, 2>() | w4_cfg_one<EPI, 4>() |
         w4_cfg_one<EPI, 6>() | w4_cfg_one<EPI, 8>() | w4_cfg_one<EPI, 24>() |
         w4_cfg_one<EPI, 40>() | w4_cfg_one<EPI, 56>();
}

}  // namespace

static int g_w4_krot = 8;
void w4_set_grouped_rot(int r) { g_w4_grouped_rot = r != 0; }
void w4_set_krot(int k) { g_w4_krot = (k == 1 || k == 2 || k == 4) ? k : 8; }
int w4_krot() { return g_w4_krot; }

int w4_num_cus() {
  static int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return cus;
  }();
  return n;
}

int launch_gemm_w4(void* c, const void* a, const void* b, const void* r, int M, int N, int K,
                   int lda, int ldb, int ldc, int ldr, int epi, int up_off, int splitk,
                   int group_m, void* slab, int64_t slab_bytes, int* counters, int n_counters,
                   int v, hipStream_t st) {
  // shape contract (checked here so a bad call never reaches the device)
  const bool glu = epi == W4_SILU || epi == W4_GELU;
  const bool res = epi == W4_RESIDUAL;
  if (epi < W4_STORE || epi > W4_GELU) return -1;
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || splitk < 1 || (K / 64) % splitk) return -1;
  if (glu ? (N % 128 || up_off != N) : (N % 256)) return -1;
  // persistent form (v & 8): one slice, and two K tiles per tile for the cross-tile prefetch
  if ((v & 8) && ((v != 8 && v != 24 && v != 40 && v != 56) || splitk != 1 || K / 64 < 2))
    return -1;
  if ((v & 4) && splitk < 2) return -1;  // the parallel combine is a split-K form
  // the per-XCD K rotation needs whole XCD rounds of workgroups: below 8 tiles, plain persistent
  if ((v & 16) && (int64_t)((M + 255) / 256) * (glu ? N / 128 : N / 256) < 8) v &= ~16;
  if (lda % 8 || ldb % 8 || (glu ? ldc % 4 : ldc % 8)) return -1;
  if (res && (ldr % 8 || r == nullptr || (uintptr_t)r % 16)) return -1;
  if ((uintptr_t)a % 16 || (uintptr_t)b % 16 || (uintptr_t)c % (glu ? 8 : 16)) return -1;
  // 32-bit buffer offsets: every staged row must sit within 2 GiB of its operand base
  if ((int64_t)min(M, 256) * lda * 2 >= (1ll << 31)) return -1;
  if ((int64_t)(glu ? up_off + 128 : 256) * ldb * 2 >= (1ll << 31)) return -1;
  // group_m < 0: K-slice-by-XCD order with row groups of -group_m (split-K forms only)
  const bool xk = group_m < 0;
  if (xk) group_m = -group_m;
  if (group_m < 1) group_m = 8;
  W4Params p{};
  p.c = (bf16_t*)c;
  p.a = (const bf16_t*)a;
  p.b = (const bf16_t*)b;
  p.r = (const bf16_t*)r;
  p.M = M; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldr = ldr;
  p.tiles_m = (M + 255) / 256;
  p.tiles_n = glu ? N / 128 : N / 256;
  p.splitk = splitk;
  p.kt_split = K / 64 / splitk;
  p.up_off = up_off;
  p.group_m = group_m;
  p.krot = g_w4_krot;
  if (xk) {
    const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
    if ((v & 8) || 8 % splitk || (tiles * splitk) % 8 || tiles % (8 / splitk)) return -1;
    p.xk = 1;
  }
  if (splitk > 1) {
    const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
    // tile counters [0, 2 tiles) and the error word at the workspace's last slot
    if (slab == nullptr || counters == nullptr || n_counters < 2 * tiles + 2 ||
        slab_bytes < tiles * splitk * 64ll * kW4Threads * 16)
      return -2;
    p.err = counters + n_counters - 1;
    p.spin_limit = splitk_spin_limit();
    // parallel combine: slices wait for each other, so every workgroup must be resident at
    // once (one per CU: the LDS ring) and a row band per slice (splitk | 256)
    if ((v & 4) && (256 % splitk || tiles * splitk > w4_num_cus())) return -1;
    p.slab = (float*)slab;
    p.counters = counters;
  }
  switch (epi) {
    case W4_STORE: return w4_launch<W4_STORE>(p, v, st);
    case W4_RESIDUAL: return w4_launch<W4_RESIDUAL>(p, v, st);
    case W4_SILU: return w4_launch<W4_SILU>(p, v, st);
    default: return w4_launch<W4_GELU>(p, v, st);
  }
}

// Grouped persistent GEMM: for g < n_grp, C[r] = epi(A[r] . B_g^T) over the rows r in
// [grp[g], grp[g + 1]) with B_g = b + g * b_grp elements (the experts of a MoE layer over
// expert-ordered rows).  grp is a DEVICE array (n_grp + 1 non-decreasing row offsets, the last
// <= max_rows): the routing kernel writes it and the launch reads it with no host sync, so the
// layer stays hipGraph-capturable.  The grid is min(CUs, tiles of max_rows rows spread over
// n_grp groups); workgroups past the actual tile count leave at once.
int launch_gemm_w4_grouped(void* c, const void* a, const void* b, const int* grp, int n_grp,
                           int max_rows, int N, int K, int lda, int ldb, int ldc, int64_t b_grp,
                           int epi, int up_off, int group_m, int ksplit, int64_t c_split,
                           hipStream_t st) {
  const bool glu = epi == W4_SILU || epi == W4_GELU;
  if (epi != W4_STORE && !glu) return -1;
  if (ksplit < 1 || (glu && ksplit != 1)) return -1;  // a gated epilogue cannot be split
  if (grp == nullptr || n_grp < 1 || max_rows < 1 || K % 64 || (K / 64) % ksplit ||
      K / 64 / ksplit < 2)
    return -1;
  if (ksplit > 1 && (c_split % 8 || (int64_t)max_rows * ldc > c_split)) return -1;
  if (glu ? (N % 128 || up_off != N) : (N % 256)) return -1;
  if (lda % 8 || ldb % 8 || (glu ? ldc % 4 : ldc % 8)) return -1;
  if ((uintptr_t)a % 16 || (uintptr_t)b % 16 || (uintptr_t)c % (glu ? 8 : 16)) return -1;
  if ((int64_t)256 * lda * 2 >= (1ll << 31)) return -1;
  if ((int64_t)(glu ? up_off + 128 : 256) * ldb * 2 >= (1ll << 31)) return -1;
  W4Params p{};
  p.c = (bf16_t*)c;
  p.a = (const bf16_t*)a;
  p.b = (const bf16_t*)b;
  p.M = max_rows; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.tiles_m = (max_rows + 255) / 256;
  p.tiles_n = glu ? N / 128 : N / 256;
  p.splitk = 1;
  p.kt_split = K / 64 / ksplit;
  p.up_off = up_off;
  p.group_m = group_m < 1 ? 8 : group_m;
  p.krot = g_w4_krot;
  p.grp = grp;
  p.n_grp = n_grp;
  p.b_grp = b_grp;
  p.ksplit = ksplit;
  p.c_split = c_split;
  // the most row tiles n_grp groups of max_rows rows in total can make
  const int64_t tiles = (int64_t)(p.tiles_m + n_grp - 1) * p.tiles_n * ksplit;
  int nwg = (int)(tiles < w4_num_cus() ? tiles : w4_num_cus());
  nwg -= nwg & 7;  // whole XCD rounds; surplus workgroups leave at once
  if (nwg < 8) nwg = 8;
  switch (epi) {
    case W4_STORE: return w4_launch_grouped<W4_STORE>(p, nwg, st);
    case W4_SILU: return w4_launch_grouped<W4_SILU>(p, nwg, st);
    default: return w4_launch_grouped<W4_GELU>(p, nwg, st);
  }
}

int64_t gemm_w4_workspace_bytes(int64_t M, int64_t N, int splitk) {
  // fp32 split-K slabs: 256 KiB per 256 x 256 tile and slice
  return splitk > 1 ? ((M + 255) / 256) * (N / 256) * splitk * 64ll * kW4Threads * 16 : 0;
}

int configure_gemm_w4() {
  return w4_cfg<W4_STORE>() | w4_cfg<W4_RESIDUAL>() | w4_cfg<W4_SILU>() | w4_cfg<W4_GELU>() |
         w4_cfg_one<W4_STORE, 104>() | w4_cfg_one<W4_SILU, 104>() | w4_cfg_one<W4_GELU, 104>() |
         w4_cfg_one<W4_STORE, 120>() | w4_cfg_one<W4_SILU, 120>() | w4_cfg_one<W4_GELU, 120>();
}

}  // namespace drtc
