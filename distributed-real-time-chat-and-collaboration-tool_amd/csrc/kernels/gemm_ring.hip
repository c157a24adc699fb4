// Ring-pipelined 4-wave CDNA4 (gfx950) bf16 GEMM, persistent:
//
//   C[M, N] = epi( A[M, K] . B[N, K]^T )      (A activations, B weights, both K-contiguous)
//
// epilogues: store / + residual (may alias C) / SiLU- or GELU-gated [gate; up].  The prefill
// projections of ref llm_server/llm_server.py:231 / :287's on-node replacement.
//
// Why a second 256 x 256 kernel next to gemm_w4: gemm_w4 (and hipBLASLt's MT256x256x64 kernel,
// whose loop it resembles) stage 64-deep K tiles in a 2-slot LDS ring - one tile in flight -
// and need THREE barriers per tile (B region free, A region free, next tile landed).  With one
// wave per SIMD every barrier skew and every LDS-issue stall is lost MFMA time (profiles/r4j:
// gemm_w4 +68 % SQ_WAIT_ANY, +72 % SQ_WAIT_INST_LDS against the library).  This kernel stages
// 32-deep K stages in a 4-slot ring (4 x 32.5 KiB):
//
//   * iteration t consumes stage t % 4, whose fragments are ALREADY in registers (read during
//     iteration t - 1), so that slot is free at once: the LDS-DMA of stage t + 4 goes into it
//     during iteration t.  Three stages are in flight (96 KiB per CU), each with 2-3 iterations
//     of latency slack (~1.0-1.5 us) instead of ~1 tile.
//   * ONE barrier per iteration (64 MFMAs): after it every wave's stage t + 2 has landed (its own
//     vmcnt first) and every wave's reads of stage t + 1 are done (lgkmcnt(0)).
//   * Per iteration and wave a fixed order pinned with sched_barrier: 64 MFMA 16x16x32 (8 x 8
//     fragments, 128 x 128 outputs, 256 accumulators), 16 ds_read_b128 of the next stage's
//     fragments (one per 3 MFMAs, Q = 2..47) into the other register set, 8 LDS-DMA of stage
//     t + 4 (one per 6 MFMAs, Q = 1..43), then vmcnt / lgkmcnt / barrier at Q = 63.
//   * LDS images (bytes within a stage), conflict-free for the 4 lane groups of ds_read_b128
//     (checked exhaustively): A 256 rows x 64 B, 16-B chunk c of row r at c ^ (-(r >> 2) & 3);
//     B 16 blocks of 16 rows x 64 B + 32 B of padding (1056-B blocks), chunk c of row q at
//     c ^ ((q >> 3) & 1).  Every DMA wave-instruction loads 16 CONSECUTIVE weight rows (gated:
//     8 consecutive gate rows and their 8 up rows) into one block.
//   * B fragment j, lane row l reads weight row 8 l + j of the wave's 128-row panel, so a lane's
//     accumulators over the 8 B fragments are 8 consecutive output columns: the epilogue stores
//     16 B per lane straight from the accumulators (4 rows x 256 contiguous bytes per
//     instruction); a gated tile pairs gate fragment j with up fragment j + 4 in a lane.
//   * Persistent: min(tiles, CUs) workgroups walk the XCD-aware, row-grouped tile order; the
//     DMA stream runs across tile seams (the last 4 iterations of a tile load the next tile's
//     first 4 stages), so a seam costs the epilogue's stores only.
//
// Contract (launch_gemm_ring): K % 128 == 0 and K >= 256 (a tile is a whole number of 4-stage
// ring trips, >= 2), N % 256 == 0 (gated: N % 128 == 0, up_off == N), 16-B aligned operands.
#include "common.h"
#include "launchers.h"

#include <utility>

namespace drtc {
int w4_num_cus();
namespace {

typedef __attribute__((address_space(3))) void* rg_lds_ptr;

constexpr int kRgThreads = 256;
constexpr int kRgA = 256 * 64;                 // A image: 256 rows x 64 B (32 K values)
constexpr int kRgBBlk = 1056;                  // B: 16-row block = 1 KiB + 32 B padding
constexpr int kRgStage = kRgA + 16 * kRgBBlk;  // 33280
constexpr int kRgLds = 4 * kRgStage;           // 133120: the 4-slot ring

enum { RG_STORE = 0, RG_RESIDUAL = 1, RG_SILU = 2, RG_GELU = 3 };
template <int EPI>
DRTC_DEVICE constexpr bool rg_glu() { return EPI == RG_SILU || EPI == RG_GELU; }

struct RgParams {
  bf16_t* c;
  const bf16_t* a;
  const bf16_t* b;
  const bf16_t* r;
  int M, N, K;  // N = columns of C
  int lda, ldb, ldc, ldr;
  int tiles_m, tiles_n, group_m;
  int up_off;
  int nk;  // 32-deep K stages per tile (a multiple of 4, >= 8)
};

// Operand panels of one tile (the DMA stream's only tile-dependent state).
struct RgPlan {
  const char* abase;  // A rows [256 tm, +256), k = 0
  const char* bbase;  // B rows of tile column tn (gated: gate rows; up rows at + up_off)
  unsigned na;        // valid A bytes from abase: DMA rows past M fall outside (read as 0)
};

// Tile-independent DMA lanes and LDS bases of this wave.
struct RgLanes {
  unsigned va[4], vb[4];  // per-lane source offsets of the wave's 4 A / 4 B instructions
  unsigned lds_a, lds_b;  // LDS byte address of its first A / B block in stage 0
};

template <int N>
DRTC_DEVICE void rg_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
  __builtin_amdgcn_s_waitcnt(imm);
}
DRTC_DEVICE void rg_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
DRTC_DEVICE void rg_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
DRTC_DEVICE bf16x8 rg_rd(const char* lds, int off) {
  return *reinterpret_cast<const bf16x8*>(lds + off);
}

DRTC_DEVICE __amdgpu_buffer_rsrc_t rg_rsrc(const char* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

// Tile coordinates of tile-order index tt (row-grouped: group_m row tiles sweep the columns).
DRTC_DEVICE void rg_tile_of(const RgParams& p, int tt, int& tm, int& tn) {
  const int gsize = p.group_m * p.tiles_n;
  const int first_m = (tt / gsize) * p.group_m;
  const int gm = min(p.tiles_m - first_m, p.group_m);
  tm = first_m + (tt % gsize) % gm;
  tn = (tt % gsize) / gm;
}

template <int EPI>
DRTC_DEVICE RgPlan rg_plan(const RgParams& p, int tm, int tn) {
  RgPlan P;
  const int rows_a = min(256, p.M - 256 * tm);
  P.abase = reinterpret_cast<const char*>(p.a + (int64_t)(256 * tm) * p.lda);
  P.na = (unsigned)(rows_a * p.lda * 2);
  P.bbase = reinterpret_cast<const char*>(p.b + (int64_t)((rg_glu<EPI>() ? 128 : 256) * tn) *
                                                    p.ldb);
  return P;
}

template <int EPI>
DRTC_DEVICE void rg_lanes(RgLanes& L, const RgParams& p, int wv, int lane, unsigned lds0) {
  // A instruction s: LDS rows 64 wv + 16 s + (lane >> 2), stored chunk lane & 3 <- source
  // chunk (lane & 3) ^ (-(row >> 2) & 3), (row >> 2) & 3 = lane >> 4
  const int ca = (lane & 3) ^ ((4 - (lane >> 4)) & 3);
#pragma unroll
  for (int s = 0; s < 4; ++s)
    L.va[s] = (unsigned)((64 * wv + 16 * s + (lane >> 2)) * p.lda * 2 + ca * 16);
  // B instruction s fills block 4 wv + s (panel h = block >> 3, block d = block & 7 of it),
  // slot row q = lane >> 2: panel weight-row index w = 16 d + q; stored chunk lane & 3 <- source
  // chunk (lane & 3) ^ ((q >> 3) & 1)
  const int q = lane >> 2;
  const int cb = (lane & 3) ^ ((q >> 3) & 1);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int blk = 4 * wv + s, h = blk >> 3, d = blk & 7;
    int row;
    if constexpr (rg_glu<EPI>()) {
      // w = 8 l + j: gate (j < 4) or up (j >= 4) row of output column 64 h + 4 l + (j & 3)
      const int w = 16 * d + q, l = w >> 3, j = w & 7;
      row = (j < 4 ? 0 : p.up_off) + 64 * h + 4 * l + (j & 3);
    } else {
      row = 128 * h + 16 * d + q;
    }
    L.vb[s] = (unsigned)(row * p.ldb * 2 + cb * 16);
  }
  L.lds_a = __builtin_amdgcn_readfirstlane(lds0 + 4096 * wv);
  L.lds_b = __builtin_amdgcn_readfirstlane(lds0 + kRgA + 4 * kRgBBlk * wv);
}

// Step Q (0..63) of iteration U (stage U of the ring): MFMA Q on the current fragment set, then
// the memory work scheduled behind it.  Every condition is a compile-time constant except the
// seam test of the wait; sched_barrier(0) pins the emitted order.
//   W 0: end wait vmcnt(16) (stages t + 3, t + 4 may be in flight); W 1: vmcnt(48) after a
//   tile seam (the previous tile's 32 epilogue stores sit between) else 16.
template <int U, int W, bool Z, bool NR, int Q>
DRTC_DEVICE void rg_step(f32x4 (&acc)[8][8], const bf16x8 (&fac)[8], const bf16x8 (&fbc)[8],
                         bf16x8 (&fan)[8], bf16x8 (&fbn)[8], const char* lds, int ra, int rb,
                         const RgLanes& L, __amdgpu_buffer_rsrc_t rak,
                         __amdgpu_buffer_rsrc_t rbk, bool seam) {
  constexpr int i = Q >> 3, j = Q & 7;
  if constexpr (Z)  // first iteration of a tile: accumulate onto 0
    acc[i][j] = mfma16(fac[i], fbc[j], (f32x4){0.f, 0.f, 0.f, 0.f});
  else
    acc[i][j] = mfma16(fac[i], fbc[j], acc[i][j]);
  constexpr int cur = U * kRgStage, nxt = ((U + 1) & 3) * kRgStage;
  // ---- LDS-DMA of stage t + 4 into slot U: 4 A instructions, then 4 B, at Q = 1 + 6 s
  if constexpr (Q == 0) asm volatile("s_mov_b32 m0, %0" : : "s"(L.lds_a + cur) : "memory");
  if constexpr (Q >= 1 && (Q - 1) % 6 == 0 && (Q - 1) / 6 < 8) {
    constexpr int s = (Q - 1) / 6;
    if constexpr (s < 4) {
      asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" : : "v"(L.va[s]), "s"(rak) : "memory");
      if constexpr (s < 3)
        asm volatile("s_add_u32 m0, m0, 0x400" ::: "memory");
      else
        asm volatile("s_mov_b32 m0, %0" : : "s"(L.lds_b + cur) : "memory");
    } else {
      asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds"
                   : : "v"(L.vb[s - 4]), "s"(rbk) : "memory");
      if constexpr (s < 7) asm volatile("s_add_u32 m0, m0, 0x420" ::: "memory");
    }
  }
  // ---- the next stage's fragments (slot U + 1): fa[0], fb[0..7], fa[1..7] at Q = 2 + 3 r
  // (NR: not here - read after the epilogue, rg_late_reads)
  if constexpr (!NR && Q >= 2 && (Q - 2) % 3 == 0 && (Q - 2) / 3 < 16) {
    constexpr int r = (Q - 2) / 3;
    if constexpr (r == 0)
      fan[0] = rg_rd(lds, nxt + ra);
    else if constexpr (r <= 8)
      fbn[r - 1] = rg_rd(lds, nxt + rb + 64 * (r - 1));
    else
      fan[r - 8] = rg_rd(lds, nxt + ra + 1024 * (r - 8));
  }
  // ---- stage t + 2 landed for every wave, every read of slot U + 1 done
  if constexpr (Q == 63) {
    if constexpr (W == 1) {
      if (seam)
        rg_vmcnt<48>();
      else
        rg_vmcnt<16>();
    } else {
      rg_vmcnt<16>();
    }
    rg_lgkm0();
    rg_barrier();
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int U, int W, bool Z, bool NR, int... Qs>
DRTC_DEVICE void rg_steps(std::integer_sequence<int, Qs...>, f32x4 (&acc)[8][8],
                          const bf16x8 (&fac)[8], const bf16x8 (&fbc)[8], bf16x8 (&fan)[8],
                          bf16x8 (&fbn)[8], const char* lds, int ra, int rb, const RgLanes& L,
                          __amdgpu_buffer_rsrc_t rak, __amdgpu_buffer_rsrc_t rbk, bool seam) {
  (rg_step<U, W, Z, NR, Qs>(acc, fac, fbc, fan, fbn, lds, ra, rb, L, rak, rbk, seam), ...);
}

// One iteration: stage U consumed (fragments in fac / fbc), stage t + 4 of plan P at K byte
// offset kb DMA'd into slot U.
template <int U, int W, bool Z, bool NR = false>
DRTC_DEVICE void rg_iter(f32x4 (&acc)[8][8], const bf16x8 (&fac)[8], const bf16x8 (&fbc)[8],
                         bf16x8 (&fan)[8], bf16x8 (&fbn)[8], const char* lds, int ra, int rb,
                         const RgLanes& L, const RgPlan& P, unsigned kb, bool seam) {
  const __amdgpu_buffer_rsrc_t rak = rg_rsrc(P.abase + kb, P.na - kb);
  const __amdgpu_buffer_rsrc_t rbk = rg_rsrc(P.bbase + kb, 0x7FFFFFFFu);
  rg_steps<U, W, Z, NR>(std::make_integer_sequence<int, 64>{}, acc, fac, fbc, fan, fbn, lds, ra, rb,
                    L, rak, rbk, seam);
}

// One ring trip = 4 iterations (slots 0..3, register sets X, Y, X, Y).  FIRST: the tile's
// first trip (iteration 0 accumulates onto 0, iterations 0 and 1 wait past a seam's stores).
// The trip DMAs stages kb0 / 64 + 4 .. + 7 of plan P (kb0 = K byte offset of its slot-0 stage).
// NR: the trip's last iteration does not read the next stage's fragments (a residual tile's
// epilogue needs their 64 registers; rg_late_reads reads them after it).
template <bool FIRST, bool NR = false>
DRTC_DEVICE void rg_trip(f32x4 (&acc)[8][8], bf16x8 (&xa)[8], bf16x8 (&xb)[8], bf16x8 (&ya)[8],
                         bf16x8 (&yb)[8], const char* lds, int ra, int rb, const RgLanes& L,
                         const RgPlan& P, unsigned kb0, bool seam) {
  rg_iter<0, FIRST ? 1 : 0, FIRST>(acc, xa, xb, ya, yb, lds, ra, rb, L, P, kb0, seam);
  rg_iter<1, FIRST ? 1 : 0, false>(acc, ya, yb, xa, xb, lds, ra, rb, L, P, kb0 + 64u, seam);
  rg_iter<2, 0, false>(acc, xa, xb, ya, yb, lds, ra, rb, L, P, kb0 + 128u, seam);
  rg_iter<3, 0, false, NR>(acc, ya, yb, xa, xb, lds, ra, rb, L, P, kb0 + 192u, seam);
}

// Fragments of slot 0 into set X, then a barrier: every wave's reads of slot 0 precede any
// wave's LDS-DMA into it (iteration 0 of the next tile).
DRTC_DEVICE void rg_late_reads(bf16x8 (&xa)[8], bf16x8 (&xb)[8], const char* lds, int ra,
                               int rb) {
  xa[0] = rg_rd(lds, ra);
#pragma unroll
  for (int j = 0; j < 8; ++j) xb[j] = rg_rd(lds, rb + 64 * j);
#pragma unroll
  for (int i = 1; i < 8; ++i) xa[i] = rg_rd(lds, ra + 1024 * i);
  rg_lgkm0();
  rg_barrier();
}

template <int EPI>
DRTC_DEVICE void rg_st(bf16_t* p, bf16x8 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p));
}

// acc[i][j][r] = C[256 tm + 128 wm + 16 i + 4 g + r][column of B fragment j, lane row l16]:
// plain, columns 256 tn + 128 wn + 8 l16 + j; gated, output column 128 tn + 64 wn + 4 l16 + j
// from gate fragment j and up fragment j + 4.  Exactly 32 store instructions per wave for a
// full tile (the seam wait counts them).
template <int EPI>
DRTC_DEVICE void rg_epilogue(const RgParams& p, f32x4 (&acc)[8][8], int tm, int tn, int wm,
                             int wn, int l16, int g) {
  if constexpr (EPI == RG_RESIDUAL) {
    // two halves of 16 rows per lane: each half's residual rows are all loaded before its
    // first store (R may alias C: a load after a store could not be hoisted above it); a
    // whole tile's 32 rows at once would not fit beside the 256 accumulators
    const int n = 256 * tn + 128 * wn + 8 * l16;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      bf16x8 rv[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = min(256 * tm + 128 * wm + 16 * (4 * hf + i) + 4 * g + r, p.M - 1);
          rv[i][r] = *reinterpret_cast<const bf16x8*>(p.r + (int64_t)m * p.ldr + n);
        }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 256 * tm + 128 * wm + 16 * (4 * hf + i) + 4 * g + r;
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[4 * hf + i][j][r] + bf2f(rv[i][r][j]));
          if (m < p.M) rg_st<EPI>(p.c + (int64_t)m * p.ldc + n, o);
        }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 256 * tm + 128 * wm + 16 * i + 4 * g + r;
      if (m >= p.M) continue;
      bf16_t* crow = p.c + (int64_t)m * p.ldc;
      if constexpr (rg_glu<EPI>()) {
        const int n = 128 * tn + 64 * wn + 4 * l16;
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = f2bf(act_value<EPI == RG_SILU ? 0 : 1>(acc[i][j][r]) * acc[i][j + 4][r]);
        __builtin_nontemporal_store(o, reinterpret_cast<bf16x4*>(crow + n));
      } else {
        const int n = 256 * tn + 128 * wn + 8 * l16;
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[i][j][r]);
        rg_st<EPI>(crow + n, o);
      }
    }
  }
}

template <int EPI>
__global__ __launch_bounds__(kRgThreads, 1) void gemm_ring_kernel(RgParams p) {
  extern __shared__ __attribute__((aligned(16))) char rg_lds[];
  // ---- XCD remap (bijective; speed only): XCD label b % 8 takes a contiguous range of the
  // tile order, so the workgroups sharing operand panels share an L2
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, qq = nwg >> 3, rmd = nwg & 7;
  int tt = (xcd < rmd ? xcd * (qq + 1) : rmd * (qq + 1) + (xcd - rmd) * qq) + (orig >> 3);
  const int ntiles = p.tiles_m * p.tiles_n;
  if (tt >= ntiles) return;
  int tm, tn;
  rg_tile_of(p, tt, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wv >> 1, wn = wv & 1, l16 = lane & 15, g = lane >> 4;
  const unsigned lds0 = (unsigned)(uintptr_t)(rg_lds_ptr)rg_lds;
  RgLanes L;
  rg_lanes<EPI>(L, p, wv, lane, lds0);
  // fragment reads (bytes within a stage): A fragment i row 128 wm + 16 i + l16, chunk g;
  // B fragment j lane row l16 = panel weight row 8 l16 + j: block 8 wn + (l16 >> 1), slot row
  // 8 (l16 & 1) + j
  const int ra = (128 * wm + l16) * 64 + ((g ^ ((4 - (l16 >> 2)) & 3)) * 16);
  const int rb = kRgA + (8 * wn + (l16 >> 1)) * kRgBBlk + (l16 & 1) * 512 + ((g ^ (l16 & 1)) * 16);
  const char* lds = rg_lds;
  RgPlan P = rg_plan<EPI>(p, tm, tn);

  // ---- prologue: stages 0..3 of the first tile into slots 0..3
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const unsigned kb = 64u * u;
    const __amdgpu_buffer_rsrc_t rak = rg_rsrc(P.abase + kb, P.na - kb);
    const __amdgpu_buffer_rsrc_t rbk = rg_rsrc(P.bbase + kb, 0x7FFFFFFFu);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(L.lds_a + u * kRgStage) : "memory");
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" : : "v"(L.va[s]), "s"(rak) : "memory");
      asm volatile("s_add_u32 m0, m0, 0x400" ::: "memory");
    }
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(L.lds_b + u * kRgStage) : "memory");
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" : : "v"(L.vb[s]), "s"(rbk) : "memory");
      asm volatile("s_add_u32 m0, m0, 0x420" ::: "memory");
    }
  }
  rg_vmcnt<24>();  // own stage 0 landed
  rg_barrier();    // everyone's
  bf16x8 xa[8], xb[8], ya[8], yb[8];
  xa[0] = rg_rd(lds, ra);
#pragma unroll
  for (int j = 0; j < 8; ++j) xb[j] = rg_rd(lds, rb + 64 * j);
#pragma unroll
  for (int i = 1; i < 8; ++i) xa[i] = rg_rd(lds, ra + 1024 * i);
  rg_vmcnt<16>();  // own stage 1 landed
  rg_lgkm0();
  rg_barrier();

  f32x4 acc[8][8];
  const int trips = p.nk >> 2;
  bool seam = false;  // the previous tile's 32 epilogue stores are in this wave's vmcnt queue
  for (;;) {
    const int tnext = tt + nwg;
    const bool more = tnext < ntiles;
    int tm2 = tm, tn2 = tn;
    if (more) rg_tile_of(p, tnext, tm2, tn2);
    // the last trip DMAs the next tile's stages 0..3 (the very last tile re-stages its own:
    // valid bytes, never read)
    const RgPlan Pn = more ? rg_plan<EPI>(p, tm2, tn2) : P;
    rg_trip<true>(acc, xa, xb, ya, yb, lds, ra, rb, L, P, 256u, seam);
    for (int r = 1; r + 1 < trips; ++r)
      rg_trip<false>(acc, xa, xb, ya, yb, lds, ra, rb, L, P, 256u * (r + 1), false);
    constexpr bool kLate = EPI == RG_RESIDUAL;
    rg_trip<false, kLate>(acc, xa, xb, ya, yb, lds, ra, rb, L, Pn, 0u, false);
    if (!more) rg_vmcnt<0>();  // no LDS-DMA may still be landing when the workgroup leaves
    // the lane index re-derived (opaque to hipcc): kept live across the K loop it is spilled
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    rg_epilogue<EPI>(p, acc, tm, tn, wm, wn, ln & 15, ln >> 4);
    if (!more) break;
    if constexpr (kLate) rg_late_reads(xa, xb, lds, ra, rb);
    // the waits of the next tile's first two iterations may skip the stores (>= 32 younger
    // VMEM ops: a full tile's 32 stores, or a residual tile's 32 loads)
    seam = EPI == RG_RESIDUAL || 256 * tm + 256 <= p.M;
    tt = tnext;
    tm = tm2;
    tn = tn2;
    P = Pn;
  }
}

template <int EPI>
int rg_launch(const RgParams& p, hipStream_t st) {
  const int ntiles = p.tiles_m * p.tiles_n;
  const int cus = w4_num_cus();
  const int nwg = min(ntiles, cus > 0 ? cus : 256);
  hipLaunchKernelGGL((gemm_ring_kernel<EPI>), dim3(nwg), dim3(kRgThreads), kRgLds, st, p);
  return (int)hipGetLastError();
}

}  // namespace

int launch_gemm_ring(void* c, const void* a, const void* b, const void* r, int M, int N, int K,
                     int lda, int ldb, int ldc, int ldr, int epi, int group_m, hipStream_t st) {
  const bool glu = epi == RG_SILU || epi == RG_GELU;
  const bool res = epi == RG_RESIDUAL;
  if (epi < RG_STORE || epi > RG_GELU) return -1;
  if (M <= 0 || N <= 0 || K < 256 || K % 128) return -1;
  if (glu ? N % 128 : N % 256) return -1;
  if (lda % 8 || ldb % 8 || (glu ? ldc % 4 : ldc % 8) || lda < K || ldb < K) return -1;
  if (res && (ldr % 8 || r == nullptr || (uintptr_t)r % 16)) return -1;
  if ((uintptr_t)a % 16 || (uintptr_t)b % 16 || (uintptr_t)c % (glu ? 8 : 16)) return -1;
  // 32-bit buffer offsets from the panel bases
  if ((int64_t)min(M, 256) * lda * 2 >= (1ll << 31)) return -1;
  if ((int64_t)(glu ? N + 128 : 256) * ldb * 2 >= (1ll << 31)) return -1;
  RgParams p{};
  p.c = (bf16_t*)c;
  p.a = (const bf16_t*)a;
  p.b = (const bf16_t*)b;
  p.r = (const bf16_t*)r;
  p.M = M; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldr = ldr;
  p.tiles_m = (M + 255) / 256;
  p.tiles_n = glu ? N / 128 : N / 256;
  p.group_m = group_m < 1 ? 8 : group_m;
  p.up_off = glu ? N : 0;
  p.nk = K / 32;
  switch (epi) {
    case RG_STORE: return rg_launch<RG_STORE>(p, st);
    case RG_RESIDUAL: return rg_launch<RG_RESIDUAL>(p, st);
    case RG_SILU: return rg_launch<RG_SILU>(p, st);
    default: return rg_launch<RG_GELU>(p, st);
  }
}

int configure_gemm_ring() {
  int e = 0;
  for (const void* f : {(const void*)gemm_ring_kernel<RG_STORE>,
                        (const void*)gemm_ring_kernel<RG_RESIDUAL>,
                        (const void*)gemm_ring_kernel<RG_SILU>,
                        (const void*)gemm_ring_kernel<RG_GELU>})
    e |= (int)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kRgLds);
  return e;
}

}  // namespace drtc
