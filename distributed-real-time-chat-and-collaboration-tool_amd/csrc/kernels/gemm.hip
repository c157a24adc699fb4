// Hand-written CDNA4 (gfx950) bf16 GEMM for the projection layers:
//
//   C[M, N] = epi( A[M, K] . B[N, K]^T )        (A activations, B weights, both K-contiguous)
//
// with the epilogue fused into the kernel:
//   EPI_STORE     C = acc
//   EPI_RESIDUAL  C = acc + R                    (R may alias C: o / down projection adding
//                                                  into the residual stream in place)
//   EPI_SILU/GELU C[:, n] = act(gate_n) * up_n    (gate|up projection of a gated MLP; B rows
//                                                  [0, I) are the gate rows, [I, 2I) the up
//                                                  rows; C has I columns, no act_glu pass)
//
// This replaces the model hop of the reference (ref llm_server/llm_server.py:231, the
// remote generate_content call) with the dominant compute of an on-node engine.
//
// Structure (cdna_hip_programming.md §5: 256^2 tile, 8 waves, LDS-DMA staging):
//   * tile 256 (rows of A) x 256 (rows of B), 512 threads = 8 waves as 2 (M) x 4 (N), each
//     wave owns 128 x 64 outputs = 8 x 4 MFMA 16x16x32 tiles (128 accumulator registers);
//   * operands staged HBM/L2 -> LDS with global_load_lds_dwordx4 (16 B per lane, no VGPR
//     round trip), the bank-conflict swizzle applied to the per-lane SOURCE address and to
//     the ds_read_b128 address (the two sides of one involution, rule 21);
//   * operands swapped in the MFMA (B fragment as the "A" operand) so each lane's four
//     accumulator registers are four CONSECUTIVE output columns of one row: the epilogue
//     stores 8 bytes per lane and the gate/up pair of a GLU column sits in one lane;
//   * XCD-aware block order: blocks that share an XCD (L2) get consecutive logical tiles,
//     grouped GROUP_M row-tiles at a time, so a weight panel is fetched into each L2 once;
//   * split-K for short-M (decode) shapes: every K slice writes an fp32 slab, the last
//     arriving slice (agent-scope release/acquire ticket, §6 Guideline 16) sums the slabs
//     and runs the epilogue - one launch, no separate reduction kernel.
//
// Pipelines (template V):
//   V1  one LDS stage per 64-deep K tile, 2 stages, one barrier per K tile, next tile's
//       DMA issued right after the barrier (the "2-phase minimum" of §5.5 T3+T4).
//   V2  K tiles split into two 32-deep halves ("phases"), 4 half regions in LDS, each
//       phase: counted vmcnt -> raw s_barrier -> DMA of the phase three ahead into the
//       region freed by the previous phase -> 12 ds_read_b128 -> 32 MFMA.  Three half
//       tiles stay in flight across every barrier (§5 'Pipelining across barriers').
//   V3  V2 with the fragments of phase q+1 read during phase q's MFMAs (register double
//       buffer): no MFMA waits on an LDS read at a phase start.
//   V5  V2's memory pipeline with the two wave groups (wr = 0 / 1) staggered by one
//       barrier: per SIMD one wave computes while its partner reads fragments and
//       issues DMA (ping-pong; cdna_hip_programming.md §5 8-phase template's stagger).
#include "common.h"
#include "launchers.h"

namespace drtc {
namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int kTM = 256, kTN = 256, kBK = 64, kThreads = 512;

// LDS-DMA of 16 B per lane (global_load_lds_dwordx4) issued through inline asm: hipcc
// models the builtin form as an outstanding LDS access and then pins lgkmcnt(0) in front
// of every MFMA group (it cannot order the DMA against the ds_reads), which serialises
// the fragment reads with the MFMAs.  Hidden from the compiler, the DMA is waited for by
// the explicit counted vmcnt + barrier of each phase (cdna_hip_programming.md §5.7 item 1).
// M0 (the wave-uniform LDS destination) is written and restored inside the statement.
DRTC_DEVICE void glds16(const bf16_t* src, bf16_t* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ptr_t)lds);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst)
      : "memory");
}

template <int N>
DRTC_DEVICE void wait_vm() {
  // gfx9 s_waitcnt immediate: vmcnt[3:0] | expcnt[6:4] = 7 | lgkmcnt[11:8] = 15 | vmcnt_hi[15:14]
  constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
  __builtin_amdgcn_s_waitcnt(imm);
}

DRTC_DEVICE void barrier_raw() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct GemmParams {
  bf16_t* c;
  const bf16_t* a;
  const bf16_t* b;
  const bf16_t* r;
  float* slab;
  int* counters;
  int M, N, K;  // N = columns of C
  int lda, ldb, ldc, ldr;
  int tiles_m, tiles_n, splitk, kt_split;  // kt_split = 64-deep K tiles per slice
  int up_off;                              // GLU: row of B where the up half starts (= I)
  int group_m;
};

enum { EPI_STORE = 0, EPI_RESIDUAL = 1, EPI_SILU = 2, EPI_GELU = 3 };

template <int EPI>
DRTC_DEVICE constexpr bool is_glu() { return EPI == EPI_SILU || EPI == EPI_GELU; }

// Tile-local B row rb (0..255) -> global row of B.  GLU tiles interleave 16-row blocks
// of gate and up rows so an output column's gate and up accumulators share a lane.
template <int EPI>
DRTC_DEVICE int64_t b_row(const GemmParams& p, int tn, int rb) {
  if constexpr (is_glu<EPI>()) {
    const int pb = rb >> 5, w = rb & 31;
    return (int64_t)(kTN / 2) * tn + 16 * pb + (w & 15) + (w >= 16 ? p.up_off : 0);
  } else {
    return (int64_t)kTN * tn + rb;
  }
}

// Bank swizzle of the 64-B-row half-tile image (V2/V3): physical 16-B chunk = logical ^
// f(q), q = (row >> 2) & 3, f = {0, 2, 3, 1}: conflict-free for the ds_read_b128 lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... (MI355X_MICROARCH.md §LDS) where lane
// l reads row l & 15, chunk l >> 4.
DRTC_DEVICE int sw4(int q) { return (0x78 >> (2 * q)) & 3; }

template <int EPI>
DRTC_DEVICE void epilogue_store(const GemmParams& p, f32x4 (&acc)[8][4], int tm, int tn, int wr,
                                int wc, int l16, int g) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = kTM * tm + 128 * wr + 16 * i + l16;
    if (m >= p.M) continue;
    bf16_t* crow = p.c + (int64_t)m * p.ldc;
    if constexpr (is_glu<EPI>()) {
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int n = (kTN / 2) * tn + 32 * wc + 16 * jp + 4 * g;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[r] = f2bf(act_value<EPI == EPI_SILU ? 0 : 1>(acc[i][2 * jp][r]) * acc[i][2 * jp + 1][r]);
        *reinterpret_cast<bf16x4*>(crow + n) = o;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = kTN * tn + 64 * wc + 16 * j + 4 * g;
        bf16x4 o;
        if constexpr (EPI == EPI_RESIDUAL) {
          const bf16x4 rv = *reinterpret_cast<const bf16x4*>(p.r + (int64_t)m * p.ldr + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r] + bf2f(rv[r]));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r]);
        }
        *reinterpret_cast<bf16x4*>(crow + n) = o;
      }
    }
  }
}

// Split-K combine: publish this slice's fp32 slab, draw a ticket, the last arriver sums
// every other slice's slab into its registers.  Returns false for non-last slices.
DRTC_DEVICE bool splitk_combine(const GemmParams& p, f32x4 (&acc)[8][4], int tile, int slice,
                                bf16_t* lds) {
  const int tid = threadIdx.x;
  const int64_t per_slice = 32ll * kThreads;  // f32x4 elements
  f32x4* mine = reinterpret_cast<f32x4*>(p.slab) + ((int64_t)tile * p.splitk + slice) * per_slice;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) mine[(i * 4 + j) * kThreads + tid] = acc[i][j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(lds);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == p.splitk - 1);
    if (last) {
      // every slice of this tile has arrived: re-arm the counter for the next launch
      __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return false;
  const f32x4* base = reinterpret_cast<const f32x4*>(p.slab) + (int64_t)tile * p.splitk * per_slice;
  for (int s = 0; s < p.splitk; ++s) {
    if (s == slice) continue;
    const f32x4* src = base + s * per_slice;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] += src[(i * 4 + j) * kThreads + tid];
  }
  return true;
}

template <int EPI, int V>
__global__ __launch_bounds__(kThreads) void gemm256_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  // ---- tile assignment: XCD remap (bijective), split-K slice fastest, grouped rows
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, qq = nwg >> 3, rmd = nwg & 7;
  const int wgid = (xcd < rmd ? xcd * (qq + 1) : rmd * (qq + 1) + (xcd - rmd) * qq) + (orig >> 3);
  const int slice = wgid % p.splitk;
  const int t = wgid / p.splitk;
  const int gsize = p.group_m * p.tiles_n;
  const int first_m = (t / gsize) * p.group_m;
  const int gm = min(p.tiles_m - first_m, p.group_m);
  const int tm = first_m + (t % gsize) % gm;
  const int tn = (t % gsize) / gm;
  const int tile = tm * p.tiles_n + tn;

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wv >> 2, wc = wv & 3, l16 = lane & 15, g = lane >> 4;
  const int k_base = slice * p.kt_split * kBK;
  const int nk = p.kt_split;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if constexpr (V == 1) {
    // ---- V1: [stage 2][row 512][64] with 128-B rows, chunk ^= (row >> 1) & 7
    constexpr int STAGE = 512 * kBK;
    const bf16_t* src[8];
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) {
      const int loc = 32 * wv + 8 * (ii & 3) + (lane >> 3);  // row within the operand tile
      const int d = (lane & 7) ^ ((loc >> 1) & 7);
      if (ii < 4) {
        const int m = min(kTM * tm + loc, p.M - 1);
        src[ii] = p.a + (int64_t)m * p.lda + k_base + 8 * d;
      } else {
        src[ii] = p.b + b_row<EPI>(p, tn, loc) * p.ldb + k_base + 8 * d;
      }
    }
    auto stage = [&](int kt, int buf) {
      bf16_t* base = lds + buf * STAGE;
#pragma unroll
      for (int ii = 0; ii < 8; ++ii) {
        const int row = (ii < 4 ? 0 : 256) + 32 * wv + 8 * (ii & 3);
        glds16(src[ii] + kt * kBK, base + row * kBK);
      }
    };
    const int rsw = (l16 >> 1) & 7;
    stage(0, 0);
    for (int kt = 0; kt < nk; ++kt) {
      wait_vm<0>();
      barrier_raw();
      if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
      const bf16_t* S = lds + (kt & 1) * STAGE;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = ((4 * s + g) ^ rsw) * 8;
        bf16x8 fb[4], fa[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = *(const bf16x8*)(S + (256 + 64 * wc + 16 * j + l16) * kBK + ch);
#pragma unroll
        for (int i = 0; i < 8; ++i) fa[i] = *(const bf16x8*)(S + (128 * wr + 16 * i + l16) * kBK + ch);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  } else {
    // ---- V2 / V3: [region 4][row 512][32] with 64-B rows (region = phase & 3,
    // phase = 2 * k_tile + half); rows 0..255 = A, 256..511 = B
    constexpr int REG = 512 * 32;
    const bf16_t* src[4];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int row = 64 * wv + 16 * ii + (lane >> 2);  // staged row 0..511
      const int d = (lane & 3) ^ sw4((lane >> 4) & 3);
      if (row < 256) {
        const int m = min(kTM * tm + row, p.M - 1);
        src[ii] = p.a + (int64_t)m * p.lda + k_base + 8 * d;
      } else {
        src[ii] = p.b + b_row<EPI>(p, tn, row - 256) * p.ldb + k_base + 8 * d;
      }
    }
    auto issue = [&](int q) {  // DMA of phase q (k tile q >> 1, half q & 1) into region q & 3
      bf16_t* base = lds + (q & 3) * REG + 64 * wv * 32;
      const int koff = (q >> 1) * kBK + (q & 1) * 32;
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) glds16(src[ii] + koff, base + 16 * ii * 32);
    };
    const int ch = (g ^ sw4((l16 >> 2) & 3)) * 8;
    const int aoff = (128 * wr + l16) * 32 + ch;
    const int boff = (256 + 64 * wc + l16) * 32 + ch;
    auto read = [&](int q, bf16x8 (&fa)[8], bf16x8 (&fb)[4]) {
      const bf16_t* R = lds + (q & 3) * REG;
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *(const bf16x8*)(R + boff + 16 * j * 32);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = *(const bf16x8*)(R + aoff + 16 * i * 32);
    };
    auto mma = [&](const bf16x8 (&fa)[8], const bf16x8 (&fb)[4]) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    };
    const int Q = 2 * nk;
    issue(0);
    if (Q > 1) issue(1);
    if (Q > 2) issue(2);
    if constexpr (V == 6) {
      // V5 with the DMA of phase q+3 issued from the COMPUTE segment of phase q,
      // one 1-KiB piece after every 8 MFMAs (an LDS-DMA issue costs ~60 cycles
      // among bare MFMAs, 100-185 inside a load segment already carrying 12
      // ds_reads: MI355X_MICROARCH.md cycle constants).  Region (q+3)&3 held
      // phase q-1, whose last reader (G1) finished it in I(2q) <= this segment;
      // the load segment of phase q waits for phase q+1 (issued in the compute
      // segment of q-2) with one younger phase (q+2) in flight.
      wait_vm<8>();  // phase 0 landed
      barrier_raw();
      if (wr == 1) barrier_raw();
      for (int q = 0; q < Q; ++q) {
        bf16x8 fa[8], fb[4];
        read(q, fa, fb);
        if (q + 2 < Q) wait_vm<4>();
        else wait_vm<0>();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        barrier_raw();
        const bool dma = q + 3 < Q;
        bf16_t* dbase = lds + ((q + 3) & 3) * REG + 64 * wv * 32;
        const int koff = ((q + 3) >> 1) * kBK + ((q + 3) & 1) * 32;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
          if ((i & 1) && dma) {
            __builtin_amdgcn_sched_barrier(0);
            glds16(src[i >> 1] + koff, dbase + 16 * (i >> 1) * 32);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        __builtin_amdgcn_s_setprio(0);
        barrier_raw();
      }
      if (wr == 0) barrier_raw();
    } else if constexpr (V == 5) {
      // Ping-pong: wave group G0 (wr = 0) and G1 (wr = 1) run the same
      // load | barrier | compute | barrier program, G1 one barrier behind, so on
      // every SIMD (one wave of each group) one wave's 32 MFMAs overlap the other
      // wave's fragment reads + DMA issue.  Interval I(n) = between barriers n-1
      // and n: G0 loads phase k in I(2k+1) and computes it in I(2k+2); G1 loads
      // it in I(2k+2) and computes in I(2k+3).  A load segment for phase k reads
      // region k, issues the DMA of phase k+3 into the region of phase k-1 (read
      // by both groups by I(2k) at the latest, with lgkmcnt(0) before that
      // barrier), then waits until its own DMA of phase k+1 landed (vmcnt of
      // the two younger phases), so phase k+1 is visible to G0's reads in
      // I(2k+3) after barriers 2k+1 (G0's wait) and 2k+2 (G1's wait).
      wait_vm<8>();  // phase 0 landed (1 and 2 may fly)
      barrier_raw();
      if (wr == 1) barrier_raw();  // the stagger
      for (int q = 0; q < Q; ++q) {
        bf16x8 fa[8], fb[4];
        read(q, fa, fb);
        if (q + 3 < Q) issue(q + 3);
        const int younger = min(2, max(0, Q - 1 - (q + 1)));
        if (younger == 2) wait_vm<8>();
        else if (younger == 1) wait_vm<4>();
        else wait_vm<0>();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): fragments in registers
        barrier_raw();
        mma(fa, fb);
        barrier_raw();
      }
      if (wr == 0) barrier_raw();  // balance G1's extra barrier
    } else if constexpr (V == 2) {
      for (int q = 0; q < Q; ++q) {
        const int ahead = Q - 1 - q;  // phases issued after q (at most 2 are outstanding)
        if (ahead >= 2) wait_vm<8>();
        else if (ahead == 1) wait_vm<4>();
        else wait_vm<0>();
        barrier_raw();
        if (q + 3 < Q) issue(q + 3);
        bf16x8 fa[8], fb[4];
        read(q, fa, fb);
        mma(fa, fb);
      }
    } else {
      // V3: fragments of phase q are read during phase q-1.  At phase q the region of
      // phase q was fully read before this barrier, so it takes the DMA of phase q + 4;
      // the wait makes phase q + 1 (read during this phase) visible.
      // Each phase waits lgkmcnt(0) before its barrier: the fragment reads of the
      // previous phase (consumed only in this phase) must have left LDS before any
      // wave re-targets their region with a DMA.
      bf16x8 fa0[8], fb0[4], fa1[8], fb1[4];
      wait_vm<(0)>();  // phases 0..2 (Q >= 2 always: K >= 64)
      barrier_raw();
      read(0, fa0, fb0);
      if (Q > 3) issue(3);  // region 3: never read yet
      for (int q = 0; q < Q; q += 2) {
        // ---- even phase q: compute fa0/fb0, read phase q + 1 into fa1/fb1
        {
          const int ahead = Q - 1 - (q + 1);  // phases issued after q + 1
          if (ahead >= 2) wait_vm<8>();
          else if (ahead == 1) wait_vm<4>();
          else wait_vm<0>();
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        barrier_raw();
        if (q + 4 < Q) issue(q + 4);
        if (q + 1 < Q) read(q + 1, fa1, fb1);
        mma(fa0, fb0);
        if (q + 1 >= Q) break;
        // ---- odd phase q + 1: compute fa1/fb1, read phase q + 2 into fa0/fb0
        {
          const int ahead = Q - 1 - (q + 2);
          if (ahead >= 2) wait_vm<8>();
          else if (ahead == 1) wait_vm<4>();
          else wait_vm<0>();
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        barrier_raw();
        if (q + 5 < Q) issue(q + 5);
        if (q + 2 < Q) read(q + 2, fa0, fb0);
        mma(fa1, fb1);
      }
    }
  }

  if (p.splitk > 1) {
    __syncthreads();
    if (!splitk_combine(p, acc, tile, slice, lds)) return;
  }
  epilogue_store<EPI>(p, acc, tm, tn, wr, wc, l16, g);
}

// ---------------------------------------------------------------- V4
// The 4-wave layout hipBLASLt's gfx950 kernels use (PMC: 4 waves/CU, 1/3 fewer LDS
// instructions than the 8-wave layout): 256 x 256 tile, waves 2 x 2, each wave 128 x 128
// outputs = 8 x 8 MFMA 16x16x32 tiles = 256 accumulator registers (the AGPR half of
// the unified file; one wave per SIMD, 512 registers).  Per 32-deep phase a wave reads
// the 8 B fragments of the NEXT phase and streams its 8 A fragments one 16-row block
// at a time, one MFMA row (8 MFMA) ahead of use: 16 ds_read_b128 per 64 MFMAs.  All
// loops fully unrolled (no runtime-indexed register arrays -> no scratch, rule 20).
template <int EPI>
DRTC_DEVICE void epilogue_store4(const GemmParams& p, f32x4 (&acc)[8][8], int tm, int tn, int wr,
                                 int wc, int l16, int g) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = kTM * tm + 128 * wr + 16 * i + l16;
    if (m >= p.M) continue;
    bf16_t* crow = p.c + (int64_t)m * p.ldc;
    if constexpr (is_glu<EPI>()) {
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        const int n = (kTN / 2) * tn + 64 * wc + 16 * jp + 4 * g;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[r] = f2bf(act_value<EPI == EPI_SILU ? 0 : 1>(acc[i][2 * jp][r]) * acc[i][2 * jp + 1][r]);
        *reinterpret_cast<bf16x4*>(crow + n) = o;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int n = kTN * tn + 128 * wc + 16 * j + 4 * g;
        bf16x4 o;
        if constexpr (EPI == EPI_RESIDUAL) {
          const bf16x4 rv = *reinterpret_cast<const bf16x4*>(p.r + (int64_t)m * p.ldr + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r] + bf2f(rv[r]));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r]);
        }
        *reinterpret_cast<bf16x4*>(crow + n) = o;
      }
    }
  }
}

DRTC_DEVICE bool splitk_combine4(const GemmParams& p, f32x4 (&acc)[8][8], int tile, int slice,
                                 bf16_t* lds) {
  constexpr int NT = 256;
  const int tid = threadIdx.x;
  const int64_t per_slice = 64ll * NT;  // f32x4 elements (256 KiB, as the 8-wave layout)
  f32x4* mine = reinterpret_cast<f32x4*>(p.slab) + ((int64_t)tile * p.splitk + slice) * per_slice;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) mine[(i * 8 + j) * NT + tid] = acc[i][j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(lds);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == p.splitk - 1);
    if (last) {
      __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return false;
  const f32x4* base = reinterpret_cast<const f32x4*>(p.slab) + (int64_t)tile * p.splitk * per_slice;
  for (int s = 0; s < p.splitk; ++s) {
    if (s == slice) continue;
    const f32x4* src = base + s * per_slice;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] += src[(i * 8 + j) * NT + tid];
  }
  return true;
}

template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm256w4_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, qq = nwg >> 3, rmd = nwg & 7;
  const int wgid = (xcd < rmd ? xcd * (qq + 1) : rmd * (qq + 1) + (xcd - rmd) * qq) + (orig >> 3);
  const int slice = wgid % p.splitk;
  const int t = wgid / p.splitk;
  const int gsize = p.group_m * p.tiles_n;
  const int first_m = (t / gsize) * p.group_m;
  const int gm = min(p.tiles_m - first_m, p.group_m);
  const int tm = first_m + (t % gsize) % gm;
  const int tn = (t % gsize) / gm;
  const int tile = tm * p.tiles_n + tn;

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wv >> 1, wc = wv & 1, l16 = lane & 15, g = lane >> 4;
  const int k_base = slice * p.kt_split * kBK;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // [region 4][row 512][32] (64-B rows): rows 0..255 A, 256..511 B; wave wv stages
  // rows [128 wv, 128 wv + 128) of every phase as 8 DMA pieces of 16 rows
  constexpr int REG = 512 * 32;
  const bf16_t* src[8];
#pragma unroll
  for (int ii = 0; ii < 8; ++ii) {
    const int row = 128 * wv + 16 * ii + (lane >> 2);
    const int d = (lane & 3) ^ sw4((lane >> 4) & 3);
    if (row < 256) {
      const int m = min(kTM * tm + row, p.M - 1);
      src[ii] = p.a + (int64_t)m * p.lda + k_base + 8 * d;
    } else {
      src[ii] = p.b + b_row<EPI>(p, tn, row - 256) * p.ldb + k_base + 8 * d;
    }
  }
  auto issue = [&](int q) {
    bf16_t* base = lds + (q & 3) * REG + 128 * wv * 32;
    const int koff = (q >> 1) * kBK + (q & 1) * 32;
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) glds16(src[ii] + koff, base + 16 * ii * 32);
  };
  const int ch = (g ^ sw4((l16 >> 2) & 3)) * 8;
  const int aoff = (128 * wr + l16) * 32 + ch;
  const int boff = (256 + 128 * wc + l16) * 32 + ch;
  auto readB = [&](int q, int j) -> bf16x8 {
    return *(const bf16x8*)(lds + (q & 3) * REG + boff + 16 * j * 32);
  };
  auto readA = [&](int q, int i) -> bf16x8 {
    return *(const bf16x8*)(lds + (q & 3) * REG + aoff + 16 * i * 32);
  };
  // (the last phase also "reads" the B fragments of a phase Q that does not exist:
  // stale LDS bytes that are never used - an unconditional read keeps the phase one
  // straight-line block for the scheduler)
  auto phase = [&](int q, bf16x8 (&fb)[8], bf16x8 (&fbn)[8]) {
    bf16x8 fa = readA(q, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16x8 fan;
      if (i < 7) fan = readA(q, i + 1);
      fbn[i] = readB(q + 1, i);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(fb[j], fa, acc[i][j]);
      if (i < 7) fa = fan;
    }
  };
  // Phase q (k tile q >> 1, half q & 1) lives in region q & 3.  Before phase q's
  // barrier each wave has waited for its own DMA of phase q + 1 (read during phase
  // q: the next B fragments) and for its LDS reads (lgkmcnt(0)); after the barrier
  // the DMA of phase q + 3 goes into the region of phase q - 1, whose last reads
  // (the A fragments of phase q - 1) retired before this barrier.
  const int Q = 2 * p.kt_split;
  issue(0);
  if (Q > 1) issue(1);
  if (Q > 2) issue(2);
  bf16x8 fb0[8], fb1[8];
  wait_vm<0>();
  barrier_raw();
#pragma unroll
  for (int j = 0; j < 8; ++j) fb0[j] = readB(0, j);
  for (int q = 0; q < Q; q += 2) {
    // ---- phase q: B of q in fb0; A of q and B of q + 1 are read during it
    {
      const int ahead = Q - 1 - (q + 1);
      if (ahead >= 2) wait_vm<16>();
      else if (ahead == 1) wait_vm<8>();
      else wait_vm<0>();
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    barrier_raw();
    if (q + 3 < Q) issue(q + 3);  // region of phase q - 1: fully read before this barrier
    phase(q, fb0, fb1);  // Q is even: phase q + 1 always exists
    {
      const int ahead = Q - 1 - (q + 2);
      if (ahead >= 2) wait_vm<16>();
      else if (ahead == 1) wait_vm<8>();
      else wait_vm<0>();
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    barrier_raw();
    if (q + 4 < Q) issue(q + 4);
    phase(q + 1, fb1, fb0);
  }

  if (p.splitk > 1) {
    __syncthreads();
    if (!splitk_combine4(p, acc, tile, slice, lds)) return;
  }
  epilogue_store4<EPI>(p, acc, tm, tn, wr, wc, l16, g);
}

template <int EPI, int V>
int launch_t(const GemmParams& p, hipStream_t st) {
  const int nwg = p.tiles_m * p.tiles_n * p.splitk;
  if constexpr (V == 4) {
    hipLaunchKernelGGL((gemm256w4_kernel<EPI>), dim3(nwg), dim3(256), 4 * 512 * 32 * 2, st, p);
    return (int)hipGetLastError();
  }

  constexpr int lds_bytes = V == 1 ? 2 * 512 * kBK * 2 : 4 * 512 * 32 * 2;
  hipLaunchKernelGGL((gemm256_kernel<EPI, V>), dim3(nwg), dim3(kThreads), lds_bytes, st, p);
  return (int)hipGetLastError();
}

template <int EPI>
int launch_e(const GemmParams& p, int variant, hipStream_t st) {
  switch (variant) {
    case 1: return launch_t<EPI, 1>(p, st);
    case 2: return launch_t<EPI, 2>(p, st);
    case 3: return launch_t<EPI, 3>(p, st);
    case 4: return launch_t<EPI, 4>(p, st);
    case 5: return launch_t<EPI, 5>(p, st);
    case 6: return launch_t<EPI, 6>(p, st);
    default: return -1;
  }
}

template <int EPI, int V>
int cfg_one() {
  constexpr int lds_bytes = V == 1 ? 2 * 512 * kBK * 2 : 4 * 512 * 32 * 2;
  return (int)hipFuncSetAttribute((const void*)gemm256_kernel<EPI, V>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
}

template <int EPI>
int cfg_epi() {
  return cfg_one<EPI, 1>() | cfg_one<EPI, 2>() | cfg_one<EPI, 3>() | cfg_one<EPI, 5>() |
         cfg_one<EPI, 6>() |
         (int)hipFuncSetAttribute((const void*)gemm256w4_kernel<EPI>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 512 * 32 * 2);
}

}  // namespace

int64_t gemm_workspace_bytes(int64_t M, int64_t N, int splitk) {
  const int64_t tiles = ((M + kTM - 1) / kTM) * ((N + kTN - 1) / kTN);
  // (the 8-wave slab: 32 f32x4 per thread x 512 threads; gemm_w4's is 64 x 256, the same
  // 256 KiB per tile and slice)
  return splitk > 1 ? tiles * splitk * 32ll * kThreads * 16 : 0;
}

int launch_gemm(void* c, const void* a, const void* b, const void* r, int M, int N, int K,
                int lda, int ldb, int ldc, int ldr, int epi, int up_off, int variant, int splitk,
                int group_m, void* slab, int64_t slab_bytes, int* counters, int n_counters,
                hipStream_t st) {
  // shape contract (checked here so a bad call never reaches the device)
  if ((variant >= 7 && variant <= 15) || variant == 31)
    return launch_gemm_w4(c, a, b, r, M, N, K, lda, ldb, ldc, ldr, epi, up_off, splitk, group_m,
                          slab, slab_bytes, counters, n_counters, variant - 7, st);
  const bool glu = epi == EPI_SILU || epi == EPI_GELU;
  if (M <= 0 || N <= 0 || K <= 0 || K % kBK || splitk < 1 || (K / kBK) % splitk) return -1;
  if (glu ? (N % (kTN / 2)) : (N % kTN)) return -1;
  if (lda % 8 || ldb % 8 || ldc % 4 || (epi == EPI_RESIDUAL && (ldr % 4 || r == nullptr))) return -1;
  if ((uintptr_t)a % 16 || (uintptr_t)b % 16 || (uintptr_t)c % 8) return -1;
  if (group_m < 1) group_m = 8;
  GemmParams p{};
  p.c = (bf16_t*)c;
  p.a = (const bf16_t*)a;
  p.b = (const bf16_t*)b;
  p.r = (const bf16_t*)r;
  p.M = M; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldr = ldr;
  p.tiles_m = (M + kTM - 1) / kTM;
  p.tiles_n = glu ? N / (kTN / 2) : N / kTN;
  p.splitk = splitk;
  p.kt_split = K / kBK / splitk;
  p.up_off = up_off;
  p.group_m = group_m;
  if (splitk > 1) {
    const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
    if (slab == nullptr || counters == nullptr || n_counters < tiles ||
        slab_bytes < tiles * splitk * 32ll * kThreads * 16)
      return -2;
    p.slab = (float*)slab;
    p.counters = counters;
  }
  switch (epi) {
    case EPI_STORE: return launch_e<EPI_STORE>(p, variant, st);
    case EPI_RESIDUAL: return launch_e<EPI_RESIDUAL>(p, variant, st);
    case EPI_SILU: return launch_e<EPI_SILU>(p, variant, st);
    case EPI_GELU: return launch_e<EPI_GELU>(p, variant, st);
    default: return -1;
  }
}

int configure_gemm() {
  return cfg_epi<EPI_STORE>() | cfg_epi<EPI_RESIDUAL>() | cfg_epi<EPI_SILU>() |
         cfg_epi<EPI_GELU>();
}

}  // namespace drtc
