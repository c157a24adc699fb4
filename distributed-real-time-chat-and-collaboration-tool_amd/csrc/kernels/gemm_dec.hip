// Hand-written CDNA4 (gfx950) bf16 GEMM for decode-batch projections (M = 256..1024 rows):
//
//   C[M, N] = epi( A[M, K] . B[N, K]^T )      (A activations, B weights, both K-contiguous)
//
// Why a second tile shape: at a decode bucket of M = 1024 rows the 8B model's o / down
// projections (N = 4096) have only 64 output tiles of 256 x 256, a quarter of the 256 CUs.
// hipBLASLt covers the CUs with stream-K and reaches 0.9-1.1 PF/s there (profiles/README.md);
// the 256^2 kernel of gemm.hip needs split-K with fp32 slabs whose traffic costs as much as
// the MFMA work (profiles/r2a_hand_gemm.md: 0.58x the library on o).  Here a 128 x 128 tile
// gives 256 tiles = one per CU with no cross-workgroup reduction, and the two SIMD slots
// that a 256^2 tile fills with its second wave row are filled by an INTRA-workgroup K
// split instead:
//
//   * 512 threads = 8 waves = 2 K groups x (2 x 2) waves; every wave owns 64 x 64 outputs
//     (4 x 4 MFMA 16x16x32 tiles, 64 accumulator registers).  Group 0 computes the even
//     32-deep K phases, group 1 the odd ones; each SIMD holds one wave of each group.  At
//     the end group 1 hands its accumulators to group 0 through LDS (64 KiB) - one sum per
//     output instead of an fp32 slab round trip through HBM.
//   * Per wave and phase: 8 ds_read_b128 (64 A rows + 64 B rows of 32 k) feed 16 MFMAs:
//     with 8 waves the LDS array runs at ~50 % of its 256 B/clk (MI355X_MICROARCH.md §LDS).
//   * Operands are staged HBM/L2 -> LDS by global_load_lds_dwordx4 (no VGPR round trip)
//     into NR regions of 256 rows x 64 B; the 16-B chunk swizzle (f(q) = {0,2,3,1}, q =
//     (row >> 2) & 3) is applied to the per-lane SOURCE address of the DMA and to the
//     ds_read address (conflict-free for the ds_read_b128 lane groups).  A step = one
//     phase per group = 64 k; NR = 8 regions keep 3 steps in flight (128 KiB, one
//     workgroup per CU), NR = 4 one step (64 KiB, two workgroups per CU for grids that
//     exceed the CU count).
//   * Operands swapped in the MFMA (B fragment as the "A" operand) so each lane's four
//     accumulator registers are four consecutive output columns of one row (8-byte stores;
//     a gated-MLP column's gate and up values sit in one lane).
//   * XCD-aware workgroup order (bijective remap, GROUP_M row tiles per group), as gemm.hip.
//
// Epilogues: store, residual add (R may alias C), SiLU/GELU-gated [gate; up] (B rows
// [0, up_off) gate, [up_off, 2 up_off) up; C has up_off columns; no act_glu pass).
//
// This is part of the on-node engine that replaces the reference's hosted model call
// (ref llm_server/llm_server.py:231).
#include "common.h"
#include "launchers.h"

namespace drtc {
namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kT = 128, kPh = 32, kRows = 2 * kT, kThr = 512;
constexpr int kReg = kRows * kPh;  // elements per LDS region (16 KiB)

// LDS-DMA of 16 B per lane, hidden from the compiler's LDS dependency tracking (see
// gemm.hip glds16: the builtin form makes hipcc pin lgkmcnt(0) before every MFMA group).
DRTC_DEVICE void dma16(const bf16_t* src, bf16_t* lds) {
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
DRTC_DEVICE void vm_wait() {
  constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
  __builtin_amdgcn_s_waitcnt(imm);
}

DRTC_DEVICE void bar() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

DRTC_DEVICE int swz(int q) { return (0x78 >> (2 * q)) & 3; }

struct DecParams {
  bf16_t* c;
  const bf16_t* a;
  const bf16_t* b;
  const bf16_t* r;
  int M, K;
  int lda, ldb, ldc, ldr;
  int tiles_m, tiles_n, up_off, group_m;
};

enum { E_STORE = 0, E_RES = 1, E_SILU = 2, E_GELU = 3 };

template <int EPI>
DRTC_DEVICE constexpr bool glu() { return EPI == E_SILU || EPI == E_GELU; }

// tile-local B row (0..127) -> global row of B; gated tiles interleave 16-row blocks of
// gate and up rows (block 2p = gate cols 16p.., block 2p+1 = the matching up rows)
template <int EPI>
DRTC_DEVICE int64_t brow(const DecParams& p, int tn, int rb) {
  if constexpr (glu<EPI>()) {
    const int pb = rb >> 5, w = rb & 31;
    return (int64_t)(kT / 2) * tn + 16 * pb + (w & 15) + (w >= 16 ? p.up_off : 0);
  } else {
    return (int64_t)kT * tn + rb;
  }
}

template <int NSTEP>
DRTC_DEVICE void wait_steps(int younger) {
  // each step = 4 DMA instructions per wave; wait until at most `younger` steps fly
  if constexpr (NSTEP >= 3) {
    if (younger >= 2) { vm_wait<8>(); return; }
  }
  if constexpr (NSTEP >= 2) {
    if (younger >= 1) { vm_wait<4>(); return; }
  }
  vm_wait<0>();
}

template <int EPI, int NR, int V>
__global__ __launch_bounds__(kThr) void gemm_dec_kernel(DecParams p) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  constexpr int D = NR / 2 - 1;  // steps in flight ahead of the one being computed
  static_assert(D >= 1 && D <= 3, "NR must be 4, 6 or 8");

  // ---- tile assignment: XCD remap (bijective), grouped row tiles
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, qq = nwg >> 3, rmd = nwg & 7;
  const int t = (xcd < rmd ? xcd * (qq + 1) : rmd * (qq + 1) + (xcd - rmd) * qq) + (orig >> 3);
  const int gsize = p.group_m * p.tiles_n;
  const int first_m = (t / gsize) * p.group_m;
  const int gm = min(p.tiles_m - first_m, p.group_m);
  const int tm = first_m + (t % gsize) % gm;
  const int tn = (t % gsize) / gm;

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wv >> 2, wr = (wv >> 1) & 1, wc = wv & 1;
  const int l16 = lane & 15, g = lane >> 4;

  // ---- DMA sources: wave wv stages rows [32 wv, 32 wv + 32) of every phase (2 x 16 rows)
  const bf16_t* src[2];
#pragma unroll
  for (int ii = 0; ii < 2; ++ii) {
    const int row = 32 * wv + 16 * ii + (lane >> 2);
    const int d = (lane & 3) ^ swz((lane >> 4) & 3);
    if (row < kT) {
      const int m = min(kT * tm + row, p.M - 1);
      src[ii] = p.a + (int64_t)m * p.lda + 8 * d;
    } else {
      src[ii] = p.b + brow<EPI>(p, tn, row - kT) * p.ldb + 8 * d;
    }
  }
  auto issue = [&](int s) {  // phases 2s, 2s+1 -> regions (2s) % NR, (2s+1) % NR
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = 2 * s + h;
      bf16_t* base = lds + (q % NR) * kReg + 32 * wv * kPh;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) dma16(src[ii] + q * kPh, base + 16 * ii * kPh);
    }
  };

  const int ch = (g ^ swz((l16 >> 2) & 3)) * 8;
  const int aoff = (64 * wr + l16) * kPh + ch;
  const int boff = (kT + 64 * wc + l16) * kPh + ch;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int S = p.K / (2 * kPh);
  auto frags = [&](int s, bf16x8 (&fa)[4], bf16x8 (&fb)[4]) {
    const bf16_t* R = lds + ((2 * s + grp) % NR) * kReg;
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = *(const bf16x8*)(R + boff + 16 * j * kPh);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = *(const bf16x8*)(R + aoff + 16 * i * kPh);
  };

  if constexpr (V == 1) {
    // ---- V1: barrier -> DMA of step s + D -> 8 fragment reads -> 16 MFMAs
#pragma unroll
    for (int s = 0; s < D; ++s)
      if (s < S) issue(s);
    for (int s = 0; s < S; ++s) {
      wait_steps<D>(min(D - 1, S - 1 - s));
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of step s - 1 retired
      bar();  // step s visible to every wave; every read of step s - 1 retired
      if (s + D < S) issue(s + D);  // into the regions of step s - 1
      bf16x8 fa[4], fb[4];
      frags(s, fa, fb);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  } else {
    // ---- V2: fragments double-buffered in registers.  Iteration s computes step s from
    // registers read during iteration s - 1, reads step s + 1, and refills the regions of
    // step s (free: every wave read them before this barrier) with step s + NR/2, one
    // DMA piece after every 4 MFMAs.  The barrier of iteration s covers "step s + 1
    // landed" (each wave's own counted vmcnt, then the barrier for the other waves) and
    // "step s fully read" (lgkmcnt(0) before it).
    constexpr int A = NR / 2;  // steps in flight
    auto piece = [&](int s, int k) {  // DMA piece k (0..3) of step s
      const int q = 2 * s + (k >> 1);
      dma16(src[k & 1] + q * kPh, lds + (q % NR) * kReg + 32 * wv * kPh + 16 * (k & 1) * kPh);
    };
#pragma unroll
    for (int s = 0; s < A; ++s)
      if (s < S) issue(s);
    // step 0 landed: younger = min(S, A) - 1 steps may fly
    {
      const int y = min(S, A) - 1;
      if (A >= 4 && y >= 3) vm_wait<12>();
      else if (A >= 3 && y >= 2) vm_wait<8>();
      else if (y >= 1) vm_wait<4>();
      else vm_wait<0>();
    }
    bar();
    bf16x8 ca[4], cb[4], na[4], nb[4];
    frags(0, ca, cb);
    auto iter = [&](int s, bf16x8 (&fa)[4], bf16x8 (&fb)[4], bf16x8 (&ga)[4], bf16x8 (&gb)[4]) {
      // younger steps allowed in flight once step s + 1 landed
      const int y = max(0, min(S - s - 2, A - 2));
      if (A >= 4 && y >= 2) vm_wait<8>();
      else if (A >= 3 && y >= 1) vm_wait<4>();
      else vm_wait<0>();
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): fragments of step s in registers
      bar();
      const bool nxt = s + 1 < S;
      const bool dma = s + A < S;
      if (nxt) frags(s + 1, ga, gb);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
        if (dma) {
          __builtin_amdgcn_sched_barrier(0);
          piece(s + A, i);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    };
    int s = 0;
    for (; s + 1 < S; s += 2) {
      iter(s, ca, cb, na, nb);
      iter(s + 1, na, nb, ca, cb);
    }
    if (s < S) iter(s, ca, cb, na, nb);
  }

  // ---- K-group reduction through LDS: group 1 -> group 0
  __syncthreads();
  f32x4* red = reinterpret_cast<f32x4*>(lds);
  const int slot = (wv & 3) * 16;
  if (grp == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[(slot + 4 * i + j) * 64 + lane] = acc[i][j];
  }
  __syncthreads();
  if (grp == 1) return;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] += red[(slot + 4 * i + j) * 64 + lane];

  // ---- epilogue
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = kT * tm + 64 * wr + 16 * i + l16;
    if (m >= p.M) continue;
    bf16_t* crow = p.c + (int64_t)m * p.ldc;
    if constexpr (glu<EPI>()) {
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int n = (kT / 2) * tn + 32 * wc + 16 * jp + 4 * g;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[r] = f2bf(act_value<EPI == E_SILU ? 0 : 1>(acc[i][2 * jp][r]) * acc[i][2 * jp + 1][r]);
        *reinterpret_cast<bf16x4*>(crow + n) = o;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = kT * tn + 64 * wc + 16 * j + 4 * g;
        bf16x4 o;
        if constexpr (EPI == E_RES) {
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

template <int NR>
constexpr int lds_bytes() { return NR * kReg * 2; }

template <int EPI, int NR, int V>
int launch_t(const DecParams& p, hipStream_t st) {
  const int nwg = p.tiles_m * p.tiles_n;
  hipLaunchKernelGGL((gemm_dec_kernel<EPI, NR, V>), dim3(nwg), dim3(kThr), lds_bytes<NR>(), st, p);
  return (int)hipGetLastError();
}

// cfg = 10 * pipeline + LDS regions (14 16 18: V1; 24 26 28: V2)
template <int EPI>
int launch_e(const DecParams& p, int cfg, hipStream_t st) {
  switch (cfg) {
    case 14: return launch_t<EPI, 4, 1>(p, st);
    case 16: return launch_t<EPI, 6, 1>(p, st);
    case 18: return launch_t<EPI, 8, 1>(p, st);
    case 24: return launch_t<EPI, 4, 2>(p, st);
    case 26: return launch_t<EPI, 6, 2>(p, st);
    case 28: return launch_t<EPI, 8, 2>(p, st);
    default: return -1;
  }
}

template <int EPI, int V>
int cfg_v() {
  int e = 0;
  e |= (int)hipFuncSetAttribute((const void*)gemm_dec_kernel<EPI, 4, V>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes<4>());
  e |= (int)hipFuncSetAttribute((const void*)gemm_dec_kernel<EPI, 6, V>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes<6>());
  e |= (int)hipFuncSetAttribute((const void*)gemm_dec_kernel<EPI, 8, V>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes<8>());
  return e;
}

template <int EPI>
int cfg_e() { return cfg_v<EPI, 1>() | cfg_v<EPI, 2>(); }

}  // namespace

int launch_gemm_dec(void* c, const void* a, const void* b, const void* r, int M, int N, int K,
                    int lda, int ldb, int ldc, int ldr, int epi, int up_off, int cfg, int group_m,
                    hipStream_t st) {
  // shape contract (checked here so a bad call never reaches the device): N = columns of C
  const bool gated = epi == E_SILU || epi == E_GELU;
  if (M <= 0 || N <= 0 || K <= 0 || K % (2 * kPh)) return -1;
  if (gated ? (N % (kT / 2) || up_off != N) : (N % kT)) return -1;
  if (lda % 8 || ldb % 8 || ldc % 4 || lda < K || ldb < K || ldc < N) return -1;
  if (epi == E_RES && (r == nullptr || ldr % 4 || ldr < N)) return -1;
  if ((uintptr_t)a % 16 || (uintptr_t)b % 16 || (uintptr_t)c % 8 ||
      (epi == E_RES && (uintptr_t)r % 8))
    return -1;
  if (epi < 0 || epi > 3) return -1;
  DecParams p{};
  p.c = (bf16_t*)c;
  p.a = (const bf16_t*)a;
  p.b = (const bf16_t*)b;
  p.r = (const bf16_t*)r;
  p.M = M; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldr = ldr;
  p.tiles_m = (M + kT - 1) / kT;
  p.tiles_n = gated ? N / (kT / 2) : N / kT;
  p.up_off = up_off;
  p.group_m = group_m < 1 ? 8 : group_m;
  switch (epi) {
    case E_STORE: return launch_e<E_STORE>(p, cfg, st);
    case E_RES: return launch_e<E_RES>(p, cfg, st);
    case E_SILU: return launch_e<E_SILU>(p, cfg, st);
    default: return launch_e<E_GELU>(p, cfg, st);
  }
}

int configure_gemm_dec() {
  return cfg_e<E_STORE>() | cfg_e<E_RES>() | cfg_e<E_SILU>() | cfg_e<E_GELU>();
}

}  // namespace drtc
