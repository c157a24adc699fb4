// XCD-partitioned decode GEMM for gfx950 (MI355X):  c[M, N] = epi( a[M, K] . b[N, K]^T )
//
// The full-batch decode projections (M = 512..1024 rows of activations, N x K weights: Llama-3-8B
// qkv / o / down) have too few 256 x 256 tiles to fill 256 CUs (o: 4 x 16 = 64) and split-K
// pays a fp32 combine that costs what it saves (profiles/r3k_decode_gemm_limits.md,
// profiles/r4f).  This kernel takes the other road:
//
//   * 128 x (32 NF) output tiles, full K, ONE workgroup per tile and per CU (o / down at
//     M = 1024: 8 x 32 = 256 tiles with NF = 4; qkv N = 6144: 8 x 32 with NF = 6).
//   * Tile order partitioned by XCD (workgroup b runs on XCD b % 8 under round-robin dispatch -
//     used for speed only, the map below is a bijection of blockIdx): XCD x owns a contiguous
//     range of the column-major tile order, i.e. a contiguous set of weight column panels and
//     ALL row tiles of each.  Every weight byte is fetched from HBM into ONE XCD's L2, and the
//     tiles_m workgroups that share a panel stream it through that L2 in K-lockstep (the
//     activations, 1-8 MB, are read by every XCD from the Infinity Cache).
//   * 4 waves, one per SIMD, 64 x (16 NF) outputs per wave (4 x NF MFMA 16x16x32 tiles); the
//     16x16x32 form, not 32x32x16: same LDS bytes per FLOP at this wave tile, and the bf16
//     16x16x32 loop holds a 12-15 % higher clock on random data (MI355X_MICROARCH.md, DVFS
//     give-back item 7).
//   * LDS: S stages x [A 128 rows | B 32 NF rows] x 128 B (one 64-deep K tile), filled by
//     LDS-DMA (buffer_load_dwordx4 ... lds, 8 rows per wave-instruction), chunk c of row r
//     stored at c ^ ((r >> 1) & 7): conflict-free ds_read_b128 of the MFMA fragments (the same
//     involution on the DMA source address and on the read address).  S - 1 K tiles in flight
//     (96 KiB per CU at NF = 4) to cover L2 / Infinity-Cache latency with one wave per SIMD.
//   * Per K tile a fixed order pinned with sched_barrier: half 0 MFMAs | ds_read of half 1;
//     [vmcnt: own DMA of tile t + 1 landed, lgkmcnt(0), ONE barrier: everyone's tile t + 1
//     landed and every read of stage t done]; half 1 MFMAs | LDS-DMA of tile t + S into stage
//     t + ds_read of tile t + 1 half 0.
//   * Epilogue through LDS (the wave's tile as bf16, then 16-B row-contiguous global stores):
//     store, or + residual (may alias c).
#include "common.h"
#include "launchers.h"

#include <utility>

namespace drtc {
namespace {

typedef __attribute__((address_space(3))) void* xd_lds_ptr;

constexpr int kXdThreads = 256;
enum { XD_STORE = 0, XD_RESIDUAL = 1 };

template <int NF, int S_ = (NF <= 4 ? 4 : 3)>
struct XdGeom {
  static constexpr int TN = 32 * NF;               // tile columns
  static constexpr int H = 4 * NF;                 // MFMAs per 32-deep K half (per wave)
  static constexpr int DA = 4, DB = NF, D = DA + DB;  // LDS-DMA instructions per wave per K tile
  static constexpr int NR = 4 + NF;                // fragment reads per wave per K half
  static constexpr int BOFF = 128 * 128;           // B region within a stage
  static constexpr int STAGE = BOFF + TN * 128;
  static constexpr int S = S_;                     // stages (K tiles in the LDS ring)
  static constexpr int LDS = S * STAGE;
  static constexpr int PITCH = 32 * NF + 16;       // epilogue bytes per wave-tile row (padded)
  static_assert(4 * 64 * PITCH <= LDS, "epilogue image must fit the stages");
  static_assert(LDS <= 160 * 1024, "LDS ring exceeds the CU's 160 KiB");
};

struct XdParams {
  bf16_t* c;
  const bf16_t* a;
  const bf16_t* b;
  const bf16_t* r;
  int M, N, K;
  int lda, ldb, ldc, ldr;
  int tiles_m, tiles_n, per_xcd;
};

template <int NF>
struct XdDma {
  __amdgpu_buffer_rsrc_t ra, rb;
  unsigned va[4];
  unsigned vb[NF];
  unsigned lds_a, lds_b;  // LDS byte address of this wave's first DMA block in stage 0
};

// Fragment read offsets within a stage (bytes): row 64 wm + l16 (A) / 16 NF wn + l16 (B),
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

// One LDS-DMA wave-instruction outside the main loop: M0 saved and restored.
DRTC_DEVICE void xd_dma(unsigned dst, unsigned voff, __amdgpu_buffer_rsrc_t rsrc, unsigned soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(dst), "v"(voff), "s"(rsrc), "s"(soff)
      : "memory");
}

// Step Q of a K tile (0 .. 8 NF - 1): MFMA Q, then the memory work scheduled behind it.  All
// conditions are compile-time constants; sched_barrier(0) pins the emitted order.
// Main-loop DMA: M0 (the LDS destination) is set at the first DMA of each operand group and
// advanced by 1 KiB after each DMA; K advances through the scalar offset (nothing else in
// this kernel uses M0).
template <int NF, int S, bool DMA, bool NEXT, int WT, bool Z, int Q>
DRTC_DEVICE void xd_step(f32x4 (&acc)[4][NF], bf16x8 (&fa0)[4], bf16x8 (&fb0)[NF],
                         bf16x8 (&fa1)[4], bf16x8 (&fb1)[NF], const char* lds, int cur, int nxt,
                         unsigned kb, const XdFrag& f, const XdDma<NF>& d) {
  using G = XdGeom<NF, S>;
  constexpr int H = G::H;
  constexpr int h = Q / H, rem = Q % H, i = rem / NF, j = rem % NF;
  if constexpr (h == 0 && Z)  // first K tile: accumulate onto 0 (no zeroed AGPRs to coalesce)
    acc[i][j] = mfma16(fa0[i], fb0[j], (f32x4){0.f, 0.f, 0.f, 0.f});
  else if constexpr (h == 0)
    acc[i][j] = mfma16(fa0[i], fb0[j], acc[i][j]);
  else
    acc[i][j] = mfma16(fa1[i], fb1[j], acc[i][j]);
  // ---- half 0: fragments of this tile's half 1, in the order half 1 consumes them
  if constexpr (h == 0 && Q >= 1 && Q <= G::NR) {
    constexpr int r = Q - 1;
    if constexpr (r == 0)
      fa1[0] = xd_rd(lds, cur + f.ra1);
    else if constexpr (r <= NF)
      fb1[r - 1] = xd_rd(lds, cur + f.rb1 + 2048 * (r - 1));
    else
      fa1[r - NF] = xd_rd(lds, cur + f.ra1 + 2048 * (r - NF));
  }
  // ---- boundary: tile t + 1 landed for every wave; every read of this stage is done
  if constexpr (NEXT && Q == H - 1) {
    xd_vmcnt<WT * G::D>();  // WT younger K tiles of this wave may still be in flight
    xd_lgkm0();
    xd_barrier();
  }
  // ---- half 1: DMA of tile t + S into this stage (A group, then B group), one per
  // H / D MFMAs; the next tile's half-0 fragments in between
  if constexpr (DMA && h == 1) {
    constexpr int s0 = ((rem * G::D) + H - 1) / H;  // DMAs issued at steps < rem: ceil
    constexpr int s1 = (((rem + 1) * G::D) + H - 1) / H;
#pragma unroll
    for (int s = s0; s < s1; ++s) {
      if (s < G::DA) {
        if (s == 0)
          asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(d.lds_a + cur) : "memory");
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
                     : : "v"(d.va[s]), "s"(d.ra), "s"(kb) : "memory");
        if (s + 1 < G::DA) asm volatile("s_add_u32 m0, m0, 0x400" ::: "memory");
      } else {
        if (s == G::DA)
          asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(d.lds_b + cur) : "memory");
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
                     : : "v"(d.vb[s - G::DA]), "s"(d.rb), "s"(kb) : "memory");
        if (s + 1 < G::D) asm volatile("s_add_u32 m0, m0, 0x400" ::: "memory");
      }
    }
  }
  if constexpr (NEXT && h == 1) {
    constexpr int r0 = (rem * G::NR + H - 1) / H;
    constexpr int r1 = ((rem + 1) * G::NR + H - 1) / H;
#pragma unroll
    for (int r = r0; r < r1; ++r) {
      if (r == 0)
        fa0[0] = xd_rd(lds, nxt + f.ra0);
      else if (r <= NF)
        fb0[r - 1] = xd_rd(lds, nxt + f.rb0 + 2048 * (r - 1));
      else
        fa0[r - NF] = xd_rd(lds, nxt + f.ra0 + 2048 * (r - NF));
    }
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int NF, int S, bool DMA, bool NEXT, int WT, bool Z, int... Qs>
DRTC_DEVICE void xd_steps(std::integer_sequence<int, Qs...>, f32x4 (&acc)[4][NF],
                          bf16x8 (&fa0)[4], bf16x8 (&fb0)[NF], bf16x8 (&fa1)[4],
                          bf16x8 (&fb1)[NF], const char* lds, int cur, int nxt, unsigned kb,
                          const XdFrag& f, const XdDma<NF>& d) {
  (xd_step<NF, S, DMA, NEXT, WT, Z, Qs>(acc, fa0, fb0, fa1, fb1, lds, cur, nxt, kb, f, d), ...);
}

template <int NF, int S, bool DMA, bool NEXT, int WT, bool Z = false>
DRTC_DEVICE void xd_tile(f32x4 (&acc)[4][NF], bf16x8 (&fa0)[4], bf16x8 (&fb0)[NF],
                         bf16x8 (&fa1)[4], bf16x8 (&fb1)[NF], const char* lds, int cur, int nxt,
                         unsigned kb, const XdFrag& f, const XdDma<NF>& d) {
  xd_steps<NF, S, DMA, NEXT, WT, Z>(std::make_integer_sequence<int, 8 * NF>{}, acc, fa0, fb0, fa1, fb1,
                          lds, cur, nxt, kb, f, d);
}

template <int NF, int S, int WT>
DRTC_DEVICE void xd_tail(f32x4 (&acc)[4][NF], bf16x8 (&fa0)[4], bf16x8 (&fb0)[NF],
                         bf16x8 (&fa1)[4], bf16x8 (&fb1)[NF], const char* lds, int cur,
                         const XdFrag& f, const XdDma<NF>& d) {
  using G = XdGeom<NF, S>;
  if constexpr (WT < 0) {
    xd_tile<NF, S, false, false, 0>(acc, fa0, fb0, fa1, fb1, lds, cur, cur, 0u, f, d);
  } else {
    const int nxt = cur + G::STAGE == G::LDS ? 0 : cur + G::STAGE;
    xd_tile<NF, S, false, true, WT>(acc, fa0, fb0, fa1, fb1, lds, cur, nxt, 0u, f, d);
    xd_tail<NF, S, WT - 1>(acc, fa0, fb0, fa1, fb1, lds, nxt, f, d);
  }
}

template <int NF, int S, int EPI>
__global__ __launch_bounds__(kXdThreads, 1) void gemm_xd_kernel(XdParams p) {
  using G = XdGeom<NF, S>;
  extern __shared__ __attribute__((aligned(16))) char xd_lds[];
  // ---- tile: XCD label b % 8 owns tiles [x per_xcd, (x + 1) per_xcd) of the column-major
  // order (all row tiles of a weight panel consecutive)
  const int b = blockIdx.x;
  const int tid = (b & 7) * p.per_xcd + (b >> 3);
  if (tid >= p.tiles_m * p.tiles_n) return;
  const int tn = tid / p.tiles_m, tm = tid - tn * p.tiles_m;
  const int m0 = 128 * tm, n0 = G::TN * tn;

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wv >> 1, wn = wv & 1, l16 = lane & 15, g = lane >> 4;
  const int nk = p.K >> 6;

  // ---- DMA plan: instruction i of wave wv fills stage rows 32 wv + 8 i + (lane >> 3) (A) /
  // 8 NF wv + 8 i + (lane >> 3) (B), lane's LDS chunk lane & 7 <- source chunk ^ swizzle.
  // A rows past M read row M - 1 (valid bytes, never stored).
  XdDma<NF> d;
  const unsigned lds0 = (unsigned)(uintptr_t)(xd_lds_ptr)xd_lds;
  {
    const int rows_a = min(128, p.M - m0);
    const char* abase = reinterpret_cast<const char*>(p.a + (int64_t)m0 * p.lda);
    const char* bbase = reinterpret_cast<const char*>(p.b + (int64_t)n0 * p.ldb);
    d.ra = __builtin_amdgcn_make_buffer_rsrc((void*)abase, (short)0, 0x7FFFFFFF, 0x00020000);
    d.rb = __builtin_amdgcn_make_buffer_rsrc((void*)bbase, (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int R = 32 * wv + 8 * i + (lane >> 3);
      const int c = (lane & 7) ^ ((R >> 1) & 7);
      d.va[i] = (unsigned)(min(R, rows_a - 1) * p.lda * 2 + c * 16);
    }
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int R = 8 * NF * wv + 8 * i + (lane >> 3);
      const int c = (lane & 7) ^ ((R >> 1) & 7);
      d.vb[i] = (unsigned)(R * p.ldb * 2 + c * 16);
    }
    d.lds_a = __builtin_amdgcn_readfirstlane(lds0 + 32 * wv * 128);
    d.lds_b = __builtin_amdgcn_readfirstlane(lds0 + G::BOFF + 8 * NF * wv * 128);
  }
  XdFrag f;
  {
    const int fx = (l16 >> 1) & 7;
    f.ra0 = (64 * wm + l16) * 128 + ((0 + g) ^ fx) * 16;
    f.ra1 = (64 * wm + l16) * 128 + ((4 + g) ^ fx) * 16;
    f.rb0 = G::BOFF + (16 * NF * wn + l16) * 128 + ((0 + g) ^ fx) * 16;
    f.rb1 = G::BOFF + (16 * NF * wn + l16) * 128 + ((4 + g) ^ fx) * 16;
  }
  const char* lds = xd_lds;

  f32x4 acc[4][NF];  // written first by the K tile 0 MFMAs (onto a zero C operand)

  // ---- prologue: K tiles 0 .. S-1 into the S stages (the launcher guarantees nk > S)
#pragma unroll
  for (int u = 0; u < G::S; ++u) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      xd_dma(d.lds_a + u * G::STAGE + 1024 * i, d.va[i], d.ra, (unsigned)u * 128u);
#pragma unroll
    for (int i = 0; i < NF; ++i)
      xd_dma(d.lds_b + u * G::STAGE + 1024 * i, d.vb[i], d.rb, (unsigned)u * 128u);
  }
  xd_vmcnt<(G::S - 1) * G::D>();
  xd_barrier();
  bf16x8 fa0[4], fb0[NF], fa1[4], fb1[NF];
  fa0[0] = xd_rd(lds, f.ra0);
#pragma unroll
  for (int j = 0; j < NF; ++j) fb0[j] = xd_rd(lds, f.rb0 + 2048 * j);
#pragma unroll
  for (int i = 1; i < 4; ++i) fa0[i] = xd_rd(lds, f.ra0 + 2048 * i);

  // ---- main loop: tile t in stage cur; its half 1 DMAs tile t + S into the same stage
  xd_tile<NF, S, true, true, G::S - 2, true>(acc, fa0, fb0, fa1, fb1, lds, 0, G::STAGE,
                                          (unsigned)G::S * 128u, f, d);
  int cur = G::STAGE;
  for (int t = 1; t + G::S < nk; ++t) {
    const int nxt = cur + G::STAGE == G::LDS ? 0 : cur + G::STAGE;
    xd_tile<NF, S, true, true, G::S - 2>(acc, fa0, fb0, fa1, fb1, lds, cur, nxt,
                                      (unsigned)(t + G::S) * 128u, f, d);
    cur = nxt;
  }
  // the last S tiles: nothing more to load; S - 2, ..., 0 younger tiles still in flight
  xd_tail<NF, S, G::S - 2>(acc, fa0, fb0, fa1, fb1, lds, cur, f, d);
  xd_vmcnt<0>();

  // ---- epilogue: the wave's 64 x 16 NF tile as bf16 into LDS, then 16-B global stores of
  // whole row segments (acc[i][j][r] = C[64 wm + 16 i + 4 g + r][16 NF wn + 16 j + l16])
  __syncthreads();  // every wave is done reading the stages
  char* ep = xd_lds + wv * 64 * G::PITCH;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<bf16_t*>(ep + (16 * i + 4 * g + r) * G::PITCH + (16 * j + l16) * 2) =
            f2bf(acc[i][j][r]);
  __syncthreads();
  constexpr int CPR = 2 * NF;  // 16-B chunks per wave-tile row
#pragma unroll
  for (int s = 0; s < CPR; ++s) {
    const int q = lane + 64 * s;
    const int row = q / CPR, ch = q - row * CPR;
    const int m = m0 + 64 * wm + row;
    if (m >= p.M) continue;
    const int n = n0 + 16 * NF * wn + 8 * ch;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(ep + row * G::PITCH + ch * 16);
    if constexpr (EPI == XD_RESIDUAL) {
      const bf16x8 rv = *reinterpret_cast<const bf16x8*>(p.r + (int64_t)m * p.ldr + n);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(rv[e]));
    }
    *reinterpret_cast<bf16x8*>(p.c + (int64_t)m * p.ldc + n) = v;
  }
}

template <int NF, int S, int EPI>
int xd_launch(const XdParams& p, hipStream_t st) {
  hipLaunchKernelGGL((gemm_xd_kernel<NF, S, EPI>), dim3(8 * p.per_xcd), dim3(kXdThreads),
                     (XdGeom<NF, S>::LDS), st, p);
  return (int)hipGetLastError();
}

template <int NF, int S>
int xd_launch_s(const XdParams& p, bool res, hipStream_t st) {
  return res ? xd_launch<NF, S, XD_RESIDUAL>(p, st) : xd_launch<NF, S, XD_STORE>(p, st);
}

template <int NF, int S>
int xd_cfg() {
  return (int)hipFuncSetAttribute((const void*)gemm_xd_kernel<NF, S, XD_STORE>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  XdGeom<NF, S>::LDS) |
         (int)hipFuncSetAttribute((const void*)gemm_xd_kernel<NF, S, XD_RESIDUAL>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  XdGeom<NF, S>::LDS);
}

// (nf, stages) forms built: nf 2 with 4 / 6 stages, nf 4 with 4 / 5, nf 6 with 3 / 4
int xd_default_stages(int nf) { return nf <= 4 ? 4 : 3; }
bool xd_form(int nf, int s) {
  return (nf == 2 && (s == 4 || s == 6)) || (nf == 4 && (s == 4 || s == 5)) ||
         (nf == 6 && (s == 3 || s == 4));
}

}  // namespace

int launch_gemm_xd(void* c, const void* a, const void* b, const void* r, int M, int N, int K,
                   int lda, int ldb, int ldc, int ldr, int epi, int nf, int stages,
                   hipStream_t st) {
  if (epi != XD_STORE && epi != XD_RESIDUAL) return -1;
  if (stages == 0) stages = xd_default_stages(nf);
  if (!xd_form(nf, stages)) return -1;
  if (lda % 8 || ldb % 8 || ldc % 8) return -1;
  if ((uintptr_t)a % 16 || (uintptr_t)b % 16 || (uintptr_t)c % 16) return -1;
  if (epi == XD_RESIDUAL && (r == nullptr || ldr % 8 || (uintptr_t)r % 16)) return -1;
  const int tn = 32 * nf;
  // shape contract: whole column tiles, K tiles beyond the ring (the first K tile is peeled),
  // 32-bit buffer offsets from each tile's operand bases
  if (M <= 0 || N <= 0 || N % tn || K % 64 || K / 64 <= stages) return -1;
  if ((int64_t)128 * lda * 2 >= (1ll << 31) || (int64_t)tn * ldb * 2 >= (1ll << 31)) return -1;
  XdParams p{};
  p.c = (bf16_t*)c;
  p.a = (const bf16_t*)a;
  p.b = (const bf16_t*)b;
  p.r = (const bf16_t*)r;
  p.M = M; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldr = ldr;
  p.tiles_m = (M + 127) / 128;
  p.tiles_n = N / tn;
  const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
  if (tiles * 8 >= (1ll << 31)) return -1;
  p.per_xcd = (int)((tiles + 7) / 8);
  const bool res = epi == XD_RESIDUAL;
  switch (nf * 16 + stages) {
    case 2 * 16 + 4: return xd_launch_s<2, 4>(p, res, st);
    case 2 * 16 + 6: return xd_launch_s<2, 6>(p, res, st);
    case 4 * 16 + 4: return xd_launch_s<4, 4>(p, res, st);
    case 4 * 16 + 5: return xd_launch_s<4, 5>(p, res, st);
    case 6 * 16 + 3: return xd_launch_s<6, 3>(p, res, st);
    default: return xd_launch_s<6, 4>(p, res, st);
  }
}

int configure_gemm_xd() {
  return xd_cfg<2, 4>() | xd_cfg<2, 6>() | xd_cfg<4, 4>() | xd_cfg<4, 5>() | xd_cfg<6, 3>() |
         xd_cfg<6, 4>();
}

}  // namespace drtc
