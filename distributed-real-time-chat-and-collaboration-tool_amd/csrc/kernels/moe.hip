// Mixture-of-experts on MFMA (gfx950): routing, grouped GEMMs, combine.
// Static launch shapes (device-side tile table), so the whole MoE layer is
// hipGraph-capturable - the decode step of Mixtral replays with no host sync.
//
//   moe_route / offsets / scatter   top-k over the router logits (+ softmax over the
//                         selected logits), stable counting sort of the (token, slot)
//                         pairs by expert, per-expert row-tile table.
//   moe_gate_up_kernel    grouped GEMM  H[p] = act(X[tok(p)] . Wg[e]^T) * (X[tok(p)] . Wu[e]^T)
//                         with the gate|up activation fused in the epilogue: a
//                         wave owns matching gate and up columns, so both MFMA
//                         accumulators of an output element sit in one lane.
//   moe_down_kernel       grouped GEMM  Z[p] = H[p] . Wd[e]^T
//   moe_combine_kernel    out[t] = sum_j w[t,j] * Z[pos(t,j)]   (fp32, fixed order:
//                         deterministic, no atomics)
//
// GEMM structure: 256-thread workgroup, 2x2 waves, 128-row tile; operands are
// K-contiguous rows (activations gathered by token, weights [N][K]) loaded as
// 16-B fragments straight into registers (register double buffer over the K
// loop), 16 MFMA 16x16x32 per wave per k-step.
#include "common.h"
#include "launchers.h"

#include <initializer_list>

namespace drtc {

constexpr int kMoeBM = 128;   // rows per tile
constexpr int kMoeMaxK = 8;   // top-k bound
constexpr int kMoeW4Rows = 256;  // auto variant 4 from this many rows per expert
constexpr int kMoeW4SplitTiles = 256;  // variant 4: down split over K below this many tiles
// variant 4 row-tile groups of the grouped gemm_w4 tile order (gate_up, down): A/B knob
static int g_moe_gm_gu = 4, g_moe_gm_dn = 8;
void moe_set_w4_group_m(int gu, int dn) {
  g_moe_gm_gu = gu > 0 ? gu : 4;
  g_moe_gm_dn = dn > 0 ? dn : 8;
}

// ---------------------------------------------------------------- routing
// Three passes over workgroups of 256 tokens (one workgroup for all T was 89 us at T = 8192,
// profiles/r6j - 2 % of a Mixtral prefill MoE layer):
//   moe_route_kernel    top-k of each token's logits (+ softmax over the selected k), and the
//                       workgroup's per-expert pair counts;
//   moe_offsets_kernel  one workgroup: expert offsets, the per-expert tile table, the expert
//                       row groups (variant 4), and each (workgroup, expert)'s first position;
//   moe_scatter_kernel  every pair to its position in expert order: within an expert, pairs of
//                       lower workgroups first, then (slot j, token) order - a STABLE order, the
//                       same for the same logits whatever the scheduling.
constexpr int kMoeRouteWG = 256;

__global__ __launch_bounds__(kMoeRouteWG) void moe_route_kernel(
    const bf16_t* __restrict__ logits, int T, int E, int k, int lts, int les,
    int* __restrict__ topi, float* __restrict__ topk_w, int* __restrict__ wg_cnt) {
  __shared__ int hist[256];
  const int tid = threadIdx.x;
  for (int e = tid; e < E; e += kMoeRouteWG) hist[e] = 0;
  __syncthreads();
  const int t = blockIdx.x * kMoeRouteWG + tid;
  if (t < T) {
    // logit (t, e) at t * lts + e * les: [T, E] rows, or the router GEMM's [E, T] output read
    // in place (lts = 1: consecutive threads read consecutive tokens of one expert row)
    const bf16_t* lr = logits + (int64_t)t * lts;
    // sorted top-8 list kept in registers (fully unrolled: no scratch)
    float v[kMoeMaxK];
    int id[kMoeMaxK];
#pragma unroll
    for (int j = 0; j < kMoeMaxK; ++j) { v[j] = -INFINITY; id[j] = 0x7fffffff; }
    for (int e = 0; e < E; ++e) {
      float x = bf2f(lr[(int64_t)e * les]);
      int xi = e;
#pragma unroll
      for (int j = 0; j < kMoeMaxK; ++j) {
        // order (value desc, id asc): a displaced entry carried down the list
        // must not overtake an equal-valued entry with a higher id
        if (x > v[j] || (x == v[j] && xi < id[j])) {
          const float tv = v[j]; const int ti = id[j];
          v[j] = x; id[j] = xi; x = tv; xi = ti;
        }
      }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kMoeMaxK; ++j) s += (j < k) ? __expf(v[j] - v[0]) : 0.f;
#pragma unroll
    for (int j = 0; j < kMoeMaxK; ++j) {
      if (j < k) {
        topk_w[t * k + j] = __expf(v[j] - v[0]) / s;
        topi[t * k + j] = id[j];
        atomicAdd(&hist[id[j]], 1);  // a count: its order does not matter
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < E; e += kMoeRouteWG) wg_cnt[blockIdx.x * E + e] = hist[e];
}

__global__ __launch_bounds__(1024) void moe_offsets_kernel(
    const int* __restrict__ wg_cnt, int G, int E, int* __restrict__ wg_base,
    int* __restrict__ tile_expert, int* __restrict__ tile_row0, int* __restrict__ tile_rows,
    int* __restrict__ n_tiles, int* __restrict__ local_range, int max_tiles, int e_off,
    int e_local, int bm, int* __restrict__ grp_off) {
  __shared__ int cnt[256], off[257], toff[257];
  const int tid = threadIdx.x;
  for (int e = tid; e < E; e += 1024) {
    int c = 0;
    for (int g = 0; g < G; ++g) c += wg_cnt[g * E + e];
    cnt[e] = c;
  }
  __syncthreads();
  if (tid == 0) {
    int o = 0, to = 0;
    for (int e = 0; e < E; ++e) {  // tiles only for this rank's experts (EP)
      const bool loc = e >= e_off && e < e_off + e_local;
      off[e] = o;
      toff[e] = to;
      o += cnt[e];
      to += loc ? (cnt[e] + bm - 1) / bm : 0;
    }
    off[E] = o;
    toff[E] = to;
    n_tiles[0] = to < max_tiles ? to : max_tiles;
    local_range[0] = off[e_off];
    local_range[1] = off[e_off + e_local];
  }
  __syncthreads();
  // variant 4: this rank's expert row groups in the sorted order (absolute positions)
  if (grp_off != nullptr && tid <= e_local) grp_off[tid] = off[e_off + tid];
  for (int e = tid; e < E; e += 1024) {
    const int nt = toff[e + 1] - toff[e];
    for (int i = 0; i < nt; ++i) {
      const int ti = toff[e] + i;
      if (ti < max_tiles) {
        tile_expert[ti] = e - e_off;  // local weight index
        tile_row0[ti] = off[e] + i * bm;
        tile_rows[ti] = min(bm, cnt[e] - i * bm);
      }
    }
    int b = off[e];
    for (int g = 0; g < G; ++g) {
      wg_base[g * E + e] = b;
      b += wg_cnt[g * E + e];
    }
  }
}

__global__ __launch_bounds__(kMoeRouteWG) void moe_scatter_kernel(
    const float* __restrict__ topk_w, const int* __restrict__ wg_base, int T, int E, int k,
    int* __restrict__ sorted_tok, float* __restrict__ sorted_w, int* __restrict__ inv_pos) {
  // inv_pos holds each pair's expert id (moe_route_kernel) and gets its position here
  __shared__ int run[256];
  __shared__ int wcnt[kMoeRouteWG / 64][256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int t = blockIdx.x * kMoeRouteWG + tid;
  const uint64_t below = (1ull << lane) - 1;
  for (int e = tid; e < E; e += kMoeRouteWG) run[e] = 0;
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    const int e = t < T ? inv_pos[t * k + j] : -1;
    int rank = 0;
    for (int x = 0; x < E; ++x) {  // this wave's pairs of expert x, in lane order
      const uint64_t m = __ballot(e == x);
      if (e == x) rank = __popcll(m & below);
      if (lane == 0) wcnt[w][x] = __popcll(m);
    }
    __syncthreads();
    if (e >= 0) {
      int r = run[e] + rank;
      for (int w2 = 0; w2 < w; ++w2) r += wcnt[w2][e];
      const int p = wg_base[blockIdx.x * E + e] + r;
      sorted_tok[p] = t;
      sorted_w[p] = topk_w[t * k + j];
      inv_pos[t * k + j] = p;
    }
    __syncthreads();
    for (int x = tid; x < E; x += kMoeRouteWG) {
      int c = 0;
#pragma unroll
      for (int w2 = 0; w2 < kMoeRouteWG / 64; ++w2) c += wcnt[w2][x];
      run[x] += c;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- GEMMs
// One grouped-GEMM kernel for both projections.  Tile 128 (pair rows) x 128
// (weight rows) x BK 64; 4 waves in 2x2, each owning a 64x64 accumulator
// (4x4 MFMA 16x16x32 tiles).  Both operands are K-contiguous rows, staged
// global -> LDS with global_load_lds_dwordx4 (16 B per lane, lane-linear LDS
// image; the gather of token rows is free because the source address is
// per lane).  Bank conflicts of the ds_read_b128 fragment reads are removed
// by an XOR swizzle of the 16-B chunk index with (row >> 1) & 7, applied to
// the per-lane SOURCE address and to the read address (the two sides of the
// same involution; cdna_hip_programming.md rule 21).  With 128-B rows two
// rows share a 256-B bank row, so (row & 1, (row >> 1) & 7) picks 16
// distinct 16-B slots for the 16 lanes of a read group: conflict-free.
// Two LDS buffers (64 KiB, 2 workgroups per CU): tile k+1 streams in while
// tile k feeds the MFMAs.
//
// MODE 0 (gate_up): B rows 0..63 = gate rows n0.., rows 64..127 = the
//   matching up rows I+n0..; the epilogue writes act(gate) * up, 64 columns.
// MODE 1 (down): B rows = output columns n0..n0+127.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int kBK = 64;
constexpr int kTileElems = 128 * kBK;  // one operand tile (16 KiB)

DRTC_DEVICE void glds16(const bf16_t* src, bf16_t* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)lds_base, 16, 0, 0);
}

template <int MODE>
__global__ __launch_bounds__(256, 2) void moe_gemm_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ a, const bf16_t* __restrict__ w,
    const int* __restrict__ sorted_tok, const int* __restrict__ tile_expert,
    const int* __restrict__ tile_row0, const int* __restrict__ tile_rows,
    const int* __restrict__ n_tiles, int K, int w_rows, int I, int ldo, int max_tiles,
    int act) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[4 * kTileElems];  // [buf][A|B][128][64]
  // XCD-aware remap: contiguous chunks of the launch order share an XCD (L2),
  // and tile (row block) varies fastest, so all row blocks of one weight
  // panel run on the same XCD and re-read the panel from its L2.
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, rmd = nwg & 7;
  const int wgid = (xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q) + (orig >> 3);
  const int tile = wgid % max_tiles, ct = wgid / max_tiles;
  if (tile >= n_tiles[0]) return;
  const int e = tile_expert[tile], r0 = tile_row0[tile], nr = tile_rows[tile];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wv >> 1, wc = wv & 1, l16 = lane & 15, g = lane >> 4;

  // staging sources: wave wv stages rows [32wv, 32wv+32) of both operands,
  // 8 rows (8 lanes x 16 B each) per glds instruction
  const bf16_t* asrc[4];
  const bf16_t* bsrc[4];
  const bf16_t* we = w + (int64_t)e * w_rows * K;
  const int n0 = MODE == 0 ? 64 * ct : 128 * ct;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 32 * wv + 8 * i + (lane >> 3);
    const int d = (lane & 7) ^ ((r >> 1) & 7);  // source chunk for this LDS slot
    const int rr = r < nr ? r : 0;
    const int64_t arow = MODE == 0 ? (int64_t)sorted_tok[r0 + rr] : (int64_t)(r0 + rr);
    asrc[i] = a + arow * K + 8 * d;
    const int wrow = MODE == 0 ? (r < 64 ? n0 + r : I + n0 + r - 64) : n0 + r;
    bsrc[i] = we + (int64_t)wrow * K + 8 * d;
  }
  auto stage = [&](int kt, int buf) {
    bf16_t* A = lds + buf * 2 * kTileElems;
    bf16_t* B = A + kTileElems;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(asrc[i] + kt * kBK, A + (32 * wv + 8 * i) * kBK);
      glds16(bsrc[i] + kt * kBK, B + (32 * wv + 8 * i) * kBK);
    }
  };
  // fragment read offsets (elements) within a tile, per k-substep s
  const int rsw = (l16 >> 1) & 7;
  const int off0 = l16 * kBK + ((0 + g) ^ rsw) * 8;
  const int off1 = l16 * kBK + ((4 + g) ^ rsw) * 8;
  int brow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    brow[j] = MODE == 0 ? (j < 2 ? 32 * wc + 16 * j : 64 + 32 * wc + 16 * (j - 2))
                        : 64 * wc + 16 * j;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / kBK;
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const bf16_t* A = lds + cur * 2 * kTileElems;
    const bf16_t* B = A + kTileElems;
    // k-substep 0 fragments first: its 16 MFMAs wait only for the first 8
    // LDS reads (lgkmcnt counts in order), substep 1's reads overlap them
    bf16x8 fa0[4], fa1[4], fb0[4], fb1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa0[i] = *(const bf16x8*)(A + (64 * wr + 16 * i) * kBK + off0);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb0[j] = *(const bf16x8*)(B + brow[j] * kBK + off0);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa1[i] = *(const bf16x8*)(A + (64 * wr + 16 * i) * kBK + off1);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb1[j] = *(const bf16x8*)(B + brow[j] * kBK + off1);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fa0[i], fb0[j], acc[i][j]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fa1[i], fb1[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    __syncthreads();  // retires the glds of tile kt+1 (vmcnt) and the reads of tile kt
  }

  // epilogue: C lane map row 4g+r, col l16 of each 16x16 tile
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 64 * wr + 16 * i + 4 * g + r;
      if (row >= nr) continue;
      bf16_t* orow = out + (int64_t)(r0 + row) * ldo;
      if constexpr (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float gt = acc[i][j][r], up = acc[i][j + 2][r];
          float av;
          if (act == 0) {
            av = gt / (1.f + __expf(-gt));
          } else {
            const float inner = 0.7978845608028654f * (gt + 0.044715f * gt * gt * gt);
            av = 0.5f * gt * (1.f + tanhf(inner));
          }
          orow[n0 + 32 * wc + 16 * j + l16] = f2bf(av * up);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) orow[n0 + 64 * wc + 16 * j + l16] = f2bf(acc[i][j][r]);
      }
    }
}

// ------------------------------------------------------ pipelined GEMM
// Same operand/epilogue contract as moe_gemm_kernel, restructured for the
// glds-pipelined regime (cdna_hip_programming.md §5 "Pipelining across
// barriers"): THREE LDS stages, two k-tiles in flight.  Each k-step waits
// with a COUNTED vmcnt (the youngest tile may stay in flight), passes a raw
// s_barrier (no vmcnt(0) drain, unlike __syncthreads with an LDS-DMA
// outstanding), then issues the tile two steps ahead into the stage freed
// by the previous step.  BM = 256 doubles the MFMA work per staged byte
// (8 waves, 4x2, each 64x64) - the prefill shape; BM = 128 keeps 4 waves.
// All LDS is one dynamic array (a second __shared__ object can make hipcc
// drain vmcnt before every ds_read: §5 trap 4a).
template <int BM>
struct PipeCfg {
  static constexpr int BN = 128;
  static constexpr int WM = BM / 64, WN = 2, NW = WM * WN, NT = NW * 64;
  static constexpr int ROWS = BM + BN;          // staged rows per k-tile
  static constexpr int GPW = ROWS / (8 * NW);   // glds per wave per stage
  static constexpr int STAGE = ROWS * kBK;      // elements per stage
  static constexpr int LDS_BYTES = 3 * STAGE * 2;
};

template <int N>
DRTC_DEVICE void wait_vmcnt() {
  // gfx9 s_waitcnt immediate: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt_hi[15:14]
  constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
  __builtin_amdgcn_s_waitcnt(imm);
}

template <int BM, int MODE>
__global__ __launch_bounds__(PipeCfg<BM>::NT, 1) void moe_gemm_pipe_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ a, const bf16_t* __restrict__ w,
    const int* __restrict__ sorted_tok, const int* __restrict__ tile_expert,
    const int* __restrict__ tile_row0, const int* __restrict__ tile_rows,
    const int* __restrict__ n_tiles, int K, int w_rows, int I, int ldo, int max_tiles,
    int act) {
  using C = PipeCfg<BM>;
  extern __shared__ __attribute__((aligned(16))) bf16_t plds[];  // [3][ROWS][64]
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, rmd = nwg & 7;
  const int wgid = (xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q) + (orig >> 3);
  const int tile = wgid % max_tiles, ct = wgid / max_tiles;
  if (tile >= n_tiles[0]) return;
  const int e = tile_expert[tile], r0 = tile_row0[tile], nr = tile_rows[tile];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wv / C::WN, wc = wv % C::WN, l16 = lane & 15, g = lane >> 4;

  const bf16_t* src[C::GPW];
  const bf16_t* we = w + (int64_t)e * w_rows * K;
  const int n0 = MODE == 0 ? (C::BN / 2) * ct : C::BN * ct;
#pragma unroll
  for (int i = 0; i < C::GPW; ++i) {
    const int r = (C::GPW * 8) * wv + 8 * i + (lane >> 3);  // staged row (A rows, then B rows)
    const int d = (lane & 7) ^ ((r >> 1) & 7);
    if (r < BM) {
      const int rr = r < nr ? r : 0;
      const int64_t arow = MODE == 0 ? (int64_t)sorted_tok[r0 + rr] : (int64_t)(r0 + rr);
      src[i] = a + arow * K + 8 * d;
    } else {
      const int br = r - BM;
      const int wrow = MODE == 0 ? (br < C::BN / 2 ? n0 + br : I + n0 + br - C::BN / 2) : n0 + br;
      src[i] = we + (int64_t)wrow * K + 8 * d;
    }
  }
  auto stage = [&](int kt, int buf) {
    bf16_t* base = plds + buf * C::STAGE + (C::GPW * 8) * wv * kBK;
#pragma unroll
    for (int i = 0; i < C::GPW; ++i) glds16(src[i] + kt * kBK, base + 8 * i * kBK);
  };
  const int rsw = (l16 >> 1) & 7;
  const int off0 = l16 * kBK + ((0 + g) ^ rsw) * 8;
  const int off1 = l16 * kBK + ((4 + g) ^ rsw) * 8;
  int brow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    brow[j] = BM + (MODE == 0 ? (j < 2 ? 32 * wc + 16 * j : C::BN / 2 + 32 * wc + 16 * (j - 2))
                              : 64 * wc + 16 * j);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / kBK;
  stage(0, 0);
  if (nk > 1) stage(1, 1);
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) wait_vmcnt<C::GPW>();  // tile kt landed; tile kt+1 may still fly
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + 2 < nk) stage(kt + 2, cur == 0 ? 2 : cur - 1);  // the stage read in step kt-1
    const bf16_t* A = plds + cur * C::STAGE;
    bf16x8 fa0[4], fa1[4], fb0[4], fb1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa0[i] = *(const bf16x8*)(A + (64 * wr + 16 * i) * kBK + off0);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb0[j] = *(const bf16x8*)(A + brow[j] * kBK + off0);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa1[i] = *(const bf16x8*)(A + (64 * wr + 16 * i) * kBK + off1);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb1[j] = *(const bf16x8*)(A + brow[j] * kBK + off1);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fa0[i], fb0[j], acc[i][j]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fa1[i], fb1[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    cur = cur == 2 ? 0 : cur + 1;
  }

#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 64 * wr + 16 * i + 4 * g + r;
      if (row >= nr) continue;
      bf16_t* orow = out + (int64_t)(r0 + row) * ldo;
      if constexpr (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float gt = acc[i][j][r], up = acc[i][j + 2][r];
          float av;
          if (act == 0) {
            av = gt / (1.f + __expf(-gt));
          } else {
            const float inner = 0.7978845608028654f * (gt + 0.044715f * gt * gt * gt);
            av = 0.5f * gt * (1.f + tanhf(inner));
          }
          orow[n0 + 32 * wc + 16 * j + l16] = f2bf(av * up);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) orow[n0 + 64 * wc + 16 * j + l16] = f2bf(acc[i][j][r]);
      }
    }
}

// Variant 4: the pairs' token rows copied into expert order, xs[p] = x[sorted_tok[p]] for this
// rank's positions (16 B per lane; a row of H bf16 per workgroup pass).
__global__ __launch_bounds__(256) void moe_gather_kernel(bf16_t* __restrict__ xs,
                                                         const bf16_t* __restrict__ x,
                                                         const int* __restrict__ sorted_tok,
                                                         const int* __restrict__ local_range,
                                                         int P, int H) {
  const int lo = local_range[0], hi = local_range[1];
  for (int p = lo + blockIdx.x; p < hi; p += gridDim.x) {
    const bf16_t* src = x + (int64_t)sorted_tok[p] * H;
    bf16_t* dst = xs + (int64_t)p * H;
    for (int c = threadIdx.x * 8; c < H; c += 256 * 8) store_bf16x8(dst + c, load_bf16x8(src + c));
  }
}

__global__ __launch_bounds__(256) void moe_combine_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ zbuf, const bf16_t* __restrict__ zbuf2,
    const float* __restrict__ topk_w, const int* __restrict__ inv_pos,
    const int* __restrict__ local_range, int T, int H, int k) {
  const int t = blockIdx.x;
  const int lo = local_range[0], hi = local_range[1];
  for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const int p = inv_pos[t * k + j];
      if (p < lo || p >= hi) continue;  // pair routed to another EP rank
      const float w = topk_w[t * k + j];
      const bf16x8 z = load_bf16x8(zbuf + (int64_t)p * H + c);
      if (zbuf2 != nullptr) {  // down split over K: the two halves' partial products
        const bf16x8 z2 = load_bf16x8(zbuf2 + (int64_t)p * H + c);
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] += w * (bf2f(z[q]) + bf2f(z2[q]));
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] += w * bf2f(z[q]);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(s[q]);
    store_bf16x8(out + (int64_t)t * H + c, o);
  }
}

// Whether grouped gemm_xd form `form` takes an expert GEMM with N output columns (gated: I)
// and reduction K (the 1x4 / 2x4 / 2x8 tiles launch_gemm_xd_grouped builds).
static bool moe_xd_ok(int form, int N, int K, bool glu) {
  const int mt = (form % 1000) / 100, nf = form / 10 % 10, sk = form % 10;
  const int st = mt == 1 ? (nf == 4 ? 4 : 0) : (mt == 2 ? (nf == 4 ? 3 : (nf == 8 ? 2 : 0)) : 0);
  if (st == 0 || sk < 1 || sk > 8 || form >= 2000) return false;
  const int tno = glu ? 16 * nf : 32 * nf;
  return N % tno == 0 && K % 64 == 0 && K / 64 / sk > st;
}

// xd form (mt * 100 + nf * 10 + splitk, + 1000 non-temporal weights) -> launcher fields
static void moe_xd_form(int form, int& mt, int& nf, int& sk) {
  mt = (form % 1000) / 100 | (form >= 1000 ? 16 : 0);
  nf = form / 10 % 10;
  sk = form % 10;
}

int launch_moe(void* out, const void* x, const void* router_logits, const void* w_gu,
               const void* w_dn, int T, int H, int I, int E, int k, int e_off, int e_local,
               int act, void* workspace, int64_t ws_bytes, int variant, int gu_form, int dn_form,
               void* slab, int64_t slab_bytes, int* counters, int n_counters, int logit_ts,
               int logit_es, hipStream_t st) {
  if (T == 0) return 0;
  if (!((logit_ts == E && logit_es == 1) || (logit_ts == 1 && logit_es >= T))) return -1;
  if (E > 256 || k > kMoeMaxK || k < 1 || k > E || H % 128 != 0 || I % 64 != 0 || H % kBK != 0 ||
      e_off < 0 || e_local < 1 || e_off + e_local > E)
    return -1;
  const int P = T * k;
  // GEMM structure: 0 = 128-row 2-barrier (small tiles, decode), 1 = 128-row
  // 3-stage pipeline, 2 = 256-row 3-stage pipeline, 3 = gemm_xd grouped mode (gate_up with
  // the GLU in its epilogue and down, forms gu_form / dn_form; 0 = by rows per expert);
  // -1 = pick by rows per expert (scripts/moe_bench.py, Mixtral shapes)
  const int rows_e = P / e_local;
  const bool auto_v = variant < 0;
  // variant 4 from one 256-row tile per expert (gemm_w4's persistent 256 x 256 tiles over
  // expert-ordered rows; Mixtral shapes, profiles/r6j: 770 / 917 / 1061 TF/s at T = 1024 /
  // 2048 / 4096 against 703 / 841 / 1019 on variant 3), gemm_xd's grouped forms from ~a
  // 96-row tile
  if (auto_v) variant = rows_e >= kMoeW4Rows ? 4 : (rows_e >= 96 ? 3 : 1);
  if (variant > 4) return -1;
  // variant 4: the persistent GEMM's prologue stages two K tiles; the down reduction is I
  if (variant == 4 && (H / 64 < 2 || I % 128 || I / 64 < 2 || H % 256)) {
    if (!auto_v) return -1;
    variant = 3;
  }
  // variant 4 with dn_form: down on a 256-row gemm_xd grouped form (the tile table's rows)
  if (variant == 4 && dn_form && ((dn_form % 1000) / 100 != 2 || !moe_xd_ok(dn_form, H, I, false))) {
    if (!auto_v) return -1;
    variant = 3;  // a down form requested for variant 3 (DRTC_MOE_DN_FORM) keeps its variant
  }
  if (variant == 3) {
    // 256-row tiles from ~1.5 tiles of rows per expert, else 128-row; 256 gated columns
    // (128 outputs) for gate_up where I allows; down with split-K 2 while the grid is below
    // ~2 rounds of CUs; non-temporal weights where an expert's rows fit one tile (each
    // weight byte is read by one workgroup)
    const bool gu_auto = gu_form == 0;  // an explicitly requested form runs as given
    if (gu_auto) {
      for (int f : rows_e >= 96 ? std::initializer_list<int>{281, 241} :
                                  std::initializer_list<int>{141})
        if (moe_xd_ok(f, I, H, true)) { gu_form = f; break; }
    }
    const int mt0 = (gu_form % 1000) / 100, bm0 = 128 * mt0;
    if (gu_auto && gu_form && gu_form < 1000 && rows_e <= bm0) gu_form += 1000;
    if (dn_form == 0 && gu_form) {
      const int64_t max_t = (P + bm0 - 1) / bm0 + e_local;
      for (int f : mt0 == 2 ? std::initializer_list<int>{282, 281, 242, 241} :
                              std::initializer_list<int>{142, 141}) {
        // split-K 2 while the grid is below ~2 rounds of CUs and its fp32 partial slots fit
        const int nf = f / 10 % 10;
        const int64_t tiles = max_t * (H / (32 * nf));
        const bool split = tiles < 512 && slab != nullptr && n_counters >= 2 * tiles + 2 &&
                           slab_bytes >= tiles * 2 * bm0 * (32 * nf) * 4;
        if (!split && f % 10 > 1) continue;
        if (moe_xd_ok(f, H, I, false)) { dn_form = f; break; }
      }
      if (dn_form && rows_e <= bm0) dn_form += 1000;
    }
    const bool ok = gu_form && dn_form && moe_xd_ok(gu_form, I, H, true) &&
                    moe_xd_ok(dn_form, H, I, false) &&
                    (gu_form % 1000) / 100 == (dn_form % 1000) / 100;  // one tile table
    if (!ok) {
      if (!auto_v) return -1;
      variant = rows_e >= 96 ? 2 : 1;  // shapes the grouped gemm_xd forms do not take
    }
  }
  const int bm = variant == 3 ? 128 * ((gu_form % 1000) / 100)
                              : (variant == 2 || variant == 4 ? 256 : 128);
  const int max_tiles = (P + bm - 1) / bm + e_local;
  // workspace carve (all 256-B aligned)
  auto align = [](int64_t v) { return (v + 255) & ~int64_t(255); };
  char* p = (char*)workspace;
  int64_t o = 0;
  int* sorted_tok = (int*)(p + o); o = align(o + 4ll * P);
  float* sorted_w = (float*)(p + o); o = align(o + 4ll * P);
  int* inv_pos = (int*)(p + o); o = align(o + 4ll * P);
  float* topk_w = (float*)(p + o); o = align(o + 4ll * P);
  int* t_e = (int*)(p + o); o = align(o + 4ll * max_tiles);
  int* t_r0 = (int*)(p + o); o = align(o + 4ll * max_tiles);
  int* t_n = (int*)(p + o); o = align(o + 4ll * max_tiles);
  int* n_tiles = (int*)(p + o); o = align(o + 4);
  int* local_range = (int*)(p + o); o = align(o + 8);
  bf16_t* hbuf = (bf16_t*)(p + o); o = align(o + 2ll * P * I);
  bf16_t* zbuf = (bf16_t*)(p + o); o = align(o + 2ll * P * H);
  int* grp_off = (int*)(p + o); o = align(o + 4ll * (e_local + 1));
  bf16_t* zbuf2 = (bf16_t*)(p + o); o = align(o + 2ll * P * H);  // (variant 4, split down)
  const int G = (T + kMoeRouteWG - 1) / kMoeRouteWG;
  int* wg_cnt = (int*)(p + o); o = align(o + 4ll * G * E);
  int* wg_base = (int*)(p + o); o = align(o + 4ll * G * E);
  if (o > ws_bytes) return -2;
  // variant 4: down split over K in two when its 256 x 256 tiles (rows spread evenly over the
  // experts) would not fill the CUs once - one tile row per expert at Mixtral decode sizes
  const int64_t dn_tiles = (int64_t)e_local * ((rows_e + 255) / 256) * (H / 256);
  const bool dn_split = variant == 4 && dn_form == 0 && dn_tiles < kMoeW4SplitTiles &&
                        (I / 64) % 2 == 0 && I / 128 >= 2;
  hipLaunchKernelGGL(moe_route_kernel, dim3(G), dim3(kMoeRouteWG), 0, st,
                     (const bf16_t*)router_logits, T, E, k, logit_ts, logit_es, inv_pos, topk_w,
                     wg_cnt);
  hipLaunchKernelGGL(moe_offsets_kernel, dim3(1), dim3(1024), 0, st, (const int*)wg_cnt, G, E,
                     wg_base, t_e, t_r0, t_n, n_tiles, local_range, max_tiles, e_off, e_local, bm,
                     variant == 4 ? grp_off : (int*)nullptr);
  hipLaunchKernelGGL(moe_scatter_kernel, dim3(G), dim3(kMoeRouteWG), 0, st, (const float*)topk_w,
                     (const int*)wg_base, T, E, k, sorted_tok, sorted_w, inv_pos);
  const dim3 g_gu((I / 64) * max_tiles), g_dn((H / 128) * max_tiles);
  if (variant == 4) {
    // xs (expert-ordered token rows) lives in zbuf: gate_up consumes it before down writes Z
    bf16_t* xs = zbuf;
    hipLaunchKernelGGL(moe_gather_kernel, dim3(min(P, 8192)), dim3(256), 0, st, xs,
                       (const bf16_t*)x, sorted_tok, local_range, P, H);
    int e = launch_gemm_w4_grouped(hbuf, xs, w_gu, grp_off, e_local, P, I, H, H, H, I,
                                   2ll * I * H, 2 + act, I, g_moe_gm_gu, 1, 0, st);
    if (e) return e;
    if (dn_form) {
      // down on gemm_xd's grouped split-K forms over the 256-row tile table (few rows per
      // expert: the persistent 256 x 256 down has H / 256 column tiles per expert only)
      int mt, nf, sk;
      moe_xd_form(dn_form, mt, nf, sk);
      e = launch_gemm_xd_grouped(zbuf, hbuf, w_dn, P, H, I, I, I, H, 0, mt, nf, sk, max_tiles,
                                 t_r0, t_n, t_e, n_tiles, nullptr, (int64_t)H * I, slab,
                                 slab_bytes, counters, n_counters, st);
    } else {
      e = launch_gemm_w4_grouped(zbuf, hbuf, w_dn, grp_off, e_local, P, H, I, I, I, H,
                                 (int64_t)H * I, 0, 0, g_moe_gm_dn, dn_split ? 2 : 1,
                                 dn_split ? (int64_t)(zbuf2 - zbuf) : 0, st);
    }
    if (e) return e;
  } else if (variant == 3) {
    int mt, nf, sk, e;
    moe_xd_form(gu_form, mt, nf, sk);
    e = launch_gemm_xd_grouped(hbuf, x, w_gu, T, I, H, H, H, I, 2 + act, mt, nf, sk, max_tiles,
                               t_r0, t_n, t_e, n_tiles, sorted_tok, 2ll * I * H, slab,
                               slab_bytes, counters, n_counters, st);
    if (e) return e;
    moe_xd_form(dn_form, mt, nf, sk);
    e = launch_gemm_xd_grouped(zbuf, hbuf, w_dn, P, H, I, I, I, H, 0, mt, nf, sk, max_tiles,
                               t_r0, t_n, t_e, n_tiles, nullptr, (int64_t)H * I, slab,
                               slab_bytes, counters, n_counters, st);
    if (e) return e;
  } else if (variant == 0) {
    hipLaunchKernelGGL(moe_gemm_kernel<0>, g_gu, dim3(256), 0, st, hbuf, (const bf16_t*)x,
                       (const bf16_t*)w_gu, sorted_tok, t_e, t_r0, t_n, n_tiles, H, 2 * I, I, I,
                       max_tiles, act);
    hipLaunchKernelGGL(moe_gemm_kernel<1>, g_dn, dim3(256), 0, st, zbuf, (const bf16_t*)hbuf,
                       (const bf16_t*)w_dn, sorted_tok, t_e, t_r0, t_n, n_tiles, I, H, I, H,
                       max_tiles, 0);
  } else if (variant == 1) {
    using Cf = PipeCfg<128>;
    hipLaunchKernelGGL((moe_gemm_pipe_kernel<128, 0>), g_gu, dim3(Cf::NT), Cf::LDS_BYTES, st, hbuf,
                       (const bf16_t*)x, (const bf16_t*)w_gu, sorted_tok, t_e, t_r0, t_n, n_tiles, H,
                       2 * I, I, I, max_tiles, act);
    hipLaunchKernelGGL((moe_gemm_pipe_kernel<128, 1>), g_dn, dim3(Cf::NT), Cf::LDS_BYTES, st, zbuf,
                       (const bf16_t*)hbuf, (const bf16_t*)w_dn, sorted_tok, t_e, t_r0, t_n,
                       n_tiles, I, H, I, H, max_tiles, 0);
  } else {
    using Cf = PipeCfg<256>;
    hipLaunchKernelGGL((moe_gemm_pipe_kernel<256, 0>), g_gu, dim3(Cf::NT), Cf::LDS_BYTES, st, hbuf,
                       (const bf16_t*)x, (const bf16_t*)w_gu, sorted_tok, t_e, t_r0, t_n, n_tiles, H,
                       2 * I, I, I, max_tiles, act);
    hipLaunchKernelGGL((moe_gemm_pipe_kernel<256, 1>), g_dn, dim3(Cf::NT), Cf::LDS_BYTES, st, zbuf,
                       (const bf16_t*)hbuf, (const bf16_t*)w_dn, sorted_tok, t_e, t_r0, t_n,
                       n_tiles, I, H, I, H, max_tiles, 0);
  }
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, st, (bf16_t*)out, zbuf,
                     dn_split ? (const bf16_t*)zbuf2 : nullptr, topk_w, inv_pos, local_range, T, H,
                     k);
  return (int)hipGetLastError();
}

int configure_moe() {
  int e = 0;
  e |= (int)hipFuncSetAttribute((const void*)moe_gemm_pipe_kernel<128, 0>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, PipeCfg<128>::LDS_BYTES);
  e |= (int)hipFuncSetAttribute((const void*)moe_gemm_pipe_kernel<128, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, PipeCfg<128>::LDS_BYTES);
  e |= (int)hipFuncSetAttribute((const void*)moe_gemm_pipe_kernel<256, 0>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, PipeCfg<256>::LDS_BYTES);
  e |= (int)hipFuncSetAttribute((const void*)moe_gemm_pipe_kernel<256, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, PipeCfg<256>::LDS_BYTES);
  return e;
}

int64_t moe_workspace_bytes(int T, int H, int I, int e_local, int k) {
  auto align = [](int64_t v) { return (v + 255) & ~int64_t(255); };
  const int64_t P = (int64_t)T * k;
  const int64_t mt = (P + kMoeBM - 1) / kMoeBM + e_local;
  // (tile tables sized for the 128-row tiles: the largest count of any variant)
  // (routing: per-workgroup counts and bases for up to 256 experts)
  const int64_t G = (T + kMoeRouteWG - 1) / kMoeRouteWG;
  return 4 * align(4 * P) + 3 * align(4 * mt) + align(4) + align(8) + align(2 * P * I) +
         2 * align(2 * P * H) + align(4 * (e_local + 1)) + 2 * align(4 * G * 256);
}

}  // namespace drtc
