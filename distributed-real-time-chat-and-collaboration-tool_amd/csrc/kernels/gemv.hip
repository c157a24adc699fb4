// Skinny projection GEMM for small-batch decode: y[M, N] = x[M, K] @ W[N, K]^T,
// M <= 16, bf16 in/out, fp32 accumulation.  Two forms: a VALU dot2 kernel
// (M <= 8, best at M <= 2) and an MFMA kernel (M <= 16), described below.
//
// Regime (cdna_hip_programming.md, "GEMV / M <= 16 decode weights"): every
// weight byte is used M <= 8 times, so the kernel is a pure HBM stream of W -
// operands go straight to VGPRs (no LDS round trip), 16-byte loads, several
// independent loads in flight per lane, products on the VALU with
// v_dot2_f32_bf16 (two bf16 products + fp32 accumulate per instruction).
//
// Decomposition: a 256-thread workgroup owns R consecutive output rows of W;
// its 4 waves split K into 512-element chunks round-robin (chunk c -> wave
// c % 4; a lane covers 8 contiguous k of a chunk), so even N = 1024-row shards
// launch N / R workgroups with 4 streaming waves each.  x (M x K, a few KB to
// a few hundred KB) is re-read by every workgroup from L2.  Partial sums are
// reduced across the 64 lanes with xor-shuffles and across the 4 waves
// through LDS.  K must be a multiple of 512 and N of R (checked by the
// launcher).
#include "common.h"
#include "launchers.h"

namespace drtc {

typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

DRTC_DEVICE float dot8(const bf16x8& a, const bf16x8& b, float acc) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bf16x2v pa = {a[2 * j], a[2 * j + 1]};
    bf16x2v pb = {b[2 * j], b[2 * j + 1]};
    acc = __builtin_amdgcn_fdot2_f32_bf16(pa, pb, acc, false);
  }
  return acc;
}

// x operand of the dot2 form: a plain row chunk, or (ACT >= 0) the gated
// activation act(gate) * up of a fused [gate | up] row computed on the fly
// (down projection: the act_glu launch disappears; up half at +K).
template <int ACT>
DRTC_DEVICE bf16x8 load_x8(const bf16_t* p, int K) {
  if constexpr (ACT < 0) {
    return load_bf16x8(p);
  } else {
    const bf16x8 g = load_bf16x8(p), u = load_bf16x8(p + K);
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(act_value<ACT>(bf2f(g[q])) * bf2f(u[q]));
    return o;
  }
}

template <int MT, int R, int ACT = -1>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(bf16_t* __restrict__ y,
                                                          const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ w, int M,
                                                          int K, int ldx, int ldy) {
  constexpr int CH = 512;  // k elements per chunk (64 lanes x 8)
  __shared__ float part[4][R * MT];
  const int n0 = blockIdx.x * R;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nch = K / CH;
  float acc[R][MT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;
  const bf16_t* wrow = w + (int64_t)n0 * K + lane * 8;
  const bf16_t* xrow = x + lane * 8;
  int c = wv;
  // two chunks per iteration: 2R weight loads (+ 2M x loads, L2 hits) in flight
  for (; c + 4 < nch; c += 8) {
    bf16x8 wa[R], wb[R], xa[MT], xb[MT];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      wa[r] = load_bf16x8(wrow + (int64_t)r * K + c * CH);
      wb[r] = load_bf16x8(wrow + (int64_t)r * K + (c + 4) * CH);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m < M) {
        xa[m] = load_x8<ACT>(xrow + (int64_t)m * ldx + c * CH, K);
        xb[m] = load_x8<ACT>(xrow + (int64_t)m * ldx + (c + 4) * CH, K);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        if (m < M) acc[r][m] = dot8(wb[r], xb[m], dot8(wa[r], xa[m], acc[r][m]));
  }
  if (c < nch) {  // odd chunk count: one left for this wave
    bf16x8 wa[R], xa[MT];
#pragma unroll
    for (int r = 0; r < R; ++r) wa[r] = load_bf16x8(wrow + (int64_t)r * K + c * CH);
#pragma unroll
    for (int m = 0; m < MT; ++m)
      if (m < M) xa[m] = load_x8<ACT>(xrow + (int64_t)m * ldx + c * CH, K);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        if (m < M) acc[r][m] = dot8(wa[r], xa[m], acc[r][m]);
  }
  // lanes -> lane 0 of each wave
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float v = acc[r][m];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      acc[r][m] = v;
    }
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int m = 0; m < MT; ++m) part[wv][r * MT + m] = acc[r][m];
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < R * MT) {
    const int r = t / MT, m = t - r * MT;
    if (m < M) {
      const float s = part[0][t] + part[1][t] + part[2][t] + part[3][t];
      y[(int64_t)m * ldy + n0 + r] = f2bf(s);
    }
  }
}

int launch_skinny_glu_gemm(void* y, const void* gu, const void* w, int M, int N, int K, int ldx,
                           int ldy, int act, hipStream_t st) {
  if (M < 1 || M > 2 || K % 512 != 0 || N % 4 != 0 || ldx % 8 != 0 || act < 0 || act > 1)
    return -1;
  const dim3 grid(N / 4), block(256);
  bf16_t* yy = (bf16_t*)y;
  const bf16_t* xx = (const bf16_t*)gu;
  const bf16_t* ww = (const bf16_t*)w;
  if (M == 1) {
    if (act == 0) skinny_gemm_kernel<1, 4, 0><<<grid, block, 0, st>>>(yy, xx, ww, M, K, ldx, ldy);
    else skinny_gemm_kernel<1, 4, 1><<<grid, block, 0, st>>>(yy, xx, ww, M, K, ldx, ldy);
  } else {
    if (act == 0) skinny_gemm_kernel<2, 4, 0><<<grid, block, 0, st>>>(yy, xx, ww, M, K, ldx, ldy);
    else skinny_gemm_kernel<2, 4, 1><<<grid, block, 0, st>>>(yy, xx, ww, M, K, ldx, ldy);
  }
  return (int)hipGetLastError();
}

// RMSNorm fused into the dot2 form (decode, M <= 4, K = hidden size with
// K % 2048 == 0): y = norm(x [+ res]) @ W^T, where h = bf16(x + res) is the
// new residual stream (written by workgroup 0 to h_out) and norm(h) =
// bf16(h * rsqrt(mean(h^2) + eps) * w) (Gemma: * (1 + w)) - the semantics of
// rmsnorm_kernel, so the separate norm launch disappears from the decode
// step.  Every workgroup needs the full-row sum of squares: its 256 threads
// hold exactly the x chunks the dot products use (CPW = K / 2048 chunks of 8
// per thread), so the prologue costs one extra load per chunk (res) and one
// barrier.  The W loads of all chunks are issued FIRST - they do not depend
// on x - so their HBM latency covers the norm prologue.  Measured (Llama-3-8B
// decode, profiles/r1l_skinny_gemm.md): a win at M = 1 only - at M = 2..4 the
// per-workgroup re-read of the M x K input costs what the saved launch gains
// (also with 8 W rows per workgroup), so ops.norm_linear fuses at M = 1.
template <int MT, int CPW, bool GEMMA, int R>
__global__ __launch_bounds__(256) void skinny_norm_gemm_kernel(
    bf16_t* __restrict__ y, bf16_t* __restrict__ h_out, const bf16_t* __restrict__ x,
    const bf16_t* __restrict__ res, const bf16_t* __restrict__ nw,
    const bf16_t* __restrict__ w, int M, int K, int ldx, int ldr, int ldh, int ldy, float eps) {
  constexpr int CH = 512;
  __shared__ float red[4][MT];
  __shared__ float part[4][R * MT];
  const int n0 = blockIdx.x * R;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  bf16x8 wa[CPW][R];
#pragma unroll
  for (int j = 0; j < CPW; ++j)
#pragma unroll
    for (int r = 0; r < R; ++r)
      wa[j][r] = load_bf16x8(w + (int64_t)(n0 + r) * K + (wv + 4 * j) * CH + lane * 8);
  bf16x8 hx[MT][CPW];
  float ss[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    ss[m] = 0.f;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int k = (wv + 4 * j) * CH + lane * 8;
      bf16x8 a = load_bf16x8(x + (int64_t)m * ldx + k);
      if (res != nullptr) {
        const bf16x8 rv = load_bf16x8(res + (int64_t)m * ldr + k);
#pragma unroll
        for (int q = 0; q < 8; ++q) a[q] = f2bf(bf2f(a[q]) + bf2f(rv[q]));
        if (blockIdx.x == 0) store_bf16x8(h_out + (int64_t)m * ldh + k, a);
      }
      hx[m][j] = a;
#pragma unroll
      for (int q = 0; q < 8; ++q) ss[m] += bf2f(a[q]) * bf2f(a[q]);
    }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const float v = wave_sum(ss[m]);
    if (lane == 0) red[wv][m] = v;
  }
  __syncthreads();
  float rstd[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
    rstd[m] = rsqrtf((red[0][m] + red[1][m] + red[2][m] + red[3][m]) / (float)K + eps);
  float acc[R][MT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;
#pragma unroll
  for (int j = 0; j < CPW; ++j) {
    const bf16x8 gv = load_bf16x8(nw + (wv + 4 * j) * CH + lane * 8);
    float ww[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) ww[q] = bf2f(gv[q]) + (GEMMA ? 1.f : 0.f);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m >= M) continue;
      bf16x8 xn;
#pragma unroll
      for (int q = 0; q < 8; ++q) xn[q] = f2bf(bf2f(hx[m][j][q]) * rstd[m] * ww[q]);
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r][m] = dot8(wa[j][r], xn, acc[r][m]);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float v = acc[r][m];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      acc[r][m] = v;
    }
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int m = 0; m < MT; ++m) part[wv][r * MT + m] = acc[r][m];
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < R * MT) {
    const int r = t / MT, m = t - r * MT;
    if (m < M) {
      const float s = part[0][t] + part[1][t] + part[2][t] + part[3][t];
      y[(int64_t)m * ldy + n0 + r] = f2bf(s);
    }
  }
}

template <int MT, bool GEMMA>
static int launch_norm_mt(bf16_t* y, bf16_t* h, const bf16_t* x, const bf16_t* res,
                          const bf16_t* nw, const bf16_t* w, int M, int N, int K, int ldx, int ldr,
                          int ldh, int ldy, float eps, hipStream_t st) {
  const dim3 grid(N / 4), block(256);
  switch (K / 2048) {
    case 1: skinny_norm_gemm_kernel<MT, 1, GEMMA, 4><<<grid, block, 0, st>>>(y, h, x, res, nw, w, M, K, ldx, ldr, ldh, ldy, eps); break;
    case 2: skinny_norm_gemm_kernel<MT, 2, GEMMA, 4><<<grid, block, 0, st>>>(y, h, x, res, nw, w, M, K, ldx, ldr, ldh, ldy, eps); break;
    case 4: skinny_norm_gemm_kernel<MT, 4, GEMMA, 4><<<grid, block, 0, st>>>(y, h, x, res, nw, w, M, K, ldx, ldr, ldh, ldy, eps); break;
    default: return -1;
  }
  return 0;
}

int launch_skinny_norm_gemm(void* y, void* h_out, const void* x, const void* res, const void* nw,
                            const void* w, int M, int N, int K, int ldx, int ldr, int ldh,
                            int ldy, float eps, bool gemma, hipStream_t st) {
  if (M < 1 || M > 4 || K % 2048 != 0 || N % 4 != 0 || ldx % 8 || (res && (ldr % 8 || ldh % 8)) ||
      (res && !h_out))
    return -1;
  bf16_t* yy = (bf16_t*)y;
  bf16_t* hh = (bf16_t*)h_out;
  const bf16_t* xx = (const bf16_t*)x;
  const bf16_t* rr = (const bf16_t*)res;
  const bf16_t* gg = (const bf16_t*)nw;
  const bf16_t* ww = (const bf16_t*)w;
  int rc;
  if (M == 1)
    rc = gemma ? launch_norm_mt<1, true>(yy, hh, xx, rr, gg, ww, M, N, K, ldx, ldr, ldh, ldy, eps, st)
               : launch_norm_mt<1, false>(yy, hh, xx, rr, gg, ww, M, N, K, ldx, ldr, ldh, ldy, eps, st);
  else if (M == 2)
    rc = gemma ? launch_norm_mt<2, true>(yy, hh, xx, rr, gg, ww, M, N, K, ldx, ldr, ldh, ldy, eps, st)
               : launch_norm_mt<2, false>(yy, hh, xx, rr, gg, ww, M, N, K, ldx, ldr, ldh, ldy, eps, st);
  else
    rc = gemma ? launch_norm_mt<4, true>(yy, hh, xx, rr, gg, ww, M, N, K, ldx, ldr, ldh, ldy, eps, st)
               : launch_norm_mt<4, false>(yy, hh, xx, rr, gg, ww, M, N, K, ldx, ldr, ldh, ldy, eps, st);
  return rc ? rc : (int)hipGetLastError();
}

// MFMA form for M <= 16: a wave multiplies T 16-row W tiles (A operand,
// straight from HBM to VGPRs) by the x^T fragment (B operand, M valid columns
// of 16, zero-padded), 16x16x32 bf16 MFMA, fp32 accumulators.  No cross-lane
// reduction at all; x is re-read once per 16*T W rows (M/(16T) of the W
// bytes), where the dot2 form re-reads it every 4 rows.  The NW waves of a
// workgroup form NW/KS row groups (16*T rows each) times KS K-splits; a
// K-split takes every KS-th 128-element step and the splits are combined
// through LDS.  k-permutation: in MFMA s (0..3) of a step, lane group
// g = l >> 4 takes k = 32 s + 8 g .. +8 - the same k for the A and B
// fragments, so the product is exact; this order makes the 4 lanes of a row
// read 64 contiguous bytes per load instruction.
template <int T, int NW, int KS>
__global__ __launch_bounds__(NW * 64) void skinny_mfma_kernel(bf16_t* __restrict__ y,
                                                             const bf16_t* __restrict__ x,
                                                             const bf16_t* __restrict__ w, int M,
                                                             int K, int ldx, int ldy) {
  constexpr int STEP = 128, RG = NW / KS;
  __shared__ f32x4 red[NW][T][64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ks = wv % KS, rg = wv / KS;
  const int n0 = (blockIdx.x * RG + rg) * (16 * T);
  const int r = lane & 15, g = lane >> 4;
  const bool xv = r < M;
  const int nst = K / STEP;
  const bf16_t* wp = w + (int64_t)(n0 + r) * K + 8 * g;
  const bf16_t* xp = x + (int64_t)(xv ? r : 0) * ldx + 8 * g;
  f32x4 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16x8 zero = {};
  int c = ks;
  for (; c + KS < nst; c += 2 * KS) {  // two steps in flight
    bf16x8 wa[2][T][4], xa[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k0 = (c + u * KS) * STEP;
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) wa[u][t][s] = load_bf16x8(wp + (int64_t)t * 16 * K + k0 + 32 * s);
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[u][s] = xv ? load_bf16x8(xp + k0 + 32 * s) : zero;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < T; ++t) acc[t] = mfma16(wa[u][t][s], xa[u][s], acc[t]);
  }
  if (c < nst) {
    bf16x8 wa[T][4], xa[4];
    const int k0 = c * STEP;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) wa[t][s] = load_bf16x8(wp + (int64_t)t * 16 * K + k0 + 32 * s);
#pragma unroll
    for (int s = 0; s < 4; ++s) xa[s] = xv ? load_bf16x8(xp + k0 + 32 * s) : zero;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < T; ++t) acc[t] = mfma16(wa[t][s], xa[s], acc[t]);
  }
  // C layout: lane l holds D[row 4*(l>>4) + v][col l&15] = y[m = l&15][n0 + 16t + 4(l>>4) + v]
  auto store = [&](f32x4 v, int row0, int l) {
    const bf16x4 o = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
    *reinterpret_cast<bf16x4*>(y + (int64_t)(l & 15) * ldy + row0 + 4 * (l >> 4)) = o;
  };
  if constexpr (KS == 1) {
    if (xv) {
#pragma unroll
      for (int t = 0; t < T; ++t) store(acc[t], n0 + 16 * t, lane);
    }
  } else {
#pragma unroll
    for (int t = 0; t < T; ++t) red[wv][t][lane] = acc[t];
    __syncthreads();
    for (int i = threadIdx.x; i < RG * T * 64; i += NW * 64) {
      const int l = i & 63, t = (i >> 6) % T, q = i / (64 * T);
      if ((l & 15) >= M) continue;
      f32x4 sum = red[q * KS][t][l];
#pragma unroll
      for (int j = 1; j < KS; ++j) sum += red[q * KS + j][t][l];
      store(sum, (blockIdx.x * RG + q) * (16 * T) + 16 * t, l);
    }
  }
}

template <int T, int NW, int KS>
static int launch_mfma(bf16_t* y, const bf16_t* x, const bf16_t* w, int M, int N, int K, int ldx,
                       int ldy, hipStream_t st) {
  constexpr int ROWS = 16 * T * (NW / KS);
  if (N % ROWS != 0) return -1;
  skinny_mfma_kernel<T, NW, KS><<<dim3(N / ROWS), dim3(NW * 64), 0, st>>>(y, x, w, M, K, ldx, ldy);
  return 0;
}

// variant: 0 = by shape, 1 = dot2 form, 2.. = MFMA form (T, NW, KS):
//   2 (1,4,4)  3 (1,8,8)  4 (2,4,4)  5 (2,8,8)  6 (1,16,16)  7 (1,8,2)  8 (1,8,1)  9 (1,16,4)
int launch_skinny_gemm(void* y, const void* x, const void* w, int M, int N, int K, int ldx,
                       int ldy, int variant, hipStream_t st) {
  constexpr int R = 4;
  bf16_t* yy = (bf16_t*)y;
  const bf16_t* xx = (const bf16_t*)x;
  const bf16_t* ww = (const bf16_t*)w;
  if (M < 1 || M > 16 || ldx % 8 != 0 || ldy % 4 != 0) return -1;
  if (variant == 0) variant = (M <= 2 && K % 512 == 0) ? 1 : 3;
  if (variant >= 2) {
    if (K % 128 != 0) return -1;
    int rc = -1;
    switch (variant) {
      case 2: rc = launch_mfma<1, 4, 4>(yy, xx, ww, M, N, K, ldx, ldy, st); break;
      case 3: rc = launch_mfma<1, 8, 8>(yy, xx, ww, M, N, K, ldx, ldy, st); break;
      case 4: rc = launch_mfma<2, 4, 4>(yy, xx, ww, M, N, K, ldx, ldy, st); break;
      case 5: rc = launch_mfma<2, 8, 8>(yy, xx, ww, M, N, K, ldx, ldy, st); break;
      case 6: rc = launch_mfma<1, 16, 16>(yy, xx, ww, M, N, K, ldx, ldy, st); break;
      case 7: rc = launch_mfma<1, 8, 2>(yy, xx, ww, M, N, K, ldx, ldy, st); break;
      case 8: rc = launch_mfma<1, 8, 1>(yy, xx, ww, M, N, K, ldx, ldy, st); break;
      case 9: rc = launch_mfma<1, 16, 4>(yy, xx, ww, M, N, K, ldx, ldy, st); break;
      default: return -1;
    }
    return rc ? rc : (int)hipGetLastError();
  }
  if (M > 8 || K % 512 != 0 || N % R != 0) return -1;
  const dim3 grid(N / R), block(256);
  if (M == 1)
    skinny_gemm_kernel<1, R><<<grid, block, 0, st>>>(yy, xx, ww, M, K, ldx, ldy);
  else if (M == 2)
    skinny_gemm_kernel<2, R><<<grid, block, 0, st>>>(yy, xx, ww, M, K, ldx, ldy);
  else if (M <= 4)
    skinny_gemm_kernel<4, R><<<grid, block, 0, st>>>(yy, xx, ww, M, K, ldx, ldy);
  else
    skinny_gemm_kernel<8, R><<<grid, block, 0, st>>>(yy, xx, ww, M, K, ldx, ldy);
  return (int)hipGetLastError();
}

}  // namespace drtc
