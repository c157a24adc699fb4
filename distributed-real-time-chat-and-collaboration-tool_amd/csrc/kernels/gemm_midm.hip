// Medium-M projection GEMM for decode batches 17..256: y[M, N] = x[M, K] @ W[N, K]^T,
// bf16 in/out, fp32 accumulation, 16x16x32 bf16 MFMA.
//
// Regime: at these M the weights are read once per call and every weight byte is used
// M times - far below the MFMA's arithmetic intensity - so the kernel is a weight
// stream, and the library's 128-256-row output tiles leave most CUs idle on the
// N = 4096-6144 projections (hipBLASLt at M = 128: o / qkv / down stream W at 2.3-2.4
// TB/s, scripts/midm_probe.py).  Here:
//   * a 256-thread workgroup owns 128 rows of W (4 waves x 2 MFMA row tiles) and one
//     K-split of them; W goes straight from HBM to VGPRs through a D-chunk register
//     ring (64-k chunks, compile-time ring slots), one pass, 16-byte loads;
//   * the x chunk [0:M_pad, 64 k] is staged once per workgroup in LDS (double buffer,
//     rows padded to 72 elements) and shared by the 4 waves; a wave multiplies each of
//     its W fragments by MG x fragments (MG = ceil(M/16) column groups);
//   * K is split over S workgroups so the grid fills every CU; splits write fp32
//     partial tiles to a slab and `midm_reduce_kernel` sums them in fixed order and
//     applies the epilogue (store, residual add, SiLU/GELU-gated [gate | up]).  With
//     S = 1 and a plain / residual epilogue the GEMM kernel writes bf16 directly.
//     No atomics or fences: the kernel boundary orders slab writes and reads, so the
//     pair replays inside a hipGraph.
// Operand mapping (as gemv.hip's MFMA form): A = W rows (lane row l & 15, k = 8 (l >> 4)
// .. +8 of the 32-k substep), B = x^T (lane column m = l & 15 of the column group,
// same k), so lane l holds D[n = 4 (l >> 4) + r][m = l & 15], r = 0..3: 4
// consecutive output columns n of one row m (16-byte stores).
#include "common.h"
#include "launchers.h"

namespace drtc {
namespace {

constexpr int kMidThreads = 256;
constexpr int kMidRows = 128;   // W rows per workgroup (4 waves x 2 tiles x 16)
constexpr int kMidKC = 64;      // k per chunk
constexpr int kMidXRow = 72;    // LDS x row stride (elements): 144 B breaks bank aliasing
// W register ring depth (chunks in flight per wave): 4, or 2 where the accumulators of
// 14-16 column groups leave no room for 4 (no scratch)
template <int MG>
constexpr int mid_depth() { return 4; }  // 8 measured slower (VGPRs, fewer valid splits)

enum { MID_STORE = 0, MID_RESIDUAL = 1, MID_SLAB = 2 };

// Occupancy: 2 workgroups per CU up to 8 column groups (M <= 128); beyond that (the
// 129-256-row buckets of the 70B decode) the 2 x MG accumulators need the AGPR half of the
// register file and the x double buffer is up to 74 KiB of LDS, so one workgroup per CU.
template <int MG>
constexpr int mid_wgs_per_cu() { return MG > 8 ? 1 : 2; }

template <int MG, int OUT>
__global__ __launch_bounds__(kMidThreads, mid_wgs_per_cu<MG>()) void midm_kernel(
    bf16_t* __restrict__ y, float* __restrict__ slab, const bf16_t* __restrict__ x,
    const bf16_t* __restrict__ w, const bf16_t* __restrict__ res, int M, int N, int K,
    int ldx, int ldy, int ldr, int n_blocks, int kps) {
  constexpr int MP = MG * 16;
  constexpr int kMidD = mid_depth<MG>();
  __shared__ __attribute__((aligned(16))) bf16_t xs[2][MP * kMidXRow];
  const int nb = blockIdx.x % n_blocks;
  const int s = blockIdx.x / n_blocks;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = nb * kMidRows + wv * 32;
  const int k_begin = s * kps;
  const int nc = kps / kMidKC;

  // ---- W register ring: [slot][tile][substep] 16-B fragments
  bf16x8 wr[kMidD][2][2];
  const bf16_t* wp0 = w + (int64_t)(n0 + r) * K + k_begin + 8 * g;
  const bf16_t* wp1 = wp0 + (int64_t)16 * K;
  auto load_w = [&](bf16x8 (&dst)[2][2], int c) {
    const int k = c * kMidKC;
    dst[0][0] = load_bf16x8(wp0 + k);
    dst[0][1] = load_bf16x8(wp0 + k + 32);
    dst[1][0] = load_bf16x8(wp1 + k);
    dst[1][1] = load_bf16x8(wp1 + k + 32);
  };
  // ---- x staging: MP rows x 64 k = MP * 8 16-B vectors, MG / 2 per thread
  constexpr int XV = MP * 8 / kMidThreads;  // = MG / 2
  static_assert(MG % 2 == 0 && XV >= 1, "MG must be even");
  // x register ring of 2 chunks: chunk j is loaded at iteration j - 2 into slot j & 1 and
  // written to LDS buffer j & 1 at iteration j - 1, so a whole iteration hides its latency
  bf16x8 xr[2][XV];
  auto load_x = [&](bf16x8 (&dst)[XV], int c) {
    const int k = k_begin + c * kMidKC;
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int v = tid + i * kMidThreads;
      const int m = v >> 3, kk = (v & 7) * 8;
      if (m < M) {
        dst[i] = load_bf16x8(x + (int64_t)m * ldx + k + kk);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) dst[i][j] = f2bf(0.f);
      }
    }
  };
  auto store_x = [&](const bf16x8 (&src)[XV], int buf) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int v = tid + i * kMidThreads;
      const int m = v >> 3, kk = (v & 7) * 8;
      store_bf16x8(&xs[buf][m * kMidXRow + kk], src[i]);
    }
  };

  f32x4 acc[2][MG];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < MG; ++q) acc[t][q] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // The loop body is branch-free (nc is a multiple of kMidD, enforced by the launcher;
  // prefetches past the last chunk re-load the last chunk instead of being skipped), so
  // hipcc can count the loads still in flight: each chunk waits for its own W fragments
  // only (counted vmcnt), not for the ring's younger loads (a conditional load made it
  // emit vmcnt(0) before every chunk - one full HBM latency per 64-k chunk).
  load_x(xr[0], 0);
#pragma unroll
  for (int d = 0; d < kMidD; ++d) load_w(wr[d], d);
  load_x(xr[1], min(1, nc - 1));
  store_x(xr[0], 0);
  __syncthreads();

  static_assert(kMidD % 2 == 0, "ring phases must keep the x slot compile-time");
  for (int c0 = 0; c0 < nc; c0 += kMidD) {
#pragma unroll
    for (int ph = 0; ph < kMidD; ++ph) {
      const int c = c0 + ph;
      {
        const int buf = ph & 1;  // == c & 1 (c0 is a multiple of kMidD, which is even)
        load_x(xr[buf], min(c + 2, nc - 1));  // slot of chunk c: stored last iteration
        const bf16_t* xb = &xs[buf][0];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
          for (int q = 0; q < MG; ++q) {
            const bf16x8 xf = load_bf16x8(xb + (q * 16 + r) * kMidXRow + sub * 32 + 8 * g);
            acc[0][q] = mfma16(wr[ph][0][sub], xf, acc[0][q]);
            acc[1][q] = mfma16(wr[ph][1][sub], xf, acc[1][q]);
          }
        }
        load_w(wr[ph], min(c + kMidD, nc - 1));
        store_x(xr[buf ^ 1], buf ^ 1);  // chunk c + 1, loaded an iteration ago
        __syncthreads();
      }
    }
  }

  // ---- epilogue: lane holds rows n = n0 + 16 t + 4 g + 0..3 of column m = 16 q + r
#pragma unroll
  for (int q = 0; q < MG; ++q) {
    const int m = q * 16 + r;
    if (m >= M) continue;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      if constexpr (OUT == MID_SLAB) {
        *reinterpret_cast<f32x4*>(slab + ((int64_t)s * M + m) * N + n) = acc[t][q];
      } else {
        f32x4 v = acc[t][q];
        if constexpr (OUT == MID_RESIDUAL) {
          const bf16x4 rv = *reinterpret_cast<const bf16x4*>(res + (int64_t)m * ldr + n);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] += bf2f(rv[j]);
        }
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j]);
        *reinterpret_cast<bf16x4*>(y + (int64_t)m * ldy + n) = o;
      }
    }
  }
}

// Sum the S fp32 partial slabs (fixed order) and apply the epilogue.
//   EPI 0: y = sum;  1: y = bf16(sum + res);  2 / 3: y[:, j] = act(sum[:, j]) *
//   sum[:, j + N/2] with SiLU / GELU-tanh (N = 2 I, the fused [gate | up] rows).
template <int EPI>
__global__ __launch_bounds__(256) void midm_reduce_kernel(bf16_t* __restrict__ y,
                                                          const float* __restrict__ slab,
                                                          const bf16_t* __restrict__ res, int M,
                                                          int N, int S, int ldy, int ldr) {
  const int NO = (EPI >= 2) ? N / 2 : N;  // output columns
  const int per_row = NO / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)M * per_row) return;
  const int m = (int)(i / per_row);
  const int n = (int)(i - (int64_t)m * per_row) * 4;
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    const float* row = slab + ((int64_t)s * M + m) * N;
    a += *reinterpret_cast<const f32x4*>(row + n);
    if constexpr (EPI >= 2) b += *reinterpret_cast<const f32x4*>(row + n + NO);
  }
  bf16x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float v = a[j];
    if constexpr (EPI == 1) v += bf2f(res[(int64_t)m * ldr + n + j]);
    if constexpr (EPI == 2) v = act_value<0>(bf2f(f2bf(a[j]))) * bf2f(f2bf(b[j]));
    if constexpr (EPI == 3) v = act_value<1>(bf2f(f2bf(a[j]))) * bf2f(f2bf(b[j]));
    o[j] = f2bf(v);
  }
  *reinterpret_cast<bf16x4*>(y + (int64_t)m * ldy + n) = o;
}

template <int MG>
int launch_mg(bf16_t* y, float* slab, const bf16_t* x, const bf16_t* w, const bf16_t* res, int M,
              int N, int K, int ldx, int ldy, int ldr, int S, int out, hipStream_t st) {
  const int n_blocks = N / kMidRows;
  const dim3 grid(n_blocks * S), block(kMidThreads);
  const int kps = K / S;
  switch (out) {
    case MID_STORE:
      midm_kernel<MG, MID_STORE><<<grid, block, 0, st>>>(y, slab, x, w, res, M, N, K, ldx, ldy, ldr, n_blocks, kps);
      break;
    case MID_RESIDUAL:
      midm_kernel<MG, MID_RESIDUAL><<<grid, block, 0, st>>>(y, slab, x, w, res, M, N, K, ldx, ldy, ldr, n_blocks, kps);
      break;
    default:
      midm_kernel<MG, MID_SLAB><<<grid, block, 0, st>>>(y, slab, x, w, res, M, N, K, ldx, ldy, ldr, n_blocks, kps);
      break;
  }
  return 0;
}

}  // namespace

int64_t midm_slab_bytes(int M, int N, int S) { return (int64_t)S * M * N * 4; }

// epi: 0 store, 1 residual add (res may alias y), 2 SiLU-GLU, 3 GELU-GLU (N = 2 I,
// y has N / 2 columns).  S = number of K splits (K % (64 S) == 0); S > 1 or a GLU
// epilogue needs `slab` (midm_slab_bytes) and runs the reduce kernel.
int launch_midm_gemm(void* y, const void* x, const void* w, const void* res, int M, int N,
                     int K, int ldx, int ldy, int ldr, int epi, int S, void* slab,
                     int64_t slab_bytes, hipStream_t st) {
  // K per split: whole register rings (4 chunks of 64)
  if (M < 1 || M > 256 || N % kMidRows || S < 1 || K % (4 * kMidKC * S) || ldx % 8 ||
      ldy % 4 ||
      epi < 0 || epi > 3 || (epi == 1 && (res == nullptr || ldr % 4)) ||
      (epi >= 2 && (N / 2) % 4))
    return -1;
  const bool use_slab = S > 1 || epi >= 2;
  if (use_slab && (slab == nullptr || slab_bytes < midm_slab_bytes(M, N, S))) return -2;
  const int out = use_slab ? MID_SLAB : (epi == 1 ? MID_RESIDUAL : MID_STORE);
  int mg = (M + 15) / 16;
  mg += mg & 1;  // even column-group counts only
  bf16_t* yy = (bf16_t*)y;
  float* sl = (float*)slab;
  const bf16_t* xx = (const bf16_t*)x;
  const bf16_t* ww = (const bf16_t*)w;
  const bf16_t* rr = (const bf16_t*)res;
  switch (mg) {
    case 2: launch_mg<2>(yy, sl, xx, ww, rr, M, N, K, ldx, ldy, ldr, S, out, st); break;
    case 4: launch_mg<4>(yy, sl, xx, ww, rr, M, N, K, ldx, ldy, ldr, S, out, st); break;
    case 6: launch_mg<6>(yy, sl, xx, ww, rr, M, N, K, ldx, ldy, ldr, S, out, st); break;
    case 8: launch_mg<8>(yy, sl, xx, ww, rr, M, N, K, ldx, ldy, ldr, S, out, st); break;
    case 10: launch_mg<10>(yy, sl, xx, ww, rr, M, N, K, ldx, ldy, ldr, S, out, st); break;
    case 12: launch_mg<12>(yy, sl, xx, ww, rr, M, N, K, ldx, ldy, ldr, S, out, st); break;
    case 14: launch_mg<14>(yy, sl, xx, ww, rr, M, N, K, ldx, ldy, ldr, S, out, st); break;
    case 16: launch_mg<16>(yy, sl, xx, ww, rr, M, N, K, ldx, ldy, ldr, S, out, st); break;
    default: return -1;
  }
  if (use_slab) {
    const int NO = epi >= 2 ? N / 2 : N;
    const int64_t items = (int64_t)M * (NO / 4);
    const dim3 rgrid((unsigned)((items + 255) / 256)), rblock(256);
    switch (epi) {
      case 0: midm_reduce_kernel<0><<<rgrid, rblock, 0, st>>>(yy, sl, rr, M, N, S, ldy, ldr); break;
      case 1: midm_reduce_kernel<1><<<rgrid, rblock, 0, st>>>(yy, sl, rr, M, N, S, ldy, ldr); break;
      case 2: midm_reduce_kernel<2><<<rgrid, rblock, 0, st>>>(yy, sl, rr, M, N, S, ldy, ldr); break;
      default: midm_reduce_kernel<3><<<rgrid, rblock, 0, st>>>(yy, sl, rr, M, N, S, ldy, ldr); break;
    }
  }
  return (int)hipGetLastError();
}

}  // namespace drtc
