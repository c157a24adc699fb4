// Memory-bound fused elementwise kernels for the decoder layer (gfx950).
//
//  * RMSNorm, optionally fused with the residual add that precedes it
//    (residual += x; out = norm(residual) * w), Llama (w) and Gemma (1 + w)
//    weight conventions.  One 256-thread workgroup per row, 16-byte bf16
//    vectors held in registers between the sum-of-squares and the scale pass,
//    so every row is read from HBM exactly once.
//  * Gated activations act(gate) * up (SiLU for Llama/Mixtral, tanh-GELU for
//    Gemma) over the fused [gate | up] GEMM output.
//  * RoPE applied in place on the fused QKV GEMM output, fused with the
//    paged KV-cache write (K token-major [blk][h][tok][d], V dim-major
//    [blk][h][d][tok], the layout the paged decode kernel reads with MFMA).
//    cos/sin come from a host-precomputed fp32 table (no device trig).
#include "common.h"
#include "launchers.h"

namespace drtc {

// ----------------------------------------------------------------- RMSNorm
template <int VPT, bool GEMMA, bool RESID>
__global__ __launch_bounds__(256) void rmsnorm_kernel(
    bf16_t* __restrict__ out, bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, int H,
    float eps, int x_stride, int out_stride, int res_stride) {
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  const bf16_t* xr = x + (int64_t)row * x_stride;
  float v[VPT][8];
  float ss = 0.f;
  // the weight row is loaded with the activations, not after the reduction: a decode-sized
  // norm (one short workgroup per row) then pays one memory latency, not two
  bf16x8 wv[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = (tid + i * 256) * 8;
    if (idx < H) wv[i] = load_bf16x8(w + idx);
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = (tid + i * 256) * 8;
    if (idx < H) {
      bf16x8 a = load_bf16x8(xr + idx);
      if constexpr (RESID) {
        bf16_t* rr = residual + (int64_t)row * res_stride + idx;
        bf16x8 r = load_bf16x8(rr);
        bf16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] = f2bf(bf2f(a[j]) + bf2f(r[j]));
        store_bf16x8(rr, s);
        a = s;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = bf2f(a[j]);
        ss += v[i][j] * v[i][j];
      }
    }
  }
  __shared__ float red[4];
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float rstd = rsqrtf(tot / (float)H + eps);
  bf16_t* orow = out + (int64_t)row * out_stride;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = (tid + i * 256) * 8;
    if (idx < H) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float ww = bf2f(wv[i][j]);
        if constexpr (GEMMA) ww += 1.f;
        o[j] = f2bf(v[i][j] * rstd * ww);
      }
      store_bf16x8(orow + idx, o);
    }
  }
}

template <bool GEMMA, bool RESID>
static void launch_rmsnorm_t(bf16_t* out, bf16_t* residual, const bf16_t* x,
                             const bf16_t* w, int rows, int H, float eps,
                             int x_stride, int out_stride, int res_stride,
                             hipStream_t st) {
  const int vpt = (H / 8 + 255) / 256;
  dim3 grid(rows), block(256);
#define DRTC_RMS_CASE(N)                                                      \
  case N:                                                                    \
    hipLaunchKernelGGL((rmsnorm_kernel<N, GEMMA, RESID>), grid, block, 0, st, \
                       out, residual, x, w, H, eps, x_stride, out_stride,     \
                       res_stride);                                           \
    break;
  switch (vpt) {
    DRTC_RMS_CASE(1)
    DRTC_RMS_CASE(2)
    DRTC_RMS_CASE(3)
    DRTC_RMS_CASE(4)
    DRTC_RMS_CASE(8)
    default:
      break;
  }
#undef DRTC_RMS_CASE
}

int launch_rmsnorm(void* out, void* residual, const void* x, const void* w,
                   int rows, int H, float eps, int x_stride, int out_stride,
                   int res_stride, bool gemma, hipStream_t st) {
  const int vpt = (H / 8 + 255) / 256;
  if (H % 8 != 0 || vpt < 1 || (vpt > 4 && vpt != 8)) return -1;
  if (rows == 0) return 0;
  auto o = (bf16_t*)out;
  auto r = (bf16_t*)residual;
  auto xx = (const bf16_t*)x;
  auto ww = (const bf16_t*)w;
  if (residual) {
    if (gemma) launch_rmsnorm_t<true, true>(o, r, xx, ww, rows, H, eps, x_stride, out_stride, res_stride, st);
    else launch_rmsnorm_t<false, true>(o, r, xx, ww, rows, H, eps, x_stride, out_stride, res_stride, st);
  } else {
    if (gemma) launch_rmsnorm_t<true, false>(o, r, xx, ww, rows, H, eps, x_stride, out_stride, res_stride, st);
    else launch_rmsnorm_t<false, false>(o, r, xx, ww, rows, H, eps, x_stride, out_stride, res_stride, st);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------- gated activations
template <int ACT>  // 0 = SiLU, 1 = tanh-GELU
__global__ __launch_bounds__(256) void act_glu_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ gu, int64_t T, int I,
    int gu_stride) {
  const int vpr = I / 8;
  const int64_t total = T * vpr;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total;
       v += (int64_t)gridDim.x * 256) {
    const int64_t t = v / vpr;
    const int c = (int)(v - t * vpr) * 8;
    const bf16_t* row = gu + t * gu_stride;
    bf16x8 g = load_bf16x8(row + c);
    bf16x8 u = load_bf16x8(row + I + c);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = f2bf(act_value<ACT>(bf2f(g[j])) * bf2f(u[j]));
    }
    store_bf16x8(out + t * I + c, o);
  }
}

int launch_act_glu(void* out, const void* gu, int64_t T, int I, int gu_stride,
                   int act, hipStream_t st) {
  if (I % 8 != 0) return -1;
  const int64_t total = T * (I / 8);
  if (total == 0) return 0;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (act == 0)
    hipLaunchKernelGGL(act_glu_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, st,
                       (bf16_t*)out, (const bf16_t*)gu, T, I, gu_stride);
  else
    hipLaunchKernelGGL(act_glu_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, st,
                       (bf16_t*)out, (const bf16_t*)gu, T, I, gu_stride);
  return (int)hipGetLastError();
}

// ------------------------------------------------------ RoPE + KV write
// qkv: [T][qkv_stride] with heads laid out q(Hq) | k(Hkv) | v(Hkv), each D.
// cos_sin: [max_pos][D] fp32, first D/2 = cos, last D/2 = sin (NeoX halves).
template <int D>
__global__ __launch_bounds__(256) void rope_kv_kernel(
    bf16_t* __restrict__ qkv, int qkv_stride, const int* __restrict__ positions,
    const int64_t* __restrict__ slots, const float* __restrict__ cos_sin,
    int Hq, int Hkv, bf16_t* __restrict__ k_cache,
    bf16_t* __restrict__ v_cache, int block_size, int write_v) {
  constexpr int HV = D / 16;  // 8-wide vectors per half-head
  const int t = blockIdx.x;
  const int pos = positions[t];
  const int64_t slot = slots ? slots[t] : -1;
  bf16_t* row = qkv + (int64_t)t * qkv_stride;
  const float* cs = cos_sin + (int64_t)pos * D;
  int64_t blk = 0, off = 0;
  if (slot >= 0) {
    blk = slot / block_size;
    off = slot - blk * block_size;
  }
  const int n_rope = (Hq + Hkv) * HV;
  for (int item = threadIdx.x; item < n_rope; item += 256) {
    const int head = item / HV;
    const int vi = item - head * HV;
    bf16_t* base = row + head * D + vi * 8;
    bf16x8 x1 = load_bf16x8(base);
    bf16x8 x2 = load_bf16x8(base + D / 2);
    bf16x8 o1, o2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = cs[vi * 8 + j];
      const float s = cs[D / 2 + vi * 8 + j];
      const float a = bf2f(x1[j]), b = bf2f(x2[j]);
      o1[j] = f2bf(a * c - b * s);
      o2[j] = f2bf(b * c + a * s);
    }
    store_bf16x8(base, o1);
    store_bf16x8(base + D / 2, o2);
    if (head >= Hq && slot >= 0) {
      const int h = head - Hq;
      bf16_t* kd = k_cache + ((blk * Hkv + h) * block_size + off) * D + vi * 8;
      store_bf16x8(kd, o1);
      store_bf16x8(kd + D / 2, o2);
    }
  }
  if (slot < 0 || !write_v) return;
  const int n_v = Hkv * (D / 8);
  for (int item = threadIdx.x; item < n_v; item += 256) {
    const int h = item / (D / 8);
    const int c = (item - h * (D / 8)) * 8;
    bf16x8 v = load_bf16x8(row + (Hq + Hkv + h) * D + c);
    // V block layout: [block_size/4 groups][D][4 tokens] (see kv_write_v)
    bf16_t* vd = v_cache + (blk * Hkv + h) * D * block_size + (off >> 2) * (4 * D) + c * 4 +
                 (off & 3);
#pragma unroll
    for (int j = 0; j < 8; ++j) vd[4 * j] = v[j];
  }
}

// v2: a single pass over rope items + V items (block = their count rounded
// up to whole waves, looping only past 1024), cos/sin read as 16-B vectors,
// and the V scatter mapped one cache dim per lane: a wave's stores then hit
// 64 consecutive 8-B slots of the dim-major V group (4 cache lines) instead of
// 8 dims per lane (every store instruction spread over 32 lines).  Same math
// and cache contents as rope_kv_kernel.
template <int D>
__global__ __launch_bounds__(1024) void rope_kv_kernel_v2(
    bf16_t* __restrict__ qkv, int qkv_stride, const int* __restrict__ positions,
    const int64_t* __restrict__ slots, const float* __restrict__ cos_sin,
    int Hq, int Hkv, bf16_t* __restrict__ k_cache,
    bf16_t* __restrict__ v_cache, int block_size, int write_v) {
  constexpr int HV = D / 16;
  const int t = blockIdx.x;
  const int n_rope = (Hq + Hkv) * HV;
  const int pos = positions[t];
  const int64_t slot = slots ? slots[t] : -1;
  const int n_items = n_rope + ((slot >= 0 && write_v) ? Hkv * (D / 2) : 0);
  bf16_t* row = qkv + (int64_t)t * qkv_stride;
  int64_t blk = 0, off = 0;
  if (slot >= 0) {
    blk = slot / block_size;
    off = slot - blk * block_size;
  }
  for (int item = threadIdx.x; item < n_items; item += blockDim.x) {
    if (item < n_rope) {
      const int head = item / HV;
      const int vi = item - head * HV;
      const float* cs = cos_sin + (int64_t)pos * D + vi * 8;
      const f32x4 ca = *reinterpret_cast<const f32x4*>(cs);
      const f32x4 cb = *reinterpret_cast<const f32x4*>(cs + 4);
      const f32x4 sa = *reinterpret_cast<const f32x4*>(cs + D / 2);
      const f32x4 sb = *reinterpret_cast<const f32x4*>(cs + D / 2 + 4);
      bf16_t* base = row + head * D + vi * 8;
      const bf16x8 x1 = load_bf16x8(base);
      const bf16x8 x2 = load_bf16x8(base + D / 2);
      bf16x8 o1, o2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = j < 4 ? ca[j] : cb[j - 4];
        const float sn = j < 4 ? sa[j] : sb[j - 4];
        const float a = bf2f(x1[j]), b = bf2f(x2[j]);
        o1[j] = f2bf(a * c - b * sn);
        o2[j] = f2bf(b * c + a * sn);
      }
      store_bf16x8(base, o1);
      store_bf16x8(base + D / 2, o2);
      if (head >= Hq && slot >= 0) {
        bf16_t* kd = k_cache + ((blk * Hkv + (head - Hq)) * block_size + off) * D + vi * 8;
        store_bf16x8(kd, o1);
        store_bf16x8(kd + D / 2, o2);
      }
    } else {
      // V block layout: [block_size/4 groups][D][4 tokens] (see kv_write_v)
      const int vitem = item - n_rope;
      const int h = vitem / (D / 2);
      const int d = vitem - h * (D / 2);
      const bf16_t* src = row + (Hq + Hkv + h) * D + d;
      bf16_t* vd = v_cache + (blk * Hkv + h) * D * block_size + (off >> 2) * (4 * D) + d * 4 +
                   (off & 3);
      const bf16_t v0 = src[0], v1 = src[D / 2];
      vd[0] = v0;
      vd[2 * D] = v1;  // dim d + D/2: 4 * (D/2) elements further
    }
  }
}

static int g_rope_variant = 2;
void set_rope_variant(int v) { g_rope_variant = v; }

int launch_rope_kv(void* qkv, int T, int qkv_stride, const int* positions,
                   const int64_t* slots, const float* cos_sin, int Hq, int Hkv,
                   int D, void* k_cache, void* v_cache, int block_size, int write_v,
                   hipStream_t st) {
  if (T == 0) return 0;
  const int items = (Hq + Hkv) * (D / 16) + (slots && write_v ? Hkv * (D / 2) : 0);
  if (g_rope_variant == 2) {
    dim3 grid(T), block(std::min(1024, (items + 63) / 64 * 64));
    switch (D) {
      case 64:
        hipLaunchKernelGGL(rope_kv_kernel_v2<64>, grid, block, 0, st, (bf16_t*)qkv, qkv_stride, positions, slots, cos_sin, Hq, Hkv, (bf16_t*)k_cache, (bf16_t*)v_cache, block_size, write_v);
        break;
      case 128:
        hipLaunchKernelGGL(rope_kv_kernel_v2<128>, grid, block, 0, st, (bf16_t*)qkv, qkv_stride, positions, slots, cos_sin, Hq, Hkv, (bf16_t*)k_cache, (bf16_t*)v_cache, block_size, write_v);
        break;
      case 256:
        hipLaunchKernelGGL(rope_kv_kernel_v2<256>, grid, block, 0, st, (bf16_t*)qkv, qkv_stride, positions, slots, cos_sin, Hq, Hkv, (bf16_t*)k_cache, (bf16_t*)v_cache, block_size, write_v);
        break;
      default:
        return -1;
    }
    return (int)hipGetLastError();
  }
  dim3 grid(T), block(256);
  switch (D) {
    case 64:
      hipLaunchKernelGGL(rope_kv_kernel<64>, grid, block, 0, st, (bf16_t*)qkv, qkv_stride, positions, slots, cos_sin, Hq, Hkv, (bf16_t*)k_cache, (bf16_t*)v_cache, block_size, write_v);
      break;
    case 128:
      hipLaunchKernelGGL(rope_kv_kernel<128>, grid, block, 0, st, (bf16_t*)qkv, qkv_stride, positions, slots, cos_sin, Hq, Hkv, (bf16_t*)k_cache, (bf16_t*)v_cache, block_size, write_v);
      break;
    case 256:
      hipLaunchKernelGGL(rope_kv_kernel<256>, grid, block, 0, st, (bf16_t*)qkv, qkv_stride, positions, slots, cos_sin, Hq, Hkv, (bf16_t*)k_cache, (bf16_t*)v_cache, block_size, write_v);
      break;
    default:
      return -1;
  }
  return (int)hipGetLastError();
}

// ------------------------------------------- prefill V write (transposed)
// V cache block layout (per kv head): 8 groups of 4 tokens, each group
// dim-major [D][4] - the decode kernel's P.V operand wants 4 consecutive
// tokens of one dim in 8 contiguous bytes, and a decode-time write of ONE
// token then touches D 8-byte slots inside a 2*D-byte span (a plain [D][32]
// dim-major block scatters it over D separate 64-B rows: ~8x the HBM write
// traffic).  In prefill a whole block's tokens are contiguous rows of the
// QKV buffer, so one workgroup per (block segment, kv head) stages the
// [32][D] tile in LDS and writes the block with 16-byte stores (two dims x
// 4 tokens each).
template <int D>
__global__ __launch_bounds__(256) void kv_write_v_kernel(
    bf16_t* __restrict__ v_cache, const bf16_t* __restrict__ qkv, int qkv_stride,
    const int* __restrict__ seg_tok, const int* __restrict__ seg_len,
    const int* __restrict__ seg_blk, int Hq, int Hkv) {
  constexpr int BS = 32;
  constexpr int ROW = D + 2;  // padded LDS row (elements)
  __shared__ bf16_t tile[BS * ROW];
  const int seg = blockIdx.x, h = blockIdx.y;
  const int t0 = seg_tok[seg], n = seg_len[seg];
  const int64_t blk = seg_blk[seg];
  const int voff = (Hq + Hkv + h) * D;
  for (int v = threadIdx.x; v < BS * (D / 8); v += 256) {
    const int t = v / (D / 8), c = (v - t * (D / 8)) * 8;
    bf16x8 x;
    if (t < n) x = load_bf16x8(qkv + (int64_t)(t0 + t) * qkv_stride + voff + c);
    else for (int j = 0; j < 8; ++j) x[j] = f2bf(0.f);
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[t * ROW + c + j] = x[j];
  }
  __syncthreads();
  bf16_t* dst = v_cache + (blk * Hkv + h) * (int64_t)D * BS;
  for (int v = threadIdx.x; v < (BS / 4) * (D / 2); v += 256) {
    const int q4 = v / (D / 2), d = (v - q4 * (D / 2)) * 2;
    bf16x8 y;
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = tile[(4 * q4 + (j & 3)) * ROW + d + (j >> 2)];
    store_bf16x8(dst + q4 * (4 * D) + d * 4, y);
  }
}

int launch_kv_write_v(void* v_cache, const void* qkv, int qkv_stride, const int* seg_tok,
                      const int* seg_len, const int* seg_blk, int nseg, int Hq, int Hkv,
                      int D, int block_size, hipStream_t st) {
  if (nseg == 0) return 0;
  if (block_size != 32) return -1;
  dim3 grid(nseg, Hkv), block(256);
  switch (D) {
    case 64:
      hipLaunchKernelGGL(kv_write_v_kernel<64>, grid, block, 0, st, (bf16_t*)v_cache, (const bf16_t*)qkv, qkv_stride, seg_tok, seg_len, seg_blk, Hq, Hkv);
      break;
    case 128:
      hipLaunchKernelGGL(kv_write_v_kernel<128>, grid, block, 0, st, (bf16_t*)v_cache, (const bf16_t*)qkv, qkv_stride, seg_tok, seg_len, seg_blk, Hq, Hkv);
      break;
    case 256:
      hipLaunchKernelGGL(kv_write_v_kernel<256>, grid, block, 0, st, (bf16_t*)v_cache, (const bf16_t*)qkv, qkv_stride, seg_tok, seg_len, seg_blk, Hq, Hkv);
      break;
    default:
      return -1;
  }
  return (int)hipGetLastError();
}

}  // namespace drtc
