// Varlen causal flash-attention forward on MFMA (gfx950), GQA/MQA-aware.
//
// Inputs are read straight out of the fused QKV GEMM output (after the
// in-place RoPE kernel), so no Q/K/V copies are made: sequence s occupies
// rows cu_seqlens[s] .. cu_seqlens[s+1] of the packed [T, qkv_stride] buffer.
//
// Work decomposition: grid = (n_q_tiles, Hq); a workgroup of 4 waves owns a
// 64-row query tile of one head (16 rows per wave).  K/V tiles of 64 keys
// are staged in LDS once per workgroup (K row-major padded to kill the
// 256-B-stride bank conflicts of the ds_read_b128 A-operand reads; V
// transposed to [d][key] so the P.V A-operand is two 8-B reads).
//
// MFMA formulation (16x16x32 bf16): the scores are computed transposed,
//   S^T[key, q] = K[key, :] . Q[q, :]   (A = K from LDS, B = Q^T in registers)
// so that the accumulator tiles of two 16-key halves become the P^T
// B-operand of O^T[d, q] += V^T[d, key] . P^T[key, q] without any lane
// movement (same token permutation trick as the decode kernel).  The online
// softmax per query column needs only two cross-lane xor-shuffles.
#include "common.h"
#include "launchers.h"

namespace drtc {

constexpr int kQT = 64;   // query rows per workgroup
constexpr int kKT = 64;   // keys per LDS tile

template <int D>
struct PrefillLds {
  static constexpr int KROW = D + 8;     // padded K row (elements)
  static constexpr int VROW = kKT + 4;   // padded V^T row (elements)
  static constexpr int K_ELEMS = kKT * KROW;
  static constexpr int V_ELEMS = D * VROW;
  static constexpr size_t BYTES = (size_t)(K_ELEMS + V_ELEMS) * 2;
};

template <int D>
__global__ __launch_bounds__(256) void prefill_attn_kernel(
    bf16_t* __restrict__ out, int out_stride, const bf16_t* __restrict__ qkv,
    int qkv_stride, int Hq, int Hkv, const int* __restrict__ cu_seqlens,
    const int* __restrict__ tile_seq, const int* __restrict__ tile_q0,
    float scale_log2e, int causal) {
  using L = PrefillLds<D>;
  constexpr int KS = D / 32;
  constexpr int NT = D / 16;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  bf16_t* k_lds = lds;
  bf16_t* vt_lds = lds + L::K_ELEMS;

  const int tile = blockIdx.x;
  const int hq = blockIdx.y;
  const int G = Hq / Hkv;
  const int hk = hq / G;
  const int seq = tile_seq[tile];
  const int q0 = tile_q0[tile];
  const int s_begin = cu_seqlens[seq];
  const int seqlen = cu_seqlens[seq + 1] - s_begin;
  const int lane = threadIdx.x & 63;
  const int w = wave_id_uniform();
  const int col = lane & 15, g = lane >> 4;
  const int qrow = q0 + 16 * w + col;  // this lane's query column (seq-local)

  // Q^T B-operand fragments.
  bf16x8 qf[KS];
  {
    const bf16_t* qp = qkv + (int64_t)(s_begin + qrow) * qkv_stride + hq * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (qrow < seqlen) qf[s] = load_bf16x8(qp + 32 * s + 8 * g);
      else for (int j = 0; j < 8; ++j) qf[s][j] = f2bf(0.f);
    }
  }
  f32x4 o[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) o[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = kNegBig, lsum = 0.f;

  const int kv_end = causal ? min(seqlen, q0 + kQT) : seqlen;
  const int ntiles = (kv_end + kKT - 1) / kKT;
  const int k_off = (Hq + hk) * D;
  const int v_off = (Hq + Hkv + hk) * D;

  for (int kt = 0; kt < ntiles; ++kt) {
    const int k0 = kt * kKT;
    // ---- stage K (row-major) and V^T (transposed) tiles
    constexpr int VPR = D / 8;  // 16-B vectors per row
    for (int v = threadIdx.x; v < kKT * VPR; v += 256) {
      const int key = v / VPR;
      const int c = (v - key * VPR) * 8;
      bf16x8 kv, vv;
      if (k0 + key < seqlen) {
        const bf16_t* rp = qkv + (int64_t)(s_begin + k0 + key) * qkv_stride;
        kv = load_bf16x8(rp + k_off + c);
        vv = load_bf16x8(rp + v_off + c);
      } else {
        for (int j = 0; j < 8; ++j) { kv[j] = f2bf(0.f); vv[j] = f2bf(0.f); }
      }
      store_bf16x8(k_lds + key * L::KROW + c, kv);
#pragma unroll
      for (int j = 0; j < 8; ++j) vt_lds[(c + j) * L::VROW + key] = vv[j];
    }
    __syncthreads();

    // ---- S^T = K . Q^T for 4 sub-tiles of 16 keys
    f32x4 sc[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      sc[st] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8 a = load_bf16x8(k_lds + (16 * st + col) * L::KROW + 32 * s + 8 * g);
        sc[st] = mfma16(a, qf[s], sc[st]);
      }
    }
    float bmax = kNegBig;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 16 * st + 4 * g + r;
        const bool ok = key < seqlen && (!causal || key <= qrow);
        sc[st][r] = ok ? sc[st][r] * scale_log2e : kNegBig;
        bmax = fmaxf(bmax, sc[st][r]);
      }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
    const float m_new = fmaxf(m, bmax);
    const float alpha = fast_exp2(m - m_new);
    m = m_new;
    bf16x8 pf[2];
    float psum = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pa = fast_exp2(sc[2 * ks][r] - m_new);
        const float pb = fast_exp2(sc[2 * ks + 1][r] - m_new);
        psum += pa + pb;
        pf[ks][r] = f2bf(pa);
        pf[ks][4 + r] = f2bf(pb);
      }
    lsum = lsum * alpha + psum;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      o[i] *= alpha;
      const bf16_t* vrow = vt_lds + (16 * i + col) * L::VROW;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x4 lo = load_bf16x4(vrow + 32 * ks + 4 * g);
        bf16x4 hi = load_bf16x4(vrow + 32 * ks + 16 + 4 * g);
        bf16x8 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) { a[j] = lo[j]; a[4 + j] = hi[j]; }
        o[i] = mfma16(a, pf[ks], o[i]);
      }
    }
    __syncthreads();
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (qrow < seqlen) {
    const float inv = 1.f / lsum;
    bf16_t* op = out + (int64_t)(s_begin + qrow) * out_stride + hq * D;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) op[16 * i + 4 * g + r] = f2bf(o[i][r] * inv);
  }
}

int launch_prefill_attn(void* out, int out_stride, const void* qkv,
                        int qkv_stride, int Hq, int Hkv, int D,
                        const int* cu_seqlens, const int* tile_seq,
                        const int* tile_q0, int ntiles, float scale, int causal,
                        hipStream_t st) {
  if (ntiles == 0) return 0;
  if (Hkv <= 0 || Hq % Hkv != 0) return -1;
  const float sl2 = scale * kLog2e;
  dim3 grid(ntiles, Hq), block(256);
  switch (D) {
    case 64:
      hipLaunchKernelGGL(prefill_attn_kernel<64>, grid, block, PrefillLds<64>::BYTES, st, (bf16_t*)out, out_stride, (const bf16_t*)qkv, qkv_stride, Hq, Hkv, cu_seqlens, tile_seq, tile_q0, sl2, causal);
      break;
    case 128:
      hipLaunchKernelGGL(prefill_attn_kernel<128>, grid, block, PrefillLds<128>::BYTES, st, (bf16_t*)out, out_stride, (const bf16_t*)qkv, qkv_stride, Hq, Hkv, cu_seqlens, tile_seq, tile_q0, sl2, causal);
      break;
    case 256:
      hipLaunchKernelGGL(prefill_attn_kernel<256>, grid, block, PrefillLds<256>::BYTES, st, (bf16_t*)out, out_stride, (const bf16_t*)qkv, qkv_stride, Hq, Hkv, cu_seqlens, tile_seq, tile_q0, sl2, causal);
      break;
    default:
      return -1;
  }
  return (int)hipGetLastError();
}

int configure_prefill() {
  return (int)hipFuncSetAttribute((const void*)prefill_attn_kernel<256>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)PrefillLds<256>::BYTES);
}

}  // namespace drtc
