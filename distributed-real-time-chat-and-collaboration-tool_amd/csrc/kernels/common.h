// Shared device helpers for the CDNA4 (gfx950) kernels of drtc_amd.
//
// Everything here is written for wave64 / MFMA on MI355X directly: 16-byte
// vector memory ops, hardware bf16 conversion (v_cvt_pk_bf16_f32), 64-lane
// shuffles and the bf16 MFMA operand types.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DRTC_DEVICE __device__ __forceinline__

typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegBig = -1.0e30f;  // finite "-inf": keeps (m_a - m_b) NaN-free

DRTC_DEVICE float bf2f(bf16_t x) { return (float)x; }
DRTC_DEVICE bf16_t f2bf(float x) { return (bf16_t)x; }  // RNE via v_cvt_pk_bf16_f32

DRTC_DEVICE bf16x8 load_bf16x8(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}
DRTC_DEVICE void store_bf16x8(bf16_t* p, bf16x8 v) {
  *reinterpret_cast<bf16x8*>(p) = v;
}
DRTC_DEVICE bf16x4 load_bf16x4(const bf16_t* p) {
  return *reinterpret_cast<const bf16x4*>(p);
}

DRTC_DEVICE float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

DRTC_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DRTC_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 16x16x32 bf16 MFMA (gfx950).  Operand maps (cdna_hip_programming.md §3):
//   A: lane l holds A[row l&15][k = 8*(l>>4) + j], j = 0..7
//   B: lane l holds B[k = 8*(l>>4) + j][col l&15]
//   C: lane l holds C[row 4*(l>>4) + r][col l&15], r = 0..3
DRTC_DEVICE f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Gated-MLP activation of the gate value (ACT 0 = SiLU, 1 = tanh-GELU); the
// one definition shared by act_glu_kernel and the fused skinny GEMM.
template <int ACT>
DRTC_DEVICE float act_value(float gf) {
  if constexpr (ACT == 0) {
    return gf / (1.f + __expf(-gf));
  } else {
    // 0.5 x (1 + tanh(u)) = x / (1 + exp(-2 u)): one exp and one divide instead of tanhf's
    // range-reduced polynomial (the GEMM epilogues that gate with it keep 256 accumulators live)
    const float k0 = 0.7978845608028654f;  // sqrt(2/pi)
    const float inner = k0 * (gf + 0.044715f * gf * gf * gf);
    return gf / (1.f + __expf(-2.f * inner));
  }
}

DRTC_DEVICE int lane_id() { return threadIdx.x & 63; }
DRTC_DEVICE int wave_id_uniform() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}
