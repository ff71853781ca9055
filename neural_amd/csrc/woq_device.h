// woq_device.h -- device helpers shared by the gfx950 WOQ kernels (woq_kernels.hip, woq_gemv.hip): fp16/bf16 bit
// conversions, the 0x6400 magic-number dequantization of one MFMA B fragment, activation loaders and the epilogue
// activations (bestla_common.hpp:121-216).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "woq_kernels.h"

namespace nad {

typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u4_t __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------ helpers
__device__ __forceinline__ float bf16_bits_to_f32(uint16_t x) { return __uint_as_float(uint32_t(x) << 16); }
__device__ __forceinline__ float f16_bits_to_f32(uint16_t x) {
  return float(__builtin_bit_cast(_Float16, x));
}

__device__ __forceinline__ float load_scale(const void* p, size_t i, int st) {
  if (st == kScaleF32) return static_cast<const float*>(p)[i];
  uint16_t h = static_cast<const uint16_t*>(p)[i];
  return st == kScaleBF16 ? bf16_bits_to_f32(h) : f16_bits_to_f32(h);
}

__device__ __forceinline__ h2_t as_h2(uint32_t v) { return __builtin_bit_cast(h2_t, v); }

// One MFMA step's B fragment (8 fp16 = exact integers q - zp) from the packed dwords.
//   c2 = (-(1024 + bias + zp)) broadcast as half2.
template <int BITS>
__device__ __forceinline__ h8_t dequant_step(const u4_t& b, int d, h2_t c2) {
  h2_t p0, p1, p2, p3;
  if constexpr (BITS == 4) {
    uint32_t w = b[d];
    p0 = as_h2(((w >> 0) & 0x000F000Fu) | 0x64006400u);
    p1 = as_h2(((w >> 4) & 0x000F000Fu) | 0x64006400u);
    p2 = as_h2(((w >> 8) & 0x000F000Fu) | 0x64006400u);
    p3 = as_h2(((w >> 12) & 0x000F000Fu) | 0x64006400u);
  } else if constexpr (BITS == 2) {
    uint32_t w = b[d >> 1];
    int sh = (d & 1) * 8;
    p0 = as_h2(((w >> (sh + 0)) & 0x00030003u) | 0x64006400u);
    p1 = as_h2(((w >> (sh + 2)) & 0x00030003u) | 0x64006400u);
    p2 = as_h2(((w >> (sh + 4)) & 0x00030003u) | 0x64006400u);
    p3 = as_h2(((w >> (sh + 6)) & 0x00030003u) | 0x64006400u);
  } else {
    uint32_t w0 = b[2 * d], w1 = b[2 * d + 1];
    p0 = as_h2(__builtin_amdgcn_perm(0x64646464u, w0, 0x04010400u));
    p1 = as_h2(__builtin_amdgcn_perm(0x64646464u, w0, 0x04030402u));
    p2 = as_h2(__builtin_amdgcn_perm(0x64646464u, w1, 0x04010400u));
    p3 = as_h2(__builtin_amdgcn_perm(0x64646464u, w1, 0x04030402u));
  }
  p0 += c2;
  p1 += c2;
  p2 += c2;
  p3 += c2;
  h8_t r;
  r[0] = p0[0];
  r[1] = p0[1];
  r[2] = p1[0];
  r[3] = p1[1];
  r[4] = p2[0];
  r[5] = p2[1];
  r[6] = p3[0];
  r[7] = p3[1];
  return r;
}

template <int BITS>
__device__ __forceinline__ constexpr int bias_of() {
  return BITS == 4 ? 8 : (BITS == 2 ? 2 : 128);
}

__device__ __forceinline__ h2_t zp_const(int bias_plus_zp) {
  _Float16 c = _Float16(-(1024 + bias_plus_zp));
  h2_t r;
  r[0] = c;
  r[1] = c;
  return r;
}

// activation element loaders -> float
template <int AT>
__device__ __forceinline__ float a_elem(const void* A, size_t idx) {
  if constexpr (AT == kActF32) return static_cast<const float*>(A)[idx];
  if constexpr (AT == kActF16) return float(static_cast<const _Float16*>(A)[idx]);
  return bf16_bits_to_f32(static_cast<const uint16_t*>(A)[idx]);
}

// load 8 consecutive activation values A[row][k0..k0+7] (zero beyond K), optional act-order gather
template <int AT>
__device__ __forceinline__ void load_a8(const void* A, int lda, int row, int k0, int K, const int32_t* shf, bool vec_ok,
                                        float (&v)[8]) {
  const size_t base = size_t(row) * lda;
  if (shf == nullptr && vec_ok && k0 + 8 <= K) {
    if constexpr (AT == kActF32) {
      const float4* p = reinterpret_cast<const float4*>(static_cast<const float*>(A) + base + k0);
      float4 x = p[0], y = p[1];
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
      v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    } else {
      uint4 x = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(A) + base + k0);
      uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        if constexpr (AT == kActF16) {
          h2_t h = as_h2(w[i]);
          v[2 * i] = float(h[0]);
          v[2 * i + 1] = float(h[1]);
        } else {
          v[2 * i] = __uint_as_float(w[i] << 16);
          v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      int k = k0 + j;
      v[j] = 0.f;
      if (k < K) v[j] = a_elem<AT>(A, base + (shf ? shf[k] : k));
    }
  }
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float gelu_f(float x) {
  return 0.5f * x * (1.f + tanhf(0.7978845834732056f * (x + 0.044714998453855515f * x * x * x)));
}

}  // namespace nad
