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

// (x & m) | c as ONE v_and_or_b32 (hipcc emits v_and_b32 + v_or_b32 for the C form: the literal mask and magic cannot
// share a VOP3 on gfx9; here the mask sits in an SGPR and the magic in a VGPR)
__device__ __forceinline__ uint32_t dq_and_or(uint32_t x, uint32_t m, uint32_t c) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(m), "v"(c));
  return r;
}

// One MFMA step's B fragment (8 fp16 = exact integers q - zp) from the packed dwords.
//   c2 = (-(1024 + bias + zp)) broadcast as half2.
template <int BITS>
__device__ __forceinline__ h8_t dequant_step(const u4_t& b, int d, h2_t c2) {
  h2_t p0, p1, p2, p3;
  if constexpr (BITS == 4) {
    uint32_t w = b[d];
    p0 = as_h2(dq_and_or(w, 0x000F000Fu, 0x64006400u));
    p1 = as_h2(dq_and_or(w >> 4, 0x000F000Fu, 0x64006400u));
    p2 = as_h2(dq_and_or(w >> 8, 0x000F000Fu, 0x64006400u));
    p3 = as_h2(dq_and_or(w >> 12, 0x000F000Fu, 0x64006400u));
  } else if constexpr (BITS == 2) {
    uint32_t w = b[d >> 1];
    int sh = (d & 1) * 8;
    p0 = as_h2(dq_and_or(w >> (sh + 0), 0x00030003u, 0x64006400u));
    p1 = as_h2(dq_and_or(w >> (sh + 2), 0x00030003u, 0x64006400u));
    p2 = as_h2(dq_and_or(w >> (sh + 4), 0x00030003u, 0x64006400u));
    p3 = as_h2(dq_and_or(w >> (sh + 6), 0x00030003u, 0x64006400u));
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

// int2 through scaled magic numbers: crumb i of each 16-bit half (bits 2i .. 2i + 1 of x) or'ed into 0x6400 is the fp16
// 1024 + 4^i q (exact: 4^i q <= 192), and fma(that, 4^-i, -(1024 * 4^-i + bias + zp)) is q - bias - zp exactly (fused,
// and every intermediate is representable).  4 v_and_or + 4 packed fp16 ops per 8 weights, plus one shift for the odd
// step of a dword -- dequant_step<2> spends a shift per crumb pair.  Same element order as dequant_step<2>.
__device__ __forceinline__ h2_t zp_const(int bias_plus_zp);
struct Dq2c {
  h2_t c0, c1, c2, c3;
};
__device__ __forceinline__ h2_t h2_splat(float v) {
  h2_t r;
  r[0] = _Float16(v);
  r[1] = _Float16(v);
  return r;
}
__device__ __forceinline__ Dq2c dq2_consts(int bias_plus_zp) {
  const float b = float(bias_plus_zp);
  return Dq2c{h2_splat(-(1024.f + b)), h2_splat(-(256.f + b)), h2_splat(-(64.f + b)), h2_splat(-(16.f + b))};
}
// x: the dword already shifted right by 8 for the odd step (b[d >> 1] >> ((d & 1) * 8))
__device__ __forceinline__ h8_t dequant2s(uint32_t x, const Dq2c& c) {
  const uint32_t mag = 0x64006400u;
  const h2_t p0 = as_h2(dq_and_or(x, 0x00030003u, mag)) + c.c0;
  const h2_t p1 = __builtin_elementwise_fma(as_h2(dq_and_or(x, 0x000C000Cu, mag)), h2_splat(0.25f), c.c1);
  const h2_t p2 = __builtin_elementwise_fma(as_h2(dq_and_or(x, 0x00300030u, mag)), h2_splat(0.0625f), c.c2);
  const h2_t p3 = __builtin_elementwise_fma(as_h2(dq_and_or(x, 0x00C000C0u, mag)), h2_splat(0.015625f), c.c3);
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
// one 32-deep step of an int2 tile (the dwords of a lane's 16 B) through the scaled magic numbers (measured faster than
// dequant_step<2>, round 3)
__device__ __forceinline__ h8_t dequant2_step(const u4_t& b, int d, int bias_plus_zp) {
  return dequant2s(b[d >> 1] >> ((d & 1) * 8), dq2_consts(bias_plus_zp));
}

// NFloat 4-bit weights (F4_BNB, F4_E2M1, F4_NF4): code -> value LUTs of bestla_utils.h:749-790, rounded to fp16 for
// the MFMA B operand (the fp32 group scale is applied after the MFMA, as for the integer formats)
static __constant__ _Float16 kF4LutH[3][16] = {
    {_Float16(0.00000000f), _Float16(5.208333333e-03f), _Float16(0.66666667f), _Float16(1.00000000f),
     _Float16(0.33333333f), _Float16(0.50000000f), _Float16(0.16666667f), _Float16(0.25000000f),
     _Float16(-0.00000000f), _Float16(-5.208333333e-03f), _Float16(-0.66666667f), _Float16(-1.00000000f),
     _Float16(-0.33333333f), _Float16(-0.50000000f), _Float16(-0.16666667f), _Float16(-0.25000000f)},
    {_Float16(0.f), _Float16(0.010416666666666666f), _Float16(0.16666666666666666f), _Float16(0.25f),
     _Float16(0.333333333333333f), _Float16(0.5f), _Float16(0.6666666666666f), _Float16(1.f), _Float16(-0.f),
     _Float16(-0.010416666666666666f), _Float16(-0.16666666666666666f), _Float16(-0.25f),
     _Float16(-0.333333333333333f), _Float16(-0.5f), _Float16(-0.6666666666666f), _Float16(-1.f)},
    {_Float16(0.f), _Float16(-0.6961928009986877f), _Float16(-0.5250730514526367f), _Float16(-0.39491748809814453f),
     _Float16(-0.28444138169288635f), _Float16(-0.18477343022823334f), _Float16(-0.09105003625154495f),
     _Float16(-1.f), _Float16(0.07958029955625534f), _Float16(0.16093020141124725f), _Float16(0.24611230194568634f),
     _Float16(0.33791524171829224f), _Float16(0.44070982933044434f), _Float16(0.5626170039176941f),
     _Float16(0.7229568362236023f), _Float16(1.0f)}};

// the 16 fp16 LUT entries as byte planes: lo[i] holds the low bytes of entries 4i..4i+3, hi[i] the high bytes
struct F4Lut {
  uint32_t lo[4], hi[4];
};
__device__ __forceinline__ F4Lut f4_lut_regs(int kind) {
  F4Lut L;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint16_t v = __builtin_bit_cast(uint16_t, kF4LutH[kind][4 * i + b]);
      lo |= uint32_t(v & 0xFF) << (8 * b);
      hi |= uint32_t(v >> 8) << (8 * b);
    }
    L.lo[i] = lo;
    L.hi[i] = hi;
  }
  return L;
}
// four codes (low nibbles of the bytes of N) -> the low / high bytes of their fp16 values: a byte permute from each
// half of the table, then a per-byte select on the code's bit 3
__device__ __forceinline__ void f4_lookup(uint32_t N, const F4Lut& L, uint32_t& lob, uint32_t& hib) {
  const uint32_t S = N & 0x07070707u;
  const uint32_t M = ((N >> 3) & 0x01010101u) * 0xFFu;
  const uint32_t l0 = __builtin_amdgcn_perm(L.lo[1], L.lo[0], S), l1 = __builtin_amdgcn_perm(L.lo[3], L.lo[2], S);
  const uint32_t h0 = __builtin_amdgcn_perm(L.hi[1], L.hi[0], S), h1 = __builtin_amdgcn_perm(L.hi[3], L.hi[2], S);
  lob = (l0 & ~M) | (l1 & M);
  hib = (h0 & ~M) | (h1 & M);
}
// one 32-deep step of a 4-bit tile (int4 element order, woq_layout.h) through the LUT -> 8 fp16 B-operand values
__device__ __forceinline__ h8_t dequant_f4(const u4_t& b, int d, const F4Lut& L) {
  const uint32_t w = b[d];
  uint32_t la, ha, lb, hb;
  f4_lookup(w & 0x0F0F0F0Fu, L, la, ha);         // slots: elements 0, 4, 1, 5
  f4_lookup((w >> 4) & 0x0F0F0F0Fu, L, lb, hb);  // slots: elements 2, 6, 3, 7
  const h2_t p01 = as_h2(__builtin_amdgcn_perm(ha, la, 0x06020400u));
  const h2_t p23 = as_h2(__builtin_amdgcn_perm(hb, lb, 0x06020400u));
  const h2_t p45 = as_h2(__builtin_amdgcn_perm(ha, la, 0x07030501u));
  const h2_t p67 = as_h2(__builtin_amdgcn_perm(hb, lb, 0x07030501u));
  h8_t r;
  r[0] = p01[0];
  r[1] = p01[1];
  r[2] = p23[0];
  r[3] = p23[1];
  r[4] = p45[0];
  r[5] = p45[1];
  r[6] = p67[0];
  r[7] = p67[1];
  return r;
}

// NFloat 8-bit weights: raw codes in the int8 layout -> the exact fp16 of f8_to_fp32 (kernel_ref.h:984-1001, which
// reads every exponent field as a normal one).  E4M3: fp16 exponent = e + 8, mantissa m << 7.  E5M2: the code is the
// fp16's top byte for e >= 1; e = 0 (2^-15 (1 + m/4)) is the fp16 subnormal (m << 7) + 0x200 -- as bit patterns the
// right value is max(c << 8, ((c << 8) >> 1) + 0x200) per half for every e < 31 (e = 31 is rejected at load).
typedef uint16_t us2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t f8_pair(uint32_t w, uint32_t sel_lo, uint32_t sel_hi, bool e5m2) {
  if (!e5m2) {
    const uint32_t t = __builtin_amdgcn_perm(0u, w, sel_lo);  // codes in the low byte of each half
    return (((t & 0x007F007Fu) << 7) + 0x20002000u) | ((t & 0x00800080u) << 8);
  }
  const uint32_t t = __builtin_amdgcn_perm(0u, w, sel_hi);    // codes in the high byte of each half
  const uint32_t mag = t & 0x7FFF7FFFu;
  const us2_t r = __builtin_elementwise_max(__builtin_bit_cast(us2_t, mag),
                                            __builtin_bit_cast(us2_t, (mag >> 1) + 0x02000200u));
  return __builtin_bit_cast(uint32_t, r) | (t & 0x80008000u);
}
__device__ __forceinline__ h8_t dequant_f8(const u4_t& b, int d, bool e5m2) {
  const uint32_t w0 = b[2 * d], w1 = b[2 * d + 1];
  const h2_t p0 = as_h2(f8_pair(w0, 0x04010400u, 0x01040004u, e5m2));
  const h2_t p1 = as_h2(f8_pair(w0, 0x04030402u, 0x03040204u, e5m2));
  const h2_t p2 = as_h2(f8_pair(w1, 0x04010400u, 0x01040004u, e5m2));
  const h2_t p3 = as_h2(f8_pair(w1, 0x04030402u, 0x03040204u, e5m2));
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

// Prefill epilogue of four consecutive outputs (row, n0 .. n0 + 3) of a gemm3 / gemm4 / split-K reduce: the fused op,
// then the store -- fp32 into w.out, or fp16 (RNE) into out16 when the FFN keeps its intermediates in fp16.
// W: the weight whose output this is (a.w, or one of gemm7's fused weights)
__device__ __forceinline__ void gemm_epilogue4(const GemmArgs& a, const SkinnyWeight& W, int row, int n0, float (&v)[4]) {
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int n = n0 + e;
    if (n >= W.n) break;
    switch (a.epi) {
      case kEpiBias:
        v[e] += W.bias[size_t(row) * W.bias_ld + n];
        break;
      case kEpiAddGelu:
        v[e] = gelu_f(v[e] + W.bias[size_t(row) * W.bias_ld + n]);
        break;
      case kEpiGelu:
        v[e] = gelu_f(v[e]);
        break;
      case kEpiSilu:
        v[e] = silu_f(v[e]);
        break;
      case kEpiResAdd:
        v[e] += a.res[size_t(row) * a.ld_res + n];
        break;
      case kEpiSiluMul:  // second GEMM of the FFN: aux holds act(x.w1)
        v[e] = (a.aux16 ? float(a.aux16[size_t(row) * a.ld_aux + n]) : a.aux[size_t(row) * a.ld_aux + n]) * v[e];
        break;
      default:
        break;
    }
  }
  const bool full = n0 + 3 < W.n;
  if (a.out16) {
    _Float16* o = a.out16 + size_t(row) * a.ldo16 + n0;
    if (full && (reinterpret_cast<uintptr_t>(o) & 7) == 0) {
      typedef _Float16 h4v __attribute__((ext_vector_type(4)));
      *reinterpret_cast<h4v*>(o) = h4v{_Float16(v[0]), _Float16(v[1]), _Float16(v[2]), _Float16(v[3])};
    } else {
#pragma unroll
      for (int e = 0; e < 4; e++)
        if (n0 + e < W.n) o[e] = _Float16(v[e]);
    }
    return;
  }
  float* o = W.out + size_t(row) * W.ldo + n0;
  if (full && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int e = 0; e < 4; e++)
      if (n0 + e < W.n) o[e] = v[e];
  }
}
__device__ __forceinline__ void gemm_epilogue4(const GemmArgs& a, int row, int n0, float (&v)[4]) {
  gemm_epilogue4(a, a.w, row, n0, v);
}

}  // namespace nad
