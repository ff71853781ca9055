// woq_i8.hip -- the int8-compute mode: what the reference computes for a weight packed for an integer core
// (comp_int8, the default of the reference's Python quantizer).
//
//   * activations: u8 per (row, weight block), exactly kernel_ref.h:1824-1883 quantize_fp_u8_colblock
//     (scale = (max - min) / 255 with the running max starting at FLT_MIN for full blocks and 0 for the ragged tail,
//     zp = u8(-min / scale + 0.5), q = u8(zp + round(x / scale) + 0.5)); kept as s8 = u8 - 128 for the MFMA;
//   * weights: the tile layout's integers as s8 (q - zp), exact;
//   * per block: s32 = sum a_u8 * b_s8 on v_mfma_i32_16x16x32_i8 (the u8 offset restored exactly as 128 * sum b), then
//     C += float(s32) * (sA * sB) and C -= (float(zpA) * sA) * reduceB, blocks in K order: the kblock core's
//     generate_f32_accumulate + generate_zp_correction (bestla_gemm.h:2983-3050), driven as
//     LauncherIntKBlock::run_block does (bestla_wrapper.h:768-831).  reduceB is the blob's bf16 reduce.
//
// Kernel shapes: a workgroup is 4 waves.  M <= 16: the 4 waves split one stripe's K range (one 16-row MFMA tile),
// partials summed through LDS; M > 16: each wave owns one stripe and 64 rows (4 MFMA row tiles).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "woq_device.h"
#include "woq_kernels.h"

#pragma clang fp contract(off)

namespace nad {
namespace i8 {

typedef int i4_t __attribute__((ext_vector_type(4)));

// x86 float -> int32 (cvttss2si): NaN and out-of-range give INT32_MIN (the reference's int(roundf(x)) on the host)
__device__ __forceinline__ int f2i_x86(float x) {
  if (__builtin_isnan(x) || x >= 2147483648.0f || x < -2147483648.0f) return INT32_MIN;
  return int(x);
}
// bestla_utils.h cast<float, uint8_t>: + 0.5, clamp to [0, 255] (std::min / std::max argument order), truncate
__device__ __forceinline__ uint32_t cast_u8(float v) {
  v = v + 0.5f;
  v = (255.f < v) ? 255.f : v;
  v = (v < 0.f) ? 0.f : v;
  return uint32_t(f2i_x86(v)) & 0xffu;
}

template <int AT>
__global__ __launch_bounds__(256) void quant_u8_kernel(QuantU8Args a) {
  const int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= int64_t(a.M) * a.ng) return;
  const int row = int(idx / a.ng), g = int(idx % a.ng);
  const int k0 = g * a.bs;
  const int len = min(a.bs, a.K - k0);
  const bool full = k0 + a.bs <= a.K;
  const size_t rb = size_t(row) * a.lda;
  auto x_at = [&](int k) { return a_elem<AT>(a.A, rb + size_t(a.shuffle ? a.shuffle[k] : k)); };
  float maxval = full ? FLT_MIN : 0.f, minval = 0.f;
  for (int j = 0; j < len; j++) {
    const float x = x_at(k0 + j);
    maxval = (x < maxval) ? maxval : x;  // std::max(x, maxval)
    minval = (minval < x) ? minval : x;  // std::min(x, minval)
  }
  const float scale = (maxval - minval) / 255.f;
  const uint32_t zp = cast_u8((0.f - minval) / scale);
  const float rscale = 1.f / scale;
  const float zpf = float(zp);
  int sum = 0;
  for (int j = 0; j < len; j++) {
    const int q = f2i_x86(roundf(x_at(k0 + j) * rscale));
    sum = int(uint32_t(sum) + uint32_t(q));
    const uint32_t u = cast_u8(zpf + float(q));
    if (a.aq) a.aq[size_t(row) * a.ldq + k0 + j] = int8_t(u ^ 0x80u);
    if (a.q_u8) a.q_u8[size_t(row) * a.ldu + k0 + j] = uint8_t(u);
  }
  if (a.aq && g == a.ng - 1)
    for (int k = a.K; k < a.kp; k++) a.aq[size_t(row) * a.ldq + k] = 0;
  if (a.sa) a.sa[size_t(row) * a.ng + g] = make_float2(scale, zpf * scale);
  const size_t so = size_t(row) * a.ld_scale + g;
  if (a.s_out) a.s_out[so] = scale;
  if (a.z_out) a.z_out[so] = uint8_t(zp);
  if (a.red_out) a.red_out[so] = float(sum) * scale;
}

// B fragment of one 32-deep step as 8 signed bytes (element j at byte j): tile layout (woq_layout.h) -> q - zp
template <int BITS>
__device__ __forceinline__ void b_step(const u4_t& b, int d, uint32_t bias, uint32_t& lo, uint32_t& hi) {
  if constexpr (BITS == 8) {
    // byte = q + 128 (S5..S8); q - zp fits s8 for every format the int8 core takes (S8 is symmetric there,
    // bestla_gemm.cpp:250), so add bias = (-zp) mod 256 per byte without carries between bytes (SWAR byte add)
    auto add_bytes = [](uint32_t x, uint32_t y) {
      return ((x & 0x7f7f7f7fu) + (y & 0x7f7f7f7fu)) ^ ((x ^ y) & 0x80808080u);
    };
    lo = add_bytes(b[2 * d] ^ 0x80808080u, bias);
    hi = add_bytes(b[2 * d + 1] ^ 0x80808080u, bias);
    return;
  } else {
    constexpr int SH = BITS;                    // field stride between the two elements sharing a byte pair
    constexpr uint32_t M = BITS == 4 ? 0x000F000Fu : 0x00030003u;
    const uint32_t w = BITS == 4 ? b[d] : (b[d >> 1] >> ((d & 1) * 8));
    const uint32_t x0 = w & M, x1 = (w >> SH) & M, x2 = (w >> (2 * SH)) & M, x3 = (w >> (3 * SH)) & M;
    // [x0.b0, x0.b2, x1.b0, x1.b2] = elements 0..3, likewise 4..7; + (128 - bias - zp) per byte, then flip the sign bit
    lo = (__builtin_amdgcn_perm(x1, x0, 0x06040200u) + bias) ^ 0x80808080u;
    hi = (__builtin_amdgcn_perm(x3, x2, 0x06040200u) + bias) ^ 0x80808080u;
  }
}

template <int BITS, int RT, bool KSPLIT>
__global__ __launch_bounds__(256) void woq_i8_kernel(I8Args a) {
  constexpr int KT = BITS == 4 ? 128 : (BITS == 2 ? 256 : 64);
  constexpr int SPT = KT / 32;
  constexpr int BIAS = BITS == 4 ? 8 : (BITS == 2 ? 2 : 128);
  __shared__ float part[KSPLIT ? 3 * 64 * 4 * RT : 1];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nl = lane & 15, kq = lane >> 4;
  const SkinnyWeight& W = a.w;
  const int s = KSPLIT ? blockIdx.y : blockIdx.y * 4 + wave;
  const int m0 = blockIdx.x * 16 * RT;
  const bool live = s < W.ns;
  const int sc = min(s, W.ns - 1);
  const int n = sc * 16 + nl;
  const int nsteps = (a.K + 31) / 32;
  const int bs = W.bs;
  const int spg = bs / 32;  // steps per group (per-channel: bs >= K, one group)
  // this wave's step range: KSPLIT splits whole groups across the 4 waves
  int st0 = 0, st1 = nsteps;
  if constexpr (KSPLIT) {
    const int g0 = (W.ng * wave) / 4, g1 = (W.ng * (wave + 1)) / 4;
    st0 = min(g0 * spg, nsteps);
    st1 = min(g1 * spg, nsteps);
  }

  i4_t acc[RT];
  float c[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; rt++) {
    acc[rt] = i4_t{0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; r++) c[rt][r] = 0.f;
  }
  int sb = 0;
  const u4_t* tiles = reinterpret_cast<const u4_t*>(W.tiles);
  const int8_t* arow[RT];
#pragma unroll
  for (int rt = 0; rt < RT; rt++) arow[rt] = a.aq + size_t(min(m0 + rt * 16 + nl, a.M - 1)) * a.ldq + kq * 8;

  // one tile and one step of A in flight ahead of the MFMA
  const int tlast = st1 > st0 ? (st1 - 1) / SPT : 0;
  auto tile_at = [&](int t) { return tiles[tile_index(W.kmajor, W.ns, W.nt, sc, min(t, tlast)) * 64 + lane]; };
  u4_t bt = tile_at(st0 / SPT), bnx = tile_at(st0 / SPT + 1);
  int tcur = st0 / SPT;
  long anx[RT];
#pragma unroll
  for (int rt = 0; rt < RT; rt++) anx[rt] = st0 < st1 ? *reinterpret_cast<const long*>(arow[rt] + st0 * 32) : 0;
  uint32_t bias = 0;
  for (int st = st0; st < st1; st++) {
    const int t = st / SPT, d = st % SPT;
    if (t != tcur) {
      bt = bnx;
      bnx = tile_at(t + 1);
      tcur = t;
    }
    long av[RT];
#pragma unroll
    for (int rt = 0; rt < RT; rt++) {
      av[rt] = anx[rt];
      if (st + 1 < st1) anx[rt] = *reinterpret_cast<const long*>(arow[rt] + (st + 1) * 32);
    }
    const int g = min(st / spg, W.ng - 1);
    if (st == st0 || st % spg == 0) {
      const int zp = W.zps ? int(W.zps[scale_row(W.kmajor, W.ns, W.ng, sc, g) * 16 + nl]) : 0;
      bias = uint32_t((128 - BIAS - zp) & 0xff) * 0x01010101u;
    }
    uint32_t lo, hi;
    b_step<BITS>(bt, d, bias, lo, hi);
    const int k0 = st * 32;
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
      acc[rt] = __builtin_amdgcn_mfma_i32_16x16x32_i8(av[rt], long(uint64_t(lo) | (uint64_t(hi) << 32)), acc[rt], 0, 0,
                                                      0);
    // sum of this lane's 8 weights (k < K only: the padded rows of a tile are not part of the block)
    const int valid = a.K - (k0 + kq * 8);
    uint32_t ml = 0xffffffffu, mh = 0xffffffffu;
    if (valid < 8) {
      ml = valid <= 0 ? 0u : (valid >= 4 ? 0xffffffffu : ((1u << (8 * valid)) - 1u));
      mh = valid <= 4 ? 0u : ((1u << (8 * (valid - 4))) - 1u);
    }
    sb = __builtin_amdgcn_sdot4(int(lo & ml), 0x01010101, sb, false);
    sb = __builtin_amdgcn_sdot4(int(hi & mh), 0x01010101, sb, false);
    const bool gend = (st + 1) % spg == 0 || st + 1 == nsteps;
    if (gend) {
      int sbt = sb;
      sbt += __shfl_xor(sbt, 16);
      sbt += __shfl_xor(sbt, 32);
      const float sB = load_scale(W.scales, scale_row(W.kmajor, W.ns, W.ng, sc, g) * 16 + nl, a.scale_t);
      const float redB = a.red ? bf16_bits_to_f32(a.red[size_t(g) * a.red_ld + n]) : 0.f;
      if (a.a_signed) {  // Q8_0 x Q4_0: sumf += sumi * d_w * d_a (vec_dot.h:201)
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int row = min(m0 + rt * 16 + kq * 4 + r, a.M - 1);
            const float2 sz = a.sa[size_t(row) * W.ng + g];
            c[rt][r] = c[rt][r] + (float(acc[rt][r]) * sB) * sz.x;
          }
      } else {
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int row = min(m0 + rt * 16 + kq * 4 + r, a.M - 1);
            const float2 sz = a.sa[size_t(row) * W.ng + g];
            const int dot = acc[rt][r] + 128 * sbt;
            c[rt][r] = c[rt][r] + float(dot) * (sz.x * sB);
            c[rt][r] = c[rt][r] - sz.y * redB;
          }
      }
#pragma unroll
      for (int rt = 0; rt < RT; rt++) acc[rt] = i4_t{0, 0, 0, 0};
      sb = 0;
    }
  }

  if constexpr (KSPLIT) {
    if (wave > 0) {
#pragma unroll
      for (int rt = 0; rt < RT; rt++)
#pragma unroll
        for (int r = 0; r < 4; r++) part[((wave - 1) * 4 * RT + rt * 4 + r) * 64 + lane] = c[rt][r];
    }
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int w = 0; w < 3; w++)
#pragma unroll
      for (int rt = 0; rt < RT; rt++)
#pragma unroll
        for (int r = 0; r < 4; r++) c[rt][r] = c[rt][r] + part[(w * 4 * RT + rt * 4 + r) * 64 + lane];
  }
  if (!live || n >= W.n) return;
#pragma unroll
  for (int rt = 0; rt < RT; rt++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = m0 + rt * 16 + kq * 4 + r;
      if (row >= a.M) continue;
      float v = c[rt][r];
      switch (a.epi) {
        case kEpiBias:
          v += W.bias[size_t(row) * W.bias_ld + n];
          break;
        case kEpiAddGelu:
          v = gelu_f(v + W.bias[size_t(row) * W.bias_ld + n]);
          break;
        case kEpiGelu:
          v = gelu_f(v);
          break;
        case kEpiSilu:
          v = silu_f(v);
          break;
        case kEpiResAdd:
          v += a.res[size_t(row) * a.ld_res + n];
          break;
        case kEpiSiluMul:  // second pass of the FFN: aux holds act(x.w1)
          v = a.aux[size_t(row) * a.ld_aux + n] * v;
          break;
        default:
          break;
      }
      W.out[size_t(row) * W.ldo + n] = v;
    }
}

}  // namespace i8

hipError_t launch_quant_u8(const QuantU8Args& a, int act_t, hipStream_t st) {
  const int64_t total = int64_t(a.M) * a.ng;
  const int blocks = int((total + 255) / 256);
  if (act_t == kActF32)
    hipLaunchKernelGGL(i8::quant_u8_kernel<kActF32>, dim3(blocks), dim3(256), 0, st, a);
  else if (act_t == kActF16)
    hipLaunchKernelGGL(i8::quant_u8_kernel<kActF16>, dim3(blocks), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(i8::quant_u8_kernel<kActBF16>, dim3(blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_i8(const I8Args& a, int bits, hipStream_t st) {
  const bool small = a.M <= 16;
  const dim3 grid(small ? 1 : (a.M + 63) / 64, small ? a.w.ns : (a.w.ns + 3) / 4);
#define NAD_I8(B)                                                                     \
  do {                                                                                \
    if (small)                                                                        \
      hipLaunchKernelGGL((i8::woq_i8_kernel<B, 1, true>), grid, dim3(256), 0, st, a); \
    else                                                                              \
      hipLaunchKernelGGL((i8::woq_i8_kernel<B, 4, false>), grid, dim3(256), 0, st, a); \
  } while (0)
  if (bits == 4)
    NAD_I8(4);
  else if (bits == 2)
    NAD_I8(2);
  else
    NAD_I8(8);
#undef NAD_I8
  return hipGetLastError();
}

}  // namespace nad
