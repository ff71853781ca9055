// woq_gguf.hip -- GGUF Q4_0 weights and Q8_0 activations.
//
// A Q4_0 row is K/32 blocks {fp16 d; u8 qs[16]} (neural_speed/core/data_types.h:79-83), value = (nibble - 8) * d with
// element j < 16 in the low nibble of qs[j] and j >= 16 in the high nibble of qs[j - 16] (vectors/cpu/quantize.h:
// 686-704).  That is exactly a symmetric int4, group-32, fp16-scale weight, so nad_q4_0_repack_kernel writes it into
// the same MFMA tile layout as a BTLA blob (woq_layout.h) and every forward kernel serves it unchanged.
//
// The reference multiplies a Q4_0 matrix by quantizing the activation rows to Q8_0 (vec_dot_type, ne_layers.c:266-273;
// quantize_row_q8_0_reference, quantize.h:422-445) and summing per block sumi * d_w * d_a (vec_dot.h:187-204).
// nad_q8_0_quant_kernel is that quantizer; woq_i8.hip's GEMM runs the block dot products in its signed-activation mode.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

#include "woq_device.h"
#include "woq_kernels.h"
#include "woq_layout.h"

#pragma clang fp contract(off)

namespace nad {

// one thread per (row n, block b): 18 bytes in, four dwords of the tile + one fp16 scale out
__global__ void nad_q4_0_repack_kernel(const uint8_t* __restrict__ src, int n, int k, DeviceWeight w) {
  const int nb = k / 32;
  const int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= int64_t(n) * nb) return;
  const int row = int(idx / nb), b = int(idx % nb);
  const uint8_t* blk = src + (size_t(row) * nb + b) * 18;
  uint8_t qs[16];
#pragma unroll
  for (int j = 0; j < 16; j++) qs[j] = blk[2 + j];
  const int s = row >> 4, nl = row & 15;
  const int t = b >> 2, d = b & 3;
  uint32_t* tiles = static_cast<uint32_t*>(w.tiles);
#pragma unroll
  for (int kq = 0; kq < 4; kq++) {
    uint32_t word = 0;
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const int j = kq * 8 + e;
      const uint32_t nib = j < 16 ? (qs[j] & 15u) : (qs[j - 16] >> 4);
      const int p = (e & 1) ? 4 + (e >> 1) : (e >> 1);  // woq_layout.h int4 element order
      word |= nib << (4 * p);
    }
    tiles[(tile_index(w.kmajor, w.ns, w.nt, s, t) * 64 + kq * 16 + nl) * 4 + d] = word;
  }
  uint16_t dh = uint16_t(blk[0]) | (uint16_t(blk[1]) << 8);
  static_cast<uint16_t*>(w.scales)[scale_row(w.kmajor, w.ns, w.ng, s, b) * 16 + nl] = dh;
}

// quantize_row_q8_0_reference: per (row, 32-block) amax, d = amax / 127, q = roundf(x / d) (x * (1 / d)), d kept fp16
template <int AT>
__global__ __launch_bounds__(256) void nad_q8_0_quant_kernel(Q80Args a) {
  const int nb = a.K / 32;
  const int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= int64_t(a.M) * nb) return;
  const int row = int(idx / nb), b = int(idx % nb);
  const size_t rb = size_t(row) * a.lda + size_t(b) * 32;
  float x[32];
  float amax = 0.0f;
#pragma unroll
  for (int j = 0; j < 32; j++) {
    x[j] = a_elem<AT>(a.A, rb + j);
    const float v = fabsf(x[j]);
    amax = amax > v ? amax : v;  // MAX(amax, fabsf(v))
  }
  const float d = amax / 127.f;
  const float id = d != 0.f ? 1.0f / d : 0.0f;
  const __half dh = __float2half_rn(d);
  const float dy = __half2float(dh);
  int8_t* out = a.blocks ? a.blocks + (size_t(row) * nb + b) * 34 : nullptr;
  if (out) {
    const uint16_t bits = __half_as_ushort(dh);
    out[0] = int8_t(bits & 0xff);
    out[1] = int8_t(bits >> 8);
  }
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const int8_t q = int8_t(int(roundf(x[j] * id)));
    if (a.aq) a.aq[size_t(row) * a.ldq + b * 32 + j] = q;
    if (out) out[2 + j] = q;
  }
  if (a.aq && b == nb - 1)
    for (int k = a.K; k < a.kp; k++) a.aq[size_t(row) * a.ldq + k] = 0;
  if (a.sa) a.sa[size_t(row) * nb + b] = make_float2(dy, 0.f);
}

hipError_t launch_q4_0_repack(const uint8_t* src, int n, int k, const DeviceWeight& w, hipStream_t st) {
  const int64_t total = int64_t(n) * (k / 32);
  hipLaunchKernelGGL(nad_q4_0_repack_kernel, dim3(int((total + 255) / 256)), dim3(256), 0, st, src, n, k, w);
  return hipGetLastError();
}

hipError_t launch_q8_0_quant(const Q80Args& a, int act_t, hipStream_t st) {
  const int64_t total = int64_t(a.M) * (a.K / 32);
  const dim3 grid(int((total + 255) / 256));
  if (act_t == kActF32)
    hipLaunchKernelGGL(nad_q8_0_quant_kernel<kActF32>, grid, dim3(256), 0, st, a);
  else if (act_t == kActF16)
    hipLaunchKernelGGL(nad_q8_0_quant_kernel<kActF16>, grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(nad_q8_0_quant_kernel<kActBF16>, grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace nad
