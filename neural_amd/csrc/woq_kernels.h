// woq_kernels.h -- launch-argument structs and launchers of the gfx950 WOQ kernels (woq_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "woq_layout.h"

namespace nad {

enum ActType : int { kActF32 = 0, kActF16 = 1, kActBF16 = 2 };

struct RepackArgs {
  // source blob (already on the device): interleaved [NPad/NTILE][KPad/PR][NTILE][PR] packed values
  const uint8_t* src_q;
  const void* src_s;
  const int8_t* src_z;
  int ntile, packrow, kpad, cstep;
  // destination geometry
  int bits, n, k, ns, nt, ng, scale_t;
  uint32_t* dst_tiles;
  void* dst_scales;
  int8_t* dst_zps;
};

struct SkinnyWeight {
  const void* tiles;
  const void* scales;
  const int8_t* zps;
  const int32_t* shuffle;
  int n, ns, nt, ng, bs;
  int ldo;
  float* out;
  const float* bias;  // bias[m * bias_ld + n] (bias_ld = 0 broadcasts one row)
  int bias_ld;
  int pad_;
};

struct SkinnyArgs {
  const void* A;
  int lda, M, K;
  int nw;               // weights in this launch (1..3); for dual epilogues w[0], w[1] pair up
  int stripe_base[4];   // prefix sums of ns over the weights (non-dual)
  int tiles_per_wave;
  int steps_per_group;  // blocksize / 32
  int scale_t;
  int epi;
  int vec_ok;           // A rows 16-B aligned (vector loads allowed)
  int a_fast;           // vec_ok && no act-order shuffle && K % (16 B / elem) == 0
  const float* res;
  int ld_res;
  float* aux;           // dual epilogue: optional silu/gelu(W0.a) output (tmp1 of the reference FFN)
  int ld_aux;
  SkinnyWeight w[3];
};

struct GemmArgs {
  const void* A;
  int lda, M, K;
  int scale_t;
  int epi;
  int vec_ok;
  const float* res;
  int ld_res;
  const float* aux;
  int ld_aux;
  SkinnyWeight w;
};

hipError_t launch_repack(const RepackArgs& a, hipStream_t stream);
hipError_t launch_skinny(const SkinnyArgs& a, int bits, int act_t, int waves_per_wg, int stripes, int ch,
                         hipStream_t stream);
hipError_t launch_gemm(const GemmArgs& a, int bits, int act_t, hipStream_t stream);

}  // namespace nad
