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
  int src_bits;         // blob element bits: 2, 3, 4, 5, 6, 7, 8 (3/5/6/7 in bit planes, bestla_prologue_b.h:512-546)
  uint64_t nel;         // NPad * KPad: plane size of the multi-plane formats
  int raw;              // F8 weights: store the 8-bit code as it is (no + 128 bias)
  int src_e8m0;         // source scales are F8_E8M0 exponents (one byte each) -> fp32 2^e
  // destination geometry (bits: the device layout's 2 / 4 / 8 -- S3 lands in the int4 layout, S5-S7 in int8)
  int bits, n, k, ns, nt, ng, scale_t, kmajor;
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
  int kmajor;         // tile / scale order (woq_layout.h tile_index, scale_row)
  int ldo;
  float* out;
  const float* bias;  // bias[m * bias_ld + n] (bias_ld = 0 broadcasts one row)
  int bias_ld;
  int f4;             // NFloat weight: 0 = F4_BNB, 1 = F4_E2M1, 2 = F4_NF4 (int4 layout, LUT), 3 = F8_E4M3,
                      // 4 = F8_E5M2 (int8 layout, raw codes); -1 = integer weight
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
  int stagger;          // gemm3: waves 4-7 half a step behind waves 0-3 (NAD_GEMM3_STAGGER)
  int fold;             // gemm3 / gemm4: group scale folded into the fp16 B fragment (DeviceWeight::fold_ok)
  int ksw;              // gemm4 (folded): waves split over K, 1 (M) x 4 (N) x 2 (K) -- each B fragment dequantized once
  // split-K (gemm3 / gemm4 when the output tiles alone cannot fill the chip): the K tiles are cut into ksplit runs of
  // ktiles (a multiple of the tiles per group); run r of tile b writes its raw fp32 partial to
  // part[(r * M + row) * ldp + n] and launch_splitk_reduce sums the runs in order and applies the epilogue.
  int ksplit;           // 0 / 1: no split
  int ktiles;
  float* part;
  int ldp;
  // FFN prefill with fp16 intermediates: out16 set = the result goes to out16[row * ldo16 + n] as fp16 (RNE) instead of
  // w.out; aux16 set = the SiLU*mul operand is read as fp16 from aux16[row * ld_aux + n]
  _Float16* out16;
  int ldo16;
  const _Float16* aux16;
  int tpg_shift;        // mid-M kernel, one group per K tile or more: log2(K tiles per group) (31: one group)
  int xcd_sg;           // mid-M kernel + its reduce: > 0 = the stripe-group count; the runs of stripe group sg on XCD
                        // sg % 8 (whole rounds of 8 groups), and the reduce workgroups that sum them there too
  int xcd_w;            // ... the stripe group's width in float4 (S stripes x 4)
  // gemm7 without split K: nwt = 2 / 3 weights of one format and K in one launch (fused QKV prefill); the column tiles
  // of weight i follow those of weight i - 1 (nbn_cut: running tile-column counts, nbn_all their total); a.w is weight 0
  int nwt;
  int nbn_cut[2];
  int nbn_all;
  SkinnyWeight wf[2];
  int xcd_tile;         // gemm7 split-K: > 0 = its tile height; XCD x runs every K run of tiles [x T/8, (x+1) T/8) (T tiles,
                        // a multiple of 8), and the reduce workgroups of those tiles run there too
  SkinnyWeight w;
};

// One problem of a batched M = 1 launch (nad_batch_*: BTLAGemmBatchDriver's independent problems, bestla_gemm.cpp:508-624)
struct GemvBatchEnt {
  const void* act;
  const void* tiles;
  const void* scales;
  const int8_t* zps;
  float* out;
  const void* pad[3];  // 64 B per entry (one scalar-cache line)
};

// Persistent stripe-stream decode GEMV (woq_gemv.hip).  All weights of one launch share K, group size, scale type and
// symmetry; for the dual epilogues w[0] = gate, w[1] = up.
struct GemvArgs {
  const void* A;
  int lda, M, K;
  int act_t;            // ActType
  int dual;             // units are {w[0] stripe s, w[1] stripe s} pairs (SiLU*mul / GELU*mul)
  int units;            // stripes (non-dual, summed over the weights) or stripe pairs (dual)
  int stripe_base[4];   // non-dual: first virtual stripe of each weight (unused entries = INT_MAX)
  int nt, ng, bs;       // tiles along K, groups along K, group size
  int tpg_mask;         // GPT == 1: tiles per group - 1 (power of two; 0x7fffffff for one group), group = t >> shift
  int tpg_shift;
  int scale_t;
  int asym;
  int epi;
  int a_fast;           // 16-B aligned rows, K % 8 == 0, no act-order shuffle: vector staging
  const int32_t* shuffle;
  const float* res;
  int ld_res;
  float* aux;
  int ld_aux;
  int part_off;         // LDS byte offset of the partial-sum slots
  uint32_t dq_mask;     // 0x000F000F and 0x64006400: int4 dequant constants, passed in so they stay in registers
  uint32_t dq_magic;
  int nwa;              // woq_chain: waves that own K slices in this op (the single-op launch's wave count)
  int norm;             // woq_chain: RMS-normalise each activation row while staging (x / rms(x) * norm_w)
  float norm_eps;
  const float* norm_w;  //   optional per-k weight (null = 1)
  int u_q, u_r;         // units per workgroup: u_q, one more for the first u_r workgroups (host-divided)
  int lean;             // M = 1 int4 single-group-per-tile launches may take woq_gemv_m1_kernel (NAD_GEMV_LEAN)
  int lean_ks;          // woq_gemv_m1_kernel: K tiles per K-slice (4, or 1 / 2 where that gives each of up to 16 waves one)
  int lean_spw;         // woq_gemv_m1_kernel: K-slices per wave at most (2; 4 for long K; 1 for narrow slices)
  SkinnyWeight w[3];
  const GemvBatchEnt* batch;  // batched M = 1 launch (woq_gemv_m1_kernel<..., BATCH>): problem p = blockIdx / batch_wpp
  int batch_wpp;              //   reads its activations / weight / output from batch[p]; u_q / u_r split one problem
  int m1_nst;                 // woq_gemv_m1_kernel: register stages in flight per wave (0 = by the stages per wave)
};

hipError_t launch_repack(const RepackArgs& a, hipStream_t stream);
hipError_t launch_skinny(const SkinnyArgs& a, int bits, int act_t, int waves_per_wg, int stripes, int ch,
                         hipStream_t stream);
hipError_t launch_gemm(const GemmArgs& a, int bits, int act_t, hipStream_t stream);
// prefill GEMM v2 (woq_gemm2.hip): int4, group = 128 * 2^j, stripe-major; A as fp16 [M][lda16] with K padded to the
// 128-deep tile (zeros), e.g. from launch_cvt_act
hipError_t launch_gemm2(const GemmArgs& a, const _Float16* A16, int lda16, hipStream_t stream);
// prefill GEMM v3 (woq_gemm2.hip): same contract as launch_gemm2; every operand staged by LDS-DMA three 64-deep half
// steps ahead with counted vmcnt (no drain at the barriers)
hipError_t launch_gemm3(const GemmArgs& a, const _Float16* A16, int lda16, hipStream_t stream);
// prefill GEMM v4 (woq_gemm4.hip): gemm3's pipeline for int4 groups of 32 / 64 and int2 groups >= 64.
// gemm4_mode: 0 = not taken, else the group mode; A as for gemm3 with K padded to the weight's K tile (128 / 256)
int gemm4_mode(int bits, int blocksize, int ng, int kpad, bool asym);

// int8-compute mode (woq_i8.hip).  Activation quantizer: one thread per (row, block); any output may be null.
struct QuantU8Args {
  const void* A;
  int lda, M, K, bs, ng;
  const int32_t* shuffle;
  int8_t* aq;           // [M][ldq] s8 = u8 - 128, zero in [K, kp)
  int ldq, kp;
  float2* sa;           // [M][ng] {scale, float(zp) * scale}
  uint8_t* q_u8;        // [M][ldu] the reference's u8 codes
  int ldu;
  float* s_out;         // [M][ld_scale]
  uint8_t* z_out;
  float* red_out;       // sum(q - zp... as kernel_ref: sum of round(x / s)) * s
  int ld_scale;
};
struct I8Args {
  const int8_t* aq;
  int ldq;
  int a_signed;         // 1: Q8_0 activations (s8, sa = {d, 0}; C += float(s32) * d_w * d_a); 0: u8 kblock mode
  const float2* sa;     // [M][ng]
  int M, K;
  const uint16_t* red;  // bf16 reduce [ng][red_ld]
  int red_ld;
  int scale_t;
  int epi;
  const float* res;
  int ld_res;
  const float* aux;
  int ld_aux;
  SkinnyWeight w;
};
// GGUF Q4_0 weights / Q8_0 activations (woq_gguf.hip)
struct Q80Args {
  const void* A;
  int lda, M, K;        // K % 32 == 0
  int8_t* aq;           // [M][ldq] s8 codes, zero in [K, kp)
  int ldq, kp;
  float2* sa;           // [M][K/32] {float(fp16 d), 0}
  int8_t* blocks;       // optional raw block_q8_0 rows [M][K/32][34]
};
hipError_t launch_q4_0_repack(const uint8_t* src, int n, int k, const DeviceWeight& w, hipStream_t stream);
hipError_t launch_q8_0_quant(const Q80Args& a, int act_t, hipStream_t stream);
hipError_t launch_quant_u8(const QuantU8Args& a, int act_t, hipStream_t stream);
hipError_t launch_i8(const I8Args& a, int bits, hipStream_t stream);
hipError_t launch_gemm4(const GemmArgs& a, int bits, const _Float16* A16, int lda16, hipStream_t stream);
// prefill GEMM v7 (woq_gemm7.hip, the default for int4 groups of 128 * 2^j): gemm3's contract (256 x 128 tiles,
// split-K partials, fp16 A padded to the 128-deep tile) with the group scale folded (needs DeviceWeight::fold_ok)
bool gemm7_ok(int bits, int blocksize, int fold_ok);
hipError_t launch_gemm7(const GemmArgs& a, int bits, int bm, const _Float16* A16, int lda16, hipStream_t stream);
// mid-M GEMM (woq_gemm_mid.hip, 17 <= M <= 64): int4 / int2, gpt groups per K tile (1, 2, 4), rf = ceil(M / 16) row
// fragments; grid = ceil(ns / S) * a.ksplit for the S of mid_geometry; a.ksplit > 1: launch_splitk_reduce follows
void mid_geometry(int bits, int gpt, int act_t, int rf, int wide, int* s, int* nw, int* spw);
int mid_lds_bytes(int rf, int s, int nw);
hipError_t launch_gemm_mid(const GemmArgs& a, int bits, int gpt, int act_t, int rf, int s, int grid, hipStream_t stream);
// sum a.ksplit partials of a split-K gemm3 / gemm4 launch in run order and apply a.epi into a.w.out (woq_gemm2.hip)
hipError_t launch_splitk_reduce(const GemmArgs& a, hipStream_t stream);
hipError_t launch_cvt_act(const void* A, int act_t, int lda, int M, int K, int Kp, const int32_t* shuffle,
                          _Float16* out, hipStream_t stream);
// groups per K tile the GEMV handles (1, 2, 4, 8) for this geometry, 0 if unsupported; *tpg = tiles per group
int gemv_groups_per_tile(int bits, int nt, int ng, int bs, int* tpg);
size_t gemv_lds_layout(GemvArgs& a, int bits, int waves, int grid);
int gemv_waves(int bits, int nt, int ng, int bs);
// M = 1: K-slices of 2 tiles for woq_gemv_m1_kernel when that gives more waves (one slice each); sets a.lean_ks and
// *waves when taken (ks_pref = NAD_GEMV_KS: 2 = 1- or 2-tile slices wherever that gives more waves, 3 = 2-tile only,
// 4 = never)
void gemv_lean_slices(GemvArgs& a, int bits, int* waves, int ks_pref);
hipError_t launch_gemv(const GemvArgs& a, int bits, int waves, int grid, size_t lds, hipStream_t stream);
// whether launch_gemv would take woq_gemv_m1_kernel for these arguments
bool gemv_uses_m1(const GemvArgs& a, int bits, int waves);
// two M = 1 launches of different formats as one (int2 a + int4 b at groups of 64 or 128, fp32 activations, sym,
// 16 waves each; a on workgroups [0, ga), b on [ga, ga + gb))
bool gemv_dual_ok(const GemvArgs& a, int bits_a, const GemvArgs& b, int bits_b, int waves);
hipError_t launch_gemv_dual(const GemvArgs& a, const GemvArgs& b, int ga, int gb, int waves, size_t lds,
                            hipStream_t stream);
// the batched M = 1 launch (requires gemv_uses_m1; grid = problems * a.batch_wpp)
hipError_t launch_gemv_batch(const GemvArgs& a, int bits, int waves, int grid, size_t lds, hipStream_t stream);

}  // namespace nad
