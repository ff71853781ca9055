// btla_format.h -- host-side model of Neural Speed's packed weight blob (NE_TYPE_BTLA tensor payload).
//
// The blob is StorageWeightKBlockNInteger (bestla/bestla/bestla_storage.h:697-834): a 48-byte header,
// then 64-B aligned buffers (quantized weights, scales, optional zero points / reduce / shuffle LUT).  This
// file reads and writes that format bit-exactly so blobs produced by the reference's quantizer load here and
// blobs produced here load in the reference.  The GPU never sees this layout: bestla_device_load_storage
// repacks it into the tile layout of woq_layout.h.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

namespace nad {

// BTLA_DTYPE (bestla/bestla/bestla.h:38-87)
enum : uint32_t {
  kF32 = 32,
  kF16 = 16,
  kBF16 = 16 | (1u << 16),
  kS8 = 8 | 0x100,
  kS4 = 4 | 0x100,
  kS2 = 2 | 0x100,
  kS3 = 3 | 0x100,
  kS5 = 5 | 0x100,
  kS6 = 6 | 0x100,
  kS7 = 7 | 0x100,
  kF4E2M1 = 4,                // EleBits4 | TypeFloat (bestla.h:82-84)
  kF4BNB = 4 | (1u << 16),
  kF4NF4 = 4 | (2u << 16),
  kF8E4M3 = 8,                // EleBits8 | TypeFloat (bestla.h:68-71)
  kF8E5M2 = 8 | (1u << 16),
  kF8E8M0 = 8 | (3u << 16),   // shared-exponent scale dtype (one int8 exponent per block)
  kDQ8_BNB = 8 | (4u << 16),
};
inline int dtype_bits(uint32_t t) { return int(t & 0xff); }
inline bool is_f8(uint32_t t) { return t == kF8E4M3 || t == kF8E5M2; }
// kernel_ref.h:984-1001 f8_to_fp32 (exponent field always read as normal) and :1721-1762 f8_mx_quantize
float f8_to_f32(uint32_t t, int8_t code);
int8_t f8_quantize(uint32_t t, float v, float scale, bool e8m0);
// NFloat 4-bit kind (0 F4_BNB, 1 F4_E2M1, 2 F4_NF4) or -1
inline int f4_kind(uint32_t t) { return t == kF4BNB ? 0 : (t == kF4E2M1 ? 1 : (t == kF4NF4 ? 2 : -1)); }
// bestla_utils.h:749-790 dequant LUTs (the values of kernel_ref.h's unpack trees)
float f4_lut(int kind, int code);
// kernel_ref.h f4_quantize (fp4_bnb_quantize :1233-1254, fp4_e2m1_quantize :1256-1297, nf4_quantize :1373-1419)
int8_t f4_quantize(int kind, float x);
// bits of the device tile layout that holds a blob's integers exactly: S2 -> 2, S3/S4 -> 4, S5..S8 -> 8
inline int device_bits(uint32_t t) {
  const int b = dtype_bits(t);
  return b <= 2 ? 2 : (b <= 4 ? 4 : 8);
}
inline bool dtype_is_int(uint32_t t) { return ((t >> 8) & 0xff) == 1; }

// ne_comp_type (neural_speed/core/data_types.h:57-63)
enum CompType : int { kCompUndef = 0, kCompF32 = 1, kCompBF16 = 2, kCompF16 = 3, kCompInt8 = 4 };

// GemmCore attributes encoded in mCoreId (bestla/bestla/bestla_gemm.h:83-128)
struct CoreInfo {
  int ntile, packrow, ktile;
  bool int_comp;  // B-side integer compute -> blob carries a BF16 reduce buffer
};
CoreInfo core_info(uint64_t core_id);
uint64_t core_id_by_name(const std::string& name);  // "avx512f", "amx_int8_kblock", ...

// Emulated host ISA for the pack path (BTLAGemmPackBSizeLocal picks the core from the packing host's ISA,
// neural_speed/core/layers/bestla_gemm.cpp:241-300).  Default SPR (the reference's published 8480L box);
// override with NAD_HOST_ISA=spr|avx512_vnni|avx512f|avx2.
int host_isa_profile();
uint64_t select_core(int comp_type, uint32_t qtype, int blocksize, bool asym, int profile);

struct Blob {
  // header (bestla_storage.h:250-357)
  uint64_t size = 0;
  uint32_t prologue = 1;  // BTLA_PROLOGUEB_IDS::WeightKBlockNInteger
  uint64_t core_id = 0;
  int npad = 0, kpad = 0, n = 0, k = 0;
  uint32_t qtype = kS4;
  int blocksize = 0, dq_blocksize = 0;
  // correction (bestla_storage.h:151-248)
  uint32_t scale_t = kF32, zp_t = kS8, red_t = kBF16;
  int cstep = 0;
  uint64_t csize = 0;
  bool asym = false, has_reduce = false, has_shuffle = false;
  // buffers: byte offsets from the blob base and sizes
  uint64_t q_off = 0, q_size = 0, s_off = 0, s_size = 0, z_off = 0, z_size = 0, r_off = 0, r_size = 0,
           shf_off = 0, shf_size = 0;
  // DQ8_BNB double-quantized scales (mDQCorrectionBuf, bestla_storage.h:158,223-231): u8 codes in the scale buffer,
  // then fp32 [updiv(ngroups * N, dq_blocksize)] block absmax + 1 offset (the mean of all scales) in this buffer
  bool has_dq = false;
  uint64_t dq_off = 0, dq_size = 0;

  int ngroups() const { return int((kpad + blocksize - 1) / blocksize); }      // rows of the scale buffer
  int ngroups_k() const { return int((k + blocksize - 1) / blocksize); }       // groups covering real K
  size_t scale_bytes() const { return scale_t == kF32 ? 4 : (scale_t == kF8E8M0 || scale_t == kDQ8_BNB ? 1 : 2); }
  // fp32 scale of (group g, column n) whatever the stored dtype (DQ8_BNB: dq8_get_fp_scale, kernel_ref.h:1981-1991)
  float scale_at(const int8_t* base, int g, int n) const;

  // describe a fresh blob (createStorage + resize, bestla_prologue_b.h:120-127, bestla_storage.h:725-753)
  static Blob describe(int n, int k, int blocksize, uint32_t qtype, uint32_t scale_t, bool asym, uint64_t core_id,
                       bool shuffle);
  // write header + buffer descriptors (assign(), bestla_storage.h:818-823); fills the *_off fields
  void write_header(int8_t* base);
  // parse (deserialize(), bestla_storage.h:831-836).  Returns false (and a message) on anything unsupported.
  bool parse(const void* buf, std::string* err);
};

// quantize_f32_sign_int_rowblock (bestla/bestla/kernel_ref.h:1608-1719), multithreaded over columns.
// src is [K][ld_src] (K rows, N columns), outputs q [K][N], scales/zp [ceil(K/bs)][N].
// F8 weights: quantize_f32_f8_rowblock_mxscale; with e8m0 the scales are the (float) shared exponents.
void quantize_kblock(const float* src, int K, int N, int ld_src, int blocksize, uint32_t qtype, int8_t* q, float* scales,
                     int8_t* zp, bool e8m0 = false);

// packQWeight (bestla_prologue_b.h:378-398) into a buffer whose header was written by Blob::write_header.
bool pack_quantized(Blob& b, int8_t* base, const int8_t* Q, int ldq, const float* S, const int8_t* Z,
                    const int* g_idx, std::string* err);

// exact unpack: Q [K][N] (signed), S [ngroups_k][N] float, Z [ngroups_k][N] (0 if sym), shuffle [K] (optional)
void unpack_quantized(const Blob& b, const int8_t* base, int8_t* Q, float* S, int8_t* Z, int* shuffle);
// BTLAGemmUnPackB semantics: W[k][n] = float(q - zp) * s  (kernel_ref.h:1027-1056)
void unpack_fp32(const Blob& b, const int8_t* base, float* W, int ldw);

// DQ8_BNB (bitsandbytes' signed 8-bit dynamic map, bestla_utils.h:794-820): code -> value
float dq8_lut(int code);
// dq8_bnb_double_quant<false> (kernel_ref.h:1952-1979): scale[0, n) -> codes (as floats, in place); dq gets
// updiv(n, dq_blocksize) + 1 floats (block absmax, then the offset).  dq must be zero-filled by the caller.
void dq8_double_quant(float* scale, size_t n, int dq_blocksize, float* dq);

// scale conversions used when storing scales in the blob's dtype
uint16_t f32_to_bf16_rne(float v);   // bestla_utils.h:146-153
uint16_t f32_to_f16_rne(float v);    // IEEE RNE (vcvtps2ph on AVX512-FP16 hosts)
float bf16_to_f32(uint16_t x);
float f16_to_f32(uint16_t x);

}  // namespace nad
