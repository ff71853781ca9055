/*
 * btla_oracle.h -- CPU restatement of the reference (hoivb612/neural, BesTLA) weight-only-quantization
 * algorithms on the WOQ matmul hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * Parity pinning: every integer/byte transform here is checked bit-for-bit against goldens produced by
 * oracle/_ref/ref_golden, a driver compiled from the reference's own bestla/bestla/kernel_ref.h +
 * bestla_utils.h (see oracle/ref/Makefile and tests/golden/make_golden.py).  The blob (de)serializer is
 * restated from bestla_storage.h text (not compilable here: it pulls xbyak) and pinned by the reference's
 * own round-trip rule (UT_StorageMemCheck, bestla/bestla/ut/bestla_prologue_b.cpp:290-331) plus the
 * field-by-field layout of bestla_storage.h:22-357,697-834.
 */
#ifndef NAD_BTLA_ORACLE_H
#define NAD_BTLA_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* BTLA_DTYPE values (bestla/bestla/bestla.h:38-87) */
#define ORC_F32 32u
#define ORC_F16 16u
#define ORC_BF16 (16u | (1u << 16))
#define ORC_S8 (8u | 0x100u)
#define ORC_S4 (4u | 0x100u)
#define ORC_S2 (2u | 0x100u)
#define ORC_F4_E2M1 (4u)                 /* EleBits4 | TypeFloat          (bestla.h:82) */
#define ORC_F4_BNB (4u | (1u << 16))     /* EleBits4 | TypeFloat | SubType1 */
#define ORC_F4_NF4 (4u | (2u << 16))     /* EleBits4 | TypeFloat | SubType2 */
#define ORC_F8_E4M3 (8u)                 /* EleBits8 | TypeFloat          (bestla.h:68-71) */
#define ORC_F8_E5M2 (8u | (1u << 16))
#define ORC_F8_E8M0 (8u | (3u << 16))    /* shared-exponent (mx) scale dtype */
#define ORC_DQ8_BNB (8u | (4u << 16))    /* double-quantized u8 scale codes (bestla.h:72) */

/* fp16/bf16 conversions (bestla/bestla/bestla_utils.h:116-229) */
uint16_t orc_f32_to_bf16(float v);
float orc_bf16_to_f32(uint16_t x);
uint16_t orc_f32_to_fp16_bestla(float v); /* utils::fp16::operator=(float), bestla_utils.h:184-196 */
uint16_t orc_f32_to_fp16_rne(float v);    /* IEEE RNE, = vcvtps2ph on AVX512-FP16/F16C hosts */
float orc_fp16_to_f32(uint16_t x);        /* bestla_utils.h:197-206 */

/* kernel_ref.h:1608-1719 quantize_f32_sign_int_rowblock (sNauto sym / asym paths) */
void orc_quantize_rowblock(const float* src, int8_t* dst, int row, int col, int ld_src, int ld_dst, float* scales,
                           int8_t* zero_points, int blocksize, int bits);

/* kernel_ref.h:39-59 padding_interleave / kernel_ref.h:62-80 revert_padding_interleave (int8) */
void orc_padding_interleave(const int8_t* src, int8_t* dst, int row, int col, int rowpad, int colpad, int src_step,
                            int dst_step, int ntile, int rowpack);
void orc_revert_padding_interleave(const int8_t* src, int8_t* dst, int row, int col, int rowpad, int colpad,
                                   int src_step, int dst_step, int ntile, int rowpack);

/* kernel_ref.h:155-165 compress_s8_s4, :330-341 compress_2bit, and the matching decompress_s4_s8/s2_s8 */
void orc_compress_s4(const int8_t* src, uint8_t* dst, size_t n);
void orc_compress_s2(const int8_t* src, uint8_t* dst, size_t n);
void orc_decompress_s4(const uint8_t* src, int8_t* dst, size_t n);
void orc_decompress_s2(const uint8_t* src, int8_t* dst, size_t n);

/* Core ids (bestla_gemm.h:83-93 CoreAttr::make_core_id; typedefs neural_speed/core/layers/bestla_defs.h:36-54) */
uint64_t orc_core_id(const char* name); /* "avx2","avx512f","amx_bf16","amx_fp16","avx512_vnni_kblock",
                                           "avx512bw_kblock","avx_vnni_kblock","avx2_vnni_kblock","amx_int8_kblock" */
int orc_core_ntile(uint64_t id);
int orc_core_packrow(uint64_t id);
int orc_core_ktile(uint64_t id);
int orc_core_is_int(uint64_t id);

/* ne_comp_type (neural_speed/core/data_types.h:57-63) -> core selection of BTLAGemmPackBSizeLocal
   (neural_speed/core/layers/bestla_gemm.cpp:241-300) for an emulated host ISA profile:
   profile 0 = Sapphire Rapids (AMX-INT8/BF16, AVX512-VNNI/BF16/FP16), 1 = AVX512-VNNI, 2 = AVX512F, 3 = AVX2 */
uint64_t orc_select_core(int comp_type, uint32_t qtype, int blocksize, int asym, int profile);

/* Packed blob (StorageWeightKBlockNInteger, bestla_storage.h:697-834) */
size_t orc_blob_size(int n, int k, int blocksize, uint32_t qtype, uint32_t stype, int asym, uint64_t core_id,
                     int shuffle);
/* full quantize + pack (BTLAGemmQuantPackB, bestla_gemm.cpp:321-398 -> WeightKBlockNInteger::packWeight) */
int orc_blob_quant_pack(void* buf, const float* B, int n, int k, int ldb, int blocksize, uint32_t qtype,
                        uint32_t stype, int asym, uint64_t core_id, int is_trans);
/* pre-quantized pack (BTLAGemmPackB, bestla_gemm.cpp:424-504 -> packQWeight + setShuffleIndices) */
int orc_blob_pack_q(void* buf, const int8_t* Q, const float* S, const int8_t* Z, int n, int k, int ldb, int blocksize,
                    uint32_t qtype, uint32_t stype, int asym, uint64_t core_id, const int* g_idx);
/* header fields: [mSize, prologue, coreid, NPad, KPad, N, K, dtype, blocksize, scaT, zpT, redT, cstep, csize,
                   asym, has_reduce, has_shuffle, q_off, q_size, s_off, s_size, z_off, z_size, r_off, r_size,
                   shf_off, shf_size]  (27 int64 values; *_off are byte offsets from the blob base) */
int orc_blob_info(const void* buf, int64_t* out27);
/* exact unpack to the integer domain: Q [K][N] signed int8, S [ceil(K/bs)][N] float, Z same shape int8 */
int orc_blob_unpack_q(const void* buf, int8_t* Q, float* S, int8_t* Z, int* shuffle);
/* BTLAGemmUnPackB (bestla_gemm.cpp:673-749): W[k][n] = float(q - zp) * s  (kernel_ref.h:1027-1056) */
int orc_blob_unpack_fp32(const void* buf, float* W, int ldb);
/* UT_ShuffleIndices LUT (bestla_prologue_b.h:337-356): out[g*bs + j] = j-th k with g_idx[k] == g */
void orc_shuffle_indices(const int* g_idx, int k, int blocksize, int* out);

/* GEMM oracles */
/* C[m][n] = sum_k A[m][k] * W[k][n], fp64 accumulation (the bar of bestla_prologue_b.cpp:510-511) */
void orc_gemm_f64(int m, int n, int k, const float* A, int lda, const float* W, int ldw, float* C, int ldc);
/* blob forward: applies the shuffle LUT to A (bestla_prologue_a.h:407-422) then unpack + orc_gemm_f64 */
int orc_blob_forward(const float* A, const void* blob, float* C, int m, int n, int k, int lda, int ldc);
/* kernel_ref.h:2489-2531 gemv_4bit_fp32_fp32 and :2712-2760 gemv_2bit_fp32_fp32 over a whole PACK_ROW=1 blob,
   float accumulation in the reference's order (MTILE = m <= 8) */
int orc_blob_gemv_ref(const float* A, const void* blob, float* C, int m, int lda, int ldc);
/* single-threaded CPU WOQ GEMV in the reference algorithm's float order, used as the timed cpu_baseline */
int orc_blob_gemv_par(const float* A, const void* blob, float* C, int m, int lda, int ldc, int threads);
int orc_blob_gemv_avx512(const float* A, const void* blob, float* C, int k_ld, int threads);
int orc_blob_gemv_timed(const float* A, const void* blob, float* C, int m, int lda, int ldc, int iters);


/* int8 compute (comp_int8): kernel_ref.h:1824-1883 quantize_fp_u8_colblock, the kblock u8s8 GEMM
   (bestla_wrapper.h:768-831 + bestla_gemm.h:2899-3050) over a blob with a reduce section, and kernel_ref.h:2371-2429
   gemv_4bit_u8s8_fp32 over unpacked operands */
void orc_quant_u8_colblock(int row, int col, const float* src, int ld_src, uint8_t* dst, int ld_dst, float* scales,
                           int ld_scale, uint8_t* zps, int blocksize, float* blkreduce);
int orc_blob_forward_int8(const float* A, const void* blob, float* C, int m, int n, int k, int lda, int ldc);
void orc_gemv_u8s8_ref(int m, int n, int k, int bs, const uint8_t* a8, const float* as, const uint8_t* azp,
                       const int8_t* q, const float* s, const int8_t* zp, float* C);


/* 3/5/6/7-bit plane (de)compression: kernel_ref.h:178-341 compress_Nbit, :412-520 decompress_sN_s8, plane offsets of
   bestla_prologue_b.h:512-546 */
int orc_compress_planes(int bits, const int8_t* src, uint8_t* dst, size_t n);
int orc_decompress_planes(int bits, const uint8_t* src, int8_t* dst, size_t n);

/* GGUF Q4_0 x Q8_0: data_types.h:79-83 blocks, data_types.h:204-228 fp32->fp16, vectors/cpu/quantize.h:243-276 / 422-445 /
   686-704, core/layers/vec_dot.h:187-204 (scalar path) */
uint16_t orc_ne_fp32_to_fp16(float f);
float orc_ne_fp16_to_fp32(uint16_t h);
void orc_q4_0_quantize_row(const float* x, uint8_t* y, int k);
void orc_q4_0_dequantize_row(const uint8_t* x, float* y, int k);
void orc_q8_0_quantize_row(const float* x, uint8_t* y, int k);
float orc_vec_dot_q4_0_q8_0(int n, const uint8_t* vx, const uint8_t* vy);
int orc_q4_0_forward(const float* A, const uint8_t* W, float* C, int m, int n, int k);


/* NFloat 4-bit weights: LUTs bestla_utils.h:749-790, quantizers kernel_ref.h:1233-1419, quantize_f32_f4_rowblock
   kernel_ref.h:1800-1822.  kind: 0 = F4_BNB, 1 = F4_E2M1, 2 = F4_NF4 */
int orc_f4_kind(uint32_t qtype);
float orc_f4_lut(int kind, int code);
int8_t orc_f4_quantize(int kind, float x);
void orc_quantize_f4_rowblock(const float* src, int8_t* dst, int row, int col, int ld_src, int ld_dst, float* scales,
                              int blocksize, int kind);


/* NFloat 8-bit weights: kernel_ref.h:1721-1762 f8_mx_quantize, :984-1001 f8_to_fp32, :1764-1800
   quantize_f32_f8_rowblock_mxscale (e8m0 != 0: F8_E8M0 scales, else F32) */
int8_t orc_f8_quantize(uint32_t t, float v, float scale, int e8m0);
float orc_f8_to_f32(uint32_t t, int8_t code);
/* DQ8_BNB double-quantized scales (kernel_ref.h:1930-1991, bestla_utils.h:794-820) */
void orc_dq8_lut(float* out256);
void orc_dq8_double_quant(float* scale, size_t n, int dq_bs, float* dq);
void orc_dq8_get_fp_scale(const uint8_t* src, float* dst, int row, int col, int dq_bs, int dq_offset_idx,
                          const float* dq, int src_stride, int dst_stride, int mN);
void orc_quantize_f8_rowblock(const float* src, int8_t* dst, int row, int col, int ld_src, int ld_dst, float* scales,
                              int blocksize, uint32_t t, int e8m0);

#ifdef __cplusplus
}
#endif
#endif
