/*
 * neural_amd.h -- C ABI of the MI355X-native weight-only-quantized (WOQ) matmul core.
 *
 * Drop-in for the BesTLA boundary of Neural Speed (hoivb612/neural).  Every entry point below keeps the name,
 * argument meaning and error behaviour of the reference interface it replaces (cited per group; paths relative to
 * the reference repo root).  Plain C types only: no torch, no HIP types (a HIP stream is passed as void* "queue").
 *
 * Build: `make -C neural_amd` -> neural_amd/libneural_amd.so (gfx950).  Link it in place of
 * neural_speed/core/layers/ne_bestla.cpp + ne_bestla_sycl.cpp + bestla_gemm.cpp.
 *
 * Errors: bool/int functions return false/nonzero; void functions (whose reference counterparts assert(0) or are
 * silently skipped, e.g. bestla_gemm.cpp:542-590) print "neural_amd: <reason>" to stderr and record it; read it with
 * nad_last_error().  Nothing is silently skipped.
 */
#ifndef NEURAL_AMD_H
#define NEURAL_AMD_H
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ===== device half: neural_speed/core/ne_bestla.h:85-112 (implemented for SYCL in
 * neural_speed/core/layers/ne_bestla_sycl.cpp:25-171).  queue == hipStream_t; device == NadDevice*. */
void* bestla_create_device(bool profile);               /* ne_bestla.h:86 */
void* bestla_get_device_queue(void* device);            /* ne_bestla.h:87 */
void bestla_release_device(void* device);               /* ne_bestla.h:88 */
size_t bestla_device_gmem_size(void* device);           /* ne_bestla.h:89 */
void* bestla_device_malloc(size_t size, void* queue);   /* ne_bestla.h:90 */
void bestla_device_free(void* ptr, void* queue);        /* ne_bestla.h:91 */
void bestla_device_memcpy(void* dstptr, const void* srcptr, size_t size, void* queue);      /* ne_bestla.h:92 */
void bestla_device_memcpy_sync(void* dstptr, const void* srcptr, size_t size, void* queue); /* ne_bestla.h:93 */
void bestla_device_sync(void* queue);                   /* ne_bestla.h:94 */
/* size of the per-tensor device descriptor embedded after ne_tensor (ne_layers.c:946-949) */
size_t bestla_device_storage_size(void);                /* ne_bestla.h:95 */
/* parse a host BTLA blob, repack it on the GPU into the MFMA tile layout inside `deviceptr` (which the caller sized
 * with the blob's byte size, model_files.h:1515-1525) and fill the host descriptor `devstor`. */
void bestla_device_load_storage(void* hoststor, void* devstor, void* deviceptr, void* queue); /* ne_bestla.h:96 */
/* Y[m][n] = X[m][k] . W^T, X/Y fp32 device pointers (row strides lda/ldo in elements), asynchronous on queue */
void bestla_device_f32f32_forward(float* activation, void* weiptr, float* output, int _m, int _n, int _k, int lda,
                                  int ldo, void* workspace, void* queue); /* ne_bestla.h:97-98 */

/* ===== host half: neural_speed/core/ne_bestla.h:21-83 (CPU implementation: core/layers/inner_product.cpp,
 * ip_fusion_qkv.cpp, ip_fusion_ffn.cpp, ne_bestla.cpp).  Same host-pointer contract; the work runs on the GPU
 * (weights uploaded once per blob and cached, activations/outputs staged over PCIe).  Pointers that are already
 * device memory are used in place. */
void bestla_init(void);                                 /* ne_bestla.h:31 */
int bestla_set_threads(int _nth);                       /* ne_bestla.h:23: host packing threads */
void* bestla_get_thread_handle(void);                   /* ne_bestla.h:25 */
unsigned long long bestla_f32f32_get_workspace_size(int _m, int _n, int _k, void* wptr); /* ne_bestla.h:33 */
void bestla_f32f32_forward(float* activation, void* weiptr, float* output, int _m, int _n, int _k, int lda, int ldo,
                           void* workspace);            /* ne_bestla.h:35-36 */
bool bestla_fusion_add_f32f32_support(void* weiptr, int _m, int _n, int _k); /* ne_bestla.h:38 */
void bestla_fusion_add_f32f32_forward(float* activation, void* weiptr, float* bias, float* output, int _m, int _n,
                                      int _k, int lda, int ldo, bool boardcast_bias, void* workspace); /* :39-40 */
unsigned long long bestla_fusion_QKV_f32f32_get_workspace_size(int _m, int _n, int _k, void* w1ptr); /* :42 */
bool bestla_fusion_QKV_f32f32_support(void* wqptr, void* wkptr, void* wvptr, int _m, int _n, int _k); /* :44 */
void bestla_fusion_QKV_f32f32_forward(float* activation, void* wqptr, void* wkptr, void* wvptr, float* output, int _m,
                                      int _n, int _k, int lda, int ldo, void* workspace); /* :46-47 */
unsigned long long bestla_fusion_FFN_f32f32_get_workspace_size(int seq, int fin, int fmid, int fout, void* w1ptr,
                                                               void* w2ptr); /* :49-50 */
bool bestla_fusion_FFN_SiLu_f32f32_support(void* w1ptr, void* w2ptr, void* w3ptr, int seq, int fin, int fmid,
                                           int fout); /* :57 */
void bestla_fusion_FFN_SiLu_f32f32_forward(float* activation, void* w1ptr, void* w2ptr, void* w3ptr, float* tmp1,
                                           float* tmp2, float* output, int seq, int fin, int fmid, int fout,
                                           void* workspace); /* :58-60 */
bool bestla_fusion_FFN_Gelu_Mul_f32f32_support(void* w1ptr, void* w2ptr, void* w3ptr, int seq, int fin, int fmid,
                                               int fout); /* :52-53 */
void bestla_fusion_FFN_Gelu_Mul_f32f32_forward(float* activation, void* w1ptr, void* w2ptr, void* w3ptr, float* tmp1,
                                               float* tmp2, float* output, int seq, int fin, int fmid, int fout,
                                               void* workspace); /* :54-56 */
bool bestla_fusion_FFN_GeLu_f32f32_support(void* w1ptr, void* w2ptr, int seq, int fin, int fmid, int fout); /* :62 */
void bestla_fusion_FFN_GeLu_f32f32_forward(float* activation, void* w1ptr, void* w2ptr, float* tmp1, float* output,
                                           int seq, int fin, int fmid, int fout, void* workspace); /* :63-64 */
bool bestla_fusion_FFN_Add_GeLu_f32f32_support(void* w1ptr, void* w2ptr, int seq, int fin, int fmid,
                                               int fout); /* :66 */
void bestla_fusion_FFN_Add_GeLu_f32f32_forward(float* activation, void* w1ptr, void* w2ptr, float* b1ptr,
                                               float* b2ptr, float* tmp1, float* output, int seq, int fin, int fmid,
                                               int fout, bool boardcast_bias, void* workspace); /* :67-69 */
void bestla_unpackweight_fp32(void* wptr, int n, int k, float* fp32data, int ld); /* ne_bestla.h:71 */
void bestla_packweight_copyattr(const float* f32ptr, void* dstpr, int n, int k, int ld, void* srcptr); /* :73 */

/* ===== pack / format API: neural_speed/core/layers/bestla_gemm.h:30-58 (C++ linkage in the reference; C here).
 * QuantType/ScaleDtype are BTLA_DTYPE values (bestla/bestla/bestla.h:38-87), CompType is ne_comp_type
 * (core/data_types.h:57-63).  The core layout is chosen for an emulated host ISA (NAD_HOST_ISA, default
 * Sapphire Rapids) exactly as BTLAGemmPackBSizeLocal does (bestla_gemm.cpp:241-300). ThreadPool may be NULL. */
typedef struct BTLA_GEMM_DATA_PACKED_PARAMS {
  const float* A; /* address of A (float32 matrix) */
  const void* B;  /* address of B (packed nbits blob) */
  float* C;       /* address of result matrix */
  int lda;        /* leading dimension of A */
  int ldc;        /* leading dimension of C */
} BTLA_GEMM_DATA_PACKED_PARAMS;     /* bestla_gemm.h:30-36 */
size_t BTLAGemmPackBSize(size_t N, size_t K, size_t BlkSize, uint32_t QuantType, uint32_t ScaleDtype, bool isAsym,
                         int CompType, int* shuffle_indice); /* bestla_gemm.h:38-39 */
bool BTLAGemmQuantPackB(void* PackedBuf, const float* FpData, size_t N, size_t K, size_t ldb, size_t BlkSize,
                        uint32_t QuantType, uint32_t ScaleDtype, bool isAsym, int CompType, bool isTrans,
                        void* ThreadPool); /* bestla_gemm.h:41-43 */
bool BTLAGemmPackB(void* PackedBuf, const int8_t* QData, const float* Scales, const int8_t* Zp, size_t N, size_t K,
                   size_t ldb, size_t BlkSize, uint32_t QuantType, uint32_t ScaleDtype, bool isAsym, int CompType,
                   int* shuffle_indice, void* ThreadPool); /* bestla_gemm.h:48-50 */
bool BTLAGemmUnPackB(float* FpData, const void* PackedBuf, size_t N, size_t K, size_t ldb,
                     void* ThreadPool); /* bestla_gemm.h:52 */
bool BTLAGemmBatchDriver(const size_t M, const size_t N, const size_t K, const size_t BatchN,
                         const BTLA_GEMM_DATA_PACKED_PARAMS* DataParams, int8_t* WorkSpace,
                         void* ThreadPool); /* bestla_gemm.h:54-55 */

/* ===== tensor-parallel communicator: neural_speed/core/parallel_context.h:21-48 (oneCCL/MPI + SHM in the reference,
 * parallel_context.cpp:19-159, shared_memory_ccl.hpp:100-139).  Implemented in csrc/parallel_context.hip: TCP
 * rendezvous from RANK/WORLD_SIZE (or OMPI_/PMI_ env), RCCL on a context stream for device buffers, a one-shot IPC
 * peer-buffer all-reduce for small device messages, host buffers staged through the device (or carried over the
 * rendezvous sockets when no GPU is present).  `count` is an element count (the reference passes byte counts at
 * ne_layers.c:5474 -- callers of this library pass elements). */
typedef struct parallel_context parallel_context;
parallel_context* init_parallel_context(void);   /* parallel_context.h:40 (process-wide singleton) */
int get_tp_size(parallel_context* p);             /* :41 */
int get_tp_rank(parallel_context* p);             /* :42 */
bool is_master(parallel_context* p);              /* :43 */
void barrier(parallel_context* p);                /* :44 (also drains this rank's device work) */
void broadcast(parallel_context* p, float* buffer, size_t count);                           /* :45, root 0 */
void alltoall(parallel_context* p, float* send_buffer, float* recv_buffer, size_t count);   /* :46, count per rank */
void reduce_add(parallel_context* p, float* send_buffer, float* recv_buffer, size_t count); /* :47, sum */
/* native: sum all-reduce of device buffers on `stream` (a hipStream_t; NULL = the null stream, as everywhere in this
 * library), asynchronous, graph-capturable */
int nad_pc_allreduce_f32(parallel_context* p, const float* send, float* recv, size_t count, void* stream);
int nad_pc_set_stream(parallel_context* p, void* stream);   /* stream of the reference entry points (default NULL) */
double nad_pc_max_f64(parallel_context* p, double v);        /* max over ranks (host value; bench timing) */
int nad_pc_status(parallel_context* p);   /* 0 ok, 1 a one-shot all-reduce gave up waiting for a peer */
int nad_pc_info(parallel_context* p);     /* bit0 GPU transport, bit1 one-shot IPC path, bit2 RCCL communicator,
                                             bit3 one-shot buffer is uncached fine-grained memory (else hipMalloc) */
const char* nad_pc_last_error(parallel_context* p);
void nad_pc_destroy(parallel_context* p);

/* ===== native extensions (no reference counterpart) */
#define NAD_ACT_F32 0
#define NAD_ACT_F16 1
#define NAD_ACT_BF16 2
/* device scale codes (nad_synthetic_weight, nad_plan_forward, nad_weight_info[8]) */
#define NAD_SCALE_F32 0
#define NAD_SCALE_BF16 1
#define NAD_SCALE_F16 2
#define NAD_EPI_NONE 0
#define NAD_EPI_BIAS 1
#define NAD_EPI_SILU_MUL 2
#define NAD_EPI_GELU_MUL 3
#define NAD_EPI_GELU 4
#define NAD_EPI_ADD_GELU 5
#define NAD_EPI_SILU 6
#define NAD_EPI_RES_ADD 7

const char* nad_last_error(void);
void nad_clear_error(void);
/* device bytes the tile layout of this blob needs (<= the blob size for every Llama/Mistral shape) */
size_t nad_device_weight_size(const void* hostblob);
/* bestla_device_load_storage with an explicit capacity check and a status return */
int nad_device_load(const void* hostblob, void* devstor, void* deviceptr, size_t capacity, void* queue);
/* descriptor summary: [magic, bits, n, k, blocksize, ns, nt, ng, scale_t, asym, has_shuffle, bytes] */
int nad_weight_info(const void* devstor, int64_t* out12);
/* the same, versioned by the caller's buffer: writes min(n, 13) values ([12] = fold_ok: every q * scale is an fp16
 * normal, the prefill GEMM may fold the scale into the fp16 weights), returns the number written or -1 */
int nad_weight_info2(const void* devstor, int64_t* out, int n);
/* re-read the NAD_* tuning / A-B switches from the environment (they are read once when the library loads, never per
 * call); not thread-safe against forwards running at the same time */
void nad_reload_knobs(void);
/* blob header summary (same fields as the oracle's orc_blob_info) */
int nad_blob_info(const void* hostblob, int64_t* out27);
/* Y = epi(X . W^T): X in fp32/fp16/bf16 (act_dtype), Y fp32.  bias: bias[m*bias_ld + n] (bias_ld 0 = broadcast);
 * res: residual[m*ld_res + n] for NAD_EPI_RES_ADD. */
int nad_device_forward(const void* act, int act_dtype, const void* devstor, float* out, int m, int n, int k, int lda,
                       int ldo, int epi, const float* bias, int bias_ld, const float* res, int ld_res, void* queue);
/* Dry run of nad_device_forward for a weight geometry (bits 2 / 4 / 8, blocksize <= 0 = per-channel, scale_t
 * NAD_SCALE_*, m rows of act_dtype): the whole host side of the call -- validation, kernel choice, geometry,
 * workspace sizing -- with every launch recorded instead of issued; no device memory is touched and no GPU is needed.
 * out (versioned by nout): [kernel NAD_KERNEL_*, grid, threads per workgroup, split-K runs, flags (bit 0: scale folded
 * into the fp16 weights; bit 1: gemm4 waves split over K), launches including pre-passes].  Returns the number of values
 * written or -1. */
#define NAD_KERNEL_GEMV_M1 1   /* woq_gemv_m1_kernel: M = 1 decode */
#define NAD_KERNEL_GEMV 2      /* woq_gemv_kernel: the stripe-stream GEMV, M <= 16 */
#define NAD_KERNEL_SKINNY 3    /* woq_skinny_kernel: decode geometries the stream does not take */
#define NAD_KERNEL_I8 4        /* woq_i8_kernel: int8-compute mode */
#define NAD_KERNEL_GEMM3 5     /* woq_gemm3_kernel: prefill, int4 groups of 128 * 2^j */
#define NAD_KERNEL_GEMM4 6     /* woq_gemm4_kernel: prefill, int4 g32 / g64, int2, int8 */
#define NAD_KERNEL_GEMM2 7     /* woq_gemm2_kernel (NAD_GEMM_KERNEL=2) */
#define NAD_KERNEL_GEMM 8      /* woq_gemm_kernel: register-staged prefill fallback */
#define NAD_KERNEL_GEMM7 9     /* woq_gemm7_kernel: prefill, int4 groups of 128 * 2^j, scale folded (default) */
#define NAD_KERNEL_MID 10      /* woq_mid_kernel: 12 (fp16) / 8 (fp32, bf16) <= M <= 64, int4 / int2 */
int nad_plan_forward(int bits, int n, int k, int blocksize, int scale_t, int asym, int m, int act_dtype, int64_t* out,
                     int nout);
/* the same dry run for a loaded device weight (its format, act-order, fold range and compute mode included) */
int nad_plan_weight(const void* devstor, int m, int act_dtype, int64_t* out, int nout);
/* fused Q/K/V (ip_fusion_qkv.cpp:22-93): out_i = X . W_i^T, one launch; W_i share K, blocksize, bits, scale dtype */
int nad_device_qkv_forward(const void* act, int act_dtype, const void* wq, const void* wk, const void* wv, float* oq,
                           float* ok, float* ov, int m, int k, int lda, int ldo_q, int ldo_k, int ldo_v, void* queue);
/* gate/up half of the fused FFN (ip_fusion_ffn.cpp:407-433): tmp2 = act(X.W1^T) * (X.W3^T), tmp1 = act(X.W1^T)
 * (optional for m <= 16).  epi: NAD_EPI_SILU_MUL / NAD_EPI_GELU_MUL. */
int nad_device_ffn_gate_up(const void* act, int act_dtype, const void* w1, const void* w3, float* tmp1, float* tmp2,
                           int m, int fin, int fmid, int lda, int epi, void* queue);
/* fused FFN (ip_fusion_ffn.cpp:407-457): tmp1 = act1(X.W1^T) [optional], tmp2 = tmp1 * (X.W3^T), out = tmp2 . W2^T.
 * epi = NAD_EPI_SILU_MUL or NAD_EPI_GELU_MUL.  tmp1 / tmp2 are scratch: for M > 16 with the pipelined GEMMs they hold
 * the intermediates as fp16 (the down GEMM reads tmp2 as its fp16 operand; NAD_FFN_F32=1 keeps fp32).  The
 * reference-named bestla_fusion_FFN_* entries always return the fp32 intermediates in tmp1 / tmp2. */
int nad_device_ffn_forward(const void* act, int act_dtype, const void* w1, const void* w2, const void* w3, float* tmp1,
                           float* tmp2, float* out, int m, int fin, int fmid, int fout, int lda, int epi, void* queue);
/* tensor-parallel slicing of a packed blob without re-quantization (the reference re-quantizes,
 * model_files.h:1538-1563).  axis 0: split N (TP_1D_ROW, column-parallel) into near-equal chunks of `unit` columns
 * (use the consumer's K group / head size so column shards line up with the next row-parallel weight's K shards);
 * axis 1: split K by whole quantization groups (TP_1D_COLUMN, row-parallel; `unit` ignored).
 * Returns the shard's blob size (dst may be NULL to query). */
size_t nad_blob_split(const void* src, int axis, int rank, int world, int unit, void* dst, size_t dst_capacity);
/* the [begin, end) range of N (axis 0) or K (axis 1) that `rank` owns */
int nad_split_range(const void* src, int axis, int rank, int world, int unit, int* begin, int* end);
/* synthetic device weight of the given geometry (random packed values, scales U[smin,smax], zps) for benchmarks */
int nad_synthetic_weight(void* devstor, void* deviceptr, size_t capacity, int bits, int n, int k, int blocksize,
                         int scale_t, int asym, uint64_t seed, void* queue);
/* device bytes of nad_synthetic_weight's layout */
size_t nad_synthetic_weight_size(int bits, int n, int k, int blocksize, int scale_t, int asym);
/* The host-pointer ABI (bestla_f32f32_forward & co., inner_product.cpp:28-36 called per node at ne_layers.c:7313)
 * keeps one device copy per blob address.  Per call the key check is O(1): the 64-byte header, the blob size and 64
 * dwords sampled at fixed positions; every pack entry of this library (BTLAGemmQuantPackB, BTLAGemmPackB,
 * bestla_packweight_copyattr, nad_blob_split) drops the copy of the buffer it writes, so a rewrite through the pack
 * API is always seen.  The cache is bounded (least recently used first out) by NAD_HOST_CACHE_MB, default 64 GiB. */
void nad_host_cache_clear(void);
/* drop the device copy of one blob.  MUST be called before a blob is freed, or rewritten in place by anything other
 * than this library's pack entries: the per-call key samples the blob, so a partial rewrite (a few groups
 * re-quantized) is not guaranteed to change it, and the forward would use the stale device copy. */
void nad_host_cache_evict(const void* blob);
/* cap on the cached device bytes (0 = the default); returns the previous cap */
size_t nad_host_cache_set_limit(size_t bytes);
/* entries and device bytes currently cached */
int nad_host_cache_stats(size_t* entries, size_t* bytes);
/* the per-call key of a host blob (what the cache compares on every forward); 0 if the blob does not parse */
unsigned long long nad_host_blob_key(const void* blob);
/* ===== int8-compute mode: the reference's comp_int8 arithmetic for weights packed for an integer core (blobs that
 * carry the bf16 reduce).  0 (default): fp16 MFMA on the exact weights.  1: activations quantized to u8 per (row,
 * weight block) as kernel_ref.h:1824-1883, s32 block dot products, the kblock core's fp32 combine
 * (bestla_wrapper.h:768-831, bestla_gemm.h:2983-3050).  Initial value from NAD_COMPUTE_INT8.  Weights without a
 * reduce keep the fp path; a fused call mixing the two kinds fails. */
int nad_set_compute_mode(int mode);
int nad_get_compute_mode(void);
/* per-thread override of the process mode (-1 clears it); thread-safe, takes precedence over nad_set_compute_mode */
int nad_set_thread_compute_mode(int mode);
/* per-weight arithmetic, as the reference selects it per blob core (bestla_gemm.cpp:516-616): -1 follow the
 * thread / process mode, 0 fp, 1 int8 (integer-core blobs and GGUF Q4_0; other weights stay fp).  Takes precedence
 * over both; a fused call whose weights resolve to different arithmetic runs each weight in its own. */
int nad_device_set_compute(void* devstor, int mode);
/* the arithmetic a forward of this weight takes now: 0 fp, 1 int8, -1 not a device weight */
int nad_device_get_compute(const void* devstor);
/* kernel::wrapper::QuantizeU8ColBlock::forward (kernel_wrapper.h:571-590) on device pointers: act [m][lda] in
 * act_dtype, q [m][ldq] u8, scales / zps [m][ld_scale] per block, blkreduce (may be NULL) = sum(round(x/s)) * s. */
int nad_quant_u8_colblock(const void* act, int act_dtype, int m, int k, int lda, int blocksize, uint8_t* q, int ldq,
                          float* scales, uint8_t* zps, int ld_scale, float* blkreduce, void* queue);
/* ===== GGUF Q4_0 (neural_speed/core/data_types.h:79-83): a Q4_0 matrix of N rows x K (K % 32 == 0), rows of K/32
 * blocks {fp16 d; u8 qs[16]} as an ne_tensor of type NE_TYPE_Q4_0 holds them, loaded into the same device layout as a
 * BTLA blob (symmetric int4, group 32, fp16 scales); every nad_device_* / bestla_device_* forward then accepts the
 * descriptor.  Compute mode 1 reproduces the reference's Q8_0 x Q4_0 arithmetic (quantize_row_q8_0_reference,
 * ne_vec_dot_q4_0_q8_0). */
size_t nad_q4_0_device_size(int n, int k);
int nad_q4_0_device_load(const void* blocks, int n, int k, void* devstor, void* deviceptr, size_t capacity, void* queue);
/* quantize_row_q8_0 (vectors/cpu/quantize.h:422-445) on device pointers: act [m][lda] -> m rows of K/32 block_q8_0 */
int nad_quant_q8_0(const void* act, int act_dtype, int m, int k, int lda, void* blocks, void* queue);
/* host convenience: (re)pack one blob into fp32 dequantized [K][N] from the device tile layout (round-trip check) */
int nad_device_unpack_fp32(const void* devstor, float* host_out, void* queue);

/* ===== batched independent decode problems: BTLAGemmBatchDriver (bestla_gemm.cpp:508-624) for device tensors.  n
 * problems y_i = x_i W_i (M = 1, fp32 x_i [K] 16-B aligned, fp32 y_i [N]) whose weights share N, K and format (int4 /
 * int2, no act-order, fp arithmetic, a geometry the M = 1 GEMV takes) run as ONE launch: workgroups are dealt out
 * problem by problem, each streaming its problem's share of the stripes.  The pointers are bound at creation (a device
 * problem table): keep the tensors alive and reuse them across runs; run is asynchronous on queue and graph-capturable.
 * create returns NULL with nad_last_error() set when the problems do not qualify. */
typedef struct nad_batch_problem {
  const void* weight; /* a loaded device weight (bestla_device_load_storage / nad_device_load) */
  const float* act;   /* [K] */
  float* out;         /* [N] */
} nad_batch_problem;
void* nad_batch_create(const nad_batch_problem* problems, int n);
int nad_batch_run(void* batch, void* queue);
void nad_batch_destroy(void* batch);

#ifdef __cplusplus
}
#endif
#endif /* NEURAL_AMD_H */
