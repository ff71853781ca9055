/*
 * neural_amd_ne.h -- the graph-facing half of Neural Speed's BesTLA seam (neural_speed/core/ne_bestla.h:21-30,76-83,
 * 99-111) re-hosted on MI355X: host threading/timer/norm/elementwise helpers, the support probes the graph planner
 * calls (ne_layers.c:11929-11967), and the device elementwise / norm / RoPE / copy / attention ops of the NS_SYCL build
 * (implemented for SYCL in neural_speed/core/layers/ne_bestla_sycl.cpp:173-880; called at ne_layers.c:4253, 4569,
 * 5634, 6406, 6593, 9248, 9913).  Implemented in neural_amd/csrc/ne_ops.hip.
 *
 * The entry points take the reference's own `struct ne_tensor*` / `struct ne_compute_params*` (declared incomplete
 * here; callers pass the structs of neural_speed/core/ne.h).  The library reads them through the layout restated below
 * (ne.h:161-199, 242-255); tests/test_ne_link.py checks every offset against the reference header.  Device queues are
 * hipStream_t.  Element values and enum codes restate neural_speed/core/data_types.h and ne.h.
 */
#ifndef NEURAL_AMD_NE_H
#define NEURAL_AMD_NE_H
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- restated layout of struct ne_tensor (ne.h:161-199; sizeof 512 on LP64) */
#define NAD_NE_MAX_DIMS 4
#define NAD_NE_MAX_OPT 36
#define NAD_NE_MAX_OP_PARAMS 32
typedef struct nad_ne_tensor {
  int32_t type;    /* enum ne_type */
  int32_t backend; /* enum ne_backend */
  int32_t n_dims;
  int64_t ne[NAD_NE_MAX_DIMS];
  size_t nb[NAD_NE_MAX_DIMS];
  int32_t op; /* enum ne_op */
  bool is_param;
  int32_t op_params[NAD_NE_MAX_OP_PARAMS / 4];
  struct nad_ne_tensor* grad;
  struct nad_ne_tensor* src0;
  struct nad_ne_tensor* src1;
  struct nad_ne_tensor* opt[NAD_NE_MAX_OPT];
  int32_t n_tasks;
  int32_t perf_runs;
  int64_t perf_cycles;
  int64_t perf_time_us;
  void* data;
  size_t size;
  char name[32];
  char padding[8];
} nad_ne_tensor;

/* ---- restated layout of struct ne_compute_params (ne.h:242-255) */
typedef struct nad_ne_compute_params {
  int32_t type; /* enum ne_task_type */
  int32_t ith, nth;
  size_t wsize;
  void* wdata;
  size_t dev_wsize;
  void* dev_wdata;
  void* dev_queue; /* hipStream_t here (sycl::queue* in the reference) */
} nad_ne_compute_params;

/* ---- enum codes used on this seam (data_types.h:32-56 ne_type, ne.h:95-98 ne_backend, ne.h:236-240 ne_task_type,
 * data_types.h ne_op) */
enum {
  NAD_NE_TYPE_F32 = 0, NAD_NE_TYPE_F16 = 1, NAD_NE_TYPE_Q4_0 = 2, NAD_NE_TYPE_Q8_0 = 8, NAD_NE_TYPE_I32 = 18,
  NAD_NE_TYPE_BTLA = 19,
  NAD_NE_BACKEND_CPU = 0, NAD_NE_BACKEND_DEVICE = 1, /* NE_BACKEND_SYCL */
  NAD_NE_TASK_INIT = 0, NAD_NE_TASK_COMPUTE = 1, NAD_NE_TASK_FINALIZE = 2,
  NAD_NE_OP_NONE = 0, NAD_NE_OP_DUP = 1, NAD_NE_OP_ADD = 2, NAD_NE_OP_MUL = 6, NAD_NE_OP_GELU = 21,
  NAD_NE_OP_SILU = 22, NAD_NE_OP_NORM = 24, NAD_NE_OP_RMS_NORM = 25, NAD_NE_OP_MUL_MAT = 28,
  NAD_NE_OP_MUL_MAT_BIAS = 29, NAD_NE_OP_MUL_MAT_ID = 30, NAD_NE_OP_CPY = 33, NAD_NE_OP_ROPE = 46,
  NAD_NE_OP_MUL_QKV = 52, NAD_NE_OP_MUL_FFN_SILU = 53, NAD_NE_OP_MUL_FFN_GELU = 54, NAD_NE_OP_MUL_FFN_GELU_MUL = 55,
  NAD_NE_OP_MUL_FFN_ADD_GELU = 56, NAD_NE_OP_MUL_ID_FFN_SILU = 57, NAD_NE_OP_MUL_ID_FFN_GELU = 58
};

struct ne_tensor;
struct ne_compute_params;
typedef void (*nad_forward_compute_fptr)(struct ne_compute_params*, struct ne_tensor*);

/* ---- host half (ne_bestla.h:21-30, 76-83; CPU implementation core/layers/ne_bestla.cpp:27-249) */
void bestla_timer(bool _init);                                                                     /* ne_bestla.h:21 */
/* INIT on thread 0, barrier, COMPUTE on nth threads, barrier, FINALIZE (ne_bestla.cpp:42-70) */
void bestla_parallel_for(nad_forward_compute_fptr fcomp, struct ne_compute_params* mainparams,
                         struct ne_tensor* node);                                                  /* ne_bestla.h:29 */
/* row-wise (RMS) normalisation, kernel_ref.h:2199-2240 order; host or device pointers (host ones are staged) */
void bestla_layernormalization(int norm_count, int norm_size, bool isrms, float epsilon, const float* FpIn,
                               float* FpOut);                                                      /* ne_bestla.h:76 */
/* out[b][i] = tensor[b*vsize + i] (*|+) vector[b*vstep + i]  (vstep 0 broadcasts one row) */
void bestla_mul(int batch, int vsize, const float* tensor, const float* vector, int vstep, float* out); /* :79 */
void bestla_add(int batch, int vsize, const float* tensor, const float* vector, int vstep, float* out); /* :80 */
/* returns enum ne_backend (an int-sized enum in the reference) */
int bestla_backend_support(struct ne_tensor* src0, struct ne_tensor* src1, int op);              /* ne_bestla.h:82 */
/* node planner probe: host + device workspace (device: the fp16 activation copy of the prefill GEMM) */
bool bestla_support(struct ne_tensor* node, int n_threads, size_t* workspace, size_t* dev_workspace); /* :83 */

/* ---- device half (ne_bestla.h:99-111; SYCL implementation ne_bestla_sycl.cpp:173-880).  Asynchronous on
 * params->dev_queue; INIT / FINALIZE phases are no-ops as in the reference. */
void bestla_device_mul_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                           const struct ne_tensor* src1, struct ne_tensor* dst);
void bestla_device_add_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                           const struct ne_tensor* src1, struct ne_tensor* dst);
void bestla_device_elewise_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                               struct ne_tensor* dst);     /* dst->op == SILU: silu, else copy */
void bestla_device_rms_norm_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                                struct ne_tensor* dst);    /* eps = ((float*)dst->op_params)[0] */
void bestla_device_rope_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                            const struct ne_tensor* src1, struct ne_tensor* dst); /* YaRN params in dst->op_params */
void bestla_device_dup_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                           struct ne_tensor* dst);         /* strided f32 -> f32 / f16 */
void bestla_device_mha_f32(const struct ne_compute_params* params, const struct ne_tensor* q,
                           const struct ne_tensor* k, const struct ne_tensor* v,
                           struct ne_tensor* dst);         /* scale, n_ctx in dst->padding */

/* ---- native: bind a caller-owned device workspace to a queue (the role of cgraph->dev_work, ne_layers.c:11947-11967)
 * for the nad_device_* entry points, which take no workspace argument.  bytes = 0 unbinds. */
int nad_bind_workspace(void* queue, void* ptr, size_t bytes);
/* device workspace the WOQ forward needs for m x k activations (0 at m <= 16) */
size_t nad_device_workspace_size(int m, int k);

#ifdef __cplusplus
}
#endif
#endif /* NEURAL_AMD_NE_H */
