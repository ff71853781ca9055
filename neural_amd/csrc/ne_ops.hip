// ne_ops.hip -- the graph-facing half of the BesTLA seam on MI355X (include/neural_amd_ne.h): host helpers and
// support probes of core/layers/ne_bestla.cpp:27-249, and the device ops of the NS_SYCL build
// (core/layers/ne_bestla_sycl.cpp:173-880) as HIP kernels on the graph's queue (hipStream_t).
//
// These ops sit around the WOQ matmul in a decode layer (RMSNorm, residual add, SiLU, RoPE, KV copies, attention);
// they are memory-bound elementwise / row work: one thread per element (grid-stride) or one wave per row, coalesced
// along the contiguous dimension.  Host pointers given to the host half are staged through the device (the library
// has no CPU compute path).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/neural_amd.h"
#include "../../include/neural_amd_ne.h"

static_assert(sizeof(nad_ne_tensor) == 512, "ne_tensor layout (ne.h:161-199)");
static_assert(offsetof(nad_ne_tensor, ne) == 16 && offsetof(nad_ne_tensor, nb) == 48 &&
                  offsetof(nad_ne_tensor, op) == 80 && offsetof(nad_ne_tensor, op_params) == 88 &&
                  offsetof(nad_ne_tensor, src0) == 128 && offsetof(nad_ne_tensor, opt) == 144 &&
                  offsetof(nad_ne_tensor, n_tasks) == 432 && offsetof(nad_ne_tensor, data) == 456 &&
                  offsetof(nad_ne_tensor, padding) == 504,
              "ne_tensor field offsets");
static_assert(sizeof(nad_ne_compute_params) == 56 && offsetof(nad_ne_compute_params, dev_queue) == 48,
              "ne_compute_params layout (ne.h:242-255)");

namespace {

const nad_ne_tensor* T(const ne_tensor* t) { return reinterpret_cast<const nad_ne_tensor*>(t); }
nad_ne_tensor* T(ne_tensor* t) { return reinterpret_cast<nad_ne_tensor*>(t); }
const nad_ne_compute_params* P(const ne_compute_params* p) {
  return reinterpret_cast<const nad_ne_compute_params*>(p);
}

void ops_err(const char* where, const char* what) { fprintf(stderr, "neural_amd: %s: %s\n", where, what); }

bool skip_phase(const ne_compute_params* params) {
  const int t = P(params)->type;
  return t == NAD_NE_TASK_INIT || t == NAD_NE_TASK_FINALIZE;
}
hipStream_t queue_of(const ne_compute_params* params) { return static_cast<hipStream_t>(P(params)->dev_queue); }

bool is_device(const void* p) {
  hipPointerAttribute_t at;
  if (!p || hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeDevice;
}

inline int grid_for(int64_t n, int block) { return int(std::min<int64_t>((n + block - 1) / block, 65536)); }

// ------------------------------------------------------------------------------------------------ kernels
struct Shape4 {
  int64_t ne[4];
  int64_t nb[4];  // bytes
};
Shape4 shape(const nad_ne_tensor* t) {
  Shape4 s;
  for (int i = 0; i < 4; i++) {
    s.ne[i] = t->ne[i];
    s.nb[i] = int64_t(t->nb[i]);
  }
  return s;
}

// dst = src0 (*|+) src1, src1 broadcast over dims 1..3 by modulo (ne_bestla_sycl.cpp:173-226 / 228-281)
template <bool MUL>
__global__ void binary_kernel(const char* s0, const char* s1, char* d, Shape4 a, Shape4 b, Shape4 o) {
  const int64_t n = a.ne[0] * a.ne[1] * a.ne[2] * a.ne[3];
  for (int64_t idx = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * blockDim.x) {
    int64_t i = idx;
    const int64_t i0 = i % a.ne[0];
    i /= a.ne[0];
    const int64_t i1 = i % a.ne[1];
    i /= a.ne[1];
    const int64_t i2 = i % a.ne[2];
    const int64_t i3 = i / a.ne[2];
    const int64_t j1 = i1 % b.ne[1], j2 = i2 % b.ne[2], j3 = i3 % b.ne[3];
    const float x = *reinterpret_cast<const float*>(s0 + i3 * a.nb[3] + i2 * a.nb[2] + i1 * a.nb[1] + i0 * 4);
    const float y = *reinterpret_cast<const float*>(s1 + j3 * (b.ne[3] == 1 ? 0 : b.nb[3]) +
                                                    j2 * (b.ne[2] == 1 ? 0 : b.nb[2]) +
                                                    j1 * (b.ne[1] == 1 ? 0 : b.nb[1]) + i0 * 4);
    *reinterpret_cast<float*>(d + i3 * o.nb[3] + i2 * o.nb[2] + i1 * o.nb[1] + i0 * 4) = MUL ? x * y : x + y;
  }
}

// flat elementwise: silu or copy (ne_bestla_sycl.cpp:283-309)
__global__ void elewise_kernel(const float* s, float* d, int64_t n, int silu) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const float x = s[i];
    d[i] = silu ? x / (1.0f + expf(-x)) : x;
  }
}

// one workgroup per row: sum of squares (fp32), scale = 1/sqrt(mean + eps) (ne_bestla_sycl.cpp:311-383)
__global__ __launch_bounds__(256) void rms_norm_kernel(const char* s, char* d, Shape4 a, Shape4 o, float eps) {
  __shared__ float red[256];
  int64_t r = blockIdx.x;
  const int64_t i1 = r % a.ne[1];
  r /= a.ne[1];
  const int64_t i2 = r % a.ne[2];
  const int64_t i3 = r / a.ne[2];
  const float* x = reinterpret_cast<const float*>(s + i3 * a.nb[3] + i2 * a.nb[2] + i1 * a.nb[1]);
  float* y = reinterpret_cast<float*>(d + i3 * o.nb[3] + i2 * o.nb[2] + i1 * o.nb[1]);
  float sum = 0.f;
  for (int64_t i = threadIdx.x; i < a.ne[0]; i += blockDim.x) sum += x[i] * x[i];
  red[threadIdx.x] = sum;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (int(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const float scale = 1.0f / sqrtf(red[0] / float(a.ne[0]) + eps);
  for (int64_t i = threadIdx.x; i < a.ne[0]; i += blockDim.x) y[i] = x[i] * scale;
}

// BTLALayerNorm over contiguous rows (bestla_gemm.cpp:751-776, kernel_ref.h:2199-2240)
__global__ __launch_bounds__(256) void layernorm_kernel(const float* in, float* out, int size, int rms, float eps) {
  __shared__ float r1[256], r2[256];
  const float* x = in + size_t(blockIdx.x) * size;
  float* y = out + size_t(blockIdx.x) * size;
  float s = 0.f, sq = 0.f;
  for (int i = threadIdx.x; i < size; i += blockDim.x) {
    s += x[i];
    sq += x[i] * x[i];
  }
  r1[threadIdx.x] = s;
  r2[threadIdx.x] = sq;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (int(threadIdx.x) < w) {
      r1[threadIdx.x] += r1[threadIdx.x + w];
      r2[threadIdx.x] += r2[threadIdx.x + w];
    }
    __syncthreads();
  }
  const float mean = r1[0] / float(size);
  const float ms = rms ? sqrtf(r2[0] / float(size) + eps) : sqrtf(r2[0] / float(size) - mean * mean + eps);
  const float inv = 1.f / ms;
  __syncthreads();  // every thread has read r1/r2 before any row is overwritten in place
  for (int i = threadIdx.x; i < size; i += blockDim.x) y[i] = rms ? x[i] * inv : (x[i] - mean) * inv;
}

// out[b][i] = t[b][i] (*|+) v[b * vstep + i]
template <bool MUL>
__global__ void rowvec_kernel(const float* t, const float* v, float* out, int batch, int vsize, int vstep) {
  const int64_t n = int64_t(batch) * vsize;
  for (int64_t idx = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * blockDim.x) {
    const int64_t b = idx / vsize, i = idx % vsize;
    const float x = t[idx], y = v[b * vstep + i];
    out[idx] = MUL ? x * y : x + y;
  }
}

struct RopeArgs {
  float freq_scale, ext_factor, attn_factor, corr0, corr1, theta_scale;
  int64_t n_past;
};

__device__ float rope_ramp(float low, float high, int64_t i0) {
  const float y = (float(i0 / 2) - low) / fmaxf(0.001f, high - low);
  return 1.0f - fminf(1.0f, fmaxf(0.0f, y));
}

// one thread per row (i1, i2, i3), pairs rotated in order with the running theta (ne_bestla_sycl.cpp:436-536)
__global__ void rope_kernel(const char* s, char* d, Shape4 a, Shape4 o, RopeArgs r) {
  const int64_t rows = o.ne[1] * o.ne[2] * o.ne[3];
  for (int64_t row = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; row < rows; row += int64_t(gridDim.x) * blockDim.x) {
    int64_t t = row;
    const int64_t i1 = t % o.ne[1];
    t /= o.ne[1];
    const int64_t i2 = t % o.ne[2];
    const int64_t i3 = t / o.ne[2];
    float theta_base = float(r.n_past + i2);
    for (int64_t i0 = 0; i0 < o.ne[0]; i0 += 2) {
      const float theta_interp = r.freq_scale * theta_base;
      float theta = theta_interp, mscale = r.attn_factor;
      if (r.ext_factor != 0.0f) {
        const float mix = rope_ramp(r.corr0, r.corr1, i0) * r.ext_factor;
        theta = theta_interp * (1 - mix) + theta_base * mix;
        mscale *= 1.0f + 0.1f * logf(1.0f / r.freq_scale);
      }
      const float c = cosf(theta) * mscale, sn = sinf(theta) * mscale;
      theta_base *= r.theta_scale;
      const float* src = reinterpret_cast<const float*>(s + i3 * a.nb[3] + i2 * a.nb[2] + i1 * a.nb[1] + i0 * a.nb[0]);
      float* dst = reinterpret_cast<float*>(d + i3 * o.nb[3] + i2 * o.nb[2] + i1 * o.nb[1] + i0 * o.nb[0]);
      const float x0 = src[0], x1 = src[1];
      dst[0] = x0 * c - x1 * sn;
      dst[1] = x0 * sn + x1 * c;
    }
  }
}

// strided f32 -> f32 / f16 copy over the dst shape (ne_bestla_sycl.cpp:538-592)
__global__ void dup_kernel(const char* s, char* d, Shape4 a, Shape4 o, int to_f16) {
  const int64_t n = o.ne[0] * o.ne[1] * o.ne[2] * o.ne[3];
  for (int64_t idx = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * blockDim.x) {
    int64_t i = idx;
    const int64_t i0 = i % o.ne[0];
    i /= o.ne[0];
    const int64_t i1 = i % o.ne[1];
    i /= o.ne[1];
    const int64_t i2 = i % o.ne[2];
    const int64_t i3 = i / o.ne[2];
    const float v = *reinterpret_cast<const float*>(s + i0 * a.nb[0] + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3]);
    char* p = d + i0 * o.nb[0] + i1 * o.nb[1] + i2 * o.nb[2] + i3 * o.nb[3];
    if (to_f16)
      *reinterpret_cast<_Float16*>(p) = _Float16(v);
    else
      *reinterpret_cast<float*>(p) = v;
  }
}

// Attention of one (batch, query row, head) per wave, online softmax over the keys in chunks of 64
// (ne_bestla_sycl.cpp:594-880 MHA::forward1: Q [b][s][h][d], K [b][h][n_ctx][d], V^T [b][h][d][n_ctx], O [b][s][h][d];
// causal mask when seq > 1).  Lane j scores key (chunk + j); lane l accumulates output dims l, l + 64, ...
constexpr int kMhaMaxD = 256;
__global__ __launch_bounds__(64) void mha_kernel(const float* Q, const float* K, const float* V, float* O, int batch,
                                                 int seq, int seq_all, int hnum, int hsize, int n_ctx, float scale) {
  __shared__ float qs[kMhaMaxD];
  __shared__ float ps[64];
  int i = blockIdx.x;
  const int ih = i % hnum;
  i /= hnum;
  const int is = i % seq;
  const int ib = i / seq;
  const int lane = threadIdx.x;
  const size_t nf = size_t(hnum) * hsize;
  const float* q = Q + size_t(ib) * seq * nf + size_t(is) * nf + size_t(ih) * hsize;
  const float* k = K + size_t(ib) * n_ctx * nf + size_t(ih) * hsize * n_ctx;
  const float* v = V + size_t(ib) * n_ctx * nf + size_t(ih) * hsize * n_ctx;
  float* out = O + size_t(ib) * seq * nf + size_t(is) * nf + size_t(ih) * hsize;
  for (int d = lane; d < hsize; d += 64) qs[d] = q[d];
  __syncthreads();
  const int n_past = seq_all - seq;
  const int limit = seq > 1 ? min(seq_all, is + n_past + 1) : seq_all;
  float m = -INFINITY, l = 0.f;
  float acc[kMhaMaxD / 64];
#pragma unroll
  for (int r = 0; r < kMhaMaxD / 64; r++) acc[r] = 0.f;
  for (int c0 = 0; c0 < limit; c0 += 64) {
    const int j = c0 + lane;
    float s = -INFINITY;
    if (j < limit) {
      const float* kr = k + size_t(j) * hsize;
      float t = 0.f;
      for (int d = 0; d < hsize; d++) t += qs[d] * kr[d];
      s = t * scale;
    }
    float cm = s;
    for (int off = 32; off > 0; off >>= 1) cm = fmaxf(cm, __shfl_xor(cm, off));
    const float mn = fmaxf(m, cm);
    const float corr = expf(m - mn);  // 0 on the first chunk (m = -inf)
    const float p = j < limit ? expf(s - mn) : 0.f;
    float ls = p;
    for (int off = 32; off > 0; off >>= 1) ls += __shfl_xor(ls, off);
    l = l * corr + ls;
    m = mn;
    __syncthreads();
    ps[lane] = p;
    __syncthreads();
    const int nk = min(64, limit - c0);
#pragma unroll
    for (int r = 0; r < kMhaMaxD / 64; r++) {
      const int d = lane + 64 * r;
      if (d < hsize) {
        const float* vr = v + size_t(d) * n_ctx + c0;
        float t = 0.f;
        for (int jj = 0; jj < nk; jj++) t += ps[jj] * vr[jj];
        acc[r] = acc[r] * corr + t;
      }
    }
  }
  const float inv = 1.f / l;
#pragma unroll
  for (int r = 0; r < kMhaMaxD / 64; r++) {
    const int d = lane + 64 * r;
    if (d < hsize) out[d] = acc[r] * inv;
  }
}

// ------------------------------------------------------------------------------------------------ staging helper
// run fn() on device pointers for host or device buffers, synchronously (the reference's host helpers return with
// the result in place): host buffers are copied in when `in`, copied back when `out`
struct Buf {
  const void* host;
  size_t bytes;
  bool in, out;
  void* dev = nullptr;
  bool staged = false;
};
template <class Fn>
bool with_device(std::vector<Buf>& bufs, Fn fn) {
  bool ok = true;
  for (auto& b : bufs) {
    if (!b.host || is_device(b.host)) {
      b.dev = const_cast<void*>(b.host);
      continue;
    }
    if (hipMalloc(&b.dev, b.bytes) != hipSuccess) {
      b.dev = nullptr;
      ok = false;
      break;
    }
    b.staged = true;
    if (b.in && hipMemcpy(b.dev, b.host, b.bytes, hipMemcpyHostToDevice) != hipSuccess) ok = false;
  }
  ok = ok && fn() && hipDeviceSynchronize() == hipSuccess;
  for (auto& b : bufs) {
    if (b.staged && b.out && ok)
      ok = hipMemcpy(const_cast<void*>(b.host), b.dev, b.bytes, hipMemcpyDeviceToHost) == hipSuccess;
    if (b.staged) (void)hipFree(b.dev);
  }
  return ok;
}

// ------------------------------------------------------------------------------------------------ host threading
int g_threads = 0;
int host_threads() {
  if (g_threads > 0) return g_threads;
  const unsigned h = std::thread::hardware_concurrency();
  return h ? int(h) : 1;
}

class PhaseBarrier {
 public:
  explicit PhaseBarrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const int gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      gen_++;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != gen; });
    }
  }

 private:
  int n_, count_ = 0, gen_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
};

}  // namespace

// ================================================================================================ host half
extern "C" void bestla_timer(bool _init) {
  static std::chrono::steady_clock::time_point t0;
  if (_init) {
    t0 = std::chrono::steady_clock::now();
  } else {
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    printf("time :%f us\n", us);
    fflush(stdout);
  }
}

extern "C" void nad_set_host_threads(int n) { g_threads = n; }

extern "C" void bestla_parallel_for(nad_forward_compute_fptr fcomp, struct ne_compute_params* mainparams,
                                    struct ne_tensor* node) {
  auto* mp = reinterpret_cast<nad_ne_compute_params*>(mainparams);
  if (mp->nth <= 1) {
    nad_ne_compute_params params = *mp;
    for (int phase : {int(NAD_NE_TASK_INIT), int(NAD_NE_TASK_COMPUTE), int(NAD_NE_TASK_FINALIZE)}) {
      params.type = phase;
      fcomp(reinterpret_cast<ne_compute_params*>(&params), node);
    }
    return;
  }
  const int nth = mp->nth;
  const int workers = std::max(nth, 1);
  PhaseBarrier bar(workers);
  auto body = [&](int tidx) {
    nad_ne_compute_params params = *mp;
    params.ith = tidx;
    params.type = NAD_NE_TASK_INIT;
    if (tidx == 0) fcomp(reinterpret_cast<ne_compute_params*>(&params), node);
    bar.wait();
    params.type = NAD_NE_TASK_COMPUTE;
    if (params.ith < params.nth) fcomp(reinterpret_cast<ne_compute_params*>(&params), node);
    bar.wait();
    params.type = NAD_NE_TASK_FINALIZE;
    if (params.ith < params.nth) fcomp(reinterpret_cast<ne_compute_params*>(&params), node);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < workers; t++) th.emplace_back(body, t);
  body(0);
  for (auto& t : th) t.join();
}

extern "C" void bestla_layernormalization(int norm_count, int norm_size, bool isrms, float epsilon, const float* FpIn,
                                          float* FpOut) {
  if (norm_count <= 0 || norm_size <= 0) return;
  const size_t bytes = size_t(norm_count) * norm_size * 4;
  const bool inplace = FpIn == FpOut;
  std::vector<Buf> bufs = {{FpIn, bytes, true, inplace}};
  if (!inplace) bufs.push_back({FpOut, bytes, false, true});
  const bool ok = with_device(bufs, [&] {
    float* out = static_cast<float*>(bufs.back().dev);
    hipLaunchKernelGGL(layernorm_kernel, dim3(norm_count), dim3(256), 0, 0, static_cast<const float*>(bufs[0].dev),
                       out, norm_size, isrms ? 1 : 0, epsilon);
    return hipGetLastError() == hipSuccess;
  });
  if (!ok) ops_err("bestla_layernormalization", "device execution failed");
}

template <bool MUL>
static void host_rowvec(const char* name, int batch, int vsize, const float* tensor, const float* vector, int vstep,
                        float* out) {
  if (batch <= 0 || vsize <= 0) return;
  const size_t tb = size_t(batch) * vsize * 4;
  const size_t vb = (size_t(batch - 1) * vstep + vsize) * 4;
  std::vector<Buf> bufs = {{tensor, tb, true, false}, {vector, vb, true, false}, {out, tb, false, true}};
  if (out == tensor) {  // in place
    bufs[0].out = true;
    bufs.pop_back();
  }
  const bool ok = with_device(bufs, [&] {
    hipLaunchKernelGGL(rowvec_kernel<MUL>, dim3(grid_for(int64_t(batch) * vsize, 256)), dim3(256), 0, 0,
                       static_cast<const float*>(bufs[0].dev), static_cast<const float*>(bufs[1].dev),
                       static_cast<float*>(bufs.back().dev), batch, vsize, vstep);
    return hipGetLastError() == hipSuccess;
  });
  if (!ok) ops_err(name, "device execution failed");
}

extern "C" void bestla_mul(int batch, int vsize, const float* tensor, const float* vector, int vstep, float* out) {
  host_rowvec<true>("bestla_mul", batch, vsize, tensor, vector, vstep, out);
}
extern "C" void bestla_add(int batch, int vsize, const float* tensor, const float* vector, int vstep, float* out) {
  host_rowvec<false>("bestla_add", batch, vsize, tensor, vector, vstep, out);
}

static bool ne_contig(const nad_ne_tensor* t) { return t->nb[0] <= t->nb[1] && t->nb[1] <= t->nb[2] && t->nb[2] <= t->nb[3]; }
static int64_t ne_rows(const nad_ne_tensor* t) { return t->ne[1] * t->ne[2] * t->ne[3]; }

// ne_bestla.cpp:176-203: the device backend takes BTLA matmuls and f32 RMS_NORM / SILU / ADD / MUL when an operand
// already lives on the device
extern "C" int bestla_backend_support(struct ne_tensor* src0p, struct ne_tensor* src1p, int op) {
  const nad_ne_tensor* s0 = T(src0p);
  const nad_ne_tensor* s1 = src1p ? T(src1p) : nullptr;
  bool on_dev = s0->backend == NAD_NE_BACKEND_DEVICE;
  if (s1) on_dev |= s1->backend == NAD_NE_BACKEND_DEVICE;
  switch (op) {
    case NAD_NE_OP_MUL_MAT:
      if (s0->type == NAD_NE_TYPE_BTLA) return on_dev ? NAD_NE_BACKEND_DEVICE : NAD_NE_BACKEND_CPU;
      break;
    case NAD_NE_OP_RMS_NORM:
    case NAD_NE_OP_SILU:
    case NAD_NE_OP_ADD:
    case NAD_NE_OP_MUL:
      if (s0->type == NAD_NE_TYPE_F32) return on_dev ? NAD_NE_BACKEND_DEVICE : NAD_NE_BACKEND_CPU;
      break;
    default:
      break;
  }
  return NAD_NE_BACKEND_CPU;
}

extern "C" size_t nad_device_workspace_size(int m, int k) {
  // K padded to the largest device K tile (256: int2), so the bound holds for every weight format
  const size_t kp = (size_t(k) + 255) / 256 * 256;
  auto a256 = [](size_t x) { return (x + 255) / 256 * 256; };
  // fp16 copy of A (tile padded), then the split-K partials of a GEMM with few output tiles (bound for any N); the
  // mid-M kernel's K-run slabs (ks x N <= 32768 fp32 per row, capi.hip run_mid) fit the same m x 128 KiB
  const size_t nbm = (size_t(m) + 255) / 256;
  const size_t gemm = a256(size_t(m) * kp * 2) + size_t(m) * 4 * 256 * 128 / nbm + 256;
  // m <= 16: the fp decode GEMV stages its activations in LDS; a weight in the int8-compute mode quantizes them into
  // u8 codes [m][kp] + per-(row, block) {scale, zp} (block >= 32); the mid-M kernel runs from 8 / 12 rows by default
  // (from any m with NAD_MID_MIN_M), so its split-K slabs are covered here too
  if (m <= 16) return std::max(a256(size_t(m) * kp) + a256(size_t(m) * (kp / 32) * 8) + 256, gemm);
  return gemm;
}

// ne_bestla.cpp:205-249 + the device workspace of this backend's prefill GEMM (the reference's SYCL path reports 0)
extern "C" bool bestla_support(struct ne_tensor* nodep, int n_threads, size_t* workspace, size_t* dev_workspace) {
  nad_ne_tensor* node = T(nodep);
  size_t ws_h = 0, ws_d = 0;
  bool support = node->backend == NAD_NE_BACKEND_DEVICE;
  switch (node->op) {
    case NAD_NE_OP_MUL_MAT_ID:
    case NAD_NE_OP_MUL_MAT_BIAS:
    case NAD_NE_OP_MUL_MAT: {
      const nad_ne_tensor* wei = node->op == NAD_NE_OP_MUL_MAT_ID ? node->opt[0] : node->src0;
      if (node->src0->type == NAD_NE_TYPE_BTLA) {
        const int m = int(node->src1->ne[1]), k = int(node->src1->ne[0]);
        if (node->src0->backend == NAD_NE_BACKEND_CPU)
          ws_h = bestla_f32f32_get_workspace_size(m, int(wei->ne[1]), k, wei->data);
        else
          ws_d = nad_device_workspace_size(m, k);
        support = true;
      }
    } break;
    case NAD_NE_OP_ROPE:
      if (node->type == NAD_NE_TYPE_BTLA) support = true;
      break;
    case NAD_NE_OP_MUL:
    case NAD_NE_OP_ADD:
      if (ne_contig(node->src1) && ne_contig(node->src0) &&
          (ne_rows(node->src1) == 1 || ne_rows(node->src1) == ne_rows(node->src0)) &&
          node->src0->ne[0] == node->src1->ne[0] && node->nb[0] == sizeof(float))
        support = true;
      break;
    case NAD_NE_OP_MUL_FFN_SILU:
    case NAD_NE_OP_MUL_FFN_GELU:
    case NAD_NE_OP_MUL_FFN_GELU_MUL:
    case NAD_NE_OP_MUL_FFN_ADD_GELU:
      if (node->src0->backend == NAD_NE_BACKEND_CPU) {
        ws_h = bestla_fusion_FFN_f32f32_get_workspace_size(int(node->src0->ne[1]), int(node->src0->ne[0]),
                                                           int(node->src1->ne[1]), int(node->opt[0]->ne[1]),
                                                           node->src1->data, node->opt[0]->data);
        support = true;
      }
      break;
    case NAD_NE_OP_MUL_ID_FFN_GELU:
    case NAD_NE_OP_MUL_ID_FFN_SILU:
      if (node->src0->backend == NAD_NE_BACKEND_CPU) {
        ws_h = bestla_fusion_FFN_f32f32_get_workspace_size(int(node->src0->ne[1]), int(node->src0->ne[0]),
                                                           int(node->opt[0]->ne[1]), int(node->opt[9]->ne[1]),
                                                           node->opt[0]->data, node->opt[9]->data);
        support = true;
      }
      break;
    case NAD_NE_OP_MUL_QKV:
      ws_h = bestla_fusion_QKV_f32f32_get_workspace_size(int(node->src0->ne[1]), int(node->src1->ne[1]),
                                                         int(node->src1->ne[0]), node->src1->data);
      support = true;
      break;
    case NAD_NE_OP_NORM:
    case NAD_NE_OP_RMS_NORM:
      if (ne_contig(node->src0)) support = true;
      break;
    default:
      break;
  }
  if (support) node->n_tasks = 1;
  *workspace = ws_h;
  *dev_workspace = ws_d;
  return support;
}

// ================================================================================================ device half
extern "C" void bestla_device_mul_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                                      const struct ne_tensor* src1, struct ne_tensor* dst) {
  if (skip_phase(params)) return;
  const auto *a = T(src0), *b = T(src1);
  auto* o = T(dst);
  const int64_t n = a->ne[0] * a->ne[1] * a->ne[2] * a->ne[3];
  hipLaunchKernelGGL(binary_kernel<true>, dim3(grid_for(n, 256)), dim3(256), 0, queue_of(params),
                     static_cast<const char*>(a->data), static_cast<const char*>(b->data), static_cast<char*>(o->data),
                     shape(a), shape(b), shape(o));
  if (hipGetLastError() != hipSuccess) ops_err("bestla_device_mul_f32", "launch failed");
}

extern "C" void bestla_device_add_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                                      const struct ne_tensor* src1, struct ne_tensor* dst) {
  if (skip_phase(params)) return;
  const auto *a = T(src0), *b = T(src1);
  auto* o = T(dst);
  const int64_t n = a->ne[0] * a->ne[1] * a->ne[2] * a->ne[3];
  hipLaunchKernelGGL(binary_kernel<false>, dim3(grid_for(n, 256)), dim3(256), 0, queue_of(params),
                     static_cast<const char*>(a->data), static_cast<const char*>(b->data), static_cast<char*>(o->data),
                     shape(a), shape(b), shape(o));
  if (hipGetLastError() != hipSuccess) ops_err("bestla_device_add_f32", "launch failed");
}

extern "C" void bestla_device_elewise_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                                          struct ne_tensor* dst) {
  if (skip_phase(params)) return;
  const auto* a = T(src0);
  auto* o = T(dst);
  const int64_t n = a->ne[0] * a->ne[1] * a->ne[2] * a->ne[3];
  hipLaunchKernelGGL(elewise_kernel, dim3(grid_for(n, 256)), dim3(256), 0, queue_of(params),
                     static_cast<const float*>(a->data), static_cast<float*>(o->data), n,
                     o->op == NAD_NE_OP_SILU ? 1 : 0);
  if (hipGetLastError() != hipSuccess) ops_err("bestla_device_elewise_f32", "launch failed");
}

extern "C" void bestla_device_rms_norm_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                                           struct ne_tensor* dst) {
  if (skip_phase(params)) return;
  const auto* a = T(src0);
  auto* o = T(dst);
  float eps;
  std::memcpy(&eps, o->op_params, sizeof(float));
  const int64_t rows = a->ne[1] * a->ne[2] * a->ne[3];
  if (rows <= 0) return;
  hipLaunchKernelGGL(rms_norm_kernel, dim3(unsigned(rows)), dim3(256), 0, queue_of(params),
                     static_cast<const char*>(a->data), static_cast<char*>(o->data), shape(a), shape(o), eps);
  if (hipGetLastError() != hipSuccess) ops_err("bestla_device_rms_norm_f32", "launch failed");
}

// ne_layers.c:9225-9234 (YaRN correction dims)
static void rope_corr_dims(int n_dims, int n_orig_ctx, float freq_base, float beta_fast, float beta_slow,
                           float dims[2]) {
  auto corr = [&](float n_rot) {
    return n_dims * logf(n_orig_ctx / (n_rot * 2 * 3.14159265358979323846f)) / (2 * logf(freq_base));
  };
  dims[0] = std::max(0.0f, floorf(corr(beta_fast)));
  dims[1] = std::min(float(n_dims - 1), ceilf(corr(beta_slow)));
}

extern "C" void bestla_device_rope_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                                       const struct ne_tensor* src1, struct ne_tensor* dst) {
  if (skip_phase(params)) return;
  const auto *a = T(src0), *b = T(src1);
  auto* o = T(dst);
  if (b->type != NAD_NE_TYPE_I32) {
    ops_err("bestla_device_rope_f32", "src1 must be the I32 rope parameter tensor");
    return;
  }
  const float* fp = reinterpret_cast<const float*>(o->op_params);
  // src1 holds {n_past, n_dims, mode, prompt_size, n_keep} (ne_bestla_sycl.cpp:455-467); read it where it lives
  int32_t ip[5] = {0, 0, 0, 0, 0};
  if (is_device(b->data)) {
    if (hipMemcpyAsync(ip, b->data, sizeof(ip), hipMemcpyDeviceToHost, queue_of(params)) != hipSuccess ||
        hipStreamSynchronize(queue_of(params)) != hipSuccess) {
      ops_err("bestla_device_rope_f32", "reading the rope parameters failed");
      return;
    }
  } else {
    std::memcpy(ip, b->data, sizeof(ip));
  }
  const float freq_base = fp[0], freq_scale = 1 / fp[1];
  const int n_orig_ctx = int(fp[2]);
  RopeArgs r{};
  r.freq_scale = freq_scale;
  r.ext_factor = fp[3];
  r.attn_factor = fp[4];
  const float beta_fast = fp[5], beta_slow = fp[6];
  const int n_dims = ip[1];
  r.n_past = ip[0];
  r.theta_scale = powf(freq_base, -2.0f / float(n_dims));
  float cd[2];
  rope_corr_dims(n_dims, n_orig_ctx, freq_base, beta_fast, beta_slow, cd);
  r.corr0 = cd[0];
  r.corr1 = cd[1];
  const int64_t rows = o->ne[1] * o->ne[2] * o->ne[3];
  hipLaunchKernelGGL(rope_kernel, dim3(grid_for(rows, 64)), dim3(64), 0, queue_of(params),
                     static_cast<const char*>(a->data), static_cast<char*>(o->data), shape(a), shape(o), r);
  if (hipGetLastError() != hipSuccess) ops_err("bestla_device_rope_f32", "launch failed");
}

extern "C" void bestla_device_dup_f32(const struct ne_compute_params* params, const struct ne_tensor* src0,
                                      struct ne_tensor* dst) {
  if (skip_phase(params)) return;
  const auto* a = T(src0);
  auto* o = T(dst);
  if (o->type != NAD_NE_TYPE_F32 && o->type != NAD_NE_TYPE_F16) {
    ops_err("bestla_device_dup_f32", "destination must be F32 or F16");
    return;
  }
  const int64_t n = o->ne[0] * o->ne[1] * o->ne[2] * o->ne[3];
  hipLaunchKernelGGL(dup_kernel, dim3(grid_for(n, 256)), dim3(256), 0, queue_of(params),
                     static_cast<const char*>(a->data), static_cast<char*>(o->data), shape(a), shape(o),
                     o->type == NAD_NE_TYPE_F16 ? 1 : 0);
  if (hipGetLastError() != hipSuccess) ops_err("bestla_device_dup_f32", "launch failed");
}

extern "C" void bestla_device_mha_f32(const struct ne_compute_params* params, const struct ne_tensor* qp,
                                      const struct ne_tensor* kp, const struct ne_tensor* vp, struct ne_tensor* dst) {
  if (skip_phase(params)) return;
  const auto *q = T(qp), *k = T(kp), *v = T(vp);
  auto* o = T(dst);
  const int hsize = int(q->ne[0]), hnum = int(q->ne[1]), seq = int(q->ne[2]), batch = int(q->ne[3]);
  const int seq_all = int(k->ne[1]);
  float scale;
  uint32_t n_ctx;
  std::memcpy(&scale, o->padding, 4);
  std::memcpy(&n_ctx, o->padding + 4, 4);
  if (hsize > kMhaMaxD || seq_all > int(n_ctx) || seq_all < seq) {
    ops_err("bestla_device_mha_f32", "unsupported head size / context (head <= 256, seq <= seq_all <= n_ctx)");
    return;
  }
  hipLaunchKernelGGL(mha_kernel, dim3(unsigned(batch * seq * hnum)), dim3(64), 0, queue_of(params),
                     static_cast<const float*>(q->data), static_cast<const float*>(k->data),
                     static_cast<const float*>(v->data), static_cast<float*>(o->data), batch, seq, seq_all, hnum, hsize,
                     int(n_ctx), scale);
  if (hipGetLastError() != hipSuccess) ops_err("bestla_device_mha_f32", "launch failed");
}
