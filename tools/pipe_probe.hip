// pipe_probe.hip -- development calibration (not product): can a decode step's dependent M = 1 matmuls run as
// separate kernels on two alternating streams, each kernel dispatched while its predecessor still runs, so that it
// streams its own weights before its input exists?
//
// Each "op" is a 256-workgroup kernel (512 threads, 64 KiB LDS: two fit per CU) that (A) loads `wkb` KiB of its own
// weights per workgroup into registers, (B) gathers the previous op's whole output vector -- 4096 8-byte {value, tag}
// granules written with sc1 stores, re-read with sc1 loads until every tag matches (the data is the flag) --, (C)
// folds both into 16 outputs per workgroup and publishes them as granules.  Modes: one stream (graph), two
// alternating streams captured into one graph, two alternating streams launched eagerly.  Every wait is bounded
// (50 ms) and counted, so a mode that orders the two branches wrongly shows give-ups instead of hanging.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x)                                                        \
  do {                                                               \
    hipError_t e = (x);                                              \
    if (e != hipSuccess) {                                           \
      printf("%s: %s\n", #x, hipGetErrorString(e));                  \
      return 1;                                                      \
    }                                                                \
  } while (0)

constexpr int kOps = 64, kWg = 256, kVec = kWg * 16;
typedef unsigned u4v __attribute__((ext_vector_type(4)));

// wkb_of(k): KiB of weights per workgroup of op k: a Llama-2-7B layer's per-CU shares cycled (QKV 96, O 32, gate/up
// 176, down 88) when wkb < 0, else wkb for every op
__device__ __host__ inline int wkb_of(int wkb, int k) {
  if (wkb >= 0) return wkb;
  const int t[4] = {96, 32, 176, 88};
  return t[k & 3];
}

// every wave holds a share of the weights (issued at dispatch) and then gathers 8 granules per lane -- all 8 loads in
// flight per pass, tags checked after the pass (a load -> check -> load loop would make 8 serial round trips per pass)
__global__ __launch_bounds__(512, 4) void op_kernel(unsigned* ctl, unsigned long long* gran, const uint4* weights,
                                                   int wkb_arg, int k, int last, unsigned long long* st) {
  extern __shared__ unsigned lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned gen = __builtin_amdgcn_readfirstlane(__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const int wkb = wkb_of(wkb_arg, k);
  const uint4* wp = weights + (size_t(k) * kWg + blockIdx.x) * size_t(176 * 64);
  const int nld = wkb * 64;  // 16-B loads of the workgroup
  u4v w[22];
#pragma unroll
  for (int i = 0; i < 22; i++) {
    const int idx = i * 512 + threadIdx.x;
    if (idx < nld) w[i] = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(wp + idx));
    else w[i] = u4v{0u, 0u, 0u, 0u};
  }
  float part = 0.f;
  unsigned long long tg = t0;
  if (k > 0) {
    const unsigned want = gen * 256u + unsigned(k);
    const unsigned long long* src = gran + size_t(k - 1) * kVec;
    unsigned pend = 0xFFu;
    unsigned spins = 0;
    while (true) {
      unsigned long long g[8];
#pragma unroll
      for (int j = 0; j < 8; j++)
        g[j] = __hip_atomic_load(src + j * 512 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 8; j++)
        if ((pend & (1u << j)) && unsigned(g[j] >> 32) == want) {
          part += __uint_as_float(unsigned(g[j]));
          pend &= ~(1u << j);
        }
      if (__all(pend == 0u)) break;
      __builtin_amdgcn_s_sleep(1);
      if (((++spins) & 63) == 0 && (__builtin_amdgcn_s_memrealtime() - t0) > 5000000ull) {  // 50 ms
        if (lane == 0) __hip_atomic_fetch_add(ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tg = __builtin_amdgcn_s_memrealtime();
#pragma unroll
  for (int i = 0; i < 22; i++) part += __uint_as_float(w[i][0] & 0x3f7fffffu) + __uint_as_float(w[i][3] & 0x3f7fffffu);
  lds[threadIdx.x] = __float_as_uint(part);
  if (threadIdx.x == 0) lds[600] = unsigned(tg), lds[601] = unsigned(tg >> 32);
  __syncthreads();
  if (threadIdx.x < 64) {
    const int o = threadIdx.x & 15, q = threadIdx.x >> 4;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) v += __uint_as_float(lds[(q * 8 + i) * 16 + o]);
    v += __shfl_down(v, 32, 64);
    v += __shfl_down(v, 16, 64);
    if (threadIdx.x < 16) {
      const unsigned long long g = (static_cast<unsigned long long>(gen * 256u + unsigned(k) + 1u) << 32) |
                                   __float_as_uint(v * 1e-6f);
      __hip_atomic_store(gran + size_t(k) * kVec + blockIdx.x * 16 + threadIdx.x, g, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (threadIdx.x == 0) {
    unsigned long long* s = st + (size_t(k) * kWg + blockIdx.x) * 4;
    s[0] = t0;
    s[1] = (static_cast<unsigned long long>(lds[601]) << 32) | lds[600];  // weights landed and input gathered
    s[2] = s[1];
    s[3] = __builtin_amdgcn_s_memrealtime();
    if (last) {
      const unsigned old = __hip_atomic_fetch_add(ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == gridDim.x * (gen + 1u) - 1u) __hip_atomic_fetch_add(ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

struct Bufs {
  unsigned* ctl;
  unsigned long long* gran;
  const uint4* weights;
  unsigned long long* st;
  int wkb;
};

static int enqueue(const Bufs& b, hipStream_t sa, hipStream_t sb, bool two, hipEvent_t fork, hipEvent_t join) {
  if (two) {
    CK(hipEventRecord(fork, sa));
    CK(hipStreamWaitEvent(sb, fork, 0));
  }
  for (int k = 0; k < kOps; k++) {
    hipStream_t s = (two && (k & 1)) ? sb : sa;
    hipLaunchKernelGGL(op_kernel, dim3(kWg), dim3(512), 64 * 1024, s, b.ctl, b.gran, b.weights, b.wkb, k,
                       k == kOps - 1 ? 1 : 0, b.st);
  }
  if (two) {
    CK(hipEventRecord(join, sb));
    CK(hipStreamWaitEvent(sa, join, 0));
  }
  return 0;
}

static int report(const char* name, const Bufs& b, float ms, int reps) {
  unsigned h[3];
  CK(hipMemcpy(h, b.ctl, 12, hipMemcpyDeviceToHost));
  std::vector<unsigned long long> s(size_t(kOps) * kWg * 4);
  CK(hipMemcpy(s.data(), b.st, s.size() * 8, hipMemcpyDeviceToHost));
  double lead = 0, wl = 0, gl = 0, post = 0, per = 0;
  int early = 0;
  double bytes = 0;
  for (int k = 0; k < kOps; k++) bytes += double(wkb_of(b.wkb, k)) * 1024 * kWg;
  for (int k = 1; k < kOps; k++) {
    unsigned long long start_min = ~0ull, prev_end_max = 0, w_max = 0, g_max = 0, end_max = 0;
    for (int g = 0; g < kWg; g++) {
      const unsigned long long* x = &s[(size_t(k) * kWg + g) * 4];
      start_min = std::min(start_min, x[0]);
      w_max = std::max(w_max, x[1]);
      g_max = std::max(g_max, x[2]);
      end_max = std::max(end_max, x[3]);
      prev_end_max = std::max(prev_end_max, s[(size_t(k - 1) * kWg + g) * 4 + 3]);
    }
    if (start_min < prev_end_max) early++;
    lead += double((long long)prev_end_max - (long long)start_min) * 0.01;
    wl += double((long long)w_max - (long long)start_min) * 0.01;
    gl += double((long long)g_max - (long long)prev_end_max) * 0.01;
    post += double((long long)end_max - (long long)std::max(g_max, w_max)) * 0.01;
    per += double((long long)end_max - (long long)prev_end_max) * 0.01;
  }
  const int n = kOps - 1;
  const double us = ms * 1e3 / (reps * kOps);
  printf("%-32s %7.3f us/op  %5.2f TB/s of weights  give-ups %u | dispatched early %d/%d, lead %.2f, first start -> "
         "weights landed (max) %.2f, prev end -> input gathered (max) %.2f, max(both) -> end %.2f, end-to-end %.2f us\n",
         name, us, bytes / (ms * 1e-3 / reps) / 1e12, h[1], early, n, lead / n, wl / n, gl / n, post / n, per / n);
  return 0;
}

static int run(const char* name, int mode, Bufs& b, hipStream_t sa, hipStream_t sb, hipEvent_t fork, hipEvent_t join) {
  const int reps = 20;
  CK(hipMemset(b.ctl, 0, 256));
  CK(hipMemset(b.gran, 0, size_t(kOps) * kVec * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipGraphExec_t ge = nullptr;
  hipGraph_t g = nullptr;
  if (mode != 2) {
    CK(hipStreamBeginCapture(sa, hipStreamCaptureModeGlobal));
    if (enqueue(b, sa, sb, mode == 1, fork, join)) return 1;
    CK(hipStreamEndCapture(sa, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  }
  auto once = [&]() -> int {
    if (mode == 2) return enqueue(b, sa, sb, true, fork, join);
    CK(hipGraphLaunch(ge, sa));
    return 0;
  };
  if (once() || once()) return 1;
  CK(hipStreamSynchronize(sa));
  CK(hipEventRecord(e0, sa));
  for (int r = 0; r < reps; r++)
    if (once()) return 1;
  CK(hipEventRecord(e1, sa));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  if (ge) {
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return report(name, b, ms, reps);
}

int main() {
  Bufs b{};
  CK(hipMalloc(&b.ctl, 256));
  CK(hipMalloc(&b.gran, size_t(kOps) * kVec * 8));
  CK(hipMalloc(&b.st, size_t(kOps) * kWg * 4 * 8));
  const size_t wbytes = size_t(kOps) * kWg * 176 * 1024;  // up to 176 KiB per workgroup per op: 2.9 GB, cold per replay
  void* wmem;
  CK(hipMalloc(&wmem, wbytes));
  CK(hipMemset(wmem, 0x11, wbytes));
  b.weights = static_cast<const uint4*>(wmem);
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(op_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                         64 * 1024));
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  for (int wkb : {0, 32, 96, 176, -1}) {
    b.wkb = wkb;
    if (wkb >= 0)
      printf("-- %d KiB of weights per workgroup per op (%.1f MB per op)\n", wkb, wkb * 1024.0 * kWg / 1e6);
    else
      printf("-- Llama-2-7B layer shares cycled: 96 / 32 / 176 / 88 KiB per workgroup (QKV, O, gate/up, down)\n");
    if (run("graph, one stream", 0, b, sa, sb, fork, join)) return 1;
    if (run("graph, two alternating streams", 1, b, sa, sb, fork, join)) return 1;
    if (run("eager, two alternating streams", 2, b, sa, sb, fork, join)) return 1;
  }
  return 0;
}
