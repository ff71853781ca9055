// pipe_probe.hip -- development calibration (not product): do dependent kernels on two alternating streams run
// co-resident on MI355X, so that kernel k+1 is dispatched (and can issue its weight loads) while kernel k still runs?
// Each "op" is a 256-workgroup kernel whose workgroups wait for the previous op's arrival counter (agent-scope
// acquire), spin `work` ns, and arrive on their own counter (release).  Modes: one stream (graph), two alternating
// streams captured into one graph (two branches), two alternating streams launched eagerly.  Every wait is bounded
// (50 ms); a give-up is recorded and reported, so a mode that serialises the two branches in the wrong order shows up
// as failures, not as a hang.
#include <hip/hip_runtime.h>

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

constexpr int kOps = 64, kWg = 256, kCnt = 64, kStride = 32;  // counters on their own 128-B lines

__global__ __launch_bounds__(512, 4) void op_kernel(unsigned* ctl, int k, int work_ns, int last,
                                                   unsigned long long* st) {
  extern __shared__ unsigned lds[];
  __shared__ unsigned gen_s;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    const unsigned gen = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    gen_s = gen;
    if (k > 0) {
      const unsigned want = unsigned(gridDim.x) * (gen + 1);
      unsigned* c = ctl + kCnt + (k - 1) * kStride;
      while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(2);
        if ((__builtin_amdgcn_s_memrealtime() - t_start) > 5000000ull) {  // 50 ms at 100 MHz
          __hip_atomic_fetch_add(ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
  }
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const unsigned long long t_go = __builtin_amdgcn_s_memrealtime();
  while ((__builtin_amdgcn_s_memrealtime() - t_go) * 10ull < unsigned(work_ns)) __builtin_amdgcn_s_sleep(1);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned gen = gen_s;
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    atomicMin(st + k * 4 + 0, t_start);
    atomicMax(st + k * 4 + 1, t_start);
    atomicMin(st + k * 4 + 2, t_go);
    atomicMax(st + k * 4 + 3, t_end);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(ctl + kCnt + k * kStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (last && old == unsigned(gridDim.x) * (gen + 1) - 1)
      __hip_atomic_fetch_add(ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static int enqueue(unsigned* ctl, int work, unsigned long long* st, hipStream_t a, hipStream_t b, bool two,
                   hipEvent_t fork, hipEvent_t join) {
  if (two) {
    CK(hipEventRecord(fork, a));
    CK(hipStreamWaitEvent(b, fork, 0));
  }
  for (int k = 0; k < kOps; k++) {
    hipStream_t s = (two && (k & 1)) ? b : a;
    hipLaunchKernelGGL(op_kernel, dim3(kWg), dim3(512), 64 * 1024, s, ctl, k, work, k == kOps - 1 ? 1 : 0, st);
  }
  if (two) {
    CK(hipEventRecord(join, b));
    CK(hipStreamWaitEvent(a, join, 0));
  }
  return 0;
}

static int report(const char* name, unsigned* ctl, unsigned long long* st, float ms, int reps) {
  unsigned h[2];
  CK(hipMemcpy(h, ctl, 8, hipMemcpyDeviceToHost));
  std::vector<unsigned long long> s(kOps * 4);
  CK(hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost));
  // overlap: op k+1 dispatched (first workgroup started) before op k's last workgroup ended
  int overl = 0;
  double disp_lead = 0, go_gap = 0;
  for (int k = 0; k + 1 < kOps; k++) {
    if (s[(k + 1) * 4 + 0] < s[k * 4 + 3]) overl++;
    disp_lead += double((long long)(s[k * 4 + 3]) - (long long)(s[(k + 1) * 4 + 0])) * 0.01;
    go_gap += double((long long)(s[(k + 1) * 4 + 2]) - (long long)(s[k * 4 + 3])) * 0.01;
  }
  printf("%-34s %8.3f us/op  give-ups %u  gen %u  | last replay: next op dispatched before prev end %d/%d, "
         "mean lead %.2f us, mean end(k)->go(k+1) %.2f us\n",
         name, ms * 1e3 / (reps * kOps), h[1], h[0], overl, kOps - 1, disp_lead / (kOps - 1), go_gap / (kOps - 1));
  return 0;
}

static int run(const char* name, int mode, int work, unsigned* ctl, unsigned long long* st, hipStream_t a,
               hipStream_t b, hipEvent_t fork, hipEvent_t join) {
  const int reps = 20;
  CK(hipMemset(ctl, 0, 4096 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto reset_st = [&]() -> int {
    std::vector<unsigned long long> init(kOps * 4);
    for (int k = 0; k < kOps; k++) init[k * 4] = init[k * 4 + 2] = ~0ull, init[k * 4 + 1] = init[k * 4 + 3] = 0;
    CK(hipMemcpyAsync(st, init.data(), init.size() * 8, hipMemcpyHostToDevice, a));
    CK(hipStreamSynchronize(a));
    return 0;
  };
  if (mode == 2) {  // eager two streams
    if (enqueue(ctl, work, st, a, b, true, fork, join)) return 1;
    CK(hipStreamSynchronize(a));
    CK(hipEventRecord(e0, a));
    for (int r = 0; r < reps; r++)
      if (enqueue(ctl, work, st, a, b, true, fork, join)) return 1;
    CK(hipEventRecord(e1, a));
    CK(hipEventSynchronize(e1));
    if (reset_st()) return 1;
    if (enqueue(ctl, work, st, a, b, true, fork, join)) return 1;
    CK(hipStreamSynchronize(a));
  } else {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(a, hipStreamCaptureModeGlobal));
    if (enqueue(ctl, work, st, a, b, mode == 1, fork, join)) return 1;
    CK(hipStreamEndCapture(a, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, a));
    CK(hipStreamSynchronize(a));
    CK(hipEventRecord(e0, a));
    for (int r = 0; r < reps; r++) CK(hipGraphLaunch(ge, a));
    CK(hipEventRecord(e1, a));
    CK(hipEventSynchronize(e1));
    if (reset_st()) return 1;
    CK(hipGraphLaunch(ge, a));
    CK(hipStreamSynchronize(a));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return report(name, ctl, st, ms, reps);
}

int main() {
  unsigned* ctl;
  unsigned long long* st;
  CK(hipMalloc(&ctl, 4096 * 4 + kCnt * 4 + kOps * kStride * 4));
  CK(hipMalloc(&st, kOps * 4 * 8));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(op_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                         64 * 1024));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  for (int work : {0, 3000, 8000}) {
    printf("-- work %d ns per op\n", work);
    if (run("graph, one stream", 0, work, ctl, st, a, b, fork, join)) return 1;
    if (run("graph, two alternating streams", 1, work, ctl, st, a, b, fork, join)) return 1;
    if (run("eager, two alternating streams", 2, work, ctl, st, a, b, fork, join)) return 1;
  }
  return 0;
}
