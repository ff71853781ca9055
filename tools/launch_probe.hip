// launch_probe.hip -- development calibration (not product): the cost of kernel-argument (kernarg segment) reads at
// the start of a launch.  k1 reads its arguments in one batch; k2 makes a second, dependent scalar load (an argument
// indexed by another argument), as a kernel does when it selects one of several weight descriptors.  Graph-replayed.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
struct Big { unsigned* out; int sel; int pad; unsigned long long f[48]; };
__global__ void k1(Big a) { if (threadIdx.x == 0) a.out[blockIdx.x] = unsigned(a.f[3]) + a.sel; }
__global__ void k2(Big a) { if (threadIdx.x == 0) a.out[blockIdx.x] = unsigned(a.f[a.sel & 31]); }
__global__ void k3(Big a) {  // three dependent rounds
  if (threadIdx.x == 0) {
    int i = int(a.f[a.sel & 31]) & 31;
    int j = int(a.f[i]) & 31;
    a.out[blockIdx.x] = unsigned(a.f[j]);
  }
}
template <class F>
int run(const char* name, F kern, Big a, hipStream_t st) {
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int r = 0; r < 64; r++) hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, st, a);
  CK(hipStreamEndCapture(st, &g)); CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st)); for (int i = 0; i < 5; i++) CK(hipGraphLaunch(ge, st)); CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-28s %7.2f us/launch\n", name, ms * 1e3 / (5 * 64));
  return 0;
}
int main() {
  Big a{}; CK(hipMalloc(&a.out, 1 << 20)); a.sel = 5; for (int i = 0; i < 48; i++) a.f[i] = (i * 7) % 31;
  hipStream_t st; CK(hipStreamCreate(&st));
  run("one kernarg batch", k1, a, st); run("two dependent batches", k2, a, st); run("three dependent batches", k3, a, st);
  run("one kernarg batch", k1, a, st); run("two dependent batches", k2, a, st); run("three dependent batches", k3, a, st);
  return 0;
}
