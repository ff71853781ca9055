// ifetch_probe.hip -- development calibration (not product): cost of executing N never-repeated 8-byte instructions
// (s_mov_b32 with a literal) per launch, one wave vs 16 waves per CU, graph-replayed.  Separates instruction-fetch
// latency from issue cost: issue-bound ~1 cycle per SALU op; fetch-bound ~ (N * 8 B / 64 B) L2 round trips.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
#define STR2(x) #x
#define STR(x) STR2(x)
template <int N>
__global__ void junk(unsigned* out) {
  asm volatile(".rept %0\n\ts_mov_b32 s20, 0x12345678\n\t.endr" :: "i"(N) : "s20");
  if (threadIdx.x == 0) out[blockIdx.x] = blockIdx.x;
}
template <int N>
int run(unsigned* out, hipStream_t st, int threads) {
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int r = 0; r < 64; r++) hipLaunchKernelGGL(junk<N>, dim3(256), dim3(threads), 0, st, out);
  CK(hipStreamEndCapture(st, &g)); CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st)); for (int i = 0; i < 5; i++) CK(hipGraphLaunch(ge, st)); CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  printf("N=%5d (%6d B code) threads %4d: %7.2f us/launch\n", N, N * 8, threads, ms * 1e3 / (5 * 64));
  return 0;
}
int main() {
  unsigned* out; CK(hipMalloc(&out, 1 << 20)); hipStream_t st; CK(hipStreamCreate(&st));
  for (int t : {64, 1024}) { run<1>(out, st, t); run<256>(out, st, t); run<1024>(out, st, t); run<2048>(out, st, t); run<4096>(out, st, t); }
  return 0;
}
