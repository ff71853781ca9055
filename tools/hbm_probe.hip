// hbm_probe.hip -- development calibration tool (not part of the product): how fast can one launch stream B bytes of
// cold HBM into the CUs on this MI355X?  A pure read kernel (every byte read once, 16 B/lane, one value written per
// thread so nothing is dead) timed over rotating buffers (1.5 GiB pool, so the 256 MB Infinity Cache never serves a
// re-read), back-to-back in one captured HIP graph, for several grid shapes.  This is the floor the decode GEMV launches
// of the same byte counts are compared against.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// mode 0: grid-stride (consecutive waves read consecutive KiB);  mode 1: each wave streams its own contiguous range
template <int UNROLL>
__global__ void read_kernel(const u4* __restrict__ p, size_t n16, unsigned* out, int mode) {
  u4 acc = {0u, 0u, 0u, 0u};
  const size_t tid = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const size_t nth = size_t(gridDim.x) * blockDim.x;
  if (mode == 0) {
    size_t i = tid;
    for (; i + (UNROLL - 1) * nth < n16; i += UNROLL * nth) {
      u4 v[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; u++) v[u] = __builtin_nontemporal_load(p + i + u * nth);
#pragma unroll
      for (int u = 0; u < UNROLL; u++) acc ^= v[u];
    }
    for (; i < n16; i += nth) acc ^= __builtin_nontemporal_load(p + i);
  } else {
    const size_t nwaves = nth / 64, wave = tid / 64, lane = tid % 64;
    const size_t per = (n16 / 64 + nwaves - 1) / nwaves;  // 1 KiB rows per wave
    const size_t r0 = wave * per, r1 = r0 + per < n16 / 64 ? r0 + per : n16 / 64;
    size_t r = r0;
    for (; r + UNROLL <= r1; r += UNROLL) {
      u4 v[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; u++) v[u] = __builtin_nontemporal_load(p + (r + u) * 64 + lane);
#pragma unroll
      for (int u = 0; u < UNROLL; u++) acc ^= v[u];
    }
    for (; r < r1; r++) acc ^= __builtin_nontemporal_load(p + r * 64 + lane);
  }
  out[tid] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// the same read with a large straight-line code footprint in front (instruction-fetch cost of a big kernel)
template <int JUNK>
__global__ void read_kernel_big(const u4* __restrict__ p, size_t n16, unsigned* out) {
  unsigned x = threadIdx.x;
#pragma unroll
  for (int i = 0; i < JUNK; i++) asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(x) : "v"(i));
  u4 acc = {x, 0u, 0u, 0u};
  const size_t tid = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const size_t nth = size_t(gridDim.x) * blockDim.x;
  for (size_t i = tid; i < n16; i += nth) acc ^= __builtin_nontemporal_load(p + i);
  out[tid] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int JUNK>
static void time_big(char* buf, size_t bytes, int copies, unsigned* out, hipStream_t st) {
  const int reps = 64;
  hipGraph_t graph;
  hipGraphExec_t exec;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL(read_kernel_big<JUNK>, dim3(512), dim3(256), 0, st,
                       reinterpret_cast<const u4*>(buf + size_t(r % copies) * bytes), bytes / 16, out);
  CK(hipStreamEndCapture(st, &graph));
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  CK(hipGraphLaunch(exec, st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < 3; i++) CK(hipGraphLaunch(exec, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / (3 * reps);
  printf("  code-footprint %6d B junk: %8.2f us  %7.1f GB/s\n", JUNK * 8, us, bytes / us / 1e3);
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
}

int main(int argc, char** argv) {
  const size_t pool = size_t(1536) << 20;
  char* buf;
  unsigned* out;
  CK(hipMalloc(&buf, pool));
  CK(hipMalloc(&out, size_t(64) << 20));
  CK(hipMemset(buf, 1, pool));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const double sizes_mb[] = {8.67, 26.0, 46.6, 23.3, 67.7};
  const int grids[][2] = {{256, 256}, {256, 512}, {256, 1024}, {512, 256}, {512, 512}, {1024, 256}, {2048, 256},
                          {4096, 256}};
  if (argc > 1 && argv[1][0] == 'o') {  // one configuration (profiling): 8.67 MB, per-wave rows, 256 x 512
    const size_t bytes = size_t(8.67e6) & ~size_t(1023);
    const int copies = int(pool / bytes);
    for (int r = 0; r < 64; r++)
      hipLaunchKernelGGL(read_kernel<4>, dim3(256), dim3(512), 0, st,
                         reinterpret_cast<const u4*>(buf + size_t(r % copies) * bytes), bytes / 16, out, 1);
    CK(hipStreamSynchronize(st));
    return 0;
  }
  if (argc > 1) {  // instruction-footprint experiment only
    const size_t bytes = size_t(8.67e6) & ~size_t(1023);
    const int copies = int(pool / bytes);
    printf("== %.2f MB, grid 512 x 256, straight-line junk in front of the read\n", bytes / 1e6);
    time_big<1>(buf, bytes, copies, out, st);
    time_big<512>(buf, bytes, copies, out, st);
    time_big<1024>(buf, bytes, copies, out, st);
    time_big<2048>(buf, bytes, copies, out, st);
    time_big<4096>(buf, bytes, copies, out, st);
    time_big<8192>(buf, bytes, copies, out, st);
    return 0;
  }
  for (double mb : sizes_mb) {
    const size_t bytes = (size_t(mb * 1e6) + 1023) & ~size_t(1023);
    const size_t n16 = bytes / 16;
    const int copies = int(pool / bytes);
    printf("== %.2f MB (%d rotating copies)\n", bytes / 1e6, copies);
    for (int mode = 0; mode < 2; mode++) {
      for (auto& g : grids) {
        const int reps = 64;
        hipGraph_t graph;
        hipGraphExec_t exec;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int r = 0; r < reps; r++)
          hipLaunchKernelGGL(read_kernel<4>, dim3(g[0]), dim3(g[1]), 0, st,
                             reinterpret_cast<const u4*>(buf + size_t(r % copies) * bytes), n16, out, mode);
        CK(hipStreamEndCapture(st, &graph));
        CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
        CK(hipGraphLaunch(exec, st));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < 3; i++) CK(hipGraphLaunch(exec, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / (3 * reps);
        printf("  %s grid %5d x %4d: %8.2f us  %7.1f GB/s\n", mode ? "per-wave  " : "grid-strd ", g[0], g[1], us,
               bytes / us / 1e3);
        CK(hipGraphExecDestroy(exec));
        CK(hipGraphDestroy(graph));
        CK(hipEventDestroy(e0));
        CK(hipEventDestroy(e1));
      }
    }
  }
  return 0;
}
