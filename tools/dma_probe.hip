// dma_probe.hip -- development calibration tool (not part of the product): the LDS-DMA weight-stream rate of the
// decode engine's loader shape, with nothing else on the CU.  One 1 KiB buffer_load_dwordx4 ... lds per 64 lanes, fills
// of 16 such pieces (16 KiB), one workgroup per CU (160 KiB LDS request), NL loader waves each keeping D fills in
// flight (counted vmcnt), no consumers.  Patterns: 0 = each workgroup streams its own contiguous region (the engine's
// stripe runs), 1 = fill f of workgroup b at (f * grid + b) * 16 KiB (neighbouring CUs read neighbouring fills).
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/dma_probe tools/dma_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef __attribute__((address_space(3))) void lds_void_t;
constexpr int kFill = 16384;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int D, int NL, int AUX, int PAT, int PIECE>
__global__ __launch_bounds__(NL * 64) void dma_kernel(const char* buf, long long per_wg, int nfill, unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(buf), 0, 0x7FFFFFFF, 0x00020000);
  constexpr int IPF = kFill / (64 * PIECE);  // DMA instructions per fill
  char* ring = smem + w * D * kFill;
  int issued = 0;
  for (int f = w; f < nfill; f += NL) {
    long long off = PAT == 0 ? blockIdx.x * per_wg + (long long)f * kFill
                             : ((long long)f * gridDim.x + blockIdx.x) * kFill;
    // the buffer offset is 32-bit: fold the high part into the base per fill
    const auto rf = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(buf) + off, 0, kFill, 0x00020000);
    (void)rs;
    char* sb = ring + (issued % D) * kFill;
    if (issued >= D) wait_vm<(D - 1) * IPF>();
#pragma unroll
    for (int i = 0; i < IPF; i++)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rf, (lds_void_t*)(sb + i * 1024), 16, i * 1024 + lane * 16, 0,
                                               0, AUX);
    issued++;
  }
  wait_vm<0>();
  if (threadIdx.x == 0) out[blockIdx.x] = *reinterpret_cast<unsigned*>(smem);
}

template <int D, int NL, int AUX, int PAT, int PIECE = 16>
static void run(const char* name, char* buf, size_t pool, unsigned* out, hipStream_t st, int grid) {
  const size_t per_launch = size_t(512) << 20;
  const int nfill = int(per_launch / grid / kFill);
  const long long per_wg = (long long)nfill * kFill;
  const int copies = int(pool / per_launch);
  auto k = dma_kernel<D, NL, AUX, PAT, PIECE>;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const int reps = 12;
  for (int r = 0; r < 2; r++)
    hipLaunchKernelGGL(k, dim3(grid), dim3(NL * 64), 160 * 1024, st, buf + size_t(r % copies) * per_launch, per_wg,
                       nfill, out);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL(k, dim3(grid), dim3(NL * 64), 160 * 1024, st, buf + size_t(r % copies) * per_launch, per_wg,
                       nfill, out);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double bytes = double(nfill) * kFill * grid;
  printf("  %-44s %8.1f us  %7.1f GB/s  (%.1f GB/s per CU)\n", name, us, bytes / us / 1e3, bytes / us / 1e3 / grid);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const size_t pool = size_t(3) << 30;
  char* buf;
  unsigned* out;
  CK(hipMalloc(&buf, pool));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(buf, 1, pool));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("== LDS-DMA stream, %d workgroups (one per CU), 512 MB per launch, cold (3 GB pool)\n", cus);
  if (getenv("DMA_PROBE_ALL")) {
    run<1, 1, 2, 0>("1 wave, 1 fill in flight, nt, contiguous", buf, pool, out, st, cus);
    run<2, 1, 2, 0>("1 wave, 2 fills, nt, contiguous", buf, pool, out, st, cus);
    run<3, 1, 2, 0>("1 wave, 3 fills, nt, contiguous", buf, pool, out, st, cus);
    run<3, 1, 0, 0>("1 wave, 3 fills, default, contiguous", buf, pool, out, st, cus);
    run<3, 1, 2, 1>("1 wave, 3 fills, nt, interleaved", buf, pool, out, st, cus);
    run<3, 2, 2, 1>("2 waves x 3 fills, nt, interleaved", buf, pool, out, st, cus);
    run<2, 4, 2, 1>("4 waves x 2 fills, nt, interleaved", buf, pool, out, st, cus);
    run<1, 8, 2, 1>("8 waves x 1 fill, nt, interleaved", buf, pool, out, st, cus);
  }
  run<1, 2, 2, 0>("2 waves x 1 fill, nt, contiguous", buf, pool, out, st, cus);
  run<2, 2, 2, 0>("2 waves x 2 fills, nt, contiguous", buf, pool, out, st, cus);
  run<3, 2, 2, 0>("2 waves x 3 fills, nt, contiguous", buf, pool, out, st, cus);
  run<3, 2, 0, 0>("2 waves x 3 fills, default, contiguous", buf, pool, out, st, cus);
  run<1, 3, 2, 0>("3 waves x 1 fill, nt, contiguous", buf, pool, out, st, cus);
  run<2, 3, 2, 0>("3 waves x 2 fills, nt, contiguous", buf, pool, out, st, cus);
  run<1, 4, 2, 0>("4 waves x 1 fill, nt, contiguous", buf, pool, out, st, cus);
  run<2, 4, 2, 0>("4 waves x 2 fills, nt, contiguous", buf, pool, out, st, cus);
  run<1, 6, 2, 0>("6 waves x 1 fill, nt, contiguous", buf, pool, out, st, cus);
  return 0;
}
