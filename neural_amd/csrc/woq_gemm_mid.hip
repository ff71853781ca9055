// woq_gemm_mid.hip -- the mid-M (17 <= M <= 64) WOQ GEMM for gfx950: one launch, every operand straight to registers.
//
// Replaces LauncherBase::gemm / run_block for batched-decode sized M (bestla/bestla/bestla_wrapper.h:471-542, the
// 2-D scheduler's cache-blocked per-thread tiles, bestla_parallel.h:421-583) where the prefill GEMMs' 256 x 128 tiles
// leave the chip idle and their split-K reduce is a second launch.
//
// Shape of the work (mid-M).  The weight bytes are what a launch of this size must move (M = 64 at
// K = N = 4096: 8.4 MB of int4 against 0.5 MB of fp16 activations), so every CU streams an equal, distinct slice of them:
// a workgroup owns S stripes (16 columns each) x a run of K tiles, the runs of one stripe group (ks of them) together
// cover K.  Its waves split the run's K tiles (wave w: tiles w, w + NW, ...; SPW stages each) and every wave covers all
// the workgroup's stripes and all M rows, so each weight byte and each activation byte is loaded exactly once per
// workgroup -- no LDS staging, no barrier in front of the arithmetic: a wave issues every load of all its stages at
// once (weights non-temporal, raw buffer loads, out-of-range offsets for rows >= M / tiles past the run: zeros, no
// branches), then dequantizes and multiplies (v_mfma_f32_16x16x32_f16 with the weights as the A operand and the
// activation rows as B, so C^T comes out with 4 consecutive columns of one row per lane; the group scale applied to an
// fp32 group partial exactly as the decode GEMV does).  The waves' partial tiles meet once in
// LDS (summed in wave order).  With ks > 1 each run's tile goes out as an fp32 slab and launch_splitk_reduce sums
// the runs in order.  (An in-launch combine -- write-through slabs, an arrival ticket per stripe group, the last run
// sums -- measured 0.4-1.5 us SLOWER per launch than the reduce launch at M = 17 .. 64: the ticket round trip and the
// last run's dependent slab reads cost more than the kernel boundary; profiles/r05_mid_*.)
#include <hip/hip_runtime.h>

#include <cstdint>

#include "woq_device.h"
#include "woq_kernels.h"

namespace nad {
namespace mid {

// Development instrumentation (make trace -> libneural_amd_trace.so): per-workgroup wall-clock stamps of the phases,
// read back with nad_mid_trace_fetch().  Compiled out of the product library.
#ifdef NAD_PHASE_TRACE
constexpr int kTraceSlots = 8, kTraceMaxWg = 16384;
__device__ unsigned long long mid_trace_buf[kTraceSlots][kTraceMaxWg];
#define MID_TRACE(slot)                                                                                        \
  do {                                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < kTraceMaxWg) mid_trace_buf[slot][blockIdx.x] = wall_clock64();       \
  } while (0)
#define MID_TRACE_MAX(slot)                                                                                    \
  do {                                                                                                         \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < kTraceMaxWg)                                                   \
      atomicMax(&mid_trace_buf[slot][blockIdx.x], (unsigned long long)wall_clock64());                         \
  } while (0)
#else
#define MID_TRACE(slot) \
  do {                  \
  } while (0)
#define MID_TRACE_MAX(slot) \
  do {                      \
  } while (0)
#endif

constexpr int kOOB = 0x7FFF0000;  // a buffer offset past every resource: the load returns 0 and touches no memory
constexpr int kAuxNT = 2;         // non-temporal: the weights are read once

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, int(bytes), 0x00020000);
}
__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t m, uint32_t c) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(m), "v"(c));
  return r;
}
__device__ __forceinline__ h2_t splat(float v) {
  h2_t r;
  r[0] = _Float16(v);
  r[1] = _Float16(v);
  return r;
}
// int4: 8 nibbles -> exact fp16 (q - bias - zp) via the 0x6400 magic (woq_gemv.hip dequant4)
__device__ __forceinline__ h8_t dq4(uint32_t w, uint32_t m0, uint32_t mag, h2_t s16, h2_t c0, h2_t c1) {
  const uint32_t w8 = w >> 8, m1 = m0 << 4;
  const h2_t p0 = as_h2(and_or(w, m0, mag)) + c0;
  const h2_t p1 = __builtin_elementwise_fma(as_h2(and_or(w, m1, mag)), s16, c1);
  const h2_t p2 = as_h2(and_or(w8, m0, mag)) + c0;
  const h2_t p3 = __builtin_elementwise_fma(as_h2(and_or(w8, m1, mag)), s16, c1);
  h8_t r;
  r[0] = p0[0];
  r[1] = p0[1];
  r[2] = p1[0];
  r[3] = p1[1];
  r[4] = p2[0];
  r[5] = p2[1];
  r[6] = p3[0];
  r[7] = p3[1];
  return r;
}
// the group scales of a lane's 4 output columns: 4 fp32, or 4 fp16 / bf16 in two dwords (the 16-bit types share code,
// selected per launch)
template <bool F32>
__device__ __forceinline__ f4_t scale4(const u4_t& x, bool bf16) {
  if constexpr (F32) return __builtin_bit_cast(f4_t, x);
  f4_t r;
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const uint32_t h = (x[e >> 1] >> ((e & 1) * 16)) & 0xFFFFu;
    r[e] = bf16 ? __uint_as_float(h << 16) : f16_bits_to_f32(uint16_t(h));
  }
  return r;
}
// 8 activations (raw 16 or 32 bytes) -> the fp16 fragment; fp32 / bf16 values split as hi = fp16(a), lo = fp16(a - hi)
// (two MFMAs: products accurate to fp32, as the decode GEMV does)
__device__ __forceinline__ float a_val(int at, const u4_t& x0, const u4_t& x1, int e) {
  if (at == kActF32) return __uint_as_float(e < 4 ? x0[e] : x1[e - 4]);
  const uint32_t w = x0[e >> 1];
  return __uint_as_float((e & 1) ? (w & 0xFFFF0000u) : (w << 16));
}
template <int AT>
__device__ __forceinline__ void a_frag(const u4_t& x0, const u4_t& x1, h8_t& hi, h8_t& lo) {
  if constexpr (AT == kActF16) {
    hi = __builtin_bit_cast(h8_t, x0);
  } else {
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const float f = a_val(AT, x0, x1, e);
      hi[e] = _Float16(f);
      lo[e] = _Float16(f - float(hi[e]));
    }
  }
}

// BITS 4 / 2 (K tile 128 / 256), GPT groups per K tile (1, 2, 4), RF row fragments (M <= 16 RF), S stripes per
// workgroup, NW waves, SPW stages (K tiles) per wave, SF32 fp32 scales (else fp16 / bf16).
template <int BITS, int GPT, bool ASYM, int AT, int RF, int S, int NW, int SPW, bool SF32>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW / 4, NW / 4))) void woq_mid_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KT = BITS == 4 ? 128 : 256, SPT = KT / 32, SPG = SPT / GPT;
  constexpr int BIAS = BITS == 4 ? 8 : 2;
  constexpr int AL = AT == kActF32 ? 2 : 1;  // 16-B loads per 8 activations
  constexpr int ESZ = AT == kActF32 ? 4 : 2;
  static_assert(SPT % GPT == 0, "groups must tile the K tile");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const SkinnyWeight& W = a.w;
  const int M = a.M, nt = W.nt, ng = W.ng, ns = W.ns;
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  const int bid = blockIdx.x;
  // round-robin placement puts workgroup b on XCD b % 8: with xcd_sg the runs of stripe group sg all go to XCD sg % 8
  // (the groups of the last incomplete round of 8 as before), so the reduce finds their slabs in that XCD's L2
  const int x8 = (a.xcd_sg >> 3) << 3, full = x8 * ks;
  int r, sg;
  if (bid < full) {
    r = (bid >> 3) % ks;
    sg = ((bid >> 3) / ks) * 8 + (bid & 7);
  } else {
    r = (bid - full) % ks;
    sg = x8 + (bid - full) / ks;
  }
  const int t0 = r * a.ktiles;
  const int t1 = min(nt, t0 + a.ktiles);
  const int tsh = a.tpg_shift;

  MID_TRACE(0);
  const auto rt = rsrc(W.tiles, uint32_t(ns) * nt * 1024u);
  const bool sbf16 = a.scale_t == kScaleBF16;
  const auto rs = rsrc(W.scales, uint32_t(ns) * ng * 16u * (SF32 ? 4u : 2u));
  const auto rz = rsrc(W.zps, ASYM ? uint32_t(ns) * ng * 16u : 0u);
  const auto ra = rsrc(a.A, uint32_t(M - 1) * a.lda * ESZ + uint32_t(a.K) * ESZ);
  const int rowb = SF32 ? 64 : 32;  // bytes per scale row of 16 columns
  const int vs = (lane >> 4) * (SF32 ? 16 : 8);  // this lane's 4 output columns (4 (lane >> 4) .. + 3)

  const uint32_t m0 = __builtin_amdgcn_readfirstlane(0x000F000Fu), mag = __builtin_amdgcn_readfirstlane(0x64006400u);
  const h2_t s16 = splat(1.f / 16.f);
  const h2_t zc0 = splat(-(1024.f + BIAS)), zc1 = splat(-(64.f + BIAS));
  f4_t acc[RF][S];
#pragma unroll
  for (int i = 0; i < RF; i++)
#pragma unroll
    for (int s = 0; s < S; s++) acc[i][s] = f4_t{0.f, 0.f, 0.f, 0.f};

  // the run in chunks of NW * SPW K tiles (one chunk when the host sized the run to it)
  for (int tc = t0; tc < t1; tc += NW * SPW) {
  // 1) every load of every stage of the chunk, back to back
  u4_t bw[SPW][S];
  u4_t sc[SPW][S][GPT];  // the 4 scales of this lane's output columns (fp32: 4 dwords; 16-bit: the first 2)
  int zp[SPW][S][GPT];
  u4_t av[SPW][RF][SPT][AL];
#pragma unroll
  for (int j = 0; j < SPW; j++) {
    const int t = tc + j * NW + wave;
    const bool live = t < t1;
#pragma unroll
    for (int s = 0; s < S; s++) {
      const int stripe = sg * S + s;
      const bool sl = live && stripe < ns;
      bw[j][s] = __builtin_bit_cast(
          u4_t, __builtin_amdgcn_raw_buffer_load_b128(rt, sl ? (stripe * nt + t) * 1024 + lane * 16 : kOOB, 0, kAuxNT));
#pragma unroll
      for (int g = 0; g < GPT; g++) {
        const int grp = GPT == 1 ? (t >> tsh) : t * GPT + g;
        const bool gl = sl && (GPT == 1 || grp < ng);
        const int row = stripe * ng + grp;
        if constexpr (SF32) {
          sc[j][s][g] = __builtin_bit_cast(u4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, gl ? row * rowb + vs : kOOB, 0, 0));
        } else {
          const auto h = __builtin_amdgcn_raw_buffer_load_b64(rs, gl ? row * rowb + vs : kOOB, 0, 0);
          sc[j][s][g] = u4_t{h[0], h[1], 0u, 0u};
        }
        if constexpr (ASYM)
          zp[j][s][g] = int(int8_t(__builtin_amdgcn_raw_buffer_load_b8(rz, gl ? row * 16 + (lane & 15) : kOOB, 0, 0)));
        else
          zp[j][s][g] = 0;
      }
    }
#pragma unroll
    for (int i = 0; i < RF; i++) {
      const int row = i * 16 + (lane & 15);
#pragma unroll
      for (int d = 0; d < SPT; d++) {
        const int k = t * KT + d * 32 + (lane >> 4) * 8;
        const int off = (live && row < M && k < a.K) ? (row * a.lda + k) * ESZ : kOOB;
#pragma unroll
        for (int h = 0; h < AL; h++)
          av[j][i][d][h] = __builtin_bit_cast(u4_t, __builtin_amdgcn_raw_buffer_load_b128(ra, off + h * 16, 0, 0));
      }
    }
  }

  // every load is in flight before the first use (left alone, the scheduler sinks each load next to its MFMA and
  // serialises the latencies)
  __builtin_amdgcn_sched_barrier(0);
  MID_TRACE_MAX(1);
  // 2) dequantize + multiply: per (stripe, group) an fp32 partial of RF fragments, scaled into the stripe's sums
#pragma unroll
  for (int j = 0; j < SPW; j++) {
    if (tc + j * NW + wave >= t1) break;  // wave-uniform: past the run (its loads returned zeros)
#pragma unroll
    for (int s = 0; s < S; s++) {
      f4_t tmp[RF];
#pragma unroll
      for (int d = 0; d < SPT; d++) {
        const int g = d / SPG;
        h8_t bf;
        if constexpr (BITS == 4) {
          if constexpr (ASYM) {
            const float z = float(zp[j][s][g]);
            bf = dq4(bw[j][s][d], m0, mag, s16, zc0 - splat(z), zc1 - splat(z));
          } else {
            bf = dq4(bw[j][s][d], m0, mag, s16, zc0, zc1);
          }
        } else {
          bf = dequant2_step(bw[j][s], d, BIAS + zp[j][s][g]);
        }
#pragma unroll
        for (int i = 0; i < RF; i++) {
          h8_t af, afl;
          a_frag<AT>(av[j][i][d][0], av[j][i][d][AL - 1], af, afl);
          // operands swapped (C^T = B^T A^T): lane l gets rows 4 (l >> 4) .. + 3 of C^T = 4 consecutive columns
          tmp[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf, af, d % SPG == 0 ? f4_t{0.f, 0.f, 0.f, 0.f} : tmp[i], 0,
                                                          0, 0);
          if constexpr (AT != kActF16) tmp[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf, afl, tmp[i], 0, 0, 0);
        }
        if ((d + 1) % SPG == 0) {
          const f4_t scl = scale4<SF32>(sc[j][s][g], sbf16);
#pragma unroll
          for (int i = 0; i < RF; i++) acc[i][s] += tmp[i] * scl;
        }
      }
    }
  }

  }  // chunk
  MID_TRACE_MAX(2);

  // 3) the waves' partial tiles meet in LDS: slot (wave, i, s) in the MFMA layout, summed in wave order.  Lane l of a
  //    slot holds row 16 i + (l & 15), columns 16 s + 4 (l >> 4) .. + 3 of the workgroup's tile
  constexpr int SLOTS = RF * S, QT = (SLOTS + NW - 1) / NW;  // slots per thread
  f4_t* red = reinterpret_cast<f4_t*>(smem);
#pragma unroll
  for (int i = 0; i < RF; i++)
#pragma unroll
    for (int s = 0; s < S; s++) red[(wave * SLOTS + i * S + s) * 64 + lane] = acc[i][s];
  __syncthreads();
  f4_t v[QT];
  int orow[QT], ocol[QT];
  const int n0t = sg * S * 16;
#pragma unroll
  for (int u = 0; u < QT; u++) {
    const int q = u * NW * 64 + int(threadIdx.x);
    const int is = q >> 6, i = is / S, s = is - i * S;
    orow[u] = i * 16 + (lane & 15);
    ocol[u] = n0t + s * 16 + (lane >> 4) * 4;
    if (q < SLOTS * 64) {
      v[u] = red[q];
#pragma unroll
      for (int w = 1; w < NW; w++) v[u] += red[w * SLOTS * 64 + q];
    }
    if (q >= SLOTS * 64 || orow[u] >= M) orow[u] = -1;  // nothing to store
    if (ocol[u] >= W.n) orow[u] = -1;
  }
  MID_TRACE(3);

  // 4) epilogue / slab
  if (ks == 1) {
#pragma unroll
    for (int u = 0; u < QT; u++) {
      if (orow[u] < 0) continue;
      float o[4] = {v[u][0], v[u][1], v[u][2], v[u][3]};
      gemm_epilogue4(a, orow[u], ocol[u], o);
    }
    MID_TRACE(5);
    return;
  }
  // split K: this run's slab (part[(r * M + row) * ldp + n], ldp % 4 == 0); launch_splitk_reduce sums them
  const uint32_t slab = uint32_t(M) * a.ldp;  // floats per run
  const auto rp = rsrc(a.part, uint32_t(ks) * slab * 4u);
#pragma unroll
  for (int u = 0; u < QT; u++) {
    if (orow[u] < 0) continue;
    const uint32_t off = (uint32_t(r) * slab + uint32_t(orow[u]) * a.ldp + ocol[u]) * 4u;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, v[u]), rp, off, 0, 0);
  }
  MID_TRACE(5);
}

}  // namespace mid

#ifdef NAD_PHASE_TRACE
extern "C" int nad_mid_trace_fetch(void* host, size_t bytes, int clear) {
  const size_t n = sizeof(mid::mid_trace_buf) < bytes ? sizeof(mid::mid_trace_buf) : bytes;
  if (host && hipMemcpyFromSymbol(host, HIP_SYMBOL(mid::mid_trace_buf), n) != hipSuccess) return -1;
  if (clear) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(mid::mid_trace_buf)) != hipSuccess) return -1;
    if (hipMemset(p, 0, sizeof(mid::mid_trace_buf)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

int mid_lds_bytes(int rf, int s, int nw) { return nw * rf * s * 1024; }

// BITS / GPT / ASYM / AT / RF / S / NW / SPW dispatch (mid_geometry: what the host plans with)
template <int BITS, int GPT, bool ASYM, int AT, int RF, int S, int NW, int SPW>
static hipError_t mid_go(const GemmArgs& a, int grid, hipStream_t st) {
  const int lds = mid_lds_bytes(RF, S, NW);
  const bool f32 = a.scale_t == kScaleF32;
  auto k = f32 ? mid::woq_mid_kernel<BITS, GPT, ASYM, AT, RF, S, NW, SPW, true>
               : mid::woq_mid_kernel<BITS, GPT, ASYM, AT, RF, S, NW, SPW, false>;
  static bool attr[2] = {};  // opt in to > 64 KiB of dynamic LDS once per instantiation
  if (!attr[f32] && lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       lds);
    if (e != hipSuccess) return e;
    attr[f32] = true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), lds, st, a);
  return hipGetLastError();
}

// Geometry per format: 4 stripes per workgroup; int4 with one group per K tile or more: 8 waves x 1 stage (K tile)
// each (round 6), except fp32 / bf16 rows at M > 48, whose raw rows, hi / lo fragments and 64 accumulators need more
// than two waves' register budget: 4 waves (one per SIMD) x 2 stages; groups of half a tile: 8 x 1 to M = 32, then 4
// waves x 1 (their scale / zero-point registers); groups of a quarter tile: 4 waves x 2 stages; int2 (256-deep tiles, 8 steps of activation fragments per stage)
// 4 x 1.  Not taken: int2 at M > 32, int4 with 4 groups per tile (g32) at M > 32.
void mid_geometry(int bits, int gpt, int act_t, int rf, int wide, int* s, int* nw, int* spw) {
  *nw = 4;
  // 8 stripes x a 512-deep run: half the activation bytes per column.  Not at 3 / 4 row fragments: measured 1.1-1.3 us
  // SLOWER than 4 stripes at M = 33 .. 64, N = 4096 (no spills; the doubled slabs outweigh the halved activation bytes;
  // profiles/r06_mid_wide_ab.txt)
  if (wide && bits == 4 && rf <= 2 && gpt <= 2) {
    *s = 8;
    *spw = 1;
    // 8 waves (measured N = 11008: fp16 M = 16 / 32 14.9 / 18.7 -> 13.1 / 15.6 us, fp32 15.7 / 21.6 -> 15.2 / 19.6;
    // profiles/r06_mid_8waves_ab.txt), except g64 at 2 row fragments (its scale registers spill)
    if (gpt == 1 || rf == 1) *nw = 8;
    return;
  }
  *s = 4;
  // int4 with one group per K tile or more: 8 waves x 1 stage -- the same 8-tile chunk as 4 waves x 2 stages, the
  // loads and the dequant / MFMA of a chunk spread over two waves per SIMD (fp16 rows M = 12 / 32 / 64 7.71 / 9.44 /
  // 12.62 -> 7.65 / 9.22 / 12.12 us; fp32 M = 48 15.2 -> 13.8; profiles/r06_mid_8waves_ab.txt); not for fp32 / bf16 rows
  // at 4 row fragments (their hi / lo stage spills at two waves per SIMD: fp32 M = 64 19.2 -> 20.0 us)
  // ... and int4 groups of half a tile (g64) at M <= 32 (M = 24 / 32: fp16 9.68 / 9.94 -> 9.29 / 9.64 us, fp32 12.09 /
  // 12.63 -> 11.23 / 11.73; profiles/r06_mid_8waves_ab.txt; beyond 2 row fragments their scale registers spill)
  if (bits == 4 && gpt == 2 && rf <= 2) {
    *nw = 8;
    *spw = 1;
    return;
  }
  if (bits == 4 && gpt == 1 && (rf <= 3 || act_t == kActF16)) {
    *nw = 8;
    *spw = 1;
    return;
  }
  *spw = bits == 4 && (rf <= 2 || gpt == 1) ? 2 : 1;
}

template <int BITS, int GPT, bool ASYM, int AT>
static hipError_t mid_rf(const GemmArgs& a, int rf, int s, int grid, hipStream_t st) {
  if constexpr (BITS == 4) {
    constexpr int SPW3 = GPT == 1 ? 2 : 1;  // M > 32
    if constexpr (GPT <= 2) {
      if (s == 8 && rf == 1) return mid_go<BITS, GPT, ASYM, AT, 1, 8, 8, 1>(a, grid, st);
      if (s == 8 && rf == 2) {
        if constexpr (GPT == 1) return mid_go<BITS, GPT, ASYM, AT, 2, 8, 8, 1>(a, grid, st);
        return mid_go<BITS, GPT, ASYM, AT, 2, 8, 4, 1>(a, grid, st);
      }
    }
    if (s != 4) return hipErrorInvalidValue;
    if constexpr (GPT <= 2) {  // 8 waves x 1 stage (mid_geometry)
      if (rf == 1) return mid_go<BITS, GPT, ASYM, AT, 1, 4, 8, 1>(a, grid, st);
      if (rf == 2) return mid_go<BITS, GPT, ASYM, AT, 2, 4, 8, 1>(a, grid, st);
    }
    if constexpr (GPT == 1) {
      if (rf == 3) return mid_go<BITS, GPT, ASYM, AT, 3, 4, 8, 1>(a, grid, st);
      if constexpr (AT == kActF16) {  // fp32 / bf16 rows at 4 row fragments: 4 waves (their hi / lo stage spills)
        if (rf == 4) return mid_go<BITS, GPT, ASYM, AT, 4, 4, 8, 1>(a, grid, st);
      }
    }
    switch (rf) {
      case 1:
        return mid_go<BITS, GPT, ASYM, AT, 1, 4, 4, 2>(a, grid, st);
      case 2:
        return mid_go<BITS, GPT, ASYM, AT, 2, 4, 4, 2>(a, grid, st);
      default:
        if constexpr (GPT == 4) {
          return hipErrorInvalidValue;  // g32 at M > 32: not taken (run_mid)
        } else {
          return rf == 3 ? mid_go<BITS, GPT, ASYM, AT, 3, 4, 4, SPW3>(a, grid, st)
                         : mid_go<BITS, GPT, ASYM, AT, 4, 4, 4, SPW3>(a, grid, st);
        }
    }
  } else {
    // int2 (8 steps of activation fragments per 256-deep stage): M <= 32 only (run_mid)
    if (s != 4) return hipErrorInvalidValue;
    return rf == 1 ? mid_go<BITS, GPT, ASYM, AT, 1, 4, 4, 1>(a, grid, st)
                   : mid_go<BITS, GPT, ASYM, AT, 2, 4, 4, 1>(a, grid, st);
  }
}

template <int BITS, int GPT, bool ASYM>
static hipError_t mid_at(const GemmArgs& a, int act_t, int rf, int s, int grid, hipStream_t st) {
  if (act_t == kActF16) return mid_rf<BITS, GPT, ASYM, kActF16>(a, rf, s, grid, st);
  if (act_t == kActBF16) return mid_rf<BITS, GPT, ASYM, kActBF16>(a, rf, s, grid, st);
  return mid_rf<BITS, GPT, ASYM, kActF32>(a, rf, s, grid, st);
}

hipError_t launch_gemm_mid(const GemmArgs& a, int bits, int gpt, int act_t, int rf, int s, int grid, hipStream_t st) {
  const bool asym = a.w.zps != nullptr;
  if (bits == 4) {
    if (gpt == 1)
      return asym ? mid_at<4, 1, true>(a, act_t, rf, s, grid, st) : mid_at<4, 1, false>(a, act_t, rf, s, grid, st);
    if (gpt == 2)
      return asym ? mid_at<4, 2, true>(a, act_t, rf, s, grid, st) : mid_at<4, 2, false>(a, act_t, rf, s, grid, st);
    return asym ? mid_at<4, 4, true>(a, act_t, rf, s, grid, st) : mid_at<4, 4, false>(a, act_t, rf, s, grid, st);
  }
  if (gpt == 1) return asym ? mid_at<2, 1, true>(a, act_t, rf, s, grid, st) : mid_at<2, 1, false>(a, act_t, rf, s, grid, st);
  if (gpt == 2) return asym ? mid_at<2, 2, true>(a, act_t, rf, s, grid, st) : mid_at<2, 2, false>(a, act_t, rf, s, grid, st);
  return asym ? mid_at<2, 4, true>(a, act_t, rf, s, grid, st) : mid_at<2, 4, false>(a, act_t, rf, s, grid, st);
}

}  // namespace nad
