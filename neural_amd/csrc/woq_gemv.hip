// woq_gemv.hip -- the decode (M <= 16) weight-only-quantized GEMV for gfx950: a persistent stripe stream.
//
// Replaces GEMVWrapper::gemv_kblock -> gemv_{4,2}bit_fp32_fp32 (bestla/bestla/bestla_wrapper.h:364-468,
// bestla/bestla/kernel_ref.h:2489-2531,2712-2760) and the fused QKV / FFN-gate-up decode launches
// (neural_speed/core/layers/ip_fusion_qkv.cpp:22-93, ip_fusion_ffn.cpp:407-457).
//
// Shape of the work.  A launch streams `units` stripes (16 output columns x all of K; for the dual SiLU*mul / GELU*mul
// epilogue a unit is the pair {gate stripe s, up stripe s}).  The grid is sized to the chip (one workgroup per CU),
// each workgroup owns a contiguous, balanced run of whole units, and its waves split the run's concatenated 1 KiB tiles
// evenly -- a wave's range may cross stripe boundaries.
//
// What the measurements on MI355X (tools/gemv_sweep.py, tools/hbm_probe.hip) shaped:
//   * a launch of this size is dominated by fixed costs, not arithmetic: everything before the first weight load and
//     every instruction executed once per launch shows up directly in the time.  So the prologue issues the
//     activation, scale and weight loads back to back with no waits in between, all bookkeeping is wave-uniform SALU
//     work (a cursor advanced per tile, the weight / stripe re-derived only at stripe boundaries), and the weight loads
//     are raw buffer loads that are never predicated -- tiles past a wave's range get an out-of-range offset, which
//     returns zeros without touching memory -- so every pipeline stage has the same vmcnt footprint and hipcc waits for
//     exactly one stage instead of draining the queue at control-flow joins;
//   * the activations are staged into LDS once per workgroup as MFMA-ready fp16 rows (fp32/bf16 inputs split
//     hi = fp16(a), lo = fp16(a - hi) so the products are fp32-accurate; the act-order gather of
//     ShuffleActivationKBlock, bestla_prologue_a.h:407-422, is applied while staging), and the workgroup's group scales
//     loads of each stage are issued with it (one dword per tile: L2-merged 32 B rows);
//   * wave w owns K-slices w, w + NW, ... (KS = 4 tiles) of every stripe in the run: a pipeline stage is one
//     (stripe, slice) -- four loads at immediate offsets from one base -- and NST stages are in flight per wave
//     (register ring, 1 or 3 chosen per launch: see NST below), the stage being computed the oldest;
//   * int4 dequantization takes 1 shift + 4 v_and_or + 4 packed fp16 ops per 8 weights (the 0x6400 magic makes
//     1024 + q and 1024 + 16 q exact fp16 without per-nibble shifts), then one
//     v_mfma_f32_16x16x32_f16 with the activation rows in the A operand; the group scale multiplies an fp32 group
//     accumulator once per group, so the weights are dequantized exactly;
//   * a wave's partial sum per stripe goes to an LDS slot; after ONE barrier the workgroup sums the slots of each
//     stripe in wave order (deterministic, no atomics) and applies the fused epilogue.
// HBM-bound by design: weights + scales are read exactly once; the only other traffic is A (L2-resident) once per WG.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "woq_device.h"
#include "woq_kernels.h"

namespace nad {

// ------------------------------------------------------------------------------------------------ phase trace
// Development instrumentation (make trace -> libneural_amd_trace.so): per-workgroup wall-clock stamps of the
// GEMV kernel's phases, read back with nad_trace_fetch().  Compiled out of the product library.
#ifdef NAD_PHASE_TRACE
constexpr int kTraceSlots = 8, kTraceMaxWg = 16384;
__device__ unsigned long long nad_trace_buf[kTraceSlots][kTraceMaxWg];
#define NAD_TRACE(slot)                                                                       \
  do {                                                                                        \
    if (threadIdx.x == 0 && blockIdx.x < kTraceMaxWg) nad_trace_buf[slot][blockIdx.x] = wall_clock64(); \
  } while (0)
#define NAD_TRACE_MAX(slot)                                                                               \
  do {                                                                                                    \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < kTraceMaxWg)                                              \
      atomicMax(&nad_trace_buf[slot][blockIdx.x], (unsigned long long)wall_clock64());                    \
  } while (0)
#else
#define NAD_TRACE(slot) \
  do {                  \
  } while (0)
#define NAD_TRACE_MAX(slot) \
  do {                      \
  } while (0)
#endif

// M = 1 kernel tail: partial-sum slots laid out per column so a 16-wave launch reduces with four 16-B LDS reads per
// output and no per-slot clamps (the general form's 16 clamped offsets + masks are ~100 scalar instructions executed
// once per launch, cold in the instruction cache: ~0.4 us per KB).  Measured (profiles/r06_gemv_tail_ab.txt, same
// box, alternating): O 4.80 -> 4.55 us, decode 946-951 -> 969-972 tok/s; bit-identical sums (same order).  A
// branch-free first weight stage (the two-armed load_stage makes hipcc wait vmcnt(0) for the activation loads before
// the first weight load) measured neutral (943-947 tok/s) and was not kept.
#ifndef NAD_GEMV_LEAN_TAIL
#define NAD_GEMV_LEAN_TAIL 1
#endif

constexpr int kOOB = 0x7FFF0000;  // a buffer offset past every resource: the load returns 0 and touches no memory

// virtual stripe -> (weight index, stripe within that weight); all wave-uniform
__device__ __forceinline__ void vstripe(const GemvArgs& a, int v, int& w, int& s) {
  if (a.dual) {
    w = v & 1;
    s = v >> 1;
  } else {
    w = (v >= a.stripe_base[1] ? 1 : 0) + (v >= a.stripe_base[2] ? 1 : 0);
    s = v - (w == 0 ? 0 : (w == 1 ? a.stripe_base[1] : a.stripe_base[2]));
  }
}

template <class T>
__device__ __forceinline__ T sel3(int w, T x0, T x1, T x2) {
  return w == 0 ? x0 : (w == 1 ? x1 : x2);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}

// ------------------------------------------------------------------------------------------------ weight stream
// Wave w owns the K-slices q = w, w + NW, w + 2 NW, ... (KS consecutive tiles each) of EVERY stripe of the workgroup's
// run, visited stripe-major.  One pipeline stage is one (stripe, slice): KS tile loads at immediate offsets from one
// stripe base, plus the slice's group scales / zero points -- a few SALU ops per stage, nothing per tile.
constexpr int KS = 4;

struct StageCursor {
  int j, q;                      // local virtual stripe, K-slice
  int s;                         // stripe within its weight
  __amdgpu_buffer_rsrc_t rt, rs, rz;
};

__device__ __forceinline__ void cursor_stripe(const GemvArgs& a, StageCursor& c, int v0) {
  int w, s;
  vstripe(a, v0 + c.j, w, s);
  const int ns = sel3(w, a.w[0].ns, a.w[1].ns, a.w[2].ns);
  const int ssz = a.scale_t == kScaleF32 ? 4 : 2;
  c.s = s;
  c.rt = rsrc(sel3(w, a.w[0].tiles, a.w[1].tiles, a.w[2].tiles), ns * a.nt * 1024);
  c.rs = rsrc(sel3(w, a.w[0].scales, a.w[1].scales, a.w[2].scales), ns * a.ng * 16 * ssz);
  c.rz = rsrc(sel3(w, a.w[0].zps, a.w[1].zps, a.w[2].zps), ns * a.ng * 16);
}

template <int GPT, int KSN = KS>
struct StageRegs {
  u4_t b[KSN];
  uint32_t sc[KSN][GPT];  // raw scale bits (the dword holding this lane's 16-bit scale, or the f32)
  int zp[KSN][GPT];
};

#ifndef NAD_TILE_AUX
#define NAD_TILE_AUX 2  // non-temporal: the weights are read once per token
#endif
// Issue one stage's loads (never predicated: past-the-end tiles / stages get the out-of-range offset), then advance.
template <int GPT, bool ASYM, int KSN = KS>
__device__ __forceinline__ void load_stage(const GemvArgs& a, StageRegs<GPT, KSN>& S, StageCursor& c, int nv, int nsl,
                                           int wave, int NW, int v0, int lane, int vs) {
  if (c.j >= nv) {  // past this wave's last stage: the same loads, all out of range, no bookkeeping
#pragma unroll
    for (int i = 0; i < KSN; i++) {
      S.b[i] = __builtin_bit_cast(u4_t, __builtin_amdgcn_raw_buffer_load_b128(c.rt, kOOB, 0, NAD_TILE_AUX));
#pragma unroll
      for (int g = 0; g < GPT; g++) {
        S.sc[i][g] = __builtin_amdgcn_raw_buffer_load_b32(c.rs, kOOB, 0, 0);
        S.zp[i][g] = ASYM ? int(int8_t(__builtin_amdgcn_raw_buffer_load_b8(c.rz, kOOB, 0, 0))) : 0;
      }
    }
    return;
  }
  const int nt = a.nt, ng = a.ng;
  const bool over = false;
  const int t0 = c.q * KSN;
  const int tb = (c.s * nt + t0) * 1024;
  const int rowb = a.scale_t == kScaleF32 ? 64 : 32;  // bytes per scale row of 16
#pragma unroll
  for (int i = 0; i < KSN; i++) {
    const bool live = !over && t0 + i < nt;
    S.b[i] = __builtin_bit_cast(u4_t, __builtin_amdgcn_raw_buffer_load_b128(c.rt, (live ? tb + i * 1024 : kOOB) + lane * 16, 0, NAD_TILE_AUX));
#pragma unroll
    for (int g = 0; g < GPT; g++) {
      const int grp = GPT == 1 ? ((t0 + i) >> a.tpg_shift) : (t0 + i) * GPT + g;
      const bool gl = live && (GPT == 1 || grp < ng);
      const int row = c.s * ng + grp;
      S.sc[i][g] = __builtin_amdgcn_raw_buffer_load_b32(c.rs, (gl ? row * rowb : kOOB) + vs, 0, 0);
      if constexpr (ASYM)
        S.zp[i][g] = int(int8_t(__builtin_amdgcn_raw_buffer_load_b8(c.rz, (gl ? row * 16 : kOOB) + (lane & 15), 0, 0)));
      else
        S.zp[i][g] = 0;
    }
  }
  c.q += NW;
  if (c.q >= nsl) {
    c.q = wave;
    c.j++;
    if (c.j < nv)
      cursor_stripe(a, c, v0);
    else
      c.rt = c.rs = c.rz = rsrc(a.w[0].tiles, 0);
  }
}

// ------------------------------------------------------------------------------------------------ dequantization
// int4: the four nibble pairs of one MFMA step's dword as exact integer fp16 (q - zp).  The 0x6400 magic leaves the
// ten mantissa bits free, so a nibble can sit at bits 0-3 (value 1024 + q) or bits 4-7 (value 1024 + 16 q):
//   pair 0 = (w & 0x000F000F) | M          = 1024 + q     -> x - (1024 + 8 + zp)
//   pair 1 = (w & 0x00F000F0) | M          = 1024 + 16 q  -> x / 16 - (64 + 8 + zp)
//   pair 2 = ((w >> 8) & 0x000F000F) | M   = 1024 + q
//   pair 3 = ((w >> 8) & 0x00F000F0) | M   = 1024 + 16 q
// = 1 shift + 4 v_and_or + 2 v_pk_add_f16 + 2 v_pk_fma_f16 per 8 weights; each pk op rounds an exact value once.
struct Dq4 {
  uint32_t m0, m1, mag;  // masks and magic, kept in registers (VOP3 takes no literals on gfx9)
  h2_t s16;
};

// (x & m) | c in one VOP3 instruction (hipcc splits it when both constants sit in SGPRs: one constant-bus read on gfx9)
__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t m, uint32_t c) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(m), "v"(c));
  return r;
}

__device__ __forceinline__ h8_t dequant4(uint32_t w, const Dq4& q, h2_t c0, h2_t c1) {
  const uint32_t w8 = w >> 8;
  const h2_t p0 = as_h2(and_or(w, q.m0, q.mag)) + c0;
  const h2_t p1 = as_h2(and_or(w, q.m1, q.mag)) * q.s16 + c1;
  const h2_t p2 = as_h2(and_or(w8, q.m0, q.mag)) + c0;
  const h2_t p3 = as_h2(and_or(w8, q.m1, q.mag)) * q.s16 + c1;
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

__device__ __forceinline__ h2_t splat(float v) {
  h2_t r;
  r[0] = _Float16(v);
  r[1] = _Float16(v);
  return r;
}

// a group scale from the dword load_stage fetched: f32 as is, 16-bit types from the half selected by `sh`
// (branch-free: the scale type is launch-uniform, selects are cheaper than branches here)
__device__ __forceinline__ float scale_bits_to_f32(uint32_t x, int st, int sh) {
  const uint32_t h = (x >> sh) & 0xFFFFu;
  const float fb = __uint_as_float(h << 16);
  const float fh = f16_bits_to_f32(uint16_t(h));
  const float f16or = st == kScaleBF16 ? fb : fh;
  return st == kScaleF32 ? __uint_as_float(x) : f16or;
}

// ... with the scale type known at compile time (ST >= 0: the int2 M = 1 instantiations, whose body applies a scale
// every 64 k at g64 -- VERDICT r5 item 4), else from the launch-uniform runtime value as above
template <int ST>
__device__ __forceinline__ float scale_to_f32(uint32_t x, int st, int sh) {
  if constexpr (ST < 0) return scale_bits_to_f32(x, st, sh);
  else if constexpr (ST == kScaleF32) return __uint_as_float(x);
  else if constexpr (ST == kScaleBF16) return __uint_as_float((x >> sh) << 16);
  else return f16_bits_to_f32(uint16_t(x >> sh));
}

// ------------------------------------------------------------------------------------------------ activation staging
// activation bits -> 8 floats of one staging unit (runtime type: staging runs once per workgroup)
__device__ __forceinline__ void unit_to_f32(int act_t, uint4 x0, uint4 x1, float (&f)[8]) {
  const uint32_t w[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  if (act_t == kActF32) {
#pragma unroll
    for (int j = 0; j < 8; j++) f[j] = __uint_as_float(w[j]);
  } else if (act_t == kActBF16) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      f[2 * j] = __uint_as_float(w[j] << 16);
      f[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const h2_t h = as_h2(w[j]);
      f[2 * j] = float(h[0]);
      f[2 * j + 1] = float(h[1]);
    }
  }
}

// write one staging unit (8 k of one row) as fp16 hi (+ lo) rows
template <int HILO>
__device__ __forceinline__ void unit_store(char* smem, const float (&f)[8], int row, int k, int M, int Kp) {
  h8_t hi, lo;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    hi[j] = _Float16(f[j]);
    lo[j] = _Float16(f[j] - float(hi[j]));
  }
  *reinterpret_cast<h8_t*>(smem + (size_t(row) * Kp + k) * 2) = hi;
  if constexpr (HILO != 0) *reinterpret_cast<h8_t*>(smem + (size_t(M + row) * Kp + k) * 2) = lo;
}

// element-wise staging (act-order gather, unaligned rows, K % 8 != 0)
template <int HILO>
__device__ __forceinline__ void stage_a_slow(const GemvArgs& a, char* smem, int units, int Kp) {
  for (int u = threadIdx.x; u < units; u += blockDim.x) {
    const int row = u / (Kp >> 3), k = (u - row * (Kp >> 3)) * 8;
    float f[8];
    for (int j = 0; j < 8; j++) {
      const int kk = k + j;
      f[j] = 0.f;
      if (kk < a.K) {
        const size_t src = size_t(row) * a.lda + (a.shuffle ? a.shuffle[kk] : kk);
        if (a.act_t == kActF32)
          f[j] = static_cast<const float*>(a.A)[src];
        else if (a.act_t == kActBF16)
          f[j] = bf16_bits_to_f32(static_cast<const uint16_t*>(a.A)[src]);
        else
          f[j] = float(static_cast<const _Float16*>(a.A)[src]);
      }
    }
    unit_store<HILO>(smem, f, row, k, a.M, Kp);
  }
}

// ------------------------------------------------------------------------------------------------ the kernel
// finer groups carry GPT scale (+ zero-point) registers per tile: those variants run at most 8 waves per workgroup
template <int GPT>
constexpr int gemv_max_threads() {
  return GPT == 1 ? 1024 : 512;
}

// NST: register stages in flight per wave (3, or 1 where no wave streams more than two stages: the ring's extra slots
// would only carry dead out-of-range loads, see m1_body)
template <int BITS, int HILO, int GPT, bool ASYM, int NST>
__global__ __launch_bounds__(gemv_max_threads<GPT>()) void woq_gemv_kernel(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KT = BITS == 4 ? 128 : (BITS == 2 ? 256 : 64);
  constexpr int SPT = KT / 32;
  static_assert(SPT % GPT == 0, "groups must tile the K tile");
  constexpr int SPG = SPT / GPT;  // steps per group when GPT > 1
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int NW = __builtin_amdgcn_readfirstlane(int(blockDim.x >> 6));
  const int M = a.M, nt = a.nt, Kp = nt * KT;
  const int R = HILO == 0 ? M : 2 * M;
  const int nsl = (nt + KS - 1) / KS;  // K-slices per stripe
  NAD_TRACE(0);
#ifdef NAD_EXP_KPREF
  {  // touch every 64-B line of the argument block in one batch so the later scalar loads hit
    const __attribute__((address_space(4))) uint32_t* kp =
        (const __attribute__((address_space(4))) uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < int(sizeof(GemvArgs) + 63) / 64; i++) s ^= kp[i * 16];
    asm volatile("; kpref %0" ::"s"(s));
  }
#endif

  // this workgroup's units (wave-uniform)
  const int G = gridDim.x, bid = blockIdx.x;
  const int u0 = int(unsigned(bid) * unsigned(a.units) / unsigned(G));
  const int u1 = int(unsigned(bid + 1) * unsigned(a.units) / unsigned(G));
  const int vpu = a.dual ? 2 : 1;
  const int v0 = u0 * vpu, nv = (u1 - u0) * vpu;
  const bool idle = wave >= nsl;  // more waves than K-slices: this wave only joins the barriers
  float* part = reinterpret_cast<float*>(smem + a.part_off);  // [nv][NW][M][16]
  const int bd = blockDim.x;

  // 1) activation loads, then the first three weight stages, back to back
  const int a_units = M * (Kp >> 3);
  constexpr int AR = 2;  // activation units per thread issued ahead of the weights
  const int esz = a.act_t == kActF32 ? 4 : 2;
  const auto ra = rsrc(a.A, (M - 1) * a.lda * esz + a.K * esz);
  uint4 x[AR][2];
  if (a.a_fast) {
#pragma unroll
    for (int q = 0; q < AR; q++) {
      const int u = q * bd + int(threadIdx.x);
      const int row = u / (Kp >> 3), k = (u - row * (Kp >> 3)) * 8;
      const int off = (u < a_units && k < a.K) ? (row * a.lda + k) * esz : kOOB;
      x[q][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
      x[q][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, off + 16, 0, 0));
    }
  }
  const int vs = a.scale_t == kScaleF32 ? (lane & 15) * 4 : (lane & 14) * 2;
  StageCursor lc;
  lc.j = idle ? nv : 0;
  lc.q = wave;
  lc.s = 0;
  lc.rt = rsrc(a.w[0].tiles, 0);  // zero records: every access out of range (idle waves, past-the-end stages)
  lc.rs = lc.rt;
  lc.rz = lc.rt;
  if (!idle && nv > 0) cursor_stripe(a, lc, v0);
  StageRegs<GPT> S[NST];
  // Only the first stage goes out before the activations are published: issuing all three first stalled the wave on
  // memory back-pressure and delayed the (already landed) activation staging by ~1-2 us (phase trace; the pre-issue
  // A/B of round 4, profiles/r04_gemv_preissue_ab.txt).
  load_stage<GPT, ASYM>(a, S[0], lc, nv, nsl, wave, NW, v0, lane, vs);
  NAD_TRACE(4);

  // 2) publish the activations (waits only for the loads issued before the weights)
  if (a.a_fast) {
#pragma unroll
    for (int q = 0; q < AR; q++) {
      const int u = q * bd + int(threadIdx.x);
      if (u < a_units) {
        const int row = u / (Kp >> 3), k = (u - row * (Kp >> 3)) * 8;
        float f[8];
        unit_to_f32(a.act_t, x[q][0], x[q][1], f);
        unit_store<HILO>(smem, f, row, k, M, Kp);
      }
    }
    for (int u = AR * bd + int(threadIdx.x); u < a_units; u += bd) {  // large M * K only
      const int row = u / (Kp >> 3), k = (u - row * (Kp >> 3)) * 8;
      const int off = k < a.K ? (row * a.lda + k) * esz : kOOB;
      const uint4 y0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
      const uint4 y1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, off + 16, 0, 0));
      float f[8];
      unit_to_f32(a.act_t, y0, y1, f);
      unit_store<HILO>(smem, f, row, k, M, Kp);
    }
  } else {
    stage_a_slow<HILO>(a, smem, a_units, Kp);
  }
  {
    uint4* zr = reinterpret_cast<uint4*>(smem + size_t(R) * Kp * 2);
    for (int i = threadIdx.x; i < (Kp >> 3); i += bd) zr[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();
#pragma unroll
  for (int i = 1; i < NST; i++) load_stage<GPT, ASYM>(a, S[i], lc, nv, nsl, wave, NW, v0, lane, vs);
  NAD_TRACE(1);

  // 3) the stream
  const int m = lane & 15;   // MFMA A row fed by this lane (and C column n)
  const int kq = lane >> 4;  // k-quarter of a 32-k step
  const int arow = HILO == 1 ? (m & 7) : m;
  const bool is_lo = HILO == 1 && m >= 8;
  const int row_hi = arow < M ? (is_lo ? M + arow : arow) : R;  // inactive rows read the zero row
  const int row_lo = arow < M ? M + arow : R;
  const char* a_hi = smem + size_t(row_hi) * Kp * 2 + kq * 16;
  const char* a_lo = smem + size_t(row_lo) * Kp * 2 + kq * 16;
  const int ssh = a.scale_t == kScaleF32 ? 0 : (lane & 1) * 16;  // this lane's half of a 16-bit scale pair
  constexpr int BIAS = BITS == 4 ? 8 : (BITS == 2 ? 2 : 128);
  Dq4 dq;
  dq.m0 = __builtin_amdgcn_readfirstlane(a.dq_mask);
  dq.m1 = dq.m0 << 4;
  dq.mag = __builtin_amdgcn_readfirstlane(a.dq_magic);
  dq.s16 = splat(1.f / 16.f);
  const h2_t zc0 = splat(-(1024.f + BIAS)), zc1 = splat(-(64.f + BIAS));

  f4_t acc = {0.f, 0.f, 0.f, 0.f};
  int cj = idle ? nv : 0, cq = wave;  // compute cursor (wave-uniform)

  auto compute_stage = [&](const StageRegs<GPT>& S) {
    if (cj >= nv) return;
    const int t0 = cq * KS;
    const char* ab = a_hi + t0 * KT * 2;
    const char* abl = a_lo + t0 * KT * 2;
    // KS independent MFMA chains (one per tile, step-major) so the scheduler can interleave them; tiles past the end
    // of K carry out-of-range (zero) weights and a zero scale, and read a valid activation row (no NaN from LDS).
    f4_t accg[KS];
#pragma unroll
    for (int d = 0; d < SPT; d++) {
      const int g = GPT == 1 ? 0 : d / SPG;
#pragma unroll
      for (int i = 0; i < KS; i++) {
        const int ti = min(t0 + i, nt - 1) - t0;
        h8_t bf;
        if constexpr (BITS == 4) {
          if constexpr (ASYM) {
            const float z = float(S.zp[i][g]);
            bf = dequant4(S.b[i][d], dq, zc0 - splat(z), zc1 - splat(z));
          } else {
            bf = dequant4(S.b[i][d], dq, zc0, zc1);
          }
        } else {
          bf = BITS == 2 ? dequant2_step(S.b[i], d, BIAS + S.zp[i][g])
                         : dequant_step<BITS>(S.b[i], d, zp_const(BIAS + S.zp[i][g]));
        }
        const h8_t af = *reinterpret_cast<const h8_t*>(ab + ti * KT * 2 + d * 64);
        const bool first = d % SPG == 0;
        accg[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, first ? f4_t{0.f, 0.f, 0.f, 0.f} : accg[i], 0, 0, 0);
        if constexpr (HILO == 2) {
          const h8_t afl = *reinterpret_cast<const h8_t*>(abl + ti * KT * 2 + d * 64);
          accg[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(afl, bf, accg[i], 0, 0, 0);
        }
      }
      if ((d + 1) % SPG == 0) {  // group end: scale each tile's group partial into the stripe sum, in tile order
#pragma unroll
        for (int i = 0; i < KS; i++) acc += accg[i] * scale_bits_to_f32(S.sc[i][g], a.scale_t, ssh);
      }
    }
    cq += NW;
    if (cq >= nsl) {  // this wave's last slice of stripe cj: publish its partial
      f4_t r = acc;
      if constexpr (HILO == 1) {
#pragma unroll
        for (int xx = 0; xx < 4; xx++) r[xx] += __shfl_down(r[xx], 32, 64);
      }
      float* ps = part + (size_t(cj) * NW + wave) * M * 16 + m;
#pragma unroll
      for (int xx = 0; xx < 4; xx++) {
        const int row = (lane >> 4) * 4 + xx;
        if (row < M && (HILO != 1 || lane < 32)) ps[row * 16] = r[xx];
      }
      acc = f4_t{0.f, 0.f, 0.f, 0.f};
      cq = wave;
      cj++;
    }
  };

  while (cj < nv) {
#pragma unroll
    for (int i = 0; i < NST; i++) {
      compute_stage(S[i]);
      load_stage<GPT, ASYM>(a, S[i], lc, nv, nsl, wave, NW, v0, lane, vs);
    }
  }
  NAD_TRACE_MAX(2);
  __syncthreads();

  // 4) sum each stripe's wave slots in wave order and apply the epilogue
  const int nout = (u1 - u0) * M * 16;
  const int nwl = min(NW, nsl);  // waves that own slices
  for (int o = threadIdx.x; o < nout; o += bd) {
    const int p = o / (M * 16), mm = (o >> 4) % M, nn = o & 15;
    float y[2] = {0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (h < vpu) {
        const float* ps = part + (size_t(p * vpu + h) * NW * M + mm) * 16 + nn;
        const size_t wst = size_t(M) * 16;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        int w = 0;
        for (; w + 3 < nwl; w += 4) {
          s0 += ps[size_t(w) * wst];
          s1 += ps[size_t(w + 1) * wst];
          s2 += ps[size_t(w + 2) * wst];
          s3 += ps[size_t(w + 3) * wst];
        }
        for (; w < nwl; w++) s0 += ps[size_t(w) * wst];
        y[h] = (s0 + s1) + (s2 + s3);
      }
    }
    int wsel, s;
    vstripe(a, v0 + p * vpu, wsel, s);
    if (a.dual) wsel = 0;
    const int n = s * 16 + nn;
    const int nmax = sel3(wsel, a.w[0].n, a.w[1].n, a.w[2].n);
    if (n >= nmax) continue;
    float* out = sel3(wsel, a.w[0].out, a.w[1].out, a.w[2].out);
    const int ldo = sel3(wsel, a.w[0].ldo, a.w[1].ldo, a.w[2].ldo);
    float v = y[0];
    switch (a.epi) {
      case kEpiBias:
        v += a.w[0].bias[size_t(mm) * a.w[0].bias_ld + n];
        break;
      case kEpiAddGelu:
        v = gelu_f(v + a.w[0].bias[size_t(mm) * a.w[0].bias_ld + n]);
        break;
      case kEpiGelu:
        v = gelu_f(v);
        break;
      case kEpiSilu:
        v = silu_f(v);
        break;
      case kEpiResAdd:
        v += a.res[size_t(mm) * a.ld_res + n];
        break;
      case kEpiSiluMul: {
        const float t1 = silu_f(y[0]);
        if (a.aux) a.aux[size_t(mm) * a.ld_aux + n] = t1;
        v = t1 * y[1];
        break;
      }
      case kEpiGeluMul: {
        const float t1 = gelu_f(y[0]);
        if (a.aux) a.aux[size_t(mm) * a.ld_aux + n] = t1;
        v = t1 * y[1];
        break;
      }
      default:
        break;
    }
    out[size_t(mm) * ldo + n] = v;
  }
  NAD_TRACE(3);
}

// ------------------------------------------------------------------------------------------------ M = 1 variant
// Every launch pays its executed code again (the instruction cache starts cold per dispatch: ~0.45 us per KB at 8
// waves per CU, tools/ifetch_probe.hip), and a decode matmul at K = 4096 streams one stripe per workgroup -- so the
// executed instruction bytes ARE the fixed cost.  This variant of the stream for M = 1 (int4 / int2, groups of a whole
// tile or a power-of-two part of one) keeps that path short: the activation type is a template parameter, the workgroup's unit range comes from host-divided
// counts (no integer division), and each wave stages only ITS K-slices of the activations into its own LDS rows
// (hi / lo fp16, plus a zero row for the MFMA rows M = 1 leaves empty), so nothing waits on a block-wide barrier before
// the stream; the one barrier is the final cross-wave reduction.
// K-slices per wave it stages: 2 (K <= waves * 2 * ks * KT), or 4 for long K (Mistral's down, K = 14336 at 7 waves)
// per wave: a zero row, then per slice {hi, lo} rows of ks * KT fp16 each
constexpr int lean_row_bytes(int bits, int ks) { return ks * (bits == 4 ? 128 : 256) * 2; }
constexpr int lean_wave_lds(int bits, int ks, int spw) { return lean_row_bytes(bits, ks) * (1 + 2 * spw); }
static int lean_ks(const GemvArgs& a) { return a.lean_ks == 1 || a.lean_ks == 2 ? a.lean_ks : KS; }
// narrow slices carry few stage registers: those launches may run 16 waves whatever the groups per tile
template <int GPT, int KSN>
constexpr int m1_max_threads() {
  return GPT == 1 || KSN <= 2 ? 1024 : 512;
}
// K-slices per wave staged: 1 for the narrow-slice launches (exactly one slice per wave: a second would only be a
// dead out-of-range activation load in front of the weights), 4 for long K, else 2
static int lean_spw(const GemvArgs& a) { return a.lean_spw == 4 ? 4 : (a.lean_spw == 1 ? 1 : 2); }

static bool lean_ok(const GemvArgs& a, int bits, int waves) {
  int tpg = 0;
  const int ks = lean_ks(a);
  const int nsl = (a.nt + ks - 1) / ks;
  const int gpt = gemv_groups_per_tile(bits, a.nt, a.ng, a.bs, &tpg);
  const bool inst = bits == 4 ? (gpt == 1 || gpt == 2) : (bits == 2 && (gpt == 1 || gpt == 2 || (gpt == 4 && !a.asym)));
  return a.lean && a.M == 1 && inst && a.a_fast && nsl <= waves * lean_spw(a);
}

// BATCH: independent problems of one shape in one launch (BTLAGemmBatchDriver, bestla_gemm.cpp:508-624): workgroup
// b serves problem b / batch_wpp -- its activations, weight and output pointers come from the problem table (one
// scalar-cache line) -- and that problem's share b % batch_wpp of the stripes, so a batch of decode-size problems
// streams like one large launch instead of paying each launch's fixed chain.
// The kernel body takes its workgroup index as an argument: woq_gemv_m1_dual_kernel runs two instantiations side by
// side in one launch.
// NST: register stages in flight per wave.  Every stage slot is loaded again right after it is computed -- with
// out-of-range offsets once the wave's run is done -- so a ring deeper than the wave's own stages only adds dead
// loads to the CU's memory queue, in front of the live ones.  Measured (profiles/r04_gemv_ring_depth_ab.txt,
// r04_gemv_nst_ab.txt): one stage (1-2 KiB per wave) is fastest until a wave streams about seven, two beyond that
// or for 1 KiB int2 stages from four (O 5.78 -> 4.83 us, down K = 11008 9.6 -> 7.8, gate/up 13.2 -> 12.2, QKV 8.6 ->
// 8.1); deeper rings are slower everywhere except the batched launch's long streams (3: 1.43 vs 1.46 us per problem).
#ifndef NAD_M1_BATCH_NST
#define NAD_M1_BATCH_NST 3
#endif
#ifndef NAD_M1_DUAL_NST
#define NAD_M1_DUAL_NST 2
#endif

template <int BITS, int GPT, int AT, bool ASYM, int KSN, int SPW, bool BATCH, int NST, int ST = -1>
__device__ __forceinline__ void m1_body(GemvArgs& a, int bid) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KT = BITS == 4 ? 128 : 256, SPT = KT / 32, SPG = SPT / GPT;
  constexpr int RB = lean_row_bytes(BITS, KSN);  // one fp16 row of a slice
  constexpr int UNITS = KSN * KT / 8;             // 8-element staging units per slice
  constexpr int UPL = UNITS >= 64 ? UNITS / 64 : 1;  // ... per lane (2-tile int4 slices: lanes < 32 hold one)
  constexpr bool PART = UNITS < 64;
  constexpr int BIAS = BITS == 4 ? 8 : 2;
  constexpr int ESZ = AT == kActF32 ? 4 : 2;
  constexpr bool HL = AT != kActF16;  // fp32 / bf16 rows split into fp16 hi + lo (MFMA rows 0 and 8)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int NW = __builtin_amdgcn_readfirstlane(int(blockDim.x >> 6));
  const int nt = a.nt;
  const int nsl = (nt + KSN - 1) / KSN;
  const bool ulane = !PART || lane < UNITS;  // this lane holds a staging unit of each slice
  NAD_TRACE(0);
  if constexpr (BATCH) {
    const int p = bid / a.batch_wpp;
    bid -= p * a.batch_wpp;
    const GemvBatchEnt e = a.batch[p];
    a.A = e.act;
    a.w[0].tiles = e.tiles;
    a.w[0].scales = e.scales;
    a.w[0].zps = e.zps;
    a.w[0].out = e.out;
  }
  const int u0 = bid * a.u_q + min(bid, a.u_r);
  const int u1 = u0 + a.u_q + (bid < a.u_r ? 1 : 0);
  const int vpu = a.dual ? 2 : 1;
  const int v0 = u0 * vpu, nv = (u1 - u0) * vpu;
  const bool idle = wave >= nsl;
  float* part = reinterpret_cast<float*>(smem + a.part_off);  // [nv][NW][16]

  // 1) this wave's activation slices (q = wave + j NW), then the first weight stage
  const auto ra = rsrc(a.A, a.K * ESZ);
  uint4 x[SPW * UPL][2];
#pragma unroll
  for (int j = 0; j < SPW * UPL; j++) {
    const int q = wave + (j / UPL) * NW, k = q * (KSN * KT) + ((j % UPL) * 64 + lane) * 8;
    const int off = (ulane && q < nsl && k < a.K) ? k * ESZ : kOOB;
    x[j][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
    if constexpr (ESZ == 4) x[j][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, off + 16, 0, 0));
  }
  const int vs = a.scale_t == kScaleF32 ? (lane & 15) * 4 : (lane & 14) * 2;
  StageCursor lc;
  lc.j = idle ? nv : 0;
  lc.q = wave;
  lc.s = 0;
  lc.rt = rsrc(a.w[0].tiles, 0);
  lc.rs = lc.rt;
  lc.rz = lc.rt;
  if (!idle && nv > 0) cursor_stripe(a, lc, v0);
  StageRegs<GPT, KSN> S[NST];
  load_stage<GPT, ASYM, KSN>(a, S[0], lc, nv, nsl, wave, NW, v0, lane, vs);
  NAD_TRACE(4);

  // 2) stage the slices into this wave's rows (LDS ops of one wave complete in order: no barrier)
  char* wrow = smem + wave * lean_wave_lds(BITS, KSN, SPW);
#pragma unroll
  for (int u = 0; u < UPL; u++)
    if (ulane) *reinterpret_cast<uint4*>(wrow + (u * 64 + lane) * 16) = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int j = 0; j < SPW * UPL; j++) {
    if (!ulane) break;
    h8_t hi, lo;
    if constexpr (AT == kActF16) {
      hi = __builtin_bit_cast(h8_t, x[j][0]);
    } else {
      float f[8];
      unit_to_f32(AT, x[j][0], x[j][1], f);
#pragma unroll
      for (int e = 0; e < 8; e++) {
        hi[e] = _Float16(f[e]);
        lo[e] = _Float16(f[e] - float(hi[e]));
      }
    }
    char* row = wrow + RB + (j / UPL) * 2 * RB + ((j % UPL) * 64 + lane) * 16;
    *reinterpret_cast<h8_t*>(row) = hi;
    if constexpr (HL) *reinterpret_cast<h8_t*>(row + RB) = lo;
  }
#pragma unroll
  for (int i = 1; i < NST; i++) load_stage<GPT, ASYM, KSN>(a, S[i], lc, nv, nsl, wave, NW, v0, lane, vs);
  NAD_TRACE(1);

  // 3) the stream: MFMA row 0 = hi (lane m 0), row 8 = lo (lane m 8), every other row reads the zero row
  const int m = lane & 15, kq = lane >> 4;
  const bool isrow = m == 0 || (HL && m == 8);
  const char* abase = wrow + (isrow ? (m == 0 ? RB : 2 * RB) : 0) + kq * 16;
  const int slice_step = isrow ? 2 * RB : 0;
  const int ssh = a.scale_t == kScaleF32 ? 0 : (lane & 1) * 16;
  Dq4 dq;
  dq.m0 = __builtin_amdgcn_readfirstlane(a.dq_mask);
  dq.m1 = dq.m0 << 4;
  dq.mag = __builtin_amdgcn_readfirstlane(a.dq_magic);
  dq.s16 = splat(1.f / 16.f);
  const h2_t zc0 = splat(-(1024.f + BIAS)), zc1 = splat(-(64.f + BIAS));

  f4_t acc = {0.f, 0.f, 0.f, 0.f};
  int cj = idle ? nv : 0, cq = wave, cs = 0;  // compute cursor: local stripe, K-slice, slice ordinal of this wave

  auto compute_stage = [&](const StageRegs<GPT, KSN>& S) {
    if (cj >= nv) return;
    const char* ab = abase + cs * slice_step;
    f4_t accg[KSN];
#pragma unroll
    for (int d = 0; d < SPT; d++) {
      const int g = GPT == 1 ? 0 : d / SPG;
#pragma unroll
      for (int i = 0; i < KSN; i++) {
        h8_t bf;
        if constexpr (BITS == 4) {
          if constexpr (ASYM) {
            const float z = float(S.zp[i][g]);
            bf = dequant4(S.b[i][d], dq, zc0 - splat(z), zc1 - splat(z));
          } else {
            bf = dequant4(S.b[i][d], dq, zc0, zc1);
          }
        } else {
          bf = BITS == 2 ? dequant2_step(S.b[i], d, BIAS + S.zp[i][g])
                         : dequant_step<BITS>(S.b[i], d, zp_const(BIAS + S.zp[i][g]));
        }
        const h8_t af = *reinterpret_cast<const h8_t*>(ab + i * KT * 2 + d * 64);
        accg[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, d % SPG == 0 ? f4_t{0.f, 0.f, 0.f, 0.f} : accg[i],
                                                         0, 0, 0);
      }
      if ((d + 1) % SPG == 0) {  // group end: scale each tile's group partial into the stripe sum, in tile order
#pragma unroll
        for (int i = 0; i < KSN; i++) acc += accg[i] * scale_to_f32<ST>(S.sc[i][g], a.scale_t, ssh);
      }
    }
    cq += NW;
    cs++;
    if (cq >= nsl) {  // this wave's last slice of stripe cj: publish its partial (row 0 + row 8 = hi + lo)
      float r = acc[0];
      if constexpr (HL) {
        r += __shfl_down(r, 32, 64);
      }
#if NAD_GEMV_LEAN_TAIL
      if (lane < 16) part[(size_t(cj) * 16 + lane) * NW + wave] = r;  // [nv][16 columns][NW]: a column's slots together
#else
      if (lane < 16) part[(size_t(cj) * NW + wave) * 16 + lane] = r;
#endif
      acc = f4_t{0.f, 0.f, 0.f, 0.f};
      cq = wave;
      cs = 0;
      cj++;
    }
  };

  while (cj < nv) {
#pragma unroll
    for (int i = 0; i < NST; i++) {
      compute_stage(S[i]);
      load_stage<GPT, ASYM, KSN>(a, S[i], lc, nv, nsl, wave, NW, v0, lane, vs);
    }
  }
  NAD_TRACE_MAX(2);
  __syncthreads();

  // 4) sum each stripe's wave slots in wave order and apply the epilogue
  const int nout = (u1 - u0) * 16;
  const int nwl = min(NW, nsl);
  // the fused epilogue of output o = (local stripe p, column nn) from its stripe sum(s) y
  auto emit = [&](int p, int nn, const float (&y)[2]) {
    int wsel, s;
    vstripe(a, v0 + p * vpu, wsel, s);
    if (a.dual) wsel = 0;
    const int n = s * 16 + nn;
    if (n >= sel3(wsel, a.w[0].n, a.w[1].n, a.w[2].n)) return;
    float* out = sel3(wsel, a.w[0].out, a.w[1].out, a.w[2].out);
    float v = y[0];
    switch (a.epi) {
      case kEpiBias:
        v += a.w[0].bias[n];
        break;
      case kEpiAddGelu:
        v = gelu_f(v + a.w[0].bias[n]);
        break;
      case kEpiGelu:
        v = gelu_f(v);
        break;
      case kEpiSilu:
        v = silu_f(v);
        break;
      case kEpiResAdd:
        v += a.res[n];
        break;
      case kEpiSiluMul: {
        const float t1 = silu_f(y[0]);
        if (a.aux) a.aux[n] = t1;
        v = t1 * y[1];
        break;
      }
      case kEpiGeluMul: {
        const float t1 = gelu_f(y[0]);
        if (a.aux) a.aux[n] = t1;
        v = t1 * y[1];
        break;
      }
      default:
        break;
    }
    out[n] = v;
  };
#if NAD_GEMV_LEAN_TAIL
  if (nwl == 16 && NW == 16) {  // 16 waves with a slice each: four 16-B reads per column, no clamps or masks
    for (int o = threadIdx.x; o < nout; o += blockDim.x) {
      const int p = o >> 4, nn = o & 15;
      float y[2] = {0.f, 0.f};
#pragma unroll
      for (int h = 0; h < 2; h++) {
        if (h < vpu) {
          const float4* ps = reinterpret_cast<const float4*>(part + (size_t(p * vpu + h) * 16 + nn) * 16);
          const float4 t0 = ps[0], t1 = ps[1], t2 = ps[2], t3 = ps[3];
          // the general order below at nwl = 16: s_i sums slots i, i + 4, i + 8, i + 12
          const float s0 = ((t0.x + t1.x) + t2.x) + t3.x, s1 = ((t0.y + t1.y) + t2.y) + t3.y;
          const float s2 = ((t0.z + t1.z) + t2.z) + t3.z, s3 = ((t0.w + t1.w) + t2.w) + t3.w;
          y[h] = (s0 + s1) + (s2 + s3);
        }
      }
      emit(p, nn, y);
    }
    NAD_TRACE(3);
    return;
  }
#endif
  for (int o = threadIdx.x; o < nout; o += blockDim.x) {
    const int p = o >> 4, nn = o & 15;
    float y[2] = {0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (h < vpu) {  // all slots read at once (one LDS round trip), summed in the general kernel's order
#if NAD_GEMV_LEAN_TAIL
        const float* ps = part + (size_t(p * vpu + h) * 16 + nn) * NW;
#define NAD_SLOT(w) ps[w]
#else
        const float* ps = part + size_t(p * vpu + h) * NW * 16 + nn;
#define NAD_SLOT(w) ps[(w) * 16]
#endif
        float t[16];
#pragma unroll
        for (int w = 0; w < 16; w++) t[w] = NAD_SLOT(min(w, nwl - 1));
#undef NAD_SLOT
        const int full = nwl & ~3;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
        for (int w = 0; w < 16; w += 4)
          if (w < full) {
            s0 += t[w];
            s1 += t[w + 1];
            s2 += t[w + 2];
            s3 += t[w + 3];
          }
#pragma unroll
        for (int w = 0; w < 16; w++)
          if (w >= full && w < nwl) s0 += t[w];
        y[h] = (s0 + s1) + (s2 + s3);
      }
    }
    emit(p, nn, y);
  }
  NAD_TRACE(3);
}

template <int BITS, int GPT, int AT, bool ASYM, int KSN, int SPW, bool BATCH, int NST, int ST>
__global__ __launch_bounds__((m1_max_threads<GPT, KSN>())) void woq_gemv_m1_kernel(GemvArgs a) {
  m1_body<BITS, GPT, AT, ASYM, KSN, SPW, BATCH, NST, ST>(a, int(blockIdx.x));
}

// Two weight formats in one decode launch: workgroups [0, ga) run format 1's body over a, the rest format 2's over b
// (each exactly its own one-format launch's arithmetic).  The int2 policies' QKV (llama_utils.cpp:269-287: int2 Q, K
// with an int4 V of the same group size) then costs one launch instead of two.  Both bodies take 16 waves at K = 4096
// (int2: 1-tile slices of 256 k, int4: 2-tile slices of 256 k); the launch takes the larger LDS image.
template <int B1, int G1, int K1, int B2, int G2, int K2, int AT>
__global__ __launch_bounds__(1024) void woq_gemv_m1_dual_kernel(GemvArgs a, GemvArgs b, int ga) {
  if (int(blockIdx.x) < ga)
    m1_body<B1, G1, AT, false, K1, 1, false, NAD_M1_DUAL_NST>(a, int(blockIdx.x));
  else
    m1_body<B2, G2, AT, false, K2, 1, false, NAD_M1_DUAL_NST>(b, int(blockIdx.x) - ga);
}

// ------------------------------------------------------------------------------------------------ launcher
template <int BITS, int HILO, int GPT, bool ASYM, int NST>
static hipError_t gemv_launch5(const GemvArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  auto k = woq_gemv_kernel<BITS, HILO, GPT, ASYM, NST>;
  static bool attr_set = false;  // opt in to > 64 KiB of dynamic LDS once per instantiation
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k, g, b, lds, st, a);
  return hipGetLastError();
}
template <int BITS, int HILO, int GPT, bool ASYM>
static hipError_t gemv_launch4(const GemvArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  // stages of the busiest wave: its (stripe, KS-tile slice) pairs
  const int nsl = (a.nt + KS - 1) / KS, waves = int(b.x / 64);
  const int spw = (a.u_q + (a.u_r ? 1 : 0)) * (a.dual ? 2 : 1) * ((nsl + waves - 1) / waves);
  const int nst = a.m1_nst == 1 ? 1 : (a.m1_nst == 3 ? 3 : (spw <= 2 ? 1 : 3));
  return nst == 1 ? gemv_launch5<BITS, HILO, GPT, ASYM, 1>(a, g, b, lds, st)
                  : gemv_launch5<BITS, HILO, GPT, ASYM, 3>(a, g, b, lds, st);
}

template <int BITS, int GPT, int AT, bool ASYM, int KSN, int SPW, int NST, int ST>
static hipError_t gemv_m1_launch6(const GemvArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  auto k = woq_gemv_m1_kernel<BITS, GPT, AT, ASYM, KSN, SPW, false, NST, ST>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k, g, b, lds, st, a);
  return hipGetLastError();
}
// register stages per wave of a single-problem launch: the most (stripe, K-slice) stages any wave streams
static int m1_stages_per_wave(const GemvArgs& a, int ksn, int waves) {
  const int nsl = (a.nt + ksn - 1) / ksn;
  return (a.u_q + (a.u_r ? 1 : 0)) * (a.dual ? 2 : 1) * ((nsl + waves - 1) / waves);
}
template <int BITS, int GPT, int AT, bool ASYM, int KSN, int SPW, int ST>
static hipError_t gemv_m1_launch5(const GemvArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  if (a.batch) {
    auto kb = woq_gemv_m1_kernel<BITS, GPT, AT, ASYM, KSN, SPW, true, NAD_M1_BATCH_NST, ST>;
    static bool attr_b = false;
    if (!attr_b) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kb), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         160 * 1024);
      if (e != hipSuccess) return e;
      attr_b = true;
    }
    hipLaunchKernelGGL(kb, g, b, lds, st, a);
    return hipGetLastError();
  }
  const int spw = m1_stages_per_wave(a, KSN, int(b.x / 64));
  const int nst = a.m1_nst == 1 || a.m1_nst == 2 ? a.m1_nst : (spw >= 7 || (KSN == 1 && spw >= 4) ? 2 : 1);
  return nst == 1 ? gemv_m1_launch6<BITS, GPT, AT, ASYM, KSN, SPW, 1, ST>(a, g, b, lds, st)
                  : gemv_m1_launch6<BITS, GPT, AT, ASYM, KSN, SPW, 2, ST>(a, g, b, lds, st);
}
// int2: the scale type as a template parameter (3 x the int2 instantiations; int4 keeps the runtime form)
#ifndef NAD_INT2_ST
#define NAD_INT2_ST 1
#endif
template <int BITS, int GPT, int AT, bool ASYM, int ST = -1>
static hipError_t gemv_m1_launch4(const GemvArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  if constexpr (BITS == 2 && ST < 0 && NAD_INT2_ST) {
    if (a.scale_t == kScaleF32) return gemv_m1_launch4<BITS, GPT, AT, ASYM, kScaleF32>(a, g, b, lds, st);
    if (a.scale_t == kScaleBF16) return gemv_m1_launch4<BITS, GPT, AT, ASYM, kScaleBF16>(a, g, b, lds, st);
    return gemv_m1_launch4<BITS, GPT, AT, ASYM, kScaleF16>(a, g, b, lds, st);
  } else {
    if (a.lean_ks == 1) return gemv_m1_launch5<BITS, GPT, AT, ASYM, 1, 1, ST>(a, g, b, lds, st);
    if (a.lean_ks == 2) return gemv_m1_launch5<BITS, GPT, AT, ASYM, 2, 1, ST>(a, g, b, lds, st);
    return a.lean_spw == 4 ? gemv_m1_launch5<BITS, GPT, AT, ASYM, KS, 4, ST>(a, g, b, lds, st)
                           : gemv_m1_launch5<BITS, GPT, AT, ASYM, KS, 2, ST>(a, g, b, lds, st);
  }
}
template <int BITS, int GPT>
static hipError_t gemv_m1_launch2(const GemvArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  if (a.act_t == kActF32) return a.asym ? gemv_m1_launch4<BITS, GPT, kActF32, true>(a, g, b, lds, st)
                                        : gemv_m1_launch4<BITS, GPT, kActF32, false>(a, g, b, lds, st);
  if (a.act_t == kActF16) return a.asym ? gemv_m1_launch4<BITS, GPT, kActF16, true>(a, g, b, lds, st)
                                        : gemv_m1_launch4<BITS, GPT, kActF16, false>(a, g, b, lds, st);
  return a.asym ? gemv_m1_launch4<BITS, GPT, kActBF16, true>(a, g, b, lds, st)
                : gemv_m1_launch4<BITS, GPT, kActBF16, false>(a, g, b, lds, st);
}
// int4 / int2 with one group per tile or 2 per tile; int2 also 4 per tile (sym only, as the general kernel).  The
// int2 instantiations (3 scale types each) compile as their own object (woq_gemv_b2.o: GEMV_PART=1) in parallel with
// the rest (GEMV_PART=0); without GEMV_PART (trace / experiment builds) one object holds everything.
#if !defined(GEMV_PART) || GEMV_PART == 1
hipError_t gemv_m1_launch_b2(const GemvArgs& a, int gpt, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  if (gpt == 1) return gemv_m1_launch2<2, 1>(a, g, b, lds, st);
  if (gpt == 2) return gemv_m1_launch2<2, 2>(a, g, b, lds, st);
  if (gpt == 4 && !a.asym) return a.act_t == kActF32 ? gemv_m1_launch4<2, 4, kActF32, false>(a, g, b, lds, st)
                                 : (a.act_t == kActF16 ? gemv_m1_launch4<2, 4, kActF16, false>(a, g, b, lds, st)
                                                       : gemv_m1_launch4<2, 4, kActBF16, false>(a, g, b, lds, st));
  return hipErrorInvalidValue;
}
#else
hipError_t gemv_m1_launch_b2(const GemvArgs& a, int gpt, dim3 g, dim3 b, size_t lds, hipStream_t st);
#endif
#if !defined(GEMV_PART) || GEMV_PART == 0
static hipError_t gemv_m1_launch(const GemvArgs& a, int bits, int gpt, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  if (bits == 4) {
    if (gpt == 1) return gemv_m1_launch2<4, 1>(a, g, b, lds, st);
    if (gpt == 2) return gemv_m1_launch2<4, 2>(a, g, b, lds, st);
    return hipErrorInvalidValue;
  }
  return gemv_m1_launch_b2(a, gpt, g, b, lds, st);
}

// Instantiated: groups of >= KT (GPT 1), KT/2 (GPT 2) and KT/4 (GPT 4), sym and asym.  Finer groups fall back to
// woq_skinny_kernel.
template <int BITS, int HILO>
static hipError_t gemv_launch2(const GemvArgs& a, int gpt, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  constexpr int SPT = (BITS == 4 ? 128 : (BITS == 2 ? 256 : 64)) / 32;
  if (gpt == 1) return a.asym ? gemv_launch4<BITS, HILO, 1, true>(a, g, b, lds, st)
                              : gemv_launch4<BITS, HILO, 1, false>(a, g, b, lds, st);
  if (gpt == 2) return a.asym ? gemv_launch4<BITS, HILO, 2, true>(a, g, b, lds, st)
                              : gemv_launch4<BITS, HILO, 2, false>(a, g, b, lds, st);
  if constexpr (SPT % 4 == 0) {
    if (gpt == 4)
      return a.asym ? gemv_launch4<BITS, HILO, 4, true>(a, g, b, lds, st)
                    : gemv_launch4<BITS, HILO, 4, false>(a, g, b, lds, st);
  }
  return hipErrorInvalidValue;
}

template <int BITS>
static hipError_t gemv_launch1(const GemvArgs& a, int hilo, int gpt, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  if (hilo == 0) return gemv_launch2<BITS, 0>(a, gpt, g, b, lds, st);
  if (hilo == 1) return gemv_launch2<BITS, 1>(a, gpt, g, b, lds, st);
  return gemv_launch2<BITS, 2>(a, gpt, g, b, lds, st);
}

// LDS layout (and its size) of one launch: activation rows, then the partial-sum slots [nv][waves][M][16]
size_t gemv_lds_layout(GemvArgs& a, int bits, int waves, int grid) {
  if (lean_ok(a, bits, waves)) {  // woq_gemv_m1_kernel: per-wave rows, then the partial slots [nv][waves][16]
    const int upw = (a.units + grid - 1) / grid;
    a.part_off = waves * lean_wave_lds(bits, lean_ks(a), lean_spw(a));
    return size_t(a.part_off) + size_t(upw) * (a.dual ? 2 : 1) * waves * 16 * 4;
  }
  const int KT = bits == 4 ? 128 : (bits == 2 ? 256 : 64);
  const int R = a.act_t == kActF16 ? a.M : 2 * a.M;
  const size_t kp = size_t(a.nt) * KT;
  const size_t abytes = (size_t(R) + 1) * kp * 2;
  const int upw = (a.units + grid - 1) / grid;  // max units per workgroup
  const size_t nv = size_t(upw) * (a.dual ? 2 : 1);
  a.part_off = int((abytes + 15) & ~size_t(15));
  return size_t(a.part_off) + nv * waves * a.M * 16 * 4;
}

// waves per workgroup: balanced K-slices per wave, at most 16 (8 for groups finer than a K tile)
int gemv_waves(int bits, int nt, int ng, int bs) {
  int tpg = 0;
  const int gpt = gemv_groups_per_tile(bits, nt, ng, bs, &tpg);
  const int maxw = gpt > 1 ? 8 : 16;
  const int nsl = (nt + KS - 1) / KS;
  const int spw = (nsl + maxw - 1) / maxw;  // slices per wave
  return (nsl + spw - 1) / spw;
}

void gemv_lean_slices(GemvArgs& a, int bits, int* waves, int ks_pref) {
  a.lean_ks = KS;
  a.lean_spw = 2;
  if (a.M == 1 && a.lean && (a.nt + KS - 1) / KS > 2 * *waves) {  // long K: up to 4 slices per wave
    a.lean_spw = 4;
    if (!lean_ok(a, bits, *waves)) a.lean_spw = 2;
    return;
  }
  // Slices of 1 or 2 tiles, one per wave, up to 16 waves (the narrowest width that fits).  bench (graph-replayed
  // token): 2-tile slices took Llama int4 g128 837 -> 853 tok/s and the Mistral int2 policy 586 -> 633 (its int2
  // K = 4096 launches from 4 waves to 8).  NAD_GEMV_KS: 2 = 1- or 2-tile, 3 = 2-tile only, 4 = 4-tile everywhere.
  if ((ks_pref != 2 && ks_pref != 3) || a.M != 1 || !a.lean) return;
  const int ks = a.nt <= 16 && ks_pref == 2 ? 1 : 2;
  const int nsl = (a.nt + ks - 1) / ks;
  if (nsl > 16 || nsl <= *waves) return;  // narrow slices only where each wave gets one and there are more waves
  if (!lean_ok(a, bits, *waves)) return;  // the 4-tile launch would not take the M = 1 kernel either
  a.lean_ks = ks;
  a.lean_spw = 1;  // one slice per wave
  if (!lean_ok(a, bits, nsl)) {
    a.lean_ks = KS;
    a.lean_spw = 2;
    return;
  }
  *waves = nsl;
}

int gemv_groups_per_tile(int bits, int nt, int ng, int bs, int* tpg) {
  const int KT = bits == 4 ? 128 : (bits == 2 ? 256 : 64);
  if (ng == 1) {
    *tpg = 0;  // one group: ends only at the last tile
    return 1;
  }
  if (bs % KT == 0) {
    *tpg = bs / KT;
    return (*tpg & (*tpg - 1)) == 0 ? 1 : 0;  // power-of-two tiles per group
  }
  if (KT % bs == 0 && bs % 32 == 0) {
    *tpg = 1;
    const int g = KT / bs;
    return (g == 2 || g == 4) ? g : 0;
  }
  return 0;
}

bool gemv_uses_m1(const GemvArgs& a, int bits, int waves) { return lean_ok(a, bits, waves); }

bool gemv_dual_ok(const GemvArgs& a, int bits_a, const GemvArgs& b, int bits_b, int waves) {
  int tpg = 0;
  const int ga = gemv_groups_per_tile(bits_a, a.nt, a.ng, a.bs, &tpg), gb = gemv_groups_per_tile(bits_b, b.nt, b.ng, b.bs, &tpg);
  const bool pair = bits_a == 2 && bits_b == 4 && ((ga == 4 && gb == 2) || (ga == 2 && gb == 1));
  return pair && !a.asym && !b.asym && a.lean_ks == 1 && b.lean_ks == 2 && a.act_t == kActF32 && b.act_t == kActF32 &&
         waves == 16 && lean_ok(a, bits_a, waves) && lean_ok(b, bits_b, waves);
}

hipError_t launch_gemv_dual(const GemvArgs& a, const GemvArgs& b, int ga, int gb, int waves, size_t lds,
                            hipStream_t stream) {
  int tpg = 0;
  const int g1 = gemv_groups_per_tile(2, a.nt, a.ng, a.bs, &tpg);
  auto go = [&](auto k) -> hipError_t {
    static bool attr = false;
    if (!attr) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         160 * 1024);
      if (e != hipSuccess) return e;
      attr = true;
    }
    hipLaunchKernelGGL(k, dim3(ga + gb), dim3(waves * 64), lds, stream, a, b, ga);
    return hipGetLastError();
  };
  if (g1 == 4) return go(woq_gemv_m1_dual_kernel<2, 4, 1, 4, 2, 2, kActF32>);  // groups of 64
  return go(woq_gemv_m1_dual_kernel<2, 2, 1, 4, 1, 2, kActF32>);              // groups of 128
}

hipError_t launch_gemv_batch(const GemvArgs& a, int bits, int waves, int grid, size_t lds, hipStream_t stream) {
  int tpg = 0;
  const int gpt = gemv_groups_per_tile(bits, a.nt, a.ng, a.bs, &tpg);
  if (gpt == 0 || !a.batch || a.batch_wpp <= 0 || !lean_ok(a, bits, waves)) return hipErrorInvalidValue;
  return gemv_m1_launch(a, bits, gpt, dim3(grid), dim3(waves * 64), lds, stream);
}

hipError_t launch_gemv(const GemvArgs& a, int bits, int waves, int grid, size_t lds, hipStream_t stream) {
  const int hilo = a.act_t == kActF16 ? 0 : (a.M <= 8 ? 1 : 2);
  int tpg = 0;
  const int gpt = gemv_groups_per_tile(bits, a.nt, a.ng, a.bs, &tpg);
  if (gpt == 0) return hipErrorInvalidValue;
  dim3 g(grid), b(waves * 64);
  if (lean_ok(a, bits, waves)) return gemv_m1_launch(a, bits, gpt, g, b, lds, stream);
  if (bits == 4) return gemv_launch1<4>(a, hilo, gpt, g, b, lds, stream);
  if (bits == 2) return gemv_launch1<2>(a, hilo, gpt, g, b, lds, stream);
  return gemv_launch1<8>(a, hilo, gpt, g, b, lds, stream);
}

#endif  // GEMV_PART 0

}  // namespace nad

#if defined(NAD_PHASE_TRACE) && (!defined(GEMV_PART) || GEMV_PART == 0)
extern "C" int nad_trace_clock_khz() {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return -1;
  return khz;
}

extern "C" int nad_trace_fetch(void* host, size_t bytes, int clear, int grid_filter) {
  (void)grid_filter;
  const size_t n = sizeof(nad::nad_trace_buf) < bytes ? sizeof(nad::nad_trace_buf) : bytes;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (host && hipMemcpyFromSymbol(host, HIP_SYMBOL(nad::nad_trace_buf), n) != hipSuccess) return -1;
  if (clear) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(nad::nad_trace_buf)) != hipSuccess) return -1;
    if (hipMemset(p, 0, sizeof(nad::nad_trace_buf)) != hipSuccess) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
  }
  return 0;
}
#endif
