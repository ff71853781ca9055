// woq_gemv.hip -- the decode (M <= 16) weight-only-quantized GEMV for gfx950: a persistent stripe stream.
//
// Replaces GEMVWrapper::gemv_kblock -> gemv_{4,2}bit_fp32_fp32 (bestla/bestla/bestla_wrapper.h:364-468,
// bestla/bestla/kernel_ref.h:2489-2531,2712-2760) and the fused QKV / FFN-gate-up decode launches
// (neural_speed/core/layers/ip_fusion_qkv.cpp:22-93, ip_fusion_ffn.cpp:407-457).
//
// Shape of the work.  A launch streams `units` stripes (16 output columns x all of K; for the dual SiLU*mul / GELU*mul
// epilogue a unit is the pair {gate stripe s, up stripe s}).  The grid is sized to the chip (a few workgroups per CU),
// each workgroup owns a contiguous, balanced run of whole units, and its waves split the run's concatenated 1 KiB tiles
// evenly -- a wave's range may cross stripe boundaries.  So:
//   * the activations are staged into LDS ONCE per workgroup (not once per stripe) as MFMA-ready fp16 rows (fp32/bf16
//     inputs split hi = fp16(a), lo = fp16(a - hi) so products are fp32-accurate), with the act-order gather of
//     ShuffleActivationKBlock (bestla_prologue_a.h:407-422) applied while staging;
//   * every wave keeps 2 x CH tiles (+ their group scales / zero points) in flight with a double-buffered register
//     pipeline, so the HBM stream never waits on compute, and no byte is loaded twice;
//   * per tile: 1 global_load_dwordx4 (16 B/lane, fully coalesced), SPT = KT/32 x {ds_read_b128 of A, 4 v_and_or +
//     4 v_pk_add_f16 (0x6400 magic dequant -> exact integer fp16), v_mfma_f32_16x16x32_f16}, one fp32 FMA of the group
//     accumulator by its scale at each group end;
//   * a wave's partial sums per stripe segment go to an LDS slot; after ONE barrier the workgroup sums the slots of
//     each stripe in wave order (deterministic, no atomics) and applies the fused epilogue.
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
__device__ int nad_trace_grid;  // record only launches with this many workgroups (0: all)
#define NAD_TRACE_ON (blockIdx.x < kTraceMaxWg)
#define NAD_TRACE(slot)                                                                              \
  do {                                                                                               \
    if (threadIdx.x == 0 && NAD_TRACE_ON) nad_trace_buf[slot][blockIdx.x] = wall_clock64(); \
  } while (0)
#define NAD_TRACE_MAX(slot)                                                                             \
  do {                                                                                                  \
    if ((threadIdx.x & 63) == 0 && NAD_TRACE_ON)                                            \
      atomicMax(&nad_trace_buf[slot][blockIdx.x], (unsigned long long)wall_clock64());                  \
  } while (0)
#define NAD_TRACE_ID()                                                                                  \
  do {                                                                                                  \
    if (threadIdx.x == 0 && NAD_TRACE_ON)                                                               \
      nad_trace_buf[kTraceSlots - 1][blockIdx.x] =                                                      \
          (unsigned long long)__smid() | ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32); \
  } while (0)
#else
#define NAD_TRACE(slot) \
  do {                  \
  } while (0)
#define NAD_TRACE_MAX(slot) \
  do {                      \
  } while (0)
#define NAD_TRACE_ID() \
  do {                 \
  } while (0)
#endif

constexpr int kGemvCH = 4;  // tiles per pipeline stage (2 stages in flight per wave)

// a group scale from the dword loaded by load_stage: f32 as is, 16-bit types from the half selected by `sh`
__device__ __forceinline__ float scale_bits_to_f32(uint32_t x, int st, int sh) {
  if (st == kScaleF32) return __uint_as_float(x);
  const uint32_t h = (x >> sh) & 0xFFFFu;
  return st == kScaleBF16 ? __uint_as_float(h << 16) : f16_bits_to_f32(uint16_t(h));
}

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

// One pipeline stage: CH weight tiles of this wave's flat range plus the raw group scale / zero-point values they need.
template <int GPT>
struct Stage {
  u4_t b[kGemvCH];
  uint32_t sc[kGemvCH][GPT];
  int zp[kGemvCH][GPT];
};

constexpr int kOOB = 0x7FFF0000;  // a buffer offset past every resource: the load returns 0 and touches no memory

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}

// The load cursor: where the next tile / group-scale / zero-point loads of this wave come from.  Everything here is
// wave-uniform (SGPRs); advancing by one tile is a handful of SALU ops, and the weight / stripe is re-derived only when
// the cursor crosses a stripe boundary.
struct LoadCursor {
  int f, f1;             // flat tile index in the workgroup's run, end of this wave's range
  int j, t;              // local virtual stripe, tile within it
  int toff, tstr;        // tile byte offset in the weight's tile array, bytes between consecutive K tiles
  int soff, gstr;        // scale-row byte offset of the tile's (first) group, bytes between consecutive groups
  int zoff, zstr;        // the same for the int8 zero points
  int g0;                // first group of the tile
  __amdgpu_buffer_rsrc_t rt, rs, rz;
};

template <int GPT>
__device__ __forceinline__ void cursor_seek(const GemvArgs& a, LoadCursor& c, int v0) {
  int w, s;
  vstripe(a, v0 + c.j, w, s);
  const int nt = a.nt, ng = a.ng;
  const int ns = sel3(w, a.w[0].ns, a.w[1].ns, a.w[2].ns);
  const int km = sel3(w, a.w[0].kmajor, a.w[1].kmajor, a.w[2].kmajor);
  const int ssz = a.scale_t == kScaleF32 ? 4 : 2;
  c.rt = rsrc(sel3(w, a.w[0].tiles, a.w[1].tiles, a.w[2].tiles), ns * nt * 1024);
  c.rs = rsrc(sel3(w, a.w[0].scales, a.w[1].scales, a.w[2].scales), ns * ng * 16 * ssz);
  c.rz = rsrc(sel3(w, a.w[0].zps, a.w[1].zps, a.w[2].zps), ns * ng * 16);
  c.toff = int(tile_index(km, ns, nt, s, c.t)) * 1024;
  c.tstr = km ? ns * 1024 : 1024;
  c.g0 = GPT == 1 ? (c.t >> a.tpg_shift) : c.t * GPT;
  const int row = int(scale_row(km, ns, ng, s, c.g0));
  c.soff = row * 16 * ssz;
  c.zoff = row * 16;
  c.gstr = (km ? ns : 1) * 16 * ssz;
  c.zstr = (km ? ns : 1) * 16;
}

template <int GPT>
__device__ __forceinline__ void cursor_next(const GemvArgs& a, LoadCursor& c, int v0) {
  c.f++;
  if (++c.t == a.nt) {
    c.t = 0;
    c.j++;
    cursor_seek<GPT>(a, c, v0);
    return;
  }
  c.toff += c.tstr;
  if constexpr (GPT == 1) {
    if ((c.t & a.tpg_mask) == 0) {
      c.g0++;
      c.soff += c.gstr;
      c.zoff += c.zstr;
    }
  } else {
    c.g0 += GPT;
    c.soff += GPT * c.gstr;
    c.zoff += GPT * c.zstr;
  }
}

// Issue the loads of the next CH tiles: per tile one buffer_load_dwordx4 (nt) of the 1 KiB tile and GPT dword loads of
// its group scales (+ zero points).  Every load is issued unconditionally -- tiles past the wave's range and groups past
// K get an out-of-range offset (no memory traffic) -- so every stage has the same vmcnt footprint and the compiler can
// wait for exactly one stage.  The per-lane work is one v_add per load.
template <int BITS, int GPT, bool ASYM>
__device__ __forceinline__ void load_stage(const GemvArgs& a, Stage<GPT>& S, LoadCursor& c, int v0, int lane, int vs) {
#pragma unroll
  for (int i = 0; i < kGemvCH; i++) {
    const bool over = c.f >= c.f1;
    S.b[i] = __builtin_bit_cast(u4_t, __builtin_amdgcn_raw_buffer_load_b128(c.rt, (over ? kOOB : c.toff) + lane * 16, 0, 2));
#pragma unroll
    for (int q = 0; q < GPT; q++) {
      const bool gin = !over && (GPT == 1 || c.g0 + q < a.ng);
#ifdef NAD_EXP_NOSCALE
      S.sc[i][q] = 0x3C003C00u;
#else
      S.sc[i][q] = __builtin_amdgcn_raw_buffer_load_b32(c.rs, (gin ? c.soff + q * c.gstr : kOOB) + vs, 0, 0);
#endif
      if constexpr (ASYM) {
        S.zp[i][q] = int(int8_t(__builtin_amdgcn_raw_buffer_load_b8(c.rz, (gin ? c.zoff + q * c.zstr : kOOB) + (lane & 15), 0, 0)));
      } else {
        S.zp[i][q] = 0;
      }
    }
    if (!over) cursor_next<GPT>(a, c, v0);
  }
}

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

// element-wise staging (act-order gather, unaligned rows, K % 8 != 0): rolled, runs before any weight load
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

template <int BITS, int HILO, int GPT, bool ASYM>
__global__ __launch_bounds__(1024) void woq_gemv_kernel(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KT = BITS == 4 ? 128 : (BITS == 2 ? 256 : 64);
  constexpr int SPT = KT / 32;
  constexpr int CH = kGemvCH;
  static_assert(SPT % GPT == 0, "groups must tile the K tile");
  constexpr int SPG = SPT / GPT;  // steps per group when GPT > 1
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int NW = __builtin_amdgcn_readfirstlane(int(blockDim.x >> 6));
  const int M = a.M, nt = a.nt, Kp = nt * KT;
  const int R = HILO == 0 ? M : 2 * M;
  NAD_TRACE(0);
  NAD_TRACE_ID();

  // this workgroup's units and this wave's flat tile range (all wave-uniform)
  const int G = gridDim.x, bid = blockIdx.x;
  const int u0 = int(unsigned(bid) * unsigned(a.units) / unsigned(G));
  const int u1 = int(unsigned(bid + 1) * unsigned(a.units) / unsigned(G));
  const int vpu = a.dual ? 2 : 1;
  const int v0 = u0 * vpu, nv = (u1 - u0) * vpu;
  const int T = nv * nt;
  const int f0 = int(unsigned(wave) * unsigned(T) / unsigned(NW));
  const int f1 = int(unsigned(wave + 1) * unsigned(T) / unsigned(NW));

  // 1) activations -> LDS (once per workgroup) overlapped with the first two weight stages
  const int a_units = M * (Kp >> 3);
  const int bd = blockDim.x;
  Stage<GPT> S0, S1;
  LoadCursor lc;
  lc.f = f0;
  lc.f1 = f1;
  {
    const int j0 = f0 / nt;
    lc.j = __builtin_amdgcn_readfirstlane(j0);
    lc.t = __builtin_amdgcn_readfirstlane(f0 - j0 * nt);
  }
  cursor_seek<GPT>(a, lc, v0);
  const int vs = a.scale_t == kScaleF32 ? (lane & 15) * 4 : (lane & 14) * 2;
  if (a.a_fast) {
    constexpr int AR = 2;  // units per thread issued ahead of the weights
    const int esz = a.act_t == kActF32 ? 4 : 2;
    const auto ra = rsrc(a.A, (M - 1) * a.lda * esz + a.K * esz);
    uint4 x[AR][2];
#pragma unroll
    for (int q = 0; q < AR; q++) {
      const int u = q * bd + int(threadIdx.x);
      const int row = u / (Kp >> 3), k = (u - row * (Kp >> 3)) * 8;
#ifdef NAD_EXP_NOA
      const int off = kOOB;
#else
      const int off = (u < a_units && k < a.K) ? (row * a.lda + k) * esz : kOOB;
#endif
      x[q][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
      x[q][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, off + 16, 0, 0));
    }
    NAD_TRACE(4);
    load_stage<BITS, GPT, ASYM>(a, S0, lc, v0, lane, vs);
    load_stage<BITS, GPT, ASYM>(a, S1, lc, v0, lane, vs);
    NAD_TRACE(5);
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
    load_stage<BITS, GPT, ASYM>(a, S0, lc, v0, lane, vs);
    load_stage<BITS, GPT, ASYM>(a, S1, lc, v0, lane, vs);
  }
  {
    uint4* zr = reinterpret_cast<uint4*>(smem + size_t(R) * Kp * 2);
    for (int i = threadIdx.x; i < (Kp >> 3); i += bd) zr[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();
  NAD_TRACE(1);

  float* part = reinterpret_cast<float*>(smem + a.part_off);  // [slot][M][16]
  const int m = lane & 15;   // MFMA A row fed by this lane
  const int kq = lane >> 4;  // k-quarter of a 32-k step
  const int arow = HILO == 1 ? (m & 7) : m;
  const bool is_lo = HILO == 1 && m >= 8;
  const int row_hi = arow < M ? (is_lo ? M + arow : arow) : R;  // inactive rows read the zero row
  const int row_lo = arow < M ? M + arow : R;
  const char* a_hi = smem + size_t(row_hi) * Kp * 2 + kq * 16;
  const char* a_lo = smem + size_t(row_lo) * Kp * 2 + kq * 16;
  const h2_t cdef = zp_const(bias_of<BITS>());
  const int ssh = a.scale_t == kScaleF32 ? 0 : (lane & 1) * 16;  // this lane's half of a 16-bit scale pair

  f4_t acc = {0.f, 0.f, 0.f, 0.f};
  f4_t accg = {0.f, 0.f, 0.f, 0.f};

  // compute cursor (wave-uniform): flat index, local stripe, tile
  int cf = f0, cj = lc.j, ct = 0;
  {
    const int j0 = f0 / nt;
    cj = __builtin_amdgcn_readfirstlane(j0);
    ct = __builtin_amdgcn_readfirstlane(f0 - j0 * nt);
  }
  auto compute_stage = [&](const Stage<GPT>& S) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      if (cf < f1) {
        const bool seg_end = (ct == nt - 1) || (cf == f1 - 1);
        const bool tile_gend = GPT == 1 ? (((ct + 1) & a.tpg_mask) == 0 || ct == nt - 1) : true;
        const int kb = ct * KT * 2;
#pragma unroll
        for (int d = 0; d < SPT; d++) {
          const int q = GPT == 1 ? 0 : d / SPG;
          h2_t c2 = cdef;
          if constexpr (ASYM) c2 = zp_const(bias_of<BITS>() + S.zp[i][q]);
#ifdef NAD_EXP_NOCOMPUTE
          if (d == 0) acc[0] += __uint_as_float(S.b[i][0] ^ S.b[i][1] ^ S.b[i][2] ^ S.b[i][3]) + scale_bits_to_f32(S.sc[i][0], a.scale_t, ssh);
          continue;
#endif
          const h8_t bf = dequant_step<BITS>(S.b[i], d, c2);
          const h8_t af = *reinterpret_cast<const h8_t*>(a_hi + kb + d * 64);
          accg = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, accg, 0, 0, 0);
          if constexpr (HILO == 2) {
            const h8_t afl = *reinterpret_cast<const h8_t*>(a_lo + kb + d * 64);
            accg = __builtin_amdgcn_mfma_f32_16x16x32_f16(afl, bf, accg, 0, 0, 0);
          }
          if constexpr (GPT > 1) {
            if ((d + 1) % SPG == 0) {
              acc += accg * scale_bits_to_f32(S.sc[i][q], a.scale_t, ssh);
              accg = f4_t{0.f, 0.f, 0.f, 0.f};
            }
          }
        }
        // GPT == 1: the group ends at this tile, or the wave's range ends inside it (a linear partial of the group)
        if (GPT == 1 && (tile_gend || seg_end)) {
          acc += accg * scale_bits_to_f32(S.sc[i][0], a.scale_t, ssh);
          accg = f4_t{0.f, 0.f, 0.f, 0.f};
        }
        if (seg_end) {
          f4_t r = acc;
          if constexpr (HILO == 1) {
#pragma unroll
            for (int x = 0; x < 4; x++) r[x] += __shfl_down(r[x], 32, 64);
          }
          // rows (lane >> 4) * 4 + x live in this lane; slot = local stripe + wave (distinct for all (wave, stripe))
          float* ps = part + size_t(cj + wave) * M * 16 + (lane & 15);
#pragma unroll
          for (int x = 0; x < 4; x++) {
            const int row = (lane >> 4) * 4 + x;
            if (row < M && (HILO != 1 || lane < 32)) ps[row * 16] = r[x];
          }
          acc = f4_t{0.f, 0.f, 0.f, 0.f};
        }
        cf++;
        if (++ct == nt) {
          ct = 0;
          cj++;
        }
      }
    }
  };

  bool first = true;
  while (cf < f1) {
    compute_stage(S0);
    if (first) NAD_TRACE_MAX(6);
    first = false;
    load_stage<BITS, GPT, ASYM>(a, S0, lc, v0, lane, vs);
    compute_stage(S1);
    load_stage<BITS, GPT, ASYM>(a, S1, lc, v0, lane, vs);
  }
  NAD_TRACE_MAX(2);
  __syncthreads();

  // 2) sum each stripe's slots in wave order and apply the epilogue
  const int nout = (u1 - u0) * M * 16;
  for (int o = threadIdx.x; o < nout; o += bd) {
    const int p = o / (M * 16), mm = (o >> 4) % M, nn = o & 15;
    float y[2] = {0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (h < vpu) {
        // waves whose ranges meet stripe j: wave(x) = ((x + 1) * NW - 1) / T holds flat tile x; empty waves skipped
        const int j = p * vpu + h;
        const int wlo = int((unsigned(j * nt + 1) * unsigned(NW) - 1u) / unsigned(T));
        const int whi = int((unsigned((j + 1) * nt) * unsigned(NW) - 1u) / unsigned(T));
        const float* ps = part + (size_t(j) * M + mm) * 16 + nn;
        const size_t wst = size_t(M) * 16;
        if (T >= NW) {  // no empty waves: four independent LDS reads per step
          float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
          int w = wlo;
          for (; w + 3 <= whi; w += 4) {
            s0 += ps[size_t(w) * wst];
            s1 += ps[size_t(w + 1) * wst];
            s2 += ps[size_t(w + 2) * wst];
            s3 += ps[size_t(w + 3) * wst];
          }
          for (; w <= whi; w++) s0 += ps[size_t(w) * wst];
          y[h] = (s0 + s1) + (s2 + s3);
        } else {
          for (int w = wlo; w <= whi; w++) {
            const bool nonempty =
                (unsigned(w + 1) * unsigned(T)) / unsigned(NW) > (unsigned(w) * unsigned(T)) / unsigned(NW);
            if (nonempty) y[h] += ps[size_t(w) * wst];
          }
        }
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

// ------------------------------------------------------------------------------------------------ launcher
template <int BITS, int HILO, int GPT, bool ASYM>
static hipError_t gemv_launch4(const GemvArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  auto k = woq_gemv_kernel<BITS, HILO, GPT, ASYM>;
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

// Instantiated: GPT 1 and 2 (group >= KT/2), sym and asym; GPT 4 (KT/4 groups) sym only.  Finer groups fall back to
// woq_skinny_kernel (their per-group scale/zero registers would spill).
template <int BITS, int HILO>
static hipError_t gemv_launch2(const GemvArgs& a, int gpt, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  constexpr int SPT = (BITS == 4 ? 128 : (BITS == 2 ? 256 : 64)) / 32;
  if (gpt == 1) return a.asym ? gemv_launch4<BITS, HILO, 1, true>(a, g, b, lds, st)
                              : gemv_launch4<BITS, HILO, 1, false>(a, g, b, lds, st);
  if (gpt == 2) return a.asym ? gemv_launch4<BITS, HILO, 2, true>(a, g, b, lds, st)
                              : gemv_launch4<BITS, HILO, 2, false>(a, g, b, lds, st);
  if constexpr (SPT % 4 == 0) {
    if (gpt == 4 && !a.asym) return gemv_launch4<BITS, HILO, 4, false>(a, g, b, lds, st);
  }
  return hipErrorInvalidValue;
}

template <int BITS>
static hipError_t gemv_launch1(const GemvArgs& a, int hilo, int gpt, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  if (hilo == 0) return gemv_launch2<BITS, 0>(a, gpt, g, b, lds, st);
  if (hilo == 1) return gemv_launch2<BITS, 1>(a, gpt, g, b, lds, st);
  return gemv_launch2<BITS, 2>(a, gpt, g, b, lds, st);
}

size_t gemv_lds_bytes(const GemvArgs& a, int bits, int waves, int grid, int* part_off, int* part_bytes) {
  const int KT = bits == 4 ? 128 : (bits == 2 ? 256 : 64);
  const int R = a.act_t == kActF16 ? a.M : 2 * a.M;
  const size_t kp = size_t(a.nt) * KT;
  const size_t abytes = (size_t(R) + 1) * kp * 2;
  const int upw = (a.units + grid - 1) / grid;  // max units per workgroup
  const size_t slots = size_t(upw) * (a.dual ? 2 : 1) + waves;
  *part_off = int(abytes);
  *part_bytes = int(slots * a.M * 16 * 4);
  return abytes + *part_bytes + (waves + 1) * 4;
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

hipError_t launch_gemv(const GemvArgs& a, int bits, int waves, int grid, size_t lds, hipStream_t stream) {
  const int hilo = a.act_t == kActF16 ? 0 : (a.M <= 8 ? 1 : 2);
  int tpg = 0;
  const int gpt = gemv_groups_per_tile(bits, a.nt, a.ng, a.bs, &tpg);
  if (gpt == 0) return hipErrorInvalidValue;
  dim3 g(grid), b(waves * 64);
  if (bits == 4) return gemv_launch1<4>(a, hilo, gpt, g, b, lds, stream);
  if (bits == 2) return gemv_launch1<2>(a, hilo, gpt, g, b, lds, stream);
  return gemv_launch1<8>(a, hilo, gpt, g, b, lds, stream);
}

}  // namespace nad

#ifdef NAD_PHASE_TRACE
extern "C" int nad_trace_clock_khz() {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return -1;
  return khz;
}

extern "C" int nad_trace_fetch(void* host, size_t bytes, int clear, int grid_filter) {
  const size_t n = sizeof(nad::nad_trace_buf) < bytes ? sizeof(nad::nad_trace_buf) : bytes;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (host && hipMemcpyFromSymbol(host, HIP_SYMBOL(nad::nad_trace_buf), n) != hipSuccess) return -1;
  if (clear) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(nad::nad_trace_buf)) != hipSuccess) return -1;
    if (hipMemset(p, 0, sizeof(nad::nad_trace_buf)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(nad::nad_trace_grid), &grid_filter, sizeof(int)) != hipSuccess) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
  }
  return 0;
}
#endif
