// woq_chain.hip -- a whole decode step's WOQ matmuls in ONE persistent launch (the decode chain).
//
// What it replaces: the sequence of device WOQ nodes one decode token runs through the ne graph
// (ne_compute_forward_mul_mat_q_f32_bestla -> bestla_device_f32f32_forward, neural_speed/core/ne_layers.c:7219-7316;
// fused QKV / FFN nodes, ne_layers.c:8050-8170), i.e. what BTLAGemmBatchDriver (core/layers/bestla_gemm.cpp:508-624)
// does for a batch of independent GEMMs, extended with the data dependencies between consecutive matmuls.
//
// Why: measured on MI355X (profiles/r01_decode_calibration.md) every separate decode launch pays ~5 us during which
// HBM is mostly idle -- the kernel boundary (~1.8 us), the prologue (cold instruction cache, activation staging,
// first weight loads ~2.5-3 us) and the epilogue (~0.7 us).  Over 129 launches per Llama-2-7B token that is about
// half of the token time.  Here one workgroup per CU stays resident for the whole step and, for every op:
//   1. issues the first three weight stages of the op (they do not depend on the activations) -- these loads stream
//      from HBM while the workgroup waits for the previous op;
//   2. wave 0 polls the per-workgroup arrival flags (one 16-B sc1 load per lane) until every workgroup has
//      published the previous op;
//   3. stages the op's activations (optionally RMS-normalised) into LDS as MFMA-ready fp16 hi/lo rows;
//   4. runs the stripe stream of woq_gemv.hip (same tiles, same dequant, same MFMA and reduction order, so every
//      op's output is bit-identical to the single-op launch);
//   5. publishes its outputs with write-through (sc1) stores, waits for them, and sets its own flag to op + 1.
// Hand-off protocol (MI355X_MICROARCH.md, "Hand-offs measured with sc1 loads", row 1): every load of chain-produced
// data (activations, residuals) is an sc1 load, every store of it an sc1 store, each storing wave waits vmcnt(0)
// before the workgroup barrier that precedes the one-lane sc1 flag store; the polling wave's loads follow its
// matching poll, the other waves' follow the barrier it then joins.  All workgroups must be co-resident: the grid is
// one workgroup per CU and the LDS request (> 80 KiB) admits no second one.  Every spin is bounded; a timeout sets
// status[0] and the launch still terminates.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "woq_chain.h"
#include "woq_device.h"
#include "woq_kernels.h"

namespace nad {
namespace chain {

// Development instrumentation (make chaintrace): per-(op, workgroup) wall-clock stamps of the chain's phases.
#ifdef NAD_CHAIN_TRACE
constexpr int kTrOps = 160, kTrWg = 256, kTrSlots = 6;
__device__ unsigned long long nad_chain_trace[kTrSlots][kTrOps][kTrWg];
#define CTRACE(slot)                                                                                      \
  do {                                                                                                    \
    if (threadIdx.x == 0 && op < kTrOps && blockIdx.x < kTrWg) nad_chain_trace[slot][op][blockIdx.x] = wall_clock64(); \
  } while (0)
#else
#define CTRACE(slot) \
  do {               \
  } while (0)
#endif

constexpr int kOOB = 0x7FFF0000;  // buffer offset past every resource: the load returns 0 and touches no memory
constexpr int kSC1 = 16;          // cache-policy aux bit of buffer loads: sc1 (bypass the CU's L1)
constexpr int KS = 4;             // tiles per K-slice (woq_gemv.hip)

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

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct StageCursor {
  int j, q, s;
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

template <bool ASYM>
struct StageRegs {
  u4_t b[KS];
  uint32_t sc[KS];
  int zp[KS];
};

// one stage = KS tiles of one (stripe, K-slice) + their group scales (never predicated: out-of-range offsets)
template <bool ASYM>
__device__ __forceinline__ void load_stage(const GemvArgs& a, StageRegs<ASYM>& S, StageCursor& c, int nv, int nsl,
                                           int wave, int NW, int v0, int lane, int vs) {
  if (c.j >= nv) {
#pragma unroll
    for (int i = 0; i < KS; i++) {
      S.b[i] = __builtin_bit_cast(u4_t, __builtin_amdgcn_raw_buffer_load_b128(c.rt, kOOB, 0, 2));
      S.sc[i] = __builtin_amdgcn_raw_buffer_load_b32(c.rs, kOOB, 0, 0);
      S.zp[i] = ASYM ? int(int8_t(__builtin_amdgcn_raw_buffer_load_b8(c.rz, kOOB, 0, 0))) : 0;
    }
    return;
  }
  const int nt = a.nt;
  const int t0 = c.q * KS;
  const int tb = (c.s * nt + t0) * 1024;
  const int rowb = a.scale_t == kScaleF32 ? 64 : 32;
#pragma unroll
  for (int i = 0; i < KS; i++) {
    const bool live = t0 + i < nt;
    S.b[i] = __builtin_bit_cast(u4_t, __builtin_amdgcn_raw_buffer_load_b128(c.rt, (live ? tb + i * 1024 : kOOB) + lane * 16, 0, 2));
    const int row = c.s * a.ng + ((t0 + i) >> a.tpg_shift);
    S.sc[i] = __builtin_amdgcn_raw_buffer_load_b32(c.rs, (live ? row * rowb : kOOB) + vs, 0, 0);
    if constexpr (ASYM)
      S.zp[i] = int(int8_t(__builtin_amdgcn_raw_buffer_load_b8(c.rz, (live ? row * 16 : kOOB) + (lane & 15), 0, 0)));
    else
      S.zp[i] = 0;
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

// (x & m) | c in one VOP3
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

// int4: 0x6400 | nibble<<0 = 1024 + q, 0x6400 | nibble<<4 = 1024 + 16 q (exact fp16), one shift per dword
__device__ __forceinline__ h8_t dequant4(uint32_t w, uint32_t m0, uint32_t m1, uint32_t mag, h2_t s16, h2_t c0,
                                         h2_t c1) {
  const uint32_t w8 = w >> 8;
  const h2_t p0 = as_h2(and_or(w, m0, mag)) + c0;
  const h2_t p1 = as_h2(and_or(w, m1, mag)) * s16 + c1;
  const h2_t p2 = as_h2(and_or(w8, m0, mag)) + c0;
  const h2_t p3 = as_h2(and_or(w8, m1, mag)) * s16 + c1;
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

__device__ __forceinline__ float scale_bits_to_f32(uint32_t x, int st, int sh) {
  const uint32_t h = (x >> sh) & 0xFFFFu;
  const float fb = __uint_as_float(h << 16);
  const float fh = f16_bits_to_f32(uint16_t(h));
  const float f16or = st == kScaleBF16 ? fb : fh;
  return st == kScaleF32 ? __uint_as_float(x) : f16or;
}

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

// ------------------------------------------------------------------------------------------------ the kernel
constexpr int AR = 3;  // activation staging units (8 elements) per thread held in registers

template <int HILO, bool ASYM>
__global__ __launch_bounds__(768) void woq_chain_kernel(const GemvArgs* __restrict__ ops, int n_ops,
                                                         unsigned* flags, unsigned* status, int npre) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KT = 128, SPT = 4, BIAS = 8;  // int4, one group per >= one K tile (host-checked)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int NW = __builtin_amdgcn_readfirstlane(int(blockDim.x >> 6));
  const int G = gridDim.x, bid = blockIdx.x, bd = blockDim.x, tid = threadIdx.x;
  const uint32_t m0 = 0x000F000Fu, m1 = 0x00F000F0u, mag = 0x64006400u;
  const h2_t s16 = splat(1.f / 16.f);
  bool gave_up = false;

  for (int op = 0; op < n_ops; op++) {
    const GemvArgs& a = ops[op];
    const int M = a.M, nt = a.nt, Kp = nt * KT;
    const int R = HILO == 0 ? M : 2 * M;
    const int nsl = (nt + KS - 1) / KS;
    const int NWa = a.nwa;  // waves owning K slices: as in the single-op launch, so the sums match it bit for bit
    const int u0 = int(unsigned(bid) * unsigned(a.units) / unsigned(G));
    const int u1 = int(unsigned(bid + 1) * unsigned(a.units) / unsigned(G));
    const int vpu = a.dual ? 2 : 1;
    const int v0 = u0 * vpu, nv = (u1 - u0) * vpu;
    const bool idle = wave >= nsl || wave >= NWa;
    float* part = reinterpret_cast<float*>(smem + a.part_off);  // [nv][NWa][M][16]
    const int vs = a.scale_t == kScaleF32 ? (lane & 15) * 4 : (lane & 14) * 2;

    // 1) the first three weight stages of this op (independent of the activations): in flight during the wait
    StageCursor lc;
    lc.j = idle ? nv : 0;
    lc.q = wave;
    lc.s = 0;
    lc.rt = rsrc(a.w[0].tiles, 0);
    lc.rs = lc.rt;
    lc.rz = lc.rt;
    if (!idle && nv > 0) cursor_stripe(a, lc, v0);
    StageRegs<ASYM> S0, S1, S2;
    CTRACE(0);
    if (wave != 0 && npre) {
      load_stage<ASYM>(a, S0, lc, nv, nsl, wave, NWa, v0, lane, vs);
      load_stage<ASYM>(a, S1, lc, nv, nsl, wave, NWa, v0, lane, vs);
      load_stage<ASYM>(a, S2, lc, nv, nsl, wave, NWa, v0, lane, vs);
    }

    // 2) wave 0 waits until every workgroup has published ops 0..op-1, then issues its own stages
    if (wave == 0) {
      if (op > 0 && !gave_up) {
        // every workgroup's flag >= op: lane l checks flags 4l..4l+3 with one sc1 16-B load (no atomics, no
        // fan-in serialisation: measured single-counter barriers cost ~7 us at 256 workgroups)
        const auto rf = rsrc(flags, G * 4);
        const unsigned target = unsigned(op);
        unsigned spins = 0;
        while (true) {
          const uint4 f4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rf, lane * 16, 0, kSC1));
          const bool ok = lane * 4 >= G || ((f4.x >= target || lane * 4 + 0 >= G) && (f4.y >= target || lane * 4 + 1 >= G) &&
                                            (f4.z >= target || lane * 4 + 2 >= G) && (f4.w >= target || lane * 4 + 3 >= G));
          if (__all(ok)) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (1u << 21)) {  // ~1 s: never expected; record it, stop waiting, and run on rather than hang
            if (lane == 0) __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            gave_up = true;
            break;
          }
        }
      }
      load_stage<ASYM>(a, S0, lc, nv, nsl, wave, NWa, v0, lane, vs);
      load_stage<ASYM>(a, S1, lc, nv, nsl, wave, NWa, v0, lane, vs);
      load_stage<ASYM>(a, S2, lc, nv, nsl, wave, NWa, v0, lane, vs);
    }
    __syncthreads();
    if (wave != 0 && !npre) {
      load_stage<ASYM>(a, S0, lc, nv, nsl, wave, NWa, v0, lane, vs);
      load_stage<ASYM>(a, S1, lc, nv, nsl, wave, NWa, v0, lane, vs);
      load_stage<ASYM>(a, S2, lc, nv, nsl, wave, NWa, v0, lane, vs);
    }
    CTRACE(1);

    // 3) stage the activations (sc1 loads: they may come from another workgroup of this launch)
    const int KU = Kp >> 3;
    const int a_units = M * KU;
    const int esz = a.act_t == kActF32 ? 4 : 2;
    const auto ra = rsrc(a.A, (M - 1) * a.lda * esz + a.K * esz);
    float f[AR][8];
#pragma unroll
    for (int q = 0; q < AR; q++) {
      const int u = q * bd + tid;
      const int row = u / KU, k = (u - row * KU) * 8;
      const int off = (u < a_units && k < a.K) ? (row * a.lda + k) * esz : kOOB;
      const uint4 x0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, kSC1));
      const uint4 x1 = a.act_t == kActF32
                           ? __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, off + 16, 0, kSC1))
                           : make_uint4(0u, 0u, 0u, 0u);
      unit_to_f32(a.act_t, x0, x1, f[q]);
    }
    if (a.norm) {  // RMSNorm of each row: per-wave row sums in LDS, combined in wave order (deterministic)
      float* slot = reinterpret_cast<float*>(smem + a.part_off);  // [NW][8] scratch: partial slots not live yet
      float rs[8];
#pragma unroll
      for (int r = 0; r < 8; r++) rs[r] = 0.f;
#pragma unroll
      for (int q = 0; q < AR; q++) {
        const int u = q * bd + tid;
        float s2 = 0.f;
#pragma unroll
        for (int j = 0; j < 8; j++) s2 += f[q][j] * f[q][j];
        const int row = u < a_units ? u / KU : 8;
#pragma unroll
        for (int r = 0; r < 8; r++) rs[r] += row == r ? s2 : 0.f;
      }
      for (int r = 0; r < M; r++) {
        float v = rs[r];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) slot[wave * 8 + r] = v;
      }
      __syncthreads();
      float inv[8];
#pragma unroll
      for (int r = 0; r < 8; r++) {
        float tot = 0.f;
        if (r < M)
          for (int w = 0; w < NW; w++) tot += slot[w * 8 + r];
        inv[r] = 1.f / sqrtf(tot / float(a.K) + a.norm_eps);
      }
#pragma unroll
      for (int q = 0; q < AR; q++) {
        const int u = q * bd + tid;
        const int row = min(u / KU, M - 1), k = (u - (u / KU) * KU) * 8;
        float r = inv[0];
#pragma unroll
        for (int rr = 1; rr < 8; rr++) r = row == rr ? inv[rr] : r;
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const float g = (a.norm_w != nullptr && k + j < a.K) ? a.norm_w[k + j] : 1.f;
          f[q][j] = f[q][j] * r * g;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < AR; q++) {
      const int u = q * bd + tid;
      if (u < a_units) unit_store<HILO>(smem, f[q], u / KU, (u - (u / KU) * KU) * 8, M, Kp);
    }
    {
      uint4* zr = reinterpret_cast<uint4*>(smem + size_t(R) * Kp * 2);
      for (int i = tid; i < (Kp >> 3); i += bd) zr[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();
    CTRACE(2);

    // 4) the stripe stream (woq_gemv.hip)
    const int m = lane & 15;
    const int kq = lane >> 4;
    const int arow = HILO == 1 ? (m & 7) : m;
    const bool is_lo = HILO == 1 && m >= 8;
    const int row_hi = arow < M ? (is_lo ? M + arow : arow) : R;
    const char* a_hi = smem + size_t(row_hi) * Kp * 2 + kq * 16;
    const int ssh = a.scale_t == kScaleF32 ? 0 : (lane & 1) * 16;
    const h2_t zc0 = splat(-(1024.f + BIAS)), zc1 = splat(-(64.f + BIAS));

    f4_t acc = {0.f, 0.f, 0.f, 0.f};
    int cj = idle ? nv : 0, cq = wave;

    auto compute_stage = [&](const StageRegs<ASYM>& S) {
      if (cj >= nv) return;
      const int t0 = cq * KS;
      const char* ab = a_hi + t0 * KT * 2;
      f4_t accg[KS];  // as woq_gemv.hip: KS independent chains, step-major, scaled per tile in tile order
#pragma unroll
      for (int d = 0; d < SPT; d++) {
#pragma unroll
        for (int i = 0; i < KS; i++) {
          const int ti = min(t0 + i, nt - 1) - t0;
          h8_t bf;
          if constexpr (ASYM) {
            const float z = float(S.zp[i]);
            bf = dequant4(S.b[i][d], m0, m1, mag, s16, zc0 - splat(z), zc1 - splat(z));
          } else {
            bf = dequant4(S.b[i][d], m0, m1, mag, s16, zc0, zc1);
          }
          const h8_t af = *reinterpret_cast<const h8_t*>(ab + ti * KT * 2 + d * 64);
          accg[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, d == 0 ? f4_t{0.f, 0.f, 0.f, 0.f} : accg[i], 0, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < KS; i++) acc += accg[i] * scale_bits_to_f32(S.sc[i], a.scale_t, ssh);
      cq += NWa;
      if (cq >= nsl) {
        f4_t r = acc;
        if constexpr (HILO == 1) {
#pragma unroll
          for (int xx = 0; xx < 4; xx++) r[xx] += __shfl_down(r[xx], 32, 64);
        }
        float* ps = part + (size_t(cj) * NWa + wave) * M * 16 + m;
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
      compute_stage(S0);
      load_stage<ASYM>(a, S0, lc, nv, nsl, wave, NWa, v0, lane, vs);
      compute_stage(S1);
      load_stage<ASYM>(a, S1, lc, nv, nsl, wave, NWa, v0, lane, vs);
      compute_stage(S2);
      load_stage<ASYM>(a, S2, lc, nv, nsl, wave, NWa, v0, lane, vs);
    }
    __syncthreads();
    CTRACE(3);

    // 5) reduce in wave order, epilogue, write-through stores; then one arrival per workgroup
    const int nout = (u1 - u0) * M * 16;
    const int nwl = min(NWa, nsl);
    for (int o = tid; o < nout; o += bd) {
      const int p = o / (M * 16), mm = (o >> 4) % M, nn = o & 15;
      float y[2] = {0.f, 0.f};
#pragma unroll
      for (int h = 0; h < 2; h++) {
        if (h < vpu) {
          const float* ps = part + (size_t(p * vpu + h) * NWa * M + mm) * 16 + nn;
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
          v += ld_sc1(a.res + size_t(mm) * a.ld_res + n);
          break;
        case kEpiSiluMul: {
          const float t1 = silu_f(y[0]);
          if (a.aux) st_sc1(a.aux + size_t(mm) * a.ld_aux + n, t1);
          v = t1 * y[1];
          break;
        }
        case kEpiGeluMul: {
          const float t1 = gelu_f(y[0]);
          if (a.aux) st_sc1(a.aux + size_t(mm) * a.ld_aux + n, t1);
          v = t1 * y[1];
          break;
        }
        default:
          break;
      }
      st_sc1(out + size_t(mm) * ldo + n, v);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(flags + bid, unsigned(op + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    CTRACE(4);
  }
}

}  // namespace chain

// ------------------------------------------------------------------------------------------------ host side
size_t chain_lds_layout(GemvArgs& a, int waves, int grid) {
  const int R = a.act_t == kActF16 ? a.M : 2 * a.M;
  const size_t kp = size_t(a.nt) * 128;
  const size_t abytes = (size_t(R) + 1) * kp * 2;
  const int upw = (a.units + grid - 1) / grid;
  const size_t nv = size_t(upw) * (a.dual ? 2 : 1);
  a.part_off = int((abytes + 15) & ~size_t(15));
  const size_t part = nv * waves * a.M * 16 * 4;
  const size_t norm_scratch = size_t(waves) * 8 * 4;  // RMSNorm per-wave row sums
  return size_t(a.part_off) + (part > norm_scratch ? part : norm_scratch);
}

hipError_t launch_chain(const GemvArgs* dev_ops, int n_ops, int hilo, int asym, int waves, int grid, size_t lds,
                        unsigned* flags, unsigned* status, int npre, hipStream_t st) {
  auto pick = [&](auto k) -> hipError_t {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(grid), dim3(waves * 64), lds, st, dev_ops, n_ops, flags, status, npre);
    return hipGetLastError();
  };
  if (hilo == 0) return asym ? pick(chain::woq_chain_kernel<0, true>) : pick(chain::woq_chain_kernel<0, false>);
  return asym ? pick(chain::woq_chain_kernel<1, true>) : pick(chain::woq_chain_kernel<1, false>);
}

}  // namespace nad

#ifdef NAD_CHAIN_TRACE
extern "C" int nad_chain_trace_fetch(void* host, size_t bytes) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const size_t n = sizeof(nad::chain::nad_chain_trace) < bytes ? sizeof(nad::chain::nad_chain_trace) : bytes;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(nad::chain::nad_chain_trace), n) == hipSuccess ? 0 : -1;
}
#endif
