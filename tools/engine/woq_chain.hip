// woq_chain.hip -- the decode weight-stream engine: a list of M = 1 WOQ matmuls in ONE persistent launch.
//
// What it replaces: the device WOQ nodes one decode step runs between two attention nodes
// (ne_compute_forward_mul_mat_q_f32_bestla -> bestla_device_f32f32_forward, neural_speed/core/ne_layers.c:7219-7316;
// the fused QKV / FFN nodes, ne_layers.c:8050-8170; op order llama.cpp:212-237,590-619,690-718), i.e. what
// BTLAGemmBatchDriver (core/layers/bestla_gemm.cpp:508-624) does for independent GEMMs, extended with the data
// dependencies between consecutive matmuls (the O -> gate/up -> down -> next QKV segment of a decoder layer).
//
// Why: a separate decode launch is bounded by its own fixed chain (kernel boundary ~1.2 us, first weight load issued
// ~0.5 us in, ~1.5 us of HBM latency before the stream runs, ~0.6 us reduce + epilogue), so one
// launch at a time cannot pass ~0.33-0.57 of the 8 TB/s roofline whatever its body does.  The weights of a decode step
// do not depend on the activations: here each CU's weight stream runs ahead of every data dependency.
//
// Shape (MI355X_MICROARCH.md rows ldsdma-fill, prefetch-credit, handoff-1to1, allgather; the engine-vs-launches row
// measured the same structure at 0.87-0.89x of separate launches for a bf16 layer):
//   * one workgroup per CU (the LDS request admits no second one), all co-resident; 10 waves: 8 consumers + 2 loaders
//     (one loader wave tops out near 20 GB/s per CU, two reach 27: tools/dma_probe.hip);
//   * every op's units (16-column stripes; {gate, up} stripe pairs for the dual SiLU*mul op) are split into balanced
//     runs per workgroup, exactly as the single-op stripe stream splits them;
//   * the LOADER waves walk the workgroup's fills for ALL ops of the launch in order (fill f by loader f mod 2) -- a
//     fill is 16 consecutive 1 KiB K tiles of one stripe + their group scales (+ zero points) -- and move each by LDS-DMA
//     (buffer_load_dwordx4 ... lds, non-temporal: read once per token) into a ring of LDS slots: one fill in flight per
//     loader (counted s_waitcnt vmcnt), a FULL word per slot published when its fill has landed, a slot re-filled only
//     when all 8 consumers have released it (FREE counter).  It never waits for activations, so it keeps streaming the
//     next op's weights while the consumers wait for that op's input;
//   * the 8 CONSUMER waves: per op, stage the input vector into LDS as MFMA-ready fp16 hi/lo rows (hi = fp16(x),
//     lo = fp16(x - hi): fp32-accurate products), optionally RMS-normalised; then for each fill consumer c takes tiles
//     c and c + 8: ds_read of the 1 KiB tile (the same 16 B per lane a global load would bring), 0x6400 magic
//     dequantisation, v_mfma_f32_16x16x32_f16 with hi in MFMA rows 0-7 and lo in rows 8-15, the group scale applied to
//     an fp32 group accumulator; partial sums per (stripe, consumer) in LDS, summed in a fixed order, fused epilogue
//     (residual add, SiLU / GELU * up);
//   * hand-offs between ops (MI355X_MICROARCH.md "Hand-offs measured with sc1 loads", granule form R2; Guideline 16):
//     each result element is published as ONE 8-byte {fp32 value, tag} granule by an agent-scope relaxed 64-bit store
//     (write-through sc1), tag = launch generation * 256 + op index + 1; a consumer reads the whole input vector with
//     sc1 buffer loads and re-reads every granule whose tag is not yet the expected one -- the data is the flag, no
//     fence, no counter.  The generation is the launch's index on its chain, taken by every workgroup at its start
//     as a ticket of a monotonic arrival counter (ticket / grid), so stale granules of the previous run never match
//     (graph replay safe, nothing to reset per call, nothing to publish at the end);
//   * every spin is bounded (~1 s); a give-up records a code in ctl[1] and the launch still terminates;
//   * one launch may hold two weight formats (the op body is a generic lambda over (bits, groups per tile)): Mistral's
//     int2 policy keeps wv / w2 at int4 (llama_utils.cpp:269-287);
// Arithmetic per op is the same for every position of the op in a launch: a one-op launch of it gives bit-identical
// outputs (tests/test_chain_gpu.py).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "woq_chain.h"
#include "woq_device.h"
#include "woq_kernels.h"

namespace nad {
namespace eng {

// Development instrumentation (make chaintrace): per-(op, workgroup) wall-clock stamps of the engine's phases.
#ifdef NAD_CHAIN_TRACE
constexpr int kTrOps = 160, kTrWg = 256, kTrSlots = 22;
__device__ unsigned long long nad_chain_trace[kTrSlots][kTrOps][kTrWg];
#define ETRACE(slot, opi, val)                                                                     \
  do {                                                                                             \
    if (lane == 0 && (opi) < kTrOps && blockIdx.x < kTrWg) nad_chain_trace[slot][opi][blockIdx.x] = (val); \
  } while (0)
#else
#define ETRACE(slot, opi, val) \
  do {                         \
  } while (0)
#endif

constexpr int NC = kEngConsumers;
constexpr int FT = kEngFillTiles;
constexpr int TPC = FT / NC;  // tiles per consumer per fill
static_assert(FT % NC == 0, "every consumer takes the same number of tiles of a fill");
constexpr int PJ = 8;                       // granule pairs per consumer lane per gather pass (12 = one pass for K = 11008 measured 1-3 % slower: 168 VGPRs)
constexpr int kOOB = 0x7FFF0000;            // buffer offset past every resource: no memory access, returns 0
constexpr int kSC1 = 16;                    // buffer-load aux: sc1 (bypass this CU's L1)
constexpr int kNT = 2;                      // buffer-load aux: non-temporal (weights, read once per token)
constexpr unsigned kSpinMax = 1u << 24;     // ~1 s of s_sleep(1) polls
// LDS control words (u32 index): FULL[16], FREE[16], consumer barrier, RMS partial sums[2][8], gather phase,
// consumers that issued the launch's first gather (start sync)
constexpr int kFull = 0, kFree = 16, kBar = 32, kNsum = 36, kGen = 60, kCtlBytes = 256;
constexpr int kPartBytes = kEngMaxStripes * NC * 16 * 4;

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return uint32_t(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p));
}
// LDS words shared between the loader and the consumers, in inline asm: hipcc puts vmcnt(0) in front of every LDS
// access it can see while an LDS-DMA is in flight, which would drain the loader's pipeline at every poll
__device__ __forceinline__ unsigned lds_ld(uint32_t a) {
  unsigned r;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
  return __builtin_amdgcn_readfirstlane(r);
}
__device__ __forceinline__ void lds_st(uint32_t a, unsigned v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_add(uint32_t a, unsigned v) {
  asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void give_up(unsigned* ctl, unsigned code) {
  __hip_atomic_store(ctl + 1, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// per-lane selection among an op's (at most 3) weights from uniform (scalar) loads of all of them -- indexing o.w[]
// with a lane-varying index would turn every field access into a vector load with full memory latency
template <class T>
__device__ __forceinline__ T sel3(int w, T x0, T x1, T x2) {
  return w == 0 ? x0 : (w == 1 ? x1 : x2);
}

// The op fields a role reads, loaded as scalars once at the op's start: the inline-asm "memory" clobbers of the LDS
// protocol would otherwise make hipcc re-load a field from the op table (a dependent scalar-cache round trip) at every
// use -- the consumer's per-op code held ~30 such load -> wait pairs.
struct OpGeom {
  int nt, ng, tpg_shift, scale_t, u_q, u_r, dual, sb1, sb2;
};
__device__ __forceinline__ OpGeom op_geom(const EngOp& o) {
  return OpGeom{o.nt, o.ng, o.tpg_shift, o.scale_t, o.u_q, o.u_r, o.dual, o.stripe_base[1], o.stripe_base[2]};
}

// virtual stripe -> (weight, stripe within it)
__device__ __forceinline__ void vstripe(const OpGeom& o, int v, int& w, int& s) {
  if (o.dual) {
    w = v & 1;
    s = v >> 1;
  } else {
    w = (v >= o.sb1 ? 1 : 0) + (v >= o.sb2 ? 1 : 0);
    s = v - (w == 0 ? 0 : (w == 1 ? o.sb1 : o.sb2));
  }
}
__device__ __forceinline__ void unit_range(const OpGeom& o, int bid, int& v0, int& nv) {
  const int u0 = bid * o.u_q + min(bid, o.u_r);
  const int nu = o.u_q + (bid < o.u_r ? 1 : 0);
  const int vpu = o.dual ? 2 : 1;
  v0 = u0 * vpu;
  nv = nu * vpu;
}
// groups of one fill (chunk c of a stripe): first group and count
template <int GPT>
__device__ __forceinline__ void fill_groups(const OpGeom& o, int t0, int& g0, int& ngc) {
  const int t1 = min(t0 + FT, o.nt);
  if constexpr (GPT == 1) {
    g0 = t0 >> o.tpg_shift;
    ngc = ((t1 - 1) >> o.tpg_shift) - g0 + 1;
  } else {
    g0 = t0 * GPT;
    ngc = (t1 - t0) * GPT;
  }
}

__device__ __forceinline__ void fill_groups_rt(const OpGeom& o, int gpt, int t0, int& g0, int& ngc) {
  const int t1 = min(t0 + FT, o.nt);
  if (gpt == 1) {
    g0 = t0 >> o.tpg_shift;
    ngc = ((t1 - 1) >> o.tpg_shift) - g0 + 1;
  } else {
    g0 = t0 * gpt;
    ngc = (t1 - t0) * gpt;
  }
}

// ------------------------------------------------------------------------------------------------ loaders
// NL loader waves share the launch's fill sequence: loader lw issues the fills f = lw, lw + NL, ... (every loader walks
// the whole sequence, skipping the others' fills), keeps D of its own in flight (counted vmcnt) and publishes them in
// its order.  One wave cannot keep more than ~2 fills usefully in flight (tools/dma_probe.hip on MI355X: 1 wave x 2-3
// fills 19-20 GB/s per CU, 2 waves x 2 fills 27 GB/s = 6.9 TB/s chip-wide, 3 waves x 1 fill 26.6).  Slot of fill f:
// f mod S; it is re-filled only when all consumers released fill f - S (FREE counter >= NC * (f / S)), so fills into one
// slot stay ordered whichever loader issues them.
template <bool ASYM, int SD, int D>
__device__ void loader(const EngOp* ops, int n_ops, char* ring, int S, int slot_bytes, uint32_t ctl_a, unsigned* ctl,
                       int lane, int lw, int NL) {
  constexpr int IPF = FT + SD + (ASYM ? 1 : 0);  // DMA instructions per fill: constant, so vmcnt counts are exact
  static_assert(D * IPF <= 63, "in-flight DMAs beyond what vmcnt counts");
  const uint32_t full_a = ctl_a + kFull * 4, free_a = ctl_a + kFree * 4;
  int slot = 0, rr = 0;   // slot of fill f, f mod NL
  unsigned round = 0;     // f / S
  int mine = 0, mpub = 0;         // own fills issued / published
  int pub_f = lw, pub_slot = lw;  // the next own fill to publish and its slot
  while (pub_slot >= S) pub_slot -= S;
  bool failed = false;
  auto publish_one = [&]() {
    lds_st(full_a + pub_slot * 4, unsigned(pub_f + 1));
    mpub++;
    pub_f += NL;
    pub_slot += NL;
    while (pub_slot >= S) pub_slot -= S;
  };
  for (int op = 0; op < n_ops; op++) {
    const EngOp& od = ops[op];
    const OpGeom o = op_geom(od);
    const void *tl0 = od.w[0].tiles, *tl1 = od.w[1].tiles, *tl2 = od.w[2].tiles;
    const void *sc0 = od.w[0].scales, *sc1 = od.w[1].scales, *sc2 = od.w[2].scales;
    const void *zp0 = od.w[0].zps, *zp1 = od.w[1].zps, *zp2 = od.w[2].zps;
    const int ns0 = od.w[0].ns, ns1 = od.w[1].ns, ns2 = od.w[2].ns;
    const int nt = o.nt, ng = o.ng, nch = (nt + FT - 1) / FT;
    const int ssz = o.scale_t == kScaleF32 ? 4 : 2;
    int v0, nv;
    unit_range(o, blockIdx.x, v0, nv);
#ifdef NAD_CHAIN_TRACE
    unsigned long long tr_wait = 0;
    bool tr_first = true;
#endif
    for (int jl = 0; jl < nv; jl++) {
      int wsel, s;
      vstripe(o, v0 + jl, wsel, s);
      const unsigned wns = unsigned(sel3(wsel, ns0, ns1, ns2));
      const auto rt = rsrc(sel3(wsel, tl0, tl1, tl2), wns * nt * 1024u);
      const auto rs = rsrc(sel3(wsel, sc0, sc1, sc2), wns * ng * 16u * ssz);
      const auto rz = rsrc(ASYM ? sel3(wsel, zp0, zp1, zp2) : sel3(wsel, tl0, tl1, tl2), ASYM ? wns * ng * 16u : 0u);
      const int tbase = s * nt * 1024 + lane * 16;
      for (int c = 0; c < nch; c++) {
        if (rr == lw) {
          if (mine - mpub == D) {  // keep at most D own fills in flight: the oldest has landed -> publish it
            wait_vm<(D - 1) * IPF>();
            publish_one();
          }
          if (round > 0) {  // this slot's previous fill must have been released by every consumer
            const unsigned need = NC * round;
            if (lds_ld(free_a + slot * 4) < need) {
#ifdef NAD_CHAIN_TRACE
              const unsigned long long tw0 = wall_clock64();
#endif
              wait_vm<0>();  // about to wait anyway: publish everything in flight first
              while (mpub < mine) publish_one();
              unsigned spins = 0;
              while (!failed && lds_ld(free_a + slot * 4) < need) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > kSpinMax) {
                  give_up(ctl, 2);
                  failed = true;
                }
              }
#ifdef NAD_CHAIN_TRACE
              tr_wait += wall_clock64() - tw0;
#endif
            }
          }
#ifdef NAD_CHAIN_TRACE
          if (tr_first && lw == 0) ETRACE(6, op, wall_clock64());
          tr_first = false;
#endif
          char* sb = ring + slot * slot_bytes;
          const int t0 = c * FT;
#pragma unroll
          for (int i = 0; i < FT; i++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (lds_void_t*)(sb + i * 1024), 16,
                                                     t0 + i < nt ? tbase + (t0 + i) * 1024 : kOOB, 0, 0, kNT);
          int g0, ngc;
          fill_groups_rt(o, od.gpt, t0, g0, ngc);
          const int sbytes = ngc * 16 * ssz, soff = (s * ng + g0) * 16 * ssz;
#pragma unroll
          for (int j = 0; j < SD; j++) {
            const int b = j * 1024 + lane * 16;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(sb + FT * 1024 + j * 1024), 16,
                                                     b < sbytes ? soff + b : kOOB, 0, 0, 0);
          }
          if constexpr (ASYM) {
            const int b = lane * 16;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rz, (lds_void_t*)(sb + FT * 1024 + SD * 1024), 16,
                                                     b < ngc * 16 ? (s * ng + g0) * 16 + b : kOOB, 0, 0, 0);
          }
          mine++;
        }
        if (++rr == NL) rr = 0;
        if (++slot == S) {
          slot = 0;
          round++;
        }
      }
    }
    if (lw == 0) ETRACE(7, op, wall_clock64());
#ifdef NAD_CHAIN_TRACE
    if (lw == 0) ETRACE(8, op, tr_wait);
#endif
  }
  wait_vm<0>();
  while (mpub < mine) publish_one();
}

// ------------------------------------------------------------------------------------------------ consumers
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
// int4: 0x6400 | nibble = 1024 + q and 0x6400 | nibble << 4 = 1024 + 16 q (exact fp16): one shift per dword
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
__device__ __forceinline__ float lds_scale(const char* p, int st) {
  if (st == kScaleF32) return *reinterpret_cast<const float*>(p);
  const uint16_t h = *reinterpret_cast<const uint16_t*>(p);
  return st == kScaleBF16 ? bf16_bits_to_f32(h) : f16_bits_to_f32(h);
}

// consumer-only barrier: an LDS arrival counter (the loader never joins)
__device__ __forceinline__ void cbar(uint32_t a, unsigned& epoch, unsigned* ctl, int lane, bool& failed) {
  epoch += NC;
  if (lane == 0) lds_add(a, 1u);
  unsigned spins = 0;
  while (!failed && lds_ld(a) < epoch) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > kSpinMax) {
      if (lane == 0) give_up(ctl, 5);
      failed = true;
    }
  }
}

template <int V>
using IC = std::integral_constant<int, V>;

// One launch holds ops of at most two weight formats (B0, G0) and (B1, G1) (bits, groups per tile; EngOp::fmt picks
// one), e.g. Mistral's int2 g64 projections beside its int4 g64 wv / w2 (llama_utils.cpp:269-287)
template <int B0, int G0, int B1, int G1, bool ASYM, int SD>
__global__ __launch_bounds__(kEngMaxThreads, 1) void woq_engine_kernel(const EngOp* __restrict__ ops, int n_ops,
                                                                       unsigned* ctl, int S, int slot_bytes, int Kp,
                                                                       int bump, int nl) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool MIXED = B0 != B1 || G0 != G1;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const uint32_t ctl_a = lds_addr(smem);
  float* part = reinterpret_cast<float*>(smem + kCtlBytes);          // [stripe][consumer][16]
  char* act = smem + kCtlBytes + kPartBytes;             // [Kp / 8] units of {hi[8], lo[8]}
  char* zrows = act + size_t(Kp) * 4;                   // kEngZeroBytes of zeros (never written)
  char* ring = zrows + kEngZeroBytes;
  if (threadIdx.x < kCtlBytes / 4) reinterpret_cast<unsigned*>(smem)[threadIdx.x] = 0u;
  if (threadIdx.x < kEngZeroBytes / 4) reinterpret_cast<unsigned*>(zrows)[threadIdx.x] = 0u;
  __syncthreads();
  if (wave >= NC) {
    const int lw = wave - NC;
    loader<ASYM, SD, 1>(ops, n_ops, ring, S, slot_bytes, ctl_a, ctl, lane, lw, nl);
    return;
  }

  const int cw = wave, cl = wave * 64 + lane;  // consumer wave, consumer lane
  const uint32_t full_a = ctl_a + kFull * 4, free_a = ctl_a + kFree * 4, bar_a = ctl_a + kBar * 4;
  float* nsum = reinterpret_cast<float*>(smem) + kNsum;
  // The launch generation (granule tags): every workgroup takes a ticket from a monotonic arrival counter at its start;
  // launches of one chain are stream-ordered, so tickets of launch L are L * grid ... L * grid + grid - 1 and
  // gen = ticket / grid.  Nothing is bumped at the end (a workgroup that starts late, or owns no stripes, still reads
  // its own launch's generation); the ticket's round trip overlaps the first op's gather and is read after its barrier.
  unsigned gticket = 0;
  if (cw == 0 && lane == 0)
    gticket = __hip_atomic_fetch_add(ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned gen = 0;  // defined after the first op's staging barrier (no op of a launch reads a granule before that)
  unsigned bar_epoch = 0;
  bool failed = false;
  const int m = lane & 15, kq = lane >> 4;
  const uint32_t mk0 = 0x000F000Fu, mk1 = 0x00F000F0u, mag = 0x64006400u;
  const h2_t s16 = splat(1.f / 16.f);
  // this lane's A operand: MFMA rows 0-7 read hi, rows 8-15 lo (rows 0 and 8 are the result); k unit u = k / 8 at byte
  // 32 u (+16: lo), so step d of tile t starts at byte t * KT * 4 + d * 128 + kq * 32
  const uint32_t a_lane = lds_addr(act) + (m >= 8 ? 16 : 0) + kq * 32;
  const uint32_t zrow_lane = lds_addr(zrows) + (m >= 8 ? 16 : 0) + kq * 32;
  const uint32_t ring_a = lds_addr(ring);
  int f = 0, slot = 0;

  // one op, for the op's weight format (a generic lambda: the format is a compile-time constant inside)
  auto op_body = [&](auto bits_c, auto gpt_c, int op) {
    constexpr int BITS = decltype(bits_c)::value, GPT = decltype(gpt_c)::value;
    constexpr int KT = BITS == 4 ? 128 : 256, SPT = KT / 32, SPG = SPT / GPT, BIAS = BITS == 4 ? 8 : 2;
    const h2_t zc0 = splat(-(1024.f + BIAS)), zc1 = splat(-(64.f + BIAS));
    const EngOp& od = ops[op];
    const OpGeom o = op_geom(od);
    const int K = od.K;
    const float* const o_act = od.act;
    const unsigned long long* const o_act_gran = od.act_gran;
    const unsigned o_act_tag = od.act_tag, o_res_tag = od.res_tag, o_tag = od.tag;
    const int o_norm = od.norm, o_epi = od.epi;
    const float o_norm_eps = od.norm_eps;
    const float* const o_norm_w = od.norm_w;
    const float* const o_res = od.res;
    const unsigned long long* const o_res_gran = od.res_gran;
    float* const o_aux = od.aux;
    const int wn0 = od.w[0].n, wn1 = od.w[1].n, wn2 = od.w[2].n;
    float *const wo0 = od.w[0].out, *const wo1 = od.w[1].out, *const wo2 = od.w[2].out;
    unsigned long long *const wg0 = od.w[0].gran, *const wg1 = od.w[1].gran, *const wg2 = od.w[2].gran;
    const int nt = o.nt, Kpo = nt * KT, nch = (nt + FT - 1) / FT;
    if (cw == 0) ETRACE(0, op, wall_clock64());
    const int st = o.scale_t, ssz = st == kScaleF32 ? 4 : 2;
    int v0, nv;
    unit_range(o, blockIdx.x, v0, nv);
    const int vpu = o.dual ? 2 : 1;
    const int nout = nv / vpu * 16;

    // 0) this lane's residual (one output per lane at most: nout <= 256), issued now, used in the epilogue
    float res_v = 0.f;
    unsigned long long res_g = 0;
    int my_n = -1;
    {
      const int oi = cl;
      if (oi < nout && o_epi == kEpiResAdd) {
        int wsel, sx;
        vstripe(o, v0 + (oi >> 4) * vpu, wsel, sx);
        const int n = sx * 16 + (oi & 15);
        if (n < sel3(wsel, wn0, wn1, wn2)) {
          my_n = n;
          if (o_res_gran)
            res_g = __hip_atomic_load(o_res_gran + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else
            res_v = o_res[n];
        }
      }
    }

    // 1) the input vector straight into the MFMA-ready fp16 rows: element pair (2q, 2q + 1) of 8-element unit
    //    u = q / 4 -> hi at byte 32 u + 4 (q & 3), lo 16 bytes further.  An RMSNorm of the input is applied as
    //    x * g here and the scalar 1 / rms(x) on the results (y = W (x * g) / rms: the same products, no second pass)
    float s2 = 0.f;
    {
      const int npair = (K + 1) / 2;  // granule / element pairs: one 16-B (8-B external) load per pair
      const bool gw = o_norm && o_norm_w;
      float sq[PJ];  // per-slot squares, summed in slot order once the pass is complete (arrival order varies)
      auto put = [&](int j, int q, float x0, float x1) {
        // explicit fma: put() is inlined at two call sites, and hipcc's fp contraction may differ between them
        sq[j] = __builtin_fmaf(x1, x1, x0 * x0);
        if (gw) {
          x0 *= o_norm_w[2 * q];
          x1 *= 2 * q + 1 < K ? o_norm_w[2 * q + 1] : 0.f;
        }
        h2_t hi, lo;
        hi[0] = _Float16(x0);
        hi[1] = _Float16(x1);
        lo[0] = _Float16(x0 - float(hi[0]));
        lo[1] = _Float16(x1 - float(hi[1]));
        char* pu = act + (q >> 2) * 32 + (q & 3) * 4;
        *reinterpret_cast<h2_t*>(pu) = hi;
        *reinterpret_cast<h2_t*>(pu + 16) = lo;
      };
      if (o_act_gran) {
        const unsigned want = gen * 256u + o_act_tag;
        const auto rg = rsrc(o_act_gran, unsigned(K) * 8u);
        for (int q0 = 0; q0 < npair; q0 += NC * 64 * PJ) {
          uint32_t pend = 0;
#pragma unroll
          for (int j = 0; j < PJ; j++) {
            sq[j] = 0.f;
            if (q0 + cl + NC * 64 * j < npair) pend |= 1u << j;
          }
          unsigned spins = 0;
          while (true) {
            uint4 g[PJ];
#pragma unroll
            for (int j = 0; j < PJ; j++)
              g[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rg, (pend >> j) & 1u ? (q0 + cl + NC * 64 * j) * 16 : kOOB, 0, kSC1));
            __builtin_amdgcn_sched_barrier(0);  // every load of the pass in flight before the first tag check
#pragma unroll
            for (int j = 0; j < PJ; j++) {
              const int q = q0 + cl + NC * 64 * j;
              // the pair's second granule is past K for odd K: its tag is never written, value 0
              const bool ok1 = 2 * q + 1 >= K || g[j].w == want;
              if (((pend >> j) & 1u) && g[j].y == want && ok1) {
                put(j, q, __uint_as_float(g[j].x), 2 * q + 1 < K ? __uint_as_float(g[j].z) : 0.f);
                pend &= ~(1u << j);
              }
            }
            if (cw == 0 && spins == 0 && q0 == 0) ETRACE(11, op, wall_clock64());  // first pass returned
            if (__all(pend == 0u) || failed) break;
            __builtin_amdgcn_s_sleep(1);
            if (++spins > kSpinMax) {
              if (lane == 0) give_up(ctl, 3);
              failed = true;
            }
          }
#pragma unroll
          for (int j = 0; j < PJ; j++) s2 += sq[j];
        }
      } else {  // an external vector (written before this launch): plain loads, all of a pass in flight at once
        const auto ra = rsrc(o_act, unsigned(K) * 4u);
        for (int q0 = 0; q0 < npair; q0 += NC * 64 * PJ) {
          uint2 g[PJ];
#pragma unroll
          for (int j = 0; j < PJ; j++) {
            const int q = q0 + cl + NC * 64 * j;
            g[j] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(ra, q < npair ? q * 8 : kOOB, 0, 0));
          }
          __builtin_amdgcn_sched_barrier(0);
          if (cw == 0 && q0 == 0) ETRACE(11, op, wall_clock64());
#pragma unroll
          for (int j = 0; j < PJ; j++) {
            const int q = q0 + cl + NC * 64 * j;
            sq[j] = 0.f;
            // odd K: the last pair's second element lies past the vector (its bytes are out of range: 0)
            if (q < npair) put(j, q, __uint_as_float(g[j].x), 2 * q + 1 < K ? __uint_as_float(g[j].y) : 0.f);
          }
#pragma unroll
          for (int j = 0; j < PJ; j++) s2 += sq[j];
        }
      }
      for (int q = npair + cl; q < Kpo / 2; q += NC * 64) {  // K tail of the last tile: zero rows
        char* pu = act + (q >> 2) * 32 + (q & 3) * 4;
        *reinterpret_cast<uint32_t*>(pu) = 0u;
        *reinterpret_cast<uint32_t*>(pu + 16) = 0u;
      }
    }
    if (cw == 0) ETRACE(1, op, wall_clock64());
    // per-consumer sums of squares, double-buffered by op parity: they are read after this op's post-stream barrier,
    // and no consumer can write this parity again before every consumer has passed the next op's one
    float* const nsum_op = nsum + (op & 1) * NC;
    if (o_norm) {
#pragma unroll
      for (int sh = 32; sh > 0; sh >>= 1) s2 += __shfl_xor(s2, sh, 64);
      if (lane == 0) nsum_op[cw] = s2;
    }
    // every consumer staged a share of the whole vector, so all meet before the stream.  (Staging only the consumer's
    // own tiles with no barrier measured 2-3 % slower per whole-token launch.)
    if (op == 0 && cw == 0 && lane == 0) lds_st(ctl_a + kGen * 4, gticket / gridDim.x);
    cbar(bar_a, bar_epoch, ctl, lane, failed);
    if (op == 0) gen = lds_ld(ctl_a + kGen * 4);
    if (cw == 0) ETRACE(2, op, wall_clock64());

    // 2) the weight stream: consumer cw takes tiles cw and cw + 8 of every fill.  One LDS round trip per fill: the FULL
    //    word and every operand of both tiles are read together (a wave's LDS reads complete in order, and the loader
    //    publishes FULL only after the fill landed, so operands read behind a FULL that says "landed" are that fill's);
    //    the slot is released as soon as they are in registers, then two interleaved MFMA chains run.
#ifdef NAD_CHAIN_TRACE
    unsigned long long tr_fw = 0;
#endif
    const int gsh = st == kScaleF32 ? 0 : (m & 1) * 16;  // this lane's scale bits within the dword read
    for (int jl = 0; jl < nv; jl++) {
      f4_t acc = {0.f, 0.f, 0.f, 0.f};
      for (int c = 0; c < nch; c++) {
        const int t0 = c * FT;
        int g0, ngc;
        fill_groups<GPT>(o, t0, g0, ngc);
        const uint32_t sb = ring_a + slot * slot_bytes;
        int tt[TPC];
        uint32_t ab[TPC], sca[TPC][GPT], zpa[TPC][GPT];
        bool valid[TPC];
#pragma unroll
        for (int h = 0; h < TPC; h++) {
          const int p = cw + h * NC, t = t0 + p;
          valid[h] = t < nt;
          tt[h] = min(t, nt - 1);
          // a ragged last fill's missing tile reads the zero rows (tile nt - 1's rows belong to another consumer, staged
          // with no barrier in between: stale bits there could be a NaN, which a zero scale does not cancel)
          ab[h] = (valid[h] ? a_lane + uint32_t(tt[h]) * KT * 4 : zrow_lane);
#pragma unroll
          for (int g = 0; g < GPT; g++) {
            const int gi = GPT == 1 ? (tt[h] >> o.tpg_shift) - g0 : p * GPT + g;
            sca[h][g] = sb + FT * 1024 + ((gi * 16 + m) * ssz & ~3);
            zpa[h][g] = sb + FT * 1024 + SD * 1024 + ((gi * 16 + m) & ~3);
          }
        }
        u4_t bq[TPC];
        h8_t af[TPC][SPT];
        uint32_t scw[TPC][GPT], zpw[TPC][GPT];
        unsigned full;
#ifdef NAD_CHAIN_TRACE
        const unsigned long long tf0 = wall_clock64();
#endif
        // every operand of both tiles in one round trip with the FULL word: one LDS round trip per fill when it has
        // landed.  If it has not, poll the FULL word alone (an operand re-read per poll by 8 waves saturates the LDS
        // and starves the loader's DMA writes), then read the operands once more.
        auto rd_ops = [&]() {
#pragma unroll
          for (int h = 0; h < TPC; h++) {
            const uint32_t tb = sb + (cw + h * NC) * 1024 + lane * 16;
            asm volatile("ds_read_b128 %0, %1" : "=v"(bq[h]) : "v"(tb) : "memory");
#pragma unroll
            for (int d = 0; d < SPT; d++) asm volatile("ds_read_b128 %0, %1" : "=v"(af[h][d]) : "v"(ab[h] + d * 128) : "memory");
#pragma unroll
            for (int g = 0; g < GPT; g++) {
              asm volatile("ds_read_b32 %0, %1" : "=v"(scw[h][g]) : "v"(sca[h][g]) : "memory");
              if constexpr (ASYM) asm volatile("ds_read_b32 %0, %1" : "=v"(zpw[h][g]) : "v"(zpa[h][g]) : "memory");
            }
          }
        };
        asm volatile("ds_read_b32 %0, %1" : "=v"(full) : "v"(full_a + slot * 4) : "memory");
        rd_ops();
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(full) : : "memory");  // full is defined here, not at its load
        if (__builtin_amdgcn_readfirstlane(full) < unsigned(f + 1) && !failed) {
          for (unsigned spins = 0;; spins++) {
            __builtin_amdgcn_s_sleep(1);
            if (lds_ld(full_a + slot * 4) >= unsigned(f + 1) || failed) break;
            if (spins > kSpinMax) {
              if (lane == 0) give_up(ctl, 1);
              failed = true;
            }
          }
          rd_ops();
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (int h = 0; h < TPC; h++) {  // registers are defined by the wait above: pin every use below it
          asm volatile("" : "+v"(bq[h]));
#pragma unroll
          for (int d = 0; d < SPT; d++) {
            asm volatile("" : "+v"(af[h][d]));
          }
#pragma unroll
          for (int g = 0; g < GPT; g++) {
            asm volatile("" : "+v"(scw[h][g]));
            if constexpr (ASYM) asm volatile("" : "+v"(zpw[h][g]));
          }
        }
        if (lane == 0) lds_add(free_a + slot * 4, 1u);  // operands in registers: the slot may be refilled
#ifdef NAD_CHAIN_TRACE
        tr_fw += wall_clock64() - tf0;
        if (cw == 0 && jl == 0 && c == 0) ETRACE(3, op, wall_clock64());
#endif
        float scf[TPC][GPT];
        int zpv[TPC][GPT];
#pragma unroll
        for (int h = 0; h < TPC; h++)
#pragma unroll
          for (int g = 0; g < GPT; g++) {
            const uint32_t x = scw[h][g];
            const uint32_t hb = (x >> gsh) & 0xFFFFu;
            const float fb = __uint_as_float(hb << 16), fh = f16_bits_to_f32(uint16_t(hb));
            const float sv = st == kScaleF32 ? __uint_as_float(x) : (st == kScaleBF16 ? fb : fh);
            scf[h][g] = valid[h] ? sv : 0.f;  // a ragged last fill: the missing tile contributes nothing
            zpv[h][g] = ASYM ? int(int8_t((zpw[h][g] >> ((m & 3) * 8)) & 0xFFu)) : 0;
          }
        f4_t accg[TPC];
#pragma unroll
        for (int d = 0; d < SPT; d++) {
          const int g = GPT == 1 ? 0 : d / SPG;
#pragma unroll
          for (int h = 0; h < TPC; h++) {
            h8_t bf;
            if constexpr (BITS == 4) {
              if constexpr (ASYM) {
                const float z = float(zpv[h][g]);
                bf = dequant4(bq[h][d], mk0, mk1, mag, s16, zc0 - splat(z), zc1 - splat(z));
              } else {
                bf = dequant4(bq[h][d], mk0, mk1, mag, s16, zc0, zc1);
              }
            } else {
              bf = dequant2_step(bq[h], d, BIAS + zpv[h][g]);
            }
            accg[h] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[h][d], bf, d % SPG == 0 ? f4_t{0.f, 0.f, 0.f, 0.f}
                                                                                       : accg[h], 0, 0, 0);
          }
          if ((d + 1) % SPG == 0) {
#pragma unroll
            for (int h = 0; h < TPC; h++) acc += accg[h] * scf[h][g];
          }
        }
        f++;
        slot = slot + 1 == S ? 0 : slot + 1;
      }
      const float r = acc[0] + __shfl_down(acc[0], 32, 64);  // row 0 (hi) + row 8 (lo)
      if (lane < 16) part[(jl * NC + cw) * 16 + lane] = r;
    }
    if (cw == 0) ETRACE(4, op, wall_clock64());
    ETRACE(12 + cw, op, wall_clock64());  // every consumer's loop end (slots 12..19)
#ifdef NAD_CHAIN_TRACE
    if (cw == 0) ETRACE(9, op, tr_fw);
#endif
    cbar(bar_a, bar_epoch, ctl, lane, failed);
    if (cw == 0) ETRACE(10, op, wall_clock64());
    float inv = 1.f;  // 1 / rms of the input
    if (o_norm) {
      float tot = 0.f;
#pragma unroll
      for (int w = 0; w < NC; w++) tot += nsum_op[w];
      inv = 1.f / sqrtf(tot / float(K) + o_norm_eps);
    }

    // 3) sum the consumers' partials in a fixed order, RMS scale, epilogue, results + granules
    const unsigned tag = gen * 256u + o_tag;
    for (int oi = cl; oi < nout; oi += NC * 64) {
      const int p = oi >> 4, nn = oi & 15;
      float y[2] = {0.f, 0.f};
#pragma unroll
      for (int h = 0; h < 2; h++) {
        if (h < vpu) {
          const float* ps = part + (p * vpu + h) * NC * 16 + nn;
          y[h] = (((ps[0] + ps[16]) + (ps[32] + ps[48])) + ((ps[64] + ps[80]) + (ps[96] + ps[112]))) * inv;
        }
      }
      int wsel, sx;
      vstripe(o, v0 + p * vpu, wsel, sx);
      const int n = sx * 16 + nn;
      if (n >= sel3(wsel, wn0, wn1, wn2)) continue;
      float* const w_out = sel3(wsel, wo0, wo1, wo2);
      unsigned long long* const w_gran = sel3(wsel, wg0, wg1, wg2);
      float val = y[0];
      if (o_epi == kEpiResAdd) {
        if (o_res_gran) {
          const unsigned want = gen * 256u + o_res_tag;
          unsigned spins = 0;
          unsigned long long x = res_g;
          while (unsigned(x >> 32) != want && !failed) {  // the early load normally already holds it
            __builtin_amdgcn_s_sleep(1);
            x = __hip_atomic_load(o_res_gran + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (++spins > kSpinMax) {
              give_up(ctl, 4);
              failed = true;
            }
          }
          res_v = __uint_as_float(unsigned(x));
        }
        val += res_v;
      } else if (o_epi == kEpiSiluMul || o_epi == kEpiGeluMul) {
        const float t1 = o_epi == kEpiSiluMul ? silu_f(y[0]) : gelu_f(y[0]);
        if (o_aux) o_aux[n] = t1;
        val = t1 * y[1];
      }
      if (w_out) w_out[n] = val;
      if (w_gran)
        __hip_atomic_store(w_gran + n, (static_cast<unsigned long long>(tag) << 32) | __float_as_uint(val),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    (void)my_n;
    if (cw == 0) ETRACE(5, op, wall_clock64());
#ifdef NAD_CHAIN_TRACE
    if (cw == 0) {  // development: how long the published stores take to complete (delays wave 0 only)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ETRACE(20, op, wall_clock64());
    }
#endif
  };
  for (int op = 0; op < n_ops; op++) {
    if (MIXED && ops[op].fmt)
      op_body(IC<B1>(), IC<G1>(), op);
    else
      op_body(IC<B0>(), IC<G0>(), op);
  }
  (void)bump;
}

}  // namespace eng

// ------------------------------------------------------------------------------------------------ host side
bool engine_geometry(EngGeometry& g, int kp) {
  g.kp = (kp + 15) / 16 * 16;
  g.slot_bytes = size_t(kEngFillTiles) * 1024 + size_t(g.sd) * 1024 + (g.asym ? 1024 : 0);
  const size_t act = size_t(g.kp) * 4;
  const size_t fixed = size_t(eng::kCtlBytes) + eng::kPartBytes + act + kEngZeroBytes;
  const size_t budget = 160 * 1024;
  if (fixed >= budget) return false;
  int s = int((budget - fixed) / g.slot_bytes);
  if (s > 16) s = 16;
  if (g.max_slots > 0 && s > g.max_slots) s = g.max_slots;
  if (g.loaders < 1 || g.loaders > kEngMaxLoaders) return false;
  if (s < g.loaders + 2) return false;  // fills in flight + at least two published ones for the consumers
  g.slots = s;
  g.lds = fixed + size_t(s) * g.slot_bytes;
  return true;
}

template <int B0, int G0, int B1, int G1, bool ASYM, int SD>
static hipError_t engine_launch5(const EngOp* ops, int n_ops, const EngGeometry& g, unsigned* ctl, int grid, int bump,
                                 hipStream_t st) {
  auto k = eng::woq_engine_kernel<B0, G0, B1, G1, ASYM, SD>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3((kEngConsumers + g.loaders) * 64), g.lds, st, ops, n_ops, ctl, g.slots,
                     int(g.slot_bytes), g.kp, bump, g.loaders);
  return hipGetLastError();
}

template <int B0, int G0, int B1, int G1>
static hipError_t engine_launch4(const EngOp* ops, int n_ops, const EngGeometry& g, unsigned* ctl, int grid, int bump,
                                 hipStream_t st) {
  if (g.sd != 1 && g.sd != 2) return hipErrorInvalidValue;
#define NAD_ENG_L(A, D) \
  if (g.asym == A && g.sd == D) return engine_launch5<B0, G0, B1, G1, A, D>(ops, n_ops, g, ctl, grid, bump, st);
  NAD_ENG_L(false, 1)
  NAD_ENG_L(false, 2)
  NAD_ENG_L(true, 1)
  NAD_ENG_L(true, 2)
#undef NAD_ENG_L
  return hipErrorInvalidValue;
}

hipError_t launch_engine(const EngOp* ops, int n_ops, const EngGeometry& g, unsigned* ctl, int grid, int bump,
                         hipStream_t st) {
  static_assert(kEngConsumers == 8, "the partial-sum order below is written for 8 consumers");
  const int f0 = g.bits * 16 + g.gpt, f1 = g.bits1 * 16 + g.gpt1;
  if (f0 == f1) {
    switch (f0) {
      case 4 * 16 + 1: return engine_launch4<4, 1, 4, 1>(ops, n_ops, g, ctl, grid, bump, st);
      case 4 * 16 + 2: return engine_launch4<4, 2, 4, 2>(ops, n_ops, g, ctl, grid, bump, st);
      case 2 * 16 + 1: return engine_launch4<2, 1, 2, 1>(ops, n_ops, g, ctl, grid, bump, st);
      case 2 * 16 + 2: return engine_launch4<2, 2, 2, 2>(ops, n_ops, g, ctl, grid, bump, st);
      case 2 * 16 + 4: return engine_launch4<2, 4, 2, 4>(ops, n_ops, g, ctl, grid, bump, st);
      default: return hipErrorInvalidValue;
    }
  }
  // mixed launches: the reference's int2 policies keep some weights at int4 with the same group size
  if (f0 == 2 * 16 + 4 && f1 == 4 * 16 + 2) return engine_launch4<2, 4, 4, 2>(ops, n_ops, g, ctl, grid, bump, st);
  if (f0 == 2 * 16 + 2 && f1 == 4 * 16 + 1) return engine_launch4<2, 2, 4, 1>(ops, n_ops, g, ctl, grid, bump, st);
  return hipErrorInvalidValue;
}

bool engine_format_pair_ok(int bits0, int gpt0, int bits1, int gpt1) {
  const int f0 = bits0 * 16 + gpt0, f1 = bits1 * 16 + gpt1;
  if (f0 == f1) return f0 == 65 || f0 == 66 || f0 == 33 || f0 == 34 || f0 == 36;
  return (f0 == 36 && f1 == 66) || (f0 == 34 && f1 == 65);
}

}  // namespace nad

#ifdef NAD_CHAIN_TRACE
extern "C" int nad_chain_trace_fetch(void* host, size_t bytes) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const size_t n = sizeof(nad::eng::nad_chain_trace) < bytes ? sizeof(nad::eng::nad_chain_trace) : bytes;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(nad::eng::nad_chain_trace), n) == hipSuccess ? 0 : -1;
}
#endif
