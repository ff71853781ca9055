// woq_chain.h -- the decode weight-stream engine (woq_chain.hip): a list of M = 1 WOQ matmuls in ONE persistent
// launch, one workgroup per CU, each CU's weights streamed by one LDS-DMA loader wave into an LDS ring while eight
// consumer waves compute, hand-offs between ops as data-tagged 8-byte granules.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "woq_kernels.h"

namespace nad {

struct EngWeight {
  const void* tiles;            // stripe-major tile layout (woq_layout.h)
  const void* scales;
  const int8_t* zps;            // asym only
  int ns, n;
  float* out;                   // [n] fp32 result (plain stores; read by kernels after this launch)
  unsigned long long* gran;     // [n] {value, tag} granules for ops of this launch that read the result (or null)
};

struct EngOp {
  EngWeight w[3];
  int nw;                       // weights (QKV: 3); dual: w[0] = gate, w[1] = up
  int dual;                     // units are {w[0] stripe u, w[1] stripe u}: out = act(x.w0) * (x.w1) into w[0]
  int units, u_q, u_r;          // units (virtual stripes, or stripe pairs); per workgroup u_q, +1 for the first u_r
  int stripe_base[4];           // non-dual: first virtual stripe of each weight (unused = INT_MAX)
  int K, nt, ng, tpg_shift;     // shared geometry: K, K tiles, groups, log2(tiles per group) (31: one group)
  int scale_t;
  // input: an external fp32 vector [K] (written before this launch), or the granules of an earlier op
  const float* act;
  const unsigned long long* act_gran;
  unsigned act_tag;
  int norm;                     // RMS-normalise the input: x / sqrt(mean(x^2) + eps) * (norm_w ? norm_w : 1)
  float norm_eps;
  const float* norm_w;
  int epi;                      // kEpiNone, kEpiResAdd, dual: kEpiSiluMul / kEpiGeluMul
  const float* res;             // residual: external [n] ...
  const unsigned long long* res_gran;  // ... or an earlier op's granules
  unsigned res_tag;
  float* aux;                   // dual: act(x.w0) (optional)
  unsigned tag;                 // this op's index in the launch + 1
  int fmt;                      // weight format of the op: 0 = the launch's first (bits, gpt), 1 = its second
  int gpt;                      // groups per K tile (the loader's scale pieces per fill)
};

// Engine geometry: 8 consumer waves + `loaders` loader waves (each keeping `depth` fills in flight), fills of 16 tiles
// (two per consumer).  Measured (trace_chain.py): 8-tile fills stream SLOWER (the loader's per-fill
// LDS round trips dominate); one loader wave tops out near 20 GB/s per CU whatever its depth (tools/dma_probe.hip).
constexpr int kEngConsumers = 8;
constexpr int kEngMaxLoaders = 4;
constexpr int kEngMaxThreads = (kEngConsumers + kEngMaxLoaders) * 64;
constexpr int kEngFillTiles = 16;
constexpr int kEngMaxStripes = 16;   // virtual stripes of one op per workgroup (partial-sum slots)
constexpr int kEngMaxK = 16384;      // input length (gather registers)
constexpr int kEngZeroBytes = 1024;  // LDS zero rows for a ragged fill's missing tile (one int2 tile's fp16 hi/lo rows)

struct EngGeometry {
  int bits, gpt, asym, sd;      // kernel instantiation: bits 4 / 2, groups per tile 1 / 2 / 4, scale DMAs per fill
  int bits1, gpt1;              // the second weight format of a mixed launch (= bits, gpt when there is one)
  int slots;                    // ring slots
  int kp;                       // activation row length (max over ops of nt * KT)
  size_t lds;                   // dynamic LDS bytes
  size_t slot_bytes;
  int loaders;                  // loader waves (one fill in flight each)
  int max_slots;                // cap on the ring's slots (A/B; 16 = as many as fit)
};

// fills g.kp/slots/lds from g.bits/gpt/asym/sd and the ops' largest padded K; false if the ring does not fit
bool engine_geometry(EngGeometry& g, int kp);
// ops: device array; ctl: [1] status (0 ok, else the first give-up code), [2] workgroup arrivals (monotonic: the launch
// generation that tags granules is arrivals / grid); bump: some op reads a result of this launch
// the (bits, groups per tile) formats one launch may hold: one of int4 g >= 128 / g64, int2 g >= 256 / g128 / g64, or the
// mixed pairs (int2 g64, int4 g64) and (int2 g128, int4 g128)
bool engine_format_pair_ok(int bits0, int gpt0, int bits1, int gpt1);
hipError_t launch_engine(const EngOp* ops, int n_ops, const EngGeometry& g, unsigned* ctl, int grid, int bump,
                         hipStream_t st);

}  // namespace nad
