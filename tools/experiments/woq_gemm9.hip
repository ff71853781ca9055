// woq_gemm9.hip -- the wide-tile prefill int4 WOQ GEMM for gfx950: 256 x 256 output tiles, groups of 128 * 2^j, the
// group scale folded into the fp16 weight fragment (as gemm7).
//
// Replaces LauncherBase::gemm / run_block + WeightKBlockNInteger::getFpWeight + the AMX / AVX512 GEMM cores
// (bestla/bestla/bestla_wrapper.h:481-542, bestla_prologue_b.h:732-838) for prefill M where the tiles fill the chip.
//
// Why a 256-column tile (prefill): the weights are 4-bit, so a tile's bytes per k are dominated by the
// activation rows (256 rows x 2 B against 256 columns x 0.5 B): gemm7's 256 x 128 tile moves 576 B per k for 65536
// flop, and its L2 -> LDS activation stream (60 GB/s per CU measured, profiles/r05_gemm6_7_diag.txt) overlaps its
// MFMAs poorly.  256 x 256 moves 640 B per k for twice the flops.  The weights are staged packed (16 KiB per 128-deep
// tile) and every wave dequantizes the fragments it multiplies; the activation tile is staged as fp16.
//
// Shape of the loop.  8 waves as 2 (M) x 4 (N), each owning 128 x 64 of the tile (8 x 4 fragments of 16 x 16, 128
// accumulator VGPRs).  A 64-deep K step u: 4 phases of 16 v_mfma_f32_16x16x32_f16 (two row fragments x four column
// fragments x two 32-deep halves) with the next phase's activation fragments read from LDS under them; the weight
// fragments of step u + 1 are read and dequantized in phase 3.  Operands are swapped (weights as the A operand, C^T
// comes out) so each lane holds 4 consecutive output columns of one row: float4 stores, no LDS transpose.
//
// Staging (LDS-DMA, 147 KiB): waves 4-7 move the activations (32 KiB per step, 8 pieces each) two steps ahead into a
// ring of 3 slots and drain them at the end of every step; waves 0-3 move the packed weight tiles (16 KiB + scale /
// zero-point rows per 128-deep tile, 4 pieces each) two tiles ahead into a ring of 3 slots, leaving the newest tile in
// flight across the step's barrier.  The split matters: DMAs retire in issue order per wave, so a wave that moved both
// would drain the weight tile (an HBM miss) every time it waited for its activations (an L2 hit); with one step of
// cover for both the kernel ran at 0.33 of the MFMA peak, latency-bound (profiles/r05_gemm9_*).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "woq_device.h"
#include "woq_kernels.h"

namespace nad {
namespace g9 {

constexpr int BM = 256, BN = 256, NS = BN / 16;  // tile rows, columns, stripes
constexpr int KT = 128;                            // K tile of the int4 layout (one packed weight tile)
constexpr int ROWB = 128;                          // bytes of one activation row per 64-deep step
constexpr int ABUF = BM * ROWB;                    // one activation slot (32 KiB)
constexpr int NA = 3;                              // activation slots
constexpr int BTILE = NS * 1024;                   // packed weights of one K tile (16 KiB)
constexpr int BSC = NS * 16 * 2;                   // their fp16 scale rows (512 B; f32 / bf16 scales: see kScaleBytes)
constexpr int BSCMAX = NS * 16 * 4;                // room for f32 scales
constexpr int BZP = NS * 16;                       // int8 zero points (256 B)
constexpr int BBUF = BTILE + BSCMAX + BZP;         // one weight slot
constexpr int NB = 3;                              // weight slots
constexpr int LDS = NA * ABUF + NB * BBUF;         // 98304 + 3 * 17664 = 151296 B
static_assert(LDS <= 160 * 1024, "LDS");

__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, -1, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, char* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ void blds4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, char* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 4, voff, soff, 0, 0);
}
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return uint32_t(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p));
}
// LDS reads in inline asm (hipcc would wait vmcnt(0) in front of every LDS read it sees while an LDS-DMA is in
// flight); consumed only after an explicit lgkmcnt wait that names them
template <int OFF>
__device__ __forceinline__ h8_t lds_b128(uint32_t addr) {
  h8_t r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ uint2 lds_b64(uint32_t addr) {
  uint2 r;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ uint32_t lds_b32(uint32_t addr) {
  uint32_t r;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}
template <class T>
__device__ __forceinline__ void tie(T& r) {
  asm volatile("" : "+v"(r));
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
// one 32-deep step's weight fragment: 8 nibbles -> fp16 (q - 8 - zp) * s, the product rounded once (gemm7's fold)
__device__ __forceinline__ h8_t dequant_fold(uint32_t w, uint32_t mag, h2_t s16, h2_t c0, h2_t c1, h2_t sc) {
  const uint32_t w8 = w >> 8;
  const h2_t p0 = (as_h2(and_or(w, 0x000F000Fu, mag)) + c0) * sc;
  const h2_t p1 = __builtin_elementwise_fma(as_h2(and_or(w, 0x00F000F0u, mag)), s16, c1) * sc;
  const h2_t p2 = (as_h2(and_or(w8, 0x000F000Fu, mag)) + c0) * sc;
  const h2_t p3 = __builtin_elementwise_fma(as_h2(and_or(w8, 0x00F000F0u, mag)), s16, c1) * sc;
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

#define G9_FENCE() __builtin_amdgcn_sched_barrier(0)
// diagnostic builds only (make g9x): 1 = no dequantization (raw bits as the operand), 2 = no MFMA, 4 = no DMA,
// 8 = no DMA wait in the loop
#ifndef NAD_G9_DEV
#define NAD_G9_DEV 0
#endif

template <bool ASYM, int ST>
__global__ __launch_bounds__(512, 1) void woq_gemm9_kernel(GemmArgs a, const _Float16* __restrict__ A16, int lda16) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int wr = wave >> 2, wc = wave & 3;  // M half, N quarter
  const SkinnyWeight& W = a.w;
  const int M = a.M, nt = W.nt, ng = W.ng, ns = W.ns;
  const int tsh = __builtin_ctz(unsigned(W.bs / KT));
  const int nl = lane & 15, kq = lane >> 4;

  // XCD-aware remap: the workgroups of one XCD are consecutive tiles of one row of tiles (shared activation rows)
  const int nbm = (M + BM - 1) / BM, nbn = (ns + NS - 1) / NS;
  const int nwg = nbm * nbn;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8, o = bid / 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + o;
  }
  const int bm = bid / nbn, bn = bid % nbn;
  const int m0 = bm * BM;
  const int nh = 2 * nt;  // 64-deep steps

  // activation DMA (waves 4-7): piece p (rows 8p .. 8p + 7 of the 256, one 1 KiB wave instruction) -> wave pieces
  // 8 (w & 3) .. + 7; lane -> row 8p + (lane >> 3), 16-B chunk (lane & 7) ^ ((row >> 1) & 7) of the 128-B row (the read
  // side's swizzle).  Weight DMA (waves 0-3): stripes 4 w .. + 3 of the tile (1 KiB each), the scale rows (8 or 4
  // stripes per 256-B piece; waves of equal parity / index move the same piece) and the zero-point rows (one piece).
  const bool aw = wave >= 4;  // the activation-DMA waves (the delayed half, see the loop)
  const int wq = wave & 3;
  uint32_t aoff[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int p = wq * 8 + i;
    const int row = p * 8 + (lane >> 3);
    const int grow = min(m0 + row, M - 1);  // rows past M re-read row M - 1 (never stored)
    aoff[i] = uint32_t(grow) * uint32_t(lda16) * 2u + uint32_t(((lane & 7) ^ ((row >> 1) & 7)) * 16);
  }
  const auto ra = brsrc(A16);
  const auto rb = brsrc(W.tiles);
  const auto rs = brsrc(W.scales);
  const auto rz = brsrc(W.zps);
  const auto rnull = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(W.tiles), 0, 0, 0x00020000);
  constexpr int SB = ST == kScaleF32 ? 4 : 2;  // scale bytes
  uint32_t boff[4];
#pragma unroll
  for (int i = 0; i < 4; i++)
    boff[i] = (uint32_t(min(bn * NS + 4 * wq + i, ns - 1)) * nt * 64 + lane) * 16;
  // scale piece: lane -> stripe (SB == 2: 8 stripes x 32 B per 256-B piece, two pieces; SB == 4: 4 stripes x 64 B,
  // four pieces) and a dword of its row
  const int spc = SB == 2 ? (wq & 1) : wq;
  const int sps = SB == 2 ? 8 : 4;  // stripes per scale piece
  const int sstripe = min(bn * NS + spc * sps + lane / (16 * SB / 4), ns - 1);
  const uint32_t svo = (uint32_t(sstripe) * ng * 16 * SB) + uint32_t(lane % (16 * SB / 4)) * 4;
  const int zstripe = min(bn * NS + (lane >> 2), ns - 1);
  const uint32_t zvo = uint32_t(zstripe) * ng * 16 + uint32_t(lane & 3) * 4;

  // activations of step v (waves 4-7); steps past the end load from the zero-record resource
  auto issue_a = [&](int v) {
    if constexpr ((NAD_G9_DEV & 4) != 0) {
      if (v >= 2) return;
    }
    const auto rA = v < nh ? ra : rnull;
    char* slot = smem + (v % NA) * ABUF + wq * 8 * 1024;
#pragma unroll
    for (int i = 0; i < 8; i++) blds16(rA, aoff[i], uint32_t(v) * ROWB, slot + i * 1024);
  };
  // weight tile t with its scale / zero-point rows (waves 0-3)
  constexpr int NBD = 4 + 1 + (ASYM ? 1 : 0);  // DMAs per tile per weight wave
  auto issue_b = [&](int t) {
    if constexpr ((NAD_G9_DEV & 4) != 0) {
      if (t >= 2) return;
    }
    const bool live = t < nt;
    char* bb = smem + NA * ABUF + (t % NB) * BBUF;
    const auto rB = live ? rb : rnull;
#pragma unroll
    for (int i = 0; i < 4; i++) blds16(rB, boff[i], uint32_t(t) * 1024, bb + (4 * wq + i) * 1024);
    const uint32_t g = uint32_t(t >> tsh) * 16 * SB;
    blds4(live ? rs : rnull, svo, g, bb + BTILE + spc * 256);
    if constexpr (ASYM) blds4(live ? rz : rnull, zvo, uint32_t(t >> tsh) * 16, bb + BTILE + BSCMAX);
  };

  // read side: activation fragment (row fragment i of the wave's 8, 32-deep half ks) of slot v
  const uint32_t roff = uint32_t((wr * 128 + nl) * ROWB);
  const uint32_t rsw0 = uint32_t(((0 * 4 + kq) ^ ((nl >> 1) & 7)) * 16);
  const uint32_t rsw1 = uint32_t(((1 * 4 + kq) ^ ((nl >> 1) & 7)) * 16);
  // weight words of the wave's stripe j: lane's 16 B, half h (8 B) of the 128-deep tile
  const uint32_t bwo = uint32_t((wc * 4) * 1024 + lane * 16);
  const uint32_t sco = uint32_t(BTILE + ((wc * 4) * 16 + (nl & ~(SB == 2 ? 1 : 0))) * SB);
  const int ssh = SB == 2 ? (nl & 1) * 16 : 0;
  const uint32_t zpo = uint32_t(BTILE + BSCMAX + (wc * 4) * 16 + nl);

  const uint32_t mag = 0x64006400u;
  const h2_t s16 = splat(1.f / 16.f);
  const h2_t zc0 = splat(-(1024.f + 8.f)), zc1 = splat(-(64.f + 8.f));
  auto scale_h2 = [&](uint32_t x) {
    if constexpr (ST == kScaleF32) return splat(__uint_as_float(x));
    const uint32_t h = (x >> ssh) & 0xFFFFu;
    if constexpr (ST == kScaleF16) return as_h2(h | (h << 16));
    return splat(__uint_as_float(h << 16));
  };

  f4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  h8_t af[2][2][2];  // [phase parity][row fragment of the phase][32-deep half]
  h8_t bf[4][2];     // dequantized weight fragments of the current step [stripe][half]
  uint2 bw[4];       // packed weight words of the next step
  uint32_t sw[4];    // scale words (read at a tile start)
  uint32_t zw[4];
  h2_t sc[4], c0[4], c1[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    c0[j] = zc0;
    c1[j] = zc1;
    sw[j] = 0u;
    zw[j] = 0u;
  }

  // phase-p activation fragments of step v into af[P]
  auto read_a = [&](auto Pc, int p, int v) {
    constexpr int P = decltype(Pc)::value;
    const uint32_t base = lds_addr(smem + (v % NA) * ABUF) + roff + uint32_t(p * 2 * 16 * ROWB);
    af[P][0][0] = lds_b128<0>(base + rsw0);
    af[P][0][1] = lds_b128<0>(base + rsw1);
    af[P][1][0] = lds_b128<16 * ROWB>(base + rsw0);
    af[P][1][1] = lds_b128<16 * ROWB>(base + rsw1);
  };
  // weight words (+ scale / zero-point words at a tile start) of step v
  auto read_b = [&](int v) {
    const int t = v >> 1, h = v & 1;
    const uint32_t bl = lds_addr(smem + NA * ABUF + (t % NB) * BBUF);
    const uint32_t wb = bl + bwo + uint32_t(h * 8);
    bw[0] = lds_b64<0>(wb);
    bw[1] = lds_b64<1024>(wb);
    bw[2] = lds_b64<2048>(wb);
    bw[3] = lds_b64<3072>(wb);
    if (h == 0) {
      sw[0] = lds_b32<0>(bl + sco);
      sw[1] = lds_b32<16 * SB>(bl + sco);
      sw[2] = lds_b32<32 * SB>(bl + sco);
      sw[3] = lds_b32<48 * SB>(bl + sco);
      if constexpr (ASYM) {
        // the zero point byte of this lane's column in each of the 4 stripes (dword-aligned reads, byte selected)
        zw[0] = lds_b32<0>((bl + zpo) & ~3u);
        zw[1] = lds_b32<16>((bl + zpo) & ~3u);
        zw[2] = lds_b32<32>((bl + zpo) & ~3u);
        zw[3] = lds_b32<48>((bl + zpo) & ~3u);
      }
    }
  };
  auto dequant_b = [&](int v) {
    if ((v & 1) == 0) {  // a tile start: its scales (and zero points)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        sc[j] = scale_h2(sw[j]);
        if constexpr (ASYM) {
          const float z = float(int(int8_t((zw[j] >> ((nl & 3) * 8)) & 0xFFu)));
          c0[j] = zc0 - splat(z);
          c1[j] = zc1 - splat(z);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if constexpr (NAD_G9_DEV & 1) {
        bf[j][0] = __builtin_bit_cast(h8_t, u4_t{bw[j].x, bw[j].y, bw[j].x, bw[j].y});
        bf[j][1] = __builtin_bit_cast(h8_t, u4_t{bw[j].y, bw[j].x, bw[j].y, bw[j].x});
      } else {
        bf[j][0] = dequant_fold(bw[j].x, mag, s16, c0[j], c1[j], sc[j]);
        bf[j][1] = dequant_fold(bw[j].y, mag, s16, c0[j], c1[j], sc[j]);
      }
    }
  };
  auto mfma_phase = [&](auto Pc, int p) {
    constexpr int P = decltype(Pc)::value;
#pragma unroll
    for (int ks = 0; ks < 2; ks++)
#pragma unroll
      for (int ii = 0; ii < 2; ii++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
          f4_t& c = acc[2 * p + ii][j];
          if constexpr (NAD_G9_DEV & 2) {
            const h8_t x = bf[j][ks], y = af[P][ii][ks];
            asm volatile("" ::"v"(x), "v"(y));
          } else {
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][ks], af[P][ii][ks], c, 0, 0, 0);
          }
        }
  };

  // prologue: activations of steps 0, 1 and weight tiles 0, 1 landed and published, then step 0's operands
  if (aw) {
    issue_a(0);
    issue_a(1);
  } else {
    issue_b(0);
    issue_b(1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  G9_FENCE();
  read_b(0);
  read_a(std::integral_constant<int, 0>{}, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  G9_FENCE();
#pragma unroll
  for (int j = 0; j < 4; j++) {
    tie(bw[j]);
    tie(sw[j]);
    tie(zw[j]);
  }
  dequant_b(0);
  // stagger: waves 4-7 run half a step behind waves 0-3 (one barrier late), so each SIMD pairs one wave's MFMA phases
  // with its partner's loads, dequantization and waits (MI355X_MICROARCH.md, two waves per SIMD, item 9).  Barrier
  // g = 2u + 1 + (wave >= 4) is wave's mid-step u, g + 1 its end of step u.  Hazards, by global barrier: waves 4-7
  // issue the activations of step u + 2 after barrier 2u + 1 into the slot of step u - 1, which waves 0-3 left at
  // barrier 2u and waves 4-7 at 2u + 1; they drain them before 2u + 3, and the first read (phase 3 of step u + 1) is
  // after 2u + 3 (waves 0-3) / 2u + 4.  Waves 0-3 issue weight tile T at step 2T - 4 (after barrier 4T - 8) into the slot
  // of tile T - 3 (last read in step 2T - 6, before barrier 4T - 9) and drain it before 4T - 2; its first read (phase 3
  // of step 2T - 1) is after 4T - 1.
  if (wave >= 4) __builtin_amdgcn_s_barrier();

  for (int u = 0; u < nh; u++) {
    G9_FENCE();
    if (aw)
      issue_a(u + 2);
    else if ((u & 1) == 0)
      issue_b((u >> 1) + 2);
    G9_FENCE();
    // phases 0 .. 2: next phase's fragments from this step's slot under this phase's MFMAs
    read_a(std::integral_constant<int, 1>{}, 1, u);
    G9_FENCE();
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");  // phase 0's fragments (4 newer reads in flight)
    G9_FENCE();
    mfma_phase(std::integral_constant<int, 0>{}, 0);
    G9_FENCE();
    read_a(std::integral_constant<int, 0>{}, 2, u);
    G9_FENCE();
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
    G9_FENCE();
    mfma_phase(std::integral_constant<int, 1>{}, 1);
    G9_FENCE();
    __builtin_amdgcn_s_barrier();  // mid-step (pairs with the partner half's end of step)
    G9_FENCE();
    read_a(std::integral_constant<int, 1>{}, 3, u);
    G9_FENCE();
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
    G9_FENCE();
    mfma_phase(std::integral_constant<int, 0>{}, 2);
    G9_FENCE();
    // phase 3: step u + 1's weight words and phase-0 fragments
    if (u + 1 < nh) {
      read_b(u + 1);
      read_a(std::integral_constant<int, 0>{}, 0, u + 1);
    }
    G9_FENCE();
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // phase 3's fragments (<= 8 newer reads in flight)
    G9_FENCE();
    mfma_phase(std::integral_constant<int, 1>{}, 3);
    G9_FENCE();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G9_FENCE();
#pragma unroll
    for (int j = 0; j < 4; j++) {
      tie(bw[j]);
      tie(sw[j]);
      tie(zw[j]);
    }
    if (u + 1 < nh) dequant_b(u + 1);
    // end of step: the activation waves drain their DMAs, the weight waves leave the newest tile in flight
    if constexpr ((NAD_G9_DEV & 8) == 0) {  // 8: diagnostic, no DMA wait in the loop (wrong results)
      if (aw)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NAD_G9_DEV & 4) ? 0 : NBD) : "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (wave < 4) __builtin_amdgcn_s_barrier();  // equal barrier counts
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  // epilogue: lane l holds columns 4 (l >> 4) .. + 3 of stripe j, row l & 15 of row fragment i
  const int n0w = bn * BN + wc * 64 + kq * 4;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int row = m0 + wr * 128 + i * 16 + nl;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int n0 = n0w + j * 16;
      if (n0 >= W.n) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      gemm_epilogue4(a, row, n0, v);
    }
  }
}

}  // namespace g9

bool gemm9_ok(int bits, int blocksize, int fold_ok) {
  const int tpg = blocksize / g9::KT;
  return bits == 4 && fold_ok && blocksize % g9::KT == 0 && (tpg & (tpg - 1)) == 0;
}

int gemm9_tiles(int m, int ns) { return ((m + g9::BM - 1) / g9::BM) * ((ns + g9::NS - 1) / g9::NS); }

hipError_t launch_gemm9(const GemmArgs& a, const _Float16* A16, int lda16, hipStream_t st) {
  const dim3 grid(gemm9_tiles(a.M, a.w.ns));
  auto go = [&](auto k, bool& done) -> hipError_t {
    if (!done) {  // opt in to the dynamic LDS once per instantiation
      hipError_t e =
          hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, g9::LDS);
      if (e != hipSuccess) return e;
      done = true;
    }
    hipLaunchKernelGGL(k, grid, dim3(512), g9::LDS, st, a, A16, lda16);
    return hipGetLastError();
  };
  static bool attr[2][3] = {};
  const bool asym = a.w.zps != nullptr;
  bool& d = attr[asym][a.scale_t];
  switch (a.scale_t) {
    case kScaleF32:
      return asym ? go(g9::woq_gemm9_kernel<true, kScaleF32>, d) : go(g9::woq_gemm9_kernel<false, kScaleF32>, d);
    case kScaleBF16:
      return asym ? go(g9::woq_gemm9_kernel<true, kScaleBF16>, d) : go(g9::woq_gemm9_kernel<false, kScaleBF16>, d);
    default:
      return asym ? go(g9::woq_gemm9_kernel<true, kScaleF16>, d) : go(g9::woq_gemm9_kernel<false, kScaleF16>, d);
  }
}

}  // namespace nad
