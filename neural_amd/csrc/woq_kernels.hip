// woq_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the weight-only-quantized matmul hot path.
//
//   nad_repack_kernel   : BTLA blob (any core layout, NTILE 24/48, PACK_ROW 1/2/4; S2-S8) -> tile layout
//                         (woq_layout.h).  Replaces convertTransStorage + fromHost of the SYCL backend
//                         (bestla/bestla/bestla_prologue_b.h:129-150, neural_speed/core/layers/ne_bestla_sycl.cpp:94-144).
//   woq_skinny_kernel   : M <= 16 ("GEMV", decode).  Replaces GEMVWrapper::gemv_kblock -> gemv_{4,2}bit_fp32_fp32
//                         (bestla/bestla/bestla_wrapper.h:364-468, kernel_ref.h:2489-2531,2712-2760).
//                         One wave streams one 16-column stripe over a K slice with fully coalesced 16 B/lane loads
//                         of 1 KiB tiles, dequantizes nibbles/crumbs/bytes to exact integer fp16 with the 0x6400
//                         magic (no LUT, no shuffles), and runs v_mfma_f32_16x16x32_f16 with the activation rows in
//                         the A operand.  fp32 activations are split hi+lo into the 16 MFMA rows (M<=8) or into two
//                         MFMA passes (M<=16) so the result is fp32-accurate; group scales are applied in fp32 once
//                         per group; the K slices of a stripe are reduced in LDS inside the workgroup (deterministic,
//                         no atomics).  HBM-bound by design: every weight byte is read exactly once.
//   woq_gemm_kernel     : M > 16 (prefill).  Replaces LauncherBase::gemm/run_block + getFpWeight + the AMX/AVX512
//                         GemmCore (bestla_wrapper.h:481-542, bestla_prologue_b.h:732-838).  128x128 block tile,
//                         4 waves of 64x64; A staged fp32->fp16 into an XOR-swizzled LDS tile; B tiles go HBM ->
//                         VGPR -> exact-integer fp16 fragments with no LDS round trip; per-group fp32 scaling of a
//                         group accumulator keeps the weight dequant exact.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "woq_device.h"
#include "woq_kernels.h"

namespace nad {


// ------------------------------------------------------------------------------------------------ repack
// signed integer q of blob element e (interleaved order).  S2/S4: crumb / nibble = q + 2^(b-1); S8: the byte;
// S1/S3/S5/S6/S7: u = q + 2^(b-1) split over a nibble plane [nel/2], a crumb plane [nel/4] and a bit plane [nel/8]
// (1 = bit, 3 = crumb|bit, 5 = nibble|bit, 6 = nibble|crumb, 7 = nibble|crumb|bit; kernel_ref.h:178-361).  S1
// repacks into the int2 tile layout (q in {-1, 0}).
__device__ __forceinline__ int blob_q(const RepackArgs& a, uint64_t e) {
  const uint8_t* q = a.src_q;
  switch (a.src_bits) {
    case 8:
      return int(int8_t(q[e]));
    case 4:
      return int((q[e >> 1] >> (4 * (e & 1))) & 0xF) - 8;
    case 2:
      return int((q[e >> 2] >> (2 * (e & 3))) & 0x3) - 2;
    default:
      break;
  }
  const int b = a.src_bits;
  const bool has4 = b >= 5, has2 = b == 3 || b >= 6, has1 = b == 1 || b == 3 || b == 5 || b == 7;
  uint64_t off = 0;
  uint32_t u = 0;
  int sh = 0;
  if (has4) {
    u = (q[e >> 1] >> (4 * (e & 1))) & 0xF;
    sh = 4;
    off = a.nel / 2;
  }
  if (has2) {
    u |= ((q[off + (e >> 2)] >> (2 * (e & 3))) & 0x3u) << sh;
    sh += 2;
    off += a.nel / 4;
  }
  if (has1) u |= ((q[off + (e >> 3)] >> (e & 7)) & 0x1u) << sh;
  return int(u) - (1 << (b - 1));
}

// One thread per output dword of the tile layout.
__global__ void nad_repack_kernel(RepackArgs a) {
  const uint64_t total = uint64_t(a.ns) * a.nt * 256;
  const int KT = a.bits == 4 ? 128 : (a.bits == 2 ? 256 : 64);
  for (uint64_t gid = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; gid < total;
       gid += uint64_t(gridDim.x) * blockDim.x) {
    const int dw = int(gid & 3);
    const int lane = int((gid >> 2) & 63);
    const uint64_t tile = gid >> 8;
    const int t = int(tile % a.nt);
    const int s = int(tile / a.nt);
    const int n = s * 16 + (lane & 15);
    const int kq = lane >> 4;
    uint32_t out = 0;
    const int per = 32 / a.bits;  // elements per dword
    for (int p = 0; p < per; p++) {
      int k;
      if (a.bits == 4) {
        int j = 2 * (p & 3) + (p >> 2);
        k = t * KT + dw * 32 + kq * 8 + j;
      } else if (a.bits == 2) {
        int h = (p & 7) >> 2, j = 2 * (p & 3) + (p >> 3);
        int d = dw * 2 + h;
        k = t * KT + d * 32 + kq * 8 + j;
      } else {
        int d = dw >> 1, j = (dw & 1) * 4 + p;
        k = t * KT + d * 32 + kq * 8 + j;
      }
      uint32_t v;
      if (n < a.n && k < a.k) {
        const uint64_t e = uint64_t(n / a.ntile) * a.ntile * a.kpad + uint64_t(k / a.packrow) * a.ntile * a.packrow +
                           uint64_t(n % a.ntile) * a.packrow + uint64_t(k % a.packrow);
        v = a.raw ? uint32_t(blob_q(a, e)) & 0xFFu
                  : uint32_t(blob_q(a, e) + (a.bits == 4 ? 8 : (a.bits == 2 ? 2 : 128)));  // device: q + 2^(bits-1)
      } else {
        v = a.raw ? 0u : (a.bits == 4 ? 8u : (a.bits == 2 ? 2u : 128u));  // q = 0 padding (F8: code 0)
      }
      out |= v << (a.bits * p);
    }
    a.dst_tiles[tile_index(a.kmajor, a.ns, a.nt, s, t) * 256 + (gid & 255)] = out;
  }
}

__global__ void nad_repack_scales_kernel(RepackArgs a) {
  const int total = a.ns * a.ng * 16;
  const int ssz = a.scale_t == kScaleF32 ? 4 : 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i & 15, g = (i >> 4) % a.ng, s = (i >> 4) / a.ng;
    const int n = s * 16 + c;
    const bool ok = n < a.n;
    const uint64_t src = uint64_t(g) * a.cstep + n;
    const uint64_t dst = scale_row(a.kmajor, a.ns, a.ng, s, g) * 16 + c;
    if (a.src_e8m0) {  // decompress_kblock_f8_fp (kernel_ref.h:1013-1015): scale = 2^(int8)e, exact in fp32
      static_cast<float*>(a.dst_scales)[dst] = ok ? ldexpf(1.f, int(reinterpret_cast<const int8_t*>(a.src_s)[src])) : 0.f;
    } else if (ssz == 4) {
      static_cast<float*>(a.dst_scales)[dst] = ok ? reinterpret_cast<const float*>(a.src_s)[src] : 0.f;
    } else {
      static_cast<uint16_t*>(a.dst_scales)[dst] = ok ? reinterpret_cast<const uint16_t*>(a.src_s)[src] : 0;
    }
    if (a.dst_zps) a.dst_zps[dst] = ok ? a.src_z[src] : 0;
  }
}


// store one staged activation vector (VEC elements of row `row` at column k) as fp16 hi (+ lo) rows
template <int AT, int VEC>
__device__ __forceinline__ void stage_store(char* smem, uint4 x, int row, int k, int Kp, int M) {
  if constexpr (AT == kActF16) {
    *reinterpret_cast<uint4*>(smem + (size_t(row) * Kp + k) * 2) = x;
  } else {
    float f[VEC];
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
    if constexpr (AT == kActF32) {
#pragma unroll
      for (int j = 0; j < 4; j++) f[j] = __uint_as_float(w[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        f[2 * j] = __uint_as_float(w[j] << 16);
        f[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
      }
    }
    _Float16 hi[VEC], lo[VEC];
#pragma unroll
    for (int j = 0; j < VEC; j++) {
      hi[j] = _Float16(f[j]);
      lo[j] = _Float16(f[j] - float(hi[j]));
    }
    char* ph = smem + (size_t(row) * Kp + k) * 2;
    char* pl = smem + (size_t(M + row) * Kp + k) * 2;
    if constexpr (VEC == 4) {
      *reinterpret_cast<uint2*>(ph) = __builtin_bit_cast(uint2, hi);
      *reinterpret_cast<uint2*>(pl) = __builtin_bit_cast(uint2, lo);
    } else {
      *reinterpret_cast<uint4*>(ph) = __builtin_bit_cast(uint4, hi);
      *reinterpret_cast<uint4*>(pl) = __builtin_bit_cast(uint4, lo);
    }
  }
}

// ------------------------------------------------------------------------------------------------ skinny (M<=16)
// Dynamic LDS map:
//   [0, a_bytes)          ALDS: the activations staged ONCE per workgroup as MFMA-ready fp16 rows [R][Kp]
//                         (Kp = nt*KT, zero padded past K; the act-order gather of ShuffleActivationKBlock,
//                         bestla_prologue_a.h:407-422, is applied while staging).  fp32/bf16 inputs are split into
//                         hi = fp16(a) rows 0..M-1 and lo = fp16(a - hi) rows M..2M-1 (R = 2M), fp16 inputs are copied
//                         (R = M); a 16-B zero block follows for lanes whose MFMA row is unused.  The main loop then
//                         does one ds_read_b128 per step for A: no conversion, no global load on the critical path.
//   [a_bytes, ...)        group scales as fp32, then zp constants (half2 bits), [nwi][ng][16] each
//   reduction scratch     reuses offset 0 after the main loop
template <int BITS, int AT, int HILO, int CH, bool ALDS>
__global__ __launch_bounds__(1024) void woq_skinny_kernel(SkinnyArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KT = BITS == 4 ? 128 : (BITS == 2 ? 256 : 64);
  constexpr int SPT = KT / 32;
  constexpr int ESZ = AT == kActF32 ? 4 : 2;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int nwaves = blockDim.x >> 6;
  const bool dual = a.epi == kEpiSiluMul || a.epi == kEpiGeluMul;

  // which weight and stripe does this workgroup own (all wave-uniform)
  int wsel = 0;
  int sid = blockIdx.x;
  if (!dual) {
#pragma unroll
    for (int i = 1; i < 3; i++)
      if (i < a.nw && sid >= a.stripe_base[i]) wsel = i;
    sid -= a.stripe_base[wsel];
  }
  const int nwi = dual ? 2 : 1;
  const int KS = nwaves / nwi;
  const int my_w = dual ? (wave / KS) : wsel;
  const int ks = wave % KS;
  const SkinnyWeight& W = a.w[my_w];
  const int s = sid;
  const int nt = W.nt, ng = W.ng;
  const int Kp = nt * KT;
  const int R = HILO == 0 ? a.M : 2 * a.M;        // staged fp16 rows
  const int zero_off = R * Kp * 2;                 // 16-B zero block
  const int a_bytes = ALDS ? zero_off + 16 : 0;
  float* lds_scale = reinterpret_cast<float*>(smem + a_bytes);
  uint32_t* lds_zc = reinterpret_cast<uint32_t*>(smem + a_bytes + size_t(nwi) * ng * 16 * 4);

  // 1) this wave's weight tiles go out first: one coalesced 16 B/lane nontemporal load per 1 KiB tile
  const int tpw = a.tiles_per_wave;
  const int tw0 = ks * tpw;
  const int tw1 = min(nt, tw0 + tpw);
  const u4_t* tile_base = reinterpret_cast<const u4_t*>(W.tiles) + lane;
  const int tss = W.kmajor ? 1 : nt, tts = W.kmajor ? W.ns : 1;  // tile (s, t) at s * tss + t * tts
  u4_t b[CH];
#pragma unroll
  for (int i = 0; i < CH; i++) {
    int t = min(tw0 + i, nt - 1);
    b[i] = __builtin_nontemporal_load(tile_base + (size_t(s) * tss + size_t(t) * tts) * 64);
  }

  const int32_t* shf = W.shuffle;
  const bool vec_ok = a.vec_ok != 0;
  // 2) stage A (whole K, all M rows) and 3) the group scales / zp constants into LDS.  Rounds of fixed-size,
  //    clamped (never predicated) loads so that the first round is in flight together with the weight tiles: the
  //    prologue costs one memory round trip.
  {
    constexpr int VEC = 16 / ESZ;
    constexpr int AR = 4;  // A vectors per thread per round
    constexpr int SR = 4;  // scale entries per thread per round
    const int bd = blockDim.x;
    const int a_vecs = ALDS ? (a.M * Kp) / VEC : 0;
    const int cnt = ng * 16;
    const bool a_fast = a.a_fast != 0;
    const int rounds = max((a_vecs + bd * AR - 1) / (bd * AR), (cnt + bd * SR - 1) / (bd * SR));
    const char* Ab = static_cast<const char*>(a.A);
    auto stage_round = [&](const int r) {
      uint4 av[AR];
      float sv[SR];
      int zv[SR];
      if constexpr (ALDS) {
        if (a_fast) {
#pragma unroll
          for (int q = 0; q < AR; q++) {
            const int v = min((r * AR + q) * bd + int(threadIdx.x), a_vecs - 1);
            const int idx = v * VEC, row = idx / Kp, k = idx - row * Kp;
            const int kc = min(k, a.K - VEC);
            av[q] = *reinterpret_cast<const uint4*>(Ab + (size_t(row) * a.lda + kc) * ESZ);
          }
        }
      }
      // scales / zero points: loop the (<= 2) weights uniformly so their pointers stay scalar
      uint32_t sraw[2][SR];
      int zraw[2][SR];
#pragma unroll
      for (int wi = 0; wi < 2; wi++) {
        if (wi < nwi) {
          const SkinnyWeight& Wl = a.w[dual ? wi : wsel];
          // branch-free: a scale is read as two 16-bit halves (stride 2 for f32, the same half twice for bf16/f16)
          const int sstr = a.scale_t == kScaleF32 ? 2 : 1;
          const uint16_t* sp = static_cast<const uint16_t*>(Wl.scales);
          const bool hz = Wl.zps != nullptr;
          const int8_t* zp = hz ? Wl.zps : static_cast<const int8_t*>(Wl.scales);
          const int zmask = hz ? -1 : 0;
#pragma unroll
          for (int q = 0; q < SR; q++) {
            const int e = min((r * SR + q) * bd + int(threadIdx.x), cnt - 1);
            const size_t ei = scale_row(Wl.kmajor, Wl.ns, Wl.ng, s, e >> 4) * 16 + (e & 15);
            const uint32_t lo = sp[ei * sstr], hi = sp[ei * sstr + sstr - 1];
            sraw[wi][q] = lo | (hi << (16 * (sstr - 1)));  // f32: lo|hi<<16; 16-bit: lo|lo
            zraw[wi][q] = int(zp[hz ? ei : 0]) & zmask;
          }
        }
      }
      if constexpr (ALDS) {
        if (a_fast) {
#pragma unroll
          for (int q = 0; q < AR; q++) {
            const int v = (r * AR + q) * bd + int(threadIdx.x);
            if (v < a_vecs) {
              const int idx = v * VEC, row = idx / Kp, k = idx - row * Kp;
              uint4 x = av[q];
              if (k >= a.K) x = make_uint4(0u, 0u, 0u, 0u);
              stage_store<AT, VEC>(smem, x, row, k, Kp, a.M);
            }
          }
        } else {  // act-order gather / unaligned rows: element-wise staging
          for (int q = 0; q < AR; q++) {
            const int v = (r * AR + q) * bd + int(threadIdx.x);
            if (v >= a_vecs) break;
            const int idx = v * VEC, row = idx / Kp, k = idx - row * Kp;
            uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < VEC; j++) {
              const int kk = k + j;
              uint32_t e = 0;
              if (kk < a.K) {
                const size_t src = size_t(row) * a.lda + (shf ? shf[kk] : kk);
                if constexpr (ESZ == 4)
                  e = static_cast<const uint32_t*>(a.A)[src];
                else
                  e = static_cast<const uint16_t*>(a.A)[src];
              }
              if constexpr (ESZ == 4)
                w[j] = e;
              else
                w[j >> 1] |= e << (16 * (j & 1));
            }
            stage_store<AT, VEC>(smem, make_uint4(w[0], w[1], w[2], w[3]), row, k, Kp, a.M);
          }
        }
        if (threadIdx.x == 0 && r == 0) *reinterpret_cast<uint4*>(smem + zero_off) = make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int wi = 0; wi < 2; wi++) {
        if (wi < nwi) {
#pragma unroll
          for (int q = 0; q < SR; q++) {
            const int e = (r * SR + q) * bd + int(threadIdx.x);
            if (e < cnt) {
              const uint32_t x = sraw[wi][q];
              float sc;
              if (a.scale_t == kScaleF32)
                sc = __uint_as_float(x);
              else if (a.scale_t == kScaleBF16)
                sc = __uint_as_float(x << 16);
              else
                sc = f16_bits_to_f32(uint16_t(x));
              lds_scale[wi * cnt + e] = sc;
              lds_zc[wi * cnt + e] = __builtin_bit_cast(uint32_t, zp_const(bias_of<BITS>() + zraw[wi][q]));
            }
          }
        }
      }
    };
    stage_round(0);  // straight-line: in flight together with the weight tiles
    for (int r = 1; r < rounds; r++) stage_round(r);
  }
  __syncthreads();

  const int m = lane & 15;   // A-operand row fed by this lane
  const int kq = lane >> 4;  // k-quarter of the 32-k step
  const int M = a.M;
  // HILO==1: rows 0..7 carry hi(A[m]), rows 8..15 lo(A[m-8]); HILO==2: two MFMA passes; HILO==0: fp16 A as is
  const int arow = HILO == 1 ? (m & 7) : m;
  const bool is_lo = HILO == 1 && m >= 8;
  const bool aact = arow < M;
  // byte offsets of this lane's staged rows (hi row arow; lo row M + arow)
  const int a_hi_off = (HILO == 1 && is_lo ? (a.M + arow) : arow) * Kp * 2;
  const int a_lo_off = (a.M + arow) * Kp * 2;
  const float* sc_l = lds_scale + (dual ? my_w : 0) * ng * 16 + (lane & 15);
  const uint32_t* zc_l = lds_zc + (dual ? my_w : 0) * ng * 16 + (lane & 15);

  f4_t acc = {0.f, 0.f, 0.f, 0.f};
  f4_t accg = {0.f, 0.f, 0.f, 0.f};
  const F4Lut f4l = f4_lut_regs(BITS == 4 && W.f4 >= 0 ? W.f4 : 0);
  // group bookkeeping in scalars: g = group of the current step, rem = steps left in it
  const int spg = a.steps_per_group;
  const int st0 = tw0 * SPT;
  int g = min(st0 / spg, ng - 1);
  int rem = spg - (st0 - g * spg);
  const int last_step = tw1 * SPT - 1;

  for (int c0 = tw0; c0 < tw1; c0 += CH) {
    if (c0 != tw0) {
#pragma unroll
      for (int i = 0; i < CH; i++) {
        int t = min(c0 + i, nt - 1);
        b[i] = __builtin_nontemporal_load(tile_base + (size_t(s) * tss + size_t(t) * tts) * 64);
      }
    }
#pragma unroll
    for (int i = 0; i < CH; i++) {
      const int t = c0 + i;
      if (t < tw1) {
#pragma unroll
        for (int d = 0; d < SPT; d++) {
          const int st = t * SPT + d;
          const int k0 = st * 32 + kq * 8;
          const h2_t c2 = as_h2(zc_l[g * 16]);
          h8_t bf;
          if (BITS == 4 && W.f4 >= 0)
            bf = dequant_f4(b[i], d, f4l);
          else if (BITS == 8 && W.f4 >= 3)
            bf = dequant_f8(b[i], d, W.f4 == 4);
          else
            bf = dequant_step<BITS>(b[i], d, c2);
          if constexpr (ALDS) {
            const h8_t af = *reinterpret_cast<const h8_t*>(smem + (aact ? a_hi_off + k0 * 2 : zero_off));
            if (HILO == 2) {
              const h8_t afl = *reinterpret_cast<const h8_t*>(smem + (aact ? a_lo_off + k0 * 2 : zero_off));
              accg = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, accg, 0, 0, 0);
              accg = __builtin_amdgcn_mfma_f32_16x16x32_f16(afl, bf, accg, 0, 0, 0);
            } else {
              accg = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, accg, 0, 0, 0);
            }
          } else {
            float av[8];
            if (aact) {
              load_a8<AT>(a.A, a.lda, arow, k0, a.K, shf, vec_ok, av);
            } else {
#pragma unroll
              for (int j = 0; j < 8; j++) av[j] = 0.f;
            }
            h8_t ah, al;
#pragma unroll
            for (int j = 0; j < 8; j++) {
              const _Float16 h = _Float16(av[j]);
              ah[j] = h;
              if (HILO != 0) al[j] = _Float16(av[j] - float(h));
            }
            if (HILO == 1) {
              accg = __builtin_amdgcn_mfma_f32_16x16x32_f16(is_lo ? al : ah, bf, accg, 0, 0, 0);
            } else if (HILO == 2) {
              accg = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bf, accg, 0, 0, 0);
              accg = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bf, accg, 0, 0, 0);
            } else {
              accg = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bf, accg, 0, 0, 0);
            }
          }
          if (rem == 1 || st == last_step) {
            acc += accg * sc_l[min(g, ng - 1) * 16];
            accg = f4_t{0.f, 0.f, 0.f, 0.f};
          }
          if (--rem == 0) {
            rem = spg;
            g = min(g + 1, ng - 1);
          }
        }
      }
    }
  }

  // 4) HILO==1 folds the lo rows (8..15, lanes 32..63) onto the hi rows (0..7, lanes 0..31)
  if (HILO == 1) {
#pragma unroll
    for (int i = 0; i < 4; i++) acc[i] += __shfl_down(acc[i], 32, 64);
  }
  // 5) reduce the K slices through LDS
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  *reinterpret_cast<f4_t*>(red + (size_t(wave) * 64 + lane) * 4) = acc;
  __syncthreads();
  for (int o = threadIdx.x; o < 256; o += blockDim.x) {
    const int mm = o >> 4, nn = o & 15;
    if (mm >= M) continue;
    const int src_lane = (mm >> 2) * 16 + nn, reg = mm & 3;
    float y0 = 0.f, y1 = 0.f;
    for (int w = 0; w < KS; w++) y0 += red[(size_t(w) * 64 + src_lane) * 4 + reg];
    if (dual)
      for (int w = 0; w < KS; w++) y1 += red[(size_t(KS + w) * 64 + src_lane) * 4 + reg];
    const SkinnyWeight& Wo = a.w[dual ? 0 : wsel];
    const int n = s * 16 + nn;
    if (n >= Wo.n) continue;
    float v = y0;
    switch (a.epi) {
      case kEpiBias:
        v += Wo.bias[size_t(mm) * Wo.bias_ld + n];
        break;
      case kEpiAddGelu:
        v = gelu_f(v + Wo.bias[size_t(mm) * Wo.bias_ld + n]);
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
        const float t1 = silu_f(y0);
        if (a.aux) a.aux[size_t(mm) * a.ld_aux + n] = t1;
        v = t1 * y1;
        break;
      }
      case kEpiGeluMul: {
        const float t1 = gelu_f(y0);
        if (a.aux) a.aux[size_t(mm) * a.ld_aux + n] = t1;
        v = t1 * y1;
        break;
      }
      default:
        break;
    }
    Wo.out[size_t(mm) * Wo.ldo + n] = v;
  }
}

// ------------------------------------------------------------------------------------------------ GEMM (M>16)
// Block 256 threads = 4 waves (2 x 2); block tile BM x BN = 128 x 128 (8 stripes); K step = one tile (KT).
// LDS A tile: [128 rows][KT fp16] with 16-B chunk XOR swizzle (chunk ^= row & 15).
template <int BITS, int AT>
__global__ __launch_bounds__(256, 2) void woq_gemm_kernel(GemmArgs a) {
  constexpr int KT = BITS == 4 ? 128 : (BITS == 2 ? 256 : 64);
  constexpr int SPT = KT / 32;
  constexpr int BM = 128, BN = 128;
  constexpr int ROWB = KT * 2;            // bytes per LDS row (fp16)
  constexpr int CHUNKS = ROWB / 16;       // 16-B chunks per row
  __shared__ __attribute__((aligned(16))) char lds_a[BM * ROWB];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const SkinnyWeight& W = a.w;

  // XCD-aware remap: consecutive workgroups (same N tile, different M tiles) land on one XCD's L2
  const int nbm = (a.M + BM - 1) / BM;
  const int nbn = (W.ns + 7) / 8;
  const int nwg = nbm * nbn;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8, o = bid / 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + o;
  }
  const int bn = bid / nbm, bm = bid % nbm;
  const int m0 = bm * BM;
  const int s0 = bn * 8 + wn * 4;         // first stripe of this wave
  const int nt = W.nt, bs = W.bs;

  f4_t acc[4][4], accg[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
      accg[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
    }
  const F4Lut f4l = f4_lut_regs(BITS == 4 && W.f4 >= 0 ? W.f4 : 0);

  // A staging map: 256 threads cover BM rows x KT k; each thread handles rows r0 + 32*i, chunk ch (8 k values)
  constexpr int TPR = CHUNKS;              // threads per row chunk group
  constexpr int ROWS_PER_PASS = 256 / TPR;
  constexpr int PASSES = BM / ROWS_PER_PASS;
  const int ch = threadIdx.x % TPR;
  const int r0 = threadIdx.x / TPR;
  const bool vec_ok = a.vec_ok != 0;
  const int32_t* shf = W.shuffle;

  const u4_t* tiles = reinterpret_cast<const u4_t*>(W.tiles);
  u4_t bcur[4], bnext[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    int s = min(s0 + j, W.ns - 1);
    bcur[j] = tiles[tile_index(W.kmajor, W.ns, nt, s, 0) * 64 + lane];
  }

  for (int t = 0; t < nt; t++) {
    // stage A(t) into LDS (fp32/bf16/fp16 -> fp16)
#pragma unroll
    for (int p = 0; p < PASSES; p++) {
      const int r = r0 + p * ROWS_PER_PASS;
      const int row = m0 + r;
      float v[8];
      if (row < a.M) {
        load_a8<AT>(a.A, a.lda, row, t * KT + ch * 8, a.K, shf, vec_ok, v);
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = 0.f;
      }
      h8_t hv;
#pragma unroll
      for (int j = 0; j < 8; j++) hv[j] = _Float16(v[j]);
      const int sw = ch ^ (r & 15 & (CHUNKS - 1));
      *reinterpret_cast<h8_t*>(lds_a + r * ROWB + sw * 16) = hv;
    }
    // prefetch next B tiles
    if (t + 1 < nt) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        int s = min(s0 + j, W.ns - 1);
        bnext[j] = tiles[tile_index(W.kmajor, W.ns, nt, s, t + 1) * 64 + lane];
      }
    }
    __syncthreads();
#pragma unroll
    for (int d = 0; d < SPT; d++) {
      const int st = t * SPT + d;
      const int g = min((st * 32) / bs, W.ng - 1);
      h8_t bf[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int s = min(s0 + j, W.ns - 1);
        const size_t zi = scale_row(W.kmajor, W.ns, W.ng, s, g) * 16 + (lane & 15);
        const int zp = W.zps ? int(W.zps[zi]) : 0;
        if (BITS == 4 && W.f4 >= 0)
          bf[j] = dequant_f4(bcur[j], d, f4l);
        else if (BITS == 8 && W.f4 >= 3)
          bf[j] = dequant_f8(bcur[j], d, W.f4 == 4);
        else
          bf[j] = dequant_step<BITS>(bcur[j], d, zp_const(bias_of<BITS>() + zp));
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int r = wm * 64 + i * 16 + (lane & 15);
        const int chunk = d * 4 + (lane >> 4);
        const int sw = chunk ^ (r & 15 & (CHUNKS - 1));
        const h8_t af = *reinterpret_cast<const h8_t*>(lds_a + r * ROWB + sw * 16);
#pragma unroll
        for (int j = 0; j < 4; j++) accg[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], accg[i][j], 0, 0, 0);
      }
      const bool gend = (((st + 1) * 32) % bs == 0) || (st == nt * SPT - 1);
      if (gend) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int s = min(s0 + j, W.ns - 1);
          const float sc = load_scale(W.scales, scale_row(W.kmajor, W.ns, W.ng, s, g) * 16 + (lane & 15), a.scale_t);
#pragma unroll
          for (int i = 0; i < 4; i++) {
            acc[i][j] += accg[i][j] * sc;
            accg[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; j++) bcur[j] = bnext[j];
  }

  // epilogue: C layout col = lane & 15, row = (lane >> 4) * 4 + reg
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int n = (s0 + j) * 16 + (lane & 15);
    if (s0 + j >= W.ns || n >= W.n) continue;
#pragma unroll
    for (int i = 0; i < 4; i++) {
#pragma unroll
      for (int rr = 0; rr < 4; rr++) {
        const int row = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + rr;
        if (row >= a.M) continue;
        float v = acc[i][j][rr];
        switch (a.epi) {
          case kEpiBias:
            v += W.bias[size_t(row) * W.bias_ld + n];
            break;
          case kEpiAddGelu:
            v = gelu_f(v + W.bias[size_t(row) * W.bias_ld + n]);
            break;
          case kEpiGelu:
            v = gelu_f(v);
            break;
          case kEpiSilu:
            v = silu_f(v);
            break;
          case kEpiResAdd:
            v += a.res[size_t(row) * a.ld_res + n];
            break;
          case kEpiSiluMul:  // second pass of the FFN: out = silu(tmp1) * (x.w3), aux holds silu(x.w1)
            v = a.aux[size_t(row) * a.ld_aux + n] * v;
            break;
          default:
            break;
        }
        W.out[size_t(row) * W.ldo + n] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ launchers
hipError_t launch_repack(const RepackArgs& a, hipStream_t stream) {
  const uint64_t total = uint64_t(a.ns) * a.nt * 256;
  int blocks = int(std::min<uint64_t>((total + 255) / 256, 65535));
  hipLaunchKernelGGL(nad_repack_kernel, dim3(blocks), dim3(256), 0, stream, a);
  int total_s = a.ns * a.ng * 16;
  int bs2 = std::min((total_s + 255) / 256, 65535);
  hipLaunchKernelGGL(nad_repack_scales_kernel, dim3(bs2), dim3(256), 0, stream, a);
  return hipGetLastError();
}

template <int BITS, int AT, int HILO, bool ALDS>
static hipError_t skinny_dispatch_ch(const SkinnyArgs& a, int ch, dim3 grid, dim3 block, size_t lds,
                                     hipStream_t stream) {
  if (ch == 4)
    hipLaunchKernelGGL((woq_skinny_kernel<BITS, AT, HILO, 4, ALDS>), grid, block, lds, stream, a);
  else
    hipLaunchKernelGGL((woq_skinny_kernel<BITS, AT, HILO, 8, ALDS>), grid, block, lds, stream, a);
  return hipGetLastError();
}

template <int BITS, int AT, int HILO>
static hipError_t skinny_dispatch_alds(const SkinnyArgs& a, bool alds, int ch, dim3 g, dim3 b, size_t lds,
                                       hipStream_t st) {
  if (alds) return skinny_dispatch_ch<BITS, AT, HILO, true>(a, ch, g, b, lds, st);
  return skinny_dispatch_ch<BITS, AT, HILO, false>(a, ch, g, b, lds, st);
}

template <int BITS>
static hipError_t skinny_dispatch_bits(const SkinnyArgs& a, int at, int hilo, bool alds, int ch, dim3 g, dim3 b,
                                       size_t lds, hipStream_t st) {
  if (at == kActF16) return skinny_dispatch_alds<BITS, kActF16, 0>(a, alds, ch, g, b, lds, st);
  if (at == kActF32) {
    if (hilo == 1) return skinny_dispatch_alds<BITS, kActF32, 1>(a, alds, ch, g, b, lds, st);
    return skinny_dispatch_alds<BITS, kActF32, 2>(a, alds, ch, g, b, lds, st);
  }
  if (hilo == 1) return skinny_dispatch_alds<BITS, kActBF16, 1>(a, alds, ch, g, b, lds, st);
  return skinny_dispatch_alds<BITS, kActBF16, 2>(a, alds, ch, g, b, lds, st);
}

static constexpr size_t kSkinnyLdsBudget = 64 * 1024;

hipError_t launch_skinny(const SkinnyArgs& a, int bits, int act_t, int waves_per_wg, int stripes, int ch,
                         hipStream_t stream) {
  const bool dual = a.epi == kEpiSiluMul || a.epi == kEpiGeluMul;
  const int nwi = dual ? 2 : 1;
  int ngmax = 0;
  for (int i = 0; i < a.nw; i++) ngmax = std::max(ngmax, a.w[i].ng);
  const int KT = bits == 4 ? 128 : (bits == 2 ? 256 : 64);
  const size_t rows = act_t == kActF16 ? size_t(a.M) : 2 * size_t(a.M);
  const size_t sc = size_t(nwi) * ngmax * 16 * 8;
  const size_t abytes = rows * a.w[0].nt * KT * 2 + 16;
  const bool alds = abytes + sc <= kSkinnyLdsBudget;
  size_t lds = std::max((alds ? abytes : 0) + sc, size_t(waves_per_wg) * 64 * 16);
  const int hilo = act_t == kActF16 ? 0 : (a.M <= 8 ? 1 : 2);
  dim3 grid(stripes), block(waves_per_wg * 64);
  if (bits == 4) return skinny_dispatch_bits<4>(a, act_t, hilo, alds, ch, grid, block, lds, stream);
  if (bits == 2) return skinny_dispatch_bits<2>(a, act_t, hilo, alds, ch, grid, block, lds, stream);
  return skinny_dispatch_bits<8>(a, act_t, hilo, alds, ch, grid, block, lds, stream);
}

template <int BITS>
static hipError_t gemm_dispatch_bits(const GemmArgs& a, int at, dim3 g, hipStream_t st) {
  if (at == kActF32)
    hipLaunchKernelGGL((woq_gemm_kernel<BITS, kActF32>), g, dim3(256), 0, st, a);
  else if (at == kActF16)
    hipLaunchKernelGGL((woq_gemm_kernel<BITS, kActF16>), g, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((woq_gemm_kernel<BITS, kActBF16>), g, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_gemm(const GemmArgs& a, int bits, int act_t, hipStream_t stream) {
  const int nbm = (a.M + 127) / 128, nbn = (a.w.ns + 7) / 8;
  dim3 grid(nbm * nbn);
  if (bits == 4) return gemm_dispatch_bits<4>(a, act_t, grid, stream);
  if (bits == 2) return gemm_dispatch_bits<2>(a, act_t, grid, stream);
  return gemm_dispatch_bits<8>(a, act_t, grid, stream);
}

}  // namespace nad

