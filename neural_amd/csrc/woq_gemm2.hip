// woq_gemm2.hip -- the prefill (M > 16) weight-only-quantized GEMM for gfx950, int4, groups of 128 * 2^j.
//
// Replaces LauncherBase::gemm / run_block + WeightKBlockNInteger::getFpWeight + the AMX / AVX512 GEMM cores
// (bestla/bestla/bestla_wrapper.h:481-542, bestla_prologue_b.h:732-838) for prefill-sized M.
//
// Structure (one workgroup per CU, 512 threads = 8 waves as 4 (M) x 2 (N), block tile 256 x 128, K step = one
// 128-deep int4 tile):
//   * A is fp16 [M][Kp] (a one-pass conversion of the fp32 / bf16 activations, nad_cvt_act_kernel, or the caller's
//     fp16 rows) and streams global -> LDS by LDS-DMA (global_load_lds_dwordx4) into a double buffer, one K step
//     ahead; the 16-B chunks of a 256-B row are XOR-swizzled by (row & 15) through the SOURCE address (the LDS image
//     of a DMA is lane-linear) so the MFMA fragment reads (16 rows x one chunk) are bank-conflict free;
//   * B needs no LDS: the tile layout (woq_layout.h) is already the v_mfma_f32_16x16x32_f16 B-fragment order, so each
//     wave loads its 4 stripes' 1 KiB tiles of the NEXT K step straight into registers (with their scales / zero
//     points) while it computes the current one, and dequantizes with the 0x6400 magic number into exact fp16
//     integers (q - zp);
//   * one fp32 group accumulator per output fragment is scaled into the result at every group end, so weights are
//     applied exactly as w = (q - zp) * s (fp32 scale multiply), the only rounding being A -> fp16 (as the reference's
//     own BF16/FP16 AMX cores round A);
//   * workgroups are remapped so that one XCD walks the N tiles of one M tile (the fp16 A rows, 8x the bytes of the
//     int4 B tiles per K step, are re-read from that XCD's L2).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "woq_device.h"
#include "woq_kernels.h"

namespace nad {
namespace g2 {

constexpr int BM = 256, BN = 128, KT = 128, ROWB = KT * 2;  // ROWB: bytes of one A row slice in LDS
constexpr int ABUF = BM * ROWB;                              // one A buffer: 64 KiB

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

// LDS-DMA of one K step of A: 256 rows x 256 B = 64 one-KiB pieces, 8 per wave; lane l of piece p fills LDS chunk
// (l & 15) of row 4p + (l >> 4) with source chunk (l & 15) ^ (row & 15).  Rows past M re-read row M-1 (their
// outputs are never stored).  The per-lane byte offsets are fixed for the whole K loop (aoff); each step only moves
// the uniform base.
__device__ __forceinline__ void stage_a(const char* base, const uint32_t (&aoff)[8], char* lbuf, int wave) {
#pragma unroll
  for (int i = 0; i < 8; i++)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + aoff[i]),
                                     (__attribute__((address_space(3))) void*)(lbuf + (wave * 8 + i) * 1024), 16, 0,
                                     0);
}

template <bool ASYM, bool TPG1>
__global__ __launch_bounds__(512, 1) void woq_gemm2_kernel(GemmArgs a, const _Float16* __restrict__ A16, int lda16) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int wm = wave >> 1, wn = wave & 1;
  const SkinnyWeight& W = a.w;
  const int M = a.M, nt = W.nt, ng = W.ng, ns = W.ns;
  const int tpg = W.bs / KT;  // tiles per group (power of two, host-checked)

  // XCD-aware remap: consecutive (remapped) ids share one XCD and walk the N tiles of ONE M tile, so the XCD's L2
  // holds that M tile's fp16 A rows (64 KiB per K step, read by every workgroup) while the int4 B tiles (8 KiB per K
  // step) stream from HBM / the Infinity Cache
  const int nbm = (M + BM - 1) / BM;
  const int nbn = (ns + 7) / 8;
  const int nwg = nbm * nbn;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8, o = bid / 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + o;
  }
  const int bm = bid / nbn, bn = bid % nbn;
  const int m0 = bm * BM;
  const int s0 = bn * 8 + wn * 4;  // this wave's first stripe
  const int nl = lane & 15;

  // per-stripe bases (clamped stripes past N read stripe ns-1: their columns are never stored)
  const u4_t* tl[4];
  int srow[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int s = min(s0 + j, ns - 1);
    tl[j] = reinterpret_cast<const u4_t*>(W.tiles) + size_t(s) * nt * 64 + lane;
    srow[j] = s * ng;
  }
  // branch-free scale fetch: the dword holding this lane's scale (f32, or a 16-bit pair), decoded at use.  A branch on
  // the scale type here made hipcc drain vmcnt(0) right after the next step's loads were issued.
  const int st = a.scale_t;
  const int ssh = st == kScaleF32 ? 0 : (nl & 1) * 16;
  const uint32_t* sbase = static_cast<const uint32_t*>(W.scales);
  auto load_b = [&](int t, u4_t (&b)[4], uint32_t (&sc)[4], int (&zp)[4]) {
    const int g = t / tpg;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      b[j] = __builtin_nontemporal_load(tl[j] + size_t(t) * 64);
      const size_t si = size_t(srow[j] + g) * 16 + nl;
      sc[j] = sbase[st == kScaleF32 ? si : (si >> 1)];
      zp[j] = ASYM ? int(W.zps[si]) : 0;
    }
  };
  auto scale_f32 = [&](uint32_t x) {
    const uint32_t h = (x >> ssh) & 0xFFFFu;
    const float fb = __uint_as_float(h << 16);
    const float fh = f16_bits_to_f32(uint16_t(h));
    const float f16or = st == kScaleBF16 ? fb : fh;
    return st == kScaleF32 ? __uint_as_float(x) : f16or;
  };
  // FOLD: this lane's two stripe scales of the current tile as fp16 pairs (fp16 scales: the stored bits, exact)
  h2_t fsc[2] = {g2::splat(1.f), g2::splat(1.f)};
  auto scale_h2 = [&](uint32_t x) {
    if (st == kScaleF16) {
      const uint32_t h = (x >> ssh) & 0xFFFFu;
      return as_h2(h | (h << 16));
    }
    return g2::splat(scale_f32(x));
  };

  f4_t acc[4][4], accg[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
      accg[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
    }

  u4_t bc[4], bx[4];
  uint32_t scc[4], scx[4];
  int zc[4], zx[4];
  uint32_t aoff[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int row = (wave * 8 + i) * 4 + (lane >> 4);
    const int grow = min(m0 + row, M - 1);
    aoff[i] = uint32_t(grow) * uint32_t(lda16) * 2u + uint32_t(((lane & 15) ^ (row & 15)) * 16);
  }
  const char* abase = reinterpret_cast<const char*>(A16);
  stage_a(abase, aoff, smem, wave);
  load_b(0, bc, scc, zc);
  __syncthreads();

  const uint32_t m0k = 0x000F000Fu, m1k = 0x00F000F0u, mag = 0x64006400u;
  const h2_t s16 = splat(1.f / 16.f);
  const h2_t zc0 = splat(-(1024.f + 8.f)), zc1 = splat(-(64.f + 8.f));
  // this lane's A fragment rows (i = 0..3) and their XOR key
  const int rbase = wm * 64 + nl;
  const int kq = lane >> 4;
  const f4_t zero = {0.f, 0.f, 0.f, 0.f};

  // one K step on the registers (b, sc, z) while the next step's A and B land in (bn, scn, zn)
  auto kstep = [&](int t, const u4_t (&b)[4], const uint32_t (&sc)[4], const int (&z)[4], u4_t (&bn)[4],
                   uint32_t (&scn)[4], int (&zn)[4]) {
    char* cur = smem + (t & 1) * ABUF;
    if (t + 1 < nt) {
      stage_a(abase + size_t(t + 1) * (KT * 2), aoff, smem + ((t + 1) & 1) * ABUF, wave);
      load_b(t + 1, bn, scn, zn);
    }
    const bool gstart = TPG1 || (t & (tpg - 1)) == 0;
    const bool gend = TPG1 || ((t + 1) & (tpg - 1)) == 0 || t == nt - 1;
#pragma unroll
    for (int d = 0; d < 4; d++) {
      h8_t bf[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if constexpr (ASYM) {
          const float zf = float(z[j]);
          bf[j] = dequant4(b[j][d], m0k, m1k, mag, s16, zc0 - splat(zf), zc1 - splat(zf));
        } else {
          bf[j] = dequant4(b[j][d], m0k, m1k, mag, s16, zc0, zc1);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int r = rbase + i * 16;
        const int ch = (d * 4 + kq) ^ (r & 15);
        const h8_t af = *reinterpret_cast<const h8_t*>(cur + r * ROWB + ch * 16);
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if (d == 0 && gstart)
            accg[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], zero, 0, 0, 0);
          else
            accg[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], accg[i][j], 0, 0, 0);
        }
      }
    }
    if (gend) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const float sf = scale_f32(sc[j]);
#pragma unroll
        for (int i = 0; i < 4; i++) acc[i][j] += accg[i][j] * sf;
      }
    }
    __syncthreads();  // next A buffer landed (vmcnt(0)), current buffer free for the step after
  };
  for (int t = 0; t < nt; t++) {
    kstep(t, bc, scc, zc, bx, scx, zx);
#pragma unroll
    for (int j = 0; j < 4; j++) {  // (unrolling by two to swap the sets instead measured slower: 256 VGPRs)
      bc[j] = bx[j];
      scc[j] = scx[j];
      zc[j] = zx[j];
    }
  }

  // epilogue: C fragment (i, j): row = m0 + wm*64 + i*16 + (lane>>4)*4 + rr, col = (s0+j)*16 + (lane&15)
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int n = (s0 + j) * 16 + nl;
    if (s0 + j >= ns || n >= W.n) continue;
#pragma unroll
    for (int i = 0; i < 4; i++) {
#pragma unroll
      for (int rr = 0; rr < 4; rr++) {
        const int row = m0 + wm * 64 + i * 16 + kq * 4 + rr;
        if (row >= M) continue;
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

// activations -> fp16 [M][Kp] (zero past K; act-order gather when shuffled): the A operand of woq_gemm2_kernel
template <int AT>
__global__ void nad_cvt_act_kernel(const void* A, int lda, int M, int K, int Kp, const int32_t* shuffle,
                                   _Float16* out) {
  const size_t total = size_t(M) * (Kp / 8);
  for (size_t u = blockIdx.x * size_t(blockDim.x) + threadIdx.x; u < total; u += size_t(gridDim.x) * blockDim.x) {
    const int row = int(u / (Kp / 8)), k0 = int(u % (Kp / 8)) * 8;
    float v[8];
    load_a8<AT>(A, lda, row, k0, K, shuffle, shuffle == nullptr && (reinterpret_cast<uintptr_t>(A) % 16 == 0) &&
                                                 ((size_t(lda) * (AT == kActF32 ? 4 : 2)) % 16 == 0), v);
    h8_t h;
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = _Float16(v[j]);
    *reinterpret_cast<h8_t*>(out + size_t(row) * Kp + k0) = h;
  }
}

}  // namespace g2

// ------------------------------------------------------------------------------------------------------------------
// gemm3: the same 256 x 128 block tile, pipelined across barriers.  In gemm2 the B tiles and scales are register loads
// beside the A LDS-DMA, so hipcc waits vmcnt(0) at their first use and at the __syncthreads: every K step exposes the
// full load latency (cdna_hip_programming.md §5 "Pipelining across barriers", trap (b)).  Here EVERY operand moves by
// LDS-DMA into one __shared__ array and each barrier waits with a counted vmcnt for the buffer the next half step reads
// only:
//   * K advances in 64-deep half steps; A (256 rows x 128 B, 32 pieces of 1 KiB, 4 per wave) is staged three half
//     steps ahead into a ring of four 32 KiB buffers;
//   * the K tile of B (8 stripes x 1 KiB, one piece per wave) and its scale / zero-point dwords (one 256 B piece each,
//     issued by every wave -- duplicate writes of identical bytes) go out with A on odd half steps into a ring of three;
//   * waves are 2 (M) x 4 (N), 128 x 32 per wave: each wave dequantizes 2 stripes (half of gemm2's per-wave VALU) and
//     reads 8 A fragments per 32-deep step;
//   * LDS image of a half step: row r = 128 B = 8 chunks of 16 B, chunk c holds A[r][8 (c ^ f(r)) .. + 7] with
//     f(r) = (r >> 1) & 7 (XOR through the DMA source address): a ds_read_b128 over 16 consecutive rows at one chunk
//     hits 16 distinct 16-B bank slots.
namespace g3 {

constexpr int BM = 256, KT = 128, ROWB = 128;        // ROWB: bytes of one A row per 64-deep half step
constexpr int HBUF = BM * ROWB;                       // one half step of A: 32 KiB
constexpr int NA = 4;                                 // A ring: three half steps in flight
constexpr int BTILES = 8 * 1024, BSC = 512, BZP = 512;
constexpr int BBUF = BTILES + BSC + BZP;              // one K tile of B: 8 stripe tiles + scale and zero-point dwords
constexpr int NBR = 3;                                // B ring
constexpr int LDS_BYTES = NA * HBUF + NBR * BBUF;     // 155 KiB

__device__ __forceinline__ void glds16(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 4, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS reads in inline asm: hipcc puts a vmcnt(0) in front of every LDS read it can see while an LDS-DMA is in flight
// (it cannot tell the buffers of one __shared__ array apart), which would drain the whole prefetch each half step.
// Results are consumed only after an explicit lgkmcnt wait that names them (wait_lgk below).
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
template <size_t... I>
__device__ __forceinline__ void lds_frags(h8_t (&f)[8], uint32_t addr, std::index_sequence<I...>) {
  ((f[I] = lds_b128<int(I) * 16 * ROWB>(addr)), ...);
}
template <class T>
__device__ __forceinline__ void tie(T& r) {
  asm volatile("" : "+v"(r));
}
template <int N, class... T>
__device__ __forceinline__ void wait_lgk(T&... regs) {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N));
  (tie(regs), ...);  // each result is redefined after the wait: no use can be scheduled above it
}
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return uint32_t(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p));
}

// FOLD: the group scale is multiplied into the fp16 B fragment (q * s rounded once to fp16, the host checked that every
// q * s of the weight is an fp16 normal, DeviceWeight::fold_ok) and the MFMAs accumulate straight into the result: no
// per-group fp32 accumulator, no group-end scaling (the reference itself dequantizes to bf16 for its AMX-BF16 core,
// bestla_prologue_b.h:732-838 getFpWeight)
template <bool ASYM, bool TPG1, bool FOLD>
__global__ __launch_bounds__(512, 1) void woq_gemm3_kernel(GemmArgs a, const _Float16* __restrict__ A16, int lda16) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int wm = wave >> 2, wn = wave & 3;
  const SkinnyWeight& W = a.w;
  const int M = a.M, nt = W.nt, ng = W.ng, ns = W.ns;
  const int tpg = W.bs / KT;
  const int tsh = __builtin_ctz(unsigned(tpg));

  // XCD-aware remap (as gemm2); with split-K the remapped id is (run, tile), so one XCD walks the N tiles of one
  // (M tile, K run) and its L2 holds that run's A rows
  const int nbm = (M + BM - 1) / BM;
  const int nbn = (ns + 7) / 8;
  const int ntile = nbm * nbn;
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;
  const int nwg = ntile * nsplit;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8, o = bid / 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + o;
  }
  const int ks = bid / ntile;
  bid -= ks * ntile;
  const int kt0 = nsplit > 1 ? ks * a.ktiles : 0;          // first K tile of this run (a multiple of tpg)
  const int ntl = nsplit > 1 ? min(a.ktiles, nt - kt0) : nt;
  const int nh = 2 * ntl;
  const int bm = bid / nbn, bn = bid % nbn;
  const int m0 = bm * BM;
  const int nl = lane & 15, kq = lane >> 4;

  // DMA sources of this lane.  A piece p = 4 wave + i: rows 8p .. 8p + 7, lane -> row 8p + (lane >> 3), chunk lane & 7
  uint32_t aoff[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int row = (wave * 4 + i) * 8 + (lane >> 3);
    const int grow = min(m0 + row, M - 1);  // rows past M re-read row M-1 (never stored)
    aoff[i] = uint32_t(grow) * uint32_t(lda16) * 2u + uint32_t(((lane & 7) ^ ((row >> 1) & 7)) * 16);
  }
  const char* abase = reinterpret_cast<const char*>(A16) + size_t(kt0) * KT * 2;
  // B: wave w copies stripe 8 bn + w (clamped: stripes past N are never stored); scale / zero-point piece w & 1 covers
  // stripes 8 bn + 4 (w & 1) + (lane >> 4), column lane & 15
  const char* btile =
      static_cast<const char*>(W.tiles) + (size_t(min(bn * 8 + wave, ns - 1)) * nt * 64 + lane) * 16 + size_t(kt0) * 1024;
  const int sstripe = min(bn * 8 + (wave & 1) * 4 + (lane >> 4), ns - 1);
  const size_t srow0 = size_t(sstripe) * ng * 16 + nl + size_t(kt0 >> tsh) * 16;
  const int st = a.scale_t;
  const uint32_t* sbase = static_cast<const uint32_t*>(W.scales);
  const uint32_t* zbase = reinterpret_cast<const uint32_t*>(W.zps);

  // batch(u): the DMAs issued at the start of half step u -- A(u + 3) and, on odd u, B tile (u + 3) / 2
  auto issue = [&](auto Hc, int u) {
    constexpr int H = decltype(Hc)::value;
    if (u + 3 >= nh) return;
    const int ua = u + 3;
    char* ab = smem + (ua & 3) * HBUF;
    const char* src = abase + size_t(ua) * ROWB;
#pragma unroll
    for (int i = 0; i < 4; i++) glds16(src + aoff[i], ab + (wave * 4 + i) * 1024);
    if constexpr (H == 1) {
      const int t = ua >> 1;
      char* bb = smem + NA * HBUF + (t % NBR) * BBUF;
      glds16(btile + size_t(t) * 1024, bb + wave * 1024);
      const size_t si = srow0 + size_t(t >> tsh) * 16;
      glds4(sbase + (st == kScaleF32 ? si : (si >> 1)), bb + BTILES + (wave & 1) * 256);
      if constexpr (ASYM) glds4(zbase + (si >> 2), bb + BTILES + BSC + (wave & 1) * 256);
    }
  };
  // VMEM instructions per odd batch besides the 4 A pieces
  constexpr int NBW = ASYM ? 3 : 2;

  f4_t acc[8][2], accg[8][2];
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) {
      acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
      accg[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
    }

  // prologue: batches -3, -2, -1 (A0 + B0, A1, A2 + B1); wait for batch -3
  issue(std::integral_constant<int, 1>{}, -3);
  issue(std::integral_constant<int, 0>{}, -2);
  issue(std::integral_constant<int, 1>{}, -1);
  if (nh > 2)
    wait_vm<8 + NBW>();
  else
    wait_vm<4>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const uint32_t m0k = 0x000F000Fu, m1k = 0x00F000F0u, mag = 0x64006400u;
  const h2_t s16 = g2::splat(1.f / 16.f);
  const h2_t zc0 = g2::splat(-(1024.f + 8.f)), zc1 = g2::splat(-(64.f + 8.f));
  // fragment reads: A row wm*128 + i*16 + nl, chunk (dd*4 + kq) ^ f(row); B / scale / zp of stripe wn*2 + j
  uint32_t roff[2];
#pragma unroll
  for (int dd = 0; dd < 2; dd++) roff[dd] = uint32_t((wm * 128 + nl) * ROWB + (((dd * 4 + kq) ^ ((nl >> 1) & 7)) * 16));
  const int boff = (wn * 2) * 1024 + lane * 16;
  const int soff = BTILES + ((wn * 2) * 16 + nl) * 4;
  const int zoff = BTILES + BSC + ((wn * 2) * 16 + nl) * 4;
  const int ssh = st == kScaleF32 ? 0 : (nl & 1) * 16;
  const int zsh = (nl & 3) * 8;
  const f4_t zero = {0.f, 0.f, 0.f, 0.f};
  auto scale_f32 = [&](uint32_t x) {
    const uint32_t h = (x >> ssh) & 0xFFFFu;
    const float fb = __uint_as_float(h << 16);
    const float fh = f16_bits_to_f32(uint16_t(h));
    const float f16or = st == kScaleBF16 ? fb : fh;
    return st == kScaleF32 ? __uint_as_float(x) : f16or;
  };
  // FOLD: this lane's two stripe scales of the current tile as fp16 pairs (fp16 scales: the stored bits, exact)
  h2_t fsc[2] = {g2::splat(1.f), g2::splat(1.f)};
  auto scale_h2 = [&](uint32_t x) {
    if (st == kScaleF16) {
      const uint32_t h = (x >> ssh) & 0xFFFFu;
      return as_h2(h | (h << 16));
    }
    return g2::splat(scale_f32(x));
  };

  // hand-over: batch(u - 2) (the buffers half step u + 1 reads) has landed for this wave; batches u - 1 and u
  // (8 A pieces + one B batch, whatever the order inside a batch) stay in flight across the barrier
  auto hand_over = [&](auto Hc, int u) {
    constexpr int H = decltype(Hc)::value;
    if constexpr (H == 0) {
      if (u + 3 < nh)
        wait_vm<8 + NBW>();
      else
        wait_vm<0>();
    } else {
      if (u + 3 < nh)
        wait_vm<8 + NBW>();
      else if (u + 3 == nh)
        wait_vm<4>();
      else
        wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // L (late, waves 4-7 when staggered): the barrier of half step u comes after its first 32-deep step, so these waves'
  // second-step MFMAs and group scaling run half a block behind waves 0-3 (MI355X_MICROARCH item 9).  Everything they
  // read from LDS for half step u (A fragments, B words, scales) is in registers before that barrier.
  auto half = [&](auto Hc, auto Lc, int u) {
    constexpr int H = decltype(Hc)::value;  // which 64 of the B tile's 128
    constexpr bool L = decltype(Lc)::value;
    const int t = u >> 1;
    const char* ab = smem + (u & 3) * HBUF;
    const char* bb = smem + NA * HBUF + (t % NBR) * BBUF;
    issue(Hc, u);
    const uint32_t al = lds_addr(ab), bl = lds_addr(bb);
    uint2 bv0 = lds_b64<H * 8>(bl + boff), bv1 = lds_b64<1024 + H * 8>(bl + boff);
    uint32_t zw0 = 0, zw1 = 0;
    if constexpr (ASYM) {
      zw0 = lds_b32<0>(bl + zoff);
      zw1 = lds_b32<64>(bl + zoff);
    }
    uint32_t fw0 = 0, fw1 = 0;
    if constexpr (FOLD && H == 0) {  // every tile carries its group's scale piece
      fw0 = lds_b32<0>(bl + soff);
      fw1 = lds_b32<64>(bl + soff);
    }
    h8_t af0[8], af1[8];
    lds_frags(af0, al + roff[0], std::make_index_sequence<8>{});
    lds_frags(af1, al + roff[1], std::make_index_sequence<8>{});
    wait_lgk<8>(bv0, bv1, zw0, zw1, fw0, fw1, af0[0], af0[1], af0[2], af0[3], af0[4], af0[5], af0[6], af0[7]);
    if constexpr (FOLD && H == 0) {
      fsc[0] = scale_h2(fw0);
      fsc[1] = scale_h2(fw1);
    }
    const uint32_t bw[2][2] = {{bv0.x, bv0.y}, {bv1.x, bv1.y}};
    int zp[2] = {0, 0};
    if constexpr (ASYM) {
      zp[0] = int(int8_t((zw0 >> zsh) & 0xFFu));
      zp[1] = int(int8_t((zw1 >> zsh) & 0xFFu));
    }
    const bool gstart = H == 0 && (TPG1 || (t & (tpg - 1)) == 0);
    const bool gend = H == 1 && (TPG1 || ((t + 1) & (tpg - 1)) == 0 || t == ntl - 1);
    uint32_t sw0 = 0, sw1 = 0;
#pragma unroll
    for (int dd = 0; dd < 2; dd++) {
      if (dd == 1) {
        wait_lgk<0>(af1[0], af1[1], af1[2], af1[3], af1[4], af1[5], af1[6], af1[7]);
        if constexpr (L) {
          if (!FOLD && gend) {
            sw0 = lds_b32<0>(bl + soff);
            sw1 = lds_b32<64>(bl + soff);
            wait_lgk<0>(sw0, sw1);
          }
          hand_over(Hc, u);
        }
      }
      h8_t bf[2];
#pragma unroll
      for (int j = 0; j < 2; j++) {
        if constexpr (ASYM) {
          const float zf = float(zp[j]);
          bf[j] = g2::dequant4(bw[j][dd], m0k, m1k, mag, s16, zc0 - g2::splat(zf), zc1 - g2::splat(zf));
        } else {
          bf[j] = g2::dequant4(bw[j][dd], m0k, m1k, mag, s16, zc0, zc1);
        }
        if constexpr (FOLD) {
          const h8_t s8 = {fsc[j][0], fsc[j][0], fsc[j][0], fsc[j][0], fsc[j][0], fsc[j][0], fsc[j][0], fsc[j][0]};
          bf[j] = bf[j] * s8;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const h8_t af = dd == 0 ? af0[i] : af1[i];
#pragma unroll
        for (int j = 0; j < 2; j++) {
          if constexpr (FOLD)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], acc[i][j], 0, 0, 0);
          else if (dd == 0 && gstart)
            accg[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], zero, 0, 0, 0);
          else
            accg[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], accg[i][j], 0, 0, 0);
        }
      }
    }
    if (!FOLD && gend) {
      if constexpr (!L) {
        sw0 = lds_b32<0>(bl + soff);
        sw1 = lds_b32<64>(bl + soff);
        wait_lgk<0>(sw0, sw1);
      }
      const float sf[2] = {scale_f32(sw0), scale_f32(sw1)};
#pragma unroll
      for (int j = 0; j < 2; j++)
#pragma unroll
        for (int i = 0; i < 8; i++) acc[i][j] += accg[i][j] * sf[j];
    }
    if constexpr (!L) hand_over(Hc, u);
  };

  if (a.stagger && wave >= 4) {
    for (int u = 0; u < nh; u += 2) {
      half(std::integral_constant<int, 0>{}, std::true_type{}, u);
      half(std::integral_constant<int, 1>{}, std::true_type{}, u + 1);
    }
  } else {
    for (int u = 0; u < nh; u += 2) {
      half(std::integral_constant<int, 0>{}, std::false_type{}, u);
      half(std::integral_constant<int, 1>{}, std::false_type{}, u + 1);
    }
  }

  // epilogue through LDS (free after the loop: the last barrier retired every read and DMA): each wave transposes its
  // 128 x 32 fp32 tile into row-major LDS rows (stride 36 floats), then writes whole 16-B row chunks -- the C fragment
  // (4 rows of one column per lane) would otherwise leave as 64 scattered dword stores per lane, an issue-bound tail
  // that all workgroups reach at once.
  float* tw = reinterpret_cast<float*>(smem) + wave * (128 * 36);
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
      for (int rr = 0; rr < 4; rr++) tw[(i * 16 + kq * 4 + rr) * 36 + j * 16 + nl] = acc[i][j][rr];
  const int s0 = bn * 8 + wn * 2;
  const int col0 = s0 * 16;
#pragma unroll 4
  for (int q = 0; q < 16; q++) {
    const int c = q * 64 + lane;
    const int rl = c >> 3, c4 = c & 7;
    const int row = m0 + wm * 128 + rl;
    const int n0 = col0 + c4 * 4;
    const float4 t = *reinterpret_cast<const float4*>(tw + rl * 36 + c4 * 4);
    if (row >= M || n0 >= W.n) continue;
    if (nsplit > 1) {  // raw partial of this K run (ldp % 4 == 0, 16-B aligned rows): the reduce applies the epilogue
      *reinterpret_cast<float4*>(a.part + (size_t(ks) * M + row) * a.ldp + n0) = t;
      continue;
    }
    float v[4] = {t.x, t.y, t.z, t.w};
    gemm_epilogue4(a, row, n0, v);
  }
}

}  // namespace g3

// ------------------------------------------------------------------------------------------------------------------
// split-K reduce: out[row][n] = epi(sum over runs r = 0 .. S-1, in order, of part[r][row][n]); 4 columns per thread
__global__ __launch_bounds__(256) void nad_splitk_reduce_kernel(GemmArgs a) {
  const SkinnyWeight& W = a.w;
  const int nq = (W.n + 3) >> 2;
  int row, n0;
  if (a.xcd_sg) {
    // the mid-M kernel's stripe groups (4 xcd_w columns): group sg's slabs were written on XCD sg % 8, read them there
    // (the last incomplete round of 8 groups in order, as the mid-M kernel places them)
    const int xw = a.xcd_w, per = (a.M * xw + 255) >> 8, x8 = (a.xcd_sg >> 3) << 3, full = x8 * per, b = int(blockIdx.x);
    int sg, u;
    if (b < full) {
      sg = ((b >> 3) / per) * 8 + (b & 7);
      u = ((b >> 3) % per) * 256 + int(threadIdx.x);
    } else {
      sg = x8 + (b - full) / per;
      u = ((b - full) % per) * 256 + int(threadIdx.x);
    }
    row = u / xw;
    n0 = (sg * xw + (u - row * xw)) * 4;
    if (row >= a.M || n0 >= W.n) return;
  } else if (a.xcd_tile) {
    // gemm7's tiles (xcd_tile rows x 128 columns): XCD x summed tiles [x T/8, (x+1) T/8), 8 rows per workgroup
    const int bmt = a.xcd_tile, per = bmt >> 3, nbn = (W.ns + 7) >> 3, ntile = ((a.M + bmt - 1) / bmt) * nbn;
    const int b = int(blockIdx.x), o = b >> 3, tile = (b & 7) * (ntile >> 3) + o / per;
    row = (tile / nbn) * bmt + (o % per) * 8 + int(threadIdx.x >> 5);
    n0 = (tile % nbn) * 128 + int(threadIdx.x & 31) * 4;
    if (row >= a.M || n0 >= W.n) return;
  } else {
    const size_t q = size_t(blockIdx.x) * 256 + threadIdx.x;
    if (q >= size_t(a.M) * nq) return;
    row = int(q / nq);
    n0 = int(q - size_t(row) * nq) * 4;
  }
  const size_t rs = size_t(a.M) * a.ldp;
  const float* p = a.part + size_t(row) * a.ldp + n0;
  // the loads of up to 8 runs in flight at once (a loop over the runs serialised their latencies: 4.7 us for 1 MB)
  float4 t[8];
#pragma unroll
  for (int r = 0; r < 8; r++)
    if (r < a.ksplit) t[r] = *reinterpret_cast<const float4*>(p + r * rs);
  float4 s = t[0];
#pragma unroll
  for (int r = 1; r < 8; r++) {
    if (r >= a.ksplit) break;
    s.x += t[r].x;
    s.y += t[r].y;
    s.z += t[r].z;
    s.w += t[r].w;
  }
  for (int r = 8; r < a.ksplit; r++) {
    const float4 u = *reinterpret_cast<const float4*>(p + r * rs);
    s.x += u.x;
    s.y += u.y;
    s.z += u.z;
    s.w += u.w;
  }
  float v[4] = {s.x, s.y, s.z, s.w};
  gemm_epilogue4(a, row, n0, v);
}

hipError_t launch_splitk_reduce(const GemmArgs& a, hipStream_t st) {
  const size_t work = a.xcd_sg     ? size_t(a.xcd_sg) * ((a.M * a.xcd_w + 255) / 256) * 256
                      : a.xcd_tile ? size_t((a.M + a.xcd_tile - 1) / a.xcd_tile) * ((a.w.ns + 7) / 8) * a.xcd_tile * 32
                                   : size_t(a.M) * ((a.w.n + 3) / 4);
  hipLaunchKernelGGL(nad_splitk_reduce_kernel, dim3(unsigned((work + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_gemm3(const GemmArgs& a, const _Float16* A16, int lda16, hipStream_t st) {
  const int nbm = (a.M + g3::BM - 1) / g3::BM, nbn = (a.w.ns + 7) / 8;
  const bool tpg1 = a.w.bs == g3::KT;
  auto go = [&](auto k) -> hipError_t {
    static bool attr[2][2][2] = {};  // opt in to 155 KiB of dynamic LDS once per instantiation
    bool& done = attr[a.w.zps != nullptr][a.w.bs == g3::KT][a.fold ? 1 : 0];
    if (!done) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         g3::LDS_BYTES);
      if (e != hipSuccess) return e;
      done = true;
    }
    hipLaunchKernelGGL(k, dim3(nbm * nbn * (a.ksplit > 1 ? a.ksplit : 1)), dim3(512), g3::LDS_BYTES, st, a, A16, lda16);
    return hipGetLastError();
  };
  const bool asym = a.w.zps != nullptr;
  if (a.fold) {
    if (asym) return tpg1 ? go(g3::woq_gemm3_kernel<true, true, true>) : go(g3::woq_gemm3_kernel<true, false, true>);
    return tpg1 ? go(g3::woq_gemm3_kernel<false, true, true>) : go(g3::woq_gemm3_kernel<false, false, true>);
  }
  if (asym) return tpg1 ? go(g3::woq_gemm3_kernel<true, true, false>) : go(g3::woq_gemm3_kernel<true, false, false>);
  return tpg1 ? go(g3::woq_gemm3_kernel<false, true, false>) : go(g3::woq_gemm3_kernel<false, false, false>);
}

hipError_t launch_cvt_act(const void* A, int act_t, int lda, int M, int K, int Kp, const int32_t* shuffle,
                          _Float16* out, hipStream_t st) {
  const size_t units = size_t(M) * (Kp / 8);
  const int blocks = int(std::min<size_t>((units + 255) / 256, 4096));
  if (act_t == kActF32)
    hipLaunchKernelGGL(g2::nad_cvt_act_kernel<kActF32>, dim3(blocks), dim3(256), 0, st, A, lda, M, K, Kp, shuffle,
                       out);
  else if (act_t == kActF16)
    hipLaunchKernelGGL(g2::nad_cvt_act_kernel<kActF16>, dim3(blocks), dim3(256), 0, st, A, lda, M, K, Kp, shuffle,
                       out);
  else
    hipLaunchKernelGGL(g2::nad_cvt_act_kernel<kActBF16>, dim3(blocks), dim3(256), 0, st, A, lda, M, K, Kp, shuffle,
                       out);
  return hipGetLastError();
}

hipError_t launch_gemm2(const GemmArgs& a, const _Float16* A16, int lda16, hipStream_t st) {
  const int nbm = (a.M + g2::BM - 1) / g2::BM, nbn = (a.w.ns + 7) / 8;
  const size_t lds = 2 * size_t(g2::ABUF);
  const bool tpg1 = a.w.bs == g2::KT;
  auto go = [&](auto k) -> hipError_t {
    static bool attr = false;  // per instantiation (distinct lambda argument types)
    (void)attr;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       int(lds));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(nbm * nbn), dim3(512), lds, st, a, A16, lda16);
    return hipGetLastError();
  };
  const bool asym = a.w.zps != nullptr;
  if (asym) return tpg1 ? go(g2::woq_gemm2_kernel<true, true>) : go(g2::woq_gemm2_kernel<true, false>);
  return tpg1 ? go(g2::woq_gemm2_kernel<false, true>) : go(g2::woq_gemm2_kernel<false, false>);
}

}  // namespace nad
