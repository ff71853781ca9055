// woq_gemm7.hip -- the default prefill (M > 16) int4 WOQ GEMM for gfx950: groups of 128 * 2^j, the group scale folded
// into the fp16 B operand.
//
// Replaces LauncherBase::gemm / run_block + WeightKBlockNInteger::getFpWeight + the AMX / AVX512 GEMM cores
// (bestla/bestla/bestla_wrapper.h:481-542, bestla_prologue_b.h:732-838) for prefill-sized M.  q * s is rounded once to
// fp16, as the reference's own AMX-BF16 / FP16 cores dequantize to a 16-bit float (DeviceWeight::fold_ok range-checks
// every q * s at load; an unfoldable weight stays on gemm3, woq_gemm2.hip, which applies the scale exactly in fp32).
//
// Why it replaced gemm3 (profiles/r05_*): gemm3 runs 8 waves as 2 (M) x 4 (N) on a 256 x 128 tile, so
// every B fragment is dequantized by both M-waves and each wave scales 64 group accumulators per group (2.65 non-MFMA
// VALU per v_mfma_f32_16x16x32_f16).  gemm7 keeps the tile and gemm3's LDS-DMA plan (A three 64-deep half steps ahead
// in a ring of four 32 KiB slots, the K tile of B + scale / zero-point dwords in a ring of three) but splits the waves
// over K: wave (wn, wk) owns the 256 x 32 partial of stripes 2 wn, 2 wn + 1 over the 32-deep step wk of every half
// step, so each B fragment is dequantized once per workgroup (1.44 VALU per MFMA measured incl. addressing) and the two
// K halves meet once, in the epilogue.  DMAs are raw buffer loads with per-lane offsets fixed for the whole loop (no
// 64-bit address arithmetic per piece); the MFMA accumulators live in VGPRs (-amdgpu-mfma-vgpr-form in the Makefile:
// left to its heuristics hipcc split them over both register files and copied them every half step).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "woq_device.h"
#include "woq_kernels.h"

namespace nad {
namespace g7 {

constexpr int KT = 128, ROWB = 128;  // ROWB: bytes of one A row per 64-deep half step
constexpr int NS = 8;                // stripes per tile (128 columns)
constexpr int EPI_LD = 36;           // epilogue transpose row stride (floats)

// One B buffer with its scale and zero-point bytes as they lie in HBM ([stripe][group][16 columns]), each region at least
// one 256-byte LDS-DMA piece.  int4 (tile mode): a whole 128-deep K tile, GPT groups per tile (4 at groups of 32, 2 at
// 64, 1 from 128 up).  int2 / int8 (half-step mode, HS): the slice of the 8 stripes one 64-deep half step reads -- a
// dword of every lane of a 256-deep int2 tile, a whole 64-deep int8 tile -- loaded every half step, so each half step
// issues the same loads and the vmcnt arithmetic stays exact; GPT groups per half step (2 at groups of 32, else 1).
template <int BITS, int GPT, int ST, bool ASYM>
struct Bbuf {
  static constexpr bool HS = BITS != 4;
  static constexpr int ESZ = ST == kScaleF32 ? 4 : 2;
  static constexpr int BSL = BITS == 4 ? 1024 : (BITS == 8 ? 1024 : 256);  // bytes per stripe per buffer
  static constexpr int SCT = NS * GPT * 16 * ESZ, ZPT = NS * GPT * 16;      // bytes a buffer uses
  static constexpr int SCR = SCT > 256 ? SCT : 256, ZPR = ASYM ? (ZPT > 256 ? ZPT : 256) : 0;
  static constexpr int BW = NS * BSL;
  static constexpr int BYTES = BW + SCR + ZPR;
};

// Geometry per tile height BMT (32, 64, 128, 256 rows; every wave covers all of them): the A ring runs DA = NA - 1 half
// steps ahead -- deeper for the short tiles, whose K runs are split-K runs of a few tiles.  Tile mode: the B ring holds
// a tile no shorter than the two half steps after its last read.  Half-step mode: B runs DB half steps ahead (DA, or 2
// where DA + 1 int8 slices would not fit beside the A ring) in a ring of DB + 1 slices.
template <int BMT, class BB>
struct Geo {
  static constexpr int RF = BMT / 16;                  // row fragments per wave
  static constexpr int HF = RF / 2;                    // fragments per half of the register rotation
  static constexpr int HBUF = BMT * ROWB;              // one half step of A
  static constexpr int PIECES = HBUF / 1024;           // A pieces per half step
  static constexpr int PA = PIECES >= 8 ? PIECES / 8 : 1;  // per wave (BMT = 32: waves 4-7 repeat pieces 0-3)
  static constexpr int NA = BMT == 256 ? 4 : (BMT == 128 ? 6 : 8);
  static constexpr int DA = NA - 1;
  static constexpr int DB = !BB::HS ? DA : (NA * HBUF + (DA + 1) * BB::BYTES <= 160 * 1024 ? DA : 2);
  static constexpr int NBR = BB::HS ? DB + 1 : (DA + 3) / 2;
  static constexpr int LDS_RING = NA * HBUF + NBR * BB::BYTES;
  static constexpr int LDS_EPI = 8 * (BMT / 2) * EPI_LD * 4;
  static constexpr int LDS = LDS_RING > LDS_EPI ? LDS_RING : LDS_EPI;
  static_assert(LDS <= 160 * 1024 && DA % 2 == 1, "geometry");
};

// LDS-DMA as raw buffer loads: 32-bit per-lane offsets fixed for the whole K loop, the moving part in an SGPR
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, -1, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, char* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ void blds4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, char* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 4, voff, soff, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// LDS reads in inline asm (hipcc would put vmcnt(0) in front of every LDS read it sees while an LDS-DMA is in flight);
// results are consumed only after an explicit lgkmcnt wait that names them
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
template <int N, class... T>
__device__ __forceinline__ void wait_lgk(T&... regs) {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N));
  (tie(regs), ...);
}
template <int B, size_t... I>
__device__ __forceinline__ void read_frags(h8_t* f, uint32_t addr, std::index_sequence<I...>) {
  ((f[B + I] = lds_b128<int(B + I) * 16 * ROWB>(addr)), ...);
}
template <int B, size_t... I>
__device__ __forceinline__ void tie_frags(h8_t* f, std::index_sequence<I...>) {
  (tie(f[B + I]), ...);
}
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return uint32_t(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p));
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
// one 32-deep step's B fragment: 8 nibbles -> fp16 (q - 8 - zp) * s, the product rounded once
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

// int8: a dword pair (8 bytes q + 128) -> fp16 (q - zp) * s: byte b becomes 1024 + b by a byte permute, c = -(1152 + zp)
__device__ __forceinline__ h8_t dequant8_fold(uint32_t w0, uint32_t w1, h2_t c, h2_t sc) {
  const h2_t p0 = (as_h2(__builtin_amdgcn_perm(0x64646464u, w0, 0x04010400u)) + c) * sc;
  const h2_t p1 = (as_h2(__builtin_amdgcn_perm(0x64646464u, w0, 0x04030402u)) + c) * sc;
  const h2_t p2 = (as_h2(__builtin_amdgcn_perm(0x64646464u, w1, 0x04010400u)) + c) * sc;
  const h2_t p3 = (as_h2(__builtin_amdgcn_perm(0x64646464u, w1, 0x04030402u)) + c) * sc;
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
// int2: one 32-deep step (the low 8 bits of each 16-bit half of x) -> fp16 (q - 2 - zp) * s: the exact integers of the
// scaled magic numbers (dequant2s), then one rounding
__device__ __forceinline__ h8_t dequant2_fold(uint32_t x, const Dq2c& q, h2_t sc) {
  const h8_t v = dequant2s(x, q);
  h8_t r;
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    h2_t p;
    p[0] = v[i];
    p[1] = v[i + 1];
    p = p * sc;
    r[i] = p[0];
    r[i + 1] = p[1];
  }
  return r;
}

#define NAD_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

// 8 waves (two per SIMD) split over K: wave (wn = w & 3, wk = w >> 2) owns the BMT x 32 partial of stripes 2 wn,
// 2 wn + 1 over the 32-deep step wk of every 64-deep half step.  Its RF A fragments per half step rotate in two halves
// around the half step's barrier: fragments 0 .. HF - 1 of half step u + 1 are read into the registers the same
// fragments of u just left (their MFMAs done, barrier of u + 1 passed), the rest after the other MFMAs.  Batches past
// the end of the K run load from a zero-record buffer, so every half step issues and waits the same counts.  A 4-wave
// form (one wave per SIMD owning both K steps) measured 5-15 % slower than gemm3 (profiles/r05_gemm6_vs_gemm3_sweep.txt);
// wider-N tiles (128 x 256, 128 x 512, 256 x 256: 8 waves as 1 or 2 (M) x 8 or 4 (N), each B fragment dequantized by
// every M-wave) 3-35 % slower than this one (profiles/r05_gemm8_tile_shapes_sweep.txt).  BMT < 256 serves 17 <= M <= 256
// with split-K runs (the mid-M range): the tile's rows are what the problem has, not 256 rows of which most re-read the
// last one.
// MW: several weights in one launch (fused QKV prefill, GemmArgs::nwt; int4 groups of 128 * 2^j, whole K) -- a
// separate instantiation, so the single-weight kernel keeps its code (the runtime selection in it cost 2-4 %,
// profiles/r06_gemm7_fused_qkv_ab.txt)
template <int BITS, int BMT, bool ASYM, int ST, int GPT, bool MW = false>
__global__ __launch_bounds__(512, 1) void woq_gemm7_kernel(GemmArgs a, const _Float16* __restrict__ A16, int lda16) {
  using BB = Bbuf<BITS, GPT, ST, ASYM>;
  using G = Geo<BMT, BB>;
  constexpr int RF = G::RF, HF = G::HF, HBUF = G::HBUF, PA = G::PA, NA = G::NA, DA = G::DA, DB = G::DB, NBR = G::NBR;
  constexpr int BBUF = BB::BYTES, BSC = BB::SCR, ESZ = BB::ESZ, BW = BB::BW;
  constexpr bool HS = BB::HS;
  constexpr int TK = BITS == 4 ? 128 : (BITS == 2 ? 256 : 64), HPT = TK / 64;  // K tile depth, half steps per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int wn = wave & 3, wk = wave >> 2;
  const int M = a.M, nt = a.w.nt, ng = a.w.ng;  // the K side: shared by fused weights
  // tile mode: K tiles per group (2^tsh); half-step mode: half steps per group (2^tsh, groups of 64 up)
  const int tpg = HS ? (a.w.bs >= 64 ? a.w.bs / 64 : 1) : (a.w.bs >= KT ? a.w.bs / KT : 1);
  const int tsh = __builtin_ctz(unsigned(tpg));

  // XCD-aware remap (one XCD walks the N tiles of one (M tile, K run)) and split-K runs, as gemm3
  const int nbm = (M + BMT - 1) / BMT;
  const int nbn = MW ? a.nbn_all : (a.w.ns + NS - 1) / NS;
  const int ntile = nbm * nbn;
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;
  const int nwg = ntile * nsplit;
  int bid = blockIdx.x, ks;
  if (a.xcd_tile) {  // every run of a tile on one XCD: the reduce reads the slabs from that XCD's L2
    const int o = bid >> 3;
    ks = o % nsplit;
    bid = (bid & 7) * (ntile >> 3) + o / nsplit;
  } else {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8, o = bid / 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + o;
    ks = bid / ntile;
    bid -= ks * ntile;
  }
  const int kt0 = nsplit > 1 ? ks * a.ktiles : 0;
  const int ntl = nsplit > 1 ? min(a.ktiles, nt - kt0) : nt;
  const int nh = HPT * ntl;            // half steps of the K run
  const int nh2 = (nh + 1) & ~1;       // the loop's (int8: an odd count ends with one all-zero half step)
  const int bm = bid / nbn;
  // fused weights: column tile of the concatenation -> (weight, its own column tile)
  const int wi = MW ? int(bid % nbn >= a.nbn_cut[0]) + int(bid % nbn >= a.nbn_cut[1]) : 0;
  const int bn = bid % nbn - (MW && wi != 0 ? a.nbn_cut[wi - 1] : 0);
  const SkinnyWeight& W = MW && wi != 0 ? a.wf[wi - 1] : a.w;
  const int ns = W.ns;
  const int m0 = bm * BMT;
  const int nl = lane & 15, kq = lane >> 4;

  // A piece p: rows 8p .. 8p + 7, lane -> row 8p + (lane >> 3), chunk (lane & 7) ^ ((row >> 1) & 7)
  uint32_t aoff[PA];
  char* adst[PA];
#pragma unroll
  for (int i = 0; i < PA; i++) {
    const int p = (wave * PA + i) % G::PIECES;
    const int row = p * 8 + (lane >> 3);
    const int grow = min(m0 + row, M - 1);  // rows past M re-read row M - 1 (never stored)
    aoff[i] = uint32_t(grow) * uint32_t(lda16) * 2u + uint32_t(((lane & 7) ^ ((row >> 1) & 7)) * 16);
    adst[i] = smem + p * 1024;
  }
  const auto ra = brsrc(reinterpret_cast<const char*>(A16) + size_t(kt0) * TK * 2);
  const auto rb = brsrc(static_cast<const char*>(W.tiles) + size_t(kt0) * 1024);
  const auto rnull = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(W.tiles), 0, 0, 0x00020000);
  const uint32_t boffd = (uint32_t(min(bn * NS + wave, ns - 1)) * nt * 64 + lane) * 16;
  // scale / zero-point pieces: wave w copies 256-byte piece w % pieces of the tile's region; lane bytes past the tile's
  // share (a region rounded up to one piece) re-read its start into the unused tail
  constexpr int st = ST;
  // scales / zero points: a lane whose group lies past the last one (the zero-padded K tail of the last tile or half
  // step) gets an offset past the resource's end, which loads 0 without touching memory
  constexpr uint32_t kOOB = 0x7FFF0000u;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(W.scales), 0, int(kOOB), 0x00020000);
  const auto rz = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(static_cast<const void*>(W.zps)), 0, int(kOOB),
                                                    0x00020000);
  // first group of B buffer v of the K run (a tile, or a half step)
  auto group_of = [&](int v) -> uint32_t {
    const uint32_t x = HS ? uint32_t(kt0 * HPT + v) : uint32_t(kt0 + v);
    return GPT > 1 ? x * GPT : x >> tsh;
  };
  auto piece_off = [&](int pieces, int total, int esz, int* dst, int* gi) {
    const int p = wave % pieces;
    *dst = p * 256;
    const int o = (p * 256 + lane * 4) % total, chunk = GPT * 16 * esz;
    const int s = min(bn * NS + o / chunk, ns - 1);
    *gi = (o % chunk) / (16 * esz);  // the lane's group within the buffer
    return uint32_t(s) * ng * 16 * esz + uint32_t(o % chunk);
  };
  int sdst = 0, zdst = 0, sgi = 0, zgi = 0;
  const uint32_t svo = piece_off(BB::SCR / 256, BB::SCT, ESZ, &sdst, &sgi);
  const uint32_t zvo = ASYM ? piece_off(BB::ZPR / 256, BB::ZPT, 1, &zdst, &zgi) : 0u;
  // the scale / zero-point pieces of buffer v (first group g)
  auto load_sz = [&](bool live, uint32_t g, char* dst) {
    const uint32_t vs = g + uint32_t(sgi) < uint32_t(ng) ? svo + g * 16 * ESZ : kOOB;
    blds4(live ? rs : rnull, vs, 0, dst + sdst);
    if constexpr (ASYM) {
      const uint32_t vz = g + uint32_t(zgi) < uint32_t(ng) ? zvo + g * 16 : kOOB;
      blds4(live ? rz : rnull, vz, 0, dst + BSC + zdst);
    }
  };

  // batch(u): A(u + DA) and -- tile mode -- when u + DA is even, B tile (u + DA) / 2 with its scale / zero-point
  // pieces; half-step mode: the B slice of half step u + DB (none in the prologue batches before it starts)
  auto issue = [&](int u) {
    const int ua = u + DA;
    const bool live = ua < nh;
    const int aslot = ua % NA;
    const auto rA = live ? ra : rnull;
#pragma unroll
    for (int i = 0; i < PA; i++) blds16(rA, aoff[i], uint32_t(ua) * ROWB, adst[i] + aslot * HBUF);
    if constexpr (HS) {
      const int ub = u + DB;
      if (ub >= 0) {
        const bool lb = ub < nh;
        char* bb = smem + NA * HBUF + (ub % NBR) * BBUF;
        if constexpr (BITS == 8)
          blds16(lb ? rb : rnull, boffd, uint32_t(ub) * 1024, bb + wave * 1024);
        else  // dword ub & 3 of every lane of int2 tile ub >> 2
          blds4(lb ? rb : rnull, boffd, uint32_t(ub >> 2) * 1024 + uint32_t(ub & 3) * 4, bb + wave * 256);
        load_sz(lb, group_of(ub), bb + BW);
      }
    } else if ((ua & 1) == 0) {
      const int t = ua >> 1;
      char* bb = smem + NA * HBUF + (t % NBR) * BBUF;
      blds16(live ? rb : rnull, boffd, uint32_t(t) * 1024, bb + wave * 1024);
      load_sz(live, group_of(t), bb + BW);
    }
  };
  // at the barrier of buffer u + 1 (the middle of half step u), batch(u + 1 - DA) has landed and batches
  // u + 2 - DA .. u (DA - 1 of them, (DA - 1) / 2 with a B tile) may be in flight; half-step mode: B(u + 1) came with
  // batch(u + 1 - DB), after which DB - 1 whole batches may be in flight
  constexpr int NB = ASYM ? 3 : 2;
  constexpr int WV = HS ? (DB - 1) * (PA + NB) : (DA - 1) * PA + (DA - 1) / 2 * NB;
  static_assert(WV < 64, "vmcnt");

  const uint32_t mag = 0x64006400u;
  const h2_t s16 = splat(1.f / 16.f);
  const h2_t zc0 = splat(-(1024.f + 8.f)), zc1 = splat(-(64.f + 8.f));
  const h2_t zc8 = splat(-(1024.f + 128.f));
  const uint32_t roff = uint32_t(nl * ROWB + (((wk * 4 + kq) ^ ((nl >> 1) & 7)) * 16));
  // this lane's B bytes of stripe 2 wn (+ 1 KiB / 256 B for 2 wn + 1) for its 32-deep step: int4 dword 2 H + wk of the
  // tile, int8 the dword pair wk, int2 the half step's dword (its 16-bit half wk)
  const int boff = BITS == 4 ? (wn * 2) * 1024 + lane * 16 + wk * 4
                             : (BITS == 8 ? (wn * 2) * 1024 + lane * 16 + wk * 8 : (wn * 2) * 256 + lane * 4);
  constexpr int BJ = BITS == 2 ? 256 : 1024;
  // this lane's scale / zero-point dword for stripe 2 wn (+ SJ for 2 wn + 1) at its first 32-deep step of the tile; the
  // step's group moves it by SH per half step
  const int gw = (HS ? GPT == 2 : GPT == 4) ? wk : 0;
  const int soff = BW + ((((wn * 2) * GPT + gw) * 16 + nl) * ESZ & ~3);
  const int zoff = BW + BSC + ((((wn * 2) * GPT + gw) * 16 + nl) & ~3);
  constexpr int SJ = GPT * 16 * ESZ, ZJ = GPT * 16;
  constexpr int SH = HS ? 0 : (GPT == 4 ? 2 * 16 * ESZ : (GPT == 2 ? 16 * ESZ : 0)), ZH = SH / ESZ;
  constexpr bool SCALE_EVERY = HS || GPT > 1;  // the scale changes within a tile / every half step
  const int ssh = st == kScaleF32 ? 0 : (nl & 1) * 16;
  const int zsh = (nl & 3) * 8;
  auto scale_h2 = [&](uint32_t x) {
    const uint32_t h = (x >> ssh) & 0xFFFFu;
    if (st == kScaleF16) return as_h2(h | (h << 16));
    const float f = st == kScaleF32 ? __uint_as_float(x)
                                    : (st == kScaleBF16 ? __uint_as_float(h << 16) : f16_bits_to_f32(uint16_t(h)));
    return splat(f);
  };

  f4_t acc[RF][2];
#pragma unroll
  for (int i = 0; i < RF; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  h8_t af[RF];
  h8_t bf[2];
  h2_t sc[2];
  h2_t c0[2] = {zc0, zc0}, c1[2] = {zc1, zc1};
  const Dq2c q2s = dq2_consts(2);
  Dq2c q2[2] = {q2s, q2s};
  if constexpr (BITS == 8) c0[0] = c0[1] = zc8;
  uint32_t bw0 = 0, bw1 = 0, bx0 = 0, bx1 = 0, sw0 = 0, sw1 = 0, zw0 = 0, zw1 = 0;

  // B words (+ scale / zp at a tile start) and A fragments 0 .. HF - 1 of half step u
  auto read_lo = [&](auto Hc, int u) {
    constexpr int H = decltype(Hc)::value;
    const int t = HS ? u : u >> 1;
    const uint32_t bl = lds_addr(smem + NA * HBUF + (t % NBR) * BBUF);
    if constexpr (BITS == 8) {
      const uint2 x0 = lds_b64<0>(bl + boff), x1 = lds_b64<BJ>(bl + boff);
      bw0 = x0.x;
      bx0 = x0.y;
      bw1 = x1.x;
      bx1 = x1.y;
    } else {
      bw0 = lds_b32<HS ? 0 : H * 8>(bl + boff);
      bw1 = lds_b32<HS ? BJ : 1024 + H * 8>(bl + boff);
    }
    if constexpr (H == 0 || SCALE_EVERY) {
      sw0 = lds_b32<H * SH>(bl + soff);
      sw1 = lds_b32<H * SH + SJ>(bl + soff);
      if constexpr (ASYM) {
        zw0 = lds_b32<H * ZH>(bl + zoff);
        zw1 = lds_b32<H * ZH + ZJ>(bl + zoff);
      }
    }
    const uint32_t al = lds_addr(smem + (u % NA) * HBUF) + roff;
    read_frags<0>(af, al, std::make_index_sequence<HF>{});
  };
  auto read_hi = [&](int u) {
    const uint32_t al = lds_addr(smem + (u % NA) * HBUF) + roff;
    read_frags<HF>(af, al, std::make_index_sequence<HF>{});
  };
  auto dequant = [&](auto Hc) {
    constexpr int H = decltype(Hc)::value;
    if constexpr (H == 0 || SCALE_EVERY) {
      sc[0] = scale_h2(sw0);
      sc[1] = scale_h2(sw1);
      if constexpr (ASYM) {
        const int z0 = int(int8_t((zw0 >> zsh) & 0xFFu)), z1 = int(int8_t((zw1 >> zsh) & 0xFFu));
        if constexpr (BITS == 4) {
          c0[0] = zc0 - splat(float(z0));
          c1[0] = zc1 - splat(float(z0));
          c0[1] = zc0 - splat(float(z1));
          c1[1] = zc1 - splat(float(z1));
        } else if constexpr (BITS == 8) {
          c0[0] = zc8 - splat(float(z0));
          c0[1] = zc8 - splat(float(z1));
        } else {  // the symmetric constants less zp: 4 packed subtractions per stripe
          const h2_t y0 = splat(float(z0)), y1 = splat(float(z1));
          q2[0] = Dq2c{q2s.c0 - y0, q2s.c1 - y0, q2s.c2 - y0, q2s.c3 - y0};
          q2[1] = Dq2c{q2s.c0 - y1, q2s.c1 - y1, q2s.c2 - y1, q2s.c3 - y1};
        }
      }
    }
    if constexpr (BITS == 4) {
      bf[0] = dequant_fold(bw0, mag, s16, c0[0], c1[0], sc[0]);
      bf[1] = dequant_fold(bw1, mag, s16, c0[1], c1[1], sc[1]);
    } else if constexpr (BITS == 8) {
      bf[0] = dequant8_fold(bw0, bx0, c0[0], sc[0]);
      bf[1] = dequant8_fold(bw1, bx1, c0[1], sc[1]);
    } else {
      const uint32_t sh = uint32_t(wk) * 8u;
      bf[0] = dequant2_fold(bw0 >> sh, q2[0], sc[0]);
      bf[1] = dequant2_fold(bw1 >> sh, q2[1], sc[1]);
    }
  };

  // prologue: batches -DA .. -1, then the operands of half step 0
#pragma unroll
  for (int v = -DA; v < 0; v++) issue(v);
  wait_vm<WV>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read_lo(std::integral_constant<int, 0>{}, 0);
  read_hi(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  tie(bw0);
  tie(bw1);
  tie(bx0);
  tie(bx1);
  tie(sw0);
  tie(sw1);
  tie(zw0);
  tie(zw1);
  dequant(std::integral_constant<int, 0>{});

  // half step u: entering, B of u is dequantized, A fragments 0 .. HF - 1 of u were issued before the rest (both may be
  // in flight).  The barrier of buffer u + 1 sits between the two MFMA halves.  (Waves 4-7 with that barrier after both
  // halves instead -- a stagger, MI355X_MICROARCH item 9 -- measured 6-15 % slower: profiles/r05_gemm7_stagger_ab.txt.)
  auto half = [&](auto Hc, int u) {
    constexpr int H = decltype(Hc)::value;
    NAD_SCHED_FENCE();
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(HF));  // fragments 0 .. HF - 1 (HF newer reads may be in flight)
    tie_frags<0>(af, std::make_index_sequence<HF>{});
    NAD_SCHED_FENCE();
    issue(u);
#pragma unroll
    for (int i = 0; i < HF; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    NAD_SCHED_FENCE();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    tie_frags<HF>(af, std::make_index_sequence<HF>{});
    wait_vm<WV>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    NAD_SCHED_FENCE();
    read_lo(std::integral_constant<int, 1 - H>{}, u + 1);
    NAD_SCHED_FENCE();
#pragma unroll
    for (int i = HF; i < RF; i++) {
      acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[0], acc[i][0], 0, 0, 0);
      acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[1], acc[i][1], 0, 0, 0);
    }
    NAD_SCHED_FENCE();
    read_hi(u + 1);
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(HF));  // the B words and fragments 0 .. HF - 1 have landed
    tie(bw0);
    tie(bw1);
    tie(bx0);
    tie(bx1);
    tie(sw0);
    tie(sw1);
    tie(zw0);
    tie(zw1);
    dequant(std::integral_constant<int, 1 - H>{});
  };
  for (int u = 0; u < nh2; u += 2) {
    half(std::integral_constant<int, 0>{}, u);
    half(std::integral_constant<int, 1>{}, u + 1);
  }
  // drain the no-op loads past the end and the last (unused) operand reads before the rings are reused
  NAD_SCHED_FENCE();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: the two K halves of each BMT x 32 tile meet in LDS ((k-half 0) + (k-half 1) for every output).  Wave
  // (wn, wk) finishes rows wk * BMT / 2 .. + BMT / 2 - 1.
  constexpr int HR = BMT / 2;
  float* const tw = reinterpret_cast<float*>(smem) + wave * (HR * EPI_LD);
  float* const tp = reinterpret_cast<float*>(smem) + (wave ^ 4) * (HR * EPI_LD);
#pragma unroll
  for (int i = 0; i < HF; i++)
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
      for (int rr = 0; rr < 4; rr++) {
        const float v = wk ? acc[i][j][rr] : acc[HF + i][j][rr];  // the partner's rows
        tp[(i * 16 + kq * 4 + rr) * EPI_LD + j * 16 + nl] = v;
      }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < HF; i++)
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
      for (int rr = 0; rr < 4; rr++) {
        float* p = tw + (i * 16 + kq * 4 + rr) * EPI_LD + j * 16 + nl;
        const float mine = wk ? acc[HF + i][j][rr] : acc[i][j][rr];
        *p = wk == 0 ? mine + *p : *p + mine;
      }
  const int col0 = (bn * NS + wn * 2) * 16;
#pragma unroll 4
  for (int q = 0; q < HR / 8; q++) {
    const int c = q * 64 + lane;
    const int rl = c >> 3, c4 = c & 7;
    const int row = m0 + wk * HR + rl;
    const int n0 = col0 + c4 * 4;
    const float4 t = *reinterpret_cast<const float4*>(tw + rl * EPI_LD + c4 * 4);
    if (row >= M || n0 >= W.n) continue;
    if (nsplit > 1) {
      *reinterpret_cast<float4*>(a.part + (size_t(ks) * M + row) * a.ldp + n0) = t;
      continue;
    }
    float v[4] = {t.x, t.y, t.z, t.w};
    gemm_epilogue4(a, W, row, n0, v);
  }
}

}  // namespace g7

#ifndef G7_BITS
#define G7_BITS 4  // this object's weight format: woq_gemm7.o 4, woq_gemm7_b2.o 2, woq_gemm7_b8.o 8 (Makefile)
#endif
#define G7_CAT2(x, y) x##y
#define G7_CAT(x, y) G7_CAT2(x, y)

hipError_t G7_CAT(launch_gemm7_b, G7_BITS)(const GemmArgs& a, int bm, const _Float16* A16, int lda16, hipStream_t st) {
  constexpr int BITS = G7_BITS;
  const int nbm = (a.M + bm - 1) / bm, nbn = a.nwt > 1 ? a.nbn_all : (a.w.ns + g7::NS - 1) / g7::NS;
  const dim3 grid(nbm * nbn * (a.ksplit > 1 ? a.ksplit : 1));
  auto go = [&](auto k, int lds, bool& done) -> hipError_t {
    if (!done) {  // opt in to the dynamic LDS once per instantiation
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         lds);
      if (e != hipSuccess) return e;
      done = true;
    }
    hipLaunchKernelGGL(k, grid, dim3(512), lds, st, a, A16, lda16);
    return hipGetLastError();
  };
  // groups per B buffer: per tile (int4) or per half step (int2 / int8)
  const int gpt = BITS == 4 ? (a.w.bs == 32 ? 4 : (a.w.bs == 64 ? 2 : 1)) : (a.w.bs == 32 ? 2 : 1);
  auto pick = [&](auto bmc) -> hipError_t {
    constexpr int BMT = decltype(bmc)::value;
    static bool attr[3][2][3] = {};
    const bool asym = a.w.zps != nullptr;
    const int gi = gpt == 4 ? 2 : gpt - 1;
    bool& d = attr[gi][asym][a.scale_t];
    static bool attr_mw[2][3] = {};
    auto sel = [&](auto asc, auto stc, auto gc) {
      constexpr bool AS = decltype(asc)::value;
      constexpr int STT = decltype(stc)::value, GP = decltype(gc)::value;
      constexpr int LDS = g7::Geo<BMT, g7::Bbuf<BITS, GP, STT, AS>>::LDS;
      if constexpr (BITS == 4 && GP == 1 && BMT >= 64) {
        if (a.nwt > 1) return go(g7::woq_gemm7_kernel<BITS, BMT, AS, STT, GP, true>, LDS, attr_mw[AS][a.scale_t]);
      }
      if (a.nwt > 1) return hipErrorInvalidValue;  // fused weights: int4 g128 * 2^j, 64-256-row tiles only
      return go(g7::woq_gemm7_kernel<BITS, BMT, AS, STT, GP>, LDS, d);
    };
    auto by_gpt = [&](auto asc, auto stc) {
      if constexpr (BITS == 4) {
        if (gpt == 4) return sel(asc, stc, std::integral_constant<int, 4>{});
      }
      return gpt == 2 ? sel(asc, stc, std::integral_constant<int, 2>{}) : sel(asc, stc, std::integral_constant<int, 1>{});
    };
    auto by_st = [&](auto asc) {
      switch (a.scale_t) {
        case kScaleF32:
          return by_gpt(asc, std::integral_constant<int, kScaleF32>{});
        case kScaleBF16:
          return by_gpt(asc, std::integral_constant<int, kScaleBF16>{});
        default:
          return by_gpt(asc, std::integral_constant<int, kScaleF16>{});
      }
    };
    return asym ? by_st(std::true_type{}) : by_st(std::false_type{});
  };
  switch (bm) {
    case 32:
      return pick(std::integral_constant<int, 32>{});
    case 64:
      return pick(std::integral_constant<int, 64>{});
    case 128:
      return pick(std::integral_constant<int, 128>{});
    default:
      return pick(std::integral_constant<int, 256>{});
  }
}

#if G7_BITS == 4
// int4: groups of 32, 64 or 128 * 2^j; int2 / int8: 32 or 64 * 2^j (a whole number of groups per 64-deep half step, or
// whole half steps per group)
bool gemm7_ok(int bits, int blocksize, int fold_ok) {
  if (!fold_ok) return false;
  if (blocksize == 32 || blocksize == 64) return bits == 4 || bits == 2 || bits == 8;
  const int unit = bits == 4 ? g7::KT : 64, r = blocksize / unit;
  return (bits == 4 || bits == 2 || bits == 8) && blocksize % unit == 0 && (r & (r - 1)) == 0;
}

hipError_t launch_gemm7_b2(const GemmArgs& a, int bm, const _Float16* A16, int lda16, hipStream_t st);
hipError_t launch_gemm7_b8(const GemmArgs& a, int bm, const _Float16* A16, int lda16, hipStream_t st);

hipError_t launch_gemm7(const GemmArgs& a, int bits, int bm, const _Float16* A16, int lda16, hipStream_t st) {
  return bits == 2   ? launch_gemm7_b2(a, bm, A16, lda16, st)
         : bits == 8 ? launch_gemm7_b8(a, bm, A16, lda16, st)
                     : launch_gemm7_b4(a, bm, A16, lda16, st);
}
#endif

}  // namespace nad
