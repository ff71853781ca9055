// woq_gemm4.hip -- the pipelined prefill GEMM (gemm3's structure) generalised to the configurations gemm3 leaves to
// the register-staged fallback: int4 with groups of 32 / 64 (the reference Python default is g32,
// neural_speed/__init__.py:150) and int2 with groups of >= 64 (Mistral int2 g64, BASELINE config 5).
//
// Replaces LauncherBase::gemm / run_block + WeightKBlockNInteger::getFpWeight (bestla/bestla/bestla_wrapper.h:481-542,
// bestla_prologue_b.h:732-838) for these weights.
//
// Same skeleton as woq_gemm3_kernel (woq_gemm2.hip): 256 x 128 block tile, 8 waves as 2 (M) x 4 (N), K in 64-deep
// half steps, A (fp16) three half steps ahead in a ring of four 32 KiB LDS buffers, every operand by LDS-DMA, counted
// vmcnt + raw s_barrier at each half step, inline-asm LDS reads.  What changes with the weight format:
//   * a 1 KiB B tile spans HPT = 2 (int4, 128 k) or 4 (int2, 256 k) half steps; it is DMA'd when the A of its first
//     half step goes out, into a ring of NBR tiles, so batch sizes follow the half step's phase in the tile and every
//     wait count is a compile-time constant of that phase;
//   * a tile carries up to GSLOTS groups: scale (and zero-point) dword pieces for all of them go out with the tile,
//     one 256 B piece per wave (slot = wave >> 1, stripe half = wave & 1; spare waves re-copy a slot: identical bytes);
//   * groups end every 2^gh_log2 half steps (>= 64 k) or after every 32-deep MFMA step (G32); at a group end the
//     group accumulators are scaled into the result (exact weights, w = (q - zp) * s in fp32);
//   * int2 crumbs dequantise like woq_device.h dequant_step<2> (0x6400 magic, 2-bit fields), one LDS dword per stripe
//     per half step.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "woq_device.h"
#include "woq_kernels.h"

namespace nad {
namespace g4 {

constexpr int BM = 256, ROWB = 128;        // ROWB: bytes of one A row per 64-deep half step
constexpr int HBUF = BM * ROWB;            // one half step of A: 32 KiB
constexpr int NA = 4;                      // A ring: three half steps in flight
constexpr int BTILES = 8 * 1024;           // one B tile of the block's 8 stripes
constexpr int LDS_BUDGET = 160 * 1024;

template <int BITS>
constexpr int hpt() {
  return BITS == 4 ? 2 : (BITS == 2 ? 4 : 1);
}
template <int BITS, bool G32>
constexpr int gslots() {
  return G32 ? 2 * hpt<BITS>() : hpt<BITS>();
}
// zero points: one byte per column per group, [slot][stripe][16] -- 128 B a slot, filled 256 B (two slots) per wave load
template <int BITS, bool G32>
constexpr int zpbytes() {
  return (gslots<BITS, G32>() < 2 ? 2 : gslots<BITS, G32>()) * 128;
}
template <int BITS, bool G32, bool ASYM>
constexpr int bbuf() {
  return BTILES + gslots<BITS, G32>() * 512 + (ASYM ? zpbytes<BITS, G32>() : 0);
}
template <int BITS, bool G32, bool ASYM>
constexpr int nbr() {
  return (LDS_BUDGET - NA * HBUF) / bbuf<BITS, G32, ASYM>() >= 3 ? 3 : 2;
}
template <int BITS, bool G32, bool ASYM>
constexpr int lds_bytes() {
  // a 2-deep ring is only safe when a tile spans more than two half steps (int2)
  static_assert(hpt<BITS>() > 2 || nbr<BITS, G32, ASYM>() == 3, "int4 / int8 need a 3-deep B ring");
  return NA * HBUF + nbr<BITS, G32, ASYM>() * bbuf<BITS, G32, ASYM>();
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
// int4: 8 nibbles of one dword -> 8 exact fp16 (q - 8 - zp), 0x6400 magic (as woq_gemm2.hip)
__device__ __forceinline__ h8_t dq4(uint32_t w, h2_t s16, h2_t c0, h2_t c1) {
  const uint32_t m0 = 0x000F000Fu, m1 = 0x00F000F0u, mag = 0x64006400u;
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
// int2: the 16-bit half `sh` (0 or 8) of a dword -> 8 exact fp16 (q - 2 - zp); field order of dequant_step<2>
__device__ __forceinline__ h8_t dq2(uint32_t w, int sh, h2_t c) {
  const uint32_t m = 0x00030003u, mag = 0x64006400u;
  const uint32_t x = w >> sh;
  const h2_t p0 = as_h2(and_or(x, m, mag)) + c;
  const h2_t p1 = as_h2(and_or(x >> 2, m, mag)) + c;
  const h2_t p2 = as_h2(and_or(x >> 4, m, mag)) + c;
  const h2_t p3 = as_h2(and_or(x >> 6, m, mag)) + c;
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

// int8: 8 bytes (two dwords) -> 8 exact fp16 (q - 128 - zp): byte b becomes the fp16 1024 + b by a byte permute
__device__ __forceinline__ h8_t dq8(uint32_t w0, uint32_t w1, h2_t c) {
  const h2_t p0 = as_h2(__builtin_amdgcn_perm(0x64646464u, w0, 0x04010400u)) + c;
  const h2_t p1 = as_h2(__builtin_amdgcn_perm(0x64646464u, w0, 0x04030402u)) + c;
  const h2_t p2 = as_h2(__builtin_amdgcn_perm(0x64646464u, w1, 0x04010400u)) + c;
  const h2_t p3 = as_h2(__builtin_amdgcn_perm(0x64646464u, w1, 0x04030402u)) + c;
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
// LDS reads in inline asm (hipcc would put a vmcnt(0) before every LDS read it can see while an LDS-DMA is in flight)
template <int OFF>
__device__ __forceinline__ h8_t lds_b128(uint32_t addr) {
  h8_t r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ u4_t lds_u128(uint32_t addr) {
  u4_t r;
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
__device__ __forceinline__ uint32_t lds_b32v(uint32_t addr) {  // runtime offset folded into the address
  uint32_t r;
  asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
template <size_t... I>
__device__ __forceinline__ void lds_frags(h8_t (&f)[8], uint32_t addr, std::index_sequence<I...>) {
  ((f[I] = lds_b128<int(I) * 16 * ROWB>(addr)), ...);
}
template <size_t... I>
__device__ __forceinline__ void lds_frags16(h8_t (&f)[16], uint32_t addr, std::index_sequence<I...>) {
  ((f[I] = lds_b128<int(I) * 16 * ROWB>(addr)), ...);
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
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return uint32_t(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p));
}

// KSW (folded launches only): the waves split over K instead of M -- 1 (M) x 4 (N) x 2 (K), wave (wn, wk) owns a
// 256 x 32 partial over the 32-deep step wk of every half step -- so each B fragment is dequantized (and scaled) once
// per workgroup instead of by both M-waves (gemm5 in woq_gemm2.hip is the same change for gemm3); the two K-halves meet
// in the epilogue
template <int BITS, bool G32, bool ASYM, bool FOLD = false, bool KSW = false>
__global__ __launch_bounds__(512, 1) void woq_gemm4_kernel(GemmArgs a, const _Float16* __restrict__ A16, int lda16,
                                                           int gh_log2) {
  static_assert(!KSW || FOLD, "the K-split wave layout keeps no per-group partials: folded launches only");
  constexpr int HPT = hpt<BITS>();
  constexpr int GS = gslots<BITS, G32>();
  constexpr int BSC = GS * 512;
  constexpr int BBUF = bbuf<BITS, G32, ASYM>();
  constexpr int NBR = nbr<BITS, G32, ASYM>();
  constexpr int NBW = ASYM ? 3 : 2;  // B-side VMEM instructions of a tile batch, per wave
  constexpr int ZPB = zpbytes<BITS, G32>();
  constexpr int BIAS = BITS == 4 ? 8 : (BITS == 2 ? 2 : 128);
  // int8: a tile is one half step, so the tile rides two half steps ahead (not three, as A does): a 4-deep tile ring
  // would not fit beside the A ring.  Its batch is [tile (u + 2), A (u + 3)], tile first.
  constexpr bool B2 = BITS == 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int wm = wave >> 2, wn = wave & 3;
  const int wk = wave >> 2;  // KSW: this wave's 32-deep step of every half step
  const SkinnyWeight& W = a.w;
  const int M = a.M, nt = W.nt, ng = W.ng, ns = W.ns;
  const int gh = 1 << gh_log2;

  // XCD-aware remap (as gemm2 / gemm3)
  const int nbm = (M + BM - 1) / BM;
  const int nbn = (ns + 7) / 8;
  const int ntile = nbm * nbn;
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;  // split-K runs of whole groups (see woq_gemm3_kernel)
  const int nwg = ntile * nsplit;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8, o = bid / 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + o;
  }
  const int ks = bid / ntile;
  bid -= ks * ntile;
  const int kt0 = nsplit > 1 ? ks * a.ktiles : 0;
  const int ntl = nsplit > 1 ? min(a.ktiles, nt - kt0) : nt;
  const int nh = HPT * ntl;  // half steps of this run
  const int bm = bid / nbn, bn = bid % nbn;
  const int m0 = bm * BM;
  const int nl = lane & 15, kq = lane >> 4;

  uint32_t aoff[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int row = (wave * 4 + i) * 8 + (lane >> 3);
    const int grow = min(m0 + row, M - 1);
    aoff[i] = uint32_t(grow) * uint32_t(lda16) * 2u + uint32_t(((lane & 7) ^ ((row >> 1) & 7)) * 16);
  }
  const char* abase = reinterpret_cast<const char*>(A16) + size_t(kt0) * HPT * ROWB;
  const char* btile = static_cast<const char*>(W.tiles) + (size_t(min(bn * 8 + wave, ns - 1)) * nt * 64 + lane) * 16;
  const int sstripe = min(bn * 8 + (wave & 1) * 4 + (lane >> 4), ns - 1);
  const size_t srow0 = size_t(sstripe) * ng * 16 + nl;
  const int slot_w = (wave >> 1) % GS;  // this wave's scale slot
  // zero-point piece of this wave: slots 2 zq, 2 zq + 1 (lanes 0-31 / 32-63), stripe (lane >> 2) & 7, 4 columns a lane
  const int zq = wave % (ZPB / 256);
  const int zslot = min(2 * zq + (lane >> 5), GS - 1);
  const size_t zrow0 = size_t(min(bn * 8 + ((lane >> 2) & 7), ns - 1)) * ng * 16 + (lane & 3) * 4;
  const int st = a.scale_t;
  const uint32_t* sbase = static_cast<const uint32_t*>(W.scales);
  const uint32_t* zbase = reinterpret_cast<const uint32_t*>(W.zps);

  // group of tile t's slot s
  auto slot_group = [&](int t, int s) {
    int g;
    if constexpr (G32)
      g = t * (2 * HPT) + s;
    else
      g = ((t * HPT) >> gh_log2) + (gh_log2 < 30 ? min(s, max(HPT >> gh_log2, 1) - 1) : 0);
    return min(g, ng - 1);
  };

  // batch(u): A(u + 3) and, when u + 3 starts a tile, that tile + its scale (+ zero-point) pieces
  auto issue_tile = [&](int t) {  // t: tile of this run (ring slot), tg: tile of the weight
    char* bb = smem + NA * HBUF + (t % NBR) * BBUF;
    const int tg = t + kt0;
    glds16(btile + size_t(tg) * 1024, bb + wave * 1024);
    const size_t si = srow0 + size_t(slot_group(tg, slot_w)) * 16;
    glds4(sbase + (st == kScaleF32 ? si : (si >> 1)), bb + BTILES + slot_w * 512 + (wave & 1) * 256);
    if constexpr (ASYM) glds4(zbase + ((zrow0 + size_t(slot_group(tg, zslot)) * 16) >> 2), bb + BTILES + BSC + zq * 256);
  };
  auto issue = [&](auto Pc, int u) {
    constexpr int P = decltype(Pc)::value;  // (u + 3) % HPT
    if constexpr (B2) {
      if (u + 2 >= 0 && u + 2 < nh) issue_tile(u + 2);
    }
    if (u + 3 >= nh) return;
    const int ua = u + 3;
    char* ab = smem + (ua & 3) * HBUF;
    const char* src = abase + size_t(ua) * ROWB;
#pragma unroll
    for (int i = 0; i < 4; i++) glds16(src + aoff[i], ab + (wave * 4 + i) * 1024);
    if constexpr (!B2 && P == 0) issue_tile(ua / HPT);
  };

  constexpr int RB = KSW ? 16 : 8;  // 16-row blocks per wave
  f4_t acc[RB][2], accg[8][2];
#pragma unroll
  for (int i = 0; i < RB; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) accg[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  // prologue: batches -3, -2, -1 (A0 + tile 0, A1, A2; the tile of half 2 goes with A2 when HPT == 2)
  issue(std::integral_constant<int, 0>{}, -3);
  issue(std::integral_constant<int, 1 % HPT>{}, -2);
  issue(std::integral_constant<int, 2 % HPT>{}, -1);
  // wait for batch -3: batches -2 and -1 may stay in flight
  if constexpr (B2) {  // batch -2 = [tile 0, A1], batch -1 = [tile 1, A2]: tile 0 landed, A1 + batch -1 in flight
    if (nh > 2)
      wait_vm<8 + NBW>();
    else if (nh > 1)
      wait_vm<4 + NBW>();
    else
      wait_vm<0>();
  } else {
    constexpr int b2 = 4 + ((1 % HPT) == 0 ? NBW : 0), b1 = 4 + ((2 % HPT) == 0 ? NBW : 0);
    if (nh > 2)
      wait_vm<b2 + b1>();
    else if (nh > 1)
      wait_vm<b2>();
    else
      wait_vm<0>();
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const h2_t s16 = splat(1.f / 16.f);
  const h2_t zc0 = splat(-(1024.f + BIAS)), zc1 = splat(-(64.f + BIAS));
  uint32_t roff[2];
#pragma unroll
  for (int dd = 0; dd < 2; dd++) roff[dd] = uint32_t((wm * 128 + nl) * ROWB + (((dd * 4 + kq) ^ ((nl >> 1) & 7)) * 16));
  // KSW: rows 0..255 (f(row) = (nl >> 1) & 7 for every 16-row block), chunk of step wk
  const uint32_t roffk = uint32_t(nl * ROWB + (((wk * 4 + kq) ^ ((nl >> 1) & 7)) * 16));
  const int boff = (wn * 2) * 1024 + lane * 16;
  const int soff = BTILES + ((wn * 2) * 16 + nl) * 4;
  const int zoff = BTILES + BSC + (wn * 2) * 16 + (nl & ~3);
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
  // FOLD (G32): the scale as an fp16 pair -- fp16 scales are the stored bits, exact; bf16 / f32 ones are rounded once
  auto scale_h8 = [&](uint32_t x) {
    _Float16 hs;
    if (st == kScaleF16)
      hs = __builtin_bit_cast(_Float16, uint16_t((x >> ssh) & 0xFFFFu));
    else
      hs = _Float16(scale_f32(x));
    return h8_t{hs, hs, hs, hs, hs, hs, hs, hs};
  };

  auto hand_over = [&](auto Hc, int u) {
    constexpr int H = decltype(Hc)::value;
    // hand-over: batch u - 2 has landed; batches u - 1 and u stay in flight
    if constexpr (B2) {  // tile u + 1 (head of batch u - 1) and A(u + 1) landed; A(u + 2) and batch u in flight
      if (u + 3 < nh)
        wait_vm<8 + NBW>();
      else if (u + 2 < nh)
        wait_vm<4 + NBW>();
      else
        wait_vm<0>();
    } else {
      constexpr int bu = 4 + (((H + 3) % HPT) == 0 ? NBW : 0);   // |batch u| (when issued)
      constexpr int bu1 = 4 + (((H + 2) % HPT) == 0 ? NBW : 0);  // |batch u - 1|
      if (u + 3 < nh)
        wait_vm<bu + bu1>();
      else if (u + 2 < nh)
        wait_vm<bu1>();
      else
        wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // L (late, waves 4-7): the barrier of half step u comes after its first 32-deep step (see woq_gemm3_kernel)
  auto half = [&](auto Hc, auto Lc, int u) {
    constexpr int H = decltype(Hc)::value;  // phase of half step u in its tile
    constexpr bool L = decltype(Lc)::value;
    const int t = u / HPT;
    const char* ab = smem + (u & 3) * HBUF;
    const char* bb = smem + NA * HBUF + (t % NBR) * BBUF;
    issue(std::integral_constant<int, (H + 3) % HPT>{}, u);
    const uint32_t al = lds_addr(ab), bl = lds_addr(bb);
    if constexpr (KSW) {
      // this wave's step wk: one B dword per stripe (int8: two), its group's scale (and zero point), 16 A fragments
      const int slot = G32 ? 2 * H + wk : (gh_log2 >= 30 ? 0 : (H >> gh_log2) % GS);
      uint32_t b0 = 0u, b1 = 0u;
      uint2 e0 = {0u, 0u}, e1 = {0u, 0u};
      if constexpr (BITS == 8) {
        e0 = lds_b64<0>(bl + boff + wk * 8);
        e1 = lds_b64<1024>(bl + boff + wk * 8);
      } else if constexpr (BITS == 4) {
        b0 = lds_b32<H * 8>(bl + boff + wk * 4);
        b1 = lds_b32<1024 + H * 8>(bl + boff + wk * 4);
      } else {
        b0 = lds_b32<H * 4>(bl + boff);
        b1 = lds_b32<1024 + H * 4>(bl + boff);
      }
      uint32_t z0 = 0u, z1 = 0u;
      if constexpr (ASYM) {
        const uint32_t za = bl + zoff + slot * 128;
        z0 = lds_b32v(za);
        z1 = lds_b32v(za + 16);
      }
      const uint32_t sa = bl + soff + slot * 512;
      uint32_t s0 = lds_b32v(sa), s1 = lds_b32v(sa + 64);
      h8_t af[16];
      lds_frags16(af, al + roffk, std::make_index_sequence<16>{});
      wait_lgk<8>(b0, b1, e0, e1, z0, z1, s0, s1, af[0], af[1], af[2], af[3], af[4], af[5], af[6], af[7]);
      if constexpr (L) {
        wait_lgk<0>(af[8], af[9], af[10], af[11], af[12], af[13], af[14], af[15]);
        hand_over(Hc, u);
      }
      h8_t bf[2];
      const uint32_t bw1[2] = {b0, b1};
      const uint2 bw8[2] = {e0, e1};
      const uint32_t zw1[2] = {z0, z1};
      const uint32_t sw1[2] = {s0, s1};
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const float zf = ASYM ? float(int(int8_t((zw1[j] >> zsh) & 0xFFu))) : 0.f;
        if constexpr (BITS == 8)
          bf[j] = dq8(bw8[j].x, bw8[j].y, zc0 - splat(zf));
        else if constexpr (BITS == 4)
          bf[j] = dq4(bw1[j], s16, zc0 - splat(zf), zc1 - splat(zf));
        else
          bf[j] = dq2(bw1[j], wk * 8, zc0 - splat(zf));
        bf[j] = bf[j] * scale_h8(sw1[j]);
      }
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
      if constexpr (!L) wait_lgk<0>(af[8], af[9], af[10], af[11], af[12], af[13], af[14], af[15]);
#pragma unroll
      for (int i = 8; i < RB; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
      if constexpr (!L) hand_over(Hc, u);
      return;
    } else {
    // B words of this half step for the wave's two stripes: int4 two dwords (one per 32-deep step), int2 one dword
    uint32_t bw[2][2];
    u4_t b8[2];
    if constexpr (BITS == 8) {
      b8[0] = lds_u128<0>(bl + boff);
      b8[1] = lds_u128<1024>(bl + boff);
      bw[0][0] = bw[0][1] = bw[1][0] = bw[1][1] = 0u;
    } else if constexpr (BITS == 4) {
      const uint2 v0 = lds_b64<H * 8>(bl + boff), v1 = lds_b64<1024 + H * 8>(bl + boff);
      bw[0][0] = v0.x;
      bw[0][1] = v0.y;
      bw[1][0] = v1.x;
      bw[1][1] = v1.y;
    } else {
      // one dword serves both 32-deep steps.  No copy into bw[j][1]: a register copy of an inline-asm LDS result would
      // be scheduled before the lgkmcnt wait and read the register before the data lands
      bw[0][0] = lds_b32<H * 4>(bl + boff);
      bw[1][0] = lds_b32<1024 + H * 4>(bl + boff);
      bw[0][1] = bw[1][1] = 0u;
    }
    // group slot(s) of this half step
    const int slot = G32 ? 2 * H : (gh_log2 >= 30 ? 0 : (H >> gh_log2) % GS);
    uint32_t zw[2][2] = {{0u, 0u}, {0u, 0u}};
    if constexpr (ASYM) {
      const uint32_t za = bl + zoff + slot * 128;
      zw[0][0] = lds_b32v(za);
      zw[1][0] = lds_b32v(za + 16);
      if constexpr (G32) {
        zw[0][1] = lds_b32v(za + 128);
        zw[1][1] = lds_b32v(za + 128 + 16);
      }
    }
    // G32: both groups' scales up front, so each 32-deep step's products scale straight into the result
    uint32_t sg[2][2] = {{0u, 0u}, {0u, 0u}};
    if constexpr (G32) {
      const uint32_t sa = bl + soff + slot * 512;
      sg[0][0] = lds_b32v(sa);
      sg[0][1] = lds_b32v(sa + 64);
      sg[1][0] = lds_b32v(sa + 512);
      sg[1][1] = lds_b32v(sa + 512 + 64);
    } else if constexpr (FOLD) {  // the half step's group: its scales fold into the B fragments of both steps
      // (each register its own LDS read: a C++ copy of an inline-asm LDS result would run before the lgkmcnt wait)
      const uint32_t sa = bl + soff + slot * 512;
      sg[0][0] = lds_b32v(sa);
      sg[0][1] = lds_b32v(sa + 64);
      sg[1][0] = lds_b32v(sa);
      sg[1][1] = lds_b32v(sa + 64);
    }
    h8_t af0[8], af1[8];
    lds_frags(af0, al + roff[0], std::make_index_sequence<8>{});
    lds_frags(af1, al + roff[1], std::make_index_sequence<8>{});
    wait_lgk<8>(b8[0], b8[1], bw[0][0], bw[0][1], bw[1][0], bw[1][1], zw[0][0], zw[0][1], zw[1][0], zw[1][1], sg[0][0], sg[0][1],
                sg[1][0], sg[1][1], af0[0], af0[1], af0[2], af0[3], af0[4], af0[5], af0[6], af0[7]);
    const bool gstart = G32 || (u & (gh - 1)) == 0;
    const bool gend = G32 || ((u + 1) & (gh - 1)) == 0 || u == nh - 1;
    uint32_t sw0 = 0, sw1 = 0;
#pragma unroll
    for (int dd = 0; dd < 2; dd++) {
      if (dd == 1) {
        wait_lgk<0>(af1[0], af1[1], af1[2], af1[3], af1[4], af1[5], af1[6], af1[7]);
        if constexpr (L) {
          if (!G32 && gend) {
            sw0 = lds_b32v(bl + soff + slot * 512);
            sw1 = lds_b32v(bl + soff + slot * 512 + 64);
            wait_lgk<0>(sw0, sw1);
          }
          hand_over(Hc, u);
        }
      }
      const int zi = G32 ? dd : 0;
      h8_t bf[2];
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const float zf = ASYM ? float(int(int8_t((zw[j][zi] >> zsh) & 0xFFu))) : 0.f;
        if constexpr (BITS == 8)
          bf[j] = dq8(b8[j][2 * dd], b8[j][2 * dd + 1], zc0 - splat(zf));
        else if constexpr (BITS == 4)
          bf[j] = dq4(bw[j][dd], s16, zc0 - splat(zf), zc1 - splat(zf));
        else
          bf[j] = dq2(bw[j][0], dd * 8, zc0 - splat(zf));
      }
      if constexpr (FOLD) {
        // the group scale folded into the fp16 B fragment (q * s rounded once; DeviceWeight::fold_ok checked that every
        // q * s is an fp16 normal): the MFMAs accumulate straight into the result -- no per-step (g32) or group-end
        // (g >= 64) scaling FMAs
#pragma unroll
        for (int j = 0; j < 2; j++) bf[j] = bf[j] * scale_h8(sg[dd][j]);
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const h8_t af = dd == 0 ? af0[i] : af1[i];
#pragma unroll
          for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], acc[i][j], 0, 0, 0);
        }
        continue;
      }
      if constexpr (G32) {
        const float sf[2] = {scale_f32(sg[dd][0]), scale_f32(sg[dd][1])};
        // software-pipelined by one row block: the products of block i are scaled in while block i + 1 multiplies,
        // so only two blocks of products are ever live
        f4_t p[2][2];
#pragma unroll
        for (int i = 0; i <= 8; i++) {
          if (i < 8) {
            const h8_t af = dd == 0 ? af0[i] : af1[i];
#pragma unroll
            for (int j = 0; j < 2; j++) p[i & 1][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], zero, 0, 0, 0);
          }
          if (i > 0) {
#pragma unroll
            for (int j = 0; j < 2; j++) {
              acc[i - 1][j] += p[(i - 1) & 1][j] * sf[j];
              tie(acc[i - 1][j]);  // pin the update here: left alone, the compiler sinks it past the hand-over
            }                      // branches and keeps every product of the half step live (spills)
          }
        }
        continue;
      }
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const h8_t af = dd == 0 ? af0[i] : af1[i];
#pragma unroll
        for (int j = 0; j < 2; j++) {
          const bool fresh = dd == 0 && gstart;
          accg[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], fresh ? zero : accg[i][j], 0, 0, 0);
        }
      }
      if (dd == 1 && gend) {  // group end: scale the group partials into the result
        if constexpr (!L) {
          const uint32_t sa = bl + soff + slot * 512;
          sw0 = lds_b32v(sa);
          sw1 = lds_b32v(sa + 64);
          wait_lgk<0>(sw0, sw1);
        }
        const float sf[2] = {scale_f32(sw0), scale_f32(sw1)};
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
          for (int i = 0; i < 8; i++) {
            acc[i][j] += accg[i][j] * sf[j];
            tie(acc[i][j]);
          }
      }
    }
    if constexpr (!L) hand_over(Hc, u);
    }
  };

  auto loop = [&](auto Lc) {
    for (int u = 0; u < nh; u += HPT) {
      half(std::integral_constant<int, 0>{}, Lc, u);
      if constexpr (HPT >= 2) half(std::integral_constant<int, 1>{}, Lc, u + 1);
      if constexpr (HPT == 4) {
        half(std::integral_constant<int, 2>{}, Lc, u + 2);
        half(std::integral_constant<int, 3>{}, Lc, u + 3);
      }
    }
  };
  if (a.stagger && wave >= 4)
    loop(std::true_type{});
  else
    loop(std::false_type{});

  // epilogue through LDS (as gemm3); KSW: the two K-halves of each 256 x 32 tile meet first (as gemm5): wave (wn, wk)
  // finishes rows wk * 128 .. + 127, its partial of the other rows goes to its partner's region
  float* tw = reinterpret_cast<float*>(smem) + wave * (128 * 36);
  if constexpr (KSW) {
    __syncthreads();
    float* const tp = reinterpret_cast<float*>(smem) + (wave ^ 4) * (128 * 36);
    // (static indices only: a wave-dependent index into acc would move the whole array to scratch memory)
    auto put = [&](auto Oc) {
      constexpr int O = decltype(Oc)::value;
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
          for (int rr = 0; rr < 4; rr++) tp[(i * 16 + kq * 4 + rr) * 36 + j * 16 + nl] = acc[(O + i) % RB][j][rr];
    };
    auto add = [&](auto Oc) {
      constexpr int O = decltype(Oc)::value;
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
          for (int rr = 0; rr < 4; rr++) tw[(i * 16 + kq * 4 + rr) * 36 + j * 16 + nl] += acc[(O + i) % RB][j][rr];
    };
    if (wk == 0)
      put(std::integral_constant<int, 8>{});
    else
      put(std::integral_constant<int, 0>{});
    __syncthreads();
    if (wk == 0)
      add(std::integral_constant<int, 0>{});
    else
      add(std::integral_constant<int, 8>{});
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j < 2; j++)
#pragma unroll
        for (int rr = 0; rr < 4; rr++) tw[(i * 16 + kq * 4 + rr) * 36 + j * 16 + nl] = acc[i][j][rr];
  }
  const int s0 = bn * 8 + wn * 2;
  const int col0 = s0 * 16;
#pragma unroll 4
  for (int q = 0; q < 16; q++) {
    const int c = q * 64 + lane;
    const int rl = c >> 3, c4 = c & 7;
    const int row = m0 + (KSW ? wk : wm) * 128 + rl;
    const int n0 = col0 + c4 * 4;
    const float4 tv = *reinterpret_cast<const float4*>(tw + rl * 36 + c4 * 4);
    if (row >= M || n0 >= W.n) continue;
    if (nsplit > 1) {  // raw partial of this K run; launch_splitk_reduce applies the epilogue
      *reinterpret_cast<float4*>(a.part + (size_t(ks) * M + row) * a.ldp + n0) = tv;
      continue;
    }
    float v[4] = {tv.x, tv.y, tv.z, tv.w};
    gemm_epilogue4(a, row, n0, v);
  }
}

}  // namespace g4

// 0 if gemm4 does not take this weight; kG32Mode for int4 groups of 32; else gh_log2 + 1 (gh_log2: log2 of half steps
// per group, 30 = one group over all of K)
constexpr int kG32Mode = 100;
int gemm4_mode(int bits, int blocksize, int ng, int kpad, bool asym) {
  if (bits != 4 && bits != 2 && bits != 8) return 0;
  (void)asym;
  if (ng == 1) return 30 + 1;  // per-channel
  if (blocksize == 32) return bits == 2 ? 0 : kG32Mode;
  if (blocksize < 64 || blocksize % 64) return 0;
  const int gh = blocksize / 64;
  if (gh & (gh - 1)) return 0;
  (void)kpad;
  return __builtin_ctz(unsigned(gh)) + 1;
}

hipError_t launch_gemm4(const GemmArgs& a, int bits, const _Float16* A16, int lda16, hipStream_t st) {
  const int mode = gemm4_mode(bits, a.w.bs, a.w.ng, a.w.nt * (bits == 4 ? 128 : (bits == 2 ? 256 : 64)), a.w.zps != nullptr);
  if (!mode) return hipErrorInvalidValue;
  const bool g32 = mode == kG32Mode;
  const int gh_log2 = g32 ? 0 : mode - 1;
  const int nbm = (a.M + g4::BM - 1) / g4::BM, nbn = (a.w.ns + 7) / 8;
  const bool asym = a.w.zps != nullptr;
  GemmArgs ga = a;
  // the stagger measured +4-14 % for int4 / int8 and neutral to -5 % for int2 (profiles/r02_gemm4_stagger.txt); with
  // the scale fold int2 gains too, +5-11 % (profiles/r03_gemm4_int2_stagger_fold.txt): off only for unfolded int2
  if (bits == 2 && !a.fold) ga.stagger = 0;
  auto go = [&](auto k, int lds) -> hipError_t {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(nbm * nbn * (a.ksplit > 1 ? a.ksplit : 1)), dim3(512), lds, st, ga, A16, lda16, gh_log2);
    return hipGetLastError();
  };
#define NAD_G4(B, G, A) go(g4::woq_gemm4_kernel<B, G, A>, g4::lds_bytes<B, G, A>())
#define NAD_G4F(B, G, A)                                                                              \
  (a.ksw ? go(g4::woq_gemm4_kernel<B, G, A, true, true>, g4::lds_bytes<B, G, A>())                    \
         : go(g4::woq_gemm4_kernel<B, G, A, true, false>, g4::lds_bytes<B, G, A>()))
  if (bits == 4) {
    if (g32 && a.fold) return asym ? NAD_G4F(4, true, true) : NAD_G4F(4, true, false);
    if (g32) return asym ? NAD_G4(4, true, true) : NAD_G4(4, true, false);
    if (a.fold) return asym ? NAD_G4F(4, false, true) : NAD_G4F(4, false, false);
    return asym ? NAD_G4(4, false, true) : NAD_G4(4, false, false);
  }
  if (bits == 8) {
    if (g32 && a.fold) return asym ? NAD_G4F(8, true, true) : NAD_G4F(8, true, false);
    if (g32) return asym ? NAD_G4(8, true, true) : NAD_G4(8, true, false);
    if (a.fold) return asym ? NAD_G4F(8, false, true) : NAD_G4F(8, false, false);
    return asym ? NAD_G4(8, false, true) : NAD_G4(8, false, false);
  }
  if (a.fold) return asym ? NAD_G4F(2, false, true) : NAD_G4F(2, false, false);
  return asym ? NAD_G4(2, false, true) : NAD_G4(2, false, false);
#undef NAD_G4
#undef NAD_G4F
}

}  // namespace nad
