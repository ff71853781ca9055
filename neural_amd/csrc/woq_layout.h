// woq_layout.h -- the MI355X-native device layout of a weight-only-quantized matrix, and the descriptor that
// bestla_device_load_storage writes into the caller's `devstor` (ne_tensor's embedded device storage,
// neural_speed/core/ne_layers.c:946-949,1022-1024).
//
// Layout (one "stripe" = 16 output features n, one "tile" = 1 KiB of packed weights):
//   tiles  : [ns][nt][64 lanes][16 B]      ns = ceil(N/16), nt = ceil(K/KT), KT = 128 (int4) / 256 (int2) / 64 (int8)
//            Lane l of a tile owns column n = 16*s + (l & 15) and k-quarter kq = l >> 4.  Its 16 bytes are the
//            B fragments of KT/32 consecutive v_mfma_f32_16x16x32_f16 steps: step d covers k = t*KT + 32*d + 8*kq + j,
//            j = 0..7, i.e. exactly the B-operand lane map of 16x16x32 (lane l: B[k = 8(l>>4)+j][n = l&15]).
//            A wave therefore streams a tile with one fully coalesced global_load_dwordx4 and feeds MFMA directly.
//   values : stored biased/unsigned: int4 q+8, int2 q+2, int8 q+128.  Inside a dword the element order is chosen so
//            that ((w >> s) & mask) | 0x6400 yields fp16 pairs (1024 + v_j, 1024 + v_j+1) with no shuffles:
//              int4 dword (one step):   nibble position p holds element j = 2p (p<4) / 2(p-4)+1 (p>=4)
//              int2 dword (two steps):  crumb position p (0..15): step h = (p&7)>>2, j = 2*(p&3) + (p>>3)
//              int8 dword pair (step):  byte b of dword w holds element j = 4w + b (v_perm places it)
//            Tile order: stripe-major [ns][nt] or K-major [nt][ns] (DeviceWeight::kmajor, tile_index()).
//   scales : [ns][ngroups][16] (or K-major [ngroups][ns][16]) in the blob's scale dtype (f32 / bf16 / f16)
//   zps    : same order as scales, int8 (asym only)
//   shuffle: [K] int32 act-order LUT (GPTQ desc_act), applied as a gather on the A operand
//   reduce : [ngroups][ns*16] bf16, integer-core blobs only (the int8-compute mode's zero-point correction)
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define NAD_HD __host__ __device__
#else
#define NAD_HD
#endif

namespace nad {

constexpr uint32_t kWeightMagic = 0x5744414eu;  // "NADW"

enum ScaleType : int32_t { kScaleF32 = 0, kScaleBF16 = 1, kScaleF16 = 2 };

struct DeviceWeight {
  uint32_t magic;
  int32_t bits;       // 2, 4, 8
  int32_t n, k;       // logical shape: out features, in features
  int32_t blocksize;  // quantization group along K
  int32_t ns, nt, ng; // stripes, tiles along K, groups along K
  int32_t scale_t;    // ScaleType
  int32_t asym;
  int32_t has_shuffle;
  int32_t kmajor;     // tile / scale-row order: 0 = stripe-major [ns][nt], 1 = K-major [nt][ns] (see tile_index)
  uint64_t bytes;     // device bytes used from the caller's buffer
  uint64_t src_core_id;
  void* tiles;
  void* scales;
  int8_t* zps;
  int32_t* shuffle;
  void* owner;        // non-null when the library allocated the device memory itself (nad_* helpers)
  void* reduce;       // bf16 [ng][red_ld]: the blob's reduce (Sum_k dequant(w) per block), integer-core blobs only
  int32_t red_ld;     // 0: no reduce
  int32_t blob_bs;    // the blob's own block size (per-channel: may exceed K; the int8-compute quantizer uses it)
  int32_t f4kind;     // NFloat weight: 0 F4_BNB, 1 F4_E2M1, 2 F4_NF4 (codes in the int4 layout, LUT dequant),
                      // 3 F8_E4M3, 4 F8_E5M2 (raw codes in the int8 layout); -1 = integer
  int32_t compute;    // per-weight arithmetic (nad_device_set_compute): 0 follow the thread / process mode, 1 fp,
                      // 2 int8 (integer-core blobs and Q4_0 only)
  int32_t fold_ok;    // every (q - zp) * scale of the weight is 0 or an fp16 normal: the prefill GEMMs may fold the
                      // group scale into the fp16 B fragment (checked at load)
};

// Tile (s, t) and scale row (s, g) positions.  K-major interleaves the stripes at every K position, so the waves of a
// decode launch -- which sweep K in near lock-step over different stripes -- read one contiguous front of HBM at any
// instant (no channel camping), and a prefill block's 8 stripes of one K tile are 8 consecutive KiB.
NAD_HD inline uint64_t tile_index(int kmajor, int ns, int nt, int s, int t) {
  return kmajor ? uint64_t(t) * ns + s : uint64_t(s) * nt + t;
}
NAD_HD inline uint64_t scale_row(int kmajor, int ns, int ng, int s, int g) {
  return kmajor ? uint64_t(g) * ns + s : uint64_t(s) * ng + g;
}

NAD_HD inline int tile_k(int bits) { return bits == 4 ? 128 : (bits == 2 ? 256 : 64); }
NAD_HD inline int steps_per_tile(int bits) { return tile_k(bits) / 32; }

inline uint64_t align256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

// fill the geometry of a DeviceWeight and return the device bytes it needs
inline uint64_t layout_geometry(DeviceWeight& w, int bits, int n, int k, int blocksize, int scale_t, bool asym,
                                bool shuffle, int kmajor = 0, bool reduce = false) {
  w.magic = kWeightMagic;
  w.kmajor = kmajor;
  w.bits = bits;
  w.n = n;
  w.k = k;
  w.blocksize = blocksize;
  w.ns = (n + 15) / 16;
  w.nt = (k + tile_k(bits) - 1) / tile_k(bits);
  w.ng = (k + blocksize - 1) / blocksize;
  w.scale_t = scale_t;
  w.asym = asym ? 1 : 0;
  w.has_shuffle = shuffle ? 1 : 0;
  uint64_t tiles = uint64_t(w.ns) * w.nt * 1024;
  uint64_t sbytes = uint64_t(w.ns) * w.ng * 16 * (scale_t == kScaleF32 ? 4 : 2);
  uint64_t zbytes = asym ? uint64_t(w.ns) * w.ng * 16 : 0;
  uint64_t shf = shuffle ? uint64_t(k) * 4 : 0;
  w.red_ld = reduce ? w.ns * 16 : 0;
  w.blob_bs = blocksize;
  w.f4kind = -1;
  w.compute = 0;
  w.fold_ok = 0;
  uint64_t rbytes = uint64_t(w.ng) * w.red_ld * 2;
  return align256(tiles) + align256(sbytes) + align256(zbytes) + align256(shf) + align256(rbytes);
}

inline void layout_assign(DeviceWeight& w, void* base) {
  char* p = static_cast<char*>(base);
  uint64_t tiles = uint64_t(w.ns) * w.nt * 1024;
  uint64_t sbytes = uint64_t(w.ns) * w.ng * 16 * (w.scale_t == kScaleF32 ? 4 : 2);
  uint64_t zbytes = w.asym ? uint64_t(w.ns) * w.ng * 16 : 0;
  w.tiles = p;
  p += align256(tiles);
  w.scales = p;
  p += align256(sbytes);
  w.zps = w.asym ? reinterpret_cast<int8_t*>(p) : nullptr;
  p += align256(zbytes);
  w.shuffle = w.has_shuffle ? reinterpret_cast<int32_t*>(p) : nullptr;
  p += w.has_shuffle ? align256(uint64_t(w.k) * 4) : 0;
  w.reduce = w.red_ld ? p : nullptr;
  p += align256(uint64_t(w.ng) * w.red_ld * 2);
  w.bytes = uint64_t(p - static_cast<char*>(base));
}

// epilogues (bestla_epilogue.h:114-166; neural_speed/core/layers/bestla_common.hpp:121-216)
enum Epilogue : int32_t {
  kEpiNone = 0,     // AccumulatorWriteBack
  kEpiBias = 1,     // ip_add: + bias[n] (broadcast) or + bias[m][n]
  kEpiSiluMul = 2,  // FFN: silu(W0.a) * (W1.a)       (ip_fusion_ffn.cpp:407-433)
  kEpiGeluMul = 3,  // FFN: gelu(W0.a) * (W1.a)
  kEpiGelu = 4,     // gelu(W0.a)
  kEpiAddGelu = 5,  // gelu(W0.a + bias)
  kEpiSilu = 6,     // swish
  kEpiResAdd = 7,   // + residual[m][n]
};

}  // namespace nad
