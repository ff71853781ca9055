// ref_golden.cpp -- golden-vector generator compiled DIRECTLY against the reference's own sources
// (/root/reference/bestla/bestla/kernel_ref.h + bestla_utils.h + bestla.h; no copies, no stand-ins).
// TEST INFRASTRUCTURE ONLY: built by oracle/ref/Makefile into oracle/_ref/ref_golden (git-ignored), run by
// tests/golden/make_golden.py in the build container; its outputs are committed under tests/golden/.
//
// Output: for each case, raw little-endian arrays <dir>/<case>.<name>.bin plus a line in <dir>/manifest.txt:
//   <case> <name> <dtype> <n_elements>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kernel_ref.h"

using namespace bestla;

static std::string g_dir;
static FILE* g_man = nullptr;

template <typename T>
static void dump(const std::string& cs, const std::string& name, const char* dt, const T* p, size_t n) {
  std::string path = g_dir + "/" + cs + "." + name + ".bin";
  FILE* f = fopen(path.c_str(), "wb");
  fwrite(p, sizeof(T), n, f);
  fclose(f);
  fprintf(g_man, "%s %s %s %zu\n", cs.c_str(), name.c_str(), dt, n);
}

// deterministic xorshift so the inputs are reproducible (they are also dumped, tests never regenerate them)
static uint32_t g_state = 20250112u;
static uint32_t rnd() {
  g_state ^= g_state << 13;
  g_state ^= g_state >> 17;
  g_state ^= g_state << 5;
  return g_state;
}
static float urand(float lo, float hi) { return lo + (hi - lo) * (float)(rnd() & 0xFFFFFF) / 16777216.f; }

static void case_quant(const char* cs, int row, int col, int bs, BTLA_DTYPE qt, bool asym, int special) {
  std::vector<float> src((size_t)row * col);
  for (auto& v : src) v = urand(-0.5f, 0.5f);
  if (special == 1) {  // an all-zero block and an all-positive block and a constant block
    for (int r = 0; r < bs && r < row; r++) src[(size_t)r * col + 0] = 0.f;
    for (int r = 0; r < bs && r < row; r++) src[(size_t)r * col + 1] = urand(0.1f, 0.4f);
    for (int r = 0; r < bs && r < row; r++) src[(size_t)r * col + 2] = -0.25f;
  }
  int nblk = (row + bs - 1) / bs;
  std::vector<int8_t> q((size_t)row * col), zp((size_t)nblk * col);
  std::vector<float> s((size_t)nblk * col);
  kernel::ref::quantize_f32_sign_int_rowblock(src.data(), q.data(), row, col, col, col, s.data(),
                                              asym ? zp.data() : nullptr, bs, qt);
  int meta[5] = {row, col, bs, (int)utils::bestla_dtype_bits(qt), asym ? 1 : 0};
  dump(cs, "meta", "i4", meta, 5);
  dump(cs, "src", "f4", src.data(), src.size());
  dump(cs, "q", "i1", q.data(), q.size());
  dump(cs, "s", "f4", s.data(), s.size());
  if (asym) dump(cs, "zp", "i1", zp.data(), zp.size());
}

static void case_interleave(const char* cs, int row, int col, int ntile, int rowpack) {
  int rowpad = utils::padto(row, rowpack * 4 > 0 ? rowpack : 1);
  rowpad = utils::padto(rowpad, rowpack);
  int colpad = utils::padto(col, ntile);
  std::vector<int8_t> src((size_t)row * col), dst((size_t)rowpad * colpad), back((size_t)row * col);
  for (auto& v : src) v = (int8_t)((int)(rnd() % 16) - 8);
  kernel::ref::padding_interleave<int8_t>(src.data(), dst.data(), row, col, rowpad, colpad, col, rowpad, ntile,
                                          rowpack);
  kernel::ref::revert_padding_interleave<int8_t>(dst.data(), back.data(), row, col, rowpad, colpad, rowpad, col,
                                                 ntile, rowpack);
  int meta[6] = {row, col, rowpad, colpad, ntile, rowpack};
  dump(cs, "meta", "i4", meta, 6);
  dump(cs, "src", "i1", src.data(), src.size());
  dump(cs, "dst", "i1", dst.data(), dst.size());
  dump(cs, "back", "i1", back.data(), back.size());
}

static void case_compress(const char* cs, size_t n) {
  std::vector<int8_t> s4(n), s2(n), d4(n), d2(n), tmp(64);
  for (auto& v : s4) v = (int8_t)((int)(rnd() % 16) - 8);
  for (auto& v : s2) v = (int8_t)((int)(rnd() % 4) - 2);
  std::vector<utils::int4x2> c4(n / 2);
  std::vector<utils::bit2x4> c2(n / 4);
  kernel::ref::compress_s8_s4(s4.data(), c4.data(), n);
  kernel::ref::compress_2bit(s2.data(), c2.data(), n);
  kernel::ref::decompress_s4_s8(c4.data(), d4.data(), n, tmp.data(), tmp.size());
  kernel::ref::decompress_s2_s8(c2.data(), d2.data(), n, tmp.data(), tmp.size());
  dump(cs, "s4", "i1", s4.data(), n);
  dump(cs, "c4", "u1", reinterpret_cast<uint8_t*>(c4.data()), n / 2);
  dump(cs, "d4", "i1", d4.data(), n);
  dump(cs, "s2", "i1", s2.data(), n);
  dump(cs, "c2", "u1", reinterpret_cast<uint8_t*>(c2.data()), n / 4);
  dump(cs, "d2", "i1", d2.data(), n);
}

// decompress_kblock_s4_s8 + decompress_kblock_s8_fp for one NTILE stripe with zero points (the getFpWeight chain)
template <int PackRow, int NTILE>
static void case_dequant_s4(const char* cs, int row, int bs, bool bf16scale) {
  int nblk = (row + bs - 1) / bs;
  std::vector<int8_t> q((size_t)row * NTILE), zp((size_t)nblk * NTILE), s8((size_t)row * NTILE), tmp(4096);
  for (auto& v : q) v = (int8_t)((int)(rnd() % 16) - 8);
  for (auto& v : zp) v = (int8_t)((int)(rnd() % 16) - 8);
  std::vector<float> sf((size_t)nblk * NTILE);
  std::vector<utils::bf16> sb((size_t)nblk * NTILE);
  for (size_t i = 0; i < sf.size(); i++) {
    sf[i] = urand(-0.02f, 0.05f);
    sb[i] = utils::bf16(sf[i]);
  }
  std::vector<utils::int4x2> c((size_t)row * NTILE / 2);
  kernel::ref::compress_s8_s4(q.data(), c.data(), q.size());
  kernel::ref::decompress_kblock_s4_s8<PackRow, NTILE>(c.data(), zp.data(), s8.data(), bs, NTILE, 0, 0, row, NTILE,
                                                       tmp.data(), tmp.size());
  std::vector<float> out((size_t)row * NTILE);
  kernel::ref::decompress_kblock_s8_fp<PackRow, NTILE, float>(
      s8.data(), out.data(), row, NTILE, bf16scale ? (void*)sb.data() : (void*)sf.data(),
      bf16scale ? BTLA_DTYPE::BF16 : BTLA_DTYPE::F32, nullptr, 0, 0, bs, NTILE, tmp.data(), tmp.size());
  int meta[5] = {row, NTILE, PackRow, bs, bf16scale ? 1 : 0};
  dump(cs, "meta", "i4", meta, 5);
  dump(cs, "packed", "u1", reinterpret_cast<uint8_t*>(c.data()), c.size());
  dump(cs, "zp", "i1", zp.data(), zp.size());
  if (bf16scale)
    dump(cs, "scale_bf16", "u2", reinterpret_cast<uint16_t*>(sb.data()), sb.size());
  else
    dump(cs, "scale", "f4", sf.data(), sf.size());
  dump(cs, "s8", "i1", s8.data(), s8.size());
  dump(cs, "out", "f4", out.data(), out.size());
}

template <int PackRow, int NTILE>
static void case_dequant_s2(const char* cs, int row, int bs) {
  int nblk = (row + bs - 1) / bs;
  std::vector<int8_t> q((size_t)row * NTILE), zp((size_t)nblk * NTILE), s8((size_t)row * NTILE), tmp(4096);
  for (auto& v : q) v = (int8_t)((int)(rnd() % 4) - 2);
  for (auto& v : zp) v = (int8_t)((int)(rnd() % 4) - 2);
  std::vector<utils::bit2x4> c((size_t)row * NTILE / 4);
  kernel::ref::compress_2bit(q.data(), c.data(), q.size());
  kernel::ref::decompress_kblock_s2_s8<PackRow, NTILE>(c.data(), zp.data(), s8.data(), bs, NTILE, 0, 0, row, NTILE,
                                                       tmp.data(), tmp.size());
  int meta[4] = {row, NTILE, PackRow, bs};
  dump(cs, "meta", "i4", meta, 4);
  dump(cs, "packed", "u1", reinterpret_cast<uint8_t*>(c.data()), c.size());
  dump(cs, "zp", "i1", zp.data(), zp.size());
  dump(cs, "s8", "i1", s8.data(), s8.size());
}

// gemv_4bit_fp32_fp32 / gemv_2bit_fp32_fp32 on one PACK_ROW=1 stripe of NTILE columns
template <int NTILE, int MTILE>
static void case_gemv(const char* cs, int bits, int k, int bs, bool asym) {
  int nblk = k / bs;
  std::vector<int8_t> q((size_t)k * NTILE), zp((size_t)nblk * NTILE);
  for (auto& v : q) v = (int8_t)((int)(rnd() % (1u << bits)) - (1 << (bits - 1)));
  for (auto& v : zp) v = (int8_t)((int)(rnd() % (1u << bits)) - (1 << (bits - 1)));
  std::vector<float> s((size_t)nblk * NTILE), A((size_t)MTILE * k), C((size_t)MTILE * NTILE);
  for (auto& v : s) v = urand(0.001f, 0.05f);
  for (auto& v : A) v = urand(-0.5f, 0.5f);
  std::vector<uint8_t> packed((size_t)k * NTILE * bits / 8);
  if (bits == 4)
    kernel::ref::compress_s8_s4(q.data(), reinterpret_cast<utils::int4x2*>(packed.data()), q.size());
  else
    kernel::ref::compress_2bit(q.data(), reinterpret_cast<utils::bit2x4*>(packed.data()), q.size());
  utils::GemvParamB<float> B;
  if (bits == 4)
    B.b4ptr = packed.data();
  else
    B.b2ptr = packed.data();
  B.sptr = s.data();
  B.zpptr = asym ? zp.data() : nullptr;
  B.nbits = bits;
  B.ldzp = NTILE;
  B.kpad = k;
  std::vector<int8_t> tmp(16384);
  if (bits == 4)
    kernel::ref::gemv_4bit_fp32_fp32<float, NTILE, MTILE>(A.data(), k, B, C.data(), NTILE, k, bs, tmp.data(),
                                                          tmp.size());
  else
    kernel::ref::gemv_2bit_fp32_fp32<float, NTILE, MTILE>(A.data(), k, B, C.data(), NTILE, k, bs, tmp.data(),
                                                          tmp.size());
  int meta[6] = {bits, k, bs, NTILE, MTILE, asym ? 1 : 0};
  dump(cs, "meta", "i4", meta, 6);
  dump(cs, "packed", "u1", packed.data(), packed.size());
  dump(cs, "scale", "f4", s.data(), s.size());
  if (asym) dump(cs, "zp", "i1", zp.data(), zp.size());
  dump(cs, "A", "f4", A.data(), A.size());
  dump(cs, "C", "f4", C.data(), C.size());
}

static void case_convert(const char* cs) {
  std::vector<float> v;
  float specials[] = {0.f,     -0.f,       1.f,        -1.f,    65504.f, 70000.f, 1e-8f, 6.1035156e-5f,
                      3e-5f,   -3e-5f,     0.33333334f, 1.0009765625f, 1.00048828125f, 2.0009765625f,
                      1e-3f,   0.0625f,    -0.0078125f, 123.456f};
  for (float f : specials) v.push_back(f);
  for (int i = 0; i < 4000; i++) {
    float mag = urand(-20.f, 12.f);
    float x = std::ldexp(urand(1.f, 2.f), (int)mag);
    if (rnd() & 1) x = -x;
    v.push_back(x);
  }
  std::vector<uint16_t> bf(v.size()), fh(v.size());
  std::vector<float> bf_back(v.size()), fh_back(v.size());
  for (size_t i = 0; i < v.size(); i++) {
    utils::bf16 b(v[i]);
    bf[i] = b.x;
    bf_back[i] = b.tofloat();
    utils::fp16 h(v[i]);
    fh[i] = h.x;
    fh_back[i] = static_cast<float>(h);
  }
  dump(cs, "f32", "f4", v.data(), v.size());
  dump(cs, "bf16", "u2", bf.data(), bf.size());
  dump(cs, "bf16_back", "f4", bf_back.data(), bf_back.size());
  dump(cs, "fp16", "u2", fh.data(), fh.size());
  dump(cs, "fp16_back", "f4", fh_back.data(), fh_back.size());
}

// kernel_ref.h:1824-1883 quantize_fp_u8_colblock (int8-compute activation quantizer)
static void case_quant_u8(const char* cs, int row, int col, int bs, float amp) {
  std::vector<float> src((size_t)row * col);
  for (auto& v : src) v = urand(-amp, amp);
  if (col >= 3 * bs) {  // row 0: an all-zero block, an all-positive block, an all-negative block
    for (int j = 0; j < bs; j++) src[j] = 0.f;
    for (int j = bs; j < 2 * bs; j++) src[j] = urand(0.1f, amp);
    for (int j = 2 * bs; j < 3 * bs; j++) src[j] = urand(-amp, -0.1f);
  }
  int nblk = (col + bs - 1) / bs;
  std::vector<uint8_t> q((size_t)row * col), zp((size_t)row * nblk);
  std::vector<float> s((size_t)row * nblk), red((size_t)row * nblk);
  kernel::ref::quantize_fp_u8_colblock<float>(row, col, src.data(), col, q.data(), col, s.data(), nblk, zp.data(), bs,
                                              red.data());
  int meta[3] = {row, col, bs};
  dump(cs, "meta", "i4", meta, 3);
  dump(cs, "src", "f4", src.data(), src.size());
  dump(cs, "q", "u1", q.data(), q.size());
  dump(cs, "s", "f4", s.data(), s.size());
  dump(cs, "zp", "u1", zp.data(), zp.size());
  dump(cs, "red", "f4", red.data(), red.size());
}

// kernel_ref.h:2371-2429 gemv_4bit_u8s8_fp32 on a PACK_ROW 4 stripe, activation quantized by quantize_fp_u8_colblock
template <int NTILE, int MTILE>
static void case_gemv_u8s8(const char* cs, int k, int bs, bool asym) {
  int nblk = k / bs;
  std::vector<int8_t> q((size_t)k * NTILE), zp((size_t)nblk * NTILE), qp((size_t)k * NTILE);
  for (auto& v : q) v = (int8_t)((int)(rnd() % 16u) - 8);
  for (auto& v : zp) v = (int8_t)((int)(rnd() % 16u) - 8);
  for (int kk = 0; kk < k; kk++)  // [k/4][NTILE][4]
    for (int n = 0; n < NTILE; n++) qp[(size_t)(kk / 4) * NTILE * 4 + n * 4 + kk % 4] = q[(size_t)kk * NTILE + n];
  std::vector<float> s((size_t)nblk * NTILE), A((size_t)MTILE * k), C((size_t)MTILE * NTILE);
  for (auto& v : s) v = urand(0.001f, 0.05f);
  for (auto& v : A) v = urand(-0.5f, 0.5f);
  std::vector<uint8_t> a8((size_t)MTILE * k), azp((size_t)MTILE * nblk);
  std::vector<float> as((size_t)MTILE * nblk);
  kernel::ref::quantize_fp_u8_colblock<float>(MTILE, k, A.data(), k, a8.data(), k, as.data(), nblk, azp.data(), bs,
                                              nullptr);
  std::vector<uint8_t> packed((size_t)k * NTILE / 2);
  kernel::ref::compress_s8_s4(qp.data(), reinterpret_cast<utils::int4x2*>(packed.data()), qp.size());
  utils::GemvParamA PA{a8.data(), as.data(), azp.data(), k, nblk};
  utils::GemvParamB<float> B;
  B.b4ptr = packed.data();
  B.sptr = s.data();
  B.zpptr = asym ? zp.data() : nullptr;
  B.nbits = 4;
  B.ldzp = NTILE;
  B.kpad = k;
  std::vector<int8_t> tmp(16384);
  kernel::ref::gemv_4bit_u8s8_fp32<float, NTILE, MTILE>(PA, B, C.data(), NTILE, k, bs, tmp.data(), tmp.size());
  int meta[6] = {4, k, bs, NTILE, MTILE, asym ? 1 : 0};
  dump(cs, "meta", "i4", meta, 6);
  dump(cs, "A", "f4", A.data(), A.size());
  dump(cs, "a8", "u1", a8.data(), a8.size());
  dump(cs, "as", "f4", as.data(), as.size());
  dump(cs, "azp", "u1", azp.data(), azp.size());
  dump(cs, "q", "i1", q.data(), q.size());
  dump(cs, "scale", "f4", s.data(), s.size());
  if (asym) dump(cs, "zp", "i1", zp.data(), zp.size());
  dump(cs, "C", "f4", C.data(), C.size());
}

// kernel_ref.h:178-341 compress_{7,6,5,3}bit (plane layouts as compressBitNWeight, bestla_prologue_b.h:512-546) and
// :448-520 decompress_s{7,6,5,3}_s8
static void case_compress_planes(const char* cs, size_t n) {
  std::vector<int8_t> tmp(64);
  for (int bits : {3, 5, 6, 7}) {
    std::vector<int8_t> src(n), dec(n);
    const int full = 1 << (bits - 1);
    for (auto& v : src) v = (int8_t)((int)(rnd() % (2u * full)) - full);
    std::vector<uint8_t> packed(n * bits / 8);
    auto* u8 = packed.data();
    if (bits == 3) {
      auto* b2 = reinterpret_cast<utils::bit2x4*>(u8);
      auto* b1 = reinterpret_cast<utils::bit1x8*>(u8 + n / 4);
      kernel::ref::compress_3bit(src.data(), b2, b1, n);
      kernel::ref::decompress_s3_s8(b2, b1, dec.data(), n, tmp.data(), tmp.size());
    } else if (bits == 5) {
      auto* b4 = reinterpret_cast<utils::bit4x2*>(u8);
      auto* b1 = reinterpret_cast<utils::bit1x8*>(u8 + n / 2);
      kernel::ref::compress_5bit(src.data(), b4, b1, n);
      kernel::ref::decompress_s5_s8(b4, b1, dec.data(), n, tmp.data(), tmp.size());
    } else if (bits == 6) {
      auto* b4 = reinterpret_cast<utils::bit4x2*>(u8);
      auto* b2 = reinterpret_cast<utils::bit2x4*>(u8 + n / 2);
      kernel::ref::compress_6bit(src.data(), b4, b2, n);
      kernel::ref::decompress_s6_s8(b4, b2, dec.data(), n, tmp.data(), tmp.size());
    } else {
      auto* b4 = reinterpret_cast<utils::bit4x2*>(u8);
      auto* b2 = reinterpret_cast<utils::bit2x4*>(u8 + n / 2);
      auto* b1 = reinterpret_cast<utils::bit1x8*>(u8 + n / 2 + n / 4);
      kernel::ref::compress_7bit(src.data(), b4, b2, b1, n);
      kernel::ref::decompress_s7_s8(b4, b2, b1, dec.data(), n, tmp.data(), tmp.size());
    }
    std::string b = std::to_string(bits);
    dump(cs, "s" + b, "i1", src.data(), n);
    dump(cs, "c" + b, "u1", packed.data(), packed.size());
    dump(cs, "d" + b, "i1", dec.data(), n);
  }
}

// kernel_ref.h:343-361 compress_1bit / :511-525 decompress_s1_s8 (S1_CLIP, one bit plane).  compress_1bit reads
// element 4 of every 8 from srcptr[j + FullRange] = srcptr[j + 1]: the golden records what the reference stores.
static void case_compress_bit1(const char* cs, size_t n) {
  std::vector<int8_t> tmp(64), src(n), dec(n);
  for (auto& v : src) v = (int8_t)((int)(rnd() % 2u) - 1);
  std::vector<uint8_t> packed(n / 8);
  auto* b1 = reinterpret_cast<utils::bit1x8*>(packed.data());
  kernel::ref::compress_1bit(src.data(), b1, n);
  kernel::ref::decompress_s1_s8(b1, dec.data(), n, tmp.data(), tmp.size());
  dump(cs, "s1", "i1", src.data(), n);
  dump(cs, "c1", "u1", packed.data(), packed.size());
  dump(cs, "d1", "i1", dec.data(), n);
}

// NFloat 4-bit: kernel_ref.h:1800-1822 quantize_f32_f4_rowblock, f4_dequantize (the unpack trees) and the
// bestla_utils.h:749-790 LUTs the SIMD kernels use
template <BTLA_DTYPE F4_T>
static void case_f4(const char* cs, int row, int col, int bs, const float* lut) {
  std::vector<float> src((size_t)row * col);
  for (auto& v : src) v = urand(-1.f, 1.f);
  for (int r = 0; r < bs && r < row; r++) src[(size_t)r * col] = 0.f;  // an all-zero block
  int nblk = (row + bs - 1) / bs;
  std::vector<int8_t> q((size_t)row * col);
  std::vector<float> s((size_t)nblk * col), deq((size_t)row * col), lutv(lut, lut + 16), tree(16);
  kernel::ref::quantize_f32_f4_rowblock<F4_T>(src.data(), q.data(), row, col, col, col, s.data(), bs);
  for (int r = 0; r < row; r++)
    for (int c = 0; c < col; c++)
      deq[(size_t)r * col + c] = kernel::ref::f4_dequantize<F4_T>(q[(size_t)r * col + c], s[(size_t)(r / bs) * col + c]);
  for (int code = 0; code < 16; code++) tree[code] = kernel::ref::f4_unpack<F4_T>((int8_t)code);
  int meta[3] = {row, col, bs};
  dump(cs, "meta", "i4", meta, 3);
  dump(cs, "src", "f4", src.data(), src.size());
  dump(cs, "q", "i1", q.data(), q.size());
  dump(cs, "s", "f4", s.data(), s.size());
  dump(cs, "deq", "f4", deq.data(), deq.size());
  dump(cs, "lut", "f4", lutv.data(), 16);
  dump(cs, "tree", "f4", tree.data(), 16);
}

// NFloat 8-bit: kernel_ref.h:1764-1800 quantize_f32_f8_rowblock_mxscale and :984-1001 f8_to_fp32 (all 256 codes)
template <BTLA_DTYPE F8_T>
static void case_f8(const char* cs, int row, int col, int bs, BTLA_DTYPE sdt, float amp) {
  std::vector<float> src((size_t)row * col);
  for (auto& v : src) v = urand(-amp, amp);
  for (int r = 0; r < bs && r < row; r++) src[(size_t)r * col] = 0.f;  // an all-zero block
  if (col > 1) src[1] = 1e-30f;                                        // an underflowing value
  int nblk = (row + bs - 1) / bs;
  std::vector<int8_t> q((size_t)row * col);
  std::vector<float> s((size_t)nblk * col), dec(256);
  kernel::ref::quantize_f32_f8_rowblock_mxscale<F8_T>(src.data(), q.data(), row, col, col, col, s.data(), bs, sdt);
  for (int c = 0; c < 256; c++) dec[c] = kernel::ref::f8_to_fp32(utils::f8((int8_t)c), F8_T);
  int meta[4] = {row, col, bs, sdt == BTLA_DTYPE::F8_E8M0 ? 1 : 0};
  dump(cs, "meta", "i4", meta, 4);
  dump(cs, "src", "f4", src.data(), src.size());
  dump(cs, "q", "i1", q.data(), q.size());
  dump(cs, "s", "f4", s.data(), s.size());
  dump(cs, "dec", "f4", dec.data(), 256);
}

// kernel_ref.h:2199-2240 layernorm<float> as BTLALayerNorm drives it (bestla_gemm.cpp:751-776: no scale / bias,
// simplified = isrms), one row at a time -- the reference of bestla_layernormalization (ne_bestla.cpp:113-116)
static void case_layernorm(const char* cs, int rows, int size, bool isrms, float eps, float amp, float offset) {
  std::vector<float> src((size_t)rows * size), dst((size_t)rows * size);
  for (auto& v : src) v = offset + urand(-amp, amp);
  for (int r = 0; r < rows; r++)
    kernel::ref::layernorm<float>(src.data() + (size_t)r * size, nullptr, nullptr, eps, size,
                                  dst.data() + (size_t)r * size, nullptr, nullptr, isrms);
  int meta[3] = {rows, size, isrms ? 1 : 0};
  dump(cs, "meta", "i4", meta, 3);
  dump(cs, "eps", "f4", &eps, 1);
  dump(cs, "src", "f4", src.data(), src.size());
  dump(cs, "dst", "f4", dst.data(), dst.size());
}

// DQ8_BNB double-quantized scales: the int4 sym scales of a [row][col] weight ([nblk][col], the ssize = N * nk_scale
// array packQWeight hands over, bestla_prologue_b.h:381-386) through kernel_ref.h:1952-1979 dq8_bnb_double_quant
// into u8 codes + dq_buf (zero-initialised like the avector doubleQuantScale resizes), and back through :1981-1991
// dq8_get_fp_scale with the offset read from the buffer's last slot (getScale, bestla_prologue_b.h:699-706)
static void case_dq8(const char* cs, int row, int col, int bs, int dq_blk, float amp) {
  std::vector<float> src((size_t)row * col);
  for (auto& v : src) v = urand(-amp, amp);
  int nblk = (row + bs - 1) / bs;
  std::vector<int8_t> q((size_t)row * col);
  std::vector<float> s((size_t)nblk * col);
  kernel::ref::quantize_f32_sign_int_rowblock(src.data(), q.data(), row, col, col, col, s.data(), nullptr, bs,
                                              BTLA_DTYPE::S4_CLIP);
  const size_t ssize = s.size(), nd = utils::updiv(ssize, (size_t)dq_blk) + 1;
  std::vector<float> work(s), dq(nd, 0.f), dec(ssize), lut(dq8_bnb_LUT, dq8_bnb_LUT + 256);
  kernel::ref::dq8_bnb_double_quant<false>(work.data(), ssize, dq_blk, dq.data());
  std::vector<uint8_t> code(ssize);
  for (size_t i = 0; i < ssize; i++) code[i] = static_cast<uint8_t>(work[i]);  // setQuantCorrection DQ8 (:313-329)
  kernel::ref::dq8_get_fp_scale(code.data(), dec.data(), nblk, col, 0, dq_blk, (int)(nd - 1), dq.data(), col, col,
                                false, col);
  int meta[4] = {row, col, bs, dq_blk};
  dump(cs, "meta", "i4", meta, 4);
  dump(cs, "s", "f4", s.data(), ssize);
  dump(cs, "code", "u1", code.data(), ssize);
  dump(cs, "dq", "f4", dq.data(), nd);
  dump(cs, "dec", "f4", dec.data(), ssize);
  dump(cs, "lut", "f4", lut.data(), 256);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <outdir>\n", argv[0]);
    return 2;
  }
  g_dir = argv[1];
  g_man = fopen((g_dir + "/manifest.txt").c_str(), "w");
  if (!g_man) return 3;
  case_quant("quant_s4_sym_g32", 128, 37, 32, BTLA_DTYPE::S4_CLIP, false, 1);
  case_quant("quant_s4_asym_g32", 128, 37, 32, BTLA_DTYPE::S4_CLIP, true, 1);
  case_quant("quant_s4_sym_g128_ragged", 300, 19, 128, BTLA_DTYPE::S4_CLIP, false, 0);
  case_quant("quant_s4_asym_g128_ragged", 300, 19, 128, BTLA_DTYPE::S4_CLIP, true, 0);
  case_quant("quant_s2_sym_g64", 256, 21, 64, BTLA_DTYPE::S2_CLIP, false, 1);
  case_quant("quant_s2_asym_g64", 256, 21, 64, BTLA_DTYPE::S2_CLIP, true, 1);
  case_quant("quant_s8_sym_g16", 96, 13, 16, BTLA_DTYPE::S8, false, 1);
  case_quant("quant_s8_asym_g128", 256, 13, 128, BTLA_DTYPE::S8, true, 0);
  case_quant("quant_s4_sym_perchannel", 200, 11, 200, BTLA_DTYPE::S4_CLIP, false, 0);
  case_interleave("ilv_n48_p1", 70, 100, 48, 1);
  case_interleave("ilv_n48_p4", 70, 100, 48, 4);
  case_interleave("ilv_n48_p2", 70, 100, 48, 2);
  case_interleave("ilv_n24_p1", 33, 50, 24, 1);
  case_interleave("ilv_n24_p4", 33, 50, 24, 4);
  case_compress("compress", 4096);
  case_dequant_s4<1, 48>("deq_s4_p1_n48_f32", 256, 32, false);
  case_dequant_s4<4, 48>("deq_s4_p4_n48_bf16", 256, 64, true);
  case_dequant_s4<2, 48>("deq_s4_p2_n48_f32", 128, 32, false);
  case_dequant_s2<1, 48>("deq_s2_p1_n48", 256, 64);
  case_dequant_s2<4, 48>("deq_s2_p4_n48", 256, 64);
  case_gemv<48, 1>("gemv_s4_m1_sym", 4, 512, 128, false);
  case_gemv<48, 4>("gemv_s4_m4_asym", 4, 512, 32, true);
  case_gemv<48, 2>("gemv_s2_m2_sym", 2, 512, 64, false);
  case_gemv<48, 1>("gemv_s2_m1_asym", 2, 256, 64, true);
  case_convert("convert");
  case_compress_planes("compress_planes", 4096);
  case_quant("quant_s3_sym_g32", 128, 37, 32, BTLA_DTYPE::S3_CLIP, false, 1);
  case_quant("quant_s3_asym_g128", 256, 19, 128, BTLA_DTYPE::S3_CLIP, true, 0);
  case_quant("quant_s5_sym_g32", 96, 13, 32, BTLA_DTYPE::S5_CLIP, false, 1);
  case_quant("quant_s6_asym_g64", 128, 13, 64, BTLA_DTYPE::S6_CLIP, true, 0);
  case_quant("quant_s7_sym_g128", 256, 11, 128, BTLA_DTYPE::S7_CLIP, false, 0);
  case_quant_u8("qu8_g32", 7, 256, 32, 0.5f);
  case_quant_u8("qu8_g128_tail", 5, 300, 128, 3.0f);
  case_quant_u8("qu8_perchannel", 4, 200, 4096, 1.0f);
  case_quant_u8("qu8_g64_big", 3, 512, 64, 1000.f);
  case_gemv_u8s8<48, 1>("gemv_u8s8_m1_sym", 512, 128, false);
  case_gemv_u8s8<48, 4>("gemv_u8s8_m4_asym", 512, 32, true);
  case_f4<BTLA_DTYPE::F4_BNB>("f4_bnb_g32", 128, 19, 32, fp4_bnb_dequant_fp32_LUT);
  case_f4<BTLA_DTYPE::F4_E2M1>("f4_e2m1_g64", 192, 13, 64, fp4_e2m1_dequant_fp32_LUT);
  case_f4<BTLA_DTYPE::F4_NF4>("f4_nf4_g32", 128, 17, 32, nf4_dequant_fp32_LUT);
  case_f4<BTLA_DTYPE::F4_NF4>("f4_nf4_perchannel", 100, 7, 100, nf4_dequant_fp32_LUT);
  case_f8<BTLA_DTYPE::F8_E4M3>("f8_e4m3_e8m0_g32", 128, 11, 32, BTLA_DTYPE::F8_E8M0, 3.f);
  case_f8<BTLA_DTYPE::F8_E5M2>("f8_e5m2_e8m0_g64", 128, 9, 64, BTLA_DTYPE::F8_E8M0, 100.f);
  case_f8<BTLA_DTYPE::F8_E4M3>("f8_e4m3_f32_g32", 96, 7, 32, BTLA_DTYPE::F32, 0.5f);
  case_f8<BTLA_DTYPE::F8_E5M2>("f8_e5m2_f32_g128", 256, 5, 128, BTLA_DTYPE::F32, 1.f);
  case_compress_bit1("compress_bit1", 4096);
  case_quant("quant_s1_sym_g32", 128, 37, 32, BTLA_DTYPE::S1_CLIP, false, 1);
  case_quant("quant_s1_asym_g64", 128, 13, 64, BTLA_DTYPE::S1_CLIP, true, 0);
  case_layernorm("layernorm_rms_4096", 5, 4096, true, 1e-5f, 2.f, 0.f);
  case_layernorm("layernorm_ln_300", 7, 300, false, 1e-6f, 1.f, 0.75f);
  case_layernorm("layernorm_rms_11008", 2, 11008, true, 1e-6f, 40.f, 0.f);
  case_layernorm("layernorm_ln_4096", 3, 4096, false, 1e-5f, 3.f, -1.5f);
  case_dq8("dq8_g32", 256, 40, 32, 32, 0.5f);           // 8 x 40 scales, dq blocks of 32: 10 full blocks
  case_dq8("dq8_g128_ragged", 384, 21, 128, 128, 2.f);  // 63 scales in one partial dq block (the :1978 slot quirk)
  case_dq8("dq8_g64_tail", 512, 100, 64, 64, 1.f);      // 800 scales = 12 full blocks + a 32-scale tail
  fclose(g_man);
  return 0;
}
