// btla_format.cpp -- bit-exact reader/writer/packer for Neural Speed's BTLA weight blobs (host side).
// Compiled with g++ -ffp-contract=off: the quantizer must round exactly like the reference's scalar code.
#include "btla_format.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

namespace nad {

namespace {

template <typename F>
void parallel_for(int n, F&& f) {
  int hw = int(std::thread::hardware_concurrency());
  const char* env = std::getenv("NAD_HOST_THREADS");
  if (env) hw = std::atoi(env);
  int nth = std::max(1, std::min({hw, n, 32}));
  if (nth <= 1) {
    for (int i = 0; i < n; i++) f(i);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nth);
  for (int t = 0; t < nth; t++)
    th.emplace_back([&, t]() {
      for (int i = t; i < n; i += nth) f(i);
    });
  for (auto& x : th) x.join();
}

inline size_t updiv(size_t a, size_t b) { return (a + b - 1) / b; }
inline size_t padto(size_t a, size_t b) { return updiv(a, b) * b; }

struct Writer {
  int8_t* p;
  template <typename T>
  void put(T v) {
    std::memcpy(p, &v, sizeof(T));
    p += sizeof(T);
  }
};
struct Reader {
  const int8_t* p;
  template <typename T>
  T get() {
    T v;
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
};

// ObjectAlignedBuffer<64> (bestla_storage.h:59-110): {size, offset-to-64B-boundary, pad, bytes}
uint64_t put_aligned(Writer& w, const int8_t* base, uint64_t bytes) {
  w.put<uint64_t>(bytes);
  uintptr_t tmp = reinterpret_cast<uintptr_t>(w.p + sizeof(uint64_t));
  uint64_t off = ((tmp + 63) / 64) * 64 - tmp;
  w.put<uint64_t>(off);
  w.p += off;
  uint64_t at = uint64_t(w.p - base);
  w.p += bytes;
  return at;
}
uint64_t get_aligned(Reader& r, const int8_t* base, uint64_t* bytes) {
  *bytes = r.get<uint64_t>();
  uint64_t off = r.get<uint64_t>();
  r.p += off;
  uint64_t at = uint64_t(r.p - base);
  r.p += *bytes;
  return at;
}

// std::min/std::max argument-order semantics, and x86 cvttss2si for float->int (NaN/overflow -> INT_MIN)
inline float smax(float a, float b) { return (a < b) ? b : a; }
inline float smin(float a, float b) { return (b < a) ? b : a; }
inline int32_t f2i(float x) {
  if (std::isnan(x) || x >= 2147483648.0f || x < -2147483648.0f) return std::numeric_limits<int32_t>::min();
  return int32_t(x);
}
inline int32_t wrap_add(int32_t a, int32_t b) { return int32_t(uint32_t(a) + uint32_t(b)); }

}  // namespace

// ----------------------------------------------------------------------------------------------- cores
static uint64_t make_core(int ntile, int packrow, int comp, int isa) {
  return uint64_t(ntile) | (uint64_t(packrow) << 8) | (uint64_t(comp) << 16) | (uint64_t(isa) << 32);
}

uint64_t core_id_by_name(const std::string& s) {
  // typedefs of neural_speed/core/layers/bestla_defs.h:36-54; ISA ids bestla.h:23-36; CompType bestla_gemm.h:22-50
  if (s == "avx2") return make_core(24, 1, 0x000, 2);
  if (s == "avx512f") return make_core(48, 1, 0x000, 4);
  if (s == "amx_bf16") return make_core(48, 2, 0x011, 9);
  if (s == "amx_fp16") return make_core(48, 2, 0x022, 11);
  if (s == "avx512_vnni_kblock") return make_core(48, 4, 0x034, 6);
  if (s == "avx512bw_kblock") return make_core(48, 4, 0x034, 5);
  if (s == "avx_vnni_kblock") return make_core(24, 4, 0x034, 3);
  if (s == "avx2_vnni_kblock") return make_core(24, 4, 0x034, 2);
  if (s == "amx_int8_kblock") return make_core(48, 4, 0x034, 10);
  if (s == "amx_int8_ss_kblock") return make_core(48, 4, 0x033, 10);
  return 0;
}

CoreInfo core_info(uint64_t id) {
  CoreInfo c;
  c.ntile = int(id & 0xff);
  c.packrow = int((id >> 8) & 0xff);
  int comp = int((id >> 16) & 0xffff);
  int isa = int((id >> 32) & 0xff);
  int bt = (comp >> 4) & 0xf;  // CompTypeHelper::get_B
  c.int_comp = (bt == 3 || bt == 4);
  if (c.packrow == 1)
    c.ktile = 1;  // Avx2N8P1 / Avx512fN16P1
  else if (isa == 9 || isa == 11)
    c.ktile = 32;  // Amx{bf16,fp16}N16P2
  else if (isa == 10)
    c.ktile = 64;  // Amxint8N16P4
  else
    c.ktile = 4;  // VNNI / BW kblock cores
  return c;
}

int host_isa_profile() {
  const char* e = std::getenv("NAD_HOST_ISA");
  if (!e) return 0;
  std::string s(e);
  if (s == "avx512_vnni") return 1;
  if (s == "avx512f") return 2;
  if (s == "avx2") return 3;
  return 0;
}

uint64_t select_core(int comp, uint32_t qtype, int bs, bool asym, int profile) {
  const bool amx = profile == 0, vnni = profile <= 1, a512 = profile <= 2;
  switch (comp) {
    case kCompInt8:
      if (dtype_is_int(qtype) && !(qtype == kS8 && asym)) {
        if (amx && bs % 64 == 0) return core_id_by_name("amx_int8_kblock");
        if (vnni && bs % 4 == 0) return core_id_by_name("avx512_vnni_kblock");
        if (a512 && bs % 4 == 0) return core_id_by_name("avx512bw_kblock");
        if (bs % 4 == 0) return core_id_by_name("avx2_vnni_kblock");
      }
      [[fallthrough]];
    case kCompBF16:
      if (amx && bs % 32 == 0) return core_id_by_name("amx_bf16");
      [[fallthrough]];
    case kCompF16:  // no AMX-FP16 on the emulated profiles
    case kCompF32:
    case kCompUndef:
      return a512 ? core_id_by_name("avx512f") : core_id_by_name("avx2");
    default:
      return 0;
  }
}

// ----------------------------------------------------------------------------------------------- blob
Blob Blob::describe(int n, int k, int blocksize, uint32_t qtype, uint32_t scale_t, bool asym, uint64_t core_id,
                    bool shuffle) {
  Blob b;
  CoreInfo ci = core_info(core_id);
  b.core_id = core_id;
  b.n = n;
  b.k = k;
  b.kpad = int(padto(size_t(k), size_t(ci.ktile)));
  b.npad = int(padto(size_t(n), size_t(ci.ntile)));
  b.blocksize = blocksize <= 0 ? b.kpad : blocksize;
  b.qtype = qtype;
  b.scale_t = scale_t;
  const bool f4 = f4_kind(qtype) >= 0 || is_f8(qtype);  // StorageWeightKBlockNFloat (bestla_storage.h:836-859)
  b.prologue = f4 ? 2 : 1;
  b.zp_t = f4 ? 0 : kS8;
  b.red_t = f4 ? 0 : kBF16;
  if (f4) asym = false;
  b.asym = asym;
  b.has_reduce = ci.int_comp && !f4;
  b.has_shuffle = shuffle;
  b.q_size = updiv(uint64_t(b.npad) * b.kpad * dtype_bits(qtype), 8);
  b.cstep = b.npad;
  b.csize = uint64_t(b.ngroups()) * b.npad;
  b.s_size = b.csize * b.scale_bytes();
  b.z_size = asym ? b.csize : 0;
  b.r_size = b.has_reduce ? b.csize * 2 : 0;
  b.shf_size = shuffle ? uint64_t(k) * 4 : 0;
  if (scale_t == kDQ8_BNB) {  // resize -> initDoubleQuantBlkSize(Block, ...) (bestla_storage.h:750-758)
    b.has_dq = true;
    b.dq_blocksize = b.blocksize;
    b.dq_size = (updiv(uint64_t(b.ngroups()) * n, uint64_t(b.dq_blocksize)) + 1) * 4;
  }
  // update_size(): every aligned buffer is charged size + 16 + 64, optional ones + 1 flag byte
  uint64_t sz = 48 + (16 + b.q_size + 64) + 24 + (16 + b.s_size + 64);
  sz += 1 + (asym ? 16 + b.z_size + 64 : 0);
  sz += 1 + (b.has_reduce ? 16 + b.r_size + 64 : 0);
  sz += 1 + (b.has_dq ? 16 + b.dq_size + 64 : 0);
  sz += 1 + (shuffle ? 16 + b.shf_size + 64 : 0);
  b.size = padto(sz, 64);
  return b;
}

void Blob::write_header(int8_t* base) {
  Writer w{base};
  w.put<uint64_t>(size);
  w.put<uint32_t>(prologue);
  w.put<uint64_t>(core_id);
  w.put<int32_t>(npad);
  w.put<int32_t>(kpad);
  w.put<int32_t>(n);
  w.put<int32_t>(k);
  w.put<uint32_t>(qtype);
  w.put<int32_t>(blocksize);
  w.put<int32_t>(dq_blocksize);
  q_off = put_aligned(w, base, q_size);
  w.put<uint32_t>(scale_t);
  w.put<uint32_t>(zp_t);
  w.put<uint32_t>(red_t);
  w.put<int32_t>(cstep);
  w.put<uint64_t>(csize);
  s_off = put_aligned(w, base, s_size);
  w.put<uint8_t>(asym ? 1 : 0);
  if (asym) z_off = put_aligned(w, base, z_size);
  w.put<uint8_t>(has_reduce ? 1 : 0);
  if (has_reduce) r_off = put_aligned(w, base, r_size);
  w.put<uint8_t>(has_dq ? 1 : 0);
  if (has_dq) dq_off = put_aligned(w, base, dq_size);
  w.put<uint8_t>(has_shuffle ? 1 : 0);
  if (has_shuffle) shf_off = put_aligned(w, base, shf_size);
}

bool Blob::parse(const void* buf, std::string* err) {
  auto fail = [&](const char* m) {
    if (err) *err = m;
    return false;
  };
  if (!buf) return fail("null blob");
  const int8_t* base = static_cast<const int8_t*>(buf);
  Reader r{base};
  size = r.get<uint64_t>();
  prologue = r.get<uint32_t>();
  if (prologue != 1 && prologue != 2)
    return fail("only WeightKBlockNInteger / WeightKBlockNFloat blobs (N-bit integer or 4-bit float weights) are supported");
  core_id = r.get<uint64_t>();
  npad = r.get<int32_t>();
  kpad = r.get<int32_t>();
  n = r.get<int32_t>();
  k = r.get<int32_t>();
  qtype = r.get<uint32_t>();
  blocksize = r.get<int32_t>();
  dq_blocksize = r.get<int32_t>();
  if (n <= 0 || k <= 0 || npad < n || kpad < k || blocksize <= 0) return fail("corrupt blob header");
  q_off = get_aligned(r, base, &q_size);
  scale_t = r.get<uint32_t>();
  zp_t = r.get<uint32_t>();
  red_t = r.get<uint32_t>();
  cstep = r.get<int32_t>();
  csize = r.get<uint64_t>();
  s_off = get_aligned(r, base, &s_size);
  asym = r.get<uint8_t>() != 0;
  if (asym) z_off = get_aligned(r, base, &z_size);
  has_reduce = r.get<uint8_t>() != 0;
  if (has_reduce) r_off = get_aligned(r, base, &r_size);
  has_dq = r.get<uint8_t>() != 0;
  if (has_dq) dq_off = get_aligned(r, base, &dq_size);
  has_shuffle = r.get<uint8_t>() != 0;
  if (has_shuffle) shf_off = get_aligned(r, base, &shf_size);
  if (prologue == 2) {
    if (f4_kind(qtype) < 0 && !is_f8(qtype))
      return fail("NFloat weight dtype must be F4_BNB, F4_E2M1, F4_NF4, F8_E4M3 or F8_E5M2");
  } else if (!dtype_is_int(qtype) || dtype_bits(qtype) < 1 || dtype_bits(qtype) > 8) {
    return fail("weight dtype must be an integer type S1_CLIP .. S8");
  }
  if (scale_t == kDQ8_BNB || has_dq) {  // IsDoubleQuant(): sym integer or NF4 weights (bestla_prologue_b.h:170-176)
    if (scale_t != kDQ8_BNB || !has_dq) return fail("DQ8_BNB scales without their double-quant buffer (or vice versa)");
    if (asym) return fail("DQ8_BNB scales are symmetric only");
    if (!dtype_is_int(qtype) && qtype != kF4NF4) return fail("DQ8_BNB scales go with integer or F4_NF4 weights");
    if (dq_blocksize <= 0 || dq_blocksize % 8 || dq_size / 4 < updiv(uint64_t(ngroups()) * n, uint64_t(dq_blocksize)) + 1)
      return fail("corrupt DQ8_BNB double-quant buffer");
  } else if (scale_t != kF32 && scale_t != kBF16 && scale_t != kF16 && !(scale_t == kF8E8M0 && is_f8(qtype))) {
    return fail("scale dtype must be F32, BF16, F16 or DQ8_BNB (F8_E8M0 with F8 weights)");
  }
  CoreInfo ci = core_info(core_id);
  if (ci.ntile <= 0 || (ci.packrow != 1 && ci.packrow != 2 && ci.packrow != 4)) return fail("unknown core id");
  if (npad % ci.ntile || kpad % ci.packrow) return fail("blob padding does not match its core");
  return true;
}

// ----------------------------------------------------------------------------------------------- scales
uint16_t f32_to_bf16_rne(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}
float bf16_to_f32(uint16_t x) {
  uint32_t u = uint32_t(x) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
uint16_t f32_to_f16_rne(float v) {
  uint32_t x;
  std::memcpy(&x, &v, 4);
  uint32_t sign = (x >> 16) & 0x8000u, ax = x & 0x7FFFFFFFu;
  if (ax > 0x7F800000u) return uint16_t(sign | 0x7E00u | ((ax >> 13) & 0x3FFu));
  if (ax >= 0x477FF000u) return uint16_t(sign | 0x7C00u);
  if (ax < 0x38800000u) {
    if (ax < 0x33000000u) return uint16_t(sign);
    uint32_t e = ax >> 23, mant = (ax & 0x7FFFFFu) | 0x800000u, sh = 126 - e;
    uint32_t q = mant >> sh, rem = mant & ((1u << sh) - 1), half = 1u << (sh - 1);
    if (rem > half || (rem == half && (q & 1u))) q++;
    return uint16_t(sign | q);
  }
  uint32_t q = (((ax >> 23) - 112) << 10) | ((ax & 0x7FFFFFu) >> 13), rem = ax & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (q & 1u))) q++;
  return uint16_t(sign | q);
}
float f16_to_f32(uint16_t h) {
  uint32_t sign = uint32_t(h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff, u;
  if (e == 0) {
    if (m == 0) {
      u = sign;
    } else {  // subnormal: normalise
      int sh = 0;
      while (!(m & 0x400)) {
        m <<= 1;
        sh++;
      }
      u = sign | (uint32_t(113 - sh) << 23) | ((m & 0x3ff) << 13);
    }
  } else if (e == 31) {
    u = sign | 0x7F800000u | (m << 13);
  } else {
    u = sign | ((e + 112) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

static inline void store_scale(uint8_t* sp, size_t i, uint32_t t, float v) {
  if (t == kF8E8M0) {  // setQuantCorrection F8_E8M0 (bestla_prologue_b.h:1198-1208): static_cast<uint8_t>(float)
    sp[i] = uint8_t(f2i(v) & 0xff);
    return;
  }
  if (t == kF32) {
    std::memcpy(sp + i * 4, &v, 4);
  } else {
    uint16_t h = (t == kBF16) ? f32_to_bf16_rne(v) : f32_to_f16_rne(v);
    std::memcpy(sp + i * 2, &h, 2);
  }
}
static inline float load_scale(const uint8_t* sp, size_t i, uint32_t t) {
  if (t == kF8E8M0) return float(std::pow(2, int(int8_t(sp[i]))));  // decompress_kblock_f8_fp (kernel_ref.h:1013-1015)
  if (t == kF32) {
    float v;
    std::memcpy(&v, sp + i * 4, 4);
    return v;
  }
  uint16_t h;
  std::memcpy(&h, sp + i * 2, 2);
  return t == kBF16 ? bf16_to_f32(h) : f16_to_f32(h);
}

// ----------------------------------------------------------------------------------------------- DQ8_BNB
// bitsandbytes' signed dynamic map (create_dynamic_map, 7 exponent bits): for decade i = 0..6 the 2^i midpoints of
// linspace(0.1, 1, 2^i + 1) scaled by 10^(i - 6), both signs, plus 0 and 1, sorted; bestla_utils.h:794-820 holds it
// rounded to 5 decimals (tests/test_dq8.py checks all 256 values against the reference's table)
float dq8_lut(int code) {
  static const std::vector<float> t = [] {
    std::vector<double> v;
    for (int i = 0; i < 7; i++) {
      const int items = (1 << i) + 1;
      for (int j = 0; j + 1 < items; j++) {
        const double b0 = 0.1 + 0.9 * j / (items - 1), b1 = 0.1 + 0.9 * (j + 1) / (items - 1);
        const double m = std::pow(10.0, i - 6) * ((b0 + b1) / 2.0);
        v.push_back(m);
        v.push_back(-m);
      }
    }
    v.push_back(0.0);
    v.push_back(1.0);
    std::sort(v.begin(), v.end());
    std::vector<float> f(256);
    for (int c = 0; c < 256; c++) f[c] = float(std::nearbyint(v[c] * 1e5) / 1e5);
    return f;
  }();
  return t[size_t(code) & 255];
}

// get_dq8_bnb (kernel_ref.h:1930-1950): binary search, nearest neighbour on a miss (ties to the upper code)
static uint8_t dq8_code(float v) {
  int lo = 0, hi = 255;
  while (lo <= hi) {
    const int mid = lo + (hi - lo) / 2;
    const float x = dq8_lut(mid);
    if (x == v) return uint8_t(mid);
    if (x < v)
      lo = mid + 1;
    else
      hi = mid - 1;
  }
  if (hi < 0) return 0;
  if (lo >= 256) return 255;
  return uint8_t(v - dq8_lut(hi) < dq8_lut(lo) - v ? hi : lo);
}

void dq8_double_quant(float* scale, size_t n, int dqb, float* dq) {
  float offset = 0.f;
  for (size_t i = 0; i < n; i++) offset += scale[i];
  offset /= float(n);
  dq[updiv(n, size_t(dqb))] = offset;
  size_t i = 0;
  auto block = [&](size_t len) {
    float absmax = std::numeric_limits<float>::min();
    for (size_t j = 0; j < len; j++) {
      scale[i + j] -= offset;
      absmax = smax(absmax, std::fabs(scale[i + j]));
    }
    for (size_t j = 0; j < len; j++) scale[i + j] = float(dq8_code(scale[i + j] / absmax));
    return absmax;
  };
  for (; i < n / dqb * dqb; i += dqb) dq[i / dqb] = block(size_t(dqb));
  // a partial last block's absmax lands one slot further, on the offset (kernel_ref.h:1978); kept for parity
  if (i < n) dq[i / dqb + 1] = block(n - i);
}

float Blob::scale_at(const int8_t* base, int g, int col) const {
  const size_t c = size_t(g) * cstep + col;
  const uint8_t* sp = reinterpret_cast<const uint8_t*>(base + s_off);
  if (!has_dq) return load_scale(sp, c, scale_t);
  float a, off;
  std::memcpy(&a, base + dq_off + (size_t(g) * n + col) / dq_blocksize * 4, 4);
  std::memcpy(&off, base + dq_off + dq_size - 4, 4);
  const float p = dq8_lut(sp[c]) * a;  // two statements: no fused multiply-add, as the reference's scalar code
  return p + off;
}

// ----------------------------------------------------------------------------------------------- quantizer
// bestla_utils.h:414-454: exponent bits 4 / 5, quantisation mantissa bits 5 / 4 (implicit one included), mx max norm
// (E4M3 448, E5M2 57344)
static float f8_maxnorm(uint32_t t) { return t == kF8E4M3 ? 448.f : 57344.f; }
void quantize_kblock(const float* src, int K, int N, int ld_src, int bs, uint32_t qtype, int8_t* q, float* scales,
                     int8_t* zp, bool e8m0) {
  if (is_f8(qtype)) {  // quantize_f32_f8_rowblock_mxscale (kernel_ref.h:1764-1800): e8m0 scales hold the exponent
    const float maxnorm = f8_maxnorm(qtype);
    const float emax = qtype == kF8E4M3 ? 8.f : 15.f;  // 2^(ebits-1), minus 1 for E5M2
    parallel_for(N, [&](int n) {
      for (int j = 0; j < K; j += bs) {
        const int len = std::min(bs, K - j);
        float scale = std::numeric_limits<float>::min();
        for (int t = 0; t < len; t++) scale = smax(scale, std::fabs(src[size_t(j + t) * ld_src + n]));
        if (e8m0) {
          if (scale == 0) scale += std::numeric_limits<float>::min();
          scale = std::floor(std::log2(scale)) - emax;
          scale = scale < -127.f ? -127.f : scale;
        } else {
          scale /= maxnorm;
        }
        scales[size_t(j / bs) * N + n] = scale;
        for (int t = 0; t < len; t++)
          q[size_t(j + t) * N + n] = f8_quantize(qtype, src[size_t(j + t) * ld_src + n], scale, e8m0);
      }
    });
    return;
  }
  const int f4 = f4_kind(qtype);
  if (f4 >= 0) {  // quantize_f32_f4_rowblock (kernel_ref.h:1800-1822): absmax from FLT_MIN, code = f4(x * (1/absmax))
    parallel_for(N, [&](int n) {
      for (int j = 0; j < K; j += bs) {
        const int len = std::min(bs, K - j);
        float absmax = std::numeric_limits<float>::min();
        for (int t = 0; t < len; t++) absmax = std::max(absmax, std::fabs(src[size_t(j + t) * ld_src + n]));
        scales[size_t(j / bs) * N + n] = absmax;
        for (int t = 0; t < len; t++)
          q[size_t(j + t) * N + n] = f4_quantize(f4, src[size_t(j + t) * ld_src + n] * (1.f / absmax));
      }
    });
    return;
  }
  const int bits = dtype_bits(qtype);
  const int full = 1 << (bits - 1), sym = full - 1;
  auto clip = [&](int32_t s) { return s < -full ? -full : (s > sym ? sym : s); };
  const int nblk = int(updiv(size_t(K), size_t(bs)));
  // parallel over (column chunk): each column is independent in the reference algorithm
  const int CH = 64;
  parallel_for(int(updiv(size_t(N), CH)), [&](int c) {
    int n0 = c * CH, n1 = std::min(N, n0 + CH);
    for (int i = n0; i < n1; i++) {
      for (int g = 0; g < nblk; g++) {
        int j = g * bs, len = std::min(bs, K - j);
        if (!zp) {  // sNauto sym (kernel_ref.h:1650-1671)
          float maxval = std::numeric_limits<float>::min(), minval = std::numeric_limits<float>::max(), absmax = 0;
          for (int t = 0; t < len; t++) {
            float x = src[size_t(j + t) * ld_src + i];
            maxval = smax(maxval, x);
            minval = smin(minval, x);
            absmax = smax(absmax, std::fabs(x));
          }
          float nval = float(sym) + 0.5f, sum = maxval + minval;
          if (std::fabs(sum) >= absmax / float(full)) nval = sum > 0.f ? float(-full) : float(full);
          float scale = absmax / nval, rscale = 1.f / scale;
          scales[size_t(g) * N + i] = scale;
          for (int t = 0; t < len; t++) {
            float v = std::roundf(src[size_t(j + t) * ld_src + i] * rscale);  // cast<float,int8_t>
            v = smax(smin(v, 127.f), -128.f);
            q[size_t(j + t) * N + i] = int8_t(clip(int8_t(f2i(v))));
          }
        } else {  // sNauto asym (kernel_ref.h:1673-1693)
          float maxval = 0.f, minval = 0.f;
          for (int t = 0; t < len; t++) {
            float x = src[size_t(j + t) * ld_src + i];
            maxval = smax(maxval, x);
            minval = smin(minval, x);
          }
          float scale = (maxval - minval) / float((1 << bits) - 1), rscale = 1.f / scale;
          scales[size_t(g) * N + i] = scale;
          int32_t z = clip(wrap_add(f2i(std::roundf((0 - minval) * rscale)), -full));
          zp[size_t(g) * N + i] = int8_t(z);
          for (int t = 0; t < len; t++)
            q[size_t(j + t) * N + i] =
                int8_t(clip(wrap_add(f2i(std::roundf(src[size_t(j + t) * ld_src + i] * rscale)), z)));
        }
      }
    }
  });
}

// ----------------------------------------------------------------------------------------------- pack
// element (k, n) -> flat index in the [NPad/NTILE][KPad/PR][NTILE][PR] interleave (kernel_ref.h:39-59)
static inline size_t ilv_index(int k, int n, int kpad, int ntile, int pr) {
  return size_t(n / ntile) * ntile * kpad + size_t(k / pr) * ntile * pr + size_t(n % ntile) * pr + (k % pr);
}

static inline int8_t read_q(const Blob& b, const uint8_t* qp, const CoreInfo& ci, int kk, int nn);

bool pack_quantized(Blob& b, int8_t* base, const int8_t* Q, int ldq, const float* S, const int8_t* Z,
                    const int* g_idx, std::string* err) {
  const CoreInfo ci = core_info(b.core_id);
  const int bits = dtype_bits(b.qtype);
  if (bits < 1 || bits > 8) {
    if (err) *err = "unsupported weight bits";
    return false;
  }
  const int rawnk = b.ngroups_k(), nk = b.ngroups();
  // setQuantCorrection (bestla_prologue_b.h:244-335): scales/zp with zero padding rows and columns
  uint8_t* sp = reinterpret_cast<uint8_t*>(base + b.s_off);
  std::vector<float> dqc;  // DQ8_BNB: packQWeight double-quantizes the [rawnk][N] scales first (bestla_prologue_b.h:381-386)
  if (b.has_dq) {
    if (nk != rawnk || b.asym) {
      if (err) *err = b.asym ? "DQ8_BNB scales are symmetric only" : "DQ8_BNB scales need K padded within its last group";
      return false;
    }
    dqc.assign(S, S + size_t(rawnk) * b.n);
    std::vector<float> dq(updiv(dqc.size(), size_t(b.dq_blocksize)) + 1, 0.f);
    dq8_double_quant(dqc.data(), dqc.size(), b.dq_blocksize, dq.data());
    std::memset(base + b.dq_off, 0, b.dq_size);
    std::memcpy(base + b.dq_off, dq.data(), dq.size() * 4);  // setDoubleQuantCorrection (:161-168)
  }
  parallel_for(nk, [&](int g) {
    for (int n = 0; n < b.npad; n++) {
      const bool in = g < rawnk && n < b.n;
      if (b.has_dq)  // setQuantCorrection DQ8_BNB (:313-329): static_cast<uint8_t>(code), zero padding
        sp[size_t(g) * b.npad + n] = in ? uint8_t(dqc[size_t(g) * b.n + n]) : 0;
      else
        store_scale(sp, size_t(g) * b.npad + n, b.scale_t, in ? S[size_t(g) * b.n + n] : 0.f);
    }
    if (b.asym) {
      int8_t* zp = base + b.z_off;
      for (int n = 0; n < b.npad; n++)
        zp[size_t(g) * b.npad + n] = (g < rawnk && n < b.n) ? Z[size_t(g) * b.n + n] : 0;
    }
  });
  if (b.has_shuffle) {  // setShuffleIndices (bestla_prologue_b.h:337-356)
    int* lut = reinterpret_cast<int*>(base + b.shf_off);
    std::vector<int> cnt(size_t(b.ngroups_k()), 0);
    for (int i = 0; i < b.k; i++) {
      int g = g_idx[i];
      if (g < 0 || g >= b.ngroups_k() || cnt[g] >= b.blocksize) {
        if (err) *err = "g_idx out of range or group overfull";
        return false;
      }
      lut[size_t(g) * b.blocksize + cnt[g]++] = i;
    }
  }
  // reorderWeight + compressWeight: walk the interleaved order directly, packing as we go
  uint8_t* qp = reinterpret_cast<uint8_t*>(base + b.q_off);
  const int ntile = ci.ntile, pr = ci.packrow, kpad = b.kpad;
  if (bits == 1 || bits == 3 || bits == 5 || bits == 6 || bits == 7) {  // bit planes (compressBitNWeight,
    // bestla_prologue_b.h:512-546 / compressBit1Weight :566-581)
    const size_t nel = size_t(b.npad) * kpad;
    std::memset(qp, 0, b.q_size);
    const bool has4 = bits >= 5, has2 = bits == 3 || bits >= 6, has1 = bits == 1 || bits == 3 || bits == 5 || bits == 7;
    const size_t o2 = has4 ? nel / 2 : 0, o1 = o2 + (has2 ? nel / 4 : 0);
    // one task per group of 8 elements so no two tasks write the same byte of any plane
    parallel_for(int(nel / 8 / 64 + 1), [&](int task) {
      for (size_t e8 = size_t(task) * 64; e8 < std::min(nel / 8, size_t(task + 1) * 64); e8++)
        for (size_t e = e8 * 8; e < e8 * 8 + 8; e++) {
          // compress_1bit (kernel_ref.h:343-361) fills the slot of element 8i + 4 from srcptr[8i + FullRange] =
          // srcptr[8i + 1]; the blob keeps that, so it matches the reference's byte for byte
          const size_t es = bits == 1 && (e & 7) == 4 ? e - 3 : e;
          const size_t st = es / (size_t(ntile) * kpad), el = es % (size_t(ntile) * kpad);
          const int kk = int(el / (size_t(ntile) * pr)) * pr + int(el % pr);
          const int nn = int(st) * ntile + int((el / pr) % ntile);
          const int8_t v = (kk < b.k && nn < b.n) ? Q[size_t(kk) * ldq + nn] : 0;
          uint32_t u = uint32_t(v + (1 << (bits - 1)));
          int sh = 0;
          if (has4) {
            qp[e / 2] |= uint8_t((u & 15u) << (4 * (e & 1)));
            sh = 4;
          }
          if (has2) {
            qp[o2 + e / 4] |= uint8_t(((u >> sh) & 3u) << (2 * (e & 3)));
            sh += 2;
          }
          if (has1) qp[o1 + e / 8] |= uint8_t(((u >> sh) & 1u) << (e & 7));
        }
    });
  } else {
  const int per_byte = 8 / bits;
  // compress_f4 (kernel_ref.h:167-176) stores the codes as they are; the integer compressors store q + 2^(bits-1)
  const int8_t bias = int8_t((bits == 8 || f4_kind(b.qtype) >= 0) ? 0 : (1 << (bits - 1)));
  const size_t stripe_elems = size_t(ntile) * kpad;
  parallel_for(b.npad / ntile, [&](int st) {
    size_t e0 = size_t(st) * stripe_elems;
    for (size_t e = 0; e < stripe_elems; e += per_byte) {
      uint8_t byte = 0;
      for (int t = 0; t < per_byte; t++) {
        size_t el = e + t;  // within stripe: [KPad/PR][NTILE][PR]
        int kk = int(el / (size_t(ntile) * pr)) * pr + int(el % pr);
        int nn = st * ntile + int((el / pr) % ntile);
        int8_t v = (kk < b.k && nn < b.n) ? Q[size_t(kk) * ldq + nn] : 0;
        if (bits == 8) {
          qp[e0 + e] = uint8_t(v);
        } else {
          byte |= uint8_t((uint8_t(v + bias) & ((1u << bits) - 1)) << (bits * t));
        }
      }
      if (bits != 8) qp[(e0 + e) / per_byte] = byte;
    }
  });
  }
  (void)ilv_index;
  if (b.has_reduce) {  // reduceWeight (bestla_prologue_b.h:455-470): sequential float sum per (block, n) -> bf16
    uint16_t* rp = reinterpret_cast<uint16_t*>(base + b.r_off);
    parallel_for(rawnk, [&](int g) {
      int k0 = g * b.blocksize, k1 = std::min(b.k, k0 + b.blocksize);
      for (int n = 0; n < b.n; n++) {
        float s = b.scale_at(base, g, n);
        int z = b.asym ? (base + b.z_off)[size_t(g) * b.cstep + n] : 0;
        float t = 0.f;
        for (int kk = k0; kk < k1; kk++)  // from the stored codes (unpackWeight): S1 keeps compress_1bit's slot 4
          t += float((bits == 1 ? read_q(b, qp, ci, kk, n) : Q[size_t(kk) * ldq + n]) - z) * s;
        rp[size_t(g) * b.cstep + n] = f32_to_bf16_rne(t);
      }
    });
  }
  return true;
}

static inline int8_t read_q(const Blob& b, const uint8_t* qp, const CoreInfo& ci, int kk, int nn) {
  size_t e = ilv_index(kk, nn, b.kpad, ci.ntile, ci.packrow);
  int bits = dtype_bits(b.qtype);
  if (bits == 8) return int8_t(qp[e]);
  if (bits == 1 || bits == 3 || bits == 5 || bits == 6 || bits == 7) {
    const size_t nel = size_t(b.npad) * b.kpad;
    const bool has4 = bits >= 5, has2 = bits == 3 || bits >= 6, has1 = bits == 1 || bits == 3 || bits == 5 || bits == 7;
    const size_t o2 = has4 ? nel / 2 : 0, o1 = o2 + (has2 ? nel / 4 : 0);
    uint32_t u = 0;
    int sh = 0;
    if (has4) {
      u = (qp[e / 2] >> (4 * (e & 1))) & 15u;
      sh = 4;
    }
    if (has2) {
      u |= ((qp[o2 + e / 4] >> (2 * (e & 3))) & 3u) << sh;
      sh += 2;
    }
    if (has1) u |= ((qp[o1 + e / 8] >> (e & 7)) & 1u) << sh;
    return int8_t(int(u) - (1 << (bits - 1)));
  }
  int per = 8 / bits;
  int v = (qp[e / per] >> (bits * (e % per))) & ((1 << bits) - 1);
  if (f4_kind(b.qtype) >= 0) return int8_t(v);  // the F4 code
  return int8_t(v - (1 << (bits - 1)));
}

void unpack_quantized(const Blob& b, const int8_t* base, int8_t* Q, float* S, int8_t* Z, int* shuffle) {
  const CoreInfo ci = core_info(b.core_id);
  const uint8_t* qp = reinterpret_cast<const uint8_t*>(base + b.q_off);
  if (Q)
    parallel_for(b.k, [&](int kk) {
      for (int nn = 0; nn < b.n; nn++) Q[size_t(kk) * b.n + nn] = read_q(b, qp, ci, kk, nn);
    });
  for (int g = 0; g < b.ngroups_k(); g++)
    for (int nn = 0; nn < b.n; nn++) {
      size_t ci2 = size_t(g) * b.cstep + nn;
      if (S) S[size_t(g) * b.n + nn] = b.scale_at(base, g, nn);
      if (Z) Z[size_t(g) * b.n + nn] = b.asym ? base[b.z_off + ci2] : 0;
    }
  if (shuffle && b.has_shuffle) std::memcpy(shuffle, base + b.shf_off, size_t(b.k) * 4);
}

void unpack_fp32(const Blob& b, const int8_t* base, float* W, int ldw) {
  const CoreInfo ci = core_info(b.core_id);
  const uint8_t* qp = reinterpret_cast<const uint8_t*>(base + b.q_off);
  parallel_for(b.k, [&](int kk) {
    int g = kk / b.blocksize;
    for (int nn = 0; nn < b.n; nn++) {
      size_t c = size_t(g) * b.cstep + nn;
      int z = b.asym ? base[b.z_off + c] : 0;
      const int f4 = f4_kind(b.qtype);
      const int8_t qv = read_q(b, qp, ci, kk, nn);
      const float sc = b.scale_at(base, g, nn);
      W[size_t(kk) * ldw + nn] = f4 >= 0 ? f4_lut(f4, qv) * sc : (is_f8(b.qtype) ? f8_to_f32(b.qtype, qv) * sc
                                                                                   : float(qv - z) * sc);
    }
  });
}

// ----------------------------------------------------------------------------------------------- NFloat 8-bit

// f8_mx_quantize (kernel_ref.h:1721-1762), one element: scale the value, round its mantissa to the format at the value's
// own exponent (clamped below at the format's minimum normal exponent), clamp to the max norm and re-pack the fp32 bits
// into sign | exponent | mantissa.  An exponent that wraps out of range stores 0 (the reference's uint8 arithmetic).
int8_t f8_quantize(uint32_t t, float v, float scale, bool e8m0) {
  v = e8m0 ? v / float(std::pow(2, scale)) : v / scale;
  const int ebits = t == kF8E4M3 ? 4 : 5, qm = t == kF8E4M3 ? 5 : 4, mbits = 7 - ebits;
  float pe = std::floor(std::log2(std::fabs(v == 0 ? v + 1 : v)));
  const float min_exp = float(2 - (1 << (ebits - 1)));
  pe = pe < min_exp ? min_exp : pe;
  v = float(v / std::pow(2, pe) * std::pow(2, qm - 2));
  const float sgn = v > 0 ? 1.f : -1.f;
  v = sgn * float(std::floor(std::fabs(v) + 0.5));
  v = float(v / std::pow(2, qm - 2) * std::pow(2, pe));
  const float mx = f8_maxnorm(t);
  v = v < -mx ? -mx : (v > mx ? mx : v);
  uint32_t u;
  std::memcpy(&u, &v, 4);
  const uint8_t sbit = uint8_t((u >> 24) & 0x80);
  uint8_t e = uint8_t(uint8_t(u >> 23) - 127 + (1 << (ebits - 1)) - 1);
  if (e > uint8_t((1 << ebits) - 1)) e = 0;
  const uint8_t m = uint8_t(((u >> 15) & 0xff) & uint8_t(0xff00u >> mbits)) >> (1 + ebits);
  return int8_t(sbit | uint8_t(e << mbits) | m);
}

// f8_to_fp32 (kernel_ref.h:984-1001): the exponent field is always a normal one, bias 2^(ebits-1) - 1
float f8_to_f32(uint32_t t, int8_t code) {
  const uint32_t x = uint32_t(uint8_t(code));
  const int ebits = t == kF8E4M3 ? 4 : 5, mbits = 7 - ebits;
  const uint32_t e = ((x & 0x7f) >> mbits) - (1u << (ebits - 1)) + 1 + 127;
  const uint32_t r = ((x & 0x80) << 24) | (e << 23) | ((x << (23 - mbits)) & 0x007fffffu);
  float f;
  std::memcpy(&f, &r, 4);
  return f;
}

// ----------------------------------------------------------------------------------------------- NFloat 4-bit
static const float kF4Lut[3][16] = {
    {0.00000000f, 5.208333333e-03f, 0.66666667f, 1.00000000f, 0.33333333f, 0.50000000f, 0.16666667f, 0.25000000f,
     -1.f * 0.00000000f, -1.f * 5.208333333e-03f, -1.f * 0.66666667f, -1.f * 1.00000000f, -1.f * 0.33333333f,
     -1.f * 0.50000000f, -1.f * 0.16666667f, -1.f * 0.25000000f},
    {0.f, 0.010416666666666666f, 0.16666666666666666f, 0.25f, 0.333333333333333f, 0.5f, 0.6666666666666f, 1.f,
     -1.f * 0.f, -1.f * 0.010416666666666666f, -1.f * 0.16666666666666666f, -1.f * 0.25f, -1.f * 0.333333333333333f,
     -1.f * 0.5f, -1.f * 0.6666666666666f, -1.f * 1.f},
    {0.f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f, -0.28444138169288635f,
     -0.18477343022823334f, -0.09105003625154495f, -1.f, 0.07958029955625534f, 0.16093020141124725f,
     0.24611230194568634f, 0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f,
     1.0f}};

float f4_lut(int kind, int code) { return kF4Lut[kind][code & 15]; }

int8_t f4_quantize(int kind, float x) {
  if (kind == 2) {  // nf4: thresholds are the midpoints of the sorted LUT; codes of 0 and -1 swapped
    if (x > 0.03979014977812767f) {
      if (x > 0.3893125355243683f) {
        if (x > 0.6427869200706482f) return x > 0.8614784181118011f ? 0xF : 0xE;
        return x > 0.5016634166240692f ? 0xD : 0xC;
      }
      if (x > 0.2035212516784668f) return x > 0.2920137718319893f ? 0xB : 0xA;
      return x > 0.1202552504837513f ? 0x9 : 0x8;
    }
    if (x > -0.33967943489551544f) {
      if (x > -0.13791173323988914f) return x > -0.045525018125772476f ? 0x0 : 0x6;
      return x > -0.23460740596055984f ? 0x5 : 0x4;
    }
    if (x > -0.6106329262256622f) return x > -0.4599952697753906f ? 0x3 : 0x2;
    return x > -0.8480964004993439f ? 0x1 : 0x7;
  }
  const int sign = x < 0 ? 0x8 : 0;
  x = std::fabs(x);
  if (kind == 0) {  // fp4 bnb
    if (x > 0.29166667f) {
      if (x > 0.583333f) return int8_t((x > 0.8333333f ? 0x3 : 0x2) + sign);
      return int8_t((x > 0.4166667f ? 0x5 : 0x4) + sign);
    }
    if (x > 0.0859375f) return int8_t((x > 0.20833333f ? 0x7 : 0x6) + sign);
    return int8_t((x > 0.00260417f ? 0x1 : 0x0) + sign);
  }
  // fp4 e2m1 (the reference's normalised table: magnitudes / 6, code 1 = 1/96)
  if (x > 1.75f / 6) {
    if (x > 3.5f / 6) return int8_t((x > 5.f / 6 ? 0x7 : 0x6) + sign);
    return int8_t((x > 2.5f / 6 ? 0x5 : 0x4) + sign);
  }
  if (x > 0.53125f / 6) return int8_t((x > 1.25f / 6 ? 0x3 : 0x2) + sign);
  return int8_t((x > 0.03125f / 6 ? 0x1 : 0x0) + sign);
}

}  // namespace nad
