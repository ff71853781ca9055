/*
 * btla_oracle.c -- scalar C restatement of the reference's WOQ packing / dequant / GEMV algorithms.
 * TEST INFRASTRUCTURE ONLY (see btla_oracle.h).  Each function cites the reference file:line it follows,
 * relative to /root/reference.
 */
#include "btla_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ scalar helpers */
typedef union {
  float f;
  uint32_t u;
} f32u;

/* bestla_utils.h:146-153 bf16::fromfloat: tmp.u += 0x7fff + lsb (no NaN special-case) */
uint16_t orc_f32_to_bf16(float v) {
  f32u t;
  t.f = v;
  uint32_t lsb = (t.u >> 16) & 1u;
  t.u += 0x7fffu + lsb;
  return (uint16_t)(t.u >> 16);
}

float orc_bf16_to_f32(uint16_t x) {
  f32u t;
  t.u = ((uint32_t)x) << 16;
  return t.f;
}

/* bestla_utils.h:184-196 fp16::operator=(float) */
uint16_t orc_f32_to_fp16_bestla(float val) {
  f32u t;
  t.f = val;
  const uint32_t b = t.u + 0x00001000u;
  const uint32_t e = (b & 0x7F800000u) >> 23;
  const uint32_t m = b & 0x007FFFFFu;
  return (uint16_t)((b & 0x80000000u) >> 16 | (e > 112) * ((((e - 112) << 10) & 0x7C00u) | m >> 13) |
                    ((e < 113) & (e > 101)) * ((((0x007FF000u + m) >> (125 - e)) + 1) >> 1) | (e > 143) * 0x7FFFu);
}

/* IEEE-754 binary16 round-to-nearest-even (vcvtps2ph with RNE on AVX512-FP16/F16C hosts) */
uint16_t orc_f32_to_fp16_rne(float v) {
  f32u t;
  t.f = v;
  uint32_t x = t.u;
  uint32_t sign = (x >> 16) & 0x8000u;
  uint32_t ax = x & 0x7FFFFFFFu;
  if (ax > 0x7F800000u) return (uint16_t)(sign | 0x7E00u | ((ax >> 13) & 0x3FFu)); /* NaN */
  if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);                         /* overflow -> inf */
  if (ax < 0x38800000u) {                                                            /* subnormal / zero */
    if (ax < 0x33000000u) return (uint16_t)sign;
    uint32_t e = ax >> 23;
    uint32_t mant = (ax & 0x7FFFFFu) | 0x800000u;
    uint32_t shift = 126 - e; /* 14..24 */
    uint32_t q = mant >> shift;
    uint32_t rem = mant & ((1u << shift) - 1);
    uint32_t half = 1u << (shift - 1);
    if (rem > half || (rem == half && (q & 1u))) q++;
    return (uint16_t)(sign | q);
  }
  uint32_t e = (ax >> 23) - 112;
  uint32_t mant = ax & 0x7FFFFFu;
  uint32_t q = (e << 10) | (mant >> 13);
  uint32_t rem = mant & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (q & 1u))) q++;
  return (uint16_t)(sign | q);
}

/* bestla_utils.h:197-206 explicit operator float */
float orc_fp16_to_f32(uint16_t x) {
  const uint32_t e = (x & 0x7C00u) >> 10;
  const uint32_t m = (uint32_t)(x & 0x03FFu) << 13;
  f32u mv;
  mv.f = (float)m;
  const uint32_t v = mv.u >> 23;
  f32u r;
  r.u = ((uint32_t)(x & 0x8000u)) << 16 | (e != 0) * ((e + 112) << 23 | m) |
        ((e == 0) & (m != 0)) * ((v - 37) << 23 | ((m << (150 - v)) & 0x007FE000u));
  return r.f;
}

/* std::max / std::min semantics (first argument wins unless strictly ordered) */
static inline float smax(float a, float b) { return (a < b) ? b : a; }
static inline float smin(float a, float b) { return (b < a) ? b : a; }

/* float -> int32 as x86 cvttss2si: NaN / out-of-range -> INT32_MIN */
static inline int32_t f2i_x86(float x) {
  if (isnan(x) || x >= 2147483648.0f || x < -2147483648.0f) return INT32_MIN;
  return (int32_t)x;
}
static inline int32_t iadd_wrap(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }

/* bestla_utils.h:507-512 cast<float,int8_t>: roundf then clamp to [-128,127] */
static inline int8_t cast_f32_s8(float v) {
  v = roundf(v);
  v = smin(v, 127.f);
  v = smax(v, -128.f);
  return (int8_t)f2i_x86(v);
}
/* bestla_utils.h:522-525 cast<float,int>: int(roundf) */
static inline int32_t cast_f32_int(float v) { return f2i_x86(roundf(v)); }

int orc_f4_kind(uint32_t qtype);
float orc_f4_lut(int kind, int code);
float orc_f8_to_f32(uint32_t t, int8_t code);
void orc_quantize_f8_rowblock(const float* src, int8_t* dst, int row, int col, int ld_src, int ld_dst, float* scales,
                              int blocksize, uint32_t t, int e8m0);
void orc_quantize_f4_rowblock(const float* src, int8_t* dst, int row, int col, int ld_src, int ld_dst, float* scales,
                              int blocksize, int kind);
int orc_compress_planes(int bits, const int8_t* src, uint8_t* dst, size_t n);
int orc_decompress_planes(int bits, const uint8_t* src, int8_t* dst, size_t n);

/* ------------------------------------------------------------------ quantizer */
/* kernel_ref.h:1608-1719.  dispatch_calc always takes the sNauto_* lambdas for integer types. */
void orc_quantize_rowblock(const float* srcptr, int8_t* dstptr, int row, int col, int ld_src, int ld_dst,
                           float* scales, int8_t* zero_points, int blocksize, int bits) {
  const int raw_blocksize = blocksize;
  const int FullValue = 1 << (bits - 1);
  const int SymValue = FullValue - 1;
#define CLIPV(s) ((s) < -FullValue ? -FullValue : ((s) > SymValue ? SymValue : (s)))
  for (int i = 0; i < col; i++) {
    int align_row_loop = row / blocksize * blocksize;
    int j = 0;
    while (j < row) {
      int bs = (j < align_row_loop) ? blocksize : row - align_row_loop;
      if (zero_points == NULL) {
        /* sNauto_calc_store_scale_and_quantv_sym, kernel_ref.h:1650-1671 */
        float maxval = 1.17549435e-38f; /* std::numeric_limits<float>::min() */
        float minval = 3.40282347e+38f;
        float absmax = 0.f;
        for (int ij = 0; ij < bs; ij++) {
          float x = srcptr[(size_t)(j + ij) * ld_src + i];
          maxval = smax(maxval, x);
          minval = smin(minval, x);
          absmax = smax(absmax, fabsf(x));
        }
        float NVal = (float)SymValue + 0.5f;
        float sum = maxval + minval;
        if (fabsf(sum) >= absmax / (float)FullValue) {
          NVal = sum > 0.f ? (float)(-FullValue) : (float)FullValue;
        }
        float scale = absmax / NVal;
        float rscale = 1.f / scale;
        scales[(size_t)(j / raw_blocksize) * ld_dst + i] = scale;
        for (int ij = 0; ij < bs; ij++) {
          int v = cast_f32_s8(srcptr[(size_t)(j + ij) * ld_src + i] * rscale);
          dstptr[(size_t)(j + ij) * ld_dst + i] = (int8_t)CLIPV(v);
        }
      } else {
        /* sNauto_calc_store_scale_and_quantv_asym, kernel_ref.h:1673-1693 */
        float maxval = 0.f, minval = 0.f;
        for (int ij = 0; ij < bs; ij++) {
          float x = srcptr[(size_t)(j + ij) * ld_src + i];
          maxval = smax(maxval, x);
          minval = smin(minval, x);
        }
        float scale = (maxval - minval) / (float)((1 << bits) - 1);
        float rscale = 1.f / scale;
        scales[(size_t)(j / raw_blocksize) * ld_dst + i] = scale;
        int32_t bzp = iadd_wrap(cast_f32_int((0 - minval) * rscale), -FullValue);
        bzp = CLIPV(bzp);
        zero_points[(size_t)(j / raw_blocksize) * ld_dst + i] = (int8_t)bzp;
        for (int ij = 0; ij < bs; ij++) {
          int32_t t = iadd_wrap(cast_f32_int(srcptr[(size_t)(j + ij) * ld_src + i] * rscale), bzp);
          t = CLIPV(t);
          dstptr[(size_t)(j + ij) * ld_dst + i] = (int8_t)t;
        }
      }
      j += bs;
    }
  }
#undef CLIPV
}

/* ------------------------------------------------------------------ interleave / compress */
/* kernel_ref.h:39-59 */
void orc_padding_interleave(const int8_t* src, int8_t* dst, int row, int col, int rowpad, int colpad, int src_step,
                            int dst_step, int ntile, int rowpack) {
  for (int i = 0; i < rowpad; i += rowpack)
    for (int j = 0; j < colpad; j += ntile)
      for (int jj = 0; jj < ntile; jj++)
        for (int ii = 0; ii < rowpack; ii++)
          dst[(size_t)i * ntile + (size_t)j * dst_step + jj * rowpack + ii] =
              ((i + ii) < row && (j + jj) < col) ? src[(size_t)(i + ii) * src_step + (j + jj)] : 0;
}

/* kernel_ref.h:62-80 */
void orc_revert_padding_interleave(const int8_t* src, int8_t* dst, int row, int col, int rowpad, int colpad,
                                   int src_step, int dst_step, int ntile, int rowpack) {
  for (int i = 0; i < rowpad; i += rowpack)
    for (int j = 0; j < colpad; j += ntile)
      for (int jj = 0; jj < ntile; jj++)
        if ((j + jj) < col)
          for (int ii = 0; ii < rowpack; ii++)
            if ((i + ii) < row)
              dst[(size_t)(i + ii) * dst_step + (j + jj)] =
                  src[(size_t)i * ntile + (size_t)j * src_step + jj * rowpack + ii];
}

/* kernel_ref.h:155-165: int4x2 {x: low nibble, y: high nibble} = value + 8 */
void orc_compress_s4(const int8_t* src, uint8_t* dst, size_t n) {
  for (size_t i = 0; i < n; i += 2)
    dst[i / 2] = (uint8_t)(((uint8_t)(src[i] + 8) & 0xF) | (((uint8_t)(src[i + 1] + 8) & 0xF) << 4));
}
/* kernel_ref.h:330-341: bit2x4 {a,b,c,d} LSB..MSB = value + 2 */
void orc_compress_s2(const int8_t* src, uint8_t* dst, size_t n) {
  for (size_t i = 0; i < n; i += 4) {
    uint8_t v = 0;
    for (int t = 0; t < 4; t++) v |= (uint8_t)(((uint8_t)(src[i + t] + 2) & 0x3) << (2 * t));
    dst[i / 4] = v;
  }
}
/* kernel_ref.h:471-479 */
void orc_decompress_s4(const uint8_t* src, int8_t* dst, size_t n) {
  for (size_t i = 0; i < n; i += 2) {
    dst[i] = (int8_t)((src[i / 2] & 0xF) - 8);
    dst[i + 1] = (int8_t)((src[i / 2] >> 4) - 8);
  }
}
/* kernel_ref.h:499-509 */
void orc_decompress_s2(const uint8_t* src, int8_t* dst, size_t n) {
  for (size_t i = 0; i < n; i += 4)
    for (int t = 0; t < 4; t++) dst[i + t] = (int8_t)(((src[i / 4] >> (2 * t)) & 3) - 2);
}

/* ------------------------------------------------------------------ core ids */
/* BTLA_ISA (bestla.h:23-36): AVX2=2, AVX_VNNI=3, AVX512F=4, AVX512BW=5, AVX512_VNNI=6, AMX_BF16=9, AMX_INT8=10,
   AMX_FP16=11.  CompType (bestla_gemm.h:22-50): FP32=0x000, BF16_FP32=0x011, FP16_FP32=0x022,
   INT8_US_FP32=0x034.  make_core_id: NTILE | PACKROW<<8 | COMP<<16 | ISA<<32 (bestla_gemm.h:91). */
static uint64_t mkid(int nt, int pr, int comp, int isa) {
  return (uint64_t)nt | ((uint64_t)pr << 8) | ((uint64_t)comp << 16) | ((uint64_t)isa << 32);
}
uint64_t orc_core_id(const char* name) {
  if (!strcmp(name, "avx2")) return mkid(24, 1, 0x000, 2);
  if (!strcmp(name, "avx512f")) return mkid(48, 1, 0x000, 4);
  if (!strcmp(name, "amx_bf16")) return mkid(48, 2, 0x011, 9);
  if (!strcmp(name, "amx_fp16")) return mkid(48, 2, 0x022, 11);
  if (!strcmp(name, "avx512_vnni_kblock")) return mkid(48, 4, 0x034, 6);
  if (!strcmp(name, "avx512bw_kblock")) return mkid(48, 4, 0x034, 5);
  if (!strcmp(name, "avx_vnni_kblock")) return mkid(24, 4, 0x034, 3);
  if (!strcmp(name, "avx2_vnni_kblock")) return mkid(24, 4, 0x034, 2);
  if (!strcmp(name, "amx_int8_kblock")) return mkid(48, 4, 0x034, 10);
  return 0;
}
int orc_core_ntile(uint64_t id) { return (int)(id & 0xff); }
int orc_core_packrow(uint64_t id) { return (int)((id >> 8) & 0xff); }
int orc_core_is_int(uint64_t id) {
  int b = (int)((id >> 16) & 0xf0) >> 4; /* CompTypeHelper::get_B, bestla_gemm.h:66-79 */
  return b == 3 || b == 4;
}
int orc_core_ktile(uint64_t id) {
  int isa = (int)((id >> 32) & 0xff);
  int pr = orc_core_packrow(id);
  if (pr == 1) return 1;                /* Avx2N8P1 / Avx512fN16P1: KTILE 1 */
  if (isa == 9 || isa == 11) return 32; /* Amxbf16N16P2 / Amxfp16N16P2 */
  if (isa == 10) return 64;             /* Amxint8N16P4 */
  return 4;                             /* VNNI / BW KBlock cores */
}

uint64_t orc_select_core(int comp_type, uint32_t qtype, int bs, int asym, int profile) {
  int amx = profile == 0, vnni = profile <= 1, a512 = profile <= 2;
  int is_int = ((qtype >> 8) & 0xff) == 1;
  switch (comp_type) {
    case 4: /* NE_COMP_INT8 */
      if (is_int && !(qtype == ORC_S8 && asym)) {
        if (amx && bs % 64 == 0) return orc_core_id("amx_int8_kblock");
        if (vnni && bs % 4 == 0) return orc_core_id("avx512_vnni_kblock");
        if (a512 && bs % 4 == 0) return orc_core_id("avx512bw_kblock");
        if (bs % 4 == 0) return orc_core_id("avx2_vnni_kblock");
      }
      /* fallthrough */
    case 2: /* NE_COMP_BF16 */
      if (amx && bs % 32 == 0) return orc_core_id("amx_bf16");
      /* fallthrough */
    case 3: /* NE_COMP_F16: AMX-FP16 absent on every profile here */
    case 1:
    case 0:
      if (a512) return orc_core_id("avx512f");
      return orc_core_id("avx2");
    default:
      return 0;
  }
}

/* ------------------------------------------------------------------ blob layout */
static int dtype_bits(uint32_t t) { return (int)(t & 0xff); }
static size_t dtype_bytes(uint32_t t) { return (size_t)((t & 0xff) / 8); }
static size_t updiv(size_t a, size_t b) { return (a + b - 1) / b; }
static size_t padto(size_t a, size_t b) { return updiv(a, b) * b; }

typedef struct {
  int npad, kpad, n, k, bs, dq_bs;
  uint32_t prologue, dtype, scat, zpt, redt;
  uint64_t coreid;
  int cstep;
  size_t csize, msize;
  int asym, has_red, has_shf;
  size_t q_size, s_size, z_size, r_size, shf_size, dq_size;
  /* offsets from blob base */
  size_t q_off, s_off, z_off, r_off, shf_off, dq_off;
  int has_dq;
} blob_t;

/* StorageWeightKBlockNInteger::resize (bestla_storage.h:725-753) + createStorage (bestla_prologue_b.h:120-127) */
static void blob_describe(blob_t* b, int n, int k, int blocksize, uint32_t qtype, uint32_t stype, int asym,
                          uint64_t coreid, int shuffle) {
  memset(b, 0, sizeof(*b));
  int ktile = orc_core_ktile(coreid), ntile = orc_core_ntile(coreid);
  b->kpad = (int)padto((size_t)k, (size_t)ktile);
  b->npad = (int)padto((size_t)n, (size_t)ntile);
  b->n = n;
  b->k = k;
  b->bs = blocksize <= 0 ? b->kpad : blocksize;
  const int is_f4 = orc_f4_kind(qtype) >= 0 || qtype == ORC_F8_E4M3 || qtype == ORC_F8_E5M2; /* NFloat */
  /* BTLA_PROLOGUEB_IDS (bestla.h:91-102): WeightKBlockNInteger = 1, WeightKBlockNFloat = 2 */
  b->prologue = is_f4 ? 2 : 1;
  b->coreid = coreid;
  b->dtype = qtype;
  b->scat = stype;
  b->zpt = is_f4 ? 0 : ORC_S8;   /* StorageWeightKBlockNFloat::resize: zp / reduce dtypes EleBitsUndef (bestla_storage.h:849) */
  b->redt = is_f4 ? 0 : ORC_BF16; /* reduce dtype fixed to BF16 by the callers, bestla_gemm.cpp:229,308,408 */
  if (is_f4) asym = 0;
  b->q_size = updiv((size_t)b->npad * b->kpad * dtype_bits(qtype), 8);
  int nk = (int)updiv((size_t)b->kpad, (size_t)b->bs);
  b->cstep = b->npad;
  b->csize = (size_t)nk * b->npad;
  b->asym = asym;
  b->has_red = is_f4 ? 0 : orc_core_is_int(coreid);
  b->has_shf = shuffle;
  b->s_size = b->csize * dtype_bytes(stype);
  b->z_size = asym ? b->csize * 1 : 0;
  b->r_size = b->has_red ? b->csize * 2 : 0;
  b->shf_size = shuffle ? (size_t)k * 4 : 0;
  if (stype == ORC_DQ8_BNB) { /* initDoubleQuantBlkSize(Block, nk_scale, ..., N) (bestla_storage.h:750-759) */
    b->has_dq = 1;
    b->dq_bs = b->bs;
    b->dq_size = (updiv((size_t)nk * n, (size_t)b->dq_bs) + 1) * sizeof(float); /* enable_double_quant :223-231 */
  }
  /* update_size (bestla_storage.h:812-816): header 48 + aligned/optional buffer sizes, padto 64 */
  size_t sz = 48;
  sz += 16 + b->q_size + 64;
  sz += 24 + (16 + b->s_size + 64);
  sz += 1 + (asym ? 16 + b->z_size + 64 : 0);
  sz += 1 + (b->has_red ? 16 + b->r_size + 64 : 0);
  sz += 1 + (b->has_dq ? 16 + b->dq_size + 64 : 0); /* mDQCorrectionBuf */
  sz += 1 + (shuffle ? 16 + b->shf_size + 64 : 0);
  b->msize = padto(sz, 64);
}

static inline void w64(int8_t** p, uint64_t v) {
  memcpy(*p, &v, 8);
  *p += 8;
}
static inline void w32(int8_t** p, uint32_t v) {
  memcpy(*p, &v, 4);
  *p += 4;
}
static inline void w8(int8_t** p, uint8_t v) {
  **p = (int8_t)v;
  *p += 1;
}
/* ObjectAlignedBuffer<64>::serializeToBuffer (bestla_storage.h:77-88): size, offset to next 64-B boundary */
static size_t aligned_buf(int8_t** p, int8_t* base, size_t size) {
  w64(p, size);
  uintptr_t tmp = (uintptr_t)(*p + 8);
  uint64_t off = ((tmp + 63) / 64 * 64) - tmp;
  w64(p, off);
  *p += off;
  size_t at = (size_t)(*p - base);
  *p += size;
  return at;
}

/* assign() (bestla_storage.h:818-823): writes the header and every buffer descriptor, returns data offsets */
static void blob_write_header(blob_t* b, int8_t* base) {
  int8_t* p = base;
  w64(&p, b->msize);
  w32(&p, b->prologue);
  w64(&p, b->coreid);
  w32(&p, (uint32_t)b->npad);
  w32(&p, (uint32_t)b->kpad);
  w32(&p, (uint32_t)b->n);
  w32(&p, (uint32_t)b->k);
  w32(&p, b->dtype);
  w32(&p, (uint32_t)b->bs);
  w32(&p, (uint32_t)b->dq_bs);
  b->q_off = aligned_buf(&p, base, b->q_size);
  w32(&p, b->scat);
  w32(&p, b->zpt);
  w32(&p, b->redt);
  w32(&p, (uint32_t)b->cstep);
  w64(&p, b->csize);
  b->s_off = aligned_buf(&p, base, b->s_size);
  w8(&p, (uint8_t)(b->asym != 0));
  if (b->asym) b->z_off = aligned_buf(&p, base, b->z_size);
  w8(&p, (uint8_t)(b->has_red != 0));
  if (b->has_red) b->r_off = aligned_buf(&p, base, b->r_size);
  w8(&p, (uint8_t)(b->has_dq != 0)); /* mDQCorrectionBuf */
  if (b->has_dq) b->dq_off = aligned_buf(&p, base, b->dq_size);
  w8(&p, (uint8_t)(b->has_shf != 0));
  if (b->has_shf) b->shf_off = aligned_buf(&p, base, b->shf_size);
}

static inline uint64_t r64(const int8_t** p) {
  uint64_t v;
  memcpy(&v, *p, 8);
  *p += 8;
  return v;
}
static inline uint32_t r32(const int8_t** p) {
  uint32_t v;
  memcpy(&v, *p, 4);
  *p += 4;
  return v;
}
static inline uint8_t r8(const int8_t** p) {
  uint8_t v = (uint8_t)**p;
  *p += 1;
  return v;
}
static size_t read_buf(const int8_t** p, const int8_t* base, size_t* size) {
  *size = r64(p);
  uint64_t off = r64(p);
  *p += off;
  size_t at = (size_t)(*p - base);
  *p += *size;
  return at;
}

/* deserialize() (bestla_storage.h:831-836) */
static int blob_parse(blob_t* b, const void* buf) {
  memset(b, 0, sizeof(*b));
  const int8_t* base = (const int8_t*)buf;
  const int8_t* p = base;
  b->msize = r64(&p);
  b->prologue = r32(&p);
  if (b->prologue != 1 && b->prologue != 2) return -1; /* WeightKBlockNInteger / WeightKBlockNFloat */
  b->coreid = r64(&p);
  b->npad = (int)r32(&p);
  b->kpad = (int)r32(&p);
  b->n = (int)r32(&p);
  b->k = (int)r32(&p);
  b->dtype = r32(&p);
  b->bs = (int)r32(&p);
  b->dq_bs = (int)r32(&p);
  b->q_off = read_buf(&p, base, &b->q_size);
  b->scat = r32(&p);
  b->zpt = r32(&p);
  b->redt = r32(&p);
  b->cstep = (int)r32(&p);
  b->csize = r64(&p);
  b->s_off = read_buf(&p, base, &b->s_size);
  b->asym = r8(&p);
  if (b->asym) b->z_off = read_buf(&p, base, &b->z_size);
  b->has_red = r8(&p);
  if (b->has_red) b->r_off = read_buf(&p, base, &b->r_size);
  b->has_dq = r8(&p);
  if (b->has_dq) b->dq_off = read_buf(&p, base, &b->dq_size);
  if (b->has_dq != (b->scat == ORC_DQ8_BNB)) return -2;
  b->has_shf = r8(&p);
  if (b->has_shf) b->shf_off = read_buf(&p, base, &b->shf_size);
  return 0;
}

size_t orc_blob_size(int n, int k, int blocksize, uint32_t qtype, uint32_t stype, int asym, uint64_t core_id,
                     int shuffle) {
  blob_t b;
  blob_describe(&b, n, k, blocksize, qtype, stype, asym, core_id, shuffle);
  return b.msize;
}

int orc_blob_info(const void* buf, int64_t* o) {
  blob_t b;
  int r = blob_parse(&b, buf);
  if (r) return r;
  int64_t v[27] = {(int64_t)b.msize, b.prologue, (int64_t)b.coreid, b.npad, b.kpad, b.n, b.k, b.dtype, b.bs,
                   b.scat, b.zpt, b.redt, b.cstep, (int64_t)b.csize, b.asym, b.has_red, b.has_shf,
                   (int64_t)b.q_off, (int64_t)b.q_size, (int64_t)b.s_off, (int64_t)b.s_size, (int64_t)b.z_off,
                   (int64_t)b.z_size, (int64_t)b.r_off, (int64_t)b.r_size, (int64_t)b.shf_off,
                   (int64_t)b.shf_size};
  memcpy(o, v, sizeof(v));
  return 0;
}

/* ------------------------------------------------------------------ DQ8_BNB double quant */
/* bestla_utils.h:794-820 dq8_bnb_LUT: bitsandbytes' signed dynamic map (7 exponent bits) rounded to 5 decimals.
   Restated from its construction: decade i = 0..6 contributes the 2^i midpoints of linspace(0.1, 1, 2^i + 1) times
   10^(i-6), both signs; plus 0 and 1; sorted.  tests/test_dq8.py pins all 256 values to the reference's table. */
static float g_dq8[256];
static int g_dq8_ready = 0;
static int cmp_d(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : (x > y ? 1 : 0);
}
static const float* dq8_table(void) {
  if (!g_dq8_ready) {
    double v[256];
    int c = 0;
    for (int i = 0; i < 7; i++) {
      int items = (1 << i) + 1;
      for (int j = 0; j + 1 < items; j++) {
        double b0 = 0.1 + 0.9 * j / (items - 1), b1 = 0.1 + 0.9 * (j + 1) / (items - 1);
        double m = pow(10.0, i - 6) * ((b0 + b1) / 2.0);
        v[c++] = m;
        v[c++] = -m;
      }
    }
    v[c++] = 0.0;
    v[c++] = 1.0;
    qsort(v, 256, sizeof(double), cmp_d);
    for (int i = 0; i < 256; i++) g_dq8[i] = (float)(nearbyint(v[i] * 1e5) / 1e5);
    g_dq8_ready = 1;
  }
  return g_dq8;
}
void orc_dq8_lut(float* out) { memcpy(out, dq8_table(), sizeof(float) * 256); }

/* kernel_ref.h:1930-1950 get_dq8_bnb */
static uint8_t dq8_encode(float v) {
  const float* t = dq8_table();
  int left = 0, right = 255;
  while (left <= right) {
    int mid = left + (right - left) / 2;
    if (t[mid] == v) return (uint8_t)mid;
    if (t[mid] < v)
      left = mid + 1;
    else
      right = mid - 1;
  }
  if (right < 0) return 0;
  if (left >= 256) return 255;
  return (v - t[right] < t[left] - v) ? (uint8_t)right : (uint8_t)left;
}

/* kernel_ref.h:1952-1979 dq8_bnb_double_quant<false>: scale[] becomes codes (as floats); dq (zero-filled by the caller,
   updiv(n, dq_bs) + 1 floats) gets each block's absmax and, last, the mean of all scales.  A partial last block writes
   its absmax one slot further (:1978), over the mean; restated as is. */
void orc_dq8_double_quant(float* scale, size_t n, int dq_bs, float* dq) {
  float offset = 0.f;
  for (size_t i = 0; i < n; i++) offset += scale[i];
  offset /= (float)n;
  dq[updiv(n, (size_t)dq_bs)] = offset;
  size_t aligned = n / dq_bs * dq_bs;
  for (size_t i = 0; i < n; i += dq_bs) {
    size_t len = i < aligned ? (size_t)dq_bs : n - i;
    float absmax = FLT_MIN;
    for (size_t j = 0; j < len; j++) {
      scale[i + j] -= offset;
      absmax = smax(absmax, fabsf(scale[i + j]));
    }
    for (size_t j = 0; j < len; j++) scale[i + j] = (float)dq8_encode(scale[i + j] / absmax);
    if (i < aligned)
      dq[i / dq_bs] = absmax;
    else
      dq[i / dq_bs + 1] = absmax;
  }
}

/* kernel_ref.h:1981-1991 dq8_get_fp_scale over [row][col] codes at src_stride, scale index (i * mN + j) / dq_bs */
void orc_dq8_get_fp_scale(const uint8_t* src, float* dst, int row, int col, int dq_bs, int dq_offset_idx,
                          const float* dq, int src_stride, int dst_stride, int mN) {
  const float* t = dq8_table();
  for (int i = 0; i < row; i++)
    for (int j = 0; j < col; j++) {
      float p = t[src[(size_t)i * src_stride + j]] * dq[((size_t)i * mN + j) / dq_bs];
      dst[(size_t)i * dst_stride + j] = p + dq[dq_offset_idx];
    }
}

/* store one scale value in the blob's scale dtype (setQuantCorrection, bestla_prologue_b.h:244-271):
   BF16 via bf16(float) RNE; F16 via the host's vcvtps2ph (IEEE RNE) on AVX512-FP16 hosts */
static void put_scale(uint8_t* sp, size_t idx, uint32_t scat, float v) {
  if (scat == ORC_F8_E8M0) { /* setQuantCorrection F8_E8M0 (bestla_prologue_b.h:1198-1208): static_cast<uint8_t> */
    sp[idx] = (uint8_t)(f2i_x86(v) & 0xff);
  } else if (scat == ORC_F32) {
    memcpy(sp + idx * 4, &v, 4);
  } else if (scat == ORC_BF16) {
    uint16_t h = orc_f32_to_bf16(v);
    memcpy(sp + idx * 2, &h, 2);
  } else {
    uint16_t h = orc_f32_to_fp16_rne(v);
    memcpy(sp + idx * 2, &h, 2);
  }
}
static float get_scale(const uint8_t* sp, size_t idx, uint32_t scat) {
  if (scat == ORC_F8_E8M0) return (float)pow(2, (int8_t)sp[idx]); /* decompress_kblock_f8_fp, kernel_ref.h:1013-1015 */
  if (scat == ORC_F32) {
    float v;
    memcpy(&v, sp + idx * 4, 4);
    return v;
  }
  uint16_t h;
  memcpy(&h, sp + idx * 2, 2);
  return scat == ORC_BF16 ? orc_bf16_to_f32(h) : orc_fp16_to_f32(h);
}

/* fp32 scale of (group g, column nn): the stored dtype, or DQ8_BNB decoded as getScale does (bestla_prologue_b.h:699-706,
   offset from the last slot of the double-quant buffer) */
static float blob_scale(const blob_t* b, const int8_t* base, int g, int nn) {
  const uint8_t* sp = (const uint8_t*)(base + b->s_off);
  size_t ci = (size_t)g * b->cstep + nn;
  if (!b->has_dq) return get_scale(sp, ci, b->scat);
  const float* dq = (const float*)(base + b->dq_off);
  float p = dq8_table()[sp[ci]] * dq[((size_t)g * b->n + nn) / b->dq_bs];
  return p + dq[b->dq_size / 4 - 1];
}

/* dequantized W[k][n] (ld = ldw) from a parsed blob: getWeight + RevertPaddingInterleave (bestla_prologue_b.h:211-242) */
static void blob_dequant(const blob_t* b, const int8_t* base, float* W, int ldw, int8_t* Qout, float* Sout,
                         int8_t* Zout) {
  int nt = orc_core_ntile(b->coreid), pr = orc_core_packrow(b->coreid);
  size_t nel = (size_t)b->npad * b->kpad;
  int8_t* flat = (int8_t*)malloc(nel);
  const uint8_t* q = (const uint8_t*)(base + b->q_off);
  int bits = dtype_bits(b->dtype);
  const int f4 = orc_f4_kind(b->dtype);
  const int f8 = b->dtype == ORC_F8_E4M3 || b->dtype == ORC_F8_E5M2;
  if (f4 >= 0)
    for (size_t e = 0; e < nel; e++) flat[e] = (int8_t)((q[e / 2] >> (4 * (e & 1))) & 15);
  else if (bits == 4)
    orc_decompress_s4(q, flat, nel);
  else if (bits == 2)
    orc_decompress_s2(q, flat, nel);
  else if (bits == 8)
    memcpy(flat, q, nel);
  else
    orc_decompress_planes(bits, q, flat, nel);
  int8_t* qkn = (int8_t*)malloc((size_t)b->k * b->n);
  orc_revert_padding_interleave(flat, qkn, b->k, b->n, b->kpad, b->npad, b->kpad, b->n, nt, pr);
  const int8_t* zp = b->asym ? base + b->z_off : NULL;
  for (int kk = 0; kk < b->k; kk++) {
    int g = kk / b->bs;
    for (int nn = 0; nn < b->n; nn++) {
      size_t ci = (size_t)g * b->cstep + nn;
      int z = zp ? zp[ci] : 0;
      float s = blob_scale(b, base, g, nn);
      int8_t qv = qkn[(size_t)kk * b->n + nn];
      if (W)
        W[(size_t)kk * ldw + nn] = f4 >= 0 ? orc_f4_lut(f4, qv) * s /* f4_dequantize, kernel_ref.h:1433-1438 */
                                   : f8 ? orc_f8_to_f32(b->dtype, qv) * s /* decompress_kblock_f8_fp :1003-1026 */
                                        : (float)(qv - z) * s;            /* kernel_ref.h:1035 */
      if (Qout) Qout[(size_t)kk * b->n + nn] = qv;
    }
  }
  int nblk = (int)updiv((size_t)b->k, (size_t)b->bs);
  for (int g = 0; g < nblk; g++)
    for (int nn = 0; nn < b->n; nn++) {
      size_t ci = (size_t)g * b->cstep + nn;
      if (Sout) Sout[(size_t)g * b->n + nn] = blob_scale(b, base, g, nn);
      if (Zout) Zout[(size_t)g * b->n + nn] = zp ? zp[ci] : 0;
    }
  free(flat);
  free(qkn);
}

/* packQWeight (bestla_prologue_b.h:378-398): setQuantCorrection -> reorderWeight -> compressWeight -> reduceWeight */
static int blob_pack_q_impl(blob_t* b, int8_t* base, const int8_t* Q, int ldb, const float* S, const int8_t* Z) {
  int nt = orc_core_ntile(b->coreid), pr = orc_core_packrow(b->coreid);
  int n = b->n, k = b->k;
  int rawnk = (int)updiv((size_t)k, (size_t)b->bs);
  int nk = (int)updiv((size_t)b->kpad, (size_t)b->bs);
  uint8_t* sp = (uint8_t*)(base + b->s_off);
  if (b->has_dq) { /* packQWeight (bestla_prologue_b.h:381-386): double-quantize the [rawnk][N] scales, then
                      setQuantCorrection stores static_cast<uint8_t>(code) with zero padding (:313-329) */
    if (b->asym || nk != rawnk) return -4;
    size_t ss = (size_t)rawnk * n, nd = updiv(ss, (size_t)b->dq_bs) + 1;
    float* codes = (float*)malloc(sizeof(float) * ss);
    float* dq = (float*)calloc(nd, sizeof(float));
    memcpy(codes, S, sizeof(float) * ss);
    orc_dq8_double_quant(codes, ss, b->dq_bs, dq);
    memset(base + b->dq_off, 0, b->dq_size);
    memcpy(base + b->dq_off, dq, nd * sizeof(float)); /* setDoubleQuantCorrection :161-168 */
    for (int g = 0; g < nk; g++)
      for (int nn = 0; nn < b->npad; nn++)
        sp[(size_t)g * b->npad + nn] = (g < rawnk && nn < n) ? (uint8_t)codes[(size_t)g * n + nn] : 0;
    free(codes);
    free(dq);
  } else {
    for (int g = 0; g < nk; g++)
      for (int nn = 0; nn < b->npad; nn++) {
        float v = (g < rawnk && nn < n) ? S[(size_t)g * n + nn] : 0.f;
        put_scale(sp, (size_t)g * b->npad + nn, b->scat, v);
      }
  }
  if (b->asym) {
    int8_t* zp = base + b->z_off;
    for (int g = 0; g < nk; g++)
      for (int nn = 0; nn < b->npad; nn++) zp[(size_t)g * b->npad + nn] = (g < rawnk && nn < n) ? Z[(size_t)g * n + nn] : 0;
  }
  size_t nel = (size_t)b->npad * b->kpad;
  int8_t* reordered = (int8_t*)malloc(nel);
  orc_padding_interleave(Q, reordered, k, n, b->kpad, b->npad, ldb, b->kpad, nt, pr);
  uint8_t* q = (uint8_t*)(base + b->q_off);
  int bits = dtype_bits(b->dtype);
  if (b->dtype == ORC_F8_E4M3 || b->dtype == ORC_F8_E5M2) /* F8: reorderWeight only (bestla_prologue_b.h:1137) */
    memcpy(q, reordered, nel);
  else if (orc_f4_kind(b->dtype) >= 0) /* compress_f4 (kernel_ref.h:167-176): codes as nibbles, element 2i low */
    for (size_t e = 0; e < nel; e += 2) q[e / 2] = (uint8_t)((reordered[e] & 15) | ((reordered[e + 1] & 15) << 4));
  else if (bits == 4)
    orc_compress_s4(reordered, q, nel);
  else if (bits == 2)
    orc_compress_s2(reordered, q, nel);
  else if (bits == 8)
    memcpy(q, reordered, nel);
  else if (orc_compress_planes(bits, reordered, q, nel) != 0) {
    free(reordered);
    return -3;
  }
  free(reordered);
  if (b->has_red) {
    /* reduceWeight (bestla_prologue_b.h:455-470) + reduce/RowReduceSum (kernel_ref.h:2132-2141): sequential float
       sum over the k < K rows of each block of the dequantized weight, stored bf16 */
    float* deq = (float*)malloc(sizeof(float) * (size_t)k * n);
    blob_dequant(b, base, deq, n, NULL, NULL, NULL);
    uint16_t* rp = (uint16_t*)(base + b->r_off);
    for (int g = 0; g < rawnk; g++)
      for (int nn = 0; nn < n; nn++) {
        float t = 0.f;
        int k0 = g * b->bs, k1 = k0 + b->bs < k ? k0 + b->bs : k;
        for (int kk = k0; kk < k1; kk++) t += deq[(size_t)kk * n + nn];
        rp[(size_t)g * b->cstep + nn] = orc_f32_to_bf16(t);
      }
    free(deq);
  }
  return 0;
}

void orc_shuffle_indices(const int* g_idx, int k, int blocksize, int* out) {
  int groups = (int)updiv((size_t)k, (size_t)blocksize);
  int* cnt = (int*)calloc((size_t)groups, sizeof(int));
  for (int i = 0; i < k; i++) {
    int g = g_idx[i];
    out[(size_t)g * blocksize + cnt[g]] = i;
    cnt[g]++;
  }
  free(cnt);
}

int orc_blob_pack_q(void* buf, const int8_t* Q, const float* S, const int8_t* Z, int n, int k, int ldb, int blocksize,
                    uint32_t qtype, uint32_t stype, int asym, uint64_t core_id, const int* g_idx) {
  blob_t b;
  blob_describe(&b, n, k, blocksize, qtype, stype, asym, core_id, g_idx != NULL);
  blob_write_header(&b, (int8_t*)buf);
  if (g_idx) orc_shuffle_indices(g_idx, k, b.bs, (int*)((int8_t*)buf + b.shf_off));
  return blob_pack_q_impl(&b, (int8_t*)buf, Q, ldb, S, asym ? Z : NULL);
}

int orc_blob_quant_pack(void* buf, const float* B, int n, int k, int ldb, int blocksize, uint32_t qtype,
                        uint32_t stype, int asym, uint64_t core_id, int is_trans) {
  blob_t b;
  blob_describe(&b, n, k, blocksize, qtype, stype, asym, core_id, 0);
  blob_write_header(&b, (int8_t*)buf);
  /* packTransposeWeight (bestla_prologue_b.h:180-185): B is [N][ldb] -> transpose to [K][N] */
  float* kn = (float*)malloc(sizeof(float) * (size_t)k * n);
  for (int kk = 0; kk < k; kk++)
    for (int nn = 0; nn < n; nn++)
      kn[(size_t)kk * n + nn] = is_trans ? B[(size_t)nn * ldb + kk] : B[(size_t)kk * ldb + nn];
  int nk = (int)updiv((size_t)k, (size_t)b.bs);
  int8_t* q = (int8_t*)malloc((size_t)k * n);
  float* s = (float*)malloc(sizeof(float) * (size_t)nk * n);
  int8_t* z = asym ? (int8_t*)malloc((size_t)nk * n) : NULL;
  /* quantizeWeight (bestla_prologue_b.h:472-488) with bsize = mBlockSize (block rows align to blocksize) */
  if (orc_f4_kind(qtype) >= 0) /* WeightKBlockNFloat::quantRowBlock (bestla_prologue_b.h:1316-1338) */
    orc_quantize_f4_rowblock(kn, q, k, n, n, n, s, b.bs, orc_f4_kind(qtype));
  else if (qtype == ORC_F8_E4M3 || qtype == ORC_F8_E5M2)
    orc_quantize_f8_rowblock(kn, q, k, n, n, n, s, b.bs, qtype, stype == ORC_F8_E8M0);
  else
    orc_quantize_rowblock(kn, q, k, n, n, n, s, z, b.bs, dtype_bits(qtype));
  int r = blob_pack_q_impl(&b, (int8_t*)buf, q, n, s, z);
  free(kn);
  free(q);
  free(s);
  free(z);
  return r;
}

int orc_blob_unpack_q(const void* buf, int8_t* Q, float* S, int8_t* Z, int* shuffle) {
  blob_t b;
  int r = blob_parse(&b, buf);
  if (r) return r;
  blob_dequant(&b, (const int8_t*)buf, NULL, 0, Q, S, Z);
  if (shuffle && b.has_shf) memcpy(shuffle, (const int8_t*)buf + b.shf_off, (size_t)b.k * 4);
  return 0;
}

int orc_blob_unpack_fp32(const void* buf, float* W, int ldb) {
  blob_t b;
  int r = blob_parse(&b, buf);
  if (r) return r;
  blob_dequant(&b, (const int8_t*)buf, W, ldb, NULL, NULL, NULL);
  return 0;
}

void orc_gemm_f64(int m, int n, int k, const float* A, int lda, const float* W, int ldw, float* C, int ldc) {
  double* acc = (double*)malloc(sizeof(double) * (size_t)n);
  for (int i = 0; i < m; i++) {
    for (int j = 0; j < n; j++) acc[j] = 0.0;
    for (int kk = 0; kk < k; kk++) {
      double a = A[(size_t)i * lda + kk];
      const float* w = W + (size_t)kk * ldw;
      for (int j = 0; j < n; j++) acc[j] += a * (double)w[j];
    }
    for (int j = 0; j < n; j++) C[(size_t)i * ldc + j] = (float)acc[j];
  }
  free(acc);
}

int orc_blob_forward(const float* A, const void* blob, float* C, int m, int n, int k, int lda, int ldc) {
  blob_t b;
  int r = blob_parse(&b, blob);
  if (r) return r;
  if (b.n != n || b.k != k) return -4;
  float* W = (float*)malloc(sizeof(float) * (size_t)k * n);
  blob_dequant(&b, (const int8_t*)blob, W, n, NULL, NULL, NULL);
  const float* Ause = A;
  float* Ash = NULL;
  int ld = lda;
  if (b.has_shf) { /* ShuffleActivationKBlockBase: A'[:, j] = A[:, idx[j]] (kernel_ref.h:27-37) */
    const int* idx = (const int*)((const int8_t*)blob + b.shf_off);
    Ash = (float*)malloc(sizeof(float) * (size_t)m * k);
    for (int i = 0; i < m; i++)
      for (int j = 0; j < k; j++) Ash[(size_t)i * k + j] = A[(size_t)i * lda + idx[j]];
    Ause = Ash;
    ld = k;
  }
  orc_gemm_f64(m, n, k, Ause, ld, W, n, C, ldc);
  free(W);
  free(Ash);
  return 0;
}

/* kernel_ref.h:2489-2531 / 2712-2760 driven over the NTILE stripes of a PACK_ROW=1 blob as GEMVWrapper::gemv_kblock
   does (bestla_wrapper.h:364-427); requires K % blocksize == 0 (blks = k / blocksize). */
int orc_blob_gemv_ref(const float* A, const void* blob, float* C, int m, int lda, int ldc) {
  blob_t b;
  int r = blob_parse(&b, blob);
  if (r) return r;
  int nt = orc_core_ntile(b.coreid);
  if (orc_core_packrow(b.coreid) != 1 || m > 8 || b.has_shf) return -5;
  int bits = dtype_bits(b.dtype);
  if (bits != 4 && bits != 2) return -6;
  const uint8_t* q = (const uint8_t*)((const int8_t*)blob + b.q_off);
  const uint8_t* sp = (const uint8_t*)((const int8_t*)blob + b.s_off);
  const int8_t* zp = b.asym ? (const int8_t*)blob + b.z_off : NULL;
  int blks = b.k / b.bs;
  float* acc = (float*)malloc(sizeof(float) * (size_t)nt * m);
  for (int n0 = 0; n0 < b.n; n0 += nt) {
    memset(acc, 0, sizeof(float) * (size_t)nt * m);
    const uint8_t* bp = q + (size_t)n0 * b.kpad * bits / 8;
    for (int ib = 0; ib < blks; ib++) {
      for (int ik = 0; ik < b.bs; ik++) {
        int kk = ib * b.bs + ik;
        for (int im = 0; im < m; im++) {
          float aval = A[(size_t)im * lda + kk];
          for (int in = 0; in < nt; in++) {
            size_t ci = (size_t)ib * b.cstep + n0 + in;
            int qv;
            if (bits == 4)
              qv = ((bp[(size_t)kk * nt / 2 + in / 2] >> (4 * (in & 1))) & 0xF) - 8;
            else
              qv = ((bp[((size_t)kk * nt + in) / 4] >> (2 * (in & 3))) & 3) - 2;
            float z = zp ? (float)zp[ci] : 0.f;
            if (bits == 4) /* kernel_ref.h:2505-2506: aval * (q - zp) * s */
              acc[im * nt + in] += aval * ((float)qv - z) * get_scale(sp, ci, b.scat);
            else /* kernel_ref.h:2733-2735: bval = (q - zp) * s; acc += aval * bval */
              acc[im * nt + in] += aval * (((float)qv - z) * get_scale(sp, ci, b.scat));
          }
        }
      }
    }
    for (int im = 0; im < m; im++)
      for (int in = 0; in < nt && n0 + in < b.n; in++) C[(size_t)im * ldc + n0 + in] = acc[im * nt + in];
  }
  free(acc);
  return 0;
}

/* The same scalar GEMV, its independent NTILE column blocks spread over `threads` OpenMP threads (every output is
 * computed by exactly the code and order of orc_blob_gemv_ref: bit-identical).  CPU-baseline timing only. */
int orc_blob_gemv_par(const float* A, const void* blob, float* C, int m, int lda, int ldc, int threads) {
  blob_t b;
  int r = blob_parse(&b, blob);
  if (r) return r;
  int nt = orc_core_ntile(b.coreid);
  if (orc_core_packrow(b.coreid) != 1 || m > 8 || b.has_shf) return -5;
  int bits = dtype_bits(b.dtype);
  if (bits != 4 && bits != 2) return -6;
  const uint8_t* q = (const uint8_t*)((const int8_t*)blob + b.q_off);
  const uint8_t* sp = (const uint8_t*)((const int8_t*)blob + b.s_off);
  const int8_t* zp = b.asym ? (const int8_t*)blob + b.z_off : NULL;
  int blks = b.k / b.bs;
  int nblk = (b.n + nt - 1) / nt;
#pragma omp parallel for schedule(static) num_threads(threads)
  for (int blk = 0; blk < nblk; blk++) {
    int n0 = blk * nt;
    float acc[48 * 8];
    memset(acc, 0, sizeof(float) * (size_t)nt * m);
    const uint8_t* bp = q + (size_t)n0 * b.kpad * bits / 8;
    for (int ib = 0; ib < blks; ib++) {
      for (int ik = 0; ik < b.bs; ik++) {
        int kk = ib * b.bs + ik;
        for (int im = 0; im < m; im++) {
          float aval = A[(size_t)im * lda + kk];
          for (int in = 0; in < nt; in++) {
            size_t ci = (size_t)ib * b.cstep + n0 + in;
            int qv;
            if (bits == 4)
              qv = ((bp[(size_t)kk * nt / 2 + in / 2] >> (4 * (in & 1))) & 0xF) - 8;
            else
              qv = ((bp[((size_t)kk * nt + in) / 4] >> (2 * (in & 3))) & 3) - 2;
            float z = zp ? (float)zp[ci] : 0.f;
            if (bits == 4)
              acc[im * nt + in] += aval * ((float)qv - z) * get_scale(sp, ci, b.scat);
            else
              acc[im * nt + in] += aval * (((float)qv - z) * get_scale(sp, ci, b.scat));
          }
        }
      }
    }
    for (int im = 0; im < m; im++)
      for (int in = 0; in < nt && n0 + in < b.n; in++) C[(size_t)im * ldc + n0 + in] = acc[im * nt + in];
  }
  return 0;
}

int orc_blob_gemv_timed(const float* A, const void* blob, float* C, int m, int lda, int ldc, int iters) {
  int r = 0;
  for (int it = 0; it < iters && r == 0; it++) r = orc_blob_gemv_ref(A, blob, C, m, lda, ldc);
  return r;
}

/* ------------------------------------------------------------------ int8 compute (comp_int8) */
/* bestla_utils.h cast<float,uint8_t>: +0.5, clamp to [0,255], truncating conversion (x86 cvttss2si, low byte) */
static inline uint8_t cast_f32_u8(float v) {
  v += 0.5f;
  v = smin(v, 255.f);
  v = smax(v, 0.f);
  return (uint8_t)(f2i_x86(v) & 0xff);
}

/* kernel_ref.h:1824-1883 quantize_fp_u8_colblock: per (row, block of `blocksize` columns) asymmetric u8.  Full blocks
   start the running max at FLT_MIN (std::numeric_limits<float>::min()), the ragged tail block at 0. */
static void quant_u8_block(const float* x, int len, float maxinit, uint8_t* dst, float* scale_out, uint8_t* zp_out,
                           float* red_out) {
  float maxval = maxinit, minval = 0.f;
  for (int j = 0; j < len; j++) {
    maxval = smax(x[j], maxval);
    minval = smin(x[j], minval);
  }
  float scale = (maxval - minval) / 255;
  uint8_t zp = cast_f32_u8((0 - minval) / scale);
  float rscale = 1.f / scale;
  *scale_out = scale;
  *zp_out = zp;
  int32_t sum = 0;
  float zpf = (float)zp;
  for (int j = 0; j < len; j++) {
    int32_t q = cast_f32_int(x[j] * rscale);
    sum = iadd_wrap(sum, q);
    dst[j] = cast_f32_u8(zpf + (float)q);
  }
  if (red_out) *red_out = (float)sum * scale;
}

void orc_quant_u8_colblock(int row, int col, const float* src, int ld_src, uint8_t* dst, int ld_dst, float* scales,
                           int ld_scale, uint8_t* zps, int blocksize, float* blkreduce) {
  int colblk = (col / blocksize) * blocksize;
  for (int i = 0; i < row; i++) {
    int j = 0;
    for (; j < colblk; j += blocksize) {
      size_t si = (size_t)(j / blocksize) + (size_t)i * ld_scale;
      quant_u8_block(src + (size_t)i * ld_src + j, blocksize, FLT_MIN, dst + (size_t)i * ld_dst + j, scales + si,
                     zps + si, blkreduce ? blkreduce + si : NULL);
    }
    if (j < col) {
      size_t si = (size_t)(j / blocksize) + (size_t)i * ld_scale;
      quant_u8_block(src + (size_t)i * ld_src + j, col - j, 0.f, dst + (size_t)i * ld_dst + j, scales + si, zps + si,
                     blkreduce ? blkreduce + si : NULL);
    }
  }
}

/* LauncherIntKBlock::run_block (bestla_wrapper.h:768-831) with a kblock u8s8 core (bestla_gemm.h:2899-3050): the
   activation (act-order gathered first, bestla_prologue_a.h:407-422) is quantized per (row, weight block) by
   quantize_fp_u8_colblock; per block: s32 = sum a_u8 * (q - zp), then C += float(s32) * (sA * sB) and
   C -= (float(zpA) * sA * 1.f) * reduceB, blocks in K order.  reduceB is the blob's bf16 reduce (Sum_k dequant(w)). */
int orc_blob_forward_int8(const float* A, const void* blob, float* C, int m, int n, int k, int lda, int ldc) {
  blob_t b;
  int r = blob_parse(&b, blob);
  if (r) return r;
  if (b.n != n || b.k != k) return -4;
  if (!b.has_red) return -5;
  const int8_t* base = (const int8_t*)blob;
  int nblk = (int)updiv((size_t)k, (size_t)b.bs);
  int8_t* Q = (int8_t*)malloc((size_t)k * n);
  float* S = (float*)malloc(sizeof(float) * (size_t)nblk * n);
  int8_t* Z = (int8_t*)malloc((size_t)nblk * n);
  blob_dequant(&b, base, NULL, 0, Q, S, Z);
  const uint16_t* red = (const uint16_t*)(base + b.r_off);
  float* Ash = (float*)malloc(sizeof(float) * (size_t)m * k);
  const int* idx = b.has_shf ? (const int*)(base + b.shf_off) : NULL;
  for (int i = 0; i < m; i++)
    for (int j = 0; j < k; j++) Ash[(size_t)i * k + j] = A[(size_t)i * lda + (idx ? idx[j] : j)];
  uint8_t* a8 = (uint8_t*)malloc((size_t)m * k);
  float* sa = (float*)malloc(sizeof(float) * (size_t)m * nblk);
  uint8_t* za = (uint8_t*)malloc((size_t)m * nblk);
  orc_quant_u8_colblock(m, k, Ash, k, a8, k, sa, nblk, za, b.bs, NULL);
  for (int i = 0; i < m; i++)
    for (int nn = 0; nn < n; nn++) {
      float c = 0.f;
      for (int g = 0; g < nblk; g++) {
        int k0 = g * b.bs, k1 = k0 + b.bs < k ? k0 + b.bs : k;
        int zb = Z[(size_t)g * n + nn];
        int32_t dot = 0;
        for (int kk = k0; kk < k1; kk++)
          dot += (int32_t)a8[(size_t)i * k + kk] * (int32_t)(Q[(size_t)kk * n + nn] - zb);
        float sA = sa[(size_t)i * nblk + g], sB = S[(size_t)g * n + nn];
        float t = sA * sB;
        c = c + (float)dot * t;
        float zc = (float)za[(size_t)i * nblk + g] * sA * 1.f;
        c = c - zc * orc_bf16_to_f32(red[(size_t)g * b.cstep + nn]);
      }
      C[(size_t)i * ldc + nn] = c;
    }
  free(Q);
  free(S);
  free(Z);
  free(Ash);
  free(a8);
  free(sa);
  free(za);
  return 0;
}

/* kernel_ref.h:2371-2429 gemv_4bit_u8s8_fp32 restated over unpacked operands: a8 [m][k] u8, as/azp [m][nblk],
   q [k][n] signed int4 values (nibble - 8), s [nblk][n], zp [nblk][n] (NULL: symmetric).  Float accumulation per
   element in the reference's order: blocks, then k in fours, then the four k of a PACK_ROW group. */
void orc_gemv_u8s8_ref(int m, int n, int k, int bs, const uint8_t* a8, const float* as, const uint8_t* azp,
                       const int8_t* q, const float* s, const int8_t* zp, float* C) {
  int blks = k / bs;
  for (int im = 0; im < m; im++)
    for (int in = 0; in < n; in++) {
      float acc = 0.f;
      for (int ib = 0; ib < blks; ib++) {
        int az = azp[(size_t)im * blks + ib];
        float asc = as[(size_t)im * blks + ib];
        float vscale = asc * s[(size_t)ib * n + in];
        int bz = zp ? zp[(size_t)ib * n + in] : 0;
        for (int ik = 0; ik < bs; ik++) {
          int kk = ib * bs + ik;
          int prod = ((int)a8[(size_t)im * k + kk] - az) * ((int)q[(size_t)kk * n + in] - bz);
          acc += (float)prod * vscale;
        }
      }
      C[(size_t)im * n + in] = acc;
    }
}

/* ------------------------------------------------------------------ GGUF Q4_0 x Q8_0 */
/* block layouts (neural_speed/core/data_types.h:79-83 and the Q8_0 block beside it): q4_0 = {fp16 d; u8 qs[16]} (18 B,
   element j < 16 in the low nibble of qs[j], element j >= 16 in the high nibble of qs[j - 16]); q8_0 = {fp16 d;
   s8 qs[32]} (34 B). */
static inline uint32_t f2b(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
static inline float b2f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
/* data_types.h:204-228 ne_compute_fp32_to_fp16 */
uint16_t orc_ne_fp32_to_fp16(float f) {
  const float scale_to_inf = 0x1.0p+112f, scale_to_zero = 0x1.0p-110f;
  float base = (fabsf(f) * scale_to_inf) * scale_to_zero;
  const uint32_t w = f2b(f), shl1_w = w + w, sign = w & 0x80000000u;
  uint32_t bias = shl1_w & 0xFF000000u;
  if (bias < 0x71000000u) bias = 0x71000000u;
  base = b2f((bias >> 1) + 0x07800000u) + base;
  const uint32_t bits = f2b(base);
  const uint32_t exp_bits = (bits >> 13) & 0x00007C00u, mantissa_bits = bits & 0x00000FFFu;
  const uint32_t nonsign = exp_bits + mantissa_bits;
  return (uint16_t)((sign >> 16) | (shl1_w > 0xFF000000u ? 0x7E00u : nonsign));
}
/* data_types.h ne_compute_fp16_to_fp32 (exact) */
float orc_ne_fp16_to_fp32(uint16_t h) { return orc_fp16_to_f32(h); }

/* vectors/cpu/quantize.h:243-276 quantize_row_q4_0_reference */
void orc_q4_0_quantize_row(const float* x, uint8_t* y, int k) {
  const int qk = 32, nb = k / qk;
  for (int i = 0; i < nb; i++) {
    float amax = 0.0f, max = 0.0f;
    for (int j = 0; j < qk; j++) {
      const float v = x[i * qk + j];
      if (amax < fabsf(v)) {
        amax = fabsf(v);
        max = v;
      }
    }
    const float d = max / -8;
    const float id = d ? 1.0f / d : 0.0f;
    uint8_t* blk = y + (size_t)i * 18;
    uint16_t dh = orc_ne_fp32_to_fp16(d);
    memcpy(blk, &dh, 2);
    for (int j = 0; j < qk / 2; ++j) {
      const float x0 = x[i * qk + 0 + j] * id;
      const float x1 = x[i * qk + qk / 2 + j] * id;
      int8_t t0 = (int8_t)(x0 + 8.5f), t1 = (int8_t)(x1 + 8.5f);
      const uint8_t xi0 = (uint8_t)(15 < t0 ? 15 : t0);
      const uint8_t xi1 = (uint8_t)(15 < t1 ? 15 : t1);
      blk[2 + j] = (uint8_t)(xi0 | (xi1 << 4));
    }
  }
}

/* vectors/cpu/quantize.h:686-704 dequantize_row_q4_0 */
void orc_q4_0_dequantize_row(const uint8_t* x, float* y, int k) {
  const int qk = 32, nb = k / qk;
  for (int i = 0; i < nb; i++) {
    uint16_t dh;
    memcpy(&dh, x + (size_t)i * 18, 2);
    const float d = orc_ne_fp16_to_fp32(dh);
    const uint8_t* qs = x + (size_t)i * 18 + 2;
    for (int j = 0; j < qk / 2; ++j) {
      const int x0 = (qs[j] & 0x0F) - 8, x1 = (qs[j] >> 4) - 8;
      y[i * qk + j + 0] = x0 * d;
      y[i * qk + j + qk / 2] = x1 * d;
    }
  }
}

/* vectors/cpu/quantize.h:422-445 quantize_row_q8_0_reference */
void orc_q8_0_quantize_row(const float* x, uint8_t* y, int k) {
  const int nb = k / 32;
  for (int i = 0; i < nb; i++) {
    float amax = 0.0f;
    for (int j = 0; j < 32; j++) {
      const float v = fabsf(x[i * 32 + j]);
      amax = amax > v ? amax : v;
    }
    const float d = amax / ((1 << 7) - 1);
    const float id = d ? 1.0f / d : 0.0f;
    uint8_t* blk = y + (size_t)i * 34;
    uint16_t dh = orc_ne_fp32_to_fp16(d);
    memcpy(blk, &dh, 2);
    for (int j = 0; j < 32; ++j) ((int8_t*)blk)[2 + j] = (int8_t)roundf(x[i * 32 + j] * id);
  }
}

/* neural_speed/core/layers/vec_dot.h:187-204 ne_vec_dot_q4_0_q8_0, scalar path */
float orc_vec_dot_q4_0_q8_0(int n, const uint8_t* vx, const uint8_t* vy) {
  const int qk = 32, nb = n / qk;
  float sumf = 0.0f;
  for (int i = 0; i < nb; i++) {
    const uint8_t* xb = vx + (size_t)i * 18;
    const uint8_t* yb = vy + (size_t)i * 34;
    const int8_t* yq = (const int8_t*)(yb + 2);
    int sumi = 0;
    for (int j = 0; j < qk / 2; ++j) {
      const int v0 = (xb[2 + j] & 0x0F) - 8, v1 = (xb[2 + j] >> 4) - 8;
      sumi += (v0 * yq[j]) + (v1 * yq[j + qk / 2]);
    }
    uint16_t dx, dy;
    memcpy(&dx, xb, 2);
    memcpy(&dy, yb, 2);
    sumf += sumi * orc_ne_fp16_to_fp32(dx) * orc_ne_fp16_to_fp32(dy);
  }
  return sumf;
}

/* ne_compute_forward_mul_mat for a Q4_0 src0 (ne_layers.c: src1 rows quantized by vec_dot_type = Q8_0, then one
   vec_dot per output): W = [n][k/32] q4_0 blocks, A [m][k] f32 -> C [m][n] */
int orc_q4_0_forward(const float* A, const uint8_t* W, float* C, int m, int n, int k) {
  if (k % 32) return -1;
  uint8_t* q8 = (uint8_t*)malloc((size_t)(k / 32) * 34);
  for (int i = 0; i < m; i++) {
    orc_q8_0_quantize_row(A + (size_t)i * k, q8, k);
    for (int j = 0; j < n; j++) C[(size_t)i * n + j] = orc_vec_dot_q4_0_q8_0(k, W + (size_t)j * (k / 32) * 18, q8);
  }
  free(q8);
  return 0;
}

/* ------------------------------------------------------------------ 1/3/5/6/7-bit planes */
/* kernel_ref.h:178-341 compress_{7,6,5,3}bit with the plane layout of compressBitNWeight (bestla_prologue_b.h:512-546):
   stored u = q + 2^(bits-1) split into a nibble plane (bit4x2: element 2i in the low nibble of byte i), a crumb plane
   (bit2x4: element 4i + j at bits 2j of byte i) and a bit plane (bit1x8: element 8i + j at bit j of byte i):
   3 = crumb [n/4] | bit [n/8];  5 = nibble [n/2] | bit [n/8];  6 = nibble [n/2] | crumb [n/4];
   7 = nibble [n/2] | crumb [n/4] | bit [n/8]; the high part of u sits in the later plane(s).
   1 = bit [n/8] (compress_1bit, kernel_ref.h:343-361), which stores element 8i + 4 from srcptr[8i + FullRange] =
   srcptr[8i + 1]: reproduced, so blobs match the reference byte for byte (golden compress_bit1). */
static void planes(int bits, size_t n, size_t* o4, size_t* o2, size_t* o1) {
  *o4 = *o2 = *o1 = (size_t)-1;
  switch (bits) {
    case 1: *o1 = 0; break;
    case 3: *o2 = 0; *o1 = n / 4; break;
    case 5: *o4 = 0; *o1 = n / 2; break;
    case 6: *o4 = 0; *o2 = n / 2; break;
    case 7: *o4 = 0; *o2 = n / 2; *o1 = n / 2 + n / 4; break;
    default: break;
  }
}
int orc_compress_planes(int bits, const int8_t* src, uint8_t* dst, size_t n) {
  size_t o4, o2, o1;
  planes(bits, n, &o4, &o2, &o1);
  if (o2 == (size_t)-1 && o1 == (size_t)-1) return -1;
  memset(dst, 0, n * bits / 8);
  for (size_t e = 0; e < n; e++) {
    unsigned u = (unsigned)(src[bits == 1 && (e & 7) == 4 ? e - 3 : e] + (1 << (bits - 1)));
    int sh = 0;
    if (o4 != (size_t)-1) {
      dst[o4 + e / 2] |= (uint8_t)((u & 15u) << (4 * (e & 1)));
      sh = 4;
    }
    if (o2 != (size_t)-1) {
      dst[o2 + e / 4] |= (uint8_t)(((u >> sh) & 3u) << (2 * (e & 3)));
      sh += 2;
    }
    if (o1 != (size_t)-1) dst[o1 + e / 8] |= (uint8_t)(((u >> sh) & 1u) << (e & 7));
  }
  return 0;
}
/* decompress_s{1,3,5,6,7}_s8 (kernel_ref.h:412-525) */
int orc_decompress_planes(int bits, const uint8_t* src, int8_t* dst, size_t n) {
  size_t o4, o2, o1;
  planes(bits, n, &o4, &o2, &o1);
  if (o2 == (size_t)-1 && o1 == (size_t)-1) return -1;
  for (size_t e = 0; e < n; e++) {
    unsigned u = 0;
    int sh = 0;
    if (o4 != (size_t)-1) {
      u = (src[o4 + e / 2] >> (4 * (e & 1))) & 15u;
      sh = 4;
    }
    if (o2 != (size_t)-1) {
      u |= ((src[o2 + e / 4] >> (2 * (e & 3))) & 3u) << sh;
      sh += 2;
    }
    if (o1 != (size_t)-1) u |= ((src[o1 + e / 8] >> (e & 7)) & 1u) << sh;
    dst[e] = (int8_t)((int)u - (1 << (bits - 1)));
  }
  return 0;
}

/* ------------------------------------------------------------------ NFloat 4-bit weights (F4_BNB, F4_E2M1, F4_NF4) */
/* dequant LUTs: bestla_utils.h:749-790 (the values the reference's unpack trees kernel_ref.h:1195-1360 return) */
static const float k_f4_lut[3][16] = {
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
/* f4 kind: 0 = F4_BNB (0x10004), 1 = F4_E2M1 (0x4 | float), 2 = F4_NF4 */
int orc_f4_kind(uint32_t qtype) {
  if (qtype == ORC_F4_BNB) return 0;
  if (qtype == ORC_F4_E2M1) return 1;
  if (qtype == ORC_F4_NF4) return 2;
  return -1;
}
float orc_f4_lut(int kind, int code) { return k_f4_lut[kind][code & 15]; }

/* kernel_ref.h:1233-1254 fp4_bnb_quantize */
static int8_t f4_bnb_q(float x) {
  int sign = x < 0 ? 0x8 : 0;
  x = fabsf(x);
  if (x > 0.29166667f) {
    if (x > 0.583333f) return (int8_t)((x > 0.8333333f ? 0x3 : 0x2) + sign);
    return (int8_t)((x > 0.4166667f ? 0x5 : 0x4) + sign);
  }
  if (x > 0.0859375f) return (int8_t)((x > 0.20833333f ? 0x7 : 0x6) + sign);
  return (int8_t)((x > 0.00260417f ? 0x1 : 0x0) + sign);
}
/* kernel_ref.h:1256-1297 fp4_e2m1_quantize */
static int8_t f4_e2m1_q(float x) {
  int sign = x < 0 ? 0x8 : 0;
  x = fabsf(x);
  if (x > 1.75f / 6) {
    if (x > 3.5f / 6) return (int8_t)((x > 5.f / 6 ? 0x7 : 0x6) + sign);
    return (int8_t)((x > 2.5f / 6 ? 0x5 : 0x4) + sign);
  }
  if (x > 0.53125f / 6) return (int8_t)((x > 1.25f / 6 ? 0x3 : 0x2) + sign);
  return (int8_t)((x > 0.03125f / 6 ? 0x1 : 0x0) + sign);
}
/* kernel_ref.h:1373-1419 nf4_quantize (codes of 0 and -1 swapped so that 0 pads as 0) */
static int8_t f4_nf4_q(float x) {
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
int8_t orc_f4_quantize(int kind, float x) {
  return kind == 0 ? f4_bnb_q(x) : (kind == 1 ? f4_e2m1_q(x) : f4_nf4_q(x));
}
/* kernel_ref.h:1800-1822 quantize_f32_f4_rowblock: per (column, K block) absmax (running max from FLT_MIN) -> scale;
   code = f4_quantize(x * (1 / absmax)) */
void orc_quantize_f4_rowblock(const float* src, int8_t* dst, int row, int col, int ld_src, int ld_dst, float* scales,
                              int blocksize, int kind) {
  for (int i = 0; i < col; i++) {
    int align = row / blocksize * blocksize;
    for (int j = 0; j < row; j += blocksize) {
      int bs = j < align ? blocksize : row - align;
      float absmax = FLT_MIN;
      for (int ij = 0; ij < bs; ij++) absmax = smax(absmax, fabsf(src[(size_t)(j + ij) * ld_src + i]));
      scales[(size_t)(j / blocksize) * ld_dst + i] = absmax;
      for (int ij = 0; ij < bs; ij++)
        dst[(size_t)(j + ij) * ld_dst + i] = orc_f4_quantize(kind, src[(size_t)(j + ij) * ld_src + i] * (1.f / absmax));
    }
  }
}

/* ------------------------------------------------------------------ NFloat 8-bit weights (F8_E4M3, F8_E5M2) */
/* bestla_utils.h:414-454 (ebits, quant mantissa bits, mx max norm) */
static int f8_ebits(uint32_t t) { return t == ORC_F8_E4M3 ? 4 : 5; }
static int f8_qmbits(uint32_t t) { return t == ORC_F8_E4M3 ? 5 : 4; }
static float f8_maxnorm(uint32_t t) {
  int ebits = f8_ebits(t), mb = f8_qmbits(t);
  double emax = pow(2, ebits - 1);
  if (t == ORC_F8_E5M2) emax -= 1;
  double max_norm = pow(2, emax);
  if (t != ORC_F8_E4M3)
    max_norm *= ((pow(2, mb - 1) - 1) / pow(2, mb - 2));
  else
    max_norm *= 1.75;
  return (float)max_norm;
}
/* kernel_ref.h:1721-1762 f8_mx_quantize (float / double steps as the reference's std:: overloads resolve them) */
int8_t orc_f8_quantize(uint32_t t, float v, float scale, int e8m0) {
  if (e8m0)
    v /= (float)pow(2, scale);
  else
    v /= scale;
  const int ebits = f8_ebits(t), qm = f8_qmbits(t), store_mantissa = 7 - ebits;
  float private_exp = floorf(log2f(fabsf(v == 0 ? v + 1 : v)));
  const float min_exp = (float)(-1 * (pow(2, ebits - 1)) + 2);
  private_exp = private_exp < min_exp ? min_exp : private_exp;
  v = (float)(v / pow(2, private_exp) * pow(2, qm - 2));
  const int sign = v > 0 ? 1 : -1;
  v = sign * (float)floor(fabsf(v) + 0.5);
  v = (float)(v / pow(2, qm - 2) * pow(2, private_exp));
  const float max_norm = f8_maxnorm(t);
  v = v < -1 * max_norm ? -1 * max_norm : (v > max_norm ? max_norm : v); /* std::clamp */
  uint32_t u;
  memcpy(&u, &v, 4);
  const uint8_t store_signbit = (uint8_t)((u >> 24) & 0x80);
  u <<= 1;
  uint8_t store_ebit = (uint8_t)(u >> 24);
  store_ebit = (uint8_t)(store_ebit - 127 + (uint8_t)pow(2, ebits - 1) - 1);
  if (store_ebit > 15 && t == ORC_F8_E4M3) store_ebit = 0;
  if (store_ebit > 31 && t == ORC_F8_E5M2) store_ebit = 0;
  store_ebit = (uint8_t)(store_ebit << store_mantissa);
  u <<= 8;
  const int8_t mask = (int8_t)(-128 >> (store_mantissa - 1));
  uint8_t store_mantissabit = (uint8_t)((u >> 24) & (uint8_t)mask);
  store_mantissabit = (uint8_t)(store_mantissabit >> (1 + ebits));
  return (int8_t)(store_signbit | store_ebit | store_mantissabit);
}
/* kernel_ref.h:984-1001 f8_to_fp32: the exponent field is always read as a normal one (no subnormals) */
float orc_f8_to_f32(uint32_t t, int8_t code) {
  uint32_t x = (uint32_t)(int32_t)code;
  uint32_t s = (x << 24) & 0x80000000u;
  const int ebits = f8_ebits(t), mb = 7 - ebits;
  uint32_t e = (x & 0x7f) >> mb;
  e = e - (uint32_t)pow(2, ebits - 1) + 1 + 127;
  e <<= 23;
  uint32_t m = (x << (23 - mb)) & 0x007fffffu;
  uint32_t r = s | e | m;
  float f;
  memcpy(&f, &r, 4);
  return f;
}
/* kernel_ref.h:1764-1800 quantize_f32_f8_rowblock_mxscale; e8m0: scales hold the (float) shared exponent */
void orc_quantize_f8_rowblock(const float* src, int8_t* dst, int row, int col, int ld_src, int ld_dst, float* scales,
                              int blocksize, uint32_t t, int e8m0) {
  for (int i = 0; i < col; i++) {
    int align = row / blocksize * blocksize;
    for (int j = 0; j < row; j += blocksize) {
      int bs = j < align ? blocksize : row - align;
      float scale = FLT_MIN;
      for (int ij = 0; ij < bs; ij++) scale = smax(scale, fabsf(src[(size_t)(j + ij) * ld_src + i]));
      if (e8m0) {
        if (scale == 0) scale += fabsf(FLT_MIN);
        scale = floorf(log2f(scale));
        float emax = (float)pow(2, f8_ebits(t) - 1);
        if (t == ORC_F8_E5M2) emax -= 1;
        scale -= emax;
        const float scale_max = (float)pow(2, 7) - 1;
        scale = scale < (-1 * scale_max) ? (-1 * scale_max) : scale;
      } else {
        scale /= f8_maxnorm(t);
      }
      scales[(size_t)(j / blocksize) * ld_dst + i] = scale;
      for (int ij = 0; ij < bs; ij++)
        dst[(size_t)(j + ij) * ld_dst + i] = orc_f8_quantize(t, src[(size_t)(j + ij) * ld_src + i], scale, e8m0);
    }
  }
}

/* The CPU baseline's GEMV with AVX-512 (test infrastructure: bench.py cpu_baseline only): the arithmetic of
 * orc_blob_gemv_ref for int4 weights at m = 1 on an NTILE-48 PACK_ROW-1 blob, reassociated the way a SIMD kernel does
 * it -- per quantization block t[col] = sum_k a_k * nibble_k by FMA chains (16 columns per zmm, the columns of a byte's
 * low and high nibbles in separate accumulators, one interleave per block), then acc += (t - (8 + zp) sum_k a_k) s with
 * the block's scales converted 16 at a time (F16C / bf16 shift) -- within
 * fp32 reassociation of the scalar restatement (tests/test_oracle_golden.py::test_avx512_gemv_matches_scalar).  The
 * reference's own AVX512F / AMX cores (kernel_avx512f.h, bestla_gemm.h) need xbyak and are unbuildable here.
 * Returns -7 when the host has no AVX-512 (the caller falls back to orc_blob_gemv_par). */
#include <immintrin.h>

__attribute__((target("avx512f,avx512bw,avx2,fma,f16c"))) static __m512 scales16(const uint8_t* sp, size_t ci,
                                                                                  uint32_t scat) {
  if (scat == ORC_F32) return _mm512_loadu_ps((const float*)(sp + ci * 4));
  const __m256i h = _mm256_loadu_si256((const __m256i*)(sp + ci * 2));
  if (scat == ORC_BF16) return _mm512_castsi512_ps(_mm512_slli_epi32(_mm512_cvtepu16_epi32(h), 16));
  return _mm512_cvtph_ps(h);
}

__attribute__((target("avx512f,avx512bw,avx2,fma,f16c"))) static void gemv4_nt48_avx512(const float* A,
                                                                                        const uint8_t* bp,
                                                                                        const uint8_t* sp,
                                                                                        const int8_t* zp,
                                                                                        const blob_t* b, int n0,
                                                                                        float* out) {
  const int nt = 48, blks = b->k / b->bs;
  /* accumulator lanes: L0 = low nibbles of bytes 0-15 (columns 0, 2, .., 30), H0 = their high nibbles (1, 3, .., 31),
     L1 / H1 the same for bytes 16-23 (columns 32 .. 47); one interleave per block restores column order */
  const __m512i ia = _mm512_setr_epi32(0, 16, 1, 17, 2, 18, 3, 19, 4, 20, 5, 21, 6, 22, 7, 23);
  const __m512i ib_ = _mm512_setr_epi32(8, 24, 9, 25, 10, 26, 11, 27, 12, 28, 13, 29, 14, 30, 15, 31);
  const __m512i m15 = _mm512_set1_epi32(15);
  const __m256i m15y = _mm256_set1_epi32(15);
  const __m512 c8 = _mm512_set1_ps(8.f);
  __m512 acc0 = _mm512_setzero_ps(), acc1 = _mm512_setzero_ps(), acc2 = _mm512_setzero_ps();
  for (int ib = 0; ib < blks; ib++) {
    __m512 tl0 = _mm512_setzero_ps(), th0 = _mm512_setzero_ps();
    __m256 tl1 = _mm256_setzero_ps(), th1 = _mm256_setzero_ps();
    float asum = 0.f;
    const uint8_t* p = bp + (size_t)ib * b->bs * nt / 2;
    const float* ak = A + (size_t)ib * b->bs;
    for (int ik = 0; ik < b->bs; ik++, p += nt / 2) {
      const float av = ak[ik];
      asum += av;
      const __m512 a = _mm512_set1_ps(av);
      const __m512i x0 = _mm512_cvtepu8_epi32(_mm_loadu_si128((const __m128i*)p));
      const __m256i x1 = _mm256_cvtepu8_epi32(_mm_loadl_epi64((const __m128i*)(p + 16)));
      tl0 = _mm512_fmadd_ps(a, _mm512_cvtepi32_ps(_mm512_and_si512(x0, m15)), tl0);
      th0 = _mm512_fmadd_ps(a, _mm512_cvtepi32_ps(_mm512_srli_epi32(x0, 4)), th0);
      tl1 = _mm256_fmadd_ps(_mm512_castps512_ps256(a), _mm256_cvtepi32_ps(_mm256_and_si256(x1, m15y)), tl1);
      th1 = _mm256_fmadd_ps(_mm512_castps512_ps256(a), _mm256_cvtepi32_ps(_mm256_srli_epi32(x1, 4)), th1);
    }
    const __m512 t0 = _mm512_permutex2var_ps(tl0, ia, th0), t1 = _mm512_permutex2var_ps(tl0, ib_, th0);
    const __m512 t2 = _mm512_permutex2var_ps(_mm512_castps256_ps512(tl1), ia, _mm512_castps256_ps512(th1));
    const size_t ci = (size_t)ib * b->cstep + n0;
    __m512 z0 = c8, z1 = c8, z2 = c8;
    if (zp) {
      z0 = _mm512_add_ps(c8, _mm512_cvtepi32_ps(_mm512_cvtepi8_epi32(_mm_loadu_si128((const __m128i*)(zp + ci)))));
      z1 = _mm512_add_ps(c8, _mm512_cvtepi32_ps(_mm512_cvtepi8_epi32(_mm_loadu_si128((const __m128i*)(zp + ci + 16)))));
      z2 = _mm512_add_ps(c8, _mm512_cvtepi32_ps(_mm512_cvtepi8_epi32(_mm_loadu_si128((const __m128i*)(zp + ci + 32)))));
    }
    const __m512 as = _mm512_set1_ps(asum);
    acc0 = _mm512_fmadd_ps(_mm512_fnmadd_ps(z0, as, t0), scales16(sp, ci, b->scat), acc0);
    acc1 = _mm512_fmadd_ps(_mm512_fnmadd_ps(z1, as, t1), scales16(sp, ci + 16, b->scat), acc1);
    acc2 = _mm512_fmadd_ps(_mm512_fnmadd_ps(z2, as, t2), scales16(sp, ci + 32, b->scat), acc2);
  }
  _mm512_storeu_ps(out, acc0);
  _mm512_storeu_ps(out + 16, acc1);
  _mm512_storeu_ps(out + 32, acc2);
}

int orc_blob_gemv_avx512(const float* A, const void* blob, float* C, int k_ld, int threads) {
  (void)k_ld;
  if (!__builtin_cpu_supports("avx512f") || !__builtin_cpu_supports("avx512bw")) return -7;
  blob_t b;
  int r = blob_parse(&b, blob);
  if (r) return r;
  if (orc_core_ntile(b.coreid) != 48 || orc_core_packrow(b.coreid) != 1 || b.has_shf || b.has_dq) return -5;
  if (dtype_bits(b.dtype) != 4) return -6;
  if (b.scat != ORC_F32 && b.scat != ORC_BF16 && b.scat != ORC_F16) return -6;
  const uint8_t* q = (const uint8_t*)((const int8_t*)blob + b.q_off);
  const uint8_t* sp = (const uint8_t*)((const int8_t*)blob + b.s_off);
  const int8_t* zp = b.asym ? (const int8_t*)blob + b.z_off : NULL;
  const int nblk = (b.n + 47) / 48;
#pragma omp parallel for schedule(static) num_threads(threads)
  for (int blk = 0; blk < nblk; blk++) {
    const int n0 = blk * 48;
    float acc[48];
    gemv4_nt48_avx512(A, q + (size_t)n0 * b.kpad / 2, sp, zp, &b, n0, acc);
    for (int in = 0; in < 48 && n0 + in < b.n; in++) C[n0 + in] = acc[in];
  }
  return 0;
}
