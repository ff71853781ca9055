// cxx_abi.cpp -- C++-linkage overloads of the pack / batch-driver API (include/neural_amd_bestla_gemm.hpp), so C++
// callers compiled against the reference's bestla_gemm.h (C++ linkage, bestla_gemm.h:30-58) link against this
// library.  Each forwards to the extern "C" entry of include/neural_amd.h, reached here through asm labels because
// BTLAGemmUnPackB / BTLAGemmBatchDriver have identical parameter lists in both linkages (one TU cannot declare both).
#include <cstddef>
#include <cstdint>

enum class BTLA_DTYPE : uint32_t;  // bestla/bestla/bestla.h:38
enum ne_comp_type : int;           // core/data_types.h:57-63
struct BTLA_GEMM_DATA_PACKED_PARAMS {  // bestla_gemm.h:30-36 (same layout as neural_amd.h's C struct)
  const float* A;
  const void* B;
  float* C;
  int lda;
  int ldc;
};

extern "C" {
size_t c_pack_size(size_t, size_t, size_t, uint32_t, uint32_t, bool, int, int*) __asm__("BTLAGemmPackBSize");
bool c_quant_pack(void*, const float*, size_t, size_t, size_t, size_t, uint32_t, uint32_t, bool, int, bool,
                  void*) __asm__("BTLAGemmQuantPackB");
bool c_pack(void*, const int8_t*, const float*, const int8_t*, size_t, size_t, size_t, size_t, uint32_t, uint32_t, bool,
            int, int*, void*) __asm__("BTLAGemmPackB");
bool c_unpack(float*, const void*, size_t, size_t, size_t, void*) __asm__("BTLAGemmUnPackB");
bool c_batch(size_t, size_t, size_t, size_t, const BTLA_GEMM_DATA_PACKED_PARAMS*, int8_t*,
             void*) __asm__("BTLAGemmBatchDriver");
void c_layernorm(int, int, bool, float, const float*, float*) __asm__("bestla_layernormalization");
}

size_t BTLAGemmPackBSize(size_t N, size_t K, size_t BlkSize, BTLA_DTYPE QuantType, BTLA_DTYPE ScaleDtype, bool isAsym,
                         ne_comp_type CompType, int* shuffle_indice) {
  return c_pack_size(N, K, BlkSize, static_cast<uint32_t>(QuantType), static_cast<uint32_t>(ScaleDtype), isAsym,
                     static_cast<int>(CompType), shuffle_indice);
}

bool BTLAGemmQuantPackB(void* PackedBuf, const float* FpData, size_t N, size_t K, size_t ldb, size_t BlkSize,
                        BTLA_DTYPE QuantType, BTLA_DTYPE ScaleDtype, bool isAsym, ne_comp_type CompType, bool isTrans,
                        void* ThreadPool) {
  return c_quant_pack(PackedBuf, FpData, N, K, ldb, BlkSize, static_cast<uint32_t>(QuantType),
                      static_cast<uint32_t>(ScaleDtype), isAsym, static_cast<int>(CompType), isTrans, ThreadPool);
}

bool BTLAGemmPackB(void* PackedBuf, const int8_t* QData, const float* Scales, const int8_t* Zp, size_t N, size_t K,
                   size_t ldb, size_t BlkSize, BTLA_DTYPE QuantType, BTLA_DTYPE ScaleDtype, bool isAsym,
                   ne_comp_type CompType, int* shuffle_indice, void* ThreadPool) {
  return c_pack(PackedBuf, QData, Scales, Zp, N, K, ldb, BlkSize, static_cast<uint32_t>(QuantType),
                static_cast<uint32_t>(ScaleDtype), isAsym, static_cast<int>(CompType), shuffle_indice, ThreadPool);
}

bool BTLAGemmUnPackB(float* FpData, const void* PackedBuf, size_t N, size_t K, size_t ldb, void* ThreadPool) {
  return c_unpack(FpData, PackedBuf, N, K, ldb, ThreadPool);
}

bool BTLAGemmBatchDriver(const size_t M, const size_t N, const size_t K, const size_t BatchN,
                         const BTLA_GEMM_DATA_PACKED_PARAMS* DataParams, int8_t* WorkSpace, void* ThreadPool) {
  return c_batch(M, N, K, BatchN, DataParams, WorkSpace, ThreadPool);
}

bool BTLALayerNorm(size_t norm_count, size_t norm_size, bool isrms, float epsilon, const float* FpIn, float* FpOut,
                   void* ThreadPool) {
  c_layernorm(static_cast<int>(norm_count), static_cast<int>(norm_size), isrms, epsilon, FpIn, FpOut);
  return true;
}
