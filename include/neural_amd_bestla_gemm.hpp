// neural_amd_bestla_gemm.hpp -- C++-linkage face of the pack / batch-driver API, for C++ callers compiled against the
// reference's neural_speed/core/layers/bestla_gemm.h:30-58 (quant_utils.cpp:256-259,343-347, main_pybind.cpp:378-402),
// whose declarations have C++ linkage and take BTLA_DTYPE (bestla/bestla/bestla.h:38) and ne_comp_type
// (core/data_types.h:57-63).  libneural_amd.so exports these mangled overloads next to the extern "C" ones of
// neural_amd.h; they forward to them.  Include this header OR the reference's bestla_gemm.h, not both.
#pragma once
#include <cstddef>
#include <cstdint>

#include "neural_amd.h"

enum class BTLA_DTYPE : uint32_t;  // values: the uint32 codes of bestla.h:38-87 (S4_CLIP = 0x104, F16 = 16, ...)
enum ne_comp_type : int;           // NE_COMP_UNDEF 0, F32 1, BF16 2, F16 3, INT8 4

size_t BTLAGemmPackBSize(size_t N, size_t K, size_t BlkSize, BTLA_DTYPE QuantType, BTLA_DTYPE ScaleDtype, bool isAsym,
                         ne_comp_type CompType, int* shuffle_indice);
bool BTLAGemmQuantPackB(void* PackedBuf, const float* FpData, size_t N, size_t K, size_t ldb, size_t BlkSize,
                        BTLA_DTYPE QuantType, BTLA_DTYPE ScaleDtype, bool isAsym, ne_comp_type CompType, bool isTrans,
                        void* ThreadPool);
bool BTLAGemmPackB(void* PackedBuf, const int8_t* QData, const float* Scales, const int8_t* Zp, size_t N, size_t K,
                   size_t ldb, size_t BlkSize, BTLA_DTYPE QuantType, BTLA_DTYPE ScaleDtype, bool isAsym,
                   ne_comp_type CompType, int* shuffle_indice, void* ThreadPool);
bool BTLALayerNorm(size_t norm_count, size_t norm_size, bool isrms, float epsilon, const float* FpIn, float* FpOut,
                   void* ThreadPool);
// BTLAGemmUnPackB / BTLAGemmBatchDriver keep their parameter lists: the library also exports their C++-mangled names
// (for callers of the reference header); from this header they resolve to the extern "C" declarations of neural_amd.h
