"""The drop-in link proof (CPU; needs the reference sources, so it runs in the build container, not on the GPU box).

1. The reference's own graph executor neural_speed/core/ne_layers.c, compiled as plain C with -DNS_SYCL (the device
   seam of ne_bestla.h:85-112), links against libneural_amd.so with --no-undefined: every bestla_* symbol it calls
   (host forward + fusions, device forward, the device elementwise/norm/RoPE/copy/attention ops, layernorm/mul/add,
   support probes, parallel_for, timer) resolves in this library.  Only the reference's out-of-scope neighbours --
   the CPU attention kernels of layers/mha_dense.h and the conv/argsort/padding-mask layers -- are stubbed, here in
   the test.
2. A C++ translation unit compiled against the reference's layers/bestla_gemm.h (C++ linkage, BTLA_DTYPE /
   ne_comp_type parameters, as quant_utils.cpp and main_pybind.cpp use it) links against the library.
3. include/neural_amd_ne.h's restated ne_tensor / ne_compute_params layout and enum codes equal the reference's
   (ne.h:161-255, data_types.h), checked by the compiler on a TU that includes both.
"""
import os
import subprocess

import pytest

REF = "/root/reference/neural_speed"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "neural_amd")

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "core", "ne_layers.c")),
                                reason="reference sources not present (GPU box)")

STUBS = r"""
/* out-of-scope neighbours of ne_layers.c (CPU attention kernels, conv / argsort / padding-mask layers) */
#include <stddef.h>
#include <stdlib.h>
#define STUB(name) void name(void) { abort(); }
STUB(bestla_fusion_attn_fp32_fp16_fp16_fp32_forward)
STUB(bestla_reordered_attn_fp32_forward)
STUB(bestla_reordered_attn_fp32_shift_rope_k)
STUB(bestla_reordered_attn_fp32_update_k)
STUB(bestla_reordered_attn_fp32_update_v)
STUB(ne_attention_padding_mask_f32_forward)
STUB(ne_compute_forward_argsort)
STUB(ne_compute_forward_conv_1d)
STUB(ne_compute_forward_conv_1d_1s)
STUB(ne_compute_forward_conv_1d_2s)
size_t bestla_fusion_attn_workspace_size(const void* p) { (void)p; abort(); }
"""


def _sh(cmd, cwd):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    assert r.returncode == 0, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return r


def _lib():
    so = os.path.join(LIBDIR, "libneural_amd.so")
    if not os.path.exists(so):
        pytest.skip("libneural_amd.so not built")
    return so


def test_ne_layers_links_against_library(tmp_path):
    _lib()
    inc = ["-I", os.path.join(REF, "core"), "-I", REF, "-I", "/root/reference"]
    _sh(["gcc", "-std=gnu11", "-O0", "-w", "-fPIC", "-DNS_SYCL", "-c", os.path.join(REF, "core", "ne_layers.c"),
         *inc, "-o", "ne_layers.o"], tmp_path)
    (tmp_path / "stubs.c").write_text(STUBS)
    _sh(["gcc", "-fPIC", "-c", "stubs.c", "-o", "stubs.o"], tmp_path)
    undef = _sh(["nm", "-u", "ne_layers.o"], tmp_path).stdout.split()
    seam = sorted({s for s in undef if s.startswith("bestla_")} - {
        "bestla_fusion_attn_fp32_fp16_fp16_fp32_forward", "bestla_reordered_attn_fp32_forward",
        "bestla_reordered_attn_fp32_shift_rope_k", "bestla_reordered_attn_fp32_update_k",
        "bestla_reordered_attn_fp32_update_v", "bestla_fusion_attn_workspace_size"})
    assert len(seam) >= 26, seam
    exported = set(_sh(["nm", "-D", "--defined-only", os.path.join(LIBDIR, "libneural_amd.so")], tmp_path)
                   .stdout.split())
    missing = [s for s in seam if s not in exported]
    assert not missing, f"seam symbols not exported: {missing}"
    _sh(["gcc", "-shared", "-o", "libne_graph.so", "ne_layers.o", "stubs.o", f"-L{LIBDIR}", "-lneural_amd",
         f"-Wl,-rpath,{LIBDIR}", "-Wl,--no-undefined", "-lm"], tmp_path)


CXX_CALLER = r"""
#include "layers/bestla_gemm.h"
// a quant_utils.cpp-style caller: every C++-linkage entry of bestla_gemm.h:38-58 plus BTLALayerNorm
void* use_all() {
  static void* f[] = {(void*)&BTLAGemmPackBSize, (void*)&BTLAGemmQuantPackB, (void*)&BTLAGemmPackB,
                      (void*)&BTLAGemmUnPackB, (void*)&BTLAGemmBatchDriver, (void*)&BTLALayerNorm};
  return f;
}
"""


def test_cxx_bestla_gemm_callers_link(tmp_path):
    _lib()
    (tmp_path / "caller.cpp").write_text(CXX_CALLER)
    _sh(["g++", "-std=c++17", "-fPIC", "-c", "caller.cpp", "-I", os.path.join(REF, "core"), "-I", REF,
         "-I", "/root/reference/bestla", "-o", "caller.o"], tmp_path)
    _sh(["g++", "-shared", "-o", "libcaller.so", "caller.o", f"-L{LIBDIR}", "-lneural_amd", f"-Wl,-rpath,{LIBDIR}",
         "-Wl,--no-undefined"], tmp_path)


LAYOUT = r"""
#include <stddef.h>
#include "ne.h"
#include "neural_amd_ne.h"
#define SAME(f) _Static_assert(offsetof(struct ne_tensor, f) == offsetof(nad_ne_tensor, f), #f);
SAME(type) SAME(backend) SAME(n_dims) SAME(ne) SAME(nb) SAME(op) SAME(is_param) SAME(op_params) SAME(grad)
SAME(src0) SAME(src1) SAME(opt) SAME(n_tasks) SAME(perf_runs) SAME(perf_cycles) SAME(perf_time_us) SAME(data)
SAME(size) SAME(name) SAME(padding)
_Static_assert(sizeof(struct ne_tensor) == sizeof(nad_ne_tensor), "ne_tensor size");
#define PSAME(f) _Static_assert(offsetof(struct ne_compute_params, f) == offsetof(nad_ne_compute_params, f), #f);
PSAME(type) PSAME(ith) PSAME(nth) PSAME(wsize) PSAME(wdata) PSAME(dev_wsize) PSAME(dev_wdata) PSAME(dev_queue)
_Static_assert(sizeof(struct ne_compute_params) == sizeof(nad_ne_compute_params), "params size");
#define E(a, b) _Static_assert((int)(a) == (int)(b), #a);
E(NE_TYPE_F32, NAD_NE_TYPE_F32) E(NE_TYPE_F16, NAD_NE_TYPE_F16) E(NE_TYPE_Q4_0, NAD_NE_TYPE_Q4_0)
E(NE_TYPE_Q8_0, NAD_NE_TYPE_Q8_0) E(NE_TYPE_I32, NAD_NE_TYPE_I32) E(NE_TYPE_BTLA, NAD_NE_TYPE_BTLA)
E(NE_BACKEND_CPU, NAD_NE_BACKEND_CPU) E(NE_BACKEND_SYCL, NAD_NE_BACKEND_DEVICE)
E(NE_TASK_INIT, NAD_NE_TASK_INIT) E(NE_TASK_COMPUTE, NAD_NE_TASK_COMPUTE) E(NE_TASK_FINALIZE, NAD_NE_TASK_FINALIZE)
E(NE_OP_DUP, NAD_NE_OP_DUP) E(NE_OP_ADD, NAD_NE_OP_ADD) E(NE_OP_MUL, NAD_NE_OP_MUL) E(NE_OP_GELU, NAD_NE_OP_GELU)
E(NE_OP_SILU, NAD_NE_OP_SILU) E(NE_OP_NORM, NAD_NE_OP_NORM) E(NE_OP_RMS_NORM, NAD_NE_OP_RMS_NORM)
E(NE_OP_MUL_MAT, NAD_NE_OP_MUL_MAT) E(NE_OP_MUL_MAT_BIAS, NAD_NE_OP_MUL_MAT_BIAS)
E(NE_OP_MUL_MAT_ID, NAD_NE_OP_MUL_MAT_ID) E(NE_OP_CPY, NAD_NE_OP_CPY) E(NE_OP_ROPE, NAD_NE_OP_ROPE)
E(NE_OP_MUL_QKV, NAD_NE_OP_MUL_QKV) E(NE_OP_MUL_FFN_SILU, NAD_NE_OP_MUL_FFN_SILU)
E(NE_OP_MUL_FFN_GELU, NAD_NE_OP_MUL_FFN_GELU) E(NE_OP_MUL_FFN_GELU_MUL, NAD_NE_OP_MUL_FFN_GELU_MUL)
E(NE_OP_MUL_FFN_ADD_GELU, NAD_NE_OP_MUL_FFN_ADD_GELU) E(NE_OP_MUL_ID_FFN_SILU, NAD_NE_OP_MUL_ID_FFN_SILU)
E(NE_OP_MUL_ID_FFN_GELU, NAD_NE_OP_MUL_ID_FFN_GELU)
int main(void) { return 0; }
"""


def test_ne_layout_matches_reference(tmp_path):
    (tmp_path / "layout.c").write_text(LAYOUT)
    _sh(["gcc", "-std=gnu11", "-fsyntax-only", "layout.c", "-I", os.path.join(REF, "core"), "-I", REF,
         "-I", "/root/reference", "-I", os.path.join(REPO, "include")], tmp_path)
