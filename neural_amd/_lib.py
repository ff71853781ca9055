"""Loader for libneural_amd.so (the C-ABI of include/neural_amd.h).

There is no fallback: if the shared library is missing or fails to load, every entry point raises.
"""
import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# NAD_LIB_PATH: development override (tools/trace_skinny.py loads the phase-trace build)
LIB_PATH = os.environ.get("NAD_LIB_PATH") or os.path.join(_HERE, "libneural_amd.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "neural_amd.h")
HEADERS = [HEADER, os.path.join(os.path.dirname(_HERE), "include", "neural_amd_ne.h")]

_p = C.c_void_p
_i = C.c_int
_sz = C.c_size_t
_u32 = C.c_uint32
_u64 = C.c_uint64
_b = C.c_bool

# name -> (restype, argtypes)
SIGNATURES = {
    "bestla_create_device": (_p, [_b]),
    "bestla_get_device_queue": (_p, [_p]),
    "bestla_release_device": (None, [_p]),
    "bestla_device_gmem_size": (_sz, [_p]),
    "bestla_device_malloc": (_p, [_sz, _p]),
    "bestla_device_free": (None, [_p, _p]),
    "bestla_device_memcpy": (None, [_p, _p, _sz, _p]),
    "bestla_device_memcpy_sync": (None, [_p, _p, _sz, _p]),
    "bestla_device_sync": (None, [_p]),
    "bestla_device_storage_size": (_sz, []),
    "bestla_device_load_storage": (None, [_p, _p, _p, _p]),
    "bestla_device_f32f32_forward": (None, [_p, _p, _p, _i, _i, _i, _i, _i, _p, _p]),
    "bestla_init": (None, []),
    "bestla_set_threads": (_i, [_i]),
    "bestla_get_thread_handle": (_p, []),
    "bestla_f32f32_get_workspace_size": (C.c_ulonglong, [_i, _i, _i, _p]),
    "bestla_f32f32_forward": (None, [_p, _p, _p, _i, _i, _i, _i, _i, _p]),
    "bestla_fusion_add_f32f32_support": (_b, [_p, _i, _i, _i]),
    "bestla_fusion_add_f32f32_forward": (None, [_p, _p, _p, _p, _i, _i, _i, _i, _i, _b, _p]),
    "bestla_fusion_QKV_f32f32_get_workspace_size": (C.c_ulonglong, [_i, _i, _i, _p]),
    "bestla_fusion_QKV_f32f32_support": (_b, [_p, _p, _p, _i, _i, _i]),
    "bestla_fusion_QKV_f32f32_forward": (None, [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p]),
    "bestla_fusion_FFN_f32f32_get_workspace_size": (C.c_ulonglong, [_i, _i, _i, _i, _p, _p]),
    "bestla_fusion_FFN_SiLu_f32f32_support": (_b, [_p, _p, _p, _i, _i, _i, _i]),
    "bestla_fusion_FFN_SiLu_f32f32_forward": (None, [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p]),
    "bestla_fusion_FFN_Gelu_Mul_f32f32_support": (_b, [_p, _p, _p, _i, _i, _i, _i]),
    "bestla_fusion_FFN_Gelu_Mul_f32f32_forward": (None, [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p]),
    "bestla_fusion_FFN_GeLu_f32f32_support": (_b, [_p, _p, _i, _i, _i, _i]),
    "bestla_fusion_FFN_GeLu_f32f32_forward": (None, [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p]),
    "bestla_fusion_FFN_Add_GeLu_f32f32_support": (_b, [_p, _p, _i, _i, _i, _i]),
    "bestla_fusion_FFN_Add_GeLu_f32f32_forward": (None, [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _b, _p]),
    "bestla_unpackweight_fp32": (None, [_p, _i, _i, _p, _i]),
    "bestla_packweight_copyattr": (None, [_p, _p, _i, _i, _i, _p]),
    "BTLAGemmPackBSize": (_sz, [_sz, _sz, _sz, _u32, _u32, _b, _i, _p]),
    "BTLAGemmQuantPackB": (_b, [_p, _p, _sz, _sz, _sz, _sz, _u32, _u32, _b, _i, _b, _p]),
    "BTLAGemmPackB": (_b, [_p, _p, _p, _p, _sz, _sz, _sz, _sz, _u32, _u32, _b, _i, _p, _p]),
    "BTLAGemmUnPackB": (_b, [_p, _p, _sz, _sz, _sz, _p]),
    "BTLAGemmBatchDriver": (_b, [_sz, _sz, _sz, _sz, _p, _p, _p]),
    "nad_last_error": (C.c_char_p, []),
    "nad_clear_error": (None, []),
    "nad_device_weight_size": (_sz, [_p]),
    "nad_device_load": (_i, [_p, _p, _p, _sz, _p]),
    "nad_weight_info": (_i, [_p, _p]),
    "nad_weight_info2": (_i, [_p, _p, _i]),
    "nad_reload_knobs": (None, []),
    "nad_plan_forward": (_i, [_i, _i, _i, _i, _i, _i, _i, _i, _p, _i]),
    "nad_plan_weight": (_i, [_p, _i, _i, _p, _i]),
    "nad_blob_info": (_i, [_p, _p]),
    "nad_device_forward": (_i, [_p, _i, _p, _p, _i, _i, _i, _i, _i, _i, _p, _i, _p, _i, _p]),
    "nad_device_qkv_forward": (_i, [_p, _i, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p]),
    "nad_device_ffn_forward": (_i, [_p, _i, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p]),
    "nad_device_ffn_gate_up": (_i, [_p, _i, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p]),
    "nad_blob_split": (_sz, [_p, _i, _i, _i, _i, _p, _sz]),
    "nad_split_range": (_i, [_p, _i, _i, _i, _i, _p, _p]),
    "nad_synthetic_weight": (_i, [_p, _p, _sz, _i, _i, _i, _i, _i, _i, _u64, _p]),
    "nad_synthetic_weight_size": (_sz, [_i, _i, _i, _i, _i, _i]),
    "nad_device_unpack_fp32": (_i, [_p, _p, _p]),
    "nad_host_cache_clear": (None, []),
    "nad_host_cache_evict": (None, [_p]),
    "nad_host_cache_set_limit": (_sz, [_sz]),
    "nad_host_cache_stats": (_i, [_p, _p]),
    "nad_host_blob_key": (C.c_ulonglong, [_p]),
    "nad_set_compute_mode": (_i, [_i]),
    "nad_get_compute_mode": (_i, []),
    "nad_set_thread_compute_mode": (_i, [_i]),
    "nad_device_set_compute": (_i, [_p, _i]),
    "nad_device_get_compute": (_i, [_p]),
    "nad_quant_u8_colblock": (_i, [_p, _i, _i, _i, _i, _i, _p, _i, _p, _p, _i, _p, _p]),
    "nad_q4_0_device_size": (_sz, [_i, _i]),
    "nad_q4_0_device_load": (_i, [_p, _i, _i, _p, _p, _sz, _p]),
    "nad_quant_q8_0": (_i, [_p, _i, _i, _i, _i, _p, _p]),
    "nad_batch_create": (_p, [_p, _i]),
    "nad_batch_run": (_i, [_p, _p]),
    "nad_batch_destroy": (None, [_p]),
    "init_parallel_context": (_p, []),
    "get_tp_size": (_i, [_p]),
    "get_tp_rank": (_i, [_p]),
    "is_master": (_b, [_p]),
    "barrier": (None, [_p]),
    "broadcast": (None, [_p, _p, _sz]),
    "alltoall": (None, [_p, _p, _p, _sz]),
    "reduce_add": (None, [_p, _p, _p, _sz]),
    "nad_pc_allreduce_f32": (_i, [_p, _p, _p, _sz, _p]),
    "nad_pc_set_stream": (_i, [_p, _p]),
    "nad_pc_max_f64": (C.c_double, [_p, C.c_double]),
    "nad_pc_status": (_i, [_p]),
    "nad_pc_info": (_i, [_p]),
    "nad_pc_last_error": (C.c_char_p, [_p]),
    "nad_pc_destroy": (None, [_p]),
    # include/neural_amd_ne.h
    "bestla_timer": (None, [_b]),
    "bestla_parallel_for": (None, [_p, _p, _p]),
    "bestla_layernormalization": (None, [_i, _i, _b, C.c_float, _p, _p]),
    "bestla_mul": (None, [_i, _i, _p, _p, _i, _p]),
    "bestla_add": (None, [_i, _i, _p, _p, _i, _p]),
    "bestla_backend_support": (_i, [_p, _p, _i]),
    "bestla_support": (_b, [_p, _i, _p, _p]),
    "bestla_device_mul_f32": (None, [_p, _p, _p, _p]),
    "bestla_device_add_f32": (None, [_p, _p, _p, _p]),
    "bestla_device_elewise_f32": (None, [_p, _p, _p]),
    "bestla_device_rms_norm_f32": (None, [_p, _p, _p]),
    "bestla_device_rope_f32": (None, [_p, _p, _p, _p]),
    "bestla_device_dup_f32": (None, [_p, _p, _p]),
    "bestla_device_mha_f32": (None, [_p, _p, _p, _p, _p]),
    "nad_bind_workspace": (_i, [_p, _p, _sz]),
    "nad_device_workspace_size": (_sz, [_i, _i]),
}


class NativeLibraryMissing(RuntimeError):
    pass


_LIB = None


def lib():
    """The loaded libneural_amd.so (raises NativeLibraryMissing if it cannot be loaded)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(f"{LIB_PATH} not found: build it with `make -C neural_amd` "
                                   "(or __graft_entry__.build()); there is no non-native fallback")
    L = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def header_symbols():
    """Function names declared in the C headers include/neural_amd.h and include/neural_amd_ne.h."""
    text = "\n".join(open(h).read() for h in HEADERS)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", text)
    skip = {"if", "defined", "sizeof", "extern", "void"}
    return sorted({n for n in names if n not in skip and not n.isupper()})


def reload_knobs():
    """The library reads its NAD_* switches once; tests and A/B tools that change them at run time call this."""
    lib().nad_reload_knobs()


def last_error():
    return lib().nad_last_error().decode()


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {last_error()}")
