"""Python mirror of Neural Speed's BesTLA operator surface, backed by the MI355X C-ABI (libneural_amd.so).

Reference entry points mirrored (paths relative to the reference repo root):
  quantize()        <- bestla_quantize          neural_speed/models/model_utils/quant_utils.cpp:269-354
  qpack()           <- bestla_qpack / Model.np_bestla_qpack
                                                quant_utils.cpp:226-266, application/main_pybind.cpp:378-402
  pack_size()       <- BTLAGemmPackBSize        neural_speed/core/layers/bestla_gemm.h:38-39
  unpack()          <- BTLAGemmUnPackB / bestla_unpackweight_fp32
  DeviceWeight      <- bestla_device_load_storage (ne_bestla.h:96; SYCL impl ne_bestla_sycl.cpp:94-144)
  DeviceWeight.forward / f32f32_forward
                    <- bestla_device_f32f32_forward (ne_bestla.h:97-98) / bestla_f32f32_forward (inner_product.cpp:28-36)
  qkv_forward()     <- bestla_fusion_QKV_f32f32_forward (ip_fusion_qkv.cpp)
  ffn_forward()     <- bestla_fusion_FFN_SiLu_f32f32_forward / _Gelu_Mul_ (ip_fusion_ffn.cpp:734-755)
  split()           <- TP weight split of model_files.h:1538-1660 (here exact: no re-quantization)

Device buffers are torch tensors (plumbing only); every arithmetic op on the path runs in the HIP kernels.
"""
import ctypes as C

import numpy as np

from ._lib import check, last_error, lib

# BTLA_DTYPE (bestla/bestla/bestla.h:38-87)
F32, F16, BF16 = 32, 16, 16 | (1 << 16)
S8, S4, S2 = 8 | 0x100, 4 | 0x100, 2 | 0x100
# ne_comp_type (neural_speed/core/data_types.h:57-63)
COMP_UNDEF, COMP_F32, COMP_BF16, COMP_F16, COMP_INT8 = 0, 1, 2, 3, 4
# activation dtypes / epilogues of the native API
ACT_F32, ACT_F16, ACT_BF16 = 0, 1, 2
EPI_NONE, EPI_BIAS, EPI_SILU_MUL, EPI_GELU_MUL, EPI_GELU, EPI_ADD_GELU, EPI_SILU, EPI_RES_ADD = range(8)

S1, S3, S5, S6, S7 = 1 | 0x100, 3 | 0x100, 5 | 0x100, 6 | 0x100, 7 | 0x100
F4_E2M1, F4_BNB, F4_NF4 = 4, 4 | (1 << 16), 4 | (2 << 16)
F8_E4M3, F8_E5M2, F8_E8M0 = 8, 8 | (1 << 16), 8 | (3 << 16)
DQ8_BNB = 8 | (4 << 16)  # double-quantized u8 scale codes + fp32 block absmax / offset (bestla_storage.h:223-231)
# quant_config.h:22-57 parse_bits ("int1" is not supported here); "fp4_bnb" names the F4_BNB type the reference packs
# but has no command-line name for
_WEIGHT_DTYPES = {"int4": S4, "int8": S8, "int2": S2, "int1": S1, "int3": S3, "int5": S5, "int6": S6, "int7": S7,
                  "fp4_e2m1": F4_E2M1, "fp4": F4_E2M1, "nf4": F4_NF4, "fp4_bnb": F4_BNB,
                  "fp8_e4m3": F8_E4M3, "fp8": F8_E4M3, "fp8_e5m2": F8_E5M2}
_SCALE_DTYPES = {"fp32": F32, "bf16": BF16, "fp16": F16, "fp8": F8_E8M0}
_COMP = {"int8": COMP_INT8, "bf16": COMP_BF16, "fp16": COMP_F16, "fp32": COMP_F32, "auto": COMP_UNDEF}
BITS = {S4: 4, S2: 2, S8: 8, S1: 1, S3: 3, S5: 5, S6: 6, S7: 7, F4_E2M1: 4, F4_BNB: 4, F4_NF4: 4, F8_E4M3: 8, F8_E5M2: 8}


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(C.c_void_p)
    return C.c_void_p(a.data_ptr())


def _aligned_buffer(size):
    """64-byte aligned, zero-filled uint8 numpy buffer (the blob serializer aligns relative to the base)."""
    raw = np.zeros(size + 64, np.uint8)
    off = (-raw.ctypes.data) % 64
    return raw[off:off + size]


def parse_weight_dtype(s):
    if s not in _WEIGHT_DTYPES:
        raise ValueError(f"unsupported weight_dtype {s!r} (supported: {sorted(_WEIGHT_DTYPES)})")
    return _WEIGHT_DTYPES[s]


def pack_size(n, k, block_size, weight_dtype=S4, scale_dtype=F32, asym=False, comp=COMP_INT8, shuffle=False):
    L = lib()
    dummy = C.c_int(0)
    return L.BTLAGemmPackBSize(n, k, block_size, weight_dtype, scale_dtype, bool(asym), comp,
                               C.byref(dummy) if shuffle else None)


def quantize(w_nk, group_size=32, weight_dtype="int4", scale_dtype="fp32", alg="sym", compute_dtype="int8"):
    """bestla_quantize (quant_utils.cpp:269-354): fp32 torch-layout weight [N][K] -> packed BTLA blob (uint8)."""
    w = np.ascontiguousarray(w_nk, dtype=np.float32)
    qt = parse_weight_dtype(weight_dtype)
    if scale_dtype not in _SCALE_DTYPES:
        raise ValueError(f"unsupported scale_dtype {scale_dtype!r} (supported: {sorted(_SCALE_DTYPES)})")
    st = _SCALE_DTYPES[scale_dtype]
    if qt in (F8_E4M3, F8_E5M2):
        st = F8_E8M0  # quant_utils.cpp:336-341: fp8 weights always get F8_E8M0 shared-exponent scales
    elif st == F8_E8M0:
        st = BF16  # quant_utils.cpp:329-335: anything but fp32 / fp16 is stored as bf16
    gsize = w.shape[1] if group_size == -1 else group_size
    return quant_pack(w, gsize, qt, st, alg == "asym", _COMP[compute_dtype])


def quant_pack(w_nk, block_size, qtype, scale_type, asym, comp):
    """BTLAGemmPackBSize + BTLAGemmQuantPackB on a torch-layout [N][K] weight with BTLA_DTYPE codes (bestla_gemm.cpp);
    unlike quantize() any scale dtype the pack API accepts may be named (e.g. F32 scales for fp8 weights)."""
    w = np.ascontiguousarray(w_nk, dtype=np.float32)
    n, k = w.shape
    gsize, qt, st = block_size, qtype, scale_type
    size = pack_size(n, k, gsize, qt, st, asym, comp)
    if not size:
        raise RuntimeError(f"no packing core for this configuration: {last_error()}")
    blob = _aligned_buffer(size)
    if not lib().BTLAGemmQuantPackB(_ptr(blob), _ptr(w), n, k, k, gsize, qt, st, asym, comp, True, None):
        raise RuntimeError(f"BTLAGemmQuantPackB failed: {last_error()}")
    return blob


def qpack(int_weight, scales, zeros=None, g_idx=None, weight_dtype="int4", group_size=128, alg="sym",
          scale_dtype="fp32", compute_dtype="int8"):
    """bestla_qpack / np_bestla_qpack: pre-quantized int8 [K][N] (+ scales [K/g][N], zeros, g_idx) -> blob.
    As in the reference (quant_utils.cpp:248-254) fp16 scale requests are stored as bf16."""
    q = np.ascontiguousarray(int_weight, dtype=np.int8)
    k, n = q.shape
    s = np.ascontiguousarray(scales, dtype=np.float32)
    asym = alg == "asym"
    z = np.ascontiguousarray(zeros, dtype=np.int8) if (asym and zeros is not None and np.size(zeros)) else None
    gi = np.ascontiguousarray(g_idx, dtype=np.int32) if (g_idx is not None and np.size(g_idx)) else None
    qt = parse_weight_dtype(weight_dtype)
    # "dq8_bnb" (no quant_utils name; the pack API's DQ8_BNB) double-quantizes the given scales at pack time
    st = F32 if scale_dtype == "fp32" else (DQ8_BNB if scale_dtype == "dq8_bnb" else BF16)
    gsize = k if group_size == -1 else group_size
    comp = _COMP[compute_dtype]
    size = pack_size(n, k, gsize, qt, st, asym, comp, gi is not None)
    if not size:
        raise RuntimeError(f"no packing core for this configuration: {last_error()}")
    blob = _aligned_buffer(size)
    if not lib().BTLAGemmPackB(_ptr(blob), _ptr(q), _ptr(s), _ptr(z), n, k, n, gsize, qt, st, asym, comp,
                               _ptr(gi), None):
        raise RuntimeError(f"BTLAGemmPackB failed: {last_error()}")
    return blob


BLOB_FIELDS = ["size", "prologue", "coreid", "npad", "kpad", "n", "k", "dtype", "bs", "scat", "zpt", "redt",
               "cstep", "csize", "asym", "has_reduce", "has_shuffle", "q_off", "q_size", "s_off", "s_size",
               "z_off", "z_size", "r_off", "r_size", "shf_off", "shf_size"]


def blob_info(blob):
    o = np.zeros(27, np.int64)
    check(lib().nad_blob_info(_ptr(blob), _ptr(o)), "nad_blob_info")
    return dict(zip(BLOB_FIELDS, (int(v) for v in o)))


def unpack(blob):
    """BTLAGemmUnPackB: dequantized fp32 [K][N]."""
    inf = blob_info(blob)
    out = np.zeros((inf["k"], inf["n"]), np.float32)
    if not lib().BTLAGemmUnPackB(_ptr(out), _ptr(blob), inf["n"], inf["k"], inf["n"], None):
        raise RuntimeError(f"BTLAGemmUnPackB failed: {last_error()}")
    return out


def split(blob, axis, rank, world, unit=1):
    """Exact TP shard of a blob: axis 0 splits N (TP_1D_ROW) in chunks of `unit` columns, axis 1 splits K by whole
    quantization groups (TP_1D_COLUMN)."""
    L = lib()
    size = L.nad_blob_split(_ptr(blob), axis, rank, world, unit, None, 0)
    if not size:
        raise RuntimeError(f"nad_blob_split failed: {last_error()}")
    out = _aligned_buffer(size)
    if L.nad_blob_split(_ptr(blob), axis, rank, world, unit, _ptr(out), size) != size:
        raise RuntimeError(f"nad_blob_split failed: {last_error()}")
    return out


def split_range(blob, axis, rank, world, unit=1):
    b, e = C.c_int(0), C.c_int(0)
    check(lib().nad_split_range(_ptr(blob), axis, rank, world, unit, C.byref(b), C.byref(e)), "nad_split_range")
    return b.value, e.value


# ---------------------------------------------------------------------------------------------------- device
KERNELS = {1: "woq_gemv_m1_kernel", 2: "woq_gemv_kernel", 3: "woq_skinny_kernel", 4: "woq_i8_kernel",
           5: "woq_gemm3_kernel", 6: "woq_gemm4_kernel", 7: "woq_gemm2_kernel", 8: "woq_gemm_kernel",
           9: "woq_gemm7_kernel", 10: "woq_mid_kernel"}


def plan_forward(bits, n, k, group_size=128, scale_dtype="fp16", asym=False, m=1, act="fp32"):
    """Which kernel a forward of this geometry launches, with what grid (nad_plan_forward: the host side of the call
    with every launch recorded instead of issued -- no GPU needed)."""
    o = np.zeros(6, np.int64)
    st = {"fp32": 0, "bf16": 1, "fp16": 2}[scale_dtype]
    at = {"fp32": 0, "fp16": 1, "bf16": 2}[act]
    r = lib().nad_plan_forward(bits, n, k, group_size, st, int(asym), m, at, _ptr(o), 6)
    if r != 6:
        raise RuntimeError(f"nad_plan_forward failed: {last_error()}")
    return dict(kernel=KERNELS.get(int(o[0]), str(int(o[0]))), grid=int(o[1]), threads=int(o[2]), ksplit=int(o[3]),
                fold=bool(o[4] & 1), ksw=bool(o[4] & 2), launches=int(o[5]))


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("neural_amd device ops need a ROCm GPU (torch.cuda.is_available() is False)")
    return torch


def _stream(stream=None):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


_ACT = {}


def _act_code(t):
    torch = _torch()
    if not _ACT:
        _ACT.update({torch.float32: ACT_F32, torch.float16: ACT_F16, torch.bfloat16: ACT_BF16})
    if t.dtype not in _ACT:
        raise TypeError(f"activation dtype {t.dtype} not supported (float32/float16/bfloat16)")
    return _ACT[t.dtype]


class DeviceWeight:
    """A WOQ weight resident in HBM in the MFMA tile layout (woq_layout.h); the reference's ne_tensor device
    storage: `desc` plays the role of the embedded descriptor (devstor), `mem` of the device buffer."""

    def __init__(self, blob=None, device=None, stream=None, _desc=None, _mem=None):
        torch = _torch()
        L = lib()
        self.desc = (C.c_uint8 * L.bestla_device_storage_size())()
        if blob is not None:
            blob = np.ascontiguousarray(blob)
            need = L.nad_device_weight_size(_ptr(blob))
            if not need:
                raise RuntimeError(f"unsupported blob: {last_error()}")
            self.mem = torch.empty(need, dtype=torch.uint8, device=device or "cuda")
            check(L.nad_device_load(_ptr(blob), self.desc, _ptr(self.mem), need, _stream(stream)),
                  "nad_device_load")
        else:
            self.mem = _mem
            C.memmove(self.desc, _desc, len(self.desc))
        o = np.zeros(13, np.int64)
        if L.nad_weight_info2(self.desc, _ptr(o), 13) != 13:
            raise RuntimeError(f"nad_weight_info2 failed: {last_error()}")
        (_, self.bits, self.n, self.k, self.blocksize, self.ns, self.nt, self.ng, self.scale_t, self.asym,
         self.has_shuffle, self.bytes, self.fold_ok) = (int(v) for v in o)

    @classmethod
    def synthetic(cls, bits, n, k, group_size=128, scale_dtype="fp16", asym=False, seed=0, device=None, stream=None):
        torch = _torch()
        L = lib()
        st = {"fp32": 0, "bf16": 1, "fp16": 2}[scale_dtype]
        need = L.nad_synthetic_weight_size(bits, n, k, group_size, st, int(asym))
        mem = torch.empty(need, dtype=torch.uint8, device=device or "cuda")
        desc = (C.c_uint8 * L.bestla_device_storage_size())()
        check(L.nad_synthetic_weight(desc, _ptr(mem), need, bits, n, k, group_size, st, int(asym), seed,
                                     _stream(stream)), "nad_synthetic_weight")
        return cls(_desc=desc, _mem=mem)

    @classmethod
    def from_q4_0(cls, blocks, n, k, device=None, stream=None):
        """A GGUF Q4_0 matrix (n rows of k/32 block_q4_0, as an NE_TYPE_Q4_0 ne_tensor holds it) in the device tile
        layout (nad_q4_0_device_load)."""
        torch = _torch()
        L = lib()
        blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
        assert blocks.size == n * (k // 32) * 18, (blocks.size, n, k)
        need = L.nad_q4_0_device_size(n, k)
        if not need:
            raise RuntimeError(last_error())
        mem = torch.empty(need, dtype=torch.uint8, device=device or "cuda")
        desc = (C.c_uint8 * L.bestla_device_storage_size())()
        check(L.nad_q4_0_device_load(_ptr(blocks), n, k, desc, _ptr(mem), need, _stream(stream)), "nad_q4_0_device_load")
        return cls(_desc=desc, _mem=mem)

    def forward(self, x, out=None, epilogue=EPI_NONE, bias=None, residual=None, stream=None):
        """out[m][n] = epi(sum_k x[m][k] * W[n][k]); x: cuda [M][K] fp32/fp16/bf16 (row stride honoured)."""
        torch = _torch()
        m, k = x.shape
        assert k == self.k, (k, self.k)
        if out is None:
            out = torch.empty((m, self.n), dtype=torch.float32, device=x.device)
        bias_ld = 0 if bias is None or bias.dim() == 1 else bias.stride(0)
        check(lib().nad_device_forward(_ptr(x), _act_code(x), self.desc, _ptr(out), m, self.n, k, x.stride(0),
                                       out.stride(0), epilogue, _ptr(bias), bias_ld, _ptr(residual),
                                       residual.stride(0) if residual is not None else 0, _stream(stream)),
              "nad_device_forward")
        return out

    __call__ = forward

    def plan(self, m, act="fp32"):
        """which kernel a forward of m rows launches (nad_plan_weight: a dry run, nothing is launched)"""
        o = np.zeros(6, np.int64)
        at = {"fp32": 0, "fp16": 1, "bf16": 2}[act]
        if lib().nad_plan_weight(self.desc, m, at, _ptr(o), 6) != 6:
            raise RuntimeError(f"nad_plan_weight failed: {last_error()}")
        return dict(kernel=KERNELS.get(int(o[0]), str(int(o[0]))), grid=int(o[1]), threads=int(o[2]),
                    ksplit=int(o[3]), fold=bool(o[4] & 1), ksw=bool(o[4] & 2), launches=int(o[5]))

    def set_compute(self, mode):
        """Per-weight arithmetic (nad_device_set_compute): None / -1 follow the thread / process mode, COMPUTE_FP or
        COMPUTE_INT8 (integer-core blobs and GGUF Q4_0 only; other weights stay fp)."""
        check(lib().nad_device_set_compute(self.desc, -1 if mode is None else int(mode)), "nad_device_set_compute")
        return self

    @property
    def compute(self):
        """the arithmetic a forward takes now: COMPUTE_FP or COMPUTE_INT8"""
        return lib().nad_device_get_compute(self.desc)

    def unpack(self, stream=None):
        """dequantized fp32 [K][N] read back from the device tile layout (repack exactness check)."""
        out = np.zeros((self.k, self.n), np.float32)
        check(lib().nad_device_unpack_fp32(self.desc, _ptr(out), _stream(stream)), "nad_device_unpack_fp32")
        return out


COMPUTE_FP, COMPUTE_INT8 = 0, 1


def set_compute_mode(mode):
    """0 (fp16 MFMA on exact weights, default) or 1: the reference's comp_int8 arithmetic for weights packed for an
    integer core (u8 activations per (row, block), s32 block dots, kblock fp32 combine).  Returns the previous mode."""
    L = lib()
    prev = L.nad_get_compute_mode()
    check(L.nad_set_compute_mode(int(mode)), "nad_set_compute_mode")
    return prev


def get_compute_mode():
    return lib().nad_get_compute_mode()


def set_thread_compute_mode(mode):
    """Per-thread override of the process mode (None / -1 clears it)."""
    check(lib().nad_set_thread_compute_mode(-1 if mode is None else int(mode)), "nad_set_thread_compute_mode")


def quant_u8_colblock(x, blocksize, stream=None):
    """kernel::wrapper::QuantizeU8ColBlock (kernel_wrapper.h:571-590) on the GPU: x cuda [M][K] fp32/fp16/bf16 ->
    (q u8 [M][K], scales f32 [M][nblk], zero points u8 [M][nblk], block reduce f32 [M][nblk])."""
    torch = _torch()
    m, k = x.shape
    nblk = -(-k // blocksize)
    q = torch.empty((m, k), dtype=torch.uint8, device=x.device)
    s = torch.empty((m, nblk), dtype=torch.float32, device=x.device)
    z = torch.empty((m, nblk), dtype=torch.uint8, device=x.device)
    red = torch.empty((m, nblk), dtype=torch.float32, device=x.device)
    check(lib().nad_quant_u8_colblock(_ptr(x), _act_code(x), m, k, x.stride(0), blocksize, _ptr(q), k, _ptr(s),
                                      _ptr(z), nblk, _ptr(red), _stream(stream)), "nad_quant_u8_colblock")
    return q, s, z, red


def quant_q8_0(x, stream=None):
    """quantize_row_q8_0 (vectors/cpu/quantize.h:422-445) on the GPU: x cuda [M][K] -> uint8 [M][K/32 * 34] blocks"""
    torch = _torch()
    m, k = x.shape
    out = torch.empty((m, k // 32 * 34), dtype=torch.uint8, device=x.device)
    check(lib().nad_quant_q8_0(_ptr(x), _act_code(x), m, k, x.stride(0), _ptr(out), _stream(stream)), "nad_quant_q8_0")
    return out


def f32f32_forward(activation, weight, output, m, n, k, lda, ldo, stream=None):
    """bestla_device_f32f32_forward with raw device tensors (void result; errors via last_error)."""
    L = lib()
    L.nad_clear_error()
    L.bestla_device_f32f32_forward(_ptr(activation), weight.desc, _ptr(output), m, n, k, lda, ldo, None,
                                   _stream(stream))
    err = last_error()
    if err:
        raise RuntimeError(err)
    return output


def qkv_forward(x, wq, wk, wv, out=None, stream=None):
    """Fused Q/K/V: returns (q, k, v) fp32, written into out[3][M][N] when given (reference layout)."""
    torch = _torch()
    m = x.shape[0]
    if out is None:
        oq = torch.empty((m, wq.n), dtype=torch.float32, device=x.device)
        ok = torch.empty((m, wk.n), dtype=torch.float32, device=x.device)
        ov = torch.empty((m, wv.n), dtype=torch.float32, device=x.device)
    else:
        oq, ok, ov = out[0], out[1], out[2]
    check(lib().nad_device_qkv_forward(_ptr(x), _act_code(x), wq.desc, wk.desc, wv.desc, _ptr(oq), _ptr(ok),
                                       _ptr(ov), m, x.shape[1], x.stride(0), oq.stride(0), ok.stride(0),
                                       ov.stride(0), _stream(stream)), "nad_device_qkv_forward")
    return oq, ok, ov


def ffn_gate_up(x, w1, w3, act="silu", tmp1=None, tmp2=None, stream=None):
    """Gate/up half of the fused FFN: tmp2 = act(x.W1^T) * (x.W3^T), tmp1 = act(x.W1^T) (ip_fusion_ffn.cpp:407-433).
    tmp1 may be None at M <= 16 (decode: one dual-weight launch); the prefill path needs it."""
    torch = _torch()
    m, fin = x.shape
    fmid = w1.n
    if tmp1 is None and m > 16:
        tmp1 = torch.empty((m, fmid), dtype=torch.float32, device=x.device)
    tmp2 = torch.empty((m, fmid), dtype=torch.float32, device=x.device) if tmp2 is None else tmp2
    epi = EPI_SILU_MUL if act == "silu" else EPI_GELU_MUL
    check(lib().nad_device_ffn_gate_up(_ptr(x), _act_code(x), w1.desc, w3.desc, _ptr(tmp1), _ptr(tmp2), m, fin, fmid,
                                       x.stride(0), epi, _stream(stream)), "nad_device_ffn_gate_up")
    return tmp2


def ffn_forward(x, w1, w2, w3, act="silu", tmp1=None, tmp2=None, out=None, stream=None):
    """Fused FFN: out = (act(x.W1^T) * (x.W3^T)) . W2^T  (ip_fusion_ffn.cpp:407-457)."""
    torch = _torch()
    m, fin = x.shape
    fmid, fout = w1.n, w2.n
    dev = x.device
    tmp1 = torch.empty((m, fmid), dtype=torch.float32, device=dev) if tmp1 is None else tmp1
    tmp2 = torch.empty((m, fmid), dtype=torch.float32, device=dev) if tmp2 is None else tmp2
    out = torch.empty((m, fout), dtype=torch.float32, device=dev) if out is None else out
    epi = EPI_SILU_MUL if act == "silu" else EPI_GELU_MUL
    check(lib().nad_device_ffn_forward(_ptr(x), _act_code(x), w1.desc, w2.desc, w3.desc, _ptr(tmp1), _ptr(tmp2),
                                       _ptr(out), m, fin, fmid, fout, x.stride(0), epi, _stream(stream)),
          "nad_device_ffn_forward")
    return out


class Batch:
    """Independent M = 1 problems y_i = x_i W_i of one weight shape as ONE launch (include/neural_amd.h nad_batch_*:
    BTLAGemmBatchDriver, bestla_gemm.cpp:508-624, for device tensors).  problems: list of (DeviceWeight, x [K] or [1][K]
    fp32 cuda tensor, y [N] or [1][N] fp32 cuda tensor); the tensors are bound at creation (keep them alive)."""

    class _P(C.Structure):
        _fields_ = [("weight", C.c_void_p), ("act", C.c_void_p), ("out", C.c_void_p)]

    def __init__(self, problems):
        arr = (Batch._P * len(problems))()
        self._keep = []
        for i, (w, x, y) in enumerate(problems):
            arr[i].weight = C.cast(w.desc, C.c_void_p)
            arr[i].act = x.data_ptr()
            arr[i].out = y.data_ptr()
            self._keep.extend((w, x, y))
        self._arr = arr
        h = lib().nad_batch_create(C.cast(arr, C.c_void_p), len(problems))
        if not h:
            raise RuntimeError(f"nad_batch_create failed: {last_error()}")
        self.handle = h

    def run(self, stream=None):
        check(lib().nad_batch_run(self.handle, _stream(stream)), "nad_batch_run")

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                lib().nad_batch_destroy(h)
            except Exception:
                pass
            self.handle = None
