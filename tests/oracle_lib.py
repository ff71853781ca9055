"""ctypes access to the oracle (oracle/liboracle.so) and the golden fixtures.  Test infrastructure only."""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")

F32, F16, BF16 = 32, 16, 16 | (1 << 16)
S8, S4, S2 = 8 | 0x100, 4 | 0x100, 2 | 0x100
S1, S3, S5, S6, S7 = 1 | 0x100, 3 | 0x100, 5 | 0x100, 6 | 0x100, 7 | 0x100
F4_E2M1, F4_BNB, F4_NF4 = 4, 4 | (1 << 16), 4 | (2 << 16)
F8_E4M3, F8_E5M2, F8_E8M0 = 8, 8 | (1 << 16), 8 | (3 << 16)
DQ8_BNB = 8 | (4 << 16)
BITS_TO_QTYPE = {8: S8, 7: S7, 6: S6, 5: S5, 4: S4, 3: S3, 2: S2, 1: S1}

_p = C.c_void_p


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_p)


class Oracle:
    _inst = None

    @classmethod
    def get(cls):
        if cls._inst is None:
            cls._inst = cls()
        return cls._inst

    def __init__(self):
        so = os.path.join(ORACLE_DIR, "liboracle.so")
        src = os.path.join(ORACLE_DIR, "btla_oracle.c")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = self.lib = C.CDLL(so)
        L.orc_blob_size.restype = C.c_size_t
        L.orc_blob_size.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_uint32, C.c_int, C.c_uint64, C.c_int]
        L.orc_core_id.restype = C.c_uint64
        L.orc_core_id.argtypes = [C.c_char_p]
        L.orc_select_core.restype = C.c_uint64
        L.orc_select_core.argtypes = [C.c_int, C.c_uint32, C.c_int, C.c_int, C.c_int]
        L.orc_blob_quant_pack.argtypes = [_p, _p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_uint32, C.c_int,
                                          C.c_uint64, C.c_int]
        L.orc_blob_pack_q.argtypes = [_p, _p, _p, _p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_uint32,
                                      C.c_int, C.c_uint64, _p]
        L.orc_blob_info.argtypes = [_p, _p]
        L.orc_blob_unpack_q.argtypes = [_p, _p, _p, _p, _p]
        L.orc_blob_unpack_fp32.argtypes = [_p, _p, C.c_int]
        L.orc_blob_forward.argtypes = [_p, _p, _p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_blob_gemv_ref.argtypes = [_p, _p, _p, C.c_int, C.c_int, C.c_int]
        L.orc_blob_gemv_timed.argtypes = [_p, _p, _p, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_blob_gemv_par.argtypes = [_p, _p, _p, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_blob_gemv_avx512.argtypes = [_p, _p, _p, C.c_int, C.c_int]
        L.orc_quantize_rowblock.argtypes = [_p, _p, C.c_int, C.c_int, C.c_int, C.c_int, _p, _p, C.c_int, C.c_int]
        L.orc_padding_interleave.argtypes = [_p, _p] + [C.c_int] * 8
        L.orc_revert_padding_interleave.argtypes = [_p, _p] + [C.c_int] * 8
        for f in ("orc_compress_s4", "orc_compress_s2", "orc_decompress_s4", "orc_decompress_s2"):
            getattr(L, f).argtypes = [_p, _p, C.c_size_t]
        L.orc_shuffle_indices.argtypes = [_p, C.c_int, C.c_int, _p]
        L.orc_f32_to_bf16.restype = C.c_uint16
        L.orc_f32_to_bf16.argtypes = [C.c_float]
        L.orc_f32_to_fp16_bestla.restype = C.c_uint16
        L.orc_f32_to_fp16_bestla.argtypes = [C.c_float]
        L.orc_f32_to_fp16_rne.restype = C.c_uint16
        L.orc_f32_to_fp16_rne.argtypes = [C.c_float]
        L.orc_fp16_to_f32.restype = C.c_float
        L.orc_fp16_to_f32.argtypes = [C.c_uint16]
        L.orc_bf16_to_f32.restype = C.c_float
        L.orc_bf16_to_f32.argtypes = [C.c_uint16]
        L.orc_core_ktile.argtypes = [C.c_uint64]
        L.orc_core_ntile.argtypes = [C.c_uint64]
        L.orc_core_packrow.argtypes = [C.c_uint64]
        L.orc_dq8_lut.argtypes = [_p]
        L.orc_dq8_double_quant.argtypes = [_p, C.c_size_t, C.c_int, _p]
        L.orc_dq8_get_fp_scale.argtypes = [_p, _p] + [C.c_int] * 4 + [_p] + [C.c_int] * 3
        L.orc_f8_to_f32.restype = C.c_float
        L.orc_f8_to_f32.argtypes = [C.c_uint32, C.c_int8]
        L.orc_quantize_f8_rowblock.argtypes = [_p, _p] + [C.c_int] * 4 + [_p, C.c_int, C.c_uint32, C.c_int]
        L.orc_f4_lut.restype = C.c_float
        L.orc_f4_lut.argtypes = [C.c_int, C.c_int]
        L.orc_f4_kind.argtypes = [C.c_uint32]
        L.orc_quantize_f4_rowblock.argtypes = [_p, _p] + [C.c_int] * 4 + [_p, C.c_int, C.c_int]
        L.orc_compress_planes.argtypes = [C.c_int, _p, _p, C.c_size_t]
        L.orc_decompress_planes.argtypes = [C.c_int, _p, _p, C.c_size_t]
        L.orc_quant_u8_colblock.argtypes = [C.c_int, C.c_int, _p, C.c_int, _p, C.c_int, _p, C.c_int, _p, C.c_int, _p]
        L.orc_blob_forward_int8.argtypes = [_p, _p, _p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_gemv_u8s8_ref.argtypes = [C.c_int] * 4 + [_p] * 7
        L.orc_q4_0_quantize_row.argtypes = [_p, _p, C.c_int]
        L.orc_q4_0_dequantize_row.argtypes = [_p, _p, C.c_int]
        L.orc_q8_0_quantize_row.argtypes = [_p, _p, C.c_int]
        L.orc_vec_dot_q4_0_q8_0.argtypes = [C.c_int, _p, _p]
        L.orc_vec_dot_q4_0_q8_0.restype = C.c_float
        L.orc_q4_0_forward.argtypes = [_p, _p, _p, C.c_int, C.c_int, C.c_int]

    # ---- helpers
    def core(self, name):
        return self.lib.orc_core_id(name.encode())

    def quantize(self, src_kn, blocksize, bits, asym):
        src = np.ascontiguousarray(src_kn, dtype=np.float32)
        row, col = src.shape
        nblk = -(-row // blocksize)
        q = np.zeros((row, col), np.int8)
        s = np.zeros((nblk, col), np.float32)
        z = np.zeros((nblk, col), np.int8) if asym else None
        self.lib.orc_quantize_rowblock(_ptr(src), _ptr(q), row, col, col, col, _ptr(s), _ptr(z), blocksize, bits)
        return q, s, z

    def blob_size(self, n, k, bs, qtype, stype, asym, core, shuffle=False):
        return self.lib.orc_blob_size(n, k, bs, qtype, stype, int(asym), core, int(shuffle))

    def quant_pack(self, W, n, k, bs, qtype, stype, asym, core, is_trans=True):
        W = np.ascontiguousarray(W, dtype=np.float32)
        size = self.blob_size(n, k, bs, qtype, stype, asym, core)
        buf = np.zeros(size + 64, np.uint8)
        off = (-buf.ctypes.data) % 64
        blob = buf[off:off + size]
        ldb = k if is_trans else n
        r = self.lib.orc_blob_quant_pack(_ptr(blob), _ptr(W), n, k, ldb, bs, qtype, stype, int(asym), core,
                                         int(is_trans))
        assert r == 0, r
        return blob

    def pack_q(self, Q, S, Z, n, k, bs, qtype, stype, asym, core, g_idx=None):
        Q = np.ascontiguousarray(Q, dtype=np.int8)
        S = np.ascontiguousarray(S, dtype=np.float32)
        Z = None if Z is None else np.ascontiguousarray(Z, dtype=np.int8)
        gi = None if g_idx is None else np.ascontiguousarray(g_idx, dtype=np.int32)
        size = self.blob_size(n, k, bs, qtype, stype, asym, core, gi is not None)
        buf = np.zeros(size + 64, np.uint8)
        off = (-buf.ctypes.data) % 64
        blob = buf[off:off + size]
        r = self.lib.orc_blob_pack_q(_ptr(blob), _ptr(Q), _ptr(S), _ptr(Z), n, k, n, bs, qtype, stype, int(asym),
                                     core, _ptr(gi))
        assert r == 0, r
        return blob

    def info(self, blob):
        o = np.zeros(27, np.int64)
        assert self.lib.orc_blob_info(_ptr(blob), _ptr(o)) == 0
        keys = ["size", "prologue", "coreid", "npad", "kpad", "n", "k", "dtype", "bs", "scat", "zpt", "redt",
                "cstep", "csize", "asym", "has_reduce", "has_shuffle", "q_off", "q_size", "s_off", "s_size",
                "z_off", "z_size", "r_off", "r_size", "shf_off", "shf_size"]
        return dict(zip(keys, (int(v) for v in o)))

    def unpack_q(self, blob):
        inf = self.info(blob)
        n, k, bs = inf["n"], inf["k"], inf["bs"]
        nblk = -(-k // bs)
        Q = np.zeros((k, n), np.int8)
        S = np.zeros((nblk, n), np.float32)
        Z = np.zeros((nblk, n), np.int8)
        shf = np.zeros(k, np.int32)
        assert self.lib.orc_blob_unpack_q(_ptr(blob), _ptr(Q), _ptr(S), _ptr(Z), _ptr(shf)) == 0
        return Q, S, Z, (shf if inf["has_shuffle"] else None)

    def unpack_fp32(self, blob):
        inf = self.info(blob)
        W = np.zeros((inf["k"], inf["n"]), np.float32)
        assert self.lib.orc_blob_unpack_fp32(_ptr(blob), _ptr(W), inf["n"]) == 0
        return W

    def forward(self, A, blob, n, k):
        A = np.ascontiguousarray(A, dtype=np.float32)
        m = A.shape[0]
        C_ = np.zeros((m, n), np.float32)
        assert self.lib.orc_blob_forward(_ptr(A), _ptr(blob), _ptr(C_), m, n, k, A.shape[1], n) == 0
        return C_

    def quant_u8(self, A, blocksize, want_reduce=False):
        """kernel_ref.h:1824-1883: -> (u8 codes [m][k], scales [m][nblk], zero points [m][nblk], block reduce)"""
        A = np.ascontiguousarray(A, dtype=np.float32)
        m, k = A.shape
        nblk = -(-k // blocksize)
        q = np.zeros((m, k), np.uint8)
        s = np.zeros((m, nblk), np.float32)
        z = np.zeros((m, nblk), np.uint8)
        red = np.zeros((m, nblk), np.float32) if want_reduce else None
        self.lib.orc_quant_u8_colblock(m, k, _ptr(A), k, _ptr(q), k, _ptr(s), nblk, _ptr(z), blocksize, _ptr(red))
        return q, s, z, red

    def forward_int8(self, A, blob, n, k):
        """int8-compute forward (kblock u8s8 core) of a blob packed for an integer core"""
        A = np.ascontiguousarray(A, dtype=np.float32)
        m = A.shape[0]
        C_ = np.zeros((m, n), np.float32)
        r = self.lib.orc_blob_forward_int8(_ptr(A), _ptr(blob), _ptr(C_), m, n, k, A.shape[1], n)
        assert r == 0, r
        return C_

    def q4_0_quantize(self, W):
        """[n][k] f32 -> [n][k/32] block_q4_0 bytes (vectors/cpu/quantize.h:243-276)"""
        W = np.ascontiguousarray(W, dtype=np.float32)
        n, k = W.shape
        out = np.zeros((n, k // 32 * 18), np.uint8)
        for r in range(n):
            self.lib.orc_q4_0_quantize_row(_ptr(W[r]), _ptr(out[r]), k)
        return out

    def q4_0_forward(self, A, W_q4, n, k):
        """the reference's Q4_0 mul_mat: Q8_0 activations, integer block dots (vec_dot.h scalar order)"""
        A = np.ascontiguousarray(A, dtype=np.float32)
        m = A.shape[0]
        C_ = np.zeros((m, n), np.float32)
        assert self.lib.orc_q4_0_forward(_ptr(A), _ptr(np.ascontiguousarray(W_q4)), _ptr(C_), m, n, k) == 0
        return C_

    def q4_0_dequant(self, W_q4, n, k):
        out = np.zeros((n, k), np.float32)
        W_q4 = np.ascontiguousarray(W_q4)
        for r in range(n):
            self.lib.orc_q4_0_dequantize_row(_ptr(W_q4[r]), _ptr(out[r]), k)
        return out

    def gemv_ref(self, A, blob, n):
        A = np.ascontiguousarray(A, dtype=np.float32)
        m = A.shape[0]
        C_ = np.zeros((m, n), np.float32)
        r = self.lib.orc_blob_gemv_ref(_ptr(A), _ptr(blob), _ptr(C_), m, A.shape[1], n)
        assert r == 0, r
        return C_


def load_ref_golden(sub="ref"):
    """tests/golden/<sub>/manifest.txt -> {case: {name: array}}"""
    d = os.path.join(GOLDEN, sub)
    out = {}
    with open(os.path.join(d, "manifest.txt")) as f:
        for line in f:
            cs, name, dt, n = line.split()
            arr = np.fromfile(os.path.join(d, f"{cs}.{name}.bin"), dtype=np.dtype(dt))
            assert arr.size == int(n)
            out.setdefault(cs, {})[name] = arr
    return out
