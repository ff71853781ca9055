"""Pin the oracle (oracle/btla_oracle.c, oracle/gptq_oracle.py) against the reference's own outputs.

Goldens: tests/golden/ref (kernel_ref.h compiled from /root/reference) and tests/golden/gptq (the reference's
convert/common.py unpack functions); see tests/golden/make_golden.py.  CPU only.
"""
import os

import numpy as np
import pytest

from oracle import gptq_oracle
from tests.oracle_lib import GOLDEN, load_ref_golden

G = load_ref_golden()


def _cases(prefix):
    return sorted(c for c in G if c.startswith(prefix))


@pytest.mark.parametrize("case", _cases("quant_"))
def test_quantizer_bit_exact(oracle, case):
    g = G[case]
    row, col, bs, bits, asym = (int(v) for v in g["meta"])
    src = g["src"].reshape(row, col)
    q, s, z = oracle.quantize(src, bs, bits, bool(asym))
    np.testing.assert_array_equal(q.reshape(-1), g["q"])
    np.testing.assert_array_equal(s.reshape(-1).view(np.uint32), g["s"].view(np.uint32))
    if asym:
        np.testing.assert_array_equal(z.reshape(-1), g["zp"])


@pytest.mark.parametrize("case", _cases("ilv_"))
def test_interleave_bit_exact(oracle, case):
    g = G[case]
    row, col, rowpad, colpad, ntile, rowpack = (int(v) for v in g["meta"])
    src = np.ascontiguousarray(g["src"])
    dst = np.zeros(rowpad * colpad, np.int8)
    oracle.lib.orc_padding_interleave(src.ctypes.data, dst.ctypes.data, row, col, rowpad, colpad, col, rowpad, ntile,
                                      rowpack)
    np.testing.assert_array_equal(dst, g["dst"])
    back = np.zeros(row * col, np.int8)
    oracle.lib.orc_revert_padding_interleave(dst.ctypes.data, back.ctypes.data, row, col, rowpad, colpad, rowpad, col,
                                             ntile, rowpack)
    np.testing.assert_array_equal(back, g["back"])
    np.testing.assert_array_equal(back, src)


def test_compress_bit_exact(oracle):
    g = G["compress"]
    n = g["s4"].size
    c4 = np.zeros(n // 2, np.uint8)
    c2 = np.zeros(n // 4, np.uint8)
    oracle.lib.orc_compress_s4(g["s4"].ctypes.data, c4.ctypes.data, n)
    oracle.lib.orc_compress_s2(g["s2"].ctypes.data, c2.ctypes.data, n)
    np.testing.assert_array_equal(c4, g["c4"])
    np.testing.assert_array_equal(c2, g["c2"])
    d4 = np.zeros(n, np.int8)
    d2 = np.zeros(n, np.int8)
    oracle.lib.orc_decompress_s4(c4.ctypes.data, d4.ctypes.data, n)
    oracle.lib.orc_decompress_s2(c2.ctypes.data, d2.ctypes.data, n)
    np.testing.assert_array_equal(d4, g["d4"])
    np.testing.assert_array_equal(d2, g["d2"])


def test_conversions_bit_exact(oracle):
    g = G["convert"]
    L = oracle.lib
    bf = np.array([L.orc_f32_to_bf16(float(v)) for v in g["f32"]], np.uint16)
    np.testing.assert_array_equal(bf, g["bf16"])
    fh = np.array([L.orc_f32_to_fp16_bestla(float(v)) for v in g["f32"]], np.uint16)
    np.testing.assert_array_equal(fh, g["fp16"])
    back = np.array([L.orc_fp16_to_f32(int(h)) for h in g["fp16"]], np.float32)
    np.testing.assert_array_equal(back.view(np.uint32), g["fp16_back"].view(np.uint32))
    bback = np.array([L.orc_bf16_to_f32(int(h)) for h in g["bf16"]], np.float32)
    np.testing.assert_array_equal(bback.view(np.uint32), g["bf16_back"].view(np.uint32))
    # IEEE RNE fp16 (the SPR host's vcvtps2ph path) agrees with numpy's float16 cast
    rne = np.array([L.orc_f32_to_fp16_rne(float(v)) for v in g["f32"]], np.uint16)
    np.testing.assert_array_equal(rne, g["f32"].astype(np.float16).view(np.uint16))


def _unpack_packrow(packed_s8, row, ntile, packrow):
    """packed [row/PR][NTILE][PR] -> [row][NTILE]"""
    t = packed_s8.reshape(row // packrow, ntile, packrow).transpose(0, 2, 1)
    return t.reshape(row, ntile)


@pytest.mark.parametrize("case", _cases("deq_s4"))
def test_dequant_s4_chain(oracle, case):
    """decompress_kblock_s4_s8 (with zp) + decompress_kblock_s8_fp == float(q - zp) * s"""
    g = G[case]
    row, nt, pr, bs, isbf = (int(v) for v in g["meta"])
    flat = np.zeros(row * nt, np.int8)
    oracle.lib.orc_decompress_s4(np.ascontiguousarray(g["packed"]).ctypes.data, flat.ctypes.data, row * nt)
    q = _unpack_packrow(flat, row, nt, pr).astype(np.int32)
    zp = g["zp"].reshape(-1, nt).astype(np.int32)
    kb = np.arange(row) // bs
    s8 = q - zp[kb]
    np.testing.assert_array_equal(_unpack_packrow(g["s8"], row, nt, pr), s8)
    if isbf:
        sc = np.array([oracle.lib.orc_bf16_to_f32(int(h)) for h in g["scale_bf16"]], np.float32).reshape(-1, nt)
    else:
        sc = g["scale"].reshape(-1, nt)
    out = (s8.astype(np.float32) * sc[kb]).astype(np.float32)
    np.testing.assert_array_equal(_unpack_packrow(g["out"], row, nt, pr).view(np.uint32), out.view(np.uint32))


@pytest.mark.parametrize("case", _cases("deq_s2"))
def test_dequant_s2_chain(oracle, case):
    g = G[case]
    row, nt, pr, bs = (int(v) for v in g["meta"])
    flat = np.zeros(row * nt, np.int8)
    oracle.lib.orc_decompress_s2(np.ascontiguousarray(g["packed"]).ctypes.data, flat.ctypes.data, row * nt)
    q = _unpack_packrow(flat, row, nt, pr).astype(np.int32)
    zp = g["zp"].reshape(-1, nt).astype(np.int32)
    s8 = q - zp[np.arange(row) // bs]
    np.testing.assert_array_equal(_unpack_packrow(g["s8"], row, nt, pr), s8)


@pytest.mark.parametrize("case", [c for c in _cases("gemv_") if not c.startswith("gemv_u8s8")])
def test_gemv_ref_matches_reference(oracle, case):
    """The oracle's stripe GEMV (used for the cpu_baseline) reproduces kernel_ref.h's gemv_{4,2}bit_fp32_fp32."""
    g = G[case]
    bits, k, bs, nt, mt, asym = (int(v) for v in g["meta"])
    # build a blob that holds exactly this stripe: PACK_ROW 1, NTILE 48 (avx512f core), F32 scales
    flat = np.zeros(k * nt, np.int8)
    fn = oracle.lib.orc_decompress_s4 if bits == 4 else oracle.lib.orc_decompress_s2
    fn(np.ascontiguousarray(g["packed"]).ctypes.data, flat.ctypes.data, k * nt)
    Q = flat.reshape(k, nt)
    S = g["scale"].reshape(-1, nt)
    Z = g["zp"].reshape(-1, nt) if asym else None
    qt = {4: 4 | 0x100, 2: 2 | 0x100}[bits]
    blob = oracle.pack_q(Q, S, Z, nt, k, bs, qt, 32, bool(asym), oracle.core("avx512f"))
    A = g["A"].reshape(mt, k)
    C = oracle.gemv_ref(A, blob, nt)
    np.testing.assert_array_equal(C.reshape(-1).view(np.uint32), g["C"].view(np.uint32))
    # and the fp64 oracle agrees with the reference GEMV within fp32 accumulation error
    ref = oracle.forward(A, blob, nt, k)
    np.testing.assert_allclose(C, ref, rtol=0, atol=1e-4 * max(1.0, float(np.abs(ref).max())))


def _gptq_cases():
    d = os.path.join(GOLDEN, "gptq")
    return sorted({f.split(".")[0] for f in os.listdir(d) if f.endswith(".cfg.txt")})


@pytest.mark.parametrize("case", _gptq_cases())
def test_gptq_awq_unpack(case):
    d = os.path.join(GOLDEN, "gptq")
    method, bits, gs, sym, K, N = open(os.path.join(d, f"{case}.cfg.txt")).read().split()
    qweight = np.load(os.path.join(d, f"{case}.qweight.npy"))
    qzeros = np.load(os.path.join(d, f"{case}.qzeros.npy"))
    if method == "awq":
        w, z = gptq_oracle.unpack_awq4(qweight, qzeros)
    elif bits == "3":
        scales = np.load(os.path.join(d, f"{case}.scales.npy"))
        w, z = gptq_oracle.unpack_gptq3(qweight, qzeros, int(gs), scales.shape[0], scales.shape[1])
    elif bits == "4":
        w, z = gptq_oracle.unpack_gptq4(qweight, qzeros)
    else:
        w, z = gptq_oracle.unpack_gptq8(qweight, qzeros, sym == "1")
    np.testing.assert_array_equal(w, np.load(os.path.join(d, f"{case}.weight.npy")))
    np.testing.assert_array_equal(z, np.load(os.path.join(d, f"{case}.zeros.npy")))


def test_blob_roundtrip_and_layout(oracle):
    """UT_StorageMemCheck rule (ut/bestla_prologue_b.cpp:290-331): deserialize -> serialize is the identity, and the
    layout follows bestla_storage.h field by field."""
    rng = np.random.default_rng(1)
    n, k, bs = 100, 256, 32
    W = rng.uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
    for core in ("avx512f", "avx512_vnni_kblock", "amx_bf16", "avx2"):
        cid = oracle.core(core)
        for stype in (32, 16 | (1 << 16), 16):
            for asym in (False, True):
                blob = oracle.quant_pack(W, n, k, bs, 4 | 0x100, stype, asym, cid)
                inf = oracle.info(blob)
                nt, pr = oracle.lib.orc_core_ntile(cid), oracle.lib.orc_core_packrow(cid)
                assert inf["size"] == blob.size
                assert inf["npad"] == -(-n // nt) * nt and inf["n"] == n and inf["k"] == k
                assert inf["q_off"] % 64 == 0 and inf["s_off"] % 64 == 0
                assert inf["q_size"] == inf["npad"] * inf["kpad"] // 2
                assert inf["has_reduce"] == (pr == 4)
                assert inf["asym"] == int(asym)
                # quantized values survive pack -> unpack exactly
                q, s, z = oracle.quantize(np.ascontiguousarray(W.T), bs, 4, asym)
                Q, S, Z, _ = oracle.unpack_q(blob)
                np.testing.assert_array_equal(Q, q)
                if stype == 32:
                    np.testing.assert_array_equal(S, s)
                if asym:
                    np.testing.assert_array_equal(Z, z)


def test_parallel_gemv_matches_scalar(oracle):
    """The OpenMP column-block GEMV used for bench.py's cpu_baseline is bit-identical to the scalar oracle GEMV."""
    from tests.oracle_lib import S4, F16
    rng = np.random.default_rng(11)
    n, k = 200, 512
    Q = rng.integers(-8, 8, size=(k, n), dtype=np.int8)
    S = rng.uniform(0.001, 0.01, size=(k // 128, n)).astype(np.float32)
    blob = oracle.pack_q(Q, S, None, n, k, 128, S4, F16, False, oracle.core("avx512f"))
    A = rng.uniform(-0.5, 0.5, size=(2, k)).astype(np.float32)
    c1 = np.zeros((2, n), np.float32)
    c2 = np.zeros((2, n), np.float32)
    assert oracle.lib.orc_blob_gemv_ref(A.ctypes.data, blob.ctypes.data, c1.ctypes.data, 2, k, n) == 0
    assert oracle.lib.orc_blob_gemv_par(A.ctypes.data, blob.ctypes.data, c2.ctypes.data, 2, k, n, 4) == 0
    np.testing.assert_array_equal(c1, c2)


def test_compress_planes_bit_exact(oracle):
    """3/5/6/7-bit plane packing (kernel_ref.h compress_Nbit / decompress_sN_s8, plane offsets of
    bestla_prologue_b.h:512-546) against the reference's own outputs"""
    g = G["compress_planes"]
    for bits in (3, 5, 6, 7):
        src = np.ascontiguousarray(g[f"s{bits}"])
        n = src.size
        c = np.zeros(n * bits // 8, np.uint8)
        assert oracle.lib.orc_compress_planes(bits, src.ctypes.data, c.ctypes.data, n) == 0
        assert np.array_equal(c, g[f"c{bits}"]), bits
        d = np.zeros(n, np.int8)
        assert oracle.lib.orc_decompress_planes(bits, np.ascontiguousarray(g[f"c{bits}"]).ctypes.data,
                                                d.ctypes.data, n) == 0
        assert np.array_equal(d, g[f"d{bits}"]) and np.array_equal(d, src), bits


def test_compress_bit1_bit_exact(oracle):
    """1-bit weights (S1_CLIP): kernel_ref.h compress_1bit / decompress_s1_s8 against the reference's own outputs.  The
    reference's compressor stores element 8i + 1 in the slot of element 8i + 4 (srcptr[j + FullRange]); the oracle
    reproduces that, so the decompressed golden differs from its source exactly there."""
    g = G["compress_bit1"]
    src = np.ascontiguousarray(g["s1"])
    n = src.size
    c = np.zeros(n // 8, np.uint8)
    assert oracle.lib.orc_compress_planes(1, src.ctypes.data, c.ctypes.data, n) == 0
    assert np.array_equal(c, g["c1"])
    d = np.zeros(n, np.int8)
    assert oracle.lib.orc_decompress_planes(1, np.ascontiguousarray(g["c1"]).ctypes.data, d.ctypes.data, n) == 0
    assert np.array_equal(d, g["d1"])
    quirk = np.arange(n) % 8 == 4
    assert np.array_equal(d[~quirk], src[~quirk]) and np.array_equal(d[quirk], src[np.nonzero(quirk)[0] - 3])


@pytest.mark.parametrize("case,kind", [("f4_bnb_g32", 0), ("f4_e2m1_g64", 1), ("f4_nf4_g32", 2),
                                       ("f4_nf4_perchannel", 2)])
def test_f4_quantizer_and_lut_bit_exact(oracle, case, kind):
    """NFloat 4-bit: the oracle's quantizer (kernel_ref.h:1233-1419,1800-1822) and LUT (bestla_utils.h:749-790)
    against the reference; the reference's unpack trees and its LUTs agree code for code"""
    g = G[case]
    row, col, bs = (int(v) for v in g["meta"])
    lut = np.array([oracle.lib.orc_f4_lut(kind, c) for c in range(16)], np.float32)
    assert np.array_equal(lut.view(np.uint32), g["lut"].view(np.uint32))
    assert np.array_equal(np.abs(g["tree"]), np.abs(g["lut"])) and np.array_equal(g["tree"], g["lut"])
    q = np.zeros((row, col), np.int8)
    nblk = -(-row // bs)
    s = np.zeros((nblk, col), np.float32)
    src = np.ascontiguousarray(g["src"].reshape(row, col))
    oracle.lib.orc_quantize_f4_rowblock(src.ctypes.data, q.ctypes.data, row, col, col, col, s.ctypes.data, bs, kind)
    assert np.array_equal(q.ravel(), g["q"]) and np.array_equal(s.ravel().view(np.uint32), g["s"].view(np.uint32))
    deq = lut[q.astype(np.int64) & 15] * np.repeat(s, bs, axis=0)[:row]
    assert np.array_equal(deq.ravel().view(np.uint32), g["deq"].view(np.uint32))


@pytest.mark.parametrize("case,t", [("f8_e4m3_e8m0_g32", 8), ("f8_e5m2_e8m0_g64", 8 | (1 << 16)),
                                    ("f8_e4m3_f32_g32", 8), ("f8_e5m2_f32_g128", 8 | (1 << 16))])
def test_f8_quantizer_and_decode_bit_exact(oracle, case, t):
    """NFloat 8-bit: f8_mx_quantize / quantize_f32_f8_rowblock_mxscale (e8m0 and f32 scales) and f8_to_fp32 for all
    256 codes, against the reference's own outputs"""
    g = G[case]
    row, col, bs, e8m0 = (int(v) for v in g["meta"])
    dec = np.array([oracle.lib.orc_f8_to_f32(t, c - 256 if c > 127 else c) for c in range(256)], np.float32)
    assert np.array_equal(dec.view(np.uint32), g["dec"].view(np.uint32))
    q = np.zeros((row, col), np.int8)
    s = np.zeros((-(-row // bs), col), np.float32)
    src = np.ascontiguousarray(g["src"].reshape(row, col))
    oracle.lib.orc_quantize_f8_rowblock(src.ctypes.data, q.ctypes.data, row, col, col, col, s.ctypes.data, bs, t, e8m0)
    assert np.array_equal(s.ravel().view(np.uint32), g["s"].view(np.uint32))
    assert np.array_equal(q.ravel(), g["q"])


def test_layernorm_golden_is_the_stated_formula():
    """The layernorm goldens (kernel_ref.h:2199-2240 via oracle/ref/ref_golden.cpp) are what the numpy restatement used
    by the device-op tests says: x / sqrt(mean(x^2) + eps) (RMS) or (x - mean) / sqrt(mean(x^2) - mean^2 + eps)."""
    G = load_ref_golden()
    for case in ("layernorm_rms_4096", "layernorm_ln_300", "layernorm_rms_11008", "layernorm_ln_4096"):
        g = G[case]
        rows, size, rms = (int(v) for v in g["meta"])
        eps = float(g["eps"][0])
        x = g["src"].reshape(rows, size).astype(np.float64)
        mean = x.mean(-1, keepdims=True)
        ms = np.sqrt((x ** 2).mean(-1, keepdims=True) + eps) if rms else \
            np.sqrt((x ** 2).mean(-1, keepdims=True) - mean ** 2 + eps)
        ref = x / ms if rms else (x - mean) / ms
        d = g["dst"].reshape(rows, size).astype(np.float64)
        assert np.abs(d - ref).max() / np.abs(ref).max() <= 2e-5, case


@pytest.mark.parametrize("stype,asym,n", [("F16", False, 200), ("BF16", True, 96), ("F32", False, 4096),
                                          ("F16", True, 1000)])
def test_avx512_gemv_matches_scalar(oracle, stype, asym, n):
    """the AVX-512 + OpenMP GEMV that bench.py's cpu_baseline times (int4, NTILE-48 blobs; per-block
    FMA chains over the raw nibbles, zero point and scale applied once per block) equals the scalar oracle within fp32
    reassociation: 1e-5 of the largest output, ragged N."""
    from tests import oracle_lib as ol
    rng = np.random.default_rng(n)
    k = 1024
    Q = rng.integers(-8, 8, size=(k, n), dtype=np.int8)
    S = rng.uniform(0.001, 0.01, size=(k // 128, n)).astype(np.float32)
    Z = rng.integers(-3, 4, size=(k // 128, n), dtype=np.int8) if asym else None
    blob = oracle.pack_q(Q, S, Z, n, k, 128, ol.S4, getattr(ol, stype), asym, oracle.core("avx512f"))
    A = rng.uniform(-0.5, 0.5, size=(1, k)).astype(np.float32)
    c1 = np.zeros((1, n), np.float32)
    c2 = np.full((1, n), np.nan, np.float32)
    assert oracle.lib.orc_blob_gemv_ref(A.ctypes.data, blob.ctypes.data, c1.ctypes.data, 1, k, n) == 0
    r = oracle.lib.orc_blob_gemv_avx512(A.ctypes.data, blob.ctypes.data, c2.ctypes.data, k, 4)
    if r == -7:
        pytest.skip("host without AVX-512")
    assert r == 0
    assert np.isfinite(c2).all()
    assert np.abs(c2 - c1).max() <= 1e-5 * np.abs(c1).max(), np.abs(c2 - c1).max() / np.abs(c1).max()
