"""int8-compute oracle (comp_int8: SURVEY a12 / a14) pinned against the reference's own code.

tests/golden/ref/qu8_* and gemv_u8s8_* come from oracle/_ref/ref_golden, which calls the reference's
kernel_ref.h:1824-1883 quantize_fp_u8_colblock and kernel_ref.h:2371-2429 gemv_4bit_u8s8_fp32 directly.  The oracle's
restatements must reproduce them bit for bit; its kblock int8 GEMM (bestla_wrapper.h:768-831) is then checked against
the reference GEMV on the same operands (the two differ only by float association and the bf16 reduce of the zero-point
correction)."""
import numpy as np
import pytest

from tests.oracle_lib import F32, S4, Oracle, load_ref_golden


@pytest.fixture(scope="module")
def golden():
    return load_ref_golden()


@pytest.fixture(scope="module")
def oracle():
    return Oracle.get()


@pytest.mark.parametrize("case", ["qu8_g32", "qu8_g128_tail", "qu8_perchannel", "qu8_g64_big"])
def test_quant_u8_bit_exact(golden, oracle, case):
    g = golden[case]
    row, col, bs = (int(v) for v in g["meta"])
    q, s, z, red = oracle.quant_u8(g["src"].reshape(row, col), bs, want_reduce=True)
    assert np.array_equal(q.ravel(), g["q"])
    assert np.array_equal(s.ravel().view(np.uint32), g["s"].view(np.uint32))
    assert np.array_equal(z.ravel(), g["zp"])
    assert np.array_equal(red.ravel().view(np.uint32), g["red"].view(np.uint32))


@pytest.mark.parametrize("case", ["gemv_u8s8_m1_sym", "gemv_u8s8_m4_asym"])
def test_gemv_u8s8_bit_exact(golden, oracle, case):
    g = golden[case]
    _, k, bs, nt, mt, asym = (int(v) for v in g["meta"])
    nblk = k // bs
    a8, as_, azp, _ = oracle.quant_u8(g["A"].reshape(mt, k), bs)
    assert np.array_equal(a8.ravel(), g["a8"]) and np.array_equal(azp.ravel(), g["azp"])
    assert np.array_equal(as_.ravel().view(np.uint32), g["as"].view(np.uint32))
    C = np.zeros((mt, nt), np.float32)
    zp = g["zp"] if asym else None
    from tests.oracle_lib import _ptr
    oracle.lib.orc_gemv_u8s8_ref(mt, nt, k, bs, _ptr(g["a8"]), _ptr(g["as"]), _ptr(g["azp"]), _ptr(g["q"]),
                                 _ptr(g["scale"]), _ptr(zp), _ptr(C))
    assert np.array_equal(C.ravel().view(np.uint32), g["C"].view(np.uint32))
    assert nblk * bs == k


@pytest.mark.parametrize("case", ["gemv_u8s8_m1_sym", "gemv_u8s8_m4_asym"])
def test_kblock_forward_matches_reference_gemv(golden, oracle, case):
    """The same weights packed for the AMX-INT8 kblock core (which carries the bf16 reduce) through the oracle's
    int8-compute GEMM: equal to the reference GEMV within the bf16 reduce's rounding."""
    g = golden[case]
    _, k, bs, nt, mt, asym = (int(v) for v in g["meta"])
    Q = g["q"].reshape(k, nt)
    S = g["scale"].reshape(k // bs, nt)
    Z = g["zp"].reshape(k // bs, nt) if asym else None
    blob = oracle.pack_q(Q, S, Z, nt, k, bs, S4, F32, bool(asym), oracle.core("amx_int8_kblock"))
    assert oracle.info(blob)["has_reduce"] == 1
    C = oracle.forward_int8(g["A"].reshape(mt, k), blob, nt, k)
    ref = g["C"].reshape(mt, nt)
    # the kblock core corrects the activation zero point with the bf16 reduce: per block the term zpA * sA * reduceB
    # carries reduceB's rounding (<= 2^-9 relative); bound the difference by that, plus float association
    nb = k // bs
    as_ = g["as"].reshape(mt, nb).astype(np.float64)
    azp = g["azp"].reshape(mt, nb).astype(np.float64)
    qz = Q.astype(np.float64) - (0 if Z is None else np.repeat(Z, bs, axis=0))
    red = (qz * np.repeat(S, bs, axis=0)).reshape(nb, bs, nt).sum(1)
    bound = (azp * as_) @ (np.abs(red) * 2.0 ** -8) + 1e-5 * np.abs(ref).max()
    assert np.all(np.abs(C - ref) <= bound)
    # with the exact reduce the kblock algebra equals the reference GEMV to float association
    a8 = g["a8"].reshape(mt, k).astype(np.float64)
    exact = sum((a8[:, b * bs:(b + 1) * bs] @ qz[b * bs:(b + 1) * bs]) * (as_[:, b:b + 1] * S[b])
                - (azp[:, b:b + 1] * as_[:, b:b + 1]) * red[b] for b in range(nb))
    assert np.abs(exact - ref).max() <= 1e-5 * np.abs(ref).max()


def test_int8_forward_close_to_fp(oracle):
    """int8 compute is a quantized approximation of the fp forward: u8 activations carry ~1/255 of each block's range"""
    rng = np.random.default_rng(3)
    n, k, m = 64, 512, 5
    W = rng.uniform(-1, 1, size=(k, n)).astype(np.float32)
    blob = oracle.quant_pack(W, n, k, 32, S4, F32, False, oracle.core("amx_int8_kblock"))
    A = rng.uniform(-1, 1, size=(m, k)).astype(np.float32)
    c8 = oracle.forward_int8(A, blob, n, k)
    cf = oracle.forward(A, blob, n, k)
    assert np.abs(c8 - cf).max() <= 2e-2 * np.abs(cf).max()
