"""DQ8_BNB double-quantized scales (bestla_storage.h:158,223-231,750-759; bestla_prologue_b.h:151-176,313-329,378-398,
699-706; kernel_ref.h:1930-1991; the LUT bestla_utils.h:794-820).

The scales of a blob are stored as u8 codes into bitsandbytes' signed dynamic map; a trailing fp32 buffer holds each
block's absmax (blocks of dq_blocksize = the quantization group, over the [groups][N] scale array) and the mean of
all scales.  The fp32 scale is LUT[code] * absmax[(g * N + n) / dq_blocksize] + mean.

Pinning: the oracle's restatement (LUT, encoder, decoder) equals the reference's kernel_ref.h outputs bit for bit
(tests/golden/ref/dq8_*, made by oracle/ref/ref_golden.cpp), including the reference's partial-last-block slot
(kernel_ref.h:1978: that block's absmax is written over the mean, its own slot stays 0).  The product's packer
(BTLAGemmQuantPackB / BTLAGemmPackB with DQ8_BNB) equals the oracle's blob byte for byte; on the GPU the weight loads
with the decoded fp32 scales and forwards within the usual bars of the oracle.
"""
import numpy as np
import pytest

from neural_amd import bestla
from tests.oracle_lib import DQ8_BNB, F4_NF4, S2, S4, S8, load_ref_golden

G = load_ref_golden()
CASES = sorted(c for c in G if c.startswith("dq8_"))


def _p(a):
    return a.ctypes.data


def test_lut_matches_reference_table(oracle):
    lut = np.zeros(256, np.float32)
    oracle.lib.orc_dq8_lut(_p(lut))
    for c in CASES:
        np.testing.assert_array_equal(lut.view(np.uint32), G[c]["lut"].view(np.uint32))
    assert np.all(np.diff(lut) >= 0) and lut[0] == np.float32(-0.99297) and lut[255] == 1.0


@pytest.mark.parametrize("case", CASES)
def test_double_quant_and_decode_bit_exact(oracle, case):
    g = G[case]
    row, col, bs, dqb = (int(v) for v in g["meta"])
    s = g["s"].copy()
    dq = np.zeros(g["dq"].size, np.float32)
    oracle.lib.orc_dq8_double_quant(_p(s), s.size, dqb, _p(dq))
    np.testing.assert_array_equal(s.astype(np.uint8), g["code"])
    np.testing.assert_array_equal(dq.view(np.uint32), g["dq"].view(np.uint32))
    nblk = -(-row // bs)
    code = np.ascontiguousarray(g["code"])
    dec = np.zeros(code.size, np.float32)
    oracle.lib.orc_dq8_get_fp_scale(_p(code), _p(dec), nblk, col, dqb, dq.size - 1, _p(dq), col, col, col)
    np.testing.assert_array_equal(dec.view(np.uint32), g["dec"].view(np.uint32))


def test_partial_block_quirk_is_the_references(oracle):
    """63 scales in one dq block of 128: no full block, so the partial block's absmax lands in slot 1 (the mean's
    slot) and slot 0 stays 0 -- every scale decodes to the same value, absmax.  The reference does this; so do we."""
    g = G["dq8_g128_ragged"]
    assert g["dq"][0] == 0.0
    assert np.all(g["dec"] == g["dq"][1])


def _core(oracle, comp, qt, bs):
    return oracle.lib.orc_select_core(comp, qt, bs, 0, 0)


PACKS = [
    # n, k, bs, qtype, comp
    (64, 256, 32, S4, 1),
    (100, 384, 128, S4, 4),    # int8 compute core: BF16 reduce from the decoded scales; N*groups % 128 != 0
    (80, 512, 64, S2, 1),
    (72, 192, 64, S8, 4),
    (40, 256, 32, F4_NF4, 1),
    (50, 1024, 1024, S4, 1),   # per-channel: one dq block of 1024 over 50 scales (the partial-block slot)
]


@pytest.mark.parametrize("cfg", PACKS)
def test_product_pack_matches_oracle(oracle, cfg):
    n, k, bs, qt, comp = cfg
    W = np.random.default_rng(n + k).uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
    blob = bestla.quant_pack(W, bs, qt, DQ8_BNB, False, comp)
    ref = oracle.quant_pack(W, n, k, bs, qt, DQ8_BNB, False, _core(oracle, comp, qt, bs))
    assert blob.size == ref.size
    np.testing.assert_array_equal(blob, ref)
    np.testing.assert_array_equal(bestla.unpack(blob).view(np.uint32), oracle.unpack_fp32(ref).view(np.uint32))


def test_pre_quantized_pack_decodes_to_reference_scales(oracle):
    """BTLAGemmPackB with DQ8_BNB on the golden case's scales: the blob's decoded scales are the reference's
    dq8_get_fp_scale output bit for bit (the whole pipeline -- encoder, buffer placement, offset slot, decoder)."""
    g = G["dq8_g64_tail"]
    row, col, bs, _ = (int(v) for v in g["meta"])
    s = g["s"].reshape(-1, col)
    q = np.random.default_rng(1).integers(-8, 8, size=(row, col)).astype(np.int8)
    blob = bestla.qpack(q, s, weight_dtype="int4", group_size=bs, scale_dtype="dq8_bnb", compute_dtype="fp32")
    ref = oracle.pack_q(q, s, None, col, row, bs, S4, DQ8_BNB, False, _core(oracle, 1, S4, bs))
    np.testing.assert_array_equal(blob, ref)
    _, S, _, _ = oracle.unpack_q(blob)
    np.testing.assert_array_equal(S.reshape(-1).view(np.uint32), g["dec"].view(np.uint32))
    W = bestla.unpack(blob)
    np.testing.assert_array_equal(W, (q.astype(np.float32) * np.repeat(S, bs, axis=0)[:row]))


def test_rejections():
    W = np.zeros((64, 256), np.float32)
    with pytest.raises(RuntimeError, match="DQ8_BNB"):
        bestla.quant_pack(W, 32, S4, DQ8_BNB, True, 1)  # asym (initDoubleQuantBlkSize asserts)
    with pytest.raises(RuntimeError, match="DQ8_BNB"):
        bestla.quant_pack(W, 32, bestla.F8_E4M3, DQ8_BNB, False, 1)
    blob = bestla.quant_pack(np.ones((64, 256), np.float32), 32, S4, DQ8_BNB, False, 1)
    with pytest.raises(RuntimeError, match="cannot be split"):
        bestla.split(blob, 0, 0, 2)


# ------------------------------------------------------------------------------------------------------------ GPU
TOL_DECODE, TOL_PREFILL = 2e-5, 1e-3


def _rel(y, ref):
    return float(np.abs(y - ref).max() / max(np.abs(ref).max(), 1e-30))


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [(512, 1024, 128, S4, 1), (300, 768, 64, S2, 4), (256, 512, 32, S8, 1),
                                 (256, 512, 32, F4_NF4, 1), (4096, 4096, 128, S4, 4)])
def test_device_forward_matches_oracle(oracle, cfg):
    import torch

    n, k, bs, qt, comp = cfg
    W = np.random.default_rng(n * 3 + k).uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
    blob = oracle.quant_pack(W, n, k, bs, qt, DQ8_BNB, False, _core(oracle, comp, qt, bs))
    w = bestla.DeviceWeight(blob)
    # the device holds the decoded fp32 scales: its dequantized weight is the reference's bit for bit
    assert np.array_equal(w.unpack().view(np.uint32), oracle.unpack_fp32(blob).view(np.uint32))
    rng = np.random.default_rng(7)
    for m, tol in ((1, TOL_DECODE), (64, TOL_PREFILL)):
        A = rng.uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
        y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
        tol = TOL_PREFILL if qt == F4_NF4 else tol  # NF4 codes run as fp16 LUT values (test_more_bits_gpu's F4 bar)
        err = _rel(y, oracle.forward(A, blob, n, k))
        assert err <= tol, (m, cfg, err)
