"""GPU parity for the 1/3/5/6/7-bit integer weights and the NFloat 4-bit weights (F4_NF4 / F4_E2M1 / F4_BNB,
bestla_prologue_b.h:1005-1342: codes in the int4 tile layout, dequantized through the bestla_utils.h:749-790 LUT whose
entries are rounded to fp16 for the MFMA B operand -- <= 2^-12 relative per weight, hence the 1e-3 bar) and the
3/5/6/7-bit integer weights (quant_config.h:22-57 "int3".."int7"; planes of
bestla_prologue_b.h:512-546).  The repack stores S1 in the int2 tile layout, S3 in the int4 one and S5-S7 in the int8 one (exact: the
integers fit), so every forward kernel serves them; checked against the oracle's fp64 forward of the same blob, the
repacked integers bit-exact, and the int8-compute mode against the oracle's kblock GEMM.  NFloat 8-bit weights (F8_E4M3 /
F8_E5M2 with F8_E8M0 or F32 scales, bestla_prologue_b.h:1198-1208, kernel_ref.h:984-1026) sit as raw codes in the int8
layout and decode to their exact fp16 values, so they take the integer formats' bars."""
import numpy as np
import pytest

from tests.conftest import gpu_available
from tests.oracle_lib import BF16, F16, F32, F4_BNB, F4_E2M1, F4_NF4, F8_E4M3, F8_E5M2, F8_E8M0, S1, S3, S5, S6, S7
from tests.test_gpu_parity import _blob, _rel_err

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from neural_amd import bestla

CASES = [
    # n, k, bs, qtype, stype, asym, comp
    (256, 1024, 128, S3, F16, False, 1),
    (200, 768, 32, S3, BF16, True, 4),
    (96, 512, 64, S5, F32, True, 1),
    (128, 1024, 32, S6, F16, False, 4),
    (64, 512, 128, S7, F32, False, 1),
    (48, 300, 1024, S3, F32, False, 1),     # per-channel, K tail
    (256, 1024, 64, S1, F16, False, 1),     # 1-bit (S1_CLIP, q in {-1, 0}) in the int2 tile layout
    (200, 768, 32, S1, BF16, True, 4),
    (72, 300, 128, S1, F32, False, 2),      # K tail
    (256, 1024, 32, F4_NF4, F32, False, 1),
    (128, 512, 64, F4_E2M1, BF16, False, 2),
    (96, 512, 32, F4_BNB, F16, False, 1),
    (80, 300, 128, F4_NF4, F32, False, 1),  # K tail
    (256, 1024, 32, F8_E4M3, F8_E8M0, False, 1),
    (128, 512, 64, F8_E5M2, F8_E8M0, False, 2),
    (96, 512, 32, F8_E4M3, F32, False, 1),
    (80, 300, 128, F8_E5M2, F32, False, 1),   # K tail
]
F4 = (F4_NF4, F4_E2M1, F4_BNB)
TOL = {1: 2e-5, 64: 1e-3}


@pytest.mark.parametrize("cfg", CASES)
def test_repack_exact(oracle, cfg):
    n, k, bs, qt, st, asym, comp = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, comp, seed=n + k)
    w = bestla.DeviceWeight(blob)
    assert w.bits == (2 if qt == S1 else (4 if qt in (S3,) + F4 else 8))
    assert np.array_equal(w.unpack().view(np.uint32), oracle.unpack_fp32(blob).view(np.uint32))


@pytest.mark.parametrize("m", [1, 4, 64, 300])
@pytest.mark.parametrize("cfg", CASES)
def test_forward_parity(oracle, cfg, m):
    n, k, bs, qt, st, asym, comp = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, comp, seed=n + k)
    w = bestla.DeviceWeight(blob)
    A = np.random.default_rng(m + n).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
    ref = oracle.forward(A, blob, n, k)
    tol = 1e-3 if qt in F4 else (TOL[1] if m <= 16 else TOL[64])
    assert _rel_err(y, ref) <= tol, _rel_err(y, ref)


@pytest.mark.parametrize("m", [1, 64])
def test_int8_mode_on_int3(oracle, m):
    n, k = 128, 1024
    blob = _blob(oracle, n, k, 32, S3, F32, True, 4, seed=9)
    w = bestla.DeviceWeight(blob)
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, k)).astype(np.float32)
    prev = bestla.set_compute_mode(bestla.COMPUTE_INT8)
    try:
        y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
    finally:
        bestla.set_compute_mode(prev)
    assert _rel_err(y, oracle.forward_int8(A, blob, n, k)) <= 1e-5


@pytest.mark.parametrize("m", [1, 64])
@pytest.mark.parametrize("qt,st", [(F8_E4M3, F8_E8M0), (F8_E5M2, F8_E8M0), (F8_E5M2, F32)])
def test_f8_small_codes(oracle, qt, st, m):
    """exponent-field-0 codes (the reference reads them as normals: 2^(1-bias) (1 + m)), zeros (code 0x80) and the
    largest codes, through the repack and both kernels"""
    n, k, bs = 64, 512, 32
    rng = np.random.default_rng(5)
    W = rng.uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
    W[:, 1::4] *= np.float32(1e-6)
    W[:, 2::8] = 0.0
    W[:, 0::bs] = np.float32(4.0)
    core = oracle.lib.orc_select_core(1, qt, bs, 0, 0)
    blob = oracle.quant_pack(W, n, k, bs, qt, st, False, core, is_trans=True)
    Q, _, _, _ = oracle.unpack_q(blob)
    assert np.any((Q.view(np.uint8) & 0x7F) >> (3 if qt == F8_E4M3 else 2) == 0)
    w = bestla.DeviceWeight(blob)
    assert np.array_equal(w.unpack().view(np.uint32), oracle.unpack_fp32(blob).view(np.uint32))
    A = np.random.default_rng(m).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
    assert _rel_err(y, oracle.forward(A, blob, n, k)) <= (TOL[1] if m <= 16 else TOL[64])
