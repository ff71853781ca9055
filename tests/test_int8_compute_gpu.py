"""GPU int8-compute mode (woq_i8.hip) against the oracle.

  * the activation quantizer (nad_quant_u8_colblock): bit-exact u8 codes, scales, zero points and block reduce vs the
    reference's own outputs (tests/golden/ref/qu8_*, kernel_ref.h:1824-1883) and vs the oracle on larger inputs;
  * the forward in mode 1: the oracle's kblock int8 GEMM (orc_blob_forward_int8: same u8 codes, same s32 block dots,
    same fp32 combine order) within 1e-5 of max|ref| -- the GPU differs only in summing K-split partials at M <= 16;
  * mode 0 on the same blob stays the fp path; fused entries in mode 1 equal their single-weight compositions.
"""
import numpy as np
import pytest

from tests.conftest import gpu_available
from tests.oracle_lib import BF16, F16, F32, S2, S4, S5, S6, S7, S8, load_ref_golden
from tests.test_gpu_parity import _blob, _rel_err

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from neural_amd import bestla

TOL_I8 = 1e-5


@pytest.fixture
def int8_mode():
    prev = bestla.set_compute_mode(bestla.COMPUTE_INT8)
    yield
    bestla.set_compute_mode(prev)


@pytest.mark.parametrize("case", ["qu8_g32", "qu8_g128_tail", "qu8_perchannel", "qu8_g64_big"])
def test_quant_u8_matches_reference_golden(case):
    g = load_ref_golden()[case]
    row, col, bs = (int(v) for v in g["meta"])
    x = torch.from_numpy(g["src"].reshape(row, col).copy()).cuda()
    q, s, z, red = (t.cpu().numpy() for t in bestla.quant_u8_colblock(x, bs))
    assert np.array_equal(q.ravel(), g["q"])
    assert np.array_equal(s.ravel().view(np.uint32), g["s"].view(np.uint32))
    assert np.array_equal(z.ravel(), g["zp"])
    assert np.array_equal(red.ravel().view(np.uint32), g["red"].view(np.uint32))


@pytest.mark.parametrize("m,k,bs,amp,act", [(64, 4096, 32, 1.0, "fp32"), (33, 4096, 128, 30.0, "fp16"),
                                            (17, 1000, 64, 0.01, "bf16"), (5, 11008, 11008, 4.0, "fp32")])
def test_quant_u8_matches_oracle(oracle, m, k, bs, amp, act):
    rng = np.random.default_rng(m + k)
    A = rng.uniform(-amp, amp, size=(m, k)).astype(np.float32)
    A[0, :bs] = 0.0                                   # an all-zero block
    A[1 % m, :bs] = np.abs(A[1 % m, :bs])             # an all-positive block
    x = torch.from_numpy(A).cuda()
    if act != "fp32":
        x = x.to(torch.float16 if act == "fp16" else torch.bfloat16)
    q, s, z, red = (t.cpu().numpy() for t in bestla.quant_u8_colblock(x, bs))
    oq, os_, oz, ored = oracle.quant_u8(x.float().cpu().numpy(), bs, want_reduce=True)
    assert np.array_equal(q, oq) and np.array_equal(z, oz)
    assert np.array_equal(s.view(np.uint32), os_.view(np.uint32))
    assert np.array_equal(red.view(np.uint32), ored.view(np.uint32))


I8_CASES = [
    # n, k, bs, qtype, stype, asym, act-order shuffle
    (256, 1024, 32, S4, F32, False, False),     # the reference Python default: int4 g32 sym, comp int8
    (200, 768, 32, S4, BF16, True, False),      # asym weights, ragged N
    (128, 2048, 128, S4, F16, True, False),     # GPTQ-style g128 asym
    (96, 1024, 1024, S4, F32, False, False),    # per-channel
    (160, 1024, 64, S2, F32, False, False),     # int2 g64
    (64, 512, 64, S2, F32, True, False),        # int2 asym
    (128, 512, 32, S8, F32, False, False),      # int8 sym
    (64, 512, 128, S4, F32, True, True),        # act-order shuffle (gather before quantization)
    (48, 300, 32, S4, F32, False, False),       # K tail inside a tile and a block
    # 5/6/7-bit asym (int8 device layout q + 128 with separate zero points; ADVICE r2: the zp was dropped there)
    (96, 512, 32, S5, F32, True, False),
    (64, 768, 64, S6, BF16, True, False),
    (80, 512, 128, S7, F32, True, False),
]


@pytest.mark.parametrize("m", [1, 4, 16, 33, 200])
@pytest.mark.parametrize("cfg", I8_CASES)
def test_int8_forward_matches_oracle(oracle, int8_mode, cfg, m):
    n, k, bs, qt, st, asym, shuf = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, 4, seed=n + k + bs, gidx=shuf)
    assert oracle.info(blob)["has_reduce"] == 1
    w = bestla.DeviceWeight(blob)
    A = np.random.default_rng(m * 7 + n).uniform(-1, 1, size=(m, k)).astype(np.float32)
    y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
    ref = oracle.forward_int8(A, blob, n, k)
    assert _rel_err(y, ref) <= TOL_I8, _rel_err(y, ref)


@pytest.mark.parametrize("act", ["fp16", "bf16"])
def test_int8_forward_half_activations(oracle, int8_mode, act):
    n, k, bs = 128, 1024, 32
    blob = _blob(oracle, n, k, bs, S4, F32, True, 4, seed=11)
    w = bestla.DeviceWeight(blob)
    for m in (3, 70):
        x = (torch.rand((m, k), device="cuda") - 0.5).to(torch.float16 if act == "fp16" else torch.bfloat16)
        ref = oracle.forward_int8(x.float().cpu().numpy(), blob, n, k)
        assert _rel_err(w.forward(x).cpu().numpy(), ref) <= TOL_I8


def test_mode_off_keeps_fp_path(oracle):
    assert bestla.get_compute_mode() == bestla.COMPUTE_FP
    n, k = 128, 1024
    blob = _blob(oracle, n, k, 32, S4, F32, False, 4, seed=5)
    w = bestla.DeviceWeight(blob)
    x = (torch.rand((8, k), device="cuda") - 0.5).half()
    y = w.forward(x).cpu().numpy()
    assert _rel_err(y, oracle.forward(x.float().cpu().numpy(), blob, n, k)) <= 2e-5
    assert _rel_err(y, oracle.forward_int8(x.float().cpu().numpy(), blob, n, k)) > 1e-4  # genuinely different math


def test_float_core_blob_stays_fp_in_int8_mode(oracle, int8_mode):
    """a blob packed for a float core has no reduce: the reference computes it in fp, and so does mode 1"""
    n, k = 64, 512
    blob = _blob(oracle, n, k, 32, S4, F32, False, 1, seed=6)
    assert oracle.info(blob)["has_reduce"] == 0
    w = bestla.DeviceWeight(blob)
    x = (torch.rand((5, k), device="cuda") - 0.5).half()
    assert _rel_err(w.forward(x).cpu().numpy(), oracle.forward(x.float().cpu().numpy(), blob, n, k)) <= 2e-5


@pytest.mark.parametrize("m", [2, 64])
def test_int8_fused_entries(oracle, int8_mode, m):
    k, nq, nkv, fmid = 512, 256, 128, 384
    bq, bk, bv = (_blob(oracle, n, k, 32, S4, F32, False, 4, seed=s) for n, s in ((nq, 1), (nkv, 2), (nkv, 3)))
    wq, wk, wv = (bestla.DeviceWeight(b) for b in (bq, bk, bv))
    x = torch.rand((m, k), device="cuda") - 0.5
    xa = x.cpu().numpy()
    oq, ok, ov = bestla.qkv_forward(x, wq, wk, wv)
    for o, b, n in ((oq, bq, nq), (ok, bk, nkv), (ov, bv, nkv)):
        assert _rel_err(o.cpu().numpy(), oracle.forward_int8(xa, b, n, k)) <= TOL_I8
    b1, b3 = (_blob(oracle, fmid, k, 32, S4, F32, False, 4, seed=s) for s in (4, 5))
    w1, w3 = bestla.DeviceWeight(b1), bestla.DeviceWeight(b3)
    tmp2 = bestla.ffn_gate_up(x, w1, w3, act="silu")
    g = oracle.forward_int8(xa, b1, fmid, k)
    u = oracle.forward_int8(xa, b3, fmid, k)
    silu = g / (1.0 + np.exp(-g))
    assert _rel_err(tmp2.cpu().numpy(), silu * u) <= 1e-4
