"""Prefill GEMMs (woq_gemm2.hip): gemm3 (default: every operand by LDS-DMA, three 64-deep half steps in flight) and
gemm2 (NAD_GEMM_KERNEL=2: A by LDS-DMA one K step ahead, B in registers).

Both run for int4 weights with group size a power-of-two multiple of 128 and M > 16 (capi.hip gemm2_ok); these
cases pin them against the oracle (fp64 GEMM on the reference's dequantized weights) on ragged M/N, K tails, all
scale dtypes, asymmetric zero points, per-channel scales and act-order shuffles.

Tolerances (north_star: 1e-3 relative):
  * fp32 activations (rounded to fp16 once by nad_cvt_act_kernel): max|y - ref| <= 1e-3 * max|ref|
  * fp16 activations (exact inputs, fp32 MFMA accumulation):      max|y - ref| <= 2e-5 * max|ref|
  * bf16 activations (exact in fp16 except below 2^-14):            max|y - ref| <= 1e-4 * max|ref|
"""
import numpy as np
import pytest

from tests.conftest import gpu_available
from tests.oracle_lib import BF16, F16, F32, S2, S4, S8
from tests.test_gpu_parity import _blob, _rel_err

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from neural_amd import bestla

TOL = {"fp32": 1e-3, "fp16": 2e-5, "bf16": 1e-4}

GEMM2_CASES = [
    # m, n, k, bs, qtype, stype, asym, comp, act-order shuffle
    (32, 64, 128, 128, S4, F16, False, 4, False),       # smallest eligible M, one K tile (two half steps)
    (257, 300, 640, 128, S4, BF16, True, 4, False),     # ragged M (one row past a block), ragged N
    (64, 128, 1024, 256, S4, F32, False, 1, False),     # 2 K tiles per group
    (100, 96, 4096, 4096, S4, F32, True, 1, False),     # per-channel
    (96, 130, 300, 128, S4, F16, False, 4, False),      # K tail (300 = 2 tiles + 44, zero padded)
    (64, 80, 512, 128, S4, F16, True, 4, True),         # act-order shuffle gathered during conversion
    (512, 384, 2048, 128, S4, F16, False, 4, False),    # several M and N blocks
    (300, 200, 768, 256, S4, BF16, True, 4, False),     # 3 K tiles at 2 tiles per group: a group ends at the tail
]


@pytest.mark.parametrize("kernel", ["7", "3", "2"])
@pytest.mark.parametrize("cfg", GEMM2_CASES)
@pytest.mark.parametrize("act", ["fp32", "fp16", "bf16"])
def test_gemm_parity(oracle, knob, kernel, cfg, act):
    """gemm3 / gemm2 (held to FOLD_TOL when the launch folds the group scale, which nad_plan_weight reports)."""
    knob("NAD_MID_MAX_M", "0")  # M <= 64 would take the mid-M kernel (tests/test_mid_gpu.py)
    knob("NAD_GEMM_KERNEL", kernel)
    m, n, k, bs, qt, st, asym, comp, shuf = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, comp, seed=m + 3 * n + k, gidx=shuf)
    w = bestla.DeviceWeight(blob)
    assert bool(w.has_shuffle) == shuf
    A = np.random.default_rng(m * 5 + n).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    x = torch.from_numpy(A).cuda()
    if act != "fp32":
        x = x.to(torch.float16 if act == "fp16" else torch.bfloat16)
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    plan = w.plan(m, act)
    y = w.forward(x).cpu().numpy()
    tol = max(TOL[act], FOLD_TOL) if plan["fold"] else TOL[act]
    assert _rel_err(y, ref) <= tol, (_rel_err(y, ref), act)


def test_gemm_kernels_agree(oracle, knob):
    """gemm3, gemm2 and the register-staged fallback (NAD_GEMM2_DISABLE=1) on the same fp16 inputs: each within fp32
    accumulation noise of the oracle and of each other; gemm3 repeatable bit for bit."""
    m, n, k = 700, 272, 1536
    blob = _blob(oracle, n, k, 128, S4, BF16, True, 4, seed=11)
    w = bestla.DeviceWeight(blob)
    knob("NAD_GEMM_KERNEL", "3")  # the exact-scale kernels (gemm7, the default, folds: test_gemm_parity)
    x = (torch.rand((m, k), device="cuda") - 0.5).half()
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    y3 = w.forward(x).cpu().numpy()
    for _ in range(3):
        assert np.array_equal(w.forward(x).cpu().numpy(), y3)
    knob("NAD_GEMM_KERNEL", "2")
    y2 = w.forward(x).cpu().numpy()
    knob("NAD_GEMM2_DISABLE", "1")
    y1 = w.forward(x).cpu().numpy()
    for y in (y3, y2, y1):
        assert _rel_err(y, ref) <= 2e-5
    assert _rel_err(y3, y2.astype(np.float64)) <= 2e-5


def test_gemm_full_size_rows(oracle):
    """BASELINE synthetic GEMM shape K = N = 4096 at M = 4096 (gemm7, scale folded): oracle on sampled rows."""
    n = k = 4096
    blob = _blob(oracle, n, k, 128, S4, F16, False, 4, seed=42)
    w = bestla.DeviceWeight(blob)
    x = (torch.rand((4096, k), device="cuda") - 0.5).half()
    y = w.forward(x).cpu().numpy()
    rows = np.random.default_rng(1).choice(4096, size=16, replace=False)
    ref = oracle.forward(x[rows].float().cpu().numpy(), blob, n, k)
    assert _rel_err(y[rows], ref) <= (FOLD_TOL if w.plan(4096, "fp16")["fold"] else 2e-5)


def test_gemm_strided_epilogues(oracle):
    """lda > k input view, ldc > n output view, bias and residual epilogues on the prefill path."""
    m, n, k = 96, 200, 1024
    blob = _blob(oracle, n, k, 128, S4, F16, False, 4, seed=12)
    w = bestla.DeviceWeight(blob)
    rng = np.random.default_rng(4)
    big = rng.uniform(-0.5, 0.5, size=(m, k + 40)).astype(np.float32)
    x = torch.from_numpy(big).cuda()[:, 8:8 + k]
    A = np.ascontiguousarray(big[:, 8:8 + k])
    ref = oracle.forward(A, blob, n, k).astype(np.float64)
    out = torch.zeros((m, n + 7), device="cuda")[:, :n]
    w.forward(x, out=out)
    assert _rel_err(out.cpu().numpy(), ref) <= TOL["fp32"]
    b = rng.uniform(-1, 1, size=(n,)).astype(np.float32)
    r = rng.uniform(-1, 1, size=(m, n)).astype(np.float32)
    y = w.forward(x, epilogue=bestla.EPI_BIAS, bias=torch.from_numpy(b).cuda()).cpu().numpy()
    assert _rel_err(y, ref + b) <= TOL["fp32"]
    y = w.forward(x, epilogue=bestla.EPI_RES_ADD, residual=torch.from_numpy(r).cuda()).cpu().numpy()
    assert _rel_err(y, ref + r) <= TOL["fp32"]


@pytest.mark.parametrize("m", [32, 200])
def test_gemm_fused_qkv_and_ffn(oracle, m):
    """Fused QKV and gate/up (SiLU*mul) prefill convert the activation once and run the GEMM per weight."""
    k = 512
    blobs = [_blob(oracle, n, k, 128, S4, F16, False, 4, seed=40 + i) for i, n in enumerate((256, 128, 128))]
    ws = [bestla.DeviceWeight(b) for b in blobs]
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, k)).astype(np.float32)
    for y, b, n in zip(bestla.qkv_forward(torch.from_numpy(A).cuda(), *ws), blobs, (256, 128, 128)):
        assert _rel_err(y.cpu().numpy(), oracle.forward(A, b, n, k)) <= TOL["fp32"]
    fin, fmid, fout = 512, 768, 512
    b1 = _blob(oracle, fmid, fin, 128, S4, F16, False, 4, seed=51)
    b3 = _blob(oracle, fmid, fin, 128, S4, F16, False, 4, seed=53)
    b2 = _blob(oracle, fout, fmid, 128, S4, F16, False, 4, seed=52)
    w1, w2, w3 = (bestla.DeviceWeight(b) for b in (b1, b2, b3))
    y = bestla.ffn_forward(torch.from_numpy(A).cuda(), w1, w2, w3, act="silu").cpu().numpy()
    h1 = oracle.forward(A, b1, fmid, fin).astype(np.float64)
    h3 = oracle.forward(A, b3, fmid, fin).astype(np.float64)
    ref = oracle.forward((h1 / (1 + np.exp(-h1)) * h3).astype(np.float32), b2, fout, fmid)
    assert _rel_err(y, ref) <= 2 * TOL["fp32"]


@pytest.mark.parametrize("m,ns,asym", [(2048, (4096, 4096, 4096), False), (1500, (4096, 3072, 3072), True)])
def test_gemm7_fused_qkv_is_the_separate_launches(oracle, knob, m, ns, asym):
    """Fused QKV prefill where each weight runs whole-K gemm7 at one tile height: ONE launch over the weights' column
    tiles (NAD_GEMM7_FUSE) -- bit-identical to one launch per weight, ragged row tiles and unequal N included; against
    the oracle on sampled rows at the fold bar."""
    k = 4096
    blobs = [_blob(oracle, n, k, 128, S4, BF16 if asym else F16, asym, 4, seed=70 + i) for i, n in enumerate(ns)]
    ws = [bestla.DeviceWeight(b) for b in blobs]
    x = (torch.rand((m, k), device="cuda") - 0.5)
    ys = [y.cpu().numpy() for y in bestla.qkv_forward(x, *ws)]
    knob("NAD_GEMM7_FUSE", "0")
    y0 = [y.cpu().numpy() for y in bestla.qkv_forward(x, *ws)]
    for a, b in zip(ys, y0):
        assert np.array_equal(a, b)
    rows = np.random.default_rng(m).choice(m, size=8, replace=False)
    A = x.cpu().numpy()[rows]
    for y, b, n in zip(ys, blobs, ns):
        assert _rel_err(y[rows], oracle.forward(A, b, n, k)) <= FOLD_TOL


GEMM4_CASES = [
    # m, n, k, bs, qtype, stype, asym, comp  -- gemm4 (woq_gemm4.hip): int4 g32 / g64, int2 groups >= 64, int8
    (64, 128, 512, 32, S4, F16, False, 4),        # int4 g32 (the reference Python default group)
    (257, 300, 640, 32, S4, BF16, False, 4),      # ragged M / N, 5 K tiles
    (96, 130, 300, 64, S4, F16, False, 4),        # int4 g64, K tail (zero padded)
    (300, 200, 768, 64, S4, BF16, True, 4),       # int4 g64 asym
    (128, 256, 1024, 64, S2, F16, False, 1),      # int2 g64 (Mistral config 5)
    (200, 96, 640, 64, S2, F32, True, 1),         # int2 g64 asym, K tail inside a 256-deep tile
    (64, 160, 1024, 128, S2, BF16, False, 4),     # int2 g128
    (100, 64, 2048, 256, S2, F16, True, 4),       # int2 g256 asym (one group per tile)
    (48, 80, 1024, 1024, S2, F32, False, 1),      # int2 per-channel
    (128, 200, 640, 32, S4, F16, True, 4),        # int4 g32 asym (compact zero-point slots)
    (64, 128, 512, 32, S8, F16, False, 4),        # int8 g32: one tile per half step, tile two half steps ahead
    (257, 300, 640, 32, S8, BF16, True, 4),       # int8 g32 asym, ragged M / N
    (96, 130, 300, 128, S8, F32, False, 1),       # int8 g128, K tail
    (200, 96, 1024, 256, S8, F16, True, 4),       # int8 g256 asym (four tiles a group)
    (48, 80, 512, 512, S8, BF16, False, 1),       # int8 per-channel
    (33, 64, 64, 64, S8, F16, True, 4),           # int8, a single half step
    (40, 48, 128, 64, S8, F16, False, 4),         # int8, two half steps
]


@pytest.mark.parametrize("ksw", ["0", "1"])
@pytest.mark.parametrize("cfg", GEMM4_CASES)
@pytest.mark.parametrize("act", ["fp32", "fp16", "bf16"])
def test_gemm4_parity(oracle, knob, cfg, act, ksw):
    """gemm4 against the oracle (NAD_GEMM4_KSW=1: folded launches with the waves split over K; NAD_GEMM_KERNEL=3 keeps
    int4 g32 / g64 on gemm4, tests/test_gemm2_gpu.py::test_gemm7_small_groups covers their default gemm7 path)."""
    knob("NAD_MID_MAX_M", "0")
    knob("NAD_GEMM_KERNEL", "3")
    knob("NAD_GEMM4_KSW", ksw)
    m, n, k, bs, qt, st, asym, comp = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, comp, seed=m + 7 * n + k)
    w = bestla.DeviceWeight(blob)
    A = np.random.default_rng(m * 3 + n).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    x = torch.from_numpy(A).cuda()
    if act != "fp32":
        x = x.to(torch.float16 if act == "fp16" else torch.bfloat16)
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    y = w.forward(x).cpu().numpy()
    # a launch that folds the group scale into the fp16 weights (q * s rounded once to fp16; the library reports it,
    # nad_plan_weight) is held to FOLD_TOL, the north_star-side bar of a product with fp16 weights; every other launch
    # keeps the exact-weight bars (test_gemm4_g32_scale_fold)
    tol = max(TOL[act], FOLD_TOL) if w.plan(m, act)["fold"] else TOL[act]
    assert _rel_err(y, ref) <= tol, (_rel_err(y, ref), act)


FOLD_TOL = 5e-4


@pytest.mark.parametrize("cfg", [c for c in GEMM4_CASES if c[3] == 64])
def test_gemm4_g64_scale_fold(oracle, knob, cfg):
    """Groups of 64 fold the group scale into the fp16 B fragment too (int4 / int2 / int8): against the oracle and the
    exact fp32 group-end scaling (NAD_GEMM4_FOLD=0)."""
    knob("NAD_GEMM_KERNEL", "3")
    m, n, k, bs, qt, st, asym, comp = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, comp, seed=m + 9 * n + k)
    w = bestla.DeviceWeight(blob)
    x = torch.from_numpy(np.random.default_rng(m + n + 1).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)).cuda().half()
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    yf = w.forward(x).cpu().numpy()
    knob("NAD_GEMM4_FOLD", "0")
    ye = w.forward(x).cpu().numpy()
    assert _rel_err(ye, ref) <= TOL["fp16"]
    assert _rel_err(yf, ref) <= FOLD_TOL
    assert _rel_err(yf, ye) <= FOLD_TOL


@pytest.mark.parametrize("cfg", [c for c in GEMM4_CASES if c[3] == 32])
def test_gemm4_g32_scale_fold(oracle, knob, cfg):
    """Groups of 32 fold the group scale into the fp16 B fragment by default (q * s rounded once to fp16; every q * s of
    these blobs is an fp16 normal, DeviceWeight::fold_ok): against the oracle at the prefill bar, and against the exact
    fp32 per-step scaling (NAD_GEMM4_FOLD=0) within the fp16 rounding of q * s (2^-11 relative per weight)."""
    knob("NAD_GEMM_KERNEL", "3")
    m, n, k, bs, qt, st, asym, comp = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, comp, seed=m + 5 * n + k)
    w = bestla.DeviceWeight(blob)
    x = torch.from_numpy(np.random.default_rng(m + n).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)).cuda().half()
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    yf = w.forward(x).cpu().numpy()
    knob("NAD_GEMM4_FOLD", "0")
    ye = w.forward(x).cpu().numpy()
    assert _rel_err(yf, ref) <= FOLD_TOL
    assert _rel_err(ye, ref) <= TOL["fp16"]
    assert _rel_err(yf, ye) <= FOLD_TOL


GEMM7_GROUP_CASES = [
    # m, n, k, bs, qtype, stype, asym -- gemm7 beyond int4 g128: int4 g32 / g64 (the group scale per 32-deep step), int2
    # and int8 (half-step mode: the B slice, scales and zero points of every 64-deep half step loaded with it)
    (2048, 512, 1024, 32, S4, F16, False),    # 256-row tiles
    (300, 384, 640, 32, S4, BF16, True),      # ragged M, 256-row tiles, 5 K tiles
    (100, 130, 512, 32, S4, F32, False),      # 128-row tile, ragged N (a partial stripe), f32 scales (the largest region)
    (257, 300, 640, 32, S4, F32, True),       # f32 asym: the 256-row tile's LDS at its largest (scales 2 KiB, zp 512 B)
    (96, 130, 300, 64, S4, F16, False),       # g64, K tail (zero padded), 128-row tile
    (300, 200, 768, 64, S4, BF16, True),      # g64 asym
    (65, 1024, 4096, 32, S4, F16, True),      # 128-row tile with split-K runs
    (200, 640, 2048, 64, S4, F32, True),      # 256-row tile with split-K runs
    (300, 256, 1024, 64, S2, F16, False),     # int2 g64 (Mistral): one group per half step
    (257, 200, 768, 64, S2, BF16, True),      # int2 g64 asym, ragged, K = 3 int2 tiles
    (100, 96, 640, 128, S2, F32, True),       # int2 g128, K tail inside a 256-deep tile, 128-row tile
    (64, 1024, 4096, 256, S2, F16, False),    # int2 g256, 64-row tile with split-K runs
    (48, 160, 1024, 1024, S2, F16, True),     # int2 per-channel (a group of 16 half steps)
    (200, 256, 1024, 32, S2, F16, False),     # int2 g32: two groups per half step
    (100, 130, 768, 32, S2, F32, True),       # int2 g32 f32 asym, ragged N, 3 int2 tiles
    (300, 256, 1024, 32, S8, F16, False),     # int8 g32: two groups per half step
    (96, 200, 512, 512, S8, BF16, True),      # int8 per-channel asym (one group of 8 half steps)
    (257, 300, 640, 32, S8, F32, True),       # int8 g32 f32 asym: the 256-row tile's int8 slices at their largest
    (96, 130, 320, 128, S8, BF16, False),     # int8 g128, an odd half-step count (5 tiles: one all-zero padding step)
    (200, 96, 1024, 256, S8, F16, True),      # int8 g256 asym
    (33, 640, 2048, 64, S8, F16, False),      # int8, 64-row tile (M = 33) with split-K runs
]


@pytest.mark.parametrize("cfg", GEMM7_GROUP_CASES)
@pytest.mark.parametrize("act", ["fp32", "fp16", "bf16"])
def test_gemm7_small_groups(oracle, knob, cfg, act):
    """gemm7 at int4 g32 / g64, int2 and int8 (q * s rounded once to fp16): against the oracle at the fold bar, against
    gemm4's folded launch (NAD_GEMM_KERNEL=3: the same fp16 weights up to the scale's own fp16 rounding; int2 g32, which
    gemm4 does not take, the generic tiled GEMM) and gemm4's exact fp32 group scales (NAD_GEMM4_FOLD=0); bit-repeatable."""
    m, n, k, bs, qt, st, asym = cfg
    knob("NAD_MID_MAX_M", "0")
    blob = _blob(oracle, n, k, bs, qt, st, asym, 4, seed=m + 11 * n + k)
    w = bestla.DeviceWeight(blob)
    plan = w.plan(m, act)
    assert plan["kernel"] == "woq_gemm7_kernel" and plan["fold"], plan
    A = np.random.default_rng(m * 5 + n).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    x = torch.from_numpy(A).cuda()
    if act != "fp32":
        x = x.to(torch.float16 if act == "fp16" else torch.bfloat16)
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    y = w.forward(x).cpu().numpy()
    assert _rel_err(y, ref) <= max(TOL[act], FOLD_TOL), (_rel_err(y, ref), plan)
    assert np.array_equal(w.forward(x).cpu().numpy(), y)
    knob("NAD_GEMM_KERNEL", "3")
    assert w.plan(m, act)["kernel"] in ("woq_gemm4_kernel", "woq_gemm_kernel")  # int2 g32: the generic tiled GEMM
    y4 = w.forward(x).cpu().numpy()
    assert _rel_err(y, y4.astype(np.float64)) <= FOLD_TOL
    knob("NAD_GEMM_KERNEL", "7")
    knob("NAD_GEMM4_FOLD", "0")
    ye = w.forward(x).cpu().numpy()
    assert _rel_err(ye, ref) <= TOL[act]
    assert _rel_err(y, ye.astype(np.float64)) <= FOLD_TOL


def test_gemm4_takes_the_fallback_configs(oracle, knob):
    """With gemm4 disabled the same inputs run the register-staged kernel: both agree within fp32 accumulation noise
    (they see identical fp16 A and exact weights).  NAD_GEMM_KERNEL=3: int2 otherwise runs gemm7."""
    knob("NAD_GEMM_KERNEL", "3")
    m, n, k = 200, 256, 1024
    blob = _blob(oracle, n, k, 64, S2, F16, True, 1, seed=5)
    w = bestla.DeviceWeight(blob)
    x = (torch.rand((m, k), device="cuda") - 0.5).half()
    y4 = w.forward(x).cpu().numpy()
    knob("NAD_GEMM4_DISABLE", "1")
    y1 = w.forward(x).cpu().numpy()
    assert _rel_err(y4, y1.astype(np.float64)) <= 2e-5


SPLITK_CASES = [
    # m, n, k, bs, asym, act -- few 256 x 128 output tiles: gemm3 runs split-K (capi.hip splitk_plan) + the ordered reduce
    (17, 4096, 4096, 128, False, "fp16"),     # smallest M past the GEMV (was the register-staged fallback)
    (31, 1024, 4096, 128, True, "fp32"),
    (64, 4096, 4096, 128, False, "fp32"),     # batched decode at the Llama O shape: 32 tiles x 8 runs of 4 K tiles
    (100, 1024, 11008, 128, True, "bf16"),    # down-like K = 86 tiles: runs of 3, the last one shorter
    (256, 2048, 4096, 256, False, "fp16"),    # 2 K tiles per group: runs of whole groups
    (512, 1536, 4096, 128, True, "fp16"),     # a TP-8 QKV shard width at a 512-token prefill chunk
    (96, 1000, 4096, 128, False, "fp16"),     # ragged N (63 stripes, 16 tiles): a tile's runs + their reduce on one XCD
]


@pytest.mark.parametrize("cfg", SPLITK_CASES)
def test_gemm_splitk_parity(oracle, knob, cfg):
    """Split-K gemm3 against the oracle, and against the same GEMM without the split (fp32 sums in another order)."""
    knob("NAD_MID_MAX_M", "0")
    m, n, k, bs, asym, act = cfg
    blob = _blob(oracle, n, k, bs, S4, F16, asym, 4, seed=m + n + k)
    w = bestla.DeviceWeight(blob)
    A = np.random.default_rng(m + 17).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    x = torch.from_numpy(A).cuda()
    if act != "fp32":
        x = x.to(torch.float16 if act == "fp16" else torch.bfloat16)
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    y = w.forward(x).cpu().numpy()
    tol = max(TOL[act], FOLD_TOL) if w.plan(m, act)["fold"] else TOL[act]  # gemm7 folds the scale (fp16 weights)
    assert _rel_err(y, ref) <= tol, (_rel_err(y, ref), act)
    knob("NAD_SPLITK_DISABLE", "1")
    y1 = w.forward(x).cpu().numpy()
    assert _rel_err(y, y1.astype(np.float64)) <= 2e-5
    knob("NAD_SPLITK_DISABLE", "0")
    knob("NAD_GEMM_KERNEL", "3")  # the exact-scale gemm3 split-K path at the exact bar
    y3 = w.forward(x).cpu().numpy()
    assert _rel_err(y3, ref) <= TOL[act], (_rel_err(y3, ref), act)


@pytest.mark.parametrize("mid", [True, False])
def test_gemm_splitk_epilogues(oracle, knob, mid):
    """The split-K reduce applies bias, residual and the FFN's SiLU*mul after summing the runs: the mid-M kernel's
    (stripe groups on one XCD) and gemm7's (NAD_MID_MAX_M=0: a tile's runs on one XCD, the scale folded)."""
    if not mid:
        knob("NAD_MID_MAX_M", "0")
    m, n, k = 48, 1024, 2048
    blob = _blob(oracle, n, k, 128, S4, F16, False, 4, seed=91)
    w = bestla.DeviceWeight(blob)
    rng = np.random.default_rng(9)
    A = rng.uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    x = torch.from_numpy(A).cuda()
    ref = oracle.forward(A, blob, n, k).astype(np.float64)
    plan = w.plan(m, "fp32")
    assert plan["kernel"] == ("woq_mid_kernel" if mid else "woq_gemm7_kernel") and plan["ksplit"] > 1, plan
    tol = TOL["fp32"] if mid else FOLD_TOL
    b = rng.uniform(-1, 1, size=(n,)).astype(np.float32)
    r = rng.uniform(-1, 1, size=(m, n)).astype(np.float32)
    y = w.forward(x, epilogue=bestla.EPI_BIAS, bias=torch.from_numpy(b).cuda()).cpu().numpy()
    assert _rel_err(y, ref + b) <= tol
    y = w.forward(x, epilogue=bestla.EPI_RES_ADD, residual=torch.from_numpy(r).cuda()).cpu().numpy()
    assert _rel_err(y, ref + r) <= tol
    fin, fmid, fout = 2048, 1024, 2048
    b1, b3, b2 = (_blob(oracle, nn, kk, 128, S4, F16, False, 4, seed=s)
                  for nn, kk, s in ((fmid, fin, 61), (fmid, fin, 63), (fout, fmid, 62)))
    w1, w2, w3 = (bestla.DeviceWeight(bb) for bb in (b1, b2, b3))
    y = bestla.ffn_forward(x, w1, w2, w3, act="silu").cpu().numpy()
    h1 = oracle.forward(A, b1, fmid, fin).astype(np.float64)
    h3 = oracle.forward(A, b3, fmid, fin).astype(np.float64)
    ref = oracle.forward((h1 / (1 + np.exp(-h1)) * h3).astype(np.float32), b2, fout, fmid)
    assert _rel_err(y, ref) <= 2 * tol


SPLITK4_CASES = [
    # m, n, k, bs, qtype, asym, act -- gemm4 formats with few output tiles: split-K runs of whole groups
    (256, 1024, 4096, 64, S2, False, "fp16"),    # Mistral k/v projection (int2 g64) at a 256-token chunk
    (64, 4096, 4096, 32, S4, True, "fp32"),      # int4 g32 asym (the reference Python default group), batched decode
    (48, 2048, 2048, 128, S8, False, "bf16"),    # int8 g128: runs of two 64-deep tiles per group
    (96, 512, 4096, 128, S2, True, "fp16"),      # int2 g128 asym, 4 half steps per tile
    (17, 4096, 4096, 32, S4, False, "fp32"),     # M just past the GEMV (was the register-staged fallback)
    (24, 1024, 4096, 64, S2, True, "bf16"),
    (31, 768, 2048, 32, S8, True, "fp16"),
]


@pytest.mark.parametrize("cfg", SPLITK4_CASES)
def test_gemm4_splitk_parity(oracle, knob, cfg):
    m, n, k, bs, qt, asym, act = cfg
    knob("NAD_MID_MAX_M", "0")
    blob = _blob(oracle, n, k, bs, qt, F16, asym, 4, seed=m + 3 * n + k)
    w = bestla.DeviceWeight(blob)
    A = np.random.default_rng(m + 5).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    x = torch.from_numpy(A).cuda()
    if act != "fp32":
        x = x.to(torch.float16 if act == "fp16" else torch.bfloat16)
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    y = w.forward(x).cpu().numpy()
    tol = max(TOL[act], FOLD_TOL) if w.plan(m, act)["fold"] else TOL[act]  # scale folded into the fp16 weights
    assert _rel_err(y, ref) <= tol, (_rel_err(y, ref), act)
    knob("NAD_SPLITK_DISABLE", "1")
    y1 = w.forward(x).cpu().numpy()
    assert _rel_err(y, y1.astype(np.float64)) <= 2e-5


@pytest.mark.parametrize("qt,bs", [(S4, 128), (S2, 64), (S4, 32)])
def test_ffn_prefill_fp16_intermediates(oracle, knob, qt, bs):
    """The prefill FFN keeps act(x.W1) and act(x.W1)*(x.W3) in fp16 (the down GEMM reads the second one as its operand
    directly): within the fp32-path tolerance of the oracle and of the fp32-intermediate path (NAD_FFN_F32=1)."""
    m, fin, fmid, fout = 160, 1024, 1536, 1024
    b1, b3, b2 = (_blob(oracle, nn, kk, bs, qt, F16, False, 4, seed=s)
                  for nn, kk, s in ((fmid, fin, 71), (fmid, fin, 73), (fout, fmid, 72)))
    w1, w2, w3 = (bestla.DeviceWeight(bb) for bb in (b1, b2, b3))
    A = np.random.default_rng(13).uniform(-1, 1, size=(m, fin)).astype(np.float32)
    x = torch.from_numpy(A).cuda()
    y = bestla.ffn_forward(x, w1, w2, w3, act="silu").cpu().numpy()
    h1 = oracle.forward(A, b1, fmid, fin).astype(np.float64)
    h3 = oracle.forward(A, b3, fmid, fin).astype(np.float64)
    ref = oracle.forward((h1 / (1 + np.exp(-h1)) * h3).astype(np.float32), b2, fout, fmid)
    assert _rel_err(y, ref) <= TOL["fp32"], _rel_err(y, ref)
    knob("NAD_FFN_F32", "1")
    y32 = bestla.ffn_forward(x, w1, w2, w3, act="silu").cpu().numpy()
    assert _rel_err(y32, ref) <= TOL["fp32"], _rel_err(y32, ref)
    assert _rel_err(y, y32.astype(np.float64)) <= TOL["fp32"]
    assert not np.array_equal(y, y32)   # the fp16 path really ran (different rounding of the intermediates)


MID_M = [17, 32, 33, 64, 100, 128, 200, 256, 512]


@pytest.mark.parametrize("m", MID_M)
@pytest.mark.parametrize("fmt", [(S4, 128, F16, False), (S4, 128, BF16, True), (S2, 64, F16, False), (S2, 64, F16, True)])
def test_gemm_mid_m(oracle, knob, m, fmt):
    """The mid-M range (17 <= M <= 512): int4 g128 runs gemm7 with a tile of 32 / 64 / 128 / 256
    rows and split-K runs (the plan reports the split), int2 g64 gemm4; fp16 activations against the oracle at the
    fold bar, and -- for int4 -- against gemm3 (exact scale, 256-row tiles) on the same inputs."""
    qt, bs, st, asym = fmt
    n, k = 1024, 2048
    blob = _blob(oracle, n, k, bs, qt, st, asym, 4, seed=m * 7 + bs)
    w = bestla.DeviceWeight(blob)
    x = (torch.from_numpy(np.random.default_rng(m).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32))
         .cuda().half())
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    plan = w.plan(m, "fp16")
    y = w.forward(x).cpu().numpy()
    assert _rel_err(y, ref) <= (FOLD_TOL if plan["fold"] else TOL["fp16"]), (_rel_err(y, ref), plan)
    if m <= (64 if qt == S4 else 32):  # the mid-M kernel (exact scales; tests/test_mid_gpu.py)
        assert plan["kernel"] == "woq_mid_kernel", plan
        return
    if qt == S4:
        assert plan["kernel"] == "woq_gemm7_kernel" and plan["ksplit"] > 1, plan
        knob("NAD_GEMM_KERNEL", "3")
        y3 = w.forward(x).cpu().numpy()
        assert _rel_err(y, y3.astype(np.float64)) <= FOLD_TOL



@pytest.mark.parametrize("edge,folds", [
    (2.0 ** -14, True),                  # the smallest scale whose q * s is an fp16 normal for every |q| >= 1
    (2.0 ** -14 * (1 - 2.0 ** -20), False),
    (65504.0 / 8, True),                 # int4 sym: qmax * s = 8 * 8188 = 65504, the largest fp16
    (65504.0 / 8 * (1 + 2.0 ** -20), False),
])
def test_fold_range_edge_scales(oracle, edge, folds):
    """the load-time fold check (capi.hip scale_in_fold_range) at the edges of the fp16 range.  A
    blob whose group scales sit exactly on an edge folds q * s into fp16 (gemm7) and is held to FOLD_TOL; one just past
    it runs the exact fp32 group-scale path (gemm3) and is held to the fp16-activation bar, both against the oracle."""
    m, n, k, g = 128, 256, 1024, 128
    rng = np.random.default_rng(17)
    q = rng.integers(-8, 8, size=(k, n)).astype(np.int8)
    s = rng.uniform(0.001, 0.01, size=(k // g, n)).astype(np.float32)
    s[::3, ::5] = np.float32(edge)       # a sprinkling of edge scales over groups and columns
    s[1, 7] = -np.float32(edge)          # the check takes |s|
    blob = bestla.qpack(q, s, weight_dtype="int4", group_size=g, alg="sym", scale_dtype="fp32", compute_dtype="fp32")
    w = bestla.DeviceWeight(blob)
    p = w.plan(m, "fp16")
    assert p["fold"] == folds, p
    assert p["kernel"] == ("woq_gemm7_kernel" if folds else "woq_gemm3_kernel"), p
    x = torch.from_numpy(rng.uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)).cuda().half()
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    y = w.forward(x).cpu().numpy()
    assert np.isfinite(y).all()
    assert _rel_err(y, ref) <= (FOLD_TOL if folds else TOL["fp16"]), _rel_err(y, ref)
