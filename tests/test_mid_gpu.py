"""The mid-M GEMM (woq_gemm_mid.hip, 12 (fp16) / 8 (fp32, bf16) <= M <= 64): operands straight to registers, the
split-K runs' slabs summed in run order by the reduce launch.

Against the oracle (fp64 GEMM on the reference's dequantized weights, bestla_wrapper.h:471-542 semantics) on the
formats the kernel takes (int4 / int2, sym / asym, groups of 32 .. per-channel, fp32 / fp16 / bf16 scales), ragged M / N,
K tails, every activation type and the epilogues; bit-identical across repeated launches and under graph replay.

Tolerance: the decode GEMV's -- the group scale is applied exactly in fp32 and fp32 / bf16 activations enter as fp16
hi + lo rows (two MFMAs), so every activation type is held to 2e-5 of max|ref|.
"""
import numpy as np
import pytest

from tests.conftest import gpu_available
from tests.oracle_lib import BF16, F16, F32, S2, S4
from tests.test_gpu_parity import _blob, _rel_err

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from neural_amd import bestla

TOL = {"fp32": 2e-5, "fp16": 2e-5, "bf16": 2e-5}

MID_CASES = [
    # m, n, k, bs, qtype, stype, asym
    (17, 4096, 4096, 128, S4, F16, False),     # just past the GEMV; the Llama O shape (4 runs, 256 workgroups)
    (64, 4096, 4096, 128, S4, F16, False),     # batched decode at 64 rows
    (33, 1000, 2048, 128, S4, BF16, True),     # ragged N (a partial stripe group), asym, bf16 scales
    (48, 512, 1000, 128, S4, F32, False),      # K tail (1000 = 7 tiles + 104), f32 scales
    (24, 768, 4096, 4096, S4, F16, True),      # per-channel asym (one group: tpg_shift 31)
    (32, 640, 2048, 256, S4, F16, False),      # groups of two K tiles
    (32, 384, 2048, 32, S4, F16, False),       # int4 g32 (the reference Python default group; M <= 32): 4 groups per tile
    (56, 320, 1024, 64, S4, BF16, True),       # int4 g64 asym: 2 groups per tile
    (32, 1024, 4096, 64, S2, F16, False),      # int2 g64 (Mistral; int2 takes M <= 32)
    (20, 1024, 4096, 64, S2, F16, True),       # int2 g64 asym
    (28, 448, 1280, 128, S2, F32, False),      # int2 g128, K tail inside a 256-deep tile
    (30, 256, 2048, 256, S2, F16, True),       # int2 g256 asym
    (64, 4096, 11008, 128, S4, F16, False),    # the Llama down shape: 86 K tiles, 11 runs
    (32, 11008, 4096, 128, S4, F16, False),    # the Llama gate shape: 8-stripe workgroups (172 instead of 344)
    (24, 9000, 4096, 128, S4, F32, False),     # 8-stripe workgroups, ragged last group (563 stripes), 3 runs
    (20, 12288, 2048, 64, S4, BF16, True),     # 8-stripe workgroups at g64 asym (2 groups per tile)
]


def _x(m, k, act, seed):
    A = np.random.default_rng(seed).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    x = torch.from_numpy(A).cuda()
    if act != "fp32":
        x = x.to(torch.float16 if act == "fp16" else torch.bfloat16)
    return x


@pytest.mark.parametrize("cfg", MID_CASES)
@pytest.mark.parametrize("act", ["fp32", "fp16", "bf16"])
def test_mid_parity(oracle, knob, cfg, act):
    m, n, k, bs, qt, st, asym = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, 4, seed=m + 5 * n + k)
    w = bestla.DeviceWeight(blob)
    plan = w.plan(m, act)
    assert plan["kernel"] == "woq_mid_kernel" and not plan["fold"], plan
    assert plan["launches"] == (1 if plan["ksplit"] == 1 else 2), plan  # split K: the reduce launch
    x = _x(m, k, act, m * 3 + n)
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    y = w.forward(x).cpu().numpy()
    assert _rel_err(y, ref) <= TOL[act], (_rel_err(y, ref), act, plan)
    for _ in range(2):  # repeatable bit for bit (the reduce sums the runs in run order)
        assert np.array_equal(w.forward(x).cpu().numpy(), y)


@pytest.mark.parametrize("ks", ["1", "2", "3", "7"])
def test_mid_k_runs(oracle, knob, ks):
    """Forced run counts (NAD_MID_KS): one run (no combine), uneven runs, runs of more than one chunk."""
    m, n, k = 40, 1024, 4096
    blob = _blob(oracle, n, k, 128, S4, F16, True, 4, seed=int(ks))
    w = bestla.DeviceWeight(blob)
    x = _x(m, k, "fp16", 5)
    ref = oracle.forward(x.float().cpu().numpy(), blob, n, k)
    knob("NAD_MID_KS", ks)
    assert w.plan(m, "fp16")["ksplit"] == int(ks)
    y = w.forward(x).cpu().numpy()
    assert _rel_err(y, ref) <= TOL["fp16"], _rel_err(y, ref)


def test_mid_matches_prefill_and_gemv(oracle, knob):
    """The same inputs through the mid-M kernel, the prefill GEMM (NAD_MID_MAX_M=0) and the GEMV's exact arithmetic at
    M = 16 rows of them: all within fp32 accumulation noise of each other."""
    m, n, k = 32, 2048, 4096
    blob = _blob(oracle, n, k, 128, S4, F16, False, 4, seed=7)
    w = bestla.DeviceWeight(blob)
    x = _x(m, k, "fp16", 8)
    y = w.forward(x).cpu().numpy()
    knob("NAD_MID_MIN_M", "17")  # fp16 rows take the mid-M kernel from 12: force the GEMV for the M = 16 cross-check
    assert w.plan(16, "fp16")["kernel"] == "woq_gemv_kernel"
    y16 = w.forward(x[:16].contiguous()).cpu().numpy()
    assert _rel_err(y[:16], y16.astype(np.float64)) <= 2e-5
    knob("NAD_MID_MAX_M", "0")
    knob("NAD_GEMM_KERNEL", "3")
    y3 = w.forward(x).cpu().numpy()
    assert _rel_err(y, y3.astype(np.float64)) <= 2e-5


def test_mid_epilogues(oracle):
    """bias, residual, SiLU and the strided views through the split-K reduce."""
    m, n, k = 48, 1000, 2048
    blob = _blob(oracle, n, k, 128, S4, F16, False, 4, seed=91)
    w = bestla.DeviceWeight(blob)
    rng = np.random.default_rng(9)
    big = rng.uniform(-0.5, 0.5, size=(m, k + 24)).astype(np.float32)
    x = torch.from_numpy(big).cuda()[:, 8:8 + k]
    A = np.ascontiguousarray(big[:, 8:8 + k])
    ref = oracle.forward(A, blob, n, k).astype(np.float64)
    assert w.plan(m, "fp32")["ksplit"] > 1
    out = torch.zeros((m, n + 12), device="cuda")[:, :n]
    w.forward(x, out=out)
    assert _rel_err(out.cpu().numpy(), ref) <= TOL["fp32"]
    b = rng.uniform(-1, 1, size=(n,)).astype(np.float32)
    r = rng.uniform(-1, 1, size=(m, n)).astype(np.float32)
    y = w.forward(x, epilogue=bestla.EPI_BIAS, bias=torch.from_numpy(b).cuda()).cpu().numpy()
    assert _rel_err(y, ref + b) <= TOL["fp32"]
    y = w.forward(x, epilogue=bestla.EPI_RES_ADD, residual=torch.from_numpy(r).cuda()).cpu().numpy()
    assert _rel_err(y, ref + r) <= TOL["fp32"]
    y = w.forward(x, epilogue=bestla.EPI_SILU).cpu().numpy()
    assert _rel_err(y, ref / (1 + np.exp(-ref))) <= TOL["fp32"]


def test_mid_fused_qkv_ffn(oracle):
    """Fused QKV and the FFN (gate/up SiLU*mul, down) at a batched-decode M through the mid-M kernel."""
    m, k = 24, 1024
    blobs = [_blob(oracle, n, k, 128, S4, F16, False, 4, seed=40 + i) for i, n in enumerate((512, 256, 256))]
    ws = [bestla.DeviceWeight(b) for b in blobs]
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, k)).astype(np.float32)
    for y, b, n in zip(bestla.qkv_forward(torch.from_numpy(A).cuda(), *ws), blobs, (512, 256, 256)):
        assert _rel_err(y.cpu().numpy(), oracle.forward(A, b, n, k)) <= TOL["fp32"]
    fin, fmid, fout = 1024, 1536, 1024
    b1 = _blob(oracle, fmid, fin, 128, S4, F16, False, 4, seed=51)
    b3 = _blob(oracle, fmid, fin, 128, S4, F16, False, 4, seed=53)
    b2 = _blob(oracle, fout, fmid, 128, S4, F16, False, 4, seed=52)
    w1, w2, w3 = (bestla.DeviceWeight(b) for b in (b1, b2, b3))
    y = bestla.ffn_forward(torch.from_numpy(A).cuda(), w1, w2, w3, act="silu").cpu().numpy()
    h1 = oracle.forward(A, b1, fmid, fin).astype(np.float64)
    h3 = oracle.forward(A, b3, fmid, fin).astype(np.float64)
    ref = oracle.forward((h1 / (1 + np.exp(-h1)) * h3).astype(np.float32), b2, fout, fmid)
    assert _rel_err(y, ref) <= 2e-3  # the FFN's intermediates (fp16 at M > 16) dominate


def test_mid_graph_replay(oracle):
    """Captured and replayed (slabs in the workspace the first eager call sized): replays repeat the result."""
    m, n, k = 64, 2048, 4096
    blob = _blob(oracle, n, k, 128, S4, F16, False, 4, seed=3)
    w = bestla.DeviceWeight(blob)
    x = _x(m, k, "fp16", 4)
    out = torch.empty((m, n), device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        w.forward(x, out=out)  # the workspace sized outside the capture
        ref = out.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(3):
                w.forward(x, out=out)
        out.zero_()
        for _ in range(4):
            g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    y = ref.cpu().numpy()
    assert _rel_err(y, oracle.forward(x.float().cpu().numpy(), blob, n, k)) <= TOL["fp16"]


@pytest.mark.parametrize("m", [2, 5, 8, 13, 16])
def test_mid_small_m(oracle, knob, m):
    """Below the default threshold (NAD_MID_MIN_M=1): the one-fragment tile with zero rows, at the decode bar."""
    n, k = 1024, 4096
    blob = _blob(oracle, n, k, 128, S4, F16, False, 4, seed=m)
    w = bestla.DeviceWeight(blob)
    knob("NAD_MID_MIN_M", "1")
    assert w.plan(m, "fp32")["kernel"] == "woq_mid_kernel"
    x = _x(m, k, "fp32", m)
    y = w.forward(x).cpu().numpy()
    assert _rel_err(y, oracle.forward(x.cpu().numpy(), blob, n, k)) <= TOL["fp32"]


@pytest.mark.parametrize("m,n,mid", [(32, 4096, True), (64, 1000, True), (128, 4096, False), (65, 1000, False)])
def test_xcd_placement_is_speed_only(oracle, knob, m, n, mid):
    """The split-K runs of a stripe group (mid-M, NAD_MID_XCD) or of a gemm7 tile (NAD_GEMM_XCD) and the reduce
    workgroups that sum them placed on one XCD: which workgroup computes which run changes, the run order of the sums
    does not -- results bit-identical to the round-5 placement, ragged N included."""
    k = 4096
    blob = _blob(oracle, n, k, 128, S4, F16, False, 4, seed=m + n)
    w = bestla.DeviceWeight(blob)
    plan = w.plan(m, "fp16")
    assert plan["kernel"] == ("woq_mid_kernel" if mid else "woq_gemm7_kernel") and plan["ksplit"] > 1, plan
    x = _x(m, k, "fp16", m)
    y = w.forward(x).cpu().numpy()
    knob("NAD_MID_XCD", "0")
    knob("NAD_GEMM_XCD", "0")
    y0 = w.forward(x).cpu().numpy()
    assert np.array_equal(y, y0)
    assert _rel_err(y, oracle.forward(x.float().cpu().numpy(), blob, n, k)) <= (2e-5 if mid else 5e-4)
