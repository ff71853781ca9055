"""Batched independent decode problems (nad_batch_*: BTLAGemmBatchDriver, bestla_gemm.cpp:508-624, for device
tensors): n M = 1 problems of one weight shape in ONE woq_gemv_m1_kernel launch, workgroups dealt out problem by
problem.

Parity bars:
  * against the oracle (fp64 GEMM on the reference's dequantized weights): 2e-5 of max|ref| per problem, the decode bar;
  * against a one-problem launch of the same weight: BIT-identical -- a stripe is reduced by the same waves, K-slices
    and wave order whichever workgroup (and however many stripes per workgroup) serves it.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from neural_amd import bestla  # noqa: E402
from tests.oracle_lib import BF16, F16, F32, S2, S4  # noqa: E402
from tests.test_gpu_parity import _blob, _rel_err  # noqa: E402

TOL_DECODE = 2e-5

CASES = [
    # problems, n, k, bs, qtype, stype, asym
    (5, 300, 1024, 128, S4, F16, False),    # ragged N (19 stripes), workgroups per problem > stripes per problem
    (3, 1024, 4096, 128, S4, BF16, True),   # asym, bf16 scales
    (4, 512, 2048, 64, S2, F16, False),     # int2 g64 (Mistral's format)
    (2, 256, 4096, 4096, S4, F32, False),   # per-channel scales
    (300, 64, 256, 128, S4, F16, False),    # more problems than CUs: one workgroup each
]


@pytest.mark.parametrize("cfg", CASES)
def test_batch_matches_oracle_and_single_launches(oracle, cfg):
    nprob, n, k, bs, qt, st, asym = cfg
    rng = np.random.default_rng(nprob * 7 + n)
    blobs = [_blob(oracle, n, k, bs, qt, st, asym, 4, seed=1000 * i + k) for i in range(min(nprob, 6))]
    ws = [bestla.DeviceWeight(b) for b in blobs]
    xs = [torch.from_numpy(rng.uniform(-0.5, 0.5, size=(1, k)).astype(np.float32)).cuda() for _ in range(nprob)]
    ys = [torch.full((1, n), float("nan"), device="cuda") for _ in range(nprob)]
    b = bestla.Batch([(ws[i % len(ws)], xs[i], ys[i]) for i in range(nprob)])
    b.run()
    torch.cuda.synchronize()
    for i in range(nprob):
        w = ws[i % len(ws)]
        single = w.forward(xs[i]).cpu().numpy()
        got = ys[i].cpu().numpy()
        assert np.array_equal(got, single), (i, float(np.abs(got - single).max()))
        if i < 6:
            ref = oracle.forward(xs[i].cpu().numpy(), blobs[i % len(blobs)], n, k)
            assert _rel_err(got, ref) <= TOL_DECODE


def test_batch_graph_replay_and_llama_shape(oracle):
    """K = N = 4096 int4 g128 (BASELINE config 2) x 64 problems, captured in a HIP graph and replayed: every problem
    equals its one-problem launch bit for bit, replay after replay."""
    n = k = 4096
    ws = [bestla.DeviceWeight.synthetic(4, n, k, 128, "fp16", False, seed=40 + i) for i in range(8)]
    g = torch.Generator(device="cpu").manual_seed(3)
    xs = [(torch.rand((1, k), generator=g) - 0.5).cuda() for _ in range(64)]
    ys = [torch.empty((1, n), device="cuda") for _ in range(64)]
    b = bestla.Batch([(ws[i % 8], xs[i], ys[i]) for i in range(64)])
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        b.run(stream=s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            b.run(stream=s)
    torch.cuda.current_stream().wait_stream(s)
    singles = [ws[i % 8].forward(xs[i]).cpu().numpy() for i in range(64)]
    for _ in range(2):
        for y in ys:
            y.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        for i in range(64):
            assert np.array_equal(ys[i].cpu().numpy(), singles[i]), i


def test_batch_rejects_mixed_shapes():
    a = bestla.DeviceWeight.synthetic(4, 256, 1024, 128, "fp16", False, seed=1)
    c = bestla.DeviceWeight.synthetic(4, 512, 1024, 128, "fp16", False, seed=2)
    x = torch.zeros((1, 1024), device="cuda")
    y1, y2 = torch.empty((1, 256), device="cuda"), torch.empty((1, 512), device="cuda")
    with pytest.raises(RuntimeError, match="differs in shape or format"):
        bestla.Batch([(a, x, y1), (c, x, y2)])


@pytest.mark.parametrize("bs", [64, 128])
def test_qkv_two_formats_one_launch(oracle, knob, bs):
    """The int2 policy's decode QKV (llama_utils.cpp:269-287: int2 Q, K and an int4 V of one group size; Mistral-7B
    shapes, 8 KV heads) as ONE launch of two formats (woq_gemv_m1_dual_kernel, NAD_GEMV_DUAL=1): bit-identical to the
    two launches it replaces (NAD_GEMV_DUAL=0), and within the decode bar of the oracle."""
    k = 4096
    shapes = [(4096, S2), (1024, S2), (1024, S4)]
    blobs = [_blob(oracle, n, k, bs, qt, F16, False, 4, seed=77 + n + i) for i, (n, qt) in enumerate(shapes)]
    ws = [bestla.DeviceWeight(b) for b in blobs]
    x = torch.from_numpy(np.random.default_rng(5).uniform(-0.5, 0.5, size=(1, k)).astype(np.float32)).cuda()
    outs = {}
    for dual in ("1", "0"):
        knob("NAD_GEMV_DUAL", dual)
        o = [torch.full((1, n), float("nan"), device="cuda") for n, _ in shapes]
        bestla.qkv_forward(x, ws[0], ws[1], ws[2], out=tuple(o))
        torch.cuda.synchronize()
        outs[dual] = [t.cpu().numpy() for t in o]
    for a, b in zip(outs["1"], outs["0"]):
        assert np.array_equal(a, b)
    for i, (n, _) in enumerate(shapes):
        ref = oracle.forward(x.cpu().numpy(), blobs[i], n, k)
        assert _rel_err(outs["1"][i], ref) <= TOL_DECODE
