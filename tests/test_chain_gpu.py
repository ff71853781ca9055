"""The persistent decode chain (woq_chain.hip, nad_chain_*): a sequence of decode GEMV ops in one launch.

Parity bar: every op of the chain runs the same tiles, dequant, MFMA and reduction order as the single-op stripe
stream (woq_gemv.hip), so chain outputs must be BIT-identical to the same ops launched one by one; the single-op path
itself is pinned against the oracle by test_gpu_parity.py.  The RMSNorm staging option is checked against a torch
fp32 reference of the same formula (x / sqrt(mean(x^2) + eps) * g) within 1e-5 relative.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _four_tile_slices(monkeypatch):
    # the chain streams 4-tile K-slices; the per-op M = 1 launch takes 2-tile slices at K <= 16 tiles (a different
    # summation order), so the bit-identity reference runs the per-op launches with 4-tile slices
    monkeypatch.setenv("NAD_GEMV_KS", "4")

from neural_amd import bestla  # noqa: E402
from neural_amd.bestla import CHAIN_GATE_UP, CHAIN_LINEAR, CHAIN_QKV, EPI_RES_ADD  # noqa: E402


def _w(n, k, seed, asym=False, stype="fp16", bs=128):
    return bestla.DeviceWeight.synthetic(4, n, k, bs, stype, asym, seed=seed)


def _layer_weights(hid, ffn, seed, asym=False):
    return dict(wq=_w(hid, hid, seed + 1, asym), wk=_w(hid, hid, seed + 2, asym), wv=_w(hid, hid, seed + 3, asym),
                wo=_w(hid, hid, seed + 4, asym), w1=_w(ffn, hid, seed + 5, asym), w3=_w(ffn, hid, seed + 6, asym),
                w2=_w(hid, ffn, seed + 7, asym))


def _build(layers, hid, ffn, m, vocab_w, norm, scale=1.0):
    dev = "cuda"
    f = dict(dtype=torch.float32, device=dev)
    xs = [torch.empty((m, hid), **f) for _ in range(2)]
    g = torch.Generator(device="cpu").manual_seed(5)
    xs[0].copy_((torch.rand((m, hid), generator=g) - 0.5) * scale)
    q, k, v = (torch.empty((m, hid), **f) for _ in range(3))
    h = torch.empty((m, hid), **f)
    t = torch.empty((m, ffn), **f)
    logits = torch.empty((m, vocab_w.n), **f)
    ops = []
    for li, L in enumerate(layers):
        x, xn = xs[li % 2], xs[(li + 1) % 2]
        ops.append(dict(kind=CHAIN_QKV, w=[L["wq"], L["wk"], L["wv"]], act=x, out=[q, k, v], norm=norm))
        ops.append(dict(kind=CHAIN_LINEAR, w=[L["wo"]], act=v, out=[h], epi=EPI_RES_ADD, res=x))
        ops.append(dict(kind=CHAIN_GATE_UP, w=[L["w1"], L["w3"]], act=h, out=[t], norm=norm))
        ops.append(dict(kind=CHAIN_LINEAR, w=[L["w2"]], act=t, out=[xn], epi=EPI_RES_ADD, res=h))
    ops.append(dict(kind=CHAIN_LINEAR, w=[vocab_w], act=xs[len(layers) % 2], out=[logits], norm=norm))
    return ops, xs, (q, k, v, h, t, logits)


def _per_op(ops):
    """The same ops, one launch each (the single-op stripe stream)."""
    for o in ops:
        if o["kind"] == CHAIN_QKV:
            q, k, v = bestla.qkv_forward(o["act"], *o["w"])
            for dst, src in zip(o["out"], (q, k, v)):
                dst.copy_(src)
        elif o["kind"] == CHAIN_GATE_UP:
            w1, w3 = o["w"]
            tmp1 = torch.empty_like(o["out"][0])
            rc = bestla.lib().nad_device_ffn_gate_up(o["act"].data_ptr(), 0, w1.desc, w3.desc, tmp1.data_ptr(),
                                                      o["out"][0].data_ptr(), o["act"].shape[0], w1.k, w1.n,
                                                      o["act"].stride(0), bestla.EPI_SILU_MUL,
                                                      torch.cuda.current_stream().cuda_stream)
            assert rc == 0, bestla.last_error()
        else:
            o["w"][0].forward(o["act"], out=o["out"][0], epilogue=o.get("epi", 0), residual=o.get("res"))


@pytest.mark.parametrize("m", [1, 2])
@pytest.mark.parametrize("asym", [False, True])
def test_chain_bit_identical_to_per_op(m, asym):
    hid, ffn = 1024, 2816  # ffn: 22 K tiles -> 6 slices over 6 waves, as Llama's 86 -> 22 over 11
    layers = [_layer_weights(hid, ffn, 100 * i, asym) for i in range(2)]
    lm = _w(1000, hid, 999, asym)
    # small input: without norms the random stack grows ~6x per matmul and must stay inside fp16 staging range
    ops, xs, bufs = _build(layers, hid, ffn, m, lm, norm=False, scale=0.01)
    x0 = xs[0].clone()
    chain = bestla.Chain(ops, m)
    chain.run()
    torch.cuda.synchronize()
    assert chain.status() == 0
    got = [b.clone() for b in bufs] + [x.clone() for x in xs]
    xs[0].copy_(x0)
    _per_op(ops)
    torch.cuda.synchronize()
    ref = list(bufs) + list(xs)
    for a, b in zip(got, ref):
        assert torch.isfinite(b).all()
        assert torch.equal(a, b), (a - b).abs().max().item()


def test_chain_llama_shapes_and_replay():
    """One Llama-2-7B layer + lm_head: bit-identical to per-op launches, repeatable, graph-capturable."""
    hid, ffn = 4096, 11008
    layers = [_layer_weights(hid, ffn, 7)]
    lm = _w(32000, hid, 77)
    ops, xs, bufs = _build(layers, hid, ffn, 1, lm, norm=False)
    x0 = xs[0].clone()
    chain = bestla.Chain(ops, 1)
    chain.run()
    torch.cuda.synchronize()
    got = [b.clone() for b in bufs]
    xs[0].copy_(x0)
    _per_op(ops)
    torch.cuda.synchronize()
    for a, b in zip(got, bufs):
        assert torch.equal(a, b)
    # graph replay of the single launch reproduces the first run exactly
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        xs[0].copy_(x0)
        with torch.cuda.graph(g, stream=s):
            chain.run(stream=s)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        xs[0].copy_(x0)
        g.replay()
        torch.cuda.synchronize()
        for a, b in zip(got, bufs):
            assert torch.equal(a, b)
    assert chain.status() == 0


def test_chain_rmsnorm_staging():
    hid, ffn = 2048, 1024
    w = _w(512, hid, 3)
    m = 2
    x = (torch.rand((m, hid), device="cuda") - 0.5) * 3
    gw = torch.rand(hid, device="cuda") + 0.5
    out = torch.empty((m, 512), device="cuda")
    chain = bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w], act=x, out=[out], norm=True, norm_eps=1e-5, norm_w=gw)], m)
    chain.run()
    xn = x / torch.sqrt((x.double() ** 2).mean(dim=1, keepdim=True) + 1e-5).float() * gw
    ref = w.forward(xn)
    torch.cuda.synchronize()
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    assert err <= 1e-5, err


def test_chain_rejects_ineligible():
    w8 = bestla.DeviceWeight.synthetic(8, 128, 256, 64, "fp16", False, seed=1)
    x = torch.zeros((1, 256), device="cuda")
    out = torch.empty((1, 128), device="cuda")
    with pytest.raises(RuntimeError, match="nad_chain_create"):
        bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w8], act=x, out=[out])], 1)
