"""The decode weight-stream engine (woq_chain.hip, nad_chain_*): M = 1 WOQ matmuls of a decode segment in one
persistent launch, weights streamed by an LDS-DMA loader wave, results handed between ops as tagged granules.

Parity bars:
  * every op of a launch computes exactly what a ONE-op launch of the same op computes (same tiles per consumer, same
    reduction order, same RMSNorm order): chain outputs are BIT-identical to the ops launched one by one, whether the
    launch is a whole token or cut at the attention nodes (the form the reference graph can dispatch);
  * against the oracle (fp64 GEMM on the reference's dequantized weights): 2e-5 of max|ref| per op (fp32 activations
    split into fp16 hi + lo, fp32 accumulation) -- the same bar as the single-op decode kernels;
  * against the per-op decode kernel (woq_gemv.hip): 1e-6 (only the order of the fp32 partial sums differs);
  * RMSNorm staging against a torch fp32 reference of x / sqrt(mean(x^2) + eps) * g: 1e-5.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from neural_amd import bestla  # noqa: E402
from neural_amd.bestla import CHAIN_GATE_UP, CHAIN_LINEAR, CHAIN_QKV, EPI_RES_ADD  # noqa: E402
from tests.oracle_lib import F16, S2, S4  # noqa: E402
from tests.test_gpu_parity import _rel_err  # noqa: E402


def _w(n, k, seed, asym=False, stype="fp16", bs=128, bits=4):
    return bestla.DeviceWeight.synthetic(bits, n, k, bs, stype, asym, seed=seed)


def _layer_weights(hid, ffn, seed, asym=False, bits=4, bs=128):
    mk = lambda n, k, s: _w(n, k, seed + s, asym, bs=bs, bits=bits)  # noqa: E731
    return dict(wq=mk(hid, hid, 1), wk=mk(hid, hid, 2), wv=mk(hid, hid, 3), wo=mk(hid, hid, 4), w1=mk(ffn, hid, 5),
                w3=mk(ffn, hid, 6), w2=mk(hid, ffn, 7))


class Stack:
    """Buffers + the op list of L decoder layers and the lm_head tail (llama.cpp op order):
    x -> RMSNorm -> QKV -> (attention: here V, exact for a single-token context) -> O + x -> RMSNorm -> gate/up
    SiLU*mul -> down + h -> next layer ... -> RMSNorm -> lm_head."""

    def __init__(self, layers, hid, ffn, lm, scale=1.0, norm_w=False):
        f = dict(dtype=torch.float32, device="cuda")
        g = torch.Generator(device="cpu").manual_seed(5)
        self.x0 = ((torch.rand((1, hid), generator=g) - 0.5) * scale).cuda()
        L = len(layers)
        self.xs = [torch.empty((1, hid), **f) for _ in range(L + 1)]
        self.q, self.k, self.v = ([torch.empty((1, hid), **f) for _ in range(L)] for _ in range(3))
        self.h = [torch.empty((1, hid), **f) for _ in range(L)]
        self.t = [torch.empty((1, ffn), **f) for _ in range(L)]
        self.logits = torch.empty((1, lm.n), **f)
        self.gw = [(torch.rand(hid, generator=g) + 0.5).cuda() if norm_w else None for _ in range(2 * L + 1)]
        self.layers, self.lm = layers, lm

    def ops(self):
        """(ops, boundaries): the whole token, and the indices where the reference graph cuts it (attention)."""
        ops, cuts = [], [1]
        for li, Lw in enumerate(self.layers):
            x = self.xs[li]
            ops.append(dict(kind=CHAIN_QKV, w=[Lw["wq"], Lw["wk"], Lw["wv"]], act=x,
                            out=[self.q[li], self.k[li], self.v[li]], norm=True, norm_w=self.gw[2 * li]))
            ops.append(dict(kind=CHAIN_LINEAR, w=[Lw["wo"]], act=self.v[li], out=[self.h[li]], epi=EPI_RES_ADD, res=x))
            ops.append(dict(kind=CHAIN_GATE_UP, w=[Lw["w1"], Lw["w3"]], act=self.h[li], out=[self.t[li]], norm=True,
                            norm_w=self.gw[2 * li + 1]))
            ops.append(dict(kind=CHAIN_LINEAR, w=[Lw["w2"]], act=self.t[li], out=[self.xs[li + 1]], epi=EPI_RES_ADD,
                            res=self.h[li]))
            cuts.append(len(ops) + 1)   # next cut: after the next layer's QKV
        ops.append(dict(kind=CHAIN_LINEAR, w=[self.lm], act=self.xs[-1], out=[self.logits], norm=True,
                        norm_w=self.gw[-1]))
        cuts[-1] = len(ops)
        return ops, cuts

    def results(self):
        return [t.clone() for t in self.xs + self.q + self.k + self.v + self.h + self.t + [self.logits]]

    def reset(self):
        for t in self.xs + self.q + self.k + self.v + self.h + self.t + [self.logits]:
            t.fill_(float("nan"))
        self.xs[0].copy_(self.x0)


def _run_chains(chains):
    for c in chains:
        c.run()
    torch.cuda.synchronize()
    for c in chains:
        assert c.status() == 0


def _same(a, b):
    assert len(a) == len(b)
    bad = [(i, (x - y).abs().max().item()) for i, (x, y) in enumerate(zip(a, b)) if not torch.equal(x, y)]
    for i, y in enumerate(b):
        assert torch.isfinite(y).all(), i
    assert not bad, bad


@pytest.mark.parametrize("asym", [False, True])
def test_chain_bit_identical_to_one_op_launches_and_cut_segments(asym):
    hid, ffn = 1024, 2816   # ffn: 22 K tiles -> two fills per stripe, the second ragged
    st = Stack([_layer_weights(hid, ffn, 100 * i, asym) for i in range(2)], hid, ffn, _w(1000, hid, 999, asym),
               norm_w=True)
    ops, cuts = st.ops()
    st.reset()
    _run_chains([bestla.Chain(ops, 1)])                         # the whole token: one launch
    whole = st.results()
    st.reset()
    _run_chains([bestla.Chain([o], 1) for o in ops])            # one launch per op
    _same(whole, st.results())
    st.reset()
    bounds = [0] + cuts
    _run_chains([bestla.Chain(ops[a:b], 1) for a, b in zip(bounds, bounds[1:])])   # cut at attention
    _same(whole, st.results())


def _per_op_kernels(st):
    """the same math through the per-op decode kernels (woq_gemv.hip) + torch for RMSNorm (fp32)"""
    def norm(x, g):
        y = x / torch.sqrt((x * x).mean(dim=1, keepdim=True) + 1e-5)
        return y * g if g is not None else y
    outs = {}
    for li, Lw in enumerate(st.layers):
        x = st.xs[li]
        q, k, v = bestla.qkv_forward(norm(x, st.gw[2 * li]), Lw["wq"], Lw["wk"], Lw["wv"])
        h = Lw["wo"].forward(st.v[li], epilogue=EPI_RES_ADD, residual=x)
        t = bestla.ffn_gate_up(norm(st.h[li], st.gw[2 * li + 1]), Lw["w1"], Lw["w3"])
        xn = Lw["w2"].forward(st.t[li], epilogue=EPI_RES_ADD, residual=st.h[li])
        outs[li] = (q, k, v, h, t, xn)
    logits = st.lm.forward(norm(st.xs[-1], st.gw[-1]))
    return outs, logits


def test_chain_matches_per_op_kernels():
    hid, ffn = 2048, 5632
    st = Stack([_layer_weights(hid, ffn, 7)], hid, ffn, _w(4000, hid, 77), norm_w=True)
    ops, _ = st.ops()
    st.reset()
    _run_chains([bestla.Chain(ops, 1)])
    outs, logits = _per_op_kernels(st)   # each op fed the chain's own inputs
    q, k, v, h, t, xn = outs[0]
    for got, ref in ((st.q[0], q), (st.k[0], k), (st.v[0], v), (st.h[0], h), (st.t[0], t), (st.xs[1], xn),
                     (st.logits, logits)):
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        assert err <= 1e-6, err


def test_chain_matches_oracle(oracle):
    """Weights packed by the oracle (the reference's blob format), each op of a launch against the oracle's fp64
    forward on that op's actual input: 2e-5."""
    hid, ffn = 1024, 2816
    rng = np.random.default_rng(3)

    def blob(n, k):
        q = rng.integers(-8, 8, size=(k, n), dtype=np.int8)
        s = rng.uniform(0.001, 0.005, size=(k // 128, n)).astype(np.float32)
        return oracle.pack_q(q, s, None, n, k, 128, S4, F16, False, oracle.lib.orc_select_core(4, S4, 128, 0, 0))
    names = [("wq", hid, hid), ("wk", hid, hid), ("wv", hid, hid), ("wo", hid, hid), ("w1", ffn, hid),
             ("w3", ffn, hid), ("w2", hid, ffn)]
    blobs = {nm: (blob(n, k), n, k) for nm, n, k in names}
    layer = {nm: bestla.DeviceWeight(b[0]) for nm, b in blobs.items()}
    lmb = blob(512, hid)
    st = Stack([layer], hid, ffn, bestla.DeviceWeight(lmb))
    ops, _ = st.ops()
    st.reset()
    _run_chains([bestla.Chain(ops, 1)])

    def rms(x):
        x = x.astype(np.float64)
        return (x / np.sqrt((x * x).mean() + 1e-5)).astype(np.float32)
    f = lambda nm, a: oracle.forward(a, blobs[nm][0], blobs[nm][1], blobs[nm][2])  # noqa: E731
    x0 = st.xs[0].cpu().numpy()
    xn = rms(x0)
    for got, nm in ((st.q[0], "wq"), (st.k[0], "wk"), (st.v[0], "wv")):
        assert _rel_err(got.cpu().numpy(), f(nm, xn)) <= 2e-5, nm
    h_ref = f("wo", st.v[0].cpu().numpy()) + x0
    assert _rel_err(st.h[0].cpu().numpy(), h_ref) <= 2e-5
    hn = rms(st.h[0].cpu().numpy())
    g, u = f("w1", hn).astype(np.float64), f("w3", hn).astype(np.float64)
    assert _rel_err(st.t[0].cpu().numpy(), g / (1 + np.exp(-g)) * u) <= 1e-4
    x1_ref = f("w2", st.t[0].cpu().numpy()) + st.h[0].cpu().numpy()
    assert _rel_err(st.xs[1].cpu().numpy(), x1_ref) <= 2e-5
    lg = oracle.forward(rms(st.xs[1].cpu().numpy()), lmb, 512, hid)
    assert _rel_err(st.logits.cpu().numpy(), lg) <= 2e-5


def test_chain_llama_shapes_graph_replay():
    """One Llama-2-7B layer + lm_head as the bench's cut launches ([QKV] [O, gate/up, down, lm_head]): bit-identical to
    the whole-token launch, and every graph replay reproduces it exactly (the launch generation moves on, stale
    granules of the previous replay never match)."""
    hid, ffn = 4096, 11008
    st = Stack([_layer_weights(hid, ffn, 7)], hid, ffn, _w(32000, hid, 77))
    ops, cuts = st.ops()
    st.reset()
    _run_chains([bestla.Chain(ops, 1)])
    whole = st.results()
    bounds = [0] + cuts
    chains = [bestla.Chain(ops[a:b], 1) for a, b in zip(bounds, bounds[1:])]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        st.reset()
        with torch.cuda.graph(g, stream=s):
            for c in chains:
                c.run(stream=s)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        st.reset()
        g.replay()
        torch.cuda.synchronize()
        _same(whole, st.results())
    for c in chains:
        assert c.status() == 0


def test_chain_rmsnorm_staging():
    hid = 2048
    w = _w(512, hid, 3)
    x = (torch.rand((1, hid), device="cuda") - 0.5) * 3
    gw = torch.rand(hid, device="cuda") + 0.5
    out = torch.empty((1, 512), device="cuda")
    chain = bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w], act=x, out=[out], norm=True, norm_eps=1e-5, norm_w=gw)], 1)
    chain.run()
    xn = x / torch.sqrt((x.double() ** 2).mean(dim=1, keepdim=True) + 1e-5).float() * gw
    ref = w.forward(xn)
    torch.cuda.synchronize()
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    assert err <= 1e-5, err


def test_chain_int2_stack():
    """int2 weights (KT = 256, two groups of 64 per... one group of 128 per tile here) through the same engine."""
    hid, ffn = 1024, 2048
    st = Stack([_layer_weights(hid, ffn, 11, bits=2, bs=128)], hid, ffn, _w(1024, hid, 12, bits=2), norm_w=True)
    ops, _ = st.ops()
    st.reset()
    _run_chains([bestla.Chain(ops, 1)])
    whole = st.results()
    st.reset()
    _run_chains([bestla.Chain([o], 1) for o in ops])
    _same(whole, st.results())
    outs, logits = _per_op_kernels(st)
    err = ((st.logits - logits).abs().max() / logits.abs().max()).item()
    assert err <= 1e-6, err


def test_chain_rejects_ineligible():
    w8 = bestla.DeviceWeight.synthetic(8, 128, 256, 64, "fp16", False, seed=1)
    x = torch.zeros((1, 256), device="cuda")
    out = torch.empty((1, 128), device="cuda")
    with pytest.raises(RuntimeError, match="nad_chain_create"):
        bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w8], act=x, out=[out])], 1)
    w4 = _w(128, 256, 2)
    with pytest.raises(RuntimeError, match="m = 1"):
        bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w4], act=torch.zeros((2, 256), device="cuda"),
                           out=[torch.empty((2, 128), device="cuda")])], 2)


def test_chain_rejects_write_after_read_hazards():
    """the engine orders only the hand-offs that go through granules, so nad_chain_create refuses
    an op whose result or aux overwrites a vector an op of the chain reads from outside it (its own input included),
    and any read of an earlier op's aux (aux has no in-launch hand-off)."""
    w = _w(256, 256, 3)
    wd = _w(256, 256, 4)
    x = torch.rand((1, 256), device="cuda")
    y = torch.empty((1, 256), device="cuda")
    z = torch.empty((1, 256), device="cuda")
    # op 1 writes op 0's external input
    with pytest.raises(RuntimeError, match="write-after-read"):
        bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w], act=x, out=[y]),
                      dict(kind=CHAIN_LINEAR, w=[wd], act=y, out=[x])], 1)
    # an op writes its own input
    with pytest.raises(RuntimeError, match="write-after-read"):
        bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w], act=x, out=[x])], 1)
    # op 1's external residual overwritten by op 2
    with pytest.raises(RuntimeError, match="write-after-read"):
        bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w], act=x, out=[y]),
                      dict(kind=CHAIN_LINEAR, w=[wd], act=y, out=[z], epi=EPI_RES_ADD, res=x),
                      dict(kind=CHAIN_LINEAR, w=[w], act=z, out=[x])], 1)
    # reading an earlier op's aux
    g1, g3 = _w(256, 256, 5), _w(256, 256, 6)
    aux = torch.empty((1, 256), device="cuda")
    t = torch.empty((1, 256), device="cuda")
    with pytest.raises(RuntimeError, match="aux"):
        bestla.Chain([dict(kind=CHAIN_GATE_UP, w=[g1, g3], act=x, out=[t], aux=aux),
                      dict(kind=CHAIN_LINEAR, w=[wd], act=aux, out=[y])], 1)
    # the legal form of the same chain still builds
    bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w], act=x, out=[y]),
                  dict(kind=CHAIN_LINEAR, w=[wd], act=y, out=[z], epi=EPI_RES_ADD, res=x)], 1)


def test_chain_mixed_formats_mistral_policy():
    """Two weight formats in one launch (Mistral-7B's int2 policy: q, k, o, gate, up, lm_head int2 g64; wv, w2 int4 g64;
    GQA so {Q, K} is one op and V its own): bit-identical across launch forms (whole token, cut at attention, one op
    per launch), every op within 1e-6 of the per-op kernels fed the chain's own inputs, and the oracle bar on the
    format boundary (int4 V and down) through those kernels' own oracle tests."""
    import bench
    cfg = dict(bench.MISTRAL, hidden=1024, ffn=2048, layers=2, vocab=1000, kv=256)
    st = bench.Stack(cfg, 0, 1, seed=17)
    forms = {}
    for name, cut in (("whole", False), ("cut", True)):
        cr = bench.ChainRunner(st, "cuda", cut=cut)
        for c in cr.chains:
            c.run()
        torch.cuda.synchronize()
        assert cr.status() == 0
        forms[name] = [t.clone() for t in cr.xs + cr.q + cr.k + cr.v + cr.h + cr.t + [cr.logits]]
        if name == "whole":
            keep = cr
    _same(forms["whole"], forms["cut"])
    cr = keep
    assert all(torch.isfinite(t).all() for t in forms["whole"])

    def norm(x):
        return x / torch.sqrt((x * x).mean(dim=1, keepdim=True) + 1e-5)
    for li, Lw in enumerate(st.layers):
        x = cr.xs[li]
        xn = norm(x)
        refs = [(cr.q[li], Lw["wq"].forward(xn)), (cr.k[li], Lw["wk"].forward(xn)), (cr.v[li], Lw["wv"].forward(xn)),
                (cr.h[li], Lw["wo"].forward(cr.o_in[li], epilogue=EPI_RES_ADD, residual=x)),
                (cr.t[li], bestla.ffn_gate_up(norm(cr.h[li]), Lw["w1"], Lw["w3"])),
                (cr.xs[li + 1], Lw["w2"].forward(cr.t[li], epilogue=EPI_RES_ADD, residual=cr.h[li]))]
        for i, (got, ref) in enumerate(refs):
            err = ((got - ref).abs().max() / ref.abs().max()).item()
            assert err <= 1e-6, (li, i, err)
    lg = st.lm_head.forward(norm(cr.xs[-1]))
    assert ((cr.logits - lg).abs().max() / lg.abs().max()).item() <= 1e-6


def test_chain_mixed_launch_may_start_with_either_format(oracle):
    """A mixed launch whose first op is the int4 member (format roles swapped at creation): each op against the oracle."""
    rng = np.random.default_rng(21)

    def blob(n, k, bits):
        lo, hi = (-8, 8) if bits == 4 else (-2, 2)
        q = rng.integers(lo, hi, size=(k, n), dtype=np.int8)
        s = rng.uniform(0.001, 0.005, size=(k // 64, n)).astype(np.float32)
        qt = S4 if bits == 4 else S2
        return oracle.pack_q(q, s, None, n, k, 64, qt, F16, False, oracle.lib.orc_select_core(4, qt, 64, 0, 0))
    k, n = 512, 256
    b4, b2 = blob(n, k, 4), blob(n, k, 2)
    w4, w2 = bestla.DeviceWeight(b4), bestla.DeviceWeight(b2)
    x = (torch.rand((1, k), device="cuda") - 0.5)
    y4, y2 = torch.empty((1, n), device="cuda"), torch.empty((1, n), device="cuda")
    ch = bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w4], act=x, out=[y4]), dict(kind=CHAIN_LINEAR, w=[w2], act=x, out=[y2])], 1)
    ch.run()
    torch.cuda.synchronize()
    assert ch.status() == 0
    xa = x.cpu().numpy()
    assert _rel_err(y4.cpu().numpy(), oracle.forward(xa, b4, n, k)) <= 2e-5
    assert _rel_err(y2.cpu().numpy(), oracle.forward(xa, b2, n, k)) <= 2e-5


def test_chain_rejects_format_pairs_it_has_no_kernel_for():
    """int4 g128 beside int2 g64 in one launch has no instantiation: refused at creation with the formats named."""
    x = torch.zeros((1, 512), device="cuda")
    a, b = torch.empty((1, 128), device="cuda"), torch.empty((1, 128), device="cuda")
    w4 = _w(128, 512, 1, bs=128, bits=4)
    w2 = _w(128, 512, 2, bs=64, bits=2)
    with pytest.raises(RuntimeError, match="cannot join"):
        bestla.Chain([dict(kind=CHAIN_LINEAR, w=[w4], act=x, out=[a]), dict(kind=CHAIN_LINEAR, w=[w2], act=x, out=[b])],
                     1)
