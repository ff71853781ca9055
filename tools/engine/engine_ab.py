"""A/B of decode-engine knobs read at nad_chain_create (environment variables): the bench's Llama-2-7B int4-g128 token
as cut launches (33 per token) and as one launch, graph-replayed, HIP events on the replay stream.
Usage: python tools/engine_ab.py VAR=v1,v2,... [VAR2=...]   (every combination; first value of each = baseline)
       ENGINE_AB_CFG=mistral for the Mistral int2 policy geometry (engine takes one format per launch: skipped then)"""
import itertools
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from neural_amd import _lib  # noqa: E402

specs = []
for a in sys.argv[1:]:
    k, v = a.split("=", 1)
    specs.append((k, v.split(",")))
stack = bench.Stack(bench.LLAMA, 0, 1)
per_op = bench.Runner(stack, 1, None, "cuda")
t_op = bench.graph_time(lambda s: per_op.step(), 20, torch)
print(json.dumps({"per_op_tok_s": round(1 / t_op, 1)}), flush=True)


def indep_time():
    """the token's matmuls as ONE launch with no data dependencies (every op reads an external vector): the engine's
    pure weight-stream rate, no hand-offs"""
    from neural_amd import bestla
    H, L = stack.cfg["hidden"], len(stack.layers)
    f = dict(dtype=torch.float32, device="cuda")
    x = torch.rand((1, H), **f) - 0.5
    t = torch.rand((1, stack.nf), **f) - 0.5
    outs = [torch.empty((1, n), **f) for n in (stack.nq, stack.nkv, stack.nkv, H, stack.nf, H, stack.nv)]
    ops = []
    for Lw in stack.layers:
        ops.append(dict(kind=bestla.CHAIN_QKV, w=[Lw["wq"], Lw["wk"], Lw["wv"]], act=x, out=outs[0:3]))
        ops.append(dict(kind=bestla.CHAIN_LINEAR, w=[Lw["wo"]], act=x, out=[outs[3]]))
        ops.append(dict(kind=bestla.CHAIN_GATE_UP, w=[Lw["w1"], Lw["w3"]], act=x, out=[outs[4]]))
        ops.append(dict(kind=bestla.CHAIN_LINEAR, w=[Lw["w2"]], act=t, out=[outs[5]]))
    ops.append(dict(kind=bestla.CHAIN_LINEAR, w=[stack.lm_head], act=x, out=[outs[6]]))
    ch = bestla.Chain(ops, 1)
    tt = bench.graph_time(lambda s: ch.run(stream=s), 20, torch)
    assert ch.status() == 0
    return tt


combos = list(itertools.product(*[v for _, v in specs])) if specs else [()]
for rep in range(2):
    for combo in combos:
        for (k, _), v in zip(specs, combo):
            os.environ[k] = v
        _lib.reload_knobs()  # the library reads its switches once
        res = {}
        for cut in (True, False):
            cr = bench.ChainRunner(stack, "cuda", cut=cut)
            t = bench.graph_time(lambda s: cr.step(stream=s), 20, torch)
            assert cr.status() == 0, "engine give-up"
            res["cut" if cut else "whole"] = round(1 / t, 1)
            del cr
        if os.environ.get("ENGINE_AB_INDEP"):
            res["indep"] = round(1 / indep_time(), 1)
        print(json.dumps({"rep": rep, **{k: v for (k, _), v in zip(specs, combo)}, **res}), flush=True)
