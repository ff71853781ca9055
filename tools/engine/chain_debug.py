"""Bisect a whole-launch vs one-op-launch mismatch of the decode engine (development tool)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from neural_amd import bestla  # noqa: E402
from tests.test_chain_gpu import Stack, _layer_weights, _w  # noqa: E402

hid, ffn = 1024, 2816
for norm_w in (True, False):
    for nl in (1, 2):
        st = Stack([_layer_weights(hid, ffn, 100 * i) for i in range(nl)], hid, ffn, _w(1000, hid, 999), norm_w=norm_w)
        ops, cuts = st.ops()
        for variant in ("asis", "nonorm"):
            if variant == "nonorm":
                for o in ops:
                    o["norm"] = False
            st.reset()
            c = bestla.Chain(ops, 1)
            c.run()
            torch.cuda.synchronize()
            whole = st.results()
            st.reset()
            cs = [bestla.Chain([o], 1) for o in ops]
            for x in cs:
                x.run()
            torch.cuda.synchronize()
            one = st.results()
            names = ([f"x{i}" for i in range(nl + 1)] + [f"q{i}" for i in range(nl)] + [f"k{i}" for i in range(nl)] +
                     [f"v{i}" for i in range(nl)] + [f"h{i}" for i in range(nl)] + [f"t{i}" for i in range(nl)] + ["lg"])
            bad = [(nm, f"{(a - b).abs().max().item():.2e}") for nm, a, b in zip(names, whole, one)
                   if not torch.equal(a, b)]
            print(f"norm_w={norm_w} layers={nl} {variant}: status {c.status()} mismatches {bad}", flush=True)
