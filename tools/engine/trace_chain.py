"""Phase trace of the decode weight-stream engine (development tool; needs `make -C neural_amd chaintrace`).

Runs the bench's Llama-2-7B stack as the cut launches (default) or the whole token as one launch (arg "whole"), then
prints per op kind the medians over workgroups of: gather (op start -> input read), stage (-> hi/lo rows staged),
first fill (-> first weight fill ready), loop (stream), publish (reduce + granules), the consumer's FULL-wait and the
loader's FREE-wait inside the op, and the op's span (first start -> last publish over workgroups).
Usage: python tools/trace_chain.py [cut|whole] [layers]"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["NAD_LIB_PATH"] = os.environ.get("NAD_LIB_PATH") or os.path.join(REPO, "neural_amd", "libneural_amd_chaintrace.so")
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from neural_amd import _lib  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "cut"
layers = int(sys.argv[2]) if len(sys.argv) > 2 else 32
cfg = dict(bench.LLAMA, layers=layers)
stack = bench.Stack(cfg, 0, 1)
cr = bench.ChainRunner(stack, "cuda", cut=(mode == "cut"))
L = _lib.lib()
L.nad_chain_trace_fetch.argtypes = [C.c_void_p, C.c_size_t]
tick = 1e-2  # wall_clock64: 100 MHz -> us
names = ["qkv", "o", "gate_up", "down"]
if mode == "cut":
    # one launch at a time (the trace buffer holds one launch): trace each segment kind once, warm
    rows = {}
    for ci, ch in enumerate(cr.chains[:3] + cr.chains[-1:]):
        for _ in range(3):
            ch.run()
        torch.cuda.synchronize()
        buf = np.zeros((22, 160, 256), np.uint64)
        ch.run()
        assert L.nad_chain_trace_fetch(buf.ctypes.data, buf.nbytes) == 0
        nops = ch.n_ops if hasattr(ch, "n_ops") else len(ch._ops)
        b = buf.astype(np.int64)
        t0 = b[0, 0].min()
        span = (b[5, nops - 1].max() - t0) * tick
        kinds = ["qkv"] if nops == 1 else ["o", "gate_up", "down", "qkv" if ci < 3 else "lm_head"]
        print(f"launch {ci}: {nops} ops, span {span:.2f} us (first op start -> last publish)")
        for op in range(nops):
            x = b[:, op]
            g1 = x[11] - x[0]
            d = dict(gather=np.median(x[1] - x[0]) * tick,
                     pass1=(np.median(g1[x[11] > 0]) * tick if (x[11] > 0).any() else 0.0),
                     stage=np.median(x[2] - x[1]) * tick,
                     first=np.median(x[3] - x[2]) * tick, loop=np.median(x[4] - x[3]) * tick,
                     publish=np.median(x[5] - x[4]) * tick, pbar=np.median(x[10] - x[4]) * tick,
                     fullwait=np.median(x[9]) * tick,
                     freewait=np.median(x[8]) * tick, start=(x[0].min() - t0) * tick,
                     end=(x[5].max() - t0) * tick, endskew=(x[5].max() - x[5].min()) * tick)
            if op > 0:  # hand-off: the previous op's LAST publish (any CU) -> this CU's input gathered
                ho = (x[1] - b[5, op - 1].max()) * tick
                d["handoff_med"], d["handoff_max"] = np.median(ho), ho.max()
            lag = [np.median(x[12 + c] - x[12]) * tick for c in range(8)]
            print("  " + kinds[op].ljust(8) + " ".join(f"{k} {v:6.2f}" for k, v in d.items()), flush=True)
            print("           loop end vs consumer 0: " + " ".join(f"{v:5.2f}" for v in lag) +
                  f"   stores done after publish: {np.median(x[20] - x[5]) * tick:5.2f}", flush=True)
else:
    ch = cr.chains[0]
    for _ in range(3):
        ch.run()
    torch.cuda.synchronize()
    buf = np.zeros((22, 160, 256), np.uint64)
    ch.run()
    assert L.nad_chain_trace_fetch(buf.ctypes.data, buf.nbytes) == 0
    b = buf.astype(np.int64)
    n = cr.n_ops
    t0 = b[0, 0].min()
    print(f"whole token: {n} ops, span {(b[5, n - 1].max() - t0) * tick:.1f} us")
    rows = {}
    for op in range(n):
        x = b[:, op]
        nm = "lm_head" if op == n - 1 else names[op % 4]
        rows.setdefault(nm, []).append(dict(
            gather=np.median(x[1] - x[0]) * tick, stage=np.median(x[2] - x[1]) * tick,
            first=np.median(x[3] - x[2]) * tick, loop=np.median(x[4] - x[3]) * tick,
            publish=np.median(x[5] - x[4]) * tick, fullwait=np.median(x[9]) * tick, freewait=np.median(x[8]) * tick,
            span=(x[5].max() - x[0].min()) * tick, endskew=(x[5].max() - x[5].min()) * tick))
    for nm, ds in rows.items():
        print(nm.ljust(8), " ".join(f"{k} {np.median([d[k] for d in ds]):6.2f}" for k in ds[0]), flush=True)
