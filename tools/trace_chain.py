"""Phase trace of the decode chain (development tool): per op, median / max over workgroups of
prefetch->barrier-passed, staging, stream, publish; and the gaps between ops.  Needs `make -C neural_amd chaintrace`."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["NAD_LIB_PATH"] = os.path.join(REPO, "neural_amd", "libneural_amd_chaintrace.so")
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from neural_amd import _lib  # noqa: E402

layers = int(sys.argv[1]) if len(sys.argv) > 1 else 32
bench.LAYERS = layers
stack = bench.Stack(0, 1)
cr = bench.ChainRunner(stack, 1, "cuda")
for _ in range(3):
    cr.step()
torch.cuda.synchronize()
L = _lib.lib()
L.nad_chain_trace_fetch.argtypes = [C.c_void_p, C.c_size_t]
buf = np.zeros((6, 160, 256), np.uint64)
cr.step()
assert L.nad_chain_trace_fetch(buf.ctypes.data, buf.nbytes) == 0
khz = 100000.0  # wall_clock64 runs at 100 MHz on MI300-class parts
tick = 1e3 / khz
n = cr.n_ops
t0 = buf[0, 0].astype(np.int64).min()
names = ["qkv", "o", "gate_up", "down"]
tot = (buf[4, n - 1].astype(np.int64).max() - t0) * tick
print(f"chain span {tot:.1f} us over {n} ops")
rows = {}
for op in range(n):
    b = buf[:, op].astype(np.int64)
    nm = names[op % 4] if op < n - 1 else "lm_head"
    d = dict(wait=np.median(b[1] - b[0]) * tick, stage=np.median(b[2] - b[1]) * tick,
             stream=np.median(b[3] - b[2]) * tick, stream_max=(b[3] - b[2]).max() * tick,
             publish=np.median(b[4] - b[3]) * tick,
             span=(b[4].max() - b[0].min()) * tick,
             start_skew=(b[0].max() - b[0].min()) * tick)
    rows.setdefault(nm, []).append(d)
for nm, ds in rows.items():
    keys = ds[0].keys()
    print(nm.ljust(8), " ".join(f"{k} {np.median([d[k] for d in ds]):6.2f}" for k in keys))
