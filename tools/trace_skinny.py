"""Phase trace of the decode (skinny) kernel on each Llama-2-7B shape -- development tool, not part of the product.

Loads neural_amd/libneural_amd_trace.so (`make -C neural_amd trace`: the same kernels with per-workgroup wall-clock
stamps at entry, after the prologue barrier, at the last wave's main-loop end and at exit), rotates enough weight
copies to defeat the 256 MB Infinity Cache, and prints per-shape: HIP-event time per launch, the traced launch's span,
and the distribution of each phase across workgroups.  Usage: python tools/trace_skinny.py [shape ...]
"""
import ctypes as C
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("NAD_LIB_PATH", os.path.join(REPO, "neural_amd", "libneural_amd_trace.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from neural_amd import _lib, bestla  # noqa: E402

SLOTS, MAXWG = 8, 16384
G = 128


def wbytes(n, k):
    return n * k // 2 + n * (k // G) * 2


def main():
    L = _lib.lib()
    L.nad_trace_fetch.restype = C.c_int
    L.nad_trace_fetch.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int]
    L.nad_trace_clock_khz.restype = C.c_int
    khz = L.nad_trace_clock_khz()
    tick_us = 1e3 / khz
    dev = torch.device("cuda")
    x = torch.empty((1, 11008), device=dev).uniform_(-1, 1)
    shapes = {  # name: (n, k, weights per launch, grid filter)
        "qkv": (4096, 4096, 3), "o": (4096, 4096, 1), "gate_up": (11008, 4096, 2), "down": (4096, 11008, 1),
        "lm_head": (32000, 4096, 1)}
    want = sys.argv[1:] or list(shapes)
    print(f"wall clock {khz} kHz; {torch.cuda.get_device_name()}")
    buf = np.zeros((SLOTS, MAXWG), np.uint64)
    for name in want:
        n, k, nw = shapes[name]
        per = nw * wbytes(n, k)
        copies = max(2, math.ceil(700e6 / per))
        ws = [[bestla.DeviceWeight.synthetic(4, n, k, G, "fp16", False, seed=1000 * i + j) for j in range(nw)]
              for i in range(copies)]
        xa = x[:, :k].contiguous()
        out = torch.empty((3, 1, n), device=dev)
        tmp = torch.empty((2, 1, n), device=dev)
        w2 = bestla.DeviceWeight.synthetic(4, 4096, n, G, "fp16", False, seed=7) if name == "gate_up" else None

        def launch(i):
            w = ws[i]
            if name == "qkv":
                bestla.qkv_forward(xa, w[0], w[1], w[2], out=out)
            elif name == "gate_up":
                bestla.ffn_forward(xa, w[0], w2, w[1], tmp1=tmp[0], tmp2=tmp[1], out=out[0, :, :4096])
            else:
                w[0].forward(xa, out=out[0])

        for i in range(copies):
            launch(i)
        torch.cuda.synchronize()
        reps = max(copies, 64)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in range(reps):
            launch(r % copies)
        e1.record()
        torch.cuda.synchronize()
        ev_us = e0.elapsed_time(e1) * 1e3 / reps
        # trace: record only launches of this grid size; the last launch's stamps survive
        grid = {"qkv": 3 * ((n + 15) // 16), "gate_up": (n + 15) // 16}.get(name, (n + 15) // 16)
        assert L.nad_trace_fetch(None, 0, 1, grid) == 0
        for i in range(copies):
            launch(i)
        assert L.nad_trace_fetch(buf.ctypes.data, buf.nbytes, 0, 0) == 0
        s0, s1, s2, s3 = (buf[i, :grid].astype(np.int64) for i in range(4))
        ids = buf[SLOTS - 1, :grid]
        t0 = s0.min()
        span = (s3.max() - t0) * tick_us
        q = lambda v: "p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f" % tuple(  # noqa: E731
            np.percentile(v * tick_us, [10, 50, 90, 100]))
        cu = ids & 0xFFFFFFFF
        xcc = ids >> 32
        per_cu = np.unique(xcc * 4096 + cu, return_counts=True)[1]
        print(f"\n== {name}: N={n} K={k} x{nw}, {per / 1e6:.2f} MB/launch, grid {grid}, copies {copies}")
        print(f"  event avg {ev_us:7.2f} us  -> {per / ev_us / 1e3:7.1f} GB/s")
        print(f"  traced span {span:7.2f} us -> {per / span / 1e3:7.1f} GB/s")
        print(f"  wg start offset   {q(s0 - t0)}")
        print(f"  prologue (->bar)  {q(s1 - s0)}")
        print(f"  main loop         {q(s2 - s1)}")
        print(f"  reduce+epilogue   {q(s3 - s2)}")
        print(f"  wg end offset     {q(s3 - t0)}")
        print(f"  CUs used {len(per_cu)}, WGs per CU min {per_cu.min()} max {per_cu.max()}, XCCs {np.unique(xcc).size}")
        del ws


if __name__ == "__main__":
    main()
