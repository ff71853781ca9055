"""Phase trace of the mid-M kernel (development tool, not part of the product): loads libneural_amd_trace.so (make -C
neural_amd trace), runs cold forwards (rotating weight copies) at K = N = 4096, and prints for the last launch the
distribution over workgroups of each stamp relative to the earliest entry: 0 entry, 1 loads issued, 2 compute done
(last wave), 3 LDS reduce done, 5 exit.
Usage: python tools/trace_mid.py [M ...]"""
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


def main():
    L = _lib.lib()
    L.nad_mid_trace_fetch.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    n = k = 4096
    copies = 48
    ws = [bestla.DeviceWeight.synthetic(4, n, k, 128, "fp16", False, seed=11 + i) for i in range(copies)]
    buf = np.zeros((SLOTS, MAXWG), np.uint64)
    for m in [int(v) for v in (sys.argv[1:] or ["17", "64"])]:
        x = (torch.rand((m, k), device="cuda") - 0.5).half()
        out = torch.empty((m, n), device="cuda")
        for i in range(copies):
            ws[i].forward(x, out=out)
        torch.cuda.synchronize()
        for rep in range(3):
            L.nad_mid_trace_fetch(None, 0, 1)
            torch.cuda.synchronize()
            ws[rep].forward(x, out=out)
            torch.cuda.synchronize()
            L.nad_mid_trace_fetch(buf.ctypes.data, buf.nbytes, 0)
            plan = ws[0].plan(m, "fp16")
            g = plan["grid"]
            t = buf[:, :g].astype(np.int64)
            t0 = t[0][t[0] > 0].min()
            print(f"M={m} rep {rep} grid {g} ksplit {plan['ksplit']}  (us from the first entry: min / median / max)")
            for s in range(7):
                v = t[s][t[s] > 0]
                if len(v) == 0:
                    continue
                d = (v - t0) / 100.0  # 100 MHz wall clock
                print(f"   stamp {s}: n={len(v):4d}  {d.min():7.2f} {np.median(d):7.2f} {d.max():7.2f}")


if __name__ == "__main__":
    main()
