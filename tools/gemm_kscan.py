"""K scan of the prefill GEMM (development tool): N=4096, M=2048, fp16 activations, K = 2048..16384, graph-replayed.
Splits a launch into a K-proportional part and a fixed part (prologue, output write-back, launch)."""
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from neural_amd import bestla
dev = "cuda"
for (n, k) in [(4096, 2048), (4096, 4096), (4096, 8192), (4096, 16384)]:
    w = bestla.DeviceWeight.synthetic(4, n, k, 128, "fp16", False, seed=3)
    x = (torch.rand((2048, k), device=dev) - 0.5).half()
    out = torch.empty((2048, n), device=dev)
    for _ in range(3): w.forward(x, out=out)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(10): w.forward(x, out=out)
    torch.cuda.current_stream().wait_stream(s)
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 10
    print(f"N={n} K={k} M=2048 graph: {us:8.1f} us  {2*2048*n*k/us/1e6:7.1f} TF/s", flush=True)
