"""Dense fp16 GEMM rate of the vendor library (torch.matmul -> hipBLASLt) at the prefill shapes, for comparison with the
fused WOQ prefill kernels: [M, K] x [K, N] with the weight pre-dequantized to fp16 (what a dequantize-then-GEMM split
would run).  Prints TF/s per shape (median of graph-replayed launches over rotated weight copies)."""
import sys

import torch

SHAPES = [("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008),
          ("lm_head", 32000, 4096)]


def main():
    ms = [int(v) for v in (sys.argv[1:] or ["2048", "4096"])]
    for dt in (torch.float16, torch.bfloat16):
        for m in ms:
            for name, n, k in SHAPES:
                copies = max(2, min(8, int(2e9 // (n * k * 2))))
                ws = [torch.randn(k, n, device="cuda", dtype=dt) * 0.01 for _ in range(copies)]
                a = torch.randn(m, k, device="cuda", dtype=dt)
                out = torch.empty(m, n, device="cuda", dtype=dt)
                for w in ws:
                    torch.matmul(a, w, out=out)
                torch.cuda.synchronize()
                times = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for w in ws * 4:
                        torch.matmul(a, w, out=out)
                    e1.record()
                    torch.cuda.synchronize()
                    times.append(e0.elapsed_time(e1) * 1e3 / (4 * copies))
                us = sorted(times)[len(times) // 2]
                print(f"{str(dt):15s} M={m:5d} {name:8s} N={n:5d} K={k:5d} {us:9.2f} us {2 * m * n * k / us / 1e6:8.1f} TF/s",
                      flush=True)
                del ws


if __name__ == "__main__":
    main()
