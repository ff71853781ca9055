"""Prefill GEMM sweep (development tool): TFLOP/s of one WOQ linear per Llama-2-7B shape at prefill M.

Usage: python tools/gemm_sweep.py [--m 2048,4096] [--act fp16,fp32] [--shapes o,gate,down,lm_head] [--reps 20]
       [--kernels 3,2] [--bits 4] [--group 128] [--asym]
Kernels: 7 / 3 / 2 = the int4 pipelined kernels, suffix k = gemm4 waves split over K (j: the library's auto choice), a = int4 g128 on gemm4 too, f / u = fold at g128 on / off (default: the library's), 4 = gemm4 (int4 g32/g64, int2), 0 = generic tiled fallback.
Each line: shape, M, activation dtype, kernel, average device time per forward (HIP events on the launch stream, back
to back launches) and TFLOP/s (2*M*N*K / time).  fp32 activations include the one-pass fp16 conversion kernel.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SHAPES = {"o": (4096, 4096), "gate": (11008, 4096), "down": (4096, 11008), "lm_head": (32000, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="2048,4096")
    ap.add_argument("--act", default="fp16,fp32")
    ap.add_argument("--shapes", default="o,gate,down,lm_head")
    ap.add_argument("--kernels", default="3,2")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--group", type=int, default=128)
    ap.add_argument("--asym", action="store_true")
    ap.add_argument("--nk", default="", help="extra N:K shapes, comma separated (named nNkK)")
    args = ap.parse_args()
    import torch
    from neural_amd import _lib, bestla
    dev = torch.device("cuda:0")
    print(torch.cuda.get_device_name(0), flush=True)
    for nk in filter(None, args.nk.split(",")):
        n_, k_ = (int(v) for v in nk.split(":"))
        SHAPES[f"n{n_}k{k_}"] = (n_, k_)
    names = args.shapes.split(",") + [f"n{n_}k{k_}" for n_, k_ in (map(int, nk.split(":")) for nk in filter(None, args.nk.split(",")))]
    for name in filter(None, names):
        n, k = SHAPES[name]
        w = bestla.DeviceWeight.synthetic(args.bits, n, k, args.group, "fp16", args.asym, seed=3)
        for m in (int(x) for x in args.m.split(",")):
            for act in args.act.split(","):
                dt = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}[act]
                x = (torch.rand((m, k), device=dev) - 0.5).to(dt)
                out = torch.empty((m, n), device=dev)
                s = torch.cuda.current_stream()
                for kname in args.kernels.split(","):
                    kern = kname
                    os.environ["NAD_GEMM_KERNEL"] = kern[0]
                    os.environ["NAD_GEMM2_DISABLE"] = "1" if kern[0] == "0" else "0"
                    os.environ["NAD_GEMM4_DISABLE"] = "1" if kern[0] != "4" else "0"
                    os.environ["NAD_GEMM3_STAGGER"] = "1" if "s" in kern[1:] else "0"
                    os.environ["NAD_GEMM4_KSW"] = "1" if "k" in kern[1:] else ("2" if "j" in kern[1:] else "0")
                    os.environ["NAD_GEMM4_ALL"] = "1" if "a" in kern[1:] else "0"
                    if "f" in kern[1:] or "u" in kern[1:]:  # else the library's default
                        os.environ["NAD_GEMM4_FOLD_ALL"] = "1" if "f" in kern[1:] else "0"
                    else:
                        os.environ.pop("NAD_GEMM4_FOLD_ALL", None)
                    _lib.reload_knobs()  # the library reads its switches once
                    for _ in range(3):
                        w.forward(x, out=out)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record(s)
                    for _ in range(args.reps):
                        w.forward(x, out=out)
                    e1.record(s)
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / args.reps
                    tf = 2.0 * m * n * k / us / 1e6
                    print(f"{name:8s} b{args.bits} g{args.group}{'a' if args.asym else 's'} N={n:5d} K={k:5d} M={m:5d} {act} gemm{kname}: {us:9.1f} us  {tf:7.1f} TFLOP/s",
                          flush=True)
                del x, out
        del w


if __name__ == "__main__":
    main()
