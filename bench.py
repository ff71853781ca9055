"""bench.py -- Llama-2-7B int4-g128 WOQ linear stack on MI355X: decode tokens/s (headline) + prefill TFLOPS.

One step = one decode token (M=1) through every weight-only-quantized linear layer of Llama-2-7B
(32 x [fused QKV, O, fused gate/up(+SiLU*mul), down] + lm_head), weights resident in HBM in the MFMA tile layout.
N GPUs = tensor parallel (the reference's docs/tensor_parallelism.md split): QKV / gate / up / lm_head split N
(column-parallel), O / down split K by whole quantization groups (row-parallel) followed by an RCCL all-reduce.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]   (N>1: launched by torch.distributed.run)
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HIDDEN, FFN, LAYERS, VOCAB = 4096, 11008, 32, 32000
GROUP = 128
METRIC = "decode tokens/sec + prefill TFLOPS, Llama-2-7B int4-g128 at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_F16_PEAK_TFLOPS = 2500.0


def shard(n, world, rank, unit=1):
    units = (n + unit - 1) // unit
    base, rem = divmod(units, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo * unit, min(n, hi * unit)


def weight_bytes(n, k, bits=4, g=GROUP, sbytes=2):
    return n * k * bits // 8 + n * ((k + g - 1) // g) * sbytes


class Stack:
    """Synthetic Llama-2-7B linear weights for one TP rank."""

    def __init__(self, rank, world, seed=1234):
        from neural_amd import bestla
        self.rank, self.world = rank, world
        q0, q1 = shard(HIDDEN, world, rank, 128)          # heads of 128
        f0, f1 = shard(FFN, world, rank, GROUP)             # gate/up N shard == down K shard
        h0, h1 = shard(HIDDEN, world, rank, GROUP)         # row-parallel K split: whole groups
        d0, d1 = shard(FFN, world, rank, GROUP)
        v0, v1 = shard(VOCAB, world, rank, 16)
        self.nq, self.nf, self.kh, self.kd, self.nv = q1 - q0, f1 - f0, h1 - h0, d1 - d0, v1 - v0
        mk = lambda n, k, s: bestla.DeviceWeight.synthetic(4, n, k, GROUP, "fp16", False, seed=s)  # noqa: E731
        self.layers = []
        for li in range(LAYERS):
            s = seed + 97 * li
            self.layers.append(dict(
                wq=mk(self.nq, HIDDEN, s + 1), wk=mk(self.nq, HIDDEN, s + 2), wv=mk(self.nq, HIDDEN, s + 3),
                wo=mk(HIDDEN, self.kh, s + 4), w1=mk(self.nf, HIDDEN, s + 5), w3=mk(self.nf, HIDDEN, s + 6),
                w2=mk(HIDDEN, self.kd, s + 7)))
        self.lm_head = mk(self.nv, HIDDEN, seed + 999)

    def launches(self, m):
        """(name, bytes, flops, count) of every WOQ launch in one step at M=m (act fp32 in / fp32 out)."""
        a = 4
        return [
            ("qkv", 3 * weight_bytes(self.nq, HIDDEN) + (m * HIDDEN + 3 * m * self.nq) * a,
             2 * m * 3 * self.nq * HIDDEN, LAYERS),
            ("o", weight_bytes(HIDDEN, self.kh) + (m * self.kh + m * HIDDEN) * a, 2 * m * HIDDEN * self.kh, LAYERS),
            ("gate_up", 2 * weight_bytes(self.nf, HIDDEN) + (m * HIDDEN + m * self.nf * 2) * a,
             2 * m * 2 * self.nf * HIDDEN, LAYERS),
            ("down", weight_bytes(HIDDEN, self.kd) + (m * self.kd + m * HIDDEN) * a, 2 * m * HIDDEN * self.kd, LAYERS),
            ("lm_head", weight_bytes(self.nv, HIDDEN) + (m * HIDDEN + m * self.nv) * a, 2 * m * self.nv * HIDDEN, 1),
        ]


class Runner:
    def __init__(self, stack, m, dist, device):
        import torch
        from neural_amd import bestla
        self.b, self.torch, self.st, self.m, self.dist = bestla, torch, stack, m, dist
        f = dict(dtype=torch.float32, device=device)
        g = torch.Generator(device="cpu").manual_seed(7)
        self.x = (torch.rand((m, HIDDEN), generator=g) - 0.5).to(device)
        self.attn = (torch.rand((m, stack.kh), generator=g) - 0.5).to(device)
        self.qkv = torch.empty((3, m, stack.nq), **f)
        self.o = torch.empty((m, HIDDEN), **f)
        self.t1 = torch.empty((m, stack.nf), **f)
        self.t2 = torch.empty((m, stack.nf), **f)
        self.t2in = (torch.rand((m, stack.kd), generator=g) - 0.5).to(device)
        assert stack.nf == stack.kd and stack.nq == stack.kh
        self.ffn = torch.empty((m, HIDDEN), **f)
        self.logits = torch.empty((m, stack.nv), **f)
        self.world = stack.world

    def step(self):
        b, st = self.b, self.st
        for L in st.layers:
            b.qkv_forward(self.x, L["wq"], L["wk"], L["wv"], out=self.qkv)
            L["wo"].forward(self.attn, out=self.o)
            if self.world > 1:
                self.dist.all_reduce(self.o)
            b.ffn_forward(self.x, L["w1"], L["w2"], L["w3"], tmp1=self.t1, tmp2=self.t2, out=self.ffn)
            if self.world > 1:
                self.dist.all_reduce(self.ffn)
        st.lm_head.forward(self.x, out=self.logits)


class ChainRunner:
    """The decode step as ONE persistent launch (nad_chain_*): every WOQ matmul of the token with its real data
    dependencies -- x -> RMSNorm -> QKV -> (attention at position 0 is the identity on V) -> O + x -> RMSNorm ->
    gate/up + SiLU*mul -> down + h -> next layer, then RMSNorm -> lm_head.  RoPE at position 0 is the identity too;
    only the attention over a KV history (out of scope) is not modelled."""

    def __init__(self, stack, m, device):
        import torch
        from neural_amd import bestla
        f = dict(dtype=torch.float32, device=device)
        g = torch.Generator(device="cpu").manual_seed(7)
        self.xs = [(torch.rand((m, HIDDEN), generator=g) - 0.5).to(device), torch.empty((m, HIDDEN), **f)]
        self.q, self.k, self.v = (torch.empty((m, stack.nq), **f) for _ in range(3))
        self.h = torch.empty((m, HIDDEN), **f)
        self.t = torch.empty((m, stack.nf), **f)
        self.logits = torch.empty((m, stack.nv), **f)
        ops = []
        for li, L in enumerate(stack.layers):
            x, xn = self.xs[li % 2], self.xs[(li + 1) % 2]
            ops.append(dict(kind=bestla.CHAIN_QKV, w=[L["wq"], L["wk"], L["wv"]], act=x, out=[self.q, self.k, self.v],
                            norm=True))
            ops.append(dict(kind=bestla.CHAIN_LINEAR, w=[L["wo"]], act=self.v, out=[self.h], epi=bestla.EPI_RES_ADD,
                            res=x))
            ops.append(dict(kind=bestla.CHAIN_GATE_UP, w=[L["w1"], L["w3"]], act=self.h, out=[self.t], norm=True))
            ops.append(dict(kind=bestla.CHAIN_LINEAR, w=[L["w2"]], act=self.t, out=[xn], epi=bestla.EPI_RES_ADD,
                            res=self.h))
        ops.append(dict(kind=bestla.CHAIN_LINEAR, w=[stack.lm_head], act=self.xs[len(stack.layers) % 2],
                        out=[self.logits], norm=True))
        self.chain = bestla.Chain(ops, m)
        self.n_ops = len(ops)

    def step(self, stream=None):
        self.chain.run(stream=stream)


def time_chain(chain_runner, reps, torch):
    """Average device time of one chain launch (= one decode token), graph-replayed, HIP events on its stream."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        chain_runner.step(stream=s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            chain_runner.step(stream=s)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def time_launches(stack, m, reps, torch):
    """Average device time of each WOQ launch shape: `reps` launches cycling through the 32 layers' distinct weights
    (cold: 3.4 GB of weights defeat the 256 MB Infinity Cache) captured in one HIP graph, timed with HIP events on the
    stream the kernels run on (graph replay: no host launch cost, only the kernel-to-kernel boundaries)."""
    from neural_amd import bestla
    r = Runner(stack, m, None, "cuda")
    ops = {
        "qkv": lambda L: bestla.qkv_forward(r.x, L["wq"], L["wk"], L["wv"], out=r.qkv),
        "o": lambda L: L["wo"].forward(r.attn, out=r.o),
        "gate_up": lambda L: bestla.ffn_forward(r.x, L["w1"], L["w2"], L["w3"], tmp1=r.t1, tmp2=r.t2, out=r.ffn),
        "down": lambda L: L["w2"].forward(r.t2in, out=r.ffn),
        "lm_head": lambda L: L["lm"].forward(r.x, out=r.logits),
    }
    # lm_head is one 66 MB matrix: time it over 5 copies so the Infinity Cache cannot serve re-reads
    lms = [stack.lm_head] + [bestla.DeviceWeight.synthetic(4, stack.nv, HIDDEN, GROUP, "fp16", False, seed=5000 + i)
                             for i in range(4)]
    res = {}
    s = torch.cuda.Stream()
    for name, fn in ops.items():
        n = reps if name != "lm_head" else 10
        layer = (lambda i: {"lm": lms[i % len(lms)]}) if name == "lm_head" else (lambda i: stack.layers[i % LAYERS])
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(4):
                fn(layer(i))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for i in range(n):
                    fn(layer(i))
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            g.replay()
            g.replay()
            e1.record(s)
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / (2 * n) * 1e-3  # seconds per launch
        del g
    del lms
    # the fused FFN op above is the gate/up dual launch + the down launch: subtract down to isolate gate/up
    res["gate_up"] = max(res["gate_up"] - res["down"], 1e-9)
    return res


def cpu_baseline():
    """The oracle's restatement of the reference GEMV (kernel_ref.h:2489-2531, gemv_4bit_fp32_fp32 order), its
    independent NTILE column blocks spread over the host cores with OpenMP (bit-identical to the scalar oracle), on one
    decoder layer's shapes + lm_head (int4 g128), extrapolated to a 32-layer token."""
    from tests.oracle_lib import Oracle, S4, F16
    orc = Oracle.get()
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))
    rng = np.random.default_rng(0)
    core = orc.core("avx512f")
    shapes = [(3 * HIDDEN, HIDDEN, LAYERS), (HIDDEN, HIDDEN, LAYERS), (2 * FFN, HIDDEN, LAYERS), (HIDDEN, FFN, LAYERS),
              (VOCAB, HIDDEN, 1)]
    total = 0.0
    spent = 0.0
    for n, k, count in shapes:
        Q = rng.integers(-8, 8, size=(k, n), dtype=np.int8)
        S = rng.uniform(0.001, 0.01, size=(k // GROUP, n)).astype(np.float32)
        blob = orc.pack_q(Q, S, None, n, k, GROUP, S4, F16, False, core)
        A = rng.uniform(-0.5, 0.5, size=(1, k)).astype(np.float32)
        Cout = np.zeros((1, n), np.float32)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            r = orc.lib.orc_blob_gemv_par(A.ctypes.data, blob.ctypes.data, Cout.ctypes.data, 1, k, n, threads)
            assert r == 0
        dt = (time.perf_counter() - t0) / reps
        spent += dt * reps
        total += dt * count
    return {"value": 1.0 / total, "unit": "tokens/s", "cores": threads, "kind": "port",
            "sample": f"oracle GEMV (kernel_ref.h gemv_4bit_fp32_fp32 order, scalar code, NTILE column blocks over "
                      f"{threads} OpenMP threads) on one decoder layer (QKV 12288x4096, O 4096x4096, gate+up "
                      f"22016x4096, down 4096x11008) + lm_head 32000x4096 int4 g128, 3 runs each ({spent:.1f} s), "
                      f"extrapolated to 32 layers + lm_head per token"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--prefill-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--per-op", action="store_true", help="headline from per-op launches instead of the decode chain")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from neural_amd import bestla  # noqa: F401  (fails loudly if the native library is missing)

    stack = Stack(rank, world)
    torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def timed(runner, steps, warmup, use_graph):
        fn = runner.step
        if use_graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                runner.step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                runner.step(**({"stream": torch.cuda.current_stream()} if isinstance(runner, ChainRunner) else {}))
            fn = g.replay
        for _ in range(warmup):
            fn()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        barrier()
        dt = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([dt], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    # ---- decode (headline): M = 1.  One GPU: the whole token as one persistent chain launch (nad_chain_*);
    # tensor parallel: per-op launches with an RCCL all-reduce after O and down.
    use_graph = world == 1 and not args.no_graph
    chain = None
    chain_tok_s = None
    if world == 1 and not args.per_op:
        chain = ChainRunner(stack, 1, "cuda")
        dt_chain = timed(chain, args.steps, args.warmup, use_graph)
        assert chain.chain.status() == 0, "decode chain hand-off timed out"
        chain_tok_s = args.steps / dt_chain
    dec = Runner(stack, 1, dist, "cuda")
    dt_op = timed(dec, args.steps, args.warmup, use_graph)
    per_op_tok_s = args.steps / dt_op
    # the headline is the faster of the two complete decode paths (both run every WOQ matmul of the token)
    if chain is not None and dt_chain >= dt_op:
        chain = None
    dt = dt_chain if chain is not None else dt_op
    tok_s = args.steps / dt

    # ---- prefill: M = 2048 tokens
    pre = Runner(stack, 2048, dist, "cuda")
    pdt = timed(pre, args.prefill_steps, 1, False)
    pflops = sum(f * c for _, _, f, c in stack.launches(2048)) * world  # whole-job FLOPs
    prefill_tflops = pflops * args.prefill_steps / pdt / 1e12

    # ---- roofline of the dominant kernel on this rank's shards.  Algorithmic bytes per SURVEY.md §8(d)
    # (bestla_benchmark.cpp:817-823): packed weights + scales + activations in/out, for every WOQ matmul of the token.
    per = time_launches(stack, 1, 64, torch)
    L1 = stack.launches(1)
    tot_bytes = sum(b * c for _, b, _, c in L1)
    per_op_time = sum(per[n] * c for n, _, _, c in L1)
    n_per_op_launches = sum(c for *_, c in L1)
    if chain is not None:
        # one woq_chain_kernel launch = one token: its average duration, HIP events on the stream it runs on
        chain_us = time_chain(chain, 20, torch)
        kernel, bytes_per_launch, launch_s = "woq_chain_kernel (whole decode step, one persistent launch)", tot_bytes, \
            chain_us
    else:
        kernel, bytes_per_launch, launch_s = "woq_gemv_kernel (decode GEMV, one launch per matmul)", \
            tot_bytes / n_per_op_launches, per_op_time / n_per_op_launches
    achieved = bytes_per_launch / launch_s / 1e9
    # HBM traffic per launch from the committed PMC pass (profiles/pmc_traffic.json: FETCH_SIZE x 2 + WRITE_SIZE, the
    # gfx950 correction of MI355X_MICROARCH.md), scaled from its measured traffic / algorithmic-bytes ratio
    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            rec = json.load(open(pmc))["woq_chain_kernel" if chain is not None else "woq_gemv_kernel"]
            traffic = int(rec["traffic_over_algorithmic"] * bytes_per_launch)
        except Exception:
            traffic = None

    if rank == 0:
        cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline()
        line = {
            "metric": METRIC,
            "value": round(tok_s, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f16",
            "data": "synthetic: random int4 codes + fp16 group scales U[0.001,0.01] in Llama-2-7B shapes (no checkpoint)",
            "config": {"workload": "Llama-2-7B int4-g128 sym decode step, M=1: 32 x [RMSNorm, fused QKV, O + residual, "
                                   "RMSNorm, gate/up + SiLU*mul, down + residual] + RMSNorm + lm_head, fp32 activations "
                                   "(attention at position 0 = V)" if chain is not None else
                                   "Llama-2-7B int4-g128 sym decode linear stack, M=1 (32 x [QKV, O, gate/up+SiLU*mul, "
                                   "down] + lm_head), fp32 activations", "group_size": GROUP, "batch": 1,
                       "tp": world, "parallelism": f"tp{world}", "cuda_graph": use_graph,
                       "decode_path": "chain (1 launch per token)" if chain is not None else "per-op launches"},
            "prefill_tflops": round(prefill_tflops, 2),
            "prefill_ms_per_2048_tokens": round(pdt / args.prefill_steps * 1e3, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel": kernel, "bytes_per_launch": int(bytes_per_launch),
                         "avg_launch_us": round(launch_s * 1e6, 3)},
            "decode_chain_tokens_per_s": None if chain_tok_s is None else round(chain_tok_s, 2),
            "per_op_launches": {"tokens_per_s": round(per_op_tok_s, 2),
                                "gemv_achieved_GBps": round(tot_bytes / per_op_time / 1e9, 1),
                                "per_shape_us": {k: round(v * 1e6, 3) for k, v in per.items()}},
            "prefill_roofline": {"bound": "mfma", "achieved": round(prefill_tflops / world, 2),
                                 "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                                 "frac": round(prefill_tflops / world / MFMA_F16_PEAK_TFLOPS, 4)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
