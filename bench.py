"""bench.py -- Llama-2-7B int4-g128 WOQ linear stack on MI355X: decode tokens/s (headline) + prefill TFLOPS.

One step = one decode token (M=1) through every weight-only-quantized linear layer of Llama-2-7B
(32 x [fused QKV, O, fused gate/up(+SiLU*mul), down] + lm_head), weights resident in HBM in the MFMA tile layout.
N GPUs = tensor parallel (the reference's docs/tensor_parallelism.md split): QKV / gate / up / lm_head split N
(column-parallel), O / down split K by whole quantization groups (row-parallel) followed by a sum all-reduce through
the library's C-ABI parallel context (nad_pc_*: RCCL over xGMI on the caller's stream).

The same JSON line also carries the other BASELINE configs as secondary workloads (never the headline `value`):
Llama-2-7B int4-g128 with GPTQ-style zero points (config 3) and Mistral-7B int2-g64 with the reference's int2 quant
policy (config 5: wv and w2 stay int4, llama_utils.cpp:269-287), each with its own algorithmic bytes and roofline.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  --gpus N > 1 without a torch.distributed environment re-launches this script as N ranks under
  torch.distributed.run (a child process, started before anything touches the GPU) and exits with its status.
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "decode tokens/sec + prefill TFLOPS, Llama-2-7B int4-g128 at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_F16_PEAK_TFLOPS = 2500.0

# model geometries; bits per weight role, group size, symmetry
LLAMA = dict(name="Llama-2-7B", hidden=4096, ffn=11008, layers=32, vocab=32000, kv=4096, head=128, group=128,
             bits=dict(q=4, k=4, v=4, o=4, gate=4, up=4, down=4, lm=4), asym=False, fuse_qkv=True)
LLAMA_ASYM = dict(LLAMA, asym=True, scale="bf16")   # GPTQ/AWQ zero points, bf16 scales as qpack stores them
# Mistral-7B: kv heads 8 (n_head_kv != n_head: the reference's CPU graph runs three matmuls, llama.cpp:212-215); int2
# policy keeps wv, w2 int4 sym.  Here nad_device_qkv_forward takes Q, K, V of different N and format: decode runs ONE
# launch of two formats ({Q, K} int2 + V int4, woq_gemv_m1_dual_kernel), prefill one GEMM per weight; every output is
# bit-identical to its own launch.
MISTRAL = dict(name="Mistral-7B", hidden=4096, ffn=14336, layers=32, vocab=32000, kv=1024, head=128, group=64,
               bits=dict(q=2, k=2, v=4, o=2, gate=2, up=2, down=4, lm=2), asym=False, fuse_qkv=False, group_qkv=True,
               int4_roles_sym=True)


def shard(n, world, rank, unit=1):
    units = (n + unit - 1) // unit
    base, rem = divmod(units, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo * unit, min(n, hi * unit)


def weight_bytes(n, k, bits, g, sbytes=2, asym=False):
    """bestla_benchmark.cpp:817-823: packed codes + one scale (+ one int8 zero point) per group."""
    groups = n * ((k + g - 1) // g)
    return n * k * bits // 8 + groups * sbytes + (groups if asym else 0)


def shard_table(cfg, world):
    """Per-rank tensor-parallel shards of the model geometry (what Stack builds on each rank; no GPU): head-aligned
    Q/K/V columns, O's K rows = that rank's heads, gate/up columns = down's K rows in whole quantization groups, vocab
    columns of lm_head in whole 16-column stripes."""
    H, F, g, hd = cfg["hidden"], cfg["ffn"], cfg["group"], cfg["head"]
    rows = []
    for r in range(world):
        q = shard(H, world, r, hd)
        kv = shard(cfg["kv"], world, r, hd)
        f = shard(F, world, r, g)
        v = shard(cfg["vocab"], world, r, 16)
        rows.append({"rank": r, "q_cols": q, "kv_cols": kv, "o_k_rows": q, "gate_up_cols": f, "down_k_rows": f,
                     "down_k_groups": (f[1] - f[0]) // g, "heads": (q[1] - q[0]) // hd, "lm_head_cols": v})
    return rows


class Stack:
    """Synthetic linear weights of one TP rank for a model geometry (random codes, scales U[0.001, 0.01])."""

    def __init__(self, cfg, rank, world, seed=1234):
        from neural_amd import bestla
        self.cfg, self.rank, self.world = cfg, rank, world
        H, F, g, hd = cfg["hidden"], cfg["ffn"], cfg["group"], cfg["head"]
        q0, q1 = shard(H, world, rank, hd)                   # whole heads
        kv0, kv1 = shard(cfg["kv"], world, rank, hd)
        f0, f1 = shard(F, world, rank, g)                    # gate/up N shard == down K shard (whole groups)
        v0, v1 = shard(cfg["vocab"], world, rank, 16)
        self.nq, self.nkv, self.nf, self.nv = q1 - q0, kv1 - kv0, f1 - f0, v1 - v0
        self.kh, self.kd = self.nq, self.nf                   # row-parallel K shards = column shards feeding them
        self.sbytes = 2
        scale = cfg.get("scale", "fp16")
        b, asym = cfg["bits"], cfg["asym"]
        # the int2 policy keeps its int4 roles symmetric (llama_utils.cpp:270-271: q4cfg.alg = sym)
        self.asym_of = lambda role: asym and not (cfg.get("int4_roles_sym") and b[role] == 4)  # noqa: E731
        mk = lambda role, n, k, s: bestla.DeviceWeight.synthetic(b[role], n, k, g, scale, self.asym_of(role),  # noqa
                                                                 seed=s)
        self.layers = []
        for li in range(cfg["layers"]):
            s = seed + 97 * li
            self.layers.append(dict(
                wq=mk("q", self.nq, H, s + 1), wk=mk("k", self.nkv, H, s + 2), wv=mk("v", self.nkv, H, s + 3),
                wo=mk("o", H, self.kh, s + 4), w1=mk("gate", self.nf, H, s + 5), w3=mk("up", self.nf, H, s + 6),
                w2=mk("down", H, self.kd, s + 7)))
        self.lm_head = mk("lm", self.nv, H, seed + 999)

    def launches(self, m):
        """(name, bytes, flops, count) of every WOQ launch in one step at M=m (act fp32 in / fp32 out)."""
        c, a, H, L = self.cfg, 4, self.cfg["hidden"], self.cfg["layers"]
        b, g = c["bits"], c["group"]
        wb = lambda role, n, k: weight_bytes(n, k, b[role], g, self.sbytes, self.asym_of(role))  # noqa: E731
        qkv = [("qkv", wb("q", self.nq, H) + wb("k", self.nkv, H) + wb("v", self.nkv, H) +
                (m * H + m * (self.nq + 2 * self.nkv)) * a, 2 * m * (self.nq + 2 * self.nkv) * H, L)]
        # {Q, K} one launch (same format), V its own -- except at M = 1, where both formats share ONE launch
        # (woq_gemv_m1_dual_kernel, NAD_GEMV_DUAL=1)
        dual = m == 1 and os.environ.get("NAD_GEMV_DUAL", "1") != "0"
        if c.get("group_qkv") and dual:
            pass                 # the fused entry above: one launch, the activations read once
        elif c.get("group_qkv"):
            qkv = [("qk", wb("q", self.nq, H) + wb("k", self.nkv, H) + (m * H + m * (self.nq + self.nkv)) * a,
                    2 * m * (self.nq + self.nkv) * H, L),
                   ("v", wb("v", self.nkv, H) + (m * H + m * self.nkv) * a, 2 * m * self.nkv * H, L)]
        elif not c["fuse_qkv"]:
            qkv = [("q", wb("q", self.nq, H) + (m * H + m * self.nq) * a, 2 * m * self.nq * H, L),
                   ("k", wb("k", self.nkv, H) + (m * H + m * self.nkv) * a, 2 * m * self.nkv * H, L),
                   ("v", wb("v", self.nkv, H) + (m * H + m * self.nkv) * a, 2 * m * self.nkv * H, L)]
        return qkv + [
            ("o", wb("o", H, self.kh) + (m * self.kh + m * H) * a, 2 * m * H * self.kh, L),
            ("gate_up", wb("gate", self.nf, H) + wb("up", self.nf, H) + (m * H + m * self.nf * 2) * a,
             2 * m * 2 * self.nf * H, L),
            ("down", wb("down", H, self.kd) + (m * self.kd + m * H) * a, 2 * m * H * self.kd, L),
            ("lm_head", wb("lm", self.nv, H) + (m * H + m * self.nv) * a, 2 * m * self.nv * H, 1),
        ]


class Runner:
    def __init__(self, stack, m, pc, device):
        import torch
        from neural_amd import bestla
        self.b, self.torch, self.st, self.m, self.pc = bestla, torch, stack, m, pc
        H = stack.cfg["hidden"]
        f = dict(dtype=torch.float32, device=device)
        g = torch.Generator(device="cpu").manual_seed(7)
        self.x = (torch.rand((m, H), generator=g) - 0.5).to(device)
        self.attn = (torch.rand((m, stack.kh), generator=g) - 0.5).to(device)
        self.qkv = torch.empty((3, m, stack.nq), **f)
        self.kv = torch.empty((2, m, stack.nkv), **f)
        self.o = torch.empty((m, H), **f)
        self.t1 = torch.empty((m, stack.nf), **f)
        self.t2 = torch.empty((m, stack.nf), **f)
        self.t2in = (torch.rand((m, stack.kd), generator=g) - 0.5).to(device)
        self.ffn = torch.empty((m, H), **f)
        self.logits = torch.empty((m, stack.nv), **f)
        self.world = stack.world

    def qkv_op(self, L):
        if self.st.cfg["fuse_qkv"]:
            self.b.qkv_forward(self.x, L["wq"], L["wk"], L["wv"], out=self.qkv)
        elif self.st.cfg.get("group_qkv"):
            self.b.qkv_forward(self.x, L["wq"], L["wk"], L["wv"], out=(self.qkv[0], self.kv[0], self.kv[1]))
        else:
            L["wq"].forward(self.x, out=self.qkv[0])
            L["wk"].forward(self.x, out=self.kv[0])
            L["wv"].forward(self.x, out=self.kv[1])

    def step(self, stream=None):
        b, st = self.b, self.st
        for L in st.layers:
            self.qkv_op(L)
            L["wo"].forward(self.attn, out=self.o)
            if self.world > 1:
                self.pc.reduce_add(self.o)
            b.ffn_forward(self.x, L["w1"], L["w2"], L["w3"], tmp1=self.t1, tmp2=self.t2, out=self.ffn)
            if self.world > 1:
                self.pc.reduce_add(self.ffn)
        st.lm_head.forward(self.x, out=self.logits)


def graph_time(fn, reps, torch):
    """Average device time of fn() (one decode token), captured once in a HIP graph and replayed `reps` times; HIP
    events recorded on the stream the kernels run on."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn(s)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
    torch.cuda.synchronize()
    del g
    return e0.elapsed_time(e1) / reps * 1e-3


def graph_times(fn, reps, torch):
    """Device time of each of `reps` replays of fn() captured once in a HIP graph (HIP events on the launch stream)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    out = []
    with torch.cuda.stream(s):
        fn(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn(s)
        g.replay()
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            g.replay()
            e1.record(s)
            e1.synchronize()
            out.append(e0.elapsed_time(e1) * 1e-3)
    torch.cuda.synchronize()
    del g
    return out


SYN_MS = [1, 2, 4, 8, 16, 17, 32, 64, 128, 256, 512, 1024, 2048, 4096]


def synthetic_sweep(torch, copies=128, reps=5, batch=64):
    """north_star's synthetic N x K x M GEMM throughput (bestla_benchmark.cpp:815-824 bytes,
    bestla_ut.h:69-76 cold-cache batching): K = N = 4096 int4 g128 sym fp16 scales, fp16 activations, M in SYN_MS.
    `copies` distinct weights (>= 1 GiB) rotated so the 256 MB Infinity Cache cannot serve them; per M one HIP graph
    of back-to-back launches replayed `reps` times -- min and median per launch.  Bytes per section 8(d) with 2-byte
    activations (in and out); M <= 64 is priced against HBM, larger M against the dense fp16 MFMA peak.
    Config 2 (M = 1) is also run as BTLAGemmBatchDriver-style batches (bestla_gemm.cpp:508-624): `batch` independent
    problems in ONE launch of the batched M = 1 GEMV (nad_batch_*); fp32 activations."""
    from neural_amd import bestla
    K = N = 4096
    g = 128
    ws = [bestla.DeviceWeight.synthetic(4, N, K, g, "fp16", False, seed=9000 + i) for i in range(copies)]
    wb = weight_bytes(N, K, 4, g, 2, False)
    gen = torch.Generator(device="cpu").manual_seed(11)
    rows = []
    for m in SYN_MS:
        x = (torch.rand((m, K), generator=gen) - 0.5).half().cuda()
        y = torch.empty((m, N), dtype=torch.float32, device="cuda")
        n = 256 if m <= 16 else (128 if m <= 256 else 32)

        def fn(st, x=x, y=y, n=n):
            for i in range(n):
                ws[i % copies].forward(x, out=y, stream=st)
        per = sorted(t / n for t in graph_times(fn, reps, torch))
        t_min, t_med = per[0], per[len(per) // 2]
        byts = wb + (m * K + m * N) * 2
        fl = 2.0 * m * N * K
        hbm = m <= 64
        gbps, tfl = byts / t_med / 1e9, fl / t_med / 1e12
        rows.append({"m": m, "us_min": round(t_min * 1e6, 3), "us_median": round(t_med * 1e6, 3),
                     "GBps": round(gbps, 1), "TFLOPs": round(tfl, 2), "bound": "hbm" if hbm else "mfma",
                     "frac": round(gbps / HBM_PEAK_GBPS if hbm else tfl / MFMA_F16_PEAK_TFLOPS, 4),
                     "kernel": bestla.plan_forward(4, N, K, g, "fp16", False, m, "fp16")["kernel"]})
        del x, y
    sets = copies // batch
    xs = [(torch.rand((1, K), generator=gen) - 0.5).cuda() for _ in range(batch)]
    ys = [torch.empty((1, N), dtype=torch.float32, device="cuda") for _ in range(batch)]
    byts = wb + (K + N) * 4
    # config 2 as BTLAGemmBatchDriver batches on the M = 1 GEMV (nad_batch_*): one launch per batch, workgroups dealt
    # out problem by problem (the batch's problems stream like one large launch)
    batches = [bestla.Batch([(ws[j * batch + i], xs[i], ys[i]) for i in range(batch)]) for j in range(sets)]

    def fb(st):
        for bb in batches:
            bb.run(stream=st)
    per = sorted(t / (sets * batch) for t in graph_times(fb, reps, torch))
    t_med = per[len(per) // 2]
    batched_gemv = {"problems_per_launch": batch, "launches_per_replay": sets,
                    "us_per_problem_min": round(per[0] * 1e6, 3), "us_per_problem_median": round(t_med * 1e6, 3),
                    "GBps": round(byts / t_med / 1e9, 1), "frac": round(byts / t_med / 1e9 / HBM_PEAK_GBPS, 4),
                    "bytes_per_problem": byts, "kernel": "woq_gemv_m1_kernel (batched: nad_batch_run)", "act": "fp32"}
    single = next(r for r in rows if r["m"] == 1)
    del batches, ws
    torch.cuda.empty_cache()
    return {"config": "K=N=4096 int4 g128 sym, fp16 scales, fp16 activations; 128 weight copies (1.1 GB) rotated "
                      "(cold); graph-replayed back-to-back launches, min / median over replays",
            "bytes_formula": "N*K/2 + N*K/128*2 + (M*K + M*N)*2 (section 8(d), 2-byte activations)",
            "per_m": rows,
            "config2_m1_single_launches": {k: single[k] for k in ("us_min", "us_median", "GBps", "frac", "kernel")},
            "config2_m1_batched": batched_gemv,
            "m4096_mfma_frac": next(r for r in rows if r["m"] == 4096)["frac"]}


def time_launches(stack, m, reps, torch):
    """Average device time of each WOQ launch shape: `reps` launches cycling through the 32 layers' distinct weights
    (cold: 3.4 GB of weights defeat the 256 MB Infinity Cache) captured in one HIP graph, timed with HIP events on the
    stream the kernels run on (graph replay: no host launch cost, only the kernel-to-kernel boundaries)."""
    from neural_amd import bestla
    r = Runner(stack, m, None, "cuda")
    ops = {
        "qkv": lambda L, s: r.qkv_op(L),
        "o": lambda L, s: L["wo"].forward(r.attn, out=r.o),
        "gate_up": lambda L, s: bestla.ffn_gate_up(r.x, L["w1"], L["w3"], tmp2=r.t2),
        "down": lambda L, s: L["w2"].forward(r.t2in, out=r.ffn),
        "lm_head": lambda L, s: L["lm"].forward(r.x, out=r.logits),
    }
    c = stack.cfg
    # lm_head is one 66 MB matrix: time it over 5 copies so the Infinity Cache cannot serve re-reads
    lms = [stack.lm_head] + [bestla.DeviceWeight.synthetic(c["bits"]["lm"], stack.nv, c["hidden"], c["group"],
                                                           c.get("scale", "fp16"), stack.asym_of("lm"), seed=5000 + i)
                             for i in range(4)]
    res = {}
    for name, fn in ops.items():
        n = reps if name != "lm_head" else 10
        layer = (lambda i: {"lm": lms[i % len(lms)]}) if name == "lm_head" else (lambda i: stack.layers[i % len(
            stack.layers)])

        def many(s, fn=fn, n=n, layer=layer):
            for i in range(n):
                fn(layer(i), s)
        res[name] = graph_time(many, 2, torch) / n
    del lms
    return res


def decode_workload(cfg, torch, reps=20, prefill=True, prefill_steps=5):
    """Secondary workload (one GPU): decode token time (graph-replayed, HIP events), its algorithmic bytes and
    roofline, and optionally the 2048-token prefill throughput."""
    st = Stack(cfg, 0, 1, seed=4321)
    run = Runner(st, 1, None, "cuda")
    t = graph_time(lambda s: run.step(), reps, torch)
    L1 = st.launches(1)
    byts = sum(b * c for _, b, _, c in L1)
    del run
    out = {"tokens_per_s": round(1.0 / t, 2), "ms_per_token": round(t * 1e3, 4), "bytes_per_token": int(byts),
           "roofline": {"bound": "hbm", "achieved": round(byts / t / 1e9, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": round(byts / t / 1e9 / HBM_PEAK_GBPS, 4)},
           "decode_path": "per-op launches", "launches_per_token": sum(c for *_, c in L1),
           "per_op_per_shape_us": {k: round(v * 1e6, 3) for k, v in time_launches(st, 1, reps, torch).items()}}
    if prefill:
        pre = Runner(st, 2048, None, "cuda")
        pdt = graph_time(lambda s: pre.step(stream=s), prefill_steps, torch)
        fl = sum(f * c for _, _, f, c in st.launches(2048))
        out["prefill_tflops"] = round(fl / pdt / 1e12, 2)
        out["prefill_ms_per_2048_tokens"] = round(pdt * 1e3, 3)
        del pre
    del st
    torch.cuda.empty_cache()
    return out


REFERENCE_PUBLISHED = {
    "decode_ms_per_token_total": 41.27, "decode_ms_per_token_woq_linear": 24.005,
    "woq_linear_tokens_per_s": round(1000.0 / 24.005, 2),
    "source": "docs/fused_attention.md:183-187,199 (Xeon Platinum 8480L, 56 threads, Llama-7B int4 sym g128 int8-compute; "
              "woq linear = MUL_QKV 6.034 + FFN_SILU 14.527 + INNER PRODUCT 3.444 ms)"}


def cpu_baseline(budget_s=12.0):
    """The oracle's restatement of the reference GEMV (kernel_ref.h:2489-2531, gemv_4bit_fp32_fp32 order), its
    independent NTILE column blocks spread over the host cores with OpenMP -- AVX-512 where the host has it (within
    fp32 reassociation, 1e-5 of max|C|, of the scalar oracle; tests/test_oracle_golden.py), else the scalar blocks
    (bit-identical) -- on one decoder layer's shapes + lm_head (int4 g128), repeated for ~budget_s seconds,
    extrapolated to a 32-layer token."""
    from tests.oracle_lib import Oracle, S4, F16
    orc = Oracle.get()
    # every host core this process may use: its affinity set, capped by the box's CPU share when the launcher sets
    # one (the GPU box exports OMP_NUM_THREADS = its share of the machine; os.cpu_count() is the whole machine)
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(usable, share) if share > 0 else usable)
    rng = np.random.default_rng(0)
    core = orc.core("avx512f")
    H, F, Lr, V, G = 4096, 11008, 32, 32000, 128
    shapes = [(3 * H, H, Lr), (H, H, Lr), (2 * F, H, Lr), (H, F, Lr), (V, H, 1)]
    prepared = []
    for n, k, count in shapes:
        Q = rng.integers(-8, 8, size=(k, n), dtype=np.int8)
        S = rng.uniform(0.001, 0.01, size=(k // G, n)).astype(np.float32)
        blob = orc.pack_q(Q, S, None, n, k, G, S4, F16, False, core)
        A = rng.uniform(-0.5, 0.5, size=(1, k)).astype(np.float32)
        prepared.append((n, k, count, blob, A, np.zeros((1, n), np.float32)))
    times = [[] for _ in prepared]
    vec = True
    t_start = time.perf_counter()
    while True:
        for i, (n, k, count, blob, A, Cout) in enumerate(prepared):
            t0 = time.perf_counter()
            r = orc.lib.orc_blob_gemv_avx512(A.ctypes.data, blob.ctypes.data, Cout.ctypes.data, k, threads) \
                if vec else -7
            if r == -7:  # no AVX-512 on this host: the scalar column blocks (same outputs, bit for bit)
                vec = False
                r = orc.lib.orc_blob_gemv_par(A.ctypes.data, blob.ctypes.data, Cout.ctypes.data, 1, k, n, threads)
            assert r == 0
            times[i].append(time.perf_counter() - t0)
        if time.perf_counter() - t_start >= budget_s:
            break
    spent = time.perf_counter() - t_start
    total = sum(float(np.median(ts)) * p[2] for ts, p in zip(times, prepared))
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(1.0 / total, 4), "unit": "tokens/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model, "host_cpus": os.cpu_count(), "usable_cpus": usable,
            "cores_note": "all CPUs this process may use (affinity), capped by the launcher's CPU share "
                          "(OMP_NUM_THREADS) when set",
            "sample": f"oracle GEMV (kernel_ref.h gemv_4bit_fp32_fp32 order; "
                      f"{'AVX-512, 16 columns per zmm, within fp32 reassociation of' if vec else 'scalar code, bit-identical to'} "
                      f"the scalar restatement; NTILE-48 column blocks over {threads} OpenMP threads) on one decoder layer (QKV "
                      f"12288x4096, O 4096x4096, gate+up 22016x4096, down 4096x11008) + lm_head 32000x4096 int4 g128, "
                      f"{len(times[0])} rounds ({spent:.1f} s of CPU work), median per shape extrapolated to 32 layers "
                      f"+ lm_head per token",
            "vectorized": "avx512" if vec else "scalar",
            "reference_published": REFERENCE_PUBLISHED,
            "note": "a vectorised restatement, not the reference's AVX512F / AMX JIT kernels (unbuildable offline: "
                    "xbyak) and not int8 compute; reference_published is the reference's own number on its own CPU"}


def latest_pmc():
    """The newest round's decode PMC traffic file: profiles/rNN_pmc_traffic_decode*.json with the highest round, the
    file listed last in that round's profiles/rNN_pmc_latest.txt when present (tools/pmc_traffic.py writes both)."""
    import glob
    import re
    prof = os.path.join(REPO, "profiles")
    best = None
    for f in glob.glob(os.path.join(prof, "r*_pmc_latest.txt")):
        rnd = int(re.match(r"r(\d+)_", os.path.basename(f)).group(1))
        names = [ln.strip() for ln in open(f) if ln.strip()]
        if names and os.path.exists(os.path.join(prof, names[-1])) and (best is None or rnd > best[0]):
            best = (rnd, os.path.join(prof, names[-1]))
    return best[1] if best else os.path.join(prof, "pmc_traffic.json")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def relaunch(args_list, n):
    """Start n ranks of this script under torch.distributed.run as a child process (nothing has touched the GPU in
    this process) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + args_list
    return subprocess.call(cmd)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--prefill-steps", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the secondary BASELINE workloads")
    ap.add_argument("--no-synthetic", action="store_true", help="skip the synthetic K=N=4096 M sweep")
    ap.add_argument("--dry-run", action="store_true", help="print the rank layout and exit (no GPU)")
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        if args.dry_run:
            print(json.dumps({"relaunch": True, "nproc_per_node": args.gpus,
                              "shards": shard_table(LLAMA, args.gpus)}))
            return 0
        return relaunch(argv, args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a wrong n_gpus")
    if args.dry_run:
        print(json.dumps({"relaunch": False, "world": world, "rank": rank, "local_rank": local,
                          "shards": shard_table(LLAMA, world)[rank:rank + 1]}))
        return 0

    import torch
    torch.cuda.set_device(local)
    from neural_amd import bestla  # noqa: F401  (fails loudly if the native library is missing)
    pc = None
    if world > 1:
        from neural_amd.parallel_context import ParallelContext
        pc = ParallelContext(device=local)  # C-ABI (nad_pc_*): RCCL communicator over the ranks
        assert pc.get_tp_size() == world, (pc.get_tp_size(), world)

    stack = Stack(LLAMA, rank, world)
    torch.cuda.synchronize()

    def barrier():
        if pc is not None:
            pc.barrier()
        torch.cuda.synchronize()

    def timed(runner, steps, warmup, use_graph):
        fn = runner.step
        if use_graph:
            # warm-up and capture on the SAME stream: the library's prefill scratch workspace is per stream (it grows
            # outside capture only), so a capture stream that never ran the shape would have none
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                runner.step()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                runner.step(stream=s)
            torch.cuda.current_stream().wait_stream(s)
            fn = g.replay
        for _ in range(warmup):
            fn()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        barrier()
        dt = time.perf_counter() - t0
        if pc is not None:
            dt = pc.max_over_ranks(dt)
        return dt

    # ---- decode (headline): M = 1, one launch per WOQ matmul (graph-replayed; the eager drop-in path beside it).
    # Tensor parallel: the same launches on this rank's shards + C-ABI all-reduce after O and down.  (The round-3/4
    # weight-stream engine -- one persistent launch per segment -- stayed slower than these launches and left the
    # product in round 5: tools/engine/)
    use_graph = not args.no_graph
    dec = Runner(stack, 1, pc, "cuda")
    dt = timed(dec, args.steps, args.warmup, use_graph)
    tok_s = args.steps / dt
    # the eager drop-in path (what ne_graph_compute does: one host call per WOQ node, no graph)
    dt_eager = timed(dec, args.steps, args.warmup, False)
    eager_tok_s = args.steps / dt_eager

    # ---- prefill: M = 2048 tokens
    pre = Runner(stack, 2048, pc, "cuda")
    # graph-replayed on one GPU (the TP ranks' 32 MiB all-reduces stay eager: RCCL under capture is not exercised)
    pdt = timed(pre, args.prefill_steps, 1, use_graph and world == 1)
    del pre
    pflops = sum(f * c for _, _, f, c in stack.launches(2048)) * world  # whole-job FLOPs
    prefill_tflops = pflops * args.prefill_steps / pdt / 1e12

    # ---- roofline of the dominant kernel on this rank's shards.  Algorithmic bytes per SURVEY.md §8(d)
    # (bestla_benchmark.cpp:817-823): packed weights + scales + activations in/out, for every WOQ matmul of the token.
    per = time_launches(stack, 1, 64, torch)
    L1 = stack.launches(1)
    tot_bytes = sum(b * c for _, b, _, c in L1)
    per_op_time = sum(per[n] * c for n, _, _, c in L1)
    n_per_op_launches = sum(c for *_, c in L1)
    kernel, bytes_per_launch, launch_s = "woq_gemv_m1_kernel (decode GEMV, one launch per matmul)", \
        tot_bytes / n_per_op_launches, per_op_time / n_per_op_launches
    achieved = bytes_per_launch / launch_s / 1e9
    traffic = None
    pmc = latest_pmc()
    if os.path.exists(pmc):
        try:
            rec = json.load(open(pmc))["woq_gemv_m1_kernel"]
            traffic = int(rec["traffic_over_algorithmic"] * bytes_per_launch)
        except Exception:
            traffic = None

    # ---- north_star's synthetic GEMM sweep (one GPU only)
    synthetic = None
    if world == 1 and not args.no_synthetic:
        synthetic = synthetic_sweep(torch)

    # ---- secondary BASELINE workloads (one GPU only)
    extra = None
    if world == 1 and not args.no_extra:
        del dec
        extra = {}
        extra["llama2_7b_int4_g128_asym_bf16scale"] = decode_workload(LLAMA_ASYM, torch)
        extra["mistral_7b_int2_g64_policy"] = decode_workload(MISTRAL, torch)
        extra["mistral_7b_int2_g64_policy"]["policy"] = "q,k,o,gate,up,lm_head int2 g64 sym; wv, w2 int4 g64 sym " \
                                                          "(llama_utils.cpp:269-287); kv heads 8: {q, k} one launch, v one"

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
            "config": {"workload": "Llama-2-7B int4-g128 sym decode linear stack, M=1 (32 x [QKV, O, gate/up+SiLU*mul, "
                                   "down] + lm_head), fp32 activations", "group_size": LLAMA["group"], "batch": 1,
                       "tp": world, "parallelism": f"tp{world}", "hip_graph": use_graph,
                       "decode_path": "per-op launches"},
            "prefill_tflops": round(prefill_tflops, 2),
            "prefill_ms_per_2048_tokens": round(pdt / args.prefill_steps * 1e3, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "traffic_source": os.path.basename(pmc) if traffic is not None else None,
                         "kernel": kernel, "bytes_per_launch": int(bytes_per_launch),
                         "avg_launch_us": round(launch_s * 1e6, 3)},
            "decode_eager_tokens_per_s": round(eager_tok_s, 2),
            "per_op_launches": {"tokens_per_s": round(tok_s, 2), "eager_tokens_per_s": round(eager_tok_s, 2),
                                "gemv_achieved_GBps": round(tot_bytes / per_op_time / 1e9, 1),
                                "per_shape_us": {k: round(v * 1e6, 3) for k, v in per.items()}},
            "prefill_roofline": {"bound": "mfma", "achieved": round(prefill_tflops / world, 2),
                                 "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                                 "frac": round(prefill_tflops / world / MFMA_F16_PEAK_TFLOPS, 4)},
            "synthetic": synthetic,
            "workloads": extra,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if pc is not None:
        pc.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
