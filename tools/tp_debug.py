"""Diagnose the 2-rank TP block on one GPU: compare every intermediate with the TP=1 computation done in-process."""
import os
import sys
import socket
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
D, F, GS = 1024, 2816, 128


def blob(seed, n, k):
    from neural_amd import bestla
    rng = np.random.default_rng(seed)
    W = rng.uniform(-1.5, 1.5, size=(n, k)).astype(np.float32) / np.sqrt(k)
    return bestla.quantize(W, GS, "int4", "fp16", "sym", "int8")


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", NAD_TP_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", NAD_PC_NO_RCCL="1")
    import torch
    torch.cuda.set_device(0)
    from neural_amd import bestla, tp
    from neural_amd.parallel_context import ParallelContext
    ctx = ParallelContext()
    print(rank, "info", ctx.info(), flush=True)
    # all-reduce unit check: distinct random data per rank
    for cnt in (() if os.environ.get("SKIP_AR") else (1, 7, 1024, 4096, 49152, 100000)):
        data = [torch.from_numpy(np.random.default_rng(1000 * r + cnt).standard_normal(cnt).astype(np.float32))
                for r in range(world)]
        expect = sum(d.double() for d in data)
        buf = data[rank].cuda()
        ctx.reduce_add(buf)
        torch.cuda.synchronize()
        err = (buf.cpu().double() - expect).abs().max().item()
        print(rank, "allreduce", cnt, "err", err, "status", ctx.status(), flush=True)
    spec = {"wq": (".attention.wq.weight", D, D), "wo": (".attention.wo.weight", D, D),
            "w1": (".feed_forward.w1.weight", F, D), "w3": (".feed_forward.w3.weight", F, D),
            "w2": (".feed_forward.w2.weight", D, F)}
    full, W = {}, {}
    for i, (key, (name, n, k)) in enumerate(spec.items()):
        b = blob(200 + i, n, k)
        full[key] = bestla.DeviceWeight(b)
        shard, rng_ = tp.shard_blob(b, tp.split_type("layers.0" + name), rank, world, unit=GS)
        W[key] = (bestla.DeviceWeight(shard), rng_)
        print(rank, key, "range", rng_, flush=True)
    x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, size=(1, D)).astype(np.float32)).cuda()
    q_full = full["wq"].forward(x)
    q_sh = W["wq"][0].forward(x)
    lo, hi = W["wq"][1]
    print(rank, "q shard err", (q_sh - q_full[:, lo:hi]).abs().max().item(), q_full.abs().max().item(), flush=True)
    h_full = full["wo"].forward(q_full)
    h_part = W["wo"][0].forward(q_sh)
    klo, khi = W["wo"][1]
    ref_part = full["wo"].forward(torch.nn.functional.pad(q_full[:, klo:khi], (klo, D - khi)))
    print(rank, "h partial err", (h_part - ref_part).abs().max().item(), flush=True)
    h = h_part.clone()
    ctx.reduce_add(h)
    torch.cuda.synchronize()
    print(rank, "status after first reduce", ctx.status(), flush=True)
    print(rank, "h reduced err", (h - h_full).abs().max().item(), h_full.abs().max().item(), flush=True)
    t_full = bestla.ffn_gate_up(h_full, full["w1"], full["w3"])
    t_sh = bestla.ffn_gate_up(h, W["w1"][0], W["w3"][0])
    flo, fhi = W["w1"][1]
    print(rank, "t shard err", (t_sh - t_full[:, flo:fhi]).abs().max().item(), t_full.abs().max().item(), flush=True)
    y_full = full["w2"].forward(t_full)
    y_part = W["w2"][0].forward(t_sh)
    klo, khi = W["w2"][1]
    print(rank, "w2 range", (klo, khi), flush=True)
    ref_part = full["w2"].forward(torch.nn.functional.pad(t_full[:, klo:khi], (klo, F - khi)))
    print(rank, "y partial err", (y_part - ref_part).abs().max().item(), flush=True)
    ctx.reduce_add(y_part)
    torch.cuda.synchronize()
    print(rank, "y reduced err", (y_part - y_full).abs().max().item(), y_full.abs().max().item(), flush=True)
    ctx.barrier()
    ctx.destroy()


if __name__ == "__main__":
    import multiprocessing as mp
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    c = mp.get_context("spawn")
    ps = [c.Process(target=worker, args=(r, 2, port)) for r in range(2)]
    [p.start() for p in ps]
    [p.join(timeout=200) for p in ps]
