"""Tensor-parallel composition on CPU: 2 (and 4) ranks through the library's C-ABI parallel context
(init_parallel_context / reduce_add / broadcast / alltoall / barrier, csrc/parallel_context.hip) over its TCP transport,
exact blob shards, row/column-parallel linears.  The per-rank matmul is the oracle here (no GPU in this container;
tests/test_tp_gpu.py runs the same composition with the HIP kernels); TP=W must reproduce TP=1 up to the all-reduce
summation order.  Pattern of the reference's TP test (tests/model-test/run_tp.sh: 2 ranks on one host vs 1 rank)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class OracleWeight:
    """test-local stand-in exposing DeviceWeight.forward's interface, computed by the oracle on the shard blob"""

    def __init__(self, blob, oracle):
        self.blob, self.o = blob, oracle
        inf = oracle.info(blob)
        self.n, self.k = inf["n"], inf["k"]

    def forward(self, x, out=None):
        y = torch.from_numpy(self.o.forward(np.ascontiguousarray(x.numpy()), self.blob, self.n, self.k))
        if out is not None:
            out.copy_(y)
            return out
        return y


def _blob(seed, n, k, gs=32):
    from neural_amd import bestla
    rng = np.random.default_rng(seed)
    W = rng.uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
    return bestla.quantize(W, gs, "int4", "bf16", "asym", "int8")


def _block(x, wq, wo, w1, w3, w2, ctx, world):
    """linear part of a decoder block: QKV-like col-parallel, O row-parallel, gate/up col, down row."""
    q = wq(x)                                   # [M, Nq_r]
    h = wo(q) if world > 1 else wo(q)           # row-parallel consumes the local columns, all-reduce inside
    g = w1(h)
    u = w3(h)
    t = g / (1 + torch.exp(-g)) * u             # SiLU(x.w1) * (x.w3), local columns
    return w2(t)


def _worker(rank, world, port, q, big=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", NAD_TP_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        from neural_amd.parallel_context import ParallelContext
        from neural_amd import tp
        from tests.oracle_lib import Oracle
        o = Oracle.get()
        ctx = ParallelContext("tcp")
        assert ctx.get_tp_size() == world and ctx.get_tp_rank() == rank
        # hidden, ffn: 10 groups of 32 give uneven K shards at world 4; world 8 takes 8 / 11 groups (2,2,2,1,...)
        d, f, gs = (256, 352, 32) if big else (128, 320, 32)
        names = {"wq": (".attention.wq.weight", d, d), "wo": (".attention.wo.weight", d, d),
                 "w1": (".feed_forward.w1.weight", f, d), "w3": (".feed_forward.w3.weight", f, d),
                 "w2": (".feed_forward.w2.weight", d, f)}
        layers = {}
        for i, (key, (name, n, k)) in enumerate(names.items()):
            blob = _blob(100 + i, n, k, gs)
            mode = tp.split_type("layers.0" + name)
            shard, rng_ = tp.shard_blob(blob, mode, rank, world, unit=gs)
            w = OracleWeight(shard, o)
            layers[key] = (tp.ColumnParallelLinear(w, rng_) if mode == tp.TP_1D_ROW else
                           tp.RowParallelLinear(w, rng_, ctx))
        # column shards of wq must line up with the K shards of wo, w1/w3 with w2
        assert layers["wq"].n_range == layers["wo"].k_range
        assert layers["w1"].n_range == layers["w2"].k_range == layers["w3"].n_range
        x = torch.from_numpy(np.random.default_rng(0).uniform(-1, 1, size=(3, d)).astype(np.float32))
        y = _block(x, layers["wq"], layers["wo"], layers["w1"], layers["w3"], layers["w2"], ctx, world)
        # broadcast / alltoall / gather helpers
        b = torch.full((4,), float(rank))
        ctx.broadcast(b, 0)
        assert torch.all(b == 0)
        send = torch.arange(world * 2, dtype=torch.float32) + 100 * rank
        recv = torch.empty_like(send)
        ctx.alltoall(send, recv)
        expect = torch.cat([torch.arange(2, dtype=torch.float32) + 2 * rank + 100 * r for r in range(world)])
        assert torch.equal(recv, expect)
        yq = layers["wq"](x)
        sizes = [hi - lo for lo, hi in (tp.shard_blob(_blob(100, d, d, gs), tp.TP_1D_ROW, r, world, unit=gs)[1]
                                        for r in range(world))]
        assert sizes[rank] == yq.shape[1]
        full_q = ctx.all_gather_cols(yq, sizes)
        assert ctx.max_over_ranks(float(rank)) == world - 1
        ctx.barrier()
        q.put((rank, y.numpy(), full_q.numpy()))
        ctx.destroy()
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put((rank, "ERR", traceback.format_exc() + str(e)))


def _run(world, big=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, big)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[1] is not None and not isinstance(r[1], str), r[2]
    return sorted(res, key=lambda r: r[0])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_tp_block_matches_single_rank(world):
    single = _run(1, world == 8)[0]
    multi = _run(world, world == 8)
    for _, y, fq in multi:
        scale = np.abs(single[1]).max()
        assert np.abs(y - single[1]).max() <= 1e-5 * scale   # only the all-reduce order differs
        np.testing.assert_array_equal(fq, single[2])          # column shards gather to the exact TP=1 output
