"""Tensor parallel on the GPU through the C-ABI: 2 ranks (both on cuda:0 -- the box has one GPU), each running the HIP
kernels on its exact blob shards (nad_blob_split), partial sums combined by the library's one-shot IPC all-reduce
(nad_pc_allreduce_f32; RCCL refuses two ranks on one device, so NAD_PC_NO_RCCL=1 here -- the 8-GPU node uses RCCL for
messages above the one-shot size).  A Llama-style block (col-parallel Q, row-parallel O + all-reduce, col-parallel
gate/up with the fused SiLU*mul epilogue, row-parallel down + all-reduce) at TP=2 must match TP=1 within 1e-5 relative
(only the summation order of the all-reduce differs) at M=1 (decode GEMV), 2e-4 at M=48 (prefill GEMM, whose fp16 input
rounding can amplify the order difference by one fp16 ulp of single elements); the all-reduce must
also replay correctly from a captured HIP graph (device-side generation counter)."""
import os
import socket

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


D, F, GS = 1024, 2816, 128      # F = 22 groups of 128: uneven K shards at TP=4, even at TP=2


def _blob(seed, n, k):  # noqa: D103
    from neural_amd import bestla
    rng = np.random.default_rng(seed)
    # ~1/sqrt(K)-scaled weights keep the block's activations O(1) like a real (RMS-normalised) layer; U[-0.5, 0.5] at
    # these widths drives SiLU(gate)*up past 65504, beyond the fp16 range the kernels compute in
    W = rng.uniform(-1.5, 1.5, size=(n, k)).astype(np.float32) / np.sqrt(k)
    return bestla.quantize(W, GS, "int4", "fp16", "sym", "int8")


def _worker(rank, world, port, q, dims=(D, F), ms=(1, 48), host_reduce=False):
    # one hardware queue per rank: W ranks share the one GPU, and with HIP's default of 4 queues per process world 8
    # oversubscribes the hardware queue slots -- a rank whose queue is not mapped cannot start its all-reduce while the
    # mapped ranks' all-reduces spin for it (bounded: they give up and report status 1)
    os.environ.update(MASTER_ADDR="127.0.0.1", NAD_TP_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", NAD_PC_NO_RCCL="1", GPU_MAX_HW_QUEUES="1")
    try:
        import torch
        torch.cuda.set_device(0)
        from neural_amd import bestla, tp
        from neural_amd.parallel_context import ParallelContext
        ctx = ParallelContext("tcp" if host_reduce else None)
        assert ctx.get_tp_size() == world and ctx.get_tp_rank() == rank
        info = ctx.info()
        if world > 1 and not host_reduce:
            assert info["oneshot"], "one-shot IPC all-reduce unavailable"
        d, f = dims
        spec = {"wq": (".attention.wq.weight", d, d), "wo": (".attention.wo.weight", d, d),
                "w1": (".feed_forward.w1.weight", f, d), "w3": (".feed_forward.w3.weight", f, d),
                "w2": (".feed_forward.w2.weight", d, f)}
        W, FULL = {}, {}
        for i, (key, (name, n, k)) in enumerate(spec.items()):
            b = _blob(200 + i, n, k)
            shard, rng_ = tp.shard_blob(b, tp.split_type("layers.0" + name), rank, world, unit=GS)
            W[key] = bestla.DeviceWeight(shard)
            FULL[key] = bestla.DeviceWeight(b)
            info["range_" + key] = rng_
        out, ref = {}, {}
        for m in ms:
            x = torch.from_numpy(np.random.default_rng(m).uniform(-1, 1, size=(m, d)).astype(np.float32)).cuda()

            def block(Wt, reduce):
                def allreduce(v):
                    if not host_reduce:
                        ctx.reduce_add(v)
                        return
                    hv = v.cpu()            # the matmuls stay on the GPU; the sum goes over the rendezvous sockets
                    ctx.reduce_add(hv)
                    v.copy_(hv)
                qh = Wt["wq"].forward(x)
                h = Wt["wo"].forward(qh)
                if reduce:
                    allreduce(h)
                t = bestla.ffn_gate_up(h, Wt["w1"], Wt["w3"], act="silu")
                y = Wt["w2"].forward(t)
                if reduce:
                    allreduce(y)
                return y
            y = block(W, True)
            y1 = block(FULL, False)     # TP=1 on the same GPU, same inputs
            torch.cuda.synchronize()
            out[m] = y.cpu().numpy()
            ref[m] = y1.cpu().numpy()
        if host_reduce:
            ctx.barrier()
            ctx.destroy()
            q.put((rank, out, True, ref, info))
            return
        # graph-captured all-reduce replayed twice
        buf = torch.full((4096,), float(rank + 1), device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                buf.mul_(1.0)
                ctx.reduce_add(buf)
        torch.cuda.current_stream().wait_stream(s)
        buf.fill_(float(rank + 1))
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        tri = world * (world + 1) / 2
        expect = tri * world if world > 1 else 1.0    # sum of (r+1) over ranks, then that sum summed again
        graph_ok = bool(torch.all(buf == expect).item())
        assert ctx.status() == 0
        ctx.barrier()
        ctx.destroy()
        q.put((rank, out, graph_ok, ref, info))
    except Exception as e:
        import traceback
        q.put((rank, "ERR", traceback.format_exc() + str(e)))


def _run(world, dims=(D, F), ms=(1, 48), host_reduce=False):
    import torch.multiprocessing as mp
    c = mp.get_context("spawn")
    q = c.Queue()
    port = _free_port()
    ps = [c.Process(target=_worker, args=(r, world, port, q, dims, ms, host_reduce)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert not isinstance(r[1], str), r[2]
    return sorted(res, key=lambda r: r[0])


def _check_tp(world, dims=(D, F), ms=(1, 48), host_reduce=False):
    single = _run(1, dims, ms)[0]
    multi = _run(world, dims, ms, host_reduce)
    for m in ms:   # TP=1 computed in the world-1 run and in each rank agree bit for bit
        np.testing.assert_array_equal(single[1][m], single[3][m])
        np.testing.assert_array_equal(multi[0][3][m], single[3][m])
    for _, out, graph_ok, _, _ in multi:
        assert graph_ok, "graph-replayed one-shot all-reduce gave a wrong sum"
        for m in ms:
            ref = single[1][m].astype(np.float64)
            err = np.abs(out[m] - ref).max() / np.abs(ref).max()
            # M=48 rounds each GEMM input to fp16: a 1e-7 change of h from the all-reduce order can move an element
            # across an fp16 rounding boundary (one ulp = 1e-3 of that element) -> allow 2e-4 there
            assert err <= (1e-5 if m <= 16 else 2e-4), (m, err)
    # every rank holds the identical reduced result (rank-order summation)
    for m in ms:
        for r in range(1, world):
            np.testing.assert_array_equal(multi[0][1][m], multi[r][1][m])
    return multi


@pytest.mark.skipif(not gpu_available(), reason="needs a GPU")
def test_tp2_hip_kernels_match_tp1():
    _check_tp(2)


@pytest.mark.skipif(not gpu_available(), reason="needs a GPU")
def test_tp4_uneven_k_shards_match_tp1():
    """World 4 on the one GPU: F = 2816 = 22 groups of 128 -> the row-parallel down weight gets
    UNEVEN K shards 6/6/5/5 groups (model_files.h:134-235 requires even splits; here whole groups, exact), the gate/up
    column shards line up with them, and which one-shot allocation actually ran is recorded."""
    multi = _check_tp(4)
    ranges = [r[4]["range_w2"] for r in multi]
    assert ranges == [(0, 768), (768, 1536), (1536, 2176), (2176, 2816)], ranges
    assert [r[4]["range_w1"] for r in multi] == ranges                 # gate/up N shard == down K shard
    allocs = {r[4]["oneshot_alloc"] for r in multi}
    assert len(allocs) == 1 and allocs <= {"uncached", "hipMalloc"}, allocs
    print(f"\nTP=4 one-shot all-reduce buffer: {allocs.pop()} (nad_pc_info bit 3); down K shards {ranges}")


@pytest.mark.skipif(not gpu_available(), reason="needs a GPU")
def test_tp8_llama_layer_shapes_match_tp1():
    """World 8 emulated on the one GPU at Llama-2-7B layer shapes (configs[3]'s split,
    model_files.h:134-235): col-parallel Q 4096 -> 512 columns (4 heads) per rank, O row-parallel over 4 x 128 k per
    rank, gate/up 11008 -> 1408 / 1280 columns, and down's K = 11008 = 86 groups of 128 cut 11 x 6 + 10 x 2 (uneven,
    whole groups, exact) with the gate/up column shards lined up; TP=8 against TP=1 within 1e-5 at M = 1 (decode GEMV)
    and M = 8.  The sums go over the rendezvous sockets (host transport): eight processes' spinning one-shot
    all-reduces on ONE GPU need all eight of their queues mapped at once, which the hardware scheduler does not promise
    (the one-shot device all-reduce is exercised at worlds 2 and 4 above; on the 8-GPU node each rank has its own GPU)."""
    multi = _check_tp(8, (4096, 11008), (1, 8), host_reduce=True)
    ranges = [r[4]["range_w2"] for r in multi]
    groups = [(e - b) // GS for b, e in ranges]
    assert groups == [11] * 6 + [10] * 2, groups
    assert ranges[0][0] == 0 and ranges[-1][1] == 11008
    assert [r[4]["range_w1"] for r in multi] == ranges
    assert [r[4]["range_wq"] for r in multi] == [(512 * i, 512 * (i + 1)) for i in range(8)]
    assert [r[4]["range_wo"] for r in multi] == [(512 * i, 512 * (i + 1)) for i in range(8)]


def _rccl_worker(q):
    """world 1 with NAD_PC_FORCE_RCCL=1: the RCCL bootstrap (unique id over the rendezvous, ncclCommInitRank) and the
    RCCL all-reduce / broadcast / alltoall calls that the 8-GPU node runs, exercised on the one GPU here."""
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", NAD_PC_FORCE_RCCL="1")
    try:
        import torch
        torch.cuda.set_device(0)
        from neural_amd.parallel_context import ParallelContext
        ctx = ParallelContext()
        info = ctx.info()
        assert info["rccl"] and not info["oneshot"], info
        x = torch.arange(1 << 20, dtype=torch.float32, device="cuda")
        y = torch.empty_like(x)
        ctx.reduce_add(x, y)
        b = torch.full((1000,), 3.0, device="cuda")
        ctx.broadcast(b)
        s = torch.arange(64, dtype=torch.float32, device="cuda")
        r = torch.empty_like(s)
        ctx.alltoall(s, r)
        h = np.arange(5000, dtype=np.float32)
        ht = torch.from_numpy(h.copy())
        ctx.reduce_add(ht)                      # host tensor: staged through the device, synchronous
        torch.cuda.synchronize()
        ok = bool(torch.equal(x, y)) and bool(torch.all(b == 3.0)) and bool(torch.equal(s, r)) and \
            bool(np.array_equal(ht.numpy(), h))
        ctx.destroy()
        q.put(("ok", ok))
    except Exception as e:
        import traceback
        q.put(("ERR", traceback.format_exc() + str(e)))


@pytest.mark.skipif(not gpu_available(), reason="needs a GPU")
def test_rccl_transport_world1():
    import torch.multiprocessing as mp
    c = mp.get_context("spawn")
    q = c.Queue()
    p = c.Process(target=_rccl_worker, args=(q,))
    p.start()
    tag, v = q.get(timeout=240)
    p.join(timeout=60)
    assert tag == "ok", v
    assert v
