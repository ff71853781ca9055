"""The reference-named fused C-ABI entries (ne_bestla.h:38-69), called exactly as ne_layers.c calls them -- with HOST
pointers (the NE CPU-tensor path: weights uploaded once per blob and cached, activations staged) -- against the oracle:
bestla_fusion_add_f32f32_forward (inner_product.cpp:132-244), bestla_fusion_QKV_f32f32_forward (ip_fusion_qkv.cpp),
bestla_fusion_FFN_{SiLu,Gelu_Mul,GeLu,Add_GeLu}_f32f32_forward (ip_fusion_ffn.cpp:734-800).  Plus the host weight
cache's invalidation (re-pack into the same buffer) and the device workspace contract (caller workspace / bound
workspace / loud failure under graph capture).

Tolerances: decode (M <= 16, fp32 activations split hi/lo): 1e-4 for the chained FFN (fp32 intermediate), 2e-5 for
single GEMMs; prefill (M > 16, activations rounded to fp16 once per GEMM): north_star's 1e-3, also for the chained FFN
(two fp16 roundings; the error actually reached at Llama / Mistral shapes is recorded by
test_model_shapes_gpu.py::test_ffn_prefill_error_at_model_shapes)."""
import ctypes as C

import numpy as np
import pytest

from tests.conftest import gpu_available
from tests.oracle_lib import F16, F32, S2, S4
from tests.test_gpu_parity import _blob, _rel_err

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from neural_amd import _lib, bestla


def _gelu(x):
    return 0.5 * x * (1 + np.tanh(0.7978845834732056 * (x + 0.044714998453855515 * x ** 3)))


def _silu(x):
    return x / (1 + np.exp(-x))


def vp(a):
    return a.ctypes.data_as(C.c_void_p)


def _wb(oracle, n, k, seed, bs=128):
    rng = np.random.default_rng(seed)
    W = (rng.uniform(-1.5, 1.5, size=(n, k)) / np.sqrt(k)).astype(np.float32)
    core = oracle.lib.orc_select_core(4, S4, bs, 0, 0)
    return oracle.quant_pack(W, n, k, bs, S4, F16, False, core, is_trans=True)


@pytest.mark.parametrize("m", [1, 5, 40])
@pytest.mark.parametrize("bcast", [True, False])
def test_fusion_add(oracle, m, bcast):
    L = _lib.lib()
    n, k = 192, 512
    blob = _wb(oracle, n, k, 1)
    rng = np.random.default_rng(m)
    A = rng.uniform(-1, 1, size=(m, k)).astype(np.float32)
    bias = rng.uniform(-1, 1, size=(n,) if bcast else (m, n)).astype(np.float32)
    out = np.zeros((m, n), np.float32)
    L.nad_clear_error()
    assert L.bestla_fusion_add_f32f32_support(vp(blob), m, n, k)
    L.bestla_fusion_add_f32f32_forward(vp(A), vp(blob), vp(bias), vp(out), m, n, k, k, n, bcast, None)
    assert _lib.last_error() == ""
    ref = oracle.forward(A, blob, n, k).astype(np.float64) + bias
    assert _rel_err(out, ref) <= (2e-5 if m <= 16 else 1e-3)


@pytest.mark.parametrize("m", [1, 9, 48])
def test_fusion_qkv(oracle, m):
    L = _lib.lib()
    n, k = 256, 1024
    blobs = [_wb(oracle, n, k, 10 + i) for i in range(3)]
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, k)).astype(np.float32)
    out = np.zeros((3, m, n), np.float32)   # Q, K, V at output, output + M*ldo, output + 2*M*ldo
    assert L.bestla_fusion_QKV_f32f32_support(vp(blobs[0]), vp(blobs[1]), vp(blobs[2]), m, n, k)
    L.nad_clear_error()
    L.bestla_fusion_QKV_f32f32_forward(vp(A), vp(blobs[0]), vp(blobs[1]), vp(blobs[2]), vp(out), m, n, k, k, n, None)
    assert _lib.last_error() == ""
    for i in range(3):
        assert _rel_err(out[i], oracle.forward(A, blobs[i], n, k)) <= (2e-5 if m <= 16 else 1e-3)


@pytest.mark.parametrize("m", [1, 4, 40])
@pytest.mark.parametrize("kind", ["SiLu", "Gelu_Mul"])
def test_fusion_ffn_three_weights(oracle, m, kind):
    L = _lib.lib()
    fin, fmid, fout = 512, 768, 384
    b1, b3, b2 = _wb(oracle, fmid, fin, 21), _wb(oracle, fmid, fin, 23), _wb(oracle, fout, fmid, 22)
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, fin)).astype(np.float32)
    tmp1 = np.zeros((m, fmid), np.float32)
    tmp2 = np.zeros((m, fmid), np.float32)
    out = np.zeros((m, fout), np.float32)
    sup = getattr(L, f"bestla_fusion_FFN_{kind}_f32f32_support")
    fwd = getattr(L, f"bestla_fusion_FFN_{kind}_f32f32_forward")
    assert sup(vp(b1), vp(b2), vp(b3), m, fin, fmid, fout)
    L.nad_clear_error()
    fwd(vp(A), vp(b1), vp(b2), vp(b3), vp(tmp1), vp(tmp2), vp(out), m, fin, fmid, fout, None)
    assert _lib.last_error() == ""
    h1 = oracle.forward(A, b1, fmid, fin).astype(np.float64)
    h3 = oracle.forward(A, b3, fmid, fin).astype(np.float64)
    t = (_silu(h1) if kind == "SiLu" else _gelu(h1)) * h3
    ref = oracle.forward(t.astype(np.float32), b2, fout, fmid)
    assert _rel_err(tmp2, t) <= (1e-4 if m <= 16 else 1e-3)
    assert _rel_err(out, ref) <= (1e-4 if m <= 16 else 1e-3)


@pytest.mark.parametrize("m", [1, 6, 40])
@pytest.mark.parametrize("kind", ["GeLu", "Add_GeLu"])
def test_fusion_ffn_two_weights(oracle, m, kind):
    """FFN_GeLu: tmp1 = gelu(X.W1), out = tmp1.W2; FFN_Add_GeLu: tmp1 = gelu(X.W1 + b1), out = tmp1.W2 + b2
    (ip_fusion_ffn.cpp:760-800, broadcast bias)."""
    L = _lib.lib()
    fin, fmid, fout = 512, 640, 256
    b1, b2 = _wb(oracle, fmid, fin, 31), _wb(oracle, fout, fmid, 32)
    rng = np.random.default_rng(m)
    A = rng.uniform(-1, 1, size=(m, fin)).astype(np.float32)
    bias1 = rng.uniform(-0.5, 0.5, size=(fmid,)).astype(np.float32)
    bias2 = rng.uniform(-0.5, 0.5, size=(fout,)).astype(np.float32)
    tmp1 = np.zeros((m, fmid), np.float32)
    out = np.zeros((m, fout), np.float32)
    L.nad_clear_error()
    if kind == "GeLu":
        assert L.bestla_fusion_FFN_GeLu_f32f32_support(vp(b1), vp(b2), m, fin, fmid, fout)
        L.bestla_fusion_FFN_GeLu_f32f32_forward(vp(A), vp(b1), vp(b2), vp(tmp1), vp(out), m, fin, fmid, fout, None)
        h = _gelu(oracle.forward(A, b1, fmid, fin).astype(np.float64))
        ref = oracle.forward(h.astype(np.float32), b2, fout, fmid).astype(np.float64)
    else:
        assert L.bestla_fusion_FFN_Add_GeLu_f32f32_support(vp(b1), vp(b2), m, fin, fmid, fout)
        L.bestla_fusion_FFN_Add_GeLu_f32f32_forward(vp(A), vp(b1), vp(b2), vp(bias1), vp(bias2), vp(tmp1), vp(out), m,
                                                    fin, fmid, fout, True, None)
        h = _gelu(oracle.forward(A, b1, fmid, fin).astype(np.float64) + bias1)
        ref = oracle.forward(h.astype(np.float32), b2, fout, fmid).astype(np.float64) + bias2
    assert _lib.last_error() == ""
    assert _rel_err(tmp1, h) <= (1e-4 if m <= 16 else 1e-3)
    assert _rel_err(out, ref) <= (1e-4 if m <= 16 else 1e-3)


def test_host_cache_sees_repack_into_same_buffer(oracle):
    """Pack, forward, re-pack DIFFERENT weights into the same buffer (BTLAGemmQuantPackB), forward again: the result
    follows the new weights (the cache was keyed by pointer + size only)."""
    L = _lib.lib()
    n, k, m = 128, 512, 2
    rng = np.random.default_rng(0)
    A = rng.uniform(-1, 1, size=(m, k)).astype(np.float32)
    size = L.BTLAGemmPackBSize(n, k, 128, S4, F16, False, 4, None)
    buf = bestla._aligned_buffer(size)
    for seed in (1, 2):
        W = rng.uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
        assert L.BTLAGemmQuantPackB(vp(buf), vp(W), n, k, k, 128, S4, F16, False, 4, True, None)
        out = np.zeros((m, n), np.float32)
        L.bestla_f32f32_forward(vp(A), vp(buf), vp(out), m, n, k, k, n, None)
        assert _rel_err(out, oracle.forward(A, buf, n, k)) <= 2e-5, seed
    # a byte-level rewrite that keeps the header (another writer): the fingerprint covers the scales
    W = rng.uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
    other = bestla._aligned_buffer(size)
    assert L.BTLAGemmQuantPackB(vp(other), vp(W), n, k, k, 128, S4, F16, False, 4, True, None)
    buf[:] = other
    out = np.zeros((m, n), np.float32)
    L.bestla_f32f32_forward(vp(A), vp(buf), vp(out), m, n, k, k, n, None)
    assert _rel_err(out, oracle.forward(A, buf, n, k)) <= 2e-5
    L.nad_host_cache_clear()


def test_host_cache_evict_contract_for_partial_rewrites(oracle):
    """the per-call key samples the blob, so a partial in-place rewrite outside the pack API (a few groups
    re-scaled) need not change it -- the documented contract (include/neural_amd.h) is nad_host_cache_evict before such
    a rewrite is used.  Checked: after the rewrite + evict the forward follows the new bytes."""
    L = _lib.lib()
    n, k, m = 96, 1024, 3
    blob = _wb(oracle, n, k, 41)
    A = np.random.default_rng(2).uniform(-1, 1, size=(m, k)).astype(np.float32)
    out = np.zeros((m, n), np.float32)
    L.bestla_f32f32_forward(vp(A), vp(blob), vp(out), m, n, k, k, n, None)
    assert _rel_err(out, oracle.forward(A, blob, n, k)) <= 2e-5
    # rewrite the scales of a handful of (group, column) entries in place: fp16 scales, halve them
    info = bestla.blob_info(blob)
    s_off = int(info["s_off"]) if "s_off" in info else None
    assert s_off is not None, info
    sc = blob[s_off:s_off + 2 * 16].view(np.float16).copy()
    blob[s_off:s_off + 2 * 16] = (sc * np.float16(0.5)).view(np.uint8)
    L.nad_host_cache_evict(vp(blob))
    L.bestla_f32f32_forward(vp(A), vp(blob), vp(out), m, n, k, k, n, None)
    assert _rel_err(out, oracle.forward(A, blob, n, k)) <= 2e-5
    L.nad_host_cache_clear()


def test_device_forward_uses_caller_workspace_and_capture_contract(oracle):
    """bestla_device_f32f32_forward runs the prefill GEMM with the caller's workspace (sized by bestla_support ->
    nad_device_workspace_size); nad_device_forward under graph capture uses a bound workspace, and without one on a
    fresh stream it fails loudly instead of switching kernels."""
    L = _lib.lib()
    n, k, m = 256, 1024, 100  # past the mid-M kernel (M <= 64 reads the activations as they are)
    blob = _wb(oracle, n, k, 5)
    w = bestla.DeviceWeight(blob)
    A = np.random.default_rng(1).uniform(-1, 1, size=(m, k)).astype(np.float32)
    ref = oracle.forward(A, blob, n, k)
    x = torch.from_numpy(A).cuda()
    ws_bytes = L.nad_device_workspace_size(m, k)
    assert ws_bytes >= m * k * 2
    ws = torch.zeros(ws_bytes, dtype=torch.uint8, device="cuda")
    y = torch.empty(m, n, device="cuda")
    L.nad_clear_error()
    s = torch.cuda.current_stream()
    L.bestla_device_f32f32_forward(C.c_void_p(x.data_ptr()), w.desc, C.c_void_p(y.data_ptr()), m, n, k, k, n,
                                   C.c_void_p(ws.data_ptr()), C.c_void_p(s.cuda_stream))
    torch.cuda.synchronize()
    assert _lib.last_error() == ""
    assert _rel_err(y.cpu().numpy(), ref) <= 1e-3
    assert int(ws.count_nonzero()) > 0            # the fp16 activation copy went into the caller's buffer
    # capture on a fresh stream: without a workspace -> loud error; with a bound one -> graph replays correctly
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        with pytest.raises(RuntimeError, match="workspace"):
            with torch.cuda.graph(g, stream=st):
                w.forward(x, out=y, stream=st)
    st2 = torch.cuda.Stream()
    st2.wait_stream(torch.cuda.current_stream())
    ws2 = torch.zeros(ws_bytes, dtype=torch.uint8, device="cuda")
    assert L.nad_bind_workspace(C.c_void_p(st2.cuda_stream), C.c_void_p(ws2.data_ptr()), ws_bytes) == 0
    y2 = torch.zeros(m, n, device="cuda")
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st2):
        with torch.cuda.graph(g2, stream=st2):
            w.forward(x, out=y2, stream=st2)
    g2.replay()
    torch.cuda.synchronize()
    assert _rel_err(y2.cpu().numpy(), ref) <= 1e-3
    L.nad_bind_workspace(C.c_void_p(st2.cuda_stream), None, 0)


@pytest.mark.parametrize("m", [8, 16])
def test_mid_m_capture_with_bound_workspace(oracle, m):
    """at M = 8..16 fp32 rows take the mid-M kernel with split-K slabs; nad_device_workspace_size(m, k)
    covers them, so graph capture with a workspace of exactly that size replays correctly (no 'needs N bytes')."""
    L = _lib.lib()
    n, k = 512, 4096
    blob = _wb(oracle, n, k, 11)
    w = bestla.DeviceWeight(blob)
    p = w.plan(m, "fp32")
    assert p["kernel"] == "woq_mid_kernel" and p["ksplit"] > 1, p
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, k)).astype(np.float32)
    ref = oracle.forward(A, blob, n, k)
    x = torch.from_numpy(A).cuda()
    ws_bytes = L.nad_device_workspace_size(m, k)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    ws = torch.zeros(ws_bytes, dtype=torch.uint8, device="cuda")
    assert L.nad_bind_workspace(C.c_void_p(st.cuda_stream), C.c_void_p(ws.data_ptr()), ws_bytes) == 0
    y = torch.zeros(m, n, device="cuda")
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.stream(st):
            with torch.cuda.graph(g, stream=st):
                w.forward(x, out=y, stream=st)
        g.replay()
        torch.cuda.synchronize()
    finally:
        L.nad_bind_workspace(C.c_void_p(st.cuda_stream), None, 0)
    assert _rel_err(y.cpu().numpy(), ref) <= 2e-5


def test_host_cache_code_only_rewrite_and_lru_bound(oracle):
    """(1) a rewrite that changes only the CODES and keeps every scale, through the pack API
    (BTLAGemmPackB into the same buffer) or by another writer followed by nad_host_cache_evict, is seen by the next
    forward; (2) the cache is bounded by device bytes, least recently used first out, and results stay exact when
    entries are evicted and re-uploaded."""
    L = _lib.lib()
    n, k, m = 128, 512, 2
    rng = np.random.default_rng(3)
    A = rng.uniform(-1, 1, size=(m, k)).astype(np.float32)
    s = rng.uniform(0.001, 0.01, size=(k // 128, n)).astype(np.float32)
    size = L.BTLAGemmPackBSize(n, k, 128, S4, F32, False, 4, None)
    buf = bestla._aligned_buffer(size)
    L.nad_host_cache_clear()

    def fwd(b):
        out = np.zeros((m, n), np.float32)
        L.nad_clear_error()
        L.bestla_f32f32_forward(vp(A), vp(b), vp(out), m, n, k, k, n, None)
        assert _lib.last_error() == ""
        return out
    for seed in (1, 2):  # same scales, new codes, through the pack API
        q = np.random.default_rng(seed).integers(-8, 8, size=(k, n), dtype=np.int8)
        assert L.BTLAGemmPackB(vp(buf), vp(q), vp(s), None, n, k, n, 128, S4, F32, False, 4, None, None)
        assert _rel_err(fwd(buf), oracle.forward(A, buf, n, k)) <= 2e-5, seed
    # another writer flips ONE code byte (no API call): evict, and the forward follows it
    info = bestla.blob_info(buf)
    buf[info["q_off"] + 7] ^= 0x11
    L.nad_host_cache_evict(vp(buf))
    assert _rel_err(fwd(buf), oracle.forward(A, buf, n, k)) <= 2e-5
    # LRU bound: room for two of these weights -> at most two entries, every forward still exact
    e, b = C.c_size_t(0), C.c_size_t(0)
    L.nad_host_cache_stats(C.byref(e), C.byref(b))
    one = b.value
    assert e.value == 1 and one > 0
    prev = L.nad_host_cache_set_limit(2 * one + 16)
    try:
        blobs = [_wb(oracle, n, k, 40 + i) for i in range(4)]
        for rnd in range(2):
            for bl in blobs:
                assert _rel_err(fwd(bl), oracle.forward(A, bl, n, k)) <= 2e-5
                L.nad_host_cache_stats(C.byref(e), C.byref(b))
                assert e.value <= 2 and b.value <= 2 * one + 16
    finally:
        L.nad_host_cache_set_limit(prev)
        L.nad_host_cache_clear()


def test_qkv_prefill_mixed_formats_keep_their_activations(oracle):
    """the shared fp16 activation copy of a QKV prefill must not be reused after a weight that rewrote the
    workspace (other K tile: int4 / int2 / int4; or an int8-compute weight in the middle)."""
    m, k = 64, 1024
    bq = _blob(oracle, 256, k, 128, S4, F16, False, 1, seed=71)
    bk = _blob(oracle, 128, k, 64, S2, F16, False, 1, seed=72)
    bv = _blob(oracle, 128, k, 128, S4, F16, False, 1, seed=73)
    bi = _blob(oracle, 128, k, 32, S4, F32, False, 4, seed=74)      # integer core: int8-capable
    x = torch.from_numpy(np.random.default_rng(9).uniform(-1, 1, size=(m, k)).astype(np.float32)).cuda()
    xa = x.cpu().numpy()
    wq, wk, wv, wi = (bestla.DeviceWeight(b) for b in (bq, bk, bv, bi))
    oq, ok, ov = bestla.qkv_forward(x, wq, wk, wv)
    for o, b, n in ((oq, bq, 256), (ok, bk, 128), (ov, bv, 128)):
        assert _rel_err(o.cpu().numpy(), oracle.forward(xa, b, n, k)) <= 1e-3
    wi.set_compute(bestla.COMPUTE_INT8)
    assert wi.compute == bestla.COMPUTE_INT8 and wq.compute == bestla.COMPUTE_FP
    oq, oi, ov = bestla.qkv_forward(x, wq, wi, wv)
    assert _rel_err(oq.cpu().numpy(), oracle.forward(xa, bq, 256, k)) <= 1e-3
    assert _rel_err(oi.cpu().numpy(), oracle.forward_int8(xa, bi, 128, k)) <= 1e-5
    assert _rel_err(ov.cpu().numpy(), oracle.forward(xa, bv, 128, k)) <= 1e-3


@pytest.mark.parametrize("m", [1, 4, 64])
def test_per_weight_compute_mode(oracle, m):
    """the int8-compute arithmetic is chosen per weight (the reference: per blob core,
    bestla_gemm.cpp:516-616) and per thread, not only by a process-global switch; a fused decode QKV whose weights
    resolve to different arithmetic runs each in its own."""
    k = 512
    b8 = [_blob(oracle, 128, k, 32, S4, F32, False, 4, seed=80 + i) for i in range(3)]   # integer-core blobs
    ws = [bestla.DeviceWeight(b) for b in b8]
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, k)).astype(np.float32)
    x = torch.from_numpy(A).cuda()
    assert bestla.get_compute_mode() == bestla.COMPUTE_FP
    assert all(w.compute == bestla.COMPUTE_FP for w in ws)
    ws[1].set_compute(bestla.COMPUTE_INT8)
    outs = bestla.qkv_forward(x, *ws)
    for i, (o, b) in enumerate(zip(outs, b8)):
        ref = oracle.forward_int8(A, b, 128, k) if i == 1 else oracle.forward(A, b, 128, k)
        assert _rel_err(o.cpu().numpy(), ref) <= (1e-5 if i == 1 else (2e-5 if m <= 16 else 1e-3)), i
    # the thread override switches the weights that follow it; the per-weight setting still wins
    ws[0].set_compute(bestla.COMPUTE_FP)
    bestla.set_thread_compute_mode(bestla.COMPUTE_INT8)
    try:
        assert [w.compute for w in ws] == [bestla.COMPUTE_FP, bestla.COMPUTE_INT8, bestla.COMPUTE_INT8]
        y2 = ws[2].forward(x).cpu().numpy()
        assert _rel_err(y2, oracle.forward_int8(A, b8[2], 128, k)) <= 1e-5
    finally:
        bestla.set_thread_compute_mode(None)
    assert ws[2].compute == bestla.COMPUTE_FP
    ws[1].set_compute(None)
    assert ws[1].compute == bestla.COMPUTE_FP
