"""GPU parity: the HIP path through the C-ABI vs the oracle (fp64 GEMM on the reference's dequantized weights).

Tolerances (north_star: 1e-3 relative, bit-exact for packing/indexing):
  * repack / unpack from the device tile layout: bit-exact vs the oracle's dequantization.
  * decode path (M <= 16, fp32 activations, hi/lo fp16 split):  max|y - ref| <= 2e-5 * max|ref|
  * prefill path (M > 16, activations rounded to fp16):          max|y - ref| <= 1e-3 * max|ref|
  * fp16 / bf16 activations (exact in fp16 up to range):          max|y - ref| <= 2e-5 * max|ref|
"""
import ctypes as C

import numpy as np
import pytest

from tests.conftest import gpu_available
from tests.oracle_lib import BF16, F16, F32, S2, S4, S8

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from neural_amd import _lib, bestla

TOL_DECODE = 2e-5
TOL_PREFILL = 1e-3


def _rel_err(y, ref):
    return float(np.abs(y.astype(np.float64) - ref).max() / max(np.abs(ref).max(), 1e-30))


def _blob(oracle, n, k, bs, qt, st, asym, comp, seed, gidx=False):
    rng = np.random.default_rng(seed)
    if not gidx:
        W = rng.uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
        core = oracle.lib.orc_select_core(comp, qt, bs, int(asym), 0)
        return oracle.quant_pack(W, n, k, bs, qt, st, asym, core, is_trans=True)
    bits = {S4: 4, S2: 2, S8: 8}[qt]
    q = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), size=(k, n)).astype(np.int8)
    s = rng.uniform(0.001, 0.005, size=(-(-k // bs), n)).astype(np.float32)
    z = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), size=s.shape).astype(np.int8) if asym else None
    g_idx = rng.permutation(np.arange(k) // bs).astype(np.int32)
    core = oracle.lib.orc_select_core(comp, qt, bs, int(asym), 0)
    return oracle.pack_q(q, s, z, n, k, bs, qt, st, asym, core, g_idx)


LAYOUTS = [
    # n, k, bs, qtype, stype, asym, comp
    (64, 256, 32, S4, F32, False, 1),
    (100, 384, 128, S4, BF16, True, 4),     # PACK_ROW 4 (AMX-int8 kblock), ragged N
    (96, 512, 64, S4, F16, False, 2),       # PACK_ROW 2 (AMX-bf16)
    (80, 512, 64, S2, F32, True, 1),
    (48, 256, 256, S2, BF16, False, 4),
    (72, 192, 64, S8, F32, False, 1),
    (40, 256, 128, S8, BF16, False, 4),
    (50, 4096, 4096, S4, F32, False, 1),    # per-channel
]


@pytest.mark.parametrize("cfg", LAYOUTS)
def test_repack_bit_exact(oracle, cfg):
    n, k, bs, qt, st, asym, comp = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, comp, seed=n + k)
    w = bestla.DeviceWeight(blob)
    np.testing.assert_array_equal(w.unpack().view(np.uint32), oracle.unpack_fp32(blob).view(np.uint32))


FWD = [
    # m, n, k, bs, qtype, stype, asym, comp
    (1, 64, 256, 32, S4, F32, False, 1),
    (1, 4096, 4096, 128, S4, F16, False, 4),
    (2, 100, 384, 128, S4, BF16, True, 4),
    (3, 96, 512, 64, S4, F16, False, 2),
    (4, 80, 512, 64, S2, F32, True, 1),
    (5, 48, 256, 256, S2, BF16, False, 4),
    (8, 72, 192, 64, S8, F32, False, 1),
    (9, 40, 256, 128, S8, BF16, True, 1),
    (16, 160, 1024, 32, S4, F32, True, 1),
    (1, 50, 4096, 4096, S4, F32, False, 1),
    (17, 64, 256, 32, S4, F32, False, 1),
    (33, 100, 384, 128, S4, BF16, True, 4),
    (128, 256, 512, 64, S2, F32, False, 1),
    (130, 72, 192, 64, S8, F32, True, 1),
    (300, 150, 640, 128, S4, F16, False, 4),
]


@pytest.mark.parametrize("cfg", FWD)
def test_forward_parity(oracle, cfg):
    m, n, k, bs, qt, st, asym, comp = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, comp, seed=m * 7 + n)
    w = bestla.DeviceWeight(blob)
    rng = np.random.default_rng(m + n + k)
    A = rng.uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    ref = oracle.forward(A, blob, n, k).astype(np.float64)
    y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
    tol = TOL_DECODE if m <= 16 else TOL_PREFILL
    assert _rel_err(y, ref) <= tol, (_rel_err(y, ref), tol)


@pytest.mark.parametrize("m", [1, 4, 12, 40])
def test_act_order_shuffle(oracle, m):
    n, k, bs = 96, 512, 64
    blob = _blob(oracle, n, k, bs, S4, F32, True, 4, seed=5, gidx=True)
    w = bestla.DeviceWeight(blob)
    assert w.has_shuffle
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, k)).astype(np.float32)
    ref = oracle.forward(A, blob, n, k)
    y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
    assert _rel_err(y, ref) <= (TOL_DECODE if m <= 16 else TOL_PREFILL)


@pytest.mark.parametrize("m", [1, 7, 64])
def test_strides_and_half_activations(oracle, m):
    n, k, bs = 112, 768, 128
    blob = _blob(oracle, n, k, bs, S4, BF16, True, 4, seed=9)
    w = bestla.DeviceWeight(blob)
    rng = np.random.default_rng(m)
    big = rng.uniform(-1, 1, size=(m, k + 24)).astype(np.float32)
    A = big[:, 8:8 + k]
    x = torch.from_numpy(big).cuda()[:, 8:8 + k]           # lda = k + 24, unaligned start
    out = torch.zeros((m, n + 5), dtype=torch.float32, device="cuda")[:, :n]
    w.forward(x, out=out)
    ref = oracle.forward(np.ascontiguousarray(A), blob, n, k)
    assert _rel_err(out.cpu().numpy(), ref) <= (TOL_DECODE if m <= 16 else TOL_PREFILL)
    for dt in (torch.float16, torch.bfloat16):
        xh = torch.from_numpy(np.ascontiguousarray(A)).cuda().to(dt)
        ref_h = oracle.forward(xh.float().cpu().numpy(), blob, n, k)
        y = w.forward(xh).cpu().numpy()
        assert _rel_err(y, ref_h) <= (TOL_DECODE if m <= 16 or dt == torch.float16 else TOL_PREFILL)


@pytest.mark.parametrize("m", [1, 3, 48])
def test_epilogues_bias_residual(oracle, m):
    n, k = 64, 256
    blob = _blob(oracle, n, k, 32, S4, F32, False, 1, seed=1)
    w = bestla.DeviceWeight(blob)
    rng = np.random.default_rng(2)
    A = rng.uniform(-1, 1, size=(m, k)).astype(np.float32)
    b = rng.uniform(-1, 1, size=(n,)).astype(np.float32)
    r = rng.uniform(-1, 1, size=(m, n)).astype(np.float32)
    ref = oracle.forward(A, blob, n, k).astype(np.float64)
    x = torch.from_numpy(A).cuda()
    y = w.forward(x, epilogue=bestla.EPI_BIAS, bias=torch.from_numpy(b).cuda()).cpu().numpy()
    tol = TOL_DECODE if m <= 16 else TOL_PREFILL
    assert _rel_err(y, ref + b) <= tol
    y = w.forward(x, epilogue=bestla.EPI_RES_ADD, residual=torch.from_numpy(r).cuda()).cpu().numpy()
    assert _rel_err(y, ref + r) <= tol


@pytest.mark.parametrize("m", [1, 5, 20])
def test_fused_qkv(oracle, m):
    k = 512
    blobs = [_blob(oracle, n, k, 128, S4, F32, False, 4, seed=i) for i, n in enumerate((128, 64, 64))]
    ws = [bestla.DeviceWeight(b) for b in blobs]
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, k)).astype(np.float32)
    q, kk, v = bestla.qkv_forward(torch.from_numpy(A).cuda(), *ws)
    for y, b, n in zip((q, kk, v), blobs, (128, 64, 64)):
        ref = oracle.forward(A, b, n, k)
        assert _rel_err(y.cpu().numpy(), ref) <= (TOL_DECODE if m <= 16 else TOL_PREFILL)


@pytest.mark.parametrize("m", [1, 4, 24])
@pytest.mark.parametrize("act", ["silu", "gelu"])
def test_fused_ffn(oracle, m, act):
    fin, fmid, fout = 256, 384, 256
    b1 = _blob(oracle, fmid, fin, 64, S4, BF16, False, 4, seed=21)
    b3 = _blob(oracle, fmid, fin, 64, S4, BF16, False, 4, seed=23)
    b2 = _blob(oracle, fout, fmid, 64, S4, BF16, False, 4, seed=22)
    w1, w2, w3 = (bestla.DeviceWeight(b) for b in (b1, b2, b3))
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, fin)).astype(np.float32)
    y = bestla.ffn_forward(torch.from_numpy(A).cuda(), w1, w2, w3, act=act).cpu().numpy()
    h1 = oracle.forward(A, b1, fmid, fin).astype(np.float64)
    h3 = oracle.forward(A, b3, fmid, fin).astype(np.float64)
    if act == "silu":
        t1 = h1 / (1 + np.exp(-h1))
    else:
        t1 = 0.5 * h1 * (1 + np.tanh(0.7978845834732056 * (h1 + 0.044714998453855515 * h1 ** 3)))
    ref = oracle.forward((t1 * h3).astype(np.float32), b2, fout, fmid)
    assert _rel_err(y, ref) <= (1e-4 if m <= 16 else TOL_PREFILL)


def test_host_abi_f32f32_forward(oracle):
    """bestla_f32f32_forward with HOST pointers (the NE CPU-tensor path) runs on the GPU and matches the oracle."""
    L = _lib.lib()
    n, k, m = 96, 512, 3
    blob = _blob(oracle, n, k, 128, S4, F32, False, 4, seed=3)
    A = np.random.default_rng(0).uniform(-1, 1, size=(m, k)).astype(np.float32)
    out = np.zeros((m, n), np.float32)
    L.nad_clear_error()
    vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    L.bestla_f32f32_forward(vp(A), vp(blob), vp(out), m, n, k, k, n, None)
    assert _lib.last_error() == ""
    assert _rel_err(out, oracle.forward(A, blob, n, k)) <= TOL_DECODE
    # BTLAGemmBatchDriver over two problems
    blob2 = _blob(oracle, n, k, 32, S2, BF16, True, 1, seed=4)
    out2 = np.zeros((m, n), np.float32)
    P = type("P", (C.Structure,), {"_fields_": [("A", C.c_void_p), ("B", C.c_void_p), ("C", C.c_void_p),
                                                 ("lda", C.c_int), ("ldc", C.c_int)]})
    arr = (P * 2)(P(vp(A).value, vp(blob).value, vp(out).value, k, n), P(vp(A).value, vp(blob2).value,
                                                                          vp(out2).value, k, n))
    assert L.BTLAGemmBatchDriver(m, n, k, 2, C.cast(arr, C.c_void_p), None, None)
    assert _rel_err(out2, oracle.forward(A, blob2, n, k)) <= TOL_DECODE


def test_pure_c_abi_device_path(oracle):
    """bestla_create_device -> bestla_device_malloc -> bestla_device_load_storage -> bestla_device_f32f32_forward,
    exactly the call sequence of ne_layers.c:7285-7311 / model_files.h:1515-1525, with no torch buffers."""
    L = _lib.lib()
    vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    dev = L.bestla_create_device(False)
    q = L.bestla_get_device_queue(dev)
    n, k, m = 200, 1024, 2
    blob = _blob(oracle, n, k, 128, S4, F32, True, 1, seed=8)
    dptr = L.bestla_device_malloc(blob.size, q)
    desc = (C.c_uint8 * L.bestla_device_storage_size())()
    L.nad_clear_error()
    L.bestla_device_load_storage(vp(blob), desc, dptr, q)
    assert _lib.last_error() == ""
    A = np.random.default_rng(1).uniform(-1, 1, size=(m, k)).astype(np.float32)
    dA = L.bestla_device_malloc(A.nbytes, q)
    dY = L.bestla_device_malloc(m * n * 4, q)
    L.bestla_device_memcpy_sync(dA, vp(A), A.nbytes, q)
    L.bestla_device_f32f32_forward(dA, desc, dY, m, n, k, k, n, None, q)
    Y = np.zeros((m, n), np.float32)
    L.bestla_device_memcpy_sync(vp(Y), dY, Y.nbytes, q)
    assert _lib.last_error() == ""
    assert _rel_err(Y, oracle.forward(A, blob, n, k)) <= TOL_DECODE
    # wrong shape -> loud error, no silent skip
    L.bestla_device_f32f32_forward(dA, desc, dY, m, n + 1, k, k, n, None, q)
    assert "shape mismatch" in _lib.last_error()
    for p in (dptr, dA, dY):
        L.bestla_device_free(p, q)
    L.bestla_release_device(dev)


def test_full_size_decode_and_prefill_properties(oracle):
    """BASELINE shapes: K=N=4096 int4 g128 at M=1 (full oracle) and M=2048 (oracle on sampled rows)."""
    n = k = 4096
    blob = _blob(oracle, n, k, 128, S4, F16, False, 4, seed=42)
    w = bestla.DeviceWeight(blob)
    rng = np.random.default_rng(0)
    A1 = rng.uniform(-0.5, 0.5, size=(1, k)).astype(np.float32)
    y1 = w.forward(torch.from_numpy(A1).cuda()).cpu().numpy()
    assert _rel_err(y1, oracle.forward(A1, blob, n, k)) <= TOL_DECODE
    A = rng.uniform(-0.5, 0.5, size=(2048, k)).astype(np.float32)
    y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
    rows = rng.choice(2048, size=24, replace=False)
    ref = oracle.forward(A[rows], blob, n, k)
    assert _rel_err(y[rows], ref) <= TOL_PREFILL
    # linearity (size-independent property): W(2a) = 2 W(a) up to fp16 subnormal rounding of the lo part
    y2 = w.forward(torch.from_numpy(2 * A1).cuda()).cpu().numpy()
    assert _rel_err(y2, 2.0 * y1.astype(np.float64)) <= 1e-6


def test_deterministic_and_graph_capturable(oracle):
    n, k = 4096, 4096
    w = bestla.DeviceWeight.synthetic(4, n, k, 128, "fp16")
    x = torch.randn(1, k, device="cuda")
    y0 = w.forward(x).clone()
    g = torch.cuda.CUDAGraph()
    out = torch.empty_like(y0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        w.forward(x, out=out)
        with torch.cuda.graph(g, stream=s):
            w.forward(x, out=out)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, y0)


GEMV_GEOM = [
    # m, n, k, bs, qtype, stype, asym, comp
    (1, 4096, 4096, 128, S4, F16, False, 4),
    (1, 1000, 4096, 256, S4, BF16, True, 4),   # a group spans 2 tiles: wave ranges split groups
    (2, 200, 1024, 64, S4, F32, True, 1),      # 2 groups per tile
    (3, 320, 2048, 32, S4, F16, False, 2),     # 4 groups per tile
    (1, 96, 11008, 128, S4, F16, False, 4),    # Llama down K
    (5, 130, 2048, 128, S2, BF16, True, 1),
    (8, 72, 768, 64, S8, F32, True, 4),
    (12, 64, 512, 128, S4, F32, False, 1),     # M 9..16: two MFMA passes (hi, lo)
    (1, 50, 4096, 4096, S4, F32, True, 1),     # per-channel
]


@pytest.mark.parametrize("cfg", GEMV_GEOM)
@pytest.mark.parametrize("geom", [(None, None), ("1", "16"), ("3", "5"), ("7", "1"), ("64", "8")])
def test_gemv_stream_geometry(oracle, knob, cfg, geom):
    """The persistent stripe-stream GEMV with forced grids / wave counts: workgroups owning many stripes, wave ranges
    crossing stripe and group boundaries, single-wave workgroups.  Same bar as the default launch."""
    grid, waves = geom
    knob("NAD_MID_MAX_M", "0")  # M >= 8 would take the mid-M kernel (tests/test_mid_gpu.py)
    if grid:
        knob("NAD_GEMV_GRID", grid)
        knob("NAD_GEMV_WAVES", waves)
    m, n, k, bs, qt, st, asym, comp = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, comp, seed=m + n + bs)
    w = bestla.DeviceWeight(blob)
    A = np.random.default_rng(n).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    ref = oracle.forward(A, blob, n, k)
    y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
    assert _rel_err(y, ref) <= TOL_DECODE


M1_SLICES = [
    # n, k, bs, qtype, stype, asym, act dtype: M = 1 launches of woq_gemv_m1_kernel with 2-tile K-slices (more waves)
    (4096, 4096, 128, S4, F16, False, "f32"),
    (1000, 4096, 256, S4, BF16, True, "f16"),
    (320, 2048, 64, S4, F32, True, "bf16"),  # 2 groups per tile, 8 waves
    (520, 3968, 128, S4, F16, False, "f32"),  # K tail: 31 tiles, the last wave's slice half out of range
    (1024, 4096, 64, S2, F16, False, "f16"),  # int2 g64 (Mistral): 4 groups per tile, 8 waves instead of 4
    (264, 2048, 128, S2, BF16, True, "f32"),
    # long K: up to 4 slices per wave (Mistral's down, 4096 x 14336 int4 g64, at 7 waves)
    (256, 14336, 64, S4, F16, False, "f16"),
    (200, 12288, 64, S4, BF16, True, "f32"),
    (128, 20480, 64, S2, F16, False, "bf16"),
]


@pytest.mark.parametrize("cfg", M1_SLICES)
@pytest.mark.parametrize("grid", [None, "1", "7"])
def test_gemv_m1_two_tile_slices(oracle, knob, cfg, grid):
    """M = 1 with 2-tile K-slices (one per wave, up to 16 waves) against the oracle,
    and within 1e-6 of a 4-tile-slice launch (a forced wave count takes 4-tile slices; only the partial-sum order
    differs).  Forced grids make
    workgroups stream many stripes through the 3-stage ring."""
    n, k, bs, qt, st, asym, adt = cfg
    if grid:
        knob("NAD_GEMV_GRID", grid)
    blob = _blob(oracle, n, k, bs, qt, st, asym, 4, seed=n + k)
    w = bestla.DeviceWeight(blob)
    A = np.random.default_rng(k).uniform(-0.5, 0.5, size=(1, k)).astype(np.float32)
    xa = torch.from_numpy(A).cuda().to(dict(f32=torch.float32, f16=torch.float16, bf16=torch.bfloat16)[adt])
    ref = oracle.forward(xa.float().cpu().numpy(), blob, n, k)
    y2 = w.forward(xa).cpu().numpy()
    knob("NAD_GEMV_WAVES", "16")
    y4 = w.forward(xa).cpu().numpy()
    assert _rel_err(y2, ref) <= TOL_DECODE
    assert _rel_err(y2, y4) <= 1e-6


@pytest.mark.parametrize("geom", [(None, None), ("2", "3"), ("5", "16")])
def test_gemv_stream_fused(oracle, knob, geom):
    """QKV (three weights in one stream) and the dual gate/up stream with SiLU*mul under forced geometries."""
    grid, waves = geom
    if grid:
        knob("NAD_GEMV_GRID", grid)
        knob("NAD_GEMV_WAVES", waves)
    k = 1024
    blobs = [_blob(oracle, n, k, 128, S4, F16, False, 4, seed=i) for i, n in enumerate((256, 80, 80))]
    ws = [bestla.DeviceWeight(b) for b in blobs]
    A = np.random.default_rng(3).uniform(-1, 1, size=(1, k)).astype(np.float32)
    for y, b, n in zip(bestla.qkv_forward(torch.from_numpy(A).cuda(), *ws), blobs, (256, 80, 80)):
        assert _rel_err(y.cpu().numpy(), oracle.forward(A, b, n, k)) <= TOL_DECODE
    fin, fmid, fout = 1024, 688, 512
    b1 = _blob(oracle, fmid, fin, 128, S4, F16, False, 4, seed=31)
    b3 = _blob(oracle, fmid, fin, 128, S4, F16, False, 4, seed=33)
    b2 = _blob(oracle, fout, fmid, 128, S4, F16, False, 4, seed=32)
    w1, w2, w3 = (bestla.DeviceWeight(b) for b in (b1, b2, b3))
    y = bestla.ffn_forward(torch.from_numpy(A).cuda(), w1, w2, w3, act="silu").cpu().numpy()
    h1 = oracle.forward(A, b1, fmid, fin).astype(np.float64)
    h3 = oracle.forward(A, b3, fmid, fin).astype(np.float64)
    ref = oracle.forward((h1 / (1 + np.exp(-h1)) * h3).astype(np.float32), b2, fout, fmid)
    assert _rel_err(y, ref) <= 1e-4


@pytest.mark.parametrize("cfg", FWD[:9])
def test_legacy_skinny_kernel(oracle, knob, cfg):
    """The per-stripe woq_skinny_kernel (used when the stream GEMV is not eligible) keeps its own parity."""
    knob("NAD_GEMV_DISABLE", "1")
    m, n, k, bs, qt, st, asym, comp = cfg
    blob = _blob(oracle, n, k, bs, qt, st, asym, comp, seed=m * 7 + n)
    w = bestla.DeviceWeight(blob)
    A = np.random.default_rng(m + n + k).uniform(-0.5, 0.5, size=(m, k)).astype(np.float32)
    ref = oracle.forward(A, blob, n, k)
    y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
    assert _rel_err(y, ref) <= TOL_DECODE


@pytest.mark.parametrize("m", [1, 3, 40])
@pytest.mark.parametrize("kinds", ["int2_policy", "all_differ"])
def test_qkv_mixed_formats(oracle, m, kinds):
    """QKV over weights of different formats and N (the Mistral int2 policy: Q, K int2 g64, V int4 g64 with 4x fewer
    rows): decode runs one stream launch per run of same-format weights ({Q, K} + {V}), each output exactly as alone."""
    k = 1024
    if kinds == "int2_policy":
        spec = [(512, 64, S2, False), (128, 64, S2, False), (128, 64, S4, False)]
    else:
        spec = [(256, 128, S4, True), (128, 64, S2, False), (128, 128, S4, False)]
    blobs = [_blob(oracle, n, k, bs, qt, F16, asym, 4, seed=70 + i) for i, (n, bs, qt, asym) in enumerate(spec)]
    ws = [bestla.DeviceWeight(b) for b in blobs]
    A = np.random.default_rng(m).uniform(-1, 1, size=(m, k)).astype(np.float32)
    x = torch.from_numpy(A).cuda()
    for y, w, b, (n, *_) in zip(bestla.qkv_forward(x, *ws), ws, blobs, spec):
        assert _rel_err(y.cpu().numpy(), oracle.forward(A, b, n, k)) <= (TOL_DECODE if m <= 16 else TOL_PREFILL)
        assert torch.equal(y, w.forward(x))    # fusion does not change a single bit


@pytest.mark.parametrize("st", [F32, BF16, F16])
@pytest.mark.parametrize("cfg", [(1024, 4096, 64, False, "f32"), (528, 2048, 128, True, "f16"),
                                 (300, 1024, 256, False, "bf16"), (4096, 4096, 64, False, "f16")])
def test_gemv_m1_int2_every_scale_type(oracle, st, cfg):
    """Round 6: the int2 M = 1 instantiations take the scale type as a template parameter (woq_gemv.hip
    gemv_m1_launch4, compiled as woq_gemv_b2.o).  Every scale type x group layout (4 / 2 / 1 groups per 256-deep tile)
    against the oracle, and the batched form of the same kernel bit-identical to single launches."""
    n, k, bs, asym, adt = cfg
    blob = _blob(oracle, n, k, bs, S2, st, asym, 4, seed=n + bs + st)
    w = bestla.DeviceWeight(blob)
    assert w.plan(1, {"f32": "fp32", "f16": "fp16", "bf16": "bf16"}[adt])["kernel"] == "woq_gemv_m1_kernel"
    A = np.random.default_rng(n + k).uniform(-0.5, 0.5, size=(1, k)).astype(np.float32)
    xa = torch.from_numpy(A).cuda().to(dict(f32=torch.float32, f16=torch.float16, bf16=torch.bfloat16)[adt])
    ref = oracle.forward(xa.float().cpu().numpy(), blob, n, k)
    y = w.forward(xa).cpu().numpy()
    assert _rel_err(y, ref) <= TOL_DECODE
    if adt == "f32":
        xs = [torch.from_numpy(np.random.default_rng(i).uniform(-1, 1, size=(k,)).astype(np.float32)).cuda()
              for i in range(3)]
        ys = [torch.empty(n, device="cuda") for _ in xs]
        bestla.Batch([(w, x, yy) for x, yy in zip(xs, ys)]).run()
        for x, yy in zip(xs, ys):
            assert torch.equal(yy, w.forward(x.view(1, k)).view(n))
