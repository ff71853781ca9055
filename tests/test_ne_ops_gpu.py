"""GPU parity of the device half of the graph seam (bestla_device_{mul,add,elewise,rms_norm,rope,dup,mha}_f32) and the
host helpers (bestla_layernormalization / bestla_mul / bestla_add) through the C-ABI, with ne_tensor structs laid out
as the reference's ne.h.  References are numpy restatements of the SYCL implementations they replace
(core/layers/ne_bestla_sycl.cpp:173-880, cited per test) and of kernel_ref.h:2199-2240 (layernorm), in float64.
Tolerance: 1e-5 relative (fp32 elementwise / row reductions; RoPE and attention use expf/sinf/cosf)."""
import ctypes as C

import numpy as np
import pytest

from tests.conftest import gpu_available
from tests.ne_structs import NE_TYPE_F16, NE_TYPE_I32, OP, params, set_op_params_f32, tensor

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from neural_amd import _lib

TOL = 1e-5


def _rel(a, b):
    b = np.asarray(b, np.float64)
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def _run(fn, *args):
    torch.cuda.synchronize()
    fn(*args)
    torch.cuda.synchronize()


def _t(x, **kw):
    """ne_tensor over a torch tensor (ne reversed from torch's shape; strides in bytes)."""
    ne = list(reversed(x.shape))
    nb = list(reversed([s * x.element_size() for s in x.stride()]))
    nb += [nb[-1] * ne[-1]] * (4 - len(nb))
    return tensor(ne, nb, data=x.data_ptr(), **kw)


@pytest.mark.parametrize("op", ["mul", "add"])
def test_binary_broadcast(op):
    """ne_bestla_sycl.cpp:173-281: dst = src0 op src1, src1 broadcast over rows by modulo."""
    L = _lib.lib()
    rng = np.random.default_rng(1)
    a = torch.from_numpy(rng.standard_normal((3, 5, 96)).astype(np.float32)).cuda()
    for bshape in ((1, 1, 96), (1, 5, 96), (3, 5, 96)):
        b = torch.from_numpy(rng.standard_normal(bshape).astype(np.float32)).cuda()
        out = torch.empty_like(a)
        p = params()
        f = L.bestla_device_mul_f32 if op == "mul" else L.bestla_device_add_f32
        _run(f, C.byref(p), C.byref(_t(a)), C.byref(_t(b)), C.byref(_t(out)))
        ref = a.cpu().numpy() * b.cpu().numpy() if op == "mul" else a.cpu().numpy() + b.cpu().numpy()
        assert _rel(out.cpu().numpy(), ref) <= TOL
    # INIT / FINALIZE phases do nothing (ne_bestla_sycl.cpp:175-177)
    out = torch.zeros_like(a)
    _run(L.bestla_device_add_f32, C.byref(params(phase=0)), C.byref(_t(a)), C.byref(_t(a)), C.byref(_t(out)))
    assert float(out.abs().max()) == 0.0


def test_elewise_silu_and_copy():
    L = _lib.lib()
    x = torch.randn(4, 1000, device="cuda")
    for op, ref in ((OP["SILU"], lambda v: v / (1 + np.exp(-v))), (OP["NONE"], lambda v: v)):
        out = torch.empty_like(x)
        _run(L.bestla_device_elewise_f32, C.byref(params()), C.byref(_t(x)), C.byref(_t(out, op=op)))
        assert _rel(out.cpu().numpy(), ref(x.cpu().numpy().astype(np.float64))) <= TOL


def test_rms_norm_rows():
    """ne_bestla_sycl.cpp:311-383: y = x / sqrt(mean(x^2) + eps) per row; eps from op_params."""
    L = _lib.lib()
    x = torch.randn(2, 3, 4096, device="cuda") * 3
    out = torch.empty_like(x)
    t = _t(out)
    set_op_params_f32(t, [1e-5])
    _run(L.bestla_device_rms_norm_f32, C.byref(params()), C.byref(_t(x)), C.byref(t))
    xv = x.cpu().numpy().astype(np.float64)
    ref = xv / np.sqrt((xv ** 2).mean(-1, keepdims=True) + 1e-5)
    assert _rel(out.cpu().numpy(), ref) <= TOL


def _rope_ref(x, n_past, n_dims, freq_base, freq_scale_inv, n_orig_ctx, ext_factor, attn_factor, beta_fast, beta_slow):
    """ne_bestla_sycl.cpp:436-536 (+ ne_layers.c:9225-9234) in float64; x [b][s][h][d]"""
    freq_scale = 1.0 / freq_scale_inv
    theta_scale = freq_base ** (-2.0 / n_dims)

    def corr(n_rot):
        return n_dims * np.log(n_orig_ctx / (n_rot * 2 * np.pi)) / (2 * np.log(freq_base))
    c0 = max(0.0, np.floor(corr(beta_fast)))
    c1 = min(n_dims - 1.0, np.ceil(corr(beta_slow)))
    out = np.empty_like(x, dtype=np.float64)
    B, S, H, D = x.shape
    for s in range(S):
        theta_base = float(n_past + s)
        for i0 in range(0, D, 2):
            theta_interp = freq_scale * theta_base
            theta, mscale = theta_interp, attn_factor
            if ext_factor != 0:
                y = (i0 // 2 - c0) / max(0.001, c1 - c0)
                ramp = 1 - min(1, max(0, y))
                mix = ramp * ext_factor
                theta = theta_interp * (1 - mix) + theta_base * mix
                mscale *= 1 + 0.1 * np.log(1 / freq_scale)
            c, sn = np.cos(theta) * mscale, np.sin(theta) * mscale
            theta_base *= theta_scale
            x0, x1 = x[:, s, :, i0].astype(np.float64), x[:, s, :, i0 + 1].astype(np.float64)
            out[:, s, :, i0] = x0 * c - x1 * sn
            out[:, s, :, i0 + 1] = x0 * sn + x1 * c
    return out


@pytest.mark.parametrize("ext", [0.0, 1.0])
def test_rope_yarn(ext):
    L = _lib.lib()
    B, S, H, D = 1, 5, 4, 128
    x = torch.randn(B, S, H, D, device="cuda")
    out = torch.empty_like(x)
    pv = np.array([7, D, 0, S, 0, 0, 0, 0], np.int32)     # n_past, n_dims, mode, prompt_size, n_keep (host tensor)
    ptens = tensor([5], ttype=NE_TYPE_I32, data=pv.ctypes.data, backend=0)
    t = _t(out)
    fp = [10000.0, 2.0, 4096.0, ext, 1.0, 32.0, 1.0, 1.0]  # base, 1/freq_scale, n_orig_ctx, ext, attn, b_fast, b_slow
    set_op_params_f32(t, fp)
    _run(L.bestla_device_rope_f32, C.byref(params()), C.byref(_t(x)), C.byref(ptens), C.byref(t))
    ref = _rope_ref(x.cpu().numpy(), 7, D, fp[0], fp[1], int(fp[2]), fp[3], fp[4], fp[5], fp[6])
    assert _rel(out.cpu().numpy(), ref) <= 2e-5


def test_dup_strided_to_f16_and_f32():
    """ne_bestla_sycl.cpp:538-592: strided f32 source (a transpose view) into contiguous f32 / f16."""
    L = _lib.lib()
    base = torch.randn(64, 48, device="cuda")
    src = base.t()                                  # [48][64] view, non-contiguous
    for dt, ttype, tol in ((torch.float32, 0, 0.0), (torch.float16, NE_TYPE_F16, 1e-3)):
        out = torch.empty(48, 64, dtype=dt, device="cuda")
        _run(L.bestla_device_dup_f32, C.byref(params()), C.byref(_t(src)), C.byref(_t(out, ttype=ttype)))
        ref = src.cpu().numpy()
        if dt == torch.float16:
            ref = ref.astype(np.float16)
        assert _rel(out.float().cpu().numpy(), ref) <= max(tol, 0.0) + 1e-7


def _mha_ref(Q, K, V, scale, seq_all):
    """MHA::forward1 (ne_bestla_sycl.cpp:704-803): Q [b][s][h][d], K [b][h][n_ctx][d], V^T [b][h][d][n_ctx]"""
    B, S, H, D = Q.shape
    n_past = seq_all - S
    O = np.zeros((B, S, H, D))
    for b in range(B):
        for s in range(S):
            for h in range(H):
                lim = s + n_past + 1 if S > 1 else seq_all
                sc = K[b, h, :lim].astype(np.float64) @ Q[b, s, h].astype(np.float64) * scale
                p = np.exp(sc - sc.max())
                p /= p.sum()
                O[b, s, h] = V[b, h, :, :lim].astype(np.float64) @ p
    return O


@pytest.mark.parametrize("seq,seq_all", [(1, 37), (1, 300), (6, 70)])
def test_mha(seq, seq_all):
    L = _lib.lib()
    B, H, D, n_ctx = 2, 4, 128, 320
    rng = np.random.default_rng(seq_all)
    Q = rng.standard_normal((B, seq, H, D)).astype(np.float32)
    K = rng.standard_normal((B, H, n_ctx, D)).astype(np.float32)
    V = rng.standard_normal((B, H, D, n_ctx)).astype(np.float32)
    q, k, v = (torch.from_numpy(a).cuda() for a in (Q, K, V))
    o = torch.zeros(B, seq, H, D, device="cuda")
    kt = tensor([D, seq_all, H, B], data=k.data_ptr())
    vt = tensor([seq_all, D, H, B], data=v.data_ptr())
    ot = _t(o)
    scale = 1.0 / np.sqrt(D)
    pad = np.zeros(2, np.uint32)
    pad.view(np.float32)[0] = scale
    pad[1] = n_ctx
    C.memmove(C.addressof(ot) + type(ot).padding.offset, pad.ctypes.data, 8)   # c_char field reads return copies
    _run(L.bestla_device_mha_f32, C.byref(params()), C.byref(_t(q)), C.byref(kt), C.byref(vt), C.byref(ot))
    assert _rel(o.cpu().numpy(), _mha_ref(Q, K, V, scale, seq_all)) <= 2e-5


@pytest.mark.parametrize("rms", [True, False])
@pytest.mark.parametrize("where", ["host", "device", "host_inplace"])
def test_host_layernorm(rms, where):
    """bestla_layernormalization = BTLALayerNorm (bestla_gemm.cpp:751-776; kernel_ref.h:2199-2240), host or device
    pointers, synchronous."""
    L = _lib.lib()
    x = (np.random.default_rng(3).standard_normal((7, 4096)) * 2 + 0.3).astype(np.float32)
    xv = x.astype(np.float64)
    mean = xv.mean(-1, keepdims=True)
    ms = np.sqrt((xv ** 2).mean(-1, keepdims=True) + 1e-6) if rms else \
        np.sqrt((xv ** 2).mean(-1, keepdims=True) - mean ** 2 + 1e-6)
    ref = xv / ms if rms else (xv - mean) / ms
    if where == "device":
        xd = torch.from_numpy(x).cuda()
        od = torch.empty_like(xd)
        L.bestla_layernormalization(7, 4096, rms, 1e-6, C.c_void_p(xd.data_ptr()), C.c_void_p(od.data_ptr()))
        out = od.cpu().numpy()
    elif where == "host":
        out = np.zeros_like(x)
        L.bestla_layernormalization(7, 4096, rms, 1e-6, x.ctypes.data, out.ctypes.data)
    else:
        out = x.copy()
        L.bestla_layernormalization(7, 4096, rms, 1e-6, out.ctypes.data, out.ctypes.data)
    assert _rel(out, ref) <= TOL


@pytest.mark.parametrize("vstep", [0, 300])
def test_host_mul_add(vstep):
    """bestla_mul / bestla_add (ne_bestla.cpp:118-168): out[b] = t[b] op v[b * vstep], host pointers."""
    L = _lib.lib()
    rng = np.random.default_rng(4)
    t = rng.standard_normal((5, 300)).astype(np.float32)
    v = rng.standard_normal((5 if vstep else 1, 300)).astype(np.float32)
    for f, op in ((L.bestla_mul, np.multiply), (L.bestla_add, np.add)):
        out = np.zeros_like(t)
        f(5, 300, t.ctypes.data, v.ctypes.data, vstep, out.ctypes.data)
        np.testing.assert_allclose(out, op(t, v if vstep else v[0]), rtol=1e-6)


LN_GOLDEN = ["layernorm_rms_4096", "layernorm_ln_300", "layernorm_rms_11008", "layernorm_ln_4096"]


@pytest.mark.parametrize("case", LN_GOLDEN)
@pytest.mark.parametrize("where", ["host", "device"])
def test_layernorm_matches_reference_golden(case, where):
    """bestla_layernormalization pinned to the REFERENCE's own output: tests/golden/ref/layernorm_* were produced by
    kernel_ref.h:2199-2240 layernorm<float> driven as BTLALayerNorm drives it (oracle/ref/ref_golden.cpp).  The
    device kernel sums the row in a tree instead of left to right, so the bar is fp32 reduction-order noise: 1e-5
    (the non-RMS form's mean(x^2) - mean^2 cancels, amplifying that noise where |mean| ~ rms)."""
    from tests.oracle_lib import load_ref_golden
    g = load_ref_golden()[case]
    rows, size, rms = (int(v) for v in g["meta"])
    eps = float(g["eps"][0])
    x = g["src"].reshape(rows, size).copy()
    if where == "device":
        xd = torch.from_numpy(x).cuda()
        od = torch.empty_like(xd)
        _lib.lib().bestla_layernormalization(rows, size, bool(rms), eps, C.c_void_p(xd.data_ptr()),
                                             C.c_void_p(od.data_ptr()))
        out = od.cpu().numpy()
    else:
        out = np.zeros_like(x)
        _lib.lib().bestla_layernormalization(rows, size, bool(rms), eps, x.ctypes.data, out.ctypes.data)
    assert _rel(out, g["dst"].reshape(rows, size)) <= TOL
