"""Host half of the graph seam (include/neural_amd_ne.h) on CPU: the planner probes bestla_support /
bestla_backend_support (restating core/layers/ne_bestla.cpp:176-249 with this backend's device workspace) and
bestla_parallel_for's INIT / COMPUTE / FINALIZE phase protocol (ne_bestla.cpp:42-70).  No GPU calls."""
import ctypes as C

import numpy as np

from neural_amd import _lib
from tests.ne_structs import (BACKEND_CPU, BACKEND_DEVICE, NE_TYPE_BTLA, NE_TYPE_F32, OP, TASK_COMPUTE,
                              TASK_FINALIZE, TASK_INIT, NeParams, NeTensor, params, tensor)


def _support(node):
    ws, dws = C.c_size_t(123), C.c_size_t(456)
    ok = _lib.lib().bestla_support(C.byref(node), 4, C.byref(ws), C.byref(dws))
    return ok, ws.value, dws.value


def test_support_mul_mat_workspaces():
    L = _lib.lib()
    w = tensor([4096, 4096], ttype=NE_TYPE_BTLA, backend=BACKEND_CPU)
    for m in (1, 2048):
        x = tensor([4096, m])
        node = tensor([4096, m], op=OP["MUL_MAT"])
        node.src0, node.src1 = C.pointer(w), C.pointer(x)
        ok, ws, dws = _support(node)
        # host weight: the reference's workspace contract M * padto(K, 128) * 4 (inner_product.cpp:20-25)
        assert ok and node.n_tasks == 1 and ws == m * 4096 * 4 and dws == 0
    w.backend = BACKEND_DEVICE
    for m in (1, 16, 2048):
        want = L.nad_device_workspace_size(m, 4096)
        x = tensor([4096, m])
        node = tensor([4096, m], op=OP["MUL_MAT"], backend=BACKEND_DEVICE)
        node.src0, node.src1 = C.pointer(w), C.pointer(x)
        ok, ws, dws = _support(node)
        assert ok and ws == 0 and dws == want
    assert L.nad_device_workspace_size(2048, 4096) >= 2048 * 4096 * 2      # fp16 copy of A


def _a256(x):
    return -(-x // 256) * 256


def test_workspace_bound_covers_every_k_tile():
    """nad_device_workspace_size bounds what the forward places in the workspace for any weight format: the fp16 copy
    of A padded to the weight's K tile (int2: 256, so K mod 256 in 1..128 needs more than a 128-rounded bound) plus the
    split-K partials behind it; at m <= 16 the int8-compute mode's u8 codes + per-block {scale, zp}."""
    L = _lib.lib()
    for k in (4096, 4097, 4160, 4224, 4300, 11008, 300, 33):
        for m in (1, 5, 16):
            kp = -(-k // 256) * 256
            need = _a256(m * kp) + _a256(m * (kp // 32) * 8)          # i8_act_bytes at the smallest group (32)
            assert L.nad_device_workspace_size(m, k) >= need, (m, k)
        for m in (1, 8, 12, 16):  # the mid-M kernel (from 8 / 12 rows by default): fp16 room + ks x N <= 32768 slabs
            a16 = _a256(m * (-(-k // 256) * 256) * 2)
            assert L.nad_device_workspace_size(m, k) >= a16 + m * 32768 * 4, (m, k)
        for m in (17, 300, 2048):
            for ktile in (64, 128, 256):
                kp = -(-k // ktile) * ktile
                a16 = _a256(m * kp * 2)
                # split-K partials: ks runs x m x ldp fp32, ks x ceil(m/256) x ceil(N/128) <= 256 -> N-independent
                part = 4 * m * 256 * 128 // -(-m // 256)
                assert L.nad_device_workspace_size(m, k) >= a16 + part, (m, k, ktile)


def test_support_elementwise_rules():
    a = tensor([64, 8])
    b = tensor([64, 1])
    node = tensor([64, 8], op=OP["ADD"], backend=BACKEND_CPU)
    node.src0, node.src1 = C.pointer(a), C.pointer(b)
    assert _support(node)[0]                   # broadcast row
    b2 = tensor([64, 3])
    node.src1 = C.pointer(b2)
    assert not _support(node)[0]               # rows neither 1 nor equal
    n2 = tensor([64, 8], op=OP["RMS_NORM"], backend=BACKEND_CPU)
    n2.src0 = C.pointer(a)
    assert _support(n2)[0]
    n3 = tensor([64, 8], op=OP["NONE"], backend=BACKEND_CPU)
    assert not _support(n3)[0]


def test_backend_support():
    L = _lib.lib()
    w = tensor([64, 64], ttype=NE_TYPE_BTLA, backend=BACKEND_DEVICE)
    x = tensor([64, 1], backend=BACKEND_CPU)
    assert L.bestla_backend_support(C.byref(w), C.byref(x), OP["MUL_MAT"]) == BACKEND_DEVICE
    w.backend = BACKEND_CPU
    assert L.bestla_backend_support(C.byref(w), C.byref(x), OP["MUL_MAT"]) == BACKEND_CPU
    f = tensor([64, 4], ttype=NE_TYPE_F32, backend=BACKEND_DEVICE)
    for op in ("RMS_NORM", "SILU", "ADD", "MUL"):
        assert L.bestla_backend_support(C.byref(f), None, OP[op]) == BACKEND_DEVICE
    assert L.bestla_backend_support(C.byref(f), None, OP["ROPE"]) == BACKEND_CPU


FPTR = C.CFUNCTYPE(None, C.POINTER(NeParams), C.POINTER(NeTensor))


def test_parallel_for_phases():
    L = _lib.lib()
    for nth in (1, 3):
        seen = []

        def fcomp(p, node):
            seen.append((p.contents.type, p.contents.ith))
        cb = FPTR(fcomp)
        mp = params(phase=TASK_COMPUTE, nth=nth)
        node = tensor([4])
        L.bestla_parallel_for(C.cast(cb, C.c_void_p), C.byref(mp), C.byref(node))
        inits = [s for s in seen if s[0] == TASK_INIT]
        comps = sorted(s[1] for s in seen if s[0] == TASK_COMPUTE)
        fins = sorted(s[1] for s in seen if s[0] == TASK_FINALIZE)
        assert inits == [(TASK_INIT, 0)]
        assert comps == list(range(nth)) and fins == list(range(nth))
        # every COMPUTE happens after INIT, every FINALIZE after all COMPUTEs
        order = [s[0] for s in seen]
        assert order.index(TASK_COMPUTE) > order.index(TASK_INIT)
        assert max(i for i, t in enumerate(order) if t == TASK_COMPUTE) < min(
            i for i, t in enumerate(order) if t == TASK_FINALIZE)


def test_timer_runs(capfd):
    L = _lib.lib()
    L.bestla_timer(True)
    L.bestla_timer(False)
    out = capfd.readouterr().out
    assert "time :" in out and "us" in out
    assert np.isfinite(float(out.split(":")[1].split()[0]))
