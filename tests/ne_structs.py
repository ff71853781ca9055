"""ctypes mirrors of include/neural_amd_ne.h (the reference's ne_tensor / ne_compute_params layout) for tests."""
import ctypes as C

import numpy as np

NE_TYPE_F32, NE_TYPE_F16, NE_TYPE_I32, NE_TYPE_BTLA = 0, 1, 18, 19
BACKEND_CPU, BACKEND_DEVICE = 0, 1
TASK_INIT, TASK_COMPUTE, TASK_FINALIZE = 0, 1, 2
OP = dict(NONE=0, DUP=1, ADD=2, MUL=6, GELU=21, SILU=22, NORM=24, RMS_NORM=25, MUL_MAT=28, MUL_MAT_BIAS=29,
          MUL_MAT_ID=30, CPY=33, ROPE=46, MUL_QKV=52, MUL_FFN_SILU=53)


class NeTensor(C.Structure):
    pass


NeTensor._fields_ = [("type", C.c_int32), ("backend", C.c_int32), ("n_dims", C.c_int32), ("ne", C.c_int64 * 4),
                     ("nb", C.c_size_t * 4), ("op", C.c_int32), ("is_param", C.c_bool), ("op_params", C.c_int32 * 8),
                     ("grad", C.POINTER(NeTensor)), ("src0", C.POINTER(NeTensor)), ("src1", C.POINTER(NeTensor)),
                     ("opt", C.POINTER(NeTensor) * 36), ("n_tasks", C.c_int32), ("perf_runs", C.c_int32),
                     ("perf_cycles", C.c_int64), ("perf_time_us", C.c_int64), ("data", C.c_void_p),
                     ("size", C.c_size_t), ("name", C.c_char * 32), ("padding", C.c_char * 8)]
assert C.sizeof(NeTensor) == 512


class NeParams(C.Structure):
    _fields_ = [("type", C.c_int32), ("ith", C.c_int32), ("nth", C.c_int32), ("wsize", C.c_size_t),
                ("wdata", C.c_void_p), ("dev_wsize", C.c_size_t), ("dev_wdata", C.c_void_p), ("dev_queue", C.c_void_p)]


assert C.sizeof(NeParams) == 56


def tensor(ne, strides_bytes=None, ttype=NE_TYPE_F32, data=0, backend=BACKEND_DEVICE, op=0):
    """ne: up to 4 dims (ne[0] innermost).  strides default to contiguous for the element size of ttype."""
    ne = list(ne) + [1] * (4 - len(ne))
    esz = 2 if ttype == NE_TYPE_F16 else 4
    if strides_bytes is None:
        nb = [esz]
        for i in range(1, 4):
            nb.append(nb[-1] * ne[i - 1])
    else:
        nb = list(strides_bytes)
    t = NeTensor()
    t.type, t.backend, t.n_dims, t.op = ttype, backend, 4, op
    for i in range(4):
        t.ne[i] = ne[i]
        t.nb[i] = nb[i]
    t.data = data
    return t


def params(queue=0, phase=TASK_COMPUTE, nth=1):
    p = NeParams()
    p.type, p.ith, p.nth, p.dev_queue = phase, 0, nth, queue
    return p


def set_op_params_f32(t, values):
    arr = np.zeros(8, np.float32)
    arr[:len(values)] = values
    C.memmove(t.op_params, arr.ctypes.data, 32)
