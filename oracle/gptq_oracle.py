"""numpy restatement of the reference's GPTQ / AWQ unpack (TEST INFRASTRUCTURE ONLY).

Follows /root/reference/neural_speed/convert/common.py:
  unpack_gptq_weight_4bits  :398-417
  unpack_gptq_weight_8bits  :353-395
  unpack_gptq_weight_3bits  :420-446  (ten 3-bit fields per int32 at bits 0..27; the int3 re-centring of :766-770)
  unpack_awq_weight         :449-464
and the int4 re-centring of convert_quantized_llama.py:72-76 (w - 8, zp - 8) that precedes
np_bestla_qpack (application/main_pybind.cpp:378-402).  Pinned by tests/golden/gptq/* (outputs of the
reference functions themselves, see tests/golden/make_golden.py).
"""
import numpy as np


def _wrap_i8(x):
    return ((np.asarray(x, dtype=np.int64) + 128) % 256 - 128).astype(np.int8)


def _wrap_u8(x):
    return (np.asarray(x, dtype=np.int64) % 256).astype(np.uint8)


def unpack_gptq4(qweight, qzeros):
    """qweight int32 [K/8, N], qzeros int32 [G, N/8] -> weight [K, N] in 0..15, zeros [G, N] in 1..16."""
    qweight = np.asarray(qweight, dtype=np.int32)
    qzeros = np.asarray(qzeros, dtype=np.int32)
    shifts = np.arange(0, 32, 4, dtype=np.int32)
    w = (qweight[:, None, :] >> shifts[None, :, None]) & 15           # [K/8, 8, N]
    z = (qzeros[:, :, None] >> shifts[None, None, :]) & 15             # [G, N/8, 8]
    return w.reshape(-1, qweight.shape[1]).astype(np.int32), (z.reshape(qzeros.shape[0], -1) + 1).astype(np.int32)


def unpack_gptq8(qweight, qzeros, sym):
    qweight = np.asarray(qweight, dtype=np.int32)
    qzeros = np.asarray(qzeros, dtype=np.int32)
    shifts = np.arange(0, 32, 8, dtype=np.int32)
    z = ((qzeros[:, :, None] >> shifts[None, None, :]) & 255).reshape(qzeros.shape[0], -1)
    if sym:
        z = _wrap_i8(_wrap_i8(z).astype(np.int64) + 1).astype(np.int32)
    else:
        z = _wrap_u8(_wrap_u8(z).astype(np.int64) + 1).astype(np.int64)
        z = _wrap_i8(z - 128).astype(np.int32)
    w = ((qweight[:, None, :] >> shifts[None, :, None]) & 255).reshape(-1, qweight.shape[1]).astype(np.int64)
    if sym:
        w = _wrap_i8(w - 128)
    else:
        w = _wrap_i8(_wrap_u8(w).astype(np.int64) - 128)
    return w.astype(np.int32), z


def unpack_gptq3(qweight, qzeros, group_size, n_groups, n):
    """qweight int32 [R, N] -> weight [group_size * n_groups, N] in 0..7 (rows past that trimmed); qzeros int32 [G, C]
    -> zeros [G, n] in 1..8 (ten fields per int32, columns past n dropped)."""
    qweight = np.asarray(qweight, dtype=np.int32)
    qzeros = np.asarray(qzeros, dtype=np.int32)
    shifts = np.arange(0, 29, 3, dtype=np.int32)                       # range(0, 32 - 3, 3): 10 fields
    w = (qweight[:, None, :] >> shifts[None, :, None]) & 7             # [R, 10, N]
    w = w.reshape(-1, qweight.shape[1])[:group_size * n_groups]
    z = ((qzeros[:, :, None] >> shifts[None, None, :]) & 7) + 1        # [G, C, 10]
    z = z.reshape(qzeros.shape[0], -1)[:, :n]
    return w.astype(np.int32), z.astype(np.int32)


def unpack_awq4(qweight, qzeros):
    """AWQ: qweight int32 [K, N/8] with nibble order [0,4,1,5,2,6,3,7]; no +1 on zeros."""
    order = [0, 4, 1, 5, 2, 6, 3, 7]
    qweight = np.asarray(qweight, dtype=np.int32)
    qzeros = np.asarray(qzeros, dtype=np.int32)
    K, C = qweight.shape
    w = np.zeros((K, C * 8), dtype=np.int32)
    z = np.zeros((qzeros.shape[0], qzeros.shape[1] * 8), dtype=np.int32)
    for col in range(C):
        for i in range(8):
            w[:, col * 8 + i] = (qweight[:, col] >> (4 * order[i])) & 15
    for col in range(qzeros.shape[1]):
        for i in range(8):
            z[:, col * 8 + i] = (qzeros[:, col] >> (4 * order[i])) & 15
    return w, z


def gidx_regroup(int_weight, g_idx, group_size):
    """convert_quantized_llama.py:46-60: rows permuted so group g's rows are contiguous."""
    out = int_weight.copy()
    seen = {}
    for i, g in enumerate(np.asarray(g_idx)):
        g = int(g)
        if g not in seen:
            seen[g] = 0
        else:
            seen[g] += 1
        out[g * group_size + seen[g]] = int_weight[i]
    return out
