"""GGUF Q4_0 x Q8_0 oracle pinned bit-exact against the reference's own code: tests/golden/gguf/* come
from oracle/_ref/gguf_golden, compiled from neural_speed/vectors/cpu/quantize.h + core/layers/vec_dot.h (scalar
paths).  The reference's AVX2 build rounds Q8_0 ties to even and forms 127/amax instead of 1/(amax/127); those codes
can differ by one on exact ties, which the GPU tests' tolerance absorbs."""
import numpy as np
import pytest

from tests.oracle_lib import Oracle, _ptr, load_ref_golden


@pytest.fixture(scope="module")
def golden():
    return load_ref_golden("gguf")


@pytest.fixture(scope="module")
def oracle():
    return Oracle.get()


@pytest.mark.parametrize("case", ["q4_0_n40_k256", "q4_0_n16_k1024"])
def test_q4_0_oracle_bit_exact(golden, oracle, case):
    g = golden[case]
    n, k, m = (int(v) for v in g["meta"])
    W = g["W"].reshape(n, k)
    q4 = oracle.q4_0_quantize(W)
    assert np.array_equal(q4.ravel(), g["q4_0"])
    deq = oracle.q4_0_dequant(q4, n, k)
    assert np.array_equal(deq.ravel().view(np.uint32), g["deq"].view(np.uint32))
    A = g["A"].reshape(m, k)
    q8 = np.zeros((m, k // 32 * 34), np.uint8)
    for i in range(m):
        oracle.lib.orc_q8_0_quantize_row(_ptr(A[i].copy()), _ptr(q8[i]), k)
    assert np.array_equal(q8.ravel(), g["q8_0"])
    C = oracle.q4_0_forward(A, q4, n, k)
    assert np.array_equal(C.ravel().view(np.uint32), g["C"].view(np.uint32))


def test_q4_0_is_int4_g32_sym_fp16_scale(golden, oracle):
    """Q4_0 = signed int4 (nibble - 8) x fp16 d per 32 k: the same dequantized values as a BTLA S4 g32 sym blob with
    fp16 scales, which is how the device layout holds it"""
    g = golden["q4_0_n40_k256"]
    n, k, _ = (int(v) for v in g["meta"])
    blocks = g["q4_0"].reshape(n, k // 32, 18)
    d = blocks[:, :, :2].copy().view(np.float16).astype(np.float32)[:, :, 0]
    qs = blocks[:, :, 2:]
    q = np.concatenate([(qs & 15).astype(np.int8) - 8, (qs >> 4).astype(np.int8) - 8], axis=2)  # [n][nb][32]
    deq = (q.astype(np.float32) * d[:, :, None]).reshape(n, k)
    assert np.array_equal(deq.view(np.uint32), g["deq"].reshape(n, k).view(np.uint32))
