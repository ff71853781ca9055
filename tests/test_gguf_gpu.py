"""GPU GGUF Q4_0 (woq_gguf.hip) against the reference's own outputs (tests/golden/gguf, from neural_speed's
quantize.h / vec_dot.h) and the oracle.

  * nad_q4_0_device_load: the device tile layout unpacks to the reference's dequantize_row_q4_0, bit for bit;
  * nad_quant_q8_0: block_q8_0 bytes identical to quantize_row_q8_0_reference;
  * compute mode 1 (the reference's arithmetic: Q8_0 activations, integer block dots, sumi * d_w * d_a): within 1e-5
    of max|ref| of the reference's ne_vec_dot_q4_0_q8_0 results (float association across blocks differs);
  * mode 0: the fp path on the exact Q4_0 weights, against the fp64 product with the dequantized matrix.
"""
import numpy as np
import pytest

from tests.conftest import gpu_available
from tests.oracle_lib import load_ref_golden
from tests.test_gpu_parity import _rel_err

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from neural_amd import bestla


@pytest.fixture(scope="module")
def golden():
    return load_ref_golden("gguf")


@pytest.fixture
def int8_mode():
    prev = bestla.set_compute_mode(bestla.COMPUTE_INT8)
    yield
    bestla.set_compute_mode(prev)


@pytest.mark.parametrize("case", ["q4_0_n40_k256", "q4_0_n16_k1024"])
def test_q4_0_load_unpacks_bit_exact(golden, case):
    g = golden[case]
    n, k, _ = (int(v) for v in g["meta"])
    w = bestla.DeviceWeight.from_q4_0(g["q4_0"], n, k)
    deq = w.unpack()                      # [K][N]
    assert np.array_equal(deq.T.copy().view(np.uint32), g["deq"].reshape(n, k).view(np.uint32))


@pytest.mark.parametrize("case", ["q4_0_n40_k256", "q4_0_n16_k1024"])
def test_q8_0_quant_bit_exact(golden, case):
    g = golden[case]
    _, k, m = (int(v) for v in g["meta"])
    x = torch.from_numpy(g["A"].reshape(m, k).copy()).cuda()
    assert np.array_equal(bestla.quant_q8_0(x).cpu().numpy().ravel(), g["q8_0"])


@pytest.mark.parametrize("case", ["q4_0_n40_k256", "q4_0_n16_k1024"])
def test_q4_0_int8_mode_matches_reference(golden, int8_mode, case):
    g = golden[case]
    n, k, m = (int(v) for v in g["meta"])
    w = bestla.DeviceWeight.from_q4_0(g["q4_0"], n, k)
    y = w.forward(torch.from_numpy(g["A"].reshape(m, k).copy()).cuda()).cpu().numpy()
    assert _rel_err(y, g["C"].reshape(m, n).astype(np.float64)) <= 1e-5


@pytest.mark.parametrize("m", [1, 5, 16, 40, 300])
@pytest.mark.parametrize("n,k", [(4096, 4096), (200, 11008)])
def test_q4_0_int8_mode_matches_oracle(oracle, int8_mode, m, n, k):
    rng = np.random.default_rng(m + n)
    Wq = oracle.q4_0_quantize(rng.uniform(-1, 1, size=(n, k)).astype(np.float32))
    w = bestla.DeviceWeight.from_q4_0(Wq, n, k)
    A = rng.uniform(-1, 1, size=(m, k)).astype(np.float32)
    y = w.forward(torch.from_numpy(A).cuda()).cpu().numpy()
    assert _rel_err(y, oracle.q4_0_forward(A, Wq, n, k).astype(np.float64)) <= 1e-5


@pytest.mark.parametrize("m", [1, 64])
def test_q4_0_fp_mode(oracle, m):
    n, k = 256, 2048
    rng = np.random.default_rng(m)
    Wq = oracle.q4_0_quantize(rng.uniform(-1, 1, size=(n, k)).astype(np.float32))
    w = bestla.DeviceWeight.from_q4_0(Wq, n, k)
    x = torch.from_numpy(rng.uniform(-1, 1, size=(m, k)).astype(np.float32)).half().cuda()
    ref = x.float().cpu().numpy().astype(np.float64) @ oracle.q4_0_dequant(Wq, n, k).T.astype(np.float64)
    # M > 16 runs the prefill GEMM (gemm7) at groups of 32, which folds the fp16 block scale into the fp16 weights (q * d rounded once:
    # tests/test_gemm2_gpu.py FOLD_TOL); the M = 1 GEMV keeps them exact
    assert _rel_err(w.forward(x).cpu().numpy(), ref) <= (2e-5 if m <= 16 else 5e-4)
