"""Regenerate the committed golden fixtures under tests/golden/ (run in the build container only).

Two sources, both the reference itself:
  1. tests/golden/gguf/  -- outputs of oracle/_ref/gguf_golden, compiled from the reference's GGUF Q4_0 / Q8_0 code
                            (neural_speed/vectors/cpu/quantize.h, core/layers/vec_dot.h; scalar paths).
     tests/golden/ref/   -- outputs of oracle/_ref/ref_golden, a driver compiled by oracle/ref/Makefile directly
                            against /root/reference/bestla/bestla/kernel_ref.h (quantizer, interleave, compress,
                            kblock decompress, scalar GEMV, bf16/fp16 conversions).
  2. tests/golden/gptq/  -- outputs of the reference's GPTQ/AWQ unpack functions
                            (/root/reference/neural_speed/convert/common.py:333-464), imported here with the absent
                            `gguf` module stubbed (it is only used by other converters in that file).

The fixtures are data (inputs + expected outputs); nothing from the reference's source text is stored.
Usage:  python tests/golden/make_golden.py
"""
import os
import subprocess
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


def make_ref():
    subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle", "ref")])
    out = os.path.join(HERE, "ref")
    os.makedirs(out, exist_ok=True)
    for f in os.listdir(out):
        os.remove(os.path.join(out, f))
    subprocess.check_call([os.path.join(REPO, "oracle", "_ref", "ref_golden"), out])
    gg = os.path.join(HERE, "gguf")
    os.makedirs(gg, exist_ok=True)
    for f in os.listdir(gg):
        os.remove(os.path.join(gg, f))
    subprocess.check_call([os.path.join(REPO, "oracle", "_ref", "gguf_golden"), gg])


def make_gptq():
    import torch

    sys.modules.setdefault("gguf", types.ModuleType("gguf"))
    sys.path.insert(0, os.path.join(REF, "neural_speed", "convert"))
    import common  # noqa: E402  (reference module, generation-time only)

    out = os.path.join(HERE, "gptq")
    os.makedirs(out, exist_ok=True)
    rng = np.random.default_rng(20250112)
    cases = {
        "gptq4_g32": dict(bits=4, K=128, N=64, gs=32, method="gptq", sym=False),
        "gptq4_g128": dict(bits=4, K=256, N=32, gs=128, method="gptq", sym=True),
        "gptq8_g64_sym": dict(bits=8, K=128, N=16, gs=64, method="gptq", sym=True),
        "gptq8_g64_asym": dict(bits=8, K=128, N=16, gs=64, method="gptq", sym=False),
        "awq4_g64": dict(bits=4, K=128, N=64, gs=64, method="awq", sym=False),
        "gptq3_g64": dict(bits=3, K=320, N=40, gs=64, method="gptq", sym=False),
    }
    for name, c in cases.items():
        bits, K, N, gs = c["bits"], c["K"], c["N"], c["gs"]
        pack = 32 // bits
        G = K // gs
        if c["method"] == "awq":
            qweight = rng.integers(-2**31, 2**31, size=(K, N // pack), dtype=np.int64).astype(np.int32)
        elif bits == 3:  # the reference reads ten 3-bit fields per int32
            qweight = rng.integers(-2**31, 2**31, size=(K // 10, N), dtype=np.int64).astype(np.int32)
        else:
            qweight = rng.integers(-2**31, 2**31, size=(K // pack, N), dtype=np.int64).astype(np.int32)
        if bits == 3:
            qzeros = rng.integers(-2**31, 2**31, size=(G, -(-N // 10)), dtype=np.int64).astype(np.int32)
        else:
            qzeros = rng.integers(-2**31, 2**31, size=(G, N // pack), dtype=np.int64).astype(np.int32)
        scales = rng.uniform(0.001, 0.005, size=(G, N)).astype(np.float16)
        qcfg = {"quant_method": c["method"], "bits": bits, "group_size": gs, "sym": c["sym"]}
        w, s, z = common.unpack_weight(torch.from_numpy(qweight), torch.from_numpy(scales),
                                       torch.from_numpy(qzeros), qcfg)
        w = w.reshape(-1, w.shape[-1]) if c["method"] != "awq" else w
        np.save(os.path.join(out, f"{name}.qweight.npy"), qweight)
        np.save(os.path.join(out, f"{name}.qzeros.npy"), qzeros)
        np.save(os.path.join(out, f"{name}.scales.npy"), scales)
        np.save(os.path.join(out, f"{name}.weight.npy"), w.to(torch.int32).numpy())
        np.save(os.path.join(out, f"{name}.zeros.npy"), z.to(torch.int32).numpy())
        with open(os.path.join(out, f"{name}.cfg.txt"), "w") as f:
            f.write(f"{c['method']} {bits} {gs} {int(c['sym'])} {K} {N}\n")


if __name__ == "__main__":
    make_ref()
    make_gptq()
    print("golden fixtures written under", HERE)
