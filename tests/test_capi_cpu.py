"""C-ABI tests that need no GPU: the library loads, exports every symbol of include/neural_amd.h, and its host
pack/unpack/split paths are bit-exact against the oracle (which is pinned to the reference's own goldens)."""
import ctypes as C

import numpy as np
import pytest

from neural_amd import _lib, bestla
from tests.oracle_lib import F32, BF16, F16, F4_BNB, F4_E2M1, F4_NF4, F8_E4M3, F8_E5M2, F8_E8M0, S1, S2, S3, S4, S5, S6, S7, S8


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    names = _lib.header_symbols()
    assert len(names) >= 50
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python signature table covers all of them
    assert set(names) <= set(_lib.SIGNATURES), set(names) - set(_lib.SIGNATURES)


def test_storage_descriptor_size():
    assert _lib.lib().bestla_device_storage_size() >= 96


CFGS = [
    # n, k, bs, qtype, stype, asym, comp
    (96, 256, 32, S4, F32, False, bestla.COMP_F32),
    (100, 300, 32, S4, BF16, True, bestla.COMP_F32),
    (77, 256, 128, S4, F16, False, bestla.COMP_INT8),   # amx_int8 kblock, PACK_ROW 4, reduce buffer
    (48, 512, 32, S4, F32, True, bestla.COMP_INT8),     # avx512_vnni kblock (32 % 64 != 0)
    (64, 256, 64, S2, F32, False, bestla.COMP_F32),
    (50, 256, 64, S2, BF16, True, bestla.COMP_INT8),
    (40, 128, 32, S8, F32, False, bestla.COMP_F32),
    (40, 128, 128, S8, F32, False, bestla.COMP_INT8),
    (96, 256, 32, S4, F32, False, bestla.COMP_BF16),    # amx_bf16: PACK_ROW 2, KTILE 32
    (33, 160, 32, S4, F32, False, bestla.COMP_F32),     # ragged N
    (64, 256, 32, S3, F32, False, bestla.COMP_F32),     # 3-bit: crumb + bit planes
    (50, 256, 128, S3, BF16, True, bestla.COMP_INT8),
    (48, 256, 32, S5, F32, True, bestla.COMP_F32),      # 5-bit: nibble + bit planes
    (48, 256, 64, S6, F16, False, bestla.COMP_INT8),    # 6-bit: nibble + crumb planes
    (40, 128, 32, S7, F32, False, bestla.COMP_F32),     # 7-bit: nibble + crumb + bit planes
    (64, 256, 32, S1, F32, False, bestla.COMP_F32),     # 1-bit: one bit plane (compress_1bit's slot-4 quirk)
    (50, 256, 64, S1, BF16, True, bestla.COMP_INT8),    # ... reduce buffer from the stored codes
    (64, 256, 32, F4_NF4, F32, False, bestla.COMP_F32),  # NFloat (prologue WeightKBlockNFloat): no zp / reduce
    (50, 256, 64, F4_E2M1, BF16, False, bestla.COMP_BF16),
    (48, 128, 32, F4_BNB, F32, False, bestla.COMP_INT8),  # int8 compute falls through to a float core
    (64, 256, 32, F8_E4M3, F8_E8M0, False, bestla.COMP_F32),  # fp8: shared-exponent (E8M0) scales
    (50, 200, 64, F8_E5M2, F8_E8M0, False, bestla.COMP_BF16),
    (48, 256, 32, F8_E4M3, F32, False, bestla.COMP_F32),      # fp8 with fp32 scales (pack API only)
    (40, 256, 128, F8_E5M2, F32, False, bestla.COMP_INT8),
]


@pytest.mark.parametrize("cfg", CFGS)
def test_quant_pack_bit_exact_vs_oracle(oracle, cfg):
    n, k, bs, qt, st, asym, comp = cfg
    rng = np.random.default_rng(n * 1000 + k)
    W = rng.uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
    W[0, :bs] = 0.0  # an all-zero block
    if qt in (F8_E4M3, F8_E5M2):
        W[1, 1:bs:2] *= np.float32(1e-6)  # tiny next to the block max: codes with exponent field 0
    if qt in (F8_E4M3, F8_E5M2) and st == F32:
        blob = bestla.quant_pack(W, bs, qt, st, asym, comp)
    else:
        blob = bestla.quantize(W, group_size=bs, weight_dtype={S4: "int4", S2: "int2", S8: "int8", S1: "int1", S3: "int3", S5: "int5", S6: "int6",
                                                           S7: "int7", F4_NF4: "nf4", F4_E2M1: "fp4_e2m1",
                                                           F4_BNB: "fp4_bnb", F8_E4M3: "fp8_e4m3", F8_E5M2: "fp8_e5m2"}[qt],
                           scale_dtype={F32: "fp32", BF16: "bf16", F16: "fp16", F8_E8M0: "fp8"}[st],
                           alg="asym" if asym else "sym",
                           compute_dtype={bestla.COMP_F32: "fp32", bestla.COMP_INT8: "int8", bestla.COMP_BF16: "bf16"}[comp])
    core = oracle.lib.orc_select_core(comp, qt, bs, int(asym), 0)
    ref = oracle.quant_pack(W, n, k, bs, qt, st, asym, core, is_trans=True)
    assert blob.size == ref.size
    np.testing.assert_array_equal(blob, ref)
    # unpack matches the oracle's dequantization exactly
    np.testing.assert_array_equal(bestla.unpack(blob).view(np.uint32), oracle.unpack_fp32(ref).view(np.uint32))


def test_qpack_gptq_with_g_idx_bit_exact(oracle):
    rng = np.random.default_rng(7)
    k, n, gs = 256, 64, 32
    q = rng.integers(-8, 8, size=(k, n)).astype(np.int8)
    s = rng.uniform(0.001, 0.005, size=(k // gs, n)).astype(np.float32)
    z = rng.integers(-8, 8, size=(k // gs, n)).astype(np.int8)
    g_idx = rng.permutation(np.arange(k) // gs).astype(np.int32)
    blob = bestla.qpack(q, s, z, g_idx, "int4", gs, "asym", "fp32", "int8")
    core = oracle.lib.orc_select_core(bestla.COMP_INT8, S4, gs, 1, 0)
    ref = oracle.pack_q(q, s, z, n, k, gs, S4, F32, True, core, g_idx)
    np.testing.assert_array_equal(blob, ref)
    Q, S, Z, shf = oracle.unpack_q(blob)
    np.testing.assert_array_equal(Q, q)
    expect = np.zeros(k, np.int32)
    oracle.lib.orc_shuffle_indices(g_idx.ctypes.data, k, gs, expect.ctypes.data)
    np.testing.assert_array_equal(shf, expect)


def test_blob_info_matches_oracle(oracle):
    rng = np.random.default_rng(3)
    W = rng.uniform(-0.5, 0.5, size=(80, 256)).astype(np.float32)
    blob = bestla.quantize(W, 64, "int4", "bf16", "asym", "int8")
    assert bestla.blob_info(blob) == oracle.info(blob)


@pytest.mark.parametrize("axis,world", [(0, 2), (0, 4), (1, 2), (1, 8)])
def test_tp_split_is_exact(oracle, axis, world):
    rng = np.random.default_rng(11)
    n, k, bs = 96, 86 * 32, 32  # 86 groups: uneven K split (11,11,11,11,11,11,10,10) at world 8
    W = rng.uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
    blob = bestla.quantize(W, bs, "int4", "bf16", "asym", "int8")
    full = bestla.unpack(blob)
    Qf, Sf, Zf, _ = oracle.unpack_q(blob)
    covered = 0
    for r in range(world):
        lo, hi = bestla.split_range(blob, axis, r, world)
        shard = bestla.split(blob, axis, r, world)
        if axis == 0:  # chunked column split lines up with a K-group consumer
            lo2, hi2 = bestla.split_range(blob, 0, r, world, unit=bs)
            assert lo2 % bs == 0 and (hi2 % bs == 0 or hi2 == n)
        part = bestla.unpack(shard)
        if axis == 0:
            np.testing.assert_array_equal(part, full[:, lo:hi])
        else:
            assert lo % bs == 0
            np.testing.assert_array_equal(part, full[lo:hi, :])
            # the shard's reduce buffer (int8 compute) equals the slice of the full one
            Qs, Ss, Zs, _ = oracle.unpack_q(shard)
            np.testing.assert_array_equal(Qs, Qf[lo:hi])
            np.testing.assert_array_equal(Ss, Sf[lo // bs:hi // bs])
        covered += hi - lo
    assert covered == (n if axis == 0 else k)


def test_packweight_copyattr_and_unpack_abi(oracle):
    L = _lib.lib()
    rng = np.random.default_rng(5)
    n, k = 64, 256
    W = rng.uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
    src = bestla.quantize(W, 32, "int4", "fp32", "sym", "fp32")
    dst = bestla._aligned_buffer(src.size)
    W2 = rng.uniform(-0.5, 0.5, size=(n, k)).astype(np.float32)
    L.bestla_packweight_copyattr(W2.ctypes.data_as(C.c_void_p), dst.ctypes.data_as(C.c_void_p), n, k, k,
                                 src.ctypes.data_as(C.c_void_p))
    np.testing.assert_array_equal(dst, bestla.quantize(W2, 32, "int4", "fp32", "sym", "fp32"))
    out = np.zeros((k, n), np.float32)
    L.bestla_unpackweight_fp32(dst.ctypes.data_as(C.c_void_p), n, k, out.ctypes.data_as(C.c_void_p), n)
    np.testing.assert_array_equal(out, oracle.unpack_fp32(dst))


def test_unsupported_inputs_fail_loudly():
    L = _lib.lib()
    bad = np.zeros(256, np.uint8)
    assert L.nad_device_weight_size(bad.ctypes.data_as(C.c_void_p)) == 0
    assert "WeightKBlockNInteger" in _lib.last_error() or "corrupt" in _lib.last_error()
    with pytest.raises(ValueError):
        bestla.quantize(np.zeros((16, 64), np.float32), 32, "int9")  # no such weight dtype (loudly)
    with pytest.raises(RuntimeError):  # F8_E8M0 scales with integer weights: rejected by the pack API
        bestla.quant_pack(np.zeros((16, 64), np.float32), 32, S4, F8_E8M0, False, bestla.COMP_F32)


def test_qpack_gptq3_bit_exact(oracle):
    """3-bit GPTQ ingest as convert/common.py:420-446,766-770 does it: unpack (ten fields per int32), re-centre by 4,
    np_bestla_qpack(weight_dtype="int3") -- the blob equals the oracle's and unpacks to (q - zp) * s"""
    import os
    from oracle import gptq_oracle
    from tests.oracle_lib import GOLDEN
    d = os.path.join(GOLDEN, "gptq")
    qweight = np.load(os.path.join(d, "gptq3_g64.qweight.npy"))
    qzeros = np.load(os.path.join(d, "gptq3_g64.qzeros.npy"))
    scales = np.load(os.path.join(d, "gptq3_g64.scales.npy")).astype(np.float32)
    w, z = gptq_oracle.unpack_gptq3(qweight, qzeros, 64, scales.shape[0], scales.shape[1])
    q = (w - 4).astype(np.int8)
    zp = (z - 4).astype(np.int8)
    k, n = q.shape
    blob = bestla.qpack(q, scales, zp, None, weight_dtype="int3", group_size=64, alg="asym", compute_dtype="int8")
    core = oracle.lib.orc_select_core(bestla.COMP_INT8, S3, 64, 1, 0)
    ref = oracle.pack_q(q, scales, zp, n, k, 64, S3, F32, True, core)
    np.testing.assert_array_equal(blob, ref)
    W = oracle.unpack_fp32(ref)
    expect = (q.astype(np.float32) - np.repeat(zp, 64, axis=0)) * np.repeat(scales, 64, axis=0)
    np.testing.assert_array_equal(W, expect)


def test_host_cache_key_is_constant_time_at_lm_head_shape():
    """The host-pointer ABI's per-call cache key (nad_host_blob_key: header + size + 64 sampled dwords) costs well under
    10 us at the lm_head shape (32000 x 4096 int4 g128, 67 MB blob) -- VERDICT r2 item 7: the old key hashed the whole
    scale section (4 MiB) byte by byte on every bestla_f32f32_forward -- and does not grow with the blob."""
    import time
    L = _lib.lib()
    rng = np.random.default_rng(0)
    keys, per_call = [], []
    for k, n in ((4096, 32000), (512, 256)):
        q = rng.integers(-8, 8, size=(k, n), dtype=np.int8)
        s = rng.uniform(0.001, 0.01, size=(k // 128, n)).astype(np.float32)
        blob = bestla.qpack(q, s, weight_dtype="int4", group_size=128, scale_dtype="fp16")
        p = C.c_void_p(blob.ctypes.data)
        keys.append(L.nad_host_blob_key(p))
        assert keys[-1] != 0
        reps = 20000
        t0 = time.perf_counter()
        for _ in range(reps):
            L.nad_host_blob_key(p)
        per_call.append((time.perf_counter() - t0) / reps)
        # another matrix packed into the same buffer changes the key (codes are sampled, not only the header)
        q2 = rng.integers(-8, 8, size=(k, n), dtype=np.int8)
        blob2 = bestla.qpack(q2, s, weight_dtype="int4", group_size=128, scale_dtype="fp16")
        blob[:] = blob2
        assert L.nad_host_blob_key(p) != keys[-1]
    assert per_call[0] < 10e-6, per_call
    assert per_call[0] < 4 * per_call[1] + 2e-6, per_call     # size-independent (ctypes call overhead included)


def test_plan_forward_kernel_choice():
    """nad_plan_forward (the host side of nad_device_forward with every launch recorded, no GPU): the decode shapes take
    the M = 1 / stripe-stream GEMVs, 17 <= M <= 64 the mid-M kernel, prefill takes gemm7 (int4 g128, the scale folded; gemm3 under NAD_GEMM_KERNEL=3)
    -- as do int4 g32 / g64, int2 and int8 (gemm4 under NAD_GEMM_KERNEL=3) -- and few output tiles split K."""
    p = bestla.plan_forward
    assert p(4, 4096, 4096, 128, m=1)["kernel"] == "woq_gemv_m1_kernel"
    assert p(2, 14336, 4096, 64, m=1)["kernel"] == "woq_gemv_m1_kernel"
    assert p(4, 4096, 4096, 128, m=4)["kernel"] == "woq_gemv_kernel"
    assert p(4, 4096, 4096, 128, m=8, act="fp16")["kernel"] == "woq_gemv_kernel"
    assert p(4, 4096, 4096, 128, m=8)["kernel"] == "woq_mid_kernel"       # fp32 rows: the mid-M kernel from 8
    assert p(4, 4096, 4096, 128, m=12, act="fp16")["kernel"] == "woq_mid_kernel"
    assert p(4, 4096, 4096, 128, m=9, act="fp16")["kernel"] == "woq_mid_kernel"      # one round of workgroups: from 9
    assert p(4, 11008, 4096, 128, m=10, act="fp16")["kernel"] == "woq_gemv_kernel"   # 344 workgroups: from 12
    r = p(4, 4096, 4096, 128, m=2048)
    assert (r["kernel"], r["fold"], r["ksplit"]) == ("woq_gemm7_kernel", True, 1)
    assert r["launches"] == 2                       # fp32 activations: one fp16 conversion pass, then the GEMM
    assert p(4, 4096, 4096, 128, m=2048, act="fp16")["launches"] == 1
    for bits, g in ((4, 32), (4, 64), (2, 64), (8, 32), (8, 128)):   # gemm7: the scale per 32-deep step / half step
        r = p(bits, 4096, 4096, g, m=2048)
        assert (r["kernel"], r["fold"]) == ("woq_gemm7_kernel", True), (bits, g, r)
    r = p(4, 4096, 4096, 128, m=64)                 # mid-M: fp32 activations read as they are, + the split-K reduce
    assert (r["kernel"], r["fold"], r["ksplit"], r["launches"]) == ("woq_mid_kernel", False, 4, 2), r
    r = p(4, 4096, 4096, 128, m=17, act="fp16")
    assert (r["kernel"], r["grid"], r["threads"]) == ("woq_mid_kernel", 256, 512), r   # 8 waves x 1 stage (int4 g128)
    r = p(4, 4096, 4096, 128, m=64)                 # fp32 rows at 4 row fragments: 4 waves x 2 stages (registers)
    assert (r["kernel"], r["threads"]) == ("woq_mid_kernel", 256), r
    assert p(4, 11008, 4096, 128, m=32)["ksplit"] == 2      # slabs within the workspace bound: ks x N <= 32768
    # 8-stripe workgroups where 4-stripe ones would take more than one per CU (M <= 32): 86 x 2 instead of 172 x 2
    assert p(4, 11008, 4096, 128, m=32)["grid"] == 172
    assert p(4, 11008, 4096, 128, m=48)["grid"] == 344     # 4 row fragments: 4 stripes only
    assert p(4, 4096, 4096, 128, m=32)["grid"] == 256
    assert p(4, 32000, 4096, 128, m=32)["ksplit"] == 1
    assert p(2, 4096, 4096, 64, m=33)["kernel"] == "woq_gemm7_kernel"   # int2 past 32 rows: the prefill GEMM
    r = p(4, 4096, 4096, 128, m=65)
    assert r["kernel"] == "woq_gemm7_kernel" and r["ksplit"] > 1 and r["launches"] == 3   # + the split-K reduce
    # gemm7's tile height (cost model, profiles/r05_gemm7_tile_height_sweep.txt) as launch geometry: M = 256 at N = 4096
    # takes 64-row tiles (128 tiles, split 2: 256 workgroups), M = 1024 128-row tiles (256, one round), M = 2048 256-row
    # (256 tiles); N = 11008 M = 640 128-row tiles (430 over 2 rounds, not 258 256-row tiles over 2)
    for m, n, grid, ks in ((256, 4096, 256, 2), (1024, 4096, 256, 1), (2048, 4096, 256, 1), (640, 11008, 430, 1)):
        r = p(4, n, 4096, 128, m=m, act="fp16")
        assert (r["kernel"], r["grid"], r["ksplit"]) == ("woq_gemm7_kernel", grid, ks), (m, n, r)
    # int8 / int2 at g128 fold too (NAD_GEMM4_FOLD_ALL default since round 4)
    assert p(8, 4096, 4096, 128, m=2048)["fold"] and p(2, 4096, 4096, 128, m=2048)["fold"]


def test_plan_gemm4_waves_split_over_k(knob):
    """gemm4's K-split wave layout (NAD_GEMM4_KSW=2, auto): on for more than one round of output tiles or K >= 8192
    (gate, down, lm_head, M = 4096), off for one round at K = 4096 (profiles/r04_gemm4_ksw_ab.txt) and under split-K.
    Shown on int8 g32 with gemm4 selected (NAD_GEMM_KERNEL=3; by default it runs gemm7)."""
    p = bestla.plan_forward
    knob("NAD_GEMM_KERNEL", "3")
    assert not p(8, 4096, 4096, 32, m=2048)["ksw"]          # 256 tiles: one round on 256 CUs
    assert p(8, 4096, 4096, 32, m=4096)["ksw"]              # 512 tiles
    assert p(8, 11008, 4096, 32, m=2048)["ksw"]             # gate: 688 tiles
    assert p(8, 4096, 11008, 32, m=2048)["ksw"]             # down: K = 11008
    r = p(8, 4096, 11008, 32, m=64)
    assert r["ksplit"] > 1 and not r["ksw"]                 # split-K launches keep the M-split waves
    assert not p(4, 4096, 4096, 128, m=4096)["ksw"]         # int4 g128: gemm3 (no K-split waves; gemm7 by default)


def test_host_cost_per_forward_under_3us():
    """the per-call host work of a forward (what an NE graph pays per WOQ node on the eager path:
    validation, kernel choice, geometry; the NAD_* switches are read once at load, not per call) stays under 3 us,
    ctypes call overhead included.  Timed through nad_plan_forward, which runs exactly that code with the launch
    recorded instead of issued."""
    import time
    L = _lib.lib()
    o = np.zeros(6, np.int64)
    ptr = o.ctypes.data

    def per_call(bits, n, k, g, m):
        best = 1e9
        for _ in range(5):
            reps = 4000
            t0 = time.perf_counter()
            for _ in range(reps):
                L.nad_plan_forward(bits, n, k, g, 2, 0, m, 0, ptr, 6)
            best = min(best, (time.perf_counter() - t0) / reps)
        return best

    # the same ctypes call rejected at its first check (bits = 3): the Python -> C call cost itself, which is ~2-3 us
    # here and varies with the machine's load, measured beside each shape and taken out
    for bits, n, k, g, m in ((4, 4096, 4096, 128, 1), (4, 22016, 4096, 128, 1), (2, 4096, 14336, 64, 1),
                             (4, 4096, 4096, 128, 2048)):
        assert L.nad_plan_forward(bits, n, k, g, 2, 0, m, 0, ptr, 6) == 6
        base = per_call(3, n, k, g, m)
        cost = per_call(bits, n, k, g, m)
        assert cost - base < 3e-6 and cost < 20e-6, (bits, n, k, m, cost, base)
