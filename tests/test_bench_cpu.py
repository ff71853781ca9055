"""bench.py's contract on CPU (no GPU): `--gpus 8 --dry-run` prints the per-rank tensor-parallel shard table the
8-GPU run would build, following docs/tensor_parallelism.md's split and the reference's loader
(model_files.h:134-235): Q/K/V column shards are whole heads, O / down are split along K by the same boundaries as the
columns feeding them, and down's K shards are whole quantization groups -- Llama-2-7B F = 11008 = 86 groups of 128 ->
11 groups on ranks 0-5 and 10 on ranks 6-7 (the reference itself requires even splits; here they are exact)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dry(gpus):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--dry-run"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_dry_run_tp8_shard_table():
    d = _dry(8)
    assert d["relaunch"] and d["nproc_per_node"] == 8
    rows = d["shards"]
    assert [r["rank"] for r in rows] == list(range(8))
    assert [r["down_k_groups"] for r in rows] == [11, 11, 11, 11, 11, 11, 10, 10]
    assert [r["heads"] for r in rows] == [4] * 8                                  # 32 heads of 128
    # contiguous, complete, head-aligned / group-aligned covers
    for key, total, unit in (("q_cols", 4096, 128), ("kv_cols", 4096, 128), ("down_k_rows", 11008, 128),
                             ("lm_head_cols", 32000, 16)):
        spans = [tuple(r[key]) for r in rows]
        assert spans[0][0] == 0 and spans[-1][1] == total, (key, spans)
        for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
            assert a1 == b0
        assert all(a % unit == 0 for a, _ in spans), (key, spans)
    for r in rows:
        assert r["o_k_rows"] == r["q_cols"] and r["gate_up_cols"] == r["down_k_rows"]


def test_dry_run_single_gpu():
    d = _dry(1)
    assert not d["relaunch"] and d["world"] == 1
    assert d["shards"][0]["down_k_groups"] == 86 and d["shards"][0]["lm_head_cols"] == [0, 32000]
