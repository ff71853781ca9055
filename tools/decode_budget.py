"""Per-token decode budget from a rocprofv3 --kernel-trace of bench.py (development tool).

Finds runs of 129 consecutive M = 1 decode GEMV dispatches (one Llama-2-7B token: 32 x [QKV, O, gate/up, down] +
lm_head), and per op role reports: algorithmic bytes, their time at 8 TB/s (spec) and at 6.3 TB/s (the achievable HBM
rate, MI355X_MICROARCH.md § HBM), the measured kernel span (trace Start -> End), the gap from the previous kernel's
End to this Start (the kernel boundary as the CP spends it), and the totals per token.
Usage: python tools/decode_budget.py <rocprofv3 output dir> [out.txt]"""
import csv
import glob
import statistics as st
import sys

H, F, V, G = 4096, 11008, 32000, 128


def wbytes(n, k):
    return n * k // 2 + n * (k // G) * 2


ROLES = [("qkv", wbytes(3 * H, H) + 4 * (H + 3 * H)), ("o", wbytes(H, H) + 4 * (H + H)),
         ("gate_up", 2 * wbytes(F, H) + 4 * (H + 2 * F)), ("down", wbytes(H, F) + 4 * (F + H))]
LM = ("lm_head", wbytes(V, H) + 4 * (H + V))

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
dec = [i for i, r in enumerate(rows) if "woq_gemv_m1" in r[2]]
tokens, run = [], []
for i in dec:
    if run and i != run[-1] + 1:
        run = []
    run.append(i)
    if len(run) == 129:
        tokens.append(run)
        run = []
if not tokens:
    sys.exit("no 129-launch decode token found")
per = {name: {"span": [], "gap": []} for name, _ in ROLES + [LM]}
tok_wall = []
for t in tokens:
    tok_wall.append((rows[t[-1]][1] - rows[t[0]][0]) / 1e3)
    for j, i in enumerate(t):
        name = LM[0] if j == 128 else ROLES[j % 4][0]
        per[name]["span"].append((rows[i][1] - rows[i][0]) / 1e3)
        if j > 0:
            per[name]["gap"].append((rows[i][0] - rows[i - 1][1]) / 1e3)
out = [f"# decode budget from {len(tokens)} traced tokens (median per op; us)",
       f"{'op':8s} {'count':>5s} {'MB':>7s} {'@8TB/s':>7s} {'@6.3TB/s':>8s} {'span':>6s} {'gap':>5s} {'span-@6.3':>9s}"]
tot = {"b8": 0, "b63": 0, "span": 0, "gap": 0}
for name, by in ROLES + [LM]:
    cnt = 1 if name == "lm_head" else 32
    sp = st.median(per[name]["span"])
    gp = st.median(per[name]["gap"]) if per[name]["gap"] else 0.0
    b8, b63 = by / 8e6, by / 6.3e6
    out.append(f"{name:8s} {cnt:5d} {by / 1e6:7.2f} {b8:7.2f} {b63:8.2f} {sp:6.2f} {gp:5.2f} {sp - b63:9.2f}")
    tot["b8"] += cnt * b8
    tot["b63"] += cnt * b63
    tot["span"] += cnt * sp
    tot["gap"] += cnt * gp
out.append(f"{'token':8s} {129:5d} {3415.34:7.1f} {tot['b8']:7.1f} {tot['b63']:8.1f} {tot['span']:6.1f} {tot['gap']:5.1f} "
           f"{tot['span'] - tot['b63']:9.1f}")
wall = st.median(tok_wall)
out.append(f"sum span + gaps = {tot['span'] + tot['gap']:.1f} us; traced token wall (first start -> last end) median "
           f"{wall:.1f} us -> {wall - tot['span']:.1f} us between kernels ({(wall - tot['span']) / 128:.2f} us per "
           f"boundary; the trace's per-pair gaps read ~0 under graph replay, the wall does not)")
print("\n".join(out))
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write("\n".join(out) + "\n")
