"""HBM traffic of the decode kernels from two rocprofv3 --pmc passes over tools/pmc_decode.py (development tool).

  rocprofv3 --pmc FETCH_SIZE -d D/fetch ... -- python tools/pmc_decode.py     (PMC_ALG_OUT=D/alg.json)
  rocprofv3 --pmc WRITE_SIZE -d D/write ... -- python tools/pmc_decode.py
  python tools/pmc_traffic.py D profiles/pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are KB (1024 B) per dispatch; FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950 reports
half the bytes of 16 B/lane streaming reads).  Per kernel family: mean traffic per dispatch vs the mean algorithmic
bytes of the same dispatches (bench.Stack.launches)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_dispatch(root, ctr):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if (r.get("Counter_Name") or r.get("Counter-Name")) != ctr:
                continue
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName")
            vals[name][r.get("Dispatch_Id") or r.get("Dispatch-Id")] += float(r.get("Counter_Value") or 0)
    return vals


def family(name):
    for fam in ("woq_gemv_m1_kernel", "woq_gemv_kernel"):
        if fam in name:
            return fam
    return None


def main():
    root, out = sys.argv[1], sys.argv[2]
    alg = json.load(open(f"{root}/alg.json"))
    fetch, write = per_dispatch(f"{root}/fetch", "FETCH_SIZE"), per_dispatch(f"{root}/write", "WRITE_SIZE")
    fam_f, fam_w = defaultdict(list), defaultdict(list)
    for name, d in fetch.items():
        if family(name):
            fam_f[family(name)] += list(d.values())
    for name, d in write.items():
        if family(name):
            fam_w[family(name)] += list(d.values())
    rec = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over tools/pmc_decode.py "
                     "(4 Llama-2-7B layers + lm_head: 3 per-op tokens); FETCH_SIZE doubled per "
                     "MI355X_MICROARCH.md (gfx950 reports half of 16 B/lane streaming reads); KB = 1024 B; "
                     "tools/pmc_traffic.py"}
    per_op_alg = alg["decode_bytes_per_token"] / alg["decode_launches_per_token"]
    for fam in fam_f:
        n = len(fam_f[fam])
        if True:
            fb = 2 * 1024 * sum(fam_f[fam]) / n
            wb = 1024 * sum(fam_w[fam]) / max(1, len(fam_w[fam]))
            rec[fam] = {"fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb, "algorithmic_bytes_per_launch":
                        per_op_alg, "dispatches": n, "traffic_over_algorithmic": round((fb + wb) / per_op_alg, 4)}
        print(fam, rec[fam])
    json.dump(rec, open(out, "w"), indent=1)
    # bench.py reads the newest round's last-listed file (bench.latest_pmc)
    import os
    import re
    m = re.match(r"(r\d+)_", os.path.basename(out))
    if m:
        with open(os.path.join(os.path.dirname(os.path.abspath(out)), f"{m.group(1)}_pmc_latest.txt"), "a") as f:
            f.write(os.path.basename(out) + "\n")


if __name__ == "__main__":
    main()
