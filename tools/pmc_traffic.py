"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv [--symbol 'gemm_glds_kernel<256, 192, 4, 2, 0>']
                                [--json out.json]

Counter values are KB per dispatch.  Corrections (MI355X_MICROARCH.md, HBM section): on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so it is doubled; WRITE_SIZE
is exact for 16-B-per-lane stores.  Only dispatches between the first and the last fusion_kernel
(the measured steps) are used; set-up work before them is excluded.
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def same_kernel(a, b):
    """Symbols equal up to gemm_glds_kernel's trailing TQ = false (as profiling.same_kernel)."""
    def norm(s):
        return re.sub(r"^(gemm_glds_kernel<(?:[^,<>]+, ){7}[^,<>]+), (?:false|0)>$", r"\1>", s)
    return norm(a) == norm(b)


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*\)$", "", re.sub(r"^void ", "", name))


def load(path):
    rows = list(csv.DictReader(open(path)))
    marks = sorted(int(r["End_Timestamp"]) for r in rows if "fusion_kernel" in r["Kernel_Name"])
    if len(marks) >= 2:
        rows = [r for r in rows if int(r["Start_Timestamp"]) >= marks[0] and int(r["End_Timestamp"]) <= marks[-1]]
    agg = defaultdict(list)
    for r in rows:
        agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return agg, max(len(marks) - 1, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--symbol", default="gemm_glds_kernel<256, 192, 4, 2, 0>")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    fe, steps = load(a.fetch)
    wr, _ = load(a.write)
    table = []
    for k in sorted(fe, key=lambda k: -sum(fe[k])):
        f = 2.0 * 1024 * sum(fe[k]) / len(fe[k])
        w = 1024 * sum(wr.get(k, [0])) / max(len(wr.get(k, [])), 1)
        table.append({"kernel": k, "launches_per_step": len(fe[k]) / steps, "fetch_bytes_per_launch": f,
                      "write_bytes_per_launch": w, "hbm_bytes_per_launch": f + w})
    for t in table[:25]:
        print(f"{t['kernel'][:48]:48s} {t['launches_per_step']:6.1f}/step  fetch {t['fetch_bytes_per_launch'] / 1e6:9.2f} MB"
              f"  write {t['write_bytes_per_launch'] / 1e6:9.2f} MB")
    dom = next((t for t in table if same_kernel(t["kernel"], a.symbol)), None)
    if a.json and dom:
        json.dump({"symbol": a.symbol, "steps": steps, "hbm_bytes_per_launch": round(dom["hbm_bytes_per_launch"]),
                   "fetch_bytes_per_launch": round(dom["fetch_bytes_per_launch"]),
                   "write_bytes_per_launch": round(dom["write_bytes_per_launch"]),
                   "corrections": "FETCH_SIZE x2 (gfx950 wide-read tally), WRITE_SIZE as reported",
                   "all_kernels": table}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
