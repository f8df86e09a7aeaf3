"""Side-by-side per-kernel average durations of several rocprofv3 --stats runs.

    python tools/kstats_cmp.py gpurun_out/<tag>/t1 gpurun_out/<tag>/t2 ... [--match effnet]
"""
import csv
import os
import re
import sys


def load(d):
    rows = {}
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
        n = re.sub(r"\(anonymous namespace\)::", "", r["Name"])
        n = re.sub(r"^void ", "", re.sub(r"\(.*$", "", n))
        rows[n] = (float(r["AverageNs"]) / 1e3, int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3)
    return rows


def main():
    dirs = [a for a in sys.argv[1:] if not a.startswith("--")]
    runs = [load(d) for d in dirs]
    names = sorted(runs[0], key=lambda n: -runs[0][n][2])
    tot = [0.0] * len(runs)
    for n in names:
        if n.startswith("__amd"):
            continue
        vals = [r.get(n, (0, 0, 0)) for r in runs]
        for i, v in enumerate(vals):
            tot[i] += v[2] / max(v[1], 1) * vals[0][1] / max(vals[0][1], 1) if v[1] else 0
        print(f"{n[:60]:60s} " + " ".join(f"{v[0]:8.1f}" for v in vals))
    totals = [sum(v[2] for k, v in r.items() if not k.startswith("__amd")) for r in runs]
    print("total us (all calls)".ljust(61) + " ".join(f"{t:8.0f}" for t in totals))


if __name__ == "__main__":
    main()
