"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite) of a bench.py run.

    python tools/rocprof_summary.py gpurun_out/prof/run_results.db [--per-step-kernel fusion_kernel]

Prints, per kernel symbol, launches per step, avg / total duration per step (us), using the
number of launches of a once-per-step kernel (the fusion MLP) as the step count.  With --by-grid
the rows are split by grid size (one row per GEMM shape).
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*\)$", "", name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per-step-kernel", default="fusion_kernel")
    ap.add_argument("--by-grid", action="store_true")
    ap.add_argument("--csv", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, duration, grid_x, workgroup_x, start, end from kernels"))
    marks = sorted(r[5] for r in rows if a.per_step_kernel in r[0])
    if len(marks) >= 2:
        # steady-state window: from the end of the first step to the end of the last one, so
        # set-up work before the first step (vault encoding, warm-up compiles) is excluded
        rows = [r for r in rows if r[4] >= marks[0] and r[5] <= marks[-1]]
        steps = len(marks) - 1
    else:
        steps = 1
    agg = defaultdict(lambda: [0, 0.0])
    for name, dur, gx, wx, _, _ in rows:
        key = short(name) + (f" grid={gx // max(wx, 1)}" if a.by_grid else "")
        agg[key][0] += 1
        agg[key][1] += dur / 1e3
    total = sum(v[1] for v in agg.values()) / steps
    out = ["kernel,launches_per_step,avg_us,us_per_step,share"]
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.append(f"\"{k}\",{n / steps:.2f},{us / n:.2f},{us / steps:.1f},{us / steps / total:.4f}")
    out.append(f"\"TOTAL (kernel time per step, {steps} steps)\",,,{total:.1f},1.0")
    text = "\n".join(out)
    print(text)
    if a.csv:
        open(a.csv, "w").write(text + "\n")


if __name__ == "__main__":
    main()
