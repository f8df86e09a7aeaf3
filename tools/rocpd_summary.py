"""Per-kernel summary of a rocprofv3 --kernel-trace database (run_results.db, ROCm 7.2's default
output): launches, average and total duration, share; --per N divides totals by N (e.g. forwards).

    python tools/rocpd_summary.py gpurun_out/x/run_results.db [--per 6] [--top 40] [--grid]
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*\)$", "", re.sub(r"^void ", "", name))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--grid", action="store_true", help="split kernels by grid size")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    agg = defaultdict(list)
    for name, dur, gx, gy, gz in c.execute("select name, duration, grid_x, grid_y, grid_z from kernels"):
        k = short(name)
        if a.match and a.match not in k:
            continue
        if a.grid:
            k += f" grid=({gx},{gy},{gz})"
        agg[k].append(dur / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"{'kernel':70s} {'n/per':>7s} {'avg_us':>9s} {'us/per':>10s} {'share':>6s}")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
        print(f"{k[:70]:70s} {len(v) / a.per:7.2f} {sum(v) / len(v):9.2f} {sum(v) / a.per:10.1f} {sum(v) / tot:6.3f}")
    print(f"{'TOTAL':70s} {'':7s} {'':9s} {tot / a.per:10.1f}")


if __name__ == "__main__":
    main()
