"""Idle gaps between consecutive kernels of one queue in a rocprofv3 --kernel-trace database
(run_results.db): for each queue, kernels sorted by start; gap = next start - previous end (µs).
Prints per queue the busy time, the summed gaps and the kernel pairs with the largest gaps, and a
per-kernel-name table of the gap that FOLLOWS each kernel (what a launch boundary after it costs).

    python tools/stream_gaps.py gpurun_out/x/t1/run_results.db [--window-kernel gap_classifier] [--top 15]
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*\)$", "", re.sub(r"^void ", "", name))[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--window-kernel", default="", help="only kernels after the first launch of this "
                    "name (set-up launches excluded) and up to its last launch")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    qcol = next((q for q in ("queue_id", "queue", "stream_id", "stream") if q in cols), None)
    rows = list(c.execute(f"select name, start, end, {qcol or '0'} from kernels order by start"))
    if a.window_kernel:
        idx = [i for i, r in enumerate(rows) if a.window_kernel in r[0]]
        if len(idx) >= 2:
            rows = rows[idx[0] + 1: idx[-1] + 1]
    byq = defaultdict(list)
    for n, s, e, q in rows:
        byq[q].append((s, e, short(n)))
    after = defaultdict(list)
    for q, ks in byq.items():
        ks.sort()
        busy = sum(e - s for s, e, _ in ks) / 1e3
        gaps = [(ks[i + 1][0] - ks[i][1]) / 1e3 for i in range(len(ks) - 1)]
        span = (ks[-1][1] - ks[0][0]) / 1e3
        print(f"queue {q}: {len(ks)} kernels, span {span:.1f} us, busy {busy:.1f} us, "
              f"gaps {sum(g for g in gaps if g > 0):.1f} us (median {sorted(gaps)[len(gaps) // 2] if gaps else 0:.2f})")
        for i, g in enumerate(gaps):
            after[ks[i][2]].append(g)
    print(f"\n{'kernel (gap that follows it)':60s} {'n':>5s} {'avg_us':>8s} {'sum_us':>9s}")
    for k, v in sorted(after.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
        print(f"{k:60s} {len(v):5d} {sum(v) / len(v):8.2f} {sum(v):9.1f}")


if __name__ == "__main__":
    main()
