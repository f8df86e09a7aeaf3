"""Concurrency of the tower streams in a rocprofv3 --kernel-trace of bench.py (default concurrent
mode): per step, the wall time (first fusion_kernel end to the next), the union of busy intervals,
the sum of kernel durations, and per stream (Stream_Id) its kernel time and span.

    python tools/concurrency_report.py gpurun_out/<tag>/t/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"], r["Queue_Id"])
                 for r in rows), key=lambda x: x[0])
    fus = [k for k in ks if "fusion_kernel" in k[2]]
    # steady-state steps: windows between consecutive fusion kernel ends (the last ~half of the run)
    wins = [(fus[i][1], fus[i + 1][1]) for i in range(len(fus) - 1)]
    wins = wins[len(wins) // 2:]
    for w0, w1 in wins[-4:]:
        inw = [k for k in ks if k[0] >= w0 and k[1] <= w1 and not k[2].startswith("__amd")]
        tot = sum(k[1] - k[0] for k in inw)
        # union
        u, cur_s, cur_e = 0, None, None
        for s, e, *_ in sorted(inw):
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    u += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            u += cur_e - cur_s
        per = defaultdict(lambda: [0, None, None, 0])
        for s, e, n, st, q in inw:
            p = per[q]
            p[0] += e - s
            p[1] = s if p[1] is None else min(p[1], s)
            p[2] = e if p[2] is None else max(p[2], e)
            p[3] += 1
        print(f"step {(w1 - w0) / 1e6:.3f} ms: busy union {u / 1e6:.3f} ms, kernel sum {tot / 1e6:.3f} ms, "
              f"overlap factor {tot / max(u, 1):.2f}")
        for q, (t, s, e, n) in sorted(per.items(), key=lambda kv: kv[1][1]):
            print(f"   queue {q}: {n:4d} kernels, {t / 1e6:.3f} ms kernel time, span {(s - w0) / 1e6:.3f} .. "
                  f"{(e - w0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
