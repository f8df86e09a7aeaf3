"""Per-step kernel totals from a rocprofv3 kernel trace (run_kernel_trace.csv), grouped by kernel
symbol with template arguments; 'steps' = launches of the one-per-step fusion kernel.

    python tools/kstats.py gpurun_out/<dir>/trace/run_kernel_trace.csv [--top 40]
"""
import argparse
import collections
import csv
import re


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\((?!anonymous).*$", "", n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    tot, cnt = collections.Counter(), collections.Counter()
    for r in csv.DictReader(open(a.csv)):
        n = short(r["Kernel_Name"])
        tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[n] += 1
    fk = [k for k in cnt if "fusion" in k]
    steps = cnt[fk[0]] if fk else 1
    print(f"steps {steps}")
    s = 0.0
    for k, v in tot.most_common(a.top):
        s += v / steps
        print(f"{v / steps / 1e3:7.3f} ms  {cnt[k] / steps:6.1f}/step  {v / cnt[k]:8.1f} us  {k[:100]}")
    print(f"sum of listed {s / 1e3:.3f} ms/step; all kernels {sum(tot.values()) / steps / 1e3:.3f} ms/step")


if __name__ == "__main__":
    main()
