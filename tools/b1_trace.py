"""Per-stream timeline of single-pair analyze_batch calls (B = 1, inputs on the device): run under
`rocprofv3 --kernel-trace` and reduce the trace with --report.

    rocprofv3 --kernel-trace -f csv rocpd -d OUT -o run -- python3 tools/b1_trace.py --calls 40
    python3 tools/b1_trace.py --report OUT/run_results.db

The report takes the last --last calls (each delimited by its fusion_kernel) and prints, per HIP
queue: span (first start .. last end), busy time (sum of kernel durations), gap time and kernel
count, plus the call's overall span -- which tower chain is the critical path and how much of it is
inter-kernel gaps (launch-latency bound) vs kernel time."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(calls: int) -> None:
    import torch
    import bench
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    eng = Engine(0, W.synthetic_detector_state(0), W.synthetic_clip_state(0), max_batch=8)
    t = bench.build_inputs(eng, 8, 0)
    one = {k: v[:1].contiguous() for k, v in t.items()}
    out = eng.alloc_outputs(1)
    for _ in range(calls):
        eng.analyze_batch(one["rid"], one["rm"], one["cid"], one["cm"], one["img"], out=out)
        torch.cuda.synchronize()


def report(db: str, last: int) -> None:
    import sqlite3
    cur = sqlite3.connect(db).cursor()
    rows = list(cur.execute("select name, start, end, queue_id from kernels order by start"))
    fus = [i for i, r in enumerate(rows) if "fusion_kernel" in r[0]]
    for c in range(len(fus) - last, len(fus)):
        a = fus[c - 1] + 1
        call = rows[a:fus[c] + 1]
        t0, t1 = call[0][1], max(r[2] for r in call)
        print(f"call {c}: {len(call)} kernels, span {(t1 - t0) / 1e3:.1f} us")
        by_q = {}
        for name, s, e, q in call:
            by_q.setdefault(q, []).append((s, e, name))
        for q, ks in sorted(by_q.items(), key=lambda kv: kv[1][0][0]):
            busy = sum(e - s for s, e, _ in ks)
            span = max(e for _, e, _ in ks) - ks[0][0]
            top = {}
            for s, e, n in ks:
                n = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:48]
                top[n] = top.get(n, 0) + (e - s)
            tops = ", ".join(f"{n} {v / 1e3:.0f}" for n, v in sorted(top.items(), key=lambda kv: -kv[1])[:4])
            print(f"  queue {q}: {len(ks):4d} kernels, start +{(ks[0][0] - t0) / 1e3:7.1f} us, span {span / 1e3:7.1f} us, "
                  f"busy {busy / 1e3:7.1f} us, gaps {(span - busy) / 1e3:7.1f} us | {tops}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=40)
    ap.add_argument("--report", default="")
    ap.add_argument("--last", type=int, default=2)
    a = ap.parse_args()
    if a.report:
        report(a.report, a.last)
    else:
        run(a.calls)
