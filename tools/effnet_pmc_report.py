"""Derived per-kernel metrics from the four PMC passes of tools/pmc_passes.sh (EfficientNet tower):
duration, resident waves per CU, wave-state shares, VALU / LDS / bank-conflict shares, MFMA busy,
HBM bytes per launch and the achieved HBM rate.

    python tools/effnet_pmc_report.py gpurun_out/<tag> [--match expand_dw,stem_dw,dwconv,se_kernel,pw_kernel]

Units (MI355X_MICROARCH.md, rocprofv3 PMC slots): SQ_WAVE_CYCLES and the SQ_WAIT_* / SQ_ACTIVE_*
counters count quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs; SQ_* counters are summed over
the chip; a wave64 VALU instruction occupies its SIMD 2 cycles (transcendentals more: the VALU
share is a lower bound); FETCH_SIZE x2 for the gfx950 wide-read tally, WRITE_SIZE as reported (KB).
"""
import argparse
import collections
import csv
import os
import re

CUS, SIMDS, XCDS = 256, 1024, 8


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return re.sub(r"\(.*$", "", re.sub(r"^void ", "", n))


def load(path):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "End_Timestamp" in r and "Start_Timestamp" in r:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="expand_dw,stem_dw,dwconv,se_kernel,pw_kernel,gemm_f16,gemm_glds,gap")
    ap.add_argument("--images", type=int, default=0,
                    help="images the profiled command pushed through the tower (all its forwards): prints MB/img")
    a = ap.parse_args()
    passes = [load(os.path.join(a.dir, f"p{i}", "run_counter_collection.csv")) for i in range(1, 5)]
    # per-dispatch means (a counter row is repeated per dimension instance: sum per dispatch first)
    cnt = collections.defaultdict(dict)
    durs = collections.defaultdict(list)
    for per, dur in passes:
        for k, cs in per.items():
            for c, vals in cs.items():
                cnt[k][c] = vals
            durs[k] += dur[k]
    match = a.match.split(",")
    if a.images:
        tot = sum(2 * sum(cs.get("FETCH_SIZE", [])) + sum(cs.get("WRITE_SIZE", []))
                  for k, cs in cnt.items() if any(m in k for m in match)) * 1024
        print(f"# HBM bytes of every matching launch (FETCH_SIZE x2 + WRITE_SIZE) / {a.images} images: "
              f"{tot / a.images / 1e6:.2f} MB per image")
    rows = []
    for k, cs in cnt.items():
        if not any(m in k for m in match):
            continue
        def m(c):
            v = cs.get(c)
            return sum(v) / max(len(v), 1) if v else float("nan")
        n = len(cs.get("GRBM_GUI_ACTIVE", [1]))
        cyc = m("GRBM_GUI_ACTIVE") / XCDS  # per-XCD cycles of one dispatch
        wave_cyc = m("SQ_WAVE_CYCLES") * 4
        res = wave_cyc / (CUS * cyc) if cyc else float("nan")
        valu = m("SQ_INSTS_VALU") * 2 / (SIMDS * cyc) if cyc else float("nan")
        lds = m("SQ_LDS_IDX_ACTIVE") / (CUS * cyc) if cyc else float("nan")
        conf = m("SQ_LDS_BANK_CONFLICT") / max(m("SQ_LDS_IDX_ACTIVE"), 1)
        mfma = m("SQ_VALU_MFMA_BUSY_CYCLES") / (SIMDS * cyc) if cyc else float("nan")
        hbm = (2 * m("FETCH_SIZE") + m("WRITE_SIZE")) * 1024
        d = sum(durs[k]) / max(len(durs[k]), 1) if durs[k] else float("nan")
        rows.append((d * n, k, d, res, m("SQ_WAIT_ANY") * 4 / wave_cyc, m("SQ_WAIT_INST_ANY") * 4 / wave_cyc,
                     m("SQ_ACTIVE_INST_ANY") * 4 / wave_cyc, valu, lds, conf, mfma, hbm / 1e6, hbm / (d * 1e3)))
    print(f"{'kernel':44s} {'us':>7s} {'waves/CU':>8s} {'wait':>5s} {'issue':>5s} {'activ':>5s} {'VALU':>5s} "
          f"{'LDS':>5s} {'bankc':>5s} {'MFMA':>5s} {'HBM MB':>7s} {'GB/s':>6s}")
    for _, k, d, res, w, wi, ac, valu, lds, conf, mfma, mb, gbs in sorted(rows, reverse=True):
        print(f"{k[:44]:44s} {d:7.1f} {res:8.1f} {w:5.2f} {wi:5.2f} {ac:5.2f} {valu:5.2f} {lds:5.2f} {conf:5.2f} "
              f"{mfma:5.2f} {mb:7.1f} {gbs:6.0f}")


if __name__ == "__main__":
    main()
