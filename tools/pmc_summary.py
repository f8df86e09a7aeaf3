"""Per-kernel averages of rocprofv3 PMC counters (counter_collection.csv of any command).

    python tools/pmc_summary.py gpurun_out/x/pass1/run_counter_collection.csv [--match effnet] [--top 30]

Prints, per kernel symbol (template arguments kept, grid size appended with --by-grid), the number
of dispatches and the mean value per dispatch of every counter in the file, plus derived ratios
when their inputs are present: MFMA busy share (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE)),
wait shares of SQ_WAVE_CYCLES, LDS bank-conflict cycles per LDS-active cycle.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*\)$", "", re.sub(r"^void ", "", name))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--by-grid", action="store_true")
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for r in csv.DictReader(open(a.csv)):
        k = short(r["Kernel_Name"])
        if a.by_grid:
            k += f" grid={r.get('Grid_Size', '?')}"
        if a.match and a.match not in k:
            continue
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for k, cs in per.items():
        n = max(len(v) for v in cs.values())
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        rows.append((sum(dur[k]) / len(dur[k]) * n, k, n, mean, sum(dur[k]) / len(dur[k])))
    rows.sort(key=lambda x: -x[0])
    for _, k, n, m, us in rows[: a.top]:
        extra = []
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    extra.append(f"{c[3:]}/WAVE={m[c] / wc:.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m and m["GRBM_GUI_ACTIVE"]:
            # MFMA busy per SIMD: busy cycles summed over 1024 SIMDs vs GUI-active cycles (8 XCDs summed)
            extra.append(f"mfma_busy={m['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * m['GRBM_GUI_ACTIVE'] / 8):.3f}")
        if "GRBM_GUI_ACTIVE" in m and us > 0:
            extra.append(f"clk={m['GRBM_GUI_ACTIVE'] / 8 / us / 1e3:.2f}GHz")
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
            extra.append(f"lds_conflict={m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.3f}")
        vals = " ".join(f"{c}={v:.4g}" for c, v in sorted(m.items()))
        print(f"{k[:60]:60s} n={n:4d} {us:9.2f}us  {' '.join(extra)}\n      {vals}")


if __name__ == "__main__":
    main()
