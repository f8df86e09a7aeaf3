"""Per-kernel roofline accounting from the library's event timing (mmf_profile_begin/end).

Peaks (MI355X, /opt/skills/guides/MI355X_MICROARCH.md): dense fp16 MFMA 2.5 PFLOP/s; HBM3E
8.0 TB/s.  `achieved` divides ALGORITHMIC work (flops of the contraction, or the minimum bytes
the op must move) by measured device time, so it is a lower bound on utilisation.
"""
from __future__ import annotations

import ctypes
import glob
import json
import os
import re
from typing import Callable, Dict, List

import torch

from .hip import check

PROFILES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
PEAK_BF16_TFLOPS = 2500.0
PEAK_HBM_GBS = 8000.0
NK = 512  # >= the library's PK_COUNT (kGemmConfigs x 5 epilogues x 5 activations + 12 other kinds)


def profile_kernels(eng, step: Callable[[], None], steps: int) -> List[Dict]:
    lib = eng.lib
    torch.cuda.synchronize()
    check(lib.mmf_profile_begin(eng.h), "mmf_profile_begin")
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    counts = (ctypes.c_int * NK)()
    ms = (ctypes.c_double * NK)()
    fl = (ctypes.c_double * NK)()
    by = (ctypes.c_double * NK)()
    n = lib.mmf_profile_end(eng.h, NK, counts, ms, fl, by)
    if n < 0:
        check(n, "mmf_profile_end")
    rows = []
    for k in range(n):
        if counts[k] == 0:
            continue
        name = lib.mmf_profile_kind_name(k).decode()
        # attention reads qkv once at ~4.2 TB/s for ~210 TFLOP/s: an HBM kernel
        mfma = name.startswith("gemm")
        rows.append({"kernel": name, "launches_per_step": counts[k] / steps, "ms_per_step": ms[k] / steps,
                     "avg_launch_us": 1000.0 * ms[k] / counts[k],
                     "tflops": fl[k] / (ms[k] / 1e3) / 1e12, "gbs": by[k] / (ms[k] / 1e3) / 1e9,
                     "flops_per_launch": fl[k] / counts[k], "bytes_per_launch": by[k] / counts[k],
                     "bound": "mfma" if mfma else "hbm"})
    rows.sort(key=lambda r: -r["ms_per_step"])
    return rows


def kind_symbol(kind: str) -> str:
    """Event-profile kind -> kernel symbol as rocprofv3 prints it (GEMM kinds only)."""
    m = re.match(r"gemm_(glds|glds_pipe2|f16)<([\d,]+)> act=(\d)(?: epi=(\d))?", kind)
    if not m:
        return kind
    dims = m.group(2).split(",")
    epi = m.group(4) or "0"
    # (then the measurement-build selector DBG, 0 in production)
    if m.group(1) == "glds":
        return f"gemm_glds_kernel<{', '.join(dims + [m.group(3), 'false', epi, '0'])}>"
    if m.group(1) == "glds_pipe2":
        return f"gemm_glds_kernel<{', '.join(dims + [m.group(3), 'true', epi, '0'])}>"
    return f"gemm_f16_kernel<{', '.join(dims)}, 1, false>"  # (PF, ASC: plain launches)


def same_kernel(a: str, b: str) -> bool:
    """Symbols equal up to gemm_glds_kernel's ninth template argument when it is the default: round 4's
    tile-queue TQ = false, or the K-loop variant KL = 0 measured in round 6 (later summaries print 8)."""
    def norm(s):
        return re.sub(r"^(gemm_glds_kernel<(?:[^,<>]+, ){7}[^,<>]+), (?:false|0)>$", r"\1>", s)
    return norm(a) == norm(b)


def pmc_traffic(symbol: str, path: str | None = None) -> float | None:
    """HBM bytes per launch of `symbol` from the committed rocprofv3 PMC passes
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py), or None."""
    files = [path] if path else sorted(glob.glob(os.path.join(PROFILES, "r*_pmc_traffic.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for row in d.get("all_kernels", []):
            if same_kernel(row["kernel"], symbol):
                return float(row["hbm_bytes_per_launch"])
    return None


def kernel_roofline(eng, step: Callable[[], None], steps: int) -> Dict:
    rows = profile_kernels(eng, step, steps)
    dom = rows[0]
    if dom["bound"] == "mfma":
        ach, peak, unit = dom["tflops"], PEAK_BF16_TFLOPS, "TFLOP/s"
    else:
        ach, peak, unit = dom["gbs"], PEAK_HBM_GBS, "GB/s"
    total = sum(r["ms_per_step"] for r in rows)
    return {"bound": dom["bound"], "kernel": dom["kernel"], "achieved": round(ach, 1), "peak": peak,
            "unit": unit, "frac": round(ach / peak, 4),
            # the library prices every launch by its own (M, N, K), so the dominant kernel's
            # algorithmic work IS what it executes (the compact last layers are separate launches)
            "executed_frac": round(ach / peak, 4),
            "traffic": pmc_traffic(kind_symbol(dom["kernel"])),
            "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/)",
            "symbol": kind_symbol(dom["kernel"]),
            "avg_launch_us": round(dom["avg_launch_us"], 2),
            "algorithmic_per_launch": round(dom["flops_per_launch"] if dom["bound"] == "mfma"
                                            else dom["bytes_per_launch"], 1),
            "kernel_ms_per_step": round(total, 3),
            "breakdown": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()
                           if k in ("kernel", "ms_per_step", "launches_per_step", "avg_launch_us", "tflops", "gbs",
                                    "bound")} for r in rows]}
