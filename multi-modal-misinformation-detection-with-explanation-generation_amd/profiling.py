"""Per-kernel roofline accounting from the library's event timing (mmf_profile_begin/end).

Peaks (MI355X, /opt/skills/guides/MI355X_MICROARCH.md): dense bf16 MFMA 2.5 PFLOP/s; HBM3E
8.0 TB/s.  `achieved` divides ALGORITHMIC work (flops of the contraction, or the minimum bytes
the op must move) by measured device time, so it is a lower bound on utilisation.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Dict, List

import torch

from .hip import check

PEAK_BF16_TFLOPS = 2500.0
PEAK_HBM_GBS = 8000.0
NK = 32


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
        mfma = name.startswith("gemm") or name == "attention"
        rows.append({"kernel": name, "launches_per_step": counts[k] / steps, "ms_per_step": ms[k] / steps,
                     "avg_launch_us": 1000.0 * ms[k] / counts[k],
                     "tflops": fl[k] / (ms[k] / 1e3) / 1e12, "gbs": by[k] / (ms[k] / 1e3) / 1e9,
                     "flops_per_launch": fl[k] / counts[k], "bytes_per_launch": by[k] / counts[k],
                     "bound": "mfma" if mfma else "hbm"})
    rows.sort(key=lambda r: -r["ms_per_step"])
    return rows


def kernel_roofline(eng, step: Callable[[], None], steps: int) -> Dict:
    rows = profile_kernels(eng, step, steps)
    dom = rows[0]
    if dom["bound"] == "mfma":
        ach, peak, unit = dom["tflops"], PEAK_BF16_TFLOPS, "TFLOP/s"
    else:
        ach, peak, unit = dom["gbs"], PEAK_HBM_GBS, "GB/s"
    total = sum(r["ms_per_step"] for r in rows)
    return {"bound": dom["bound"], "kernel": dom["kernel"], "achieved": round(ach, 1), "peak": peak,
            "unit": unit, "frac": round(ach / peak, 4), "traffic": None,
            "avg_launch_us": round(dom["avg_launch_us"], 2),
            "algorithmic_per_launch": round(dom["flops_per_launch"] if dom["bound"] == "mfma"
                                            else dom["bytes_per_launch"], 1),
            "kernel_ms_per_step": round(total, 3),
            "breakdown": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()
                           if k in ("kernel", "ms_per_step", "launches_per_step", "avg_launch_us", "tflops", "gbs",
                                    "bound")} for r in rows]}
