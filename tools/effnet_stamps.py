"""Per-block phase stamps of the EfficientNet depthwise / fused-front kernels (diagnostic build).

    make -C <pkg>/csrc -j8 BUILD=build_stamp LIB=../../variants/stamp/libmmf_hip.so EXTRA=-DMMF_EFF_STAMP
    MMF_HIP_LIB=variants/stamp/libmmf_hip.so python tools/effnet_stamps.py [--batch 256]

Each stamping kernel (effnet.hip, EST_* macros) records per block: s_memrealtime at start / end and
s_memtime after each phase (wave 0, after the phase's barrier where there is one).  Printed per
kernel instantiation: blocks, kernel span, mean resident blocks per CU (sum of block lifetimes /
span / 256 CUs), the median block lifetime, the effective clock (memtime / realtime ticks) and the
median cycles of each phase segment.  The stamps cost cycles of their own (a waitcnt each): read the
SHARES, not the absolute times.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REGIONS = 25
BLOCKS, SLOTS = 16384, 32
NAMES = {
    0: "expand_dw<3,1,1,..> (stage 2.2)", 2: "expand_dw<3,2,1,..> (stage 2.1)", 3: "expand_dw<3,2,2,..> (stage 4.1)",
    5: "expand_dw<5,1,2,..> (stage 3.2)", 6: "expand_dw<5,2,1,..> (stage 3.1)", 24: "stem_dw",
}


def region_name(r):
    if r in NAMES:
        return NAMES[r]
    if 8 <= r < 24:
        q, tt = divmod(r - 8, 4)
        k = 5 if q >= 2 else 3
        s = 2 if q % 2 else 1
        t = {0: 8, 1: 14, 2: 7, 3: 16}[tt]
        return f"dwconv<{k},{s},T={t}>"
    return f"region {r}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    import mmf_amd.hip as hip
    import mmf_amd.synthetic as syn
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    lib = hip.load()
    if not hasattr(lib, "mmf_debug_eff_stamp"):
        raise SystemExit("not a stamp build (set MMF_HIP_LIB to a -DMMF_EFF_STAMP library)")
    eng = Engine(0, W.synthetic_detector_state(0), None, max_batch=a.batch)
    img = torch.from_numpy(syn.images(a.batch, 3)).cuda()
    for _ in range(a.iters):  # warm (clock, caches); stamps off
        eng.effnet_forward(img)
    torch.cuda.synchronize()
    buf = torch.zeros(REGIONS * BLOCKS * SLOTS, dtype=torch.int64, device="cuda")
    lib.mmf_debug_eff_stamp.argtypes = [ctypes.c_void_p]
    assert lib.mmf_debug_eff_stamp(ctypes.c_void_p(buf.data_ptr())) == 0
    eng.effnet_forward(img)
    torch.cuda.synchronize()
    assert lib.mmf_debug_eff_stamp(ctypes.c_void_p(0)) == 0
    st = buf.view(REGIONS, BLOCKS, SLOTS).cpu().numpy().astype(np.int64)
    print(f"B = {a.batch}; times in us (realtime 100 MHz), phases in shader cycles (median over blocks)")
    for r in range(REGIONS):
        n = st[r, :, SLOTS - 1]
        used = n > 0
        if not used.any():
            continue
        s = st[r, used]
        t0, t1 = s[:, 0], s[:, 1]
        span = (t1.max() - t0.min()) / 100.0
        life = (t1 - t0) / 100.0
        resident = life.sum() / span / 256.0
        nst = int(n[used].max())
        ph = np.diff(s[:, 2:nst + 1], axis=1)
        clk = (s[:, nst] - s[:, 2]) / np.maximum(t1 - t0, 1) * 0.1  # GHz
        print(f"{region_name(r):34s} blocks {used.sum():6d} span {span:7.1f}  resident/CU {resident:4.2f}  "
              f"life p50 {np.median(life):6.2f} p90 {np.percentile(life, 90):6.2f}  clk {np.median(clk):.2f} GHz")
        med = np.median(ph, axis=0)
        tot = med.sum()
        print("    phases (cycles): " + "  ".join(f"{int(m)}" for m in med) + f"   (sum {int(tot)})")
        # start-time profile: how many blocks start in each tenth of the span
        hist, _ = np.histogram((t0 - t0.min()) / 100.0, bins=10, range=(0, span))
        print("    starts per tenth of span: " + " ".join(str(int(x)) for x in hist))


if __name__ == "__main__":
    main()
