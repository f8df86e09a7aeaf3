"""Per-phase cycles of the persistent encoder GEMM (diagnostic build).

    make -C <pkg>/csrc -j8 BUILD=build_gstamp LIB=../../variants/gstamp/libmmf_hip.so EXTRA=-DMMF_GEMM_STAMP
    MMF_HIP_LIB=variants/gstamp/libmmf_hip.so python tools/gemm_stamps.py [--shapes rob_o,rob_fc2,...]

gemm.hip's GST macros record, per workgroup (wave 0), s_memtime at every tile's start, after its first
K-step and after its K loop, plus one stamp after the last tile (and s_memrealtime at start / end).
Per shape (the production tile choice, or --config), over all workgroups (medians):
  first    tile 0's first K-step: the prologue DMA of both slabs + 1 K-step of MFMAs
  k0       a later tile's first K-step: its slab 0 was prefetched under the previous tile's last
           K-step, slab 1 is fetched during this one (exposed fill latency)
  kstep    steady K-steps: (K loop - first K-step) / (nk - 1)
  epi      a tile's epilogue: next tile's start - this tile's K-loop end (stores issued, not drained)
  tail     the last tile's epilogue + the drain to the kernel's end
Shares are of the median workgroup's life.  The stamps cost cycles of their own (an s_waitcnt each,
and sched_barriers around them): read the shares, not the absolute times.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SLOTS = 96
SHAPES = {  # name: (M, N, K, act)
    "rob_qkv": (32768, 2304, 768, 0), "rob_o": (32768, 768, 768, 0), "rob_fc1": (32768, 3072, 768, 1),
    "rob_fc2": (32768, 768, 3072, 0), "vit_qkv": (12800, 2304, 768, 0), "vit_o": (12800, 768, 768, 0),
    "vit_fc1": (12800, 3072, 768, 2), "vit_fc2": (12800, 768, 3072, 0), "txt_qkv": (19712, 1536, 512, 0),
    "txt_o": (19712, 512, 512, 0), "txt_fc1": (19712, 2048, 512, 2), "txt_fc2": (19712, 512, 2048, 0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="rob_o,rob_fc2,rob_fc1,rob_qkv,vit_o,vit_fc2,txt_o,txt_fc2")
    ap.add_argument("--config", type=int, default=-1, help="forced gemm_config (default: production choice)")
    ap.add_argument("--warm", type=int, default=30)
    ap.add_argument("--phases", action="store_true",
                    help="a -DMMF_GEMM_STAMP=2 build: the four phase stamps of K-steps 1..20 of each workgroup's first tile")
    a = ap.parse_args()
    import mmf_amd.hip as hip
    lib = hip.load()
    if not hasattr(lib, "mmf_debug_gemm_stamp"):
        raise SystemExit("not a stamp build (set MMF_HIP_LIB to a -DMMF_GEMM_STAMP library)")
    lib.mmf_debug_gemm_stamp.argtypes = [ctypes.c_void_p]
    hip.set_process_option("gemm_config", a.config)
    dev = torch.device("cuda")
    buf = torch.zeros(256 * SLOTS, dtype=torch.int64, device=dev)
    g = torch.Generator(device=dev).manual_seed(5)
    print("median cycles per workgroup phase (shares of the median workgroup life); clk = memtime / realtime")
    for name in a.shapes.split(","):
        M, N, K, act = SHAPES[name]
        A = (torch.randn(M, K, device=dev, generator=g) * 0.5).half()
        W = (torch.randn(N, K, device=dev, generator=g) * 0.03).half()
        bias = torch.randn(N, device=dev, generator=g) * 0.1
        C = torch.empty(M, N, device=dev, dtype=torch.float16)

        def run():
            hip.check(lib.mmf_gemm_f16(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(), None, None, C.data_ptr(), N,
                                       M, N, K, act, hip.stream_ptr()))
        for _ in range(a.warm):
            run()
        torch.cuda.synchronize()
        buf.zero_()
        assert lib.mmf_debug_gemm_stamp(ctypes.c_void_p(buf.data_ptr())) == 0
        run()
        torch.cuda.synchronize()
        assert lib.mmf_debug_gemm_stamp(ctypes.c_void_p(0)) == 0
        st = buf.view(256, SLOTS).cpu().numpy()
        used = st[:, 2] > 0
        nk = K // 64
        if a.phases:
            phases(name, M, N, K, st, used, nk)
            continue
        first, k0, kstep, epi, tail, life, clk, ntile = [], [], [], [], [], [], [], []
        for r in st[used]:
            n = int(r[2])
            ts = r[3:min(n, SLOTS)]
            nt = (len(ts) - 1) // 3
            ntile.append(nt)
            for i in range(nt):
                t0, t1, t2 = ts[3 * i], ts[3 * i + 1], ts[3 * i + 2]
                (first if i == 0 else k0).append(t1 - t0)
                if nk > 1:
                    kstep.append((t2 - t1) / (nk - 1))
                nxt = ts[3 * i + 3]
                (epi if i + 1 < nt else tail).append(nxt - t2)
            life.append(ts[-1] - ts[0])
            clk.append((ts[-1] - ts[0]) / max(r[1] - r[0], 1) * 0.1)
        med = lambda v: float(np.median(v)) if len(v) else float("nan")  # noqa: E731
        L = med(life)
        nt = med(ntile)
        parts = {"first": med(first), "k0": med(k0), "kstep": med(kstep), "epi": med(epi), "tail": med(tail)}
        # share of the life: first + (nt - 1) k0 + nt (nk - 1) kstep + (nt - 1) epi + tail
        shares = {"first": parts["first"], "k0": (nt - 1) * parts["k0"] if nt > 1 else 0.0,
                  "ksteps": nt * (nk - 1) * parts["kstep"], "epi": (nt - 1) * parts["epi"] if nt > 1 else 0.0,
                  "tail": parts["tail"]}
        tf = 2.0 * M * N * K / (L / (med(clk) * 1e9)) / 1e12 if L > 0 else 0.0
        print(f"{name:8s} M={M} N={N} K={K}: {used.sum()} WGs, {nt:.0f} tiles/WG, life {L / 1e3:.1f} k cycles "
              f"at {med(clk):.2f} GHz (~{tf:.0f} TFLOP/s)")
        print("    per phase: " + "  ".join(f"{k} {v:.0f}" for k, v in parts.items()))
        print("    shares:    " + "  ".join(f"{k} {100 * v / L:.1f}%" for k, v in shares.items()))
    hip.set_process_option("gemm_config", -1)


def phases(name, M, N, K, st, used, nk):
    """Per steady K-step (wave 0, steps 1..min(nk - 1, 20) of the first tile), cycles spent
    issuing the next slab's LDS-DMA (dma), issuing the fragment reads and MFMAs until the last MFMA
    is issued (reads+mfma: the partner wave's MFMAs share the pipe), waiting at the step barrier --
    vmcnt(0) for the DMA plus the slowest wave (barrier), and from the barrier to the next step's
    start (loop)."""
    steps = min(nk - 1, 20)
    rows = []
    for r in st[used]:
        t = r[3:3 + 4 * steps].reshape(steps, 4).astype(np.float64)
        if (t <= 0).any():
            continue
        for i in range(steps):
            nxt = t[i + 1, 0] if i + 1 < steps else np.nan
            rows.append((t[i, 1] - t[i, 0], t[i, 2] - t[i, 1], t[i, 3] - t[i, 2], nxt - t[i, 3], t[i, 3] - t[i, 0]))
    a = np.array(rows)
    # shader clock over each workgroup's life: s_memtime (slots 94 / 95) against s_memrealtime
    # (slots 0 / 1, 100 MHz)
    clk = [(r[95] - r[94]) / max(r[1] - r[0], 1) * 0.1 for r in st[used] if r[95] > r[94] > 0 and r[1] > r[0]]
    med = np.nanmedian(a, axis=0)
    p90 = np.nanpercentile(a, 90, axis=0)
    names = ("dma", "reads+mfma", "barrier", "loop", "step")
    print(f"{name:8s} M={M} N={N} K={K}: {used.sum()} WGs x {steps} steady K-steps (wave 0; 48 MFMAs x 2 waves = "
          f"1536 pipe cycles per step)")
    print("    median cycles: " + "  ".join(f"{n} {v:.0f}" for n, v in zip(names, med)))
    print("    p90 cycles:    " + "  ".join(f"{n} {v:.0f}" for n, v in zip(names, p90)))
    print("    share of the median step: " + "  ".join(f"{n} {100 * v / med[4]:.0f}%" for n, v in zip(names[:3], med[:3])))
    if clk:
        print(f"    shader clock over the workgroup's life: median {np.median(clk):.2f} GHz")


if __name__ == "__main__":
    main()
