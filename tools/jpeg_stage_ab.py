"""A/B of the host entropy stage alone (no GPU): dense coefficient planes (mmf_jpeg_entropy, straight
into the staging buffer) vs packed records (mmf_jpeg_entropy_packed into a per-thread scratch +
copy into the staging buffer: mmf_jpeg_stage_packed), n synthetic 640x480 q90 4:2:0 JPEGs over a thread pool, alternated."""
import argparse
import ctypes
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mmf_amd import hip  # noqa: E402
from tests import jpeg_cases as C  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--workers", type=int, default=min(16, len(os.sched_getaffinity(0))))
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--progressive", action="store_true", help="progressive files (both legs)")
a = ap.parse_args()
L = hip.load()
datas = [C.encode(C.photo_like(640, 480, seed=i % 16), quality=90, subsampling=2, progressive=a.progressive)
         for i in range(a.n)]
info = np.zeros(16, np.int32)
L.mmf_jpeg_header(datas[0], len(datas[0]), info.ctypes.data)
blocks = int(info[11])
dense = np.empty(a.n * blocks * 128, np.uint8)
stage = np.empty(a.n * int(L.mmf_jpeg_packed_bound(blocks)), np.uint8)
boff = np.empty(a.n * blocks, np.uint32)
qt = np.empty(a.n * 192, np.uint16)
pool = ThreadPoolExecutor(a.workers)


def f_dense(k):
    d = datas[k]
    return L.mmf_jpeg_entropy(d, len(d), dense.ctypes.data + k * blocks * 128, qt.ctypes.data + k * 384)


cursor = np.zeros(1, np.int64)
rec_off = np.zeros(a.n, np.int64)


def f_packed(k):  # the product's staging call (jpeg.py): decode + reserve + copy in one C call
    d = datas[k]
    return L.mmf_jpeg_stage_packed(d, len(d), stage.ctypes.data, stage.size, cursor.ctypes.data,
                                   boff.ctypes.data + k * blocks * 4, qt.ctypes.data + k * 384,
                                   rec_off.ctypes.data + k * 8)


ptrs = (ctypes.c_char_p * a.n)(*datas)
lens = np.array([len(d) for d in datas], np.int64)
bases = np.arange(a.n, dtype=np.int64) * blocks
rcs = np.zeros(a.n, np.int32)


def batch_call():
    return L.mmf_jpeg_stage_packed_batch(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, a.n, stage.ctypes.data,
                                         stage.size, cursor.ctypes.data, boff.ctypes.data, bases.ctypes.data,
                                         qt.ctypes.data, rec_off.ctypes.data, a.workers, rcs.ctypes.data)


res = {"dense": [], "packed": [], "packed_batch": []}
for r in range(a.reps + 1):
    for name, f in (("dense", f_dense), ("packed", f_packed)):
        cursor[0] = 0
        t = time.perf_counter()
        assert not any(pool.map(f, range(a.n)))
        if r:
            res[name].append((time.perf_counter() - t) * 1e3)
    cursor[0] = 0
    t = time.perf_counter()
    assert batch_call() == 0 and not rcs.any()
    if r:
        res["packed_batch"].append((time.perf_counter() - t) * 1e3)
print(f"n={a.n} workers={a.workers} blocks/img={blocks} packed bytes/img={cursor[0] / a.n / 1e3:.0f} KB "
      f"dense {blocks * 128 / 1e3:.0f} KB")
for k, v in res.items():
    print(f"{k}: median {np.median(v):.2f} ms  min {min(v):.2f} ms  ({a.n / np.median(v) * 1e3:.0f} img/s)")
