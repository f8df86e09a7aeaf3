import sys, time, os, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import bench
import mmf_amd.weights as W
from mmf_amd.engine import Engine
eng = Engine(0, W.synthetic_detector_state(0), W.synthetic_clip_state(0), max_batch=256)
t = bench.build_inputs(eng, 256, 0)
out = eng.alloc_outputs(256)
def step():
    eng.analyze_batch(t["rid"], t["rm"], t["cid"], t["cm"], t["img"], out=out)
for _ in range(5): step()
torch.cuda.synchronize()
res = {}
for trial in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter(); step(); t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
    res[f"single_{trial}"] = (round((t1-t0)*1e3, 3), round((t2-t0)*1e3, 3))
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20): step()
t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
res["20_enqueue_ms_per_step"] = round((t1-t0)/20*1e3, 3)
res["20_total_ms_per_step"] = round((t2-t0)/20*1e3, 3)
print(json.dumps(res))
