import torch, ctypes, sys, statistics
sys.path.insert(0, '.')
import mmf_amd.hip as hip
lib = hip.load()
dev = torch.device('cuda')
def run(M, N, K, act, iters=30):
    A = torch.randn(M, K, device=dev).half(); W = (torch.randn(N, K, device=dev) * 0.05).half()
    b = torch.randn(N, device=dev); C = torch.empty(M, N, device=dev, dtype=torch.float16)
    f = lambda: hip.check(lib.mmf_gemm_f16_ex(A.data_ptr(), K, W.data_ptr(), K, b.data_ptr(), None, None, 0, C.data_ptr(), N, M, N, K, act, hip.stream_ptr()))
    for _ in range(3): f()
    ts = []
    for r in range(5):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); [f() for _ in range(iters)]; e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters * 1e3)
    return statistics.median(ts)
for (M, N, K) in [(32768, 3072, 768), (12800, 3072, 768), (19712, 2048, 512)]:
    print(M, N, K, {a: round(run(M, N, K, a), 1) for a in (0, 1, 2, 0, 1, 2)})
