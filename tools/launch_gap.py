"""Where do the inter-kernel gaps of the timed loop come from?  Times K
back-to-back forward launches (a) alone, (b) with a hipEventRecord after each,
(c) host loop only (no sync), on one 8192^2 frame set."""
import ctypes, os, sys, time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuda-dct-idct_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import hpdct
from bench import HipEvents
dev = torch.device("cuda:0")
n = 8192; K = 400
imgs = [torch.randint(0, 256, (n, n), dtype=torch.uint8, device=dev) for _ in range(4)]
outs = [torch.empty((n, n), dtype=torch.float32, device=dev) for _ in range(4)]
st = torch.cuda.current_stream()
calls = [hpdct.bind("fwd", imgs[i], outs[i], stream=st) for i in range(4)]
hip = HipEvents(st, 1024)
for _ in range(3):
    for i in range(20): calls[i % 4]()
    torch.cuda.synchronize()
    t0 = time.perf_counter(); hip.record(0)
    for i in range(K): calls[i % 4]()
    hip.record(1); torch.cuda.synchronize(); t1 = time.perf_counter()
    a = hip.elapsed(0, 1) / K * 1e3
    ha = (t1 - t0) / K * 1e6
    t0 = time.perf_counter(); hip.record(0)
    for i in range(K):
        calls[i % 4](); hip.record(2 + i)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    b = hip.elapsed(0, 1 + K) / K * 1e3
    hb = (t1 - t0) / K * 1e6
    t0 = time.perf_counter()
    for i in range(K): calls[i % 4]()
    t1 = time.perf_counter(); torch.cuda.synchronize()
    hc = (t1 - t0) / K * 1e6
    print(f"back-to-back {a:.2f} us/launch (host {ha:.2f}) | with events {b:.2f} (host {hb:.2f}) | host enqueue only {hc:.2f} us")
