import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "cuda-dct-idct_amd"))
import torch, hpdct
dev = torch.device("cuda", 0); stream = torch.cuda.current_stream()
H = W = 8192
img = [torch.empty((H, W), dtype=torch.uint8, device=dev) for _ in range(16)]
for s, t in enumerate(img): hpdct.fill_hash_u8(t, seed=3 + s)
coef = [torch.empty((H, W), dtype=torch.float32, device=dev) for _ in range(2)]
rf = [torch.empty((H, W), dtype=torch.float32, device=dev) for _ in range(2)]
r8 = [torch.empty((H, W), dtype=torch.uint8, device=dev) for _ in range(2)]
sums = torch.zeros(3, dtype=torch.int64, device=dev)
def region(calls, reps):
    for c in calls[:4]: c()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for i in range(reps): calls[i % len(calls)]()
    b.record(stream); torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps
warm = hpdct.bind("fwd", img[0], coef[0], stream=stream)
for _ in range(20000): warm()
torch.cuda.synchronize()
for rep in range(2):
    u8 = [hpdct.bind_roundtrip(img[s], coef[s % 2], r8[s % 2], sums, stream=stream) for s in range(16)]
    f32 = [hpdct.bind_roundtrip(img[s], coef[s % 2], rf[s % 2], sums, stream=stream) for s in range(16)]
    nos = [hpdct.bind_roundtrip(img[s], coef[s % 2], rf[s % 2], None, stream=stream) for s in range(16)]
    print("u8 recon + sums %.2f us | f32 recon + sums %.2f us | f32 recon no sums %.2f us" % (region(u8, 600), region(f32, 600), region(nos, 600)), flush=True)
