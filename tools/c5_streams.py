"""C5 stream-count sweep: hpdct_stream_forward over N pinned 4096^2 frames
with 1..8 HIP streams, fp32 and int8 outputs (frames/s, PCIe GB/s)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-dct-idct_amd"))


def main():
    import torch
    import hpdct
    n, frames = 4096, int(sys.argv[1]) if len(sys.argv) > 1 else 256
    pool = []
    for k in range(8):
        t = torch.empty((n, n), dtype=torch.uint8).pin_memory()
        t.copy_(torch.from_numpy(hpdct.fill_rand_u8(n * n, 42 + k).reshape(n, n)))
        pool.append(t)
    for dtype, ob in ((torch.float32, 4), (torch.int8, 1)):
        outs = [torch.empty((n, n), dtype=dtype).pin_memory() for _ in range(8)]
        fr = [pool[i % 8] for i in range(frames)]
        oo = [outs[i % 8] for i in range(frames)]
        for ns in (1, 2, 3, 4, 6, 8):
            hpdct.stream_forward(fr[:8], oo[:8], nstreams=ns)
            ms = min(hpdct.stream_forward(fr, oo, nstreams=ns) for _ in range(2))
            moved = frames * n * n * (1 + ob)
            print(f"{str(dtype):14s} streams={ns}  {frames / (ms * 1e-3):8.1f} frames/s  "
                  f"{moved / (ms * 1e-3) / 1e9:6.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
