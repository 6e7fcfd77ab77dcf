#!/usr/bin/env python3
"""Print the README's accuracy table (README.md:64-69: PEEN / MSE /
compression factor for 6..10 retained coefficients and the standard table)
for an image, computed with the gfx950 kernels.  The reference's "Circuit"
image is absent, so by default two synthetic 512x512 frames are used: a
smooth natural-like scene and the benchmark's uniform noise.

usage: python tools/quality_table.py [image.pgm|image.jpg ...]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuda-dct-idct_amd"))


def scene(n=512, seed=7):
    y, x = np.mgrid[0:n, 0:n].astype(np.float64) / n
    rng = np.random.default_rng(seed)
    img = 90 + 60 * np.sin(6 * x + 2 * y) + 40 * np.cos(9 * y * x)
    for _ in range(12):
        cx, cy, r = rng.uniform(0, 1, 2).tolist() + [rng.uniform(0.03, 0.15)]
        img[(x - cx) ** 2 + (y - cy) ** 2 < r * r] += rng.uniform(-70, 70)
    img += rng.normal(0, 2.0, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def load(path):
    from PIL import Image
    a = np.asarray(Image.open(path).convert("L"))
    h, w = a.shape[0] // 8 * 8, a.shape[1] // 8 * 8
    return np.ascontiguousarray(a[:h, :w])


def main():
    import torch
    import hpdct
    import hpdct_quality as Qm
    imgs = {p: load(p) for p in sys.argv[1:]} or {
        "synthetic scene 512x512": scene(),
        "uniform noise 512x512 (srand(42) rand()%256)": hpdct.fill_rand_u8(512 * 512, 42).reshape(512, 512)}
    for name, img in imgs.items():
        x = torch.from_numpy(img).cuda()
        rows = Qm.readme_table(x)
        print(f"\n{name}")
        print(f"{'':22s}" + "".join(f"{r['mode']:>12s}" for r in rows))
        for key, label in (("peen_pct_u8", "PEEN (%)"), ("mse_u8", "MSE"), ("compression_factor", "Compr. Factor")):
            print(f"{label:22s}" + "".join(f"{r[key]:12.2f}" for r in rows))


if __name__ == "__main__":
    main()
