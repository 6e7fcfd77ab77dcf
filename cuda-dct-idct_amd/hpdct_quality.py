"""Quality metrics of the DCT/IDCT round trip: the README's accuracy table
(README.md:62-69: PEEN, MSE and compression factor for the standard
quantisation table and for k = 6..10 retained coefficients).  The reference
publishes the numbers but ships no code and no "Circuit" image, so the
definitions are pinned here:

  PEEN  = 100 * sqrt( sum (x - y)^2 / sum x^2 )       (percentage error energy norm)
  MSE   = mean (x - y)^2
  retained-k: keep the first k coefficients of every 8x8 tile in JPEG zig-zag
        order, zero the rest, no quantisation; then the inverse transform
  CF    = size(JPEG q=100 of x) / size(JPEG q=100 of y)  (our reading of the
        README's "Compr. Factor": the reconstruction re-encoded like the
        reference's save_grayscale_jpeg, quality 100, main_newAppr.cu:136;
        unpinned -- no reference code or data to check it against)

x is the original uint8 image, y the reconstruction: fp32 as produced by the
inverse (no clamp, like idct_all_blocks_cuda) or uint8 after the reference's
clamp + truncate (convertToUnsignedChar, utils.cu:18-24).  The transforms run
through the gfx950 kernels (hpdct.forward / hpdct.inverse); only the
zig-zag masking and the reductions use torch.
"""
from __future__ import annotations

import io

import numpy as np

import hpdct

# JPEG zig-zag scan: ZIGZAG[n] = row-major index (8*v + u) of the n-th coefficient
ZIGZAG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
          12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
          35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
          58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]


def retain_mask(k: int) -> np.ndarray:
    """8x8 float32 mask keeping the first k zig-zag coefficients."""
    if not 0 <= k <= 64:
        raise ValueError("k must be in 0..64")
    m = np.zeros(64, np.float32)
    m[ZIGZAG[:k]] = 1.0
    return m.reshape(8, 8)


def peen_mse(x, y):
    """(PEEN %, MSE) of reconstruction y against original x (any shapes equal)."""
    xd = x.double()
    d = xd - y.double()
    se = float((d * d).sum())
    sx = float((xd * xd).sum())
    return (100.0 * (se / sx) ** 0.5 if sx > 0 else 0.0), se / x.numel()


def jpeg_bytes(img_u8: np.ndarray, quality: int = 100) -> int:
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(img_u8), mode="L").save(buf, format="JPEG", quality=quality)
    return buf.tell()


def evaluate(image, retain=None, with_cf: bool = True) -> dict:
    """Round-trip one uint8 image (CUDA tensor, H and W multiples of 8).
    retain=None: the standard path (library quant table); retain=k: keep k
    zig-zag coefficients per tile without quantisation."""
    import torch
    if retain is None:
        q = hpdct.forward(image)
        rec = hpdct.inverse(q)
        nonzero = float((q != 0).float().mean())
    else:
        c = hpdct.forward(image, quantise=False)
        h, w = c.shape[-2], c.shape[-1]
        m = torch.from_numpy(retain_mask(retain)).to(c.device)
        c = (c.view(-1, 8, w // 8, 8) * m.view(1, 8, 1, 8)).reshape(c.shape).contiguous()
        rec = hpdct.inverse(c, dequantise=False)
        nonzero = float((c != 0).float().mean())
    rec8 = hpdct.inverse(q, out_dtype=torch.uint8) if retain is None else \
        hpdct.inverse(c, out_dtype=torch.uint8, dequantise=False)
    peen, mse = peen_mse(image, rec)
    peen8, mse8 = peen_mse(image, rec8)
    out = {"mode": "standard" if retain is None else f"retain{retain}", "peen_pct": peen, "mse": mse,
           "peen_pct_u8": peen8, "mse_u8": mse8, "nonzero_coef_fraction": nonzero}
    if with_cf:
        out["compression_factor"] = jpeg_bytes(image.cpu().numpy()) / jpeg_bytes(rec8.cpu().numpy())
    return out


def readme_table(image, ks=(6, 7, 8, 9, 10)) -> list:
    """The README's accuracy table (README.md:64-69) for one image."""
    return [evaluate(image, retain=k) for k in ks] + [evaluate(image)]
