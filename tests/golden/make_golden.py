#!/usr/bin/env python3
"""Regenerate the committed golden fixtures under tests/golden/.

Sources:
  * the CPU oracle (oracle/hpdct_oracle.c) for every DCT/IDCT vector -- these
    pin the GPU path to the oracle and the oracle to itself across changes;
  * the reference's OWN host utilities (/root/reference/utils.cu compiled by
    oracle/Makefile into oracle/_ref/libref_utils.so) for the uint8<->fp32
    conversions -- outputs of the reference run here;
  * glibc rand() (via ctypes) for the synthetic-input stream of
    benchmark_newAppr.cu:46-51.
The reference ships no fixtures of its own.

Also: ref_tables.json -- every Q / T table initialiser in the reference's .cu
sources (quant_matrix / q_matrix / transform_matrix), extracted from the text
and converted as the reference's compiler does, (float)(double)literal, kept as
fp32 bit patterns with file:line.  `--tables-only` regenerates just that file.

Usage: python tests/golden/make_golden.py [--tables-only]
       (needs oracle built and /root/reference present; _ref optional)
"""
import ctypes
import hashlib
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def special_floats() -> np.ndarray:
    v = [0.0, -0.0, 0.4, 0.5, 0.99, 1.0, 1.5, 127.5, 254.99, 255.0, 255.5, 256.0, 300.0, -0.5, -1.0, -300.0,
         1e30, -1e30, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 128.0, 37.9999]
    return np.array(v, np.float32)


REFERENCE = "/root/reference"
TABLE_RE = re.compile(r"float\s+(quant_matrix|q_matrix|transform_matrix)\s*\[[^\]]*\]\s*=\s*\{([^}]*)\}")


def extract_tables(root: str = REFERENCE) -> dict:
    """{"<file>:<line>": {"name", "bits"}} for every table initialiser in the
    reference's .cu text.  bits[i] = fp32 bit pattern of (float)(double)lit."""
    out = {}
    for dirpath, _, files in os.walk(root):
        if "/.git" in dirpath:
            continue
        for fn in sorted(files):
            if not fn.endswith(".cu"):
                continue
            path = os.path.join(dirpath, fn)
            text = open(path, encoding="utf-8", errors="replace").read()
            for m in TABLE_RE.finditer(text):
                lits = [t for t in re.split(r"[\s,]+", m.group(2)) if t]
                assert len(lits) == 64, (path, m.group(1), len(lits))
                vals = np.array([np.float32(float(t.rstrip("fF"))) for t in lits], np.float32)
                line = text.count("\n", 0, m.start()) + 1
                out[f"{os.path.relpath(path, root)}:{line}"] = {
                    "name": m.group(1), "bits": [int(b) for b in vals.view(np.uint32)]}
    return dict(sorted(out.items()))


def write_tables() -> None:
    tabs = extract_tables()
    assert "main_newAppr.cu:60" in tabs and "main_newAppr.cu:73" in tabs, sorted(tabs)
    doc = {"generator": "tests/golden/make_golden.py (extract_tables)",
           "conversion": "(float)(double)literal, as stored by `float x[64] = {...}`",
           "tables": tabs}
    with open(os.path.join(HERE, "ref_tables.json"), "w") as fh:
        json.dump(doc, fh, indent=1)
    print("wrote", os.path.join(HERE, "ref_tables.json"), len(tabs), "tables")


def main() -> None:
    if os.path.isdir(REFERENCE):
        write_tables()
    else:
        print("/root/reference absent: ref_tables.json NOT regenerated", file=sys.stderr)
    if "--tables-only" in sys.argv[1:]:
        return
    manifest = {"generator": "tests/golden/make_golden.py", "seed": 42, "configs": {}}

    # C1: 256x256, srand(42) rand()%256 (benchmark_newAppr.cu:44-51)
    n = 256
    img = O.rand_u8(n * n).reshape(n, n)
    q = O.fdct(img)
    assert np.abs(q).max() <= 127
    np.save(os.path.join(HERE, "c1_256_seed42_q_i8.npy"), q.astype(np.int8))
    raw = O.fdct(img, quant=False)
    rt = O.idct(q)
    manifest["configs"]["c1_256"] = {
        "input_sha256": sha(img),
        "q_f32_sha256": sha(q),
        "coef_f32_sha256": sha(raw),
        "roundtrip_f32_sha256": sha(rt),
        "q_nofma_mismatches": int((O.fdct(img, nofma=True) != q).sum()),
        "q_recip_mismatches": int((O.fdct(img, recip=True) != q).sum()),
        "max_abs_q": float(np.abs(q).max()),
    }

    # 64x64 round-trip planes kept verbatim (fp32)
    small = img[:64, :64].copy()
    np.save(os.path.join(HERE, "rt64_unquant_f32.npy"),
            O.idct(O.fdct(small, quant=False), dequant=False))
    np.save(os.path.join(HERE, "rt64_quant_f32.npy"), O.idct(O.fdct(small)))

    # C2 / C3 digests (the planes are too large to commit)
    for name, n in (("c2_1024", 1024), ("c3_8192", 8192)):
        img = O.rand_u8(n * n).reshape(n, n)
        q = O.fdct(img)
        rt = O.idct(q)
        r8 = O.to_u8(rt)
        peen, mse = O.quality(img.astype(np.float32), rt)
        peen8, mse8 = O.quality(img.astype(np.float32), r8.astype(np.float32))
        x64 = img.astype(np.int64)
        manifest["configs"][name] = {
            "input_sha256": sha(img),
            "q_f32_sha256": sha(q),
            "roundtrip_f32_sha256": sha(rt),
            # the one-pass round trip's uint8 reconstruction (convertToUnsignedChar
            # of R + 128) and its exact quality sums (hpdct_roundtrip_sums)
            "roundtrip_u8_sha256": sha(r8),
            "sum_x2": int((x64 * x64).sum()),
            "sse_u8": int(((x64 - r8.astype(np.int64)) ** 2).sum()),
            "sse_f32_fx": O.rt_sse_f32_fx(img, rt),
            "q_nofma_mismatches": int((O.fdct(img, nofma=True) != q).sum()),
            "q_recip_mismatches": int((O.fdct(img, recip=True) != q).sum()),
            "max_abs_q": float(np.abs(q).max()),
            "peen_f32": peen, "mse_f32": mse, "peen_u8": peen8, "mse_u8": mse8,
        }
        del img, q, rt, r8, x64

    # glibc rand() stream: first 64 values of rand()%256 after srand(42)
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(42)
    manifest["rand42_mod256_first64"] = [libc.rand() % 256 for _ in range(64)]

    # the reference's own conversions, run here (oracle/_ref)
    R = O.ref_utils()
    if R is None:
        print("oracle/_ref not built: reference conversion fixtures NOT regenerated", file=sys.stderr)
    else:
        u8 = np.arange(256, dtype=np.uint8)
        f = np.empty(256, np.float32)
        R._Z14convertToFloatPKhPfm(u8.ctypes.data, f.ctypes.data, 256)
        xs = np.concatenate([special_floats(), np.linspace(-20, 280, 3001, dtype=np.float32)])
        uc = np.empty(xs.size, np.uint8)
        R._Z21convertToUnsignedCharPKfPhm(xs.ctypes.data, uc.ctypes.data, xs.size)
        np.savez(os.path.join(HERE, "ref_utils_convert.npz"), u8_in=u8, f32_out=f, f32_in=xs, u8_out=uc)
        manifest["ref_utils_convert"] = "ref_utils_convert.npz (generated from /root/reference/utils.cu)"

    with open(os.path.join(HERE, "golden.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
