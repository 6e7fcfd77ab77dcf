"""The per-position quantiser forms for the default JPEG table
(csrc/hpdct_quant_forms.h), re-derived on the CPU:

  - the exhaustive proof tests/tools/verify_quant_pos.c is compiled and run:
    for every table position it checks the 3-op forms F (bias 0.49999997) and
    H (bias 0.5) against round(C / Q) (utils_kernels.cu:42) for EVERY fp32 C up
    to that position's bound 128 * |T_v|_1 * |T_u|_1 (* (1 + 2^-16)); its masks
    must equal the ones compiled into the kernels;
  - the bounds themselves are re-derived here from the T norms (numpy), and
    checked against the largest |C| the oracle produces on extreme tiles;
  - a brute-force numpy cross-check of the masks on a sample of C values.
"""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "tools", "verify_quant_pos.c")
HDR = os.path.join(ROOT, "cuda-dct-idct_amd", "csrc", "hpdct_quant_forms.h")


def header_masks():
    text = open(HDR).read()
    f = int(re.search(r"kJpegF = (0x[0-9a-f]+)ull", text).group(1), 16)
    h = int(re.search(r"kJpegH = (0x[0-9a-f]+)ull", text).group(1), 16)
    return f, h


@pytest.fixture(scope="module")
def proof(tmp_path_factory):
    d = tmp_path_factory.mktemp("vqp")
    exe = str(d / "verify_quant_pos")
    r = subprocess.run(["gcc", "-O2", "-mfma", "-msse4.1", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", SRC,
                        "-o", exe, "-lm"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_proof_masks_equal_kernel_masks(proof):
    m = re.search(r"masks F (0x[0-9a-f]+) H (0x[0-9a-f]+)", proof)
    assert m, proof[-500:]
    assert (int(m.group(1), 16), int(m.group(2), 16)) == header_masks()
    assert "F or H at 39 of 64" in proof


def test_bounds_from_t_norms(oracle, proof):
    T = oracle.default_transform().astype(np.float64)
    n = np.abs(T).sum(axis=1)
    bound = 128.0 * np.outer(n, n)
    assert bound.max() == pytest.approx(1024.0, rel=1e-6) and bound.min() == pytest.approx(256.0, rel=1e-6)
    # the proof's printed bounds are these (x (1 + 2^-16))
    rows = re.findall(r"^\s*(\d+)\s+(\d) (\d)\s+(\d+)\s+([\d.]+)", proof, re.M)
    assert len(rows) == 64
    for p, v, u, q, b in rows:
        assert float(b) == pytest.approx(bound[int(v), int(u)] * (1 + 2.0 ** -16), abs=0.006)
        assert float(q) == oracle.default_quant().reshape(-1)[int(p)]


def test_bound_is_attained_not_exceeded(oracle):
    """The worst-case tiles for a few positions (X = 127 where T_v x T_u > 0,
    -128 where < 0, and the sign-flipped one) through the oracle's unquantised
    forward: |C| reaches the bound's order and never exceeds it."""
    T = oracle.default_transform().astype(np.float64)
    n = np.abs(T).sum(axis=1)
    for v, u in [(0, 0), (0, 2), (2, 2), (3, 3), (7, 7), (1, 5)]:
        s = np.sign(np.outer(T[v], T[u]))
        for sign in (1, -1):
            x = np.where(sign * s > 0, 255, 0).astype(np.uint8)
            c = oracle.fdct(x, quant=False)[v, u]
            b = 128.0 * n[v] * n[u] * (1 + 2.0 ** -16)
            assert abs(c) <= b
            assert abs(c) >= 0.99 * 127.0 * n[v] * n[u]


def test_masks_sampled_in_numpy(oracle):
    """Independent of the C proof: on 2^21 random C per position, up to the
    bound, the chosen form equals roundf(C / Q) (numpy fp32; fma emulated in
    float64, exact for these magnitudes: |C * r| < 2^11 with 24+24 product bits
    fits 53 bits, then one rounding to fp32)."""
    f_mask, h_mask = header_masks()
    Q = oracle.default_quant().reshape(-1).astype(np.float32)
    T = oracle.default_transform().astype(np.float64)
    n = np.abs(T).sum(axis=1)
    rng = np.random.default_rng(3)
    for p in range(64):
        form = "F" if (f_mask >> p) & 1 else "H" if (h_mask >> p) & 1 else None
        if form is None:
            continue
        b = 128.0 * n[p // 8] * n[p % 8]
        c = rng.uniform(-b, b, 1 << 21).astype(np.float32)
        # the tie neighbourhoods, where the forms can fail: (k + 1/2) Q and its fp32 neighbours
        k = np.arange(0, int(b // Q[p]) + 1, dtype=np.float32)
        ties = ((k + np.float32(0.5)) * Q[p]).astype(np.float32)
        ties = ties[np.abs(ties) <= b]
        near = np.concatenate([np.nextafter(ties, np.float32(0)), ties, np.nextafter(ties, np.float32(2048))])
        c = np.concatenate([c, near, -near])
        ref = np.round(c / Q[p])  # numpy rounds half to even: fix ties to half-away below
        d = (c / Q[p]).astype(np.float32)
        ref = np.where(np.abs(d - np.trunc(d)) == np.float32(0.5), np.trunc(d) + np.sign(d), np.rint(d))
        r = np.float32(1.0) / Q[p]
        bias = np.float32(0.49999997) if form == "F" else np.float32(0.5)
        exact = c.astype(np.float64) * np.float64(r) + np.copysign(np.float64(bias), c)
        got = np.trunc(exact.astype(np.float32))
        assert np.array_equal(got, ref.astype(np.float32)), (p, form)
