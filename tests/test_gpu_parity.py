"""GPU parity: the gfx950 kernels against the CPU oracle, through the C-ABI.

Bar: quantised coefficients and every fp32 plane BIT-EXACT (the oracle
restates the reference's fp32 FMA chain, IEEE division and roundf), compared
as uint32 bit patterns (so -0.0 must match too).  NaN outputs compare by
position (payload bits are not part of the contract).
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(np.where(na, 0, a.view(np.uint32)), np.where(nb, 0, b.view(np.uint32)))


def mismatches(a, b):
    return int((np.ascontiguousarray(a, np.float32).view(np.uint32) != np.ascontiguousarray(b, np.float32).view(np.uint32)).sum())


@pytest.fixture(autouse=True, params=["tile", "octet", "duo"])
def mapping(request, hp, monkeypatch):
    """Every parity case runs under each forced work mapping (one, eight or
    two lanes per tile; two: the fp32 -> fp32 kernels and, since round 6, the
    uint8 -> quantised fp32 forward of whole 32-tile runs); child processes
    inherit HPDCT_MAPPING.  AUTO picks among these per frame size."""
    monkeypatch.setenv("HPDCT_MAPPING", request.param)
    hp.set_mapping(request.param)
    yield request.param
    hp.set_mapping("auto")


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(GOLD, "golden.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def c1(oracle):
    return oracle.rand_u8(256 * 256, 42).reshape(256, 256)


def to_dev(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def to_host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


# --------------------------------------------------------------------- forward
def test_c1_forward_u8_f32_bitexact(hp, oracle, dev, c1, golden):
    q = to_host(hp.forward(to_dev(c1, dev)))
    ref = oracle.fdct(c1)
    assert mismatches(q, ref) == 0
    assert sha(q) == golden["configs"]["c1_256"]["q_f32_sha256"]


def test_c1_forward_f32_input_bitexact(hp, oracle, dev, c1, golden):
    img = c1.astype(np.float32)
    t = to_dev(img, dev)
    q = to_host(hp.forward(t))
    assert sha(q) == golden["configs"]["c1_256"]["q_f32_sha256"]
    assert np.array_equal(to_host(t), img)  # native API does not mutate


def test_c1_forward_int8_matches_golden(hp, dev, c1):
    import torch
    q = to_host(hp.forward(to_dev(c1, dev), out_dtype=torch.int8))
    assert np.array_equal(q, np.load(os.path.join(GOLD, "c1_256_seed42_q_i8.npy")))


def test_forward_unquantised_bitexact(hp, oracle, dev, c1, golden):
    c = to_host(hp.forward(to_dev(c1, dev), quantise=False))
    assert sha(c) == golden["configs"]["c1_256"]["coef_f32_sha256"]
    c32 = to_host(hp.forward(to_dev(c1.astype(np.float32), dev), quantise=False))
    assert bits_equal(c32, oracle.fdct(c1, quant=False))


def test_forward_no_level_shift(hp, oracle, dev, c1):
    c = to_host(hp.forward(to_dev(c1, dev), quantise=False, level_shift=False))
    assert bits_equal(c, oracle.fdct(c1, quant=False, shift=False))


def test_runtime_transform_equals_builtin(hp, oracle, dev, c1):
    # the caller's T (device buffer) takes the dense-FMA kernel; same bits
    T = to_dev(hp.default_transform(), dev)
    a = to_host(hp.forward(to_dev(c1, dev), transform=T))
    b = to_host(hp.forward(to_dev(c1.astype(np.float32), dev), transform=T))
    ref = oracle.fdct(c1)
    assert bits_equal(a, ref) and bits_equal(b, ref)


def test_builtin_immediates_equal_reference_text_tables(hp, dev, c1):
    """The built-in T (instruction immediates, zero terms skipped) against
    T and Q as extracted from main_newAppr.cu:60-81's text
    (tests/golden/ref_tables.json), passed as the caller's T / Q (all 64
    terms as runtime operands, IEEE division): bit-identical coefficients
    and reconstructions."""
    import torch
    doc = json.load(open(os.path.join(GOLD, "ref_tables.json")))["tables"]
    T = np.array(doc["main_newAppr.cu:73"]["bits"], np.uint32).view(np.float32).reshape(8, 8)
    Q = np.array(doc["main_newAppr.cu:60"]["bits"], np.uint32).view(np.float32).reshape(8, 8)
    builtin = to_host(hp.forward(to_dev(c1, dev)))
    builtin8 = to_host(hp.forward(to_dev(c1, dev), out_dtype=torch.int8))
    hp.set_quant_table(Q)
    try:
        ext = to_host(hp.forward(to_dev(c1, dev), transform=to_dev(T, dev)))
        ext_inv = to_host(hp.inverse(to_dev(ext, dev), transform=to_dev(T, dev)))
    finally:
        hp.set_quant_table(None)
    assert bits_equal(builtin, ext)
    assert np.array_equal(builtin8.astype(np.float32), ext)
    assert bits_equal(to_host(hp.inverse(to_dev(builtin, dev))), ext_inv)


def test_custom_transform_and_quant(hp, oracle, dev, c1):
    rng = np.random.default_rng(5)
    T = np.linalg.qr(rng.standard_normal((8, 8)))[0].astype(np.float32)
    Q = rng.integers(1, 120, (8, 8)).astype(np.float32)
    hp.set_quant_table(Q)
    try:
        got = to_host(hp.forward(to_dev(c1, dev), transform=to_dev(T, dev)))
        got32 = to_host(hp.forward(to_dev(c1.astype(np.float32), dev), transform=to_dev(T, dev)))
        builtin = to_host(hp.forward(to_dev(c1, dev)))
    finally:
        hp.set_quant_table(None)
    assert bits_equal(got, oracle.fdct(c1, T=T, Q=Q))
    assert bits_equal(got32, oracle.fdct(c1, T=T, Q=Q))
    assert bits_equal(builtin, oracle.fdct(c1, Q=Q))


@pytest.mark.parametrize("qtab", ["fractional", "large", "ones", "max255"])
def test_quant_table_paths(hp, oracle, dev, c1, qtab):
    """Integer tables in 1..255 take the verified 3-op quotient, anything else
    IEEE division: both must equal the oracle (IEEE C/Q) bit for bit."""
    rng = np.random.default_rng(11)
    Q = {"fractional": rng.uniform(1.0, 50.0, (8, 8)),
         "large": rng.integers(200, 5000, (8, 8)),
         "ones": np.ones((8, 8)),
         "max255": np.full((8, 8), 255.0)}[qtab].astype(np.float32)
    hp.set_quant_table(Q)
    try:
        got = to_host(hp.forward(to_dev(c1, dev)))
        got_nq = to_host(hp.forward(to_dev(np.full((16, 16), 255, np.uint8), dev)))
    finally:
        hp.set_quant_table(None)
    assert bits_equal(got, oracle.fdct(c1, Q=Q))
    assert bits_equal(got_nq, oracle.fdct(np.full((16, 16), 255, np.uint8), Q=Q))


SHAPES = [(8, 8), (8, 16), (16, 8), (24, 40), (8, 4096), (520, 8), (1000, 1008), (72, 2056)]


@pytest.mark.parametrize("h,w", SHAPES)
def test_forward_shapes(hp, oracle, dev, h, w):
    img = np.random.default_rng(h * 7919 + w).integers(0, 256, (h, w), dtype=np.uint8)
    assert bits_equal(to_host(hp.forward(to_dev(img, dev))), oracle.fdct(img))
    assert bits_equal(to_host(hp.forward(to_dev(img.astype(np.float32), dev))), oracle.fdct(img))


@pytest.mark.parametrize("h,w", SHAPES)
def test_fp32_paths_shapes(hp, oracle, dev, h, w):
    """Every fp32 -> fp32 kernel at ragged shapes (partial waves, tile rows
    narrower than a wave's tiles, waves straddling tile rows): the inverse, the
    forward with the X-128 write-back, and the cublasDCTv2 order both ways
    with its write-backs (row-first duo kernel unless the mapping is TILE)."""
    img = np.random.default_rng(h * 31 + w).integers(0, 256, (h, w)).astype(np.float32)
    q = oracle.fdct(img)
    assert bits_equal(to_host(hp.inverse(to_dev(q, dev))), oracle.idct(q))
    x = to_dev(img, dev)
    got = to_host(hp.forward(x, writeback_shift=True))
    assert bits_equal(got, q)
    assert bits_equal(to_host(x), img - 128.0)
    x = to_dev(img, dev)
    qr = to_host(hp.forward(x, row_first=True, writeback_shift=True))
    assert bits_equal(qr, oracle.fdct(img, row_first=True))
    assert bits_equal(to_host(x), img - 128.0)
    qd = to_dev(qr, dev)
    rr = to_host(hp.inverse(qd, row_first=True, writeback_dequant=True))
    assert bits_equal(rr, oracle.idct(qr, row_first=True))
    qtab = np.tile(oracle.default_quant(), (h // 8, w // 8))
    assert bits_equal(to_host(qd), qr * qtab)


def test_forward_extremes(hp, oracle, dev):
    t = oracle.default_transform()
    tiles = []
    for v in range(8):
        for u in range(8):
            s = np.sign(np.outer(t[v], t[u]))
            tiles.append(np.where(s > 0, 255, 0))
            tiles.append(np.where(s > 0, 0, 255))
    tiles += [np.zeros((8, 8)), np.full((8, 8), 255), np.full((8, 8), 128)]
    img = np.concatenate(tiles, axis=1).astype(np.uint8)  # 8 x (8*131)
    img = np.ascontiguousarray(img)
    q = to_host(hp.forward(to_dev(img, dev)))
    assert bits_equal(q, oracle.fdct(img))
    assert np.abs(q).max() <= 98
    import torch
    q8 = to_host(hp.forward(to_dev(img, dev), out_dtype=torch.int8))
    assert np.array_equal(q8, oracle.fdct(img).astype(np.int8))


def test_forward_nonfinite_fp32_input(hp, oracle, dev):
    img = np.random.default_rng(1).uniform(-1e3, 1e3, (16, 32)).astype(np.float32)
    img[1, 2] = np.inf
    img[9, 20] = np.nan
    img[12, 5] = -np.inf
    img[3, 30] = 3.0e38
    img[5, 17] = 1e-42  # denormal
    got = to_host(hp.forward(to_dev(img, dev)))
    assert bits_equal(got, oracle.fdct(img))
    got = to_host(hp.forward(to_dev(img, dev), quantise=False))
    assert bits_equal(got, oracle.fdct(img, quant=False))


@pytest.mark.parametrize("lo,hi", [(0.0, 255.0), (-700.0, 700.0), (-3000.0, 3000.0)])
def test_fp32_input_quotient_range_check(hp, oracle, dev, lo, hi):
    """fp32 input over three coefficient ranges: every |C| within the 3-op
    quotient's verified |C| <= 4096 (pixel values), a mix, and mostly beyond
    it.  fp32 input with an integer 1..255 table takes the checked 3-op
    quotient per output row in the duo kernels (kVarFastDivChecked): rows
    whose |C| all stay <= 4096 use it, any other row IEEE division, so the
    three ranges drive both branches.  Bit-exact with the built-in and with
    the caller's T."""
    import torch
    img = np.random.default_rng(7).uniform(lo, hi, (256, 1024)).astype(np.float32)
    if lo == 0.0:
        img = np.round(img)
    ref = oracle.fdct(img)
    assert bits_equal(to_host(hp.forward(to_dev(img, dev))), ref)
    T = torch.from_numpy(oracle.default_transform()).to(dev)
    assert bits_equal(to_host(hp.forward(to_dev(img, dev), transform=T)), ref)


def test_batch_of_frames(hp, oracle, dev):
    frames = np.random.default_rng(2).integers(0, 256, (3, 64, 128), dtype=np.uint8)
    got = to_host(hp.forward(to_dev(frames, dev)))
    for f in range(3):
        assert bits_equal(got[f], oracle.fdct(frames[f]))


def test_tile_independence(hp, dev, c1):
    a = to_host(hp.forward(to_dev(c1, dev)))
    img = c1.copy()
    img[64:72, 128:136] = 255 - img[64:72, 128:136]
    b = to_host(hp.forward(to_dev(img, dev)))
    d = a != b
    d[64:72, 128:136] = False
    assert not d.any()


def test_non_default_stream_and_determinism(hp, dev, c1):
    import torch
    s = torch.cuda.Stream()
    x = to_dev(c1, dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        a = hp.forward(x)
    s.synchronize()
    b = hp.forward(x, stream=s)
    s.synchronize()
    assert torch.equal(a, b)


def test_misaligned_pointer_rejected(hp, dev):
    import torch
    buf = torch.zeros(8 * 8 + 1, dtype=torch.float32, device=dev)
    with pytest.raises(hp.HpdctError) as e:
        hp.forward(buf[1:].view(8, 8))
    assert e.value.status == 1


# --------------------------------------------------------------------- inverse
def test_c1_inverse_f32_bitexact(hp, oracle, dev, c1, golden):
    q = oracle.fdct(c1)
    r = to_host(hp.inverse(to_dev(q, dev)))
    assert sha(r) == golden["configs"]["c1_256"]["roundtrip_f32_sha256"]
    assert bits_equal(r, oracle.idct(q))


def test_inverse_outputs_and_inputs(hp, oracle, dev, c1):
    import torch
    q = oracle.fdct(c1)
    ref = oracle.idct(q)
    ref8 = oracle.to_u8(ref)
    assert np.array_equal(to_host(hp.inverse(to_dev(q, dev), out_dtype=torch.uint8)), ref8)
    qi8 = to_dev(q.astype(np.int8), dev)
    assert bits_equal(to_host(hp.inverse(qi8)), ref)
    assert np.array_equal(to_host(hp.inverse(qi8, out_dtype=torch.uint8)), ref8)


def test_inverse_unquantised_and_runtime_T(hp, oracle, dev, c1):
    c = oracle.fdct(c1, quant=False)
    r = to_host(hp.inverse(to_dev(c, dev), dequantise=False))
    assert bits_equal(r, oracle.idct(c, dequant=False))
    assert np.abs(r - c1).max() < 1e-4
    T = to_dev(hp.default_transform(), dev)
    r2 = to_host(hp.inverse(to_dev(c, dev), dequantise=False, transform=T))
    assert bits_equal(r2, r)
    rng = np.random.default_rng(9)
    Tc = np.linalg.qr(rng.standard_normal((8, 8)))[0].astype(np.float32)
    q = oracle.fdct(c1, T=Tc)
    assert bits_equal(to_host(hp.inverse(to_dev(q, dev), transform=to_dev(Tc, dev))), oracle.idct(q, T=Tc))


def test_golden_rt64(hp, dev, c1):
    small = np.ascontiguousarray(c1[:64, :64])
    a = to_host(hp.inverse(hp.forward(to_dev(small, dev), quantise=False), dequantise=False))
    b = to_host(hp.inverse(hp.forward(to_dev(small, dev))))
    assert bits_equal(a, np.load(os.path.join(GOLD, "rt64_unquant_f32.npy")))
    assert bits_equal(b, np.load(os.path.join(GOLD, "rt64_quant_f32.npy")))


# --------------------------------------------------------------------- compat surface
_COMPAT_SCRIPT = r"""
import sys, numpy as np, torch
sys.path[:0] = [{pkg!r}, {orc!r}]
import hpdct, oracle
dev = torch.device("cuda:0")
c1 = oracle.rand_u8(256 * 256, 42).reshape(256, 256)
img = torch.from_numpy(c1.astype(np.float32)).to(dev)
T = torch.from_numpy(hpdct.default_transform()).to(dev)
res = torch.empty_like(img)
hpdct.dct_all_blocks_cuda(img, 256, 256, T, res)
q = oracle.fdct(c1)
assert np.array_equal(res.cpu().numpy().view(np.uint32), q.view(np.uint32)), "forward"
assert np.array_equal(img.cpu().numpy(), c1.astype(np.float32) - 128.0), "in-place X-128"
out = torch.empty_like(img)
hpdct.idct_all_blocks_cuda(res, 256, 256, T, out)
assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle.idct(q).view(np.uint32)), "inverse"
bad = torch.empty((12, 16), device=dev)
sys.stdout.flush()
hpdct.dct_all_blocks_cuda(bad, 12, 16, T, torch.empty_like(bad))  # must print and exit(EXIT_FAILURE)
print("NOT REACHED")
"""


def test_compat_entry_points():
    """The reference-named C++ entry points (hpdct_compat.h) in a child
    process: they print the timing line and exit() on error, like the
    reference's CHECK_CUDA."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _COMPAT_SCRIPT.format(pkg=os.path.join(root, "cuda-dct-idct_amd"), orc=os.path.join(root, "oracle"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 1, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    assert "DCT (256,256): " in p.stdout and "IDCT (256,256): " in p.stdout and " ms" in p.stdout
    assert "not a positive multiple of 8" in p.stdout
    assert "NOT REACHED" not in p.stdout and "AssertionError" not in p.stderr


# --------------------------------------------------------------------- cublasDCTv2 order
def test_row_first_paths(hp, oracle, dev, c1):
    import torch
    img = c1.astype(np.float32)
    T = to_dev(hp.default_transform(), dev)
    for tr in (None, T):
        q = to_host(hp.forward(to_dev(img, dev), row_first=True, transform=tr))
        assert bits_equal(q, oracle.fdct(c1, row_first=True))
        c = to_host(hp.forward(to_dev(img, dev), row_first=True, quantise=False, transform=tr))
        assert bits_equal(c, oracle.fdct(c1, row_first=True, quant=False))
        qd = to_dev(q, dev)
        r = to_host(hp.inverse(qd, row_first=True, writeback_dequant=True, transform=tr))
        assert bits_equal(r, oracle.idct(q, row_first=True))
        assert bits_equal(to_host(qd), q * oracle.default_quant()[np.arange(256) % 8][:, np.arange(256) % 8])
    # the HpApprDCT inverse with the dequant write-back
    q = oracle.fdct(c1)
    qd = to_dev(q, dev)
    r = to_host(hp.inverse(qd, writeback_dequant=True))
    assert bits_equal(r, oracle.idct(q))
    assert not bits_equal(to_host(qd), q)


_CUBLAS_SCRIPT = r"""
import sys, numpy as np, torch
sys.path[:0] = [{pkg!r}, {orc!r}]
import hpdct, oracle
dev = torch.device("cuda:0")
c1 = oracle.rand_u8(256 * 256, 42).reshape(256, 256)
img = torch.from_numpy(c1.astype(np.float32)).to(dev)
T = torch.from_numpy(hpdct.default_transform()).to(dev)
res = torch.empty_like(img)
hpdct.dct_all_blocks(img, 256, 256, T, res)
q = oracle.fdct(c1, row_first=True)
assert np.array_equal(res.cpu().numpy().view(np.uint32), q.view(np.uint32)), "forward"
assert np.array_equal(img.cpu().numpy(), c1.astype(np.float32) - 128.0), "in-place X-128"
out = torch.empty_like(img)
hpdct.idct_all_blocks(res, 256, 256, T, out)
assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle.idct(q, row_first=True).view(np.uint32)), "inverse"
Q = np.tile(oracle.default_quant(), (32, 32))
assert np.array_equal(res.cpu().numpy(), q * Q), "in-place q*Q"
print("CUBLAS-SURFACE-OK")
"""


def test_cublas_surface_entry_points():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _CUBLAS_SCRIPT.format(pkg=os.path.join(root, "cuda-dct-idct_amd"), orc=os.path.join(root, "oracle"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-2000:])
    assert "CUBLAS-SURFACE-OK" in p.stdout and "DCT (256,256): " in p.stdout and "IDCT (256,256): " in p.stdout


# --------------------------------------------------------------------- C5 host streaming
@pytest.mark.parametrize("nstreams", [1, 3])
def test_stream_forward_host_batch(hp, oracle, dev, nstreams):
    import torch
    h, w = 64, 136
    pool = [torch.from_numpy(oracle.rand_u8(h * w, 42 + k).reshape(h, w)).pin_memory() for k in range(3)]
    frames = [pool[i % 3] for i in range(10)]
    outs = [torch.full((h, w), -7.0).pin_memory() for _ in range(10)]
    ms = hp.stream_forward(frames, outs, nstreams=nstreams)
    assert ms > 0
    for f, o in zip(frames, outs):
        assert bits_equal(o.numpy(), oracle.fdct(f.numpy()))
    outs8 = [torch.zeros((h, w), dtype=torch.int8).pin_memory() for _ in range(4)]
    hp.stream_forward(frames[:4], outs8, nstreams=nstreams)
    for f, o in zip(frames[:4], outs8):
        assert np.array_equal(o.numpy(), oracle.fdct(f.numpy()).astype(np.int8))
    with pytest.raises(hp.HpdctError):
        hp.stream_forward(frames[:2], outs[:1])


# --------------------------------------------------------------------- A/B baselines
@pytest.mark.parametrize("kind", ["reference_3pass", "fastappr_3pass"])
@pytest.mark.parametrize("h,w", [(256, 256), (24, 72), (64, 8)])
def test_baselines_bitexact(hp, oracle, dev, kind, h, w):
    import torch
    img8 = np.random.default_rng(h + w).integers(0, 256, (h, w), dtype=np.uint8)
    img = to_dev(img8.astype(np.float32), dev)
    tmp = torch.empty_like(img)
    res = torch.empty_like(img)
    T = to_dev(hp.default_transform(), dev)
    hp.baseline_forward(kind, img, tmp, res, T)
    assert bits_equal(to_host(res), oracle.fdct(img8))
    assert np.array_equal(to_host(img), img8.astype(np.float32) - 128.0)


# --------------------------------------------------------------------- generator
@pytest.mark.parametrize("n,first", [(4096, 0), (1000, 12345), (17, 3)])
def test_fill_hash_matches_oracle(hp, oracle, dev, n, first):
    import torch
    buf = torch.empty(n, dtype=torch.uint8, device=dev)
    hp.fill_hash_u8(buf, 42, first)
    assert np.array_equal(to_host(buf), oracle.hash_u8(n, 42, first))


@pytest.mark.parametrize("h,w", [(6560, 1280), (4376, 1920)])
def test_video_widths_large_frames(hp, oracle, dev, h, w):
    """Frames large enough for the one-lane-per-tile kernels under AUTO, at
    widths that are not multiples of 512 px: 64-tile sets straddle two tile
    rows (the kVarStraddle variant's two-run staged stores).  Forward to fp32
    and int8, inverse from int8, and the one-pass round trip, all bit-exact."""
    import torch
    img = oracle.hash_u8(h * w, seed=17).reshape(h, w)
    x = to_dev(img, dev)
    q_ref = oracle.fdct(img)
    r_ref = oracle.idct(q_ref)
    q = hp.forward(x)
    assert bits_equal(to_host(q), q_ref)
    q8 = hp.forward(x, torch.empty((h, w), dtype=torch.int8, device=dev))
    assert np.array_equal(to_host(q8), q_ref.astype(np.int8))
    assert bits_equal(to_host(hp.inverse(q8)), r_ref)
    coef, rec8, _ = hp.roundtrip(x, recon_dtype=torch.uint8, sums=False)
    assert bits_equal(to_host(coef), q_ref)
    assert np.array_equal(to_host(rec8), oracle.to_u8(r_ref))
    # fp32 reconstruction: a second LDS-staged plane through the straddling sets
    coef, recf, sums = hp.roundtrip(x, recon_dtype=torch.float32, sums=True)
    assert bits_equal(to_host(coef), q_ref)
    assert bits_equal(to_host(recf), r_ref)
    assert sums["sum_x2"] == int((img.astype(np.int64) ** 2).sum())


@pytest.mark.parametrize("h,w", [(4104, 8200), (6000, 8008), (2048, 16384)])
@pytest.mark.parametrize("qtab", ["jpeg", "fractional"])
def test_capped_packed_forward_large_frames(hp, oracle, dev, h, w, qtab):
    """u8 -> fp32 frames of more than 32 sets per CU take the one-wave,
    residency-capped (7 per CU), packed-fp32 kernel (hpdct_launch.hpp
    fdct_tile_go): 4104 x 8200 (32.1 sets per CU), 6000 x 8008 (45.8); frames
    of up to 32 take the uncapped 1024-thread kernel: 2048 x 16384 (the C4
    8-way slab, exactly 32).  Ragged widths (tiles_x not a multiple of 64:
    sets straddle tile rows) and a ragged last set; the JPEG table (per-position
    forms, 3-op quotient elsewhere) and a fractional table (IEEE division per
    half).  Bit-exact vs the oracle."""
    img = oracle.hash_u8(h * w, seed=h + w).reshape(h, w)
    Q = None
    if qtab == "fractional":
        Q = np.random.default_rng(5).uniform(1.0, 50.0, (8, 8)).astype(np.float32)
        hp.set_quant_table(Q)
    try:
        got = to_host(hp.forward(to_dev(img, dev)))
    finally:
        if Q is not None:
            hp.set_quant_table(None)
    ref = oracle.fdct(img) if Q is None else oracle.fdct(img, Q=Q)
    assert bits_equal(got, ref), mismatches(got, ref)


def test_capped_duo_writebacks_large_frame(hp, oracle, dev):
    """fp32 frames of >= 64 duo waves per CU (here 4096 x 8200: 524,800 tiles,
    16,400 waves of 32 tiles on 256 CUs) take the one-wave, residency-capped
    duo kernels (hpdct_launch.hpp DuoShape): the rows-first forward with the
    X-128 write-back, the rows-first inverse with the q*Q write-back and the
    reference-order inverse with the q*Q write-back; since round 6 also the
    reference-order forward (dct_all_blocks_cuda's kernel, checked quotient)
    with the built-in and the caller's T, with and without its write-back.
    Ragged width (tiles_x = 1025).  Bit-exact, the write-back planes included
    (ADVICE r3)."""
    h, w = 4096, 8200
    img = oracle.hash_u8(h * w, seed=77).reshape(h, w).astype(np.float32)
    ref = oracle.fdct(img)
    T = to_dev(oracle.default_transform(), dev)
    for transform in (None, T):
        x = to_dev(img, dev)
        got = hp.forward(x, transform=transform, writeback_shift=True)
        assert bits_equal(to_host(got), ref), mismatches(to_host(got), ref)
        assert bits_equal(to_host(x), img - np.float32(128))
        got = hp.forward(to_dev(img, dev), transform=transform)
        assert bits_equal(to_host(got), ref), mismatches(to_host(got), ref)
    x = to_dev(img, dev)
    q = hp.forward(x, row_first=True, writeback_shift=True)
    q_ref = oracle.fdct(img, row_first=True)
    assert bits_equal(to_host(q), q_ref), mismatches(to_host(q), q_ref)
    assert bits_equal(to_host(x), img - np.float32(128))
    dq_ref = q_ref * np.tile(oracle.default_quant().astype(np.float32), (h // 8, w // 8))
    qd = q.clone()
    r = hp.inverse(qd, row_first=True, writeback_dequant=True)
    assert bits_equal(to_host(r), oracle.idct(q_ref, row_first=True))
    assert bits_equal(to_host(qd), dq_ref)
    qd = q.clone()
    r = hp.inverse(qd, writeback_dequant=True)
    assert bits_equal(to_host(r), oracle.idct(q_ref))
    assert bits_equal(to_host(qd), dq_ref)


def _hardest_tiles(oracle, per_pos=6, n_tiles=1 << 18, seed=11):
    """Tiles whose unquantised coefficient C at some position (v, u) lies
    closest to a rounding boundary (k + 1/2) * Q of the default table, found by
    the oracle among n_tiles random tiles, plus each position's two
    extreme tiles (|C| at that position's bound): the inputs where a quotient
    form that is not exact would show.  One row of tiles, 8 x (8 * count)."""
    rng = np.random.default_rng(seed)
    w = 8 * n_tiles
    img = rng.integers(0, 256, (8, w), dtype=np.uint8)
    c = oracle.fdct(img, quant=False).reshape(8, n_tiles, 8).transpose(1, 0, 2).reshape(n_tiles, 64)
    q = oracle.default_quant().reshape(64).astype(np.float64)
    frac = np.abs(np.abs(c.astype(np.float64)) / q - np.floor(np.abs(c.astype(np.float64)) / q) - 0.5)
    pick = set()
    for p in range(64):
        pick.update(np.argsort(frac[:, p], kind="stable")[:per_pos].tolist())
    tiles = [img[:, 8 * t:8 * t + 8] for t in sorted(pick)]
    T = oracle.default_transform().astype(np.float64)
    for v in range(8):
        for u in range(8):
            s = np.sign(np.outer(T[v], T[u]))
            for sign in (1, -1):
                tiles.append(np.where(sign * s > 0, 255, 0).astype(np.uint8))
    while len(tiles) % 64:  # whole 64-tile sets: a 512-px multiple width
        tiles.append(rng.integers(0, 256, (8, 8), dtype=np.uint8))
    return np.ascontiguousarray(np.concatenate(tiles, axis=1))


@pytest.fixture(scope="module")
def hardest(oracle):
    img = _hardest_tiles(oracle)
    return img, oracle.fdct(img)


def test_quantiser_hardest_tiles(hp, dev, hardest):
    """The default JPEG table's per-position quantiser forms (kVarJpegQ,
    hpdct_quant_forms.h) and the 6-op form on the tiles nearest a rounding
    boundary at every position and on the extreme tiles: fp32 and int8
    output bit-exact against the oracle's IEEE division + roundf, in every
    mapping (the tile kernels are the ones with the forms)."""
    import torch
    img, ref = hardest
    x = to_dev(img, dev)
    assert bits_equal(to_host(hp.forward(x)), ref), mismatches(to_host(hp.forward(x)), ref)
    got8 = to_host(hp.forward(x, out_dtype=torch.int8))
    assert np.array_equal(got8.astype(np.float32), ref)
    # the same tiles in a frame large enough for the capped packed kernel (> 32 sets per CU)
    h = 8 * (-(-(33 * 256 * 64 * 64) // img.size))
    big = np.ascontiguousarray(np.tile(img, (h // 8, 1)))
    refb = np.tile(ref, (h // 8, 1))
    xb = to_dev(big, dev)
    assert bits_equal(to_host(hp.forward(xb)), refb)
    assert np.array_equal(to_host(hp.forward(xb, out_dtype=torch.int8)).astype(np.float32), refb)
    coef, rec, _ = hp.roundtrip(xb, sums=True)
    assert bits_equal(to_host(coef), refb)


def _retile(strip, tiles_x, tile_rows):
    """The 8 x 8N strip's tiles laid out row-major into a tile_rows x tiles_x
    grid of tiles, cycling through them (tiles are position-independent, so
    the oracle's strip output retiles the same way)."""
    n = strip.shape[1] // 8
    t = strip.reshape(8, n, 8).transpose(1, 0, 2)  # (n, 8, 8)
    idx = np.arange(tile_rows * tiles_x) % n
    g = t[idx].reshape(tile_rows, tiles_x, 8, 8).transpose(0, 2, 1, 3)
    return np.ascontiguousarray(g.reshape(tile_rows * 8, tiles_x * 8))


@pytest.mark.parametrize("mapping", ["tile", "octet"])
def test_quantiser_hardest_tiles_forced_mapping(hp, dev, hardest, mapping):
    """the small hardest-tiles frame under AUTO runs the octet
    kernels; forced to the tile mapping it runs the uncapped 1024-thread tile
    kernels with the JPEG forms (fp32 and int8) and the tile round trip."""
    import torch
    img, ref = hardest
    x = to_dev(img, dev)
    hp.set_mapping(mapping)
    try:
        f32 = to_host(hp.forward(x))
        i8 = to_host(hp.forward(x, out_dtype=torch.int8))
        coef, _, _ = hp.roundtrip(x, sums=True)
        coef = to_host(coef)
    finally:
        hp.set_mapping("auto")
    assert bits_equal(f32, ref), mismatches(f32, ref)
    assert np.array_equal(i8.astype(np.float32), ref)
    assert bits_equal(coef, ref)


@pytest.mark.parametrize("sets_per_cu", [16, 40])
@pytest.mark.parametrize("tiles_x", [77, 512])
def test_quantiser_hardest_tiles_mid_big_ragged(hp, dev, hardest, sets_per_cu, tiles_x):
    """The hardest tiles in frames of 16 sets per CU (the uncapped 1024-thread
    tile kernel) and 40 (the capped one-wave kernels), at a width of 77 tiles
    (every 64-tile set straddles two tile rows: kVarStraddle with kVarJpegQ)
    and of 512 tiles: fp32, int8 and the round trip's coefficients."""
    import torch
    img, ref = hardest
    tile_rows = -(-(sets_per_cu * 256 * 64) // tiles_x)
    big, refb = _retile(img, tiles_x, tile_rows), _retile(ref, tiles_x, tile_rows)
    x = to_dev(big, dev)
    f32 = to_host(hp.forward(x))
    assert bits_equal(f32, refb), mismatches(f32, refb)
    assert np.array_equal(to_host(hp.forward(x, out_dtype=torch.int8)).astype(np.float32), refb)
    coef, _, _ = hp.roundtrip(x, sums=True)
    assert bits_equal(to_host(coef), refb)


# --------------------------------------------------------------------- full-size configs
def test_c2_1024_bitexact(hp, oracle, dev, golden):
    img = oracle.rand_u8(1024 * 1024).reshape(1024, 1024)
    q = to_host(hp.forward(to_dev(img, dev)))
    assert sha(q) == golden["configs"]["c2_1024"]["q_f32_sha256"]
    r = to_host(hp.inverse(to_dev(q, dev)))
    assert sha(r) == golden["configs"]["c2_1024"]["roundtrip_f32_sha256"]


def test_c3_8192_roundtrip(hp, oracle, dev, golden):
    g = golden["configs"]["c3_8192"]
    img = oracle.rand_u8(8192 * 8192).reshape(8192, 8192)
    x = to_dev(img, dev)
    qd = hp.forward(x)
    q = to_host(qd)
    assert sha(q) == g["q_f32_sha256"]
    r = to_host(hp.inverse(qd))
    assert sha(r) == g["roundtrip_f32_sha256"]
    peen, mse = oracle.quality(img.astype(np.float32), r)
    assert abs(mse - g["mse_f32"]) < 1e-6 and abs(peen - g["peen_f32"]) < 1e-6
    assert 370 < mse < 380 and 12.9 < peen < 13.3
    # size-independent properties at full size
    c = hp.forward(x, quantise=False)
    rt = hp.inverse(c, dequantise=False)
    import torch
    assert float((rt - x.float()).abs().max()) < 1e-4
    assert float(qd.abs().max()) <= 98


# --------------------------------------------------------------------- beyond 32-bit indexing
@pytest.mark.parametrize("out", ["f32", "i8"])
def test_beyond_int32_pixel_count(hp, oracle, dev, out):
    """A 32776 x 65536 frame (2^31 + 2^19 pixels): the reference's int indices
    overflow here; every offset in the kernels is 64-bit.  The
    frame is generated on the device by the stateless hash, so the oracle can
    regenerate any 8-row slab; tiles are independent, so crops of the output
    are checked against the oracle on the same crops of the input (top, middle
    and bottom slabs, left and right edges), forward and (fp32) inverse."""
    import torch
    h, w, seed = 32776, 65536, 7
    x = torch.empty((h, w), dtype=torch.uint8, device=dev)
    hp.fill_hash_u8(x, seed=seed)
    y = hp.forward(x, out_dtype=torch.float32 if out == "f32" else torch.int8)
    r = hp.inverse(y) if out == "f32" else None
    torch.cuda.synchronize()
    try:
        for r0 in (0, (h // 16) * 8, h - 8):
            slab = oracle.hash_u8(8 * w, seed=seed, first_index=r0 * w).reshape(8, w)
            for c0 in (0, w - 1024):
                crop = np.ascontiguousarray(slab[:, c0:c0 + 1024])
                q_ref = oracle.fdct(crop)
                got = y[r0:r0 + 8, c0:c0 + 1024].cpu().numpy()
                if out == "f32":
                    assert bits_equal(got, q_ref), (r0, c0)
                    assert bits_equal(r[r0:r0 + 8, c0:c0 + 1024].cpu().numpy(), oracle.idct(q_ref)), (r0, c0)
                else:
                    assert np.array_equal(got.astype(np.float32), q_ref), (r0, c0)
    finally:
        del x, y, r
        torch.cuda.empty_cache()
