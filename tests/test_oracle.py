"""CPU checks of the oracle itself (it is the checker of every GPU test).

Pins: glibc rand() (the reference's input stream, benchmark_newAppr.cu:46-51),
the T/Q tables (main_newAppr.cu:60-81), the reference's own host conversions
(utils.cu:10-24, run here from oracle/_ref), known answers that follow from
the algorithm, and the committed golden fixtures (tests/golden/).
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(GOLD, "golden.json")) as fh:
        return json.load(fh)


# ---------------------------------------------------------------- input stream
def test_rand_matches_glibc(oracle, golden):
    libc = ctypes.CDLL("libc.so.6")
    for seed in (42, 0, 1, 7, 2**31 - 1, 2**32 - 1):
        g = (ctypes.c_uint32 * 35)()
        oracle.lib().oracle_srand(g, seed)
        libc.srand(ctypes.c_uint(seed))
        assert all(oracle.lib().oracle_rand(g) == libc.rand() for _ in range(1000)), seed
    a = oracle.rand_u8(64, 42)
    assert a.tolist() == golden["rand42_mod256_first64"]
    # first 16 values of rand()%256 after srand(42)
    assert a[:16].tolist() == [70, 100, 49, 41, 100, 134, 237, 156, 215, 31, 194, 7, 37, 72, 32, 162]


def test_hash_generator_is_stateless(oracle):
    full = oracle.hash_u8(10000, seed=42)
    part = oracle.hash_u8(3000, seed=42, first_index=7000)
    assert np.array_equal(full[7000:], part)
    assert 120 < full.mean() < 135


# ---------------------------------------------------------------- tables
def test_transform_bits_and_orthonormality(oracle):
    t = oracle.default_transform()
    bits = sorted(set(np.abs(t).view(np.uint32).ravel().tolist()))
    # a, b, 0.5, 2b, 2a as float32 bit patterns
    assert bits == [0, 0x3E64F92E, 0x3EB504F3, 0x3EE4F92E, 0x3F000000, 0x3F3504F3]
    assert int((t != 0).sum()) == 44
    t64 = t.astype(np.float64)
    assert np.abs(t64 @ t64.T - np.eye(8)).max() < 4e-8


def test_quant_table(oracle):
    q = oracle.default_quant()
    assert q[0].tolist() == [16, 11, 10, 16, 24, 40, 51, 61]
    assert q[7].tolist() == [72, 92, 95, 98, 112, 100, 103, 99]


# ---------------------------------------------------------------- known answers
def test_kat_all_128_is_zero(oracle):
    img = np.full((16, 24), 128, np.uint8)
    assert not oracle.fdct(img, quant=False).any()
    assert not oracle.fdct(img).any()


@pytest.mark.parametrize("v", [0, 1, 100, 127, 128, 129, 200, 255])
def test_kat_constant_tile_dc(oracle, v):
    img = np.full((8, 8), v, np.uint8)
    c = oracle.fdct(img, quant=False)
    # DC = 8 (v - 128) up to fp32 rounding of a^2; every AC ~ 0
    assert abs(c[0, 0] - 8.0 * (v - 128)) <= 1e-4 * max(1, abs(v - 128))
    ac = c.copy()
    ac[0, 0] = 0
    assert np.abs(ac).max() < 1e-4
    q = oracle.fdct(img)
    assert q[0, 0] == np.round(8.0 * (v - 128) / 16.0) or abs(q[0, 0] - 8.0 * (v - 128) / 16.0) <= 0.5 + 1e-6


def test_kat_impulse_is_outer_product(oracle):
    t = oracle.default_transform().astype(np.float64)
    for (i, j) in [(0, 0), (3, 5), (7, 2)]:
        img = np.full((8, 8), 128, np.uint8)
        img[i, j] = 228  # +100 impulse
        c = oracle.fdct(img, quant=False).astype(np.float64)
        expect = 100.0 * np.outer(t[:, i], t[:, j])
        assert np.abs(c - expect).max() < 1e-4


def test_kat_extremes_and_int8_bound(oracle):
    # the pattern that maximises |C[v][u]| is sign(T_v (x) T_u): |q| stays << 127
    t = oracle.default_transform()
    worst = 0.0
    for v in range(8):
        for u in range(8):
            s = np.sign(np.outer(t[v], t[u]))
            for sign in (1, -1):
                img = np.where(sign * s > 0, 255, 0).astype(np.uint8)
                worst = max(worst, float(np.abs(oracle.fdct(img)).max()))
    assert worst <= 98.0  # SURVEY.md section 8a row a4 bound, max at (0,2)


def test_tiles_are_independent(oracle):
    img = oracle.rand_u8(32 * 48).reshape(32, 48)
    base = oracle.fdct(img)
    img2 = img.copy()
    img2[8:16, 16:24] ^= 0x5A
    c2 = oracle.fdct(img2)
    diff = base != c2
    diff[8:16, 16:24] = False
    assert not diff.any()


def test_roundtrip_properties(oracle):
    img = oracle.rand_u8(256 * 256).reshape(256, 256)
    rt = oracle.idct(oracle.fdct(img, quant=False), dequant=False)
    assert np.abs(rt - img).max() < 1e-4  # 3.8e-5 measured
    ones = np.ones((8, 8), np.float32)
    rt1 = oracle.idct(oracle.fdct(img, Q=ones), Q=ones)
    assert np.abs(rt1 - img).max() < 1.5


def test_u8_and_f32_inputs_agree(oracle):
    img = oracle.rand_u8(64 * 64, seed=3).reshape(64, 64)
    assert np.array_equal(oracle.fdct(img).view(np.uint32), oracle.fdct(img.astype(np.float32)).view(np.uint32))


# ---------------------------------------------------------------- golden fixtures
def test_golden_c1(oracle, golden):
    g = golden["configs"]["c1_256"]
    img = oracle.rand_u8(256 * 256).reshape(256, 256)
    assert sha(img) == g["input_sha256"]
    q = oracle.fdct(img)
    assert sha(q) == g["q_f32_sha256"]
    assert np.array_equal(q.astype(np.int8), np.load(os.path.join(GOLD, "c1_256_seed42_q_i8.npy")))
    assert sha(oracle.fdct(img, quant=False)) == g["coef_f32_sha256"]
    assert sha(oracle.idct(q)) == g["roundtrip_f32_sha256"]
    # the arithmetic is order/FMA sensitive
    assert int((oracle.fdct(img, nofma=True) != q).sum()) == g["q_nofma_mismatches"] == 36
    assert int((oracle.fdct(img, recip=True) != q).sum()) == g["q_recip_mismatches"] == 5


def test_golden_rt64(oracle):
    img = oracle.rand_u8(256 * 256).reshape(256, 256)[:64, :64].copy()
    a = oracle.idct(oracle.fdct(img, quant=False), dequant=False)
    b = oracle.idct(oracle.fdct(img))
    assert np.array_equal(a.view(np.uint32), np.load(os.path.join(GOLD, "rt64_unquant_f32.npy")).view(np.uint32))
    assert np.array_equal(b.view(np.uint32), np.load(os.path.join(GOLD, "rt64_quant_f32.npy")).view(np.uint32))


def test_golden_c2(oracle, golden):
    g = golden["configs"]["c2_1024"]
    img = oracle.rand_u8(1024 * 1024).reshape(1024, 1024)
    assert sha(img) == g["input_sha256"]
    q = oracle.fdct(img)
    assert sha(q) == g["q_f32_sha256"]
    rt = oracle.idct(q)
    assert sha(rt) == g["roundtrip_f32_sha256"]
    peen, mse = oracle.quality(img.astype(np.float32), rt)
    assert abs(mse - g["mse_f32"]) < 1e-9 and abs(peen - g["peen_f32"]) < 1e-9


@pytest.mark.slow
def test_golden_c3(oracle, golden):
    g = golden["configs"]["c3_8192"]
    img = oracle.rand_u8(8192 * 8192).reshape(8192, 8192)
    assert sha(img) == g["input_sha256"]
    assert sha(oracle.fdct(img)) == g["q_f32_sha256"]


# ---------------------------------------------------------------- the reference's own code
def test_conversions_match_reference_fixture(oracle):
    z = np.load(os.path.join(GOLD, "ref_utils_convert.npz"))
    assert np.array_equal(z["f32_out"], z["u8_in"].astype(np.float32))
    assert np.array_equal(oracle.to_u8(z["f32_in"]), z["u8_out"])


def test_conversions_match_reference_live(oracle):
    R = oracle.ref_utils()
    if R is None:
        pytest.skip("oracle/_ref not built (reference sources absent)")
    xs = np.concatenate([np.random.default_rng(0).uniform(-50, 300, 20000).astype(np.float32),
                         np.array([np.nan, np.inf, -np.inf, -0.0, 255.999], np.float32)])
    uc = np.empty(xs.size, np.uint8)
    R._Z21convertToUnsignedCharPKfPhm(xs.ctypes.data, uc.ctypes.data, xs.size)
    assert np.array_equal(oracle.to_u8(xs), uc)


# ---------------------------------------------------------------- cublasDCTv2 order
def test_row_first_order(oracle):
    """main_cublass_2.cu:228-235/288-295: the same transform with the row pass
    first.  Unquantised it agrees with the HpApprDCT order to fp32 rounding;
    quantised, values near a rounding boundary may move by one step."""
    img = oracle.rand_u8(256 * 256).reshape(256, 256)
    a = oracle.fdct(img, quant=False)
    b = oracle.fdct(img, quant=False, row_first=True)
    assert 0 < np.abs(a - b).max() < 1e-4
    qa, qb = oracle.fdct(img), oracle.fdct(img, row_first=True)
    assert np.abs(qa - qb).max() <= 1.0 and 0 < int((qa != qb).sum()) < 200
    rt = oracle.idct(b, dequant=False, row_first=True)
    assert np.abs(rt - img).max() < 1e-4
    # separable transform of an impulse: identical in both orders
    imp = np.full((8, 8), 128, np.uint8)
    imp[2, 5] = 200
    assert np.array_equal(oracle.fdct(imp, quant=False), oracle.fdct(imp, quant=False, row_first=True)) or \
        np.abs(oracle.fdct(imp, quant=False) - oracle.fdct(imp, quant=False, row_first=True)).max() < 1e-5


@pytest.mark.parametrize("h,w,threads", [(64, 96, 3), (8, 40, 4), (256, 256, 16)])
def test_fdct_threads_equals_fdct(oracle, h, w, threads):
    """The all-cores CPU baseline (bench.py cpu_baseline.all_cores) bands the
    frame by tile rows; tiles are independent, so it is bit-identical."""
    img = oracle.rand_u8(h * w, 7).reshape(h, w)
    a = oracle.fdct_threads(img, threads)
    b = oracle.fdct(img)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_rt_sse_f32_definition_known_answers():
    """oracle_rt_sse_f32_fx (the round trip's sse_f32 definition, checked bit
    for bit against the GPU in tests/test_gpu_roundtrip.py): known answers."""
    import oracle
    img = np.full((16, 24), 100, dtype=np.uint8)
    assert oracle.rt_sse_f32_fx(img, img.astype(np.float32)) == 0
    # e = -1 everywhere: each of the 4 chains of a tile holds 16, a tile 64
    assert oracle.rt_sse_f32_fx(img, img.astype(np.float32) + 1.0) == 6 * 64 * 65536
    # e = 0.5 at one pixel only
    r = img.astype(np.float32)
    r[3, 5] -= 0.5
    assert oracle.rt_sse_f32_fx(img, r) == 65536 // 4
    # a non-finite chain sets bit 63 and adds nothing
    r[0, 0] = np.inf
    v = oracle.rt_sse_f32_fx(img, r)
    assert v >> 63 == 1 and (v & ((1 << 63) - 1)) == 65536 // 4
