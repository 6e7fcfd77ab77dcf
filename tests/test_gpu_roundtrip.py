"""GPU parity of the one-pass round trip (hpdct_roundtrip_u8, BASELINE config
C3: forward DCT + IDCT with the PEEN/MSE check) against the CPU oracle.

Bar: the coefficients and both reconstructions are BIT-EXACT to
oracle.fdct / oracle.idct / oracle.to_u8 (convertToUnsignedChar) -- the same
contract as the two separate kernels; sum_x2 and sse_u8 are exact integers;
sse_f32 is a sum of per-tile fp32 partials, so it is checked to a relative
REL_SSE_F32 of the float64 sum.
"""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_SSE_F32 = 1e-6
SHAPES = [(8, 8), (8, 16), (16, 8), (24, 40), (8, 4096), (520, 8), (1000, 1008), (72, 2056), (256, 256)]
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(GOLD, "golden.json")) as fh:
        return json.load(fh)


def to_dev(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def to_host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def expected(oracle, img, Q=None):
    q = oracle.fdct(img, Q=Q)
    r = oracle.idct(q, Q=Q)
    r8 = oracle.to_u8(r)
    x = img.astype(np.float64)
    sums = {"sum_x2": int((img.astype(np.int64) ** 2).sum()),
            "sse_u8": int(((img.astype(np.int64) - r8.astype(np.int64)) ** 2).sum()),
            "sse_f32": float(((x - r.astype(np.float64)) ** 2).sum())}
    return q, r, r8, sums


def check_sums(got, want):
    assert got["sum_x2"] == want["sum_x2"]
    assert got["sse_u8"] == want["sse_u8"]
    assert abs(got["sse_f32"] - want["sse_f32"]) <= REL_SSE_F32 * max(want["sse_f32"], 1.0)


@pytest.mark.parametrize("h,w", SHAPES)
def test_roundtrip_shapes(hp, oracle, dev, h, w):
    import torch
    img = np.random.default_rng(h * 131 + w).integers(0, 256, (h, w), dtype=np.uint8)
    q, r, r8, sums = expected(oracle, img)
    x = to_dev(img, dev)
    coef, rec8, got = hp.roundtrip(x, recon_dtype=torch.uint8, sums=True)
    assert bits_equal(to_host(coef), q)
    assert np.array_equal(to_host(rec8), r8)
    check_sums(got, sums)
    coef, recf, none = hp.roundtrip(x, recon_dtype=torch.float32, sums=False)
    assert none is None
    assert bits_equal(to_host(coef), q)
    assert bits_equal(to_host(recf), r)


def test_roundtrip_equals_two_kernels(hp, dev):
    """Same bits as hpdct_forward + hpdct_inverse on the device."""
    import torch
    x = torch.empty((512, 1024), dtype=torch.uint8, device=dev)
    hp.fill_hash_u8(x, seed=3)
    q2 = hp.forward(x)
    r2 = hp.inverse(q2, out_dtype=torch.uint8)
    coef, rec, _ = hp.roundtrip(x, recon_dtype=torch.uint8)
    torch.cuda.synchronize()
    assert torch.equal(coef.view(torch.int32), q2.view(torch.int32))
    assert torch.equal(rec, r2)


def test_roundtrip_sums_only_and_no_sums(hp, oracle, dev):
    img = oracle.rand_u8(64 * 128, 5).reshape(64, 128)
    q, _, _, sums = expected(oracle, img)
    coef, rec, got = hp.roundtrip(to_dev(img, dev), recon_dtype=None, sums=True)
    assert rec is None
    assert bits_equal(to_host(coef), q)
    check_sums(got, sums)
    coef, rec, got = hp.roundtrip(to_dev(img, dev), recon_dtype=None, sums=False)
    assert got is None and rec is None
    assert bits_equal(to_host(coef), q)


def test_roundtrip_sums_repeat_and_streams(hp, oracle, dev):
    """The sums are written (not accumulated) by each launch: the kernel adds
    into the library's slot for the sums pointer and a one-wave kernel moves
    it over the struct, so back-to-back launches of different grid sizes, a
    garbage-filled sums buffer, and launches on a second stream all give this
    frame's totals."""
    import torch
    a = oracle.rand_u8(64 * 128, 11).reshape(64, 128)
    b = oracle.rand_u8(520 * 1008, 12).reshape(520, 1008)
    want_a, want_b = expected(oracle, a)[3], expected(oracle, b)[3]
    xa, xb = to_dev(a, dev), to_dev(b, dev)
    side = torch.cuda.Stream(device=dev)
    bufs = []
    for i, (x, strm) in enumerate([(xa, None), (xb, None), (xa, side), (xa, None), (xb, side), (xb, side),
                                    (xa, None)]):
        buf = torch.full((3,), -1234567, dtype=torch.int64, device=dev)
        coef = torch.empty(x.shape, dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        hp.bind_roundtrip(x, coef, None, buf, stream=side if strm is side else None)()
        bufs.append((buf, want_a if x is xa else want_b))
    torch.cuda.synchronize()
    for buf, want in bufs:
        check_sums(hp.sums_from_buffer(buf), want)


def test_roundtrip_in_a_hip_graph(hp, oracle, dev):
    """hpdct_roundtrip_u8 captured into a HIP graph (the round trip and the
    sums finish kernel, or the memset fallback when the sums pointer is new
    and its slot would need an allocation inside the capture) next to an
    accumulate launch: every replay overwrites the one-pass sums with the
    frame's totals and adds the other frame's into the ring slot once more;
    coefficients are the frame's each time."""
    import torch
    a = oracle.rand_u8(64 * 128, 31).reshape(64, 128)
    b = oracle.rand_u8(72 * 256, 32).reshape(72, 256)
    qa, _, _, want_a = expected(oracle, a)
    want_b = expected(oracle, b)[3]
    xa, xb = to_dev(a, dev), to_dev(b, dev)
    ca = torch.empty(xa.shape, dtype=torch.float32, device=dev)
    cb = torch.empty(xb.shape, dtype=torch.float32, device=dev)
    sums = torch.full((3,), -9, dtype=torch.int64, device=dev)
    ring = torch.zeros(3, dtype=torch.int64, device=dev)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(g):
            hp.bind_roundtrip(xa, ca, None, sums)()
            hp.bind_roundtrip(xb, cb, None, ring, accumulate=True)()
    torch.cuda.synchronize()
    for k in range(1, 4):
        sums.fill_(-1)
        ca.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        check_sums(hp.sums_from_buffer(sums), want_a)
        assert bits_equal(to_host(ca), qa)
        got = hp.sums_from_buffer(ring)
        assert got["sum_x2"] == k * want_b["sum_x2"] and got["sse_u8"] == k * want_b["sse_u8"]


def test_roundtrip_sums_slots_many_buffers(hp, oracle, dev):
    """hpdct_roundtrip_u8's sums slots (hpdct_roundtrip.hip): one per sums
    pointer, handed out from zeroed 256-slot (4 MiB) chunks and left zero by
    every launch's fold.  1100 distinct sums buffers (five chunks) each get the
    frame's totals, then another frame's on reuse; an accumulate launch on a
    slotted buffer goes through the same slot and its fold adds the frame's
    sums to what the buffer holds; an overwrite after it writes the totals
    again."""
    import torch
    a = oracle.rand_u8(64 * 128, 41).reshape(64, 128)
    b = oracle.rand_u8(72 * 256, 42).reshape(72, 256)
    want_a, want_b = expected(oracle, a)[3], expected(oracle, b)[3]
    xa, xb = to_dev(a, dev), to_dev(b, dev)
    ca = torch.empty(xa.shape, dtype=torch.float32, device=dev)
    cb = torch.empty(xb.shape, dtype=torch.float32, device=dev)

    def all_rows(buf, want):
        rows = buf.cpu()
        assert torch.equal(rows, rows[:1].expand_as(rows))
        check_sums(hp.sums_from_buffer(rows[0]), want)

    many = torch.full((1100, 3), -7, dtype=torch.int64, device=dev)
    for i in range(many.shape[0]):
        hp.bind_roundtrip(xa, ca, None, many[i])()
    torch.cuda.synchronize()
    all_rows(many, want_a)
    for i in range(many.shape[0]):
        hp.bind_roundtrip(xb, cb, None, many[i])()
    torch.cuda.synchronize()
    all_rows(many, want_b)
    hp.bind_roundtrip(xa, ca, None, many[5], accumulate=True)()
    torch.cuda.synchronize()
    s5 = hp.sums_from_buffer(many[5])
    assert s5["sum_x2"] == want_a["sum_x2"] + want_b["sum_x2"] and s5["sse_u8"] == want_a["sse_u8"] + want_b["sse_u8"]
    hp.bind_roundtrip(xa, ca, None, many[5])()
    torch.cuda.synchronize()
    check_sums(hp.sums_from_buffer(many[5]), want_a)


def test_roundtrip_accumulate_adds_into_caller_zeroed_sums(hp, oracle, dev):
    """hpdct_roundtrip_u8_accumulate: the round trip and its fold, which adds
    each frame's sums to the caller's struct.  A zeroed ring of per-frame slots gives the per-frame
    totals; two frames sharing a slot give the sum of both (exact integer
    fields, sse_f32 to the fixed-point unit); coefficients and reconstruction
    are the same bits as hpdct_roundtrip_u8."""
    import torch
    a = oracle.rand_u8(64 * 512, 21).reshape(64, 512)
    b = oracle.rand_u8(64 * 512, 22).reshape(64, 512)
    xa, xb = to_dev(a, dev), to_dev(b, dev)
    ring = torch.zeros((3, 3), dtype=torch.int64, device=dev)
    coef = torch.empty(xa.shape, dtype=torch.float32, device=dev)
    rec = torch.empty(xa.shape, dtype=torch.uint8, device=dev)
    hp.bind_roundtrip(xa, coef, rec, ring[0], accumulate=True)()
    hp.bind_roundtrip(xb, torch.empty_like(coef), None, ring[1], accumulate=True)()
    hp.bind_roundtrip(xa, torch.empty_like(coef), None, ring[2], accumulate=True)()
    hp.bind_roundtrip(xb, torch.empty_like(coef), None, ring[2], accumulate=True)()
    torch.cuda.synchronize()
    sa, sb, sab = (hp.sums_from_buffer(ring[i]) for i in range(3))
    check_sums(sa, expected(oracle, a)[3])
    check_sums(sb, expected(oracle, b)[3])
    assert sab["sum_x2"] == sa["sum_x2"] + sb["sum_x2"] and sab["sse_u8"] == sa["sse_u8"] + sb["sse_u8"]
    assert sab["sse_f32"] == sa["sse_f32"] + sb["sse_f32"]
    c2, r2, _ = hp.roundtrip(xa, recon_dtype=torch.uint8, sums=True)
    assert bits_equal(to_host(coef), to_host(c2)) and np.array_equal(to_host(rec), to_host(r2))
    with pytest.raises(hp.HpdctError):
        hp.bind_roundtrip(xa, coef, None, None, accumulate=True)


@pytest.mark.parametrize("qtab", ["jpeg_q90", "fractional", "ones", "max255", "large"])
def test_roundtrip_quant_tables(hp, oracle, dev, qtab):
    """Integer tables in 1..255 whose quotients fit int8 take the packed fast
    path; every other table (fractional, all-ones, > 255) the general one."""
    import torch
    rng = np.random.default_rng(17)
    base = oracle.default_quant()
    Q = {"jpeg_q90": np.clip(np.floor((base * 20 + 50) / 100), 1, 255),
         "fractional": rng.uniform(1.0, 50.0, (8, 8)),
         "ones": np.ones((8, 8)),
         "max255": np.full((8, 8), 255.0),
         "large": rng.integers(200, 5000, (8, 8))}[qtab].astype(np.float32)
    img = rng.integers(0, 256, (64, 192), dtype=np.uint8)
    q, r, r8, sums = expected(oracle, img, Q=Q)
    hp.set_quant_table(Q)
    try:
        coef, rec8, got = hp.roundtrip(to_dev(img, dev), recon_dtype=torch.uint8, sums=True)
        _, recf, _ = hp.roundtrip(to_dev(img, dev), recon_dtype=torch.float32)
        torch.cuda.synchronize()
    finally:
        hp.set_quant_table(None)
    assert bits_equal(to_host(coef), q)
    assert np.array_equal(to_host(rec8), r8)
    assert bits_equal(to_host(recf), r)
    check_sums(got, sums)


def nan_aware_bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(np.where(na, 0, a.view(np.uint32)),
                                                     np.where(nb, 0, b.view(np.uint32)))


@pytest.mark.parametrize("tiny", [1e-40, -1e-40, 1e-38])
def test_roundtrip_extreme_quant_table(hp, oracle, dev, tiny):
    """A subnormal / tiny entry of a caller's table (accepted: finite and
    non-zero) makes round(C/Q) infinite under IEEE division; the reference's
    inverse then multiplies those infinities by the zero entries of T and gets
    NaN (0 * inf).  The one-pass round trip must agree with the oracle and
    with forward + standalone inverse: full chain for such waves.  The integer
    sums stay exact (the uint8 reconstruction clamps NaN to 0)."""
    import torch
    rng = np.random.default_rng(99)
    Q = rng.uniform(1.0, 40.0, (8, 8)).astype(np.float32)
    Q[0, 2] = np.float32(tiny)
    Q[3, 1] = np.float32(tiny)
    img = rng.integers(0, 256, (64, 4096), dtype=np.uint8)
    img[:, 512:] = 128  # tiles with C == 0: 0 / tiny = 0 stays finite there
    q, r, r8, sums = expected(oracle, img, Q=Q)
    assert np.isinf(q).any() and np.isnan(r).any()
    hp.set_quant_table(Q)
    try:
        x = to_dev(img, dev)
        coef, rec8, got = hp.roundtrip(x, recon_dtype=torch.uint8, sums=True)
        _, recf, _ = hp.roundtrip(x, recon_dtype=torch.float32)
        two = hp.inverse(hp.forward(x))
        torch.cuda.synchronize()
    finally:
        hp.set_quant_table(None)
    assert bits_equal(to_host(coef), q)
    assert np.array_equal(to_host(rec8), r8)
    assert nan_aware_bits_equal(to_host(recf), r)
    assert nan_aware_bits_equal(to_host(two), r)
    assert got["sum_x2"] == sums["sum_x2"] and got["sse_u8"] == sums["sse_u8"]
    # NaN reconstructions: the fp32 error sum has no finite value, and the
    # device says so (sticky HPDCT_SSE_F32_INVALID -> inf), it never reads as
    # a small number (the field used to wrap modulo 2^64)
    assert not np.isfinite(sums["sse_f32"]) and got["sse_f32"] == float("inf")


def test_roundtrip_extremes(hp, oracle, dev):
    """All-0 / all-255 / sign-pattern tiles: the largest |q| and the most
    clamping in the uint8 reconstruction."""
    import torch
    t = oracle.default_transform()
    tiles = []
    for v in range(8):
        for u in range(8):
            s = np.sign(np.outer(t[v], t[u]))
            tiles.append(np.where(s > 0, 255, 0))
            tiles.append(np.where(s > 0, 0, 255))
    tiles += [np.zeros((8, 8)), np.full((8, 8), 255), np.full((8, 8), 128)]
    img = np.ascontiguousarray(np.concatenate(tiles, axis=1).astype(np.uint8))
    q, r, r8, sums = expected(oracle, img)
    coef, rec8, got = hp.roundtrip(to_dev(img, dev), recon_dtype=torch.uint8, sums=True)
    assert bits_equal(to_host(coef), q)
    assert np.array_equal(to_host(rec8), r8)
    check_sums(got, sums)


def test_roundtrip_rejects_bad_arguments(hp, dev):
    import torch
    x = torch.zeros((16, 16), dtype=torch.uint8, device=dev)
    with pytest.raises(hp.HpdctError):
        hp.roundtrip(x[:, :12].contiguous())  # width not a multiple of 8
    buf = torch.zeros(16 * 16 + 4, dtype=torch.float32, device=dev)
    with pytest.raises(hp.HpdctError):
        hp.roundtrip(x, coef=buf[1:257].view(16, 16))  # misaligned coefficient plane


@pytest.fixture(scope="module")
def c3_frame(oracle, dev):
    img = oracle.rand_u8(8192 * 8192).reshape(8192, 8192)
    return img, to_dev(img, dev)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_c3_8192_roundtrip_one_pass(hp, oracle, dev, golden, c3_frame):
    """C3 at full size with the fp32 reconstruction: coefficients and
    reconstruction match the golden digests of the oracle; PEEN/MSE from the
    device sums match the golden values of both reconstructions."""
    import torch
    g = golden["configs"]["c3_8192"]
    img, x = c3_frame
    coef, recf, got = hp.roundtrip(x, recon_dtype=torch.float32, sums=True)
    assert _sha(to_host(coef)) == g["q_f32_sha256"]
    assert _sha(to_host(recf)) == g["roundtrip_f32_sha256"]
    px = 8192 * 8192
    q = hp.quality_from_sums(got, px)
    assert abs(q["mse_f32"] - g["mse_f32"]) < 1e-5 * g["mse_f32"]
    assert abs(q["peen_f32_pct"] - g["peen_f32"]) < 1e-5 * g["peen_f32"]
    assert abs(q["mse_u8"] - g["mse_u8"]) < 1e-9 * g["mse_u8"]
    assert abs(q["peen_u8_pct"] - g["peen_u8"]) < 1e-9 * g["peen_u8"]
    assert got["sum_x2"] == g["sum_x2"] and got["sse_u8"] == g["sse_u8"]
    assert got["sse_f32"] * 65536 == g["sse_f32_fx"]


@pytest.mark.parametrize("accumulate", [False, True])
def test_c3_8192_benched_one_pass_u8_recon(hp, dev, golden, c3_frame, accumulate):
    """the configuration bench.py times as
    extras.c3_roundtrip.one_pass (and one_pass_sums_ring), at the config's
    size: uint8 reconstruction + sums through bind_roundtrip on a side stream,
    i.e. the two-lanes-per-tile kernel (roundtrip_duo_kernel<sums, JPEG forms,
    u8>) and the spread-slot fold.  Coefficients, the uint8 reconstruction and
    all three sums equal the oracle's (golden digests and exact integers,
    tests/golden/make_golden.py), twice in a row with one sums buffer: the
    overwrite gives the frame's sums both times (the fold leaves the slot
    zero), accumulate twice the frame's."""
    import torch
    g = golden["configs"]["c3_8192"]
    _, x = c3_frame
    coef = torch.full((8192, 8192), float("nan"), dtype=torch.float32, device=dev)
    rec = torch.full((8192, 8192), 7, dtype=torch.uint8, device=dev)
    buf = torch.zeros(3, dtype=torch.int64, device=dev) if accumulate else torch.full((3,), -5, dtype=torch.int64,
                                                                                       device=dev)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    call = hp.bind_roundtrip(x, coef, rec, buf, stream=side, accumulate=accumulate)
    for k in (1, 2):
        call()
        side.synchronize()
        got = hp.sums_from_buffer(buf)
        m = k if accumulate else 1
        assert got["sum_x2"] == m * g["sum_x2"] and got["sse_u8"] == m * g["sse_u8"], k
        assert got["sse_f32"] * 65536 == m * g["sse_f32_fx"], k
    assert _sha(to_host(coef)) == g["q_f32_sha256"]
    assert _sha(to_host(rec)) == g["roundtrip_u8_sha256"]
    hp.release_sums(buf)


def test_roundtrip_accumulate_two_streams_one_sums(hp, oracle, dev):
    """accumulate launches that share one sums buffer on
    two streams at once (one spread slot, two round trips and two folds in
    flight) lose nothing: the fold takes the slot with atomic exchanges and
    adds with atomic adds.  Many launches, interleaved over two streams with
    no ordering between them, add up to exactly n x the frame's sums."""
    import torch
    a = oracle.rand_u8(512 * 2048, 77).reshape(512, 2048)
    want = expected(oracle, a)[3]
    x = to_dev(a, dev)
    buf = torch.zeros(3, dtype=torch.int64, device=dev)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    for s in (s1, s2):
        s.wait_stream(torch.cuda.current_stream())
    coefs = [torch.empty(a.shape, dtype=torch.float32, device=dev) for _ in range(2)]
    calls = [hp.bind_roundtrip(x, coefs[i], None, buf, stream=s, accumulate=True) for i, s in enumerate((s1, s2))]
    n = 40
    for i in range(n):
        calls[i % 2]()
    torch.cuda.synchronize()
    got = hp.sums_from_buffer(buf)
    assert got["sum_x2"] == n * want["sum_x2"] and got["sse_u8"] == n * want["sse_u8"]
    fx = oracle.rt_sse_f32_fx(a, oracle.idct(oracle.fdct(a)))
    assert got["sse_f32"] * 65536 == n * fx
    hp.release_sums(buf)


def test_roundtrip_release_sums_reuses_slots(hp, oracle, dev):
    """hpdct_roundtrip_release_sums: a released buffer's slot
    goes back to the library and is handed to the next new sums pointer; every
    buffer still gets its frame's sums, before and after."""
    import torch
    a = oracle.rand_u8(64 * 256, 91).reshape(64, 256)
    want = expected(oracle, a)[3]
    x = to_dev(a, dev)
    coef = torch.empty(a.shape, dtype=torch.float32, device=dev)
    for rnd in range(3):
        bufs = [torch.full((3,), -1, dtype=torch.int64, device=dev) for _ in range(300)]
        for b in bufs:
            hp.bind_roundtrip(x, coef, None, b)()
        torch.cuda.synchronize()
        for b in bufs:
            check_sums(hp.sums_from_buffer(b), want)
        for b in bufs:
            hp.release_sums(b)
        del bufs
    hp.release_sums(torch.zeros(3, dtype=torch.int64, device=dev))  # never used: a no-op


@pytest.mark.parametrize("mapping", ["auto", "tile"])
@pytest.mark.parametrize("h,w", [(8, 256), (64, 512), (1000, 1008), (256, 2048), (2048, 4096)])
def test_sse_f32_is_the_four_chain_definition(hp, oracle, dev, mapping, h, w):
    """sse_f32_fx bit for bit against the oracle's restatement of its
    definition (oracle_rt_sse_f32_fx: four fp32 chains per tile, one per
    (row parity, column parity) class, each rounded to 2^-16): the
    two-lanes-per-tile kernel (AUTO, widths a multiple of 256) and the tile
    kernel (forced, or ragged widths, or the fp32 reconstruction) give the
    same value; accumulate mode adds it."""
    import torch
    img = np.random.default_rng(h * 7 + w).integers(0, 256, (h, w), dtype=np.uint8)
    q = oracle.fdct(img)
    r = oracle.idct(q)
    want = oracle.rt_sse_f32_fx(img, r)
    assert want < (1 << 53)
    x = to_dev(img, dev)
    hp.set_mapping(mapping)
    try:
        _, _, s8 = hp.roundtrip(x, recon_dtype=torch.uint8, sums=True)
        _, _, s0 = hp.roundtrip(x, sums=True)
        _, _, sf = hp.roundtrip(x, recon_dtype=torch.float32, sums=True)
        buf = torch.zeros(3, dtype=torch.int64, device=dev)
        coef = torch.empty((h, w), dtype=torch.float32, device=dev)
        call = hp.bind_roundtrip(x, coef, None, buf, accumulate=True)
        call()
        call()
        acc = hp.sums_from_buffer(buf)
    finally:
        hp.set_mapping("auto")
    for got in (s8, s0, sf):
        assert got["sse_f32"] * 65536 == want
    assert acc["sse_f32"] * 65536 == 2 * want
    assert acc["sse_u8"] == 2 * s8["sse_u8"] and acc["sum_x2"] == 2 * s8["sum_x2"]


@pytest.mark.parametrize("recon", ["u8", "f32"])
def test_roundtrip_beyond_the_duo_width_bound(hp, oracle, dev, recon):
    """the duo round trip addresses a wave's rows with 32-bit
    byte offsets, valid below 2^22 pixels of width; a wider frame (here
    2^22 + 256 px, a multiple of 256 that would otherwise take the duo
    kernel) must take the tile kernel and stay bit-exact, sums included, with
    either reconstruction."""
    import torch
    w = (1 << 22) + 256
    img = np.random.default_rng(123).integers(0, 256, (8, w), dtype=np.uint8)
    q, r, r8, sums = expected(oracle, img)
    rdt = torch.uint8 if recon == "u8" else torch.float32
    coef, rec, got = hp.roundtrip(to_dev(img, dev), recon_dtype=rdt, sums=True)
    assert bits_equal(to_host(coef), q)
    if recon == "u8":
        assert np.array_equal(to_host(rec), r8)
    else:
        assert bits_equal(to_host(rec), r)
    assert got["sum_x2"] == sums["sum_x2"] and got["sse_u8"] == sums["sse_u8"]
    assert got["sse_f32"] * 65536 == oracle.rt_sse_f32_fx(img, r)
