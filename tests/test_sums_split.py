"""The duo round trip's sse_f32 split (rt_sse_split in
cuda-dct-idct_amd/csrc/hpdct_rt_duo.hpp): a chain's fixed-point value
fx = rint(chain * 2^16), an integer-valued fp32 below 2^40, is carried as two
32-bit halves hi = floor(fx * 2^-22), lo = fma(-hi, 2^22, fx), and the wave
sums are rebuilt as (sum hi) << 22 + sum lo.  This checks the arithmetic the
kernel relies on, in fp32 as the kernel computes it: hi * 2^22 + lo == fx
exactly, lo < 2^22, hi < 2^18, and the 32-bit wave sums cannot wrap at the
kernel's bound (64 lanes x 2 chains x 8 runs).  CPU only."""
import numpy as np

SCALE = np.float32(65536.0)


def split(chain):
    fx = np.rint(chain.astype(np.float32) * SCALE).astype(np.float32)
    good = fx < np.float32(2.0 ** 40)
    h = np.floor(fx * np.float32(2.0 ** -22)).astype(np.float32)
    # fma(-h, 2^22, fx): the exact difference is an integer below 2^22, so one
    # rounding of it (float64 here, then fp32) is exact
    lo = (fx.astype(np.float64) - h.astype(np.float64) * 2.0 ** 22).astype(np.float32)
    return fx, h, lo, good


def test_split_recombines_exactly():
    rng = np.random.default_rng(5)
    chains = np.concatenate([
        rng.uniform(0.0, 2.0 ** 24, 200_000),            # the whole valid range of a chain
        rng.uniform(0.0, 64.0, 100_000),                 # typical per-tile sums
        np.array([0.0, 2.0 ** -17, 2.0 ** -16, 0.5, 1.0, 2.0 ** 6 - 2.0 ** -16, 2.0 ** 6, 2.0 ** 24 - 1.0]),
    ]).astype(np.float32)
    fx, h, lo, good = split(chains)
    assert good.all()
    hi_i = h.astype(np.int64)
    lo_i = lo.astype(np.int64)
    assert (lo == np.floor(lo)).all() and (h == np.floor(h)).all()
    assert (lo_i >= 0).all() and (lo_i < 2 ** 22).all()
    assert (hi_i >= 0).all() and (hi_i < 2 ** 18).all()
    assert ((hi_i << 22) + lo_i == fx.astype(np.int64)).all()


def test_invalid_chains_flag():
    with np.errstate(invalid="ignore", over="ignore"):
        fx, h, lo, good = split(np.array([2.0 ** 24, 3e30, np.inf, np.nan], dtype=np.float32))
    assert not good.any()


def test_wave_sums_fit_32_bits():
    # per lane: 2 chains per run, at most 8 runs (static_assert kSets <= 8), 64 lanes
    terms = 64 * 2 * 8
    assert terms * (2 ** 22 - 1) < 2 ** 32          # sum of lo
    assert terms * (2 ** 18 - 1) < 2 ** 32          # sum of hi
    # sse_u8 and sum_x2 per lane and run: 32 pixels of at most 255^2
    assert 64 * 8 * 32 * 255 ** 2 < 2 ** 32
