"""ctypes view of the CPU oracle (hpdct_oracle.c) and of the reference's own
host utilities compiled here (_ref/libref_utils.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / the timed CPU baseline,
never by the product path.  Parity status: partially pinned (see
hpdct_oracle.c header and DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "libhpdct_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_utils.so")

QUANT = 1
NOFMA = 2
RECIP = 4
NOSHIFT = 8
ROWFIRST = 16

_lib = None
_ref = None


def build() -> None:
    """Compile the oracle (and _ref when /root/reference is present)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        for name in ("oracle_fdct", "oracle_fdct_u8", "oracle_idct"):
            f = getattr(L, name)
            f.argtypes = [vp, i64, i64, vp, vp, vp, ctypes.c_int]
            f.restype = None
        L.oracle_fill_rand_u8.argtypes = [vp, i64, ctypes.c_uint32]
        L.oracle_fill_hash_u8.argtypes = [vp, i64, ctypes.c_uint64, i64]
        L.oracle_quality.argtypes = [vp, vp, i64, vp, vp]
        L.oracle_rt_sse_f32_fx.argtypes = [vp, vp, i64, i64]
        L.oracle_rt_sse_f32_fx.restype = ctypes.c_uint64
        L.oracle_u8_to_f32.argtypes = [vp, vp, i64]
        L.oracle_f32_to_u8.argtypes = [vp, vp, i64]
        L.oracle_default_quant.argtypes = [vp]
        L.oracle_default_transform.argtypes = [vp]
        L.oracle_srand.argtypes = [vp, ctypes.c_uint32]
        L.oracle_rand.argtypes = [vp]
        L.oracle_rand.restype = ctypes.c_int32
        _lib = L
    return _lib


def ref_utils():
    """The reference's utils.cu compiled here, or None if not built."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        R = ctypes.CDLL(REF_SO)
        R._Z14convertToFloatPKhPfm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        R._Z14convertToFloatPKhPfm.restype = None
        R._Z21convertToUnsignedCharPKfPhm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        R._Z21convertToUnsignedCharPKfPhm.restype = None
        R._Z16arrays_are_closePKfS0_mf.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                   ctypes.c_float]
        R._Z16arrays_are_closePKfS0_mf.restype = ctypes.c_bool
        _ref = R
    return _ref


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def default_quant() -> np.ndarray:
    q = np.empty(64, np.float32)
    lib().oracle_default_quant(_p(q))
    return q.reshape(8, 8)


def default_transform() -> np.ndarray:
    t = np.empty(64, np.float32)
    lib().oracle_default_transform(_p(t))
    return t.reshape(8, 8)


def rand_u8(n: int, seed: int = 42) -> np.ndarray:
    a = np.empty(int(n), np.uint8)
    lib().oracle_fill_rand_u8(_p(a), int(n), seed)
    return a


def hash_u8(n: int, seed: int, first_index: int = 0) -> np.ndarray:
    a = np.empty(int(n), np.uint8)
    lib().oracle_fill_hash_u8(_p(a), int(n), ctypes.c_uint64(seed), int(first_index))
    return a


def _tables(T, Q):
    t = None if T is None else np.ascontiguousarray(np.asarray(T, np.float32).reshape(64))
    q = None if Q is None else np.ascontiguousarray(np.asarray(Q, np.float32).reshape(64))
    return t, q


def fdct(img: np.ndarray, T=None, Q=None, quant=True, nofma=False, recip=False, shift=True,
         row_first=False) -> np.ndarray:
    """Forward transform of a (H, W) uint8 or float32 image (not mutated)."""
    img = np.ascontiguousarray(img)
    h, w = img.shape[-2] if img.ndim > 1 else 1, img.shape[-1]
    h = img.size // w
    out = np.empty(img.shape, np.float32)
    t, q = _tables(T, Q)
    mode = (QUANT if quant else 0) | (NOFMA if nofma else 0) | (RECIP if recip else 0) | (0 if shift else NOSHIFT) | \
        (ROWFIRST if row_first else 0)
    fn = lib().oracle_fdct_u8 if img.dtype == np.uint8 else lib().oracle_fdct
    if img.dtype not in (np.uint8, np.float32):
        raise TypeError(img.dtype)
    fn(_p(img), h, w, None if t is None else _p(t), None if q is None else _p(q), _p(out), mode)
    return out


def fdct_threads(img: np.ndarray, threads: int) -> np.ndarray:
    """fdct (default tables, quantised) of a (H, W) uint8 image split into
    `threads` bands of whole tile rows, one ctypes call per band on a thread
    pool (ctypes drops the GIL): the all-cores CPU baseline.
    Tiles are independent, so the result equals fdct(img) bit for bit."""
    from concurrent.futures import ThreadPoolExecutor
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.empty(img.shape, np.float32)
    trows = h // 8
    cuts = [8 * (trows * k // threads) for k in range(threads + 1)]

    def band(k):
        r0, r1 = cuts[k], cuts[k + 1]
        if r1 > r0:
            lib().oracle_fdct_u8(_p(img[r0:r1]), r1 - r0, w, None, None, _p(out[r0:r1]), QUANT)

    with ThreadPoolExecutor(max_workers=threads) as pool:
        list(pool.map(band, range(threads)))
    return out


def idct(coef: np.ndarray, T=None, Q=None, dequant=True, nofma=False, shift=True, row_first=False) -> np.ndarray:
    coef = np.ascontiguousarray(coef, dtype=np.float32)
    w = coef.shape[-1]
    h = coef.size // w
    out = np.empty(coef.shape, np.float32)
    t, q = _tables(T, Q)
    mode = (QUANT if dequant else 0) | (NOFMA if nofma else 0) | (0 if shift else NOSHIFT) | (ROWFIRST if row_first else 0)
    lib().oracle_idct(_p(coef), h, w, None if t is None else _p(t), None if q is None else _p(q), _p(out), mode)
    return out


def to_u8(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32)
    o = np.empty(a.shape, np.uint8)
    lib().oracle_f32_to_u8(_p(a), _p(o), a.size)
    return o


def rt_sse_f32_fx(img: np.ndarray, r: np.ndarray) -> int:
    """The round trip's sse_f32_fx (hpdct_oracle.c oracle_rt_sse_f32_fx): img
    uint8 (h x w), r the fp32 reconstruction R + 128 of the same shape."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    r = np.ascontiguousarray(r, dtype=np.float32)
    return int(lib().oracle_rt_sse_f32_fx(_p(img), _p(r), img.shape[0], img.shape[1]))


def quality(x: np.ndarray, y: np.ndarray):
    """(PEEN %, MSE)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.ascontiguousarray(y, dtype=np.float32)
    peen = ctypes.c_double()
    mse = ctypes.c_double()
    lib().oracle_quality(_p(x), _p(y), x.size, ctypes.byref(peen), ctypes.byref(mse))
    return peen.value, mse.value
