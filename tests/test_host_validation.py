"""Host-side argument checks of the Python boundary (hpdct.py), no GPU.

The C-ABI sees raw pointers only, so buffer sizes, dtypes, devices and the
transform's shape are checked in Python before any call reaches the library
(a short `out` or a host transform would be an out-of-bounds
device access or a GPU page fault).  Device tensors are stood in for by a
duck-typed object carrying the attributes the checks read; every case here
must raise HpdctError before the library is called.
"""
import pytest


class FakeDev:
    """Minimal stand-in for a CUDA tensor (shape, dtype, device, contiguity)."""

    def __init__(self, shape, dtype, device="cuda:0", contiguous=True, cuda=True):
        import torch
        self.shape = tuple(shape)
        self.dtype = dtype
        self.device = torch.device(device)
        self.is_cuda = cuda
        self._contig = contiguous

    def dim(self):
        return len(self.shape)

    def numel(self):
        n = 1
        for s in self.shape:
            n *= s
        return n

    def is_contiguous(self):
        return self._contig

    def data_ptr(self):
        raise AssertionError("the library must not be reached")


@pytest.fixture()
def t():
    import torch
    return torch


def test_forward_rejects_short_out(hp, t):
    img = FakeDev((64, 64), t.uint8)
    with pytest.raises(hp.HpdctError, match="holds"):
        hp.forward(img, FakeDev((64, 32), t.float32))


def test_forward_rejects_bad_out_dtype_and_device(hp, t):
    img = FakeDev((64, 64), t.uint8)
    with pytest.raises(hp.HpdctError):
        hp.forward(img, FakeDev((64, 64), t.float64))
    with pytest.raises(hp.HpdctError, match="is on"):
        hp.forward(img, FakeDev((64, 64), t.float32, device="cuda:1"))
    with pytest.raises(hp.HpdctError, match="CUDA"):
        hp.forward(img, FakeDev((64, 64), t.float32, cuda=False))
    with pytest.raises(hp.HpdctError, match="contiguous"):
        hp.forward(img, FakeDev((64, 64), t.float32, contiguous=False))


def test_forward_rejects_height_width_past_the_source(hp, t):
    img = FakeDev((64, 64), t.uint8)
    with pytest.raises(hp.HpdctError, match="needs"):
        hp.forward(img, FakeDev((128, 64), t.float32), height=128, width=64)
    with pytest.raises(hp.HpdctError, match="negative"):
        hp.forward(img, FakeDev((64, 64), t.float32), height=-8, width=64)


def test_transform_must_be_64_device_floats(hp, t):
    img = FakeDev((64, 64), t.float32)
    out = FakeDev((64, 64), t.float32)
    for bad in (FakeDev((8, 8), t.float32, cuda=False),    # host pointer: a GPU page fault
                FakeDev((8, 7), t.float32),                # 56 floats
                FakeDev((8, 8), t.float64),
                FakeDev((8, 8), t.float32, contiguous=False),
                FakeDev((8, 8), t.float32, device="cuda:3")):
        with pytest.raises(hp.HpdctError):
            hp.forward(img, out, transform=bad)
        with pytest.raises(hp.HpdctError):
            hp.inverse(img, out, transform=bad)
    with pytest.raises(hp.HpdctError):
        hp.dct_all_blocks_cuda(img, 64, 64, None, out)


def test_inverse_and_bind_reject_short_out(hp, t):
    coef = FakeDev((64, 64), t.float32)
    with pytest.raises(hp.HpdctError):
        hp.inverse(coef, FakeDev((63, 64), t.float32))
    with pytest.raises(hp.HpdctError):
        hp.inverse(coef, FakeDev((64, 64), t.int8))  # int8 is not a pixel output
    with pytest.raises(hp.HpdctError):
        hp.bind("fwd", FakeDev((64, 64), t.uint8), FakeDev((8, 64), t.float32))
    with pytest.raises(hp.HpdctError):
        hp.bind("inv", coef, FakeDev((64, 64), t.float32, device="cuda:2"))
    with pytest.raises(ValueError):
        hp.bind("sideways", coef, coef)


def test_compat_wrappers_check_buffers(hp, t):
    T = FakeDev((8, 8), t.float32)
    img = FakeDev((64, 64), t.float32)
    with pytest.raises(hp.HpdctError):
        hp.dct_all_blocks_cuda(img, 64, 128, T, FakeDev((64, 128), t.float32))  # image too small
    with pytest.raises(hp.HpdctError):
        hp.idct_all_blocks_cuda(img, 64, 64, T, FakeDev((32, 64), t.float32))   # result too small
    with pytest.raises(hp.HpdctError):
        hp.dct_all_blocks(img, 64, 64, FakeDev((8, 8), t.float32, cuda=False), img)


def test_roundtrip_checks_every_plane(hp, t):
    img = FakeDev((64, 64), t.uint8)
    coef = FakeDev((64, 64), t.float32)
    with pytest.raises(hp.HpdctError):
        hp.bind_roundtrip(img, FakeDev((64, 60), t.float32))
    with pytest.raises(hp.HpdctError):
        hp.bind_roundtrip(img, coef, FakeDev((64, 64), t.int8))
    with pytest.raises(hp.HpdctError):
        hp.bind_roundtrip(img, coef, None, FakeDev((2,), t.int64))
    with pytest.raises(hp.HpdctError):
        hp.bind_roundtrip(img, coef, None, FakeDev((3,), t.float32))
    with pytest.raises(hp.HpdctError):
        hp.bind_roundtrip(FakeDev((64, 64), t.float32), coef)


def test_stream_forward_checks_every_host_entry(hp, t):
    f = t.zeros((64, 64), dtype=t.uint8)
    out = t.empty((64, 64), dtype=t.float32)
    with pytest.raises(hp.HpdctError):
        hp.stream_forward([f, t.zeros((32, 64), dtype=t.uint8)], [out, out.clone()])
    with pytest.raises(hp.HpdctError):
        hp.stream_forward([f, f], [out, t.empty((64, 64), dtype=t.int8)])
    with pytest.raises(hp.HpdctError):
        hp.stream_forward([f], [t.empty((64, 32), dtype=t.float32)])
    with pytest.raises(hp.HpdctError):
        hp.stream_forward([f.float()], [out])
    with pytest.raises(hp.HpdctError):
        hp.stream_forward([f[:, ::2]], [t.empty((64, 32), dtype=t.float32)])
    with pytest.raises(hp.HpdctError):
        hp.stream_forward([f], [t.empty((64, 64), dtype=t.float64)])
    with pytest.raises(hp.HpdctError):
        hp.stream_forward([f], [])


def test_fill_hash_checks_its_plane(hp, t):
    with pytest.raises(hp.HpdctError):
        hp.fill_hash_u8(FakeDev((64,), t.float32), seed=1)
    with pytest.raises(hp.HpdctError):
        hp.fill_hash_u8(t.zeros(64, dtype=t.uint8), seed=1)  # host tensor


def test_forward_frames_checks_every_plane(hp, t):
    f = FakeDev((64, 64), t.uint8)
    o = FakeDev((64, 64), t.float32)
    with pytest.raises(hp.HpdctError, match="shape"):
        hp.forward_frames([f, FakeDev((32, 128), t.uint8)], [o, o])
    with pytest.raises(hp.HpdctError):
        hp.forward_frames([f, FakeDev((64, 64), t.float32)], [o, o])
    with pytest.raises(hp.HpdctError, match="coefficient planes"):
        hp.forward_frames([f, f], [o])
    with pytest.raises(hp.HpdctError, match="holds"):
        hp.forward_frames([f], [FakeDev((64, 32), t.float32)])
    with pytest.raises(hp.HpdctError, match="dtype"):
        hp.forward_frames([f, f], [o, FakeDev((64, 64), t.int8)])
    with pytest.raises(hp.HpdctError):
        hp.forward_frames([f, FakeDev((64, 64), t.uint8, device="cuda:1")], [o, o])
    with pytest.raises(hp.HpdctError):
        hp.forward_frames([FakeDev((64, 64), t.uint8, contiguous=False)], [o])
    assert hp.forward_frames([], []) == []


def test_stream_context_arguments_rejected(hp):
    """hpdct_stream_create validates before touching a device; run/destroy
    on a NULL context are a status / a no-op."""
    import ctypes
    L = hp.load_library()
    h = ctypes.c_void_p()
    assert L.hpdct_stream_create(ctypes.byref(h), 64, 64, hp.F32, 0) == 1    # nstreams 0
    assert L.hpdct_stream_create(ctypes.byref(h), 64, 64, hp.F32, 17) == 1   # > 16
    assert L.hpdct_stream_create(ctypes.byref(h), 64, 64, hp.U8, 2) == 2     # coefficients f32 / i8
    assert L.hpdct_stream_create(ctypes.byref(h), 64, 60, hp.F32, 2) == 1    # width not a multiple of 8
    assert L.hpdct_stream_create(None, 64, 64, hp.F32, 2) == 1
    assert not h.value
    P = ctypes.c_void_p * 1
    assert L.hpdct_stream_run(None, P(1), P(1), 1, None) == 1
    assert L.hpdct_stream_destroy(None) == 0
    # the one-shot form: an empty batch is a no-op without device work
    ms = ctypes.c_float(-1.0)
    assert L.hpdct_stream_forward(P(1), P(1), 0, 64, 64, hp.F32, 2, ctypes.byref(ms)) == 0 and ms.value == 0.0
