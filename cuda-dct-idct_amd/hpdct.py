"""hpdct -- Python host-side mirror of the reference's DCT/IDCT call surface,
bound to the gfx950 library ``lib/libhpdct.so`` through its C-ABI
(``include/hpdct.h``) with ctypes.

PyTorch only supplies device memory and streams here: tensors are passed to
the library as raw device pointers and the kernels run on torch's current HIP
stream (or the one given).  There is no CPU or PyTorch fallback: if the
shared library is missing, every entry point raises ``HpdctLibraryError``.

Reference names mirrored (file:line into GerryDps/CUDA-DCT-IDCT):
  dct_all_blocks_cuda(image, h, w, T, result)   main_newAppr.cu:252-291
  idct_all_blocks_cuda(coef, h, w, T, result)   main_newAppr.cu:293-332
  set_quant_table(q)      cudaMemcpyToSymbol(const_quant_matrix, ...) :19,70
  convert_to_float / convert_to_unsigned_char   utils.cu:10-24
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HPDCT_LIB", os.path.join(_HERE, "lib", "libhpdct.so"))

# include/hpdct.h
U8, I8, F32 = 0, 1, 2
FLAG_NO_QUANT = 0x1
FLAG_WRITEBACK_SHIFT = 0x2
FLAG_NO_SHIFT = 0x4
FLAG_ROW_FIRST = 0x8
FLAG_WRITEBACK_DEQUANT = 0x10

STATUS = {
    0: "HPDCT_SUCCESS",
    1: "HPDCT_ERROR_INVALID_VALUE",
    2: "HPDCT_ERROR_UNSUPPORTED",
    3: "HPDCT_ERROR_RANGE",
    4: "HPDCT_ERROR_DEVICE",
}

# every symbol include/hpdct.h, hpdct_baseline.h (A/B and measurement only)
# and hpdct_compat.h declare
C_SYMBOLS = [
    "hpdct_version", "hpdct_build_info", "hpdct_status_string", "hpdct_last_error_string",
    "hpdct_default_quant_table", "hpdct_default_transform",
    "hpdct_set_quant_table", "hpdct_get_quant_table",
    "hpdct_forward", "hpdct_inverse",
    "hpdct_forward_u8_f32", "hpdct_forward_u8_i8", "hpdct_inverse_f32_f32",
    "hpdct_fill_hash_u8", "hpdct_fill_rand_u8", "hpdct_u8_to_f32", "hpdct_f32_to_u8",
    "hpdct_baseline_forward", "hpdct_stream_forward", "hpdct_set_mapping", "hpdct_get_mapping",
    "hpdct_roundtrip_u8", "hpdct_roundtrip_u8_accumulate", "hpdct_forward_frames",
    "hpdct_stream_create", "hpdct_stream_run", "hpdct_stream_destroy", "hpdct_decode_i8_f32",
    "hpdct_roundtrip_release_sums", "hpdct_floor_probe", "hpdct_copy_ceiling",
]
MAPPINGS = {"auto": 0, "tile": 1, "octet": 2, "duo": 3}
BASELINES = {"reference_3pass": 0, "fastappr_3pass": 1}
COMPAT_SYMBOLS = {
    "dct_all_blocks_cuda": "_Z19dct_all_blocks_cudaPfiiPKfS_",
    "idct_all_blocks_cuda": "_Z20idct_all_blocks_cudaPKfiiS0_Pf",
    # cublasDCTv2 surface (main_cublass_2.cu:36-37); last argument: cublasHandle_t (ignored)
    "dct_all_blocks": "_Z14dct_all_blocksPfiiPKfS_P13cublasContext",
    "idct_all_blocks": "_Z15idct_all_blocksPfiiPKfS_P13cublasContext",
}


class HpdctLibraryError(RuntimeError):
    """libhpdct.so is missing or failed to load (no fallback exists)."""


class HpdctError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS.get(status, status)}: {message}")
        self.status = status


_lib = None


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Load (once) and return the native library; raise loudly if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    # libhpdct.so and torch both need libamdhip64.so.7 and the first one loaded
    # wins the soname for the whole process.  Two HIP runtimes (torch's bundled
    # copy and /opt/rocm's) in one process see no device, so let torch load
    # its runtime first and bind the library to that same instance.
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - host-only use without torch
        pass
    if not os.path.exists(p):
        raise HpdctLibraryError(
            f"{p} not found: build it with `make -C cuda-dct-idct_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:  # pragma: no cover - depends on the loader
        raise HpdctLibraryError(f"cannot load {p}: {e}") from e
    vp, i64, u32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint32
    lib.hpdct_version.restype = ctypes.c_char_p
    lib.hpdct_build_info.restype = ctypes.c_char_p
    lib.hpdct_decode_i8_f32.argtypes = [vp, vp, i64, vp]
    lib.hpdct_decode_i8_f32.restype = ctypes.c_int
    lib.hpdct_floor_probe.argtypes = [ctypes.c_int, vp, vp, i64, i64, vp]
    lib.hpdct_floor_probe.restype = ctypes.c_int
    lib.hpdct_copy_ceiling.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp, ctypes.c_int, i64, ctypes.c_int, vp]
    lib.hpdct_copy_ceiling.restype = ctypes.c_int
    lib.hpdct_roundtrip_release_sums.argtypes = [vp]
    lib.hpdct_roundtrip_release_sums.restype = ctypes.c_int
    lib.hpdct_status_string.restype = ctypes.c_char_p
    lib.hpdct_status_string.argtypes = [ctypes.c_int]
    lib.hpdct_last_error_string.restype = ctypes.c_char_p
    for f in (lib.hpdct_default_quant_table, lib.hpdct_default_transform):
        f.argtypes = [vp]
        f.restype = None
    lib.hpdct_set_quant_table.argtypes = [vp]
    lib.hpdct_get_quant_table.argtypes = [vp]
    for f in (lib.hpdct_forward, lib.hpdct_inverse):
        f.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, i64, i64, vp, ctypes.c_uint, vp]
        f.restype = ctypes.c_int
    for f in (lib.hpdct_forward_u8_f32, lib.hpdct_forward_u8_i8, lib.hpdct_inverse_f32_f32):
        f.argtypes = [vp, vp, i64, i64, vp]
        f.restype = ctypes.c_int
    lib.hpdct_fill_hash_u8.argtypes = [vp, i64, ctypes.c_uint64, i64, vp]
    lib.hpdct_fill_hash_u8.restype = ctypes.c_int
    lib.hpdct_fill_rand_u8.argtypes = [vp, i64, u32]
    lib.hpdct_fill_rand_u8.restype = None
    lib.hpdct_u8_to_f32.argtypes = [vp, vp, i64]
    lib.hpdct_u8_to_f32.restype = None
    lib.hpdct_f32_to_u8.argtypes = [vp, vp, i64]
    lib.hpdct_f32_to_u8.restype = None
    lib.hpdct_set_mapping.argtypes = [ctypes.c_int]
    lib.hpdct_set_mapping.restype = ctypes.c_int
    lib.hpdct_get_mapping.argtypes = []
    lib.hpdct_get_mapping.restype = ctypes.c_int
    lib.hpdct_stream_forward.argtypes = [vp, vp, i64, i64, i64, ctypes.c_int, ctypes.c_int, vp]
    lib.hpdct_stream_forward.restype = ctypes.c_int
    lib.hpdct_stream_create.argtypes = [vp, i64, i64, ctypes.c_int, ctypes.c_int]
    lib.hpdct_stream_run.argtypes = [vp, vp, vp, i64, vp]
    lib.hpdct_stream_destroy.argtypes = [vp]
    for f in (lib.hpdct_stream_create, lib.hpdct_stream_run, lib.hpdct_stream_destroy):
        f.restype = ctypes.c_int
    lib.hpdct_forward_frames.argtypes = [vp, vp, ctypes.c_int, i64, i64, i64, vp]
    lib.hpdct_forward_frames.restype = ctypes.c_int
    lib.hpdct_baseline_forward.argtypes = [ctypes.c_int, vp, vp, vp, i64, i64, vp, vp]
    lib.hpdct_baseline_forward.restype = ctypes.c_int
    for f in (lib.hpdct_roundtrip_u8, lib.hpdct_roundtrip_u8_accumulate):
        f.argtypes = [vp, vp, vp, ctypes.c_int, vp, i64, i64, vp]
        f.restype = ctypes.c_int
    for name, mangled in COMPAT_SYMBOLS.items():
        f = getattr(lib, mangled)
        f.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp] + ([vp] if not name.endswith("_cuda") else [])
        f.restype = None
    if path is None:
        _lib = lib
    return lib


def _check(status: int) -> None:
    if status != 0:
        msg = load_library().hpdct_last_error_string().decode(errors="replace")
        raise HpdctError(status, msg)


def version() -> str:
    return load_library().hpdct_version().decode()


def build_info() -> str:
    """'src=<sha256 of csrc/ + include/> git=<rev> arch=gfx950' stamped at build
    time (src_digest.py)."""
    return load_library().hpdct_build_info().decode()


def provenance() -> dict:
    """The loaded library's build stamp and whether it matches the sources of
    this tree (bench.py / smoke() report it)."""
    import src_digest
    return src_digest.provenance(build_info())


def set_mapping(name: str) -> None:
    """Kernel work mapping, process-wide: "auto" (per frame size), "tile"
    (one lane per 8x8 tile), "octet" (eight lanes per tile) or "duo" (two
    lanes per tile, fp32 -> fp32 kernels).  Results are bit-identical; for
    A/B timing and tests (include/hpdct.h)."""
    if name not in MAPPINGS:
        raise ValueError(f"mapping must be one of {sorted(MAPPINGS)}")
    _check(load_library().hpdct_set_mapping(MAPPINGS[name]))


def get_mapping() -> str:
    m = load_library().hpdct_get_mapping()
    return {v: k for k, v in MAPPINGS.items()}[m]


# ---------------------------------------------------------------------------
# tables
# ---------------------------------------------------------------------------
def default_quant_table() -> np.ndarray:
    q = np.empty(64, np.float32)
    load_library().hpdct_default_quant_table(q.ctypes.data)
    return q.reshape(8, 8)


def default_transform() -> np.ndarray:
    t = np.empty(64, np.float32)
    load_library().hpdct_default_transform(t.ctypes.data)
    return t.reshape(8, 8)


def set_quant_table(q) -> None:
    """Library-owned Q (replaces cudaMemcpyToSymbol(const_quant_matrix, ...)).
    ``None`` restores the default JPEG luminance table."""
    lib = load_library()
    if q is None:
        _check(lib.hpdct_set_quant_table(None))
        return
    a = np.ascontiguousarray(np.asarray(q, dtype=np.float32).reshape(64))
    _check(lib.hpdct_set_quant_table(a.ctypes.data))


def get_quant_table() -> np.ndarray:
    q = np.empty(64, np.float32)
    _check(load_library().hpdct_get_quant_table(q.ctypes.data))
    return q.reshape(8, 8)


# ---------------------------------------------------------------------------
# device entry points (torch tensors in HBM)
# ---------------------------------------------------------------------------
def _torch():
    import torch
    return torch


def _dtype_code(t) -> int:
    torch = _torch()
    m = {torch.uint8: U8, torch.int8: I8, torch.float32: F32}
    if t.dtype not in m:
        raise HpdctError(2, f"unsupported tensor dtype {t.dtype}")
    return m[t.dtype]


def _stream_ptr(stream):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _hw(t, height, width):
    if height is None or width is None:
        if t.dim() < 2:
            raise HpdctError(1, "pass height/width for a flat tensor")
        height = t.numel() // t.shape[-1] if t.shape[-1] else 0
        width = t.shape[-1]
    h, w = int(height), int(width)
    if h < 0 or w < 0:
        raise HpdctError(1, f"negative frame shape {h}x{w}")
    if h * w > t.numel():
        raise HpdctError(1, f"a {h}x{w} frame needs {h * w} elements, the source holds {t.numel()}")
    return h, w


def _device_plane(t, what: str, device, need: int, dtypes=None):
    """The C-ABI cannot see buffer sizes: every device plane is checked here
    (CUDA, contiguous, on `device`, >= `need` elements, dtype allowed)."""
    if not hasattr(t, "is_cuda") or not t.is_cuda:
        raise HpdctError(1, f"{what} must be a CUDA tensor")
    if not t.is_contiguous():
        raise HpdctError(1, f"{what} must be contiguous")
    if device is not None and t.device != device:
        raise HpdctError(1, f"{what} is on {t.device}, the source on {device}")
    if t.numel() < need:
        raise HpdctError(1, f"{what} holds {t.numel()} elements, {need} needed")
    if dtypes is not None and t.dtype not in dtypes:
        raise HpdctError(2, f"{what} dtype {t.dtype} not in {list(dtypes)}")


def _transform_ptr(transform, device):
    """None (built-in T) or a contiguous 64-element float32 CUDA tensor."""
    if transform is None:
        return None
    torch = _torch()
    _device_plane(transform, "transform", device, 64, (torch.float32,))
    if transform.numel() != 64:
        raise HpdctError(1, f"transform must hold 64 floats, not {transform.numel()}")
    return ctypes.c_void_p(transform.data_ptr())


def _planes(src, dst, direction: str, height, width):
    """Shape and buffer checks of one forward/inverse launch; returns (h, w)."""
    torch = _torch()
    what = "image" if direction == "fwd" else "coefficients"
    ins = (torch.uint8, torch.float32) if direction == "fwd" else (torch.int8, torch.float32)
    outs = (torch.float32, torch.int8) if direction == "fwd" else (torch.float32, torch.uint8)
    _device_plane(src, what, None, 0, ins)
    h, w = _hw(src, height, width)
    _device_plane(dst, "out", src.device, h * w, outs)
    return h, w


def forward(image, out=None, *, out_dtype=None, transform=None, quantise=True, writeback_shift=False,
            level_shift=True, row_first=False, height=None, width=None, stream=None):
    """Fused forward pass on the GPU: round((T.(X-128).T^T)/Q) per 8x8 tile.

    image: CUDA tensor, uint8 or float32, (..., H, W) contiguous (a stack of
    frames is treated as one (F*H) x W image).  Returns the coefficient
    tensor (float32 by default, int8 on request) in the reference layout."""
    torch = _torch()
    _device_plane(image, "image", None, 0)
    if out is None:
        out = torch.empty(image.shape, dtype=out_dtype or torch.float32, device=image.device)
    h, w = _planes(image, out, "fwd", height, width)
    flags = (0 if quantise else FLAG_NO_QUANT) | (FLAG_WRITEBACK_SHIFT if writeback_shift else 0) | \
        (0 if level_shift else FLAG_NO_SHIFT) | (FLAG_ROW_FIRST if row_first else 0)
    tptr = _transform_ptr(transform, image.device)
    _check(load_library().hpdct_forward(ctypes.c_void_p(image.data_ptr()), _dtype_code(image),
                                        ctypes.c_void_p(out.data_ptr()), _dtype_code(out), h, w, tptr,
                                        flags, _stream_ptr(stream)))
    return out


def inverse(coef, out=None, *, out_dtype=None, transform=None, dequantise=True, level_shift=True,
            row_first=False, writeback_dequant=False, height=None, width=None, stream=None):
    """Fused inverse pass: T^T.(q*Q).T + 128 per tile.  out float32 (no clamp,
    as the reference) or uint8 (clamp + truncate, convertToUnsignedChar)."""
    torch = _torch()
    _device_plane(coef, "coefficients", None, 0)
    if out is None:
        out = torch.empty(coef.shape, dtype=out_dtype or torch.float32, device=coef.device)
    h, w = _planes(coef, out, "inv", height, width)
    flags = (0 if dequantise else FLAG_NO_QUANT) | (0 if level_shift else FLAG_NO_SHIFT) | \
        (FLAG_ROW_FIRST if row_first else 0) | (FLAG_WRITEBACK_DEQUANT if writeback_dequant else 0)
    tptr = _transform_ptr(transform, coef.device)
    _check(load_library().hpdct_inverse(ctypes.c_void_p(coef.data_ptr()), _dtype_code(coef),
                                        ctypes.c_void_p(out.data_ptr()), _dtype_code(out), h, w, tptr,
                                        flags, _stream_ptr(stream)))
    return out


def bind(direction: str, src, dst, *, transform=None, quantise=True, level_shift=True, writeback_shift=False,
         row_first=False, writeback_dequant=False, stream=None, height=None, width=None):
    """Pre-resolve every argument of one forward ("fwd") or inverse ("inv")
    launch and return a zero-argument callable: the per-call host cost is one
    ctypes call (used by bench.py's timed loop)."""
    if direction not in ("fwd", "inv"):
        raise ValueError('direction must be "fwd" or "inv"')
    h, w = _planes(src, dst, direction, height, width)
    lib = load_library()
    fn = {"fwd": lib.hpdct_forward, "inv": lib.hpdct_inverse}[direction]
    flags = (0 if quantise else FLAG_NO_QUANT) | (0 if level_shift else FLAG_NO_SHIFT) | \
        (FLAG_WRITEBACK_SHIFT if writeback_shift else 0) | (FLAG_ROW_FIRST if row_first else 0) | \
        (FLAG_WRITEBACK_DEQUANT if writeback_dequant else 0)
    args = (ctypes.c_void_p(src.data_ptr()), _dtype_code(src), ctypes.c_void_p(dst.data_ptr()), _dtype_code(dst),
            h, w, _transform_ptr(transform, src.device), flags, _stream_ptr(stream))

    def call():
        st = fn(*args)
        if st:
            _check(st)
    return call


SSE_F32_UNIT = 1.0 / 65536.0  # HPDCT_SSE_F32_UNIT
SSE_F32_INVALID = 1 << 63     # HPDCT_SSE_F32_INVALID


def _roundtrip_args(image, coef, recon, sums_buf, height, width, stream):
    torch = _torch()
    _device_plane(image, "image", None, 0, (torch.uint8,))
    h, w = _hw(image, height, width)
    _device_plane(coef, "coefficients", image.device, h * w, (torch.float32,))
    if recon is not None:
        _device_plane(recon, "reconstruction", image.device, h * w, (torch.uint8, torch.float32))
    if sums_buf is not None:
        _device_plane(sums_buf, "sums buffer", image.device, 3, (torch.int64,))
    return (ctypes.c_void_p(image.data_ptr()), ctypes.c_void_p(coef.data_ptr()),
            None if recon is None else ctypes.c_void_p(recon.data_ptr()),
            F32 if recon is None else _dtype_code(recon),
            None if sums_buf is None else ctypes.c_void_p(sums_buf.data_ptr()), h, w, _stream_ptr(stream))


def sums_from_buffer(sums_buf) -> dict:
    """The 3 x uint64 device struct hpdct_roundtrip_sums (held in an int64
    tensor) as {"sse_f32", "sse_u8", "sum_x2"} (synchronises)."""
    v = [int(x) & ((1 << 64) - 1) for x in sums_buf.cpu().tolist()]
    # bit 63: some tile's fp32 error sum was non-finite or too large to add
    # (HPDCT_SSE_F32_INVALID): no finite sse_f32 exists for the frame
    sse_f32 = float("inf") if v[0] & SSE_F32_INVALID else v[0] * SSE_F32_UNIT
    return {"sse_f32": sse_f32, "sse_u8": v[1], "sum_x2": v[2]}


def quality_from_sums(sums: dict, pixels: int) -> dict:
    """PEEN (%) and MSE of both reconstructions from the round-trip sums
    (PEEN = 100 sqrt(sse / sum x^2), MSE = sse / pixels; hpdct_quality.py)."""
    sx = float(sums["sum_x2"])
    return {"mse_f32": sums["sse_f32"] / pixels, "peen_f32_pct": 100.0 * (sums["sse_f32"] / sx) ** 0.5,
            "mse_u8": sums["sse_u8"] / pixels, "peen_u8_pct": 100.0 * (sums["sse_u8"] / sx) ** 0.5}


def roundtrip(image, coef=None, recon=None, *, recon_dtype=None, sums=False, height=None, width=None,
              stream=None):
    """One-pass C3 round trip on the GPU (hpdct_roundtrip_u8): uint8 frame ->
    fp32 quantised coefficients, the reconstruction (uint8 clamp + truncate or
    fp32, when recon or recon_dtype is given) and, with sums=True, the quality
    sums.  Bit-identical to forward() followed by inverse().
    Returns (coef, recon or None, sums dict or None); reading the sums
    synchronises the stream."""
    torch = _torch()
    if coef is None:
        coef = torch.empty(image.shape, dtype=torch.float32, device=image.device)
    if recon is None and recon_dtype is not None:
        recon = torch.empty(image.shape, dtype=recon_dtype, device=image.device)
    sums_buf = torch.empty(3, dtype=torch.int64, device=image.device) if sums else None
    _check(load_library().hpdct_roundtrip_u8(*_roundtrip_args(image, coef, recon, sums_buf, height, width, stream)))
    return coef, recon, (sums_from_buffer(sums_buf) if sums else None)


def bind_roundtrip(image, coef, recon=None, sums_buf=None, *, stream=None, height=None, width=None,
                   accumulate=False):
    """Pre-resolved round-trip launch (like bind): a zero-argument callable.
    sums_buf: an int64 CUDA tensor of 3 elements, or None.  accumulate=True:
    the frame's sums are added to sums_buf, which the caller zeroes
    (hpdct_roundtrip_u8_accumulate: the same kernels, the finish adds)."""
    if accumulate and sums_buf is None:
        raise HpdctError(1, "accumulate=True needs a sums buffer")
    args = _roundtrip_args(image, coef, recon, sums_buf, height, width, stream)
    lib = load_library()
    fn = lib.hpdct_roundtrip_u8_accumulate if accumulate else lib.hpdct_roundtrip_u8

    def call():
        st = fn(*args)
        if st:
            _check(st)
    return call


def baseline_forward(kind: str, image, tmp, result, transform, stream=None) -> None:
    """A/B baselines (include/hpdct_baseline.h): the reference's 3-launch
    HpApprDCT structure or the fastApprDCT row-per-thread structure on the GPU.
    Mutates `image` to X-128 like the reference."""
    if kind not in BASELINES:
        raise ValueError(f"kind must be one of {sorted(BASELINES)}")
    torch = _torch()
    _device_plane(image, "image", None, 0, (torch.float32,))
    h, w = _hw(image, None, None)
    for t, what in ((tmp, "tmp"), (result, "result")):
        _device_plane(t, what, image.device, h * w, (torch.float32,))
    if _transform_ptr(transform, image.device) is None:
        raise HpdctError(1, "the baselines take the caller's transform (64 floats on the device)")
    st = load_library().hpdct_baseline_forward(BASELINES[kind], ctypes.c_void_p(image.data_ptr()),
                                               ctypes.c_void_p(tmp.data_ptr()), ctypes.c_void_p(result.data_ptr()),
                                               h, w, ctypes.c_void_p(transform.data_ptr()), _stream_ptr(stream))
    if st:
        raise HpdctError(st, "baseline launch failed")


def _frame_list(frames, outs, out_dtype):
    """Checks of one frame list (the C-ABI sees only the pointer tables):
    every frame a contiguous uint8 CUDA tensor of one shape on one device,
    every out a contiguous plane of h*w elements of one coefficient dtype."""
    torch = _torch()
    frames = list(frames)
    if not frames:
        return frames, [], 0, 0
    _device_plane(frames[0], "frame 0", None, 0, (torch.uint8,))
    h, w = _hw(frames[0], None, None)
    shape, dev = tuple(frames[0].shape), frames[0].device
    for i, f in enumerate(frames):
        _device_plane(f, f"frame {i}", dev, h * w, (torch.uint8,))
        if tuple(f.shape) != shape:
            raise HpdctError(1, f"frame {i}: shape {tuple(f.shape)}, frame 0 is {shape}")
    if outs is None:
        outs = [torch.empty(shape, dtype=out_dtype or torch.float32, device=dev) for _ in frames]
    outs = list(outs)
    if len(outs) != len(frames):
        raise HpdctError(1, f"{len(frames)} frames but {len(outs)} coefficient planes")
    odt = outs[0].dtype
    for i, o in enumerate(outs):
        _device_plane(o, f"out {i}", dev, h * w, (torch.float32, torch.int8))
        if o.dtype != odt:
            raise HpdctError(1, f"out {i}: dtype {o.dtype}, out 0 is {odt}")
    return frames, outs, h, w


def forward_frames(frames, outs=None, *, out_dtype=None, stream=None):
    """A list of independent uint8 frames (CUDA tensors of one shape, need not
    be contiguous with each other) -> their quantised coefficients, one kernel
    launch per 64 frames (hpdct_forward_frames).  Built-in T, library Q.
    Bit-identical to forward() per frame; returns the list of outs."""
    frames, outs, h, w = _frame_list(frames, outs, out_dtype)
    n = len(frames)
    if n == 0:
        return outs
    fp = (ctypes.c_void_p * n)(*[f.data_ptr() for f in frames])
    op = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
    _check(load_library().hpdct_forward_frames(fp, op, _dtype_code(outs[0]), n, h, w, _stream_ptr(stream)))
    return outs


def bind_frames(frames, outs, *, stream=None):
    """forward_frames with every argument resolved once: a zero-argument
    callable (bench.py's timed loop)."""
    frames, outs, h, w = _frame_list(frames, outs, None)
    n = len(frames)
    fp = (ctypes.c_void_p * n)(*[f.data_ptr() for f in frames])
    op = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
    fn, args = load_library().hpdct_forward_frames, (fp, op, _dtype_code(outs[0]), n, h, w, _stream_ptr(stream))

    def call():
        st = fn(*args)
        if st:
            _check(st)
    return call


def _stream_lists(frames, outs):
    """Checks of a C5 batch; returns (n, h, w, out dtype code, frame and out pointer arrays)."""
    torch = _torch()
    n = len(frames)
    if n != len(outs) or n == 0:
        raise HpdctError(1, "frames and outs must be non-empty lists of equal length")
    h, w = _hw(frames[0], None, None)
    # the library copies h*w bytes in and h*w coefficients out per frame from
    # these host pointers: every entry must be exactly that large
    shape, odt = tuple(frames[0].shape), outs[0].dtype
    if odt not in (torch.float32, torch.int8):
        raise HpdctError(2, f"coefficient planes must be float32 or int8, not {odt}")
    for i, (f, o) in enumerate(zip(frames, outs)):
        if f.is_cuda or o.is_cuda:
            raise HpdctError(1, f"frame {i}: frames and outs are host (pinned) tensors")
        if not (f.is_contiguous() and o.is_contiguous()):
            raise HpdctError(1, f"frame {i}: host tensors must be contiguous")
        if f.dtype != torch.uint8 or tuple(f.shape) != shape:
            raise HpdctError(1, f"frame {i}: expected a uint8 {shape} frame, got {f.dtype} {tuple(f.shape)}")
        if o.dtype != odt or o.numel() != h * w:
            raise HpdctError(1, f"out {i}: expected {h * w} {odt} elements, got {o.numel()} {o.dtype}")
    fp = (ctypes.c_void_p * n)(*[f.data_ptr() for f in frames])
    op = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
    return n, h, w, _dtype_code(outs[0]), fp, op


def stream_forward(frames, outs, nstreams: int = 3) -> float:
    """Config C5: host-resident (pinned) uint8 frames -> host coefficient planes
    with H2D / kernel / D2H overlapped over `nstreams` HIP streams.  `frames`
    and `outs` are equal-length lists of CPU tensors (entries may repeat).
    Returns the device-timed milliseconds of the whole batch.  One-shot:
    streams and device buffers are made and freed per call (StreamContext
    keeps them)."""
    n, h, w, odt, fp, op = _stream_lists(frames, outs)
    ms = ctypes.c_float()
    _check(load_library().hpdct_stream_forward(fp, op, n, h, w, odt, int(nstreams), ctypes.byref(ms)))
    return ms.value


class StreamContext:
    """A persistent C5 pipeline (hpdct_stream_create / _run / _destroy): the
    HIP streams, the device ring (one input + one output frame per stream)
    and the timing events are created once, on the current device, for
    height x width frames and one coefficient dtype; run() streams a batch
    through them like stream_forward()."""

    def __init__(self, height: int, width: int, out_dtype, nstreams: int = 3):
        torch = _torch()
        if out_dtype not in (torch.float32, torch.int8):
            raise HpdctError(2, f"coefficient planes must be float32 or int8, not {out_dtype}")
        self.height, self.width, self.out_dtype = int(height), int(width), out_dtype
        self.handle = ctypes.c_void_p()
        _check(load_library().hpdct_stream_create(ctypes.byref(self.handle), self.height, self.width,
                                                  F32 if out_dtype == torch.float32 else I8, int(nstreams)))

    def run(self, frames, outs) -> float:
        if not self.handle:
            raise HpdctError(1, "stream context is closed")
        n, h, w, _, fp, op = _stream_lists(frames, outs)
        if (h, w) != (self.height, self.width) or outs[0].dtype != self.out_dtype:
            raise HpdctError(1, f"context is for {self.height}x{self.width} -> {self.out_dtype} frames")
        ms = ctypes.c_float()
        _check(load_library().hpdct_stream_run(self.handle, fp, op, n, ctypes.byref(ms)))
        return ms.value

    def close(self) -> None:
        if self.handle:
            _check(load_library().hpdct_stream_destroy(self.handle))
            self.handle = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fill_hash_u8(out, seed: int, first_index: int = 0, stream=None):
    """Device-side synthetic frame: out[i] = splitmix64(seed, first_index+i) & 255."""
    _device_plane(out, "out", None, 0, (_torch().uint8,))
    _check(load_library().hpdct_fill_hash_u8(ctypes.c_void_p(out.data_ptr()), out.numel(),
                                             ctypes.c_uint64(seed), first_index, _stream_ptr(stream)))
    return out


def decode_i8_f32(q, out=None, stream=None):
    """int8 wire coefficients -> the fp32 coefficient plane (HIP kernel,
    hpdct_decode_i8_f32): equal in value to the fp32 forward's output."""
    torch = _torch()
    _device_plane(q, "q", None, 0, (torch.int8,))
    if out is None:
        out = torch.empty(q.shape, dtype=torch.float32, device=q.device)
    _device_plane(out, "out", q.device, q.numel(), (torch.float32,))
    _check(load_library().hpdct_decode_i8_f32(ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                              q.numel(), _stream_ptr(stream)))
    return out


PROBE_EMPTY, PROBE_COPY = 0, 1


def bind_floor_probe(kind: int, img=None, out=None, height: int = 0, width: int = 0, stream=None):
    """Measurement floor of the uint8 -> fp32 forward of a height x width
    frame (hpdct_floor_probe), as a zero-argument callable like bind():
    PROBE_EMPTY an empty kernel on that forward's grid, PROBE_COPY the same
    grid copying img (uint8) to out as fp32."""
    torch = _torch()
    ip = op = None
    if kind == PROBE_COPY:
        _device_plane(img, "img", None, int(height) * int(width), (torch.uint8,))
        _device_plane(out, "out", img.device, int(height) * int(width), (torch.float32,))
        ip, op = ctypes.c_void_p(img.data_ptr()), ctypes.c_void_p(out.data_ptr())
    fn = load_library().hpdct_floor_probe
    args = (int(kind), ip, op, int(height), int(width), _stream_ptr(stream))

    def call():
        st = fn(*args)
        if st:
            _check(st)
    return call


def floor_probe(kind: int, img=None, out=None, height: int = 0, width: int = 0, stream=None) -> None:
    bind_floor_probe(kind, img, out, height, width, stream)()


def bind_copy_ceiling(src, out0, out1=None, *, cap_waves: int = 0, stream=None):
    """The copy ceiling of a kernel that reads src and writes out0 (and out1)
    (hpdct_copy_ceiling, include/hpdct_baseline.h): the same bytes per pixel,
    no arithmetic, at most cap_waves resident one-wave workgroups per CU
    (0: no cap).  A zero-argument callable like bind().  Measurement only."""
    _device_plane(src, "src", None, 0)
    n = src.numel()
    for name, t in (("out0", out0), ("out1", out1)):
        if t is not None:
            _device_plane(t, name, src.device, n)
    args = (ctypes.c_void_p(src.data_ptr()), _dtype_code(src), ctypes.c_void_p(out0.data_ptr()), _dtype_code(out0),
            None if out1 is None else ctypes.c_void_p(out1.data_ptr()), F32 if out1 is None else _dtype_code(out1),
            n, int(cap_waves), _stream_ptr(stream))
    fn = load_library().hpdct_copy_ceiling

    def call():
        st = fn(*args)
        if st:
            _check(st)
    return call


def release_sums(sums_buf) -> None:
    """Return the library's 16 KiB spread slot kept for this sums buffer
    (hpdct_roundtrip_release_sums); call when no round trip with it is in
    flight (e.g. before freeing a ring of sums buffers)."""
    _device_plane(sums_buf, "sums_buf", None, 3, (_torch().int64,))
    _check(load_library().hpdct_roundtrip_release_sums(ctypes.c_void_p(sums_buf.data_ptr())))


# ---------------------------------------------------------------------------
# the reference's own C++ entry points (compat layer, synchronous, prints)
# ---------------------------------------------------------------------------
def _compat_call(key, image_matrix, img_height, img_width, transform_matrix, result, *extra):
    """Buffer checks the C++ entry points cannot make (they see raw pointers):
    fp32 CUDA planes of >= h*w elements and a 64-float device T.  Shape
    errors the reference itself reports (W, H not multiples of 8) are left to
    the library, which prints and exits like CHECK_CUDA."""
    torch = _torch()
    h, w = int(img_height), int(img_width)
    need = max(h, 0) * max(w, 0)
    _device_plane(image_matrix, "image_matrix", None, need, (torch.float32,))
    _device_plane(result, "result", image_matrix.device, need, (torch.float32,))
    tptr = _transform_ptr(transform_matrix, image_matrix.device)
    if tptr is None:
        raise HpdctError(1, "transform_matrix: the reference entry points take the caller's device T")
    f = getattr(load_library(), COMPAT_SYMBOLS[key])
    f(ctypes.c_void_p(image_matrix.data_ptr()), h, w, tptr, ctypes.c_void_p(result.data_ptr()), *extra)


def dct_all_blocks_cuda(image_matrix, img_height: int, img_width: int, transform_matrix, result) -> None:
    """main_newAppr.cu:252-291 semantics: device fp32 buffers, caller's T,
    X-128 left in image_matrix, timing line on stdout, exits on error."""
    _compat_call("dct_all_blocks_cuda", image_matrix, img_height, img_width, transform_matrix, result)


def idct_all_blocks_cuda(image_matrix, img_height: int, img_width: int, transform_matrix, result) -> None:
    """main_newAppr.cu:293-332 semantics."""
    _compat_call("idct_all_blocks_cuda", image_matrix, img_height, img_width, transform_matrix, result)


def dct_all_blocks(image_matrix, img_height: int, img_width: int, transform_matrix, result, handle=None) -> None:
    """cublasDCTv2 surface (main_cublass_2.cu:197-252): row pass first, X-128
    left in image_matrix; the cuBLAS handle is accepted and ignored."""
    _compat_call("dct_all_blocks", image_matrix, img_height, img_width, transform_matrix, result, handle)


def idct_all_blocks(image_matrix, img_height: int, img_width: int, transform_matrix, result, handle=None) -> None:
    """main_cublass_2.cu:257-311: q*Q left in image_matrix, D.T first."""
    _compat_call("idct_all_blocks", image_matrix, img_height, img_width, transform_matrix, result, handle)


# ---------------------------------------------------------------------------
# host helpers (no device work)
# ---------------------------------------------------------------------------
def fill_rand_u8(n: int, seed: int = 42) -> np.ndarray:
    """srand(seed); rand() % 256, n values (benchmark_newAppr.cu:46-51)."""
    a = np.empty(int(n), np.uint8)
    load_library().hpdct_fill_rand_u8(a.ctypes.data, int(n), ctypes.c_uint32(seed))
    return a


def convert_to_float(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint8)
    o = np.empty(a.shape, np.float32)
    load_library().hpdct_u8_to_f32(a.ctypes.data, o.ctypes.data, a.size)
    return o


def convert_to_unsigned_char(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32)
    o = np.empty(a.shape, np.uint8)
    load_library().hpdct_f32_to_u8(a.ctypes.data, o.ctypes.data, a.size)
    return o


# ---------------------------------------------------------------------------
# row-shard layer over RCCL (include/hpdct_dist.h, lib/libhpdct_dist.so):
# BASELINE config C4.  The reference has no multi-GPU code.
# ---------------------------------------------------------------------------
DIST_LIB_PATH = os.environ.get("HPDCT_DIST_LIB", os.path.join(_HERE, "lib", "libhpdct_dist.so"))
DIST_SYMBOLS = [
    "hpdct_shard_rows", "hpdct_comm_init_all", "hpdct_comm_unique_id", "hpdct_comm_init_rank",
    "hpdct_comm_destroy", "hpdct_comm_rank", "hpdct_comm_size", "hpdct_comm_device",
    "hpdct_group_start", "hpdct_group_end", "hpdct_forward_slab", "hpdct_gather_rows", "hpdct_forward_sharded",
    "hpdct_gather_decode_i8",
]
UNIQUE_ID_BYTES = 128
_dist = None


def load_dist_library() -> ctypes.CDLL:
    """Load (once) libhpdct_dist.so; it needs librccl.so.1 (inside a torch
    process that is torch's own RCCL, already loaded under the same soname)."""
    global _dist
    if _dist is not None:
        return _dist
    load_library()
    if not os.path.exists(DIST_LIB_PATH):
        raise HpdctLibraryError(f"{DIST_LIB_PATH} not found: build it with `make -C cuda-dct-idct_amd`")
    try:
        lib = ctypes.CDLL(DIST_LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the loader
        raise HpdctLibraryError(f"cannot load {DIST_LIB_PATH}: {e}") from e
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.hpdct_shard_rows.argtypes = [i64, ci, ci, vp, vp]
    lib.hpdct_comm_init_all.argtypes = [vp, ci, vp]
    lib.hpdct_comm_unique_id.argtypes = [vp]
    lib.hpdct_comm_init_rank.argtypes = [vp, ci, vp, ci, ci]
    lib.hpdct_comm_destroy.argtypes = [vp]
    for f in (lib.hpdct_comm_rank, lib.hpdct_comm_size, lib.hpdct_comm_device):
        f.argtypes = [vp]
        f.restype = ci
    lib.hpdct_group_start.argtypes = []
    lib.hpdct_group_end.argtypes = []
    lib.hpdct_forward_slab.argtypes = [vp, vp, vp, ci, i64, i64, vp]
    lib.hpdct_gather_rows.argtypes = [vp, vp, vp, ci, i64, i64, ci, vp]
    lib.hpdct_forward_sharded.argtypes = [vp, vp, vp, ci, vp, i64, i64, ci, vp]
    lib.hpdct_gather_decode_i8.argtypes = [vp, vp, vp, vp, i64, i64, ci, vp]
    for name in DIST_SYMBOLS:
        if name not in ("hpdct_comm_rank", "hpdct_comm_size", "hpdct_comm_device"):
            getattr(lib, name).restype = ci
    _dist = lib
    return lib


def shard_rows_native(height: int, world: int, rank: int):
    """(first_row, rows) of `rank` from the C-ABI (hpdct_shard_rows)."""
    first, rows = ctypes.c_int64(), ctypes.c_int64()
    _check(load_dist_library().hpdct_shard_rows(int(height), int(world), int(rank), ctypes.byref(first),
                                                ctypes.byref(rows)))
    return first.value, rows.value


def comm_unique_id() -> bytes:
    """ncclGetUniqueId (rank 0 creates it, the caller hands it to every rank)."""
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    _check(load_dist_library().hpdct_comm_unique_id(buf))
    return buf.raw


class Comm:
    """An RCCL communicator of the row-shard layer (hpdct_comm)."""

    def __init__(self, handle: int):
        self.handle = ctypes.c_void_p(handle)

    @classmethod
    def init_all(cls, devices):
        """One communicator per device of this process (ncclCommInitAll)."""
        devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        hs = (ctypes.c_void_p * len(devices))()
        _check(load_dist_library().hpdct_comm_init_all(hs, len(devices), devs))
        return [cls(h) for h in hs]

    @classmethod
    def init_rank(cls, nranks: int, unique_id: bytes, rank: int, device: int):
        """One communicator per process (ncclCommInitRank on `device`)."""
        if len(unique_id) != UNIQUE_ID_BYTES:
            raise HpdctError(1, f"unique id must be {UNIQUE_ID_BYTES} bytes")
        h = ctypes.c_void_p()
        uid = ctypes.create_string_buffer(bytes(unique_id), UNIQUE_ID_BYTES)
        _check(load_dist_library().hpdct_comm_init_rank(ctypes.byref(h), int(nranks), uid, int(rank), int(device)))
        return cls(h.value)

    @property
    def rank(self) -> int:
        return load_dist_library().hpdct_comm_rank(self.handle)

    @property
    def size(self) -> int:
        return load_dist_library().hpdct_comm_size(self.handle)

    @property
    def device(self) -> int:
        return load_dist_library().hpdct_comm_device(self.handle)

    def destroy(self) -> None:
        if self.handle:
            _check(load_dist_library().hpdct_comm_destroy(self.handle))
            self.handle = ctypes.c_void_p()


def group_start() -> None:
    _check(load_dist_library().hpdct_group_start())


def group_end() -> None:
    _check(load_dist_library().hpdct_group_end())


def forward_slab(comm: Comm, slab, coef_slab, height: int, width: int, stream=None) -> None:
    """The fused forward kernel on this rank's slab (hpdct_forward_slab):
    slab = rows x width uint8 of the height x width frame, rows from
    shard_rows_native(height, comm.size, comm.rank)."""
    torch = _torch()
    _, rows = shard_rows_native(height, comm.size, comm.rank)
    _device_plane(slab, "slab", None, rows * width, (torch.uint8,))
    _device_plane(coef_slab, "coefficient slab", slab.device, rows * width, (torch.float32, torch.int8))
    _check(load_dist_library().hpdct_forward_slab(comm.handle, ctypes.c_void_p(slab.data_ptr()),
                                                  ctypes.c_void_p(coef_slab.data_ptr()), _dtype_code(coef_slab),
                                                  int(height), int(width), _stream_ptr(stream)))


def gather_rows(comm: Comm, slab, frame, height: int, width: int, root: int = 0, stream=None) -> None:
    """Every rank's slab to the root's height x width `frame` over RCCL
    (hpdct_gather_rows); `frame` is ignored (may be None) off the root."""
    _, rows = shard_rows_native(height, comm.size, comm.rank)
    _device_plane(slab, "slab", None, rows * width)
    fp = None
    if comm.rank == root:
        _device_plane(frame, "frame", slab.device, int(height) * int(width), (slab.dtype,))
        fp = ctypes.c_void_p(frame.data_ptr())
    _check(load_dist_library().hpdct_gather_rows(comm.handle, ctypes.c_void_p(slab.data_ptr()), fp,
                                                 _dtype_code(slab), int(height), int(width), int(root),
                                                 _stream_ptr(stream)))


def gather_decode_i8(comm: Comm, slab8, frame8, frame, height: int, width: int, root: int = 0,
                     stream=None) -> None:
    """The int8 wire format's gather (hpdct_gather_decode_i8): every rank but
    the root sends its int8 slab; the root, whose own slab is already fp32 at
    its rows of `frame` (pass slab8=None there), receives the peers' slabs
    into the int8 scratch `frame8` and decodes them into `frame`.  frame8 and
    frame are ignored (may be None) off the root."""
    torch = _torch()
    n = int(height) * int(width)
    sp = f8 = ff = None
    if comm.rank != root:
        _, rows = shard_rows_native(height, comm.size, comm.rank)
        _device_plane(slab8, "slab", None, rows * int(width), (torch.int8,))
        sp = ctypes.c_void_p(slab8.data_ptr())
    else:
        _device_plane(frame8, "frame8", None, n, (torch.int8,))
        _device_plane(frame, "frame", frame8.device, n, (torch.float32,))
        f8, ff = ctypes.c_void_p(frame8.data_ptr()), ctypes.c_void_p(frame.data_ptr())
    _check(load_dist_library().hpdct_gather_decode_i8(comm.handle, sp, f8, ff, int(height), int(width), int(root),
                                                      _stream_ptr(stream)))
