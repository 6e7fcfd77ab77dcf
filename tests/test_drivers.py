"""The HIP-native counterparts of the reference's two programs
(benchmark_newAppr.cu:33-119, main_newAppr.cu:26-168), run as processes on the
GPU: same CLI, same stdout lines, same output image.  The JPEG round trip is
compared byte-for-byte with what the reference's own save_grayscale_jpeg
(utils.cu:98-147, compiled in oracle/_ref) writes for the expected pixels."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "cuda-dct-idct_amd", "bin")


def run(args, **kw):
    return subprocess.run(args, capture_output=True, text=True, timeout=300, **kw)


def test_benchmark_cli():
    p = run([os.path.join(BIN, "benchmark_hpdct"), "256"])
    assert p.returncode == 0, p.stdout + p.stderr
    assert re.search(r"^DCT \(256,256\): [0-9.]+ ms$", p.stdout, re.M)
    assert re.search(r"^IDCT \(256,256\): [0-9.]+ ms$", p.stdout, re.M)
    p = run([os.path.join(BIN, "benchmark_hpdct")])
    assert p.returncode == 1 and "Use:" in p.stdout


def test_benchmark_cli_repeated_runs():
    """Optional run count (tools/size_sweep.py): the reference's call sequence
    and lines repeated, one DCT and one IDCT line per run."""
    p = run([os.path.join(BIN, "benchmark_hpdct"), "64", "3"])
    assert p.returncode == 0, p.stdout + p.stderr
    assert len(re.findall(r"^DCT \(64,64\): [0-9.]+ ms$", p.stdout, re.M)) == 3
    assert len(re.findall(r"^IDCT \(64,64\): [0-9.]+ ms$", p.stdout, re.M)) == 3


def _write_pgm(path, img):
    with open(path, "wb") as fh:
        fh.write(b"P5\n%d %d\n255\n" % (img.shape[1], img.shape[0]))
        fh.write(img.tobytes())


def _read_pgm(path):
    data = open(path, "rb").read()
    m = re.match(rb"P5\s+(\d+)\s+(\d+)\s+255\s", data)
    w, h = int(m.group(1)), int(m.group(2))
    return np.frombuffer(data[m.end():], np.uint8).reshape(h, w)


def test_interactive_pgm(tmp_path, oracle):
    img = oracle.rand_u8(64 * 72, 9).reshape(64, 72)
    src, dst = tmp_path / "in.pgm", tmp_path / "out.pgm"
    _write_pgm(src, img)
    p = run([os.path.join(BIN, "main_hpdct"), str(src), str(dst)])
    assert p.returncode == 0, p.stdout + p.stderr
    expect = oracle.to_u8(oracle.idct(oracle.fdct(img)))
    assert np.array_equal(_read_pgm(dst), expect)
    assert "Printing the 8x8 of result[] (matrix coming from the dct)" in p.stdout
    assert "Image saved successfully to" in p.stdout
    # first printed coefficient row equals the oracle's
    q = oracle.fdct(img)
    block = p.stdout.split("(matrix coming from the dct)\n", 1)[1].splitlines()[0]
    assert [float(v) for v in block.split()] == [float(v) for v in q[0, :8]]


def test_interactive_crops_to_multiple_of_8(tmp_path, oracle):
    img = oracle.rand_u8(30 * 45, 3).reshape(30, 45)
    src, dst = tmp_path / "in.pgm", tmp_path / "out.pgm"
    _write_pgm(src, img)
    p = run([os.path.join(BIN, "main_hpdct"), str(src), str(dst)])
    assert p.returncode == 0, p.stdout + p.stderr
    crop = np.ascontiguousarray(img[:24, :40])
    assert np.array_equal(_read_pgm(dst), oracle.to_u8(oracle.idct(oracle.fdct(crop))))


def test_interactive_jpeg_matches_reference_writer(tmp_path, oracle):
    R = oracle.ref_utils()
    if R is None:
        pytest.skip("oracle/_ref (the reference's utils.cu) not built")
    R._Z19save_grayscale_jpegPKcPhiii.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_int]
    R._Z19save_grayscale_jpegPKcPhiii.restype = ctypes.c_int
    img = oracle.rand_u8(48 * 64, 5).reshape(48, 64)
    src, dst, ref = tmp_path / "in.jpg", tmp_path / "out.jpg", tmp_path / "ref.jpg"
    assert R._Z19save_grayscale_jpegPKcPhiii(str(src).encode(), img.ctypes.data, 64, 48, 100) == 1
    # decode the input the way the reference does (load_jpeg_as_matrix)
    R._Z19load_jpeg_as_matrixPKcPiS1_S1_.restype = ctypes.c_void_p
    w, h, ch = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    ptr = R._Z19load_jpeg_as_matrixPKcPiS1_S1_(str(src).encode(), ctypes.byref(w), ctypes.byref(h), ctypes.byref(ch))
    assert (w.value, h.value, ch.value) == (64, 48, 1)
    pixels = np.ctypeslib.as_array((ctypes.c_uint8 * (64 * 48)).from_address(ptr)).reshape(48, 64).copy()
    p = run([os.path.join(BIN, "main_hpdct"), str(src), str(dst)])
    assert p.returncode == 0, p.stdout + p.stderr
    expect = np.ascontiguousarray(oracle.to_u8(oracle.idct(oracle.fdct(pixels))))
    assert R._Z19save_grayscale_jpegPKcPhiii(str(ref).encode(), expect.ctypes.data, 64, 48, 100) == 1
    assert open(dst, "rb").read() == open(ref, "rb").read()
