"""CPU-side checks of the C-ABI boundary (no compute calls: there is no GPU here).

- libhpdct.so loads and exports every function include/*.h declares, with
  the reference's C++ mangled names for the compat entry points;
- argument validation fails with the documented status before any device
  work is attempted;
- the host helpers reproduce the reference's input stream and conversions.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")


DIST_HEADER = "hpdct_dist.h"  # declares libhpdct_dist.so (the RCCL row-shard layer), not libhpdct.so


def header_functions(only=None):
    names = set()
    for fn in os.listdir(INCLUDE):
        if not fn.endswith(".h") or (fn == DIST_HEADER) != (only == DIST_HEADER):
            continue
        text = open(os.path.join(INCLUDE, fn)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for m in re.finditer(r"\b([A-Za-z_]\w*)\s*\([^;{}()]*\)\s*;", text):
            names.add(m.group(1))
    return names


def exported_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_exports_every_declared_symbol(hp):
    declared = header_functions()
    assert {"hpdct_forward", "hpdct_inverse", "dct_all_blocks_cuda", "idct_all_blocks_cuda"} <= declared
    syms = exported_symbols(hp.LIB_PATH)
    for name in declared:
        if name in hp.COMPAT_SYMBOLS:
            assert hp.COMPAT_SYMBOLS[name] in syms, name
        else:
            assert name in syms, name
    assert set(hp.C_SYMBOLS) | set(hp.COMPAT_SYMBOLS) == declared


def test_dist_library_exports_every_declared_symbol(hp):
    declared = header_functions(only=DIST_HEADER)
    assert {"hpdct_gather_rows", "hpdct_forward_slab", "hpdct_comm_init_all"} <= declared
    syms = exported_symbols(hp.DIST_LIB_PATH)
    for name in declared:
        assert name in syms, name
    assert set(hp.DIST_SYMBOLS) == declared


def test_compat_mangling_matches_reference_signatures(tmp_path):
    # what g++ emits for the reference's own declarations (main_newAppr.cu:23-24)
    src = tmp_path / "decl.cpp"
    src.write_text(
        "void dct_all_blocks_cuda(float* image_matrix, const int img_height, const int img_width,"
        " const float* transform_matrix, float* result) {}\n"
        "void idct_all_blocks_cuda(const float* image_matrix, const int img_height, const int img_width,"
        " const float* transform_matrix, float* result) {}\n")
    obj = tmp_path / "decl.o"
    subprocess.run(["g++", "-c", str(src), "-o", str(obj)], check=True)
    out = subprocess.run(["nm", str(obj)], capture_output=True, text=True, check=True).stdout
    assert "_Z19dct_all_blocks_cudaPfiiPKfS_" in out
    assert "_Z20idct_all_blocks_cudaPKfiiS0_Pf" in out
    # cublasDCTv2 (main_cublass_2.cu:36-37), with cuBLAS's handle typedef
    src.write_text(
        "typedef struct cublasContext *cublasHandle_t;\n"
        "void dct_all_blocks(float *image_matrix, int img_height, int img_width, const float *transform_matrix,"
        " float *result, cublasHandle_t handle) {}\n"
        "void idct_all_blocks(float *image_matrix, int img_height, int img_width, const float *transform_matrix,"
        " float *result, cublasHandle_t handle) {}\n")
    subprocess.run(["g++", "-c", str(src), "-o", str(obj)], check=True)
    out = subprocess.run(["nm", str(obj)], capture_output=True, text=True, check=True).stdout
    assert "_Z14dct_all_blocksPfiiPKfS_P13cublasContext" in out
    assert "_Z15idct_all_blocksPfiiPKfS_P13cublasContext" in out


def test_kernels_are_gfx950_code_objects(hp):
    data = open(hp.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"_ZN5hpdct11fdct_kernel" in data and b"_ZN5hpdct11idct_kernel" in data


def test_version_and_status_strings(hp):
    assert "gfx950" in hp.version()
    L = hp.load_library()
    assert L.hpdct_status_string(0) == b"success"
    assert L.hpdct_status_string(3).startswith(b"quantised")


def test_build_provenance_matches_tree(hp):
    """The library carries the digest of the csrc/ + include/ it was built from
    (src_digest.py, stamped by the Makefile); a stale build (sources edited,
    library not rebuilt) fails here, and bench.py / smoke() print the same
    check on the GPU box."""
    info = hp.build_info()
    assert info.startswith("src=") and "arch=gfx950" in info
    prov = hp.provenance()
    assert prov["lib_matches_sources"] is True, prov


def test_tables_match_reference(hp, oracle):
    assert np.array_equal(hp.default_transform().view(np.uint32), oracle.default_transform().view(np.uint32))
    assert np.array_equal(hp.default_quant_table(), oracle.default_quant())


def ref_tables():
    """Q / T initialisers extracted from the reference's own .cu text
    (tests/golden/make_golden.py extract_tables), fp32 bit patterns."""
    import json
    doc = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_tables.json")))
    return {k: np.array(v["bits"], np.uint32) for k, v in doc["tables"].items()}, doc["tables"]


def test_tables_pinned_to_reference_text(hp, oracle):
    """The library's tables (the SAME constexpr arrays the kernels compile to
    immediates, csrc/hpdct_tables.h) and the oracle's are bit-identical to
    (float)(double)literal of main_newAppr.cu:60-81 and
    Benchmark_code/benchmark_newAppr.cu:54-75, and every other table in the
    reference agrees with them."""
    bits, meta = ref_tables()
    q_ref, t_ref = bits["main_newAppr.cu:60"], bits["main_newAppr.cu:73"]
    assert np.array_equal(bits["Benchmark_code/benchmark_newAppr.cu:54"], q_ref)
    assert np.array_equal(bits["Benchmark_code/benchmark_newAppr.cu:67"], t_ref)
    for k, v in bits.items():
        want = t_ref if meta[k]["name"] == "transform_matrix" else q_ref
        assert np.array_equal(v, want), k
    assert np.array_equal(hp.default_transform().reshape(-1).view(np.uint32), t_ref)
    assert np.array_equal(hp.default_quant_table().reshape(-1).view(np.uint32), q_ref)
    assert np.array_equal(oracle.default_transform().reshape(-1).view(np.uint32), t_ref)
    assert np.array_equal(oracle.default_quant().reshape(-1).view(np.uint32), q_ref)
    assert np.array_equal(hp.get_quant_table().reshape(-1).view(np.uint32), q_ref)


def test_kernel_tables_share_one_source():
    """hpdct_tile.hpp (kernel immediates) and hpdct_api.cpp (host C-ABI) both
    take the tables from hpdct_tables.h; neither restates a literal."""
    csrc = os.path.join(ROOT, "cuda-dct-idct_amd", "csrc")
    for fn in ("hpdct_tile.hpp", "hpdct_api.cpp"):
        text = open(os.path.join(csrc, fn)).read()
        assert '#include "hpdct_tables.h"' in text, fn
        assert "0.35355339" not in text and "121, 120, 101" not in text, fn


def test_quant_table_state(hp):
    q = np.arange(1, 65, dtype=np.float32).reshape(8, 8)
    hp.set_quant_table(q)
    try:
        assert np.array_equal(hp.get_quant_table(), q)
    finally:
        hp.set_quant_table(None)
    assert np.array_equal(hp.get_quant_table(), hp.default_quant_table())
    bad = np.ones(64, np.float32)
    bad[5] = 0.0
    with pytest.raises(hp.HpdctError) as e:
        hp.set_quant_table(bad)
    assert e.value.status == 1
    bad[5] = np.nan
    with pytest.raises(hp.HpdctError):
        hp.set_quant_table(bad)
    assert np.array_equal(hp.get_quant_table(), hp.default_quant_table())


def test_mapping_state(hp):
    assert hp.get_mapping() == "auto"
    try:
        for m in ("tile", "octet", "duo", "auto"):
            hp.set_mapping(m)
            assert hp.get_mapping() == m
        assert hp.load_library().hpdct_set_mapping(7) == 1  # HPDCT_ERROR_INVALID_VALUE
        assert hp.get_mapping() == "auto"
        with pytest.raises(ValueError):
            hp.set_mapping("wave")
    finally:
        hp.set_mapping("auto")


def test_mapping_from_environment(tmp_path):
    """HPDCT_MAPPING seeds the process-wide mapping (the GPU tests' child
    processes rely on it); an unknown value falls back to auto."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import hpdct; print(hpdct.get_mapping())"
            % os.path.join(ROOT, "cuda-dct-idct_amd"))
    for env_val, want in (("octet", "octet"), ("tile", "tile"), ("duo", "duo"), ("bogus", "auto")):
        env = dict(os.environ, HPDCT_MAPPING=env_val)
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
        assert out.stdout.strip() == want


@pytest.mark.parametrize("h,w", [(0, 8), (8, 0), (12, 8), (8, 20), (-8, 8), (7, 7)])
def test_bad_shapes_rejected_before_device_work(hp, h, w):
    L = hp.load_library()
    dummy = ctypes.c_void_p(256)  # never dereferenced: validation fails first
    st = L.hpdct_forward(dummy, hp.U8, ctypes.c_void_p(4096), hp.F32, h, w, None, 0, None)
    assert st == 1
    assert b"multiples of 8" in L.hpdct_last_error_string()
    st = L.hpdct_inverse(dummy, hp.F32, ctypes.c_void_p(4096), hp.F32, h, w, None, 0, None)
    assert st == 1


def test_decode_arguments_rejected(hp):
    """hpdct_decode_i8_f32 validates before any device work: n == 0 is a no-op
    (NULL allowed), NULL / negative / misaligned pointers are rejected."""
    L = hp.load_library()
    a, b = ctypes.c_void_p(1 << 20), ctypes.c_void_p(1 << 30)
    assert L.hpdct_decode_i8_f32(None, None, 0, None) == 0
    assert L.hpdct_decode_i8_f32(None, b, 64, None) == 1
    assert L.hpdct_decode_i8_f32(a, None, 64, None) == 1
    assert L.hpdct_decode_i8_f32(a, b, -1, None) == 1
    assert L.hpdct_decode_i8_f32(ctypes.c_void_p((1 << 20) + 2), b, 64, None) == 1
    assert L.hpdct_decode_i8_f32(a, ctypes.c_void_p((1 << 30) + 8), 64, None) == 1
    assert b"aligned" in L.hpdct_last_error_string()


def test_bad_arguments_rejected(hp):
    L = hp.load_library()
    a, b = ctypes.c_void_p(1 << 20), ctypes.c_void_p(1 << 30)
    assert L.hpdct_forward(None, hp.U8, b, hp.F32, 8, 8, None, 0, None) == 1
    assert L.hpdct_forward(a, hp.I8, b, hp.F32, 8, 8, None, 0, None) == 2  # int8 is not an image type
    assert L.hpdct_forward(a, hp.U8, b, hp.U8, 8, 8, None, 0, None) == 2
    assert L.hpdct_forward(a, hp.U8, b, hp.I8, 8, 8, None, hp.FLAG_NO_QUANT, None) == 2
    assert L.hpdct_forward(a, hp.U8, b, hp.F32, 8, 8, None, hp.FLAG_WRITEBACK_SHIFT, None) == 2
    assert L.hpdct_forward(a, hp.U8, b, hp.F32, 8, 8, None, 0x80, None) == 2
    assert L.hpdct_forward(ctypes.c_void_p((1 << 20) + 4), hp.F32, b, hp.F32, 8, 8, None, 0, None) == 1
    assert L.hpdct_forward(a, hp.F32, ctypes.c_void_p((1 << 20) + 64), hp.F32, 8, 8, None, 0, None) == 1  # overlap
    assert L.hpdct_inverse(a, hp.U8, b, hp.F32, 8, 8, None, 0, None) == 2
    assert L.hpdct_inverse(a, hp.F32, b, hp.I8, 8, 8, None, 0, None) == 2
    assert L.hpdct_inverse(a, hp.F32, b, hp.F32, 8, 8, None, hp.FLAG_WRITEBACK_SHIFT, None) == 2
    # cublasDCTv2 options are fp32 -> fp32 only; the dequant write-back needs dequantisation
    assert L.hpdct_forward(a, hp.U8, b, hp.F32, 8, 8, None, hp.FLAG_ROW_FIRST, None) == 2
    assert L.hpdct_forward(a, hp.F32, b, hp.F32, 8, 8, None, hp.FLAG_WRITEBACK_DEQUANT, None) == 2
    assert L.hpdct_inverse(a, hp.I8, b, hp.F32, 8, 8, None, hp.FLAG_ROW_FIRST, None) == 2
    assert L.hpdct_inverse(a, hp.F32, b, hp.U8, 8, 8, None, hp.FLAG_WRITEBACK_DEQUANT, None) == 2
    assert L.hpdct_inverse(a, hp.F32, b, hp.F32, 8, 8, None,
                           hp.FLAG_WRITEBACK_DEQUANT | hp.FLAG_NO_QUANT, None) == 2
    # int8 output refused when the table can overflow int8
    hp.set_quant_table(np.ones(64, np.float32))
    try:
        assert L.hpdct_forward(a, hp.U8, b, hp.I8, 8, 8, None, 0, None) == 3
    finally:
        hp.set_quant_table(None)


def test_roundtrip_arguments_rejected(hp):
    """hpdct_roundtrip_u8 validates before any device work (no GPU here)."""
    L = hp.load_library()
    a, b, c, s = (ctypes.c_void_p(1 << 20), ctypes.c_void_p(1 << 30), ctypes.c_void_p(1 << 31),
                  ctypes.c_void_p(1 << 32))
    rt = L.hpdct_roundtrip_u8
    assert rt(a, b, c, hp.U8, s, 8, 12, None) == 1           # width not a multiple of 8
    assert rt(None, b, c, hp.U8, s, 8, 8, None) == 1         # null image
    assert rt(a, None, c, hp.U8, s, 8, 8, None) == 1         # null coefficients
    assert rt(a, b, c, hp.I8, s, 8, 8, None) == 2            # int8 is not a reconstruction type
    assert rt(a, ctypes.c_void_p((1 << 30) + 4), c, hp.U8, s, 8, 8, None) == 1  # misaligned coefficients
    assert rt(a, b, c, hp.F32, ctypes.c_void_p((1 << 32) + 4), 8, 8, None) == 1  # misaligned sums
    assert rt(a, ctypes.c_void_p((1 << 20) + 16), None, hp.U8, None, 8, 8, None) == 1  # image/coef overlap
    assert rt(a, b, ctypes.c_void_p((1 << 30) + 64), hp.U8, None, 8, 8, None) == 1  # coef/recon overlap
    assert rt(a, b, c, hp.U8, ctypes.c_void_p((1 << 31) + 8), 8, 8, None) == 1  # sums inside the recon
    assert b"overlap" in L.hpdct_last_error_string()
    assert ctypes.sizeof(ctypes.c_uint64 * 3) == 24  # hpdct_roundtrip_sums: three uint64
    acc = L.hpdct_roundtrip_u8_accumulate
    assert acc(a, b, c, hp.U8, None, 8, 8, None) == 1          # accumulate needs the sums struct
    assert b"sums" in L.hpdct_last_error_string()
    assert acc(a, b, c, hp.U8, s, 8, 12, None) == 1            # same validation as hpdct_roundtrip_u8
    assert acc(a, b, c, hp.I8, s, 8, 8, None) == 2


def test_product_header_declares_only_the_path(hp):
    """include/hpdct.h is the path's API; the measurement
    probes (the C2 floors, the copy ceilings) are declared in hpdct_baseline.h
    beside the A/B baselines, not in the product header."""
    text = open(os.path.join(INCLUDE, "hpdct.h")).read()
    for name in ("hpdct_floor_probe", "hpdct_copy_ceiling", "hpdct_baseline_forward", "hpdct_probe_kind"):
        assert name not in text, name
    base = open(os.path.join(INCLUDE, "hpdct_baseline.h")).read()
    for name in ("hpdct_floor_probe", "hpdct_copy_ceiling", "hpdct_baseline_forward"):
        assert name + "(" in base, name


def test_copy_ceiling_and_release_arguments(hp):
    """hpdct_copy_ceiling validates before any device work (no GPU here);
    hpdct_roundtrip_release_sums of an unknown pointer or NULL is a no-op."""
    L = hp.load_library()
    a, b, c = ctypes.c_void_p(1 << 20), ctypes.c_void_p(1 << 30), ctypes.c_void_p(1 << 31)
    cc = L.hpdct_copy_ceiling
    assert cc(a, hp.U8, b, hp.F32, None, 0, 2048 * 3, -1, None) == 1        # negative cap
    assert cc(a, hp.U8, b, hp.F32, None, 0, 2000, 0, None) == 1             # n not a multiple of 2048
    assert cc(a, hp.U8, b, hp.F32, None, 0, 0, 0, None) == 1
    assert cc(None, hp.U8, b, hp.F32, None, 0, 2048, 0, None) == 1
    assert cc(a, hp.U8, ctypes.c_void_p((1 << 30) + 4), hp.F32, None, 0, 2048, 0, None) == 1  # misaligned
    assert cc(a, hp.U8, b, hp.F32, ctypes.c_void_p((1 << 31) + 8), hp.U8, 2048, 0, None) == 1
    assert cc(a, 7, b, hp.F32, None, 0, 2048, 0, None) == 2                  # unknown type
    assert cc(a, hp.U8, b, hp.F32, c, 9, 2048, 0, None) == 2
    assert L.hpdct_roundtrip_release_sums(None) == 0
    assert L.hpdct_roundtrip_release_sums(ctypes.c_void_p(1 << 33)) == 0


def test_forward_frames_arguments_rejected(hp):
    """hpdct_forward_frames validates the whole pointer table before any
    device work (no GPU here): shape, counts, nulls, alignment, overlaps."""
    L = hp.load_library()
    P = ctypes.c_void_p * 3
    ins = P(1 << 20, 1 << 21, 1 << 20)           # a repeated input is allowed
    outs = P(1 << 30, (1 << 30) + (1 << 22), 1 << 31)
    ff = L.hpdct_forward_frames
    assert ff(ins, outs, hp.F32, 0, 64, 64, None) == 0   # empty list: no-op
    assert ff(ins, outs, hp.F32, -1, 64, 64, None) == 1
    assert ff(ins, outs, hp.F32, 3, 64, 60, None) == 1   # width not a multiple of 8
    assert ff(None, outs, hp.F32, 3, 64, 64, None) == 1
    assert ff(ins, outs, hp.U8, 3, 64, 64, None) == 2    # coefficients are f32 or i8
    assert ff(P(1 << 20, None, 1 << 20), outs, hp.F32, 3, 64, 64, None) == 1
    assert ff(P(1 << 20, (1 << 21) + 4, 1 << 20), outs, hp.F32, 3, 64, 64, None) == 1  # misaligned frame
    assert ff(ins, P(1 << 30, (1 << 30) + (1 << 22) + 8, 1 << 31), hp.F32, 3, 64, 64, None) == 1  # f32: 16 B
    assert ff(ins, P(1 << 30, (1 << 30) + 64, 1 << 31), hp.F32, 3, 64, 64, None) == 1  # two outs overlap
    assert b"overlap" in L.hpdct_last_error_string()
    assert ff(ins, P(1 << 30, (1 << 21) + 64, 1 << 31), hp.I8, 3, 64, 64, None) == 1  # out inside an input
    hp.set_quant_table(np.ones(64, np.float32))
    try:
        assert ff(ins, outs, hp.I8, 3, 64, 64, None) == 3  # int8 overflow with this table
    finally:
        hp.set_quant_table(None)
    # a garbage count: the span table cannot be allocated; a status, not an
    # exception across the C ABI (std::terminate)
    assert ff(ins, outs, hp.F32, 1 << 62, 64, 64, None) == 1
    assert b"hpdct_forward_frames" in L.hpdct_last_error_string()
    # a large list from a small repeated pool: the overlap sweep is O(n log n)
    n = 20000
    many_in = (ctypes.c_void_p * n)(*[(1 << 20) + (k % 4) * (1 << 16) for k in range(n)])
    many_out = (ctypes.c_void_p * n)(*[(1 << 32) + k * (1 << 16) for k in range(n)])
    many_out[n - 1] = (1 << 20) + 8  # the last plane lands on a pool input
    t0 = time.perf_counter()
    assert ff(many_in, many_out, hp.I8, n, 64, 64, None) == 1
    assert time.perf_counter() - t0 < 1.0
    assert b"overlap" in L.hpdct_last_error_string()


def test_host_rand_matches_glibc(hp, oracle):
    assert np.array_equal(hp.fill_rand_u8(100000, 42), oracle.rand_u8(100000, 42))
    assert np.array_equal(hp.fill_rand_u8(5000, 7), oracle.rand_u8(5000, 7))


def test_host_conversions_match_reference(hp, oracle):
    z = np.load(os.path.join(ROOT, "tests", "golden", "ref_utils_convert.npz"))
    assert np.array_equal(hp.convert_to_float(z["u8_in"]), z["f32_out"])
    assert np.array_equal(hp.convert_to_unsigned_char(z["f32_in"]), z["u8_out"])
