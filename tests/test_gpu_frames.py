"""GPU parity of hpdct_forward_frames: a list of separately allocated uint8
frames in one launch per 64 frames (the answer to config C2's dispatch-bound
single-frame launches; the reference has no batch entry, dct_all_blocks_cuda
takes one image, main_newAppr.cu:252).

Every frame's coefficients must equal hpdct_forward on that frame alone BIT FOR
BIT, and sampled frames equal the CPU oracle (the checker only).  Cases: more
than 64 frames (two launches, the second ragged), a width that is not a
multiple of 512 px (the straddle-capable stores), the C2 1024^2 frame size in
fp32 and int8, an input pool repeated across the list, and a custom integer
quant table (the verified fast quotient) against an IEEE-division one.  Since
round 6 a large enough fp32 list of whole-run widths runs on the duo forward
(1024^2 x 33, 256 x 2048 x 70 in two launches) while each frame alone takes
the octet kernel: the two mappings must agree bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames(hp, dev, n, h, w, seed0):
    import torch
    out = []
    for k in range(n):
        x = torch.empty((h, w), dtype=torch.uint8, device=dev)
        hp.fill_hash_u8(x, seed=seed0 + k)
        out.append(x)
        # a spacer allocation so the frames are not one contiguous plane
        out.append(torch.empty(4096 + 64 * k, dtype=torch.uint8, device=dev))
    return out[0::2]


def _bits(t):
    import torch
    return t.view(torch.int32) if t.dtype == torch.float32 else t


@pytest.mark.parametrize("out_dtype", ["float32", "int8"])
@pytest.mark.parametrize("h,w,n", [(64, 136, 70), (1024, 1024, 33), (48, 4096, 3), (8, 8, 1), (256, 2048, 70)])
def test_frames_equal_per_frame_forward(hp, dev, out_dtype, h, w, n):
    import torch
    dt = getattr(torch, out_dtype)
    frames = _frames(hp, dev, n, h, w, seed0=100 + h + w)
    outs = hp.forward_frames(frames, out_dtype=dt)
    for k, (x, y) in enumerate(zip(frames, outs)):
        ref = hp.forward(x, out_dtype=dt)
        assert torch.equal(_bits(ref), _bits(y)), f"frame {k} of {n} ({h}x{w}, {out_dtype})"


def test_frames_vs_oracle_and_repeated_pool(hp, oracle, dev):
    import torch
    pool = _frames(hp, dev, 3, 64, 1040, seed0=7)
    frames = [pool[k % 3] for k in range(130)]  # inputs repeat; outputs are distinct
    outs = hp.forward_frames(frames)
    torch.cuda.synchronize()
    for k in (0, 1, 2, 64, 65, 129):
        ref = oracle.fdct(frames[k].cpu().numpy())
        assert np.array_equal(outs[k].cpu().numpy().view(np.uint32), ref.view(np.uint32)), f"frame {k}"
    for k in range(3, 130):
        assert torch.equal(_bits(outs[k]), _bits(outs[k % 3]))


@pytest.mark.parametrize("table", ["integer", "fractional"])
def test_frames_custom_quant_table(hp, oracle, dev, table):
    """Integer table in 1..255: the verified 3-op quotient; fractional: IEEE
    division.  Both must match the oracle under that table."""
    import torch
    q = np.arange(1, 65, dtype=np.float32) * (1.0 if table == "integer" else 1.37)
    hp.set_quant_table(q)
    try:
        frames = _frames(hp, dev, 5, 16, 512, seed0=900)
        outs = hp.forward_frames(frames)
        torch.cuda.synchronize()
        for k, (x, y) in enumerate(zip(frames, outs)):
            ref = oracle.fdct(x.cpu().numpy(), Q=q)
            assert np.array_equal(y.cpu().numpy().view(np.uint32), ref.view(np.uint32)), f"frame {k}"
    finally:
        hp.set_quant_table(None)


def test_frames_on_a_side_stream(hp, dev):
    import torch
    s = torch.cuda.Stream()
    frames = _frames(hp, dev, 4, 256, 256, seed0=55)
    torch.cuda.synchronize()
    outs = [torch.empty((256, 256), dtype=torch.float32, device=dev) for _ in frames]
    with torch.cuda.stream(s):
        call = hp.bind_frames(frames, outs, stream=s)
        call()
    s.synchronize()
    for x, y in zip(frames, outs):
        assert torch.equal(_bits(hp.forward(x)), _bits(y))


@pytest.mark.parametrize("pattern", ["u8_f32", "u8_i8", "f32_f32", "f32_f32_f32inplace", "u8_f32_u8", "u8_f32_f32"])
@pytest.mark.parametrize("cap", [0, 4])
def test_copy_ceiling_moves_the_kernels_bytes(hp, dev, pattern, cap):
    """hpdct_copy_ceiling (include/hpdct_baseline.h), the ceiling bench.py puts
    beside every kernel, really reads and writes every byte it is charged for:
    each output element is the input element converted (u8 -> f32 exactly,
    f32 -> 1 B by truncation of the value), the in-place write-back included."""
    import torch
    n = 2048 * 37
    gen = torch.Generator(device="cpu").manual_seed(7)
    src_u8 = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=gen).to(dev)
    src_f32 = src_u8.float()
    kinds = pattern.split("_")
    src = src_u8 if kinds[0] == "u8" else src_f32.clone()
    dt = {"u8": torch.uint8, "i8": torch.int8, "f32": torch.float32, "f32inplace": torch.float32}
    o0 = torch.full((n,), 77, dtype=dt[kinds[1]], device=dev)
    o1 = None
    if len(kinds) > 2:
        o1 = src if kinds[2] == "f32inplace" else torch.full((n,), 77, dtype=dt[kinds[2]], device=dev)
    hp.bind_copy_ceiling(src, o0, o1, cap_waves=cap)()
    torch.cuda.synchronize()
    want = {torch.float32: src_f32, torch.uint8: src_u8, torch.int8: src_u8.view(torch.int8)}
    assert torch.equal(o0, want[o0.dtype])
    if o1 is not None:
        assert torch.equal(o1, want[o1.dtype])
