"""Quality metrics (README.md:62-69 table; definitions in hpdct_quality)."""
import numpy as np
import pytest


def _zigzag_reference():
    # walk the anti-diagonals, alternating direction (the JPEG scan)
    order = []
    for s in range(15):
        cells = [(v, s - v) for v in range(8) if 0 <= s - v < 8]
        if s % 2 == 0:
            cells.reverse()  # even diagonals run bottom-left -> top-right
        order += [8 * v + u for v, u in cells]
    return order


def test_zigzag_table():
    import hpdct_quality as Qm
    assert sorted(Qm.ZIGZAG) == list(range(64))
    assert Qm.ZIGZAG == _zigzag_reference()
    m = Qm.retain_mask(6)
    assert int(m.sum()) == 6 and m[0, 0] == m[0, 1] == m[1, 0] == m[2, 0] == m[1, 1] == m[0, 2] == 1
    assert Qm.retain_mask(64).all() and not Qm.retain_mask(0).any()
    with pytest.raises(ValueError):
        Qm.retain_mask(65)


def _oracle_retain(oracle, img, k):
    import hpdct_quality as Qm
    c = oracle.fdct(img, quant=False)
    h, w = c.shape
    c = (c.reshape(h // 8, 8, w // 8, 8) * Qm.retain_mask(k)[None, :, None, :]).reshape(h, w)
    return oracle.idct(c.astype(np.float32), dequant=False)


@pytest.mark.gpu
def test_quality_matches_oracle(hp, oracle, dev):
    import torch
    import hpdct_quality as Qm
    img = oracle.rand_u8(64 * 128, 4).reshape(64, 128)
    x = torch.from_numpy(img).to(dev)
    std = Qm.evaluate(x)
    peen, mse = oracle.quality(img.astype(np.float32), oracle.idct(oracle.fdct(img)))
    assert abs(std["peen_pct"] - peen) < 1e-9 and abs(std["mse"] - mse) < 1e-9
    assert std["compression_factor"] > 0
    for k in (1, 6, 10, 64):
        r = Qm.evaluate(x, retain=k, with_cf=False)
        peen, mse = oracle.quality(img.astype(np.float32), _oracle_retain(oracle, img, k))
        assert abs(r["peen_pct"] - peen) < 1e-9 and abs(r["mse"] - mse) < 1e-9, k
    full = Qm.evaluate(x, retain=64, with_cf=False)
    assert full["mse"] < 1e-8  # all coefficients kept, no quantisation: exact to fp32 rounding
