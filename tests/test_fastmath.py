"""The fast factor math of csrc/common.h (ftanh_pos, fatanh_pos), restated in float32 numpy with
correctly rounded exp2 / log2 / reciprocal (the device's v_exp / v_log / v_rcp are within 1 ulp
of those), against float64 over the inputs the row maps give them: the polynomial branches and
the switch point 0.25 keep the error under 6 ulp.  The device functions themselves are pinned
by tests/test_gpu_parity.py::test_row_maps_fast_factor_math."""
import numpy as np

F = np.float32
LOG2E, LN2 = F(1.4426950408889634), F(0.6931471805599453)


def ftanh_pos(x):
    x = x.astype(F)
    x2 = x * x
    p = F(62 / 2835) * x2 + F(-17 / 315)
    p = p * x2 + F(2 / 15)
    p = p * x2 + F(-1 / 3)
    p = (x * x2) * p + x
    e = np.exp2(x * (F(-2) * LOG2E)).astype(F)
    q = (F(1) - e) * (F(1) / (F(1) + e))
    return np.where(x < F(0.25), p, q).astype(F)


def fatanh_pos(s):
    s = s.astype(F)
    s2 = s * s
    p = F(1 / 11) * s2 + F(1 / 9)
    for c in (1 / 7, 1 / 5, 1 / 3):
        p = p * s2 + F(c)
    p = (s * s2) * p + s
    q = (F(0.5) * LN2) * np.log2((F(1) + s) * (F(1) / (F(1) - s))).astype(F)
    return np.where(s < F(0.25), p, q).astype(F)


def _rel(got, ref):
    return np.abs(got.astype(np.float64) - ref) / np.maximum(np.abs(ref), 1e-30)


def test_ftanh_pos_within_6_ulp():
    x = np.concatenate([np.logspace(-8, 1.5, 100000), np.linspace(0, 4, 100001)]).astype(F)
    assert _rel(ftanh_pos(x), np.tanh(x.astype(np.float64))).max() < 6 * 2.0 ** -23


def test_fatanh_pos_within_6_ulp():
    s = np.concatenate([np.logspace(-8, -1e-7, 100000), np.linspace(0, 1 - 1e-6, 100001)]).astype(F)
    s = np.minimum(s, F(1 - 1e-6))  # log0's clamp (hyperbolic_ops.py:115)
    assert _rel(fatanh_pos(s), np.arctanh(s.astype(np.float64))).max() < 6 * 2.0 ** -23
