"""The colour spec of cost_type 1 (f4): deterministic float transcendentals and the reference's
CIEDE2000 term order (perception_amd/csrc/pcore_colour.h, shared by the GPU kernel and the oracle),
checked against independent numpy / Python float64 evaluations."""
import math

import numpy as np
import pytest

import oracle


def _ulps(a, b):
    a = np.float32(a)
    b = np.float32(b)
    ia = np.array([a]).view(np.int32)[0].astype(np.int64)
    ib = np.array([b]).view(np.int32)[0].astype(np.int64)
    if ia < 0:
        ia = -(ia & 0x7FFFFFFF)
    if ib < 0:
        ib = -(ib & 0x7FFFFFFF)
    return abs(ia - ib)


@pytest.mark.parametrize("fn,ref,lo,hi", [("sin_f", math.sin, -30.0, 30.0), ("cos_f", math.cos, -30.0, 30.0),
                                          ("exp_f", math.exp, -120.0, 5.0)])
def test_transcendentals_within_one_ulp(fn, ref, lo, hi):
    xs = np.concatenate([np.linspace(lo, hi, 20001, dtype=np.float32),
                         np.random.default_rng(1).uniform(lo, hi, 20000).astype(np.float32)])
    worst = 0
    for x in xs:
        worst = max(worst, _ulps(oracle.colour_math(fn, x), np.float32(ref(float(x)))))
    assert worst <= 1


def test_atan2_special_cases_and_accuracy():
    pi32 = np.float32(math.pi)
    assert oracle.colour_math("atan2_f", 0.0, 1.0) == 0.0
    assert oracle.colour_math("atan2_f", 0.0, -1.0) == pi32
    assert oracle.colour_math("atan2_f", -0.0, -1.0) == -pi32
    assert math.copysign(1.0, oracle.colour_math("atan2_f", -0.0, 1.0)) < 0
    assert oracle.colour_math("atan2_f", 0.0, -0.0) == pi32
    assert oracle.colour_math("atan2_f", 1.0, 0.0) == np.float32(math.pi / 2)
    rng = np.random.default_rng(2)
    worst = 0
    for y, x in rng.uniform(-120, 120, (20000, 2)).astype(np.float32):
        worst = max(worst, _ulps(oracle.colour_math("atan2_f", y, x), np.float32(math.atan2(float(y), float(x)))))
    assert worst <= 1


def _rgb2lab_py(c):
    r, g, b = c[2] / 255.0, c[1] / 255.0, c[0] / 255.0
    lin = [((v + 0.055) / 1.055) ** 2.4 * 100.0 if v > 0.04045 else v / 12.92 * 100.0 for v in (r, g, b)]
    r, g, b = lin
    x = (r * 0.4124564 + g * 0.3575761 + b * 0.1804375) / 95.047
    y = (r * 0.2126729 + g * 0.7151522 + b * 0.0721750) / 100.00
    z = (r * 0.0193339 + g * 0.1191920 + b * 0.9503041) / 108.883
    f = [v ** (1.0 / 3.0) if v > 0.008856 else 7.787 * v + 16.0 / 116.0 for v in (x, y, z)]
    return np.array([116.0 * f[1] - 16, 500 * (f[0] - f[1]), 200 * (f[1] - f[2])], np.float32)


def test_rgb2lab_matches_python_double():
    rng = np.random.default_rng(3)
    for c in list(rng.integers(0, 256, (300, 3))) + [[0, 0, 0], [255, 255, 255], [128, 128, 128], [10, 0, 0]]:
        assert np.allclose(oracle.rgb2lab(c), _rgb2lab_py(c), rtol=0, atol=2e-5)


def _ciede_ref_double(l1, a1, b1, l2, a2, b2):
    """compute_costs.cuh:90-158 evaluated in float64 throughout (no float rounding)."""
    pi = math.pi
    c1, c2 = math.hypot(a1, b1), math.hypot(a2, b2)
    mc = (c1 + c2) / 2
    mc7 = mc ** 7
    g = 0.5 * (1 - math.sqrt(mc7 / (mc7 + 6103515625.0)))
    a1p, a2p = a1 * (1 + g), a2 * (1 + g)
    c1, c2 = math.hypot(a1p, b1), math.hypot(a2p, b2)
    h1 = math.fmod(math.atan2(b1, a1p) + 2 * pi, 2 * pi)
    h2 = math.fmod(math.atan2(b2, a2p) + 2 * pi, 2 * pi)
    dL, dC = l2 - l1, c2 - c1
    dh = h2 - h1 if abs(h2 - h1) <= pi else (h2 - h1 - 2 * pi if h2 > h1 else h2 - h1 + 2 * pi)
    dH = 2 * math.sqrt(c1 * c2) * math.sin(dh / 2)
    mL = (l1 + l2) / 2
    mc = (c1 + c2) / 2
    mc7 = mc ** 7
    if abs(h1 - h2) <= pi + 1e-5:
        mH = (h1 + h2) / 2
    elif h1 + h2 < 2 * pi:
        mH = (h1 + h2 + 2 * pi) / 2
    else:
        mH = (h1 + h2 - 2 * pi) / 2
    T = (1 - 0.17 * math.cos(mH - math.radians(30)) + 0.24 * math.cos(2 * mH) + 0.32 * math.cos(3 * mH + math.radians(6))
         - 0.2 * math.cos(4 * mH - math.radians(63)))
    sl = 1 + 0.015 * (mL - 50) ** 2 / math.sqrt(20 + (mL - 50) ** 2)
    sc = 1 + 0.045 * mc
    sh = 1 + 0.015 * mc * T
    rc = 2 * math.sqrt(mc7 / (mc7 + 6103515625.0))
    rt = -math.sin(math.radians(60 * math.exp(-(((math.degrees(mH) - 275) / 25) ** 2)))) * rc
    return math.sqrt((dL / sl) ** 2 + (dC / sc) ** 2 + (dH / sh) ** 2 + rt * dC / sc * dH / sh)


def test_colour_distance_follows_the_reference_formula():
    rng = np.random.default_rng(4)
    cols = rng.integers(0, 256, (400, 2, 3))
    for c1, c2 in cols:
        l1, l2 = oracle.rgb2lab(c1), oracle.rgb2lab(c2)
        d = oracle.colour_distance(l1, l2)
        ref = _ciede_ref_double(*map(float, l1), *map(float, l2))
        assert abs(d - ref) <= 1e-4 * max(1.0, ref), (c1, c2, d, ref)
    same = oracle.rgb2lab([90, 90, 90])
    assert oracle.colour_distance(same, same) == 0.0
