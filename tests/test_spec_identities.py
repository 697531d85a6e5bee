"""Exact identities the kernel arithmetic (gqmap_math.h) relies on when it
replaces a reference expression by a cheaper one with the same values."""
import math
from fractions import Fraction

import numpy as np


def _matlab_round_ge1(y: float) -> float:
    """max(round(y), 1) with MATLAB's round (half away from zero), in exact
    rational arithmetic; NaN -> 1 (MATLAB's max ignores NaN)."""
    if math.isnan(y):
        return 1.0
    r = math.floor(abs(Fraction(y)) + Fraction(1, 2))
    return max(float(r if y >= 0 else -r), 1.0)


def _kernel_round_ge1(y: float) -> float:
    """gqmap_math.h round_ge1: trunc(max(y, 1/2) + 1/2) in IEEE doubles
    (Python floats are IEEE doubles; fmax ignores NaN)."""
    yy = 0.5 if (math.isnan(y) or y < 0.5) else y
    return float(math.trunc(yy + 0.5))


def test_round_ge1_identity():
    # sample_ctf4 (legacy/gqmap_ctf.m:96): positions rounded to the 1/64 grid
    rng = np.random.default_rng(0)
    ys = list(rng.uniform(-200.0, 64 * 2600.0, 50000))
    # neighbours of half-integers and of the binade edges, where y + 1/2 rounds
    for k in range(-2, 40):
        for base in (2.0 ** k - 0.5, 2.0 ** k - 1.5, 2.0 ** k + 0.5):
            v_up = v_dn = base
            for _ in range(4):
                v_up = float(np.nextafter(v_up, np.inf))
                v_dn = float(np.nextafter(v_dn, -np.inf))
                ys += [v_up, v_dn]
            ys.append(base)
    ys += [n + 0.5 for n in range(-5, 200)] + [0.49999999999999994, 0.5, -0.5, float("nan"), -1e300]
    bad = [y for y in ys if _matlab_round_ge1(y) != _kernel_round_ge1(y)]
    assert not bad, bad[:5]


def test_fract_identity():
    # axis_cell_abs without clamps: X - (double)(int)X == X - floor(X) for X >= 1
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(1.0, 3000.0, 100000), np.arange(1.0, 100.0),
                         np.nextafter(np.arange(2.0, 100.0), 0.0)])
    for x in xs:
        assert x - float(int(x)) == x - math.floor(x)


def test_last_cell_identity():
    # axis_cell_abs / axis_cell without the cap: a sample clamped to the last
    # column / row (X == No, Y == Mo) interpolates cell n at fraction 0 instead
    # of the reference's cell n-1 at fraction 1 -- the same value (up to the
    # sign of a zero), fp64 and fp32, with zero, negative and fractional taps
    import oracle.oracle as O
    rng = np.random.default_rng(2)
    for Mo, No in ((7, 9), (16, 20), (5, 5)):
        for kind in ("int", "frac", "zeros"):
            if kind == "int":
                I2 = rng.integers(0, 256, (Mo, No)).astype(np.float64)
            elif kind == "frac":
                I2 = rng.normal(0.0, 50.0, (Mo, No))
            else:
                I2 = np.zeros((Mo, No))
                I2[rng.integers(0, Mo, 4), rng.integers(0, No, 4)] = -3.0
            VV = O.get_vv(np.asfortranarray(I2))
            n = 4000
            X = rng.uniform(-5.0, No + 5.0, n)
            Y = rng.uniform(-5.0, Mo + 5.0, n)
            sel = rng.integers(0, 4, n)
            X[sel == 1] = No
            Y[sel == 2] = Mo
            X[sel == 3], Y[sel == 3] = No, Mo
            X[:8] = [No, No + 1e-9, No - 1e-12, 1.0, No, 0.5, No, No]
            Y[:8] = [Mo, 2.5, Mo, Mo, 1.0, Mo, Mo - 0.5, Mo + 3.0]
            for fp32 in (False, True):
                if fp32 and kind == "frac":
                    continue  # fp32 frames hold exact (integer) values
                a = O.emu_sample(VV, Mo, No, X, Y, fp32=fp32, cap=False)
                b = O.emu_sample(VV, Mo, No, X, Y, fp32=fp32, cap=True)
                assert np.all(np.isfinite(a))
                np.testing.assert_array_equal(a, b)


def _fma(a: float, b: float, c: float) -> float:
    """IEEE fused multiply-add: the exact a*b + c rounded once (float() of a
    Fraction is correctly rounded)."""
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def test_div_rcp_is_correctly_rounded():
    # gqmap_math.h div_rcp (literal mode, device): with r = RN(1/y),
    # q = RN(x r), q = RN(q + RN(x - q y) r) twice, equals RN(x/y) -- here for
    # the literal engine's operands: x = XI^2 - XJ^2 of Gauss-Hermite nodes
    # (|x| < 64), y = sqrtpr = sqrt(1 - p^2) with |p| <= corr_tor < 1.
    rng = np.random.default_rng(5)
    xs = list(rng.uniform(-60.0, 60.0, 3000)) + list(rng.uniform(-1e-3, 1e-3, 500)) + [0.0, 1.0, -1.0, 59.999]
    ys = list(np.sqrt(1 - rng.uniform(-0.999, 0.999, 3000) ** 2)) + [1.0, 0.5, math.sqrt(1 - 0.999 ** 2)]
    bad = 0
    for i, x in enumerate(xs):
        y = float(ys[i % len(ys)])
        r = 1.0 / y
        q = x * r
        q = _fma(_fma(-q, y, x), r, q)
        q = _fma(_fma(-q, y, x), r, q)
        bad += q != x / y
    assert bad == 0


def test_legacy_df2_sums_are_exact_negations():
    # gqmap_legacy.hip k_legacy_grad: the reference's c2 += df2 (df2 = -df1)
    # chain, from +0, equals 0 - (the c1 += df1 chain) bit for bit -- zero
    # terms of either sign and exact cancellations included -- so s2 = 0 - s1
    # (legacy/gqmap_cpu.m:40-53).
    rng = np.random.default_rng(9)
    for trial in range(400):
        n = int(rng.integers(1, 40))
        df1 = list(rng.normal(0, 10.0 ** rng.integers(-8, 3), n))
        for j in range(n):  # zeros of both signs and exact cancellations
            u = rng.random()
            if u < 0.15:
                df1[j] = 0.0
            elif u < 0.3:
                df1[j] = -0.0
            elif u < 0.4 and j > 0:
                df1[j] = -df1[j - 1]
        c1 = 0.0
        c2 = 0.0
        for d in df1:
            c1 += d
            c2 += -d
        assert math.copysign(1.0, c2) == math.copysign(1.0, 0.0 - c1) and c2 == 0.0 - c1, (trial, df1)
