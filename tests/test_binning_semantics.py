"""The groupies pair rule under numba and without it.

The reference's AggregateTrapz._loop (interp.py:156-207) adds ``(a_i + a_{i+1}) / 2`` to a
float32 accumulator.  Compiled by numba, ``a_i + a_{i+1}`` is float32, ``/ 2`` promotes to
float64 and the float64 sum is rounded to float32 on the store.  The golden fixture was made
with numba's ``njit`` as the identity (tests/golden/binharness.py), where numpy 1.26 keeps
everything in float32.  The oracle and the GPU follow the numba form.  These tests show that
the two forms give the same bits for every normal float32 input — so the fixture pins the real
reference — and that only a subnormal pair sum can tell them apart.  The fixture has none.

Argument: ``f32(pair) / 2`` is exact in float32 unless the pair sum is subnormal.  The exact
sum of two float32 values whose exponents differ by at most 29 fits in 53 bits, so the float64
sum is exact and is rounded once, as the float32 addition is.  For a larger exponent
difference the smaller term is below 2^-28 of the larger, and both forms return the larger
term.
"""
import numpy as np

import oracle.frei_oracle as O


def _numba_form(acc, a, b):
    pair = (a + b).astype(np.float32)
    return (acc.astype(np.float64) + pair.astype(np.float64) / 2).astype(np.float32)


def _float32_form(acc, a, b):
    pair = (a + b).astype(np.float32)
    half = (pair / np.float32(2)).astype(np.float32)
    return (acc + half).astype(np.float32)


def _random_f32(rng, n, lo_exp, hi_exp):
    m = rng.uniform(1.0, 2.0, n)
    e = rng.integers(lo_exp, hi_exp, n)
    s = rng.choice([-1.0, 1.0], n)
    return (s * np.ldexp(m, e)).astype(np.float32)


def test_pair_rule_forms_agree_on_normal_float32():
    rng = np.random.default_rng(5)
    n = 2_000_000
    with np.errstate(over="ignore"):
        for lo, hi in ((-120, 120), (-40, 10), (-5, 5)):
            acc = _random_f32(rng, n, lo, hi)
            a = _random_f32(rng, n, lo, hi)
            b = np.where(rng.random(n) < 0.5, a, _random_f32(rng, n, lo, hi)).astype(np.float32)
            x, y = _numba_form(acc, a, b), _float32_form(acc, a, b)
            fin = np.isfinite(x) & np.isfinite(y)
            pair = (a + b).astype(np.float32)
            normal = np.abs(pair) >= np.finfo(np.float32).tiny
            assert np.array_equal(x[fin & normal], y[fin & normal])
            assert np.array_equal(np.isfinite(x), np.isfinite(y))


def test_pair_rule_forms_differ_only_for_subnormal_pairs():
    # a subnormal pair sum loses its last bit when halved in float32 but not in float64
    tiny = np.float32(np.finfo(np.float32).smallest_subnormal)       # 2^-149
    acc = np.array([tiny], dtype=np.float32)
    a = np.array([tiny], dtype=np.float32)
    b = np.array([np.float32(0.0)], dtype=np.float32)
    x, y = _numba_form(acc, a, b), _float32_form(acc, a, b)
    # float32: 2^-150 rounds to 0, acc stays 2^-149; float64: 1.5 * 2^-149 ties to 2^-148
    assert x[0] == 2 * tiny and y[0] == tiny


def test_golden_cross_section_pins_the_numba_form(golden):
    """The fixture's input has no subnormal (or zero-crossing) pair sums, so the harness's
    float32 arithmetic and numba's float64 promotion give identical binned tables: the golden
    groupies output pins the reference as numba runs it."""
    B = golden("binning.npz")
    x = np.asarray(B["xsec"], dtype=np.float32)
    pair = x[..., 1:] + x[..., :-1]
    assert np.all((pair == 0) | (np.abs(pair) >= np.finfo(np.float32).tiny))
    for case in ("g1", "g2"):
        start, end = O.bin_ranges(B["xsec_wl"], B[f"{case}_wl_bins"])
        rows = x.reshape(-1, x.shape[-1])
        n = end - start
        acc32 = np.zeros((rows.shape[0], start.size), dtype=np.float32)
        for j in range(int(n.max()) - 1):
            m = j + 1 < n
            i = start[m] + j
            acc32[:, m] = _float32_form(acc32[:, m], rows[:, i], rows[:, i + 1])
        ref = acc32.astype(np.float64) * (B[f"{case}_wl_bins"][1:] - B[f"{case}_wl_bins"][:-1]) * 1e-3
        out = O.bin_groupies_rows(rows, start, end, B[f"{case}_wl_bins"])
        assert np.array_equal(out, ref)
