"""The limb-bound contract of the field arithmetic (dkg_amd/csrc/fe25519.h, ge25519.h), checked by
tools/fe_bounds.py on worst-case bounds -- a property random tests cannot establish -- and a
check that the checker itself detects overflows (it is not vacuous)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import fe_bounds as F  # noqa: E402


def test_terms_follow_the_header():
    """fe_mul has 10 x 10 products, fe_sq the 55 distinct ones, read from fe25519.h, in both
    flavours, and the two flavours sum the same products into each column."""
    import random

    for fl in ("ps", "cs"):
        assert sum(len(v) for v in F._parse_terms(f"fe_mul_{fl}").values()) == 100
        assert sum(len(v) for v in F._parse_terms(f"fe_sq_{fl}").values()) == 55
    rng = random.Random(5)
    for _ in range(50):
        f = [rng.getrandbits(26) for _ in range(10)]
        g = [rng.getrandbits(26) for _ in range(10)]
        assert F._columns("fe_mul_ps", f, g, "x") == F._columns("fe_mul_cs", f, g, "x")
        assert F._columns("fe_sq_ps", f, f, "x") == F._columns("fe_sq_cs", f, f, "x")


def test_no_overflow_anywhere():
    tight = F.run()
    assert F.violations == [], F.violations
    # the stated TIGHT bound of fe25519.h
    assert all(x < (1 << 26) + (1 << 6) for x in tight[0::2])
    assert all(x < (1 << 25) + (1 << 12) for x in tight[1::2])
    assert F.main() == 0


def test_checker_detects_violations():
    F.violations.clear()
    F.fe_mul([1 << 29] * 10, [1 << 27] * 10, "probe")        # 19 * 2^27 fits, the columns do not
    assert any("probe column" in v for v in F.violations)
    F.violations.clear()
    F.fe_mul([1 << 26] * 10, [1 << 28] * 10, "probe")        # 19 * 2^28 > 2^32
    assert any("pre-multiply x19" in v for v in F.violations)
    F.violations.clear()
    F.fe_sub([0] * 10, [1 << 27] * 10, "probe")              # subtrahend above 2p: would wrap
    assert any("subtrahend" in v for v in F.violations)
    F.violations.clear()
    F.fe_mul([int(2 ** 28.0)] * 10, [int(2 ** 27.75)] * 10, "probe")  # the stated admissible corner
    F.fe_mul([int(2 ** 28.32)] * 10, [int(2 ** 27.585)] * 10, "probe")
    F.fe_mul([1 << 29] * 10, [1 << 26] * 10, "probe")
    assert F.violations == []


def test_dedicated_addition_is_exact_or_flags():
    """The stepping's dedicated addition (points.h ge_add_ded_lds) returns p + q or a point with
    Z = 0, never a wrong point, over random pairs and every pair of 8-torsion offsets with equal,
    opposite, doubled and random prime-order parts (tools/ded_check.py); random pairs never flag."""
    import ded_check

    stats, random_flags = ded_check.run(seed=2, nrand=32)
    assert stats["wrong"] == 0 and random_flags == 0
    assert stats["Z=0"] > 0  # the exceptional cases exist and are caught


def test_tight_zero_representations():
    """fe_tight_zero's rule on fe_mul / fe_sq outputs: with limbs bounded as tools/fe_bounds.py
    derives (limbs 1 and 5 below 2 * 2^25 - 1, the rest in their widths), 0 and p have one
    representation each (all zero / p's canonical limbs)."""
    W = F.W
    p_limbs = [(2**255 - 19 >> sum(W[:i])) & ((1 << W[i]) - 1) for i in range(10)]
    assert p_limbs == [0x3ffffed] + [(1 << W[i]) - 1 for i in range(1, 10)]
    # a representation of p (or 0) other than the canonical one needs some limb to hold at least
    # one extra unit of its width: limb i >= 2^W[i] + canonical -- beyond every derived bound
    z = F.fe_mul([F.MASK[i] for i in range(10)], [F.MASK[i] for i in range(10)], "x")
    for i in range(10):
        assert z[i] < (1 << W[i]) + p_limbs[i] if i in (1, 5) else z[i] <= F.MASK[i]
