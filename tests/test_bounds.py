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


def test_pair_products_are_generated_from_the_singles():
    """fe_mul2 / fe_sq2 (the interleaved pair products) are generated from fe_mul_ps / fe_sq_ps by
    tools/gen_fe_pair.py, so the bounds checked above cover them only while the header holds exactly
    what the generator makes of the current single products."""
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_fe_pair.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


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


def test_lazy_horner_bounds():
    """The share evaluation's lazy reduction (sc25519.h sc_lazy_step / sc_lazy_fold, k_share_eval
    for x < 2^13), restated limb by limb: at the worst case -- accumulator just below 2^254,
    coefficients l - 1, x = 8191, SC_LAZY_STEPS = 5 steps between folds -- no 64-bit limb sum or
    10-limb accumulator overflows, the fold never goes negative and lands below 2^254 again, and
    the value stays congruent to the Horner value mod l."""
    L = 2**252 + 27742317777372353535851937790883648493
    D = L - 2**252
    limbs = lambda v, k: [(v >> (32 * i)) & 0xffffffff for i in range(k)]  # noqa: E731
    val = lambda l: sum(x << (32 * i) for i, x in enumerate(l))  # noqa: E731

    def step(v, x, c):
        t, out, cl = 0, [], limbs(c, 8)
        for i in range(10):
            t = v[i] * x + (cl[i] if i < 8 else 0) + (t >> 32)
            assert t < 2**64
            out.append(t & 0xffffffff)
        assert t >> 32 == 0, "10-limb accumulator overflow"
        return out

    def fold(v):
        h = [(v[7] >> 28) | ((v[8] << 4) & 0xffffffff), (v[8] >> 28) | ((v[9] << 4) & 0xffffffff), v[9] >> 28]
        dl, p, acc, hiacc = limbs(D, 4), [], 0, 0
        for k in range(7):
            for i in range(3):
                if 0 <= k - i < 4:
                    m = h[i] * dl[k - i]
                    acc += m & 0xffffffff
                    hiacc += m >> 32
            assert acc < 2**64
            p.append(acc & 0xffffffff)
            acc, hiacc = (acc >> 32) + hiacc, 0
        Ll, c, out = limbs(L, 8), 0, []
        for i in range(8):
            c += (v[i] if i < 7 else v[7] & 0x0fffffff) + Ll[i] - (p[i] if i < 7 else 0)
            out.append(c & 0xffffffff)
            c >>= 32
        assert c == 0, "fold went negative or past 2^256"
        return out + [0, 0]

    x = 8191
    for start in (2**254 - 1, L - 1, 0):
        v, want = limbs(start, 10), start
        for _ in range(5):
            v = step(v, x, L - 1)
            want = want * x + L - 1
        v = fold(v)
        assert val(v) < 2**254 and val(v) % L == want % L
