#!/usr/bin/env python3
"""Worst-case limb-bound checker for the GF(2^255-19) arithmetic of dkg_amd/csrc/fe25519.h and the
group formulas of dkg_amd/csrc/ge25519.h / points.h, as written.

Every field element is abstracted by ten upper bounds (one per 32-bit limb; lower bound 0 -- every
operation is unsigned).  The primitives are restated limb for limb from fe25519.h, and fe_mul /
fe_sq take their product terms (which limb pairs, which operand carries the x19 fold and the x2 / x4
weights) straight from the header text, so the checker cannot drift from the code.  It asserts:
  * every 32-bit limb result (fe_add, fe_sub, fe_neg, fe_carry, the x19 / x2 / x4 pre-multiplies
    of fe_mul / fe_sq) stays below 2^32, and fe_sub / fe_neg never wrap (subtrahend <= 2p limbwise);
  * every 64-bit column sum of fe_mul / fe_sq in both flavours (product scanning: on top of the
    carry out of the previous column, and the x19 fold of the top carry; column sums: every
    intermediate of the carry pass fe_carry64) stays below 2^64, every 32-bit value below 2^32;
  * fe_tobytes32's canonical reduction sees a value below 2p (one conditional subtraction suffices).
The group formulas (ge_to_cached, ge_add, ge_sub, ge_madd, ge_msub, ge_dbl / _rt / _lean,
ge_add_signed, ge_add_lds incl. its negated path, ge_madd_signed / ge_madd_lds and the affine
addends of k_affine_pieces, the stepping's dedicated ge_add_ded_lds (and fe_tight_zero's operand), the comb entry selection of combw_mul_add,
ristretto_eq, decode / encode) are run on the bounds; point coordinates are iterated to a fixpoint
(every stored coordinate is again an input), so the invariant "a coordinate is TIGHT" is closed.

Run:  python tools/fe_bounds.py      (prints the derived bounds; exit status 1 on any violation)
tests/test_bounds.py runs it on the CPU.
"""
import math
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FE_H = os.path.join(ROOT, "dkg_amd", "csrc", "fe25519.h")
GE_H = os.path.join(ROOT, "dkg_amd", "csrc", "ge25519.h")

W = [26 if i % 2 == 0 else 25 for i in range(10)]           # limb widths (radix 2^25.5)
OFF = [sum(W[:i]) for i in range(10)]                        # bit offsets 0, 26, 51, ...
MASK = [(1 << w) - 1 for w in W]
P2 = [0x7ffffda] + [0x3fffffe if i % 2 else 0x7fffffe for i in range(1, 10)]  # fe_const::P2_*
U32, U64 = 1 << 32, 1 << 64
P = 2**255 - 19

violations = []
worst = {}  # check name -> (max value seen, limit)


def check(name, value, limit):
    """Record value < limit (a bound that must hold)."""
    w = worst.get(name)
    if w is None or value > w[0]:
        worst[name] = (value, limit)
    if value >= limit:
        violations.append(f"{name}: {value} (2^{math.log2(value):.3f}) >= 2^{math.log2(limit):.0f}")


def vmax(*fes):
    return [max(f[i] for f in fes) for i in range(10)]


def log2s(f):
    return "[" + ", ".join(f"{math.log2(x):.2f}" if x else "0" for x in f) + "]"


# ---------------- fe25519.h primitives ----------------
def fe_add(a, b, where="fe_add"):
    r = [a[i] + b[i] for i in range(10)]
    for i in range(10):
        check(f"{where} limb", r[i], U32)
    return r


def fe_sub(a, b, where="fe_sub"):
    """r = a + 2p - b: b must not exceed 2p limbwise (no wrap), and a + 2p must fit."""
    for i in range(10):
        check(f"{where} subtrahend <= 2p limb", b[i], P2[i] + 1)
    r = [a[i] + P2[i] for i in range(10)]
    for i in range(10):
        check(f"{where} limb", r[i], U32)
    return r


def fe_neg(a, where="fe_neg"):
    for i in range(10):
        check(f"{where} operand <= 2p limb", a[i], P2[i] + 1)
    return list(P2)


def fe_carry(a, where="fe_carry"):
    c = [a[i] >> W[i] for i in range(10)]
    r = [0] * 10
    check(f"{where} 19*c9", 19 * c[9], U32)
    r[0] = min(a[0], MASK[0]) + 19 * c[9]
    for i in range(1, 10):
        r[i] = min(a[i], MASK[i]) + c[i - 1]
    for i in range(10):
        check(f"{where} limb", r[i], U32)
    return r


def fe_scan(cols, where):
    """The product-scanning reduction of fe25519.h (FE_LIMB / FE_FOLD): column k is accumulated on
    top of the carry out of column k-1 (one 64-bit register, v_mad_u64_u32 chains), limb k is its
    low W[k] bits; the carry out of limb 9 is folded x19 into limb 0 and that carry into limb 1."""
    r, h = [0] * 10, 0
    for k in range(10):
        h += cols[k]
        check(f"{where} column + carry", h, U64)
        r[k] = min(h, MASK[k])
        h >>= W[k]
    check(f"{where} 19 * (carry >> 32) (32-bit product)", 19 * (h >> 32), U32)
    t = r[0] + 19 * h
    check(f"{where} fold", t, U64)
    r[0] = min(t, MASK[0])
    r[1] += t >> W[0]
    check(f"{where} limb 1 after fold", r[1], U32)
    return r


def fe_carry64(h, where):
    """fe_carry64 of fe25519.h (the column-sum flavour's carry pass), statement by statement."""
    h = list(h)
    for x in h:
        check(f"{where} column", x, U64)

    def step(i, j, fold=1):
        c = h[i] >> W[i]
        h[j] += c * fold
        check(f"{where} carry into h{j}", h[j], U64)
        h[i] = min(h[i], MASK[i])

    for i, j in [(0, 1), (4, 5), (1, 2), (5, 6), (2, 3), (6, 7), (3, 4), (7, 8), (4, 5), (8, 9)]:
        step(i, j)
    step(9, 0, 19)
    step(0, 1)
    for i in range(10):
        check(f"{where} carried limb fits u32", h[i], U32)
    return h


_MUL_TERMS = {}


def _body(func, end):
    src = open(FE_H).read()
    body = src[src.index(f"DKG_DEV void {func}("):]
    return body[:body.index(end)]


def _parse_terms(func):
    """Column k of `func` in fe25519.h as a list of (operand, operand) names: for the
    product-scanning flavour (fe_mul_ps / fe_sq_ps / fe_mul_small_ps) the mad_first / mad_acc calls
    before FE_LIMB(r, k, h); for the column-sum flavour (fe_mul_cs / fe_sq_cs) the mul32 terms of
    `uint64_t hk = ...`."""
    if func in _MUL_TERMS:
        return _MUL_TERMS[func]
    cols = {}
    if func.endswith("_cs"):
        for m in re.finditer(r"uint64_t h(\d) = (.*?);", _body(func, "fe_carry64("), re.S):
            cols[int(m.group(1))] = re.findall(r"mul32\((\w+), (\w+)\)", m.group(2))
    else:
        body, last = _body(func, "FE_FOLD("), 0
        for m in re.finditer(r"FE_LIMB\(r, (\d), h\)", body):
            cols[int(m.group(1))] = re.findall(r"mad_(?:first\(|acc\(h, )([\w.\[\]]+), ([\w.\[\]]+)\)",
                                               body[last:m.start()])
            last = m.end()
    assert sorted(cols) == list(range(10)), f"{func}: could not parse the ten columns"
    _MUL_TERMS[func] = cols
    return cols


def _operand(name, f, g, where):
    """Bound of an operand name of fe_mul / fe_sq: f3, g7, f1_2, g9_19, f5_4, ... (the pre-multiply
    is a 32-bit product in the code: checked)."""
    m = re.fullmatch(r"([fg])(\d)(?:_(\d+))?", name)
    assert m, name
    base = (f if m.group(1) == "f" else g)[int(m.group(2))]
    k = int(m.group(3) or 1)
    if k != 1:
        check(f"{where} pre-multiply x{k}", base * k, U32)
    return base * k


def _columns(func, f, g, where):
    cols = _parse_terms(func)
    return [sum(_operand(x, f, g, where) * _operand(y, f, g, where) for x, y in cols[k]) for k in range(10)]


def fe_mul(f, g, where="fe_mul"):
    """Both flavours of fe25519.h (dkgk: product scanning, dkgk_ilp: column sums) on the same
    inputs; the result bound is the larger of the two."""
    return vmax(fe_scan(_columns("fe_mul_ps", f, g, where), where),
                fe_carry64(_columns("fe_mul_cs", f, g, where), where))


def fe_sq(f, where="fe_sq"):
    return vmax(fe_scan(_columns("fe_sq_ps", f, f, where), where),
                fe_carry64(_columns("fe_sq_cs", f, f, where), where))


def fe_mul_small(a, k, where="fe_mul_small"):
    cols = _parse_terms("fe_mul_small_ps")
    assert all(c == [(f"a.v[{i}]", "k")] for i, c in cols.items()), "fe_mul_small: unexpected terms"
    return vmax(fe_scan([a[i] * k for i in range(10)], where), fe_carry64([a[i] * k for i in range(10)], where))


def fe_tobytes32(a, where="fe_tobytes32"):
    t = fe_carry(fe_carry(a, where), where)
    value = sum(t[i] << OFF[i] for i in range(10))
    check(f"{where} value below 2p (one conditional subtraction)", value, 2 * P)
    return t


def const(limbs):
    return list(limbs)


def fe_const_from_header(name):
    src = open(GE_H).read()
    m = re.search(name + r"\[10\] = \{(.*?)\};", src, re.S)
    return [int(x, 16) for x in re.findall(r"0x[0-9a-f]+", m.group(1))]


ONE = [1] + [0] * 9
ZERO = [0] * 10


# ---------------- ge25519.h formulas (as written) ----------------
def ge_to_cached(p):
    X, Y, Z, T = p
    ypx = fe_add(Y, X, "to_cached Y+X")               # left uncarried (fe_mul's g operand only)
    ymx = fe_sub(Y, X, "to_cached Y-X")
    z2 = fe_add(Z, Z, "to_cached 2Z")
    t2d = fe_mul(T, D2, "to_cached T*2d")
    return (ypx, ymx, z2, t2d)


def ge_cached_neg(c):
    return (c[1], c[0], c[2], fe_carry(fe_neg(c[3], "cached_neg"), "cached_neg"))


def ge_add(p, q, where="ge_add", swap=False):
    """ge_add (ge_sub: swap selects Y-X <-> Y+X and the sign of c, same bounds up to order)."""
    X, Y, Z, T = p
    YpX, YmX, Z2, T2d = q
    qa, qb = (YpX, YmX) if swap else (YmX, YpX)
    t = fe_sub(Y, X, where)
    a = fe_mul(t, qa, where)
    t = fe_add(Y, X, where)
    b = fe_mul(t, qb, where)
    e = fe_sub(b, a, where)
    h = fe_add(b, a, where)
    a = fe_mul(T, T2d, where)                       # c
    b = fe_mul(Z, Z2, where)                        # d
    if swap:
        t = fe_add(b, a, where)                     # f = d + c
        b = fe_sub(b, a, where)                     # g = d - c
    else:
        t = fe_sub(b, a, where)                     # f = d - c
        b = fe_add(b, a, where)                     # g = d + c
    return (fe_mul(e, t, where), fe_mul(b, h, where), fe_mul(t, b, where), fe_mul(e, h, where))


def ge_madd(p, q, where="ge_madd", minus=False):
    X, Y, Z, T = p
    ypx, ymx, xy2d = q
    t = fe_sub(Y, X, where)
    a = fe_mul(t, ypx if minus else ymx, where)
    t = fe_add(Y, X, where)
    b = fe_mul(t, ymx if minus else ypx, where)
    e = fe_sub(b, a, where)
    h = fe_add(b, a, where)
    a = fe_mul(T, xy2d, where)
    b = fe_add(Z, Z, where)
    if minus:
        t = fe_add(b, a, where)
        b = fe_sub(b, a, where)
        return (fe_mul(t, e, where), fe_mul(b, h, where), fe_mul(b, t, where), fe_mul(e, h, where))
    t = fe_sub(b, a, where)
    b = fe_add(b, a, where)
    return (fe_mul(t, e, where), fe_mul(b, h, where), fe_mul(t, b, where), fe_mul(e, h, where))


def ge_dbl(p, where="ge_dbl"):
    """ge_dbl<with_t> and ge_dbl_rt (same statements)."""
    X, Y, Z, T = p
    a, b, c = fe_sq(X, where), fe_sq(Y, where), fe_sq(Z, where)
    c = fe_add(c, c, where)
    t = fe_sq(fe_add(X, Y, where), where)
    h = fe_add(a, b, where)
    e = fe_sub(h, t, where)
    g = fe_sub(a, b, where)
    f = fe_carry(fe_add(c, g, where), where)
    return (fe_mul(e, f, where), fe_mul(g, h, where), fe_mul(f, g, where), fe_mul(e, h, where))


def ge_dbl_lean(p, where="ge_dbl_lean"):
    X, Y, Z, T = p
    a, b = fe_sq(X, where), fe_sq(Y, where)
    h = fe_add(a, b, where)
    g = fe_sub(a, b, where)
    t = fe_sq(Z, where)
    t = fe_add(t, t, where)
    t = fe_carry(fe_add(t, g, where), where)
    a = fe_sq(fe_add(X, Y, where), where)
    b = fe_sub(h, a, where)
    return (fe_mul(b, t, where), fe_mul(g, h, where), fe_mul(t, g, where), fe_mul(b, h, where))


def ge_add_signed(p, q, where="ge_add_signed"):
    """Both signs: qa / qb are selected from (Y+X, Y-X), and a = +-c is carried before fe_sub."""
    X, Y, Z, T = p
    YpX, YmX, Z2, T2d = q
    qa = qb = vmax(YpX, YmX)
    t = fe_sub(Y, X, where)
    a = fe_mul(t, qa, where)
    t = fe_add(Y, X, where)
    b = fe_mul(t, qb, where)
    e = fe_sub(b, a, where)
    h = fe_add(b, a, where)
    a = fe_mul(T, T2d, where)
    b = fe_mul(Z, Z2, where)
    na = fe_neg(a, where)
    a = vmax(a, na)                                 # fe_cmov (no carry: 2p - c <= 2p)
    t = fe_sub(b, a, where)
    b = fe_add(b, a, where)
    return (fe_mul(e, t, where), fe_mul(b, h, where), fe_mul(t, b, where), fe_mul(e, h, where))


def ge_add_lds(p, q, where="ge_add_lds"):
    """points.h ge_add_lds, both signs: neg swaps the two reads and negates c (fe_neg + fe_carry)."""
    X, Y, Z, T = p
    YpX, YmX, Z2, T2d = q
    sel = vmax(YpX, YmX)
    t = fe_sub(Y, X, where)
    a = fe_mul(t, sel, where)
    t = fe_add(Y, X, where)
    b = fe_mul(t, sel, where)
    e = fe_sub(b, a, where)
    h = fe_add(b, a, where)
    a = fe_mul(T, T2d, where)
    a = vmax(a, fe_neg(a, where))                   # if (neg) fe_neg (no carry)
    b = fe_mul(Z, Z2, where)
    t = fe_sub(b, a, where)
    b = fe_add(b, a, where)
    return (fe_mul(e, t, where), fe_mul(b, h, where), fe_mul(t, b, where), fe_mul(e, h, where))


def ge_madd_signed(p, q, where="ge_madd_signed"):
    """ge25519.h ge_madd_signed and points.h ge_madd_lds, both signs: the two reads selected from
    (y+x, y-x), a = +-c (fe_neg, no carry), d = 2Z carried."""
    X, Y, Z, T = p
    ypx, ymx, xy2d = q
    sel = vmax(ypx, ymx)
    t = fe_sub(Y, X, where)
    a = fe_mul(t, sel, where)
    t = fe_add(Y, X, where)
    b = fe_mul(t, sel, where)
    e = fe_sub(b, a, where)
    h = fe_add(b, a, where)
    a = fe_mul(T, xy2d, where)
    a = vmax(a, fe_neg(a, where))
    b = fe_carry(fe_add(Z, Z, where), where)
    t = fe_sub(b, a, where)
    b = fe_add(b, a, where)
    return (fe_mul(e, t, where), fe_mul(b, h, where), fe_mul(t, b, where), fe_mul(e, h, where))


def affine_addend(p, where="affine_pieces"):
    """kernels.hip k_affine_pieces: zi = inv * prefix (products of Z), x = X zi, y = Y zi,
    2dxy = (T zi) 2d; y+x and y-x left uncarried like the cached form."""
    X, Y, Z, T = p
    zi = fe_mul(fe_mul(Z, Z, where), Z, where)
    x, y = fe_mul(X, zi, where), fe_mul(Y, zi, where)
    return (fe_add(y, x, where), fe_sub(y, x, where), fe_mul(fe_mul(T, zi, where), D2, where))


def ge_to_cached_ded(p):
    X, Y, Z, T = p
    return (fe_add(Y, X, "to_cached_ded"), fe_sub(Y, X, "to_cached_ded"), fe_add(Z, Z, "to_cached_ded"),
            fe_add(T, T, "to_cached_ded 2T"))


def tight_zero_ok(z, where):
    """fe25519.h fe_tight_zero: limbs within their widths except 1 and 5, which stay below
    2 * 2^25 - 1 (so 0 and p each have one representation)."""
    for i in range(10):
        lim = (2 * (MASK[i] + 1) - 1) if i in (1, 5) else MASK[i] + 1
        check(f"{where} fe_tight_zero operand limb {i}", z[i], lim)


def ge_add_ded(p, q, where="ge_add_ded_lds"):
    """points.h ge_add_ded_lds (dedicated addition, q = ge_to_cached_ded): X3 = E F, Y3 = G H,
    T3 = E H, Z3 = G F with F, H the second operands; Z3 feeds fe_tight_zero."""
    X, Y, Z, T = p
    YpX, YmX, Z2, T2 = q
    t = fe_sub(Y, X, where)
    a = fe_mul(t, YpX, where)
    t = fe_add(Y, X, where)
    b = fe_mul(t, YmX, where)
    f = fe_sub(b, a, where)
    g = fe_add(b, a, where)
    c = fe_mul(Z, T2, where)
    d = fe_mul(T, Z2, where)
    e = fe_add(d, c, where)
    h = fe_sub(d, c, where)
    z3 = fe_mul(g, f, where)
    tight_zero_ok(z3, where)
    return (fe_mul(e, f, where), fe_mul(g, h, where), z3, fe_mul(e, h, where))


def comb8_entry(tab_ypx, tab_ymx, tab_xy2d):
    """points.h combw_mul_add: the selected affine entry, incl. identity (1, 1, 0) and -Q =
    (y-x, y+x, 2p - xy2d) -- the negated xy2d is NOT carried."""
    sel = vmax(tab_ypx, tab_ymx, ONE)
    for i in range(10):
        check("comb8 2p - xy2d operand", tab_xy2d[i], P2[i] + 1)
    return (sel, sel, vmax(tab_xy2d, P2))


def fe_abs(a, where):
    n = fe_carry(fe_neg(a, where), where)
    fe_tobytes32(a, where)                          # fe_isneg
    return vmax(a, n)


def fe_pow_chain(z, where):
    """fe_pow22523 / fe_invert: squarings and products of tight values only."""
    t = fe_sq(z, where)
    return fe_mul(t, z, where)


def sqrt_ratio_m1(u, v, where="sqrt_ratio"):
    v3 = fe_mul(fe_sq(v, where), v, where)
    v7 = fe_mul(fe_sq(v3, where), v, where)
    t = fe_pow_chain(fe_mul(u, v7, where), where)
    t = fe_mul(t, v3, where)
    r = fe_mul(t, u, where)
    chk = fe_mul(fe_sq(r, where), v, where)
    neg_u = fe_carry(fe_neg(u, where), where)
    neg_u_i = fe_mul(neg_u, SQRT_M1, where)
    for x in (u, neg_u, neg_u_i):
        fe_tobytes32(fe_sub(chk, x, where), where)  # fe_iszero
    r = vmax(r, fe_mul(r, SQRT_M1, where))
    return fe_abs(r, where)


def ristretto_decode(where="decode"):
    s = list(MASK)                                   # fe_frombytes32: 255 bits, maybe >= p
    fe_tobytes32(s, where)                           # the canonical re-encoding check
    ss = fe_sq(s, where)
    u1 = fe_carry(fe_sub(ONE, ss, where), where)
    u2 = fe_carry(fe_add(ONE, ss, where), where)
    u2sq = fe_sq(u2, where)
    t = fe_mul(fe_sq(u1, where), D, where)
    t = fe_carry(fe_add(t, u2sq, where), where)
    v = fe_carry(fe_neg(t, where), where)
    t = fe_mul(v, u2sq, where)
    inv = sqrt_ratio_m1(ONE, t, where)
    den_x = fe_mul(inv, u2, where)
    den_y = fe_mul(fe_mul(inv, den_x, where), v, where)
    t = fe_mul(fe_carry(fe_add(s, s, where), where), den_x, where)
    X = fe_abs(t, where)
    Y = fe_mul(u1, den_y, where)
    T = fe_mul(X, Y, where)
    fe_tobytes32(T, where)
    fe_tobytes32(Y, where)
    return (X, Y, ONE, T)


def ristretto_encode(p, where="encode"):
    X, Y, Z, T = p
    t = fe_add(Z, Y, where)
    u1 = fe_mul(t, fe_sub(Z, Y, where), where)
    u2 = fe_mul(X, Y, where)
    t = fe_mul(fe_sq(u2, where), u1, where)
    inv = sqrt_ratio_m1(ONE, t, where)
    den1, den2 = fe_mul(inv, u1, where), fe_mul(inv, u2, where)
    z_inv = fe_mul(fe_mul(den1, den2, where), T, where)
    ix0, iy0 = fe_mul(X, SQRT_M1, where), fe_mul(Y, SQRT_M1, where)
    ench = fe_mul(den1, INVSQRT_A_MINUS_D, where)
    fe_tobytes32(fe_mul(T, z_inv, where), where)
    x, y, den_inv = vmax(X, iy0), vmax(Y, ix0), vmax(den2, ench)
    fe_tobytes32(fe_mul(x, z_inv, where), where)
    y = vmax(y, fe_carry(fe_neg(y, where), where))
    t = fe_mul(den_inv, fe_sub(Z, y, where), where)
    fe_tobytes32(fe_abs(t, where), where)


def ristretto_elligator(where="elligator"):
    t0 = fe_carry(list(MASK), where)
    r = fe_mul(fe_sq(t0, where), SQRT_M1, where)
    u = fe_mul(fe_add(r, ONE, where), ONE_MINUS_D_SQ, where)
    tmp = fe_carry(fe_neg(fe_add(fe_mul(r, D, where), ONE, where), where), where)
    v = fe_mul(tmp, fe_add(r, D, where), where)
    s = sqrt_ratio_m1(u, v, where)
    s_prime = fe_carry(fe_neg(fe_abs(fe_mul(s, t0, where), where), where), where)
    s = vmax(s, s_prime)
    c = vmax(fe_carry(fe_neg(ONE, where), where), r)
    n = fe_mul(fe_mul(c, fe_sub(r, ONE, where), where), D_MINUS_ONE_SQ, where)
    n = fe_carry(fe_sub(n, v, where), where)
    w0 = fe_mul(fe_carry(fe_add(s, s, where), where), v, where)
    w1 = fe_mul(n, SQRT_AD_MINUS_ONE, where)
    tmp = fe_sq(s, where)
    w2 = fe_carry(fe_sub(ONE, tmp, where), where)
    w3 = fe_add(ONE, tmp, where)
    return (fe_mul(w0, w3, where), fe_mul(w2, w1, where), fe_mul(w1, w3, where), fe_mul(w0, w2, where))


def ristretto_eq(p, q):
    a = fe_mul(p[0], q[1], "eq")
    b = fe_mul(p[1], q[0], "eq")
    fe_tobytes32(fe_sub(a, b, "eq"), "eq tobytes")
    a = fe_mul(p[1], q[1], "eq")
    b = fe_mul(p[0], q[0], "eq")
    fe_tobytes32(fe_sub(a, b, "eq"), "eq tobytes")


# ---------------- the closed invariant ----------------
D = fe_const_from_header("D")
D2 = fe_const_from_header("D2")
SQRT_M1 = fe_const_from_header("SQRT_M1")
INVSQRT_A_MINUS_D = fe_const_from_header("INVSQRT_A_MINUS_D")
ONE_MINUS_D_SQ = fe_const_from_header("ONE_MINUS_D_SQ")
D_MINUS_ONE_SQ = fe_const_from_header("D_MINUS_ONE_SQ")
SQRT_AD_MINUS_ONE = fe_const_from_header("SQRT_AD_MINUS_ONE")


def run():
    global violations, worst
    violations, worst = [], {}
    # TIGHT: the output bound of fe_mul / fe_sq on any admissible inputs; iterate: start from the
    # canonical limb widths and widen with every producer until nothing grows.
    tight = [MASK[i] for i in range(10)]
    for _ in range(10):
        pt = (tight, tight, tight, tight)
        c = ge_to_cached(pt)
        outs = [ge_add(pt, c), ge_add(pt, c, "ge_sub", swap=True), ge_dbl(pt), ge_dbl_lean(pt),
                ge_add_signed(pt, c), ge_add_lds(pt, c), ge_add(pt, ge_cached_neg(c), "ge_add(-q)")]
        aff = (fe_carry(fe_add(tight, tight)), fe_carry(fe_sub(tight, tight)), fe_mul(fe_mul(tight, tight), D2))
        outs += [ge_madd(pt, comb8_entry(*aff), "comb8 madd"), ge_madd(pt, aff, "ge_msub", minus=True)]
        outs += [ge_madd_signed(pt, affine_addend(pt)), ge_add_ded(pt, ge_to_cached_ded(pt))]
        outs += [ristretto_decode(), ristretto_elligator()]
        ristretto_encode(pt)
        new = vmax(tight, *[x for o in outs for x in o])
        # fe_carry outputs (decode's fe_abs, cached forms) are also stored coordinates
        new = vmax(new, fe_carry(fe_neg(tight)), fe_carry(fe_add(tight, tight)))
        if new == tight:
            break
        tight = new
    else:
        violations.append("no fixpoint for the coordinate bound")
    pt = (tight, tight, tight, tight)
    ristretto_eq(pt, pt)
    fe_tobytes32(tight)
    fe_mul_small(tight, (1 << 12) - 1)
    return tight


def main():
    tight = run()
    f_max = max(tight)
    print("TIGHT coordinate bound (log2 per limb):", log2s(tight))
    print("TIGHT max limb: 2^%.4f" % math.log2(f_max))
    groups = {}
    for name, (v, lim) in worst.items():  # the worst case of each kind of check over all call sites
        kind = name.split(" ", 1)[1] if " " in name else name
        kind = re.sub(r"h\d$", "h*", kind)
        if kind not in groups or v / lim > groups[kind][0] / groups[kind][1]:
            groups[kind] = (v, lim, name)
    print("worst case per check (value, limit, where):")
    for kind in sorted(groups):
        v, lim, name = groups[kind]
        print(f"  {kind:52s} 2^{math.log2(v) if v else 0:7.3f} < 2^{math.log2(lim):.0f}   ({name.split(' ')[0]})")
    if os.environ.get("FE_BOUNDS_VERBOSE"):
        for name in sorted(worst):
            v, lim = worst[name]
            print(f"  {name:48s} max 2^{math.log2(v) if v else 0:7.3f}  limit 2^{math.log2(lim):.0f}")
    if violations:
        print("VIOLATIONS:")
        for v in violations:
            print("  " + v)
        return 1
    print("OK: no 32-bit limb, pre-multiply or 64-bit column overflow; fe_sub/fe_neg never wrap")
    return 0


if __name__ == "__main__":
    sys.exit(main())
