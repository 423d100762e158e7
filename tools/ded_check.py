#!/usr/bin/env python3
"""Numeric check of the stepping's dedicated addition (points.h ge_add_ded_lds, HWCD 2008
"add-2008-hwcd-4" for a = -1) against the complete group law (tools/r255.py add):

  * on random pairs of points (random projective scaling) it returns p + q with Z != 0;
  * over every pair of 8-torsion offsets T1, T2 and the relations q = p, q = -p, q = 2p, q random
    (p = a g + T1, q = b g + T2), it either returns p + q exactly or a point with Z = 0 -- never a
    wrong point with Z != 0.  That is what makes the stepping's redo rule exact: a workgroup whose
    sums all came out with Z != 0 holds the complete formula's values.
Usage: python tools/ded_check.py   (exit status 1 on a wrong sum); tests/test_bounds.py runs it.
"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import r255 as R  # noqa: E402

P = R.P


def ded(p, q):
    """ge_add_ded_lds on (X, Y, Z, T) and the cached (Y+X, Y-X, 2Z, 2T) of q."""
    ypx, ymx, z2, t2 = (q.Y + q.X) % P, (q.Y - q.X) % P, 2 * q.Z % P, 2 * q.T % P
    A = (p.Y - p.X) * ypx % P
    B = (p.Y + p.X) * ymx % P
    F, G = (B - A) % P, (B + A) % P
    C, Dd = p.Z * t2 % P, p.T * z2 % P
    E, H = (Dd + C) % P, (Dd - C) % P
    return R.Pt(E * F, G * H, G * F, E * H)


def same(a, b):
    return all((u * b.Z - v * a.Z) % P == 0 for u, v in ((a.X, b.X), (a.Y, b.Y), (a.T, b.T)))


def scaled(p, s):
    return R.Pt(p.X * s, p.Y * s, p.Z * s, p.T * s)


def mul_full(p, k):  # k * p without reducing k mod l (torsion survives)
    r = R.IDENTITY
    while k:
        if k & 1:
            r = R.add(r, p)
        p = R.add(p, p)
        k >>= 1
    return r


def torsion(rng):
    """The 8 points of E[8] as l * (random curve points)."""
    out = {}
    while len(out) < 8:
        y = rng.randrange(P)
        x2 = (1 - y * y) * pow((-1 - R.D * y * y) % P, P - 2, P) % P
        x = pow(x2, (P + 3) // 8, P)
        if x * x % P != x2:
            x = x * pow(2, (P - 1) // 4, P) % P
        if x * x % P != x2:
            continue
        t = mul_full(R.Pt(x, y, 1, x * y), R.L)
        zi = pow(t.Z, P - 2, P)
        out[(t.X * zi % P, t.Y * zi % P)] = None
    return [R.Pt(x, y, 1, x * y) for x, y in out]


def run(seed=1, nrand=64):
    rng = random.Random(seed)
    g = R.from_uniform_bytes(bytes(range(64)))
    stats = {"sum": 0, "Z=0": 0, "wrong": 0}

    def one(p, q):
        r = ded(p, q)
        if r.Z % P == 0:
            stats["Z=0"] += 1
        elif same(r, R.add(p, q)):
            stats["sum"] += 1
        else:
            stats["wrong"] += 1

    for _ in range(nrand):
        one(scaled(R.mul(g, rng.randrange(1, R.L)), rng.randrange(1, P)), R.mul(g, rng.randrange(1, R.L)))
    rand_exc = stats["Z=0"]
    for t1 in torsion(rng):
        for t2 in torsion(rng):
            for rel in range(4):
                a = rng.randrange(1, R.L)
                b = (a, R.L - a, 2 * a % R.L, rng.randrange(1, R.L))[rel]
                one(scaled(R.add(R.mul(g, a), t1), rng.randrange(1, P)), R.add(R.mul(g, b), t2))
    one(R.IDENTITY, R.IDENTITY)
    one(g, R.IDENTITY)
    return stats, rand_exc


if __name__ == "__main__":
    st, rx = run()
    print(st, "exceptional among random pairs:", rx)
    sys.exit(1 if st["wrong"] or rx else 0)
