"""Checker (test infrastructure only): the reference's finalise rules restated on the CPU oracle.

Phases<Phase4>::proceed (committee.rs:625-688) and Phases<Phase5>::finalise (committee.rs:726-805)
as every party runs them, on Python integers mod l and the oracle's group operations
(tests/oracle_lib.py).  Small committees only (pure-Python loops).  Pinned against the libsodium
fixtures finalise_parties_*.json by tests/test_oracle.py, then used by the GPU tests as the
checker of dkg_finalise_parties and of the ceremony-level mpk on random faulty committees.
"""
from tests import oracle_lib as O

L = 2**252 + 27742317777372353535851937790883648493
ID = bytes(32)


def scalar(b: bytes) -> int:
    return int.from_bytes(b, "little") % L


def lagrange_at_zero(ys, xs):
    """polynomial.rs:162-184 at x = 0 (xs distinct)."""
    res = 0
    for xa, ya in zip(xs, ys):
        num = den = 1
        for xb in xs:
            if xb != xa:
                num = num * (0 - xb) % L
                den = den * (xa - xb) % L
        res = (res + num * pow(den, -1, L) * ya) % L
    return res


def gsum(points):
    """Sum of compressed points (oracle MSM with unit scalars); the identity for none."""
    if not points:
        return ID
    one = (1).to_bytes(32, "little")
    return O.msm(one * len(points), b"".join(points))


def g_mul(k: int) -> bytes:
    return O.base_mul((k % L).to_bytes(32, "little"))


def party_finalise(p, n, t, qualified, recon, A0, share, own_A0=None, disclosed=None, r2_error=None,
                   r4_error=None):
    """(status, index, mpk) of party p (0-based).  share(i, j) -> s_ij as int; A0[i] the broadcast
    A_i0 (32 bytes); own_A0 the party's own A_p0 from its init state (default A0[p])."""
    disclosed = disclosed or [1] * n
    if r2_error and r2_error[p]:
        return "R2_ERROR", -1, None                           # committee.rs:340-347
    if r4_error and r4_error[p]:
        return "R4_ERROR", -1, None                           # :567-569
    if sum(qualified) - sum(recon) <= t:
        return "PHASE4_ERROR", -1, None                       # :673-677
    final = [q ^ r for q, r in zip(qualified, recon)]         # :733-739
    terms, secret = [], 0
    for i in range(n):
        if recon[i] and qualified[i]:
            xs, ys = [p + 1], [share(i, p)]                   # own index and share (:754-761)
            for q in range(n):
                # :763-775; a party that failed Phase1/Phase3 never broadcasts phase 5 (:684)
                if (q != p and disclosed[q] and final[q] and not (r2_error and r2_error[q])
                        and not (r4_error and r4_error[q])):
                    xs.append(q + 1)
                    ys.append(share(i, q))
            if len(xs) < t:                                   # :779-781 (threshold, not t + 1)
                return "INSUFFICIENT", i, None
            secret = (secret + lagrange_at_zero(ys, xs)) % L  # :784-789
        elif i == p:
            terms.append(own_A0 if own_A0 is not None else A0[p])  # committed_shares[my-1] (:190)
        elif qualified[i]:
            terms.append(A0[i])                               # :790-795
        else:
            return "PANIC", i, None                           # expect() on None (:791-794)
    return "OK", -1, gsum(terms + [g_mul(secret)])


def final_party_mpk(n, qualified, recon, A0, share, r2_error=None, r4_error=None, t=None):
    """The master public key every finalising final party computes when all disclosures arrive: the
    reconstructed secrets are interpolated over the final parties that disclose -- a party whose
    Phase1 or Phase3 proceed failed (r2 / r4 error, committee.rs:340-347, 567-569, 684) never
    broadcasts its phase-5 shares.  None when those are fewer than t (InsufficientSharesForRecovery
    for every finalising party, :779-781; t must be given then)."""
    final = [q and not r for q, r in zip(qualified, recon)]
    err = [bool((r2_error and r2_error[j]) or (r4_error and r4_error[j])) for j in range(n)]
    xs = [j + 1 for j in range(n) if final[j] and not err[j]]
    if any(recon) and t is not None and len(xs) < t:
        return None
    secret = sum(lagrange_at_zero([share(i, x - 1) for x in xs], xs) for i in range(n) if recon[i]) % L
    return gsum([A0[i] for i in range(n) if final[i]] + [g_mul(secret)])
