"""Fault-injected parity at the BASELINE sizes (configs 2-5), through the C ABI, against the CPU oracle.

The oracle (tests/oracle_lib.py: dalek-3's algorithms, a vartime MSM per pair, committee.rs:287-305,
532-548) recomputes WHOLE decision rows of the tampered dealers; the honest rows are checked by
properties.  Config numbers are SURVEY.md 8(d)'s (= BASELINE.json configs[0..4]): 2 is n=256 (t=127),
3 is n=1024 (t=511: the headline schedule -- cost-model split U=4 with pieces of 128 positions,
short lattice multipliers, two dealer-chunk streams, rounds 2 and 4 fused -- and forced U=2 / 3 /
5), 4 is n=4096 (t=2047, whose pieces exceed 512 positions: the block-chained stepping,
kernels.hip k_stepping<512> with its up/down boundary streams), 5 is the 10,000-ceremony batch of
n=64 (t=31: the per-wave binomial and the stepping's dead-position repack); plus n=1100 (t=549)
with a short last piece.
"""
import random

import pytest

import dkg_amd
from dkg_amd import ACCEPT, MISSING, REJECT, SELF, SKIPPED
from tests import finalise_ref as FR
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

H = bytes.fromhex
L = 2**252 + 27742317777372353535851937790883648493
CK = b"Example of a shared string."


@pytest.fixture(scope="module")
def be():
    b = dkg_amd.Backend(0)
    yield b
    b.close()


def _rand_point(rng):
    return O.base_mul(rng.randrange(1, L).to_bytes(32, "little"))


def _bump(buf, off):
    v = (int.from_bytes(buf[off:off + 32], "little") + 1) % L
    buf[off:off + 32] = v.to_bytes(32, "little")


def _inject(rng, n, t, E, A, s, sp, base=0):
    """Tamper dealers base..base+4: E, A [..][t+1][32], s, sp [..][n][32] are bytearrays whose row 0
    is dealer `base` (a rank's block of a sharded run; base = 0: the whole committee).  Returns
    {local dealer: description}.  Receivers and coefficient positions are chosen across the stepping
    blocks (multiples of 512) and the degree-split pieces; dealer base+2's unchecked self-share sits
    at the GLOBAL diagonal j = base + 2."""
    N = t + 1
    js = sorted({0, 1, min(511, n - 1), min(512, n - 1), n // 2, n - 1, rng.randrange(n)} - {0})
    for j in js:                                           # dealer 0: flipped shares
        _bump(s, 32 * (0 * n + j))
    _bump(sp, 32 * (0 * n + n - 2))                        # ... and one flipped randomness share
    for k in sorted({0, N // 2, N - 1}):                   # dealer 1: replaced E coefficients
        E[32 * (1 * N + k):32 * (1 * N + k) + 32] = _rand_point(rng)
    A[32 * (2 * N + N - 1):32 * (2 * N + N)] = _rand_point(rng)  # dealer 2: a replaced A coefficient
    _bump(s, 32 * (2 * n + base + 2))                      # ... and its unchecked self-share
    E[32 * (3 * N + N // 3) + 31] |= 0x80                  # dealer 3: an undecodable E row (MISSING)
    for j in (7, n - 3):                                   # dealer 4: randomness only (round 2 only)
        _bump(sp, 32 * (4 * n + j))
    return {0: "shares", 1: "E", 2: "A+self", 3: "E undecodable", 4: "randomness"}


# (dealer, round) pairs whose whole rows the oracle recomputes; every other row of the tampered
# dealers is fixed by the tampering itself (untouched data accepts; an undecodable E row is MISSING)
FULL_ROWS = [(0, 2), (0, 4), (1, 2), (2, 4), (4, 2)]


def _expected_rows(n, t, h, E, A, s, sp, full=FULL_ROWS, sample=None, base=0):
    """{(local dealer, round): expected raw decision row} for dealers base..base+4 (SKIPPED not
    applied; E, A, s, sp as _inject's, row 0 = dealer base).  Rows in `full` come from the oracle;
    with `sample` (a receiver list) the (4, 2) row is checked by the oracle at those receivers only
    and completed analytically (large n)."""
    N = t + 1
    exp = {}
    for i in range(5):
        g = base + i
        for rnd in (2, 4):
            row = bytearray(SELF if j == g else ACCEPT for j in range(n))
            if (i, rnd) == (3, 2):
                row = bytearray(SELF if j == g else MISSING for j in range(n))
            exp[(i, rnd)] = row
    for j in (7, n - 3):
        if j != base + 4:
            exp[(4, 2)][j] = REJECT
    rows = lambda buf, w, i: bytes(buf[w * i:w * (i + 1)])  # noqa: E731
    for (i, rnd) in full:
        if sample is not None and (i, rnd) == (4, 2):
            continue
        C = E if rnd == 2 else A
        acc, _ = O.verify_rows(n, t, rnd, rows(C, 32 * N, i), h, rows(s, 32 * n, i),
                               rows(sp, 32 * n, i) if rnd == 2 else None, base + i, base + i + 1, 0, n)
        exp[(i, rnd)] = bytearray(acc)
    if sample is not None:
        for j in sample:
            acc, _ = O.verify_rows(n, t, 2, rows(E, 32 * N, 4), h, rows(s, 32 * n, 4), rows(sp, 32 * n, 4),
                                   base + 4, base + 5, j, j + 1)
            assert acc[0] == exp[(4, 2)][j], ("oracle disagrees with the injected fault", j)
    return {k: bytes(v) for k, v in exp.items()}


def _check_rows(n, dec2, dec4, qualified, exp, ctx):
    """dec2 / dec4: row accessors of the ceremony outputs (dec4 with SKIPPED for disqualified
    dealers).  Tampered dealers' rows equal `exp`; every other row accepts."""
    for i in range(n):
        r2, r4 = bytes(dec2(i)), bytes(dec4(i))
        if i < 5:
            assert r2 == exp[(i, 2)], (ctx, i, "round 2")
            e4 = exp[(i, 4)] if qualified[i] else bytes(SELF if j == i else SKIPPED for j in range(n))
            assert r4 == e4, (ctx, i, "round 4")
        else:
            row = bytes(SELF if j == i else ACCEPT for j in range(n))
            assert r2 == row and r4 == row, (ctx, i)


@pytest.mark.parametrize("n,t,split,combine", [(256, 127, 0, 0), (1024, 511, 0, 0), (1024, 511, 2, 0),
                                               (1024, 511, 3, 0), (1024, 511, 3, 1), (1024, 511, 5, 0),
                                               (1024, 511, 5, 1), (1024, 511, 6, 0)])
def test_faults_baseline_sizes(be, n, t, split, combine):
    """Configs 2 and 3 with the default schedule (for n=1024 the headline one: U=4 from the cost
    model, pieces of 128 positions recombined with short lattice multipliers, every piece of a
    column in one 512-lane stepping workgroup, two dealer-chunk streams, rounds 2 and 4 fused), and
    forced U=2 / U=3 (171 + 171 + 170, the last piece a step late; short multipliers and powers of
    j^L) / U=5 (five-piece short multipliers, and powers) / U=6 (powers, pairwise Horner in y^2): tampered shares, randomness, E and A
    coefficients, an undecodable E row and a tampered self-share.  Whole rows of every tampered
    dealer equal the oracle's per-pair MSM checks; qualification, reconstruction, final shares and
    the final parties' mpk follow the reference's rules (committee.rs:311-398, 454-467, 660-805)."""
    N = t + 1
    h = be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes([n % 251]) * 32, 11, 0, n, t)
    E, A, s, sp = (bytearray(x) for x in be.share_gen(a, b, n, n, t))
    rng = random.Random(n)
    faulty = _inject(rng, n, t, E, A, s, sp)
    be.set_split(split)
    be.set_combine(combine)
    try:
        r = be.ceremony_verify(bytes(E), bytes(A), bytes(s), bytes(sp), n, t)
        U, comb = be.last_split(), be.last_combine()
    finally:
        be.set_split(0)
        be.set_combine(0)
    if split:
        assert U == split
    elif n == 1024:
        assert U == 4, "the headline schedule uses the cost model's U=4 at n=1024"
    assert comb == (0 if U == 1 else 1 if (combine == 1 or U > 5) else 2)
    assert sorted(faulty) == [0, 1, 2, 3, 4]
    exp = _expected_rows(n, t, h, E, A, s, sp)
    qualified = [0 if i in (0, 1, 3, 4) else 1 for i in range(n)]
    assert r.qualified == qualified
    _check_rows(n, lambda i: r.dec2[i * n:(i + 1) * n], lambda i: r.dec4[i * n:(i + 1) * n], qualified, exp, (n, U))
    recon = [int(i == 2) for i in range(n)]
    assert r.reconstruct == recon and r.phase4_error == 0
    complaints = [sum(1 for i in range(n) if i != j and r.dec2[i * n + j] == REJECT) for j in range(n)]
    assert r.complaints2 == complaints
    share = lambda i, j: int.from_bytes(s[32 * (i * n + j):32 * (i * n + j) + 32], "little")  # noqa: E731
    for j in random.Random(1).sample(range(n), 4):
        assert int.from_bytes(r.final_share[32 * j:32 * j + 32], "little") == \
            sum(share(i, j) for i in range(n) if qualified[i]) % L
    A0 = [bytes(A[32 * N * i:32 * N * i + 32]) for i in range(n)]
    assert r.mpk == FR.final_party_mpk(n, qualified, recon, A0, share)
    # the mpk is the honest one: dealer 2's secret recovered from the final parties, its bad s_22 unused
    sec = sum(int.from_bytes(a[32 * N * i:32 * N * i + 32], "little") for i in range(n) if qualified[i]) % L
    assert r.mpk == O.base_mul(sec.to_bytes(32, "little"))


def _device_committee(be, n, t, master, ceremony):
    import torch

    N = t + 1
    dev = torch.device("cuda", 0)
    ta = torch.empty(32 * n * N, dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    be.dealer_coefficients_device(master, ceremony, 1, 0, n, t, ta.data_ptr(), tb.data_ptr())
    tE = torch.empty(32 * n * N, dtype=torch.uint8, device=dev)
    tA = torch.empty_like(tE)
    ts = torch.empty(32 * n * n, dtype=torch.uint8, device=dev)
    tsp = torch.empty_like(ts)
    be.share_gen_device(n, n, t, ta.data_ptr(), tb.data_ptr(), tE.data_ptr(), tA.data_ptr(), ts.data_ptr(),
                        tsp.data_ptr())
    return ta, tE, tA, ts, tsp


def _shard_verify_all(be, n, t, tE, tA, ts, tsp):
    import torch

    dev = ts.device
    o2 = torch.zeros(n * n, dtype=torch.uint8, device=dev)
    o4 = torch.zeros_like(o2)
    oA = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
    op = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
    be.ceremony_shard_verify_device(n, t, 0, n, tE.data_ptr(), tA.data_ptr(), ts.data_ptr(), tsp.data_ptr(),
                                    o2.data_ptr(), o4.data_ptr(), oA.data_ptr(), op.data_ptr())
    return o2.view(n, n), o4.view(n, n)


# (U, piece length L) per run; the last piece holds t + 1 - (U - 1) L coefficients
@pytest.mark.parametrize("n,t,splits", [(1100, 549, ((1, 550), (3, 192), (2, 320))),
                                        (4096, 2047, ((2, 1024), (1, 2048), (3, 683), (4, 512)))])
def test_faults_multiblock_stepping(be, golden, n, t, splits):
    """Pieces longer than 512 positions take the block-chained stepping (k_stepping<512>, the top
    block streaming its per-step values down): n=1100, t=549 unsplit (2 blocks of 275) and n=4096,
    t=2047 at U=2 (2 blocks of 512 per piece) and unsplit (4 blocks).  Short last pieces, the piece
    length rounded up to whole waves: n=1100 at U=3 (192 + 192 + 166, per-piece stepping tables,
    the last one in its own launch, joining the binomial 26 steps late) and U=2 (320 + 230, 90 steps
    late), n=4096 at U=3 (683 + 683 + 682 in 2 blocks each) and U=4 (config E's split).  Split
    runs recombine with short lattice multipliers (the default).  The committee is built on the
    device (dkg_share_gen_device), tampered there, and verified as one shard of all dealers; whole
    rows of the tampered dealers equal the oracle's (MSM over t+1 = 550 / 2048 points, Pippenger
    w=7 / w=8).  At n=4096 the committee uses the seed of tests/golden/spot_n4096_t2047.json, whose
    libsodium commitments and shares it must reproduce."""
    import torch

    N = t + 1
    spot = golden("spot_n4096_t2047.json") if n == 4096 else None
    master = H(spot["master_seed"]) if spot else bytes([3]) * 32
    h = be.env_init(t, n, CK)
    ta, tE, tA, ts, tsp = _device_committee(be, n, t, master, 0)
    if spot:  # golden spot dealers (libsodium) inside the device-generated committee
        assert h.hex() == spot["h"]
        for d in spot["dealers"]:
            i = d["dealer"]
            assert bytes(tE[32 * N * i:32 * N * (i + 1)].cpu().numpy()).hex() == d["E"]
            assert bytes(tA[32 * N * i:32 * N * (i + 1)].cpu().numpy()).hex() == d["A"]
            for pr in d["pairs"]:
                j = pr["receiver"]
                assert bytes(ts[32 * (i * n + j):32 * (i * n + j + 1)].cpu().numpy()).hex() == pr["s"]
                assert bytes(tsp[32 * (i * n + j):32 * (i * n + j + 1)].cpu().numpy()).hex() == pr["s_prime"]
    # tamper dealers 0..4 on the host copies of their rows, write them back
    D5 = 5
    E = bytearray(tE[:32 * N * D5].cpu().numpy().tobytes())
    A = bytearray(tA[:32 * N * D5].cpu().numpy().tobytes())
    s = bytearray(ts[:32 * n * D5].cpu().numpy().tobytes())
    sp = bytearray(tsp[:32 * n * D5].cpu().numpy().tobytes())
    _inject(random.Random(n + 1), n, t, E, A, s, sp)
    for t_, b_ in ((tE, E), (tA, A), (ts, s), (tsp, sp)):
        t_[:len(b_)] = torch.frombuffer(bytearray(b_), dtype=torch.uint8).to(t_.device)
    sample = [7, n - 3] + random.Random(n).sample(range(8, n - 3), 30) if n > 2000 else None
    exp = _expected_rows(n, t, h, E, A, s, sp, sample=sample)
    for U, plen in splits:
        be.set_split(U)
        try:
            d2, d4 = _shard_verify_all(be, n, t, tE, tA, ts, tsp)
            assert be.last_split() == U and be.last_split_len() == plen
        finally:
            be.set_split(0)
        h2 = d2[:D5].cpu().numpy()
        h4 = d4[:D5].cpu().numpy()
        # shard rows carry the raw decisions (SKIPPED is applied by the combine step)
        for i in range(D5):
            assert bytes(h2[i]) == exp[(i, 2)], (n, U, i, "round 2")
            assert bytes(h4[i]) == exp[(i, 4)], (n, U, i, "round 4")
        # honest rows (dealers >= 5) on the device: ACCEPT everywhere but the SELF diagonal
        eye = torch.eye(n, dtype=torch.bool, device=d2.device)[D5:]
        for d in (d2[D5:], d4[D5:]):
            assert bool(((d == ACCEPT) | (eye & (d == SELF))).all()) and int((d == SELF).sum()) == n - D5


def test_batch_config5_full_size(be):
    """BASELINE config 5 at its real size: 10,000 honest n=64, t=31 ceremonies in one batch from
    device coefficients (640,000 dealer rows).  Every pair of every ceremony accepts in both rounds,
    every ceremony qualifies all 64 dealers, every ceremony's mpk == g * sum_i a_i0
    (committee.rs:1633-1647), and sampled ceremonies' final shares interpolate to the secret."""
    import numpy as np
    import torch

    B, n, t = 10000, 64, 31
    N = t + 1
    be.env_init(t, n, CK)
    dev = torch.device("cuda", 0)
    ta = torch.empty(B * n * N * 32, dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    be.dealer_coefficients_device(b"\x5c" * 32, 0, B, 0, n, t, ta.data_ptr(), tb.data_ptr())
    r = dkg_amd.ceremony_batch_device(be, B, n, t, ta.data_ptr(), tb.data_ptr(), big=True)
    assert r.n_qualified == [n] * B and set(r.phase4_error) == {0}
    d2 = np.frombuffer(r.dec2, dtype=np.uint8).reshape(B, n, n)
    d4 = np.frombuffer(r.dec4, dtype=np.uint8).reshape(B, n, n)
    eye = np.eye(n, dtype=bool)[None]
    for d in (d2, d4):
        assert ((d == ACCEPT) | (eye & (d == SELF))).all() and int((d == SELF).sum()) == B * n
    a0 = ta.view(B * n, N, 32)[:, 0, :].cpu().numpy()
    for c in range(B):
        sec = sum(int.from_bytes(a0[c * n + i].tobytes(), "little") for i in range(n)) % L
        assert r.mpk[c] == O.base_mul(sec.to_bytes(32, "little")), c
    rng = random.Random(5)
    for c in [0, B - 1] + rng.sample(range(B), 6):
        xs = rng.sample(range(1, n + 1), t + 1)
        fs = [int.from_bytes(r.final_share[32 * (c * n + x - 1):32 * (c * n + x)], "little") for x in xs]
        sec = sum(int.from_bytes(a0[c * n + i].tobytes(), "little") for i in range(n)) % L
        assert FR.lagrange_at_zero(fs, xs) == sec, c


def test_batch_faulty_members_at_scale(be, golden):
    """A batch of 2,500 n=10, t=4 ceremonies in which the fault fixtures sit at the first, middle and
    last positions (row offsets up to 25,000 dealers): each member equals its golden ceremony bit for
    bit, the honest filler ceremonies equal the honest golden."""
    names = ["fault_self_share_n10_t4.json", "fault_share_flip_n10_t4.json", "fault_a_many_n10_t4.json",
             "fault_recon_only_n10_t4.json"]
    honest = golden("ceremony_n10_t4.json")
    fx = [golden(x) for x in names]
    B, n, t = 2500, 10, 4
    be.env_init(t, n, CK)
    at = {0: fx[0], 1249: fx[1], 1250: fx[2], B - 1: fx[3]}
    cs = [at.get(c, honest) for c in range(B)]
    E = b"".join(H(c["E"]) for c in cs)
    A = b"".join(H(c["A"]) for c in cs)
    s = b"".join(H(c["s"]) for c in cs)
    sp = b"".join(H(c["s_prime"]) for c in cs)
    r = dkg_amd.ceremony_batch_verify(be, B, n, t, E, A, s, sp)
    for k in sorted(set(at) | {1, 777, B - 2}):
        c, d = cs[k], r.ceremony(k)
        assert "".join(str(x) for x in d["dec2"]) == c["dec2"], k
        assert "".join(str(x) for x in d["dec4"]) == c["dec4"], k
        assert d["qualified"] == c["qualified"] and d["reconstruct"] == c["reconstruct"], k
        assert d["r4_error"] == [int(x) for x in c["r4_error"]] and d["phase4_error"] == int(c["phase4_error"]), k
        assert d["final_share"].hex() == c["final_share"] and d["mpk"].hex() == c["mpk"], k
    hm = H(honest["mpk"])
    assert sum(1 for c in range(B) if r.mpk[c] == hm) == B - len(at)


@pytest.mark.parametrize("n,t", [(130, 64), (300, 149), (517, 258)])
def test_recombination_modes_agree_on_faults(be, n, t):
    """Ragged sizes with tampered dealers (shares, E, A, an undecodable row, randomness): every split
    U = 2..5 recombined with short lattice multipliers, U = 3..5 with powers of j^L and U = 6 give the
    same decision matrices, qualification and mpk as the unsplit tables."""
    be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes([t % 251]) * 32, 5, 0, n, t)
    E, A, s, sp = (bytearray(x) for x in be.share_gen(a, b, n, n, t))
    _inject(random.Random(n * 7 + t), n, t, E, A, s, sp)
    runs = {}
    try:
        for split, comb, add in ((1, 0, 0), (2, 0, 0), (3, 0, 0), (4, 0, 0), (2, 0, 1), (3, 0, 1), (4, 0, 1),
                                 (3, 1, 0), (4, 1, 0), (5, 0, 0), (5, 1, 0), (5, 0, 1), (6, 0, 0)):
            be.set_split(split)
            be.set_combine(comb)
            be.set_addends(add)
            r = be.ceremony_verify(bytes(E), bytes(A), bytes(s), bytes(sp), n, t)
            assert be.last_split() == split
            short = split <= 4 or (split == 5 and add == 0)  # five pieces: affine addends only
            assert be.last_combine() == (0 if split == 1 else 2 if (comb == 0 and short) else 1)
            runs[(split, comb, add)] = r
    finally:
        be.set_split(0)
        be.set_combine(0)
        be.set_addends(0)
    ref = runs.pop((1, 0, 0))
    assert ref.qualified[:5] == [0, 0, 1, 0, 0] and all(ref.qualified[5:])
    for key, r in runs.items():
        assert r.dec2 == ref.dec2 and r.dec4 == ref.dec4, key
        assert r.qualified == ref.qualified and r.reconstruct == ref.reconstruct and r.mpk == ref.mpk, key


@pytest.mark.parametrize("n,t,split", [(1024, 511, 4), (1024, 511, 3), (1100, 549, 1)])
def test_stepping_redo_at_scale(be, n, t, split):
    """The stepping's exact fallback at the BASELINE size and in each stepping layout -- whole-column
    slots (U=4), per-piece tables (U=3: 171-position pieces) and 512-lane blocks chained through
    boundary streams (n=1100 unsplit: 550 positions): an E row made the identity (committee.rs:1127)
    makes its dedicated additions exceptional; the marked workgroups are redone by the complete
    formula, and every output equals the complete formula's run.  The same rows trip the per-step
    binomial's dedicated additions (e_{m-1} + e_m of two identities has Z = 0): its guard word makes
    the driver rerun the whole verification with the complete formula (binomial_reruns() == 1) -- on
    the headline schedule at n=1024 (two chunk streams, lane-pair early steps, column-sum copy) --
    and a committee without them reruns nothing."""
    be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes([split]) * 32, 3, 0, n, t)
    E, A, s, sp = (bytearray(x) for x in be.share_gen(a, b, n, n, t))
    N = t + 1
    _bump(s, 32 * (5 * n + 9))  # an ordinary fault
    out = []
    try:
        be.set_split(split)
        # the honest control: no identity rows, no binomial rerun (and no stepping redo)
        r0 = be.ceremony_verify(bytes(E), bytes(A), bytes(s), bytes(sp), n, t)
        assert be.binomial_reruns() == 0 and be.stepping_redos() == 0
        assert r0.dec2[5 * n:6 * n].count(REJECT) == 1
        for d in (3, n - 2):  # dealers in the first and the last stepping workgroups
            E[32 * d * N:32 * (d + 1) * N] = bytes(32 * N)
        for formula in (0, 1):
            be.set_stepping_formula(formula)
            r = be.ceremony_verify(bytes(E), bytes(A), bytes(s), bytes(sp), n, t)
            assert be.last_split() == split
            out.append((r.dec2, r.dec4, r.qualified, r.reconstruct, r.mpk, r.final_share, be.stepping_redos(),
                        be.binomial_reruns()))
    finally:
        be.set_stepping_formula(0)
        be.set_split(0)
    assert out[0][:6] == out[1][:6]
    assert out[0][6] > 0 and out[1][6] == 0
    assert out[0][7] == 1 and out[1][7] == 0  # the dedicated binomial's rerun guard fired (formula 0 only)
    dec2 = out[0][0]
    for d in (3, n - 2):
        row = dec2[d * n:(d + 1) * n]
        assert row.count(REJECT) == n - 1 and row[d] == SELF
    assert dec2[5 * n + 9] == REJECT and dec2[5 * n:6 * n].count(REJECT) == 1


def _rank_rows(be, n, t, d0, d1, tE, tA, ts, tsp):
    """Rank [d0, d1)'s rows through dkg_ceremony_shard_verify_device on views of the committee."""
    import torch

    N, D = t + 1, d1 - d0
    dev = ts.device
    o2 = torch.zeros(D * n, dtype=torch.uint8, device=dev)
    o4 = torch.zeros_like(o2)
    oA = torch.zeros(D * 32, dtype=torch.uint8, device=dev)
    op = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
    be.ceremony_shard_verify_device(n, t, d0, d1, tE[32 * N * d0:].data_ptr(), tA[32 * N * d0:].data_ptr(),
                                    ts[32 * n * d0:].data_ptr(), tsp[32 * n * d0:].data_ptr(), o2.data_ptr(),
                                    o4.data_ptr(), oA.data_ptr(), op.data_ptr())
    return o2.view(D, n), o4.view(D, n)


def _tamper_rank(be, n, t, d0, tE, tA, ts, tsp, seed):
    """_inject on the first five dealers of the rank starting at d0, written back to the device."""
    import torch

    N, D5 = t + 1, 5
    E = bytearray(tE[32 * N * d0:32 * N * (d0 + D5)].cpu().numpy().tobytes())
    A = bytearray(tA[32 * N * d0:32 * N * (d0 + D5)].cpu().numpy().tobytes())
    s = bytearray(ts[32 * n * d0:32 * n * (d0 + D5)].cpu().numpy().tobytes())
    sp = bytearray(tsp[32 * n * d0:32 * n * (d0 + D5)].cpu().numpy().tobytes())
    _inject(random.Random(seed), n, t, E, A, s, sp, base=d0)
    for t_, b_, w in ((tE, E, 32 * N), (tA, A, 32 * N), (ts, s, 32 * n), (tsp, sp, 32 * n)):
        t_[w * d0:w * d0 + len(b_)] = torch.frombuffer(bytearray(b_), dtype=torch.uint8).to(t_.device)
    return E, A, s, sp


def _check_rank(n, d0, d2, d4, exp, ctx):
    """Rank rows: the five tampered dealers equal `exp`; every other row ACCEPT with SELF at j == i."""
    import torch

    D = d2.shape[0]
    h2, h4 = d2[:5].cpu().numpy(), d4[:5].cpu().numpy()
    for i in range(5):
        assert bytes(h2[i]) == exp[(i, 2)], (ctx, d0 + i, "round 2")
        assert bytes(h4[i]) == exp[(i, 4)], (ctx, d0 + i, "round 4")
    honest = torch.full((D - 5, n), ACCEPT, dtype=torch.uint8, device=d2.device)
    idx = torch.arange(5, D, device=d2.device)
    honest[idx - 5, d0 + idx] = SELF  # the GLOBAL diagonal j = d0 + i
    assert torch.equal(d2[5:], honest) and torch.equal(d4[5:], honest), ctx


@pytest.mark.parametrize("rank", [1, 4, 7])
def test_shard_ranks_n4096(be, rank):
    """BASELINE config 4's per-rank shape: rank r in {1, 4, 7} of the 8-way dealer split at n=4096,
    t=2047 (512 dealers, d0 = 512 r) through dkg_ceremony_shard_verify_device, faults inside the
    rank's range (tampered shares and randomness, replaced E and A coefficients, an undecodable E row,
    a tampered self-share at the global diagonal j = d0 + 2).  Whole rows of the tampered dealers equal
    the oracle's per-pair MSM checks (committee.rs:287-305, 532-548); the other 507 rows accept
    everywhere except their global SELF diagonal."""
    import torch

    n, t, ws = 4096, 2047, 8
    h = be.env_init(t, n, CK)
    ta, tE, tA, ts, tsp = _device_committee(be, n, t, bytes([41]) * 32, 0)
    del ta
    d0, d1 = dkg_amd.shard_range(n, ws, rank)
    assert (d0, d1) == (512 * rank, 512 * (rank + 1))
    E, A, s, sp = _tamper_rank(be, n, t, d0, tE, tA, ts, tsp, seed=rank)
    d2, d4 = _rank_rows(be, n, t, d0, d1, tE, tA, ts, tsp)
    U = be.last_split()
    exp = _expected_rows(n, t, h, E, A, s, sp, sample=[7, n - 3] + random.Random(rank).sample(range(8, n - 3), 16),
                         base=d0)
    _check_rank(n, d0, d2, d4, exp, (n, rank, U))
    torch.cuda.synchronize()


def test_shard_ranks_n1024_all_match_single(be):
    """Config 3 (n=1024) split 8 ways (128 dealers per rank: the latency-bound shard -- column-sum
    binomial copy on every step, one stream, 2-waves-per-SIMD stepping), faults inside EVERY rank's
    range (40 tampered dealers).  Per rank: whole rows of its tampered dealers equal the oracle's.
    Then the eight ranks' blocks, gathered, through the library's combine, reconstruction and
    finalise (tests/shard_play.py) equal the single-GPU ceremony on the same broadcasts bit for bit:
    decision matrices, qualified / complaints / r2 and r4 errors / reconstruction set, final and
    public shares, mpk (committee.rs:287-305, 311-398, 454-467, 532-569, 660-805)."""
    import torch

    from tests import shard_play

    n, t, ws = 1024, 511, 8
    N = t + 1
    h = be.env_init(t, n, CK)
    ta, tE, tA, ts, tsp = _device_committee(be, n, t, bytes([43]) * 32, 2)
    del ta
    exps = {}
    for r in range(ws):
        d0, _ = dkg_amd.shard_range(n, ws, r)
        E, A, s, sp = _tamper_rank(be, n, t, d0, tE, tA, ts, tsp, seed=100 + r)
        exps[r] = _expected_rows(n, t, h, E, A, s, sp, base=d0)

    def call(r, d0, d1, o2, o4, oA, op):
        be.ceremony_shard_verify_device(n, t, d0, d1, tE[32 * N * d0:].data_ptr(), tA[32 * N * d0:].data_ptr(),
                                        ts[32 * n * d0:].data_ptr(), tsp[32 * n * d0:].data_ptr(), o2.data_ptr(),
                                        o4.data_ptr(), oA.data_ptr(), op.data_ptr())
        D = d1 - d0
        _check_rank(n, d0, o2[:D * n].view(D, n), o4[:D * n].view(D, n), exps[r], (n, r, be.last_split()))
        return ts[32 * n * d0:]

    p = shard_play.play(be, n, t, ws, call, ts.device)
    single = be.ceremony_verify(bytes(tE.cpu().numpy()), bytes(tA.cpu().numpy()), bytes(ts.cpu().numpy()),
                                bytes(tsp.cpu().numpy()), n, t)
    o = p.outcome
    assert p.dec2 == bytes(single.dec2) and p.dec4 == bytes(single.dec4)
    assert o.qualified == single.qualified and o.reconstruct == single.reconstruct
    assert o.complaints2 == single.complaints2 and o.r2_error == single.r2_error and o.r4_error == single.r4_error
    assert o.phase4_error == bool(single.phase4_error) and o.n_qualified == single.n_qualified
    assert p.final_share == single.final_share and p.public_share == single.public_share
    assert p.mpk == single.mpk and p.mpk != bytes(32)
    bad = {dkg_amd.shard_range(n, ws, r)[0] + i for r in range(ws) for i in (0, 1, 3, 4)}
    assert o.qualified == [int(i not in bad) for i in range(n)]
    assert o.reconstruct == [int(i in {dkg_amd.shard_range(n, ws, r)[0] + 2 for r in range(ws)}) for i in range(n)]


def test_shard_stepping_redo_n1024(be):
    """The 8-way n=1024 shard's stepping (256 columns x 4 pieces, 2 waves per SIMD) with identity E
    and A rows inside rank 0's dealers: their columns' dedicated additions are exceptional, the
    complete-formula redo must run, and every output of the rank equals the complete formula's
    (dkg_ctx_set_stepping_formula 1); the identity rows are rejected by every other receiver, honest
    rows accepted (committee.rs:287-305, 532-548).  (A lane-pair variant of the dedicated pass was
    built against this test and measured slower: profiles/r05_step_pair_ab.txt.)"""
    import torch

    n, t, ws = 1024, 511, 8
    N = t + 1
    be.env_init(t, n, CK)
    _, tE, tA, ts, tsp = _device_committee(be, n, t, bytes([59]) * 32, 3)
    d0, d1 = dkg_amd.shard_range(n, ws, 0)
    D = d1 - d0
    outs = []

    def rows():
        o2 = torch.zeros(D * n, dtype=torch.uint8, device=ts.device)
        o4 = torch.zeros_like(o2)
        oA = torch.zeros(D * 32, dtype=torch.uint8, device=ts.device)
        op = torch.zeros(n * 32, dtype=torch.uint8, device=ts.device)
        be.ceremony_shard_verify_device(n, t, d0, d1, tE.data_ptr(), tA.data_ptr(), ts.data_ptr(), tsp.data_ptr(),
                                        o2.data_ptr(), o4.data_ptr(), oA.data_ptr(), op.data_ptr())
        return o2, o4

    h2, h4 = rows()  # the honest rank: the binomial's guard word stays clear
    assert be.binomial_reruns() == 0 and be.stepping_redos() == 0
    assert h2.view(D, n)[0].eq(ACCEPT).sum().item() == n - 1
    for d, buf in ((7, tE), (9, tA)):  # identity rows (committee.rs:1127 style)
        buf[32 * N * d:32 * N * (d + 1)] = 0
    try:
        for formula in (0, 1):
            be.set_stepping_formula(formula)
            o2 = torch.zeros(D * n, dtype=torch.uint8, device=ts.device)
            o4 = torch.zeros_like(o2)
            oA = torch.zeros(D * 32, dtype=torch.uint8, device=ts.device)
            op = torch.zeros(n * 32, dtype=torch.uint8, device=ts.device)
            be.ceremony_shard_verify_device(n, t, d0, d1, tE.data_ptr(), tA.data_ptr(), ts.data_ptr(), tsp.data_ptr(),
                                            o2.data_ptr(), o4.data_ptr(), oA.data_ptr(), op.data_ptr())
            assert be.last_split() == 4, be.last_split()
            outs.append((bytes(o2.cpu().numpy()), bytes(o4.cpu().numpy()), bytes(oA.cpu().numpy()),
                         bytes(op.cpu().numpy()), be.stepping_redos(), be.binomial_reruns()))
    finally:
        be.set_stepping_formula(0)
    assert outs[0][:4] == outs[1][:4]
    assert outs[0][4] > 0 and outs[1][4] == 0  # the dedicated pass marked the identity rows' workgroups
    # the shard's per-step binomial (dedicated additions) met Z = 0 and the call reran with the
    # complete formula; its rows are the complete-formula run's (above)
    assert outs[0][5] == 1 and outs[1][5] == 0
    d2, d4 = outs[0][0], outs[0][1]
    row = lambda m, i, v: bytes(SELF if j == i else v for j in range(n)) == m[i * n:(i + 1) * n]  # noqa: E731
    assert row(d2, 7, REJECT) and row(d4, 9, REJECT)  # identity rows: every other receiver rejects
    assert all(row(d2, i, ACCEPT) for i in (0, 8, 9, D - 1)) and all(row(d4, i, ACCEPT) for i in (0, 8, D - 1))


@pytest.mark.parametrize("n,t", [(64, 31), (100, 49), (41, 20)])
def test_stepping_tail_repack_faults(be, n, t):
    """The dead-position repack of short unsplit tables (kernels.hip stepping_tail_phases: the last
    steps on halved segments, the live positions carried in a compact state) on tampered committees
    with an identity E row and A row (exceptional dedicated additions: each phase's marked workgroups
    are redone from that phase's starting state), alone and batched: the same decision matrices,
    qualification and mpk as the plain stepping (dkg_ctx_set_stepping 3), and the tampered dealers'
    rows equal the oracle's per-pair MSM checks (committee.rs:287-305, 532-548)."""
    h = be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes([n]) * 32, 6, 0, n, t)
    E, A, s, sp = (bytearray(x) for x in be.share_gen(a, b, n, n, t))
    _inject(random.Random(n + 17), n, t, E, A, s, sp)
    N = t + 1
    for d, buf in ((7, E), (9, A)):  # identity rows (committee.rs:1127 style)
        buf[32 * N * d:32 * N * (d + 1)] = bytes(32 * N)
    out = []
    try:
        for mode in (3, 0):
            be.set_stepping(mode)
            r = be.ceremony_verify(bytes(E), bytes(A), bytes(s), bytes(sp), n, t)
            assert be.last_split() == 1
            out.append((r.dec2, r.dec4, r.qualified, r.reconstruct, r.mpk, r.final_share, be.stepping_redos()))
            B = 3  # the same committee three times in one batch: column offsets of later ceremonies
            rb = dkg_amd.ceremony_batch_verify(be, B, n, t, bytes(E) * B, bytes(A) * B, bytes(s) * B,
                                               bytes(sp) * B)
            for c in range(B):
                d = rb.ceremony(c)
                assert bytes(d["dec2"]) == bytes(r.dec2) and bytes(d["dec4"]) == bytes(r.dec4), (mode, c)
    finally:
        be.set_stepping(0)
    assert out[0] == out[1][:6] + (out[0][6],)
    assert out[1][6] > 0  # the identity rows took the complete-formula redo in the repacked phases
    exp = _expected_rows(n, t, h, E, A, s, sp)
    d2, d4, q = out[1][0], out[1][1], out[1][2]
    for i in range(5):
        assert bytes(d2[i * n:(i + 1) * n]) == exp[(i, 2)], (i, "round 2")
        # round 4 of a disqualified dealer is not checked: SKIPPED (committee.rs:522)
        want4 = exp[(i, 4)] if q[i] else bytes(SELF if j == i else SKIPPED for j in range(n))
        assert bytes(d4[i * n:(i + 1) * n]) == want4, (i, "round 4")
    assert bytes(d2[7 * n:8 * n]).count(REJECT) == n - 1 and bytes(d4[9 * n:10 * n]).count(REJECT) == n - 1


def _first_diffs(x, y, n, k=8):
    """(row, column, x, y) of the first k entries where x and y differ."""
    x, y = bytes(x) if not isinstance(x, (list, tuple)) else x, bytes(y) if not isinstance(y, (list, tuple)) else y
    return [(i // n, i % n, x[i], y[i]) for i in range(min(len(x), len(y))) if x[i] != y[i]][:k]


def test_stepping_tail_repack_unsplit_n1024(be):
    """n=1024, t=511 forced unsplit runs the repack on 512-lane tables, 8 phases
    of one table per workgroup at first (grid.x = columns for P = 512 and 256): the redo flag words
    of every phase must fit the allocation (kernels.hip stepping_flag_words), or a dropped flag
    would skip the complete-formula redo of an exceptional addition.  Identity E and A rows make
    every phase's additions exceptional; the repack and the plain stepping (mode 3) must agree,
    and the tampered dealers' rows equal the oracle's per-pair MSM checks (committee.rs:287-305,
    532-548)."""
    n, t = 1024, 511
    h = be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes([77]) * 32, 6, 0, n, t)
    E, A, s, sp = (bytearray(x) for x in be.share_gen(a, b, n, n, t))
    _inject(random.Random(1024 + 17), n, t, E, A, s, sp)
    N = t + 1
    for d, buf in ((7, E), (9, A), (n - 1, E)):  # identity rows, one in the last dealer group
        buf[32 * N * d:32 * N * (d + 1)] = bytes(32 * N)
    out = []
    try:
        be.set_split(1)
        for mode in (3, 0):
            be.set_stepping(mode)
            r = be.ceremony_verify(bytes(E), bytes(A), bytes(s), bytes(sp), n, t)
            assert be.last_split() == 1
            out.append((r.dec2, r.dec4, r.qualified, r.reconstruct, r.mpk, r.final_share, be.stepping_redos()))
    finally:
        be.set_stepping(0)
        be.set_split(0)
    for k, name in enumerate(("dec2", "dec4", "qualified", "reconstruct", "mpk", "final_share")):
        same = out[0][k] == out[1][k]  # a plain bool: pytest's diff of 1-MB values takes minutes
        assert same, (name, _first_diffs(out[0][k], out[1][k], n))
    assert out[1][6] > 0
    exp = _expected_rows(n, t, h, E, A, s, sp)
    d2, d4, q = out[1][0], out[1][1], out[1][2]
    for i in range(5):
        assert bytes(d2[i * n:(i + 1) * n]) == exp[(i, 2)], (i, "round 2")
        want4 = exp[(i, 4)] if q[i] else bytes(SELF if j == i else SKIPPED for j in range(n))
        assert bytes(d4[i * n:(i + 1) * n]) == want4, (i, "round 4")
    for d, dd in ((7, d2), (9, d4), (n - 1, d2)):
        assert bytes(dd[d * n:(d + 1) * n]).count(REJECT) == n - 1, d


@pytest.mark.parametrize("n,t,split", [(1024, 511, 4), (1024, 511, 3), (1100, 549, 2), (300, 149, 1)])
def test_binomial_schedules_match_at_scale(be, n, t, split):
    """The binomial schedules (dkg_ctx_set_binomial: lane pairs for no / every / the latency-bound
    steps, the mixed m-fastest XCD-grouped item order for every / no / the many-round steps) at the
    BASELINE size and on ragged ones (n=1100 at U=2: a short last piece joining 90 steps late; n=300
    unsplit: a padded column group), with tampered dealers: identical decision matrices,
    qualification, reconstruction and mpk."""
    be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes([split + 7]) * 32, 9, 0, n, t)
    E, A, s, sp = (bytearray(x) for x in be.share_gen(a, b, n, n, t))
    _inject(random.Random(n + split), n, t, E, A, s, sp)
    out = []
    try:
        be.set_split(split)
        for mode in (1, 2, 3, 4, 0):
            be.set_binomial(mode)
            r = be.ceremony_verify(bytes(E), bytes(A), bytes(s), bytes(sp), n, t)
            assert be.last_split() == split
            out.append((r.dec2, r.dec4, r.qualified, r.reconstruct, r.mpk, r.final_share))
    finally:
        be.set_binomial(0)
        be.set_split(0)
    assert all(o == out[0] for o in out[1:])
    assert out[0][2][:5] == [0, 0, 1, 0, 0] and out[0][3][:5] == [0, 0, 1, 0, 0]


@pytest.mark.parametrize("n,t,split", [(100, 49, 0), (300, 149, 2), (1100, 549, 0), (65, 32, 3)])
def test_honest_ragged_no_stepping_redo(be, n, t, split):
    """Identity padding columns (a dealer count that is not a multiple of 64) are the identity, whose
    dedicated additions always have Z = 0: they must not mark their workgroups for the complete redo
    (runtime passes the real dealer count to k_stepping).  An honest ragged ceremony redoes nothing,
    and dkg_ctx_stepping_redos reports the last verification only (0 after a receiver-view call)."""
    be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes([n % 251]) * 32, 4, 0, n, t)
    try:
        be.set_split(split)
        r = be.ceremony(a, b, n, t)
    finally:
        be.set_split(0)
    assert r.qualified == [1] * n and r.n_qualified == n
    assert be.stepping_redos() == 0, (n, t, be.last_split())
    assert be.binomial_reruns() == 0, (n, t, be.last_split())
