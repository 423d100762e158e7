"""Parity of the HIP path (through the C ABI) with the golden fixtures and the CPU oracle.

Every test here runs the gfx950 kernels in dkg_amd/libdkg_amd.so; the oracle (tests/oracle_lib.py)
and the libsodium-generated fixtures are the checkers.  Bit-exact comparison throughout: this path
is integer arithmetic, so there is no tolerance.
"""
import random

import pytest

import dkg_amd
from dkg_amd import ACCEPT, MISSING, REJECT, SELF
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


def dec_str(raw):
    return "".join(str(x) for x in raw)


def test_env_and_commitment_key(be, golden):
    g = golden("kat_group.json")
    h = be.env_init(4, 10, CK)
    assert h.hex() == g["hash_to_group"][0]["P"]  # commitment.rs:13-17
    with pytest.raises(dkg_amd.DkgError):
        dkg_amd.Environment(be, 5, 10)  # BASELINE config 1: committee.rs:73 rejects t=5, n=10
    for e in g["hash_to_group"][1:]:
        m = H(e["msg"])
        assert be.env_init(0, 2, m).hex() == e["P"]
    be.env_init(4, 10, CK)


def test_fixed_base_generator(be, golden):
    g = golden("kat_group.json")
    ks = [e["k"].to_bytes(32, "little") for e in g["base_multiples"]] + [H(e["k"]) for e in g["base_mul"]]
    exp = [e["P"] for e in g["base_multiples"]] + [e["P"] for e in g["base_mul"]]
    out = be.fixed_base_batch(b"".join(ks))
    assert [out[32 * i:32 * i + 32].hex() for i in range(len(ks))] == exp


def test_fixed_base_other_point(be, golden):
    for e in golden("kat_group.json")["mul"]:
        assert be.fixed_base_batch(H(e["k"]), base=H(e["P"])).hex() == e["kP"]
    # the caller base's comb is cached by its bytes: repeats, alternations, and the generator and the
    # commitment key passed as explicit bases (their own combs) give the same products
    muls = golden("kat_group.json")["mul"]
    for e in muls + muls[::-1] + muls:
        assert be.fixed_base_batch(H(e["k"]), base=H(e["P"])).hex() == e["kP"]
    g = golden("kat_group.json")
    gen = bytes.fromhex("e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76")
    e = g["base_mul"][0]
    assert be.fixed_base_batch(H(e["k"]), base=gen).hex() == e["P"]
    h = be.env_init(4, 10, CK)
    k = (123456789).to_bytes(32, "little")
    assert be.fixed_base_batch(k, base=h) == bytes(O.msm(k, h))
    with pytest.raises(dkg_amd.DkgError):
        be.fixed_base_batch(k, base=b"\xff" * 32)  # does not decode
    assert be.fixed_base_batch(H(muls[0]["k"]), base=H(muls[0]["P"])).hex() == muls[0]["kP"]


def test_clock_probe_and_device_id(be):
    """bench.py's measurement aids: the shader clock under full occupancy and the PCI bus id."""
    c = be.clock_probe()
    assert 500 < c["sclk_mhz"] < 4000 and c["busy_ms"] > 0.05, c
    bus = be.pci_bus_id()
    assert len(bus.split(":")) == 3 and "." in bus, bus


def test_points_valid(be, golden):
    g = golden("kat_group.json")
    bad = b"".join(H(x) for x in g["invalid_encodings"])
    assert set(be.points_valid(bad)) == {0}
    good = b"".join(H(e["P"]) for e in g["base_multiples"])
    assert set(be.points_valid(good)) == {1}


@pytest.mark.parametrize("idx", range(10))
def test_msm_batch(be, golden, idx):
    c = golden("kat_group.json")["msm"][idx]
    N = c["N"]
    if N == 0:
        return
    assert be.msm_batch(H(c["scalars"]), H(c["points"]), 1, N).hex() == c["out"]


def test_msm_batch_many(be, golden):
    cases = [c for c in golden("kat_group.json")["msm"] if c["N"] == 32]
    sc = b"".join(H(c["scalars"]) for c in cases) * 3
    pt = b"".join(H(c["points"]) for c in cases) * 3
    out = be.msm_batch(sc, pt, 3 * len(cases), 32)
    assert [out[32 * i:32 * i + 32].hex() for i in range(3 * len(cases))] == [c["out"] for c in cases] * 3


def test_msm_decode_error(be, golden):
    bad = H(golden("kat_group.json")["invalid_encodings"][0])
    with pytest.raises(dkg_amd.DkgError) as ei:
        be.msm_batch(bytes(32), bad, 1, 1)
    assert ei.value.code == -2


def test_poly_eval(be, golden):
    s = golden("kat_scalar.json")
    kt = s["poly_tests"]
    coeffs = b"".join(c.to_bytes(32, "little") for c in kt["coeffs"])
    assert be.poly_eval_batch(coeffs, 1, 5, [kt["x"]]) == kt["value"].to_bytes(32, "little")
    for e in s["poly_eval"]:
        pts = [x for x in e["points"] if x < 2**24]
        N = len(H(e["coeffs"])) // 32
        out = be.poly_eval_batch(H(e["coeffs"]), 1, N, pts)
        exp = [v for x, v in zip(e["points"], e["values"]) if x < 2**24]
        assert [out[32 * i:32 * i + 32].hex() for i in range(len(pts))] == exp


CEREMONIES = ["ceremony_n2_t0.json", "ceremony_n3_t1.json", "ceremony_n10_t4.json",
              "ceremony_n11_t5.json", "ceremony_n16_t7.json"]
FAULTS = ["fault_e_identity_n10_t4.json", "fault_share_flip_n10_t4.json",
          "fault_a_generator_n10_t4.json", "fault_over_threshold_n10_t4.json", "fault_a_many_n10_t4.json",
          "fault_self_share_n10_t4.json", "fault_recon_only_n10_t4.json", "fault_recon_r2err_n16_t3.json",
          "fault_recon_insufficient_n16_t3.json"]


@pytest.mark.parametrize("name", CEREMONIES)
def test_share_gen(be, golden, name):
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(H(c["master_seed"]), c["ceremony"], 0, n, t)
    assert a.hex() == c["a"] and b.hex() == c["b"]
    E, A, s, sp = be.share_gen(a, b, n, n, t)
    assert E.hex() == c["E"]
    assert A.hex() == c["A"]
    assert s.hex() == c["s"]
    assert sp.hex() == c["s_prime"]


@pytest.mark.parametrize("name", CEREMONIES + FAULTS)
def test_verify_pairs(be, golden, name):
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    d2 = be.verify_pairs(n, t, 2, 0, n, H(c["E"]), H(c["s"]), H(c["s_prime"]))
    assert dec_str(d2) == c["dec2"]
    d4 = dec_str(be.verify_pairs(n, t, 4, 0, n, H(c["A"]), H(c["s"])))
    for i in range(n * n):
        if c["dec4"][i] != "3":
            assert d4[i] == c["dec4"][i], (name, i // n, i % n)
    # dealer sub-range (a sharded rank's rows)
    d0, d1 = n // 3, n - 1
    N = t + 1
    part = be.verify_pairs(n, t, 2, d0, d1, H(c["E"])[32 * N * d0:32 * N * d1],
                           H(c["s"])[32 * n * d0:32 * n * d1], H(c["s_prime"])[32 * n * d0:32 * n * d1])
    assert dec_str(part) == c["dec2"][n * d0:n * d1]


@pytest.mark.parametrize("name", ["ceremony_n16_t7.json", "fault_share_flip_n10_t4.json",
                                  "fault_e_identity_n10_t4.json"])
def test_verify_receiver(be, golden, name):
    """One party's view (what Phases<Phase1>::proceed computes for receiver j)."""
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    s, sp = H(c["s"]), H(c["s_prime"])
    for j in range(n):
        col = b"".join(s[32 * (i * n + j):32 * (i * n + j) + 32] for i in range(n))
        colp = b"".join(sp[32 * (i * n + j):32 * (i * n + j) + 32] for i in range(n))
        d = be.verify_receiver(n, t, 2, j, H(c["E"]), col, colp)
        assert dec_str(d) == "".join(c["dec2"][i * n + j] for i in range(n)), j


def _check_ceremony(c, r, n):
    assert r.E.hex() == c["E"] if r.E is not None and "a" in c else True
    assert dec_str(r.dec2) == c["dec2"]
    assert dec_str(r.dec4) == c["dec4"]
    assert r.qualified == c["qualified"]
    assert r.r2_error == [int(x) for x in c["r2_error"]]
    assert r.complaints2 == c["complaints2"]
    assert r.reconstruct == c["reconstruct"]
    assert r.r4_error == [int(x) for x in c["r4_error"]]
    assert r.phase4_error == int(c["phase4_error"])
    assert r.final_share.hex() == c["final_share"]
    assert r.public_share.hex() == c["public_share"]
    assert r.mpk.hex() == c["mpk"]


@pytest.mark.parametrize("name", CEREMONIES)
def test_ceremony_honest(be, golden, name):
    """full_valid_run (committee.rs:1518-1656): every output of every party, bit for bit."""
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(H(c["master_seed"]), c["ceremony"], 0, n, t)
    r = be.ceremony(a, b, n, t)
    assert r.E.hex() == c["E"] and r.A.hex() == c["A"]
    assert r.s.hex() == c["s"] and r.s_prime.hex() == c["s_prime"]
    _check_ceremony(c, r, n)


@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("name", FAULTS)
def test_ceremony_faults(be, golden, name, overlap):
    """misbehaving_parties / invalid_phase_2 / phase_4 style fault injection (committee.rs:1105-1313),
    with the round-4 checks overlapped with rounds 2-3 (default) and in protocol order."""
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    be.set_overlap(overlap)
    try:
        r = be.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
    finally:
        be.set_overlap(True)
    _check_ceremony(c, r, n)


def test_ceremony_n64(be, golden):
    c = golden("ceremony_n64_t31.json")
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(H(c["master_seed"]), c["ceremony"], 0, n, t)
    r = be.ceremony(a, b, n, t)
    assert r.E.hex() == c["E"] and r.A.hex() == c["A"]
    assert r.s.hex() == c["s"] and r.s_prime.hex() == c["s_prime"]
    _check_ceremony(c, r, n)


@pytest.mark.parametrize("name", ["spot_n256_t127.json", "spot_n1024_t511.json"])
def test_spot_vectors(be, golden, name):
    sp = golden(name)
    n, t = sp["n"], sp["t"]
    be.env_init(t, n, CK)
    for d in sp["dealers"]:
        i = d["dealer"]
        a, b = dkg_amd.dealer_coefficients(H(sp["master_seed"]), 0, i, 1, t)
        E, A, s, s_p = be.share_gen(a, b, 1, n, t)
        assert E.hex() == d["E"] and A.hex() == d["A"]
        for pr in d["pairs"]:
            j = pr["receiver"]
            assert s[32 * j:32 * j + 32].hex() == pr["s"] and s_p[32 * j:32 * j + 32].hex() == pr["s_prime"]
        dec = be.verify_pairs(n, t, 2, i, i + 1, E, s, s_p)
        exp = [SELF if j == i else ACCEPT for j in range(n)]
        assert list(dec) == exp
        # flip one share: exactly that pair is rejected (committee.rs:305)
        j = d["pairs"][0]["receiver"]
        bad = bytearray(s)
        bad[32 * j] ^= 1
        dec = be.verify_pairs(n, t, 2, i, i + 1, E, bytes(bad), s_p)
        assert [k for k in range(n) if dec[k] == REJECT] == ([j] if j != i else [])


def _gsum(values):
    return sum(values) % L


@pytest.mark.parametrize("n,t,split", [(256, 127, 0), (1024, 511, 0), (1024, 511, 1), (1024, 511, 3),
                                       (1024, 511, 4), (1024, 511, 6), (1024, 511, 7)])
def test_ceremony_large_properties(be, n, t, split):
    """BASELINE configs 2 and 3 at full size: size-independent properties plus oracle spot pairs,
    with the cost model's degree split (0), none (1) and forced ragged / 4-way splits."""
    be.env_init(t, n, CK)
    master = bytes([7]) * 32
    a, b = dkg_amd.dealer_coefficients(master, 3, 0, n, t)
    be.set_split(split)
    try:
        r = be.ceremony(a, b, n, t)
        if split:
            assert be.last_split() == split
    finally:
        be.set_split(0)
    N = t + 1
    # every share verifies in both rounds, nobody complains, everyone is qualified
    assert r.dec2.count(bytes([ACCEPT])) == n * (n - 1) and r.dec4.count(bytes([ACCEPT])) == n * (n - 1)
    assert r.qualified == [1] * n and r.complaints2 == [0] * n
    # mpk == g * sum_i a_i0  (committee.rs:1633-1647)
    secret = _gsum(int.from_bytes(a[32 * N * i:32 * N * i + 32], "little") for i in range(n))
    assert r.mpk == O.base_mul(secret.to_bytes(32, "little"))
    # final share j == sum_i s_ij and mpk == g * Lagrange(t+1 final shares)
    fs = [int.from_bytes(r.final_share[32 * j:32 * j + 32], "little") for j in range(n)]
    rng = random.Random(n)
    for j in rng.sample(range(n), 3):
        assert fs[j] == _gsum(int.from_bytes(r.s[32 * (i * n + j):32 * (i * n + j) + 32], "little")
                              for i in range(n))
    xs = rng.sample(range(1, n + 1), t + 1)
    lag = 0
    for xa in xs:
        coef = 1
        for xb in xs:
            if xb != xa:
                coef = coef * (-xb) * pow(xa - xb, -1, L) % L
        lag = (lag + coef * fs[xa - 1]) % L
    assert lag == secret
    # oracle: a few (dealer, receiver) pairs recomputed the reference's way (vartime MSM)
    for _ in range(3):
        i, j = rng.randrange(n), rng.randrange(n)
        if i == j:
            continue
        acc, _rc = O.verify_pairs(n, t, 2, r.E, be.h, r.s, r.s_prime, i, i + 1, j, j + 1)
        assert acc[0] == 1
    # commitments of a sampled dealer re-derived by the oracle
    i = rng.randrange(n)
    E, A, s, sp = O.share_gen(1, n, t, a[32 * N * i:32 * N * (i + 1)], b[32 * N * i:32 * N * (i + 1)], be.h)
    assert E == r.E[32 * N * i:32 * N * (i + 1)] and A == r.A[32 * N * i:32 * N * (i + 1)]
    assert s == r.s[32 * n * i:32 * n * (i + 1)] and sp == r.s_prime[32 * n * i:32 * n * (i + 1)]


@pytest.mark.parametrize("n,t", [(200, 99), (512, 255)])
@pytest.mark.parametrize("round_", [2, 4])
def test_chunked_streams_identical(be, round_, n, t):
    """Dealer chunks on 1..8 HIP streams (dkg_ctx_set_streams) give identical decisions, with
    flipped shares and one undecodable dealer.  n=200 (ragged: not a multiple of 64) is below both
    chunk gates of verify_device (runtime.hip: saturating binomial, W*L*n >= 5e7 lane-steps) and
    runs one pipeline whatever nsub; n=512 (6.7e7 lane-steps) takes the chunked path for nsub > 1."""
    N = t + 1
    be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes([9]) * 32, 1, 0, n, t)
    E, A, s, sp = be.share_gen(a, b, n, n, t)
    C = bytearray(E if round_ == 2 else A)
    s = bytearray(s)
    rng = random.Random(round_ * 1000 + n)
    flips = {(rng.randrange(n), rng.randrange(n)) for _ in range(40)}
    for i, j in flips:
        s[32 * (i * n + j) + 5] ^= 0x10
    bad_dealer = 137
    C[32 * (N * bad_dealer + 3) + 31] |= 0x80  # bit 255 set: does not decode (groups.rs:78-81)
    exp = bytearray(ACCEPT for _ in range(n * n))
    for i, j in flips:
        exp[i * n + j] = REJECT
    for j in range(n):  # no decodable broadcast: MISSING in round 2 (no complaint), REJECT in round 4
        exp[bad_dealer * n + j] = MISSING if round_ == 2 else REJECT
    for i in range(n):
        exp[i * n + i] = SELF
    try:
        for nsub in (1, 3, 8):
            be.set_streams(nsub)
            d = be.verify_pairs(n, t, round_, 0, n, bytes(C), bytes(s), sp if round_ == 2 else None)
            assert bytes(d) == bytes(exp), nsub
    finally:
        be.set_streams(2)


def _check_played(p, c, n, ws):
    """A played sharded run (tests/shard_play.py) against a golden ceremony, and the library's combine
    against the checker's rules (tests/combine_ref.py) on the same gathered rows."""
    from tests import combine_ref as CR

    assert dec_str(p.dec2) == c["dec2"]
    assert dec_str(p.dec4) == c["dec4"]
    o = p.outcome
    assert o.qualified == c["qualified"] and o.reconstruct == c["reconstruct"]
    assert o.complaints2 == c["complaints2"]
    assert o.r2_error == [int(x) for x in c["r2_error"]]
    assert o.r4_error == [int(x) for x in c["r4_error"]]
    assert o.phase4_error == c["phase4_error"] and o.n_qualified == sum(c["qualified"])
    ref = CR.combine(p.dec2, p.raw4, n, int(c["t"]))
    assert ref.qualified.tolist() == o.qualified and ref.reconstruct.tolist() == o.reconstruct
    assert ref.r4_error.tolist() == o.r4_error and bytes(ref.dec4) == p.dec4
    assert p.final_share.hex() == c["final_share"]
    assert p.public_share.hex() == c["public_share"]
    # Phases<Phase4>::proceed fails for everyone without a master key (committee.rs:673-677): zero
    assert p.mpk.hex() == c["mpk"]


@pytest.mark.parametrize("name,ws", [("ceremony_n16_t7.json", 2), ("ceremony_n64_t31.json", 3),
                                     ("ceremony_n11_t5.json", 4)])
def test_sharded_ceremony_matches_golden(be, golden, name, ws):
    """dkg_ceremony_shard_device for every rank of a ws-way dealer split (played in one process), the
    gathered padded blocks, and the library's combine and finalise (dkg_shard_combine_device,
    dkg_shard_finalise_device) reproduce the single-GPU golden ceremony bit for bit."""
    import torch

    from tests import shard_play

    c = golden(name)
    n, t = c["n"], c["t"]
    N = t + 1
    be.env_init(t, n, CK)
    dev = torch.device("cuda", 0)
    a, b = dkg_amd.dealer_coefficients(H(c["master_seed"]), c["ceremony"], 0, n, t)
    keep = []

    def call(r, d0, d1, o2, o4, oA, op):
        ta = torch.frombuffer(bytearray(a[32 * N * d0:32 * N * d1] or b"\0"), dtype=torch.uint8).to(dev)
        tb = torch.frombuffer(bytearray(b[32 * N * d0:32 * N * d1] or b"\0"), dtype=torch.uint8).to(dev)
        keep.extend((ta, tb))
        be.ceremony_shard_device(n, t, d0, d1, ta.data_ptr(), tb.data_ptr(), o2.data_ptr(), o4.data_ptr(),
                                 oA.data_ptr(), op.data_ptr())
        return None

    p = shard_play.play(be, n, t, ws, call, dev)
    _check_played(p, c, n, ws)


@pytest.mark.parametrize("ws", [1, 2, 3])
@pytest.mark.parametrize("name", FAULTS + ["ceremony_n16_t7.json"])
def test_sharded_verify_faults(be, golden, name, ws):
    """dkg_ceremony_shard_verify_device on the fixtures' broadcasts (faulty commitments / shares):
    every rank's rows, the library's combine, the reconstruction of a dealer accused in round 4 on its
    owning rank (fault_a_generator: committee.rs:660-670, 747-783) and the library's finalise give the
    single-GPU golden decisions, final shares, public shares and mpk bit for bit."""
    import torch

    from tests import shard_play

    c = golden(name)
    n, t = c["n"], c["t"]
    N = t + 1
    be.env_init(t, n, CK)
    dev = torch.device("cuda", 0)
    E, A, s, sp = (H(c[k]) for k in ("E", "A", "s", "s_prime"))
    keep = []

    def put(x):
        v = torch.frombuffer(bytearray(x or b"\0"), dtype=torch.uint8).to(dev)
        keep.append(v)
        return v

    def call(r, d0, d1, o2, o4, oA, op):
        tE, tA = put(E[32 * N * d0:32 * N * d1]), put(A[32 * N * d0:32 * N * d1])
        ts, tsp = put(s[32 * n * d0:32 * n * d1]), put(sp[32 * n * d0:32 * n * d1])
        be.ceremony_shard_verify_device(n, t, d0, d1, tE.data_ptr(), tA.data_ptr(), ts.data_ptr(), tsp.data_ptr(),
                                        o2.data_ptr(), o4.data_ptr(), oA.data_ptr(), op.data_ptr())
        return ts

    p = shard_play.play(be, n, t, ws, call, dev)
    _check_played(p, c, n, ws)


@pytest.mark.parametrize("seed", range(12))
def test_shard_combine_random_matrices(be, seed):
    """dkg_shard_combine_device against the checker's rules (tests/combine_ref.py) on random decision
    matrices in the padded gather layout: random REJECT densities (from none to over-threshold
    columns), MISSING rows, random round-4 accusations (including rows of disqualified dealers, which
    the combine must turn SKIPPED) and ragged rank partitions (ws up to 8, n not a multiple of ws)."""
    import numpy as np
    import torch

    from tests import combine_ref as CR

    rng = np.random.default_rng(seed)
    n = int(rng.choice([3, 10, 33, 64, 257, 1024]))
    t = int(rng.integers(0, (n + 1) // 2))
    if 2 * t >= n + 1:
        t = (n - 1) // 2
    ws = int(rng.choice([w for w in (1, 2, 3, 5, 8) if w <= n]))
    p2, p4 = float(rng.choice([0.0, 0.001, 0.02, 0.3])), float(rng.choice([0.0, 0.002, 0.05, 0.5]))
    dec2 = np.where(rng.random((n, n)) < p2, REJECT, ACCEPT).astype(np.uint8)
    for i in rng.choice(n, size=int(rng.integers(0, 4)), replace=False) if n > 3 else []:
        dec2[i, :] = MISSING
    dec4 = np.where(rng.random((n, n)) < p4, REJECT, ACCEPT).astype(np.uint8)
    np.fill_diagonal(dec2, SELF)
    np.fill_diagonal(dec4, SELF)
    be.env_init(t, n, CK)
    dev = torch.device("cuda", 0)
    g2 = torch.from_numpy(CR.pad(dec2, ws, n, n)).to(dev)
    g4 = torch.from_numpy(CR.pad(dec4, ws, n, n)).to(dev)
    c2 = torch.empty(n * n, dtype=torch.uint8, device=dev)
    c4 = torch.empty_like(c2)
    o = be.shard_combine_device(n, t, ws, g2.data_ptr(), g4.data_ptr(), c2.data_ptr(), c4.data_ptr())
    ref = CR.combine(dec2, dec4, n, t)
    ctx = (seed, n, t, ws, p2, p4)
    assert bytes(c2.cpu().numpy()) == bytes(dec2), ctx
    assert bytes(c4.cpu().numpy()) == bytes(ref.dec4), ctx
    assert o.qualified == ref.qualified.tolist(), ctx
    assert o.complaints2 == ref.complaints2.tolist(), ctx
    assert o.r2_error == ref.r2_error.tolist(), ctx
    assert o.reconstruct == ref.reconstruct.tolist(), ctx
    assert o.r4_error == ref.r4_error.tolist(), ctx
    assert o.phase4_error == ref.phase4_error and o.n_qualified == int(ref.qualified.sum()), ctx
    # the optional compacted outputs may be omitted
    o2 = be.shard_combine_device(n, t, ws, g2.data_ptr(), g4.data_ptr())
    assert (o2.qualified, o2.reconstruct, o2.r4_error) == (o.qualified, o.reconstruct, o.r4_error)


def _check_batch_member(c, d, n):
    """One ceremony of a BatchResult against its golden file (same fields as _check_ceremony)."""
    assert dec_str(d["dec2"]) == c["dec2"]
    assert dec_str(d["dec4"]) == c["dec4"]
    assert d["qualified"] == c["qualified"]
    assert d["r2_error"] == [int(x) for x in c["r2_error"]]
    assert d["complaints2"] == c["complaints2"]
    assert d["reconstruct"] == c["reconstruct"]
    assert d["r4_error"] == [int(x) for x in c["r4_error"]]
    assert d["phase4_error"] == int(c["phase4_error"])
    assert d["final_share"].hex() == c["final_share"]
    assert d["public_share"].hex() == c["public_share"]
    assert d["mpk"].hex() == c["mpk"]


@pytest.mark.parametrize("overlap", [True, False])
def test_batch_verify_goldens(be, golden, overlap):
    """BASELINE config 5 path: five n=10, t=4 ceremonies (one honest, four with the fault injections
    of committee.rs:1105-1313) verified as ONE batch give each golden ceremony's outputs bit for bit."""
    names = ["ceremony_n10_t4.json"] + [x for x in FAULTS if "_n10_t4" in x]
    cs = [golden(x) for x in names]
    n, t = 10, 4
    assert all((c["n"], c["t"]) == (n, t) for c in cs)
    be.env_init(t, n, CK)
    E = b"".join(H(c["E"]) for c in cs)
    A = b"".join(H(c["A"]) for c in cs)
    s = b"".join(H(c["s"]) for c in cs)
    sp = b"".join(H(c["s_prime"]) for c in cs)
    be.set_overlap(overlap)
    try:
        r = dkg_amd.ceremony_batch_verify(be, len(cs), n, t, E, A, s, sp)
    finally:
        be.set_overlap(True)
    for k, c in enumerate(cs):
        _check_batch_member(c, r.ceremony(k), n)


@pytest.mark.parametrize("name", FAULTS + ["ceremony_n64_t31.json", "ceremony_n11_t5.json"])
def test_check_split_combs_goldens(be, golden, name):
    """The fused round-2/4 check as two launches, one per fixed-base comb (dkg_ctx_set_check 1: g*s
    parked in device memory between them), unsplit and split tables, one and two chunk streams,
    alone and batched: every output bit-exact against the fixture (committee.rs:287-305, 532-548)."""
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    try:
        be.set_check(1)
        for pieces, streams in ((1, 2), (min(3, t + 1), 1), (0, 2)):
            be.set_split(pieces)
            be.set_streams(streams)
            r = be.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
            _check_ceremony(c, r, n)
        rb = dkg_amd.ceremony_batch_verify(be, 3, n, t, *(H(c[k]) * 3 for k in ("E", "A", "s", "s_prime")))
        for k in range(3):
            _check_batch_member(c, rb.ceremony(k), n)
    finally:
        be.set_check(0)
        be.set_split(0)
        be.set_streams(2)


def test_batch_verify_disclosure_goldens(be, golden):
    """Final parties with round-2 errors never disclose in phase 5 (committee.rs:340-347, 684): a batch
    of the n=16, t=3 fixtures in which they leave exactly t disclosures (a wrong recovered secret, as
    the reference) and fewer (no mpk) -- each member equals its golden ceremony bit for bit."""
    names = ["fault_recon_r2err_n16_t3.json", "fault_recon_insufficient_n16_t3.json", "fault_recon_r2err_n16_t3.json"]
    cs = [golden(x) for x in names]
    n, t = 16, 3
    be.env_init(t, n, CK)
    r = dkg_amd.ceremony_batch_verify(be, len(cs), n, t, *(b"".join(H(c[k]) for c in cs)
                                                          for k in ("E", "A", "s", "s_prime")))
    for k, c in enumerate(cs):
        _check_batch_member(c, r.ceremony(k), n)
    assert r.mpk[1] == bytes(32) and r.mpk[0] == r.mpk[2] != bytes(32)


def test_batch_device_matches_single(be, golden):
    """Honest batch from device coefficients (dkg_ceremony_batch_device) = the golden n=16 ceremony
    plus independent ceremonies each re-run alone through dkg_ceremony_run."""
    import torch

    c0 = golden("ceremony_n16_t7.json")
    n, t = c0["n"], c0["t"]
    N = t + 1
    be.env_init(t, n, CK)
    seeds = [(H(c0["master_seed"]), c0["ceremony"])] + [(bytes([7 + k]) * 32, 100 + k) for k in range(4)]
    coeffs = [dkg_amd.dealer_coefficients(m, cid, 0, n, t) for m, cid in seeds]
    dev = torch.device("cuda", 0)
    ta = torch.frombuffer(bytearray(b"".join(a for a, _ in coeffs)), dtype=torch.uint8).to(dev)
    tb = torch.frombuffer(bytearray(b"".join(b for _, b in coeffs)), dtype=torch.uint8).to(dev)
    r = dkg_amd.ceremony_batch_device(be, len(seeds), n, t, ta.data_ptr(), tb.data_ptr(), big=True)
    _check_batch_member(c0, r.ceremony(0), n)
    for k, (a, b) in enumerate(coeffs[1:], start=1):
        single = be.ceremony(a, b, n, t)
        d = r.ceremony(k)
        assert d["mpk"] == single.mpk and d["final_share"] == single.final_share
        assert d["public_share"] == single.public_share and d["dec2"] == single.dec2 and d["dec4"] == single.dec4
        assert d["qualified"] == single.qualified and d["n_qualified"] == n
        secret = sum(int.from_bytes(a[32 * N * i:32 * N * i + 32], "little") for i in range(n)) % L
        assert d["mpk"] == O.base_mul(secret.to_bytes(32, "little"))
    assert r.ms["total"] > 0


@pytest.mark.parametrize("c0,B,d0,D,t", [(0, 1, 0, 10, 4), (5, 3, 2, 7, 31), (9, 2, 0, 3, 0), (1, 1, 100, 5, 511)])
def test_dealer_coefficients_device(be, c0, B, d0, D, t):
    """On-device seeded coefficients are bit-identical to the host convention."""
    import torch

    N = t + 1
    master = bytes(range(32))
    dev = torch.device("cuda", 0)
    ta = torch.zeros(B * D * N * 32, dtype=torch.uint8, device=dev)
    tb = torch.zeros_like(ta)
    be.dealer_coefficients_device(master, c0, B, d0, D, t, ta.data_ptr(), tb.data_ptr())
    ga, gb = bytes(ta.cpu().numpy()), bytes(tb.cpu().numpy())
    for c in range(B):
        a, b = dkg_amd.dealer_coefficients(master, c0 + c, d0, D, t)
        assert ga[32 * N * D * c:32 * N * D * (c + 1)] == a
        assert gb[32 * N * D * c:32 * N * D * (c + 1)] == b


@pytest.mark.parametrize("overlap", [True, False])
def test_ceremony_undecodable_broadcast(be, golden, overlap):
    """A dealer whose round-1 broadcast does not decode (CompressedRistretto::decompress -> None,
    groups.rs:78-81) is missing data: disqualified by everyone WITHOUT a complaint
    (committee.rs:331-335), so complaints / r2 errors stay as in the honest run; its round-4 row is
    SKIPPED and it drops out of the final shares and the master key."""
    c = golden("ceremony_n10_t4.json")
    n, t = c["n"], c["t"]
    N = t + 1
    be.env_init(t, n, CK)
    bad = 3
    E = bytearray(H(c["E"]))
    E[32 * (N * bad + 2) + 31] |= 0x80  # bit 255 set: not a canonical encoding
    be.set_overlap(overlap)
    try:
        r = be.ceremony_verify(bytes(E), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
    finally:
        be.set_overlap(True)
    assert [r.dec2[bad * n + j] for j in range(n)] == [SELF if j == bad else MISSING for j in range(n)]
    assert r.complaints2 == c["complaints2"] == [0] * n and r.r2_error == [0] * n
    assert r.qualified == [0 if i == bad else 1 for i in range(n)]
    assert [r.dec4[bad * n + j] for j in range(n)] == [SELF if j == bad else 3 for j in range(n)]
    s = H(c["s"])
    a = H(c["a"])
    fs = b"".join((sum(int.from_bytes(s[32 * (i * n + j):32 * (i * n + j) + 32], "little")
                       for i in range(n) if i != bad) % L).to_bytes(32, "little") for j in range(n))
    assert r.final_share == fs
    secret = sum(int.from_bytes(a[32 * N * i:32 * N * i + 32], "little") for i in range(n) if i != bad) % L
    assert r.mpk == O.base_mul(secret.to_bytes(32, "little"))


# ---------------- full (encrypted-share) mode: elgamal.rs / procedure_keys.rs ----------------
FULL = ["full_n4_t1.json", "full_n10_t4.json", "full_faults_n10_t4.json"]


def test_member_keys_golden(be, golden):
    """Seeded member keys sorted by public key (committee.rs:134-135) as in the fixtures."""
    for name in ("full_n4_t1.json", "full_n10_t4.json"):
        c = golden(name)
        sk, pk = be.member_keys(H(c["master_seed"]), c["ceremony"], c["n"])
        assert sk.hex() == c["member_sk"] and pk.hex() == c["member_pk"]


def test_hybrid_kat_device(be, golden):
    """Device encryption / decryption of the libsodium hybrid vectors (elgamal.rs:134-193): each KAT
    is a 1-dealer x 1-recipient batch whose two ciphertexts carry msg (w = 0) and msg reversed (w = 1)."""
    k = golden("kat_hybrid.json")
    for c in k["hybrid"]:
        msg = H(c["msg"])
        if int.from_bytes(msg, "little") >= L:
            continue  # the share arrays hold canonical scalars
        r = H(c["r"]) * 2
        e1, ct = be.encrypt_shares(H(c["pk"]), msg, msg, r, 1, 1)
        assert e1[:32].hex() == c["e1"] and ct[:32].hex() == c["e2"]
        assert e1[32:] == e1[:32] and ct[32:] == ct[:32]
        s, sp, ok = be.decrypt_shares(H(c["sk"]), e1, ct, 1, 1)
        assert s == msg and sp == msg and ok == b"\x01\x01"


@pytest.mark.parametrize("name", FULL)
def test_full_mode_verify_golden(be, golden, name):
    """Receivers decrypt the (possibly tampered) golden ciphertexts on the GPU and run rounds 2-5:
    every output bit for bit, including the complaints raised by tampered ciphertexts."""
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    r = be.ceremony_verify_full(H(c["E"]), H(c["A"]), H(c["e1"]), H(c["ct"]), H(c["member_sk"]), n, t)
    assert r.s.hex() == c["s"] and r.s_prime.hex() == c["s_prime"]
    _check_ceremony(c, r, n)


@pytest.mark.parametrize("name", ["full_n4_t1.json", "full_n10_t4.json"])
def test_full_mode_device_ceremony(be, golden, name):
    """Whole full-mode ceremony on the device from seeded coefficients, encryption randomness and
    member keys; the ciphertexts the device produced decrypt (on the oracle) to the golden shares."""
    import torch

    c = golden(name)
    n, t = c["n"], c["t"]
    N = t + 1
    be.env_init(t, n, CK)
    master = H(c["master_seed"])
    dev = torch.device("cuda", 0)
    ta = torch.empty(32 * n * N, dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    tr = torch.empty(64 * n * n, dtype=torch.uint8, device=dev)
    be.dealer_coefficients_device(master, c["ceremony"], 1, 0, n, t, ta.data_ptr(), tb.data_ptr())
    be.enc_randomness_device(master, c["ceremony"], 1, 0, n, n, t, tr.data_ptr())
    assert bytes(tr.cpu().numpy()).hex() == c["enc_r"]
    sk, pk = be.member_keys(master, c["ceremony"], n)
    r = be.ceremony_full_device(ta.data_ptr(), tb.data_ptr(), tr.data_ptr(), sk, pk, n, t)
    assert r.mpk.hex() == c["mpk"] and r.qualified == c["qualified"] and r.n_qualified == n
    # the host-buffer encryption entry point reproduces the golden wire ciphertexts
    e1, ct = be.encrypt_shares(pk, H(c["s"]), H(c["s_prime"]), H(c["enc_r"]), n, n)
    assert e1.hex() == c["e1"] and ct.hex() == c["ct"]


def test_full_mode_key_tables_follow_the_keys(be):
    """The member keys' comb tables are kept across full-mode ceremonies and rebuilt when the keys
    change (compared byte for byte): three ceremonies of the same size with keys A, B, A must each
    decrypt their own ciphertexts -- stale tables would encrypt to the previous keys and every
    receiver would reject."""
    import torch

    n, t = 16, 7
    N = t + 1
    be.env_init(t, n, CK)
    dev = torch.device("cuda", 0)
    ta = torch.empty(32 * n * N, dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    tr = torch.empty(64 * n * n, dtype=torch.uint8, device=dev)
    be.dealer_coefficients_device(b"\x11" * 32, 0, 1, 0, n, t, ta.data_ptr(), tb.data_ptr())
    be.enc_randomness_device(b"\x11" * 32, 0, 1, 0, n, n, t, tr.data_ptr())
    keys = [be.member_keys(m, 0, n) for m in (b"\x21" * 32, b"\x22" * 32)]
    mpks = []
    for sk, pk in (keys[0], keys[1], keys[0]):
        r = be.ceremony_full_device(ta.data_ptr(), tb.data_ptr(), tr.data_ptr(), sk, pk, n, t)
        assert r.n_qualified == n and r.qualified == [1] * n
        mpks.append(r.mpk)
    assert mpks[0] == mpks[1] == mpks[2]  # the same coefficients: the same master key


def test_full_mode_oracle_random(be):
    """Random keys / messages / randomness: device encryption equals the CPU oracle's, and device
    decryption inverts it (a wrong key does not)."""
    rng = random.Random(11)
    D, n = 3, 5
    sks = [rng.randrange(1, L).to_bytes(32, "little") for _ in range(n)]
    pks = [O.base_mul(k) for k in sks]
    s = b"".join(rng.randrange(L).to_bytes(32, "little") for _ in range(D * n))
    sp = b"".join(rng.randrange(L).to_bytes(32, "little") for _ in range(D * n))
    r = b"".join(rng.randrange(L).to_bytes(32, "little") for _ in range(2 * D * n))
    e1, ct = be.encrypt_shares(b"".join(pks), s, sp, r, D, n)
    for i in range(D):
        for q in range(n):
            for w, msg in ((0, sp), (1, s)):
                k = 2 * (i * n + q) + w
                oe1, oct_ = O.hybrid_encrypt(pks[q], r[32 * k:32 * k + 32], msg[32 * (i * n + q):32 * (i * n + q) + 32])
                assert (oe1, oct_) == (e1[32 * k:32 * k + 32], ct[32 * k:32 * k + 32])
    ds, dsp, ok = be.decrypt_shares(b"".join(sks), e1, ct, D, n)
    assert ds == s and dsp == sp and set(ok) == {1}
    wrong = b"".join(sks[1:] + sks[:1])
    ds2, _, _ = be.decrypt_shares(wrong, e1, ct, D, n)
    assert ds2 != s


def test_full_mode_decryption_slices(be):
    """The width-4 decryption runs in recipient slices of at most 16,384 waves (one 40-KB odd-multiple
    table slot per wave of a launch, reused by the next slice): at D=1100, n=512 that is two launches
    (455 + 57 recipients).  Every one of the 1.1 M items decrypts to its plaintext, and a sample of
    ciphertexts equals the CPU oracle's (elgamal.rs:134-193)."""
    rng = random.Random(12)
    D, n = 1100, 512
    sks = [rng.randrange(1, L).to_bytes(32, "little") for _ in range(n)]
    pks = be.fixed_base_batch(b"".join(sks))
    s = b"".join(rng.randrange(L).to_bytes(32, "little") for _ in range(D * n))
    sp = b"".join(rng.randrange(L).to_bytes(32, "little") for _ in range(D * n))
    r = b"".join(rng.randrange(L).to_bytes(32, "little") for _ in range(2 * D * n))
    e1, ct = be.encrypt_shares(pks, s, sp, r, D, n)
    for i, q, w in [(0, 0, 0), (D - 1, n - 1, 1), (700, 455, 1), (3, 454, 0)] + \
            [(rng.randrange(D), rng.randrange(n), rng.randrange(2)) for _ in range(4)]:
        k = 2 * (i * n + q) + w
        msg = (sp, s)[w][32 * (i * n + q):32 * (i * n + q) + 32]
        assert O.hybrid_encrypt(pks[32 * q:32 * q + 32], r[32 * k:32 * k + 32], msg) == \
            (e1[32 * k:32 * k + 32], ct[32 * k:32 * k + 32]), (i, q, w)
    ds, dsp, ok = be.decrypt_shares(b"".join(sks), e1, ct, D, n)
    assert ds == s and dsp == sp and set(ok) == {1}


def test_complaint_proofs_device(be, golden):
    """SURVEY 8 f2 through the ABI, all complaints of a kind in one batched call: proofs of
    misbehaviour byte for byte (broadcast.rs:189-226), round-1 verdicts incl. the swapped-role quirk
    (:50-99, 271-274) and round-3 verdicts incl. forged claims (:105-135), as in the fixtures."""
    from tests.test_oracle import VERDICT, _complaint_inputs
    c = golden("complaints_n10_t4.json")
    full = golden(c["source"])
    assert full["h"] == be.env_init(full["t"], full["n"], CK).hex()
    rows = [_complaint_inputs(c, full, x) for x in c["round1"]]
    sk, pk, enc, E, proof = (b"".join(r[k] for r in rows) for k in range(5))
    w = b"".join(H(v) for x in c["round1"] for v in x["w"])
    got = be.misbehaviour_prove(sk, enc, w)
    for b, x in enumerate(c["round1"]):
        if x["verdict"] != "InvalidProofOfMisbehaviour":
            assert got[192 * b:192 * b + 192] == proof[192 * b:192 * b + 192], x
    res = be.complaint1_verify(full["t"], [x["accuser"] for x in c["round1"]], pk, enc, E, proof)
    assert res == [VERDICT[x["verdict"]] for x in c["round1"]]
    # an undecodable key in the proof is a decode failure, not a verdict
    bad = bytearray(proof[:192])
    bad[0:32] = b"\xff" * 32
    assert be.complaint1_verify(full["t"], [c["round1"][0]["accuser"]], pk[:32], enc[:128], E[:32 * (full["t"] + 1)],
                                bytes(bad)) == [-1]
    p3 = golden(c["round3_source"])
    N = p3["t"] + 1
    assert p3["h"] == be.env_init(p3["t"], p3["n"], CK).hex()
    r3 = c["round3"]
    Eb, Ab = H(p3["E"]), H(p3["A"])
    Es = b"".join(Eb[32 * N * (x["accused"] - 1):32 * N * x["accused"]] for x in r3)
    As = b"".join(Ab[32 * N * (x["accused"] - 1):32 * N * x["accused"]] for x in r3)
    res = be.complaint3_verify(p3["t"], [x["accuser"] for x in r3], b"".join(H(x["share"]) for x in r3),
                               b"".join(H(x["randomness"]) for x in r3), Es, As)
    assert res == [VERDICT[x["verdict"]] for x in r3]
    assert be.misbehaviour_prove(b"", b"", b"") == b""


def test_ceremony_from_broadcasts(be, golden):
    """a committee's broadcasts through the intake (dkg_amd.broadcast) and
    dkg_ceremony_verify_fetched.  Dealers 3 and 7 send no / a malformed phase-1 broadcast (MISSING,
    disqualified without complaints, committee.rs:331-335); dealers 5 and 10 send no / a malformed
    phase-3 broadcast (accused by everyone, :549-555, and reconstructed).  The expected outputs are
    restated here from the reference's rules on the fixture's values."""
    from dkg_amd.broadcast import BroadcastPhase1, BroadcastPhase3, verify_broadcasts
    from tests.test_broadcast import committee_broadcasts

    c = golden("ceremony_n10_t4.json")
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    p1, p3 = committee_broadcasts(c)
    p1[2] = None
    p1[6] = BroadcastPhase1(p1[6].committed_coefficients[:t], p1[6].encrypted_shares)
    p3[4] = None
    p3[9] = BroadcastPhase3(p3[9].committed_coefficients + p3[9].committed_coefficients[:1])
    for overlap in (True, False):
        be.set_overlap(overlap)
        r = verify_broadcasts(be, n, t, p1, p3)
        miss, acc = {2, 6}, {4, 9}
        exp2 = [[2 if i == j else (MISSING if i in miss else ACCEPT) for j in range(n)] for i in range(n)]
        exp4 = [[2 if i == j else (3 if i in miss else (REJECT if i in acc else ACCEPT)) for j in range(n)]
                for i in range(n)]
        assert list(r.dec2) == [x for row in exp2 for x in row]
        assert list(r.dec4) == [x for row in exp4 for x in row]
        qualified = [int(i not in miss) for i in range(n)]
        assert r.qualified == qualified and r.complaints2 == [0] * n and r.r2_error == [0] * n
        assert r.reconstruct == [int(i in acc) for i in range(n)]
        honest4 = [1 + sum(1 for i in range(n) if i != j and exp4[i][j] == ACCEPT) for j in range(n)]
        assert r.r4_error == [int(h < t + 1) for h in honest4] and r.phase4_error == 0
        s, a = H(c["s"]), H(c["a"])
        fs = [sum(int.from_bytes(s[32 * (i * n + j):32 * (i * n + j + 1)], "little") for i in range(n) if qualified[i]) % L
              for j in range(n)]
        assert r.final_share == b"".join(x.to_bytes(32, "little") for x in fs)
        sec = sum(int.from_bytes(a[32 * (t + 1) * i:32 * (t + 1) * i + 32], "little") for i in range(n) if qualified[i]) % L
        assert r.mpk == O.base_mul(sec.to_bytes(32, "little"))  # committee.rs:1633-1647 property
    be.set_overlap(True)


@pytest.mark.parametrize("pieces", [2, 3, 4, 5])
@pytest.mark.parametrize("name", FAULTS + ["ceremony_n16_t7.json", "ceremony_n11_t5.json"])
def test_degree_split_goldens(be, golden, name, pieces):
    """The degree-split evaluation (P = sum_u x^(uL) Q_u, recombined per receiver by k_combine) forced
    on the fixtures, fused and in protocol order, including ragged pieces (t+1 not a multiple of U)
    and pieces of one coefficient: every output bit-exact."""
    c = golden(name)
    n, t = c["n"], c["t"]
    if pieces > t + 1:
        pytest.skip("more pieces than coefficients")
    be.env_init(t, n, CK)
    try:
        be.set_split(pieces)
        for overlap in (True, False):
            be.set_overlap(overlap)
            r = be.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
            assert be.last_split() == pieces
            _check_ceremony(c, r, n)
    finally:
        be.set_split(0)
        be.set_overlap(True)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("name", FAULTS + ["ceremony_n16_t7.json", "ceremony_n64_t31.json"])
def test_field_modes_goldens(be, golden, name, mode):
    """Both copies of the verification kernels (dkgk: product-scanning field multiplication, dkgk_ilp:
    column sums; dkg_ctx_set_field_mode) forced for every launch, with and without a degree split:
    every output bit-exact against the fixture."""
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    try:
        be.set_field_mode(mode)
        for pieces in (1, min(3, t + 1)):
            be.set_split(pieces)
            r = be.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
            _check_ceremony(c, r, n)
    finally:
        be.set_field_mode(0)
        be.set_split(0)


@pytest.mark.parametrize("field", [1, 2])
@pytest.mark.parametrize("name", FAULTS + ["ceremony_n64_t31.json", "ceremony_n16_t7.json", "ceremony_n3_t1.json"])
def test_binomial_schedules_goldens(be, golden, name, field):
    """The schedules of the binomial-basis Horner (dkg_ctx_set_binomial): one launch per step with
    lane pairs (k_binom_pair) for the latency-bound steps or for every step or none, and the mixed
    (m-fastest, XCD-grouped) item order for every step or none, in both field-multiplication copies,
    with and without a degree split (short last pieces included), one and two chunk streams: every
    output bit-exact against the fixture."""
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    try:
        be.set_field_mode(field)
        # default; no lane pairs; lane pairs for every step; per step as default; per wave; per wave
        # with the operands prefetched one item ahead
        for mode in (0, 1, 2, 3, 4, 5):
            be.set_binomial(mode)
            for pieces, streams in ((1, 2), (min(3, t + 1), 1), (min(2, t + 1), 2)):
                be.set_split(pieces)
                be.set_streams(streams)
                r = be.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
                _check_ceremony(c, r, n)
    finally:
        be.set_field_mode(0)
        be.set_binomial(0)
        be.set_split(0)
        be.set_streams(2)


@pytest.mark.parametrize("field", [1, 2])
def test_binomial_dedicated_redo(be, golden, field):
    """The per-wave binomial's dedicated additions (runtime.hip DKG_BINOM_WAVE_DED) meet Z = 0 on a
    dealer whose commitments are all the identity (the fault of committee.rs:1127): e_{m-1} + e_m of
    two identities gives the all-zero quadruple, which the projective equality test would find equal
    to ANY point -- a false accept of that dealer's honest shares.  Its column group must be redone
    with the complete formula: every receiver rejects it (identity != g*s + h*s'), and every output
    equals the complete formula's.  The per-step schedule (mode 1; DKG_BINOM_STEP_DED=1, the default)
    marks one word instead and its driver reruns the whole verification with the complete formula --
    here through the ceremony and the dealer-shard entry point alike.  Builds without the per-wave
    redo or the rerun fail here (profiles/r05_binom_ded_ab.txt)."""
    import torch
    c = golden("ceremony_n64_t31.json")
    n, t = c["n"], c["t"]
    N = t + 1
    be.env_init(t, n, CK)
    E, A = bytearray(H(c["E"])), bytearray(H(c["A"]))
    s, sp = bytearray(H(c["s"])), bytearray(H(c["s_prime"]))
    bad = 5
    for buf in (E, A):
        buf[32 * N * bad:32 * N * (bad + 1)] = bytes(32 * N)  # the identity's encoding, every coefficient
    outs = {}
    try:
        be.set_field_mode(field)
        be.set_split(1)
        be.set_binomial(1)  # the honest broadcasts: the dedicated per-step binomial needs no rerun
        r = be.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
        _check_ceremony(c, r, n)
        assert be.binomial_reruns() == 0
        # formula 0: dedicated additions in the per-step (mode 1, no lane pairs) and the per-wave
        # (mode 4) binomial, each with its redo; formula 1: the complete formula throughout (reference)
        for formula, mode in ((0, 1), (0, 4), (1, 1)):
            be.set_stepping_formula(formula)
            be.set_binomial(mode)
            r = be.ceremony_verify(bytes(E), bytes(A), bytes(s), bytes(sp), n, t)
            # only the dedicated per-step schedule reran (the per-wave one redoes its groups in place)
            assert be.binomial_reruns() == (1 if (formula, mode) == (0, 1) else 0), (formula, mode)
            row = list(r.dec2[bad * n:(bad + 1) * n])  # round 4 then skips the disqualified dealer
            assert row == [SELF if j == bad else REJECT for j in range(n)], (formula, mode, row)
            assert not r.qualified[bad]
            outs[(formula, mode)] = (bytes(r.dec2), bytes(r.dec4), list(r.qualified), r.final_share,
                                     r.public_share, r.mpk)
            if mode == 1:  # one rank holding every dealer: dkg_ceremony_shard_verify_device's rows
                dev = torch.device("cuda", 0)
                ins = [torch.frombuffer(bytearray(x), dtype=torch.uint8).to(dev) for x in (E, A, s, sp)]
                o2, o4 = (torch.zeros(n * n, dtype=torch.uint8, device=dev) for _ in range(2))
                oA, op = (torch.zeros(32 * n, dtype=torch.uint8, device=dev) for _ in range(2))
                be.ceremony_shard_verify_device(n, t, 0, n, *(x.data_ptr() for x in ins), o2.data_ptr(),
                                                o4.data_ptr(), oA.data_ptr(), op.data_ptr())
                assert be.binomial_reruns() == (1 if formula == 0 else 0), (formula, "shard")
                srow = o2[bad * n:(bad + 1) * n].tolist()
                assert srow == [SELF if j == bad else REJECT for j in range(n)], (formula, "shard", srow)
                outs[(formula, "shard")] = (bytes(o2.cpu().numpy()), bytes(op.cpu().numpy()))
    finally:
        be.set_stepping_formula(0)
        be.set_field_mode(0)
        be.set_binomial(0)
        be.set_split(0)
    assert outs[(0, 1)] == outs[(1, 1)] and outs[(0, 4)] == outs[(1, 1)]
    assert outs[(0, "shard")] == outs[(1, "shard")]


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("name", FAULTS + ["ceremony_n64_t31.json"])
def test_stepping_modes_goldens(be, golden, name, mode):
    """Stepping workgroup slots forced per column (1: all pieces of a column in one slot) or per
    piece (2), on split tables with ragged and short last pieces: every output bit-exact."""
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    try:
        be.set_stepping(mode)
        for pieces in {2, min(3, t + 1), min(5, t + 1)}:
            be.set_split(pieces)
            r = be.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
            _check_ceremony(c, r, n)
    finally:
        be.set_stepping(0)
        be.set_split(0)


@pytest.mark.parametrize("name", FAULTS + ["ceremony_n64_t31.json"])
def test_stepping_formulas_goldens(be, golden, name):
    """The stepping's dedicated additions (default; workgroups that met an exceptional pair redone by
    the complete formula) and the complete formula alone give every output bit-exact, unsplit and
    split into 2..4 pieces.  An E row made the identity (committee.rs:1127) makes every addition of
    its tables exceptional: the redo path runs; honest tables never need it."""
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    try:
        for pieces in sorted({1, 2, min(3, t + 1), min(4, t + 1)}):
            be.set_split(pieces)
            redos = []
            for formula in (0, 1):
                be.set_stepping_formula(formula)
                r = be.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
                _check_ceremony(c, r, n)
                redos.append(be.stepping_redos())
            assert redos[1] == 0
            if name.startswith("fault_e_identity"):
                assert redos[0] > 0, "the identity row must take the complete-formula redo"
            elif name.startswith("ceremony_"):  # n = 64: no identity padding columns either
                assert redos[0] == 0, "an honest ceremony needs no redo"
        if name.startswith("ceremony_"):
            # dealer 5's E row made the identity (committee.rs:1127) in a table without padding:
            # both formulas agree, and only the dedicated one needed the redo
            E = bytearray(H(c["E"]))
            E[5 * (t + 1) * 32:6 * (t + 1) * 32] = bytes(32 * (t + 1))
            be.set_split(0)
            out = []
            for formula in (0, 1):
                be.set_stepping_formula(formula)
                r = be.ceremony_verify(bytes(E), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
                out.append((r.dec2, r.dec4, r.qualified, r.mpk, be.stepping_redos()))
            assert out[0][:4] == out[1][:4] and out[0][4] > 0 and out[1][4] == 0
            assert r.dec2[5 * n:6 * n].count(0) == n - 1  # every other receiver complains about dealer 5
    finally:
        be.set_stepping_formula(0)
        be.set_split(0)


@pytest.mark.parametrize("mode,addends", [(1, 0), (2, 0), (2, 1)])
@pytest.mark.parametrize("name", FAULTS + ["ceremony_n64_t31.json"])
def test_combine_modes_goldens(be, golden, name, mode, addends):
    """Recombination with powers of j^L (1) or with short lattice multipliers (2: R holds b_j P(j),
    the checks scale the shares by b_j; addends affine Niels (0) or cached projective (1)) for 2..5
    pieces: every output bit-exact."""
    c = golden(name)
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    try:
        be.set_combine(mode)
        be.set_addends(addends)
        for pieces in sorted({2, min(3, t + 1), min(4, t + 1), min(5, t + 1)}):
            be.set_split(pieces)
            r = be.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
            _check_ceremony(c, r, n)
            # short multipliers: up to 4 pieces with either addend form, 5 with affine addends only
            short = mode == 2 and (pieces <= 4 or (pieces == 5 and addends == 0))
            assert be.last_combine() == (2 if short else 1) or pieces == 1
    finally:
        be.set_combine(0)
        be.set_addends(0)
        be.set_split(0)


@pytest.mark.parametrize("pieces", [1, 2, 3])
def test_degree_split_n256_matches_unsplit(be, pieces):
    """n = 256, t = 127 (BASELINE config 2) from device coefficients with one E row made undecodable
    and one A row replaced: the split and unsplit runs give identical decision matrices, and the
    honest rows accept everywhere."""
    import torch

    n, t = 256, 127
    N = t + 1
    be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes(range(32)), 9, 0, n, t)
    r0 = be.ceremony(a, b, n, t)
    E, A = bytearray(r0.E), bytearray(r0.A)
    E[32 * N * 17:32 * N * 17 + 32] = b"\xff" * 32
    A[32 * N * 200 + 32 * 5:32 * N * 200 + 32 * 6] = r0.A[32 * N * 3:32 * N * 3 + 32]
    try:
        be.set_split(pieces)
        r = be.ceremony_verify(bytes(E), bytes(A), r0.s, r0.s_prime, n, t)
        assert be.last_split() == pieces
    finally:
        be.set_split(0)
    dec2 = torch.frombuffer(bytearray(r.dec2), dtype=torch.uint8).reshape(n, n)
    dec4 = torch.frombuffer(bytearray(r.dec4), dtype=torch.uint8).reshape(n, n)
    assert set(dec2[17].tolist()) == {MISSING, SELF}
    assert set(dec4[200].tolist()) == {REJECT, SELF}
    ok2 = [i for i in range(n) if i != 17]
    ok4 = [i for i in range(n) if i not in (17, 200)]
    assert set(dec2[ok2].reshape(-1).tolist()) == {ACCEPT, SELF}
    assert set(dec4[ok4].reshape(-1).tolist()) == {ACCEPT, SELF}
    assert r.reconstruct == [int(i == 200) for i in range(n)]


@pytest.fixture
def interp(be):
    be.set_verify_mode("interp")
    yield be
    be.set_verify_mode("group")


@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("name", CEREMONIES + FAULTS + ["ceremony_n64_t31.json"])
def test_interp_mode_goldens(interp, golden, name, overlap):
    """Committee verification by interpolation (dkg_ctx_set_verify_mode 1) on every fixture: all
    outputs bit-exact.  The fault fixtures exercise both of its branches: dealers whose
    commitments are not g F + h F' (E := identity, A := generator, a flipped share among
    receivers 1..t+1) are re-verified with difference tables; a flipped randomness share beyond
    t+1 is decided by its own group equation."""
    c = golden(name)
    n, t = c["n"], c["t"]
    interp.env_init(t, n, CK)
    interp.set_overlap(overlap)
    try:
        r = interp.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
    finally:
        interp.set_overlap(True)
    _check_ceremony(c, r, n)
    expect_fallback = set(FAULTS)
    assert (interp.fallback_rows() > 0) == (name in expect_fallback), interp.fallback_rows()


@pytest.mark.parametrize("j,which", [(12, "s"), (12, "s_prime"), (3, "s"), (15, "both")])
def test_interp_mode_flipped_shares(be, golden, j, which):
    """A single tampered share of an honest n=16, t=7 ceremony, beyond and within receivers 1..t+1:
    group and interpolation modes give the same decision matrices, equal to the oracle's
    per-pair MSM check (committee.rs:287-305, 532-541)."""
    c = golden("ceremony_n16_t7.json")
    n, t = c["n"], c["t"]
    be.env_init(t, n, CK)
    s, sp = bytearray(H(c["s"])), bytearray(H(c["s_prime"]))
    i = 5
    for name, buf in (("s", s), ("s_prime", sp)):
        if which in (name, "both"):
            k = 32 * (i * n + j)
            buf[k] ^= 1
    out = {}
    for mode in ("group", "interp"):
        be.set_verify_mode(mode)
        try:
            r = be.ceremony_verify(H(c["E"]), H(c["A"]), bytes(s), bytes(sp), n, t)
        finally:
            be.set_verify_mode("group")
        out[mode] = (r.dec2, r.dec4, r.mpk, r.final_share)
    assert out["group"] == out["interp"]
    acc2, _ = O.verify_pairs(n, t, 2, H(c["E"]), H(c["h"]), bytes(s), bytes(sp), 0, n, 0, n)
    acc4, _ = O.verify_pairs(n, t, 4, H(c["A"]), H(c["h"]), bytes(s), bytes(sp), 0, n, 0, n)
    assert list(out["group"][0]) == list(acc2)
    d4 = list(out["group"][1])
    assert all(d4[q] == acc4[q] for q in range(n * n) if d4[q] != 3)
    assert out["group"][0][i * n + j] == REJECT


@pytest.mark.parametrize("n,t", [(256, 127), (1024, 511)])
def test_interp_mode_large(interp, n, t):
    """Configs 2 and 3 end to end from device coefficients in interpolation mode: same decisions,
    mpk and final shares as the difference-table mode, and no fallback on an honest ceremony."""
    import torch

    interp.env_init(t, n, CK)
    N = t + 1
    dev = torch.device("cuda", 0)
    ta = torch.empty(n * N * 32, dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    interp.dealer_coefficients_device(b"\x33" * 32, 2, 1, 0, n, t, ta.data_ptr(), tb.data_ptr())
    r1 = interp.ceremony_device(ta.data_ptr(), tb.data_ptr(), n, t)
    assert interp.fallback_rows() == 0
    interp.set_verify_mode("group")
    r0 = interp.ceremony_device(ta.data_ptr(), tb.data_ptr(), n, t)
    assert r1.mpk == r0.mpk and r1.qualified == r0.qualified == [1] * n and r1.complaints2 == [0] * n


def test_interp_mode_batch_and_shard(interp, golden):
    """Batched ceremonies (config-5 path) and the dealer-sharded rows in interpolation mode."""
    _ = golden
    n, t, B = 64, 31, 6
    N = t + 1
    interp.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(b"\x44" * 32, 0, 0, n, t)
    import torch

    dev = torch.device("cuda", 0)
    ta = torch.empty(B * n * N * 32, dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    interp.dealer_coefficients_device(b"\x44" * 32, 0, B, 0, n, t, ta.data_ptr(), tb.data_ptr())
    res1 = dkg_amd.ceremony_batch_device(interp, B, n, t, ta.data_ptr(), tb.data_ptr())
    interp.set_verify_mode("group")
    res0 = dkg_amd.ceremony_batch_device(interp, B, n, t, ta.data_ptr(), tb.data_ptr())
    assert res1.mpk == res0.mpk and res1.n_qualified == res0.n_qualified == [n] * B
    interp.set_verify_mode("interp")
    # one rank of a 3-way shard on tampered broadcasts (fixture): equal to the group mode's rows
    c = golden("fault_share_flip_n10_t4.json")
    n, t = c["n"], c["t"]
    N = t + 1
    interp.env_init(t, n, CK)
    E, A, s, sp = (H(c[k]) for k in ("E", "A", "s", "s_prime"))
    d0, d1 = 3, 7
    D = d1 - d0

    def put(x):
        return torch.frombuffer(bytearray(x), dtype=torch.uint8).to(dev)

    outs = []
    for mode in ("interp", "group"):
        interp.set_verify_mode(mode)
        o2 = torch.zeros(D * n, dtype=torch.uint8, device=dev)
        o4 = torch.zeros_like(o2)
        oA = torch.zeros(D * 32, dtype=torch.uint8, device=dev)
        op = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
        tE, tA = put(E[32 * N * d0:32 * N * d1]), put(A[32 * N * d0:32 * N * d1])
        ts, tsp = put(s[32 * n * d0:32 * n * d1]), put(sp[32 * n * d0:32 * n * d1])
        interp.ceremony_shard_verify_device(n, t, d0, d1, tE.data_ptr(), tA.data_ptr(), ts.data_ptr(), tsp.data_ptr(),
                                            o2.data_ptr(), o4.data_ptr(), oA.data_ptr(), op.data_ptr())
        outs.append([bytes(x.cpu().numpy()) for x in (o2, o4, oA, op)])
    assert outs[0] == outs[1]
    assert dec_str(outs[0][0]) == c["dec2"][d0 * n:d1 * n]


@pytest.mark.parametrize("seed", range(40))
def test_random_ceremonies_vs_oracle(be, seed):
    """Random committees (3 <= n < 48, every valid t) with random faults -- tampered shares or
    randomness, a replaced E or A coefficient, an undecodable commitment -- under a random schedule
    (verify mode, degree split, fused or protocol order): the decisions equal the oracle's per-pair
    MSM checks (committee.rs:287-305, 532-548) and the final shares and mpk equal the reference's
    rules recomputed here (committee.rs:454-462, 726-805)."""
    rng = random.Random(7000 + seed)
    n = rng.randrange(3, 48)
    t = rng.randrange(0, (n + 1) // 2)
    N = t + 1
    h = be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes(rng.randrange(256) for _ in range(32)), seed, 0, n, t)
    E, A, s, sp = (bytearray(x) for x in O.share_gen(n, n, t, a, b, h))
    faults = []
    for _ in range(rng.randrange(0, 4)):
        kind = rng.choice(["s", "sp", "E", "A", "Ebad", "self"])
        i = rng.randrange(n)
        if kind in ("s", "sp", "self"):
            j = i if kind == "self" else rng.choice([x for x in range(n) if x != i])
            buf = sp if kind == "sp" else s
            v = (int.from_bytes(buf[32 * (i * n + j):32 * (i * n + j) + 32], "little") + 1) % L
            buf[32 * (i * n + j):32 * (i * n + j) + 32] = v.to_bytes(32, "little")
            if kind == "self":  # the unchecked self-share plus an A fault on the same dealer
                A[32 * i * N:32 * i * N + 32] = O.base_mul(rng.randrange(1, L).to_bytes(32, "little"))
        elif kind in ("E", "A"):
            k = rng.randrange(N)
            buf = E if kind == "E" else A
            buf[32 * (i * N + k):32 * (i * N + k) + 32] = O.base_mul(rng.randrange(1, L).to_bytes(32, "little"))
        else:
            k = rng.randrange(N)
            E[32 * (i * N + k):32 * (i * N + k) + 32] = b"\xff" * 32
        faults.append((kind, i))
    mode, split, overlap = rng.choice(["group", "interp"]), rng.choice([0, 1, 2, 3]), rng.choice([True, False])
    be.set_verify_mode(mode)
    be.set_split(min(split, N))
    be.set_overlap(overlap)
    try:
        r = be.ceremony_verify(bytes(E), bytes(A), bytes(s), bytes(sp), n, t)
    finally:
        be.set_verify_mode("group")
        be.set_split(0)
        be.set_overlap(True)
    ctx = (n, t, faults, mode, split, overlap)
    acc2, _ = O.verify_pairs(n, t, 2, bytes(E), h, bytes(s), bytes(sp), 0, n, 0, n)
    acc4, _ = O.verify_pairs(n, t, 4, bytes(A), h, bytes(s), None, 0, n, 0, n)
    assert list(r.dec2) == list(acc2), ctx
    qualified = [int(all(r.dec2[i * n + j] in (ACCEPT, SELF) for j in range(n))) for i in range(n)]
    assert r.qualified == qualified, ctx
    for q in range(n * n):
        i, j = divmod(q, n)
        if i == j:
            assert r.dec4[q] == SELF
        elif not qualified[i]:
            assert r.dec4[q] == 3, ctx  # SKIPPED
        else:
            assert r.dec4[q] == acc4[q], ctx
    recon = [int(qualified[i] and any(r.dec4[i * n + j] == REJECT for j in range(n) if j != i)) for i in range(n)]
    assert r.reconstruct == recon, ctx
    fs = b"".join((sum(int.from_bytes(s[32 * (i * n + j):32 * (i * n + j) + 32], "little")
                       for i in range(n) if qualified[i]) % L).to_bytes(32, "little") for j in range(n))
    assert r.final_share == fs, ctx
    # mpk: what every final party computes (committee.rs:726-805), none if Phase4 fails (:673-677)
    A0 = [bytes(A[32 * N * i:32 * N * i + 32]) for i in range(n)]
    share = lambda i, j: int.from_bytes(s[32 * (i * n + j):32 * (i * n + j) + 32], "little")  # noqa: E731
    if sum(qualified) - sum(recon) <= t:
        assert r.phase4_error == 1 and r.mpk == bytes(32), ctx
    else:
        assert r.phase4_error == 0 and r.mpk == FR.final_party_mpk(n, qualified, recon, A0, share), ctx
    # per-party finalise with a random set of missing phase-5 disclosures (dkg_finalise_parties)
    disclosed = [int(rng.random() < 0.7) for _ in range(n)]
    pf = be.finalise_parties(n, t, qualified, recon, b"".join(A0), bytes(s), r.r2_error, r.r4_error, disclosed)
    names = {"OK": 0, "R2_ERROR": 1, "R4_ERROR": 2, "PHASE4_ERROR": 3, "INSUFFICIENT": 4, "PANIC": 5}
    for p in range(n):
        st, idx, mk = FR.party_finalise(p, n, t, qualified, recon, A0, share, disclosed=disclosed,
                                        r2_error=r.r2_error, r4_error=r.r4_error)
        assert (pf.status[p], pf.recovery_index[p]) == (names[st], idx), (ctx, p)
        assert pf.mpk[p] == (mk or bytes(32)), (ctx, p)


@pytest.mark.parametrize("name", ["finalise_parties_n10_t4.json", "finalise_parties_recon_n10_t4.json"])
def test_finalise_parties_golden(be, golden, name):
    """dkg_finalise_parties: every party's Phases<Phase5>::finalise outcome (committee.rs:726-805) --
    missing disclosures, exactly-t-point interpolation (a wrong secret, as the reference computes it),
    InsufficientSharesForRecovery, the reference's panic on a disqualified dealer, earlier round
    failures, a reconstructed dealer's own tampered self-share -- against the libsodium fixture."""
    f = golden(name)
    c = golden(f["source"])
    n, t = c["n"], c["t"]
    N = t + 1
    be.env_init(t, n, CK)
    A0 = b"".join(H(c["A"])[32 * N * i:32 * N * i + 32] for i in range(n))
    names = {"OK": 0, "R2_ERROR": 1, "R4_ERROR": 2, "PHASE4_ERROR": 3, "INSUFFICIENT": 4, "PANIC": 5}
    for case in f["cases"]:
        pf = be.finalise_parties(n, t, c["qualified"], c["reconstruct"], A0, H(c["s"]), case.get("r2_error"),
                                 case.get("r4_error"), case.get("disclosed"))
        assert pf.status == [names[x] for x in case["status"]], case["name"]
        assert pf.recovery_index == case["index"], case["name"]
        assert [m.hex() for m in pf.mpk] == case["mpk"], case["name"]


def test_ceremony_n4096_device(be):
    """BASELINE config 4 (n = 4096, t = 2047) end to end on one GPU from device-generated
    coefficients: every share of both rounds verifies and mpk == g * sum_i a_i0 (committee.rs:
    1633-1647); then rank 0 of the 8-way dealer split (dkg_ceremony_shard_device) accepts its rows."""
    import torch

    n, t = 4096, 2047
    N = t + 1
    be.env_init(t, n, CK)
    master = bytes([4]) * 32
    dev = torch.device("cuda", 0)
    ta = torch.empty(32 * n * N, dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    be.dealer_coefficients_device(master, 0, 1, 0, n, t, ta.data_ptr(), tb.data_ptr())
    r = be.ceremony_device(ta.data_ptr(), tb.data_ptr(), n, t)
    assert r.qualified == [1] * n and r.complaints2 == [0] * n and r.n_qualified == n
    a0 = ta.view(n, N, 32)[:, 0, :].cpu().numpy()
    secret = sum(int.from_bytes(bytes(a0[i]), "little") for i in range(n)) % L
    assert r.mpk == O.base_mul(secret.to_bytes(32, "little"))
    D = n // 8
    o2 = torch.empty(D * n, dtype=torch.uint8, device=dev)
    o4 = torch.empty_like(o2)
    oA = torch.empty(D * 32, dtype=torch.uint8, device=dev)
    op = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    be.ceremony_shard_device(n, t, 0, D, ta.data_ptr(), tb.data_ptr(), o2.data_ptr(), o4.data_ptr(), oA.data_ptr(),
                             op.data_ptr())
    import numpy as np

    honest = np.full((D, n), ACCEPT, dtype=np.uint8)
    honest[np.arange(D), np.arange(D)] = SELF  # rank 0 owns dealers 0..D-1: SELF at j == i
    assert np.array_equal(o2.view(D, n).cpu().numpy(), honest)
    assert np.array_equal(o4.view(D, n).cpu().numpy(), honest)


_NT_CHILD = r"""
import json, sys
sys.path.insert(0, %r)
import dkg_amd
c = json.load(open(%r))
be = dkg_amd.Backend(0)
be.env_init(c["t"], c["n"], b"Example of a shared string.")
be.set_split(1)
be.set_binomial(1)
H = bytes.fromhex
r = be.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), c["n"], c["t"])
print(json.dumps({"dec2": "".join(str(x) for x in r.dec2), "dec4": "".join(str(x) for x in r.dec4),
                  "final_share": r.final_share.hex(), "mpk": r.mpk.hex(), "reruns": be.binomial_reruns()}))
be.close()
"""


@pytest.mark.parametrize("knobs", [{"DKG_BINOM_NT_BYTES": "1e30"}, {"DKG_BINOM_NT_BYTES": "0"},
                                   {"DKG_BINOM_NT_BYTES": "3e5"},
                                   {"DKG_BINOM_IL_WAVES": "1e9", "DKG_BINOM_ILP_WAVES": "0"}],
                         ids=["plain", "nontemporal", "by_footprint", "paired_chains"])
def test_binomial_store_kinds_env(golden, knobs):
    """The per-step binomial's rows stored plainly (DKG_BINOM_NT_BYTES=1e30), nontemporally (0, the
    default) or by step footprint (3e5: steps 1-6 plain, the later ones nontemporal), and every step
    on the product-scanning copy with paired m-chains (k_binom_step<.., IL>: DKG_BINOM_IL_WAVES above
    any step, no column-sum steps) -- the env knobs are read once per process, so each runs in a
    child: the same decisions, final shares and mpk as the golden ceremony."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "tests", "golden", "ceremony_n64_t31.json")
    env = dict(os.environ, **knobs)
    p = subprocess.run([sys.executable, "-c", _NT_CHILD % (root, path)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    got = json.loads(p.stdout.strip().splitlines()[-1])
    c = golden("ceremony_n64_t31.json")
    assert got == {"dec2": c["dec2"], "dec4": c["dec4"], "final_share": c["final_share"], "mpk": c["mpk"],
                   "reruns": 0}
