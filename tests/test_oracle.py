"""Pin the CPU oracle against the golden fixtures (libsodium-generated, tools/gen_golden.py).

These run on CPU only.  They are the reason the oracle may be trusted as the checker for the HIP
path: every group / scalar / ceremony output it produces equals an independent implementation.
"""
import ctypes

import pytest

from tests import oracle_lib as O

H = bytes.fromhex


def chunks(hexstr, size=32):
    b = H(hexstr)
    return [b[i:i + size] for i in range(0, len(b), size)]


def test_base_multiples(golden):
    g = golden("kat_group.json")
    for e in g["base_multiples"]:
        k = e["k"].to_bytes(32, "little")
        assert O.base_mul(k).hex() == e["P"], e["k"]
    for e in g["base_mul"]:
        assert O.base_mul(H(e["k"])).hex() == e["P"]


def test_hash_to_group_and_uniform(golden):
    g = golden("kat_group.json")
    for e in g["hash_to_group"]:
        m = H(e["msg"])
        out, _ = O.call32("or_pt_hash_to_group", m, len(m))
        assert out.hex() == e["P"]
    # CommitmentKey::generate(b"Example of a shared string.") (commitment.rs:13-17)
    assert g["hash_to_group"][0]["P"].startswith("242496c4")
    for e in g["from_uniform_bytes"]:
        out, _ = O.call32("or_pt_from_uniform_bytes", H(e["in"]))
        assert out.hex() == e["P"]


def test_point_ops(golden):
    g = golden("kat_group.json")
    for e in g["add"]:
        assert O.call32("or_pt_add", H(e["P"]), H(e["Q"]))[0].hex() == e["sum"]
        assert O.call32("or_pt_sub", H(e["P"]), H(e["Q"]))[0].hex() == e["diff"]
        assert O.call32("or_pt_neg", H(e["P"]))[0].hex() == e["neg_P"]
        assert O.lib().or_pt_eq(H(e["P"]), H(e["P"])) == 1
        assert O.lib().or_pt_eq(H(e["P"]), H(e["Q"])) == 0
    for e in g["mul"]:
        assert O.call32("or_pt_mul", H(e["P"]), H(e["k"]))[0].hex() == e["kP"]


def test_invalid_encodings(golden):
    for b in golden("kat_group.json")["invalid_encodings"]:
        assert O.lib().or_pt_valid(H(b)) == 0, b
    assert O.lib().or_pt_valid(bytes(32)) == 1  # identity decodes


@pytest.mark.parametrize("idx", range(10))
def test_msm(golden, idx):
    c = golden("kat_group.json")["msm"][idx]
    assert O.msm(H(c["scalars"]), H(c["points"])).hex() == c["out"], c["N"]


def test_scalar_ops(golden):
    s = golden("kat_scalar.json")
    for e in s["reduce_wide"]:
        assert O.call32("or_sc_reduce_wide", H(e["in"]))[0].hex() == e["out"]
    for e in s["ops"]:
        a, b = H(e["a"]), H(e["b"])
        assert O.call32("or_sc_add", a, b)[0].hex() == e["add"]
        assert O.call32("or_sc_sub", a, b)[0].hex() == e["sub"]
        assert O.call32("or_sc_mul", a, b)[0].hex() == e["mul"]
        assert O.call32("or_sc_neg", a)[0].hex() == e["neg_a"]
        assert O.call32("or_sc_invert", a)[0].hex() == e["inv_a"]


def test_polynomial_kats(golden):
    s = golden("kat_scalar.json")
    # polynomial.rs:240-249: (1 + 3x) of degree 4 at 3 == 10
    kt = s["poly_tests"]
    coeffs = b"".join(c.to_bytes(32, "little") for c in kt["coeffs"])
    assert O.poly_eval(coeffs, kt["x"].to_bytes(32, "little")) == kt["value"].to_bytes(32, "little")
    for e in s["poly_eval"]:
        for x, v in zip(e["points"], e["values"]):
            assert O.poly_eval(H(e["coeffs"]), x.to_bytes(32, "little")).hex() == v
    lg = s["lagrange"]
    xs = b"".join(x.to_bytes(32, "little") for x in lg["xs"])
    ys = b"".join(y.to_bytes(32, "little") for y in lg["ys"])
    out = ctypes.create_string_buffer(32)
    O.lib().or_lagrange(out, bytes(32), ys, xs, 3)
    assert int.from_bytes(out.raw, "little") == lg["at_zero"] == 13


def test_dealer_rng(golden):
    r = golden("kat_scalar.json")["dealer_rng"]
    seed = O.dealer_seed(H(r["master"]), r["ceremony"], r["dealer"])
    assert seed.hex() == r["seed"]
    out = ctypes.create_string_buffer(128)
    O.lib().or_chacha20_stream(seed, 0, out, 128)
    assert out.raw.hex() == r["stream_head"]
    a, b = O.dealer_coeffs(seed, r["t"])
    assert chunks(a.hex()) == [H(x) for x in r["a"]]
    assert chunks(b.hex()) == [H(x) for x in r["b"]]


CEREMONIES = ["ceremony_n2_t0.json", "ceremony_n3_t1.json", "ceremony_n10_t4.json",
              "ceremony_n11_t5.json", "ceremony_n16_t7.json"]
FAULTS = ["fault_e_identity_n10_t4.json", "fault_share_flip_n10_t4.json",
          "fault_a_generator_n10_t4.json", "fault_over_threshold_n10_t4.json", "fault_a_many_n10_t4.json",
          "fault_self_share_n10_t4.json", "fault_recon_only_n10_t4.json", "fault_recon_r2err_n16_t3.json",
          "fault_recon_insufficient_n16_t3.json"]


@pytest.mark.parametrize("name", CEREMONIES)
def test_share_gen(golden, name):
    c = golden(name)
    n, t = c["n"], c["t"]
    master = H(c["master_seed"])
    a = b"".join(O.dealer_coeffs(O.dealer_seed(master, c["ceremony"], i), t)[0] for i in range(n))
    b = b"".join(O.dealer_coeffs(O.dealer_seed(master, c["ceremony"], i), t)[1] for i in range(n))
    assert a.hex() == c["a"] and b.hex() == c["b"]
    E, A, s, sp = O.share_gen(n, n, t, a, b, H(c["h"]))
    assert E.hex() == c["E"]
    assert A.hex() == c["A"]
    assert s.hex() == c["s"]
    assert sp.hex() == c["s_prime"]


def _decisions(c, rnd):
    n, t = c["n"], c["t"]
    C = H(c["E"] if rnd == 2 else c["A"])
    acc, rc = O.verify_pairs(n, t, rnd, C, H(c["h"]), H(c["s"]), H(c["s_prime"]), 0, n, 0, n)
    return acc, rc


@pytest.mark.parametrize("name", CEREMONIES + FAULTS)
def test_round2_round4_decisions(golden, name):
    c = golden(name)
    n = c["n"]
    acc, rc = _decisions(c, 2)
    assert rc == 0
    assert "".join(str(x) for x in acc) == c["dec2"]
    acc4, rc = _decisions(c, 4)
    exp4 = c["dec4"]
    got4 = "".join(str(x) for x in acc4)
    # dec4 marks disqualified dealers "3" (skipped, committee.rs:522); the oracle checks every pair
    for i in range(n * n):
        if exp4[i] != "3":
            assert got4[i] == exp4[i], (name, i // n, i % n)


def test_ceremony_n64(golden):
    c = golden("ceremony_n64_t31.json")
    acc, rc = _decisions(c, 2)
    assert rc == 0 and "".join(str(x) for x in acc) == c["dec2"]


def test_spot_n256(golden):
    sp = golden("spot_n256_t127.json")
    n, t = sp["n"], sp["t"]
    for d in sp["dealers"]:
        # per-pair reference check on the committed vector (vartime MSM over t+1 = 128 points)
        for pr in d["pairs"]:
            j = pr["receiver"]
            pw = b"".join(pow(j + 1, k, 2**252 + 27742317777372353535851937790883648493).to_bytes(32, "little")
                          for k in range(t + 1))
            assert O.msm(pw, H(d["E"])).hex() == pr["rhs2"]


# ---------------- full (encrypted-share) mode: elgamal.rs / procedure_keys.rs ----------------
FULL = ["full_n4_t1.json", "full_n10_t4.json", "full_faults_n10_t4.json"]


def test_hybrid_kat(golden):
    """Oracle hybrid encryption (elgamal.rs:134-193) against the libsodium vectors."""
    k = golden("kat_hybrid.json")
    for c in k["hybrid"]:
        e1, e2 = O.hybrid_encrypt(H(c["pk"]), H(c["r"]), H(c["msg"]))
        assert (e1.hex(), e2.hex()) == (c["e1"], c["e2"])
        assert O.hybrid_decrypt(H(c["sk"]), e1, e2).hex() == c["msg"]
        assert O.call32("or_pt_mul", H(c["pk"]), H(c["r"]))[0].hex() == c["K"]
    assert O.member_sk(bytes(32), 0, 0).hex() == k["member_sk0"]


def _member_keys(master, ceremony, n):
    sks = [O.member_sk(master, ceremony, j) for j in range(n)]
    pks = [O.base_mul(sk) for sk in sks]
    order = sorted(range(n), key=lambda j: pks[j])  # procedure_keys.rs:26-40, committee.rs:134-135
    return [sks[j] for j in order], [pks[j] for j in order]


@pytest.mark.parametrize("name", FULL)
def test_full_mode_ceremony(golden, name):
    """Full mode end to end on the oracle: sorted member keys, the draw order of the encryption
    randomness, every ciphertext of the honest pairs, decryption of the (possibly tampered) wire
    ciphertexts, and the round-2/4 decisions on the decrypted shares."""
    c = golden(name)
    n, t = c["n"], c["t"]
    master = H(c["master_seed"])
    sks, pks = _member_keys(master, c["ceremony"], n)
    assert b"".join(sks).hex() == c["member_sk"] and b"".join(pks).hex() == c["member_pk"]
    r = b"".join(O.enc_randomness(O.dealer_seed(master, c["ceremony"], i), t, n) for i in range(n))
    assert r.hex() == c["enc_r"]
    a = b"".join(O.dealer_coeffs(O.dealer_seed(master, c["ceremony"], i), t)[0] for i in range(n))
    b = b"".join(O.dealer_coeffs(O.dealer_seed(master, c["ceremony"], i), t)[1] for i in range(n))
    E, A, s, sp = O.share_gen(n, n, t, a, b, H(c["h"]))
    e1w, ctw = H(c["e1"]), H(c["ct"])
    tampered = {(f["dealer"] - 1, f["receiver"] - 1) for f in c["faults"]}
    dec_s, dec_sp = bytearray(32 * n * n), bytearray(32 * n * n)
    for i in range(n):
        for q in range(n):
            for w, msg in ((0, sp), (1, s)):  # randomness ciphertext first (committee.rs:171-172)
                k = 2 * (i * n + q) + w
                if (i, q) not in tampered:
                    e1, e2 = O.hybrid_encrypt(pks[q], r[32 * k:32 * k + 32], msg[32 * (i * n + q):32 * (i * n + q) + 32])
                    assert (e1, e2) == (e1w[32 * k:32 * k + 32], ctw[32 * k:32 * k + 32]), (i, q, w)
                m = O.hybrid_decrypt(sks[q], e1w[32 * k:32 * k + 32], ctw[32 * k:32 * k + 32])
                red = O.call32("or_sc_reduce", bytes(m[:31]) + bytes([m[31] & 0x7f]))[0]  # from_bits, reduced
                (dec_sp if w == 0 else dec_s)[32 * (i * n + q):32 * (i * n + q) + 32] = red
    assert bytes(dec_s).hex() == c["s"] and bytes(dec_sp).hex() == c["s_prime"]
    assert _decisions(c, 2)[0] == bytes(int(x) for x in c["dec2"])


# ---------------- complaint proofs: dl_equality/zkp.rs, broadcast.rs ----------------
VERDICT = {"Ok": 0, "InvalidProofOfMisbehaviour": 1, "FalseClaimedInequality": 2, "FalseClaimedEquality": 3}


def _complaint_inputs(c, full, x):
    n, t = full["n"], full["t"]
    N = t + 1
    q, i = x["accuser"] - 1, x["accused"] - 1
    k = 2 * (i * n + q)
    e1, ct = H(full["e1"]), H(full["ct"])
    enc = e1[32 * k:32 * k + 32] + ct[32 * k:32 * k + 32] + e1[32 * k + 32:32 * k + 64] + ct[32 * k + 32:32 * k + 64]
    pf = x["proof"]
    proof = b"".join(H(pf[f]) for f in ("share_key", "randomness_key", "c1", "r1", "c2", "r2"))
    return (H(full["member_sk"])[32 * q:32 * q + 32], H(full["member_pk"])[32 * q:32 * q + 32], enc,
            H(full["E"])[32 * N * i:32 * N * (i + 1)], proof)


def test_complaint_proofs_oracle(golden):
    """ProofOfMisbehaviour::generate / MisbehavingPartiesRound1::verify (broadcast.rs:50-99, 181-283,
    incl. the swapped-role quirk of :271-274) and MisbehavingPartiesRound3::verify (:105-135) on the
    oracle against the libsodium fixtures: proofs byte for byte, verdicts including forged claims."""
    c = golden("complaints_n10_t4.json")
    full = golden(c["source"])
    t = full["t"]
    for x in c["round1"]:
        sk, pk, enc, E, proof = _complaint_inputs(c, full, x)
        w = b"".join(H(v) for v in x["w"])
        if x["verdict"] != "InvalidProofOfMisbehaviour":
            assert O.misbehaviour_prove(sk, enc, w) == proof
        assert O.complaint1_verify(H(full["h"]), t, x["accuser"], pk, enc, E, proof) == VERDICT[x["verdict"]]
    p3 = golden(c["round3_source"])
    n, N = p3["n"], p3["t"] + 1
    for x in c["round3"]:
        i = x["accused"] - 1
        rc = O.complaint3_verify(H(p3["h"]), p3["t"], x["accuser"], H(x["share"]), H(x["randomness"]),
                                 H(p3["E"])[32 * N * i:32 * N * (i + 1)], H(p3["A"])[32 * N * i:32 * N * (i + 1)])
        assert rc == VERDICT[x["verdict"]], x


# ---------------- finalise (committee.rs:625-805) per party: tests/finalise_ref.py ----------------
def _fin_inputs(c):
    n, t = c["n"], c["t"]
    N = t + 1
    A0 = [H(c["A"])[32 * N * i:32 * N * i + 32] for i in range(n)]
    s = H(c["s"])
    return n, t, A0, lambda i, j: int.from_bytes(s[32 * (i * n + j):32 * (i * n + j) + 32], "little")


@pytest.mark.parametrize("name", CEREMONIES + FAULTS)
def test_ceremony_mpk_rule(golden, name):
    """The ceremony-level mpk of the fixtures is what every final party computes (an all-zero mpk
    when Phases<Phase4>::proceed fails for everyone, committee.rs:673-677)."""
    from tests.finalise_ref import final_party_mpk
    c = golden(name)
    n, t, A0, share = _fin_inputs(c)
    if c["phase4_error"]:
        assert c["mpk"] == "00" * 32
    else:
        mpk = final_party_mpk(n, c["qualified"], c["reconstruct"], A0, share,
                              [int(x) for x in c["r2_error"]], [int(x) for x in c["r4_error"]], t)
        assert (mpk or bytes(32)).hex() == c["mpk"]


@pytest.mark.parametrize("name", ["finalise_parties_n10_t4.json", "finalise_parties_recon_n10_t4.json"])
def test_finalise_parties_fixtures(golden, name):
    """Per-party finalise (missing disclosures, t-point interpolation, InsufficientSharesForRecovery,
    the reference's panic on a disqualified dealer, earlier round failures) restated on the oracle
    reproduces the libsodium fixture for every party."""
    from tests.finalise_ref import party_finalise
    f = golden(name)
    c = golden(f["source"])
    n, t, A0, share = _fin_inputs(c)
    for case in f["cases"]:
        for p in range(n):
            st, idx, mpk = party_finalise(p, n, t, c["qualified"], c["reconstruct"], A0, share,
                                          disclosed=case.get("disclosed"), r2_error=case.get("r2_error"),
                                          r4_error=case.get("r4_error"))
            assert (st, idx) == (case["status"][p], case["index"][p]), (case["name"], p)
            assert (mpk or bytes(32)).hex() == case["mpk"][p], (case["name"], p)
