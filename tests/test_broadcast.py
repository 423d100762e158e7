"""Broadcast messages and the committee-wide intake (dkg_amd/broadcast.py):
byte layouts round-trip, malformed messages are refused, and from_broadcast's shape rules
(committee.rs:841-852, 940-946) give the fetched masks.  The GPU half (the fetched ceremony) is
tests/test_gpu.py::test_ceremony_from_broadcasts."""
import random

import pytest

from dkg_amd.broadcast import (BroadcastPhase1, BroadcastPhase2, BroadcastPhase3, BroadcastPhase4,
                               BroadcastPhase5, EncryptedShares, MisbehavingPartiesRound1,
                               MisbehavingPartiesRound3, intake_phase1, intake_phase3)

H = bytes.fromhex


def committee_broadcasts(c):
    """The plaintext-mode phase-1 / phase-3 broadcasts of a golden ceremony."""
    n, N = c["n"], c["t"] + 1
    E, A, s, sp = (H(c[k]) for k in ("E", "A", "s", "s_prime"))
    p1 = [BroadcastPhase1([E[32 * (N * i + k):32 * (N * i + k + 1)] for k in range(N)],
                          [EncryptedShares(q + 1, s[32 * (i * n + q):32 * (i * n + q + 1)],
                                           sp[32 * (i * n + q):32 * (i * n + q + 1)]) for q in range(n)])
          for i in range(n)]
    p3 = [BroadcastPhase3([A[32 * (N * i + k):32 * (N * i + k + 1)] for k in range(N)]) for i in range(n)]
    return p1, p3


def test_roundtrip_all_phases(golden):
    rng = random.Random(3)
    rb = lambda k: bytes(rng.randrange(256) for _ in range(k))  # noqa: E731
    p1, p3 = committee_broadcasts(golden("ceremony_n10_t4.json"))
    for m in p1:
        assert BroadcastPhase1.from_bytes(m.to_bytes()) == m
    full = BroadcastPhase1([rb(32)] * 3, [EncryptedShares(q + 1, rb(64), rb(64)) for q in range(4)])
    assert BroadcastPhase1.from_bytes(full.to_bytes()) == full
    for m in p3:
        assert BroadcastPhase3.from_bytes(m.to_bytes()) == m
    b2 = BroadcastPhase2([MisbehavingPartiesRound1(3, 1, rb(128), rb(192)), MisbehavingPartiesRound1(7, 2, rb(128), rb(192))])
    assert BroadcastPhase2.from_bytes(b2.to_bytes()) == b2
    b4 = BroadcastPhase4([MisbehavingPartiesRound3(2, rb(32), rb(32))])
    assert BroadcastPhase4.from_bytes(b4.to_bytes()) == b4
    b5 = BroadcastPhase5([None, rb(32), None])
    assert BroadcastPhase5.from_bytes(b5.to_bytes()) == b5
    assert BroadcastPhase2.from_bytes(BroadcastPhase2([]).to_bytes()).misbehaving_parties == []


def test_malformed_bytes_refused(golden):
    p1, p3 = committee_broadcasts(golden("ceremony_n3_t1.json"))
    b = p1[0].to_bytes()
    with pytest.raises(ValueError):
        BroadcastPhase1.from_bytes(b[:-1])
    with pytest.raises(ValueError):
        BroadcastPhase1.from_bytes(b + b"\0")
    bad_mode = bytearray(b)
    bad_mode[4 + 32 * 2 + 4 + 4] = 7  # mode byte of the first EncryptedShares
    with pytest.raises(ValueError):
        BroadcastPhase1.from_bytes(bytes(bad_mode))
    with pytest.raises(ValueError):
        BroadcastPhase3.from_bytes(p3[0].to_bytes()[:40])


def test_intake_shape_rules(golden):
    c = golden("ceremony_n10_t4.json")
    n, t = c["n"], c["t"]
    N = t + 1
    p1, p3 = committee_broadcasts(c)
    p1[2] = None                                                             # did not broadcast
    p1[6] = BroadcastPhase1(p1[6].committed_coefficients[:t], p1[6].encrypted_shares)         # t entries
    p1[8] = BroadcastPhase1(p1[8].committed_coefficients, p1[8].encrypted_shares[:n - 1])     # n-1 shares
    p3[4] = None
    p3[9] = BroadcastPhase3(p3[9].committed_coefficients + p3[9].committed_coefficients[:1])  # t+2 entries
    got = intake_phase1(n, t, p1)
    assert list(got.fetched1) == [0 if i in (2, 6, 8) else 1 for i in range(n)]
    E = H(c["E"])
    for i in (0, 1, 3):
        assert got.E[32 * N * i:32 * N * (i + 1)] == E[32 * N * i:32 * N * (i + 1)]
        assert got.share[32 * n * i:32 * n * (i + 1)] == H(c["s"])[32 * n * i:32 * n * (i + 1)]
    A, f3 = intake_phase3(n, t, p3)
    assert list(f3) == [0 if i in (4, 9) else 1 for i in range(n)]
    assert A[:32 * N] == H(c["A"])[:32 * N]
    with pytest.raises(ValueError):
        intake_phase1(n, t, p1[:-1])
    # a full-mode share in a plaintext-mode committee is not fetched data either
    p1b, _ = committee_broadcasts(c)
    p1b[0].encrypted_shares[3] = EncryptedShares(4, bytes(64), bytes(64))
    assert intake_phase1(n, t, p1b).fetched1[0] == 0
    assert list(got.fetch_invalid) == [0] * n


def test_intake_recipient_index(golden):
    """A share whose recipient_index is not the receiver's own makes that receiver's Phase1::proceed
    return Err(FetchedInvalidData) (committee.rs:277-280): flagged per receiver; a party's own
    broadcast is never fetched by itself, so its own mislabelled entry is not a failure."""
    c = golden("ceremony_n10_t4.json")
    n, t = c["n"], c["t"]
    p1, _ = committee_broadcasts(c)
    e = p1[3].encrypted_shares[5]
    p1[3].encrypted_shares[5] = EncryptedShares(7, e.share, e.randomness)      # dealer 4 -> receiver 6
    e = p1[1].encrypted_shares[1]
    p1[1].encrypted_shares[1] = EncryptedShares(9, e.share, e.randomness)      # dealer 2's own entry
    got = intake_phase1(n, t, p1)
    assert list(got.fetch_invalid) == [int(q == 5) for q in range(n)]
    assert list(got.fetched1) == [1] * n
