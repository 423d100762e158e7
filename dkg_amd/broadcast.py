"""Broadcast messages of the protocol and the committee-wide broadcast intake.

The reference keeps its broadcasts as in-memory structs (broadcast.rs:16-30, 155-178) and turns the
list a party fetched into per-sender state with MembersFetchedState1..5::from_broadcast
(committee.rs:818-1035).  This module mirrors those structs, gives them a byte layout for the wire
(the reference defines none; points are 32-byte compressed Ristretto, groups.rs:72-76, scalars
32-byte little-endian canonical, groups.rs:23-27, integers u32 little-endian):

  EncryptedShares   u32 recipient_index | u8 mode | share | randomness
                    mode 0 (plaintext, the headline mode): 32-byte scalars
                    mode 1 (full mode): 64-byte HybridCiphertext e1 || e2 each (elgamal.rs:110-113)
  BroadcastPhase1   u32 N | N points | u32 m | m x EncryptedShares
  BroadcastPhase2   u32 k | k x (u32 accused | u8 error | 128-byte ciphertexts | 192-byte proof)
  BroadcastPhase3   u32 N | N points
  BroadcastPhase4   u32 k | k x (u32 accused | share | randomness)
  BroadcastPhase5   u32 n | n x (u8 present | 32-byte share)

and packs a committee's phase-1 / phase-3 broadcasts into the dense arrays of the C ABI with the
intake rules of from_broadcast: an absent broadcast, or one whose committed_coefficients do not
have t+1 entries or whose encrypted_shares do not have n entries (committee.rs:841-852, 940-946),
is "no fetched data" -- fetched[i] = 0, which dkg_ceremony_verify_fetched turns into DKG_MISSING in
round 2 (committee.rs:331-335) and a round-4 accusation (committee.rs:549-555).
"""
import struct
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

_U32 = struct.Struct("<I")


class _Reader:
    def __init__(self, b: bytes):
        self.b, self.o = b, 0

    def take(self, k: int) -> bytes:
        if self.o + k > len(self.b):
            raise ValueError("truncated broadcast message")
        v = self.b[self.o:self.o + k]
        self.o += k
        return v

    def u32(self) -> int:
        return _U32.unpack(self.take(4))[0]

    def u8(self) -> int:
        return self.take(1)[0]

    def done(self):
        if self.o != len(self.b):
            raise ValueError("trailing bytes in broadcast message")


def _points(r: _Reader) -> List[bytes]:
    return [r.take(32) for _ in range(r.u32())]


def _put_points(pts: Sequence[bytes]) -> bytes:
    assert all(len(p) == 32 for p in pts)
    return _U32.pack(len(pts)) + b"".join(pts)


@dataclass
class EncryptedShares:
    """broadcast.rs:16-20: the dealer's share and randomness for one recipient (1-based index)."""
    recipient_index: int
    share: bytes          # 32-byte scalar (plaintext mode) or 64-byte hybrid ciphertext e1 || e2
    randomness: bytes

    @property
    def mode(self) -> int:
        return 0 if len(self.share) == 32 else 1

    def to_bytes(self) -> bytes:
        w = 32 if self.mode == 0 else 64
        assert len(self.share) == w and len(self.randomness) == w
        return _U32.pack(self.recipient_index) + bytes([self.mode]) + self.share + self.randomness

    @classmethod
    def read(cls, r: _Reader) -> "EncryptedShares":
        idx, mode = r.u32(), r.u8()
        if mode not in (0, 1):
            raise ValueError("unknown share mode")
        w = 32 if mode == 0 else 64
        return cls(idx, r.take(w), r.take(w))


@dataclass
class BroadcastPhase1:
    """broadcast.rs:155-158: committed coefficients E_i and the shares for every recipient."""
    committed_coefficients: List[bytes]
    encrypted_shares: List[EncryptedShares]

    def to_bytes(self) -> bytes:
        return (_put_points(self.committed_coefficients) + _U32.pack(len(self.encrypted_shares))
                + b"".join(e.to_bytes() for e in self.encrypted_shares))

    @classmethod
    def from_bytes(cls, b: bytes) -> "BroadcastPhase1":
        r = _Reader(b)
        E = _points(r)
        shares = [EncryptedShares.read(r) for _ in range(r.u32())]
        r.done()
        return cls(E, shares)


@dataclass
class MisbehavingPartiesRound1:
    """broadcast.rs:37-42 with the ciphertexts the proof refers to (dkg_complaint1_verify layout)."""
    accused_index: int
    accusation_error: int     # DkgError discriminant of the accuser's failed check
    ciphertexts: bytes        # 128 B: e1_rand || ct_rand || e1_share || ct_share
    proof: bytes              # 192 B ProofOfMisbehaviour


@dataclass
class BroadcastPhase2:
    misbehaving_parties: List[MisbehavingPartiesRound1]

    def to_bytes(self) -> bytes:
        out = [_U32.pack(len(self.misbehaving_parties))]
        for m in self.misbehaving_parties:
            assert len(m.ciphertexts) == 128 and len(m.proof) == 192
            out.append(_U32.pack(m.accused_index) + bytes([m.accusation_error]) + m.ciphertexts + m.proof)
        return b"".join(out)

    @classmethod
    def from_bytes(cls, b: bytes) -> "BroadcastPhase2":
        r = _Reader(b)
        ms = [MisbehavingPartiesRound1(r.u32(), r.u8(), r.take(128), r.take(192)) for _ in range(r.u32())]
        r.done()
        return cls(ms)


@dataclass
class BroadcastPhase3:
    """broadcast.rs:166-168: the dealer's A_i."""
    committed_coefficients: List[bytes]

    def to_bytes(self) -> bytes:
        return _put_points(self.committed_coefficients)

    @classmethod
    def from_bytes(cls, b: bytes) -> "BroadcastPhase3":
        r = _Reader(b)
        A = _points(r)
        r.done()
        return cls(A)


@dataclass
class MisbehavingPartiesRound3:
    """broadcast.rs:103-108: accused index and the accuser's decrypted share / randomness."""
    accused_index: int
    decrypted_share: bytes
    decrypted_randomness: bytes


@dataclass
class BroadcastPhase4:
    misbehaving_parties: List[MisbehavingPartiesRound3]

    def to_bytes(self) -> bytes:
        return _U32.pack(len(self.misbehaving_parties)) + b"".join(
            _U32.pack(m.accused_index) + m.decrypted_share + m.decrypted_randomness for m in self.misbehaving_parties)

    @classmethod
    def from_bytes(cls, b: bytes) -> "BroadcastPhase4":
        r = _Reader(b)
        ms = [MisbehavingPartiesRound3(r.u32(), r.take(32), r.take(32)) for _ in range(r.u32())]
        r.done()
        return cls(ms)


@dataclass
class BroadcastPhase5:
    """broadcast.rs:175-177: per party, the disclosed share of a reconstructed dealer or None."""
    misbehaving_parties: List[Optional[bytes]]

    def to_bytes(self) -> bytes:
        return _U32.pack(len(self.misbehaving_parties)) + b"".join(
            b"\x00" + bytes(32) if s is None else b"\x01" + s for s in self.misbehaving_parties)

    @classmethod
    def from_bytes(cls, b: bytes) -> "BroadcastPhase5":
        r = _Reader(b)
        out: List[Optional[bytes]] = []
        for _ in range(r.u32()):
            present, share = r.u8(), r.take(32)
            out.append(share if present else None)
        r.done()
        return cls(out)


# ---------------- committee-wide intake (MembersFetchedState1/3::from_broadcast) ----------------
@dataclass
class Phase1Intake:
    E: bytes             # [n][t+1][32]; rows of unfetched dealers are zero (never decided on)
    share: bytes         # [n dealer][n recipient][w] (w = 32 plaintext, 64 full mode)
    randomness: bytes
    fetched1: bytes      # [n] 1 = the dealer's phase-1 data was fetched
    fetch_invalid: bytes  # [n] 1 = receiver q's Phases<Phase1>::proceed returns Err(FetchedInvalidData)


def intake_phase1(n: int, t: int, msgs: Sequence[Optional[BroadcastPhase1]], mode: int = 0) -> Phase1Intake:
    """Every party's phase-1 broadcast (msgs[i] from dealer i+1, None if it did not broadcast) as the
    committee sees it: from_broadcast's shape rule (committee.rs:841-852) per dealer; recipient q
    takes encrypted_shares[q] (:856-858, by position, as the reference does).  A fetched share whose
    recipient_index is not q+1 makes receiver q's round 2 abort with FetchedInvalidData
    (committee.rs:277-280): flagged in fetch_invalid[q].  The rest of such a party's protocol is not
    modelled (it never broadcasts again); its column of decisions is still computed."""
    if len(msgs) != n:
        raise ValueError("one entry per party expected")
    N, w = t + 1, 32 if mode == 0 else 64
    E, S, R, ok = bytearray(32 * n * N), bytearray(w * n * n), bytearray(w * n * n), bytearray(n)
    bad = bytearray(n)
    for i, m in enumerate(msgs):
        if m is None or len(m.committed_coefficients) != N or len(m.encrypted_shares) != n:
            continue
        if any(e.mode != mode for e in m.encrypted_shares):
            continue
        ok[i] = 1
        E[32 * N * i:32 * N * (i + 1)] = b"".join(m.committed_coefficients)
        for q, e in enumerate(m.encrypted_shares):
            S[w * (i * n + q):w * (i * n + q + 1)] = e.share
            R[w * (i * n + q):w * (i * n + q + 1)] = e.randomness
            if e.recipient_index != q + 1 and q != i:  # a party never fetches its own broadcast
                bad[q] = 1
    return Phase1Intake(bytes(E), bytes(S), bytes(R), bytes(ok), bytes(bad))


def intake_phase3(n: int, t: int, msgs: Sequence[Optional[BroadcastPhase3]]) -> Tuple[bytes, bytes]:
    """(A [n][t+1][32], fetched3 [n]) under MembersFetchedState3::from_broadcast (committee.rs:930-963)."""
    if len(msgs) != n:
        raise ValueError("one entry per party expected")
    N = t + 1
    A, ok = bytearray(32 * n * N), bytearray(n)
    for i, m in enumerate(msgs):
        if m is None or len(m.committed_coefficients) != N:
            continue
        ok[i] = 1
        A[32 * N * i:32 * N * (i + 1)] = b"".join(m.committed_coefficients)
    return bytes(A), bytes(ok)


def verify_broadcasts(be, n: int, t: int, phase1: Sequence[Optional[BroadcastPhase1]],
                      phase3: Sequence[Optional[BroadcastPhase3]]):
    """Rounds 2-5 of a plaintext-mode committee on its broadcasts (one dkg_ceremony_verify_fetched)."""
    p1 = intake_phase1(n, t, phase1, mode=0)
    A, f3 = intake_phase3(n, t, phase3)
    r = be.ceremony_verify_fetched(p1.E, A, p1.share, p1.randomness, p1.fetched1, f3, n, t)
    r.fetch_invalid = list(p1.fetch_invalid)  # receivers whose round 2 aborts (committee.rs:277-280)
    return r
