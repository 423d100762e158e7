"""Python host API over the C ABI, mirroring the reference's operator surface for this path.

Reference interface -> here:
  Environment::init(threshold, nr_members, ck_gen_bytes)      committee.rs:72-83  -> Environment
  PrimeGroupElement::vartime_multiscalar_multiplication        traits.rs:234-237   -> Backend.msm_batch
  Mul<Scalar> (generator / h)                                  traits.rs:212       -> Backend.fixed_base_batch
  Polynomial::evaluate                                         polynomial.rs:68-74 -> Backend.poly_eval_batch
  PrimeGroupElement::from_bytes (validity)                     groups.rs:78-81     -> Backend.points_valid
  Phases<Initialise>::init (all dealers)                       committee.rs:124-216 -> Backend.share_gen
  Phases<Phase1>::proceed / Phases<Phase3>::proceed checks     committee.rs:273-338, 520-559
                                                               -> Backend.verify_pairs / verify_receiver
  the all-parties test driver (full_valid_run)                 committee.rs:1518-1656 -> Backend.ceremony
Scalars and points are 32-byte encodings (bytes), exactly the reference's wire values.
"""
import ctypes
from collections.abc import Sequence
from dataclasses import dataclass
from typing import List, Optional

from . import _lib
from ._lib import BatchOut, CeremonyOut, DkgError

CK_DEFAULT = b"Example of a shared string."


def _check(ctx, rc):
    if rc != _lib.DKG_OK:
        msg = _lib.lib().dkg_ctx_last_error(ctx).decode() if ctx else ""
        raise DkgError(rc, msg)


def env_check(threshold: int, nr_members: int) -> None:
    """committee.rs:73 `assert!(threshold < (nr_members + 1) / 2)` -> DkgError(DKG_E_ARG)."""
    rc = _lib.lib().dkg_env_check(threshold, nr_members)
    if rc != _lib.DKG_OK:
        raise DkgError(rc, f"threshold {threshold} must be < (nr_members + 1) / 2 = {(nr_members + 1) // 2}")


def dealer_coefficients(master: bytes, ceremony: int, d0: int, D: int, t: int):
    """Seeded Polynomial::random pair per dealer (hiding first, committee.rs:143-146): (a, b)."""
    N = t + 1
    a = ctypes.create_string_buffer(32 * D * N)
    b = ctypes.create_string_buffer(32 * D * N)
    rc = _lib.lib().dkg_dealer_coeffs(master, ceremony, d0, D, t, a, b)
    if rc != _lib.DKG_OK:
        raise DkgError(rc, "dealer_coeffs")
    return a.raw, b.raw


def enc_randomness(master: bytes, ceremony: int, d0: int, D: int, n: int, t: int) -> bytes:
    """Encryption randomness [D][n][2][32] continuing each dealer's seeded stream (committee.rs:171-172)."""
    r = ctypes.create_string_buffer(max(64 * D * n, 1))
    rc = _lib.lib().dkg_enc_randomness(master, ceremony, d0, D, n, t, r)
    if rc != _lib.DKG_OK:
        raise DkgError(rc, "enc_randomness")
    return r.raw[:64 * D * n]


def split_multipliers(n: int, L: int, pieces: int):
    """Short recombination vectors [(b_j, a_j1, ..)] of receivers j = 1..n for a `pieces`-way split
    of piece length L (a_ju = b_j j^(uL) mod l; dkg_split_multipliers, host-only)."""
    mag = ctypes.create_string_buffer(32 * n * pieces)
    sign = ctypes.create_string_buffer(n * pieces)
    rc = _lib.lib().dkg_split_multipliers(n, L, pieces, mag, sign)
    if rc != _lib.DKG_OK:
        raise DkgError(rc, "split_multipliers")
    sg = [1 if b < 128 else -1 for b in sign.raw]
    m = mag.raw  # one copy (each .raw access copies the whole buffer)
    return [[sg[j * pieces + u] * int.from_bytes(m[(j * pieces + u) * 32:(j * pieces + u + 1) * 32], "little")
             for u in range(pieces)] for j in range(n)]


@dataclass
class CeremonyResult:
    n: int
    t: int
    mpk: bytes
    qualified: List[int]
    r2_error: List[int]
    r4_error: List[int]
    complaints2: List[int]
    reconstruct: List[int]
    n_qualified: int
    phase4_error: int
    ms: dict
    E: Optional[bytes] = None
    A: Optional[bytes] = None
    s: Optional[bytes] = None
    s_prime: Optional[bytes] = None
    dec2: Optional[bytes] = None
    dec4: Optional[bytes] = None
    final_share: Optional[bytes] = None
    public_share: Optional[bytes] = None


@dataclass
class PartyFinalise:
    """Per-party outcome of Phases<Phase5>::finalise (dkg_finalise_parties): status[p] is one of
    dkg_amd._lib.FIN_* and recovery_index[p] the dealer of InsufficientSharesForRecovery (else -1)."""
    mpk: List[bytes]
    status: List[int]
    recovery_index: List[int]


class Backend:
    """One GPU (one process per GPU).  Owns a dkg_ctx."""

    def __init__(self, device: int = 0):
        L = _lib.lib()
        h = ctypes.c_void_p()
        rc = L.dkg_ctx_create(device, ctypes.byref(h))
        if rc != _lib.DKG_OK:
            raise DkgError(rc, f"dkg_ctx_create(device={device}) failed (is a gfx950 GPU visible?)")
        self._ctx = h
        self.device = device
        self.h: Optional[bytes] = None

    def close(self):
        if self._ctx:
            _lib.lib().dkg_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self):
        return self._ctx

    def set_streams(self, nsub: int):
        """Dealer-chunk streams of the round-2/4 checks (1 = serialised, phase times recorded)."""
        _check(self._ctx, _lib.lib().dkg_ctx_set_streams(self._ctx, nsub))

    def set_verify_mode(self, mode):
        """0 / "group": difference tables (every P_i(j) in the group, default); 1 / "interp":
        committee verification by interpolation (identical decisions; dkg_ctx_set_verify_mode)."""
        m = {"group": 0, "interp": 1}.get(mode, mode)
        _check(self._ctx, _lib.lib().dkg_ctx_set_verify_mode(self._ctx, int(m)))

    def fallback_rows(self) -> int:
        return _lib.lib().dkg_ctx_fallback_rows(self._ctx)

    def set_split(self, pieces: int):
        """Degree split of the difference tables (0 = cost model, 1 = off); results are identical."""
        _check(self._ctx, _lib.lib().dkg_ctx_set_split(self._ctx, pieces))

    def set_field_mode(self, mode: int):
        """Field multiplication of the verification kernels: 0 by occupancy, 1 product scanning,
        2 column sums; results are identical."""
        _check(self._ctx, _lib.lib().dkg_ctx_set_field_mode(self._ctx, mode))

    def set_binomial(self, mode: int):
        """Binomial schedule (dkg_ctx_set_binomial): 0 (default) per-wave Horner loops for tables of
        many column groups, else one launch per step with lane pairs for the latency-bound steps; 1
        per step without lane pairs; 2 per step with lane pairs everywhere; 3 per step as 0; 4 per
        wave always; 5 per wave always with each item's operand prefetched during the previous item."""
        _check(self._ctx, _lib.lib().dkg_ctx_set_binomial(self._ctx, mode))

    def set_check(self, mode: int):
        """Fused round-2/4 checks: 0 one launch over both combs (default), 1 one launch per comb with
        g*s parked between them (dkg_ctx_set_check); decisions are identical."""
        _check(self._ctx, _lib.lib().dkg_ctx_set_check(self._ctx, mode))

    def set_stepping(self, mode: int):
        """Stepping slots: 0 cost model, 1 one per column (all pieces of a split table), 2 one per
        piece, 3 as 0 without the dead-position repack of short unsplit tables; results are identical."""
        _check(self._ctx, _lib.lib().dkg_ctx_set_stepping(self._ctx, mode))

    def set_combine(self, mode: int):
        """Recombination of a degree split: 0 short lattice multipliers for 2..4 pieces (default),
        1 powers of y = j^L; decisions are identical (dkg_ctx_set_combine)."""
        _check(self._ctx, _lib.lib().dkg_ctx_set_combine(self._ctx, mode))

    def set_stepping_formula(self, mode: int):
        """Stepping additions: 0 dedicated formula with complete redo of the workgroups that met an
        exceptional pair (default), 1 complete formula only; decisions are identical."""
        _check(self._ctx, _lib.lib().dkg_ctx_set_stepping_formula(self._ctx, mode))

    def stepping_redos(self) -> int:
        """Workgroups of the last verification's stepping redone by the complete formula."""
        r = _lib.lib().dkg_ctx_stepping_redos(self._ctx)
        if r < 0:
            raise DkgError(_lib.DKG_E_DEVICE, "dkg_ctx_stepping_redos failed")
        return r

    def binomial_reruns(self) -> int:
        """1 when the last ceremony / shard call reran its verification with the complete formula
        (a dedicated addition of the per-step binomial met an exceptional pair), else 0."""
        return _lib.lib().dkg_ctx_binomial_reruns(self._ctx)

    def clock_probe(self, iters: int = 200_000) -> dict:
        """Shader clock under full VALU occupancy (dkg_ctx_clock_probe): {"sclk_mhz", "busy_ms"}."""
        mhz, ms = ctypes.c_double(), ctypes.c_double()
        _check(self._ctx, _lib.lib().dkg_ctx_clock_probe(self._ctx, iters, ctypes.byref(mhz), ctypes.byref(ms)))
        return {"sclk_mhz": mhz.value, "busy_ms": ms.value}

    def pci_bus_id(self) -> str:
        """PCI bus id of this context's device ("dddd:bb:dd.f")."""
        return device_pci_bus_id(self.device)

    def set_addends(self, mode: int):
        """Addends of the short-multiplier recombination: 0 affine Niels (default), 1 cached
        projective; decisions are identical (dkg_ctx_set_addends)."""
        _check(self._ctx, _lib.lib().dkg_ctx_set_addends(self._ctx, mode))

    def last_combine(self) -> int:
        """0 no split, 1 powers of y, 2 short multipliers (the last verification)."""
        return _lib.lib().dkg_ctx_last_combine(self._ctx)

    def last_binomial(self) -> int:
        """0 one launch per Horner step, 1 per-wave loops (k_binom_wave) in the last verification."""
        return _lib.lib().dkg_ctx_last_binomial(self._ctx)

    def last_split(self) -> int:
        return _lib.lib().dkg_ctx_last_split(self._ctx)

    def last_split_len(self) -> int:
        """Piece length L of the last split (the last piece holds t + 1 - (U - 1) L coefficients)."""
        return _lib.lib().dkg_ctx_last_split_len(self._ctx)

    def set_overlap(self, on: bool):
        """Verify rounds 2 and 4 as one fused pipeline (default) or in protocol order."""
        _check(self._ctx, _lib.lib().dkg_ctx_set_overlap(self._ctx, 1 if on else 0))

    def phase_times(self, tag="r24") -> dict:
        """Device ms of binomial / stepping / combine / check in the last ceremony's checks: tag "r24" (rounds
        2 and 4 fused, the default schedule), "r2" or "r4" (protocol order), "full" (the hybrid
        encryption / decryption kernels of the last full-mode ceremony).  Only recorded with
        set_streams(1); -1 otherwise."""
        L = _lib.lib()
        if isinstance(tag, int):
            tag = f"r{tag}"
        names = (("interpolate", "coef_check", "decide", "fallback") if tag == "interp"
                 else ("enc_mul", "enc_encode", "enc_sym", "dec_decode", "dec_mul", "dec_encode", "dec_sym")
                 if tag == "full" else ("binomial", "stepping", "combine", "check"))
        return {k: L.dkg_ctx_phase_ms(self._ctx, f"{tag}.{k}".encode()) for k in names}

    def env_init(self, threshold: int, nr_members: int, ck_gen_bytes: bytes = CK_DEFAULT) -> bytes:
        out = ctypes.create_string_buffer(32)
        _check(self._ctx, _lib.lib().dkg_env_init(self._ctx, threshold, nr_members, ck_gen_bytes,
                                                   len(ck_gen_bytes), out))
        self.h = out.raw
        return out.raw

    # ---- trait-level batches
    def msm_batch(self, scalars: bytes, points: bytes, B: int, N: int) -> bytes:
        out = ctypes.create_string_buffer(32 * max(B, 1))
        _check(self._ctx, _lib.lib().dkg_msm_batch(self._ctx, B, N, scalars, points, out))
        return out.raw[: 32 * B]

    def fixed_base_batch(self, scalars: bytes, base: Optional[bytes] = None) -> bytes:
        count = len(scalars) // 32
        out = ctypes.create_string_buffer(32 * max(count, 1))
        _check(self._ctx, _lib.lib().dkg_fixed_base_batch(self._ctx, base, count, scalars, out))
        return out.raw[: 32 * count]

    def poly_eval_batch(self, coeffs: bytes, D: int, N: int, xs: List[int]) -> bytes:
        M = len(xs)
        arr = (ctypes.c_uint32 * max(M, 1))(*xs)
        out = ctypes.create_string_buffer(32 * max(D * M, 1))
        _check(self._ctx, _lib.lib().dkg_poly_eval_batch(self._ctx, D, N, coeffs, M, arr, out))
        return out.raw[: 32 * D * M]

    def points_valid(self, points: bytes) -> bytes:
        count = len(points) // 32
        out = ctypes.create_string_buffer(max(count, 1))
        _check(self._ctx, _lib.lib().dkg_points_valid_batch(self._ctx, count, points, out))
        return out.raw[:count]

    # ---- round 1
    def share_gen(self, a: bytes, b: bytes, D: int, n: int, t: int):
        N = t + 1
        E, A = ctypes.create_string_buffer(32 * D * N), ctypes.create_string_buffer(32 * D * N)
        s, sp = ctypes.create_string_buffer(32 * D * n), ctypes.create_string_buffer(32 * D * n)
        _check(self._ctx, _lib.lib().dkg_share_gen(self._ctx, D, n, t, a, b, E, A, s, sp))
        return E.raw, A.raw, s.raw, sp.raw

    def share_gen_device(self, D: int, n: int, t: int, d_a: int, d_b: int, d_E: Optional[int], d_A: Optional[int],
                         d_s: int, d_sp: int):
        """dkg_share_gen on device buffers (pointers): compressed E/A [D][t+1][32], shares [D][n][32]."""
        vp = ctypes.c_void_p
        _check(self._ctx, _lib.lib().dkg_share_gen_device(self._ctx, D, n, t, vp(d_a), vp(d_b), vp(d_E), vp(d_A),
                                                           vp(d_s), vp(d_sp)))

    # ---- rounds 2 / 4
    def verify_pairs(self, n: int, t: int, rnd: int, d0: int, d1: int, C: bytes, s: bytes,
                     s_prime: Optional[bytes] = None) -> bytes:
        dec = ctypes.create_string_buffer(max((d1 - d0) * n, 1))
        _check(self._ctx, _lib.lib().dkg_verify_pairs(self._ctx, n, t, rnd, d0, d1, C, s, s_prime, dec))
        return dec.raw[: (d1 - d0) * n]

    def verify_receiver(self, n: int, t: int, rnd: int, j: int, C: bytes, s_col: bytes,
                        sp_col: Optional[bytes] = None) -> bytes:
        dec = ctypes.create_string_buffer(max(n, 1))
        _check(self._ctx, _lib.lib().dkg_verify_receiver(self._ctx, n, t, rnd, j, C, s_col, sp_col, dec))
        return dec.raw[:n]

    # ---- whole ceremony
    def _ceremony_out(self, n, t, big):
        N = t + 1
        bufs = {}
        o = CeremonyOut()
        sizes = {"qualified": n, "r2_error": n, "r4_error": n, "complaints2": 4 * n, "reconstruct": n}
        if big:
            sizes.update({"E": 32 * n * N, "A": 32 * n * N, "s": 32 * n * n, "s_prime": 32 * n * n,
                          "dec2": n * n, "dec4": n * n, "final_share": 32 * n, "public_share": 32 * n})
        for k, v in sizes.items():
            bufs[k] = ctypes.create_string_buffer(v)
            setattr(o, k, ctypes.cast(bufs[k], ctypes.c_void_p))
        return o, bufs

    def _result(self, n, t, o, bufs, big):
        import struct
        r = CeremonyResult(
            n=n, t=t, mpk=bytes(o.mpk), qualified=list(bufs["qualified"].raw[:n]),
            r2_error=list(bufs["r2_error"].raw[:n]), r4_error=list(bufs["r4_error"].raw[:n]),
            complaints2=list(struct.unpack(f"<{n}i", bufs["complaints2"].raw[: 4 * n])),
            reconstruct=list(bufs["reconstruct"].raw[:n]), n_qualified=o.n_qualified,
            phase4_error=o.phase4_error,
            ms={"round1": o.ms_round1, "round2": o.ms_round2, "round3": o.ms_round3, "round4": o.ms_round4,
                "finalise": o.ms_finalise, "total": o.ms_total})
        if big:
            for k in ("E", "A", "s", "s_prime", "dec2", "dec4", "final_share", "public_share"):
                setattr(r, k, bufs[k].raw)
        return r

    def ceremony(self, a: bytes, b: bytes, n: int, t: int) -> CeremonyResult:
        o, bufs = self._ceremony_out(n, t, True)
        _check(self._ctx, _lib.lib().dkg_ceremony_run(self._ctx, n, t, a, b, ctypes.byref(o)))
        return self._result(n, t, o, bufs, True)

    def ceremony_verify(self, E: bytes, A: bytes, s: bytes, s_prime: bytes, n: int, t: int) -> CeremonyResult:
        o, bufs = self._ceremony_out(n, t, True)
        for k in ("E", "A", "s", "s_prime"):
            setattr(o, k, None)
        _check(self._ctx, _lib.lib().dkg_ceremony_verify(self._ctx, n, t, E, A, s, s_prime, ctypes.byref(o)))
        r = self._result(n, t, o, bufs, True)
        r.E, r.A, r.s, r.s_prime = E, A, s, s_prime
        return r

    def ceremony_verify_fetched(self, E: bytes, A: bytes, s: bytes, s_prime: bytes, fetched1: bytes,
                                fetched3: bytes, n: int, t: int) -> CeremonyResult:
        """ceremony_verify after the broadcast intake (MembersFetchedState1/3::from_broadcast):
        fetched1[i] / fetched3[i] = 0 for a dealer whose phase-1 / phase-3 broadcast is absent or
        malformed (see dkg_amd.broadcast)."""
        o, bufs = self._ceremony_out(n, t, True)
        for k in ("E", "A", "s", "s_prime"):
            setattr(o, k, None)
        _check(self._ctx, _lib.lib().dkg_ceremony_verify_fetched(self._ctx, n, t, E, A, s, s_prime, fetched1,
                                                                 fetched3, ctypes.byref(o)))
        r = self._result(n, t, o, bufs, True)
        r.E, r.A, r.s, r.s_prime = E, A, s, s_prime
        return r

    def ceremony_device(self, d_a: int, d_b: int, n: int, t: int) -> CeremonyResult:
        """d_a, d_b: device pointers (e.g. torch tensor .data_ptr()) to [n][t+1][32] scalars."""
        o, bufs = self._ceremony_out(n, t, False)
        _check(self._ctx, _lib.lib().dkg_ceremony_run_device(self._ctx, n, t, ctypes.c_void_p(d_a),
                                                              ctypes.c_void_p(d_b), ctypes.byref(o)))
        return self._result(n, t, o, bufs, False)

    # ---- full (encrypted-share) mode
    def member_keys(self, master: bytes, ceremony: int, n: int):
        """Seeded member communication keys, sorted by public key (party q+1 owns sk[q]): (sk, pk)."""
        sk, pk = ctypes.create_string_buffer(32 * n), ctypes.create_string_buffer(32 * n)
        _check(self._ctx, _lib.lib().dkg_member_keys(self._ctx, master, ceremony, n, sk, pk))
        return sk.raw, pk.raw

    def encrypt_shares(self, pk: bytes, s: bytes, s_prime: bytes, r: bytes, D: int, n: int):
        e1, ct = ctypes.create_string_buffer(64 * D * n), ctypes.create_string_buffer(64 * D * n)
        _check(self._ctx, _lib.lib().dkg_encrypt_shares(self._ctx, D, n, pk, s, s_prime, r, e1, ct))
        return e1.raw, ct.raw

    def decrypt_shares(self, sk: bytes, e1: bytes, ct: bytes, D: int, n: int):
        s, sp, ok = (ctypes.create_string_buffer(32 * D * n), ctypes.create_string_buffer(32 * D * n),
                     ctypes.create_string_buffer(2 * D * n))
        _check(self._ctx, _lib.lib().dkg_decrypt_shares(self._ctx, D, n, sk, e1, ct, s, sp, ok))
        return s.raw, sp.raw, ok.raw

    def enc_randomness_device(self, master: bytes, ceremony0: int, B: int, d0: int, D: int, n: int, t: int, d_r: int):
        _check(self._ctx, _lib.lib().dkg_enc_randomness_device(self._ctx, master, ceremony0, B, d0, D, n, t,
                                                                ctypes.c_void_p(d_r)))

    def ceremony_full_device(self, d_a: int, d_b: int, d_r: int, sk: bytes, pk: bytes, n: int, t: int):
        o, bufs = self._ceremony_out(n, t, False)
        vp = ctypes.c_void_p
        _check(self._ctx, _lib.lib().dkg_ceremony_run_full_device(self._ctx, n, t, vp(d_a), vp(d_b), vp(d_r), sk, pk,
                                                                   ctypes.byref(o)))
        return self._result(n, t, o, bufs, False)

    def ceremony_verify_full(self, E: bytes, A: bytes, e1: bytes, ct: bytes, sk: bytes, n: int, t: int):
        o, bufs = self._ceremony_out(n, t, True)
        for k in ("E", "A"):
            setattr(o, k, None)
        _check(self._ctx, _lib.lib().dkg_ceremony_verify_full(self._ctx, n, t, E, A, e1, ct, sk, ctypes.byref(o)))
        r = self._result(n, t, o, bufs, True)
        r.E, r.A = E, A
        return r

    # ---- complaint proofs (broadcast.rs)
    def misbehaviour_prove(self, sk: bytes, enc: bytes, w: bytes) -> bytes:
        """ProofOfMisbehaviour::generate for B = len(sk) // 32 complaints: proofs [B][192]."""
        B = len(sk) // 32
        out = ctypes.create_string_buffer(max(192 * B, 1))
        _check(self._ctx, _lib.lib().dkg_misbehaviour_prove(self._ctx, B, sk, enc, w, out))
        return out.raw[:192 * B]

    def complaint1_verify(self, t: int, accusers: List[int], pk: bytes, enc: bytes, E: bytes, proofs: bytes):
        B = len(accusers)
        acc = (ctypes.c_uint32 * max(B, 1))(*accusers)
        res = (ctypes.c_int32 * max(B, 1))()
        _check(self._ctx, _lib.lib().dkg_complaint1_verify(self._ctx, B, t, acc, pk, enc, E, proofs, res))
        return list(res)[:B]

    def complaint3_verify(self, t: int, accusers: List[int], share: bytes, randomness: bytes, E: bytes, A: bytes):
        B = len(accusers)
        acc = (ctypes.c_uint32 * max(B, 1))(*accusers)
        res = (ctypes.c_int32 * max(B, 1))()
        _check(self._ctx, _lib.lib().dkg_complaint3_verify(self._ctx, B, t, acc, share, randomness, E, A, res))
        return list(res)[:B]

    def dealer_coefficients_device(self, master: bytes, ceremony0: int, B: int, d0: int, D: int, t: int,
                                   d_a: int, d_b: int):
        """dkg_dealer_coeffs on the GPU for B ceremonies: rows [B*D][t+1][32] at device pointers."""
        vp = ctypes.c_void_p
        _check(self._ctx, _lib.lib().dkg_dealer_coeffs_device(self._ctx, master, ceremony0, B, d0, D, t, vp(d_a),
                                                               vp(d_b)))

    def ceremony_shard_device(self, n, t, d0, d1, d_a, d_b, d_dec2, d_dec4, d_A0, d_partial) -> float:
        ms = ctypes.c_double()
        vp = ctypes.c_void_p
        _check(self._ctx, _lib.lib().dkg_ceremony_shard_device(self._ctx, n, t, d0, d1, vp(d_a), vp(d_b),
                                                                vp(d_dec2), vp(d_dec4), vp(d_A0),
                                                                vp(d_partial), ctypes.byref(ms)))
        return ms.value

    def ceremony_shard_verify_device(self, n, t, d0, d1, d_E, d_A, d_s, d_sp, d_dec2, d_dec4, d_A0,
                                     d_partial) -> float:
        """Rounds 2-5 of this rank's dealers [d0, d1) on received broadcasts (device pointers)."""
        ms = ctypes.c_double()
        vp = ctypes.c_void_p
        _check(self._ctx, _lib.lib().dkg_ceremony_shard_verify_device(
            self._ctx, n, t, d0, d1, vp(d_E), vp(d_A), vp(d_s), vp(d_sp), vp(d_dec2), vp(d_dec4), vp(d_A0),
            vp(d_partial), ctypes.byref(ms)))
        return ms.value

    def ceremony_shard_recon_device(self, n, t, d0, d1, qualified, reconstruct, d_s: Optional[int], d_terms: int,
                                    r2_error=None, r4_error=None) -> bool:
        """After the exchange: replace the terms of this rank's reconstructed dealers by g * a_i0
        interpolated over the disclosing final parties' shares (no r2 / r4 error; d_s None = the
        last shard call's rows).  Returns True when fewer than t final parties disclose
        (InsufficientSharesForRecovery for everyone: no mpk; the terms are untouched)."""
        vp = ctypes.c_void_p
        opt = lambda m: None if m is None else bytes(bytearray(m))  # noqa: E731
        fails = ctypes.c_int32(0)
        _check(self._ctx, _lib.lib().dkg_ceremony_shard_recon_device(
            self._ctx, n, t, d0, d1, bytes(bytearray(qualified)), bytes(bytearray(reconstruct)), opt(r2_error),
            opt(r4_error), vp(d_s), vp(d_terms), ctypes.byref(fails)))
        return bool(fails.value)

    def finalise_parties(self, n: int, t: int, qualified, reconstruct, A0: bytes, s: bytes, r2_error=None,
                         r4_error=None, disclosed=None) -> "PartyFinalise":
        """Phases<Phase5>::finalise as every party runs it (committee.rs:726-805), with optional
        per-party earlier failures and missing phase-5 disclosures (dkg_finalise_parties)."""
        mpk = ctypes.create_string_buffer(32 * max(n, 1))
        st = (ctypes.c_int32 * max(n, 1))()
        ri = (ctypes.c_int32 * max(n, 1))()
        mask = lambda x: None if x is None else bytes(bytearray(x))  # noqa: E731
        _check(self._ctx, _lib.lib().dkg_finalise_parties(
            self._ctx, n, t, mask(qualified), mask(reconstruct), mask(r2_error), mask(r4_error), mask(disclosed),
            A0, s, mpk, st, ri))
        m = mpk.raw
        return PartyFinalise([m[32 * p:32 * p + 32] for p in range(n)], list(st)[:n], list(ri)[:n])

    def shard_combine_device(self, n: int, t: int, world_size: int, d_dec2_g: int, d_dec4_g: int,
                             d_dec2: Optional[int] = None, d_dec4: Optional[int] = None,
                             packed: bool = False, arrays: bool = False) -> "ShardOutcome":
        """Combine step of the sharded run (dkg_shard_combine_device): the common round-2/4 outcome
        from the all-gathered [ws][R][n] decision blocks (device pointers; with packed, the
        [ws][R][packed_row_words(n)] bitmaps of dkg_shard_combine_packed_device); d_dec2 / d_dec4
        optionally receive the compacted [n][n] matrices (dec4 with SKIPPED rows).  arrays: the
        per-party outcomes as numpy arrays (uint8 / int32) instead of lists -- no per-element
        conversion on the multi-GPU driver's path."""
        q, r2e, rc, r4e = (ctypes.create_string_buffer(max(n, 1)) for _ in range(4))
        c = (ctypes.c_int32 * max(n, 1))()
        o = _lib.ShardOutcome(ctypes.cast(q, ctypes.c_void_p), ctypes.cast(c, ctypes.c_void_p),
                              ctypes.cast(r2e, ctypes.c_void_p), ctypes.cast(rc, ctypes.c_void_p),
                              ctypes.cast(r4e, ctypes.c_void_p), 0, 0)
        vp = ctypes.c_void_p
        fn = _lib.lib().dkg_shard_combine_packed_device if packed else _lib.lib().dkg_shard_combine_device
        _check(self._ctx, fn(self._ctx, n, t, world_size, vp(d_dec2_g), vp(d_dec4_g), vp(d_dec2), vp(d_dec4),
                             ctypes.byref(o)))
        if arrays:
            import numpy as np

            u8 = lambda b: np.frombuffer(b.raw, dtype=np.uint8, count=n).copy()  # noqa: E731
            return ShardOutcome(u8(q), np.frombuffer(c, dtype=np.int32, count=n).copy(), u8(r2e), u8(rc), u8(r4e),
                                o.n_qualified, bool(o.phase4_error))
        return ShardOutcome(list(q.raw[:n]), list(c)[:n], list(r2e.raw[:n]), list(rc.raw[:n]), list(r4e.raw[:n]),
                            o.n_qualified, bool(o.phase4_error))

    def decisions_pack_device(self, rows: int, nvalid: int, n: int, d0: int, d_dec: int, d_packed: int):
        """Raw decision rows of dealers d0.. (device [nvalid][n] bytes) -> the packed bitmaps the ranks
        all-gather (device [rows][packed_row_words(n)] u32; dkg_decisions_pack_device).  Raises if a
        row holds values the encoding cannot carry."""
        vp = ctypes.c_void_p
        _check(self._ctx, _lib.lib().dkg_decisions_pack_device(self._ctx, rows, nvalid, n, d0, vp(d_dec),
                                                                vp(d_packed)))

    def shard_finalise_device(self, n: int, t: int, world_size: int, d_terms_g: int, d_partials_g: int, qualified,
                              phase4_error: bool, d_final_share: int, d_public_share: Optional[int] = None) -> bytes:
        """Finalise of the sharded run (dkg_shard_finalise_device): final shares (and public shares)
        into device buffers; returns the mpk (zero when phase4_error)."""
        mpk = ctypes.create_string_buffer(32)
        vp = ctypes.c_void_p
        _check(self._ctx, _lib.lib().dkg_shard_finalise_device(
            self._ctx, n, t, world_size, vp(d_terms_g), vp(d_partials_g), bytes(bytearray(qualified)),
            int(bool(phase4_error)), vp(d_final_share), vp(d_public_share), mpk))
        return mpk.raw

    def scalar_sum_device(self, rows: int, n: int, d_in: int, d_mask: Optional[int], d_out: int):
        """out[j] = sum over rows r with mask[r] of in[r][j] mod l (device pointers)."""
        vp = ctypes.c_void_p
        _check(self._ctx, _lib.lib().dkg_scalar_sum_device(self._ctx, rows, n, vp(d_in), vp(d_mask), vp(d_out)))

    def point_sum_device(self, count: int, d_points: int, d_mask: Optional[int], d_out: int):
        """out = sum of the compressed points[c] with mask[c] (device pointers)."""
        vp = ctypes.c_void_p
        _check(self._ctx, _lib.lib().dkg_point_sum_device(self._ctx, count, vp(d_points), vp(d_mask), vp(d_out)))


class _ShardView(Backend):
    """A shard's dkg_ctx inside a MultiBackend (owned by the multi-device context: close is a no-op)."""

    def __init__(self, ctx, owner):
        self._ctx, self.h, self._owner = ctx, None, owner

    def close(self):
        self._ctx = None


class MultiBackend:
    """Several GPUs driven from ONE process (dkg_multi_*, SURVEY.md section 8(b) threading row): the
    ceremony sharded by dealer over `devices`, exchanged by peer copies into devices[0], combined and
    finalised there.  Results equal Backend.ceremony / ceremony_verify's except that E, A, s,
    s_prime are not returned (they stay on the shards' devices).  A device may repeat."""

    def __init__(self, devices):
        L = _lib.lib()
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        rc = L.dkg_multi_create(devs, len(devices), ctypes.byref(h))
        if rc != _lib.DKG_OK:
            raise DkgError(rc, f"dkg_multi_create(devices={list(devices)}) failed (are gfx950 GPUs visible?)")
        self._m = h
        self.devices = list(devices)
        self.h: Optional[bytes] = None

    def close(self):
        if self._m:
            _lib.lib().dkg_multi_destroy(self._m)
            self._m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != _lib.DKG_OK:
            raise DkgError(rc, _lib.lib().dkg_multi_last_error(self._m).decode())

    def __len__(self):
        return _lib.lib().dkg_multi_size(self._m)

    def shard(self, i: int) -> Backend:
        """Shard i's context, for its tuning knobs (set_split, set_streams, ...)."""
        ctx = _lib.lib().dkg_multi_ctx(self._m, i)
        if not ctx:
            raise DkgError(_lib.DKG_E_ARG, f"no shard {i}")
        return _ShardView(ctypes.c_void_p(ctx), self)

    def phase_ms(self) -> dict:
        L = _lib.lib()
        return {k: L.dkg_multi_phase_ms(self._m, k.encode())
                for k in ("shard_max", "shard_min", "exchange", "combine", "recon", "finalise")}

    def env_init(self, threshold: int, nr_members: int, ck_gen_bytes: bytes = CK_DEFAULT) -> bytes:
        out = ctypes.create_string_buffer(32)
        self._check(_lib.lib().dkg_multi_env_init(self._m, threshold, nr_members, ck_gen_bytes, len(ck_gen_bytes),
                                                  out))
        self.h = out.raw
        return out.raw

    def _out(self, n, t):
        o, bufs = Backend._ceremony_out(None, n, t, True)
        for k in ("E", "A", "s", "s_prime"):
            setattr(o, k, None)
        return o, bufs

    def _result(self, n, t, o, bufs):
        r = Backend._result(None, n, t, o, bufs, False)
        for k in ("dec2", "dec4", "final_share", "public_share"):
            setattr(r, k, bufs[k].raw)
        return r

    def ceremony(self, a: bytes, b: bytes, n: int, t: int) -> CeremonyResult:
        o, bufs = self._out(n, t)
        self._check(_lib.lib().dkg_multi_ceremony_run(self._m, n, t, a, b, ctypes.byref(o)))
        return self._result(n, t, o, bufs)

    def ceremony_device(self, d_as, d_bs, n: int, t: int) -> CeremonyResult:
        """d_as[i], d_bs[i]: device pointers on devices[i] to shard i's dealers' coefficients."""
        k = len(self.devices)
        pa = (ctypes.c_void_p * k)(*d_as)
        pb = (ctypes.c_void_p * k)(*d_bs)
        o, bufs = self._out(n, t)
        self._check(_lib.lib().dkg_multi_ceremony_run_device(self._m, n, t, pa, pb, ctypes.byref(o)))
        return self._result(n, t, o, bufs)

    def ceremony_verify(self, E: bytes, A: bytes, s: bytes, s_prime: bytes, n: int, t: int) -> CeremonyResult:
        o, bufs = self._out(n, t)
        self._check(_lib.lib().dkg_multi_ceremony_verify(self._m, n, t, E, A, s, s_prime, ctypes.byref(o)))
        return self._result(n, t, o, bufs)


@dataclass
class ShardOutcome:
    """The common outcome of a sharded ceremony (dkg_shard_combine_device), identical on every rank."""
    qualified: List[int]
    complaints2: List[int]
    r2_error: List[int]
    reconstruct: List[int]
    r4_error: List[int]
    n_qualified: int
    phase4_error: bool


def shard_range(n: int, world_size: int, rank: int):
    """Dealers [d0, d1) of `rank` (dkg_shard_range: contiguous, sizes differ by at most one)."""
    d0, d1 = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.lib().dkg_shard_range(n, world_size, rank, ctypes.byref(d0), ctypes.byref(d1))
    return d0.value, d1.value


def device_pci_bus_id(device: int) -> str:
    """PCI bus id ("dddd:bb:dd.f") of HIP device `device` (dkg_device_pci_bus_id)."""
    b = ctypes.create_string_buffer(64)
    rc = _lib.lib().dkg_device_pci_bus_id(device, b, len(b))
    if rc != _lib.DKG_OK:
        raise DkgError(rc, f"dkg_device_pci_bus_id({device}) failed")
    return b.value.decode()


def shard_rows(n: int, world_size: int) -> int:
    """Padded per-rank block height R of the all-gathers (dkg_shard_rows)."""
    return _lib.lib().dkg_shard_rows(n, world_size)


def packed_row_words(n: int) -> int:
    """u32 words of one packed decision row (dkg_packed_row_words: ceil(n/32) ACCEPT-bit words + a kind word)."""
    return _lib.lib().dkg_packed_row_words(n)


@dataclass
class BatchResult:
    """Outputs of B independent ceremonies (row c*n + i = party i of ceremony c)."""
    B: int
    n: int
    t: int
    mpk: List[bytes]
    n_qualified: List[int]
    phase4_error: bytes
    qualified: bytes
    r2_error: bytes
    r4_error: bytes
    complaints2: "Int32s"  # list-like: indexing, slices (lists), iteration, == with a list
    reconstruct: bytes
    final_share: Optional[bytes]
    public_share: Optional[bytes]
    dec2: Optional[bytes]
    dec4: Optional[bytes]
    ms: dict

    def ceremony(self, c: int) -> dict:
        """The outputs of ceremony c in the layout of a single CeremonyResult."""
        n = self.n
        r = slice(c * n, (c + 1) * n)
        d = {"mpk": self.mpk[c], "n_qualified": self.n_qualified[c], "phase4_error": self.phase4_error[c],
             "qualified": list(self.qualified[r]),
             "r2_error": list(self.r2_error[r]), "r4_error": list(self.r4_error[r]),
             "complaints2": self.complaints2[r],
             "reconstruct": list(self.reconstruct[r])}
        for k in ("final_share", "public_share"):
            v = getattr(self, k)
            d[k] = v[32 * n * c:32 * n * (c + 1)] if v is not None else None
        for k in ("dec2", "dec4"):
            v = getattr(self, k)
            d[k] = v[n * n * c:n * n * (c + 1)] if v is not None else None
        return d


def _batch_out(B, n, big):
    import struct  # noqa: F401
    V = B * n
    sizes = {"mpk": 32 * B, "n_qualified": 4 * B, "phase4_error": B, "qualified": V, "r2_error": V, "r4_error": V,
             "complaints2": 4 * V,
             "reconstruct": V}
    if big:
        sizes.update({"final_share": 32 * V, "public_share": 32 * V, "dec2": V * n, "dec4": V * n})
    o = BatchOut()
    bufs = {}
    for k, v in sizes.items():
        bufs[k] = ctypes.create_string_buffer(max(v, 1))
        setattr(o, k, ctypes.cast(bufs[k], ctypes.c_void_p))
    return o, bufs


class Int32s(Sequence):
    """Little-endian int32 rows of a batch output, converted to Python ints only where read: a
    10,000-ceremony batch holds 640,000 of them, and building the whole list up front costs more
    host time than the ceremonies' round 3.  A read-only Sequence (len, indexing, slices -> list,
    iteration, `in`, index, count, == against any sequence); tolist() / list(x) for a list (JSON,
    concatenation).  Unhashable, like the list it stands for."""

    def __init__(self, raw: bytes):
        self._mv = memoryview(raw).cast("i")

    def __len__(self):
        return len(self._mv)

    def __getitem__(self, i):
        return self._mv[i].tolist() if isinstance(i, slice) else self._mv[i]

    def __iter__(self):
        return iter(self._mv.tolist())

    def __eq__(self, other):
        try:
            return self._mv.tolist() == list(other)
        except TypeError:
            return NotImplemented

    __hash__ = None

    def __add__(self, other):
        return self._mv.tolist() + list(other)

    def __repr__(self):
        return f"Int32s({self._mv.tolist()!r})" if len(self) <= 16 else f"Int32s(<{len(self)} values>)"

    def tolist(self):
        return self._mv.tolist()


def _batch_result(B, n, t, o, bufs):
    import struct
    V = B * n
    g = lambda k, size: bufs[k].raw[:size] if k in bufs else None  # noqa: E731
    mpk = bufs["mpk"].raw  # one copy (each .raw access copies the whole buffer)
    return BatchResult(
        B=B, n=n, t=t, mpk=[mpk[32 * c:32 * c + 32] for c in range(B)],
        n_qualified=list(struct.unpack(f"<{B}i", bufs["n_qualified"].raw[:4 * B])),
        phase4_error=g("phase4_error", B),
        qualified=g("qualified", V), r2_error=g("r2_error", V), r4_error=g("r4_error", V),
        complaints2=Int32s(bufs["complaints2"].raw[:4 * V]),
        reconstruct=g("reconstruct", V), final_share=g("final_share", 32 * V), public_share=g("public_share", 32 * V),
        dec2=g("dec2", V * n), dec4=g("dec4", V * n),
        ms={"round1": o.ms_round1, "checks": o.ms_checks, "round3": o.ms_round3, "finalise": o.ms_finalise,
            "total": o.ms_total})


def ceremony_batch_device(be: "Backend", B: int, n: int, t: int, d_a: int, d_b: int, big: bool = False) -> BatchResult:
    """B honest ceremonies from device coefficients [B*n][t+1][32] (dkg_ceremony_batch_device).  The
    output buffers are kept on the backend for the next batch of the same shape (the result holds
    copies): a 10,000-ceremony batch no longer allocates and zeroes ~5 MB of host buffers per call."""
    key = (B, n, big)
    cache = getattr(be, "_batch_bufs", None)
    if cache is None or cache[0] != key:
        cache = (key,) + _batch_out(B, n, big)
        be._batch_bufs = cache
    o, bufs = cache[1], cache[2]
    _check(be.ctx, _lib.lib().dkg_ceremony_batch_device(be.ctx, B, n, t, ctypes.c_void_p(d_a), ctypes.c_void_p(d_b),
                                                          ctypes.byref(o)))
    return _batch_result(B, n, t, o, bufs)


def ceremony_batch_verify(be: "Backend", B: int, n: int, t: int, E: bytes, A: bytes, s: bytes,
                          s_prime: bytes) -> BatchResult:
    """Receiver side of B ceremonies from (possibly tampered) broadcast values (dkg_ceremony_batch_verify)."""
    o, bufs = _batch_out(B, n, True)
    _check(be.ctx, _lib.lib().dkg_ceremony_batch_verify(be.ctx, B, n, t, E, A, s, s_prime, ctypes.byref(o)))
    return _batch_result(B, n, t, o, bufs)


class Environment:
    """committee.rs:24-28 / :72-83 — threshold, nr_members and the Pedersen commitment key h."""

    def __init__(self, backend: Backend, threshold: int, nr_members: int, ck_gen_bytes: bytes = CK_DEFAULT):
        env_check(threshold, nr_members)
        self.threshold = threshold
        self.nr_members = nr_members
        self.commitment_key = backend.env_init(threshold, nr_members, ck_gen_bytes)
