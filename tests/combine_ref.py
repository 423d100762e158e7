"""Checker (test infrastructure only): the sharded run's combine step restated in numpy.

The rules every party applies to the all-gathered decision rows (committee.rs:311-347, 370-398,
515-569, 660-677), written independently of the library's round2_outcome / round4_outcome
(dkg_amd/csrc/runtime.hip), so that tests can compare dkg_shard_combine_device against it on golden,
random and fault-injected decision matrices.  Also the compaction of padded per-rank blocks.
"""
from dataclasses import dataclass

import numpy as np

REJECT, ACCEPT, SELF, SKIPPED, MISSING = 0, 1, 2, 3, 4


def _u8(x):
    """uint8 array view of bytes / bytearray / arrays / tensors already on the host."""
    if isinstance(x, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(x), dtype=np.uint8)
    return np.asarray(x, dtype=np.uint8)


def dealer_range(rank, ws, n):
    return (rank * n) // ws, ((rank + 1) * n) // ws


def rows_per_rank(ws, n):
    return max(dealer_range(r, ws, n)[1] - dealer_range(r, ws, n)[0] for r in range(ws))


def compact(gathered, ws, n, width):
    """[ws][R][width] padded blocks (flat) -> dense [n][width] (numpy uint8)."""
    R = rows_per_rank(ws, n)
    g = _u8(gathered).reshape(ws, R, width)
    return np.concatenate([g[r, :dealer_range(r, ws, n)[1] - dealer_range(r, ws, n)[0]] for r in range(ws)])


def pad(dense, ws, n, width, fill=0xEE):
    """dense [n][width] -> the [ws][R][width] layout an all-gather produces (padding rows = fill)."""
    R = rows_per_rank(ws, n)
    d = _u8(dense).reshape(n, width)
    out = np.full((ws, R, width), fill, dtype=np.uint8)
    for r in range(ws):
        a, b = dealer_range(r, ws, n)
        out[r, :b - a] = d[a:b]
    return out.reshape(-1)


@dataclass
class Outcome:
    dec2: np.ndarray
    dec4: np.ndarray          # SKIPPED rows applied
    qualified: np.ndarray
    complaints2: np.ndarray
    r2_error: np.ndarray
    reconstruct: np.ndarray
    r4_error: np.ndarray
    phase4_error: bool


def combine(dec2, dec4, n, t) -> Outcome:
    """A REJECT by receiver j is a complaint of j against dealer i and a valid complaint disqualifies i
    for everyone (committee.rs:311-316, 370-398); MISSING (undecodable broadcast) disqualifies without
    a complaint (:331-335); more than t complaints raise MisbehaviourHigherThreshold for j (:340-347);
    disqualified dealers are skipped in round 4 (:522); a round-4 REJECT puts a qualified dealer in the
    reconstruction set (:660-670); receiver j counts itself plus the qualified dealers it accepted in
    round 4 (:515-516, 567-569); qualified minus reconstructable <= t fails Phase4 (:673-677)."""
    dec2 = _u8(dec2).reshape(n, n)
    dec4 = _u8(dec4).reshape(n, n).copy()
    rej2 = dec2 == REJECT
    qualified = (~(rej2 | (dec2 == MISSING)).any(axis=1)).astype(np.uint8)
    complaints = rej2.sum(axis=0).astype(np.int32)
    r2_error = (complaints > t).astype(np.uint8)
    off = ~np.eye(n, dtype=bool)
    raw4 = dec4.copy()
    dec4[(qualified == 0)[:, None] & off] = SKIPPED
    recon = ((raw4 == REJECT) & (qualified == 1)[:, None]).any(axis=1).astype(np.uint8)
    honest4 = 1 + ((raw4 == ACCEPT) & off & (qualified == 1)[:, None]).sum(axis=0)
    r4_error = (honest4 < t + 1).astype(np.uint8)
    honest = qualified & (1 - recon)
    return Outcome(dec2, dec4, qualified, complaints, r2_error, recon, r4_error, bool(int(honest.sum()) <= t))
