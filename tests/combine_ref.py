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


def packed_words(n):
    """u32 words per packed decision row (include/dkg_amd.h dkg_packed_row_words)."""
    return (n + 31) // 32 + 1


def pack_rows(dec, rows, nvalid, n, d0):
    """Raw decision rows of dealers d0..d0+nvalid-1 ([nvalid][n] uint8) -> [rows][W+1] uint32, the
    encoding of dkg_decisions_pack_device restated: ACCEPT bits (bit j % 32 of word j // 32), then the
    row kind (0 checked, 1 MISSING row, 2 SKIPPED row); the diagonal is implied; padding rows zero.
    Raises ValueError on a row the encoding cannot carry."""
    W = (n + 31) // 32
    out = np.zeros((rows, W + 1), dtype=np.uint32)
    d = _u8(dec).reshape(-1)[:nvalid * n].reshape(nvalid, n)
    for r in range(nvalid):
        row, self_ = d[r], d0 + r
        off = np.ones(n, dtype=bool)
        off[self_] = False
        if row[self_] != SELF:
            raise ValueError(f"row {r}: diagonal is not SELF")
        vals = set(row[off].tolist())
        kind = 1 if vals == {MISSING} else 2 if vals == {SKIPPED} else 0
        if kind == 0 and not vals <= {REJECT, ACCEPT}:
            raise ValueError(f"row {r}: values {sorted(vals)} do not fit the packed encoding")
        if kind == 0:
            bits = np.zeros(32 * W, dtype=np.uint64)
            bits[:n] = (row == ACCEPT) & off
            out[r, :W] = (bits.reshape(W, 32) << np.arange(32, dtype=np.uint64)).sum(axis=1).astype(np.uint32)
        out[r, W] = kind
    return out


def unpack_ranks(gathered, ws, n):
    """All-gathered packed blocks [ws][R][W+1] (flat uint32) -> dense [n][n] uint8 decisions."""
    R, W = rows_per_rank(ws, n), (n + 31) // 32
    g = np.asarray(gathered, dtype=np.uint32).reshape(ws, R, W + 1)
    out = np.empty((n, n), dtype=np.uint8)
    for r in range(ws):
        a, b = dealer_range(r, ws, n)
        for k in range(b - a):
            i, kind = a + k, int(g[r, k, W])
            if kind:
                out[i] = MISSING if kind == 1 else SKIPPED
            else:
                bits = (g[r, k, :W, None].astype(np.uint64) >> np.arange(32, dtype=np.uint64)) & 1
                out[i] = bits.reshape(-1)[:n].astype(np.uint8)
            out[i, i] = SELF
    return out


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
