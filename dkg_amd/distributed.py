"""Multi-GPU ceremony: one process per GPU, the ceremony sharded by dealer.

Rank r owns dealers [r*n/ws, (r+1)*n/ws): it generates their commitments and shares and checks their
rows against all n receivers on its GPU (dkg_ceremony_shard_device).  The protocol's exchange step --
every party learns every complaint (committee.rs:311-331, 370-398) and the round-3/5 broadcasts
(committee.rs:454-467, 790-795) -- is a set of all-gathers (RCCL over xGMI with the "nccl" backend,
gloo in the CPU tests) of:
  * the round-2 / round-4 decision rows,
  * every dealer's compressed master-key term (A_i0, or g * a_i0 recovered by Lagrange
    interpolation on the owning rank for dealers accused in round 4),
  * each rank's partial final shares (sum over its qualified dealers of s_ij).
combine_decisions() then derives, identically on every rank, what receivers_rounds() in runtime.hip
derives on one GPU: qualified set, complaints, r2 errors, round-4 SKIPPED marks, reconstruction set.
"""
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ._lib import ACCEPT, MISSING, REJECT, SKIPPED


def dealer_range(rank: int, world_size: int, n: int):
    """Dealers owned by `rank` (contiguous, sizes differ by at most one)."""
    return (rank * n) // world_size, ((rank + 1) * n) // world_size


def max_rows(world_size: int, n: int) -> int:
    return max(dealer_range(r, world_size, n)[1] - dealer_range(r, world_size, n)[0] for r in range(world_size))


@dataclass
class Decisions:
    dec2: np.ndarray          # [n][n] uint8 (a torch tensor on the exchange device when combined there)
    dec4: np.ndarray          # [n][n] uint8, SKIPPED rows for disqualified dealers (idem)
    qualified: np.ndarray     # [n] uint8
    complaints2: np.ndarray   # [n] int32, complaints raised by receiver j
    r2_error: np.ndarray      # [n] uint8, receiver j saw more than t complaints
    reconstruct: np.ndarray   # [n] uint8, qualified dealers accused in round 4
    r4_error: np.ndarray      # [n] uint8, receiver j saw fewer than t+1 honest dealers in round 4
    honest: np.ndarray        # [n] uint8, qualified and not reconstructed (their A_i0 enter mpk)
    phase4_error: bool        # qualified minus reconstructable <= t: Phase4::proceed fails (:673-677)


def combine_decisions(dec2, dec4, n: int, t: int) -> Decisions:
    """See _combine_np; torch tensors (e.g. the gathered rows, still on the GPU) are combined on
    their device and only the per-party vectors come back to the host (dec2 / dec4 stay tensors)."""
    if not isinstance(dec2, np.ndarray) and hasattr(dec2, "device"):
        return _combine_torch(dec2, dec4, n, t)
    return _combine_np(dec2, dec4, n, t)


def _combine_torch(dec2, dec4, n: int, t: int) -> Decisions:
    import torch

    d2 = dec2.reshape(n, n)
    d4 = dec4.reshape(n, n).clone()
    rej2 = d2 == REJECT
    qualified = ~(rej2 | (d2 == MISSING)).any(dim=1)
    complaints = rej2.sum(dim=0, dtype=torch.int32)
    off = ~torch.eye(n, dtype=torch.bool, device=d2.device)
    d4[(~qualified)[:, None] & off] = SKIPPED
    recon = ((d4 == REJECT) & off & qualified[:, None]).any(dim=1)
    honest = qualified & ~recon
    honest4 = 1 + ((d4 == ACCEPT) & off & qualified[:, None]).sum(dim=0)
    small = torch.stack([qualified.to(torch.int32), complaints, (complaints > t).to(torch.int32), recon.to(torch.int32),
                         (honest4 < t + 1).to(torch.int32), honest.to(torch.int32)]).cpu().numpy()
    q, c, r2e, rc, r4e, h = small
    hon = h.astype(np.uint8)
    return Decisions(d2, d4, q.astype(np.uint8), c.astype(np.int32), r2e.astype(np.uint8), rc.astype(np.uint8),
                     r4e.astype(np.uint8), hon, bool(int(hon.sum()) <= t))


def _combine_np(dec2: np.ndarray, dec4: np.ndarray, n: int, t: int) -> Decisions:
    """Host combine of the gathered decision matrices, the same rules as the single-GPU driver:
    a REJECT by receiver j is a complaint of j against dealer i (committee.rs:311-316) and a valid
    complaint disqualifies i for everyone (:370-398); more than t complaints raise
    MisbehaviourHigherThreshold for j (:340-347); disqualified dealers are skipped in round 4 (:522);
    a round-4 REJECT puts the dealer in the reconstruction set (:660-670)."""
    dec2 = np.asarray(dec2, dtype=np.uint8).reshape(n, n)
    dec4 = np.array(dec4, dtype=np.uint8).reshape(n, n)
    rej2 = dec2 == REJECT
    # MISSING (undecodable broadcast) disqualifies without a complaint (committee.rs:331-335)
    qualified = (~(rej2 | (dec2 == MISSING)).any(axis=1)).astype(np.uint8)
    complaints = rej2.sum(axis=0).astype(np.int32)
    r2_error = (complaints > t).astype(np.uint8)
    off = ~np.eye(n, dtype=bool)
    skip = (qualified == 0)[:, None] & off
    dec4[skip] = SKIPPED
    recon = ((dec4 == REJECT) & off & (qualified == 1)[:, None]).any(axis=1).astype(np.uint8)
    honest = (qualified & (1 - recon)).astype(np.uint8)
    # receiver j counts itself plus the qualified dealers it accepted in round 4 (:515-516, 567-569)
    honest4 = 1 + ((dec4 == ACCEPT) & off & (qualified == 1)[:, None]).sum(axis=0)
    r4_error = (honest4 < t + 1).astype(np.uint8)
    return Decisions(dec2, dec4, qualified, complaints, r2_error, recon, r4_error, honest,
                     bool(int(honest.sum()) <= t))


@dataclass
class ShardResult:
    decisions: Decisions
    final_share: Optional[bytes]   # [n][32] s_j (committee.rs:454-462)
    mpk: Optional[bytes]           # 32 bytes (committee.rs:790-795), honest case
    ms_shard: float                # device time of this rank's share gen + checks


class ShardedCeremony:
    """One rank's view of a dealer-sharded ceremony.  `be` is this rank's dkg_amd.Backend (its GPU),
    `dist` an initialised torch.distributed, `device` the torch device the exchanged buffers live on
    (cuda:local for RCCL; cpu works with gloo)."""

    def __init__(self, be, dist, n: int, t: int, device):
        import torch

        self.torch = torch
        self.be, self.dist, self.n, self.t, self.dev = be, dist, n, t, device
        self.ws, self.rank = dist.get_world_size(), dist.get_rank()
        self.staged = dist.get_backend() == "gloo" and getattr(device, "type", str(device)) != "cpu"
        self.d0, self.d1 = dealer_range(self.rank, self.ws, n)
        D, R = self.d1 - self.d0, max_rows(self.ws, n)
        u8 = dict(dtype=torch.uint8, device=device)
        self.dec2 = torch.zeros(R * n, **u8)
        self.dec4 = torch.zeros(R * n, **u8)
        self.A0 = torch.zeros(R * 32, **u8)
        self.part = torch.zeros(n * 32, **u8)
        self.g_dec2 = torch.empty(self.ws * R * n, **u8)
        self.g_dec4 = torch.empty(self.ws * R * n, **u8)
        self.g_A0 = torch.empty(self.ws * R * 32, **u8)
        self.g_part = torch.empty(self.ws * n * 32, **u8)
        self.D, self.R = D, R

    def _fence(self):
        """The library runs on its own HIP streams: before it reads buffers torch produced (the
        gathered rows, concatenations, uploads) or overwrites buffers a collective may still read,
        the work queued on torch's stream -- including an RCCL collective, which torch's current
        stream waits for -- must have completed."""
        if getattr(self.dev, "type", str(self.dev)) == "cuda":
            self.torch.cuda.current_stream(self.dev).synchronize()

    def _all_gather(self, out, inp):
        if self.staged:  # gloo with device buffers: through host memory (rehearsal / CPU runs)
            o = out.cpu()
            self.dist.all_gather_into_tensor(o, inp.cpu())
            out.copy_(o)
        else:
            self.dist.all_gather_into_tensor(out, inp)

    def exchange(self):
        """All-gather the padded per-rank rows; returns (dec2 [n][n], dec4 [n][n], A0 [n][32])
        tensors with the padding removed, and the gathered partial sums [ws][n][32]."""
        self._all_gather(self.g_dec2, self.dec2)
        self._all_gather(self.g_dec4, self.dec4)
        self._all_gather(self.g_A0, self.A0)
        self._all_gather(self.g_part, self.part)
        n, R = self.n, self.R
        rows = []
        for r in range(self.ws):
            a, b = dealer_range(r, self.ws, n)
            rows.append((r * R, r * R + (b - a)))
        torch = self.torch
        dec2 = torch.cat([self.g_dec2[s * n:e * n] for s, e in rows])
        dec4 = torch.cat([self.g_dec4[s * n:e * n] for s, e in rows])
        A0 = torch.cat([self.g_A0[s * 32:e * 32] for s, e in rows])
        return dec2, dec4, A0, self.g_part

    def run(self, d_a: int, d_b: int, finalise: bool = True) -> ShardResult:
        """Share gen + rounds 2/4 for this rank's dealers (device pointers d_a, d_b to its [D][t+1][32]
        coefficients), exchange, combine.  With finalise, also the round-3 final shares (sum of the
        gathered partials) and the master public key (sum of the qualified dealers' terms), both on
        the GPU."""
        self._fence()
        ms = self.be.ceremony_shard_device(self.n, self.t, self.d0, self.d1, d_a, d_b, self.dec2.data_ptr(),
                                           self.dec4.data_ptr(), self.A0.data_ptr(), self.part.data_ptr())
        return self._finish(ms, finalise)

    def run_verify(self, d_E: int, d_A: int, d_s: int, d_sp: int, finalise: bool = True) -> ShardResult:
        """Rounds 2-5 on received broadcasts: this rank's dealers' commitments d_E, d_A [D][t+1][32]
        (compressed, as broadcast in phases 1 and 3) and their shares d_s, d_sp [D][n][32]."""
        self._fence()
        ms = self.be.ceremony_shard_verify_device(self.n, self.t, self.d0, self.d1, d_E, d_A, d_s, d_sp,
                                                  self.dec2.data_ptr(), self.dec4.data_ptr(),
                                                  self.A0.data_ptr(), self.part.data_ptr())
        return self._finish(ms, finalise, d_s)

    def _finish(self, ms: float, finalise: bool, d_s: Optional[int] = None) -> ShardResult:
        n, t = self.n, self.t
        dec2, dec4, A0, parts = self.exchange()
        dec = combine_decisions(dec2, dec4, n, t)
        fs = mpk = None
        if finalise:
            torch = self.torch
            fs_t = torch.empty(n * 32, dtype=torch.uint8, device=self.dev)
            self._fence()
            self.be.scalar_sum_device(self.ws, n, parts.data_ptr(), None, fs_t.data_ptr())
            fs = bytes(fs_t.cpu().numpy())
            if dec.reconstruct.any() and not dec.phase4_error:
                # a dealer accused in round 4 (committee.rs:660-670) enters mpk as g * a_i0 over the
                # final parties' shares (:747-789): the owning rank replaces its term and the terms
                # are gathered again (the interpolation points depend on every rank's rows)
                self._fence()
                self.be.ceremony_shard_recon_device(n, t, self.d0, self.d1, dec.qualified, dec.reconstruct, d_s,
                                                    self.A0.data_ptr())
                self._all_gather(self.g_A0, self.A0)
                A0 = torch.cat([self.g_A0[r * self.R * 32:(r * self.R + b - a) * 32]
                                for r, (a, b) in enumerate(dealer_range(q, self.ws, n) for q in range(self.ws))])
            if not dec.phase4_error:  # else Phases<Phase4>::proceed fails for everyone: no mpk (:673-677)
                # the terms are A_i0 for honest dealers and g * a_i0 for the reconstructable set, so
                # the sum runs over the qualified set
                mask = torch.from_numpy(dec.qualified).to(self.dev)
                mpk_t = torch.empty(32, dtype=torch.uint8, device=self.dev)
                self._fence()
                self.be.point_sum_device(n, A0.data_ptr(), mask.data_ptr(), mpk_t.data_ptr())
                mpk = bytes(mpk_t.cpu().numpy())
        return ShardResult(dec, fs, mpk, ms)
