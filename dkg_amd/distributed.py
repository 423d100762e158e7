"""Multi-GPU ceremony: one process per GPU, the ceremony sharded by dealer.

Rank r owns dealers [r*n/ws, (r+1)*n/ws) (dkg_shard_range): it generates their commitments and
shares and checks their rows against all n receivers on its GPU (dkg_ceremony_shard_device).  The
protocol's exchange step -- every party learns every complaint (committee.rs:311-331, 370-398) and
the round-3/5 broadcasts (committee.rs:454-467, 790-795) -- is a set of all-gathers (RCCL over xGMI
with the "nccl" backend, gloo in the CPU tests) of:
  * the round-2 / round-4 decision rows, packed as bitmaps (dkg_decisions_pack_device: one ACCEPT
    bit per pair plus a row-kind word -- SELF, MISSING rows and SKIPPED are implied; n=4096: 516
    bytes per row instead of 4096),
  * every dealer's compressed master-key term (A_i0, or g * a_i0 recovered by Lagrange
    interpolation on the owning rank for dealers accused in round 4),
  * each rank's partial final shares (sum over its qualified dealers of s_ij).
This module holds only the collectives.  The protocol layer runs in the library, behind the C ABI:
dkg_shard_combine_device derives the common outcome (qualified set, complaints, r2 errors, SKIPPED
rows, reconstruction set, r4 errors, Phase4 failure) with the single-GPU drivers' own code, and
dkg_shard_finalise_device the final shares, public shares and mpk (include/dkg_amd.h).
"""
import time
from dataclasses import dataclass
from typing import Any, Dict, Optional

import numpy as np

from .api import shard_range, shard_rows


def dealer_range(rank: int, world_size: int, n: int):
    """Dealers owned by `rank` (dkg_shard_range: contiguous, sizes differ by at most one)."""
    return shard_range(n, world_size, rank)


def max_rows(world_size: int, n: int) -> int:
    """Padded block height R of every rank's gathered rows (dkg_shard_rows)."""
    return shard_rows(n, world_size)


@dataclass
class Decisions:
    dec2: Any                 # [n][n] uint8 tensor on the exchange device
    dec4: Any                 # [n][n] uint8 tensor, SKIPPED rows for disqualified dealers
    qualified: np.ndarray     # [n] uint8
    complaints2: np.ndarray   # [n] int32, complaints raised by receiver j
    r2_error: np.ndarray      # [n] uint8, receiver j saw more than t complaints
    reconstruct: np.ndarray   # [n] uint8, qualified dealers accused in round 4
    r4_error: np.ndarray      # [n] uint8, receiver j saw fewer than t+1 honest dealers in round 4
    phase4_error: bool        # qualified minus reconstructable <= t: Phase4::proceed fails (:673-677)


class ShardResult:
    """One rank's outputs of a sharded ceremony.
    final_share  [n][32] s_j (committee.rs:454-462) and public_share [n][32] g * s_j (:463-467): bytes,
                 copied from the device when first read (a device copy is kept, so a later run does
                 not change them; a timed loop that never reads them pays no host round trip)
    mpk          32 bytes (committee.rs:790-795); None when Phase4 fails
    ms_shard     device time of this rank's share gen + checks
    ms_steps     host wall ms of the steps after the shard: "exchange" (the all-gather, fenced),
                 "combine" (dkg_shard_combine_device + outcome copies), "recon" (round-4
                 reconstruction + its gather; 0 when nobody was accused), "finalise"
                 (dkg_shard_finalise_device)"""

    def __init__(self, decisions: Decisions, final_share, public_share, mpk: Optional[bytes], ms_shard: float,
                 ms_steps: Optional[Dict[str, float]] = None):
        self.decisions, self._fs, self._pub = decisions, final_share, public_share
        self.mpk, self.ms_shard, self.ms_steps = mpk, ms_shard, dict(ms_steps or {})

    @staticmethod
    def _host(v):
        return v if v is None or isinstance(v, (bytes, bytearray)) else bytes(v.cpu().numpy())

    @property
    def final_share(self) -> Optional[bytes]:
        self._fs = self._host(self._fs)
        return self._fs

    @property
    def public_share(self) -> Optional[bytes]:
        self._pub = self._host(self._pub)
        return self._pub


class ShardedCeremony:
    """One rank's view of a dealer-sharded ceremony.  `be` is this rank's dkg_amd.Backend (its GPU),
    `dist` an initialised torch.distributed, `device` the torch device the exchanged buffers live on
    (cuda:local for RCCL; cpu works with gloo)."""

    def __init__(self, be, dist, n: int, t: int, device, packed: bool = True):
        import torch

        self.torch = torch
        self.be, self.dist, self.n, self.t, self.dev = be, dist, n, t, device
        self.packed = packed
        self.ws, self.rank = dist.get_world_size(), dist.get_rank()
        self.staged = dist.get_backend() == "gloo" and getattr(device, "type", str(device)) != "cpu"
        self.d0, self.d1 = dealer_range(self.rank, self.ws, n)
        D, R = self.d1 - self.d0, max_rows(self.ws, n)
        u8 = dict(dtype=torch.uint8, device=device)
        # One send block per rank, gathered in ONE collective: [round-2 rows | round-4 rows | master-key
        # terms [R][32] | partial final shares [n][32]], the rows packed ([R][W+1] u32 bitmaps,
        # dkg_packed_row_words) or raw ([R][n] bytes).  The library writes straight into its views.
        if packed:
            from .api import packed_row_words

            self.W1 = packed_row_words(n)
            S2 = 4 * R * self.W1
        else:
            S2 = R * n
        self.S2, self.S = S2, 2 * S2 + R * 32 + n * 32
        self.send = torch.zeros(self.S, **u8)
        self.A0 = self.send[2 * S2:2 * S2 + R * 32]
        self.part = self.send[2 * S2 + R * 32:]
        if packed:
            self.dec2 = torch.zeros(R * n, **u8)  # raw rows, packed into the send block
            self.dec4 = torch.zeros(R * n, **u8)
            self.p2 = self.send[:S2].view(torch.int32)
            self.p4 = self.send[S2:2 * S2].view(torch.int32)
            i32 = dict(dtype=torch.int32, device=device)
            self.g_dec2 = torch.empty(self.ws * R * self.W1, **i32)
            self.g_dec4 = torch.empty(self.ws * R * self.W1, **i32)
        else:
            self.dec2, self.dec4 = self.send[:S2], self.send[S2:2 * S2]
            self.g_dec2 = torch.empty(self.ws * R * n, **u8)
            self.g_dec4 = torch.empty(self.ws * R * n, **u8)
        self.g_all = torch.empty(self.ws * self.S, **u8)
        self.g_A0 = torch.empty(self.ws * R * 32, **u8)
        self.g_part = torch.empty(self.ws * n * 32, **u8)
        self.c_dec2 = torch.empty(n * n, **u8)   # compacted by the combine
        self.c_dec4 = torch.empty(n * n, **u8)
        self.fs = torch.empty(n * 32, **u8)
        self.pub = torch.empty(n * 32, **u8)
        self.D, self.R = D, R

    def _fence(self):
        """The library runs on its own HIP streams: before it reads buffers torch produced (the
        gathered rows, uploads) or overwrites buffers a collective may still read, the work queued
        on torch's stream -- including an RCCL collective, which torch's current stream waits for --
        must have completed."""
        if getattr(self.dev, "type", str(self.dev)) == "cuda":
            self.torch.cuda.current_stream(self.dev).synchronize()

    def _all_gather(self, out, inp):
        if self.staged:  # gloo with device buffers: through host memory (rehearsal / CPU runs)
            o = out.cpu()
            self.dist.all_gather_into_tensor(o, inp.cpu())
            out.copy_(o)
        else:
            self.dist.all_gather_into_tensor(out, inp)

    def _pack(self, dec, out):
        """This rank's raw rows [D][n] -> its packed block [R][W+1] (dkg_decisions_pack_device)."""
        self.be.decisions_pack_device(self.R, self.D, self.n, self.d0, dec.data_ptr(), out.data_ptr())

    def exchange_bytes(self) -> int:
        """Bytes one rank contributes to the all-gather of one ceremony (without the round-4
        reconstruction's second gather of the master-key terms)."""
        return self.S

    def exchange(self):
        """All-gather every rank's send block (one collective), then split the gathered [ws][S] blocks
        on the device into the decision rows (round 2, round 4; packed bitmaps [ws][R][W+1] or bytes
        [ws][R][n]), the master-key terms [ws][R][32] and the partial final shares [ws][n][32]."""
        if self.packed:
            self._pack(self.dec2, self.p2)
            self._pack(self.dec4, self.p4)
        self._all_gather(self.g_all, self.send)
        S2, R, ws = self.S2, self.R, self.ws
        g = self.g_all.view(ws, self.S)
        self.g_dec2.view(self.torch.uint8).view(ws, S2).copy_(g[:, :S2])
        self.g_dec4.view(self.torch.uint8).view(ws, S2).copy_(g[:, S2:2 * S2])
        self.g_A0.view(ws, R * 32).copy_(g[:, 2 * S2:2 * S2 + R * 32])
        self.g_part.view(ws, self.n * 32).copy_(g[:, 2 * S2 + R * 32:])
        return self.g_dec2, self.g_dec4, self.g_A0, self.g_part

    def run(self, d_a: int, d_b: int, finalise: bool = True) -> ShardResult:
        """Share gen + rounds 2/4 for this rank's dealers (device pointers d_a, d_b to its [D][t+1][32]
        coefficients), exchange, combine.  With finalise, also the round-3 final shares and public
        shares and the master public key, on the GPU."""
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
        n, t, ws = self.n, self.t, self.ws
        steps = {}
        c0 = time.perf_counter()
        self.exchange()
        self._fence()
        c1 = time.perf_counter()
        steps["exchange"] = (c1 - c0) * 1e3
        o = self.be.shard_combine_device(n, t, ws, self.g_dec2.data_ptr(), self.g_dec4.data_ptr(),
                                         self.c_dec2.data_ptr(), self.c_dec4.data_ptr(), packed=self.packed,
                                         arrays=True)
        dec = Decisions(self.c_dec2.view(n, n), self.c_dec4.view(n, n), np.array(o.qualified, dtype=np.uint8),
                        np.array(o.complaints2, dtype=np.int32), np.array(o.r2_error, dtype=np.uint8),
                        np.array(o.reconstruct, dtype=np.uint8), np.array(o.r4_error, dtype=np.uint8),
                        o.phase4_error)
        c2 = time.perf_counter()
        steps["combine"] = (c2 - c1) * 1e3
        if not finalise:
            return ShardResult(dec, None, None, None, ms, steps)
        no_mpk = dec.phase4_error
        if dec.reconstruct.any() and not dec.phase4_error:
            # a dealer accused in round 4 (committee.rs:660-670) enters mpk as g * a_i0 over the
            # disclosing final parties' shares (:747-789): the owning rank replaces its term and the
            # terms are gathered again (the interpolation points depend on every rank's rows).  Fewer
            # than t disclosing parties: nobody recovers (:779-781), the same verdict on every rank.
            no_mpk = self.be.ceremony_shard_recon_device(n, t, self.d0, self.d1, dec.qualified, dec.reconstruct, d_s,
                                                         self.A0.data_ptr(), dec.r2_error, dec.r4_error)
            if not no_mpk:
                self._all_gather(self.g_A0, self.A0)
                self._fence()
        c3 = time.perf_counter()
        steps["recon"] = (c3 - c2) * 1e3
        mpk = self.be.shard_finalise_device(n, t, ws, self.g_A0.data_ptr(), self.g_part.data_ptr(), dec.qualified,
                                            no_mpk, self.fs.data_ptr(), self.pub.data_ptr())
        # device copies of this run's shares (the buffers are reused), read back only when asked for
        fs, pub = self.fs.clone(), self.pub.clone()
        steps["finalise"] = (time.perf_counter() - c3) * 1e3
        return ShardResult(dec, fs, pub, None if no_mpk else mpk, ms, steps)
