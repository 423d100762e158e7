"""Test helper (not a test module): every rank of a ws-way dealer-sharded run played in ONE process
on GPU 0, with the all-gathers replaced by their result -- each rank's padded block placed at
r * R in the gathered buffers, exactly what all_gather_into_tensor delivers -- and the protocol layer
run by the library (dkg_shard_combine_device, dkg_ceremony_shard_recon_device,
dkg_shard_finalise_device), as dkg_amd/distributed.py drives it across processes."""
from dataclasses import dataclass
from typing import Any, List

import dkg_amd


@dataclass
class Played:
    dec2: bytes          # compacted [n][n] (raw round-2 decisions)
    dec4: bytes          # compacted [n][n], SKIPPED applied
    raw4: bytes          # the ranks' raw round-4 rows, compacted
    outcome: Any         # dkg_amd.api.ShardOutcome
    final_share: bytes
    public_share: bytes
    mpk: bytes
    rank_dec2: List[bytes]
    rank_dec4: List[bytes]


def play(be, n, t, ws, shard_call, dev):
    """shard_call(r, d0, d1, o2, o4, oA, op) runs rank r's dkg_ceremony_shard[_verify]_device into the
    given device buffers and returns the rank's share-row tensor for the reconstruction (or None to
    use the ctx's last shard rows -- only valid for ws == 1)."""
    import torch

    R = dkg_amd.shard_rows(n, ws)
    u8 = dict(dtype=torch.uint8, device=dev)
    g2 = torch.full((ws * R * n,), 0xEE, **u8)
    g4 = torch.full((ws * R * n,), 0xEE, **u8)
    gA = torch.zeros(ws * R * 32, **u8)
    gp = torch.zeros(ws * n * 32, **u8)
    shares, rd2, rd4 = [], [], []
    for r in range(ws):
        d0, d1 = dkg_amd.shard_range(n, ws, r)
        D = d1 - d0
        o2 = g2[r * R * n:(r + 1) * R * n]
        o4 = g4[r * R * n:(r + 1) * R * n]
        oA = gA[r * R * 32:(r + 1) * R * 32]
        op = gp[r * n * 32:(r + 1) * n * 32]
        shares.append(shard_call(r, d0, d1, o2, o4, oA, op))
        rd2.append(bytes(o2[:D * n].cpu().numpy()))
        rd4.append(bytes(o4[:D * n].cpu().numpy()))
    c2 = torch.empty(n * n, **u8)
    c4 = torch.empty(n * n, **u8)
    o = be.shard_combine_device(n, t, ws, g2.data_ptr(), g4.data_ptr(), c2.data_ptr(), c4.data_ptr())
    no_mpk = o.phase4_error
    if any(o.reconstruct) and not o.phase4_error:
        for r in range(ws):
            d0, d1 = dkg_amd.shard_range(n, ws, r)
            if d1 > d0:
                s = shares[r]
                no_mpk = be.ceremony_shard_recon_device(n, t, d0, d1, o.qualified, o.reconstruct,
                                                        None if s is None else s.data_ptr(), gA[r * R * 32:].data_ptr(),
                                                        o.r2_error, o.r4_error)
    fs = torch.empty(n * 32, **u8)
    pub = torch.empty(n * 32, **u8)
    mpk = be.shard_finalise_device(n, t, ws, gA.data_ptr(), gp.data_ptr(), o.qualified, no_mpk, fs.data_ptr(),
                                   pub.data_ptr())
    return Played(bytes(c2.cpu().numpy()), bytes(c4.cpu().numpy()), b"".join(rd4), o, bytes(fs.cpu().numpy()),
                  bytes(pub.cpu().numpy()), mpk, rd2, rd4)
