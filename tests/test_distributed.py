"""Multi-process (world_size 2, gloo, CPU) tests of the dealer-sharded exchange and combine
(dkg_amd/distributed.py).  Each rank holds only its dealers' rows of a golden ceremony; after the
all-gathers every rank must derive the golden qualified set, complaints, r2 errors, round-4 SKIPPED
marks, reconstruction set and final shares.  The GPU half of the sharded path
(dkg_ceremony_shard_device) is covered by tests/test_gpu.py::test_sharded_ceremony_matches_golden.
"""
import json
import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = 2**252 + 27742317777372353535851937790883648493
NAMES = ["ceremony_n11_t5.json", "fault_share_flip_n10_t4.json", "fault_a_generator_n10_t4.json",
         "fault_over_threshold_n10_t4.json", "fault_e_identity_n10_t4.json", "ceremony_n3_t1.json",
         "fault_a_many_n10_t4.json"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, ws, port, names, errq):
    import torch
    import torch.distributed as dist

    from dkg_amd.distributed import ShardedCeremony, combine_decisions, dealer_range

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
        for name in names:
            with open(os.path.join(ROOT, "tests", "golden", name)) as f:
                c = json.load(f)
            n, t = c["n"], c["t"]
            N = t + 1
            sc = ShardedCeremony(None, dist, n, t, torch.device("cpu"))
            d0, d1 = dealer_range(rank, ws, n)
            assert (sc.d0, sc.d1) == (d0, d1)
            rng = random.Random(rank)
            dec2 = bytes(int(x) for x in c["dec2"][d0 * n:d1 * n])
            # a shard's raw round-4 rows hold real check results even for disqualified dealers:
            # replace the golden SKIPPED marks by arbitrary 0/1, combine must restore them
            dec4 = bytes(rng.randrange(2) if x == "3" else int(x) for x in c["dec4"][d0 * n:d1 * n])
            A = bytes.fromhex(c["A"])
            A0 = b"".join(A[32 * N * i:32 * N * i + 32] for i in range(d0, d1))
            qualified_own = [all(c["dec2"][i * n + j] != "0" for j in range(n)) for i in range(d0, d1)]
            s = bytes.fromhex(c["s"])
            part = b"".join(
                (sum(int.from_bytes(s[32 * (i * n + j):32 * (i * n + j) + 32], "little")
                     for k, i in enumerate(range(d0, d1)) if qualified_own[k]) % L).to_bytes(32, "little")
                for j in range(n))
            sc.dec2[:len(dec2)] = torch.frombuffer(bytearray(dec2), dtype=torch.uint8) if dec2 else sc.dec2[:0]
            sc.dec4[:len(dec4)] = torch.frombuffer(bytearray(dec4), dtype=torch.uint8) if dec4 else sc.dec4[:0]
            if A0:
                sc.A0[:len(A0)] = torch.frombuffer(bytearray(A0), dtype=torch.uint8)
            sc.part[:] = torch.frombuffer(bytearray(part), dtype=torch.uint8)
            g2, g4, gA0, gpart = sc.exchange()
            assert bytes(g2.numpy()) == bytes(int(x) for x in c["dec2"]), name
            assert bytes(gA0.numpy()) == b"".join(A[32 * N * i:32 * N * i + 32] for i in range(n)), name
            d = combine_decisions(g2.numpy(), g4.numpy(), n, t)
            assert d.qualified.tolist() == c["qualified"], name
            assert d.complaints2.tolist() == c["complaints2"], name
            assert d.r2_error.tolist() == [int(x) for x in c["r2_error"]], name
            assert d.reconstruct.tolist() == c["reconstruct"], name
            assert d.r4_error.tolist() == [int(x) for x in c["r4_error"]], name
            assert d.phase4_error == c["phase4_error"], name
            assert "".join(str(x) for x in d.dec4.reshape(-1).tolist()) == c["dec4"], name
            parts = gpart.numpy().reshape(ws, n, 32)
            fs = b"".join((sum(int.from_bytes(bytes(parts[r, j]), "little") for r in range(ws)) % L)
                          .to_bytes(32, "little") for j in range(n))
            assert fs.hex() == c["final_share"], name
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # report to the parent; a hung peer is cut by the join timeout
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


@pytest.mark.parametrize("ws", [2, 3])
def test_sharded_exchange_gloo(ws):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, ws, port, NAMES, errq)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not alive, "rank hung"
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_combine_single_process(golden):
    """combine_decisions alone on every golden ceremony (no exchange)."""
    from dkg_amd.distributed import combine_decisions

    for name in NAMES + ["ceremony_n64_t31.json"]:
        c = golden(name)
        n, t = c["n"], c["t"]
        dec2 = np.frombuffer(bytes(int(x) for x in c["dec2"]), dtype=np.uint8)
        dec4 = np.frombuffer(bytes(1 if x == "3" else int(x) for x in c["dec4"]), dtype=np.uint8)
        d = combine_decisions(dec2, dec4, n, t)
        assert d.qualified.tolist() == c["qualified"]
        assert d.reconstruct.tolist() == c["reconstruct"]
        assert d.r4_error.tolist() == [int(x) for x in c["r4_error"]]
        assert d.phase4_error == c["phase4_error"]
        assert "".join(str(x) for x in d.dec4.reshape(-1).tolist()) == c["dec4"]


def test_combine_torch_matches_numpy(golden):
    """The device-side combine (torch tensors, as ShardedCeremony hands over the gathered rows)
    equals the numpy combine on every golden ceremony."""
    import torch

    from dkg_amd.distributed import combine_decisions

    for name in NAMES + ["ceremony_n64_t31.json"]:
        c = golden(name)
        n, t = c["n"], c["t"]
        dec2 = np.frombuffer(bytes(int(x) for x in c["dec2"]), dtype=np.uint8).copy()
        dec4 = np.frombuffer(bytes(1 if x == "3" else int(x) for x in c["dec4"]), dtype=np.uint8).copy()
        a = combine_decisions(dec2, dec4, n, t)
        b = combine_decisions(torch.from_numpy(dec2), torch.from_numpy(dec4), n, t)
        for f in ("qualified", "complaints2", "r2_error", "reconstruct", "r4_error", "honest"):
            assert getattr(a, f).tolist() == getattr(b, f).tolist(), (name, f)
        assert a.dec4.reshape(-1).tolist() == b.dec4.reshape(-1).tolist() and a.phase4_error == b.phase4_error
