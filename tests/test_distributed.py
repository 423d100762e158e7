"""Multi-process (world_size 2/3, gloo, CPU) tests of the dealer-sharded exchange
(dkg_amd/distributed.py).  Each rank holds only its dealers' rows of a golden ceremony; after the
all-gathers every rank must hold every rank's blocks, from which the combine rules
(tests/combine_ref.py, the checker of the library's dkg_shard_combine_device) derive the golden
qualified set, complaints, r2 errors, round-4 SKIPPED marks, reconstruction set and final shares.
The GPU half of the sharded path (dkg_ceremony_shard_device, dkg_shard_combine_device,
dkg_shard_finalise_device) is covered by tests/test_gpu.py and tests/test_gpu_dist.py.
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

    from dkg_amd.distributed import ShardedCeremony, dealer_range
    from tests import combine_ref as CR

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
        for name, packed in [(x, p) for x in names for p in (False, True)]:
            with open(os.path.join(ROOT, "tests", "golden", name)) as f:
                c = json.load(f)
            n, t = c["n"], c["t"]
            N = t + 1
            sc = ShardedCeremony(None, dist, n, t, torch.device("cpu"), packed=packed)
            if packed:  # the library's packing restated (tests/combine_ref.py pack_rows)
                sc._pack = lambda dec, out, sc=sc: out.copy_(torch.from_numpy(
                    CR.pack_rows(dec.numpy()[:sc.D * sc.n], sc.R, sc.D, sc.n, sc.d0).view(np.int32).reshape(-1)))
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
            if packed:
                assert g2.numel() == ws * sc.R * CR.packed_words(n)
                g2, g4 = (CR.unpack_ranks(g.numpy().view(np.uint32), ws, n) for g in (g2, g4))
            else:
                g2, g4 = CR.compact(g2.numpy(), ws, n, n), CR.compact(g4.numpy(), ws, n, n)
            gA0 = CR.compact(gA0.numpy(), ws, n, 32)
            assert bytes(g2) == bytes(int(x) for x in c["dec2"]), name
            assert bytes(gA0) == b"".join(A[32 * N * i:32 * N * i + 32] for i in range(n)), name
            d = CR.combine(g2, g4, n, t)
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


def test_combine_ref_on_goldens(golden):
    """The checker's combine rules (tests/combine_ref.py) reproduce every golden ceremony's outcome
    from its raw decision matrices (round-4 SKIPPED marks replaced by arbitrary checks)."""
    from tests import combine_ref as CR

    for name in NAMES + ["ceremony_n64_t31.json"]:
        c = golden(name)
        n, t = c["n"], c["t"]
        dec2 = np.frombuffer(bytes(int(x) for x in c["dec2"]), dtype=np.uint8)
        dec4 = np.frombuffer(bytes(1 if x == "3" else int(x) for x in c["dec4"]), dtype=np.uint8)
        d = CR.combine(dec2, dec4, n, t)
        assert d.qualified.tolist() == c["qualified"]
        assert d.complaints2.tolist() == c["complaints2"]
        assert d.reconstruct.tolist() == c["reconstruct"]
        assert d.r4_error.tolist() == [int(x) for x in c["r4_error"]]
        assert d.phase4_error == c["phase4_error"]
        assert "".join(str(x) for x in d.dec4.reshape(-1).tolist()) == c["dec4"]


def test_shard_partition_matches_library():
    """The padded gather layout the checker assumes is the library's partition (dkg_shard_range,
    dkg_shard_rows: C entry points without a device)."""
    import dkg_amd
    from tests import combine_ref as CR

    for n in (2, 3, 10, 11, 64, 1024, 1100, 4096):
        for ws in (1, 2, 3, 5, 8):
            if ws > n:
                continue
            assert dkg_amd.shard_rows(n, ws) == CR.rows_per_rank(ws, n)
            assert [dkg_amd.shard_range(n, ws, r) for r in range(ws)] == [CR.dealer_range(r, ws, n) for r in range(ws)]
            rows = [dkg_amd.shard_range(n, ws, r) for r in range(ws)]
            assert rows[0][0] == 0 and rows[-1][1] == n and all(rows[r][1] == rows[r + 1][0] for r in range(ws - 1))


class OracleBackend:
    """Stand-in for dkg_amd.Backend on CPU tensors (test double, oracle arithmetic): the device
    entry points ShardedCeremony calls, computed by the CPU oracle and written through the
    tensors' pointers.  Lets the whole ShardedCeremony.run_verify orchestration -- exchange,
    combine, the reconstruction exchange, finalise -- run in gloo processes without a GPU."""

    def __init__(self, h):
        self.h = h

    @staticmethod
    def _rd(ptr, size):
        import ctypes
        return ctypes.string_at(ptr, size)

    @staticmethod
    def _wr(ptr, data):
        import ctypes
        ctypes.memmove(ptr, data, len(data))

    def ceremony_shard_verify_device(self, n, t, d0, d1, dE, dA, ds, dsp, o2, o4, oA, op):
        from tests import oracle_lib as O
        N, D = t + 1, d1 - d0
        if D:
            E, A = self._rd(dE, 32 * N * D), self._rd(dA, 32 * N * D)
            s, sp = self._rd(ds, 32 * n * D), self._rd(dsp, 32 * n * D)
            pe, ps = bytes(32 * N * d0), bytes(32 * n * d0)  # the oracle indexes absolute dealers
            r2, _ = O.verify_pairs(n, t, 2, pe + E, self.h, ps + s, ps + sp, d0, d1, 0, n)
            r4, _ = O.verify_pairs(n, t, 4, pe + A, self.h, ps + s, None, d0, d1, 0, n)
            self._wr(o2, r2)
            self._wr(o4, r4)
            self._wr(oA, b"".join(A[32 * N * i:32 * N * i + 32] for i in range(D)))
            q = [all(r2[i * n + j] in (1, 2) for j in range(n)) for i in range(D)]
            part = b"".join((sum(int.from_bytes(s[32 * (i * n + j):32 * (i * n + j) + 32], "little")
                                 for i in range(D) if q[i]) % L).to_bytes(32, "little") for j in range(n))
        else:
            part = bytes(32 * n)
        self._wr(op, part)
        self._shares = (d0, d1, self._rd(ds, 32 * n * D) if D else b"")
        return 0.0

    def ceremony_shard_recon_device(self, n, t, d0, d1, qualified, reconstruct, d_s, d_terms, r2_error=None,
                                    r4_error=None):
        from tests import finalise_ref as FR
        s = self._rd(d_s, 32 * n * (d1 - d0))
        # the disclosing final parties (no r2 / r4 error: committee.rs:340-347, 567-569, 684)
        final = [int(q and not r and not (r2_error is not None and r2_error[j]) and
                     not (r4_error is not None and r4_error[j]))
                 for j, (q, r) in enumerate(zip(qualified, reconstruct))]
        xs = [j + 1 for j in range(n) if final[j]]
        if any(reconstruct) and len(xs) < t:
            return True  # InsufficientSharesForRecovery for everyone (:779-781)
        for i in range(d0, d1):
            if reconstruct[i]:
                row = s[32 * n * (i - d0):32 * n * (i - d0 + 1)]
                ys = [int.from_bytes(row[32 * (x - 1):32 * x], "little") for x in xs]
                self._wr(d_terms + 32 * (i - d0), FR.g_mul(FR.lagrange_at_zero(ys, xs)))
        return False

    def decisions_pack_device(self, rows, nvalid, n, d0, d_dec, d_packed):
        from tests import combine_ref as CR
        raw = np.frombuffer(self._rd(d_dec, nvalid * n), dtype=np.uint8) if nvalid else np.zeros(0, np.uint8)
        self._wr(d_packed, CR.pack_rows(raw, rows, nvalid, n, d0).tobytes())

    def shard_combine_device(self, n, t, ws, d_dec2_g, d_dec4_g, d_dec2=None, d_dec4=None, packed=False,
                             arrays=False):
        from dkg_amd.api import ShardOutcome
        from tests import combine_ref as CR
        R = CR.rows_per_rank(ws, n)
        if packed:
            sz = 4 * ws * R * CR.packed_words(n)
            g2, g4 = (CR.unpack_ranks(np.frombuffer(self._rd(d, sz), dtype=np.uint32), ws, n)
                      for d in (d_dec2_g, d_dec4_g))
        else:
            g2 = CR.compact(np.frombuffer(self._rd(d_dec2_g, ws * R * n), dtype=np.uint8), ws, n, n)
            g4 = CR.compact(np.frombuffer(self._rd(d_dec4_g, ws * R * n), dtype=np.uint8), ws, n, n)
        d = CR.combine(g2, g4, n, t)
        if d_dec2:
            self._wr(d_dec2, bytes(d.dec2))
        if d_dec4:
            self._wr(d_dec4, bytes(d.dec4))
        cv = (lambda a: np.asarray(a).copy()) if arrays else (lambda a: a.tolist())
        return ShardOutcome(cv(d.qualified), cv(d.complaints2), cv(d.r2_error), cv(d.reconstruct), cv(d.r4_error),
                            int(d.qualified.sum()), d.phase4_error)

    def shard_finalise_device(self, n, t, ws, d_terms_g, d_partials_g, qualified, phase4_error, d_fs, d_pub=None):
        from tests import combine_ref as CR
        from tests import finalise_ref as FR
        data = self._rd(d_partials_g, 32 * ws * n)
        fs = [sum(int.from_bytes(data[32 * (r * n + j):32 * (r * n + j) + 32], "little") for r in range(ws)) % L
              for j in range(n)]
        self._wr(d_fs, b"".join(x.to_bytes(32, "little") for x in fs))
        if d_pub:
            self._wr(d_pub, b"".join(FR.g_mul(x) for x in fs))
        R = CR.rows_per_rank(ws, n)
        terms = bytes(CR.compact(np.frombuffer(self._rd(d_terms_g, 32 * ws * R), dtype=np.uint8), ws, n, 32))
        if phase4_error:
            return bytes(32)
        return FR.gsum([terms[32 * i:32 * i + 32] for i in range(n) if qualified[i]])


def _run_verify_main(rank, ws, port, names, errq):
    import torch
    import torch.distributed as dist

    from dkg_amd.distributed import ShardedCeremony, dealer_range

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
        for name in names:
            with open(os.path.join(ROOT, "tests", "golden", name)) as f:
                c = json.load(f)
            n, t = c["n"], c["t"]
            N = t + 1
            d0, d1 = dealer_range(rank, ws, n)
            H = bytes.fromhex
            E, A, s, sp = (H(c[k]) for k in ("E", "A", "s", "s_prime"))
            put = lambda x: torch.frombuffer(bytearray(x or b"\0"), dtype=torch.uint8)  # noqa: E731
            tE, tA = put(E[32 * N * d0:32 * N * d1]), put(A[32 * N * d0:32 * N * d1])
            ts, tsp = put(s[32 * n * d0:32 * n * d1]), put(sp[32 * n * d0:32 * n * d1])
            sc = ShardedCeremony(OracleBackend(H(c["h"])), dist, n, t, torch.device("cpu"))
            res = sc.run_verify(tE.data_ptr(), tA.data_ptr(), ts.data_ptr(), tsp.data_ptr())
            d = res.decisions
            assert d.qualified.tolist() == c["qualified"] and d.reconstruct.tolist() == c["reconstruct"], name
            assert res.final_share.hex() == c["final_share"], name
            assert res.public_share.hex() == c["public_share"], name
            if c["phase4_error"] or c["mpk"] == "00" * 32:
                assert res.mpk is None, name
            else:
                assert res.mpk.hex() == c["mpk"], name
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


@pytest.mark.parametrize("ws", [2, 3])
def test_sharded_run_verify_gloo(ws):
    """ShardedCeremony.run_verify end to end over gloo with the oracle standing in for the GPU:
    the reconstruction exchange of dealers accused in round 4 (fault_a_generator, fault_self_share
    with a tampered self-share, fault_recon_only; final parties with round-2 errors that never
    disclose, leaving t points and then fewer -- no mpk) and the Phase4 failure (fault_a_many: no mpk)."""
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    names = ["fault_a_generator_n10_t4.json", "fault_self_share_n10_t4.json", "fault_recon_only_n10_t4.json",
             "fault_a_many_n10_t4.json", "ceremony_n11_t5.json", "fault_recon_r2err_n16_t3.json",
             "fault_recon_insufficient_n16_t3.json"]
    procs = [ctx.Process(target=_run_verify_main, args=(r, ws, port, names, errq)) for r in range(ws)]
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
