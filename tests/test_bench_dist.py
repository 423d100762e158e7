"""CPU tests of bench.py's own multi-rank launcher (`--gpus N` without torchrun): a rank that dies
must end the whole run with a non-zero exit within seconds -- its peers, blocked in a collective the
dead rank never joins, are stopped by the launcher instead of waiting for the collective timeout.
DKG_BENCH_FAIL_RANK (bench.fault_rehearsal) injects the failure after the gloo process group is up;
no GPU is touched."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(fail_rank, gpus=2):
    env = dict(os.environ, DKG_BENCH_FAIL_RANK=str(fail_rank))
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dist-backend", "gloo",
                        "--dist-timeout", "300"], env=env, capture_output=True, text=True, timeout=240)
    return p, time.time() - t0


def test_failed_rank_ends_the_run_fast():
    p, dt = _run(1)
    assert p.returncode != 0, p.stderr[-2000:]
    assert "rank 1 exited with 1" in p.stderr, p.stderr[-2000:]
    # far below the 300-s collective timeout: the launcher stopped rank 0 out of its barrier
    assert dt < 60, dt
    assert p.stdout == ""  # no result line from a failed run


def test_failed_rank_zero_of_three():
    p, dt = _run(0, gpus=3)
    assert p.returncode != 0 and dt < 60, (p.returncode, dt, p.stderr[-2000:])


def test_all_ranks_succeed():
    p, dt = _run(-1)
    assert p.returncode == 0, p.stderr[-2000:]


def _self_check_rank(rank, ws, port, wrong, errq, outq, backend="gloo", shared=False):
    """One gloo rank of bench.sharded_self_check on a stand-in sharded result: the rank's dealers'
    coefficients, the honest outcome, the mpk g * sum_i a_i0 (or a wrong one) and step times."""
    import random
    from types import SimpleNamespace

    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    from dkg_amd.distributed import dealer_range
    from tests import oracle_lib as O

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
        n, t = 10, 4
        N = t + 1
        rng = random.Random(7)
        a = [[rng.randrange(bench.L) for _ in range(N)] for _ in range(n)]  # every rank: the same ceremony
        d0, d1 = dealer_range(rank, ws, n)
        ta = torch.frombuffer(bytearray(b"".join(x.to_bytes(32, "little") for i in range(d0, d1) for x in a[i])),
                              dtype=torch.uint8)
        secret = sum(a[i][0] for i in range(n)) % bench.L
        mpk = O.base_mul(((secret + (wrong == -2)) % bench.L).to_bytes(32, "little"))  # -2: all wrong
        dec = SimpleNamespace(qualified=np.ones(n, np.uint8), r2_error=np.zeros(n, np.uint8),
                              r4_error=np.zeros(n, np.uint8), phase4_error=False)
        res = SimpleNamespace(decisions=dec, mpk=mpk, ms_shard=1.0 + rank,
                              ms_steps={"exchange": 0.5 * (rank + 1), "combine": 0.2, "recon": 0.0, "finalise": 0.3})
        bus = "0000:05:00.0" if shared else f"0000:{0x05 + 0x10 * rank:02x}:00.0"
        be = SimpleNamespace(fixed_base_batch=O.base_mul, pci_bus_id=lambda: bus)
        # backend "nccl" here only selects bench's RCCL-side checks; the tensors stay on the CPU
        args = SimpleNamespace(dist_backend=backend)
        try:
            out = bench.sharded_self_check(args, dist, be, res, ta, d1 - d0, N, torch.device("cpu"))
        except AssertionError as e:
            out = {"assertion": str(e)}
        except SystemExit as e:
            out = {"exit": str(e)}
        outq.put((rank, out))
        dist.destroy_process_group()
    except BaseException as e:
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


def _self_check(ws, wrong, backend="gloo", shared=False):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    errq, outq = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_self_check_rank, args=(r, ws, port, wrong, errq, outq, backend, shared))
             for r in range(ws)]
    for p in procs:
        p.start()
    outs = dict(outq.get(timeout=240) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive and errq.empty()
    return outs


def test_sharded_self_check_gloo():
    """bench.sharded_self_check (the N > 1 line's mpk check and per-rank step spread) over gloo: the
    all-gathered partial sums of a_i0 reproduce the mpk, and `rank_ms` holds the min / max over ranks
    of the shard time and of every host step."""
    outs = _self_check(3, wrong=-1)
    for r in range(3):
        o = outs[r]
        assert o["mpk_check"].startswith("mpk == g"), o
        rm = o["rank_ms"]
        assert rm["shard_device"] == {"min": 1.0, "max": 3.0}
        assert rm["exchange"] == {"min": 0.5, "max": 1.5}
        assert rm["combine"] == {"min": 0.2, "max": 0.2} and rm["recon"] == {"min": 0.0, "max": 0.0}
        # every rank's device, all-gathered in rank order
        assert o["rank_devices"] == ["0000:05:00.0", "0000:15:00.0", "0000:25:00.0"], o
        assert o["distinct_devices"] == 3 and o["dist"] == {"backend": "gloo", "world_size": 3}


def test_sharded_self_check_shared_device_gloo_rehearsal():
    """The gloo rehearsal on one GPU: every rank reports the same device and the line says so."""
    outs = _self_check(2, wrong=-1, shared=True)
    for r in range(2):
        assert outs[r]["rank_devices"] == ["0000:05:00.0"] * 2 and outs[r]["distinct_devices"] == 1


def test_sharded_self_check_rccl_refuses_shared_devices():
    """Under RCCL the N > 1 line must come from N distinct devices: ranks sharing one fail."""
    outs = _self_check(2, wrong=-1, backend="nccl", shared=True)
    assert all("share devices" in outs[r].get("exit", "") for r in range(2)), outs


def test_sharded_self_check_catches_a_wrong_mpk():
    """Every rank holds the same (wrong) mpk after the exchange, so every rank fails the check (in the
    bench, the launcher then ends the run non-zero)."""
    outs = _self_check(2, wrong=-2)
    assert all("sharded mpk" in outs[r]["assertion"] for r in range(2)), outs
