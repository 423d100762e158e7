"""The dealer-sharded multi-GPU path as ONE unit across processes: ShardedCeremony.run /
run_verify + dkg_ceremony_shard_device / _shard_verify_device + the all-gathers + the library's
combine, reconstruction exchange and finalise (dkg_amd/distributed.py), in 2 and 3 spawned ranks that
share GPU 0 over gloo and in one rank over RCCL (tests/dist_worker.py).  Every combined output equals
the single-GPU golden ceremony."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("ws,backend", [(2, "gloo"), (3, "gloo"), (1, "nccl")])
def test_sharded_ceremony_processes(tmp_path, golden, ws, backend):
    """gloo: 2 and 3 ranks sharing GPU 0 (exchange staged through host memory).  nccl: one rank over
    RCCL -- the real all_gather_into_tensor on device buffers and the stream fences around the
    library's calls (one GPU per rank, so world size 1 here; the driver's 8-GPU node runs more)."""
    out = tmp_path / "dist.json"
    port = _free_port()
    procs = []
    for r in range(ws):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(ws), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), DKG_DIST_BACKEND=backend)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_worker.py"), str(out)],
                                      env=env))
    try:
        rcs = [p.wait(timeout=100) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * ws, rcs
    res = json.loads(out.read_text())
    assert len(res) == 7
    for name, got in res.items():
        c = golden(name)
        for k in ("dec2", "dec4", "qualified", "reconstruct", "complaints2", "final_share", "public_share"):
            assert got[k] == c[k], (name, k)
        assert got["r4_error"] == [int(x) for x in c["r4_error"]], name
        assert got["phase4_error"] == c["phase4_error"], name
        if c["phase4_error"]:
            assert got["mpk"] is None, name  # Phases<Phase4>::proceed fails for everyone (committee.rs:673-677)
        else:
            assert got["mpk"] == c["mpk"], name
