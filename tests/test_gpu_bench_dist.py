"""The N > 1 bench line on a GPU: `bench.py --gpus N --dist-backend gloo` as a
fresh child process, its ranks sharing GPU 0 -- the launcher (bench.spawn_ranks), the dealer-sharded
ceremony with its all-gathers, the combine / reconstruction / finalise (dkg_amd/distributed.py), the
mpk self-check (bench.sharded_self_check) and the per-rank roofline pass: the code the driver's
multi-GPU run executes first, with gloo standing in for RCCL.  The line is a check that the path
runs, not a scaling figure (the ranks share one GPU).  With DKG_SAVE_LINES=<dir> the JSON lines are
also written there (gpurun_out/ on the GPU box, copied to profiles/)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("gpus", [2, 3])
def test_bench_multi_rank_gloo_on_one_gpu(gpus):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dist-backend", "gloo",
           "--steps", "2", "--warmup", "1", "--no-cpu", "--no-interp", "--dist-timeout", "120"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, p.stdout[-2000:]  # exactly one result line, from rank 0
    out = json.loads(lines[0])
    save = os.environ.get("DKG_SAVE_LINES")
    if save:
        os.makedirs(save, exist_ok=True)
        with open(os.path.join(save, f"bench_gloo{gpus}.json"), "w") as f:
            f.write(lines[0] + "\n")
    assert out["n_gpus"] == gpus and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == f"dealer-sharded x{gpus}"
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["value"] == pytest.approx(out["config"]["pairs_per_step"] / (out["ms_per_step"] / 1e3), rel=1e-6)
    assert out["mpk_check"].startswith("mpk == g")
    # the rehearsal's ranks share GPU 0: one device, named by its PCI bus id on every rank
    assert len(out["rank_devices"]) == gpus and len(set(out["rank_devices"])) == 1, out["rank_devices"]
    assert out["distinct_devices"] == 1 and out["dist"] == {"backend": "gloo", "world_size": gpus}
    clk = out["sclk_mhz"]
    assert 500 < clk["before"] < 4000 and 500 < clk["after"] < 4000, clk
    rm = out["rank_ms"]
    assert set(rm) == {"shard_device", "exchange", "combine", "recon", "finalise"}
    for k, v in rm.items():
        assert 0 <= v["min"] <= v["max"], (k, v)
    assert rm["shard_device"]["min"] > 0
    ex = out["exchange"]  # the decisions travel as packed bitmaps (dkg_decisions_pack_device)
    assert ex["decisions"] == "packed bitmaps" and ex["bytes_per_rank"] < ex["bytes_per_rank_byte_rows"]
    rl = out["roofline"]
    assert rl["bound"] and rl["peak"] > 0 and 0 < rl["frac"] <= 1.2, rl
    assert 0 < rl["instr_frac"] < rl["frac"], rl
    if gpus == 2 and rl["kernel"] == "stepping":  # the one-GPU profile's (n, t, U, L) = this shard's
        assert rl["instr_frac"] < rl["frac_counter_lower_bound"] <= rl["frac"] * 1.01, rl
