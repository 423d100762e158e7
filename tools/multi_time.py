"""Wall time of one ceremony through the in-library multi-device context (dkg_multi_*, one process
driving several GPUs) against one context, from device-resident coefficients.

On a node with K GPUs, `--devices 0,1,...,K-1` times the real fan-out (shard threads + the peer-copy
gather into the first device); on a one-GPU box `--devices 0,0` shares the GPU between the shards
(a check of the orchestration cost, not a scaling figure).  Prints one JSON line per repetition
with the context's step times (dkg_multi_phase_ms).
usage: python3 tools/multi_time.py [n t] [--devices 0,1] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int, nargs="?", default=1024)
    ap.add_argument("t", type=int, nargs="?", default=511)
    ap.add_argument("--devices", default="0,0")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    import dkg_amd

    n, t = args.n, args.t
    N = t + 1
    devs = [int(x) for x in args.devices.split(",")]
    a, b = dkg_amd.dealer_coefficients(bytes(range(32)), 1, 0, n, t)
    single = dkg_amd.Backend(devs[0])
    single.env_init(t, n)
    ta, tb = (torch.frombuffer(bytearray(x), dtype=torch.uint8).to(f"cuda:{devs[0]}") for x in (a, b))
    m = dkg_amd.MultiBackend(devs)
    m.env_init(t, n)
    bufs = []
    for i, d in enumerate(devs):
        d0, d1 = dkg_amd.shard_range(n, len(devs), i)
        bufs.append([torch.frombuffer(bytearray(x[32 * N * d0:32 * N * d1]), dtype=torch.uint8).to(f"cuda:{d}")
                     for x in (a, b)])
    want = single.ceremony_device(ta.data_ptr(), tb.data_ptr(), n, t).mpk
    for rep in range(args.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r1 = single.ceremony_device(ta.data_ptr(), tb.data_ptr(), n, t)
        t1 = time.perf_counter()
        r = m.ceremony_device([x[0].data_ptr() for x in bufs], [x[1].data_ptr() for x in bufs], n, t)
        t2 = time.perf_counter()
        assert r.mpk == want == r1.mpk and r.n_qualified == n
        if rep:  # the first round builds tables and lattice multipliers
            print(json.dumps({"n": n, "t": t, "devices": devs, "single_ms": round((t1 - t0) * 1e3, 2),
                              "multi_ms": round((t2 - t1) * 1e3, 2),
                              "multi_steps_ms": {k: round(v, 3) for k, v in m.phase_ms().items()}}), flush=True)
    m.close()
    single.close()


if __name__ == "__main__":
    main()
