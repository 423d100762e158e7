"""Per-rank device time of the dealer-sharded ceremony at N GPUs, emulated on ONE GPU.

Rank 0 of an N-way split owns dealers [0, n/N); dkg_ceremony_shard_device runs exactly what that
rank runs (share gen + round-2/4 checks of its rows against all n receivers + partial sums).  The
RCCL all-gathers that follow are not included (they move n^2 * 2 bytes of decisions plus ~n*64 B).
usage: python3 tools/shard_time.py [n t] [--no-overlap] [--streams K] [--split U] [--stepping M] [--field F]
                                  [--combine C] [--binomial B] [--ws 1,2,4,8]
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
    ap.add_argument("--ws", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--split", type=int, default=0, help="degree split (0: cost model)")
    ap.add_argument("--stepping", type=int, default=0, help="stepping slots: 0 model, 1 per column, 2 per piece, 3 no dead-position repack")
    ap.add_argument("--field", type=int, default=0, help="field multiply: 0 by occupancy, 1 product scanning, 2 column sums")
    ap.add_argument("--combine", type=int, default=0, help="recombination: 0 short multipliers (U <= 4), 1 powers of j^L")
    ap.add_argument("--binomial", type=int, default=0, help="binomial schedule (dkg_ctx_set_binomial): 0 default, 1 no lane pairs, 2 lane pairs for all steps, 3 per step as 0, 4 per-wave loops")
    args = ap.parse_args()
    import torch

    import dkg_amd

    n, t = args.n, args.t
    N = t + 1
    be = dkg_amd.Backend(0)
    be.set_overlap(not args.no_overlap)
    be.set_streams(args.streams)
    be.set_split(args.split)
    be.set_stepping(args.stepping)
    be.set_field_mode(args.field)
    be.set_combine(args.combine)
    be.set_binomial(args.binomial)
    be.env_init(t, n)
    dev = torch.device("cuda", 0)
    res = {}
    for ws in (int(x) for x in args.ws.split(",")):
        D = n // ws
        a, b = dkg_amd.dealer_coefficients(b"\xbe" * 32, 0, 0, D, t)
        ta = torch.frombuffer(bytearray(a), dtype=torch.uint8).to(dev)
        tb = torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
        o2 = torch.empty(D * n, dtype=torch.uint8, device=dev)
        o4 = torch.empty_like(o2)
        oA = torch.empty(D * 32, dtype=torch.uint8, device=dev)
        op = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        args_ = (n, t, 0, D, ta.data_ptr(), tb.data_ptr(), o2.data_ptr(), o4.data_ptr(), oA.data_ptr(),
                 op.data_ptr())
        be.ceremony_shard_device(*args_)  # warm-up (allocations)
        ms = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            be.ceremony_shard_device(*args_)
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
        if not os.environ.get("DKG_EXP_TIMING_ONLY"):  # experiment builds that compute wrong values
            assert bool((o2.view(D, n) != 0).all()), "an honest shard rejected a share"
        res[ws] = round(min(ms), 2)
        ph = be.phase_times("r24" if not args.no_overlap else "r4")
        print(json.dumps({"n": n, "t": t, "ws": ws, "dealers": D, "ms_wall": res[ws],
                          "overlap": not args.no_overlap, "streams": args.streams, "split": be.last_split(),
                          "split_len": be.last_split_len(), "stepping": args.stepping, "field": args.field, "combine": be.last_combine(),
                          "binomial": args.binomial,
                          "phases_ms_if_serialised": {k: round(v, 3) for k, v in ph.items()}}), flush=True)
    base = res.get(1)
    if base:
        print(json.dumps({"speedup_vs_1": {k: round(base / v, 2) for k, v in res.items()}}))
    be.close()


if __name__ == "__main__":
    main()
