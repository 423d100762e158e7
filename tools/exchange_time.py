"""Host-side cost of the multi-GPU exchange + combine (dkg_amd/distributed.py), measured on ONE GPU:
a world-size-1 RCCL group runs ShardedCeremony.run() for the shard of an N-way split (rank 0's
dealers) and the time is compared with the bare shard (dkg_ceremony_shard_device).
usage: python3 tools/exchange_time.py [--ws-emulated 8] [n t]"""
import argparse
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int, nargs="?", default=1024)
    ap.add_argument("t", type=int, nargs="?", default=511)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    import dkg_amd
    from dkg_amd.distributed import ShardedCeremony

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    n, t = args.n, args.t
    be = dkg_amd.Backend(0)
    be.env_init(t, n)
    dev = torch.device("cuda", 0)
    N = t + 1
    ta = torch.empty(n * N * 32, dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    be.dealer_coefficients_device(b"\xbe" * 32, 0, 1, 0, n, t, ta.data_ptr(), tb.data_ptr())
    sc = ShardedCeremony(be, dist, n, t, dev)
    sc.run(ta.data_ptr(), tb.data_ptr())
    torch.cuda.synchronize()
    full, shard = [], []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        r = sc.run(ta.data_ptr(), tb.data_ptr())
        torch.cuda.synchronize()
        full.append((time.perf_counter() - t0) * 1e3)
        shard.append(r.ms_shard)
    # the parts of ShardedCeremony._finish, one by one (device work synchronised after each)
    parts = {}

    def timed(name, f):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = f()
        torch.cuda.synchronize()
        parts[name] = min(parts.get(name, 1e9), (time.perf_counter() - t0) * 1e3)
        return out

    for _ in range(args.reps):
        timed("shard_device", lambda: be.ceremony_shard_device(n, t, sc.d0, sc.d1, ta.data_ptr(), tb.data_ptr(),
                                                               sc.dec2.data_ptr(), sc.dec4.data_ptr(),
                                                               sc.A0.data_ptr(), sc.part.data_ptr()))
        if sc.packed:
            timed("pack", lambda: (sc._pack(sc.dec2, sc.p2), sc._pack(sc.dec4, sc.p4)))
        timed("all_gathers", sc.exchange)  # packs again when packed
        o = timed("combine", lambda: be.shard_combine_device(n, t, 1, sc.g_dec2.data_ptr(), sc.g_dec4.data_ptr(),
                                                             sc.c_dec2.data_ptr(), sc.c_dec4.data_ptr(),
                                                             packed=sc.packed))
        q = [int(x) for x in o.qualified]
        timed("finalise", lambda: be.shard_finalise_device(n, t, 1, sc.g_A0.data_ptr(), sc.g_part.data_ptr(), q,
                                                           bool(o.phase4_error), sc.fs.data_ptr(), sc.pub.data_ptr()))
        timed("copy_out", lambda: (bytes(sc.fs.cpu().numpy()), bytes(sc.pub.cpu().numpy())))
    after = sorted(f - s for f, s in zip(full, shard))  # per run: wall minus the shard's device span
    print(json.dumps({"n": n, "t": t, "run_ms": round(min(full), 3), "shard_device_ms": round(min(shard), 3),
                      "exchange_and_combine_ms": round(min(full) - min(shard), 3),
                      "after_shard_ms_median": round(after[len(after) // 2], 3),
                      "after_shard_ms_min": round(after[0], 3),
                      "parts_ms": {k: round(v, 3) for k, v in parts.items()}}))
    be.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
