"""One rank of tests/test_gpu_dist.py (not a test module): a dealer-sharded ceremony end to end
through dkg_amd.distributed.ShardedCeremony on GPU 0, ranks sharing the GPU over gloo (the
rehearsal mode of bench.py --dist-backend gloo), or one rank over RCCL (DKG_DIST_BACKEND=nccl: the
real collectives and the device-side fences, world size 1 on a one-GPU box).  Started as a child process with RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT set; rank 0 writes every ceremony's combined outputs as
JSON to argv[1].  With argv[2] = a directory holding cfg.json and a tampered committee's E.bin,
A.bin, s.bin, sp.bin (tests/test_gpu_dist.py, BASELINE size), each rank reads its dealers' slices
of those and runs them, plus an honest ceremony of cfg's seed; digests of the large outputs."""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (before libdkg_amd.so: its HIP runtime must be torch's)
import torch.distributed as dist  # noqa: E402

import dkg_amd  # noqa: E402
from dkg_amd.distributed import ShardedCeremony, dealer_range  # noqa: E402

HONEST = ["ceremony_n16_t7.json", "ceremony_n64_t31.json"]
FAULTS = ["fault_a_generator_n10_t4.json", "fault_self_share_n10_t4.json", "fault_recon_only_n10_t4.json",
          "fault_a_many_n10_t4.json", "fault_share_flip_n10_t4.json", "fault_recon_r2err_n16_t3.json",
          "fault_recon_insufficient_n16_t3.json"]
H = bytes.fromhex


def golden(name):
    with open(os.path.join(ROOT, "tests", "golden", name)) as f:
        return json.load(f)


def summary(res):
    d = res.decisions
    b = lambda x: bytes(x.reshape(-1).cpu().numpy()) if hasattr(x, "cpu") else bytes(x.reshape(-1))  # noqa: E731
    return {"dec2": "".join(str(v) for v in b(d.dec2)), "dec4": "".join(str(v) for v in b(d.dec4)),
            "qualified": [int(x) for x in d.qualified], "reconstruct": [int(x) for x in d.reconstruct],
            "complaints2": [int(x) for x in d.complaints2], "r4_error": [int(x) for x in d.r4_error],
            "phase4_error": bool(d.phase4_error), "final_share": res.final_share.hex(),
            "public_share": res.public_share.hex() if res.public_share is not None else None,
            "mpk": res.mpk.hex() if res.mpk is not None else None}


def digest(res):
    """summary() with the n x n decision matrices and the share vectors as SHA-256 digests."""
    d = summary(res)
    for k in ("dec2", "dec4", "final_share", "public_share"):
        d[k] = hashlib.sha256(d[k].encode()).hexdigest() if d[k] is not None else None
    return d


def big(be, dev, rank, ws, d):
    with open(os.path.join(d, "cfg.json")) as f:
        cfg = json.load(f)
    n, t = cfg["n"], cfg["t"]
    N = t + 1
    be.env_init(t, n)
    d0, d1 = dealer_range(rank, ws, n)

    def load(name, w):  # this rank's dealers' rows only
        a = np.fromfile(os.path.join(d, name), dtype=np.uint8, count=w * (d1 - d0), offset=w * d0)
        return torch.from_numpy(a).to(dev)

    tE, tA, ts, tsp = load("E.bin", 32 * N), load("A.bin", 32 * N), load("s.bin", 32 * n), load("sp.bin", 32 * n)
    out = {"tampered": digest(ShardedCeremony(be, dist, n, t, dev).run_verify(
        tE.data_ptr(), tA.data_ptr(), ts.data_ptr(), tsp.data_ptr()))}
    a, b = dkg_amd.dealer_coefficients(H(cfg["master_seed"]), cfg["ceremony"], d0, d1 - d0, t)
    ta, tb = (torch.frombuffer(bytearray(x), dtype=torch.uint8).to(dev) for x in (a, b))
    out["honest"] = digest(ShardedCeremony(be, dist, n, t, dev).run(ta.data_ptr(), tb.data_ptr()))
    return out


def main(out_path, big_dir=None):
    rank = int(os.environ["RANK"])
    backend = os.environ.get("DKG_DIST_BACKEND", "gloo")
    dev = torch.device("cuda", 0)
    if backend == "nccl":  # RCCL: one GPU per rank, so world size 1 on a one-GPU box
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    ws = dist.get_world_size()
    be = dkg_amd.Backend(0)
    put = lambda x: torch.frombuffer(bytearray(x or b"\0"), dtype=torch.uint8).to(dev)  # noqa: E731
    out = {}
    if big_dir:
        out = big(be, dev, rank, ws, big_dir)
        dist.barrier()
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump(out, f)
        be.close()
        dist.destroy_process_group()
        return
    for name in HONEST:  # share generation + checks of this rank's dealers, exchange, combine, finalise
        c = golden(name)
        n, t = c["n"], c["t"]
        be.env_init(t, n)
        d0, d1 = dealer_range(rank, ws, n)
        a, b = dkg_amd.dealer_coefficients(H(c["master_seed"]), c["ceremony"], d0, d1 - d0, t)
        ta, tb = put(a), put(b)  # keep both alive: a freed temporary's memory would be handed to the next
        out[name] = summary(ShardedCeremony(be, dist, n, t, dev).run(ta.data_ptr(), tb.data_ptr()))
    for name in FAULTS:  # received (tampered) broadcasts: rounds 2-5 incl. the reconstruction exchange
        c = golden(name)
        n, t = c["n"], c["t"]
        N = t + 1
        be.env_init(t, n)
        d0, d1 = dealer_range(rank, ws, n)
        E, A, s, sp = (H(c[k]) for k in ("E", "A", "s", "s_prime"))
        tE, tA = put(E[32 * N * d0:32 * N * d1]), put(A[32 * N * d0:32 * N * d1])
        ts, tsp = put(s[32 * n * d0:32 * n * d1]), put(sp[32 * n * d0:32 * n * d1])
        sc = ShardedCeremony(be, dist, n, t, dev)
        out[name] = summary(sc.run_verify(tE.data_ptr(), tA.data_ptr(), ts.data_ptr(), tsp.data_ptr()))
    dist.barrier()
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(out, f)
    be.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(*sys.argv[1:3])
