"""Time the trait-boundary batched MSM (dkg_msm_batch: Straus, 4-bit windows split over a
workgroup) for a few (B, N) shapes; host->device upload and decode included."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401  (HIP runtime first)

    import dkg_amd
    from tests import oracle_lib as O

    L = 2**252 + 27742317777372353535851937790883648493
    rng = random.Random(5)
    be = dkg_amd.Backend(0)
    base = [O.base_mul(rng.randrange(1, L).to_bytes(32, "little")) for _ in range(64)]
    for B, N in [(1, 512), (1, 2048), (64, 32), (1024, 32), (256, 512)]:
        pts = b"".join(base[(i * 7) % 64] for i in range(B * N))
        sc = b"".join(rng.randrange(L).to_bytes(32, "little") for _ in range(B * N))
        be.msm_batch(sc, pts, B, N)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            be.msm_batch(sc, pts, B, N)
        ms = (time.perf_counter() - t0) / reps * 1e3
        print(json.dumps({"B": B, "N": N, "ms": round(ms, 3), "terms_per_s": B * N / ms * 1e3}), flush=True)
    be.close()


if __name__ == "__main__":
    main()
