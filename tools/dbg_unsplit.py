"""Diagnosis of the n=1024, t=511 forced-unsplit ceremony (tests/test_gpu_scale.py
test_stepping_tail_repack_unsplit_n1024): the same tampered committee under the stepping's
dead-position repack (mode 0) and without it (mode 3), one and two chunk streams, each run twice on a
fresh context; prints, per run, how its decision matrices differ from the first run's.
usage: python3 tools/dbg_unsplit.py [--identity 0|1]"""
import argparse
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--identity", type=int, default=1)
    ap.add_argument("--n", type=int, default=1024)
    args = ap.parse_args()
    import dkg_amd
    from tests.test_gpu_scale import CK, _inject

    n = args.n
    t = (n - 1) // 2
    be = dkg_amd.Backend(0)
    be.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(bytes([77]) * 32, 6, 0, n, t)
    E, A, s, sp = (bytearray(x) for x in be.share_gen(a, b, n, n, t))
    _inject(random.Random(n + 17), n, t, E, A, s, sp)
    N = t + 1
    if args.identity:
        for d, buf in ((7, E), (9, A), (n - 1, E)):
            buf[32 * N * d:32 * N * (d + 1)] = bytes(32 * N)
    ref = None
    be.set_split(1)
    for mode, streams in ((3, 1), (3, 1), (3, 2), (0, 1), (0, 1), (0, 2), (0, 2), (3, 2)):
        be.set_stepping(mode)
        be.set_streams(streams)
        r = be.ceremony_verify(bytes(E), bytes(A), bytes(s), bytes(sp), n, t)
        d2, d4 = bytes(r.dec2), bytes(r.dec4)
        out = {"mode": mode, "streams": streams, "split": be.last_split(), "redos": be.stepping_redos(),
               "n_qualified": r.n_qualified}
        if ref is None:
            ref = (d2, d4, r.mpk)
        else:
            for name, x, y in (("dec2", d2, ref[0]), ("dec4", d4, ref[1])):
                diff = [k for k in range(n * n) if x[k] != y[k]]
                out[name + "_diffs"] = len(diff)
                out[name + "_first"] = [(k // n, k % n, x[k], y[k]) for k in diff[:8]]
                out[name + "_rows"] = sorted({k // n for k in diff})[:16]
            out["mpk_same"] = r.mpk == ref[2]
        print(json.dumps(out), flush=True)
    be.close()


if __name__ == "__main__":
    main()
