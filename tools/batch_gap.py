"""Config 5's wall time against its device time, step by step: where the host spends the gap.

For each step: the wall time of the library call (dkg_ceremony_batch_device, which returns after its
own synchronisation), the device span it reports (first to last event), and the Python wrapper's
result assembly.  Usage: python tools/batch_gap.py [--steps K] [--config B5]"""
import argparse
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--config", default="B5")
    a = ap.parse_args()
    import torch

    import bench
    import dkg_amd
    from dkg_amd import _lib, api

    B, n, t = bench.BATCH[a.config]
    N = t + 1
    be = dkg_amd.Backend(0)
    be.env_init(t, n)
    ta = torch.empty(B * n * N * 32, dtype=torch.uint8, device="cuda")
    tb = torch.empty_like(ta)
    be.dealer_coefficients_device(b"\xb5" * 32, 0, B, 0, n, t, ta.data_ptr(), tb.data_ptr())
    o, bufs = api._batch_out(B, n, False)
    lib = _lib.lib()
    for k in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = lib.dkg_ceremony_batch_device(be.ctx, B, n, t, ctypes.c_void_p(ta.data_ptr()),
                                           ctypes.c_void_p(tb.data_ptr()), ctypes.byref(o))
        t1 = time.perf_counter()
        res = api._batch_result(B, n, t, o, bufs)
        t2 = time.perf_counter()
        assert rc == 0
        print(f"step {k}: call {1e3 * (t1 - t0):.2f} ms, device span {o.ms_total:.2f} ms "
              f"(checks {o.ms_checks:.2f}, round3 {o.ms_round3:.2f}, finalise {o.ms_finalise:.2f}), "
              f"wrapper {1e3 * (t2 - t1):.2f} ms, qualified {min(res.n_qualified)}", flush=True)


if __name__ == "__main__":
    main()
