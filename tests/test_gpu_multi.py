"""The in-library multi-device context (dkg_multi_*, include/dkg_amd.h; dkg_amd/csrc/multi.cpp): one
process sharding a ceremony by dealer over several devices, one host thread per shard, exchanged by
peer copies into the first device.  On a one-GPU box the devices repeat ([0, 0], [0, 0, 0]): the
shards then share the GPU and the peer copies are device-local, which exercises every step of the
N-device path (ranges, padded gathers, combine, reconstruction on the owning shard, finalise).
Checked byte for byte against the libsodium goldens and the single-context run."""
import hashlib

import pytest

import dkg_amd
from tests.test_gpu import CEREMONIES, CK, FAULTS, H, _check_ceremony

pytestmark = pytest.mark.gpu

SHARDS = [[0], [0, 0], [0, 0, 0]]


@pytest.fixture(scope="module", params=SHARDS, ids=lambda d: f"ws{len(d)}")
def mb(request):
    m = dkg_amd.MultiBackend(request.param)
    yield m
    m.close()


@pytest.fixture(scope="module")
def be():
    b = dkg_amd.Backend(0)
    yield b
    b.close()


@pytest.mark.parametrize("name", CEREMONIES + ["ceremony_n64_t31.json"])
def test_multi_honest_goldens(mb, golden, name):
    c = golden(name)
    n, t = c["n"], c["t"]
    if len(mb) > n:
        pytest.skip("more shards than dealers")
    mb.env_init(t, n, CK)
    a, b = dkg_amd.dealer_coefficients(H(c["master_seed"]), c["ceremony"], 0, n, t)
    r = mb.ceremony(a, b, n, t)
    assert r.E is None
    _check_ceremony(c, r, n)
    ms = mb.phase_ms()
    assert all(v >= 0 for v in ms.values()), ms
    assert r.ms["total"] > 0


@pytest.mark.parametrize("name", FAULTS)
def test_multi_fault_goldens(mb, golden, name):
    """Tampered broadcasts (committee.rs:1105-1313), including round-4 reconstruction on the owning
    shard and the disclosure-dependent mpk (fault_recon_*)."""
    c = golden(name)
    n, t = c["n"], c["t"]
    mb.env_init(t, n, CK)
    r = mb.ceremony_verify(H(c["E"]), H(c["A"]), H(c["s"]), H(c["s_prime"]), n, t)
    _check_ceremony(c, r, n)


def _digest(r):
    return {k: hashlib.sha256(getattr(r, k)).hexdigest() for k in ("dec2", "dec4", "final_share", "public_share")} | {
        "mpk": r.mpk.hex(), "qualified": r.qualified, "reconstruct": r.reconstruct, "r4_error": r.r4_error}


def test_multi_n1024_matches_single_context(be, golden):
    """BASELINE's headline size over two shards, from host coefficients and from per-shard device
    buffers, against one context's run of the same ceremony."""
    import torch

    n, t = 1024, 511
    a, b = dkg_amd.dealer_coefficients(bytes(range(32)), 7, 0, n, t)
    be.env_init(t, n, CK)
    want = _digest(be.ceremony(a, b, n, t))
    assert want["qualified"] == [1] * n
    m = dkg_amd.MultiBackend([0, 0])
    try:
        m.env_init(t, n, CK)
        assert _digest(m.ceremony(a, b, n, t)) == want
        N = t + 1
        bufs = []
        for i in range(2):
            d0, d1 = dkg_amd.shard_range(n, 2, i)
            bufs.append([torch.frombuffer(bytearray(x[32 * N * d0:32 * N * d1]), dtype=torch.uint8).to("cuda:0")
                         for x in (a, b)])
        r = m.ceremony_device([x[0].data_ptr() for x in bufs], [x[1].data_ptr() for x in bufs], n, t)
        assert _digest(r) == want
        ms = m.phase_ms()
        assert ms["shard_max"] >= ms["shard_min"] > 0
    finally:
        m.close()


def test_multi_rejects_bad_arguments(golden):
    with pytest.raises(dkg_amd.DkgError):
        dkg_amd.MultiBackend([])
    with pytest.raises(dkg_amd.DkgError):
        dkg_amd.MultiBackend([0, 99])
    m = dkg_amd.MultiBackend([0, 0, 0])
    try:
        m.env_init(0, 2, CK)
        a, b = dkg_amd.dealer_coefficients(bytes(32), 0, 0, 2, 0)
        with pytest.raises(dkg_amd.DkgError):
            m.ceremony(a, b, 2, 0)  # three shards, two dealers
        with pytest.raises(dkg_amd.DkgError):
            m.ceremony(a, b, 2, 1)  # committee.rs:73
    finally:
        m.close()
