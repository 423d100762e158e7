"""Packed decision rows (dkg_decisions_pack_device, dkg_shard_combine_packed_device): the bitmaps the
ranks of a sharded ceremony all-gather (north_star: "RCCL all-gather ... of the complaint /
verification bitmaps"; committee.rs:311-347 -- every party learns every complaint) instead of n bytes
per row.  The packed words equal the checker's restatement (tests/combine_ref.py pack_rows), and the
packed combine gives the byte combine's outcome and matrices bit for bit on random matrices in the
padded rank layout; rows the encoding cannot carry are refused, not truncated."""
import numpy as np
import pytest

import dkg_amd
from dkg_amd import ACCEPT, MISSING, REJECT, SELF, SKIPPED
from tests import combine_ref as CR

pytestmark = pytest.mark.gpu
CK = b"shared commitment key"


@pytest.fixture(scope="module")
def be():
    b = dkg_amd.Backend(0)
    yield b
    b.close()


def _raw(rng, n, round_):
    p = float(rng.choice([0.0, 0.01, 0.3, 0.9]))
    dec = np.where(rng.random((n, n)) < p, REJECT, ACCEPT).astype(np.uint8)
    if round_ == 2 and n > 3:
        for i in rng.choice(n, size=int(rng.integers(0, 4)), replace=False):
            dec[i, :] = MISSING
    np.fill_diagonal(dec, SELF)
    return dec


@pytest.mark.parametrize("seed", range(10))
def test_packed_combine_equals_byte_combine(be, seed):
    import torch

    rng = np.random.default_rng(100 + seed)
    n = int(rng.choice([2, 3, 10, 31, 32, 33, 64, 100, 257, 1024]))
    t = int(rng.integers(0, (n + 1) // 2))
    ws = int(rng.integers(1, min(8, n) + 1))
    R, W1 = CR.rows_per_rank(ws, n), dkg_amd.packed_row_words(n)
    assert W1 == CR.packed_words(n)
    dec2, dec4 = _raw(rng, n, 2), _raw(rng, n, 4)
    be.env_init(t, n, CK)
    dev = torch.device("cuda", 0)
    g = {}
    for name, dec in (("2", dec2), ("4", dec4)):
        packed = torch.randint(-2**31, 2**31 - 1, (ws * R * W1,), dtype=torch.int32).to(dev)  # stale words
        for r in range(ws):
            d0, d1 = dkg_amd.shard_range(n, ws, r)
            rows = torch.from_numpy(np.ascontiguousarray(dec[d0:d1])).to(dev)
            be.decisions_pack_device(R, d1 - d0, n, d0, rows.data_ptr(), packed[r * R * W1:].data_ptr())
            got = packed[r * R * W1:(r + 1) * R * W1].cpu().numpy().view(np.uint32).reshape(R, W1)
            assert (got == CR.pack_rows(dec[d0:d1], R, d1 - d0, n, d0)).all(), (seed, name, r)
        g[name] = packed
        assert (CR.unpack_ranks(packed.cpu().numpy().view(np.uint32), ws, n) == dec).all()
    c2, c4 = (torch.empty(n * n, dtype=torch.uint8, device=dev) for _ in range(2))
    o = be.shard_combine_device(n, t, ws, g["2"].data_ptr(), g["4"].data_ptr(), c2.data_ptr(), c4.data_ptr(),
                                packed=True)
    b2 = torch.from_numpy(CR.pad(dec2, ws, n, n)).to(dev)
    b4 = torch.from_numpy(CR.pad(dec4, ws, n, n)).to(dev)
    e2, e4 = (torch.empty(n * n, dtype=torch.uint8, device=dev) for _ in range(2))
    ob = be.shard_combine_device(n, t, ws, b2.data_ptr(), b4.data_ptr(), e2.data_ptr(), e4.data_ptr())
    assert o == ob, (seed, n, t, ws)
    assert torch.equal(c2, e2) and torch.equal(c4, e4)
    assert bytes(c2.cpu().numpy()) == bytes(dec2)


@pytest.mark.parametrize("bad", ["skipped_in_checked_row", "partial_missing", "diagonal", "value_5"])
def test_pack_refuses_rows_it_cannot_carry(be, bad):
    import torch

    n, d0 = 40, 3
    dec = _raw(np.random.default_rng(7), n, 2)[d0:d0 + 4].copy()
    dec[:] = ACCEPT
    for r in range(4):
        dec[r, d0 + r] = SELF
    if bad == "skipped_in_checked_row":
        dec[1, 9] = SKIPPED
    elif bad == "partial_missing":
        dec[2, :] = MISSING
        dec[2, d0 + 2] = SELF
        dec[2, 30] = ACCEPT
    elif bad == "diagonal":
        dec[0, d0] = ACCEPT
    else:
        dec[3, 0] = 5
    with pytest.raises(ValueError):
        CR.pack_rows(dec, 4, 4, n, d0)
    dev = torch.device("cuda", 0)
    rows = torch.from_numpy(dec).to(dev)
    out = torch.zeros(4 * dkg_amd.packed_row_words(n), dtype=torch.int32, device=dev)
    with pytest.raises(dkg_amd.DkgError):
        be.decisions_pack_device(4, 4, n, d0, rows.data_ptr(), out.data_ptr())
