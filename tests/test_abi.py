"""CPU-only checks of the boundary: the C ABI library loads and exports every symbol that
include/dkg_amd.h declares; host-side logic (seeded coefficients, environment check, error path
without a GPU) behaves like the reference."""
import ctypes
import os
import re

import pytest

import dkg_amd
from dkg_amd import _lib
from tests import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "dkg_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dkg_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 18
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(_lib.EXPORTED)


def test_env_check_matches_reference_assert():
    # committee.rs:73: assert!(threshold < (nr_members + 1) / 2)
    for t, n in [(0, 1), (0, 2), (1, 3), (4, 10), (5, 11), (511, 1024), (2047, 4096)]:
        dkg_amd.env_check(t, n)
    for t, n in [(5, 10), (1, 2), (2, 3), (512, 1024), (0, 0)]:
        with pytest.raises(dkg_amd.DkgError):
            dkg_amd.env_check(t, n)


@pytest.mark.parametrize("t", [0, 3, 31])
def test_dealer_coefficients_match_oracle(t):
    master = bytes(range(32))
    a, b = dkg_amd.dealer_coefficients(master, 5, 3, 4, t)
    N = t + 1
    for i in range(4):
        oa, ob = O.dealer_coeffs(O.dealer_seed(master, 5, 3 + i), t)
        assert a[32 * N * i:32 * N * (i + 1)] == oa and b[32 * N * i:32 * N * (i + 1)] == ob


def test_dealer_coefficients_golden(golden):
    c = golden("ceremony_n10_t4.json")
    a, b = dkg_amd.dealer_coefficients(bytes.fromhex(c["master_seed"]), c["ceremony"], 0, c["n"], c["t"])
    assert a.hex() == c["a"] and b.hex() == c["b"]


def test_no_gpu_fails_loudly():
    """Without a visible GPU the product path raises; it never falls back to the CPU."""
    if _lib.lib().dkg_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(dkg_amd.DkgError):
        dkg_amd.Backend(0)
    with pytest.raises(dkg_amd.DkgError):
        dkg_amd.MultiBackend([0, 0])


@pytest.mark.parametrize("name", ["full_n4_t1.json", "full_n10_t4.json"])
def test_enc_randomness_golden(golden, name):
    """Host encryption randomness (committee.rs:171-172 draw order) against the libsodium fixture."""
    c = golden(name)
    r = dkg_amd.enc_randomness(bytes.fromhex(c["master_seed"]), c["ceremony"], 0, c["n"], c["n"], c["t"])
    assert r.hex() == c["enc_r"]


def test_split_multipliers():
    """Short recombination vectors (lattice.cpp): a_ju = b_j j^(uL) mod l exactly, b_j > 0, and
    entries near l^((U-1)/U) (the cheapest chain among small combinations of the reduced basis, a
    few bits above the shortest row): <= 132 / 174 / 195 / 208 bits for 2 / 3 / 4 / 5 pieces (253
    for the powers)."""
    import dkg_amd

    ell = 2**252 + 27742317777372353535851937790883648493
    for U, Lp, bound in ((2, 256, 132), (3, 171, 174), (4, 128, 195), (3, 683, 174), (5, 103, 208), (5, 410, 208)):
        rows = dkg_amd.split_multipliers(300, Lp, U)
        assert len(rows) == 300
        for j, row in enumerate(rows, 1):
            y = pow(j, Lp, ell)
            assert row[0] > 0
            assert all((row[u] - row[0] * pow(y, u, ell)) % ell == 0 for u in range(U))
            # the powers themselves are kept where their chain is cheaper (j = 2, 4 at U = 5: y a
            # power of two, NAFs of weight 1)
            powers = [pow(y, u, ell) for u in range(U)]
            assert max(abs(v).bit_length() for v in row) <= bound or row == powers, (U, j)
    with pytest.raises(dkg_amd.DkgError):
        dkg_amd.split_multipliers(10, 5, 6)


def test_split_cost_model():
    """The degree-split cost model (runtime.hip choose_split) picks a split where the binomial
    dominates (n=1024, t=511 and n=4096, t=2047) and none for small tables (config 5)."""
    L = _lib.lib()
    ms = lambda cols, n, t, U: L.dkg_split_model_ms(cols, n, t, U)  # noqa: E731
    assert ms(2048, 1024, 511, 2) < 0.9 * ms(2048, 1024, 511, 1)
    # n=1024 with short recombination multipliers: U=4 (4 x 128) measured ahead of U=3 (171 + 171 +
    # 170) and U=2 (profiles/r02_lattice_ab.txt)
    assert min(range(1, 9), key=lambda U: ms(2048, 1024, 511, U)) == 4
    assert L.dkg_split_len(2048, 1024, 511, 3) == 171 and L.dkg_split_len(2048, 1024, 511, 2) == 256
    assert L.dkg_split_len(2048, 1024, 511, 4) == 128
    # n=1100, U=2: 275 + 275 would leave 45 idle lanes per 320-lane stepping table: 320 + 230
    assert L.dkg_split_len(2304, 1100, 549, 2) == 320 and L.dkg_split_len(2304, 1100, 549, 3) == 192
    assert L.dkg_split_len(64, 10, 4, 6) == 0
    assert min(range(1, 17), key=lambda U: ms(8192, 4096, 2047, U)) == 4
    # dealer shards of n=1024 (2 rows per dealer): smaller shards split more (a shorter dependent
    # binomial chain; measured profiles/r01_shard_scaling_n1024_v13.txt for U in 1, 2, 4, 8)
    picks = [min(range(1, 9), key=lambda U: ms(c, 1024, 511, U)) for c in (2048, 1024, 512, 256)]
    # measured best at 1, 2, 4 and 8 ranks with 2..4 short pieces (profiles/r02_lattice_ab.txt); with
    # five short pieces (round 4) the model ties U=4 and U=5 at 4 ranks and prefers U=5 at 8 (the
    # automatic choice prices U=5 with powers unless built with DKG_AUTO_SHORT5: unmeasured there)
    assert picks[:2] == [4, 4] and picks[2] in (4, 5) and picks[3] in (4, 5)
    assert ms(16384, 64, 31, 1) < ms(16384, 64, 31, 2)
    assert ms(64, 10, 4, 6) == -1.0  # more pieces than coefficients
