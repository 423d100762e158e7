"""ctypes loader for the CPU oracle (oracle/build/libdkg_oracle.so) — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker / timed CPU baseline.  The product path (dkg_amd) never imports it.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("DKG_ORACLE_LIB", os.path.join(ROOT, "oracle", "build", "libdkg_oracle.so"))

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        _lib = ctypes.CDLL(LIB)
        sz = ctypes.c_size_t
        _lib.or_msm.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, ctypes.c_char_p]
        _lib.or_poly_eval.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_char_p]
        _lib.or_share_gen.argtypes = [sz, sz, sz, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                      ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                      ctypes.c_int]
        _lib.or_verify_pairs.argtypes = [sz, sz, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p,
                                         ctypes.c_char_p, ctypes.c_char_p, sz, sz, sz, sz, ctypes.c_char_p,
                                         ctypes.c_int]
        _lib.or_verify_pairs_rows.argtypes = _lib.or_verify_pairs.argtypes
        _lib.or_dealer_coeffs.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, ctypes.c_char_p]
        _lib.or_dealer_seed.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]
        _lib.or_lagrange.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, sz]
        _lib.or_blake2b.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz]
        _lib.or_chacha20_stream.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, sz]
        _lib.or_pt_hash_to_group.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz]
        _lib.or_sc_from_u64.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
        cp = ctypes.c_char_p
        _lib.or_chacha20_ietf_xor.argtypes = [cp, cp, sz, cp, cp]
        _lib.or_hybrid_encrypt.argtypes = [cp, cp, cp, cp, cp, sz]
        _lib.or_hybrid_decrypt.argtypes = [cp, cp, cp, cp, sz]
        _lib.or_member_sk.argtypes = [cp, cp, ctypes.c_uint32, ctypes.c_uint32]
        _lib.or_enc_randomness.argtypes = [cp, cp, sz, sz]
        _lib.or_misbehaviour_prove.argtypes = [cp, cp, cp, cp]
        _lib.or_complaint1_verify.argtypes = [cp, sz, ctypes.c_uint32, cp, cp, cp, cp]
        _lib.or_complaint3_verify.argtypes = [cp, sz, ctypes.c_uint32, cp, cp, cp, cp]
    return _lib


def _b(n):
    return ctypes.create_string_buffer(n)


def call32(name, *args):
    out = _b(32)
    rc = getattr(lib(), name)(out, *args)
    return out.raw, rc


def base_mul(k):
    return call32("or_pt_base_mul", k)[0]


def msm(scalars: bytes, points: bytes):
    n = len(scalars) // 32
    out, rc = call32("or_msm", n, scalars, points)
    return out if rc == 0 else None


def poly_eval(coeffs: bytes, x: bytes):
    out = _b(32)
    lib().or_poly_eval(out, coeffs, len(coeffs) // 32, x)
    return out.raw


def dealer_seed(master: bytes, ceremony: int, dealer: int):
    out = _b(32)
    lib().or_dealer_seed(out, master, ceremony, dealer)
    return out.raw


def dealer_coeffs(seed: bytes, t: int):
    a, b = _b(32 * (t + 1)), _b(32 * (t + 1))
    lib().or_dealer_coeffs(seed, t, a, b)
    return a.raw, b.raw


def share_gen(D, n, t, a, b, h, nthreads=0):
    N = t + 1
    E, A, s, sp = _b(32 * D * N), _b(32 * D * N), _b(32 * D * n), _b(32 * D * n)
    lib().or_share_gen(D, n, t, a, b, h, E, A, s, sp, nthreads)
    return E.raw, A.raw, s.raw, sp.raw


def verify_pairs(n, t, rnd, C, h, s, sp, d0, d1, r0, r1, nthreads=0):
    acc = _b((d1 - d0) * (r1 - r0))
    rc = lib().or_verify_pairs(n, t, rnd, C, h, s, sp or b"", d0, d1, r0, r1, acc, nthreads)
    return acc.raw, rc


def verify_rows(n, t, rnd, C, h, s, sp, d0, d1, r0, r1, nthreads=0):
    """verify_pairs on row-local arrays holding dealers d0..d1-1 only (C [d1-d0][t+1], s / sp
    [d1-d0][n]); the SELF diagonal stays at the global dealer index."""
    acc = _b((d1 - d0) * (r1 - r0))
    rc = lib().or_verify_pairs_rows(n, t, rnd, C, h, s, sp or b"", d0, d1, r0, r1, acc, nthreads)
    return acc.raw, rc


def hybrid_encrypt(pk: bytes, r: bytes, msg: bytes):
    e1, e2 = _b(32), _b(len(msg))
    rc = lib().or_hybrid_encrypt(e1, e2, pk, r, msg, len(msg))
    return (e1.raw, e2.raw) if rc == 0 else None


def hybrid_decrypt(sk: bytes, e1: bytes, e2: bytes):
    m = _b(len(e2))
    rc = lib().or_hybrid_decrypt(m, sk, e1, e2, len(e2))
    return m.raw if rc == 0 else None


def member_sk(master: bytes, ceremony: int, member: int):
    out = _b(32)
    lib().or_member_sk(out, master, ceremony, member)
    return out.raw


def enc_randomness(seed: bytes, t: int, n: int):
    out = _b(64 * n)
    lib().or_enc_randomness(out, seed, t, n)
    return out.raw


def misbehaviour_prove(sk: bytes, enc: bytes, w: bytes):
    out = _b(192)
    rc = lib().or_misbehaviour_prove(out, sk, enc, w)
    return out.raw if rc == 0 else None


def complaint1_verify(h, t, accuser, pk, enc, E, proof):
    return lib().or_complaint1_verify(h, t, accuser, pk, enc, E, proof)


def complaint3_verify(h, t, accuser, share, randomness, E, A):
    return lib().or_complaint3_verify(h, t, accuser, share, randomness, E, A)
