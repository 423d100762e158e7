#!/usr/bin/env python3
"""Benchmark: verified shares/sec (whole node) for the n=1024, t=511 DKG ceremony (BASELINE.json).

One step = one full plaintext-mode ceremony on synthetic seeded coefficients already resident in
HBM: round-1 share generation (commitments E/A + all n^2 share evaluations), round-2 checks of all
n(n-1) shares, round-3 share aggregation, round-4 checks, finalise (master public key).
value = n(n-1) verified shares per ceremony x steps / wall time (max over ranks).

N GPUs (torchrun, one process per GPU): the SAME ceremony is sharded by dealer; every rank
generates and verifies its dealers' rows for all receivers, then RCCL all-gathers (over xGMI) the
decision rows, the A_i0 commitments and the final-share partial sums (strong scaling).

Also printed in the same JSON line: the roofline of the dominant kernel (VALU issue slots, with the
PMC-measured HBM bytes per launch) and the CPU baseline: the
dalek-algorithm-matched C oracle timed on a bounded sample of the same ceremony (share generation
and round-2 and round-4 checks of a subset of dealers against all receivers) on every host thread
this process may use, extrapolated to the whole ceremony.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

L = 2**252 + 27742317777372353535851937790883648493
CONFIGS = {"D": (1024, 511), "C": (256, 127), "E": (4096, 2047), "B": (64, 31)}
BATCH = {"B5": (10000, 64, 31)}  # BASELINE config 5: 10,000 independent n=64, t=31 ceremonies

# Peak VALU issue rate of one MI355X: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = one full-rate wave64
# instruction per 2 cycles per SIMD (v_add_u32 reaches 0.85 of it: profiles/r02_ubench_intrate3.txt).
# Work is counted on the implemented schedule: closed-form call counts of each group primitive x its
# static gfx950 count (tools/count_valu.py), in two units:
#   slots -- VALU issue slots: half-rate instructions (v_mad_u64_u32, v_mul_lo_u32, shifts, 3-operand
#            fused ops, carry adds; measured by tools/ubench/intrate*.hip) count 2, full-rate 1.  This
#            is the roofline's work: frac = 1 means every issue cycle of every SIMD was used.
#   instr -- plain VALU instruction count (the round-1 unit, reported beside it as instr_frac).
INT32_PEAK = 256 * 4 * 32 * 2.4e9
VALU = {"fe_mul": (140, 256), "fe_sq": (109, 185), "ge_add": (1184, 2152), "ge_add_signed": (1228, 2200),
        "ge_madd_signed": (1130, 1992), "ge_madd_signed_not": (1001, 1744), "ge_add_signed_not": (1100, 1954),
        "ge_add_ded": (1198, 2180), "ge_to_cached_ded": (70, 70),
        "fe_tight_zero": (16, 31), "ge_dbl_t": (1058, 1855), "ge_dbl_not": (930, 1611), "comb_window": (1181, 2074),
        "combw_window": (1171, 2037), "ge_to_cached": (193, 309), "eq": (633, 1151), "sc_mont_mul": (580, 834)}
INSTR = {k: v[0] for k, v in VALU.items()}
# an addition followed by a doubling skips T (ge_add_signed / ge_madd_signed / ge_add_lds with_t = false):
# one product less; the "_not" counts are measured for the signed forms, ge_add's is derived
NO_T = {"ge_add_signed": "ge_add_signed_not", "ge_madd_signed": "ge_madd_signed_not"}


def add_cost(VALU, name, with_t=True):
    if with_t:
        return VALU[name]
    if name in NO_T:
        return VALU[NO_T[name]]
    return VALU[name] - (VALU["ge_add_signed"] - VALU["ge_add_signed_not"])
def combw_windows():
    """Mixed additions per scalar of the fixed-base combs of g and h (points.h, radix 2^DKG_COMBW_BITS
    of the loaded build: dkg_fixed_base_windows)."""
    global _COMBW
    if _COMBW is None:
        import dkg_amd
        _COMBW = dkg_amd.lib().dkg_fixed_base_windows()
    return _COMBW


_COMBW = None


def key_comb_windows():
    """Mixed additions per scalar of the member keys' combs (full mode's encryption; dkg_key_comb_windows)."""
    import dkg_amd
    return dkg_amd.lib().dkg_key_comb_windows()
SLOTS = {k: v[1] for k, v in VALU.items()}


def dalek_msm_fp_mults(N):
    """SURVEY.md 8(d) cost model of curve25519-dalek 3.x's vartime_multiscalar_mul over N points in
    Fp multiplications: Straus below 190 points, else Pippenger with w = 6 / 7 / 8 (N < 500 / 800 /
    above) over ceil(256 / w) digits (w = 8: 33, the carry digit)."""
    if N < 190:
        return 1792 + 408 * N
    w = 6 if N < 500 else 7 if N < 800 else 8
    digits = -(-256 // w) if w < 8 else 33
    return digits * (8 * N + 18 * (2 ** (w - 1) - 1)) + (digits - 1) * (7 * w + 10) + N


VARBASE_MUL = 2403  # dalek-3 constant-time variable-base scalar multiplication, Fp-mults


def ref_equiv(n, t, value):
    """The reference-equivalent work rate: W2 = MSM(t+1) + 2 variable-base muls + 9
    Fp-mults per verified share (the receiver's round-2 check, committee.rs:287-305), W4 = MSM + 1
    mul (round 4, :532-548); value x W2 is what the reference's per-pair MSM schedule would have to
    sustain to match this throughput."""
    msm = dalek_msm_fp_mults(t + 1)
    w2, w4 = msm + 2 * VARBASE_MUL + 9, msm + VARBASE_MUL
    return {"W2_fp_mults_per_share": w2, "W4_fp_mults_per_share": w4,
            "ref_equiv_W2_fp_mults_per_s": value * w2, "ref_equiv_W2_W4_fp_mults_per_s": value * (w2 + w4),
            "note": "dalek-3 cost model of the reference's per-pair checks (SURVEY.md 8(d)) x verified shares/s"}


def kernel_rooflines(ph, work, work_i):
    """Per-kernel VALU roofline of a serialised pass: ph = device ms per kernel (HIP events)."""
    rl = {}
    for k in work:
        ms = ph.get(k, 0.0)
        if ms > 0:
            rl[k] = {"ms_per_pass": round(ms, 3), "valu_slots": work[k], "valu_instr": work_i[k],
                     "achieved_T_slots": work[k] / (ms / 1e3) / 1e12, "frac": work[k] / (ms / 1e3) / INT32_PEAK,
                     "instr_frac": work_i[k] / (ms / 1e3) / INT32_PEAK}
    return rl


def roofline_line(rl, dom, work_text):
    ach = rl[dom]["achieved_T_slots"]
    return {"bound": "valu-issue", "kernel": dom, "achieved": ach, "peak": INT32_PEAK / 1e12,
            "unit": "T VALU issue slots/s", "frac": ach / (INT32_PEAK / 1e12), "instr_frac": rl[dom]["instr_frac"],
            "traffic": None, "work": work_text, "all_kernels": rl}


# Full mode (hybrid encryption, hybrid.hip): per item (dealer, recipient, w) closed forms.  Encode /
# decode: one fe_pow22523 (252 squarings + 11 products) plus the Ristretto map's products
# (ge25519.h ristretto_encode / ristretto_decode: 11 and 13 more); Blake2b-512 of one block (12
# rounds x 8 G: six 64-bit adds at 3 slots, four 64-bit xors at 2, three non-trivial 64-bit
# rotates at 4) + one ChaCha20 block (20 rounds x 4 quarter-rounds: 4 adds, 4 xors, 4 rotates at 2)
# + the 32-byte XOR: an op-count model (its loops defeat a static count).
HY_ENCODE = (252, 22)   # (fe_sq, fe_mul)
HY_DECODE = (252, 24)
HY_SYM_SLOTS = 12 * 8 * (6 * 3 + 4 * 2 + 3 * 4) + 20 * 4 * (4 + 4 + 4 * 2) + 64


def hybrid_valu(n, sk, VALU=SLOTS):
    """Closed-form VALU work of full mode's encryption and decryption of all 2 n^2 items (n dealers x n
    recipients x {randomness, share}): k_enc_mul (the windows of g's comb and of pk_q's own global comb
    per item: dkg_fixed_base_windows + dkg_key_comb_windows), k_dec_mul_w4 (sk_q's width-4 window, wave-uniform: a doubling per digit below the
    top, an addition per nonzero digit, the odd multiples), the encode / decode kernels and k_sym_xor
    (model above)."""
    items = 2 * n * n
    enc = items * (combw_windows() + key_comb_windows()) * VALU["combw_window"]
    dec = 0
    for q in range(n):
        ds = _wnaf(int.from_bytes(sk[32 * q:32 * q + 32], "little"), 4)
        # k_dec_mul_w4: the odd multiples R, 3R, 5R, 7R (one doubling, three additions, four cached
        # forms); then from the top nonzero digit down: an addition per nonzero digit (the first onto
        # the identity), a doubling per digit below the top (T when an addition or the end follows)
        c = VALU["ge_dbl_t"] + 3 * VALU["ge_add"] + 5 * VALU["ge_to_cached"]
        top = max((i for i, d in enumerate(ds) if d), default=-1)
        for i in range(top, -1, -1):
            if i != top:
                c += VALU["ge_dbl_t"] if (ds[i] or i == 0) else VALU["ge_dbl_not"]
            if ds[i]:  # a doubling follows unless i = 0: no T
                c += add_cost(VALU, "ge_add_signed", i == 0)
        dec += 2 * n * c
    encode = HY_ENCODE[0] * VALU["fe_sq"] + HY_ENCODE[1] * VALU["fe_mul"]
    decode = HY_DECODE[0] * VALU["fe_sq"] + HY_DECODE[1] * VALU["fe_mul"]
    sym = HY_SYM_SLOTS if VALU is SLOTS else HY_SYM_SLOTS * 0.7
    return {"enc_mul": enc, "enc_encode": 2 * items * encode, "enc_sym": items * sym,
            "dec_decode": items * decode, "dec_mul": dec, "dec_encode": items * encode, "dec_sym": items * sym}


PT_BYTES = 160  # one extended point, 40 u32 words (SoA)
AFF_BYTES = 128  # kernels.hip AFFP_WORDS: one affine addend slot
TRAFFIC_DIR = os.path.join(ROOT, "profiles", "pmc_traffic")


def algorithmic_bytes(kernel, n, t, U, plen=None, per_wave=False, batch=1):
    """(bytes per launch, launches per pass) of a check-pipeline kernel in the serialised fused pass:
    2n columns (E and A rows) x U pieces (split_pieces: L positions, a shorter last one; DESIGN.md
    sections 3-4), times `batch` ceremonies.  per_wave: the binomial ran as per-wave Horner loops
    (k_binom_wave, one launch): per column the initial copy of C_t, then per step one load (the old
    e_{m-1}; e_m is carried in registers) and one store per live position and the copy of C_k."""
    if batch > 1:
        b, nl = algorithmic_bytes(kernel, n, t, U, plen, per_wave)
        return (None, None) if b is None else (b * batch, nl)
    pieces, Lp0 = split_pieces(t, U, plen)
    cols = 2 * n
    if kernel == "binomial" and per_wave:
        per_col = sum(2 * PT_BYTES + sum(2 * PT_BYTES * (1 + max(r - (Lp0 - Lp), 0)) for r in range(1, Lp0))
                      for Lp in pieces)
        return cols * per_col, 1
    if kernel == "binomial":  # step r: position 0 copies C_k (load+store), positions 1..r' load 2, store 1
        # (r' = r for full pieces, r - (L - Lp) for a short last piece, which starts late)
        per_pass = sum(cols * (2 * PT_BYTES + max(r - (Lp0 - Lp), 0) * 3 * PT_BYTES)
                       for r in range(1, Lp0) for Lp in pieces)
        return per_pass / max(Lp0 - 1, 1), max(Lp0 - 1, 1)
    if kernel == "stepping":  # the table once, then D_0 out per (piece, receiver) + its dense Z (40 B)
        nblk = -(-Lp0 // 512)
        zb = 40 if U > 1 else 0  # the Z copy exists for the affine recombination addends (U > 1)
        return cols * ((t + 1) * PT_BYTES + U * n * (PT_BYTES + zb)) / nblk, nblk
    if kernel == "combine":  # U affine piece values (128-B slots) in, P(j) out per (column, receiver)
        return 2 * n * n * (U * AFF_BYTES + PT_BYTES), 1
    if kernel == "check":  # s and s' (32 B each), b_j P(j) of the E and A columns (160 B each), 2 decisions,
        # and one 128-B comb entry per window of g and of h: the radix-2^19 tables (470 MB per base)
        # live in HBM beyond the Infinity Cache, so every window's entry is a read of the algorithm
        return n * n * (2 * 32 + 2 * PT_BYTES + 2 + 2 * combw_windows() * 128), 1
    if kernel == "affine":  # per stepped value: Z twice (the stepping's dense 40-B copy), the point, a
        # block prefix (48 B written and read per 4 points), the 128-B affine slot out
        return 2 * n * U * n * (2 * 40 + PT_BYTES + 2 * 12 + AFF_BYTES), 1
    return None, None


def pmc_traffic(kernel, n, t, U, plen=None, batch=1, mode="plain"):
    """HBM-side bytes per launch of `kernel` from the committed PMC passes (tools/profile.sh ->
    tools/pmc_summary.py --traffic, one file per workload in profiles/pmc_traffic/), when one was
    taken on this workload (n, t, split, piece length, batch, mode); else None."""
    want = {"n": n, "t": t, "split": U, "split_len": plen if plen is not None else split_pieces(t, U)[1],
            "batch": batch, "mode": mode}
    # DKG_PMC_TRAFFIC_DIR (a profile pass of the same GPU call, not yet committed) first, then the
    # committed files, newest round first (names start with the round tag)
    paths = []
    for d in [os.environ.get("DKG_PMC_TRAFFIC_DIR"), TRAFFIC_DIR]:
        try:
            paths += [os.path.join(d, x) for x in sorted(os.listdir(d), reverse=True) if x.endswith(".json")]
        except (OSError, TypeError):
            pass
    for path in paths:
        try:
            with open(path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        key = dict(doc.get("key", {}))
        if key.get("split_len") is None:
            key["split_len"] = split_pieces(t, U)[1]
        if key == want and kernel in doc.get("kernels", {}):
            k = doc["kernels"][kernel]
            return k["bytes_per_launch"], doc["source"], k.get("valu_int64_share"), k.get("effective_clock_mhz")
    return None


def add_traffic(line, dom, ms_pass, n, t, U, plen, per_wave=False, batch=1, mode="plain"):
    """roofline.algorithmic_bytes_per_launch / algorithmic_GBps / traffic (PMC) of the dominant kernel."""
    alg, launches = algorithmic_bytes(dom, n, t, U, plen, per_wave, batch)
    pmc = pmc_traffic(dom, n, t, U, plen, batch, mode)
    rl = line["roofline"]
    if alg is not None:
        rl["algorithmic_bytes_per_launch"] = alg
        rl["algorithmic_GBps"] = alg / (ms_pass / launches / 1e3) / 1e9
    if pmc is not None:
        rl["traffic"] = pmc[0]
        rl["traffic_unit"] = "HBM-side bytes per launch (average)"
        rl["traffic_source"] = pmc[1]
        rl["traffic_measured_on"] = (f"profile box ({pmc[1]}): PMC FETCH_SIZE/WRITE_SIZE passes of the same "
                                     "workload, not counters taken during this run")
        if alg:
            rl["traffic_over_algorithmic"] = pmc[0] / alg
        if pmc[2] is not None:
            # the counters' own lower bound on the slot fraction: every SQ_INSTS_VALU_INT64 instruction
            # is half rate (2 slots), the rest counted as full rate
            rl["valu_int64_share"] = pmc[2]
            rl["frac_counter_lower_bound"] = rl["instr_frac"] * (1 + pmc[2])
    # the clock the chip held during each kernel in the profiled pass (GRBM_GUI_ACTIVE / 8 / time,
    # MI355X_MICROARCH.md "DVFS give-back"): integer-VALU load is power-limited, so the 2.4-GHz peak
    # overstates what a kernel could issue; frac_at_profile_clock = frac x 2400 / that clock
    for name, k in [(dom, rl)] + list(rl.get("all_kernels", {}).items()):
        got = pmc_traffic(name, n, t, U, plen, batch, mode)
        if got is not None and got[3]:
            k["effective_clock_mhz_profile"] = round(got[3], 1)
            k["frac_at_profile_clock"] = k["frac"] * 2400.0 / got[3]


def spawn_ranks(args, poll_s=0.2):
    """`--gpus N` (N > 1) without a launcher: start N fresh worker processes of this script, one per
    GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (what torchrun sets),
    before this process touches the GPU; rank 0 prints the JSON line.  Every child is polled: the
    first one to exit non-zero ends the run -- its peers, blocked in a collective it will never
    join, are terminated (then killed) at once -- and its exit code is returned; 0 when all succeed."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    failed = 0
    while not failed and any(p.returncode is None for p in procs):
        time.sleep(poll_s)
        for r, p in enumerate(procs):
            if p.poll() not in (None, 0):
                failed = p.returncode
                print(f"bench.py: rank {r} exited with {failed}; stopping the other ranks", file=sys.stderr)
                break
    if failed:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(deadline - time.time(), 0.1))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        return failed if failed > 0 else 1
    return 0


def clock_fields(before, after):
    """The shader clock just before and just after the timed region (Backend.clock_probe: 4 waves per
    SIMD on every CU, s_memtime against s_memrealtime): boxes differ by several percent in clock,
    and the line says which clock its number was taken at."""
    return {"sclk_mhz": {"before": round(before["sclk_mhz"], 1), "after": round(after["sclk_mhz"], 1)},
            "sclk_probe": "median over 4 waves/SIMD x all CUs of s_memtime cycles per s_memrealtime us, "
                          f"{before['busy_ms']:.2f} ms probe launches outside the timed region"}


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def init_dist(args, local):
    """One process per GPU over RCCL ("nccl").  --dist-backend gloo is a rehearsal mode for boxes
    with fewer GPUs than ranks: ranks share GPUs (local % device_count) and the exchange is staged
    through host memory; its timings say nothing about xGMI.  A collective that waits longer than
    --dist-timeout seconds fails the rank instead of hanging it."""
    import datetime

    import torch
    import torch.distributed as dist

    timeout = datetime.timedelta(seconds=args.dist_timeout)
    if args.dist_backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
    else:
        dist.init_process_group("gloo", timeout=timeout)
    return dist


def fault_rehearsal(args, rank):
    """DKG_BENCH_FAIL_RANK=r (tests/test_bench_dist.py): rank r exits 1 right after the process group
    is up, the others enter a barrier it never joins -- the failure a crashed rank leaves behind.
    No GPU is touched, so the launcher's fail-fast path is testable on CPU."""
    bad = int(os.environ["DKG_BENCH_FAIL_RANK"])
    import datetime

    import torch.distributed as dist

    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.dist_timeout))
    if rank == bad:
        print(f"rank {rank}: injected failure", file=sys.stderr)
        sys.exit(1)
    dist.barrier()
    dist.destroy_process_group()


def gpu_index(args, local):
    import torch

    return local % torch.cuda.device_count() if args.dist_backend == "gloo" else local


def _naf(m):
    digits = []
    v = m
    while v:
        if v & 1:
            d = 2 - (v & 3)
            v -= d
        else:
            d = 0
        digits.append(d)
        v >>= 1
    return digits


def _wnaf(m, w):
    """Width-w non-adjacent form, least significant digit first (odd digits |d| < 2^(w-1))."""
    digits = []
    v = m
    while v:
        if v & 1:
            d = v & ((1 << w) - 1)
            if d >= 1 << (w - 1):
                d -= 1 << w
            v -= d
        else:
            d = 0
        digits.append(d)
        v >>= 1
    return digits


def split_pieces(t, U, plen=None):
    """Piece lengths of a U-way degree split with piece length plen (runtime.hip split_len:
    ceil((t+1)/U), or that rounded up to a multiple of 64; the last piece holds the rest)."""
    N = t + 1
    plen = plen or -(-N // U)
    last = N - (U - 1) * plen
    return [plen] * (U - 1) + [last if last > 0 else plen], plen  # runtime.hip last_piece_len


def affine_point_valu(VALU=SLOTS):
    """k_affine_pieces per stepped value: blocks of 4 points cost 31 fe_mul + 8 fe_add/fe_sub
    (counted as ~1/10 of a product each), one inversion (254 fe_sq + 11 fe_mul) per 32 points."""
    return (31 * VALU["fe_mul"] + 0.8 * VALU["fe_mul"]) / 4 + (254 * VALU["fe_sq"] + 11 * VALU["fe_mul"]) / 32


def short_combine_valu(mults, VALU=SLOTS, affine=True):
    """k_combine_short per (column, receiver row of `mults`): U cached addends (the first KL in LDS:
    ge_add, the rest in VGPRs: ge_add_signed), one joint chain over the U NAFs of the short vector.
    affine (k_combine_aff, the default addends): mixed additions (ge_madd_signed, LDS ones priced
    the same), no cached conversion, and k_affine_pieces' normalisation of the U addends."""
    total = 0
    for row in mults:
        U = len(row)
        KL = 1 if U == 2 else 2
        ds = [_naf(abs(v)) for v in row]
        top = max(len(d) for d in ds) - 1
        c = U * (affine_point_valu(VALU) if affine else VALU["ge_to_cached"])
        for i in range(top, -1, -1):
            nz = [u for u in range(U) if i < len(ds[u]) and ds[u][i] != 0]
            if i != top:
                c += VALU["ge_dbl_t"] if (nz or i == 0) else VALU["ge_dbl_not"]
            # the last addition of a position above 0 is followed by a doubling: no T
            for u in nz:
                wt = i == 0 or u != nz[-1]
                if affine:
                    c += add_cost(VALU, "ge_madd_signed", wt)
                else:
                    c += add_cost(VALU, "ge_add" if u < KL else "ge_add_signed", wt)
        total += c
    return total


def binom_digits(m):
    """The kernels' recoding of a binomial multiplier m (points.h small_recode): signed digits, least
    significant first, top digit +1 -- the NAF with a leading 1 0 -1 turned into 1 1."""
    ds = _naf(m)
    if len(ds) >= 3 and ds[-1] == 1 and ds[-2] == 0 and ds[-3] == -1:
        ds = ds[:-3] + [1, 1]
    return ds


def binom_item_valu(m, VALU=SLOTS, ded=True):
    """One binomial item e_m <- m (e_{m-1} + e_m) (kernels.hip k_binom_step / k_binom_wave): the first
    addition, then the NAF chain of m on the sum's cached form.  ded (the default with the dedicated
    stepping additions): the product-free cached forms, dedicated additions and a zero test of every
    addition's Z (fe_tight_zero); else the complete formula (cached form with the product by 2d)."""
    cached = VALU["ge_to_cached_ded"] if ded else VALU["ge_to_cached"]
    zt = VALU["fe_tight_zero"] if ded else 0
    c = cached + (VALU["ge_add_ded"] if ded else VALU["ge_add"]) + zt  # e_{m-1} + e_m
    ds = binom_digits(m)
    if len(ds) > 1:
        c += cached
        for i in range(len(ds) - 2, -1, -1):
            nz = ds[i] != 0
            c += VALU["ge_dbl_t"] if (nz or i == 0) else VALU["ge_dbl_not"]
            if nz:  # a doubling follows unless i = 0: no T (the dedicated signed form costs the same)
                c += add_cost(VALU, "ge_add_signed", i == 0) + zt
    return c


def algorithmic_valu(n, t, rnd=2, U=1, VALU=SLOTS, plen=None, mults=None, affine=True, ded=True):
    """Closed-form VALU work (issue slots, or instructions with VALU=INSTR) of one verification round
    over all n dealers as implemented (DESIGN.md "Work per unit"): binomial-basis Horner on U pieces
    (split_pieces: L coefficients each but a shorter last one), stepping, recombination by
    y_j = j^L (U > 1; with `mults`, the short multipliers of api.split_multipliers), fixed-base
    check (with `mults`, of b_j s: one more Montgomery product per scalar)."""
    pieces, L_ = split_pieces(t, U, plen)
    cost_m = {m: binom_item_valu(m, VALU, ded) for m in range(1, L_)}
    # position m of a piece of length Lp is live for Lp-m steps (a short last piece starts late)
    binom = sum(sum(cost_m[m] * (Lp - m) for m in range(1, Lp)) for Lp in pieces)
    # stepping: every lane converts each step; position p adds at step j (0..n-1) only while
    # p + j < n (k_stepping skips dead positions), so sum_j min(Lp - 1, n - j) additions
    def adds(Lp):
        m = min(Lp - 1, n)
        return m * (m + 1) // 2 + (n - m) * m
    # (ded: the dedicated addition + fe_tight_zero on its Z, and the product-free cached form; the
    # complete redo of marked workgroups does not occur on honest tables)
    cached, add = ((VALU["ge_to_cached_ded"], VALU["ge_add_ded"] + VALU["fe_tight_zero"]) if ded
                   else (VALU["ge_to_cached"], VALU["ge_add"]))
    stepping = sum(n * Lp * cached + adds(Lp) * add for Lp in pieces)
    combine = 0
    if U > 1 and mults is not None:
        combine = short_combine_valu(mults, VALU, affine)
    elif U > 1:  # k_combine: pairwise Horner in y^2 with joint NAF chains (kernels.hip)
        for j in range(1, n + 1):
            y = pow(j, L_, L)
            d1, d2 = _naf(y), _naf(y * y % L)
            c = 0
            if U % 2 == 0:  # top pair: y Q + Q'
                c += 2 * VALU["ge_to_cached"] + VALU["ge_add"]
                for i in range(len(d1) - 2, -1, -1):
                    nz = d1[i] != 0
                    c += VALU["ge_dbl_t"] if (nz or i == 0) else VALU["ge_dbl_not"]
                    if nz:
                        c += add_cost(VALU, "ge_add_signed", i == 0)
            joint = 3 * VALU["ge_to_cached"] + VALU["ge_add"]  # two addends, Q_2v, + Q_2v
            for i in range(max(len(d1), len(d2)) - 1, -1, -1):
                e1 = d1[i] if i < len(d1) else 0
                e2 = d2[i] if i < len(d2) else 0
                joint += VALU["ge_dbl_t"] if (e1 or e2 or i == 0) else VALU["ge_dbl_not"]
                if e2:
                    joint += add_cost(VALU, "ge_add_signed", e1 != 0 or i == 0)
                if e1:
                    joint += add_cost(VALU, "ge_add_signed", i == 0)
            c += ((U + 1) // 2 - 1) * joint
            combine += c
    nsc = 2 if rnd == 2 else 1
    scale = nsc * VALU["sc_mont_mul"] if mults is not None else 0
    check = n * (nsc * combw_windows() * VALU["combw_window"] + VALU["eq"] + scale)
    return {"binomial": binom * n, "stepping": stepping * n, "combine": combine * n, "check": check * n}


def fused_valu(n, t, U=1, VALU=SLOTS, plen=None, mults=None, affine=True, ded=True):
    """Work of the fused round-2 + round-4 pipeline: both tables' binomial, stepping and
    recombination; one check kernel computing g*s once (24 radix-2^11 comb windows), h*s' (24 more)
    and both equalities per pair (with `mults`: s and s' scaled by b_j first)."""
    w2 = algorithmic_valu(n, t, 2, U, VALU, plen, mults, affine, ded)
    w4 = algorithmic_valu(n, t, 4, U, VALU, plen, mults, affine, ded)
    out = {k: w2[k] + w4[k] for k in ("binomial", "stepping", "combine")}
    scale = 2 * VALU["sc_mont_mul"] if mults is not None else 0
    out["check"] = n * n * (2 * combw_windows() * VALU["combw_window"] + 2 * VALU["eq"] + scale)
    return out


def host_cpu():
    """(threads to use, description): every core of this process's affinity mask, capped by a cgroup
    CPU quota when one is set (a GPU box grants a share of a larger machine), and the CPU model."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cores = min(aff, quota) if quota else aff
    return cores, {"cpu_model": model, "affinity_cores": aff, "cgroup_quota_cores": quota,
                   "os_cpu_count": os.cpu_count()}


def cpu_baseline(n, t, seconds_target=20.0, ceremonies=1):
    """Reference-algorithm CPU baseline of the WHOLE ceremony, extrapolated from a bounded sample.
    The oracle follows dalek-3's u64 algorithms (5x51 field, radix-16 variable-base mul, Straus /
    Pippenger MSM at dalek's thresholds) loop for loop with committee.rs.  On blocks of dealers
    (8 up to n = 1024, 2 above: a block of n = 4096 dealers is 2 x 8190 MSMs of 2048 points) it times
    round-1 share generation (commitments + all n shares, committee.rs:148-186), round-2 checks
    (:287-305) and round-4 checks (:532-548) against all receivers on every host core, until about
    `seconds_target` seconds, moving on to the next ceremony (other seeds) when one is complete
    (small n, config 5); the ceremony time is n x (share gen per dealer) + n(n-1) x (round-2 +
    round-4 per pair) -- rounds 3 and 5 are negligible -- and value = n(n-1) / that time (the same
    rate in verified shares/s for `ceremonies` independent ceremonies)."""
    import ctypes

    from tests import oracle_lib as O
    import dkg_amd

    cores, cpu = host_cpu()
    lib = O.lib()
    lib.or_bench_fe_mul.restype = ctypes.c_double
    lib.or_bench_fe_mul.argtypes = [ctypes.c_uint64]
    lib.or_bench_msm.restype = ctypes.c_double
    lib.or_bench_msm.argtypes = [ctypes.c_size_t, ctypes.c_int]
    fe_ns = lib.or_bench_fe_mul(5_000_000)
    msm_ms = lib.or_bench_msm(t + 1, 3)
    master = b"\x05" * 32
    nd = min(n, 8 if n <= 1024 else 2)
    h = O.call32("or_pt_hash_to_group", b"Example of a shared string.", 27)[0]
    t_gen = t_r2 = t_r4 = 0.0
    dealers = pairs = 0
    cer = d0 = 0
    warm = False
    while t_gen + t_r2 + t_r4 < seconds_target:
        if d0 + nd > n:  # this ceremony is complete: the next one
            if n > 1024:
                break
            cer, d0 = cer + 1, 0
        a, b = dkg_amd.dealer_coefficients(master, cer, d0, nd, t)
        t0 = time.perf_counter()
        E, A, s, sp = O.share_gen(nd, n, t, a, b, h, cores)
        t_gen += time.perf_counter() - t0
        # rows of the sampled dealers at their own indices (the diagonal stays global)
        if not warm:
            O.verify_rows(n, t, 2, E, h, s, sp, d0, d0 + nd, 0, 1, cores)  # warm the thread pool
            warm = True
        t0 = time.perf_counter()
        acc2, _ = O.verify_rows(n, t, 2, E, h, s, sp, d0, d0 + nd, 0, n, cores)
        t_r2 += time.perf_counter() - t0
        t0 = time.perf_counter()
        acc4, _ = O.verify_rows(n, t, 4, A, h, s, None, d0, d0 + nd, 0, n, cores)
        t_r4 += time.perf_counter() - t0
        assert set(acc2) <= {1, 2} and set(acc4) <= {1, 2}
        dealers += nd
        d0 += nd
        pairs += sum(1 for x in acc2 if x == 1)
    gen_per_dealer, r2_per_pair, r4_per_pair = t_gen / dealers, t_r2 / pairs, t_r4 / pairs
    ceremony_s = n * gen_per_dealer + n * (n - 1) * (r2_per_pair + r4_per_pair)
    what = (f"{dealers // n} whole ceremonies + {dealers % n} dealers" if dealers >= n
            else f"{dealers} dealers x all {n} receivers")
    return {"value": n * (n - 1) / ceremony_s, "unit": "verified shares/s", "cores": cores, "kind": "port",
            "ceremony_s_extrapolated": ceremony_s, "batch_s_extrapolated": ceremony_s * ceremonies,
            "round1_ms_per_dealer": gen_per_dealer * 1e3, "round2_ms_per_pair": r2_per_pair * 1e3,
            "round4_ms_per_pair": r4_per_pair * 1e3,
            "fe_mul_ns_1thread": fe_ns, f"msm_N{t + 1}_ms_1thread": msm_ms, **cpu,
            "sample": f"{what} at n={n}, t={t} ({pairs} pairs): share generation, round-2 and round-4 checks "
                      f"(vartime MSM over t+1={t + 1} points per pair, dalek-3's algorithms) timed on {cores} "
                      f"threads in {t_gen + t_r2 + t_r4:.1f} s; time of {ceremonies} ceremon"
                      f"{'ies' if ceremonies > 1 else 'y'} extrapolated linearly in dealers and pairs"}


def bench_batch(args, ws, rank, local):
    """BASELINE config 5: B independent ceremonies per step (replicas only: with N GPUs each rank
    runs its own B ceremonies, no collective -- weak scaling).  Coefficients are generated on the
    GPU (dkg_dealer_coeffs_device) and stay in HBM; one step = rounds 1-5 of all B ceremonies."""
    import torch

    import dkg_amd

    B, n, t = BATCH[args.config]
    N = t + 1
    local = gpu_index(args, local)
    torch.cuda.set_device(local)
    dist = init_dist(args, local) if ws > 1 else None
    be = dkg_amd.Backend(local)
    be.set_streams(args.streams)
    be.set_overlap(not args.no_overlap)
    be.set_verify_mode(args.verify)
    be.set_binomial(args.binomial)
    be.set_check(args.check)
    be.set_stepping(args.stepping)
    be.env_init(t, n)
    dev = torch.device("cuda", local)
    ta = torch.empty(B * n * N * 32, dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    be.dealer_coefficients_device(b"\xb5" * 32, rank * B, B, 0, n, t, ta.data_ptr(), tb.data_ptr())

    def step():
        return dkg_amd.ceremony_batch_device(be, B, n, t, ta.data_ptr(), tb.data_ptr())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    clk0 = be.clock_probe()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    clk1 = be.clock_probe()
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    assert all(q == n for q in res.n_qualified), "an honest ceremony disqualified a dealer"
    # per-kernel device times: one extra serialised batch (one chunk stream)
    be.set_streams(1)
    step()
    torch.cuda.synchronize()
    be.set_streams(args.streams)
    ph = be.phase_times("r24")
    U, Ls = be.last_split(), be.last_split_len()
    mults = dkg_amd.split_multipliers(n, Ls, U) if be.last_combine() == 2 else None
    work = {k: v * B for k, v in fused_valu(n, t, U, plen=Ls, mults=mults).items()}
    work_i = {k: v * B for k, v in fused_valu(n, t, U, INSTR, Ls, mults).items()}
    rl = kernel_rooflines(ph, work, work_i)
    pairs = B * n * (n - 1) * ws  # whole node: every rank runs its own B ceremonies
    out = {"metric": f"verified shares/sec (whole node) of {B} independent n={n},t={t} ceremonies per GPU "
                     f"x {ws} GPU(s) (BASELINE config 5)",
           "value": pairs * args.steps / elapsed, "unit": "verified shares/s", "n_gpus": ws, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u32 (GF(2^255-19), Z_l)",
           "data": "synthetic: seeded ChaCha20 coefficients generated on the GPU, honest ceremonies",
           "config": {"workload": f"{B} ceremonies n={n}, t={t} per GPU (share gen + round-2/4 checks + "
                                  f"finalise of each)", "ceremonies_per_gpu": B, "n": n, "t": t,
                      "pairs_per_step": pairs, "parallelism": f"replicas x{ws}" if ws > 1 else "single GPU"},
           "ceremonies_per_s": B * ws * args.steps / elapsed,
           "phases_ms": {k: round(v, 3) for k, v in res.ms.items()}}
    out["config"]["degree_split"] = U
    out["ref_equiv"] = ref_equiv(n, t, out["value"])
    out.update(clock_fields(clk0, clk1))
    out["config"]["binomial"] = "per-wave loops" if be.last_binomial() else "one launch per step"
    if rl:
        dom = max(rl, key=lambda k: rl[k]["ms_per_pass"])
        out["roofline"] = roofline_line(rl, dom, f"{work[dom]:.4g} VALU issue slots ({work_i[dom]:.4g} instructions) "
                                                 f"per batch: {B} x the closed form of one ceremony's fused "
                                                 f"round-2/4 pipeline; device time in a serialised batch")
        add_traffic(out, dom, rl[dom]["ms_per_pass"], n, t, U, Ls, bool(be.last_binomial()), B)
    if rank == 0 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(n, t, 20.0, ceremonies=B)
        out["gpu_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    if rank == 0:
        emit(out)
    be.close()
    if dist:
        dist.destroy_process_group()


def sharded_self_check(args, dist, be, res, ta, D, N, dev):
    """N > 1: the honest sharded ceremony must qualify everyone with no round errors, and the mpk
    every rank derived (sum of the gathered A_i0, dkg_shard_finalise_device) must equal g * sum_i a_i0
    -- each rank sums its dealers' constant terms mod l, the partial sums are all-gathered, and the
    total goes through the fixed-base path (a different computation from the commitments').  Returns
    the per-rank spread of the last timed step: shard device ms and the exchange / combine /
    reconstruction / finalise host ms (min and max over ranks)."""
    import torch

    d = res.decisions
    assert d.qualified.all(), "an honest sharded ceremony disqualified a dealer"
    assert not d.r2_error.any() and not d.r4_error.any() and not d.phase4_error, "round error in an honest ceremony"
    xdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    own = ta[:D * N * 32].view(D, N, 32)[:, 0, :].cpu().numpy() if D else []
    part = sum(int.from_bytes(bytes(r), "little") for r in own) % L
    mine = torch.frombuffer(bytearray(part.to_bytes(32, "little")), dtype=torch.uint8).to(xdev)
    allp = torch.empty(32 * dist.get_world_size(), dtype=torch.uint8, device=xdev)
    dist.all_gather_into_tensor(allp, mine)
    raw = bytes(allp.cpu().numpy())
    secret = sum(int.from_bytes(raw[32 * r:32 * r + 32], "little") for r in range(dist.get_world_size())) % L
    expect = be.fixed_base_batch(secret.to_bytes(32, "little"))
    assert res.mpk == expect, "sharded mpk != g * sum of the dealers' a_i0"
    # which device each rank ran on: the N > 1 line must show N distinct GPUs under RCCL (under the
    # gloo rehearsal ranks share one GPU and the count is 1)
    bus = be.pci_bus_id().encode()[:31].ljust(32, b"\0")
    mine = torch.frombuffer(bytearray(bus), dtype=torch.uint8).to(xdev)
    allb = torch.empty(32 * dist.get_world_size(), dtype=torch.uint8, device=xdev)
    dist.all_gather_into_tensor(allb, mine)
    rawb = bytes(allb.cpu().numpy())
    rank_devices = [rawb[32 * r:32 * r + 32].rstrip(b"\0").decode() for r in range(dist.get_world_size())]
    distinct = len(set(rank_devices))
    if args.dist_backend == "nccl" and distinct != dist.get_world_size():
        raise SystemExit(f"RCCL ranks share devices: {rank_devices}")
    keys = ["shard_device", "exchange", "combine", "recon", "finalise"]
    vals = [res.ms_shard] + [res.ms_steps.get(k, 0.0) for k in keys[1:]]
    mine = torch.tensor(vals, dtype=torch.float64, device=xdev)
    allv = torch.empty(len(vals) * dist.get_world_size(), dtype=torch.float64, device=xdev)
    dist.all_gather_into_tensor(allv, mine)
    per = allv.cpu().view(-1, len(vals)).tolist()
    return {"mpk_check": "mpk == g * sum_i a_i0 (partial sums all-gathered)",
            "rank_devices": rank_devices, "distinct_devices": distinct,
            "dist": {"backend": args.dist_backend, "world_size": dist.get_world_size()},
            "rank_ms": {k: {"min": round(min(r[i] for r in per), 3), "max": round(max(r[i] for r in per), 3)}
                        for i, k in enumerate(keys)},
            "rank_ms_note": "last timed step; shard_device = HIP-event time of the rank's share gen + checks, the "
                            "rest host wall time of the steps after it (all-gathers fenced, combine, round-4 "
                            "reconstruction, finalise)"}


_RESULT_OUT = None


def keep_stdout_for_result():
    """The result line must be the only line on stdout: RCCL's banner, the gloo backend and native
    libraries write to fd 1.  Keep a private copy of stdout for emit() and point fd 1 (and Python's
    sys.stdout) at stderr for everything else."""
    global _RESULT_OUT
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def emit(out):
    f = _RESULT_OUT or sys.stdout
    f.write(json.dumps(out) + "\n")
    f.flush()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="D", choices=sorted(CONFIGS) + sorted(BATCH))
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-interp", action="store_true",
                    help="skip the side measurement of the opt-in interpolation verify mode")
    ap.add_argument("--streams", type=int, default=2, help="dealer-chunk streams of the round-2/4 checks")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo = rehearsal with ranks sharing GPUs")
    ap.add_argument("--dist-timeout", type=float, default=180.0,
                    help="seconds a collective may wait for its peers before the rank fails")
    ap.add_argument("--verify", default="group", choices=["group", "interp"],
                    help="group: every P_i(j) computed in the group (default); interp: committee verification "
                         "by interpolation (identical decisions, DESIGN.md section 2)")
    ap.add_argument("--split", type=int, default=0, help="degree split U of the difference tables (0: cost model)")
    ap.add_argument("--combine", type=int, default=0,
                    help="recombination of a degree split: 0 short lattice multipliers (U <= 4), 1 powers of j^L")
    ap.add_argument("--step-formula", type=int, default=0, choices=[0, 1],
                    help="stepping additions: 0 dedicated (complete redo where exceptional), 1 complete")
    ap.add_argument("--addends", type=int, default=0, choices=[0, 1],
                    help="short-multiplier recombination addends: 0 affine Niels, 1 cached projective")
    ap.add_argument("--field", type=int, default=0,
                    help="field multiply of the checks: 0 per launch by occupancy, 1 product scanning, 2 column sums")
    ap.add_argument("--binomial", type=int, default=0, choices=[0, 1, 2, 3, 4, 5],
                    help="binomial schedule (dkg_ctx_set_binomial): 0 default (per-wave Horner loops for tables of many column groups, else per step with lane pairs for the latency-bound steps), 1 per step without lane pairs, 2 per step with lane pairs for every step, 3 per step as 0, 4 per wave always, 5 per wave with operands prefetched one item ahead")
    ap.add_argument("--check", type=int, default=0, choices=[0, 1],
                    help="fused checks (dkg_ctx_set_check): 0 one launch, 1 one launch per fixed-base comb")
    ap.add_argument("--stepping", type=int, default=0, choices=[0, 1, 2, 3],
                    help="stepping slots (dkg_ctx_set_stepping): 0 cost model, 1 per column, 2 per piece, 3 no dead-position repack")
    ap.add_argument("--no-overlap", action="store_true", help="verify round 4 after round 3 (protocol order) instead of fused with round 2")
    ap.add_argument("--mode", default="plain", choices=["plain", "full"],
                    help="plain: shares in the clear (headline); full: hybrid-encrypted shares (SURVEY 8 f1)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    keep_stdout_for_result()
    ws, rank, local = dist_env()
    if ws != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={ws} ranks")
    if "DKG_BENCH_FAIL_RANK" in os.environ:
        return fault_rehearsal(args, rank)
    if args.config in BATCH:
        return bench_batch(args, ws, rank, local)
    n, t = CONFIGS[args.config]

    import torch

    local = gpu_index(args, local)
    torch.cuda.set_device(local)
    import dkg_amd

    dist = init_dist(args, local) if ws > 1 else None
    be = dkg_amd.Backend(local)
    be.set_streams(args.streams)
    be.set_overlap(not args.no_overlap)
    be.set_split(args.split)
    be.set_field_mode(args.field)
    be.set_combine(args.combine)
    be.set_addends(args.addends)
    be.set_stepping_formula(args.step_formula)
    be.set_binomial(args.binomial)
    be.set_check(args.check)
    be.set_stepping(args.stepping)
    be.set_verify_mode(args.verify)
    h = be.env_init(t, n)
    N = t + 1
    master = b"\xbe" * 32
    d0, d1 = (rank * n) // ws, ((rank + 1) * n) // ws
    D = d1 - d0
    dev = torch.device("cuda", local)
    # seeded coefficients generated on the GPU (bit-identical to dkg_amd.dealer_coefficients)
    ta = torch.empty(max(D * N * 32, 32), dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    be.dealer_coefficients_device(master, 0, 1, d0, D, t, ta.data_ptr(), tb.data_ptr())
    torch.cuda.synchronize()

    if ws == 1 and args.mode == "full":
        tr = torch.empty(64 * n * n, dtype=torch.uint8, device=dev)
        be.enc_randomness_device(master, 0, 1, 0, n, n, t, tr.data_ptr())
        msk, mpk = be.member_keys(master, 0, n)

        def step():
            return be.ceremony_full_device(ta.data_ptr(), tb.data_ptr(), tr.data_ptr(), msk, mpk, n, t)
    elif ws == 1:
        def step():
            return be.ceremony_device(ta.data_ptr(), tb.data_ptr(), n, t)
    else:
        from dkg_amd.distributed import ShardedCeremony

        sc = ShardedCeremony(be, dist, n, t, dev)

        def step():
            # shard (share gen + checks of this rank's dealers), RCCL all-gathers, combine, round-3
            # final shares and mpk on the GPU (dkg_amd/distributed.py)
            return sc.run(ta.data_ptr(), tb.data_ptr())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    clk0 = be.clock_probe()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    clk1 = be.clock_probe()
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    if ws == 1:  # an honest ceremony: every dealer qualifies
        assert res.n_qualified == n, "an honest ceremony disqualified a dealer"
    shard_stats = None
    if ws > 1:
        shard_stats = sharded_self_check(args, dist, be, res, ta, D, N, dev)
    pairs = n * (n - 1)
    value = pairs * args.steps / elapsed
    metric = f"verified shares/sec (whole node) at n={n},t={t}; full-ceremony wall time"
    if args.mode == "full":
        metric += " -- FULL mode (hybrid-encrypted shares, SURVEY 8 f1)"
    out = {
        "metric": metric,
        "value": value, "unit": "verified shares/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32 (GF(2^255-19), Z_l)",
        "data": "synthetic: seeded ChaCha20 coefficients (SURVEY.md 8d), honest ceremony",
        "config": {"workload": f"one DKG ceremony n={n}, t={t} (share gen + round-2/4 checks + finalise)",
                   "n": n, "t": t, "pairs_per_step": pairs,
                   "parallelism": f"dealer-sharded x{ws}" if ws > 1 else "single GPU"},
    }
    out["ref_equiv"] = ref_equiv(n, t, value)
    out.update(clock_fields(clk0, clk1))
    if args.mode == "full":
        out["config"]["mode"] = "full: shares hybrid-encrypted (elgamal.rs) and decrypted by each receiver"
    if rank == 0 and ws == 1 and res is not None and args.mode == "full":
        out["phases_ms"] = {k: round(v, 3) for k, v in res.ms.items()}
        # per-kernel roofline of the whole full-mode ceremony: one serialised extra ceremony
        be.set_streams(1)
        step()
        torch.cuda.synchronize()
        be.set_streams(args.streams)
        ph = dict(be.phase_times("r24"))
        ph.update(be.phase_times("full"))
        U, Ls = be.last_split(), be.last_split_len()
        mults = dkg_amd.split_multipliers(n, Ls, U) if be.last_combine() == 2 else None
        work = fused_valu(n, t, U, plen=Ls, mults=mults)
        work_i = fused_valu(n, t, U, INSTR, Ls, mults)
        work.update(hybrid_valu(n, msk))
        work_i.update(hybrid_valu(n, msk, INSTR))
        rl = kernel_rooflines(ph, work, work_i)
        dom = max(rl, key=lambda k: rl[k]["ms_per_pass"])
        out["roofline"] = roofline_line(rl, dom, f"{work[dom]:.4g} VALU issue slots ({work_i[dom]:.4g} instructions) "
                                                 f"per full-mode ceremony (closed form; hybrid kernels: "
                                                 f"bench.py hybrid_valu); device time in a serialised ceremony")
        add_traffic(out, dom, rl[dom]["ms_per_pass"], n, t, U, Ls, bool(be.last_binomial()), 1, "full")
        if not args.no_cpu:
            cb = cpu_baseline(n, t)
            lib = __import__("tests.oracle_lib", fromlist=["lib"]).lib()
            lib.or_bench_hybrid.restype = ctypes.c_double
            lib.or_bench_hybrid.argtypes = [ctypes.c_size_t, ctypes.c_int]
            items = 2 * n * n
            sample = 40000
            per_item = lib.or_bench_hybrid(sample, cb["cores"])
            assert per_item > 0, "oracle hybrid round trip failed"
            full_s = cb["ceremony_s_extrapolated"] + items * per_item
            cb.update({"value": n * (n - 1) / full_s, "ceremony_s_extrapolated": full_s,
                       "hybrid_us_per_item": per_item * 1e6,
                       "sample": cb["sample"] + f"; plus hybrid encryption + decryption of {sample} sampled "
                                                f"items (elgamal.rs:134-193), extrapolated to all {items}"})
            out["cpu_baseline"] = cb
            out["gpu_vs_cpu"] = value / cb["value"]
    if args.verify == "interp":
        out["metric"] += " -- committee verification by interpolation (identical decisions)"
        out["config"]["verify"] = ("interp: shares at receivers 1..t+1 fix F, F'; commitments tested once; "
                                   "remaining pairs by scalar comparison (DESIGN.md section 2)")
    if rank == 0 and ws == 1 and res is not None and args.verify == "interp" and args.mode != "full":
        out["phases_ms"] = {k: round(v, 3) for k, v in res.ms.items()}
        out["verify_phases_ms"] = {k: round(v, 3) for k, v in be.phase_times("interp").items()}
        out["fallback_rows"] = be.fallback_rows()
    elif rank == 0 and ws == 1 and res is not None and args.mode != "full":
        out["phases_ms"] = {k: round(v, 3) for k, v in res.ms.items()}
        out["config"]["verify_streams"] = args.streams
        out["config"]["rounds_2_4_fused"] = not args.no_overlap
        ov = not args.no_overlap
        U, Ls = be.last_split(), be.last_split_len()
        mults = dkg_amd.split_multipliers(n, Ls, U) if be.last_combine() == 2 else None
        out["config"]["degree_split"] = U
        out["config"]["split_pieces"] = split_pieces(t, U, Ls)[0]
        out["config"]["recombination"] = {0: "none", 1: "powers of j^L", 2: "short lattice multipliers"}[be.last_combine()]
        aff, ded = args.addends == 0, args.step_formula == 0
        out["config"]["recombination_addends"] = "affine Niels" if aff else "cached projective"
        out["config"]["stepping_additions"] = "dedicated (complete redo where exceptional)" if ded else "complete"
        out["stepping_redos"] = be.stepping_redos()
        w2 = algorithmic_valu(n, t, 2, U, plen=Ls, mults=mults, affine=aff, ded=ded)
        w4 = algorithmic_valu(n, t, 4, U, plen=Ls, mults=mults, affine=aff, ded=ded)
        work = fused_valu(n, t, U, plen=Ls, mults=mults, affine=aff, ded=ded) if ov else w2
        work_i = (fused_valu(n, t, U, INSTR, Ls, mults, aff, ded) if ov
                  else algorithmic_valu(n, t, 2, U, INSTR, Ls, mults, aff, ded))
        # per-kernel device times need the serialised schedule (one chunk stream): one extra,
        # untimed ceremony in the same round order as the timed ones
        be.set_streams(1)
        ser = step()
        torch.cuda.synchronize()
        be.set_streams(args.streams)
        ph = be.phase_times("r24" if ov else "r2")
        out["checks_serialised_ms"] = round(ser.ms["round2"], 3)
        # VALU efficiency of all checks: closed-form work of rounds 2 and 4 (as scheduled) over the
        # timed ceremony's rounds 2-4 wall time
        vms = res.ms["round2"] + res.ms["round3"] + res.ms["round4"]
        wall = work if ov else {k: w2[k] + w4[k] for k in w2}
        out["checks_valu_frac"] = sum(wall.values()) / (vms / 1e3) / INT32_PEAK
        rl = kernel_rooflines(ph, work, work_i)
        dom = max(rl, key=lambda k: rl[k]["ms_per_pass"]) if rl else None
        if dom:
            what = "rounds 2+4 (fused pipeline)" if ov else "round 2"
            out["roofline"] = roofline_line(rl, dom, f"{work[dom]:.4g} VALU issue slots ({work_i[dom]:.4g} "
                                            f"instructions) per pass over {what} (closed form); device time of "
                                            f"the kernel's launches (HIP events) in a serialised pass")
            if ov:
                add_traffic(out, dom, rl[dom]["ms_per_pass"], n, t, U, Ls, bool(be.last_binomial()))
        if not args.no_interp:
            # the opt-in committee verification on the same inputs, reported
            # beside the headline, never as it: every P_i(j) is NOT computed in the group there
            be.set_verify_mode("interp")
            step()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                ri = step()
            torch.cuda.synchronize()
            ms_i = (time.perf_counter() - t1) / args.steps * 1e3
            be.set_verify_mode("group")
            assert ri.n_qualified == n and ri.mpk == res.mpk, "interpolation mode disagrees with the group mode"
            out["interp_mode"] = {"ms_per_step": ms_i, "value": pairs / (ms_i / 1e3), "unit": "verified shares/s",
                                  "note": "opt-in dkg_ctx_set_verify_mode(ctx, 1): committee verification by "
                                          "interpolation, identical decisions; not the headline"}
        if not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(n, t)
            out["gpu_vs_cpu"] = value / out["cpu_baseline"]["value"]
    if shard_stats is not None:
        out.update(shard_stats)
        # the all-gathered decisions are packed bitmaps (dkg_decisions_pack_device): bytes one rank
        # contributes per ceremony, against the n-byte rows, here and at BASELINE config 4
        R4, W4 = dkg_amd.shard_rows(4096, 8), dkg_amd.packed_row_words(4096)
        out["exchange"] = {"decisions": "packed bitmaps" if sc.packed else "bytes",
                           "bytes_per_rank": sc.exchange_bytes(),
                           "bytes_per_rank_byte_rows": 2 * sc.R * n + sc.A0.numel() + sc.part.numel(),
                           "n4096_ws8_bytes_per_rank": 2 * R4 * 4 * W4 + 32 * R4 + 32 * 4096,
                           "n4096_ws8_bytes_per_rank_byte_rows": 2 * R4 * 4096 + 32 * R4 + 32 * 4096}
    if ws > 1 and args.mode != "full" and args.verify == "group":
        # per-GPU roofline of this rank's shard: one extra serialised pass (every rank joins its
        # collectives); the rank's work is its D dealers' share of the closed form
        be.set_streams(1)
        sc.run(ta.data_ptr(), tb.data_ptr())
        torch.cuda.synchronize()
        be.set_streams(args.streams)
        ph = be.phase_times("r24" if not args.no_overlap else "r2")
        U, Ls = be.last_split(), be.last_split_len()
        mults = dkg_amd.split_multipliers(n, Ls, U) if be.last_combine() == 2 else None
        D = ((rank + 1) * n) // ws - (rank * n) // ws
        aff, ded = args.addends == 0, args.step_formula == 0
        work = {k: v * D / n for k, v in fused_valu(n, t, U, plen=Ls, mults=mults, affine=aff, ded=ded).items()}
        work_i = {k: v * D / n for k, v in fused_valu(n, t, U, INSTR, Ls, mults, aff, ded).items()}
        rl = kernel_rooflines(ph, work, work_i)
        out["config"]["degree_split"] = U
        if rl:
            dom = max(rl, key=lambda k: rl[k]["ms_per_pass"])
            out["roofline"] = roofline_line(rl, dom, f"rank 0's shard ({D} dealers): {work[dom]:.4g} VALU issue "
                                                     f"slots per pass (closed form); device time in a serialised pass")
            # the counters' lower bound needs the kernel's INT64 share, a per-lane instruction mix that
            # does not depend on the dealer count: the one-GPU profile of the same (n, t, U, L) gives it
            # (its byte count does depend on D, so `traffic` stays unmeasured here)
            pmc = pmc_traffic(dom, n, t, U, Ls)
            if pmc is not None and pmc[2] is not None:
                r = out["roofline"]
                r["valu_int64_share"] = pmc[2]
                r["valu_int64_share_source"] = (pmc[1] + " -- the same kernel at the one-GPU workload "
                                                "(n, t, U, L); the instruction mix per lane is independent of D")
                r["frac_counter_lower_bound"] = r["instr_frac"] * (1 + pmc[2])
    if rank == 0:
        emit(out)
    be.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
