#!/usr/bin/env python3
"""Static VALU instruction count of each group/field primitive as compiled for gfx950.

Compiles tiny kernels that loop over one primitive and counts the VALU instructions of the hottest
basic block in the ISA.  bench.py's roofline multiplies these counts by the closed-form number of
primitive calls of the implemented schedule (the "algorithmic" work: no PMC, no guesswork).
Usage: python tools/count_valu.py  (prints a JSON dict; copy into bench.py VALU_PER_OP).
"""
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRIMS = {
    "fe_mul": ("fe a, b; LD10(a.v, 0); LD10(b.v, 640);", "fe_mul(a, a, b);", "ST10(a.v);"),
    "fe_sq": ("fe a; LD10(a.v, 0);", "fe_sq(a, a);", "ST10(a.v);"),
    "ge_add": ("ge_p3 p; ge_cached q; LDP(p, 0); LDP(q, 2560);", "ge_add(p, p, q);", "STP(p);"),
    "ge_add_signed": ("ge_p3 p; ge_cached q; LDP(p, 0); LDP(q, 2560); bool ng = o[9999] & 1;",
                      "ge_add_signed(p, p, q, ng); ng = !ng;", "STP(p);"),
    "ge_dbl_t": ("ge_p3 p; LDP(p, 0);", "ge_dbl_rt(p, p, true);", "STP(p);"),
    "ge_dbl_not": ("ge_p3 p; LDP(p, 0);", "ge_dbl_rt(p, p, false);", "STP(p);"),
    "ge_add_ded": ("ge_p3 p; LDP(p, 0);", "ge_add_ded_lds(p, p, o + 2560 + threadIdx.x, 64);", "STP(p);"),
    "ge_to_cached_ded": ("ge_p3 p; ge_cached q; LDP(p, 0);",
                         "ge_to_cached_ded(q, p); p.X = q.T2d; p.Y = q.YpX; p.Z = q.Z2; p.T = q.YmX;",
                         "STP(p);"),
    "fe_tight_zero": ("fe a; LD10(a.v, 0); uint32_t acc = 0;", "acc += fe_tight_zero(a) ? 1u : 0u; a.v[0] ^= acc;",
                      "ST10(a.v);"),
    "ge_madd_signed": ("ge_p3 p; ge_aff q; LDP(p, 0); LD10(q.ypx.v, 3000); LD10(q.ymx.v, 3640); LD10(q.xy2d.v, 4280); "
                       "bool ng = o[9999] & 1;", "ge_madd_signed(p, p, q, ng); ng = !ng;", "STP(p);"),
    "ge_madd_signed_not": ("ge_p3 p; ge_aff q; LDP(p, 0); LD10(q.ypx.v, 3000); LD10(q.ymx.v, 3640); "
                           "LD10(q.xy2d.v, 4280); bool ng = o[9999] & 1;",
                           "ge_madd_signed(p, p, q, ng, false); ng = !ng; p.T.v[0] ^= ng;", "STP(p);"),
    "ge_add_signed_not": ("ge_p3 p; ge_cached q; LDP(p, 0); LDP(q, 2560); bool ng = o[9999] & 1;",
                          "ge_add_signed(p, p, q, ng, false); ng = !ng; p.T.v[0] ^= ng;", "STP(p);"),
    "ge_madd": ("ge_p3 p; ge_aff q; LDP(p, 0); LD10(q.ypx.v, 3000); LD10(q.ymx.v, 3640); LD10(q.xy2d.v, 4280);",
                "ge_madd(p, p, q);", "STP(p);"),
    "comb_window": ("ge_p3 p; LDP(p, 0); sc x; for (int i_ = 0; i_ < 8; i_++) x.v[i_] = o[9000 + i_];",
                    "comb_mul_add(p, x, o + 20000); x.v[0] ^= p.X.v[0];", "STP(p);"),
    "combw_window": ("ge_p3 p; LDP(p, 0); sc x; for (int i_ = 0; i_ < 8; i_++) x.v[i_] = o[9000 + i_];",
                     "combw_mul_add(p, x, o + 20000); x.v[0] ^= p.X.v[0];", "STP(p);"),
    "eq": ("ge_p3 p, q; LDP(p, 0); LDP(q, 2560);", "if (ristretto_eq(p, q)) p.X.v[0] ^= 1; else q.Y.v[1] ^= 3;",
           "STP(p); STP(q);"),
    "sc_mont_mul": ("sc x, f; for (int i_ = 0; i_ < 8; i_++) { x.v[i_] = o[9000 + i_ * 64 + threadIdx.x]; "
                    "f.v[i_] = o[9600 + i_ * 64 + threadIdx.x]; }",
                    "sc_mont_mul(x, x, f);", "for (int i_ = 0; i_ < 8; i_++) o[i_ * 64 + threadIdx.x] = x.v[i_];"),
    "ge_to_cached": ("ge_p3 p; ge_cached q; LDP(p, 0);",
                     "ge_to_cached(q, p); p.X = q.T2d; p.Y = q.YpX; p.Z = q.Z2; p.T = q.YmX;",
                     "STP(p);"),
}
HDR = r'''
#include "%s/dkg_amd/csrc/points.h"
#define LD10(dst, off) for (int i_ = 0; i_ < 10; i_++) (dst)[i_] = o[(off) + i_ * 64 + threadIdx.x];
#define ST10(src) for (int i_ = 0; i_ < 10; i_++) o[i_ * 64 + threadIdx.x] = (src)[i_];
#define LDP(p, off) { uint32_t* w_ = (uint32_t*)&(p); for (int i_ = 0; i_ < 40; i_++) w_[i_] = o[(off) + i_ * 64 + threadIdx.x]; }
#define STP(p) { uint32_t* w_ = (uint32_t*)&(p); for (int i_ = 0; i_ < 40; i_++) o[i_ * 64 + threadIdx.x] = w_[i_]; }
''' % ROOT


# gfx950 VALU issue cost in units of a full-rate wave64 instruction (2 cycles on a SIMD32), measured
# by tools/ubench/intrate*.hip (profiles/r01_ubench_intrate*.txt, profiles/r02_ubench_intrate3.txt):
# only plain 32-bit add/sub/logic/move/select issue at full rate; v_mad_u64_u32, v_mul_lo_u32,
# every shift, the 3-operand fused ops (v_add3, v_lshl_add, v_lshl_or, v_and_or, v_bfe, v_alignbit)
# and the carry-chain adds issue at half rate.
FULL_RATE = ("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32",
             "v_mov_b32", "v_cndmask_b32", "v_not_b32")


def issue_slots(ins):
    op = ins.split()[0].replace("_e32", "").replace("_e64", "").replace("_sdwa", "")
    return 1 if op in FULL_RATE else 2


def main():
    src = HDR
    for name, (pro, body, epi) in PRIMS.items():
        src += f'extern "C" __global__ void k_{name}(uint32_t* o, int n) {{ {pro} for (int it = 0; it < n; it++) {{ {body} }} {epi} }}\n'
    d = tempfile.mkdtemp()
    with open(os.path.join(d, "k.hip"), "w") as f:
        f.write(src)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-S", "--cuda-device-only", "-o",
                           os.path.join(d, "k.s"), os.path.join(d, "k.hip")])
    s = open(os.path.join(d, "k.s")).read()
    out = {}
    for name in PRIMS:
        body = s[s.index(f"k_{name}:"):]
        body = body[:body.index("s_endpgm")]
        blocks = re.split(r"\n\.LBB\d+_\d+:", body)
        best = max(blocks, key=lambda b: sum(1 for l in b.split("\n") if l.strip().startswith("v_")))
        ins = [l.strip() for l in best.split("\n") if l.strip().startswith("v_")]
        out[name] = {"valu": len(ins), "slots": sum(issue_slots(i) for i in ins),
                     "mad_u64": sum(1 for i in ins if i.startswith("v_mad_u64_u32"))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
