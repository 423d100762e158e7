import re, subprocess, sys
FULL = ("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_mov_b32", "v_cndmask_b32", "v_not_b32")
def slots(op):
    op = op.replace("_e32", "").replace("_e64", "").replace("_sdwa", "")
    if op in FULL: return 1
    return 2 if op.startswith("v_") else 0
src, out = sys.argv[1], sys.argv[2]
inc = sys.argv[3]
subprocess.check_call(["/opt/rocm/bin/hipcc","--offload-arch=gfx950","-O3","-std=c++17","-S","--cuda-device-only","-I",inc,"-o",out,src], stderr=subprocess.DEVNULL)
s = open(out).read()
for m in re.finditer(r"\n(_Z\w*(k_binom_step|k_stepping|k_combine|k_check|k_affine)\w*):[^\n]*\n", s):
    name = m.group(1); body = s[m.end():]; body = body[:body.index("s_endpgm")]
    ops = [l.split()[0] for l in body.split("\n") if l.strip().startswith("v_")]
    tot = sum(slots(o) for o in ops)
    mads = sum(1 for o in ops if o.startswith("v_mad_u64_u32"))
    movs = sum(1 for o in ops if o.startswith("v_mov"))
    vg = re.search(r"\.amdhsa_next_free_vgpr (\d+)", s[s.index(".amdhsa_kernel " + name):])
    print(f"{m.group(2):14s} ops {len(ops):6d} slots {tot:6d} mads {mads:5d} movs {movs:4d} vgpr {vg.group(1)} {name[15:70]}")
