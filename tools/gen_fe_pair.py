"""Generate the pair field products fe_mul_ps2 / fe_sq_ps2 in dkg_amd/csrc/fe25519.h.

Each is the single product (fe_mul_ps / fe_sq_ps) written twice with suffixed locals and its
statements interleaved, so consecutive v_mad_u64_u32 belong to different chains; every chain keeps
its own carry-out SGPR pair (cc_a / cc_b) so the hardware sees no back-to-back write of one SGPR.
The generated text replaces the block between the BEGIN/END markers (inserted before
fe_mul_small_ps the first time).  Run from the repository root: python tools/gen_fe_pair.py
"""
import re
p='dkg_amd/csrc/fe25519.h'
s=open(p).read()
def body(fn):
    i=s.index('DKG_DEV void %s('%fn); j=s.index('\n}\n',i)
    b=s[s.index('{',i)+1:j]
    toks=[]
    for line in b.split('\n'):
        line=line.strip()
        if not line or line.startswith('//'): continue
        if line.startswith('FE_LIMB') or line.startswith('FE_FOLD'):
            toks.append(line); continue
        for st in line.split(';'):
            st=st.strip()
            if st and not st.startswith('//'): toks.append(st+';')
    return toks
def ren(st, sfx):
    # the volatile mads with the chain's own carry-out pair (cc_a / cc_b)
    st=re.sub(r'mad_acc\(([^;]*)\);', lambda m: 'mad_acc_v(%s, cc_%s);' % (m.group(1), sfx), st)
    st=re.sub(r'mad_first\(([^;]*)\);', lambda m: 'mad_first_v(%s, cc_%s);' % (m.group(1), sfx), st)
    st=re.sub(r'\b(f\d+(?:_\d+)?|g\d+(?:_\d+)?|h)\b', lambda m: m.group(1)+'_'+sfx, st)
    st=st.replace('f.v[', 'f%s.v['%sfx).replace('g.v[', 'g%s.v['%sfx)
    st=re.sub(r'FE_LIMB\(r,', 'FE_LIMB(r%s,'%sfx, st)
    st=re.sub(r'FE_FOLD\(r,', 'FE_FOLD(r%s,'%sfx, st)
    return st
def gen(fn, newname, sig):
    toks=body(fn)
    out=['DKG_DEV void %s(%s) {'%(newname,sig), '  uint64_t cc_a = 0, cc_b = 0;  // carry-out pairs, one per chain']
    for t in toks:
        out.append('  '+ren(t,'a'))
        out.append('  '+ren(t,'b'))
    out.append('  asm volatile("" : : "s"(cc_a), "s"(cc_b));  // both pairs live to the end: distinct registers')
    out.append('}')
    return '\n'.join(out)
code=("// Two independent products in one instruction stream (pair versions of fe_mul_ps / fe_sq_ps):\n"
      "// statement by statement interleaved, so consecutive v_mad_u64_u32 belong to different chains and\n"
      "// need no hazard wait state between them (the single chain puts an s_nop 0 between its back-to-back\n"
      "// mads).  All inputs are read before the first output limb is written: outputs may alias inputs.\n"
      "// Generated from the single versions (tools/gen_fe_pair.py); the same terms in the same order.\n")
code+=gen('fe_mul_ps','fe_mul_ps2','fe& ra, const fe& fa, const fe& ga, fe& rb, const fe& fb, const fe& gb')+'\n\n'
code+=gen('fe_sq_ps','fe_sq_ps2','fe& ra, const fe& fa, fe& rb, const fe& fb')+'\n'
begin='// ---- BEGIN generated pair products (tools/gen_fe_pair.py)\n'
end='// ---- END generated pair products\n'
if begin in s:
    i=s.index(begin); j=s.index(end)+len(end)
    s=s[:i]+begin+code+end+s[j:]
else:
    anchor='DKG_DEV void fe_mul_small_ps('
    i=s.index(anchor)
    s=s[:i]+begin+code+end+'\n'+s[i:]
open(p,'w').write(s)
print('ok', len(code.split('\n')))
