"""Generate the pair field products fe_mul_ps2 / fe_sq_ps2 in dkg_amd/csrc/fe25519.h.

Each is the single product (fe_mul_ps / fe_sq_ps) written twice with suffixed locals and its
statements interleaved, so consecutive v_mad_u64_u32 belong to different chains; every chain keeps
its own carry-out SGPR pair (cc_a / cc_b) so the hardware sees no back-to-back write of one SGPR.
The generated text replaces the block between the BEGIN/END markers (inserted before
fe_mul_small_ps the first time): python tools/gen_fe_pair.py.  --four adds the four-chain flavour
fe_mul_ps4 / fe_sq_ps4 (two accumulators per product; DKG_FE_PAIR=2, for A/B builds: measured
slower); --check only compares.
"""
import os
import re
import sys
p=os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'dkg_amd', 'csrc', 'fe25519.h')
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
    st=re.sub(r'\b(f\d+(?:_\d+)?|g\d+(?:_\d+)?|h|l)\b', lambda m: m.group(1)+'_'+sfx, st)
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
def columns(fn):
    """(prologue statements, [(terms, limb statement)], epilogue statements) of a single product;
    a term is (x, y) of one mad."""
    pro, cols, epi, cur = [], [], [], []
    for t in body(fn):
        m = re.match(r'(?:uint64_t h = )?mad_(?:first|acc)\((?:h, )?(\w+), (\w+)\);$', t)
        if m:
            cur.append((m.group(1), m.group(2)))
        elif t.startswith('FE_LIMB'):
            cols.append((cur, t)); cur = []
        elif t.startswith('FE_FOLD'):
            epi.append(t)
        else:
            pro.append(t)
    return pro, cols, epi
def gen4(fn, newname, sig):
    """Each product's column split over two accumulators (h: the carry and the even terms, l: the
    odd terms, summed before the limb is cut) and the two products interleaved: four independent
    mad chains, each with its own carry-out SGPR pair."""
    pro, cols, epi = columns(fn)
    out = ['DKG_DEV void %s(%s) {' % (newname, sig),
           '  uint64_t cc_ha = 0, cc_hb = 0, cc_la = 0, cc_lb = 0;  // carry-out pairs, one per chain',
           '  uint64_t h_a, h_b, l_a, l_b;']
    for t in pro:
        out.append('  ' + ren(t, 'a')); out.append('  ' + ren(t, 'b'))
    for k, (terms, limb) in enumerate(cols):
        for i, (x, y) in enumerate(terms):
            acc = 'h' if i % 2 == 0 else 'l'
            for sfx in 'ab':
                xs, ys = ren(x, sfx), ren(y, sfx)
                if (acc == 'h' and k == 0 and i == 0) or (acc == 'l' and i == 1):
                    out.append('  %s_%s = mad_first_v(%s, %s, cc_%s%s);' % (acc, sfx, xs, ys, acc, sfx))
                else:
                    out.append('  mad_acc_v(%s_%s, %s, %s, cc_%s%s);' % (acc, sfx, xs, ys, acc, sfx))
        if len(terms) > 1:
            out.append('  h_a += l_a;'); out.append('  h_b += l_b;')
        out.append('  ' + ren(limb, 'a')); out.append('  ' + ren(limb, 'b'))
    for t in epi:
        out.append('  ' + ren(t, 'a')); out.append('  ' + ren(t, 'b'))
    out.append('  asm volatile("" : : "s"(cc_ha), "s"(cc_hb), "s"(cc_la), "s"(cc_lb));  // distinct registers')
    out.append('}')
    return '\n'.join(out)
code=("// Two independent products in one instruction stream (pair versions of fe_mul_ps / fe_sq_ps):\n"
      "// statement by statement interleaved, so consecutive v_mad_u64_u32 belong to different chains and\n"
      "// need no hazard wait state between them (the single chain puts an s_nop 0 between its back-to-back\n"
      "// mads).  All inputs are read before the first output limb is written: outputs may alias inputs.\n"
      "// Generated from the single versions (tools/gen_fe_pair.py); the same terms in the same order.\n")
code+=gen('fe_mul_ps','fe_mul_ps2','fe& ra, const fe& fa, const fe& ga, fe& rb, const fe& fb, const fe& gb')+'\n\n'
code+=gen('fe_sq_ps','fe_sq_ps2','fe& ra, const fe& fa, fe& rb, const fe& fb')+'\n\n'
if '--four' in sys.argv:  # the four-chain flavour (DKG_FE_PAIR=2), measured 4-5 % slower: A/B builds only
    code+=("// Four chains: each product's column summed in two accumulators (the carry and the even terms,\n"
           "// the odd terms), the two products interleaved: one s_nop per four mads instead of two, for a\n"
           "// 64-bit add per column (profiles/r06_pair_ab.txt: slower).\n")
    code+=gen4('fe_mul_ps','fe_mul_ps4','fe& ra, const fe& fa, const fe& ga, fe& rb, const fe& fb, const fe& gb')+'\n\n'
    code+=gen4('fe_sq_ps','fe_sq_ps4','fe& ra, const fe& fa, fe& rb, const fe& fb')+'\n'
begin='// ---- BEGIN generated pair products (tools/gen_fe_pair.py)\n'
end='// ---- END generated pair products\n'
if begin in s:
    i=s.index(begin); j=s.index(end)+len(end)
    out=s[:i]+begin+code+end+s[j:]
else:
    anchor='DKG_DEV void fe_mul_small_ps('
    i=s.index(anchor)
    out=s[:i]+begin+code+end+'\n'+s[i:]
if '--check' in sys.argv:  # tests/test_bounds.py: the header holds what the single products generate
    if out != s:
        print('fe25519.h: the generated pair products are stale; run python tools/gen_fe_pair.py')
        sys.exit(1)
    print('ok: generated pair products up to date')
else:
    open(p,'w').write(out)
    print('ok', len(code.split('\n')))
