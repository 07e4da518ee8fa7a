"""Static check of the stream-wave ring in the compiled pass kernel (pass_cfg 6): inside the loop,
no instruction other than the slot asm (MFMA / ds_read / global_load) may touch a ring, chunk or
accumulator register, and every ring wait is vmcnt(SR - 1).  Usage: python scripts/check_stream_isa.py <file.s>"""
import re
import sys

s = open(sys.argv[1]).read()
nm = re.search(r'^(_Z11pass_kernel\w+Li48EEv8PassArgs):', s, re.M).group(1)
i = s.index(nm + ':')
j = s.index('.Lfunc_end', i)
body = s[i:j].split('\n')


def regs(tok):
    m = re.match(r'v\[(\d+):(\d+)\]', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', tok)
    return {int(m.group(1))} if m else set()


mf = [k for k, l in enumerate(body) if 'v_mfma_f32_16x16x32_bf16' in l and ', 0' not in l.split('bf16', 1)[1][-4:]]
guard = set()
for k in mf:
    ops = [t.strip() for t in body[k].split('bf16', 1)[1].split(',')]
    for t in ops[:3]:
        guard |= regs(t)
for k in range(len(body)):
    if 'global_load_dwordx4' in body[k] and ' nt' in body[k]:
        guard |= regs(body[k].split()[1].rstrip(','))
lo, hi = min(mf) - 200, max(mf) + 200
bad = []
for k in range(lo, hi):
    l = body[k].strip()
    if not l or l.startswith((';', '.')) or l.endswith(':'):
        continue
    op = l.split()[0]
    if op.startswith(('v_mfma', 'ds_read_b128', 'global_load_dwordx4', 's_')):
        continue
    toks = [t.strip(',') for t in l.split()[1:]]
    touched = set()
    for t in toks:
        touched |= regs(t)
    if touched & guard:
        # the flush's diagonal select reads the accumulator after its nop block (s_nop 7 x 3)
        back = '\n'.join(body[max(0, k - 12):k])
        if op == 'v_cndmask_b32_e32' and back.count('s_nop 7') >= 3:
            continue
        bad.append((k, l))
print(f"{len(mf)} MFMA slots, {len(guard)} guarded VGPRs")
for k, l in bad[:40]:
    print("TOUCH", k, l)
w = re.findall(r's_waitcnt vmcnt\((\d+)\) lgkmcnt\((\d+)\)', s[i:j])
print("slot waits:", sorted(set(w)))
sys.exit(1 if bad else 0)
