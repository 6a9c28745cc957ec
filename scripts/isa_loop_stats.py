"""Instruction mix per basic block of a kernel in a hipcc -S listing.
usage: python scripts/isa_loop_stats.py file.s kernel_substring [min_block_len]"""
import collections
import re
import sys

path, name = sys.argv[1], sys.argv[2]
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 40
s = open(path).read()
starts = [m.start() for m in re.finditer(r'^(_Z\S*' + re.escape(name) + r'\S*):', s, re.M)]
for st in starts[:1]:
    end = s.index('.Lfunc_end', st)
    lines = s[st:end].split('\n')
    print(lines[0])
    blocks, cur = [], None
    for l in lines[1:]:
        t = l.strip()
        if re.match(r'^(\.LBB\S+|;\s*%bb\.\d+):', t) or (t.endswith(':') and not t.startswith('.')):
            cur = [t.split()[0], collections.Counter(), 0]
            blocks.append(cur)
            continue
        if t.startswith('; %bb.'):
            cur = [t, collections.Counter(), 0]
            blocks.append(cur)
            continue
        if not t or t.startswith(('.', ';')) or cur is None:
            continue
        op = t.split()[0]
        cls = ('valu' if op.startswith('v_') else 'salu' if op.startswith('s_') else
               'lds' if op.startswith('ds_') else 'vmem' if op.startswith(('global_', 'buffer_', 'flat_')) else 'other')
        cur[1][cls] += 1
        cur[1]['op:' + op] += 1
        cur[2] += 1
    for b in blocks:
        if b[2] >= minlen:
            c = b[1]
            top = sorted(((v, k[3:]) for k, v in c.items() if k.startswith('op:')), reverse=True)[:18]
            print(f"{b[0]} n={b[2]} valu={c['valu']} salu={c['salu']} lds={c['lds']} vmem={c['vmem']}")
            print('   ', ', '.join(f'{k}:{v}' for v, k in top))
