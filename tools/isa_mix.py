"""Instruction mix of a kernel's main K loop (the innermost loop containing MFMAs) in a .s file.
usage: python tools/isa_mix.py file.s mangled_name [top]"""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
name = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 0
i = [k for k, l in enumerate(lines) if l.startswith(name + ':')][0]
j = i
while not lines[j].startswith('.Lfunc_end'):
    j += 1
body = lines[i:j]
# loops: a label L and a later backward branch to L; pick the largest one containing MFMAs
labels = {l.split(':')[0]: k for k, l in enumerate(body) if re.match(r'^\.LBB\d+_\d+:', l)}
best = None
for k, l in enumerate(body):
    m = re.search(r's_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)', l)
    if not m:
        continue
    tgt = m.group(1) or m.group(2)
    if tgt in labels and labels[tgt] < k:
        seg = body[labels[tgt]:k + 1]
        nm = sum(1 for x in seg if x.strip().startswith('v_mfma'))
        if nm and (best is None or k - labels[tgt] > best[1] - best[0]):
            best = (labels[tgt], k)
seg = body[best[0]:best[1] + 1]
cnt, ops = {}, {}
for l in seg:
    t = l.strip()
    if not t or t.startswith(';') or t.startswith('.'):
        continue
    op = t.split()[0]
    cls = ('mfma' if op.startswith('v_mfma') else 'valu' if op.startswith('v_') else
           'salu' if op.startswith('s_') else 'lds' if op.startswith('ds_') else
           'vmem' if op.startswith(('global', 'buffer')) else 'other')
    cnt[cls] = cnt.get(cls, 0) + 1
    if cls in ('valu', 'salu'):
        ops[op] = ops.get(op, 0) + 1
print(name[:60], 'loop lines', best[1] - best[0], cnt)
if top:
    print(sorted(ops.items(), key=lambda x: -x[1])[:top])
