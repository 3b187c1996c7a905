"""Instruction mix of the loops of one kernel in a hipcc .s file.

    python tools/isa_count.py file.s mangled_kernel_name
Prints each loop's instruction counts by mnemonic (VALU / SALU / MFMA / memory).
"""
import sys
from collections import Counter


def main():
    lines = open(sys.argv[1]).read().split('\n')
    name = sys.argv[2]
    i = [k for k, l in enumerate(lines) if l.startswith(name + ':')][0]
    j = i
    while not lines[j].startswith('.Lfunc_end'):
        j += 1
    body = lines[i:j]
    hdrs = [k for k, l in enumerate(body) if 'Loop Header' in l]
    for h in hdrs:
        lab = body[h].split(':')[0]
        tag = 'Header=' + lab[2:] + ' '
        blk = [k for k, l in enumerate(body) if tag in l and 'in Loop' in l] + [h]
        ends = [k for k, l in enumerate(body) if lab in l and 'branch' in l]
        if not ends:
            continue
        s, e = min(blk), max(ends + blk)
        c = Counter()
        for l in body[s:e + 1]:
            t = l.strip().split(' ')[0]
            if not t or t.startswith(';') or t.startswith('.'):
                continue
            c[t] += 1
        mf = sum(v for k, v in c.items() if k.startswith('v_mfma'))
        va = sum(v for k, v in c.items() if k.startswith('v_') and not k.startswith('v_mfma'))
        sa = sum(v for k, v in c.items() if k.startswith('s_'))
        print('loop %s: lines %d-%d  mfma %d  valu %d  s_* %d  total %d' % (lab, s, e, mf, va, sa, sum(c.values())))
        for k, v in c.most_common(30):
            print('   %5d %s' % (v, k))


if __name__ == '__main__':
    main()
