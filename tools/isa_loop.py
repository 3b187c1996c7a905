"""Print the main-loop skeleton (waits, barriers, DMA, MFMA counts) of one kernel in a .s file.
usage: python tools/isa_loop.py file.s mangled_name_substring"""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
start = [i for i, l in enumerate(lines) if l.startswith(sys.argv[2]) and l.split(':')[0].endswith('EEv8GemmArgs') or (l.startswith(sys.argv[2]) and ':' in l and not l.startswith('\t'))]
i = start[0]
j = i
while not lines[j].startswith('.Lfunc_end'):
    j += 1
body = lines[i:j]
cnt = {}
for l in body:
    for key in ['v_mfma', 'global_load_lds', 'ds_read', 's_waitcnt', 's_barrier', 'scratch_', 'global_store', 'ds_write']:
        if key in l:
            cnt[key] = cnt.get(key, 0) + 1
print(len(body), 'lines', cnt)
run = {}
for l in body:
    t = l.strip()
    if re.match(r'^\.LBB', t) or 's_waitcnt' in t or 's_barrier' in t or 's_cbranch' in t or 's_branch' in t:
        if run:
            print('   ', run)
            run = {}
        print(t)
    else:
        for key in ['v_mfma', 'global_load_lds', 'ds_read', 'ds_write', 'global_store', 'global_load']:
            if t.startswith(key):
                run[key] = run.get(key, 0) + 1
if run:
    print('   ', run)
for l in lines[j:j + 400]:
    if re.search(r'\.(vgpr_count|sgpr_count|agpr_count|private_segment_fixed_size|group_segment_fixed_size):', l):
        print(l.strip())
