"""Summarise a rocprofv3 kernel_stats.csv: top kernels, families, ms per step."""
import csv, sys, re
path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 12
r = [x for x in csv.DictReader(open(path)) if 'spin_kernel' not in x['Name']]  # bench's host-queue spin
tot = sum(float(x['TotalDurationNs']) for x in r)
fam = {}
for x in r:
    n = x['Name']
    k = ('gemm' if 'gemm_kernel' in n else 'bn' if re.search(r'bn_', n) else 'coatt' if ('coatt' in n or 'softmax' in n or 'col_stats' in n or 'prow' in n or 'dscore' in n) else 'splitk' if 'splitk' in n else 'other')
    fam[k] = fam.get(k, 0) + float(x['TotalDurationNs'])
print("total %.2f ms/step over %g steps" % (tot / steps / 1e6, steps))
for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
    print("  %-8s %6.2f ms/step %5.1f%%" % (k, v / steps / 1e6, 100 * v / tot))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print('%6.2f%% %8.1fus %6d  %s' % (100 * float(x['TotalDurationNs']) / tot, float(x['AverageNs']) / 1e3, int(x['Calls']), x['Name'][:110]))
