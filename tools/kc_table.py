"""Tabulate tools/gpu_kernel_counters.sh output (gpurun_out/kc_*) per op, per GB."""
import collections
import csv
import glob
import statistics
import sys

ORDER = ['c2swap'] * 3 + ['c4swap'] * 3 + ['c3swap'] * 3 + ['c5T'] * 3 + ['c5pack'] * 3 + ['c5pack_chunk'] + ['c5v2k'] * 3
OPS = ['c2swap', 'c4swap', 'c3swap', 'c5T', 'c5pack', 'c5v2k']
BYTES = {'c2swap': 4.194304e9, 'c4swap': 2 * 10000 * 1024 * 1024 * 2, 'c3swap': 2 * 4096 * 256 * 256 * 32 * 4,
         'c5T': 2 * 64 ** 5 * 8, 'c5pack': 20.7e9, 'c5v2k': 22.31e9}
KERNELS = ('k_transpose', 'k_rowcopy', 'k_recmap_lds', 'k_recmap_parts')
root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out'
res = collections.defaultdict(dict)
for f in sorted(glob.glob(root + '/kc_[0-9]*/**/*counter_collection.csv', recursive=True)):
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if not any(k in r['Kernel_Name'] for k in KERNELS):
            continue
        d = disp.setdefault(r['Dispatch_Id'], {})
        d[r['Counter_Name']] = d.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    for op, d in zip(ORDER, disp.values()):
        for c, v in d.items():
            res[op].setdefault(c, []).append(v)
ctrs = sorted({c for op in res for c in res[op]})
print('| counter (median of 3 launches) / GB of algorithmic bytes | ' + ' | '.join(OPS) + ' |')
print('|---' * (len(OPS) + 1) + '|')
for c in ctrs:
    cells = []
    for op in OPS:
        v = res[op].get(c)
        cells.append('%.3g' % (statistics.median(v) / (BYTES[op] / 1e9)) if v else '-')
    print('| %s | %s |' % (c, ' | '.join(cells)))
