"""Tabulate tools/gpu_scatter_counters.sh output: python tools/scatter_counter_table.py <TAG>."""
import collections, csv, glob, statistics, sys
T = sys.argv[1]
P = 76 * 76 * 64 ** 3 * 8
BYTES = {'c5k2v': 2 * P, 'c5unchunk': P + 64 ** 5 * 8, 'c4swap': 2 * 10000 * 1024 * 1024 * 2}
OPS = ['c5k2v', 'c5unchunk', 'c4swap']
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob('gpurun_out/%s_sc_[0-9]*/**/*counter_collection.csv' % T, recursive=True)):
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if 'k_recmap_scatter' not in r['Kernel_Name'] and 'k_rowcopy' not in r['Kernel_Name']:
            continue
        d = disp.setdefault(int(r['Dispatch_Id']), {})
        d[r['Counter_Name']] = d.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    ds = [disp[k] for k in sorted(disp)]
    for i, d in enumerate(ds):
        op = OPS[i // 4]
        for c, v in d.items():
            res[op][c].append(v)
ctrs = sorted({c for op in res for c in res[op]})
print('| counter (median of 4 launches) | ' + ' | '.join(OPS) + ' | k2v/unchunk per GB |')
print('|---' * (len(OPS) + 2) + '|')
for c in ctrs:
    vals = {op: statistics.median(res[op][c]) for op in OPS if res[op].get(c)}
    cells = ['%.4g' % vals[op] if op in vals else '-' for op in OPS]
    ratio = (vals['c5k2v'] / BYTES['c5k2v']) / (vals['c5unchunk'] / BYTES['c5unchunk']) if 'c5k2v' in vals and vals.get('c5unchunk') else float('nan')
    print('| %s | %s | %.3f |' % (c, ' | '.join(cells), ratio))
