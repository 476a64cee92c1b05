"""Summarise rocprofv3 PMC passes (scripts/profile.sh) into profiles/.

HBM traffic per fs_local_train launch, corrected as MI355X_MICROARCH.md's HBM section
prescribes: gfx950 FETCH_SIZE counts exactly half the bytes of a wide coalesced
(16 B/lane) streaming read -> x2; WRITE_SIZE is exact for 16 B/lane stores and is used
as is; both are KiB -> x1024.  Writes profiles/traffic_local_train.json (read by
bench.py for roofline.traffic) and profiles/<tag>_pmc_summary.txt.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, 'gpurun_out', 'pmc')
tag = sys.argv[2] if len(sys.argv) > 2 else 'r01'
vals = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(src, 'p*', '*counter_collection.csv'))):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '')
        vals[(k, r['Counter_Name'])].append(float(r['Counter_Value']))
lines = []
for (k, c), v in sorted(vals.items()):
    lines.append('%-55s %-28s n=%-3d mean=%.6g' % (k[:55], c, len(v), sum(v) / len(v)))
out = os.path.join(ROOT, 'profiles', '%s_pmc_summary.txt' % tag)
with open(out, 'w') as fh:
    fh.write('\n'.join(lines) + '\n')
print('\n'.join(lines))


def mean(k, c):
    v = vals.get((k, c))
    return sum(v) / len(v) if v else None


lt = [k for k, _ in vals if 'local_train' in k]
if lt:
    k = sorted(set(lt))[0]
    fetch, write = mean(k, 'FETCH_SIZE'), mean(k, 'WRITE_SIZE')
    if fetch is not None and write is not None:
        rec = {'kernel': k, 'fetch_kib_raw': fetch, 'write_kib_raw': write,
               'bytes_per_launch': 2 * fetch * 1024 + write * 1024,
               'correction': 'FETCH_SIZE*2*1024 + WRITE_SIZE*1024 (gfx950, MI355X_MICROARCH.md HBM section)',
               'source': tag}
        with open(os.path.join(ROOT, 'profiles', 'traffic_local_train.json'), 'w') as fh:
            json.dump(rec, fh, indent=1)
        print('traffic', rec)
