"""Summarise rocprofv3 PMC passes (scripts/pmc_capture.sh) into profiles/.

    python scripts/pmc_summary.py <tag> <kernel-substring> [round [source_rev]]

HBM traffic per launch of the named kernel, corrected as MI355X_MICROARCH.md's HBM section
prescribes: gfx950 FETCH_SIZE counts exactly half the bytes of a wide coalesced (16 B/lane)
streaming read -> x2; WRITE_SIZE is exact for 16 B/lane stores -> as is; both KiB -> x1024.
Writes profiles/<round>/pmc_<tag>.txt (every counter, every kernel) and, for the named
kernel, profiles/traffic_<kernel-substring>_<tag>.json with the kernel-source revision it was
measured on (bench.py ignores a traffic file whose revision differs from the running sources).
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    tag, kname = sys.argv[1], sys.argv[2]
    rnd = sys.argv[3] if len(sys.argv) > 3 else 'r02'
    src = os.path.join(ROOT, 'gpurun_out', 'pmc_' + tag)
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(src, 'p*', '**', '*counter_collection.csv'), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '')
            vals[(k, r['Counter_Name'])].append(float(r['Counter_Value']))
    # the kernel-source revision the passes ran on (written by pmc_capture.sh on the GPU box)
    # (source_rev.json: the revision of all device sources ("null") and of each measured kernel's)
    revs = {}
    if os.path.exists(os.path.join(src, 'source_rev.json')):
        revs = json.load(open(os.path.join(src, 'source_rev.json')))
    elif os.path.exists(os.path.join(src, 'source_rev.txt')):
        revs = {'null': open(os.path.join(src, 'source_rev.txt')).read().strip()}
    kkey = kname.replace('_kernel', '')
    rev = revs.get(kkey) or revs.get('null') or (sys.argv[4] if len(sys.argv) > 4 else None)
    if not rev:
        raise SystemExit('no source_rev.json in %s: pass the revision the capture ran on as argv[4]' % src)
    lines = ['# PMC summary %s (kernel sources %s); per-dispatch means' % (tag, rev)]
    for (k, c), v in sorted(vals.items()):
        lines.append('%-60s %-26s n=%-3d mean=%.6g' % (k[:60], c, len(v), sum(v) / len(v)))
    os.makedirs(os.path.join(ROOT, 'profiles', rnd), exist_ok=True)
    with open(os.path.join(ROOT, 'profiles', rnd, 'pmc_%s.txt' % tag), 'w') as fh:
        fh.write('\n'.join(lines) + '\n')
    print('\n'.join(lines))

    def mean(k, c):
        v = vals.get((k, c))
        return sum(v) / len(v) if v else None

    ks = sorted({k for k, _ in vals if kname in k})
    for k in ks:
        fetch, write = mean(k, 'FETCH_SIZE'), mean(k, 'WRITE_SIZE')
        if fetch is None or write is None:
            continue
        rec = {'kernel': k, 'fetch_kib_raw': fetch, 'write_kib_raw': write,
               'bytes_per_launch': 2 * fetch * 1024 + write * 1024,
               'correction': 'FETCH_SIZE*2*1024 + WRITE_SIZE*1024 (gfx950, MI355X_MICROARCH.md HBM section)',
               'source': '%s/pmc_%s.txt' % (rnd, tag), 'source_rev': rev,
               'lds_bank_conflict_cycles': mean(k, 'SQ_LDS_BANK_CONFLICT'),
               'lds_active_cycles': mean(k, 'SQ_LDS_IDX_ACTIVE'),
               'mfma_busy_cycles': mean(k, 'SQ_VALU_MFMA_BUSY_CYCLES'),
               'grbm_gui_active': mean(k, 'GRBM_GUI_ACTIVE')}
        # MFMA utilisation: SQ_VALU_MFMA_BUSY_CYCLES is summed over every SIMD of the chip
        # (32 per v_mfma_f32_16x16x4_f32 = its issue cycles on one SIMD; checked against the
        # launch's MFMA count), GRBM_GUI_ACTIVE over the 8 XCDs (MI355X_MICROARCH.md, DVFS
        # item) -> busy / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) = the fraction of the chip's
        # MFMA issue cycles spent in MFMAs during the launch
        if rec['mfma_busy_cycles'] is not None and rec['grbm_gui_active']:
            rec['mfma_busy'] = rec['mfma_busy_cycles'] / (1024.0 * rec['grbm_gui_active'] / 8.0)
            rec['mfma_busy_note'] = ('SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs): '
                                     'chip-wide MFMA pipe busy fraction over the launch')
        name = kname.replace('_kernel', '')
        with open(os.path.join(ROOT, 'profiles', 'traffic_%s_%s.json' % (name, tag)), 'w') as fh:
            json.dump(rec, fh, indent=1)
        print('traffic', tag, rec)
        break


if __name__ == '__main__':
    main()
