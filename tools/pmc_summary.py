"""Summarise rocprofv3 --pmc CSV passes per kernel (dev tool; not part of the product).

usage: python tools/pmc_summary.py gpurun_out/pmc_*  [--match resblk]
Counters are summed over dispatches of a kernel; FETCH_SIZE is reported x2 (gfx950 correction,
MI355X_MICROARCH.md HBM/rocprofv3 section) and both FETCH/WRITE_SIZE are KiB.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(dirs):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in dirs:
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r['Kernel_Name']
                tot[k][r['Counter_Name']] += float(r['Counter_Value'])
                disp[k].add((d, r['Dispatch_Id']))
    return tot, disp


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    match = None
    if '--match' in sys.argv:
        match = sys.argv[sys.argv.index('--match') + 1]
        args = [a for a in args if a != match]
    tot, disp = load(args)
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0)):
        if match and match not in k:
            continue
        if 'anonymous' not in k:
            continue
        name = k.replace('(anonymous namespace)::', '')[:90]
        nd = max(1, len({x[1] for x in disp[k]}))
        print(f'== {name}')
        out = []
        for key in sorted(c):
            v = c[key]
            if key == 'FETCH_SIZE':
                v *= 2
            out.append(f'{key}={v:.4g}')
        print('   ' + '  '.join(out))
        w = c.get('SQ_WAVES', 0)
        if w:
            per = {x: c[x] / w for x in ('SQ_INSTS_VALU', 'SQ_INSTS_MFMA', 'SQ_INSTS_LDS',
                                         'SQ_INSTS_VMEM_RD', 'SQ_INSTS_VMEM_WR') if x in c}
            print('   per wave: ' + '  '.join(f'{x[8:]}={v:.1f}' for x, v in per.items()))
        wc = c.get('SQ_WAVE_CYCLES', 0)
        if wc:
            print('   wave-cycle share: ' + '  '.join(
                f'{x[3:]}={c[x] / wc:.2f}' for x in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY',
                                                     'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_MFMA')
                if x in c))


if __name__ == '__main__':
    main()
