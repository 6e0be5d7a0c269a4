"""Cross-check bench.py's live roofline timing against the committed rocprofv3 kernel stats.

bench.py times the dominant stage's launches with HIP events on the library stream
(`roofline.avg_launch_ms` over `roofline.launches`); the rocprof `--kernel-trace --stats` summary of
the same workload lists every kernel.  This sums the stage's kernels in the summary and prints both
averages (they should agree within a few per cent; the runs are separate processes, often on
separate boxes).  Usage: python tools/roofline_check.py [round tag, default r1]
"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAGE_KERNELS = {'conv': ('resblk_kernel', 'rbs_kernel', 'conv_h3_kernel', 'conv_kernel', 'siu_kernel',
                          'siu_pair_kernel', 'siu_chain_kernel', 'odu_kernel'),
                 'od_fe': ('od_fe_kernel', 'od_fe3_kernel'), 'si_fe': ('si_fe_kernel',),
                 'nr': ('nr_stft_kernel', 'nr_gmax_kernel', 'nr_rows_kernel', 'nr_gate_kernel', 'nr_ola_kernel')}
# kernels of a stage's family that bench.py books under another stage (the SI Dense head runs as a
# 1x1 conv_h3 launch: stage 'head')
EXCLUDE = {'conv': ('conv_h3_kernel<1, 1, 32, 128',)}
PAIRS = [('od_pipeline', 'od_pipeline_kernel_stats'), ('si_pipeline', 'si_pipeline_kernel_stats'),
         ('od_features', 'od_features_kernel_stats'), ('noise_gate', 'noise_gate_kernel_stats')]


def main(tag='r1'):
    for wl, stats in PAIRS:
        bj = os.path.join(REPO, 'profiles', f'{tag}_bench_{wl}.json')
        sc = os.path.join(REPO, 'profiles', f'{tag}_{stats}.csv')
        if not (os.path.exists(bj) and os.path.exists(sc)):
            continue
        b = json.load(open(bj))
        for roof in (b['roofline'], b.get('roofline_conv')):
            if roof:
                check(wl, roof, sc)


def check(wl, roof, sc):
    names = STAGE_KERNELS.get(roof.get('kernel'), ())
    rows = [r for r in csv.DictReader(open(sc)) if any(k in r['Name'] for k in names) and
            not any(k in r['Name'] for k in EXCLUDE.get(roof.get('kernel'), ()))]
    calls = sum(int(r['Calls']) for r in rows)
    tot = sum(int(r['TotalDurationNs']) for r in rows) / 1e6
    if roof.get('kernel') == 'nr':   # bench counts one "launch" per nr_gate_launch (5 kernels)
        calls = calls // 5 if calls else 0
    avg = tot / calls if calls else float('nan')
    print(f"{wl:12s} stage {roof.get('kernel'):6s} bench: {roof.get('launches')} launches, "
          f"avg {roof.get('avg_launch_ms', float('nan')):.4f} ms | rocprof: {calls} launches, "
          f"avg {avg:.4f} ms | ratio {avg / roof.get('avg_launch_ms', float('nan')):.3f}")


if __name__ == '__main__':
    main(*sys.argv[1:])
