"""Per-kernel summary of a rocprofv3 results database (rocpd sqlite), optionally against an older
kernel-stats CSV or database: python tools/prof_db.py run_results.db [baseline.{csv,db}] [--csv out]"""
import csv
import sqlite3
import sys


def load(path):
    if path.endswith('.csv'):
        return {r['Name']: (int(r['Calls']), float(r['TotalDurationNs']), float(r['AverageNs']))
                for r in csv.DictReader(open(path))}
    c = sqlite3.connect(path)
    return {n: (k, float(s), float(a)) for n, k, s, a in
            c.execute('select name, count(*), sum(end-start), avg(end-start) from kernels group by name')}


def main():
    argv = sys.argv[1:]
    if '--csv' in argv:   # its value is an output path, not a baseline
        i = argv.index('--csv')
        argv = argv[:i] + argv[i + 2:]
    args = [a for a in argv if not a.startswith('--')]
    cur = load(args[0])
    base = load(args[1]) if len(args) > 1 else {}
    if '--csv' in sys.argv:
        out = sys.argv[sys.argv.index('--csv') + 1]
        with open(out, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage'])
            tot = sum(v[1] for v in cur.values())
            for n, (k, s, a) in sorted(cur.items(), key=lambda kv: -kv[1][1]):
                w.writerow([n, k, int(s), round(a, 1), round(100 * s / tot, 4)])
    tot = sum(v[1] for v in cur.values())
    for n, (k, s, a) in sorted(cur.items(), key=lambda kv: -kv[1][1])[:30]:
        if n.startswith('void at::') or 'elementwise' in n:
            continue
        b = base.get(n)
        print('%5.1f%% %5d avg %8.3f ms%s  %s' % (100 * s / tot, k, a / 1e6,
              ('  (was %8.3f)' % (b[2] / 1e6)) if b else '', n[:110]))


if __name__ == '__main__':
    main()
