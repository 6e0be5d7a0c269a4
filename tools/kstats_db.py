"""Dev: per-kernel median durations from a rocprofv3 results .db (rocpd sqlite):
python3 tools/kstats_db.py <db> [top]"""
import collections
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 10
cols = [r[1] for r in con.execute('pragma table_info(kernels)')]
name = [c for c in cols if 'name' in c][0]
agg = collections.defaultdict(list)
for r in con.execute('select * from kernels'):
    d = dict(zip(cols, r))
    agg[d[name]].append(d['end'] - d['start'])
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    v = sorted(v)
    print(f'{len(v):6d} calls  median {v[len(v) // 2] / 1e3:9.2f} us  total {sum(v) / 1e6:9.3f} ms  {k[:90]}')
