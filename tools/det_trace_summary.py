"""Per-call kernel breakdown of a detect_only.py rocprofv3 kernel trace: the last detect call (split at the input
kernel image_s2d), kernels grouped by name.  python tools/det_trace_summary.py <run_kernel_trace.csv> [top]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
calls, cur = [], None
for r in rows:
    if 'image_s2d' in r['Kernel_Name']:
        cur = []
        calls.append(cur)
    if cur is not None:
        cur.append(r)
last = calls[-1]
dur = lambda r: (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000  # noqa: E731
span = (int(last[-1]['End_Timestamp']) - int(last[0]['Start_Timestamp'])) / 1000
print(f'{len(calls)} calls; last: {len(last)} kernels, span {span:.1f} us, busy {sum(map(dur, last)):.1f} us')
g = collections.defaultdict(list)
for r in last:
    g[r['Kernel_Name'][:80]].append(dur(r))
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f'{len(v):4d} {sum(v):8.1f} us  {k}')
