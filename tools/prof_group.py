"""Group a rocprofv3 kernel_stats.csv by kernel family (template arguments stripped): per-step us and share."""
import collections
import csv
import re
import sys


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    g = collections.defaultdict(lambda: [0.0, 0])
    for r in rows:
        k = re.sub(r'^void ', '', r['Name']).replace('(anonymous namespace)::', '').split('(')[0]
        k = re.sub(r'<.*', '', k)
        g[k][0] += float(r['TotalDurationNs']) / steps / 1e3
        g[k][1] += int(r['Calls'])
    tot = sum(v[0] for v in g.values())
    print('| kernel family | us/step | calls/step | % |\n|---|---|---|---|')
    for k, v in sorted(g.items(), key=lambda x: -x[1][0]):
        if v[0] / tot > 0.002:
            print(f'| {k} | {v[0]:.1f} | {v[1] / steps:.1f} | {100 * v[0] / tot:.1f} |')
    print(f'\ntotal GPU kernel time per step: {tot / 1e3:.2f} ms')


if __name__ == '__main__':
    main(sys.argv[1], float(sys.argv[2]))
