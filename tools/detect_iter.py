"""Kernel mix of one detect iteration from a rocprofv3 kernel_trace.csv of tools/gpu/detect_only.py (iterations
split at the NMS greedy kernel): python tools/detect_iter.py <kernel_trace.csv> [iteration] [top]"""
import collections
import csv
import re
import sys


def main(path, k=20, top=25):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    its, cur = [], []
    for r in rows:
        cur.append(r)
        if 'nms_greedy' in r['Kernel_Name']:
            its.append(cur)
            cur = []
    it = its[min(k, len(its) - 1)]
    c = collections.defaultdict(lambda: [0, 0.0])
    for r in it:
        n = re.sub(r'\(.*', '', r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', ''))[:80]
        c[n][0] += 1
        c[n][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    for n, (cnt, us) in sorted(c.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f'{cnt:4d} {us:8.1f} us  {n}')
    span = (int(it[-1]['End_Timestamp']) - int(it[0]['Start_Timestamp'])) / 1e3
    print(f'iteration span {span:.1f} us, kernel sum {sum(v[1] for v in c.values()):.1f} us, {len(it)} kernels')


if __name__ == '__main__':
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
