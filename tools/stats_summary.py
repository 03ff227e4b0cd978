"""Summarise a rocprofv3 kernel_stats.csv as a markdown table: python tools/stats_summary.py <csv> [steps] [top]"""
import csv
import sys


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    print('| kernel | calls/step | ms/step | avg us | % |')
    print('|---|---|---|---|---|')
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
        t = float(r['TotalDurationNs'])
        print('| %s | %.1f | %.2f | %.1f | %.2f |' % (r['Name'][:110], int(r['Calls']) / steps, t / 1e6 / steps,
                                                 float(r['AverageNs']) / 1e3, 100 * t / tot))
    print('\ntotal GPU kernel time: %.2f ms/step (%d steps incl. warmup)' % (tot / 1e6 / steps, steps))


if __name__ == '__main__':
    main()
