"""Summarise a rocprofv3 kernel_stats.csv (top kernels by total time)."""
import csv
import sys


def main(path, top=25, out=None):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    lines = ['| kernel | calls | total ms | avg us | % |', '|---|---|---|---|---|']
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
        n = r['Name'].replace('(anonymous namespace)::', '').replace('void ', '')
        n = n.split('(')[0] if not n.startswith('__') else n
        lines.append(f"| {n[:110]} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    lines.append(f'\ntotal GPU kernel time: {tot / 1e6:.2f} ms')
    txt = '\n'.join(lines)
    if out:
        open(out, 'w').write(txt + '\n')
    print(txt)


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25, sys.argv[3] if len(sys.argv) > 3 else None)
