"""Per conv-family launch statistics from a rocprofv3 kernel_trace.csv (the cross-check of bench.py's roofline
avg_launch_us): python tools/family_stats.py <kernel_trace.csv> [skip_first_fraction]"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import family, kernels_per_call  # noqa: E402


def main(path):
    fams = {}
    for r in csv.DictReader(open(path)):
        name = r.get('Kernel_Name') or r.get('KernelName') or ''
        f = family(name)
        if f is None:
            continue
        d = float(r['End_Timestamp']) - float(r['Start_Timestamp'])
        e = fams.setdefault(f, [0, 0.0])
        e[0] += 1.0 / kernels_per_call(name)  # per dmy_conv_* call (bench.py's unit)
        e[1] += d
    out = {f: {'calls': round(n), 'avg_call_us': round(t / n / 1e3, 2), 'total_ms': round(t / 1e6, 2)}
           for f, (n, t) in fams.items()}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1])
