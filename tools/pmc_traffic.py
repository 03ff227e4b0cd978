"""HBM bytes per launch of each conv kernel family from rocprofv3 --pmc passes of a bench command.

python tools/pmc_traffic.py <config> gpurun_out/pmc_<tag>      (reads <prefix>_fetch and <prefix>_write)

Adds {config: {family: {...}}} to profiles/pmc_traffic.json, which bench.py reads to fill
roofline.traffic.  Bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 summed over the family's dispatches
(gfx950: FETCH_SIZE counts half of a wide coalesced stream, MI355X_MICROARCH.md §HBM), divided by
the number of calls (a stride-2 data-grad call is its 4 parity-class dispatches, as in bench.py's KernelTimer).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
FAMILIES = {'conv_fwd': ('conv_fwd',), 'conv_dgrad': ('conv_dgrad',), 'conv_wgrad': ('conv_wgrad',)}


def _targs(name, token):
    i = name.index(token) + len(token)
    return [a.strip() for a in name[i:name.index('>', i)].split(',')]


def kernels_per_call(name):
    """bench.py times one dmy_conv_* CALL per KernelTimer record; the stride-2 data-grad call launches one
    conv_fwd_v3<..., BUF = 3> kernel per output-parity class (4), every other call one family kernel"""
    if 'conv_fwd_v3<' in name:
        args = _targs(name, 'conv_fwd_v3<')
        if len(args) > 5 and args[5] == '3':
            return 4
    return 1


def family(name):
    # the implicit-GEMM kernels shared by forward and data-grad: the DG template argument picks the family
    if 'conv_fwd_v3<' in name:  # <BM, BN, NS, P1, DG, BUF>
        args = _targs(name, 'conv_fwd_v3<')
        return 'conv_dgrad' if len(args) > 4 and args[4] == 'true' else 'conv_fwd'
    if 'conv_fwd_w<' in name:  # <BM, BN, P1, DG>
        args = _targs(name, 'conv_fwd_w<')
        return 'conv_dgrad' if len(args) > 3 and args[3] == 'true' else 'conv_fwd'
    if 'conv_fwd_f8<' in name:
        return 'conv_fwd_f8'
    if 'conv_p1p<' in name:  # <BM, BN, NS, WTR, DG>
        args = _targs(name, 'conv_p1p<')
        return 'conv_dgrad' if len(args) > 4 and args[4] == 'true' else 'conv_fwd'
    if 'conv3_halo64<' in name:  # <DG>
        return 'conv_dgrad' if _targs(name, 'conv3_halo64<')[0] == 'true' else 'conv_fwd'
    if 'conv_p1s<' in name or 'conv_sk<' in name or 'conv_p1_persist<' in name:
        if 'conv_p1_persist<' in name:
            args = _targs(name, 'conv_p1_persist<')
            return 'conv_dgrad' if len(args) > 2 and args[2] == 'true' else 'conv_fwd'
        return 'conv_fwd'
    for fam, keys in FAMILIES.items():
        if any(k in name for k in keys):
            return fam
    return None


def main(config, prefix):
    res = {}
    for p, counter, mult in (('fetch', 'FETCH_SIZE', 2.0), ('write', 'WRITE_SIZE', 1.0)):
        disp = load(prefix + '_' + p)
        for did, (name, _grid, dur, ctrs) in disp.items():
            fam = family(name)
            if fam is None or counter not in ctrs:
                continue
            r = res.setdefault(fam, {'fetch_launches': 0, 'write_launches': 0, 'read_bytes': 0.0, 'write_bytes': 0.0,
                                     'ns': 0.0})
            r[p + '_launches'] += 1.0 / kernels_per_call(name)  # per dmy_conv_* call, as bench.py's records
            r['read_bytes' if p == 'fetch' else 'write_bytes'] += mult * ctrs[counter] * 1024
            if p == 'fetch':
                r['ns'] += dur
    out = {}
    for fam, r in res.items():
        n = max(r['fetch_launches'], 1)
        per = r['read_bytes'] / n + r['write_bytes'] / max(r['write_launches'], 1)
        out[fam] = {'bytes_per_launch': per, 'launches': round(r['fetch_launches']),
                    'read_bytes_per_launch': r['read_bytes'] / n,
                    'write_bytes_per_launch': r['write_bytes'] / max(r['write_launches'], 1),
                    'avg_launch_us_profiled': r['ns'] / n / 1e3,
                    'source': os.path.basename(prefix) + '_{fetch,write} (rocprofv3 --kernel-trace --pmc)'}
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    db[config] = out
    json.dump(db, open(OUT, 'w'), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
