"""Summarise rocprofv3 --pmc passes (tools/gpu/pmc.sh) per run of consecutive same-kernel dispatches.

python tools/pmc_summary.py gpurun_out/pmc_<tag> [out.md]

Reads <prefix>_{mfma,fetch,write}/**/{counter_collection,kernel_trace}.csv.  Per group:
  clock   = GRBM_GUI_ACTIVE / 8 / duration          (GRBM counts are summed over the 8 XCDs)
  mfma    = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)   (MFMA-busy share)
  hbm     = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 B  (gfx950: FETCH_SIZE counts half of a wide
            coalesced stream, MI355X_MICROARCH.md §HBM)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def _find(d, name):
    hits = glob.glob(os.path.join(d, '**', f'*{name}'), recursive=True)
    return hits[0] if hits else None


def _key(row, *names):
    low = {k.lower(): k for k in row}
    for n in names:
        if n.lower() in low:
            return row[low[n.lower()]]
    raise KeyError(names)


def short(n):
    n = n.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0] if not n.startswith('__') else n


def load(d):
    """dispatch id -> (kernel name, grid, duration ns, {counter: value})"""
    out = {}
    kt = _find(d, 'kernel_trace.csv')
    if kt:
        for r in csv.DictReader(open(kt)):
            did = int(_key(r, 'Dispatch_Id'))
            dur = int(_key(r, 'End_Timestamp')) - int(_key(r, 'Start_Timestamp'))
            grid = _key(r, 'Grid_Size_X', 'Grid_Size', 'Grid_Size_x')
            out[did] = [short(_key(r, 'Kernel_Name')), grid, dur, {}]
    cc = _find(d, 'counter_collection.csv')
    if cc:
        for r in csv.DictReader(open(cc)):
            did = int(_key(r, 'Dispatch_Id'))
            ent = out.setdefault(did, [short(_key(r, 'Kernel_Name')), _key(r, 'Grid_Size', 'Grid_Size_X'), 0, {}])
            c = _key(r, 'Counter_Name')
            ent[3][c] = ent[3].get(c, 0.0) + float(_key(r, 'Counter_Value'))
    return out


def groups(disp):
    """consecutive dispatches with the same (kernel, grid) -> list of dispatch ids"""
    gs, cur, last = [], [], None
    for did in sorted(disp):
        k = tuple(disp[did][:2])
        if k != last and cur:
            gs.append(cur)
            cur = []
        cur.append(did)
        last = k
    if cur:
        gs.append(cur)
    return gs


def main(prefix, out=None):
    passes = {p: load(prefix + '_' + p) for p in ('mfma', 'fetch', 'write') if os.path.isdir(prefix + '_' + p)}
    base = passes.get('mfma') or next(iter(passes.values()))
    lines = ['| # | kernel | grid | n | avg us | clock GHz | MFMA busy | LDS conflict / active | HBM MB/launch | HBM GB/s |',
             '|---|---|---|---|---|---|---|---|---|---|']
    agg = defaultdict(lambda: defaultdict(float))
    for gi, ids in enumerate(groups(base)):
        name, grid = base[ids[0]][:2]
        vals = defaultdict(float)
        for p, disp in passes.items():
            for did in ids:
                if did in disp:
                    for c, v in disp[did][3].items():
                        vals[c] += v / len(ids)
        dur = sum(base[i][2] for i in ids) / len(ids)
        gg = vals.get('GRBM_GUI_ACTIVE', 0.0) / 8
        clock = gg / dur if dur and gg else float('nan')
        mf = vals['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * gg) if gg and 'SQ_VALU_MFMA_BUSY_CYCLES' in vals else float('nan')
        ldsr = (vals['SQ_LDS_BANK_CONFLICT'] / vals['SQ_LDS_IDX_ACTIVE']
                if vals.get('SQ_LDS_IDX_ACTIVE') else float('nan'))
        hbm = (2 * vals.get('FETCH_SIZE', 0.0) + vals.get('WRITE_SIZE', 0.0)) * 1024
        lines.append(f'| {gi} | {name[:70]} | {grid} | {len(ids)} | {dur / 1e3:.1f} | {clock:.2f} | {mf:.3f} | '
                     f'{ldsr:.3f} | {hbm / 1e6:.1f} | {hbm / dur if dur else 0:.0f} |')
        a = agg[name]
        a['n'] += len(ids)
        a['ns'] += dur * len(ids)
        a['hbm'] += hbm * len(ids)
        a['busy'] += vals.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0) * len(ids)
        a['gg'] += gg * len(ids)
    lines += ['', '| kernel | launches | avg us | MFMA busy (time-weighted) | HBM MB/launch |', '|---|---|---|---|---|']
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]['ns']):
        mf = a['busy'] / (1024 * a['gg']) if a['gg'] else float('nan')
        lines.append(f"| {name[:70]} | {int(a['n'])} | {a['ns'] / a['n'] / 1e3:.1f} | {mf:.3f} | {a['hbm'] / a['n'] / 1e6:.1f} |")
    txt = '\n'.join(lines)
    if out:
        open(out, 'w').write(txt + '\n')
    print(txt)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
