"""HBM bytes per call of each conv kernel family from rocprofv3 --pmc passes of a bench command.

python tools/pmc_traffic.py <config> gpurun_out/pmc_<tag>      (reads <prefix>_fetch, <prefix>_write, and the bench
                                                                JSON line the profiled command printed, <prefix>_fetch.log)

The population is the bench's own: bench.py times one record per dmy_conv_* CALL (its KernelTimer
kinds conv_fwd / conv_dgrad / conv_wgrad / conv_bwd1x1 / conv_fwd_f8), and a call may launch several kernels (a
stride-2 data-grad its parity classes, a k > 1 weight-grad its GEMM-order kernel and the OIHW scatter, a split-K reduce,
the fused 1x1 backward its slot reduce).  So every dispatch is assigned to the C-ABI call family that launches it,
from the kernel name and its DG (data-grad) template argument -- `family()` below is that table -- and the family's
bytes are divided by the number of CALLS the same command made, read from its bench line:
    calls = roofline.kernels[family].launches x (warmup + 2 x steps) / steps
(the profiled command runs `warmup` steps, the `steps` timed steps and the roofline pass of `steps` more; every step
makes the same calls).  Bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950: FETCH_SIZE counts half of a wide
coalesced stream, MI355X_MICROARCH.md §HBM).  Not attributed: the hipMemsetAsync fills of the k > 1 weight-grad
GEMM-order buffers (a runtime fill kernel shared with torch's own fills; K x 9C x 4 B per layer, < 0.2 % of the
family's bytes).

Adds {config: {family: {...}, '_per_step': {...}}} to profiles/pmc_traffic.json; bench.py reads bytes_per_call as
roofline.traffic and checks calls_per_step against its own launch count.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')


def _targs(name, token):
    i = name.index(token) + len(token)
    return [a.strip() for a in name[i:name.index('>', i)].split(',')]


# kernel -> index of its DG template argument (the kernels forward and data-grad share)
_DG_ARG = {'conv_fwd_v3<': 4,     # <BM, BN, NS, P1, DG, BUF>
           'conv_fwd_w<': 3,      # <BM, BN, P1, DG>
           'conv_fwd_8p<': 1,     # <P1, DG>
           'conv_p1p<': 4,        # <BM, BN, NS, WTR, DG, ...>
           'conv3_halo64<': 0,    # <DG, EVAL>
           'conv_p1_persist<': 2,
           'conv_p1s<': 3}        # <KD, NTH, G3, DG>: output-heavy 1x1 forwards, the stem, output-heavy 1x1 data-grads
_FWD = ('conv_sk<', 'conv_fwd_split<', 'splitk_epi_kernel', 'conv_fwd_kernel<')
_DGRAD = ('conv_dgrad_s2_v3<', 'conv_dgrad_q2', 'conv_s2p<', 'conv_dgrad_kernel<')
_WGRAD = ('conv_wgrad_v3<', 'conv_wgrad_v3n<', 'conv_wgrad_v4<', 'conv_wgrad_w<', 'conv_wgrad_tap<', 'conv_wgrad_kernel<',
          'wgrad_to_oihw_kernel', 'wgrad_s2d_to_oihw_kernel', 'wgrad_split_reduce')
_BWD1 = ('conv1x1_bwd_bn<', 'conv1x1_bwd_bn', 'wgrad_slots_reduce')


def family(name):
    """the dmy_conv_* call family (bench.py KernelTimer kind) that launches kernel `name`, or None"""
    for tok, i in _DG_ARG.items():
        if tok in name:
            args = _targs(name, tok)
            return 'conv_dgrad' if len(args) > i and args[i] == 'true' else 'conv_fwd'
    if 'conv_fwd_f8<' in name:
        return 'conv_fwd_f8'
    if any(t in name for t in _BWD1):
        return 'conv_bwd1x1'
    if any(t in name for t in _WGRAD):
        return 'conv_wgrad'
    if any(t in name for t in _DGRAD):
        return 'conv_dgrad'
    if any(t in name for t in _FWD):
        return 'conv_fwd'
    return None


def bench_line(path):
    """the JSON line a bench.py run printed (last line starting with '{"metric"')"""
    line = None
    with open(path, errors='replace') as f:
        for s in f:
            if s.startswith('{"metric"'):
                line = s
    if line is None:
        raise SystemExit(f'{path}: no bench JSON line (the profiled command must be bench.py)')
    return json.loads(line)


def main(config, prefix):
    b = bench_line(prefix + '_fetch.log')
    steps, warm = b['steps'], b['warmup']
    nsteps = warm + 2 * steps
    kern = b['roofline']['kernels']
    acc = {}
    for p, counter, mult in (('fetch', 'FETCH_SIZE', 2.0), ('write', 'WRITE_SIZE', 1.0)):
        disp = load(prefix + '_' + p)
        for did, (name, _grid, dur, ctrs) in disp.items():
            fam = family(name)
            if fam is None or counter not in ctrs:
                continue
            r = acc.setdefault(fam, {'read': 0.0, 'write': 0.0, 'ns': 0.0, 'dispatches': 0})
            r['read' if p == 'fetch' else 'write'] += mult * ctrs[counter] * 1024
            if p == 'fetch':
                r['ns'] += dur
                r['dispatches'] += 1
    out, tot_pmc, tot_alg = {}, 0.0, 0.0
    for fam, r in sorted(acc.items()):
        if fam not in kern:
            print(f'warning: {fam}: {r["dispatches"]} dispatches but no bench calls of that kind', file=sys.stderr)
            continue
        cps = kern[fam]['launches'] / steps  # calls per step, from the bench's own records
        calls = cps * nsteps
        alg_step = kern[fam]['gbps'] * 1e9 * kern[fam]['ms'] * 1e-3  # algorithmic bytes per step (bench records)
        pmc_step = (r['read'] + r['write']) / nsteps
        tot_pmc += pmc_step
        tot_alg += alg_step
        out[fam] = {'bytes_per_call': (r['read'] + r['write']) / calls, 'read_bytes_per_call': r['read'] / calls,
                    'write_bytes_per_call': r['write'] / calls, 'calls_per_step': cps,
                    'dispatches_per_step': r['dispatches'] / nsteps,
                    'pmc_bytes_per_step': pmc_step, 'algorithmic_bytes_per_step': alg_step,
                    'pmc_over_algorithmic': pmc_step / alg_step if alg_step else None,
                    'avg_call_us_profiled': r['ns'] / calls / 1e3,
                    'source': os.path.basename(prefix) + '_{fetch,write} (rocprofv3 --kernel-trace --pmc FETCH_SIZE / '
                              f'WRITE_SIZE; bench.py --steps {steps} --warmup {warm}: {nsteps} training steps)'}
    out['_per_step'] = {'pmc_bytes': tot_pmc, 'algorithmic_bytes': tot_alg,
                        'pmc_over_algorithmic': tot_pmc / tot_alg if tot_alg else None,
                        'families': sorted(k for k in out if not k.startswith('_'))}
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    db[config] = out
    json.dump(db, open(OUT, 'w'), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
