"""MFMA-busy per conv kernel family from a rocprofv3 --pmc pass of a bench command.

python tools/pmc_mfma.py <config> gpurun_out/<dir of the mfma pass>

Counters (one pass): SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE (+ SQ_BUSY_CYCLES).  Per dispatch
  busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)   (GRBM is summed over the 8 XCDs)
and per family the time-weighted mean over its dispatches (= sum MFMA-busy cycles / sum SIMD-cycles).  Families as
bench.py's roofline (tools/pmc_traffic.family), plus 'conv_3x3': every dispatch of a kernel that only runs k > 1
layers (implicit-GEMM tiles with P1 = false, the halo kernel, the tap-fused weight-grad, the stride-2 data-grad) --
the north-star's ">= 40 % MFMA on 3x3 implicit-GEMM" is read off that row.  Writes {config: {family: {...}}} into
profiles/pmc_mfma.json, which bench.py copies into roofline.kernels[family].mfma_busy.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402
from pmc_traffic import family, _targs  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'profiles', 'pmc_mfma.json')


def is_3x3(name):
    """a dispatch of a k > 1 layer: the kernels that only run them, and the shared implicit-GEMM tiles with P1 = false"""
    if any(t in name for t in ('conv3_halo64<', 'conv_wgrad_tap<', 'conv_dgrad_s2_v3<', 'conv_dgrad_q2', 'conv_s2p<',
                               'conv_fwd_f8<')):
        return True
    if 'conv_p1s<' in name:  # <KD, NTH, G3, DG>: G3 = the space-to-depth stem's 3x3 gather
        return _targs(name, 'conv_p1s<')[2] == 'true'
    for tok, i in (('conv_fwd_w<', 2), ('conv_fwd_v3<', 3), ('conv_fwd_8p<', 0)):  # the P1 template argument
        if tok in name:
            return _targs(name, tok)[i] == 'false'
    return False


def main(cfg, d):
    disp = load(d)
    acc = {}
    for _, (name, _grid, dur, vals) in disp.items():
        if 'SQ_VALU_MFMA_BUSY_CYCLES' not in vals or not vals.get('GRBM_GUI_ACTIVE'):
            continue
        fams = [f for f in (family(name), 'conv_3x3' if is_3x3(name) else None) if f]
        for f in fams:
            a = acc.setdefault(f, dict(busy=0.0, simd_cycles=0.0, dispatches=0, ns=0.0))
            a['busy'] += vals['SQ_VALU_MFMA_BUSY_CYCLES']
            a['simd_cycles'] += 1024 * vals['GRBM_GUI_ACTIVE'] / 8
            a['dispatches'] += 1
            a['ns'] += dur
    res = {f: dict(mfma_busy=round(a['busy'] / a['simd_cycles'], 4), dispatches=a['dispatches'],
                   avg_us=round(a['ns'] / a['dispatches'] / 1e3, 2), source=os.path.basename(d.rstrip('/')) +
                   ' (rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE)')
           for f, a in acc.items()}
    allres = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            allres = json.load(f)
    allres[cfg] = res
    with open(OUT, 'w') as f:
        json.dump(allres, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
