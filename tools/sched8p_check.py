"""Formal check of the LDS-DMA half-tile schedule of v3::conv_fwd_8p (csrc/conv.hip): RAW and WAR hazards between the
8 waves of a block, under the gfx950 ordering rules of cdna_hip_programming.md §5 ("Read a staged buffer one phase
AFTER the wait that retires it"; WAR: a restage only after the readers' lgkmcnt and a barrier both passed).

Model.  Each wave runs a program of events: ISSUE(slot, fill) (its 2 LDS-DMA instructions of one half-tile), WAIT(n)
(s_waitcnt vmcnt(n): every ISSUE but the last n/2 of this wave has landed), READ(slot, fill) (ds_reads of a half),
LGKM (the wave's ds_reads are complete), BAR (s_barrier: every wave's k-th BAR is one event).  A READ of fill f of slot s
is safe iff for every wave X there is a barrier index b such that X retired its ISSUE of f before its b-th BAR and the
reader performs the READ after its own b-th BAR.  An ISSUE of fill f into slot s is safe iff for every reader of the
previous fill there is a b with that reader's LGKM (after the READ) before its b-th BAR and the ISSUE after the
issuer's b-th BAR.  The two groups of 4 waves run staggered by one barrier (group 1 passes one extra barrier first).

python tools/sched8p_check.py [nk ...]   (exits 1 on a hazard)
"""
import sys

NA, NB = 3, 2  # A half-tiles triple-buffered (6 slots), B double-buffered (4 slots): 10 x 16 KiB = 160 KiB


def slot(op, h, t):
    return ('A', (t % NA) * 2 + h) if op == 'A' else ('B', (t % NB) * 2 + h)


def issues_in_phase(u, p, nk):
    """the half-tile a wave issues in phase p of K tile u (steady state): p0 B1(u+1), p1 A0(u+2), p2 A1(u+2),
    p3 B0(u+2)"""
    t, op, h = {0: (u + 1, 'B', 1), 1: (u + 2, 'A', 0), 2: (u + 2, 'A', 1), 3: (u + 2, 'B', 0)}[p]
    return [(op, h, t)] if t < nk else []


def reads_in_phase(p):
    """halves a wave reads in phase p of its tile: p0 A-sub0 + B-sub0, p1 B-sub1, p2 A-sub1, p3 none"""
    return {0: ['A', 'B'], 1: ['B'], 2: ['A'], 3: []}[p]


def program(wid, nk):
    grp = wid >> 2
    wm, wn = wid % 2, wid // 2  # tile mapping: A half = wm, B half = wn // 2
    ev = []
    # prologue: tile 0 whole, tile 1's A0, A1, B0 (the stream order of each operand is kept)
    pro = [('A', 0, 0), ('A', 1, 0), ('B', 0, 0), ('B', 1, 0)]
    if nk > 1:
        pro += [('A', 0, 1), ('A', 1, 1), ('B', 0, 1)]
    for op, h, t in pro:
        ev.append(('ISSUE', slot(op, h, t), (op, h, t)))
    ev.append(('WAIT', 6 if nk > 1 else 0))
    ev.append(('BAR',))
    if grp == 1:
        ev.append(('BAR',))
    for u in range(nk):
        for p in range(4):
            for op in reads_in_phase(p):
                h = wm if op == 'A' else wn // 2
                ev.append(('READ', slot(op, h, u), (op, h, u)))
            for op, h, t in issues_in_phase(u, p, nk):
                ev.append(('ISSUE', slot(op, h, t), (op, h, t)))
            if p == 3 and u + 1 < nk:
                # tile u+1 must have landed: outstanding = halves issued after B1(u+1) = A0, A1, B0 of u+2 (if any)
                ev.append(('WAIT', 6 if u + 2 < nk else 0))
            ev.append(('BAR',))
            ev.append(('LGKM',))
            ev.append(('BAR',))
    if grp == 0:
        ev.append(('BAR',))
    return ev


def check(nk, nw=8):
    progs = [program(w, nk) for w in range(nw)]
    nbar = [sum(1 for e in p if e[0] == 'BAR') for p in progs]
    assert len(set(nbar)) == 1, nbar
    # per wave: barrier count before each event; retirement of issues
    info = []
    for w, prog in enumerate(progs):
        b = 0
        issued = []  # (fill, event index)
        retire_bar = {}  # fill -> barrier count at the WAIT that retired it (retired before barrier b+1)
        reads = []  # (slot, fill, bar count at read, bar count at the following LGKM)
        pending_reads = []
        issues = []  # (slot, fill, bar count at issue)
        for e in prog:
            if e[0] == 'BAR':
                b += 1
            elif e[0] == 'ISSUE':
                issued.append(e[2])
                issues.append((e[1], e[2], b))
            elif e[0] == 'WAIT':
                n = e[1] // 2
                for f in issued[:len(issued) - n] if n else issued:
                    retire_bar.setdefault(f, b)
            elif e[0] == 'READ':
                pending_reads.append((e[1], e[2], b))
            elif e[0] == 'LGKM':
                for s, f, rb in pending_reads:
                    reads.append((s, f, rb, b))
                pending_reads = []
        info.append(dict(retire=retire_bar, reads=reads, issues=issues))
    errs = []
    # RAW: a READ of fill f at barrier count rb needs every wave to have retired f at a barrier count < rb... the
    # wave's WAIT happened while its barrier count was c, i.e. before its (c+1)-th barrier; the reader read after its
    # rb-th barrier: safe iff c + 1 <= rb
    for w, d in enumerate(info):
        for s, f, rb, _ in d['reads']:
            for x, dx in enumerate(info):
                c = dx['retire'].get(f)
                if c is None or c + 1 > rb:
                    errs.append(f'RAW: wave {w} reads {f} (slot {s}) after barrier {rb}; wave {x} retires it at {c}')
    # WAR: an ISSUE of fill f into slot s at barrier count ib needs every READ of the previous fill of s finished
    # (its LGKM at barrier count lb, i.e. before barrier lb+1) with lb + 1 <= ib
    for x, dx in enumerate(info):
        for s, f, ib in dx['issues']:
            prev = [(w, f2, lb) for w, d in enumerate(info) for s2, f2, rb, lb in d['reads']
                    if s2 == s and f2 != f and f2[2] < f[2]]
            for w, f2, lb in prev:
                if lb + 1 > ib:
                    errs.append(f'WAR: wave {x} issues {f} into slot {s} at barrier {ib}; wave {w} finishes reading '
                                f'{f2} at {lb}')
    # every read sees the fill it expects: the slot's most recent issued fill by the time of the read is f
    return errs


if __name__ == '__main__':
    nks = [int(v) for v in sys.argv[1:]] or [1, 2, 3, 4, 5, 8, 9, 36]
    bad = 0
    for nk in nks:
        e = check(nk)
        print(f'nk={nk}: {"ok" if not e else str(len(e)) + " hazards"}')
        for x in e[:8]:
            print('   ', x)
        bad += len(e)
    sys.exit(1 if bad else 0)
