"""CPU: the C ABI (include/dmayolo.h) is one signature in three places, and all three are checked here.

  * the .hip definitions: csrc/common.h includes the header, so every DMY_API definition must match its declaration
    or the translation unit does not compile (test_mismatched_definition_fails_to_compile proves the mechanism);
  * the ctypes tables (dmayolo/_lib.py SIGNATURES + the optimizer bindings in dmayolo/optim.py): argument count,
    each argument's ctypes type and the return type are derived from the header's C types and compared per symbol;
  * the shared library exports every declared symbol.
No compute calls (no GPU here)."""
import ctypes
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'dmayolo.h')
CSRC = os.path.join(ROOT, 'dma-yolo_amd', 'csrc')

_DECL = re.compile(r'^\s*(int|long)\s+(dmy_\w+)\s*\(([^)]*)\)\s*;', re.M | re.S)
_SCALAR = {'int': ctypes.c_int, 'long': ctypes.c_long, 'float': ctypes.c_float, 'double': ctypes.c_double}


def _strip_comments(src):
    return re.sub(r'//[^\n]*', ' ', re.sub(r'/\*.*?\*/', ' ', src, flags=re.S))


def header_decls():
    """name -> (return ctypes type, [argument ctypes types]) from the header's C declarations."""
    out = {}
    for ret, name, args in _DECL.findall(_strip_comments(open(HEADER).read())):
        args = ' '.join(args.split())
        types = []
        if args and args != 'void':
            for a in args.split(','):
                a = a.strip()
                if '*' in a:
                    types.append(ctypes.c_void_p)
                    continue
                base = re.sub(r'\b(const|unsigned)\b', ' ', a).split()[0]  # 'long long x' -> 'long'
                assert base in _SCALAR, (name, a)
                types.append(_SCALAR[base])
        out[name] = (_SCALAR[ret], types)
    return out


def header_symbols():
    return sorted(header_decls())


def _bound():
    """every ctypes binding the product uses: _lib.SIGNATURES plus those optim.py sets itself"""
    from dmayolo import _lib
    import dmayolo.optim  # noqa: F401  (binds the optimizer symbols on _lib.lib)
    b = {}
    for name in header_symbols():
        fn = getattr(_lib.lib, name)
        b[name] = (fn.restype, list(fn.argtypes or []))
    return b


def test_header_nonempty():
    assert len(header_symbols()) >= 100


def test_every_definition_is_declared():
    defs = set()
    for f in glob.glob(os.path.join(CSRC, '*.hip')):
        defs |= set(re.findall(r'DMY_API\s+\w+\s+(dmy_\w+)\s*\(', open(f).read()))
    hs = set(header_symbols())
    assert defs == hs, (sorted(defs - hs), sorted(hs - defs))
    assert '#include "../../include/dmayolo.h"' in open(os.path.join(CSRC, 'common.h')).read()


def test_library_exports_every_header_symbol():
    from dmayolo import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_signatures_match_header():
    from dmayolo import _lib
    bound = _bound()
    unbound = [s for s in header_symbols() if s not in _lib.SIGNATURES and s not in _lib.SELF_BOUND]
    assert not unbound, unbound
    bad = []
    for name, (ret, args) in header_decls().items():
        bret, bargs = bound[name]
        if bret is not ret or len(bargs) != len(args) or any(a is not b for a, b in zip(args, bargs)):
            bad.append((name, ret.__name__, [a.__name__ for a in args], getattr(bret, '__name__', bret),
                        [a.__name__ for a in bargs]))
    assert not bad, bad
    stale = [s for s in _lib.SIGNATURES if s not in header_decls()]
    assert not stale, stale


@pytest.mark.skipif(not shutil.which(os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')), reason='hipcc absent')
def test_mismatched_definition_fails_to_compile(tmp_path):
    """a definition whose argument list drifts from the header (long -> int) is a compile error, a matching one is not"""
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')

    def syntax(body):
        src = tmp_path / 'probe.hip'
        src.write_text(f'#include "{os.path.join(CSRC, "common.h")}"\n{body}\n')
        return subprocess.run([hipcc, '--offload-arch=gfx950', '-std=c++17', '-fsyntax-only', str(src)],
                              capture_output=True, text=True)
    good = syntax('DMY_API int dmy_bn_partial_rows(long M) { return (int)M; }')
    assert good.returncode == 0, good.stderr[-2000:]
    bad = syntax('DMY_API int dmy_bn_partial_rows(int M) { return M; }')
    assert bad.returncode != 0 and 'conflicting types' in bad.stderr, bad.stderr[-2000:]


def test_size_queries_cpu_only():
    from dmayolo import _lib
    assert _lib.lib.dmy_conv_fwd_partial_rows(1000, 32) == 2 * ((1000 + 63) // 64)
    assert _lib.lib.dmy_bn_partial_rows(10) == 1
