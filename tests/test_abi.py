"""CPU: the C-ABI library loads and exports every symbol include/dmayolo.h declares (no compute)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, 'include', 'dmayolo.h')).read()
    return sorted(set(re.findall(r'^\s*(?:int|long)\s+(dmy_\w+)\s*\(', src, re.M)))


def test_header_nonempty():
    assert len(header_symbols()) > 40


def test_library_exports_every_header_symbol():
    from dmayolo import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_bindings_cover_header():
    from dmayolo import _lib
    import dmayolo.optim  # noqa: F401  (binds the optimizer symbols)
    extra = {'dmy_chunk_size', 'dmy_sgd', 'dmy_adam', 'dmy_ema', 'dmy_amp_check', 'dmy_amp_update'}
    unbound = [s for s in header_symbols() if s not in _lib.SIGNATURES and s not in extra]
    assert not unbound, unbound


def test_size_queries_cpu_only():
    from dmayolo import _lib
    assert _lib.lib.dmy_conv_fwd_partial_rows(1000, 32) == 2 * ((1000 + 63) // 64)
    assert _lib.lib.dmy_bn_partial_rows(10) == 1
