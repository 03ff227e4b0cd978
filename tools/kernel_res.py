"""Print register / LDS / spill metadata of kernels in the built library (gfx950 code object inside .hip_fatbin).

python tools/kernel_res.py [name-substring ...]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'libdmayolo_hip.so')
LLVM = '/opt/rocm/lib/llvm/bin'


def code_objects(path):
    data = open(path, 'rb').read()
    magic = b'__CLANG_OFFLOAD_BUNDLE__'
    pos = 0
    while True:
        i = data.find(magic, pos)
        if i < 0:
            return
        n = struct.unpack_from('<Q', data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from('<QQQ', data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if 'gfx950' in triple:
                yield data[i + off:i + off + size]
        pos = i + 1


def main():
    pats = sys.argv[1:]
    with tempfile.TemporaryDirectory() as d:
        for ci, co in enumerate(code_objects(LIB)):
            f = os.path.join(d, f'co{ci}.o')
            open(f, 'wb').write(co)
            out = subprocess.run([f'{LLVM}/llvm-readelf', '--notes', f], capture_output=True, text=True).stdout
            for blk in re.split(r'\n  - \.agpr_count', out)[1:]:
                name = re.search(r'\.name:\s+(\S+)', blk)
                if not name or (pats and not any(p in name.group(1) for p in pats)):
                    continue
                dem = subprocess.run(['c++filt', name.group(1)], capture_output=True, text=True).stdout
                vals = {k: re.search(rf'\.{k}:\s+(\d+)', blk) for k in
                        ('vgpr_count', 'sgpr_count', 'vgpr_spill_count', 'sgpr_spill_count', 'group_segment_fixed_size',
                         'private_segment_fixed_size')}
                agpr = re.match(r':\s+(\d+)', blk)
                print(dem.strip()[:110], {k: int(v.group(1)) for k, v in vals.items() if v},
                      'agpr', agpr.group(1) if agpr else '?')


if __name__ == '__main__':
    main()
