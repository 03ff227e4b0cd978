"""compare the probe's v_cvt_pk_fp8_f32 bytes with torch's float8_e4m3fn conversion (RNE) of the same floats"""
import numpy as np, torch
raw = open('gpurun_out/probe_cvt.bin', 'rb').read()
n = 4096
x = np.frombuffer(raw[:4 * n], dtype=np.float32)
q = np.frombuffer(raw[4 * n:], dtype=np.uint8)
xc = np.clip(x, -448, 448)
ref = torch.from_numpy(xc.copy()).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
bad = np.nonzero(ref != q)[0]
print('cvt mismatches (clipped inputs):', len(bad), [(float(x[i]), int(q[i]), int(ref[i])) for i in bad[:10]])
big = np.abs(x) > 448
print('out-of-range inputs:', int(big.sum()), 'their bytes:', sorted(set(int(v) for v in q[big]))[:8])
