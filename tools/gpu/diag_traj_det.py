"""Is the device-run fp32 oracle trajectory deterministic under torch.use_deterministic_algorithms?  Runs the oracle
trajectory of each trajectory case for a few steps twice (warn_only: the warnings name the ops without a deterministic
implementation) and reports whether the loss curves are bit-identical; then the fp64 CPU-vs-GPU first-step pin."""
import os
import sys
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd'), os.path.join(ROOT, 'tests')]
os.environ.setdefault('CUBLAS_WORKSPACE_CONFIG', ':4096:8')
import torch  # noqa: E402
import trajectory_util as tu  # noqa: E402
from test_gpu_trajectory import CASES  # noqa: E402
from dmayolo.synthetic import HYP_VISDRONE, scaled_hyp  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
torch.use_deterministic_algorithms(True, warn_only=True)
for case, (yml, gw, gd, img, bs, nb, _, nc, fp8, _) in CASES.items():
    cfg = tu.load_cfg(yml, gw, gd)
    batches = tu.make_batches(nb, bs, img, nc)
    m, sd = tu.product_model(cfg, nc, fp8=False)
    hyp = scaled_hyp(HYP_VISDRONE, nc, img, m.model[-1].nl)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        a, _ = tu.oracle_trajectory(cfg, nc, sd, batches, hyp, steps, None)
        b, _ = tu.oracle_trajectory(cfg, nc, sd, batches, hyp, steps, None)
    ops = sorted({str(x.message).split(' does not have')[0][:90] for x in w if 'deterministic' in str(x.message)})
    print(f'{case}: identical={torch.equal(a, b)} max|diff|={float((a - b).abs().max()):.3e} nondeterministic ops: {ops}',
          flush=True)
    print(f'  fp64 pin (loss, outputs, grad): {tu.pin_device_oracle(cfg, nc, sd, batches[0], hyp)}', flush=True)
