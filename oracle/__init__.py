"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the DMA-YOLO hot path.

A from-scratch fp32 PyTorch-CPU restatement of the reference algorithms
(Yaling-Li/DMA-YOLO, models/common.py, models/yolo.py, utils/loss.py, utils/metrics.py,
utils/general.py).  It is the checker, never the thing measured or shipped:
only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.

Parity pin: every function here is checked against golden vectors captured from the
reference itself in this container (tools/gen_golden.py -> tests/golden/*.npz), see
tests/test_oracle_golden.py.  The one third-party boundary, torchvision.ops.nms, is
restated from torchvision's documented CPU algorithm.
"""
