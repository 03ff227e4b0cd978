"""dmayolo — MI355X-native (gfx950) DMA-YOLO detection path.

Import layout mirrors the reference's plugin boundary:
  dmayolo.models.yolo   (Model, parse_model, Detect)     <- models/yolo.py
  dmayolo.models.common (Conv, C3, SCConv, CA, ...)       <- models/common.py, models/cspcm.py
  dmayolo.utils.loss    (ComputeLoss)                     <- utils/loss.py
  dmayolo.utils.general (non_max_suppression, ...)        <- utils/general.py
"""
from . import _lib  # noqa: F401  (fails loudly when the HIP library is missing)

__version__ = '0.1.0'
