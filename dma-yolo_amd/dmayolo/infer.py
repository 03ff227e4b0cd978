"""Graph-replayed inference (detect.py:175-243's model call, SURVEY.md §8(d) "detect p50 ms incl. NMS").

At batch 1 the eval forward is ~60 small kernel launches, and issuing them from Python costs more than
running them.  GraphedDetector records one eval forward (every launch goes to torch's current stream,
ctypes launches included) into a HIP graph with a static input buffer and replays it with a single
launch.  NMS stays outside the graph: it reads one candidate count back to the host (variable-length
output).

The graph bakes in the prepped weights and eval BN coefficients of the moment of capture: a call
re-captures automatically when a parameter / buffer changed since (torch _version or
functional.PARAM_GEN for our in-place optimizer / EMA / BN kernels), when the input shape changes, or
when the model switched to train mode.
"""
import torch

from . import functional as Fn


class GraphedDetector:
    def __init__(self, model, warmup=2):
        self.model = model
        self.warmup = warmup
        self.graph = None
        self.key = None

    def _state_key(self, x):
        return (tuple(x.shape), x.dtype, x.device, Fn.PARAM_GEN[0], sum(t._version for t in self._ts))

    def _capture(self, x):
        self.model.eval()
        self._ts = list(self.model.parameters()) + list(self.model.buffers())
        self.static_in = x.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.no_grad():
            for _ in range(self.warmup):  # fills every per-layer cache (prepped weights, BN coefficients, grids)
                self.model(self.static_in)
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph), torch.no_grad():
            self.static_out = self.model(self.static_in)
        self.key = self._state_key(x)

    @torch.no_grad()
    def __call__(self, x):
        """eval forward of `x` (same shape / dtype each call for replay): returns (z, per-level outputs)"""
        if self.model.training:
            self.model.eval()
        if self.graph is None or self._state_key(x) != self.key:
            self._capture(x)
        self.static_in.copy_(x)
        self.graph.replay()
        return self.static_out
