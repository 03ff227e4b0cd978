"""Graph-replayed inference (detect.py:175-243's model call, SURVEY.md §8(d) "detect p50 ms incl. NMS").

At batch 1 the eval forward is ~60 small kernel launches, and issuing them from Python costs more than
running them.  GraphedDetector records one eval forward (every launch goes to torch's current stream,
ctypes launches included) into a HIP graph with a static input buffer and replays it with a single
launch.  `detect()` records the NMS kernels into the same graph (utils.general.nms_launch: no host read
inside), so a detection is one graph launch and one host read of the keep counts (variable-length output,
SURVEY §8(b)); eager NMS issued its 5-7 launches from Python after the forward, ~100-170 us of host gaps
per call.  When some image had more candidates than the recorded sort capacity (the read says so) the call
falls back to the eager NMS at the exact capacity once, and the next call re-records at that capacity.

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

    def _capture_detect(self, x, nms_args):
        from .utils.general import nms_prepare, nms_launch, nms_buffers
        self._capture(x)  # warm-up forwards fill every per-layer cache; the forward-only graph stays usable
        z = self.static_out[0]
        pred, plan = nms_prepare(z, **nms_args)  # NMS plan from the recorded output's shape (the cap hint)
        # the detect graph owns its input buffer, its state key and its NMS counter / pinned counts: __call__ may
        # re-record the forward-only graph (and replace static_in) without this graph noticing otherwise
        self.dstatic_in = x.clone()
        bufs = nms_buffers(x.device, x.shape[0])
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            for _ in range(self.warmup):
                nms_launch(pred, plan, bufs=bufs)
        torch.cuda.synchronize()
        self.dgraph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.dgraph, stream=cs), torch.no_grad():
            out = self.model(self.dstatic_in)
            dpred = out[0].detach().float().contiguous()  # nms_prepare's conversion (the plan, cls_ok included, is made)
            self.dstate = (out, plan, plan['cap']) + nms_launch(dpred, plan, bufs=bufs)
        self.dbufs = bufs
        self.dkey = (self._state_key(x), tuple(sorted((k, str(v)) for k, v in nms_args.items())), plan['cap'])

    @torch.no_grad()
    def detect(self, x, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False, multi_label=False,
               max_det=300):
        """eval forward + non_max_suppression (utils/general.py:633-725 arguments, merge=False) as one graph replay:
        returns (list of (k, 6) detections per image, (z, per-level outputs)).  The detections are views of the
        graph's static output buffer, valid until the next call (as the forward's outputs are)."""
        from .utils.general import nms_finish, non_max_suppression, _CAP_HINT
        if self.model.training:
            self.model.eval()
        args = dict(conf_thres=conf_thres, iou_thres=iou_thres, classes=classes, agnostic=agnostic,
                    multi_label=multi_label, max_det=max_det)
        key = tuple(sorted((k, str(v)) for k, v in args.items()))
        cur = getattr(self, 'dkey', None)
        if (cur is None or self._state_key(x) != cur[0] or cur[1] != key or
                _CAP_HINT.get(self.dstate[1]['key'], cur[2]) != cur[2]):
            self._capture_detect(x, args)
        self.dstatic_in.copy_(x)
        self.dgraph.replay()
        out, plan, cap, cnt, dets = self.dstate
        res = nms_finish(plan, cap, cnt, dets)
        if res is None:  # more candidates than the recorded capacity: this call eager at the exact one, next re-records
            res = non_max_suppression(out[0], **args)
        return res, out

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
