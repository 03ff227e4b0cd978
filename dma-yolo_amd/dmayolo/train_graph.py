"""Graph-replayed training step (train.py:400-454 on one GPU).

A yolov5s@640 bs64 step is ~670 kernels; issued one by one they leave the GPU idle between dependent
launches for a few microseconds each (~2 ms per step measured in the rocprofv3 trace).
GraphedTrainStep records forward + loss + backward once into a HIP graph (torch.cuda.CUDAGraph; the
ctypes launches go to the capturing stream) and replays it; optimizer.step() and the EMA update stay
eager, because their scalars (lr / momentum from the warmup and LambdaLR schedules, the EMA decay)
change between steps and are kernel arguments.

Static-shape contract and how it is kept general:
  * images: one shape per graph; a new shape re-captures.
  * targets: copied into a zero-padded buffer of capacity `tcap` (grown and re-captured when a batch
    has more).  A zero row (w = h = 0) can never match: its anchor ratio max(r, 1/r) is inf, so
    build_targets rejects it for every anchor (utils/loss.py:233-236) -- padding changes nothing.
  * gradients: captured with param.grad unset, so autograd leaves static gradient tensors (the
    weight-gradient arena slices among them) on the parameters; every replay rewrites them.  Do not
    call optimizer.zero_grad(set_to_none=True) between calls: __call__ runs the whole step.
  * the call that (re)captures runs its batch eagerly (a real step, which also warms every per-layer
    cache and the optimizer state); replays start with the next call.
Single process only: the DDP path (world > 1) keeps the eager step.
"""
import torch


class GraphedTrainStep:
    def __init__(self, model, compute_loss, optimizer, ema=None, tcap=256):
        self.model, self.compute_loss, self.optimizer, self.ema = model, compute_loss, optimizer, ema
        self.tcap = tcap
        self.graph = None
        self.shape = None
        self.captures = 0

    def _eager(self, imgs, t):
        self.optimizer.zero_grad(set_to_none=True)
        loss, items = self.compute_loss(self.model(imgs), t)
        loss.backward()
        self.optimizer.step()
        if self.ema is not None:
            self.ema.update(self.model)
        return loss, items

    def _capture(self, imgs, targets):
        nt = targets.shape[0]
        while self.tcap < nt:
            self.tcap *= 2
        dev = imgs.device
        self.static_imgs = imgs.clone()
        self.static_t = torch.zeros((self.tcap, 6), dtype=torch.float32, device=dev)
        self.static_t[:nt].copy_(targets)
        cur = torch.cuda.current_stream()
        s = torch.cuda.Stream()
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            loss, items = self._eager(self.static_imgs, self.static_t)  # this call's real step
            loss, items = loss.detach().clone(), items.detach().clone()
        cur.wait_stream(s)
        self.optimizer.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            sl, si = self.compute_loss(self.model(self.static_imgs), self.static_t)
            sl.backward()
        self.static_loss, self.static_items = sl.detach(), si.detach()
        self.grads = [(q, q.grad) for q in self.model.parameters() if q.grad is not None]
        self.shape = tuple(imgs.shape)
        self.captures += 1
        return loss, items

    def __call__(self, imgs, targets):
        """one training step on (imgs [N, 3, H, W] uint8/float on the GPU, targets [nt, 6] normalised):
        returns (loss [1], items [3]) like ComputeLoss"""
        if not self.model.training:
            self.model.train()
        nt = targets.shape[0]
        if (self.graph is None or tuple(imgs.shape) != self.shape or nt > self.tcap
                or any(q.grad is not g for q, g in self.grads)):  # static gradients detached (zero_grad(None))
            return self._capture(imgs, targets)
        self.static_imgs.copy_(imgs)
        self.static_t.zero_()
        self.static_t[:nt].copy_(targets)
        self.graph.replay()
        self.optimizer.step()
        if self.ema is not None:
            self.ema.update(self.model)
        return self.static_loss, self.static_items
