"""Product-free reproduction 2 for the rocprofv3 --pmc SIGSEGV: torch kernels only, dispatched the way a training step
dispatches them -- forward on the main thread, backward on the autograd engine's device thread, and a second stream
joined by events (HIP writes barrier packets ahead of the dispatches).  A small conv net trained for `steps` steps.
Run under rocprofv3 --kernel-trace --pmc FETCH_SIZE -- python tools/gpu/pmc_wrap_repro2.py [steps]"""
import sys

import torch

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
torch.manual_seed(0)
net = torch.nn.Sequential(*[m for _ in range(12) for m in (torch.nn.Conv2d(32, 32, 3, padding=1),
                                                          torch.nn.BatchNorm2d(32), torch.nn.SiLU())]).cuda()
opt = torch.optim.SGD(net.parameters(), lr=1e-3, momentum=0.9)
x = torch.randn(4, 32, 32, 32, device='cuda')
side = torch.cuda.Stream()
for i in range(steps):
    y = net(x)
    ev = torch.cuda.Event()
    ev.record()
    with torch.cuda.stream(side):
        side.wait_event(ev)
        aux = (y.detach() * 2).sum()
    torch.cuda.current_stream().wait_stream(side)
    loss = y.square().mean() + 0 * aux
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)
    if i % 50 == 49:
        torch.cuda.synchronize()
        print(f'step {i + 1}: loss {float(loss):.4f}', flush=True)
torch.cuda.synchronize()
print('done')
