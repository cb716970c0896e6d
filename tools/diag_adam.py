"""Diagnostic: packed Adam (optim.Adam) vs the plain multi-tensor kernel, per tensor and step."""
import torch
from relativisticgan_amd import kernels as K
from relativisticgan_amd.optim import Adam

DEV = "cuda"
torch.manual_seed(21)
g4, gt = K.ConvGeom(4, 2, 1, False), K.ConvGeom(4, 2, 1, True)
conv = torch.nn.Parameter(torch.randn(256, 128, 4, 4, device=DEV) * 0.05)
vec = torch.nn.Parameter(torch.randn(256, device=DEV))
x = torch.randn(2, 128, 16, 16, device=DEV).contiguous(memory_format=torch.channels_last)
K.conv_fwd(x, conv, g4, cache=True)
for with_layout in (False, True):
    params = [conv, vec] if with_layout else [torch.nn.Parameter(conv.detach().clone()), vec]
    for p in params:
        p.grad = torch.randn_like(p) * 1e-3
    twins = [torch.nn.Parameter(p.detach().clone()) for p in params]
    for p, q in zip(params, twins):
        q.grad = p.grad.clone()
    opt, ref = Adam(params, lr=1e-3, betas=(0.5, 0.999)), Adam(twins, lr=1e-3, betas=(0.5, 0.999))
    for step in range(2):
        opt.step()
        hyper, _, dstep = ref._group_dev(0, ref.param_groups[0], DEV, ref.state.get(twins[0]) or None)
        for q in twins:
            st = ref.state[q]
            if not st:
                st["step"] = torch.tensor(0.0)
                st["exp_avg"] = torch.zeros_like(q)
                st["exp_avg_sq"] = torch.zeros_like(q)
        K.adam(twins, [q.grad for q in twins], [ref.state[q]["exp_avg"] for q in twins],
               [ref.state[q]["exp_avg_sq"] for q in twins], hyper, dstep)
        for q in twins:
            ref.state[q]["step"] += 1
        torch.cuda.synchronize()
        print("layout", with_layout, "step", step, "dev steps", opt._dev[0][2].item(), dstep.item(), flush=True)
        for i, (p, q) in enumerate(zip(params, twins)):
            d = (p.detach() - q.detach()).abs()
            print("  param", i, tuple(p.shape), "max|dp|", d.max().item(), "n diff", int((d > 0).sum()),
                  "m eq", torch.equal(opt.state[p]["exp_avg"], ref.state[q]["exp_avg"]),
                  "v eq", torch.equal(opt.state[p]["exp_avg_sq"], ref.state[q]["exp_avg_sq"]), flush=True)
