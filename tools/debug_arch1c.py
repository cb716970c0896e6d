import copy, sys
sys.path.insert(0, ".")
import torch
from oracle.reference_cpu import build_D, build_G, make_param as oparam, weights_init as owi
from relativisticgan_amd.config import make_param
from relativisticgan_amd.nets import DCGAN_D, DCGAN_G
from relativisticgan_amd import kernels as K

def rel(a, b):
    a = a.detach().double().cpu().reshape(-1); b = b.detach().double().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()

case = dict(arch=1, image_size=32, batch_size=8, z_size=16, loss_D=1, no_batch_norm_D=True)
torch.manual_seed(3)
po = oparam(cuda=False, **case)
Go, Do = build_G(po), build_D(po)
Go.apply(owi); Do.apply(owi)
G = DCGAN_G(make_param(**case)); G.load_state_dict(Go.state_dict()); G.cuda()
D = DCGAN_D(make_param(**case))
Go64, Do64 = copy.deepcopy(Go).double(), copy.deepcopy(Do).double()
z = torch.randn(8, 16, 1, 1)
out64 = Go64(z.double())
x64 = out64.detach().clone().requires_grad_(True)
Do64(x64).backward(torch.randn(8).double())
g = x64.grad.detach()
# fp64 intermediates: output of each model child
acts64 = {}
h = Go64.dense(z.double().view(-1, 16)).view(-1, 512, 4, 4)
h.retain_grad(); acts64["dense"] = h
for i, m in enumerate(Go64.model):
    h = m(h); h.retain_grad(); acts64[i] = h
h.backward(g)
# ours: run plan layers manually
hh = z.cuda(); outs = []
for L in G._plan:
    hh = L.run(hh, True); hh.retain_grad(); outs.append(hh)
hh.backward(g.float().cuda())
# plan layer k output corresponds to model index: dense, 2 (after ReLU of block0), 5, 8, 10
idx = ["dense", 2, 5, 8, 10]
for k, o in zip(idx, outs):
    print(k, "act", f"{rel(o, acts64[k]):.2e}", "grad", f"{rel(o.grad, acts64[k].grad):.2e}", f"|grad64| {acts64[k].grad.norm():.3e}")
# now the last BN: compare BN-backward given identical upstream grad (fp64 -> fp32)
L = G._plan[3]
print("layer3 spec", L.spec.geom, L.spec.act, L.spec.bn)
# BN backward of layer 3 in isolation with the fp64 upstream grad
y3 = None
