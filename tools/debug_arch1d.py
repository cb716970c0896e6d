"""Isolate layer 3 (ConvT 128->64 + BN + ReLU) backward of arch-1 G on the failing data."""
import copy, sys
sys.path.insert(0, ".")
import torch
import torch.nn.functional as F
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
# fp64 activations and grads around block 2 (model 6,7,8): input = model[5] output
h = Go64.dense(z.double().view(-1, 16)).view(-1, 512, 4, 4)
acts = [h]
for m in Go64.model:
    h = m(h); h.retain_grad(); acts.append(h)
h.backward(g)
xin = acts[6].detach()            # input of ConvT model.6 (post-ReLU of block 1)
gout = acts[9].grad.detach()       # grad at model.8 output (post-ReLU block 2)
conv, bn = Go64.model[6], Go64.model[7]
W64, b64 = conv.weight.detach(), conv.bias.detach()
gam, bet = bn.weight.detach(), bn.bias.detach()
def layer(x, W, b, gm, bt):
    y = F.conv_transpose2d(x, W, b, stride=2, padding=1)
    return F.relu(F.batch_norm(y, None, None, gm, bt, training=True, eps=1e-5)), y
# exact
xe = xin.clone().requires_grad_(True)
ae, ye = layer(xe, W64, b64, gam, bet); ye.retain_grad(); ae.backward(gout)
# torch fp32
x3 = xin.float().clone().requires_grad_(True)
a3, y3 = layer(x3, W64.float(), b64.float(), gam.float(), bet.float()); y3.retain_grad(); a3.backward(gout.float())
# ours: ConvLayerFn via plan layer 3
L3 = G._plan[3]
xo = xin.float().cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
ao = L3.run(xo, True)
ao.backward(gout.float().cuda().contiguous(memory_format=torch.channels_last))
print("fwd out: ours", f"{rel(ao, ae):.2e}", "torch32", f"{rel(a3, ae):.2e}")
print("dx:      ours", f"{rel(xo.grad, xe.grad):.2e}", "torch32", f"{rel(x3.grad, xe.grad):.2e}", "|dx|", xe.grad.norm().item())
# component test: BN backward alone from exact y and exact grad
yy = ye.detach()
st = K.bn_stats(yy.float().cuda().contiguous(memory_format=torch.channels_last), 1e-5, 0.1)
dyo, dgo, dbo = K.bn_backward(gout.float().cuda().contiguous(memory_format=torch.channels_last),
                              yy.float().cuda().contiguous(memory_format=torch.channels_last), st,
                              gam.float().cuda(), bet.float().cuda(), "relu", 0.0)
y3b = yy.float().clone().requires_grad_(True); gm3 = gam.float().clone().requires_grad_(True)
F.relu(F.batch_norm(y3b, None, None, gm3, bet.float(), training=True, eps=1e-5)).backward(gout.float())
print("BN dy:   ours", f"{rel(dyo, ye.grad):.2e}", "torch32", f"{rel(y3b.grad, ye.grad):.2e}", "|dy|", ye.grad.norm().item(),
      "|g|", gout.norm().item())
# dgrad alone from exact dy
dxo = K.conv_dgrad(ye.grad.float().cuda().contiguous(memory_format=torch.channels_last), W64.float().cuda(),
                   K.ConvGeom(4, 2, 1, True), tuple(xin.shape))
dx3 = torch.nn.grad.conv_transpose2d_input if hasattr(torch.nn.grad, "conv_transpose2d_input") else None
xx = xin.float().clone().requires_grad_(True)
F.conv_transpose2d(xx, W64.float(), None, stride=2, padding=1).backward(ye.grad.float())
xx64 = xin.clone().requires_grad_(True)
F.conv_transpose2d(xx64, W64, None, stride=2, padding=1).backward(ye.grad)
print("dgrad:   ours", f"{rel(dxo, xx64.grad):.2e}", "torch32", f"{rel(xx.grad, xx64.grad):.2e}")
# stats precision
m64 = yy.mean((0, 2, 3)); v64 = yy.var((0, 2, 3), unbiased=False)
print("mean rel", f"{rel(st[:64], m64):.2e}", "invstd rel", f"{rel(st[64:], 1/torch.sqrt(v64+1e-5)):.2e}")
print("mean/std ratio", (m64.abs() / v64.sqrt()).max().item())
