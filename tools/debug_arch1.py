"""Debug: per-parameter G gradient errors (ours / torch fp32 vs fp64) for arch 1."""
import copy
import sys
sys.path.insert(0, ".")
import torch
from oracle.reference_cpu import build_D, build_G, make_param as oparam, weights_init as owi
from relativisticgan_amd.config import make_param
from relativisticgan_amd.nets import DCGAN_D, DCGAN_G

def rel(a, b):
    a = a.detach().double().cpu().reshape(-1); b = b.detach().double().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()

case = dict(arch=1, image_size=32, batch_size=8, z_size=16, loss_D=1, no_batch_norm_D=True)
torch.manual_seed(3)
po = oparam(cuda=False, **case)
Go, Do = build_G(po), build_D(po)
Go.apply(owi); Do.apply(owi)
G = DCGAN_G(make_param(**case)); G.load_state_dict(Go.state_dict()); G.cuda()
Go64, Go32 = copy.deepcopy(Go).double(), copy.deepcopy(Go)
z = torch.randn(8, 16, 1, 1)
out64 = Go64(z.double()); out32 = Go32(z); fake = G(z.cuda())
g = torch.randn_like(out64) * 1e-3
fake.backward(g.float().cuda()); out32.backward(g.float()); out64.backward(g)
for (n, q), (_, q32), (_, q64) in zip(G.named_parameters(), Go32.named_parameters(), Go64.named_parameters()):
    print(f"{n:25s} ours {rel(q.grad, q64.grad):.2e}  torch32 {rel(q32.grad, q64.grad):.2e}  |g| {q64.grad.norm():.3e}")
for (n, b), (_, b64) in zip(G.named_buffers(), Go64.named_buffers()):
    if "running" in n:
        print(n, f"{rel(b, b64):.2e}")
