"""Debug: arch-1 G grads with the D-derived upstream gradient of test_modules_gpu."""
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
D = DCGAN_D(make_param(**case)); D.load_state_dict(Do.state_dict()); D.cuda()
Go64, Go32 = copy.deepcopy(Go).double(), copy.deepcopy(Go)
Do64 = copy.deepcopy(Do).double()
z = torch.randn(8, 16, 1, 1)
out64 = Go64(z.double()); out32 = Go32(z); fake = G(z.cuda())
x64 = out64.detach().clone().requires_grad_(True)
y64 = Do64(x64)
gy = torch.randn(8)
y64.backward(gy.double())
g = x64.grad.detach()
print("upstream |g|", g.norm().item(), "per-sample norms", g.flatten(1).norm(dim=1))
# per-channel mean of g relative to its norm (BN null-space content)
fake.backward(g.float().cuda()); out32.backward(g.float()); out64.backward(g)
for (n, q), (_, q32), (_, q64) in zip(G.named_parameters(), Go32.named_parameters(), Go64.named_parameters()):
    print(f"{n:25s} ours {rel(q.grad, q64.grad):.2e}  torch32 {rel(q32.grad, q64.grad):.2e}  |g| {q64.grad.norm():.3e}")
