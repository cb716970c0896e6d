"""Where do activation-sign flips happen (parity test, arch-1 config)?"""
import sys
sys.path.insert(0, ".")
import torch
from tests.test_parity_gpu import oracle_steps, gpu_step, _feed
from tests.oracle_replay import param_for, dataset_for
from relativisticgan_amd.train import Trainer

name = sys.argv[1] if len(sys.argv) > 1 else "rahinge_arch1"
p, init, steps = oracle_steps(name, 1)
p.rgan_rng = "host"
t = Trainer(p, dataset_for(name).to("cuda"))
st = steps[0]
got = gpu_step(t, st)
from oracle.reference_cpu import Trainer as OT
pre_acts = []
tt = OT(param_for(name), dataset_for(name), dtype=torch.float64)
tt.G.load_state_dict(st["pre"]["G"]); tt.D.load_state_dict(st["pre"]["D"])
names = {}
hooks = []
for net, nn_ in ((tt.G, "G"), (tt.D, "D")):
    for mname, m in net.named_modules():
        if isinstance(m, (torch.nn.ReLU, torch.nn.LeakyReLU, torch.nn.SELU)):
            hooks.append(m.register_forward_pre_hook(
                lambda mod, inp, key=f"{nn_}.{mname}": pre_acts.append((key, inp[0].detach().clone()))))
tt.iteration(0, feed={k: v.double() for k, v in _feed(st).items()})
for h in hooks:
    h.remove()
ours = [m for _, m in got["masks"]]  # (net tag, mask) entries
print(len(ours), len(pre_acts))
for k, ((key, z), m) in enumerate(zip(pre_acts, ours)):
    e = (z > 0)
    diff = (e != m)
    n = int(diff.sum())
    if n:
        zz = z[diff].abs()
        print(f"call {k:3d} {key:22s} shape {tuple(z.shape)} flips {n:5d}  max|z| at flips {zz.max().item():.3e}  "
              f"min {zz.min().item():.3e}  rms z {z.pow(2).mean().sqrt().item():.3e}  zeros_exact {(z == 0).sum().item()}")
