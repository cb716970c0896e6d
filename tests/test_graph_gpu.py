"""HIP-graph replay of a training iteration (bench.py's timed mode) == eager iterations.

bench.py captures one Trainer.iteration as a HIP graph and replays it (no Python/ctypes per
launch).  Two trainers from the same seed run the same fed inputs: A eagerly, B by replays
of one captured iteration whose static input buffers are refilled before each replay.  The
kernels are deterministic, so parameters, optimizer state and BN/spectral buffers must
agree bitwise after every step.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

CFGS = {
    "ralsgan": dict(loss_D=7),
    "wgangp": dict(loss_D=3),
    "rahinge_spectral": dict(loss_D=8, spectral=True),
}


def _trainer(cfg):
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.train import Trainer, synthetic_images
    p = make_param(image_size=32, batch_size=8, G_h_size=16, D_h_size=16, seed=1, print_every=10 ** 9,
                   rgan_rng="device", **cfg)
    return Trainer(p, synthetic_images(64, 32, device="cuda"))


def _feed(t, gen):
    p = t.p
    f = {"x_D": torch.rand(8, 3, 32, 32, device="cuda", generator=gen) * 2 - 1,
         "z_D": torch.randn(8, p.z_size, 1, 1, device="cuda", generator=gen),
         "z_G": torch.randn(8, p.z_size, 1, 1, device="cuda", generator=gen),
         "x_G": torch.rand(8, 3, 32, 32, device="cuda", generator=gen) * 2 - 1,
         "u": torch.rand(8, 1, 1, 1, device="cuda", generator=gen)}
    return f


def _state(t):
    out = {f"G.{k}": v.detach().clone() for k, v in t.G.state_dict().items()}
    out.update({f"D.{k}": v.detach().clone() for k, v in t.D.state_dict().items()})
    for name, opt in (("optG", t.optG), ("optD", t.optD)):
        for i, (p, st) in enumerate(opt.state.items()):
            out[f"{name}.{i}.m"] = st["exp_avg"].detach().clone()
            out[f"{name}.{i}.v"] = st["exp_avg_sq"].detach().clone()
    return out


@pytest.mark.parametrize("name", sorted(CFGS))
def test_graph_replay_matches_eager(name):
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    A, B = _trainer(CFGS[name]), _trainer(CFGS[name])
    feeds = [_feed(A, gen) for _ in range(4)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        A.iteration(1, feed=feeds[0])
        B.iteration(1, feed=feeds[0])
    static = {k: v.clone() for k, v in feeds[0].items()}
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        B.iteration(2, feed=static)
    for j in range(1, 4):
        with torch.cuda.stream(side):
            A.iteration(1 + j, feed=feeds[j])
            for k, v in feeds[j].items():
                static[k].copy_(v)
        with torch.cuda.stream(side):
            graph.replay()
        torch.cuda.synchronize()
        sa, sb = _state(A), _state(B)
        bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
        assert not bad, (name, j, bad[:8])
