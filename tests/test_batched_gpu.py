"""The G step's batched D pass (--rgan_batch_G): [D(G(z)); D(x)] as one pass over 2B samples
with per-call BatchNorm and the backward over the D(G(z)) rows only (GLI:673-707 run D(fake)
with a graph, then D(x) of a fresh real batch without one).

* batched == the separate calls, from the same seed and device draws: the G step's outputs,
  loss and G's gradients (before the optimizer step) and D's BN running statistics agree to
  fp32 summation-order differences (the batched GEMMs split K differently);
* the laid-out path (G writes its output and the gather its images into one buffer, no
  concatenation) under HIP-graph replay == eager iterations, bitwise (device RNG: replays
  draw fresh numbers, as eager iterations do).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(kind, batch_G, **kw):
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.train import Trainer, synthetic_images
    cfg = dict(loss_D=kind, image_size=32, batch_size=8, G_h_size=16, D_h_size=16, seed=3, print_every=10 ** 9,
               rgan_rng="device", rgan_batch_G=batch_G)
    cfg.update(kw)
    return Trainer(make_param(**cfg), synthetic_images(64, 32, device="cuda"))


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("kind", [5, 6, 7, 8])
def test_batched_G_step_matches_separate_calls(kind):
    got = {}
    for batch_G in (True, False):
        t = _trainer(kind, batch_G)
        assert t.batch_G == batch_G
        rec = {}

        def hook(tag, r, t=t, rec=rec):
            if tag == "G":
                rec.update({k: v.detach().clone() for k, v in r.items() if torch.is_tensor(v)})
                rec.update({"grad." + n: q.grad.detach().clone() for n, q in t.G.named_parameters()})

        t.iteration(0, hooks=hook)
        torch.cuda.synchronize()
        rec.update({"D." + k: v.detach().clone() for k, v in t.D.state_dict().items() if "running" in k})
        got[batch_G] = rec
    a, b = got[True], got[False]
    assert set(a) == set(b)
    for k in sorted(b):
        if k in ("z", "x"):
            assert torch.equal(a[k], b[k]), k  # same device draws, same order
            continue
        tol = 2e-4 if k.startswith("grad.") else 2e-5
        assert _rel(a[k], b[k]) < tol, (kind, k, _rel(a[k], b[k]))


def _state(t):
    out = {f"G.{k}": v.detach().clone() for k, v in t.G.state_dict().items()}
    out.update({f"D.{k}": v.detach().clone() for k, v in t.D.state_dict().items()})
    for name, opt in (("optG", t.optG), ("optD", t.optD)):
        for i, st in enumerate(opt.state.values()):
            out[f"{name}.{i}.m"] = st["exp_avg"].detach().clone()
            out[f"{name}.{i}.v"] = st["exp_avg_sq"].detach().clone()
    return out


def test_batched_G_step_graph_replay_matches_eager():
    A, B = _trainer(7, True), _trainer(7, True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        A.iteration(1)
        B.iteration(1)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        B.iteration(2)
    for j in range(1, 4):
        with torch.cuda.stream(side):
            A.iteration(1 + j)
            graph.replay()
        torch.cuda.synchronize()
        sa, sb = _state(A), _state(B)
        bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
        assert not bad, (j, bad[:8])
