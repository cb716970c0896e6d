"""Checkpoint parity (GLI:536-552 load, GLI:733-747 save) in both directions.

reference -> build: ``tests/golden/ralsgan_ckpt_state_01.pth`` was written by the
  unmodified reference itself (``--gen_every 2 --save True`` after two iterations,
  tests/golden/make_golden.py; pinned bitwise against the oracle's ``checkpoint()`` dict by
  tests/test_oracle_golden.py).  ``train.main --load`` resumes it on the GPU for one
  iteration, and the oracle resumed from the same file runs the same iteration.  Both runs
  re-seed and draw exactly as the reference does after a resume (GLI:537-560).
build -> reference: the GPU trainer's ``state()`` file loads into the oracle (strict
  state_dict keys, torch Adam state) and the next iteration matches the GPU's own.

Tolerances (as the step-parity tests): errD / errG rel 1e-4; parameters after the step
max|dp| <= 2.02 x the largest Adam update in the tensor plus 1e-7.
"""
import os
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu

ARGS = dict(loss_D=7, image_size=32, batch_size=8, z_size=16, G_h_size=8, D_h_size=8, seed=1)


def _oracle(extra=None):
    from oracle.reference_cpu import Trainer, make_param, synthetic_images
    torch.set_num_threads(4)
    kw = dict(ARGS, cuda=False, print_every=1000, gen_extra_images=0)
    kw.update(extra or {})
    return Trainer(make_param(**kw), synthetic_images(64, 32))


def _check_step(pre, ours, ref, what):
    for side in ("G", "D"):
        a, b, p0 = ours[side], ref[side], pre[side]
        for k in b:
            if k.endswith("num_batches_tracked"):
                assert int(a[k]) == int(b[k]), (what, side, k)
                continue
            x, y = a[k].double().cpu(), b[k].double()
            if "running" in k:
                assert ((x - y).norm() / y.norm()).item() < 1e-4, (what, side, k)
                continue
            upd = (y - p0[k].double()).abs().max().item()
            assert (x - y).abs().max().item() <= 2.02 * upd + 1e-7, (what, side, k)


REF_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ralsgan_ckpt_state_01.pth")


def test_resume_reference_checkpoint_through_cli():
    from oracle.reference_cpu import load_checkpoint
    from relativisticgan_amd.train import main
    root = tempfile.mkdtemp()
    path = REF_FILE                                   # written by the reference (GLI:737)
    ck = torch.load(path, weights_only=True)
    pre = {"G": {k: v.clone() for k, v in ck["G_state"].items()},
           "D": {k: v.clone() for k, v in ck["D_state"].items()}}
    # the reference resumed: re-seeded build, load, iteration 2 (GLI:537-560)
    ref2 = _oracle()
    it0, _ = load_checkpoint(ref2, torch.load(path, weights_only=True))
    ref2.iteration(it0)
    # the build resumed through its CLI (--load), one iteration
    argv = ["--loss_D", "7", "--image_size", "32", "--batch_size", "8", "--z_size", "16", "--G_h_size", "8",
            "--D_h_size", "8", "--seed", "1", "--n_iter", "3", "--print_every", "1000", "--gen_every", "1000",
            "--gen_extra_images", "0", "--save", "False", "--output_folder", os.path.join(root, "out"),
            "--extra_folder", os.path.join(root, "extra"), "--rgan_synthetic", "64", "--load", path]
    t = main(argv)
    torch.cuda.synchronize()
    for mine, want in ((t.errD, ref2.errD), (t.errG, ref2.errG)):
        assert abs(mine.item() - want.item()) <= 1e-4 * abs(want.item())
    _check_step(pre, {"G": t.G.state_dict(), "D": t.D.state_dict()},
                {"G": ref2.G.state_dict(), "D": ref2.D.state_dict()}, "ref->build")
    # optimizer state continued from the file: step counts 2 -> 3
    st = t.optD.state_dict()["state"]
    assert all(float(v["step"]) == 3.0 for v in st.values())


def test_build_checkpoint_loads_into_reference():
    from oracle.reference_cpu import load_checkpoint, make_param, synthetic_images
    from relativisticgan_amd.config import make_param as build_param
    from relativisticgan_amd.train import Trainer
    root = tempfile.mkdtemp()
    t = Trainer(build_param(print_every=1000, **ARGS), synthetic_images(64, 32).cuda())
    for i in range(2):
        t.iteration(i)
    path = os.path.join(root, "state_01.pth")
    torch.save(t.state(2, 1), path)                   # the build's file
    ck = torch.load(path, weights_only=True, map_location="cpu")
    ref = _oracle()
    it0, cur = load_checkpoint(ref, ck)               # strict keys, torch Adam / scheduler state
    assert (it0, cur) == (2, 1)
    pre = {"G": {k: v.clone() for k, v in ref.G.state_dict().items()},
           "D": {k: v.clone() for k, v in ref.D.state_dict().items()}}
    # the same draws on both sides: teacher-force the build's iteration 2 with the oracle's
    feed = {}
    rec = ref.iteration(it0)
    feed = {"x_D": rec.D["x"], "z_D": rec.D["z"], "z_G": rec.G["z"], "x_G": rec.G["x"]}
    t.iteration(it0, feed={k: v.cuda() for k, v in feed.items()})
    torch.cuda.synchronize()
    for mine, want in ((t.errD, ref.errD), (t.errG, ref.errG)):
        assert abs(mine.item() - want.item()) <= 1e-4 * abs(want.item())
    _check_step(pre, {"G": t.G.state_dict(), "D": t.D.state_dict()},
                {"G": ref.G.state_dict(), "D": ref.D.state_dict()}, "build->ref")
