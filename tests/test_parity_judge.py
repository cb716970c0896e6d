"""CPU checks of the GPU parity judge itself (tests/test_parity_gpu.py).

The mask-forced float64 step must be the exact step whenever the forced signs are the
exact step's own (so "forced" can only differ from "exact" through the GPU's branch
choices), and the teacher-forcing state must survive being loaded twice (torch's Adam
bumps the loaded ``step`` tensors in place).
"""
import pytest
import torch

from tests.test_parity_gpu import _rel, oracle_exact_step, oracle_steps, per_net


@pytest.mark.parametrize("name", ["ralsgan", "ralsgan_selu", "wgangp", "rahinge_arch1", "sgan_pac2_gp"])
def test_forced_with_own_masks_is_exact(name):
    _, _, steps = oracle_steps(name, 2)
    st = steps[1]                       # iteration 1: Adam state loaded from the pre-step state
    ex = oracle_exact_step(name, st)
    fo = oracle_exact_step(name, st, force=per_net(ex["masks"]))
    again = oracle_exact_step(name, st)
    for sec in ("D", "gradD", "postD", "G", "gradG", "postG", "postD_G"):
        for k, v in ex[sec].items():
            if torch.is_tensor(v) and v.is_floating_point():
                assert _rel(fo[sec][k], v) <= 1e-15, (sec, k)
                assert torch.equal(again[sec][k], v), (sec, k)


def test_forced_masks_change_the_branch():
    """Flipping one forced sign in D's first activation moves D's first-layer gradient."""
    _, _, steps = oracle_steps("ralsgan", 1)
    st = steps[0]
    ex = oracle_exact_step("ralsgan", st)
    masks = per_net(ex["masks"])
    m = masks["D"][0].clone()
    m.view(-1)[0] = ~m.view(-1)[0]
    masks["D"][0] = m
    fo = oracle_exact_step("ralsgan", st, force=masks)
    k = "main.Start-Conv2d.weight"
    assert _rel(fo["gradD"][k], ex["gradD"][k]) > 1e-6
