"""CPU checks of the GPU parity judge itself (tests/test_parity_gpu.py).

The mask-forced float64 step must be the exact step whenever the forced signs are the
exact step's own (so "forced" can only differ from "exact" through the GPU's branch
choices), and the teacher-forcing state must survive being loaded twice (torch's Adam
bumps the loaded ``step`` tensors in place).
"""
import pytest
import torch

from tests.test_parity_gpu import (ELEM_FACTOR, TOL_GRAD, _rel, check_premise, compare, oracle_exact_step,
                                   oracle_steps, per_net)


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


def _as_gpu(ex):
    """A stand-in 'GPU step': the exact step's results rounded to fp32 (arithmetic-exact)."""
    out = {}
    for sec in ("D", "G", "gradD", "gradG", "postD", "postG", "postD_G"):
        out[sec] = {k: (v.float() if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in ex[sec].items()}
    return out


def test_premise_rejects_a_large_wrong_sign():
    """The forced judge adopts the GPU's activation signs only where the exact pre-activation
    is within rounding of 0: the exact step's own signs pass, one flipped sign on a
    large-magnitude element fails (check_premise)."""
    _, _, steps = oracle_steps("ralsgan", 1)
    st = steps[0]
    ex = oracle_exact_step("ralsgan", st)
    recs, errs = check_premise(ex["masks"], ex)
    assert not recs and not errs
    masks = list(ex["masks"])
    tag, m = masks[0]
    near = ex["near"][0]
    x_rms = near[1]
    m = m.clone()
    # an element far from 0: any not recorded in the near set (|x| > NEAR_STORE * RMS)
    flat = m.view(-1)
    k = next(i for i in range(flat.numel()) if i not in set(near[2].tolist()))
    flat[k] = ~flat[k]
    masks[0] = (tag, m)
    recs, errs = check_premise(masks, ex)
    assert errs and recs[0]["flips"] == 1 and recs[0]["max_abs_over_rms"] == float("inf"), (recs, errs, x_rms)


def test_elementwise_bound_rejects_one_corrupted_element():
    """One gradient element off by 5e-3 x RMS moves the tensor's rel-L2 by far less than the
    2e-4 tolerance, but fails the elementwise bound against the forced step."""
    p, _, steps = oracle_steps("ralsgan", 1)
    st = steps[0]
    ex = oracle_exact_step("ralsgan", st)
    got = _as_gpu(ex)
    assert compare(p, st, got, ex, [], forced=ex) == []
    name = max(got["gradD"], key=lambda n: got["gradD"][n].numel())
    g = got["gradD"][name]
    rms = g.double().pow(2).mean().sqrt().item()
    bad = g.clone()
    bad.view(-1)[g.numel() // 2] += 5e-3 * rms
    assert _rel(bad, ex["gradD"][name]) < TOL_GRAD  # rel-L2 alone would pass it
    assert 5e-3 > ELEM_FACTOR * TOL_GRAD
    got["gradD"][name] = bad
    errs = compare(p, st, got, ex, [], forced=ex)
    assert len(errs) == 1 and name in errs[0] and "max|gpu - forced|" in errs[0], errs
