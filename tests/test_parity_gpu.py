"""Step parity: the MI355X training step vs the oracle (pinned bitwise to the reference).

For every fixture config the oracle (CPU, fp32) replays the reference loop and exposes,
per iteration, the pre-step state, the drawn inputs and the results.  The GPU trainer is
teacher-forced from the same pre-step state and inputs, and again between its D step and
its G step (the G step starts from the oracle's post-D-step D, as does the fp64 run).  Each compared tensor T must
satisfy (tolerances stated here):

  direct:    rel_L2(T_gpu, T_oracle32) <= TOL[kind]                      OR
  forced:    rel_L2(T_gpu, T_forced) <= TOL[kind]                        OR
  envelope:  rel_L2(T_gpu, T_exact) <= max(TOL[kind], 4 * rel_L2(T_oracle32, T_exact))

where T_exact is the same teacher-forced step run by the oracle in float64, and T_forced
is that float64 step run with every ReLU / LeakyReLU / SELU taking the branch the GPU
took (the mask-forced judge: the GPU's recorded activation signs replace the signs of the
exact pre-activations; equal to T_exact when no sign differs).  It measures the GPU's
arithmetic at the same tolerance as "direct", without the O(1) gradient jump a near-zero
pre-activation landing on the other side of a kink causes (see below).  The
envelope form admits exactly the cases where fp32 itself is ill-conditioned (conv
biases feeding BatchNorm have an exact gradient of 0, so both fp32 results are
roundoff; BN-backward cancellation in arch 1), and nothing else.

The forced judge proves its premise (``check_premise``): wherever a GPU activation sign
differs from the exact step's, the exact pre-activation must be within rounding of 0,
|x_exact| <= TAU_FLIP * RMS of that activation call -- a genuinely wrong sign of a
large-magnitude element fails the test instead of being adopted by the forced step.  Outputs
and gradients that pass directly or against the forced step must also pass elementwise:
max|T_gpu - T_forced| <= ELEM_FACTOR * TOL[kind] * RMS(T_forced), so a few corrupted elements
of a large tensor fail although they barely move its rel-L2 (tests/test_parity_judge.py
checks both failure modes on CPU).  The full-size configs run twice: on the fp32 MFMA
and with the opt-in fp32-on-bf16x6 GEMMs (``-bf16x6`` ids), judged identically.

ReLU', LeakyReLU' and SELU' jump at 0.  Every forward activation sign of the GPU step
is compared with the exact step (autograd.ACT_TRACE vs forward hooks on the oracle's
activation modules, same call order); when a pre-activation within rounding of 0 lands
on the other side (a "flip"), the forward values move by ~(1-alpha)|v| (negligible) but
the gradient through that element changes by O(1).  Only the tensors a flip can reach
are relaxed (to FLIP_TOL = 3e-2 relative, Adam's element-fraction bound to 5%):
  * a flip in D's layer L during the D step's D(x) / D(x_fake): the D gradients (and
    post-Adam D parameters) of layers <= L -- backprop reaches only the layers before it;
  * a flip in the gradient-penalty pass D(x_hat): every D gradient and the penalty (the
    double backward differentiates the whole dgrad chain);
  * a flip in G's layer L during the G step: G's gradients of layers <= L;
  * a flip in D(fake) during the G step: every G gradient (dD/dx flows into G);
  * flips in no-grad forwards (G(z) in the D step, D(x) in the G step, G(z_test)): none.
With RGAN_PARITY_AUDIT=<dir> every config writes <dir>/<name>.json: per tensor the
direct error, the envelope errors when used, and whether a flip relaxed it.

  TOL: outputs / losses / GP 1e-4; gradients 2e-4; BN running stats, spectral u/v 1e-4.
  Parameters after Adam: max|p_gpu - p_exact| <= 2.02 x the largest update the exact or
  the oracle step makes in the tensor (Adam's first steps are sign steps, so a near-zero
  gradient may flip: 2*lr at step 1) and at most max(1%, 2x the oracle's own share + 0.5%) of elements off by more
  than 1e-6.  Where a mask-forced step exists, the post-Adam parameters are measured against
  it as well and the closer of the two counts (as for gradients: after a flip the GPU's
  gradient is the forced step's, and Adam's sign steps turn every near-zero gradient element
  the flip moved into a full-size parameter difference from the exact step).
"""
import copy
import json
import os

import pytest
import torch

from tests.golden.configs import CONFIGS, FULL_SIZE
from tests.oracle_replay import dataset_for, param_for

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL_OUT, TOL_GRAD, TOL_BUF = 1e-4, 2e-4, 1e-4
FLIP_TOL = 3e-2
# Mask-forced judge premise: the GPU may take the other branch of a kink only where the exact
# pre-activation is within rounding of 0: |x_exact| <= TAU_FLIP * RMS(x_exact) of that
# activation call (fp32 rounding of a pre-activation is ~1e-6 of its RMS: 100x margin).
TAU_FLIP = 1e-4
NEAR_STORE = 1e-3   # the exact step records pre-activations within this of 0 (x RMS)
# Elementwise bound of outputs and gradients against the mask-forced step: max|gpu - forced|
# <= ELEM_FACTOR * tol * RMS(forced) (rel-L2 alone lets a few corrupted elements of a large
# tensor through).
ELEM_FACTOR = 10


def _rel(a, b):
    a = a.detach().double().cpu().reshape(-1)
    b = b.detach().double().cpu().reshape(-1)
    den = b.norm()
    if den == 0:
        return (a - b).norm().item()
    return ((a - b).norm() / den).item()


def _cap(cur, t, tag, r):
    if tag == "D":
        cur["D"] = {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in r.items()}
        cur["gradD"] = {n: q.grad.detach().clone() for n, q in t.D.named_parameters()}
    elif tag == "D.post":
        cur["postD"] = {k: v.detach().clone() for k, v in t.D.state_dict().items()}
    elif tag == "G":
        cur["G"] = {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in r.items()}
        cur["gradG"] = {n: q.grad.detach().clone() for n, q in t.G.named_parameters()}
    elif tag == "G.post":
        cur["postG"] = {k: v.detach().clone() for k, v in t.G.state_dict().items()}
        cur["postD_G"] = {k: v.detach().clone() for k, v in t.D.state_dict().items()}


def _threads(name):
    """Host threads for the CPU oracle: 4 for the small fixtures, the lease's cores (at most
    16, the GPU box's share) for the full-size BASELINE configs."""
    if name not in FULL_SIZE:
        return 4
    return max(1, min(16, len(os.sched_getaffinity(0))))


def oracle_steps(name, n_iter):
    """Oracle fp32 replay: per iteration pre-state, inputs, outputs, grads, post-state."""
    from oracle.reference_cpu import Trainer
    torch.set_num_threads(_threads(name))
    p = param_for(name)
    steps, cur, holder = [], {}, {}
    t = Trainer(p, dataset_for(name), hooks=lambda tag, r: _cap(cur, holder["t"], tag, r))
    holder["t"] = t
    init = {"G": copy.deepcopy(t.G.state_dict()), "D": copy.deepcopy(t.D.state_dict()), "z_test": t.z_test.clone()}
    for i in range(n_iter):
        pre = {"G": copy.deepcopy(t.G.state_dict()), "D": copy.deepcopy(t.D.state_dict()),
               "optG": copy.deepcopy(t.optG.state_dict()), "optD": copy.deepcopy(t.optD.state_dict())}
        cur.clear()
        t.iteration(i)
        steps.append(dict(cur, pre=pre, i=i))
    return p, init, steps


def _feed(st):
    f = {"x_D": st["D"]["x"], "z_D": st["D"]["z"], "z_G": st["G"]["z"]}
    if "u" in st["D"]:
        f["u"] = st["D"]["u"]
    if "x" in st["G"]:
        f["x_G"] = st["G"]["x"]
    return f


def _force_activations(net, queue):
    """Make every ReLU / LeakyReLU / SELU of ``net`` take its branch from ``queue`` (the GPU's
    recorded activation signs, in call order) instead of from the sign of its input: the
    exact step then runs the GPU's piecewise-linear branch everywhere, so what remains
    between the two is arithmetic, not which side of a kink a near-zero value fell on."""
    def make(mod):
        def fwd(x):
            if not queue:
                raise RuntimeError("forced activation masks exhausted")
            m = queue.pop(0).to(x.device).contiguous()  # GPU masks are NHWC-strided; keep x's layout
            if m.shape != x.shape:
                raise RuntimeError(f"forced mask shape {tuple(m.shape)} vs {tuple(x.shape)}")
            if isinstance(mod, torch.nn.ReLU):
                return torch.where(m, x, torch.zeros_like(x))
            if isinstance(mod, torch.nn.LeakyReLU):
                return torch.where(m, x, x * mod.negative_slope)
            a, sc = 1.6732632423543772848170429916717, 1.0507009873554804934193349852946  # torch SELU
            return torch.where(m, sc * x, sc * a * torch.expm1(x))
        return fwd
    for mod in net.modules():
        if isinstance(mod, (torch.nn.ReLU, torch.nn.LeakyReLU, torch.nn.SELU)):
            mod.forward = make(mod)


def _near_hooks(net, tag, out):
    """Forward pre-hooks recording, per kinked activation call of the exact step, RMS(x) of
    the pre-activation x and every element with |x| <= NEAR_STORE * RMS(x) (flat index and
    value): what ``check_premise`` needs to bound |x| wherever the GPU took the other sign.
    x is read before the module runs (the reference's LeakyReLU is in place)."""
    def pre(mod, inp):
        x = inp[0].detach()
        rms = x.double().pow(2).mean().sqrt().item()
        flat = x.reshape(-1)
        idx = torch.nonzero(flat.abs() <= NEAR_STORE * rms).reshape(-1)
        out.append((tag, rms, idx.cpu(), flat[idx].double().cpu()))
    return [m.register_forward_pre_hook(pre) for m in net.modules()
            if isinstance(m, (torch.nn.ReLU, torch.nn.LeakyReLU, torch.nn.SELU))]


def check_premise(got_masks, exact):
    """The mask-forced judge's premise: the GPU may take the other side of a kink than the
    exact step only where the exact pre-activation is within rounding of 0.  For every
    activation call (per net, call order) and every element whose GPU sign differs from the
    exact sign: |x_exact| / RMS(x_exact) <= TAU_FLIP.  Returns (records, errors)."""
    mine = per_net(got_masks)
    ex_m = per_net(exact["masks"])
    near = {tag: [(r, i, v) for t_, r, i, v in exact["near"] if t_ == tag] for tag in ("G", "D")}
    recs, errs = [], []
    for tag in ("G", "D"):
        assert len(mine[tag]) == len(ex_m[tag]) == len(near[tag]), (tag, len(mine[tag]), len(ex_m[tag]))
        for call, (a, b, (rms, idx, val)) in enumerate(zip(mine[tag], ex_m[tag], near[tag])):
            flips = torch.nonzero((a.reshape(-1).cpu() != b.reshape(-1).cpu())).reshape(-1)
            if flips.numel() == 0:
                continue
            # idx is sorted (torch.nonzero): locate each flip among the recorded near elements
            pos = torch.searchsorted(idx, flips).clamp(max=max(idx.numel() - 1, 0))
            hit = (idx[pos] == flips) if idx.numel() else torch.zeros_like(flips, dtype=torch.bool)
            far = int((~hit).sum())
            ratio = (val[pos[hit]].abs().max().item() if bool(hit.any()) else 0.0) / max(rms, 1e-300)
            if far:
                ratio = float("inf")
            recs.append({"net": tag, "call": call, "flips": int(flips.numel()), "max_abs_over_rms": ratio})
            if ratio > TAU_FLIP:
                errs.append(f"{tag} activation call {call}: {flips.numel()} sign flips, max |x_exact| / RMS = "
                            f"{ratio:.2e} > {TAU_FLIP:.0e}" + (f" ({far} beyond {NEAR_STORE:.0e})" if far else ""))
    return recs, errs


def oracle_exact_step(name, st, force=None):
    """The same teacher-forced step in float64 (the 'exact' reference for the envelope).
    With ``force`` ({"G": [masks], "D": [masks]} in each net's call order) every kinked
    activation follows the given signs (the mask-forced judge, see ``compare``).  Without,
    ``cur["near"]`` holds every pre-activation within NEAR_STORE of 0 (``check_premise``)."""
    from oracle.reference_cpu import Trainer
    cur, holder = {}, {}
    def hook(tag, r):
        _cap(cur, holder["t"], tag, r)
        if tag == "D.post":  # the G step starts from the oracle's post-D-step D (see gpu_step)
            holder["t"].D.load_state_dict(st["postD"])
    # float64 on the device (checker only: ATen's double convolutions with MIOpen off, as
    # tests/test_kernels_gpu.py builds its fp64 references); the fp32 replay above stays on the
    # host, where it is pinned bitwise to the reference
    dev = DEV if torch.cuda.is_available() else "cpu"  # (the CPU judge tests: tests/test_parity_judge.py)
    t = Trainer(param_for(name), dataset_for(name), hooks=hook, dtype=torch.float64, device=dev)
    holder["t"] = t
    pre = copy.deepcopy(st["pre"])  # torch Adam keeps the loaded `step` tensors and bumps them in place
    t.G.load_state_dict(pre["G"])
    t.D.load_state_dict(pre["D"])
    if pre["optG"]["state"]:
        t.optG.load_state_dict(pre["optG"])
        t.optD.load_state_dict(pre["optD"])
    if force is not None:
        queues = {tag: list(ms) for tag, ms in force.items()}
        _force_activations(t.G, queues["G"])
        _force_activations(t.D, queues["D"])
    masks, near = [], []
    hooks = [m.register_forward_hook(lambda mod, inp, out, tag=tag: masks.append((tag, (out.detach() > 0).cpu())))
             for net, tag in ((t.G, "G"), (t.D, "D")) for m in net.modules()
             if isinstance(m, (torch.nn.ReLU, torch.nn.LeakyReLU, torch.nn.SELU))]
    if force is None:
        hooks += _near_hooks(t.G, "G", near) + _near_hooks(t.D, "D", near)
    with torch.backends.cudnn.flags(enabled=False):
        t.iteration(st["i"], feed={k: v.double().to(dev) for k, v in _feed(st).items()})
    for h in hooks:
        h.remove()
    for sec in ("D", "gradD", "postD", "G", "gradG", "postG", "postD_G"):
        if sec in cur:
            cur[sec] = {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in cur[sec].items()}
    if force is not None and any(queues.values()):
        raise RuntimeError("forced activation masks left over: " + str({k: len(v) for k, v in queues.items()}))
    cur["masks"] = masks
    cur["near"] = near
    return cur


def gpu_step(t, st):
    from relativisticgan_amd import autograd
    got = {}
    autograd.ACT_TRACE = []
    autograd.ACT_TAGS = []
    autograd.ACT_LAYERS = []
    pre = copy.deepcopy(st["pre"])
    t.G.load_state_dict(pre["G"])
    t.D.load_state_dict(pre["D"])
    if pre["optG"]["state"]:
        t.optG.load_state_dict(pre["optG"])
        t.optD.load_state_dict(pre["optD"])
    try:
        split = {}

        def hook(tag, r):
            if tag == "D":  # everything traced so far belongs to the D step
                split["D"] = len(autograd.ACT_TRACE)
            _cap(got, t, tag, r)
            if tag == "D.post":
                # teacher-force the G step too: it starts from the oracle's post-D-step D.
                # Adam's first steps are sign steps, so D after a fp32 step differs from
                # fp64 by +-lr on near-zero-gradient elements; the G step would otherwise
                # inherit that (and every activation flip it causes in D(fake)).
                t.D.load_state_dict(st["postD"])
        t.iteration(st["i"], feed={k: v.to(DEV) for k, v in _feed(st).items()}, hooks=hook)
        masks = list(zip(autograd.ACT_TAGS, autograd.ACT_TRACE))
        got["trace_info"] = [(tag, li, "D" if k < split["D"] else "G")
                             for k, (tag, li) in enumerate(zip(autograd.ACT_TAGS, autograd.ACT_LAYERS))]
    finally:
        autograd.ACT_TRACE = None
    got["postG"] = {k: v.detach().clone() for k, v in t.G.state_dict().items()}
    got["postD_G"] = {k: v.detach().clone() for k, v in t.D.state_dict().items()}
    torch.cuda.synchronize()
    info = got.pop("trace_info")
    out = {k: {n: (v.cpu() if torch.is_tensor(v) else v) for n, v in d.items()} for k, d in got.items()}
    out["masks"] = masks
    out["trace_info"] = info
    return out


def per_net(trace):
    """(tag, mask) entries -> per-net mask streams, call order kept within each net (the
    GPU D step runs G(z) before its one batched D pass; the reference interleaves them)."""
    return {tag: [m for t, m in trace if t == tag] for tag in ("G", "D")}


def locate_flips(ours, exact, info):
    """Activation-sign disagreements between the GPU and the exact forward passes, as
    [(net, plan layer, phase, call index within the phase, count)]."""
    streams = {tag: [(m, inf) for (t_, m), inf in zip(ours, info) if t_ == tag] for tag in ("G", "D")}
    exact = per_net(exact)
    out = []
    for tag in ("G", "D"):
        mine = streams[tag]
        assert len(mine) == len(exact[tag]), f"{tag} activation trace length {len(mine)} vs {len(exact[tag])}"
        per_call = len({li for _, (_, li, _) in mine}) or 1   # kinked layers per call of this net
        seen = {}
        for (a, (_, li, ph)), b in zip(mine, exact[tag]):
            assert a.shape == b.shape, (tag, a.shape, b.shape)
            k = seen.get(ph, 0)
            seen[ph] = k + 1
            n = int((a != b).sum())
            if n:
                out.append((tag, li, ph, k // per_call, n))
    return out


def layer_of_params(net):
    """parameter name -> index of its fused layer in the net's plan."""
    ids = {id(q): n for n, q in net.named_parameters()}
    out = {}
    for li, layer in enumerate(net._plan):
        for mod in (layer.conv, layer.bn):
            if mod is None:
                continue
            for q in mod.parameters(recurse=False):
                if id(q) in ids:
                    out[ids[id(q)]] = li
    return out


def flip_reach(flips, p, lay_G, lay_D, g_step_fake_call=0):
    """Which tensors the located flips can move (see the module docstring)."""
    reach = set()
    gp = p.loss_D == 3 or p.grad_penalty
    for tag, li, ph, call, _n in flips:
        if getattr(p, "pac", 1) == 2 and tag == "G" and ph == "D":
            ph = "G"  # PacGAN: the G step backpropagates through the D step's G(z) (PAC:674)
        if ph == "D" and tag == "D":
            if gp and call >= 2:       # D(x), D(x_fake), then the penalty's D(x_hat)
                reach |= {f"gradD.{n}" for n in lay_D} | {"D.gp"}
            else:
                reach |= {f"gradD.{n}" for n, l in lay_D.items() if l <= li}
        elif ph == "G" and tag == "G":
            reach |= {f"gradG.{n}" for n, l in lay_G.items() if l <= li}
        elif ph == "G" and tag == "D" and call == g_step_fake_call:
            reach |= {f"gradG.{n}" for n in lay_G}
    reach |= {"postD." + k[len("gradD."):] for k in reach if k.startswith("gradD.")}
    reach |= {"postG." + k[len("gradG."):] for k in reach if k.startswith("gradG.")}
    return reach


def _lookup(d, label):
    """got/exact dicts are keyed by section ("D", "gradD", "postD", ...) then name."""
    sec, _, key = label.partition(".")
    return d.get(sec, {}).get(key)


def _elem(a, b):
    """max |a - b| / RMS(b) (elementwise error on the reference tensor's own scale)."""
    a = a.detach().double().cpu().reshape(-1)
    b = b.detach().double().cpu().reshape(-1)
    rms = b.pow(2).mean().sqrt().item() if b.numel() else 0.0
    d = (a - b).abs().max().item() if b.numel() else 0.0
    return d / rms if rms > 0 else d


def compare(p, st, got, exact, report, reach=frozenset(), forced=None):
    errs = []

    def check(label, g, o, x, tol, elem=False):
        e_dir = _rel(g, o)
        rec = {"tensor": f"it{st['i']}.{label}", "direct": e_dir, "tol": tol}
        report.append(rec)
        xf = _lookup(forced, label) if forced is not None else None

        def elem_ok():
            # elementwise against the mask-forced step (the GPU's own branches, computed
            # exactly): a few corrupted elements move rel-L2 of a large tensor by almost
            # nothing, but never pass this (ELEM_FACTOR x tol of the tensor's RMS).  Not for
            # envelope tensors (ill-conditioned in fp32: exact gradient ~0)
            if not elem or xf is None:
                return True
            rec["elem_vs_forced"] = e_el = _elem(g, xf)
            if e_el <= ELEM_FACTOR * tol:
                return True
            rec["via"] = "FAIL"
            errs.append(f"{label}: max|gpu - forced| / RMS = {e_el:.2e} > {ELEM_FACTOR * tol:.1e} "
                        f"(rel-L2 vs oracle {e_dir:.2e})")
            return False

        if e_dir <= tol:
            if elem_ok():
                rec["via"] = "direct"
            return
        if xf is not None:
            rec["gpu_vs_forced"] = e_f = _rel(g, xf)
            if e_f <= tol:  # the GPU's own branch decisions, computed exactly: same result
                if elem_ok():
                    rec["via"] = "forced"
                return
        e_gx, e_ox = _rel(g, x), _rel(o, x)
        rec.update(gpu_vs_exact=e_gx, oracle_vs_exact=e_ox)
        if e_gx <= max(tol, 4 * e_ox):
            rec["via"] = "envelope"
            return
        if label in reach and e_dir <= FLIP_TOL:
            rec["via"] = "flip"
            return
        rec["via"] = "FAIL"
        errs.append(f"{label}: gpu-vs-oracle {e_dir:.2e}, gpu-vs-exact {e_gx:.2e}, "
                    f"oracle-vs-exact {e_ox:.2e}{' (flip-reachable)' if label in reach else ''}")

    for side, keys in (("D", ("y_pred", "y_pred_fake", "errD", "gp")), ("G", ("y_pred", "y_pred_fake", "errG"))):
        for k in keys:
            if k in st[side]:
                check(f"{side}.{k}", got[side][k], st[side][k], exact[side][k], TOL_OUT, elem=True)
    for gk in ("gradD", "gradG"):
        for n, o in st[gk].items():
            check(f"{gk}.{n}", got[gk][n], o, exact[gk][n], TOL_GRAD, elem=True)
    i = st["i"]
    for label, lr in (("postD", p.lr_D * (1 - p.decay) ** i), ("postG", p.lr_G * (1 - p.decay) ** i)):
        for k, o in st[label].items():
            g, x = got[label][k], exact[label][k]
            if k.endswith("num_batches_tracked"):
                if int(g) != int(o):
                    errs.append(f"{label}.{k}: {int(g)} != {int(o)}")
                continue
            if "running" in k or k.endswith("weight_u") or k.endswith("weight_v"):
                check(f"{label}.{k}", g, o, x, TOL_BUF)
                continue
            d = (g.double() - x.double()).abs()
            dref = (o.double() - x.double()).abs()
            xf = _lookup(forced, f"{label}.{k}") if forced is not None else None
            frac_f = None
            if xf is not None:  # the GPU's own branches, computed exactly, then the same Adam step
                df = (g.double() - xf.double()).abs()
                frac_f = (df > 1e-6).double().mean().item()
                if frac_f < (d > 1e-6).double().mean().item():
                    d = df
            # a sign-flipped Adam update moves an element by at most 2x the largest update
            # made in this tensor (2*lr at step 1); for biases feeding BN the exact update is
            # 0 while the oracle's own fp32 step moves them by +-lr, so both count
            pre = st["pre"]["D" if label == "postD" else "G"][k].double()
            upd = max((x.double() - pre).abs().max().item(), (o.double() - pre).abs().max().item())
            bound = 2.02 * upd + 1e-7
            if d.max().item() > bound:
                errs.append(f"{label}.{k}: max|dp| {d.max().item():.3e} > {bound:.3e}")
            frac, fref = (d > 1e-6).double().mean().item(), (dref > 1e-6).double().mean().item()
            report.append({"tensor": f"it{i}.{label}.{k}", "adam_max_dp": d.max().item(), "adam_bound": bound,
                           "frac_off": frac, "oracle_frac_off": fref, "frac_off_vs_forced": frac_f,
                           "flip_reachable": f"{label}.{k}" in reach})
            if frac > max(0.05 if f"{label}.{k}" in reach else 0.01, 2 * fref + 0.005):
                errs.append(f"{label}.{k}: {frac:.2%} of elements off by >1e-6 (oracle fp32: {fref:.2%})")
    for k, o in st["postD_G"].items():  # D buffers after the G step (BN stats / spectral u,v move there too)
        if "running" in k or k.endswith("weight_u") or k.endswith("weight_v"):
            check(f"postD_G.{k}", got["postD_G"][k], o, exact["postD_G"][k], TOL_BUF)
    return errs


# The oracle's fp32 replay and the exact fp64 steps of the last config, shared by its fp32 and
# bf16x6 GPU runs (one config at a time: the full-size states are GBs).
_CACHE = {}


def _oracle_for(name, n_iter):
    if _CACHE.get("name") != name:
        _CACHE.clear()
        _CACHE["name"] = name
        _CACHE["oracle"] = oracle_steps(name, n_iter)
        _CACHE["exact"] = {}
    return _CACHE["oracle"]


def _exact_for(name, st):
    ex = _CACHE["exact"]
    if st["i"] not in ex:
        ex[st["i"]] = oracle_exact_step(name, st)
    return ex[st["i"]]


# every fixture config on the fp32 MFMA path; the full-size BASELINE configs also with the
# opt-in fp32-on-bf16x6 GEMMs (rgan_set_gemm_emulation), judged identically.  The
# bf16x6 rows qualify an opt-in variant that is never the bench's `value`: they carry the
# `gpu_emu` marker and run only when it is selected (`-m gpu_emu`), not in the default `-m gpu`
# suite (tests/conftest.py); their audit is committed (profiles/round*_parity_summary.json)
PARITY_CASES = [pytest.param(n, False, id=n) for n in CONFIGS] + \
               [pytest.param(n, True, id=n + "-bf16x6", marks=pytest.mark.gpu_emu) for n in FULL_SIZE]


@pytest.mark.parametrize("name,emu", PARITY_CASES)
def test_step_parity_teacher_forced(name, emu):
    from relativisticgan_amd import kernels
    from relativisticgan_amd.train import Trainer
    n_iter = CONFIGS[name]["args"].get("n_iter", 3)
    p, init, steps = _oracle_for(name, n_iter)
    print(f"[parity {name}] oracle fp32 replay done", flush=True)
    p = copy.deepcopy(p)
    p.rgan_rng = "host"
    prev = kernels.set_gemm_emulation(emu)
    try:
        t = Trainer(p, dataset_for(name).to(DEV))
        # the initial state comes from the same CPU init calls: bitwise equal
        for k, v in init["G"].items():
            assert torch.equal(t.G.state_dict()[k].cpu(), v), f"G init {k}"
        for k, v in init["D"].items():
            assert torch.equal(t.D.state_dict()[k].cpu(), v), f"D init {k}"
        assert torch.equal(t.z_test.cpu(), init["z_test"])
        lay_G, lay_D = layer_of_params(t.G), layer_of_params(t.D)
        errs, report, flips_all, premise = [], [], [], []
        for st in steps:
            got = gpu_step(t, st)
            print(f"[parity {name}{'-bf16x6' if emu else ''}] it{st['i']}: GPU step done", flush=True)
            exact = _exact_for(name, st)
            print(f"[parity {name}] it{st['i']}: exact fp64 step done", flush=True)
            recs, perrs = check_premise(got["masks"], exact)
            premise += [dict(r, it=st["i"]) for r in recs]
            errs += [f"it{st['i']} premise: {e}" for e in perrs]
            flips = locate_flips(got["masks"], exact["masks"], got["trace_info"])
            try:
                forced = oracle_exact_step(name, st, force=per_net(got["masks"])) if flips else exact
            except RuntimeError as e:  # a call order the per-net queues cannot follow (none known)
                print(f"{name}: no mask-forced judge: {e}")
                forced = None
            flips_all += [dict(it=st["i"], net=f[0], layer=f[1], phase=f[2], call=f[3], elements=f[4]) for f in flips]
            reach = flip_reach(flips, p, lay_G, lay_D)
            errs += [f"it{st['i']} {e}" for e in compare(p, st, got, exact, report, reach, forced)]
            del got, forced
    finally:
        kernels.set_gemm_emulation(prev)
    tens = [r for r in report if "via" in r]
    by = {v: sum(1 for r in tens if r["via"] == v) for v in ("direct", "forced", "envelope", "flip", "FAIL")}
    worst = max(tens, key=lambda r: r["direct"] / r["tol"])
    elem = [r for r in tens if "elem_vs_forced" in r]
    worst_el = max(elem, key=lambda r: r["elem_vs_forced"] / r["tol"]) if elem else None
    tag = name + ("-bf16x6" if emu else "")
    summary = {"config": tag, "gemm_arith": "bf16x6" if emu else "fp32", "tensors": len(tens), **by,
               "flips": flips_all, "premise": premise,
               "premise_max_abs_over_rms": max((r["max_abs_over_rms"] for r in premise), default=0.0),
               "tau_flip": TAU_FLIP, "elem_factor": ELEM_FACTOR,
               "worst_elem_vs_forced": ({"tensor": worst_el["tensor"], "max_over_rms": worst_el["elem_vs_forced"],
                                         "tol": worst_el["tol"]} if worst_el else None),
               "worst_direct": {"tensor": worst["tensor"], "rel": worst["direct"], "tol": worst["tol"]},
               "exceptions": [r for r in tens if r["via"] != "direct"]}
    print(f"{tag}: {len(tens)} tensors: {by['direct']} direct, {by['forced']} direct vs the mask-forced fp64 step, "
          f"{by['envelope']} via fp64 envelope, "
          f"{by['flip']} flip-relaxed, {by['FAIL']} failed; flips {sum(f['elements'] for f in flips_all)} "
          f"(max |x_exact|/RMS {summary['premise_max_abs_over_rms']:.2e}); worst elementwise "
          f"{(worst_el['elem_vs_forced'] / worst_el['tol']) if worst_el else 0:.2f} x tol")
    out_dir = os.environ.get("RGAN_PARITY_AUDIT")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"{tag}.json"), "w") as f:
            json.dump(dict(summary, report=report), f, indent=1)
    assert not errs, "\n".join(errs[:30])
