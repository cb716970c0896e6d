"""CPU-only checks of the product surface (no GPU compute).

* the C-ABI library loads and exports every function include/rgan.h declares;
* the CLI accepts the reference's flags with the same defaults (GLI:17-62);
* DCGAN_G / DCGAN_D reproduce the reference's state_dict keys and -- since parameter
  init runs on the CPU generator -- its initial values bitwise (golden fixtures);
* the product path refuses CPU tensors (no CPU fallback exists).
"""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from tests.golden.configs import CONFIGS, PINNED
from tests.oracle_replay import load_golden, param_for

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    src = open(os.path.join(ROOT, "include", "rgan.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(rgan_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    from relativisticgan_amd import _lib
    lib = _lib.lib()
    declared = _declared_functions()
    assert len(declared) >= 30
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared) == set(_lib.EXPORTED), set(declared) ^ set(_lib.EXPORTED)
    assert b"gfx950" in lib.rgan_version()
    # rgan_adam_packed's float[2] step (count + arrival ticket) is ABI revision 2 (include/rgan.h)
    hdr = open(os.path.join(ROOT, "include", "rgan.h")).read()
    want = int(re.search(r"#define RGAN_ABI_VERSION (\d+)", hdr).group(1))
    assert lib.rgan_abi_version() == want == 4
    assert lib.rgan_version().endswith(b"abi%d" % want)


def test_library_rejects_bad_descriptors():
    from relativisticgan_amd import _lib
    lib = _lib.lib()
    d = _lib.RganConv()
    d.batch, d.cin, d.hin, d.win, d.cout, d.hout, d.wout = 2, 3, 8, 8, 4, 5, 5  # inconsistent hout
    d.kh = d.kw = 4
    d.stride, d.pad = 2, 1
    assert lib.rgan_conv_workspace(ctypes.byref(d), 0, 0) == 0
    d.hout = d.wout = 4
    for i, s in enumerate((192, 64, 8, 1)):
        d.xs[i] = s
    for i, s in enumerate((64, 1, 16, 4)):
        d.ys[i] = s
    assert lib.rgan_conv_workspace(ctypes.byref(d), 0, 0) > 0
    assert lib.rgan_loss_head(9, 0, None, None, 8, None, None, None, None) == 1001


def test_cli_matches_reference_flags():
    from oracle.reference_cpu import make_parser as oracle_parser
    from relativisticgan_amd.config import make_parser
    ours = {a.dest: a.default for a in make_parser()._actions if a.dest != "help"}
    ref = {a.dest: a.default for a in oracle_parser()._actions if a.dest != "help"}
    for k, v in ref.items():
        assert k in ours, k
        if k in ("input_folder", "output_folder", "inception_folder", "extra_folder", "CIFAR10_input_folder"):
            continue  # paths: the oracle blanks them
        assert ours[k] == v, (k, ours[k], v)


@pytest.mark.parametrize("name", PINNED)
def test_nets_state_dict_and_init_match_reference(name):
    """Keys, shapes and initial values of G and D == the reference's (fixture sha1s)."""
    import hashlib
    import random
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.nets import DCGAN_D, DCGAN_G, weights_init
    g = load_golden(name)
    p = param_for(name)
    ours = make_param(**{k: v for k, v in vars(p).items() if not k.startswith("rgan_")})
    random.seed(p.seed)
    np.random.seed(p.seed)
    torch.manual_seed(p.seed)
    G, D = DCGAN_G(ours), DCGAN_D(ours)
    G.apply(weights_init)
    D.apply(weights_init)
    for prefix, net in (("init.G.", G), ("init.D.", D)):
        sd = net.state_dict()
        want = {k[len(prefix):].split("@")[0] for k in g if k.startswith(prefix)}
        assert set(sd) == want, set(sd) ^ want
        for k, v in sd.items():
            full = prefix + k
            arr = v.detach().cpu().numpy()
            if full in g:
                assert np.array_equal(arr, g[full]), k
            else:
                sha = hashlib.sha1(arr.astype(np.float32).reshape(-1).tobytes()).hexdigest()
                assert sha == bytes(g[full + "@sha1"]).decode(), k


def test_cli_script_profiles():
    """--rgan_script: the art script is GLI with other defaults (art:20-60), PAC packs 2."""
    from relativisticgan_amd.config import parse
    art = parse(["--rgan_script", "GAN_losses_iter_art"])
    assert (art.image_size, art.loss_D, art.gen_every, art.gen_extra_images, art.pac) == (128, 7, 2000, 2000, 1)
    assert parse(["--rgan_script", "GAN_losses_iter_art", "--loss_D", "6"]).loss_D == 6
    assert parse(["--rgan_script", "GAN_losses_iter_PAC"]).pac == 2
    gli = parse([])
    assert (gli.image_size, gli.loss_D, gli.pac) == (64, 1, 1)


ORDER_CASES = list(CONFIGS) + ["arch1_spectral"]


@pytest.mark.parametrize("name", ORDER_CASES)
def test_parameter_and_state_dict_order_match_reference(name):
    """Parameter order == the reference's (torch optimizers load state by POSITION:
    spectral_norm registers weight_orig after bias), and state_dict key order too."""
    from oracle.reference_cpu import build_D, build_G
    from oracle.reference_cpu import make_param as oracle_param
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.nets import DCGAN_D, DCGAN_G
    if name == "arch1_spectral":
        kw = dict(arch=1, image_size=32, batch_size=8, z_size=16, loss_D=8, spectral=True, spectral_G=True)
    else:
        kw = {k: v for k, v in vars(param_for(name)).items() if not k.startswith("rgan_")}
    ours, ref = make_param(**kw), oracle_param(**{k: v for k, v in kw.items() if k != "cuda"})
    for mine, theirs in ((DCGAN_G(ours), build_G(ref)), (DCGAN_D(ours), build_D(ref))):
        assert [n for n, _ in mine.named_parameters()] == [n for n, _ in theirs.named_parameters()]
        assert list(mine.state_dict()) == list(theirs.state_dict())
        for (n, a), (_, b) in zip(mine.named_parameters(), theirs.named_parameters()):
            assert a.shape == b.shape, n


def test_adam_rejects_mismatched_state():
    from relativisticgan_amd.optim import Adam
    a, b = torch.nn.Parameter(torch.zeros(3)), torch.nn.Parameter(torch.zeros(2, 5))
    src = torch.optim.Adam([b, a])  # reversed order
    for q in (a, b):
        q.grad = torch.ones_like(q)
    src.step()
    opt = Adam([a, b])
    with pytest.raises(ValueError):
        opt.load_state_dict(src.state_dict())


def test_product_refuses_cpu_tensors():
    from relativisticgan_amd import kernels as K
    from relativisticgan_amd._lib import RganError
    x = torch.randn(1, 4, 8, 8)
    w = torch.randn(8, 4, 4, 4)
    with pytest.raises(RganError):
        K.conv_fwd(x, w, K.ConvGeom(4, 2, 1, False))
