"""Pin the ORACLE against the reference's own outputs (golden fixtures).

The fixtures in tests/golden were captured by running the unmodified reference
(tests/golden/make_golden.py); here the oracle replays each config and every
recorded tensor must be bitwise identical (sha1 for large tensors).  CPU only.
"""
import numpy as np
import pytest

from tests.golden.configs import PINNED
from tests.oracle_replay import golden_meta, load_golden, replay


@pytest.mark.parametrize("name", PINNED)
def test_oracle_bitwise_matches_reference(name):
    g = load_golden(name)
    meta = golden_meta(g)
    got, _ = replay(name, n_iter=meta["n_iter"], threads=meta["threads"])
    want_keys = {k for k in g if k != "meta.json"}
    missing = want_keys - set(got)
    assert not missing, f"oracle did not produce: {sorted(missing)[:10]}"
    bad = []
    for k in sorted(want_keys):
        a, b = g[k], got[k]
        if k.endswith("@sample") or k.endswith("@sum"):
            continue  # covered by the sha1 of the same tensor
        if a.shape != b.shape or not np.array_equal(a, b):
            bad.append(k)
    assert not bad, f"{len(bad)} tensors differ, e.g. {bad[:8]}"


def test_oracle_pac2_semantics():
    """PacGAN-2 oracle (parity unpinned, see tests/golden/configs.py): D sees 2B samples
    packed channel-wise, z is drawn for 2B per step, and the G step reuses the D step's
    G(z) (PAC:673-674), so G's BatchNorm runs once per iteration, not twice."""
    from tests.oracle_replay import dataset_for, param_for
    from oracle.reference_cpu import Trainer
    p = param_for("ralsgan_pac2")
    recs = {}
    t = Trainer(p, dataset_for("ralsgan_pac2"), hooks=lambda tag, r: recs.__setitem__(tag, dict(r)))
    nbt0 = int(t.G.state_dict()["main.Start-BatchNorm2d.num_batches_tracked"])
    t.iteration(1)  # i=1: no print_every sample forward
    B, S = p.batch_size, p.image_size
    assert tuple(recs["D"]["x"].shape) == (B, 2 * p.n_colors, S, S)
    assert tuple(recs["D"]["z"].shape) == (2 * B, p.z_size, 1, 1)
    assert tuple(recs["G"]["z"].shape) == (2 * B, p.z_size, 1, 1)
    assert int(t.G.state_dict()["main.Start-BatchNorm2d.num_batches_tracked"]) == nbt0 + 1
