"""Pin the ORACLE against the reference's own outputs (golden fixtures).

The fixtures in tests/golden were captured by running the unmodified reference
(tests/golden/make_golden.py); here the oracle replays each config and every
recorded tensor must be bitwise identical (sha1 for large tensors).  CPU only.
"""
import numpy as np
import pytest

from tests.golden.configs import CONFIGS
from tests.oracle_replay import golden_meta, load_golden, replay


@pytest.mark.parametrize("name", list(CONFIGS))
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
