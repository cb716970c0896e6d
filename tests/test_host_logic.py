"""Host-side logic of the round-3 fusions, on the CPU (no kernel launches).

* loss heads: the unit backward seed registry (a dead seed's address must not stay "unit");
* autograd.LayerLink: the kernels.Post it builds for the lower layer (rows of the gradient
  segment, per-segment statistics rows, act-only vs BatchNorm mode);
* ConvLayerFn: forward inputs == backward outputs (autograd requires one gradient slot per input);
* --rgan_batch_G is a CLI flag with the reference's argparse bool convention.
"""
import gc
import inspect

import torch

from relativisticgan_amd import autograd as AG
from relativisticgan_amd import losses


def test_unit_seed_registry():
    one = losses.unit_seed("cpu")
    assert losses._is_unit(one)
    other = torch.ones((), dtype=torch.float32)
    assert not losses._is_unit(other)
    ptr = one.data_ptr()
    del one
    gc.collect()
    assert ptr not in losses._UNIT_SEEDS


def test_layer_link_post_rows_and_segments():
    link = AG.LayerLink()
    assert link.post(4, 1) is None  # nothing recorded: no post-op
    y = torch.randn(8, 16, 4, 4).contiguous(memory_format=torch.channels_last)
    stats = torch.randn(2, 32)  # two batch segments' (mean, invstd)
    link.mode, link.act, link.alpha, link.x, link.stats = 2, "lrelu", 0.2, y, stats
    link.gamma, link.beta, link.segs = torch.ones(16), torch.zeros(16), 2
    p = link.post(4, 1)  # the G step's restricted backward: first segment only
    assert p.mode == 2 and p.nseg == 1 and p.x.shape[0] == 4 and p.x.data_ptr() == y.data_ptr()
    assert torch.equal(p.stats, stats[:1])
    p2 = link.post(8, 2)  # the batched D step: both segments
    assert p2.nseg == 2 and torch.equal(p2.stats, stats)
    link1 = AG.LayerLink()
    a = torch.randn(8, 16, 4, 4)
    link1.mode, link1.act, link1.alpha, link1.x = 1, "relu", 0.0, a
    p3 = link1.post(8, 2)
    assert p3.mode == 1 and p3.stats is None and p3.x.shape[0] == 8


def test_conv_layer_fn_arity():
    n_in = len(inspect.signature(AG.ConvLayerFn.forward).parameters) - 1  # minus ctx
    src = inspect.getsource(AG.ConvLayerFn)
    # every return of backward / _create_graph_backward hands back one slot per forward input
    assert f"[None] * {n_in}" in src
    tail = ", ".join(["None"] * (n_in - 5))
    assert f"return dx, dw, db, dgamma, dbeta, {tail}\n" in src


def test_batch_G_flag():
    from relativisticgan_amd.config import make_param, parse
    assert make_param().rgan_batch_G is None
    p = parse(["--rgan_batch_G", "False"])
    assert p.rgan_batch_G is False


def test_throughput_meter_line():
    """train.main's SURVEY §5 log suffix: img/s of the global batch and MFMA% of one GPU from
    the conv FLOPs of an iteration (the same count bench.py uses)."""
    from relativisticgan_amd import perf

    m = perf.ThroughputMeter.__new__(perf.ThroughputMeter)
    m.flops, m.images, m.t0, m.i0 = 1.573e12, 32, None, None
    m.excluded = 0.0
    assert m.tick(0, 10.0) is None          # first point: nothing to report yet
    line = m.tick(10, 12.0)                 # 10 iterations in 2 s = 5 it/s
    assert line == "[10] img/s: 160.0 MFMA%%: %.1f" % (100.0 * 5 * 1.573e12 / perf.FP32_MFMA_PEAK)
    # host-side output work (sample PNG, checkpoint) is left out of the interval
    m.exclude(1.5)
    line = m.tick(20, 16.0)                 # 10 iterations in 4 s - 1.5 s = 4 it/s
    assert line == "[20] img/s: 128.0 MFMA%%: %.1f" % (100.0 * 4 * 1.573e12 / perf.FP32_MFMA_PEAK)
    assert perf.FP32_MFMA_PEAK == 157.3e12  # (the meter on a real trainer: tests/test_cli_gpu.py)


def test_pack_cache_drops_views_of_shrunk_storage():
    """kernels._PackCache keeps, per packed view of a parameter (arch 1's dense layers viewed as
    convolutions), the view's geometry on its base.  When the parameter's storage is later
    swapped for a smaller one (``p.data = ...``), rebuilding that view would read past the
    storage: _weight returns None and refresh / layouts_of drop the entry instead of raising
    inside the optimizer step (advisor, round 5)."""
    import weakref
    from relativisticgan_amd import kernels as K
    cache = K._PackCache()
    p = torch.nn.Parameter(torch.randn(8192, 128))
    view = p.view(512, 4, 4, 128)
    geo = (tuple(view.shape), tuple(view.stride()), view.storage_offset())
    key = ("k",)
    ent = (weakref.ref(p), p._version, torch.empty(4), p.data_ptr(), None, 0, geo)
    cache.entries[key] = ent
    assert cache._weight(ent) is not None and tuple(cache._weight(ent).shape) == (512, 4, 4, 128)
    p.data = torch.randn(16, 128)  # smaller storage under the same parameter
    assert cache._weight(ent) is None
    assert cache.layouts_of([p]) == [] and key not in cache.entries
    cache.entries[key] = ent
    cache.refresh([p])  # no lib call: nothing current to repack
    assert key not in cache.entries
