"""The oracle's restatement of the reference's --n_gpu data_parallel forward (GLI:393,
GLI:455), which the per-shard-BN multi-GPU parity test (tests/test_dp_gpu.py) checks
against.  CPU; parity unpinned against the reference itself (no multi-GPU CUDA here):
these tests pin the restatement to torch's documented DataParallel behaviour."""
import torch
import torch.nn as nn

from oracle.reference_cpu import Trainer, data_parallel_emulated
from tests.oracle_replay import dataset_for, param_for


def test_scatter_gather_and_replica0_buffers():
    torch.manual_seed(0)
    net = nn.Sequential(nn.Conv2d(3, 8, 3, 1, 1), nn.BatchNorm2d(8), nn.ReLU())
    x = torch.randn(6, 3, 5, 5)
    ref = nn.Sequential(nn.Conv2d(3, 8, 3, 1, 1), nn.BatchNorm2d(8), nn.ReLU())
    ref.load_state_dict(net.state_dict())
    y = data_parallel_emulated(net, x, 2)
    # each replica normalises its own chunk (torch.chunk scatter), outputs concatenated
    ref1 = nn.Sequential(nn.Conv2d(3, 8, 3, 1, 1), nn.BatchNorm2d(8), nn.ReLU())
    ref1.load_state_dict(ref.state_dict())
    y0 = ref(x[:3])
    y1 = ref1(x[3:])
    assert torch.equal(y, torch.cat([y0, y1]))
    # replica 0's running statistics persist, replica 1's are discarded
    assert torch.equal(net[1].running_mean, ref[1].running_mean)
    assert torch.equal(net[1].running_var, ref[1].running_var)
    assert int(net[1].num_batches_tracked) == 1
    # gradients of the shared parameters sum over the replicas
    y.sum().backward()
    (y0.sum() + y1.sum()).backward()
    assert torch.allclose(net[0].weight.grad, ref[0].weight.grad + ref1[0].weight.grad, rtol=1e-5, atol=1e-6)
    # uneven batch: chunk sizes ceil(B/n), fewer replicas when B < n
    assert data_parallel_emulated(net, torch.randn(5, 3, 5, 5), 2).shape[0] == 5
    assert data_parallel_emulated(net, torch.randn(1, 3, 5, 5), 4).shape[0] == 1


def _step(name, shards, **extra):
    torch.set_num_threads(4)
    rec = {}

    def hooks(tag, r):
        if tag in ("D", "G"):
            rec[tag] = {k: v.detach().clone() for k, v in r.items()}
    t = Trainer(param_for(name, dp_shards=shards, **extra), dataset_for(name), hooks=hooks)
    t.iteration(0)
    return rec, t


def test_without_batchnorm_sharding_changes_nothing_but_rounding():
    a, ta = _step("ralsgan", 1, no_batch_norm_G=True, no_batch_norm_D=True)
    b, tb = _step("ralsgan", 2, no_batch_norm_G=True, no_batch_norm_D=True)
    for tag in ("D", "G"):
        for k in a[tag]:
            assert torch.allclose(a[tag][k], b[tag][k], rtol=1e-4, atol=1e-6), (tag, k)
    for (n, p), (_, q) in zip(ta.G.named_parameters(), tb.G.named_parameters()):
        assert (p - q).abs().max() <= 2 * 2 * 1e-4 * 1.01, n


def test_batchnorm_statistics_are_per_shard():
    a, _ = _step("ralsgan", 1)
    b, _ = _step("ralsgan", 2)
    assert torch.equal(a["D"]["x"], b["D"]["x"])          # same inputs
    assert not torch.allclose(a["D"]["y_pred"], b["D"]["y_pred"], rtol=1e-3)  # different BN stats
