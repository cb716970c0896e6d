"""Data-parallel algebra on CPU: world_size-2 gloo processes (no GPU).

Checks the collective helpers of relativisticgan_amd.dp and the exchange protocol the
build uses against single-process global-batch math:
  * SyncBN forward: per-rank (count, mean, M2) all-gathered and merged in rank order
    == the global batch statistics;
  * SyncBN backward: all-reduced (sum g, sum g*(y-mean)) == global sums;
  * relativistic loss heads: the 3-phase protocol (local sums of r/f -> all-reduce ->
    local sums of a, b, a', b' -> all-reduce -> grads) reproduces the global-batch loss
    and gradients of the reference expressions (GLI:634-641, 698-709);
  * bucketed gradient all-reduce == per-tensor sum.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.reference_cpu import head_G, head_relativistic_D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from relativisticgan_amd import dp
    dp.setup()
    return dp


def _local_moments(y):
    C = y.shape[1]
    t = y.transpose(0, 1).reshape(C, -1).double()
    n = torch.full((C,), float(t.shape[1]), dtype=torch.float64)
    mean = t.mean(1)
    m2 = ((t - mean[:, None]) ** 2).sum(1)
    return torch.cat([n, mean, m2])


def _ra_terms(kind, side, r, f, mr, mf):
    """Per-element a(r - m_f), b(f - m_r) and derivatives."""
    g = side == 2
    dr_, df_ = r - mf, f - mr
    sp = torch.nn.functional.softplus
    if kind == 6:
        a = sp(dr_) if g else sp(-dr_)
        da = torch.sigmoid(dr_) if g else torch.sigmoid(dr_) - 1
        b = sp(-df_) if g else sp(df_)
        db = torch.sigmoid(df_) - 1 if g else torch.sigmoid(df_)
    elif kind == 7:
        sa, sb = (dr_ + 1, df_ - 1) if g else (dr_ - 1, df_ + 1)
        a, da, b, db = sa * sa, 2 * sa, sb * sb, 2 * sb
    else:
        ha, hb = (1 + dr_, 1 - df_) if g else (1 - dr_, 1 + df_)
        a, b = ha.clamp_min(0), hb.clamp_min(0)
        da = (ha > 0).double() * (1 if g else -1)
        db = (hb > 0).double() * (-1 if g else 1)
    return a, b, da, db


def _worker(rank, world, port, q):
    try:
        dp = _init(rank, world, port)
        torch.manual_seed(0)
        B, C = 16, 6
        y = torch.randn(B, C, 5, 5, dtype=torch.float64) * 3 + 1
        r_all = torch.randn(B, dtype=torch.float64)
        f_all = torch.randn(B, dtype=torch.float64)
        lo, hi = rank * B // world, (rank + 1) * B // world
        # SyncBN forward
        mom = dp.all_gather_cat(_local_moments(y[lo:hi]))
        mean, var, n = dp.merge_moments(mom, C)
        assert torch.allclose(mean, y.mean((0, 2, 3)), atol=1e-12)
        assert torch.allclose(var, y.var((0, 2, 3), unbiased=False), atol=1e-12)
        assert torch.all(n == B * 25)
        # SyncBN backward sums
        g = torch.randn_like(y)
        loc = torch.cat([g[lo:hi].sum((0, 2, 3)), (g[lo:hi] * (y[lo:hi] - mean.view(1, -1, 1, 1))).sum((0, 2, 3))])
        dp.all_reduce_sum(loc)
        glob = torch.cat([g.sum((0, 2, 3)), (g * (y - mean.view(1, -1, 1, 1))).sum((0, 2, 3))])
        assert torch.allclose(loc, glob, atol=1e-10)
        # relativistic heads, 3-phase protocol vs the reference expressions on the global batch
        ones, zeros = torch.ones(B, dtype=torch.float64), torch.zeros(B, dtype=torch.float64)
        for kind in (6, 7, 8):
            for side in (0, 2):
                r, f = r_all[lo:hi], f_all[lo:hi]
                s = dp.all_reduce_sum(torch.stack([r.sum(), f.sum()]))
                mr, mf = s[0] / B, s[1] / B
                a, b, da, db = _ra_terms(kind, side, r, f, mr, mf)
                s2 = dp.all_reduce_sum(torch.stack([a.sum(), b.sum(), da.sum(), db.sum()]))
                loss = (s2[0] / B + s2[1] / B) / 2
                grad_r = 0.5 / B * (da - s2[3] / B)
                grad_f = 0.5 / B * (db - s2[2] / B)
                rr = r_all.clone().requires_grad_(True)
                ff = f_all.clone().requires_grad_(True)
                ref = (head_relativistic_D(kind, rr, ff, ones, zeros) if side == 0
                       else head_G(kind, ff, rr, ones, zeros))
                ref.backward()
                assert abs(loss.item() - ref.item()) < 1e-12, (kind, side)
                assert torch.allclose(grad_r, rr.grad[lo:hi], atol=1e-12), (kind, side)
                assert torch.allclose(grad_f, ff.grad[lo:hi], atol=1e-12), (kind, side)
        # bucketed gradient all-reduce
        ps = [torch.nn.Parameter(torch.zeros(s)) for s in ((3, 4), (7,), (2, 2, 2))]
        for k, prm in enumerate(ps):
            prm.grad = torch.full(prm.shape, float(rank + 1 + k))
        dp.allreduce_grads(ps, bucket_bytes=40)
        for k, prm in enumerate(ps):
            assert torch.all(prm.grad == sum(rk + 1 + k for rk in range(world)))
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_dp_collectives_and_protocol_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(120)
    res = [q.get() for _ in range(world)]
    assert all(msg == "ok" for _, msg in res), res


def _make_params(seed=3):
    torch.manual_seed(seed)
    shapes = [(16, 6), (16,), (8, 16), (8,), (1, 8), (1,), (5,)]
    return [torch.nn.Parameter(torch.randn(sh) * 0.5) for sh in shapes]


def _losses(params, rank):
    """Two losses of rank ``rank``; the last parameter gets a gradient from loss 1 only."""
    w1, b1, w2, b2, w3, b3, extra = params
    g = torch.Generator().manual_seed(100 + rank)
    x1, x2 = torch.randn(4, 6, generator=g), torch.randn(4, 6, generator=g)

    def f(x):
        h = torch.tanh(x @ w1.t() + b1)
        h = torch.tanh(h @ w2.t() + b2)
        return h @ w3.t() + b3
    return f(x1).pow(2).mean() + (extra * (rank + 1)).sum(), f(x2).sin().mean()


def _reducer_worker(rank, world, port, q):
    try:
        dp = _init(rank, world, port)
        params = _make_params()
        red = dp.GradReducer(params, bucket_bytes=60)  # several buckets
        assert len(red.buckets) > 2
        ref = _make_params()
        want = [torch.zeros_like(prm) for prm in params]
        for rk in range(world):
            l1, l2 = _losses(ref, rk)
            for w_, g_ in zip(want, torch.autograd.grad(l1 + l2, ref)):
                w_ += g_
        for step in range(2):  # the reducer re-arms cleanly on the next step
            for prm in params:
                prm.grad = None
            l1, l2 = _losses(params, rank)
            l1.backward()  # first backward: not armed
            red.arm()
            l2.backward()  # last backward: buckets launch from the hooks
            red.finish()
            for prm, w_ in zip(params, want):
                assert torch.allclose(prm.grad, w_, atol=1e-6), (step, prm.shape)
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_overlapped_grad_reducer_gloo_world2():
    """dp.GradReducer: buckets launched from post-accumulate hooks during the last
    backward (own communicator), grads from earlier backwards included, == global SUM."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_reducer_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(120)
    res = [q.get() for _ in range(world)]
    assert all(msg == "ok" for _, msg in res), res


def _seed_worker(rank, world, port, q):
    try:
        dp = _init(rank, world, port)
        from relativisticgan_amd.config import make_param
        from relativisticgan_amd.train import Trainer, synthetic_images
        # no --seed: each rank would draw its own random seed; rank 0's must win
        import random
        random.seed(1000 + rank)
        p = make_param(loss_D=7, image_size=32, batch_size=8, z_size=16, G_h_size=8, D_h_size=8, seed=None)
        t = Trainer(p, synthetic_images(16, 32, device="cpu"), device="cpu")
        seeds = [None] * world
        dist.all_gather_object(seeds, p.seed)
        assert len(set(seeds)) == 1, seeds
        flat = torch.cat([v.reshape(-1).float() for v in list(t.G.state_dict().values()) +
                          list(t.D.state_dict().values())])
        z = t.z_test.reshape(-1)
        all_flat = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(all_flat, flat)
        assert all(torch.equal(all_flat[0], f) for f in all_flat), "replicas start from different weights"
        all_z = [torch.empty_like(z) for _ in range(world)]
        dist.all_gather(all_z, z.contiguous())
        assert not torch.equal(all_z[0], all_z[1]), "z_test shards must differ (one global draw, sliced)"
        # --n_gpu must match the process count (GLI:393-394 data_parallel is per-process here)
        try:
            Trainer(make_param(loss_D=7, image_size=32, batch_size=8, z_size=16, G_h_size=8, D_h_size=8, seed=1,
                               n_gpu=4), synthetic_images(16, 32, device="cpu"), device="cpu")
            raise AssertionError("--n_gpu 4 with 2 processes was accepted")
        except ValueError:
            pass
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_dp_unseeded_replicas_agree_gloo_world2():
    """Without --seed every rank draws random.randint; the Trainer broadcasts rank 0's
    seed so the replicas start from identical weights."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_seed_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(180)
    res = [q.get() for _ in range(world)]
    assert all(msg == "ok" for _, msg in res), res


def test_n_gpu_without_processes_fails_loudly():
    """A single process with --n_gpu 2 would silently use whole-batch BN (GLI:455-456 runs
    data_parallel with per-shard BN): the build refuses instead."""
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.train import Trainer, synthetic_images
    p = make_param(loss_D=7, image_size=32, batch_size=8, z_size=16, G_h_size=8, D_h_size=8, seed=1, n_gpu=2)
    with pytest.raises(ValueError, match="n_gpu"):
        Trainer(p, synthetic_images(16, 32, device="cpu"), device="cpu")


class _WgradLike(torch.autograd.Function):
    """y = x * w; backward writes dL/dw the way the fused conv layers do under data
    parallelism: into w's gradient-bucket slice when dp.grad_view hands one out."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x * w

    @staticmethod
    def backward(ctx, g):
        from relativisticgan_amd import dp
        x, w = ctx.saved_tensors
        dw = (g * x).sum(0)
        into = dp.grad_view(w)
        if into is not None:
            into.copy_(dw)
            dw = into
        return g * w, dw


def _bucket_view_worker(rank, world, port, q):
    try:
        dp = _init(rank, world, port)
        g = torch.Generator().manual_seed(7)
        w1 = torch.nn.Parameter(torch.randn(5, generator=g))
        w2 = torch.nn.Parameter(torch.randn(3, generator=g))
        bn = torch.nn.Parameter(torch.randn(4, generator=g))   # gradient produced outside the bucket
        red = dp.GradReducer([w1, w2, bn], bucket_bytes=1 << 20)
        assert len(red.buckets) == 1

        def losses(rk):
            gx = torch.Generator().manual_seed(50 + rk)
            xa, xb = torch.randn(6, 5, generator=gx), torch.randn(6, 5, generator=gx)
            # w1 used twice in ONE backward (as D(x), D(fake)): one slice, summed correctly
            ya, yb = _WgradLike.apply(xa, w1), _WgradLike.apply(xb, w1)
            y2 = _WgradLike.apply(torch.randn(2, 3, generator=gx), w2)
            return ya.pow(2).mean() + yb.sin().mean() + y2.sum() + (bn * (rk + 1)).pow(2).sum()

        want = [torch.zeros_like(t) for t in (w1, w2, bn)]
        for rk in range(world):
            ref = [t.detach().clone().requires_grad_(True) for t in (w1, w2, bn)]
            gx = torch.Generator().manual_seed(50 + rk)
            xa, xb = torch.randn(6, 5, generator=gx), torch.randn(6, 5, generator=gx)
            x2 = torch.randn(2, 3, generator=gx)
            lref = (xa * ref[0]).pow(2).mean() + (xb * ref[0]).sin().mean() + (x2 * ref[1]).sum() + \
                (ref[2] * (rk + 1)).pow(2).sum()
            for w_, g_ in zip(want, torch.autograd.grad(lref, ref)):
                w_ += g_
        for step in range(2):
            for t in (w1, w2, bn):
                t.grad = None
            red.arm()
            losses(rank).backward()
            # the layer-written gradients are the bucket's own storage (no copy)
            flat = red.flats[0]
            assert w2.grad.data_ptr() == flat[red.offset[id(w2)]:].data_ptr()
            red.finish()
            for t, w_ in zip((w1, w2, bn), want):
                assert torch.allclose(t.grad, w_, atol=1e-5), (step, t.shape)
                assert flat.data_ptr() <= t.grad.data_ptr() < flat.data_ptr() + 4 * flat.numel()
        assert dp.grad_view(w1) is None  # has a gradient now
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_gradient_bucket_views_gloo_world2():
    """Gradient-as-bucket-view: layers write weight gradients into their bucket slices
    (dp.grad_view), autograd adopts them as .grad, the bucket is all-reduced in place
    (gradients produced elsewhere are copied in), a weight used by two calls in one
    backward gets its slice once, and the result is the global SUM."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_view_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(120)
    res = [q.get() for _ in range(world)]
    assert all(msg == "ok" for _, msg in res), res


def _forced_worker(rank, world, port, q):
    try:
        dp = _init(rank, world, port)
        assert not dp.active()  # one rank: plain single-process mode by default
        dp.setup(force=True)
        assert dp.active() and dp.world() == 1 and dp._S.grad_group is not None
        t = torch.arange(6.0)
        assert torch.equal(dp.all_reduce_sum(t.clone()), t)
        assert torch.equal(dp.all_gather_cat(t), t)
        params = _make_params()
        red = dp.GradReducer(params, bucket_bytes=60)
        ref = _make_params()
        l1, l2 = _losses(ref, 0)
        want = torch.autograd.grad(l1 + l2, ref)
        l1, l2 = _losses(params, 0)
        l1.backward()
        red.arm()
        l2.backward()
        red.finish()
        for prm, w_ in zip(params, want):
            assert torch.allclose(prm.grad, w_, atol=1e-6)
        # finish() ran the forced rank's wait / rebind path: nothing left in flight, the
        # per-step hand-out set cleared, and every .grad is its slice of the reduced bucket
        assert red.inflight == [] and red.handed == set() and not red.armed
        for prm in params:
            bi, off = red.where[id(prm)], red.offset[id(prm)]
            assert prm.grad.data_ptr() == red.region(bi, off, prm).data_ptr()
        # a second step re-arms and hands out slices again
        for prm in params:
            prm.grad = None
        l1, l2 = _losses(params, 0)
        l1.backward()
        red.arm()
        l2.backward()
        red.finish()
        for prm, w_ in zip(params, want):
            assert torch.allclose(prm.grad, w_, atol=1e-6)
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        from relativisticgan_amd import dp as _dp
        _dp.reset()
        if dist.is_initialized():
            dist.destroy_process_group()


def test_forced_dp_one_rank_gloo():
    """dp.setup(force=True) with one rank (the one-GPU rehearsal of the RCCL path,
    bench.py --force-dp): the machinery switches on -- second communicator, collectives,
    bucketed reducer -- and every exchange is the identity."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    pr = ctx.Process(target=_forced_worker, args=(0, 1, _free_port(), q))
    pr.start()
    pr.join(120)
    res = q.get()
    assert res[1] == "ok", res
