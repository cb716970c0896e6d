"""The reference's training loop (GLI:559-714) on the MI355X build.

``Trainer`` reproduces the loop body's exact call order -- sample-image G(z_test)
every ``print_every`` (it mutates G's BN running stats, GLI:563-565), D step with the
two-backward heads 1-4 / one-backward heads 5-8, optional WGAN-GP, D Adam, G step
with a fresh real batch and a no-graph D(x) for heads 5-8, G Adam, LR decay -- and
the reference's RNG consumption order when ``rgan_rng == 'host'``.

Run as a script it is the reference CLI (``python -m relativisticgan_amd.train --loss_D 7 ...``)
with synthetic images (``--rgan_synthetic N``; torchvision / image folders are out of
scope), the same log line (GLI:723) and the same checkpoint dict (GLI:737-747).
"""
import os
import random
import sys
import time

import numpy
import torch

from . import autograd, dp
from .config import TITLES, parse
from .kernels import DeviceRNG
from .losses import gradient_penalty, loss_D, loss_D_cat, loss_D_fake, loss_D_real, loss_G, loss_G_cat, unit_seed
from .nets import DCGAN_D, DCGAN_G, weights_init
from .optim import Adam
from .perf import ThroughputMeter


def synthetic_images(n, size, n_colors=3, seed=1234, device="cuda"):
    """uint8 -> (u8/255 - 0.5)/0.5, the bench/fixture image set."""
    g = torch.Generator().manual_seed(seed)
    u8 = torch.randint(0, 256, (n, n_colors, size, size), generator=g, dtype=torch.uint8)
    return ((u8.float() / 255.0 - 0.5) / 0.5).to(device)


class Trainer:
    """State of one training run (G, D, optimizers, schedulers, buffers)."""

    def __init__(self, param, images, device="cuda", seed_all=True):
        p = self.p = param
        self.device = torch.device(device)
        world = dp.world()
        n_gpu = getattr(p, "n_gpu", 1) or 1
        if n_gpu > 1 and n_gpu != world:
            # GLI:393-394,455-456: --n_gpu N runs torch's data_parallel over N GPUs inside
            # forward (per-shard BatchNorm).  Here every GPU is its own process: a single
            # process would silently train with whole-batch BN statistics instead.
            raise ValueError(f"--n_gpu {n_gpu} with {world} process(es): launch one process per GPU "
                             f"(torchrun --nproc-per-node {n_gpu}); each rank then normalises its own shard "
                             "like the reference's data_parallel")
        if seed_all:
            if p.seed is None:
                p.seed = random.randint(1, 10000)
            if world > 1:
                # every replica must start from the same weights / z_test / batch draws:
                # rank 0's (possibly random) seed is everyone's
                import torch.distributed as dist
                box = [p.seed]
                dist.broadcast_object_list(box, src=0, group=dp.group())
                p.seed = box[0]
            random.seed(p.seed)
            numpy.random.seed(p.seed)
            torch.manual_seed(p.seed)
        self.images = images
        self.world, self.rank = dp.world(), dp.rank()
        if p.batch_size % self.world:
            raise ValueError(f"batch_size {p.batch_size} not divisible by {self.world} ranks")
        self.B = p.batch_size // self.world
        # construction + init on the CPU generator: same draws as the reference (GLI:463-477)
        self.G = DCGAN_G(p)
        self.D = DCGAN_D(p)
        self.G.apply(weights_init)
        self.D.apply(weights_init)
        z_test = torch.FloatTensor(p.batch_size, p.z_size, 1, 1).normal_(0, 1)  # GLI:497
        self.G.to(self.device)
        self.D.to(self.device)
        self.z_test = self._shard(z_test).to(self.device)
        self.optD = Adam(self.D.parameters(), lr=p.lr_D, betas=(p.beta1, p.beta2), weight_decay=p.weight_decay)
        self.optG = Adam(self.G.parameters(), lr=p.lr_G, betas=(p.beta1, p.beta2), weight_decay=p.weight_decay)
        self.decayD = torch.optim.lr_scheduler.ExponentialLR(self.optD, gamma=1 - p.decay)
        self.decayG = torch.optim.lr_scheduler.ExponentialLR(self.optG, gamma=1 - p.decay)
        # gradient SUM all-reduce overlapped with the last backward of each step (world > 1,
        # or the data-parallel path forced on one rank: dp.setup(force=True))
        self.redD = dp.GradReducer(self.D.parameters()) if dp.active() else None
        self.redG = dp.GradReducer(self.G.parameters()) if dp.active() else None
        self._pending_G, self._pending_decay_G = None, False
        # under DP, G's optimizer step waits for the next use of G (flush) so its gradient
        # all-reduce overlaps the next D forward; a PiecewiseGraph capture steps it in place
        self.defer_G = True
        self.host_rng = getattr(p, "rgan_rng", "host") == "host"
        if not self.host_rng and self.device.type != "cuda":
            raise ValueError("--rgan_rng device draws in HIP kernels: it needs a CUDA (HIP) device, "
                             f"got {self.device}; use --rgan_rng host")
        # --rgan_rng device: counter-based draws in HIP kernels (same seed on every rank)
        self.dev_rng = (None if self.host_rng else
                        DeviceRNG(p.seed if p.seed is not None else torch.initial_seed(), self.device))
        self.pac = getattr(p, "pac", 1)  # 2: code/GAN_losses_iter_PAC.py
        # one batched D pass per D step where the nets allow it (--rgan_batch_D).  Default
        # (auto): on, under data parallelism too.  G's gradient buckets all-reduce while G's
        # own backward runs (GradReducer), so the deferred G step (flush, right before the
        # batched pass's G(z)) only waits for the last bucket; separate D(x) / D(x_fake)
        # passes would hide that tail behind D(x) but cost ~2 % more kernel time at C3
        # (bench dp_path_n1, round 5: 436.8 vs 446.0 img/s)
        bd = getattr(p, "rgan_batch_D", None)
        bd = True if bd is None else bool(bd)
        self.batch_D = bd and self.pac == 1 and self.D.segmentable
        # the G step's D(G(z)) and D(x) (heads 5-8) as one batched pass (--rgan_batch_G,
        # default on, under data parallelism too: nothing overlaps with its D(x) forward)
        bg = getattr(p, "rgan_batch_G", None)
        self.batch_G = (True if bg is None else bool(bg)) and self.pac == 1 and self.D.segmentable
        self._fake_D = None
        self._one = None
        self.errD = self.errG = None
        self.last = {}
        # set by whoever captures iterations into HIP graphs (bench.py, dp.PiecewiseGraph users):
        # replays advance the device-side state only (Adam's device step counters, the device
        # LR), while the host mirrors (state['step'], the schedulers) froze at capture time
        self.graph_captured = False

    # -- inputs (host order = reference order; device = throughput mode)
    def _shard(self, t):
        return t[self.rank * self.B:(self.rank + 1) * self.B]

    def _shard_pac(self, t):
        """Global [pac*B, ...] draw -> this rank's [pac*B_local, ...] (each packing slot's
        shard, so packing the local part gives the rank's shard of the packed batch)."""
        if self.pac == 1:
            return self._shard(t)
        B = self.p.batch_size
        return torch.cat([t[k * B + self.rank * self.B:k * B + (self.rank + 1) * self.B] for k in range(self.pac)])

    def _pack(self, t):
        """[pac*b, C, ...] -> [b, pac*C, ...]: torch.cat([t[0:b], t[b:2b]], 1) (PAC:582,609,674,682)."""
        if self.pac == 1:
            return t
        b = t.shape[0] // self.pac
        return torch.cat([t[k * b:(k + 1) * b] for k in range(self.pac)], 1)

    def _real(self, feed, key, out=None):
        if feed is not None and key in feed:
            return feed[key]
        from .kernels import gather_images
        n = self.p.batch_size * self.pac
        if self.host_rng:
            idx = numpy.random.choice(self.images.shape[0], size=n, replace=False)
            idx = self._shard_pac(torch.from_numpy(idx.astype(numpy.int64))).to(self.device, non_blocking=True)
        else:
            idx = self._shard_pac(self.dev_rng.choice(self.images.shape[0], n))
        return self._pack(gather_images(self.images, idx, out=out if self.pac == 1 else None))

    def _normal(self, feed, key, shape):
        if feed is not None and key in feed:
            return feed[key]
        if self.host_rng:
            return self._shard_pac(torch.empty(shape).normal_(0, 1)).to(self.device, non_blocking=True)
        # every rank draws the global batch from the same device generator and keeps its
        # shard: ranks see different z, and the union is the 1-process draw
        return self._shard_pac(self.dev_rng.normal(shape))

    def _uniform(self, feed, key, shape):
        if feed is not None and key in feed:
            return feed[key]
        if self.host_rng:
            return self._shard(torch.empty(shape).uniform_(0, 1)).to(self.device, non_blocking=True)
        return self._shard(self.dev_rng.uniform(shape))

    def _generate_D(self, z, out=None):
        """The D step's fake batch.  Single samples: G(z) without a graph (GLI copies it into
        x_fake's .data), written into ``out`` when given.  PacGAN: keep G's graph for the G
        step (PAC:674) and pack."""
        if self.pac == 1:
            with torch.no_grad():
                return self.G(z, out=out)
        self._zbuf = z.clone()  # the reference's persistent z buffer (GLI:490)
        self._fake_D = self.G(self._zbuf)
        return self._pack(self._fake_D).detach()

    @staticmethod
    def _arm(red):
        if red is not None:
            red.arm()

    def _backward(self, loss):
        """loss.backward() (GLI:605/624/644/658/710) with a cached device 1.0 as the seed
        gradient (autograd would fill a fresh ones tensor on every call)."""
        one = self._one
        if one is None or one.device != loss.device or one.dtype != loss.dtype:
            one = self._one = unit_seed(loss.device, loss.dtype)
        with autograd.owning_grads():  # the fused layers write their weight .grad directly
            loss.backward(one)

    def _set_D_grad(self, flag):
        for q in self.D.parameters():
            q.requires_grad = flag

    # -- one iteration (GLI:560-714)
    def iteration(self, i, feed=None, hooks=None):
        p, D, G = self.p, self.D, self.G
        kind = p.loss_D
        gp_on = kind == 3 or p.grad_penalty
        zshape = (p.batch_size * self.pac, p.z_size, 1, 1)
        if i % p.print_every == 0:
            self.flush()
            with torch.no_grad():
                self.fake_test = G(self.z_test)  # GLI:564 (sample image; BN running stats move)
        self._set_D_grad(True)
        for _ in range(p.Diters):
            D.zero_grad()
            pair = None
            if self.batch_D and self.pac == 1:
                # the real batch and G's fake batch are written back to back into one buffer:
                # the batched D pass reads it as is (no concatenation)
                pair = torch.empty((2 * self.B, p.n_colors, p.image_size, p.image_size), dtype=torch.float32,
                                   device=self.device)
            x = self._real(feed, "x_D", out=pair[:self.B] if pair is not None else None)
            if self.batch_D:
                # D(x) and D(x_fake) as one batched pass (per-call BN statistics kept):
                # the draws keep the reference's order (x, then z); D(x) does not read G
                z = self._normal(feed, "z_D", zshape)
                self.flush()
                x_fake = self._generate_D(z, out=pair[self.B:] if pair is not None else None)
                laid_out = (pair is not None and x.data_ptr() == pair.data_ptr()
                            and x_fake.data_ptr() == pair[self.B:].data_ptr())
                y_all = D.forward_pair(x, x_fake, cat=pair if laid_out else None)
                y_pred, y_pred_fake = y_all[:self.B], y_all[self.B:]
                # heads 1-4: err_real.backward(); err_fake.backward() accumulate = one backward
                # of the sum (GLI:605, 624); heads 5-8: errD.backward() (GLI:644)
                errD = loss_D_cat(kind, y_all)
                if not gp_on:
                    self._arm(self.redD)
                self._backward(errD)
                errD = errD.detach()
            elif kind <= 4:
                y_pred = D(x)
                err_real = loss_D_real(kind, y_pred)
                self._backward(err_real)
                z = self._normal(feed, "z_D", zshape)
                self.flush()
                x_fake = self._generate_D(z)
                y_pred_fake = D(x_fake)
                err_fake = loss_D_fake(kind, y_pred_fake)
                if not gp_on:
                    self._arm(self.redD)
                self._backward(err_fake)
                errD = err_real.detach() + err_fake.detach()
            else:
                y_pred = D(x)
                z = self._normal(feed, "z_D", zshape)
                self.flush()
                x_fake = self._generate_D(z)
                y_pred_fake = D(x_fake)
                errD = loss_D(kind, y_pred, y_pred_fake)
                if not gp_on:
                    self._arm(self.redD)
                self._backward(errD)
            rec = {"x": x, "z": z, "y_pred": y_pred.detach(), "y_pred_fake": y_pred_fake.detach(),
                   "errD": errD.detach()}
            if gp_on:
                u = self._uniform(feed, "u", (p.batch_size, 1, 1, 1))
                gp = gradient_penalty(D, x, x_fake, u, p.penalty)
                self._arm(self.redD)
                self._backward(gp)
                rec.update(u=u, gp=gp.detach())
            if self.redD is not None:
                self.redD.finish()
            if hooks:
                hooks("D", rec)
            self.optD.step()
            if hooks:
                hooks("D.post", rec)
        self.errD = errD
        self.last["D"] = rec
        self._set_D_grad(False)
        for _ in range(p.Giters):
            self.flush()
            G.zero_grad()
            z = self._normal(feed, "z_G", zshape)
            pair_G = None
            if self.batch_G and kind > 4:
                # D(G(z)) and the fresh real batch's D(x) as one batched pass: G writes its
                # output and the gather its images into one buffer, back to back
                pair_G = torch.empty((2 * self.B, p.n_colors, p.image_size, p.image_size), dtype=torch.float32,
                                     device=self.device)
                fake = G(z, out=pair_G[:self.B])
            elif self.pac == 1:
                fake = G(z)
            else:
                # PAC:673-674: the G step reuses the D step's G(z) (graph kept; G's weights
                # have not moved).  The fresh z is written into the persistent z buffer
                # through .data (PAC:673), which that graph saved for G's first layer without
                # a version bump: the first layer's weight gradient reads the NEW z.
                self._zbuf.data.copy_(z)
                fake, self._fake_D = self._pack(self._fake_D), None
            recG = {"z": z}
            if pair_G is not None:
                # GLI:674 then GLI:677-682 + 695-707: the draw order (z, then the real batch)
                # and the BN call order (D(fake), then D(x)) are the reference's
                x = self._real(feed, "x_G", out=pair_G[self.B:])
                laid_out = (fake.data_ptr() == pair_G.data_ptr()
                            and x.data_ptr() == pair_G[self.B:].data_ptr())
                y_all = D.forward_pair_G(fake, x, cat=pair_G if laid_out else None)
                y_pred_fake, y_pred = y_all[:self.B], y_all[self.B:].detach()
                recG.update(x=x, y_pred=y_pred)
                errG = loss_G_cat(kind, y_all)
            else:
                y_pred_fake = D(fake)
                y_pred = None
                if kind > 4:
                    x = self._real(feed, "x_G")
                    with torch.no_grad():
                        y_pred = D(x)
                    recG.update(x=x, y_pred=y_pred)
                errG = loss_G(kind, y_pred_fake, y_pred)
            self._arm(self.redG)
            self._backward(errG)
            recG.update(y_pred_fake=y_pred_fake.detach(), errG=errG.detach())
            self._pending_G = (hooks, recG)
            if self.redG is None or not self.defer_G:
                self._step_G()
        self.errG = errG
        self.last["G"] = recG
        self.decayD.step()
        if self._pending_G is None:
            self.decayG.step()
        else:
            self._pending_decay_G = True

    def _step_G(self):
        hooks, recG = self._pending_G
        self._pending_G = None
        if self.redG is not None:
            self.redG.finish()
        if hooks:
            hooks("G", recG)
        self.optG.step()
        if hooks:
            hooks("G.post", recG)

    def flush(self):
        """Under data parallelism G's optimizer step (and its LR decay) is deferred to the
        next use of G: the G gradients' all-reduce then overlaps the next iteration's
        real-batch D forward, which does not read G (GLI:580-590 draw x and run D(x) before
        G(z)).  The order of every draw and every result is unchanged.  Called before any
        G forward, before checkpoints, and by callers that stop iterating."""
        if self._pending_G is not None:
            self._step_G()
        if self._pending_decay_G:
            self._pending_decay_G = False
            self.decayG.step()

    # -- checkpoint (GLI:536-552, 733-747): same dict keys as the reference
    def state(self, i, current_set_images=0):
        if self.graph_captured:
            raise RuntimeError("Trainer.state(): iterations were replayed from a captured HIP graph, so the "
                               "host-side Adam step counts and LR schedulers are stale; checkpoint an eagerly "
                               "stepped trainer")
        self.flush()
        return {"i": i, "current_set_images": current_set_images, "G_state": self.G.state_dict(),
                "D_state": self.D.state_dict(), "G_optimizer": self.optG.state_dict(),
                "D_optimizer": self.optD.state_dict(), "G_scheduler": self.decayG.state_dict(),
                "D_scheduler": self.decayD.state_dict(), "z_test": _gather_batch(self.z_test)}

    def load(self, ckpt):
        self.flush()
        self.G.load_state_dict(ckpt["G_state"])
        self.D.load_state_dict(ckpt["D_state"])
        self.optG.load_state_dict(ckpt["G_optimizer"])
        self.optD.load_state_dict(ckpt["D_optimizer"])
        self.decayG.load_state_dict(ckpt["G_scheduler"])
        self.decayD.load_state_dict(ckpt["D_scheduler"])
        self.z_test.copy_(self._shard(ckpt["z_test"].to(self.device)) if ckpt["z_test"].shape[0] != self.B
                          else ckpt["z_test"])
        return ckpt["i"], ckpt["current_set_images"]

    def log_line(self, i, elapsed):
        """GLI:723."""
        d, g = self.errD.item(), self.errG.item()
        return '[%d] Diff: %.4f loss_D: %.4f loss_G: %.4f time:%.4f' % (i, -d + g, d, g, elapsed)


def _gather_batch(t):
    """Concatenate every rank's shard along the batch (rank order); identity on one rank."""
    if not dp.active():
        return t
    import torch.distributed as dist
    parts = [torch.empty_like(t) for _ in range(dp.world())]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts)


def load_images(p, device="cuda"):
    """The training set in HBM: --rgan_synthetic N synthetic images, or --input_folder as
    torchvision's ImageFolder + Resize + ToTensor + Normalize would give it (GLI:159-169),
    decoded once into uint8 (relativisticgan_amd.data)."""
    if p.rgan_synthetic:
        return synthetic_images(p.rgan_synthetic, p.image_size, p.n_colors, device=device)
    if p.CIFAR10:
        raise SystemExit("--CIFAR10: torchvision's CIFAR-10 loader unpickles python batches; convert the set "
                         "to an image folder and pass --input_folder instead")
    from .data import load_image_folder
    return load_image_folder(p.input_folder, p.image_size, p.n_colors, device=device)


def run_dirs(p, title):
    """GLI:86-100: <output_folder>/<title>-<run> with logs/ and images/ (first free run
    number); the extra-image folder is created when images will be generated."""
    run = 0
    base = f"{p.output_folder}/{title}-{run}"
    while os.path.exists(base):
        run += 1
        base = f"{p.output_folder}/{title}-{run}"
    os.makedirs(os.path.join(base, "logs"))
    os.makedirs(os.path.join(base, "images"))
    if p.gen_extra_images > 0:
        os.makedirs(p.extra_folder, exist_ok=True)
    return base


def generate_extra_images(G, p, folder, device="cuda"):
    """GLI:752-768: empty (or create) `folder`, then write gen_extra_images G samples,
    100 per G call, as fake_samples_%05d.png of fake*.5+.5.  G stays in train mode like the
    reference (its BN batch statistics and running stats move).  Under data parallelism
    every rank draws the same 100 z, runs its shard (SyncBN = the 100-batch statistics)
    and writes its shard's files."""
    from .images import save_images
    if dp.rank() == 0:
        if os.path.exists(folder):
            for root, _dirs, files in os.walk(folder):
                for f in files:
                    os.unlink(os.path.join(root, f))
        else:
            os.makedirs(folder)
    if dp.active():
        import torch.distributed as dist
        dist.barrier()
    world, rank = dp.world(), dp.rank()
    if 100 % world:
        raise ValueError(f"extra images are drawn 100 per batch: not divisible by {world} ranks")
    per = 100 // world
    ext_curr = 0
    with torch.no_grad():
        for _ in range(int(p.gen_extra_images / 100)):
            z = torch.randn(100, p.z_size, 1, 1, device=device)[rank * per:(rank + 1) * per]
            fake = G(z)
            save_images(fake, [os.path.join(folder, "fake_samples_%05d.png" % (ext_curr + rank * per + k))
                               for k in range(per)])
            ext_curr += 100


def main(argv=None):
    from .images import save_image
    p = parse(argv)
    start = time.time()
    if not torch.cuda.is_available():
        raise SystemExit("this build trains on MI355X GPUs only")
    if "RANK" in os.environ and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
        dp.setup(sync_bn=p.rgan_sync_bn)
    title = TITLES[p.loss_D] + ("seed%i" % p.seed if p.seed is not None else "")
    lead = dp.rank() == 0
    base = run_dirs(p, title) if lead else None
    log = open(os.path.join(base, "logs", "log.txt"), "w") if lead else None

    def say(s):
        if lead:
            print(s, flush=True)
            print(s, file=log, flush=True)
    images = load_images(p)
    t = Trainer(p, images)
    say(p)
    say(f"Random Seed: {p.seed}")
    iter_offset, current_set_images = 0, 0
    if p.load:
        iter_offset, current_set_images = t.load(torch.load(p.load, map_location="cuda", weights_only=True))
        say(f"Resumed from iteration {current_set_images * p.gen_every}.")
    say(t.G)
    say(t.D)
    meter = ThroughputMeter(t) if p.rgan_perf_log else None
    if meter is not None:
        meter.tick(iter_offset, time.time())
    def output_clock():
        """Start of host-side output work left out of the perf line's interval (the device
        finishes the queued training work first, so none of it is excluded)."""
        if meter is None:
            return None
        torch.cuda.synchronize()
        return time.time()

    def output_done(t_out):
        if t_out is not None:
            meter.exclude(time.time() - t_out)

    for i in range(iter_offset, p.n_iter):
        t.iteration(i)
        if i % p.print_every == 0:  # GLI:563-565 (the sample batch was drawn inside the iteration)
            t_out = output_clock()
            grid = _gather_batch(t.fake_test)
            if lead:
                save_image(grid, os.path.join(base, "images", "fake_samples_iter%05d.png" % i), normalize=True)
            output_done(t_out)
        if (i + 1) % p.print_every == 0:
            say(t.log_line(i, time.time() - start))  # the reference's line, unchanged (GLI:723-726)
            if meter is not None:  # plus img/s and MFMA%, on a line of its own
                perf = meter.tick(i + 1, time.time())
                if perf:
                    say(perf)
        if (i + 1) % p.gen_every == 0:
            t_out = output_clock()
            current_set_images += 1
            if p.save:
                st = t.state(i + 1, current_set_images)  # collective under DP (z_test shards)
                if lead:
                    os.makedirs(os.path.join(p.extra_folder, "models"), exist_ok=True)
                    torch.save(st, os.path.join(p.extra_folder, "models", "state_%02d.pth" % current_set_images))
                    say("Models saved")
            if p.gen_extra_images > 0:
                t.flush()
                generate_extra_images(t.G, p, "%s/%01d/" % (p.extra_folder, current_set_images))
            output_done(t_out)
    t.flush()
    if log:
        log.close()
    return t


if __name__ == "__main__":
    main(sys.argv[1:])
