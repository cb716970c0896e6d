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

from . import dp
from .config import TITLES, parse
from .losses import gradient_penalty, loss_D, loss_D_fake, loss_D_real, loss_G
from .nets import DCGAN_D, DCGAN_G, weights_init
from .optim import Adam


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
        if seed_all:
            if p.seed is None:
                p.seed = random.randint(1, 10000)
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
        # gradient SUM all-reduce overlapped with the last backward of each step (world > 1)
        self.redD = dp.GradReducer(self.D.parameters()) if self.world > 1 else None
        self.redG = dp.GradReducer(self.G.parameters()) if self.world > 1 else None
        self.host_rng = getattr(p, "rgan_rng", "host") == "host"
        self.errD = self.errG = None
        self.last = {}

    # -- inputs (host order = reference order; device = throughput mode)
    def _shard(self, t):
        return t[self.rank * self.B:(self.rank + 1) * self.B]

    def _real(self, feed, key):
        if feed is not None and key in feed:
            return feed[key]
        from .kernels import gather_images
        if self.host_rng:
            idx = numpy.random.choice(self.images.shape[0], size=self.p.batch_size, replace=False)
            idx = self._shard(torch.from_numpy(idx.astype(numpy.int64))).to(self.device, non_blocking=True)
        else:
            idx = torch.randperm(self.images.shape[0], device=self.device)[:self.p.batch_size]
            idx = self._shard(idx)
        return gather_images(self.images, idx)

    def _normal(self, feed, key, shape):
        if feed is not None and key in feed:
            return feed[key]
        if self.host_rng:
            return self._shard(torch.empty(shape).normal_(0, 1)).to(self.device, non_blocking=True)
        # every rank draws the global batch from the same device generator and keeps its
        # shard: ranks see different z, and the union is the 1-process draw
        return self._shard(torch.randn(shape, device=self.device))

    def _uniform(self, feed, key, shape):
        if feed is not None and key in feed:
            return feed[key]
        if self.host_rng:
            return self._shard(torch.empty(shape).uniform_(0, 1)).to(self.device, non_blocking=True)
        return self._shard(torch.rand(shape, device=self.device))

    @staticmethod
    def _arm(red):
        if red is not None:
            red.arm()

    def _set_D_grad(self, flag):
        for q in self.D.parameters():
            q.requires_grad = flag

    # -- one iteration (GLI:560-714)
    def iteration(self, i, feed=None, hooks=None):
        p, D, G = self.p, self.D, self.G
        kind = p.loss_D
        gp_on = kind == 3 or p.grad_penalty
        zshape = (p.batch_size, p.z_size, 1, 1)
        if i % p.print_every == 0:
            with torch.no_grad():
                self.fake_test = G(self.z_test)  # GLI:564 (sample image; BN running stats move)
        self._set_D_grad(True)
        for _ in range(p.Diters):
            D.zero_grad()
            x = self._real(feed, "x_D")
            y_pred = D(x)
            if kind <= 4:
                err_real = loss_D_real(kind, y_pred)
                err_real.backward()
                z = self._normal(feed, "z_D", zshape)
                with torch.no_grad():
                    x_fake = G(z)
                y_pred_fake = D(x_fake)
                err_fake = loss_D_fake(kind, y_pred_fake)
                if not gp_on:
                    self._arm(self.redD)
                err_fake.backward()
                errD = err_real.detach() + err_fake.detach()
            else:
                z = self._normal(feed, "z_D", zshape)
                with torch.no_grad():
                    x_fake = G(z)
                y_pred_fake = D(x_fake)
                errD = loss_D(kind, y_pred, y_pred_fake)
                if not gp_on:
                    self._arm(self.redD)
                errD.backward()
            rec = {"x": x, "z": z, "y_pred": y_pred.detach(), "y_pred_fake": y_pred_fake.detach(),
                   "errD": errD.detach()}
            if gp_on:
                u = self._uniform(feed, "u", (p.batch_size, 1, 1, 1))
                gp = gradient_penalty(D, x, x_fake, u, p.penalty)
                self._arm(self.redD)
                gp.backward()
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
            G.zero_grad()
            z = self._normal(feed, "z_G", zshape)
            fake = G(z)
            y_pred_fake = D(fake)
            y_pred = None
            recG = {"z": z}
            if kind > 4:
                x = self._real(feed, "x_G")
                with torch.no_grad():
                    y_pred = D(x)
                recG.update(x=x, y_pred=y_pred)
            errG = loss_G(kind, y_pred_fake, y_pred)
            self._arm(self.redG)
            errG.backward()
            recG.update(y_pred_fake=y_pred_fake.detach(), errG=errG.detach())
            if self.redG is not None:
                self.redG.finish()
            if hooks:
                hooks("G", recG)
            self.optG.step()
            if hooks:
                hooks("G.post", recG)
        self.errG = errG
        self.last["G"] = recG
        self.decayD.step()
        self.decayG.step()

    # -- checkpoint (GLI:536-552, 733-747): same dict keys as the reference
    def state(self, i, current_set_images=0):
        return {"i": i, "current_set_images": current_set_images, "G_state": self.G.state_dict(),
                "D_state": self.D.state_dict(), "G_optimizer": self.optG.state_dict(),
                "D_optimizer": self.optD.state_dict(), "G_scheduler": self.decayG.state_dict(),
                "D_scheduler": self.decayD.state_dict(), "z_test": self.z_test}

    def load(self, ckpt):
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


def main(argv=None):
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
    n = p.rgan_synthetic or 1024
    images = synthetic_images(n, p.image_size, p.n_colors)
    t = Trainer(p, images)
    print(p)
    print(f"Random Seed: {p.seed}")
    iter_offset, current_set_images = 0, 0
    if p.load:
        iter_offset, current_set_images = t.load(torch.load(p.load, map_location="cuda", weights_only=False))
    print(t.G)
    print(t.D)
    for i in range(iter_offset, p.n_iter):
        t.iteration(i)
        if (i + 1) % p.print_every == 0 and dp.rank() == 0:
            print(t.log_line(i, time.time() - start), flush=True)
        if (i + 1) % p.gen_every == 0:
            current_set_images += 1
            if p.save and dp.rank() == 0:
                os.makedirs(os.path.join(p.extra_folder, "models"), exist_ok=True)
                torch.save(t.state(i + 1, current_set_images),
                           os.path.join(p.extra_folder, "models", "state_%02d.pth" % current_set_images))
                print("Models saved")
    return t


if __name__ == "__main__":
    main(sys.argv[1:])
