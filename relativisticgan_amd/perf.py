"""Throughput accounting shared by the trainer's log line and bench.py.

``conv_flops_per_iteration`` is the algorithmic conv FLOP count of one reference iteration
(SURVEY §8(d)); ``MFMA%`` = those FLOPs per second over the fp32 MFMA peak of the GPUs that
ran them.
"""
import torch

FP32_MFMA_PEAK = 157.3e12  # MI355X_MICROARCH.md: Peak FP32 (matrix) = vector peak


def conv_flops_per_iteration(t):
    """Algorithmic conv FLOPs of one reference iteration, F = forward conv
    FLOPs (2*MACs) per net, d0/g0 = the image-side first layers (no data gradient needed):
      relativistic heads 5-8: 9 F_D + 4 F_G - 2 d0 - g0  (D step: D(x), D(fake) fwd+wgrad+
        dgrad, G fwd; G step: G fwd, D(fake) fwd + dgrad, G wgrad + dgrad, D(x) fwd);
      heads 1-4: the G step has no D(x): 8 F_D + 4 F_G - 2 d0 - g0;
      gradient penalty (GLI:646-658): + D(x_hat) fwd, its create-graph dgrad chain, and the
        double backward (adjoint conv fwd + wgrad per dgrad, then wgrad + dgrad back through
        the forward): 6 F_D - d0 - 3 F_end."""
    def layer_flops(net, x_shape):
        out, h = [], torch.zeros(x_shape, device="meta")
        for layer in net._plan:
            c = layer.conv
            geom = layer.spec.geom
            if layer.in_view is not None:
                h = torch.zeros((h.shape[0],) + tuple(layer.in_view), device="meta")
            B, cin, H, W = h.shape
            w = c.w if hasattr(c, "w") else c.weight
            if layer.w_view is not None:
                w = w.view(*layer.w_view)
            cout = w.shape[1] if geom.transposed else w.shape[0]
            Ho, Wo = geom.out_hw(H, W)
            pix = H * W if geom.transposed else Ho * Wo
            out.append(2.0 * B * cin * cout * geom.k * geom.k * pix)
            h = torch.zeros((B, cout, Ho, Wo), device="meta")
            if layer.out_view is not None:
                h = torch.zeros((B,) + tuple(layer.out_view), device="meta")
        return out
    p = t.p
    fg = layer_flops(t.G, (t.B, p.z_size, 1, 1))
    fd = layer_flops(t.D, (t.B, p.n_colors * getattr(p, "pac", 1), p.image_size, p.image_size))
    total = 9 * sum(fd) + 4 * sum(fg) - 2 * fd[0] - fg[0]
    if p.loss_D <= 4:
        total -= sum(fd)
    if p.loss_D == 3 or p.grad_penalty:
        total += 6 * sum(fd) - fd[0] - 3 * fd[-1]
    return total


class ThroughputMeter:
    """img/s and MFMA% between two log points of a training run (``train.main``): SURVEY §5's
    "same line, plus img/s and MFMA%".  ``tick(i)`` at a log point (after the reference line,
    whose ``.item()`` already waited for the GPU) returns the suffix line for the iterations
    since the previous tick."""

    def __init__(self, trainer):
        self.flops = conv_flops_per_iteration(trainer)  # this rank's share of the batch
        self.images = trainer.p.batch_size  # global batch per iteration
        self.t0 = None
        self.i0 = None
        self.excluded = 0.0

    def exclude(self, seconds):
        """Leave ``seconds`` of host-side output work (sample-grid PNGs, checkpoint files, the
        extra-image dump: GLI:565, 729-770) out of the current interval, so the line reports
        training throughput -- the same iterations bench.py times (the caller synchronises the
        device before starting that clock, so no training work is excluded)."""
        self.excluded += seconds

    def tick(self, i, now):
        line = None
        span = (now - self.t0 - self.excluded) if self.t0 is not None else 0.0
        if self.t0 is not None and i > self.i0 and span > 0:
            it_s = (i - self.i0) / span
            # img/s of the whole job; MFMA% of this GPU (every rank runs the same share)
            line = "[%d] img/s: %.1f MFMA%%: %.1f" % (i, it_s * self.images, 100.0 * it_s * self.flops / FP32_MFMA_PEAK)
        self.t0, self.i0, self.excluded = now, i, 0.0
        return line
