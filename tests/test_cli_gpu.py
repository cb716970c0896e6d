"""The reference CLI end to end on the MI355X (GLI:17-62, 86-100, 536-552, 560-768):
run folders, log file, the normalize=True sample grid every print_every, checkpoints with
the reference's dict keys every gen_every, the extra FID images, and --load resume."""
import os
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_train_cli_outputs_and_resume():
    from PIL import Image
    from relativisticgan_amd.train import main
    root = tempfile.mkdtemp()
    out, extra = os.path.join(root, "out"), os.path.join(root, "extra")
    args = ["--loss_D", "7", "--image_size", "32", "--batch_size", "8", "--z_size", "16", "--G_h_size", "8",
            "--D_h_size", "8", "--seed", "1", "--n_iter", "4", "--print_every", "2", "--gen_every", "3",
            "--gen_extra_images", "200", "--output_folder", out, "--extra_folder", extra,
            "--rgan_synthetic", "64"]
    main(args)
    base = os.path.join(out, "RaLSGAN_seed1-0")
    assert os.path.isfile(os.path.join(base, "logs", "log.txt"))
    log = open(os.path.join(base, "logs", "log.txt")).read()
    assert "[1] Diff:" in log and "[3] Diff:" in log and "Models saved" in log
    # the reference line unchanged, then img/s and MFMA% on a line of its own
    import re
    perf = re.findall(r"^\[(\d+)\] img/s: ([0-9.]+) MFMA%: ([0-9.]+)$", log, re.M)
    assert perf and all(float(v) > 0 for _, v, _ in perf), log[-400:]
    for i in (0, 2):
        img = np.asarray(Image.open(os.path.join(base, "images", "fake_samples_iter%05d.png" % i)))
        assert img.shape == (32 + 2 + 2, 8 * (32 + 2) + 2, 3)  # make_grid: 8 per row, padding 2
    files = sorted(os.listdir(os.path.join(extra, "1")))
    assert files == ["fake_samples_%05d.png" % k for k in range(200)]
    assert np.asarray(Image.open(os.path.join(extra, "1", files[0]))).shape == (32, 32, 3)
    ck = torch.load(os.path.join(extra, "models", "state_01.pth"), weights_only=True)
    assert set(ck) == {"i", "current_set_images", "G_state", "D_state", "G_optimizer", "D_optimizer",
                       "G_scheduler", "D_scheduler", "z_test"}
    assert ck["i"] == 3 and ck["current_set_images"] == 1
    # resume: a second run continues from iteration 3 with the saved state
    t2 = main(args + ["--load", os.path.join(extra, "models", "state_01.pth"), "--n_iter", "4"])
    assert os.path.isdir(os.path.join(out, "RaLSGAN_seed1-1"))
    assert torch.isfinite(t2.errD) and torch.isfinite(t2.errG)


def test_generate_from_checkpoint():
    from PIL import Image
    from relativisticgan_amd.config import make_param
    from relativisticgan_amd.generate import main as gen
    from relativisticgan_amd.train import Trainer, synthetic_images
    root = tempfile.mkdtemp()
    p = make_param(loss_D=7, image_size=32, batch_size=8, z_size=16, G_h_size=8, D_h_size=8, seed=1)
    t = Trainer(p, synthetic_images(64, 32))
    t.iteration(0)
    path = os.path.join(root, "state_01.pth")
    torch.save(t.state(1, 1), path)
    folder = gen(["--load", path, "--image_size", "32", "--z_size", "16", "--G_h_size", "8",
                  "--gen_extra_images", "100", "--extra_folder", os.path.join(root, "extra"), "--seed", "3"])
    files = sorted(os.listdir(folder))
    assert len(files) == 100
    assert np.asarray(Image.open(os.path.join(folder, files[-1]))).shape == (32, 32, 3)


def test_train_cli_from_image_folder():
    from tests.test_data import _make_folder
    from relativisticgan_amd.train import main
    root = tempfile.mkdtemp()
    folder = _make_folder(os.path.join(root, "data"))
    t = main(["--loss_D", "6", "--image_size", "32", "--batch_size", "4", "--z_size", "16", "--G_h_size", "8",
              "--D_h_size", "8", "--seed", "1", "--n_iter", "2", "--print_every", "1000", "--gen_extra_images", "0",
              "--output_folder", os.path.join(root, "out"), "--input_folder", folder, "--save", "False"])
    assert t.images.dtype == torch.uint8 and tuple(t.images.shape) == (5, 3, 32, 32)
    assert torch.isfinite(t.errD) and torch.isfinite(t.errG)
