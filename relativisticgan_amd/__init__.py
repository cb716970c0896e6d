"""MI355X-native (gfx950) training core for RelativisticGAN's DCGAN / standard-CNN GAN step.

Hot path: hand-written HIP kernels (librgan.so, C-ABI in include/rgan.h) behind the
reference's surface (GLI = code/GAN_losses_iter.py): DCGAN_G / DCGAN_D modules with the
reference's state_dict names, the eight --loss_D heads, WGAN-GP, spectral norm, Adam.
"""
__version__ = "0.1.0"
