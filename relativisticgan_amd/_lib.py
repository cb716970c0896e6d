"""ctypes binding of the C-ABI library (include/rgan.h -> relativisticgan_amd/librgan.so).

The HIP library is the only compute backend: if it is missing or fails to load, every
op raises -- there is no CPU or eager-PyTorch fallback.  Torch is used for device
memory (caching allocator) and the current HIP stream only.
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RGAN_LIB") or os.path.join(HERE, "librgan.so")  # RGAN_LIB: experiment builds (tools/build_variant.py)

ACT = {"none": 0, "relu": 1, "lrelu": 2, "tanh": 3, "sigmoid": 4, "selu": 5}

c_int, c_ll, c_f, c_d, c_sz, c_vp = (ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_double,
                                     ctypes.c_size_t, ctypes.c_void_p)


class RganConv(ctypes.Structure):
    _fields_ = [("batch", c_int), ("cin", c_int), ("hin", c_int), ("win", c_int),
                ("cout", c_int), ("hout", c_int), ("wout", c_int),
                ("kh", c_int), ("kw", c_int), ("stride", c_int), ("pad", c_int),
                ("transposed", c_int), ("xs", c_ll * 4), ("ys", c_ll * 4)]


class RganPost(ctypes.Structure):
    _fields_ = [("mode", c_int), ("act", c_int), ("alpha", c_f), ("nseg", c_int), ("x", c_vp), ("stats", c_vp),
                ("gamma", c_vp), ("beta", c_vp), ("part", c_vp), ("part_segments", c_ll)]


class RganAdamPack(ctypes.Structure):
    _fields_ = [("tensor", c_int), ("which", c_int), ("d", ctypes.POINTER(RganConv)), ("packed", c_vp)]


class RganSnLayer(ctypes.Structure):
    _fields_ = [("W", c_vp), ("rows", c_int), ("cols", c_int), ("lo", c_int), ("rs", c_ll), ("hs", c_ll),
                ("u", c_vp), ("v", c_vp), ("u_copy", c_vp), ("v_copy", c_vp), ("inv_sigma", c_vp)]


# name -> (restype, argtypes)
_SIGS = {
    "rgan_conv_workspace": (c_sz, [ctypes.POINTER(RganConv), c_int, c_int]),
    "rgan_conv_pack_floats": (c_sz, [ctypes.POINTER(RganConv), c_int]),
    "rgan_conv_pack": (c_int, [ctypes.POINTER(RganConv), c_int, c_vp, c_vp, c_vp]),
    "rgan_conv_pack_batch": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rgan_conv_fwd": (c_int, [ctypes.POINTER(RganConv), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_f, c_vp, c_sz,
                              c_vp]),
    "rgan_conv_bn_segments": (c_ll, [ctypes.POINTER(RganConv), c_int]),
    "rgan_conv_fwd_bn": (c_int, [ctypes.POINTER(RganConv), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp,
                                 c_ll, c_int, ctypes.POINTER(c_int), c_vp]),
    "rgan_bn_segment_stats_n": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_int, c_f, c_f, c_vp, c_vp, c_vp, c_vp,
                                        c_vp]),
    "rgan_bn_backward_segments": (c_int, [c_vp, c_vp, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_f, c_vp, c_vp,
                                          c_vp, c_vp, c_vp]),
    "rgan_bn_apply_segments": (c_int, [c_vp, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_f, c_vp, c_vp]),
    "rgan_bn_segment_apply": (c_int, [c_vp, c_ll, c_int, c_int, c_vp, c_ll, c_int, c_f, c_f, c_vp, c_vp, c_vp, c_vp,
                                      c_vp, c_int, c_f, c_vp, c_vp, c_vp]),
    "rgan_bn_segment_stats": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_f, c_f, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_vp]),
    "rgan_conv_post_segments": (c_ll, [ctypes.POINTER(RganConv), c_int, c_int, c_int, ctypes.POINTER(c_int)]),
    "rgan_conv_post": (c_int, [ctypes.POINTER(RganConv), c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz,
                               ctypes.POINTER(RganPost), ctypes.POINTER(c_int), c_vp]),
    "rgan_bn_backward_parts": (c_int, [c_vp, c_vp, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_ll, c_int, c_vp,
                                       c_vp, c_vp, c_vp, c_vp]),
    "rgan_g1_fwd_bn": (c_int, [c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_f, c_f, c_vp, c_vp, c_vp, c_int, c_f,
                               c_vp, c_vp, c_vp, c_vp]),
    "rgan_g1_wgrad": (c_int, [c_vp, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp]),
    "rgan_conv_dgrad": (c_int, [ctypes.POINTER(RganConv), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "rgan_conv_wgrad": (c_int, [ctypes.POINTER(RganConv), c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_sz, c_vp]),
    "rgan_conv_wgrad_rows": (c_int, [ctypes.POINTER(RganConv), c_vp, c_vp, c_vp, c_vp, ctypes.c_longlong, c_int, c_vp,
                                     c_sz, c_vp]),
    "rgan_nn_fold_weight": (c_int, [c_vp, c_int, c_int, c_vp, c_vp]),
    "rgan_patches_k4s2": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "rgan_patch_weight": (c_int, [c_vp, c_int, c_int, c_ll, c_ll, c_vp, c_vp]),
    "rgan_unpatch_grad": (c_int, [c_vp, c_int, c_int, c_ll, c_ll, c_vp, c_int, c_vp]),
    "rgan_nn_unfold_grad": (c_int, [c_vp, c_int, c_int, c_vp, c_vp]),
    "rgan_gather_images_u8": (c_int, [c_vp, c_vp, c_int, c_ll, c_vp, c_vp]),
    "rgan_minmax_ws_bytes": (c_sz, [c_ll]),
    "rgan_minmax": (c_int, [c_vp, c_ll, c_vp, c_vp, c_vp]),
    "rgan_images_to_u8": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_f, c_f, c_vp, c_int, c_int, c_int, c_vp,
                                  c_vp]),
    "rgan_bn_partial_bytes": (c_sz, [c_ll, c_int]),
    "rgan_bn_stats": (c_int, [c_vp, c_ll, c_int, c_ll, c_ll, c_f, c_f, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rgan_bn_moments": (c_int, [c_vp, c_ll, c_int, c_ll, c_ll, c_vp, c_vp, c_vp]),
    "rgan_bn_finalize": (c_int, [c_vp, c_int, c_int, c_f, c_f, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rgan_bn_backward_sums": (c_int, [c_vp, c_ll, c_ll, c_vp, c_ll, c_int, c_ll, c_ll, c_vp, c_vp, c_vp, c_int,
                                      c_f, c_vp, c_vp, c_vp]),
    "rgan_bn_backward_apply": (c_int, [c_vp, c_ll, c_ll, c_vp, c_ll, c_int, c_ll, c_ll, c_vp, c_vp, c_vp, c_int,
                                       c_f, c_vp, c_ll, c_vp, c_ll, c_ll, c_vp, c_vp, c_vp]),
    "rgan_bn_apply": (c_int, [c_vp, c_ll, c_int, c_ll, c_ll, c_vp, c_vp, c_vp, c_int, c_f, c_vp, c_ll, c_ll,
                              c_vp]),
    "rgan_bn_backward": (c_int, [c_vp, c_ll, c_ll, c_vp, c_ll, c_int, c_ll, c_ll, c_vp, c_vp, c_vp, c_int, c_f,
                                 c_vp, c_ll, c_ll, c_vp, c_vp, c_vp, c_vp]),
    "rgan_bn_backward_apply_ex": (c_int, [c_vp, c_ll, c_ll, c_vp, c_ll, c_int, c_ll, c_ll, c_vp, c_vp, c_vp, c_int,
                                          c_f, c_vp, c_ll, c_vp, c_vp, c_ll, c_ll, c_vp, c_vp, c_int, c_vp]),
    "rgan_bn_affine_grads": (c_int, [c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_vp]),
    "rgan_bn_backward_sums_apply": (c_int, [c_vp, c_vp, c_ll, c_int, c_vp, c_vp, c_vp, c_int, c_f, c_vp, c_vp, c_vp,
                                            c_vp, c_int, c_vp, c_vp, c_vp]),
    "rgan_bn_dd_partial_bytes": (c_sz, [c_ll, c_int]),
    "rgan_bn_dd_sums": (c_int, [c_vp, c_vp, c_vp, c_ll, c_int, c_ll, c_ll, c_vp, c_vp, c_vp, c_int, c_f, c_int, c_vp,
                                c_ll, c_vp, c_vp, c_vp]),
    "rgan_bn_dd_apply": (c_int, [c_vp, c_vp, c_vp, c_ll, c_int, c_ll, c_ll, c_vp, c_vp, c_vp, c_int, c_f, c_vp, c_vp,
                                 c_vp, c_vp, c_vp, c_ll, c_vp, c_vp, c_vp, c_vp, c_int, c_vp]),
    "rgan_act_dd": (c_int, [c_vp, c_vp, c_vp, c_ll, c_int, c_f, c_vp, c_vp, c_vp]),
    "rgan_act_backward": (c_int, [c_vp, c_vp, c_ll, c_int, c_f, c_vp, c_vp]),
    "rgan_act_backward_ex": (c_int, [c_vp, c_vp, c_vp, c_ll, c_int, c_f, c_vp, c_vp]),
    "rgan_channel_sum": (c_int, [c_vp, c_ll, c_int, c_ll, c_ll, c_vp, c_int, c_vp, c_vp]),
    "rgan_loss_head": (c_int, [c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "rgan_loss_head_pair": (c_int, [c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "rgan_loss_head_joint": (c_int, [c_int, c_vp, c_int, c_vp, c_vp, c_vp]),
    "rgan_loss_head_dist": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                    c_vp]),
    "rgan_scale": (c_int, [c_vp, c_vp, c_ll, c_vp, c_vp]),
    "rgan_gp_interp": (c_int, [c_vp, c_vp, c_vp, c_int, c_ll, c_vp, c_vp]),
    "rgan_gp_penalty": (c_int, [c_vp, c_int, c_ll, c_f, c_int, c_vp, c_vp, c_vp]),
    "rgan_gp_penalty_backward": (c_int, [c_vp, c_vp, c_int, c_ll, c_f, c_int, c_vp, c_vp, c_vp]),
    "rgan_spectral_ws_bytes": (c_sz, [c_int, c_int]),
    "rgan_spectral_power": (c_int, [c_vp, c_int, c_int, c_ll, c_ll, c_int, c_f, c_vp, c_vp, c_vp, c_int, c_vp,
                                    c_vp]),
    "rgan_spectral_batch_ws_bytes": (c_sz, [c_int, c_vp]),
    "rgan_spectral_power_batch": (c_int, [c_int, c_vp, c_f, c_vp, c_vp]),
    "rgan_spectral_backward": (c_int, [c_vp, c_vp, c_int, c_int, c_ll, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_int,
                                       c_vp, c_vp]),
    "rgan_adam": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rgan_adam_packed": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "rgan_adam_step_inc": (c_int, [c_vp, c_vp]),
    "rgan_lr_decay": (c_int, [c_vp, c_d, c_vp]),
    "rgan_gather_images": (c_int, [c_vp, c_vp, c_int, c_ll, c_vp, c_vp]),
    "rgan_rng_fill": (c_int, [c_vp, c_ll, c_int, ctypes.c_ulonglong, c_vp, c_vp]),
    "rgan_rng_choice": (c_int, [c_vp, c_int, c_int, ctypes.c_ulonglong, c_vp, c_vp]),
    "rgan_set_gemm_emulation": (c_int, [c_int]),
    "rgan_profile_begin": (c_int, [c_int]),
    "rgan_profile_end": (c_int, [c_vp, c_vp, c_vp]),
    "rgan_profile_kernel": (c_int, [c_int, ctypes.c_char_p, c_int, c_vp, c_vp, c_vp]),
    "rgan_version": (ctypes.c_char_p, []),
    "rgan_abi_version": (c_int, []),
}

EXPORTED = tuple(_SIGS)
_LIB = None


def lib():
    """Load librgan.so once; raise if it is missing (no fallback path exists)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python relativisticgan_amd/build.py` "
                               "(the MI355X HIP kernels are the only implementation)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


class RganError(RuntimeError):
    pass


def check(rc, what):
    if rc != 0:
        raise RganError(f"{what} failed (code {rc}{', invalid arguments' if rc == 1001 else ''})")


def stream():
    return c_vp(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    return None if t is None else c_vp(t.data_ptr())


def workspace(nbytes, device):
    """Scratch from torch's caching allocator (the kernels never allocate)."""
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


def require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RganError("relativisticgan_amd ops run on the MI355X only (got a CPU tensor); "
                            "there is no CPU fallback")
