"""ctypes binding of libmiattack.so (the C ABI declared in include/miattack.h).

The product path has no CPU fallback: if the library is missing or no GPU is present, the first
call raises. torch is imported before the library is opened so that the process holds ONE HIP
runtime (torch's libamdhip64, whose SONAME the library's dependency resolves to).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# MIA_F32_ARITH=native loads the A/B build whose fp32 convs run v_mfma_f32_16x16x4_f32
# (csrc/Makefile `native`); the default build runs them as exact three-way bf16 splits
# (conv_common.h, mfma_chunk<float>). Everything else is the same source.
F32_ARITH = os.environ.get("MIA_F32_ARITH", "bf16x6")
if F32_ARITH not in ("bf16x6", "native"):
    raise ValueError(f"MIA_F32_ARITH must be bf16x6 or native, not {F32_ARITH!r}")
LIB_PATH = os.path.join(HERE, "libmiattack.so" if F32_ARITH == "bf16x6"
                        else "libmiattack_f32native.so")
# Tuning A/B only (tools/gpu/*_ab.sh): MIA_LIB_VARIANT=<name> loads libmiattack_<name>.so, a build
# of the same sources with extra compile-time switches (csrc/Makefile `variant`).
if os.environ.get("MIA_LIB_VARIANT"):
    LIB_PATH = os.path.join(HERE, f"libmiattack_{os.environ['MIA_LIB_VARIANT']}.so")

c_int, c_float, c_int64, c_void_p = ctypes.c_int, ctypes.c_float, ctypes.c_int64, ctypes.c_void_p
P = c_void_p

MIA_F32, MIA_F16, MIA_BF16 = 0, 1, 2
ACT_NONE, ACT_RELU, ACT_LRELU_S2, ACT_PRELU = 0, 1, 2, 3


class ConvArgs(ctypes.Structure):
    """Mirror of ``mia_conv_args`` (include/miattack.h)."""
    _fields_ = [
        ("x", P), ("w", P), ("y", P),
        ("N", c_int), ("H", c_int), ("W", c_int), ("Cin", c_int), ("Cout", c_int), ("Kpad", c_int),
        ("y_cstride", c_int), ("act_in", c_int),
        ("in_scale", P), ("out_scale", P), ("bias", P), ("noise", P), ("noise_w", c_float),
        ("act_out", c_int), ("shuffle_out", c_int),
        ("aux_x", P), ("act_aux", c_int), ("sdot", P),
        ("tap_a", P), ("tap_t", P), ("tap_coef", c_float), ("mask_a", P),
        ("accumulate", c_int),
        ("bab_demod", P), ("bab_noise", P), ("bab_noise_w", c_float), ("bab_bias", P),
        ("bab_q", P),
        ("mask_slope", P), ("act_slope", P), ("csum", P),
        ("w_split", P),
    ]


class ConvGroup(ctypes.Structure):
    """Mirror of ``mia_conv_group``."""
    _fields_ = [("w", P), ("kh", c_int), ("kw", c_int), ("pad_y", c_int), ("pad_x", c_int),
                ("ho", c_int), ("wo", c_int), ("ay", c_int), ("by", c_int), ("ax", c_int),
                ("bx", c_int), ("w_split", P)]


class ConvBatch(ctypes.Structure):
    """Mirror of ``mia_conv_batch``."""
    _fields_ = [("n_in", c_int), ("n_out", c_int), ("c_off", c_int)]


class GemmSeg(ctypes.Structure):
    """Mirror of ``mia_gemm_seg``."""
    _fields_ = [("A", P), ("B", P), ("sam", c_int64), ("sak", c_int64), ("sbk", c_int64),
                ("sbn", c_int64), ("K", c_int)]


class GemmGroup(ctypes.Structure):
    """Mirror of ``mia_gemm_group``."""
    _fields_ = [("C", P), ("bias", P), ("scm", c_int64), ("scn", c_int64), ("M", c_int),
                ("N", c_int), ("alpha", c_float), ("beta", c_float), ("nseg", c_int),
                ("seg", GemmSeg * 2)]


# name -> (restype, argtypes); every function declared in include/miattack.h
SIGNATURES = {
    "mia_version": (c_int, []),
    "mia_last_error_string": (ctypes.c_char_p, []),
    "mia_conv_workspace_size": (c_int64, [c_int, c_int, c_int, c_int, c_int]),
    "mia_reduction_workspace_size": (c_int64, [c_int, c_int, c_int]),
    "mia_reserve_reduction_scratch": (c_int, [c_int64, P]),
    "mia_reduction_scratch_bytes": (c_int64, [P]),
    "mia_release_reduction_scratch": (c_int, [P]),
    "mia_set_tuning": (c_int, [ctypes.c_char_p, c_int]),
    "mia_get_tuning": (c_int, [ctypes.c_char_p, ctypes.POINTER(c_int)]),
    "mia_conv_kpad": (c_int, [c_int, c_int]),
    "mia_conv3x3": (c_int, [ctypes.POINTER(ConvArgs), c_int, P]),
    "mia_modulate_weights": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_conv3x3_wmod": (c_int, [ctypes.POINTER(ConvArgs), c_int64, c_int, P]),
    "mia_modconv_fwd": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P,
                                c_float, P, c_int, c_int, P]),
    "mia_modconv_bwd": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, c_int, P, P,
                                c_int, P]),
    "mia_vgg_conv_relu_fwd": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                      P]),
    "mia_vgg_conv_dgrad": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P,
                                   c_float, P, c_int, P]),
    "mia_vgg_conv_relu_dgrad": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P,
                                        P, c_float, P, c_int, P]),
    "mia_upconv_kpad": (c_int, [c_int, c_int, c_int]),
    "mia_upconv_fwd": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P, c_int, P]),
    "mia_upconv_fwd_halo": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, P, c_int, P]),
    "mia_upconv_fwd_halo_split": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P, c_int,
                                          P]),
    "mia_upconv_blur_fwd": (c_int, [P, P, P, P, c_float, P, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_upconv_blur_bwd": (c_int, [P, P, c_int, c_int, c_int, c_int, P]),
    "mia_upconv_dgrad": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P, c_int, P, P, c_int,
                                 P]),
    "mia_upconv_dgrad_fused": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P, P, P, c_int, P, P,
                                       c_float, P, P, c_int, P]),
    "mia_upconv_dgrad_fused_split": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, P, P, P, c_int,
                                             P, P, c_float, P, P, c_int, P]),
    "mia_bias_act_fwd": (c_int, [P, P, c_float, P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_bias_act_bwd": (c_int, [P, P, P, c_float, P, P, P, P, c_int, c_int, c_int, c_int, c_int,
                                 c_int, c_int, P]),
    "mia_upfirdn2d_fwd": (c_int, [P, P, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int, c_int,
                                  P]),
    "mia_upfirdn2d_bwd": (c_int, [P, P, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int, c_int,
                                  P]),
    "mia_torgb_fwd": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_torgb_bwd": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                              P]),
    "mia_torgb_bwd_front": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, P, P, c_float,
                                    P, P, c_int, P]),
    "mia_maxpool2_fwd": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_maxpool2_bwd": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P, c_float, c_int,
                                 c_int, P]),
    "mia_avgpool_fwd": (c_int, [P, P, c_int, c_int, c_int, c_int, P]),
    "mia_avgpool_bwd": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_image_to_nhwc": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_mse_sum": (c_int, [P, P, P, c_int, c_int64, c_float, c_int, P]),
    "mia_mse_grad_f32": (c_int, [P, P, P, c_int64, c_float, c_int, P]),
    "mia_mse_fwd_bwd": (c_int, [P, P, P, P, c_int, c_int64, c_float, c_float, c_int, c_int, P]),
    "mia_tap_grad": (c_int, [P, P, P, c_int64, c_float, c_int, c_int, P]),
    "mia_image_grad": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_float, c_int, P]),
    "mia_pgd_update": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_float, c_float,
                               c_float, c_float, c_float, P, c_int, P]),
    "mia_grad_assemble": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_float,
                                  c_float, P, c_int, P]),
    "mia_cw_init": (c_int, [P, P, c_int64, P]),
    "mia_cw_tanh": (c_int, [P, P, c_int64, P]),
    "mia_cw_grad": (c_int, [P, P, P, P, c_int64, c_float, c_float, P]),
    "mia_cw_select": (c_int, [P, P, P, P, P, P, c_int, c_int64, c_float, P]),
    "mia_random_start": (c_int, [P, P, P, c_int64, c_float, c_float, c_float, P]),
    "mia_sign_project": (c_int, [P, P, P, c_int64, c_float, c_float, c_float, c_float, P]),
    "mia_ssim_workspace_size": (c_int64, [c_int, c_int, c_int]),
    "mia_ssim2": (c_int, [P, P, c_int, c_int, c_int, c_float, P, c_int64, P, P]),
    "mia_adam_step": (c_int, [P, P, P, P, c_int64, c_float, c_float, c_float, c_float, c_int, P]),
    "mia_patch_update": (c_int, [P, P, P, P, P, c_int64, c_int64, c_float, c_float, P]),
    "mia_gemm_f32": (c_int, [c_int, c_int, c_int, c_float, P, c_int64, c_int64, P, c_int64,
                             c_int64, c_float, P, c_int64, c_int64, P, P]),
    "mia_gemm_f32_grouped": (c_int, [ctypes.POINTER(GemmGroup), c_int, P]),
    "mia_sum_slices": (c_int, [P, P, c_int, c_int, c_int, P]),
    "mia_style_demod": (c_int, [P, P, P, c_int, c_int, c_int, c_float, P]),
    "mia_demod_bwd": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_float, P]),
    "mia_pixel_norm": (c_int, [P, P, c_int, c_int, c_float, P]),
    "mia_truncate": (c_int, [P, P, c_float, P, c_int, c_int, P]),
    "mia_repeat": (c_int, [P, P, c_int64, c_int, P]),
    "mia_memset": (c_int, [P, c_int, c_int64, P]),
    "mia_conv2d_kpad": (c_int, [c_int, c_int, c_int]),
    "mia_conv2d_planes": (c_int, [ctypes.POINTER(ConvArgs), c_int, ctypes.POINTER(ConvGroup),
                                  c_int, c_int, c_int, c_int64, c_int, P]),
    "mia_conv2d": (c_int, [ctypes.POINTER(ConvArgs), c_int, ctypes.POINTER(ConvGroup), c_int,
                           c_int, c_int, c_int, P]),
    "mia_conv2d_batched": (c_int, [ctypes.POINTER(ConvArgs), c_int, ctypes.POINTER(ConvGroup),
                                   ctypes.POINTER(ConvBatch), c_int, c_int, c_int, c_int, P]),
    "mia_conv_s2_dgrad_halo": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P, P, c_int, c_int,
                                       P]),
    "mia_conv_s2_dgrad_halo_multi": (c_int, [P, c_int, P, P, P, c_int, c_int, c_int, c_int, P, P,
                                             c_int, c_int, P]),
    "mia_se_fwd": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_float, P]),
    "mia_se_apply": (c_int, [P, P, P, c_int, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_chan_sum_parts": (c_int, [c_int, c_int]),
    "mia_chan_sum": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_chan_dot": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_se_bwd": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_float, P]),
    "mia_se_fwd_parts": (c_int, [P, c_int, P, P, P, P, c_int, c_int, c_int, c_float, P]),
    "mia_se_bwd_parts": (c_int, [P, c_int, P, P, P, P, P, c_int, c_int, c_int, c_float, P]),
    "mia_se_grad_scale": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, P]),
    "mia_prelu_bwd_scale": (c_int, [P, P, P, P, P, c_int64, c_int, c_int, P]),
    "mia_prelu_fwd": (c_int, [P, P, P, c_int64, c_int, c_int, P]),
    "mia_subsample_add": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "mia_cast": (c_int, [P, c_int, P, c_int, c_int64, c_float, P]),
    "mia_bilinear_fwd": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                 P]),
    "mia_bilinear_bwd": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                 P]),
}

_lib = None


class MiaError(RuntimeError):
    pass


def load():
    """Open the library (once). Raises if it was not built — there is no fallback path."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    if not os.path.exists(LIB_PATH):
        raise MiaError(f"{LIB_PATH} missing: build it with __graft_entry__.build() "
                       "(make -C csrc); the attack path has no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise MiaError(f"{name} failed ({rc}): {lib.mia_last_error_string().decode()}")
    return rc


def set_tuning(name, value):
    """Set a kernel-variant switch (include/miattack.h); returns the previous value."""
    old = get_tuning(name)
    call("mia_set_tuning", name.encode(), int(value))
    return old


def get_tuning(name):
    v = c_int(0)
    call("mia_get_tuning", name.encode(), ctypes.byref(v))
    return v.value
