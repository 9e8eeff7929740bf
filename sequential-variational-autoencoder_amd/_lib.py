"""ctypes binding of libsvae_hip.so (the C ABI declared in include/svae_hip.h).

The library is loaded after ``torch`` so that its ``libamdhip64.so.7`` dependency
resolves to the HIP runtime torch already mapped (one runtime per process: device
pointers from torch tensors are valid inside the library).  There is no fallback:
if the library is missing or fails to load, every entry point raises.
"""
import contextlib
import ctypes
import os

import torch  # noqa: F401  (must be imported before the HIP library is mapped)

_HERE = os.path.dirname(os.path.abspath(__file__))
# SVAE_LIB: another build of the library (A/B runs of compile-time variants)
LIB_PATH = os.environ.get("SVAE_LIB") or os.path.join(_HERE, "libsvae_hip.so")
# the -DSVAE_KNOBS build (csrc/knobs.h): the A/B tuning switches read from the environment
KNOBS_PATH = os.path.join(_HERE, "libsvae_hip_knobs.so")

_c_float_p = ctypes.POINTER(ctypes.c_float)


class SvaeConfig(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int32), ("height", ctypes.c_int32), ("width", ctypes.c_int32),
        ("channels", ctypes.c_int32), ("levels", ctypes.c_int32), ("mc_steps", ctypes.c_int32),
        ("filter_sizes", ctypes.c_int32 * 10), ("latent_dims", ctypes.c_int32 * 8),
        ("intermediate_reconstruction", ctypes.c_int32),
        ("first_step_loss_coeff", ctypes.c_float), ("latent_prior_stddev", ctypes.c_float),
        ("latent_mean_clip", ctypes.c_float), ("range_lo", ctypes.c_float), ("range_hi", ctypes.c_float),
        ("min_highway", ctypes.c_float), ("max_highway", ctypes.c_float), ("dtype", ctypes.c_int32),
        ("share_theta", ctypes.c_int32), ("share_phi", ctypes.c_int32),
        ("predict_latent_code", ctypes.c_int32), ("predict_latent_code_with_regularization", ctypes.c_int32),
        ("unregularized_steps_mask", ctypes.c_uint32 * 2),
        ("use_uniform_prior", ctypes.c_int32), ("add_noise_to_chain", ctypes.c_int32),
        ("noise_stddevs", ctypes.c_float * 64), ("predict_generator_noise", ctypes.c_int32),
        ("predict_generator_stddev_max", ctypes.c_float), ("stddev_layers", ctypes.c_int32),
        ("stddev_filter_sizes", ctypes.c_int32 * 8), ("add_improvement_maximization_loss", ctypes.c_int32),
        ("latent_pred_loss_coeff", ctypes.c_float), ("external_generator_from", ctypes.c_int32),
    ]


class SvaeParamDesc(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 96), ("ndim", ctypes.c_int32), ("shape", ctypes.c_int32 * 4),
                ("offset", ctypes.c_int64), ("init", ctypes.c_int32), ("flags", ctypes.c_int32)]


BUF_XHAT, BUF_MU, BUF_SIGMA, BUF_Z, BUF_STEP_STATS, BUF_REC_IMG, BUF_KL_IMG, BUF_DZ = range(8)
BUF_SAMPLE, BUF_STDDEV, BUF_IMP_IMG = 8, 9, 10
ACT_NONE, ACT_RELU, ACT_LRELU = 0, 1, 2

_lib = None


# void (*svae_step_hook)(void* user, int t)   (include/svae_hip.h)
STEP_HOOK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int)


_loaded = {}


def lib():
    """Load (once) and return the library; raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    _lib = _load(LIB_PATH)
    return _lib


@contextlib.contextmanager
def knob_build():
    """Within the block, lib() is the -DSVAE_KNOBS build (the tests that hold an A/B switch of
    csrc/knobs.h bitwise to the default path set SVAE_* and create their networks inside it)."""
    global _lib
    prev = lib()
    _lib = _load(KNOBS_PATH)
    try:
        yield _lib
    finally:
        _lib = prev


def _load(path):
    if path in _loaded:
        return _loaded[path]
    if not os.path.exists(path):
        raise RuntimeError("%s not built; run __graft_entry__.build() or "
                           "python sequential-variational-autoencoder_amd/build.py" % path)
    L = ctypes.CDLL(path)
    L.svae_build_hash.argtypes = []
    L.svae_build_hash.restype = ctypes.c_char_p
    built = (L.svae_build_hash() or b"").decode()
    # the library must be built from this tree's sources (a stale binary shipped with a newer tree is never
    # run); SVAE_LIB variant builds (A/B of modified copies) are exempt
    if not os.environ.get("SVAE_LIB"):
        from . import build as _build
        want = _build.src_hash()
        if built != want:
            raise RuntimeError("%s was built from other sources (hash %s, tree %s); run __graft_entry__.build()"
                               % (path, built, want))
    vp, i32, i64, f32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64
    cfgp = ctypes.POINTER(SvaeConfig)
    sig = {
        "svae_param_count": ([cfgp, ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i32)], i32),
        "svae_param_layout": ([cfgp, ctypes.POINTER(SvaeParamDesc), i32], i32),
        "svae_create": ([cfgp, i32, ctypes.POINTER(vp)], i32),
        "svae_destroy": ([vp], i32),
        "svae_last_error": ([vp], ctypes.c_char_p),
        "svae_bind": ([vp, vp, vp], i32),
        "svae_workspace_bytes": ([vp], i64),
        "svae_forward": ([vp, vp, vp, vp, f32, vp], i32),
        "svae_backward": ([vp, vp], i32),
        "svae_generate": ([vp, vp, vp], i32),
        "svae_adam": ([vp, f32, i64, f32, vp], i32),
        "svae_adam_range": ([vp, i64, i64, f32, i64, f32, vp], i32),
        "svae_backward_adam": ([vp, f32, i64, f32, vp], i32),
        "svae_adam_state": ([vp, i32, vp, vp, i64, vp], i32),
        "svae_copy_out": ([vp, i32, i32, vp, i64, vp], i32),
        "svae_op_conv": ([vp, i32, i32, i32, vp, i32, i32, i32, vp, vp], i32),
        "svae_op_conv_dgrad": ([vp, i32, i32, i32, vp, i32, i32, i32, vp, vp], i32),
        "svae_op_conv_wgrad": ([vp, i32, i32, i32, vp, i32, i32, i32, vp, vp, i64, vp], i32),
        "svae_op_bn_act": ([vp, i64, i32, vp, i32, vp, vp, vp, vp, i64, vp], i32),
        "svae_op_bn_act_bwd": ([vp, vp, vp, i64, i32, vp, vp, i32, vp, vp, vp, i64, vp], i32),
        "svae_op_fc": ([vp, i32, i32, vp, i32, vp, vp], i32),
        "svae_op_gather_bf16": ([vp, i32, i32, i32, vp, i32, i32, i32, i32, vp, vp, i64, vp], i32),
        "svae_op_wgrad_bf16": ([vp, i32, i32, i32, vp, i32, i32, i32, i32, vp, vp, i64, vp], i32),
        "svae_probe_begin": ([vp, i32, i32], i32),
        "svae_probe_end": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_double),
                            ctypes.POINTER(ctypes.c_double)], i32),
        "svae_kernel_name": ([i32], ctypes.c_char_p),
        "svae_set_backward_hook": ([vp, STEP_HOOK, vp], i32),
        "svae_hook_stream": ([vp], vp),
        "svae_set_chain_noise": ([vp, vp], i32),
        "svae_set_external_grads": ([vp, vp, vp], i32),
        "svae_bind_imp": ([vp, vp], i32),
        "svae_backward_imp": ([vp, vp], i32),
        "svae_adam_imp": ([vp, f32, i64, f32, vp], i32),
        "svae_imp_range": ([vp, ctypes.POINTER(i64)], i32),
        # PixelCNN++ head (include/svae_pcnn.h)
        "svae_pcnn_wnorm": ([vp, vp, i32, i32, i32, vp, vp, i32, vp, i32, vp], i32),
        "svae_pcnn_wnorm_bwd": ([vp, vp, vp, vp, i32, i32, i32, vp, vp, vp], i32),
        "svae_pcnn_conv": ([vp, i32, i32, i32, i32, i32, i32, vp, i32, vp, vp, i32, i32, i32, i32, i32, i32, i32,
                            i32, i32, i32, i32, i32, vp], i32),
        "svae_pcnn_conv_act_bwd": ([vp, i32, i32, i32, i32, i32, vp, i32, vp, i32, i32, i32, i32, i32, i32, i32, i32,
                                    i32, i32, i32, vp, i32, i32, vp, f32, u64, vp], i32),
        "svae_pcnn_conv_wgrad": ([vp, i32, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32,
                                  i32, i32, vp, vp, vp, i64, vp], i32),
        "svae_pcnn_wnorm_planes": ([vp, vp, i32, i32, i32, vp, vp, i32, vp, i32, i32, vp, vp], i32),
        "svae_pcnn_split_planes": ([vp, i64, i32, i32, i32, vp, i32, i32, vp, vp], i32),
        "svae_pcnn_split_h16_premax": ([vp, i64, i32, i32, vp, i32, vp, vp], i32),
        "svae_pcnn_conv_planes": ([vp, i32, i32, i32, i32, i32, i32, i64, vp, i32, i32, vp, vp, vp, vp, i32, i32,
                                   i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp], i32),
        "svae_pcnn_conv_wgrad_planes": ([vp, i32, i32, i32, i32, i32, i32, i64, vp, i32, i32, i64, i32, vp, vp, i32,
                                         i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, i64, vp], i32),
        "svae_pcnn_colsum": ([vp, i64, i32, i32, i32, i32, i32, vp, i32, vp, vp], i32),
        "svae_pcnn_colsum_absmax": ([vp, i64, i32, i32, vp, i32, vp, vp, vp], i32),
        "svae_pcnn_im2col_h16": ([vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp, vp], i32),
        "svae_pcnn_conv_planes_amax": ([vp, i32, i32, i32, i32, i32, i32, i64, vp, i32, i32, vp, vp, vp, vp, i32, i32,
                                        i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp], i32),
        "svae_pcnn_nonlin_h16": ([vp, i64, i32, i32, i32, vp, f32, f32, u64, vp, vp, i32, vp, vp], i32),
        "svae_pcnn_mask_edge": ([vp, i32, i32, i32, i32, i32, i32, vp], i32),
        "svae_pcnn_nonlin": ([vp, i64, i32, i32, i32, vp, f32, u64, vp, i32, i32, vp], i32),
        "svae_pcnn_nonlin_absmax": ([vp, i64, i32, i32, i32, vp, f32, u64, vp, i32, vp, vp], i32),
        "svae_pcnn_nonlin_bwd": ([vp, i64, i32, i32, i32, vp, f32, u64, vp, i32, vp, i32, i32, i32, vp, vp, vp], i32),
        "svae_pcnn_dropout_mask": ([i64, f32, u64, vp, vp], i32),
        "svae_pcnn_gate": ([vp, i32, vp, vp, i64, i32, i32, vp, i32, vp], i32),
        "svae_pcnn_gate_amax": ([vp, i32, vp, vp, i64, i32, i32, vp, i32, vp, vp], i32),
        "svae_pcnn_gate_bwd": ([vp, vp, vp, i32, i64, i32, i32, vp, i32, vp, vp, vp, vp], i32),
        "svae_pcnn_gemm_small": ([vp, i32, i32, vp, i32, i32, vp, i32, i32, i32, i32, f32, vp], i32),
        "svae_pcnn_imgsum": ([vp, i32, i32, i32, i32, vp, vp, vp], i32),
        "svae_pcnn_copy": ([vp, i32, i64, i32, vp, i32, i32, vp], i32),
        "svae_pcnn_pad_ones": ([vp, i64, i32, vp, i32, vp], i32),
        "svae_pcnn_mixlogistic": ([vp, vp, i64, i32, vp, vp, f32, vp], i32),
        "svae_pcnn_sum": ([vp, i64, vp, vp, vp], i32),
        "svae_pcnn_sample": ([vp, vp, vp, i32, i32, i32, vp, i32, i32, i32, vp], i32),
        "svae_pcnn_highway": ([vp, vp, vp, vp, i32, i64, f32, f32, vp, vp, vp], i32),
        "svae_pcnn_wn_init": ([vp, i64, i32, i32, f32, vp, vp, vp, vp], i32),
        "svae_pcnn_adam": ([vp, vp, vp, vp, i64, f32, i64, f32, vp], i32),
        "svae_pcnn_ema": ([vp, vp, i64, f32, vp], i32),
        "svae_pcnn_sample_bwd": ([vp, vp, vp, i32, i32, i32, vp, i32, vp, vp], i32),
        "svae_pcnn_highway_bwd": ([vp, vp, vp, vp, i32, i64, f32, f32, vp, vp, vp, i32, vp, vp], i32),
        "svae_pcnn_dropout": ([vp, i64, i32, i32, vp, vp, i32, vp], i32),
        "svae_pcnn_sqerr": ([vp, vp, i32, i64, f32, vp, vp, vp], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _loaded[path] = L
    return L


EXPORTED = ["svae_param_count", "svae_param_layout", "svae_create", "svae_destroy", "svae_last_error",
            "svae_bind", "svae_workspace_bytes", "svae_forward", "svae_backward", "svae_adam", "svae_copy_out",
            "svae_op_conv", "svae_op_conv_dgrad", "svae_op_conv_wgrad", "svae_op_bn_act",
            "svae_op_bn_act_bwd", "svae_op_fc", "svae_probe_begin", "svae_probe_end", "svae_kernel_name",
            "svae_op_gather_bf16", "svae_op_wgrad_bf16", "svae_generate", "svae_set_backward_hook",
            "svae_hook_stream", "svae_adam_range", "svae_backward_adam", "svae_adam_state",
            "svae_set_chain_noise", "svae_bind_imp", "svae_backward_imp", "svae_adam_imp", "svae_imp_range",
            "svae_set_external_grads", "svae_build_hash"]
# include/svae_pcnn.h (the PixelCNN++ head)
PCNN_EXPORTED = ["svae_pcnn_wnorm", "svae_pcnn_wnorm_bwd", "svae_pcnn_conv", "svae_pcnn_conv_wgrad", "svae_pcnn_colsum",
                 "svae_pcnn_colsum_absmax", "svae_pcnn_im2col_h16", "svae_pcnn_conv_planes_amax",
                 "svae_pcnn_nonlin_h16", "svae_pcnn_gate_amax",
                 "svae_pcnn_mask_edge", "svae_pcnn_nonlin", "svae_pcnn_nonlin_bwd", "svae_pcnn_gate",
                 "svae_pcnn_gate_bwd", "svae_pcnn_gemm_small", "svae_pcnn_imgsum", "svae_pcnn_copy",
                 "svae_pcnn_pad_ones", "svae_pcnn_mixlogistic", "svae_pcnn_sum", "svae_pcnn_sample",
                 "svae_pcnn_highway", "svae_pcnn_wn_init", "svae_pcnn_adam", "svae_pcnn_ema", "svae_pcnn_sample_bwd",
                 "svae_pcnn_highway_bwd", "svae_pcnn_dropout", "svae_pcnn_sqerr",
                 "svae_pcnn_dropout_mask", "svae_pcnn_conv_act_bwd", "svae_pcnn_wnorm_planes",
                 "svae_pcnn_split_planes", "svae_pcnn_conv_planes", "svae_pcnn_conv_wgrad_planes",
                 "svae_pcnn_split_h16_premax", "svae_pcnn_nonlin_absmax"]

# bf16 GEMM instance ids (csrc/kernels.h KernelId) for svae_probe_begin
KID_IGEMM_BF16_256x32 = 2
KID_IGEMM_BF16_128x64 = 4
KID_IGEMM_BF16_128x128 = 6
KID_IGEMM_BF16_64x128 = 8
KID_WGRAD_BF16_128x32 = 10
KID_WGRAD_BF16_128x64 = 12
KID_WGRAD_BF16_128x128 = 14
KID_HALO_256x32 = 16
KID_HALO_128x64 = 18
KID_HALO_128x128 = 20
KID_HALO_64x128 = 21
KID_WHALO_32_S1 = 22
KID_WHALO_32_S2 = 23
KID_WHALO2_S1 = 26   # wgrad_halo2_kernel<...>: every instance of the stride-1 halo weight-GEMM
KID_HALO_KW = 27     # igemm_halo_kw_kernel<...>: the wave-split gather-GEMM (main stream)
KID_WHALO2_S2 = 28   # wgrad_halo2_kernel<..., S = 2>: the stride-2 instances
KID_HALO_X3 = 29     # gather_x3_kernel<...>: the split mode's fp16-plane wave-split gather (main stream)


def check(rc, ctx=None):
    if rc != 0:
        msg = lib().svae_last_error(ctx)
        raise RuntimeError("libsvae_hip error %d: %s" % (rc, msg.decode() if msg else "?"))


def ptr(t):
    """Raw device (or host) pointer of a contiguous tensor, or None."""
    if t is None:
        return None
    assert t.is_contiguous(), "tensor must be contiguous"
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
