"""ctypes binding of libupr.so (include/upr.h).

The library is built in-tree (csrc/Makefile -> lib/libupr.so).  There is no
fallback: if the library is missing or fails to load, every entry point raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("UPR_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libupr.so"))

UPR_F32 = 0
UPR_F16 = 1
UPR_MODEL_IENET_ONLY = 1
UPR_MODEL_HEAD_ONLY = 2

UPR_OK = 0
UPR_ERR_ARG = -1
UPR_ERR_SHAPE = -2
UPR_ERR_MISSING_PARAM = -3
UPR_ERR_WORKSPACE = -4
UPR_ERR_UNSUPPORTED = -5


class UprTensorDesc(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p),
                ("data", ctypes.POINTER(ctypes.c_float)),
                ("ndim", ctypes.c_int),
                ("shape", ctypes.c_int64 * 4)]


class UprOpStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 64),
                ("kind", ctypes.c_int),
                ("calls", ctypes.c_int),
                ("ms", ctypes.c_double),
                ("flops", ctypes.c_double),
                ("bytes", ctypes.c_double)]


UPR_OP_CONV_IGEMM = 0
UPR_OP_OTHER = 1
UPR_CALIB_MFMA_F16 = 0
UPR_CALIB_HBM_COPY = 1

c_int, c_size_t, c_void_p, c_float = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_float
c_u8p = ctypes.POINTER(ctypes.c_uint8)

# name -> (restype, argtypes); mirrors include/upr.h exactly
SIGNATURES = {
    "upr_model_create": (c_int, [ctypes.POINTER(UprTensorDesc), c_int, c_int, c_int, c_int, c_int,
                                 ctypes.POINTER(c_void_p)]),
    "upr_model_workspace": (c_size_t, [c_void_p, c_int, c_int, c_int]),
    "upr_model_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_size_t, c_void_p]),
    "upr_model_destroy": (None, [c_void_p]),
    "upr_model_forks": (ctypes.c_longlong, [c_void_p]),
    "upr_model_profile": (c_int, [c_void_p, c_int]),
    "upr_model_profile_read": (c_int, [c_void_p, ctypes.POINTER(UprOpStat), c_int, ctypes.POINTER(c_int)]),
    "upr_status_string": (ctypes.c_char_p, [c_int]),
    "upr_conv2d_nhwc": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "upr_quantize_u8": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    "upr_letterbox": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                              c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "upr_to_u8_hwc": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "upr_rgb2lab_u8": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "upr_lab2rgb_u8": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "upr_clahe_u8": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int, c_int, c_void_p]),
    "upr_clahe_enhance_workspace": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "upr_clahe_enhance": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int, c_int, c_int,
                                  c_void_p]),
    "upr_gray_hist": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "upr_multiscale": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                               c_void_p]),
    "upr_multiscale_features": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "upr_content_aware_workspace": (c_size_t, [c_int, c_int, c_int]),
    "upr_content_aware": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int,
                                  c_int, c_int, c_void_p]),
    "upr_lab_tables": (None, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "upr_retinex_decompose": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_void_p]),
    "upr_retinex_decompose_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                          c_int, c_int, c_int, c_void_p]),
    "upr_calib_run": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_size_t, c_int, ctypes.POINTER(c_float),
                              c_void_p]),
}


class UprView(ctypes.Structure):
    """include/upr_train.h UprView: element strides of (batch, row, col, channel)."""
    _fields_ = [("data", ctypes.c_void_p), ("sb", ctypes.c_int64), ("sh", ctypes.c_int64),
                ("sw", ctypes.c_int64), ("sc", ctypes.c_int64)]


class UprLossParams(ctypes.Structure):
    """include/upr_train.h UprLossParams: the loss modules' constructor arguments."""
    _fields_ = [("patch", ctypes.c_int), ("base_exposure", ctypes.c_float), ("smooth_lambda", ctypes.c_float),
                ("smooth_alpha", ctypes.c_float), ("decouple_lambda", ctypes.c_float), ("freq_high", ctypes.c_float),
                ("freq_low", ctypes.c_float), ("dynamic_smooth", ctypes.c_int),
                ("illu_channels", ctypes.c_int)]


class UprPackJob(ctypes.Structure):
    """include/upr_train.h UprPackJob: one re-pack of upr_t_pack_weights."""
    _fields_ = [("w", ctypes.c_void_p), ("out32", ctypes.c_void_p), ("out16", ctypes.c_void_p), ("Co", ctypes.c_int),
                ("Ci", ctypes.c_int), ("kh", ctypes.c_int), ("kw", ctypes.c_int), ("mode", ctypes.c_int),
                ("n", ctypes.c_int)]


_vp = ctypes.POINTER(UprView)
c_u64, c_i64p = ctypes.c_uint64, ctypes.c_void_p
_i, _p, _f = c_int, c_void_p, c_float

# mirrors include/upr_train.h exactly
SIGNATURES.update({
    "upr_t_zero": (_i, [_p, c_size_t, _p]),
    "upr_t_conv_direct": (_i, [_vp, _i, _i, _i, _i, _p, _p, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _p]),
    "upr_t_conv_dgrad_c3_16": (_i, [_p, _i, _i, _i, _p, _i, _vp, _i, _p]),
    "upr_t_conv_direct16": (_i, [_vp, _i, _i, _i, _i, _p, _p, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _p, _i,
                                 _p]),
    "upr_t_conv_direct_dgrad": (_i, [_vp, _i, _i, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _p]),
    "upr_t_conv_direct_wgrad": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p]),
    "upr_t_conv_stem_wgrad_relu16": (_i, [_vp, _p, _p, _i, _i, _i, _p, _p, _p]),
    "upr_t_conv_direct_wgrad_relu": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p,
                                          _p]),
    "upr_t_conv_mfma": (_i, [_p, _i, _i, _i, _i, _i, _i, _p, _p, _i, _i, _i, _i, _i, _i, _p, _i, _i, _p, _i, _i,
                             _i, _p]),
    "upr_t_conv_mfma16": (_i, [_p, _i, _i, _i, _i, _i, _i, _p, _p, _i, _i, _i, _i, _i, _i, _p, _i, _i, _p, _i, _i,
                               _i, _p, _i, _p, _i, _p]),
    "upr_t_cast_f16": (_i, [_p, _p, c_size_t, _p]),
    "upr_t_conv_wgrad": (_i, [_p, _i, _i, _i, _i, _i, _i, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p]),
    "upr_t_conv_wgrad16": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p]),
    "upr_t_conv_mfma16_relu_bwd": (_i, [_p, _i, _i, _i, _i, _p, _i, _i, _i, _i, _i, _p, _i, _i, _p, _i, _p, _i, _i,
                                        _p]),
    "upr_t_conv_mfma16_relu_bwd_cs": (_i, [_p, _i, _i, _i, _i, _i, _p, _i, _i, _i, _i, _i, _p, _i, _i, _p, _i, _p,
                                           _i, _i, _p]),
    "upr_t_conv_wgrad_into": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i,
                                   _p, _p]),
    "upr_t_pack_weight": (_i, [_p, _p, _i, _i, _i, _i, _i, _p]),
    "upr_t_pack_weights": (_i, [_p, _i, _i, _p]),
    "upr_t_unpack_grad": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _p]),
    "upr_t_zero_upsample": (_i, [_p, _i, _i, _i, _i, _i, _i, _p, _p]),
    "upr_t_bn_stats": (_i, [_p, _i, _i, _i, _i, _p, _p]),
    "upr_t_bn_finalize": (_i, [_p, _i, _i, _f, _f, _p, _p, _p, _p, _p, _p]),
    "upr_t_bn_eval_stats": (_i, [_p, _p, _i, _f, _p, _p, _p]),
    "upr_t_bn_apply": (_i, [_p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _i, _i, _p]),
    "upr_t_bn_apply16": (_i, [_p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _i, _i, _p, _p]),
    "upr_t_bn_bwd_reduce": (_i, [_p, _i, _i, _p, _i, _i, _p, _p, _i, _i, _p, _p]),
    "upr_t_bn_bwd_apply": (_i, [_p, _i, _i, _p, _i, _i, _p, _p, _p, _p, _i, _i, _p, _p, _p, _i, _i, _i, _i, _p]),
    "upr_t_chan_sum": (_i, [_p, _i, _i, _i, _i, _p, _i, _p]),
    "upr_t_chan_sum_ws": (_i, [_p, _i, _i, _i, _i, _p, _i, _p, _p]),
    "upr_t_reduce_acc_doubles": (_i, [_i]),
    "upr_t_bn_bwd_fused": (_i, [_p, _i, _i, _p, _i, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _i, _i, _i, _i, _p,
                                _p]),
    "upr_t_bn_stats16": (_i, [_p, _i, _i, _p, _p]),
    "upr_t_bn_stats16_fin": (_i, [_p, _i, _i, _p, _f, _f, _p, _p, _p, _p, _p, _p]),
    "upr_t_bn_apply16h": (_i, [_p, _i, _i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _i, _i, _p, _i, _p]),
    "upr_t_bn_apply16h_cs": (_i, [_p, _i, _i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _i, _i, _p, _i, _i, _p]),
    "upr_t_bn_bwd_fused16": (_i, [_p, _p, _i, _i, _p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _i, _i, _i, _i,
                                  _p, _i, _p]),
    "upr_t_chan_sum16": (_i, [_p, _i, _i, _p, _i, _p, _p]),
    "upr_t_chan_sum16s": (_i, [_p, _i, _i, _i, _p, _i, _p, _p]),
    "upr_t_zero_upsample16h": (_i, [_p, _i, _i, _i, _i, _p, _p]),
    "upr_t_zero_upsample16": (_i, [_p, _i, _i, _i, _i, _i, _i, _p, _p]),
    "upr_t_relu_mask": (_i, [_p, _i, _i, _p, _i, _i, _i, _i, _p]),
    "upr_t_relu_mask16": (_i, [_p, _i, _i, _p, _i, _i, _i, _i, _p, _i, _p]),
    "upr_t_copy": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _p]),
    "upr_t_pointwise": (_i, [_p, _p, _p, c_size_t, _i, _p, _p, _f, c_u64, _p]),
    "upr_t_texture_complexity": (_i, [_p, _i, _i, _i, _i, _i, _p, _p, _p]),
    "upr_t_maxpool": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _p]),
    "upr_t_maxpool_bwd": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _p]),
    "upr_t_maxpool_code": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _p, _p, _p]),
    "upr_t_maxpool16_code": (_i, [_p, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _p, _p, _p]),
    "upr_t_relu_mask16h": (_i, [_p, _i, _i, _p, _i, _i, _i, _p, _i, _p]),
    "upr_t_copy16": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _p, _i, _p]),
    "upr_t_bilinear16": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _i, _p, _i, _p]),
    "upr_t_add16": (_i, [_p, _p, _p, c_size_t, _p, _p]),
    "upr_t_maxpool_bwd_code": (_i, [_p, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _p]),
    "upr_t_maxpool_bwd_code16": (_i, [_p, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p]),
    "upr_t_bilinear": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _i, _p]),
    "upr_t_bilinear_bwd": (_i, [_vp, _i, _i, _i, _i, _i, _i, _vp, _p]),
    "upr_t_pixel_sum": (_i, [_p, _i, _i, _i, _i, _i, _f, _p, _i, _p]),
    "upr_t_broadcast": (_i, [_p, _i, _i, _i, _f, _p, _i, _i, _i, _p]),
    "upr_t_broadcast16": (_i, [_p, _i, _i, _i, _f, _p, _i, _i, _p]),
    "upr_t_fam_ca_apply": (_i, [_p, _p, _i, _i, _i, _p, _p, _p]),
    "upr_t_fam_sa_apply": (_i, [_p, _p, _i, _i, _i, _p, _p, _p]),
    "upr_t_fam_sa_bwd": (_i, [_p, _p, _p, _i, _i, _i, _p, _p, _p]),
    "upr_t_fam_sa_bwd_cs": (_i, [_p, _i, _p, _p, _i, _i, _i, _p, _p, _p]),
    "upr_t_fam_ca_bwd": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p]),
    "upr_t_fam_pool_bwd": (_i, [_p, _p, _p, _i, _i, _i, _p]),
    "upr_t_fam_pool_bwd16": (_i, [_p, _p, _p, _i, _i, _i, _p, _p]),
    "upr_t_head_fwd": (_i, [_p, _p, _p, _i, _i, _i, _p]),
    "upr_t_retinex_fwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _p]),
    "upr_t_retinex_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p]),
    "upr_t_enhance_fwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _p]),
    "upr_t_enhance_bwd": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _p]),
    "upr_t_loss_workspace": (c_size_t, [_i, _i, _i]),
    "upr_t_loss_workspace_p": (c_size_t, [_i, _i, _i, _i]),
    "upr_t_loss_pixel_p": (_i, [_p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p, _i, _f, _f, _f, _f, _f, _i, _p, _p]),
    "upr_t_loss_pixel": (_i, [_p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p, _i, _f, _f, _f, _f, _f, _i, _p]),
    "upr_t_mse": (_i, [_p, _p, c_size_t, _p, _p, _f, _p]),
    "upr_t_mse16": (_i, [_p, _p, c_size_t, _p, _p, _f, _p]),
    "upr_t_vgg_norm": (_i, [_p, _p, _i, _i, _i, _p]),
    "upr_t_vgg_norm_bwd": (_i, [_p, _p, _i, _i, _i, _p]),
    "upr_t_freq": (_i, [_p, _p, _i, _i, _i, _p, _p, _f, _p]),
    "upr_t_freq_p": (_i, [_p, _p, _i, _i, _i, _p, _p, _f, _f, _f, _p]),
    "upr_t_add_real": (_i, [_p, _p, c_size_t, _f, _p]),
    "upr_t_scale_acc": (_i, [_p, _i, _f, _p, _p]),
    "upr_t_loss_total": (_i, [_p, _f, _f, _f, _f, _f, _f, _p]),
    "upr_t_sqsum": (_i, [_p, c_size_t, _p, _p]),
    "upr_t_unscale": (_i, [_p, c_size_t, _p, _p, _p]),
    "upr_t_adam": (_i, [_p, _p, _p, _p, c_size_t, _p, _f, _f, _f, _f, _f, _f, _i, _p, _p]),
})

_lib = None


class UprError(RuntimeError):
    pass


def lib():
    """Load libupr.so once; raise loudly if it is absent (no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise UprError(f"libupr.so not found at {LIB_PATH}: build it with `make -C "
                           f"retinex-image-enhancement_amd/csrc` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def status_string(rc):
    return lib().upr_status_string(int(rc)).decode()


def check(rc, what):
    """Map a C status to the reference's error behaviour: shape/argument errors
    raise ValueError/RuntimeError like torch would; HIP errors raise UprError."""
    if rc == UPR_OK:
        return
    msg = f"{what}: {status_string(rc)} (status {rc})"
    if rc in (UPR_ERR_SHAPE,):
        raise RuntimeError(msg)
    if rc in (UPR_ERR_ARG, UPR_ERR_MISSING_PARAM):
        raise ValueError(msg)
    raise UprError(msg)
