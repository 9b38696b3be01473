"""ctypes binding of libsdfr.so (the C ABI declared in include/sdfr.h).

The library is built in-tree by ``make -C sdface-gan_amd`` (or
``__graft_entry__.build()``) into ``sdface-gan_amd/lib/libsdfr.so``.  There is
no fallback: if the library is missing or a call fails, a RuntimeError is
raised naming the entry point and the library's own message.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("SDFR_LIB", PKG_DIR / "lib" / "libsdfr.so"))

_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_f32 = ctypes.c_float
_int = ctypes.c_int

SDFR_OK = 0
SDFR_EINVAL = -1
SDFR_ELAUNCH = -2
SDFR_EUNSUPPORTED = -3
ABI_VERSION = 13
FIELD_F16X3 = 0
FIELD_FP32 = 1

# every symbol include/sdfr.h declares outside its SDFR_ABLATION block (tests check the
# product .so exports all of them and nothing else with the sdfr_ prefix)
ABLATION_EXPORTS = ("sdfr_debug_set_field_variant", "sdfr_debug_set_encode_mode")
EXPORTS = (
    "sdfr_abi_version", "sdfr_last_error",
    "sdfr_grid_encode_forward", "sdfr_grid_encode_backward",
    "sdfr_grid_encode_backward_ws_bytes", "sdfr_grid_encode_backward_ws",
    "sdfr_sh_encode_forward", "sdfr_sh_encode_backward",
    "sdfr_render_ngp_workspace_bytes", "sdfr_render_ngp_forward",
    "sdfr_render_ngp_encode_only", "sdfr_debug_sin_probe",
    "sdfr_debug_sin_rev_probe", "sdfr_camera_extrinsics",
    "sdfr_render_siren_workspace_bytes", "sdfr_render_siren_forward",
    "sdfr_render_pack_bytes", "sdfr_render_ngp_pack", "sdfr_render_siren_pack",
    "sdfr_render_fc_workspace_bytes", "sdfr_render_fc_forward", "sdfr_render_fc_pack",
    "sdfr_fused_bias_act", "sdfr_mapping_linear", "sdfr_decoder_styles", "sdfr_upfirdn2d", "sdfr_styled_epilogue", "sdfr_modulate_to_nhwc",
    "sdfr_modulate_to_nhwc_split",
    "sdfr_conv_pack_bytes", "sdfr_conv_pack_weights", "sdfr_conv3x3_f16x3",
    "sdfr_conv3x3_f16x3_ws", "sdfr_conv_ws_bytes", "sdfr_set_conv_t_mode",
    "sdfr_conv3x3_f16x3_act", "sdfr_conv_act_ws_bytes", "sdfr_rgb_finish",
    "sdfr_conv_t_act", "sdfr_conv_t_act_supported",
    "sdfr_mc_workspace_bytes", "sdfr_mc_count", "sdfr_mc_emit",
    "sdfr_linear_pack_bytes", "sdfr_linear_pack", "sdfr_linear_f16x3",
    "sdfr_linear_wgrad_ws_bytes", "sdfr_linear_wgrad_f16x3",
    "sdfr_film_linear_f16x3", "sdfr_film_backward_ws_bytes", "sdfr_film_backward",
    "sdfr_film_backward_grad_ws_bytes", "sdfr_film_backward_grad",
    "sdfr_linear_head_forward", "sdfr_linear_head_ws_bytes", "sdfr_linear_head_backward",
)


class NgpWeights(ctypes.Structure):
    """sdfr_ngp_weights (include/sdfr.h)."""
    _fields_ = [
        ("embeddings", _vp), ("offsets", _vp), ("num_levels", _u32),
        ("log2_per_level_scale", _f32), ("base_resolution", _u32), ("bound", _f32),
        ("input_w", _vp), ("input_b", _vp),
        ("pts_w", _vp * 3), ("pts_b", _vp * 3), ("pts_gw", _vp * 3), ("pts_gb", _vp * 3),
        ("pts_bw", _vp * 3), ("pts_bb", _vp * 3),
        ("views_w", _vp), ("views_b", _vp),
        ("views_gw", _vp), ("views_gb", _vp), ("views_bw", _vp), ("views_bb", _vp),
        ("sigma_w", _vp), ("sigma_b", _vp), ("rgb_w", _vp), ("rgb_b", _vp),
        ("sigmoid_beta", _vp),
    ]


class SirenWeights(ctypes.Structure):
    """sdfr_siren_weights (include/sdfr.h)."""
    _fields_ = [
        ("depth", _u32), ("width", _u32),
        ("pts_w", _vp * 8), ("pts_b", _vp * 8), ("pts_gw", _vp * 8), ("pts_gb", _vp * 8),
        ("pts_bw", _vp * 8), ("pts_bb", _vp * 8),
        ("views_w", _vp), ("views_b", _vp),
        ("views_gw", _vp), ("views_gb", _vp), ("views_bw", _vp), ("views_bb", _vp),
        ("sigma_w", _vp), ("sigma_b", _vp), ("rgb_w", _vp), ("rgb_b", _vp),
        ("sigmoid_beta", _vp),
    ]


class FcWeights(ctypes.Structure):
    """sdfr_fc_weights (include/sdfr.h)."""
    _fields_ = [
        ("depth", _u32), ("width", _u32),
        ("x_in_w", _vp), ("x_in_b", _vp), ("style_w", _vp), ("style_b", _vp),
        ("pts_w", _vp * 7), ("pts_b", _vp * 7),
        ("views_w", _vp), ("views_b", _vp),
        ("sigma_w", _vp), ("sigma_b", _vp), ("rgb_w", _vp), ("rgb_b", _vp),
        ("sigmoid_beta", _vp),
    ]


class NgpRenderArgs(ctypes.Structure):
    """sdfr_ngp_render_args (include/sdfr.h)."""
    _fields_ = [
        ("B", _u32), ("H", _u32), ("W", _u32), ("N", _u32),
        ("cam", _vp), ("focal", _vp), ("near_", _vp), ("far_", _vp), ("styles", _vp),
        ("pix_x", _vp), ("pix_y", _vp), ("t_vals", _vp), ("t_rand", _vp), ("sigma_noise", _vp),
        ("t_rand_per_sample", _int), ("offset_sampling", _int), ("static_viewdirs", _int),
        ("z_normalize", _int), ("force_background", _int), ("with_sdf", _int),
        ("rgb", _vp), ("features", _vp), ("sdf", _vp), ("xyz", _vp), ("mask", _vp),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t),
        ("stage_events", _vp * 4), ("field_precision", _int), ("prepacked", _vp),
        ("max_field_segments", _u32),
        ("styles_event", _vp), ("field_event", _vp),
        ("features_split", _vp), ("features_mod", _vp),
    ]


class StyledEpilogueArgs(ctypes.Structure):
    """sdfr_styled_epilogue_args (include/sdfr.h)."""
    _fields_ = [
        ("B", _u32), ("C", _u32), ("H", _u32), ("W", _u32),
        ("conv", _vp), ("blur_up", _int), ("fir", _f32 * 4),
        ("demod", _vp), ("noise", _vp), ("noise_weight", _vp), ("bias", _vp),
        ("negative_slope", _f32), ("act_scale", _f32),
        ("s_next", _vp), ("y", _vp), ("rgb_w", _vp), ("rgb_b", _vp), ("skip", _vp), ("rgb", _vp),
        ("y_split", _vp),
    ]


class StyleArgs(ctypes.Structure):
    """sdfr_style_args (include/sdfr.h)."""
    _fields_ = [
        ("B", _u32), ("n_latent", _u32), ("K", _u32), ("latent", _vp),
        ("L", _u32), ("cmax", _u32), ("mod_w", _vp), ("mod_b", _vp),
        ("mod_index", _u32 * 16), ("mod_c", _u32 * 16), ("mod_off", _u32 * 16), ("mods", _vp),
        ("J", _u32), ("omax", _u32), ("dem_w", _vp), ("dem_eps", _vp),
        ("dem_layer", _u32 * 16), ("dem_c", _u32 * 16), ("dem_off", _u32 * 16), ("demods", _vp),
    ]


class ConvActArgs(ctypes.Structure):
    """sdfr_conv_act_args (include/sdfr.h)."""
    _fields_ = [
        ("x_split", _vp), ("packed", _vp),
        ("B", _u32), ("H", _u32), ("W", _u32), ("Cin", _u32), ("Cout", _u32),
        ("demod", _vp), ("noise", _vp), ("noise_weight", _vp), ("bias", _vp),
        ("negative_slope", _f32), ("act_scale", _f32),
        ("s_next", _vp), ("y_split", _vp), ("rgb_w", _vp), ("rgb_partial", _vp),
        ("ws", _vp), ("ws_bytes", ctypes.c_size_t),
        ("rgb_base", _vp), ("rgb_s", _vp),
    ]


class ConvTActArgs(ctypes.Structure):
    """sdfr_conv_t_act_args (include/sdfr.h, ABI 13)."""
    _fields_ = [
        ("x_split", _vp), ("packed", _vp),
        ("B", _u32), ("H", _u32), ("W", _u32), ("Cin", _u32), ("Cout", _u32),
        ("fir", _f32 * 4),
        ("demod", _vp), ("noise", _vp), ("noise_weight", _vp), ("bias", _vp),
        ("negative_slope", _f32), ("act_scale", _f32),
        ("s_next", _vp), ("y_split", _vp), ("raw", _vp),
    ]


_lib = None


def lib():
    """Load libsdfr.so once; raise if it is absent (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(
            f"sdface-gan_amd: HIP library {LIB_PATH} is missing; build it with "
            "`make -C sdface-gan_amd` or `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(str(LIB_PATH))
    L.sdfr_abi_version.restype = _int
    L.sdfr_last_error.restype = ctypes.c_char_p
    L.sdfr_grid_encode_forward.argtypes = [_vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32, _f32,
                                           _u32, _vp, _u32, _int, _u32, _vp]
    L.sdfr_grid_encode_backward.argtypes = [_vp, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32,
                                            _f32, _u32, _vp, _vp, _u32, _int, _u32, _vp]
    L.sdfr_grid_encode_backward_ws_bytes.argtypes = [_u32, _u32, _u32, _u32, _f32, _u32, _int]
    L.sdfr_grid_encode_backward_ws_bytes.restype = ctypes.c_size_t
    L.sdfr_grid_encode_backward_ws.argtypes = (L.sdfr_grid_encode_backward.argtypes[:-1]
                                               + [_vp, ctypes.c_size_t, _vp])
    L.sdfr_sh_encode_forward.argtypes = [_vp, _vp, _u32, _u32, _u32, _vp, _vp]
    L.sdfr_sh_encode_backward.argtypes = [_vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp]
    L.sdfr_render_ngp_workspace_bytes.restype = ctypes.c_size_t
    L.sdfr_render_ngp_workspace_bytes.argtypes = [_u32, _u32, _u32, _u32, _u32]
    L.sdfr_render_ngp_forward.argtypes = [ctypes.POINTER(NgpWeights),
                                          ctypes.POINTER(NgpRenderArgs), _vp]
    L.sdfr_render_ngp_encode_only.argtypes = [ctypes.POINTER(NgpWeights),
                                              ctypes.POINTER(NgpRenderArgs), _vp]
    for name in ABLATION_EXPORTS:           # profiling builds only (make ABLATION=1)
        if hasattr(L, name):
            getattr(L, name).argtypes = [_int]
    L.sdfr_render_siren_workspace_bytes.restype = ctypes.c_size_t
    L.sdfr_render_siren_workspace_bytes.argtypes = [_u32]
    L.sdfr_render_pack_bytes.argtypes = [_int]
    L.sdfr_render_pack_bytes.restype = ctypes.c_size_t
    L.sdfr_render_ngp_pack.argtypes = [ctypes.POINTER(NgpWeights), _vp, _vp]
    L.sdfr_render_siren_pack.argtypes = [ctypes.POINTER(SirenWeights), _vp, _vp]
    L.sdfr_render_siren_forward.argtypes = [ctypes.POINTER(SirenWeights),
                                            ctypes.POINTER(NgpRenderArgs), _vp]
    L.sdfr_render_fc_workspace_bytes.restype = ctypes.c_size_t
    L.sdfr_render_fc_workspace_bytes.argtypes = [_u32, _u32, _u32, _u32]
    L.sdfr_render_fc_pack.argtypes = [ctypes.POINTER(FcWeights), _vp, _vp]
    L.sdfr_render_fc_forward.argtypes = [ctypes.POINTER(FcWeights),
                                         ctypes.POINTER(NgpRenderArgs), _vp]
    L.sdfr_debug_sin_probe.argtypes = [_vp, _vp, _vp, _u32, _vp]
    L.sdfr_debug_sin_rev_probe.argtypes = [_vp, _vp, _u32, _vp]
    L.sdfr_camera_extrinsics.argtypes = [_vp, _vp, _u32, _f32, _f32, _f32, _vp, _vp, _vp, _vp,
                                         _vp, _vp]
    L.sdfr_fused_bias_act.argtypes = [_vp, _vp, _vp, _vp, ctypes.c_uint64, _u32, _u32, _int, _int,
                                      _f32, _f32, _vp]
    L.sdfr_mapping_linear.argtypes = [_vp, _vp, _vp, _vp, _u32, _u32, _u32, _f32, _f32, _int, _f32,
                                      _f32, _int, _vp]
    L.sdfr_decoder_styles.argtypes = [ctypes.POINTER(StyleArgs), _vp]
    L.sdfr_upfirdn2d.argtypes = [_vp, _vp, _vp, _u32, _u32, _u32, _u32, _u32] + [_int] * 8 + [_vp]
    L.sdfr_styled_epilogue.argtypes = [ctypes.POINTER(StyledEpilogueArgs), _vp]
    L.sdfr_modulate_to_nhwc.argtypes = [_vp, _vp, _vp, _u32, _u32, _u32, _vp]
    L.sdfr_modulate_to_nhwc_split.argtypes = [_vp, _vp, _vp, _u32, _u32, _u32, _vp]
    L.sdfr_conv_pack_bytes.restype = ctypes.c_size_t
    L.sdfr_conv_pack_bytes.argtypes = [_u32, _u32]
    L.sdfr_conv_pack_weights.argtypes = [_vp, _f32, _u32, _u32, _vp, _vp, _vp]
    L.sdfr_conv3x3_f16x3.argtypes = [_vp, _vp, _vp, _u32, _u32, _u32, _u32, _u32, _int, _vp]
    L.sdfr_conv3x3_f16x3_ws.argtypes = [_vp, _vp, _vp, _u32, _u32, _u32, _u32, _u32, _int, _vp,
                                        ctypes.c_size_t, _vp]
    L.sdfr_conv_ws_bytes.argtypes = [_u32, _u32, _u32, _u32, _int]
    L.sdfr_conv_ws_bytes.restype = ctypes.c_size_t
    L.sdfr_set_conv_t_mode.argtypes = [_int]
    L.sdfr_set_conv_t_mode.restype = _int
    L.sdfr_conv3x3_f16x3_act.argtypes = [ctypes.POINTER(ConvActArgs), _vp]
    L.sdfr_conv_t_act.argtypes = [ctypes.POINTER(ConvTActArgs), _vp]
    L.sdfr_conv_t_act_supported.argtypes = [_u32, _u32, _u32, _u32, _u32]
    L.sdfr_conv_t_act_supported.restype = _int
    L.sdfr_conv_act_ws_bytes.argtypes = [_u32, _u32, _u32, _u32]
    L.sdfr_conv_act_ws_bytes.restype = ctypes.c_size_t
    _i64 = ctypes.c_int64
    L.sdfr_mc_workspace_bytes.argtypes = [_u32, _u32, _u32]
    L.sdfr_mc_workspace_bytes.restype = ctypes.c_size_t
    L.sdfr_mc_count.argtypes = [_vp, _u32, _u32, _u32, _i64, _i64, _i64, _f32, _vp,
                                ctypes.c_size_t, ctypes.POINTER(_u32), _vp]
    L.sdfr_mc_emit.argtypes = [_vp, _u32, _u32, _u32, _i64, _i64, _i64, _f32, _vp,
                               ctypes.c_size_t, _vp, _vp, _vp]
    L.sdfr_rgb_finish.argtypes = [_vp, _vp, _u32, _vp, _vp, ctypes.POINTER(_f32), _u32, _u32,
                                  _u32, _vp]
    L.sdfr_linear_pack_bytes.argtypes = [_u32, _u32]
    L.sdfr_linear_pack_bytes.restype = ctypes.c_size_t
    L.sdfr_linear_pack.argtypes = [_vp, _u32, _u32, _int, _vp, _vp]
    L.sdfr_linear_f16x3.argtypes = [_vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp]
    L.sdfr_linear_wgrad_ws_bytes.argtypes = [_u32, _u32, _u32]
    L.sdfr_linear_wgrad_ws_bytes.restype = ctypes.c_size_t
    L.sdfr_linear_wgrad_f16x3.argtypes = [_vp, _vp, _vp, _u32, _u32, _u32, _vp, ctypes.c_size_t,
                                          _vp]
    L.sdfr_film_linear_f16x3.argtypes = [_vp] * 7 + [_u32] * 4 + [_vp]
    L.sdfr_film_backward_ws_bytes.argtypes = [_u32, _u32, _u32]
    L.sdfr_film_backward_ws_bytes.restype = ctypes.c_size_t
    L.sdfr_film_backward.argtypes = [_vp] * 8 + [_u32] * 3 + [_vp, ctypes.c_size_t, _vp]
    L.sdfr_film_backward_grad_ws_bytes.argtypes = [_u32, _u32, _u32]
    L.sdfr_film_backward_grad_ws_bytes.restype = ctypes.c_size_t
    L.sdfr_film_backward_grad.argtypes = [_vp] * 11 + [_u32] * 3 + [_vp, ctypes.c_size_t, _vp]
    L.sdfr_linear_head_forward.argtypes = [_vp] * 4 + [_u32] * 3 + [_vp]
    L.sdfr_linear_head_ws_bytes.argtypes = [_u32, _u32, _u32]
    L.sdfr_linear_head_ws_bytes.restype = ctypes.c_size_t
    L.sdfr_linear_head_backward.argtypes = [_vp] * 6 + [_u32] * 3 + [_vp, ctypes.c_size_t, _vp]
    v = L.sdfr_abi_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"libsdfr ABI {v} != expected {ABI_VERSION}; rebuild the library")
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != SDFR_OK:
        msg = lib().sdfr_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(t):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
