"""ctypes binding of libugpg.so (the C-ABI declared in include/ugpg.h).

The library is built in-tree by ``ug-pg-unet_amd/build.py`` (or
``__graft_entry__.build()``).  There is deliberately no fallback: if the shared
library is missing every hot-path op raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(os.environ.get("UGPG_LIB", Path(__file__).resolve().parent / "libugpg.so"))

c_float_p = C.c_void_p
_i, _i64, _f, _p, _sz = C.c_int, C.c_int64, C.c_float, C.c_void_p, C.c_size_t


class Src(C.Structure):
    """ugpg_src_t: lazily-activated NHWC operand."""
    _fields_ = [("data", _p), ("scale", _p), ("shift", _p), ("C", _i), ("data_bf16", _p)]


class ConvDesc(C.Structure):
    """ugpg_conv_t."""
    _fields_ = [("B", _i), ("H", _i), ("W", _i), ("src", Src * 2), ("wpk", _p), ("bias", _p),
                ("Cout", _i), ("out", _p * 2), ("out_split", _i), ("accumulate", _i * 2),
                ("stats", _p), ("stats_slots", _i), ("wfmt", _i), ("bnb_y", _p),
                ("bnb_y_bf16", _p), ("bnb_mean", _p), ("bnb_invstd", _p), ("bnb_scale", _p), ("bnb_shift", _p),
                ("bnb_part", _p), ("bnb_slots", _i), ("out_bf16", _p)]


class Bnb(C.Structure):
    """ugpg_bnb_t."""
    _fields_ = [("y", _p), ("y_bf16", _p), ("mean", _p), ("invstd", _p), ("scale", _p),
                ("shift", _p), ("part", _p), ("nslots", _i)]


class BwdRoute(C.Structure):
    """ugpg_bwd_route_t."""
    _fields_ = [("kind", _i), ("src", _p), ("argmax", _p), ("w", _p), ("nc", _i), ("B", _i),
                ("H", _i), ("W", _i)]


class PackItem(C.Structure):
    """ugpg_pack_item_t."""
    _fields_ = [("w", _p), ("wpk", _p), ("Cout", _i), ("Cin", _i), ("Cin_pad", _i), ("mode", _i)]


class BnLazy(C.Structure):
    """ugpg_bn_lazy_t."""
    _fields_ = [("da", _p), ("y", _p), ("mean", _p), ("invstd", _p), ("scale", _p), ("shift", _p),
                ("coef", _p), ("dy_out", _p), ("route_src", _p), ("route_argmax", _p),
                ("y_bf16", _p)]


class WgradDesc(C.Structure):
    """ugpg_wgrad_t."""
    _fields_ = [("B", _i), ("H", _i), ("W", _i), ("src", Src * 2), ("dy", _p), ("dy_bf16", _p),
                ("Cout", _i), ("dw", _p), ("Cin_real", _i), ("db", _p), ("accumulate", _i), ("math", _i),
                ("dy_bn", C.POINTER(BnLazy))]


# name -> (restype, argtypes); must match include/ugpg.h exactly
SIGNATURES = {
    "ugpg_version": (C.c_char_p, []),
    "ugpg_build_id": (C.c_char_p, []),
    "ugpg_last_error": (C.c_char_p, []),
    "ugpg_conv3x3_fwd": (_i, [C.POINTER(ConvDesc), _p]),
    "ugpg_conv3x3_fwd_ntiles": (_i, [_i, _i, _i, _i, _i, _i]),
    "ugpg_pack_conv3x3_bytes": (_sz, [_i, _i, _i]),
    "ugpg_pack_conv3x3_batch": (_i, [C.POINTER(PackItem), _i, _i, _p]),
    "ugpg_pack_conv3x3": (_i, [_p, _p, _i, _i, _i, _i, _i, _p]),
    "ugpg_conv3x3_wgrad_workspace": (_sz, [C.POINTER(WgradDesc)]),
    "ugpg_conv3x3_wgrad": (_i, [C.POINTER(WgradDesc), _p, _sz, _p]),
    "ugpg_bn_finalize": (_i, [_p, _i, _i, _p, _p, _p, _p, _p, _f, _f, _p, _p, _p, _p, _p]),
    "ugpg_bn_stats_pack": (_i, [_p, _i, _i, _p, _p]),
    "ugpg_bn_finalize_merged": (_i, [_p, _i, _i, _p, _p, _p, _p, _p, _f, _f, _p, _p, _p, _p, _p]),
    "ugpg_bn_relu_bwd_reduce": (_i, [_p, _p, _p, _i64, _i, _p, _p, _p, _p, _p, _i, _p]),
    "ugpg_bn_bwd_partials_pack": (_i, [_p, _i, _i, _i64, _p, _p]),
    "ugpg_bn_bwd_partials_unpack": (_i, [_p, _i64, _p, _i, _i, _p]),
    "ugpg_bn_eval_params": (_i, [_p, _p, _p, _p, _f, _i, _p, _p, _p]),
    "ugpg_bn_relu_bwd_workspace": (_sz, [_i64, _i]),
    "ugpg_bn_relu_bwd": (_i, [_p, _p, _p, _i64, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _p,
                              _sz, _p]),
    "ugpg_bn_relu_bwd_partials_workspace": (_sz, [_i]),
    "ugpg_bn_relu_bwd_partials": (_i, [_p, _i, _p, _p, _p, _p, _i64, _i, _p, _p, _p, _p, _p, _p,
                                       _p, _p, _p, _i, _p, _sz, _p]),
    "ugpg_bn_relu_bwd_partials_routed": (_i, [C.POINTER(BwdRoute), _p, _i, _p, _p, _p, _i64, _i, _p,
                                              _p, _p, _p, _p, _p, _p, _p, _p, _i, _p, _sz, _p]),
    "ugpg_bn_relu_apply": (_i, [Src, _i64, _p, _p]),
    "ugpg_maxpool2_fwd": (_i, [Src, _i, _i, _i, _p, _p, _p, _p]),
    "ugpg_maxpool2_bwd": (_i, [_p, _p, _i, _i, _i, _i, _p, _i, _p]),
    "ugpg_maxpool2_bwd_bnb": (_i, [_p, _p, _i, _i, _i, _i, _p, _i, C.POINTER(Bnb), _p]),
    "ugpg_maxpool2_bwd_partials": (_i, [_p, _p, _i, _i, _i, _i, _p, C.POINTER(Bnb), _p]),
    "ugpg_bnb_slots": (_i, [_i64, _i]),
    "ugpg_bilinear_nhwc_fwd": (_i, [Src, _i, _i, _i, _p, _i, _i, _p, _p]),
    "ugpg_bilinear_nhwc_bwd": (_i, [_p, _i, _i, _i, _i, _p, _i, _i, _i, _p]),
    "ugpg_bilinear_nhwc_bwd_bnb": (_i, [_p, _i, _i, _i, _i, _p, _i, _i, _i, C.POINTER(Bnb), _p]),
    "ugpg_cast_f32_bf16": (_i, [_p, _p, _i64, _p]),
    "ugpg_cast_bf16_f32": (_i, [_p, _p, _i64, _p]),
    "ugpg_resize_nchw": (_i, [_p, _i, _i, _i, _i, _p, _i, _i, _i, _p]),
    "ugpg_resize_nchw_bwd": (_i, [_p, _i, _i, _i, _i, _p, _i, _i, _p]),
    "ugpg_nchw_to_nhwc": (_i, [_p, _i, _i, _i, _i, _p, _i, _p]),
    "ugpg_nhwc_to_nchw": (_i, [_p, _i, _i, _i, _i, _i, _p, _i, _p]),
    "ugpg_head_fwd": (_i, [Src, _i64, _p, _p, _i, _p, _p]),
    "ugpg_heads_combine": (_i, [_p, _p, _i, _i, _i, _i, _i, _p, _p]),
    "ugpg_heads_split_bwd": (_i, [_p, _i, _i, _i, _i, _p, _p, _i, _p]),
    "ugpg_head_bwd_workspace": (_sz, [_i64, _i, _i]),
    "ugpg_head_bwd": (_i, [Src, _i64, _p, _i, _p, _p, _p, _p, _i, _p, _sz, _p]),
    "ugpg_head_bwd_bnb_slots": (_i, [_i64]),
    "ugpg_head_bwd_bnb": (_i, [Src, _i64, _p, _i, _p, _p, _p, _p, _i, _p, _sz, C.POINTER(Bnb), _p]),
    "ugpg_ug_loss_workspace": (_sz, [_i64]),
    "ugpg_ug_loss_fwd": (_i, [_p, _p, _p, _i, _i, _i, _i, _p, _f, _p, _p, _sz, _p]),
    "ugpg_ug_loss_bwd": (_i, [_p, _p, _p, _i, _i, _i, _i, _p, _f, _p, _p, _p]),
    "ugpg_weighted_mean_fwd": (_i, [_p, _p, _i, _i, _i, _i, _f, _p, _p, _sz, _p]),
    "ugpg_weighted_mean_bwd": (_i, [_p, _i, _i, _i, _i, _f, _p, _p, _p]),
    "ugpg_seg_metrics_workspace": (_sz, [_i]),
    "ugpg_seg_metrics": (_i, [_p, _p, _i, _i, _p, _p, _sz, _p]),
    "ugpg_seg_eval_workspace": (_sz, [_i, _i]),
    "ugpg_seg_eval": (_i, [_p, _p, _i, _i, _p, _p, _sz, _p]),
    "ugpg_predict_mask": (_i, [_p, _i, _i, _i, _p, _i, _i, _p]),
    "ugpg_mean_std_workspace": (_sz, [_i64]),
    "ugpg_mean_std": (_i, [_p, _i64, _p, _p, _sz, _p]),
    "ugpg_comm_id_bytes": (_sz, []),
    "ugpg_comm_unique_id": (_i, [_p, _sz]),
    "ugpg_comm_init": (_i, [C.POINTER(_p), _i, _i, _p, _sz, _i]),
    "ugpg_comm_allreduce": (_i, [_p, _p, _p, _sz, _i, _i, _p]),
    "ugpg_comm_broadcast": (_i, [_p, _p, _p, _sz, _i, _i, _p]),
    "ugpg_comm_destroy": (_i, [_p]),
    "ugpg_metrics_pack": (_i, [_p, _i, _i, C.c_double, _p, _p]),
    "ugpg_metrics_unpack": (_i, [_p, _i, _i, C.c_uint, _p, _p]),
    "ugpg_rmsprop_step": (_i, [_p, _p, _p, _i64, _f, _f, _f, _f, _f, _p]),
    "ugpg_avgpool_fwd": (_i, [Src, _i, _i, _p, _p]),
    "ugpg_avgpool_bwd": (_i, [_p, _i, _i, _i, _p, _i, _p]),
    "ugpg_linear_fwd": (_i, [_p, _p, _p, _i, _i, _i, _i, _p, _p]),
    "ugpg_linear_bwd": (_i, [_p, _p, _p, _i, _i, _i, _p, _p, _p, _p]),
    "ugpg_dropout_mask": (_i, [_p, _i64, _f, C.c_uint64, _p]),
    "ugpg_ce_ug_fwd": (_i, [_p, _p, _p, _p, _i, _i, _f, _p, _p, _p]),
    "ugpg_ce_ug_bwd": (_i, [_p, _p, _p, _p, _i, _i, _p, _p, _p]),
    "ugpg_adam_step": (_i, [_p, _p, _p, _p, _i64, _f, _f, _f, _f, _f, _i64, _f, _p]),
    "ugpg_relu_bwd": (_i, [_p, _p, _p, _i64, _p]),
    "ugpg_mul": (_i, [_p, _p, _p, _i64, _p]),
    "ugpg_resample_aa_u8": (_i, [_p, _i64, _i, _i, _i, _p, _p, _i, _p, _p]),
    "ugpg_resize_nearest_u8": (_i, [_p, _i64, _i, _i, _i, _p, _p, _p, _i, _i, _p]),
    "ugpg_augment_param_sizes": (_i, [C.POINTER(_i), C.POINTER(_i)]),
    "ugpg_augment_geom": (_i, [_p, _p, _i, _i64, _p, _p, _p, _p, _p]),
    "ugpg_augment_color": (_i, [_p, _p, _i, _i64, _p, _p, _p, _p, _p, _p]),
    "ugpg_rasterize_polygons_ws_size": (_sz, [_i64, _i64]),
    "ugpg_rasterize_polygons": (_i, [_p, _p, _i64, _i64, _p, _i, _i, _i, _p, _sz, _p]),
}


def _check_fresh(lib) -> None:
    """Refuse an in-tree libugpg.so built from other sources than the ones beside it (a
    stale prebuilt library travelling with the tree): the content part
    of its embedded ugpg_build_id() must equal build.content_id() of csrc/ + include/.  The
    compile configuration (flags, UGPG_ARCH, defines) is not compared: it is the builder's,
    not this process's environment.  Skipped for an explicit UGPG_LIB (A/B
    variants are built from other defines on purpose)."""
    if "UGPG_LIB" in os.environ:
        return
    bpy = Path(__file__).resolve().parent.parent / "build.py"
    if not bpy.exists():
        return
    import importlib.util
    spec = importlib.util.spec_from_file_location("_ugpg_build", bpy)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    want = mod.content_id()
    fn = getattr(lib, "ugpg_build_id", None)
    got = None
    if fn is not None:
        fn.restype, fn.argtypes = C.c_char_p, []
        got = fn().decode().split("-")[0]
    if got != want:
        raise ImportError(
            f"ugpg: {LIB_PATH} is stale (built from sources {got}, tree has {want}) -- "
            "rebuild it with `python ug-pg-unet_amd/build.py`. There is no CPU fallback.")


class _Lib:
    def __init__(self):
        self._lib = None

    def load(self):
        if self._lib is None:
            if not LIB_PATH.exists():
                raise ImportError(
                    f"ugpg: native library {LIB_PATH} not found -- build it with "
                    "`python ug-pg-unet_amd/build.py` (hipcc, gfx950). There is no CPU fallback.")
            lib = C.CDLL(str(LIB_PATH))
            _check_fresh(lib)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            self._lib = lib
        return self._lib

    def __getattr__(self, name):
        return getattr(self.load(), name)


lib = _Lib()


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib.ugpg_last_error().decode(errors="replace")
        raise RuntimeError(f"ugpg {what} failed ({rc}): {msg}")


def version() -> str:
    return lib.ugpg_version().decode()
