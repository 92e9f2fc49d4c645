"""ctypes binding of libclearvae_hip.so (the C-ABI declared in include/clearvae.h).

Every struct below mirrors include/clearvae.h field for field.  The library is loaded after
``import torch`` so that it binds to the HIP runtime torch already loaded (same SONAME), which is
what makes torch's device pointers and ``torch.cuda.current_stream().cuda_stream`` valid here.

There is deliberately no CPU fallback: if the shared object is missing or cannot be loaded,
:func:`lib` raises, and every op that needs it fails loudly.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_int64, c_size_t, c_uint64, c_void_p

import torch  # noqa: F401  (must be imported before the HIP library is dlopen'ed)

_HERE = os.path.dirname(os.path.abspath(__file__))
# CVHIP_LIB overrides the in-tree library (kernel-variant experiments only)
LIB_PATH = os.environ.get("CVHIP_LIB") or os.path.join(_HERE, "libclearvae_hip.so")

REC_REPL = 32  # CV_REC_REPL
TICKET_WORDS = 130  # CV_TICKET_WORDS


def stat_repl(C: int) -> int:
    """CV_STAT_REPL(C) of include/clearvae.h: replicas of a C-feature fp64 statistics buffer."""
    return 8 if C >= 256 else 16 if C >= 64 else 32

XF_NONE, XF_BNRELU, XF_BNBWD = 0, 1, 2
STAT_NONE, STAT_FWD, STAT_BWD = 0, 1, 2
SIM = {"cosine": 0, "l2": 1, "modified_l2": 2, "jeffrey": 3, "mahalanobis": 4}
MI_NONE, MI_CLUBSAMPLE, MI_L1OUT = 0, 1, 2
MMA_FP32, MMA_BF16 = 0, 1  # CV_MMA_*
GROUP = {"MLVAE": 0, "GVAE": 1}  # CV_GROUP_*
PRECISION = {"fp32": MMA_FP32, "bf16": MMA_BF16}


class cv_bn(ctypes.Structure):
    _fields_ = [
        ("gamma", c_void_p),
        ("beta", c_void_p),
        ("stat", c_void_p),
        ("gstat", c_void_p),
        ("running_mean", c_void_p),
        ("running_var", c_void_p),
        ("C", c_int),
        ("count", c_int),
        ("train", c_int),
        ("eps", c_float),
        ("cfwd", c_void_p),
        ("cbwd", c_void_p),
        ("ticket", c_void_p),
    ]


class cv_operand(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("y", c_void_p), ("xf", c_int), ("nchw", c_int), ("bn", cv_bn)]


class cv_epilogue(ctypes.Structure):
    _fields_ = [
        ("stat_mode", c_int),
        ("stat_out", c_void_p),
        ("stat_div", c_int),
        ("ey", c_void_p),
        ("ebn", cv_bn),
        ("erelu", c_int),
    ]


class cv_conv(ctypes.Structure):
    _fields_ = [
        ("n", c_int),
        ("c_in", c_int),
        ("h_in", c_int),
        ("w_in", c_int),
        ("c_out", c_int),
        ("h_out", c_int),
        ("w_out", c_int),
        ("kh", c_int),
        ("kw", c_int),
        ("stride", c_int),
        ("pad", c_int),
        ("transposed", c_int),
        ("mma", c_int),
    ]


class cv_linear(ctypes.Structure):
    _fields_ = [
        ("n", c_int),
        ("in_features", c_int),
        ("out_features", c_int),
        ("in_pix", c_int),
        ("in_ch", c_int),
        ("out_pix", c_int),
        ("out_ch", c_int),
        ("mma", c_int),
    ]


class cv_wgrad_defer(ctypes.Structure):
    _fields_ = [("part", c_void_p), ("split", c_int), ("M", c_int), ("N", c_int), ("ntot", c_int), ("cb", c_int),
                ("kk", c_int), ("gweight", c_void_p), ("gbias", c_void_p)]


class cv_tc_disc(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("w1", "b1", "w2", "b2")] + [("zdim", c_int)]


class cv_tc_grad(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("w1", "b1", "w2", "b2")]


class cv_latent_chain(ctypes.Structure):
    _fields_ = [("heads", c_void_p), ("z", c_void_p), ("dz", c_void_p), ("d", c_int), ("rec_in", c_void_p),
                ("losses", c_void_p)]


class cv_ntxent_branch(ctypes.Structure):
    _fields_ = [
        ("mu", c_void_p),
        ("logvar", c_void_p),
        ("ld", c_int),
        ("ps", c_int),
        ("dmu", c_void_p),
        ("dlogvar", c_void_p),
        ("gld", c_int),
        ("gscale", c_void_p),
        ("gmul", c_float),
        ("loss_out", c_void_p),
        ("lse", c_void_p),
    ]


class cv_mlp(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("w1", "b1", "w2", "b2", "w3", "b3", "w4", "b4")] + [
        ("dx", c_int),
        ("h", c_int),
        ("dy", c_int),
    ]


class cv_mlp_grad(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("w1", "b1", "w2", "b2", "w3", "b3", "w4", "b4")]


_P = POINTER
# name -> (restype, argtypes)
class cv_conv_pack(ctypes.Structure):
    _fields_ = [("src", c_void_p), ("gather", c_void_p), ("scatter", c_void_p),
                ("cs", c_int), ("cb", c_int), ("kh", c_int), ("kw", c_int)]


_SIGS = {
    "cv_pack_conv_weights": (c_int, [_P(cv_conv_pack), c_int, c_void_p]),
    "cv_pack_conv_weights_zero": (c_int, [_P(cv_conv_pack), c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "cv_adam_pack_step": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                _P(cv_conv_pack), c_int, c_void_p]),
    "cv_adam_pack_step_part": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                _P(cv_conv_pack), c_int, c_int, c_void_p]),
    "cv_pack_conv_weights_zero_copy": (
        c_int, [_P(cv_conv_pack), c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "cv_conv_forward": (c_int, [_P(cv_conv), _P(cv_operand), c_void_p, c_void_p, c_void_p, _P(cv_epilogue), c_void_p]),
    "cv_conv_backward_data": (c_int, [_P(cv_conv), _P(cv_operand), c_void_p, c_void_p, _P(cv_epilogue), c_void_p]),
    "cv_conv_forward_kpack": (
        c_int, [_P(cv_conv), _P(cv_operand), c_void_p, c_void_p, c_void_p, c_void_p, _P(cv_epilogue), c_void_p]),
    "cv_conv_backward_data_kpack": (
        c_int, [_P(cv_conv), _P(cv_operand), c_void_p, c_void_p, c_void_p, _P(cv_epilogue), c_void_p]),
    "cv_conv_backward_weight": (
        c_int,
        [_P(cv_conv), _P(cv_operand), _P(cv_operand), c_void_p, c_void_p, c_int, c_void_p, c_size_t, c_void_p],
    ),
    "cv_conv_backward_weight_deferred": (
        c_int,
        [_P(cv_conv), _P(cv_operand), _P(cv_operand), c_void_p, c_void_p, c_void_p, c_size_t, _P(cv_wgrad_defer),
         c_void_p],
    ),
    "cv_conv_backward_deferred": (
        c_int,
        [_P(cv_conv), _P(cv_operand), c_void_p, c_void_p, _P(cv_epilogue), _P(cv_operand), c_void_p, c_void_p,
         c_void_p, c_size_t, _P(cv_wgrad_defer), c_void_p],
    ),
    "cv_conv_backward_deferred_kpack": (
        c_int,
        [_P(cv_conv), _P(cv_operand), c_void_p, c_void_p, c_void_p, _P(cv_epilogue), _P(cv_operand), c_void_p,
         c_void_p, c_void_p, c_size_t, _P(cv_wgrad_defer), c_void_p],
    ),
    "cv_conv_backward_deferred_kpack_side": (
        c_int,
        [_P(cv_conv), _P(cv_operand), c_void_p, c_void_p, c_void_p, _P(cv_epilogue), _P(cv_operand), c_void_p,
         c_void_p, c_void_p, c_size_t, _P(cv_wgrad_defer), c_void_p, c_void_p],
    ),
    "cv_linear_backward_weight_deferred": (
        c_int,
        [_P(cv_linear), _P(cv_operand), _P(cv_operand), c_void_p, c_void_p, c_void_p, c_size_t, _P(cv_wgrad_defer),
         c_void_p],
    ),
    "cv_step_reduce": (
        c_int,
        [_P(cv_wgrad_defer), c_int, _P(cv_bn), c_int, _P(c_void_p), _P(c_void_p), c_int, c_float, _P(c_void_p),
         c_void_p],
    ),
    "cv_step_reduce_adam": (
        c_int,
        [_P(cv_wgrad_defer), c_int, _P(cv_bn), c_int, _P(c_void_p), _P(c_void_p), c_int, c_float, _P(c_void_p),
         c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cv_conv_wgrad_workspace_bytes": (c_size_t, [_P(cv_conv), c_int]),
    "cv_linear_wgrad_workspace_bytes": (c_size_t, [_P(cv_linear), c_int]),
    "cv_linear_forward": (
        c_int,
        [_P(cv_linear), _P(cv_operand), c_void_p, c_void_p, c_void_p, c_int, _P(cv_epilogue), c_void_p],
    ),
    "cv_linear_backward_data": (
        c_int,
        [_P(cv_linear), _P(cv_operand), c_void_p, c_void_p, c_int, _P(cv_epilogue), c_void_p],
    ),
    "cv_linear_backward_weight": (
        c_int,
        [_P(cv_linear), _P(cv_operand), _P(cv_operand), c_void_p, c_void_p, c_int, c_void_p, c_size_t, c_void_p],
    ),
    "cv_declinear_backward_weight": (
        c_int,
        [_P(cv_linear), c_void_p, c_void_p, _P(cv_bn), c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cv_decoder_input_supported": (c_int, [c_int, c_int, c_int]),
    "cv_decoder_input_forward": (
        c_int,
        [_P(cv_linear), c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, _P(cv_bn), c_void_p,
         c_void_p, c_void_p, c_void_p],
    ),
    "cv_decoder_input_backward": (
        c_int,
        [_P(cv_linear), c_void_p, c_void_p, _P(cv_bn), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cv_heads_forward_supported": (c_int, [c_int, c_int, c_int, c_int]),
    "cv_heads_forward": (
        c_int,
        [_P(cv_linear), c_void_p, _P(cv_bn), c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p,
         c_void_p],
    ),
    "cv_heads_backward_supported": (c_int, [c_int, c_int, c_int, c_int]),
    "cv_heads_backward": (
        c_int,
        [_P(cv_linear), c_void_p, c_void_p, c_void_p, _P(cv_bn), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cv_heads_backward_chain": (
        c_int,
        [_P(cv_linear), c_void_p, _P(cv_latent_chain), c_void_p, c_void_p, _P(cv_bn), c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p],
    ),
    "cv_bn_apply": (c_int, [_P(cv_bn), c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "cv_bn_update_running": (c_int, [_P(cv_bn), c_int, c_float, _P(c_void_p), c_void_p]),
    "cv_bn_update_running_sets": (c_int, [_P(cv_bn), c_int, c_int, c_float, _P(c_void_p), c_void_p]),
    "cv_bn_batch_stats": (c_int, [_P(cv_bn), c_void_p, c_void_p, c_void_p]),
    "cv_output_forward": (c_int, [_P(cv_bn), c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "cv_output_loss": (
        c_int,
        [_P(cv_bn), c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p],
    ),
    "cv_convt_output_loss": (
        c_int,
        [_P(cv_conv), _P(cv_operand), c_void_p, c_void_p, c_void_p, _P(cv_epilogue), _P(cv_bn), c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cv_output_backward": (
        c_int,
        [_P(cv_bn), c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    ),
    "cv_reparam_forward": (
        c_int,
        [c_void_p, c_int, c_int, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cv_sample_forward": (c_int, [c_void_p, c_void_p, ctypes.c_long, c_void_p, c_uint64, c_void_p, c_void_p,
                                  c_void_p]),
    "cv_sample_backward": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_long, c_void_p, c_void_p, c_int,
                                   c_void_p]),
    "cv_kl": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    ),
    "cv_latent_combine": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p],
    ),
    "cv_ntxent_aux": (
        c_int,
        [_P(cv_ntxent_branch), c_int, c_void_p, c_int, c_int, c_int, c_float, c_int, c_int, c_void_p],
    ),
    "cv_ntxent_aux_flush": (c_int, [c_void_p]),
    "cv_ntxent_aux_discard": (c_int, []),
    "cv_debug_wgrad_self": (c_int, [c_int]),
    "cv_latent_combine_workspace_bytes": (c_size_t, []),
    "cv_latent_combine_dz_workspace_bytes": (c_size_t, [c_int, c_int]),
    "cv_latent_combine_dz": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, _P(cv_linear), c_float, c_float, c_float, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    ),
    "cv_ntxent_aux_pending": (c_int, []),
    "cv_ntxent_aux_combine": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cv_latent_combine_acc": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p],
    ),
    "cv_mse_sum": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "cv_ntxent": (
        c_int,
        [_P(cv_ntxent_branch), c_int, c_void_p, c_int, c_int, c_int, c_float, c_int, c_int, c_void_p],
    ),
    "cv_latent_step": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p,
         c_void_p, _P(cv_ntxent_branch), c_int, c_void_p, c_int, c_float, c_void_p],
    ),
    "cv_tc_workspace_bytes": (c_size_t, [c_int]),
    "cv_tc_forward": (
        c_int,
        [_P(cv_tc_disc), c_void_p, c_int, c_float, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p],
    ),
    "cv_tc_learning_step": (c_int, [_P(cv_tc_disc), c_void_p, c_int, c_void_p, c_void_p, _P(cv_tc_grad), c_void_p]),
    "cv_group_workspace_bytes": (c_size_t, [c_int, c_int]),
    "cv_group_forward": (
        c_int,
        [c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
         c_void_p, c_int, c_uint64, c_void_p, c_void_p, c_void_p],
    ),
    "cv_group_backward": (
        c_int,
        [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_float, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p],
    ),
    "cv_group_evidence_backward": (
        c_int,
        [c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
         c_void_p],
    ),
    "cv_resize_plan_words": (c_size_t, [c_int, c_int, c_int, c_int]),
    "cv_resize_plan": (c_int, [c_int, c_int, c_int, c_int, c_void_p, c_size_t]),
    "cv_resize_tile_rows": (c_int, [c_void_p, c_int]),
    "cv_load_batch_u8": (
        c_int,
        [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cv_mi_workspace_bytes": (c_size_t, [c_int]),
    "cv_mi_forward": (
        c_int,
        [c_int, _P(cv_mlp), c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_uint64, c_void_p, c_void_p,
         c_void_p, c_void_p],
    ),
    "cv_mi_backward": (
        c_int,
        [c_int, _P(cv_mlp), c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p,
         c_void_p, c_int, c_int, _P(cv_mlp_grad), c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    ),
    "cv_mi_learning_step": (
        c_int,
        [_P(cv_mlp), c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, _P(cv_mlp_grad), c_void_p,
         c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p],
    ),
    "cv_adam_step": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cv_bn_param_grads": (c_int, [_P(cv_bn), c_int, _P(c_void_p), _P(c_void_p), c_void_p]),
    "cv_zero": (c_int, [c_void_p, c_size_t, c_void_p]),
    "cv_graph_begin": (c_int, [c_void_p]),
    "cv_graph_end": (c_int, [c_void_p, POINTER(c_void_p)]),
    "cv_graph_launch": (c_int, [c_void_p, c_void_p]),
    "cv_graph_destroy": (c_int, [c_void_p]),
    "cv_zero_many": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "cv_copy_many": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "cv_last_error": (ctypes.c_char_p, []),
    "cv_version": (c_int, []),
    "cv_debug_force_generic_gemm": (c_int, [c_int]),
    "cv_debug_direct_count": (c_int, [c_int]),
    "cv_debug_direct_minwg": (c_int, [c_int]),
    "cv_debug_direct_gather_rule": (c_int, [c_int]),
    "cv_debug_dual": (c_int, [c_int]),
    "cv_debug_pm": (c_int, [c_int]),
    "cv_debug_aux": (c_int, [c_int]),
    "cv_debug_aux_count": (c_int, [c_int]),
    "cv_debug_nt_reg": (c_int, [c_int]),
    "cv_debug_pm_count": (c_int, [c_int]),
    "cv_debug_dual_count": (c_int, [c_int]),
    "cv_debug_kernel_log": (c_int, [c_int]),
    "cv_debug_kernel_names": (c_int, [ctypes.c_char_p, c_size_t]),
    "cv_gemm_workspace_bytes": (c_size_t, []),
    "cv_set_gemm_workspace": (c_int, [c_void_p, c_size_t]),
}

EXPORTED = tuple(_SIGS)

_LIB = None


class HipLibraryError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load the shared object and declare every prototype (no GPU needed)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise HipLibraryError(
            f"libclearvae_hip.so not found at {path}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)"
        )
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def lib():
    return load()


def check(rc: int, what: str):
    if rc != 0:
        msg = _LIB.cv_last_error().decode() if _LIB is not None else "?"
        raise RuntimeError(f"{what}: {msg}")


def call(name: str, *args):
    rc = getattr(lib(), name)(*args)
    check(rc, name)


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


_GEMM_WS: dict = {}


def ensure_gemm_workspace(device) -> None:
    """Register the device's GEMM workspace with the library once (cv_set_gemm_workspace: the in-launch
    split-K of under-filled long-K convolutions); a zeroed torch buffer kept alive for the process."""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx in _GEMM_WS:
        return
    nbytes = int(lib().cv_gemm_workspace_bytes())
    buf = torch.zeros((nbytes + 15) // 16 * 4, dtype=torch.float32, device=torch.device("cuda", idx))
    with torch.cuda.device(idx):
        call("cv_set_gemm_workspace", buf.data_ptr(), buf.numel() * 4)
    _GEMM_WS[idx] = buf


def gemm_workspace(device) -> torch.Tensor:
    """The device's registered GEMM workspace (ensure_gemm_workspace)."""
    ensure_gemm_workspace(device)
    device = torch.device(device)
    return _GEMM_WS[device.index if device.index is not None else torch.cuda.current_device()]


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


class StepGraph:
    """An executable HIP graph of library calls, launched without PyTorch's CUDAGraph.replay() (which
    refreshes the framework's RNG state with two host-to-device copies before every launch)."""

    def __init__(self, record):
        """record(stream_handle) enqueues the calls; captured on a private stream."""
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        exe = c_void_p()
        with torch.cuda.stream(side):
            s = side.cuda_stream
            call("cv_graph_begin", s)
            try:
                record(s)
            except BaseException:
                dummy = c_void_p()
                lib().cv_graph_end(s, ctypes.byref(dummy))
                if dummy.value:
                    lib().cv_graph_destroy(dummy)
                raise
            call("cv_graph_end", s, ctypes.byref(exe))
        cur.wait_stream(side)
        self.exec = exe

    def replay(self, stream=None):
        call("cv_graph_launch", self.exec, stream_handle() if stream is None else stream)

    def __del__(self):
        try:
            if self.exec and self.exec.value:
                lib().cv_graph_destroy(self.exec)
                self.exec = None
        except Exception:  # interpreter shutdown
            pass

