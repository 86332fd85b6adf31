"""ctypes bindings of the native libraries (``_native/*.so``).

The HIP path fails LOUDLY when its library is missing or stale: on a GPU box
``kernels()`` raises instead of silently falling back to PyTorch/MIOpen.
Building happens in-tree (``python -m imagent_amd.build`` or
``__graft_entry__.build()``); ``IMAGENT_AUTOBUILD=1`` builds on first use.
"""

from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (must be imported first: our libs bind to torch's HIP/RCCL)

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_NATIVE = os.path.join(_PKG, "_native")
_lock = threading.Lock()
_libs = {}


class NativeLibraryMissing(RuntimeError):
    pass


def _path(name: str) -> str:
    if name == "kernels" and os.environ.get("IMAGENT_KERNELS_LIB"):  # A/B builds (build.build_kernels_variant)
        return os.environ["IMAGENT_KERNELS_LIB"]
    return os.path.join(_NATIVE, f"libimagent_{name}.so")


def _load(name: str):
    with _lock:
        if name in _libs:
            return _libs[name]
        p = _path(name)
        if not os.path.exists(p) and os.environ.get("IMAGENT_AUTOBUILD", "0") == "1":
            from .. import build
            build.build_all(verbose=False)
        if not os.path.exists(p):
            raise NativeLibraryMissing(
                f"{p} not found - build it with `python -m imagent_amd.build` "
                "(the HIP path never falls back to PyTorch kernels silently)")
        lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
        _declare(name, lib)
        _libs[name] = lib
        return lib


def kernels():
    return _load("kernels")


def comm():
    return _load("comm")


def runtime():
    return _load("runtime")


def available(name: str = "kernels") -> bool:
    return os.path.exists(_path(name))


def loaded_paths():
    return {k: _path(k) for k in _libs}


# --------------------------------------------------------------------------
# argument structs (mirror csrc/kernels/*.hip)
# --------------------------------------------------------------------------

class IGemmArgs(C.Structure):
    _fields_ = [
        ("X", C.c_void_p), ("Wk", C.c_void_p), ("Y", C.c_void_p), ("bias", C.c_void_p),
        ("stats", C.c_void_p),
        ("N", C.c_int), ("H", C.c_int), ("W", C.c_int), ("C", C.c_int),
        ("OH", C.c_int), ("OW", C.c_int), ("M", C.c_int),
        ("Nout", C.c_int), ("ldb", C.c_int),
        ("sA", C.c_int),
        ("nth", C.c_int), ("ntw", C.c_int), ("dh0", C.c_int), ("dhs", C.c_int), ("dw0", C.c_int),
        ("dws", C.c_int), ("kh0", C.c_int), ("khs", C.c_int), ("kw0", C.c_int), ("kws", C.c_int),
        ("KW", C.c_int),
        ("YH", C.c_int), ("YW", C.c_int), ("sY", C.c_int), ("oy", C.c_int), ("ox", C.c_int),
        ("ldy", C.c_int),
        ("flags", C.c_int),
        ("bnx", C.c_void_p), ("bnym", C.c_void_p), ("bnsave", C.c_void_p), ("bngamma", C.c_void_p),
        ("bnbeta", C.c_void_p), ("bnx2", C.c_void_p), ("bnsave2", C.c_void_p),
        ("xexp", C.c_void_p), ("wexp", C.c_void_p), ("shift", C.c_void_p),
        ("xbn", C.c_void_p),
        ("X2", C.c_void_p), ("C2", C.c_int),
        ("Y8", C.c_void_p), ("y8exp", C.c_void_p), ("y8amax", C.c_void_p),
    ]


class LarsDesc(C.Structure):
    """optim.hip LarsDesc: one parameter tensor of the flat arena."""
    _fields_ = [("p", C.c_void_p), ("g", C.c_void_p), ("buf", C.c_void_p), ("shadow", C.c_void_p),
                ("n", C.c_long), ("adapt", C.c_int), ("pad", C.c_int)]


class QDesc(C.Structure):
    """fp8.hip QDesc: one weight tensor of the per-step e4m3 quantisation."""
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("n4", C.c_long), ("exp", C.c_void_p),
                ("amax", C.c_void_p), ("dstT", C.c_void_p), ("T", C.c_int), ("Ci", C.c_int)]


class WgradArgs(C.Structure):
    _fields_ = [
        ("dY", C.c_void_p), ("X", C.c_void_p), ("dW", C.c_void_p),
        ("N", C.c_int), ("H", C.c_int), ("W", C.c_int), ("Ci", C.c_int), ("Co", C.c_int),
        ("OH", C.c_int), ("OW", C.c_int), ("M", C.c_int),
        ("KH", C.c_int), ("KW", C.c_int), ("stride", C.c_int), ("pad", C.c_int),
        ("m_per_split", C.c_int),
        ("mg_ohw", C.c_uint32), ("sh_ohw", C.c_uint32), ("mg_ow", C.c_uint32), ("sh_ow", C.c_uint32),
        ("stem", C.c_int), ("xbn", C.c_void_p),
    ]


class RunDesc(C.Structure):
    _fields_ = [
        ("sums", C.c_void_p), ("rmean", C.c_void_p), ("rvar", C.c_void_p), ("nbt", C.c_void_p),
        ("C", C.c_int), ("inv_cnt", C.c_float), ("unbias", C.c_float), ("momentum", C.c_float),
    ]


class AffDesc(C.Structure):
    _fields_ = [
        ("gamma", C.c_void_p), ("beta", C.c_void_p), ("rmean", C.c_void_p), ("rvar", C.c_void_p),
        ("out", C.c_void_p), ("C", C.c_int), ("eps", C.c_float),
    ]


class TDesc(C.Structure):
    _fields_ = [
        ("src", C.c_void_p), ("dst", C.c_void_p),
        ("Co", C.c_int), ("T", C.c_int), ("Ci", C.c_int), ("tile0", C.c_int),
    ]


def _declare(name: str, lib) -> None:
    vp, i32, i64, f32 = C.c_void_p, C.c_int, C.c_long, C.c_float
    if name == "kernels":
        sigs = {
            "imk_conv_igemm": [C.POINTER(IGemmArgs), i32, vp],
            "imk_conv_wgrad": [C.POINTER(WgradArgs), i32, vp],
            "imk_conv_wgrad_variant": [C.POINTER(WgradArgs), i32, i32, vp],
            "imk_conv_launches": [],
            # fp32 path (f32.hip)
            "imk_conv_f32": [C.POINTER(IGemmArgs), vp],
            "imk_set_f32_split": [i32],
            "imk_wgrad_f32": [vp, vp, vp] + [i32] * 11 + [vp],
            "imk_bn_slab_floats_f32": [i32],
            "imk_bn_stats_f32": [vp, vp, vp, vp, vp, vp, i64, i32, f32, f32, vp],
            "imk_bn_fold_slab_f32": [vp, vp, vp, vp, vp, i64, i32, f32, f32, vp],
            "imk_bn_bwd_slab_f32": [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, vp],
            "imk_bn_apply_f32": [vp, vp, vp, vp, vp, vp, i64, i32, i32, vp],
            "imk_bn_bwd_f32": [vp] * 11 + [i64, i32, vp],
            "imk_maxpool_f32": [vp, vp, vp] + [i32] * 9 + [vp],
            "imk_maxpool_bwd_f32": [vp, vp, vp] + [i32] * 9 + [vp],
            "imk_avgpool_f32": [vp, vp, i32, i32, i32, vp],
            "imk_avgpool_bwd_f32": [vp, vp, i32, i32, i32, vp],
            "imk_colsum_f32": [vp, vp, i32, i32, vp],
            "imk_normalize_u8_f32": [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp],
            "imk_xent_bwd_f32": [vp, vp, vp, vp, vp, i32, i32, f32, vp],
            "imk_bn_fwd": [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, f32, i32, vp, vp, vp,
                           vp, vp, vp, vp, vp, i32, vp],
            "imk_bn_bwd": [vp] * 17 + [i64, i32, i32, i32, vp],
            "imk_bn_bwd_apply": [vp] * 14 + [i64, i32, i32, vp, i32, i32, vp],
            "imk_bn_running_update": [vp, i32, vp],
            "imk_bn_eval_affine": [vp, i32, vp],
            "imk_set_deterministic": [i32],
            "imk_bn_stats_det": [vp, vp, vp, vp, i64, i32, vp],
            "imk_bn_stats_finalize": [vp, vp, vp, i32, i32, i64, vp],
            "imk_bn_finalize_affine": [vp, vp, vp, vp, vp, vp, i32, i32, i64, f32, i32, vp],
            "imk_maxpool_fwd": [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp],
            "imk_maxpool_bwd": [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp],
            "imk_maxpool_fwd_bn": [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32,
                                   C.c_float, vp],
            "imk_maxpool_bwd_bnr": [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32,
                                    vp],
            "imk_avgpool_fwd": [vp, vp, i32, i32, i32, vp],
            "imk_avgpool_bwd": [vp, vp, i32, i32, i32, vp],
            "imk_xent_fwd": [vp, vp, vp, vp, vp, i32, i32, f32, vp],
            "imk_xent_bwd": [vp, vp, vp, vp, vp, i32, i32, f32, vp],
            "imk_colsum_bf16": [vp, vp, i32, i32, vp],
            "imk_stem_grad_fold": [vp, vp, i32, i32, i32, i32, vp],
            "imk_memset0": [vp, i64, vp],
            "imk_stem_pad": [vp, vp, i32, i32, i32, i32, vp],
            "imk_bn_bwd_coef_T": [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, vp],
            "imk_bn_gram_fwd_stats": [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, f32, vp],
            "imk_bn_bwd_coef": [vp, vp, vp, vp, vp, vp, i64, i32, vp],
            "imk_bn_gram_dgrad_weights": [vp, i32, vp, vp, vp, vp, i32, i32, vp],
            "imk_bn_gram_q": [vp, i32, vp, vp, i32, i32, vp],
            "imk_stem_wgrad_bnx": [C.POINTER(WgradArgs), vp, vp, vp],
            "imk_gram_sym": [vp, vp, i64, i32, i32, vp],
            "imk_bn_gram_wgrad_fixup": [vp, vp, vp, vp, vp, vp, i32, i32, vp],
            "imk_bn_gram_p": [vp, vp, vp, vp, i64, i32, i32, vp],
            "imk_sgd": [vp, vp, vp, vp, i64, f32, f32, f32, f32, i32, i32, f32, vp],
            "imk_cast_bf16": [vp, vp, i64, vp],
            "imk_uncast_bf16": [vp, vp, i64, vp],
            "imk_normalize_u8": [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp],
            "imk_resize_normalize_u8": [vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp],
            "imk_transpose_batched": [vp, i32, i32, vp],
            "imk_stream_create_cumask": [i32, C.POINTER(vp)],
            "imk_igemm_args_size": [], "imk_wgrad_args_size": [], "imk_bn_rundesc_size": [], "imk_bn_affdesc_size": [],
            "imk_tdesc_size": [], "imk_bn_bwd_scratch_floats": [i32],
            "imk_quant_fp8": [vp, vp, i64, vp, vp, vp],
            "imk_fp8_update_exp": [vp, vp, i32, i32, vp],
            "imk_quant_fp8_weights": [vp, i32, i64, i32, vp],
            "imk_qdesc_size": [], "imk_lars_desc_size": [],
            "imk_lars_step": [vp, i32, i64, vp, f32, f32, f32, f32, f32, i32, vp],
        }
        for fn, args in sigs.items():
            f = getattr(lib, fn)
            f.argtypes = args
            f.restype = C.c_int
        lib.imk_bn_stats_det_floats.argtypes = [i64, i32]
        lib.imk_bn_stats_det_floats.restype = C.c_long
        # ABI guard: the ctypes mirrors must match the compiled structs
        for fn, st in [("imk_igemm_args_size", IGemmArgs), ("imk_wgrad_args_size", WgradArgs),
                       ("imk_bn_rundesc_size", RunDesc), ("imk_bn_affdesc_size", AffDesc), ("imk_tdesc_size", TDesc),
                       ("imk_qdesc_size", QDesc), ("imk_lars_desc_size", LarsDesc)]:
            n = getattr(lib, fn)()
            if n != C.sizeof(st):
                raise RuntimeError(f"{fn}: native {n} B != ctypes {C.sizeof(st)} B - rebuild")
    elif name == "comm":
        lib.imc_last_error.restype = C.c_char_p
        lib.imc_unique_id_bytes.restype = i32
        lib.imc_get_unique_id.argtypes = [C.c_char_p]
        lib.imc_version.restype = i32
        lib.imc_comm_init.argtypes = [C.c_char_p, i32, i32, i32, i32, C.POINTER(vp)]
        lib.imc_comm_destroy.argtypes = [vp]
        lib.imc_comm_stream.argtypes = [vp]
        lib.imc_comm_stream.restype = vp
        lib.imc_stream_join_from.argtypes = [vp, vp]
        lib.imc_stream_join_into.argtypes = [vp, vp]
        lib.imc_allreduce.argtypes = [vp, vp, C.c_uint64, i32, i32, vp]
        lib.imc_allreduce_group.argtypes = [vp, i32, C.POINTER(vp), C.POINTER(C.c_uint64), i32, i32, vp]
        lib.imc_broadcast.argtypes = [vp, vp, C.c_uint64, i32, i32, vp]
        lib.imc_allgather.argtypes = [vp, vp, vp, C.c_uint64, i32, vp]
        lib.imc_reduce_scatter.argtypes = [vp, vp, vp, C.c_uint64, i32, i32, vp]
        lib.imc_synchronize.argtypes = [vp]
        lib.imc_async_error.argtypes = [vp]
        lib.imc_abort.argtypes = [vp]
        lib.imc_comm_init_start.argtypes = [C.c_char_p, i32, i32, i32, i32, i32, C.POINTER(vp)]
        lib.imc_comm_poll.argtypes = [vp]
        lib.imc_comm_nranks.argtypes = [vp]
        lib.imc_comm_set_stream_mode.argtypes = [vp, i32]
        lib.imc_stream_create.argtypes = [i32, i32, C.POINTER(vp)]
        lib.imc_stream_destroy.argtypes = [vp]
    elif name == "runtime":
        lib.imr_plan_buckets.argtypes = [i32, C.POINTER(C.c_int64), C.c_int64, C.c_int64, C.c_int64,
                                         C.POINTER(C.c_int32)]
        lib.imr_plan_buckets.restype = i32
        lib.imr_tracker_new.argtypes = [i32, C.POINTER(C.c_int32), i32]
        lib.imr_tracker_new.restype = vp
        lib.imr_tracker_free.argtypes = [vp]
        lib.imr_tracker_mark.argtypes = [vp, i32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.imr_tracker_mark.restype = i32
        lib.imr_tracker_finalize.argtypes = [vp, C.c_void_p]
        lib.imr_tracker_finalize.restype = i32
        lib.imr_tracker_last_order.argtypes = [vp, C.c_void_p]
        lib.imr_tracker_last_order.restype = i32
        lib.imr_tracker_iterations.argtypes = [vp]
        lib.imr_tracker_iterations.restype = C.c_int64
        # packed uint8 image records (csrc/runtime/records.cpp, data/records.py)
        lib.imr_records_header_bytes.restype = i32
        lib.imr_records_open.argtypes = [C.c_char_p, i32, i32]
        lib.imr_records_open.restype = vp
        lib.imr_records_close.argtypes = [vp]
        lib.imr_records_close.restype = None
        lib.imr_records_info.argtypes = [vp, vp]
        lib.imr_records_info.restype = None
        lib.imr_records_labels.argtypes = [vp, vp]
        lib.imr_records_labels.restype = None
        lib.imr_records_submit.argtypes = [vp, i32, vp, i32, vp, vp]
        lib.imr_records_submit.restype = i32
        lib.imr_records_wait.argtypes = [vp, i32]
        lib.imr_records_wait.restype = i32


STAT_SLOTS = 32  # conv epilogue statistics slab depth (csrc/kernels/conv_igemm.hip)


def ptr(t) -> int:
    """Device/host pointer of a tensor (None -> 0)."""
    return 0 if t is None else t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def zero_(t) -> None:
    """t.zero_() for a contiguous device tensor as one hipMemsetAsync on the current stream (no ATen fill launch in
    the training step); CPU / non-contiguous tensors: t.zero_()."""
    if t.is_cuda and t.is_contiguous() and available():
        check(kernels().imk_memset0(t.data_ptr(), t.numel() * t.element_size(), stream_ptr(t.device)), "memset")
    else:
        t.zero_()


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")
