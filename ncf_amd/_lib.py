"""ctypes bindings of the two in-tree native libraries.

* ``libncf_hip.so``     -- HIP kernels + C ABI, declared in ``include/ncf_hip.h``
* ``libncf_sampler.so`` -- host C++ negative sampler, ``include/ncf_sampler.h``

There is no fallback: if a library is missing or a call returns an error code,
this module raises.  ``torch`` is imported first so that the HIP runtime torch
ships (SONAME ``libamdhip64.so.7``) is the one ``libncf_hip.so`` binds to, and
streams/pointers from torch are valid in our launches.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede loading libncf_hip.so)

_HERE = os.path.dirname(os.path.abspath(__file__))
# NCF_HIP_LIB=<variant> selects ncf_amd/libncf_hip_<variant>.so (diag = phase stamps
# compiled in; other variants are experiment builds of the Makefile's `variant` target)
_VARIANT = os.environ.get("NCF_HIP_LIB", "")
HIP_LIB_PATH = os.path.join(_HERE, f"libncf_hip_{_VARIANT}.so" if _VARIANT else "libncf_hip.so")
SAMPLER_LIB_PATH = os.path.join(_HERE, "libncf_sampler.so")

NCF_OK = 0
NCF_E_UNSUPPORTED = -1
NCF_E_ARG = -2
NCF_E_LAUNCH = -3
MODEL_GMF, MODEL_MLP, MODEL_NEUMF = 0, 1, 2
DZ_BCE, DZ_DLOGIT, DZ_KD = 0, 1, 2
ABI_VERSION = 19  # include/ncf_hip.h NCF_ABI_VERSION
PATH_FUSED, PATH_LAYERED = 1, 2  # ncf_supported()
LAYOUT_PER_ROW_L0, LAYOUT_WG_SHIFT, LAYOUT_WG_MASK = 0x1, 8, 0xFFF  # ncf_layout.flags (ncf_layout_tune)
LAYOUT_LAYERED = 0x2  # ncf_layout.flags: training on the layered path even where a fused kernel exists
LAYOUT_GEO_SHIFT, LAYOUT_GEO_MASK = 20, 0x3  # ncf_layout.flags: fused-step geometry (0..3: 8, 4, 2, 1 waves)
PREP_CANONICAL = 0x1  # ncf_prepare_epoch2 flags: canonical row order inside item runs (data parallel)
PROBE_BLOCKS = 2048  # include/ncf_hip.h NCF_PROBE_BLOCKS (ncf_probe_gather_scatter's sink: x 256 floats)
LAYOUT_FACT_DEFER_DX = 0x8  # ncf_layout.flags: factored step leaves G for ncf_adam_step_fact (sharded zero1)
LAYOUT_USER_STORE = 0x10  # ncf_layout.flags (ncf_layout_tune): user-side gradients stored, summed per user
MODEL_CODES = {"GMF": MODEL_GMF, "MLP": MODEL_MLP, "NeuMF-end": MODEL_NEUMF, "NeuMF-pre": MODEL_NEUMF}

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_vp = ctypes.c_void_p


class NcfLayout(ctypes.Structure):
    _fields_ = [("ug", c_i64), ("ig", c_i64), ("um", c_i64), ("im", c_i64),
                ("w", c_i64 * 4), ("b", c_i64 * 4), ("wp", c_i64), ("bp", c_i64),
                ("tower_begin", c_i64), ("tower_len", c_i64), ("total", c_i64),
                ("user_num", c_i32), ("item_num", c_i32), ("factor_num", c_i32),
                ("num_layers", c_i32), ("model_type", c_i32), ("flags", c_i32),
                ("dropout", ctypes.c_float), ("dropout_seed", ctypes.c_uint32)]

    @property
    def loss_slot(self) -> int:
        return int(self.tower_begin + self.tower_len)


class NcfStepCtl(ctypes.Structure):
    _fields_ = [("batch", c_i64), ("adam_t", c_i64), ("n_total", c_i64), ("reserved", c_i64),
                ("snap_batch", c_i64), ("snap_t", c_i64)]


class NcfOwnerPlan(ctypes.Structure):
    """include/ncf_hip.h ncf_owner_plan (dp_mode "owner", ABI 17)."""
    _fields_ = [("world", c_i32), ("rank", c_i32), ("max_u", c_i32), ("max_i", c_i32),
                ("n_total", c_i64), ("batch_global", c_i64), ("nb", c_i64),
                ("row_u", c_i32), ("row_i", c_i32), ("chunk_u", c_i32), ("chunk_i", c_i32),
                ("nchunk_u", c_i64), ("nchunk_i", c_i64), ("record_ints", c_i64), ("lists_bytes", c_i64),
                ("send_floats", c_i64), ("param_floats", c_i64), ("tail_offset", c_i64), ("off", c_i64 * 4)]


class NcfAisBufs(ctypes.Structure):
    """include/ncf_hip.h ncf_ais_bufs (in-step Adam, ABI 18)."""
    _fields_ = [("params_b", c_vp), ("exp_avg_b", c_vp), ("exp_avg_sq_b", c_vp), ("grads_1", c_vp),
                ("grads_2", c_vp), ("state", c_vp)]


_OWNER = ctypes.POINTER(NcfOwnerPlan)
_AIS = ctypes.POINTER(NcfAisBufs)
_LAY = ctypes.POINTER(NcfLayout)
_HIP_PROTOS = {
    "ncf_abi_version": (ctypes.c_int, []),
    "ncf_supported": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "ncf_layout_init": (ctypes.c_int, [ctypes.c_int] * 5 + [ctypes.POINTER(NcfLayout)]),
    "ncf_slab_rows": (ctypes.c_int, []),
    "ncf_layout_tune": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_i64]),
    "ncf_train_step": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_i64, c_vp, c_vp]),
    "ncf_train_step_kd": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                         c_i64, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                         ctypes.c_float, c_vp, c_i64, c_vp, c_vp]),
    "ncf_kd_feature_step": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, ctypes.POINTER(NcfLayout), c_vp,
                                           c_vp, c_vp, c_i64, ctypes.c_int, ctypes.c_int,
                                           c_vp, c_vp, ctypes.c_float, c_vp, c_vp, ctypes.c_float, c_vp, c_vp]),
    "ncf_forward": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "ncf_workspace_bytes": (c_i64, [ctypes.POINTER(NcfLayout), c_i64]),
    "ncf_forward_workspace_bytes": (c_i64, [ctypes.POINTER(NcfLayout), c_i64]),
    "ncf_pack_rows": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "ncf_zero_f32": (ctypes.c_int, [c_vp, c_i64, c_vp]),
    "ncf_expand_grads": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_vp, c_vp]),
    "ncf_reduce_slab": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_vp, c_vp]),
    "ncf_slab_stride": (c_i64, [ctypes.POINTER(NcfLayout)]),
    "ncf_debug_set_diag": (ctypes.c_int, [ctypes.c_int]),
    "ncf_debug_set_user_store": (ctypes.c_int, [ctypes.c_int]),
    "ncf_debug_set_per_row": (ctypes.c_int, [ctypes.c_int]),
    "ncf_debug_set_geometry": (ctypes.c_int, [ctypes.c_int]),
    "ncf_probe_gather_scatter": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_vp, c_vp, c_i64,
                                                ctypes.c_int, c_vp]),
    "ncf_debug_set_stamps": (ctypes.c_int, [c_vp]),
    "ncf_adam_step": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(c_i64), ctypes.c_int, c_vp,
                                     ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                     c_i64, c_vp, c_i64, c_vp]),
    "ncf_adam_step_fact": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_vp, c_vp, c_vp,
                                          ctypes.POINTER(c_i64), ctypes.c_int, c_i64, c_vp, c_i64, c_vp, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_double, ctypes.c_double, c_i64, c_vp, c_i64,
                                          c_vp]),
    "ncf_reduce_adam_step": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_vp, c_vp, c_vp,
                                            ctypes.POINTER(c_i64), ctypes.c_int, c_vp, ctypes.c_double,
                                            ctypes.c_double, ctypes.c_double, ctypes.c_double, c_vp, c_i64, c_vp]),
    "ncf_sgd_step": (ctypes.c_int, [c_vp, c_vp, ctypes.POINTER(c_i64), ctypes.c_int, c_vp, ctypes.c_double,
                                    c_i64, c_vp, c_i64, c_vp]),
    "ncf_gather_epoch": (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "ncf_prepare_epoch_workspace": (c_i64, [c_i64, c_i64, ctypes.c_int]),
    "ncf_prepare_epoch": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, ctypes.c_int, c_vp, c_vp, c_i64, c_vp]),
    "ncf_prepare_epoch2": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_i64,
                                          c_vp]),
    "ncf_hr_ndcg": (ctypes.c_int, [c_vp, c_vp, c_i64, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp]),
    "ncf_fact_mode": (ctypes.c_int, [c_vp]),
    "ncf_reduce_rows": (ctypes.c_int, [c_vp]),
    "ncf_dropout_hash": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, c_i64,
                                           ctypes.c_uint32]),
    "ncf_fact_partials_bytes": (c_i64, [c_vp]),
    "ncf_randperm_workspace": (c_i64, [c_i64]),
    "ncf_randperm": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "ncf_build_rows": (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, ctypes.c_int, c_vp, c_vp]),
    "ncf_user_order": (ctypes.c_int, [c_vp, c_i64, c_i64, ctypes.c_int, ctypes.c_int, c_vp, c_vp]),
    "ncf_uses_user_order": (ctypes.c_int, [c_vp]),
    "ncf_touched_bytes": (c_i64, [c_i64, c_i64, ctypes.c_int, ctypes.c_int]),
    "ncf_batch_touched": (ctypes.c_int, [c_vp, c_i64, c_i64, ctypes.c_int, ctypes.c_int, c_vp, c_vp]),
    "ncf_lazy_adam_step": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_vp, c_vp, c_vp,
                                          ctypes.POINTER(c_i64), ctypes.c_int, c_vp,
                                          ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                          c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "ncf_touched_packed_floats": (c_i64, [ctypes.POINTER(NcfLayout), ctypes.POINTER(c_i64), ctypes.c_int, c_i64]),
    "ncf_touched_pack": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, ctypes.POINTER(c_i64), ctypes.c_int,
                                        c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "ncf_lazy_adam_step_packed": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_vp, ctypes.POINTER(c_i64),
                                                 ctypes.c_int, c_vp, ctypes.c_double, ctypes.c_double,
                                                 ctypes.c_double, ctypes.c_double, c_vp, c_i64, c_vp, c_i64, c_i64,
                                                 c_vp, c_vp, c_i64, c_vp, c_vp]),
    "ncf_lazy_adam_flush": (ctypes.c_int, [ctypes.POINTER(NcfLayout), c_vp, c_vp, c_vp, c_vp,
                                           ctypes.POINTER(c_i64), ctypes.c_int, c_vp,
                                           ctypes.c_double, ctypes.c_double, ctypes.c_double, c_vp, c_vp, c_i64,
                                           c_vp]),
    "ncf_owner_plan_init": (ctypes.c_int, [_LAY, ctypes.POINTER(c_i64), ctypes.c_int, c_i64, c_i64, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int, _OWNER]),
    "ncf_owner_lists": (ctypes.c_int, [_OWNER, _LAY, c_vp, c_vp, c_vp, c_vp]),
    "ncf_owner_pack": (ctypes.c_int, [_OWNER, _LAY, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "ncf_owner_adam": (ctypes.c_int, [_OWNER, _LAY, c_vp, c_vp, c_vp, ctypes.POINTER(c_i64), ctypes.c_int, c_vp, c_vp,
                                      ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, c_vp, c_i64,
                                      c_vp, c_vp, c_vp]),
    "ncf_owner_unpack": (ctypes.c_int, [_OWNER, _LAY, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "ncf_ais_supported": (ctypes.c_int, [_LAY]),
    "ncf_ais_begin": (ctypes.c_int, [_LAY, c_vp, c_vp, c_vp, c_vp, _AIS, ctypes.POINTER(c_i64), ctypes.c_int, c_vp,
                                     c_vp]),
    "ncf_train_step_ais": (ctypes.c_int, [_LAY, c_vp, c_vp, c_vp, c_vp, _AIS, ctypes.POINTER(c_i64), ctypes.c_int,
                                          c_vp, c_vp, c_vp, c_i64, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                          ctypes.c_double, c_vp, c_i64, c_i64, c_vp]),
    "ncf_ais_bump": (ctypes.c_int, [c_vp, _AIS, c_i64, c_vp]),
    "ncf_ais_flush": (ctypes.c_int, [_LAY, c_vp, c_vp, c_vp, c_vp, _AIS, ctypes.POINTER(c_i64), ctypes.c_int, c_vp,
                                     ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, c_vp, c_i64,
                                     c_vp]),
}

_SAMPLER_PROTOS = {
    "ncf_sampler_create": (c_vp, [c_vp, c_vp, c_i64, c_i32, c_i32]),
    "ncf_sampler_destroy": (None, [c_vp]),
    "ncf_sampler_contains": (ctypes.c_int, [c_vp, c_i32, c_i32]),
    "ncf_mt_seed": (None, [ctypes.c_uint32, c_vp, c_vp]),
    "ncf_sampler_sample": (c_i64, [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp]),
    "ncf_mt_words": (None, [c_vp, c_vp, c_i64, c_vp]),
    "ncf_sampler_create2": (c_vp, [c_vp, c_i64, c_vp, c_vp, c_i64, c_i32, c_i32]),
    "ncf_sampler_set_threads": (ctypes.c_int, [c_vp, c_i32]),
    "ncf_sampler_stats": (ctypes.c_int, [c_vp, c_vp, c_i32]),
    "ncf_mt_jump": (ctypes.c_int, [c_vp, c_i64]),
    "ncf_words_create": (c_vp, [c_i32]),
    "ncf_words_destroy": (None, [c_vp]),
    "ncf_words_fill": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp]),
}

_lock = threading.Lock()
_hip = None
_sampler = None


def _load(path, protos, what):
    if not os.path.exists(path):
        raise RuntimeError(
            f"{what} not found at {path}: build it with `make -C ncf_amd/csrc` "
            "(or `python -c 'import __graft_entry__ as g; g.build()'`). There is no fallback path.")
    lib = ctypes.CDLL(path)
    for name, (res, args) in protos.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def hip():
    """The loaded libncf_hip.so (raises if it is missing)."""
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                lib = _load(HIP_LIB_PATH, _HIP_PROTOS, "libncf_hip.so")
                if lib.ncf_abi_version() != ABI_VERSION:
                    raise RuntimeError("libncf_hip.so ABI mismatch; rebuild")
                _hip = lib
    return _hip


def sampler_lib():
    global _sampler
    if _sampler is None:
        with _lock:
            if _sampler is None:
                _sampler = _load(SAMPLER_LIB_PATH, _SAMPLER_PROTOS, "libncf_sampler.so")
    return _sampler


def check(code: int, what: str):
    if code != NCF_OK:
        names = {NCF_E_UNSUPPORTED: "unsupported shape", NCF_E_ARG: "bad argument", NCF_E_LAUNCH: "HIP launch failed"}
        raise RuntimeError(f"{what}: {names.get(code, 'error')} (code {code})")


def layout(user_num: int, item_num: int, factor_num: int, num_layers: int, model_type) -> NcfLayout:
    mode = MODEL_CODES[model_type] if isinstance(model_type, str) else int(model_type)
    lay = NcfLayout()
    check(hip().ncf_layout_init(int(user_num), int(item_num), int(factor_num), int(num_layers), mode,
                                ctypes.byref(lay)), "ncf_layout_init")
    return lay


def supported(model_type, factor_num: int, num_layers: int) -> int:
    """PATH_FUSED, PATH_LAYERED, or 0 for an invalid shape (ncf_supported)."""
    mode = MODEL_CODES[model_type] if isinstance(model_type, str) else int(model_type)
    return int(hip().ncf_supported(mode, int(factor_num), int(num_layers)))


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()
