"""ctypes binding of libvoxnav.so -- the C-ABI declared in include/voxnav.h.

There is no fallback: if the HIP library is missing or fails to load, every
entry point raises.  (The CPU restatement under oracle/ is test
infrastructure and is never used by the product path.)
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import _build

VN_OBS_DIM = 80
VN_VARIANT_CUBIC = 0
VN_VARIANT_SIMPLE = 1
VN_ABI_VERSION = 2
VN_STATE_FIELDS = 16
VN_MAX_L = 16
STATE_FIELDS = (
    "x", "y", "z", "facing", "last_action", "step_count", "visited_count", "bump_count",
    "done", "last_bump", "near_wall", "was_near_wall", "cells_insight_down", "room",
    "max_steps", "next_seed",
)


class VnRoomSet(C.Structure):
    _fields_ = [("n_rooms", C.c_int32), ("whd", C.c_void_p), ("walls", C.c_void_p), ("fixed_start", C.c_void_p),
                ("goal", C.c_void_p)]


class VnConfig(C.Structure):
    _fields_ = [
        ("local_map_length", C.c_int32), ("use_room_draw", C.c_int32), ("autoreset", C.c_int32),
        ("variant", C.c_int32), ("crash_penalty", C.c_double), ("finish_percentage", C.c_double),
        ("agent_id_base", C.c_int64), ("seed_stride", C.c_int64),
    ]


class VnInfo(C.Structure):
    _fields_ = [
        ("n_agents", C.c_int32), ("n_rooms", C.c_int32), ("local_map_length", C.c_int32),
        ("pad_w", C.c_int32), ("pad_d", C.c_int32), ("pad_h", C.c_int32),
        ("belief_bytes_per_agent", C.c_int64), ("device_bytes", C.c_int64),
        ("variant", C.c_int32), ("obs_dim", C.c_int32),
    ]


class VoxnavError(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None

P = C.c_void_p
_SIGS = {
    "vn_last_error": (C.c_char_p, []),
    "vn_abi_version": (C.c_int, []),
    "vn_create": (C.c_int, [C.POINTER(VnRoomSet), C.c_int32, C.POINTER(VnConfig), C.c_int32, C.POINTER(P)]),
    "vn_destroy": (C.c_int, [P]),
    "vn_get_info": (C.c_int, [P, C.POINTER(VnInfo)]),
    "vn_reset": (C.c_int, [P, P, P, P, P]),
    "vn_step": (C.c_int, [P, P, P, P, P, P, P, P, P]),
    "vn_step_random": (C.c_int, [P, C.c_uint64, C.c_uint64, C.c_int32, P, P, P, P, P, P, P, P]),
    "vn_export_state": (C.c_int, [P, P, P]),
    "vn_kernel_label": (C.c_int, [P, C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_int32]),
    "vn_export_belief": (C.c_int, [P, P, P]),
    "vn_gae": (C.c_int, [P, P, P, P, P, C.c_int32, C.c_int32, C.c_double, C.c_double, P, P, P]),
    "vn_lstm_cell": (C.c_int, [P, C.c_int64, P, P, P, P, P, P, P, C.c_int32, C.c_int32, C.c_int32, P]),
    "vn_policy_head": (C.c_int, [P, P, C.c_int32, C.c_int32, P, P, C.c_int32, P, P, C.c_uint64, C.c_uint64,
                                 C.c_int64, C.c_int32, P, P, P, P]),
    "vn_lstm_cell_masked": (C.c_int, [P, C.c_int64, P, P, P, P, P, P, P, C.c_int32, C.c_int32, C.c_int32, P]),
    "vn_lstm_cell_bf16": (C.c_int, [P, C.c_int64, P, P, P, P, P, P, P, P, C.c_int32, C.c_int32, C.c_int32, P]),
    "vn_policy_head_bf16": (C.c_int, [P, P, C.c_int32, C.c_int32, P, P, C.c_int32, P, P, C.c_uint64, C.c_uint64,
                                      C.c_int64, C.c_int32, P, P, P, P]),
    "vn_lstm_fused_bf16": (C.c_int, [P, C.c_int32, P, P, C.c_int32, P, P, P, P, P, P, C.c_int32, C.c_int32,
                                     C.c_int32, P]),
    "vn_lstm_fused_bf16_masked": (C.c_int, [P, C.c_int32, P, P, C.c_int32, P, P, P, P, P, P, C.c_int32, C.c_int32,
                                            C.c_int32, P]),
    "vn_lstm_fused_f32": (C.c_int, [P, C.c_int32, P, P, C.c_int32, P, P, P, P, P, C.c_int32, C.c_int32, C.c_int32,
                                    P]),
    "vn_linear_f32": (C.c_int, [C.c_int32, P, C.c_int64, P, P, P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, P]),
    "vn_mlp_head_f32": (C.c_int, [C.c_int32, P, C.c_int64, C.c_int32, C.c_int32, P, P, P, P, P, C.c_int32, P, P,
                                  C.c_uint64, C.c_uint64, C.c_int64, C.c_int32, P, P, P, C.c_int32, P]),
    "vn_collect_compact": (C.c_int, [P, P, C.c_int32, P, P, P]),
    "vn_collect_bootstrap": (C.c_int, [P, P, C.c_int32, C.c_double, P, P]),
    "vn_collect_stash": (C.c_int, [P, P, P, P, C.c_int32, C.c_int32, P, C.c_int32, P, C.c_int32, P, C.c_int32, P, P,
                                   P, P, C.c_int32, P]),
    "vn_monitor_step": (C.c_int, [P, P, P, P, C.c_int32, P, P, P, P, P]),
    "vn_collect_post_step": (C.c_int, [P, P, C.c_int32, C.c_int32, P, P, P, P, P, P, P, P, C.c_int32, P, C.c_int32,
                                       P, C.c_int32, P, P, P, P, C.c_int32, P, P, P, P, C.c_int32, P]),
    "vn_episode_start": (C.c_int, [P, P, C.c_int32, P, P, P, P, C.c_int32, C.c_int32, P]),
    "vn_lstm_seq_pack_size": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, P, P]),
    "vn_lstm_seq_fwd_mfma": (C.c_int, [P, C.c_int32, P, P, P, P, P, P, P, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                       P]),
    "vn_lstm_seq_bwd_mfma": (C.c_int, [P, P, P, P, P, P, P, P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, P]),
    "vn_lstm_rows_supported": (C.c_int, [C.c_int32, C.c_int32, C.c_int32]),
    "vn_lstm_rows_part_floats": (C.c_int, [C.c_int32, P]),
    "vn_lstm_rows_fwd": (C.c_int, [P, C.c_int32, P, P, P, P, P, C.c_int64, P, P, P, P, P, P, P, P, P, P,
                                   C.c_int32, C.c_int32, C.c_int32, P]),
    "vn_lstm_rows_bwd": (C.c_int, [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, C.c_int32, C.c_int32, C.c_int32,
                                   P]),
    "vn_ppo_loss_part_floats": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, P, P]),
    "vn_ppo_loss": (C.c_int, [P, P, C.c_int64, P, P, P, P, P, P, P, P, P, C.c_int32, C.c_int32, C.c_int32, C.c_float,
                              C.c_float, C.c_float, C.c_int32, P, P, P, P, P, P, P, P]),
    "vn_grad_norm": (C.c_int, [P, P, C.c_int32, C.c_float, P, P, P, P]),
    "vn_adam_step": (C.c_int, [P, P, P, P, P, P, C.c_int32, P, P, C.c_float, C.c_float, C.c_float, C.c_float,
                               C.c_int64, P]),
    "vn_minibatch_rows": (C.c_int, [P, C.c_int32, C.c_int32, C.c_int32, P, C.c_int32, P, P, P]),
    "vn_gemm_f32_linear": (C.c_int, [P, C.c_int64, C.c_int64, P, C.c_int64, C.c_int64, P, C.c_int64, P, C.c_int64,
                                     C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, P]),
    "vn_gemm_f32_dx": (C.c_int, [P, P, C.c_int64, C.c_int64, P, C.c_int64, C.c_int64, P, C.c_int64, C.c_int64,
                                 C.c_int32, C.c_int32, C.c_int32, C.c_int32, P]),
    "vn_gemm_f32_tn": (C.c_int, [P, P, C.c_int64, C.c_int64, P, C.c_int64, C.c_int64, P, C.c_int64, P, C.c_int32,
                                 C.c_int32, C.c_int32, C.c_int32, C.c_int32, P, P, C.c_int32, P]),
}
EXPORTED_SYMBOLS = tuple(_SIGS)


def _bind(lib, strict: bool = True):
    for name, (res, args) in _SIGS.items():
        if not strict and not hasattr(lib, name):
            continue                      # an older A/B build without this entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.vn_abi_version() != VN_ABI_VERSION:
        raise VoxnavError("libvoxnav ABI version mismatch")
    return lib


def load_variant(path):
    """Load another build of the library (A/B benchmarking); separate handle."""
    import torch  # noqa: F401
    return _bind(C.CDLL(str(path)), strict=False)


def load(build_if_missing: bool = True):
    """Load libvoxnav.so (building it with hipcc first if it is stale)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if build_if_missing and _build.needs_build():
            _build.build()
        if not _build.LIB.exists():
            raise VoxnavError(f"HIP library missing: {_build.LIB} (run __graft_entry__.build())")
        # torch first: its libamdhip64.so.7 then satisfies our NEEDED entry, so
        # the process has one HIP runtime.
        import torch  # noqa: F401
        # VOXNAV_LIB: another build of the library in the product's place
        # (A/B timing of diagnostics builds under _lib/variants only)
        alt = os.environ.get("VOXNAV_LIB")
        _lib = _bind(C.CDLL(str(alt if alt else _build.LIB)), strict=not alt)
        return _lib


def check(rc: int, what: str = "voxnav"):
    if rc != 0:
        msg = load().vn_last_error().decode(errors="replace")
        raise VoxnavError(f"{what} failed ({rc}): {msg}")
