"""ctypes binding of the C ABI in ``include/tt_mi355x.h`` (libtt_mi355x.so, gfx950).

The library is loaded after ``import torch`` so that its ``libamdhip64.so.7`` dependency resolves to
the HIP runtime torch already loaded (one runtime per process: torch's streams and device pointers
are then valid in our kernels). There is no CPU fallback: if the library is missing or does not
export every symbol the header declares, loading raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libtt_mi355x.so"
# measurement scripts only: an experiment build (TT_EXPERIMENTS=1, built with
# `python -m two_tower_recommender_model_amd.build --experiments`) sits beside the release library
EXP_LIB_PATH = Path(__file__).resolve().parent / "lib_exp" / "libtt_mi355x.so"
# same-box A/B libraries of the measurement scripts (scripts/exp_ab.sh): only these two places
_AB_DIRS = ("lib_prev", "lib_var")


def _experiment_lib():
    """TT_EXPERIMENT_LIB (measurement scripts only): "1" = the experiment build above, or a
    ``libtt_mi355x.so`` under this package's ``lib_prev/`` or ``lib_var/<name>/`` (an A/B of an
    earlier build of this tree). Anything else is refused: the product loads no other library."""
    exp = os.environ.get("TT_EXPERIMENT_LIB", "")
    if not exp:
        return None
    if exp == "1":
        return EXP_LIB_PATH
    p = Path(exp).resolve()
    pkg = Path(__file__).resolve().parent
    if p.name == "libtt_mi355x.so" and any(pkg / d in p.parents for d in _AB_DIRS):
        return p
    raise TTError(f"TT_EXPERIMENT_LIB={exp!r}: only '1' (lib_exp/) or a libtt_mi355x.so under "
                  f"{', '.join(d + '/' for d in _AB_DIRS)} of the package")

TT_OK = 0
TT_I32, TT_I64, TT_F32, TT_BF16 = 0, 1, 2, 3
TT_POOL_SUM, TT_POOL_MEAN = 0, 1
TT_TOWER_GENERAL_T1 = 1
TT_MAX_FEATURES = 64
TT_MAX_TABLES = 64


class TableMeta(C.Structure):
    _fields_ = [
        ("weight_offset", C.c_int64),
        ("state_offset", C.c_int64),
        ("num_rows", C.c_int64),
        ("dim", C.c_int32),
        ("_pad", C.c_int32),
    ]


class FeatureMeta(C.Structure):
    _fields_ = [("table", C.c_int32), ("out_offset", C.c_int32), ("out_row", C.c_int64)]


class ShardSeg(C.Structure):
    _fields_ = [("cap", C.c_int64), ("key_index", C.c_int64), ("cnt_index", C.c_int64), ("pos_in", C.c_int32),
                ("pos_out", C.c_int32)]


class TowerShape(C.Structure):
    _fields_ = [
        ("L", C.c_int32),
        ("width", C.c_int32 * 4),
        ("in_dim", C.c_int32 * 2),
        ("in_col", C.c_int32 * 2),
        ("flags", C.c_int32),
    ]


# ---- launch plans (tt_launch): the multi-role fused launches -------------------------------------
ROLE_WGRAD, ROLE_UPDATE, ROLE_INSERT, ROLE_RESOLVE = 0x01, 0x02, 0x04, 0x08
ROLE_ADAGRAD, ROLE_ROUTE_COUNT, ROLE_ROUTE_PLACE, ROLE_GATHER = 0x10, 0x20, 0x40, 0x80


class WgradRole(C.Structure):
    _fields_ = [("loss", C.c_void_p), ("adam_step_state", C.c_void_p), ("adam_lr", C.c_float),
                ("adam_beta1", C.c_float), ("adam_beta2", C.c_float)]


class UpdateRole(C.Structure):
    _fields_ = [("params", C.c_void_p), ("exp_avg", C.c_void_p), ("exp_avg_sq", C.c_void_p), ("eps", C.c_float),
                ("beta1", C.c_float), ("beta2", C.c_float), ("weight_decay", C.c_float), ("grads_out", C.c_void_p),
                ("replicated", C.c_int32), ("copies", C.c_int32), ("base", C.c_void_p),
                ("offsets", C.POINTER(C.c_int64)), ("scale", C.c_float)]


class InsertRole(C.Structure):
    _fields_ = [("next_cols", C.POINTER(C.c_void_p)), ("id_dtype", C.c_int32),
                ("num_embeddings", C.POINTER(C.c_int64)), ("dedup_tables", C.POINTER(C.c_int32)),
                ("next_dedup_ws", C.c_void_p), ("dedup_ws_bytes", C.c_size_t), ("dedup_max_lookups", C.c_int64)]


class ResolveRole(C.Structure):
    _fields_ = [("dedup_ws", C.c_void_p)]


class AdagradRole(C.Structure):
    _fields_ = [("tables", C.POINTER(TableMeta)), ("T", C.c_int32), ("F", C.c_int32),
                ("features", C.POINTER(FeatureMeta)), ("B", C.c_int64), ("grad", C.c_void_p), ("ldg", C.c_int64),
                ("weights", C.c_void_p), ("state", C.c_void_p), ("lr", C.c_float), ("eps", C.c_float),
                ("dedup_ws", C.c_void_p), ("dedup_ws_bytes", C.c_size_t), ("dedup_max_lookups", C.c_int64),
                ("multi_only", C.c_int32)]


class RouteRole(C.Structure):
    _fields_ = [("F", C.c_int32), ("id_dtype", C.c_int32), ("cols", C.POINTER(C.c_void_p)),
                ("num_embeddings", C.POINTER(C.c_int64)), ("block_sizes", C.POINTER(C.c_int64)),
                ("owners", C.POINTER(C.c_int32)), ("W", C.c_int32), ("segs", C.c_void_p), ("send", C.c_void_p),
                ("pos_in", C.c_void_p), ("pos_out", C.c_void_p), ("overflow", C.c_void_p), ("route_ws", C.c_void_p),
                ("route_ws_bytes", C.c_size_t)]


TT_PEER_MAXW = 16
TT_PEER_HANDLE_BYTES = 64


class PeerDirect(C.Structure):
    """tt_peer_direct_t (ABI 4): a producer's stores straight into the destinations' receive buffers."""
    _fields_ = [("W", C.c_int32), ("_pad", C.c_int32), ("first_row", C.c_int64 * TT_PEER_MAXW),
                ("row0", C.c_void_p * TT_PEER_MAXW), ("copy_src", C.c_void_p * TT_PEER_MAXW),
                ("copy_dst", C.c_void_p * TT_PEER_MAXW), ("copy_len", C.c_int64 * TT_PEER_MAXW),
                ("epoch", C.c_void_p)]


class PeerWait(C.Structure):
    """tt_peer_wait_t (ABI 4): a consumer launch's in-launch signal / wait of such an exchange."""
    _fields_ = [("W", C.c_int32), ("sys", C.c_int32), ("flag", C.c_void_p * TT_PEER_MAXW), ("flags", C.c_void_p),
                ("epoch", C.c_void_p), ("err", C.c_void_p), ("timeout_ticks", C.c_int64)]


class GatherRole(C.Structure):
    _fields_ = [("weights", C.c_void_p), ("tables", C.POINTER(TableMeta)), ("T", C.c_int32), ("recv", C.c_void_p),
                ("block_i64", C.c_int64), ("counts_i64", C.c_int64), ("seg_off", C.POINTER(C.c_int64)),
                ("slots", C.c_int64), ("rows_out", C.c_void_p), ("out_stride", C.c_int64), ("bad", C.c_void_p),
                ("dedup_ws", C.c_void_p), ("dedup_ws_bytes", C.c_size_t), ("dedup_max_lookups", C.c_int64),
                ("direct", C.POINTER(PeerDirect))]


class LaunchPlan(C.Structure):
    _fields_ = [("roles", C.c_uint32), ("shape", C.POINTER(TowerShape)), ("B", C.c_int64),
                ("workspace", C.c_void_p), ("ws_bytes", C.c_size_t), ("wgrad", WgradRole), ("update", UpdateRole),
                ("insert", InsertRole), ("resolve", ResolveRole), ("adagrad", AdagradRole), ("route", RouteRole),
                ("gather", GatherRole), ("wait", C.POINTER(PeerWait))]


class PeerPut(C.Structure):
    _fields_ = [("W", C.c_int32), ("rank", C.c_int32), ("src", C.c_void_p),
                ("src_off", C.c_int64 * TT_PEER_MAXW), ("len", C.c_int64 * TT_PEER_MAXW),
                ("dst", C.c_void_p * TT_PEER_MAXW), ("flag", C.c_void_p * TT_PEER_MAXW), ("state", C.c_void_p),
                ("same_device", C.c_int32), ("_pad", C.c_int32)]


def launch(plan: LaunchPlan, stream: int, what: str = "launch") -> None:
    """tt_launch(plan) on ``stream``; raises on a non-zero status. Keep every array the plan points
    to alive until the call returns (the launch copies what it needs into kernel arguments)."""
    check(load().tt_launch(C.byref(plan), stream), what)


_vp = C.c_void_p
_i32 = C.c_int32
_i64 = C.c_int64
_f32 = C.c_float
_sz = C.c_size_t
_int = C.c_int
_pvp = C.POINTER(C.c_void_p)
_pi64 = C.POINTER(C.c_int64)
_pi32 = C.POINTER(C.c_int32)
_ptm = C.POINTER(TableMeta)
_pfm = C.POINTER(FeatureMeta)
_psh = C.POINTER(TowerShape)

# name -> (restype, argtypes); the compute entry points are exactly those counted by
# tt_num_entry_points() in csrc/api.cpp.
SIGNATURES = {
    "tt_last_error_string": (C.c_char_p, []),
    "tt_abi_version": (_int, []),
    "tt_num_entry_points": (_int, []),
    "tt_kjt_build_workspace_bytes": (_sz, [_i64]),
    "tt_kjt_build_mod_dropzero": (
        _int,
        [_int, _i64, _pvp, _int, _pi64, _vp, _vp, _vp, _vp, _vp, _sz, _vp],
    ),
    "tt_kjt_single_hot_cols": (_int, [_int, _i64, _vp, _int, _vp, _pi64, _pvp, _vp, _vp, _int, _vp, _vp]),
    "tt_complete_cumsum_workspace_bytes": (_sz, [_i64]),
    "tt_kjt_route_workspace_bytes": (_sz, [_int, _i64, _int]),
    "tt_kjt_route": (_int, [_int, _i64, _vp, _int, _vp, _pi64, _pi64, _vp, _int, _i64, _i64, _vp, _vp, _vp, _sz, _vp]),
    "tt_kjt_unpack_workspace_bytes": (_sz, [_int, _int, _i64]),
    "tt_kjt_unpack": (_int, [_int, _int, _i64, _vp, _i64, _i64, _vp, _int, _vp, _vp, _vp, _vp, _sz, _vp]),
    "tt_pooled_partials_sum": (_int, [_int, _int, _i64, _int, _vp, _i64, _i64, _vp, _vp, _i64, _vp]),
    "tt_pooled_grad_pack": (_int, [_int, _int, _i64, _int, _vp, _i64, _vp, _vp, _i64, _i64, _vp]),
    "tt_complete_cumsum": (_int, [_vp, _i64, _vp, _vp, _sz, _vp]),
    "tt_kjt_permute": (
        _int,
        [_int, _i64, _vp, _vp, _vp, _int, _vp, _pi32, _int, _vp, _vp, _vp, _vp, _vp],
    ),
    "tt_block_bucketize_workspace_bytes": (_sz, [_int, _i64, _int]),
    "tt_block_bucketize": (
        _int,
        [_int, _i64, _vp, _vp, _vp, _int, _pi64, _int, _vp, _vp, _vp, _vp, _sz, _vp],
    ),
    "tt_pooled_fwd": (
        _int,
        [_vp, _ptm, _int, _pfm, _int, _i64, _vp, _int, _vp, _int, _vp, _i64, _int, _vp, _vp],
    ),
    "tt_bwd_workspace_bytes": (_sz, [_i64]),
    "tt_bwd_workspace_init": (_int, [_vp, _sz, _i64, _vp]),
    "tt_bwd_prepare": (
        _int,
        [_ptm, _int, _pfm, _int, _i64, _vp, _int, _vp, _int, _vp, _sz, _i64, _vp],
    ),
    "tt_bwd_rowwise_adagrad": (
        _int,
        [_ptm, _int, _pfm, _int, _i64, _vp, _i64, _vp, _int, _vp, _vp, _f32, _f32, _vp, _sz, _i64, _vp],
    ),
    "tt_pooled_bwd_dense": (
        _int,
        [_ptm, _int, _pfm, _int, _i64, _vp, _i64, _vp, _int, _vp, _int, _vp, _int, _vp],
    ),
    "tt_linear_fwd": (_int, [_int, _pvp, _int, _i64, _pvp, _pvp, _i64, _int, _int, _pvp, _i64, _int, _int, _vp]),
    "tt_linear_bwd_data": (_int, [_int, _pvp, _pvp, _i64, _pvp, _i64, _int, _int, _pvp, _i64, _int, _int, _vp]),
    "tt_linear_bwd_weight_workspace_bytes": (_sz, [_int, _i64, _int, _int]),
    "tt_linear_bwd_weight": (
        _int,
        [_int, _pvp, _pvp, _i64, _pvp, _int, _i64, _i64, _int, _int, _pvp, _pvp, _int, _int, _vp, _sz, _vp],
    ),
    "tt_dot_bce_workspace_bytes": (_sz, [_i64]),
    "tt_dot_bce_workspace_init": (_int, [_vp, _sz, _i64, _vp]),
    "tt_dot_bce_fwd_bwd": (
        _int,
        [_vp, _i64, _vp, _i64, _i64, _int, _vp, _int, _vp, _vp, _vp, _i64, _vp, _i64, _f32, _vp, _sz, _vp],
    ),
    "tt_adam_step": (_int, [_vp, _vp, _vp, _vp, _i64, _f32, _f32, _f32, _f32, _f32, _vp, _vp]),
    "tt_pooled_fwd_cols": (_int, [_vp, _ptm, _int, _pfm, _int, _i64, _pvp, _int, _pi64, _vp, _i64, _vp]),
    "tt_bwd_prepare_cols": (_int, [_ptm, _int, _pfm, _int, _i64, _pvp, _int, _pi64, _vp, _sz, _i64, _vp]),
    "tt_dedup_workspace_bytes": (_sz, [_i64]),
    "tt_dedup_workspace_init": (_int, [_vp, _sz, _i64, _vp]),
    "tt_dedup_insert_cols": (_int, [_ptm, _int, _pfm, _int, _i64, _pvp, _int, _pi64, _vp, _sz, _i64, _vp]),
    "tt_dedup_insert_segments": (_int, [_vp, _vp, _i64, _i64, _vp, _sz, _i64, _vp]),
    "tt_dedup_rowwise_adagrad": (
        _int,
        [_ptm, _int, _pfm, _int, _i64, _vp, _i64, _vp, _vp, _f32, _f32, _vp, _sz, _i64, _vp],
    ),
    "tt_tower_num_params": (C.c_int64, [_psh]),
    "tt_tower_workspace_bytes": (_sz, [_psh, _i64]),
    "tt_tower_workspace_init": (_int, [_psh, _i64, _vp, _sz, _vp]),
    "tt_tower_fwd_bwd": (_int, [_psh, _i64, _vp, _i64, _vp, _vp, _vp, _int, _f32, _vp, _vp, _sz, _vp]),
    "tt_tower_wgrad": (_int, [_psh, _i64, _vp, _vp, _sz, _vp]),
    "tt_tower_fwd_bwd_gather": (
        _int,
        [_psh, _i64, _pvp, _int, _pi64, _pvp, _vp, _i64, _vp, _vp, _vp, _int, _f32, _vp, _pi32, _vp, _sz, _i64,
         _vp, _sz, _vp],
    ),
    "tt_tower_fwd_bwd_kjt": (
        _int,
        [_psh, _i64, _vp, _int, _vp, _pi64, _pvp, _vp, _i64, _vp, _vp, _vp, _int, _f32, _vp, _vp, _sz, _vp],
    ),
    "tt_tower_update_pre": (_int, [_psh, _i64, _vp, _vp, _vp, _f32, _f32, _f32, _f32, _vp, _vp, _sz, _vp]),
    "tt_tower_wgrad_pre": (_int, [_psh, _i64, _vp, _vp, _sz, _vp, _f32, _f32, _f32, _vp, _sz, _i64, _vp]),
    "tt_dedup_resolve": (_int, [_vp, _sz, _i64, _vp]),
    "tt_shard_route_workspace_bytes": (_sz, [_int, _i64]),
    "tt_shard_route_cols": (
        _int,
        [_int, _i64, _pvp, _int, _pi64, _pi64, _pi32, _int, _i64, _vp, _vp, _vp, _vp, _sz, _vp],
    ),
    "tt_shard_gather_rows": (_int, [_vp, _ptm, _int, _int, _int, _i64, _vp, _vp, _vp, _vp, _sz, _i64, _vp]),
    "tt_shard_gather_rows_bf16": (_int, [_vp, _ptm, _int, _int, _int, _i64, _vp, _vp, _vp, _vp, _sz, _i64, _vp]),
    "tt_tower_adam_grads": (
        _int,
        [_psh, _i64, _vp, _vp, _vp, _vp, _f32, _f32, _f32, _f32, _f32, _vp, _vp, _sz, _vp],
    ),
    "tt_tower_fwd_bwd_indexed": (
        _int,
        [_psh, _i64, _pvp, _pvp, _pvp, _vp, _vp, _int, _f32, _vp, _vp, _sz, _vp],
    ),
    "tt_tower_fwd_bwd_indexed_bf16": (
        _int,
        [_psh, _i64, _pvp, _pvp, _pvp, _vp, _vp, _int, _f32, _vp, _vp, _sz, _vp],
    ),
    "tt_tower_update": (
        _int,
        [_psh, _i64, _vp, _vp, _vp, _f32, _f32, _f32, _f32, _f32, _vp, _int, _vp, _vp, _sz, _vp],
    ),
    "tt_shard_route_segs": (
        _int,
        [_int, _i64, _pvp, _int, _pi64, _pi64, _pi32, _int, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp],
    ),
    "tt_shard_gather_segs_bf16": (
        _int,
        [_vp, _ptm, _int, _int, _int, _vp, _i64, _i64, _pi64, _i64, _vp, _i64, _vp, _vp, _sz, _i64, _vp],
    ),
    "tt_tower_fwd_bwd_indexed2_bf16": (
        _int,
        [_psh, _i64, _pvp, _pvp, _pvp, _pvp, _vp, _vp, _int, _f32, _vp, _vp, _sz, C.POINTER(PeerDirect), _vp],
    ),
    "tt_tower_grads_replicated": (_int, [_psh, _i64, _vp, _vp, _int, _pi64, _f32, _vp, _sz, _vp]),
    "tt_tower_fwd_bwd_gather_update": (
        _int,
        [_psh, _i64, _pvp, _int, _pi64, _pvp, _pvp, _vp, _i64, _vp, _vp, _vp, _int, _f32, _vp, _f32, _f32, _vp, _sz,
         _i64, _pvp, _vp, _sz, _vp],
    ),
    "tt_tower_adam_pre_grads_sum": (
        _int, [_psh, _i64, _vp, _vp, _int, _i64, _vp, _vp, _f32, _f32, _f32, _f32, _vp, _sz, C.POINTER(PeerWait), _vp],
    ),
    "tt_tower_fwd_bwd_indexed_multi_bf16": (
        _int,
        [_psh, _i64, _int, _vp, _vp, _vp, _vp, _vp, _vp, _int, _f32, _vp, _vp, _sz, _vp],
    ),
    "tt_bwd_rowwise_adagrad_part": (
        _int, [_ptm, _int, _pfm, _int, _i64, _vp, _i64, _vp, _int, _vp, _vp, _f32, _f32, _vp, _sz, _i64, _int, _vp],
    ),
    "tt_launch": (_int, [C.c_void_p, _vp]),
    "tt_peer_alloc": (_int, [_sz, _pvp]),
    "tt_peer_free": (_int, [_vp]),
    "tt_peer_export": (_int, [_vp, _vp, _pi64]),
    "tt_peer_import": (_int, [_vp, _pvp]),
    "tt_peer_unimport": (_int, [_vp]),
    "tt_peer_exchange": (_int, [C.c_void_p, _vp, _vp, C.c_double, _vp]),
    "tt_kjt_admit": (_int, [_int, _i64, _vp, _int, _i64, _vp, _pi64, _pi64, _pi32, _int, _vp, _vp]),
    "tt_table_prefault": (_int, [_vp, _sz, _sz, _vp, _vp]),
    "tt_table_alloc": (_int, [_sz, _pvp, C.POINTER(C.c_int)]),
    "tt_table_free": (_int, [_vp]),
}

COMPUTE_ENTRY_POINTS = [
    "tt_kjt_build_mod_dropzero",
    "tt_kjt_single_hot_cols",
    "tt_kjt_route",
    "tt_kjt_unpack",
    "tt_pooled_partials_sum",
    "tt_pooled_grad_pack",
    "tt_complete_cumsum",
    "tt_kjt_permute",
    "tt_block_bucketize",
    "tt_pooled_fwd",
    "tt_bwd_workspace_init",
    "tt_bwd_prepare",
    "tt_bwd_rowwise_adagrad",
    "tt_pooled_bwd_dense",
    "tt_linear_fwd",
    "tt_linear_bwd_data",
    "tt_linear_bwd_weight",
    "tt_dot_bce_workspace_init",
    "tt_dot_bce_fwd_bwd",
    "tt_adam_step",
    "tt_tower_workspace_init",
    "tt_tower_fwd_bwd",
    "tt_tower_wgrad",
    "tt_tower_fwd_bwd_gather",
    "tt_tower_fwd_bwd_kjt",
    "tt_tower_update",
    "tt_pooled_fwd_cols",
    "tt_bwd_prepare_cols",
    "tt_dedup_workspace_init",
    "tt_dedup_insert_cols",
    "tt_dedup_insert_segments",
    "tt_dedup_rowwise_adagrad",
    "tt_tower_fwd_bwd_indexed",
    "tt_tower_wgrad_pre",
    "tt_dedup_resolve",
    "tt_shard_route_cols",
    "tt_shard_gather_rows",
    "tt_shard_gather_rows_bf16",
    "tt_tower_fwd_bwd_indexed_bf16",
    "tt_tower_adam_grads",
    "tt_tower_update_pre",
    "tt_shard_route_segs",
    "tt_shard_gather_segs_bf16",
    "tt_tower_fwd_bwd_indexed2_bf16",
    "tt_tower_grads_replicated",
    "tt_tower_fwd_bwd_gather_update",
    "tt_tower_adam_pre_grads_sum",
    "tt_tower_fwd_bwd_indexed_multi_bf16",
    "tt_bwd_rowwise_adagrad_part",
    "tt_launch",
    "tt_peer_exchange",
    "tt_kjt_admit",
    "tt_table_prefault",
]

_lib = None
_lock = threading.Lock()


class TTError(RuntimeError):
    pass


def load(path: os.PathLike | None = None):
    """Load (once) and return the ctypes library with argtypes set. Raises if absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = Path(path) if path else _experiment_lib() or LIB_PATH
        if not p.exists():
            raise TTError(
                f"libtt_mi355x.so not found at {p}: build it with "
                "`python -m two_tower_recommender_model_amd.build` (no CPU fallback exists)"
            )
        lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)  # AttributeError if a declared symbol is missing
            fn.restype = res
            fn.argtypes = args
        if lib.tt_num_entry_points() != len(COMPUTE_ENTRY_POINTS):
            raise TTError("libtt_mi355x.so entry-point count does not match the header")
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str = "") -> None:
    if rc != TT_OK:
        msg = load().tt_last_error_string()
        msg = msg.decode() if msg else ""
        raise TTError(f"{what or 'tt call'} failed (status {rc}): {msg}")


def ptr(t) -> int:
    """Device (or host) address of a tensor, or 0 for None."""
    if t is None:
        return 0
    return t.data_ptr()


def ptr_array(ts):
    arr = (C.c_void_p * len(ts))()
    for i, t in enumerate(ts):
        arr[i] = ptr(t) if t is not None else None
    return arr


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def id_dtype_code(dtype: torch.dtype) -> int:
    if dtype == torch.int64:
        return TT_I64
    if dtype == torch.int32:
        return TT_I32
    raise TTError(f"ids must be int32 or int64, got {dtype}")


_hip = None


def graph_upload(g: "torch.cuda.CUDAGraph", device=None) -> None:
    """hipGraphUpload of a captured graph on the current stream: the executable graph's first
    launch then carries no upload (a timed run that replays graphs for the first time would pay
    it inside the timed region). Runs no kernel; a no-op where the runtime lacks the call."""
    global _hip
    if _hip is None:
        try:
            _hip = C.CDLL("libamdhip64.so", mode=C.RTLD_GLOBAL)
            _hip.hipGraphUpload.restype = C.c_int
            _hip.hipGraphUpload.argtypes = [C.c_void_p, C.c_void_p]
        except (OSError, AttributeError):
            _hip = False
    if _hip:
        rc = _hip.hipGraphUpload(C.c_void_p(g.raw_cuda_graph_exec()), C.c_void_p(stream_handle(device)))
        if rc != 0:
            raise TTError(f"hipGraphUpload failed ({rc})")
