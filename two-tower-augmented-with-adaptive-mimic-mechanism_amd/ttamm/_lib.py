"""ctypes binding of libttamm.so (the C ABI declared in include/ttamm.h).

This is the only place Python talks to the native library.  Every product code path on a
ROCm device goes through here; there is no CPU fallback — a missing library raises.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

import torch

TTAMM_OK = 0
TTAMM_E_INVALID = 1
TTAMM_E_RUNTIME = 2
TTAMM_E_HIP = 3

MAX_LINEAR = 6
FUSION_IDENTITY, FUSION_SUM, FUSION_GATED, FUSION_CONCAT = 0, 1, 2, 3
ACT_RELU, ACT_GELU, ACT_TANH, ACT_SELU = 0, 1, 2, 3  # ttamm.h TTAMM_ACT_*
OPT_SPARSE_ADAM, OPT_DENSE = 0, 1
STATUS_SAMPLER_EXHAUSTED = 1
STATUS_INDEX_OUT_OF_RANGE = 2
STATUS_LOOKAHEAD_MISMATCH = 4  # row-sharded step: a batch other than the prepared look-ahead's
STATUS_POISON = STATUS_SAMPLER_EXHAUSTED | STATUS_INDEX_OUT_OF_RANGE | STATUS_LOOKAHEAD_MISMATCH  # bits that stop every later step

_NATIVE_DIR = Path(__file__).resolve().parent / "_native"
LIB_PATH = _NATIVE_DIR / "libttamm.so"

c_f = ctypes.c_float
c_d = ctypes.c_double
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_vp = ctypes.c_void_p


class Linear(ctypes.Structure):
    _fields_ = [
        ("weight", c_vp),
        ("bias", c_vp),
        ("weight_exp_avg", c_vp),
        ("weight_exp_avg_sq", c_vp),
        ("bias_exp_avg", c_vp),
        ("bias_exp_avg_sq", c_vp),
        ("in_features", c_i32),
        ("out_features", c_i32),
    ]


class Table(ctypes.Structure):
    _fields_ = [
        ("weight", c_vp),
        ("exp_avg", c_vp),
        ("exp_avg_sq", c_vp),
        ("rows", c_i64),
        ("dim", c_i32),
        ("optimizer", c_i32),
        ("last_step", c_vp),
        ("has_padding_idx", c_i32),
        ("padding_idx", c_i64),
        ("max_norm", c_d),
        ("touched", c_vp),
    ]


class Tower(ctypes.Structure):
    _fields_ = [
        ("id", Table),
        ("mimic", Table),
        ("features", c_vp),
        ("feat_ld", c_i64),
        ("feat_dim", c_i32),
        ("fusion", c_i32),
        ("n_linear", c_i32),
        ("dropout", c_f),
        ("activation", c_i32),
        ("linear", Linear * MAX_LINEAR),
        ("gate", Linear * 2),
        ("matmul_bf16", c_i32),
        ("features_bf16", c_vp),
        ("feat_bf16_ld", c_i64),
        ("features_planes", c_vp),
        ("feat_planes_ld", c_i64),
    ]


class HParams(ctypes.Structure):
    _fields_ = [
        ("lr", c_d),
        ("beta1", c_d),
        ("beta2", c_d),
        ("eps", c_d),
        ("weight_decay", c_d),
        ("decoupled_weight_decay", c_i32),
        ("sparse_lr", c_d),
        ("sparse_beta1", c_d),
        ("sparse_beta2", c_d),
        ("sparse_eps", c_d),
        ("dense_step", c_i64),
        ("sparse_step", c_i64),
        ("lambda_mimic_user", c_d),
        ("lambda_mimic_item", c_d),
        ("lambda_category_alignment", c_d),
        ("grad_clip_norm", c_d),
        ("dense_optimizer", c_i32),
        ("momentum", c_d),
        ("dampening", c_d),
        ("nesterov", c_i32),
        ("sgd_first_step", c_i32),
    ]


class Batch(ctypes.Structure):
    _fields_ = [
        ("users", c_vp),
        ("pos_items", c_vp),
        ("neg_items", c_vp),
        ("batch", c_i64),
        ("num_neg", c_i32),
        ("sample_negatives", c_i32),
        ("pos_offsets", c_vp),
        ("pos_values", c_vp),
        ("seed", c_u64),
        ("counter", c_u64),
        ("user_keep_mask", c_vp * MAX_LINEAR),
        ("item_keep_mask", c_vp * MAX_LINEAR),
    ]


class StepArgs(ctypes.Structure):
    _fields_ = [
        ("user", Tower),
        ("item", Tower),
        ("mimic_enabled", c_i32),
        ("hp", HParams),
        ("b", Batch),
        ("loss_out", c_vp),
        ("loss_accum", c_vp),
        ("status", c_vp),
        ("workspace", c_vp),
        ("workspace_bytes", ctypes.c_size_t),
        ("timing_events", c_vp * 14),
        # row-sharded multi-GPU step (ttamm.h TTAMM_PHASE_*)
        ("phase", c_i32),
        ("row_base", c_i64),
        ("global_batch", c_i64),
        ("num_items_global", c_i64),
        ("item_rows", c_vp),
        ("item_row_keys", c_vp),
        ("n_item_rows", c_i64),
        ("item_rows_capacity", c_i64),
        ("item_fwd_out", c_vp),
        ("item_fwd_in", c_vp),
        ("item_bwd_out", c_vp),
        ("item_bwd_in", c_vp),
        ("table_sumsq", c_vp),
        ("dense_grads", c_vp),
        # deferred exact AdamW(g = 0) on tables with last_step
        ("adam_history", c_vp),
        ("history_capacity", c_i32),
        ("replay_slices", c_i32),
        ("aux_stream", c_vp),
        ("item_categories", c_vp),
        ("num_categories", c_i64),
        ("major_category", c_i64),
        ("steps_applied", c_vp),
        ("in_batch", c_i32),
        ("inbatch_local", c_vp),
        ("inbatch_items", c_vp),
        ("inbatch_dp_all", c_vp),
        ("inbatch_dp", c_vp),
        ("table_g0_math", c_i32),
        ("item_slot", c_vp),
        ("cal_stats", c_vp),
        ("cal_scatter", c_vp),
        ("item_rows_ld", c_i64),
        # compact exchange rows (ttamm_exchange_compact_supported)
        ("exchange_counts", c_vp),
        ("exchange_counts_ld", c_i64),
        ("exchange_world", c_i32),
    ]


ABI_VERSION = 25  # ttamm.h TTAMM_ABI_VERSION
G0_EXACT = 0  # ttamm.h TTAMM_G0_EXACT
DENSE_ADAM = 0  # ttamm.h TTAMM_DENSE_ADAM
DENSE_SGD = 1  # ttamm.h TTAMM_DENSE_SGD
G0_FAST = 1  # ttamm.h TTAMM_G0_FAST

# ttamm.h TTAMM_PHASE_*
PHASE_ALL = 0
PHASE_SAMPLE = 1
PHASE_ITEM_FWD = 2
PHASE_USER_FWD = 4
PHASE_USER = 8
PHASE_ITEM_BWD = 16
PHASE_DENSE = 32
PHASE_INBATCH_SRC = 64
PHASE_INBATCH = 128
PHASE_SCORE = 256
PHASE_TOWERS_BWD = 512
PHASE_TABLES = 1024
PHASE_CAL_STATS = 2048
PHASE_CAL_SCATTER = 4096


# Symbol table: name -> (restype, argtypes).  tests/ check every one is exported and that this
# table covers every function declared in include/ttamm.h.
SIGNATURES = {
    "ttamm_abi_version": (ctypes.c_int, []),
    "ttamm_last_error": (ctypes.c_char_p, []),
    "ttamm_developer_build": (ctypes.c_int, []),
    "ttamm_train_step_workspace_size": (ctypes.c_size_t, [ctypes.POINTER(StepArgs)]),
    "ttamm_train_step": (ctypes.c_int, [ctypes.POINTER(StepArgs), c_vp]),
    "ttamm_dense_grad_floats": (c_i64, [ctypes.POINTER(StepArgs)]),
    "ttamm_exchange_compact_supported": (ctypes.c_int, [ctypes.POINTER(StepArgs)]),
    "ttamm_adam_history_entry_bytes": (ctypes.c_size_t, []),
    "ttamm_retrieval_topk_workspace_size": (ctypes.c_size_t, [c_i64, c_i64, c_i32, c_i32]),
    "ttamm_normalize_rows": (ctypes.c_int, [c_vp, c_i64, c_i32, c_i64, c_vp]),
    "ttamm_to_bf16": (ctypes.c_int, [c_vp, c_i64, c_i32, c_i64, c_vp, c_i64, c_vp]),
    "ttamm_to_planes": (ctypes.c_int, [c_vp, c_i64, c_i32, c_i64, c_vp, c_i64, c_vp]),
    "ttamm_stream_create_cu_limited": (ctypes.c_int, [c_i32, ctypes.POINTER(c_vp)]),
    "ttamm_stream_destroy": (ctypes.c_int, [c_vp]),
    "ttamm_route_scratch_bytes": (ctypes.c_size_t, [c_i64, c_i32]),
    "ttamm_route_rows": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_i64,
                                        c_vp, c_vp,
                                        ctypes.c_size_t, c_vp]),
    "ttamm_epoch_batch": (ctypes.c_int, [c_vp, c_vp, c_i64, ctypes.c_uint64, c_i64, c_i32, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "ttamm_candidate_topk": (
        ctypes.c_int,
        [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp],
    ),
    "ttamm_retrieval_topk": (
        ctypes.c_int,
        [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp],
    ),
    "ttamm_flush_tables": (ctypes.c_int, [ctypes.POINTER(StepArgs), c_vp]),
    "ttamm_gather_rows": (ctypes.c_int, [c_vp, c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "ttamm_tower_forward_workspace_size": (ctypes.c_size_t, [ctypes.POINTER(Tower), c_i64]),
    "ttamm_tower_forward": (
        ctypes.c_int,
        [ctypes.POINTER(Tower), c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, ctypes.c_size_t, c_vp],
    ),
    "ttamm_tower_grad_floats": (ctypes.c_size_t, [ctypes.POINTER(Tower)]),
    "ttamm_tower_train_workspace_size": (ctypes.c_size_t, [ctypes.POINTER(Tower), c_i64]),
    "ttamm_tower_train_forward": (
        ctypes.c_int,
        [ctypes.POINTER(Tower), c_vp, c_vp, c_i64, c_vp, ctypes.c_uint64, ctypes.c_uint64, c_vp, c_vp,
         ctypes.c_size_t, c_vp],
    ),
    "ttamm_tower_train_backward": (
        ctypes.c_int,
        [ctypes.POINTER(Tower), c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp],
    ),
    "ttamm_scatter_add_rows": (
        ctypes.c_int,
        [c_vp, c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, ctypes.c_float, c_i64, c_vp],
    ),
    "ttamm_mimic_augment": (ctypes.c_int, [c_vp, c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "ttamm_mse_loss": (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "ttamm_sample_negatives": (
        ctypes.c_int,
        [c_vp, c_i64, c_i32, c_i64, c_vp, c_vp, c_i64, c_u64, c_u64, c_i64, c_vp, c_vp, c_vp],
    ),
    "ttamm_check_rows": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "ttamm_coalesce_workspace_bytes": (ctypes.c_size_t, [c_i64, c_i64]),
    "ttamm_coalesce_rows": (
        ctypes.c_int,
        [c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp],
    ),
    "ttamm_sparse_adam_rows": (
        ctypes.c_int,
        [c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_i64, c_d, c_d, c_d, c_d, c_i64, c_vp],
    ),
    "ttamm_adamw_dense": (
        ctypes.c_int,
        [c_vp, c_vp, c_vp, c_vp, c_i64, c_d, c_d, c_d, c_d, c_d, c_i32, c_i64, c_vp],
    ),
    "ttamm_inbatch_workspace_size": (ctypes.c_size_t, [c_i64, c_i64, c_i32]),
    "ttamm_inbatch_bce": (
        ctypes.c_int,
        [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64, ctypes.c_float, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp,
         ctypes.c_size_t, c_vp],
    ),
}

_lib: Optional[ctypes.CDLL] = None


def library_path() -> Path:
    override = os.environ.get("TTAMM_LIBRARY")
    return Path(override) if override else LIB_PATH


def load() -> ctypes.CDLL:
    """Load libttamm.so.  Raises RuntimeError if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not path.exists():
        raise RuntimeError(
            f"libttamm.so not found at {path}; build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(make -C two-tower-augmented-with-adaptive-mimic-mechanism_amd/csrc)"
        )
    lib = ctypes.CDLL(str(path))
    for name, (restype, argtypes) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = restype
        fn.argtypes = argtypes
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc == TTAMM_OK:
        return
    msg = load().ttamm_last_error().decode("utf-8", "replace")
    if rc == TTAMM_E_INVALID:
        raise ValueError(msg)
    raise RuntimeError(msg)


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def check_index_range(idx: torch.Tensor, rows: int) -> None:
    """nn.Embedding's check (encoders.py:222-223 runs F.embedding): an id outside [0, rows)
    raises IndexError("index out of range in self").  One device->host read; used by the module
    (eval) entry points, while the fused step reports bad ids through its status word."""
    if idx.numel() == 0:
        return
    lo, hi = torch.aminmax(idx.reshape(-1))
    if int(lo) < 0 or int(hi) >= rows:
        raise IndexError("index out of range in self")


def require_rocm(t: torch.Tensor, what: str) -> None:
    """The product path runs only on a ROCm device; CPU tensors are rejected (no fallback)."""
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{what}: ttamm executes on an MI355X (ROCm) device; got a tensor on '{t.device}'. "
            "Move the model and inputs to the GPU."
        )
