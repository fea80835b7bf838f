"""ctypes binding of librecsys_hip.so (C ABI: include/recsys_hip.h).

The library is loaded on first use.  There is no fallback: if the .so is
missing or a call returns non-zero, a RuntimeError is raised.  ``import torch``
happens first so the process's single HIP runtime is torch's (the .so links
against ``libamdhip64.so.7``, which the dynamic loader resolves to the copy
torch already mapped).
"""
import ctypes as C
import os

import torch  # noqa: F401  (must be loaded before the HIP library)

PKG = os.path.dirname(os.path.abspath(__file__))
# RS_LIB_VARIANT=x loads librecsys_hip.x.so from the package directory instead (A/B timing of two builds in one
# GPU session; the default is the in-tree build)
LIB_PATH = os.path.join(PKG, "librecsys_hip.so" if not os.environ.get("RS_LIB_VARIANT")
                        else f"librecsys_hip.{os.environ['RS_LIB_VARIANT']}.so")

F32, BF16 = 0, 1

i32, i64, u64, f32, f64, vp = C.c_int, C.c_int64, C.c_uint64, C.c_float, C.c_double, C.c_void_p


class Epilogue(C.Structure):
    """Mirror of ``rs_epilogue`` (include/recsys_hip.h)."""
    _fields_ = [
        ("bias", vp), ("alpha", f32), ("act", i32),
        ("aux", vp), ("aux_out", vp), ("ldaux", i64),
        ("drop_p", f32), ("drop_seed", u64), ("seed_base", vp), ("drop_ld", i64),
        ("resid", vp), ("ldres", i64),
        ("rowmask_ids", vp), ("accumulate", i32),
        ("post_drop_p", f32), ("post_drop_seed", u64), ("rows_dev", vp),
    ]


class WgradProblem(C.Structure):
    """Mirror of ``rs_wgrad_problem``."""
    _fields_ = [("dY", vp), ("lddy", i64), ("X", vp), ("ldx", i64), ("N", i64), ("K", i64), ("dW", vp), ("db", vp)]


class ReduceSegment(C.Structure):
    """Mirror of ``rs_reduce_segment``."""
    _fields_ = [("src", vp), ("stride", i64), ("splits", i64), ("n", i64), ("out", vp)]


ACT_NONE, ACT_RELU, ACT_GELU, ACT_RELU_BWD, ACT_GELU_BWD = 0, 1, 2, 3, 4

# name -> argtypes (all return int)
SIGNATURES = {
    "rs_gemm": [i32, i32, i32, i64, i64, i64, vp, i64, vp, i64, vp, i64, i32, C.POINTER(Epilogue), i32, vp, vp],
    "rs_gemm_ln": [i64, i64, i64, vp, i64, vp, vp, f32, vp, i64, vp, i64, C.POINTER(Epilogue), vp, i64, vp, vp, vp],
    "rs_reduce_slabs": [vp, i32, i64, vp, i32, vp],
    "rs_reduce_slabs2": [vp, i32, i64, vp, i64, vp, i32, vp],
    "rs_linear_wgrad": [i32, i64, i64, i64, vp, i64, vp, i64, vp, vp, i32, i32, vp, vp, vp],
    "rs_colsum": [i32, vp, i64, i64, i64, vp, vp, i32, vp],
    "rs_embed_fwd": [i32, i32, vp, i64, i64, vp, vp, i64, f32, f32, u64, vp, vp, vp],
    "rs_embed_bwd": [i32, i32, vp, i64, i64, vp, i64, f32, f32, u64, vp, vp, vp, i32, vp],
    "rs_layernorm_fwd": [i32, i32, vp, i64, i64, i64, vp, vp, f32, vp, i64, vp, vp, vp],
    "rs_layernorm_bwd_nparts": [i32, i64, i64],
    "rs_layernorm_bwd_drop": [i32, i32, vp, i64, vp, i64, i64, i64, vp, vp, vp, f32, vp, i64, i32, vp, vp, vp, f32,
                              u64, u64, vp, vp, vp, vp],
    "rs_layernorm_bwd": [i32, i32, vp, i64, vp, i64, i64, i64, vp, vp, vp, f32, vp, i64, i32, vp, vp, vp, vp],
    "rs_attn_fwd": [i32, i64, i64, i64, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, f32, i32, vp, f32, u64, vp, vp],
    "rs_attn_row_delta": [i32, i64, i64, i64, i64, vp, i64, vp, i64, vp, vp],
    "rs_attn_bwd": [i32, i64, i64, i64, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, vp, i64, vp, i64,
                    vp, i64, f32, i32, vp, f32, u64, vp, vp, vp],
    "rs_sampled_logits_fwd": [i32, vp, i64, i64, vp, vp, vp, vp, vp, vp],
    "rs_sampled_logits_bwd": [i32, vp, i64, i64, vp, vp, vp, vp, vp, vp, i32, vp, vp],
    "rs_bce_fwd": [vp, vp, vp, i64, vp, vp, vp, vp],
    "rs_bce_bwd": [vp, vp, vp, i64, vp, vp, vp, vp, vp],
    "rs_ce_fwd": [vp, i64, i64, i64, vp, vp, vp, vp, vp, vp],
    "rs_ce_bwd": [i32, vp, i64, i64, i64, vp, vp, vp, vp, vp, i64, vp, vp],
    "rs_compact_rows": [vp, i64, i64, vp, vp, vp, vp],
    "rs_gather_rows": [i32, vp, i64, i64, vp, vp, i64, vp, i64, vp, vp, vp],
    "rs_scatter_rows": [i32, vp, i64, i64, vp, i64, vp, i64, vp],
    "rs_candidate_scores": [i32, vp, i64, i64, i64, vp, vp, vp, i64, i64, vp, vp],
    "rs_gemm_n256_splits": [i64, i64],
    "rs_gemm_n256": [i32, i64, i64, vp, i64, vp, i64, vp, i64, i32, i64, vp, vp, vp],
    "rs_adam_prepare": [vp, vp, vp, vp, vp],
    "rs_adam_step": [i64, vp, vp, vp, vp, vp, vp, vp, i32, vp],
    "rs_adam_step_wg": [i64, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp],
    "rs_adam_step_marked": [i64, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, vp, i64, i64, i32, vp],
    "rs_graph_upload": [vp, vp],
    "rs_adam_prepare_step": [i64, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp, i32, i64, vp, vp],
    "rs_adam_prepare_step_loss": [i64, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp, i32, i64, vp, vp, vp, vp],
    "rs_adam_prepare_step_marked": [i64, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp, i32, i64, vp, vp, vp, vp, vp,
                                    i64, i64, i32, vp],
    "rs_cast_bf16": [i64, vp, vp, vp],
    "rs_l2_penalty": [vp, vp, vp, i64, f32, vp, vp, vp, vp],
    "rs_dropout_rowmask": [i32, vp, i64, i64, i64, f32, u64, vp, i64, vp, vp, vp, vp],
    "rs_dropout2": [i32, vp, i64, i64, i64, f32, u64, u64, vp, i64, vp, vp, vp],
    "rs_vocab_ce_ws_numel": [i64, i64],
    "rs_vocab_ce_fwd": [i64, i64, i64, vp, i64, vp, i64, vp, vp, vp, vp, vp, vp, vp],
    "rs_vocab_ce_bwd": [i64, i64, i64, vp, i64, vp, i64, vp, vp, vp, vp, vp, vp, vp, i64, vp],
    "rs_vocab_head_supported": [i64],
    "rs_vocab_head_fwd": [i64, i64, i64, vp, i64, vp, i64, vp, vp, vp, vp, vp, vp, vp],
    "rs_vocab_head_bwd": [i64, i64, i64, vp, i64, vp, i64, vp, vp, vp, vp, vp, vp, vp, i64, i64, vp],
    "rs_vocab_shard_lse": [i64, i64, i64, vp, i64, vp, i64, vp, vp, vp, vp, vp],
    "rs_vocab_shard_label_logits": [i64, i64, vp, i64, vp, i64, vp, vp, i64, i64, vp, vp],
    "rs_vocab_shard_combine": [i32, i64, vp, vp, vp, vp, vp, vp],
    "rs_seed_advance": [vp, vp],
    "rs_sas_block_parts": [i64],
    "rs_touched_rows_ws_numel": [i64],
    "rs_touched_rows": [vp, i64, i64, vp, vp, vp, vp, vp],
    "rs_rows_pack": [vp, i64, i64, vp, vp, vp, i64, vp],
    "rs_rows_unpack": [vp, i64, i64, vp, vp, vp],
    "rs_sas_block_in": [i64, i64, vp, i64, vp, vp, f32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
    "rs_sas_block_in_count_parts": [i64],
    "rs_sas_block_grid": [i64],
    "rs_sas_block_out_head": [i64, i64, vp, vp, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32,
                              u64, u64, vp, vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
    "rs_sas_block_in_embed": [i64, i64, vp, i64, vp, vp, f32, f32, u64, vp, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp,
                              vp, vp, vp, vp, vp, vp],
    "rs_sas_block_out": [i64, i64, vp, vp, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32,
                         u64, u64, vp, vp],
    "rs_sas_block_out_bwd": [i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, u64, u64,
                             vp, vp],
    "rs_sas_block_out_bwd_delta": [i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, u64,
                                   u64, vp, vp, vp, vp],
    "rs_sas_block_in_bwd": [i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
    "rs_wgrad_grouped": [i32, C.POINTER(WgradProblem), i64, i64, vp, i64, i32, C.POINTER(ReduceSegment), vp],
    "rs_reduce_segments": [i32, C.POINTER(ReduceSegment), i32, vp],
    "rs_wgrad_grouped_slab_numel": [i32, C.POINTER(WgradProblem), i64, i64],
    "rs_wgrad_grouped_tile": [i32, C.POINTER(WgradProblem)],
    "rs_wgrad_grouped_tile_max": [i32, C.POINTER(WgradProblem), i32],
    "rs_wgrad_grouped_max": [i32, C.POINTER(WgradProblem), i64, i64, vp, i64, i32, C.POINTER(ReduceSegment), i32, vp],
    "rs_item_index_ws_bytes": [i32, i64, i64, i64],
    "rs_item_index_build": [i32, vp, vp, vp, i64, i64, i64, vp, i64, vp],
    "rs_item_index_layout": [i32, i64, i64, i64, C.POINTER(i64)],
    "rs_sas_head_fwd": [i64, i64, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
    "rs_sas_head_finish": [i64, vp, vp, vp, vp],
    "rs_sas_head_bwd": [i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
    "rs_item_grad": [vp, i32, i64, i64, i64, vp, f32, f32, u64, vp, vp, vp, vp, vp, vp],
    "rs_item_grad_marked": [vp, i32, i64, i64, i64, vp, f32, f32, u64, vp, vp, vp, vp, vp, vp, vp, vp],
    "rs_item_grad_f32": [vp, i32, i64, i64, i64, vp, f32, f32, u64, vp, vp, vp, vp, vp, vp],
    "rs_wgrad_grouped_pos": [i32, C.POINTER(WgradProblem), i64, i64, vp, i64, i32, C.POINTER(ReduceSegment),
                             vp, i64, vp, i64, f32, u64, vp, vp, vp],
    "rs_wgrad_grouped_pos_stats": [i32, C.POINTER(WgradProblem), i64, i64, vp, i64, i32, C.POINTER(ReduceSegment),
                                   vp, i64, vp, i64, f32, u64, vp, vp, vp, i64, vp, vp, vp, vp],
    "rs_transpose_bf16": [i64, vp, i64, vp, vp, vp],
    "rs_sas_sample": [vp, vp, i64, i64, i64, i64, vp, u64, vp, vp, vp, vp],
    "rs_bert_mask": [vp, vp, i64, i64, i64, i64, f64, vp, vp, u64, vp, vp, vp],
    "rs_sas_sample_draws": [vp, vp, i64, i64, i64, i64, vp, u64, vp, vp, vp, vp, vp],
    "rs_bert_mask_draws": [vp, vp, i64, i64, i64, i64, f64, vp, vp, u64, vp, vp, vp, vp],
    "rs_splitk_scatter_rows": [i32, vp, i32, i64, i64, vp, i64, vp, i64, vp],
    "rs_rank_metrics": [vp, vp, i64, i64, i32, vp, vp, vp, vp],
    "rs_kernel_stamps": [vp, vp, i32],
    "rs_kernel_stamp_count": [],
    "rs_kernel_stamp_kinds": [C.POINTER(i32), i32],
    "rs_wall_clock_khz": [C.POINTER(i32)],
    "rs_attn_bwd_plan": [i64, i64, i64, i32, vp, C.POINTER(i32)],
    "rs_abi_version": [],
}

RESTYPES = {"rs_wgrad_grouped_slab_numel": C.c_int64, "rs_sas_block_parts": C.c_int64,
            "rs_touched_rows_ws_numel": C.c_int64, "rs_item_index_ws_bytes": C.c_int64,
            "rs_vocab_ce_ws_numel": C.c_int64,
            "rs_sas_block_in_count_parts": C.c_int64,
            "rs_sas_block_grid": C.c_int64, "rs_layernorm_bwd_nparts": C.c_int64}

_lib = None


def lib():
    """Load (once) and return the native library; raise if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"librecsys_hip.so not found at {LIB_PATH}; build it with "
                "`python recommender-baseline-model_amd/build.py` (there is no CPU fallback)")
        h = C.CDLL(LIB_PATH)
        for name, argt in SIGNATURES.items():
            fn = getattr(h, name)
            fn.argtypes = argt
            fn.restype = RESTYPES.get(name, C.c_int)
        _lib = h
    return _lib


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream
