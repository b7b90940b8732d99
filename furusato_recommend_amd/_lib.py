"""ctypes binding of libmirec.so (the C ABI declared in include/mirec.h).

This is the Python side of the drop-in boundary: every device call goes
through these entry points with raw device pointers and the current HIP
stream.  There is no CPU fallback — if the shared library is missing the
import fails loudly (build it with ``python -c "import __graft_entry__ as g;
g.build()"`` or ``make -C furusato_recommend_amd/csrc``).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_float, c_int, c_int32, c_int64,
                    c_size_t, c_uint64, c_void_p, c_char_p)

import torch  # noqa: F401  (binds libmirec to torch's HIP runtime: same SONAME)

_HERE = os.path.dirname(os.path.abspath(__file__))
# MIREC_LIB selects an alternative build for A/B timing (tools/bench_variants.py)
LIB_PATH = os.environ.get("MIREC_LIB") or os.path.join(_HERE, "libmirec.so")

MIREC_OK = 0
IN_PRESCALED, IN_RAW, IN_SPARSE, IN_NONE = 0, 1, 2, 3
SUPPORTED_DIMS = (4, 8, 16, 32, 64, 128, 256)


class MirecError(RuntimeError):
    pass


class CSR(Structure):
    """mirec_csr_t (include/mirec.h)."""
    _fields_ = [
        ("rowptr", c_void_p), ("col", c_void_p), ("dinv", c_void_p),
        ("n_rows", c_int64), ("nnz", c_int64), ("split", c_int32),
        ("_pad", c_int32), ("n_long", c_int64), ("n_seg", c_int64),
        ("long_rows", c_void_p), ("long_segptr", c_void_p),
        ("seg_row", c_void_p), ("seg_beg", c_void_p),
        ("col_sorted", c_void_p), ("n_sorted", c_int64),
    ]


class AdamH(Structure):
    """mirec_adam_hparams_t."""
    _fields_ = [
        ("one_minus_beta1", c_float), ("beta2", c_float),
        ("one_minus_beta2", c_float), ("neg_step_size", c_float),
        ("bc2_sqrt", c_float), ("eps", c_float),
    ]


class Prop(Structure):
    """mirec_prop_t."""
    _fields_ = [
        ("dim", c_int32), ("in_mode", c_int32), ("x_in", c_void_p),
        ("slot", c_void_p), ("seed_in", c_void_p), ("seed", c_void_p),
        ("addend", c_void_p), ("seed2", c_void_p), ("divisor", c_float),
        ("_pad", c_float), ("out", c_void_p), ("xs_out", c_void_p),
        ("param", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
        ("adam", AdamH), ("partial", c_void_p), ("row_mask", c_void_p),
        ("in_mask", c_void_p), ("out_mask", c_void_p), ("row_list", c_void_p),
        ("row_count", c_void_p),
        ("row_list_cap", c_int64), ("narrow_max", c_int32), ("_pad2", c_int32),
        ("wide_list", c_void_p), ("wide_count", c_void_p),
    ]


class RowGradGroup(Structure):
    """mirec_row_grad_group_t (one group of table-gradient row contributions)."""
    _fields_ = [
        ("ids", c_void_p), ("grad_out", c_void_p), ("n_targets", c_int64), ("k", c_int32),
        ("mean", c_int32), ("dropout_p", c_float), ("_pad", c_int32), ("seed", c_uint64),
    ]


TABLE_GRAD_MAX_GROUPS = 8


class RowBlock(Structure):
    """mirec_row_block_t (one source block of mirec_owner_sum)."""
    _fields_ = [("ids", c_void_p), ("rows", c_void_p), ("n", c_int64)]

# name -> (restype, argtypes); the single source of truth for the exports
# test (tests/test_abi.py checks these against include/mirec.h).
SIGNATURES = {
    "mirec_strerror": (c_char_p, [c_int]),
    "mirec_abi_version": (c_int, []),
    "mirec_last_hip_error": (c_int, []),
    "mirec_struct_sizes": (c_int, [POINTER(c_size_t), POINTER(c_size_t), POINTER(c_size_t)]),
    "mirec_csr_bipartite": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64,
                                    c_void_p, c_void_p, c_void_p]),
    "mirec_csr_sort_rows": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "mirec_csr_from_coo": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                                   c_void_p, c_void_p]),
    "mirec_parse_interactions": (c_int, [c_void_p, c_int64, c_int64, c_int32, POINTER(c_int64),
                                         POINTER(c_int64), POINTER(c_int64), POINTER(c_int64),
                                         c_void_p, c_void_p, c_void_p]),
    "mirec_csr_long_rows": (c_int, [c_void_p, c_int64, c_int32, POINTER(c_int64),
                                    POINTER(c_int64), c_void_p, c_void_p, c_void_p,
                                    c_void_p]),
    "mirec_propagate": (c_int, [POINTER(CSR), POINTER(Prop), c_void_p]),
    "mirec_prescale": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    "mirec_shard_pack": (c_int, [c_void_p, c_int64, c_int32, c_int32, c_int32, c_int64, c_int64,
                                 c_void_p, c_void_p]),
    "mirec_shard_unpack": (c_int, [c_void_p, c_int64, c_int32, c_int32, c_int32, c_int64,
                                   c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mirec_frontier": (c_int, [POINTER(CSR), c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                               c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_int32, c_void_p]),
    "mirec_mask_compact_pair": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p]),
    "mirec_small_sort_workspace": (c_int, [c_int64, POINTER(c_size_t)]),
    "mirec_small_sort_pairs": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p,
                                       c_size_t, c_void_p]),
    "mirec_mask_compact": (c_int, [POINTER(CSR), c_void_p, c_int32, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_int32, c_void_p]),
    "mirec_distinct_rows_workspace": (c_int64, [c_int64]),
    "mirec_distinct_rows": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p,
                                    c_void_p, c_void_p, c_size_t, c_void_p]),
    "mirec_distinct_rows_unseen": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "mirec_stamped_rows": (c_int, [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p,
                                   c_void_p, c_size_t, c_void_p]),
    "mirec_scatter_rows": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    "mirec_owner_sum_workspace": (c_int64, [c_int32, c_int64]),
    "mirec_owner_sum": (c_int, [POINTER(RowBlock), c_int32, c_int64, c_int64, c_int32, c_void_p,
                                c_size_t, c_void_p, c_void_p]),
    "mirec_gather_rows_counted": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                          c_void_p, c_void_p]),
    "mirec_route_pack": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int32, c_int32, c_int64,
                                 c_void_p, c_void_p]),
    "mirec_gather_rows_routed": (c_int, [c_void_p, c_int64, c_void_p, c_int32, c_int32, c_int64,
                                         c_int32, c_void_p, c_void_p]),
    "mirec_bpr_forward": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int32, c_int64,
                                  c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    "mirec_bpr_loss": (c_int, [c_void_p, c_void_p, c_int64, c_float, c_void_p, c_void_p,
                               c_void_p]),
    "mirec_bpr_seed_workspace": (c_int, [c_int64, c_int64, POINTER(c_size_t)]),
    "mirec_bpr_seed": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int32, c_int64,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_float, c_float, c_int32, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_size_t, c_void_p]),
    "mirec_bpr_seed_reset": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "mirec_seed_dense": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                 c_int32, c_void_p, c_int32, c_void_p]),
    "mirec_seed_pack": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    "mirec_seed_merge_workspace": (c_int, [c_int64, c_int64, POINTER(c_size_t)]),
    "mirec_seed_merge": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int64,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                 c_void_p]),
    "mirec_adam_multi": (c_int, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 POINTER(AdamH), c_void_p]),
    "mirec_adam_dense": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                 POINTER(AdamH), c_void_p]),
    "mirec_adam_multi_dev": (c_int, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_void_p]),
    "mirec_adam_dense_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p,
                                     c_void_p]),
    "mirec_sample_fanout": (c_int, [POINTER(CSR), c_void_p, c_int64, c_int32, c_uint64,
                                    c_uint64, c_void_p, c_void_p]),
    "mirec_pack_seed_nodes": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                                      c_void_p]),
    "mirec_sample_fanout_norep": (c_int, [POINTER(CSR), c_void_p, c_int64, c_int32, c_uint64,
                                          c_uint64, c_void_p, c_void_p]),
    "mirec_gather_rows": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    "mirec_scatter_add_rows": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_void_p,
                                       c_void_p]),
    "mirec_fanout_mean": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_float,
                                  c_uint64, c_void_p, c_void_p]),
    "mirec_fanout_mean_bwd": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_float,
                                      c_uint64, c_void_p, c_void_p]),
    "mirec_fanout_mean_gather": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                         c_float, c_uint64, c_void_p, c_void_p]),
    "mirec_fanout_mean_gather_bwd": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                             c_float, c_uint64, c_void_p, c_void_p]),
    "mirec_fanout_mean_gather_bwd_sorted_workspace": (c_int, [c_int64, c_int32, c_int32,
                                                              POINTER(c_size_t)]),
    "mirec_fanout_mean_gather_bwd_sorted": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                                    c_float, c_uint64, c_int32, c_void_p,
                                                    c_void_p, c_size_t, c_void_p]),
    "mirec_row_grad_group_size": (c_int64, []),
    "mirec_table_grad_workspace": (c_int, [POINTER(RowGradGroup), c_int32, c_int32, c_int32,
                                           POINTER(c_size_t)]),
    "mirec_table_grad_sorted": (c_int, [POINTER(RowGradGroup), c_int32, c_int32, c_int32,
                                        c_void_p, c_void_p, c_int32, c_void_p, c_size_t,
                                        c_void_p]),
    "mirec_table_grad_sorted_rows": (c_int, [POINTER(RowGradGroup), c_int32, c_int32, c_int32,
                                             c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_size_t, c_void_p]),
    "mirec_table_grad_atomic": (c_int, [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                        c_int32, c_void_p]),
    "mirec_table_grad_dense": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int32,
                                       c_int64, c_int32, c_void_p, c_void_p]),
    "mirec_adam_table_sumsq_floats": (c_int64, [c_int64, c_int32]),
    "mirec_owner_adam": (c_int, [POINTER(RowBlock), c_int32, c_int64, c_int64, c_int32, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_int64, POINTER(AdamH), c_void_p,
                                 c_void_p, c_void_p, c_size_t, c_void_p]),
    "mirec_adam_table": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p,
                                 c_void_p, c_int32, c_int64, c_int32, POINTER(AdamH), c_void_p,
                                 c_void_p, c_void_p]),
    "mirec_adam_table_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p,
                                     c_void_p, c_int32, c_int64, c_int32, c_void_p, c_void_p,
                                     c_void_p, c_void_p]),
    "mirec_norm_coef": (c_int, [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_void_p,
                                c_void_p]),
    "mirec_attention_fwd": (c_int, [c_void_p, c_int64, c_int32, c_int32, c_int32, c_void_p,
                                    c_void_p]),
    "mirec_attention_bwd": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32,
                                    c_void_p, c_void_p]),
    "mirec_attention_varlen_fwd": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                           c_void_p, c_void_p]),
    "mirec_attention_varlen_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                           c_int32, c_void_p, c_void_p]),
    "mirec_attention_bucketed_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int32, c_int32,
                                             c_void_p, c_void_p]),
    "mirec_attention_bucketed_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                             c_int32, c_void_p, c_void_p]),
    "mirec_attention_wave_supported": (c_int, [c_int32]),
    "mirec_attention_ordered_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                            c_int32, c_void_p, c_void_p]),
    "mirec_attention_ordered_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                            c_int32, c_int32, c_void_p, c_void_p]),
    "mirec_attention_length_order": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                             c_int64, c_int32, c_void_p]),
    "mirec_attention_packed_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                           c_int32, c_int32, c_void_p, c_int64, c_void_p]),
    "mirec_attention_packed_bwd_lse": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_void_p, c_int64, c_int32, c_int32, c_void_p,
                                               c_int64, c_void_p]),
    "mirec_attention_wave_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                         c_int32, c_void_p, c_void_p, c_int64, c_void_p]),
    "mirec_attention_wave_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_int64, c_int32, c_int32, c_int32, c_void_p,
                                         c_void_p, c_void_p]),
    "mirec_resnorm_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                  c_int32, c_int32, c_float, c_uint64, c_void_p, c_float,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mirec_gemm_resnorm": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_int32, c_float, c_uint64,
                                   c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p]),
    "mirec_gemm_nn_resnorm_bwd_work_floats": (c_int64, [c_int64, c_int32]),
    "mirec_gemm_nn_resnorm_bwd": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_int32, c_float, c_uint64, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p]),
    "mirec_resnorm_reduce_partials": (c_int, [c_void_p, c_int64, c_int32, c_void_p, c_void_p,
                                              c_void_p, c_void_p]),
    "mirec_resnorm_work_floats": (c_int64, [c_int64, c_int32]),
    "mirec_segment_mean": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_void_p,
                                   c_void_p]),
    "mirec_segment_mean_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int32,
                                       c_void_p, c_void_p]),
    "mirec_bpr_rows_loss": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_void_p,
                                    c_float, c_void_p, c_void_p, c_void_p]),
    "mirec_bpr_rows_loss_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                        c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p]),
    "mirec_slice_norms_work_floats": (c_int64, []),
    "mirec_slice_norms": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "mirec_norm_terms": (c_int, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
                                 c_int32, c_void_p, c_void_p, c_void_p]),
    "mirec_norm_terms_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                     c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "mirec_norm_terms_bwd_acc": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                         c_void_p, c_void_p, c_void_p]),
    "mirec_seq_sample": (c_int, [c_void_p, c_int64, c_void_p, c_int32, c_void_p, c_int64,
                                 c_uint64, c_uint64, c_void_p, c_void_p]),
    "mirec_seq_pack": (c_int, [c_void_p, c_int64, c_void_p, c_int32, c_void_p, c_void_p,
                               c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p]),
    "mirec_zero_tail_rows": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int32, c_void_p]),
    "mirec_gemm_nt": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32,
                              c_void_p]),
    "mirec_gemm_nn_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                 c_int64, c_int32, c_int32, c_void_p]),
    "mirec_gemm_nt_ex": (c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_int32, c_int32, c_int64, c_int32, c_int32,
                                 c_void_p]),
    "mirec_gemm_tn_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                 c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p]),
    "mirec_gemm_tn_work_floats": (c_int64, [c_int64, c_int32, c_int32]),
    "mirec_col_sums_work_floats": (c_int64, [c_int64, c_int32]),
    "mirec_col_sums": (c_int, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p]),
    "mirec_gemm_tn": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32,
                              c_void_p, c_void_p]),
    "mirec_resnorm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_int64, c_int32, c_int32, c_float, c_uint64, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p]),
    "mirec_score_topk_workspace": (c_int64, [c_int64, c_int64, c_int32]),
    "mirec_score_topk": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int32, c_void_p,
                                 c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p,
                                 c_size_t, c_void_p]),
    "mirec_topk_masked": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_int64,
                                  c_int32, c_void_p, c_void_p, c_void_p]),
    "mirec_bpr_sample_capped_workspace": (c_int, [c_int64, c_int64, POINTER(c_size_t)]),
    "mirec_bpr_sample_capped": (c_int, [POINTER(CSR), c_int64, c_int64, c_int64, c_int32,
                                        c_uint64, c_uint64, c_int32, c_int32, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_size_t, c_void_p]),
    "mirec_bpr_sample": (c_int, [POINTER(CSR), c_int64, c_int64, c_int64, c_uint64,
                                 c_uint64, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p]),
    "mirec_bpr_sample_ex": (c_int, [POINTER(CSR), c_void_p, c_int64, c_int64, c_int64, c_uint64,
                                    c_uint64, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p]),
    "mirec_bpr_sample_capped_ex": (c_int, [POINTER(CSR), c_void_p, c_int64, c_int64, c_int64,
                                           c_int32, c_uint64, c_uint64, c_int32, c_int32, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_size_t, c_void_p]),
    "mirec_pos_cdf_build": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "mirec_cpu_bpr_sample": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                     c_int64, c_uint64, c_uint64, c_int32, c_int32, c_void_p,
                                     c_void_p, c_void_p, c_void_p, c_int32]),
    "mirec_cpu_bpr_sample_capped": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                            c_int64, c_int64, c_int32, c_uint64, c_uint64,
                                            c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_int32]),
    "mirec_cpu_bpr_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                   c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_float,
                                   c_void_p, c_void_p, c_int32]),
    "mirec_cpu_bpr_grad": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int64, c_void_p,
                                   c_void_p, c_void_p, c_int64, c_float, c_float, c_void_p,
                                   c_int32]),
    "mirec_cpu_adam": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p,
                               c_int32]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: the HIP engine is not built. Run "
            "`make -C furusato_recommend_amd/csrc` (or __graft_entry__.build()). "
            "There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mirec_abi_version() != 1:
        raise ImportError("libmirec.so ABI version mismatch")
    sizes = [c_size_t(0) for _ in range(3)]
    lib.mirec_struct_sizes(*(ctypes.byref(x) for x in sizes))
    want = (ctypes.sizeof(CSR), ctypes.sizeof(Prop), ctypes.sizeof(AdamH))
    if tuple(x.value for x in sizes) != want:
        raise ImportError(f"struct layout mismatch: lib {[x.value for x in sizes]} vs {want}")
    if lib.mirec_row_grad_group_size() != ctypes.sizeof(RowGradGroup):
        raise ImportError("struct layout mismatch: mirec_row_grad_group_t")
    return lib


lib = _load()


def check(rc: int, what: str = "") -> None:
    if rc != MIREC_OK:
        msg = lib.mirec_strerror(rc).decode()
        if rc == 3:
            msg += f" (hipError {lib.mirec_last_hip_error()})"
        raise MirecError(f"{what}: {msg}")


def ptr(t) -> int | None:
    """Device/host pointer of a tensor (None for None)."""
    return None if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    """The current HIP stream of ``device`` (default: the current device) —
    the raw handle straight from the C++ side: torch.cuda.current_stream()
    spends ~13 us of host time per call in device-index bookkeeping, and a
    GraphSAGE micro-batch makes ~230 of these calls."""
    if device is None:
        return _raw_stream(_cur_device())
    return torch.cuda.current_stream(device).cuda_stream


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_device = torch._C._cuda_getDevice


def adam_hparams(lr: float, beta1: float, beta2: float, eps: float, step: int) -> AdamH:
    """Per-step scalars of torch.optim.Adam (torch/optim/adam.py:534-547)."""
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    return AdamH(one_minus_beta1=1 - beta1, beta2=beta2, one_minus_beta2=1 - beta2,
                 neg_step_size=-(lr / bc1), bc2_sqrt=bc2 ** 0.5, eps=eps)
