"""Kernel name -> (family, role): the one table tools/traffic_table.py, tools/rocprof_summary.py and
tools/step_trace.py share, so a new kernel cannot be counted by one tool and dropped by another.

A family is what one C-ABI call's op-log entry stands for (bench.py writes the op log through
ldmseg.ops.native's launch profiler):
  igemm        ldm_conv2d (tile / halo / wide / ring / big / ars kernels), ldm_conv_in, ldm_feedforward,
               ldm_transformer_in, ldm_unet_tail; the split-K reductions attach to the op before them
  attention    ldm_attention(_ws / _fp8); the split-KV merge attaches to the op before it, the fp8
               K/V quantisation to the op after it
  group_norm   ldm_group_norm (gn_apply / gn_small); gn_stats (no producer statistics) is "pre"
  layer_norm   ldm_layer_norm
  linear_rows  ldm_linear_rows (time-embedding MLP on a few rows)
Roles: "p" primary (one per op-log entry), "post" belongs to the op before it, "pre" to the op
after it.  Kernels outside every family (layout glue, torch fills / copies) are None.
"""
import re

KINDS = [
    ("igemm", r"(igemm_kernel|igemm_big_kernel|conv3_halo_kernel|gemm_ars2?_kernel|gemm_wide_kernel|"
              r"gemm_ring_kernel|conv_in_kernel)<|feedforward_kernel|transformer_in_kernel|unet_tail_kernel", "p"),
    ("igemm", r"splitk_(epilogue|gn)_kernel<", "post"),
    ("attention", r"attn(32|_d40|_f8)?_kernel<", "p"),
    ("attention", r"attn_kv_combine", "post"),
    ("attention", r"attn_f8_prep", "pre"),
    ("group_norm", r"gn_apply|gn_small", "p"),
    ("group_norm", r"gn_stats", "pre"),
    ("layer_norm", r"ln_kernel<", "p"),
    ("linear_rows", r"linear_rows_kernel", "p"),
]


def kind_of(name):
    """(family, role) of a kernel name, or (None, None)."""
    for fam, rx, role in KINDS:
        if re.search(rx, name):
            return fam, role
    return None, None
