"""ctypes binding of libsavqa.so (C ABI declared in include/savqa.h).

The library is built in-tree (structured-alignment-vqa_amd/libsavqa.so) by
`make -C structured-alignment-vqa_amd/csrc` or __graft_entry__.build(). There is no
fallback: every op raises if the library (or a HIP device) is missing.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsavqa.so")

c_i64 = C.c_int64
c_i32 = C.c_int32
c_u64 = C.c_uint64
c_f = C.c_float
c_p = C.c_void_p


class GemmDesc(C.Structure):
    _fields_ = [
        ("M", c_i64), ("N", c_i64), ("K", c_i64),
        ("A", c_p), ("lda", c_i64), ("a_trans", c_i32), ("prec", c_i32),
        ("a_rows", c_p),
        ("B", c_p), ("ldb", c_i64), ("b_trans", c_i32), ("_pad1", c_i32),
        ("b_rows", c_p),
        ("C", c_p), ("ldc", c_i64),
        ("c_group", c_i64), ("c_stride", c_i64), ("c_offset", c_i64),
        ("c_rows", c_p),
        ("bias", c_p),
        ("rowvec", c_p), ("ldrv", c_i64), ("rowvec_period", c_i64),
        ("resid", c_p), ("ldr", c_i64),
        ("mask", c_p), ("ldmask", c_i64), ("mask_arows", c_i64),
        ("rowscale", c_p),
        ("alpha", c_f), ("beta", c_f),
        ("relu", c_i32), ("atomic", c_i32), ("split_k", c_i32), ("_pad2", c_i32),
        ("colsum_a", c_p),
        ("ws", c_p), ("ws_elems", c_i64),
        ("b_planes", c_p),
    ]


class GemmLpDesc(C.Structure):
    """savqa_gemm_lp_desc (include/savqa.h)."""
    _fields_ = [
        ("M", c_i64), ("N", c_i64), ("K", c_i64),
        ("A", c_p), ("lda", c_i64), ("a_trans", c_i32), ("a_type", c_i32),
        ("a_rows", c_p),
        ("a_scale", c_p), ("lds_a", c_i64),
        ("B", c_p), ("ldb", c_i64), ("b_trans", c_i32), ("b_type", c_i32),
        ("b_scale", c_p), ("lds_b", c_i64),
        ("C", c_p), ("ldc", c_i64),
        ("Cb", c_p), ("ldcb", c_i64),
        ("c_group", c_i64), ("c_stride", c_i64), ("c_offset", c_i64),
        ("bias", c_p),
        ("rowvec", c_p), ("ldrv", c_i64), ("rowvec_period", c_i64),
        ("resid", c_p), ("ldr", c_i64),
        ("mask", c_p), ("ldmask", c_i64), ("mask_arows", c_i32), ("mask_type", c_i32),
        ("alpha", c_f),
        ("relu", c_i32), ("atomic", c_i32), ("split_k", c_i32),
        ("tile_hint", c_i32),
        ("c_rows", c_p), ("n_store", c_i64),
        ("ws", c_p), ("ws_elems", c_i64),
        ("colsum_a", c_p),
        ("bits_out", c_p), ("ldbits", c_i64),
    ]


class CollateField(C.Structure):
    """savqa_collate_field (include/savqa.h)."""
    _fields_ = [
        ("kind", c_i32), ("elem_bytes", c_i32), ("square", c_i32), ("reserved", c_i32),
        ("T", c_i64), ("row_elems", c_i64), ("fill", C.c_uint64),
        ("src", c_p), ("off", c_p), ("dst", c_p),
    ]


class PlanesJob(C.Structure):
    """savqa_x6_planes_job (include/savqa.h)."""
    _fields_ = [
        ("B", c_p), ("ldb", c_i64), ("b_trans", c_i32), ("reserved", c_i32),
        ("N", c_i64), ("K", c_i64), ("out", c_p),
    ]


# name -> argtypes (restype is always int except savqa_last_error)
_SIGS = {
    "savqa_version": [],
    "savqa_struct_sizes": [c_p, c_i32],
    "savqa_gemm": [c_p, C.POINTER(GemmDesc)],
    "savqa_gemm_plan": [C.POINTER(GemmDesc), c_p],
    "savqa_gemm_ws_elems": [C.POINTER(GemmDesc)],
    "savqa_colsum_acc": [c_p, c_p, c_i64, c_i64, c_i64, c_p],
    "savqa_gemm_lp": [c_p, C.POINTER(GemmLpDesc)],
    "savqa_gemm_lp_supported": [C.POINTER(GemmLpDesc)],
    "savqa_gemm_lp_plan": [C.POINTER(GemmLpDesc), c_p],
    "savqa_gemm_lp_ws_elems": [C.POINTER(GemmLpDesc)],
    "savqa_cast_bf16": [c_p, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_i64],
    "savqa_widen_bf16": [c_p, c_p, c_i64, c_i64, c_i64, c_p, c_i64],
    "savqa_mark_rows": [c_p, c_p, c_i64, c_i64, c_p],
    "savqa_zero_rows": [c_p, c_p, c_i64, c_i64, c_p],
    "savqa_adam_rows": [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_f, c_f, c_f, c_f, c_f, c_f,
                        c_f],
    "savqa_quant_fp8": [c_p, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_i64,
                        c_i64],
    "savqa_dequant_fp8_bf16": [c_p, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64],
    "savqa_colsum_bf16": [c_p, c_p, c_i64, c_i64, c_i64, c_p],
    "savqa_gather_rows_bf16": [c_p, c_p, c_i64, c_p, c_i64, c_i64, c_p, c_i64],
    "savqa_ln_fwd": [c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_f, c_p, c_p, c_p, c_p, c_p, c_p,
                     c_p],
    "savqa_ln_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p,
                     c_i64, c_p],
    "savqa_ln_bwd_workspace_bytes": [c_i64],
    "savqa_rowflag": [c_p, c_p, c_i64, c_i64, c_i64, c_p],
    "savqa_gattn_fwd": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p,
                        c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p],
    "savqa_gattn_bwd": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p,
                        c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64,
                        c_p, c_i64],
    "savqa_gattn_fwd_bf16": [c_p, c_i32, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p,
                             c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p],
    "savqa_gattn_bwd_bf16": [c_p, c_i32, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p,
                             c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64,
                             c_p, c_i64],
    "savqa_gattn_fwd_flash": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p,
                              c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p],
    "savqa_gattn_bwd_flash": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p,
                              c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p,
                              c_p, c_i64, c_p, c_i64, c_p, c_i64],
    "savqa_gattn_q1s_ws_bytes": [c_i64, c_i64, c_i64],
    "savqa_gattn_flash_ws_bytes": [c_i64, c_i64, c_i64, c_i64, c_i32],
    "savqa_gattn_fwd_flash_ws": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p,
                                 c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64],
    "savqa_gattn_bwd_flash_ws": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p,
                                 c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p,
                                 c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64],
    "savqa_gattn_fwd_q1s": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64, c_i64,
                            c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64],
    "savqa_gattn_bwd_q1s": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64, c_i64,
                            c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64,
                            c_p, c_i64],
    "savqa_rel_entries_fwd": [c_p, c_p, c_i32, c_i64, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_p],
    "savqa_rel_entries_bwd": [c_p, c_p, c_i32, c_i64, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_p,
                              c_p, c_p],
    "savqa_rel_loss_ws_bytes": [c_i64, c_i64, c_i64],
    "savqa_rel_loss_fwd": [c_p, c_p, c_i64, c_i64, c_p, c_p, c_i64, c_p, c_f, c_p, c_p, c_p, c_p, c_p,
                           c_i64],
    "savqa_rel_macro_fwd": [c_p, c_p, c_i64, c_i64, c_p, c_p, c_p, c_i64, c_i64, c_p],
    "savqa_rel_macro_bwd": [c_p, c_p, c_i64, c_i64, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_p],
    "savqa_rel_loss_bwd": [c_p, c_p, c_i64, c_i64, c_p, c_p, c_i64, c_p, c_f, c_p, c_p, c_p, c_p,
                           c_p, c_p, c_p, c_p, c_i64],
    "savqa_axpby": [c_p, c_p, c_p, c_i64, c_f, c_f, c_p],
    "savqa_collate": [c_p, C.POINTER(CollateField), c_i32, c_i64],
    "savqa_collate_edges": [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p],
    "savqa_graph_build": [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p, c_p, c_p],
    "savqa_dec_init": [c_p, c_p, c_i64, c_f, c_p, c_i64, c_i64, c_u64, c_i32, c_f, c_p],
    "savqa_dec_init_bwd": [c_p, c_p, c_i64, c_i64, c_i64, c_f, c_u64, c_i32, c_f, c_p, c_p],
    "savqa_dropout": [c_p, c_p, c_i64, c_u64, c_i32, c_f, c_p],
    "savqa_posadd_dropout": [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_u64, c_i32, c_i32, c_f, c_p],
    "savqa_posadd_dropout_bwd": [c_p, c_p, c_i64, c_i64, c_i64, c_u64, c_i32, c_i32, c_f, c_p,
                                 c_p],
    "savqa_period_sum_acc": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p],
    "savqa_copy_rows": [c_p, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_i64],
    "savqa_mil_fwd": [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_f, c_p, c_p, c_p],
    "savqa_mil_bwd": [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_f, c_p, c_p, c_p, c_p, c_p],
    "savqa_mil_bwd_bf16": [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_f, c_p, c_p, c_p, c_p,
                           c_p],
    "savqa_index_put_rows": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p],
    "savqa_segment_add_rows": [c_p, c_p, c_i64, c_p, c_p, c_i64, c_i64, c_p, c_i64],
    "savqa_x6_weight_planes": [c_p, c_p, c_i64, c_i32, c_i64, c_i64, c_p],
    "savqa_x6_weight_planes_bytes": [c_i64, c_i64],
    "savqa_x6_weight_planes_batch": [c_p, c_p, c_i32],
    "savqa_index_get_rows": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p],
    "savqa_loss_fwd": [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f, c_p, c_i32, c_p, c_p, c_p, c_p],
    "savqa_scale_by": [c_p, c_p, c_p, c_i64, c_p],
    "savqa_rowscale_mask": [c_p, c_p, c_p, c_p, c_i64, c_i64, c_p],
    "savqa_affine": [c_p, c_p, c_i64, c_f, c_f, c_p],
    "savqa_gather_rows": [c_p, c_p, c_p, c_i64, c_i64, c_f, c_p],
    "savqa_scatter_rows": [c_p, c_p, c_p, c_i64, c_i64, c_f, c_i64, c_p],
    "savqa_adam": [c_p, c_p, c_p, c_p, c_p, c_i64, c_f, c_f, c_f, c_f, c_f, c_f, c_f],
    "savqa_adam_shadow": [c_p, c_p, c_p, c_p, c_p, c_i64, c_f, c_f, c_f, c_f, c_f, c_f, c_f, c_p],
}

_I64_RET = {"savqa_ln_bwd_workspace_bytes", "savqa_gemm_ws_elems", "savqa_gattn_q1s_ws_bytes",
            "savqa_rel_loss_ws_bytes", "savqa_gemm_lp_ws_elems", "savqa_x6_weight_planes_bytes",
            "savqa_gattn_flash_ws_bytes"}

_lib = None


class SavqaError(RuntimeError):
    pass


def load(path: str = None):
    """Load libsavqa.so and bind every declared entry point (raises if absent).
    SAVQA_LIB overrides the path (A/B timing of alternative builds of the same ABI)."""
    global _lib
    if _lib is not None:
        return _lib
    if path is None:
        path = os.environ.get("SAVQA_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise SavqaError(f"libsavqa.so not built ({path}); run __graft_entry__.build() "
                         "or `make -C structured-alignment-vqa_amd/csrc`")
    lib = C.CDLL(path)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int64 if name in _I64_RET else C.c_int
    lib.savqa_last_error.argtypes = []
    lib.savqa_last_error.restype = C.c_char_p
    _lib = lib
    return lib


def exported_symbols():
    return list(_SIGS) + ["savqa_last_error"]


def call(name: str, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.savqa_last_error().decode("utf-8", "replace")
        raise SavqaError(f"{name} failed (rc={rc}): {msg}")
    return rc
