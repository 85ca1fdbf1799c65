"""ctypes binding of ``libnsgcoder.so`` (C ABI declared in ``include/nsg_coder.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``hipcc --offload-arch=gfx950``).  There is
no CPU fallback: if the shared object is missing or cannot be loaded, :func:`lib` raises, and every
coder entry point fails loudly.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = PKG / "_build" / "libnsgcoder.so"
# tools/ may point at an alternative build of the SAME source (compile-time tuning variants)
if os.environ.get("NSG_CODER_LIB"):
    LIB_PATH = Path(os.environ["NSG_CODER_LIB"]).resolve()

NS_OK, NS_ERR_CONFIG, NS_ERR_UNSUPPORTED, NS_ERR_HIP = 0, -1, -2, -3
NS_DTYPE_F32, NS_DTYPE_F16, NS_DTYPE_F64 = 0, 1, 2  # F64: provider probability rows (rank coder)
NS_ST_DONE, NS_ST_ERR_RANGE, NS_ST_ERR_DIVERGE, NS_ST_EXACT_SUM = 1, 2, 4, 8
NS_STEP_FORCE_EXACT_SUM = 1
NS_STEP_FINISH_SENT = 16
NS_STEP_DIAG_STREAM_ONLY, NS_STEP_DIAG_NO_CANDIDATES, NS_STEP_DIAG_SKIP_CDF = 2, 4, 8
NS_MAX_BANNED = 8

EXPORTS = ("ns_create", "ns_destroy", "ns_last_error", "ns_version", "ns_max_topk", "ns_set_split_max_batch",
           "ns_init_state",
           "ns_encode_step", "ns_decode_step", "ns_set_sentence_end", "ns_set_stats", "ns_sample_step", "ns_set_rank_export",
           "ns_rank_encode_step", "ns_set_rank_rows", "ns_rank_decode_step", "ns_token_probs",
           "ns_read_counters", "ns_decode_attention", "ns_decode_attention_dev", "ns_decode_attention_prefix",
           "ns_decode_attention_fp8", "ns_decode_attention_ex", "ns_quantize_fp8",
           "ns_score_rows", "ns_lm_gemm", "ns_lm_gemm_config", "ns_lm_gemm_configs", "ns_lm_layernorm",
           "ns_lm_layernorm_count",
           "ns_lm_embed_ln", "ns_lm_embed_seq_ln", "ns_seq_attention", "ns_lm_ln_gemm",
           "ns_decode_attention_paged", "ns_lm_embed_ln_rows", "ns_lm_layernorm_rows",
           "ns_frac_create", "ns_frac_destroy", "ns_frac_last_error", "ns_frac_init", "ns_frac_encode_step",
           "ns_frac_decode_step", "ns_frac_set_slots", "ns_frac_scratch_bytes")
NS_LM_EPI_STORE, NS_LM_EPI_GELU, NS_LM_EPI_RESIDUAL, NS_LM_EPI_STORE_F32 = 0, 1, 2, 3
NS_KV_FP16, NS_KV_FP8 = 0, 1


class NsStreamState(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64), ("bit_pos", ctypes.c_int64),
                ("ntokens", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class NsStepTrace(ctypes.Structure):
    _fields_ = [("k", ctypes.c_int32), ("kprime", ctypes.c_int32), ("sel", ctypes.c_int32),
                ("n", ctypes.c_int32), ("token", ctypes.c_int32), ("exact", ctypes.c_int32),
                ("S", ctypes.c_double)]


assert ctypes.sizeof(NsStreamState) == 32 and ctypes.sizeof(NsStepTrace) == 32

_lib = None


class NativeLibraryError(RuntimeError):
    """The HIP coder library is missing or unusable (never silently replaced by a CPU path)."""


class NsRankQuality(ctypes.Structure):
    """``ns_rank_quality`` (include/nsg_coder.h)."""

    _fields_ = [("top_k", ctypes.c_int32), ("cap_bits", ctypes.c_int32), ("top_p", ctypes.c_double),
                ("min_prob", ctypes.c_double), ("prob_temp", ctypes.c_double)]


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise NativeLibraryError(
            f"{LIB_PATH} is missing: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()')")
    try:
        L = ctypes.CDLL(str(LIB_PATH))
    except OSError as exc:  # pragma: no cover - environment specific
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {exc}") from exc
    vp, i32p, u8p, i64p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_void_p, ctypes.c_void_p
    L.ns_create.restype = vp
    L.ns_create.argtypes = [ctypes.c_int] * 6
    L.ns_destroy.restype = None
    L.ns_destroy.argtypes = [vp]
    L.ns_last_error.restype = ctypes.c_char_p
    L.ns_last_error.argtypes = [vp]
    L.ns_version.restype = ctypes.c_char_p
    L.ns_version.argtypes = []
    L.ns_max_topk.restype = ctypes.c_int
    L.ns_max_topk.argtypes = [ctypes.c_int]
    L.ns_init_state.restype = ctypes.c_int
    L.ns_init_state.argtypes = [vp, vp, ctypes.c_int, vp]
    L.ns_encode_step.restype = ctypes.c_int
    L.ns_encode_step.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int, u8p, ctypes.c_int64, i64p, vp, vp, vp,
                                 ctypes.c_int64, ctypes.c_double, ctypes.c_int, i32p, ctypes.c_int, vp,
                                 ctypes.c_uint32, vp]
    L.ns_decode_step.restype = ctypes.c_int
    L.ns_decode_step.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_int64,
                                 ctypes.c_double, ctypes.c_int, i32p, ctypes.c_int, vp, ctypes.c_uint32, vp]
    L.ns_set_sentence_end.restype = ctypes.c_int
    L.ns_set_sentence_end.argtypes = [vp, vp]
    L.ns_rank_encode_step.restype = ctypes.c_int
    L.ns_rank_encode_step.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int, vp, ctypes.c_int64, vp, vp, vp, vp, vp,
                                      ctypes.c_int64, ctypes.c_double, ctypes.POINTER(NsRankQuality), vp,
                                      ctypes.c_uint32, vp]
    L.ns_rank_decode_step.restype = ctypes.c_int
    L.ns_rank_decode_step.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_int64,
                                      ctypes.c_double, ctypes.POINTER(NsRankQuality), vp, ctypes.c_uint32, vp]
    L.ns_token_probs.restype = ctypes.c_int
    L.ns_token_probs.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                                 ctypes.POINTER(NsRankQuality), vp, ctypes.c_int64, vp, vp]
    L.ns_set_rank_rows.restype = ctypes.c_int
    L.ns_set_rank_rows.argtypes = [vp, vp, vp, ctypes.c_int64, ctypes.c_int]
    L.ns_set_rank_export.restype = ctypes.c_int
    L.ns_set_rank_export.argtypes = [vp, vp, ctypes.c_int]
    L.ns_set_stats.restype = ctypes.c_int
    L.ns_set_stats.argtypes = [vp, vp]
    L.ns_sample_step.restype = ctypes.c_int
    L.ns_sample_step.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, vp, vp,
                                 vp, ctypes.c_int64, ctypes.c_double, ctypes.c_int, i32p, ctypes.c_int, vp, vp,
                                 ctypes.c_uint32, vp]
    L.ns_read_counters.restype = ctypes.c_int
    L.ns_read_counters.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    L.ns_score_rows.restype = ctypes.c_int
    L.ns_score_rows.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp]
    L.ns_decode_attention_dev.restype = ctypes.c_int
    L.ns_decode_attention_dev.argtypes = [vp, ctypes.c_int64, vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, vp, ctypes.c_int64,
                                          ctypes.c_float, vp]
    L.ns_decode_attention.restype = ctypes.c_int
    L.ns_decode_attention.argtypes = [vp, ctypes.c_int64, vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_float, vp]
    i64, ci = ctypes.c_int64, ctypes.c_int
    for name in ("ns_decode_attention_prefix", "ns_decode_attention_fp8"):
        f = getattr(L, name)
        f.restype = ci
        f.argtypes = [vp, i64, vp, vp, i64, i64, i64, vp, vp, i64, ci, ci, ci, ci, ci, vp, ci, ci, vp, i64,
                      ctypes.c_float, vp]
    L.ns_decode_attention_ex.restype = ci
    L.ns_decode_attention_ex.argtypes = [vp, i64, vp, vp, i64, i64, i64, vp, vp, i64, ci, ci, ci, ci, ci, vp, ci, ci, ci,
                                         vp, i64, vp, vp, i64, ctypes.c_float, vp]
    L.ns_decode_attention_paged.restype = ci
    L.ns_decode_attention_paged.argtypes = [vp, i64, vp, i64, ci, i64, vp, vp, i64, ci, ci, ci, ci, vp, ci, ci, vp, i64,
                                            vp, vp, i64, ctypes.c_float, vp]
    L.ns_lm_embed_ln_rows.restype = ci
    L.ns_lm_embed_ln_rows.argtypes = [vp, vp, vp, ci, ci, vp, vp, i64, vp, vp, vp, i64, ci, ci, ctypes.c_float, vp]
    L.ns_lm_layernorm_rows.restype = ci
    L.ns_lm_layernorm_rows.argtypes = [vp, i64, vp, vp, vp, i64, ci, ci, ctypes.c_float, vp, vp]
    L.ns_quantize_fp8.restype = ci
    L.ns_quantize_fp8.argtypes = [vp, vp, i64, vp]
    L.ns_lm_gemm.restype = ci
    L.ns_lm_gemm.argtypes = [vp, i64, vp, i64, vp, vp, i64, ci, ci, ci, ci, vp]
    L.ns_lm_gemm_config.restype = ci
    L.ns_lm_gemm_config.argtypes = [vp, i64, vp, i64, vp, vp, i64, ci, ci, ci, ci, ci, vp]
    L.ns_lm_gemm_configs.restype = ci
    L.ns_lm_gemm_configs.argtypes = []
    L.ns_lm_layernorm.restype = ci
    L.ns_lm_layernorm.argtypes = [vp, i64, vp, vp, vp, i64, ci, ci, ctypes.c_float, vp]
    L.ns_lm_layernorm_count.restype = ci
    L.ns_lm_layernorm_count.argtypes = [vp, i64, vp, vp, vp, i64, ci, ci, ctypes.c_float, vp, vp]
    L.ns_set_split_max_batch.restype = ci
    L.ns_set_split_max_batch.argtypes = [ci]
    L.ns_lm_embed_ln.restype = ci
    L.ns_lm_embed_ln.argtypes = [vp, vp, vp, ci, ci, ci, vp, vp, i64, vp, vp, vp, i64, ci, ci, ctypes.c_float, vp]
    L.ns_lm_ln_gemm.restype = ci
    L.ns_lm_ln_gemm.argtypes = [vp, i64, vp, vp, ctypes.c_float, vp, i64, vp, vp, i64, ci, ci, ci, ci, vp, i64, vp]
    L.ns_lm_embed_seq_ln.restype = ci
    L.ns_lm_embed_seq_ln.argtypes = [vp, vp, vp, ci, ci, ci, vp, i64, vp, vp, vp, i64, ci, ci, ctypes.c_float, vp]
    L.ns_seq_attention.restype = ci
    L.ns_seq_attention.argtypes = [vp, i64, vp, i64, ci, ci, ci, ci, ctypes.c_float, vp]
    L.ns_frac_create.restype = vp
    L.ns_frac_create.argtypes = [ci, ci, ci]
    L.ns_frac_destroy.restype = None
    L.ns_frac_destroy.argtypes = [vp]
    L.ns_frac_last_error.restype = ctypes.c_char_p
    L.ns_frac_last_error.argtypes = [vp]
    L.ns_frac_init.restype = ci
    L.ns_frac_init.argtypes = [vp, ci, vp, vp]
    L.ns_frac_encode_step.restype = ci
    L.ns_frac_encode_step.argtypes = [vp, ci, vp, vp, i64, vp, vp, i64, i64, i64, vp, vp, vp, vp]
    L.ns_frac_decode_step.restype = ci
    L.ns_frac_decode_step.argtypes = [vp, ci, vp, vp, i64, vp, vp, vp, i64, i64, vp, i64, vp, vp, vp]
    L.ns_frac_set_slots.restype = ci
    L.ns_frac_set_slots.argtypes = [vp, vp, ci]
    L.ns_frac_scratch_bytes.restype = i64
    L.ns_frac_scratch_bytes.argtypes = [vp, ci, i64, i64, i64]
    _lib = L
    return L


def version() -> str:
    return lib().ns_version().decode()


def set_split_max_batch(max_batch: int) -> int:
    """Steps of at most max_batch streams use the split (workgroup-per-stream) coder form (negative: the
    automatic limit); returns the previous setting (-1: automatic).  Speed only: both forms give the same tokens
    and bits."""
    return int(lib().ns_set_split_max_batch(int(max_batch)))


def max_topk(dtype_code: int) -> int:
    return int(lib().ns_max_topk(int(dtype_code)))
