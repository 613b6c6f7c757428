"""ctypes binding of liblaspj.so (include/laspj.h).

This is the Python stand-in for the Erlang NIF that would bind the same entry points
(INTEGRATION.md).  It fails loudly: if the HIP library is missing or does not load,
every caller gets LaspjUnavailable — there is no CPU fallback anywhere in lasp_amd.
"""

from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# LASPJ_LIB: another build of the library (A/B timing of kernel variants, tools/)
LIB_PATH = os.environ.get("LASPJ_LIB") or os.path.join(HERE, "liblaspj.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "laspj.h")

ABI_VERSION = 2
OK = 0
E_INVAL, E_NOMEM, E_DEVICE, E_SHAPE, E_KIND, E_RANGE, E_COMM, E_UNSUPPORTED, E_FUN = (
    -1, -2, -3, -4, -5, -6, -7, -8, -9)
KIND_ORSET, KIND_GSET, KIND_ORSET_CONCAT, KIND_ORSET_PRODUCT, KIND_GSET_PRODUCT = 1, 2, 3, 4, 5
KIND_GCOUNTER = 6
KIND_ORSET_PRODUCT_WIDE = 7
KIND_ORSET_WIDE = 10
KIND_ORSET_LIST, KIND_GSET_LIST = 8, 9
LIST_PAIR = 1 << 62          # key item: {X, Y} of element slots (bits 31-61, 0-30)
LIST_COMPOUND = 1 << 62      # token item: [Tx, Ty] of tokens (bits 31-61, 0-30)
LIST_REMOVED = 1 << 63       # token item: the {Token, true} flag
# from_binary statuses (laspj_orset_etf_read)
DEC_OK, DEC_INVALID_BINARY, DEC_UNSUPPORTED_VERSION, DEC_MALFORMED, DEC_UNKNOWN_TERM, \
    DEC_UNREPRESENTABLE, DEC_EQUAL_TERMS = 0, 1, 2, 3, 4, 5, 6
OP_ADD, OP_REMOVE, OP_INSERT = 1, 2, 3
OP_FLAG_NEW_CALL = 1
OPST_APPLIED, OPST_NOT_PRESENT, OPST_ROLLED_BACK, OPST_KEY_EXISTS = 0, 1, 2, 3
TUNE_STREAM_GRID, TUNE_STREAM_UNROLL, TUNE_STREAM_NT, TUNE_ETF_KERNEL = 1, 2, 3, 4
TUNE_REDUCE_KERNEL = 5
TUNE_PRODUCT_ROWS = 6
TUNE_PRODUCT_COLS = 7
TUNE_ETF_READ = 8
TUNE_ETF_SEG = 9
TUNE_LIST_WALK = 10
TUNE_NIF_PASSES = 14
TUNE_LIST_CHUNK = 15
NIF_OK, NIF_FALLBACK = 0, 1           # verdicts of the NIF-level entry points
NIF_STATS = 20


class LaspjUnavailable(RuntimeError):
    """liblaspj.so is not built / not loadable: the engine has no fallback."""


class LaspjError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"laspj status {status}: {msg}")
        self.status = status


class BatchInfo(C.Structure):
    _fields_ = [("kind", C.c_int32), ("elements", C.c_uint32), ("replicas", C.c_uint64),
                ("bytes_per_replica", C.c_uint64), ("bytes", C.c_uint64),
                ("elements_r", C.c_uint32), ("token_words", C.c_uint32),
                ("cells_per_replica", C.c_uint64)]


class Op(C.Structure):
    _fields_ = [("replica", C.c_uint64), ("element", C.c_uint32), ("kind", C.c_uint8),
                ("slot", C.c_uint8), ("flags", C.c_uint8), ("pad", C.c_uint8)]


class ListOrder(C.Structure):
    _fields_ = [("krank", C.c_void_p), ("nkeys", C.c_uint32), ("ntokens", C.c_uint32),
                ("grank", C.c_void_p)]


class AEStep(C.Structure):
    """laspj_ae_step: one step of an anti-entropy round's plan."""
    _fields_ = [("group", C.c_uint32), ("op", C.c_int32), ("peer", C.c_int32),
                ("buf", C.c_int32), ("offset", C.c_uint64), ("words", C.c_uint64),
                ("src", C.c_uint64), ("nsrc", C.c_uint32), ("tag", C.c_uint32)]


AE_SEND, AE_RECV, AE_REDUCE, AE_ALLREDUCE_MAX = 1, 2, 3, 4
AE_BUF_STATE, AE_BUF_RECV = 0, 1


class Incr(C.Structure):
    _fields_ = [("replica", C.c_uint64), ("actor", C.c_uint32), ("reserved", C.c_uint32),
                ("amount", C.c_uint64)]


vp = C.c_void_p
vpp = C.POINTER(C.c_void_p)
i = C.c_int
u32 = C.c_uint32
u64 = C.c_uint64

# name -> (restype, argtypes); mirrors include/laspj.h one to one
SIGNATURES = {
    "laspj_abi_version": (i, []),
    "laspj_strerror": (C.c_char_p, [i]),
    "laspj_device_count": (i, [C.POINTER(i)]),
    "laspj_ctx_create": (i, [i, vpp]),
    "laspj_ctx_destroy": (i, [vp]),
    "laspj_ctx_last_error": (C.c_char_p, [vp]),
    "laspj_ctx_synchronize": (i, [vp]),
    "laspj_ctx_set_tuning": (i, [vp, i, C.c_int64]),
    "laspj_buf_create": (i, [vp, u64, vpp]),
    "laspj_buf_destroy": (i, [vp]),
    "laspj_buf_bytes": (u64, [vp]),
    "laspj_buf_upload": (i, [vp, vp, u64, vp, u64]),
    "laspj_buf_download": (i, [vp, vp, u64, vp, u64]),
    "laspj_buf_device_ptr": (i, [vp, vpp]),
    "laspj_orset_batch_create": (i, [vp, u64, u32, vpp]),
    "laspj_gset_batch_create": (i, [vp, u64, u32, vpp]),
    "laspj_batch_destroy": (i, [vp]),
    "laspj_batch_wrap": (i, [vp, C.c_int32, vp, u64, u64, u32, vpp]),
    "laspj_batch_reduce_chunks": (i, [vp, vp, vp, u32]),
    "laspj_batch_join_n": (i, [vp, vp, vp, u32]),
    "laspj_batch_bind_many": (i, [vp, u32, vp, vp, vp, vp]),
    "laspj_batch_bind_many_host": (i, [vp, u32, vp, vp, vp, vp]),
    "laspj_batch_inflation_many": (i, [vp, u32, vp, vp, i, vp]),
    "laspj_batch_info_get": (i, [vp, C.POINTER(BatchInfo)]),
    "laspj_batch_device_ptr": (i, [vp, vpp]),
    "laspj_batch_download_range": (i, [vp, vp, u64, u64, vp]),
    "laspj_batch_upload": (i, [vp, vp, u64, u64, vp]),
    "laspj_batch_download": (i, [vp, vp, u64, u64, vp]),
    "laspj_batch_clear": (i, [vp, vp]),
    "laspj_batch_fill_synthetic": (i, [vp, vp, u64, u64]),
    "laspj_batch_fill_synthetic_tokens": (i, [vp, vp, u64, u64, u32]),
    "laspj_orset_fragment": (i, [vp, vp, u32, vp]),
    "laspj_orset_precondition_context": (i, [vp, vp, vp]),
    "laspj_orset_gather_inflation": (i, [vp, vp, vp, vp, vp, i, vp]),
    "laspj_orset_gather_inflation_keyed": (i, [vp, vp, vp, vp, vp, vp, vp, i, vp]),
    "laspj_batch_join": (i, [vp, vp, vp, vp]),
    "laspj_orset_join": (i, [vp, vp, vp, vp]),
    "laspj_orset_reduce": (i, [vp, vp, vp, u32]),
    "laspj_orset_value": (i, [vp, vp, vp]),
    "laspj_orset_removed": (i, [vp, vp, vp]),
    "laspj_orset_stats": (i, [vp, vp, vp]),
    "laspj_orset_equal": (i, [vp, vp, vp, vp]),
    "laspj_orset_inflation": (i, [vp, vp, vp, i, vp]),
    "laspj_orset_apply_ops": (i, [vp, vp, C.POINTER(Op), u64, C.POINTER(C.c_int32)]),
    "laspj_orset_union": (i, [vp, vp, vp, vp]),
    "laspj_orset_filter": (i, [vp, vp, vp, vp]),
    "laspj_orset_concat_batch_create": (i, [vp, u64, u32, vpp]),
    "laspj_orset_intersection": (i, [vp, vp, vp, vp]),
    "laspj_orset_product_batch_create": (i, [vp, u64, u32, u32, vpp]),
    "laspj_orset_product": (i, [vp, vp, vp, vp]),
    "laspj_orset_product_diag": (i, [vp, vp, vp, vp]),
    "laspj_orset_product_wide_batch_create": (i, [vp, u64, u32, u32, vpp]),
    "laspj_orset_gather": (i, [vp, vp, vp, vp]),
    "laspj_gset_union": (i, [vp, vp, vp, vp]),
    "laspj_gset_intersection": (i, [vp, vp, vp, vp]),
    "laspj_gset_filter": (i, [vp, vp, vp, vp]),
    "laspj_gset_product_batch_create": (i, [vp, u64, u32, u32, vpp]),
    "laspj_gset_product": (i, [vp, vp, vp, vp]),
    "laspj_gset_gather": (i, [vp, vp, vp, vp]),
    "laspj_gset_join": (i, [vp, vp, vp, vp]),
    "laspj_gset_reduce": (i, [vp, vp, vp, u32]),
    "laspj_gset_stats": (i, [vp, vp, vp]),
    "laspj_gset_equal": (i, [vp, vp, vp, vp]),
    "laspj_gset_inflation": (i, [vp, vp, vp, i, vp]),
    "laspj_gset_apply_ops": (i, [vp, vp, C.POINTER(Op), u64, C.POINTER(C.c_int32)]),
    "laspj_gcounter_batch_create": (i, [vp, u64, u32, vpp]),
    "laspj_gcounter_join": (i, [vp, vp, vp, vp]),
    "laspj_gcounter_value": (i, [vp, vp, vp]),
    "laspj_gcounter_threshold": (i, [vp, vp, u64, i, vp]),
    "laspj_gcounter_inflation": (i, [vp, vp, vp, i, vp]),
    "laspj_gcounter_equal": (i, [vp, vp, vp, vp]),
    "laspj_gcounter_apply_increments": (i, [vp, vp, C.POINTER(Incr), u64]),
    "laspj_gcounter_reduce": (i, [vp, vp, vp, u32]),
    "laspj_etf_dict_create": (i, [vp, u32, vp, vp, vp, vp, vp, vp, vpp]),
    "laspj_etf_dict_destroy": (i, [vp]),
    "laspj_orset_etf_size": (i, [vp, vp, vp, i, vp, C.POINTER(u64)]),
    "laspj_orset_etf_write": (i, [vp, vp, vp, i, i, vp, vp]),
    "laspj_gset_etf_size": (i, [vp, vp, vp, i, vp, C.POINTER(u64)]),
    "laspj_gset_etf_write": (i, [vp, vp, vp, i, i, vp, vp]),
    "laspj_orset_etf_read": (i, [vp, vp, vp, i, i, vp, vp, vp]),
    "laspj_gset_etf_read": (i, [vp, vp, vp, i, i, vp, vp, vp]),
    "laspj_comm_unique_id": (i, [vp]),
    "laspj_comm_init_rank": (i, [vp, i, vp, i, vpp]),
    "laspj_comm_init_all": (i, [vp, i, vp]),
    "laspj_comm_destroy": (i, [vp]),
    "laspj_comm_info": (i, [vp, C.POINTER(i), C.POINTER(i)]),
    "laspj_antientropy": (i, [vp, vp, vp, vp]),
    "laspj_antientropy_group": (i, [vp, vp, vp, vp, i]),
    "laspj_antientropy_loopback": (i, [vp, i, vp, vp, u64]),
    "laspj_antientropy_plan": (i, [C.c_int32, i, i, u64, u64, C.POINTER(AEStep), u64,
                                   C.POINTER(u64)]),
    "laspj_list_batch_create": (i, [vp, C.c_int32, u64, u32, u32, vpp]),
    "laspj_list_counts": (i, [vp, vp, vp]),
    "laspj_list_upload": (i, [vp, vp, u64, u32, vp, vp, vp]),
    "laspj_list_download": (i, [vp, vp, u64, vp, vp, vp]),
    "laspj_list_from_set": (i, [vp, vp, vp, vp, u32, vp]),
    "laspj_list_merge": (i, [vp, vp, vp, vp, C.POINTER(ListOrder)]),
    "laspj_list_equal": (i, [vp, vp, vp, C.POINTER(ListOrder), vp]),
    "laspj_list_inflation": (i, [vp, vp, vp, i, C.POINTER(ListOrder), vp]),
    "laspj_list_bind": (i, [vp, vp, vp, vp, C.POINTER(ListOrder), vp]),
    "laspj_list_value": (i, [vp, vp, vp]),
    "laspj_list_union": (i, [vp, vp, vp, vp, C.POINTER(ListOrder)]),
    "laspj_list_intersection": (i, [vp, vp, vp, vp, C.POINTER(ListOrder)]),
    "laspj_list_intersection_set": (i, [vp, vp, vp, vp, vp]),
    "laspj_list_product": (i, [vp, vp, vp, vp]),
    "laspj_list_map": (i, [vp, vp, vp, vp, u32, i]),
    "laspj_list_filter": (i, [vp, vp, vp, vp, u32, i]),
    "laspj_list_fold": (i, [vp, vp, vp, vp, vp, u32, i]),
    "laspj_term_compare": (i, [vp, C.c_size_t, vp, C.c_size_t, C.POINTER(i)]),
    "laspj_dict_create": (i, [vpp]),
    "laspj_dict_destroy": (i, [vp]),
    "laspj_dict_add": (i, [vp, C.c_int32, vp, vp, u64, i, vp]),
    "laspj_dict_info": (i, [vp, C.POINTER(u32), C.POINTER(u64), C.POINTER(u64)]),
    "laspj_dict_export": (i, [vp, u32, vp, vp, vp, vp, vp, vp]),
    "laspj_dict_encode": (i, [vp, C.c_int32, vp, vp, u64, i, u32, vp, vp]),
    "laspj_orset_etf_merge": (i, [vp, vp, u64, vp, u64, vpp, C.POINTER(u64),
                                  C.POINTER(C.c_int32)]),
    "laspj_orset_etf_merge_many": (i, [vp, u32, vp, vp, vp, vp, vp, vp, vp]),
    "laspj_orset_etf_value": (i, [vp, vp, u64, vpp, C.POINTER(u64), C.POINTER(C.c_int32)]),
    "laspj_orset_etf_equal": (i, [vp, vp, u64, vp, u64, C.POINTER(C.c_int32),
                                  C.POINTER(C.c_int32)]),
    "laspj_orset_etf_inflation": (i, [vp, vp, u64, vp, u64, i, C.POINTER(C.c_int32),
                                      C.POINTER(C.c_int32)]),
    "laspj_gset_etf_merge": (i, [vp, vp, u64, vp, u64, vpp, C.POINTER(u64),
                                 C.POINTER(C.c_int32)]),
    "laspj_gset_etf_merge_many": (i, [vp, u32, vp, vp, vp, vp, vp, vp, vp]),
    "laspj_gset_etf_value": (i, [vp, vp, u64, vpp, C.POINTER(u64), C.POINTER(C.c_int32)]),
    "laspj_gset_etf_equal": (i, [vp, vp, u64, vp, u64, C.POINTER(C.c_int32),
                                 C.POINTER(C.c_int32)]),
    "laspj_gset_etf_inflation": (i, [vp, vp, u64, vp, u64, i, C.POINTER(C.c_int32),
                                     C.POINTER(C.c_int32)]),
    "laspj_var_create": (i, [vp, C.c_int32, vpp]),
    "laspj_var_destroy": (i, [vp]),
    "laspj_var_etf_bind": (i, [vp, vp, u64, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "laspj_var_etf_bind_many": (i, [vp, u32, vp, vp, vp, vp, vp]),
    "laspj_var_etf_write": (i, [vp, vp, u64, C.POINTER(C.c_int32)]),
    "laspj_var_etf_read": (i, [vp, vpp, C.POINTER(u64), C.POINTER(C.c_int32)]),
    "laspj_var_etf_value": (i, [vp, vpp, C.POINTER(u64), C.POINTER(C.c_int32)]),
    "laspj_var_etf_threshold": (i, [vp, vp, u64, i, C.POINTER(C.c_int32),
                                    C.POINTER(C.c_int32)]),
    "laspj_var_resident": (i, [vp, C.POINTER(C.c_int32)]),
    "laspj_var_create_replica": (i, [vp, vpp]),
    "laspj_var_union": (i, [vp, vp, vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "laspj_var_etf_update": (i, [vp, vp, u64, C.POINTER(C.c_int32), vpp, C.POINTER(u64), vpp,
                                 C.POINTER(u32), C.POINTER(C.c_int32)]),
    "laspj_list_etf_args": (i, [vp, C.c_int32, vp, u64, vpp, C.POINTER(u64),
                                C.POINTER(C.c_int32)]),
    "laspj_list_etf_map": (i, [vp, C.c_int32, vp, u64, vp, u64, vpp, C.POINTER(u64),
                               C.POINTER(C.c_int32)]),
    "laspj_list_etf_filter": (i, [vp, C.c_int32, vp, u64, vp, u64, vpp, C.POINTER(u64),
                                  C.POINTER(C.c_int32)]),
    "laspj_list_etf_fold": (i, [vp, C.c_int32, vp, u64, vp, u64, vpp, C.POINTER(u64),
                                C.POINTER(C.c_int32)]),
    "laspj_list_etf_union": (i, [vp, C.c_int32, vp, u64, vp, u64, vpp, C.POINTER(u64),
                                 C.POINTER(C.c_int32)]),
    "laspj_list_etf_intersection": (i, [vp, C.c_int32, vp, u64, vp, u64, vpp, C.POINTER(u64),
                                        C.POINTER(C.c_int32)]),
    "laspj_list_etf_product": (i, [vp, C.c_int32, vp, u64, vp, u64, vpp, C.POINTER(u64),
                                   C.POINTER(C.c_int32)]),
    "laspj_list_etf_value": (i, [vp, C.c_int32, vp, u64, vpp, C.POINTER(u64),
                                 C.POINTER(C.c_int32)]),
    "laspj_list_etf_bind": (i, [vp, C.c_int32, vp, u64, vp, u64, vpp, C.POINTER(u64),
                                C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "laspj_orset_wide_batch_create": (i, [vp, u64, u32, u32, vpp]),
    "laspj_orset_widen": (i, [vp, vp, vp]),
    "laspj_nif_stats": (i, [vp, vp, u32]),
    "laspj_nif_reset": (i, [vp]),
    "laspj_event_create": (i, [vp, vpp]),
    "laspj_event_destroy": (i, [vp]),
    "laspj_event_record": (i, [vp, vp]),
    "laspj_event_elapsed_ms": (i, [vp, vp, C.POINTER(C.c_float)]),
}

_lib = None


def load():
    """Load liblaspj.so (built in-tree by __graft_entry__.build()) or raise."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LaspjUnavailable(
            f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    try:
        L = C.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the box
        raise LaspjUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.laspj_abi_version() != ABI_VERSION:
        raise LaspjUnavailable("ABI version mismatch")
    _lib = L
    return L


def check(status: int, ctx=None) -> None:
    if status != OK:
        L = load()
        msg = L.laspj_strerror(status).decode()
        if ctx is not None:
            detail = L.laspj_ctx_last_error(ctx)
            if detail:
                msg += f": {detail.decode()}"
        raise LaspjError(status, msg)
