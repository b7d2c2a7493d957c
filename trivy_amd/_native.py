"""ctypes binding of libtrivy_secret.so (include/trivy_secret.h).

The library is the product: rule compilation, the exact Go-semantics resolver and the
HIP kernels all live in it.  Importing this module fails loudly when the library has
not been built (`python -m trivy_amd.build`); there is no Python fallback.
"""
import ctypes as C
import os

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtrivy_secret.so")
# measurement builds of the same sources with other compile-time tunings (tools/)
if os.environ.get("TSG_LIB_VARIANT"):
    LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                            "libtrivy_secret_%s.so" % os.environ["TSG_LIB_VARIANT"])

TSG_OK = 0
TSG_ERR_CONFIG = -1
TSG_ERR_ARG = -2
TSG_ERR_GPU = -3
TSG_ERR_NOMEM = -4
TSG_ERR_INTERNAL = -5


class AllowRuleDesc(C.Structure):
    _fields_ = [("id", C.c_char_p), ("description", C.c_char_p), ("regex", C.c_char_p),
                ("path", C.c_char_p)]


class RuleDesc(C.Structure):
    _fields_ = [("id", C.c_char_p), ("category", C.c_char_p), ("title", C.c_char_p),
                ("severity", C.c_char_p), ("regex", C.c_char_p),
                ("keywords", C.POINTER(C.c_char_p)), ("n_keywords", C.c_uint32),
                ("path", C.c_char_p), ("allow_rules", C.POINTER(AllowRuleDesc)),
                ("n_allow_rules", C.c_uint32), ("exclude_regexes", C.POINTER(C.c_char_p)),
                ("n_exclude_regexes", C.c_uint32), ("secret_group_name", C.c_char_p)]


class RulesetInfo(C.Structure):
    _fields_ = [("n_rules", C.c_uint32), ("n_keywords", C.c_uint32), ("n_groups", C.c_uint32),
                ("n_hostonly", C.c_uint32), ("kw_states", C.c_uint32),
                ("max_group_states", C.c_uint32), ("table_bytes", C.c_uint64),
                ("kw_classes", C.c_uint32), ("k1x_literals", C.c_uint32)]


TSG_CTX_EMULATE = 1


class CtxOptions(C.Structure):
    _fields_ = [("chunk_bytes", C.c_uint32), ("ext_cap", C.c_uint32),
                ("cand_capacity", C.c_uint32), ("host_threads", C.c_int32),
                ("adapt_mib", C.c_uint32), ("flags", C.c_uint32), ("slot_mib", C.c_uint32),
                ("max_slots", C.c_uint32)]


class SlotView(C.Structure):
    _fields_ = [("id", C.c_uint32), ("data", C.c_void_p), ("data_cap", C.c_uint64),
                ("offsets", C.POINTER(C.c_uint64)), ("files_cap", C.c_uint32),
                ("paths", C.c_void_p), ("paths_cap", C.c_uint64),
                ("path_offsets", C.POINTER(C.c_uint64))]


class LayerView(C.Structure):
    _fields_ = [("data", C.c_void_p), ("offsets", C.POINTER(C.c_uint64)), ("nfiles", C.c_uint32),
                ("paths", C.c_void_p), ("path_offsets", C.POINTER(C.c_uint64)),
                ("opq", C.c_void_p), ("opq_len", C.c_size_t), ("wh", C.c_void_p),
                ("wh_len", C.c_size_t), ("walked", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("k1_ms", C.c_double), ("k2_ms", C.c_double), ("aux_ms", C.c_double),
                ("resolve_ms", C.c_double), ("bytes", C.c_uint64), ("k2_bytes", C.c_uint64),
                ("candidates", C.c_uint64), ("files_resolved", C.c_uint64),
                ("k2_launches", C.c_uint32), ("overflow", C.c_uint32),
                ("gate_ms", C.c_double), ("k2_items", C.c_uint64),
                ("k1_hot_states", C.c_uint32), ("h2d_ms", C.c_double),
                ("groups_skipped", C.c_uint32), ("batches", C.c_uint64),
                ("sum_bytes", C.c_uint64), ("sum_k1_ms", C.c_double),
                ("sum_gate_ms", C.c_double), ("sum_k2_ms", C.c_double),
                ("sum_h2d_ms", C.c_double), ("sum_d2h_ms", C.c_double),
                ("sum_resolve_ms", C.c_double), ("wait_ms", C.c_double),
                ("k2_tail_bytes", C.c_uint32), ("k2_tail_max", C.c_uint32),
                ("k2_long_tails", C.c_uint32), ("k2_replays", C.c_uint32),
                ("prep_ms", C.c_double), ("meta_ms", C.c_double),
                ("sum_prep_ms", C.c_double), ("sum_meta_ms", C.c_double),
                ("k1x_records", C.c_uint32), ("k1x_inline", C.c_uint32),
                ("k1f_listed", C.c_uint32), ("k1f_arrivals", C.c_uint32),
                ("event_chunks", C.c_uint32), ("k1_filter", C.c_uint32),
                ("k1_clock_ms", C.c_double), ("chain_clock_ms", C.c_double), ("post_k1_clock_ms", C.c_double),
                ("sum_k1_clock_ms", C.c_double), ("sum_chain_clock_ms", C.c_double),
                ("sum_post_k1_clock_ms", C.c_double)]


# (name, restype, argtypes) -- every symbol include/trivy_secret.h declares
_P = C.c_void_p
_U8P = C.POINTER(C.c_uint8)
_U64P = C.POINTER(C.c_uint64)
_I64P = C.POINTER(C.c_int64)
SIGNATURES = [
    ("tsg_ruleset_compile", C.c_int, [C.POINTER(RuleDesc), C.c_uint32, C.POINTER(AllowRuleDesc),
                                      C.c_uint32, C.POINTER(C.c_char_p), C.c_uint32,
                                      C.POINTER(_P), C.c_char_p, C.c_size_t]),
    ("tsg_ruleset_destroy", None, [_P]),
    ("tsg_ruleset_allow_path", C.c_int, [_P, C.c_char_p, C.c_size_t]),
    ("tsg_ruleset_get_info", C.c_int, [_P, C.POINTER(RulesetInfo)]),
    ("tsg_scan_cpu", C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    ("tsg_scan_cpu_batch", C.c_int, [_P, _P, _U64P, C.c_uint32, _P, _U64P, C.c_int,
                                     C.POINTER(_P)]),
    ("tsg_result_data", _P, [_P, C.POINTER(C.c_size_t)]),
    ("tsg_result_free", None, [_P]),
    ("tsg_result_summary", C.c_int, [_P, _U64P, _U64P, _U64P]),
    ("tsg_ctx_create", C.c_int, [C.c_int, _P, C.POINTER(CtxOptions), C.POINTER(_P)]),
    ("tsg_ctx_destroy", None, [_P]),
    ("tsg_batch_upload", C.c_int, [_P, _P, _U64P, C.c_uint32, _P, _U64P, C.POINTER(C.c_uint32)]),
    ("tsg_batch_kernels", C.c_int, [_P, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_size_t,
                                    C.POINTER(C.c_uint32), C.c_size_t]),
    ("tsg_batch_collect", C.c_int, [_P, C.c_uint64, C.POINTER(_P)]),
    ("tsg_batch_pending", C.c_int, [_P]),
    ("tsg_scan_batch", C.c_int, [_P, _P, _U64P, C.c_uint32, _P, _U64P, C.POINTER(_P)]),
    ("tsg_ctx_get_stats", C.c_int, [_P, C.POINTER(Stats)]),
    ("tsg_slot_acquire", C.c_int, [_P, C.c_uint64, C.c_uint32, C.c_uint64, C.POINTER(SlotView)]),
    ("tsg_slot_submit", C.c_int, [_P, C.c_uint32, C.c_uint32, _U64P]),
    ("tsg_slot_release", C.c_int, [_P, C.c_uint32]),
    ("tsg_queue_create", C.c_int, [_P, C.c_uint32, C.POINTER(_P)]),
    ("tsg_queue_scan", C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
                                 C.POINTER(_P)]),
    ("tsg_queue_flush", C.c_int, [_P]),
    ("tsg_queue_destroy", None, [_P]),
    ("tsg_multi_create", C.c_int, [C.POINTER(C.c_int), C.c_uint32, _P, C.POINTER(CtxOptions),
                                   C.POINTER(_P)]),
    ("tsg_multi_size", C.c_int, [_P]),
    ("tsg_multi_ctx", C.c_int, [_P, C.c_uint32, C.POINTER(_P)]),
    ("tsg_multi_scan_batch", C.c_int, [_P, _P, _U64P, C.c_uint32, _P, _U64P, C.POINTER(_P)]),
    ("tsg_multi_get_stats", C.c_int, [_P, C.c_uint32, C.POINTER(Stats)]),
    ("tsg_multi_destroy", None, [_P]),
    ("tsg_last_error", C.c_char_p, []),
    ("tsg_test_knob", C.c_int, [C.c_char_p, C.c_char_p]),
    ("tsg_regex_compile", C.c_int, [C.c_char_p, C.POINTER(_P), C.c_char_p, C.c_size_t]),
    ("tsg_regex_free", None, [_P]),
    ("tsg_regex_num_slots", C.c_int, [_P]),
    ("tsg_regex_match", C.c_int, [_P, C.c_char_p, C.c_size_t]),
    ("tsg_regex_find_all", C.c_int64, [_P, C.c_char_p, C.c_size_t, C.c_int, _I64P, C.c_size_t]),
    ("tsg_regex_find_all_engine", C.c_int64, [_P, C.c_char_p, C.c_size_t, C.c_int, C.c_int, _I64P, C.c_size_t]),
    ("tsg_regex_dfa_ends", C.c_int64, [_P, C.c_char_p, C.c_size_t, C.c_uint32, _I64P,
                                       C.c_size_t]),
    ("tsg_scan_batch_emulated", C.c_int, [_P, _P, _U64P, C.c_uint32, _P, _U64P, C.c_uint32,
                                          C.POINTER(_P)]),
    ("tsg_emulate_candidate_stats", C.c_int, [_P, _P, _U64P, C.c_uint32, C.c_uint32, _U64P,
                                              _U64P]),
    ("tsg_ruleset_rule_plan", C.c_int, [_P, C.c_uint32, C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int64)]),
    ("tsg_emulate_k1", C.c_int, [_P, _P, _U64P, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32),
                                 C.c_size_t, C.POINTER(C.c_uint32), C.c_size_t]),
    ("tsg_layer_pack", C.c_int, [_P, _P, C.c_uint64, C.POINTER(C.c_char_p), C.c_uint32,
                                 C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p, C.POINTER(_P)]),
    ("tsg_layer_pack_shard", C.c_int, [_P, _P, C.c_uint64, C.POINTER(C.c_char_p), C.c_uint32,
                                       C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p, C.c_uint32,
                                       C.c_uint32, C.POINTER(_P)]),
    ("tsg_layer_get", C.c_int, [_P, C.POINTER(LayerView)]),
    ("tsg_layer_range_walk", C.c_int, [_P, C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(_P),
                                       _U64P]),
    ("tsg_layer_range_sync", C.c_int, [_P, C.c_uint64, _U64P]),
    ("tsg_layer_range_dirs", C.c_int, [_P, C.POINTER(C.c_char_p), C.c_uint32,
                                       C.POINTER(C.c_void_p), _U64P]),
    ("tsg_layer_range_pack", C.c_int, [_P, _P, C.POINTER(C.c_char_p), C.c_uint32,
                                       C.POINTER(C.c_char_p), C.c_uint32, C.POINTER(C.c_char_p),
                                       C.c_uint32, C.c_char_p, C.POINTER(_P)]),
    ("tsg_layer_range_free", None, [_P]),
    ("tsg_fs_pack", C.c_int, [_P, C.c_char_p, C.POINTER(C.c_char_p), C.c_uint32,
                              C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p, C.POINTER(_P)]),
    ("tsg_fs_pack_shard", C.c_int, [_P, C.c_char_p, C.POINTER(C.c_char_p), C.c_uint32,
                                    C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p, C.c_uint32,
                                    C.c_uint32, C.POINTER(_P)]),
    ("tsg_layer_pack_slot", C.c_int, [_P, _P, C.c_uint64, C.POINTER(C.c_char_p), C.c_uint32,
                                      C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p,
                                      C.POINTER(C.c_uint32), C.POINTER(_P)]),
    ("tsg_layer_range_pack_slot", C.c_int, [_P, _P, C.POINTER(C.c_char_p), C.c_uint32,
                                            C.POINTER(C.c_char_p), C.c_uint32,
                                            C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p,
                                            C.POINTER(C.c_uint32), C.POINTER(_P)]),
    ("tsg_fs_pack_slot", C.c_int, [_P, C.c_char_p, C.POINTER(C.c_char_p), C.c_uint32,
                                   C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p,
                                   C.POINTER(C.c_uint32), C.POINTER(_P)]),
    ("tsg_layer_scan", C.c_int, [_P, _P, C.c_uint64, C.POINTER(C.c_char_p), C.c_uint32,
                                 C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p, C.POINTER(_P),
                                 C.POINTER(_P)]),
    ("tsg_fs_scan", C.c_int, [_P, C.c_char_p, C.POINTER(C.c_char_p), C.c_uint32,
                              C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p, C.POINTER(_P),
                              C.POINTER(_P)]),
    ("tsg_layer_free", None, [_P]),
    ("tsg_go_sort_perm", C.c_int, [_P, _U64P, _I64P, C.c_uint32, C.POINTER(C.c_uint32)]),
    ("tsg_ruleset_rule_anchor", C.c_int, [_P, C.c_uint32, C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_int64), C.c_char_p, C.c_size_t]),
    ("tsg_emulate_k1f", C.c_int, [_P, _P, _U64P, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32),
                                  C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_size_t,
                                  C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_uint64)]),
    ("tsg_ruleset_k1_literal", C.c_int, [_P, C.c_uint32, C.c_char_p, C.c_uint32,
                                         C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
]

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libtrivy_secret.so is not built; run `python -m trivy_amd.build` "
                              "(expected at %s)" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class NativeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (code %d)" % (msg, code))
        self.code = code


def knob(name, value=None):
    """tsg_test_knob: set (value) or reset (None) a process-wide test / measurement knob."""
    check(lib().tsg_test_knob(name.encode(), None if value is None else str(value).encode()))


def check(rc):
    if rc != TSG_OK:
        raise NativeError(rc, lib().tsg_last_error().decode("utf-8", "replace"))
    return rc
