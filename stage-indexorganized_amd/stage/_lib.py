"""ctypes binding of libstage_hip.so (include/stage_hip.h).

The library is the product: if it is missing or fails to load, every entry point raises.
There is no CPU fallback anywhere in this package.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("STAGE_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libstage_hip.so")

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u16p = ctypes.POINTER(ctypes.c_uint16)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_vp = ctypes.c_void_p


class StageParams(ctypes.Structure):
    _fields_ = [
        ("split_threshold", ctypes.c_uint32),
        ("merge_threshold", ctypes.c_uint32),
        ("leaf_node_size", ctypes.c_uint32),
        ("payload_size", ctypes.c_uint32),
        ("key_width", ctypes.c_uint32),
        ("device", ctypes.c_int32),
    ]


# every exported symbol: name -> (restype, argtypes)
SIGNATURES = {
    "stage_last_error": (ctypes.c_char_p, []),
    "stage_version": (ctypes.c_char_p, []),
    "stage_table_create": (ctypes.c_int, [ctypes.POINTER(StageParams), ctypes.POINTER(c_vp)]),
    "stage_table_destroy": (ctypes.c_int, [c_vp]),
    "stage_insert": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint16, c_vp, ctypes.c_uint64, ctypes.c_int,
                                    ctypes.c_uint32, c_u8p]),
    "stage_load_ycsb": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, c_u64p]),
    "stage_load_keys": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, c_u64p]),
    "stage_update": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint16, ctypes.c_uint32, c_vp, ctypes.c_uint32,
                                    ctypes.c_uint32, c_u8p]),
    "stage_commit_update": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint32,
                                           c_u8p]),
    "stage_finalize_update": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint16, ctypes.c_uint32, c_u8p]),
    "stage_delete": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint16, ctypes.c_uint32, c_u8p]),
    "stage_update_batch": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint16,
                                          ctypes.c_uint32, c_vp, ctypes.c_uint32, c_vp, c_vp, c_vp, c_vp, c_u64p]),
    "stage_update_batch_device": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_uint64, ctypes.c_uint32, c_vp,
                                                 ctypes.c_uint32, c_vp, c_vp, c_vp, c_vp, c_u64p, c_vp]),
    "stage_insert_key": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, c_vp, ctypes.c_uint32, c_u8p]),
    "stage_insert_key_inflight": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, c_vp, ctypes.c_uint32, c_u8p]),
    "stage_commit_insert_key": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, ctypes.c_uint32, c_u8p]),
    "stage_load_rows": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint32, ctypes.c_uint16, c_vp, ctypes.c_uint32,
                                       ctypes.c_uint64, ctypes.c_uint32, c_vp, c_u64p]),
    "stage_update_key": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, ctypes.c_uint32, c_vp, ctypes.c_uint32,
                                        ctypes.c_uint32, c_u8p]),
    "stage_commit_update_key": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint32,
                                               c_u8p]),
    "stage_delete_key": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, ctypes.c_uint32, c_u8p]),
    "stage_abort_update_key": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, c_u8p]),
    "stage_abort_insert_key": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, c_u8p]),
    "stage_key_words": (ctypes.c_uint32, [c_vp]),
    "stage_sync": (ctypes.c_int, [c_vp]),
    "stage_tpcc_stock_level": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp]),
    "stage_ch_query2_batch": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_int32, c_vp,
                                             ctypes.c_uint32, c_vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                             c_vp, c_vp]),
    "stage_ch_query2_batch_async": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_int32, c_vp,
                                                   ctypes.c_uint32, c_vp, ctypes.c_uint64, ctypes.c_int, c_vp]),
    "stage_ch_query2_wait": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), c_vp]),
    "stage_ch_query2": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_int32, ctypes.c_uint32,
                                       ctypes.c_uint32, c_vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_int32), c_vp]),
    "stage_index_scan_batch": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_uint64, ctypes.c_uint32, c_vp, c_vp,
                                              c_vp, c_vp]),
    "stage_index_scan_first_batch": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_uint64, ctypes.c_uint32,
                                                    ctypes.c_uint32, c_vp, c_vp, c_vp]),
    "stage_set_shard_chunks": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "stage_probe_sharded_loopback": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_int,
                                                    c_vp]),
    "stage_probe_sharded_ex": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, ctypes.c_int, c_vp]),
    "stage_sharded_owner_rows": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.POINTER(c_vp), c_u64p]),
    "stage_set_shard_dedupe": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "stage_set_shard_key_bits": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "stage_set_write_overlap": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "stage_scratch_plan_check": (ctypes.c_int, [ctypes.c_int, c_vp, ctypes.c_int]),
    "stage_settle": (ctypes.c_int, [c_vp]),
    "stage_rccl_info": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_char_p,
                                       ctypes.c_uint64]),
    "stage_sharded_stats": (ctypes.c_int, [c_vp, ctypes.c_int, c_u64p, c_u64p, c_u64p]),
    "stage_sharded_stats_ex": (ctypes.c_int, [c_vp, ctypes.c_int, c_u64p, ctypes.c_int]),
    "stage_comm_allreduce_f64": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double), ctypes.c_uint64, ctypes.c_int]),
    "stage_comm_allgather_f64": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double), ctypes.c_uint64,
                                                ctypes.POINTER(ctypes.c_double)]),
    "stage_export_leaf_images": (ctypes.c_int64, [c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp]),
    "stage_import_leaf_images": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, ctypes.c_uint32, c_vp, c_vp, c_u64p]),
    "stage_export_locations": (ctypes.c_int64, [c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp]),
    "stage_resolve_locations": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp]),
    "stage_host_alloc": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(c_vp)]),
    "stage_host_free": (ctypes.c_int, [c_vp]),
    "stage_probe_host": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp]),
    "stage_reader_create": (ctypes.c_int, [c_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(c_vp)]),
    "stage_reader_create_resident": (ctypes.c_int, [c_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                    ctypes.POINTER(c_vp)]),
    "stage_reader_read": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint16, ctypes.c_uint32, c_vp, c_vp]),
    "stage_reader_stats": (ctypes.c_int, [c_vp, c_vp]),
    "stage_reader_destroy": (ctypes.c_int, [c_vp]),
    "stage_sync_info": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double), c_vp]),
    "stage_stats": (ctypes.c_int, [c_vp, c_vp]),
    "stage_record_stride": (ctypes.c_uint32, [c_vp]),
    "stage_leaf_capacity": (ctypes.c_uint32, [c_vp]),
    "stage_traverse_batch": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_uint64, ctypes.c_int, c_vp]),
    "stage_export_leaves": (ctypes.c_int64, [c_vp, ctypes.c_uint32, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp]),
    "stage_probe_batch": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp]),
    "stage_probe_batch_ex": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp]),
    "stage_reader_read_ex": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_int,
                                            c_vp, c_vp, c_vp]),
    "stage_update_key_owned": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, ctypes.c_uint32, c_vp, ctypes.c_uint32,
                                              ctypes.c_uint32, c_u8p]),
    "stage_delete_key_owned": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, c_u8p]),
    "stage_set_output_layout": (ctypes.c_int, [c_vp, ctypes.c_uint32, ctypes.c_uint32]),
    "stage_scan_batch": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_uint64, ctypes.c_uint32, c_vp, c_vp, c_vp]),
    "stage_resolve_batch": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_uint64, ctypes.c_int, c_vp, c_vp]),
    "stage_set_probe_tuning": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int]),
    "stage_set_probe_store": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "stage_murmur64a_batch": (ctypes.c_int, [c_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                             ctypes.c_uint64, c_vp, c_vp]),
    "stage_comm_unique_id": (ctypes.c_int, [c_vp]),
    "stage_comm_init": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int]),
    "stage_comm_destroy": (ctypes.c_int, [c_vp]),
    "stage_probe_sharded": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp]),
    "stage_set_device": (ctypes.c_int, [ctypes.c_int]),
    "stage_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "stage_dev_alloc": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(c_vp)]),
    "stage_dev_free": (ctypes.c_int, [c_vp]),
    "stage_dev_memset": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_uint64, c_vp]),
    "stage_memcpy_h2d": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp]),
    "stage_memcpy_d2h": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp]),
    "stage_stream_create": (ctypes.c_int, [ctypes.POINTER(c_vp)]),
    "stage_stream_destroy": (ctypes.c_int, [c_vp]),
    "stage_stream_sync": (ctypes.c_int, [c_vp]),
    "stage_device_sync": (ctypes.c_int, []),
    "stage_event_create": (ctypes.c_int, [ctypes.POINTER(c_vp)]),
    "stage_event_destroy": (ctypes.c_int, [c_vp]),
    "stage_event_record": (ctypes.c_int, [c_vp, c_vp]),
    "stage_event_elapsed": (ctypes.c_int, [c_vp, c_vp, ctypes.POINTER(ctypes.c_float)]),
    "stage_fastrandom_next": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, c_vp]),
    "stage_zipf_draws": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_double, ctypes.c_uint64, ctypes.c_uint64, c_vp,
                                        ctypes.c_int]),
    "stage_zipf_zeta": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_double, c_vp]),
    "stage_ycsb_ops": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double, c_vp, c_vp]),
    "stage_probe_identify": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp]),
    "stage_reader_read_ident": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint16, ctypes.c_uint32, c_vp, c_vp,
                                               c_vp]),
    "stage_record_meta_key": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint16, c_u64p, c_vp, c_u8p]),
    "stage_location_cells": (ctypes.c_int, [c_vp]),
    "stage_location_cell": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.POINTER(c_vp)]),
    "stage_copy_get": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp]),
    "stage_copy_readers": (ctypes.c_int, [c_vp, ctypes.c_uint32, c_vp, ctypes.c_uint32, c_u32p]),
    "stage_copy_add_reader": (ctypes.c_int, [c_vp, ctypes.c_uint32, ctypes.c_uint32]),
    "stage_copy_wr_count": (ctypes.c_int, [c_vp, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "stage_copy_update_ps": (ctypes.c_int, [c_vp, ctypes.c_uint32, ctypes.c_uint32]),
}


class StageError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libstage_hip.so once; raise if it is absent (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise StageError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = lib().stage_last_error().decode(errors="replace")
        raise StageError(f"{what}: rc={rc}: {msg}")
    return rc
