"""MI355X-native index-organized probe/scan path of Stage (sheepTnT/Stage-IndexOrganized).

Python is glue here: the product is lib/libstage_hip.so (HIP kernels for gfx950, host table
builder, C-ABI in include/stage_hip.h).
"""
from ._lib import LIB_PATH, SIGNATURES, StageError, lib
from .table import (PROBE_OUT_DTYPE, PROBE_OUT16_DTYPE, Q2_REC_DTYPE, ch_query2, ch_query2_batch, ch_query2_batch_async, REPLY_DIRECT, REPLY_OWNER, REPLY_PEER, REPLY_ROWS, RC_DIRTY, RC_INVALID, RC_KEY_EXISTS, RC_NOT_FOUND, RC_NOT_NEEDED_UPDATE, RC_OK,
                    ST_CHAIN_MISS, ST_COPY, ST_FAIL_INVALID_TS, ST_LATEST, ST_NOT_FOUND, ST_OLD, DeviceBuffer, Event,
                    Reader, Stream, Table, device_count, pinned_empty, fastrandom, murmur64a_device, owner_rows, probe_sharded_loopback,
                    comm_allgather, comm_allreduce, rccl_info, set_shard_dedupe, set_shard_key_bits, sharded_stats,
                    sharded_stats_ex,
                    ycsb_ops, zipf_draws, zipf_zeta)

__all__ = [
    "LIB_PATH", "SIGNATURES", "Q2_REC_DTYPE", "ch_query2", "ch_query2_batch", "ch_query2_batch_async", "StageError", "lib", "PROBE_OUT_DTYPE", "PROBE_OUT16_DTYPE", "Table", "DeviceBuffer", "Stream", "Event", "pinned_empty",
    "murmur64a_device", "zipf_draws", "zipf_zeta", "Reader", "probe_sharded_loopback", "owner_rows", "set_shard_dedupe", "set_shard_key_bits",
    "rccl_info", "sharded_stats", "sharded_stats_ex", "comm_allreduce", "comm_allgather", "REPLY_ROWS", "REPLY_OWNER", "REPLY_PEER", "REPLY_DIRECT", "fastrandom", "ycsb_ops", "device_count", "ST_NOT_FOUND", "ST_LATEST", "ST_COPY", "ST_OLD",
    "ST_FAIL_INVALID_TS", "ST_CHAIN_MISS", "RC_OK", "RC_INVALID", "RC_KEY_EXISTS", "RC_NOT_FOUND",
    "RC_NOT_NEEDED_UPDATE", "RC_DIRTY",
]
