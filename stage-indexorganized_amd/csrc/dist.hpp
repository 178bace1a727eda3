// dist.hpp -- hash-sharded multi-GPU probe front-end (one process per GPU, RCCL over xGMI).
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <string>
#include <vector>

#include "kernel_api.hpp"
#include "stage_core.hpp"

namespace stage {

struct ShardComm {
    void *comm = nullptr;  // ncclComm_t
    int rank = 0, world = 1;
    // device scratch (grown on demand)
    void *dest = nullptr, *cursor = nullptr, *perm = nullptr, *send = nullptr, *recv = nullptr;
    void *rout = nullptr, *rrec = nullptr, *bout = nullptr, *brec = nullptr, *cnt = nullptr;
    void *lkeys = nullptr, *lrids = nullptr;
    void *fan = nullptr;             // [send position] caller positions the request serves (FanRange)
    uint64_t cap_local = 0, cap_remote = 0;
    uint32_t rec_stride = 0;
    int chunks = 1;                  // overlapped exchange chunks (same on every rank)
    hipStream_t cs = nullptr;        // RCCL transfers
    hipStream_t us = nullptr;        // fan-out of returned results / owner-reply expand
    hipStream_t ps = nullptr;        // fan-out probes of own requests (beside the remote probes)
    hipEvent_t ev_fork = nullptr, ev_own = nullptr;
    std::vector<hipEvent_t> evs;     // per-chunk keys / probe / results events + join
    uint64_t owner_rows = 0;         // rows left in rrec by the last owner-reply probe
    // request coalescing: equal (key, read id) requests of a chunk are routed once and their
    // result is expanded to every caller position (a Zipf batch is ~half duplicates)
    bool dedupe = true;
    void *dd_skeys = nullptr, *dd_iota = nullptr, *dd_sidx = nullptr, *dd_flag = nullptr, *dd_useq = nullptr;
    void *uidx = nullptr, *ukeys = nullptr, *urids = nullptr, *upos = nullptr, *dd_cub = nullptr, *dd_nu = nullptr;
    void *urange = nullptr, *flist = nullptr;  // request -> run of flist; flist = caller positions in key order
    uint64_t dd_cap = 0, dd_cub_bytes = 0, dd_cub_items = 0;
    int key_bits = 64;               // coalescing sorts on the low key_bits bits (any value is correct)
    // the last sharded probe: caller keys, requests routed (after coalescing), of which remote
    uint64_t last_n = 0, last_routed = 0, last_remote = 0;
    uint64_t last_received = 0;      // requests this rank probed as owner (own + other ranks')
    void *ctl = nullptr;             // control-plane scratch (doubles)
    uint64_t ctl_cap = 0;
    // STAGE_REPLY_PEER: the owner keeps the rows of the remote requests it probed in one of its
    // two row buffers (by call parity), and each caller's fan-out reads them there -- over xGMI,
    // through the owner's buffers opened by IPC handle (loopback: the other shard's pointers)
    void *prow[2] = {nullptr, nullptr};  // this rank's row buffers
    uint64_t prow_cap = 0;               // rows each of them holds
    uint32_t prow_stride = 0;            // ... of this many bytes
    std::vector<uint64_t> peer_cap;      // every rank's prow_cap, as every rank computes it
    uint32_t peer_stride = 0;            // the row stride peer_cap was planned for
    std::vector<void *> peer_row[2];     // [parity][rank]: where rank's row buffers are here
    std::vector<void *> opened;          // IPC mappings to close
    void *hbuf = nullptr;                // handle / count exchange scratch
    uint64_t hbuf_cap = 0;
    int parity = 0;
    // STAGE_REPLY_DIRECT: each owner probes a remote request straight into its caller's output
    // (status record and row at the first caller position of the request's run, carried in the
    // request record) through the caller's d_out / d_records opened by IPC handle; the caller
    // copies only the duplicates of its coalesced requests.  The callers' buffers change from
    // call to call: their (handle, offset) pairs travel with the counts, and a peer's mapping is
    // reopened when its pair changes (loopback: the other shard's pointers).
    void *lpads = nullptr;               // [received request] its first caller position
    void *fdest = nullptr, *fdest_h = nullptr;  // per chunk, the two remote ranges' FanDest tables (device, pinned)
    struct DirectBuf {                   // one caller buffer as exported: allocation handle + offset
        uint8_t handle[64];
        uint64_t off;
    };
    std::vector<DirectBuf> dseen;        // [2 * rank + {out, rec}] the handles the mappings were opened for
    std::vector<void *> dbase;           // [2 * rank + {out, rec}] their mapped allocation bases
    std::vector<std::vector<void *>> dopen;  // [rank] its IPC mappings to close
    std::vector<void *> dpeer[2];        // [{out, rec}][rank]: the caller buffers as mapped here
    ~ShardComm();
};

int shard_unique_id(uint8_t *id128);
// RCCL version the process runs (ncclGetVersion), the version of the headers the library was
// built against (NCCL_VERSION_CODE) and the file ncclGetVersion resolved to
int shard_rccl_info(int *runtime_code, int *header_code, char *path, uint64_t path_len);
// chunks: overlapped exchange chunks, identical on every rank (<= 0: STAGE_SHARD_CHUNKS, or 4; 1 at world 1)
int shard_init(ShardComm &c, const uint8_t *id128, int rank, int world, int chunks);
int shard_default_chunks(int world);
bool shard_default_dedupe();  // STAGE_SHARD_DEDUPE=0 turns request coalescing off
// control plane on the communicator: op 0 sum, 1 max, 2 min (in place); allgather: out[r*n + i]
int shard_allreduce_f64(ShardComm &c, double *v, uint64_t n, int op);
int shard_allgather_f64(ShardComm &c, const double *in, uint64_t n, double *out);
int shard_probe(ShardComm &c, const DevTable &t, const ProbeTuning &tune, const uint64_t *d_keys,
                const uint32_t *d_rids, uint64_t n, stage_probe_out_dev *d_out, uint8_t *d_recs, int reply,
                hipStream_t s);

// single-process rehearsal of shard_probe for W shards on one device (device copies in place
// of the RCCL transfers): the routing, offsets and permutations are the same code
int shard_init_loopback(ShardComm &c, int rank, int world, int chunks);
int shard_probe_loopback(const std::vector<ShardComm *> &cs, const std::vector<const DevTable *> &ts,
                         const ProbeTuning &tune, const std::vector<const uint64_t *> &keys,
                         const std::vector<const uint32_t *> &rids, const std::vector<uint64_t> &n,
                         const std::vector<stage_probe_out_dev *> &outs, std::vector<uint8_t *> recs, int reply,
                         hipStream_t s);

void set_error(const std::string &msg);

}  // namespace stage
