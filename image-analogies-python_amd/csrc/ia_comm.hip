// ia_comm.hip — multi-GPU exchange for the sharded A-database.
// One process per GPU; the DB rows of a level are split contiguously over ranks.  Each
// wave every rank produces, per query, the exact (fp64 distance, global row) winner of its
// shard and that row's weighted distance (ShardRec); one RCCL all-gather over xGMI (M x
// 32 B per rank, latency-bound) gives every rank all shards' records, and k_finish reduces
// them with the same lexicographic (distance, lowest row) rule as np.argmin.  Coherence /
// kappa / update then run identically on every rank from replicated state: no further
// collective.
#include "ia_internal.h"

#include <rccl/rccl.h>

#include <cstring>

namespace ia {

struct Comm {
    ncclComm_t c;
    int nranks, rank;
};

static int nccl_fail(ncclResult_t r, const char *what) {
    set_error(std::string(what) + ": " + ncclGetErrorString(r));
    return IA_E_COMM;
}

int comm_nranks(void *comm) { return comm ? reinterpret_cast<Comm *>(comm)->nranks : 1; }

int comm_allgather(void *comm, const void *send, void *recv, size_t bytes, hipStream_t st) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    IA_ARG(bytes % 8 == 0, "comm_allgather: whole 8-byte words");
    ncclResult_t r = ncclAllGather(send, recv, bytes / 8, ncclUint64, c->c, st);
    if (r != ncclSuccess) return nccl_fail(r, "ncclAllGather");
    return IA_OK;
}

}  // namespace ia

using namespace ia;

extern "C" {

int ia_comm_unique_id(uint8_t out[128]) {
    IA_ARG(out, "ia_comm_unique_id: null");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
    memcpy(out, &id, 128);
    return IA_OK;
}

int ia_comm_init(const uint8_t uid[128], int nranks, int rank, void **comm) {
    IA_ARG(uid && comm && nranks >= 1 && rank >= 0 && rank < nranks, "ia_comm_init: bad args");
    ncclUniqueId id;
    memcpy(&id, uid, 128);
    Comm *c = new Comm{nullptr, nranks, rank};
    ncclResult_t r = ncclCommInitRank(&c->c, nranks, id, rank);
    if (r != ncclSuccess) { delete c; return nccl_fail(r, "ncclCommInitRank"); }
    *comm = c;
    return IA_OK;
}

int ia_comm_destroy(void *comm) {
    if (!comm) return IA_OK;
    Comm *c = reinterpret_cast<Comm *>(comm);
    ncclResult_t r = ncclCommDestroy(c->c);
    delete c;
    if (r != ncclSuccess) return nccl_fail(r, "ncclCommDestroy");
    return IA_OK;
}

int ia_comm_nranks(void *comm) { return comm_nranks(comm); }

}  // extern "C"
