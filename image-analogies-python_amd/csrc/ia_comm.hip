// ia_comm.hip — multi-GPU exchange for the sharded A-database.
// One process per GPU; the DB rows of a level are split contiguously over ranks.  Each
// wave every rank produces, per query, the exact (fp64 distance, global row) winner of its
// shard and that row's weighted distance (ShardRec); one RCCL all-gather over xGMI (M x
// 32 B per rank, latency-bound) gives every rank all shards' records, and k_finish reduces
// them with the same lexicographic (distance, lowest row) rule as np.argmin.  Coherence /
// kappa / update then run identically on every rank from replicated state: no further
// collective.
//
// The second form of the same exchange is device-side (PeerView, ia_internal.h): each rank's
// receive box is IPC-mapped into every rank; the exact stage's kernel publishes its winner
// into every box, and k_peer_finish collects all ranks' winners from its own box and
// finishes the pixel — no host call and no collective kernel per wave.
#include "ia_finish.h"

#include <rccl/rccl.h>

#include <cstring>

namespace ia {

struct Peer {
    PeerView v{};                  // device view (box pointers of all ranks)
    unsigned long long *mine = nullptr;
    size_t bytes = 0;
    int mem_kind = 0;              // 0 uncached, 1 fine-grained, 2 plain device memory
    unsigned int epoch = 0;        // host counter: one per wave, identical on every rank
};
struct Comm {
    ncclComm_t c;
    int nranks, rank;
    Peer *peer;                    // non-null: the device-side exchange (no RCCL)
};

static int nccl_fail(ncclResult_t r, const char *what) {
    set_error(std::string(what) + ": " + ncclGetErrorString(r));
    return IA_E_COMM;
}

int comm_nranks(void *comm) { return comm ? reinterpret_cast<Comm *>(comm)->nranks : 1; }

int comm_peer_mcap(void *comm) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    return c && c->peer ? c->peer->v.mcap : 0;
}

// the device-side exchange's view for the next wave (nranks 0: an RCCL communicator)
PeerView comm_peer_wave(void *comm) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    if (!c || !c->peer) return PeerView{};
    PeerView v = c->peer->v;
    v.epoch = ++c->peer->epoch;
    return v;
}

// handshake: every rank publishes (rank, rank) as query 0 of one wave and collects all;
// then each lane checks rank g's granules carry exactly (g, g)
__global__ __launch_bounds__(64) void k_peer_check(PeerView p, int *ok) {
    const int lane = threadIdx.x;
    peer_publish(p, 0, (double)p.rank, p.rank, lane);
    double d = INFINITY;
    long long i = 0x7fffffffffffffffLL;
    const bool got = peer_collect(p, 0, lane, d, i);
    bool mine = true;
    if (got && lane < p.nranks) {
        const unsigned long long *c = peer_cell(peer_box(p, p.rank), p, lane, 0);
        const unsigned long long g0 = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long g1 = __hip_atomic_load(c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long g2 = __hip_atomic_load(c + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const double dg = __longlong_as_double((long long)(((g1 & 0xffffffffULL) << 32) | (g0 & 0xffffffffULL)));
        mine = dg == (double)lane && (long long)(g2 & 0xffffffffULL) == lane;
    }
    const bool all = __all(mine);
    if (lane == 0) *ok = got && all && d == 0.0 && i == 0;
}

// protocol stress (diagnostic): wave w, query q, rank g publishes d = 1 + ((w * 7 + q * 3
// + g * 5) % 13), row = (g << 24) | ((w & 0xfff) << 12) | q; every collected granule is
// checked against that, and the minimum against the expected rank
__device__ __forceinline__ double stress_d(int w, int q, int g) { return 1.0 + (double)((w * 7 + q * 3 + g * 5) % 13); }
__device__ __forceinline__ long long stress_row(int w, int q, int g) {
    return ((long long)g << 24) | ((long long)(w & 0xfff) << 12) | q;
}
__global__ __launch_bounds__(64) void k_peer_stress(PeerView p, int w, int *bad) {
    const int q = blockIdx.x, lane = threadIdx.x;
    peer_publish(p, q, stress_d(w, q, p.rank), stress_row(w, q, p.rank), lane);
    double d = INFINITY;
    long long i = 0x7fffffffffffffffLL;
    const bool got = peer_collect(p, q, lane, d, i);
    bool fine = got;
    if (got && lane < p.nranks) {
        const unsigned long long *c = peer_cell(peer_box(p, p.rank), p, lane, q);
        const unsigned long long g0 = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long g1 = __hip_atomic_load(c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long g2 = __hip_atomic_load(c + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const double dg = __longlong_as_double((long long)(((g1 & 0xffffffffULL) << 32) | (g0 & 0xffffffffULL)));
        fine = dg == stress_d(w, q, lane) && (long long)(g2 & 0xffffffffULL) == stress_row(w, q, lane);
    }
    double ed = INFINITY;
    long long ei = 0x7fffffffffffffffLL;
    for (int g = 0; g < p.nranks; ++g) fin_best(ed, ei, stress_d(w, q, g), stress_row(w, q, g));
    const bool all = __all(fine);
    if (lane == 0 && !(all && d == ed && i == ei)) atomicAdd(bad, 1);
}

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
    Comm *c = new Comm{nullptr, nranks, rank, nullptr};
    ncclResult_t r = ncclCommInitRank(&c->c, nranks, id, rank);
    if (r != ncclSuccess) { delete c; return nccl_fail(r, "ncclCommInitRank"); }
    *comm = c;
    return IA_OK;
}

int ia_comm_destroy(void *comm) {
    if (!comm) return IA_OK;
    Comm *c = reinterpret_cast<Comm *>(comm);
    if (c->peer) {
        Peer *p = c->peer;
        hipError_t e = hipDeviceSynchronize();
        for (int g = 0; g < c->nranks; ++g)
            if (g != c->rank && p->v.box[g]) {
                const hipError_t e2 = hipIpcCloseMemHandle(p->v.box[g]);
                if (e == hipSuccess) e = e2;
            }
        if (p->mine) { const hipError_t e2 = hipFree(p->mine); if (e == hipSuccess) e = e2; }
        if (p->v.err) { const hipError_t e2 = hipFree(p->v.err); if (e == hipSuccess) e = e2; }
        if (p->v.trace) { const hipError_t e2 = hipFree(p->v.trace); if (e == hipSuccess) e = e2; }
        delete p;
        delete c;
        IA_HIP(e);
        return IA_OK;
    }
    ncclResult_t r = ncclCommDestroy(c->c);
    delete c;
    if (r != ncclSuccess) return nccl_fail(r, "ncclCommDestroy");
    return IA_OK;
}

int ia_peer_create(int nranks, int rank, int mcap, void **comm, uint8_t handle[64]) {
    IA_ARG(comm && handle && nranks >= 1 && nranks <= IA_PEER_MAX && rank >= 0 && rank < nranks &&
               mcap >= 1,
           "ia_peer_create: bad args");
    static_assert(sizeof(hipIpcMemHandle_t) == 64, "hipIpcMemHandle_t size");
    Peer *p = new Peer;
    p->bytes = peer_box_words(nranks, mcap) * sizeof(unsigned long long);
    // uncached device memory: a peer's stores and this rank's polls meet in HBM, never in a
    // stale cache line of either GPU; fine-grained, then plain memory if the device refuses
    const unsigned flags[2] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
    void *m = nullptr;
    hipError_t e = hipErrorOutOfMemory;
    for (int k = 0; k < 2 && e != hipSuccess; ++k) {
        e = hipExtMallocWithFlags(&m, p->bytes, flags[k]);
        p->mem_kind = k;
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        // plain (coarse-grained) memory: another GPU's stores need not become visible to
        // this GPU's polls (they may be served from its L2), so across GPUs this form is
        // refused and every rank takes the RCCL exchange; ranks sharing one GPU
        // (IA_SHARE_GPU=1) meet in that GPU's own memory and may use it
        if (nranks > 1 && !env_int("IA_SHARE_GPU", 0)) {
            delete p;
            set_error("ia_peer_create: neither uncached nor fine-grained device memory for the "
                      "receive box (plain memory is not coherent across GPUs)");
            return IA_E_UNSUPPORTED;
        }
        e = hipMalloc(&m, p->bytes);
        p->mem_kind = 2;
    }
    if (e != hipSuccess) { delete p; IA_HIP(e); }
    p->mine = reinterpret_cast<unsigned long long *>(m);
    unsigned int *err = nullptr;
    e = hipMalloc(&err, 256);
    if (e == hipSuccess) e = hipMemset(err, 0, 256);
    if (e == hipSuccess) e = hipMemset(p->mine, 0, p->bytes);   // epochs start at 1
    if (e == hipSuccess && env_int("IA_PEER_TRACE", 0)) {
        double *tr = nullptr;
        e = hipMalloc(&tr, 1024 * 8 * 12 * sizeof(double));
        p->v.trace = tr;
        if (e == hipSuccess) e = hipMemset(tr, 0, 1024 * 8 * 12 * sizeof(double));
    }
    hipIpcMemHandle_t h;
    if (e == hipSuccess) e = hipIpcGetMemHandle(&h, p->mine);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(p->mine);
        if (err) (void)hipFree(err);
        delete p;
        IA_HIP(e);
    }
    memcpy(handle, &h, 64);
    p->v.err = err;
    p->v.nranks = nranks;
    p->v.rank = rank;
    p->v.mcap = mcap;
    p->v.box[rank] = p->mine;
    *comm = new Comm{nullptr, nranks, rank, p};
    return IA_OK;
}

int ia_peer_connect(void *comm, const uint8_t *handles) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    IA_ARG(c && c->peer && handles, "ia_peer_connect: not a peer exchange");
    for (int g = 0; g < c->nranks; ++g) {
        if (g == c->rank) continue;
        hipIpcMemHandle_t h;
        memcpy(&h, handles + 64 * g, 64);
        void *p = nullptr;
        IA_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        c->peer->v.box[g] = reinterpret_cast<unsigned long long *>(p);
    }
    return IA_OK;
}

int ia_peer_check(void *comm, void *stream) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    IA_ARG(c && c->peer, "ia_peer_check: not a peer exchange");
    hipStream_t st = S(stream);
    int *ok = nullptr;
    IA_HIP(hipMalloc(&ok, sizeof(int)));
    k_peer_check<<<1, 64, 0, st>>>(comm_peer_wave(comm), ok);
    hipError_t e = hipGetLastError();
    int h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, ok, sizeof(int), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(ok);
    IA_HIP(e);
    if (!h) {
        set_error("ia_peer_check: the ranks' records did not arrive (peer exchange unusable)");
        return IA_E_COMM;
    }
    return IA_OK;
}

int ia_peer_status(void *comm) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    IA_ARG(c && c->peer, "ia_peer_status: not a peer exchange");
    unsigned int e = 0;
    IA_HIP(hipDeviceSynchronize());
    IA_HIP(hipMemcpy(&e, c->peer->v.err, sizeof(e), hipMemcpyDeviceToHost));
    if (e) {
        set_error("peer exchange: a wait for another rank's records timed out");
        return IA_E_TIMEOUT;
    }
    return IA_OK;
}

int ia_diag_peer_stress(void *comm, int nwaves, int M, int *bad, void *stream) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    IA_ARG(c && c->peer && bad && nwaves >= 1 && M >= 1 && M <= c->peer->v.mcap && M < 4096,
           "ia_diag_peer_stress: bad args");
    hipStream_t st = S(stream);
    int *dbad = nullptr;
    IA_HIP(hipMalloc(&dbad, sizeof(int)));
    hipError_t e = hipMemsetAsync(dbad, 0, sizeof(int), st);
    for (int w = 0; w < nwaves && e == hipSuccess; ++w) {
        k_peer_stress<<<M, 64, 0, st>>>(comm_peer_wave(comm), w, dbad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(bad, dbad, sizeof(int), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(dbad);
    IA_HIP(e);
    return IA_OK;
}

int ia_diag_peer_trace(void *comm, double *out) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    IA_ARG(c && c->peer && c->peer->v.trace && out, "ia_diag_peer_trace: no trace (IA_PEER_TRACE=1)");
    IA_HIP(hipDeviceSynchronize());
    IA_HIP(hipMemcpy(out, c->peer->v.trace, 1024 * 8 * 12 * sizeof(double), hipMemcpyDeviceToHost));
    return IA_OK;
}

int ia_peer_mem_kind(void *comm) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    return c && c->peer ? c->peer->mem_kind : -1;
}

int ia_comm_nranks(void *comm) { return comm_nranks(comm); }

}  // extern "C"
