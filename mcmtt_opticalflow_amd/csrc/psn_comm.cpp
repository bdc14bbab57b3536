// RCCL (over xGMI) all-gather of fixed-size per-camera tracklet slots.
//
// The reference hands every camera's stTrack2DResult to the 3D associator
// in-process (std::vector<stTrack2DResult> result2D, psn_where/PSNWhere.cpp:253,
// 264, 269; consumed at PSNWhere_Associator3D.cpp:1105-1116 with index == camID).
// With one camera per GPU the same hand-off becomes ONE ncclAllGather per frame
// of a fixed-size slot per rank, so the gathered buffer is ordered by rank ==
// camera index as Associator3D requires.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <new>

#include "psn_lk.h"

struct psn_comm {
    ncclComm_t comm = nullptr;
    int device = 0;
    int nranks = 0, rank = 0;
};

static_assert(sizeof(ncclUniqueId) <= PSN_COMM_UNIQUE_ID_BYTES, "unique id size");

extern "C" {

int psn_comm_get_unique_id(void *id_out) {
    if (!id_out) return PSN_LK_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return PSN_LK_ERR_COMM;
    memset(id_out, 0, PSN_COMM_UNIQUE_ID_BYTES);
    memcpy(id_out, &id, sizeof(id));
    return PSN_LK_OK;
}

int psn_comm_init(int nranks, int rank, int device, const void *unique_id, psn_comm **out) {
    if (!out || !unique_id || nranks <= 0 || rank < 0 || rank >= nranks) return PSN_LK_ERR_ARG;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return PSN_LK_ERR_HIP;
    psn_comm *c = new (std::nothrow) psn_comm();
    if (!c) return PSN_LK_ERR_NOMEM;
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    if (ncclCommInitRank(&c->comm, nranks, id, rank) != ncclSuccess) {
        delete c;
        return PSN_LK_ERR_COMM;
    }
    c->device = device;
    c->nranks = nranks;
    c->rank = rank;
    *out = c;
    return PSN_LK_OK;
}

int psn_comm_allgather(psn_comm *c, const void *d_send, void *d_recv, size_t bytes_per_rank, void *hip_stream) {
    if (!c || !d_send || !d_recv) return PSN_LK_ERR_ARG;
    if (hipSetDevice(c->device) != hipSuccess) return PSN_LK_ERR_HIP;
    if (ncclAllGather(d_send, d_recv, bytes_per_rank, ncclUint8, c->comm, (hipStream_t)hip_stream) != ncclSuccess)
        return PSN_LK_ERR_COMM;
    return PSN_LK_OK;
}

void psn_comm_destroy(psn_comm *c) {
    if (!c) return;
    if (c->comm) ncclCommDestroy(c->comm);
    delete c;
}

}  // extern "C"
