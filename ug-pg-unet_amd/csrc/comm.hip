// RCCL communicator of the data-parallel path (SURVEY.md §8b "ugpg_comm_{init,allreduce,
// destroy}", §8e).  The reference is single-process (no collectives anywhere); this is the
// exchange step the build adds: a SUM/AVG all-reduce of the flat gradient buffer and a
// broadcast for replica synchronisation, over RCCL (xGMI inside a node), stream-ordered on
// the caller's HIP stream, no allocation, no host synchronisation.  Rendezvous: rank 0
// creates the unique id (ugpg_comm_unique_id) and hands its bytes to the other ranks by
// any out-of-band channel (ugpg/dist.py uses the torch.distributed store).
#include <rccl/rccl.h>

#include <cstring>
#include <new>

#include "common.h"

namespace ugpg {
namespace {
struct Comm {
    ncclComm_t nc;
    int rank, nranks, device;
};

int nccl_status(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return UGPG_OK;
    set_error("%s: %s", what, ncclGetErrorString(r));
    return UGPG_ERR_COMM;
}

bool nccl_type(int dtype, ncclDataType_t& t, size_t& bytes) {
    switch (dtype) {
        case UGPG_DT_F32: t = ncclFloat32; bytes = 4; return true;
        case UGPG_DT_BF16: t = ncclBfloat16; bytes = 2; return true;
        case UGPG_DT_F64: t = ncclFloat64; bytes = 8; return true;
        case UGPG_DT_I64: t = ncclInt64; bytes = 8; return true;
        default: return false;
    }
}
}  // namespace
}  // namespace ugpg

using namespace ugpg;

extern "C" size_t ugpg_comm_id_bytes(void) { return sizeof(ncclUniqueId); }

extern "C" int ugpg_comm_unique_id(unsigned char* out, size_t n) {
    if (!out || n < sizeof(ncclUniqueId)) {
        set_error("comm_unique_id: buffer of %zu bytes < %zu", n, sizeof(ncclUniqueId));
        return UGPG_ERR_INVALID;
    }
    ncclUniqueId id;
    if (int e = nccl_status(ncclGetUniqueId(&id), "comm_unique_id")) return e;
    std::memcpy(out, &id, sizeof(id));
    return UGPG_OK;
}

extern "C" int ugpg_comm_init(ugpg_comm_t* comm, int nranks, int rank, const unsigned char* id,
                              size_t id_bytes, int device) {
    if (!comm || !id || id_bytes < sizeof(ncclUniqueId) || nranks < 1 || rank < 0 ||
        rank >= nranks || device < 0) {
        set_error("comm_init: bad arguments (nranks %d rank %d device %d)", nranks, rank, device);
        return UGPG_ERR_INVALID;
    }
    *comm = nullptr;
    if (hipSetDevice(device) != hipSuccess) {
        set_error("comm_init: hipSetDevice(%d) failed", device);
        return UGPG_ERR_COMM;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    Comm* c = new (std::nothrow) Comm{nullptr, rank, nranks, device};
    if (!c) {
        set_error("comm_init: out of host memory");
        return UGPG_ERR_COMM;
    }
    if (int e = nccl_status(ncclCommInitRank(&c->nc, nranks, uid, rank), "comm_init")) {
        delete c;
        return e;
    }
    *comm = reinterpret_cast<ugpg_comm_t>(c);
    return UGPG_OK;
}

extern "C" int ugpg_comm_allreduce(ugpg_comm_t comm, const void* send, void* recv, size_t count,
                                   int dtype, int op, void* stream) {
    Comm* c = reinterpret_cast<Comm*>(comm);
    ncclDataType_t t;
    size_t bytes;
    if (!c || !send || !recv || !nccl_type(dtype, t, bytes) || op < UGPG_OP_SUM ||
        op > UGPG_OP_MAX) {
        set_error("comm_allreduce: bad arguments (dtype %d op %d)", dtype, op);
        return UGPG_ERR_INVALID;
    }
    if (count == 0) return UGPG_OK;
    const ncclRedOp_t r = op == UGPG_OP_SUM ? ncclSum : op == UGPG_OP_AVG ? ncclAvg : ncclMax;
    return nccl_status(ncclAllReduce(send, recv, count, t, r, c->nc, as_stream(stream)),
                       "comm_allreduce");
}

extern "C" int ugpg_comm_broadcast(ugpg_comm_t comm, const void* send, void* recv, size_t count,
                                   int dtype, int root, void* stream) {
    Comm* c = reinterpret_cast<Comm*>(comm);
    ncclDataType_t t;
    size_t bytes;
    if (!c || !recv || (c->rank == root && !send) || !nccl_type(dtype, t, bytes) || root < 0 ||
        root >= c->nranks) {
        set_error("comm_broadcast: bad arguments (dtype %d root %d)", dtype, root);
        return UGPG_ERR_INVALID;
    }
    if (count == 0) return UGPG_OK;
    return nccl_status(ncclBroadcast(send, recv, count, t, root, c->nc, as_stream(stream)),
                       "comm_broadcast");
}

extern "C" int ugpg_comm_destroy(ugpg_comm_t comm) {
    Comm* c = reinterpret_cast<Comm*>(comm);
    if (!c) return UGPG_OK;
    const int e = nccl_status(ncclCommDestroy(c->nc), "comm_destroy");
    delete c;
    return e;
}
