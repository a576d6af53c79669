// comm.hip -- RCCL (librccl.so.1, resolved with dlopen so the single-GPU path has no RCCL
// dependency) for edge-sharded Gauss-Newton: one in-place f64 sum all-reduce of the
// compact block-sparse system per iteration, enqueued on the GN stream (no host sync).
// When torch is imported first, dlopen returns torch's already-loaded RCCL.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/m3s_backend.h"
#include "m3s_comm.h"
#include "m3s_common.h"

namespace {

typedef int nccl_result_t;
typedef struct { char internal[M3S_COMM_ID_BYTES]; } nccl_unique_id_t;
typedef void* nccl_comm_t;
constexpr int kNcclFloat64 = 8;  // ncclFloat64 (rccl.h)
constexpr int kNcclSum = 0;      // ncclSum

struct Rccl {
    void* h = nullptr;
    nccl_result_t (*get_unique_id)(nccl_unique_id_t*) = nullptr;
    nccl_result_t (*comm_init_rank)(nccl_comm_t*, int, nccl_unique_id_t, int) = nullptr;
    nccl_result_t (*comm_destroy)(nccl_comm_t) = nullptr;
    nccl_result_t (*all_reduce)(const void*, void*, size_t, int, int, nccl_comm_t,
                                hipStream_t) = nullptr;
    const char* (*err_str)(nccl_result_t) = nullptr;
};

Rccl* rccl() {
    static Rccl r;
    static bool tried = false;
    if (!tried) {
        tried = true;
        const char* names[] = {"librccl.so.1", "librccl.so"};
        for (const char* n : names) {
            r.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
            if (r.h) break;
        }
        if (r.h) {
            r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.h, "ncclGetUniqueId");
            r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.h, "ncclCommInitRank");
            r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
            r.all_reduce = (decltype(r.all_reduce))dlsym(r.h, "ncclAllReduce");
            r.err_str = (decltype(r.err_str))dlsym(r.h, "ncclGetErrorString");
        }
    }
    if (!r.h || !r.get_unique_id || !r.comm_init_rank || !r.all_reduce) return nullptr;
    return &r;
}

const char* estr(Rccl* r, nccl_result_t e) { return (r && r->err_str) ? r->err_str(e) : "?"; }

}  // namespace

namespace m3s {
int comm_allreduce_sum_f64(void* comm, double* buf, size_t count, hipStream_t stream) {
    Rccl* r = rccl();
    if (!r) {
        set_error("RCCL not available (dlopen librccl.so.1 failed)");
        return M3S_ERR_COMM;
    }
    nccl_result_t e = r->all_reduce(buf, buf, count, kNcclFloat64, kNcclSum, (nccl_comm_t)comm, stream);
    if (e != 0) {
        set_error("ncclAllReduce failed: %s", estr(r, e));
        return M3S_ERR_COMM;
    }
    return M3S_OK;
}
}  // namespace m3s

extern "C" int m3s_comm_get_unique_id(void* id_out) {
    Rccl* r = rccl();
    if (!r) {
        m3s::set_error("RCCL not available (dlopen librccl.so.1 failed)");
        return M3S_ERR_COMM;
    }
    nccl_unique_id_t id;
    nccl_result_t e = r->get_unique_id(&id);
    if (e != 0) {
        m3s::set_error("ncclGetUniqueId failed: %s", estr(r, e));
        return M3S_ERR_COMM;
    }
    std::memcpy(id_out, id.internal, M3S_COMM_ID_BYTES);
    return M3S_OK;
}

extern "C" int m3s_comm_init(const void* id_in, int nranks, int rank, void** comm_out) {
    Rccl* r = rccl();
    if (!r) {
        m3s::set_error("RCCL not available (dlopen librccl.so.1 failed)");
        return M3S_ERR_COMM;
    }
    nccl_unique_id_t id;
    std::memcpy(id.internal, id_in, M3S_COMM_ID_BYTES);
    nccl_comm_t c = nullptr;
    nccl_result_t e = r->comm_init_rank(&c, nranks, id, rank);
    if (e != 0) {
        m3s::set_error("ncclCommInitRank failed: %s", estr(r, e));
        return M3S_ERR_COMM;
    }
    *comm_out = c;
    return M3S_OK;
}

extern "C" int m3s_comm_destroy(void* comm) {
    Rccl* r = rccl();
    if (!r || !r->comm_destroy) return M3S_ERR_COMM;
    return r->comm_destroy((nccl_comm_t)comm) == 0 ? M3S_OK : M3S_ERR_COMM;
}
