// comm.hip -- the per-iteration collective of edge-sharded Gauss-Newton: an in-place all-gather
// of the ranks' per-edge records (default: every rank then assembles ALL edges in edge order, as
// one GPU does) or an in-place f64 sum all-reduce of the assembled block system.
//
// A communicator handle is one of
//   * RCCL (production): librccl.so.1 resolved with dlopen so the single-GPU path has no RCCL
//     dependency; the all-reduce is enqueued on the GN stream (no host sync).  When torch is
//     imported first, dlopen returns torch's already-loaded RCCL.
//   * host callback (test hook, m3s_comm_init_host): the stream is drained, the buffer staged
//     to pinned host memory, handed to the callback (e.g. a torch.distributed gloo
//     all_reduce), and copied back.  Lets several processes sharing one GPU (or a CPU-only
//     rehearsal of the exchange) run the product op's sharded path.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
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
    nccl_result_t (*all_gather)(const void*, void*, size_t, int, nccl_comm_t, hipStream_t) = nullptr;
    const char* (*err_str)(nccl_result_t) = nullptr;
    nccl_result_t (*comm_count)(nccl_comm_t, int*) = nullptr;
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
            r.all_gather = (decltype(r.all_gather))dlsym(r.h, "ncclAllGather");
            r.err_str = (decltype(r.err_str))dlsym(r.h, "ncclGetErrorString");
            r.comm_count = (decltype(r.comm_count))dlsym(r.h, "ncclCommCount");
        }
    }
    if (!r.h || !r.get_unique_id || !r.comm_init_rank || !r.all_reduce) return nullptr;
    return &r;
}

const char* estr(Rccl* r, nccl_result_t e) { return (r && r->err_str) ? r->err_str(e) : "?"; }

enum { kCommRccl = 1, kCommHost = 2 };
constexpr unsigned kCommMagic = 0x6d33636du;  // "m3cm"

struct Comm {
    unsigned magic = kCommMagic;
    int kind = 0;
    int nranks = 1, rank = 0;
    nccl_comm_t nccl = nullptr;
    m3s_host_allreduce_fn fn = nullptr;
    void* user = nullptr;
    double* host = nullptr;  // pinned staging buffer (host kind)
    size_t host_cap = 0;
};

Comm* as_comm(void* h) {
    Comm* c = static_cast<Comm*>(h);
    return (c && c->magic == kCommMagic) ? c : nullptr;
}

}  // namespace

namespace m3s {
bool comm_is_async(void* comm) {
    const Comm* c = as_comm(comm);
    return c != nullptr && c->kind == kCommRccl;
}

int comm_allreduce_sum_f64(void* comm, double* buf, size_t count, hipStream_t stream) {
    Comm* c = as_comm(comm);
    if (!c) {
        set_error("all-reduce: not an m3s communicator handle");
        return M3S_ERR_COMM;
    }
    if (count == 0) return M3S_OK;
    if (c->kind == kCommHost) {
        if (c->host_cap < count) {
            if (c->host) M3S_HIP_CHECK(hipHostFree(c->host));
            c->host = nullptr;
            c->host_cap = 0;
            M3S_HIP_CHECK(hipHostMalloc((void**)&c->host, count * sizeof(double), hipHostMallocDefault));
            c->host_cap = count;
        }
        M3S_HIP_CHECK(hipMemcpyAsync(c->host, buf, count * sizeof(double), hipMemcpyDeviceToHost, stream));
        M3S_HIP_CHECK(hipStreamSynchronize(stream));
        const int rc = c->fn(c->user, c->host, count);
        if (rc != 0) {
            set_error("host all-reduce callback failed (%d)", rc);
            return M3S_ERR_COMM;
        }
        M3S_HIP_CHECK(hipMemcpyAsync(buf, c->host, count * sizeof(double), hipMemcpyHostToDevice, stream));
        // the staging buffer is reused by the next call: the copy must have read it
        M3S_HIP_CHECK(hipStreamSynchronize(stream));
        return M3S_OK;
    }
    Rccl* r = rccl();
    if (!r) {
        set_error("RCCL not available (dlopen librccl.so.1 failed)");
        return M3S_ERR_COMM;
    }
    nccl_result_t e = r->all_reduce(buf, buf, count, kNcclFloat64, kNcclSum, c->nccl, stream);
    if (e != 0) {
        set_error("ncclAllReduce failed: %s", estr(r, e));
        return M3S_ERR_COMM;
    }
    return M3S_OK;
}

int comm_rank_size(void* comm, int* rank, int* nranks) {
    Comm* c = as_comm(comm);
    if (!c) {
        set_error("comm: not an m3s communicator handle");
        return M3S_ERR_COMM;
    }
    *rank = c->rank;
    *nranks = c->nranks;
    return M3S_OK;
}

int comm_allgather_f64(void* comm, double* buf, size_t count, hipStream_t stream) {
    Comm* c = as_comm(comm);
    if (!c) {
        set_error("all-gather: not an m3s communicator handle");
        return M3S_ERR_COMM;
    }
    if (count == 0 || c->nranks == 1) return M3S_OK;
    if (c->kind == kCommHost) {
        // test hook: the other ranks' blocks zeroed, then the sum all-reduce (x + 0 = x exactly)
        double* own = buf + (size_t)c->rank * count;
        if (c->rank > 0) M3S_HIP_CHECK(hipMemsetAsync(buf, 0, sizeof(double) * (size_t)c->rank * count, stream));
        const size_t after = (size_t)(c->nranks - 1 - c->rank) * count;
        if (after) M3S_HIP_CHECK(hipMemsetAsync(own + count, 0, sizeof(double) * after, stream));
        return comm_allreduce_sum_f64(comm, buf, count * (size_t)c->nranks, stream);
    }
    Rccl* r = rccl();
    if (!r || !r->all_gather) {
        set_error("RCCL all-gather not available (dlopen librccl.so.1 / ncclAllGather)");
        return M3S_ERR_COMM;
    }
    nccl_result_t e = r->all_gather(buf + (size_t)c->rank * count, buf, count, kNcclFloat64, c->nccl, stream);
    if (e != 0) {
        set_error("ncclAllGather failed: %s", estr(r, e));
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
    M3S_REQUIRE(comm_out, "comm init: null output");
    nccl_comm_t nc = nullptr;
    nccl_result_t e = r->comm_init_rank(&nc, nranks, id, rank);
    if (e != 0) {
        m3s::set_error("ncclCommInitRank failed: %s", estr(r, e));
        return M3S_ERR_COMM;
    }
    Comm* c = new Comm();
    c->kind = kCommRccl;
    c->nranks = nranks;
    c->rank = rank;
    c->nccl = nc;
    *comm_out = c;
    return M3S_OK;
}

extern "C" int m3s_comm_init_host(m3s_host_allreduce_fn fn, void* user, int nranks, int rank,
                                  void** comm_out) {
    M3S_REQUIRE(fn && comm_out, "comm init (host): null callback or output");
    M3S_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "comm init (host): bad rank %d of %d",
                rank, nranks);
    Comm* c = new Comm();
    c->kind = kCommHost;
    c->nranks = nranks;
    c->rank = rank;
    c->fn = fn;
    c->user = user;
    *comm_out = c;
    return M3S_OK;
}

extern "C" int m3s_comm_size(void* comm, int* nranks_out) {
    Comm* c = as_comm(comm);
    if (!c || !nranks_out) {
        m3s::set_error("comm size: not an m3s communicator handle");
        return M3S_ERR_COMM;
    }
    if (c->kind == kCommRccl) {
        Rccl* r = rccl();
        int n = 0;
        if (!r || !r->comm_count || r->comm_count(c->nccl, &n) != 0) {
            m3s::set_error("ncclCommCount failed");
            return M3S_ERR_COMM;
        }
        *nranks_out = n;
        return M3S_OK;
    }
    *nranks_out = c->nranks;
    return M3S_OK;
}

extern "C" int m3s_comm_destroy(void* comm) {
    Comm* c = as_comm(comm);
    if (!c) {
        m3s::set_error("comm destroy: not an m3s communicator handle");
        return M3S_ERR_COMM;
    }
    int rc = M3S_OK;
    if (c->kind == kCommRccl) {
        Rccl* r = rccl();
        if (!r || !r->comm_destroy || r->comm_destroy(c->nccl) != 0) rc = M3S_ERR_COMM;
    }
    if (c->host) (void)hipHostFree(c->host);
    c->magic = 0;
    delete c;
    return rc;
}
