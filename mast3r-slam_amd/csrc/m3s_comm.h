// m3s_comm.h -- RCCL communicator used for the per-iteration Hessian all-reduce.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace m3s {
// Sum-all-reduce of `count` doubles in place on `stream` (RCCL ring over xGMI).
int comm_allreduce_sum_f64(void* comm, double* buf, size_t count, hipStream_t stream);
// This rank and the rank count of the handle (as created).
int comm_rank_size(void* comm, int* rank, int* nranks);
// All-gather of `count` doubles per rank on `stream`: rank r's block lands at buf + r * count, and
// the rank's own block is read from buf + rank * count (in place, ncclAllGather's convention).
int comm_allgather_f64(void* comm, double* buf, size_t count, hipStream_t stream);
// true when the handle's collectives are only enqueued on the stream (RCCL); the host-callback
// kind drains the stream and blocks the calling thread until every rank has arrived
bool comm_is_async(void* comm);
}  // namespace m3s
