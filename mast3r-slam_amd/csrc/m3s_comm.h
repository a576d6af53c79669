// m3s_comm.h -- RCCL communicator used for the per-iteration Hessian all-reduce.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace m3s {
// Sum-all-reduce of `count` doubles in place on `stream` (RCCL ring over xGMI).
int comm_allreduce_sum_f64(void* comm, double* buf, size_t count, hipStream_t stream);
}  // namespace m3s
