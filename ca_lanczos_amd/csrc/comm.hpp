// comm.hpp -- communicators for the row-slab distributed path.
//
// Two implementations behind one interface:
//  * RCCL over xGMI (kind 1): ncclAllReduce for the fused Gram blocks,
//    grouped ncclSend/ncclRecv for the per-SpMV halo, on the context stream.
//  * host-staged callbacks (kind 2): device buffers are staged through pinned
//    host memory and handed to user callbacks (e.g. torch.distributed/gloo).
//    Used to test the distributed driver with several ranks on one GPU.
#pragma once

#include <rccl/rccl.h>

#include <vector>

#include "cal_internal.hpp"

namespace cal {

struct Comm {
    int nranks = 1;
    int rank = 0;
    int kind = 0;  // 1 rccl, 2 host
    ncclComm_t nccl = nullptr;
    cal_allreduce_fn ar = nullptr;
    cal_exchange_fn ex = nullptr;
    void* user = nullptr;
    double* h_stage = nullptr;  // pinned
    size_t stage_cap = 0;
    // RCCL: the deep halo exchange runs here, overlapped with the interior
    // matrix powers (runtime.cpp powers_dev); ev_q: q ready, ev_halo: received
    hipStream_t stream = nullptr;
    hipEvent_t ev_q = nullptr, ev_halo = nullptr;
    // counters since the last cal_comm_stats(reset): collectives issued and
    // the doubles they carry (the multi-rank bench line)
    int64_t n_allreduce = 0, d_allreduce = 0, n_halo = 0, d_halo = 0;
};

void comm_destroy(cal_ctx* c);
// Host-vector exchange with one peer (setup phase; both sides call it).
int comm_exchange_host(cal_ctx* c, int peer, const std::vector<double>& send, std::vector<double>& recv);
// Host-vector sum-allreduce (setup phase).
int comm_allreduce_host(cal_ctx* c, std::vector<double>& buf);

}  // namespace cal
