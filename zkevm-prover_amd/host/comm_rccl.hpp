// zkgpu_comm over RCCL (xGMI between the GPUs of a node); included by
// starks.cpp.  librccl is opened at run time, so the prover library carries
// no link dependency on it and a process that never shards never loads it.
// One exchange = ncclSend / ncclRecv of every operation inside one
// ncclGroupStart / ncclGroupEnd, enqueued on the zkgpu stream: RCCL matches
// the sends and receives of a peer pair in order, and later zkgpu work on the
// stream is ordered after the transfers.
//
// Failure: a peer that failed (or never reaches this exchange) leaves this
// rank's receive kernels spinning.  So each exchange waits for its transfers
// with a deadline (comm_wait, ZKGPU_COMM_TIMEOUT_S), polling the
// communicator's asynchronous error; on an error or the deadline it aborts
// the communicator (ncclCommAbort: the transfer kernels see the abort flag and
// exit) and fails, and every later exchange fails at once.  A rank whose proof
// fails locally aborts through zkgpu_comm.abort (ShardedStarks::prove).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <thread>

namespace zkgpu_host {

struct RcclApi {
    void *so = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
    decltype(&ncclCommGetAsyncError) get_async_error = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;

    int load()
    {
        if (so) return 0;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return fail("zkgpu_comm_rccl: cannot open librccl: %s", dlerror());
#define ZK_SYM(f, name)                                                                      \
    f = (decltype(f))dlsym(h, name);                                                         \
    if (!f) return fail("zkgpu_comm_rccl: librccl lacks %s", name);
        ZK_SYM(get_unique_id, "ncclGetUniqueId");
        ZK_SYM(comm_init_rank, "ncclCommInitRank");
        ZK_SYM(comm_destroy, "ncclCommDestroy");
        ZK_SYM(comm_abort, "ncclCommAbort");
        ZK_SYM(get_async_error, "ncclCommGetAsyncError");
        ZK_SYM(send, "ncclSend");
        ZK_SYM(recv, "ncclRecv");
        ZK_SYM(group_start, "ncclGroupStart");
        ZK_SYM(group_end, "ncclGroupEnd");
        ZK_SYM(error_string, "ncclGetErrorString");
#undef ZK_SYM
        so = h;
        return 0;
    }
};

static RcclApi g_rccl;

// (comm_timeout_s / comm_wait: comm_host.hpp, included first)

struct RcclCtx {
    ncclComm_t comm = nullptr;
    bool failed = false;   // an exchange failed or this rank aborted: every later one fails
    bool aborted = false;  // ncclCommAbort ran (the communicator is gone)
    hipEvent_t done = nullptr;
};

static int rccl_abort(void *vctx)
{
    RcclCtx *c = (RcclCtx *)vctx;
    c->failed = true;
    if (c->comm && !c->aborted) {
        (void)g_rccl.comm_abort(c->comm);
        c->aborted = true;
        c->comm = nullptr;
    }
    return 0;
}

static int rccl_exchange(void *vctx, const zkgpu_comm_op *ops, uint32_t n_ops)
{
    RcclCtx *ctx = (RcclCtx *)vctx;
    if (ctx->failed)
        return fail("rccl exchange: the communicator failed earlier (a timed-out or failed exchange, or this rank "
                    "aborted)");
    ncclComm_t c = ctx->comm;
    hipStream_t s = (hipStream_t)zkgpu_get_stream();
    ncclResult_t r = g_rccl.group_start();
    if (r != ncclSuccess) return fail("ncclGroupStart: %s", g_rccl.error_string(r));
    ncclResult_t first = ncclSuccess;
    for (uint32_t k = 0; k < n_ops; k++) {
        const zkgpu_comm_op &o = ops[k];
        r = o.send ? g_rccl.send(o.buf, o.bytes, ncclUint8, o.peer, c, s)
                   : g_rccl.recv(o.buf, o.bytes, ncclUint8, o.peer, c, s);
        if (r != ncclSuccess && first == ncclSuccess) first = r;
    }
    r = g_rccl.group_end();
    if (first != ncclSuccess || r != ncclSuccess) {
        rccl_abort(ctx);
        return fail("ncclSend/ncclRecv/ncclGroupEnd: %s", g_rccl.error_string(first != ncclSuccess ? first : r));
    }
    if (!n_ops) return 0;
    if (!ctx->done && hipEventCreateWithFlags(&ctx->done, hipEventDisableTiming) != hipSuccess) {
        rccl_abort(ctx);
        return fail("rccl exchange: hipEventCreate failed");
    }
    if (hipEventRecord(ctx->done, s) != hipSuccess) {
        rccl_abort(ctx);
        return fail("rccl exchange: hipEventRecord failed");
    }
    ncclResult_t ae = ncclSuccess;
    const double limit = comm_timeout_s();
    const int w = comm_wait(
        [&]() {
            const hipError_t q = hipEventQuery(ctx->done);
            return q == hipSuccess ? 1 : q == hipErrorNotReady ? 0 : -1;
        },
        [&]() {
            return g_rccl.get_async_error(c, &ae) != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress);
        },
        limit);
    if (w) {
        rccl_abort(ctx);
        if (w == -2)
            return fail("rccl exchange of %u operations: not complete after %.0f s (a peer failed or stopped; "
                        "communicator aborted)", n_ops, limit);
        return fail("rccl exchange of %u operations failed: %s (communicator aborted)", n_ops,
                    ae != ncclSuccess ? g_rccl.error_string(ae) : "stream error");
    }
    return 0;
}

}  // namespace zkgpu_host
