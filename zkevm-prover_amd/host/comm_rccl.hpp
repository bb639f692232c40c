// zkgpu_comm over RCCL (xGMI between the GPUs of a node); included by
// starks.cpp.  librccl is opened at run time, so the prover library carries
// no link dependency on it and a process that never shards never loads it.
// One exchange = ncclSend / ncclRecv of every operation inside one
// ncclGroupStart / ncclGroupEnd, enqueued on the zkgpu stream: RCCL matches
// the sends and receives of a peer pair in order, and later zkgpu work on the
// stream is ordered after the transfers.
#include <dlfcn.h>
#include <rccl/rccl.h>

namespace zkgpu_host {

struct RcclApi {
    void *so = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
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

struct RcclCtx {
    ncclComm_t comm = nullptr;
};

static int rccl_exchange(void *ctx, const zkgpu_comm_op *ops, uint32_t n_ops)
{
    ncclComm_t c = ((RcclCtx *)ctx)->comm;
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
    if (first != ncclSuccess) return fail("ncclSend/ncclRecv: %s", g_rccl.error_string(first));
    if (r != ncclSuccess) return fail("ncclGroupEnd: %s", g_rccl.error_string(r));
    return 0;
}

}  // namespace zkgpu_host
