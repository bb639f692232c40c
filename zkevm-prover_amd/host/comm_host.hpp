// zkgpu_comm through host shared memory between the processes of one machine;
// included by starks.cpp.  For ranks that cannot use RCCL -- several
// processes sharing one GPU (the multi-rank tests of the C++ driver), or a
// machine without xGMI peers.  Every rank owns an outbox in a POSIX shared
// memory segment: an exchange copies the rank's send slices into its outbox
// (device -> host, after the zkgpu stream drains), waits at a process-shared
// barrier, copies each receive from the sending rank's outbox (the k-th
// receive from a peer takes that peer's k-th send to this rank), and waits
// again so outboxes can be reused.  Capacity (bytes per rank and exchange) is
// fixed at creation; a larger exchange fails loudly.
#include <fcntl.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <thread>

namespace zkgpu_host {

struct HostCommHeader {
    std::atomic<uint32_t> ready;
    uint32_t world;
    uint64_t capacity;
    pthread_barrier_t barrier;
};

struct HostCommEntry {
    int32_t peer;
    uint32_t pad;
    uint64_t bytes, off;
};

static const uint32_t HOST_COMM_MAX_OPS = 1u << 16;

struct HostCommCtx {
    uint8_t *base = nullptr;
    uint64_t size = 0;
    uint32_t rank = 0, world = 0;
    uint64_t capacity = 0;

    static uint64_t header_bytes() { return (sizeof(HostCommHeader) + 4095) & ~4095ULL; }
    uint64_t box_bytes() const { return 8 + HOST_COMM_MAX_OPS * sizeof(HostCommEntry) + capacity; }
    HostCommHeader *hdr() const { return (HostCommHeader *)base; }
    uint8_t *box(uint32_t r) const { return base + header_bytes() + (uint64_t)r * box_bytes(); }
    uint64_t &n_entries(uint32_t r) const { return *(uint64_t *)box(r); }
    HostCommEntry *entries(uint32_t r) const { return (HostCommEntry *)(box(r) + 8); }
    uint8_t *data(uint32_t r) const { return box(r) + 8 + HOST_COMM_MAX_OPS * sizeof(HostCommEntry); }
    int wait() const
    {
        const int rc = pthread_barrier_wait(&hdr()->barrier);
        return (rc == 0 || rc == PTHREAD_BARRIER_SERIAL_THREAD) ? 0 : fail("host comm: barrier failed");
    }
};

static int host_exchange(void *vctx, const zkgpu_comm_op *ops, uint32_t n_ops)
{
    HostCommCtx &c = *(HostCommCtx *)vctx;
    uint64_t off = 0, n = 0;
    HostCommEntry *tab = c.entries(c.rank);
    for (uint32_t k = 0; k < n_ops; k++) {
        const zkgpu_comm_op &o = ops[k];
        if (o.peer < 0 || (uint32_t)o.peer >= c.world || (uint32_t)o.peer == c.rank)
            return fail("host comm: bad peer %d", o.peer);
        if (!o.send) continue;
        if (n == HOST_COMM_MAX_OPS || off + o.bytes > c.capacity)
            return fail("host comm: exchange exceeds the %llu-byte outbox", (unsigned long long)c.capacity);
        CK(zkgpu_memcpy_d2h(c.data(c.rank) + off, o.buf, o.bytes));
        tab[n++] = HostCommEntry{o.peer, 0, o.bytes, off};
        off += o.bytes;
    }
    c.n_entries(c.rank) = n;
    if (c.wait()) return -1;
    std::vector<uint64_t> cursor(c.world, 0);
    for (uint32_t k = 0; k < n_ops; k++) {
        const zkgpu_comm_op &o = ops[k];
        if (o.send) continue;
        const uint32_t s = (uint32_t)o.peer;
        const HostCommEntry *st = c.entries(s);
        const uint64_t ns = c.n_entries(s);
        uint64_t &i = cursor[s];
        while (i < ns && st[i].peer != (int32_t)c.rank) i++;
        if (i == ns) return fail("host comm: rank %u sent rank %u fewer slices than it receives", s, c.rank);
        if (st[i].bytes != o.bytes)
            return fail("host comm: slice of %llu bytes from rank %u, receive of %llu", (unsigned long long)st[i].bytes,
                        s, (unsigned long long)o.bytes);
        CK(zkgpu_memcpy_h2d(o.buf, c.data(s) + st[i].off, o.bytes));
        i++;
    }
    return c.wait();
}

}  // namespace zkgpu_host
