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
#include <cstdlib>
#include <string>
#include <thread>

namespace zkgpu_host {

struct HostCommHeader {
    std::atomic<uint32_t> ready;
    uint32_t world;
    uint64_t capacity;
    uint64_t run;                 // this run's tag (run_tag_hash): a stale segment never matches
    // error[k % 3]: a rank failed inside exchange k.  One slot per exchange
    // (cleared two exchanges ahead, see host_exchange): a rank still reading
    // exchange k's flag never sees a failure a faster rank raised in k + 1
    std::atomic<uint32_t> error[3];
    pthread_barrier_t barrier;
};

// 64-bit tag of this run: ZKGPU_RUN_ID if set, else the launcher's pid
// (ranks started by one launcher share their parent)
static uint64_t run_tag_hash()
{
    const char *e = getenv("ZKGPU_RUN_ID");
    const std::string t = e && *e ? std::string(e) : "ppid" + std::to_string((long)getppid());
    uint64_t h = 1469598103934665603ULL;
    for (char ch : t) h = (h ^ (uint8_t)ch) * 1099511628211ULL;
    return h | 1;  // never 0 (a fresh segment)
}

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
    uint64_t seq = 0;  // exchanges done (the same on every rank: exchanges are collective)

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

// Every rank reaches both barriers whatever happens: a rank that fails
// raises this exchange's error flag and still waits, so one rank's error is
// every rank's non-zero return for the same exchange instead of a hang in the
// barrier.  Exchange k uses slot k % 3; after barrier 1 of exchange k every
// rank has finished exchange k - 1 (its reads included), so slot (k + 1) % 3
// -- last read in exchange k - 2 -- is cleared there, and no rank can raise it
// for exchange k + 1 before passing barrier 2 of k, which waits for every
// rank's clear.
static int host_exchange(void *vctx, const zkgpu_comm_op *ops, uint32_t n_ops)
{
    HostCommCtx &c = *(HostCommCtx *)vctx;
    HostCommHeader *h = c.hdr();
    std::atomic<uint32_t> &err = h->error[c.seq % 3];
    std::atomic<uint32_t> &next = h->error[(c.seq + 1) % 3];
    c.seq++;
    int rc = 0;
    uint64_t off = 0, n = 0;
    HostCommEntry *tab = c.entries(c.rank);
    for (uint32_t k = 0; k < n_ops && !rc; k++) {
        const zkgpu_comm_op &o = ops[k];
        if (o.peer < 0 || (uint32_t)o.peer >= c.world || (uint32_t)o.peer == c.rank) {
            rc = fail("host comm: bad peer %d", o.peer);
            break;
        }
        if (!o.send) continue;
        if (n == HOST_COMM_MAX_OPS || off + o.bytes > c.capacity) {
            rc = fail("host comm: exchange exceeds the %llu-byte outbox", (unsigned long long)c.capacity);
            break;
        }
        if (zkgpu_memcpy_d2h(c.data(c.rank) + off, o.buf, o.bytes)) {
            rc = fail("host comm: device -> outbox copy failed: %s", zkgpu_last_error());
            break;
        }
        tab[n++] = HostCommEntry{o.peer, 0, o.bytes, off};
        off += o.bytes;
    }
    c.n_entries(c.rank) = n;
    if (rc) err.store(1);
    if (c.wait()) return -1;
    next.store(0);
    if (err.load()) {
        (void)c.wait();
        return rc ? rc : fail("host comm: another rank failed in this exchange");
    }
    std::vector<uint64_t> cursor(c.world, 0);
    for (uint32_t k = 0; k < n_ops && !rc; k++) {
        const zkgpu_comm_op &o = ops[k];
        if (o.send) continue;
        const uint32_t s = (uint32_t)o.peer;
        const HostCommEntry *st = c.entries(s);
        const uint64_t ns = c.n_entries(s);
        uint64_t &i = cursor[s];
        while (i < ns && st[i].peer != (int32_t)c.rank) i++;
        if (i == ns) {
            rc = fail("host comm: rank %u sent rank %u fewer slices than it receives", s, c.rank);
        } else if (st[i].bytes != o.bytes) {
            rc = fail("host comm: slice of %llu bytes from rank %u, receive of %llu", (unsigned long long)st[i].bytes, s,
                      (unsigned long long)o.bytes);
        } else if (zkgpu_memcpy_h2d(o.buf, c.data(s) + st[i].off, o.bytes)) {
            rc = fail("host comm: outbox -> device copy failed: %s", zkgpu_last_error());
        }
        i++;
    }
    if (rc) err.store(1);
    if (c.wait()) return -1;
    if (err.load()) return rc ? rc : fail("host comm: another rank failed in this exchange");
    return 0;
}

}  // namespace zkgpu_host
