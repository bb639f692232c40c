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
//
// No wait is unbounded: the barrier is a counter in the segment polled with a
// deadline (comm_wait, ZKGPU_COMM_TIMEOUT_S); a rank that gives up there, or
// aborts (zkgpu_comm.abort: its proof failed), marks the segment broken and
// every rank's next wait fails -- a failed or stopped rank cannot leave its
// peers waiting forever.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <string>
#include <thread>

namespace zkgpu_host {

// seconds a rank waits for its peers in one exchange (ZKGPU_COMM_TIMEOUT_S,
// default 120: the largest exchange, a fork-9 stage-1 commit at W = 8, moves
// ~16 GB per rank in ~0.1 s over xGMI; the rest is the ranks' skew)
static double comm_timeout_s()
{
    const char *e = getenv("ZKGPU_COMM_TIMEOUT_S");
    const double t = e ? atof(e) : 0.0;
    return t > 0 ? t : 120.0;
}

// Poll done() until it returns 1 (0: not yet, < 0: failed), with err()
// checked on the way; returns 0, -1 (failed) or -2 (deadline).  Short sleeps
// after the first polls keep a waiting rank off its CPU core.
template <class Done, class Err>
static int comm_wait(Done done, Err err, double timeout_s)
{
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (uint64_t spin = 0;; spin++) {
        const int d = done();
        if (d > 0) return 0;
        if (d < 0 || err()) return -1;
        if (std::chrono::duration<double>(clk::now() - t0).count() > timeout_s) return -2;
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(spin > 4096 ? 200 : 20));
    }
}

struct HostCommHeader {
    std::atomic<uint32_t> ready;    // 1: set up; 2: creation failed (a late rank fails too)
    std::atomic<uint32_t> arrived;  // ranks that have mapped the segment (creation)
    uint32_t world;
    uint64_t capacity;
    uint64_t run;                 // this run's tag (run_tag_hash): a stale segment never matches
    // error[k % 3]: a rank failed inside exchange k.  One slot per exchange
    // (cleared two exchanges ahead, see host_exchange): a rank still reading
    // exchange k's flag never sees a failure a faster rank raised in k + 1
    std::atomic<uint32_t> error[3];
    // the barrier: arrivals of the current generation, the generation
    std::atomic<uint32_t> bar_count, bar_gen;
    // a rank aborted or a barrier timed out: every later wait fails
    std::atomic<uint32_t> broken;
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
    // every rank of the world: the last arrival resets the count and
    // advances the generation the others poll (with the deadline)
    int wait() const
    {
        HostCommHeader *h = hdr();
        if (h->broken.load()) return fail("host comm: a rank aborted or timed out in an earlier exchange");
        const uint32_t g = h->bar_gen.load(std::memory_order_acquire);
        if (h->bar_count.fetch_add(1, std::memory_order_acq_rel) + 1 == world) {
            h->bar_count.store(0, std::memory_order_relaxed);
            h->bar_gen.fetch_add(1, std::memory_order_release);
            return 0;
        }
        const double limit = comm_timeout_s();
        const int w = comm_wait([&]() { return h->bar_gen.load(std::memory_order_acquire) != g ? 1 : 0; },
                                [&]() { return h->broken.load() != 0; }, limit);
        if (!w) return 0;
        h->broken.store(1);
        if (w == -2) return fail("host comm: not every rank reached the exchange within %.0f s (a peer failed or stopped)", limit);
        return fail("host comm: a rank aborted (its proof failed)");
    }
};

static int host_abort(void *vctx)
{
    ((HostCommCtx *)vctx)->hdr()->broken.store(1);
    return 0;
}

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
#ifdef ZKGPU_COMM_TEST_HOOK  // tests/cpp/comm_host_check.cpp: widen the window before the flag is read
    ZKGPU_COMM_TEST_HOOK(c);
#endif
    if (err.load()) return rc ? rc : fail("host comm: another rank failed in this exchange");
    return 0;
}

// zkgpu_comm_host_create (include/zkgpu_stark.h)
static int host_comm_create(zkgpu_comm *comm, const char *name, uint32_t world, uint32_t rank, uint64_t capacity)
{
    memset(comm, 0, sizeof *comm);
    if (!world || rank >= world || !name || name[0] != '/')
        return fail("zkgpu_comm_host_create: need rank < world and a name starting with '/'");
    auto *c = new HostCommCtx();
    c->rank = rank;
    c->world = world;
    c->capacity = capacity;
    c->size = HostCommCtx::header_bytes() + (uint64_t)world * c->box_bytes();
    const uint64_t run = run_tag_hash();
    void *m = MAP_FAILED;
    if (rank == 0) {
        shm_unlink(name);
        int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd >= 0 && ftruncate(fd, (off_t)c->size)) {
            close(fd);
            fd = -1;
        }
        if (fd >= 0) {
            m = mmap(nullptr, c->size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            close(fd);
        }
        if (m == MAP_FAILED) {
            delete c;
            return fail("zkgpu_comm_host_create: shared memory %s of %llu bytes not available", name,
                        (unsigned long long)c->size);
        }
        c->base = (uint8_t *)m;
        HostCommHeader *h = c->hdr();
        h->bar_count.store(0);
        h->bar_gen.store(0);
        h->broken.store(0);
        h->world = world;
        h->capacity = capacity;
        h->run = run;
        for (auto &e : h->error) e.store(0);
        h->arrived.store(0);
        h->ready.store(1, std::memory_order_release);
    } else {
        // wait (up to 60 s) for rank 0's segment of THIS run: a segment left
        // under the name by an earlier run (other tag, or not yet unlinked by
        // rank 0) is unmapped and looked up again
        for (int t = 0; t < 6000 && m == MAP_FAILED; t++) {
            const int fd = shm_open(name, O_RDWR, 0600);
            struct stat st;
            if (fd >= 0 && !fstat(fd, &st) && (uint64_t)st.st_size >= c->size)
                m = mmap(nullptr, c->size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            if (fd >= 0) close(fd);
            if (m != MAP_FAILED) {
                const HostCommHeader *h = (const HostCommHeader *)m;
                if (h->ready.load(std::memory_order_acquire) != 1 || h->run != run) {
                    munmap(m, c->size);
                    m = MAP_FAILED;
                } else if (h->world != world || h->capacity != capacity) {
                    munmap(m, c->size);
                    delete c;
                    return fail("zkgpu_comm_host_create: segment %s belongs to another world", name);
                }
            }
            if (m == MAP_FAILED) std::this_thread::sleep_for(std::chrono::milliseconds(10));
        }
        if (m == MAP_FAILED) {
            delete c;
            return fail("zkgpu_comm_host_create: shared memory %s of this run not available", name);
        }
        c->base = (uint8_t *)m;
    }
    // every rank has mapped the segment (counted, with a time limit: a rank
    // that never arrives fails the others here instead of leaving them in a
    // barrier), then its name is no longer needed
    {
        HostCommHeader *h = c->hdr();
        h->arrived.fetch_add(1);
        bool all = false;
        for (int t = 0; t < 12000 && h->ready.load() == 1 && !(all = h->arrived.load() >= world); t++)
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        // a rank that gave up marks the segment failed (ready = 2) before it
        // leaves: a late arrival then fails here too, instead of entering the
        // first exchange without the others
        if (!all || h->ready.load() != 1) {
            h->ready.store(2);
            const uint32_t n = h->arrived.load();
            if (rank == 0) shm_unlink(name);
            munmap(m, c->size);
            delete c;
            return fail("zkgpu_comm_host_create: %u of %u ranks arrived within 60 s", n, world);
        }
    }
    if (rank == 0) shm_unlink(name);
    comm->rank = rank;
    comm->world = world;
    comm->ctx = c;
    comm->exchange = host_exchange;
    comm->abort = host_abort;
    return 0;
}

static void host_comm_destroy(zkgpu_comm *comm)
{
    if (!comm || !comm->ctx) return;
    auto *c = (HostCommCtx *)comm->ctx;
    munmap(c->base, c->size);
    delete c;
    comm->ctx = nullptr;
    comm->exchange = nullptr;
    comm->abort = nullptr;
}

}  // namespace zkgpu_host
