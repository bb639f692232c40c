// CPU multi-process check of the host-staged exchange (host/comm_host.hpp),
// the zkgpu_comm the row-sharded prover uses when ranks share a machine
// without RCCL peers.  W processes (fork) open one shared-memory
// communicator and run:
//   1. exchanges of the prover's patterns -- all-to-all with per-pair sizes,
//      ring shifts (halo refresh / spill), all-gather -- with every byte
//      checked, and
//   2. an error in exchange k + 1 raised by a fast rank while a slow rank is
//      still reading exchange k's flag (the hook below widens that window):
//      exchange k must succeed on every rank, k + 1 fail on every rank, and
//      no rank may hang;
//   3. a failed rank: the last rank aborts the communicator (zkgpu_comm.abort,
//      what the prover does when its proof fails) instead of exchanging --
//      every other rank's exchange fails at once; then, on a second
//      communicator, the last rank stops without exchanging -- every other
//      rank fails within the exchange deadline (ZKGPU_COMM_TIMEOUT_S = 2 s),
//      and every exchange after that fails at once.
// The device copies are host memcpy here (the harness defines the two
// libzkgpu calls the exchange makes), so the test needs no GPU.
// Build: g++ -O2 -std=c++17 -pthread -o comm_host_check tests/cpp/comm_host_check.cpp -lrt
// Run:   comm_host_check <world>   (exit 0 = pass)
#include <signal.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/wait.h>

#include <chrono>
#include <thread>
#include <vector>

#include "../../include/zkgpu.h"
#include "../../include/zkgpu_stark.h"

extern "C" int zkgpu_memcpy_d2h(void *dst, const void *src, uint64_t bytes)
{
    memcpy(dst, src, bytes);
    return 0;
}
extern "C" int zkgpu_memcpy_h2d(void *dst, const void *src, uint64_t bytes)
{
    memcpy(dst, src, bytes);
    return 0;
}
extern "C" const char *zkgpu_last_error(void) { return "(host memcpy)"; }

namespace zkgpu_host {
static char g_err[512];
static int fail(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return -1;
}
static int g_slow_rank = -1;  // this rank sleeps between barrier 2 and the flag read
}  // namespace zkgpu_host

#define ZKGPU_COMM_TEST_HOOK(c)                                                                                   \
    do {                                                                                                          \
        if ((int)(c).rank == zkgpu_host::g_slow_rank) std::this_thread::sleep_for(std::chrono::milliseconds(30)); \
    } while (0)
#include "../../zkevm-prover_amd/host/comm_host.hpp"

using namespace zkgpu_host;

static uint8_t pattern(uint32_t from, uint32_t to, uint32_t round, uint64_t i)
{
    return (uint8_t)(from * 131 + to * 17 + round * 7 + i * 29 + (i >> 8));
}

static int run_rank(const char *name, uint32_t W, uint32_t R)
{
    zkgpu_comm comm;
    if (host_comm_create(&comm, name, W, R, 1 << 20)) {
        fprintf(stderr, "rank %u: create: %s\n", R, g_err);
        return 2;
    }
    int bad = 0;
    // 1. the prover's exchange patterns, 60 rounds, bytes checked
    for (uint32_t round = 0; round < 60 && !bad; round++) {
        std::vector<zkgpu_comm_op> ops;
        std::vector<std::vector<uint8_t>> sbuf(W), rbuf(W);
        auto bytes = [&](uint32_t from, uint32_t to) -> uint64_t {
            switch (round % 3) {
            case 0: return 1 + (from * 7 + to * 3 + round) % 5000;  // all-to-all, ragged
            case 1: return to == (from + 1) % W ? 4096 + round : 0;  // ring shift (halo / spill)
            default: return 512;                                      // all-gather
            }
        };
        for (uint32_t d = 0; d < W; d++) {
            if (d == R || !bytes(R, d)) continue;
            sbuf[d].resize(bytes(R, d));
            for (uint64_t i = 0; i < sbuf[d].size(); i++) sbuf[d][i] = pattern(R, d, round, i);
            ops.push_back(zkgpu_comm_op{(int32_t)d, 1, sbuf[d].data(), sbuf[d].size()});
        }
        for (uint32_t s = 0; s < W; s++) {
            if (s == R || !bytes(s, R)) continue;
            rbuf[s].assign(bytes(s, R), 0);
            ops.push_back(zkgpu_comm_op{(int32_t)s, 0, rbuf[s].data(), rbuf[s].size()});
        }
        if (ops.size() > 2ULL * (W - 1)) bad = 1;  // the prover's bound holds for these patterns too
        if (!ops.empty() && host_exchange(comm.ctx, ops.data(), (uint32_t)ops.size())) {
            fprintf(stderr, "rank %u round %u: %s\n", R, round, g_err);
            bad = 1;
        }
        for (uint32_t s = 0; s < W && !bad; s++)
            for (uint64_t i = 0; i < rbuf[s].size(); i++)
                if (rbuf[s][i] != pattern(s, R, round, i)) {
                    fprintf(stderr, "rank %u round %u: byte %llu from %u wrong\n", R, round, (unsigned long long)i, s);
                    bad = 1;
                    break;
                }
    }
    // 2. exchange k succeeds everywhere although rank 0 fails in k + 1 while
    // the last rank still reads k's flag
    g_slow_rank = (int)W - 1;
    std::vector<uint8_t> a(64, (uint8_t)R), b(64 * W);
    auto ring = [&](bool poison) {
        std::vector<zkgpu_comm_op> ops;
        const uint32_t nx = (R + 1) % W, pv = (R + W - 1) % W;
        // a poisoned exchange: rank 0 names itself as a peer (refused in phase 1)
        ops.push_back(zkgpu_comm_op{(int32_t)(poison && R == 0 ? 0 : nx), 1, a.data(), 64});
        ops.push_back(zkgpu_comm_op{(int32_t)pv, 0, b.data(), 64});
        return host_exchange(comm.ctx, ops.data(), (uint32_t)ops.size());
    };
    for (int k = 0; k < 8 && !bad; k++) {
        if (ring(false)) {
            fprintf(stderr, "rank %u: clean exchange %d failed: %s\n", R, k, g_err);
            bad = 1;
        }
    }
    if (!bad && !ring(true)) {
        fprintf(stderr, "rank %u: the poisoned exchange succeeded\n", R);
        bad = 1;
    }
    g_slow_rank = -1;
    host_comm_destroy(&comm);
    // 3. a failed rank, then a stopped one
    using clk = std::chrono::steady_clock;
    auto secs = [](clk::time_point t) { return std::chrono::duration<double>(clk::now() - t).count(); };
    for (int variant = 0; variant < 2 && !bad; variant++) {
        char nm[80];
        snprintf(nm, sizeof nm, "%s_f%d", name, variant);
        zkgpu_comm c2;
        if (host_comm_create(&c2, nm, W, R, 1 << 16)) {
            fprintf(stderr, "rank %u: create %s: %s\n", R, nm, g_err);
            return 2;
        }
        std::vector<uint8_t> x(64, 1), y(64);
        const uint32_t nx = (R + 1) % W, pv = (R + W - 1) % W;
        zkgpu_comm_op ops[2] = {{(int32_t)nx, 1, x.data(), 64}, {(int32_t)pv, 0, y.data(), 64}};
        if (host_exchange(c2.ctx, ops, 2)) {  // a clean exchange first
            fprintf(stderr, "rank %u variant %d: clean exchange failed: %s\n", R, variant, g_err);
            bad = 1;
        }
        const auto t0 = clk::now();
        if (R == W - 1) {
            if (variant == 0) {
                c2.abort(c2.ctx);
            } else {
                std::this_thread::sleep_for(std::chrono::milliseconds(3500));  // stopped: never exchanges
            }
        } else {
            const int rc = host_exchange(c2.ctx, ops, 2);
            const double el = secs(t0);
            const double lim = variant == 0 ? 1.5 : 3.0;  // abort: at once; stopped: the 2 s deadline
            if (!rc || el > lim || (variant == 1 && el < 1.5)) {
                fprintf(stderr, "rank %u variant %d: exchange rc %d after %.2f s (%s)\n", R, variant, rc, el, g_err);
                bad = 1;
            }
            const auto t1 = clk::now();
            if (!host_exchange(c2.ctx, ops, 2) || secs(t1) > 0.5) {
                fprintf(stderr, "rank %u variant %d: the exchange after the failure did not fail at once\n", R, variant);
                bad = 1;
            }
        }
        host_comm_destroy(&c2);
    }
    return bad;
}

int main(int argc, char **argv)
{
    const uint32_t W = argc > 1 ? (uint32_t)atoi(argv[1]) : 2;
    char name[64];
    snprintf(name, sizeof name, "/zkgpu_cc_%d", (int)getpid());
    setenv("ZKGPU_RUN_ID", name, 1);
    setenv("ZKGPU_COMM_TIMEOUT_S", "2", 1);
    std::vector<pid_t> kids;
    for (uint32_t r = 0; r < W; r++) {
        const pid_t p = fork();
        if (p == 0) {
            alarm(60);  // a hang is a failure, not a stuck test
            _exit(run_rank(name, W, r));
        }
        kids.push_back(p);
    }
    int bad = 0;
    for (pid_t p : kids) {
        int st = 0;
        waitpid(p, &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st)) bad = 1;
    }
    shm_unlink(name);
    printf("%s: %u ranks\n", bad ? "FAIL" : "ok", W);
    return bad;
}
