// zkgpu_batch_prover -- the batch-proof STARK of Prover::genBatchProof
// (src/prover/prover.cpp:565-590) driven by the reference's own inputs:
//
//   config JSON (config.cpp:231-242 keys)
//     zkevmStarkInfo      <circuit>.starkinfo.json   (StarkInfo::load, stark_info.cpp:21-454)
//     zkevmConstPols      constant polynomials, N x nConstants u64 rows (starks.hpp:94-116)
//     zkevmConstantsTree  constant tree; its root must equal the tree built
//                         from zkevmConstPols (the prover's verkey)
//     zkevmCmPols         committed trace, N x nCm1 u64 rows (commit_pols.hpp)
//     zkevmVerkey         optional {"constRoot": [...]} checked like the tree
//     outputPath          directory for the outputs
//     zkgpuPublics        the public inputs as a JSON array (the publics.json
//                         the reference writes, prover.cpp:657); genBatchProof
//                         computes them from the executor's Main columns
//                         (prover.cpp:480-560), which this driver does not run
//
//   outputs (json2file layout, utils.cpp:212-222)
//     <outputPath>/batch_proof.proof.json   FRIProof::proofs.proof2json() + "publics"
//     <outputPath>/batch_proof.zkin.json    proof2zkinStark() + "publics"
//
// The expression code comes from the starkinfo's step code (step2prev ...
// step52ns), run as GPU programs (ProverInfo, host/stark_info.cpp); for the
// zkEVM's parser bytecode, StepsGPU (host/zkgpu_steps.hpp) is the binding.
//
// Usage: zkgpu_batch_prover [--shard RANK/WORLD --comm rccl:<id file>|host:</shm name> [--device D]] <config.json>
//        (--shard: one rank of ONE proof row-sharded over WORLD processes,
//        zkgpu_stark_create_sharded; every rank runs this command with the
//        same config, rank 0 writes the outputs.  rccl: rank 0 writes the
//        RCCL id to the file, the others wait for it; host: shared-memory
//        exchange for ranks sharing a GPU.  --device defaults to RANK for
//        rccl, 0 for host.)
//        zkgpu_batch_prover --info <starkinfo.json>                 (derived prover description; no GPU)
//        zkgpu_batch_prover --zkin <starkinfo.json> <flat proof> <publics.json> <outdir>
//                                                                   (proof JSON of a flat proof; no GPU)
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <memory>
#include <thread>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/zkgpu.h"
#include "../../include/zkgpu_stark.h"
#include "zkgpu_fri_proof.hpp"
#include "zkgpu_json.hpp"
#include "zkgpu_stark_info.hpp"

using zkgpu::json::Value;

static std::string read_text(const std::string &path)
{
    std::ifstream f(path, std::ios::binary);
    if (!f.good()) throw std::runtime_error("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

static std::vector<uint64_t> read_u64(const std::string &path, uint64_t expect)
{
    const std::string b = read_text(path);
    if (b.size() != expect * 8)
        throw std::runtime_error(path + ": " + std::to_string(b.size()) + " bytes, expected " + std::to_string(expect * 8));
    std::vector<uint64_t> v(expect);
    memcpy(v.data(), b.data(), b.size());
    return v;
}

static void write_json(const std::string &path, const Value &j)
{
    std::ofstream f(path, std::ios::binary);
    if (!f.good()) throw std::runtime_error("cannot create " + path);
    f << zkgpu::json::dump4(j) << "\n";
    if (!f.good()) throw std::runtime_error("write failed: " + path);
}

static std::vector<uint64_t> read_publics(const std::string &path, uint64_t n)
{
    const Value j = zkgpu::json::parse(read_text(path));
    if (j.size() != n) throw std::runtime_error(path + ": expected " + std::to_string(n) + " public inputs");
    std::vector<uint64_t> p(n);
    for (uint64_t i = 0; i < n; i++) p[i] = j[i].u64();
    return p;
}

static void write_outputs(const std::string &dir, const uint64_t *flat, uint64_t len, const zkgpu_stark_info &info,
                          const std::vector<uint64_t> &publics)
{
    mkdir(dir.c_str(), 0775);
    Value proof = zkgpu::proof2json(flat, len, info);
    Value zkin = zkgpu::proof2zkinStark(proof);
    Value pub = Value::array();
    for (uint64_t v : publics) pub.push(Value::str(std::to_string(v % 0xFFFFFFFF00000001ULL)));
    proof.set("publics", pub);  // prover.cpp:586-588
    zkin.set("publics", pub);
    write_json(dir + "/batch_proof.proof.json", proof);
    write_json(dir + "/batch_proof.zkin.json", zkin);
}

static uint64_t flat_len(const zkgpu_stark_info &in)
{
    // include/zkgpu_stark.h proof layout
    uint64_t L = 16 + 3ULL * in.n_ev;
    for (uint32_t si = 1; si < in.n_fri_steps; si++)
        L += 4 + (uint64_t)in.n_queries * (3ULL << (in.fri_steps[si - 1] - in.fri_steps[si])) +
             (uint64_t)in.n_queries * in.fri_steps[si] * 4;
    L += (uint64_t)in.n_queries * (in.n_cm1 + in.n_cm2 + in.n_cm3 + in.n_cm4 + in.n_const);
    L += 5ULL * in.n_queries * in.n_bits_ext * 4;
    L += 3ULL << in.fri_steps[in.n_fri_steps - 1];
    return L;
}

static void check_root(const char *what, const uint64_t got[4], const uint64_t want[4])
{
    for (int i = 0; i < 4; i++)
        if (got[i] != want[i])
            throw std::runtime_error(std::string(what) + ": constant root differs from the tree built from zkevmConstPols");
}

struct Shard {
    uint32_t rank = 0, world = 1;
    std::string comm;  // "" (single GPU), "rccl:<file>", "host:<name>"
    int device = -1;
};

// The RCCL id through a file: rank 0 writes it (atomic rename), the others
// poll.  Every file carries this run's tag -- ZKGPU_RUN_ID if set, else the
// launcher's pid (ranks started by one launcher share their parent) -- and a
// reader takes only a file with its own tag, so a file left by an earlier run
// at the same path is never mistaken for this run's id.  Rank 0 removes the
// file once the communicator exists (every rank has read it by then).
static std::string run_tag()
{
    const char *e = getenv("ZKGPU_RUN_ID");
    return e && *e ? std::string(e) : "ppid" + std::to_string((long)getppid());
}

static const char RCCL_ID_MAGIC[8] = {'Z', 'K', 'G', 'P', 'U', 'I', 'D', '1'};

static void rccl_id_file(const std::string &path, uint32_t rank, uint8_t id[128])
{
    const std::string tag = run_tag();
    if (rank == 0) {
        if (zkgpu_comm_rccl_unique_id(id)) throw std::runtime_error(std::string("rccl id: ") + zkgpu_stark_last_error());
        const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
        std::ofstream f(tmp, std::ios::binary);
        const uint32_t n = (uint32_t)tag.size();
        f.write(RCCL_ID_MAGIC, 8);
        f.write((const char *)&n, 4);
        f.write(tag.data(), n);
        f.write((const char *)id, 128);
        f.close();
        if (!f.good() || std::rename(tmp.c_str(), path.c_str())) throw std::runtime_error("cannot write " + path);
        return;
    }
    for (int t = 0; t < 6000; t++) {
        std::ifstream f(path, std::ios::binary);
        char magic[8];
        uint32_t n = 0;
        if (f.good() && f.read(magic, 8) && !memcmp(magic, RCCL_ID_MAGIC, 8) && f.read((char *)&n, 4) && n < 4096) {
            std::string got(n, '\0');
            if (f.read(&got[0], n) && got == tag && f.read((char *)id, 128) && f.gcount() == 128) return;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    throw std::runtime_error("no RCCL id for run " + tag + " in " + path + " after 60 s");
}

static int prove(const std::string &config_path, const Shard &sh)
{
    const Value cfg = zkgpu::json::parse(read_text(config_path));
    auto key = [&](const char *k) { return cfg[k].string(); };
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const zkgpu::StarkInfo si = zkgpu::StarkInfo::from_file(key("zkevmStarkInfo"));
    const zkgpu::ProverInfo pinfo(si);
    const zkgpu_stark_info &info = pinfo.info();
    const uint64_t N = 1ULL << info.n_bits;
    const std::vector<uint64_t> consts = read_u64(key("zkevmConstPols"), N * info.n_const);
    const std::vector<uint64_t> cm1 = read_u64(key("zkevmCmPols"), N * info.n_cm1);
    std::vector<uint64_t> publics(info.n_publics, 0);
    if (info.n_publics) publics = read_publics(key("zkgpuPublics"), info.n_publics);

    void *h = nullptr;
    zkgpu_comm comm{};
    struct CommGuard {
        zkgpu_comm *c;
        bool host;
        ~CommGuard()
        {
            if (host)
                zkgpu_comm_host_destroy(c);
            else
                zkgpu_comm_rccl_destroy(c);
        }
    };
    std::unique_ptr<CommGuard> comm_guard;
    if (sh.comm.empty()) {
        if (sh.device >= 0 && zkgpu_init(sh.device)) throw std::runtime_error(std::string("init: ") + zkgpu_last_error());
        if (zkgpu_stark_create(&h, &info)) throw std::runtime_error(std::string("create: ") + zkgpu_stark_last_error());
    } else {
        const bool host = sh.comm.rfind("host:", 0) == 0;
        const int dev = sh.device >= 0 ? sh.device : (host ? 0 : (int)sh.rank);
        if (zkgpu_init(dev)) throw std::runtime_error(std::string("init: ") + zkgpu_last_error());
        int rc;
        if (host) {
            rc = zkgpu_comm_host_create(&comm, sh.comm.c_str() + 5, sh.world, sh.rank, 1ULL << 30);
        } else if (sh.comm.rfind("rccl:", 0) == 0) {
            uint8_t id[128];
            rccl_id_file(sh.comm.substr(5), sh.rank, id);
            rc = zkgpu_comm_rccl_create(&comm, id, sh.world, sh.rank);
            if (!rc && sh.rank == 0) std::remove(sh.comm.substr(5).c_str());  // every rank has joined
        } else {
            throw std::runtime_error("--comm must be rccl:<file> or host:</name>");
        }
        if (rc) throw std::runtime_error(std::string("comm: ") + zkgpu_stark_last_error());
        comm_guard.reset(new CommGuard{&comm, host});
        if (zkgpu_stark_create_sharded(&h, &info, &comm))
            throw std::runtime_error(std::string("create: ") + zkgpu_stark_last_error());
    }
    struct Guard {
        void *h;
        ~Guard() { zkgpu_stark_destroy(h); }
    } guard{h};
    if (zkgpu_stark_set_const(h, consts.data()) || zkgpu_stark_set_cm1(h, cm1.data()) ||
        zkgpu_stark_set_publics(h, publics.data()))
        throw std::runtime_error(std::string("load: ") + zkgpu_stark_last_error());
    uint64_t verkey[4];
    zkgpu_stark_verkey(h, verkey);
    {
        // constant tree file: header, LDE, nodes; the root is its last 4 elements
        const std::string t = read_text(key("zkevmConstantsTree"));
        if (t.size() < 32 || t.size() % 8) throw std::runtime_error("zkevmConstantsTree: bad size");
        uint64_t root[4];
        memcpy(root, t.data() + t.size() - 32, 32);
        check_root("zkevmConstantsTree", root, verkey);
    }
    if (cfg.contains("zkevmVerkey")) {
        const Value vk = zkgpu::json::parse(read_text(key("zkevmVerkey")));
        uint64_t root[4];
        for (int i = 0; i < 4; i++) root[i] = vk["constRoot"][i].u64();
        check_root("zkevmVerkey", root, verkey);
    }
    const auto t1 = clk::now();
    const uint64_t len = zkgpu_stark_proof_len(h);
    if (len != flat_len(info)) throw std::runtime_error("proof length mismatch");
    std::vector<uint64_t> flat(len);
    if (zkgpu_stark_prove(h, flat.data())) throw std::runtime_error(std::string("prove: ") + zkgpu_stark_last_error());
    const auto t2 = clk::now();
    if (sh.rank == 0) write_outputs(key("outputPath"), flat.data(), len, info, publics);
    const auto t3 = clk::now();
    auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
    fprintf(stderr, "zkgpu_batch_prover[%u/%u]: load %.1f ms, STARK_PROOF_BATCH_PROOF %.1f ms, json %.1f ms\n", sh.rank,
            sh.world, ms(t1 - t0), ms(t2 - t1), ms(t3 - t2));
    return 0;
}

int main(int argc, char **argv)
{
    try {
        if (argc == 3 && !strcmp(argv[1], "--info")) {
            const zkgpu::StarkInfo si = zkgpu::StarkInfo::from_file(argv[2]);
            printf("%s\n", zkgpu::json::dump4(zkgpu::ProverInfo(si).to_json()).c_str());
            return 0;
        }
        if (argc == 6 && !strcmp(argv[1], "--zkin")) {
            const zkgpu::StarkInfo si = zkgpu::StarkInfo::from_file(argv[2]);
            const zkgpu::ProverInfo pinfo(si);
            const uint64_t len = flat_len(pinfo.info());
            const std::vector<uint64_t> flat = read_u64(argv[3], len);
            write_outputs(argv[5], flat.data(), len, pinfo.info(), read_publics(argv[4], si.nPublics));
            return 0;
        }
        Shard sh;
        int a = 1;
        while (a + 1 < argc && argv[a][0] == '-' && argv[a][1] == '-') {
            const std::string opt = argv[a];
            if (opt == "--shard") {
                unsigned r = 0, w = 0;
                if (sscanf(argv[a + 1], "%u/%u", &r, &w) != 2 || !w || r >= w)
                    throw std::runtime_error("--shard takes RANK/WORLD");
                sh.rank = r;
                sh.world = w;
            } else if (opt == "--comm") {
                sh.comm = argv[a + 1];
            } else if (opt == "--device") {
                sh.device = atoi(argv[a + 1]);
            } else {
                break;
            }
            a += 2;
        }
        if (sh.world > 1 && sh.comm.empty())
            throw std::runtime_error("--shard with WORLD > 1 needs --comm");
        if (argc == a + 1 && argv[a][0] != '-') return prove(argv[a], sh);
        fprintf(stderr,
                "usage: %s [--shard RANK/WORLD --comm rccl:<file>|host:</name> [--device D]] <config.json>\n"
                "       %s --info <starkinfo.json>\n"
                "       %s --zkin <starkinfo.json> <flat proof> <publics.json> <outdir>\n",
                argv[0], argv[0], argv[0]);
        return 2;
    } catch (const std::exception &e) {
        fprintf(stderr, "zkgpu_batch_prover: %s\n", e.what());
        return 1;
    }
}
