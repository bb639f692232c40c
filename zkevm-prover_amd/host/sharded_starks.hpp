// ShardedStarks: ONE proof of one trace over the GPUs of a node, one process
// per GPU (BASELINE configs[4]); included by starks.cpp.
//
// The reference proves on one host (Starks::genProof, starks.cpp:9-404).  Here
// the extended (2n) domain -- the bytes and the hashing -- is partitioned by
// ROWS over W ranks (B = 2n / W rows each), and every step that touches it
// works on the rank's rows:
//
//   commit (stages 1-3 and the constants, starks.cpp:53-57,134-138,215-219)
//       rank r extends its column share of the section (extendPol, no
//       communication), ONE exchange sends every other rank its row block of
//       those columns -- straight from the LDE output, each (column, rank)
//       slice is contiguous -- plus the 2^blowup halo rows after the block
//       (read by next-row constraints), received directly into the
//       halo-padded block (ld B + 2^blowup); each rank hashes its rows as an
//       exact subtree (merkleTreeGL.cpp:37-44 layout), the W sub-roots are
//       all-gathered and the top log2 W levels hashed on every rank.
//   stage 4  the quotient program on the rank's rows (x_i = 7 w^(rB+i),
//       halo rows, zkgpu_zxp_eval_block_dev); q (2n x 3) is gathered, the
//       INTT / split / NTT (starks.cpp:255-296) run on every rank, each
//       commits its rows of the pieces.
//   stage 5  evmap on the rank's n-domain rows, partial sums all-gathered and
//       added mod p; the FRI program on the rank's rows, f gathered.
//   FRI      folds on every rank (2n x 3 elements); a layer tree whose
//       groups split into W blocks is row-sharded like the commits (each
//       rank hashes its groups' subtree, sub-roots all-gathered, openings
//       served by the owning rank); smaller layers on every rank.
//   queries  each s0 opening by the rank owning its row (subtree siblings +
//       top levels), all-gathered.
// The n-domain sections are whole on every rank; calculateZ is row-sharded
// (each rank its N/W-row block, a scan of the W block totals, the blocks
// all-gathered); the other n-domain stage work (step2 / H1H2 / step3prev /
// step3, starks.cpp:67-211) runs on every rank.  The
// transcript runs on every rank on identical inputs; the proof is the
// single-GPU proof bit for bit.
//
// Every exchange is a zkgpu_comm call (RCCL over xGMI in production, see
// comm_rccl.hpp; the tests plug a host-staged one); a rank never sends to
// itself -- its own slices are device copies.

class ShardedStarks : public Starks
{
public:
    zkgpu_comm comm{};
    uint32_t W = 1, R = 0;
    uint64_t B = 0, H = 0, BH = 0;
    uint64_t *ext = nullptr;   // LDE of the rank's column share (max share x NE)
    uint64_t *gath = nullptr;  // q / f gathered (3 x NE)
    uint64_t *cm4 = nullptr;   // quotient pieces, whole extended domain (n_cm4 x NE)
    uint64_t *xchg = nullptr;  // all-gather staging, W slots
    uint64_t slot = 0;
    struct Tree {
        uint64_t *nodes = nullptr;
        const uint64_t *block = nullptr;
        uint64_t ld = 0;
        uint32_t ncols = 0;
        std::vector<std::vector<uint64_t>> top;  // [0]: W sub-roots ... [last]: root
    };
    Tree trees[5];  // cm1, cm2, cm3, cm4, constants
    std::vector<Tree> ftrees;  // FRI layers (row-sharded where the groups split)
    std::vector<zkgpu_comm_op> ops;

    int create_sharded(const zkgpu_stark_info *in, const zkgpu_comm *c)
    {
        comm = *c;
        W = c->world;
        R = c->rank;
        if (!W || (W & (W - 1)) || R >= W || (W > 1 && !c->exchange))
            return fail("stark_create_sharded: world %u must be a power of two, rank %u < world, exchange set", W, R);
        if (load(in)) return -1;
        H = 1ULL << eb;
        if (NE % W || N % W || NE / W < 2 * H)
            return fail("stark_create_sharded: 2^%u rows do not split into %u blocks of >= %llu rows", info.n_bits_ext,
                        W, (unsigned long long)(2 * H));
        B = NE / W;
        BH = B + H;
        if (alloc()) return -1;
        return build_const();
    }

    static uint32_t ceil_div(uint32_t a, uint32_t b) { return (a + b - 1) / b; }
    void share(uint32_t ncols, uint32_t r, uint32_t &lo, uint32_t &hi) const  // balanced contiguous column split
    {
        const uint32_t base = ncols / W, extra = ncols % W;
        lo = r * base + (r < extra ? r : extra);
        hi = lo + base + (r < extra ? 1 : 0);
    }

    int alloc() override
    {
        if (alloc_n() || alloc_fri()) return -1;
        const uint32_t blk_secs[4] = {SEC_CM1_2NS, SEC_CM2_2NS, SEC_CM3_2NS, SEC_CONST_2NS};
        const uint32_t blk_w[4] = {info.n_cm1, info.n_cm2, info.n_cm3, info.n_const};
        uint32_t max_share = 1;
        for (int k = 0; k < 4; k++) {
            if (dalloc(&S.sec[blk_secs[k]], (uint64_t)(blk_w[k] ? blk_w[k] : 1) * BH)) return -1;
            S.ld[blk_secs[k]] = BH;
            S.ncols[blk_secs[k]] = blk_w[k];
            max_share = std::max(max_share, ceil_div(blk_w[k], W));
        }
        if (dalloc(&cm4, (uint64_t)(info.n_cm4 ? info.n_cm4 : 1) * NE)) return -1;
        S.sec[SEC_CM4_2NS] = cm4 + (uint64_t)R * B;
        S.ld[SEC_CM4_2NS] = NE;
        S.ncols[SEC_CM4_2NS] = info.n_cm4;
        for (uint32_t s : {(uint32_t)SEC_Q_2NS, (uint32_t)SEC_F_2NS}) {
            if (dalloc(&S.sec[s], 3 * B)) return -1;
            S.ld[s] = B;
            S.ncols[s] = 3;
        }
        if (dalloc(&gath, 3 * NE) || dalloc(&ext, (uint64_t)max_share * NE)) return -1;
        for (auto &t : trees)
            if (dalloc(&t.nodes, zkgpu_gl_merkle_num_elements(B))) return -1;
        slot = std::max<uint64_t>(4, std::max<uint64_t>(3ULL * info.n_ev, (uint64_t)q() * s0_record()));
        ftrees.assign(fri_steps.size(), Tree{});
        for (size_t si = 1; si < fri_steps.size(); si++) {
            const uint64_t ngroups = 1ULL << fri_steps[si], width = (3ULL << fri_steps[si - 1]) / ngroups;
            if (!fri_sharded(ngroups)) continue;
            if (dalloc(&ftrees[si].nodes, zkgpu_gl_merkle_num_elements(ngroups / W))) return -1;
            slot = std::max<uint64_t>(slot, (uint64_t)q() * (width + 4ULL * fri_steps[si]));
        }
        return dalloc(&xchg, slot * W);
    }

    uint64_t s0_record() const
    {
        return (uint64_t)info.n_cm1 + info.n_cm2 + info.n_cm3 + info.n_cm4 + info.n_const + 20ULL * info.n_bits_ext;
    }

    int exchange()
    {
        if (ops.empty()) return 0;
        if (comm.exchange(comm.ctx, ops.data(), (uint32_t)ops.size()))
            return fail("zkgpu_comm exchange of %zu operations failed (rank %u of %u)", ops.size(), R, W);
        ops.clear();
        return 0;
    }
    void op(uint32_t peer, int send, const void *buf, uint64_t bytes)
    {
        ops.push_back(zkgpu_comm_op{(int32_t)peer, send, const_cast<void *>(buf), bytes});
    }

    // every rank's n words (host) -> out[W x n] in rank order
    int allgather(const uint64_t *mine, uint64_t n, std::vector<uint64_t> &out)
    {
        if (n > slot) return fail("allgather: %llu words exceed the staging slot", (unsigned long long)n);
        out.assign(W * n, 0);
        if (W == 1) {
            memcpy(out.data(), mine, n * 8);
            return 0;
        }
        CK(zkgpu_memcpy_h2d(xchg + R * slot, mine, n * 8));
        for (uint32_t d = 0; d < W; d++)
            if (d != R) op(d, 1, xchg + R * slot, n * 8);
        for (uint32_t s = 0; s < W; s++)
            if (s != R) op(s, 0, xchg + s * slot, n * 8);
        if (exchange()) return -1;
        for (uint32_t s = 0; s < W; s++) CK(zkgpu_memcpy_d2h(out.data() + s * n, xchg + s * slot, n * 8));
        return 0;
    }

    // the rank's 3 x B block (ld B) of q or f -> full (3 x NE, ld NE) on every rank
    int gather_rows(const uint64_t *blk, uint64_t *full)
    {
        for (uint32_t d = 0; d < W; d++)
            if (d != R)
                for (int c = 0; c < 3; c++) op(d, 1, blk + c * B, B * 8);
        for (uint32_t s = 0; s < W; s++)
            if (s != R)
                for (int c = 0; c < 3; c++) op(s, 0, full + c * NE + s * B, B * 8);
        for (int c = 0; c < 3; c++) CK(zkgpu_memcpy_d2d(full + c * NE + R * B, blk + c * B, B * 8));
        return exchange();
    }

    static void hash_node(uint64_t out[4], const uint64_t *l, const uint64_t *r)
    {
        uint64_t in[12] = {0}, o[12];
        memcpy(in, l, 32);
        memcpy(in + 4, r, 32);
        zkgpu_gl_poseidon_full_host(o, in);
        memcpy(out, o, 32);
    }

    // subtree of the rank's rows + the top levels over the gathered sub-roots
    int merkelize(Tree &t, const uint64_t *blk, uint64_t ld, uint32_t ncols, uint64_t root[4])
    {
        CK(zkgpu_gl_merkletree_dev(t.nodes, blk, ld, ncols, B));
        t.block = blk;
        t.ld = ld;
        t.ncols = ncols;
        return top_levels(t, B, root);
    }

    // the W sub-roots all-gathered, the top log2 W levels hashed on the host
    int top_levels(Tree &t, uint64_t rows, uint64_t root[4])
    {
        uint64_t sub[4];
        CK(zkgpu_memcpy_d2h(sub, t.nodes + zkgpu_gl_merkle_num_elements(rows) - 4, 32));
        t.top.assign(1, {});
        if (allgather(sub, 4, t.top[0])) return -1;
        while (t.top.back().size() > 4) {
            const std::vector<uint64_t> &lv = t.top.back();
            std::vector<uint64_t> nx(lv.size() / 2);
            for (size_t i = 0; i < nx.size() / 4; i++) hash_node(&nx[4 * i], &lv[8 * i], &lv[8 * i + 4]);
            t.top.push_back(std::move(nx));
        }
        memcpy(root, t.top.back().data(), 32);
        return 0;
    }

    // LDE of the rank's column share, column -> row exchange (with halo), subtree
    int commit_cols(Tree &t, uint32_t sec_e, const uint64_t *src_n, uint32_t ncols, uint64_t root[4],
                    const char *lde_name, const char *xchg_name, const char *tree_name)
    {
        uint32_t lo, hi;
        share(ncols, R, lo, hi);
        uint64_t *blk = S.sec[sec_e];
        tstart();
        if (hi > lo) CK(zkgpu_gl_extend_pol_dev(ext, NE, src_n + (uint64_t)lo * N, N, NE, N, hi - lo));
        if (lde_name && tstop(lde_name)) return -1;
        tstart();
        for (uint32_t d = 0; d < W; d++) {
            if (d == R) continue;
            const uint64_t hb = (uint64_t)((d + 1) % W) * B;  // the halo: the next block's first rows
            for (uint32_t c = 0; c < hi - lo; c++) {
                op(d, 1, ext + c * NE + (uint64_t)d * B, B * 8);
                op(d, 1, ext + c * NE + hb, H * 8);
            }
        }
        for (uint32_t s = 0; s < W; s++) {
            if (s == R) continue;
            uint32_t slo, shi;
            share(ncols, s, slo, shi);
            for (uint32_t c = slo; c < shi; c++) {
                op(s, 0, blk + (uint64_t)c * BH, B * 8);
                op(s, 0, blk + (uint64_t)c * BH + B, H * 8);
            }
        }
        const uint64_t hb = (uint64_t)((R + 1) % W) * B;
        for (uint32_t c = lo; c < hi; c++) {
            CK(zkgpu_memcpy_d2d(blk + (uint64_t)c * BH, ext + (c - lo) * NE + (uint64_t)R * B, B * 8));
            CK(zkgpu_memcpy_d2d(blk + (uint64_t)c * BH + B, ext + (c - lo) * NE + hb, H * 8));
        }
        if (exchange()) return -1;
        if (xchg_name && tstop(xchg_name)) return -1;
        tstart();
        if (merkelize(t, blk, BH, ncols, root)) return -1;
        if (tree_name && tstop(tree_name)) return -1;
        return 0;
    }

    bool fri_sharded(uint64_t ngroups) const { return W > 1 && ngroups % W == 0 && ngroups / W >= 2; }

    // FRI layer tree: each rank hashes its block of groups (friProve.cpp:125-133)
    int fri_commit(size_t si, uint64_t ngroups, uint64_t width, uint64_t root[4]) override
    {
        if (!fri_sharded(ngroups)) return Starks::fri_commit(si, ngroups, width, root);
        const uint64_t bl = ngroups / W;
        Tree &t = ftrees[si];
        t.block = fri_aux[si] + (uint64_t)R * bl * width;
        t.ld = width;
        CK(zkgpu_gl_merkletree_rows_dev(t.nodes, t.block, width, bl));
        return top_levels(t, bl, root);
    }

    // openings served by the rank owning the group, the records all-gathered
    int fri_open(size_t si, uint64_t ngroups, uint64_t width, const std::vector<uint64_t> &yq, uint64_t *vals,
                 uint64_t *sibs) override
    {
        if (!fri_sharded(ngroups)) return Starks::fri_open(si, ngroups, width, yq, vals, sibs);
        const uint64_t bl = ngroups / W, levels = fri_steps[si];
        uint32_t log_b = 0;
        while ((1ULL << log_b) < bl) log_b++;
        const uint64_t rec = width + 4 * levels;
        const Tree &t = ftrees[si];
        std::vector<uint64_t> mine((uint64_t)q() * rec, 0), own, local;
        for (uint32_t qi = 0; qi < q(); qi++)
            if (yq[qi] / bl == R) {
                own.push_back(qi);
                local.push_back(yq[qi] % bl);
            }
        if (!own.empty()) {
            std::vector<uint64_t> v(own.size() * width + 1), sb(own.size() * log_b * 4 + 1);
            CK(zkgpu_gl_merkle_open_rows_dev(v.data(), sb.data(), t.nodes, t.block, width, bl, local.data(),
                                             own.size()));
            for (size_t k = 0; k < own.size(); k++) {
                uint64_t *r = &mine[own[k] * rec];
                memcpy(r, &v[k * width], width * 8);
                memcpy(r + width, &sb[k * log_b * 4], log_b * 32ULL);
                uint64_t *top = r + width + log_b * 4;
                uint32_t j = R;
                for (size_t lv = 0; lv + 1 < t.top.size(); lv++, j >>= 1, top += 4)
                    memcpy(top, &t.top[lv][4 * (j ^ 1)], 32);
            }
        }
        std::vector<uint64_t> all;
        if (allgather(mine.data(), mine.size(), all)) return -1;
        for (uint32_t qi = 0; qi < q(); qi++) {
            const uint64_t *r = &all[(yq[qi] / bl) * mine.size() + qi * rec];
            memcpy(vals + (uint64_t)qi * width, r, width * 8);
            memcpy(sibs + (uint64_t)qi * levels * 4, r + width, levels * 32);
        }
        return 0;
    }

    int commit_const() override
    {
        return commit_cols(trees[4], SEC_CONST_2NS, S.sec[SEC_CONST_N], info.n_const, verkey, nullptr, nullptr,
                           nullptr);
    }

    // F_p^3 product on the host (x^3 = x + 1)
    static void mul3(uint64_t r[3], const uint64_t a[3], const uint64_t b[3])
    {
        const uint64_t c0 = mul(a[0], b[0]), c1 = (uint64_t)(((unsigned __int128)mul(a[0], b[1]) + mul(a[1], b[0])) % P);
        const uint64_t c2 = (uint64_t)(((unsigned __int128)mul(a[0], b[2]) + mul(a[1], b[1]) + mul(a[2], b[0])) % P);
        const uint64_t c3 = (uint64_t)(((unsigned __int128)mul(a[1], b[2]) + mul(a[2], b[1])) % P);
        const uint64_t c4 = mul(a[2], b[2]);
        // x^3 = x + 1, x^4 = x^2 + x
        r[0] = (uint64_t)(((unsigned __int128)c0 + c3) % P);
        r[1] = (uint64_t)(((unsigned __int128)c1 + c3 + c4) % P);
        r[2] = (uint64_t)(((unsigned __int128)c2 + c4) % P);
    }

    // calculateZ (starks.cpp:146-224, polinomial.hpp:586-607) over the rank's
    // N/W-row block: z = prod of the ratios before each row, the block total
    // all-gathered, the block redone with z0 = the product of the earlier
    // ranks' totals (rank 0's is already final), then the blocks all-gathered
    // so every rank holds the whole column (the n-domain sections are whole)
    int z_all() override
    {
        const uint64_t nb = N / W, r0 = (uint64_t)R * nb;
        for (uint32_t zi = 0; zi < info.n_zctx; zi++) {
            uint64_t *z = S.sec[SEC_CM3_N] + (uint64_t)zctx[3 * zi + 2] * N;
            const uint64_t *num = S.sec[SEC_TMP_N] + (uint64_t)zctx[3 * zi] * N;
            const uint64_t *den = S.sec[SEC_TMP_N] + (uint64_t)zctx[3 * zi + 1] * N;
            const uint64_t one[3] = {1, 0, 0};
            uint64_t tot[3];
            CK(zkgpu_calculate_z_block_dev(z + r0, N, num + r0, N, den + r0, N, nb, one, tot));
            std::vector<uint64_t> all;
            if (allgather(tot, 3, all)) return -1;
            uint64_t pre[3] = {1, 0, 0}, acc[3] = {1, 0, 0};
            for (uint32_t s = 0; s < W; s++) {
                if (s == R) memcpy(pre, acc, 24);
                mul3(acc, acc, &all[3 * s]);
            }
            if (acc[0] != 1 || acc[1] || acc[2]) return fail("calculateZ: grand product %u does not close", zi);
            if (pre[0] != 1 || pre[1] || pre[2])
                CK(zkgpu_calculate_z_block_dev(z + r0, N, num + r0, N, den + r0, N, nb, pre, tot));
            for (uint32_t d = 0; d < W; d++)
                if (d != R)
                    for (int c = 0; c < 3; c++) op(d, 1, z + (uint64_t)c * N + r0, nb * 8);
            for (uint32_t s = 0; s < W; s++)
                if (s != R)
                    for (int c = 0; c < 3; c++) op(s, 0, z + (uint64_t)c * N + (uint64_t)s * nb, nb * 8);
            if (exchange()) return -1;
        }
        return 0;
    }

    // an extended-domain program over the rank's rows
    int run_block(const Prog &p, const uint64_t ch[24], const uint64_t *evals, uint32_t n_ev, const uint64_t *xd,
                  const uint64_t *xdw)
    {
        uint32_t log_b = 0;
        while ((1ULL << log_b) < B) log_b++;
        const uint64_t x0 = mul(7, pw(w_of(info.n_bits_ext), (uint64_t)R * B));
        CK(zkgpu_zxp_eval_block_dev(p.instr.data(), (uint32_t)p.instr.size(), p.opnd.data(), (uint32_t)p.opnd.size(),
                                    p.n_tmp1 ? p.n_tmp1 : 1, p.n_tmp3 ? p.n_tmp3 : 1, &S, log_b, info.n_bits_ext, ch,
                                    publics.data(), (uint32_t)publics.size(), evals, n_ev, xd, xdw, eb, x0));
        return 0;
    }

    int prove(uint64_t *out) override
    {
        timers.clear();
        auto tall = clk::now();
        Transcript tr;
        tr.put(verkey, 4);
        tr.put(publics.data(), publics.size());
        uint64_t ch[24] = {0};
        uint64_t roots[4][4];
        std::vector<uint64_t> evals(3 * info.n_ev);
        // STAGE 1 (starks.cpp:49-63)
        if (commit_cols(trees[0], SEC_CM1_2NS, S.sec[SEC_CM1_N], info.n_cm1, roots[0], "STARK_STEP_1_LDE",
                        "STARK_STEP_1_EXCHANGE", "STARK_STEP_1_MERKLETREE"))
            return -1;
        tr.put(roots[0], 4);
        // STAGE 2 (:65-144), n domain on every rank
        tr.get_field(ch + 0);
        tr.get_field(ch + 3);
        tstart();
        if (run(step2, false, ch, evals.data(), 0)) return -1;
        if (tstop("STARK_STEP_2_CALCULATE_EXPS")) return -1;
        if (info.n_pu) {
            tstart();
            if (h1h2_all()) return -1;
            if (tstop("STARK_STEP_2_CALCULATEH1H2")) return -1;
        }
        if (commit_cols(trees[1], SEC_CM2_2NS, S.sec[SEC_CM2_N], info.n_cm2, roots[1], "STARK_STEP_2_LDE",
                        "STARK_STEP_2_EXCHANGE", "STARK_STEP_2_MERKLETREE"))
            return -1;
        tr.put(roots[1], 4);
        // STAGE 3 (:146-224)
        tr.get_field(ch + 6);
        tr.get_field(ch + 9);
        tstart();
        if (run(step3prev, false, ch, evals.data(), 0)) return -1;
        if (tstop("STARK_STEP_3_CALCULATE_EXPS")) return -1;
        tstart();
        if (z_all()) return -1;
        if (tstop("STARK_STEP_3_CALCULATE_Z")) return -1;
        if (!step3.instr.empty()) {
            tstart();
            if (run(step3, false, ch, evals.data(), 0)) return -1;
            if (tstop("STARK_STEP_3_CALCULATE_EXPS_2")) return -1;
        }
        if (commit_cols(trees[2], SEC_CM3_2NS, S.sec[SEC_CM3_N], info.n_cm3, roots[2], "STARK_STEP_3_LDE",
                        "STARK_STEP_3_EXCHANGE", "STARK_STEP_3_MERKLETREE"))
            return -1;
        tr.put(roots[2], 4);
        // STAGE 4 (:226-296): the quotient on the rank's rows
        tr.get_field(ch + 12);
        tstart();
        if (run_block(step42ns, ch, evals.data(), 0, nullptr, nullptr)) return -1;
        if (tstop("STARK_STEP_4_CALCULATE_EXPS_2NS")) return -1;
        tstart();
        if (gather_rows(S.sec[SEC_Q_2NS], gath) || quotient_pieces(gath, cm4)) return -1;
        if (tstop("STARK_STEP_4_CALCULATE_EXPS_2NS_INTT_NTT")) return -1;
        tstart();
        if (merkelize(trees[3], cm4 + (uint64_t)R * B, NE, info.n_cm4, roots[3])) return -1;
        if (tstop("STARK_STEP_4_MERKLETREE")) return -1;
        tr.put(roots[3], 4);
        // STAGE 5 (:298-392)
        tstart();
        uint64_t *xi = ch + 21;
        tr.get_field(xi);
        if (lagrange_xi(xi)) return -1;
        if (tstop("STARK_STEP_5_LEv_LpEv")) return -1;
        tstart();
        {
            const uint64_t nloc = N / W;
            std::vector<uint64_t> part(3 * info.n_ev), all;
            if (evmap_rows((uint64_t)R * nloc, nloc, part.data()) || allgather(part.data(), part.size(), all))
                return -1;
            for (size_t i = 0; i < evals.size(); i++) {
                unsigned __int128 acc = 0;
                for (uint32_t s = 0; s < W; s++) acc += all[s * evals.size() + i];
                evals[i] = (uint64_t)(acc % P);
            }
        }
        if (tstop("STARK_STEP_5_EVMAP")) return -1;
        tr.put(evals.data(), evals.size());
        tr.get_field(ch + 15);
        tr.get_field(ch + 18);
        tstart();
        CK(zkgpu_xdivxsub_dev(xdiv, xdivw, xi, info.n_bits, info.n_bits_ext));
        if (tstop("STARK_STEP_5_XDIVXSUB")) return -1;
        tstart();
        const uint64_t xo = 3ULL * R * B;  // xdiv rows are interleaved F_p^3
        if (run_block(step52ns, ch, evals.data(), info.n_ev, xdiv + xo, xdivw + xo)) return -1;
        if (gather_rows(S.sec[SEC_F_2NS], gath)) return -1;
        CK(zkgpu_cols3_to_interleaved_dev(fri_pol[0], gath, NE, NE));
        if (tstop("STARK_STEP_5_CALCULATE_EXPS")) return -1;
        return fri_and_queries(tr, &roots[0][0], evals, out, tall);
    }

    // each query row is opened by the rank owning it, the records all-gathered
    int open_s0(const std::vector<uint64_t> &ys, uint64_t *&w) override
    {
        const uint32_t widths[5] = {info.n_cm1, info.n_cm2, info.n_cm3, info.n_cm4, info.n_const};
        const uint64_t rec = s0_record();
        uint32_t log_b = 0;
        while ((1ULL << log_b) < B) log_b++;
        std::vector<uint64_t> mine((uint64_t)q() * rec, 0), own, local;
        for (uint32_t qi = 0; qi < q(); qi++)
            if (ys[qi] / B == R) {
                own.push_back(qi);
                local.push_back(ys[qi] % B);
            }
        uint64_t voff = 0;
        for (int t = 0; t < 5; t++) {
            const uint64_t soff = (uint64_t)info.n_cm1 + info.n_cm2 + info.n_cm3 + info.n_cm4 + info.n_const +
                                  (uint64_t)t * info.n_bits_ext * 4;
            if (!own.empty()) {
                std::vector<uint64_t> vals(own.size() * widths[t] + 1), sibs(own.size() * log_b * 4 + 1);
                CK(zkgpu_gl_merkle_open_dev(vals.data(), sibs.data(), trees[t].nodes, trees[t].block, trees[t].ld,
                                            widths[t], B, local.data(), own.size()));
                for (size_t k = 0; k < own.size(); k++) {
                    uint64_t *r = &mine[own[k] * rec];
                    memcpy(r + voff, &vals[k * widths[t]], widths[t] * 8ULL);
                    memcpy(r + soff, &sibs[k * log_b * 4], log_b * 32ULL);
                    uint64_t *top = r + soff + log_b * 4;
                    uint32_t j = R;
                    for (size_t lv = 0; lv + 1 < trees[t].top.size(); lv++, j >>= 1, top += 4)
                        memcpy(top, &trees[t].top[lv][4 * (j ^ 1)], 32);
                }
            }
            voff += widths[t];
        }
        std::vector<uint64_t> all;
        if (allgather(mine.data(), mine.size(), all)) return -1;
        auto record = [&](uint32_t qi) { return &all[(ys[qi] / B) * mine.size() + qi * rec]; };
        voff = 0;
        for (int t = 0; t < 5; t++) {
            for (uint32_t qi = 0; qi < q(); qi++, w += widths[t]) memcpy(w, record(qi) + voff, widths[t] * 8ULL);
            voff += widths[t];
        }
        for (int t = 0; t < 5; t++)
            for (uint32_t qi = 0; qi < q(); qi++, w += 4ULL * info.n_bits_ext)
                memcpy(w, record(qi) + voff + (uint64_t)t * info.n_bits_ext * 4, 32ULL * info.n_bits_ext);
        return 0;
    }
};
