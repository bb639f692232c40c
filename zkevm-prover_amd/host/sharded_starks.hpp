// ShardedStarks: ONE proof of one trace over the GPUs of a node, one process
// per GPU (BASELINE configs[4]); included by starks.cpp.
//
// The reference proves on one host (Starks::genProof, starks.cpp:9-404).  Here
// BOTH domains are partitioned by ROWS over W ranks, so no rank holds a whole
// section of the trace:
//
//   n domain   rank r holds rows [r nb, (r+1) nb) of cm1_n / cm2_n / cm3_n /
//       tmpExp_n / const_n (nb = N / W) plus the next block's first hn rows
//       (hn = the largest row shift the stage programs use: next-row reads,
//       shifted stores), ld = nb + hn.  The stage programs (step2prev /
//       step3prev / step3, starks.cpp:73,155,193) run on the rank's rows
//       (zkgpu_zxp_eval_block_dev, x_i = w^(r nb + i)); afterwards the rows
//       a shifted store wrote past the block go to the next rank (the
//       single-GPU store writes (i + s) mod N) and every written column's halo
//       is refreshed from the next rank, cyclically (the last rank's halo is
//       row 0: the wrap-around of the reference's (i + 1) % N).  calculateZ:
//       each rank its block, a scan of the W block totals, the block redone
//       with the product of the earlier ranks' totals (polinomial.hpp:586-607).
//       calculateH1H2 (starks.cpp:104-127), a global multiset sort: distinct
//       keys routed to their owner ranks, counts back to the table rows'
//       ranks, each rank deals its table rows' copies and sends every piece
//       of the multiset to the rank holding those h1/h2 rows (h1h2_sharded).
//   commit (stages 1-3 and the constants, starks.cpp:53-57,134-138,215-219)
//       the NTT transpose: the rank's rows of every column go to the rank
//       owning the column (all-to-all; each (column, rank) slice is contiguous
//       on both sides, received straight into the LDE input), the rank extends
//       its column share (extendPol, no communication), and a second all-to-all
//       sends every other rank its 2n-domain row block of those columns plus
//       the 2^blowup halo rows after it (halos packed, one message per peer).
//       Each rank hashes its rows as an exact subtree (merkleTreeGL.cpp:37-44
//       layout), the W sub-roots are all-gathered, the top log2 W levels
//       hashed on every rank.
//   stage 4  the quotient program on the rank's 2n rows (x_i = 7 w^(rB+i),
//       halo rows); the split (starks.cpp:255-296) by column owners: q column
//       j goes to rank j mod W, which interpolates it over the whole domain,
//       splits it into the q_deg pieces and evaluates them; every rank gets
//       its row blocks of all pieces back and commits its rows.
//   stage 5  LEv / LpEv (closed form) and evmap on the rank's n-domain rows,
//       partial sums all-gathered and added mod p; xDivXSub and the FRI
//       program on the rank's 2n rows.
//   FRI      layer 1 and the first fold over the ranks: one all-to-all
//       gives each rank all elements of its block of layer-1 groups (tree rows
//       and fold input, fri_transpose_layer), the folded 2^steps[1] elements
//       are all-gathered; the later folds (<= 1/16 of f) on every rank; a
//       layer tree whose groups split into W blocks is row-sharded like the
//       commits.
//   queries  each s0 opening by the rank owning its row (subtree siblings +
//       top levels), all-gathered.
// The constants are set up once (build / load, untimed) on a transient whole
// copy, committed, and cut to the rank's rows.  The transcript runs on every
// rank on identical inputs; the proof is the single-GPU proof bit for bit.
//
// Every exchange is a zkgpu_comm call (RCCL over xGMI in production, see
// comm_rccl.hpp; the tests plug a host-staged one); a rank never sends to
// itself -- its own slices are device copies.

class ShardedStarks : public Starks
{
public:
    zkgpu_comm comm{};
    uint32_t W = 1, R = 0;
    uint64_t B = 0, H = 0, BH = 0;     // 2n domain: block rows, halo rows (2^blowup), ld (>= B + H)
    uint64_t nb = 0, hn = 0, ldn = 0;  // n domain: block rows, halo rows, ld (>= nb + hn)
    uint64_t *ext = nullptr;    // LDE of the rank's column share (max share x NE)
    uint64_t *coln = nullptr;   // the rank's column share over all N rows (max share x N): the LDE input
    uint64_t *gath = nullptr;   // q / f gathered (3 x NE)
    uint64_t *cm4 = nullptr;    // quotient pieces, whole extended domain (n_cm4 x NE)
    uint64_t *xchg = nullptr;   // all-gather staging, W slots
    uint64_t *hsend = nullptr, *hrecv = nullptr;  // halo / spill / 2n-halo staging (hcap words each)
    // per-peer packing: every exchange posts at most one send and one receive
    // per peer (2 (W - 1) operations), whatever the column count -- a rank's
    // slices for a peer are gathered into its region of pack_s (stride_s
    // words per peer), a peer's message lands in its region of pack_r
    uint64_t *pack_s = nullptr, *pack_r = nullptr;
    // peer d's send region (the rank's own never is one: W - 1 regions)
    uint64_t *psend(uint32_t d) const { return pack_s + (uint64_t)(d < R ? d : d - 1) * stride_s; }
    uint64_t stride_s = 0, stride_r = 0;
    uint32_t max_ops = 0;  // largest exchange so far (operations posted by this rank)
    // this proof's exchanges: count, bytes this rank sent, the largest one's
    // sent bytes (reported as COUNT_COMM_* beside the stage timers)
    uint64_t n_exch = 0, sent_bytes = 0, max_sent = 0;
    uint64_t *puw = nullptr;    // W = 1: one plookup's f, t, h1, h2 over the whole n domain (12 x N)
    // W > 1, calculateH1H2 over the ranks (h1h2_sharded): route records out /
    // in (5 words each), the owner's returns out / in, the multiset segment
    // (3 x (nb + N): the rank's table rows can hold up to nb + N copies), the
    // per-row counts and starts (u32)
    uint64_t *hs_send = nullptr, *hs_recv = nullptr, *hs_ret = nullptr, *hs_ret_in = nullptr, *hs_seg = nullptr;
    uint32_t *hs_cnt = nullptr, *hs_start = nullptr;
    uint64_t hs_recv_cap = 0;
    uint64_t slot = 0, hcap = 0;
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

    // the n-domain columns a program writes: all of them (halo refresh) and,
    // by (section, row shift > 0), the shifted stores (spill to the next rank)
    struct Stores {
        std::vector<uint32_t> cols[5];
        std::vector<std::pair<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>>> shifted;
    };
    Stores st1, st2, st3p, st3;

    // shape only (no GPU): what create_sharded checks and allocates
    int shape(const zkgpu_stark_info *in, uint32_t world, uint32_t rank, bool init)
    {
        W = world;
        R = rank;
        if (!W || (W & (W - 1)) || R >= W)
            return fail("stark_create_sharded: world %u must be a power of two, rank %u < world", W, R);
        if (load(in, init)) return -1;
        H = 1ULL << eb;
        if (NE % W || N % W || NE / W < 2 * H)
            return fail("stark_create_sharded: 2^%u rows do not split into %u blocks of >= %llu rows", info.n_bits_ext,
                        W, (unsigned long long)(2 * H));
        B = NE / W;
        // leading dimensions padded to whole 512-byte runs: every column starts
        // on a cache-line boundary (an LDE into a block with ld 2^24 + 2 ran 12 %
        // slower than into ld 2^24)
        BH = B + ((H + 63) & ~63ULL);
        nb = N / W;
        hn = 0;
        const Prog *progs[4] = {&step1, &step2, &step3prev, &step3};
        Stores *sts[4] = {&st1, &st2, &st3p, &st3};
        for (int k = 0; k < 4; k++)
            if (stores_of(*progs[k], *sts[k])) return -1;
        if (hn > nb)
            return fail("stark_create_sharded: row shift %llu exceeds the %llu-row n-domain block of %u ranks",
                        (unsigned long long)hn, (unsigned long long)nb, W);
        ldn = nb + ((hn + 63) & ~63ULL);
        return 0;
    }

    int create_sharded(const zkgpu_stark_info *in, const zkgpu_comm *c)
    {
        comm = *c;
        if (shape(in, c->world, c->rank, true)) return abort_comm(-1);
        if (c->world > 1 && !c->exchange) return fail("stark_create_sharded: the communicator has no exchange");
        read_fail_hook();
        if (fit_lde_batch() || check_budget() || alloc()) return abort_comm(-1);
        return abort_comm(build_const());
    }

    // LDE column batches of 32 / 64 columns when the default (2^31 words of
    // scratch: 128 columns at 2^24 rows, 25.8 GB of workspaces) would not fit
    // beside the rank's sections (fork-9 widths at 2^23 over 2 ranks); the
    // smaller batches cost 2-3 % of LDE rate.  Process-wide
    // (zkgpu_set_lde_batch_cols), set only when needed.
    int fit_lde_batch()
    {
        uint64_t avail = 0, total = 0, need = 0;
        CK(zkgpu_device_memory(&avail, &total));
        for (uint64_t cap : {(uint64_t)0, (uint64_t)64, (uint64_t)32}) {
            lde_batch_cap = cap;
            if (plan(&need)) return -1;
            if (need <= avail) break;
        }
        if (lde_batch_cap) zkgpu_set_lde_batch_cols(lde_batch_cap);
        return 0;
    }

    // n-domain shifts of a program (reads and stores; sets hn) and its stores
    int stores_of(const Prog &p, Stores &st)
    {
        std::map<std::pair<uint32_t, uint32_t>, uint32_t> shift_of;  // (section, column) -> store shift
        std::map<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>> by_shift;
        for (const zxp_operand &o : p.opnd) {
            if ((o.kind != ZXP_COL && o.kind != ZXP_COL3) || o.a > SEC_CONST_N) continue;
            const int32_t sh = (int32_t)o.c;
            if (sh < 0)
                return fail("stark_create_sharded: negative row shift %d (the row-sharded prover reads ahead only)", sh);
            hn = std::max<uint64_t>(hn, (uint64_t)sh);
        }
        for (const zxp_instr &in : p.instr) {
            if (in.dst >= p.opnd.size()) return fail("stark_create_sharded: instruction destination out of range");
            const zxp_operand &o = p.opnd[in.dst];
            if ((o.kind != ZXP_COL && o.kind != ZXP_COL3) || o.a > SEC_CONST_N) continue;
            for (uint32_t c = o.b; c < o.b + (o.kind == ZXP_COL3 ? 3u : 1u); c++) {
                auto it = shift_of.find({o.a, c});
                if (it != shift_of.end()) {
                    if (it->second != o.c)
                        return fail("stark_create_sharded: section %u column %u stored at two row shifts", o.a, c);
                    continue;
                }
                shift_of[{o.a, c}] = o.c;
                st.cols[o.a].push_back(c);
                if (o.c) by_shift[{o.a, o.c}].push_back(c);
            }
        }
        for (auto &kv : by_shift) st.shifted.push_back(kv);
        return 0;
    }

    static uint32_t ceil_div(uint32_t a, uint32_t b) { return (a + b - 1) / b; }
    void share(uint32_t ncols, uint32_t r, uint32_t &lo, uint32_t &hi) const  // balanced contiguous column split
    {
        const uint32_t base = ncols / W, extra = ncols % W;
        lo = r * base + (r < extra ? r : extra);
        hi = lo + base + (r < extra ? 1 : 0);
    }
    uint64_t r0() const { return (uint64_t)R * nb; }  // global n-domain row of local row 0
    uint32_t max_share() const
    {
        return std::max({1u, ceil_div(info.n_cm1, W), ceil_div(info.n_cm2, W), ceil_div(info.n_cm3, W),
                         ceil_div(info.n_const, W)});
    }

    int alloc() override
    {
        if (alloc_fri()) return -1;
        memset(&S, 0, sizeof S);
        const uint32_t widths_n[5] = {info.n_cm1, info.n_cm2, info.n_cm3, info.n_tmp, info.n_const};
        uint32_t wmax = 1;
        for (int s = 0; s < 5; s++) {
            if (dalloc(&S.sec[s], (uint64_t)(widths_n[s] ? widths_n[s] : 1) * ldn)) return -1;
            S.ld[s] = ldn;
            S.ncols[s] = widths_n[s];
            wmax = std::max(wmax, widths_n[s]);
        }
        const uint32_t blk_secs[4] = {SEC_CM1_2NS, SEC_CM2_2NS, SEC_CM3_2NS, SEC_CONST_2NS};
        const uint32_t blk_w[4] = {info.n_cm1, info.n_cm2, info.n_cm3, info.n_const};
        for (int k = 0; k < 4; k++) {
            if (dalloc(&S.sec[blk_secs[k]], (uint64_t)(blk_w[k] ? blk_w[k] : 1) * BH)) return -1;
            S.ld[blk_secs[k]] = BH;
            S.ncols[blk_secs[k]] = blk_w[k];
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
        const uint64_t ms = max_share();
        // ext: the LDE of the share, and before it the transposes' receive
        // staging (W slots of ms x ldn words: more than ms x NE only for tiny
        // domains, where the 64-row halo padding is not small against nb)
        if (dalloc(&gath, 3 * NE) ||
            (W > 1 && (dalloc(&ext, std::max<uint64_t>(ms * NE, (uint64_t)W * ms * ldn)) || dalloc(&coln, ms * N))))
            return -1;
        // halo staging: the n-domain halos / spills of every column
        hcap = (uint64_t)5 * wmax * std::max<uint64_t>(hn, 1);
        if (dalloc(&hsend, hcap) || dalloc(&hrecv, hcap)) return -1;
        if (W > 1) {
            // send: a commit's column share with its halo, ld BH (the largest);
            // the quotient's q columns / piece blocks; a plookup's f / t
            // receive: q columns, piece blocks, f rows, a plookup's f / t (the
            // n-domain transpose lands in ext, free at that point)
            const uint64_t piece = 3ULL * info.q_deg * (B + nb);
            stride_s = std::max<uint64_t>({ms * BH, 3 * B, piece, 6 * nb});
            stride_r = std::max<uint64_t>({3 * B, piece, 6 * nb});
            if (dalloc(&pack_s, (W - 1) * stride_s) || dalloc(&pack_r, W * stride_r)) return -1;
        }
        if (info.n_pu && W == 1 && dalloc(&puw, 12 * N)) return -1;
        if (info.n_pu && W > 1) {
            // a rank sends <= 2 nb records (its distinct t and f keys); an
            // owner expects ~2 N / W of them, room for twice that (every rank
            // checks every owner's total before the exchange, h1h2_sharded)
            hs_recv_cap = std::min<uint64_t>(2 * N, 4 * N / W + 4096);
            uint64_t *cs = nullptr;
            if (dalloc(&hs_send, 5 * 2 * nb) || dalloc(&hs_recv, 5 * hs_recv_cap) || dalloc(&hs_ret, hs_recv_cap) ||
                dalloc(&hs_ret_in, 2 * nb) || dalloc(&hs_seg, 3 * (nb + N)) || dalloc(&cs, nb))
                return -1;
            hs_cnt = (uint32_t *)cs;
            hs_start = hs_cnt + nb;
        }
        for (auto &t : trees)
            if (dalloc(&t.nodes, zkgpu_gl_merkle_num_elements(B))) return -1;
        slot = std::max<uint64_t>({4, 2ULL * W, 3ULL * info.n_ev, (uint64_t)q() * s0_record()});
        ftrees.assign(fri_steps.size(), Tree{});
        for (size_t si = 1; si < fri_steps.size(); si++) {
            const uint64_t ngroups = 1ULL << fri_steps[si], width = (3ULL << fri_steps[si - 1]) / ngroups;
            if (!fri_sharded(ngroups)) continue;
            if (dalloc(&ftrees[si].nodes, zkgpu_gl_merkle_num_elements(ngroups / W))) return -1;
            slot = std::max<uint64_t>(slot, (uint64_t)q() * (width + 4ULL * fri_steps[si]));
        }
        return dalloc(&xchg, slot * W);
    }

    // the constants' whole copy while they are set up and committed (set_const:
    // plus the row-major staging of the host's rows)
    // the constants' whole copy lives in coln and set_const's row-major
    // staging in ext when they are large enough (both are free during setup:
    // the constant commit extends from the whole copy into ext after the
    // staging is done), else in transient allocations
    uint64_t const_words() const { return (uint64_t)(info.n_const ? info.n_const : 1) * N; }
    uint64_t ext_words() const
    {
        return W > 1 ? std::max<uint64_t>((uint64_t)max_share() * NE, (uint64_t)W * max_share() * ldn) : 0;
    }
    uint64_t coln_words() const { return W > 1 ? (uint64_t)max_share() * N : 0; }
    uint64_t setup_bytes() const override
    {
        return 8 * ((coln_words() >= const_words() ? 0 : const_words()) + (ext_words() >= const_words() ? 0 : const_words()));
    }
    // a setup buffer of `words`: `have` (of `cap` words) when it fits, else a
    // transient allocation (*owned set)
    int setup_buffer(uint64_t **p, uint64_t *have, uint64_t cap, uint64_t words, void **owned)
    {
        *owned = nullptr;
        if (have && cap >= words) {
            *p = have;
            return 0;
        }
        CK(zkgpu_dev_malloc(owned, words * 8));
        *p = (uint64_t *)*owned;
        return 0;
    }
    uint64_t lde_cols_max() const override { return max_share(); }
    uint64_t prog_rows_max() const override { return std::max(B, nb); }

    uint64_t s0_record() const
    {
        return (uint64_t)info.n_cm1 + info.n_cm2 + info.n_cm3 + info.n_cm4 + info.n_const + 20ULL * info.n_bits_ext;
    }

    // Collective: every rank calls it at the same point of the proof, with
    // whatever it has to send and receive -- possibly nothing (a rank whose
    // multiset segment is all its own rows, calculateH1H2): the host exchange
    // is a barrier per call, so a rank that skipped an empty exchange would
    // pair its next one with the others' current one.
    //
    // A rank that cannot take part (it refuses the exchange, or fails before
    // it) returns an error; prove() / create_sharded() then abort the
    // communicator (zkgpu_comm.abort), which fails the peers' exchanges
    // instead of leaving them waiting for this rank.
    int exchange()
    {
        if (W == 1) {
            ops.clear();
            return 0;
        }
        max_ops = std::max(max_ops, (uint32_t)ops.size());
        if (ops.size() > 2ULL * (W - 1)) {
            const size_t n = ops.size();
            ops.clear();
            return fail("exchange of %zu operations: more than one send and one receive per peer", n);
        }
        if (fail_at && n_exch_total + 1 == fail_at) {  // test hook (ZKGPU_TEST_FAIL_EXCHANGE)
            ops.clear();
            return fail("injected failure before exchange %llu on rank %u", (unsigned long long)fail_at, R);
        }
        n_exch_total++;
        // the exchange's device interval (stream marks around it; resolved
        // with the stage timers): bytes / time = the achieved link rate
        uint32_t m0 = UINT32_MAX;
        if (n_marks + 3 < ZKGPU_MARKS && !zkgpu_mark(n_marks)) m0 = n_marks++;
        if (comm.exchange(comm.ctx, ops.data(), (uint32_t)ops.size())) {
            const std::string why = last_error_text();
            return fail("zkgpu_comm exchange of %zu operations failed (rank %u of %u): %s", ops.size(), R, W,
                        why.c_str());
        }
        uint64_t sent = 0;
        for (const zkgpu_comm_op &o : ops)
            if (o.send) sent += o.bytes;
        if (m0 != UINT32_MAX && !zkgpu_mark(n_marks)) pend_x.push_back({{m0, n_marks++}, sent});
        n_exch++;
        sent_bytes += sent;
        max_sent = std::max(max_sent, sent);
        ops.clear();
        return 0;
    }
    // the injected failure of the tests: rank r fails before its k-th
    // exchange (ZKGPU_TEST_FAIL_EXCHANGE = "r:k"), k counted from creation
    uint64_t fail_at = 0, n_exch_total = 0;
    void read_fail_hook()
    {
        const char *e = getenv("ZKGPU_TEST_FAIL_EXCHANGE");
        unsigned r = 0;
        unsigned long long k = 0;
        if (e && sscanf(e, "%u:%llu", &r, &k) == 2 && r == R) fail_at = k;
    }
    // a failed sharded call on this rank: release the peers
    int abort_comm(int rc)
    {
        if (rc && W > 1 && comm.abort) {
            const std::string why = last_error_text();
            (void)comm.abort(comm.ctx);
            fail("%s (rank %u aborted the communicator)", why.c_str(), R);
        }
        return rc;
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

    // the rank's 3 x B block (ld B: one contiguous 3B-word message) of f ->
    // full (3 x NE, ld NE) on every rank
    int gather_rows(const uint64_t *blk, uint64_t *full)
    {
        for (uint32_t d = 0; d < W; d++)
            if (d != R) op(d, 1, blk, 3 * B * 8);
        for (uint32_t s = 0; s < W; s++)
            if (s != R) op(s, 0, pack_r + s * stride_r, 3 * B * 8);
        CK(zkgpu_copy_rows_dev(full, NE, (uint64_t)R * B, nullptr, blk, B, 0, 0, nullptr, 3, B));
        if (exchange()) return -1;
        for (uint32_t s = 0; s < W; s++)
            if (s != R) CK(zkgpu_copy_rows_dev(full, NE, (uint64_t)s * B, nullptr, pack_r + s * stride_r, B, 0, 0, nullptr, 3, B));
        return 0;
    }

    // quotient split (starks.cpp:255-296) by column owners: q column j
    // (j < 3) belongs to rank j mod W.  The q blocks go to the owners (one
    // message per peer), each owner interpolates its column over the whole
    // extended domain, splits it into q_deg pieces (output columns 3p + j) and
    // evaluates them on the extended and the n domain; every rank gets the
    // row blocks of all pieces back (one message per owner).  Replaces the
    // transform of all three columns on every rank.
    std::vector<uint32_t> q_owned(uint32_t r) const
    {
        std::vector<uint32_t> j;
        for (uint32_t c = r; c < 3; c += W) j.push_back(c);
        return j;
    }
    std::vector<uint32_t> pieces_of(const std::vector<uint32_t> &js) const
    {
        std::vector<uint32_t> c;
        for (uint32_t p = 0; p < info.q_deg; p++)
            for (uint32_t j : js) c.push_back(3 * p + j);
        return c;
    }
    int quotient_sharded()
    {
        const std::vector<uint32_t> mine = q_owned(R), my_pieces = pieces_of(mine);
        const uint64_t *qb = S.sec[SEC_Q_2NS];
        // 1. q blocks to the column owners; the owned columns whole in gath
        for (uint32_t d = 0; d < W; d++) {
            const std::vector<uint32_t> js = q_owned(d);
            if (d == R || js.empty()) continue;
            CK(zkgpu_copy_rows_dev(psend(d), B, 0, nullptr, qb, B, 0, 0, js.data(), (uint32_t)js.size(), B));
            op(d, 1, psend(d), js.size() * B * 8);
        }
        if (!mine.empty()) {
            for (uint32_t s = 0; s < W; s++)
                if (s != R) op(s, 0, pack_r + s * stride_r, mine.size() * B * 8);
            CK(zkgpu_copy_rows_dev(gath, NE, (uint64_t)R * B, nullptr, qb, B, 0, 0, mine.data(), (uint32_t)mine.size(), B));
        }
        if (exchange()) return -1;
        for (uint32_t s = 0; s < W && !mine.empty(); s++)
            if (s != R)
                CK(zkgpu_copy_rows_dev(gath, NE, (uint64_t)s * B, nullptr, pack_r + s * stride_r, B, 0, 0, nullptr,
                                       (uint32_t)mine.size(), B));
        // 2. the owner's pieces (quotient_pieces for its columns)
        const uint64_t shift_in = pw(inv(7), N);
        for (size_t k = 0; k < mine.size(); k++) {
            const uint32_t j = mine[k];
            CK(zkgpu_gl_ntt_dev(qq1 + k * NE, NE, gath + k * NE, NE, NE, 1, 1));
            for (uint32_t p = 0; p < info.q_deg; p++) CK(zkgpu_memset_dev(qq2 + (uint64_t)(3 * p + j) * NE, 0, NE * 8));
            CK(zkgpu_qsplit_cols_dev(qq2 + (uint64_t)j * NE, NE, qq1 + k * NE, NE, N, info.q_deg, shift_in, 1, 3));
            CK(zkgpu_gl_ntt_dev(cm4 + (uint64_t)j * NE, 3 * NE, qq2 + (uint64_t)j * NE, 3 * NE, NE, info.q_deg, 0));
            for (uint32_t p = 0; p < info.q_deg; p++)
                CK(zkgpu_memcpy_d2d(cm4_n + (uint64_t)(3 * p + j) * N, qq2 + (uint64_t)(3 * p + j) * NE, N * 8));
            CK(zkgpu_scale_by_powers_dev(cm4_n + (uint64_t)j * N, 3 * N, info.q_deg, N, inv(7)));
            CK(zkgpu_gl_ntt_dev(cm4_n + (uint64_t)j * N, 3 * N, cm4_n + (uint64_t)j * N, 3 * N, N, info.q_deg, 0));
        }
        // 3. every rank its row blocks of every piece (extended and n domain)
        const uint32_t np = (uint32_t)my_pieces.size();
        for (uint32_t d = 0; d < W && np; d++) {
            if (d == R) continue;
            uint64_t *m = psend(d);
            CK(zkgpu_copy_rows_dev(m, B, 0, nullptr, cm4, NE, (uint64_t)d * B, 0, my_pieces.data(), np, B));
            CK(zkgpu_copy_rows_dev(m + (uint64_t)np * B, nb, 0, nullptr, cm4_n, N, (uint64_t)d * nb, 0, my_pieces.data(),
                                   np, nb));
            op(d, 1, m, (uint64_t)np * (B + nb) * 8);
        }
        for (uint32_t s = 0; s < W; s++) {
            const uint32_t ns = (uint32_t)pieces_of(q_owned(s)).size();
            if (s != R && ns) op(s, 0, pack_r + s * stride_r, (uint64_t)ns * (B + nb) * 8);
        }
        if (exchange()) return -1;
        for (uint32_t s = 0; s < W; s++) {
            const std::vector<uint32_t> ps = pieces_of(q_owned(s));
            if (s == R || ps.empty()) continue;
            const uint32_t ns = (uint32_t)ps.size();
            CK(zkgpu_copy_rows_dev(cm4, NE, (uint64_t)R * B, ps.data(), pack_r + s * stride_r, B, 0, 0, nullptr, ns, B));
            CK(zkgpu_copy_rows_dev(cm4_n, N, r0(), ps.data(), pack_r + s * stride_r + (uint64_t)ns * B, nb, 0, 0,
                                   nullptr, ns, nb));
        }
        return 0;
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

    // ---- n domain
    // the NTT transpose: rows [0, nb) of every column of n-domain section sec
    // to the rank owning the column; the rank's share [lo, hi) arrives in
    // coln (ld N) at rows [s nb, (s+1) nb) from rank s
    // One message per peer: the peer's columns [dlo, dhi) of the block are
    // contiguous (ld ldn; their halo / padding rows travel along, ~64 / nb of
    // the bytes); received into ext (free until the LDE), then placed.
    int rows_to_share(uint32_t sec, uint32_t ncols)
    {
        uint32_t lo, hi;
        share(ncols, R, lo, hi);
        const uint64_t slot = (uint64_t)max_share() * ldn;
        for (uint32_t d = 0; d < W; d++) {
            uint32_t dlo, dhi;
            share(ncols, d, dlo, dhi);
            if (d == R || dhi == dlo) continue;
            op(d, 1, S.sec[sec] + (uint64_t)dlo * ldn, (uint64_t)(dhi - dlo) * ldn * 8);
        }
        for (uint32_t s = 0; s < W && hi > lo; s++)
            if (s != R) op(s, 0, ext + s * slot, (uint64_t)(hi - lo) * ldn * 8);
        if (hi > lo)
            CK(zkgpu_copy_rows_dev(coln, N, r0(), nullptr, S.sec[sec] + (uint64_t)lo * ldn, ldn, 0, 0, nullptr, hi - lo, nb));
        if (exchange()) return -1;
        for (uint32_t s = 0; s < W && hi > lo; s++)
            if (s != R)
                CK(zkgpu_copy_rows_dev(coln, N, (uint64_t)s * nb, nullptr, ext + s * slot, ldn, 0, 0, nullptr, hi - lo, nb));
        return 0;
    }

    // rows [0, hn) of every written column -> the previous rank's halo rows
    // [nb, nb + hn) (the last rank's halo is the domain's first rows)
    int refresh_halos(const std::vector<uint32_t> cols[5])
    {
        if (!hn) return 0;
        uint64_t off = 0;
        for (uint32_t s = 0; s < 5; s++) {
            const uint32_t n = (uint32_t)cols[s].size();
            if (!n) continue;
            if (off + (uint64_t)n * hn > hcap) return fail("halo refresh: %u columns exceed the staging", n);
            CK(zkgpu_copy_rows_dev(hsend + off, hn, 0, nullptr, S.sec[s], ldn, 0, 0, cols[s].data(), n, hn));
            off += (uint64_t)n * hn;
        }
        if (!off) return 0;
        const uint64_t *in = hsend;
        if (W > 1) {
            op((R + W - 1) % W, 1, hsend, off * 8);
            op((R + 1) % W, 0, hrecv, off * 8);
            if (exchange()) return -1;
            in = hrecv;
        }
        off = 0;
        for (uint32_t s = 0; s < 5; s++) {
            const uint32_t n = (uint32_t)cols[s].size();
            if (!n) continue;
            CK(zkgpu_copy_rows_dev(S.sec[s], ldn, nb, cols[s].data(), in + off, hn, 0, 0, nullptr, n, hn));
            off += (uint64_t)n * hn;
        }
        return 0;
    }

    // a store at row shift s writes local rows [s, nb + s): rows [nb, nb + s)
    // are the next rank's first s rows (the single-GPU store wraps mod N)
    int spill(const Stores &st)
    {
        if (st.shifted.empty()) return 0;
        uint64_t off = 0;
        for (const auto &g : st.shifted) {
            const uint32_t sec = g.first.first, sh = g.first.second, n = (uint32_t)g.second.size();
            if (off + (uint64_t)n * sh > hcap) return fail("shifted-store spill exceeds the staging");
            CK(zkgpu_copy_rows_dev(hsend + off, sh, 0, nullptr, S.sec[sec], ldn, nb, 0, g.second.data(), n, sh));
            off += (uint64_t)n * sh;
        }
        const uint64_t *in = hsend;
        if (W > 1) {
            op((R + 1) % W, 1, hsend, off * 8);
            op((R + W - 1) % W, 0, hrecv, off * 8);
            if (exchange()) return -1;
            in = hrecv;
        }
        off = 0;
        for (const auto &g : st.shifted) {
            const uint32_t sec = g.first.first, sh = g.first.second, n = (uint32_t)g.second.size();
            CK(zkgpu_copy_rows_dev(S.sec[sec], ldn, 0, g.second.data(), in + off, sh, 0, 0, nullptr, n, sh));
            off += (uint64_t)n * sh;
        }
        return 0;
    }

    // an n-domain stage program over the rank's rows, then the spill of its
    // shifted stores and the halo refresh of everything it wrote
    int run_n(const Prog &p, const Stores &st, const uint64_t ch[24])
    {
        if (p.instr.empty()) return 0;
        uint32_t log_nb = 0;
        while ((1ULL << log_nb) < nb) log_nb++;
        const uint64_t ev0[3] = {0, 0, 0};
        CK(zkgpu_zxp_eval_block_dev(p.instr.data(), (uint32_t)p.instr.size(), p.opnd.data(), (uint32_t)p.opnd.size(),
                                    p.n_tmp1 ? p.n_tmp1 : 1, p.n_tmp3 ? p.n_tmp3 : 1, &S, log_nb, info.n_bits, ch,
                                    publics.data(), (uint32_t)publics.size(), ev0, 0, nullptr, nullptr, 0,
                                    pw(w_of(info.n_bits), r0())));
        if (spill(st)) return -1;
        return refresh_halos(st.cols);
    }

    const uint64_t *ncol(uint32_t ev_sec, uint32_t col, uint64_t row, uint64_t &ld) const override
    {
        if (ev_sec == SEC_CM4_2NS) return Starks::ncol(ev_sec, col, row, ld);  // the pieces are whole
        ld = ldn;
        const uint32_t s = ev_sec == SEC_CONST_2NS ? (uint32_t)SEC_CONST_N : ev_sec - SEC_CM1_2NS + SEC_CM1_N;
        return S.sec[s] + (uint64_t)col * ldn + (row - r0());
    }

    // ---- setup and trace
    // constants: a transient whole copy (rand + L_first + step0, or the
    // host's rows), committed from it, then cut to the rank's rows
    int const_from_whole(uint64_t *whole)
    {
        uint32_t lo, hi;
        share(info.n_const, R, lo, hi);
        if (commit_cols(trees[4], SEC_CONST_2NS, whole + (uint64_t)lo * N, N, info.n_const, verkey, nullptr, nullptr,
                        nullptr))
            return -1;
        CK(zkgpu_copy_rows_dev(S.sec[SEC_CONST_N], ldn, 0, nullptr, whole, N, r0(), info.n_bits, nullptr,
                               info.n_const, ldn));
        CK(zkgpu_synchronize());
        return 0;
    }

    int build_const() override
    {
        void *w = nullptr;
        uint64_t *whole = nullptr;
        if (setup_buffer(&whole, coln, coln_words(), const_words(), &w)) return -1;
        const zkgpu_sections blocks = S;
        S.sec[SEC_CONST_N] = whole;  // Starks::build_const's fill on the whole domain ...
        S.ld[SEC_CONST_N] = N;
        int rc = fill_const();
        S = blocks;
        if (!rc) rc = const_from_whole(whole);  // ... then the commit and the cut
        if (w) zkgpu_dev_free(w);
        if (!rc) init_publics();
        return rc;
    }

    int set_const(const uint64_t *rows) override
    {
        void *w = nullptr, *t = nullptr;
        uint64_t *whole = nullptr, *tmp = nullptr;
        if (setup_buffer(&whole, coln, coln_words(), const_words(), &w)) return -1;
        int rc = setup_buffer(&tmp, ext, ext_words(), const_words(), &t);
        if (!rc) rc = zkgpu_memcpy_h2d(tmp, rows, (uint64_t)info.n_const * N * 8);
        if (!rc) rc = zkgpu_rows_to_cols_dev(whole, N, tmp, N, info.n_const);
        if (!rc) rc = zkgpu_synchronize();
        if (t) zkgpu_dev_free(t);
        if (rc) {
            if (w) zkgpu_dev_free(w);
            return fail("set_const: %s", zkgpu_last_error());
        }
        rc = const_from_whole(whole);
        if (w) zkgpu_dev_free(w);
        return rc;
    }

    int commit_const() override { return fail("stark (sharded): constants are committed from their whole copy"); }
    // the rank's rows of the next proof's trace, loaded during this prove (as
    // set_cm1: rows [r0, r0 + ldn) mod N, so up to two host pieces)
    int set_cm1_async(const uint64_t *rows) override
    {
        if (take_cm1_async(false)) return -1;
        const uint64_t w = info.n_cm1, first = std::min(ldn, N - r0());
        if (cm1_next_alloc(ldn, 2)) return -1;
        if (zkgpu_load_rows_async(cm1_next, ldn, rows + r0() * w, first, w, 0, cm1_xfer[0], xfer_bytes, &cm1_ticket[0]) ||
            (ldn > first && zkgpu_load_rows_async(cm1_next + first, ldn, rows, ldn - first, w, 0, cm1_xfer[1], xfer_bytes,
                                                  &cm1_ticket[1]))) {
            cm1_pending = true;  // wait for whatever started
            (void)take_cm1_async(false);
            return fail("set_cm1_async: %s", zkgpu_last_error());
        }
        cm1_pending = true;
        return 0;
    }
    int get_cm1(uint64_t *) override { return fail("stark (sharded): get_cm1 is single-GPU only"); }

    // the executor's row-major buffer: the rank takes rows [r0, r0 + ldn) mod N
    int set_cm1(const uint64_t *rows) override
    {
        void *t = nullptr;
        uint64_t *tmp = nullptr;
        const uint64_t w = info.n_cm1, first = std::min(ldn, N - r0());
        // the row-major staging in ext (free between proofs) when it fits
        if (setup_buffer(&tmp, ext, ext_words(), std::max<uint64_t>(1, w * ldn), &t)) return -1;
        int rc = zkgpu_memcpy_h2d(tmp, rows + r0() * w, first * w * 8);
        if (!rc && ldn > first) rc = zkgpu_memcpy_h2d(tmp + first * w, rows, (ldn - first) * w * 8);
        if (!rc) rc = zkgpu_rows_to_cols_dev(S.sec[SEC_CM1_N], ldn, tmp, ldn, info.n_cm1);
        if (!rc) rc = zkgpu_synchronize();
        if (t) zkgpu_dev_free(t);
        if (rc) return fail("set_cm1: %s", zkgpu_last_error());
        return 0;
    }

    int witness() override
    {
        CK(zkgpu_memset_dev(S.sec[SEC_CM1_N], 0, (uint64_t)info.n_cm1 * ldn * 8));
        CK(zkgpu_rand_cols_rows_dev(S.sec[SEC_CM1_N], ldn, random_cols.data(), (uint32_t)random_cols.size(), r0(), ldn,
                                    info.n_bits, info.seed, 0));
        uint64_t ch[24] = {0};
        if (run_n(step1, st1, ch)) return -1;
        CK(zkgpu_synchronize());
        return 0;
    }

    // ---- commits
    // LDE of the rank's column share (src: its first column, ld src_ld),
    // column -> row exchange (halos packed), subtree
    int commit_cols(Tree &t, uint32_t sec_e, const uint64_t *src, uint64_t src_ld, uint32_t ncols, uint64_t root[4],
                    const char *lde_name, const char *xchg_name, const char *tree_name)
    {
        uint32_t lo, hi;
        share(ncols, R, lo, hi);
        uint64_t *blk = S.sec[sec_e];
        if (W == 1) {  // one rank: the LDE straight into the block, then its halo (the first rows)
            tstart();
            CK(zkgpu_gl_extend_pol_dev(blk, BH, src, src_ld, NE, N, ncols));
            CK(zkgpu_copy_rows_dev(blk, BH, B, nullptr, blk, BH, 0, 0, nullptr, ncols, H));
            if (lde_name && tstop(lde_name)) return -1;
            tstart();
            if (merkelize(t, blk, BH, ncols, root)) return -1;
            if (tree_name && tstop(tree_name)) return -1;
            return 0;
        }
        tstart();
        if (hi > lo) CK(zkgpu_gl_extend_pol_dev(ext, NE, src, src_ld, NE, N, hi - lo));
        if (lde_name && tstop(lde_name)) return -1;
        tstart();
        // peer d's rows [d B, d B + B + H) (mod NE: the halo of the last
        // block wraps) of the share, packed with the block's own ld BH: the
        // message lands as whole block columns [lo, hi) on the peer
        uint32_t log_ne = 0;
        while ((1ULL << log_ne) < NE) log_ne++;
        for (uint32_t d = 0; d < W; d++) {
            if (d == R || hi == lo) continue;
            CK(zkgpu_copy_rows_dev(psend(d), BH, 0, nullptr, ext, NE, (uint64_t)d * B, log_ne, nullptr,
                                   hi - lo, B + H));
            op(d, 1, psend(d), (uint64_t)(hi - lo) * BH * 8);
        }
        for (uint32_t s = 0; s < W; s++) {
            uint32_t slo, shi;
            share(ncols, s, slo, shi);
            if (s == R || shi == slo) continue;
            op(s, 0, blk + (uint64_t)slo * BH, (uint64_t)(shi - slo) * BH * 8);
        }
        if (hi > lo)
            CK(zkgpu_copy_rows_dev(blk + (uint64_t)lo * BH, BH, 0, nullptr, ext, NE, (uint64_t)R * B, log_ne, nullptr,
                                   hi - lo, B + H));
        if (exchange()) return -1;
        if (xchg_name && tstop(xchg_name)) return -1;
        tstart();
        if (merkelize(t, blk, BH, ncols, root)) return -1;
        if (tree_name && tstop(tree_name)) return -1;
        return 0;
    }

    // a stage's n-domain section: transpose to column shares, then commit
    int commit_n(Tree &t, uint32_t sec_n, uint32_t sec_e, uint32_t ncols, uint64_t root[4], const char *lde_name,
                 const char *xchg_name, const char *tree_name)
    {
        if (W == 1)  // the rank holds every row: no transpose
            return commit_cols(t, sec_e, S.sec[sec_n], ldn, ncols, root, lde_name, xchg_name, tree_name);
        tstart();
        if (rows_to_share(sec_n, ncols)) return -1;
        if (xchg_name && tstop((std::string(xchg_name) + "_T").c_str())) return -1;
        return commit_cols(t, sec_e, coln, N, ncols, root, lde_name, xchg_name, tree_name);
    }

    bool fri_sharded(uint64_t ngroups) const { return W > 1 && ngroups % W == 0 && ngroups / W >= 2; }

    // ---- FRI's first layer over the ranks (friProve.cpp:44-133)
    // Layer 1's group g < w = 2^steps[1] holds the kk = 2^(steps[0] - steps[1])
    // elements f[g + k w], and the first fold maps exactly those to folded
    // element g.  Rank R's f rows [R B, (R+1) B) are k in [R kk/W, (R+1) kk/W)
    // of every group, so ONE all-to-all (rank s sends d its kk/W chunks of d's
    // bl = w / W groups, 3 columns: 3 NE / W^2 words per peer) leaves each rank
    // all kk elements of its bl groups: its block of layer 1's tree rows
    // (getTransposed) and the input of its block of the first fold.  The fold
    // output (1/kk of f) is then all-gathered and the later, smaller layers run
    // as before.  Replaces the all-gather of f (3 NE words to every rank) and
    // the fold of the whole 2^steps[0] domain on every rank.
    // Invariant: when this holds, fri_pol[0] is never filled (f stays in the
    // rank's row blocks, S.sec[SEC_F_2NS]); the FRI loop passes a null pol to
    // fri_transpose_layer(0, ...), whose override below reads the blocks.
    bool fri_pol0_filled() const override { return !fri_first_sharded(); }
    bool fri_first_sharded() const
    {
        if (W == 1 || fri_steps.size() < 2) return false;
        const uint64_t w = 1ULL << fri_steps[1], kk = 1ULL << (fri_steps[0] - fri_steps[1]);
        return kk % W == 0 && fri_sharded(w);
    }

    int fri_transpose_layer(size_t si, uint64_t *aux, const uint64_t *pol, uint64_t degree, uint32_t nb) override
    {
        if (si != 0 || !fri_first_sharded()) return Starks::fri_transpose_layer(si, aux, pol, degree, nb);
        (void)pol;  // null here (fri_pol0_filled)
        const uint64_t w = 1ULL << nb, kk = NE / w, kw = kk / W, bl = w / W, msg = 3 * kw * bl;
        const uint64_t *f = S.sec[SEC_F_2NS];  // the rank's f rows: 3 columns, ld B
        // one message per peer, column-major bl x 3 kw (column 3 kc + c: chunk
        // kc, component c); the rank's own lands straight in gath
        for (uint32_t d = 0; d < W; d++) {
            uint64_t *m = d == R ? gath + (uint64_t)R * msg : psend(d);
            for (uint64_t kc = 0; kc < kw; kc++)
                CK(zkgpu_copy_rows_dev(m + kc * 3 * bl, bl, 0, nullptr, f + kc * w + (uint64_t)d * bl, B, 0, 0, nullptr,
                                       3, bl));
            if (d != R) op(d, 1, m, msg * 8);
        }
        for (uint32_t s = 0; s < W; s++)
            if (s != R) op(s, 0, gath + (uint64_t)s * msg, msg * 8);
        if (exchange()) return -1;
        // gath is now a column-major bl x 3 kk matrix, column 3 k + c = element
        // k (from rank k / kw), component c: the row-major transpose is the
        // groups' getTransposed rows
        CK(zkgpu_cols_to_rows_dev(aux + (uint64_t)R * bl * 3 * kk, gath, bl, bl, 3 * kk));
        return 0;
    }

    int fri_fold_step(size_t si, uint64_t *dst, const uint64_t *src, uint32_t pol_bits, uint32_t out_bits,
                      const uint64_t sx[3], uint64_t shift_inv) override
    {
        if (si != 1 || !fri_first_sharded())
            return Starks::fri_fold_step(si, dst, src, pol_bits, out_bits, sx, shift_inv);
        const uint64_t w = 1ULL << out_bits, bl = w / W, kk = 1ULL << (pol_bits - out_bits);
        CK(zkgpu_fri_fold_rows_dev(dst + 3ULL * R * bl, fri_aux[1] + (uint64_t)R * bl * 3 * kk, (uint64_t)R * bl, bl,
                                   pol_bits, out_bits, sx, shift_inv));
        for (uint32_t d = 0; d < W; d++)
            if (d != R) op(d, 1, dst + 3ULL * R * bl, 3 * bl * 8);
        for (uint32_t s = 0; s < W; s++)
            if (s != R) op(s, 0, dst + 3ULL * s * bl, 3 * bl * 8);
        return exchange();
    }

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
    // block: z = prod of the ratios before each row, the block total
    // all-gathered, the block redone with z0 = the product of the earlier
    // ranks' totals (rank 0's is already final); then the z halos
    int z_all() override
    {
        Stores zs;
        for (uint32_t zi = 0; zi < info.n_zctx; zi++) {
            uint64_t *z = S.sec[SEC_CM3_N] + (uint64_t)zctx[3 * zi + 2] * ldn;
            const uint64_t *num = S.sec[SEC_TMP_N] + (uint64_t)zctx[3 * zi] * ldn;
            const uint64_t *den = S.sec[SEC_TMP_N] + (uint64_t)zctx[3 * zi + 1] * ldn;
            const uint64_t one[3] = {1, 0, 0};
            uint64_t tot[3];
            CK(zkgpu_calculate_z_block_dev(z, ldn, num, ldn, den, ldn, nb, one, tot));
            std::vector<uint64_t> all;
            if (allgather(tot, 3, all)) return -1;
            uint64_t pre[3] = {1, 0, 0}, acc[3] = {1, 0, 0};
            for (uint32_t s = 0; s < W; s++) {
                if (s == R) memcpy(pre, acc, 24);
                mul3(acc, acc, &all[3 * s]);
            }
            if (acc[0] != 1 || acc[1] || acc[2]) return fail("calculateZ: grand product %u does not close", zi);
            if (pre[0] != 1 || pre[1] || pre[2])
                CK(zkgpu_calculate_z_block_dev(z, ldn, num, ldn, den, ldn, nb, pre, tot));
            for (uint32_t c = 0; c < 3; c++) zs.cols[SEC_CM3_N].push_back(zctx[3 * zi + 2] + c);
        }
        return refresh_halos(zs.cols);
    }

    // calculateH1H2 of plookup k over the ranks (zkgpu_h1h2_shard_*,
    // include/zkgpu.h): each rank routes its distinct t / f keys to the key's
    // owner, the owner finds each key's last table row and its f count, the
    // counts go back to the table rows' ranks, every rank deals its table
    // rows' copies into its segment of the 2N-long multiset (offset = the
    // earlier ranks' totals) and sends each piece to the rank holding those
    // h1 / h2 rows.  Five exchanges (two of them small all-gathers), at most
    // one message per peer each; the data moved is the distinct keys and the
    // multiset, not f and t to every rank.
    int h1h2_sharded(uint32_t k)
    {
        const uint32_t *q = &pu[5 * k];
        const uint32_t d = q[4];
        const uint64_t *f = S.sec[SEC_TMP_N] + (uint64_t)q[0] * ldn, *t = S.sec[SEC_TMP_N] + (uint64_t)q[1] * ldn;
        uint64_t *h1 = S.sec[SEC_CM2_N] + (uint64_t)q[2] * ldn, *h2 = S.sec[SEC_CM2_N] + (uint64_t)q[3] * ldn;
        // 1. the rank's records, bucketed by owner
        std::vector<uint32_t> nt(W), nf(W);
        CK(zkgpu_h1h2_shard_route(hs_send, 2 * nb, nt.data(), nf.data(), f, ldn, t, ldn, nb, r0(), d, W));
        std::vector<uint64_t> mine(2 * W), all;
        for (uint32_t o = 0; o < W; o++) {
            mine[2 * o] = nt[o];
            mine[2 * o + 1] = nf[o];
        }
        if (allgather(mine.data(), 2 * W, all)) return -1;
        auto nt_of = [&](uint32_t s, uint32_t o) { return all[(uint64_t)s * 2 * W + 2 * o]; };
        auto nr_of = [&](uint32_t s, uint32_t o) { return all[(uint64_t)s * 2 * W + 2 * o] + all[(uint64_t)s * 2 * W + 2 * o + 1]; };
        std::vector<uint64_t> soff(W + 1, 0), roff(W + 1, 0);
        for (uint32_t o = 0; o < W; o++) soff[o + 1] = soff[o] + nr_of(R, o);
        for (uint32_t s = 0; s < W; s++) roff[s + 1] = roff[s] + nr_of(s, R);
        for (uint32_t o = 0; o < W; o++) {  // the same verdict on every rank, before anything moves
            uint64_t tot = 0;
            for (uint32_t s = 0; s < W; s++) tot += nr_of(s, o);
            if (tot > hs_recv_cap)
                return fail("calculateH1H2 (sharded): rank %u owns %llu keys, more than its %llu-record buffer", o,
                            (unsigned long long)tot, (unsigned long long)hs_recv_cap);
        }
        // 2. records to their owners
        const uint64_t RW = 5 * 8;  // bytes per record
        for (uint32_t o = 0; o < W; o++)
            if (o != R && nr_of(R, o)) op(o, 1, hs_send + 5 * soff[o], nr_of(R, o) * RW);
        for (uint32_t s = 0; s < W; s++)
            if (s != R && nr_of(s, R)) op(s, 0, hs_recv + 5 * roff[s], nr_of(s, R) * RW);
        if (nr_of(R, R)) CK(zkgpu_memcpy_d2d(hs_recv + 5 * roff[R], hs_send + 5 * soff[R], nr_of(R, R) * RW));
        if (exchange()) return -1;
        // 3. the owner's side, then each t record's count back to its sender
        uint64_t miss = ~0ULL;
        CK(zkgpu_h1h2_shard_owner(hs_ret, hs_recv, roff[W], d, &miss));
        for (uint32_t s = 0; s < W; s++)
            if (s != R && nt_of(s, R)) op(s, 1, hs_ret + roff[s], nt_of(s, R) * 8);
        for (uint32_t o = 0; o < W; o++)
            if (o != R && nt_of(R, o)) op(o, 0, hs_ret_in + soff[o], nt_of(R, o) * 8);
        if (nt_of(R, R)) CK(zkgpu_memcpy_d2d(hs_ret_in + soff[R], hs_ret + roff[R], nt_of(R, R) * 8));
        if (exchange()) return -1;
        // 4. counts, the rank's multiset total; totals and the smallest missing f row everywhere
        uint64_t tot = 0;
        CK(zkgpu_h1h2_shard_counts(hs_start, hs_cnt, &tot, hs_send, hs_ret_in, soff[W], nb, r0()));
        const uint64_t tm[2] = {tot, miss};
        std::vector<uint64_t> tms;
        if (allgather(tm, 2, tms)) return -1;
        uint64_t gmiss = ~0ULL, O = 0, sum = 0;
        std::vector<uint64_t> off(W);
        for (uint32_t s = 0; s < W; s++) {
            gmiss = std::min(gmiss, tms[2 * s + 1]);
            off[s] = sum;
            sum += tms[2 * s];
        }
        if (gmiss != ~0ULL)
            return fail("Polinomial::calculateH1H2() Number not included: w=%llu plookup_number=%u",
                        (unsigned long long)gmiss, k);
        if (sum != 2 * N) return fail("calculateH1H2 (sharded): the multiset has %llu entries, not 2N", (unsigned long long)sum);
        O = off[R];
        // 5. the rank's segment [O, O + tot) of the multiset, each piece to the rank holding its h rows
        const uint64_t sld = tot ? tot : 1;
        CK(zkgpu_h1h2_shard_deal(hs_seg, sld, t, ldn, hs_start, hs_cnt, nb, d));
        auto piece = [&](uint64_t o0, uint64_t len, uint32_t e, uint64_t &a, uint64_t &b) {
            a = std::max<uint64_t>(o0, 2ULL * e * nb);
            b = std::min<uint64_t>(o0 + len, 2ULL * (e + 1) * nb);
            return a < b;
        };
        for (uint32_t e = 0; e < W; e++) {
            uint64_t a, b;
            if (!piece(O, tot, e, a, b)) continue;
            if (e == R) {
                CK(zkgpu_h1h2_shard_place(h1, ldn, h2, ldn, hs_seg + (a - O), sld, a, b - a, r0(), d));
                continue;
            }
            CK(zkgpu_copy_rows_dev(psend(e), b - a, 0, nullptr, hs_seg, sld, a - O, 0, nullptr, d, b - a));
            op(e, 1, psend(e), (b - a) * d * 8);
        }
        std::vector<std::pair<uint64_t, uint64_t>> got(W, {0, 0});
        for (uint32_t s = 0; s < W; s++) {
            uint64_t a, b;
            if (s == R || !piece(off[s], tms[2 * s], R, a, b)) continue;
            got[s] = {a, b};
            op(s, 0, pack_r + s * stride_r, (b - a) * d * 8);
        }
        if (exchange()) return -1;
        for (uint32_t s = 0; s < W; s++)
            if (got[s].second > got[s].first)
                CK(zkgpu_h1h2_shard_place(h1, ldn, h2, ldn, pack_r + s * stride_r, got[s].second - got[s].first,
                                          got[s].first, got[s].second - got[s].first, r0(), d));
        return 0;
    }

    // calculateH1H2 (starks.cpp:104-127) of every plookup: over the ranks
    // (h1h2_sharded), then the h1 / h2 halos; one rank: the whole-column form
    int h1h2_all() override
    {
        if (W > 1) {
            Stores hs;
            for (uint32_t k = 0; k < info.n_pu; k++) {
                if (h1h2_sharded(k)) return -1;
                const uint32_t *q = &pu[5 * k];
                for (uint32_t c = 0; c < q[4]; c++) {
                    hs.cols[SEC_CM2_N].push_back(q[2] + c);
                    hs.cols[SEC_CM2_N].push_back(q[3] + c);
                }
            }
            return refresh_halos(hs.cols);
        }
        for (uint32_t k = 0; k < info.n_pu; k++) {
            const uint32_t *q = &pu[5 * k];
            const uint32_t d = q[4];
            uint64_t *fw = puw, *tw = puw + 3 * N, *h1w = puw + 6 * N, *h2w = puw + 9 * N;
            std::vector<uint32_t> ft;
            for (uint32_t part = 0; part < 2; part++)
                for (uint32_t c = 0; c < d; c++) ft.push_back(q[part] + c);
            std::vector<uint32_t> dst;  // f columns 0..d-1 of fw, t columns of tw (= fw + 3N)
            for (uint32_t part = 0; part < 2; part++)
                for (uint32_t c = 0; c < d; c++) dst.push_back(3 * part + c);
            CK(zkgpu_copy_rows_dev(fw, N, r0(), dst.data(), S.sec[SEC_TMP_N], ldn, 0, 0, ft.data(), 2 * d, nb));
            uint64_t miss = 0;
            const int rc = zkgpu_h1h2_dev(h1w, N, h2w, N, fw, N, tw, N, N, d, &miss);
            if (rc) {
                if (miss != ~0ULL)
                    return fail("Polinomial::calculateH1H2() Number not included: w=%llu plookup_number=%u",
                                (unsigned long long)miss, k);
                return fail("calculateH1H2: %s", zkgpu_last_error());
            }
            CK(zkgpu_copy_rows_dev(S.sec[SEC_CM2_N] + (uint64_t)q[2] * ldn, ldn, 0, nullptr, h1w, N, r0(), info.n_bits,
                                   nullptr, d, ldn));
            CK(zkgpu_copy_rows_dev(S.sec[SEC_CM2_N] + (uint64_t)q[3] * ldn, ldn, 0, nullptr, h2w, N, r0(), info.n_bits,
                                   nullptr, d, ldn));
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
        const int rc = abort_comm(prove_sharded(out));
        const int rc2 = take_cm1_async(true);  // a queued trace becomes cm1_n (set_cm1_async)
        return rc ? rc : rc2;
    }

    int prove_sharded(uint64_t *out)
    {
        timers.clear();
        pend_t.clear();
        pend_x.clear();
        n_marks = 0;
        n_exch = sent_bytes = max_sent = 0;
        auto tall = clk::now();
        Transcript tr;
        tr.put(verkey, 4);
        tr.put(publics.data(), publics.size());
        uint64_t ch[24] = {0};
        uint64_t roots[4][4];
        std::vector<uint64_t> evals(3 * info.n_ev);
        // STAGE 1 (starks.cpp:49-63)
        if (commit_n(trees[0], SEC_CM1_N, SEC_CM1_2NS, info.n_cm1, roots[0], "STARK_STEP_1_LDE",
                     "STARK_STEP_1_EXCHANGE", "STARK_STEP_1_MERKLETREE"))
            return -1;
        tr.put(roots[0], 4);
        // STAGE 2 (:65-144), n domain on the rank's rows
        tr.get_field(ch + 0);
        tr.get_field(ch + 3);
        tstart();
        if (run_n(step2, st2, ch)) return -1;
        if (tstop("STARK_STEP_2_CALCULATE_EXPS")) return -1;
        if (info.n_pu) {
            tstart();
            if (h1h2_all()) return -1;
            if (tstop("STARK_STEP_2_CALCULATEH1H2")) return -1;
        }
        if (commit_n(trees[1], SEC_CM2_N, SEC_CM2_2NS, info.n_cm2, roots[1], "STARK_STEP_2_LDE",
                     "STARK_STEP_2_EXCHANGE", "STARK_STEP_2_MERKLETREE"))
            return -1;
        tr.put(roots[1], 4);
        // STAGE 3 (:146-224)
        tr.get_field(ch + 6);
        tr.get_field(ch + 9);
        tstart();
        if (run_n(step3prev, st3p, ch)) return -1;
        if (tstop("STARK_STEP_3_CALCULATE_EXPS")) return -1;
        tstart();
        if (z_all()) return -1;
        if (tstop("STARK_STEP_3_CALCULATE_Z")) return -1;
        if (!step3.instr.empty()) {
            tstart();
            if (run_n(step3, st3, ch)) return -1;
            if (tstop("STARK_STEP_3_CALCULATE_EXPS_2")) return -1;
        }
        if (commit_n(trees[2], SEC_CM3_N, SEC_CM3_2NS, info.n_cm3, roots[2], "STARK_STEP_3_LDE",
                     "STARK_STEP_3_EXCHANGE", "STARK_STEP_3_MERKLETREE"))
            return -1;
        tr.put(roots[2], 4);
        // STAGE 4 (:226-296): the quotient on the rank's rows
        tr.get_field(ch + 12);
        tstart();
        if (run_block(step42ns, ch, evals.data(), 0, nullptr, nullptr)) return -1;
        if (tstop("STARK_STEP_4_CALCULATE_EXPS_2NS")) return -1;
        tstart();
        if (quotient_sharded()) return -1;
        if (tstop("STARK_STEP_4_CALCULATE_EXPS_2NS_INTT_NTT")) return -1;
        tstart();
        if (merkelize(trees[3], cm4 + (uint64_t)R * B, NE, info.n_cm4, roots[3])) return -1;
        if (tstop("STARK_STEP_4_MERKLETREE")) return -1;
        tr.put(roots[3], 4);
        // STAGE 5 (:298-392)
        tstart();
        uint64_t *xi = ch + 21;
        tr.get_field(xi);
        if (lagrange_xi(xi, r0(), nb)) return -1;  // the rank's rows only
        if (tstop("STARK_STEP_5_LEv_LpEv")) return -1;
        tstart();
        {
            std::vector<uint64_t> part(3 * info.n_ev), all;
            if (evmap_rows(r0(), nb, part.data()) || allgather(part.data(), part.size(), all)) return -1;
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
        CK(zkgpu_xdivxsub_rows_dev(xdiv, xdivw, xi, info.n_bits, info.n_bits_ext, (uint64_t)R * B, B));
        if (tstop("STARK_STEP_5_XDIVXSUB")) return -1;
        tstart();
        const uint64_t xo = 3ULL * R * B;  // xdiv rows are interleaved F_p^3
        if (run_block(step52ns, ch, evals.data(), info.n_ev, xdiv + xo, xdivw + xo)) return -1;
        if (!fri_first_sharded()) {  // else f stays in row blocks (fri_transpose_layer)
            if (gather_rows(S.sec[SEC_F_2NS], gath)) return -1;
            CK(zkgpu_cols3_to_interleaved_dev(fri_pol[0], gath, NE, NE));
        }
        if (tstop("STARK_STEP_5_CALCULATE_EXPS")) return -1;
        const int rc = fri_and_queries(tr, &roots[0][0], evals, out, tall);
        // a count, not a time: the largest exchange this rank posted (every
        // exchange is at most one send and one receive per peer, 2 (W - 1))
        // and the communicator's world and this proof's exchange volume
        if (W > 1) {
            timers.emplace_back("COUNT_COMM_MAX_OPS", (double)max_ops);
            timers.emplace_back("COUNT_COMM_EXCHANGE_MS", xchg_ms);  // device time inside the exchanges
            timers.emplace_back("COUNT_COMM_LARGEST_EXCHANGE_MS", xchg_max_ms);  // of the largest one (bytes sent)
            timers.emplace_back("COUNT_COMM_WORLD", (double)comm.world);
            timers.emplace_back("COUNT_COMM_EXCHANGES", (double)n_exch);
            timers.emplace_back("COUNT_COMM_BYTES_SENT", (double)sent_bytes);
            timers.emplace_back("COUNT_COMM_MAX_BYTES_SENT", (double)max_sent);
        }
        return rc;
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
