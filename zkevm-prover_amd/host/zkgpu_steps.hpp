// zkgpu_steps.hpp -- a Steps (src/starkpil/steps.hpp:21-58) whose bytecode
// evaluators run on the MI355X.
//
// Starks::genProof calls the generated expression code through the virtual
// Steps interface: step2prev_parser_first_avx at starks.cpp:73,
// step3prev_parser_first_avx at :155, step3_parser_first_avx at :193,
// step42ns_parser_first_avx at :241 and step52ns_parser_first_avx at :371
// (the avx512 variants at :79,161,199,247,377).  ZkevmSteps implements them
// as AVX2 interpreters of its op*/args* bytecode (zkevm.chelpers.*.parser.cpp).
// StepsGPU keeps the bytecode and, for each call, converts it once
// (zkgpu_parser_convert, milliseconds), stages the sections of the memory map the
// program touches to HBM, runs it as a compiled gfx950 kernel and writes the
// columns it stores back into StepsParams.pols / q_2ns / f_2ns
// (zkgpu_steps_parser_eval, include/zkgpu_parser.h).  Same results as the
// AVX2 interpreter (tests/test_parser.py, tests/test_gpu_parser.py).
//
// In a zkevm-prover build:
//     zkgpu::BytecodeProgram progs[5] = {{op2prev, NOPS2prev, args2prev, NARGS2prev}, ...};
//     zkgpu::StepsGPU<Steps, StepsParams> zkevmSteps(map, nMap, starkInfo.starkStruct.nBits,
//                                                    starkInfo.starkStruct.nBitsExt, starkInfo.nPublics, progs);
//     starkZkevm->genProof(fproof, publics, zkevmVerkey, &zkevmSteps);   // prover.cpp:577
// where `map` lists the StarkInfo sections (mapOffsets / mapSectionsN,
// stark_info.cpp:473-482) as zkgpu_pols_section entries.  Every whole-domain
// entry point of the interface -- _parser_first_avx / _avx512 and the
// scalar _parser_first / _avx_jump variants (steps.hpp:39-56; the jump tables
// of zkevm.chelpers.step3.parser.cpp:978 / step42ns.parser.cpp:1475 evaluate
// the same bytecode) -- runs the program on the GPU; none is the base class's
// silent no-op.  The per-row entry points (step*_first / _i / _last) belong to
// the non-parser code path (definitions.hpp:79-90 selects the parsers for
// zkEVM) and fail loudly.
//
// keep_mirrors(true): sections stay on the device between calls
// (zkgpu_steps_mirror); the caller invalidates a section its own code writes
// (invalidate(section pointer), see include/zkgpu_parser.h for the genProof
// call sites); step2prev, the first program of a proof, drops every mirror.
//
// Errors follow the reference (zklog.error + exitProcess, exit_process.cpp:7)
// through zkgpu::error_handler() of host/zkgpu_goldilocks.hpp.
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/zkgpu_parser.h"
#include "zkgpu_goldilocks.hpp"

namespace zkgpu {

struct BytecodeProgram {
    const uint64_t *ops = nullptr;  // op*[NOPS_]
    uint64_t n_ops = 0;
    const uint64_t *args = nullptr;  // args*[NARGS_]
    uint64_t n_args = 0;
};

// StepsBase: the reference's Steps; Params: its StepsParams (steps.hpp:4-17).
template <class StepsBase, class Params>
class StepsGPU : public StepsBase
{
public:
    StepsGPU(const zkgpu_pols_section *map, uint32_t n_map, uint32_t n_bits, uint32_t n_bits_ext, uint32_t n_publics,
             const BytecodeProgram progs[5])
        : map_(map, map + n_map), n_bits_(n_bits), n_bits_ext_(n_bits_ext), n_publics_(n_publics)
    {
        for (int k = 0; k < 5; k++) progs_[k] = progs[k];
    }

    void step2prev_parser_first_avx(Params &p, uint64_t nrows, uint64_t) override { run(ZKGPU_STEP2PREV, p, nrows); }
    void step2prev_parser_first_avx512(Params &p, uint64_t nrows, uint64_t) override
    {
        run(ZKGPU_STEP2PREV, p, nrows);
    }
    void step3prev_parser_first_avx(Params &p, uint64_t nrows, uint64_t) override { run(ZKGPU_STEP3PREV, p, nrows); }
    void step3prev_parser_first_avx512(Params &p, uint64_t nrows, uint64_t) override
    {
        run(ZKGPU_STEP3PREV, p, nrows);
    }
    void step3_parser_first_avx(Params &p, uint64_t nrows, uint64_t) override { run(ZKGPU_STEP3, p, nrows); }
    void step3_parser_first_avx512(Params &p, uint64_t nrows, uint64_t) override { run(ZKGPU_STEP3, p, nrows); }
    void step42ns_parser_first_avx(Params &p, uint64_t nrows, uint64_t) override { run(ZKGPU_STEP42NS, p, nrows); }
    void step42ns_parser_first_avx512(Params &p, uint64_t nrows, uint64_t) override
    {
        run(ZKGPU_STEP42NS, p, nrows);
    }
    void step52ns_parser_first_avx(Params &p, uint64_t nrows, uint64_t) override { run(ZKGPU_STEP52NS, p, nrows); }
    void step52ns_parser_first_avx512(Params &p, uint64_t nrows, uint64_t) override
    {
        run(ZKGPU_STEP52NS, p, nrows);
    }
    // the scalar and jump-table variants of the same evaluations
    void step3_parser_first(Params &p, uint64_t nrows, uint64_t) override { run(ZKGPU_STEP3, p, nrows); }
    void step3_parser_first_avx_jump(Params &p, uint64_t nrows, uint64_t) override { run(ZKGPU_STEP3, p, nrows); }
    void step42ns_parser_first(Params &p, uint64_t nrows, uint64_t) override { run(ZKGPU_STEP42NS, p, nrows); }
    void step42ns_parser_first_avx_jump(Params &p, uint64_t nrows, uint64_t) override
    {
        run(ZKGPU_STEP42NS, p, nrows);
    }
    void step52ns_parser_first(Params &p, uint64_t nrows, uint64_t) override { run(ZKGPU_STEP52NS, p, nrows); }

    // device mirrors of the sections between calls (include/zkgpu_parser.h)
    void keep_mirrors(bool on) { check(zkgpu_steps_mirror(on ? 1 : 0), "StepsGPU::keep_mirrors"); }
    template <typename E>
    void invalidate(const E *section)
    {
        check(zkgpu_steps_invalidate(section), "StepsGPU::invalidate");
    }

    // per-row entry points of the non-parser path: not offered on the GPU
    void step2prev_first(Params &, uint64_t) override { per_row("step2prev_first"); }
    void step2prev_i(Params &, uint64_t) override { per_row("step2prev_i"); }
    void step2prev_last(Params &, uint64_t) override { per_row("step2prev_last"); }
    void step3prev_first(Params &, uint64_t) override { per_row("step3prev_first"); }
    void step3prev_i(Params &, uint64_t) override { per_row("step3prev_i"); }
    void step3prev_last(Params &, uint64_t) override { per_row("step3prev_last"); }
    void step3_first(Params &, uint64_t) override { per_row("step3_first"); }
    void step3_i(Params &, uint64_t) override { per_row("step3_i"); }
    void step3_last(Params &, uint64_t) override { per_row("step3_last"); }
    void step42ns_first(Params &, uint64_t) override { per_row("step42ns_first"); }
    void step42ns_i(Params &, uint64_t) override { per_row("step42ns_i"); }
    void step42ns_last(Params &, uint64_t) override { per_row("step42ns_last"); }
    void step52ns_first(Params &, uint64_t) override { per_row("step52ns_first"); }
    void step52ns_i(Params &, uint64_t) override { per_row("step52ns_i"); }
    void step52ns_last(Params &, uint64_t) override { per_row("step52ns_last"); }

private:
    std::vector<zkgpu_pols_section> map_;
    uint32_t n_bits_, n_bits_ext_, n_publics_;
    BytecodeProgram progs_[5];

    static void per_row(const char *what)
    {
        error_handler()(what, ZKGPU_ERR_ARG, "StepsGPU evaluates whole domains (the *_parser_first_avx entry points)");
    }

    void run(uint32_t parser, Params &p, uint64_t nrows)
    {
        ensure_init();
        const uint64_t dom = 1ULL << (parser >= ZKGPU_STEP42NS ? n_bits_ext_ : n_bits_);
        if (nrows != dom) error_handler()("StepsGPU", ZKGPU_ERR_ARG, "nrows is not the program's domain");
        const BytecodeProgram &b = progs_[parser];
        const bool ext = parser >= ZKGPU_STEP42NS;
        zkgpu_steps_params sp;
        sp.pols = u64p(p.pols);
        sp.const_pols = u64p((const decltype(p.pols))(ext ? p.pConstPols2ns->address() : p.pConstPols->address()));
        sp.n_const = ext ? p.pConstPols2ns->numPols() : p.pConstPols->numPols();
        sp.challenges = u64p(p.challenges.address());
        sp.evals = u64p(p.evals.address());
        sp.n_evals = (uint32_t)p.evals.degree();
        sp.publics = u64p(p.publicInputs);
        sp.n_publics = n_publics_;
        sp.xdiv = parser == ZKGPU_STEP52NS ? u64p(p.xDivXSubXi.address()) : nullptr;
        sp.xdivw = parser == ZKGPU_STEP52NS ? u64p(p.xDivXSubWXi.address()) : nullptr;
        sp.q_2ns = parser == ZKGPU_STEP42NS ? u64p(p.q_2ns) : nullptr;
        sp.f_2ns = parser == ZKGPU_STEP52NS ? u64p(p.f_2ns) : nullptr;
        check(zkgpu_steps_parser_eval(parser, b.ops, b.n_ops, b.args, b.n_args, map_.data(), (uint32_t)map_.size(),
                                      n_bits_, n_bits_ext_, &sp),
              "StepsGPU::parser");
    }
};

}  // namespace zkgpu
