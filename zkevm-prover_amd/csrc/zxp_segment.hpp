// Segmented expression programs (csrc/zxp_segment.cpp): a compiled ZXP
// program too large for one kernel is cut into consecutive segments, each run
// as its own kernel over every row.  An SSA temporary defined in one segment
// and read in a later one is carried through a scratch column (column-major,
// one u64 per row): the defining segment stores it, later segments read it as
// a column.  Plain host C++.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/zkgpu_zxp.h"

namespace zk {

// pseudo section index of the scratch columns (resolved by the JIT, never
// part of zkgpu_sections)
constexpr uint32_t ZXP_SEC_SCRATCH = 12;

struct ZxpSegment {
    std::vector<zxp_instr> instr;
    std::vector<zxp_operand> opnd;  // the program's operands + scratch COL / COL3 operands
    std::vector<zxp_term> term;     // this segment's DOT terms (sources remapped)
    uint32_t n_tmp1 = 0, n_tmp3 = 0;
    uint32_t carry_in = 0, carry_out = 0;  // scratch words read / written per row
};

// Cuts `cp` into n_seg segments (n_seg >= 2; fewer when the program is short)
// at points where few temporary words are live, balancing an estimate of the
// VALU work.  Returns 0 and the scratch columns needed, or < 0 on a malformed
// program.
int zxp_segment(const zxp_compiled &cp, uint32_t n_seg, std::vector<ZxpSegment> &out, uint32_t &n_scratch);

// VALU-work estimate of one compiled instruction (cut balancing, stats)
uint32_t zxp_instr_cost(const zxp_compiled &cp, uint32_t k);

}  // namespace zk
