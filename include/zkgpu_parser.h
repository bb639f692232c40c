/*
 * zkgpu_parser.h -- the reference's zkEVM Steps bytecode on the GPU.
 *
 * The reference evaluates its constraint / expression code as bytecode: an
 * opcode array op*[] and an argument array args*[] per program
 * (src/starkpil/zkevm/chelpers/zkevm.chelpers.<step>.parser.hpp), run by
 * ZkevmSteps::<step>_parser_first_avx (…<step>.parser.cpp), called from
 * Starks::genProof at starks.cpp:73 (step2prev), :155 (step3prev), :193
 * (step3), :241 (step42ns) and :371 (step52ns) through the virtual Steps
 * interface (steps.hpp:21-58).  An argument that addresses the memory map is
 * an absolute element offset into StepsParams.pols plus a row stride: the
 * StarkInfo mapOffsets / mapSectionsN of its section (stark_info.cpp:473-482).
 *
 * zkgpu_parser_convert turns one such program into a ZXP program
 * (include/zkgpu_zxp.h) over column-major device sections, which
 * zkgpu_zxp_eval_dev compiles (csrc/zxp_compile.cpp) and runs as a run-time
 * compiled straight-line gfx950 kernel (csrc/zxp_jit.hip).  Every opcode of
 * the five AVX2 case tables is covered (step42ns fused opcodes 84-92, the
 * stage-3 column stores 86-120 including the shifted stores 101-114 / 119,
 * step52ns' accumulator form).
 *
 * zkgpu_steps_parser_eval is the drop-in for one Steps::<step>_parser_first_avx
 * call on the reference's host buffers (row-major memory map): it converts,
 * stages the sections the program touches to the device, runs it, and writes
 * the columns it stores back (host/zkgpu_steps.hpp wraps it as a Steps).
 */
#ifndef ZKGPU_PARSER_H
#define ZKGPU_PARSER_H
#include <stdint.h>

#include "zkgpu_zxp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* parser ids: the five bytecode programs of ZkevmSteps (zkevmSteps.hpp) */
enum {
    ZKGPU_STEP2PREV = 0, /* step2prev_parser_first_avx, n-domain  (starks.cpp:73)  */
    ZKGPU_STEP3PREV = 1, /* step3prev_parser_first_avx, n-domain  (starks.cpp:155) */
    ZKGPU_STEP3 = 2,     /* step3_parser_first_avx,     n-domain  (starks.cpp:193) */
    ZKGPU_STEP42NS = 3,  /* step42ns_parser_first_avx,  2n-domain (starks.cpp:241) */
    ZKGPU_STEP52NS = 4   /* step52ns_parser_first_avx,  2n-domain (starks.cpp:371) */
};

/* one section of the reference's memory map (StarkInfo.mapOffsets.section[s],
 * mapSectionsN.section[s]) and the ZXP section (SEC_*) it becomes */
typedef struct {
    uint32_t section; /* SEC_CM1_N .. SEC_CM4_2NS (include/zkgpu_zxp.h) */
    uint32_t reserved;
    uint64_t offset; /* first element of the section in StepsParams.pols */
    uint64_t width;  /* row stride = number of columns */
} zkgpu_pols_section;

/* Bytecode -> ZXP program.  n_bits / n_bits_ext: the circuit's domains (the
 * shifted accesses' modulus must be 2^n_bits for the n-domain programs and
 * 2^n_bits_ext for step42ns / step52ns).  Constant-pol operands become
 * SEC_CONST_N (n-domain programs) or SEC_CONST_2NS columns, q_2ns / f_2ns
 * SEC_Q_2NS / SEC_F_2NS.  out->instr / out->opnd stay valid until the next
 * call on the calling thread.  Returns 0 or ZKGPU_ERR_ARG (unknown opcode,
 * argument overrun, an address outside every section, a wrong modulus). */
int zkgpu_parser_convert(uint32_t parser, const uint64_t *ops, uint64_t n_ops, const uint64_t *args, uint64_t n_args,
                         const zkgpu_pols_section *secs, uint32_t n_secs, uint32_t n_bits, uint32_t n_bits_ext,
                         zxp_program *out);

/* StepsParams (steps.hpp:4-17), host side, for zkgpu_steps_parser_eval */
typedef struct {
    uint64_t *pols;             /* params.pols: the memory map (row-major sections), host */
    const uint64_t *const_pols; /* pConstPols (n-domain programs) / pConstPols2ns, row-major n_const wide */
    uint64_t n_const;           /* numPols */
    const uint64_t *challenges; /* 8 x 3 */
    const uint64_t *evals;      /* n_evals x 3 */
    uint32_t n_evals;
    uint32_t n_publics;
    const uint64_t *publics; /* publicInputs */
    const uint64_t *xdiv;    /* xDivXSubXi, 2^n_bits_ext x 3 (step52ns) or NULL */
    const uint64_t *xdivw;   /* xDivXSubWXi */
    uint64_t *q_2ns;         /* 2^n_bits_ext x 3 out (step42ns) or NULL */
    uint64_t *f_2ns;         /* 2^n_bits_ext x 3 out (step52ns) or NULL */
} zkgpu_steps_params;

/* One Steps::<step>_parser_first_avx(params, nrows, nrowsBatch) on the GPU:
 * sections of the map the program reads are copied to the device (row-major
 * -> column-major), the program runs over its whole domain, and the sections
 * it writes (and q_2ns / f_2ns) are copied back into the host buffers.
 * Synchronous.  Requires zkgpu_init. */
int zkgpu_steps_parser_eval(uint32_t parser, const uint64_t *ops, uint64_t n_ops, const uint64_t *args,
                            uint64_t n_args, const zkgpu_pols_section *secs, uint32_t n_secs, uint32_t n_bits,
                            uint32_t n_bits_ext, const zkgpu_steps_params *p);

/* Section mirrors across calls (one proof stages each section once).  With
 * mirroring on, the device copy of every section a call touches is kept
 * (keyed by host address, rows and width) and reused by later calls while
 * valid; a program's own stores keep it valid (written on the device, then
 * copied back).  Host code that writes a section between calls -- in
 * Starks::genProof calculateH1H2 (cm2_n, starks.cpp:104-127), calculateZ
 * (cm3_n, :165-189), every extendPol (cm*_2ns, :53,134,215) and the quotient
 * split (cm4_2ns, :255-296) -- must invalidate it first.  A ZKGPU_STEP2PREV
 * call starts a proof (starks.cpp:73) and invalidates every mirror itself:
 * the executor rewrites the witness in the same host map before each proof
 * (prover.cpp:94-116) without announcing it.  Off by default; turning it off
 * releases the mirrors. */
int zkgpu_steps_mirror(int enable);
int zkgpu_steps_invalidate(const void *host_section); /* NULL: every mirror */
void zkgpu_steps_release_mirrors(void);
uint64_t zkgpu_steps_mirror_bytes(void); /* device bytes the mirrors hold */

#ifdef __cplusplus
}
#endif
#endif /* ZKGPU_PARSER_H */
