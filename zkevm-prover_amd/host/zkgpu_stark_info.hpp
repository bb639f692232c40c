// zkgpu_stark_info.hpp -- the reference's StarkInfo (stark_info.hpp:269-336),
// loaded from the same <circuit>.starkinfo.json (StarkInfo::load,
// stark_info.cpp:21-454), and its translation into the instance description
// of the GPU prover (include/zkgpu_stark.h).
//
//   StarkInfo::load   every key stark_info.cpp:21-454 reads, same defaults
//                     (absent "prime" / "p" / "id" = false / 0 / 0, null
//                     entries of exps_n / q_2ns / cm4_n / cm4_2ns / tmpExp_n
//                     = 0), same errors (unknown section / op / type)
//   ProverInfo        the memory-map widths (mapSectionsN), evMap as
//                     (section_2ns, col, dim, prime) through cm_2ns / qs /
//                     varPolMap (starks.cpp:556-611), the plookup and grand-
//                     product contexts through exp2pol / cm_n in the order
//                     transposeH1H2Columns / transposeZColumns take them
//                     (starks.cpp:406-520), and the step code
//                     (step2prev / step3prev / step3 / step42ns / step52ns
//                     "first") as ZXP programs
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/zkgpu_stark.h"
#include "zkgpu_json.hpp"

namespace zkgpu {

// eSection (stark_info.hpp:42-55)
enum ESection {
    S_CM1_N = 0,
    S_CM1_2NS = 1,
    S_CM2_N = 2,
    S_CM2_2NS = 3,
    S_CM3_N = 4,
    S_CM3_2NS = 5,
    S_CM4_N = 6,
    S_CM4_2NS = 7,
    S_TMPEXP_N = 8,
    S_Q_2NS = 9,
    S_F_2NS = 10,
    S_MAX = 11
};
ESection string2section(const std::string &s);
extern const char *const SECTION_NAMES[S_MAX];

struct StepTypeJ {
    std::string type;  // tmp exp eval challenge tree1..4 number x Z public xDivXSubXi xDivXSubWXi cm const q Zi tmpExp f
    uint64_t id = 0;
    bool prime = false;
    uint64_t p = 0;
    std::string value;
};
struct StepOperationJ {
    std::string op;  // add sub mul copy
    StepTypeJ dest;
    std::vector<StepTypeJ> src;
};
struct StepJ {
    std::vector<StepOperationJ> first;
    uint64_t tmpUsed = 0;
};
struct VarPolMapJ {
    ESection section;
    uint64_t dim, sectionPos;
};
struct PeCtxJ {
    uint64_t tExpId, fExpId, zId, c1Id, numId, denId, c2Id;
};
struct PuCtxJ {
    uint64_t tExpId, fExpId, h1Id, h2Id, zId, c1Id, numId, denId, c2Id;
};
struct CiCtxJ {
    uint64_t zId, numId, denId, c1Id, c2Id;
};
struct EvMapJ {
    enum Type { cm = 0, _const = 1, q = 2 } type;
    uint64_t id;
    bool prime;
};

struct StarkInfo {
    uint64_t nBits = 0, nBitsExt = 0, nQueries = 0;
    std::string verificationHashType;
    std::vector<uint64_t> stepsNBits;  // starkStruct.steps[].nBits
    uint64_t mapTotalN = 0, nConstants = 0, nPublics = 0, nCm1 = 0, nCm2 = 0, nCm3 = 0, nCm4 = 0, friExpId = 0,
             nExps = 0, qDim = 0, qDeg = 0;
    uint64_t mapDeg[S_MAX] = {}, mapOffsets[S_MAX] = {}, mapSectionsN[S_MAX] = {}, mapSectionsN1[S_MAX] = {},
             mapSectionsN3[S_MAX] = {};
    std::vector<uint64_t> mapSections[S_MAX];
    std::vector<VarPolMapJ> varPolMap;
    std::vector<uint64_t> qs, cm_n, cm_2ns;
    std::vector<PeCtxJ> peCtx;
    std::vector<PuCtxJ> puCtx;
    std::vector<CiCtxJ> ciCtx;
    std::vector<EvMapJ> evMap;
    StepJ step2prev, step3prev, step3, step42ns, step52ns;
    std::vector<uint64_t> exps_n, q_2nsVector, cm4_nVector, cm4_2nsVector, tmpExp_n;
    std::map<std::string, uint64_t> exp2pol;

    void load(const json::Value &j);  // stark_info.cpp:21-454
    static StarkInfo from_file(const std::string &path);
};

// The GPU prover's instance description derived from a StarkInfo; owns every
// array the zkgpu_stark_info points into.
struct ZxpProgram {
    std::vector<zxp_instr> instr;
    std::vector<zxp_operand> opnd;
    uint32_t n_tmp1 = 0, n_tmp3 = 0;
    zkgpu_zxp_prog view() const;
};

class ProverInfo
{
public:
    explicit ProverInfo(const StarkInfo &si);
    const zkgpu_stark_info &info() const { return info_; }
    const ZxpProgram &program(const std::string &name) const;  // step2prev step3prev step3 step42ns step52ns
    json::Value to_json() const;                               // the derived description (tests, --info)

private:
    zkgpu_stark_info info_;
    std::vector<uint32_t> ev_, zctx_, pu_;
    std::map<std::string, ZxpProgram> progs_;
};

// a step's "first" code as a ZXP program (throws std::runtime_error on
// operands the GPU programs do not take: tree1..4, Z, tmpExp)
ZxpProgram step_to_zxp(const StarkInfo &si, const StepJ &step, bool ext, const char *name);

}  // namespace zkgpu
