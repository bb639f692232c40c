"""Bisect a ZXP program GPU vs oracle: evaluate every instruction prefix and
compare the prefix's last destination (test infrastructure)."""
import sys
import os
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zkevm-prover_amd")]
import torch  # noqa
import zkgpu
from zkgpu.synthetic import SyntheticStark, SEC_Q_2NS, COPY, COL3
from oracle.stark_prover import OracleStark


class Pref:
    def __init__(self, ins, opn, n1, n3, dom_ext):
        self.ins, self.opn, self.n_tmp1, self.n_tmp3, self.domain_ext = ins, opn, n1, n3, dom_ext

    def arrays(self):
        return self.ins, self.opn


zkgpu.init(0)
inst = SyntheticStark(n_bits=8, blowup_bits=1, t=4, m=2, n_queries=8)
o = OracleStark(inst)
o.witness()
o.prove()
prog = inst.programs["step42ns"]
ins, opn = prog.arrays()
secs = {k: (zkgpu.to_device(np.ascontiguousarray(a.T)), a.shape[0], a.shape[1]) for k, a in o.S.items()}
NE = o.NE
q = torch.zeros((3, NE), dtype=torch.int64, device="cuda:0")
secs[SEC_Q_2NS] = (q, NE, 3)
qidx = [i for i in range(opn.shape[0]) if opn[i, 0] == COL3 and opn[i, 1] == SEC_Q_2NS][0]
print("instructions", ins.shape[0], "operands", opn.shape[0])
for k in range(1, ins.shape[0] + 1):
    pi = ins[:k].copy()
    dst = pi[-1, 1]
    if opn[dst, 0] != COL3:
        pi = np.vstack([pi, np.array([[COPY, qidx, dst, 0]], np.uint32)])
    pr = Pref(pi, opn, prog.n_tmp1, prog.n_tmp3, 1)
    o.S[10][:] = 0
    o.run(pr, o.challenges, np.zeros(3, np.uint64))
    zkgpu.zxp_eval_dev(pr, secs, inst.n_bits_ext, o.challenges, o.publics, extend_bits=o.eb, x_start=7)
    torch.cuda.synchronize()
    got = zkgpu.from_device(q).T
    ok = np.array_equal(got, o.S[10])
    if not ok:
        bad = np.argwhere(got != o.S[10])
        i0 = bad[0][0]
        print("FIRST MISMATCH at prefix", k, "instr", ins[k - 1].tolist(), "a", opn[ins[k - 1, 2]].tolist(),
              "b", opn[ins[k - 1, 3]].tolist(), "dst", opn[ins[k - 1, 1]].tolist(), "rows bad", len(set(bad[:, 0])),
              "row", i0, "got", got[i0].tolist(), "want", o.S[10][i0].tolist())
        prev = ins[:k - 1]
        break
else:
    print("all prefixes match")
