#!/usr/bin/env python3
"""Derive the sparse partial-round form of Poseidon-GL and emit it as a header.

The reference evaluates the permutation in its textbook form
(`poseidon_g_executor.cpp:201-231`): every one of the 22 partial rounds adds a
12-lane constant, applies x^7 to lane 0 and multiplies by the 12x12 MDS.  The
same permutation can be rewritten exactly (Poseidon paper, appendix B:
"optimised partial rounds") so that

    s += PRE                  (full 12-lane constant, once)
    s[1..11] = D0 * s[1..11]  (dense 11x11 "initial matrix", once)
    for k in 0..21:
        s0 = s0^7 ; s0 += POST[k]             (POST[21] = 0)
        s0' = 25*s0 + <W[k], s[1..11]> ; s[j] += V[k][j] * s0   (sparse S_k)

Derivation (all arithmetic mod p):
  * constants: walking backwards, the lanes-1..11 part of a round constant
    commutes with the lane-0 S-box, and a vector added after round k-1's MDS
    equals M^-1 times it added before that MDS; lane 0 of what crosses an
    S-box stays behind as POST.  Only round 0 keeps a full vector (PRE).
  * matrices: any N with block form [[n00, w^T], [v, N^]] factors as
    S * D with D = diag(1, N^) applied first and
    S = [[n00, (N^-T w)^T], [v, I]].  D touches lanes 1..11 only, so it
    commutes with the lane-0 S-box and constant and folds into the previous
    round's matrix; after 22 steps the leftover D is the initial matrix.
    Row 0 is never changed, so n00 stays MDS[0][0] = 25 (small).

The input is the product's committed round-constant header (data from the
reference's table); the result is checked here against the textbook form on
random states before anything is written.  Output:
  zkevm-prover_amd/csrc/poseidon_gl_sparse.h

Usage: python tools/gen_poseidon_sparse.py
"""
import os
import random
import re

P = 0xFFFFFFFF00000001
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MCIRC = [17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20]
MDIAG = [8] + [0] * 11
RF_HALF, RP = 4, 22


def load_rc():
    text = open(os.path.join(ROOT, "zkevm-prover_amd/csrc/poseidon_gl_constants.h")).read()
    vals = [int(t, 16) for t in re.findall(r"0x([0-9a-f]{16})ULL", text)]
    assert len(vals) == 360
    return vals


def mds():
    return [[(MCIRC[(y - x) % 12] + (MDIAG[x] if x == y else 0)) for y in range(12)] for x in range(12)]


def matmul(a, b):
    n, m, k = len(a), len(b[0]), len(b)
    return [[sum(a[i][t] * b[t][j] for t in range(k)) % P for j in range(m)] for i in range(n)]


def matvec(a, v):
    return [sum(a[i][t] * v[t] for t in range(len(v))) % P for i in range(len(a))]


def transpose(a):
    return [list(r) for r in zip(*a)]


def inverse(a):
    n = len(a)
    m = [list(r) + [1 if i == j else 0 for j in range(n)] for i, r in enumerate(a)]
    for c in range(n):
        piv = next(r for r in range(c, n) if m[r][c] % P)
        m[c], m[piv] = m[piv], m[c]
        inv = pow(m[c][c], P - 2, P)
        m[c] = [x * inv % P for x in m[c]]
        for r in range(n):
            if r != c and m[r][c]:
                f = m[r][c]
                m[r] = [(x - f * y) % P for x, y in zip(m[r], m[c])]
    return [r[n:] for r in m]


def perm_textbook(st, rc):
    M = mds()
    st = list(st)
    for r in range(2 * RF_HALF + RP):
        st = [(s + rc[r * 12 + i]) % P for i, s in enumerate(st)]
        if r < RF_HALF or r >= RF_HALF + RP:
            st = [pow(s, 7, P) for s in st]
        else:
            st[0] = pow(st[0], 7, P)
        st = matvec(M, st)
    return st


def derive(rc):
    M = mds()
    Minv = inverse(M)
    # constants (backwards over the partial rounds)
    carry = [0] * 12
    post = [0] * RP
    pre = None
    for k in range(RP - 1, -1, -1):
        c = rc[(RF_HALF + k) * 12:(RF_HALF + k + 1) * 12]
        post[k] = carry[0]
        full = [(c[i] + (carry[i] if i else 0)) % P for i in range(12)]
        if k > 0:
            carry = matvec(Minv, full)
        else:
            pre = full
    # matrices (backwards)
    W, V = [None] * RP, [None] * RP
    N = M
    for k in range(RP - 1, -1, -1):
        n00 = N[0][0]
        w = N[0][1:]
        v = [N[i][0] for i in range(1, 12)]
        Nh = [row[1:] for row in N[1:]]
        assert n00 == M[0][0]
        what = matvec(transpose(inverse(Nh)), w)
        W[k], V[k] = what, v
        D = [[1] + [0] * 11] + [[0] + Nh[i] for i in range(11)]
        N = matmul(D, M) if k > 0 else None
        if k == 0:
            D0 = Nh
    return pre, post, D0, W, V


def perm_sparse(st, rc, pre, post, D0, W, V):
    M = mds()
    st = list(st)
    for r in range(RF_HALF):
        st = [pow((s + rc[r * 12 + i]) % P, 7, P) for i, s in enumerate(st)]
        st = matvec(M, st)
    st = [(s + pre[i]) % P for i, s in enumerate(st)]
    st = [st[0]] + matvec(D0, st[1:])
    for k in range(RP):
        s0 = (pow(st[0], 7, P) + post[k]) % P
        n0 = (M[0][0] * s0 + sum(W[k][j] * st[1 + j] for j in range(11))) % P
        st = [n0] + [(st[1 + j] + V[k][j] * s0) % P for j in range(11)]
    for r in range(RF_HALF + RP, 2 * RF_HALF + RP):
        st = [pow((s + rc[r * 12 + i]) % P, 7, P) for i, s in enumerate(st)]
        st = matvec(M, st)
    return st


BLOCK = 11  # partial rounds per block of the device evaluator


def limbs6(c):
    """Coefficient c as 6 u32 limbs: 22/21/21-bit limbs of c and of c*2^32 mod p.
    A lazy lane a = a0 + a1*2^32 times c == a0*c + a1*(c*2^32): both products land
    in the same three accumulators of weight 2^0, 2^22, 2^43."""
    c %= P
    c2 = c * (1 << 32) % P
    return [c & 0x3FFFFF, (c >> 22) & 0x1FFFFF, c >> 43, c2 & 0x3FFFFF, (c2 >> 22) & 0x1FFFFF, c2 >> 43]


def limbs3(k):
    k %= P
    return [k & 0x3FFFFF, (k >> 22) & 0x1FFFFF, k >> 43]


def derive_blocks(rc, pre, post, D0, W, V):
    """Dot-product form of the partial rounds used by the device code.

    Device state after the first four full rounds (whose last MDS already added
    PRE): x = lane 0, L = D0 * lanes[1..11] (materialised).  Per block of
    BLOCK rounds k = k0..k0+BLOCK-1 with y_k = x_k^7 (raw S-box output,
    s0_k = y_k + POST[k]):
        x_{k+1} = 25 s0_k + W_k . L(k0) + sum_{k0<=i<k} (W_k . V_i) s0_i
        L(k0+BLOCK) = L(k0) + sum_i V_i s0_i
    Every POST term and, in the last block, the round-26 constants are folded
    into per-dot constant offsets.  Returns (d0_table, block_tables), u32 lists.
    """
    M = mds()
    c26 = rc[(RF_HALF + RP) * 12:(RF_HALF + RP + 1) * 12]
    d0 = []
    for i in range(11):
        d0 += limbs3(0)
        for j in range(11):
            d0 += limbs6(D0[i][j])
    blocks = []
    for b in range(RP // BLOCK):
        k0 = b * BLOCK
        last = b == RP // BLOCK - 1
        t = []
        for tt in range(BLOCK):
            k = k0 + tt
            coef_y = {k: M[0][0]}
            for i in range(k0, k):
                coef_y[i] = sum(W[k][j] * V[i][j] for j in range(11)) % P
            const = sum(cy * post[i] for i, cy in coef_y.items()) % P
            if last and tt == BLOCK - 1:
                const = (const + c26[0]) % P
            t += limbs3(const)
            t += limbs6(coef_y[k])
            for j in range(11):
                t += limbs6(W[k][j])
            for i in range(k0, k):
                t += limbs6(coef_y[i])
        for j in range(11):
            const = sum(V[i][j] * post[i] for i in range(k0, k0 + BLOCK)) % P
            if last:
                const = (const + c26[1 + j]) % P
            t += limbs3(const)
            for i in range(k0, k0 + BLOCK):
                t += limbs6(V[i][j])
        blocks.append(t)
    assert all(len(x) == len(blocks[0]) for x in blocks)
    return d0, blocks


def perm_blocks(st, rc, pre, d0, blocks):
    """Evaluate the permutation exactly as the device code does (tables only)."""
    M = mds()
    st = [(s + rc[i]) % P for i, s in enumerate(st)]
    for r in range(RF_HALF):
        st = [pow(s, 7, P) for s in st]
        st = matvec(M, st)
        nxt = rc[(r + 1) * 12:(r + 2) * 12] if r < RF_HALF - 1 else pre
        st = [(s + c) % P for s, c in zip(st, nxt)]

    def coef(l6):
        return (l6[0] + (l6[1] << 22) + (l6[2] << 43)) % P

    def const(l3):
        return (l3[0] + (l3[1] << 22) + (l3[2] << 43)) % P

    x = st[0]
    L = []
    for i in range(11):
        base = i * 69
        L.append((const(d0[base:base + 3]) + sum(coef(d0[base + 3 + 6 * j:base + 9 + 6 * j]) * st[1 + j]
                                                   for j in range(11))) % P)
    for tb in blocks:
        pos = 0
        ys = []
        for tt in range(BLOCK):
            y = pow(x, 7, P)
            ys.append(y)
            acc = const(tb[pos:pos + 3]); pos += 3
            acc += coef(tb[pos:pos + 6]) * y; pos += 6
            for j in range(11):
                acc += coef(tb[pos:pos + 6]) * L[j]; pos += 6
            for i in range(tt):
                acc += coef(tb[pos:pos + 6]) * ys[i]; pos += 6
            x = acc % P
        newL = []
        for j in range(11):
            acc = const(tb[pos:pos + 3]) + L[j]; pos += 3
            for i in range(BLOCK):
                acc += coef(tb[pos:pos + 6]) * ys[i]; pos += 6
            newL.append(acc % P)
        L = newL
    st = [x] + L
    for r in range(RF_HALF + RP, 2 * RF_HALF + RP):
        st = [pow(s, 7, P) for s in st]
        st = matvec(M, st)
        if r < 2 * RF_HALF + RP - 1:
            st = [(s + c) % P for s, c in zip(st, rc[(r + 1) * 12:(r + 2) * 12])]
    return st


def emit(path, pre, post, D0, W, V, d0tab=None, btabs=None):
    def arr(name, vals, per=4):
        out = [f"static constexpr uint64_t {name}[{len(vals)}] = {{"]
        for i in range(0, len(vals), per):
            out.append("    " + ", ".join(f"0x{v:016x}ULL" for v in vals[i:i + per]) + ",")
        out.append("};")
        return out

    lines = [
        "// GENERATED by tools/gen_poseidon_sparse.py -- do not edit.",
        "// Poseidon-GL partial rounds in sparse form (exactly equal to the textbook",
        "// permutation of poseidon_g_executor.cpp:201-231; see the generator's docstring).",
        "#ifndef ZKGPU_POSEIDON_GL_SPARSE_H",
        "#define ZKGPU_POSEIDON_GL_SPARSE_H",
        "#include <stdint.h>",
        "// full constant added once before the partial rounds",
    ]
    lines += arr("ZKGPU_PSP_PRE", pre)
    lines += ["// lane-0 constant added after the S-box of partial round k"]
    lines += arr("ZKGPU_PSP_POST", post)
    lines += ["// dense 11x11 initial matrix on lanes 1..11, row-major"]
    lines += arr("ZKGPU_PSP_D0", [x for r in D0 for x in r])
    lines += ["// row 0 of S_k (lanes 1..11): s0' = 25*s0 + sum W[k][j] s[1+j]"]
    lines += arr("ZKGPU_PSP_W", [x for r in W for x in r])
    lines += ["// column 0 of S_k: s[1+j] += V[k][j] * s0"]
    lines += arr("ZKGPU_PSP_V", [x for r in V for x in r])
    if d0tab is not None:
        def arr32(name, vals, per=12):
            out = [f"static constexpr uint32_t {name}[{len(vals)}] = {{"]
            for i in range(0, len(vals), per):
                out.append("    " + ", ".join(f"0x{v:06x}u" for v in vals[i:i + per]) + ",")
            out.append("};")
            return out
        lines += ["// device block form (see derive_blocks): limb tables, u32",
                  f"#define ZKGPU_PSB_BLOCK {BLOCK}",
                  f"#define ZKGPU_PSB_NBLOCKS {len(btabs)}",
                  f"#define ZKGPU_PSB_BLOCK_WORDS {len(btabs[0])}"]
        lines += arr32("ZKGPU_PSB_D0", d0tab)
        lines += arr32("ZKGPU_PSB_BLOCKS", [w for t in btabs for w in t])
    lines += ["#endif  // ZKGPU_POSEIDON_GL_SPARSE_H", ""]
    with open(path, "w") as f:
        f.write("\n".join(lines))


def main():
    rc = load_rc()
    pre, post, D0, W, V = derive(rc)
    assert post[RP - 1] == 0
    rnd = random.Random(12)
    for _ in range(64):
        st = [rnd.randrange(P) for _ in range(12)]
        assert perm_sparse(st, rc, pre, post, D0, W, V) == perm_textbook(st, rc)
    d0tab, btabs = derive_blocks(rc, pre, post, D0, W, V)
    for _ in range(16):
        st = [rnd.randrange(P) for _ in range(12)]
        assert perm_blocks(st, rc, pre, d0tab, btabs) == perm_textbook(st, rc)
    emit(os.path.join(ROOT, "zkevm-prover_amd/csrc/poseidon_gl_sparse.h"), pre, post, D0, W, V, d0tab, btabs)
    print("sparse and block forms verified on random states; header written")


if __name__ == "__main__":
    main()
