/*
 * oracle/merkle.c -- TEST INFRASTRUCTURE ONLY (CPU oracle).
 *
 * MerkleTreeGL (src/starkpil/merkleTree/merkleTreeGL.{hpp:9-79,cpp:5-44}) with
 * PoseidonGoldilocks::merkletree semantics (submodule, absent):
 *   nodes[0 .. 4h)          leaf digests, leaf i = linear_hash(row i, ncols)
 *   then each level appended, node = hash(L || R || 0,0,0,0)[0..3],
 *   root = last 4 elements; getTreeNumElements = 4h + 4(h-1) (hpp:58-61).
 * getGroupProof (cpp:12-22) = the row's ncols values followed by the sibling
 * digests bottom-up, sibling index idx^1 at each level (genMerkleProof :24-35).
 * Heights are powers of two in every reference use (starks.hpp:185-189,
 * friProve.cpp:120), which is what this restatement supports.
 */
#include <stdlib.h>
#include <string.h>
#include "gl.h"
#include "oracle.h"

uint64_t oc_merkle_num_elements(uint64_t nrows)
{
    return nrows == 0 ? 0 : 4 * nrows + 4 * (nrows - 1);
}

void oc_merkletree(uint64_t *nodes, const uint64_t *src, uint64_t ncols, uint64_t nrows)
{
    if (nrows == 0) return;
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < nrows; i++) oc_linear_hash(nodes + 4 * i, src + i * ncols, ncols);
    uint64_t off = 0, pending = nrows;
    while (pending > 1) {
        uint64_t next = pending / 2;
        uint64_t *lvl = nodes + off;
        uint64_t *dst = nodes + off + 4 * pending;
#pragma omp parallel for schedule(static)
        for (uint64_t i = 0; i < next; i++) {
            uint64_t in[12] = {0};
            memcpy(in, lvl + 8 * i, 8 * sizeof(uint64_t));
            oc_poseidon_hash(dst + 4 * i, in);
        }
        off += 4 * pending;
        pending = next;
    }
}

void oc_merkle_root(uint64_t root[4], const uint64_t *nodes, uint64_t nrows)
{
    memcpy(root, nodes + oc_merkle_num_elements(nrows) - 4, 4 * sizeof(uint64_t));
}

uint64_t oc_merkle_proof_size(uint64_t nrows)
{
    uint64_t l = 0;
    while ((1ULL << l) < nrows) l++;
    return nrows > 1 ? l : 0;
}

void oc_merkle_group_proof(uint64_t *proof, const uint64_t *nodes, const uint64_t *src,
                           uint64_t ncols, uint64_t nrows, uint64_t idx)
{
    memcpy(proof, src + idx * ncols, ncols * sizeof(uint64_t));
    uint64_t *sib = proof + ncols;
    uint64_t off = 0, pending = nrows;
    while (pending > 1) {
        memcpy(sib, nodes + off + 4 * (idx ^ 1), 4 * sizeof(uint64_t));
        sib += 4;
        off += 4 * pending;
        pending >>= 1;
        idx >>= 1;
    }
}

void oc_merkle_root_from_proof(uint64_t root_out[4], const uint64_t *vals, uint64_t ncols,
                               const uint64_t *siblings, uint64_t nsiblings, uint64_t idx)
{
    uint64_t cur[4];
    oc_linear_hash(cur, vals, ncols);
    for (uint64_t l = 0; l < nsiblings; l++) {
        uint64_t in[12] = {0};
        if (idx & 1) {
            memcpy(in, siblings + 4 * l, 4 * sizeof(uint64_t));
            memcpy(in + 4, cur, 4 * sizeof(uint64_t));
        } else {
            memcpy(in, cur, 4 * sizeof(uint64_t));
            memcpy(in + 4, siblings + 4 * l, 4 * sizeof(uint64_t));
        }
        oc_poseidon_hash(cur, in);
        idx >>= 1;
    }
    for (int i = 0; i < 4; i++) root_out[i] = gl_canon(cur[i]);
}
