// zkgpu_goldilocks.hpp -- C++ host adapter: the reference's Goldilocks-library
// class surface (NTT_Goldilocks, PoseidonGoldilocks, MerklehashGoldilocks)
// implemented on top of the libzkgpu C-ABI (include/zkgpu.h).
//
// A zkevm-prover build swaps `#include "ntt_goldilocks.hpp"` /
// `"poseidon_goldilocks.hpp"` / `"merklehash_goldilocks.hpp"` (the absent
// src/goldilocks submodule, .gitmodules:1-3) for this header; the call sites in
// src/starkpil (starks.cpp:53,134,215,262,285,326-327; merkleTreeGL.cpp:40-42;
// transcript.cpp:23,46; friProve.cpp:100-102) compile unchanged because the
// names, argument order and meaning are the reference's.  Element is any
// 8-byte trivially-copyable type holding the u64 (Goldilocks::Element is
// `struct { uint64_t fe; }`).
//
// Error behaviour mirrors the reference: a failing call logs and ends the
// process (zklog.error + exitProcess(), exit_process.cpp:7); install a
// different handler with zkgpu::set_error_handler.
#pragma once
#include <vector>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string.h>

#include <type_traits>

#include "../../include/zkgpu.h"

namespace zkgpu {

using ErrorHandler = void (*)(const char *where, int code, const char *msg);

inline void default_error_handler(const char *where, int code, const char *msg)
{
    fprintf(stderr, "zkgpu error in %s (%d): %s\n", where, code, msg);
    exit(-1);  // exitProcess() in the reference
}

inline ErrorHandler &error_handler()
{
    static ErrorHandler h = default_error_handler;
    return h;
}
inline void set_error_handler(ErrorHandler h) { error_handler() = h; }

inline void check(int rc, const char *where)
{
    if (rc != ZKGPU_OK) error_handler()(where, rc, zkgpu_last_error());
}

inline void ensure_init(int device = -1)
{
    static bool done = false;
    if (!done) {
        check(zkgpu_init(device), "zkgpu_init");
        done = true;
    }
}

template <typename E>
inline uint64_t *u64p(E *p)
{
    static_assert(sizeof(E) == 8 && std::is_trivially_copyable<E>::value, "Element must be one u64");
    return reinterpret_cast<uint64_t *>(p);
}
template <typename E>
inline const uint64_t *u64p(const E *p)
{
    static_assert(sizeof(E) == 8 && std::is_trivially_copyable<E>::value, "Element must be one u64");
    return reinterpret_cast<const uint64_t *>(p);
}

// NTT_Goldilocks(maxDomainSize, nThreads, extension) -- starks.hpp:81-82.
// nThreads/extension/buffer/nphase/nblock are CPU tuning knobs of the
// reference; the GPU path ignores them (same results).
class NTT_Goldilocks
{
public:
    explicit NTT_Goldilocks(uint64_t maxDomainSize, uint32_t nThreads = 0, int extension = 1)
        : maxDomainSize_(maxDomainSize)
    {
        (void)nThreads;
        (void)extension;
        ensure_init();
    }

    template <typename E>
    void NTT(E *dst, E *src, uint64_t size, uint64_t ncols = 1, E *buffer = nullptr, uint64_t nphase = 3,
             uint64_t nblock = 1)
    {
        (void)buffer, (void)nphase, (void)nblock;
        check(zkgpu_gl_ntt(u64p(dst), u64p(src), size, ncols, 0), "NTT_Goldilocks::NTT");
    }

    template <typename E>
    void INTT(E *dst, E *src, uint64_t size, uint64_t ncols = 1, E *buffer = nullptr, uint64_t nphase = 3,
              uint64_t nblock = 1)
    {
        (void)buffer, (void)nphase, (void)nblock;
        check(zkgpu_gl_ntt(u64p(dst), u64p(src), size, ncols, 1), "NTT_Goldilocks::INTT");
    }

    template <typename E>
    void extendPol(E *output, E *input, uint64_t N_Extended, uint64_t N, uint64_t ncols, E *buffer = nullptr,
                   uint64_t nphase = 3, uint64_t nblock = 1)
    {
        (void)buffer, (void)nphase, (void)nblock;
        check(zkgpu_gl_extend_pol(u64p(output), u64p(input), N_Extended, N, ncols), "NTT_Goldilocks::extendPol");
    }

    uint64_t maxDomainSize() const { return maxDomainSize_; }

private:
    uint64_t maxDomainSize_;
};

// PoseidonGoldilocks static API -- transcript.cpp:23,46, merkleTreeGL.cpp:40-42
struct PoseidonGoldilocks {
    template <typename E>
    static void hash_full_result(E *out, const E *in)
    {
        ensure_init();
        check(zkgpu_gl_poseidon_full(u64p(out), u64p(in)), "PoseidonGoldilocks::hash_full_result");
    }
    template <typename E>
    static void hash(E *out, const E *in)
    {
        ensure_init();
        check(zkgpu_gl_poseidon_hash(u64p(out), u64p(in)), "PoseidonGoldilocks::hash");
    }
    template <typename E>
    static void linear_hash(E *out, E *in, uint64_t size)
    {
        ensure_init();
        check(zkgpu_gl_linear_hash(u64p(out), u64p(in), size), "PoseidonGoldilocks::linear_hash");
    }
    template <typename E>
    static void merkletree(E *tree, E *input, uint64_t num_cols, uint64_t num_rows)
    {
        ensure_init();
        check(zkgpu_gl_merkletree(u64p(tree), u64p(input), num_cols, num_rows), "PoseidonGoldilocks::merkletree");
    }
    // the reference selects these by __AVX512__ (merkleTreeGL.cpp:39-43)
    template <typename E>
    static void merkletree_avx(E *tree, E *input, uint64_t num_cols, uint64_t num_rows)
    {
        merkletree(tree, input, num_cols, num_rows);
    }
    template <typename E>
    static void merkletree_avx512(E *tree, E *input, uint64_t num_cols, uint64_t num_rows)
    {
        merkletree(tree, input, num_cols, num_rows);
    }
};

// MerklehashGoldilocks -- stark_info.hpp:332, build_const_tree.cpp:566-569
struct MerklehashGoldilocks {
    static uint64_t getTreeNumElements(uint64_t numRows) { return zkgpu_gl_merkle_num_elements(numRows); }
    template <typename E>
    static void root(E *out, E *tree, uint64_t numElementsTree)
    {
        for (int i = 0; i < 4; i++) out[i] = tree[numElementsTree - 4 + i];
    }
};

// MerkleTreeGL -- merkleTreeGL.hpp:8-80 / merkleTreeGL.cpp:5-48.  Same members,
// constructors and host-memory semantics (source row-major height x width,
// nodes in the reference layout), so Starks (starks.hpp:186-190) and
// FRIProve (friProve.cpp) use it unchanged; merkelize() runs on the GPU.
template <typename E>
class MerkleTreeGLT
{
public:
    uint64_t height = 0;
    uint64_t width = 0;
    E *source = nullptr;
    E *nodes = nullptr;
    bool isSourceAllocated = false;
    bool isNodesAllocated = false;

    MerkleTreeGLT() {}
    // constant-tree file image: [width, height, source..., nodes...]
    explicit MerkleTreeGLT(E *tree)
    {
        width = u64p(tree)[0];
        height = u64p(tree)[1];
        source = &tree[2];
        nodes = &tree[2 + height * width];
    }
    MerkleTreeGLT(uint64_t _height, uint64_t _width, E *_source) : height(_height), width(_width), source(_source)
    {
        if (source == nullptr) {
            source = (E *)calloc(height * width, sizeof(E));
            isSourceAllocated = true;
        }
        nodes = (E *)calloc(getTreeNumElements(), sizeof(E));
        isNodesAllocated = true;
    }
    ~MerkleTreeGLT()
    {
        if (isSourceAllocated) free(source);
        if (isNodesAllocated) free(nodes);
    }
    MerkleTreeGLT(const MerkleTreeGLT &) = delete;
    MerkleTreeGLT &operator=(const MerkleTreeGLT &) = delete;

    void copySource(E *_source) { memcpy(source, _source, height * width * sizeof(E)); }
    void merkelize() { PoseidonGoldilocks::merkletree(nodes, source, width, height); }
    uint64_t getTreeNumElements() { return height * 4 + (height - 1) * 4; }
    void getRoot(E *root) { memcpy(root, &nodes[getTreeNumElements() - 4], 4 * sizeof(E)); }
    // values of row idx followed by one sibling digest per level (leaves up)
    void getGroupProof(E *proof, uint64_t idx)
    {
        memcpy(proof, &source[idx * width], width * sizeof(E));
        E *p = proof + width;
        uint64_t offset = 0, n = height * 4;  // elements on this level (genMerkleProof)
        while (n > 4) {
            memcpy(p, &nodes[offset + (idx ^ 1) * 4], 4 * sizeof(E));
            p += 4;
            const uint64_t next = ((n - 1) / 8 + 1) * 4;
            offset += next * 2;
            n = next;
            idx >>= 1;
        }
    }
    uint64_t MerkleProofSize()
    {
        uint64_t s = 0;
        for (uint64_t n = 1; n < height; n <<= 1) s++;  // ceil(log2(height))
        return s;
    }
};

// bctree (tools/starkpil/bctree/build_const_tree.cpp:536-603, GL hash):
// interpolate + merkletree in one GPU call; returns the whole const-tree file
// image [nPols, nExt, LDE row-major, nodes] that MerkleTreeGLT(E *tree) and
// Starks (starks.hpp:193-223) load.  The verkey constRoot is image[size-4..].
template <typename E>
inline std::vector<E> buildConstTree(const E *constPols, uint64_t nPols, uint32_t nBits, uint32_t nBitsExt)
{
    ensure_init();
    std::vector<E> image(zkgpu_const_tree_num_elements(nPols, nBitsExt));
    check(zkgpu_build_const_tree(u64p(image.data()), u64p(constPols), nPols, nBits, nBitsExt), "buildConstTree");
    return image;
}

// Executor hand-off (prover.cpp:94-116, commit_pols.hpp:18): stream the
// committed-pols buffer the executor filled (row-major, stride = width) into a
// device column-major section without an intermediate host transpose.
template <typename E>
inline void loadCommittedPols(uint64_t *devCols, uint64_t ld, const E *rows, uint64_t nRows, uint64_t width,
                              bool pinSource = true)
{
    ensure_init();
    check(zkgpu_load_rows_dev(devCols, ld, u64p(rows), nRows, width, 0, pinSource ? 1 : 0), "loadCommittedPols");
}

}  // namespace zkgpu
