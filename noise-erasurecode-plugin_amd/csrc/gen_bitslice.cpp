// gen_bitslice.cpp -- writes the HIP source of the bit-sliced encode kernels
// (bitslice.hpp) for the (k, n) codes given on the command line.
//
//   gen_bitslice [-x|-X] [-g GEOMETRY] [-p PREFETCH] OUT.hip K:N [K:N ...]   (-x/-X: movement-only diagnostics)
//
// The encode matrix comes from the engine's own gf256.cpp
// (systematic_matrix, the matrix infectious.NewFEC builds, main.go:73/:248),
// so the generated wiring and the table kernels share one definition; the
// generated file also embeds the matrix and rsmi.cpp checks it at start-up.
//
// Kernel shape (per lane): 32 bytes of each shard (two 16-byte columns, one
// from each half of the wave's 2 KiB window, so every load instruction is a
// contiguous 1 KiB per wave) are transposed into 8 bit planes P0..P7 (plane p
// holds bit p of each of the 32 bytes).  For a coefficient c, output plane q
// of c*x is the XOR of the planes P_p with bit q of c*2^p set.  The 16
// XOR combinations of P0..P3 (C1) and of P4..P7 (C2) are built once per
// shard, so each (output plane, shard) costs one 3-way XOR:
// acc = acc ^ C1[s1] ^ C2[s2], with s1/s2 baked into the instruction stream.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gf256.hpp"

namespace {

int kPrefetch = 4;  // shards whose loads are in flight ahead of the one being coded (-p N)
int kRecPrefetch = 0;  // the same for the syndrome reconstruct (-P N; 0: as -p)
// -x: movement-only encode and reconstruct (diagnostic builds): the same
// loads, stores and block shape, but shard j is only XORed into parity row
// j mod m (no transpose, no network; the reconstruct stores row r mod m as
// output r: no syndromes, no solve).  Gives the memory system's rate for the kernel's
// own access pattern; never part of a product build.  -X: the same with
// every shard XORed into one row's registers and that row stored m times
// (few VGPRs, so more waves per SIMD than the real kernel).
bool kMovementOnly = false;
bool kMovementLowReg = false;
// Column geometry of a block's 512 16-byte columns per shard (-g N).
// 0: each wave owns a contiguous 2 KiB window (lane: columns l and 64 + l);
// 1: every load instruction of the block covers a contiguous 4 KiB (lane of
//    wave w: columns 64w + l and 256 + 64w + l), like the split-table kernel.
int kGeometry = 0;
constexpr int kRecMaxK = 64;  // reconstruct: survivor slots are read one per lane of a wave
constexpr int kRecMaxM = 32;  // reconstruct: parity-row masks are 32-bit words (bitslice.hpp BsStripeMask)
// Reconstruct network row guards (-G N, -E / -e): one wave-uniform branch
// per group of N parity rows (a group runs if any of its rows is needed), and
// whether the branch is marked likely-taken (needed rows fall through;
// without the hint hipcc moves most row bodies out of line, two taken
// branches per executed row).  Default groups of 2 with the hint: config 5,
// 20 steps x 3 reps against one unhinted guard per row (profiles/r03z/):
// 16 erasures -1.3%, the 1-16 mix -0.4 to -0.5%, RS(8,14) equal; groups of 4
// are -3% at 16 erasures but +0.5% on the mix.
int kRowGroup = 2;
bool kRowExpect = true;
// Reconstruct column windows per block (-I N): a block runs its prologue
// (descriptor, pattern ids, ballots, split tables) once and then codes N
// consecutive 8 KiB windows of its stripe in turn.
int kRecIters = 1;
// Outputs per solve group of the reconstruct (-R N): each group recomputes
// the syndromes' bit fields once and applies every group row's tables.
int kRecRows = 4;
// Row-subset reconstruct variants (-T a,b,...; -T 0: none): the top parity
// rows each covers, generated for codes with at least kTopMinM parity rows.
std::vector<int> kTops = {4, 8};
int kTopPrefetch = 0;  // prefetch depth of the row-subset variants (-Q N; 0: as the full kernel)
// Row guards in the row-subset variants (-u: on).  Off by default: with a
// wave-uniform branch around each of a few rows the register allocator copies
// the live accumulators in and out at every join (t4: 5,184 v_mov_b64 in the
// ISA, ~3k of its ~10k VALU per wave), which costs more than coding the
// unused top rows.
bool kTopGuard = false;
// Diagnostic builds only (-M): the reconstruct also derives its masks from
// the pattern's id rows (ballots, the pre-r03 prologue), prints any
// disagreement with the host's mask record and codes with the derived ones.
bool kDebugMasks = false;
// Reconstruct loads as buffer loads (default; -Z restores the round-3 zero
// page): every input gets a buffer resource (base in SGPRs, 32-bit lane
// offsets, no address VALU); an absent input's resource has num_records 0, so
// its loads return zeros without touching memory (no zero page, no per-load
// offset selects).  Same-box A/B, 10 steps x 2 (profiles/r04c/): config 5
// reconstruct fresh 1-16 -1.7%, 16 erasures -1.1%, RS(8,14) -2.5%.
bool kBufferLoads = true;
// Reconstruct inputs entered through an opaque asm on their load registers
// (round 3; -Y restores it) so their transpose stayed after the prefetch.
// Without it (default) the vmcnt waits are unchanged and hipcc transposes in
// the load registers instead of copying them out first: 264 fewer VALU in
// the RS(64,16) kernel's ISA, same-box A/B 10 steps x 2 (profiles/r04h/):
// config 5 fresh -0.4..-0.9%, pool -0.4..-0.8%, 16 erasures -0.1%.
bool kInputBarrier = false;
// Solve tail (default; -l: off): outputs past e in the last group of R are
// skipped by a wave-uniform branch per (syndrome, output) instead of coded as
// padding (for e uniform in 1..16, 1.5 of every 10 outputs coded were
// padding); the syndrome's bit fields are extracted once per group for all
// outputs.  With -W, same-box A/B against neither, config 5, 5 steps x 2
// (profiles/r06c/): fresh 1-16 -1.2%, pool of 256 -1.5%, e = 16 -1.0%.
bool kSolveTail = true;
// Solve in bit planes (-S; measured slower, so off: the split-table solve):
// the syndromes stay in planes, and an output gets c * s as the XOR of the
// planes of 2^b * s over the set bits b of c -- 2^b * s is s advanced b times
// by the fixed map x -> 2x (a plane rotation plus 3 XORs, shared by every
// output), the bits of c are wave-uniform scalar branches.  Per (output,
// syndrome) pair and 32 bytes: ~4 x 8 XORs + 21 / R shared, where the split
// tables issue 24 v_perm (slow class) + 16 XOR + the syndrome's bit fields;
// each parity survivor is transposed into planes instead of its row out of
// them, and each output leaves the planes at its store.  Same-box A/B,
// config 5, 5 steps x 2 (profiles/r06b/): e = 16 23.3 vs 22.1 ms, fresh
// 1-16 17.4 vs 16.8, pool of 256 15.4 vs 14.7 -- fewer VALU, but the 512
// wave-uniform branches per output group (s_bitcmp + s_cbranch per bit) cost
// more than the v_perm tables they replace.
bool kPlaneSolve = false;
// Transpose stages 4 and 2 with one 64-bit left shift per pair of words
// (-W): v_lshlrev_b64 issues at the rate of one v_lshlrev_b32 (profiles/
// r02bm/shift64.log), so each stage needs 2 slow shifts instead of 4; the
// bits a 64-bit shift carries across the word boundary land where the select
// mask keeps the other operand.  On by default (-w: off; A/B in kSolveTail's
// note); the bit-sliced encode is at its movement ceiling either way (13.97-
// 14.18 vs 14.06 ms, profiles/r06c/enc.log).
bool kShift64 = true;
constexpr int kTopMinM = 12;

void emit_common(FILE* f) {
    std::fputs("// GENERATED by gen_bitslice.cpp -- do not edit (rebuilt by the Makefile).\n", f);
    std::fprintf(f, "// The reconstruct's solve: in bit planes (1; gen_bitslice -S) or split tables (0).\n"
                    "#define BS_PLANE_SOLVE %d\n"
                    "// Transpose stages 4 and 2 with 64-bit left shifts (gen_bitslice -W).\n"
                    "#define BS_SHIFT64 %d\n", kPlaneSolve && !kMovementOnly ? 1 : 0, kShift64 ? 1 : 0);
    std::fputs(R"(
#include "bitslice.hpp"
#include "gf_device.hpp"
#include "xcd.hpp"

namespace rsmi {
namespace {

typedef unsigned int bs_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const bs_u32x4 BsGlobalCU4;
typedef __attribute__((address_space(1))) bs_u32x4 BsGlobalU4;

__device__ __forceinline__ uint32_t bs_xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Swap the high sub-field of a with the low sub-field of b (an involution).
// Written with the gfx950 issue rates in mind (tools/ubench/valu_rates.hip,
// profiles/r02bm/): v_bitop3, v_lshrrev, v_add and v_xor issue ~1.45x as
// fast as v_bfi, v_perm and every left shift.  The two field selects are
// v_bitop3 (M ? x : y, truth table 0xCA) instead of the v_bfi hipcc picks,
// and the 1-bit left shift is an add.
template <int S, uint32_t M>
__device__ __forceinline__ void bs_swap(uint32_t& a, uint32_t& b) {
#if BS_SWAP_BFI
    const uint32_t na = (a & M) | ((b << S) & ~M);
    const uint32_t nb = ((a >> S) & M) | (b & ~M);
#else
    uint32_t bl;
    if constexpr (S == 1) asm("v_add_u32 %0, %1, %1" : "=v"(bl) : "v"(b));
    else bl = b << S;
    const uint32_t na = __builtin_amdgcn_bitop3_b32(M, a, bl, 0xCA);
    const uint32_t nb = __builtin_amdgcn_bitop3_b32(M, a >> S, b, 0xCA);
#endif
    a = na;
    b = nb;
}

// Two swaps whose b words are consecutive: one 64-bit left shift for both
// (BS_SHIFT64).  The S bits b0 carries into the low end of b1's shifted word
// sit where M selects a1, so they never reach the result.
template <int S, uint32_t M>
__device__ __forceinline__ void bs_swap2(uint32_t& a0, uint32_t& a1, uint32_t& b0, uint32_t& b1) {
    // (inline asm: left to itself hipcc splits the 64-bit shift back into
    // 32-bit shifts and ors)
    uint64_t bb;
    asm("v_lshlrev_b64 %0, %2, %1" : "=v"(bb) : "v"(static_cast<uint64_t>(b1) << 32 | b0), "i"(S));
    const uint32_t na0 = __builtin_amdgcn_bitop3_b32(M, a0, static_cast<uint32_t>(bb), 0xCA);
    const uint32_t na1 = __builtin_amdgcn_bitop3_b32(M, a1, static_cast<uint32_t>(bb >> 32), 0xCA);
    const uint32_t nb0 = __builtin_amdgcn_bitop3_b32(M, a0 >> S, b0, 0xCA);
    const uint32_t nb1 = __builtin_amdgcn_bitop3_b32(M, a1 >> S, b1, 0xCA);
    a0 = na0; a1 = na1; b0 = nb0; b1 = nb1;
}

// 8 words of 4 bytes <-> 8 bit planes: word index and in-byte bit index
// exchange their three bits, one delta-swap stage per bit.  Plane p ends up
// holding bit p of byte (w, b) at bit position 8b + w.
__device__ __forceinline__ void bs_stage4(uint32_t (&w)[8]) {
#if BS_SHIFT64
    bs_swap2<4, 0x0F0F0F0Fu>(w[0], w[1], w[4], w[5]); bs_swap2<4, 0x0F0F0F0Fu>(w[2], w[3], w[6], w[7]);
#else
    bs_swap<4, 0x0F0F0F0Fu>(w[0], w[4]); bs_swap<4, 0x0F0F0F0Fu>(w[1], w[5]);
    bs_swap<4, 0x0F0F0F0Fu>(w[2], w[6]); bs_swap<4, 0x0F0F0F0Fu>(w[3], w[7]);
#endif
}
__device__ __forceinline__ void bs_stage2(uint32_t (&w)[8]) {
#if BS_SHIFT64
    bs_swap2<2, 0x33333333u>(w[0], w[1], w[2], w[3]); bs_swap2<2, 0x33333333u>(w[4], w[5], w[6], w[7]);
#else
    bs_swap<2, 0x33333333u>(w[0], w[2]); bs_swap<2, 0x33333333u>(w[1], w[3]);
    bs_swap<2, 0x33333333u>(w[4], w[6]); bs_swap<2, 0x33333333u>(w[5], w[7]);
#endif
}
__device__ __forceinline__ void bs_stage1(uint32_t (&w)[8]) {
    bs_swap<1, 0x55555555u>(w[0], w[1]); bs_swap<1, 0x55555555u>(w[2], w[3]);
    bs_swap<1, 0x55555555u>(w[4], w[5]); bs_swap<1, 0x55555555u>(w[6], w[7]);
}
// Opaque to the optimiser: without it the compiler folds the last swap
// stage into the plane combinations (and + bitop3 per use instead of one
// bfi per plane), about 50 extra VALU ops per shard.
__device__ __forceinline__ void bs_pin8(uint32_t (&w)[8]) {
    asm volatile("" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]));
}
__device__ __forceinline__ void bs_to_planes(uint32_t (&w)[8]) { bs_stage4(w); bs_stage2(w); bs_stage1(w); bs_pin8(w); }
__device__ __forceinline__ void bs_from_planes(uint32_t (&w)[8]) { bs_stage1(w); bs_stage2(w); bs_stage4(w); }

// x -> 2x (GF(2^8), poly 0x11D) on 8 bit planes: bit q of 2x is bit q - 1
// of x, and bit 7 of x folds back as 0x1D (bits 0, 2, 3, 4).
__device__ __forceinline__ __attribute__((unused)) void bs_mul2(uint32_t (&y)[8]) {
    const uint32_t h = y[7];
    y[7] = y[6]; y[6] = y[5]; y[5] = y[4];
    y[4] = y[3] ^ h; y[3] = y[2] ^ h; y[2] = y[1] ^ h;
    y[1] = y[0]; y[0] = h;
}

// The 16 XOR combinations of 4 planes (c[0] unused).
__device__ __forceinline__ void bs_combos(const uint32_t* p, uint32_t (&c)[16]) {
    c[1] = p[0]; c[2] = p[1]; c[3] = p[0] ^ p[1];
    c[4] = p[2]; c[5] = p[2] ^ p[0]; c[6] = p[2] ^ p[1]; c[7] = p[2] ^ c[3];
    c[8] = p[3];
#pragma unroll
    for (int i = 1; i < 8; ++i) c[8 + i] = p[3] ^ c[i];
}

__device__ __forceinline__ void bs_load(uint32_t (&x)[8], const uint8_t* shard, uint32_t offa, uint32_t offb) {
    const bs_u32x4 u = __builtin_nontemporal_load((BsGlobalCU4*)(shard + offa));
    const bs_u32x4 v = __builtin_nontemporal_load((BsGlobalCU4*)(shard + offb));
    x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w;
    x[4] = v.x; x[5] = v.y; x[6] = v.z; x[7] = v.w;
}

// Buffer-resource form (gen_bitslice -B): base and range in SGPRs, the lane
// offset in one VGPR; num_records 0 makes every load return zeros.  A present
// input's range is the whole 32-bit offset space (num_records 0xFFFFFFFF):
// rsmi.cpp accepts shards of up to 2^28 16-byte columns, so the last column
// ends at 2^32 - 16 -- in range.  (0x7FFFFFFF, round 4, read zeros for every
// column past 2 GiB; tests/test_gpu_parity.py test_bitslice_rec_past_2gib.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bs_rsrc(const uint8_t* base, bool present) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), static_cast<short>(0),
                                             present ? static_cast<int>(0xFFFFFFFFu) : 0, 0x00020000);
}
__device__ __forceinline__ void bs_load_buf(uint32_t (&x)[8], __amdgpu_buffer_rsrc_t r, uint32_t offa, uint32_t offb) {
    const bs_u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r, offa, 0, 2);  // 2: nt
    const bs_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, offb, 0, 2);
    x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w;
    x[4] = v.x; x[5] = v.y; x[6] = v.z; x[7] = v.w;
}

__device__ __forceinline__ void bs_store(uint8_t* shard, uint32_t off, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const bs_u32x4 v = {a, b, c, d};
    __builtin_nontemporal_store(v, (BsGlobalU4*)(shard + off));
}

#define BS_FENCE() asm volatile("" ::: "memory")

)", f);
    std::fprintf(f, "// Column geometry %d (gen_bitslice -g): this lane's two 16-byte columns.\n"
                    "__device__ __forceinline__ void bs_cols(uint32_t blk, uint32_t wave, uint32_t lane, uint32_t& ca, uint32_t& cb) {\n",
                 kGeometry);
    if (kGeometry == 1)
        std::fprintf(f, "    ca = blk * 512u + wave * 64u + lane;\n    cb = ca + 256u;\n}\n\n");
    else
        std::fprintf(f, "    ca = blk * 512u + wave * 128u + lane;\n    cb = ca + 64u;\n}\n\n");
}

// Pins accumulators [o0, o1) (multiples of 8): a shard's XORs complete
// before the next shard's loads and transposes (otherwise the scheduler
// interleaves shards and spills).
void emit_acc_fence(FILE* f, int o0, int o1) {
    for (int o = o0; o < o1; o += 8)
        std::fprintf(f, "        asm volatile(\"\" : \"+v\"(acc[%d]), \"+v\"(acc[%d]), \"+v\"(acc[%d]), \"+v\"(acc[%d]), "
                        "\"+v\"(acc[%d]), \"+v\"(acc[%d]), \"+v\"(acc[%d]), \"+v\"(acc[%d]));\n",
                     o, o + 1, o + 2, o + 3, o + 4, o + 5, o + 6, o + 7);
}

// XOR network of data shard j (its plane combinations c1/c2 built): output
// plane q of parity row t gets c1[s1] ^ c2[s2], the planes of bits 0-3 and
// 4-7 of x whose images under c = E[k+t][j] have bit q set.  assign: the
// accumulators are written, not updated (first shard of the encode).
// row_guard (reconstruct): a wave-uniform mask of the parity rows the
// pattern needs; the other rows' XORs are branched over.
void emit_network(FILE* f, const std::vector<uint8_t>& E, int k, int m, int j, bool assign,
                  const char* row_guard = nullptr, int t0 = 0) {
    for (int t = t0; t < m; ++t) {
        const int G = row_guard ? kRowGroup : 1;
        // A group opens at its first row (or at t0, mid-group, in a row-subset
        // variant whose T0 is not a multiple of G) and closes at its last row;
        // its mask covers exactly the rows from t to that last row.
        if (row_guard && (t == t0 || t % G == 0)) {
            const int rows = std::min(G - t % G, m - t);
            const unsigned gm = (rows >= 32 ? 0xFFFFFFFFu : ((1u << rows) - 1u));
            if (kRowExpect)
                std::fprintf(f, "        if (__builtin_expect(((%s >> %d) & 0x%xu) != 0u, 1)) {\n", row_guard, t, gm);
            else
                std::fprintf(f, "        if ((%s >> %d) & 0x%xu) {\n", row_guard, t, gm);
        }
        const uint8_t c = E[static_cast<size_t>(k + t) * k + j];
        uint8_t col[8];  // col[p] = c * 2^p
        for (int pb = 0; pb < 8; ++pb) col[pb] = rsmi::gmul(c, static_cast<uint8_t>(1u << pb));
        for (int q = 0; q < 8; ++q) {
            int s1 = 0, s2 = 0;
            for (int pb = 0; pb < 4; ++pb) s1 |= ((col[pb] >> q) & 1) << pb;
            for (int pb = 4; pb < 8; ++pb) s2 |= ((col[pb] >> q) & 1) << (pb - 4);
            const int o = (t - t0) * 8 + q;
            if (assign) {
                if (s1 && s2) std::fprintf(f, "        acc[%d] = c1[%d] ^ c2[%d];\n", o, s1, s2);
                else if (s1) std::fprintf(f, "        acc[%d] = c1[%d];\n", o, s1);
                else if (s2) std::fprintf(f, "        acc[%d] = c2[%d];\n", o, s2);
                else std::fprintf(f, "        acc[%d] = 0u;\n", o);
            } else {
                if (s1 && s2) std::fprintf(f, "        acc[%d] = bs_xor3(acc[%d], c1[%d], c2[%d]);\n", o, o, s1, s2);
                else if (s1) std::fprintf(f, "        acc[%d] ^= c1[%d];\n", o, s1);
                else if (s2) std::fprintf(f, "        acc[%d] ^= c2[%d];\n", o, s2);
            }
        }
        if (row_guard && (t % kRowGroup == kRowGroup - 1 || t == m - 1)) std::fprintf(f, "        }\n");
    }
}

void emit_kernel(FILE* f, int k, int n) {
    const int m = n - k;
    const std::vector<uint8_t> E = rsmi::systematic_matrix(k, n);
    const std::string name = "rs_bitslice_k" + std::to_string(k) + "_m" + std::to_string(m);
    const int P = m * 8;  // output planes

    std::fprintf(f, "const uint8_t %s_matrix[%d] = {", name.c_str(), m * k);
    for (int i = 0; i < m * k; ++i)
        std::fprintf(f, "%s%u", i ? "," : "", E[static_cast<size_t>(k) * k + i]);
    std::fprintf(f, "};\n\n");

    std::fprintf(f, "__global__ __launch_bounds__(256) void %s(BitsliceArgs a) {\n", name.c_str());
    std::fprintf(f,
                 "    // A stripe's blocks run on one XCD, in order (xcd.hpp).\n"
                 "    const uint32_t bx = a.xcd ? xcd_block(blockIdx.x, a.xcd * a.blocks_per_stripe, gridDim.x) : blockIdx.x;\n"
                 "    const uint64_t s = bx / a.blocks_per_stripe;\n"
                 "    const uint32_t blk = bx - static_cast<uint32_t>(s) * a.blocks_per_stripe;\n"
                 "    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;\n"
                 "    const uint32_t last = a.ncols16 - 1u;\n"
                 "    uint32_t ca, cb;\n"
                 "    bs_cols(blk, wave, lane, ca, cb);\n"
                 "    if (ca > last) return;  // whole 16-B columns past the shard: nothing to code\n"
                 "    const uint32_t offa = ca * 16u, offb = (cb <= last ? cb : last) * 16u;\n"
                 "    const uint8_t* d = a.data + s * a.data_ss;\n"
                 "    uint8_t* p = a.parity + s * a.parity_ss;\n"
                 "    uint32_t acc[%d];\n"
                 "    uint32_t x[%d][8];\n",
                 P, kPrefetch + 1);
    for (int j = 0; j < kPrefetch && j < k; ++j)
        std::fprintf(f, "    bs_load(x[%d], d + %du * a.pitch, offa, offb);\n", j, j);
    for (int j = 0; j < k; ++j) {
        const int buf = j % (kPrefetch + 1);
        std::fprintf(f, "    // shard %d\n    BS_FENCE();\n", j);
        if (j + kPrefetch < k)
            std::fprintf(f, "    bs_load(x[%d], d + %du * a.pitch, offa, offb);\n", (j + kPrefetch) % (kPrefetch + 1),
                         j + kPrefetch);
        // The shard's words enter the XOR network only here, so its transpose
        // is not hoisted next to the loads (which would wait for the prefetch).
        std::fprintf(f, "    asm volatile(\"\" : \"+v\"(x[%d][0]), \"+v\"(x[%d][1]), \"+v\"(x[%d][2]), \"+v\"(x[%d][3]), "
                        "\"+v\"(x[%d][4]), \"+v\"(x[%d][5]), \"+v\"(x[%d][6]), \"+v\"(x[%d][7]));\n",
                     buf, buf, buf, buf, buf, buf, buf, buf);
        if (kMovementOnly) {
            const int rows = kMovementLowReg ? 1 : m;
            if (j == 0) std::fprintf(f, "    for (int i = 0; i < %d; ++i) acc[i] = 0u;\n", rows * 8);
            for (int q = 0; q < 8; ++q)
                std::fprintf(f, "    acc[%d] ^= x[%d][%d];\n", (j % rows) * 8 + q, buf, q);
            continue;
        }
        std::fprintf(f, "    {\n        bs_to_planes(x[%d]);\n        uint32_t c1[16], c2[16];\n"
                        "        bs_combos(&x[%d][0], c1);\n        bs_combos(&x[%d][4], c2);\n",
                     buf, buf, buf);
        emit_network(f, E, k, m, j, j == 0);
        emit_acc_fence(f, 0, P);
        std::fprintf(f, "    }\n");
    }
    std::fprintf(f, "    BS_FENCE();\n");
    std::fprintf(f, "    const bool okb = cb <= last;\n");
    std::fprintf(f, "#pragma unroll\n    for (int t = 0; t < %d; ++t) {\n", m);
    std::fprintf(f, "        const int r = %s;\n", kMovementLowReg ? "0" : "t");
    std::fprintf(f,
                 "        uint32_t w[8] = {acc[8 * r], acc[8 * r + 1], acc[8 * r + 2], acc[8 * r + 3],\n"
                 "                         acc[8 * r + 4], acc[8 * r + 5], acc[8 * r + 6], acc[8 * r + 7]};\n"
                 "        bs_from_planes(w);\n"
                 "        uint8_t* o = p + static_cast<uint64_t>(t) * a.pitch;\n"
                 "        bs_store(o, offa, w[0], w[1], w[2], w[3]);\n"
                 "        if (okb) bs_store(o, offb, w[4], w[5], w[6], w[7]);\n"
                 "    }\n}\n\n");

    std::fprintf(f,
                 "hipError_t launch_%s(const BitsliceArgs& a, hipStream_t stream) {\n"
                 "    const uint64_t blocks = a.stripes * a.blocks_per_stripe;\n"
                 "    if (blocks == 0) return hipSuccess;\n"
                 "    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;\n"
                 "    hipLaunchKernelGGL(%s, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream, a);\n"
                 "    return hipGetLastError();\n}\n\n",
                 name.c_str(), name.c_str());
}

// Bit-sliced reconstruct (bitslice.hpp): inputs are the present data shards
// (network) and the parity survivors (XORed into their rows' planes, giving
// the syndromes); then the e outputs are split-table products of the
// syndromes with the decode rows' parity-survivor columns.  kRows outputs per
// pass keep the accumulators, syndromes and tables within 256 VGPRs.
//
// top < m: a row-subset variant whose network, accumulators and tables cover
// only the top `top` parity rows (m - top .. m - 1).  Rebuild fills erased
// data slots with the highest-numbered parity survivors, so stripes with few
// erasures use only top rows; the host routes a stripe here when every
// parity row its pattern uses (syndromes and erased-parity outputs) is one
// of them.  Fewer accumulators -> fewer VGPRs -> more waves per SIMD.
std::string rec_name(int k, int m, int top) {
    return "rs_bitslice_rec_k" + std::to_string(k) + "_m" + std::to_string(m) +
           (top < m ? "_t" + std::to_string(top) : std::string());
}

void emit_reconstruct(FILE* f, int k, int n, int top) {
    const int PF = top < n - k && kTopPrefetch > 0 ? kTopPrefetch : kRecPrefetch > 0 ? kRecPrefetch : kPrefetch;
    const int m = n - k;
    const int T0 = m - top;  // first parity row covered
    const std::vector<uint8_t> E = rsmi::systematic_matrix(k, n);
    const std::string name = rec_name(k, m, top);
    const int P = top * 8;
    const int N = k + top;  // inputs: data 0..k-1, then parity rows T0..m-1
    const int kRows = kRecRows;
    const int NG = (m + kRows - 1) / kRows;
    auto prow = [&](int j) { return T0 + (j - k); };  // parity row of input j >= k
    auto pres = [&](int j) {
        return j < k ? "((dmask >> " + std::to_string(j) + ") & 1ull)"
                     : "((pmask >> " + std::to_string(prow(j)) + ") & 1u)";
    };
    auto ptr = [&](int j) { return "shard(" + std::to_string(j < k ? j : k + prow(j)) + "u)"; };

    // kPtrs: shard addresses from the caller's table (rs_reconstruct_ptrs);
    // a separate instantiation, so the strided kernel carries no trace of it.
    std::fprintf(f, "template <bool kPtrs>\n__global__ __launch_bounds__(256) void %s(BitsliceRecArgs a) {\n", name.c_str());
    std::fprintf(f, "    constexpr int K = %d, M = %d, R = %d, NG = %d, TOP = %d, T0 = %d;\n", k, m, kRows, NG, top, T0);
    std::fprintf(f, "%s", R"(#if BS_PLANE_SOLVE
    // The syndrome coefficients: byte o of row t - T0 multiplies syndrome t
    // into output o (zero past the outputs and for parity rows that are not
    // survivors); one word holds a solve group's R = 4 outputs.
    __shared__ uint32_t mcoef[TOP][(NG * R + 3) / 4];
#else
    // Split tables of the syndrome coefficients: mtab[o][t - T0] multiplies
    // syndrome t into output o (zero past the outputs and for parity rows
    // that are not survivors).
    __shared__ uint32_t mtab[NG * R][TOP][5];
#endif
    // A stripe's blocks run on one XCD, in order (xcd.hpp).
    const uint32_t bx = a.xcd ? xcd_block(blockIdx.x, a.xcd * a.blocks_per_stripe, gridDim.x) : blockIdx.x;
    const uint64_t sv = bx / a.blocks_per_stripe;
    const uint32_t blk = bx - static_cast<uint32_t>(sv) * a.blocks_per_stripe;
    // The descriptor and its mask record (below), both scalar loads issued
    // back to back -- from the uploaded arrays, or (a small call) from the
    // kernel arguments.
    const BsStripeMask mk = a.stripe_desc ? a.stripe_mask[sv] : a.inl_mask[sv];
    const uint2 desc = a.stripe_desc ? a.stripe_desc[sv] : a.inl_desc[sv];
    const uint64_t s = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(desc.x));
    const uint32_t sw = __builtin_amdgcn_readfirstlane(desc.y);
    const uint32_t pat = sw >> 8, e = sw & 0xFFu;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t last = a.ncols16 - 1u;
    uint8_t* d = a.data + s * a.data_ss;
    uint8_t* p = a.parity + s * a.parity_ss;
    // Shard id i's address: the strided layout, or the caller's table
    // (pointer mode, one scalar load per input).
    const uint64_t* sptr = kPtrs ? a.shard_ptrs + s * static_cast<uint64_t>(K + M) : nullptr;
    auto shard = [&](uint32_t i) -> uint8_t* {
        if constexpr (kPtrs) return reinterpret_cast<uint8_t*>(sptr[i]);
        return i < static_cast<uint32_t>(K) ? d + static_cast<uint64_t>(i) * a.pitch
                                            : p + static_cast<uint64_t>(i - K) * a.pitch;
    };
    // Rebuild's slots: data shard j present <=> slot j holds shard j; each
    // erased data slot holds a parity survivor.  The host's mask record comes
    // with the descriptor (one scalar round trip, bitslice.hpp BsStripeMask),
    // so the first data loads need no dependent load of the pattern's ids.
    // (readfirstlane returns int: each word goes through uint32_t, or a set
    // bit 31 of dlo would sign-extend over the high word.)
    uint64_t dmask = static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(mk.dhi))) << 32 |
                     static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(mk.dlo));
    uint32_t pmask = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(mk.pmask));
    uint32_t qmask = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(mk.qmask));
    // The pattern's output ids, one per lane, requested before the data: a
    // fresh pattern's row is an L2 miss, and read by scalar loads inside the
    // solve it stalled every output group (readlane below instead).
    // (Every lane loads, clamped into the row: no exec-masked branch ahead
    // of the data loads.  Ids past e are never used.)
    const uint32_t did_l = a.dst[static_cast<size_t>(pat) * a.dst_stride + min(lane, a.dst_stride - 1u)];
)");
    if (kDebugMasks)
        std::fprintf(f, "%s", R"(    {
        const uint32_t sid = lane < static_cast<uint32_t>(K) ? a.src[static_cast<size_t>(pat) * K + lane] : 0xFFFFFFFFu;
        const uint32_t did = lane < e ? a.dst[static_cast<size_t>(pat) * a.dst_stride + lane] : 0xFFFFFFFFu;
        const uint64_t dm2 = __builtin_amdgcn_ballot_w64(sid == lane);
        uint32_t pm2 = 0u, qm2 = 0u;
#pragma unroll
        for (int t = 0; t < M; ++t) {
            const uint64_t b = __builtin_amdgcn_ballot_w64(sid == static_cast<uint32_t>(K + t));
            pm2 |= b ? (1u << t) : 0u;
            qm2 |= __builtin_amdgcn_ballot_w64(did == static_cast<uint32_t>(K + t)) ? (1u << t) : 0u;
        }
        if (threadIdx.x == 0 && blk == 0 && (dm2 != dmask || pm2 != pmask || qm2 != qmask))
            printf("RSMI_MASK_MISMATCH sv=%llu s=%llu pat=%u e=%u host d=%016llx p=%x q=%x dev d=%016llx p=%x q=%x\n",
                   (unsigned long long)sv, (unsigned long long)s, pat, e, (unsigned long long)dmask, pmask, qmask,
                   (unsigned long long)dm2, pm2, qm2);
        dmask = dm2; pmask = pm2; qmask = qm2;
    }
)");
    std::fprintf(f, "%s", R"(    // Parity rows the pattern uses (syndromes of Rebuild's parity survivors,
    // q rows of erased parity): the network skips the others.
    const uint32_t rmask = pmask | qmask;
    (void)rmask;  // unguarded row-subset variants
)");
    if (kRecIters > 1)
        std::fprintf(f, "    for (uint32_t it = 0; it < %du; ++it) {\n"
                        "    const uint32_t win = blk * %du + it;\n"
                        "    if (win * 512u > last) break;  // past the shard: uniform\n", kRecIters, kRecIters);
    else
        std::fprintf(f, "    {\n    const uint32_t win = blk, it = 0u;\n");
    std::fprintf(f, "%s", R"(    uint32_t ca, cb;
    bs_cols(win, wave, lane, ca, cb);
    const bool oka = ca <= last, okb = cb <= last;  // lanes past the shard code a clamped column, never stored
    const uint32_t offa = (oka ? ca : last) * 16u, offb = (okb ? cb : last) * 16u;
)");
    std::fprintf(f, "    uint32_t acc[%d];\n#pragma unroll\n    for (int i = 0; i < %d; ++i) acc[i] = 0u;\n", P, P);
    std::fprintf(f, "    uint32_t x[%d][8];\n", PF + 1);
    // Every input's load is issued, unconditionally: an absent input loads
    // the 2 KiB zero page at the wave's own lane offsets (the same lines for
    // every block, so they stay in L2: no HBM traffic) and its network step
    // is skipped.  Loads under a branch made the compiler wait for every load
    // in flight (vmcnt(0)) at each input, i.e. no prefetch at all.
    if (!kBufferLoads)  // (buffer loads: absent inputs get an empty range, no zero page)
        std::fprintf(f, "    const uint32_t zoffa = lane * 16u, zoffb = 1024u + lane * 16u;\n");
    auto emit_load = [&](int j, int buf) {
        const std::string pr = pres(j);
        if (kBufferLoads)
            std::fprintf(f, "    bs_load_buf(x[%d], bs_rsrc(%s, %s), offa, offb);\n", buf, ptr(j).c_str(), pr.c_str());
        else
            std::fprintf(f, "    bs_load(x[%d], %s ? %s : a.zpage, %s ? offa : zoffa, %s ? offb : zoffb);\n", buf,
                         pr.c_str(), ptr(j).c_str(), pr.c_str(), pr.c_str());
    };
    for (int j = 0; j < PF && j < N; ++j) emit_load(j, j);
    std::fprintf(f, "%s", R"(    // slot_t[t]: the erased data slot parity survivor t fills.  Rebuild walks
    // the slots upwards and gives each erased one the highest remaining
    // share, so the erased slots in ascending order take the survivors from
    // the top (scalar bit scans, after the first loads are issued).
    uint32_t slot_t[M];
    {
        uint64_t er = ~dmask & (K == 64 ? ~0ull : ((1ull << (K & 63)) - 1ull));
#pragma unroll
        for (int t = M - 1; t >= 0; --t) {
            const bool sv_t = (pmask >> t) & 1u;
            // The host's record has exactly one parity survivor per erased
            // data slot (rsmi.cpp stripe_mask; tests/test_gpu_parity.py pins
            // the straddling sets).  min: a record breaking that (er empty)
            // still cannot index past the pattern's row -- wrong bytes, never
            // a fault; the -M diagnostic build reports it.
            slot_t[t] = sv_t ? min(static_cast<uint32_t>(__builtin_ctzll(er)), static_cast<uint32_t>(K - 1)) : 0u;
)");
    if (kDebugMasks)
        std::fprintf(f, "%s", R"(            if (sv_t && er == 0ull && threadIdx.x == 0 && blk == 0)
                printf("RSMI_MASK_SLOT_OVERFLOW s=%llu pat=%u t=%d pmask=%x\n", (unsigned long long)s, pat, t, pmask);
)");
    std::fprintf(f, "%s", R"(            er = sv_t ? (er & (er - 1ull)) : er;
        }
    }
)");
    // The solve's coefficients are requested here, behind the first inputs'
    // loads, and turned into LDS tables only after the last input.  Building
    // them here (round 4) needed the byte at once: vmcnt(0) drained the
    // prefetch of every block before input PF's loads could issue -- a full
    // memory latency per block, in the movement twin as well.
    const int CPT = (NG * kRows * top + 255) / 256;  // coefficients per thread
    std::fprintf(f, "    constexpr int CPT = %d;  // decode coefficients per thread\n", CPT);
    std::fprintf(f, "%s", R"(    uint32_t tcoef[CPT];
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
        const uint32_t idx = threadIdx.x + 256u * q;
        const uint32_t o = idx / TOP, t = T0 + (idx - o * TOP);
        uint32_t slot = 0u;
#pragma unroll
        for (int u = 0; u < M; ++u) slot = t == static_cast<uint32_t>(u) ? slot_t[u] : slot;
        tcoef[q] = 0u;
        if (it == 0u && idx < static_cast<uint32_t>(NG * R * TOP) && o < e && ((pmask >> t) & 1u))
            tcoef[q] = a.coef[(static_cast<size_t>(pat) * M + o) * K + slot];
    }
)");
    for (int j = 0; j < N; ++j) {
        const int buf = j % (PF + 1);
        std::fprintf(f, "    // input %d (%s)\n    BS_FENCE();\n", j, j < k ? "data" : "parity");
        if (j + PF < N)
            emit_load(j + PF, (j + PF) % (PF + 1));
        std::fprintf(f, "    if (%s) {\n", pres(j).c_str());
        const std::string xb = "x[" + std::to_string(buf) + "]";
        if (kInputBarrier)
            std::fprintf(f, "        asm volatile(\"\" : \"+v\"(%s[0]), \"+v\"(%s[1]), \"+v\"(%s[2]), \"+v\"(%s[3]), "
                            "\"+v\"(%s[4]), \"+v\"(%s[5]), \"+v\"(%s[6]), \"+v\"(%s[7]));\n",
                         xb.c_str(), xb.c_str(), xb.c_str(), xb.c_str(), xb.c_str(), xb.c_str(), xb.c_str(), xb.c_str());
        if (kMovementOnly) {
            // movement twin: the input only enters one row's accumulators
            const int t = (j % top) * 8;
            for (int q = 0; q < 8; ++q) std::fprintf(f, "        acc[%d] ^= %s[%d];\n", t + q, xb.c_str(), q);
            std::fprintf(f, "    }\n");
            continue;
        }
        if (j < k) {
            std::fprintf(f, "        bs_to_planes(%s);\n", xb.c_str());
            std::fprintf(f, "        uint32_t c1[16], c2[16];\n        bs_combos(&%s[0], c1);\n"
                            "        bs_combos(&%s[4], c2);\n", xb.c_str(), xb.c_str());
            emit_network(f, E, k, m, j, false, top < m && !kTopGuard ? nullptr : "rmask", T0);
            emit_acc_fence(f, 0, P);
        } else if (kPlaneSolve) {
            // Parity survivor t: row t's network sum is complete (data inputs
            // come first); the survivor's planes are XORed in, and acc row t
            // holds syndrome t in planes for the plane solve.
            const int t = j - k;  // accumulator row (parity row T0 + t)
            std::fprintf(f, "        bs_to_planes(%s);\n", xb.c_str());
            for (int q = 0; q < 8; ++q) std::fprintf(f, "        acc[%d] ^= %s[%d];\n", t * 8 + q, xb.c_str(), q);
            emit_acc_fence(f, t * 8, t * 8 + 8);
        } else {
            // Parity survivor t: row t's network sum is complete (data inputs
            // come first), so the row goes back to bytes here and the
            // survivor's bytes are XORed in as loaded -- no transpose of the
            // survivor.  acc row t then holds syndrome t in bytes.
            const int t = j - k;  // accumulator row (parity row T0 + t)
            std::fprintf(f, "        uint32_t w[8] = {acc[%d], acc[%d], acc[%d], acc[%d], acc[%d], acc[%d], acc[%d], acc[%d]};\n"
                            "        bs_from_planes(w);\n",
                         t * 8, t * 8 + 1, t * 8 + 2, t * 8 + 3, t * 8 + 4, t * 8 + 5, t * 8 + 6, t * 8 + 7);
            for (int q = 0; q < 8; ++q) std::fprintf(f, "        acc[%d] = w[%d] ^ %s[%d];\n", t * 8 + q, q, xb.c_str(), q);
            emit_acc_fence(f, t * 8, t * 8 + 8);
        }
        std::fprintf(f, "    }\n");
    }
    // The solve's split tables (coefficients requested in the prologue).
    std::fprintf(f, "%s", R"(    BS_FENCE();
    if (it == 0u) {
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            const uint32_t idx = threadIdx.x + 256u * q;
            const uint32_t o = idx / TOP, t = idx - o * TOP;
#if BS_PLANE_SOLVE
            if (idx < static_cast<uint32_t>(NG * R * TOP)) reinterpret_cast<uint8_t*>(&mcoef[t][0])[o] = static_cast<uint8_t>(tcoef[q]);
#else
            if (idx < static_cast<uint32_t>(NG * R * TOP)) gfd::build_tables(tcoef[q], &mtab[o][t][0]);
#endif
        }
    }
)");
    if (kMovementOnly) {
        // movement twin: output r stores accumulator row r mod TOP (same
        // stores, descriptors and mask record as the real kernel).
        std::fprintf(f, "%s", R"(    BS_FENCE();
    if (it == 0u) __syncthreads();
#pragma unroll 1
    for (uint32_t r = 0; r < e; ++r) {
        const uint32_t oid = static_cast<uint32_t>(__builtin_amdgcn_readlane(did_l, r));
        uint32_t w[8];
        const uint32_t row = r % static_cast<uint32_t>(TOP);
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = 0u;
#pragma unroll
        for (int t = 0; t < TOP; ++t)
            if (row == static_cast<uint32_t>(t)) {
#pragma unroll
                for (int i = 0; i < 8; ++i) w[i] = acc[8 * t + i];
            }
        uint8_t* o = shard(oid);
        if (oka) bs_store(o, offa, w[0], w[1], w[2], w[3]);
        if (okb) bs_store(o, offb, w[4], w[5], w[6], w[7]);
    }
    }  // column window
}

)");
    } else if (kPlaneSolve) {
    std::fprintf(f, "%s", R"(    BS_FENCE();
    if (it == 0u) __syncthreads();  // mcoef complete
    // Outputs in groups of R: out = (q row of an erased parity output) + the
    // sum over syndromes t of c(o, t) * s_t, all in planes.  For each syndrome
    // the planes y = 2^b * s_t are advanced b = 0..7 (bs_mul2) and XORed into
    // every output whose coefficient has bit b set (wave-uniform branches).
#pragma unroll 1
    for (uint32_t g = 0; g < e; g += R) {
        uint32_t oid[R];
#pragma unroll
        for (int r = 0; r < R; ++r)
            oid[r] = g + r < e ? static_cast<uint32_t>(__builtin_amdgcn_readlane(did_l, g + r)) : 0xFFFFFFFFu;
        uint32_t out[R][8];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int w = 0; w < 8; ++w) out[r][w] = 0u;
#pragma unroll
        for (int t = T0; t < M; ++t) {
            const int at = 8 * (t - T0);  // row t's accumulators
            if ((pmask >> t) & 1u) {
                // Syndrome t's planes enter here (keeps the scheduler from
                // hoisting every syndrome's advances together).
                asm volatile("" : "+v"(acc[at + 0]), "+v"(acc[at + 1]), "+v"(acc[at + 2]), "+v"(acc[at + 3]),
                                  "+v"(acc[at + 4]), "+v"(acc[at + 5]), "+v"(acc[at + 6]), "+v"(acc[at + 7]));
                // c(g + r, t) for r < R: byte r of one LDS word, made scalar
                const uint32_t cw = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(mcoef[t - T0][g >> 2]));
                uint32_t y[8];
#pragma unroll
                for (int w = 0; w < 8; ++w) y[w] = acc[at + w];
#pragma unroll
                for (int b = 0; b < 8; ++b) {
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        if ((cw >> (8 * r + b)) & 1u) {
#pragma unroll
                            for (int w = 0; w < 8; ++w) out[r][w] ^= y[w];
                        }
                    if (b < 7) bs_mul2(y);
                }
            }
            if ((qmask >> t) & 1u) {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (oid[r] == static_cast<uint32_t>(K + t)) {
#pragma unroll
                        for (int w = 0; w < 8; ++w) out[r][w] ^= acc[at + w];
                    }
            }
#pragma unroll
            for (int r = 0; r < R; ++r)
                asm volatile("" : "+v"(out[r][0]), "+v"(out[r][1]), "+v"(out[r][2]), "+v"(out[r][3]),
                                  "+v"(out[r][4]), "+v"(out[r][5]), "+v"(out[r][6]), "+v"(out[r][7])::"memory");
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (g + r >= e) break;
            bs_from_planes(out[r]);
            uint8_t* o = shard(oid[r]);
            if (oka) bs_store(o, offa, out[r][0], out[r][1], out[r][2], out[r][3]);
            if (okb) bs_store(o, offb, out[r][4], out[r][5], out[r][6], out[r][7]);
        }
    }
    }  // column window
}

)");
    } else {
    std::fprintf(f, "%s", R"(    BS_FENCE();
    if (it == 0u) __syncthreads();  // mtab complete
    // The parity outputs' q rows back to bytes (syndrome rows already are).
#pragma unroll
    for (int t = T0; t < M; ++t)
        if ((qmask >> t) & 1u) {
            uint32_t w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = acc[8 * (t - T0) + i];
            bs_from_planes(w);
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[8 * (t - T0) + i] = w[i];
        }
)");
    std::fprintf(f, "#pragma unroll 1\n    for (uint32_t g = 0; g < e; g += R) {\n%s",
                 kSolveTail ? R"SOLVE(        uint32_t oid[R];
#pragma unroll
        for (int r = 0; r < R; ++r)
            oid[r] = g + r < e ? static_cast<uint32_t>(__builtin_amdgcn_readlane(did_l, g + r)) : 0xFFFFFFFFu;
        uint32_t out[R][8];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int w = 0; w < 8; ++w) out[r][w] = 0u;
#pragma unroll
        for (int t = T0; t < M; ++t) {
            const int at = 8 * (t - T0);  // row t's accumulators
            if ((pmask >> t) & 1u) {
                // Syndrome t's words enter here (otherwise the scheduler
                // hoists every syndrome's bit fields: ~100 extra VGPRs).
                asm volatile("" : "+v"(acc[at + 0]), "+v"(acc[at + 1]), "+v"(acc[at + 2]), "+v"(acc[at + 3]),
                                  "+v"(acc[at + 4]), "+v"(acc[at + 5]), "+v"(acc[at + 6]), "+v"(acc[at + 7]));
                uint32_t T[R][5];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int i = 0; i < 5; ++i) T[r][i] = mtab[g + r][t - T0][i];
                // Fields of the syndrome's 8 words once; each output of the
                // group is coded only if it exists (no padded outputs when
                // e is not a multiple of R).
                gfd::Fields fl[8];
#pragma unroll
                for (int w = 0; w < 8; ++w) fl[w] = gfd::fields(acc[at + w]);
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (r == 0 || g + r < e) {
#pragma unroll
                        for (int w = 0; w < 8; ++w) out[r][w] = gfd::gf_mac(out[r][w], T[r], fl[w].a, fl[w].b, fl[w].c);
                    }
            }
            if ((qmask >> t) & 1u) {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (oid[r] == static_cast<uint32_t>(K + t)) {
#pragma unroll
                        for (int w = 0; w < 8; ++w) out[r][w] ^= acc[at + w];
                    }
            }
#pragma unroll
            for (int r = 0; r < R; ++r)
                asm volatile("" : "+v"(out[r][0]), "+v"(out[r][1]), "+v"(out[r][2]), "+v"(out[r][3]),
                                  "+v"(out[r][4]), "+v"(out[r][5]), "+v"(out[r][6]), "+v"(out[r][7])::"memory");
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (g + r >= e) break;
            uint8_t* o = shard(oid[r]);
            if (oka) bs_store(o, offa, out[r][0], out[r][1], out[r][2], out[r][3]);
            if (okb) bs_store(o, offb, out[r][4], out[r][5], out[r][6], out[r][7]);
        }
)SOLVE"
                            : R"SOLVE(        uint32_t oid[R];
#pragma unroll
        for (int r = 0; r < R; ++r)
            oid[r] = g + r < e ? static_cast<uint32_t>(__builtin_amdgcn_readlane(did_l, g + r)) : 0xFFFFFFFFu;
        uint32_t out[R][8];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int w = 0; w < 8; ++w) out[r][w] = 0u;
#pragma unroll
        for (int t = T0; t < M; ++t) {
            const int at = 8 * (t - T0);  // row t's accumulators
            if ((pmask >> t) & 1u) {
                // Syndrome t's words enter here (otherwise the scheduler
                // hoists every syndrome's bit fields: ~100 extra VGPRs).
                asm volatile("" : "+v"(acc[at + 0]), "+v"(acc[at + 1]), "+v"(acc[at + 2]), "+v"(acc[at + 3]),
                                  "+v"(acc[at + 4]), "+v"(acc[at + 5]), "+v"(acc[at + 6]), "+v"(acc[at + 7]));
                uint32_t T[R][5];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int i = 0; i < 5; ++i) T[r][i] = mtab[g + r][t - T0][i];
#pragma unroll
                for (int w = 0; w < 8; ++w) {
                    const gfd::Fields fl = gfd::fields(acc[at + w]);
#pragma unroll
                    for (int r = 0; r < R; ++r) out[r][w] = gfd::gf_mac(out[r][w], T[r], fl.a, fl.b, fl.c);
                }
            }
            if ((qmask >> t) & 1u) {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (oid[r] == static_cast<uint32_t>(K + t)) {
#pragma unroll
                        for (int w = 0; w < 8; ++w) out[r][w] ^= acc[at + w];
                    }
            }
#pragma unroll
            for (int r = 0; r < R; ++r)
                asm volatile("" : "+v"(out[r][0]), "+v"(out[r][1]), "+v"(out[r][2]), "+v"(out[r][3]),
                                  "+v"(out[r][4]), "+v"(out[r][5]), "+v"(out[r][6]), "+v"(out[r][7])::"memory");
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (g + r >= e) break;
            uint8_t* o = shard(oid[r]);
            if (oka) bs_store(o, offa, out[r][0], out[r][1], out[r][2], out[r][3]);
            if (okb) bs_store(o, offb, out[r][4], out[r][5], out[r][6], out[r][7]);
        }
)SOLVE");
    std::fprintf(f, "%s", R"(    }
    }  // column window
}

)");
    }  // the solve (not in the movement twin)
    std::fprintf(f,
                 "hipError_t launch_%s(const BitsliceRecArgs& a, hipStream_t stream) {\n"
                 "    const uint64_t blocks = a.count * a.blocks_per_stripe;\n"
                 "    if (blocks == 0) return hipSuccess;\n"
                 "    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;\n"
                 "    if (a.shard_ptrs)\n"
                 "        hipLaunchKernelGGL(%s<true>, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream, a);\n"
                 "    else\n"
                 "        hipLaunchKernelGGL(%s<false>, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream, a);\n"
                 "    return hipGetLastError();\n}\n\n",
                 name.c_str(), name.c_str(), name.c_str());
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 2 && (std::string(argv[1]) == "-x" || std::string(argv[1]) == "-X")) {
        kMovementOnly = true;
        kMovementLowReg = std::string(argv[1]) == "-X";
        argv += 1;
        argc -= 1;
    }
    for (;;) {  // -S (plane solve), -W / -w (64-bit transpose shifts on / off), -l (no solve tail)
        if (argc >= 2 && std::string(argv[1]) == "-S") kPlaneSolve = true;
        else if (argc >= 2 && std::string(argv[1]) == "-W") kShift64 = true;
        else if (argc >= 2 && std::string(argv[1]) == "-w") kShift64 = false;
        else if (argc >= 2 && std::string(argv[1]) == "-l") kSolveTail = false;
        else break;
        argv += 1;
        argc -= 1;
    }
    if (argc >= 3 && std::string(argv[1]) == "-G") {
        kRowGroup = std::atoi(argv[2]);
        if (kRowGroup < 1 || kRowGroup > 16) {
            std::fprintf(stderr, "bad row group %s\n", argv[2]);
            return 2;
        }
        argv += 2;
        argc -= 2;
    }
    if (argc >= 3 && std::string(argv[1]) == "-R") {
        kRecRows = std::atoi(argv[2]);
        if (kRecRows < 1 || kRecRows > 16) {
            std::fprintf(stderr, "bad solve group %s\n", argv[2]);
            return 2;
        }
        argv += 2;
        argc -= 2;
    }
    if (argc >= 3 && std::string(argv[1]) == "-I") {
        kRecIters = std::atoi(argv[2]);
        if (kRecIters < 1 || kRecIters > 8) {
            std::fprintf(stderr, "bad reconstruct iterations %s\n", argv[2]);
            return 2;
        }
        argv += 2;
        argc -= 2;
    }
    if (argc >= 3 && std::string(argv[1]) == "-T") {
        kTops.clear();
        for (const char* q = argv[2]; *q;) {
            const int v = std::atoi(q);
            if (v < 0 || v > 64) {
                std::fprintf(stderr, "bad top rows %s\n", argv[2]);
                return 2;
            }
            if (v > 0) kTops.push_back(v);
            while (*q && *q != ',') ++q;
            if (*q == ',') ++q;
        }
        argv += 2;
        argc -= 2;
    }
    if (argc >= 3 && std::string(argv[1]) == "-Q") {
        kTopPrefetch = std::atoi(argv[2]);
        if (kTopPrefetch < 1 || kTopPrefetch > 8) {
            std::fprintf(stderr, "bad top-variant prefetch depth %s\n", argv[2]);
            return 2;
        }
        argv += 2;
        argc -= 2;
    }
    if (argc >= 2 && std::string(argv[1]) == "-M") {
        kDebugMasks = true;
        argv += 1;
        argc -= 1;
    }
    if (argc >= 2 && std::string(argv[1]) == "-B") {
        kBufferLoads = true;
        argv += 1;
        argc -= 1;
    }
    if (argc >= 2 && std::string(argv[1]) == "-Z") {
        kBufferLoads = false;
        argv += 1;
        argc -= 1;
    }
    if (argc >= 2 && std::string(argv[1]) == "-N") {
        kInputBarrier = false;
        argv += 1;
        argc -= 1;
    }
    if (argc >= 2 && std::string(argv[1]) == "-Y") {
        kInputBarrier = true;
        argv += 1;
        argc -= 1;
    }
    if (argc >= 2 && std::string(argv[1]) == "-L") {
        kSolveTail = true;
        argv += 1;
        argc -= 1;
    }
    if (argc >= 2 && std::string(argv[1]) == "-u") {
        kTopGuard = true;
        argv += 1;
        argc -= 1;
    }
    if (argc >= 2 && std::string(argv[1]) == "-E") {
        kRowExpect = true;
        argv += 1;
        argc -= 1;
    }
    if (argc >= 2 && std::string(argv[1]) == "-e") {
        kRowExpect = false;
        argv += 1;
        argc -= 1;
    }
    if (argc >= 3 && std::string(argv[1]) == "-g") {
        kGeometry = std::atoi(argv[2]);
        argv += 2;
        argc -= 2;
    }
    if (argc >= 3 && std::string(argv[1]) == "-p") {
        kPrefetch = std::atoi(argv[2]);
        if (kPrefetch < 1 || kPrefetch > 8) {
            std::fprintf(stderr, "bad prefetch depth %s\n", argv[2]);
            return 2;
        }
        argv += 2;
        argc -= 2;
    }
    if (argc >= 3 && std::string(argv[1]) == "-P") {
        kRecPrefetch = std::atoi(argv[2]);
        if (kRecPrefetch < 1 || kRecPrefetch > 8) {
            std::fprintf(stderr, "bad reconstruct prefetch depth %s\n", argv[2]);
            return 2;
        }
        argv += 2;
        argc -= 2;
    }
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s [-x|-X] [-S] [-W|-w] [-l] [-G ROWS] [-R OUTPUTS] [-I ITERS] [-T TOPS] [-Q TOP_PREFETCH] [-M] [-B|-Z] [-N|-Y] [-L] [-u] [-E|-e] [-g GEOMETRY] [-p PREFETCH] [-P REC_PREFETCH] OUT.hip K:N [K:N ...]\n", argv[0]);
        return 2;
    }
    if (kPlaneSolve && kRecRows != 4) {
        std::fprintf(stderr, "the plane solve codes R = 4 outputs per group (-R 4, or -s)\n");
        return 2;
    }
    std::vector<std::pair<int, int>> codes;
    for (int i = 2; i < argc; ++i) {
        int k = 0, n = 0;
        if (std::sscanf(argv[i], "%d:%d", &k, &n) != 2 || k < 1 || n <= k || n > 256) {
            std::fprintf(stderr, "bad code %s\n", argv[i]);
            return 2;
        }
        codes.push_back({k, n});
    }
    FILE* f = std::fopen(argv[1], "w");
    if (!f) return 1;
    emit_common(f);
    // Row-subset reconstruct variants (emit_reconstruct top < m): the listed
    // tops that are below m, for codes with at least kTopMinM parity rows.
    auto tops_of = [](int m) {
        std::vector<int> t;
        if (m >= kTopMinM)
            for (int v : kTops)
                if (v < m) t.push_back(v);
        return t;
    };
    for (auto [k, n] : codes) {
        emit_kernel(f, k, n);
        if (k <= kRecMaxK && n - k <= kRecMaxM) {
            emit_reconstruct(f, k, n, n - k);
            for (int top : tops_of(n - k)) emit_reconstruct(f, k, n, top);
        }
    }
    std::fprintf(f, "}  // namespace\n\nconst BitsliceKernel* bitslice_kernel(int k, int m) {\n"
                    "    static const BitsliceKernel table[] = {\n");
    for (auto [k, n] : codes) {
        const int m = n - k;
        const std::string name = "rs_bitslice_k" + std::to_string(k) + "_m" + std::to_string(m);
        const std::string rec = rec_name(k, m, m);
        if (k <= kRecMaxK && n - k <= kRecMaxM) {
            const std::vector<int> tops = tops_of(m);
            std::string tv = "{", tl = "{", tn = "{";
            for (size_t i = 0; i < tops.size(); ++i) {
                const std::string r = rec_name(k, m, tops[i]);
                tv += (i ? ", " : "") + std::to_string(tops[i]);
                tl += (i ? ", launch_" : "launch_") + r;
                tn += (i ? ", \"" : "\"") + r.substr(3) + "\"";
            }
            tv += "}";
            tl += "}";
            tn += "}";
            std::fprintf(f, "        {%d, %d, \"%s\", %s_matrix, launch_%s, \"%s\", launch_%s, %d, %zu, %s, %s, %s},\n", k, m,
                         name.c_str() + 3, name.c_str(), name.c_str(), rec.c_str() + 3, rec.c_str(), kRecIters, tops.size(),
                         tops.empty() ? "{}" : tv.c_str(), tops.empty() ? "{}" : tl.c_str(),
                         tops.empty() ? "{}" : tn.c_str());
        } else {
            std::fprintf(f, "        {%d, %d, \"%s\", %s_matrix, launch_%s, nullptr, nullptr, 1, 0, {}, {}, {}},\n", k, m,
                         name.c_str() + 3, name.c_str(), name.c_str());
        }
    }
    std::fprintf(f, "    };\n    for (const BitsliceKernel& b : table)\n"
                    "        if (b.k == k && b.m == m) return &b;\n    return nullptr;\n}\n\n}  // namespace rsmi\n");
    return std::fclose(f) == 0 ? 0 : 1;
}
