// blake2b.hip -- batched BLAKE2b (RFC 7693) kernel, see blake2b.hpp.
#include "blake2b.hpp"

namespace rsmi {
namespace {

constexpr uint32_t kQuads = 16;  // messages per 64-lane block (one wave)

__constant__ uint64_t kIV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                                0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};

// RFC 7693 sigma, rows 0..9 (rounds 10 and 11 reuse rows 0 and 1).
constexpr uint8_t kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
};

// Per (round row r, lane j): the message word indexes lane j's two G calls
// read, packed as bytes {col x, col y, diag x, diag y}.
struct SigmaLanes {
    uint32_t w[10][4];
};
constexpr SigmaLanes make_sigma_lanes() {
    SigmaLanes s{};
    for (int r = 0; r < 10; ++r)
        for (int j = 0; j < 4; ++j)
            s.w[r][j] = uint32_t(kSigma[r][2 * j]) | uint32_t(kSigma[r][2 * j + 1]) << 8 |
                        uint32_t(kSigma[r][8 + 2 * j]) << 16 | uint32_t(kSigma[r][9 + 2 * j]) << 24;
    return s;
}
__constant__ SigmaLanes kSigLanes = make_sigma_lanes();

// 64-bit rotations as funnel shifts of the 32-bit halves (v_alignbit_b32):
// two ops for n < 32, none for n = 32.
__device__ __forceinline__ uint64_t pack64(uint32_t lo, uint32_t hi) {
    return static_cast<uint64_t>(lo) | (static_cast<uint64_t>(hi) << 32);
}
template <int N>
__device__ __forceinline__ uint64_t rotr64(uint64_t x) {
    const uint32_t lo = static_cast<uint32_t>(x), hi = static_cast<uint32_t>(x >> 32);
    if constexpr (N == 32) {
        return pack64(hi, lo);
    } else if constexpr (N < 32) {
        return pack64(__builtin_amdgcn_alignbit(hi, lo, N), __builtin_amdgcn_alignbit(lo, hi, N));
    } else {  // rotr by 32 + (N - 32)
        return pack64(__builtin_amdgcn_alignbit(lo, hi, N - 32), __builtin_amdgcn_alignbit(hi, lo, N - 32));
    }
}

__device__ __forceinline__ void G(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t x, uint64_t y) {
    a = a + b + x;
    d = rotr64<32>(d ^ a);
    c = c + d;
    b = rotr64<24>(b ^ c);
    a = a + b + y;
    d = rotr64<16>(d ^ a);
    c = c + d;
    b = rotr64<63>(b ^ c);
}

// Lane j of a quad takes the value of lane (j + R) mod 4 (DPP quad_perm).
template <int R>
__device__ __forceinline__ uint64_t quad_rot(uint64_t v) {
    constexpr int ctrl = ((0 + R) & 3) | (((1 + R) & 3) << 2) | (((2 + R) & 3) << 4) | (((3 + R) & 3) << 6);
    const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(static_cast<uint32_t>(v)), ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(static_cast<uint32_t>(v >> 32)), ctrl, 0xF, 0xF, false);
    return static_cast<uint64_t>(static_cast<uint32_t>(lo)) | (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32);
}

// Bytes [off, off + 32) of a message (zero past len) as 8 little-endian
// dwords.  Aligned interior pieces take two 16-byte loads; otherwise
// dword-aligned loads that hold at least one message byte (never a word
// wholly past the end) are funnel-shifted into place.
__device__ __forceinline__ void load32(const uint8_t* base, uint64_t len, uint64_t off, uint32_t (&w)[8]) {
    const uint8_t* p = base + off;
    if (off + 32 <= len && (reinterpret_cast<uintptr_t>(p) & 15u) == 0) {
        const uint4 u = *reinterpret_cast<const uint4*>(p);
        const uint4 v = *reinterpret_cast<const uint4*>(p + 16);
        w[0] = u.x; w[1] = u.y; w[2] = u.z; w[3] = u.w;
        w[4] = v.x; w[5] = v.y; w[6] = v.z; w[7] = v.w;
        return;
    }
    const uintptr_t pa = reinterpret_cast<uintptr_t>(p);
    const uint32_t sh = static_cast<uint32_t>(pa & 3u);
    const uint32_t* al = reinterpret_cast<const uint32_t*>(pa - sh);
    const uintptr_t end = reinterpret_cast<uintptr_t>(base) + len;  // one past the last byte
    uint32_t raw[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const uintptr_t a = pa - sh + 4u * i;
        raw[i] = (i < 8 || sh) && a < end ? al[i] : 0u;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t x = sh ? __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh) : raw[i];
        const uint64_t pos = off + 4u * i;  // message offset of byte 0 of word i
        const uint64_t valid = pos >= len ? 0 : len - pos;
        if (valid < 4) x &= valid ? (1u << (8u * static_cast<uint32_t>(valid))) - 1u : 0u;
        w[i] = x;
    }
}

__global__ __launch_bounds__(64) void blake2b_kernel(Blake2bArgs a) {
    __shared__ uint64_t blk[kQuads][16];
    const uint32_t lane = threadIdx.x, j = lane & 3u, qi = lane >> 2;
    const uint32_t q = blockIdx.x * kQuads + qi;
    const bool live = q < a.count;
    const uint32_t msg = live ? (a.order ? a.order[q] : q) : 0u;
    const uint8_t* base = live ? reinterpret_cast<const uint8_t*>(a.ptrs[msg]) : nullptr;
    const uint64_t len = live ? a.lens[msg] : 0;
    const uint64_t nb = live ? (len ? (len + 127) / 128 : 1) : 0;
    uint32_t so[10];
#pragma unroll
    for (int r = 0; r < 10; ++r) so[r] = kSigLanes.w[r][j];
    // Parameter block: digest length, key length 0, fanout 1, depth 1.
    uint64_t h0 = kIV[j] ^ (j == 0 ? (0x01010000ull ^ a.digest_len) : 0ull);
    uint64_t h1 = kIV[4 + j];
    const uint64_t iv_c = kIV[j], iv_d = kIV[4 + j];
    uint64_t* mb = blk[qi];
    uint32_t nxt[8] = {};
    if (nb) load32(base, len, 32u * j, nxt);
    for (uint64_t b = 0; b < nb; ++b) {
        // The quad's lanes each place 32 bytes of block b in LDS.
        mb[4 * j + 0] = static_cast<uint64_t>(nxt[0]) | static_cast<uint64_t>(nxt[1]) << 32;
        mb[4 * j + 1] = static_cast<uint64_t>(nxt[2]) | static_cast<uint64_t>(nxt[3]) << 32;
        mb[4 * j + 2] = static_cast<uint64_t>(nxt[4]) | static_cast<uint64_t>(nxt[5]) << 32;
        mb[4 * j + 3] = static_cast<uint64_t>(nxt[6]) | static_cast<uint64_t>(nxt[7]) << 32;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (b + 1 < nb) load32(base, len, (b + 1) * 128u + 32u * j, nxt);  // next block in flight
        const bool last = b + 1 == nb;
        const uint64_t t = last ? len : (b + 1) * 128u;  // bytes compressed so far (t1 = 0)
        uint64_t va = h0, vb = h1, vc = iv_c, vd = iv_d;
        if (j == 0) vd ^= t;
        if (j == 2 && last) vd = ~vd;  // f0: final block
#pragma unroll
        for (int r = 0; r < 12; ++r) {
            const uint32_t s = so[r % 10];
            G(va, vb, vc, vd, mb[s & 15u], mb[(s >> 8) & 15u]);
            vb = quad_rot<1>(vb);
            vc = quad_rot<2>(vc);
            vd = quad_rot<3>(vd);
            G(va, vb, vc, vd, mb[(s >> 16) & 15u], mb[s >> 24]);
            vb = quad_rot<3>(vb);
            vc = quad_rot<2>(vc);
            vd = quad_rot<1>(vd);
        }
        h0 ^= va ^ vc;
        h1 ^= vb ^ vd;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // block b's words read before they are overwritten
    }
    if (!live) return;
    // Lane j holds h[j] (digest bytes 8j..8j+7) and h[4+j] (bytes 32+8j..).
    uint8_t* o = a.out + static_cast<uint64_t>(msg) * a.digest_len;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t p0 = 8u * j + i, p1 = 32u + 8u * j + i;
        if (p0 < a.digest_len) o[p0] = static_cast<uint8_t>(h0 >> (8 * i));
        if (p1 < a.digest_len) o[p1] = static_cast<uint8_t>(h1 >> (8 * i));
    }
}

}  // namespace

hipError_t launch_blake2b(const Blake2bArgs& a, hipStream_t stream) {
    if (a.count == 0) return hipSuccess;
    if (a.digest_len < 1 || a.digest_len > 64) return hipErrorInvalidValue;
    const uint32_t blocks = (a.count + kQuads - 1) / kQuads;
    hipLaunchKernelGGL(blake2b_kernel, dim3(blocks), dim3(64), 0, stream, a);
    return hipGetLastError();
}

}  // namespace rsmi
