/*
 * rs_oracle.h -- CPU restatement of the Reed-Solomon codec the reference
 * plugin uses (github.com/vivint/infectious, version unpinned: the reference
 * has no go.mod / vendor tree).
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * / CPU baseline -- never as the product path.
 *
 * Parity status: the evaluation points {0, a^1 .. a^(n-1)} of the systematic
 * Vandermonde matrix are restated from the upstream algorithm, not pinned by
 * an upstream known-answer vector (none exists in /root/reference).
 * Reconstructed data is self-verifying (must equal the original input); the
 * Shard wire format is pinned separately by tests/golden.  See DESIGN.md
 * "Parity status".
 */
#ifndef RS_ORACLE_H
#define RS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORC_OK = 0,
    ORC_EINVAL_KN = -1,        /* "requires 1 <= k <= n <= 256"            */
    ORC_ELEN = -2,             /* "input length must be a multiple of k"   */
    ORC_ENOT_ENOUGH = -3,      /* NotEnoughShares                          */
    ORC_EBAD_ID = -4,          /* "invalid share id"                       */
    ORC_ESINGULAR = -5,        /* "singular matrix"                        */
    ORC_ENOSHARES = -6,        /* "must specify at least one share"        */
    ORC_ETOO_MANY = -7,        /* TooManyErrors (Berlekamp-Welch)          */
};

/* GF(2^8), poly 0x11D, generator 2. */
uint8_t orc_gf_mul(uint8_t a, uint8_t b);
uint8_t orc_gf_inv(uint8_t a);
uint8_t orc_gf_exp(int i);
int orc_gf_log(uint8_t a);

/* infectious.NewFEC(k, n): fills enc (n*k, row-major, systematic).
 * point_offset: 1 = points {0, a^1, ..., a^(n-1)} (infectious, default),
 *               0 = points {0, a^0, ..., a^(n-2)} (zfec). */
int orc_fec_matrix(int k, int n, int point_offset, uint8_t *enc);

/* infectious (*FEC).Encode: input of len bytes (len % k == 0) -> parity
 * shares k..n-1, each len/k bytes, written contiguously to parity. */
int orc_encode(const uint8_t *enc, int k, int n, const uint8_t *input,
               size_t len, uint8_t *parity);

/* infectious (*FEC).Decode(dst, shares) restricted to the Rebuild path
 * (Correct is a no-op for exactly k distinct shares, the only case the
 * reference plugin produces, main.go:65).  numbers[cnt], shares[cnt] each of
 * share_len bytes.  Sorts (numbers, shares) in place like infectious.
 * dst receives k*share_len bytes. */
int orc_decode(const uint8_t *enc, int k, int n, int *numbers,
               const uint8_t **shares, int cnt, size_t share_len,
               uint8_t *dst);

/* Berlekamp-Welch correction of one byte column (infectious Correct /
 * berlekampWelch, the Decode path for more than k shares): nums[r] share
 * numbers, ys[r] received bytes.  Finds the nearest codeword within
 * floor((r-k)/2) errors (trying 1, 2, ... errors) and writes its value at
 * every share number 0..n-1 to out[n].  Returns the number of corrected
 * symbols, or ORC_ETOO_MANY when none exists (ORC_ENOT_ENOUGH if r - k < 2).
 * Restates the result of infectious's algorithm (a unique nearest codeword);
 * its behaviour for columns it cannot solve is not pinned. */
int orc_bw_column(const uint8_t *enc, int k, int n, const int *nums, const uint8_t *ys, int r,
                  uint8_t *out);

/* Decode with correction: Correct (syndrome + Berlekamp-Welch on every
 * inconsistent column) then Rebuild, for cnt >= k distinct shares. */
int orc_decode_correct(const uint8_t *enc, int k, int n, int *numbers, const uint8_t **shares,
                       int cnt, size_t share_len, uint8_t *dst);

/* infectious invertMatrix (Gauss-Jordan over GF(2^8)), in place. */
int orc_invert(uint8_t *a, int k);

/* z[i] ^= c * x[i]  -- scalar mul_table addmul (infectious generic path). */
void orc_addmul(uint8_t *z, const uint8_t *x, uint8_t c, size_t len);
/* Same result via split-nibble PSHUFB tables (infectious amd64 path as
 * described upstream), AVX2 when available, else scalar. */
void orc_addmul_simd(uint8_t *z, const uint8_t *x, uint8_t c, size_t len);

/* Batched encode for the CPU baseline: stripes of k contiguous shards of S
 * bytes at data + s*k*S; parity at parity + s*m*S.  simd selects addmul
 * flavour; threads > 1 splits stripes across pthreads. Returns ORC_OK. */
int orc_encode_batch(const uint8_t *enc, int k, int n, const uint8_t *data,
                     uint8_t *parity, size_t S, size_t stripes, int simd,
                     int threads);

/* Batched reconstruct for the CPU baseline / checks: stripe s has data at
 * data + s*k*S and parity at parity + s*m*S; erased[s*n + i] != 0 marks
 * shard i as missing.  Every erased shard is regenerated in place via
 * Rebuild's survivor choice + invertMatrix + matrix x stripe.  Returns
 * ORC_OK or the first error. */
int orc_reconstruct_batch(const uint8_t *enc, int k, int n, uint8_t *data, uint8_t *parity,
                          size_t S, size_t stripes, const uint8_t *erased, int simd,
                          int threads);

/* Generic matrix x stripe: out[t] = sum_c coef[t*k+c] * in[c] over S bytes.
 * (Rebuild's inner loop; also used for batched reconstruct checks.) */
void orc_matmul_stripe(const uint8_t *coef, int rows, int k,
                       const uint8_t *const *in, uint8_t *const *out,
                       size_t S, int simd);

/* Splitmix64 synthetic stripe generator (bench / tests): fills len bytes
 * with the byte stream of splitmix64 seeded with seed. */
void orc_fill_splitmix(uint8_t *buf, size_t len, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif
