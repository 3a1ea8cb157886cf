// gf256.hpp -- host-side GF(2^8) algebra of the engine: field tables, the
// systematic encode matrix (what infectious.NewFEC builds, main.go:73/:248)
// and the decode-matrix construction of (*FEC).Rebuild (main.go:77).
//
// This is the product's own implementation (generic Gauss-Jordan over the
// full Vandermonde matrix); the restatement of infectious's polynomial
// inverted-VDM algorithm lives in oracle/ and is only used to check it.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace rsmi {

constexpr uint32_t kPoly = 0x11D;  // x^8 + x^4 + x^3 + x^2 + 1, generator 2

struct Field {
    uint8_t exp[512];
    uint8_t log[256];
    uint8_t inv[256];
    uint8_t mul[256][256];
    Field();
};

const Field& field();

inline uint8_t gmul(uint8_t a, uint8_t b) { return field().mul[a][b]; }

// Evaluation point of row r of the Vandermonde matrix: 0 for r = 0, 2^r else.
uint8_t eval_point(int r);

// n x k row-major systematic matrix: top k rows identity, bottom rows
// V[k..n-1] * inverse(V[0..k-1]), V[r][c] = eval_point(r)^c.
std::vector<uint8_t> systematic_matrix(int k, int n);

// In-place inverse of a k x k matrix; false if singular.
bool invert(uint8_t* a, int k);

// Rebuild's survivor choice (infectious Rebuild, restated in oracle/):
// slot i takes share i if present, otherwise the highest-numbered remaining
// share.  present[n] flags; returns the k chosen shard ids in slot order, or
// an empty vector when fewer than k are present.
std::vector<int> choose_survivors(const uint8_t* present, int k, int n);
// The same into out[k] (no allocation); returns k, or 0 when fewer than k
// are present.  n <= 256.
int choose_survivors_into(const uint8_t* present, int k, int n, int* out);

// Decode rows for a set of survivors: for every shard id in `targets`, the
// row d such that shard[target] = sum_c d[c] * shard[survivors[c]].
// Returns false if the survivor submatrix is singular.
bool decode_rows(const std::vector<uint8_t>& enc, int k, int n,
                 const std::vector<int>& survivors, const std::vector<int>& targets,
                 std::vector<uint8_t>& rows_out);

// Berlekamp-Welch on one byte column (infectious Correct): nums[r] share
// numbers with received bytes ys[r].  Finds the nearest codeword within
// floor((r-k)/2) errors and writes its symbol for every share number to
// out[n]; returns the number of received symbols it disagrees with, or -1 if
// there is no such codeword.  Codeword symbol i is P(x_i) for a polynomial P
// of degree < k, x_0 = 0, x_i = 2^i (the systematic code's evaluation view).
int bw_column(int k, int n, const int* nums, const uint8_t* ys, int r, uint8_t* out);

// Split-table words for one coefficient c, as the HIP kernels consume them
// with v_perm_b32: w[0..1] = c*{0..7}, w[2..3] = c*{0,8,..,56},
// w[4] = c*{0,64,128,192} (byte i of each word = entry i).
void coef_tables(uint8_t c, uint32_t w[5]);

}  // namespace rsmi
