// gf256.cpp -- see gf256.hpp.
#include "gf256.hpp"

#include <cstring>

namespace rsmi {

Field::Field() {
    // exp[i] = 2^i by repeated doubling modulo the polynomial.
    uint32_t x = 1;
    for (int i = 0; i < 255; ++i) {
        exp[i] = static_cast<uint8_t>(x);
        exp[i + 255] = static_cast<uint8_t>(x);
        log[x] = static_cast<uint8_t>(i);
        x <<= 1;
        if (x & 0x100) x ^= kPoly;
    }
    exp[510] = exp[0];
    exp[511] = exp[1];
    log[0] = 0;  // unused: 0 has no logarithm
    inv[0] = 0;
    for (int a = 1; a < 256; ++a) inv[a] = exp[255 - log[a]];
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            mul[a][b] = (a && b) ? exp[log[a] + log[b]] : 0;
}

const Field& field() {
    static const Field f;
    return f;
}

uint8_t eval_point(int r) { return r == 0 ? 0 : field().exp[r % 255]; }

static uint8_t gpow(uint8_t x, int e) {
    if (e == 0) return 1;
    if (x == 0) return 0;
    const Field& f = field();
    return f.exp[(f.log[x] * e) % 255];
}

bool invert(uint8_t* a, int k) {
    // Gauss-Jordan on [A | I] with row pivoting.
    const Field& f = field();
    std::vector<uint8_t> aug(static_cast<size_t>(k) * 2 * k, 0);
    const int w = 2 * k;
    for (int r = 0; r < k; ++r) {
        std::memcpy(&aug[r * w], a + r * k, k);
        aug[r * w + k + r] = 1;
    }
    for (int col = 0; col < k; ++col) {
        int piv = -1;
        for (int r = col; r < k; ++r)
            if (aug[r * w + col]) { piv = r; break; }
        if (piv < 0) return false;
        if (piv != col)
            for (int c = 0; c < w; ++c) std::swap(aug[piv * w + c], aug[col * w + c]);
        const uint8_t s = f.inv[aug[col * w + col]];
        for (int c = 0; c < w; ++c) aug[col * w + c] = f.mul[s][aug[col * w + c]];
        for (int r = 0; r < k; ++r) {
            if (r == col) continue;
            const uint8_t fac = aug[r * w + col];
            if (!fac) continue;
            for (int c = 0; c < w; ++c) aug[r * w + c] ^= f.mul[fac][aug[col * w + c]];
        }
    }
    for (int r = 0; r < k; ++r) std::memcpy(a + r * k, &aug[r * w + k], k);
    return true;
}

std::vector<uint8_t> systematic_matrix(int k, int n) {
    const Field& f = field();
    std::vector<uint8_t> V(static_cast<size_t>(n) * k);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) V[r * k + c] = gpow(eval_point(r), c);
    std::vector<uint8_t> top(V.begin(), V.begin() + static_cast<size_t>(k) * k);
    invert(top.data(), k);  // Vandermonde with distinct points: never singular
    std::vector<uint8_t> E(static_cast<size_t>(n) * k, 0);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (int i = 0; i < k; ++i) acc ^= f.mul[V[r * k + i]][top[i * k + c]];
            E[r * k + c] = acc;
        }
    // The top block is exactly the identity by construction; pin it.
    for (int r = 0; r < k; ++r)
        for (int c = 0; c < k; ++c) E[r * k + c] = (r == c);
    return E;
}

int choose_survivors_into(const uint8_t* present, int k, int n, int* out) {
    int avail = 0;
    for (int i = 0; i < n; ++i) avail += present[i] ? 1 : 0;
    if (avail < k) return 0;
    uint8_t used[256] = {};
    int hi = n - 1;
    for (int i = 0; i < k; ++i) {
        if (present[i] && !used[i]) {
            out[i] = i;
            used[i] = 1;
            continue;
        }
        while (hi >= 0 && (!present[hi] || used[hi])) --hi;
        out[i] = hi;
        used[hi] = 1;
    }
    return k;
}

std::vector<int> choose_survivors(const uint8_t* present, int k, int n) {
    std::vector<int> out(static_cast<size_t>(k));
    out.resize(static_cast<size_t>(choose_survivors_into(present, k, n, out.data())));
    return out;
}

// Rebuild-shaped survivor sets (every present data shard in its own slot,
// the d erased data slots filled by parity shares): the rows follow from the
// d x d inverse of B = enc[parity survivors][erased data] -- the same
// construction as the GPU kernel (gf_invert.hip) and the same bytes as the
// full inverse, which is unique.  Returns false if surv has another shape.
static bool decode_rows_structured(const std::vector<uint8_t>& enc, int k, const std::vector<int>& surv,
                                   const std::vector<int>& targets, std::vector<uint8_t>& rows, bool* singular) {
    const Field& f = field();
    std::vector<int> D, pos(k, -1);  // erased data slots; slot -> index in D
    for (int i = 0; i < k; ++i) {
        if (surv[i] == i) continue;
        if (surv[i] < k) return false;
        pos[i] = static_cast<int>(D.size());
        D.push_back(i);
    }
    const int d = static_cast<int>(D.size());
    std::vector<uint8_t> B(static_cast<size_t>(d) * d);
    for (int a = 0; a < d; ++a)
        for (int b = 0; b < d; ++b) B[a * d + b] = enc[static_cast<size_t>(surv[D[a]]) * k + D[b]];
    if (d > 0 && !invert(B.data(), d)) {
        *singular = true;
        return true;
    }
    // G[b][j]: erased data D_b as a combination of the survivor slots
    std::vector<uint8_t> G(static_cast<size_t>(d) * k, 0);
    for (int b = 0; b < d; ++b)
        for (int j = 0; j < k; ++j) {
            if (pos[j] >= 0) {
                G[b * k + j] = B[b * d + pos[j]];
                continue;
            }
            uint8_t acc = 0;
            for (int a = 0; a < d; ++a) acc ^= f.mul[B[b * d + a]][enc[static_cast<size_t>(surv[D[a]]) * k + j]];
            G[b * k + j] = acc;
        }
    rows.assign(targets.size() * static_cast<size_t>(k), 0);
    for (size_t t = 0; t < targets.size(); ++t) {
        const int id = targets[t];
        uint8_t* row = &rows[t * k];
        if (id < k) {
            if (pos[id] >= 0) std::memcpy(row, &G[static_cast<size_t>(pos[id]) * k], k);
            else row[id] = 1;  // present in its own slot
            continue;
        }
        const uint8_t* e = &enc[static_cast<size_t>(id) * k];
        for (int j = 0; j < k; ++j) row[j] = pos[j] < 0 ? e[j] : 0;
        for (int b = 0; b < d; ++b) {
            const uint8_t c = e[D[b]];
            if (!c) continue;
            for (int j = 0; j < k; ++j) row[j] ^= f.mul[c][G[b * k + j]];
        }
    }
    return true;
}

bool decode_rows(const std::vector<uint8_t>& enc, int k, int n, const std::vector<int>& surv,
                 const std::vector<int>& targets, std::vector<uint8_t>& rows) {
    (void)n;
    bool singular = false;
    if (decode_rows_structured(enc, k, surv, targets, rows, &singular)) return !singular;
    const Field& f = field();
    std::vector<uint8_t> M(static_cast<size_t>(k) * k);
    for (int i = 0; i < k; ++i) std::memcpy(&M[i * k], &enc[static_cast<size_t>(surv[i]) * k], k);
    if (!invert(M.data(), k)) return false;
    // shard[t] = enc[t] . data = enc[t] . (M^-1 . survivors)
    rows.assign(targets.size() * static_cast<size_t>(k), 0);
    for (size_t t = 0; t < targets.size(); ++t) {
        const uint8_t* e = &enc[static_cast<size_t>(targets[t]) * k];
        for (int c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (int i = 0; i < k; ++i) acc ^= f.mul[e[i]][M[i * k + c]];
            rows[t * k + c] = acc;
        }
    }
    return true;
}

int bw_column(int k, int n, const int* nums, const uint8_t* ys, int r, uint8_t* out) {
    const Field& f = field();
    for (int t = 1; 2 * t <= r - k; ++t) {
        // Unknowns: Q's k+t coefficients, E's t low coefficients (E monic).
        // Row i: sum_j q_j x^j + y sum_l e_l x^l = y x^t   (char 2)
        const int nq = k + t, cols = nq + t, w = cols + 1;
        std::vector<uint8_t> A(static_cast<size_t>(r) * w);
        for (int i = 0; i < r; ++i) {
            const uint8_t x = eval_point(nums[i]), y = ys[i];
            uint8_t* row = &A[static_cast<size_t>(i) * w];
            uint8_t xp = 1;
            for (int j = 0; j < nq; ++j) {
                row[j] = xp;
                if (j < t) row[nq + j] = f.mul[y][xp];
                if (j == t) row[cols] = f.mul[y][xp];
                xp = f.mul[xp][x];
            }
            if (t >= nq) row[cols] = f.mul[y][gpow(x, t)];
        }
        // reduced row echelon form
        std::vector<int> pivcol;
        int rank = 0;
        for (int col = 0; col < cols && rank < r; ++col) {
            int p = -1;
            for (int i = rank; i < r; ++i)
                if (A[static_cast<size_t>(i) * w + col]) { p = i; break; }
            if (p < 0) continue;
            if (p != rank)
                for (int j = 0; j < w; ++j) std::swap(A[static_cast<size_t>(p) * w + j], A[static_cast<size_t>(rank) * w + j]);
            uint8_t* pr = &A[static_cast<size_t>(rank) * w];
            const uint8_t inv = f.inv[pr[col]];
            for (int j = 0; j < w; ++j) pr[j] = f.mul[inv][pr[j]];
            for (int i = 0; i < r; ++i) {
                uint8_t* ri = &A[static_cast<size_t>(i) * w];
                if (i == rank || !ri[col]) continue;
                const uint8_t fac = ri[col];
                for (int j = 0; j < w; ++j) ri[j] ^= f.mul[fac][pr[j]];
            }
            pivcol.push_back(col);
            ++rank;
        }
        bool consistent = true;
        for (int i = rank; i < r && consistent; ++i)
            if (A[static_cast<size_t>(i) * w + cols]) consistent = false;
        if (!consistent) continue;
        std::vector<uint8_t> u(cols, 0);  // one solution, free variables 0
        for (int i = 0; i < rank; ++i) u[pivcol[i]] = A[static_cast<size_t>(i) * w + cols];
        // P = Q / E by long division (E monic, degree t)
        std::vector<uint8_t> q(u.begin(), u.begin() + nq), e(t + 1), p(k, 0);
        for (int l = 0; l < t; ++l) e[l] = u[nq + l];
        e[t] = 1;
        for (int d = nq - 1; d >= t; --d) {
            const uint8_t cf = q[d];
            p[d - t] = cf;
            if (cf)
                for (int l = 0; l <= t; ++l) q[d - t + l] ^= f.mul[cf][e[l]];
        }
        bool rem = false;
        for (int d = 0; d < t; ++d) rem |= q[d] != 0;
        if (rem) continue;
        auto eval = [&](uint8_t x) {
            uint8_t v = 0;
            for (int d = k - 1; d >= 0; --d) v = f.mul[v][x] ^ p[d];
            return v;
        };
        int bad = 0;
        for (int i = 0; i < r; ++i) bad += eval(eval_point(nums[i])) != ys[i];
        if (bad > t) continue;
        for (int i = 0; i < n; ++i) out[i] = eval(eval_point(i));
        return bad;
    }
    return -1;
}

void coef_tables(uint8_t c, uint32_t w[5]) {
    const Field& f = field();
    auto pack = [&](int base, int step, int count) {
        uint32_t v = 0;
        for (int i = 0; i < count; ++i) v |= uint32_t(f.mul[c][(base + i * step) & 0xff]) << (8 * i);
        return v;
    };
    w[0] = pack(0, 1, 4);
    w[1] = pack(4, 1, 4);
    w[2] = pack(0, 8, 4);
    w[3] = pack(32, 8, 4);
    w[4] = pack(0, 64, 4);
}

}  // namespace rsmi
