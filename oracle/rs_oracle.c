/*
 * rs_oracle.c -- CPU restatement of the Reed-Solomon code behind the
 * reference plugin's shard path.  TEST INFRASTRUCTURE ONLY (see rs_oracle.h):
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
 * never by the product library.
 *
 * What it restates and where the reference calls it:
 *   - infectious.NewFEC(k, n)           /root/reference/main.go:73, :248
 *   - (*FEC).Encode(input, output)      /root/reference/main.go:262
 *       (shardInput main.go:243-267: contiguous k-way split, data shares
 *        0..k-1 alias the input, parity k..n-1)
 *   - (*FEC).Decode(nil, shares)        /root/reference/main.go:77
 *       (= Correct + Rebuild; the plugin passes exactly k shares, main.go:65,
 *        for which Correct's syndrome matrix has zero rows)
 *   - infectious.Share{Number, Data}    /root/reference/main.go:57-69, :254-258
 * The algorithm itself lives in the third-party package
 * github.com/vivint/infectious (unpinned, absent from /root/reference): GF(2^8)
 * with polynomial x^8+x^4+x^3+x^2+1 (0x11D) and generator 2, systematic
 * matrix = V[k..n-1] * inverse(V[0..k-1]) with V[r][c] = x_r^c,
 * x_0 = 0, x_r = 2^r (r >= 1).  Parity bytes: "parity unpinned" against
 * upstream (no known-answer vector in the reference).
 */
#include "rs_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

/* ---------------- GF(2^8) tables (infectious gf_exp/gf_log/gf_inverse/
 * gf_mul_table, generated the zfec way from Pp = "101110001") ------------- */
static uint8_t g_exp[510];
static int g_log[256];
static uint8_t g_inv[256];
static uint8_t g_mul[256][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void gf_init(void) {
    const char *pp = "101110001"; /* coefficients of x^0 .. x^8 */
    uint8_t mask = 1;
    g_exp[8] = 0;
    for (int i = 0; i < 8; i++, mask <<= 1) {
        g_exp[i] = mask;
        g_log[g_exp[i]] = i;
        if (pp[i] == '1') g_exp[8] ^= mask;
    }
    g_log[g_exp[8]] = 8;
    mask = 1u << 7;
    for (int i = 9; i < 255; i++) {
        if (g_exp[i - 1] >= mask)
            g_exp[i] = (uint8_t)(g_exp[8] ^ (uint8_t)((g_exp[i - 1] ^ mask) << 1));
        else
            g_exp[i] = (uint8_t)(g_exp[i - 1] << 1);
        g_log[g_exp[i]] = i;
    }
    g_log[0] = 255;
    for (int i = 0; i < 255; i++) g_exp[i + 255] = g_exp[i];
    g_inv[0] = 0;
    g_inv[1] = 1;
    for (int i = 2; i < 256; i++) g_inv[i] = g_exp[255 - g_log[i]];
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            g_mul[a][b] = (a == 0 || b == 0) ? 0 : g_exp[(g_log[a] + g_log[b]) % 255];
}
static inline void gf_ready(void) { pthread_once(&g_once, gf_init); }

uint8_t orc_gf_mul(uint8_t a, uint8_t b) { gf_ready(); return g_mul[a][b]; }
uint8_t orc_gf_inv(uint8_t a) { gf_ready(); return g_inv[a]; }
uint8_t orc_gf_exp(int i) { gf_ready(); return g_exp[((i % 255) + 255) % 255]; }
int orc_gf_log(uint8_t a) { gf_ready(); return g_log[a]; }

/* ---------------- addmul ---------------------------------------------- */
void orc_addmul(uint8_t *z, const uint8_t *x, uint8_t c, size_t len) {
    gf_ready();
    if (c == 0) return; /* infectious skips c == 0 */
    const uint8_t *row = g_mul[c];
    for (size_t i = 0; i < len; i++) z[i] ^= row[x[i]];
}

#if defined(__x86_64__)
__attribute__((target("avx2")))
static void addmul_avx2(uint8_t *z, const uint8_t *x, uint8_t c, size_t len) {
    uint8_t lo[16], hi[16];
    for (int i = 0; i < 16; i++) {
        lo[i] = g_mul[c][i];
        hi[i] = g_mul[c][i << 4];
    }
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)lo));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)hi));
    const __m256i m4 = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= len; i += 32) {
        __m256i v = _mm256_loadu_si256((const __m256i *)(x + i));
        __m256i l = _mm256_and_si256(v, m4);
        __m256i h = _mm256_and_si256(_mm256_srli_epi64(v, 4), m4);
        __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h));
        __m256i o = _mm256_loadu_si256((const __m256i *)(z + i));
        _mm256_storeu_si256((__m256i *)(z + i), _mm256_xor_si256(o, p));
    }
    const uint8_t *row = g_mul[c];
    for (; i < len; i++) z[i] ^= row[x[i]];
}
#endif

void orc_addmul_simd(uint8_t *z, const uint8_t *x, uint8_t c, size_t len) {
    gf_ready();
    if (c == 0) return;
#if defined(__x86_64__)
    if (__builtin_cpu_supports("avx2")) {
        addmul_avx2(z, x, c, len);
        return;
    }
#endif
    orc_addmul(z, x, c, len);
}

/* ---------------- createInvertedVdm (infectious / zfec _invert_vdm) -------
 * Inverse of the k x k Vandermonde V[r][c] = p_r^c, written row-major into
 * vdm (vdm[i*k + j] = inverse[i][j]).  Points p_0 = 0, p_r = 2^(r-1+off). */
static void inverted_vdm(uint8_t *vdm, int k, int off) {
    if (k == 1) {
        vdm[0] = 1;
        return;
    }
    uint8_t *b = calloc((size_t)k, 1), *c = calloc((size_t)k, 1), *p = calloc((size_t)k, 1);
    p[0] = 0;
    for (int r = 1; r < k; r++) p[r] = orc_gf_exp(r - 1 + off);
    /* c = coefficients of P(x) = prod (x - p_i) (leading x^k implicit) */
    c[k - 1] = p[0];
    for (int i = 1; i < k; i++) {
        for (int j = k - 1 - (i - 1); j < k - 1; j++) c[j] ^= g_mul[p[i]][c[j + 1]];
        c[k - 1] ^= p[i];
    }
    for (int row = 0; row < k; row++) {
        uint8_t xx = p[row], t = 1;
        b[k - 1] = 1;
        for (int i = k - 2; i >= 0; i--) {
            b[i] = c[i + 1] ^ g_mul[xx][b[i + 1]];
            t = g_mul[xx][t] ^ b[i];
        }
        for (int col = 0; col < k; col++) vdm[col * k + row] = g_mul[g_inv[t]][b[col]];
    }
    free(b);
    free(c);
    free(p);
}

int orc_fec_matrix(int k, int n, int off, uint8_t *enc) {
    gf_ready();
    if (k <= 0 || n <= 0 || k > 256 || n > 256 || k > n) return ORC_EINVAL_KN;
    uint8_t *tmp = calloc((size_t)n * k, 1);
    inverted_vdm(tmp, k, off);
    /* bottom rows: temp[i] = gf_exp[((i/k)*(i%k)) % 255] (points 2^r) */
    for (int i = k * k; i < n * k; i++) {
        int r = i / k, col = i % k;
        tmp[i] = orc_gf_exp((r - 1 + off) * col);
    }
    memset(enc, 0, (size_t)n * k);
    for (int i = 0; i < k; i++) enc[i * (k + 1)] = 1;
    for (int r = k; r < n; r++)
        for (int col = 0; col < k; col++) {
            uint8_t acc = 0;
            for (int i = 0; i < k; i++) acc ^= g_mul[tmp[r * k + i]][tmp[i * k + col]];
            enc[r * k + col] = acc;
        }
    free(tmp);
    return ORC_OK;
}

int orc_encode(const uint8_t *enc, int k, int n, const uint8_t *input, size_t len,
               uint8_t *parity) {
    gf_ready();
    if (len % (size_t)k != 0) return ORC_ELEN;
    size_t bs = len / (size_t)k;
    for (int i = k; i < n; i++) {
        uint8_t *buf = parity + (size_t)(i - k) * bs;
        memset(buf, 0, bs);
        for (int j = 0; j < k; j++) orc_addmul(buf, input + (size_t)j * bs, enc[i * k + j], bs);
    }
    return ORC_OK;
}

/* ---------------- invertMatrix (zfec _invert_mat restated) -------------- */
int orc_invert(uint8_t *a, int k) {
    gf_ready();
    int *indxc = calloc((size_t)k, sizeof(int)), *indxr = calloc((size_t)k, sizeof(int));
    int *ipiv = calloc((size_t)k, sizeof(int));
    uint8_t *id_row = calloc((size_t)k, 1);
    int rc = ORC_OK;
    for (int col = 0; col < k; col++) {
        int irow = -1, icol = -1;
        if (ipiv[col] != 1 && a[col * k + col] != 0) {
            irow = col;
            icol = col;
        } else {
            for (int row = 0; row < k && irow < 0; row++) {
                if (ipiv[row] == 1) continue;
                for (int ix = 0; ix < k; ix++) {
                    if (ipiv[ix] == 0) {
                        if (a[row * k + ix] != 0) {
                            irow = row;
                            icol = ix;
                            break;
                        }
                    } else if (ipiv[ix] > 1) {
                        rc = ORC_ESINGULAR;
                        goto out;
                    }
                }
            }
        }
        if (irow < 0) {
            rc = ORC_ESINGULAR;
            goto out;
        }
        ipiv[icol]++;
        if (irow != icol)
            for (int ix = 0; ix < k; ix++) {
                uint8_t t = a[irow * k + ix];
                a[irow * k + ix] = a[icol * k + ix];
                a[icol * k + ix] = t;
            }
        indxr[col] = irow;
        indxc[col] = icol;
        uint8_t *pivot_row = a + icol * k;
        uint8_t c = pivot_row[icol];
        if (c == 0) {
            rc = ORC_ESINGULAR;
            goto out;
        }
        if (c != 1) {
            c = g_inv[c];
            pivot_row[icol] = 1;
            for (int ix = 0; ix < k; ix++) pivot_row[ix] = g_mul[c][pivot_row[ix]];
        }
        id_row[icol] = 1;
        if (memcmp(pivot_row, id_row, (size_t)k) != 0) {
            for (int ix = 0; ix < k; ix++) {
                if (ix == icol) continue;
                uint8_t *p = a + ix * k;
                uint8_t cc = p[icol];
                p[icol] = 0;
                orc_addmul(p, pivot_row, cc, (size_t)k);
            }
        }
        id_row[icol] = 0;
    }
    for (int col = k - 1; col >= 0; col--)
        if (indxr[col] != indxc[col])
            for (int row = 0; row < k; row++) {
                uint8_t t = a[row * k + indxr[col]];
                a[row * k + indxr[col]] = a[row * k + indxc[col]];
                a[row * k + indxc[col]] = t;
            }
out:
    free(indxc);
    free(indxr);
    free(ipiv);
    free(id_row);
    return rc;
}

/* ---------------- Decode = Correct (no-op for k shares) + Rebuild -------- */
int orc_decode(const uint8_t *enc, int k, int n, int *numbers, const uint8_t **shares,
               int cnt, size_t share_len, uint8_t *dst) {
    gf_ready();
    if (cnt < k) return ORC_ENOT_ENOUGH;
    if (cnt == 0) return ORC_ENOSHARES;
    /* sort.Sort(byNumber(shares)) -- insertion sort, stable enough here */
    for (int i = 1; i < cnt; i++) {
        int num = numbers[i];
        const uint8_t *sh = shares[i];
        int j = i - 1;
        while (j >= 0 && numbers[j] > num) {
            numbers[j + 1] = numbers[j];
            shares[j + 1] = shares[j];
            j--;
        }
        numbers[j + 1] = num;
        shares[j + 1] = sh;
    }
    /* Correct -> syndromeMatrix counts distinct share numbers ("keepers");
     * with fewer than k distinct shares the k x shareCount Vandermonde cannot
     * be standardized and Decode fails (duplicates never reach Rebuild). */
    {
        uint8_t seen[256] = {0};
        int distinct = 0;
        for (int i = 0; i < cnt; i++) {
            if (numbers[i] < 0 || numbers[i] >= n) return ORC_EBAD_ID;
            if (!seen[numbers[i]]) { seen[numbers[i]] = 1; distinct++; }
        }
        if (distinct < k) return ORC_ESINGULAR;
    }
    uint8_t *m_dec = calloc((size_t)k * k, 1);
    int *indexes = calloc((size_t)k, sizeof(int));
    const uint8_t **sv = calloc((size_t)k, sizeof(*sv));
    int b_iter = 0, e_iter = cnt - 1, rc = ORC_OK;
    for (int i = 0; i < k; i++) {
        int id;
        const uint8_t *d;
        if (numbers[b_iter] == i) {
            id = numbers[b_iter];
            d = shares[b_iter];
            b_iter++;
        } else {
            id = numbers[e_iter];
            d = shares[e_iter];
            e_iter--;
        }
        if (id >= n || id < 0) {
            rc = ORC_EBAD_ID;
            goto out;
        }
        if (id < k) {
            m_dec[i * (k + 1)] = 1;
            memcpy(dst + (size_t)id * share_len, d, share_len);
        } else {
            memcpy(m_dec + (size_t)i * k, enc + (size_t)id * k, (size_t)k);
        }
        sv[i] = d;
        indexes[i] = id;
    }
    rc = orc_invert(m_dec, k);
    if (rc != ORC_OK) goto out;
    for (int i = 0; i < k; i++) {
        if (indexes[i] < k) continue;
        uint8_t *buf = dst + (size_t)i * share_len;
        memset(buf, 0, share_len);
        for (int col = 0; col < k; col++) orc_addmul(buf, sv[col], m_dec[i * k + col], share_len);
    }
out:
    free(m_dec);
    free(indexes);
    free(sv);
    return rc;
}

void orc_matmul_stripe(const uint8_t *coef, int rows, int k, const uint8_t *const *in,
                       uint8_t *const *out, size_t S, int simd) {
    gf_ready();
    for (int t = 0; t < rows; t++) {
        memset(out[t], 0, S);
        for (int c = 0; c < k; c++) {
            if (simd)
                orc_addmul_simd(out[t], in[c], coef[t * k + c], S);
            else
                orc_addmul(out[t], in[c], coef[t * k + c], S);
        }
    }
}

/* ---------------- batched encode (CPU baseline) ------------------------ */
typedef struct {
    const uint8_t *enc, *data;
    uint8_t *parity;
    int k, n, simd;
    size_t S, s0, s1;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *j = arg;
    int m = j->n - j->k;
    const uint8_t *in[256];
    uint8_t *out[256];
    for (size_t s = j->s0; s < j->s1; s++) {
        for (int c = 0; c < j->k; c++) in[c] = j->data + (s * (size_t)j->k + (size_t)c) * j->S;
        for (int t = 0; t < m; t++) out[t] = j->parity + (s * (size_t)m + (size_t)t) * j->S;
        orc_matmul_stripe(j->enc + (size_t)j->k * j->k, m, j->k, in, out, j->S, j->simd);
    }
    return NULL;
}

int orc_encode_batch(const uint8_t *enc, int k, int n, const uint8_t *data, uint8_t *parity,
                     size_t S, size_t stripes, int simd, int threads) {
    gf_ready();
    if (threads < 1) threads = 1;
    if ((size_t)threads > stripes) threads = (int)(stripes ? stripes : 1);
    pthread_t tid[256];
    batch_job jobs[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (batch_job){enc, data, parity, k, n, simd, S,
                              stripes * (size_t)t / (size_t)threads,
                              stripes * (size_t)(t + 1) / (size_t)threads};
        if (threads == 1)
            batch_worker(&jobs[t]);
        else
            pthread_create(&tid[t], NULL, batch_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return ORC_OK;
}

/* ---------------- Correct / Berlekamp-Welch --------------------------- */
/* Codeword symbol i of the systematic code is P(x_i) for the polynomial P
 * (degree < k) through the data symbols, with x_0 = 0, x_i = 2^i: c = E.d =
 * V.(V_t^-1 d).  BW: find Q (deg < k+t) and monic E (deg t) with
 * Q(x_i) = y_i E(x_i) for all received i; then P = Q / E. */
static uint8_t pt_of(int num) { return num == 0 ? 0 : g_exp[num % 255]; }

static uint8_t gpow8(uint8_t x, int e) {
    if (e == 0) return 1;
    if (x == 0) return 0;
    return g_exp[(g_log[x] * e) % 255];
}

/* Solves A (rows x cols+1 augmented, row-major) by Gaussian elimination; on
 * success (consistent) writes one solution (free variables 0) to sol[cols]. */
static int solve_aug(uint8_t *A, int rows, int cols, uint8_t *sol) {
    const int w = cols + 1;
    int *pivcol = malloc(sizeof(int) * (size_t)(rows > 0 ? rows : 1));
    int rank = 0;
    for (int c = 0; c < cols && rank < rows; c++) {
        int p = -1;
        for (int r = rank; r < rows; r++)
            if (A[r * w + c]) { p = r; break; }
        if (p < 0) continue;
        if (p != rank)
            for (int j = 0; j < w; j++) { uint8_t t = A[p * w + j]; A[p * w + j] = A[rank * w + j]; A[rank * w + j] = t; }
        uint8_t inv = g_inv[A[rank * w + c]];
        for (int j = 0; j < w; j++) A[rank * w + j] = g_mul[inv][A[rank * w + j]];
        for (int r = 0; r < rows; r++) {
            if (r == rank || !A[r * w + c]) continue;
            uint8_t f = A[r * w + c];
            for (int j = 0; j < w; j++) A[r * w + j] ^= g_mul[f][A[rank * w + j]];
        }
        pivcol[rank++] = c;
    }
    for (int r = rank; r < rows; r++)
        if (A[r * w + cols]) { free(pivcol); return 0; } /* inconsistent */
    memset(sol, 0, (size_t)cols);
    for (int r = 0; r < rank; r++) sol[pivcol[r]] = A[r * w + cols];
    free(pivcol);
    return 1;
}

int orc_bw_column(const uint8_t *enc, int k, int n, const int *nums, const uint8_t *ys, int r,
                  uint8_t *out) {
    (void)enc;
    gf_ready();
    const int emax = (r - k) / 2;
    if (emax <= 0) return ORC_ENOT_ENOUGH;
    for (int t = 1; t <= emax; t++) {
        const int nq = k + t, cols = nq + t;
        uint8_t *A = calloc((size_t)r * (cols + 1), 1), *u = calloc((size_t)cols, 1);
        for (int i = 0; i < r; i++) {
            const uint8_t x = pt_of(nums[i]), y = ys[i];
            uint8_t *row = A + (size_t)i * (cols + 1);
            for (int j = 0; j < nq; j++) row[j] = gpow8(x, j);
            for (int l = 0; l < t; l++) row[nq + l] = g_mul[y][gpow8(x, l)];
            row[cols] = g_mul[y][gpow8(x, t)];
        }
        int ok = solve_aug(A, r, cols, u);
        if (ok) {
            /* Q(x) = sum q_j x^j (q = u[0..nq)), E(x) = x^t + sum e_l x^l */
            uint8_t *q = malloc((size_t)nq), *e = malloc((size_t)t + 1);
            memcpy(q, u, (size_t)nq);
            for (int l = 0; l < t; l++) e[l] = u[nq + l];
            e[t] = 1;
            /* P = Q / E (long division, E monic) */
            uint8_t *pp = calloc((size_t)k, 1);
            for (int d = nq - 1; d >= t; d--) {
                const uint8_t c = q[d];
                pp[d - t] = c;
                if (c)
                    for (int l = 0; l <= t; l++) q[d - t + l] ^= g_mul[c][e[l]];
            }
            for (int d = 0; d < t; d++) if (q[d]) ok = 0; /* remainder */
            if (ok) {
                int bad = 0;
                for (int i = 0; i < r; i++) {
                    uint8_t x = pt_of(nums[i]), v = 0;
                    for (int d = k - 1; d >= 0; d--) v = g_mul[v][x] ^ pp[d];
                    if (v != ys[i]) bad++;
                }
                if (bad > t) ok = 0;
                else {
                    for (int i = 0; i < n; i++) {
                        uint8_t x = pt_of(i), v = 0;
                        for (int d = k - 1; d >= 0; d--) v = g_mul[v][x] ^ pp[d];
                        out[i] = v;
                    }
                    free(q); free(e); free(pp); free(A); free(u);
                    return bad;
                }
            }
            free(q); free(e); free(pp);
        }
        free(A);
        free(u);
    }
    return ORC_ETOO_MANY;
}

int orc_decode_correct(const uint8_t *enc, int k, int n, int *numbers, const uint8_t **shares,
                       int cnt, size_t S, uint8_t *dst) {
    gf_ready();
    if (cnt < k) return ORC_ENOT_ENOUGH;
    for (int i = 0; i < cnt; i++)
        if (numbers[i] < 0 || numbers[i] >= n) return ORC_EBAD_ID;
    /* sort by number */
    for (int i = 1; i < cnt; i++) {
        int num = numbers[i];
        const uint8_t *sh = shares[i];
        int j = i - 1;
        while (j >= 0 && numbers[j] > num) { numbers[j + 1] = numbers[j]; shares[j + 1] = shares[j]; j--; }
        numbers[j + 1] = num;
        shares[j + 1] = sh;
    }
    /* private copies, corrected in place (infectious mutates the shares) */
    uint8_t **cp = malloc(sizeof(uint8_t *) * (size_t)cnt);
    for (int i = 0; i < cnt; i++) { cp[i] = malloc(S ? S : 1); memcpy(cp[i], shares[i], S); }
    int rc = ORC_OK;
    if (cnt > k) {
        /* consistency: every share must equal enc[num] . data, data being
         * the codeword through the first k shares */
        int *kn = malloc(sizeof(int) * (size_t)k);
        const uint8_t **kp = malloc(sizeof(*kp) * (size_t)k);
        uint8_t *d = malloc((size_t)k * (S ? S : 1));
        for (int i = 0; i < k; i++) { kn[i] = numbers[i]; kp[i] = cp[i]; }
        rc = orc_decode(enc, k, n, kn, kp, k, S, d);
        uint8_t *ys = malloc((size_t)cnt), *outv = malloc((size_t)n);
        for (size_t col = 0; col < S && rc == ORC_OK; col++) {
            int consistent = 1;
            for (int i = k; i < cnt && consistent; i++) {
                uint8_t v = 0;
                for (int j = 0; j < k; j++) v ^= g_mul[enc[numbers[i] * k + j]][d[(size_t)j * S + col]];
                if (v != cp[i][col]) consistent = 0;
            }
            if (consistent) continue;
            for (int i = 0; i < cnt; i++) ys[i] = cp[i][col];
            int c = orc_bw_column(enc, k, n, numbers, ys, cnt, outv);
            if (c < 0) { rc = c; break; }
            for (int i = 0; i < cnt; i++) cp[i][col] = outv[numbers[i]];
        }
        free(kn); free(kp); free(d); free(ys); free(outv);
    }
    if (rc == ORC_OK) rc = orc_decode(enc, k, n, numbers, (const uint8_t **)cp, cnt, S, dst);
    for (int i = 0; i < cnt; i++) free(cp[i]);
    free(cp);
    return rc;
}

/* ---------------- batched reconstruct (CPU baseline) ------------------ */
typedef struct {
    const uint8_t *enc, *erased;
    uint8_t *data, *parity;
    int k, n, simd, rc;
    size_t S, s0, s1;
} rec_job;

static void *rec_worker(void *arg) {
    rec_job *j = arg;
    const int k = j->k, n = j->n, m = n - k;
    uint8_t *shard[256];
    const uint8_t *in[256];
    uint8_t *out[256];
    uint8_t *M = malloc((size_t)k * k), *rows = malloc((size_t)m * k);
    int surv[256], lost[256];
    for (size_t s = j->s0; s < j->s1 && j->rc == ORC_OK; s++) {
        const uint8_t *er = j->erased + s * (size_t)n;
        for (int i = 0; i < k; i++) shard[i] = j->data + (s * (size_t)k + (size_t)i) * j->S;
        for (int i = 0; i < m; i++) shard[k + i] = j->parity + (s * (size_t)m + (size_t)i) * j->S;
        int e = 0;
        for (int i = 0; i < n; i++)
            if (er[i]) lost[e++] = i;
        if (e == 0) continue;
        if (e > m) { j->rc = ORC_ENOT_ENOUGH; break; }
        /* Rebuild's choice: slot i takes shard i if present, else the
         * highest-numbered remaining present shard. */
        int hi = n - 1, used[256] = {0};
        for (int i = 0; i < k; i++) {
            if (!er[i]) { surv[i] = i; used[i] = 1; continue; }
            while (er[hi] || used[hi]) hi--;
            surv[i] = hi;
            used[hi] = 1;
        }
        for (int i = 0; i < k; i++) memcpy(M + (size_t)i * k, j->enc + (size_t)surv[i] * k, (size_t)k);
        if (orc_invert(M, k) != ORC_OK) { j->rc = ORC_ESINGULAR; break; }
        for (int t = 0; t < e; t++)
            for (int c = 0; c < k; c++) {
                uint8_t acc = 0;
                for (int i = 0; i < k; i++) acc ^= g_mul[j->enc[(size_t)lost[t] * k + i]][M[i * k + c]];
                rows[t * k + c] = acc;
            }
        for (int i = 0; i < k; i++) in[i] = shard[surv[i]];
        for (int t = 0; t < e; t++) out[t] = shard[lost[t]];
        orc_matmul_stripe(rows, e, k, in, out, j->S, j->simd);
    }
    free(M);
    free(rows);
    return NULL;
}

int orc_reconstruct_batch(const uint8_t *enc, int k, int n, uint8_t *data, uint8_t *parity,
                          size_t S, size_t stripes, const uint8_t *erased, int simd,
                          int threads) {
    gf_ready();
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if ((size_t)threads > stripes) threads = (int)(stripes ? stripes : 1);
    pthread_t tid[256];
    rec_job jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (rec_job){enc, erased, data, parity, k, n, simd, ORC_OK, S,
                            stripes * (size_t)t / (size_t)threads,
                            stripes * (size_t)(t + 1) / (size_t)threads};
        if (threads == 1)
            rec_worker(&jobs[t]);
        else
            pthread_create(&tid[t], NULL, rec_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    for (int t = 0; t < threads; t++)
        if (jobs[t].rc != ORC_OK) return jobs[t].rc;
    return ORC_OK;
}

/* ---------------- synthetic data ------------------------------------- */
static inline uint64_t splitmix_at(uint64_t seed, uint64_t q) {
    uint64_t z = seed + (q + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_fill_splitmix(uint8_t *buf, size_t len, uint64_t seed) {
    size_t q = 0;
    for (; (q + 1) * 8 <= len; q++) {
        uint64_t v = splitmix_at(seed, q);
        memcpy(buf + q * 8, &v, 8);
    }
    if (q * 8 < len) {
        uint64_t v = splitmix_at(seed, q);
        memcpy(buf + q * 8, &v, len - q * 8);
    }
}
