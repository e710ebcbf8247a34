/*
 * bed_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's BED-decode / standardize / subset arithmetic,
 * used as the parity checker for the HIP product path (libsnpmi.so) and as the
 * `cpu_baseline` ("port") leg of bench.py.  Nothing under pysnptools_amd/ may link,
 * load or call this file; the product path has no CPU fallback.
 *
 * Where the algorithm lives:
 *   The reference (PySnpTools 0.5.10) delegates the native arithmetic of this path to the
 *   third-party Rust package `bed-reader` (constraint `bed-reader>=0.2.36`, setup.py:26,
 *   requirements.txt:10), which is NOT vendored in /root/reference and is not installed.
 *   Its published algorithm is restated here from the reference's call sites:
 *     decode      bed.py:337-343   (open_bed.read(index=(iid_idx,sid_idx), order, dtype))
 *     standardize standardizer.py:90-133 (standardize_f32/f64(val,is_beta,a,b,apply,use_stats,stats))
 *     subset      util/__init__.py:271-393 (subset_f64_f64 / subset_f32_f64 / subset_f32_f32)
 *   and pinned (tests/test_oracle.py) against the reference's own fixtures:
 *     tests/datasets/all_chr.maf0.001.N300.pst.npz   (decoded matrix, bit-exact)
 *     pysnptools/examples/toydata10.snp.npz          (first 10 SNPs of toydata, bit-exact)
 *     pysnptools/examples/toydata.kernel.npz         (Unit GRM of toydata)
 *     the standardizer.py:37-42 doctest digits       (one-pass stats, f64)
 *   and against golden vectors produced by running the reference's Python path
 *   (tools/make_golden.py, force_python_only=True).
 *
 * Semantics:
 *   .bed = 3-byte magic 6C 1B 01, then SNP-major columns of ceil(N/4) bytes.
 *   code(i) = (b[i>>2] >> 2*(i&3)) & 3
 *   count_A1=False: {0:0, 1:missing, 2:1, 3:2};  count_A1=True: {0:2, 1:missing, 2:1, 3:0}
 *   missing = NaN (float) or -127 (int8)   (bed.py:54-56, test.py:288-295)
 *   one-pass stats: mean = S1/n, std = sqrt(S2/n - mean*mean), std <= 0 (or NaN with n>0)
 *     -> +inf; n == 0 -> mean = std = NaN.  Pinned for f64 bit-exactly by the doctest digits
 *     standardizer.py:41-42 (0.23354968324845735); the NaN rule is the Python path's
 *     behaviour (standardizer.py:150-157; bed-reader would raise NoIndividuals).
 *   Unit apply: x = (x - mean) / std, NaN -> 0                  (standardizer.py:160-163)
 *   Beta apply: maf = mean/2, folded to <= .5, w = BetaPDF(maf;a,b) (f64),
 *               x = (x - mean) * w, NaN -> 0, use_stats & std==inf -> 0 (standardizer.py:199-211)
 *   Precision rule (both dtypes): stats and the apply arithmetic run in f64 and are rounded
 *   once to T.  For f64 this IS the one-pass formula above.  For f32, evaluating the
 *   one-pass formula in f32 arithmetic (var = S2/n - mean^2 cancels) misses the 1e-5
 *   relative bar against the reference Python path (measured 1.47e-5 on N300), so the
 *   f32 result is the f64 result rounded once -- within 1 ulp of exact.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#pragma STDC FP_CONTRACT OFF

static int set_threads(int num_threads) {
#ifdef _OPENMP
    if (num_threads > 0) omp_set_num_threads(num_threads);
    return omp_get_max_threads();
#else
    (void)num_threads;
    return 1;
#endif
}

int oracle_max_threads(void) { return set_threads(0); }

/* value of a 2-bit code; returns 0..2 or -1 for missing (bed.py:337-343 via bed-reader) */
static inline int code_value(int code, int count_a1) {
    static const int lut_a2[4] = {0, -1, 1, 2};
    static const int lut_a1[4] = {2, -1, 1, 0};
    return count_a1 ? lut_a1[code] : lut_a2[code];
}

static inline int code_at(const uint8_t* col, uint64_t iid) {
    return (col[iid >> 2] >> (2 * (iid & 3))) & 3;
}

#define DEFINE_DECODE(NAME, T, MISSING)                                                        \
    int NAME(const uint8_t* body, uint64_t n_iid, uint64_t n_sid, int count_a1,                \
             const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,             \
             uint64_t n_out_sid, int order_c, T* out, int num_threads) {                       \
        uint64_t bpc = (n_iid + 3) / 4;                                                       \
        set_threads(num_threads);                                                              \
        for (uint64_t r = 0; r < n_out_iid; r++)                                               \
            if (iid_idx[r] >= n_iid) return 1;                                                 \
        for (uint64_t j = 0; j < n_out_sid; j++)                                               \
            if (sid_idx[j] >= n_sid) return 2;                                                 \
        _Pragma("omp parallel for schedule(static)")                                           \
        for (int64_t j = 0; j < (int64_t)n_out_sid; j++) {                                     \
            const uint8_t* col = body + sid_idx[j] * bpc;                                      \
            for (uint64_t r = 0; r < n_out_iid; r++) {                                         \
                int v = code_value(code_at(col, iid_idx[r]), count_a1);                        \
                T x = v < 0 ? (T)(MISSING) : (T)v;                                             \
                if (order_c) out[r * n_out_sid + j] = x;                                       \
                else out[j * n_out_iid + r] = x;                                               \
            }                                                                                  \
        }                                                                                      \
        return 0;                                                                              \
    }

DEFINE_DECODE(oracle_decode_f64, double, NAN)
DEFINE_DECODE(oracle_decode_f32, float, NAN)
DEFINE_DECODE(oracle_decode_i8, int8_t, -127)

/* Beta(a,b) density in f64: the weight of standardizer.py:204-205 (scipy.stats.beta.pdf) */
double oracle_beta_pdf(double x, double a, double b) {
    if (!(x >= 0.0 && x <= 1.0)) return 0.0;
    double lbeta = lgamma(a) + lgamma(b) - lgamma(a + b);
    return pow(x, a - 1.0) * pow(1.0 - x, b - 1.0) / exp(lbeta);
}

/* One-pass stats from sums (n, S1, S2); f64 arithmetic for every dtype (see header). */
static void stats_from_sums(double n, double s1, double s2, double* mean, double* std) {
    if (n == 0) {
        *mean = NAN;
        *std = NAN;
        return;
    }
    double m = s1 / n;
    double var = s2 / n - m * m;
    double sd = sqrt(var);
    if (!(sd > 0)) sd = INFINITY;
    *mean = m;
    *std = sd;
}

/* Per-SNP apply as a function of one observed value v (NaN -> 0), rounded once to T. */
static double apply_value(double v, double mean, double std, int is_beta, double w, int zero_col) {
    if (v != v || zero_col) return 0.0;
    return is_beta ? (v - mean) * w : (v - mean) / std;
}

static double beta_weight(double mean, double a, double b) {
    double maf = mean / 2.0;
    if (maf > 0.5) maf = 1.0 - maf;
    return oracle_beta_pdf(maf, a, b);
}

/* Per-column standardize, in place.  stats is C-order [cols][2] (mean, std). */
#define DEFINE_STANDARDIZE(NAME, T)                                                            \
    int NAME(T* val, uint64_t rows, uint64_t cols, int order_c, int is_beta, double a,         \
             double b, int use_stats, T* stats, int num_threads) {                             \
        set_threads(num_threads);                                                              \
        _Pragma("omp parallel for schedule(dynamic, 16)")                                      \
        for (int64_t j = 0; j < (int64_t)cols; j++) {                                          \
            uint64_t rs = order_c ? cols : 1, base = order_c ? (uint64_t)j : (uint64_t)j * rows;\
            double mean, std;                                                                  \
            if (use_stats) {                                                                   \
                mean = (double)stats[2 * j];                                                   \
                std = (double)stats[2 * j + 1];                                                \
            } else {                                                                           \
                double n = 0, s1 = 0, s2 = 0;                                                  \
                for (uint64_t r = 0; r < rows; r++) {                                          \
                    T x = val[base + r * rs];                                                  \
                    if (x == x) { n += 1; s1 += (double)x; s2 += (double)x * (double)x; }     \
                }                                                                              \
                stats_from_sums(n, s1, s2, &mean, &std);                                       \
                stats[2 * j] = (T)mean;                                                        \
                stats[2 * j + 1] = (T)std;                                                     \
            }                                                                                  \
            double w = is_beta ? beta_weight(mean, a, b) : 0.0;                                \
            int zero_col = is_beta && use_stats && isinf(std);                                 \
            for (uint64_t r = 0; r < rows; r++) {                                              \
                T* px = &val[base + r * rs];                                                   \
                *px = (T)apply_value((double)*px, mean, std, is_beta, w, zero_col);            \
            }                                                                                  \
        }                                                                                      \
        return 0;                                                                              \
    }

DEFINE_STANDARDIZE(oracle_standardize_f64, double)
DEFINE_STANDARDIZE(oracle_standardize_f32, float)

/*
 * Fused decode + one-pass standardize straight from the packed bytes (the composition
 * Bed.read().standardize() runs natively: bed.py:337-343 then standardizer.py:114/120).
 * Stats come from integer code counts, which equal the dtype sums exactly (values are
 * 0/1/2), so this is bit-identical to decode followed by oracle_standardize_*.
 * This is the CPU baseline timed by bench.py.
 */
#define DEFINE_DECODE_STD(NAME, T)                                                             \
    int NAME(const uint8_t* body, uint64_t n_iid, uint64_t n_sid, int count_a1,                \
             const uint64_t* sid_idx, uint64_t n_out_sid, int is_beta, double a, double b,     \
             T* out, T* stats, int num_threads) {                                              \
        uint64_t bpc = (n_iid + 3) / 4;                                                       \
        set_threads(num_threads);                                                              \
        _Pragma("omp parallel for schedule(dynamic, 4)")                                       \
        for (int64_t j = 0; j < (int64_t)n_out_sid; j++) {                                     \
            const uint8_t* col = body + sid_idx[j] * bpc;                                      \
            uint64_t cnt[4] = {0, 0, 0, 0};                                                    \
            for (uint64_t i = 0; i < n_iid; i++) cnt[code_at(col, i)]++;                       \
            uint64_t c_hi = count_a1 ? cnt[0] : cnt[3];                                        \
            double mean, std;                                                                  \
            stats_from_sums((double)(n_iid - cnt[1]), (double)(cnt[2] + 2 * c_hi),             \
                            (double)(cnt[2] + 4 * c_hi), &mean, &std);                         \
            stats[2 * j] = (T)mean;                                                            \
            stats[2 * j + 1] = (T)std;                                                         \
            double w = is_beta ? beta_weight(mean, a, b) : 0.0;                                \
            T lut[4];                                                                          \
            for (int c = 0; c < 4; c++) {                                                      \
                int v = code_value(c, count_a1);                                               \
                lut[c] = (T)apply_value(v < 0 ? NAN : (double)v, mean, std, is_beta, w, 0);    \
            }                                                                                  \
            T* o = out + (uint64_t)j * n_iid;                                                  \
            for (uint64_t i = 0; i < n_iid; i++) o[i] = lut[code_at(col, i)];                  \
        }                                                                                      \
        return 0;                                                                              \
    }

DEFINE_DECODE_STD(oracle_decode_standardize_f64, double)
DEFINE_DECODE_STD(oracle_decode_standardize_f32, float)

/* sub_matrix gather (util/__init__.py:271-393): out[i,j,k] = val[row[i], col[j], k]. */
#define DEFINE_SUBSET(NAME, S, D)                                                              \
    int NAME(const S* val, uint64_t r, uint64_t c, uint64_t k, int in_order_c,                 \
             const uint64_t* ri, uint64_t nr, const uint64_t* ci, uint64_t nc, int out_order_c,\
             D* out) {                                                                         \
        for (uint64_t i = 0; i < nr; i++) if (ri[i] >= r) return 1;                            \
        for (uint64_t j = 0; j < nc; j++) if (ci[j] >= c) return 2;                            \
        for (uint64_t i = 0; i < nr; i++)                                                      \
            for (uint64_t j = 0; j < nc; j++)                                                  \
                for (uint64_t q = 0; q < k; q++) {                                             \
                    uint64_t src = in_order_c ? (ri[i] * c + ci[j]) * k + q                    \
                                              : ri[i] + r * (ci[j] + c * q);                   \
                    uint64_t dst = out_order_c ? (i * nc + j) * k + q : i + nr * (j + nc * q); \
                    out[dst] = (D)val[src];                                                    \
                }                                                                              \
        return 0;                                                                              \
    }

DEFINE_SUBSET(oracle_subset_f64_f64, double, double)
DEFINE_SUBSET(oracle_subset_f32_f64, float, double)
DEFINE_SUBSET(oracle_subset_f32_f32, float, float)

/*
 * Synthetic BED generator restatement (CPU twin of the device generator in
 * pysnptools_amd/csrc/synth.hip).  Counter-based so any column can be regenerated
 * independently: genotype of (sid, iid) = f(splitmix64(seed, sid, iid)).
 * MAF per SNP is drawn from the SnpGen curve (snpreader/snpgen.py:140-151), passed in
 * as a 100-point table (x, cdf).
 */
static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

uint32_t oracle_synth_thresholds(uint64_t seed, uint64_t sid, const double* maf_x,
                                 const double* maf_cdf, int n_pts, double miss_rate,
                                 uint32_t* thr /* [3]: t2, t1, tmiss */) {
    uint64_t h = splitmix64(seed * 0xD1B54A32D192ED03ull ^ (sid + 1) * 0x8CB92BA72F3D8DD7ull);
    double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
    int k = 0;
    while (k < n_pts - 1 && u > maf_cdf[k]) k++;
    double maf = maf_x[k];
    double p2 = maf * maf, p1 = 2.0 * maf * (1.0 - maf);
    double s = 4294967296.0;
    double t2 = p2 * s, t12 = (p2 + p1) * s, tm = miss_rate * s;
    thr[0] = t2 >= s ? 0xFFFFFFFFu : (uint32_t)t2;
    thr[1] = t12 >= s ? 0xFFFFFFFFu : (uint32_t)t12;
    thr[2] = tm >= s ? 0xFFFFFFFFu : (uint32_t)tm;
    return (uint32_t)k;
}

static inline int synth_code(uint64_t seed, uint64_t sid, uint64_t iid, const uint32_t* thr) {
    uint64_t h = splitmix64((seed + 0x632BE59BD9B4E019ull) ^ (sid * 0x9E6C63D0676A9A99ull) ^
                            (iid * 0xC2B2AE3D27D4EB4Full));
    uint32_t ug = (uint32_t)h, um = (uint32_t)(h >> 32);
    if (um < thr[2]) return 1;       /* missing */
    if (ug < thr[0]) return 3;       /* value 2 (count_A1=False) */
    if (ug < thr[1]) return 2;       /* value 1 */
    return 0;                        /* value 0 */
}

/* writes n_sid columns of pitch bytes each (pitch >= ceil(n_iid/4)); pad bits are 0 */
int oracle_synth_bed(uint64_t seed, uint64_t n_iid, uint64_t sid0, uint64_t n_sid, uint64_t pitch,
                     const double* maf_x, const double* maf_cdf, int n_pts, double miss_rate,
                     uint8_t* out, int num_threads) {
    uint64_t bpc = (n_iid + 3) / 4;
    if (pitch < bpc) return 1;
    set_threads(num_threads);
    _Pragma("omp parallel for schedule(static)")
    for (int64_t j = 0; j < (int64_t)n_sid; j++) {
        uint32_t thr[3];
        uint64_t sid = sid0 + (uint64_t)j;
        oracle_synth_thresholds(seed, sid, maf_x, maf_cdf, n_pts, miss_rate, thr);
        uint8_t* col = out + (uint64_t)j * pitch;
        memset(col, 0, pitch);
        for (uint64_t i = 0; i < n_iid; i++)
            col[i >> 2] |= (uint8_t)(synth_code(seed, sid, i, thr) << (2 * (i & 3)));
    }
    return 0;
}

/* Per-SNP code counts (c0, c1=missing, c2, c3) over all iids, and the one-pass stats they give
 * (same formula as above; f64).  Lets a checker get the stats of a wide matrix without
 * materialising the decoded values. */
/* byte_code_count[b][c]: how many of the 4 two-bit codes packed in byte b equal c */
static uint8_t byte_code_count[256][4];
static void init_byte_code_count(void) {
    for (int b = 0; b < 256; b++)
        for (int k = 0; k < 4; k++) byte_code_count[b][(b >> (2 * k)) & 3]++;
}
__attribute__((constructor)) static void oracle_init(void) { init_byte_code_count(); }

int oracle_snp_stats(const uint8_t* body, uint64_t n_iid, uint64_t n_sid, int count_a1, double* stats,
                     int num_threads) {
    uint64_t bpc = (n_iid + 3) / 4;
    set_threads(num_threads);
    _Pragma("omp parallel for schedule(dynamic, 4)")
    for (int64_t j = 0; j < (int64_t)n_sid; j++) {
        const uint8_t* col = body + (uint64_t)j * bpc;
        uint64_t cnt[4] = {0, 0, 0, 0};
        /* whole bytes through a table of per-byte code counts, then the iids of a partial last byte */
        const uint64_t full = n_iid / 4;
        for (uint64_t q = 0; q < full; q++)
            for (int c = 0; c < 4; c++) cnt[c] += byte_code_count[col[q]][c];
        for (uint64_t i = full * 4; i < n_iid; i++) cnt[code_at(col, i)]++;
        uint64_t c_hi = count_a1 ? cnt[0] : cnt[3];
        stats_from_sums((double)(n_iid - cnt[1]), (double)(cnt[2] + 2 * c_hi), (double)(cnt[2] + 4 * c_hi),
                        &stats[2 * j], &stats[2 * j + 1]);
    }
    return 0;
}
