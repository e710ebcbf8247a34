// Memory-bound kernels of the BED path (gfx950):
//   k_snp_stats      packed codes -> per-SNP counts -> stats + 4-entry value LUT
//   k_decode_f/_c    packed codes + LUT -> values (F or C order)
//   k_repack         iid gather of packed columns (arbitrary iid index lists)
//   k_std_dense_*    standardize an arbitrary float matrix in place (SnpData.standardize)
//   k_subset         sub_matrix gather (util/__init__.py:271-393)
//   k_grm_extract    upper-triangle GRM tiles -> K[ri, ci] (symmetric mirror + scale)
//   k_synth          counter-based synthetic genotypes
// Reference semantics: SURVEY.md Appendix B; bed-reader call sites bed.py:337-343,
// standardizer.py:90-211.  Built with -ffp-contract=off: the stats/LUT arithmetic is f64,
// rounded once to the output dtype, and must not be contracted into FMAs.
#include "snpmi_internal.hpp"

namespace snpmi {
namespace {

constexpr int kWave = 64;
constexpr int kBlock = 256;

__device__ __forceinline__ double stats_mean_std(double n, double s1, double s2, double* sd_out) {
    if (n == 0.0) {
        *sd_out = __builtin_nan("");
        return __builtin_nan("");
    }
    double m = s1 / n;
    double var = s2 / n - m * m;
    double sd = sqrt(var);
    if (!(sd > 0.0)) sd = __builtin_inf();
    *sd_out = sd;
    return m;
}

// Beta(a,b) density at the folded MAF (standardizer.py:199-205); f64.
__device__ __forceinline__ double beta_weight(double mean, double a, double b) {
    double maf = mean / 2.0;
    if (maf > 0.5) maf = 1.0 - maf;
    if (!(maf >= 0.0 && maf <= 1.0)) return 0.0;
    double lbeta = lgamma(a) + lgamma(b) - lgamma(a + b);
    return pow(maf, a - 1.0) * pow(1.0 - maf, b - 1.0) / exp(lbeta);
}

// The same function behind a call: in k_std_cols_f it runs once per column on one thread, and
// inlined its lgamma / pow would set the register count of the whole kernel (~35 VGPRs more,
// which the column-in-registers path cannot spare).  Same code, so the same bits.
__device__ __attribute__((noinline)) double beta_weight_call(double mean, double a, double b) {
    return beta_weight(mean, a, b);
}

// value of code c (count_A1 selects the A1 LUT); -1 = missing
__device__ __forceinline__ int code_value(int c, int count_a1) {
    // count_A1=False {0,-,1,2}; count_A1=True {2,-,1,0}
    if (c == 1) return -1;
    int v = (c == 0) ? 0 : (c == 2 ? 1 : 2);
    return count_a1 ? 2 - v : v;
}

template <typename T>
__device__ __forceinline__ T lut_missing() { return (T)__builtin_nan(""); }
template <>
__device__ __forceinline__ int8_t lut_missing<int8_t>() { return (int8_t)-127; }

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// ------------------------------------------------------------------ per-SNP stats + LUT
// W waves per SNP column, 4/W SNPs per 256-thread block; 16-byte loads (64 iids per
// lane-load), 4 in flight per lane.  W = 1 for short columns; W = 4 for long ones,
// where one wave per SNP left 2 waves per SIMD streaming 125 KB columns (latency-bound).
template <typename T, int W, int U = 8>
__global__ __launch_bounds__(kBlock) void k_snp_stats(const uint8_t* __restrict__ packed, uint64_t pitch,
                                                      uint64_t n, uint64_t m, int count_a1, int std_kind,
                                                      double a, double b, int use_stats, T* __restrict__ stats,
                                                      T* __restrict__ lut) {
    constexpr int kS = kBlock / kWave / W;  // SNPs per block
    __shared__ uint32_t red[kBlock / kWave][3];
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave, sub = wave % W;
    const uint64_t s = (uint64_t)blockIdx.x * kS + wave / W;
    const bool valid = s < m;
    if (W == 1 && !valid) return;
    if (std_kind == SNPMI_STD_NONE) {
        if (valid && sub == 0 && lane < 4) {
            int v = code_value(lane, count_a1);
            lut[4 * s + lane] = v < 0 ? lut_missing<T>() : (T)v;
        }
        return;  // block-uniform (std_kind): no barrier below is skipped by part of the block
    }
    double mean, sd;
    if (use_stats) {
        if (!valid || sub != 0) return;  // block-uniform branch (use_stats); no barrier follows
        mean = (double)stats[2 * s];
        sd = (double)stats[2 * s + 1];
    } else {
        uint32_t c1 = 0, c2 = 0, c3 = 0;
        if (valid) {
            const uint4* col = reinterpret_cast<const uint4*>(packed + s * pitch);
            // per 32-bit word (16 codes; bit 0 of a code = lo, bit 1 = hi): lo-count, hi-count
            // and both-count (code 3); code 1 (missing) = lo - both, code 2 = hi - both.  7 VALU
            // per word (the kernel was VALU-co-bound at 13 with a per-word tail test)
            uint32_t clo = 0, chi = 0;
            auto count_word = [&](uint32_t x) {
                clo += __popc(x & 0x55555555u);
                chi += __popc(x & 0xAAAAAAAAu);
                c3 += __popc(x & (x >> 1) & 0x55555555u);
            };
            auto count16 = [&](const uint4& v) {
                count_word(v.x);
                count_word(v.y);
                count_word(v.z);
                count_word(v.w);
            };
            const uint64_t nfull = n / 64;  // 16-B items of 64 iids, all inside the column
            constexpr uint64_t step = (uint64_t)W * kWave;
            uint64_t q = (uint64_t)sub * kWave + lane;
            for (; q + (U - 1) * step < nfull; q += U * step) {  // U independent 16-B loads in flight
                uint4 v[U];
#pragma unroll
                for (int u = 0; u < U; u++) v[u] = col[q + u * step];
#pragma unroll
                for (int u = 0; u < U; u++) count16(v[u]);
            }
            for (; q < nfull; q += step) count16(col[q]);
            if (q == nfull && n % 64) {  // the column's last, partial item: codes of iids >= n masked off
                const uint4 v = col[q];
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint64_t ib = q * 64 + 16 * k;
                    const uint64_t valid_i = n > ib ? min<uint64_t>(n - ib, 16) : 0;
                    const uint32_t mk = valid_i >= 16 ? 0xffffffffu : ((1u << (2 * valid_i)) - 1u);
                    count_word(w4[k] & mk);
                }
            }
            c1 = clo - c3;
            c2 = chi - c3;
        }
        c1 = wave_sum_u32(c1);
        c2 = wave_sum_u32(c2);
        c3 = wave_sum_u32(c3);
        if constexpr (W > 1) {
            if (lane == 0) {
                red[wave][0] = c1;
                red[wave][1] = c2;
                red[wave][2] = c3;
            }
            __syncthreads();
            if (!valid || sub != 0) return;
#pragma unroll
            for (int w = 1; w < W; w++) {
                c1 += red[wave + w][0];
                c2 += red[wave + w][1];
                c3 += red[wave + w][2];
            }
        }
        uint64_t c0 = n - c1 - c2 - c3;
        uint64_t chi = count_a1 ? c0 : c3;  // count of value 2
        double nobs = (double)(n - c1);
        mean = stats_mean_std(nobs, (double)(c2 + 2 * chi), (double)(c2 + 4 * chi), &sd);
        if (lane == 0) {
            stats[2 * s] = (T)mean;
            stats[2 * s + 1] = (T)sd;
        }
    }
    if (lane < 4) {
        double w = std_kind == SNPMI_STD_BETA ? beta_weight(mean, a, b) : 0.0;
        bool zero_col = std_kind == SNPMI_STD_BETA && use_stats && __builtin_isinf(sd);
        int v = code_value(lane, count_a1);
        double x;
        if (v < 0 || zero_col) x = 0.0;
        else if (std_kind == SNPMI_STD_BETA) x = ((double)v - mean) * w;
        else x = ((double)v - mean) / sd;
        lut[4 * s + lane] = (T)x;
    }
}

// ------------------------------------------------------------------ decode, F order
// 4-entry LUT select, written so hipcc emits three v_cndmask (no divergent branches:
// the nested-ternary form compiled to exec-mask branches around every element).
template <typename T>
__device__ __forceinline__ T sel4(T l0, T l1, T l2, T l3, uint32_t c) {
    const bool b0 = (c & 1u) != 0, b1 = (c & 2u) != 0;
    const T lo = b0 ? l1 : l0;
    const T hi = b0 ? l3 : l2;
    return b1 ? hi : lo;
}

// Wave work item = (column j, chunk of 1024 iids).  Each lane loads one dword (16 iids);
// codes are redistributed with ds_bpermute (__shfl) so every store instruction writes 1 KiB
// contiguous (f32: 4 rounds of 16-B stores; f64: 8 rounds; i8: one 16-B store per lane).
// U items per wave per iteration with all U loads issued first (memory-level parallelism);
// stores are non-temporal (write-once stream).  Measured on MI355X (tools/ubench.py):
// U=4 + nt + 8 blocks per 4 waves of work-cap -> 5.2 TB/s vs 3.6 TB/s for U=1, plain stores.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef double f64x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <typename V>
__device__ __forceinline__ void store_nt(V* p, const V& v) {
    __builtin_nontemporal_store(v, p);
}
// XCD-sliced item order: the grid is a multiple of 8 and block b works as logical block
// (b mod 8) G/8 + b/8, so each XCD writes a contiguous 1/8 of every grid pass
template <typename T, int U>
__global__ __launch_bounds__(kBlock) void k_decode_f(const uint8_t* __restrict__ packed, uint64_t pitch, uint64_t n,
                                                     uint64_t m, const T* __restrict__ lut, T* __restrict__ out,
                                                     uint64_t ld) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t chunks = (n + 1023) / 1024;
    const uint64_t total = chunks * m;
    const uint64_t groups = (total + U - 1) / U;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / kWave);
    const uint64_t lb = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    for (uint64_t gi = lb * (kBlock / kWave) + threadIdx.x / kWave; gi < groups; gi += nwaves) {
        uint32_t w[U];
        uint64_t jv[U], cv[U];
        bool val[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t it = gi * U + u;
            const uint64_t j = it / chunks, c = it - j * chunks;
            jv[u] = j;
            cv[u] = c;
            val[u] = it < total;  // wave-uniform
            const bool ok = val[u] && (c * 1024 + 16 * (uint64_t)lane < n);
            w[u] = ok ? reinterpret_cast<const uint32_t*>(packed + j * pitch)[c * 64 + lane] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (!val[u]) continue;
            const uint64_t j = jv[u], i0 = cv[u] * 1024;
            const T l0 = lut[4 * j], l1 = lut[4 * j + 1], l2 = lut[4 * j + 2], l3 = lut[4 * j + 3];
            T* o = out + j * ld + i0;
            if constexpr (sizeof(T) == 4) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const uint32_t src = __shfl(w[u], r * 16 + (lane >> 2), kWave);
                    const uint32_t byte = (src >> (8 * (lane & 3))) & 0xffu;
                    const uint64_t i = i0 + r * 256 + 4 * lane;
                    f32x4_t v;
                    v.x = sel4(l0, l1, l2, l3, byte & 3u);
                    v.y = sel4(l0, l1, l2, l3, (byte >> 2) & 3u);
                    v.z = sel4(l0, l1, l2, l3, (byte >> 4) & 3u);
                    v.w = sel4(l0, l1, l2, l3, byte >> 6);
                    if (i + 4 <= n) {
                        store_nt(reinterpret_cast<f32x4_t*>(o + r * 256 + 4 * lane), v);
                    } else {
                        for (int t = 0; t < 4; t++)
                            if (i + t < n) o[r * 256 + 4 * lane + t] = v[t];
                    }
                }
            } else if constexpr (sizeof(T) == 8) {
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const uint32_t src = __shfl(w[u], r * 8 + (lane >> 3), kWave);
                    const uint32_t byte = (src >> (8 * ((lane >> 1) & 3))) & 0xffu;
                    const uint32_t sh = 4 * (lane & 1);
                    const uint64_t i = i0 + r * 128 + 2 * lane;
                    f64x2_t v;
                    v.x = sel4(l0, l1, l2, l3, (byte >> sh) & 3u);
                    v.y = sel4(l0, l1, l2, l3, (byte >> (sh + 2)) & 3u);
                    if (i + 2 <= n) {
                        store_nt(reinterpret_cast<f64x2_t*>(o + r * 128 + 2 * lane), v);
                    } else if (i < n) {
                        o[r * 128 + 2 * lane] = v.x;
                    }
                }
            } else {
                // int8: lane writes 16 bytes for its own dword; byte LUT via v_perm_b32
                const uint32_t lw = (uint32_t)(uint8_t)l0 | ((uint32_t)(uint8_t)l1 << 8) |
                                    ((uint32_t)(uint8_t)l2 << 16) | ((uint32_t)(uint8_t)l3 << 24);
                u32x4_t q;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t bb = (w[u] >> (8 * k)) & 0xffu;
                    const uint32_t selb = (bb & 3u) | ((bb & 0xCu) << 6) | ((bb & 0x30u) << 12) | ((bb & 0xC0u) << 18);
                    q[k] = __builtin_amdgcn_perm(0u, lw, selb);
                }
                const uint64_t i = i0 + 16 * lane;
                if (i + 16 <= n) {
                    store_nt(reinterpret_cast<u32x4_t*>(o + 16 * lane), q);
                } else if (i < n) {
                    for (uint64_t t = 0; i + t < n; t++)
                        reinterpret_cast<uint8_t*>(o)[16 * lane + t] = (uint8_t)(q[t >> 2] >> (8 * (t & 3)));
                }
            }
        }
    }
}


// Fused stats + decode, one workgroup per SNP column (large N): pass 1 counts the codes
// (packed column read once from HBM), the LUT is built in f64 by one lane, pass 2 re-reads
// the column (L2 / Infinity-Cache resident) and streams the values out with non-temporal
// 16-B stores.  Saves the separate k_snp_stats launch and its HBM read.
template <int U>
__global__ __launch_bounds__(kBlock) void k_decode_std_col_f32(const uint8_t* __restrict__ packed, uint64_t pitch,
                                                               uint64_t n, int count_a1, int std_kind, double a,
                                                               double b, int use_stats, float* __restrict__ stats,
                                                               float* __restrict__ lut_out, float* __restrict__ out,
                                                               uint64_t ld) {
    __shared__ uint32_t red[3][kBlock / kWave];
    __shared__ float lutsh[4];
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    const uint64_t j = blockIdx.x;
    const uint8_t* colp = packed + j * pitch;
    if (std_kind == SNPMI_STD_NONE) {
        if (threadIdx.x < 4) {
            int v = code_value(threadIdx.x, count_a1);
            lutsh[threadIdx.x] = v < 0 ? __builtin_nanf("") : (float)v;
        }
    } else {
        double mean = 0, sd = 0;
        if (!use_stats) {
            const uint4* col = reinterpret_cast<const uint4*>(colp);
            const uint64_t nq = (n + 63) / 64;
            uint32_t c1 = 0, c2 = 0, c3 = 0;
            for (uint64_t q0 = threadIdx.x; q0 < nq; q0 += kBlock * 4) {
                uint4 vv[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint64_t q = q0 + (uint64_t)u * kBlock;
                    vv[u] = q < nq ? col[q] : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint64_t q = q0 + (uint64_t)u * kBlock;
                    uint32_t w4[4] = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        uint32_t w = w4[k];
                        uint32_t lo = w & 0x55555555u, hi = (w >> 1) & 0x55555555u;
                        const uint64_t ib = q * 64 + 16 * k;
                        if (ib + 16 > n) {
                            const uint64_t valid = n > ib ? n - ib : 0;
                            const uint32_t mk = valid >= 16 ? 0xFFFFFFFFu : (((1u << (2 * valid)) - 1u) & 0x55555555u);
                            lo &= mk;
                            hi &= mk;
                        }
                        c3 += __popc(lo & hi);
                        c2 += __popc(hi & ~lo);
                        c1 += __popc(lo & ~hi);
                    }
                }
            }
            c1 = wave_sum_u32(c1);
            c2 = wave_sum_u32(c2);
            c3 = wave_sum_u32(c3);
            if (lane == 0) {
                red[0][wave] = c1;
                red[1][wave] = c2;
                red[2][wave] = c3;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                uint64_t t1 = 0, t2 = 0, t3 = 0;
                for (int q = 0; q < kBlock / kWave; q++) {
                    t1 += red[0][q];
                    t2 += red[1][q];
                    t3 += red[2][q];
                }
                const uint64_t c0 = n - t1 - t2 - t3, chi = count_a1 ? c0 : t3;
                mean = stats_mean_std((double)(n - t1), (double)(t2 + 2 * chi), (double)(t2 + 4 * chi), &sd);
                stats[2 * j] = (float)mean;
                stats[2 * j + 1] = (float)sd;
            }
        } else if (threadIdx.x == 0) {
            mean = (double)stats[2 * j];
            sd = (double)stats[2 * j + 1];
        }
        if (threadIdx.x == 0) {
            const double w = std_kind == SNPMI_STD_BETA ? beta_weight(mean, a, b) : 0.0;
            const bool zero_col = std_kind == SNPMI_STD_BETA && use_stats && __builtin_isinf(sd);
            for (int c = 0; c < 4; c++) {
                const int v = code_value(c, count_a1);
                double x;
                if (v < 0 || zero_col) x = 0.0;
                else if (std_kind == SNPMI_STD_BETA) x = ((double)v - mean) * w;
                else x = ((double)v - mean) / sd;
                lutsh[c] = (float)x;
            }
        }
    }
    __syncthreads();
    const float l0 = lutsh[0], l1 = lutsh[1], l2 = lutsh[2], l3 = lutsh[3];
    if (threadIdx.x < 4 && lut_out) lut_out[4 * j + threadIdx.x] = lutsh[threadIdx.x];
    const uint64_t chunks = (n + 1023) / 1024;
    const uint32_t* col = reinterpret_cast<const uint32_t*>(colp);
    float* ocol = out + j * ld;
    for (uint64_t c0 = (uint64_t)wave * U; c0 < chunks; c0 += (uint64_t)(kBlock / kWave) * U) {
        uint32_t w[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t c = c0 + u;
            w[u] = (c < chunks && c * 1024 + 16 * (uint64_t)lane < n) ? col[c * 64 + lane] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t c = c0 + u;
            if (c >= chunks) break;
            const uint64_t i0 = c * 1024;
            float* o = ocol + i0;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const uint32_t src = __shfl(w[u], r * 16 + (lane >> 2), kWave);
                const uint32_t byte = (src >> (8 * (lane & 3))) & 0xffu;
                const uint64_t i = i0 + r * 256 + 4 * lane;
                f32x4_t v;
                v.x = sel4(l0, l1, l2, l3, byte & 3u);
                v.y = sel4(l0, l1, l2, l3, (byte >> 2) & 3u);
                v.z = sel4(l0, l1, l2, l3, (byte >> 4) & 3u);
                v.w = sel4(l0, l1, l2, l3, byte >> 6);
                if (i + 4 <= n) {
                    __builtin_nontemporal_store(v, reinterpret_cast<f32x4_t*>(o + r * 256 + 4 * lane));
                } else {
                    for (int t = 0; t < 4; t++)
                        if (i + t < n) o[r * 256 + 4 * lane + t] = v[t];
                }
            }
        }
    }
}

// ------------------------------------------------------------------ decode, C order
// Tile = 64 SNPs x 64 iids staged in LDS, rows written SNP-fastest.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_decode_c(const uint8_t* __restrict__ packed, uint64_t pitch, uint64_t n,
                                                     uint64_t m, const T* __restrict__ lut, T* __restrict__ out,
                                                     uint64_t ld) {
    __shared__ uint32_t sh[64][5];
    __shared__ T shl[64][4];
    const int t = threadIdx.x;
    const uint64_t tiles_i = (n + 63) / 64, tiles_j = (m + 63) / 64;
    const uint64_t nwords = (n + 15) / 16;
    for (uint64_t tile = blockIdx.x; tile < tiles_i * tiles_j; tile += gridDim.x) {
        const uint64_t tj = tile / tiles_i, ti = tile - tj * tiles_i;
        const uint64_t i0 = ti * 64, j0 = tj * 64;
        {
            const int cj = t >> 2, dw = t & 3;
            uint32_t w = 0;
            if (j0 + cj < m && i0 / 16 + dw < nwords)
                w = reinterpret_cast<const uint32_t*>(packed + (j0 + cj) * pitch)[i0 / 16 + dw];
            sh[cj][dw] = w;
            if (t < 64 && j0 + t < m) {
#pragma unroll
                for (int k = 0; k < 4; k++) shl[t][k] = lut[4 * (j0 + t) + k];
            }
        }
        __syncthreads();
        const int jj = t & 63, r0 = t >> 6;
        if (j0 + jj < m) {
#pragma unroll 4
            for (int q = 0; q < 16; q++) {
                const int r = r0 + 4 * q;
                if (i0 + r < n) {
                    uint32_t code = (sh[jj][r >> 4] >> (2 * (r & 15))) & 3u;
                    out[(i0 + r) * ld + j0 + jj] = shl[jj][code];
                }
            }
        }
        __syncthreads();
    }
}

// C order, register-resident codes: one wave per tile of 256 iids x (64*V) SNPs (V = 16 bytes /
// sizeof(T): 4 f32 or 2 f64 SNPs per lane).  Each lane loads the 64-byte code segments of its
// V SNPs (256 iids each) into registers, then walks the 256 rows: per row it extracts V codes
// and writes one 16-byte vector, so every store instruction of the wave covers 1 KiB of one
// output row.  No LDS, no barriers.  Needs ld % V == 0 (16-B aligned rows).
template <typename T, bool ROWMAJOR = false>
__global__ __launch_bounds__(kBlock) void k_decode_c_reg(const uint8_t* __restrict__ packed, uint64_t pitch,
                                                         uint64_t n, uint64_t m, const T* __restrict__ lut,
                                                         T* __restrict__ out, uint64_t ld) {
    constexpr int V = 16 / sizeof(T);
    typedef T vec_t __attribute__((ext_vector_type(V)));
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t ti_n = (n + 255) / 256, tj_n = (m + 64 * V - 1) / (64 * V);
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / kWave);
    for (uint64_t it = (uint64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave; it < ti_n * tj_n; it += nwaves) {
        // ROWMAJOR: consecutive waves take neighbouring SNP ranges of the same 256 rows, so the
        // stores in flight cover whole output rows (DRAM page locality) instead of 1 KiB pieces
        // of many rows
        const uint64_t tj = ROWMAJOR ? it % tj_n : it / ti_n, ti = ROWMAJOR ? it / tj_n : it - tj * ti_n;
        const uint64_t i0 = ti * 256, jl = tj * 64 * V + (uint64_t)V * lane;
        uint32_t w[V][16];
        T l[V][4];
#pragma unroll
        for (int v = 0; v < V; v++) {
            const uint64_t j = jl + v;
            if (j < m) {
                const u32x4_t* c = reinterpret_cast<const u32x4_t*>(packed + j * pitch + i0 / 4);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const u32x4_t x = c[q];  // pitch % 64 == 0: the 64 bytes are inside the column
                    w[v][4 * q] = x[0], w[v][4 * q + 1] = x[1], w[v][4 * q + 2] = x[2], w[v][4 * q + 3] = x[3];
                }
#pragma unroll
                for (int k = 0; k < 4; k++) l[v][k] = lut[4 * j + k];
            } else {
#pragma unroll
                for (int q = 0; q < 16; q++) w[v][q] = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) l[v][k] = (T)0;
            }
        }
        const bool full = jl + V <= m;
        const uint64_t rows = n - i0 < 256 ? n - i0 : 256;
        // q fully unrolled (w[v][q] stays in registers), e rolled up to 4 (a fully unrolled
        // 256-row nest made the compiler index w dynamically -- 272 B/lane of scratch)
#pragma unroll
        for (int q = 0; q < 16; q++) {
#pragma unroll 4
            for (int e = 0; e < 16; e++) {
                const uint64_t r = 16 * q + e;
                if (r < rows) {
                    vec_t o;
#pragma unroll
                    for (int v = 0; v < V; v++) o[v] = sel4(l[v][0], l[v][1], l[v][2], l[v][3], (w[v][q] >> (2 * e)) & 3u);
                    T* dst = out + (i0 + r) * ld + jl;
                    if (full) {
                        store_nt(reinterpret_cast<vec_t*>(dst), o);
                    } else {
#pragma unroll
                        for (int v = 0; v < V; v++)
                            if (jl + v < m) dst[v] = o[v];
                    }
                }
            }
        }
    }
}

// ------------------------------------------------------------------ iid gather (repack)
__global__ __launch_bounds__(kBlock) void k_repack(const uint8_t* __restrict__ src, uint64_t sp,
                                                   const uint64_t* __restrict__ idx, uint64_t n_out, uint64_t m,
                                                   uint8_t* __restrict__ dst, uint64_t dp) {
    const uint64_t nd = (n_out + 15) / 16;
    const uint64_t total = nd * m;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t j = t / nd, d = t - j * nd;
        const uint8_t* col = src + j * sp;
        uint32_t w = 0;
#pragma unroll 4
        for (int k = 0; k < 16; k++) {
            const uint64_t r = 16 * d + k;
            if (r < n_out) {
                const uint64_t i = idx[r];
                w |= (uint32_t)((col[i >> 2] >> (2 * (i & 3))) & 3u) << (2 * k);
            }
        }
        reinterpret_cast<uint32_t*>(dst + j * dp)[d] = w;
    }
}

// iid gather with the source columns staged in LDS.  One 1024-thread workgroup walks groups of
// K SNP columns (K = 4 / 2 / 1 as K columns fit in 150 KiB of LDS), the columns of a group
// interleaved by dword (LDS dword w*K + c = dword w of column c), so ONE plan entry serves all
// K columns: a ds_read_b32/b64/b128 returns the dword holding the source code in every column.
// The plan (k_repack_plan, once per call) is one u32 per output code: LDS byte address << 5 |
// bit offset of the code in its dword, so a code costs one LDS read + v_bfe + v_lshl_or; output
// codes past n_out point at a zero dword behind the columns.  The next group's columns are
// loaded into registers while the current group gathers (global latency under LDS work), and
// every dword of the destination pitch is written (no separate memset).  k_repack (global
// gathers) is the fallback for columns over 150 KiB.
constexpr uint64_t kRepackLds = 150 * 1024;
// u32x4 of each column of the next group held per thread: ceil(150 KiB / 16 B / K / 1024) for K = 1, 2, 4
constexpr int kRepackPre[3] = {10, 5, 3};

__host__ __device__ inline int repack_k(uint64_t nq) {
    const uint64_t bytes = nq * 16;
    return 4 * bytes + 16 <= kRepackLds ? 4 : 2 * bytes + 16 <= kRepackLds ? 2 : 1;
}

constexpr uint64_t kRepackChunk = 8192;  // default output codes per windowed workgroup (512 words)

// win == nullptr: absolute LDS addresses (whole columns, zero dword behind them at u32x4 nq);
// else per kRepackChunk-code output chunk c the source window starts at u32x4 win[c] and the zero
// dword sits behind the widest window (u32x4 zq)
__global__ void k_repack_plan(const uint64_t* __restrict__ idx, uint64_t n_out, uint64_t n_pad, uint64_t zq, int K,
                              const uint32_t* __restrict__ win, uint64_t chunk, uint32_t* __restrict__ plan) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_pad; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = r < n_out ? idx[r] : 0;
        const uint64_t base = win ? 4ull * win[r / chunk] : 0;
        const uint64_t w = r < n_out ? (i >> 4) - base : 4 * zq;
        plan[r] = (uint32_t)(((w * K * 4) << 5) | ((i & 15) << 1));
    }
}

// source window of each kRepackChunk-code output chunk: lohi[2c] = min, lohi[2c+1] = max of its
// source iids (u32 atomics; lohi preset to {~0, 0} per chunk), 2048 codes per workgroup
__global__ __launch_bounds__(256) void k_repack_window(const uint64_t* __restrict__ idx, uint64_t n_out,
                                                       uint64_t chunk, uint32_t* __restrict__ lohi) {
    const uint64_t r0 = (uint64_t)blockIdx.x * 2048;
    uint32_t lo = ~0u, hi = 0;
    for (uint64_t r = r0 + threadIdx.x; r < min(r0 + 2048, n_out); r += 256) {
        const uint32_t i = (uint32_t)idx[r];
        lo = min(lo, i);
        hi = max(hi, i);
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
    }
    if ((threadIdx.x & 63) == 0 && r0 < n_out) {
        const uint64_t c = r0 / chunk;
        atomicMin(lohi + 2 * c, lo);
        atomicMax(lohi + 2 * c + 1, hi);
    }
}

// Windowed gather for index lists with locality (sorted, reversed, strided subsets -- what
// intersect_apply produces when the iid orders agree): a 256-thread workgroup (chunk c, group g)
// stages only the source window of output chunk c (512 words) for K columns, K x window <= 40
// KiB so four workgroups share a CU and one's loads overlap the others' gathers; sources are read
// once and each plan entry serves K columns.
template <int K>
__global__ __launch_bounds__(256) void k_repack_win(const uint8_t* __restrict__ src, uint64_t sp, uint64_t nq,
                                                    uint64_t zq, uint64_t nchunks, uint64_t chunk_words, uint64_t m,
                                                    const uint32_t* __restrict__ win,
                                                    const uint32_t* __restrict__ plan, uint64_t n_out,
                                                    uint8_t* __restrict__ dst, uint64_t dp) {
    extern __shared__ u32x4_t colw[];
    typedef uint32_t vk_t __attribute__((ext_vector_type(K)));
    const int t = threadIdx.x;
    const uint64_t c = blockIdx.x % nchunks, g = blockIdx.x / nchunks;
    const uint64_t lo4 = win[c], n4 = min(zq, nq - lo4);
    uint32_t* l = reinterpret_cast<uint32_t*>(colw);
    for (uint64_t q = t; q < n4; q += 256) {
        u32x4_t v[K];
#pragma unroll
        for (int cc = 0; cc < K; cc++) {
            const uint64_t j = g * K + cc;
            v[cc] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(src + (j < m ? j : m - 1) * sp) + lo4 + q);
        }
        if constexpr (K == 1) {
            colw[q] = v[0];
        } else {
#pragma unroll
            for (int e = 0; e < 4; e++) {
                vk_t x;
#pragma unroll
                for (int cc = 0; cc < K; cc++) x[cc] = v[cc][e];
                *reinterpret_cast<vk_t*>(l + (4 * q + e) * K) = x;
            }
        }
    }
    if (t < K) l[4 * zq * K + t] = 0;
    __syncthreads();
    const uint64_t nd = (n_out + 15) / 16, ndp = dp / 4;
    const uint64_t d0 = c * chunk_words, d1 = c + 1 == nchunks ? ndp : min(d0 + chunk_words, ndp);
    const uint8_t* lb = reinterpret_cast<const uint8_t*>(colw);
    for (uint64_t d = d0 + t; d < d1; d += 256) {
        vk_t w = {};
        if (d < nd) {
            const u32x4_t* pp = reinterpret_cast<const u32x4_t*>(plan + 16 * d);
#pragma unroll
            for (int v = 0; v < 4; v++) {
                const u32x4_t e4 = pp[v];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t e = e4[k];
                    const vk_t x = *reinterpret_cast<const vk_t*>(lb + (e >> 5));
#pragma unroll
                    for (int cc = 0; cc < K; cc++) w[cc] |= __builtin_amdgcn_ubfe(x[cc], e & 31u, 2) << (2 * (4 * v + k));
                }
            }
        }
#pragma unroll
        for (int cc = 0; cc < K; cc++)
            if (g * K + cc < m) reinterpret_cast<uint32_t*>(dst + (g * K + cc) * dp)[d] = w[cc];
    }
}

// Lane-interleaved form of k_repack_win (the default windowed gather): a wave owns 1024-code
// output segments; at step k lane t gathers code 64k + t, so the 64 lanes of one LDS read fetch
// neighbouring source codes (same or consecutive u32x4: broadcast, no bank conflict, where the
// dword-per-lane form had lanes 16 codes apart = 2-way conflicts), and each lane packs its 16
// codes into one dword.  A 16x16 transpose of 2-bit pairs inside each 16-lane row (4 butterfly
// stages, DPP + v_alignbit + v_bfi) turns those into output dwords: lane 16q + i holds dword
// 4i + q of the segment, so one store per column still covers 256 contiguous bytes.  The plan is
// u16 (window dword << 4 | code in dword), stored per lane (entry [segment][lane][k]) so a lane
// reads its 2 segments' 32 entries as four 16-B loads issued before the window loads.
__device__ __forceinline__ uint32_t dpp_xor(uint32_t v, int s) {
    // partner lane i ^ 2^s within each 16-lane row (gfx9 DPP has no row_xmask: i^4 = (i^7)^3,
    // i^8 = (i^15)^7)
    const int x = (int)v;
    if (s == 0) return (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);
    if (s == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);
    if (s == 2)
        return (uint32_t)__builtin_amdgcn_update_dpp(0, __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false),
                                                     0x1B, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(0, __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false), 0x141,
                                                 0xF, 0xF, false);
}

template <int K>
__global__ __launch_bounds__(256) void k_repack_win16(const uint8_t* __restrict__ src, uint64_t sp, uint64_t nq,
                                                      uint64_t zq, uint64_t nchunks, uint64_t m,
                                                      const uint32_t* __restrict__ win,
                                                      const uint16_t* __restrict__ plan, uint8_t* __restrict__ dst,
                                                      uint64_t dp) {
    extern __shared__ u32x4_t colw[];
    typedef uint32_t vk_t __attribute__((ext_vector_type(K)));
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint64_t c = blockIdx.x % nchunks, g = blockIdx.x / nchunks;
    // this lane's plan entries of segments 2*wave and 2*wave+1 of chunk c (16 u16 each)
    u32x4_t pe[4];
    {
        const u32x4_t* pp = reinterpret_cast<const u32x4_t*>(plan + (c * 8 + 2 * wave) * 1024 + 16 * lane);
        pe[0] = pp[0];
        pe[1] = pp[1];
        pe[2] = pp[128];  // next segment: + 1024 u16 = 128 u32x4
        pe[3] = pp[129];
    }
    const uint64_t lo4 = win[c], n4 = min(zq, nq - lo4);
    uint32_t* l = reinterpret_cast<uint32_t*>(colw);
    for (uint64_t q = t; q < n4; q += 256) {
        u32x4_t v[K];
#pragma unroll
        for (int cc = 0; cc < K; cc++) {
            const uint64_t j = g * K + cc;
            v[cc] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(src + (j < m ? j : m - 1) * sp) + lo4 + q);
        }
        if constexpr (K == 1) {
            colw[q] = v[0];
        } else {
#pragma unroll
            for (int e = 0; e < 4; e++) {
                vk_t x;
#pragma unroll
                for (int cc = 0; cc < K; cc++) x[cc] = v[cc][e];
                *reinterpret_cast<vk_t*>(l + (4 * q + e) * K) = x;
            }
        }
    }
    if (t < K) l[4 * zq * K + t] = 0;
    __syncthreads();
    const uint8_t* lb = reinterpret_cast<const uint8_t*>(colw);
    const uint64_t ndp = dp / 4;
    const int i = lane & 15, q = lane >> 4;
#pragma unroll
    for (int sg = 0; sg < 2; sg++) {
        uint32_t a[K];
#pragma unroll
        for (int cc = 0; cc < K; cc++) a[cc] = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t word = pe[2 * sg + (k >> 3)][(k >> 1) & 3];
            const uint32_t e = (k & 1) ? word >> 16 : word & 0xffffu;
            const vk_t x = *reinterpret_cast<const vk_t*>(lb + (e >> 4) * (4 * K));
#pragma unroll
            for (int cc = 0; cc < K; cc++) a[cc] |= __builtin_amdgcn_ubfe(x[cc], 2 * (e & 15u), 2) << (2 * k);
        }
        // 16 x 16 transpose of 2-bit pairs within each row: stage s swaps bit s of the lane index
        // with bit s of the pair index
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const uint32_t m0 = s == 0 ? 0x33333333u : s == 1 ? 0x0F0F0F0Fu : s == 2 ? 0x00FF00FFu : 0x0000FFFFu;
            const bool hi = (i >> s) & 1;
            const uint32_t mk = hi ? ~m0 : m0;
            const uint32_t rot = hi ? 2u << s : 32u - (2u << s);
#pragma unroll
            for (int cc = 0; cc < K; cc++) {
                const uint32_t y = dpp_xor(a[cc], s);
                const uint32_t sy = __builtin_amdgcn_alignbit(y, y, rot);
                a[cc] = (a[cc] & mk) | (sy & ~mk);
            }
        }
        const uint64_t d = (c * 8 + 2 * wave + sg) * 64 + 4 * i + q;
        if (d < ndp) {
#pragma unroll
            for (int cc = 0; cc < K; cc++)
                if (g * K + cc < m) reinterpret_cast<uint32_t*>(dst + (g * K + cc) * dp)[d] = a[cc];
        }
    }
}

// u16 lane-interleaved plan of k_repack_win16: code r of chunk c (8192 codes, 8 segments of 1024)
// at [r & ~1023] + 16 * (r & 63) + ((r >> 6) & 15); entries past n_out point at the zero dword
__global__ void k_repack_plan16(const uint64_t* __restrict__ idx, uint64_t n_out, uint64_t n_all, uint64_t zq,
                                const uint32_t* __restrict__ win, uint16_t* __restrict__ plan) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_all; r += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t e = (uint32_t)(4 * zq) << 4;
        if (r < n_out) {
            const uint64_t i = idx[r];
            e = (uint32_t)(((i >> 4) - 4ull * win[r / kRepackChunk]) << 4) | (uint32_t)(i & 15);
        }
        plan[(r & ~1023ull) + 16 * (r & 63) + ((r >> 6) & 15)] = (uint16_t)e;
    }
}

template <int K>
__global__ __launch_bounds__(1024) void k_repack_lds(const uint8_t* __restrict__ src, uint64_t sp, uint64_t nq,
                                                     uint64_t m, const uint32_t* __restrict__ plan, uint64_t n_out,
                                                     uint8_t* __restrict__ dst, uint64_t dp) {
    extern __shared__ u32x4_t colq[];  // K * nq u32x4 + one zero u32x4
    typedef uint32_t vk_t __attribute__((ext_vector_type(K)));
    const int t = threadIdx.x;
    const uint64_t ng = (m + K - 1) / K;
    const uint64_t nd = (n_out + 15) / 16, ndp = dp / 4;
    constexpr int PRE = kRepackPre[K >> 1];  // u32x4 per column per thread held in registers
    u32x4_t pre[K][PRE];
    auto fetch = [&](uint64_t g) {
#pragma unroll
        for (int c = 0; c < K; c++) {
            const uint64_t j = g * K + c;
            const u32x4_t* s = reinterpret_cast<const u32x4_t*>(src + (j < m ? j : m - 1) * sp);
#pragma unroll
            for (int u = 0; u < PRE; u++) {
                const uint64_t q = (uint64_t)t + 1024u * u;
                pre[c][u] = q < nq ? __builtin_nontemporal_load(s + q) : (u32x4_t){0, 0, 0, 0};
            }
        }
    };
    auto park = [&]() {
        uint32_t* l = reinterpret_cast<uint32_t*>(colq);
#pragma unroll
        for (int u = 0; u < PRE; u++) {
            const uint64_t q = (uint64_t)t + 1024u * u;
            if (q < nq) {
                if constexpr (K == 1) {
                    colq[q] = pre[0][u];
                } else {
#pragma unroll
                    for (int e = 0; e < 4; e++) {  // dword 4q+e of every column: one K-dword store
                        vk_t v;
#pragma unroll
                        for (int c = 0; c < K; c++) v[c] = pre[c][u][e];
                        *reinterpret_cast<vk_t*>(l + (4 * q + e) * K) = v;
                    }
                }
            }
        }
        if (t < K) l[4 * nq * K + t] = 0;
    };
    uint64_t g = blockIdx.x;
    if (g >= ng) return;
    fetch(g);
    for (; g < ng; g += gridDim.x) {
        __syncthreads();  // the previous group's gather is done with LDS
        park();
        __syncthreads();
        if (g + gridDim.x < ng) fetch(g + gridDim.x);  // in flight during this group's gather
        const uint8_t* lb = reinterpret_cast<const uint8_t*>(colq);
        for (uint64_t d = t; d < ndp; d += 1024) {
            vk_t w = {};
            if (d < nd) {
                const u32x4_t* pp = reinterpret_cast<const u32x4_t*>(plan + 16 * d);
#pragma unroll
                for (int v = 0; v < 4; v++) {
                    const u32x4_t e4 = pp[v];
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t e = e4[k];
                        const vk_t x = *reinterpret_cast<const vk_t*>(lb + (e >> 5));
#pragma unroll
                        for (int c = 0; c < K; c++)
                            w[c] |= __builtin_amdgcn_ubfe(x[c], e & 31u, 2) << (2 * (4 * v + k));
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < K; c++)
                if (g * K + c < m) reinterpret_cast<uint32_t*>(dst + (g * K + c) * dp)[d] = w[c];
        }
    }
}

// ------------------------------------------------------------------ dense f32 block -> codes + LUT
// A standardized genotype column takes at most 4 distinct values (codes 0/2/3 and the imputed 0 of
// missing, or their Identity values), so a dense f32 GRM operand of such columns is re-encoded
// EXACTLY as 2-bit codes + a per-SNP f32 LUT of the distinct bit patterns, and the GRM runs on the
// packed fp16x2 SYRK (0.25 B per value instead of 4.6 B of stage images).  One 256-thread
// workgroup per column: (1) each thread collects up to 4 distinct bit patterns of its values,
// (2) four block-wide min-reductions over the patterns give the column's sorted distinct set,
// and a block OR flags a column with a fifth value (*flag |= 1: the caller keeps the dense path),
// (3) every output word of 16 codes is written, the pad words of the pitch included.
__global__ __launch_bounds__(256) void k_dense_codes(const float* __restrict__ Z, uint64_t ldz, uint64_t n,
                                                     uint8_t* __restrict__ packed, uint64_t pitch,
                                                     float* __restrict__ lut, unsigned int* __restrict__ flag) {
    const uint64_t s = blockIdx.x;
    const uint32_t* col = reinterpret_cast<const uint32_t*>(Z + s * ldz);
    const int t = threadIdx.x;
    uint32_t u[4];
    int cnt = 0;
    bool over = false;
    for (uint64_t r = t; r < n; r += 256) {
        const uint32_t v = col[r];
        bool seen = false;
#pragma unroll
        for (int k = 0; k < 4; k++) seen |= k < cnt && u[k] == v;
        if (!seen) {
            if (cnt < 4) {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (k == cnt) u[k] = v;
                cnt++;
            } else {
                over = true;
            }
        }
    }
    __shared__ uint32_t red[256];
    __shared__ uint32_t uniq[5];
    __shared__ int anyover;
    if (t == 0) anyover = 0;
    __syncthreads();
    if (over) anyover = 1;
    // distinct set in ascending bit order: round k takes the smallest pattern above round k-1's
    uint32_t last = 0;
    int nu = 0;
    for (int k = 0; k < 5; k++) {
        uint32_t cand = 0xffffffffu;
        bool has = false;
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (j < cnt && (k == 0 || u[j] > last) && u[j] <= cand) {
                cand = u[j];
                has = true;
            }
        red[t] = has ? cand : 0xffffffffu;
        uint32_t hasv = has ? 1u : 0u;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (t < w) red[t] = min(red[t], red[t + w]);
            __syncthreads();
        }
        // a pattern equal to 0xffffffff would be ambiguous with "none": count holders separately
        const uint32_t mn = red[0];
        __syncthreads();
        red[t] = hasv;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (t < w) red[t] |= red[t + w];
            __syncthreads();
        }
        const bool found = red[0] != 0;
        __syncthreads();
        if (!found) break;
        if (t == 0) uniq[k] = mn;
        last = mn;
        nu = k + 1;
    }
    __syncthreads();
    if (nu > 4) anyover = 1;
    __syncthreads();
    if (anyover) {
        if (t == 0) atomicOr(flag, 1u);
        return;
    }
    if (t < 4) lut[4 * s + t] = t < nu ? __uint_as_float(uniq[t]) : 0.f;
    // unused slots never match (a value equal to uniq[0] must get code 0)
    const bool h1 = nu > 1, h2 = nu > 2, h3 = nu > 3;
    const uint32_t u1 = h1 ? uniq[1] : 0, u2 = h2 ? uniq[2] : 0, u3 = h3 ? uniq[3] : 0;
    uint32_t* o = reinterpret_cast<uint32_t*>(packed + s * pitch);
    const uint64_t nw = (n + 15) / 16, nwp = pitch / 4;
    for (uint64_t w = t; w < nwp; w += 256) {
        uint32_t word = 0;
        if (w < nw) {
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint64_t r = 16 * w + k;
                if (r < n) {
                    const uint32_t v = col[r];
                    const uint32_t c = (h1 && v == u1) ? 1u : (h2 && v == u2) ? 2u : (h3 && v == u3) ? 3u : 0u;
                    word |= c << (2 * k);
                }
            }
        }
        o[w] = word;
    }
}

// ------------------------------------------------------------------ dense standardize
template <typename T>
__device__ __forceinline__ T apply_one(T x, double mean, double sd, int is_beta, double w, bool zero_col) {
    if (x != x || zero_col) return (T)0;
    double d = (double)x - mean;
    return (T)(is_beta ? d * w : d / sd);
}

// F order, round 3: one wave per column, 4-B accesses, two passes -- the general path for columns
// holding values other than 0/1/2/NaN (`only`: the columns k_std_cols_f flagged), and A/B variant
// "std" 1 for every column.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_std_dense_f(T* __restrict__ val, uint64_t rows, uint64_t cols,
                                                        uint64_t ld, int std_kind, double a, double b, int use_stats,
                                                        T* __restrict__ stats, const uint8_t* __restrict__ only) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / kWave);
    const int is_beta = std_kind == SNPMI_STD_BETA;
    for (uint64_t j = (uint64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave; j < cols; j += nwaves) {
        if (only && !only[j]) continue;  // the columns k_std_cols_f handed over (non-genotype values)
        T* c = val + j * ld;
        double mean, sd;
        if (use_stats) {
            mean = (double)stats[2 * j];
            sd = (double)stats[2 * j + 1];
        } else {
            double n = 0, s1 = 0, s2 = 0;
            for (uint64_t i = lane; i < rows; i += kWave) {
                T x = c[i];
                if (x == x) {
                    double dx = (double)x;
                    n += 1.0;
                    s1 += dx;
                    s2 += dx * dx;
                }
            }
            n = wave_sum_f64(n);
            s1 = wave_sum_f64(s1);
            s2 = wave_sum_f64(s2);
            mean = stats_mean_std(n, s1, s2, &sd);
            if (lane == 0) {
                stats[2 * j] = (T)mean;
                stats[2 * j + 1] = (T)sd;
            }
        }
        const double w = is_beta ? beta_weight(mean, a, b) : 0.0;
        const bool zero_col = is_beta && use_stats && __builtin_isinf(sd);
        for (uint64_t i = lane; i < rows; i += kWave) c[i] = apply_one(c[i], mean, sd, is_beta, w, zero_col);
    }
}

// Per-column apply constants, computed once per column by ONE thread (beta_weight's lgamma/pow
// stay out of the hot loop) and shared through LDS: the standardized values of the genotype values
// 0/1/2 (+0.0, 1.0, 2.0 by bit pattern, so -0.0 still takes apply_one), computed by apply_one
// itself so the lookup is bit-identical to the per-element formula.  Anything else (non-genotype
// floats, NaN) takes apply_one with the column's mean / sd / weight -- the per-element f64 divide
// runs only for those.
struct ColConst {
    double mean, sd, w;
    int zero_col;
    double l[3];
};

template <typename T, bool BETA = true>
__device__ __forceinline__ void col_const(ColConst& cc, double mean, double sd, int is_beta, double a, double b,
                                          int use_stats) {
    cc.mean = mean;
    cc.sd = sd;
    cc.w = BETA && is_beta ? beta_weight_call(mean, a, b) : 0.0;
    cc.zero_col = is_beta && use_stats && __builtin_isinf(sd);
    for (int v = 0; v < 3; v++) cc.l[v] = (double)apply_one((T)v, mean, sd, is_beta, cc.w, cc.zero_col != 0);
}

__device__ __forceinline__ uint64_t tbits(float x) { return __float_as_uint(x); }
__device__ __forceinline__ uint64_t tbits(double x) { return (uint64_t)__double_as_longlong(x); }

// genotype lookup: 0..2 for +0.0 / 1.0 / 2.0, 3 for anything else
template <typename T>
__device__ __forceinline__ int geno_of(T x) {
    const uint64_t u = tbits(x);
    return u == tbits((T)0) ? 0 : u == tbits((T)1) ? 1 : u == tbits((T)2) ? 2 : 3;
}

template <typename T>
__device__ __forceinline__ void acc_stat(T x, double& n, double& s1, double& s2) {
    if (x == x) {
        const double dx = (double)x;
        n += 1.0;
        s1 += dx;
        s2 += dx * dx;
    }
}

template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t col_rsrc(T* p, uint64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(sgpr_ptr(p), (short)0, (int)__builtin_amdgcn_readfirstlane((uint32_t)bytes),
                                             0x00020000);
}

// F order, genotype-valued columns (0 / 1 / 2 / NaN -- a decoded .bed): one NT-thread workgroup per
// column (grid-stride over columns), 16-B buffer loads and stores through a per-column resource
// whose range check drops the accesses past the column (no per-vector branches; the zeros they read
// are taken out of the observation count).  The column's aligned body is NV vectors per thread per
// chunk; when it fits one chunk the values stay in registers between the stats reduction and the
// table apply, so the column is read from HBM once and written once (the algorithmic 2 x 4 B per f32
// value); longer columns (or use_stats) read it again per chunk.  A misaligned head / tail (< 16 B
// each) are single elements owned by the first threads.  Stats: per-thread partial sums in T are
// exact integers for such values, i.e. the f64 sums of any order, then bed-reader's one-pass
// mean / std (stats_mean_std) -- bit-identical to the f64 path.  A column with any other value is
// left untouched and flagged (flags[j] = 1, *any = 1) for k_std_dense_f.
template <typename T, int NT, int NV, bool BETA>
__global__ __launch_bounds__(NT) void k_std_cols_f(T* __restrict__ val, uint64_t rows, uint64_t cols, uint64_t ld,
                                                   int std_kind, double a, double b, int use_stats,
                                                   T* __restrict__ stats, uint8_t* __restrict__ flags,
                                                   unsigned int* __restrict__ any) {
    constexpr int VE = 16 / sizeof(T);
    typedef T vec __attribute__((ext_vector_type(VE)));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    constexpr int NW = NT / kWave;
    __shared__ double red[3][NW];
    __shared__ T lut[3];
    const int t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
    const int is_beta = BETA && std_kind == SNPMI_STD_BETA;
    constexpr uint64_t chunk = (uint64_t)NT * NV;  // vectors per chunk
    for (uint64_t j = blockIdx.x; j < cols; j += gridDim.x) {
        T* c = val + j * ld;
        uint64_t h = ((16 - (reinterpret_cast<uintptr_t>(c) & 15)) & 15) / sizeof(T);
        if (h > rows) h = rows;
        const uint64_t nvec = (rows - h) / VE;
        const uint64_t tail0 = h + nvec * VE;
        const __amdgpu_buffer_rsrc_t rs = col_rsrc(c + h, nvec * 16);
        // the one scalar this thread owns (head element t, or tail element t - h)
        const uint64_t se = (uint64_t)t < h ? (uint64_t)t : tail0 + (uint64_t)t - h;
        const bool has_s = (uint64_t)t < h || se < rows;
        const T xs = has_s ? c[se] : (T)0;
        const bool resident = nvec <= chunk;
        u32x4 r[NV];
        // pass 1 (whole column): partial sums, observation count, and the genotype check
        T p1 = 0, p2 = 0;
        uint32_t cnt = 0;
        bool oth = false;
        auto take = [&](T x) {  // (-0.0 counts as "other": apply_one keeps its sign when mean == 0)
            const bool ok = x == x;
            const T xv = ok ? x : (T)0;
            p1 += xv;
            p2 += xv * xv;
            cnt += ok;
            oth |= ok && geno_of(x) == 3;
        };
        if (has_s) take(xs);
        if (!use_stats || !resident) {
            for (uint64_t q0 = 0; q0 < nvec; q0 += chunk) {
                const uint32_t vo = (uint32_t)((q0 + t) * 16);
#pragma unroll
                for (int k = 0; k < NV; k++) r[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, k * NT * 16, 2);
                // vectors of this thread past the column (zero-filled by the range check)
                const uint32_t left = (uint32_t)(nvec - q0), mine = left > (uint32_t)t ? left - (uint32_t)t : 0u;
                const uint32_t good = mine >= (uint32_t)((NV - 1) * NT + 1) ? NV : (mine + NT - 1) / NT;
                cnt -= (uint32_t)((NV - good) * VE);
#pragma unroll
                for (int k = 0; k < NV; k++) {
                    const vec x = __builtin_bit_cast(vec, r[k]);
#pragma unroll
                    for (int e = 0; e < VE; e++) take(x[e]);
                    __builtin_amdgcn_sched_barrier(0);  // one vector's temporaries at a time
                }
            }
        } else {  // use_stats, one chunk: load it here, check it below
            const uint32_t vo = (uint32_t)t * 16;
#pragma unroll
            for (int k = 0; k < NV; k++) r[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, k * NT * 16, 2);
#pragma unroll
            for (int k = 0; k < NV; k++) {
                const vec x = __builtin_bit_cast(vec, r[k]);
#pragma unroll
                for (int e = 0; e < VE; e++) take(x[e]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (__syncthreads_or(oth)) {  // not a genotype column: k_std_dense_f takes it
            if (t == 0) {
                flags[j] = 1;
                atomicOr(any, 1u);
            }
            continue;  // (the barrier above also ordered the previous column's LDS reads)
        }
        if (!use_stats) {
            // exact small integers per thread, summed in f64 across the workgroup
            const double n = wave_sum_f64((double)cnt), s1 = wave_sum_f64((double)p1),
                         s2 = wave_sum_f64((double)p2);
            if (lane == 0) {
                red[0][wv] = n;
                red[1][wv] = s1;
                red[2][wv] = s2;
            }
            __syncthreads();
            if (t == 0) {
                double tn = 0, t1 = 0, t2 = 0;
                for (int q = 0; q < NW; q++) {
                    tn += red[0][q];
                    t1 += red[1][q];
                    t2 += red[2][q];
                }
                double sd;
                const double mean = stats_mean_std(tn, t1, t2, &sd);
                stats[2 * j] = (T)mean;
                stats[2 * j + 1] = (T)sd;
                ColConst cc;
                col_const<T, BETA>(cc, mean, sd, is_beta, a, b, use_stats);
                for (int v = 0; v < 3; v++) lut[v] = (T)cc.l[v];
            }
        } else if (t == 0) {
            ColConst cc;
            col_const<T, BETA>(cc, (double)stats[2 * j], (double)stats[2 * j + 1], is_beta, a, b, use_stats);
            for (int v = 0; v < 3; v++) lut[v] = (T)cc.l[v];
        }
        __syncthreads();
        const T l0 = lut[0], l1 = lut[1], l2 = lut[2];
        auto map = [&](T x) { return x == (T)1 ? l1 : x == (T)2 ? l2 : x == x ? l0 : (T)0; };  // +0 / NaN
        if (has_s) c[se] = map(xs);
        for (uint64_t q0 = 0; q0 < nvec; q0 += chunk) {
            const uint32_t vo = (uint32_t)((q0 + t) * 16);
            if (!resident) {
#pragma unroll
                for (int k = 0; k < NV; k++) r[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, k * NT * 16, 2);
            }
#pragma unroll
            for (int k = 0; k < NV; k++) {
                const vec x = __builtin_bit_cast(vec, r[k]);
                vec o;
#pragma unroll
                for (int e = 0; e < VE; e++) o[e] = map(x[e]);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rs, vo, k * NT * 16, 2);
                __builtin_amdgcn_sched_barrier(0);  // one vector's registers at a time
            }
        }
        __syncthreads();  // lut / red are reused by the next column
    }
}

// C order with 16-B row segments (row pitch and base 16-B aligned): a 256-thread workgroup owns
// 64*VE adjacent columns, each lane VE of them (one 16-B load per row), the 4 waves walk rows.
// Two passes over the slab (stats, then apply): a C-order column cannot stay on chip.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_std_cols_c16(T* __restrict__ val, uint64_t rows, uint64_t cols,
                                                         uint64_t ld, int std_kind, double a, double b,
                                                         int use_stats, T* __restrict__ stats) {
    constexpr int VE = 16 / sizeof(T);
    typedef T vec __attribute__((ext_vector_type(VE)));
    constexpr int NW = kBlock / kWave;
    constexpr int CW = kWave * VE;  // columns per workgroup
    __shared__ double red[3][NW][CW];
    __shared__ ColConst cc[CW];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int is_beta = std_kind == SNPMI_STD_BETA;
    for (uint64_t j0 = (uint64_t)blockIdx.x * CW; j0 < cols; j0 += (uint64_t)gridDim.x * CW) {
        const uint64_t jl = j0 + (uint64_t)lane * VE;  // this lane's first column
        const int nv = jl >= cols ? 0 : (int)min<uint64_t>(VE, cols - jl);
        if (use_stats) {
            if (wv == 0)
                for (int e = 0; e < nv; e++)
                    col_const<T>(cc[lane * VE + e], (double)stats[2 * (jl + e)], (double)stats[2 * (jl + e) + 1],
                                 is_beta, a, b, use_stats);
        } else {
            double n[VE], s1[VE], s2[VE];
#pragma unroll
            for (int e = 0; e < VE; e++) n[e] = s1[e] = s2[e] = 0;
            if (nv == VE) {
                for (uint64_t i = wv; i < rows; i += NW) {
                    const vec x = __builtin_nontemporal_load(reinterpret_cast<const vec*>(val + i * ld + jl));
#pragma unroll
                    for (int e = 0; e < VE; e++) acc_stat(x[e], n[e], s1[e], s2[e]);
                }
            } else if (nv > 0) {
                for (uint64_t i = wv; i < rows; i += NW)
                    for (int e = 0; e < nv; e++) acc_stat(val[i * ld + jl + e], n[e], s1[e], s2[e]);
            }
#pragma unroll
            for (int e = 0; e < VE; e++) {
                red[0][wv][lane * VE + e] = n[e];
                red[1][wv][lane * VE + e] = s1[e];
                red[2][wv][lane * VE + e] = s2[e];
            }
            __syncthreads();
            if (wv == 0)
                for (int e = 0; e < nv; e++) {
                    const int q = lane * VE + e;
                    double tn = 0, t1 = 0, t2 = 0;
                    for (int w2 = 0; w2 < NW; w2++) {
                        tn += red[0][w2][q];
                        t1 += red[1][w2][q];
                        t2 += red[2][w2][q];
                    }
                    double sd;
                    const double mean = stats_mean_std(tn, t1, t2, &sd);
                    stats[2 * (jl + e)] = (T)mean;
                    stats[2 * (jl + e) + 1] = (T)sd;
                    col_const<T>(cc[q], mean, sd, is_beta, a, b, use_stats);
                }
        }
        __syncthreads();
        if (nv > 0) {
            T l[VE][3];
#pragma unroll
            for (int e = 0; e < VE; e++)
#pragma unroll
                for (int v = 0; v < 3; v++) l[e][v] = (T)cc[lane * VE + e].l[v];
            auto slow = [&](T x, int e) {
                const ColConst& k = cc[lane * VE + e];
                return apply_one(x, k.mean, k.sd, is_beta, k.w, k.zero_col != 0);
            };
            if (nv == VE) {
                for (uint64_t i = wv; i < rows; i += NW) {
                    vec* p = reinterpret_cast<vec*>(val + i * ld + jl);
                    const vec x = __builtin_nontemporal_load(p);
                    vec o;
                    bool other = false;
#pragma unroll
                    for (int e = 0; e < VE; e++) {
                        const int g = geno_of(x[e]);
                        o[e] = g == 0 ? l[e][0] : g == 1 ? l[e][1] : l[e][2];
                        other |= g == 3;
                    }
                    if (other) {
#pragma unroll
                        for (int e = 0; e < VE; e++)
                            if (geno_of(x[e]) == 3) o[e] = slow(x[e], e);
                    }
                    __builtin_nontemporal_store(o, p);
                }
            } else {
                for (uint64_t i = wv; i < rows; i += NW)
                    for (int e = 0; e < nv; e++) val[i * ld + jl + e] = slow(val[i * ld + jl + e], e);
            }
        }
        __syncthreads();
    }
}

// C order, round 3 (and rows that are not 16-B aligned): a block owns 64 adjacent columns; lanes
// walk columns, waves walk rows.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_std_dense_c(T* __restrict__ val, uint64_t rows, uint64_t cols,
                                                        uint64_t ld, int std_kind, double a, double b, int use_stats,
                                                        T* __restrict__ stats) {
    __shared__ double red[3][4][64];
    __shared__ double fin[2][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int is_beta = std_kind == SNPMI_STD_BETA;
    for (uint64_t j0 = (uint64_t)blockIdx.x * 64; j0 < cols; j0 += (uint64_t)gridDim.x * 64) {
        const uint64_t j = j0 + lane;
        const bool ok = j < cols;
        if (use_stats) {
            if (wv == 0 && ok) {
                fin[0][lane] = (double)stats[2 * j];
                fin[1][lane] = (double)stats[2 * j + 1];
            }
        } else {
            double n = 0, s1 = 0, s2 = 0;
            if (ok)
                for (uint64_t i = wv; i < rows; i += 4) {
                    T x = val[i * ld + j];
                    if (x == x) {
                        double dx = (double)x;
                        n += 1.0;
                        s1 += dx;
                        s2 += dx * dx;
                    }
                }
            red[0][wv][lane] = n;
            red[1][wv][lane] = s1;
            red[2][wv][lane] = s2;
            __syncthreads();
            if (wv == 0) {
                double tn = 0, t1 = 0, t2 = 0;
                for (int q = 0; q < 4; q++) {
                    tn += red[0][q][lane];
                    t1 += red[1][q][lane];
                    t2 += red[2][q][lane];
                }
                double sd;
                double mean = stats_mean_std(tn, t1, t2, &sd);
                fin[0][lane] = mean;
                fin[1][lane] = sd;
                if (ok) {
                    stats[2 * j] = (T)mean;
                    stats[2 * j + 1] = (T)sd;
                }
            }
        }
        __syncthreads();
        if (ok) {
            const double mean = fin[0][lane], sd = fin[1][lane];
            const double w = is_beta ? beta_weight(mean, a, b) : 0.0;
            const bool zero_col = is_beta && use_stats && __builtin_isinf(sd);
            for (uint64_t i = wv; i < rows; i += 4) val[i * ld + j] = apply_one(val[i * ld + j], mean, sd, is_beta, w, zero_col);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ sub_matrix gather
template <typename S, typename D>
__global__ __launch_bounds__(kBlock) void k_subset(const S* __restrict__ in, uint64_t rows, uint64_t cols, uint64_t k,
                                                   int in_c, const uint64_t* __restrict__ ri, uint64_t nr,
                                                   const uint64_t* __restrict__ ci, uint64_t nc, int out_c,
                                                   D* __restrict__ out) {
    const uint64_t total = nr * nc * k;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t i, j, q;
        if (out_c) {
            q = t % k;
            const uint64_t rest = t / k;
            j = rest % nc;
            i = rest / nc;
        } else {
            i = t % nr;
            const uint64_t rest = t / nr;
            j = rest % nc;
            q = rest / nc;
        }
        const uint64_t r = ri[i], c = ci[j];
        const uint64_t src = in_c ? (r * cols + c) * k + q : r + rows * (c + cols * q);
        out[t] = (D)in[src];
    }
}

// ------------------------------------------------------------------ C -> F transpose (64x64 LDS tiles)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_transpose(const T* __restrict__ in, uint64_t rows, uint64_t cols,
                                                      T* __restrict__ out, uint64_t ld) {
    __shared__ T tile[64][65];
    const uint64_t tr = (rows + 63) / 64, tc = (cols + 63) / 64;
    const int x = threadIdx.x & 63, y = threadIdx.x >> 6;
    for (uint64_t b = blockIdx.x; b < tr * tc; b += gridDim.x) {
        const uint64_t bi = b % tr, bj = b / tr;
        for (int q = y; q < 64; q += 4) {
            const uint64_t i = bi * 64 + q, j = bj * 64 + x;
            tile[q][x] = (i < rows && j < cols) ? in[i * cols + j] : (T)0;
        }
        __syncthreads();
        for (int q = y; q < 64; q += 4) {
            const uint64_t j = bj * 64 + q, i = bi * 64 + x;
            if (i < rows && j < cols) out[j * ld + i] = tile[x][q];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ GRM tiles -> K
__device__ __forceinline__ uint64_t tile_index(uint64_t ti, uint64_t tj) { return tj * (tj + 1) / 2 + ti; }

template <typename T>
__global__ __launch_bounds__(kBlock) void k_grm_extract(const T* __restrict__ tiles, const uint64_t* __restrict__ ri,
                                                        uint64_t nr, const uint64_t* __restrict__ ci, uint64_t nc,
                                                        int out_c, double scale, T* __restrict__ out) {
    const uint64_t total = nr * nc;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t r, c;
        if (out_c) {
            r = t / nc;
            c = t - r * nc;
        } else {
            c = t / nr;
            r = t - c * nr;
        }
        uint64_t i = ri ? ri[r] : r, j = ci ? ci[c] : c;
        if (i > j) {
            const uint64_t s = i;
            i = j;
            j = s;
        }
        const T v = tiles[tile_index(i / kTile, j / kTile) * (kTile * kTile) + (i % kTile) * kTile + (j % kTile)];
        out[t] = scale == 1.0 ? v : (T)((double)v * scale);
    }
}

// Full rows [r0, r0+nr) of K (row-major, n columns, identity column index) from the
// upper-triangle tiles: one 64x64 output block per workgroup pass, read in its upper-triangle
// orientation (rows of 64 contiguous tile elements, 16-B loads) into LDS and written row by row
// with 16-B stores -- through the LDS transpose when the block lies below the diagonal.  The
// generic k_grm_extract reads the mirrored half one element per 128-element tile row (a 32-B
// sector per 4-B value): 32 ms for a 50k x 50k f32 K against ~3 ms here.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_grm_extract_rows(const T* __restrict__ tiles, uint64_t n, uint64_t r0,
                                                             uint64_t nr, double scale, T* __restrict__ out) {
    constexpr int V = 16 / sizeof(T);  // elements per 16-B vector
    constexpr int TPR = 64 / V;        // threads per 64-element row
    constexpr int RPP = kBlock / TPR;  // rows per pass
    typedef T vec_t __attribute__((ext_vector_type(V)));
    __shared__ T S[64][64 + 1];
    const int t = threadIdx.x, x = t % TPR;
    const uint64_t rb0 = r0 / 64, nbr = (r0 + nr + 63) / 64 - rb0, nbc = (n + 63) / 64;
    for (uint64_t b = blockIdx.x; b < nbr * nbc; b += gridDim.x) {
        const uint64_t R0 = (rb0 + b / nbc) * 64, C0 = (b % nbc) * 64;
        const uint64_t A0 = R0 < C0 ? R0 : C0, B0 = R0 < C0 ? C0 : R0;
        for (int y = t / TPR; y < 64; y += RPP) {
            const uint64_t i = A0 + y, j0 = B0 + (uint64_t)x * V;
            T v[V];
            if (A0 != B0 && i < n && j0 + V <= n) {
                // i < j for the whole block; the V elements sit in one 128-element tile row
                const vec_t q = *reinterpret_cast<const vec_t*>(
                    tiles + tile_index(i / kTile, j0 / kTile) * (kTile * kTile) + (i % kTile) * kTile + (j0 % kTile));
#pragma unroll
                for (int e = 0; e < V; e++) v[e] = q[e];
            } else {
#pragma unroll
                for (int e = 0; e < V; e++) {
                    const uint64_t j = j0 + e, ii = i < j ? i : j, jj = i < j ? j : i;
                    v[e] = (i < n && j < n) ? tiles[tile_index(ii / kTile, jj / kTile) * (kTile * kTile) +
                                                    (ii % kTile) * kTile + (jj % kTile)]
                                            : (T)0;
                }
            }
#pragma unroll
            for (int e = 0; e < V; e++) S[y][x * V + e] = v[e];
        }
        __syncthreads();
        const bool up = R0 <= C0;
        for (int y = t / TPR; y < 64; y += RPP) {
            const uint64_t r = R0 + y, c0 = C0 + (uint64_t)x * V;
            if (r < r0 || r >= r0 + nr || c0 >= n) continue;
            vec_t w;
#pragma unroll
            for (int e = 0; e < V; e++) {
                const T v = up ? S[y][x * V + e] : S[x * V + e][y];
                w[e] = scale == 1.0 ? v : (T)((double)v * scale);
            }
            T* o = out + (r - r0) * n + c0;
            if (c0 + V <= n && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
                *reinterpret_cast<vec_t*>(o) = w;
            } else {
                for (int e = 0; e < V; e++)
                    if (c0 + e < n) o[e] = w[e];
            }
        }
        __syncthreads();
    }
}

// The whole K (rows 0..n-1): one workgroup per upper-triangle 64x64 block (I <= J), read ONCE from
// the tiles with 16-B loads into LDS and written twice -- as block (I, J) straight and as its
// mirror (J, I) through the LDS transpose -- so the tiles cross HBM once (half the reads of
// k_grm_extract_rows, which loads every upper block for both output positions).  A diagonal block
// mirrors its own upper half.  Blocks are visited in triangular order, the grid strides over them.
// BS = 128 for f32 (a block is exactly one 64 KB tile, 512-B row segments both ways), 64 for f64
// (the same 512-B rows in half the LDS).  PIPE: the next block's loads are issued into registers
// before the current block's stores, so a workgroup keeps reads in flight while it writes.
template <typename T, int BS, int NT = kBlock, bool PIPE = false>
__global__ __launch_bounds__(NT) void k_grm_extract_sym(const T* __restrict__ tiles, uint64_t n, double scale,
                                                        T* __restrict__ out) {
    constexpr int V = 16 / sizeof(T);  // elements per 16-B vector
    constexpr int TPR = BS / V;        // threads per BS-element row
    constexpr int RPP = NT / TPR;      // rows per pass
    constexpr int NR = BS / RPP;       // rows per thread
    static_assert(BS % RPP == 0, "block rows must split evenly over the passes");
    typedef T vec_t __attribute__((ext_vector_type(V)));
    __shared__ T S[BS][BS + 1];
    const int t = threadIdx.x, x = t % TPR, y0 = t / TPR;
    const uint64_t nb = (n + BS - 1) / BS, total = nb * (nb + 1) / 2;
    auto coords = [&](uint64_t L, uint64_t& I, uint64_t& J) {
        J = (uint64_t)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
        while ((J + 1) * (J + 2) / 2 <= L) J++;
        while (J * (J + 1) / 2 > L) J--;
        I = L - J * (J + 1) / 2;
    };
    vec_t v[NR];
    auto fetch = [&](uint64_t I, uint64_t J) {
        const uint64_t R0 = I * BS, C0 = J * BS;
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const uint64_t i = R0 + y0 + r * RPP, j0 = C0 + (uint64_t)x * V;
            if (I != J && i < n && j0 + V <= n) {
                v[r] = *reinterpret_cast<const vec_t*>(tiles + tile_index(i / kTile, j0 / kTile) * (kTile * kTile) +
                                                       (i % kTile) * kTile + (j0 % kTile));
            } else {
#pragma unroll
                for (int e = 0; e < V; e++) {
                    const uint64_t j = j0 + e, ii = i < j ? i : j, jj = i < j ? j : i;
                    v[r][e] = (i < n && j < n) ? tiles[tile_index(ii / kTile, jj / kTile) * (kTile * kTile) +
                                                       (ii % kTile) * kTile + (jj % kTile)]
                                               : (T)0;
                }
            }
        }
    };
    uint64_t L = blockIdx.x, I = 0, J = 0;
    if (L < total) {
        coords(L, I, J);
        fetch(I, J);
    }
    for (; L < total; L += gridDim.x) {
#pragma unroll
        for (int r = 0; r < NR; r++)
#pragma unroll
            for (int e = 0; e < V; e++) S[y0 + r * RPP][x * V + e] = scale == 1.0 ? v[r][e] : (T)((double)v[r][e] * scale);
        __syncthreads();
        const uint64_t R0 = I * BS, C0 = J * BS;
        const bool diag = I == J;
        const uint64_t Ln = L + gridDim.x;
        if (PIPE && Ln < total) {
            coords(Ln, I, J);
            fetch(I, J);
        }
        for (int pass = 0; pass < (diag ? 1 : 2); pass++) {
            const uint64_t rb = pass ? C0 : R0, cb = pass ? R0 : C0;
            for (int y = y0; y < BS; y += RPP) {
                const uint64_t r = rb + y, c0 = cb + (uint64_t)x * V;
                if (r >= n || c0 >= n) continue;
                vec_t w;
#pragma unroll
                for (int e = 0; e < V; e++) w[e] = pass ? S[x * V + e][y] : S[y][x * V + e];
                T* o = out + r * n + c0;
                if (c0 + V <= n && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
                    __builtin_nontemporal_store(w, reinterpret_cast<vec_t*>(o));
                } else {
                    for (int e = 0; e < V; e++)
                        if (c0 + e < n) o[e] = w[e];
                }
            }
        }
        __syncthreads();
        if (!PIPE && Ln < total) {
            coords(Ln, I, J);
            fetch(I, J);
        }
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_grm_trace(const T* __restrict__ tiles, uint64_t n, double* trace) {
    __shared__ double red[kBlock / kWave];
    double s = 0;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x)
        s += (double)tiles[tile_index(i / kTile, i / kTile) * (kTile * kTile) + (i % kTile) * (kTile + 1)];
    s = wave_sum_f64(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0;
        for (int q = 0; q < kBlock / kWave; q++) t += red[q];
        *trace = t;
    }
}

// cfg5: K[ri, ci] from one part's dense 256x256 blocks (syrk.hip part_layout).  Entries whose
// block this part owns are read (upper-triangle orientation: K[i, j] = K[min, max], so the result
// is exactly symmetric, as k_grm_extract's), all others are 0 -- the sum of every part's output
// (one owner per entry; x + 0 is exact) is the sub-matrix.  lslot[L] = local slot of upper-triangle
// block L = J(J+1)/2 + I, -1 where another part owns it.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_part_extract(const T* __restrict__ blocks, const int32_t* __restrict__ lslot,
                                                         const uint64_t* __restrict__ ri, uint64_t nr,
                                                         const uint64_t* __restrict__ ci, uint64_t nc, int out_c,
                                                         double scale, T* __restrict__ out) {
    const uint64_t total = nr * nc;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t r, c;
        if (out_c) {
            r = t / nc;
            c = t - r * nc;
        } else {
            c = t / nr;
            r = t - c * nr;
        }
        uint64_t i = ri ? ri[r] : r, j = ci ? ci[c] : c;
        if (i > j) {
            const uint64_t s = i;
            i = j;
            j = s;
        }
        const uint64_t I = i / 256, J = j / 256;
        const int32_t w = lslot[J * (J + 1) / 2 + I];
        T v = (T)0;
        if (w >= 0) {
            v = blocks[(uint64_t)w * 65536 + (i % 256) * 256 + (j % 256)];
            if (scale != 1.0) v = (T)((double)v * scale);
        }
        out[t] = v;
    }
}

// sum of the K diagonal entries i < n held by one part (one workgroup, fixed reduction order)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_part_trace(const T* __restrict__ blocks, const int32_t* __restrict__ dslot,
                                                       uint64_t n, double* trace) {
    __shared__ double red[kBlock / kWave];
    double s = 0;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const int32_t w = dslot[i / 256];
        if (w >= 0) s += (double)blocks[(uint64_t)w * 65536 + (i % 256) * 257];
    }
    s = wave_sum_f64(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0;
        for (int q = 0; q < kBlock / kWave; q++) t += red[q];
        *trace = t;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_dense_trace(const T* __restrict__ K, uint64_t n, double* trace) {
    __shared__ double red[kBlock / kWave];
    double s = 0;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) s += (double)K[i * n + i];
    s = wave_sum_f64(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0;
        for (int q = 0; q < kBlock / kWave; q++) t += red[q];
        *trace = t;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_scale(T* __restrict__ p, uint64_t count, double scale) {
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += (uint64_t)gridDim.x * blockDim.x)
        p[t] = (T)((double)p[t] * scale);
}

// sum of squares in f64 (SNP-side DiagKtoN, diag_K_to_N.py:75-95): grid-stride partial sums,
// one f64 atomic per workgroup
template <typename T>
__global__ __launch_bounds__(kBlock) void k_sumsq(const T* __restrict__ p, uint64_t count, double* __restrict__ out) {
    __shared__ double red[kBlock / kWave];
    double s = 0;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += (uint64_t)gridDim.x * blockDim.x) {
        const double x = (double)p[t];
        s += x * x;
    }
    s = wave_sum_f64(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0;
        for (int q = 0; q < kBlock / kWave; q++) t += red[q];
        atomicAdd(out, t);
    }
}

// ------------------------------------------------------------------ exact f32 GRM diagonal
// K_ii = sum_s v_s(c_is)^2 is the largest entry of each K row and, in an f32 MFMA accumulation
// chain, the one that rounds worst: it grows by ~1 per SNP (a rare variant adds ~1/(2 maf) at
// once) while each step's increments are small, so after a few thousand SNPs the chain absorbs
// them at ulp(K_ii)/2 (the round-3 maxima of |dK| / max diag all sat on the
// diagonal).  These kernels give every f32 SYRK launch an exact diagonal: before the SYRK the
// current tile diagonal is saved as f64 (0 when not accumulating), k_diag_sq adds the launch's
// sum_s v^2 in f64 (each square of an f32 value is exact in f64; one f64 add per SNP), and after
// the SYRK the tile diagonal is overwritten with the f64 value rounded once to f32.
// Layout: dslot == nullptr -> upper-triangle 128x128 tiles (index tj(tj+1)/2 + ti, row-major);
// else the 256x256 blocks of one cfg5 part (syrk.hip part_layout): dslot[J] = the local slot of
// diagonal block J (-1 where another part owns it), row-major blocks.
__device__ __forceinline__ int64_t diag_offset(uint64_t i, const int32_t* __restrict__ dslot) {
    if (!dslot) {
        const uint64_t t = i / 128, r = i % 128;
        return (int64_t)((t * (t + 1) / 2 + t) * 128 * 128 + r * 128 + r);
    }
    const int32_t w = dslot[i / 256];
    const uint64_t r = i % 256;
    return w < 0 ? -1 : (int64_t)((uint64_t)w * 256 * 256 + r * 256 + r);
}

__global__ __launch_bounds__(kBlock) void k_diag_save(const float* __restrict__ K, uint64_t n,
                                                      const int32_t* __restrict__ dslot, int accumulate,
                                                      double* __restrict__ diag) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t o = diag_offset(i, dslot);
        diag[i] = (accumulate && o >= 0) ? (double)K[o] : 0.0;
    }
}

// grid.x: 16-iid words (one packed dword per thread and SNP, coalesced across the wave),
// grid.y: SNP slices (enough threads to fill the chip at any n); each slice's f64 partial sums go
// to their own row of `part` (plain stores), folded into diag in slice order by k_diag_fold -- the
// same bits on every run (f64 atomics would add the slices in arrival order)
__global__ __launch_bounds__(kBlock) void k_diag_sq(const uint8_t* __restrict__ packed, uint64_t pitch, uint64_t n,
                                                    uint64_t m, const float* __restrict__ lut, uint64_t per_slice,
                                                    uint64_t part_ld, double* __restrict__ part) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nw = (n + 15) / 16;
    if (w >= nw) return;
    const uint64_t s0 = (uint64_t)blockIdx.y * per_slice, s1 = min(m, s0 + per_slice);
    double acc[16];
#pragma unroll
    for (int k = 0; k < 16; k++) acc[k] = 0.0;
    for (uint64_t s = s0; s < s1; s++) {
        const uint32_t word = reinterpret_cast<const uint32_t*>(packed + s * pitch)[w];
        const float4 l = reinterpret_cast<const float4*>(lut)[s];  // the same address on every lane
        const double q0 = (double)l.x * (double)l.x, q1 = (double)l.y * (double)l.y, q2 = (double)l.z * (double)l.z,
                     q3 = (double)l.w * (double)l.w;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t c = (word >> (2 * k)) & 3u;
            acc[k] += c == 0 ? q0 : c == 1 ? q1 : c == 2 ? q2 : q3;
        }
    }
    double2* dst = reinterpret_cast<double2*>(part + (uint64_t)blockIdx.y * part_ld + 16 * w);
#pragma unroll
    for (int k = 0; k < 8; k++) dst[k] = make_double2(acc[2 * k], acc[2 * k + 1]);
}

__global__ __launch_bounds__(kBlock) void k_diag_fold(uint64_t n, uint64_t slices, uint64_t part_ld,
                                                      const double* __restrict__ part, double* __restrict__ diag) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        double s = diag[i];
        for (uint64_t y = 0; y < slices; y++) s += part[y * part_ld + i];
        diag[i] = s;
    }
}

__global__ __launch_bounds__(kBlock) void k_diag_patch(float* __restrict__ K, uint64_t i0, uint64_t i1,
                                                       const int32_t* __restrict__ dslot, const double* __restrict__ diag) {
    for (uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < i1; i += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t o = diag_offset(i, dslot);
        if (o >= 0) K[o] = (float)diag[i];
    }
}

// ------------------------------------------------------------------ synthetic genotypes
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// CPU twin: oracle/bed_oracle.c oracle_synth_bed (bit-identical by construction).
__global__ __launch_bounds__(kBlock) void k_synth(uint8_t* __restrict__ packed, uint64_t pitch, uint64_t n,
                                                  uint64_t sid0, uint64_t m, uint64_t seed, double miss_rate,
                                                  const double* __restrict__ maf_x, const double* __restrict__ maf_cdf,
                                                  int n_pts) {
    const uint64_t nd = pitch / 4;
    const uint64_t total = nd * m;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t j = t / nd, d = t - j * nd;
        const uint64_t sid = sid0 + j;
        uint32_t w = 0;
        if (16 * d < n) {
            const uint64_t h = splitmix64(seed * 0xD1B54A32D192ED03ull ^ (sid + 1) * 0x8CB92BA72F3D8DD7ull);
            const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
            int lo = 0, hi = n_pts - 1;  // first k with u <= cdf[k], capped at n_pts-1
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (u > maf_cdf[mid]) lo = mid + 1;
                else hi = mid;
            }
            const double maf = maf_x[lo];
            const double p2 = maf * maf, p1 = 2.0 * maf * (1.0 - maf);
            const double sc = 4294967296.0;
            const double t2 = p2 * sc, t12 = (p2 + p1) * sc, tm = miss_rate * sc;
            const uint32_t th2 = t2 >= sc ? 0xFFFFFFFFu : (uint32_t)t2;
            const uint32_t th12 = t12 >= sc ? 0xFFFFFFFFu : (uint32_t)t12;
            const uint32_t thm = tm >= sc ? 0xFFFFFFFFu : (uint32_t)tm;
            const uint64_t kb = (seed + 0x632BE59BD9B4E019ull) ^ (sid * 0x9E6C63D0676A9A99ull);
            for (int k = 0; k < 16; k++) {
                const uint64_t i = 16 * d + k;
                if (i >= n) break;
                const uint64_t hh = splitmix64(kb ^ (i * 0xC2B2AE3D27D4EB4Full));
                const uint32_t ug = (uint32_t)hh, um = (uint32_t)(hh >> 32);
                uint32_t code = um < thm ? 1u : (ug < th2 ? 3u : (ug < th12 ? 2u : 0u));
                w |= code << (2 * k);
            }
        }
        reinterpret_cast<uint32_t*>(packed + j * pitch)[d] = w;
    }
}

// Fused stats + decode with the packed column held in LDS (one 1024-thread workgroup per SNP,
// column <= kLdsColMax bytes, i.e. N <= ~600k): pass 1 streams the column HBM -> LDS once and
// counts its codes; one lane turns the counts into f64 stats + the LUT exactly as k_snp_stats
// does; pass 2 decodes from LDS with the k_decode_f store pattern (each wave store = 1 KiB
// contiguous, non-temporal).  The packed bytes are read from HBM once instead of twice.
constexpr int kLdsBlock = 1024;
constexpr uint64_t kLdsColMax = 150 * 1024;

__global__ __launch_bounds__(kLdsBlock) void k_decode_std_lds_f32(const uint8_t* __restrict__ packed, uint64_t pitch,
                                                                 uint64_t n, int count_a1, int std_kind, double a,
                                                                 double b, int use_stats, float* __restrict__ stats,
                                                                 float* __restrict__ lut_out, float* __restrict__ out,
                                                                 uint64_t ld) {
    extern __shared__ u32x4_t col[];
    __shared__ uint32_t red[3][kLdsBlock / kWave];
    __shared__ float lutsh[4];
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    const uint64_t j = blockIdx.x;
    const u32x4_t* src = reinterpret_cast<const u32x4_t*>(packed + j * pitch);
    const uint64_t nq = (n + 63) / 64;  // 16-byte words holding the column's codes
    const bool count = std_kind != SNPMI_STD_NONE && !use_stats;
    uint32_t c1 = 0, c2 = 0, c3 = 0;
    for (uint64_t q = threadIdx.x; q < nq; q += kLdsBlock) {
        const u32x4_t v = __builtin_nontemporal_load(src + q);
        col[q] = v;
        if (count) {
            const uint32_t w4[4] = {v[0], v[1], v[2], v[3]};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t lo = w4[k] & 0x55555555u, hi = (w4[k] >> 1) & 0x55555555u;
                const uint64_t ib = q * 64 + 16 * k;
                if (ib + 16 > n) {
                    const uint64_t valid = n > ib ? n - ib : 0;
                    const uint32_t mk = ((1u << (2 * valid)) - 1u) & 0x55555555u;  // valid < 16 here
                    lo &= mk;
                    hi &= mk;
                }
                c3 += __popc(lo & hi);
                c2 += __popc(hi & ~lo);
                c1 += __popc(lo & ~hi);
            }
        }
    }
    if (count) {
        c1 = wave_sum_u32(c1);
        c2 = wave_sum_u32(c2);
        c3 = wave_sum_u32(c3);
        if (lane == 0) {
            red[0][wave] = c1;
            red[1][wave] = c2;
            red[2][wave] = c3;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (std_kind == SNPMI_STD_NONE) {
            for (int c = 0; c < 4; c++) {
                const int v = code_value(c, count_a1);
                lutsh[c] = v < 0 ? __builtin_nanf("") : (float)v;
            }
        } else {
            double mean, sd;
            if (count) {
                uint64_t t1 = 0, t2 = 0, t3 = 0;
                for (int q = 0; q < kLdsBlock / kWave; q++) {
                    t1 += red[0][q];
                    t2 += red[1][q];
                    t3 += red[2][q];
                }
                const uint64_t c0 = n - t1 - t2 - t3, chi = count_a1 ? c0 : t3;
                mean = stats_mean_std((double)(n - t1), (double)(t2 + 2 * chi), (double)(t2 + 4 * chi), &sd);
                stats[2 * j] = (float)mean;
                stats[2 * j + 1] = (float)sd;
            } else {
                mean = (double)stats[2 * j];
                sd = (double)stats[2 * j + 1];
            }
            const double w = std_kind == SNPMI_STD_BETA ? beta_weight(mean, a, b) : 0.0;
            const bool zero_col = std_kind == SNPMI_STD_BETA && use_stats && __builtin_isinf(sd);
            for (int c = 0; c < 4; c++) {
                const int v = code_value(c, count_a1);
                double x;
                if (v < 0 || zero_col) x = 0.0;
                else if (std_kind == SNPMI_STD_BETA) x = ((double)v - mean) * w;
                else x = ((double)v - mean) / sd;
                lutsh[c] = (float)x;
            }
        }
        for (int c = 0; c < 4; c++) lut_out[4 * j + c] = lutsh[c];
    }
    __syncthreads();
    const float l0 = lutsh[0], l1 = lutsh[1], l2 = lutsh[2], l3 = lutsh[3];
    const uint32_t* cw = reinterpret_cast<const uint32_t*>(col);
    float* o = out + j * ld;
    const uint64_t chunks = (n + 1023) / 1024;
    for (uint64_t c = wave; c < chunks; c += kLdsBlock / kWave) {
        const uint64_t i0 = c * 1024;
        const uint32_t wv = (i0 + 16 * (uint64_t)lane < n) ? cw[c * 64 + lane] : 0u;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t srcw = __shfl(wv, r * 16 + (lane >> 2), kWave);
            const uint32_t byte = (srcw >> (8 * (lane & 3))) & 0xffu;
            const uint64_t i = i0 + r * 256 + 4 * lane;
            f32x4_t v;
            v.x = sel4(l0, l1, l2, l3, byte & 3u);
            v.y = sel4(l0, l1, l2, l3, (byte >> 2) & 3u);
            v.z = sel4(l0, l1, l2, l3, (byte >> 4) & 3u);
            v.w = sel4(l0, l1, l2, l3, byte >> 6);
            if (i + 4 <= n) {
                store_nt(reinterpret_cast<f32x4_t*>(o + i), v);
            } else {
                for (int t = 0; t < 4; t++)
                    if (i + t < n) o[i + t] = v[t];
            }
        }
    }
}

inline unsigned grid_for(uint64_t work, uint64_t per_block, unsigned cap = 65536) {
    uint64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

}  // namespace

// ====================================================================== launchers
int g_variant_decode = 0;  // tuning hook (snpmi_set_kernel_variant); no variants at present
int g_diag_exact = 1;     // exact f32 GRM diagonal (k_diag_*), hook "diag"
int g_variant_std = 0;      // dense standardize: 0 = k_std_cols_f / k_std_cols_c16, 1 = round 3's kernels
// whole-K extraction: 0 = k_grm_extract_sym, 1 = round 3's k_grm_extract_rows, 2-4 = other block
// shapes, 5-7 = the pipelined (PIPE) kernel in three shapes
int g_variant_extract = 0;

#define SNPMI_LAUNCH_CHECK() SNPMI_HIP(hipGetLastError())

void launch_snp_stats(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, int count_a1, int std_kind,
                      double a, double b, int use_stats, int dtype, void* stats, void* lut, hipStream_t st) {
    if (m == 0) return;
    // 4 waves per SNP once a column is >= 16 KiB (tools/ubench.py / bench A/B: decode variant 6
    // forces one wave per SNP)
    const bool wide = n >= 65536 && g_variant_decode != 6;
#define SNPMI_STATS(T, W, kind)                                                                                    \
    k_snp_stats<T, W><<<(unsigned)ceil_div(m, kBlock / kWave / W), kBlock, 0, st>>>(                               \
        packed, pitch, n, m, count_a1, kind, a, b, dtype == SNPMI_DT_I8 ? 0 : use_stats, (T*)stats, (T*)lut)
#define SNPMI_STATS_U(T, W, U, kind)                                                                               \
    k_snp_stats<T, W, U><<<(unsigned)ceil_div(m, kBlock / kWave / W), kBlock, 0, st>>>(                            \
        packed, pitch, n, m, count_a1, kind, a, b, dtype == SNPMI_DT_I8 ? 0 : use_stats, (T*)stats, (T*)lut)
    if (dtype == SNPMI_DT_F32) {
        // A/B of the load depth (decode variants 7 / 9: 4 / 16 loads in flight per lane) and of
        // 2 waves per SNP (variant 8)
        if (wide && g_variant_decode == 7) SNPMI_STATS_U(float, 4, 4, std_kind);
        else if (wide && g_variant_decode == 9) SNPMI_STATS_U(float, 4, 16, std_kind);
        else if (wide && g_variant_decode == 8) SNPMI_STATS(float, 2, std_kind);
        else if (wide) SNPMI_STATS(float, 4, std_kind);
        else SNPMI_STATS(float, 1, std_kind);
    } else if (dtype == SNPMI_DT_F64) {
        if (wide) SNPMI_STATS(double, 4, std_kind);
        else SNPMI_STATS(double, 1, std_kind);
    } else {
        SNPMI_STATS(int8_t, 1, SNPMI_STD_NONE);
    }
#undef SNPMI_STATS
#undef SNPMI_STATS_U
    SNPMI_LAUNCH_CHECK();
}

void launch_decode(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const void* lut, int dtype,
                   int order_c, void* out, uint64_t ld, hipStream_t st) {
    if (m == 0 || n == 0) return;
    if (!order_c) {
        // 4 work items per wave; 8x more blocks than resident waves can hold (measured best)
        const uint64_t waves = ceil_div(ceil_div(n, 1024) * m, 4);
        const unsigned g = grid_for(waves, kBlock / kWave, 256 * 16 * 8);
        // XCD-sliced item order (each XCD writes a contiguous 1/8 of every grid pass; the grid
        // is a multiple of 8 so the block permutation is a bijection): 0.712 vs 0.755 ms per
        // 2048-SNP block at 500k iids, mean over 12 output buffers on 2 boxes (profiles/r02q)
        const unsigned g8 = (unsigned)round_up(g, 8);
        if (dtype == SNPMI_DT_F32)
            k_decode_f<float, 4><<<g8, kBlock, 0, st>>>(packed, pitch, n, m, (const float*)lut, (float*)out, ld);
        else if (dtype == SNPMI_DT_F64)
            k_decode_f<double, 4><<<g8, kBlock, 0, st>>>(packed, pitch, n, m, (const double*)lut, (double*)out, ld);
        else
            k_decode_f<int8_t, 4><<<g8, kBlock, 0, st>>>(packed, pitch, n, m, (const int8_t*)lut, (int8_t*)out, ld);
    } else {
        if (dtype != SNPMI_DT_I8 && g_variant_decode != 2 && ld % (16 / dtype_size(dtype)) == 0 &&
            reinterpret_cast<uintptr_t>(out) % 16 == 0 && pitch % 64 == 0) {
            const uint64_t V = 16 / dtype_size(dtype);
            const uint64_t waves = ceil_div(n, 256) * ceil_div(m, 64 * V);
            const unsigned g = grid_for(waves, kBlock / kWave, 256 * 16);
            // tools/ubench.py decode_c: row tiles fastest 5.51 TB/s at 100k x 16384 (row-major order
            // 4.97, the 64x64 LDS-tile kernel 4.51); all three ~4.4 at 500k x 4096
            if (dtype == SNPMI_DT_F32 && g_variant_decode == 3)
                k_decode_c_reg<float, true><<<g, kBlock, 0, st>>>(packed, pitch, n, m, (const float*)lut, (float*)out, ld);
            else if (dtype == SNPMI_DT_F32)
                k_decode_c_reg<float, false><<<g, kBlock, 0, st>>>(packed, pitch, n, m, (const float*)lut, (float*)out,
                                                                   ld);
            else
                k_decode_c_reg<double, false><<<g, kBlock, 0, st>>>(packed, pitch, n, m, (const double*)lut,
                                                                    (double*)out, ld);
            SNPMI_LAUNCH_CHECK();
            return;
        }
        const uint64_t tiles = ceil_div(n, 64) * ceil_div(m, 64);
        const unsigned g = grid_for(tiles, 1, 256 * 8);
        if (dtype == SNPMI_DT_F32)
            k_decode_c<float><<<g, kBlock, 0, st>>>(packed, pitch, n, m, (const float*)lut, (float*)out, ld);
        else if (dtype == SNPMI_DT_F64)
            k_decode_c<double><<<g, kBlock, 0, st>>>(packed, pitch, n, m, (const double*)lut, (double*)out, ld);
        else
            k_decode_c<int8_t><<<g, kBlock, 0, st>>>(packed, pitch, n, m, (const int8_t*)lut, (int8_t*)out, ld);
    }
    SNPMI_LAUNCH_CHECK();
}

void launch_decode_std_fused(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, int count_a1,
                             int std_kind, double a, double b, int use_stats, void* stats, void* lut, void* out,
                             uint64_t ld, hipStream_t st) {
    if (m == 0 || n == 0) return;
    const uint64_t col_bytes = ceil_div(n, 64) * 16;
    if (g_variant_decode != 1 && col_bytes <= kLdsColMax) {
        SNPMI_HIP(hipFuncSetAttribute((const void*)k_decode_std_lds_f32, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kLdsColMax));
        k_decode_std_lds_f32<<<(unsigned)m, kLdsBlock, col_bytes, st>>>(packed, pitch, n, count_a1, std_kind, a, b,
                                                                        use_stats, (float*)stats, (float*)lut,
                                                                        (float*)out, ld);
    } else {
        k_decode_std_col_f32<4><<<(unsigned)m, kBlock, 0, st>>>(packed, pitch, n, count_a1, std_kind, a, b, use_stats,
                                                                (float*)stats, (float*)lut, (float*)out, ld);
    }
    SNPMI_LAUNCH_CHECK();
}

// u32 entries: one per output code (k_repack_plan), or two u16 per code over whole 8192-code
// chunks (k_repack_plan16)
uint64_t repack_plan_entries(uint64_t n_out) {
    const uint64_t n = std::max<uint64_t>(n_out, 1);
    return std::max(round_up(n, 16), ceil_div(n, kRepackChunk) * kRepackChunk / 2);
}
uint64_t repack_win_entries(uint64_t n_out) { return 3 * ceil_div(std::max<uint64_t>(n_out, 1), 4096) + 64; }

// Build the gather plan for one index list (once per call).  Narrow per-chunk source windows
// (the widest <= half a column and fitting K >= 1 columns in 40 KiB) select the windowed kernel;
// the choice needs the windows on the host, so this synchronises the stream once.
RepackPlan launch_repack_plan(const uint64_t* idx, uint64_t n_out, uint64_t n_src, uint32_t* plan, uint32_t* win,
                              hipStream_t st) {
    RepackPlan P;
    const uint64_t nq = ceil_div(ceil_div(n_src, 4), 16), n_pad = repack_plan_entries(n_out);
    if (n_out == 0) return P;
    // tuning hook (decode variants 9-11): chunk of 16384 / 4096 codes, or two columns per group;
    // measured 500k -> 250k x 8192 SNPs (rev2 / sorted half): 16384 0.402 ms, 8192 0.386, 32768
    // 0.468, K = 2 0.518 (profiles/r02e/ubench_repack_win.jsonl)
    const uint64_t chunk = g_variant_decode == 9 ? 16384 : g_variant_decode == 10 ? 4096 : kRepackChunk;
    const uint64_t nchunks = ceil_div(n_out, chunk);
    if (win != nullptr && nchunks > 1 && g_variant_decode != 8) {
        uint32_t* lohi = win + nchunks;
        std::vector<uint32_t> h(2 * nchunks);
        for (uint64_t c = 0; c < nchunks; c++) h[2 * c] = ~0u, h[2 * c + 1] = 0;
        SNPMI_HIP(hipMemcpyAsync(lohi, h.data(), h.size() * 4, hipMemcpyHostToDevice, st));
        k_repack_window<<<(unsigned)ceil_div(n_out, 2048), 256, 0, st>>>(idx, n_out, chunk, lohi);
        SNPMI_LAUNCH_CHECK();
        SNPMI_HIP(hipMemcpyAsync(h.data(), lohi, h.size() * 4, hipMemcpyDeviceToHost, st));
        SNPMI_HIP(hipStreamSynchronize(st));
        std::vector<uint32_t> lo4(nchunks);
        uint64_t w = 0;
        for (uint64_t c = 0; c < nchunks; c++) {
            lo4[c] = h[2 * c] >> 6;
            w = std::max<uint64_t>(w, (h[2 * c + 1] >> 6) - lo4[c] + 1);
        }
        const uint64_t budget = 40 * 1024 - 16;  // >= four workgroups per CU
        int K = 4 * w * 16 <= budget ? 4 : 2 * w * 16 <= budget ? 2 : w * 16 <= budget ? 1 : 0;
        if (g_variant_decode == 11 && K == 4) K = 2;
        if (K > 0 && 2 * w <= nq) {
            SNPMI_HIP(hipMemcpyAsync(win, lo4.data(), nchunks * 4, hipMemcpyHostToDevice, st));
            // lane-interleaved gather (k_repack_win16) when the zero dword's index fits the u16
            // entry; decode variant 17 keeps the dword-per-lane k_repack_win for A/B runs
            if (chunk == kRepackChunk && 4 * w < 4096 && g_variant_decode != 17) {
                const uint64_t n_all = nchunks * kRepackChunk;
                k_repack_plan16<<<grid_for(n_all, kBlock, 4096), kBlock, 0, st>>>(idx, n_out, n_all, w, win,
                                                                                 (uint16_t*)plan);
                SNPMI_LAUNCH_CHECK();
                SNPMI_HIP(hipStreamSynchronize(st));  // lo4 is a local vector
                P.plan = plan;
                P.win = win;
                P.K = K;
                P.zq = w;
                P.nchunks = nchunks;
                P.chunk_words = chunk / 16;
                P.lanes = true;
                return P;
            }
            k_repack_plan<<<grid_for(n_pad, kBlock, 4096), kBlock, 0, st>>>(idx, n_out, n_pad, w, K, win, chunk, plan);
            SNPMI_LAUNCH_CHECK();
            SNPMI_HIP(hipStreamSynchronize(st));  // lo4 is a local vector
            P.plan = plan;
            P.win = win;
            P.K = K;
            P.zq = w;
            P.nchunks = nchunks;
            P.chunk_words = chunk / 16;
            return P;
        }
    }
    if (nq * 16 + 16 > kRepackLds) return P;  // k_repack (global gathers) reads idx directly
    const int K = repack_k(nq);
    k_repack_plan<<<grid_for(n_pad, kBlock, 4096), kBlock, 0, st>>>(idx, n_out, n_pad, nq, K, nullptr, 1, plan);
    SNPMI_LAUNCH_CHECK();
    P.plan = plan;
    P.K = K;
    P.zq = nq;
    return P;
}

void launch_repack(const uint8_t* src, uint64_t src_pitch, uint64_t n_src, const uint64_t* idx, const RepackPlan& P,
                   uint64_t n_out, uint64_t n_sid, uint8_t* dst, uint64_t dst_pitch, hipStream_t st) {
    if (n_sid == 0) return;
    const uint64_t nq = ceil_div(ceil_div(n_src, 4), 16);  // 16-B words of a source column
    const bool fits = src_pitch % 16 == 0 && dst_pitch % 4 == 0 && n_sid < (1ull << 31);
    if (P.plan != nullptr && P.win != nullptr && fits) {
        const uint64_t ng = ceil_div(n_sid, (uint64_t)P.K);
        SNPMI_REQUIRE(ng * P.nchunks < (1ull << 31), SNPMI_E_ARG, "too many repack workgroups");
        const size_t lds = (size_t)(P.K * P.zq + 1) * 16;
        if (P.lanes) {
#define SNPMI_REPACK_WIN16(KK)                                                                                     \
    k_repack_win16<KK><<<(unsigned)(ng * P.nchunks), 256, lds, st>>>(src, src_pitch, nq, P.zq, P.nchunks, n_sid,    \
                                                                    P.win, (const uint16_t*)P.plan, dst, dst_pitch)
            if (P.K == 4) {
                SNPMI_REPACK_WIN16(4);
            } else if (P.K == 2) {
                SNPMI_REPACK_WIN16(2);
            } else {
                SNPMI_REPACK_WIN16(1);
            }
#undef SNPMI_REPACK_WIN16
            SNPMI_LAUNCH_CHECK();
            return;
        }
#define SNPMI_REPACK_WIN(KK)                                                                                       \
    k_repack_win<KK><<<(unsigned)(ng * P.nchunks), 256, lds, st>>>(src, src_pitch, nq, P.zq, P.nchunks,             \
                                                                  P.chunk_words, n_sid,                             \
                                                                   P.win, P.plan, n_out, dst, dst_pitch)
        if (P.K == 4) {
            SNPMI_REPACK_WIN(4);
        } else if (P.K == 2) {
            SNPMI_REPACK_WIN(2);
        } else {
            SNPMI_REPACK_WIN(1);
        }
#undef SNPMI_REPACK_WIN
    } else if (P.plan != nullptr && nq * 16 + 16 <= kRepackLds && fits) {
        const int K = P.K;
        SNPMI_REQUIRE(nq <= (uint64_t)kRepackPre[K >> 1] * 1024, SNPMI_E_ARG, "repack staging exceeds its registers");
        const uint64_t ng = ceil_div(n_sid, (uint64_t)K);
        // one workgroup per CU (LDS), each walking several groups so the next one's loads overlap
        const unsigned grid = (unsigned)std::min<uint64_t>(ng, 256 * 2);
        const size_t lds = (size_t)(K * nq + 1) * 16;
#define SNPMI_REPACK(KK)                                                                                            \
    SNPMI_HIP(hipFuncSetAttribute((const void*)k_repack_lds<KK>, hipFuncAttributeMaxDynamicSharedMemorySize,      \
                                  (int)kRepackLds));                                                                \
    k_repack_lds<KK><<<grid, 1024, lds, st>>>(src, src_pitch, nq, n_sid, P.plan, n_out, dst, dst_pitch)
        if (K == 4) {
            SNPMI_REPACK(4);
        } else if (K == 2) {
            SNPMI_REPACK(2);
        } else {
            SNPMI_REPACK(1);
        }
#undef SNPMI_REPACK
    } else {
        SNPMI_HIP(hipMemsetAsync(dst, 0, n_sid * dst_pitch, st));
        if (n_out == 0) return;
        const unsigned g = grid_for(ceil_div(n_out, 16) * n_sid, kBlock);
        k_repack<<<g, kBlock, 0, st>>>(src, src_pitch, idx, n_out, n_sid, dst, dst_pitch);
    }
    SNPMI_LAUNCH_CHECK();
}

void launch_dense_codes(const float* Z, uint64_t ldz, uint64_t n, uint64_t m, uint8_t* packed, uint64_t pitch,
                        float* lut, unsigned int* flag, hipStream_t st) {
    SNPMI_HIP(hipMemsetAsync(flag, 0, sizeof(unsigned int), st));
    if (m == 0) return;
    SNPMI_REQUIRE(m < (1ull << 31) && pitch % 4 == 0 && pitch * 4 >= n, SNPMI_E_ARG, "bad dense-codes shape");
    k_dense_codes<<<(unsigned)m, 256, 0, st>>>(Z, ldz, n, packed, pitch, lut, flag);
    SNPMI_LAUNCH_CHECK();
}

void launch_dense_standardize(void* val, uint64_t rows, uint64_t cols, uint64_t ld, int order_c, int dtype,
                              int std_kind, double a, double b, int use_stats, void* stats, hipStream_t st) {
    if (cols == 0 || std_kind == SNPMI_STD_NONE) return;
    const size_t es = dtype == SNPMI_DT_F32 ? 4 : 8;
    if (!order_c) {
        auto general = [&](const uint8_t* only) {
            const unsigned gw = grid_for(cols, kBlock / kWave);
            if (dtype == SNPMI_DT_F32)
                k_std_dense_f<float><<<gw, kBlock, 0, st>>>((float*)val, rows, cols, ld, std_kind, a, b, use_stats,
                                                            (float*)stats, only);
            else
                k_std_dense_f<double><<<gw, kBlock, 0, st>>>((double*)val, rows, cols, ld, std_kind, a, b, use_stats,
                                                             (double*)stats, only);
            SNPMI_LAUNCH_CHECK();
        };
        if (g_variant_std == 1) {  // A/B: round 3's wave-per-column kernel for every column
            general(nullptr);
            return;
        }
        // genotype columns: one workgroup per column, the smallest (threads, vectors per thread)
        // that keeps the whole column in registers, else 1024 x 8 in chunks (two reads); columns
        // with other values are flagged and then standardized by the general kernel
        Device& d = device();
        uint8_t* flags = (uint8_t*)d.get(Device::S_STDFLAG, round_up(cols, 256) + 256);
        unsigned int* any = (unsigned int*)(flags + round_up(cols, 256));
        SNPMI_HIP(hipMemsetAsync(flags, 0, round_up(cols, 256) + 4, st));
        const uint64_t nvec = rows * es / 16 + 1;
        const unsigned g = (unsigned)std::min<uint64_t>(cols, 1u << 20);
        const bool beta = std_kind == SNPMI_STD_BETA;
#define SNPMI_STD_F(NT, NV, BETA)                                                                                   \
    do {                                                                                                            \
        if (dtype == SNPMI_DT_F32)                                                                                  \
            k_std_cols_f<float, NT, NV, BETA><<<g, NT, 0, st>>>((float*)val, rows, cols, ld, std_kind, a, b,        \
                                                                use_stats, (float*)stats, flags, any);              \
        else                                                                                                        \
            k_std_cols_f<double, NT, NV, BETA><<<g, NT, 0, st>>>((double*)val, rows, cols, ld, std_kind, a, b,      \
                                                                 use_stats, (double*)stats, flags, any);            \
    } while (0)
        if (beta) {
            if (nvec <= 256 * 4) SNPMI_STD_F(256, 4, true);
            else if (nvec <= 256 * 16) SNPMI_STD_F(256, 16, true);
            else if (nvec <= 1024 * 8) SNPMI_STD_F(1024, 8, true);
            else if (nvec <= 1024 * 16) SNPMI_STD_F(1024, 16, true);
            else SNPMI_STD_F(1024, 8, true);
        } else if (nvec <= 256 * 4) SNPMI_STD_F(256, 4, false);
        else if (nvec <= 256 * 16) SNPMI_STD_F(256, 16, false);
        else if (nvec <= 1024 * 8) SNPMI_STD_F(1024, 8, false);
        else if (nvec <= 1024 * 16) SNPMI_STD_F(1024, 16, false);
        else SNPMI_STD_F(1024, 8, false);
#undef SNPMI_STD_F
        SNPMI_LAUNCH_CHECK();
        unsigned int h_any = 0;
        SNPMI_HIP(hipMemcpyAsync(&h_any, any, 4, hipMemcpyDeviceToHost, st));
        SNPMI_HIP(hipStreamSynchronize(st));
        if (h_any) general(flags);
        return;
    }
    const bool vec16 = reinterpret_cast<uintptr_t>(val) % 16 == 0 && (ld * es) % 16 == 0 && g_variant_std != 1;
    if (vec16) {
        const unsigned g = grid_for(cols, kWave * (16 / es));
        if (dtype == SNPMI_DT_F32)
            k_std_cols_c16<float><<<g, kBlock, 0, st>>>((float*)val, rows, cols, ld, std_kind, a, b, use_stats,
                                                        (float*)stats);
        else
            k_std_cols_c16<double><<<g, kBlock, 0, st>>>((double*)val, rows, cols, ld, std_kind, a, b, use_stats,
                                                         (double*)stats);
    } else {
        const unsigned g = grid_for(cols, 64);
        if (dtype == SNPMI_DT_F32)
            k_std_dense_c<float><<<g, kBlock, 0, st>>>((float*)val, rows, cols, ld, std_kind, a, b, use_stats,
                                                       (float*)stats);
        else
            k_std_dense_c<double><<<g, kBlock, 0, st>>>((double*)val, rows, cols, ld, std_kind, a, b, use_stats,
                                                        (double*)stats);
    }
    SNPMI_LAUNCH_CHECK();
}

void launch_subset(const void* in, int in_dt, uint64_t rows, uint64_t cols, uint64_t k, int in_c, const uint64_t* ri,
                   uint64_t nr, const uint64_t* ci, uint64_t nc, int out_c, void* out, int out_dt, hipStream_t st) {
    const uint64_t total = nr * nc * k;
    if (total == 0) return;
    const unsigned g = grid_for(total, kBlock);
    if (in_dt == SNPMI_DT_F64 && out_dt == SNPMI_DT_F64)
        k_subset<double, double><<<g, kBlock, 0, st>>>((const double*)in, rows, cols, k, in_c, ri, nr, ci, nc, out_c,
                                                       (double*)out);
    else if (in_dt == SNPMI_DT_F32 && out_dt == SNPMI_DT_F64)
        k_subset<float, double><<<g, kBlock, 0, st>>>((const float*)in, rows, cols, k, in_c, ri, nr, ci, nc, out_c,
                                                      (double*)out);
    else if (in_dt == SNPMI_DT_F32 && out_dt == SNPMI_DT_F32)
        k_subset<float, float><<<g, kBlock, 0, st>>>((const float*)in, rows, cols, k, in_c, ri, nr, ci, nc, out_c,
                                                     (float*)out);
    else
        throw Error(SNPMI_E_ARG, "unsupported subset dtype pair");
    SNPMI_LAUNCH_CHECK();
}

void launch_transpose_to_f(const void* in, uint64_t rows, uint64_t cols, int dtype, void* out, uint64_t ld,
                           hipStream_t st) {
    if (rows == 0 || cols == 0) return;
    const unsigned g = grid_for(ceil_div(rows, 64) * ceil_div(cols, 64), 1, 256 * 8);
    if (dtype == SNPMI_DT_F32)
        k_transpose<float><<<g, kBlock, 0, st>>>((const float*)in, rows, cols, (float*)out, ld);
    else
        k_transpose<double><<<g, kBlock, 0, st>>>((const double*)in, rows, cols, (double*)out, ld);
    SNPMI_LAUNCH_CHECK();
}

void launch_grm_extract(const void* tiles, uint64_t, int dtype, const uint64_t* ri, uint64_t nr, const uint64_t* ci,
                        uint64_t nc, int order_c, double scale, void* out, hipStream_t st) {
    if (nr == 0 || nc == 0) return;
    const unsigned g = grid_for(nr * nc, kBlock, 256 * 32);
    if (dtype == SNPMI_DT_F32)
        k_grm_extract<float><<<g, kBlock, 0, st>>>((const float*)tiles, ri, nr, ci, nc, order_c, scale, (float*)out);
    else
        k_grm_extract<double><<<g, kBlock, 0, st>>>((const double*)tiles, ri, nr, ci, nc, order_c, scale,
                                                    (double*)out);
    SNPMI_LAUNCH_CHECK();
}

void launch_grm_extract_rows(const void* tiles, uint64_t n, int dtype, uint64_t r0, uint64_t nr, double scale,
                             void* out, hipStream_t st) {
    if (nr == 0 || n == 0) return;
    if (r0 == 0 && nr == n && g_variant_extract == 0) {  // the whole K: each upper block read once
        const uint64_t bs = dtype == SNPMI_DT_F32 ? 128 : 64, nb = (n + bs - 1) / bs;
        const unsigned g = grid_for(nb * (nb + 1) / 2, 1, 256 * 16);
        // f32: 128x128 blocks (one 64 KB tile) on 512 threads; f64: 64x64 on 256 (the other
        // shapes of hook "extract" 2-4 were within 2-6% either way, profiles/r04f/extract_ab.jsonl)
        if (dtype == SNPMI_DT_F32)
            k_grm_extract_sym<float, 128, 512><<<g, 512, 0, st>>>((const float*)tiles, n, scale, (float*)out);
        else
            k_grm_extract_sym<double, 64><<<g, kBlock, 0, st>>>((const double*)tiles, n, scale, (double*)out);
        SNPMI_LAUNCH_CHECK();
        return;
    }
    if (r0 == 0 && nr == n && g_variant_extract >= 5) {  // A/B: the pipelined read-once kernel
        const int v = g_variant_extract;
        const bool f32 = dtype == SNPMI_DT_F32;
        const uint64_t bs = v == 6 || (v == 5 && f32) ? 128 : 64, nb = (n + bs - 1) / bs;
        const unsigned g = grid_for(nb * (nb + 1) / 2, 1, 256 * 16);
        if (f32) {
            if (v == 5) k_grm_extract_sym<float, 128, 512, true><<<g, 512, 0, st>>>((const float*)tiles, n, scale, (float*)out);
            else if (v == 6) k_grm_extract_sym<float, 128, 1024, true><<<g, 1024, 0, st>>>((const float*)tiles, n, scale, (float*)out);
            else k_grm_extract_sym<float, 64, kBlock, true><<<g, kBlock, 0, st>>>((const float*)tiles, n, scale, (float*)out);
        } else {
            if (v == 5) k_grm_extract_sym<double, 64, kBlock, true><<<g, kBlock, 0, st>>>((const double*)tiles, n, scale, (double*)out);
            else if (v == 6) k_grm_extract_sym<double, 128, 1024, true><<<g, 1024, 0, st>>>((const double*)tiles, n, scale, (double*)out);
            else k_grm_extract_sym<double, 64, 512, true><<<g, 512, 0, st>>>((const double*)tiles, n, scale, (double*)out);
        }
        SNPMI_LAUNCH_CHECK();
        return;
    }
    if (r0 == 0 && nr == n && g_variant_extract >= 2) {  // A/B shapes of the read-once kernel
        const int v = g_variant_extract;
        const uint64_t bs = v == 2 || v == 4 ? 128 : 64, nb = (n + bs - 1) / bs;
        const unsigned g = grid_for(nb * (nb + 1) / 2, 1, 256 * 16);
        if (dtype == SNPMI_DT_F32) {
            if (v == 2) k_grm_extract_sym<float, 128, 512><<<g, 512, 0, st>>>((const float*)tiles, n, scale, (float*)out);
            else if (v == 3) k_grm_extract_sym<float, 64><<<g, kBlock, 0, st>>>((const float*)tiles, n, scale, (float*)out);
            else k_grm_extract_sym<float, 128, 1024><<<g, 1024, 0, st>>>((const float*)tiles, n, scale, (float*)out);
        } else {
            if (v == 2) k_grm_extract_sym<double, 128, 512><<<g, 512, 0, st>>>((const double*)tiles, n, scale, (double*)out);
            else if (v == 3) k_grm_extract_sym<double, 64, 512><<<g, 512, 0, st>>>((const double*)tiles, n, scale, (double*)out);
            else k_grm_extract_sym<double, 128, 1024><<<g, 1024, 0, st>>>((const double*)tiles, n, scale, (double*)out);
        }
        SNPMI_LAUNCH_CHECK();
        return;
    }
    const uint64_t blocks = ((r0 + nr + 63) / 64 - r0 / 64) * ((n + 63) / 64);
    const unsigned g = grid_for(blocks, 1, 256 * 16);
    if (dtype == SNPMI_DT_F32)
        k_grm_extract_rows<float><<<g, kBlock, 0, st>>>((const float*)tiles, n, r0, nr, scale, (float*)out);
    else
        k_grm_extract_rows<double><<<g, kBlock, 0, st>>>((const double*)tiles, n, r0, nr, scale, (double*)out);
    SNPMI_LAUNCH_CHECK();
}

void launch_grm_trace(const void* tiles, uint64_t n, int dtype, double* trace_dev, hipStream_t st) {
    if (dtype == SNPMI_DT_F32)
        k_grm_trace<float><<<1, kBlock, 0, st>>>((const float*)tiles, n, trace_dev);
    else
        k_grm_trace<double><<<1, kBlock, 0, st>>>((const double*)tiles, n, trace_dev);
    SNPMI_LAUNCH_CHECK();
}

void launch_part_extract(const void* blocks, const int32_t* lslot, int dtype, const uint64_t* ri, uint64_t nr,
                         const uint64_t* ci, uint64_t nc, int order_c, double scale, void* out, hipStream_t st) {
    if (nr == 0 || nc == 0) return;
    const unsigned g = grid_for(nr * nc, kBlock, 256 * 32);
    if (dtype == SNPMI_DT_F32)
        k_part_extract<float><<<g, kBlock, 0, st>>>((const float*)blocks, lslot, ri, nr, ci, nc, order_c, scale,
                                                    (float*)out);
    else
        k_part_extract<double><<<g, kBlock, 0, st>>>((const double*)blocks, lslot, ri, nr, ci, nc, order_c, scale,
                                                     (double*)out);
    SNPMI_LAUNCH_CHECK();
}

void launch_part_trace(const void* blocks, const int32_t* dslot, uint64_t n, int dtype, double* trace_dev,
                       hipStream_t st) {
    if (dtype == SNPMI_DT_F32)
        k_part_trace<float><<<1, kBlock, 0, st>>>((const float*)blocks, dslot, n, trace_dev);
    else
        k_part_trace<double><<<1, kBlock, 0, st>>>((const double*)blocks, dslot, n, trace_dev);
    SNPMI_LAUNCH_CHECK();
}

void launch_dense_trace(const void* K, uint64_t n, int dtype, double* trace_dev, hipStream_t st) {
    if (dtype == SNPMI_DT_F32)
        k_dense_trace<float><<<1, kBlock, 0, st>>>((const float*)K, n, trace_dev);
    else
        k_dense_trace<double><<<1, kBlock, 0, st>>>((const double*)K, n, trace_dev);
    SNPMI_LAUNCH_CHECK();
}

void launch_dense_scale(void* p, uint64_t count, int dtype, double scale, hipStream_t st) {
    if (count == 0) return;
    const unsigned g = grid_for(count, kBlock, 256 * 32);
    if (dtype == SNPMI_DT_F32)
        k_scale<float><<<g, kBlock, 0, st>>>((float*)p, count, scale);
    else
        k_scale<double><<<g, kBlock, 0, st>>>((double*)p, count, scale);
    SNPMI_LAUNCH_CHECK();
}

void launch_sumsq(const void* p, uint64_t count, int dtype, double* out_dev, hipStream_t st) {
    SNPMI_HIP(hipMemsetAsync(out_dev, 0, sizeof(double), st));
    if (count == 0) return;
    const unsigned g = grid_for(count, kBlock, 1024);
    if (dtype == SNPMI_DT_F32)
        k_sumsq<float><<<g, kBlock, 0, st>>>((const float*)p, count, out_dev);
    else
        k_sumsq<double><<<g, kBlock, 0, st>>>((const double*)p, count, out_dev);
    SNPMI_LAUNCH_CHECK();
}

// Streaming device copy (16-B loads/stores, 4 in flight per thread, grid-stride): the measured
// HBM copy peak bench.py reports beside the decode roofline (hipMemcpy D2D's blit kernel
// reached only 4.9 TB/s on the same box).
__global__ __launch_bounds__(kBlock) void k_copy16(const u32x4_t* __restrict__ src, u32x4_t* __restrict__ dst,
                                                   uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const u32x4_t a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride);
        const u32x4_t c = __builtin_nontemporal_load(src + i + 2 * stride);
        const u32x4_t d = __builtin_nontemporal_load(src + i + 3 * stride);
        __builtin_nontemporal_store(a, dst + i);
        __builtin_nontemporal_store(b, dst + i + stride);
        __builtin_nontemporal_store(c, dst + i + 2 * stride);
        __builtin_nontemporal_store(d, dst + i + 3 * stride);
    }
    for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

void launch_copy16(const void* src, void* dst, uint64_t bytes, hipStream_t st) {
    const uint64_t n16 = bytes / 16;
    if (n16 == 0) return;
    k_copy16<<<grid_for(ceil_div(n16, 4), kBlock, 256 * 8 * 4), kBlock, 0, st>>>((const u32x4_t*)src, (u32x4_t*)dst, n16);
    SNPMI_LAUNCH_CHECK();
}

// tiles = (accumulate ? tiles : 0) + sum of `slices` partial tile sets (split-K GRM), in order
__global__ __launch_bounds__(kBlock) void k_tile_reduce(const f32x4_t* __restrict__ part, unsigned slices,
                                                        uint64_t n4, f32x4_t* __restrict__ tiles, int accumulate) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * kBlock) {
        f32x4_t acc = accumulate ? tiles[i] : (f32x4_t){0.f, 0.f, 0.f, 0.f};
        for (unsigned s = 0; s < slices; s++) acc += part[s * n4 + i];
        tiles[i] = acc;
    }
}

void launch_tile_reduce(const float* partial, unsigned slices, uint64_t elems, float* tiles, int accumulate,
                        hipStream_t st) {
    const uint64_t n4 = elems / 4;  // tile sets are multiples of 128x128 floats
    if (n4 == 0) return;
    k_tile_reduce<<<grid_for(n4, kBlock, 256 * 16), kBlock, 0, st>>>((const f32x4_t*)partial, slices, n4,
                                                                      (f32x4_t*)tiles, accumulate);
    SNPMI_LAUNCH_CHECK();
}

void launch_diag_begin(const float* K, uint64_t n, const int32_t* dslot, int accumulate, double* diag, hipStream_t st) {
    if (n == 0) return;
    k_diag_save<<<grid_for(n, kBlock), kBlock, 0, st>>>(K, n, dslot, accumulate, diag);
    SNPMI_LAUNCH_CHECK();
}

// SNP slices of k_diag_sq: ~1M (word, slice) threads, slices of >= 64 SNPs.  Each thread's loop has
// one dependent code load per SNP, so the kernel is latency-bound and needs the waves: round 4's
// ~262k threads (9 slices at 500k iids) ran a 32768-SNP block in 6.1 ms (0.7 TB/s of codes)
static uint64_t diag_slices(uint64_t n, uint64_t m) {
    const uint64_t nw = (n + 15) / 16;
    return std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(std::max<uint64_t>(m, 1), 64), ceil_div(1024 * 1024, nw)));
}
// diag (n f64, from round_up(n, 16)) followed by the per-slice partial rows
uint64_t diag_scratch_bytes(uint64_t n, uint64_t m) {
    return (1 + diag_slices(n, m)) * round_up(std::max<uint64_t>(n, 1), 16) * sizeof(double);
}

void launch_diag_sq(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const float* lut, double* diag,
                    hipStream_t st) {
    if (n == 0 || m == 0) return;
    const uint64_t nw = (n + 15) / 16, bx = ceil_div(nw, kBlock), ld = round_up(n, 16);
    const uint64_t per = ceil_div(m, diag_slices(n, m)), slices = ceil_div(m, per);
    double* part = diag + ld;
    k_diag_sq<<<dim3((unsigned)bx, (unsigned)slices), kBlock, 0, st>>>(packed, pitch, n, m, lut, per, ld, part);
    SNPMI_LAUNCH_CHECK();
    k_diag_fold<<<grid_for(n, kBlock), kBlock, 0, st>>>(n, slices, ld, part, diag);
    SNPMI_LAUNCH_CHECK();
}

void launch_diag_patch(float* K, uint64_t n, uint64_t i0, uint64_t i1, const int32_t* dslot, const double* diag,
                       hipStream_t st) {
    i1 = std::min(i1, n);
    if (i0 >= i1) return;
    k_diag_patch<<<grid_for(i1 - i0, kBlock), kBlock, 0, st>>>(K, i0, i1, dslot, diag);
    SNPMI_LAUNCH_CHECK();
}

void launch_diag_end(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const float* lut, float* K,
                     const int32_t* dslot, double* diag, hipStream_t st) {
    if (n == 0) return;
    launch_diag_sq(packed, pitch, n, m, lut, diag, st);
    launch_diag_patch(K, n, 0, n, dslot, diag, st);
}

void launch_synth(uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t sid0, uint64_t m, uint64_t seed,
                  double miss_rate, const double* maf_x, const double* maf_cdf, int n_pts, hipStream_t st) {
    if (m == 0) return;
    const unsigned g = grid_for(pitch / 4 * m, kBlock, 256 * 32);
    k_synth<<<g, kBlock, 0, st>>>(packed, pitch, n, sid0, m, seed, miss_rate, maf_x, maf_cdf, n_pts);
    SNPMI_LAUNCH_CHECK();
}

}  // namespace snpmi
