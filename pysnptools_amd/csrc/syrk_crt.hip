// f64 GRM of packed SNPs on the int8 MFMA pipe: exact integer products in a residue number system.
//
// Reference: SnpReader._read_kernel (snpreader.py:637-668) accumulates K = sum_b Z_b Z_b^T in
// float64 (the reference's default dtype).  gfx950's f64 MFMA peaks at 78.6 TFLOP/s; its int8
// MFMA at ~5 POP/s.  Per launch (one SNP block, m SNPs):
//   1. every LUT value a (standardized value of a SNP for one of its 4 codes) becomes the integer
//      q = rint(a * 2^(F - e)), |q| <= 2^F, with e = the block's exponent (max |a| <= 2^e); the
//      quantisation error is <= 2^(e - F - 1), i.e. 2^-(F+1) of the block's largest value;
//   2. K_int = sum_s q_is q_js is an exact integer with |K_int| <= m 2^2F < P/2, P = product of
//      R pairwise-coprime moduli p <= 256; for each modulus the int8 MFMA computes
//      sum_s rho(q_is) rho(q_js) with rho = q mod p in [-p/2, p/2) (|rho| <= 128, exact int32
//      accumulation for m <= 2^17) and the epilogue keeps it mod p (one byte per K element);
//   3. k_crt rebuilds K_int from its R residues (Garner's mixed-radix digits, exact), converts to
//      f64 (Horner, one rounding per step) and adds K_int 2^(2(e - F)) to the f64 K tiles.
// kR = 15 moduli (P ~ 2^117.8): F = floor((log2 P - 1 - log2 m) / 2) = 51 at m = 10k, so every
// value keeps its bits down to 2^-52 of the block's largest -- the f64 product K's own rounding
// level.  That F is fixed by the worst case |K_int| <= m 2^2F; the block's actual bound is
// |K_int,ij| <= sqrt(K_int,ii K_int,jj) <= max_i sum_s q_is^2 (Cauchy-Schwarz), which k_crt_bound
// computes per iid on the device (rare-variant LUT values set e, so typical blocks sit 10-13 bits
// below the worst case), and only the first R <= kR moduli with P_R > 2 max_i sum_s q_is^2 run
// (the SYRK workgroups of moduli >= R exit at once, k_crt's Garner stops at R).  A block whose LUT holds NaN/Inf raises a flag on the device and the f64 MFMA kernel
// (gated on the flag) computes it instead.
#include "snpmi_internal.hpp"

#include <cmath>

namespace snpmi {
namespace {

constexpr int kR = 15;
// pairwise coprime, <= 256 (symmetric residues fit int8): 2^8, 3*5*17, 11*23, 251, 13*19, 241, 239,
// 233, 229, 227, 223, 7*31, 211, 199, 197 -- P ~ 2^117.8
constexpr int mod_of(int i) {
    constexpr int m[kR] = {256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197};
    return m[i];
}
__constant__ int kMod[kR] = {256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197};

constexpr int BW = 256;    // block edge (iids)
constexpr int SK = 128;    // SNPs per LDS stage (four 32-deep MFMA k-steps): 147 KiB of LDS, double-buffered
constexpr int RS = 288;    // LDS bytes per SNP row (256 iids + 32: the 8 rows of a transposed read hit distinct banks)

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void tile_coords(uint64_t L, uint32_t& ti, uint32_t& tj) {
    uint64_t j = (uint64_t)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while ((j + 1) * (j + 2) / 2 <= L) j++;
    while (j * (j + 1) / 2 > L) j--;
    tj = (uint32_t)j;
    ti = (uint32_t)(L - j * (j + 1) / 2);
}

__device__ __forceinline__ int pi16(int p) { return 4 * (p & 3) + (p >> 2); }

// ---------------------------------------------------------------- block exponent + range flag
// ctl[0] = e (max |a| <= 2^e, 0 for an all-zero block), ctl[1] = 1 if any LUT value is NaN/Inf
__global__ __launch_bounds__(1024) void k_crt_exp(const double* __restrict__ lut, uint64_t cnt, int* __restrict__ ctl) {
    double M = 0.0;
    int bad = 0;
    for (uint64_t i = threadIdx.x; i < cnt; i += 1024) {
        const double v = lut[i];
        if (!isfinite(v)) bad = 1;
        else M = fmax(M, fabs(v));
    }
    __shared__ double red[1024];
    __shared__ int rb[1024];
    red[threadIdx.x] = M;
    rb[threadIdx.x] = bad;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
            rb[threadIdx.x] |= rb[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        int e = 0;
        if (red[0] > 0.0) frexp(red[0], &e);  // red = f 2^e, f in [0.5, 1)
        ctl[0] = e;
        ctl[1] = rb[0];
    }
}

// residue LUT: lutr[r * mpad + s] byte c = rho_r(q_s[c]) (int8), zero for s >= m
// qsq[4 s + c] = q_s[c]^2 in f64 (the bound table of k_crt_bound; 0 for s >= m)
__global__ __launch_bounds__(256) void k_crt_lut(const double* __restrict__ lut, uint64_t m, uint64_t mpad, int F,
                                                 const int* __restrict__ ctl, uint32_t* __restrict__ lutr,
                                                 double* __restrict__ qsq) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= mpad) return;
    const int e = ctl[0];
    long long q[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const double a = s < m && !ctl[1] ? lut[4 * s + c] : 0.0;
        q[c] = (long long)rint(ldexp(a, F - e));
        qsq[4 * s + c] = (double)q[c] * (double)q[c];
    }
#pragma unroll
    for (int r = 0; r < kR; r++) {
        const long long p = kMod[r];
        uint32_t w = 0;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            long long x = q[c] % p;
            if (x < 0) x += p;
            if (x >= (p + 1) / 2) x -= p;  // [-128, 127] for 256, +-(p-1)/2 otherwise
            w |= ((uint32_t)x & 0xffu) << (8 * c);
        }
        lutr[(uint64_t)r * mpad + s] = w;
    }
}

// ---------------------------------------------------------------- per-block modulus count
// S[i] += sum_s q_is^2 over a slice of kBoundSlice SNPs: thread = 16 iids (one code dword per SNP,
// the SNP's 4 table values are wave-uniform), one f64 atomic add per iid and slice.  f64 sums of
// integers <= 2^104: relative error <= kBoundSlice 2^-53 per slice, covered by k_crt_r's margin.
constexpr int kBoundSlice = 256;
__global__ __launch_bounds__(256) void k_crt_bound(const uint8_t* __restrict__ P, uint64_t pitch, uint64_t n,
                                                   uint64_t m, const double* __restrict__ qsq,
                                                   const int* __restrict__ ctl, double* __restrict__ S) {
    if (ctl[1]) return;
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= (n + 15) / 16) return;
    const uint64_t s0 = (uint64_t)blockIdx.y * kBoundSlice, s1 = min(m, s0 + kBoundSlice);
    double acc[16];
#pragma unroll
    for (int k = 0; k < 16; k++) acc[k] = 0.0;
    for (uint64_t s = s0; s < s1; s++) {
        const uint32_t x = *reinterpret_cast<const uint32_t*>(P + s * pitch + 4 * w);
        const double t0 = qsq[4 * s], t1 = qsq[4 * s + 1], t2 = qsq[4 * s + 2], t3 = qsq[4 * s + 3];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t c = (x >> (2 * k)) & 3u;
            acc[k] += c & 2u ? (c & 1u ? t3 : t2) : (c & 1u ? t1 : t0);
        }
    }
#pragma unroll
    for (int k = 0; k < 16; k++)
        if (16 * w + k < n) atomicAdd(S + 16 * w + k, acc[k]);
}

// ctl[2] = R: the fewest moduli with P_R > 2 max_i S[i] (1 + 2^-20); plog[r] = log2 P_{r+1} (host)
struct CrtLog {
    double plog[kR];
    int per_block;  // 0: every block runs the launch-wide ctl[2] moduli (hook "crt_block" = 0)
};
__global__ __launch_bounds__(1024) void k_crt_r(const double* __restrict__ S, uint64_t n, CrtLog L,
                                               int* __restrict__ ctl, unsigned long long* __restrict__ rec) {
    double M = 0.0;
    for (uint64_t i = threadIdx.x; i < n; i += 1024) M = fmax(M, S[i]);
    __shared__ double red[1024];
    red[threadIdx.x] = M;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        int R = kR;
        if (!ctl[1]) {
            const double need = red[0] > 0.0 ? log2(red[0] * (1.0 + 0x1p-20)) + 1.0 : 0.0;
            R = 1;
            while (R < kR && L.plog[R - 1] <= need) R++;
        }
        ctl[2] = R;
        if (rec) {
            atomicAdd(rec, (unsigned long long)R);
            atomicAdd(rec + 1, 1ull);
        }
    }
}

// Per 256-iid panel p: lgp[p] = log2(max_{i in p} S[i] (1 + 2^-20)) (-inf for an all-zero panel).
// The block (bi, bj) then needs only the moduli with P_R > 2 sqrt(M_bi M_bj): |K_int,ij| <=
// sqrt(S_i S_j) <= sqrt(M_bi M_bj) (Cauchy-Schwarz).  The launch-wide R (ctl[2]) is the largest of
// these; blocks whose panels hold no extreme iid (the rare-variant carriers that set max_i S[i])
// skip one modulus or more, and K_int is exact either way, so K is the same bits.
__global__ __launch_bounds__(256) void k_crt_panels(const double* __restrict__ S, uint64_t n, const int* __restrict__ ctl,
                                                    double* __restrict__ lgp) {
    if (ctl[1]) return;
    const uint64_t i = (uint64_t)blockIdx.x * BW + threadIdx.x;
    __shared__ double red[256];
    red[threadIdx.x] = i < n ? S[i] : 0.0;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) lgp[blockIdx.x] = red[0] > 0.0 ? log2(red[0] * (1.0 + 0x1p-20)) : -__builtin_inf();
}

// moduli the 256-block (bi, bj) needs (1 <= R_b <= ctl[2]); the same formula as k_crt_r's
__device__ __forceinline__ int block_moduli(const double* __restrict__ lgp, uint32_t bi, uint32_t bj, const CrtLog& L,
                                            const int* __restrict__ ctl) {
    if (!L.per_block) return ctl[2];
    const double need = 0.5 * (lgp[bi] + lgp[bj]) + 1.0;
    int R = 1;
    while (R < kR && L.plog[R - 1] <= need) R++;
    return R;
}

__device__ __forceinline__ v2i lds_tr8(const uint8_t* p) {
    return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)p);
}

// acc mod p -> [0, p), one byte per element at its true (row, col) in the 256 x 256 block (a wave's
// 128 x 64 = 4 x 2 tiles of v_mfma_i32_32x32x32_i8 accumulators, wave (wm, wn) of a 2 x 4 layout)
__device__ __forceinline__ void crt_epilogue(const v16i (&acc)[4][2], uint32_t r, uint64_t nblk, uint64_t bx, int wm,
                                             int wn, int lane, uint8_t* __restrict__ res) {
    const int p = kMod[r];
    const double invp = 1.0 / (double)p;
    uint8_t* O = res + ((uint64_t)r * nblk + bx) * (BW * BW);
    const int hh = lane >> 5, colp = 16 * ((lane >> 4) & 1) + pi16(lane & 15);
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) {
            uint8_t* bp = O + (wm * 128 + 32 * x + hh) * BW + wn * 64 + 32 * y + colp;
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const int v = acc[x][y][q];
                int rr = v - p * (int)floor((double)v * invp);
                rr += rr < 0 ? p : 0;
                rr -= rr >= p ? p : 0;
                bp[(16 * (q >> 3) + 4 * (q & 3) + 2 * ((q >> 2) & 1)) * BW] = (uint8_t)rr;
            }
        }
}

// ---------------------------------------------------------------- residue SYRK
// Grid (1-D, round_up(nblk, 8) * kR workgroups): workgroup w runs on XCD w % 8; its kR consecutive
// slots there are the kR moduli of block 8 (w / 8 / kR) + w % 8, so the workgroups an XCD holds at
// once share their code panels in that XCD's L2 (FETCH 951 -> 149 GB per 62.5k-SNP launch at 50k
// iids vs a (blocks, moduli) grid, profiles/r05m).  Block (bi, bj) = upper-triangle 256-block
// b0 + bx (or slot b0 + bx of a cfg5 part's layout), modulus kMod[r].
// 8 waves (2 x 4), each 128 x 64 = 4 x 2 v_mfma_i32_32x32x32_i8 tiles.
// LDS: per stage and panel SKT SNP rows x 256 iids of int8 residues ([k][iid], RS-byte rows, the
// 16 iids of a group in pi16 order as the loader's byte permutes leave them), double-buffered.
// Loader: thread (panel lp, 16-iid group d, row block kq) expands SKT/16 consecutive SNP rows
// per stage: one code dword per row, 16-B LUT loads, 4 v_perm per row.  MFMA operand
// (32x32x32 i8): lane l holds row l&31, k = 16(l>>5) + j (j < 16), read as two
// ds_read_b64_tr_b8 of 8 SNP rows: within a 16-lane group, lane 2j+p addresses row j, bytes
// 8p..8p+7 and receives column (its group-lane index) of the 8 rows (tools/probe/tr8_probe.hip).
// Per 32-SNP k-step: the next k-step's fragments are read under this one's 8 MFMAs, and a
// share of the next stage's rows is expanded and stored; one barrier per stage.  The loader runs
// unconditionally (the last stage expands into the idle buffer, its code loads clamp to the last
// stage) so each k-step's MFMAs and loader VALU share a basic block.
// Epilogue: residue of each int32 sum, one byte per element, written as a dense 256 x 256 block
// (true iid order) at res + (r * nblk + bx) * 65536.
template <int SKT>
__global__ __launch_bounds__(512, 1) void k_syrk_i8r(const uint8_t* __restrict__ P, uint64_t pitch, uint64_t kdim,
                                                     uint64_t mpad, const uint32_t* __restrict__ lutr,
                                                     const int* __restrict__ ctl, uint64_t b0, uint64_t nblk,
                                                     uint8_t* __restrict__ res, const double* __restrict__ lgp, CrtLog L,
                                                     const uint32_t* __restrict__ part_tab = nullptr) {
    constexpr int KS = SKT / 32, RPT = SKT / 16, PNL = SKT * RS, STG = 2 * PNL;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STG];
    if (ctl[1]) return;  // non-finite LUT: the f64 MFMA kernel runs instead
    const uint32_t w = blockIdx.x, q = w >> 3, u = q / kR;
    const uint32_t r = q - u * kR, bx = 8 * u + (w & 7);
    if (bx >= nblk) return;
    const uint32_t* lr = lutr + (uint64_t)r * mpad;
    uint32_t bi, bj;
    if (part_tab) {  // cfg5: slot b0 + bx of the part's layout (syrk.hip part_layout)
        const uint32_t c = part_tab[b0 + bx];
        bi = c & 0xffffu;
        bj = c >> 16;
    } else {
        tile_coords(b0 + bx, bi, bj);
    }
    if ((int)r >= block_moduli(lgp, bi, bj, L, ctl)) return;  // this block's K_int fits the first R_b moduli
    const uint64_t i0 = (uint64_t)bi * BW, j0 = (uint64_t)bj * BW;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    // loader role: panel lp (wave-uniform), rows RPT kq .. RPT kq + RPT-1 of the stage, 16-iid
    // group d.  Code loads: wave-uniform 64-bit base + 32-bit per-lane offset, the row clamped to
    // the block's last SNP (its LUT words are zero past kdim: lutr is zero-padded to mpad)
    const int lp = __builtin_amdgcn_readfirstlane(t >> 8), kq = (t >> 4) & 15, d = t & 15;
    const uint8_t* pbase = P + (lp ? j0 : i0) / 4;
    const uint32_t pit = (uint32_t)pitch;
    const uint32_t* lq = lr + RPT * kq;
    // transposed-read role: group g = lane>>4 covers k half h = g>>1 and columns 16(g&1)..+15
    const int g = lane >> 4, jj = (lane & 15) >> 1, pp = lane & 1;
    const int rd = (16 * (g >> 1) + jj) * RS + 16 * (g & 1) + 8 * pp;

    v16i acc[4][2];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = (v16i){};
    const uint64_t nst = (kdim + SKT - 1) / SKT;

    uint32_t cw[RPT];
    uint4 cl[RPT / 4];
    auto load = [&](uint64_t st) {
        const uint8_t* sb = pbase + st * SKT * pitch;
        const uint32_t lim = (uint32_t)(kdim - 1 - st * SKT);  // st < nst: >= 0
#pragma unroll
        for (int h = 0; h < RPT; h++) {
            const uint32_t row = min((uint32_t)(RPT * kq + h), lim);
            cw[h] = *reinterpret_cast<const uint32_t*>(sb + (row * pit + 4 * d));
        }
#pragma unroll
        for (int v = 0; v < RPT / 4; v++)  // lutr is zero-padded to mpad >= nst * SKT
            cl[v] = *reinterpret_cast<const uint4*>(lq + SKT * st + 4 * v);
    };
    auto store = [&](uint8_t* S, int h0, int h1) {
#pragma unroll
        for (int h = h0; h < h1; h++) {
            const uint4 c4 = cl[h >> 2];
            const uint32_t L = (h & 3) == 0 ? c4.x : (h & 3) == 1 ? c4.y : (h & 3) == 2 ? c4.z : c4.w;
            uint4 o;
            o.x = __builtin_amdgcn_perm(L, L, cw[h] & 0x03030303u);
            o.y = __builtin_amdgcn_perm(L, L, (cw[h] >> 2) & 0x03030303u);
            o.z = __builtin_amdgcn_perm(L, L, (cw[h] >> 4) & 0x03030303u);
            o.w = __builtin_amdgcn_perm(L, L, (cw[h] >> 6) & 0x03030303u);
            *reinterpret_cast<uint4*>(S + lp * PNL + (RPT * kq + h) * RS + 16 * d) = o;
        }
    };
    auto frag = [&](const uint8_t* S, int panel, int ks, int col) -> v4i {
        const uint8_t* b = S + panel * PNL + 32 * ks * RS + rd + col;
        const v2i x = lds_tr8(b), y = lds_tr8(b + 8 * RS);
        return (v4i){x.x, x.y, y.x, y.y};
    };
    auto frags = [&](const uint8_t* S, int ks, v4i (&A)[4], v4i (&B)[2]) {
#pragma unroll
        for (int x = 0; x < 4; x++) A[x] = frag(S, 0, ks, wm * 128 + 32 * x);
#pragma unroll
        for (int y = 0; y < 2; y++) B[y] = frag(S, 1, ks, wn * 64 + 32 * y);
    };

    load(0);
    store(lds, 0, RPT);
    load(nst > 1 ? 1 : 0);  // stage s+2's loads are issued at the end of stage s
    __syncthreads();
    for (uint64_t s = 0; s < nst; s++) {
        const uint8_t* cur = lds + (s & 1) * STG;
        uint8_t* nxt = lds + ((s + 1) & 1) * STG;
        v4i a[2][4], b[2][2];
        frags(cur, 0, a[0], b[0]);
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            if (ks + 1 < KS) frags(cur, ks + 1, a[(ks + 1) & 1], b[(ks + 1) & 1]);
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 2; y++)
                    acc[x][y] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[ks & 1][x], b[ks & 1][y], acc[x][y], 0, 0, 0);
            store(nxt, ks * RPT / KS, (ks + 1) * RPT / KS);
        }
        load(s + 2 < nst ? s + 2 : nst - 1);
        __syncthreads();
    }
    crt_epilogue(acc, r, nblk, bx, wm, wn, lane, res);
}

// Warp-specialised form of k_syrk_i8r (round 6): the same block, LDS image and MFMA tiling, with
// the loader moved out of the MFMA waves.  12 waves (3 per SIMD): waves 0-7 only read fragments
// (ds_read_b64_tr_b8) and issue MFMAs; waves 8-11 (one per SIMD) expand stage s+1's codes into
// the idle LDS buffer and issue stage s+2's code / LUT loads while the MFMA waves compute stage
// s.  One barrier per stage, as before.  Cycle budget per 128-SNP stage and CU (MI355X_MICROARCH
// §LDS): MFMA 2048 cycles per SIMD; fragment reads 8 waves x 4 k-steps x 12 ds_read_b64_tr_b8 x 2
// = 768 LDS cycles; residue image 64 ds_write_b128 x 13 = 832 transfer cycles -- the same 1600 LDS
// cycles, but the MFMA waves no longer issue the 13-cycle stores themselves, wait on code loads
// (vmcnt) or spend their issue slots on the expansion VALU, which put 14% of their cycles in
// SQ_WAIT_INST_LDS and 23% in SQ_WAIT_ANY (profiles/r05z/pmc_sq_crt.json).  The register budget of
// 3 waves per SIMD (<= 168 VGPRs) leaves the MFMA waves single-buffered fragments for the A panel.
// Two schedule settings on top (hook "crt" = 2 turns both off; same residues either way, int32
// sums being exact in any order), measured in one process at 50k x 62.5k (profiles/r06s):
// ROTA -- the A fragments of k-step ks+1 are read one 32-row tile at a time right after that
//   tile's two MFMAs of k-step ks (sched_group_barrier keeps the order; the compiler otherwise
//   issues all 12 reads after the 7th MFMA), -1% (r06o); the B reads of ks+1 spread over the
//   first two MFMAs and the A reads one per MFMA instead of B first then A in pairs: -1.3% / -0.7%
//   more on two boxes (profiles/r06se);
// MPRIO -- static issue priority for the MFMA waves over the loader waves, the younger MFMA half
//   (waves 4-7) one level above the older (MI355X_MICROARCH "two waves per SIMD" item 4): -2%
//   more; the loader waves at the higher priority instead +6%, pacing their stores with s_sleep
//   +7..35%, capping their LDS stores in flight -0.3% (r06o, r06q, r06r).
// Together 666.7 vs 687.7 ms per launch (-3.0%), -1.7% at 4100 iids, -2.6% on a cfg5 part.
// Lost against this kernel, all bit-identical (profiles/r06x): the residue image in 256-B lines
// stored by ds_write_addtid_b32 (2 transfer cycles per 256 B instead of 13 per KiB) -0.5%; a ring of
// three 64-SNP buffers whose next-stage fragments are read before the barrier +15%, and with LDS
// full/empty counters instead of barriers +29% (64-SNP stages double the per-stage costs).  Loader
// ablations: without the expansion VALU -7.8%, with one store in four -8%: the loader's VALU and
// its stores each take ~8% from the MFMA waves.  Also lost (profiles/r06y): the codes spread to one
// selector byte per iid by a per-launch pre-pass (no shift / mask VALU in the loader, 4x the code
// bytes) +32%; the loader's code loads issued two stages ahead (two register sets) +2.8%, issued
// one stage ahead but before the stores instead of after them +13%.
template <int SKT, bool ROTA = true, int MPRIO = 2>
__global__ __launch_bounds__(768, 1) void k_syrk_i8w(const uint8_t* __restrict__ P, uint64_t pitch, uint64_t kdim,
                                                     uint64_t mpad, const uint32_t* __restrict__ lutr,
                                                     const int* __restrict__ ctl, uint64_t b0, uint64_t nblk,
                                                     uint8_t* __restrict__ res, const double* __restrict__ lgp, CrtLog L,
                                                     const uint32_t* __restrict__ part_tab = nullptr) {
    constexpr int KS = SKT / 32, RPL = SKT / 8, PNL = SKT * RS, STG = 2 * PNL;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STG];
    if (ctl[1]) return;  // non-finite LUT: the f64 MFMA kernel runs instead
    const uint32_t w = blockIdx.x, q = w >> 3, u = q / kR;
    const uint32_t r = q - u * kR, bx = 8 * u + (w & 7);
    if (bx >= nblk) return;
    uint32_t bi, bj;
    if (part_tab) {
        const uint32_t c = part_tab[b0 + bx];
        bi = c & 0xffffu;
        bj = c >> 16;
    } else {
        tile_coords(b0 + bx, bi, bj);
    }
    if ((int)r >= block_moduli(lgp, bi, bj, L, ctl)) return;  // this block's K_int fits the first R_b moduli
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const uint64_t nst = (kdim + SKT - 1) / SKT;
    if (wave >= 8) {
        // loader: thread lt = (panel lp, row block kq of RPL rows, 16-iid group d)
        const int lt = t - 512;
        const int lp = __builtin_amdgcn_readfirstlane(lt >> 7), kq = (lt >> 4) & 7, d = lt & 15;
        const uint8_t* pbase = P + (uint64_t)(lp ? bj : bi) * (BW / 4);
        const uint32_t pit = (uint32_t)pitch;
        const uint32_t* lq = lutr + (uint64_t)r * mpad + RPL * kq;
        uint32_t cw[RPL];
        uint4 cl[RPL / 4];
        auto load = [&](uint64_t st) {
            const uint8_t* sb = pbase + st * SKT * pitch;
            const uint32_t lim = (uint32_t)(kdim - 1 - st * SKT);
#pragma unroll
            for (int h = 0; h < RPL; h++) {
                const uint32_t row = min((uint32_t)(RPL * kq + h), lim);
                cw[h] = *reinterpret_cast<const uint32_t*>(sb + (row * pit + 4 * d));
            }
#pragma unroll
            for (int v = 0; v < RPL / 4; v++) cl[v] = *reinterpret_cast<const uint4*>(lq + SKT * st + 4 * v);
        };
        auto store = [&](uint8_t* S) {
#pragma unroll
            for (int h = 0; h < RPL; h++) {
                const uint4 c4 = cl[h >> 2];
                const uint32_t L = (h & 3) == 0 ? c4.x : (h & 3) == 1 ? c4.y : (h & 3) == 2 ? c4.z : c4.w;
                uint4 o;
                o.x = __builtin_amdgcn_perm(L, L, cw[h] & 0x03030303u);
                o.y = __builtin_amdgcn_perm(L, L, (cw[h] >> 2) & 0x03030303u);
                o.z = __builtin_amdgcn_perm(L, L, (cw[h] >> 4) & 0x03030303u);
                o.w = __builtin_amdgcn_perm(L, L, (cw[h] >> 6) & 0x03030303u);
                *reinterpret_cast<uint4*>(S + lp * PNL + (RPL * kq + h) * RS + 16 * d) = o;
            }
        };
        load(0);
        store(lds);
        load(nst > 1 ? 1 : 0);
        __syncthreads();
        for (uint64_t s = 0; s < nst; s++) {
            store(lds + ((s + 1) & 1) * STG);  // stage s+1 (past the end: into the idle buffer, unread)
            load(s + 2 < nst ? s + 2 : nst - 1);
            __syncthreads();
        }
        return;
    }
    if constexpr (MPRIO > 1) {  // the younger MFMA half one level above the older (guide item 4)
        if (wave >= 4) __builtin_amdgcn_s_setprio(MPRIO);
        else __builtin_amdgcn_s_setprio(MPRIO - 1);
    } else if constexpr (MPRIO > 0) {
        __builtin_amdgcn_s_setprio(MPRIO);
    }
    const int wm = wave >> 2, wn = wave & 3;
    const int g = lane >> 4, jj = (lane & 15) >> 1, pp = lane & 1;
    const int rd = (16 * (g >> 1) + jj) * RS + 16 * (g & 1) + 8 * pp;
    v16i acc[4][2];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = (v16i){};
    auto frag = [&](const uint8_t* S, int panel, int ks, int col) -> v4i {
        const uint8_t* b = S + panel * PNL + 32 * ks * RS + rd + col;
        const v2i x = lds_tr8(b), y = lds_tr8(b + 8 * RS);
        return (v4i){x.x, x.y, y.x, y.y};
    };
    __syncthreads();
    for (uint64_t s = 0; s < nst; s++) {
        const uint8_t* cur = lds + (s & 1) * STG;
        v4i b[2][2];
#pragma unroll
        for (int y = 0; y < 2; y++) b[0][y] = frag(cur, 1, 0, wn * 64 + 32 * y);
        if constexpr (ROTA) {
            v4i a[4];
#pragma unroll
            for (int x = 0; x < 4; x++) a[x] = frag(cur, 0, 0, wm * 128 + 32 * x);
#pragma unroll
            for (int ks = 0; ks < KS; ks++) {
                if (ks + 1 < KS) {
#pragma unroll
                    for (int y = 0; y < 2; y++) b[(ks + 1) & 1][y] = frag(cur, 1, ks + 1, wn * 64 + 32 * y);
                }
#pragma unroll
                for (int x = 0; x < 4; x++) {
#pragma unroll
                    for (int y = 0; y < 2; y++)
                        acc[x][y] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[x], b[ks & 1][y], acc[x][y], 0, 0, 0);
                    if (ks + 1 < KS) a[x] = frag(cur, 0, ks + 1, wm * 128 + 32 * x);
                }
                // keep that order -- the compiler otherwise issues all 12 reads after the 7th MFMA:
                // the 12 reads of k-step ks+1 spread over this k-step's 8 MFMAs, each A tile's right
                // behind its two MFMAs (B, B | B, B, A0 | A0 | A1 | A1 | A2 | A2 | A3, A3)
                if (ks + 1 < KS) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
                    for (int i = 0; i < 5; i++) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                } else {
                    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                }
            }
            __syncthreads();
            continue;
        }
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            v4i a[4];
#pragma unroll
            for (int x = 0; x < 4; x++) a[x] = frag(cur, 0, ks, wm * 128 + 32 * x);
            if (ks + 1 < KS) {
#pragma unroll
                for (int y = 0; y < 2; y++) b[(ks + 1) & 1][y] = frag(cur, 1, ks + 1, wn * 64 + 32 * y);
            }
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 2; y++)
                    acc[x][y] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[x], b[ks & 1][y], acc[x][y], 0, 0, 0);
        }
        __syncthreads();
    }
    crt_epilogue(acc, r, nblk, bx, wm, wn, lane, res);
}

// ---------------------------------------------------------------- reconstruction
// two elements per thread (packed f32 math: v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32); the
// residues of the R planes -> K_int (Garner, exact: all digit arithmetic is on integers < 2^24
// held in f32) -> f64 -> K tiles.
typedef float f2 __attribute__((ext_vector_type(2)));

// y - p round(y / p): round by the 1.5 * 2^23 magic constant (|y / p| < 2^22), exact for the
// integers here; for odd p the result is the canonical residue in [-(p-1)/2, (p-1)/2] (no ties:
// y / p is at least 1/(2p) from a half-integer and the f32 quotient errs by < 2^-8 of that)
template <int I>
__device__ __forceinline__ f2 mod_sym(f2 y) {
    constexpr float p = (float)mod_of(I), ip = 1.0f / (float)mod_of(I), M = 12582912.0f;
    const f2 t = (y * ip + M) - M;
    return __builtin_elementwise_fma((f2)(-p), t, y);
}

template <int I>
struct Garner {
    // y = (sum_{j<I} v_j W_j) mod p_I by Horner over the digits, W_j = prod_{k<j} p_k
    template <int J>
    __device__ static __forceinline__ f2 horner(const f2 (&v)[kR], f2 y) {
        if constexpr (J < 0) {
            return y;
        } else {
            y = __builtin_elementwise_fma(y, (f2)((float)mod_of(J)), v[J]);  // |y| < 2^16, exact
            return horner<J - 1>(v, mod_sym<I>(y));
        }
    }
};

// inverse of W_i = prod_{j<i} p_j modulo p_i (host-computed, passed by value)
struct CrtConst {
    float inv[kR];
};

// digits I >= R are zero: K_int is the balanced mixed-radix number of the first R digits
template <int I>
__device__ __forceinline__ void digits(f2 (&v)[2][kR], const uint8_t* __restrict__ res, uint64_t plane,
                                       uint64_t e_off, const CrtConst& cc, int R) {
    if constexpr (I < kR) {
        if (I < R) {
            const uint32_t x = *reinterpret_cast<const uint32_t*>(res + (uint64_t)I * plane + e_off);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const f2 ri = {(float)((x >> (16 * h)) & 0xffu), (float)((x >> (16 * h + 8)) & 0xffu)};
                const f2 y = Garner<I>::template horner<I - 2>(v[h], v[h][I - 1]);
                v[h][I] = mod_sym<I>((ri - y) * cc.inv[I]);  // |.| < 2^17: exact
            }
        } else {
#pragma unroll
            for (int h = 0; h < 2; h++) v[h][I] = (f2){0.0f, 0.0f};
        }
        digits<I + 1>(v, res, plane, e_off, cc, R);
    }
}

// grid: 64 workgroups per 256-block (four rows each), 256 threads = 4 rows x 64 column quads;
// one 4-B load per residue plane and thread, two independent packed-f32 Garner chains
// part (cfg5): the block of slot b0 + blk is written whole (256 x 256 row-major, f64) at
// tiles + (b0 + blk) * 65536, as the f32 part kernels write theirs
__global__ __launch_bounds__(256) void k_crt(const uint8_t* __restrict__ res, uint64_t b0, uint64_t nblk, uint64_t n,
                                             const int* __restrict__ ctl, int F, CrtConst cc, double* __restrict__ tiles,
                                             int accumulate, const uint32_t* __restrict__ part_tab,
                                             const double* __restrict__ lgp, CrtLog L,
                                             unsigned long long* __restrict__ rec) {
    if (ctl[1]) return;
    const uint64_t blk = blockIdx.x >> 6;
    const int row = 4 * (blockIdx.x & 63) + (threadIdx.x >> 6), col = 4 * (threadIdx.x & 63);
    const bool part = part_tab != nullptr;
    uint32_t bi, bj;
    if (part) {
        const uint32_t c = part_tab[b0 + blk];
        bi = c & 0xffffu;
        bj = c >> 16;
    } else {
        tile_coords(b0 + blk, bi, bj);
    }
    const int R = block_moduli(lgp, bi, bj, L, ctl);  // the moduli k_syrk_i8* ran for this block
    if (rec && (blockIdx.x & 63) == 0 && threadIdx.x == 0) {
        atomicAdd(rec + 2, (unsigned long long)R);
        atomicAdd(rec + 3, 1ull);
    }
    uint64_t ti = 0, tj = 0;
    if (!part) {
        ti = 2 * (uint64_t)bi + (row >> 7);
        tj = 2 * (uint64_t)bj + (col >> 7);
        const uint64_t nt128 = (n + 127) / 128;
        if (ti > tj || tj >= nt128) return;
    }
    const uint64_t e_off = (blk * BW + row) * BW + col, plane = nblk * (BW * BW);
    f2 v[2][kR];
    {
        const uint32_t x = *reinterpret_cast<const uint32_t*>(res + e_off);
#pragma unroll
        for (int h = 0; h < 2; h++) {  // modulus 256: symmetric digit in [-128, 127]
            const int r0 = (x >> (16 * h)) & 0xff, r1 = (x >> (16 * h + 8)) & 0xff;
            v[h][0] = (f2){(float)(r0 >= 128 ? r0 - 256 : r0), (float)(r1 >= 128 ? r1 - 256 : r1)};
        }
    }
    digits<1>(v, res, plane, e_off, cc, R);
    const int sh = 2 * (ctl[0] - F);
    double2* T = reinterpret_cast<double2*>(
        part ? tiles + ((b0 + blk) * BW + row) * BW + col
             : tiles + (tj * (tj + 1) / 2 + ti) * (uint64_t)(128 * 128) + (row & 127) * 128 + (col & 127));
#pragma unroll
    for (int h = 0; h < 2; h++) {
        double X0 = (double)v[h][kR - 1].x, X1 = (double)v[h][kR - 1].y;
#pragma unroll
        for (int i = kR - 2; i >= 0; i--) {
            X0 = fma(X0, (double)mod_of(i), (double)v[h][i].x);
            X1 = fma(X1, (double)mod_of(i), (double)v[h][i].y);
        }
        double2 k = make_double2(ldexp(X0, sh), ldexp(X1, sh));
        if (accumulate) {
            const double2 o = T[h];
            k.x += o.x;
            k.y += o.y;
        }
        T[h] = k;
    }
}

}  // namespace

// --------------------------------------------------------------------------- host side
static double log2_modulus_product() {
    double s = 0;
    for (int i = 0; i < kR; i++) s += std::log2((double)mod_of(i));
    return s;
}

static CrtConst crt_constants() {
    CrtConst c{};
    c.inv[0] = 1.0f;
    for (int i = 1; i < kR; i++) {
        const long p = mod_of(i);
        long w = 1;
        for (int j = 0; j < i; j++) w = w * (mod_of(j) % p) % p;
        long inv = 1;
        while ((w * inv) % p != 1) inv++;
        c.inv[i] = (float)inv;
    }
    return c;
}

// largest F with 2 m 2^2F < P (|K_int| <= m 2^2F must sit inside (-P/2, P/2))
int crt_fraction_bits(uint64_t m) {
    const double f = (log2_modulus_product() - 1.0 - std::log2((double)std::max<uint64_t>(m, 1)) - 1e-9) / 2.0;
    return std::min(52, (int)std::floor(f));
}

// hook "crt": 1 = k_syrk_i8w (loader waves, default: 684 vs 697 ms per 50k x 62.5k launch in one
// process, profiles/r06g; 666.7 with its read order + wave priorities, r06s), 2 = k_syrk_i8w
// without those two, 0 = k_syrk_i8r (loader in every wave)
int g_crt_kernel = 1;
// hook "crt_block": 1 = moduli per 256-block from its panels' bounds (default), 0 = launch-wide R
int g_crt_block = 1;

uint64_t crt_max_snps() { return 1ull << 16; }  // keeps F >= 50 and the int32 sums exact
int crt_moduli() { return kR; }

// ctl (256 B) | residue LUT (kR x mpad u32) | bound table (4 x mpad f64) | per-iid bound sums (n f64) |
// per-panel log2 bounds (ceil(n / 256) f64)
uint64_t crt_lut_bytes(uint64_t m, uint64_t n) {
    const uint64_t mpad = round_up(std::max<uint64_t>(m, 1), SK);
    return 256 + (uint64_t)kR * mpad * 4 + mpad * 32 + round_up(std::max<uint64_t>(n, 1), 2) * 8 +
           round_up(ceil_div(std::max<uint64_t>(n, 1), BW), 2) * 8;
}

static CrtLog crt_logs() {
    CrtLog L{};
    double s = 0;
    for (int i = 0; i < kR; i++) L.plog[i] = (s += std::log2((double)mod_of(i)));
    return L;
}

// The residue chunks of launch_syrk_packed_crt's overlapped form as block columns [c0, c1): each
// chunk holds as many whole block columns as `res_bytes` of residues allow (at least one; block
// column c ends at block (c+1)(c+2)/2).  A function of n and res_bytes only, so every rank of an
// overlapped collective cuts the same chunks (api.hip sum_plan).
std::vector<std::pair<uint64_t, uint64_t>> crt_column_chunks(uint64_t n, uint64_t res_bytes) {
    const uint64_t nb = ceil_div(n, BW), total = nb * (nb + 1) / 2;
    const uint64_t per = std::max<uint64_t>(1, res_bytes / ((uint64_t)kR * BW * BW));
    std::vector<std::pair<uint64_t, uint64_t>> out;
    uint64_t col = 0;
    for (uint64_t b0 = 0; b0 < total;) {
        uint64_t col1 = col;
        while (col1 < nb && (col1 + 1) * (col1 + 2) / 2 <= b0 + std::min(per, total - b0)) col1++;
        if (col1 == col) col1 = col + 1;  // one column at least (<= nb <= per blocks in practice)
        out.push_back({col, col1});
        b0 = col1 * (col1 + 1) / 2;
        col = col1;
    }
    return out;
}

// K_tiles (+)= Z Z^T for packed codes + f64 LUT; ws_lut: crt_lut_bytes(m); res: res_bytes of
// scratch (>= kR * 65536); gate: device u32 set when the block must run on the f64 MFMA instead
void launch_syrk_packed_crt(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const double* lut,
                            double* tiles, int accumulate, void* ws_lut, uint8_t* res, uint64_t res_bytes,
                            unsigned long long* rec, hipStream_t st, const std::function<void()>* before_chunks,
                            const std::function<void(uint64_t, uint64_t)>* after_chunk, const uint32_t* part_tab,
                            uint64_t part_blocks) {
    SNPMI_REQUIRE(m > 0 && m <= crt_max_snps(), SNPMI_E_ARG, "crt SYRK: SNP count per launch out of range");
    SNPMI_REQUIRE(!part_tab || !after_chunk, SNPMI_E_ARG, "crt SYRK: column chunks of a part");
    const uint64_t nb = ceil_div(n, BW), total = part_tab ? part_blocks : nb * (nb + 1) / 2;
    if (total == 0) return;
    const uint64_t mpad = round_up(m, SK);
    int* ctl = (int*)ws_lut;
    uint32_t* lutr = (uint32_t*)((uint8_t*)ws_lut + 256);
    double* qsq = (double*)(lutr + (uint64_t)kR * mpad);
    double* S = qsq + 4 * mpad;
    double* lgp = S + round_up(std::max<uint64_t>(n, 1), 2);
    const int F = crt_fraction_bits(m);
    k_crt_exp<<<1, 1024, 0, st>>>(lut, 4 * m, ctl);
    k_crt_lut<<<(unsigned)ceil_div(mpad, 256), 256, 0, st>>>(lut, m, mpad, F, ctl, lutr, qsq);
    SNPMI_HIP(hipMemsetAsync(S, 0, n * sizeof(double), st));
    k_crt_bound<<<dim3((unsigned)ceil_div(ceil_div(n, 16), 256), (unsigned)ceil_div(m, kBoundSlice)), 256, 0, st>>>(
        packed, pitch, n, m, qsq, ctl, S);
    static const CrtLog logs0 = crt_logs();
    CrtLog logs = logs0;
    logs.per_block = g_crt_block;
    k_crt_r<<<1, 1024, 0, st>>>(S, n, logs, ctl, rec);
    k_crt_panels<<<(unsigned)nb, 256, 0, st>>>(S, n, ctl, lgp);
    const uint64_t per = std::max<uint64_t>(1, res_bytes / ((uint64_t)kR * BW * BW));
    static const CrtConst cc = crt_constants();
    if (before_chunks) (*before_chunks)();
    // after_chunk: chunks end at block-column boundaries (crt_column_chunks)
    const std::vector<std::pair<uint64_t, uint64_t>> cols =
        after_chunk ? crt_column_chunks(n, res_bytes) : std::vector<std::pair<uint64_t, uint64_t>>();
    size_t ci = 0;
    for (uint64_t b0 = 0, cnt = 0; b0 < total; b0 += cnt) {
        cnt = std::min(per, total - b0);
        if (after_chunk) {
            SNPMI_REQUIRE(ci < cols.size() && cols[ci].first * (cols[ci].first + 1) / 2 == b0, SNPMI_E_ARG,
                          "crt SYRK: column chunks out of step");
            cnt = cols[ci].second * (cols[ci].second + 1) / 2 - b0;
            SNPMI_REQUIRE(cnt <= per, SNPMI_E_ARG, "crt SYRK: one block column exceeds the residue scratch");
        }
        SNPMI_REQUIRE(cnt < (1ull << 23), SNPMI_E_ARG, "crt SYRK: chunk too large");
        // the kR moduli of a block on one XCD at once (FETCH 951 -> 149 GB per 62.5k-SNP
        // launch at 50k iids, the clock 2.21 -> 2.36 GHz, -3.6%: profiles/r05m)
        if (g_crt_kernel == 1)
            k_syrk_i8w<SK><<<(unsigned)(round_up(cnt, 8) * kR), 768, 0, st>>>(packed, pitch, m, mpad, lutr, ctl, b0,
                                                                            cnt, res, lgp, logs, part_tab);
        else if (g_crt_kernel == 2)
            k_syrk_i8w<SK, false, 0><<<(unsigned)(round_up(cnt, 8) * kR), 768, 0, st>>>(packed, pitch, m, mpad, lutr, ctl,
                                                                                      b0, cnt, res, lgp, logs, part_tab);
        else
            k_syrk_i8r<SK><<<(unsigned)(round_up(cnt, 8) * kR), 512, 0, st>>>(packed, pitch, m, mpad, lutr, ctl, b0,
                                                                            cnt, res, lgp, logs, part_tab);
        k_crt<<<(unsigned)(cnt * 64), 256, 0, st>>>(res, b0, cnt, n, ctl, F, cc, tiles, accumulate, part_tab, lgp, logs,
                                                    rec);
        if (after_chunk) {
            SNPMI_HIP(hipGetLastError());
            (*after_chunk)(cols[ci].first, cols[ci].second);
            ci++;
        }
    }
    SNPMI_HIP(hipGetLastError());
}

}  // namespace snpmi
