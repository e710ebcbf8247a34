// SnpKernel GRM on the MFMA cores: K_tiles += Z Z^T over one block of SNPs.
//
// Reference: SnpReader._read_kernel (snpreader.py:637-668) computes K = sum_b Z_b Z_b^T with
// NumPy (OpenBLAS ?syrk for the whole-matrix case, snpdata.py:203-206).  Here:
//   * K is held as the upper-triangle 128x128 tiles of the symmetric N x N matrix
//     (tile (ti,tj), ti <= tj, at index tj*(tj+1)/2 + ti, row-major inside) -- half the
//     HBM bytes, and the unit of the RCCL all-reduce.
//   * one workgroup (4 waves, 2x2) owns one tile; each wave owns 64x64 of it.
//   * f32: v_mfma_f32_32x32x2_f32 (exact f32 FMA chain), 2x2 MFMA tiles per wave, BK=32.
//     f64: v_mfma_f64_16x16x4_f64, 4x4 MFMA tiles per wave, BK=16.
//   * operand tiles are staged in LDS as [k][iid] (iid contiguous), double-buffered with a
//     register prefetch of stage s+1 under the MFMAs of stage s.
//   * PACKED loader: reads 2-bit codes straight from the packed BED block (32 bytes per SNP
//     per 128-iid tile) and expands them through the per-SNP 4-entry LUT written by
//     k_snp_stats -- decode + Unit/Beta standardization fused into the GEMM staging, so the
//     standardized Z never exists in HBM.  DENSE loader: an F-order float matrix (SnpData).
#include "snpmi_internal.hpp"

#include <algorithm>
#include <vector>

namespace snpmi {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int BM = kTile;  // 128

__device__ __forceinline__ void tile_coords(uint64_t L, uint32_t& ti, uint32_t& tj) {
    uint64_t j = (uint64_t)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while ((j + 1) * (j + 2) / 2 <= L) j++;
    while (j * (j + 1) / 2 > L) j--;
    tj = (uint32_t)j;
    ti = (uint32_t)(L - j * (j + 1) / 2);
}

// 4-entry LUT select, written so hipcc emits three v_cndmask (no divergent branches:
// the nested-ternary form compiled to exec-mask branches around every element).
template <typename T>
__device__ __forceinline__ T sel4(T l0, T l1, T l2, T l3, uint32_t c) {
    const bool b0 = (c & 1u) != 0, b1 = (c & 2u) != 0;
    const T lo = b0 ? l1 : l0;
    const T hi = b0 ? l3 : l2;
    return b1 ? hi : lo;
}

// v_bfi_b32: (m & a) | (~m & b).  hipcc does not form it from the C expression (it emits
// and/or/not/xor), so it is issued directly; a plain VOP3 VALU op needs no wait states.
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}

// 2-bit code at bit `sh` of w -> one of four 32-bit LUT words, 5 VALU per value:
// two v_bfe_i32 (bit -> 0 / ~0 mask) and three v_bfi_b32 selects (no v_cmp / VCC traffic).
__device__ __forceinline__ float sel4m(uint32_t l0, uint32_t l1, uint32_t l2, uint32_t l3, uint32_t w, uint32_t sh) {
    const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int)w, sh, 1u);
    const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int)w, sh + 1u, 1u);
    return __uint_as_float(bfi(m1, bfi(m0, l3, l2), bfi(m0, l1, l0)));
}

// ====================================================================== f32
namespace f32k {
constexpr int LDA = BM;  // floats per LDS row

// dense: F-order Z, ldz % 4 == 0; thread t moves float4 #(t + 256 q) of the BK x 128 tile
template <int BK>
__device__ __forceinline__ void load_dense(const float* __restrict__ Z, uint64_t ldz, uint64_t kdim, uint64_t k0,
                                           uint64_t i0, uint64_t j0, float4 (&ra)[BK / 8], float4 (&rb)[BK / 8]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < BK / 8; q++) {
        const int f = t + 256 * q;
        const int k = f >> 5, i4 = f & 31;
        const bool ok = k0 + k < kdim;
        const uint64_t kk = ok ? k0 + k : kdim - 1;  // clamped address, value zeroed below
        float4 va = *reinterpret_cast<const float4*>(Z + kk * ldz + i0 + 4 * i4);
        float4 vb = *reinterpret_cast<const float4*>(Z + kk * ldz + j0 + 4 * i4);
        if (!ok) {
            va = make_float4(0.f, 0.f, 0.f, 0.f);
            vb = va;
        }
        ra[q] = va;
        rb[q] = vb;
    }
}

template <int BK>
__device__ __forceinline__ void store_dense(float* As, float* Bs, const float4 (&ra)[BK / 8], const float4 (&rb)[BK / 8]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < BK / 8; q++) {
        const int f = t + 256 * q;
        const int k = f >> 5, i4 = f & 31;
        *reinterpret_cast<float4*>(As + k * LDA + 4 * i4) = ra[q];
        *reinterpret_cast<float4*>(Bs + k * LDA + 4 * i4) = rb[q];
    }
}

// packed: op = t>>7 (A: rows i0, B: rows j0); 128 threads x BK/16 dwords cover
// BK SNPs x 8 dwords (128 iids); each dword expands to 16 floats through the SNP's LUT.
struct PRegs {
    uint32_t w;
    float4 lut;
};

template <int BK>
__device__ __forceinline__ void load_packed(const uint8_t* __restrict__ P, uint64_t pitch, uint64_t kdim, uint64_t k0,
                                            uint64_t i0, uint64_t j0, const float* __restrict__ lut,
                                            PRegs (&r)[BK / 16]) {
    const int t = threadIdx.x;
    const int op = t >> 7, tt = t & 127;
    const uint64_t base = op ? j0 : i0;
#pragma unroll
    for (int q = 0; q < BK / 16; q++) {
        const int dw = tt + 128 * q;
        const int k = dw >> 3, d = dw & 7;
        const uint64_t kk = k0 + k;
        if (kk < kdim) {
            r[q].w = *reinterpret_cast<const uint32_t*>(P + kk * pitch + base / 4 + 4 * d);
            r[q].lut = *reinterpret_cast<const float4*>(lut + 4 * kk);
        } else {
            r[q].w = 0;
            r[q].lut = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
}

// The 4 float4 stores of a thread are rotated by (d>>1) so the 8 lanes of each
// ds_write_b128 group hit 8 distinct 16-B bank slots (conflict-free; was 4-way).
template <int BK>
__device__ __forceinline__ void store_packed(float* As, float* Bs, const PRegs (&r)[BK / 16]) {
    const int t = threadIdx.x;
    const int op = t >> 7, tt = t & 127;
    float* S = op ? Bs : As;
#pragma unroll
    for (int q = 0; q < BK / 16; q++) {
        const int dw = tt + 128 * q;
        const int k = dw >> 3, d = dw & 7;
        const uint32_t w = r[q].w;
        const float l0 = r[q].lut.x, l1 = r[q].lut.y, l2 = r[q].lut.z, l3 = r[q].lut.w;
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int vv = (v + (d >> 1)) & 3;
            const uint32_t b = w >> (8 * vv);
            float4 o;
            o.x = sel4(l0, l1, l2, l3, b & 3u);
            o.y = sel4(l0, l1, l2, l3, (b >> 2) & 3u);
            o.z = sel4(l0, l1, l2, l3, (b >> 4) & 3u);
            o.w = sel4(l0, l1, l2, l3, (b >> 6) & 3u);
            *reinterpret_cast<float4*>(S + k * LDA + 16 * d + 4 * vv) = o;
        }
    }
}

template <int BK>
__device__ __forceinline__ void compute(const float* As, const float* Bs, f32x16 (&acc)[2][2], int wm, int wn,
                                        int lane) {
    const int kr = lane >> 5, c = lane & 31;
#pragma unroll
    for (int kk = 0; kk < BK / 2; kk++) {
        const int row = (2 * kk + kr) * LDA;
        const float a0 = As[row + wm * 64 + c];
        const float a1 = As[row + wm * 64 + 32 + c];
        const float b0 = Bs[row + wn * 64 + c];
        const float b1 = Bs[row + wn * 64 + 32 + c];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
}

template <bool PACKED, int BK, int MINB>
__global__ __launch_bounds__(256, MINB) void k_syrk(const void* __restrict__ src, uint64_t ld, uint64_t kdim,
                                                    const float* __restrict__ lut, float* __restrict__ tiles,
                                                    int accumulate) {
    __shared__ __attribute__((aligned(16))) float lds[2][2][BK * LDA];
    uint32_t ti, tj;
    tile_coords(blockIdx.x, ti, tj);
    const uint64_t i0 = (uint64_t)ti * BM, j0 = (uint64_t)tj * BM;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    f32x16 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = (f32x16){};

    const uint64_t nst = (kdim + BK - 1) / BK;
    float4 ra[BK / 8], rb[BK / 8];
    PRegs rp[BK / 16 > 0 ? BK / 16 : 1];
    if constexpr (PACKED) {
        load_packed<BK>((const uint8_t*)src, ld, kdim, 0, i0, j0, lut, rp);
        store_packed<BK>(lds[0][0], lds[0][1], rp);
    } else {
        load_dense<BK>((const float*)src, ld, kdim, 0, i0, j0, ra, rb);
        store_dense<BK>(lds[0][0], lds[0][1], ra, rb);
    }
    __syncthreads();
    for (uint64_t s = 0; s < nst; s++) {
        const int buf = s & 1;
        const bool more = s + 1 < nst;
        if (more) {
            if constexpr (PACKED) load_packed<BK>((const uint8_t*)src, ld, kdim, (s + 1) * BK, i0, j0, lut, rp);
            else load_dense<BK>((const float*)src, ld, kdim, (s + 1) * BK, i0, j0, ra, rb);
        }
        compute<BK>(lds[buf][0], lds[buf][1], acc, wm, wn, lane);
        if (more) {
            if constexpr (PACKED) store_packed<BK>(lds[buf ^ 1][0], lds[buf ^ 1][1], rp);
            else store_dense<BK>(lds[buf ^ 1][0], lds[buf ^ 1][1], ra, rb);
        }
        __syncthreads();
    }
    // epilogue: C/D layout of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    float* T = tiles + (uint64_t)blockIdx.x * (BM * BM);
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++) {
            float* base = T + (wm * 64 + mt * 32 + 4 * (lane >> 5)) * BM + wn * 64 + nt * 32 + (lane & 31);
            if (accumulate) {  // wave-uniform branch; 16 loads in flight, then 16 stores
                float old[16];
#pragma unroll
                for (int r = 0; r < 16; r++) old[r] = base[((r & 3) + 8 * (r >> 2)) * BM];
#pragma unroll
                for (int r = 0; r < 16; r++) acc[mt][nt][r] += old[r];
            }
#pragma unroll
            for (int r = 0; r < 16; r++) base[((r & 3) + 8 * (r >> 2)) * BM] = acc[mt][nt][r];
        }
}

}  // namespace f32k

// ====================================================================== f32, 256x256 blocks
// 8 waves (2 x 4), each 128 x 64 = 4 x 2 MFMA 32x32 tiles.  Per MFMA this stages half the
// codes of the 128x128 kernel (the 2-bit -> f32 LUT expansion is VALU, and gfx950 runs the
// f32 MFMA at the f32 VALU rate, so expansion instructions directly displace MFMAs).
// Output goes to the same 128x128 upper-triangle tile store: wave (wm, wn) of block
// (bi, bj) owns 128-tile (2bi + wm, 2bj + wn/2); lower-quadrant / out-of-range waves skip.
namespace f32w {
constexpr int BW = 256, BK = 16, LDA = 256;

// write/accumulate a wave's 128x64 of the 256x256 block: into the 128x128 upper-triangle tile
// store (replicated K), or (LOCAL, cfg5) into the rank's dense 256x256 block at blockIdx.x.
template <bool LOCAL>
__device__ __forceinline__ void epilogue(f32x16 (&acc)[4][2], float* __restrict__ tiles, uint64_t n, uint32_t bi,
                                         uint32_t bj, int accumulate, int lane, int wm, int wn,
                                         uint64_t local_block) {
    float* T;
    uint64_t ldo;
    if constexpr (LOCAL) {
        T = tiles + local_block * (BW * BW) + (uint64_t)(wm * 128) * BW + (wn >> 1) * 128;
        ldo = BW;
    } else {
        const uint64_t nt128 = (n + 127) / 128;
        const uint64_t ti = 2 * (uint64_t)bi + wm, tj = 2 * (uint64_t)bj + (wn >> 1);
        if (ti > tj || tj >= nt128) return;  // wave-uniform
        T = tiles + (tj * (tj + 1) / 2 + ti) * (uint64_t)(BM * BM);
        ldo = BM;
    }
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) {
            float* bp = T + (32 * x + 4 * (lane >> 5)) * ldo + (wn & 1) * 64 + 32 * y + (lane & 31);
            if (accumulate) {
                float old[16];
#pragma unroll
                for (int r = 0; r < 16; r++) old[r] = bp[((r & 3) + 8 * (r >> 2)) * ldo];
#pragma unroll
                for (int r = 0; r < 16; r++) acc[x][y][r] += old[r];
            }
#pragma unroll
            for (int r = 0; r < 16; r++) bp[((r & 3) + 8 * (r >> 2)) * ldo] = acc[x][y][r];
        }
}

// LOCAL (cfg5, K too large to replicate): workgroup w computes block part_tab[w] of this part's
// layout (part_layout) and writes it as a full 256x256 row-major block at tiles + w * 65536 (no
// cross-rank reduction is needed).
// IL: the next stage's LUT expansion + ds_write is split into 4 pieces issued between the
// MFMA groups of the current stage (after kk = 1, 3, 5, 7) instead of after all of them.
// ROT: odd SNP rows of the LDS panels are stored rotated by 32 floats, so the two k-rows one
// ds_read_b32 of the MFMA A/B operands touches (lanes 0-31: row 2kk, lanes 32-63: row
// 2kk+1; rows are 1 KiB = a multiple of the 64-bank width) land on disjoint banks.
template <int MINB, bool LOCAL = false, bool IL = false, bool ROT = false>
__global__ __launch_bounds__(512, MINB) void k_syrk256(const uint8_t* __restrict__ P, uint64_t pitch, uint64_t n,
                                                      uint64_t kdim, const float* __restrict__ lut,
                                                      float* __restrict__ tiles, int accumulate,
                                                      const uint32_t* __restrict__ part_tab = nullptr) {
    __shared__ __attribute__((aligned(16))) float lds[2][2][BK * LDA];
    uint32_t bi, bj;
    if constexpr (LOCAL) {  // slot blockIdx.x of the part's layout table (part_layout)
        bi = part_tab[blockIdx.x] & 0xffffu;
        bj = part_tab[blockIdx.x] >> 16;
    } else {
        tile_coords(blockIdx.x, bi, bj);
    }
    const uint64_t i0 = (uint64_t)bi * BW, j0 = (uint64_t)bj * BW;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int t = threadIdx.x, op = t >> 8, tt = t & 255;
    const int kq = tt >> 4, d = tt & 15;
    const uint64_t base = op ? j0 : i0;
    const int kr = lane >> 5, c = lane & 31;
    f32x16 acc[4][2];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = (f32x16){};
    const uint64_t nst = (kdim + BK - 1) / BK;

    uint32_t w;
    float4 l;
    auto load = [&](uint64_t k0) {
        const uint64_t kk = k0 + kq;
        if (kk < kdim) {
            w = *reinterpret_cast<const uint32_t*>(P + kk * pitch + base / 4 + 4 * d);
            l = *reinterpret_cast<const float4*>(lut + 4 * kk);
        } else {
            w = 0;
            l = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store_part = [&](float* S, int v) {
        const uint32_t u0 = __float_as_uint(l.x), u1 = __float_as_uint(l.y), u2 = __float_as_uint(l.z),
                       u3 = __float_as_uint(l.w);
        const int vv = (v + (d >> 1)) & 3;
        const uint32_t sh = 8 * vv;
        float4 o;
        o.x = sel4m(u0, u1, u2, u3, w, sh);
        o.y = sel4m(u0, u1, u2, u3, w, sh + 2);
        o.z = sel4m(u0, u1, u2, u3, w, sh + 4);
        o.w = sel4m(u0, u1, u2, u3, w, sh + 6);
        const int col = ROT ? ((16 * d + 4 * vv + 32 * (kq & 1)) & (LDA - 1)) : 16 * d + 4 * vv;
        *reinterpret_cast<float4*>(S + kq * LDA + col) = o;
    };
    auto store = [&](float* S) {
        const uint32_t u0 = __float_as_uint(l.x), u1 = __float_as_uint(l.y), u2 = __float_as_uint(l.z),
                       u3 = __float_as_uint(l.w);
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int vv = (v + (d >> 1)) & 3;  // conflict-free ds_write_b128 slots
            const uint32_t sh = 8 * vv;
            float4 o;
            o.x = sel4m(u0, u1, u2, u3, w, sh);
            o.y = sel4m(u0, u1, u2, u3, w, sh + 2);
            o.z = sel4m(u0, u1, u2, u3, w, sh + 4);
            o.w = sel4m(u0, u1, u2, u3, w, sh + 6);
            const int col = ROT ? ((16 * d + 4 * vv + 32 * (kq & 1)) & (LDA - 1)) : 16 * d + 4 * vv;
            *reinterpret_cast<float4*>(S + kq * LDA + col) = o;
        }
    };

    load(0);
    store(op ? lds[0][1] : lds[0][0]);
    __syncthreads();
    for (uint64_t s = 0; s < nst; s++) {
        const int buf = s & 1;
        const bool more = s + 1 < nst;
        if (more) load((s + 1) * BK);
        const float* As = lds[buf][0];
        const float* Bs = lds[buf][1];
#pragma unroll
        for (int kk = 0; kk < BK / 2; kk++) {
            const int row = (2 * kk + kr) * LDA;
            float a[4], b[2];
            const int rot = ROT ? 32 * kr : 0;
#pragma unroll
            for (int x = 0; x < 4; x++) a[x] = As[row + ((wm * 128 + 32 * x + rot) & (LDA - 1)) + c];
#pragma unroll
            for (int y = 0; y < 2; y++) b[y] = Bs[row + ((wn * 64 + 32 * y + rot) & (LDA - 1)) + c];
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 2; y++)
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[x], b[y], acc[x][y], 0, 0, 0);
            if constexpr (IL) {
                if (more && (kk & 1)) store_part(op ? lds[buf ^ 1][1] : lds[buf ^ 1][0], kk >> 1);
            }
        }
        if constexpr (!IL) {
            if (more) store(op ? lds[buf ^ 1][1] : lds[buf ^ 1][0]);
        }
        __syncthreads();
    }
    epilogue<LOCAL>(acc, tiles, n, bi, bj, accumulate, lane, wm, wn, blockIdx.x);
}

// dense operand: Z (f32, F order, column k at Z + k*ldz, ldz >= round_up(n, 256), ldz % 4 == 0)
// streamed global -> LDS by global_load_lds_dwordx4 (no VGPR round trip, no VALU): one
// wave-instruction moves one 1 KiB SNP row of a 256-iid panel; odd rows are rotated by 32
// floats through the SOURCE address (the LDS image of a glds is lane-linear) so the two rows a
// ds_read_b32 of the MFMA operands touches hit disjoint banks.  SNP rows >= kdim are zero-filled
// by ds_write (wave-uniform branch).
// XCD remap: the hardware deals consecutive workgroups round-robin over the 8 XCDs (each with
// its own L2); remapping so that XCD x runs a contiguous range of the block list keeps blocks
// that share a panel (same column bj, neighbouring bi) on one L2 (bijective for any count).
__device__ __forceinline__ uint64_t xcd_remap(uint64_t orig, uint64_t nwg) {
    const uint64_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <bool LOCAL = false, int BKD = 16, int NBUF = 2, bool XCD = false>
__global__ __launch_bounds__(512, 1) void k_syrk256d(const float* __restrict__ Z, uint64_t ldz, uint64_t n,
                                                    uint64_t kdim, float* __restrict__ tiles, int accumulate,
                                                    uint32_t part_rank = 0, uint32_t part_world = 1,
                                                    const uint32_t* __restrict__ gate = nullptr,
                                                    const uint32_t* __restrict__ part_tab = nullptr) {
    static_assert(NBUF == 2 || NBUF == 3, "2 or 3 LDS stages");
    constexpr int G = 2 * BKD / 8;  // glds per wave per stage (8 waves, one 1 KiB row each)
    __shared__ __attribute__((aligned(16))) float lds[NBUF][2][BKD * LDA];
    if (gate && *gate == 0) return;  // fallback of the dense fp16x2 kernel (range flag raised)
    const uint64_t wg = XCD ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    uint32_t bi, bj;
    if constexpr (LOCAL) {  // slot wg of the part's layout table (part_layout)
        bi = part_tab[wg] & 0xffffu;
        bj = part_tab[wg] >> 16;
    } else {
        tile_coords(wg, bi, bj);
    }
    (void)part_rank;
    (void)part_world;
    const uint64_t i0 = (uint64_t)bi * BW, j0 = (uint64_t)bj * BW;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int kr = lane >> 5, c = lane & 31;
    f32x16 acc[4][2];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = (f32x16){};
    const uint64_t nst = (kdim + BKD - 1) / BKD;
    auto issue = [&](uint64_t k0, int buf) {
#pragma unroll
        for (int q = 0; q < G; q++) {
            const int r = wave * G + q;  // 2*BKD rows per stage: 2 panels x BKD SNPs
            const int panel = r / BKD, k = r % BKD;
            float* dst = &lds[buf][panel][k * LDA];
            const uint64_t kk = k0 + k;
            if (kk < kdim) {
                const float* src = Z + kk * ldz + (panel ? j0 : i0) + ((4 * lane + 32 * (k & 1)) & (BW - 1));
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                                 (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
            } else {
                reinterpret_cast<float4*>(dst)[lane] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    };
    auto compute = [&](int buf) {
        const float* As = lds[buf][0];
        const float* Bs = lds[buf][1];
#pragma unroll
        for (int kk = 0; kk < BKD / 2; kk++) {
            const int row = (2 * kk + kr) * LDA;
            const int rot = 32 * kr;
            float a[4], b[2];
#pragma unroll
            for (int x = 0; x < 4; x++) a[x] = As[row + ((wm * 128 + 32 * x - rot) & (LDA - 1)) + c];
#pragma unroll
            for (int y = 0; y < 2; y++) b[y] = Bs[row + ((wn * 64 + 32 * y - rot) & (LDA - 1)) + c];
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 2; y++)
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[x], b[y], acc[x][y], 0, 0, 0);
        }
    };
    if constexpr (NBUF == 2) {
        issue(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (uint64_t s = 0; s < nst; s++) {
            const int buf = s & 1;
            if (s + 1 < nst) issue((s + 1) * BKD, buf ^ 1);
            compute(buf);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    } else {
        // 3 stages, one raw barrier per stage; a counted vmcnt leaves stage s+1 in flight
        issue(0, 0);
        if (nst > 1) issue(BKD, 1);
        for (uint64_t s = 0; s < nst; s++) {
            if (s + 1 < nst) {
                if constexpr (G == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (s + 2 < nst) issue((s + 2) * BKD, (int)((s + 2) % 3));
            compute((int)(s % 3));
        }
    }
    epilogue<LOCAL>(acc, tiles, n, bi, bj, accumulate, lane, wm, wn, wg);
}

// ---------------------------------------------------------------- f32 GRM on the bf16 MFMA pipe
// The f32 MFMA (32x32x2) runs at 1/16 of the bf16 MFMA rate on gfx950.  Every f32 value of Z
// is the sum of three bf16 values, EXACTLY: a0 = bf16(a), a1 = bf16(a - a0), a2 = a - a0 - a1
// (a has 24 significant bits; each bf16 carries 8, and the residuals are exact in f32).  Then
//   a*b = sum_{p,q} a_p b_q;   the six terms with p + q <= 2 are kept, the dropped ones are
//   below 2^-23 |a b| -- the rounding level of one f32 multiply -- and every bf16 x bf16
// product is exact in the f32 accumulator.  So K = sum over 6 bf16 MFMA products (f32 accumulate)
// carries f32 accuracy at 16/6 = 2.7x the f32-MFMA peak.  The split is per SNP, on its 4-entry
// LUT (k_lut_bf3), so the loader expands 2-bit codes straight into three bf16 planes with one
// v_perm_b32 per 2 values per plane -- the standardized Z never exists in HBM.
//
// LDS image (per stage): [panel A/B][plane 3][k 16][iid 256, row stride 288 bf16 = 576 B].
// MFMA operands (v_mfma_f32_32x32x16_bf16: lane l holds A[iid l&31][k 8(l>>5)..+7]) come out of
// the SNP-major image with ds_read_b64_tr_b16 (4 k-rows x 16 iids per 16-lane group, delivered
// column-major).  576 B = 16 dwords (mod 64) per k-row puts the 4 rows x 2 groups of a 32-lane
// half on 64 distinct banks; the loader's two 16-B ds_write_b128 per row piece are ordered by
// (d >> 2) & 1 so each 8-lane store group covers all 32 write banks.
//
// Cheap expansion: the LUT of plane p is byte-planar (word 2p = low bytes of L0..L3, word 2p+1 =
// high bytes), so the v_perm selector of a value with code c is just (c, c + 4).  With
// v_j = (w >> 2j) & 0x03030303 (byte q = code of iid 4q + j), one v_perm of (v_j | 0x04040404,
// v_j) gives the selector of the iid pair (j, 4 + j) and another that of (8 + j, 12 + j).  The
// LDS rows therefore hold each 16-iid group in the order pi(p) = 4 (p & 3) + (p >> 2) (a 4x4
// transpose, an involution), on both panels alike; K's rows and columns come out permuted the
// same way and the epilogue writes element (p, p') to (pi(p), pi(p')).
constexpr int B3_RS = 288;                     // bf16 per LDS k-row
constexpr int B3_PLANE = BK * B3_RS;           // bf16 per plane of one panel (BK = 16 SNPs)
constexpr int B3_STAGE = 2 * 3 * B3_PLANE;     // bf16 per stage (2 panels x 3 planes)

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef short i16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ i16x4_t lds_tr16(const short* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4_t*)p);
}

__device__ __forceinline__ int pi16(int p) { return 4 * (p & 3) + (p >> 2); }

// f32w::epilogue with the pi-permuted rows/columns of k_syrk_bf3
template <bool LOCAL>
__device__ __forceinline__ void epilogue_pi(f32x16 (&acc)[4][2], float* __restrict__ tiles, uint64_t n, uint32_t bi,
                                            uint32_t bj, int accumulate, int lane, int wm, int wn,
                                            uint64_t local_block) {
    float* T;
    uint64_t ldo;
    if constexpr (LOCAL) {
        T = tiles + local_block * (BW * BW) + (uint64_t)(wm * 128) * BW + (wn >> 1) * 128;
        ldo = BW;
    } else {
        const uint64_t nt128 = (n + 127) / 128;
        const uint64_t ti = 2 * (uint64_t)bi + wm, tj = 2 * (uint64_t)bj + (wn >> 1);
        if (ti > tj || tj >= nt128) return;  // wave-uniform
        T = tiles + (tj * (tj + 1) / 2 + ti) * (uint64_t)(BM * BM);
        ldo = BM;
    }
    const int hh = lane >> 5, colp = 16 * ((lane >> 4) & 1) + pi16(lane & 15);
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) {
            float* bp = T + (32 * x + hh) * ldo + (wn & 1) * 64 + 32 * y + colp;
            // accumulator register r sits at row (r&3) + 8(r>>2) + 4hh of the subtile, i.e. at
            // pi-row 16(r>>3) + 4(r&3) + 2((r>>2)&1) + hh
            if (accumulate) {
                float old[16];
#pragma unroll
                for (int r = 0; r < 16; r++) old[r] = bp[(16 * (r >> 3) + 4 * (r & 3) + 2 * ((r >> 2) & 1)) * ldo];
#pragma unroll
                for (int r = 0; r < 16; r++) acc[x][y][r] += old[r];
            }
#pragma unroll
            for (int r = 0; r < 16; r++) bp[(16 * (r >> 3) + 4 * (r & 3) + 2 * ((r >> 2) & 1)) * ldo] = acc[x][y][r];
        }
}

// Segmented accumulation (f32 GRM accuracy): the f32 MFMA accumulators absorb a long chain of
// small additions into a large running sum (a rare variant's z^2 ~ n puts K_ii at ~1e5 early, then
// every later 16-product step rounds at ulp(1e5)/2, and the tiny z^2 = 2 maf of rare SNPs at the
// major genotype are lost), so a launch over 62.5k SNPs lands ~3e-5 of max diag from the f64 GRM
// where NumPy's float32 K (OpenBLAS K-panels of a few hundred SNPs, then K += per block) is ~3e-7
// (tools/diag_f32_accuracy.py, profiles/r03acc).  Every `seg.snps` SNPs a workgroup adds its
// accumulators into a private scratch slot and restarts them at zero, so no f32 chain is longer
// than that; the final epilogue adds the slot back.  The slot is in register-native layout
// ([wave][32 f32x4][64 lanes], one 16-B buffer load + store per 4 accumulators, lane offset in one
// VGPR, the rest constant soffsets -- with flat addresses the compiler hoists 32 loop-invariant
// 64-bit addresses out of the k-loop and spills ~210 VGPRs), from a pool taken by atomic CAS
// (SegCtx).  Flush points are staggered by workgroup (phase = wg mod trips).
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct SegFlush {
    // Every `trips` trips the accumulators are flushed into the workgroup's slot and restart: the
    // first flush stores them, later ones add to the slot with fire-and-forget f32 buffer atomics
    // (the slot is private to the wave, so the adds never contend and their order is fixed), so a
    // flush waits on nothing.  A read-modify-write flush (32 loads + 32 stores per lane at one
    // barrier) cost +4.1% at 8192 SNPs.
    uint32_t trips = 0, trip = 0;
    bool any = false;  // a segment was flushed into the slot
    uint32_t slot = 0;
    __amdgpu_buffer_rsrc_t rs;
    int voff = 0;

    // call once per kernel by every thread (contains a barrier when segmentation is on)
    __device__ SegFlush(const SegCtx& c, uint32_t snps_per_trip, uint64_t wg, uint64_t total_trips, uint32_t* sh) {
        if (c.snps == 0) return;
        trips = max(1u, c.snps / snps_per_trip);
        trip = (uint32_t)(wg % trips);
        if (trips - trip >= total_trips) {  // no flush in this workgroup: no slot needed
            trips = 0;
            return;
        }
        if (threadIdx.x == 0) {
            uint32_t i = (uint32_t)((wg * 97u) % c.nslots);
            while (atomicCAS(c.flags + i, 0u, 1u) != 0u) i = i + 1 == c.nslots ? 0 : i + 1;
            *sh = i;
        }
        __syncthreads();
        slot = *sh;
        const int wave = threadIdx.x >> 6;
        float* base = c.scratch + (uint64_t)slot * kSegSlotFloats + (uint64_t)wave * (32 * 64 * 4);
        rs = __builtin_amdgcn_make_buffer_rsrc(sgpr_ptr(base), 0, 32 * 64 * 16, 0x00020000);
        voff = (threadIdx.x & 63) * 4;
    }
    // call once per trip; true when the accumulators should be flushed now
    __device__ bool due(bool more) {
        if (!trips || ++trip < trips) return false;
        trip = 0;
        return more;
    }
    // slot layout per wave: sub-tile k = x*2+y, element e at float index (k*16 + e)*64 + lane
    __device__ void flush(f32x16 (&a)[4][2]) {
        if (any) {
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 2; y++)
#pragma unroll
                    for (int e = 0; e < 16; e++)
                        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(a[x][y][e], rs, voff, ((x * 2 + y) * 16 + e) * 256, 0);
        } else {
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 2; y++)
#pragma unroll
                    for (int e = 0; e < 16; e++) {
                        const float v = a[x][y][e];  // (bit_cast of the element lvalue itself reads element 0)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rs, voff, ((x * 2 + y) * 16 + e) * 256, 0);
                    }
        }
#pragma unroll
        for (int x = 0; x < 4; x++)
#pragma unroll
            for (int y = 0; y < 2; y++) a[x][y] = (f32x16){};
        any = true;
    }
    // before the final epilogue: add the flushed segments back into the accumulators
    __device__ void finish(f32x16 (&a)[4][2]) {
        if (!any) return;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's adds have landed in L2
#pragma unroll
        for (int x = 0; x < 4; x++)
#pragma unroll
            for (int y = 0; y < 2; y++)
#pragma unroll
                for (int e = 0; e < 16; e++)  // glc: past the CU's vector cache
                    a[x][y][e] += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, ((x * 2 + y) * 16 + e) * 256, 1));
    }
    // after the final epilogue, by every thread: give the slot back
    __device__ void release(const SegCtx& c) {
        if (!trips) return;
        __syncthreads();  // every wave has read its part of the slot back
        if (threadIdx.x == 0) {
            __threadfence();
            atomicExch(c.flags + slot, 0u);
        }
    }
};

// f32 GRM on the bf16 MFMA pipe (the fallback of k_syrk_h2 for LUTs outside fp16's range, and of
// the dense-operand path): three exact bf16 planes per value, six products p+q <= 2.  Loader: the
// codes / LUT of stage s+1 (16 SNPs) are expanded and stored plane by plane between the MFMA groups
// of stage s, with the workgroup barrier in the middle of the stage (see the loop).
struct B3Regs {
    uint32_t w;
    uint4 la, lb;  // plane LUT words: (lo0, hi0, lo1, hi1), (lo2, hi2, -, -)
};

template <bool LOCAL = false, bool XCD = false, int MODE = 5>
__global__ __launch_bounds__(512, 1) void k_syrk_bf3(const uint8_t* __restrict__ P, uint64_t pitch, uint64_t n,
                                                     uint64_t kdim, const uint32_t* __restrict__ lut3,
                                                     float* __restrict__ tiles, int accumulate,
                                                     uint32_t part_rank = 0, uint32_t part_world = 1,
                                                     uint64_t kslice = 0, uint64_t slice_elems = 0,
                                                     const uint32_t* __restrict__ gate = nullptr, SegCtx seg = SegCtx(),
                                                     uint64_t wg0 = 0, const uint32_t* __restrict__ part_tab = nullptr) {
    static_assert(MODE == 5, "k_syrk_bf3: the interleaved loader with the mid-stage barrier (MODE 5)");
    __shared__ __attribute__((aligned(16))) short lds[2 * B3_STAGE];
    if (gate && *gate == 0) return;  // fallback of k_syrk_h2: runs only when its range flag is set
    if (gridDim.y > 1) {  // split-K: slice blockIdx.y covers SNPs [y*kslice, +kslice) into its own partial K
        const uint64_t k0 = (uint64_t)blockIdx.y * kslice;
        P += k0 * pitch;
        lut3 += 8 * k0;
        kdim = min(kslice, kdim - k0);
        tiles += (uint64_t)blockIdx.y * slice_elems;
    }
    // wg0: first block of a column-group launch (triangular order), as in k_syrk_h2
    const uint64_t wg = wg0 + (XCD ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x);
    uint32_t bi, bj;
    if constexpr (LOCAL) {  // slot wg of the part's layout table (part_layout)
        bi = part_tab[wg] & 0xffffu;
        bj = part_tab[wg] >> 16;
    } else {
        tile_coords(wg, bi, bj);
    }
    const uint64_t i0 = (uint64_t)bi * BW, j0 = (uint64_t)bj * BW;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    // loader role: panel, SNP row k of the stage, 16-iid group d
    const int lp = t >> 8, lk = (t >> 4) & 15, ld_ = t & 15;
    // the two 16-B halves of a 32-B segment are stored swapped in segments with bit 2 set
    // (sw = (d >> 2) & 1): the 8 lanes of a ds_write_b128 group then hit 8 distinct 16-B bank
    // slots.  (Ordering the two stores instead does not work: the compiler reorders them --
    // PMC showed 8 conflict cycles per ds_write_b128.)  The transposed reads undo the swap.
    const int sw = (ld_ >> 2) & 1;
    // packed codes of (SNP k0 + lk, iids base + 16 ld_ ..): walked by pointer, clamped to the last
    // SNP past kdim (its values are zeroed through the LUT: lut3 is zero-padded to a multiple of BK)
    const uint8_t* wp = P + (lp ? j0 : i0) / 4 + 4 * ld_ + (uint64_t)lk * pitch;
    const uint8_t* wlast = P + (lp ? j0 : i0) / 4 + 4 * ld_ + (kdim - 1) * pitch;
    const uint32_t* lp3 = lut3 + 8 * lk;
    // transposed-read role: lane 4q+p of group g supplies row 8(g>>1)+q, cols 16(g&1)+4p
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int rd_off = (8 * (g >> 1) + q) * B3_RS + 16 * (g & 1) + 4 * pp;
    // segment of a fragment column c (multiple of 32) + 16(g&1): swapped iff bit 2 of c/16 + (g&1)
    // is set, i.e. for A (c = wm*128 + 32x) iff x >= 2, for B (c = wn*64 + 32y) iff wn is odd;
    // the lane's 8-byte piece then moves by +-8 bf16 (first / second half)
    const int dswz = (pp >> 1) ? -8 : 8;
    const int rd_offB = rd_off + ((wn & 1) ? dswz : 0);

    f32x16 acc[4][2];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = (f32x16){};
    const uint64_t nst = (kdim + BK - 1) / BK;

    auto load = [&](uint64_t st, B3Regs& r) {
        const uint8_t* a = wp + st * BK * pitch;
        r.w = *reinterpret_cast<const uint32_t*>(a <= wlast ? a : wlast);
        r.la = *reinterpret_cast<const uint4*>(lp3 + 8 * BK * st);
        r.lb = *reinterpret_cast<const uint4*>(lp3 + 8 * BK * st + 4);
    };
    auto make_sel = [&](uint32_t w, uint32_t (&sel)[8]) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t v = (w >> (2 * j)) & 0x03030303u;  // byte q: code of iid 4q + j
            const uint32_t o = v | 0x04040404u;
            sel[2 * j] = __builtin_amdgcn_perm(o, v, 0x05010400u);      // iids (j, 4 + j)
            sel[2 * j + 1] = __builtin_amdgcn_perm(o, v, 0x07030602u);  // iids (8 + j, 12 + j)
        }
    };
    auto store_plane = [&](short* S, int pl, const B3Regs& r, const uint32_t (&sel)[8]) {
        const uint32_t lo = pl == 0 ? r.la.x : pl == 1 ? r.la.z : r.lb.x;
        const uint32_t hi = pl == 0 ? r.la.y : pl == 1 ? r.la.w : r.lb.y;
        uint4 v0, v1;
        v0.x = __builtin_amdgcn_perm(hi, lo, sel[0]);
        v0.y = __builtin_amdgcn_perm(hi, lo, sel[1]);
        v0.z = __builtin_amdgcn_perm(hi, lo, sel[2]);
        v0.w = __builtin_amdgcn_perm(hi, lo, sel[3]);
        v1.x = __builtin_amdgcn_perm(hi, lo, sel[4]);
        v1.y = __builtin_amdgcn_perm(hi, lo, sel[5]);
        v1.z = __builtin_amdgcn_perm(hi, lo, sel[6]);
        v1.w = __builtin_amdgcn_perm(hi, lo, sel[7]);
        uint4* r4 = reinterpret_cast<uint4*>(S + (lp * 3 + pl) * B3_PLANE + lk * B3_RS + 16 * ld_);
        r4[sw] = v0;
        r4[sw ^ 1] = v1;
    };
    auto store = [&](short* S, const B3Regs& r) {
        uint32_t sel[8];
        make_sel(r.w, sel);
#pragma unroll
        for (int pl = 0; pl < 3; pl++) store_plane(S, pl, r, sel);
    };
    auto frag = [&](const short* S, int panel, int pl, int col, int off) -> bf16x8_t {
        const short* b = S + (panel * 3 + pl) * B3_PLANE + off + col;
        const i16x4_t r0 = lds_tr16(b), r1 = lds_tr16(b + 4 * B3_RS);
        return __builtin_bit_cast(bf16x8_t, (i16x8_t)__builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    {
        // The loader with the workgroup barrier in the middle of the stage: after
        // MFMA group 3 (stage s+1's planes are all stored) every wave reads stage s+1's B planes
        // 0-1 into a second register set during groups 4-5, so the next stage starts after its
        // 8 A-plane-0 reads instead of 20 transposed LDS reads.  Stage s's own A planes and B
        // plane 2 are read before its barrier -- after it, its buffer may be overwritten
        // (stage s+2's stores during stage s+1's groups 1-3).  256 VGPRs per wave at 2 waves
        // per SIMD: 128 hold the accumulators, so only part of the next stage is prefetched.
        auto fragB = [&](const short* S, int pl, bf16x8_t (&b)[2]) {
#pragma unroll
            for (int y = 0; y < 2; y++) b[y] = frag(S, 1, pl, wn * 64 + 32 * y, rd_offB);
        };
        auto fragsA = [&](const short* S, int pa, bf16x8_t (&a)[4]) {
#pragma unroll
            for (int x = 0; x < 4; x++) a[x] = frag(S, 0, pa, wm * 128 + 32 * x, x >= 2 ? rd_off + dswz : rd_off);
        };
        auto group = [&](const bf16x8_t (&a)[4], const bf16x8_t (&b)[2]) {
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 2; y++)
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[x], b[y], acc[x][y], 0, 0, 0);
        };
        B3Regs r;
        load(0, r);
        store(lds, r);
        if (nst > 1) load(1, r);
        __syncthreads();
        bf16x8_t B0s[2], B1s[2], B0t[2], B1t[2];
        __shared__ uint32_t seg_slot;
        SegFlush sf(seg, 2 * BK, wg, (nst + 1) / 2, &seg_slot);
        fragB(lds, 0, B0s);
        fragB(lds, 1, B1s);
        // The loader runs unconditionally (the last stage expands into the idle buffer, its code
        // loads clamp to the last stage), so each MFMA group and its loader VALU share one basic
        // block, and the schedule is pinned to one VALU after each MFMA (sched_group_barrier)
        // instead of the group's 8 MFMAs followed by a VALU burst.  N=50k: 307.2-315.0 vs
        // 303.3-307.1 TFLOP/s with the barrier-guarded form; 2 or 3 VALU per MFMA 305-307,
        // unconditional hooks without the pin 306.1, + the next B reads pinned between the
        // group 4-5 MFMAs 293.4 (profiles/r01i/ubench_syrk_bf3_interleave.jsonl).
        constexpr bool kUncond = true;
        auto pin = [&]() {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // VALU
            }
        };
        auto stage = [&](uint64_t s, bf16x8_t (&B0)[2], bf16x8_t (&B1)[2], bf16x8_t (&B0n)[2], bf16x8_t (&B1n)[2]) {
            const short* cur = lds + (s & 1) * B3_STAGE;
            short* nxt = lds + ((s + 1) & 1) * B3_STAGE;
            const bool more = kUncond || s + 1 < nst;
            bf16x8_t A0[4], B2[2], A1[4], A2[4];
            fragsA(cur, 0, A0);
            fragB(cur, 2, B2);
            fragsA(cur, 1, A1);
            uint32_t sel[8];
            group(A0, B0);
            if (more) make_sel(r.w, sel);
            pin();
            group(A0, B1);
            if (more) store_plane(nxt, 0, r, sel);
            pin();
            group(A0, B2);
            fragsA(cur, 2, A2);
            if (more) store_plane(nxt, 1, r, sel);
            pin();
            group(A1, B0);
            if (more) store_plane(nxt, 2, r, sel);
            pin();
            if constexpr (kUncond) load(s + 2 < nst ? s + 2 : nst - 1, r);
            else if (more && s + 2 < nst) load(s + 2, r);
            __syncthreads();
            if (more) {
                fragB(nxt, 0, B0n);
                fragB(nxt, 1, B1n);
            }
            group(A1, B1);
            group(A2, B0);
        };
        // two stages per trip so the two fragment sets keep fixed registers (no copies)
        for (uint64_t s = 0; s < nst; s += 2) {
            stage(s, B0s, B1s, B0t, B1t);
            if (s + 1 < nst) stage(s + 1, B0t, B1t, B0s, B1s);
            if (sf.due(s + 2 < nst)) sf.flush(acc);
        }
        sf.finish(acc);
        epilogue_pi<LOCAL>(acc, tiles, n, bi, bj, accumulate, lane, wm, wn, wg);
        sf.release(seg);
    }
}

// per-SNP f32 LUT [m][4] -> bf16x3 split LUT [mpad][8] u32, byte-planar: plane p at word 2p
// (low bytes of the bf16 of codes 0..3) and 2p+1 (high bytes).  RNE rounding; NaN (Identity
// LUT) stays NaN.  Entries m .. mpad-1 are zero (the SYRK loader's tail SNPs).
__device__ __forceinline__ uint32_t bf16_rne(float f) {
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7f800000u) == 0x7f800000u) return (u >> 16) | ((u & 0xffffu) ? 0x40u : 0u);
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__global__ __launch_bounds__(256) void k_lut_bf3(const float* __restrict__ lut, uint64_t m, uint64_t mpad,
                                                 uint32_t* __restrict__ lut3) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= mpad) return;
    uint32_t h[3][4] = {};
    if (s < m) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const float v = lut[4 * s + c];
            const uint32_t a0 = bf16_rne(v);
            const float r1 = v - __uint_as_float(a0 << 16);
            const uint32_t a1 = bf16_rne(r1);
            const float r2 = r1 - __uint_as_float(a1 << 16);
            h[0][c] = a0;
            h[1][c] = a1;
            h[2][c] = bf16_rne(r2);
        }
    }
    uint32_t o[8];
#pragma unroll
    for (int p = 0; p < 3; p++) {
        o[2 * p] = (h[p][0] & 0xff) | ((h[p][1] & 0xff) << 8) | ((h[p][2] & 0xff) << 16) | ((h[p][3] & 0xff) << 24);
        o[2 * p + 1] = (h[p][0] >> 8) | ((h[p][1] >> 8) << 8) | ((h[p][2] >> 8) << 16) | ((h[p][3] >> 8) << 24);
    }
    o[6] = o[7] = 0;
    reinterpret_cast<uint4*>(lut3 + 8 * s)[0] = make_uint4(o[0], o[1], o[2], o[3]);
    reinterpret_cast<uint4*>(lut3 + 8 * s)[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

// ---------------------------------------------------------------- f32 GRM as fp16x2 (3 products)
// fp16 carries 11 significant bits, so two fp16 values hold 22 of an f32's 24: a0 = f16(a),
// a1 = f16(a - a0) (a - a0 is exact in f32).  The error of a0 + a1 is <= 2^-22 |a| while a1 is
// normal in fp16, and <= 2^-25 absolute once it is subnormal.  Keeping a0 b0 + a0 b1 + a1 b0
// (every fp16 x fp16 product exact in the f32 accumulator; the dropped a1 b1 is <= 2^-22 |ab|)
// costs 3 MFMAs per f32 product instead of bf16x3's 6.  fp16's range is the price: the split
// is used only when every SNP's largest |LUT value| M_s lies in [2^-2, 2^15) (or is 0 / NaN),
// which bounds the error of each product by ~2^-21 M_s^2 -- the magnitude of the SNP's largest
// K contribution -- and keeps a0 finite.  Unit always qualifies: M_s = max(mu, 2 - mu) / sigma
// >= 1 and <= 2 sqrt(n).  Beta weights can span 2^24 (Beta(1,25) at MAF 0.5 is 1.5e-6): then
// k_lut_h2 raises *flag and the bf16x3 kernel (gated on the same flag) computes the block.
//
// LUT: [mpad][4] u32, byte-planar like k_lut_bf3: word 2p / 2p+1 = low / high bytes of the fp16
// plane p of codes 0..3.
__global__ __launch_bounds__(256) void k_lut_h2(const float* __restrict__ lut, uint64_t m, uint64_t mpad,
                                                uint32_t* __restrict__ lut2, uint32_t* __restrict__ flag) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= mpad) return;
    uint32_t h[2][4] = {};
    if (s < m) {
        float M = 0.f;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const float v = lut[4 * s + c];
            M = fmaxf(M, fabsf(v));  // NaN entries are ignored (they stay NaN in both planes)
            const _Float16 a0 = (_Float16)v;
            const _Float16 a1 = (_Float16)(v - (float)a0);
            h[0][c] = __builtin_bit_cast(uint16_t, a0);
            h[1][c] = __builtin_bit_cast(uint16_t, a1);
        }
        if (M != 0.f && !(M >= 0.25f && M < 32768.f)) atomicOr(flag, 1u);
    }
    uint32_t o[4];
#pragma unroll
    for (int p = 0; p < 2; p++) {
        o[2 * p] = (h[p][0] & 0xff) | ((h[p][1] & 0xff) << 8) | ((h[p][2] & 0xff) << 16) | ((h[p][3] & 0xff) << 24);
        o[2 * p + 1] = (h[p][0] >> 8) | ((h[p][1] >> 8) << 8) | ((h[p][2] >> 8) << 16) | ((h[p][3] >> 8) << 24);
    }
    reinterpret_cast<uint4*>(lut2)[s] = make_uint4(o[0], o[1], o[2], o[3]);
}

// dense f32 block Z ([sid][ldz], F order) -> two fp16 planes for k_syrk_h2<.., DENSE>:
// planes[(s * 2 + p) * ldz + 16 d + pi(i)] = plane p of Z[s][16 d + i] (the packed loader's
// in-group order), rows >= n zero; a column whose max |z| is outside [2^-2, 2^15) (and not 0)
// raises *flag.  One 256-thread block per SNP column.
template <bool WRITE = true>
__global__ __launch_bounds__(256) void k_split_h2(const float* __restrict__ Z, uint64_t ldz, uint64_t n,
                                                  uint16_t* __restrict__ planes, uint32_t* __restrict__ flag) {
    const uint64_t s = blockIdx.x;
    const float* col = Z + s * ldz;
    uint16_t* p0 = planes + s * 2 * ldz;
    uint16_t* p1 = p0 + ldz;
    float M = 0.f;
    for (uint64_t r = threadIdx.x; r < ldz; r += 256) {
        const float v = r < n ? col[r] : 0.f;
        M = fmaxf(M, fabsf(v));
        const _Float16 a0 = (_Float16)v;
        const _Float16 a1 = (_Float16)(v - (float)a0);
        if constexpr (WRITE) {
            const uint64_t o = (r & ~15ull) + (uint64_t)pi16((int)(r & 15));
            p0[o] = __builtin_bit_cast(uint16_t, a0);
            p1[o] = __builtin_bit_cast(uint16_t, a1);
        }
    }
    __shared__ float red[256];
    red[threadIdx.x] = M;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float m = red[0];
        if (m != 0.f && !(m >= 0.25f && m < 32768.f)) atomicOr(flag, 1u);
    }
}

// dense f32 block Z ([sid][ldz]) -> the stage images of k_syrk_h2<.., 6, true>: for 16-SNP step
// t and 256-iid block b, plane p, a [16][288] fp16 tile laid out as the packed loader's LDS rows
// (pi order in each 16-iid group, 16-B halves swapped in groups with bit 2 set); SNPs >= m and
// iids >= n are zero.  Grid (nb, steps), one thread per iid.  The range flag comes from
// k_split_h2<false> (column max only).
__global__ __launch_bounds__(256) void k_image_h2(const float* __restrict__ Z, uint64_t ldz, uint64_t n, uint64_t m,
                                                  short* __restrict__ img) {
    const uint64_t b = blockIdx.x, t = blockIdx.y, nbk = gridDim.x;
    const int i = threadIdx.x, d = i >> 4, q = pi16(i & 15), sw = (d >> 2) & 1;
    const int pos = 16 * d + 8 * ((q >> 3) ^ sw) + (q & 7);
    short* o0 = img + ((t * nbk + b) * 2) * (uint64_t)B3_PLANE + pos;
    short* o1 = o0 + B3_PLANE;
    const uint64_t iid = b * 256 + i;
#pragma unroll 4
    for (int k = 0; k < 16; k++) {
        const uint64_t snp = t * 16 + k;
        const float v = (snp < m && iid < n) ? Z[snp * ldz + iid] : 0.f;
        const _Float16 a0 = (_Float16)v;
        const _Float16 a1 = (_Float16)(v - (float)a0);
        o0[k * B3_RS] = __builtin_bit_cast(short, a0);
        o1[k * B3_RS] = __builtin_bit_cast(short, a1);
    }
}

typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));

// Same block structure, loader roles and LDS image as k_syrk_bf3 (two fp16 planes per panel
// instead of three bf16 planes); per 16-SNP k-step each wave runs 3 groups of 8
// v_mfma_f32_32x32x16_f16: (A0,B0), (A0,B1), (A1,B0).  Runs only when *flag == 0 (see k_lut_h2).
// MODE 4 (packed codes): 32-SNP stages (two k-steps, one barrier per 32 SNPs); stage s+1's codes
// (loaded one stage ahead) are expanded and stored plane by plane beside the MFMA groups of stage
// s, the loads of stage s+2 are issued, then the barrier; stage s+1's B fragments are read under
// the last group.  The loader's ds_write_b64 stores place 8-B piece j of 16-iid group d at slot
// (j + (d >> 2)) & 3 of the group's 32-B segment (a rotation): the 16 lanes of each ds_write_b64
// group then hit 32 distinct banks (the 16-B-half swap the ds_write_b128 form needed left them 2-way
// conflicted, PMC SQ_LDS_BANK_CONFLICT = 29% of SQ_LDS_IDX_ACTIVE, profiles/r04n); the transposed
// fragment reads undo the rotation per lane.  k_syrk_h2s (below) is the same kernel with the loader
// in its own waves -- the default since round 6; this form stays for the split-K grids and as
// hook "h2" = 0.
// MODE 6 (DENSE): the operand is a dense float block already rewritten by k_image_h2 as stage
// images (the exact LDS rows the packed loader would build, swap layout), moved into LDS by
// LDS-DMA.
template <bool LOCAL = false, int MODE = 4, bool DENSE = false>
__global__ __launch_bounds__(512, 1) void k_syrk_h2(const uint8_t* __restrict__ P, uint64_t pitch, uint64_t n,
                                                    uint64_t kdim, const uint32_t* __restrict__ lut2,
                                                    const uint32_t* __restrict__ flag, float* __restrict__ tiles,
                                                    int accumulate, uint32_t part_rank = 0, uint32_t part_world = 1,
                                                    uint64_t kslice = 0, uint64_t slice_elems = 0,
                                                    SegCtx seg = SegCtx(), const uint32_t* __restrict__ order = nullptr,
                                                    uint64_t wg0 = 0) {
    static_assert(MODE == 4 || (MODE == 6 && DENSE), "k_syrk_h2: MODE 4 (packed) or MODE 6 (dense stage images)");
    // wg0: first block of this launch in the full grid's order (a column group of the triangle,
    // launch_syrk_packed_h2_cols); block identity, storage and SegFlush phase follow wg0 + blockIdx.x
    constexpr int KS = 2, SBK = KS * BK;  // two 16-SNP k-steps per LDS stage
    constexpr int PLANE = KS * B3_PLANE, STAGE = 2 * 2 * PLANE;
    constexpr bool kRot = MODE == 4;
    __shared__ __attribute__((aligned(16))) short lds[2 * STAGE];
    if (*flag) return;  // a SNP of this block is outside fp16's range: k_syrk_bf3 runs instead
    if (gridDim.y > 1) {
        const uint64_t k0 = (uint64_t)blockIdx.y * kslice;
        P += k0 * pitch;
        lut2 += 4 * k0;
        kdim = min(kslice, kdim - k0);
        tiles += (uint64_t)blockIdx.y * slice_elems;
    }
    const uint64_t wg = wg0 + blockIdx.x;
    uint32_t bi, bj;
    if constexpr (DENSE) {
        // lut2 = block order table (supertile_order): the 256 blocks in flight share 32 panels
        const uint32_t c = lut2[wg];
        bi = c & 0xffffu;
        bj = c >> 16;
    } else if (LOCAL || order) {  // block order table (supertile_order) / the part's layout table (part_layout)
        const uint32_t c = order[wg];
        bi = c & 0xffffu;
        bj = c >> 16;
    } else {
        tile_coords(wg, bi, bj);
    }
    // LOCAL: slot wg of the part's layout table is the block's storage slot and SegFlush phase
    const uint64_t blk = wg;
    const uint64_t i0 = (uint64_t)bi * BW, j0 = (uint64_t)bj * BW;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int lp = t >> 8, lk = (t >> 4) & 15, ld_ = t & 15;
    const uint8_t* wp = P + (lp ? j0 : i0) / 4 + 4 * ld_ + (uint64_t)lk * pitch;
    const uint8_t* wlast = P + (lp ? j0 : i0) / 4 + 4 * ld_ + (kdim - 1) * pitch;
    const uint32_t* lp2 = lut2 + 4 * lk;
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int rd_base = (8 * (g >> 1) + q) * B3_RS + 16 * (g & 1);
    const int rd_off = rd_base + 4 * pp;
    const int dswz = (pp >> 1) ? -8 : 8;
    // swap layout (MODE 6 images): A fragments x >= 2 and B fragments of odd wn sit in swapped
    // segments; rotation layout (MODE 4): a fragment column c lies in segments rotated by (c / 64) & 3
    const int rd_offA0 = kRot ? rd_base + 4 * ((pp + 2 * wm) & 3) : rd_off;
    const int rd_offA1 = kRot ? rd_base + 4 * ((pp + 2 * wm + 1) & 3) : rd_off + dswz;
    const int rd_offB = kRot ? rd_base + 4 * ((pp + wn) & 3) : rd_off + ((wn & 1) ? dswz : 0);
    const int wrot = (ld_ >> 2) & 3;  // this lane's group rotation (store side)

    f32x16 acc[4][2];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = (f32x16){};
    const uint64_t nst = (kdim + SBK - 1) / SBK;

    uint32_t rw[KS];
    uint4 rl[KS];
    auto load = [&](uint64_t st) {
#pragma unroll
        for (int h = 0; h < KS; h++) {
            const uint8_t* a = wp + (st * SBK + h * BK) * pitch;
            rw[h] = *reinterpret_cast<const uint32_t*>(a <= wlast ? a : wlast);
            rl[h] = *reinterpret_cast<const uint4*>(lp2 + 4 * (SBK * st + h * BK));
        }
    };
    auto make_sel = [&](uint32_t w, uint32_t (&sel)[8]) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t v = (w >> (2 * j)) & 0x03030303u;
            const uint32_t o = v | 0x04040404u;
            sel[2 * j] = __builtin_amdgcn_perm(o, v, 0x05010400u);
            sel[2 * j + 1] = __builtin_amdgcn_perm(o, v, 0x07030602u);
        }
    };
    auto store_plane = [&](short* S, int pl, int h, const uint32_t (&sel)[8]) {
        const uint32_t lo = pl == 0 ? rl[h].x : rl[h].z;
        const uint32_t hi = pl == 0 ? rl[h].y : rl[h].w;
        // two ds_write_b64 per 16-B half (6 LDS-transfer cycles per wave-instruction vs 13 for
        // ds_write_b128; volatile + explicit LDS address space so they are neither re-merged nor
        // turned into flat stores): +1.2-1.3%, bit-identical K (profiles/r03crt/ubench_lds_store_width.jsonl)
        typedef __attribute__((address_space(3))) volatile uint64_t lds_u64;
        lds_u64* qq = (lds_u64*)(S + (lp * 2 + pl) * PLANE + (lk + BK * h) * B3_RS + 16 * ld_);
#pragma unroll
        for (int j = 0; j < 4; j++)
            qq[(wrot + j) & 3] = (uint64_t)__builtin_amdgcn_perm(hi, lo, sel[2 * j]) |
                                 ((uint64_t)__builtin_amdgcn_perm(hi, lo, sel[2 * j + 1]) << 32);
    };
    auto frag = [&](const short* S, int panel, int pl, int h, int col, int off) -> f16x8_t {
        const short* b = S + (panel * 2 + pl) * PLANE + h * BK * B3_RS + off + col;
        const i16x4_t r0 = lds_tr16(b), r1 = lds_tr16(b + 4 * B3_RS);
        return __builtin_bit_cast(f16x8_t, (i16x8_t)__builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    auto fragB = [&](const short* S, int pl, int h, f16x8_t (&b)[2]) {
#pragma unroll
        for (int y = 0; y < 2; y++) b[y] = frag(S, 1, pl, h, wn * 64 + 32 * y, rd_offB);
    };
    auto fragsA = [&](const short* S, int pa, int h, f16x8_t (&a)[4]) {
#pragma unroll
        for (int x = 0; x < 4; x++) a[x] = frag(S, 0, pa, h, wm * 128 + 32 * x, x >= 2 ? rd_offA1 : rd_offA0);
    };
    auto group = [&](const f16x8_t (&a)[4], const f16x8_t (&b)[2]) {
#pragma unroll
        for (int x = 0; x < 4; x++)
#pragma unroll
            for (int y = 0; y < 2; y++)
                acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[x], b[y], acc[x][y], 0, 0, 0);
    };
    __shared__ uint32_t seg_slot;
    if constexpr (MODE == 6) {
        // DENSE stage images (k_image_h2): P = [16-SNP step t][256-iid block b][plane][16 rows x
        // 288 fp16], exactly the LDS rows the packed loader writes, so a stage is 8 contiguous
        // 9 KiB pieces moved by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction,
        // 9 per wave) -- no VGPR staging, no ds_write; one barrier per 32 SNPs
        const uint64_t nbk = (n + 255) / 256;  // = the image grid's x
        const short* img = reinterpret_cast<const short*>(P);
        auto issue = [&](uint64_t st, short* S) {
#pragma unroll
            for (int j = 0; j < 9; j++) {
                const int c = wave * 9 + j;  // 72 pieces: [panel][plane][h][piece]
                const int panel = c / 36, rem = c % 36, pl = rem / 18, h = (rem / 9) & 1, piece = rem % 9;
                const uint64_t b = panel ? bj : bi;
                const short* src = img + (((2 * st + h) * nbk + b) * 2 + pl) * (uint64_t)B3_PLANE + piece * 512 + 8 * lane;
                short* dst = S + (panel * 2 + pl) * PLANE + h * B3_PLANE + piece * 512;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                                 (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
            }
        };
        issue(0, lds);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        SegFlush sf(seg, SBK, blk, nst, &seg_slot);
        for (uint64_t s = 0; s < nst; s++) {
            const short* cur = lds + (s & 1) * STAGE;
            if (s + 1 < nst) issue(s + 1, lds + ((s + 1) & 1) * STAGE);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                f16x8_t A0[4], A1[4], B0[2], B1[2];
                fragsA(cur, 0, h, A0);
                fragB(cur, 0, h, B0);
                fragB(cur, 1, h, B1);
                fragsA(cur, 1, h, A1);
                group(A0, B0);
                group(A0, B1);
                group(A1, B0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (sf.due(s + 1 < nst)) sf.flush(acc);
        }
        sf.finish(acc);
        epilogue_pi<LOCAL>(acc, tiles, n, bi, bj, accumulate, lane, wm, wn, blk);
        sf.release(seg);
        return;
    }
    // f32 accuracy: SegFlush (above) cuts the accumulation chains every seg SNPs inside this loop.
    const uint64_t send = nst;  // the loader clamps its stage index to send - 1
    f16x8_t B0s[2], B1s[2], B0t[2], B1t[2];
    auto prologue = [&](uint64_t s0) {
        load(s0);
#pragma unroll
        for (int h = 0; h < KS; h++) {
            uint32_t sel[8];
            make_sel(rw[h], sel);
            store_plane(lds, 0, h, sel);
            store_plane(lds, 1, h, sel);
        }
        load(s0 + 1 < send ? s0 + 1 : send - 1);
        __syncthreads();
        fragB(lds, 0, 0, B0s);
        fragB(lds, 1, 0, B1s);
    };
    // The loader runs unconditionally (the last stage expands into the idle buffer and its code
    // loads clamp to the last stage) so each MFMA group and its VALU share one basic block.
    auto stage = [&](uint64_t s, f16x8_t (&B0)[2], f16x8_t (&B1)[2], f16x8_t (&B0n)[2], f16x8_t (&B1n)[2]) {
        const short* cur = lds + (s & 1) * STAGE;
        short* nxt = lds + ((s + 1) & 1) * STAGE;
        // k-step 0 with the prefetched B, k-step 1 read from cur before the barrier (after it,
        // stage s+1's stores may overwrite cur); the expansion of stage s+1 (2 k-steps x 2 planes)
        // rides on groups 0-3
        f16x8_t Ax[4], Ay[4], C0[2], C1[2];
        fragsA(cur, 0, 0, Ax);
        fragsA(cur, 1, 0, Ay);
        uint32_t sel[8];
        group(Ax, B0);
        make_sel(rw[0], sel);
        store_plane(nxt, 0, 0, sel);
        group(Ax, B1);
        store_plane(nxt, 1, 0, sel);
        fragB(cur, 0, 1, C0);
        fragB(cur, 1, 1, C1);
        fragsA(cur, 0, 1, Ax);
        group(Ay, B0);
        make_sel(rw[1], sel);
        store_plane(nxt, 0, 1, sel);
        fragsA(cur, 1, 1, Ay);
        group(Ax, C0);
        store_plane(nxt, 1, 1, sel);
        group(Ax, C1);
        load(s + 2 < send ? s + 2 : send - 1);
        __syncthreads();
        fragB(nxt, 0, 0, B0n);
        fragB(nxt, 1, 0, B1n);
        group(Ay, C0);
    };
    SegFlush sf(seg, 2 * SBK, blk, (nst + 1) / 2, &seg_slot);
    prologue(0);
    for (uint64_t s = 0; s < nst; s += 2) {
        stage(s, B0s, B1s, B0t, B1t);
        if (s + 1 < nst) stage(s + 1, B0t, B1t, B0s, B1s);
        if (sf.due(s + 2 < nst)) sf.flush(acc);
    }
    sf.finish(acc);
    epilogue_pi<LOCAL>(acc, tiles, n, bi, bj, accumulate, lane, wm, wn, blk);
    sf.release(seg);
}

// Warp-specialised k_syrk_h2 (MODE 4 layout, round 6): the same block, products, LDS image (ROT
// rotation) and SegFlush, with the loader moved out of the MFMA waves.  12 waves (3 per SIMD):
// waves 0-7 only read fragments (ds_read_b64_tr_b16) and issue the 3 x 8 MFMAs of each 16-SNP
// k-step; waves 8-11 (one per SIMD) expand stage s+1's codes into the idle LDS buffer -- 4 SNP rows
// x 2 planes per thread and stage, ds_write_b64 -- and issue stage s+2's code / LUT loads while the
// MFMA waves compute stage s.  One barrier per 32-SNP stage, as in MODE 4.  Register budget of 3
// waves per SIMD (<= 168): the MFMA waves hold each k-step's B planes and ONE A plane at a time.
template <bool LOCAL = false>
__global__ __launch_bounds__(768, 1) void k_syrk_h2s(const uint8_t* __restrict__ P, uint64_t pitch, uint64_t n,
                                                     uint64_t kdim, const uint32_t* __restrict__ lut2,
                                                     const uint32_t* __restrict__ flag, float* __restrict__ tiles,
                                                     int accumulate, uint32_t part_rank = 0, uint32_t part_world = 1,
                                                     uint64_t kslice = 0, uint64_t slice_elems = 0,
                                                     SegCtx seg = SegCtx(), const uint32_t* __restrict__ order = nullptr,
                                                     uint64_t wg0 = 0) {
    constexpr int KS = 2, SBK = KS * BK;
    constexpr int PLANE = KS * B3_PLANE, STAGE = 2 * 2 * PLANE;
    __shared__ __attribute__((aligned(16))) short lds[2 * STAGE];
    if (*flag) return;  // a SNP of this block is outside fp16's range: k_syrk_bf3 runs instead
    if (gridDim.y > 1) {
        const uint64_t k0 = (uint64_t)blockIdx.y * kslice;
        P += k0 * pitch;
        lut2 += 4 * k0;
        kdim = min(kslice, kdim - k0);
        tiles += (uint64_t)blockIdx.y * slice_elems;
    }
    const uint64_t wg = wg0 + blockIdx.x;
    uint32_t bi, bj;
    if (LOCAL || order) {
        const uint32_t c = order[wg];
        bi = c & 0xffffu;
        bj = c >> 16;
    } else {
        tile_coords(wg, bi, bj);
    }
    const uint64_t blk = wg;
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const uint64_t nst = (kdim + SBK - 1) / SBK;
    __shared__ uint32_t seg_slot;
    SegFlush sf(seg, 2 * SBK, blk, (nst + 1) / 2, &seg_slot);  // every wave: it holds a barrier
    if (wave >= 8) {
        // loader thread lt = (panel lp, SNP rows lk + 8u of the stage (u < 4), 16-iid group ld_)
        const int lt = t - 512;
        const int lp = __builtin_amdgcn_readfirstlane(lt >> 7), lk = (lt >> 4) & 7, ld_ = lt & 15;
        const uint64_t c0 = (uint64_t)(lp ? bj : bi) * BW;
        const uint8_t* wp = P + c0 / 4 + 4 * ld_ + (uint64_t)lk * pitch;
        const uint8_t* wlast = P + c0 / 4 + 4 * ld_ + (kdim - 1) * pitch;
        const int wrot = (ld_ >> 2) & 3;
        uint32_t rw[4];
        uint4 rl[4];
        auto load = [&](uint64_t st) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint8_t* a = wp + (st * SBK + 8 * u) * pitch;
                rw[u] = *reinterpret_cast<const uint32_t*>(a <= wlast ? a : wlast);
                rl[u] = *reinterpret_cast<const uint4*>(lut2 + 4 * (SBK * st + lk + 8 * u));
            }
        };
        auto store = [&](short* S) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                uint32_t sel[8];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t v = (rw[u] >> (2 * j)) & 0x03030303u;
                    const uint32_t o = v | 0x04040404u;
                    sel[2 * j] = __builtin_amdgcn_perm(o, v, 0x05010400u);
                    sel[2 * j + 1] = __builtin_amdgcn_perm(o, v, 0x07030602u);
                }
#pragma unroll
                for (int pl = 0; pl < 2; pl++) {
                    const uint32_t lo = pl == 0 ? rl[u].x : rl[u].z;
                    const uint32_t hi = pl == 0 ? rl[u].y : rl[u].w;
                    typedef __attribute__((address_space(3))) volatile uint64_t lds_u64;
                    lds_u64* q = (lds_u64*)(S + (lp * 2 + pl) * PLANE + (lk + 8 * u) * B3_RS + 16 * ld_);
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        q[(wrot + j) & 3] = (uint64_t)__builtin_amdgcn_perm(hi, lo, sel[2 * j]) |
                                            ((uint64_t)__builtin_amdgcn_perm(hi, lo, sel[2 * j + 1]) << 32);
                }
            }
        };
        load(0);
        store(lds);
        load(nst > 1 ? 1 : 0);
        __syncthreads();
        for (uint64_t s = 0; s < nst; s++) {
            store(lds + ((s + 1) & 1) * STAGE);  // stage s+1 (past the end: the idle buffer, unread)
            load(s + 2 < nst ? s + 2 : nst - 1);
            __syncthreads();
        }
        sf.release(seg);
        return;
    }
    const int wm = wave >> 2, wn = wave & 3;
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int rd_base = (8 * (g >> 1) + q) * B3_RS + 16 * (g & 1);
    const int rd_offA0 = rd_base + 4 * ((pp + 2 * wm) & 3), rd_offA1 = rd_base + 4 * ((pp + 2 * wm + 1) & 3);
    const int rd_offB = rd_base + 4 * ((pp + wn) & 3);
    f32x16 acc[4][2];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = (f32x16){};
    auto frag = [&](const short* S, int panel, int pl, int h, int col, int off) -> f16x8_t {
        const short* b = S + (panel * 2 + pl) * PLANE + h * BK * B3_RS + off + col;
        const i16x4_t r0 = lds_tr16(b), r1 = lds_tr16(b + 4 * B3_RS);
        return __builtin_bit_cast(f16x8_t, (i16x8_t)__builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    auto group = [&](const f16x8_t (&a)[4], const f16x8_t (&b)[2]) {
#pragma unroll
        for (int x = 0; x < 4; x++)
#pragma unroll
            for (int y = 0; y < 2; y++)
                acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[x], b[y], acc[x][y], 0, 0, 0);
    };
    __syncthreads();
    for (uint64_t s = 0; s < nst; s++) {
        const short* cur = lds + (s & 1) * STAGE;
#pragma unroll
        for (int h = 0; h < KS; h++) {
            f16x8_t A[4], B0[2], B1[2];
#pragma unroll
            for (int y = 0; y < 2; y++) {
                B0[y] = frag(cur, 1, 0, h, wn * 64 + 32 * y, rd_offB);
                B1[y] = frag(cur, 1, 1, h, wn * 64 + 32 * y, rd_offB);
            }
#pragma unroll
            for (int x = 0; x < 4; x++) A[x] = frag(cur, 0, 0, h, wm * 128 + 32 * x, x >= 2 ? rd_offA1 : rd_offA0);
            group(A, B0);
            group(A, B1);
#pragma unroll
            for (int x = 0; x < 4; x++) A[x] = frag(cur, 0, 1, h, wm * 128 + 32 * x, x >= 2 ? rd_offA1 : rd_offA0);
            group(A, B0);
        }
        __syncthreads();
        if ((s & 1) && sf.due(s + 1 < nst)) sf.flush(acc);
    }
    sf.finish(acc);
    epilogue_pi<LOCAL>(acc, tiles, n, bi, bj, accumulate, lane, wm, wn, blk);
    sf.release(seg);
}

}  // namespace f32w

// ====================================================================== f64
namespace f64k {
constexpr int BK = 16;
constexpr int LDA = BM + 16;  // doubles per LDS row: +32 dwords shifts row k+1 by half the banks

struct PRegs {
    uint32_t w;
    double l[4];
};

// packed: op = t>>7; 128 threads cover BK=16 SNPs x 8 dwords.
__device__ __forceinline__ void load_packed(const uint8_t* __restrict__ P, uint64_t pitch, uint64_t kdim, uint64_t k0,
                                            uint64_t i0, uint64_t j0, const double* __restrict__ lut, PRegs& r) {
    const int t = threadIdx.x;
    const int op = t >> 7, tt = t & 127;
    const int k = tt >> 3, d = tt & 7;
    const uint64_t base = op ? j0 : i0;
    const uint64_t kk = k0 + k;
    if (kk < kdim) {
        r.w = *reinterpret_cast<const uint32_t*>(P + kk * pitch + base / 4 + 4 * d);
        const double2 x = *reinterpret_cast<const double2*>(lut + 4 * kk);
        const double2 y = *reinterpret_cast<const double2*>(lut + 4 * kk + 2);
        r.l[0] = x.x;
        r.l[1] = x.y;
        r.l[2] = y.x;
        r.l[3] = y.y;
    } else {
        r.w = 0;
        r.l[0] = r.l[1] = r.l[2] = r.l[3] = 0.0;
    }
}

__device__ __forceinline__ void store_packed(double* As, double* Bs, const PRegs& r) {
    const int t = threadIdx.x;
    const int op = t >> 7, tt = t & 127;
    const int k = tt >> 3, d = tt & 7;
    double* S = op ? Bs : As;
#pragma unroll
    for (int v = 0; v < 8; v++) {
        double2 o;
        o.x = sel4(r.l[0], r.l[1], r.l[2], r.l[3], (r.w >> (4 * v)) & 3u);
        o.y = sel4(r.l[0], r.l[1], r.l[2], r.l[3], (r.w >> (4 * v + 2)) & 3u);
        *reinterpret_cast<double2*>(S + k * LDA + 16 * d + 2 * v) = o;
    }
}

// same, with the select done on the two 32-bit halves by v_bfi_b32 (8 VALU per value)
// ROT: write chunk (v + (d>>1) + 4(k&1)) & 7 at step v so that each 16-lane quarter of the
// wave hits 16 distinct 4-bank groups (row stride 288 dwords = 32 mod 64 banks; without
// the rotation all 64 lanes of a ds_write_b128 land on 2 groups).
template <int V0 = 0, int V1 = 8, bool ROT = false>
__device__ __forceinline__ void store_packed_bfi(double* As, double* Bs, const PRegs& r) {
    const int t = threadIdx.x;
    const int op = t >> 7, tt = t & 127;
    const int k = tt >> 3, d = tt & 7;
    double* S = op ? Bs : As;
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const uint64_t u = (uint64_t)__double_as_longlong(r.l[c]);
        lo[c] = (uint32_t)u;
        hi[c] = (uint32_t)(u >> 32);
    }
    const int rot = ROT ? (d >> 1) + 4 * (k & 1) : 0;
#pragma unroll
    for (int v0 = V0; v0 < V1; v0++) {
        const int v = (v0 + rot) & 7;
        double o[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t sh = 4 * v + 2 * h;
            const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int)r.w, sh, 1u);
            const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int)r.w, sh + 1u, 1u);
            const uint32_t a = bfi(m1, bfi(m0, lo[3], lo[2]), bfi(m0, lo[1], lo[0]));
            const uint32_t b = bfi(m1, bfi(m0, hi[3], hi[2]), bfi(m0, hi[1], hi[0]));
            o[h] = __longlong_as_double((long long)(((uint64_t)b << 32) | a));
        }
        *reinterpret_cast<double2*>(S + k * LDA + 16 * d + 2 * v) = make_double2(o[0], o[1]);
    }
}

// one stage's MFMAs: 16 SNPs x the wave's 64 x 64 (4 x 4 v_mfma_f64_16x16x4f64 tiles)
__device__ __forceinline__ void compute(const double* As, const double* Bs, f64x4 (&acc)[4][4], int wm, int wn,
                                        int lane) {
    const int kr = lane >> 4, c = lane & 15;
#pragma unroll
    for (int kk = 0; kk < BK / 4; kk++) {
        const int row = (4 * kk + kr) * LDA;
        double a[4], b[4];
#pragma unroll
        for (int x = 0; x < 4; x++) {
            a[x] = As[row + wm * 64 + 16 * x + c];
            b[x] = Bs[row + wn * 64 + 16 * x + c];
        }
#pragma unroll
        for (int x = 0; x < 4; x++)
#pragma unroll
            for (int y = 0; y < 4; y++) acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], b[y], acc[x][y], 0, 0, 0);
    }
}

// The stage's MFMAs with the next stage's LDS store (bfi select) spread between its MFMA groups, so
// the select VALU issues while the wave's own MFMAs are in flight instead of after them.
template <bool ROT = false>
__device__ __forceinline__ void compute_store(const double* As, const double* Bs, f64x4 (&acc)[4][4], int wm, int wn,
                                              int lane, double* Ns, double* Nb, const PRegs& r, bool more) {
    const int kr = lane >> 4, c = lane & 15;
#pragma unroll
    for (int kk = 0; kk < BK / 4; kk++) {
        const int row = (4 * kk + kr) * LDA;
        double a[4], b[4];
#pragma unroll
        for (int x = 0; x < 4; x++) {
            a[x] = As[row + wm * 64 + 16 * x + c];
            b[x] = Bs[row + wn * 64 + 16 * x + c];
        }
#pragma unroll
        for (int x = 0; x < 4; x++)
#pragma unroll
            for (int y = 0; y < 4; y++) acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], b[y], acc[x][y], 0, 0, 0);
        if (more) {
            if (kk == 0) store_packed_bfi<0, 2, ROT>(Ns, Nb, r);
            if (kk == 1) store_packed_bfi<2, 4, ROT>(Ns, Nb, r);
            if (kk == 2) store_packed_bfi<4, 6, ROT>(Ns, Nb, r);
            if (kk == 3) store_packed_bfi<6, 8, ROT>(Ns, Nb, r);
        }
    }
}

// f64 16x16x4 C/D layout: col = lane&15, row = (lane>>4) + 4*r.  T: the 128x128 output tile,
// row stride ldo (BM for the tile store, 256 inside a cfg5 part's dense block)
__device__ __forceinline__ void epilogue(f64x4 (&acc)[4][4], double* __restrict__ T, uint64_t ldo, int accumulate,
                                         int lane, int wm, int wn) {
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 4; y++) {
            double* base = T + (wm * 64 + 16 * x + (lane >> 4)) * ldo + wn * 64 + 16 * y + (lane & 15);
            if (accumulate) {
                double old[4];
#pragma unroll
                for (int r = 0; r < 4; r++) old[r] = base[4 * r * ldo];
#pragma unroll
                for (int r = 0; r < 4; r++) acc[x][y][r] += old[r];
            }
#pragma unroll
            for (int r = 0; r < 4; r++) base[4 * r * ldo] = acc[x][y][r];
        }
}

// f64 GRM of packed codes on the f64 MFMA (the CRT path's fallback for a non-finite LUT, and hook
// "f64" = 1): 128x128 tiles, 4 waves; the select of stage s+1's values is interleaved with stage s's
// MFMAs and stored bank-rotated (compute_store<true>): 60.5 TFLOP/s = 0.77 of 78.6 at N = 32768
// (tools/ubench.py syrk --dtype f64).  part_tab (cfg5): quadrant q of slot w of the part's layout.
__global__ __launch_bounds__(256, 2) void k_syrk(const uint8_t* __restrict__ src, uint64_t ld, uint64_t kdim,
                                                 const double* __restrict__ lut, double* __restrict__ tiles,
                                                 int accumulate, const int* __restrict__ gate = nullptr,
                                                 const uint32_t* __restrict__ part_tab = nullptr) {
    __shared__ __attribute__((aligned(16))) double lds[2][2][BK * LDA];
    if (gate && *gate == 0) return;  // fallback of the CRT path: runs only when its flag is set
    uint32_t ti, tj;
    double* T;
    uint64_t ldo = BM;
    if (part_tab) {  // cfg5: quadrant q of slot w of the part's layout, written into its dense block
        const uint64_t w = blockIdx.x >> 2, q = blockIdx.x & 3;
        ti = 2 * (part_tab[w] & 0xffffu) + (uint32_t)(q & 1);
        tj = 2 * (part_tab[w] >> 16) + (uint32_t)(q >> 1);
        T = tiles + w * 65536 + (q & 1) * 128 * 256 + (q >> 1) * 128;
        ldo = 256;
    } else {
        tile_coords(blockIdx.x, ti, tj);
        T = tiles + (uint64_t)blockIdx.x * (BM * BM);
    }
    const uint64_t i0 = (uint64_t)ti * BM, j0 = (uint64_t)tj * BM;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    f64x4 acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 4; y++) acc[x][y] = (f64x4){};

    const uint64_t nst = (kdim + BK - 1) / BK;
    PRegs rp;
    load_packed(src, ld, kdim, 0, i0, j0, lut, rp);
    store_packed(lds[0][0], lds[0][1], rp);
    __syncthreads();
    for (uint64_t s = 0; s < nst; s++) {
        const int buf = s & 1;
        const bool more = s + 1 < nst;
        if (more) load_packed(src, ld, kdim, (s + 1) * BK, i0, j0, lut, rp);
        compute_store<true>(lds[buf][0], lds[buf][1], acc, wm, wn, lane, lds[buf ^ 1][0], lds[buf ^ 1][1], rp, more);
        __syncthreads();
    }
    epilogue(acc, T, ldo, accumulate, lane, wm, wn);
}

// Dense f64 operand (F order, ldz >= round_up(n, 128)) streamed global -> LDS with
// global_load_lds_dwordx4: one wave-instruction = one 128-double (1 KiB) SNP row of a panel,
// rows padded to LDA (allowed: no instruction crosses a row).  No VALU in the loader.
__global__ __launch_bounds__(256, 2) void k_syrk_glds(const double* __restrict__ Z, uint64_t ldz, uint64_t kdim,
                                                      double* __restrict__ tiles, int accumulate) {
    __shared__ __attribute__((aligned(16))) double lds[2][2][BK * LDA];
    uint32_t ti, tj;
    tile_coords(blockIdx.x, ti, tj);
    const uint64_t i0 = (uint64_t)ti * BM, j0 = (uint64_t)tj * BM;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    f64x4 acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 4; y++) acc[x][y] = (f64x4){};
    const uint64_t nst = (kdim + BK - 1) / BK;
    auto issue = [&](uint64_t k0, int buf) {
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int r = wave * 8 + q;  // 32 rows per stage: 2 panels x BK
            const int panel = r >> 4, k = r & (BK - 1);
            double* dst = &lds[buf][panel][k * LDA];
            const uint64_t kk = k0 + k;
            if (kk < kdim) {
                const double* src = Z + kk * ldz + (panel ? j0 : i0) + 2 * lane;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                                 (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
            } else {
                reinterpret_cast<double2*>(dst)[lane] = make_double2(0.0, 0.0);
            }
        }
    };
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (uint64_t s = 0; s < nst; s++) {
        const int buf = s & 1;
        if (s + 1 < nst) issue((s + 1) * BK, buf ^ 1);
        compute(lds[buf][0], lds[buf][1], acc, wm, wn, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    epilogue(acc, tiles + (uint64_t)blockIdx.x * (BM * BM), BM, accumulate, lane, wm, wn);
}
}  // namespace f64k

}  // namespace

int g_variant_syrk = 0;  // tuning hook (snpmi_set_kernel_variant "syrk")
// 8192: 4.9e-6 of max diag at 50k x 100k on SnpGen-shaped data (21.8% missing) for +2.2% time;
// 4096: 2.6e-6 for +3.8%; 16384: 6.9e-6 for +1.9%; none: 3.2e-5 (profiles/r03acc, r03seg)
int g_seg_snps = 12288;  // tuning hook "seg" (round 4: 12288 with the exact f64 diagonal, k_diag_*)

// host-side segmentation for the f32-MFMA kernels without SegFlush (fallbacks and small-N
// kernels): one launch per <= g_seg_snps / 2 SNPs, each accumulating onto the previous ones
// (v_mfma_f32_32x32x2f32 adds 2 SNPs per rounding step where the fp16 kernels add 16 x 3 products)
template <class F>
static void for_segments(uint64_t m, int accumulate, F&& launch) {
    const uint64_t seg = g_seg_snps > 0 ? round_up((uint64_t)g_seg_snps / 2, 64) : m;
    for (uint64_t c0 = 0; c0 < m; c0 += seg) launch(c0, std::min(seg, m - c0), accumulate || c0 > 0);
}

void launch_syrk_packed(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const void* lut, int dtype,
                        void* tiles, int accumulate, hipStream_t st) {
    const uint64_t nt = n_tiles_upper(n);
    if (nt == 0) return;
    SNPMI_REQUIRE(nt < (1ull << 31), SNPMI_E_ARG, "too many GRM tiles for one launch");
    if (m == 0) {
        if (!accumulate) SNPMI_HIP(hipMemsetAsync(tiles, 0, nt * BM * BM * dtype_size(dtype), st));
        return;
    }
    if (dtype == SNPMI_DT_F32) {
        const float* L = (const float*)lut;
        float* Tt = (float*)tiles;
        // Kernel choice (tools/ubench.py syrk, MI355X): 256x256 / 8 waves reaches 129 TFLOP/s at
        // N=50k (82%) vs 118 for 128x128 / 4 waves; below ~4k iids the 256 tiles leave CUs idle.
        const uint64_t nb = ceil_div(n, 256);
        // Reached for f32 only when the product path is forced off the fp16x2/bf16x3 kernels
        // (variant 20; below N = 4096 the 128x128 kernel, variant 5)
        const bool big = g_variant_syrk != 5 && n >= 4096;
        for_segments(m, accumulate, [&](uint64_t c0, uint64_t cnt, int acc) {
            if (big)
                f32w::k_syrk256<1><<<(unsigned)(nb * (nb + 1) / 2), 512, 0, st>>>(packed + c0 * pitch, pitch, n, cnt,
                                                                                 L + 4 * c0, Tt, acc);
            else
                f32k::k_syrk<true, 16, 4><<<(unsigned)nt, 256, 0, st>>>(packed + c0 * pitch, pitch, cnt, L + 4 * c0, Tt,
                                                                       acc);
            SNPMI_HIP(hipGetLastError());
        });
        return;
    }
    else {
        const double* L = (const double*)lut;
        double* Tt = (double*)tiles;
        // tools/ubench.py syrk --dtype f64 (N=32768, 8192 SNPs): plain loader 51.3 TFLOP/s, select
        // interleaved with the MFMAs 56.1, that + bank-rotated LDS stores (MODE 4) 60.5 (77% of
        // 78.6); MFMA-only ablation 71.5.
        f64k::k_syrk<<<(unsigned)nt, 256, 0, st>>>(packed, pitch, m, L, Tt, accumulate);
    }
    SNPMI_HIP(hipGetLastError());
}

void launch_syrk_packed_f64_gated(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const double* lut,
                                  double* tiles, int accumulate, const int* gate, hipStream_t st,
                                  const uint32_t* part_tab, uint64_t part_blocks) {
    const uint64_t nt = part_tab ? 4 * part_blocks : n_tiles_upper(n);
    if (nt == 0 || m == 0) return;
    SNPMI_REQUIRE(nt < (1ull << 31), SNPMI_E_ARG, "too many GRM tiles for one launch");
    f64k::k_syrk<<<(unsigned)nt, 256, 0, st>>>(packed, pitch, m, lut, tiles, accumulate, gate, part_tab);
    SNPMI_HIP(hipGetLastError());
}

// cfg5 ownership of K (round 5).  The upper triangle of 256-iid blocks is cut into S x S-block
// supertiles (S = part_unit: 16 once there are enough supertiles to deal out, else smaller),
// dealt round-robin in triangular order: supertile T = J(J+1)/2 + I belongs to part T mod world.
// A part stores its blocks densely in walk order -- its supertiles in T order, each supertile's
// blocks column by column (bj outer, bi <= bj inner) -- and every LOCAL kernel reads block
// (bi, bj) of workgroup w from that table (entry bi | bj << 16) and writes it to slot w.  So the
// ~256 blocks in flight share ~32 code panels, as in the replicated kernel's supertile order,
// instead of the ~108 of round 4's single-block round-robin ownership.
uint64_t part_unit(uint64_t nb, int world) {
    for (uint64_t S = 16; S > 1; S /= 2) {
        const uint64_t ns = ceil_div(nb, S);
        if (ns * (ns + 1) / 2 >= 4 * (uint64_t)std::max(world, 1)) return S;
    }
    return 1;
}

static uint64_t supertile_blocks(uint64_t nb, uint64_t S, uint64_t I, uint64_t J) {
    const uint64_t c = std::min(S, nb - S * J);
    return I == J ? c * (c + 1) / 2 : std::min(S, nb - S * I) * c;
}

uint64_t grm_part_blocks(uint64_t n, int rank, int world) {
    const uint64_t nb = ceil_div(n, 256), S = part_unit(nb, world), ns = ceil_div(nb, S);
    uint64_t cnt = 0;
    for (uint64_t J = 0, T = 0; J < ns; J++)
        for (uint64_t I = 0; I <= J; I++, T++)
            if (T % (uint64_t)world == (uint64_t)rank) cnt += supertile_blocks(nb, S, I, J);
    return cnt;
}

void part_layout(uint64_t nb, int rank, int world, std::vector<uint32_t>& tab) {
    SNPMI_REQUIRE(nb < 65536, SNPMI_E_ARG, "partitioned GRM: too many 256-iid blocks (n >= 2^24)");
    tab.clear();
    const uint64_t S = part_unit(nb, world), ns = ceil_div(nb, S);
    for (uint64_t J = 0, T = 0; J < ns; J++)
        for (uint64_t I = 0; I <= J; I++, T++) {
            if (T % (uint64_t)world != (uint64_t)rank) continue;
            for (uint64_t bj = S * J; bj < std::min(S * J + S, nb); bj++)
                for (uint64_t bi = S * I; bi < std::min(S * I + S, bj + 1); bi++)
                    tab.push_back((uint32_t)(bi | (bj << 16)));
        }
}

void launch_syrk_packed_part(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const void* lut,
                             int rank, int world, void* blocks, int accumulate, hipStream_t st) {
    const uint64_t nloc = grm_part_blocks(n, rank, world);
    if (nloc == 0) return;
    SNPMI_REQUIRE(nloc < (1ull << 31), SNPMI_E_ARG, "too many GRM blocks for one launch");
    if (m == 0) {
        if (!accumulate) SNPMI_HIP(hipMemsetAsync(blocks, 0, nloc * 256 * 256 * sizeof(float), st));
        return;
    }
    const uint32_t* tab = part_tables(ceil_div(n, 256), rank, world).tab;
    for_segments(m, accumulate, [&](uint64_t c0, uint64_t cnt, int acc) {
        f32w::k_syrk256<1, true><<<(unsigned)nloc, 512, 0, st>>>(packed + c0 * pitch, pitch, n, cnt,
                                                                 (const float*)lut + 4 * c0, (float*)blocks, acc, tab);
        SNPMI_HIP(hipGetLastError());
    });
}

uint64_t lut_bf3_entries(uint64_t m) { return round_up(std::max<uint64_t>(m, 1), (uint64_t)2 * f32w::BK); }

void launch_lut_bf3(const float* lut, uint64_t m, uint32_t* lut3, hipStream_t st) {
    const uint64_t mpad = lut_bf3_entries(m);
    f32w::k_lut_bf3<<<(unsigned)ceil_div(mpad, 256), 256, 0, st>>>(lut, m, mpad, lut3);
    SNPMI_HIP(hipGetLastError());
}

void launch_lut_h2(const float* lut, uint64_t m, uint32_t* lut2, uint32_t* flag, hipStream_t st) {
    const uint64_t mpad = lut_bf3_entries(m);
    SNPMI_HIP(hipMemsetAsync(flag, 0, sizeof(uint32_t), st));
    f32w::k_lut_h2<<<(unsigned)ceil_div(mpad, 256), 256, 0, st>>>(lut, m, mpad, lut2, flag);
    SNPMI_HIP(hipGetLastError());
}

// Upper-triangle 256-iid blocks in supertile order: 16x16-block supertiles (I <= J) in
// triangular order, blocks (bi <= bj) inside each; entry = bi | bj << 16.  The dense fp16x2
// SYRK streams 4.6 B per value per panel, so the ~256 blocks in flight must share panels: in the
// plain column order they touch ~nb A panels at once, in this order 32.  xcd: workgroup w
// runs on XCD w % 8, so each supertile's blocks are dealt out of 8 4 (bi) x 8 (bj) sub-tiles
// round-robin -- measured within noise of the plain order (ubench variant 45), so the product
// uses the plain order.  Pure host function; the caller keeps the table on its device.
void supertile_order(uint64_t nb, bool xcd, std::vector<uint32_t>& tab) {
    tab.clear();
    const uint64_t ns = ceil_div(nb, 16);
    for (uint64_t J = 0; J < ns; J++)
        for (uint64_t I = 0; I <= J; I++) {
            std::vector<uint32_t> sub[8];
            for (uint64_t bj = 16 * J; bj < std::min(16 * J + 16, nb); bj++)
                for (uint64_t bi = 16 * I; bi < std::min(16 * I + 16, bj + 1); bi++)
                    sub[xcd ? ((bi - 16 * I) / 4 + 4 * ((bj - 16 * J) / 8)) : 0].push_back((uint32_t)(bi | (bj << 16)));
            size_t pos[8] = {0, 0, 0, 0, 0, 0, 0, 0}, left = 0;
            for (int x = 0; x < 8; x++) left += sub[x].size();
            for (int x = 0; left > 0; x = (x + 1) & 7)
                if (pos[x] < sub[x].size()) {
                    tab.push_back(sub[x][pos[x]++]);
                    left--;
                }
        }
}


// hook "h2": 1 = k_syrk_h2s (loader waves, default: 256.6 vs 270.0 ms per 50k x 62.5k launch in one
// process, profiles/r06g), 0 = k_syrk_h2 MODE 4 (loader in every wave)
int g_h2_kernel = 1;
int g_dense_chunk = 0;  // tuning / test hook (snpmi_set_kernel_variant "dense_chunk"): force chunk SNPs

uint64_t dense_h2_chunk_snps(uint64_t n) {
    if (g_dense_chunk > 0) return round_up((uint64_t)g_dense_chunk, 32);
    // stage-image scratch per 32-SNP stage: nb blocks x 2 steps x 2 planes x 9216 B; chunks of
    // <= 4 GiB of images (>= 1024 SNPs), and < 2^20 SNPs (k_image_h2's grid.y = 16-SNP steps)
    const uint64_t nb = ceil_div(n, 256), per32 = nb * 2 * 2 * 9216;
    uint64_t c = (4ull << 30) / per32 * 32;
    c = std::max<uint64_t>(c, 1024);
    return std::min<uint64_t>(c, (1ull << 19));
}

uint64_t dense_h2_scratch_bytes(uint64_t n, uint64_t m) {
    const uint64_t nb = ceil_div(n, 256), c = std::min(round_up(std::max<uint64_t>(m, 1), 32), dense_h2_chunk_snps(n));
    return round_up(c, 32) / 16 * nb * 2 * 9216;
}

// Dense f32 operand Z ([sid][ldz], ld = round_up(n, 256), n >= 4096) -> K tiles on the fp16 MFMA
// pipe: the range check (k_split_h2<false>, column max -> flag) runs over the whole block, then
// per SNP chunk k_image_h2 rewrites the chunk once as stage images (the exact LDS rows of the
// packed loader, 4.6 B per value) that k_syrk_h2<MODE 6> moves into LDS by DMA; k_syrk256d (the
// f32 MFMA) computes the block instead when the flag is raised.  order = supertile_order table
// on the device; img = dense_h2_scratch_bytes(n, m).
void launch_syrk_dense_h2(const float* Z, uint64_t ldz, uint64_t n, uint64_t m, uint16_t* img, uint32_t* flag,
                          const uint32_t* order, float* tiles, int accumulate, hipStream_t st) {
    const uint64_t nb = ceil_div(n, 256), g = nb * (nb + 1) / 2;
    if (g == 0) return;
    SNPMI_REQUIRE(g < (1ull << 31) && m < (1ull << 31) && nb < 65536, SNPMI_E_ARG,
                  "too many GRM blocks / SNPs for one launch");
    SNPMI_REQUIRE(ldz % 256 == 0 && ldz >= nb * 256, SNPMI_E_ARG, "dense GRM operand needs ldz = round_up(n, 256)");
    if (m == 0) {
        if (!accumulate) SNPMI_HIP(hipMemsetAsync(tiles, 0, n_tiles_upper(n) * BM * BM * sizeof(float), st));
        return;
    }
    SNPMI_HIP(hipMemsetAsync(flag, 0, sizeof(uint32_t), st));
    // Measured N=50k, 10k SNPs: 60.5 ms in one launch vs 3 x 50 ms for the VGPR-staged
    // dense loader (removed: it spilled 160 B/lane) (profiles/r01k/).  A 4-slot, 16-SNP-step
    // DMA ring (3 steps in flight) was tried: with dwordx3 pieces the LDS image came out wrong
    // (NaN), with dword pieces it was correct but 272 ms (18 DMA instructions per wave per step).
    f32w::k_split_h2<false><<<(unsigned)m, 256, 0, st>>>(Z, ldz, n, nullptr, flag);
    SNPMI_HIP(hipGetLastError());
    const uint64_t C = dense_h2_chunk_snps(n);
    for (uint64_t c0 = 0; c0 < m; c0 += C) {
        const uint64_t cnt = std::min(C, m - c0), steps = 2 * ceil_div(cnt, (uint64_t)32);
        f32w::k_image_h2<<<dim3((unsigned)nb, (unsigned)steps), 256, 0, st>>>(Z + c0 * ldz, ldz, n, cnt, (short*)img);
        SNPMI_HIP(hipGetLastError());
        f32w::k_syrk_h2<false, 6, true><<<(unsigned)g, 512, 0, st>>>((const uint8_t*)img, ldz, n, cnt, order, flag,
                                                                      tiles, accumulate || c0 > 0, 0, 1, 0, 0,
                                                                      seg_ctx());
        SNPMI_HIP(hipGetLastError());
    }
    for_segments(m, accumulate, [&](uint64_t c0, uint64_t cnt, int acc) {
        f32w::k_syrk256d<><<<(unsigned)g, 512, 0, st>>>(Z + c0 * ldz, ldz, n, cnt, tiles, acc, 0, 1, flag);
        SNPMI_HIP(hipGetLastError());
    });
}

void launch_syrk_packed_bf3(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const uint32_t* lut3,
                            float* tiles, int accumulate, hipStream_t st, const H2Lut* h2) {
    const uint64_t nb = ceil_div(n, 256), g = nb * (nb + 1) / 2;
    if (g == 0) return;
    SNPMI_REQUIRE(g < (1ull << 31), SNPMI_E_ARG, "too many GRM blocks for one launch");
    SNPMI_REQUIRE(pitch % 64 == 0 && pitch * 4 >= nb * 256, SNPMI_E_ARG, "packed pitch must cover round_up(n, 256) iids");
    if (m == 0) {
        if (!accumulate) SNPMI_HIP(hipMemsetAsync(tiles, 0, n_tiles_upper(n) * BM * BM * sizeof(float), st));
        return;
    }
    // MI355X, N=50k, 10k SNPs (tools/ubench.py syrk, 7 interleaved rounds, profiles/r01g):
    // loader interleaved between the MFMA groups (MODE 1, now 33) 302.9 TFLOP/s, + XCD remap (32)
    // 303.3, expansion after the MFMAs (30) 306.6, + XCD remap (31) 305.3 -- equal within run
    // noise; 39 (no loader, ablation) 380-382, at a 8% higher clock (PMC GRBM_GUI_ACTIVE).
    // Default MODE 2 (mid-stage barrier, next B planes prefetched into registers): 311.0 vs
    // 307.1 for MODE 1 at N=50k, 304.1 vs 300.5 at N=30k (profiles/r01i/ubench_syrk_bf3_mode2.jsonl);
    // SIMD partners staggered by one loader slot (waves 4-7 expand before group 0, runtime
    // plane index, 3 VGPRs spilled) lost: 296.8 vs 313.5 (ubench_syrk_bf3_stagger.jsonl).
    if (h2) {
        // MI355X, N=50k, 10k SNPs (tools/ubench.py syrk, profiles/r01j/ubench_syrk_h2_modes.jsonl):
        // 32-SNP stages, compiler-ordered loader (MODE 4) 577 TFLOP/s; 16-SNP stages 505-564;
        // bf16x3 300-313.  Round 6: the loader in its own waves (k_syrk_h2s) 256.6 vs 270.0 ms per
        // 50k x 62.5k launch (profiles/r06g).  Supertile block order: the ~256 blocks in flight share
        // ~32 code panels instead of ~nb (+1.7-2.4% vs the triangular order, profiles/r03crt).
        if (g_h2_kernel == 1)
            f32w::k_syrk_h2s<false><<<(unsigned)g, 768, 0, st>>>(packed, pitch, n, m, h2->lut2, h2->flag, tiles,
                                                                accumulate, 0, 1, 0, 0, seg_ctx(),
                                                                packed_block_order(ceil_div(n, 256)));
        else
            f32w::k_syrk_h2<false, 4><<<(unsigned)g, 512, 0, st>>>(packed, pitch, n, m, h2->lut2, h2->flag, tiles,
                                                                  accumulate, 0, 1, 0, 0, seg_ctx(),
                                                                  packed_block_order(ceil_div(n, 256)));
        SNPMI_HIP(hipGetLastError());
        f32w::k_syrk_bf3<false, false, 5><<<(unsigned)g, 512, 0, st>>>(packed, pitch, n, m, lut3, tiles, accumulate, 0, 1, 0, 0,
                                                                      h2->flag, seg_ctx());
        SNPMI_HIP(hipGetLastError());
        return;
    }
    f32w::k_syrk_bf3<false, false, 5><<<(unsigned)g, 512, 0, st>>>(packed, pitch, n, m, lut3, tiles, accumulate, 0, 1, 0,
                                                                  0, nullptr, seg_ctx());
    SNPMI_HIP(hipGetLastError());
}

// One column group of the default f32 SYRK: the upper-triangle 256-blocks [L0, L1) -- whole
// supertile columns, so the same blocks sit at [L0, L1) of both the supertile table (k_syrk_h2)
// and the triangular order (the bf16x3 range fallback) -- each kernel with its full-grid block
// identity (wg0 = L0), so a launch split into column groups writes the same K bit for bit as the
// whole launch.  Used to overlap the K-tile collective of finished groups with the next group's
// SYRK (api.hip grm_add_packed_reduce).
void launch_syrk_packed_h2_cols(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const uint32_t* lut3,
                                float* tiles, int accumulate, hipStream_t st, const H2Lut* h2, uint64_t L0,
                                uint64_t L1) {
    const uint64_t nb = ceil_div(n, 256), g = nb * (nb + 1) / 2;
    SNPMI_REQUIRE(h2 && L0 < L1 && L1 <= g && g < (1ull << 31), SNPMI_E_ARG, "bad SYRK column group");
    SNPMI_REQUIRE(pitch % 64 == 0 && pitch * 4 >= nb * 256, SNPMI_E_ARG, "packed pitch must cover round_up(n, 256) iids");
    if (m == 0) return;
    if (g_h2_kernel == 1)
        f32w::k_syrk_h2s<false><<<(unsigned)(L1 - L0), 768, 0, st>>>(packed, pitch, n, m, h2->lut2, h2->flag, tiles,
                                                                    accumulate, 0, 1, 0, 0, seg_ctx(),
                                                                    packed_block_order(nb), L0);
    else
        f32w::k_syrk_h2<false, 4><<<(unsigned)(L1 - L0), 512, 0, st>>>(packed, pitch, n, m, h2->lut2, h2->flag, tiles,
                                                                      accumulate, 0, 1, 0, 0, seg_ctx(),
                                                                      packed_block_order(nb), L0);
    SNPMI_HIP(hipGetLastError());
    f32w::k_syrk_bf3<false, false, 5><<<(unsigned)(L1 - L0), 512, 0, st>>>(packed, pitch, n, m, lut3, tiles, accumulate,
                                                                          0, 1, 0, 0, h2->flag, seg_ctx(), L0);
    SNPMI_HIP(hipGetLastError());
}

// split-K form for grids too small to fill the chip (N <~ 16k): `slices` partial tile sets in
// `partial` (each n_tiles_upper(n) * 128^2 floats, overwritten), then a deterministic reduce
void launch_syrk_packed_bf3_split(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const uint32_t* lut3,
                                  int slices, float* partial, float* tiles, int accumulate, hipStream_t st,
                                  const H2Lut* h2) {
    const uint64_t nb = ceil_div(n, 256), g = nb * (nb + 1) / 2;
    const uint64_t elems = n_tiles_upper(n) * BM * BM;
    const uint64_t kslice = round_up(ceil_div(m, (uint64_t)slices), (uint64_t)2 * f32w::BK);
    const unsigned S = (unsigned)ceil_div(m, kslice);
    SNPMI_REQUIRE(g < (1ull << 31) && S >= 1, SNPMI_E_ARG, "bad split");
    if (h2) {
        if (g_h2_kernel == 1)
            f32w::k_syrk_h2s<><<<dim3((unsigned)g, S), 768, 0, st>>>(packed, pitch, n, m, h2->lut2, h2->flag, partial, 0, 0,
                                                                    1, kslice, elems, seg_ctx(), packed_block_order(nb));
        else
            f32w::k_syrk_h2<><<<dim3((unsigned)g, S), 512, 0, st>>>(packed, pitch, n, m, h2->lut2, h2->flag, partial, 0, 0,
                                                                   1, kslice, elems, seg_ctx(), packed_block_order(nb));
        SNPMI_HIP(hipGetLastError());
    }
    f32w::k_syrk_bf3<false, false, 5><<<dim3((unsigned)g, S), 512, 0, st>>>(packed, pitch, n, m, lut3, partial, 0, 0, 1,
                                                                          kslice, elems, h2 ? h2->flag : nullptr,
                                                                          seg_ctx());
    SNPMI_HIP(hipGetLastError());
    launch_tile_reduce(partial, S, elems, tiles, accumulate, st);
}

void launch_syrk_packed_bf3_part(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const uint32_t* lut3,
                                 int rank, int world, float* blocks, int accumulate, hipStream_t st,
                                 const H2Lut* h2) {
    const uint64_t nloc = grm_part_blocks(n, rank, world);
    if (nloc == 0) return;
    SNPMI_REQUIRE(nloc < (1ull << 31), SNPMI_E_ARG, "too many GRM blocks for one launch");
    SNPMI_REQUIRE(pitch % 64 == 0 && pitch * 4 >= ceil_div(n, 256) * 256, SNPMI_E_ARG,
                  "packed pitch must cover round_up(n, 256) iids");
    if (m == 0) {
        if (!accumulate) SNPMI_HIP(hipMemsetAsync(blocks, 0, nloc * 256 * 256 * sizeof(float), st));
        return;
    }
    const uint32_t* tab = part_tables(ceil_div(n, 256), rank, world).tab;
    if (h2) {
        if (g_h2_kernel == 1)
            f32w::k_syrk_h2s<true><<<(unsigned)nloc, 768, 0, st>>>(packed, pitch, n, m, h2->lut2, h2->flag, blocks,
                                                                  accumulate, 0, 1, 0, 0, seg_ctx(), tab);
        else
            f32w::k_syrk_h2<true><<<(unsigned)nloc, 512, 0, st>>>(packed, pitch, n, m, h2->lut2, h2->flag, blocks,
                                                                  accumulate, 0, 1, 0, 0, seg_ctx(), tab);
        SNPMI_HIP(hipGetLastError());
    }
    f32w::k_syrk_bf3<true, false, 5><<<(unsigned)nloc, 512, 0, st>>>(packed, pitch, n, m, lut3, blocks, accumulate,
                                                                     0, 1, 0, 0, h2 ? h2->flag : nullptr, seg_ctx(),
                                                                     0, tab);
    SNPMI_HIP(hipGetLastError());
}

void launch_syrk_dense_part(const float* Z, uint64_t ldz, uint64_t n, uint64_t m, int rank, int world, void* blocks,
                            int accumulate, hipStream_t st) {
    const uint64_t nloc = grm_part_blocks(n, rank, world);
    if (nloc == 0) return;
    SNPMI_REQUIRE(nloc < (1ull << 31), SNPMI_E_ARG, "too many GRM blocks for one launch");
    SNPMI_REQUIRE(ldz % 4 == 0 && ldz >= ceil_div(n, 256) * 256, SNPMI_E_ARG, "dense GRM operand needs ldz >= round_up(n, 256)");
    if (m == 0) {
        if (!accumulate) SNPMI_HIP(hipMemsetAsync(blocks, 0, nloc * 256 * 256 * sizeof(float), st));
        return;
    }
    const uint32_t* tab = part_tables(ceil_div(n, 256), rank, world).tab;
    for_segments(m, accumulate, [&](uint64_t c0, uint64_t cnt, int acc) {
        f32w::k_syrk256d<true><<<(unsigned)nloc, 512, 0, st>>>(Z + c0 * ldz, ldz, n, cnt, (float*)blocks, acc, 0, 1,
                                                               nullptr, tab);
        SNPMI_HIP(hipGetLastError());
    });
}

void launch_syrk_dense(const void* Z, uint64_t ldz, uint64_t n, uint64_t m, int dtype, void* tiles, int accumulate,
                       hipStream_t st) {
    const uint64_t nt = n_tiles_upper(n);
    if (nt == 0) return;
    SNPMI_REQUIRE(nt < (1ull << 31), SNPMI_E_ARG, "too many GRM tiles for one launch");
    SNPMI_REQUIRE(ldz % 4 == 0 && ldz >= n_tiles_1d(n) * BM, SNPMI_E_ARG, "dense GRM operand needs padded ldz");
    if (m == 0) {
        if (!accumulate) SNPMI_HIP(hipMemsetAsync(tiles, 0, nt * BM * BM * dtype_size(dtype), st));
        return;
    }
    if (dtype == SNPMI_DT_F32) {
        const uint64_t nb = ceil_div(n, 256);
        const unsigned g = (unsigned)(nb * (nb + 1) / 2);
        const float* Zf = (const float*)Z;
        float* Tf = (float*)tiles;
        if (n >= 4096 && ldz >= nb * 256 && g_variant_syrk != 5)
            for_segments(m, accumulate, [&](uint64_t c0, uint64_t cnt, int acc) {
                f32w::k_syrk256d<><<<g, 512, 0, st>>>(Zf + c0 * ldz, ldz, n, cnt, Tf, acc);
                SNPMI_HIP(hipGetLastError());
            });
        else
            for_segments(m, accumulate, [&](uint64_t c0, uint64_t cnt, int acc) {
                f32k::k_syrk<false, 16, 4><<<(unsigned)nt, 256, 0, st>>>(Zf + c0 * ldz, ldz, cnt, nullptr, Tf, acc);
                SNPMI_HIP(hipGetLastError());
            });
    }
    else {
        f64k::k_syrk_glds<<<(unsigned)nt, 256, 0, st>>>((const double*)Z, ldz, m, (double*)tiles, accumulate);
    }
    SNPMI_HIP(hipGetLastError());
}

}  // namespace snpmi
