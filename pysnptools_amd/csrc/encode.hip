// BED encoder: genotype values -> SNP-major 2-bit codes.
//
// Replaces bed-reader's to_bed body encoder (reference call site snpreader/bed.py:300-314).
// Inverse of the decode LUT: count_A1=False 0->00, 1->10, 2->11, missing->01;
// count_A1=True 0->11, 1->10, 2->00, missing->01.  Missing is NaN for f32/f64 and -127 for
// int8; any other value is counted in *bad (the caller raises ValueError).  Pad codes of
// the last byte (iids >= n) are 00, as in every .bed the reference writes.
//
// Both kernels are HBM-read bound (4-8 B in per 2 bits out):
//   k_encode_f  (F order, column-contiguous input): one wave per (SNP, 1024-iid chunk); lane l
//               reads 16 consecutive values (64 B f32) and writes ONE 32-bit word, so each
//               wave writes 256 contiguous bytes.  Requires ld % 16 == 0 (16-B aligned rows).
//   k_encode_c  (C order, iid-major input): one wave per (64 SNPs x 256 iids) tile; lane = SNP,
//               each load instruction reads one row segment of 64 consecutive values, and each
//               lane ends with 64 packed bytes of its SNP (four 16-B stores).
#include <algorithm>

#include "snpmi_internal.hpp"

namespace snpmi {
namespace {

constexpr int kBlock = 256;
constexpr int kWave = 64;

// value -> 2-bit code (bad values -> 01 and flagged)
template <typename T>
__device__ __forceinline__ uint32_t code_of(T v, uint32_t c0, uint32_t c2, uint32_t& bad) {
    if (v != v) return 1u;
    if (v == (T)0) return c0;
    if (v == (T)1) return 2u;
    if (v == (T)2) return c2;
    bad = 1u;
    return 1u;
}
template <>
__device__ __forceinline__ uint32_t code_of<int8_t>(int8_t v, uint32_t c0, uint32_t c2, uint32_t& bad) {
    if (v == -127) return 1u;
    if (v == 0) return c0;
    if (v == 1) return 2u;
    if (v == 2) return c2;
    bad = 1u;
    return 1u;
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef double f64x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// 16 consecutive values as one 16-B-aligned vector group (streamed once: non-temporal)
template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
    __device__ static void load(const float* p, float (&v)[16]) {
        const f32x4_t* q = reinterpret_cast<const f32x4_t*>(p);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            f32x4_t x = __builtin_nontemporal_load(q + k);
            v[4 * k] = x.x, v[4 * k + 1] = x.y, v[4 * k + 2] = x.z, v[4 * k + 3] = x.w;
        }
    }
};
template <>
struct Vec16<double> {
    __device__ static void load(const double* p, double (&v)[16]) {
        const f64x2_t* q = reinterpret_cast<const f64x2_t*>(p);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            f64x2_t x = __builtin_nontemporal_load(q + k);
            v[2 * k] = x.x, v[2 * k + 1] = x.y;
        }
    }
};
template <>
struct Vec16<int8_t> {
    __device__ static void load(const int8_t* p, int8_t (&v)[16]) {
        u32x4_t x = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = (int8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
};

template <typename T>
__global__ __launch_bounds__(kBlock) void k_encode_f(const T* __restrict__ val, uint64_t ld, uint64_t n,
                                                      uint64_t m, uint32_t c0, uint32_t c2,
                                                      uint8_t* __restrict__ packed, uint64_t pitch,
                                                      unsigned int* __restrict__ bad_count) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t chunks = (n + 1023) / 1024;
    const uint64_t items = chunks * m;
    const uint64_t wave0 = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
    const uint64_t nwaves = (uint64_t)gridDim.x * kBlock / kWave;
    uint32_t bad = 0;
    for (uint64_t it = wave0; it < items; it += nwaves) {
        const uint64_t j = it / chunks, c = it - j * chunks;
        const uint64_t i0 = c * 1024 + 16 * (uint64_t)lane;
        const uint64_t byte = i0 >> 2;
        if (byte >= pitch) continue;
        uint32_t w = 0;
        if (i0 + 16 <= n) {
            T v[16];
            Vec16<T>::load(val + j * ld + i0, v);
#pragma unroll
            for (int k = 0; k < 16; k++) w |= code_of<T>(v[k], c0, c2, bad) << (2 * k);
        } else {
            for (int k = 0; k < 16; k++)
                if (i0 + k < n) w |= code_of<T>(val[j * ld + i0 + k], c0, c2, bad) << (2 * k);
        }
        *reinterpret_cast<uint32_t*>(packed + j * pitch + byte) = w;
    }
    if (bad) atomicAdd(bad_count, 1u);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_encode_c(const T* __restrict__ val, uint64_t ld, uint64_t n,
                                                      uint64_t m, uint32_t c0, uint32_t c2,
                                                      uint8_t* __restrict__ packed, uint64_t pitch,
                                                      unsigned int* __restrict__ bad_count) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t tj = (m + 63) / 64, ti = (n + 255) / 256;
    const uint64_t items = tj * ti;
    const uint64_t wave0 = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
    const uint64_t nwaves = (uint64_t)gridDim.x * kBlock / kWave;
    uint32_t bad = 0;
    for (uint64_t it = wave0; it < items; it += nwaves) {
        const uint64_t bi = it / tj, bj = it - bi * tj;  // consecutive waves: neighbouring SNP tiles
        const uint64_t j = bj * 64 + lane, i0 = bi * 256;
        const bool live = j < m;
        uint32_t w[16];
        if (i0 + 256 <= n) {
#pragma unroll
            for (int q = 0; q < 16; q++) {
                uint32_t x = 0;
#pragma unroll
                for (int k = 0; k < 16; k++)
                    if (live) x |= code_of<T>(val[(i0 + 16 * q + k) * ld + j], c0, c2, bad) << (2 * k);
                w[q] = x;
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; q++) {
                uint32_t x = 0;
                for (int k = 0; k < 16; k++) {
                    const uint64_t i = i0 + 16 * q + k;
                    if (live && i < n) x |= code_of<T>(val[i * ld + j], c0, c2, bad) << (2 * k);
                }
                w[q] = x;
            }
        }
        if (live) {
            // i0/4 and pitch are multiples of 64, so the 64 bytes stay inside the column's pitch
            uint4* dst = reinterpret_cast<uint4*>(packed + j * pitch + (i0 >> 2));
#pragma unroll
            for (int q = 0; q < 4; q++) dst[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
        }
    }
    if (bad) atomicAdd(bad_count, 1u);
}

inline unsigned grid_cap(uint64_t waves, unsigned cap) {
    uint64_t g = (waves + kBlock / kWave - 1) / (kBlock / kWave);
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

}  // namespace

void launch_encode(const void* val, int dtype, int order_c, uint64_t ld, uint64_t n, uint64_t m, int count_a1,
                   uint8_t* packed, uint64_t pitch, unsigned int* bad_dev, hipStream_t st) {
    if (n == 0 || m == 0) return;
    const uint32_t c0 = count_a1 ? 3u : 0u, c2 = count_a1 ? 0u : 3u;
    if (!order_c) {
        const unsigned g = grid_cap(((n + 1023) / 1024) * m, 256 * 16 * 4);
        if (dtype == SNPMI_DT_F32)
            k_encode_f<float><<<g, kBlock, 0, st>>>((const float*)val, ld, n, m, c0, c2, packed, pitch, bad_dev);
        else if (dtype == SNPMI_DT_F64)
            k_encode_f<double><<<g, kBlock, 0, st>>>((const double*)val, ld, n, m, c0, c2, packed, pitch, bad_dev);
        else
            k_encode_f<int8_t><<<g, kBlock, 0, st>>>((const int8_t*)val, ld, n, m, c0, c2, packed, pitch, bad_dev);
    } else {
        const unsigned g = grid_cap(((m + 63) / 64) * ((n + 255) / 256), 256 * 16 * 4);
        if (dtype == SNPMI_DT_F32)
            k_encode_c<float><<<g, kBlock, 0, st>>>((const float*)val, ld, n, m, c0, c2, packed, pitch, bad_dev);
        else if (dtype == SNPMI_DT_F64)
            k_encode_c<double><<<g, kBlock, 0, st>>>((const double*)val, ld, n, m, c0, c2, packed, pitch, bad_dev);
        else
            k_encode_c<int8_t><<<g, kBlock, 0, st>>>((const int8_t*)val, ld, n, m, c0, c2, packed, pitch, bad_dev);
    }
    SNPMI_HIP(hipGetLastError());
}

}  // namespace snpmi
