// Internal declarations shared by the libsnpmi translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/snpmi.h"

namespace snpmi {

// ------------------------------------------------------------------ errors
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

#define SNPMI_HIP(expr)                                                                     \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            throw ::snpmi::Error(SNPMI_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define SNPMI_REQUIRE(cond, code, msg)                 \
    do {                                               \
        if (!(cond)) throw ::snpmi::Error(code, msg);  \
    } while (0)

// Run `body` translating exceptions into status codes + thread-local messages.
template <class F>
int guarded(F&& body) {
    try {
        body();
        return SNPMI_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_last_error("host allocation failed");
        return SNPMI_E_NOMEM;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return SNPMI_E_ARG;
    }
}

// ------------------------------------------------------------------ wave-uniform values
// A 64-bit value (an address) made wave-uniform, i.e. moved to SGPRs.  __builtin_amdgcn_readfirstlane
// takes and returns a 32-bit *int*: each half is widened through uint32_t here, because a cast of
// the int straight to uint64_t sign-extends a low word whose bit 31 is set -- the cause of round 5's
// illegal memory access (a SegFlush slot address, profiles/r05sub/README.md).  Every 64-bit value
// built from readfirstlane goes through this helper (tests/test_sgpr_widening.py checks the sources).
__device__ __forceinline__ uint64_t sgpr_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | (uint64_t)lo;
}
__device__ __forceinline__ void* sgpr_ptr(const void* p) {
    return reinterpret_cast<void*>(sgpr_u64(reinterpret_cast<uint64_t>(p)));
}

// ------------------------------------------------------------------ geometry
constexpr int kTile = 128;                      // GRM tile edge (iids)
inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
inline uint64_t round_up(uint64_t a, uint64_t b) { return ceil_div(a, b) * b; }
inline uint64_t packed_pitch(uint64_t n_iid) { return round_up(ceil_div(n_iid, 4), 64); }
inline uint64_t n_tiles_1d(uint64_t n) { return ceil_div(n, kTile); }
inline uint64_t n_tiles_upper(uint64_t n) { uint64_t t = n_tiles_1d(n); return t * (t + 1) / 2; }
inline size_t dtype_size(int dt) { return dt == SNPMI_DT_F64 ? 8 : dt == SNPMI_DT_F32 ? 4 : 1; }

// ------------------------------------------------------------------ per-device state
// host -> device staging of file chunks: a ring of kPieces pinned pieces of <= kPieceBytes
constexpr int kPieces = 4;
constexpr uint64_t kPieceBytes = 32ull << 20;

struct Device {
    int id = -1;
    hipStream_t stream = nullptr;  // compute: every kernel
    hipStream_t copy = nullptr;    // DMA: host<->device copies of streamed chunks, overlapping compute
    hipStream_t aux = nullptr;     // second compute stream (snpmi_set_stream 2): e.g. block k+1's stats
                                   // beside block k's write-bound decode
    int cu_count = 0;
    // grow-only scratch slots
    enum Slot { S_PACKED, S_PACKED2, S_IDX, S_IDX2, S_LUT, S_STATS, S_OUT, S_TILES, S_K, S_DENSE,
                S_DENSE2, S_RED, S_SESSION, S_PACKED_B, S_ZBLK, S_IDX32, S_LUT3, S_H2, S_OUT_B, S_STATS_B,
                S_WIN, S_DPACK, S_DLUT, S_CRTREC, S_SEG, S_STDFLAG, S_DIAG, S_NUM };
    void* buf[S_NUM] = {};
    // chunk pipeline events (slot = chunk parity), all on-device ordering, no host spin:
    hipEvent_t staged[2] = {};    // copy stream: H2D of pinned slot done (host may refill it)
    hipEvent_t consumed[2] = {};  // compute stream: kernels done reading device packed slot
    hipEvent_t produced[2] = {};  // compute stream: output slot written (its D2H may start)
    hipEvent_t bounce[2] = {};    // copy stream: D2H into pinned bounce slot done
    hipEvent_t fence = nullptr;   // compute stream: "all work so far", for a copy to wait on
    hipEvent_t piece[kPieces] = {};  // copy stream: H2D from pinned piece q done (host may refill it)
    uint64_t piece_next = 0;         // next piece of the ring (stage_chunk)
    size_t cap[S_NUM] = {};
    // upper-triangle 256-iid block order tables of the dense fp16x2 SYRK, built once per
    // (nb, xcd) and kept on this device (guarded by the device's own mutex)
    uint32_t* order_tab[2] = {};
    uint64_t order_nb[2] = {};
    // the cfg5 part layout (part_layout table + diagonal slots), per (nb, rank, world)
    void* part_tab = nullptr;
    uint64_t part_key[3] = {};
    void* get(Slot s, size_t bytes);
    void release();
};

Device& device();                 // current device of this thread (lazily initialised)
hipStream_t stream();  // the calling thread's current stream (compute, or aux after snpmi_set_stream(2))

// pinned host staging buffers (grow-only, per thread)
void* pinned(int slot, size_t bytes);
void release_pinned();

// ------------------------------------------------------------------ kernel launchers (kernels.hip)
extern int g_variant_decode;
extern int g_variant_std;
extern int g_variant_extract;
extern int g_variant_syrk;
extern int g_dense_chunk;
extern int g_h2_kernel;  // packed fp16x2 SYRK form (hook "h2"): 0 = k_syrk_h2, 1 = warp-specialised k_syrk_h2s
// f32 GRM accumulation segments (syrk.hip SegFlush): every `snps` SNPs a workgroup adds its MFMA
// accumulators into a private scratch slot (register-native layout, 256 KiB: 8 waves x 32 x 64
// lanes x 16 B) and restarts them, so no f32 chain is longer than `snps`; the slot is taken from a
// pool of `nslots` by atomic compare-and-swap on `flags` (0 = free) when the workgroup starts and
// released when it ends.  snps = 0: one chain per launch.  Tuning hook "seg" (g_seg_snps).
extern int g_seg_snps;
struct SegCtx {
    uint32_t snps = 0;
    uint32_t nslots = 0;
    uint32_t* flags = nullptr;
    float* scratch = nullptr;
};
constexpr uint32_t kSegSlots = 1024;                 // > the resident workgroups of one launch (<= 256 x 2)
constexpr uint64_t kSegSlotFloats = 8 * 32 * 64 * 4;  // per workgroup
SegCtx seg_ctx();                                     // api.hip: the current device's pool (lazily allocated)
// api.hip: device table of supertile_order(nb, false) for the current device (cached per nb): the
// block order of the packed fp16x2 SYRK
const uint32_t* packed_block_order(uint64_t nb);
// cfg5 K partition (syrk.hip part_layout): part `rank` of `world` owns whole S x S-block
// supertiles (S = part_unit) dealt round-robin; its blocks are stored densely in the order of its
// layout table (entry bi | bj << 16 per local slot).  part_tables: that table and the local slot
// of each diagonal block (bi = bj = J; -1 if another part owns it) on the current device (cached)
uint64_t part_unit(uint64_t nb, int world);
void part_layout(uint64_t nb, int rank, int world, std::vector<uint32_t>& tab);
struct PartTables {
    const uint32_t* tab = nullptr;
    const int32_t* dslot = nullptr;
    const int32_t* lslot = nullptr;  // per upper-triangle block L = J(J+1)/2 + I: local slot or -1
};
PartTables part_tables(uint64_t nb, int rank, int world);
void launch_snp_stats(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, int count_a1,
                      int std_kind, double a, double b, int use_stats, int dtype, void* stats, void* lut,
                      hipStream_t st);
void launch_decode(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, const void* lut,
                   int dtype, int order_c, void* out, uint64_t ld, hipStream_t st);
void launch_decode_std_fused(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, int count_a1,
                             int std_kind, double a, double b, int use_stats, void* stats, void* lut, void* out,
                             uint64_t ld, hipStream_t st);
// iid gather: plan = repack_plan_entries(n_out) u32 and win = repack_win_entries(n_out) u32 of
// scratch, built once per index list (launch_repack_plan, which may synchronise the stream once)
struct RepackPlan {
    const uint32_t* plan = nullptr;  // nullptr: global-gather fallback (reads idx)
    const uint32_t* win = nullptr;   // per-chunk source windows (windowed kernel) or nullptr
    int K = 1;                       // columns per workgroup
    uint64_t zq = 0;                 // u32x4 per staged column (window or whole column)
    uint64_t nchunks = 1;
    uint64_t chunk_words = 0;        // output words per windowed workgroup
    bool lanes = false;              // u16 lane-interleaved plan of k_repack_win16
};
uint64_t repack_plan_entries(uint64_t n_out);
uint64_t repack_win_entries(uint64_t n_out);
RepackPlan launch_repack_plan(const uint64_t* idx, uint64_t n_out, uint64_t n_src, uint32_t* plan, uint32_t* win,
                              hipStream_t st);
void launch_repack(const uint8_t* src, uint64_t src_pitch, uint64_t n_src, const uint64_t* idx, const RepackPlan& plan,
                   uint64_t n_out, uint64_t n_sid, uint8_t* dst, uint64_t dst_pitch, hipStream_t st);
// dense f32 columns with <= 4 distinct values -> 2-bit codes + f32 LUT [m][4] (exact); *flag = 1
// if any column has more (then packed/lut are incomplete)
void launch_dense_codes(const float* Z, uint64_t ldz, uint64_t n, uint64_t m, uint8_t* packed, uint64_t pitch,
                        float* lut, unsigned int* flag, hipStream_t st);
void launch_dense_standardize(void* val, uint64_t rows, uint64_t cols, uint64_t ld, int order_c, int dtype,
                              int std_kind, double a, double b, int use_stats, void* stats, hipStream_t st);
void launch_subset(const void* in, int in_dt, uint64_t rows, uint64_t cols, uint64_t k, int in_order_c,
                   const uint64_t* ri, uint64_t nr, const uint64_t* ci, uint64_t nc, int out_order_c,
                   void* out, int out_dt, hipStream_t st);
void launch_transpose_to_f(const void* in, uint64_t rows, uint64_t cols, int dtype, void* out, uint64_t ld,
                           hipStream_t st);
// rows [r0, r0+nr) of the full K (identity columns), row-major, LDS-transposed mirror half
void launch_grm_extract_rows(const void* tiles, uint64_t n, int dtype, uint64_t r0, uint64_t nr, double scale,
                             void* out, hipStream_t st);
void launch_grm_extract(const void* tiles, uint64_t n, int dtype, const uint64_t* ri, uint64_t nr,
                        const uint64_t* ci, uint64_t nc, int order_c, double scale, void* out, hipStream_t st);
void launch_grm_trace(const void* tiles, uint64_t n, int dtype, double* trace_dev, hipStream_t st);
// cfg5 part blocks -> K[ri, ci] restricted to this part's blocks (0 elsewhere; the parts' outputs
// sum to the sub-matrix) / the part's share of trace(K) (kernels.hip k_part_*)
void launch_part_extract(const void* blocks, const int32_t* lslot, int dtype, const uint64_t* ri, uint64_t nr,
                         const uint64_t* ci, uint64_t nc, int order_c, double scale, void* out, hipStream_t st);
void launch_part_trace(const void* blocks, const int32_t* dslot, uint64_t n, int dtype, double* trace_dev,
                       hipStream_t st);
// exact f32 GRM diagonal around one f32 SYRK launch (kernels.hip k_diag_*): begin saves the current
// diagonal as f64 (0 unless accumulating), end adds sum_s lut_s[code]^2 in f64 and writes it back
// rounded once.  dslot == nullptr: upper-triangle tiles; else the blocks of one cfg5 part
// (PartTables::dslot: local slot of each diagonal block, -1 if not owned).
extern int g_diag_exact;  // hook "diag": 1 (default) = on, 0 = the SYRK's own diagonal
void launch_diag_begin(const float* K, uint64_t n, const int32_t* dslot, int accumulate, double* diag, hipStream_t st);
void launch_diag_end(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const float* lut, float* K,
                     const int32_t* dslot, double* diag, hipStream_t st);
// diag: diag_scratch_bytes(n, m) of device scratch (n f64 + per-slice partial rows, folded in a
// fixed order so the diagonal is the same bits on every run)
uint64_t diag_scratch_bytes(uint64_t n, uint64_t m);
// launch_diag_end in two steps: the f64 squares of all iids, then the write-back of iids [i0, i1)
void launch_diag_sq(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const float* lut, double* diag,
                    hipStream_t st);
void launch_diag_patch(float* K, uint64_t n, uint64_t i0, uint64_t i1, const int32_t* dslot, const double* diag,
                       hipStream_t st);
// rccl.hip: in-place sum over the ranks of a device range on stream st (root < 0: all-reduce)
void rccl_sum_on(void* buf, uint64_t count, int dtype, int root, hipStream_t st);
bool rccl_ready();
void launch_dense_scale(void* p, uint64_t count, int dtype, double scale, hipStream_t st);
void launch_sumsq(const void* p, uint64_t count, int dtype, double* out_dev, hipStream_t st);
void launch_dense_trace(const void* K, uint64_t n, int dtype, double* trace_dev, hipStream_t st);
void launch_copy16(const void* src, void* dst, uint64_t bytes, hipStream_t st);  // 16-B aligned
void launch_synth(uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t sid0, uint64_t n_sid, uint64_t seed,
                  double miss_rate, const double* maf_x_dev, const double* maf_cdf_dev, int n_pts, hipStream_t st);
void launch_encode(const void* val, int dtype, int order_c, uint64_t ld, uint64_t n, uint64_t m, int count_a1,
                   uint8_t* packed, uint64_t pitch, unsigned int* bad_dev, hipStream_t st);  // encode.hip

// ------------------------------------------------------------------ MFMA SYRK (syrk.hip)
void launch_syrk_packed(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, const void* lut,
                        int dtype, void* tiles, int accumulate, hipStream_t st);
uint64_t grm_part_blocks(uint64_t n, int rank, int world);
void launch_syrk_packed_part(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const void* lut,
                             int rank, int world, void* blocks, int accumulate, hipStream_t st);
void launch_syrk_dense_part(const float* Z, uint64_t ldz, uint64_t n, uint64_t m, int rank, int world, void* blocks,
                            int accumulate, hipStream_t st);
void launch_syrk_dense(const void* Z, uint64_t ldz, uint64_t n_iid, uint64_t n_sid, int dtype, void* tiles,
                       int accumulate, hipStream_t st);
// f32 GRM on the bf16 MFMA pipe (bf16x3 split, f32 accuracy); lut3 = scratch of 32 B per SNP
uint64_t lut_bf3_entries(uint64_t m);  // 8 u32 each, zero-padded to a multiple of the SYRK stage
void launch_lut_bf3(const float* lut, uint64_t m, uint32_t* lut3, hipStream_t st);
// fp16x2 split (3 MFMA products, f32 accuracy while every SNP's LUT fits fp16's range): lut2 =
// 16 B per SNP (lut_bf3_entries), flag = 1 u32 raised by k_lut_h2 when a SNP does not fit; with
// h2 given, the SYRK launchers run k_syrk_h2 and the bf16x3 kernel gated on the flag.
struct H2Lut {
    const uint32_t* lut2;
    const uint32_t* flag;
};
void launch_lut_h2(const float* lut, uint64_t m, uint32_t* lut2, uint32_t* flag, hipStream_t st);
// dense f32 operand (ld = round_up(n, 256), n >= 4096) on the fp16 MFMA pipe: range check, then
// per SNP chunk (dense_h2_chunk_snps) LDS stage images (img: dense_h2_scratch_bytes) + the
// fp16x2 SYRK in supertile block order (order: device table of supertile_order), the f32-MFMA
// k_syrk256d gated on the range flag
void supertile_order(uint64_t nb, bool xcd, std::vector<uint32_t>& tab);
uint64_t dense_h2_chunk_snps(uint64_t n);
uint64_t dense_h2_scratch_bytes(uint64_t n, uint64_t m);
void launch_syrk_dense_h2(const float* Z, uint64_t ldz, uint64_t n, uint64_t m, uint16_t* img, uint32_t* flag,
                          const uint32_t* order, float* tiles, int accumulate, hipStream_t st);
void launch_syrk_packed_bf3(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const uint32_t* lut3,
                            float* tiles, int accumulate, hipStream_t st, const H2Lut* h2 = nullptr);
void launch_syrk_packed_h2_cols(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const uint32_t* lut3,
                                float* tiles, int accumulate, hipStream_t st, const H2Lut* h2, uint64_t L0,
                                uint64_t L1);
void launch_syrk_packed_bf3_split(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const uint32_t* lut3,
                                  int slices, float* partial, float* tiles, int accumulate, hipStream_t st,
                                  const H2Lut* h2 = nullptr);
void launch_tile_reduce(const float* partial, unsigned slices, uint64_t elems, float* tiles, int accumulate,
                        hipStream_t st);
// f64 GRM of packed SNPs on the int8 MFMA pipe (syrk_crt.hip): residues modulo crt_moduli()
// moduli, CRT back to f64.  ws_lut = crt_lut_bytes(m, n) of scratch (its first ints: block
// exponent, the non-finite flag, the moduli count R this block needs), res = residue scratch
// (>= crt_moduli() * 64 KiB; more = fewer launches); m <= crt_max_snps(); rec (device, may be
// NULL): rec[0] += R, rec[1] += 1 per launch
int crt_moduli();
extern int g_crt_kernel;  // residue SYRK form (hook "crt"): 0 = k_syrk_i8r, 1 = warp-specialised k_syrk_i8w
extern int g_crt_block;   // hook "crt_block": 1 = moduli per 256-block (default), 0 = launch-wide R
uint64_t crt_max_snps();
uint64_t crt_lut_bytes(uint64_t m, uint64_t n);
int crt_fraction_bits(uint64_t m);
// block columns [c0, c1) of each residue chunk of the overlapped form (after_chunk below)
std::vector<std::pair<uint64_t, uint64_t>> crt_column_chunks(uint64_t n, uint64_t res_bytes);
// before_chunks (optional) is enqueued after the per-launch bound/moduli kernels and before the
// first residue chunk; after_chunk(c0, c1) (optional) after the chunk whose blocks are the whole
// block columns [c0, c1) (chunks are then cut at column boundaries, so each one's tiles are one
// contiguous range): the overlapped collective of api.hip grm_add_packed_reduce.
void launch_syrk_packed_crt(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const double* lut,
                            double* tiles, int accumulate, void* ws_lut, uint8_t* res, uint64_t res_bytes,
                            unsigned long long* rec, hipStream_t st,
                            const std::function<void()>* before_chunks = nullptr,
                            const std::function<void(uint64_t, uint64_t)>* after_chunk = nullptr,
                            const uint32_t* part_tab = nullptr, uint64_t part_blocks = 0);
// part_tab (cfg5): tiles = the part's part_blocks dense 256x256 f64 blocks in the order of its
// layout table (PartTables::tab); no after_chunk.
// the f64-MFMA packed SYRK, run only when the device word *gate is non-zero (the CRT path's flag);
// with part_tab: into the part's dense blocks (all four 128-quadrants of each)
void launch_syrk_packed_f64_gated(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const double* lut,
                                  double* tiles, int accumulate, const int* gate, hipStream_t st,
                                  const uint32_t* part_tab = nullptr, uint64_t part_blocks = 0);
void launch_syrk_packed_bf3_part(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const uint32_t* lut3,
                                 int rank, int world, float* blocks, int accumulate, hipStream_t st,
                                 const H2Lut* h2 = nullptr);

}  // namespace snpmi
