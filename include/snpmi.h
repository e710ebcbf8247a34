/*
 * snpmi.h -- C ABI of libsnpmi.so, the MI355X-native (gfx950, HIP) implementation of
 * PySnpTools' BED decode -> slice -> standardize -> SnpKernel GRM path.
 *
 * The reference crosses into native code through the Rust/PyO3 module `bed_reader`
 * and NumPy BLAS; every host entry point below replaces one of those call sites
 * (paths relative to /root/reference/pysnptools):
 *
 *   snpmi_bed_check              bed_reader.open_bed(...) format check    snpreader/bed.py:137-145
 *   snpmi_bed_read_{f32,f64,i8}  open_bed(...).read(index,order,dtype)     snpreader/bed.py:337-343
 *   snpmi_standardize_{f32,f64}  bed_reader.standardize_f32/f64(...)       standardizer/standardizer.py:114,120
 *   snpmi_subset_*               bed_reader.subset_f64_f64/f32_f64/f32_f32 util/__init__.py:341-375
 *   snpmi_bed_read_standardize_* Bed.read() + SnpData.standardize() fused  snpreader/snpreader.py:606-621
 *   snpmi_grm_bed_{f32,f64}      SnpReader._read_kernel block loop         snpreader/snpreader.py:623-668
 *   snpmi_grm_dense_{f32,f64}    SnpData._read_kernel (val.dot(val.T))     snpreader/snpdata.py:190-214
 *   snpmi_diag_k_to_n_{f32,f64}  DiagKtoN._standardize_kernel              standardizer/diag_K_to_N.py:54-64
 *
 * Conventions (mirroring bed-reader's):
 *   - The caller owns every host buffer; outputs are written in place.  Index arrays are
 *     NumPy `uintp` (== uint64_t on LP64).  A NULL index array means "all, in order".
 *   - `order_c` = 1 for C order (row-major, SNP fastest), 0 for F order (iid fastest).
 *   - `stats` arrays are C-order [n_sid][2] = (mean, std) in the value dtype.
 *   - Missing values decode to NaN (float) or -127 (int8).  count_a1 selects the A1 LUT
 *     {2,NaN,1,0} instead of {0,NaN,1,2}.
 *   - Every function returns 0 on success or one of the SNPMI_E_* codes; the message of
 *     the calling thread's last failure is available from snpmi_last_error().
 *   - `num_threads` sizes the host-side gather pool only; all arithmetic runs on the GPU.
 *     There is no CPU fallback: without a HIP device every compute entry point fails
 *     with SNPMI_E_HIP.
 *   - K outputs are n_out x n_out, symmetric; order_c selects the layout of non-square
 *     subsets produced by snpmi_kernel_subset_*.
 *   - Value and K buffers (`out`, `val`, `K_out`, `K`, subset in/out) may be HOST memory or
 *     DEVICE memory of the current device (snpmi_dev_alloc / hipMalloc; HIP unified
 *     addressing tells them apart).  Device buffers are computed on in place or written
 *     directly, with no host staging: this is the array-module seam of the reference
 *     (util/__init__.py:652-730, ARRAY_MODULE=cupy keeps SnpData/KernelData values on the GPU),
 *     used by pysnptools_amd.hbm.  Stats and index arrays are always host memory.  A device
 *     buffer of another device fails with SNPMI_E_ARG.
 *
 * Deliberate semantics where the reference's two paths differ (the reference calls bed-reader's
 * native standardize by default, standardizer.py:114,120, but none of its fixtures pins the
 * native behaviour below; these follow the reference's Python path, standardizer.py:136-211,
 * which its goldens do pin -- "parity unpinned" against bed-reader itself):
 *   - a SNP with no observed value (n = 0) trains NaN stats and standardizes to an all-zero
 *     column; bed-reader's native code would raise NoIndividuals.
 *   - Beta with a trained/given mean outside [0, 2]: maf = mean/2 (folded to <= 0.5) leaves
 *     [0, 1] and the weight is 0 -- scipy.stats.beta.pdf's value there -- so the column
 *     standardizes to zeros; bed-reader would raise IllegalSnpMean.
 *   - f32 stats and LUTs are computed in f64 and rounded once (the one-pass formula in f32
 *     arithmetic misses the reference Python path by 1.47e-5 on N300); bed-reader's f32 native
 *     path has no fixture.  The claim is "matches the reference Python path", not bed-reader.
 */
#ifndef SNPMI_H
#define SNPMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SNPMI_OK 0
#define SNPMI_E_ARG 1     /* bad argument (shape, dtype, order, NULL pointer)        */
#define SNPMI_E_INDEX 2   /* iid/sid index out of range                              */
#define SNPMI_E_FORMAT 3  /* not a SNP-major .bed file, or size mismatch             */
#define SNPMI_E_IO 4      /* open/read/mmap failure                                  */
#define SNPMI_E_HIP 5     /* HIP runtime error (includes "no device")                */
#define SNPMI_E_NOMEM 6   /* device or pinned allocation failed                      */
#define SNPMI_E_RCCL 7    /* RCCL error                                              */

/* standardizer kinds (standardizer/{identity,unit,beta}.py) */
#define SNPMI_STD_NONE 0  /* raw values (Identity)                                   */
#define SNPMI_STD_UNIT 1  /* (x - mean) / std, NaN -> 0                              */
#define SNPMI_STD_BETA 2  /* (x - mean) * BetaPDF(maf; a, b), NaN -> 0               */

/* dtypes for the device-resident API */
#define SNPMI_DT_F32 0
#define SNPMI_DT_F64 1
#define SNPMI_DT_I8 2

/* ---------------------------------------------------------------- runtime */
const char* snpmi_last_error(void);
int snpmi_version(void);
int snpmi_device_count(int* count);
int snpmi_set_device(int device);            /* device used by later calls of this thread */
int snpmi_get_device(int* device);
int snpmi_release_cache(void);               /* free cached device/pinned scratch          */
int snpmi_device_info(int device, char* name, size_t name_len, uint64_t* total_mem, int* cu_count);
/* the box a measurement ran on: 16-byte device UUID, PCI domain / bus / device, max SCLK (kHz) */
int snpmi_device_ids(int dev, uint8_t* uuid16, int* pci, int* clock_khz);
/* select a kernel variant by name; 0 = default.  Public switches: "f64" (0 = f64 GRMs as int8
 * residues + CRT, 1 = on the f64 MFMA), "seg" (SNPs per f32 GRM accumulation chain, default 12288,
 * 0 = one chain per launch).  The rest ("decode", "syrk", "part_order" (1 = the cfg5 part
 * kernel in triangular block order), ...) are A/B hooks for benches. */
int snpmi_set_kernel_variant(const char* kernel, int variant);
int snpmi_get_kernel_variant(const char* kernel, int* variant);  /* current value of a hook above */

/* ---------------------------------------------------------------- BED reading (bed-reader read_*) */
int snpmi_bed_check(const char* path, uint64_t n_iid, uint64_t n_sid);
int snpmi_bed_read_f32(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                       const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                       uint64_t n_out_sid, int order_c, float* out, int num_threads);
int snpmi_bed_read_f64(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                       const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                       uint64_t n_out_sid, int order_c, double* out, int num_threads);
int snpmi_bed_read_i8(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                      const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                      uint64_t n_out_sid, int order_c, int8_t* out, int num_threads);

/* ---------------------------------------------------------------- .fam/.bim metadata (host, threaded)
 * Replaces the text parsing behind bed-reader open_bed's properties (fid/iid/sid/chromosome/
 * cm_position/bp_position; snpreader/bed.py:137-194).  Lines are split on whitespace, blank
 * lines skipped.  scan: number of rows and the widest field of columns 0..n_cols-1 (every line
 * must have >= min_fields fields, else SNPMI_E_FORMAT).  strings: column `col` as fixed-width
 * NUL-padded rows of `width` bytes.  f64: column `col` parsed as a float (SNPMI_E_FORMAT if
 * it is not one).  No GPU is needed. */
int snpmi_text_scan(const char* path, int min_fields, int n_cols, uint64_t* n_rows, uint64_t* widths,
                    int num_threads);
int snpmi_text_strings(const char* path, int col, uint64_t n_rows, uint64_t width, char* out, int num_threads);
int snpmi_text_f64(const char* path, int col, uint64_t n_rows, double* out, int num_threads);

/* ---------------------------------------------------------------- BED writing (bed-reader to_bed body)
 * Replaces the genotype half of `to_bed(filepath, val, properties, count_A1, ...)`
 * (snpreader/bed.py:300-314); the .fam/.bim text is written by the host.  val is
 * n_iid x n_sid (F or C order); values must be 0, 1, 2 or missing (NaN; -127 for int8),
 * anything else -> SNPMI_E_ARG (ValueError) and no file is left behind. */
int snpmi_bed_write_f32(const char* path, const float* val, uint64_t n_iid, uint64_t n_sid, int order_c,
                        int count_a1, int num_threads);
int snpmi_bed_write_f64(const char* path, const double* val, uint64_t n_iid, uint64_t n_sid, int order_c,
                        int count_a1, int num_threads);
int snpmi_bed_write_i8(const char* path, const int8_t* val, uint64_t n_iid, uint64_t n_sid, int order_c,
                       int count_a1, int num_threads);

/* ---------------------------------------------------------------- standardize (bed-reader standardize_*) */
int snpmi_standardize_f32(float* val, uint64_t rows, uint64_t cols, int order_c, int is_beta,
                          double a, double b, int apply_in_place, int use_stats, float* stats,
                          int num_threads);
int snpmi_standardize_f64(double* val, uint64_t rows, uint64_t cols, int order_c, int is_beta,
                          double a, double b, int apply_in_place, int use_stats, double* stats,
                          int num_threads);

/* ---------------------------------------------------------------- subset (bed-reader subset_*) */
/* out[i,j,q] = val[row_idx[i], col_idx[j], q]; val is rows x cols x k in in_order_c. */
int snpmi_subset_f64_f64(const double* val, uint64_t rows, uint64_t cols, uint64_t k, int in_order_c,
                         const uint64_t* row_idx, uint64_t n_rows, const uint64_t* col_idx,
                         uint64_t n_cols, int out_order_c, double* out, int num_threads);
int snpmi_subset_f32_f64(const float* val, uint64_t rows, uint64_t cols, uint64_t k, int in_order_c,
                         const uint64_t* row_idx, uint64_t n_rows, const uint64_t* col_idx,
                         uint64_t n_cols, int out_order_c, double* out, int num_threads);
int snpmi_subset_f32_f32(const float* val, uint64_t rows, uint64_t cols, uint64_t k, int in_order_c,
                         const uint64_t* row_idx, uint64_t n_rows, const uint64_t* col_idx,
                         uint64_t n_cols, int out_order_c, float* out, int num_threads);

/* ---------------------------------------------------------------- fused read + standardize */
int snpmi_bed_read_standardize_f32(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                                   const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                                   uint64_t n_out_sid, int order_c, int std_kind, double a, double b,
                                   int use_stats, float* stats, float* out, int num_threads);
int snpmi_bed_read_standardize_f64(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                                   const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                                   uint64_t n_out_sid, int order_c, int std_kind, double a, double b,
                                   int use_stats, double* stats, double* out, int num_threads);

/* ---------------------------------------------------------------- GRM (SnpKernel) */
/* K_out: n_out_iid x n_out_iid (symmetric).  stats: [n_out_sid][2] in/out (in if use_stats).
 * diag_k_to_n != 0 additionally applies DiagKtoN on the device and returns the factor. */
int snpmi_grm_bed_f32(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                      const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                      uint64_t n_out_sid, int std_kind, double a, double b, int use_stats,
                      float* stats, int diag_k_to_n, double* factor, float* K_out, int num_threads);
int snpmi_grm_bed_f64(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                      const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                      uint64_t n_out_sid, int std_kind, double a, double b, int use_stats,
                      double* stats, int diag_k_to_n, double* factor, double* K_out, int num_threads);
int snpmi_grm_dense_f32(const float* val, uint64_t rows, uint64_t cols, int order_c, int std_kind,
                        double a, double b, int use_stats, float* stats, int diag_k_to_n,
                        double* factor, float* K_out);
int snpmi_grm_dense_f64(const double* val, uint64_t rows, uint64_t cols, int order_c, int std_kind,
                        double a, double b, int use_stats, double* stats, int diag_k_to_n,
                        double* factor, double* K_out);
/* GRM over several .bed files that share the iids -- DistributedBed / _MergeSIDs pieces,
 * per-chromosome shards (distributedbed.py:16-207, pstreader/_mergecols.py:117-159, reached
 * from SnpReader._read_kernel snpreader.py:623-668 on a merged reader).  begin ->
 * add_bed (any number; stats per file as in snpmi_grm_bed_*) -> end (DiagKtoN + copy-out).
 * For one process per GPU, add this rank's files, then all-reduce the session tiles
 * (snpmi_grm_session_tiles + snpmi_rccl_allreduce_sum) before end. */
int snpmi_grm_begin(uint64_t n_out_iid, int dtype);
int snpmi_grm_add_bed_f32(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                          const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                          uint64_t n_out_sid, int std_kind, double a, double b, int use_stats,
                          float* stats, int num_threads);
int snpmi_grm_add_bed_f64(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                          const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                          uint64_t n_out_sid, int std_kind, double a, double b, int use_stats,
                          double* stats, int num_threads);
/* snpmi_grm_add_bed_{f32,f64} as the session's LAST add (a rank's SNP span of a .bed) + the K-tile
 * collective (1 = reduce onto root, 2 = all-reduce, 0 = none), overlapped on the file stream's last
 * chunk as in snpmi_grm_add_packed_reduce_*: shard.grm_sharded under RCCL (snpreader.py:623-668
 * per rank, then the sum over ranks).  Same K bit for bit as the add followed by the collective. */
int snpmi_grm_add_bed_reduce_f32(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1, const uint64_t* iid_idx,
                                 uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid, int std_kind,
                                 double a, double b, int use_stats, float* stats, int num_threads, int collective,
                                 int root, int parts);
int snpmi_grm_add_bed_reduce_f64(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1, const uint64_t* iid_idx,
                                 uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid, int std_kind,
                                 double a, double b, int use_stats, double* stats, int num_threads, int collective,
                                 int root, int parts);
/* add Z Z^T of an already standardized rows x cols block (F or C order) to the session */
int snpmi_grm_add_dense_f32(const float* val, uint64_t rows, uint64_t cols, int order_c);
int snpmi_grm_add_dense_f64(const double* val, uint64_t rows, uint64_t cols, int order_c);
/* add packed SNP columns already in HBM ([n_sid][pitch] bytes, pitch = snpmi_packed_pitch(n_iid),
 * every iid of the session) -- the per-rank shard of shard.grm_sharded / bench.py's cfg4 leg
 * (the block loop of snpreader.py:651-655 over a device-resident BED body).  The library runs
 * one stats + one SYRK launch per <= 65536 SNPs.  stats [n_sid][2]: host memory (synchronous) or
 * device memory (the call only enqueues on the library stream). */
int snpmi_grm_add_packed_f32(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, int count_a1,
                             int std_kind, double a, double b, int use_stats, float* stats);
int snpmi_grm_add_packed_f64(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, int count_a1,
                             int std_kind, double a, double b, int use_stats, double* stats);
/* snpmi_grm_add_packed_f32 (the session's LAST add) + the K-tile collective of the SNP-sharded
 * GRM (snpmi_rccl_reduce_sum / _allreduce_sum; collective 1 = reduce onto root, 2 = all-reduce,
 * 0 = none), overlapped: the last SNP chunk's SYRK runs as `parts` column groups of the triangle
 * (same K bit for bit) and each finished group's contiguous tile range is summed on the aux stream
 * under the next group's SYRK; the compute stream waits for the last sum.  Host stats (or a path
 * without column groups) run the add and then the collective, unoverlapped.  syrk_done (optional hipEvent_t from snpmi_event_create) is
 * recorded after the last group's SYRK.  Replaces the add + reduce pair of shard.ShardedGrm
 * (the rank loop of snpreader.py:651-655 followed by the sum over ranks). */
int snpmi_grm_add_packed_reduce_f32(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                                    int count_a1, int std_kind, double a, double b, int use_stats, float* stats,
                                    int collective, int root, int parts, void* syrk_done);
/* f64: the groups are the int8-CRT path's residue chunks of the last launch (cut at block-column
 * boundaries; `parts` is ignored) */
int snpmi_grm_add_packed_reduce_f64(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                                    int count_a1, int std_kind, double a, double b, int use_stats, double* stats,
                                    int collective, int root, int parts, void* syrk_done);
int snpmi_grm_session_tiles(void** tiles, uint64_t* count);   /* device tiles + element count */
/* The session's K-tile collective over the ranks (1 = reduce onto root, 2 = all-reduce), without
 * an add: the same RCCL calls, in the same order, as snpmi_grm_add_*_reduce_* with the same
 * `parts` -- a rank that owns no SNPs (or added its SNPs unoverlapped) joins the others' ranged sums
 * with this call.  The calls depend only on n, dtype, parts and the kernel configuration, never on
 * a rank's SNP count.  Replaces the sum over ranks after the block loop of snpreader.py:651-655. */
int snpmi_grm_session_sum(int collective, int root, int parts);
/* K_out NULL: end the session without a result (a non-root rank after snpmi_rccl_reduce_sum) */
int snpmi_grm_end(int diag_k_to_n, double* factor, void* K_out);
int snpmi_diag_k_to_n_f32(float* K, uint64_t n, double* factor);
/* SNP-side DiagKtoN (standardizer/diag_K_to_N.py:75-95): factor = rows / sum(val^2) (f64
 * accumulation); val *= sqrt(factor) unless |factor - 1| <= 1e-15.  val is any contiguous
 * rows x cols array (order does not matter). */
int snpmi_diag_k_to_n_snps_f32(float* val, uint64_t rows, uint64_t cols, double* factor);
int snpmi_diag_k_to_n_snps_f64(double* val, uint64_t rows, uint64_t cols, double* factor);
/* val[i] *= scale for a contiguous host array (DiagKtoNTrained.standardize, diag_K_to_N.py:101-159) */
int snpmi_scale_f32(float* val, uint64_t count, double scale);
int snpmi_scale_f64(double* val, uint64_t count, double scale);
int snpmi_diag_k_to_n_f64(double* K, uint64_t n, double* factor);

/* ---------------------------------------------------------------- device-resident API
 * Buffers below are device pointers from snpmi_dev_alloc; work is enqueued on the
 * library's per-device stream (use snpmi_stream_sync / events).  Packed BED data on the
 * device is [n_sid][pitch] bytes with pitch % 64 == 0 (snpmi_packed_pitch). */
uint64_t snpmi_packed_pitch(uint64_t n_iid);
int snpmi_dev_alloc(void** ptr, uint64_t bytes);
int snpmi_dev_free(void* ptr);
/* page-locked host memory (the staging side of streamed SNP blocks) */
int snpmi_host_alloc(void** ptr, uint64_t bytes);
int snpmi_host_free(void* ptr);
int snpmi_dev_memset(void* ptr, int value, uint64_t bytes);
int snpmi_memcpy_h2d(void* dst, const void* src, uint64_t bytes);
int snpmi_memcpy_d2h(void* dst, const void* src, uint64_t bytes);
/* device -> device on the library stream (asynchronous; bench.py's measured copy peak) */
int snpmi_dev_memcpy_d2d(void* dst, const void* src, uint64_t bytes);
int snpmi_stream_sync(void);
int snpmi_event_create(void** ev);
int snpmi_event_destroy(void* ev);
int snpmi_event_record(void* ev);
int snpmi_event_elapsed_ms(void* start, void* stop, float* ms);
/* Streaming: the library keeps TWO streams per device -- compute (every kernel above) and copy
 * (DMA).  The file-backed entry points pipeline their chunks across them (H2D of chunk c+1 and
 * D2H of chunk c-1 overlap the kernels of chunk c); these calls let a caller build the same
 * pipeline over its own pinned buffers (snpmi_host_alloc).  on_copy: 0 = compute, 1 = copy.
 * kind: 0 = host->device, 1 = device->host, 2 = device->device.  snpmi_stream_sync waits for
 * both streams. */
int snpmi_memcpy_async(void* dst, const void* src, uint64_t bytes, int kind, int on_copy);
/* on_copy above may also be 2: the aux compute stream.  snpmi_set_stream(which) makes the calling
 * thread's stateless device calls (snpmi_dev_snp_stats / _decode / _decode_standardize /
 * _grm_extract / _memset / _memcpy_d2d, snpmi_event_record, the RCCL calls) enqueue on the compute
 * stream (0, the default) or on the aux stream (2), so a caller can run block k+1's stats beside
 * block k's decode (bench.py --overlap-stats); order the two with snpmi_event_record_on /
 * snpmi_stream_wait_event.  The file-backed and GRM-session entry points always use the compute
 * stream. */
int snpmi_set_stream(int which);
int snpmi_event_record_on(void* ev, int on_copy);
int snpmi_stream_wait_event(void* ev, int on_copy);   /* that stream waits for ev (no host wait) */
int snpmi_event_sync(void* ev);

/* counter-based synthetic genotypes (SnpGen MAF curve, snpreader/snpgen.py:140-151) */
int snpmi_dev_synth_bed(uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t sid0, uint64_t n_sid,
                        uint64_t seed, double miss_rate, const double* maf_x, const double* maf_cdf,
                        int n_pts);
/* the same workload on host threads (streamed cfg5 legs): SNPs [sid0, sid0+n_sid) with the MAF
 * table of snpmi_dev_synth_bed, one 32-bit hash per genotype (a different stream than the device
 * generator, same distribution) */
int snpmi_host_synth_bed(uint8_t* dst, uint64_t pitch, uint64_t n_iid, uint64_t sid0, uint64_t n_sid, uint64_t seed,
                         double miss_rate, const double* maf_x, const double* maf_cdf, int n_pts, int num_threads);
/* selected .bed columns (all iids) into a host buffer at `pitch` bytes per column (zero pad) --
 * the gather half of the file readers (bed.py:337-343), for the cfg5 plan's per-rank shares */
int snpmi_bed_gather_packed(const char* path, uint64_t n_iid, uint64_t n_sid, const uint64_t* sid_idx, uint64_t n_sel,
                            uint64_t pitch, uint8_t* dst, int num_threads);
/* per-SNP code counts -> stats [n_sid][2] (dtype) and value LUT [n_sid][4] (dtype) */
int snpmi_dev_snp_stats(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                        int count_a1, int std_kind, double a, double b, int use_stats, int dtype,
                        void* stats, void* lut);
/* packed + LUT -> values, column j at out + j*ld (F) or row i at out + i*ld (C) */
int snpmi_dev_decode(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                     const void* lut, int dtype, int order_c, void* out, uint64_t ld);
/* fused per-SNP stats + decode (f32, F order): one pass per column, LUT/stats written too */
int snpmi_dev_decode_standardize(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                                 int count_a1, int std_kind, double a, double b, int use_stats, int dtype,
                                 void* stats, void* lut, void* out, uint64_t ld);
/* values (dtype, F: column j at val + j*ld with ld % 16 == 0; C: row i at val + i*ld) -> packed
 * codes; *bad_values (if non-NULL; synchronises) = number of waves that saw a value outside
 * {0,1,2,missing} (0 = all valid) */
int snpmi_dev_encode(const void* val, int dtype, int order_c, uint64_t ld, uint64_t n_iid, uint64_t n_sid,
                     int count_a1, uint8_t* packed, uint64_t pitch, uint64_t* bad_values);
/* iid gather: dst column j = src column j restricted to iids idx[0..n_out) */
int snpmi_dev_repack(const uint8_t* src, uint64_t src_pitch, uint64_t n_src_iid, const uint64_t* idx,
                     uint64_t n_out_iid, uint64_t n_sid, uint8_t* dst, uint64_t dst_pitch);
/* GRM tiles: K_tiles holds the upper-triangle 128x128 tiles of an n x n K
 * (snpmi_grm_tile_bytes); accumulate != 0 adds to it. */
uint64_t snpmi_grm_tile_bytes(uint64_t n_iid, int dtype);
int snpmi_dev_syrk_packed(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                          const void* lut, int dtype, void* K_tiles, int accumulate);
/* cfg5 mode (K too large to replicate): the upper triangle of the n x n K as 256x256
 * blocks, grouped into S x S-block supertiles (S = 16 once there are >= 4 supertiles per part,
 * else the largest power of two that gives as many) dealt round-robin in triangular supertile
 * order: supertile T = J(J+1)/2 + I belongs to part T mod part_world.  Part `part_rank` stores its
 * n_local blocks densely, each a full row-major 256x256 f32 block at blocks + b*65536, in its
 * walk order (its supertiles in T order, inside each block column by block column);
 * snpmi_grm_part_coords gives block b's (row0, col0), snpmi_grm_part_coords_all all of them
 * ([n_local][2]).  Every rank reads all SNPs; no reduction is needed.  The K sub-matrices the
 * reference's KernelReader serves (kernelreader.py:245-302) are read back from these blocks. */
uint64_t snpmi_grm_part_blocks(uint64_t n_iid, int part_rank, int part_world);
int snpmi_grm_part_coords(uint64_t n_iid, int part_rank, int part_world, uint64_t local_block,
                          uint64_t* row0, uint64_t* col0);
int snpmi_grm_part_coords_all(uint64_t n_iid, int part_rank, int part_world, uint64_t* coords);
int snpmi_dev_syrk_packed_part(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                               const void* lut, int part_rank, int part_world, void* blocks, int accumulate);
/* the same in float64 (the reference's default GRM dtype, snpreader.py:528,623): f64 LUT [n_sid][4],
 * blocks of 256x256 f64; computed on the int8 MFMA as exact residue products + CRT */
int snpmi_dev_syrk_packed_part_f64(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                                   const double* lut, int part_rank, int part_world, double* blocks, int accumulate);
/* cfg5 from a .bed file (SnpReader._read_kernel, snpreader.py:623-668, with K partitioned as
 * above): this rank streams every selected SNP, standardizes it with stats over all selected
 * iids (stats in/out as snpmi_grm_bed_f32), accumulates only its own blocks and writes them to
 * blocks_out[snpmi_grm_part_blocks][256][256] (rows/cols past n are padding).  blocks_out may be
 * host memory (copied out at the end) or device memory (accumulated in place: K stays in HBM). */
int snpmi_grm_part_bed_f32(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                           const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid,
                           int std_kind, double a, double b, int use_stats, float* stats, int part_rank,
                           int part_world, float* blocks_out, int num_threads);
int snpmi_grm_part_bed_f64(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                           const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid,
                           int std_kind, double a, double b, int use_stats, double* stats, int part_rank,
                           int part_world, double* blocks_out, int num_threads);
/* K[ri[r], ci[c]] (ri/ci host arrays, NULL = identity; order_c: out row-major) restricted to the
 * blocks part `part_rank` owns, 0 elsewhere, times `scale` (DiagKtoN) -- summed over the parts the
 * sub-matrix; out host or device.  The reader of a partitioned K (shard.PartitionedKernel, the
 * KernelReader._read of kernelreader.py:245-302 / snpkernel.py:78-101 for a K that is not
 * replicated).  IndexError for indices >= n. */
int snpmi_grm_part_extract_f32(const float* blocks, uint64_t n_iid, int part_rank, int part_world, const uint64_t* ri,
                               uint64_t nr, const uint64_t* ci, uint64_t nc, int order_c, double scale, float* out);
int snpmi_grm_part_extract_f64(const double* blocks, uint64_t n_iid, int part_rank, int part_world, const uint64_t* ri,
                               uint64_t nr, const uint64_t* ci, uint64_t nc, int order_c, double scale, double* out);
/* this part's share of trace(K) (DiagKtoN over a partitioned K, diag_K_to_N.py:54-59) */
int snpmi_grm_part_trace_f32(const float* blocks, uint64_t n_iid, int part_rank, int part_world, double* trace);
int snpmi_grm_part_trace_f64(const double* blocks, uint64_t n_iid, int part_rank, int part_world, double* trace);
/* free / total HBM of the current device (hipMemGetInfo): whether a replicated K fits */
int snpmi_device_memory(uint64_t* free_bytes, uint64_t* total_bytes);
int snpmi_dev_syrk_dense(const void* Z, uint64_t ldz, uint64_t n_iid, uint64_t n_sid, int dtype,
                         void* K_tiles, int accumulate);
/* tiles -> K[ri[r], ci[c]] (ri/ci NULL = identity), scaled by `scale` */
int snpmi_dev_grm_extract(const void* K_tiles, uint64_t n_iid, int dtype, const uint64_t* ri, uint64_t nr,
                          const uint64_t* ci, uint64_t nc, int order_c, double scale, void* out);
int snpmi_dev_grm_trace(const void* K_tiles, uint64_t n_iid, int dtype, double* trace);
/* float64 GRMs run on the int8 MFMA as residues modulo the first R of 15 coprime moduli, R chosen
 * per SNP block on the device from the block's own bound max_i sum_s q_is^2:
 * sum of R and number of such blocks on this device since the last reset (synchronous). */
int snpmi_crt_moduli_stats(uint64_t* sum_r, uint64_t* launches, int reset);
/* per 256-block: each block (bi, bj) runs only the moduli with P_R > 2 sqrt(M_bi M_bj), M_p = the
 * largest sum_s q_is^2 of its iid panel p (Cauchy-Schwarz per block; K is the same bits as with the
 * launch-wide R): sum of R_b and number of blocks since the last reset (synchronous). */
int snpmi_crt_block_moduli_stats(uint64_t* sum_rb, uint64_t* blocks, int reset);

/* ---------------------------------------------------------------- RCCL (one process per GPU) */
int snpmi_rccl_unique_id(uint8_t* id, uint64_t id_len);   /* id_len >= 128 */
int snpmi_rccl_init(int nranks, int rank, const uint8_t* id, uint64_t id_len);
int snpmi_rccl_allreduce_sum(void* buf, uint64_t count, int dtype);
/* In-place sum of the K tiles onto rank `root` only (the caller of read_kernel holds K:
 * snpreader.py:623-668 returns K to its one process); ncclReduce moves half the bytes of the
 * all-reduce over xGMI.  buf on non-root ranks is left unspecified. */
int snpmi_rccl_reduce_sum(void* buf, uint64_t count, int dtype, int root);
/* cfg5: every rank contributes bytes_per_rank bytes; recv gets them concatenated in rank
 * order (send may alias recv + rank * bytes_per_rank) */
int snpmi_rccl_allgather(const void* send, void* recv, uint64_t bytes_per_rank);
/* host-value all-reduce (op 0 = sum, 1 = max) of f64 scalars, synchronous; barrier = 1-elem sum */
int snpmi_rccl_host_allreduce_f64(double* values, uint64_t count, int op);
int snpmi_rccl_barrier(void);
int snpmi_rccl_comm_count(int* count);                    /* ncclCommCount: ranks in the communicator */
int snpmi_rccl_destroy(void);
/* Collective trace of this process (lock-free; callable from another thread while one sits in a
 * collective): out[0..11] = calls, all-reduces, reduces, all-gathers, host all-reduces (barriers /
 * max), bytes enqueued, signature of the (kind, count, root) sequence (FNV-1a: the same calls in the
 * same order give the same value on every rank), last kind (1 all-reduce, 2 reduce, 3 all-gather,
 * 4 host), last count, 1 while inside a blocking host all-reduce, completed host all-reduces,
 * communicator present.  n = entries wanted (<= 12). */
int snpmi_rccl_trace(uint64_t* out, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif /* SNPMI_H */
