// libsnpmi C ABI (include/snpmi.h): host orchestration of the BED -> GRM path on one GPU.
//
// Data flow of every file-backed entry point (one SNP chunk at a time):
//   mmap(.bed) --gather selected columns, pitch-padded--> pinned host buffer
//     --H2D--> packed codes in HBM --[k_repack: iid subset]--> k_snp_stats (stats + LUT)
//     --> k_decode_f/c (values)  or  MFMA SYRK into upper-triangle K tiles
//     --> D2H into the caller's NumPy buffer.
// The packed codes are 16x (f32) / 32x (f64) smaller than the values, so only packed bytes
// cross PCIe on the way in.
#include <fcntl.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

#include "snpmi_internal.hpp"

#include <type_traits>

namespace snpmi {

// ====================================================================== errors / devices
static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }

static std::mutex g_dev_mutex;
static std::vector<Device*> g_devices;
static thread_local int g_cur_dev = -1;

static int default_device() {
    const char* e = std::getenv("PST_DEVICE");
    return e ? std::atoi(e) : 0;
}

static int num_devices() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

Device& device() {
    if (g_cur_dev < 0) g_cur_dev = default_device();
    std::lock_guard<std::mutex> lk(g_dev_mutex);
    const int n = num_devices();
    SNPMI_REQUIRE(n > 0, SNPMI_E_HIP, "no HIP device available (libsnpmi has no CPU fallback)");
    SNPMI_REQUIRE(g_cur_dev < n, SNPMI_E_ARG, "device index out of range");
    if ((int)g_devices.size() < n) g_devices.resize(n, nullptr);
    Device*& d = g_devices[g_cur_dev];
    SNPMI_HIP(hipSetDevice(g_cur_dev));
    if (!d) {
        d = new Device();
        d->id = g_cur_dev;
        SNPMI_HIP(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
        SNPMI_HIP(hipStreamCreateWithFlags(&d->copy, hipStreamNonBlocking));
        SNPMI_HIP(hipStreamCreateWithFlags(&d->aux, hipStreamNonBlocking));
        for (hipEvent_t* set : {d->staged, d->consumed, d->produced, d->bounce})
            for (int s = 0; s < 2; s++) SNPMI_HIP(hipEventCreateWithFlags(&set[s], hipEventDisableTiming));
        for (int s = 0; s < kPieces; s++) SNPMI_HIP(hipEventCreateWithFlags(&d->piece[s], hipEventDisableTiming));
        SNPMI_HIP(hipEventCreateWithFlags(&d->fence, hipEventDisableTiming));
        hipDeviceProp_t p;
        SNPMI_HIP(hipGetDeviceProperties(&p, g_cur_dev));
        d->cu_count = p.multiProcessorCount;
    }
    return *d;
}

static thread_local int g_sel_stream = 0;  // snpmi_set_stream: 0 compute, 2 aux

hipStream_t stream() {
    Device& d = device();
    return g_sel_stream == 2 ? d.aux : d.stream;
}

void* Device::get(Slot s, size_t bytes) {
    if (bytes == 0) bytes = 256;
    if (cap[s] < bytes) {
        if (buf[s]) SNPMI_HIP(hipFree(buf[s]));
        buf[s] = nullptr;
        cap[s] = 0;
        size_t want = round_up(bytes, 1 << 20);
        if (hipMalloc(&buf[s], want) != hipSuccess) {
            (void)hipGetLastError();
            buf[s] = nullptr;
            throw Error(SNPMI_E_NOMEM, "hipMalloc of " + std::to_string(want) + " bytes failed");
        }
        cap[s] = want;
    }
    return buf[s];
}

void Device::release() {
    for (int s = 0; s < S_NUM; s++) {
        if (buf[s]) (void)hipFree(buf[s]);
        buf[s] = nullptr;
        cap[s] = 0;
    }
    for (int x = 0; x < 2; x++) {
        if (order_tab[x]) (void)hipFree(order_tab[x]);
        order_tab[x] = nullptr;
        order_nb[x] = 0;
    }
    if (part_tab) (void)hipFree(part_tab);
    part_tab = nullptr;
    for (int i = 0; i < 3; i++) part_key[i] = 0;
}

// pinned staging (two slots so a chunk can be gathered while the previous one uploads)
static std::mutex g_pin_mutex;
constexpr int kPinSlots = 6 + kPieces;  // 0: encoder, 2: stats, 4/5: D2H bounce, 6..: H2D piece ring
static void* g_pin[kPinSlots] = {};
static size_t g_pin_cap[kPinSlots] = {};

void* pinned(int slot, size_t bytes) {
    std::lock_guard<std::mutex> lk(g_pin_mutex);
    if (g_pin_cap[slot] < bytes) {
        if (g_pin[slot]) (void)hipHostFree(g_pin[slot]);
        g_pin[slot] = nullptr;
        g_pin_cap[slot] = 0;
        size_t want = round_up(bytes, 1 << 20);
        if (hipHostMalloc(&g_pin[slot], want, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            throw Error(SNPMI_E_NOMEM, "pinned allocation failed");
        }
        g_pin_cap[slot] = want;
    }
    return g_pin[slot];
}

void release_pinned() {
    std::lock_guard<std::mutex> lk(g_pin_mutex);
    for (int s = 0; s < kPinSlots; s++) {
        if (g_pin[s]) (void)hipHostFree(g_pin[s]);
        g_pin[s] = nullptr;
        g_pin_cap[s] = 0;
    }
}

// one API call at a time per process: scratch slots and the stream are shared
static std::recursive_mutex g_call_mutex;

// ====================================================================== host helpers
static int resolve_threads(int num_threads) {
    if (num_threads > 0) return std::min(num_threads, 64);
    unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc, 16u));
}

template <class F>
static void parallel_for(uint64_t n, int nthreads, F&& fn, uint64_t grain = 64) {
    if (n == 0) return;
    nthreads = (int)std::min<uint64_t>((uint64_t)nthreads, n);
    if (nthreads <= 1 || n < grain) {
        for (uint64_t i = 0; i < n; i++) fn(i);
        return;
    }
    std::atomic<uint64_t> next(0);
    std::vector<std::thread> th;
    th.reserve(nthreads);
    for (int t = 0; t < nthreads; t++)
        th.emplace_back([&] {
            for (;;) {
                uint64_t s = next.fetch_add(grain);
                if (s >= n) break;
                uint64_t e = std::min(n, s + grain);
                for (uint64_t i = s; i < e; i++) fn(i);
            }
        });
    for (auto& t : th) t.join();
}

// Device -> pageable host copy of `rows` rows of `width` bytes (device pitch spitch, host
// pitch dpitch) on the COPY stream, ordered after the compute stream's work so far (or after
// `after`).  A plain hipMemcpy to pageable memory runs at ~16 GB/s (the runtime's own bounce +
// a single-threaded copy); here 256 MiB pieces DMA into two pinned bounce buffers while host
// threads copy the previous piece out, so PCIe and the host copy overlap -- and, because the
// DMA sits on its own stream, kernels enqueued before this call keep running beside it.
static void d2h_rows(Device& d, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows,
                     int nthreads, hipEvent_t after = nullptr) {
    if (rows == 0 || width == 0) return;
    if (!after) {
        SNPMI_HIP(hipEventRecord(d.fence, d.stream));
        after = d.fence;
    }
    SNPMI_HIP(hipStreamWaitEvent(d.copy, after, 0));
    const size_t total = width * rows;
    if (total < (32u << 20)) {
        SNPMI_HIP(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, hipMemcpyDeviceToHost, d.copy));
        SNPMI_HIP(hipStreamSynchronize(d.copy));
        return;
    }
    const size_t per = std::max<size_t>(1, (256u << 20) / width);
    uint8_t* bounce[2] = {(uint8_t*)pinned(4, per * width), (uint8_t*)pinned(5, per * width)};
    hipEvent_t* ev = d.bounce;
    auto drain = [&](size_t r0, size_t nr, int slot) {
        SNPMI_HIP(hipEventSynchronize(ev[slot]));
        const uint8_t* b = bounce[slot];
        uint8_t* o = (uint8_t*)dst + r0 * dpitch;
        if (dpitch == width) {
            const size_t bytes = nr * width, per_t = round_up(ceil_div(bytes, (size_t)nthreads), 4096);
            parallel_for(
                ceil_div(bytes, per_t), nthreads,
                [&](uint64_t q) {
                    const size_t a = q * per_t, e = std::min(bytes, a + per_t);
                    std::memcpy(o + a, b + a, e - a);
                },
                1);
        } else {
            parallel_for(
                nr, nthreads, [&](uint64_t r) { std::memcpy(o + r * dpitch, b + r * width, width); },
                std::max<uint64_t>(1, (1u << 20) / width));
        }
    };
    size_t prev_r0 = 0, prev_n = 0;
    int i = 0;
    for (size_t r0 = 0; r0 < rows; r0 += per, i++) {
        const size_t nr = std::min(per, rows - r0);
        const int slot = i & 1;
        SNPMI_HIP(hipMemcpy2DAsync(bounce[slot], width, (const uint8_t*)src + r0 * spitch, spitch, width, nr,
                                   hipMemcpyDeviceToHost, d.copy));
        SNPMI_HIP(hipEventRecord(ev[slot], d.copy));
        if (i > 0) drain(prev_r0, prev_n, slot ^ 1);
        prev_r0 = r0;
        prev_n = nr;
    }
    drain(prev_r0, prev_n, (i - 1) & 1);
}

// contiguous byte range as rows of 4 MiB (+ a tail) through the pipelined copy above.  (The
// same bounce for host->device measured no faster than the runtime's pageable H2D: the
// source pages are already resident, while a D2H into fresh NumPy memory pays page faults
// that the threaded copy-out spreads over cores.)
static void d2h_bytes(Device& d, void* dst, const void* src, size_t bytes, int nthreads) {
    const size_t w = 4u << 20, rows = bytes / w, tail = bytes - rows * w;
    d2h_rows(d, dst, w, src, w, w, rows, nthreads);
    if (tail) d2h_rows(d, (uint8_t*)dst + rows * w, tail, (const uint8_t*)src + rows * w, tail, tail, 1, nthreads);
}

struct BedMap {
    int fd = -1;
    const uint8_t* base = nullptr;
    size_t size = 0;
    uint64_t bpc = 0;
    ~BedMap() {
        // unmapping a page-cache mapping of a few GB tears down ~1M page-table entries (~4 ms at
        // 1.25 GB, measured between the last SYRK and the K extraction, profiles/r03h): every
        // gather from it has returned, so a large mapping goes away off the call's critical path
        if (base && size >= (64u << 20)) {
            std::thread([p = (void*)base, n = size] { munmap(p, n); }).detach();
        } else if (base) {
            munmap((void*)base, size);
        }
        if (fd >= 0) close(fd);
    }
    const uint8_t* column(uint64_t s) const { return base + 3 + s * bpc; }
};

// bed-reader's open_bed format check (magic 6C 1B 01 = SNP-major) + size check.
static void open_bed(BedMap& m, const char* path, uint64_t n_iid, uint64_t n_sid) {
    SNPMI_REQUIRE(path != nullptr, SNPMI_E_ARG, "path is NULL");
    m.fd = open(path, O_RDONLY);
    SNPMI_REQUIRE(m.fd >= 0, SNPMI_E_IO, std::string("cannot open ") + path);
    struct stat st;
    SNPMI_REQUIRE(fstat(m.fd, &st) == 0, SNPMI_E_IO, std::string("cannot stat ") + path);
    m.size = (size_t)st.st_size;
    m.bpc = ceil_div(n_iid, 4);
    SNPMI_REQUIRE(m.size >= 3, SNPMI_E_FORMAT, std::string("file too short to be a .bed file: ") + path);
    void* p = mmap(nullptr, m.size, PROT_READ, MAP_SHARED, m.fd, 0);
    SNPMI_REQUIRE(p != MAP_FAILED, SNPMI_E_IO, std::string("mmap failed: ") + path);
    m.base = (const uint8_t*)p;
    SNPMI_REQUIRE(m.base[0] == 0x6C && m.base[1] == 0x1B, SNPMI_E_FORMAT,
                  std::string("not a PLINK .bed file (bad magic): ") + path);
    SNPMI_REQUIRE(m.base[2] == 0x01, SNPMI_E_FORMAT,
                  std::string("only SNP-major .bed files are supported: ") + path);
    SNPMI_REQUIRE(m.size == 3 + n_sid * m.bpc, SNPMI_E_FORMAT,
                  std::string(".bed size does not match .fam/.bim counts: ") + path);
    (void)madvise(p, m.size, MADV_SEQUENTIAL);
}

static void check_index(const uint64_t* idx, uint64_t n, uint64_t bound, const char* what) {
    if (!idx) return;
    for (uint64_t i = 0; i < n; i++)
        SNPMI_REQUIRE(idx[i] < bound, SNPMI_E_INDEX,
                      std::string(what) + " index " + std::to_string(idx[i]) + " out of range (count " +
                          std::to_string(bound) + ")");
}

static bool is_identity(const uint64_t* idx, uint64_t n, uint64_t bound) {
    if (!idx) return true;
    if (n != bound) return false;
    for (uint64_t i = 0; i < n; i++)
        if (idx[i] != i) return false;
    return true;
}

// Gather SNP columns [c0, c0+cnt) of the selection into `dst` with `pitch` bytes each.
// g_gather 0 (default): memcpy from the mmap; 1: pread() per column into the pinned piece.  A/B on
// a 50k x 100k file in the page cache (tools/exp_gather.py, profiles/r03j): the full 1.25 GB read
// into HBM at 37-47 GB/s of packed codes with the mmap vs 32-35 GB/s with pread, so the mmap stays
static int g_gather = 0;
static void gather_columns(const BedMap& m, const uint64_t* sid_idx, uint64_t c0, uint64_t cnt, uint64_t pitch,
                           uint8_t* dst, int nthreads) {
    const bool use_pread = g_gather == 1;
    parallel_for(cnt, nthreads, [&](uint64_t j) {
        const uint64_t s = sid_idx ? sid_idx[c0 + j] : c0 + j;
        uint8_t* d = dst + j * pitch;
        if (use_pread) {
            size_t got = 0;
            while (got < m.bpc) {
                const ssize_t r = pread(m.fd, d + got, m.bpc - got, (off_t)(3 + s * m.bpc + got));
                if (r <= 0) break;
                got += (size_t)r;
            }
            if (got < m.bpc) std::memcpy(d + got, m.column(s) + got, m.bpc - got);  // short read: the mapping
        } else {
            std::memcpy(d, m.column(s), m.bpc);
        }
        if (pitch > m.bpc) std::memset(d + m.bpc, 0, pitch - m.bpc);
    });
}

// Device-side iid selection state for one call.
struct IidPlan {
    uint64_t n_in, n_out, pitch_in, pitch_out;
    bool repack;
    uint64_t* idx_dev = nullptr;
    RepackPlan plan;                // gather plan of k_repack_lds / k_repack_win
};

static IidPlan plan_iids(Device& d, const uint64_t* iid_idx, uint64_t n_iid, uint64_t n_out) {
    IidPlan p;
    p.n_in = n_iid;
    p.n_out = iid_idx ? n_out : n_iid;
    p.pitch_in = packed_pitch(n_iid);
    p.pitch_out = packed_pitch(p.n_out);
    p.repack = !is_identity(iid_idx, p.n_out, n_iid);
    if (p.repack && p.n_out) {
        p.idx_dev = (uint64_t*)d.get(Device::S_IDX, p.n_out * 8);
        SNPMI_HIP(hipMemcpyAsync(p.idx_dev, iid_idx, p.n_out * 8, hipMemcpyHostToDevice, d.stream));
        uint32_t* plan = (uint32_t*)d.get(Device::S_IDX32, repack_plan_entries(p.n_out) * 4);
        uint32_t* win = (uint32_t*)d.get(Device::S_WIN, repack_win_entries(p.n_out) * 4);
        p.plan = launch_repack_plan(p.idx_dev, p.n_out, p.n_in, plan, win, d.stream);
    }
    return p;
}

// Upload SNP chunk [c0, c0+cnt) and return the device packed buffer for the selected iids.
// Chunks alternate between two device buffers (slot = chunk parity).  The H2D runs on the copy
// stream: it waits only for the kernels that last read this device slot (chunk c-2, event
// `consumed`), so the upload of chunk c overlaps the kernels of chunk c-1.  The compute stream
// waits on `staged` before touching the chunk.  Callers record consumed[slot] on the compute
// stream after the chunk's last kernel (chunk_done).
//
// The host side goes through a ring of kPieces pinned pieces of <= kPieceBytes (not one pinned
// buffer per chunk): the host gathers piece q+1 from the mmap while piece q crosses PCIe, and
// only 4 x 32 MiB is ever pinned -- a first call no longer pays for pinning two chunk-sized
// buffers (~0.5 GB at 50k iids), and ranks sharing a host hold less locked memory.  The host
// blocks only when the ring is full, i.e. until chunk c-2's kernels are done.
static const uint8_t* stage_chunk(Device& d, const BedMap& m, const uint64_t* sid_idx, uint64_t c0, uint64_t cnt,
                                  const IidPlan& p, int nthreads, int slot) {
    uint8_t* dev = (uint8_t*)d.get(slot ? Device::S_PACKED_B : Device::S_PACKED, cnt * p.pitch_in);
    SNPMI_HIP(hipStreamWaitEvent(d.copy, d.consumed[slot], 0));
    const uint64_t per = std::max<uint64_t>(1, kPieceBytes / p.pitch_in);
    for (uint64_t q0 = 0; q0 < cnt; q0 += per) {
        const uint64_t qn = std::min(per, cnt - q0);
        const int ps = (int)(d.piece_next++ % kPieces);
        SNPMI_HIP(hipEventSynchronize(d.piece[ps]));  // this pinned piece's previous H2D has finished
        uint8_t* host = (uint8_t*)pinned(6 + ps, std::min(cnt, per) * p.pitch_in);
        gather_columns(m, sid_idx, c0 + q0, qn, p.pitch_in, host, nthreads);
        SNPMI_HIP(hipMemcpyAsync(dev + q0 * p.pitch_in, host, qn * p.pitch_in, hipMemcpyHostToDevice, d.copy));
        SNPMI_HIP(hipEventRecord(d.piece[ps], d.copy));
    }
    SNPMI_HIP(hipEventRecord(d.staged[slot], d.copy));
    SNPMI_HIP(hipStreamWaitEvent(d.stream, d.staged[slot], 0));
    if (!p.repack) return dev;
    uint8_t* dev2 = (uint8_t*)d.get(Device::S_PACKED2, cnt * p.pitch_out);
    launch_repack(dev, p.pitch_in, p.n_in, p.idx_dev, p.plan, p.n_out, cnt, dev2, p.pitch_out, d.stream);
    return dev2;
}

static void chunk_done(Device& d, int slot) { SNPMI_HIP(hipEventRecord(d.consumed[slot], d.stream)); }

// Value / K buffers may be HOST or DEVICE memory (unified virtual addressing): a pointer into a
// snpmi_dev_alloc / hipMalloc allocation of the current device is computed on in place or
// written directly, without the host staging -- the device-resident SnpData / KernelData of
// pysnptools_amd.hbm (the reference's array-module seam, util/__init__.py:652-730).  Stats
// arrays stay host memory.
static bool is_device_ptr(Device& d, const void* p) {
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable host memory is unknown to HIP
        return false;
    }
    if (at.type != hipMemoryTypeDevice) return false;
    SNPMI_REQUIRE(at.device == d.id, SNPMI_E_ARG,
                  "device buffer belongs to device " + std::to_string(at.device) + ", the call runs on device " +
                      std::to_string(d.id));
    return true;
}

template <typename T>
struct DT;
template <>
struct DT<float> {
    static constexpr int v = SNPMI_DT_F32;
};
template <>
struct DT<double> {
    static constexpr int v = SNPMI_DT_F64;
};
template <>
struct DT<int8_t> {
    static constexpr int v = SNPMI_DT_I8;
};

static uint64_t chunk_snps(uint64_t per_snp_bytes, uint64_t budget = 1ull << 30) {
    uint64_t c = std::max<uint64_t>(1, budget / std::max<uint64_t>(per_snp_bytes, 1));
    return std::min<uint64_t>(c, 1ull << 16);
}

// ====================================================================== BED read (+ standardize)
template <typename T>
static void bed_read_impl(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1, const uint64_t* iid_idx,
                          uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid, int order_c, int std_kind,
                          double a, double b, int use_stats, T* stats, T* out, int num_threads) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    SNPMI_REQUIRE(out != nullptr || (n_out_iid == 0 || n_out_sid == 0), SNPMI_E_ARG, "out is NULL");
    BedMap m;
    open_bed(m, path, n_iid, n_sid);
    const uint64_t n_out = iid_idx ? n_out_iid : n_iid;
    const uint64_t m_out = sid_idx ? n_out_sid : n_sid;
    check_index(iid_idx, n_out, n_iid, "iid");
    check_index(sid_idx, m_out, n_sid, "sid");
    if (m_out == 0) return;
    Device& d = device();
    const int nthreads = resolve_threads(num_threads);
    IidPlan p = plan_iids(d, iid_idx, n_iid, n_out);
    const int dt = DT<T>::v;
    const bool dev_out = is_device_ptr(d, out);
    // device output: decode straight into it when its columns (F) meet the 16-B vector-store
    // alignment of k_decode_f, else through the block buffer + a device-to-device copy; C order
    // always straight (k_decode_c_reg checks alignment itself, k_decode_c has none)
    const bool direct = dev_out && (order_c || (reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                                                (n_out * sizeof(T)) % 16 == 0));
    const uint64_t ldF = round_up(std::max<uint64_t>(n_out, 1), 16);
    const uint64_t C = chunk_snps(p.pitch_in + p.pitch_out + ldF * sizeof(T));
    const bool stats_out = std_kind != SNPMI_STD_NONE && !use_stats;
    // Three-stage pipeline over SNP chunks, two slots each: host gather + H2D (copy stream) of
    // chunk c, stats + decode of chunk c (compute stream), D2H + host copy-out of chunk c-1 (copy
    // stream, after `produced`).  PCIe runs both directions at once and the kernels of chunk c
    // hide under the copy-out of chunk c-1.
    struct Pending {
        uint64_t c0 = 0, cnt = 0, ldc = 0;
        int slot = 0;
        T* dev_out = nullptr;
        T* st_dev = nullptr;
        bool valid = false;
    } pending;
    auto drain = [&](const Pending& q) {
        if (n_out > 0 && dev_out && !direct) {
            SNPMI_HIP(hipStreamWaitEvent(d.copy, d.produced[q.slot], 0));
            SNPMI_HIP(hipMemcpy2DAsync(out + q.c0 * n_out, n_out * sizeof(T), q.dev_out, ldF * sizeof(T),
                                       n_out * sizeof(T), q.cnt, hipMemcpyDeviceToDevice, d.copy));
            SNPMI_HIP(hipStreamSynchronize(d.copy));  // the block buffer slot is reused two chunks on
        } else if (n_out > 0 && !dev_out) {
            if (!order_c)
                d2h_rows(d, out + q.c0 * n_out, n_out * sizeof(T), q.dev_out, ldF * sizeof(T), n_out * sizeof(T),
                         q.cnt, nthreads, d.produced[q.slot]);
            else
                d2h_rows(d, out + q.c0, m_out * sizeof(T), q.dev_out, q.ldc * sizeof(T), q.cnt * sizeof(T), n_out,
                         nthreads, d.produced[q.slot]);
        }
    };
    // per-SNP stats stay on the device for the whole call and cross PCIe once each way (a per-chunk
    // D2H on the copy stream would wait for that chunk's kernels and stall the next upload)
    T* st_all = (T*)d.get(Device::S_STATS, m_out * 2 * sizeof(T));
    if (std_kind != SNPMI_STD_NONE && use_stats)
        SNPMI_HIP(hipMemcpyAsync(st_all, stats, m_out * 2 * sizeof(T), hipMemcpyHostToDevice, d.stream));
    for (uint64_t c0 = 0, ci = 0; c0 < m_out; c0 += C, ci++) {
        const uint64_t cnt = std::min(C, m_out - c0);
        const int slot = (int)(ci & 1);
        const uint8_t* packed = stage_chunk(d, m, sid_idx, c0, cnt, p, nthreads, slot);
        T* lut = (T*)d.get(Device::S_LUT, cnt * 4 * sizeof(T));
        T* st_dev = st_all + 2 * c0;
        launch_snp_stats(packed, p.pitch_out, n_out, cnt, count_a1, std_kind, a, b, use_stats, dt, st_dev, lut,
                         d.stream);
        Pending q;
        q.c0 = c0;
        q.cnt = cnt;
        q.slot = slot;
        q.st_dev = st_dev;
        q.valid = true;
        if (n_out > 0 && direct) {
            if (!order_c) launch_decode(packed, p.pitch_out, n_out, cnt, lut, dt, 0, out + c0 * n_out, n_out, d.stream);
            else launch_decode(packed, p.pitch_out, n_out, cnt, lut, dt, 1, out + c0, m_out, d.stream);
        } else if (n_out > 0) {
            const Device::Slot os = slot ? Device::S_OUT_B : Device::S_OUT;
            if (!order_c) {
                q.dev_out = (T*)d.get(os, cnt * ldF * sizeof(T));
                launch_decode(packed, p.pitch_out, n_out, cnt, lut, dt, 0, q.dev_out, ldF, d.stream);
            } else {
                // rows padded to 16 B on the device (k_decode_c_reg vector stores), tight on the host
                q.ldc = sizeof(T) < 4 ? cnt : round_up(cnt, 16 / sizeof(T));
                q.dev_out = (T*)d.get(os, q.ldc * n_out * sizeof(T));
                launch_decode(packed, p.pitch_out, n_out, cnt, lut, dt, 1, q.dev_out, q.ldc, d.stream);
            }
        }
        chunk_done(d, slot);
        SNPMI_HIP(hipEventRecord(d.produced[slot], d.stream));
        if (pending.valid) drain(pending);
        pending = q;
    }
    if (pending.valid) drain(pending);
    if (stats_out) SNPMI_HIP(hipMemcpyAsync(stats, st_all, m_out * 2 * sizeof(T), hipMemcpyDeviceToHost, d.stream));
    SNPMI_HIP(hipStreamSynchronize(d.stream));
    SNPMI_HIP(hipStreamSynchronize(d.copy));
}

// ====================================================================== BED write (to_bed body)
// Values (caller's host array, n_iid x n_sid, F or C) -> .bed file: magic + SNP-major packed
// columns of ceil(n/4) bytes.  SNP chunks go H2D, are encoded by k_encode_f/c, and come back
// as packed bytes (16x / 32x smaller) that are written with one fwrite per chunk.
template <typename T>
static void bed_write_impl(const char* path, const T* val, uint64_t n, uint64_t m, int order_c, int count_a1) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    SNPMI_REQUIRE(path != nullptr, SNPMI_E_ARG, "path is NULL");
    SNPMI_REQUIRE(val != nullptr || n == 0 || m == 0, SNPMI_E_ARG, "val is NULL");
    Device& d = device();
    FILE* f = std::fopen(path, "wb");
    SNPMI_REQUIRE(f != nullptr, SNPMI_E_IO, std::string("cannot create ") + path);
    struct Closer {
        FILE*& f;
        const char* path;
        bool ok = false;
        ~Closer() {
            if (f) std::fclose(f);
            if (!ok) std::remove(path);
        }
    } closer{f, path};
    const uint8_t magic[3] = {0x6C, 0x1B, 0x01};
    SNPMI_REQUIRE(std::fwrite(magic, 1, 3, f) == 3, SNPMI_E_IO, std::string("write failed: ") + path);
    const uint64_t bpc = ceil_div(n, 4), pitch = packed_pitch(n);
    const int dt = DT<T>::v;
    unsigned int* bad_dev = (unsigned int*)d.get(Device::S_RED, 256);
    if (n > 0 && m > 0) {
        const uint64_t ldF = round_up(n, 16);
        const uint64_t C = order_c ? std::min<uint64_t>(round_up(chunk_snps(n * sizeof(T) + pitch), 64), 1ull << 16)
                                   : chunk_snps(ldF * sizeof(T) + pitch);
        for (uint64_t c0 = 0; c0 < m; c0 += C) {
            const uint64_t cnt = std::min(C, m - c0);
            T* dev_val = (T*)d.get(Device::S_DENSE, cnt * (order_c ? n : ldF) * sizeof(T));
            uint8_t* dev_packed = (uint8_t*)d.get(Device::S_PACKED, cnt * pitch);
            uint8_t* host = (uint8_t*)pinned(0, cnt * bpc);
            SNPMI_HIP(hipMemsetAsync(bad_dev, 0, sizeof(unsigned int), d.stream));
            if (!order_c) {
                SNPMI_HIP(hipMemcpy2DAsync(dev_val, ldF * sizeof(T), val + c0 * n, n * sizeof(T), n * sizeof(T), cnt,
                                           hipMemcpyDefault, d.stream));  // host or device values
                launch_encode(dev_val, dt, 0, ldF, n, cnt, count_a1, dev_packed, pitch, bad_dev, d.stream);
            } else {
                SNPMI_HIP(hipMemcpy2DAsync(dev_val, cnt * sizeof(T), val + c0, m * sizeof(T), cnt * sizeof(T), n,
                                           hipMemcpyDefault, d.stream));
                launch_encode(dev_val, dt, 1, cnt, n, cnt, count_a1, dev_packed, pitch, bad_dev, d.stream);
            }
            unsigned int bad = 0;
            SNPMI_HIP(hipMemcpyAsync(&bad, bad_dev, sizeof(bad), hipMemcpyDeviceToHost, d.stream));
            SNPMI_HIP(hipMemcpy2DAsync(host, bpc, dev_packed, pitch, bpc, cnt, hipMemcpyDeviceToHost, d.stream));
            SNPMI_HIP(hipStreamSynchronize(d.stream));
            SNPMI_REQUIRE(bad == 0, SNPMI_E_ARG,
                          "Expect values to be 0, 1, 2 or missing (NaN, or -127 for int8)");
            SNPMI_REQUIRE(std::fwrite(host, 1, cnt * bpc, f) == cnt * bpc, SNPMI_E_IO,
                          std::string("write failed: ") + path);
        }
    }
    SNPMI_REQUIRE(std::fclose(f) == 0, SNPMI_E_IO, std::string("write failed: ") + path);
    f = nullptr;
    closer.ok = true;
}

// ====================================================================== dense standardize / subset
template <typename T>
static void standardize_impl(T* val, uint64_t rows, uint64_t cols, int order_c, int is_beta, double a, double b,
                             int apply_in_place, int use_stats, T* stats) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    SNPMI_REQUIRE(stats != nullptr, SNPMI_E_ARG, "stats is NULL");
    if (cols == 0) return;
    Device& d = device();
    const size_t bytes = rows * cols * sizeof(T);
    const bool dev = is_device_ptr(d, val);
    // a device val is standardized in place (a scratch copy when only the stats are wanted)
    T* dv = dev && apply_in_place ? val : (T*)d.get(Device::S_DENSE, bytes);
    T* ds = (T*)d.get(Device::S_STATS, cols * 2 * sizeof(T));
    const int nthreads = resolve_threads(0);
    if (dv != val) SNPMI_HIP(hipMemcpyAsync(dv, val, bytes, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                                           d.stream));
    if (use_stats) SNPMI_HIP(hipMemcpyAsync(ds, stats, cols * 2 * sizeof(T), hipMemcpyHostToDevice, d.stream));
    launch_dense_standardize(dv, rows, cols, order_c ? cols : rows, order_c, DT<T>::v,
                             is_beta ? SNPMI_STD_BETA : SNPMI_STD_UNIT, a, b, use_stats, ds, d.stream);
    if (apply_in_place && !dev) d2h_bytes(d, val, dv, bytes, nthreads);
    if (!use_stats) SNPMI_HIP(hipMemcpyAsync(stats, ds, cols * 2 * sizeof(T), hipMemcpyDeviceToHost, d.stream));
    SNPMI_HIP(hipStreamSynchronize(d.stream));
}

template <typename S, typename D>
static void subset_impl(const S* val, uint64_t rows, uint64_t cols, uint64_t k, int in_c, const uint64_t* ri,
                        uint64_t nr, const uint64_t* ci, uint64_t nc, int out_c, D* out) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    SNPMI_REQUIRE(k >= 1, SNPMI_E_ARG, "k must be >= 1");
    SNPMI_REQUIRE(ri && ci, SNPMI_E_ARG, "subset needs explicit row and column indices");
    check_index(ri, nr, rows, "row");
    check_index(ci, nc, cols, "col");
    if (nr * nc == 0) return;
    Device& d = device();
    const size_t in_bytes = rows * cols * k * sizeof(S);
    const bool dev_in = is_device_ptr(d, val), dev_out = is_device_ptr(d, out);
    const S* dv = dev_in ? val : (const S*)d.get(Device::S_DENSE, in_bytes);
    uint64_t* dri = (uint64_t*)d.get(Device::S_IDX, nr * 8);
    uint64_t* dci = (uint64_t*)d.get(Device::S_IDX2, nc * 8);
    D* dout = dev_out ? out : (D*)d.get(Device::S_OUT, nr * nc * k * sizeof(D));
    if (!dev_in) SNPMI_HIP(hipMemcpyAsync((S*)dv, val, in_bytes, hipMemcpyHostToDevice, d.stream));
    SNPMI_HIP(hipMemcpyAsync(dri, ri, nr * 8, hipMemcpyHostToDevice, d.stream));
    SNPMI_HIP(hipMemcpyAsync(dci, ci, nc * 8, hipMemcpyHostToDevice, d.stream));
    launch_subset(dv, DT<S>::v, rows, cols, k, in_c, dri, nr, dci, nc, out_c, dout, DT<D>::v, d.stream);
    if (!dev_out) d2h_bytes(d, out, dout, nr * nc * k * sizeof(D), resolve_threads(0));
    SNPMI_HIP(hipStreamSynchronize(d.stream));
}

// ====================================================================== GRM
// f32 GRM of a packed SNP block, N >= 4096: two phases per sub-block of SNPs -- k_decode_f
// writes the standardized block Z (f32, F order, ld = round_up(N, 256)) to HBM (0.4 ms per
// 10k SNPs at N=50k), then the dense SYRK streams Z into LDS with global_load_lds and runs
// MFMA-only (no VALU in its loader): 136.7 TFLOP/s vs 130.9 for the fused LUT-expanding
// kernel (tools/ubench.py syrk / syrk_dense, N=50k, 10k SNPs).  Sub-blocks keep Z <= 16 GiB.
static bool use_two_phase(int dt, uint64_t n) {
    if (g_variant_syrk != 0 && g_variant_syrk != 20 && g_variant_syrk != 71) return false;
    return dt == SNPMI_DT_F32 ? n >= 4096 : n >= 1024;
}

template <typename T, class F>
static void for_z_blocks(Device& d, const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, const T* lut,
                         F&& syrk) {
    const uint64_t ldz = round_up(n, 256);
    uint64_t sub = std::min<uint64_t>(m, std::max<uint64_t>(256, (16ull << 30) / (ldz * sizeof(T))));
    sub = std::min<uint64_t>(m, std::max<uint64_t>(16, sub / 16 * 16));
    T* Z = (T*)d.get(Device::S_ZBLK, sub * ldz * sizeof(T));
    if (ldz > n)  // pad iids read by the last panel: keep them finite (they only feed K(i,j), i or j >= n)
        SNPMI_HIP(hipMemset2DAsync(Z + n, ldz * sizeof(T), 0, (ldz - n) * sizeof(T), sub, d.stream));
    for (uint64_t s0 = 0; s0 < m; s0 += sub) {
        const uint64_t cnt = std::min(sub, m - s0);
        launch_decode(packed + s0 * pitch, pitch, n, cnt, lut + 4 * s0, DT<T>::v, 0, Z, ldz, d.stream);
        syrk((const T*)Z, ldz, cnt, s0 > 0);
    }
}

// f32 GRM of packed SNPs: default = the bf16 MFMA pipe (k_syrk_bf3: bf16x3 split of each SNP's
// f32 LUT, six bf16 products per f32 product, f32 accumulate): 309 TFLOP/s at N=50k, 10k SNPs
// vs 136 for the f32-MFMA two-phase path (variant 20) -- tools/ubench.py syrk.
// Variants: 30 = plain loader, 31 = + XCD remap, 33 = end-of-stage barrier, 34 = mid-stage
// barrier without the pinned VALU interleave, 35 = default kernel without split-K, 39 =
// ablation (no loader); 4/5/20 = f32 MFMA.
static int g_variant_syrk_split = 0;  // tuning hook: 0 = auto, 1 = off, S = force S slices
static int g_dense_codes = 1;         // tuning / test hook: 0 = dense operands never re-encoded

static bool use_bf3(int dt) {
    return dt == SNPMI_DT_F32 && (g_variant_syrk == 0 || (g_variant_syrk >= 30 && g_variant_syrk <= 69));
}
// default: the fp16x2 kernel (k_syrk_h2, 3 products) with the bf16x3 kernel as its range
// fallback; 30-39 force bf16x3 alone
static bool use_h2() { return g_variant_syrk == 0 || (g_variant_syrk >= 40 && g_variant_syrk <= 69); }

// split-K slices for the bf16x3 SYRK when the 256x256-block grid leaves CUs idle in its last
// round: minimise rounds-per-slice ceil(g*S / CUs) / S, +1% per extra slice (partial sets + the
// reduce), >= 1024 SNPs per slice.  Measured (tools/ubench.py syrk, m = 20k): N=10k 213 -> 242
// TFLOP/s at S=4, N=5k 199 -> 217 at S=6 -- the slice counts this model picks.
static int bf3_split_slices(uint64_t n, uint64_t m, int cus) {
    if (g_variant_syrk == 35 || g_variant_syrk == 45 || g_variant_syrk_split == 1) return 1;
    if (g_variant_syrk_split > 1) return g_variant_syrk_split;
    const uint64_t nb = ceil_div(n, 256), g = nb * (nb + 1) / 2, C = (uint64_t)std::max(cus, 1);
    const double unsplit = (double)ceil_div(g, C);
    int best = 1;
    double best_cost = unsplit;
    for (int S = 2; S <= 8 && m / (uint64_t)S >= 1024; S++) {
        const double cost = (double)ceil_div(g * S, C) / S * (1.0 + 0.01 * (S - 1));
        if (cost < best_cost) {
            best = S;
            best_cost = cost;
        }
    }
    return best_cost < 0.97 * unsplit ? best : 1;
}

// bf16x3 LUT (32 B per SNP); with h2, also the fp16x2 LUT (16 B per SNP) and its range flag,
// all in one scratch slot
static const uint32_t* lut_bf3(Device& d, const float* lut, uint64_t m, H2Lut* h2 = nullptr) {
    const uint64_t e = lut_bf3_entries(m);
    uint32_t* l3 = (uint32_t*)d.get(Device::S_LUT3, e * 48 + 256);
    launch_lut_bf3(lut, m, l3, d.stream);
    if (h2) {
        uint32_t* l2 = l3 + 8 * e;
        uint32_t* flag = l2 + 4 * e;
        launch_lut_h2(lut, m, l2, flag, d.stream);
        h2->lut2 = l2;
        h2->flag = flag;
    }
    return l3;
}

// f64 GRM of packed SNPs: default = the int8 MFMA residue path (syrk_crt.hip; variant 70 forces
// it), 71 = the f64 MFMA two-phase path (decode to a dense f64 block, then k_syrk_glds).
static int g_f64_mfma = 0;  // public switch "f64" (pysnptools_amd.set_grm_f64): 1 = every f64 GRM on the f64 MFMA
static bool use_crt(int dt) {
    return dt == SNPMI_DT_F64 && !g_f64_mfma &&
           (g_variant_syrk == 0 || (g_variant_syrk >= 70 && g_variant_syrk != 71 && g_variant_syrk <= 99));
}

// f32 segment scratch pool of the current device (syrk.hip SegFlush): kSegSlots slots of 256 KiB
// + their flags, zeroed once when the pool is first allocated (slots are released by the kernels)
SegCtx seg_ctx() {
    SegCtx c;
    c.snps = g_seg_snps > 0 ? (uint32_t)g_seg_snps : 0u;
    if (!c.snps) return c;
    Device& d = device();
    const bool fresh = d.cap[Device::S_SEG] == 0;
    const uint64_t bytes = (uint64_t)kSegSlots * kSegSlotFloats * sizeof(float) + kSegSlots * sizeof(uint32_t);
    uint8_t* base = (uint8_t*)d.get(Device::S_SEG, bytes);
    c.nslots = kSegSlots;
    c.scratch = (float*)base;
    c.flags = (uint32_t*)(base + (uint64_t)kSegSlots * kSegSlotFloats * sizeof(float));
    if (fresh) {  // once per device; complete before any stream's first SYRK can take a slot
        SNPMI_HIP(hipMemsetAsync(c.flags, 0, kSegSlots * sizeof(uint32_t), d.stream));
        SNPMI_HIP(hipStreamSynchronize(d.stream));
    }
    return c;
}

// CRT moduli counters on the device: [0] sum of the launch-wide R, [1] launches (k_crt_r); [2] sum
// of the per-block R_b, [3] blocks (k_crt)
static unsigned long long* crt_record(Device& d) {
    const bool fresh = d.cap[Device::S_CRTREC] == 0;
    auto* rec = (unsigned long long*)d.get(Device::S_CRTREC, 32);
    if (fresh) SNPMI_HIP(hipMemsetAsync(rec, 0, 32, d.stream));
    return rec;
}

static void syrk_packed_crt(Device& d, const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m,
                            const double* lut, double* tiles, int accumulate) {
    const uint64_t nb = ceil_div(n, 256), blocks = nb * (nb + 1) / 2;
    // residue scratch: one byte per modulus and element of the 256-blocks, at most 4 GiB (then chunked)
    const uint64_t res_bytes = std::min<uint64_t>(blocks * (uint64_t)crt_moduli() * 65536, 4ull << 30);
    uint8_t* res = (uint8_t*)d.get(Device::S_ZBLK, res_bytes);
    const uint64_t step = crt_max_snps();
    void* ws = d.get(Device::S_LUT3, crt_lut_bytes(std::min(m, step), n));
    unsigned long long* rec = crt_record(d);
    for (uint64_t s0 = 0; s0 < m; s0 += step) {
        const uint64_t cnt = std::min(step, m - s0);
        const int acc = accumulate || s0 > 0;
        launch_syrk_packed_crt(packed + s0 * pitch, pitch, n, cnt, lut + 4 * s0, tiles, acc, ws, res, res_bytes,
                               rec, d.stream);
        // NaN/Inf in this chunk's LUT: the f64 MFMA kernel computes it (gated on the device flag)
        launch_syrk_packed_f64_gated(packed + s0 * pitch, pitch, n, cnt, lut + 4 * s0, tiles, acc,
                                     (const int*)ws + 1, d.stream);
    }
}

static void syrk_packed_f32_body(Device& d, const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m,
                                 const void* lut, int dt, void* tiles, int accumulate);

static void syrk_packed_auto(Device& d, const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m,
                             const void* lut, int dt, void* tiles, int accumulate) {
    if (use_crt(dt) && m > 0 && n > 0) {
        syrk_packed_crt(d, packed, pitch, n, m, (const double*)lut, (double*)tiles, accumulate);
        return;
    }
    if (dt == SNPMI_DT_F32 && g_diag_exact && m > 0 && n > 0) {  // exact diagonal around the SYRK
        double* diag = (double*)d.get(Device::S_DIAG, diag_scratch_bytes(n, m));
        launch_diag_begin((const float*)tiles, n, nullptr, accumulate, diag, d.stream);
        syrk_packed_f32_body(d, packed, pitch, n, m, lut, dt, tiles, accumulate);
        launch_diag_end(packed, pitch, n, m, (const float*)lut, (float*)tiles, nullptr, diag, d.stream);
        return;
    }
    syrk_packed_f32_body(d, packed, pitch, n, m, lut, dt, tiles, accumulate);
}

static void syrk_packed_f32_body(Device& d, const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m,
                                 const void* lut, int dt, void* tiles, int accumulate) {
    if (use_bf3(dt)) {
        H2Lut h2;
        const bool h = use_h2() && m > 0;
        const uint32_t* l3 = lut_bf3(d, (const float*)lut, m, h ? &h2 : nullptr);
        const int S = bf3_split_slices(n, m, d.cu_count);
        if (S > 1) {
            float* part = (float*)d.get(Device::S_ZBLK, (uint64_t)S * n_tiles_upper(n) * kTile * kTile * sizeof(float));
            launch_syrk_packed_bf3_split(packed, pitch, n, m, l3, S, part, (float*)tiles, accumulate, d.stream,
                                         h ? &h2 : nullptr);
        } else {
            launch_syrk_packed_bf3(packed, pitch, n, m, l3, (float*)tiles, accumulate, d.stream, h ? &h2 : nullptr);
        }
        return;
    }
    if (!use_two_phase(dt, n) || m == 0) {
        launch_syrk_packed(packed, pitch, n, m, lut, dt, tiles, accumulate, d.stream);
        return;
    }
    auto run = [&](const void* Z, uint64_t ldz, uint64_t cnt, bool more) {
        launch_syrk_dense(Z, ldz, n, cnt, dt, tiles, accumulate || more, d.stream);
    };
    if (dt == SNPMI_DT_F32) for_z_blocks(d, packed, pitch, n, m, (const float*)lut, run);
    else for_z_blocks(d, packed, pitch, n, m, (const double*)lut, run);
}

static void syrk_packed_part_body(Device& d, const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m,
                                  const float* lut, int rank, int world, void* blocks, int accumulate);

static void syrk_packed_part_auto(Device& d, const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m,
                                  const float* lut, int rank, int world, void* blocks, int accumulate) {
    if (g_diag_exact && m > 0 && n > 0) {  // exact diagonal of the part's diagonal blocks
        double* diag = (double*)d.get(Device::S_DIAG, diag_scratch_bytes(n, m));
        const int32_t* dslot = part_tables(ceil_div(n, 256), rank, world).dslot;
        launch_diag_begin((const float*)blocks, n, dslot, accumulate, diag, d.stream);
        syrk_packed_part_body(d, packed, pitch, n, m, lut, rank, world, blocks, accumulate);
        launch_diag_end(packed, pitch, n, m, lut, (float*)blocks, dslot, diag, d.stream);
        return;
    }
    syrk_packed_part_body(d, packed, pitch, n, m, lut, rank, world, blocks, accumulate);
}

// f64 part (cfg5 in the reference's default dtype): the int8 CRT path over the part's layout
// (launch_syrk_packed_crt with the layout table: residue chunks of the part's blocks, K written as
// dense f64 blocks), its f64-MFMA fallback gated on the non-finite flag; hook "f64" = 1: every
// block on the f64 MFMA
static void syrk_packed_part_f64(Device& d, const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m,
                                 const double* lut, int rank, int world, double* blocks, int accumulate) {
    const uint64_t nloc = grm_part_blocks(n, rank, world);
    if (nloc == 0) return;
    SNPMI_REQUIRE(4 * nloc < (1ull << 31), SNPMI_E_ARG, "too many GRM blocks for one launch");
    SNPMI_REQUIRE(pitch % 64 == 0 && pitch * 4 >= ceil_div(n, 256) * 256, SNPMI_E_ARG,
                  "packed pitch must cover round_up(n, 256) iids");
    if (m == 0) {
        if (!accumulate) SNPMI_HIP(hipMemsetAsync(blocks, 0, nloc * 256 * 256 * sizeof(double), d.stream));
        return;
    }
    const PartTables pt = part_tables(ceil_div(n, 256), rank, world);
    const uint64_t step = crt_max_snps();
    if (!use_crt(SNPMI_DT_F64)) {
        for (uint64_t s0 = 0; s0 < m; s0 += step)
            launch_syrk_packed_f64_gated(packed + s0 * pitch, pitch, n, std::min(step, m - s0), lut + 4 * s0, blocks,
                                         accumulate || s0 > 0, nullptr, d.stream, pt.tab, nloc);
        return;
    }
    const uint64_t res_bytes = std::min<uint64_t>(nloc * (uint64_t)crt_moduli() * 65536, 4ull << 30);
    uint8_t* res = (uint8_t*)d.get(Device::S_ZBLK, res_bytes);
    void* ws = d.get(Device::S_LUT3, crt_lut_bytes(std::min(m, step), n));
    unsigned long long* rec = crt_record(d);
    for (uint64_t s0 = 0; s0 < m; s0 += step) {
        const uint64_t cnt = std::min(step, m - s0);
        const int acc = accumulate || s0 > 0;
        launch_syrk_packed_crt(packed + s0 * pitch, pitch, n, cnt, lut + 4 * s0, blocks, acc, ws, res, res_bytes, rec,
                               d.stream, nullptr, nullptr, pt.tab, nloc);
        launch_syrk_packed_f64_gated(packed + s0 * pitch, pitch, n, cnt, lut + 4 * s0, blocks, acc, (const int*)ws + 1,
                                     d.stream, pt.tab, nloc);
    }
}

static void syrk_packed_part_body(Device& d, const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m,
                                  const float* lut, int rank, int world, void* blocks, int accumulate) {
    if (use_bf3(SNPMI_DT_F32)) {
        H2Lut h2;
        const bool h = use_h2() && m > 0;
        const uint32_t* l3 = lut_bf3(d, lut, m, h ? &h2 : nullptr);
        launch_syrk_packed_bf3_part(packed, pitch, n, m, l3, rank, world, (float*)blocks, accumulate, d.stream,
                                    h ? &h2 : nullptr);
        return;
    }
    if (!use_two_phase(SNPMI_DT_F32, n) || m == 0) {
        launch_syrk_packed_part(packed, pitch, n, m, lut, rank, world, blocks, accumulate, d.stream);
        return;
    }
    for_z_blocks(d, packed, pitch, n, m, lut, [&](const float* Z, uint64_t ldz, uint64_t cnt, bool more) {
        launch_syrk_dense_part(Z, ldz, n, cnt, rank, world, blocks, accumulate || more, d.stream);
    });
}
// Finish a GRM held as tiles on the device: optional DiagKtoN, then K (n x n) to the host,
// extracted in row blocks so the device never needs a second full-size K.
template <typename T>
static void grm_finish(Device& d, const T* tiles, uint64_t n, int diag_k_to_n, double* factor, T* K_out) {
    double scale = 1.0;
    if (diag_k_to_n) {
        double* tr = (double*)d.get(Device::S_RED, 64);
        launch_grm_trace(tiles, n, DT<T>::v, tr, d.stream);
        double trace = 0;
        SNPMI_HIP(hipMemcpyAsync(&trace, tr, 8, hipMemcpyDeviceToHost, d.stream));
        SNPMI_HIP(hipStreamSynchronize(d.stream));
        const double f = (double)n / trace;
        if (factor) *factor = f;
        if (std::fabs(f - 1.0) > 1e-15) scale = f;  // diag_K_to_N.py:56-59
    }
    if (n == 0) return;
    const bool dev = is_device_ptr(d, K_out);
    const uint64_t rows_per = dev ? n : std::max<uint64_t>(1, std::min<uint64_t>(n, (1ull << 30) / (n * sizeof(T))));
    for (uint64_t r0 = 0; r0 < n; r0 += rows_per) {
        const uint64_t nr = std::min(rows_per, n - r0);
        // a device K_out is written in one extraction launch, no host copy; a host K_out goes
        // through 1 GiB row blocks (d2h_rows returns once the block has landed, so the next
        // extraction may reuse the staging buffer)
        T* dk = dev ? K_out : (T*)d.get(Device::S_K, nr * n * sizeof(T));
        launch_grm_extract_rows(tiles, n, DT<T>::v, r0, nr, scale, dk, d.stream);
        if (!dev) d2h_rows(d, K_out + r0 * n, n * sizeof(T), dk, n * sizeof(T), n * sizeof(T), nr, resolve_threads(0));
    }
    SNPMI_HIP(hipStreamSynchronize(d.stream));
}

// Stream the SNP columns of one .bed through stats and `syrk(packed, pitch, n, cnt, lut,
// accumulate)` (first = overwrite).  Returns true if anything was written.
template <typename T, class Syrk>
static bool grm_stream_bed(Device& d, bool first, const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                           const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid,
                           int std_kind, double a, double b, int use_stats, T* stats, int num_threads, Syrk&& syrk) {
    BedMap m;
    open_bed(m, path, n_iid, n_sid);
    const uint64_t n_out = iid_idx ? n_out_iid : n_iid;
    const uint64_t m_out = sid_idx ? n_out_sid : n_sid;
    check_index(iid_idx, n_out, n_iid, "iid");
    check_index(sid_idx, m_out, n_sid, "sid");
    SNPMI_REQUIRE(stats != nullptr || std_kind == SNPMI_STD_NONE || m_out == 0, SNPMI_E_ARG, "stats is NULL");
    const int nthreads = resolve_threads(num_threads);
    const int dt = DT<T>::v;
    IidPlan p = plan_iids(d, iid_idx, n_iid, n_out);
    // ~0.5 GiB of packed codes per chunk keeps >= 2 chunks in flight for cfg4-sized inputs
    const uint64_t C = chunk_snps(p.pitch_in + p.pitch_out, 1ull << 29);
    const bool has_stats = std_kind != SNPMI_STD_NONE && m_out > 0 && n_out > 0;
    // stats of every chunk stay on the device (16 B per SNP) and cross PCIe once, before / after
    // the chunk loop: a per-chunk stats D2H on the compute stream shares a DMA engine with the
    // next chunk's H2D and held that upload until the chunk's SYRK had finished (profiles/r03h)
    T* st_host = has_stats ? (T*)pinned(2, m_out * 2 * sizeof(T)) : nullptr;
    T* st_all = (T*)d.get(Device::S_STATS, std::max<uint64_t>(m_out, 1) * 2 * sizeof(T));
    if (has_stats && use_stats) {
        std::memcpy(st_host, stats, m_out * 2 * sizeof(T));
        SNPMI_HIP(hipMemcpyAsync(st_all, st_host, m_out * 2 * sizeof(T), hipMemcpyHostToDevice, d.stream));
    }
    bool wrote = false;
    // the first chunk is an eighth of the others: its gather + upload is the one that cannot hide
    // under a SYRK, the later ones stage while the previous chunk computes
    const uint64_t C1 = std::max<uint64_t>(std::min<uint64_t>(C, 2048), C / 8);
    if (m_out > C1 && n_out > 0) {  // size both device slots for a full chunk up front: no regrowth
        const uint64_t cmax = std::min(C, m_out);  // (a free + alloc) between the first two chunks
        SNPMI_HIP(hipStreamSynchronize(d.copy));
        for (int slot = 0; slot < 2; slot++) (void)d.get(slot ? Device::S_PACKED_B : Device::S_PACKED, cmax * p.pitch_in);
        if (p.repack) (void)d.get(Device::S_PACKED2, cmax * p.pitch_out);
    }
    for (uint64_t c0 = 0, ci = 0; c0 < m_out && n_out > 0; ci++) {
        const uint64_t cnt = std::min(ci == 0 ? C1 : C, m_out - c0);
        const uint8_t* packed = stage_chunk(d, m, sid_idx, c0, cnt, p, nthreads, (int)(ci & 1));
        T* lut = (T*)d.get(Device::S_LUT, std::min(C, m_out) * 4 * sizeof(T));
        T* st_dev = st_all + 2 * c0;
        launch_snp_stats(packed, p.pitch_out, n_out, cnt, count_a1, std_kind, a, b, use_stats, dt, st_dev, lut,
                         d.stream);
        syrk(packed, p.pitch_out, n_out, cnt, (const T*)lut, !(first && !wrote));
        wrote = true;
        chunk_done(d, (int)(ci & 1));
        c0 += cnt;
    }
    if (has_stats && !use_stats && n_out > 0)
        SNPMI_HIP(hipMemcpyAsync(st_host, st_all, m_out * 2 * sizeof(T), hipMemcpyDeviceToHost, d.stream));
    SNPMI_HIP(hipStreamSynchronize(d.stream));
    SNPMI_HIP(hipStreamSynchronize(d.copy));
    if (has_stats && !use_stats && n_out > 0) std::memcpy(stats, st_host, m_out * 2 * sizeof(T));
    if (n_out == 0 && std_kind != SNPMI_STD_NONE && !use_stats) {
        for (uint64_t j = 0; j < m_out; j++) stats[2 * j] = stats[2 * j + 1] = (T)NAN;
    }
    return wrote;
}

// Accumulate the SNP columns of one .bed into the replicated upper-triangle tiles.
template <typename T>
static bool grm_add_bed(Device& d, T* tiles, bool first, const char* path, uint64_t n_iid, uint64_t n_sid,
                        int count_a1, const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                        uint64_t n_out_sid, int std_kind, double a, double b, int use_stats, T* stats,
                        int num_threads) {
    return grm_stream_bed<T>(d, first, path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid, std_kind,
                             a, b, use_stats, stats, num_threads,
                             [&](const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t cnt, const T* lut, bool acc) {
                                 syrk_packed_auto(d, packed, pitch, n, cnt, lut, DT<T>::v, tiles, acc);
                             });
}

template <typename T>
static void grm_bed_impl(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1, const uint64_t* iid_idx,
                         uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid, int std_kind, double a,
                         double b, int use_stats, T* stats, int diag_k_to_n, double* factor, T* K_out,
                         int num_threads) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    const uint64_t n_out = iid_idx ? n_out_iid : n_iid;
    SNPMI_REQUIRE(K_out != nullptr || n_out == 0, SNPMI_E_ARG, "K_out is NULL");
    Device& d = device();
    const uint64_t tile_bytes = n_tiles_upper(n_out) * kTile * kTile * sizeof(T);
    T* tiles = (T*)d.get(Device::S_TILES, tile_bytes);
    if (!grm_add_bed<T>(d, tiles, true, path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid,
                        std_kind, a, b, use_stats, stats, num_threads))
        SNPMI_HIP(hipMemsetAsync(tiles, 0, tile_bytes, d.stream));
    grm_finish(d, tiles, n_out, diag_k_to_n, factor, K_out);
}

// ---------------------------------------------------------------------- GRM session (several .bed files)
struct GrmSession {
    bool active = false;
    bool wrote = false;
    uint64_t n = 0;
    int dtype = SNPMI_DT_F32;
};
static GrmSession g_session;

static void* session_tiles(Device& d) {
    return d.get(Device::S_SESSION, n_tiles_upper(g_session.n) * kTile * kTile * dtype_size(g_session.dtype));
}

// supertile block order of the dense fp16x2 SYRK, kept on the device per (nb, xcd); built once
// (blocking copy from a local vector), callers hold g_call_mutex
static const uint32_t* dense_order(Device& d, uint64_t nb, bool xcd) {
    if (d.order_nb[xcd] != nb || !d.order_tab[xcd]) {
        std::vector<uint32_t> tab;
        supertile_order(nb, xcd, tab);
        if (d.order_tab[xcd]) SNPMI_HIP(hipFree(d.order_tab[xcd]));
        d.order_tab[xcd] = nullptr;
        d.order_nb[xcd] = 0;
        if (hipMalloc(&d.order_tab[xcd], tab.size() * sizeof(uint32_t)) != hipSuccess) {
            (void)hipGetLastError();
            throw Error(SNPMI_E_NOMEM, "hipMalloc of the block order table failed");
        }
        SNPMI_HIP(hipMemcpy(d.order_tab[xcd], tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        d.order_nb[xcd] = nb;
    }
    return d.order_tab[xcd];
}

// the packed fp16x2 SYRK's block order (syrk.hip): the same supertile table, cached per nb
const uint32_t* packed_block_order(uint64_t nb) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    return dense_order(device(), nb, false);
}

// the cfg5 part layout of part `rank` of `world` on the current device (syrk.hip part_layout):
// one allocation = the layout table (u32 per local block) + the diagonal-slot table (i32 per block
// column) + the block-slot table (i32 per upper-triangle block), cached per (nb, rank, world)
PartTables part_tables(uint64_t nb, int rank, int world) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    Device& d = device();
    const uint64_t key[3] = {nb, (uint64_t)rank, (uint64_t)world};
    const uint64_t ntab = grm_part_blocks(nb * 256, rank, world), off = round_up(std::max<uint64_t>(ntab, 1), 64);
    const uint64_t off2 = off + round_up(std::max<uint64_t>(nb, 1), 64), total = nb * (nb + 1) / 2;
    if (!d.part_tab || d.part_key[0] != key[0] || d.part_key[1] != key[1] || d.part_key[2] != key[2]) {
        std::vector<uint32_t> tab;
        part_layout(nb, rank, world, tab);
        SNPMI_REQUIRE(tab.size() == ntab, SNPMI_E_ARG, "part layout size mismatch");
        std::vector<int32_t> dslot(nb, -1), lslot(total, -1);
        for (uint64_t w = 0; w < tab.size(); w++) {
            const uint64_t bi = tab[w] & 0xffffu, bj = tab[w] >> 16;
            if (bi == bj) dslot[bj] = (int32_t)w;
            lslot[bj * (bj + 1) / 2 + bi] = (int32_t)w;
        }
        std::vector<uint32_t> buf(off2 + total);
        std::copy(tab.begin(), tab.end(), buf.begin());
        std::memcpy(buf.data() + off, dslot.data(), nb * sizeof(int32_t));
        std::memcpy(buf.data() + off2, lslot.data(), total * sizeof(int32_t));
        if (d.part_tab) SNPMI_HIP(hipFree(d.part_tab));
        d.part_tab = nullptr;
        for (int i = 0; i < 3; i++) d.part_key[i] = 0;
        if (hipMalloc(&d.part_tab, buf.size() * sizeof(uint32_t)) != hipSuccess) {
            (void)hipGetLastError();
            d.part_tab = nullptr;
            throw Error(SNPMI_E_NOMEM, "hipMalloc of the part layout table failed");
        }
        SNPMI_HIP(hipMemcpy(d.part_tab, buf.data(), buf.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        for (int i = 0; i < 3; i++) d.part_key[i] = key[i];
    }
    PartTables t;
    t.tab = (const uint32_t*)d.part_tab;
    t.dslot = (const int32_t*)((const uint32_t*)d.part_tab + off);
    t.lslot = (const int32_t*)((const uint32_t*)d.part_tab + off2);
    return t;
}

// dense GRM operand on the device: f32 with n >= 4096 and the default variant takes the fp16x2
// split kernel in SNP chunks of bounded stage-image scratch (falls back to the f32-MFMA
// k_syrk256d on the device-side range flag, or when the scratch cannot be allocated)
static void syrk_packed_auto(Device& d, const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m,
                             const void* lut, int dt, void* tiles, int accumulate);

static void syrk_dense_auto(Device& d, const void* Z, uint64_t ldz, uint64_t n, uint64_t m, int dt, void* tiles,
                            int accumulate) {
    if (dt == SNPMI_DT_F32 && g_variant_syrk == 0 && m > 0 && g_dense_codes) {
        // genotype-valued columns (<= 4 distinct values each, e.g. a standardized SnpData): exact
        // re-encoding as codes + LUT, then the packed fp16x2 SYRK; one host sync for the flag
        const uint64_t pitch = packed_pitch(n);
        uint8_t* packed = (uint8_t*)d.get(Device::S_DPACK, m * pitch);
        float* lut = (float*)d.get(Device::S_DLUT, m * 16 + 256);
        unsigned int* flag = (unsigned int*)(lut + 4 * m);
        launch_dense_codes((const float*)Z, ldz, n, m, packed, pitch, lut, flag, d.stream);
        unsigned int f = 1;
        SNPMI_HIP(hipMemcpyAsync(&f, flag, sizeof(f), hipMemcpyDeviceToHost, d.stream));
        SNPMI_HIP(hipStreamSynchronize(d.stream));
        if (f == 0) {
            syrk_packed_auto(d, packed, pitch, n, m, lut, dt, tiles, accumulate);
            return;
        }
    }
    if (dt == SNPMI_DT_F32 && g_variant_syrk == 0 && n >= 4096 && m > 0 && ldz % 256 == 0) {
        const uint64_t nb = ldz / 256;
        const uint64_t scratch = round_up(dense_h2_scratch_bytes(n, m), 256);
        uint16_t* img = nullptr;
        try {
            img = (uint16_t*)d.get(Device::S_H2, scratch + 256);
        } catch (const Error& e) {
            if (e.code != SNPMI_E_NOMEM) throw;
            img = nullptr;  // HBM is full: the f32-MFMA kernel needs no scratch
        }
        if (img) {
            uint32_t* flag = (uint32_t*)((uint8_t*)img + scratch);
            launch_syrk_dense_h2((const float*)Z, ldz, n, m, img, flag, dense_order(d, nb, false), (float*)tiles,
                                 accumulate, d.stream);
            return;
        }
    }
    launch_syrk_dense(Z, ldz, n, m, dt, tiles, accumulate, d.stream);
}

template <typename T>
static void grm_dense_impl(const T* val, uint64_t rows, uint64_t cols, int order_c, int std_kind, double a, double b,
                           int use_stats, T* stats, int diag_k_to_n, double* factor, T* K_out) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    SNPMI_REQUIRE(K_out != nullptr || rows == 0, SNPMI_E_ARG, "K_out is NULL");
    Device& d = device();
    const int dt = DT<T>::v;
    const uint64_t ldz = round_up(std::max<uint64_t>(rows, 1), 256);  // 256-iid panels of the glds SYRK
    T* Z = (T*)d.get(Device::S_DENSE, ldz * std::max<uint64_t>(cols, 1) * sizeof(T));
    if (cols > 0 && rows > 0) {
        if (!order_c) {
            SNPMI_HIP(hipMemcpy2DAsync(Z, ldz * sizeof(T), val, rows * sizeof(T), rows * sizeof(T), cols,
                                       hipMemcpyDefault, d.stream));  // host or device val
        } else if (is_device_ptr(d, val)) {
            launch_transpose_to_f(val, rows, cols, dt, Z, ldz, d.stream);
        } else {
            T* Zc = (T*)d.get(Device::S_DENSE2, rows * cols * sizeof(T));
            SNPMI_HIP(hipMemcpyAsync(Zc, val, rows * cols * sizeof(T), hipMemcpyHostToDevice, d.stream));
            launch_transpose_to_f(Zc, rows, cols, dt, Z, ldz, d.stream);
        }
    }
    if (std_kind != SNPMI_STD_NONE && cols > 0) {
        T* ds = (T*)d.get(Device::S_STATS, cols * 2 * sizeof(T));
        if (use_stats) SNPMI_HIP(hipMemcpyAsync(ds, stats, cols * 2 * sizeof(T), hipMemcpyHostToDevice, d.stream));
        launch_dense_standardize(Z, rows, cols, ldz, 0, dt, std_kind, a, b, use_stats, ds, d.stream);
        if (!use_stats) SNPMI_HIP(hipMemcpyAsync(stats, ds, cols * 2 * sizeof(T), hipMemcpyDeviceToHost, d.stream));
    }
    const uint64_t tile_bytes = n_tiles_upper(rows) * kTile * kTile * sizeof(T);
    T* tiles = (T*)d.get(Device::S_TILES, tile_bytes);
    if (rows > 0) syrk_dense_auto(d, Z, ldz, rows, cols, dt, tiles, 0);
    grm_finish(d, tiles, rows, diag_k_to_n, factor, K_out);
}

template <typename T>
static void diag_k_to_n_impl(T* K, uint64_t n, double* factor) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    if (n == 0) return;
    Device& d = device();
    const bool dev = is_device_ptr(d, K);  // device K: traced and scaled in place
    T* dk = dev ? K : (T*)d.get(Device::S_K, n * n * sizeof(T));
    double* tr = (double*)d.get(Device::S_RED, 64);
    if (!dev) SNPMI_HIP(hipMemcpyAsync(dk, K, n * n * sizeof(T), hipMemcpyHostToDevice, d.stream));
    launch_dense_trace(dk, n, DT<T>::v, tr, d.stream);
    double trace = 0;
    SNPMI_HIP(hipMemcpyAsync(&trace, tr, 8, hipMemcpyDeviceToHost, d.stream));
    SNPMI_HIP(hipStreamSynchronize(d.stream));
    const double f = (double)n / trace;
    if (factor) *factor = f;
    if (std::fabs(f - 1.0) > 1e-15) {
        launch_dense_scale(dk, n * n, DT<T>::v, f, d.stream);
        if (!dev) SNPMI_HIP(hipMemcpyAsync(K, dk, n * n * sizeof(T), hipMemcpyDeviceToHost, d.stream));
        SNPMI_HIP(hipStreamSynchronize(d.stream));
    }
}

// SNP-side DiagKtoN (diag_K_to_N.py:75-95): factor = rows / sum(val^2); val *= sqrt(factor)
// when |factor - 1| > 1e-15.  scale_only: val *= scale (trained DiagKtoN / kernel rescale).
template <typename T>
static void snp_scale_impl(T* val, uint64_t count, double rows, int scale_only, double scale, double* factor) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    if (count == 0) {
        if (factor) *factor = rows / 0.0;
        return;
    }
    Device& d = device();
    const bool dev = is_device_ptr(d, val);  // device val: scaled in place
    T* dv = dev ? val : (T*)d.get(Device::S_DENSE, count * sizeof(T));
    if (!dev) SNPMI_HIP(hipMemcpyAsync(dv, val, count * sizeof(T), hipMemcpyHostToDevice, d.stream));
    double s = scale;
    if (!scale_only) {
        double* ss = (double*)d.get(Device::S_RED, 64);
        launch_sumsq(dv, count, DT<T>::v, ss, d.stream);
        double sum = 0;
        SNPMI_HIP(hipMemcpyAsync(&sum, ss, 8, hipMemcpyDeviceToHost, d.stream));
        SNPMI_HIP(hipStreamSynchronize(d.stream));
        const double f = rows / sum;
        if (factor) *factor = f;
        if (!(std::fabs(f - 1.0) > 1e-15)) return;
        s = std::sqrt(f);
    }
    launch_dense_scale(dv, count, DT<T>::v, s, d.stream);
    if (dev) SNPMI_HIP(hipStreamSynchronize(d.stream));
    else d2h_bytes(d, val, dv, count * sizeof(T), resolve_threads(0));
}

// Z Z^T of an already standardized dense block (rows = iids, cols = SNPs, F or C) added to the
// session's tiles: the generic SnpReader._read_kernel block loop (snpreader.py:651-655) for
// readers/standardizers the fused BED path does not cover, with K kept in HBM.
template <typename T>
static void grm_add_dense_impl(const T* val, uint64_t rows, uint64_t cols, int order_c) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    SNPMI_REQUIRE(g_session.active, SNPMI_E_ARG, "no GRM session (call snpmi_grm_begin)");
    SNPMI_REQUIRE(g_session.dtype == DT<T>::v, SNPMI_E_ARG, "dtype differs from snpmi_grm_begin");
    SNPMI_REQUIRE(rows == g_session.n, SNPMI_E_ARG, "iid count differs from snpmi_grm_begin");
    SNPMI_REQUIRE(val != nullptr || rows == 0 || cols == 0, SNPMI_E_ARG, "val is NULL");
    if (rows == 0 || cols == 0) return;
    Device& d = device();
    T* tiles = (T*)session_tiles(d);
    const uint64_t ldz = round_up(rows, 256);
    T* Z = (T*)d.get(Device::S_DENSE, ldz * cols * sizeof(T));
    if (!order_c) {
        SNPMI_HIP(hipMemcpy2DAsync(Z, ldz * sizeof(T), val, rows * sizeof(T), rows * sizeof(T), cols,
                                   hipMemcpyDefault, d.stream));  // host or device val
    } else if (is_device_ptr(d, val)) {
        launch_transpose_to_f(val, rows, cols, DT<T>::v, Z, ldz, d.stream);
    } else {
        T* Zc = (T*)d.get(Device::S_DENSE2, rows * cols * sizeof(T));
        SNPMI_HIP(hipMemcpyAsync(Zc, val, rows * cols * sizeof(T), hipMemcpyHostToDevice, d.stream));
        launch_transpose_to_f(Zc, rows, cols, DT<T>::v, Z, ldz, d.stream);
    }
    syrk_dense_auto(d, Z, ldz, rows, cols, DT<T>::v, tiles, g_session.wrote ? 1 : 0);
    g_session.wrote = true;
    SNPMI_HIP(hipStreamSynchronize(d.stream));
}

// Packed SNP columns already in HBM ([m][pitch] bytes, every iid of the session) added to the
// session: per chunk of <= 2^16 SNPs one stats launch (LUT) and one SYRK launch, so a rank's
// whole SNP shard accumulates in registers over up to 65536 SNPs per K-tile round trip instead
// of one per 10k block (the reference's block_size bounds host memory, snpreader.py:651).
// stats may be host memory (copied synchronously) or device memory (the call then only enqueues).
template <typename T>
static void grm_add_packed_impl(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, int count_a1,
                                int std_kind, double a, double b, int use_stats, T* stats) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    SNPMI_REQUIRE(g_session.active, SNPMI_E_ARG, "no GRM session (call snpmi_grm_begin)");
    SNPMI_REQUIRE(g_session.dtype == DT<T>::v, SNPMI_E_ARG, "dtype differs from snpmi_grm_begin");
    SNPMI_REQUIRE(n == g_session.n, SNPMI_E_ARG, "iid count differs from snpmi_grm_begin");
    SNPMI_REQUIRE(pitch % 64 == 0 && pitch >= ceil_div(n, 4), SNPMI_E_ARG, "pitch must be snpmi_packed_pitch");
    SNPMI_REQUIRE(std_kind >= SNPMI_STD_NONE && std_kind <= SNPMI_STD_BETA, SNPMI_E_ARG, "bad standardizer kind");
    SNPMI_REQUIRE(stats != nullptr || std_kind == SNPMI_STD_NONE || m == 0, SNPMI_E_ARG, "stats is NULL");
    if (m == 0 || n == 0) return;
    SNPMI_REQUIRE(packed != nullptr, SNPMI_E_ARG, "packed is NULL");
    Device& d = device();
    SNPMI_REQUIRE(is_device_ptr(d, packed), SNPMI_E_ARG, "packed must be device memory of the current device");
    T* tiles = (T*)session_tiles(d);
    const bool host_stats = stats && std_kind != SNPMI_STD_NONE && !is_device_ptr(d, stats);
    // equal chunks of <= 2^16 SNPs (the int32 / CRT accumulation cap), multiples of 256
    const uint64_t nchunk = ceil_div(m, 1ull << 16);
    const uint64_t step = std::min<uint64_t>(1ull << 16, round_up(ceil_div(m, nchunk), 256));
    for (uint64_t s0 = 0; s0 < m; s0 += step) {
        const uint64_t cnt = std::min(step, m - s0);
        const uint8_t* src = packed + s0 * pitch;
        T* lut = (T*)d.get(Device::S_LUT, cnt * 4 * sizeof(T));
        T* st = (stats && !host_stats) ? stats + 2 * s0 : (T*)d.get(Device::S_STATS, cnt * 2 * sizeof(T));
        if (host_stats && use_stats)
            SNPMI_HIP(hipMemcpyAsync(st, stats + 2 * s0, cnt * 2 * sizeof(T), hipMemcpyHostToDevice, d.stream));
        launch_snp_stats(src, pitch, n, cnt, count_a1, std_kind, a, b, use_stats, DT<T>::v, st, lut, d.stream);
        syrk_packed_auto(d, src, pitch, n, cnt, lut, DT<T>::v, tiles, g_session.wrote ? 1 : 0);
        g_session.wrote = true;
        if (host_stats && !use_stats) {
            SNPMI_HIP(hipMemcpyAsync(stats + 2 * s0, st, cnt * 2 * sizeof(T), hipMemcpyDeviceToHost, d.stream));
            SNPMI_HIP(hipStreamSynchronize(d.stream));  // S_STATS is reused by the next chunk
        }
    }
    if (host_stats) SNPMI_HIP(hipStreamSynchronize(d.stream));
}
// Column groups of the upper triangle for an overlapped collective: ranges [L0, L1) of 256-block
// indices covering whole supertile columns (16 block columns).  The last group holds ~1/4 of the
// blocks (its sum is the exposed tail), the others split the first ~3/4 evenly; every group
// boundary costs about one round of workgroups (~4 ms at 50k iids, profiles/r04l), so the bench
// uses 2 groups.
struct ColGroup {
    uint64_t L0, L1;  // 256-block index range (supertile table and triangular order alike)
    uint64_t c0, c1;  // block columns [c0, c1)
};
static std::vector<ColGroup> column_groups(uint64_t nb, int parts) {
    const uint64_t ns = ceil_div(nb, 16);
    auto B = [&](uint64_t c) { c = std::min(c, nb); return c * (c + 1) / 2; };
    const uint64_t P = (uint64_t)std::max<int64_t>(1, std::min<int64_t>(parts, (int64_t)ns));
    std::vector<ColGroup> out;
    uint64_t J = 0;
    for (uint64_t p = 0; p < P && J < ns; p++) {
        const uint64_t target = p + 1 == P ? B(nb) : (uint64_t)((double)B(nb) * 0.75 * (double)(p + 1) / (double)(P - 1));
        uint64_t J1 = J + 1;
        while (J1 < ns && B(16 * J1) < target) J1++;
        if (p + 1 == P) J1 = ns;
        out.push_back({B(16 * J), B(16 * J1), std::min(16 * J, nb), std::min(16 * J1, nb)});
        J = J1;
    }
    return out;
}

// snpmi_grm_add_packed_f32 followed by the K-tile collective (collective 1 = ncclReduce onto
// root, 2 = ncclAllReduce, 0 = none), overlapped: the last SNP chunk's SYRK runs as `parts` column
// groups of the triangle (launch_syrk_packed_h2_cols, the same K bit for bit), and as soon as a
// group's SYRK and diagonal write-back are done its contiguous range of tiles is summed over the
// ranks on the aux stream while the next group's SYRK runs.  The compute stream waits for the last
// sum before the call returns, so later work sees the combined K.  Paths without column groups
// (split-K grids, the tuning variants, the f32 MFMA fallbacks) run the SYRK whole and sum after it.
// syrk_done (optional hipEvent_t) is recorded on the compute stream after the last group's SYRK.
static int g_last_groups = 0;  // column groups of the last overlapped collective (read-only hook "overlap_groups")

// Events of one overlapped collective: compute-stream events the aux stream waits on before each
// group's sum, then one aux event the compute stream waits on; destroyed at the end.
// The RCCL calls of the last K-tile collective (read-only hooks "overlap_calls" / "overlap_sig":
// their number and a hash of their element ranges -- tests check every rank issues the same ones)
static int g_last_sum_calls = 0;
static uint64_t g_last_sum_sig = 0;

struct OverlapSums {
    Device& d;
    int collective, root, dtype;
    std::vector<hipEvent_t> evs;
    OverlapSums(Device& dev, int coll, int rt, int dt) : d(dev), collective(coll), root(rt), dtype(dt) {
        g_last_sum_calls = 0;
        g_last_sum_sig = 1469598103934665603ull;
    }
    ~OverlapSums() {
        for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    }
    hipEvent_t event() {
        hipEvent_t e;
        SNPMI_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        evs.push_back(e);
        return e;
    }
    // the tiles of 128-tile columns [t0, t1) are final on the compute stream: sum them on aux
    void range(void* tiles, uint64_t n, uint64_t t0, uint64_t t1) {
        if (!collective) return;
        const uint64_t nt = n_tiles_1d(n);
        auto T = [&](uint64_t t) { t = std::min(t, nt); return t * (t + 1) / 2 * (uint64_t)(kTile * kTile); };
        const uint64_t e0 = T(t0), e1 = T(t1);
        if (e1 <= e0) return;
        g_last_sum_calls++;
        g_last_sum_sig = (g_last_sum_sig ^ (e0 * 0x9E3779B97F4A7C15ull + e1)) * 1099511628211ull;
        hipEvent_t e = event();
        SNPMI_HIP(hipEventRecord(e, d.stream));
        SNPMI_HIP(hipStreamWaitEvent(d.aux, e, 0));
        rccl_sum_on((uint8_t*)tiles + e0 * dtype_size(dtype), e1 - e0, dtype, root, d.aux);
    }
    void join() {
        if (!collective) return;
        hipEvent_t e = event();
        SNPMI_HIP(hipEventRecord(e, d.aux));
        SNPMI_HIP(hipStreamWaitEvent(d.stream, e, 0));
    }
};

// Whether the last SYRK of an f32 GRM can run as column groups (launch_syrk_packed_h2_cols) --
// decided from state every rank shares (n, parts, the kernel configuration), never from the rank's
// own SNP count: ranks whose spans differ by a SNP, or that own none, must issue the same RCCL
// calls.  The split-K check uses the largest chunk: a chunk of fewer SNPs only narrows
// the slice counts bf3_split_slices may choose, so "no split at 65536" holds for every chunk.
static bool f32_groupable(Device& d, uint64_t n, int parts) {
    return n > 0 && use_bf3(SNPMI_DT_F32) && use_h2() && g_diag_exact && parts > 1 &&
           bf3_split_slices(n, 1ull << 16, d.cu_count) == 1 && ceil_div(n, 256) < 65536;
}

static uint64_t crt_res_bytes(uint64_t n) {
    const uint64_t nb = ceil_div(n, 256);
    return std::min<uint64_t>(nb * (nb + 1) / 2 * (uint64_t)crt_moduli() * 65536, 4ull << 30);
}

// The K-tile collective of one session as RCCL calls: 128-tile column ranges [t0, t1) of the
// triangle, each one in-place sum.  f32: the column groups of the overlapped SYRK; f64 on the CRT
// path: its column-aligned residue chunks; otherwise one range over the whole triangle.  Every path
// that sums a session's tiles (overlapped or not, with or without SNPs on this rank) issues exactly
// these calls, in this order.
struct SumPlan {
    std::vector<std::pair<uint64_t, uint64_t>> ranges;
    bool grouped = false;  // the ranges are the overlapped SYRK's groups
};
static SumPlan sum_plan(Device& d, uint64_t n, int dtype, int parts) {
    SumPlan p;
    if (dtype == SNPMI_DT_F32 && f32_groupable(d, n, parts)) {
        for (const auto& g : column_groups(ceil_div(n, 256), parts)) p.ranges.push_back({2 * g.c0, 2 * g.c1});
        p.grouped = true;
    } else if (dtype == SNPMI_DT_F64 && use_crt(SNPMI_DT_F64) && n > 0) {
        for (const auto& c : crt_column_chunks(n, crt_res_bytes(n))) p.ranges.push_back({2 * c.first, 2 * c.second});
        p.grouped = true;
    } else {
        p.ranges.push_back({0, n_tiles_1d(n)});
    }
    return p;
}

// The plan's sums after everything enqueued so far on the compute stream (aux stream, then the
// compute stream waits for the last one)
static void sum_by_plan(Device& d, const SumPlan& p, void* tiles, uint64_t n, int collective, int rt, int dtype) {
    OverlapSums sums(d, collective, rt, dtype);
    for (const auto& r : p.ranges) sums.range(tiles, n, r.first, r.second);
    sums.join();
}

// The overlapped last SYRK of an f32 GRM: `cnt` SNPs (device codes + f32 LUT) added into `tiles`
// in column groups (launch_syrk_packed_h2_cols, K bit-identical to one launch) with the exact
// diagonal written back per group, each group's tiles summed over the ranks on the aux stream
// under the next group's SYRK.  Returns the group count.
static int grouped_reduce_f32(Device& d, const uint8_t* src, uint64_t pitch, uint64_t n, uint64_t cnt,
                              const float* lut, float* tiles, int acc, int collective, int rt, int parts,
                              hipEvent_t syrk_done) {
    H2Lut h2;
    const uint32_t* l3 = lut_bf3(d, lut, cnt, &h2);
    double* diag = (double*)d.get(Device::S_DIAG, diag_scratch_bytes(n, cnt));
    launch_diag_begin(tiles, n, nullptr, acc, diag, d.stream);
    launch_diag_sq(src, pitch, n, cnt, lut, diag, d.stream);
    const auto groups = column_groups(ceil_div(n, 256), parts);
    OverlapSums sums(d, collective, rt, SNPMI_DT_F32);
    for (const auto& gr : groups) {
        launch_syrk_packed_h2_cols(src, pitch, n, cnt, l3, tiles, acc, d.stream, &h2, gr.L0, gr.L1);
        // block columns [c0, c1): diagonal iids [256 c0, 256 c1), 128-tile columns [2 c0, 2 c1)
        launch_diag_patch(tiles, n, 256 * gr.c0, 256 * gr.c1, nullptr, diag, d.stream);
        sums.range(tiles, n, 2 * gr.c0, 2 * gr.c1);
    }
    if (syrk_done) SNPMI_HIP(hipEventRecord(syrk_done, d.stream));
    sums.join();
    return (int)groups.size();
}

// f64 counterpart: the groups are the CRT path's residue chunks of the last <= crt_max_snps() SNPs
// (launch_syrk_packed_crt cuts them at block-column boundaries when given after_chunk; ~5 at 50k
// iids, so no extra launch boundary), each chunk's f64 tiles summed on the aux stream once its
// CRT reconstruction is done.  The f64-MFMA fallback of a non-finite LUT (gated on the device
// flag) runs before the chunks, so every sum sees final tiles.
static int crt_reduce_f64(Device& d, const uint8_t* src, uint64_t pitch, uint64_t n, uint64_t cnt, const double* lut,
                          double* tiles, int acc, int collective, int rt, hipEvent_t syrk_done) {
    const uint64_t step = crt_max_snps();
    if (cnt > step) {  // the leading SNPs the plain way, the last <= step overlapped
        const uint64_t lead = ((cnt - 1) / step) * step;
        syrk_packed_crt(d, src, pitch, n, lead, lut, tiles, acc);
        src += lead * pitch;
        lut += 4 * lead;
        cnt -= lead;
        acc = 1;
    }
    const uint64_t res_bytes = crt_res_bytes(n);
    uint8_t* res = (uint8_t*)d.get(Device::S_ZBLK, res_bytes);
    void* ws = d.get(Device::S_LUT3, crt_lut_bytes(cnt, n));
    unsigned long long* rec = crt_record(d);
    const SumPlan plan = sum_plan(d, n, SNPMI_DT_F64, 1);
    OverlapSums sums(d, collective, rt, SNPMI_DT_F64);
    size_t groups = 0;
    const std::function<void()> pre = [&] {
        launch_syrk_packed_f64_gated(src, pitch, n, cnt, lut, tiles, acc, (const int*)ws + 1, d.stream);
    };
    const std::function<void(uint64_t, uint64_t)> after = [&](uint64_t c0, uint64_t c1) {
        SNPMI_REQUIRE(groups < plan.ranges.size() && plan.ranges[groups] == std::make_pair(2 * c0, 2 * c1),
                      SNPMI_E_ARG, "CRT chunks differ from the collective plan");
        groups++;
        sums.range(tiles, n, 2 * c0, 2 * c1);
    };
    launch_syrk_packed_crt(src, pitch, n, cnt, lut, tiles, acc, ws, res, res_bytes, rec, d.stream, &pre, &after);
    SNPMI_REQUIRE(groups == plan.ranges.size(), SNPMI_E_ARG, "CRT chunks differ from the collective plan");
    if (syrk_done) SNPMI_HIP(hipEventRecord(syrk_done, d.stream));
    sums.join();
    return (int)groups;
}

// the session's collective after an unoverlapped add (or on a rank without SNPs): the same RCCL
// calls as the overlapped path (sum_plan); zeros join the sum if nothing was added
template <typename T>
static void session_sum_planned(Device& d, int collective, int rt, int parts, hipEvent_t syrk_done) {
    T* t = (T*)session_tiles(d);
    const uint64_t count = n_tiles_upper(g_session.n) * kTile * kTile;
    if (!g_session.wrote) {
        SNPMI_HIP(hipMemsetAsync(t, 0, count * sizeof(T), d.stream));
        g_session.wrote = true;
    }
    if (syrk_done) SNPMI_HIP(hipEventRecord(syrk_done, d.stream));
    if (collective) sum_by_plan(d, sum_plan(d, g_session.n, DT<T>::v, parts), t, g_session.n, collective, rt, DT<T>::v);
}

template <typename T>
static void check_reduce_args(int collective, int parts) {
    SNPMI_REQUIRE(g_session.active, SNPMI_E_ARG, "no GRM session (call snpmi_grm_begin)");
    SNPMI_REQUIRE(g_session.dtype == DT<T>::v, SNPMI_E_ARG, "dtype differs from snpmi_grm_begin");
    SNPMI_REQUIRE(collective >= 0 && collective <= 2, SNPMI_E_ARG, "collective must be 0 (none), 1 (reduce), 2 (all-reduce)");
    SNPMI_REQUIRE(collective == 0 || rccl_ready(), SNPMI_E_ARG, "RCCL communicator not initialised");
    SNPMI_REQUIRE(parts >= 1, SNPMI_E_ARG, "parts must be >= 1");
}

// snpmi_grm_add_packed_{f32,f64} (the session's last add) + the K-tile collective, overlapped:
// the last SNP chunk (same chunking as grm_add_packed_impl) runs through grouped_reduce_f32 /
// crt_reduce_f64.  Host stats, or a path without groups, add first and sum after.
template <typename T>
static void grm_add_packed_reduce_impl(const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t m, int count_a1,
                                       int std_kind, double a, double b, int use_stats, T* stats, int collective,
                                       int root, int parts, hipEvent_t syrk_done) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    check_reduce_args<T>(collective, parts);
    Device& d = device();
    const int rt = collective == 1 ? root : -1;
    const bool f64 = DT<T>::v == SNPMI_DT_F64;
    const uint64_t nchunk = m ? ceil_div(m, 1ull << 16) : 1;
    const uint64_t step = std::min<uint64_t>(1ull << 16, round_up(ceil_div(m, nchunk), 256));
    (void)f64;
    const bool grouped = m > 0 && n > 0 && n == g_session.n && sum_plan(d, n, DT<T>::v, parts).grouped &&
                         (std_kind == SNPMI_STD_NONE || (stats && is_device_ptr(d, stats)));
    g_last_groups = 1;
    if (!grouped) {
        grm_add_packed_impl<T>(packed, pitch, n, m, count_a1, std_kind, a, b, use_stats, stats);
        session_sum_planned<T>(d, collective, rt, parts, syrk_done);
        return;
    }
    SNPMI_REQUIRE(pitch % 64 == 0 && pitch >= ceil_div(n, 4), SNPMI_E_ARG, "pitch must be snpmi_packed_pitch");
    SNPMI_REQUIRE(std_kind >= SNPMI_STD_NONE && std_kind <= SNPMI_STD_BETA, SNPMI_E_ARG, "bad standardizer kind");
    SNPMI_REQUIRE(packed != nullptr && is_device_ptr(d, packed), SNPMI_E_ARG,
                  "packed must be device memory of the current device");
    const uint64_t s_last = ((m - 1) / step) * step;
    if (s_last > 0) grm_add_packed_impl<T>(packed, pitch, n, s_last, count_a1, std_kind, a, b, use_stats, stats);
    T* tiles = (T*)session_tiles(d);
    const int acc = g_session.wrote ? 1 : 0;
    const uint64_t cnt = m - s_last;
    const uint8_t* src = packed + s_last * pitch;
    T* lut = (T*)d.get(Device::S_LUT, cnt * 4 * sizeof(T));
    launch_snp_stats(src, pitch, n, cnt, count_a1, std_kind, a, b, use_stats, DT<T>::v,
                     stats ? stats + 2 * s_last : (T*)d.get(Device::S_STATS, cnt * 2 * sizeof(T)), lut, d.stream);
    g_session.wrote = true;
    if constexpr (std::is_same<T, double>::value)
        g_last_groups = crt_reduce_f64(d, src, pitch, n, cnt, lut, tiles, acc, collective, rt, syrk_done);
    else
        g_last_groups = grouped_reduce_f32(d, src, pitch, n, cnt, lut, tiles, acc, collective, rt, parts, syrk_done);
}

// snpmi_grm_add_bed_{f32,f64} (the session's last add: a rank's SNP span of a .bed) + the K-tile
// collective, overlapped the same way on the file stream's last chunk.
template <typename T>
static void grm_add_bed_reduce_impl(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,
                                    const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,
                                    uint64_t n_out_sid, int std_kind, double a, double b, int use_stats, T* stats,
                                    int num_threads, int collective, int root, int parts) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    check_reduce_args<T>(collective, parts);
    SNPMI_REQUIRE((iid_idx ? n_out_iid : n_iid) == g_session.n, SNPMI_E_ARG, "iid count differs from snpmi_grm_begin");
    Device& d = device();
    const int rt = collective == 1 ? root : -1;
    const uint64_t n = g_session.n, total = sid_idx ? n_out_sid : n_sid;
    T* tiles = (T*)session_tiles(d);
    uint64_t done = 0;
    int groups = 1;
    const SumPlan plan = sum_plan(d, n, DT<T>::v, parts);
    const bool wrote = grm_stream_bed<T>(
        d, !g_session.wrote, path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid, std_kind, a, b,
        use_stats, stats, num_threads,
        [&](const uint8_t* packed, uint64_t pitch, uint64_t nn, uint64_t cnt, const T* lut, bool acc) {
            done += cnt;
            const bool last = done == total;
            if (last && plan.grouped) {
                if constexpr (std::is_same<T, double>::value)
                    groups = crt_reduce_f64(d, packed, pitch, nn, cnt, lut, tiles, acc, collective, rt, nullptr);
                else
                    groups = grouped_reduce_f32(d, packed, pitch, nn, cnt, lut, tiles, acc, collective, rt, parts,
                                                nullptr);
                return;
            }
            syrk_packed_auto(d, packed, pitch, nn, cnt, lut, DT<T>::v, tiles, acc);
            if (last && collective) sum_by_plan(d, plan, tiles, n, collective, rt, DT<T>::v);
        });
    g_last_groups = groups;
    if (wrote && done == total) {
        g_session.wrote = true;
        return;  // the last chunk summed the tiles
    }
    session_sum_planned<T>(d, collective, rt, parts, nullptr);  // no SNP on this rank: zeros join the sum
}
}  // namespace snpmi

// ====================================================================== exported C ABI
using namespace snpmi;

extern "C" {

const char* snpmi_last_error(void) { return g_last_error.c_str(); }
int snpmi_version(void) { return 1; }

int snpmi_device_count(int* count) {
    return guarded([&] {
        SNPMI_REQUIRE(count != nullptr, SNPMI_E_ARG, "count is NULL");
        *count = num_devices();
        (void)hipGetLastError();
    });
}

int snpmi_set_device(int dev) {
    return guarded([&] {
        SNPMI_REQUIRE(dev >= 0 && dev < num_devices(), SNPMI_E_ARG, "device index out of range");
        g_cur_dev = dev;
        (void)device();
    });
}

int snpmi_get_device(int* dev) {
    return guarded([&] {
        SNPMI_REQUIRE(dev != nullptr, SNPMI_E_ARG, "dev is NULL");
        *dev = g_cur_dev < 0 ? default_device() : g_cur_dev;
    });
}

int snpmi_release_cache(void) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
        std::lock_guard<std::mutex> lk2(g_dev_mutex);
        for (Device* d : g_devices)
            if (d) {
                SNPMI_HIP(hipSetDevice(d->id));
                SNPMI_HIP(hipStreamSynchronize(d->stream));
                d->release();
            }
        release_pinned();
    });
}

int snpmi_device_info(int dev, char* name, size_t name_len, uint64_t* total_mem, int* cu_count) {
    return guarded([&] {
        hipDeviceProp_t p;
        SNPMI_HIP(hipGetDeviceProperties(&p, dev));
        if (name && name_len) {
            std::strncpy(name, p.gcnArchName, name_len - 1);
            name[name_len - 1] = 0;
        }
        if (total_mem) *total_mem = p.totalGlobalMem;
        if (cu_count) *cu_count = p.multiProcessorCount;
    });
}

int snpmi_device_ids(int dev, uint8_t* uuid16, int* pci, int* clock_khz) {
    return guarded([&] {
        hipDeviceProp_t p;
        SNPMI_HIP(hipGetDeviceProperties(&p, dev));
        if (uuid16) std::memcpy(uuid16, p.uuid.bytes, 16);
        if (pci) {
            pci[0] = p.pciDomainID;
            pci[1] = p.pciBusID;
            pci[2] = p.pciDeviceID;
        }
        if (clock_khz) *clock_khz = p.clockRate;
    });
}

int snpmi_set_kernel_variant(const char* kernel, int variant) {
    return guarded([&] {
        SNPMI_REQUIRE(kernel != nullptr, SNPMI_E_ARG, "kernel name is NULL");
        if (std::strcmp(kernel, "decode") == 0) g_variant_decode = variant;
        else if (std::strcmp(kernel, "std") == 0) g_variant_std = variant;
        else if (std::strcmp(kernel, "diag") == 0) g_diag_exact = variant != 0;
        else if (std::strcmp(kernel, "extract") == 0) g_variant_extract = variant;
        else if (std::strcmp(kernel, "syrk") == 0) {
            // the shipped default chain and the kernels it falls back to: 36 = the bf16x3 kernel
            // alone (fp16x2 range fallback), 20 = the f32-MFMA kernels (dense-operand range
            // fallback), 5 = the 128x128 small-N kernels, 71 = f64 GRMs on the f64 MFMA (the CRT
            // path's non-finite fallback).  The A/B ablations of earlier rounds were deleted (round 6);
            // the shipped forms' own A/B switches are the hooks "h2" and "crt".
            SNPMI_REQUIRE(variant == 0 || variant == 5 || variant == 20 || variant == 36 || variant == 71, SNPMI_E_ARG,
                          "syrk variant " + std::to_string(variant) + " is not a shipped kernel (0, 5, 20, 36, 71)");
            g_variant_syrk = variant;
        }
        else if (std::strcmp(kernel, "syrk_split") == 0) g_variant_syrk_split = variant;
        else if (std::strcmp(kernel, "dense_chunk") == 0) g_dense_chunk = std::max(variant, 0);
        else if (std::strcmp(kernel, "dense_codes") == 0) g_dense_codes = variant;
        else if (std::strcmp(kernel, "seg") == 0) g_seg_snps = std::max(variant, 0);
        else if (std::strcmp(kernel, "gather") == 0) g_gather = variant;  // host gather A/B (0 mmap, 1 pread)
        else if (std::strcmp(kernel, "h2") == 0) {
            SNPMI_REQUIRE(variant == 0 || variant == 1, SNPMI_E_ARG, "h2 SYRK: 0 = k_syrk_h2, 1 = k_syrk_h2s");
            g_h2_kernel = variant;
        }
        else if (std::strcmp(kernel, "crt") == 0) {
            SNPMI_REQUIRE(variant >= 0 && variant <= 2, SNPMI_E_ARG,
                          "crt residue SYRK: 0 = k_syrk_i8r, 1 = k_syrk_i8w, 2 = k_syrk_i8w without its read "
                          "order / wave priorities");
            g_crt_kernel = variant;
        }
        else if (std::strcmp(kernel, "crt_block") == 0) {
            SNPMI_REQUIRE(variant == 0 || variant == 1, SNPMI_E_ARG, "crt moduli: 0 = launch-wide R, 1 = per 256-block");
            g_crt_block = variant;
        }
        else if (std::strcmp(kernel, "f64") == 0) {
            SNPMI_REQUIRE(variant == 0 || variant == 1, SNPMI_E_ARG, "f64 GRM path: 0 = int8 residues + CRT, 1 = f64 MFMA");
            g_f64_mfma = variant;
        }
        else throw Error(SNPMI_E_ARG, std::string("unknown kernel ") + kernel);
    });
}

int snpmi_get_kernel_variant(const char* kernel, int* variant) {
    return guarded([&] {
        SNPMI_REQUIRE(kernel != nullptr && variant != nullptr, SNPMI_E_ARG, "kernel name or output is NULL");
        if (std::strcmp(kernel, "decode") == 0) *variant = g_variant_decode;
        else if (std::strcmp(kernel, "std") == 0) *variant = g_variant_std;
        else if (std::strcmp(kernel, "diag") == 0) *variant = g_diag_exact;
        else if (std::strcmp(kernel, "overlap_groups") == 0) *variant = g_last_groups;
        else if (std::strcmp(kernel, "overlap_calls") == 0) *variant = g_last_sum_calls;
        else if (std::strcmp(kernel, "overlap_sig") == 0) *variant = (int)(g_last_sum_sig & 0x7fffffff);
        else if (std::strcmp(kernel, "extract") == 0) *variant = g_variant_extract;
        else if (std::strcmp(kernel, "syrk") == 0) *variant = g_variant_syrk;
        else if (std::strcmp(kernel, "syrk_split") == 0) *variant = g_variant_syrk_split;
        else if (std::strcmp(kernel, "dense_chunk") == 0) *variant = g_dense_chunk;
        else if (std::strcmp(kernel, "dense_codes") == 0) *variant = g_dense_codes;
        else if (std::strcmp(kernel, "seg") == 0) *variant = g_seg_snps;
        else if (std::strcmp(kernel, "gather") == 0) *variant = g_gather;
        else if (std::strcmp(kernel, "crt") == 0) *variant = g_crt_kernel;
        else if (std::strcmp(kernel, "crt_block") == 0) *variant = g_crt_block;
        else if (std::strcmp(kernel, "h2") == 0) *variant = g_h2_kernel;
        else if (std::strcmp(kernel, "f64") == 0) *variant = g_f64_mfma;
        else throw Error(SNPMI_E_ARG, std::string("unknown kernel ") + kernel);
    });
}

int snpmi_bed_check(const char* path, uint64_t n_iid, uint64_t n_sid) {
    return guarded([&] {
        BedMap m;
        open_bed(m, path, n_iid, n_sid);
    });
}

#define SNPMI_BED_READ(SUFFIX, T)                                                                                  \
    int snpmi_bed_read_##SUFFIX(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,                  \
                                const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,             \
                                uint64_t n_out_sid, int order_c, T* out, int num_threads) {                       \
        return guarded([&] {                                                                                       \
            bed_read_impl<T>(path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid, order_c,       \
                             SNPMI_STD_NONE, 0.0, 0.0, 0, (T*)nullptr, out, num_threads);                         \
        });                                                                                                        \
    }
SNPMI_BED_READ(f32, float)
SNPMI_BED_READ(f64, double)
SNPMI_BED_READ(i8, int8_t)

#define SNPMI_BED_READ_STD(SUFFIX, T)                                                                              \
    int snpmi_bed_read_standardize_##SUFFIX(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,      \
                                            const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx, \
                                            uint64_t n_out_sid, int order_c, int std_kind, double a, double b,    \
                                            int use_stats, T* stats, T* out, int num_threads) {                   \
        return guarded([&] {                                                                                       \
            SNPMI_REQUIRE(std_kind == SNPMI_STD_NONE || stats != nullptr, SNPMI_E_ARG, "stats is NULL");          \
            bed_read_impl<T>(path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid, order_c,       \
                             std_kind, a, b, use_stats, stats, out, num_threads);                                 \
        });                                                                                                        \
    }
SNPMI_BED_READ_STD(f32, float)
SNPMI_BED_READ_STD(f64, double)

#define SNPMI_BED_WRITE(SUFFIX, T)                                                                                 \
    int snpmi_bed_write_##SUFFIX(const char* path, const T* val, uint64_t n_iid, uint64_t n_sid, int order_c,    \
                                 int count_a1, int) {                                                               \
        return guarded([&] { bed_write_impl<T>(path, val, n_iid, n_sid, order_c, count_a1); });                   \
    }
SNPMI_BED_WRITE(f32, float)
SNPMI_BED_WRITE(f64, double)
SNPMI_BED_WRITE(i8, int8_t)

int snpmi_dev_encode(const void* val, int dtype, int order_c, uint64_t ld, uint64_t n_iid, uint64_t n_sid,
                     int count_a1, uint8_t* packed, uint64_t pitch, uint64_t* bad_values) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);  // shared scratch slots
        SNPMI_REQUIRE(pitch % 64 == 0 && pitch >= ceil_div(n_iid, 4), SNPMI_E_ARG, "pitch must be a multiple of 64 >= ceil(n/4)");
        SNPMI_REQUIRE(order_c || ld % 16 == 0, SNPMI_E_ARG, "F-order ld must be a multiple of 16");
        SNPMI_REQUIRE(order_c ? ld >= n_sid : ld >= n_iid, SNPMI_E_ARG, "ld too small");
        Device& d = device();
        unsigned int* bad_dev = (unsigned int*)d.get(Device::S_RED, 256);
        SNPMI_HIP(hipMemsetAsync(bad_dev, 0, sizeof(unsigned int), d.stream));
        launch_encode(val, dtype, order_c, ld, n_iid, n_sid, count_a1, packed, pitch, bad_dev, d.stream);
        if (bad_values) {
            unsigned int bad = 0;
            SNPMI_HIP(hipMemcpyAsync(&bad, bad_dev, sizeof(bad), hipMemcpyDeviceToHost, d.stream));
            SNPMI_HIP(hipStreamSynchronize(d.stream));
            *bad_values = bad;
        }
    });
}

int snpmi_grm_begin(uint64_t n_out_iid, int dtype) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
        SNPMI_REQUIRE(dtype == SNPMI_DT_F32 || dtype == SNPMI_DT_F64, SNPMI_E_ARG, "GRM dtype must be f32 or f64");
        Device& d = device();
        g_session = GrmSession{true, false, n_out_iid, dtype};
        (void)session_tiles(d);
    });
}

#define SNPMI_GRM_ADD(SUFFIX, T, DTV)                                                                               \
    int snpmi_grm_add_bed_##SUFFIX(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,                 \
                                   const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,            \
                                   uint64_t n_out_sid, int std_kind, double a, double b, int use_stats, T* stats,   \
                                   int num_threads) {                                                                \
        return guarded([&] {                                                                                         \
            std::lock_guard<std::recursive_mutex> lk(g_call_mutex);                                                  \
            SNPMI_REQUIRE(g_session.active, SNPMI_E_ARG, "no GRM session (call snpmi_grm_begin)");                  \
            SNPMI_REQUIRE(g_session.dtype == DTV, SNPMI_E_ARG, "dtype differs from snpmi_grm_begin");               \
            SNPMI_REQUIRE((iid_idx ? n_out_iid : n_iid) == g_session.n, SNPMI_E_ARG,                                \
                          "iid count differs from snpmi_grm_begin");                                                 \
            Device& d = device();                                                                                    \
            T* tiles = (T*)session_tiles(d);                                                                         \
            if (grm_add_bed<T>(d, tiles, !g_session.wrote, path, n_iid, n_sid, count_a1, iid_idx, n_out_iid,        \
                               sid_idx, n_out_sid, std_kind, a, b, use_stats, stats, num_threads))                   \
                g_session.wrote = true;                                                                              \
        });                                                                                                          \
    }
SNPMI_GRM_ADD(f32, float, SNPMI_DT_F32)
SNPMI_GRM_ADD(f64, double, SNPMI_DT_F64)

int snpmi_grm_add_packed_f32(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, int count_a1,
                             int std_kind, double a, double b, int use_stats, float* stats) {
    return guarded([&] { grm_add_packed_impl<float>(packed, pitch, n_iid, n_sid, count_a1, std_kind, a, b, use_stats, stats); });
}
int snpmi_grm_add_packed_f64(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, int count_a1,
                             int std_kind, double a, double b, int use_stats, double* stats) {
    return guarded([&] { grm_add_packed_impl<double>(packed, pitch, n_iid, n_sid, count_a1, std_kind, a, b, use_stats, stats); });
}

int snpmi_grm_add_packed_reduce_f32(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                                    int count_a1, int std_kind, double a, double b, int use_stats, float* stats,
                                    int collective, int root, int parts, void* syrk_done) {
    return guarded([&] {
        grm_add_packed_reduce_impl<float>(packed, pitch, n_iid, n_sid, count_a1, std_kind, a, b, use_stats, stats,
                                          collective, root, parts, (hipEvent_t)syrk_done);
    });
}

int snpmi_grm_add_packed_reduce_f64(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                                    int count_a1, int std_kind, double a, double b, int use_stats, double* stats,
                                    int collective, int root, int parts, void* syrk_done) {
    // parts: the CRT path's own residue chunks are the groups
    return guarded([&] {
        grm_add_packed_reduce_impl<double>(packed, pitch, n_iid, n_sid, count_a1, std_kind, a, b, use_stats, stats,
                                           collective, root, std::max(parts, 1), (hipEvent_t)syrk_done);
    });
}

int snpmi_grm_add_bed_reduce_f32(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1, const uint64_t* iid_idx,
                                 uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid, int std_kind,
                                 double a, double b, int use_stats, float* stats, int num_threads, int collective,
                                 int root, int parts) {
    return guarded([&] {
        grm_add_bed_reduce_impl<float>(path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid, std_kind,
                                       a, b, use_stats, stats, num_threads, collective, root, parts);
    });
}
int snpmi_grm_add_bed_reduce_f64(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1, const uint64_t* iid_idx,
                                 uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid, int std_kind,
                                 double a, double b, int use_stats, double* stats, int num_threads, int collective,
                                 int root, int parts) {
    return guarded([&] {
        grm_add_bed_reduce_impl<double>(path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid,
                                        std_kind, a, b, use_stats, stats, num_threads, collective, root,
                                        std::max(parts, 1));
    });
}

int snpmi_grm_add_dense_f32(const float* val, uint64_t rows, uint64_t cols, int order_c) {
    return guarded([&] { grm_add_dense_impl<float>(val, rows, cols, order_c); });
}
int snpmi_grm_add_dense_f64(const double* val, uint64_t rows, uint64_t cols, int order_c) {
    return guarded([&] { grm_add_dense_impl<double>(val, rows, cols, order_c); });
}

int snpmi_grm_session_tiles(void** tiles, uint64_t* count) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
        SNPMI_REQUIRE(g_session.active, SNPMI_E_ARG, "no GRM session (call snpmi_grm_begin)");
        Device& d = device();
        void* t = session_tiles(d);
        const uint64_t cnt = n_tiles_upper(g_session.n) * kTile * kTile;
        if (!g_session.wrote) {
            SNPMI_HIP(hipMemsetAsync(t, 0, cnt * dtype_size(g_session.dtype), d.stream));
            SNPMI_HIP(hipStreamSynchronize(d.stream));
            g_session.wrote = true;
        }
        if (tiles) *tiles = t;
        if (count) *count = cnt;
    });
}

int snpmi_grm_session_sum(int collective, int root, int parts) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
        SNPMI_REQUIRE(g_session.active, SNPMI_E_ARG, "no GRM session (call snpmi_grm_begin)");
        Device& d = device();
        const int rt = collective == 1 ? root : -1;
        g_last_groups = 1;
        if (g_session.dtype == SNPMI_DT_F64) {
            check_reduce_args<double>(collective, parts);
            session_sum_planned<double>(d, collective, rt, parts, nullptr);
        } else {
            check_reduce_args<float>(collective, parts);
            session_sum_planned<float>(d, collective, rt, parts, nullptr);
        }
    });
}

int snpmi_grm_end(int diag_k_to_n, double* factor, void* K_out) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
        SNPMI_REQUIRE(g_session.active, SNPMI_E_ARG, "no GRM session (call snpmi_grm_begin)");
        Device& d = device();
        g_session.active = false;
        if (!K_out) {  // end without a result (a non-root rank after an RCCL reduce, an aborted GRM)
            SNPMI_HIP(hipStreamSynchronize(d.stream));
            if (factor) *factor = NAN;
            return;
        }
        void* t = session_tiles(d);
        if (!g_session.wrote)
            SNPMI_HIP(hipMemsetAsync(t, 0, n_tiles_upper(g_session.n) * kTile * kTile * dtype_size(g_session.dtype),
                                     d.stream));
        if (g_session.dtype == SNPMI_DT_F32)
            grm_finish(d, (const float*)t, g_session.n, diag_k_to_n, factor, (float*)K_out);
        else
            grm_finish(d, (const double*)t, g_session.n, diag_k_to_n, factor, (double*)K_out);
    });
}

int snpmi_standardize_f32(float* val, uint64_t rows, uint64_t cols, int order_c, int is_beta, double a, double b,
                          int apply_in_place, int use_stats, float* stats, int) {
    return guarded([&] { standardize_impl<float>(val, rows, cols, order_c, is_beta, a, b, apply_in_place, use_stats, stats); });
}
int snpmi_standardize_f64(double* val, uint64_t rows, uint64_t cols, int order_c, int is_beta, double a, double b,
                          int apply_in_place, int use_stats, double* stats, int) {
    return guarded([&] { standardize_impl<double>(val, rows, cols, order_c, is_beta, a, b, apply_in_place, use_stats, stats); });
}

int snpmi_subset_f64_f64(const double* val, uint64_t rows, uint64_t cols, uint64_t k, int in_c, const uint64_t* ri,
                         uint64_t nr, const uint64_t* ci, uint64_t nc, int out_c, double* out, int) {
    return guarded([&] { subset_impl<double, double>(val, rows, cols, k, in_c, ri, nr, ci, nc, out_c, out); });
}
int snpmi_subset_f32_f64(const float* val, uint64_t rows, uint64_t cols, uint64_t k, int in_c, const uint64_t* ri,
                         uint64_t nr, const uint64_t* ci, uint64_t nc, int out_c, double* out, int) {
    return guarded([&] { subset_impl<float, double>(val, rows, cols, k, in_c, ri, nr, ci, nc, out_c, out); });
}
int snpmi_subset_f32_f32(const float* val, uint64_t rows, uint64_t cols, uint64_t k, int in_c, const uint64_t* ri,
                         uint64_t nr, const uint64_t* ci, uint64_t nc, int out_c, float* out, int) {
    return guarded([&] { subset_impl<float, float>(val, rows, cols, k, in_c, ri, nr, ci, nc, out_c, out); });
}

#define SNPMI_GRM_BED(SUFFIX, T)                                                                                    \
    int snpmi_grm_bed_##SUFFIX(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1,                    \
                               const uint64_t* iid_idx, uint64_t n_out_iid, const uint64_t* sid_idx,              \
                               uint64_t n_out_sid, int std_kind, double a, double b, int use_stats, T* stats,     \
                               int diag, double* factor, T* K_out, int num_threads) {                             \
        return guarded([&] {                                                                                        \
            grm_bed_impl<T>(path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid, std_kind, a, b,  \
                            use_stats, stats, diag, factor, K_out, num_threads);                                   \
        });                                                                                                         \
    }
SNPMI_GRM_BED(f32, float)
SNPMI_GRM_BED(f64, double)

int snpmi_grm_dense_f32(const float* val, uint64_t rows, uint64_t cols, int order_c, int std_kind, double a, double b,
                        int use_stats, float* stats, int diag, double* factor, float* K_out) {
    return guarded([&] { grm_dense_impl<float>(val, rows, cols, order_c, std_kind, a, b, use_stats, stats, diag, factor, K_out); });
}
int snpmi_grm_dense_f64(const double* val, uint64_t rows, uint64_t cols, int order_c, int std_kind, double a,
                        double b, int use_stats, double* stats, int diag, double* factor, double* K_out) {
    return guarded([&] { grm_dense_impl<double>(val, rows, cols, order_c, std_kind, a, b, use_stats, stats, diag, factor, K_out); });
}
int snpmi_diag_k_to_n_snps_f32(float* val, uint64_t rows, uint64_t cols, double* factor) {
    return guarded([&] { snp_scale_impl<float>(val, rows * cols, (double)rows, 0, 1.0, factor); });
}
int snpmi_diag_k_to_n_snps_f64(double* val, uint64_t rows, uint64_t cols, double* factor) {
    return guarded([&] { snp_scale_impl<double>(val, rows * cols, (double)rows, 0, 1.0, factor); });
}
int snpmi_scale_f32(float* val, uint64_t count, double scale) {
    return guarded([&] { snp_scale_impl<float>(val, count, 0.0, 1, scale, nullptr); });
}
int snpmi_scale_f64(double* val, uint64_t count, double scale) {
    return guarded([&] { snp_scale_impl<double>(val, count, 0.0, 1, scale, nullptr); });
}
int snpmi_diag_k_to_n_f32(float* K, uint64_t n, double* factor) {
    return guarded([&] { diag_k_to_n_impl<float>(K, n, factor); });
}
int snpmi_diag_k_to_n_f64(double* K, uint64_t n, double* factor) {
    return guarded([&] { diag_k_to_n_impl<double>(K, n, factor); });
}

// ---------------------------------------------------------------------- device-resident API
uint64_t snpmi_packed_pitch(uint64_t n_iid) { return packed_pitch(n_iid); }
uint64_t snpmi_grm_tile_bytes(uint64_t n_iid, int dtype) {
    return n_tiles_upper(n_iid) * kTile * kTile * dtype_size(dtype);
}

int snpmi_dev_alloc(void** ptr, uint64_t bytes) {
    return guarded([&] {
        SNPMI_REQUIRE(ptr != nullptr, SNPMI_E_ARG, "ptr is NULL");
        (void)device();
        if (hipMalloc(ptr, bytes ? bytes : 256) != hipSuccess) {
            (void)hipGetLastError();
            throw Error(SNPMI_E_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
        }
    });
}
int snpmi_host_alloc(void** ptr, uint64_t bytes) {
    return guarded([&] {
        SNPMI_REQUIRE(ptr != nullptr, SNPMI_E_ARG, "ptr is NULL");
        (void)device();
        if (hipHostMalloc(ptr, bytes ? bytes : 256, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            throw Error(SNPMI_E_NOMEM, "hipHostMalloc of " + std::to_string(bytes) + " bytes failed");
        }
    });
}
int snpmi_host_free(void* ptr) {
    return guarded([&] {
        (void)device();
        SNPMI_HIP(hipHostFree(ptr));
    });
}
int snpmi_dev_free(void* ptr) {
    return guarded([&] {
        (void)device();
        SNPMI_HIP(hipFree(ptr));
    });
}
int snpmi_dev_memset(void* ptr, int value, uint64_t bytes) {
    return guarded([&] { SNPMI_HIP(hipMemsetAsync(ptr, value, bytes, stream())); });
}
int snpmi_memcpy_h2d(void* dst, const void* src, uint64_t bytes) {
    return guarded([&] {
        SNPMI_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream()));
        SNPMI_HIP(hipStreamSynchronize(stream()));
    });
}
int snpmi_memcpy_d2h(void* dst, const void* src, uint64_t bytes) {
    return guarded([&] {
        SNPMI_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream()));
        SNPMI_HIP(hipStreamSynchronize(stream()));
    });
}
int snpmi_dev_memcpy_d2d(void* dst, const void* src, uint64_t bytes) {
    return guarded([&] {
        const bool aligned = reinterpret_cast<uintptr_t>(dst) % 16 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0;
        const uint64_t body = aligned ? bytes / 16 * 16 : 0;
        if (body) launch_copy16(src, dst, body, stream());
        if (bytes > body)
            SNPMI_HIP(hipMemcpyAsync((uint8_t*)dst + body, (const uint8_t*)src + body, bytes - body,
                                     hipMemcpyDeviceToDevice, stream()));
    });
}
int snpmi_stream_sync(void) {
    return guarded([&] {
        Device& d = device();
        SNPMI_HIP(hipStreamSynchronize(d.stream));
        SNPMI_HIP(hipStreamSynchronize(d.copy));
        SNPMI_HIP(hipStreamSynchronize(d.aux));
    });
}

int snpmi_set_stream(int which) {
    return guarded([&] {
        SNPMI_REQUIRE(which == 0 || which == 2, SNPMI_E_ARG, "stream must be 0 (compute) or 2 (aux)");
        g_sel_stream = which;
    });
}

// ---------------------------------------------------------------------- copy stream (streaming API)
static hipStream_t pick_stream(Device& d, int on_copy) {
    return on_copy == 1 ? d.copy : on_copy == 2 ? d.aux : d.stream;
}

int snpmi_memcpy_async(void* dst, const void* src, uint64_t bytes, int kind, int on_copy) {
    return guarded([&] {
        SNPMI_REQUIRE(kind >= 0 && kind <= 2, SNPMI_E_ARG, "kind must be 0 (H2D), 1 (D2H) or 2 (D2D)");
        Device& d = device();
        const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                              : hipMemcpyDeviceToDevice;
        if (bytes) SNPMI_HIP(hipMemcpyAsync(dst, src, bytes, k, pick_stream(d, on_copy)));
    });
}
int snpmi_event_record_on(void* ev, int on_copy) {
    return guarded([&] {
        Device& d = device();
        SNPMI_HIP(hipEventRecord((hipEvent_t)ev, pick_stream(d, on_copy)));
    });
}
int snpmi_stream_wait_event(void* ev, int on_copy) {
    return guarded([&] {
        Device& d = device();
        SNPMI_HIP(hipStreamWaitEvent(pick_stream(d, on_copy), (hipEvent_t)ev, 0));
    });
}
int snpmi_event_sync(void* ev) {
    return guarded([&] { SNPMI_HIP(hipEventSynchronize((hipEvent_t)ev)); });
}
int snpmi_event_create(void** ev) {
    return guarded([&] {
        (void)device();
        SNPMI_HIP(hipEventCreate((hipEvent_t*)ev));
    });
}
int snpmi_event_destroy(void* ev) {
    return guarded([&] { SNPMI_HIP(hipEventDestroy((hipEvent_t)ev)); });
}
int snpmi_event_record(void* ev) {
    return guarded([&] { SNPMI_HIP(hipEventRecord((hipEvent_t)ev, stream())); });
}
int snpmi_event_elapsed_ms(void* start, void* stop, float* ms) {
    return guarded([&] {
        SNPMI_HIP(hipEventSynchronize((hipEvent_t)stop));
        SNPMI_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    });
}

int snpmi_dev_synth_bed(uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t sid0, uint64_t n_sid, uint64_t seed,
                        double miss_rate, const double* maf_x, const double* maf_cdf, int n_pts) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);  // shared scratch slots
        SNPMI_REQUIRE(pitch % 4 == 0 && pitch >= ceil_div(n_iid, 4), SNPMI_E_ARG, "bad pitch");
        SNPMI_REQUIRE(n_pts > 0 && n_pts <= 1024, SNPMI_E_ARG, "bad MAF table");
        Device& d = device();
        double* tab = (double*)d.get(Device::S_RED, 2 * n_pts * sizeof(double));
        SNPMI_HIP(hipMemcpyAsync(tab, maf_x, n_pts * 8, hipMemcpyHostToDevice, d.stream));
        SNPMI_HIP(hipMemcpyAsync(tab + n_pts, maf_cdf, n_pts * 8, hipMemcpyHostToDevice, d.stream));
        launch_synth(packed, pitch, n_iid, sid0, n_sid, seed, miss_rate, tab, tab + n_pts, n_pts, d.stream);
        SNPMI_HIP(hipStreamSynchronize(d.stream));
    });
}

// ---------------------------------------------------------------------- host-side synthetic source
// A stand-in for "gather the selected .bed columns from the page cache into pinned memory" when a
// workload is too large to write to disk (cfg5: 125 GB of packed codes): the streamed GRM legs
// generate each SNP block on host threads while the GPU works on the previous one.  Per SNP the
// MAF comes from the same counter hash and MAF table as k_synth; per genotype one 32-bit hash
// (lowbias32 of seed/SNP key ^ iid * golden ratio) split into missing / hom-alt / het / hom-ref
// with the joint probabilities miss, (1-miss) p^2, (1-miss) 2p(1-p), rest -- k_synth's
// distribution, a cheaper stream (AVX2 when the host has it).  Restated in NumPy by
// tests/test_host_synth.py.
namespace {
inline uint64_t h_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
inline uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
struct SynthCol {
    uint32_t kb, thm, t3, t2;
};
inline uint32_t synth_code(uint32_t u, const SynthCol& c) {
    const uint32_t a = u - c.thm;
    return u < c.thm ? 1u : a < c.t3 ? 3u : a - c.t3 < c.t2 ? 2u : 0u;
}
// packed words [d0, d0+nw) of one column (16 iids per word; iids >= n are 0)
void synth_words_scalar(uint32_t* w, uint64_t d0, uint64_t nw, uint64_t n, const SynthCol& c) {
    for (uint64_t q = 0; q < nw; q++) {
        uint32_t x = 0;
        for (uint32_t k = 0; k < 16; k++) {
            const uint64_t i = 16 * (d0 + q) + k;
            if (i >= n) break;
            x |= synth_code(lowbias32(c.kb ^ ((uint32_t)i * 0x9E3779B9u)), c) << (2 * k);
        }
        w[q] = x;
    }
}
__attribute__((target("avx2"))) void synth_words_avx2(uint32_t* w, uint64_t d0, uint64_t nw, uint64_t n,
                                                      const SynthCol& c) {
    const __m256i sgn = _mm256_set1_epi32((int)0x80000000u);
    const __m256i vkb = _mm256_set1_epi32((int)c.kb), G = _mm256_set1_epi32((int)0x9E3779B9u);
    const __m256i M1 = _mm256_set1_epi32(0x7feb352d), M2 = _mm256_set1_epi32((int)0x846ca68bu);
    const __m256i thm_s = _mm256_set1_epi32((int)(c.thm ^ 0x80000000u)), t3_s = _mm256_set1_epi32((int)(c.t3 ^ 0x80000000u)),
                  t2_s = _mm256_set1_epi32((int)(c.t2 ^ 0x80000000u)), thm = _mm256_set1_epi32((int)c.thm),
                  t3 = _mm256_set1_epi32((int)c.t3), two = _mm256_set1_epi32(2), three = _mm256_set1_epi32(3),
                  one = _mm256_set1_epi32(1);
    const __m256i lane = _mm256_setr_epi32(0, 16, 32, 48, 64, 80, 96, 112);
    const uint64_t full = std::min<uint64_t>(nw, n / 16 > d0 ? n / 16 - d0 : 0);  // words with 16 real iids
    uint64_t q = 0;
    for (; q + 8 <= full; q += 8) {
        __m256i i = _mm256_add_epi32(_mm256_set1_epi32((int)(uint32_t)(16 * (d0 + q))), lane);
        __m256i x = _mm256_setzero_si256();
        for (int k = 0; k < 16; k++) {
            __m256i h = _mm256_xor_si256(vkb, _mm256_mullo_epi32(i, G));
            h = _mm256_xor_si256(h, _mm256_srli_epi32(h, 16));
            h = _mm256_mullo_epi32(h, M1);
            h = _mm256_xor_si256(h, _mm256_srli_epi32(h, 15));
            h = _mm256_mullo_epi32(h, M2);
            h = _mm256_xor_si256(h, _mm256_srli_epi32(h, 16));
            const __m256i miss = _mm256_cmpgt_epi32(thm_s, _mm256_xor_si256(h, sgn));  // u < thm (unsigned)
            const __m256i a = _mm256_sub_epi32(h, thm);
            const __m256i hom = _mm256_cmpgt_epi32(t3_s, _mm256_xor_si256(a, sgn));
            const __m256i het = _mm256_cmpgt_epi32(t2_s, _mm256_xor_si256(_mm256_sub_epi32(a, t3), sgn));
            __m256i code = _mm256_and_si256(het, two);
            code = _mm256_blendv_epi8(code, three, hom);
            code = _mm256_blendv_epi8(code, one, miss);
            x = _mm256_or_si256(x, _mm256_sll_epi32(code, _mm_cvtsi32_si128(2 * k)));
            i = _mm256_add_epi32(i, one);
        }
        _mm256_storeu_si256((__m256i*)(w + q), x);
    }
    if (q < nw) synth_words_scalar(w + q, d0 + q, nw - q, n, c);
}
}  // namespace

int snpmi_host_synth_bed(uint8_t* dst, uint64_t pitch, uint64_t n_iid, uint64_t sid0, uint64_t n_sid, uint64_t seed,
                         double miss_rate, const double* maf_x, const double* maf_cdf, int n_pts, int num_threads) {
    return guarded([&] {
        SNPMI_REQUIRE(dst != nullptr || n_sid == 0, SNPMI_E_ARG, "dst is NULL");
        SNPMI_REQUIRE(pitch % 4 == 0 && pitch >= ceil_div(n_iid, 4), SNPMI_E_ARG, "bad pitch");
        SNPMI_REQUIRE(n_pts > 0 && n_pts <= 1024 && maf_x && maf_cdf, SNPMI_E_ARG, "bad MAF table");
        SNPMI_REQUIRE(n_iid < (1ull << 32), SNPMI_E_ARG, "host synth: n_iid must be < 2^32");
        const bool avx2 = __builtin_cpu_supports("avx2");
        const uint64_t nd = pitch / 4, per = 2048;  // words per work item (32 KiB of codes)
        const uint64_t items_per_col = ceil_div(nd, per);
        const double sc = 4294967296.0;
        auto thr = [&](double t) { return t >= sc ? 0xFFFFFFFFu : (uint32_t)t; };
        parallel_for(
            n_sid * items_per_col, resolve_threads(num_threads),
            [&](uint64_t it) {
                const uint64_t j = it / items_per_col, d0 = (it % items_per_col) * per;
                const uint64_t sid = sid0 + j;
                const uint64_t h = h_splitmix64(seed * 0xD1B54A32D192ED03ull ^ (sid + 1) * 0x8CB92BA72F3D8DD7ull);
                const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
                int lo = 0, hi = n_pts - 1;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (u > maf_cdf[mid]) lo = mid + 1;
                    else hi = mid;
                }
                const double maf = maf_x[lo], keep = 1.0 - miss_rate;
                SynthCol c;
                c.kb = (uint32_t)(h_splitmix64((seed + 0x632BE59BD9B4E019ull) ^ (sid * 0x9E6C63D0676A9A99ull)) >> 32);
                c.thm = thr(miss_rate * sc);
                c.t3 = thr(keep * maf * maf * sc);
                c.t2 = thr(keep * 2.0 * maf * (1.0 - maf) * sc);
                uint32_t* w = reinterpret_cast<uint32_t*>(dst + j * pitch) + d0;
                const uint64_t nw = std::min(per, nd - d0);
                if (avx2) synth_words_avx2(w, d0, nw, n_iid, c);
                else synth_words_scalar(w, d0, nw, n_iid, c);
            },
            4);
    });
}

// selected .bed columns (all iids, ceil(n/4) bytes each, zero-padded to `pitch`) into a host
// buffer -- the host half of stage_chunk, for callers that run their own upload (the cfg5 plan:
// each rank gathers only its share of a SNP block, shard.PartitionedGrm)
int snpmi_bed_gather_packed(const char* path, uint64_t n_iid, uint64_t n_sid, const uint64_t* sid_idx, uint64_t n_sel,
                            uint64_t pitch, uint8_t* dst, int num_threads) {
    return guarded([&] {
        BedMap m;
        open_bed(m, path, n_iid, n_sid);
        SNPMI_REQUIRE(pitch >= m.bpc, SNPMI_E_ARG, "pitch is smaller than a column");
        SNPMI_REQUIRE(dst != nullptr || n_sel == 0, SNPMI_E_ARG, "dst is NULL");
        check_index(sid_idx, n_sel, n_sid, "sid");
        gather_columns(m, sid_idx, 0, n_sel, pitch, dst, resolve_threads(num_threads));
    });
}

int snpmi_dev_snp_stats(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, int count_a1,
                        int std_kind, double a, double b, int use_stats, int dtype, void* stats, void* lut) {
    return guarded([&] {
        SNPMI_REQUIRE(pitch % 64 == 0 && pitch >= ceil_div(n_iid, 4), SNPMI_E_ARG, "pitch must be snpmi_packed_pitch");
        launch_snp_stats(packed, pitch, n_iid, n_sid, count_a1, std_kind, a, b, use_stats, dtype, stats, lut, stream());
    });
}

int snpmi_dev_decode(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, const void* lut,
                     int dtype, int order_c, void* out, uint64_t ld) {
    return guarded([&] {
        SNPMI_REQUIRE(pitch % 64 == 0 && pitch >= ceil_div(n_iid, 4), SNPMI_E_ARG, "pitch must be snpmi_packed_pitch");
        if (!order_c) SNPMI_REQUIRE(ld % 16 == 0 && ld >= n_iid, SNPMI_E_ARG, "F-order ld must be >= n_iid, % 16");
        else SNPMI_REQUIRE(ld >= n_sid, SNPMI_E_ARG, "C-order ld must be >= n_sid");
        launch_decode(packed, pitch, n_iid, n_sid, lut, dtype, order_c, out, ld, stream());
    });
}

int snpmi_dev_decode_standardize(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                                 int count_a1, int std_kind, double a, double b, int use_stats, int dtype,
                                 void* stats, void* lut, void* out, uint64_t ld) {
    return guarded([&] {
        SNPMI_REQUIRE(dtype == SNPMI_DT_F32, SNPMI_E_ARG, "fused decode+standardize is f32 only");
        SNPMI_REQUIRE(pitch % 64 == 0 && pitch >= ceil_div(n_iid, 4), SNPMI_E_ARG, "pitch must be snpmi_packed_pitch");
        SNPMI_REQUIRE(ld % 16 == 0 && ld >= n_iid, SNPMI_E_ARG, "F-order ld must be >= n_iid, % 16");
        launch_decode_std_fused(packed, pitch, n_iid, n_sid, count_a1, std_kind, a, b, use_stats, stats, lut, out, ld,
                                stream());
    });
}

int snpmi_dev_repack(const uint8_t* src, uint64_t src_pitch, uint64_t n_src, const uint64_t* idx, uint64_t n_out,
                     uint64_t n_sid, uint8_t* dst, uint64_t dst_pitch) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);  // shared scratch slots
        SNPMI_REQUIRE(dst_pitch % 64 == 0 && dst_pitch >= ceil_div(n_out, 4), SNPMI_E_ARG, "bad dst pitch");
        Device& d = device();
        uint32_t* plan = (uint32_t*)d.get(Device::S_IDX32, repack_plan_entries(n_out) * 4);
        uint32_t* win = (uint32_t*)d.get(Device::S_WIN, repack_win_entries(n_out) * 4);
        const RepackPlan P = launch_repack_plan(idx, n_out, n_src, plan, win, d.stream);
        launch_repack(src, src_pitch, n_src, idx, P, n_out, n_sid, dst, dst_pitch, d.stream);
    });
}

int snpmi_dev_syrk_packed(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, const void* lut,
                          int dtype, void* K_tiles, int accumulate) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);  // shared scratch slots
        SNPMI_REQUIRE(dtype == SNPMI_DT_F32 || dtype == SNPMI_DT_F64, SNPMI_E_ARG, "GRM dtype must be f32/f64");
        SNPMI_REQUIRE(pitch % 64 == 0 && pitch >= ceil_div(n_iid, 4), SNPMI_E_ARG, "pitch must be snpmi_packed_pitch");
        syrk_packed_auto(device(), packed, pitch, n_iid, n_sid, lut, dtype, K_tiles, accumulate);
    });
}

uint64_t snpmi_grm_part_blocks(uint64_t n_iid, int part_rank, int part_world) {
    if (part_world < 1 || part_rank < 0 || part_rank >= part_world) return 0;
    return grm_part_blocks(n_iid, part_rank, part_world);
}

// host copy of the last part layout asked for (snpmi_grm_part_coords is called per block)
static std::mutex g_layout_mutex;
static std::vector<uint32_t> g_layout;
static uint64_t g_layout_key[3] = {~0ull, 0, 0};
static const std::vector<uint32_t>& host_layout(uint64_t nb, int rank, int world) {
    if (g_layout_key[0] != nb || g_layout_key[1] != (uint64_t)rank || g_layout_key[2] != (uint64_t)world) {
        part_layout(nb, rank, world, g_layout);
        g_layout_key[0] = nb;
        g_layout_key[1] = (uint64_t)rank;
        g_layout_key[2] = (uint64_t)world;
    }
    return g_layout;
}

int snpmi_grm_part_coords(uint64_t n_iid, int part_rank, int part_world, uint64_t local_block, uint64_t* row0,
                          uint64_t* col0) {
    return guarded([&] {
        SNPMI_REQUIRE(part_world >= 1 && part_rank >= 0 && part_rank < part_world, SNPMI_E_ARG, "bad partition");
        std::lock_guard<std::mutex> lk(g_layout_mutex);
        const auto& tab = host_layout(ceil_div(n_iid, 256), part_rank, part_world);
        SNPMI_REQUIRE(local_block < tab.size(), SNPMI_E_INDEX, "block out of range");
        if (row0) *row0 = (uint64_t)(tab[local_block] & 0xffffu) * 256;
        if (col0) *col0 = (uint64_t)(tab[local_block] >> 16) * 256;
    });
}

int snpmi_grm_part_coords_all(uint64_t n_iid, int part_rank, int part_world, uint64_t* coords) {
    return guarded([&] {
        SNPMI_REQUIRE(part_world >= 1 && part_rank >= 0 && part_rank < part_world, SNPMI_E_ARG, "bad partition");
        std::lock_guard<std::mutex> lk(g_layout_mutex);
        const auto& tab = host_layout(ceil_div(n_iid, 256), part_rank, part_world);
        SNPMI_REQUIRE(coords != nullptr || tab.empty(), SNPMI_E_ARG, "coords is NULL");
        for (uint64_t w = 0; w < tab.size(); w++) {
            coords[2 * w] = (uint64_t)(tab[w] & 0xffffu) * 256;
            coords[2 * w + 1] = (uint64_t)(tab[w] >> 16) * 256;
        }
    });
}

// cfg5 from a file (K too large to replicate): rank part_rank of part_world streams EVERY SNP of
// the .bed (stats need all iids of a SNP; each rank computes them itself -- no exchange) and
// accumulates only its own 256x256 K blocks (snpmi_grm_part_coords) in HBM, then copies them to
// blocks_out (n_local x 65536 f32, row-major blocks; may be a memory-mapped file).
}  // extern "C"

namespace snpmi {
template <typename T>
static void grm_part_bed_impl(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1, const uint64_t* iid_idx,
                              uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid, int std_kind, double a,
                              double b, int use_stats, T* stats, int part_rank, int part_world, T* blocks_out,
                              int num_threads) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    SNPMI_REQUIRE(part_world >= 1 && part_rank >= 0 && part_rank < part_world, SNPMI_E_ARG, "bad rank / world");
    const uint64_t n_out = iid_idx ? n_out_iid : n_iid;
    const uint64_t nloc = grm_part_blocks(n_out, part_rank, part_world);
    SNPMI_REQUIRE(blocks_out != nullptr || nloc == 0, SNPMI_E_ARG, "blocks_out is NULL");
    Device& d = device();
    const uint64_t bytes = std::max<uint64_t>(nloc, 1) * 256 * 256 * sizeof(T);
    // blocks_out in device memory: the SYRK accumulates into it directly (K stays in HBM, no
    // scratch, no copy-out); host memory: scratch tiles + a pinned-bounce copy at the end
    const bool dev_out = nloc && is_device_ptr(d, blocks_out);
    T* blocks = dev_out ? blocks_out : (T*)d.get(Device::S_TILES, bytes);
    const bool wrote = grm_stream_bed<T>(
        d, true, path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid, std_kind, a, b, use_stats,
        stats, num_threads,
        [&](const uint8_t* packed, uint64_t pitch, uint64_t n, uint64_t cnt, const T* lut, bool acc) {
            if constexpr (std::is_same<T, double>::value)
                syrk_packed_part_f64(d, packed, pitch, n, cnt, lut, part_rank, part_world, blocks, acc);
            else
                syrk_packed_part_auto(d, packed, pitch, n, cnt, lut, part_rank, part_world, blocks, acc);
        });
    if (!wrote) SNPMI_HIP(hipMemsetAsync(blocks, 0, dev_out ? nloc * 256 * 256 * sizeof(T) : bytes, d.stream));
    const size_t bb = 256 * 256 * sizeof(T);  // one block per "row" of the pinned-bounce copy
    if (nloc && !dev_out) d2h_rows(d, blocks_out, bb, blocks, bb, bb, nloc, resolve_threads(num_threads));
    SNPMI_HIP(hipStreamSynchronize(d.stream));
}
}  // namespace snpmi

extern "C" {

// cfg5 from a file (K too large to replicate): rank part_rank of part_world streams EVERY SNP of
// the .bed (stats need all iids of a SNP; each rank computes them itself -- no exchange) and
// accumulates only its own 256x256 K blocks (snpmi_grm_part_coords) in HBM, then copies them to
// blocks_out (n_local x 65536 values, row-major blocks; may be a memory-mapped file).
int snpmi_grm_part_bed_f32(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1, const uint64_t* iid_idx,
                           uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid, int std_kind, double a,
                           double b, int use_stats, float* stats, int part_rank, int part_world, float* blocks_out,
                           int num_threads) {
    return guarded([&] {
        grm_part_bed_impl<float>(path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid, std_kind, a, b,
                                 use_stats, stats, part_rank, part_world, blocks_out, num_threads);
    });
}
int snpmi_grm_part_bed_f64(const char* path, uint64_t n_iid, uint64_t n_sid, int count_a1, const uint64_t* iid_idx,
                           uint64_t n_out_iid, const uint64_t* sid_idx, uint64_t n_out_sid, int std_kind, double a,
                           double b, int use_stats, double* stats, int part_rank, int part_world, double* blocks_out,
                           int num_threads) {
    return guarded([&] {
        grm_part_bed_impl<double>(path, n_iid, n_sid, count_a1, iid_idx, n_out_iid, sid_idx, n_out_sid, std_kind, a,
                                  b, use_stats, stats, part_rank, part_world, blocks_out, num_threads);
    });
}

int snpmi_dev_syrk_packed_part(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid, const void* lut,
                               int part_rank, int part_world, void* blocks, int accumulate) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);  // shared scratch slots
        SNPMI_REQUIRE(part_world >= 1 && part_rank >= 0 && part_rank < part_world, SNPMI_E_ARG, "bad partition");
        SNPMI_REQUIRE(pitch % 64 == 0 && pitch >= ceil_div(n_iid, 4), SNPMI_E_ARG, "pitch must be snpmi_packed_pitch");
        syrk_packed_part_auto(device(), packed, pitch, n_iid, n_sid, (const float*)lut, part_rank, part_world, blocks,
                              accumulate);
    });
}

}  // extern "C"

namespace snpmi {
// K[ri, ci] restricted to part `part_rank`'s blocks (the rest 0): the parts' outputs summed over
// the ranks are the sub-matrix (snpmi_grm_part_extract_*, the PartitionedKernel reader)
template <typename T>
static void part_extract_impl(const T* blocks, uint64_t n, int part_rank, int part_world, const uint64_t* ri,
                              uint64_t nr, const uint64_t* ci, uint64_t nc, int order_c, double scale, T* out) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    SNPMI_REQUIRE(part_world >= 1 && part_rank >= 0 && part_rank < part_world, SNPMI_E_ARG, "bad partition");
    SNPMI_REQUIRE(out != nullptr || nr * nc == 0, SNPMI_E_ARG, "out is NULL");
    Device& d = device();
    const uint64_t nloc = grm_part_blocks(n, part_rank, part_world);
    SNPMI_REQUIRE(nloc == 0 || (blocks && is_device_ptr(d, blocks)), SNPMI_E_ARG,
                  "blocks must be device memory of the current device");
    for (uint64_t k = 0; ri && k < nr; k++) SNPMI_REQUIRE(ri[k] < n, SNPMI_E_INDEX, "iid0 index out of range");
    for (uint64_t k = 0; ci && k < nc; k++) SNPMI_REQUIRE(ci[k] < n, SNPMI_E_INDEX, "iid1 index out of range");
    SNPMI_REQUIRE(ri || nr <= n, SNPMI_E_INDEX, "iid0 count exceeds n");
    SNPMI_REQUIRE(ci || nc <= n, SNPMI_E_INDEX, "iid1 count exceeds n");
    if (nr * nc == 0) return;
    const PartTables pt = part_tables(ceil_div(n, 256), part_rank, part_world);
    uint64_t* dri = nullptr;
    uint64_t* dci = nullptr;
    if (ri) {
        dri = (uint64_t*)d.get(Device::S_IDX, nr * 8);
        SNPMI_HIP(hipMemcpyAsync(dri, ri, nr * 8, hipMemcpyHostToDevice, d.stream));
    }
    if (ci) {
        dci = (uint64_t*)d.get(Device::S_IDX2, nc * 8);
        SNPMI_HIP(hipMemcpyAsync(dci, ci, nc * 8, hipMemcpyHostToDevice, d.stream));
    }
    const bool dev = is_device_ptr(d, out);
    T* o = dev ? out : (T*)d.get(Device::S_K, nr * nc * sizeof(T));
    launch_part_extract(blocks, pt.lslot, DT<T>::v, dri, nr, dci, nc, order_c, scale, o, d.stream);
    if (!dev) SNPMI_HIP(hipMemcpyAsync(out, o, nr * nc * sizeof(T), hipMemcpyDeviceToHost, d.stream));
    SNPMI_HIP(hipStreamSynchronize(d.stream));
}

template <typename T>
static void part_trace_impl(const T* blocks, uint64_t n, int part_rank, int part_world, double* trace) {
    std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
    SNPMI_REQUIRE(part_world >= 1 && part_rank >= 0 && part_rank < part_world, SNPMI_E_ARG, "bad partition");
    SNPMI_REQUIRE(trace != nullptr, SNPMI_E_ARG, "trace is NULL");
    Device& d = device();
    *trace = 0.0;
    if (n == 0 || grm_part_blocks(n, part_rank, part_world) == 0) return;
    SNPMI_REQUIRE(blocks && is_device_ptr(d, blocks), SNPMI_E_ARG, "blocks must be device memory of the current device");
    const PartTables pt = part_tables(ceil_div(n, 256), part_rank, part_world);
    double* tr = (double*)d.get(Device::S_RED, 64);
    launch_part_trace(blocks, pt.dslot, n, DT<T>::v, tr, d.stream);
    SNPMI_HIP(hipMemcpyAsync(trace, tr, 8, hipMemcpyDeviceToHost, d.stream));
    SNPMI_HIP(hipStreamSynchronize(d.stream));
}
}  // namespace snpmi

extern "C" {

int snpmi_grm_part_extract_f32(const float* blocks, uint64_t n_iid, int part_rank, int part_world, const uint64_t* ri,
                               uint64_t nr, const uint64_t* ci, uint64_t nc, int order_c, double scale, float* out) {
    return guarded([&] { part_extract_impl<float>(blocks, n_iid, part_rank, part_world, ri, nr, ci, nc, order_c, scale, out); });
}
int snpmi_grm_part_extract_f64(const double* blocks, uint64_t n_iid, int part_rank, int part_world, const uint64_t* ri,
                               uint64_t nr, const uint64_t* ci, uint64_t nc, int order_c, double scale, double* out) {
    return guarded([&] { part_extract_impl<double>(blocks, n_iid, part_rank, part_world, ri, nr, ci, nc, order_c, scale, out); });
}
int snpmi_grm_part_trace_f32(const float* blocks, uint64_t n_iid, int part_rank, int part_world, double* trace) {
    return guarded([&] { part_trace_impl<float>(blocks, n_iid, part_rank, part_world, trace); });
}
int snpmi_grm_part_trace_f64(const double* blocks, uint64_t n_iid, int part_rank, int part_world, double* trace) {
    return guarded([&] { part_trace_impl<double>(blocks, n_iid, part_rank, part_world, trace); });
}
int snpmi_device_memory(uint64_t* free_bytes, uint64_t* total_bytes) {
    return guarded([&] {
        device();
        size_t f = 0, t = 0;
        SNPMI_HIP(hipMemGetInfo(&f, &t));
        if (free_bytes) *free_bytes = f;
        if (total_bytes) *total_bytes = t;
    });
}

int snpmi_dev_syrk_packed_part_f64(const uint8_t* packed, uint64_t pitch, uint64_t n_iid, uint64_t n_sid,
                                   const double* lut, int part_rank, int part_world, double* blocks, int accumulate) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);  // shared scratch slots
        SNPMI_REQUIRE(part_world >= 1 && part_rank >= 0 && part_rank < part_world, SNPMI_E_ARG, "bad partition");
        SNPMI_REQUIRE(pitch % 64 == 0 && pitch >= ceil_div(n_iid, 4), SNPMI_E_ARG, "pitch must be snpmi_packed_pitch");
        syrk_packed_part_f64(device(), packed, pitch, n_iid, n_sid, lut, part_rank, part_world, blocks, accumulate);
    });
}

int snpmi_dev_syrk_dense(const void* Z, uint64_t ldz, uint64_t n_iid, uint64_t n_sid, int dtype, void* K_tiles,
                         int accumulate) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);  // shared scratch slots
        SNPMI_REQUIRE(dtype == SNPMI_DT_F32 || dtype == SNPMI_DT_F64, SNPMI_E_ARG, "GRM dtype must be f32/f64");
        syrk_dense_auto(device(), Z, ldz, n_iid, n_sid, dtype, K_tiles, accumulate);
    });
}

int snpmi_dev_grm_extract(const void* K_tiles, uint64_t n_iid, int dtype, const uint64_t* ri, uint64_t nr,
                          const uint64_t* ci, uint64_t nc, int order_c, double scale, void* out) {
    return guarded([&] {
        // the whole K (K symmetric, so either order): the tile-blocked extraction
        if (!ri && !ci && nr == n_iid && nc == n_iid)
            launch_grm_extract_rows(K_tiles, n_iid, dtype, 0, n_iid, scale, out, stream());
        else
            launch_grm_extract(K_tiles, n_iid, dtype, ri, nr, ci, nc, order_c, scale, out, stream());
    });
}

static void crt_stats(uint64_t* a, uint64_t* b, int reset, int which) {
    Device& d = device();
    unsigned long long h[2] = {0, 0};
    unsigned long long* rec = crt_record(d) + 2 * which;
    SNPMI_HIP(hipMemcpyAsync(h, rec, sizeof(h), hipMemcpyDeviceToHost, d.stream));
    if (reset) SNPMI_HIP(hipMemsetAsync(rec, 0, sizeof(h), d.stream));
    SNPMI_HIP(hipStreamSynchronize(d.stream));
    *a = h[0];
    *b = h[1];
}

int snpmi_crt_moduli_stats(uint64_t* sum_r, uint64_t* launches, int reset) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
        SNPMI_REQUIRE(sum_r != nullptr && launches != nullptr, SNPMI_E_ARG, "NULL output");
        crt_stats(sum_r, launches, reset, 0);
    });
}

int snpmi_crt_block_moduli_stats(uint64_t* sum_rb, uint64_t* blocks, int reset) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);
        SNPMI_REQUIRE(sum_rb != nullptr && blocks != nullptr, SNPMI_E_ARG, "NULL output");
        crt_stats(sum_rb, blocks, reset, 1);
    });
}

int snpmi_dev_grm_trace(const void* K_tiles, uint64_t n_iid, int dtype, double* trace) {
    return guarded([&] {
        std::lock_guard<std::recursive_mutex> lk(g_call_mutex);  // shared scratch slots
        Device& d = device();
        double* tr = (double*)d.get(Device::S_RED, 64);
        launch_grm_trace(K_tiles, n_iid, dtype, tr, d.stream);
        SNPMI_HIP(hipMemcpyAsync(trace, tr, 8, hipMemcpyDeviceToHost, d.stream));
        SNPMI_HIP(hipStreamSynchronize(d.stream));
    });
}

}  // extern "C"
