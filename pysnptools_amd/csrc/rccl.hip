// RCCL over xGMI for the SNP-sharded GRM: one process per GPU, each rank
// accumulates the upper-triangle K tiles of its SNP blocks, then one in-place ncclReduce(sum)
// of the tile buffer produces K on the rank that returns it (ncclAllReduce when every rank
// needs K, e.g. shard.grm_pieces).  In the K-partitioned
// mode (cfg5) each rank uploads 1/p of a packed SNP block and ncclAllGather rebuilds the
// whole block on every rank (packed codes are 16x smaller than the f32 values).  The unique id is
// exchanged by the caller (bench.py: rank 0 writes it to an O_EXCL node-local file named by
// the launcher; the package never imports torch, whose own HIP runtime would load beside ours).
#include <rccl/rccl.h>

#include <atomic>

#include "snpmi_internal.hpp"

namespace {
ncclComm_t g_comm = nullptr;
int g_comm_dev = -1;  // the device the communicator was created on

// Collective trace (snpmi_rccl_trace): every RCCL call this process enqueues is counted, by kind,
// with its element/byte count folded into a running signature -- the same calls in the same order
// give the same signature on every rank, so a per-rank dump after a stall (bench.py's watchdog)
// shows which rank issued a different or an extra collective.  Lock-free: a watchdog thread reads
// it while the main thread is blocked inside a collective.
enum TraceKind { TK_ALLREDUCE = 1, TK_REDUCE = 2, TK_ALLGATHER = 3, TK_HOST = 4 };
std::atomic<uint64_t> g_tr_calls{0}, g_tr_kind[5], g_tr_bytes{0}, g_tr_sig{1469598103934665603ull};
std::atomic<uint64_t> g_tr_last_kind{0}, g_tr_last_count{0}, g_tr_blocking{0}, g_tr_blocked_calls{0};
void trace(int kind, uint64_t count, uint64_t bytes, int root) {
    g_tr_calls.fetch_add(1, std::memory_order_relaxed);
    g_tr_kind[kind].fetch_add(1, std::memory_order_relaxed);
    g_tr_bytes.fetch_add(bytes, std::memory_order_relaxed);
    g_tr_last_kind.store((uint64_t)kind, std::memory_order_relaxed);
    g_tr_last_count.store(count, std::memory_order_relaxed);
    // FNV-1a over (kind, count, root): rank-independent for the plan's calls
    uint64_t h = g_tr_sig.load(std::memory_order_relaxed);
    for (uint64_t x : {(uint64_t)kind, count, (uint64_t)(int64_t)root}) h = (h ^ x) * 1099511628211ull;
    g_tr_sig.store(h, std::memory_order_relaxed);
}
// the host all-reduce (barriers, max-over-ranks) waits on the stream inside the call: a rank
// stuck there has g_tr_blocking set
struct Blocking {
    Blocking() { g_tr_blocking.store(1); }
    ~Blocking() {
        g_tr_blocking.store(0);
        g_tr_blocked_calls.fetch_add(1);
    }
};

#define SNPMI_NCCL(expr)                                                                     \
    do {                                                                                     \
        ncclResult_t r_ = (expr);                                                            \
        if (r_ != ncclSuccess)                                                               \
            throw ::snpmi::Error(SNPMI_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)
// the communicator exists and the calling thread drives the device it was built on (the
// library's current device is per thread; a collective on another device's stream would pair a
// device-0 communicator with device r's buffers)
void require_comm() {
    SNPMI_REQUIRE(g_comm != nullptr, SNPMI_E_ARG, "RCCL communicator not initialised");
    SNPMI_REQUIRE(snpmi::device().id == g_comm_dev, SNPMI_E_ARG,
                  "RCCL communicator was created on device " + std::to_string(g_comm_dev) +
                      " but this thread drives device " + std::to_string(snpmi::device().id));
}
}  // namespace

namespace snpmi {
// in-place sum of a device f32/f64 range over the ranks on stream st: ncclReduce onto root, or
// ncclAllReduce for root < 0 (api.hip grm_add_packed_reduce: one per finished column group, on the
// aux stream, under the next group's SYRK)
void rccl_sum_on(void* buf, uint64_t count, int dtype, int root, hipStream_t st) {
    require_comm();
    SNPMI_REQUIRE(dtype == SNPMI_DT_F32 || dtype == SNPMI_DT_F64, SNPMI_E_ARG, "sum dtype must be f32/f64");
    const ncclDataType_t t = dtype == SNPMI_DT_F64 ? ncclFloat64 : ncclFloat32;
    if (root < 0) {
        trace(TK_ALLREDUCE, count, count * dtype_size(dtype), -1);
        SNPMI_NCCL(ncclAllReduce(buf, buf, count, t, ncclSum, g_comm, st));
        return;
    }
    int nranks = 0;
    SNPMI_NCCL(ncclCommCount(g_comm, &nranks));
    SNPMI_REQUIRE(root < nranks, SNPMI_E_ARG, "reduce root out of range");
    trace(TK_REDUCE, count, count * dtype_size(dtype), root);
    SNPMI_NCCL(ncclReduce(buf, buf, count, t, ncclSum, root, g_comm, st));
}
bool rccl_ready() { return g_comm != nullptr; }
}  // namespace snpmi

using namespace snpmi;

extern "C" {

int snpmi_rccl_unique_id(uint8_t* id, uint64_t id_len) {
    return guarded([&] {
        SNPMI_REQUIRE(id && id_len >= sizeof(ncclUniqueId), SNPMI_E_ARG, "id buffer too small");
        ncclUniqueId u;
        SNPMI_NCCL(ncclGetUniqueId(&u));
        std::memcpy(id, &u, sizeof(u));
    });
}

int snpmi_rccl_init(int nranks, int rank, const uint8_t* id, uint64_t id_len) {
    return guarded([&] {
        SNPMI_REQUIRE(id && id_len >= sizeof(ncclUniqueId), SNPMI_E_ARG, "id buffer too small");
        SNPMI_REQUIRE(g_comm == nullptr, SNPMI_E_ARG, "RCCL communicator already initialised");
        const int dev = device().id;  // binds this thread's current HIP device
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        SNPMI_NCCL(ncclCommInitRank(&g_comm, nranks, u, rank));
        g_comm_dev = dev;
    });
}

int snpmi_rccl_allreduce_sum(void* buf, uint64_t count, int dtype) {
    return guarded([&] {
        require_comm();
        ncclDataType_t t = dtype == SNPMI_DT_F64 ? ncclFloat64 : ncclFloat32;
        SNPMI_REQUIRE(dtype == SNPMI_DT_F32 || dtype == SNPMI_DT_F64, SNPMI_E_ARG, "all-reduce dtype must be f32/f64");
        trace(TK_ALLREDUCE, count, count * dtype_size(dtype), -1);
        SNPMI_NCCL(ncclAllReduce(buf, buf, count, t, ncclSum, g_comm, stream()));
    });
}

int snpmi_rccl_reduce_sum(void* buf, uint64_t count, int dtype, int root) {
    return guarded([&] {
        require_comm();
        SNPMI_REQUIRE(dtype == SNPMI_DT_F32 || dtype == SNPMI_DT_F64, SNPMI_E_ARG, "reduce dtype must be f32/f64");
        int nranks = 0;
        SNPMI_NCCL(ncclCommCount(g_comm, &nranks));
        SNPMI_REQUIRE(root >= 0 && root < nranks, SNPMI_E_ARG, "reduce root out of range");
        const ncclDataType_t t = dtype == SNPMI_DT_F64 ? ncclFloat64 : ncclFloat32;
        trace(TK_REDUCE, count, count * dtype_size(dtype), root);
        SNPMI_NCCL(ncclReduce(buf, buf, count, t, ncclSum, root, g_comm, stream()));
    });
}

int snpmi_rccl_allgather(const void* send, void* recv, uint64_t bytes_per_rank) {
    return guarded([&] {
        require_comm();
        SNPMI_REQUIRE(send != nullptr && recv != nullptr, SNPMI_E_ARG, "all-gather buffer is NULL");
        trace(TK_ALLGATHER, bytes_per_rank, bytes_per_rank, -1);
        SNPMI_NCCL(ncclAllGather(send, recv, bytes_per_rank, ncclUint8, g_comm, stream()));
    });
}

int snpmi_rccl_host_allreduce_f64(double* values, uint64_t count, int op) {
    return guarded([&] {
        require_comm();
        SNPMI_REQUIRE(values != nullptr && count > 0 && count <= 4096, SNPMI_E_ARG, "bad host all-reduce buffer");
        Device& d = device();
        double* buf = (double*)d.get(Device::S_RED, count * sizeof(double));
        trace(TK_HOST, count, count * sizeof(double), op);
        Blocking blocking;
        SNPMI_HIP(hipMemcpyAsync(buf, values, count * sizeof(double), hipMemcpyHostToDevice, d.stream));
        SNPMI_NCCL(ncclAllReduce(buf, buf, count, ncclFloat64, op == 1 ? ncclMax : ncclSum, g_comm, d.stream));
        SNPMI_HIP(hipMemcpyAsync(values, buf, count * sizeof(double), hipMemcpyDeviceToHost, d.stream));
        SNPMI_HIP(hipStreamSynchronize(d.stream));
    });
}

int snpmi_rccl_barrier(void) {
    double one = 1.0;
    return snpmi_rccl_host_allreduce_f64(&one, 1, 0);
}

int snpmi_rccl_comm_count(int* count) {
    return guarded([&] {
        SNPMI_REQUIRE(g_comm != nullptr, SNPMI_E_ARG, "RCCL communicator not initialised");
        SNPMI_REQUIRE(count != nullptr, SNPMI_E_ARG, "count is NULL");
        SNPMI_NCCL(ncclCommCount(g_comm, count));
    });
}

int snpmi_rccl_trace(uint64_t* out, uint64_t n) {
    // no lock, no HIP call: safe from a watchdog thread while another thread sits in a collective
    if (!out) return SNPMI_E_ARG;
    const uint64_t v[12] = {g_tr_calls.load(),      g_tr_kind[TK_ALLREDUCE].load(), g_tr_kind[TK_REDUCE].load(),
                            g_tr_kind[TK_ALLGATHER].load(), g_tr_kind[TK_HOST].load(), g_tr_bytes.load(),
                            g_tr_sig.load(),        g_tr_last_kind.load(),  g_tr_last_count.load(),
                            g_tr_blocking.load(),   g_tr_blocked_calls.load(), (uint64_t)(g_comm != nullptr)};
    for (uint64_t i = 0; i < n && i < 12; i++) out[i] = v[i];
    return SNPMI_OK;
}

int snpmi_rccl_destroy(void) {
    return guarded([&] {
        if (g_comm) {
            SNPMI_HIP(hipStreamSynchronize(stream()));
            SNPMI_NCCL(ncclCommDestroy(g_comm));
            g_comm = nullptr;
            g_comm_dev = -1;
        }
    });
}

}  // extern "C"
