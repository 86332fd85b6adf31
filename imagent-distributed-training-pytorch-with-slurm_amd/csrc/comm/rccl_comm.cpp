// Native RCCL communicator with its own (normal-priority) HIP comm stream.
//
// Replaces what the reference gets from c10d ProcessGroupNCCL + NCCL
// (/root/reference/imagenet.py:270-273 init, :85 metric all-reduce, and the
// DDP bucket all-reduces issued from inside loss.backward(), :128).
//
// MI355X-first choices:
//  * one communicator per process (one process per GPU), bootstrapped from an
//    ncclUniqueId that the Python side ships through the c10d TCPStore;
//  * every collective runs on OUR comm stream (normal priority: a high-priority
//    queue parked on barrier packets throttles the compute queues, measured
//    -15 % img/s, parallel/comm.py stream_mode), ordered after the producing
//    compute stream by a HIP event and
//    re-joined by one event wait before the optimizer step - no host syncs;
//  * gradient buckets use ncclAvg (pre-scaling folded into the collective);
//  * RCCL picks multi-channel rings / direct algorithms over the 7 xGMI links
//    on its own when P2P is enabled - we never disable P2P (cf. the
//    reference's NCCL_P2P_DISABLE=1, imagenet.sh:19).
//
// C ABI for ctypes. Built with hipcc and linked against the librccl.so that
// torch ships (the same library c10d uses), see imagent_amd/build.py.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

namespace {

thread_local char g_err[512] = {0};

#define HIPCHK(x)                                                                     \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            snprintf(g_err, sizeof(g_err), "%s: %s", #x, hipGetErrorString(e_));      \
            return -1;                                                                \
        }                                                                             \
    } while (0)

#define NCCLCHK(x)                                                                    \
    do {                                                                              \
        ncclResult_t r_ = (x);                                                        \
        if (r_ != ncclSuccess) {                                                      \
            snprintf(g_err, sizeof(g_err), "%s: %s", #x, ncclGetErrorString(r_));     \
            return -2;                                                                \
        }                                                                             \
    } while (0)

struct Comm {
    // written once by init; imc_abort never clears it (readers test `aborting`), so no thread sees a
    // half-updated handle
    ncclComm_t comm = nullptr;
    // set by imc_abort (the watchdog thread) BEFORE the communicator is torn down: enqueue
    // paths spinning in settle() on the main thread see it and bail out instead of touching
    // a communicator that ncclCommAbort is freeing
    std::atomic<bool> aborting{false};
    // calls currently inside RCCL with this communicator (InFlight guards); imc_abort waits for it to
    // drain (bounded) before ncclCommAbort frees the communicator
    std::atomic<int> inflight{0};
    // who tears the communicator down, decided once (compare-exchange from 0): 1 = imc_abort (the watchdog),
    // 2 = imc_comm_destroy. The loser never touches the handle: a destroy that loses waits for `torn`, an abort
    // that loses returns (destroy's settle() sees `aborting` and aborts instead of finalising). The Comm object
    // itself is never freed (a few hundred bytes per communicator), so a watchdog that fires after destroy
    // returned reads valid memory and leaves.
    std::atomic<int> owner{0};
    std::atomic<bool> torn{false};  // the owner is done with the handle (last store of the owner)
    hipStream_t stream = nullptr;
    int rank = 0, nranks = 1, device = 0, n_events = 64, stream_mode = 0;
    std::vector<hipEvent_t> events;   // ring of reusable events
    size_t next_event = 0;
    hipEvent_t next() {
        hipEvent_t e = events[next_event];
        next_event = (next_event + 1) % events.size();
        return e;
    }
};

ncclDataType_t to_nccl(int32_t dt) {
    switch (dt) {
        case 0: return ncclFloat32;
        case 1: return ncclBfloat16;
        case 2: return ncclFloat16;
        case 3: return ncclInt64;
        case 4: return ncclInt32;
        case 5: return ncclUint8;
        case 6: return ncclFloat64;
        default: return ncclFloat32;
    }
}

ncclRedOp_t to_op(int32_t op) {
    switch (op) {
        case 0: return ncclSum;
        case 1: return ncclAvg;
        case 2: return ncclMax;
        case 3: return ncclMin;
        default: return ncclSum;
    }
}

}  // namespace

extern "C" {

const char* imc_last_error() { return g_err; }

int32_t imc_unique_id_bytes() { return (int32_t)sizeof(ncclUniqueId); }

int32_t imc_get_unique_id(char* out) {
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof(id));
    return 0;
}

int32_t imc_version() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
}

// Wait out ncclInProgress on a non-blocking communicator (enqueue calls return
// it while lazy connection set-up finishes in RCCL's own thread). Bounded: an
// abort from the watchdog thread, or SETTLE_LIMIT_S without progress, ends the
// wait with an error instead of spinning on a communicator being torn down.
constexpr double SETTLE_LIMIT_S = 600.0;

static ncclResult_t settle(Comm* c, ncclResult_t r) {
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress) {
        if (c->aborting.load(std::memory_order_acquire)) return ncclInvalidUsage;
        ncclResult_t st = ncclSuccess;
        ncclResult_t q = ncclCommGetAsyncError(c->comm, &st);
        if (q != ncclSuccess) return q;
        r = st;
        if (r == ncclInProgress &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > SETTLE_LIMIT_S)
            return ncclSystemError;
    }
    return r;
}

// A call's use of the communicator: counted in `inflight` from before the aborting check to the
// end of the call (sequentially consistent with imc_abort's flag-then-drain, so either the call sees
// the flag or the abort sees the call).
struct InFlight {
    Comm* c;
    bool ok;
    explicit InFlight(Comm* c_) : c(c_) {
        c->inflight.fetch_add(1, std::memory_order_seq_cst);
        ok = !c->aborting.load(std::memory_order_seq_cst);
    }
    ~InFlight() { c->inflight.fetch_sub(1, std::memory_order_seq_cst); }
    InFlight(const InFlight&) = delete;
    InFlight& operator=(const InFlight&) = delete;
};

#define NCCLCALL(c, x)                                                                \
    do {                                                                              \
        InFlight g_(c);                                                               \
        if (!g_.ok) {                                                                 \
            snprintf(g_err, sizeof(g_err), "communicator aborted");                   \
            return -3;                                                                \
        }                                                                             \
        ncclResult_t r_ = settle((c), (x));                                           \
        if (r_ != ncclSuccess) {                                                      \
            snprintf(g_err, sizeof(g_err), "%s: %s", #x, ncclGetErrorString(r_));     \
            return -2;                                                                \
        }                                                                             \
    } while (0)

// Start creating the communicator and its comm stream on `device`.
// nonblocking != 0: ncclCommInitRankConfig(blocking = 0) returns at once and
// imc_comm_poll() reports progress, so a rank whose peer failed can abort the
// half-built communicator (imc_abort) instead of waiting in the bootstrap
// forever. nonblocking == 0: classic blocking ncclCommInitRank.
int32_t imc_comm_init_start(const char* id_bytes, int32_t nranks, int32_t rank, int32_t device,
                            int32_t n_events, int32_t nonblocking, void** out) {
    HIPCHK(hipSetDevice(device));
    Comm* c = new Comm();
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    c->n_events = n_events < 4 ? 4 : n_events;
    ncclUniqueId id;
    std::memcpy(&id, id_bytes, sizeof(id));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = nonblocking ? 0 : 1;
    ncclResult_t r = ncclCommInitRankConfig(&c->comm, nranks, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
        snprintf(g_err, sizeof(g_err), "ncclCommInitRankConfig: %s", ncclGetErrorString(r));
        if (c->comm) ncclCommAbort(c->comm);
        delete c;
        return -2;
    }
    *out = c;
    return 0;
}

// Once the communicator is ready: create the comm stream and its events.
// Created AFTER RCCL's own init (which makes its internal streams): HIP hands
// streams to the GPU_MAX_HW_QUEUES hardware queues round-robin in creation
// order, and creating ours first was measured to land the wgrad side stream
// on a shared queue (R50/1024: 12.0k -> 10.6k img/s on one MI355X).
// Stream kinds: 0 plain, 1 highest priority, 2 full-CU-mask stream (the HIP
// runtime gives a CU-masked stream a hardware queue of its own instead of
// sharing one of the GPU_MAX_HW_QUEUES round-robin queues, so a barrier packet
// on it can never stall another stream's kernels queued behind it).
static int32_t create_stream(int32_t mode, hipStream_t* out) {
    if (mode == 2) {
        int dev = 0, ncu = 0;
        HIPCHK(hipGetDevice(&dev));
        HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        std::vector<uint32_t> mask((ncu + 31) / 32, 0xffffffffu);
        HIPCHK(hipExtStreamCreateWithCUMask(out, (uint32_t)mask.size(), mask.data()));
        return 0;
    }
    if (mode == 1) {
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        // `hi` is the numerically smallest == highest priority.
        HIPCHK(hipStreamCreateWithPriority(out, hipStreamNonBlocking, hi));
        return 0;
    }
    HIPCHK(hipStreamCreateWithFlags(out, hipStreamNonBlocking));
    return 0;
}

static int32_t finish_setup(Comm* c) {
    if (c->stream) return 0;
    int32_t rc = create_stream(c->stream_mode, &c->stream);
    if (rc) return rc;
    c->events.resize(c->n_events);
    for (auto& e : c->events) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return 0;
}

// Kind of comm stream finish_setup() creates (see create_stream); call before
// the communicator is ready.
int32_t imc_comm_set_stream_mode(void* h, int32_t mode) {
    static_cast<Comm*>(h)->stream_mode = mode;
    return 0;
}

// A stream of the given kind for other users (the weight-gradient side stream).
int32_t imc_stream_create(int32_t device, int32_t mode, void** out) {
    HIPCHK(hipSetDevice(device));
    hipStream_t s = nullptr;
    int32_t rc = create_stream(mode, &s);
    *out = s;
    return rc;
}

int32_t imc_stream_destroy(void* s) {
    HIPCHK(hipStreamDestroy((hipStream_t)s));
    return 0;
}

// 0: ready, 1: still initialising, < 0: failed (message in imc_last_error).
int32_t imc_comm_poll(void* h) {
    Comm* c = static_cast<Comm*>(h);
    if (!c || !c->comm) {
        snprintf(g_err, sizeof(g_err), "communicator aborted");
        return -3;
    }
    ncclResult_t st = ncclSuccess;
    {
        InFlight g(c);
        if (!g.ok) {
            snprintf(g_err, sizeof(g_err), "communicator aborted");
            return -3;
        }
        ncclResult_t q = ncclCommGetAsyncError(c->comm, &st);
        if (q != ncclSuccess) st = q;
    }
    if (st == ncclInProgress) return 1;
    if (st != ncclSuccess) {
        snprintf(g_err, sizeof(g_err), "ncclCommInitRank: %s", ncclGetErrorString(st));
        return -2;
    }
    return finish_setup(c);
}

// Blocking creation (kept for tools): start + wait.
int32_t imc_comm_init(const char* id_bytes, int32_t nranks, int32_t rank, int32_t device,
                      int32_t n_events, void** out) {
    int32_t rc = imc_comm_init_start(id_bytes, nranks, rank, device, n_events, 0, out);
    return rc ? rc : imc_comm_poll(*out);
}

int32_t imc_comm_nranks(void* h) {
    Comm* c = static_cast<Comm*>(h);
    int n = -1;
    if (!c || !c->comm) return n;
    InFlight g(c);
    if (g.ok && ncclCommCount(c->comm, &n) != ncclSuccess) n = -1;
    return n;
}

int32_t imc_comm_destroy(void* h) {
    Comm* c = static_cast<Comm*>(h);
    if (!c) return 0;
    int expect = 0;
    if (c->owner.compare_exchange_strong(expect, 2, std::memory_order_seq_cst)) {
        // drain the comm stream by polling, not a blocking sync: a collective hung on a dead peer never finishes,
        // and the watchdog's imc_abort (which lost the ownership race to this destroy) only raises `aborting` --
        // seeing it, this thread stops waiting and calls ncclCommAbort itself, which unblocks the stream
        while (c->stream && !c->aborting.load(std::memory_order_seq_cst) && hipStreamQuery(c->stream) == hipErrorNotReady)
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        if (c->comm) {
            // a non-blocking communicator finalises asynchronously; settle() leaves early once a concurrent
            // imc_abort raised `aborting` (that abort lost the ownership race and does not touch the handle)
            if (!c->aborting.load(std::memory_order_seq_cst) && settle(c, ncclCommFinalize(c->comm)) == ncclSuccess)
                ncclCommDestroy(c->comm);
            else
                ncclCommAbort(c->comm);
        }
        c->torn.store(true, std::memory_order_seq_cst);
    } else if (expect == 1) {
        // the watchdog's abort owns the teardown: wait for it (bounded by its drain + ncclCommAbort)
        while (!c->torn.load(std::memory_order_seq_cst)) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    } else {
        return 0;  // destroyed before
    }
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& e : c->events) (void)hipEventDestroy(e);
    c->events.clear();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    c->stream = nullptr;
    return 0;
}

void* imc_comm_stream(void* h) { return static_cast<Comm*>(h)->stream; }

// comm stream waits for everything issued so far on `src`.
int32_t imc_stream_join_from(void* h, void* src) {
    Comm* c = static_cast<Comm*>(h);
    hipEvent_t e = c->next();
    HIPCHK(hipEventRecord(e, (hipStream_t)src));
    HIPCHK(hipStreamWaitEvent(c->stream, e, 0));
    return 0;
}

// `dst` waits for everything issued so far on the comm stream.
int32_t imc_stream_join_into(void* h, void* dst) {
    Comm* c = static_cast<Comm*>(h);
    hipEvent_t e = c->next();
    HIPCHK(hipEventRecord(e, c->stream));
    HIPCHK(hipStreamWaitEvent((hipStream_t)dst, e, 0));
    return 0;
}

// In-place all-reduce of `count` elements at `ptr` on the comm stream,
// ordered after the work already issued on `src` (pass null to skip).
int32_t imc_allreduce(void* h, void* ptr, uint64_t count, int32_t dtype, int32_t op, void* src) {
    Comm* c = static_cast<Comm*>(h);
    if (src) {
        int32_t rc = imc_stream_join_from(h, src);
        if (rc) return rc;
    }
    NCCLCALL(c, ncclAllReduce(ptr, ptr, count, to_nccl(dtype), to_op(op), c->comm, c->stream));
    return 0;
}

// Several all-reduces fused into one RCCL group launch.
int32_t imc_allreduce_group(void* h, int32_t n, void** ptrs, const uint64_t* counts,
                            int32_t dtype, int32_t op, void* src) {
    Comm* c = static_cast<Comm*>(h);
    if (src) {
        int32_t rc = imc_stream_join_from(h, src);
        if (rc) return rc;
    }
    InFlight g(c);
    if (!g.ok) {
        snprintf(g_err, sizeof(g_err), "communicator aborted");
        return -3;
    }
    NCCLCHK(ncclGroupStart());
    for (int32_t i = 0; i < n; ++i)
        NCCLCHK(ncclAllReduce(ptrs[i], ptrs[i], counts[i], to_nccl(dtype), to_op(op), c->comm,
                              c->stream));
    NCCLCALL(c, ncclGroupEnd());
    return 0;
}

int32_t imc_broadcast(void* h, void* ptr, uint64_t count, int32_t dtype, int32_t root, void* src) {
    Comm* c = static_cast<Comm*>(h);
    if (src) {
        int32_t rc = imc_stream_join_from(h, src);
        if (rc) return rc;
    }
    NCCLCALL(c, ncclBroadcast(ptr, ptr, count, to_nccl(dtype), root, c->comm, c->stream));
    return 0;
}

int32_t imc_allgather(void* h, const void* send, void* recv, uint64_t count, int32_t dtype,
                      void* src) {
    Comm* c = static_cast<Comm*>(h);
    if (src) {
        int32_t rc = imc_stream_join_from(h, src);
        if (rc) return rc;
    }
    NCCLCALL(c, ncclAllGather(send, recv, count, to_nccl(dtype), c->comm, c->stream));
    return 0;
}

int32_t imc_reduce_scatter(void* h, const void* send, void* recv, uint64_t recv_count,
                           int32_t dtype, int32_t op, void* src) {
    Comm* c = static_cast<Comm*>(h);
    if (src) {
        int32_t rc = imc_stream_join_from(h, src);
        if (rc) return rc;
    }
    NCCLCALL(c, ncclReduceScatter(send, recv, recv_count, to_nccl(dtype), to_op(op), c->comm,
                                  c->stream));
    return 0;
}

int32_t imc_synchronize(void* h) {
    Comm* c = static_cast<Comm*>(h);
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

// Non-blocking health check (failure detection): returns the async error
// state of the communicator (0 == ok).
int32_t imc_async_error(void* h) {
    Comm* c = static_cast<Comm*>(h);
    if (!c || !c->comm) return -3;
    InFlight g(c);
    if (!g.ok) return -3;  // aborted
    ncclResult_t st = ncclSuccess;
    ncclCommGetAsyncError(c->comm, &st);
    return st == ncclInProgress ? 0 : (int32_t)st;
}

// Failure path (the watchdog thread): flag first, wait (bounded) until no call is inside RCCL with
// this communicator -- an enqueue spinning in settle() sees the flag and leaves -- then abort
// (unblocks kernels waiting on dead peers). The Comm object and its handle are never freed or
// cleared here; later calls fail on the flag.
constexpr double ABORT_DRAIN_S = 5.0;

int32_t imc_abort(void* h) {
    Comm* c = static_cast<Comm*>(h);
    if (!c) return 0;
    c->aborting.store(true, std::memory_order_seq_cst);
    int expect = 0;
    if (!c->owner.compare_exchange_strong(expect, 1, std::memory_order_seq_cst)) return 0;  // destroy / abort ran
    if (c->comm) {
        const auto t0 = std::chrono::steady_clock::now();
        while (c->inflight.load(std::memory_order_seq_cst) > 0 &&
               std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < ABORT_DRAIN_S)
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        const int left = c->inflight.load(std::memory_order_seq_cst);
        if (left > 0)
            fprintf(stderr, "[imagent rccl] abort: drain timed out after %.0f s with %d call(s) still inside RCCL\n",
                    ABORT_DRAIN_S, left);
        ncclCommAbort(c->comm);
    }
    c->torn.store(true, std::memory_order_seq_cst);
    return 0;
}

}  // extern "C"
