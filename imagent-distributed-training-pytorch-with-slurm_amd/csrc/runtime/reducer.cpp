// Native gradient-bucket runtime: bucket planner + per-iteration ready tracker.
//
// This is the bookkeeping half of the c10d DDP Reducer that the reference
// gets implicitly from `DistributedDataParallel(model, ...)`
// (/root/reference/imagenet.py:316; [torch] include/torch/csrc/distributed/
// c10d/reducer.hpp:30-31,73,79,135,275-285). The data half (flat gradient
// arena, RCCL all-reduce on a side HIP stream) lives in csrc/comm.
//
// Design (MI355X-first, not a translation of reducer.cpp):
//  * gradients live in ONE flat fp32 arena laid out in bucket order, so a
//    bucket is a contiguous slice and needs no copy-in/copy-out;
//  * buckets are launched strictly in index order (every rank issues its
//    collectives in the same order - required for RCCL correctness even if
//    the local ready order differs);
//  * the tracker records the observed ready order of an iteration so the
//    Python side can rebuild the layout once (torch DDP rebuilds after
//    iteration 1, [torch] nn/parallel/distributed.py:1551);
//  * errors the c10d reducer reports ("marked ready twice", "expected to
//    have finished reduction") are surfaced as return codes.
//
// Plain C ABI so it can be loaded with ctypes and has no torch/HIP deps.

#include <cstdint>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

extern "C" {

// Greedy size-capped bucketing over tensors in the given order.
// The first bucket is capped at `first_cap` bytes, later ones at `cap`
// (torch: kDefaultFirstBucketBytes = 1 MiB, kDefaultBucketBytesCap = 25 MiB).
// A bucket is closed as soon as it reaches its cap. `last_cap` > 0: the LAST
// bucket is at most that many bytes (or one tensor): the trailing tensors are
// split off the greedy last bucket -- it is the one all-reduce that cannot
// overlap backward (issued after the last gradient), so it is kept small.
// Returns #buckets.
int32_t imr_plan_buckets(int32_t n, const int64_t* nbytes, int64_t first_cap, int64_t cap, int64_t last_cap,
                         int32_t* bucket_of) {
    if (n <= 0) return 0;
    int32_t b = 0;
    int64_t acc = 0;
    int64_t limit = first_cap > 0 ? first_cap : cap;
    for (int32_t i = 0; i < n; ++i) {
        bucket_of[i] = b;
        acc += nbytes[i];
        if (acc >= limit && i + 1 < n) {
            ++b;
            acc = 0;
            limit = cap;
        }
    }
    if (last_cap > 0) {
        int32_t start = n - 1;  // first tensor of the tail (at least the last tensor)
        int64_t tail = nbytes[n - 1];
        while (start > 0 && bucket_of[start - 1] == b && tail + nbytes[start - 1] <= last_cap)
            tail += nbytes[--start];
        if (start > 0 && bucket_of[start - 1] == b) {  // the greedy last bucket holds more: split it
            ++b;
            for (int32_t i = start; i < n; ++i) bucket_of[i] = b;
        }
    }
    return b + 1;
}

struct Tracker {
    std::mutex mu;
    int32_t nparams = 0, nbuckets = 0;
    std::vector<int32_t> bucket_of;     // param -> bucket
    std::vector<int32_t> bucket_size;   // #params per bucket
    std::vector<int32_t> pending;       // per bucket, this iteration
    std::vector<uint8_t> marked;        // per param, this iteration
    std::vector<int32_t> order_cur, order_last;
    int32_t next_bucket = 0;            // first bucket not yet launched
    int64_t iterations = 0;
};

void* imr_tracker_new(int32_t nparams, const int32_t* bucket_of, int32_t nbuckets) {
    Tracker* t = new (std::nothrow) Tracker();
    if (!t) return nullptr;
    t->nparams = nparams;
    t->nbuckets = nbuckets;
    t->bucket_of.assign(bucket_of, bucket_of + nparams);
    t->bucket_size.assign(nbuckets, 0);
    for (int32_t i = 0; i < nparams; ++i) {
        if (bucket_of[i] < 0 || bucket_of[i] >= nbuckets) { delete t; return nullptr; }
        t->bucket_size[bucket_of[i]]++;
    }
    t->pending = t->bucket_size;
    t->marked.assign(nparams, 0);
    t->order_cur.reserve(nparams);
    return t;
}

void imr_tracker_free(void* h) { delete static_cast<Tracker*>(h); }

// Mark a parameter's gradient as final for this iteration.
// On success returns 0 and sets [*first, *first + *count) to the buckets
// that may now be launched (in order). -1: already marked this iteration
// (a parameter used twice in one forward); -2: bad index.
int32_t imr_tracker_mark(void* h, int32_t param, int32_t* first, int32_t* count) {
    Tracker* t = static_cast<Tracker*>(h);
    std::lock_guard<std::mutex> g(t->mu);
    *first = t->next_bucket;
    *count = 0;
    if (param < 0 || param >= t->nparams) return -2;
    if (t->marked[param]) return -1;
    t->marked[param] = 1;
    t->order_cur.push_back(param);
    t->pending[t->bucket_of[param]]--;
    while (t->next_bucket < t->nbuckets && t->pending[t->next_bucket] == 0) {
        t->next_bucket++;
        (*count)++;
    }
    return 0;
}

// End of backward: returns the number of buckets that were NOT launched
// (0 == every gradient arrived) and resets the state for the next iteration.
// `unready` (optional, size nparams) receives 1 for each param never marked.
int32_t imr_tracker_finalize(void* h, uint8_t* unready) {
    Tracker* t = static_cast<Tracker*>(h);
    std::lock_guard<std::mutex> g(t->mu);
    int32_t missing = t->nbuckets - t->next_bucket;
    if (unready) for (int32_t i = 0; i < t->nparams; ++i) unready[i] = t->marked[i] ? 0 : 1;
    t->order_last.swap(t->order_cur);
    t->order_cur.clear();
    t->pending = t->bucket_size;
    std::fill(t->marked.begin(), t->marked.end(), 0);
    t->next_bucket = 0;
    t->iterations++;
    return missing;
}

// Observed ready order of the last finalized iteration. Returns its length.
int32_t imr_tracker_last_order(void* h, int32_t* out) {
    Tracker* t = static_cast<Tracker*>(h);
    std::lock_guard<std::mutex> g(t->mu);
    if (out) std::memcpy(out, t->order_last.data(), t->order_last.size() * sizeof(int32_t));
    return static_cast<int32_t>(t->order_last.size());
}

int64_t imr_tracker_iterations(void* h) { return static_cast<Tracker*>(h)->iterations; }

int32_t imr_version() { return 1; }

}  // extern "C"
