// Internal helpers shared by the libmpo.so translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <map>
#include <tuple>
#include <mutex>
#include <string>
#include <utility>

#include "../../include/mpo.h"

namespace mpo {

// Thread-local message of the last failure (returned by mpo_last_error()).
void set_error(const char* fmt, ...);
void clear_error();

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Carve consecutive 256-B aligned regions out of a caller workspace.
struct WsCarver {
    char* base;
    size_t used = 0;
    explicit WsCarver(void* p) : base(static_cast<char*>(p)) {}
    template <class T>
    T* take(size_t count) {
        used = align_up(used, 256);
        T* p = base ? reinterpret_cast<T*>(base + used) : nullptr;
        used += count * sizeof(T);
        return p;
    }
};

// Makes the device a stream belongs to current for the scope of an entry point
// and restores the caller's afterwards: entry points that query or configure the
// device (hipFuncSetAttribute, attributes, pinned-pointer lookups) then target the
// stream's GPU whatever device the calling thread has current.
struct StreamDeviceScope {
    int prev = -1, dev = -1;
    explicit StreamDeviceScope(hipStream_t s) {
        if (s == nullptr || hipGetDevice(&prev) != hipSuccess || hipStreamGetDevice(s, &dev) != hipSuccess) {
            (void)hipGetLastError();
            prev = dev = -1;
            return;
        }
        if (dev != prev && hipSetDevice(dev) != hipSuccess) {
            (void)hipGetLastError();
            prev = dev = -1;
        }
    }
    ~StreamDeviceScope() {
        if (prev >= 0 && dev != prev) (void)hipSetDevice(prev);
    }
    StreamDeviceScope(const StreamDeviceScope&) = delete;
    StreamDeviceScope& operator=(const StreamDeviceScope&) = delete;
};

// A second stream for independent launches of one step, on the caller's stream's
// device, forked from / joined into that stream with events (created on first use,
// re-created if the caller moves to another device).  get() returns nullptr when
// disabled or when the stream / events cannot be created (the step then runs
// serially on the caller's stream).
// The side streams themselves come from one process-wide pool per (device, caller
// stream, slot): every population engine stepped from the same caller stream shares
// them, so a process that holds several engines (a search: one per population,
// DenseNet and MNIST) keeps the same few streams -- with one pair of streams per
// engine, a 40-member engine stepped 15% slower while a second, idle engine was alive
// (6.53 vs 5.69 ms; 5.69 with pooled streams: profiles/r05/shard_ratio_probe.log).
// Engines stepped from DISTINCT caller streams get distinct side streams (r06), so a
// join never waits for another caller's work: the ABI's "thread-safe across streams"
// contract holds for them (tests/test_train_gpu.py::
// test_engines_on_two_threads_and_streams_keep_their_bits).  Engines sharing a caller
// stream are serialised by that stream anyway.  The fork / join events stay per engine.
inline hipStream_t pooled_side_stream(int dev, hipStream_t caller, int slot) {
    static std::mutex mu;
    static std::map<std::tuple<int, hipStream_t, int>, hipStream_t> pool;
    std::lock_guard<std::mutex> lk(mu);
    auto it = pool.find({dev, caller, slot});
    if (it != pool.end()) return it->second;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dev);
    hipStream_t st = nullptr;
    const bool ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
    (void)hipSetDevice(cur);
    if (!ok) { (void)hipGetLastError(); return nullptr; }
    pool[{dev, caller, slot}] = st;   // lives for the process
    return st;
}

struct SideStream {
    bool enabled = true;
    int slot = 0;   // which pooled stream (0: the side stream, 1: a third stream)
    hipStream_t side = nullptr;
    hipStream_t caller = nullptr;   // the caller stream `side` was pooled for
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int device = -1;
    SideStream() = default;
    SideStream(const SideStream&) = delete;
    SideStream& operator=(const SideStream&) = delete;
    ~SideStream() { release(); }
    void release() {
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (ev_join) (void)hipEventDestroy(ev_join);
        side = nullptr;   // pooled: not destroyed
        caller = nullptr;
        ev_fork = ev_join = nullptr;
        device = -1;
    }
    hipStream_t get(hipStream_t s) {
        if (!enabled) return nullptr;
        int dev = 0;
        if (hipStreamGetDevice(s, &dev) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
        if (side && dev == device) {
            if (s == caller) return side;
            side = pooled_side_stream(dev, s, slot);   // same device, another caller stream
            if (!side) { release(); enabled = false; return nullptr; }
            caller = s;
            return side;
        }
        release();
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(dev);
        side = pooled_side_stream(dev, s, slot);
        caller = s;
        const bool ok = side && hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming) == hipSuccess &&
                        hipEventCreateWithFlags(&ev_join, hipEventDisableTiming) == hipSuccess;
        (void)hipSetDevice(cur);
        if (!ok) { (void)hipGetLastError(); release(); enabled = false; return nullptr; }
        device = dev;
        return side;
    }
    // s2 starts after everything enqueued on s so far
    hipError_t fork(hipStream_t s, hipStream_t s2) {
        if (hipError_t e = hipEventRecord(ev_fork, s)) return e;
        return hipStreamWaitEvent(s2, ev_fork, 0);
    }
    // s continues after everything enqueued on s2 so far
    hipError_t join(hipStream_t s, hipStream_t s2) {
        if (hipError_t e = hipEventRecord(ev_join, s2)) return e;
        return hipStreamWaitEvent(s, ev_join, 0);
    }
};

// Static (compile-time) LDS bytes of a kernel, from its code object.
inline size_t static_lds_bytes(const void* kern) {
    hipFuncAttributes at{};
    if (hipFuncGetAttributes(&at, kern) != hipSuccess) {
        (void)hipGetLastError();
        return SIZE_MAX / 2;
    }
    return at.sharedSizeBytes;
}

// One pending L-BFGS-B round of one GP refit (gp_fit.hip): `batch` thetas of the
// problem (X, y, n) in the layout mpo_gp_lml_grad_host uses.  lml_launch_rounds
// evaluates the rounds of several refits in one launch set (same d, every n
// lml_groupable: the fused split sweep), enqueued on `s`, not synchronised.
struct LmlRound {
    const double* X;
    const double* y;
    int n, d, batch;
    double* theta_dev;         // [batch][d+2] device: the build's copy of theta_src
    const double* theta_src;   // [batch][d+2] pinned host, device view
    double* out;               // pinned host, device view: lml [batch] | grad [batch][d+2] | info
    double* ws;                // 256-B aligned, mpo_gp_lml_ws_bytes(n, d, batch)
};
bool lml_groupable(int n, int d);
int lml_launch_rounds(const LmlRound* r, int count, hipStream_t s);

}  // namespace mpo

#define MPO_CHECK_ARG(cond, ...)              \
    do {                                      \
        if (!(cond)) {                        \
            ::mpo::set_error(__VA_ARGS__);    \
            return MPO_EINVAL;                \
        }                                     \
    } while (0)

#define MPO_HIP(call)                                                             \
    do {                                                                          \
        hipError_t e_ = (call);                                                   \
        if (e_ != hipSuccess) {                                                   \
            ::mpo::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call,           \
                             hipGetErrorString(e_));                              \
            return MPO_EHIP;                                                      \
        }                                                                         \
    } while (0)

#define MPO_LAUNCH_CHECK() MPO_HIP(hipGetLastError())

#define MPO_GUARD_BEGIN try {
#define MPO_GUARD_END                                         \
    }                                                         \
    catch (...) {                                             \
        ::mpo::set_error("unexpected C++ exception");         \
        return MPO_EHIP;                                      \
    }
