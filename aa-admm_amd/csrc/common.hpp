// Shared host/device utilities for the aa_admm HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

namespace aa {

enum Status { OK = 0, ERR_ARG = -1, ERR_STATE = -2, ERR_DEVICE = -3, ERR_NUMERIC = -4 };

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define AA_HIP(call)                                                                                   \
    do {                                                                                               \
        hipError_t e_ = (call);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            throw ::aa::Error(::aa::ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_) +    \
                                                    " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")"); \
    } while (0)

#define AA_CHECK_LAUNCH() AA_HIP(hipGetLastError())

// Owning device buffer (hipMalloc'd, never resized inside a time step).
template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    explicit DevBuf(size_t count) { alloc(count); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; return *this; }
    ~DevBuf() { release(); }
    void alloc(size_t count) {
        release();
        n = count;
        if (count) AA_HIP(hipMalloc(&p, count * sizeof(T)));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr; n = 0;
    }
    void upload(const std::vector<T>& h, hipStream_t s) {
        if (h.size() != n) alloc(h.size());
        if (n) AA_HIP(hipMemcpyAsync(p, h.data(), n * sizeof(T), hipMemcpyHostToDevice, s));
    }
    void upload(const T* h, size_t count, hipStream_t s) {
        if (count != n) alloc(count);
        if (n) AA_HIP(hipMemcpyAsync(p, h, n * sizeof(T), hipMemcpyHostToDevice, s));
    }
    void zero(hipStream_t s) { if (n) AA_HIP(hipMemsetAsync(p, 0, n * sizeof(T), s)); }
    size_t bytes() const { return n * sizeof(T); }
};

// Pinned (page-locked) host staging buffer that only grows. Host <-> device copies of setup data
// and of the host-staged all-reduce go through it, so they are plain DMA in stream order: the
// 4-rank partition test saw a top front's last column stale after a pageable hipMemcpyAsync +
// hipStreamSynchronize on one of four processes sharing the GPU (round 5).
template <typename T>
struct PinnedBuf {
    T* p = nullptr;
    size_t n = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() { if (p) (void)hipHostFree(p); }
    T* get(size_t count) {
        if (count > n) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            n = 0;
            AA_HIP(hipHostMalloc(reinterpret_cast<void**>(&p), count * sizeof(T), hipHostMallocDefault));
            n = count;
        }
        return p;
    }
};

// Records what `enqueue` puts on stream s into an instantiated graph. Returns false -- with the
// stream out of capture mode and nothing recorded kept -- when any part fails (e.g. a collective
// the communication library cannot capture); the caller then launches eagerly.
template <class F>
bool capture_graph(hipStream_t s, F&& enqueue, hipGraph_t* graph, hipGraphExec_t* exec) {
    *graph = nullptr;
    *exec = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    bool ok = true;
    try {
        enqueue();
    } catch (const Error&) {
        ok = false;
    }
    hipGraph_t g = nullptr;
    if (hipStreamEndCapture(s, &g) != hipSuccess) ok = false;
    if (ok && hipGraphInstantiate(exec, g, nullptr, nullptr, 0) != hipSuccess) {
        ok = false;
        *exec = nullptr;
    }
    if (!ok) {
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        return false;
    }
    *graph = g;
    return true;
}

constexpr int kBlock = 256;
inline int blocks_for(long long n, int block = kBlock) { return (int)((n + block - 1) / block); }

}  // namespace aa
