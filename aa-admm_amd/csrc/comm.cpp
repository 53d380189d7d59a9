// RCCL and host-callback transports of aa::Comm (see comm.hpp).
#include "comm.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>

#include "common.hpp"

namespace aa {

namespace {

// librccl entry points, resolved once (types from the header, symbols at run time)
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

// Directory of the shared object that defines `addr` ("" if unknown).
std::string object_dir(const void* addr) {
    Dl_info info;
    if (!addr || !dladdr(addr, &info) || !info.dli_fname) return "";
    std::string f = info.dli_fname;
    size_t k = f.rfind('/');
    return k == std::string::npos ? std::string() : f.substr(0, k);
}

std::string object_path(const void* addr) {
    Dl_info info;
    if (!addr || !dladdr(addr, &info) || !info.dli_fname) return "";
    return info.dli_fname;
}

std::string hip_runtime_dir() { return object_dir(reinterpret_cast<const void*>(&hipGetDeviceCount)); }

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    static std::string err;
    std::call_once(once, [] {
        // RCCL from the directory of the HIP runtime this library is bound to, so a process never
        // pairs one ROCm release's HIP with another's RCCL; the loader's search only as a fallback
        void* h = nullptr;
        std::string dir = hip_runtime_dir();
        if (!dir.empty()) h = dlopen((dir + "/librccl.so.1").c_str(), RTLD_NOW | RTLD_GLOBAL);
        for (const char* name : {"librccl.so.1", "librccl.so"}) {
            if (h) break;
            h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
        }
        if (!h) { err = std::string("cannot load librccl: ") + dlerror(); return; }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.error_string) {
            err = "librccl: missing symbols";
            r = Rccl{};
        }
    });
    if (!r.all_reduce) throw Error(ERR_DEVICE, err.empty() ? "librccl unavailable" : err);
    return r;
}

// Whether a partitioned step records its device all-reduces into the step's hipGraph (see
// RcclComm::capturable). The rehearsal transport follows the same rule, so bench.py --rehearse
// times the launch mode a real P-GPU run uses.
bool rccl_graph() {
    const char* e = std::getenv("AA_RCCL_GRAPH");
    return e && e[0] == '1';
}

void nccl_check(ncclResult_t rc, const char* what) {
    if (rc != ncclSuccess) throw Error(ERR_DEVICE, std::string(what) + ": " + rccl().error_string(rc));
}

class RcclComm final : public Comm {
public:
    RcclComm(const unsigned char id[128], int rank, int size) {
        rank_ = rank; size_ = size;
        ncclUniqueId uid;
        static_assert(sizeof(uid) == 128, "ncclUniqueId must be 128 bytes");
        std::memcpy(&uid, id, 128);
        nccl_check(rccl().comm_init_rank(&comm_, size, uid, rank), "ncclCommInitRank");
    }
    ~RcclComm() override {
        if (comm_) (void)rccl().comm_destroy(comm_);
        if (hs_) (void)hipStreamDestroy(hs_);
    }
    void allreduce_sum(const double* src, double* dst, size_t n, hipStream_t s) override {
        if (n == 0) return;
        nccl_check(rccl().all_reduce(src, dst, n, ncclDouble, ncclSum, comm_, s), "ncclAllReduce");
    }
    void allreduce_sum_host(double* buf, size_t n) override {
        if (n == 0) return;
        // through pinned staging (common.hpp PinnedBuf), copies and the sum ordered on one stream;
        // every device sum this rank enqueued before (the solver's stream is non-blocking) has
        // finished first, so the ranks' collectives reach the communicator in program order
        AA_HIP(hipDeviceSynchronize());
        double* h = stage_.get(n);
        std::memcpy(h, buf, n * sizeof(double));
        if (dstage_.n < n) dstage_.alloc(n);
        double* d = dstage_.p;
        if (!hs_) AA_HIP(hipStreamCreateWithFlags(&hs_, hipStreamNonBlocking));
        AA_HIP(hipMemcpyAsync(d, h, n * sizeof(double), hipMemcpyHostToDevice, hs_));
        nccl_check(rccl().all_reduce(d, d, n, ncclDouble, ncclSum, comm_, hs_), "ncclAllReduce");
        AA_HIP(hipMemcpyAsync(h, d, n * sizeof(double), hipMemcpyDeviceToHost, hs_));
        AA_HIP(hipStreamSynchronize(hs_));
        std::memcpy(buf, h, n * sizeof(double));
    }
    // Eager by default: a partitioned step with RCCL launches its kernels and all-reduces
    // without a hipGraph (the device-side control still needs no host sync, and at P ranks the
    // kernels are long enough for the host to stay ahead). AA_RCCL_GRAPH=1 records
    // ncclAllReduce into the step's graph instead (a failed capture on any rank drops every
    // rank back to eager launches) -- opt-in until a multi-rank RCCL capture has been verified.
    bool capturable() const override { return rccl_graph(); }

private:
    ncclComm_t comm_ = nullptr;
    PinnedBuf<double> stage_;
    DevBuf<double> dstage_;
    hipStream_t hs_ = nullptr;
};

class HostComm final : public Comm {
public:
    HostComm(HostAllreduceFn fn, void* user, int rank, int size) : fn_(fn), user_(user) { rank_ = rank; size_ = size; }
    void allreduce_sum(const double* src, double* dst, size_t n, hipStream_t s) override {
        if (n == 0) return;
        double* b = buf_.get(n);   // pinned: the copies are stream-ordered DMA (common.hpp PinnedBuf)
        AA_HIP(hipMemcpyAsync(b, src, n * sizeof(double), hipMemcpyDeviceToHost, s));
        AA_HIP(hipStreamSynchronize(s));
        allreduce_sum_host(b, n);
        AA_HIP(hipMemcpyAsync(dst, b, n * sizeof(double), hipMemcpyHostToDevice, s));
        AA_HIP(hipStreamSynchronize(s));
    }
    void allreduce_sum_host(double* buf, size_t n) override {
        if (n == 0) return;
        if (fn_(buf, (long long)n, user_) != 0) throw Error(ERR_DEVICE, "host all-reduce callback failed");
        if (verify_) check_same(buf, n);
    }
    bool capturable() const override { return false; }

private:
    // AA_COMM_VERIFY=1 (tests): every rank must hold the same bits after a sum -- a 64-bit FNV-1a
    // hash of the result, its halves summed over the ranks, must equal size x this rank's
    void check_same(const double* buf, size_t n) {
        unsigned long long h = 1469598103934665603ull;
        const unsigned char* b = reinterpret_cast<const unsigned char*>(buf);
        for (size_t i = 0; i < n * sizeof(double); ++i) { h ^= b[i]; h *= 1099511628211ull; }
        double v[2] = {(double)(h >> 32), (double)(h & 0xffffffffull)}, mine[2] = {v[0], v[1]};
        if (fn_(v, 2, user_) != 0) throw Error(ERR_DEVICE, "host all-reduce callback failed");
        if (v[0] != size_ * mine[0] || v[1] != size_ * mine[1])
            throw Error(ERR_DEVICE, "host all-reduce: the ranks hold different sums (" + std::to_string(n) + " values)");
    }
    HostAllreduceFn fn_;
    void* user_;
    PinnedBuf<double> buf_;
    bool verify_ = std::getenv("AA_COMM_VERIFY") && std::getenv("AA_COMM_VERIFY")[0] == '1';
};

// Rehearsal transport: ONE rank of a P-way partition on its own GPU, every other rank absent.
// A device all-reduce leaves the local values (dst = src), a host all-reduce multiplies by P
// (as if every rank held the same values: the setup's scene-identity checks pass, agreement
// flags stay set). The numbers it produces are not a solution -- it exists to time one rank's
// kernels of a P-GPU run (bench.py --rehearse P), launched the way production launches them
// (eager unless AA_RCCL_GRAPH=1, as the RCCL transport).
class SoloComm final : public Comm {
public:
    SoloComm(int rank, int size) { rank_ = rank; size_ = size; }
    void allreduce_sum(const double* src, double* dst, size_t n, hipStream_t s) override {
        if (n && src != dst) AA_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDevice, s));
    }
    void allreduce_sum_host(double* buf, size_t n) override {
        for (size_t i = 0; i < n; ++i) buf[i] *= size_;
    }
    bool capturable() const override { return rccl_graph(); }
    bool rehearsal() const override { return true; }
};

}  // namespace

std::string runtime_libraries() {
    try { (void)rccl(); } catch (const Error&) {}   // loads librccl (no device call); absent = empty path
    auto sym = [](const char* name) -> const void* { return dlsym(RTLD_DEFAULT, name); };
    const std::pair<const char*, const char*> probes[] = {
        {"amdhip64", "hipMalloc"}, {"hsa-runtime64", "hsa_init"}, {"rocblas", "rocblas_create_handle"},
        {"rocsolver", "rocsolver_dpotrf"}, {"rccl", "ncclAllReduce"}};
    std::string out;
    for (const auto& p : probes) out += std::string(p.first) + "=" + object_path(sym(p.second)) + "\n";
    return out;
}

std::unique_ptr<Comm> make_solo_comm(int rank, int size) { return std::unique_ptr<Comm>(new SoloComm(rank, size)); }

void rccl_unique_id(unsigned char out[128]) {
    ncclUniqueId uid;
    nccl_check(rccl().get_unique_id(&uid), "ncclGetUniqueId");
    std::memcpy(out, &uid, 128);
}

std::unique_ptr<Comm> make_rccl_comm(const unsigned char id[128], int rank, int size) {
    return std::unique_ptr<Comm>(new RcclComm(id, rank, size));
}

std::unique_ptr<Comm> make_host_comm(HostAllreduceFn fn, void* user, int rank, int size) {
    if (!fn) throw Error(ERR_ARG, "host all-reduce: null callback");
    return std::unique_ptr<Comm>(new HostComm(fn, user, rank, size));
}

}  // namespace aa
