// Inter-GPU reductions of the partitioned solver.
//
// The reference is a single OpenMP process (no MPI / NCCL anywhere). When the mesh is split
// over several MI355X (one process per GPU), each ADMM iteration needs a handful of SUM
// all-reduces of small fp64 vectors: residual block partials, the Anderson partials, and the
// separator rows of the partitioned global solve (tens of kB). Two transports:
//   * RCCL over xGMI (production): ncclAllReduce enqueued on the solver's stream, so the
//     reduction is ordered with the kernels and the ADMM loop needs no host round trip.
//     librccl is opened at run time (dlopen) so the library loads without it and shares
//     the copy a PyTorch process already holds.
//   * host callback: the stream is synchronised, the vector staged through host memory and
//     handed to a caller-supplied function (e.g. torch.distributed over gloo). Used to run
//     several ranks on ONE GPU in tests; never graph-capturable.
// Both give every rank bit-identical sums, so the device-side control decisions (Anderson
// reject, break) agree on all ranks without further communication.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <memory>
#include <string>
#include <vector>

namespace aa {

typedef int (*HostAllreduceFn)(double* buf, long long n, void* user);

class Comm {
public:
    virtual ~Comm() = default;
    int rank() const { return rank_; }
    int size() const { return size_; }
    // dst = SUM over ranks of src (n doubles in device memory, src == dst allowed), ordered on stream s
    virtual void allreduce_sum(const double* src, double* dst, size_t n, hipStream_t s) = 0;
    // in-place SUM of a host array (setup-time agreements); blocking
    virtual void allreduce_sum_host(double* buf, size_t n) = 0;
    virtual bool capturable() const = 0;   // may be recorded into a hipGraph
    virtual bool rehearsal() const { return false; }   // solo timing rehearsal: results are not a solution

protected:
    int rank_ = 0, size_ = 1;
};

void rccl_unique_id(unsigned char out[128]);
// "name=path\n" of the HIP, HSA, rocBLAS, rocSOLVER and RCCL objects this process has bound (dladdr)
std::string runtime_libraries();
std::unique_ptr<Comm> make_rccl_comm(const unsigned char id[128], int rank, int size);
std::unique_ptr<Comm> make_host_comm(HostAllreduceFn fn, void* user, int rank, int size);
std::unique_ptr<Comm> make_solo_comm(int rank, int size);   // timing rehearsal of one rank (comm.cpp)

}  // namespace aa
