// GPU backend of the multifrontal factorization's large fronts (rocSOLVER / rocBLAS).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>

#include "comm.hpp"
#include "spd_direct.hpp"

namespace aa {

// fronts of order >= min_front (AA_DENSE_MIN_FRONT, default 1024) are assembled and factored on
// the GPU of stream s; AA_DENSE_GPU=0 keeps the whole factorization on the host
std::unique_ptr<DenseFrontBackend> make_gpu_front_backend(hipStream_t s);

// Loads the backend's rocBLAS / rocSOLVER code objects on the stream's device once per process
// (one synthetic SPD front of the smallest GPU order through the same calls); returns the wall
// ms it took (0 if that device is already warm, or AA_DENSE_GPU=0)
double warm_gpu_front_backend(hipStream_t s);

// multifrontal_cholesky with the GPU backend (or on the host only, AA_DENSE_GPU=0)
// The partitioned factorization of rank `rank` over `comm` (PartFactor; part r = rank r): host
// fronts summed by comm's host all-reduce, device fronts by its all-reduce on stream s.
// Null (every rank factors the whole matrix) for a rehearsal communicator, one rank, or
// AA_PART_FACTOR=0.
std::unique_ptr<PartFactor> make_part_factor(Comm* comm, int rank, hipStream_t s);

// part: partitioned (one rank's share, see PartFactor)
SupernodalFactor factor_on_device(const CsrMatrix& A, const NdTree& tree, hipStream_t s, const PartFactor* part = nullptr);

}  // namespace aa
