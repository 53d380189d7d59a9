// GPU backend of the multifrontal factorization's large fronts (rocSOLVER / rocBLAS).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>

#include "spd_direct.hpp"

namespace aa {

// fronts of order >= min_front (AA_DENSE_MIN_FRONT, default 1024) are assembled and factored on
// the GPU of stream s; AA_DENSE_GPU=0 keeps the whole factorization on the host
std::unique_ptr<DenseFrontBackend> make_gpu_front_backend(hipStream_t s);

// multifrontal_cholesky with the GPU backend (or on the host only, AA_DENSE_GPU=0)
SupernodalFactor factor_on_device(const CsrMatrix& A, const NdTree& tree, hipStream_t s);

}  // namespace aa
