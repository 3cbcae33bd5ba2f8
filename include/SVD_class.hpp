// SVD_class.hpp -- drop-in replacement for the reference's include/SVD_class.hpp: the same
// `enum class SVDMethod` and `template<SVDMethod method> class SVD` (constructor, compute(),
// getU/getS/getV, protected setData for subclasses such as PCA_class.hpp:12), backed by the MI355X
// engine (rsvd_svd, dense_api.cpp) through include/rsvd.hpp.
//
//   Jacobi / ParallelJacobi (SVD_class.hpp:100-180, :223-333): U m x k, S k (descending), V n x k,
//     k = min(m, n) <= 4096.  Both reference methods converge to the same SVD (up to signs of
//     singular-vector pairs); the GPU runs one-sided Jacobi on the QR-preconditioned triangle.
//   Power (SVD_class.hpp:183-219, src/PM.cpp): the reference's layouts -- U m x m and V n x n
//     identity-initialised with u_i in column i of U and v_i in ROW i of V, S of length min(m, n),
//     cut to the first i columns on an early stop (sigma < 1e-12).  Any n.  Start vectors come
//     from the Philox stream (RSVD_SEED) instead of std::random_device.
// compute() prints nothing (the reference writes progress lines to stdout, :80-95).
#ifndef SVD_CLASS_HPP
#define SVD_CLASS_HPP

#include <Eigen/Dense>

#include "rsvd.hpp"

using Mat_m = Eigen::MatrixXd;
using Vec_v = Eigen::VectorXd;

#ifndef RSVD_SVDMETHOD_DECLARED
#define RSVD_SVDMETHOD_DECLARED
enum class SVDMethod { Jacobi, Power, ParallelJacobi };
#endif

template <SVDMethod method>
class SVD : public rsvd::SVDT<static_cast<rsvd::Method>(static_cast<int>(method)), Mat_m, Vec_v> {
    using Base = rsvd::SVDT<static_cast<rsvd::Method>(static_cast<int>(method)), Mat_m, Vec_v>;

public:
    SVD(const Mat_m &data, const int &r = 0) : Base(data, r) {}
};

#endif
