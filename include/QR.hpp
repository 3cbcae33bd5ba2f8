// QR.hpp -- drop-in replacement for the reference's include/QR.hpp (same names and signatures on
// Eigen types), backed by the MI355X engine (rsvd_qr, dense_api.cpp) through include/rsvd.hpp.
//
//   void qr_decomposition_full(const Mat_m &A, Mat_m &Q, Mat_m &R);     QR.hpp:15, src/QR.cpp:22-41
//   void qr_decomposition_reduced(const Mat_m &A, Mat_m &Q, Mat_m &R);  QR.hpp:16, src/QR.cpp:43-80
//
// Q has orthonormal columns, A = Q R, R upper triangular (trapezoidal for the full QR) with the
// Givens sign convention: R(j,j) >= 0 except where the reference's sweep never rotates (leading
// columns whose sub-diagonal is already zero keep the sign of A(j,j); a square Q has det +1).  The
// reduced form requires rows >= cols (std::invalid_argument otherwise, where the reference's Eigen
// block would assert).  Any size (past 512 columns: blocked CGS2 + CholeskyQR3, dense_big.cpp).
// The reference header also declares `Mat_m givens_rotation(double, double)` without defining it
// (QR.hpp:14 vs src/QR.cpp:12); the defined overload is provided here.
#ifndef QR_HPP
#define QR_HPP

#include <Eigen/Dense>
#include <cmath>

#include "rsvd.hpp"

using Mat_m = Eigen::MatrixXd;
using Vec_v = Eigen::VectorXd;

inline void givens_rotation(double a, double b, Eigen::Matrix2d &G) {  // src/QR.cpp:12-20
    const double r = std::hypot(a, b);
    const double c = a / r, s = -b / r;
    G << c, -s, s, c;
}

inline void qr_decomposition_full(const Mat_m &A, Mat_m &Q, Mat_m &R) { rsvd::qr_full(A, Q, R); }

inline void qr_decomposition_reduced(const Mat_m &A, Mat_m &Q, Mat_m &R) { rsvd::qr_reduced(A, Q, R); }

#endif
