// rSVD.hpp -- drop-in replacement for the reference's include/rSVD.hpp (same names, same
// signatures, same Eigen types), backed by the MI355X engine through include/rsvd.hpp.
//
//   void intermediate_step(const Mat_m &A, Mat_m &Q, const Mat_m &Omega, int l, int q);  rSVD.hpp:13
//   void rSVD(Mat_m &A, Mat_m &U, Vec_v &S, Mat_m &V, int l, SVDMethod method);         rSVD.hpp:14
//   Mat_m generateOmega(int n, int l);                                                   rSVD.hpp:15
//   void rSVD(Mat_m &A, Mat_m &U, Vec_v &S, Mat_m &V, int l);  image_compression/include/rSVD.hpp
//
// Link with -lrsvd_hip (rsvd_kamaneh_raganato_terrana_amd/librsvd_hip.so).  Needs Eigen >= 3.3
// (as the reference does); no MPI requirement.  SVDMethod is declared here (the reference declares
// it in SVD_class.hpp:28-32 and includes that header from rSVD.hpp, so callers see it either way).
#ifndef rSVD_H
#define rSVD_H

#include <Eigen/Dense>

#include "rsvd.hpp"

using Mat_m = Eigen::MatrixXd;
using Vec_v = Eigen::VectorXd;

#ifndef RSVD_SVDMETHOD_DECLARED
#define RSVD_SVDMETHOD_DECLARED
enum class SVDMethod { Jacobi, Power, ParallelJacobi };
#endif

inline void intermediate_step(const Mat_m &A, Mat_m &Q, const Mat_m &Omega, int l, int q) {
    rsvd::intermediate_step(A, Q, Omega, l, q);
}

inline void rSVD(Mat_m &A, Mat_m &U, Vec_v &S, Mat_m &V, int l, SVDMethod method) {
    rsvd::rsvd(A, U, S, V, l, static_cast<rsvd::Method>(static_cast<int>(method)), /*q=*/2);  // src/rSVD.cpp:83
}

inline Mat_m generateOmega(int n, int l) { return rsvd::generate_omega<Mat_m>(n, l); }

// image_compression/include/rSVD.hpp: void rSVD(MatrixXd& A, MatrixXd& U, VectorXd& S, MatrixXd& V,
// int l) -- q = 1 and the power-method small SVD with V = VT^T in columns
// (image_compression/src/rSVD.cpp:77-118, src/SVD.cpp:31-55).  An overload of the 6-argument form.
inline void rSVD(Mat_m &A, Mat_m &U, Vec_v &S, Mat_m &V, int l) {
    rsvd::rsvd_columns(A, U, S, V, l, rsvd::Method::PowerImageCompression, /*q=*/1);
}

#endif
