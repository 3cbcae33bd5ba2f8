// eigen_dropin_test.cpp -- the reference's own call shapes, compiled against the Eigen-typed drop-in
// headers include/rSVD.hpp, include/QR.hpp and include/SVD_class.hpp (here over the minimal Eigen API
// stand-in tests/cpp/eigen_shim, Eigen being absent from the image):
//   rSVD(A, U, S, V, l, SVDMethod::Jacobi)            tests/rSVD_test.cpp:72  (I_100, l = 16)
//   intermediate_step / generateOmega                 include/rSVD.hpp:13,15
//   qr_decomposition_reduced / _full, givens_rotation include/QR.hpp:14-16
//   SVD<SVDMethod::...> svd(B); svd.compute(); getU/getS/getV   tests/svd_test.cpp:58
//   a PCA_class.hpp:11-47-style subclass calling the protected setData, then compute()
//   std::invalid_argument("Unsupported SVD method")   src/rSVD.cpp:123
//   rsvd::distributed_init (library-owned RCCL, world 1) + rsvd_local_rows
// Built on the CPU by tests/test_cpp_dropin.py; run on a GPU (exit 0 and "PASSED" = pass).
#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "QR.hpp"
#include "SVD_class.hpp"
#include "rSVD.hpp"

static int fails = 0;
#define CHECK(cond, ...)                       \
    do {                                       \
        if (!(cond)) {                         \
            std::printf("FAIL: " __VA_ARGS__); \
            std::printf("\n");                 \
            ++fails;                           \
        }                                      \
    } while (0)

// PCA_class.hpp:11-47 in miniature: the subclass centres its data, hands it to the protected
// setData and calls compute(); explainedVariance() reads getS() (PCA_class.hpp:73-76).
template <SVDMethod method>
class MiniPCA : public SVD<method> {
public:
    explicit MiniPCA(const Mat_m& data) : SVD<method>(data), data_(data) {
        Mat_m c = data_;
        for (Eigen::Index j = 0; j < c.cols(); ++j) {
            double mu = 0.0;
            for (Eigen::Index i = 0; i < c.rows(); ++i) mu += c(i, j);
            mu /= (double)c.rows();
            for (Eigen::Index i = 0; i < c.rows(); ++i) c(i, j) -= mu;
        }
        SVD<method>::setData(c);
        SVD<method>::compute();
    }
    Vec_v explainedVariance() const {
        Vec_v s = SVD<method>::getS();
        for (Eigen::Index i = 0; i < s.size(); ++i) s[i] /= std::sqrt((double)(data_.rows() - 1));
        return s;
    }

private:
    Mat_m data_;
};

static double resid(const Mat_m& A, const Mat_m& U, const Vec_v& S, const Mat_m& V) {
    double e2 = 0.0;
    for (Eigen::Index i = 0; i < A.rows(); ++i)
        for (Eigen::Index j = 0; j < A.cols(); ++j) {
            double a = A(i, j);
            for (Eigen::Index k = 0; k < S.size(); ++k) a -= U(i, k) * S[k] * V(j, k);
            e2 += a * a;
        }
    return std::sqrt(e2);
}

int main() {
    // tests/rSVD_test.cpp:56-72 on input/sparse_matrix100.mtx (= I_100), l = k + p = 16
    const int n = 100, l = 16;
    Mat_m A = Mat_m::Identity(n, n), U, V;
    Vec_v S;
    rSVD(A, U, S, V, l, SVDMethod::Jacobi);
    CHECK(U.rows() == n && U.cols() == l && V.rows() == n && V.cols() == l && S.size() == l, "rSVD shapes");
    double smax = 0.0;
    for (int i = 0; i < l; ++i) smax = std::fmax(smax, std::fabs(S[i] - 1.0));
    CHECK(smax < 1e-12, "rSVD S != 1 (%g)", smax);
    CHECK(std::fabs(resid(A, U, S, V) - std::sqrt(100.0 - l)) < 1e-10, "rSVD residual");

    Mat_m Om = generateOmega(n, l), Q;
    CHECK(Om.rows() == n && Om.cols() == l, "generateOmega shape");
    intermediate_step(A, Q, Om, l, 2);
    CHECK(Q.rows() == n && Q.cols() == l, "intermediate_step shape");

    // QR(): A = Q R on a small full-rank matrix; givens_rotation as src/QR.cpp:12-20
    Mat_m B(7, 4);
    for (int i = 0; i < 7; ++i)
        for (int j = 0; j < 4; ++j) B(i, j) = 1.0 / (1.0 + i + 2 * j) + (i == j);
    Mat_m Qr, Rr, Qf, Rf;
    qr_decomposition_reduced(B, Qr, Rr);
    qr_decomposition_full(B, Qf, Rf);
    CHECK(Qr.rows() == 7 && Qr.cols() == 4 && Rr.rows() == 4 && Rr.cols() == 4, "reduced QR shapes");
    CHECK(Qf.rows() == 7 && Qf.cols() == 7 && Rf.rows() == 7 && Rf.cols() == 4, "full QR shapes");
    double qe = 0.0;
    for (int i = 0; i < 7; ++i)
        for (int j = 0; j < 4; ++j) {
            double a = B(i, j);
            for (int k = 0; k < 4; ++k) a -= Qr(i, k) * Rr(k, j);
            qe = std::fmax(qe, std::fabs(a));
        }
    CHECK(qe < 1e-12, "A != QR (%g)", qe);
    for (int j = 0; j < 4; ++j) CHECK(Rr(j, j) > 0.0, "R diag sign");
    Eigen::Matrix2d G;
    givens_rotation(3.0, 4.0, G);
    CHECK(std::fabs(G(0, 0) - 0.6) < 1e-15 && std::fabs(G(0, 1) - 0.8) < 1e-15 && std::fabs(G(1, 0) + 0.8) < 1e-15 &&
              std::fabs(G(1, 1) - 0.6) < 1e-15,
          "givens_rotation");

    // SVD<method> as tests/svd_test.cpp:58 and src/rSVD.cpp:99-103
    SVD<SVDMethod::Jacobi> svd(B);
    svd.compute();
    CHECK(std::fabs(resid(B, svd.getU(), svd.getS(), svd.getV())) < 1e-12, "SVD<Jacobi> reconstruction");
    SVD<SVDMethod::ParallelJacobi> psvd(B);
    psvd.compute();
    CHECK(std::fabs(psvd.getS()[0] - svd.getS()[0]) < 1e-12 * svd.getS()[0], "SVD<ParallelJacobi> sigma_1");

    // the PCA subclass path (protected setData + compute)
    MiniPCA<SVDMethod::Jacobi> pca(B);
    Vec_v ev = pca.explainedVariance();
    CHECK(ev.size() == 4 && ev[0] >= ev[1] && ev[1] >= ev[2] && ev[2] >= ev[3] && ev[3] >= 0.0, "PCA variances");

    // src/rSVD.cpp:123
    bool threw = false;
    try {
        rSVD(A, U, S, V, l, static_cast<SVDMethod>(7));
    } catch (const std::invalid_argument& e) {
        threw = std::string(e.what()) == "Unsupported SVD method";
    }
    CHECK(threw, "unsupported method must throw std::invalid_argument");

    // library-owned RCCL at world 1 (the id would be MPI_Bcast from rank 0 at world > 1)
    unsigned char id[RSVD_COMM_ID_BYTES];
    rsvd::unique_id(id);
    rsvd::distributed_init(id, 0, 1);
    Mat_m Ul, Vl;
    Vec_v Sl;
    rsvd::rsvd_local_rows(A, Ul, Sl, Vl, l);
    CHECK(Ul.rows() == n && Sl.size() == l, "rsvd_local_rows shapes");
    CHECK(std::fabs(resid(A, Ul, Sl, Vl) - std::sqrt(100.0 - l)) < 1e-10, "rsvd_local_rows residual");

    std::printf(fails ? "FAILED (%d)\n" : "PASSED\n", fails);
    return fails ? 1 : 0;
}
