// dropin_test.cpp -- exercises include/rsvd.hpp (the generic C++ adapter under include/rSVD.hpp,
// include/QR.hpp and include/SVD_class.hpp) with a minimal column-major matrix type, the way
// tests/rSVD_test.cpp calls rSVD() on Eigen matrices: I_100 with l = 16 must give S == 1 and
// ||A - U S V^T||_F = sqrt(100 - 16); an unsupported method must throw
// std::invalid_argument("Unsupported SVD method").  Also: QR() (A = Q R, Q^T Q = I, R upper)
// and SVD<method> (reconstruction; the Power layouts and early stop of SVD_class.hpp:183-219).
// Build: make -C tests/cpp ; run on a GPU: tests/cpp/dropin_test  (exit 0 = pass)
#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <vector>

#include "rsvd.hpp"

struct HostMat {  // column-major, ld == rows
    long r = 0, c = 0;
    std::vector<double> v;
    long rows() const { return r; }
    long cols() const { return c; }
    long size() const { return r * c; }
    double* data() { return v.data(); }
    const double* data() const { return v.data(); }
    void resize(long rr, long cc) { r = rr; c = cc; v.assign((size_t)rr * cc, 0.0); }
    double& operator()(long i, long j) { return v[(size_t)i + (size_t)j * r]; }
    double operator()(long i, long j) const { return v[(size_t)i + (size_t)j * r]; }
};
struct HostVec {
    std::vector<double> v;
    long size() const { return (long)v.size(); }
    double* data() { return v.data(); }
    void resize(long n) { v.assign((size_t)n, 0.0); }
};

static int fails = 0;
#define CHECK(cond, ...)                      \
    do {                                      \
        if (!(cond)) {                        \
            std::printf("FAIL: " __VA_ARGS__); \
            std::printf("\n");                \
            ++fails;                          \
        }                                     \
    } while (0)

int main() {
    const int n = 100, l = 16;
    HostMat A;
    A.resize(n, n);
    for (int i = 0; i < n; ++i) A(i, i) = 1.0;
    HostMat U, V;
    HostVec S;
    U.resize(n, n);  // pre-sizing is ignored, as with Eigen assignment
    rsvd::rsvd(A, U, S, V, l, rsvd::Method::Jacobi);
    CHECK(U.rows() == n && U.cols() == l && V.rows() == n && V.cols() == l && S.size() == l, "output shapes");
    double smax = 0, err2 = 0;
    for (int i = 0; i < l; ++i) smax = std::fmax(smax, std::fabs(S.v[i] - 1.0));
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double a = A(i, j);
            for (int k = 0; k < l; ++k) a -= U(i, k) * S.v[k] * V(j, k);
            err2 += a * a;
        }
    CHECK(smax < 1e-12, "S == 1 (max dev %g)", smax);
    CHECK(std::fabs(std::sqrt(err2) - std::sqrt(84.0)) < 1e-10, "||A - USV^T|| = %.15f", std::sqrt(err2));

    HostMat Om = rsvd::generate_omega<HostMat>(n, l);
    HostMat Q;
    rsvd::intermediate_step(A, Q, Om, l, 2);
    double orth = 0;
    for (int a = 0; a < l; ++a)
        for (int b = 0; b < l; ++b) {
            double d = 0;
            for (int i = 0; i < n; ++i) d += Q(i, a) * Q(i, b);
            orth = std::fmax(orth, std::fabs(d - (a == b)));
        }
    CHECK(orth < 1e-12, "Q^T Q == I (dev %g)", orth);

    // rSVD with Method::Power: the reference's layouts (U m x l, S l, V = the n x n V_, rows v_i)
    rsvd::rsvd(A, U, S, V, l, rsvd::Method::Power);
    CHECK(U.rows() == n && U.cols() == l && S.size() == l && V.rows() == n && V.cols() == n, "Power rSVD shapes");
    double pdev = 0;
    for (int i = 0; i < l; ++i) pdev = std::fmax(pdev, std::fabs(S.v[i] - 1.0));
    CHECK(pdev < 1e-12 && V(n - 1, n - 1) == 1.0, "Power rSVD on I: S == 1 (dev %g), identity rows of V_", pdev);

    // image_compression's 5-argument rSVD: q = 1, power method, V in columns
    rsvd::rsvd_columns(A, U, S, V, l, rsvd::Method::Power, 1);
    CHECK(U.rows() == n && U.cols() == l && V.rows() == n && V.cols() == l && S.size() == l, "5-arg rSVD shapes");

    bool threw = false;
    try {
        rsvd::rsvd(A, U, S, V, l, static_cast<rsvd::Method>(7));
    } catch (const std::invalid_argument& e) {
        threw = std::string(e.what()) == "Unsupported SVD method";
    }
    CHECK(threw, "unsupported method throws std::invalid_argument");
    // ---- QR(): reduced and full ----------------------------------------------------------------
    {
        const int qm = 50, qn = 20;
        HostMat B;
        B.resize(qm, qn);
        unsigned st = 12345u;
        for (auto& x : B.v) x = ((st = st * 1664525u + 1013904223u) >> 8) / 16777216.0 - 0.5;
        for (int full = 0; full < 2; ++full) {
            HostMat Q, R;
            if (full) rsvd::qr_full(B, Q, R); else rsvd::qr_reduced(B, Q, R);
            const long kq = full ? qm : qn;
            CHECK(Q.rows() == qm && Q.cols() == kq && R.rows() == kq && R.cols() == qn, "QR shapes (full=%d)", full);
            double oe = 0, re = 0, lo = 0;
            for (long a = 0; a < kq; ++a)
                for (long b = 0; b < kq; ++b) {
                    double d = 0;
                    for (long i = 0; i < qm; ++i) d += Q(i, a) * Q(i, b);
                    oe = std::fmax(oe, std::fabs(d - (a == b)));
                }
            for (long i = 0; i < qm; ++i)
                for (long j = 0; j < qn; ++j) {
                    double d = 0;
                    for (long t = 0; t < kq; ++t) d += Q(i, t) * R(t, j);
                    re = std::fmax(re, std::fabs(d - B(i, j)));
                }
            for (long i = 0; i < kq; ++i)
                for (long j = 0; j < qn && j < i; ++j) lo = std::fmax(lo, std::fabs(R(i, j)));
            CHECK(oe < 1e-13 && re < 1e-13 && lo == 0.0, "QR full=%d: orth %g recon %g lower %g", full, oe, re, lo);
        }
        bool threw = false;
        try {
            HostMat W, Q, R;
            W.resize(3, 5);
            rsvd::qr_reduced(W, Q, R);
        } catch (const std::invalid_argument&) {
            threw = true;
        }
        CHECK(threw, "reduced QR of a wide matrix throws std::invalid_argument");
    }
    // ---- SVD<Jacobi>: reconstruction; SVD<Power>: layouts and early stop ----------------------------
    {
        const int sm = 40, sn = 25;
        HostMat B;  // graded spectrum 2 * 0.8^j (+ small noise): the power method converges
        B.resize(sm, sn);
        unsigned st = 777u;
        for (auto& x : B.v) x = 1e-3 * (((st = st * 1664525u + 1013904223u) >> 8) / 16777216.0 - 0.5);
        for (int j = 0; j < sn; ++j) B(j, j) += 2.0 * std::pow(0.8, j);
        rsvd::SVDT<rsvd::Method::Jacobi, HostMat, HostVec> sj(B);
        sj.compute();
        HostMat Uj = sj.getU(), Vj = sj.getV();
        HostVec Sj = sj.getS();
        CHECK(Uj.rows() == sm && Uj.cols() == sn && Vj.rows() == sn && Vj.cols() == sn && Sj.size() == sn, "SVD shapes");
        double re = 0;
        for (long i = 0; i < sm; ++i)
            for (long j = 0; j < sn; ++j) {
                double d = 0;
                for (long t = 0; t < sn; ++t) d += Uj(i, t) * Sj.v[t] * Vj(j, t);
                re = std::fmax(re, std::fabs(d - B(i, j)));
            }
        CHECK(re < 1e-13, "SVD<Jacobi> reconstruction %g", re);
        rsvd::SVDT<rsvd::Method::Power, HostMat, HostVec> sp(B, 4);
        sp.compute();
        HostMat Up = sp.getU(), Vp = sp.getV();
        HostVec Sp = sp.getS();
        CHECK(Up.rows() == sm && Up.cols() == sm && Vp.rows() == sn && Vp.cols() == sn && Sp.size() == sn,
              "SVD<Power> layouts: U m x m, V n x n, S min(m, n)");
        double sd = 0, vd = 0;
        for (int i = 0; i < 4; ++i) {
            sd = std::fmax(sd, std::fabs(Sp.v[i] - Sj.v[i]) / Sj.v[0]);
            double dot = 0;  // v_i is ROW i of the Power V
            for (long t = 0; t < sn; ++t) dot += Vp(i, t) * Vj(t, i);
            vd = std::fmax(vd, 1.0 - std::fabs(dot));
        }
        CHECK(sd < 1e-10 && vd < 1e-9, "SVD<Power> vs SVD<Jacobi>: S %g, v %g", sd, vd);
        CHECK(Up(0, sm - 1) == 0.0 && Up(sm - 1, sm - 1) == 1.0 && Vp(sn - 1, sn - 1) == 1.0, "identity beyond dim");
        HostMat R2;  // rank 2: the power method stops after two triplets
        R2.resize(sm, sn);
        for (long i = 0; i < sm; ++i)
            for (long j = 0; j < sn; ++j) R2(i, j) = 0.01 * ((i + 1.0) * (j % 3 + 1.0) + 0.5 * (i % 2) * (j + 1.0));
        rsvd::SVDT<rsvd::Method::Power, HostMat, HostVec> se(R2);
        se.compute();
        CHECK(se.getU().cols() == 2 && se.getV().cols() == 2 && se.getS().size() == 2 && se.getV().rows() == sn,
              "SVD<Power> early stop keeps 2 columns");
    }
    std::printf("%s (%d failures)\n", fails ? "FAILED" : "PASSED", fails);
    return fails ? 1 : 0;
}
