// dropin_test.cpp -- exercises include/rsvd.hpp (the generic C++ adapter under include/rSVD.hpp)
// with a minimal column-major matrix type, the way tests/rSVD_test.cpp calls rSVD() on Eigen
// matrices: I_100 with l = 16 must give S == 1 and ||A - U S V^T||_F = sqrt(100 - 16); an
// unsupported method must throw std::invalid_argument("Unsupported SVD method").
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

    bool threw = false;
    try {
        rsvd::rsvd(A, U, S, V, l, static_cast<rsvd::Method>(7));
    } catch (const std::invalid_argument& e) {
        threw = std::string(e.what()) == "Unsupported SVD method";
    }
    CHECK(threw, "unsupported method throws std::invalid_argument");
    std::printf("%s (%d failures)\n", fails ? "FAILED" : "PASSED", fails);
    return fails ? 1 : 0;
}
