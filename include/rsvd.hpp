// rsvd.hpp -- header-only C++ adapter over the C ABI (rsvd_c.h, librsvd_hip.so).
//
// Generic over the caller's matrix types: any column-major dense matrix type with
//     rows(), cols(), data() (contiguous, leading dimension == rows()), resize(r, c)
// and vector type with size(), data(), resize(n) -- Eigen::MatrixXd / Eigen::VectorXd satisfy
// this, so include/rSVD.hpp can give the reference's exact signatures on Eigen types, and the
// adapter itself is testable without Eigen (tests/cpp/dropin_test.cpp).
//
// Semantics follow the reference (AMSC22-23/rSVD_Kamaneh_Raganato_Terrana):
//   rsvd::rsvd(A, U, S, V, l, method)     <- rSVD()            src/rSVD.cpp:72-133 (q = 2, :83)
//   rsvd::intermediate_step(A, Q, Om, l, q) <- intermediate_step src/rSVD.cpp:57-70
//   rsvd::generate_omega<Mat>(n, l)      <- generateOmega     src/rSVD.cpp:12-55
// Outputs are resized as Eigen assignment would (U m x l, S l, V n x l; caller pre-sizing is
// ignored, tests/rSVD_test.cpp:69-71).  Errors never cross the C ABI as exceptions; the adapter
// maps RSVD_ERR_UNSUPPORTED for a method to std::invalid_argument("Unsupported SVD method")
// (src/rSVD.cpp:123) and every other failure to std::runtime_error.
//
// Process model: one handle per process on device RSVD_DEVICE (default: LOCAL_RANK modulo the
// device count, else 0), created on first use.  Omega is drawn from the counter-based Philox
// stream; the reference's std::random_device seeding is replaced by RSVD_SEED (default
// 0x5EED0001) advanced once per call, so runs are reproducible.
#ifndef RSVD_HPP
#define RSVD_HPP

#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <string>

#include "rsvd_c.h"

namespace rsvd {

enum class Method { Jacobi = RSVD_SVD_JACOBI, Power = RSVD_SVD_POWER, ParallelJacobi = RSVD_SVD_PARALLEL_JACOBI };

class Context {
public:
    static Context& instance() {
        static Context ctx;
        return ctx;
    }
    rsvd_handle_t handle() {
        std::call_once(once_, [this] { init(); });
        if (!h_) throw std::runtime_error(std::string("rsvd: no HIP device: ") + rsvd_status_string(status_));
        return h_;
    }
    uint64_t next_seed() { return seed_++; }
    ~Context() {
        if (h_) rsvd_destroy(h_);
    }

private:
    Context() {
        const char* s = std::getenv("RSVD_SEED");
        seed_ = s ? std::strtoull(s, nullptr, 0) : 0x5EED0001ull;
    }
    void init() {
        int dev = 0;
        if (const char* d = std::getenv("RSVD_DEVICE")) dev = std::atoi(d);
        else if (const char* lr = std::getenv("LOCAL_RANK")) dev = std::atoi(lr);
        status_ = rsvd_create(dev, &h_);
        if (status_ == RSVD_ERR_INVALID_ARG && dev != 0) status_ = rsvd_create(0, &h_);  // fewer devices than ranks
        if (status_ != RSVD_OK) h_ = nullptr;
    }
    std::once_flag once_;
    rsvd_handle_t h_ = nullptr;
    int status_ = RSVD_OK;
    uint64_t seed_ = 0;
};

inline void check(int status, const char* what) {
    if (status == RSVD_OK) return;
    const char* detail = rsvd_last_error(Context::instance().handle());
    const std::string msg = std::string(what) + ": " + rsvd_status_string(status) + (detail && *detail ? std::string(" (") + detail + ")" : "");
    if (status == RSVD_ERR_UNSUPPORTED && detail && std::string(detail).find("Unsupported SVD method") != std::string::npos)
        throw std::invalid_argument("Unsupported SVD method");
    if (status == RSVD_ERR_INVALID_ARG) throw std::invalid_argument(msg);
    throw std::runtime_error(msg);
}

// rSVD(A, U, S, V, l, method) with q power iterations (the reference hard-codes q = 2).
template <class Mat, class Vec>
void rsvd(const Mat& A, Mat& U, Vec& S, Mat& V, int l, Method method, int q = 2) {
    const int64_t m = A.rows(), n = A.cols();
    const int64_t d = l < n ? l : n;
    U.resize(m, d);
    S.resize(d);
    V.resize(n, d);
    Context& c = Context::instance();
    check(rsvd_run_host_f64(c.handle(), m, n, A.data(), m, l, q, static_cast<int32_t>(method), nullptr,
                            c.next_seed(), U.data(), S.data(), V.data()),
          "rSVD");
}

// intermediate_step(A, Q, Omega, l, q): Q (m x l) orthonormal basis of range((A A^T)^q A Omega).
template <class Mat>
void intermediate_step(const Mat& A, Mat& Q, const Mat& Omega, int l, int q) {
    const int64_t m = A.rows(), n = A.cols();
    if (Omega.rows() != n || Omega.cols() < l) throw std::invalid_argument("intermediate_step: Omega must be n x l");
    Q.resize(m, l);
    check(rsvd_range_finder_host_f64(Context::instance().handle(), m, n, A.data(), m, Omega.data(), l, q, Q.data()),
          "intermediate_step");
}

// generateOmega(n, l): n x l i.i.d. N(0, 1).
template <class Mat>
Mat generate_omega(int n, int l) {
    Mat Om;
    Om.resize(n, l);
    Context& c = Context::instance();
    check(rsvd_generate_omega_host_f64(c.handle(), n, l, c.next_seed(), Om.data()), "generateOmega");
    return Om;
}

}  // namespace rsvd

#endif  // RSVD_HPP
