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

enum class Method {
    Jacobi = RSVD_SVD_JACOBI,
    Power = RSVD_SVD_POWER,
    ParallelJacobi = RSVD_SVD_PARALLEL_JACOBI,
    PowerImageCompression = RSVD_SVD_POWER_IC  // image_compression's power-method SVD (5-argument rSVD)
};

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

// ---- multi-GPU (one process per GPU, as the reference's MPI ranks: src/rSVD.cpp:15,20-23) ----
// The process's handle joins an RCCL communicator owned by the library (rsvd_comm_init): rank 0
// draws the id, the caller broadcasts it (MPI_Bcast of RSVD_COMM_ID_BYTES bytes -- where the
// reference broadcasts Omega, :52) and every rank calls distributed_init.  Afterwards
// rsvd_local_rows runs the row-sharded rSVD on this rank's rows of A (rsvd_row_partition, the
// :20-23 split): U comes back as this rank's rows, S and V complete on every rank.
inline void unique_id(void* id /* RSVD_COMM_ID_BYTES */) {
    const int st = rsvd_comm_unique_id(id);
    if (st != RSVD_OK) throw std::runtime_error(std::string("rsvd_comm_unique_id: ") + rsvd_status_string(st));
}
inline void check(int status, const char* what);
inline void distributed_init(const void* id, int rank, int world, bool shard_n = true) {
    check(rsvd_comm_init(Context::instance().handle(), id, rank, world, shard_n ? 1 : 0), "rsvd_comm_init");
}

// rSVD(A, U, S, V, l, method) with q power iterations (the reference hard-codes q = 2).
// rSVD with the outputs as the C ABI returns them: U m x d, S d, V n x d with the right singular
// vectors in COLUMNS for every method (d = min(l, n)).  With Method::PowerImageCompression and
// q = 1 this is image_compression's 5-argument rSVD(A, U, S, V, l) (image_compression/src/rSVD.cpp:
// 77-118: q = 1, power-method small SVD with V = VT^T, image_compression/src/SVD.cpp:31-55).
template <class Mat, class Vec>
void rsvd_columns(const Mat& A, Mat& U, Vec& S, Mat& V, int l, Method method, int q) {
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

// The row-sharded rSVD after distributed_init: A_local = this rank's rows of the global A (the
// partition of rsvd_row_partition), U_local its rows of U, S and V the whole of them.
template <class Mat, class Vec>
void rsvd_local_rows(const Mat& A_local, Mat& U_local, Vec& S, Mat& V, int l, Method method = Method::Jacobi,
                     int q = 2) {
    rsvd_columns(A_local, U_local, S, V, l, method, q);
}

// Method::Power returns what the reference's rSVD returns for it (src/rSVD.cpp:106-113 with
// SVD_class.hpp:183-219): U m x l, S l and V = the n x n V_ of SVD<Power> (v_i^T in row i, identity
// rows beyond), each cut to the first `kept` columns when the power method stops early.
template <class Mat, class Vec>
void rsvd(const Mat& A, Mat& U, Vec& S, Mat& V, int l, Method method, int q = 2) {
    rsvd_columns(A, U, S, V, l, method, q);
    if (method != Method::Power) return;
    const int64_t m = A.rows(), n = A.cols();
    const int64_t d = l < n ? l : n;
    Context& c = Context::instance();
    rsvd_info_t info{};
    check(rsvd_get_info(c.handle(), &info), "rSVD");
    const int64_t kept = info.power_kept;
    Mat Vf;  // V_ (n x n): identity, v_i^T in row i < kept
    Vf.resize(n, n);
    for (int64_t e = 0; e < n * n; ++e) Vf.data()[e] = 0.0;
    for (int64_t i = 0; i < n; ++i) Vf.data()[i + i * n] = 1.0;
    for (int64_t i = 0; i < kept; ++i)
        for (int64_t t = 0; t < n; ++t) Vf.data()[i + t * n] = V.data()[t + i * n];
    if (kept >= d) {
        V = Vf;
        return;
    }
    const int64_t kk = kept > 0 ? kept : 1;  // SVD_class.hpp:199-206: zero 1-column result at i == 0
    Mat U2, V2;
    Vec S2;
    U2.resize(m, kk);
    V2.resize(n, kk);
    S2.resize(kk);
    for (int64_t e = 0; e < m * kk; ++e) U2.data()[e] = kept ? U.data()[e] : 0.0;
    for (int64_t e = 0; e < n * kk; ++e) V2.data()[e] = kept ? Vf.data()[e] : 0.0;
    for (int64_t i = 0; i < kk; ++i) S2.data()[i] = kept ? S.data()[i] : 0.0;
    U = U2;
    V = V2;
    S = S2;
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

// qr_decomposition_reduced(A, Q, R) (src/QR.cpp:43-80): Q m x n, R n x n; requires m >= n.
template <class Mat>
void qr_reduced(const Mat& A, Mat& Q, Mat& R) {
    const int64_t m = A.rows(), n = A.cols();
    Q.resize(m, n);
    R.resize(n, n);
    check(rsvd_qr_host_f64(Context::instance().handle(), m, n, A.data(), m, 0, Q.data(), R.data()),
          "qr_decomposition_reduced");
}

// qr_decomposition_full(A, Q, R) (src/QR.cpp:22-41): Q m x m, R m x n.
template <class Mat>
void qr_full(const Mat& A, Mat& Q, Mat& R) {
    const int64_t m = A.rows(), n = A.cols();
    Q.resize(m, m);
    R.resize(m, n);
    check(rsvd_qr_host_f64(Context::instance().handle(), m, n, A.data(), m, 1, Q.data(), R.data()),
          "qr_decomposition_full");
}

// SVD<method> (include/SVD_class.hpp:35-219) over any Mat / Vec pair of the kind above.
// Jacobi / ParallelJacobi: U m x k, S k, V n x k (k = min(m, n), :107-108).  Power: U m x m and
// V n x n start as identities, u_i goes to column i of U and v_i to ROW i of V (:82-83, :213-214),
// S has min(m, n) entries; an early stop after i < dim triplets (sigma < 1e-12) keeps the first i
// columns of each, as conservativeResize does (:198-208).  compute() prints nothing.
template <Method M, class Mat, class Vec>
class SVDT {
public:
    explicit SVDT(const Mat& data, const int& r = 0) : data_(data), r_(r) {}
    void compute() {
        const int64_t m = data_.rows(), n = data_.cols(), k = m < n ? m : n;
        Context& c = Context::instance();
        if (M != Method::Power) {
            U_.resize(m, k);
            S_.resize(k);
            V_.resize(n, k);
            int32_t kept = 0;
            check(rsvd_svd_host_f64(c.handle(), m, n, data_.data(), m, static_cast<int32_t>(M), 0, 0, U_.data(),
                                    S_.data(), V_.data(), &kept),
                  "SVD::compute");
            return;
        }
        const int64_t dim = r_ ? r_ : k;
        Mat u, v;
        Vec s;
        u.resize(m, k);
        v.resize(n, k);
        s.resize(k);
        int32_t kept = 0;
        check(rsvd_svd_host_f64(c.handle(), m, n, data_.data(), m, RSVD_SVD_POWER, r_, c.next_seed(), u.data(),
                                s.data(), v.data(), &kept),
              "SVD::compute");
        if (kept == 0) {  // :199-202
            U_.resize(m, 1);
            S_.resize(1);
            V_.resize(n, 1);
            fill(U_, 0.0), fill(V_, 0.0), fill(S_, 0.0);
            return;
        }
        U_.resize(m, m);
        V_.resize(n, n);
        S_.resize(k);
        identity(U_), identity(V_), fill(S_, 0.0);
        for (int64_t i = 0; i < kept; ++i) {
            for (int64_t t = 0; t < m; ++t) U_.data()[t + i * m] = u.data()[t + i * m];
            for (int64_t t = 0; t < n; ++t) V_.data()[i + t * n] = v.data()[t + i * n];
            S_.data()[i] = s.data()[i];
        }
        if (kept < dim) {  // conservativeResize to the first `kept` columns
            U_ = leading_cols(U_, kept);
            V_ = leading_cols(V_, kept);
            Vec s2;
            s2.resize(kept);
            for (int64_t i = 0; i < kept; ++i) s2.data()[i] = S_.data()[i];
            S_ = s2;
        }
    }
    Mat getU() const { return U_; }
    Vec getS() const { return S_; }
    Mat getV() const { return V_; }

protected:
    void setData(const Mat& data) { data_ = data; }

private:
    template <class X>
    static void fill(X& x, double v) {
        const int64_t nn = (int64_t)x.size();
        for (int64_t i = 0; i < nn; ++i) x.data()[i] = v;
    }
    static void identity(Mat& x) {
        fill(x, 0.0);
        const int64_t r = x.rows(), cc = x.cols();
        for (int64_t i = 0; i < r && i < cc; ++i) x.data()[i + i * r] = 1.0;
    }
    static Mat leading_cols(const Mat& x, int64_t cols) {
        Mat y;
        y.resize(x.rows(), cols);
        for (int64_t i = 0; i < x.rows() * cols; ++i) y.data()[i] = x.data()[i];
        return y;
    }
    Mat U_, V_, data_;
    Vec S_;
    int r_;
};

}  // namespace rsvd

#endif  // RSVD_HPP
