/**
 * @file Core.hpp
 * @brief Core types of the SVGDCpp API mirror (reference: include/SVGDCpp/Core.hpp).
 *
 * The reference is header-only C++ over Eigen3 + CppAD.  Neither library is
 * part of this build: the hot path runs in the HIP library behind the C ABI
 * (svgdcpp_amd/svgd_capi.h) and the model log-gradient uses closed forms.
 * For source compatibility with the reference's callers (the example
 * programs, tests/test_svgd.cpp) this header provides a small column-major dense
 * matrix with the Eigen spellings those callers use (Eigen::MatrixXd,
 * VectorXd, Vector2d, Matrix2d, ::Random/::Zero/::Constant/::Identity, the
 * comma initialiser, operator<<, isApprox).  Define SVGDCPP_WITH_EIGEN to use
 * a real Eigen installation instead.
 */
#ifndef SVGDCPP_AMD_CORE_HPP
#define SVGDCPP_AMD_CORE_HPP

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <initializer_list>
#include <iomanip>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "Exceptions.hpp"

#ifdef SVGDCPP_WITH_EIGEN
#include <Eigen/Core>
#include <Eigen/LU>
#else

namespace svgdcpp
{
class VectorXd;

/** Dense column-major double matrix (the subset of Eigen::MatrixXd the API uses). */
class MatrixXd
{
public:
    MatrixXd() = default;
    MatrixXd(long rows, long cols) : rows_(rows), cols_(cols), data_((size_t)(rows * cols), 0.0) {}

    long rows() const { return rows_; }
    long cols() const { return cols_; }
    long size() const { return rows_ * cols_; }
    double *data() { return data_.data(); }
    const double *data() const { return data_.data(); }

    double &operator()(long r, long c) { return data_[(size_t)(c * rows_ + r)]; }
    double operator()(long r, long c) const { return data_[(size_t)(c * rows_ + r)]; }
    double &operator()(long i) { return data_[(size_t)i]; }
    double operator()(long i) const { return data_[(size_t)i]; }

    void resize(long rows, long cols)
    {
        rows_ = rows;
        cols_ = cols;
        data_.assign((size_t)(rows * cols), 0.0);
    }

    /** Eigen 3.3/3.4 Random(): -1 + 2*rand()/RAND_MAX, filled column-major. */
    static MatrixXd Random(long rows, long cols)
    {
        MatrixXd m(rows, cols);
        for (auto &v : m.data_)
            v = -1.0 + (2.0 * (double)std::rand()) / (double)RAND_MAX;
        return m;
    }
    static MatrixXd Zero(long rows, long cols) { return MatrixXd(rows, cols); }
    static MatrixXd Constant(long rows, long cols, double v)
    {
        MatrixXd m(rows, cols);
        std::fill(m.data_.begin(), m.data_.end(), v);
        return m;
    }
    static MatrixXd Identity(long rows, long cols)
    {
        MatrixXd m(rows, cols);
        for (long i = 0; i < std::min(rows, cols); ++i)
            m(i, i) = 1.0;
        return m;
    }

    inline VectorXd col(long c) const;
    template <class V> void setCol(long c, const V &v)
    {
        for (long r = 0; r < rows_; ++r)
            (*this)(r, c) = v(r);
    }

    MatrixXd transpose() const
    {
        MatrixXd t(cols_, rows_);
        for (long c = 0; c < cols_; ++c)
            for (long r = 0; r < rows_; ++r)
                t(c, r) = (*this)(r, c);
        return t;
    }

    double squaredNorm() const
    {
        double s = 0.0;
        for (double v : data_)
            s += v * v;
        return s;
    }
    double norm() const { return std::sqrt(squaredNorm()); }

    /** Eigen's fuzzy comparison: |a-b| <= prec * min(|a|, |b|). */
    bool isApprox(const MatrixXd &o, double prec = 1e-12) const
    {
        if (o.rows_ != rows_ || o.cols_ != cols_)
            return false;
        MatrixXd d = *this;
        d -= o;
        return d.norm() <= prec * std::min(norm(), o.norm());
    }

    MatrixXd &operator+=(const MatrixXd &o)
    {
        check(o);
        for (size_t i = 0; i < data_.size(); ++i)
            data_[i] += o.data_[i];
        return *this;
    }
    MatrixXd &operator-=(const MatrixXd &o)
    {
        check(o);
        for (size_t i = 0; i < data_.size(); ++i)
            data_[i] -= o.data_[i];
        return *this;
    }
    MatrixXd &operator*=(double s)
    {
        for (double &v : data_)
            v *= s;
        return *this;
    }
    MatrixXd &operator/=(double s)
    {
        for (double &v : data_)
            v /= s;
        return *this;
    }

    /** Comma initialiser, row-major fill order like Eigen's operator<<. */
    class CommaInit
    {
    public:
        CommaInit(MatrixXd &m, double v) : m_(m) { put(v); }
        CommaInit &operator,(double v)
        {
            put(v);
            return *this;
        }

    private:
        void put(double v)
        {
            if (k_ >= m_.size())
                throw DimensionMismatchException("Too many coefficients passed to comma initializer.");
            m_((long)(k_ / m_.cols()), (long)(k_ % m_.cols())) = v;
            ++k_;
        }
        MatrixXd &m_;
        long k_ = 0;
    };
    CommaInit operator<<(double v) { return CommaInit(*this, v); }

protected:
    void check(const MatrixXd &o) const
    {
        if (o.rows_ != rows_ || o.cols_ != cols_)
            throw DimensionMismatchException("Matrix sizes do not match.");
    }
    long rows_ = 0, cols_ = 0;
    std::vector<double> data_;
};

/** Column vector (Eigen::VectorXd). */
class VectorXd : public MatrixXd
{
public:
    VectorXd() = default;
    explicit VectorXd(long n) : MatrixXd(n, 1) {}
    VectorXd(const MatrixXd &m) : MatrixXd(m)
    {
        if (m.cols() != 1)
            throw DimensionMismatchException("Not a column vector.");
    }
    static VectorXd Zero(long n) { return VectorXd(n); }
    static VectorXd Constant(long n, double v) { return VectorXd(MatrixXd::Constant(n, 1, v)); }
    static VectorXd Random(long n) { return VectorXd(MatrixXd::Random(n, 1)); }
    void resize(long n) { MatrixXd::resize(n, 1); }
    double &operator[](long i) { return (*this)(i); }
    double operator[](long i) const { return (*this)(i); }
    using MatrixXd::operator();
};

/** Fixed-size spellings used by the reference examples. */
class Vector2d : public VectorXd
{
public:
    Vector2d() : VectorXd(2) {}
    Vector2d(double a, double b) : VectorXd(2)
    {
        (*this)(0) = a;
        (*this)(1) = b;
    }
};

class Matrix2d : public MatrixXd
{
public:
    Matrix2d() : MatrixXd(2, 2) {}
    Matrix2d(const MatrixXd &m) : MatrixXd(m) {}
};

inline VectorXd MatrixXd::col(long c) const
{
    VectorXd v(rows_);
    for (long r = 0; r < rows_; ++r)
        v(r) = (*this)(r, c);
    return v;
}

inline MatrixXd operator+(MatrixXd a, const MatrixXd &b) { return a += b; }
inline MatrixXd operator-(MatrixXd a, const MatrixXd &b) { return a -= b; }
inline MatrixXd operator*(double s, MatrixXd a) { return a *= s; }
inline MatrixXd operator*(MatrixXd a, double s) { return a *= s; }
inline MatrixXd operator/(MatrixXd a, double s) { return a /= s; }
inline MatrixXd operator*(const MatrixXd &a, const MatrixXd &b)
{
    if (a.cols() != b.rows())
        throw DimensionMismatchException("Matrix product dimensions do not match.");
    MatrixXd c(a.rows(), b.cols());
    for (long j = 0; j < b.cols(); ++j)
        for (long k = 0; k < a.cols(); ++k)
            for (long i = 0; i < a.rows(); ++i)
                c(i, j) += a(i, k) * b(k, j);
    return c;
}
inline bool operator==(const MatrixXd &a, const MatrixXd &b)
{
    if (a.rows() != b.rows() || a.cols() != b.cols())
        return false;
    return std::equal(a.data(), a.data() + a.size(), b.data());
}

/** Eigen-style printing: every coefficient right-aligned to the widest one. */
inline std::ostream &operator<<(std::ostream &os, const MatrixXd &m)
{
    std::vector<std::string> s((size_t)m.size());
    size_t w = 0;
    for (long r = 0; r < m.rows(); ++r)
        for (long c = 0; c < m.cols(); ++c)
        {
            std::ostringstream o;
            o.copyfmt(os);
            o.width(0);
            o << m(r, c);
            s[(size_t)(r * m.cols() + c)] = o.str();
            w = std::max(w, o.str().size());
        }
    for (long r = 0; r < m.rows(); ++r)
    {
        if (r)
            os << '\n';
        for (long c = 0; c < m.cols(); ++c)
        {
            if (c)
                os << ' ';
            os << std::setw((int)w) << s[(size_t)(r * m.cols() + c)];
        }
    }
    return os;
}

/** Gauss-Jordan inverse with partial pivoting (Eigen's .inverse() on small matrices). */
inline MatrixXd Inverse(const MatrixXd &a)
{
    const long d = a.rows();
    if (a.cols() != d)
        throw DimensionMismatchException("Only square matrices can be inverted.");
    MatrixXd m = a, inv = MatrixXd::Identity(d, d);
    for (long c = 0; c < d; ++c)
    {
        long p = c;
        for (long r = c + 1; r < d; ++r)
            if (std::fabs(m(r, c)) > std::fabs(m(p, c)))
                p = r;
        for (long q = 0; q < d; ++q)
        {
            std::swap(m(c, q), m(p, q));
            std::swap(inv(c, q), inv(p, q));
        }
        const double piv = m(c, c);
        for (long q = 0; q < d; ++q)
        {
            m(c, q) /= piv;
            inv(c, q) /= piv;
        }
        for (long r = 0; r < d; ++r)
        {
            if (r == c)
                continue;
            const double f = m(r, c);
            for (long q = 0; q < d; ++q)
            {
                m(r, q) -= f * m(c, q);
                inv(r, q) -= f * inv(c, q);
            }
        }
    }
    return inv;
}

inline double Determinant(const MatrixXd &a)
{
    const long d = a.rows();
    MatrixXd m = a;
    double det = 1.0;
    for (long c = 0; c < d; ++c)
    {
        long p = c;
        for (long r = c + 1; r < d; ++r)
            if (std::fabs(m(r, c)) > std::fabs(m(p, c)))
                p = r;
        if (m(p, c) == 0.0)
            return 0.0;
        if (p != c)
        {
            det = -det;
            for (long q = 0; q < d; ++q)
                std::swap(m(c, q), m(p, q));
        }
        det *= m(c, c);
        for (long r = c + 1; r < d; ++r)
        {
            const double f = m(r, c) / m(c, c);
            for (long q = c; q < d; ++q)
                m(r, q) -= f * m(c, q);
        }
    }
    return det;
}
} // namespace svgdcpp

namespace Eigen
{
using MatrixXd = svgdcpp::MatrixXd;
using VectorXd = svgdcpp::VectorXd;
using Vector2d = svgdcpp::Vector2d;
using Matrix2d = svgdcpp::Matrix2d;
} // namespace Eigen

#endif // SVGDCPP_WITH_EIGEN

/** Core.hpp:239: row-count comparison helper. */
template <typename T1, typename T2>
inline bool CompareVectorSizes(const T1 &a, const T2 &b)
{
    return a.rows() == b.rows();
}

/**
 * Core.hpp:273-296 configures CppAD for OpenMP.  The device path is always
 * parallel and the built-in host models are thread-safe, so this is a no-op
 * kept for source compatibility.
 */
inline void SetupForParallelMode() {}

#endif
