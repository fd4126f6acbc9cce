/**
 * @file Exceptions.hpp
 * @brief Error types of the SVGDCpp API (reference: include/SVGDCpp/Exceptions.hpp:16-56).
 *
 * Same names, same "SVGDCpp: [... Error] " message prefixes.  The C ABI
 * (svgdcpp_amd/svgd_capi.h) reports errors as codes plus a prefixed message;
 * ThrowFromCode() maps them back onto these types.
 */
#ifndef SVGDCPP_AMD_EXCEPTIONS_HPP
#define SVGDCPP_AMD_EXCEPTIONS_HPP

#include <exception>
#include <stdexcept>
#include <string>

#include "../svgdcpp_amd/svgd_capi.h"

#define SVGDCPP_LOG_PREFIX std::string("SVGDCpp: ")

/** Dimension mismatch errors (Exceptions.hpp:23-36). */
class DimensionMismatchException : public std::exception
{
public:
    explicit DimensionMismatchException(const std::string &message, bool raw = false)
        : message_(raw ? message : SVGDCPP_LOG_PREFIX + "[Dimension Error] " + message) {}
    const char *what() const noexcept override { return message_.c_str(); }

private:
    std::string message_;
};

/** Unset value errors (Exceptions.hpp:43-56). */
class UnsetException : public std::exception
{
public:
    explicit UnsetException(const std::string &message, bool raw = false)
        : message_(raw ? message : SVGDCPP_LOG_PREFIX + "[Unset Error] " + message) {}
    const char *what() const noexcept override { return message_.c_str(); }

private:
    std::string message_;
};

namespace svgdcpp
{
/** Rethrow a C-ABI failure as the exception type the reference would throw. */
inline void ThrowFromCode(int code, const std::string &msg)
{
    switch (code)
    {
    case SVGD_OK:
        return;
    case SVGD_ERR_DIM:
        throw DimensionMismatchException(msg, true);
    case SVGD_ERR_UNSET:
        throw UnsetException(msg, true);
    case SVGD_ERR_ARG:
        throw std::invalid_argument(msg);
    default:
        throw std::runtime_error(msg);
    }
}
} // namespace svgdcpp

#endif
