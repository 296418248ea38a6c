// Shared host-side plumbing for the C-ABI: thread-local error text and the
// guard macro every extern "C" entry point uses to turn C++ exceptions into
// status codes (no exception ever crosses the C boundary).
#pragma once

#include <cstdint>
#include <cstdio>
#include <new>
#include <stdexcept>
#include <string>

#include "../../../include/graphsage_amd.h"

namespace gs {

void set_error(const std::string& msg);

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] inline void fail(int code, const std::string& msg) { throw Error(code, msg); }

#define GS_REQUIRE(cond, code, msg)                                   \
    do {                                                              \
        if (!(cond)) ::gs::fail((code), std::string(__func__) + ": " + (msg)); \
    } while (0)

}  // namespace gs

#define GS_API_BEGIN try {
#define GS_API_END                                        \
    }                                                     \
    catch (const ::gs::Error& e) {                        \
        ::gs::set_error(e.what());                        \
        return e.code;                                    \
    }                                                     \
    catch (const std::bad_alloc&) {                       \
        ::gs::set_error(std::string(__func__) + ": out of host memory"); \
        return GS_ENOMEM;                                 \
    }                                                     \
    catch (const std::exception& e) {                     \
        ::gs::set_error(std::string(__func__) + ": " + e.what()); \
        return GS_EINVAL;                                 \
    }                                                     \
    return GS_OK;
