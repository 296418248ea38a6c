// Thread-local error text behind gs_last_error() and the library version.
#include <string>

#include "common.hpp"

namespace gs {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace gs

extern "C" {
const char* gs_last_error(void) { return gs::g_last_error.c_str(); }
const char* gs_version(void) { return "graphsage_amd 0.1.0 (gfx950)"; }
}
