// abi.cpp -- error channel and version of the libkaolin_hip.so C ABI.
#include <string>

#include "common.h"

namespace kl {
static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
}  // namespace kl

extern "C" const char *kl_last_error(void) { return kl::g_last_error.c_str(); }
extern "C" int kl_abi_version(void) { return 1; }
