// kinhip_host.h -- internal host helpers shared by the C-ABI translation units.
#pragma once
#include <string>

namespace kinhip {
// Records a thread-local message for kin_last_error() and returns code.
int set_error(int code, const std::string& msg);
}  // namespace kinhip
