// Shared status helper: sets the calling thread's ozec_last_error() message and returns `code`.
#pragma once
#include <string>

namespace ozec {
int set_error(int code, const std::string &msg);
}  // namespace ozec
