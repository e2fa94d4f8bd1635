// errors.h -- shared thread-local error text of the C ABI (tfhe_mi355_last_error).
#pragma once
#include <string>

namespace tfhe_mi355 {
inline std::string &last_error_text() {
    static thread_local std::string s;
    return s;
}
}  // namespace tfhe_mi355
