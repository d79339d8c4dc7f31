// Shared host-side helpers for libdeltareplay.
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>
#include <stdexcept>
#include <vector>

#include "../../include/deltareplay.h"

namespace dr {

// Errors travel as exceptions inside the library and become (status, message) at the C ABI.
struct Error : std::runtime_error {
  int status;
  Error(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};

[[noreturn]] inline void fail(int status, const std::string& msg) { throw Error(status, msg); }

template <typename... A>
std::string fmt(const char* f, A... a) {
  char buf[1024];
  snprintf(buf, sizeof buf, f, a...);
  return buf;
}

}  // namespace dr
