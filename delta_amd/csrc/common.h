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

// DeltaErrors.actionNotFoundException (D/DeltaErrors.scala:553-560): the stripMargin'd text of the
// reference, leading newline and trailing indentation included.
inline std::string action_not_found(const char* action, int64_t version) {
  return fmt("\nThe %s of your Delta table couldn't be recovered while Reconstructing\nversion: %lld. Did you "
             "manually delete files in the _delta_log directory?\nSet "
             "spark.databricks.delta.stateReconstructionValidation.enabled\nto \"false\" to skip validation.\n       ",
             action, (long long)version);
}

}  // namespace dr
