// Error plumbing for the C ABI: px.statuspb.Code return values plus a thread-local message
// (the reference's Status/StatusOr convention, src/common/base/status.h:150-160, without
// exceptions crossing the boundary).
#pragma once

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/pxg.h"

namespace pxg {

inline std::string& LastErrorRef() {
  static thread_local std::string e;
  return e;
}

inline int32_t SetError(int32_t code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  LastErrorRef() = buf;
  return code;
}

}  // namespace pxg
