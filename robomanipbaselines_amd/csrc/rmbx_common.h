// Shared helpers for the rmbx C-ABI translation units (HIP, gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "rmbx.h"

namespace rmbx {

// Thread-local last-error string returned by rmbx_last_error().
void set_error(const char* fmt, ...);

}  // namespace rmbx

#define RMBX_CHECK_ARG(cond, ...)          \
  do {                                     \
    if (!(cond)) {                         \
      rmbx::set_error(__VA_ARGS__);        \
      return RMBX_ERR_ARG;                 \
    }                                      \
  } while (0)

#define RMBX_CHECK_HIP(expr)                                                          \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      rmbx::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                      __LINE__);                                                      \
      return RMBX_ERR_HIP;                                                            \
    }                                                                                 \
  } while (0)

#define RMBX_CHECK_LAUNCH() RMBX_CHECK_HIP(hipGetLastError())
