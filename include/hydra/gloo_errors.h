// include/hydra/gloo_errors.h -- the shim's failures as Gloo's own exception types.
//
// For a caller built against Gloo (its headers on the include path).  Include this header
// INSTEAD of (or before) hydra/gloo_reduce.h: every shim then reports
//   a timeout (HYDRA_ERR_TIMEOUT)   as ::gloo::IoException     (gloo/gloo/common/error.h:45; what
//                                                              tcp/unbound_buffer.cc:80-84 throws)
//   any other failure               as ::gloo::EnforceNotMet   (gloo/gloo/common/logging.h:21,42;
//                                                              what GLOO_ENFORCE throws)
// so the reference's callers catch them where they already catch Gloo's.  Per call site the
// policy can also be named explicitly: hostSum<float, hydra::gloo_compat::GlooErrors>().
#pragma once

#ifdef HYDRA_GLOO_REDUCE_H_INCLUDED
#error "include hydra/gloo_errors.h before hydra/gloo_reduce.h (it sets the shim's default error policy)"
#endif

#include <string>

#include "gloo/common/error.h"
#include "gloo/common/logging.h"

namespace hydra {
namespace gloo_compat {

struct GlooErrors {
  [[noreturn]] static void enforce_failed(int code, const std::string& msg, const char* call) {
    throw ::gloo::EnforceNotMet(__FILE__, __LINE__, call,
                                "[hydra_hip] " + msg + " (status " + std::to_string(code) + ")");
  }
  [[noreturn]] static void io_failed(int code, const std::string& msg, const char* call) {
    throw ::gloo::IoException("[hydra_hip] " + std::string(call) + ": " + msg + " (status " +
                              std::to_string(code) + ")");
  }
};

}  // namespace gloo_compat
}  // namespace hydra

#define HYDRA_GLOO_ERRORS ::hydra::gloo_compat::GlooErrors
#include "gloo_reduce.h"
