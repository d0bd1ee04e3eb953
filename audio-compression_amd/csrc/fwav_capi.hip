// fwav_capi.hip — C-ABI plumbing shared by every entry point of libfwav.so (see include/fwav.h).
#include <cstdarg>

#include "fwav_common.h"
#include "../../include/fwav.h"

namespace fwav {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace fwav

extern "C" {

const char* fwav_last_error(void) { return fwav::g_err; }

int fwav_abi_version(void) { return 5; }

#ifndef FWAV_SOURCE_DIGEST
#define FWAV_SOURCE_DIGEST "unknown"
#endif
// SHA-256 of the sources + compiler flags (fwav/_digest.py), passed in by __graft_entry__.build.
const char* fwav_build_digest(void) { return FWAV_SOURCE_DIGEST; }

// Block until all work queued on `stream` is done; reports asynchronous kernel faults.
int fwav_stream_sync(void* stream) {
  hipError_t e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) {
    fwav::set_error("hipStreamSynchronize: %s", hipGetErrorString(e));
    return FWAV_ERR_HIP;
  }
  return FWAV_OK;
}

}  // extern "C"
