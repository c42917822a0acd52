// Library-level entry points of libmuz.so (version / error strings).
#include <hip/hip_runtime.h>

#include "../../include/muz.h"

extern "C" {

const char* muz_version(void) { return "libmuz 0.1 (gfx950)"; }

const char* muz_error_string(int code) {
  switch (code) {
    case MUZ_OK: return "ok";
    case MUZ_E_INVALID: return "invalid argument";
    case MUZ_E_UNSUPPORTED: return "unsupported configuration";
    default: return hipGetErrorString((hipError_t)code);
  }
}

}  // extern "C"
