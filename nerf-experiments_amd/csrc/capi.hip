// Library-level C-ABI helpers (version, status strings).
#include "common.h"

extern "C" int nerf_abi_version(void) { return 4; }

extern "C" const char* nerf_status_string(int status) {
    switch (status) {
        case NERF_OK: return "ok";
        case NERF_ERR_INVALID_ARG: return "invalid argument (shape, stride, alignment or null pointer)";
        case NERF_ERR_UNSUPPORTED: return "unsupported configuration";
        case NERF_ERR_LAUNCH: return "HIP kernel launch failed";
        case NERF_ERR_WORKSPACE: return "workspace missing or too small";
        default: return "unknown status";
    }
}
