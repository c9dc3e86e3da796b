// Library-level C-ABI helpers (version, status strings).
#include "common.h"

extern "C" int nerf_abi_version(void) { return 10; }

extern "C" int64_t nerf_struct_size(int32_t which) {
    switch (which) {
        case 0: return (int64_t)sizeof(nerf_pe_params);
        case 1: return (int64_t)sizeof(nerf_fused_layer);
        case 2: return (int64_t)sizeof(nerf_fused_encoding);
        case 3: return (int64_t)sizeof(nerf_hashgrid_params);
        case 4: return (int64_t)sizeof(nerf_adam_batch);
        case 5: return (int64_t)sizeof(nerf_seg);
        case 6: return (int64_t)sizeof(nerf_fused_composite);
        default: return -1;
    }
}

// each translation unit that holds diagnostic switches reports its own compile flags (a variant
// build recompiles only that unit: tools/build_variant.sh)
extern "C" int32_t nerf_tu_build_flags_mlp_fused(void);
extern "C" int32_t nerf_tu_build_flags_linear_x3(void);

extern "C" int32_t nerf_build_flags(void) {
    return NERF_TU_BUILD_FLAGS | nerf_tu_build_flags_mlp_fused() | nerf_tu_build_flags_linear_x3();
}

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
