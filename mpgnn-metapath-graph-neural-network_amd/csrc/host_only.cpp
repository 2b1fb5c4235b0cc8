// Host-only build of the plan builder and file readers (csrc/Makefile target `asan`): the
// sanitizer library libmpgnn_host_asan.so links plan.cpp + io.cpp with this file instead of
// the gfx950 kernels (ASan/UBSan host build). Only the plan-thread option exists
// here; every other option is a kernel switch and reports MPGNN_ERR_UNSUPPORTED.
#include "mpgnn_rgcn.h"
#include "plan_internal.h"

extern "C" int32_t mpgnn_set_option(int32_t option, int64_t value) {
    if (option == MPGNN_OPT_PLAN_THREADS) {
        if (value < 0 || value > 256) {
            mpgnn::set_last_error("MPGNN_OPT_PLAN_THREADS: must be 0..256");
            return MPGNN_ERR_ARG;
        }
        mpgnn::g_plan_threads = (int)value;
        return MPGNN_OK;
    }
    mpgnn::set_last_error("host-only library: kernel options are not available");
    return MPGNN_ERR_UNSUPPORTED;
}

extern "C" int32_t mpgnn_get_option(int32_t option, int64_t* value) {
    if (option == MPGNN_OPT_PLAN_THREADS && value) {
        *value = mpgnn::g_plan_threads;
        return MPGNN_OK;
    }
    mpgnn::set_last_error("host-only library: kernel options are not available");
    return MPGNN_ERR_UNSUPPORTED;
}

// the plans of the host-only build carry the shipped kernel switches (there are no kernels)
mpgnn::Options mpgnn::default_options() { return mpgnn::Options{}; }

// no kernels in the host-only build: the plan's device node maps are not built (the fused
// mode-SINGLE layer builds a relation's map per call when they are absent)
int32_t mpgnn::build_rel_node_maps(mpgnn_plan*, void*) { return MPGNN_OK; }

// no device build in the host-only library
int32_t mpgnn::sync_host_tables(mpgnn_plan*) { return MPGNN_OK; }
void mpgnn::free_device_plan(mpgnn_plan*) {}
extern "C" int32_t mpgnn_plan_create_device(const int64_t*, const int64_t*, int64_t, int64_t, int64_t, int64_t, int32_t,
                                            int32_t, void*, mpgnn_plan** out) {
    if (out) *out = nullptr;
    mpgnn::set_last_error("host-only library: no device plan build");
    return MPGNN_ERR_UNSUPPORTED;
}
