// launch_util.hpp -- host-side helpers shared by the libg2048 translation units that launch the
// env kernels (g2048.hip, env_rollout.hip): the launch status, alignment check and RngArgs copy.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "step.hpp"
#include "../../include/g2048.h"

namespace {

inline int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}

inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0u; }

inline g2048::RngArgs rng_args(const g2048_rng *r) {
    g2048::RngArgs a{};
    if (r) {
        a.seed = r->seed;
        a.counter = r->counter;
        a.counter_dev = r->counter_dev;
        a.env_base = r->env_base;
        a.mt = r->mt_state;
        a.inject = r->inject;
    }
    return a;
}

}  // namespace
