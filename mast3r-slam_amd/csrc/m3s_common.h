// m3s_common.h -- shared host-side helpers of libm3s_backend (error state, HIP checks).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

namespace m3s {

// Thread-local last-error message (m3s_last_error()).
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
const char* get_error();

// Host resources (pinned buffers, events) cached per host thread are released by m3s_shutdown()
// -- registered with atexit when the library is loaded, and by the Python module -- never by
// static or thread-local destructors: those run inside exit(), where the HIP runtime or a
// profiler's interception layer may already be finalised.  `release(obj)` frees obj's HIP
// resources; it is called once, under the registry's lock, with the HIP runtime alive.
void register_host_resource(void* obj, void (*release)(void*));

}  // namespace m3s

#define M3S_HIP_CHECK(expr)                                                              \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess) {                                                          \
            m3s::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                           __LINE__);                                                    \
            return M3S_ERR_HIP;                                                          \
        }                                                                                \
    } while (0)

#define M3S_REQUIRE(cond, ...)          \
    do {                                \
        if (!(cond)) {                  \
            m3s::set_error(__VA_ARGS__); \
            return M3S_ERR_INVALID;     \
        }                               \
    } while (0)

// Launch-error check after a kernel launch.
#define M3S_LAUNCH_CHECK() M3S_HIP_CHECK(hipGetLastError())
