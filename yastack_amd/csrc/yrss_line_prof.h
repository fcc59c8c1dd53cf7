// yrss_line_prof.h — the line scatter's phase clock, for measurement builds
// only (tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1, read by
// tools/line_prof.py).  In every other build LPROF / LPROF_ENTRY are no-ops
// and YRSS_LINE_PROF_HOST_FN is empty, so libyrss.so carries neither the
// clock nor its entry point (tests/test_abi.py).
#ifndef YRSS_LINE_PROF_H
#define YRSS_LINE_PROF_H

#ifdef YRSS_PROF_LINES
#ifndef YRSS_TOOLS_BUILD
#error "YRSS_PROF_LINES is a measurement build: tools/build_ab_lib.sh only"
#endif
// per workgroup and span, the realtime clock at each phase boundary, read by
// thread 0 (t, g, g0: the line scatter's thread, span and first span)
__device__ uint64_t g_line_prof[2048 * 8 * 8];
#define LPROF(k)                                                                       \
    do {                                                                               \
        if (t == 0 && blockIdx.x < 2048u && g - g0 < 8u)                              \
            g_line_prof[(blockIdx.x * 8u + (g - g0)) * 8u + (k)] =                     \
                __builtin_amdgcn_s_memrealtime();                                      \
    } while (0)
// kernel entry, slot 7 of span 0
#define LPROF_ENTRY()                                                                  \
    do {                                                                               \
        if (t == 0 && blockIdx.x < 2048u)                                              \
            g_line_prof[(blockIdx.x * 8u) * 8u + 7u] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// prologue milestones, slots 1-5 of the unused span-7 row (slot 0 stays 0,
// so the row never counts as a span)
#define LPROF_PRO(k)                                                                   \
    do {                                                                               \
        if (t == 0 && blockIdx.x < 2048u)                                              \
            g_line_prof[(blockIdx.x * 8u + 7u) * 8u + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// the host side (inside the library's extern "C" block): read, then clear (a
// later batch with fewer workgroups leaves no stale rows)
#define YRSS_LINE_PROF_HOST_FN                                                         \
    int yrss_debug_line_prof(void *out, size_t bytes)                                  \
    {                                                                                  \
        const size_t n = bytes < sizeof(g_line_prof) ? bytes : sizeof(g_line_prof);    \
        if (hipDeviceSynchronize() != hipSuccess ||                                    \
            hipMemcpyFromSymbol(out, HIP_SYMBOL(g_line_prof), n, 0,                    \
                                hipMemcpyDeviceToHost) != hipSuccess)                  \
            return -EIO;                                                               \
        static uint64_t zero[2048 * 8 * 8];                                            \
        return hipMemcpyToSymbol(HIP_SYMBOL(g_line_prof), zero, sizeof(zero), 0,       \
                                 hipMemcpyHostToDevice) == hipSuccess                  \
                   ? (int)n                                                            \
                   : -EIO;                                                             \
    }
#else
#define LPROF(k) \
    do {         \
    } while (0)
#define LPROF_ENTRY() \
    do {              \
    } while (0)
#define LPROF_PRO(k) \
    do {             \
    } while (0)
#define YRSS_LINE_PROF_HOST_FN
#endif

#endif /* YRSS_LINE_PROF_H */
