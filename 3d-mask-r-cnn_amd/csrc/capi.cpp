// Non-kernel parts of the C-ABI: error string, version.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace m3d {
static thread_local char g_err[512] = "";
// the det of the entry point running on this thread (DetScope), NULL outside one
static thread_local const m3d_det_t* t_det = nullptr;

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

DetState det() {
    if (!t_det || !t_det->on) return DetState{0, nullptr, 0};
    return DetState{1, t_det->scratch, t_det->bytes};
}

int det_check(const m3d_det_t* d) {
    if (d && d->on && (!d->scratch || d->bytes < 4096 || (reinterpret_cast<uintptr_t>(d->scratch) & 15)))
        return einval("deterministic reductions: det->scratch must be a 16-byte aligned device scratch of >= 4096 "
                      "bytes");
    return M3D_OK;
}

DetScope::DetScope(const m3d_det_t* d) : prev(t_det) { t_det = d; }
DetScope::~DetScope() { t_det = prev; }
}  // namespace m3d

extern "C" const char* m3d_last_error(void) { return m3d::g_err; }
// 2: m3d_proposal_decode(n_anchors, err); 3: per-call m3d_det_t and caller-owned
// fork events (no process-wide state)
extern "C" int m3d_abi_version(void) { return 3; }

// ---- stream fork / join ----------------------------------------------------
// The training step forks every layer's weight gradient onto a side stream.
// torch's wait_stream records a default event, whose completion performs a
// system-scope release (L2 write-back + invalidate) on the recording stream:
// measured as a ~7.5 us bubble on the compute queue per fork.  These events
// use a device-scope release (mode 1) or no system-scope fence (mode 2, the
// training step's default: -0.2 ms per 128^3 step): the waiting stream is on
// the same device, so agent-scope visibility is all it needs.  The events are
// the caller's (m3d.nn keeps a ring per device), so nothing here is shared.
extern "C" int m3d_fork_event_create(int32_t mode, void** ev) {
    using namespace m3d;
    if (mode < 0 || mode > 2) return einval("fork_event_create: mode must be 0, 1 or 2");
    if (!ev) return einval("fork_event_create: ev is NULL");
    const unsigned flags = hipEventDisableTiming | (mode == 1 ? hipEventReleaseToDevice : 0u) |
                           (mode == 2 ? hipEventDisableSystemFence : 0u);
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, flags) != hipSuccess) return check_launch("fork_event_create");
    *ev = reinterpret_cast<void*>(e);
    return M3D_OK;
}

extern "C" int m3d_fork_event_destroy(void* ev) {
    using namespace m3d;
    if (!ev) return M3D_OK;
    if (hipEventDestroy(reinterpret_cast<hipEvent_t>(ev)) != hipSuccess) return check_launch("fork_event_destroy");
    return M3D_OK;
}

extern "C" int m3d_stream_fork(m3d_stream_t from, m3d_stream_t to, void* ev) {
    using namespace m3d;
    if (!ev) return einval("stream_fork: ev is NULL (m3d_fork_event_create)");
    hipEvent_t e = reinterpret_cast<hipEvent_t>(ev);
    if (hipEventRecord(e, st(from)) != hipSuccess) return check_launch("stream_fork: hipEventRecord");
    if (hipStreamWaitEvent(st(to), e, 0) != hipSuccess) return check_launch("stream_fork: hipStreamWaitEvent");
    return M3D_OK;
}
