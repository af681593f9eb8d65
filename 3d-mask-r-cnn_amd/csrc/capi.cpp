// Non-kernel parts of the C-ABI: error string, version.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace m3d {
static thread_local char g_err[512] = "";
static DetState g_det = {0, nullptr, 0};

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

const DetState& det() { return g_det; }
}  // namespace m3d

extern "C" const char* m3d_last_error(void) { return m3d::g_err; }
extern "C" int m3d_abi_version(void) { return 2; }  // 2: m3d_proposal_decode(n_anchors, err)

extern "C" int m3d_set_deterministic(int32_t on, void* scratch, size_t bytes) {
    if (on && (!scratch || bytes < 4096 || (reinterpret_cast<uintptr_t>(scratch) & 15)))
        return m3d::einval("set_deterministic: needs a 16-byte aligned device scratch of >= 4096 bytes");
    m3d::g_det = on ? m3d::DetState{1, scratch, bytes} : m3d::DetState{0, nullptr, 0};
    return M3D_OK;
}

extern "C" int32_t m3d_get_deterministic(void) { return m3d::g_det.on; }

// ---- stream fork / join ----------------------------------------------------
// The training step forks every layer's weight gradient onto a side stream.
// torch's wait_stream records a default event, whose completion performs a
// system-scope release (L2 write-back + invalidate) on the recording stream:
// measured as a ~7.5 us bubble on the compute queue per fork.  These events
// use a device-scope release (mode 1) or no system-scope fence (mode 2, the
// training step's default: -0.2 ms per 128^3 step): the waiting stream is on
// the same device, so agent-scope visibility is all it needs.
#include <mutex>

namespace m3d {
constexpr int kEvRing = 64, kMaxDev = 16;
struct EvRing {
    hipEvent_t ev[kEvRing];
    int next = 0;
    bool init = false;
};
static EvRing g_rings[kMaxDev][3];
static std::mutex g_ring_mu;
}  // namespace m3d

extern "C" int m3d_stream_fork(m3d_stream_t from, m3d_stream_t to, int32_t mode) {
    using namespace m3d;
    if (mode < 0 || mode > 2) return einval("stream_fork: mode must be 0, 1 or 2");
    int dev = 0;
    if (hipStreamGetDevice(st(from), &dev) != hipSuccess || dev < 0 || dev >= kMaxDev)
        return check_launch("stream_fork: hipStreamGetDevice");
    hipEvent_t ev;
    {
        std::lock_guard<std::mutex> lk(g_ring_mu);
        EvRing& r = g_rings[dev][mode];
        if (!r.init) {
            const unsigned flags = hipEventDisableTiming |
                                   (mode == 1 ? hipEventReleaseToDevice : 0u) |
                                   (mode == 2 ? hipEventDisableSystemFence : 0u);
            int cur = 0;
            hipGetDevice(&cur);
            hipSetDevice(dev);
            for (int i = 0; i < kEvRing; ++i) {
                if (hipEventCreateWithFlags(&r.ev[i], flags) != hipSuccess) {
                    hipSetDevice(cur);
                    return check_launch("stream_fork: hipEventCreateWithFlags");
                }
            }
            hipSetDevice(cur);
            r.init = true;
        }
        ev = r.ev[r.next];
        r.next = (r.next + 1) % kEvRing;
    }
    if (hipEventRecord(ev, st(from)) != hipSuccess) return check_launch("stream_fork: hipEventRecord");
    if (hipStreamWaitEvent(st(to), ev, 0) != hipSuccess) return check_launch("stream_fork: hipStreamWaitEvent");
    return M3D_OK;
}
