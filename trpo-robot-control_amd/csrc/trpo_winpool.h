/* trpo_winpool.h -- the process-lifetime pool of uncached peer windows (trpo_peer.hip), as plain C so
 * that its policy is testable without a GPU (tests/test_winpool.py compiles it with gcc).
 *
 * Why a pool (round 5): under the ROCm 7.0 runtime a PyTorch wheel bundles, hipFree of an
 * uncached window left every LATER context of the process computing a wrong first FVP; keeping the
 * windows for the life of the process avoids the trigger.  It is a mitigation, not a root cause.
 *
 * What happens to a window when its context goes (winpool_give):
 *   - its exchange failed or was abandoned (a poll timed out, trpo_peer_set_error): LEAK it.  A peer of
 *     that group may still finish a late push into it, and a pooled window restarts its exchange numbers
 *     at 1, so such a push could carry a tag the next group expects;
 *   - otherwise PARK it while the pool has room (the next peer context of the same size takes it back);
 *   - pool full: FREE it only under the HIP runtime the library was built against; under another
 *     runtime LEAK it and say so on stderr (the overflow is no longer a silent hipFree). */
#ifndef TRPO_WINPOOL_H
#define TRPO_WINPOOL_H

#include <stddef.h>

#define WINPOOL_CAP 16

enum { WINPOOL_PARKED = 0, WINPOOL_FREED = 1, WINPOOL_LEAKED_FAILED = 2, WINPOOL_LEAKED_FULL = 3 };

typedef struct {
    void *p;
    size_t bytes;
    int device;
} winpool_slot;

typedef struct {
    winpool_slot slot[WINPOOL_CAP];
    int n;
    int warned;
} winpool;

/* a parked window of this device and size, or NULL (the caller then allocates a new one) */
static inline void *winpool_take(winpool *w, int device, size_t bytes) {
    for (int i = 0; i < w->n; ++i)
        if (w->slot[i].device == device && w->slot[i].bytes == bytes) {
            void *p = w->slot[i].p;
            w->slot[i] = w->slot[--w->n];
            return p;
        }
    return NULL;
}

/* decides (and records) what happens to a released window; the caller frees it on WINPOOL_FREED and
 * prints the warning when *warn is set (once per process) */
static inline int winpool_give(winpool *w, void *p, size_t bytes, int device, int failed, int runtime_built,
                               int *warn) {
    *warn = 0;
    if (failed) return WINPOOL_LEAKED_FAILED;
    if (w->n < WINPOOL_CAP) {
        w->slot[w->n].p = p;
        w->slot[w->n].bytes = bytes;
        w->slot[w->n].device = device;
        ++w->n;
        return WINPOOL_PARKED;
    }
    if (runtime_built) return WINPOOL_FREED;
    if (!w->warned) {
        w->warned = 1;
        *warn = 1;
    }
    return WINPOOL_LEAKED_FULL;
}

#endif
