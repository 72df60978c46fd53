// Episode-aware ring arithmetic of the VectorReplayBuffer shared by the kernels that walk
// prev/next chains on device (stack.hip, replay.hip).
//
// ReplayBufferManager prev/next (tianshou/data/buffer/manager.py:259-297, the numba
// _prev_index/_next_index).  Sub-buffer b owns storage rows [b*size, (b+1)*size)
// (vecbuf.py:33-37: equal sub-buffers), holds lengths[b] rows and last wrote last_index[b];
// a row whose done flag is set, or the last written row, ends an episode, so prev() does not
// step back across it and next() does not step forward across it.
#pragma once
#include "tsrl_common.h"

namespace tsrl {

struct Ring {
    const uint8_t* done;
    const int64_t* last_index;
    const int64_t* lengths;
    int64_t size;     // rows per sub-buffer
    int64_t maxsize;  // size * num
};

__device__ __forceinline__ int64_t pmod(int64_t a, int64_t m) {
    const int64_t r = a % m;
    return r < 0 ? r + m : r;
}

// manager.py:259-277
__device__ __forceinline__ int64_t ring_prev(const Ring& g, int64_t i) {
    i = pmod(i, g.maxsize);
    const int64_t b = i / g.size;
    const int64_t start = b * g.size;
    const int64_t cur = max(g.lengths[b], (int64_t)1);
    const int64_t sub = pmod(i - start - 1, cur);
    const int64_t end = (g.done[sub + start] != 0) | (sub + start == g.last_index[b]);
    return pmod(sub + end, cur) + start;
}

// manager.py:280-297
__device__ __forceinline__ int64_t ring_next(const Ring& g, int64_t i) {
    i = pmod(i, g.maxsize);
    const int64_t b = i / g.size;
    const int64_t start = b * g.size;
    const int64_t cur = max(g.lengths[b], (int64_t)1);
    const int64_t end = (g.done[i] != 0) | (i == g.last_index[b]);
    return pmod(i - start + 1 - end, cur) + start;
}

// The episode-end flag of compute_nstep_return (base.py:433-434): done, or the unfinished
// last row of a non-empty sub-buffer (unfinished_index, manager.py:68-74) -- i.e. exactly the
// rows next() does not step across.
__device__ __forceinline__ bool ring_end(const Ring& g, int64_t i) {
    const int64_t b = i / g.size;
    return g.done[i] != 0 || (i == g.last_index[b] && g.lengths[b] > 0);
}

}  // namespace tsrl
