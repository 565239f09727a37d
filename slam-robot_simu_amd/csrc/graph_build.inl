// graph_build.inl -- the edge set's block structure built on the device
// (included by graph_api.hip).
//
// updateEstPose (graph_based_slam.py:452-514) accumulates every edge's four
// 3x3 blocks into H at (bfr, bfr), (bfr, aft), (aft, bfr), (aft, aft) and its
// two 3-vectors into b, in edge order (:484-492), over the distinct times of
// the edge set in ascending order (the index of :457-467).  The structure the
// Gauss-Newton iterations reuse -- distinct times, the BSR slots of H (row
// major), the diagonal slot per row, and the accumulation plans (which edge
// parts land in each slot / each b row, in edge order) -- is sorts, uniques
// and binary searches: rocPRIM radix sorts (stable: equal keys keep edge
// order) and small hand-written kernels, no host pass over the edges.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>

namespace slam {

// first index in sorted a[0, n) with a[i] >= v
__device__ __forceinline__ int64_t gb_lower_bound(const int64_t* __restrict__ a, int64_t n,
                                                  const int64_t v) {
    int64_t lo = 0;
    while (n > 0) {
        const int64_t h = n >> 1;
        if (a[lo + h] < v) {
            lo += h + 1;
            n -= h + 1;
        } else {
            n = h;
        }
    }
    return lo;
}

// both endpoint times of every edge
__global__ void gb_times_kernel(const int64_t E, const slam_graph_edge* __restrict__ ed,
                                int64_t* __restrict__ tl) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    tl[2 * e] = ed[e].time_bfr;
    tl[2 * e + 1] = ed[e].time_aft;
}

// endpoint ranks and the slot keys r * nt + c: the diagonal of every time
// (rows 0 .. nt-1 of a block of nt_ub entries, the rest a sentinel) and both
// off-diagonal blocks of every edge; the b plan's row keys and values
__global__ void gb_keys_kernel(const int64_t E, const slam_graph_edge* __restrict__ ed,
                               const int64_t* __restrict__ times, const int64_t* __restrict__ nt_p,
                               const int64_t nt_ub, int64_t* __restrict__ rb, int64_t* __restrict__ ra,
                               int64_t* __restrict__ keys, int64_t* __restrict__ bkey,
                               int64_t* __restrict__ bval) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = *nt_p;
    if (i < nt_ub) keys[2 * E + i] = (i < nt) ? i * nt + i : INT64_MAX;
    if (i >= E) return;
    const int64_t b = gb_lower_bound(times, nt, ed[i].time_bfr);
    const int64_t a = gb_lower_bound(times, nt, ed[i].time_aft);
    rb[i] = b;
    ra[i] = a;
    keys[2 * i] = b * nt + a;
    keys[2 * i + 1] = a * nt + b;
    bkey[2 * i] = b;                    // b rows: (edge, side) in edge order (:488-492)
    bkey[2 * i + 1] = a;
    bval[2 * i] = 2 * i;
    bval[2 * i + 1] = 2 * i + 1;
}

// the slot of each edge part c = 4 e + {bb, ba, ab, aa} (updateEstPose :484-487)
__global__ void gb_parts_kernel(const int64_t E, const int64_t* __restrict__ rb,
                                const int64_t* __restrict__ ra, const int64_t* __restrict__ nt_p,
                                const int64_t* __restrict__ ukeys, const int64_t* __restrict__ ns_p,
                                int64_t* __restrict__ sl, int64_t* __restrict__ cval) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= 4 * E) return;
    const int64_t nt = *nt_p, ns = *ns_p, e = c >> 2, k = c & 3;
    const int64_t r = (k < 2) ? rb[e] : ra[e];
    const int64_t q = (k == 0 || k == 2) ? rb[e] : ra[e];
    sl[c] = gb_lower_bound(ukeys, ns, r * nt + q);
    cval[c] = c;
}

// per slot: row, column, the diagonal slot of its row; per row: its first slot
__global__ void gb_slots_kernel(const int64_t* __restrict__ ukeys, const int64_t* __restrict__ ns_p,
                                const int64_t* __restrict__ nt_p, const int64_t cap,
                                int64_t* __restrict__ srow, int64_t* __restrict__ scol,
                                int64_t* __restrict__ dslot, int64_t* __restrict__ rptr) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ns = *ns_p, nt = *nt_p;
    if (s < ns) {
        const int64_t r = ukeys[s] / nt, c = ukeys[s] % nt;
        srow[s] = r;
        scol[s] = c;
        if (r == c) dslot[r] = s;
    }
    if (s <= nt && s < cap) rptr[s] = gb_lower_bound(ukeys, ns, s * nt);
}

// CSR offsets of a sorted key array: off[i] = #keys < i, i in [0, m]
__global__ void gb_offsets_kernel(const int64_t* __restrict__ sorted, const int64_t n,
                                  const int64_t* __restrict__ m_p, const int64_t cap,
                                  int64_t* __restrict__ off) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= *m_p && i < cap) off[i] = gb_lower_bound(sorted, n, i);
}

// drop the sentinel slot (present when nt < nt_ub)
__global__ void gb_count_kernel(const int64_t* __restrict__ ukeys, int64_t* __restrict__ ns_p) {
    const int64_t ns = *ns_p;
    if (ns > 0 && ukeys[ns - 1] == INT64_MAX) *ns_p = ns - 1;
}

int bits_for(uint64_t v) {
    int b = 1;
    while (b < 64 && (v >> b)) ++b;
    return b;
}

}  // namespace slam
