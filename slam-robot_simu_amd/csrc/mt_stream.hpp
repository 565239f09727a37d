// mt_stream.hpp -- the device replica of NumPy's legacy RandomState stream
// (rng_api.hip), as an in-library interface for the filters that draw from it.
//
// One draw request, enqueued on a stream with no host synchronisation (so it
// can be captured in a hipGraph):
//   [n_pre doubles (random_sample), or one if *pre_flag] then G normals
//   (legacy gauss, the cached normal first).
// It advances the device state exactly as NumPy would after the same calls.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mt19937.hpp"

namespace slam {

struct MtDeviceState {
    uint32_t key[kMtN];
    int32_t pos;
    int32_t has_gauss;
    double gauss;
    // request scratch (written by the emit pass, read by the finish pass)
    int64_t j_end;          // words consumed through the last accepted pair
    double new_gauss;
    int32_t short_draw;     // candidate bound exhausted (never in practice)
    int32_t pad;
};

struct MtBuffers {
    int device = 0;
    MtDeviceState* st = nullptr;
    GlibcLogTable* tab = nullptr;   // device copy of glibc's log table
    uint32_t* X = nullptr;          // untempered stream: the key, then generated blocks
    unsigned* bcnt = nullptr;       // accepted candidates per count block
    int64_t* boff = nullptr;        // their exclusive prefix
    double* normals = nullptr;      // G normals of the last request
    double* pre = nullptr;          // n_pre doubles of the last request (standalone use)
    int64_t g_cap = 0;              // normals per request this allocation holds
    int64_t pre_cap = 0;            // doubles before the normals
    int64_t cand_cap = 0;           // candidate pairs examined per request
    int64_t nblk = 0;               // blocks of 624 generated per request
    int64_t nb_count = 0;           // count / emit blocks
};

// glibc's log table from this process's libm, checked against log() (cached).
int glibc_log_table(GlibcLogTable* out);

// Size the buffers for requests of up to g_cap normals after up to pre_cap
// doubles (grow-only; frees and reallocates).
int mt_reserve(MtBuffers& b, int64_t g_cap, int64_t pre_cap, int device);
void mt_free(MtBuffers& b);

int mt_set_state(MtBuffers& b, const uint32_t* key, int32_t pos, int32_t has_gauss, double gauss,
                 hipStream_t s);
int mt_get_state(const MtBuffers& b, uint32_t* key, int32_t* pos, int32_t* has_gauss, double* gauss,
                 hipStream_t s);   // synchronises s

// Enqueue one request of g normals (into b.normals) after the pre-draw:
// n_pre doubles into pre_out[0..n_pre) (pre_flag == nullptr), or, with
// pre_flag, one double if *pre_flag != 0 (NaN otherwise) into
// pre_out[pre_index ? *pre_index : 0]; every pre-draw is scaled by pre_scale.
// status (nullable) gets bit 8 (256) if the candidate bound was exhausted.
int mt_enqueue(const MtBuffers& b, int64_t n_pre, const int32_t* pre_flag, double pre_scale,
               double* pre_out, const int32_t* pre_index, int64_t g, int32_t* status, hipStream_t s);

}  // namespace slam
