// mt_stream.hpp -- the device replica of NumPy's legacy RandomState stream
// (rng_api.hip), as an in-library interface for the filters that draw from it.
//
// One draw request, enqueued on a stream with no host synchronisation (so it
// can be captured in a hipGraph):
//   [n_pre doubles (random_sample), or one if *pre_flag] then G normals
//   (legacy gauss, the cached normal first).
// It advances the device state exactly as NumPy would after the same calls.
//
// The untempered MT19937 sequence lives in a ring of words indexed by stream
// position (word 0 = key[0] of the state set last).  It is produced in rounds
// of R segments x S words, one workgroup per segment: a segment starts from
// its "pre-window" (the 624 words ending just before it) and runs the
// recurrence; the pre-window of the same segment one round later is the
// window R*S words further on, obtained by jump-ahead -- x^(R S) mod phi(x)
// (phi: MT19937's characteristic polynomial) applied as an XOR of shifted
// windows of the segment's own first 19937 + 623 words.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mt19937.hpp"

namespace slam {

constexpr int kMtDeg = 19937;                       // degree of phi
constexpr int kMtQWords = (kMtDeg + 63) / 64;       // 312
constexpr int kMtConvWords = kMtDeg + kMtN - 1;     // words one jump reads (20560)
constexpr int kMtMinSeg = 33 * kMtN;                // segment length when R > 1 (>= kMtConvWords + 1)
constexpr int kMtMaxSegs = 256;

struct MtDeviceState {
    int64_t p;              // stream position of the next word
    int64_t g1;             // words [.., g1) are generated
    int32_t has_gauss;
    int32_t short_draw;     // candidate bound exhausted (never in practice)
    double gauss;
    int64_t j_end;          // request scratch: words consumed through the last accepted pair
    double new_gauss;
};

struct MtBuffers {
    int device = 0;
    MtDeviceState* st = nullptr;
    GlibcLogTable* tab = nullptr;   // device copy of glibc's log table
    uint32_t* X = nullptr;          // ring of cap (a power of two) words: word k at X[k & (cap - 1)]
    int64_t cap = 0;
    uint32_t* seg = nullptr;        // [R][624] pre-windows of the next round's segments
    uint32_t* q = nullptr;          // x^(R S) mod phi: its set bits as 16-bit offsets (R > 1)
    int32_t n_idx = 0;              // offsets (a multiple of 16, padded)
    unsigned* bcnt = nullptr;       // accepted candidates per count block
    unsigned* bpre = nullptr;       // [nb + 1] their exclusive prefix (many blocks only)
    double* normals = nullptr;      // G normals of the last request
    double* pre = nullptr;          // n_pre doubles of the last request (standalone use)
    int64_t g_cap = 0;              // normals per request this allocation holds
    int64_t pre_cap = 0;            // doubles before the normals
    int64_t cand_cap = 0;           // candidate pairs examined per request
    int64_t nb_count = 0;           // count / emit blocks
    int64_t need = 0;               // words a request may read past the position (+ margins)
    int32_t R = 1;                  // segments per round
    int64_t S = 0;                  // words per segment (a multiple of 624)
};

// glibc's log table from this process's libm, checked against log() (cached).
int glibc_log_table(GlibcLogTable* out);

// Size the buffers for requests of up to g_cap normals after up to pre_cap
// doubles (grow-only; a regrow keeps the stream state).
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

// Host jump-ahead (tests): the pre-window J words after `win` (both 624 words;
// word 0's low 31 bits are not part of the state and come back unspecified).
int mt_jump_window_host(const uint32_t* win, uint64_t J, uint32_t* out);

}  // namespace slam
