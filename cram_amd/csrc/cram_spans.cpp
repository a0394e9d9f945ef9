// Host-side passage spans -> credibility weights (re_weighting.py:100-111), batched over prompts.
//
// The reference scans the whole offset mapping once per passage in Python
// (re_weighting.py:105-109: the LAST token whose start offset is <= the passage's first / last
// character).  Here every prompt's token starts are checked for monotonicity once; monotone rows
// (the normal case) use a binary search per passage boundary, others fall back to the same
// last-match scan, so non-monotone offset maps (special tokens at (0,0) in the middle) give the
// reference's answer too.  Weights are written as fp16 bits: score -> fp32 -> fp16 (RNE), the
// conversion chain of torch.full(..., scores[i]).to(torch.float16) (re_weighting.py:110).
#include <cstdint>
#include <cstring>

#include "cram_attn.h"

// The build's source hash (cram_amd/build.py: sha256 of every source, header and flag), embedded as a tag the
// Python side reads from the .so file itself, so a stale library is rebuilt by content, never by mtime.
#ifdef CRAM_SOURCE_HASH
extern "C" __attribute__((used, visibility("default"))) const char cram_source_hash_tag[] =
    "CRAM_SOURCE_HASH=" CRAM_SOURCE_HASH;
#endif

namespace {

uint16_t f32_to_f16_bits(float f) {
    _Float16 h = static_cast<_Float16>(f);   // RNE, IEEE binary16 (inf/nan preserved)
    uint16_t b;
    std::memcpy(&b, &h, sizeof(b));
    return b;
}

// max{t : start[t] <= c}, or -1
int64_t last_le_scan(const int64_t* start, int64_t T, int64_t c) {
    for (int64_t t = T - 1; t >= 0; --t)
        if (start[t] <= c) return t;
    return -1;
}

int64_t last_le_sorted(const int64_t* start, int64_t T, int64_t c) {
    int64_t lo = 0, hi = T;                    // first t with start[t] > c
    while (lo < hi) {
        int64_t mid = lo + (hi - lo) / 2;
        if (start[mid] <= c) lo = mid + 1; else hi = mid;
    }
    return lo - 1;
}

}  // namespace

extern "C" int cram_passage_weights(int B, const int64_t* cu_tok, const int64_t* tok_start, const int64_t* cu_par,
                                    const int64_t* char_lo, const int64_t* char_hi, const float* score,
                                    int32_t* span_lo, int32_t* span_hi, uint16_t* w16) {
    if (B < 0 || !cu_tok || !cu_par || (cu_tok[B] > 0 && (!tok_start || !w16)) ||
        (cu_par[B] > 0 && (!char_lo || !char_hi || !score || !span_lo || !span_hi)))
        return CRAM_ERR_INVALID_ARG;
    const uint16_t one = f32_to_f16_bits(1.0f);
    for (int b = 0; b < B; ++b) {
        const int64_t t0 = cu_tok[b], T = cu_tok[b + 1] - cu_tok[b];
        const int64_t p0 = cu_par[b], P = cu_par[b + 1] - cu_par[b];
        if (T < 0 || P < 0) return CRAM_ERR_INVALID_ARG;
        const int64_t* st = tok_start + t0;
        uint16_t* w = w16 + t0;
        bool sorted = true;
        for (int64_t t = 1; t < T && sorted; ++t) sorted = st[t - 1] <= st[t];
        for (int64_t t = 0; t < T; ++t) w[t] = one;
        for (int64_t p = p0; p < p0 + P; ++p) {
            if (char_lo[p] < 0 || char_hi[p] < char_lo[p]) return CRAM_ERR_INVALID_ARG;   // passage not found
            int64_t a = sorted ? last_le_sorted(st, T, char_lo[p]) : last_le_scan(st, T, char_lo[p]);
            int64_t e = sorted ? last_le_sorted(st, T, char_hi[p]) : last_le_scan(st, T, char_hi[p]);
            if (a < 0 || e < 0) return CRAM_ERR_INVALID_ARG;
            span_lo[p] = static_cast<int32_t>(a);
            span_hi[p] = static_cast<int32_t>(e);
            const uint16_t v = f32_to_f16_bits(score[p]);
            for (int64_t t = a; t <= e; ++t) w[t] = v;                                     // later passages overwrite
        }
    }
    return CRAM_OK;
}
