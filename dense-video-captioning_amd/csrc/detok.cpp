// detok.cpp -- host-side caption detokenisation for the evaluation pass (reference: Translator.rtranslate,
// data/video_dataset.py:172-180, which PostProcess calls once per query and video, pdvc/pdvc.py:493-546).
// Every row: the ids up to its first 0; none -> the empty caption; else the words joined by single spaces,
// then a full stop.  All rows go into one byte buffer (row r ends at row_end[r]), so the caller builds the
// Python strings from one buffer instead of one join per caption (the Python join cost ~8 us per caption:
// 0.2 s of a 256-video evaluation step).
#include <cstdint>
#include <cstring>

#include "pdvc_msda.h"

extern "C" int pdvc_set_error(int code, const char* fmt, ...);  // pdvc_status.cpp

extern "C" int pdvc_detokenize(const int64_t* seqs, int rows, int len, const char* words, const int64_t* word_off,
                               int num_words, char* out, int64_t out_cap, int64_t* row_end) {
    if (rows < 0 || len < 0 || num_words < 1) return pdvc_set_error(PDVC_ERR_INVALID_ARG, "pdvc_detokenize: invalid sizes");
    if ((rows > 0 && len > 0 && !seqs) || !words || !word_off || !out || !row_end)
        return pdvc_set_error(PDVC_ERR_INVALID_ARG, "pdvc_detokenize: NULL pointer");
    int64_t pos = 0;
    for (int r = 0; r < rows; ++r) {
        const int64_t* s = seqs + (int64_t)r * len;
        int n = 0;
        while (n < len && s[n] != 0) ++n;
        for (int i = 0; i < n; ++i) {
            const int64_t w = s[i];
            if (w < 1 || w >= num_words)
                return pdvc_set_error(PDVC_ERR_INVALID_ARG, "pdvc_detokenize: word id %lld outside [1, %d)", (long long)w,
                                      num_words);
            const int64_t a = word_off[w], b = word_off[w + 1];
            if (b < a) return pdvc_set_error(PDVC_ERR_INVALID_ARG, "pdvc_detokenize: word_off decreases at id %lld", (long long)w);
            if (pos + (b - a) + 2 > out_cap) return pdvc_set_error(PDVC_ERR_INVALID_ARG, "pdvc_detokenize: output full");
            if (i) out[pos++] = ' ';
            std::memcpy(out + pos, words + a, (size_t)(b - a));
            pos += b - a;
        }
        if (n) {
            if (pos + 1 > out_cap) return pdvc_set_error(PDVC_ERR_INVALID_ARG, "pdvc_detokenize: output full");
            out[pos++] = '.';
        }
        row_end[r] = pos;
    }
    return PDVC_OK;
}
