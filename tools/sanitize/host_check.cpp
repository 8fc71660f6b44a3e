// Edge cases of the library's host-only entry points (csrc/detok.cpp, csrc/pdvc_status.cpp) for the sanitizer pass
// (tools/sanitize/run.sh): every output buffer is a heap block of exactly the size passed, so a write past it is an
// ASan report; every case checks the return code and, where it succeeds, the bytes.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pdvc_msda.h"

extern "C" int pdvc_set_error(int code, const char* fmt, ...);
extern "C" int pdvc_detokenize(const int64_t* seqs, int rows, int len, const char* words, const int64_t* word_off,
                               int num_words, char* out, int64_t out_cap, int64_t* row_end);

static int fails = 0;
#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                  \
        }                                                             \
    } while (0)

struct Vocab {  // ids 1..n-1 -> words; id 0 is the end token
    std::string words;
    std::vector<int64_t> off{0, 0};
    explicit Vocab(const std::vector<std::string>& w) {
        for (const auto& s : w) {
            words += s;
            off.push_back((int64_t)words.size());
        }
    }
    int num() const { return (int)off.size() - 1; }
};

// detokenise into an exact-size heap buffer of `cap` bytes
static int run(const Vocab& v, const std::vector<int64_t>& seqs, int rows, int len, int64_t cap, std::string* out,
               std::vector<int64_t>* ends) {
    char* buf = static_cast<char*>(std::malloc(cap > 0 ? (size_t)cap : 1));
    int64_t* re = static_cast<int64_t*>(std::malloc(sizeof(int64_t) * (rows > 0 ? rows : 1)));
    const int rc = pdvc_detokenize(seqs.empty() ? nullptr : seqs.data(), rows, len, v.words.data(), v.off.data(),
                                   v.num(), buf, cap, re);
    if (rc == PDVC_OK) {
        *out = std::string(buf, rows ? (size_t)re[rows - 1] : 0);
        ends->assign(re, re + rows);
    }
    std::free(buf);
    std::free(re);
    return rc;
}

int main() {
    const Vocab v({"a", "caf\xc3\xa9", "longerword"});
    std::string s;
    std::vector<int64_t> e;
    // ordinary rows: words joined by spaces, a full stop; a row starting with 0 is empty; a full-length row
    CHECK(run(v, {1, 2, 0, 0, 1, 3, 3, 3, 3}, 3, 3, 64, &s, &e) == PDVC_OK);
    CHECK(s == "a caf\xc3\xa9." "longerword longerword longerword.");
    CHECK(e.size() == 3 && e[0] == 8 && e[1] == 8);
    // exact fit, and one byte short (an error, nothing written past the block)
    const int64_t need = (int64_t)std::strlen("longerword longerword longerword.");
    CHECK(run(v, {3, 3, 3}, 1, 3, need + 1, &s, &e) == PDVC_OK);  // (+1: the bound reserves a separator byte)
    CHECK(run(v, {3, 3, 3}, 1, 3, need - 1, &s, &e) == PDVC_ERR_INVALID_ARG);
    CHECK(run(v, {3}, 1, 1, 1, &s, &e) == PDVC_ERR_INVALID_ARG);
    // no rows, zero-length rows
    CHECK(run(v, {}, 0, 5, 1, &s, &e) == PDVC_OK);
    CHECK(run(v, {}, 4, 0, 1, &s, &e) == PDVC_OK && e.size() == 4 && e[3] == 0);
    // ids outside [1, num_words): errors
    CHECK(run(v, {1, 9}, 1, 2, 64, &s, &e) == PDVC_ERR_INVALID_ARG);
    CHECK(run(v, {-2}, 1, 1, 64, &s, &e) == PDVC_ERR_INVALID_ARG);
    // a word table whose offsets run backwards: an error, not a negative-length copy
    Vocab bad({"x", "y"});
    bad.off[2] = 5;
    CHECK(run(bad, {2}, 1, 1, 64, &s, &e) == PDVC_ERR_INVALID_ARG);
    // NULL pointers and negative sizes
    char one;
    int64_t re1;
    CHECK(pdvc_detokenize(nullptr, 1, 1, v.words.data(), v.off.data(), v.num(), &one, 1, &re1) == PDVC_ERR_INVALID_ARG);
    CHECK(pdvc_detokenize(nullptr, -1, 1, v.words.data(), v.off.data(), v.num(), &one, 1, &re1) == PDVC_ERR_INVALID_ARG);
    // the error message: formatted, truncated to the thread-local buffer, NUL-terminated
    std::string longmsg(2000, 'z');
    CHECK(pdvc_set_error(-7, "%s", longmsg.c_str()) == -7);
    const char* m = pdvc_last_error();
    CHECK(m != nullptr && std::strlen(m) < 2000 && std::strlen(m) > 100 && m[0] == 'z');
    CHECK(pdvc_set_error(-3, "code %d %s", 42, "x") == -3 && std::string(pdvc_last_error()) == "code 42 x");
    CHECK(pdvc_abi_version() == PDVC_ABI_VERSION);
    if (fails) return 1;
    std::printf("host_check: all cases passed\n");
    return 0;
}
