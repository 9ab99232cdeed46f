// Host-side readers for the reference's on-disk interaction formats.
//
// The reference parses its text files line by line in Python (utils/dataset.py):
//   * load_negative_file (:245-256): per line, line.split('\t')[1:] -> int() each field; the first
//     field is the "(u,i)" key and is dropped.  The Allrecipes test/valid negative files are
//     68,768 x 999 and 29,000 x 999 ids (~285 MB of text), ~17 s of a ~25 s load in Python.
//   * load_valid_test_file_as_dict / load_*_file_as_list / load_training_file_as_matrix (:93-176):
//     int(arr[0]), int(arr[1]) and (training file) float(arr[2]) per line.
// Here the file is memory-mapped and split into byte ranges at line boundaries, one std::thread per
// range: pass 1 counts rows and fields (fr_io_open), the caller allocates, pass 2 parses straight
// into the caller's arrays (fr_io_fill).  Field rules follow Python's int()/float() as the reference
// calls them: surrounding whitespace is stripped, an empty or malformed field is an error (the
// reference raises ValueError there), an empty line of a negative file is a row with no ids.
//
// The evaluation candidate lists (EvalByUserDataloader, dataloader.py:228-302) remove each positive
// from the user's negatives with list.remove -- the first remaining occurrence, in place, so the
// removal persists across evaluations.  fr_io_remove_positives restates that over an alive mask.
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "fr_engine.h"

namespace fr {
void set_error(const std::string& msg);  // fr_error.cpp
}

namespace {

struct Range {
    int64_t begin, end;      // byte range [begin, end), starting at a line start
    int64_t rows = 0;        // lines starting in the range
    int64_t fields = 0;      // values those lines contribute
    int64_t row0 = 0, val0 = 0;  // prefix sums
    int64_t bad_line = -1;   // first malformed line (0-based within the range), -1 if none
    std::string msg;
};

}  // namespace

struct fr_io_table {
    int mode = 0;
    const char* data = nullptr;
    int64_t size = 0;
    std::vector<Range> ranges;
    int64_t rows = 0, values = 0;
};

namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

// int(field): optional sign, decimal digits, optional '_' between digits, surrounding whitespace
bool parse_int(const char* b, const char* e, int64_t* out) {
    while (b < e && is_space(*b)) ++b;
    while (e > b && is_space(e[-1])) --e;
    if (b == e) return false;
    bool neg = false;
    if (*b == '+' || *b == '-') { neg = *b == '-'; ++b; }
    if (b == e || *b < '0' || *b > '9') return false;
    uint64_t v = 0;
    const uint64_t lim = neg ? uint64_t(INT64_MAX) + 1 : uint64_t(INT64_MAX);  // int64 range (the id arrays')
    bool prev_digit = false;
    for (; b < e; ++b) {
        char c = *b;
        if (c >= '0' && c <= '9') {
            const uint64_t d = uint64_t(c - '0');
            if (v > (lim - d) / 10) return false;  // outside int64: no wrapped id
            v = v * 10 + d;
            prev_digit = true;
        } else if (c == '_' && prev_digit && b + 1 < e && b[1] >= '0' && b[1] <= '9') {
            prev_digit = false;
        } else {
            return false;
        }
    }
    *out = neg ? (v ? -int64_t(v - 1) - 1 : 0) : int64_t(v);
    return true;
}

// float(field) via strtod on a bounded copy
bool parse_float(const char* b, const char* e, double* out) {
    while (b < e && is_space(*b)) ++b;
    while (e > b && is_space(e[-1])) --e;
    if (b == e || e - b > 63) return false;
    char buf[64];
    std::memcpy(buf, b, size_t(e - b));
    buf[e - b] = 0;
    char* end = nullptr;
    errno = 0;
    double v = std::strtod(buf, &end);
    if (end != buf + (e - b)) return false;
    *out = v;
    return true;
}

inline const char* line_end(const char* p, const char* end) {
    const void* nl = std::memchr(p, '\n', size_t(end - p));
    return nl ? static_cast<const char*>(nl) : end;
}

// pass 1: rows and fields per range
void count_range(const fr_io_table& t, Range& r) {
    const char* p = t.data + r.begin;
    const char* end = t.data + r.end;
    while (p < end) {
        const char* le = line_end(p, end);
        ++r.rows;
        if (t.mode == FR_IO_NEGATIVE) {
            // fields after the first = tabs in the line
            int64_t tabs = 0;
            for (const char* q = p; q < le; ++q) tabs += (*q == '\t');
            r.fields += tabs;
        } else {
            r.fields += 2;
        }
        p = le + 1;
    }
}

void set_bad(Range& r, int64_t line, const char* what, const char* b, const char* e) {
    if (r.bad_line >= 0) return;
    r.bad_line = line;
    r.msg = std::string(what) + " '" + std::string(b, size_t(std::min<int64_t>(e - b, 40))) + "'";
}

// pass 2: parse into the caller's arrays
void fill_range(const fr_io_table& t, Range& r, int64_t* values, int64_t* offsets, double* aux) {
    const char* p = t.data + r.begin;
    const char* end = t.data + r.end;
    int64_t row = r.row0, val = r.val0, line = 0;
    while (p < end) {
        const char* le = line_end(p, end);
        if (t.mode == FR_IO_NEGATIVE) {
            const char* f = static_cast<const char*>(std::memchr(p, '\t', size_t(le - p)));
            if (offsets) offsets[row] = val;
            while (f) {
                const char* fb = f + 1;
                const char* fe = static_cast<const char*>(std::memchr(fb, '\t', size_t(le - fb)));
                const char* stop = fe ? fe : le;
                int64_t v = 0;
                if (!parse_int(fb, stop, &v)) set_bad(r, line, "invalid literal for int() with base 10:", fb, stop);
                values[val++] = v;
                f = fe;
            }
        } else {
            const char* f0e = static_cast<const char*>(std::memchr(p, '\t', size_t(le - p)));
            int64_t u = 0, i = 0;
            double rating = NAN;
            if (!f0e) {
                set_bad(r, line, "expected at least two tab-separated fields:", p, le);
            } else {
                const char* f1b = f0e + 1;
                const char* f1e = static_cast<const char*>(std::memchr(f1b, '\t', size_t(le - f1b)));
                if (!parse_int(p, f0e, &u)) set_bad(r, line, "invalid literal for int() with base 10:", p, f0e);
                if (!parse_int(f1b, f1e ? f1e : le, &i))
                    set_bad(r, line, "invalid literal for int() with base 10:", f1b, f1e ? f1e : le);
                if (f1e && aux) {
                    const char* f2b = f1e + 1;
                    const char* f2e = static_cast<const char*>(std::memchr(f2b, '\t', size_t(le - f2b)));
                    if (!parse_float(f2b, f2e ? f2e : le, &rating))
                        set_bad(r, line, "could not convert string to float:", f2b, f2e ? f2e : le);
                }
            }
            values[2 * row] = u;
            values[2 * row + 1] = i;
            if (aux) aux[row] = rating;
            val += 2;
        }
        ++row;
        ++line;
        p = le + 1;
    }
}

// threads <= 0: min(hardware threads, 16) with >= 4 MB of text each; an explicit count is kept
// (at most one thread per byte), so small files can exercise the range cuts
int pick_threads(int threads, int64_t size) {
    if (threads > 0) return int(std::max<int64_t>(1, std::min<int64_t>(threads, size)));
    unsigned hc = std::thread::hardware_concurrency();
    int64_t n = std::min<unsigned>(hc ? hc : 1, 16);
    return int(std::max<int64_t>(1, std::min<int64_t>(n, size >> 22)));
}

// per-user passes: >= 256 users per thread unless a count is given
int user_threads(int threads, int64_t n_users) {
    if (threads > 0) return int(std::max<int64_t>(1, std::min<int64_t>(threads, n_users)));
    unsigned hc = std::thread::hardware_concurrency();
    int64_t n = std::min<unsigned>(hc ? hc : 1, 16);
    return int(std::max<int64_t>(1, std::min<int64_t>(n, n_users / 256 + 1)));
}

template <class F>
void run_threads(int n, F&& f) {
    if (n == 1) { f(0); return; }
    std::vector<std::thread> th;
    th.reserve(size_t(n));
    for (int k = 0; k < n; ++k) th.emplace_back(f, k);
    for (auto& x : th) x.join();
}

}  // namespace

extern "C" {

int fr_io_open(const char* path, int mode, int threads, fr_io_table** out, int64_t* rows, int64_t* values) {
    if (!path || !out || !rows || !values || (mode != FR_IO_NEGATIVE && mode != FR_IO_RATING)) {
        fr::set_error("fr_io_open: bad argument");
        return FR_EINVAL;
    }
    *out = nullptr;
    auto io_fail = [&](int e) {
        fr::set_error(std::string(path) + ": " + std::strerror(e));
        return FR_EIO;
    };
    int fd = ::open(path, O_RDONLY);
    if (fd < 0) return io_fail(errno);
    struct stat st;
    if (::fstat(fd, &st) != 0) { int e = errno; ::close(fd); return io_fail(e); }
    auto* t = new fr_io_table();
    t->mode = mode;
    t->size = int64_t(st.st_size);
    if (t->size > 0) {
        void* m = ::mmap(nullptr, size_t(t->size), PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) { int e = errno; ::close(fd); delete t; return io_fail(e); }
        ::madvise(m, size_t(t->size), MADV_SEQUENTIAL);
        t->data = static_cast<const char*>(m);
    }
    ::close(fd);
    int n = pick_threads(threads, t->size);
    // cut points at line starts
    std::vector<int64_t> cut(size_t(n) + 1, t->size);
    cut[0] = 0;
    for (int k = 1; k < n; ++k) {
        int64_t c = t->size * k / n;
        c = std::max(c, cut[size_t(k) - 1]);
        if (c > 0 && c < t->size) {
            const char* le = line_end(t->data + c - 1, t->data + t->size);  // line containing byte c-1
            c = (le - t->data) + 1;
        }
        cut[size_t(k)] = std::min(c, t->size);
    }
    for (int k = 0; k < n; ++k) {
        Range r;
        r.begin = cut[size_t(k)];
        r.end = cut[size_t(k) + 1];
        t->ranges.push_back(r);
    }
    run_threads(n, [t](int k) { count_range(*t, t->ranges[size_t(k)]); });
    for (auto& r : t->ranges) {
        r.row0 = t->rows;
        r.val0 = t->values;
        t->rows += r.rows;
        t->values += r.fields;
    }
    *rows = t->rows;
    *values = t->values;
    *out = t;
    return FR_OK;
}

int fr_io_fill(fr_io_table* t, int64_t* values, int64_t* offsets, double* aux, int64_t* bad_line) {
    if (!t || (t->values > 0 && !values) || (t->mode == FR_IO_NEGATIVE && !offsets)) {
        fr::set_error("fr_io_fill: bad argument");
        return FR_EINVAL;
    }
    if (bad_line) *bad_line = 0;
    int n = int(t->ranges.size());
    run_threads(n, [&](int k) { fill_range(*t, t->ranges[size_t(k)], values, offsets, aux); });
    if (t->mode == FR_IO_NEGATIVE) offsets[t->rows] = t->values;
    for (auto& r : t->ranges) {
        if (r.bad_line >= 0) {
            int64_t line = r.row0 + r.bad_line + 1;  // 1-based
            if (bad_line) *bad_line = line;
            fr::set_error("line " + std::to_string(line) + ": " + r.msg);
            return FR_EPARSE;
        }
    }
    return FR_OK;
}

void fr_io_close(fr_io_table* t) {
    if (!t) return;
    if (t->data) ::munmap(const_cast<char*>(t->data), size_t(t->size));
    delete t;
}

int fr_io_remove_positives(const int64_t* neg, const int64_t* neg_off, uint8_t* alive, const int64_t* pos,
                           const int64_t* pos_off, int64_t n_users, int64_t* lens, int64_t* total, int threads) {
    if (n_users < 0 || !neg_off || !pos_off || !lens || !total || (n_users > 0 && (!alive || !neg || !pos))) {
        fr::set_error("fr_io_remove_positives: bad argument");
        return FR_EINVAL;
    }
    int n = user_threads(threads, n_users);
    run_threads(n, [&](int k) {
        int64_t u0 = n_users * k / n, u1 = n_users * (k + 1) / n;
        for (int64_t u = u0; u < u1; ++u) {
            int64_t nb = neg_off[u], ne = neg_off[u + 1];
            for (int64_t j = pos_off[u]; j < pos_off[u + 1]; ++j) {
                int64_t p = pos[j];
                for (int64_t q = nb; q < ne; ++q) {
                    if (alive[q] && neg[q] == p) { alive[q] = 0; break; }
                }
            }
            int64_t c = 0;
            for (int64_t q = nb; q < ne; ++q) c += alive[q];
            lens[u] = (pos_off[u + 1] - pos_off[u]) + c;
        }
    });
    int64_t sum = 0;
    for (int64_t u = 0; u < n_users; ++u) sum += lens[u];
    *total = sum;
    return FR_OK;
}

int fr_io_candidates(const int64_t* neg, const int64_t* neg_off, const uint8_t* alive, const int64_t* pos,
                      const int64_t* pos_off, const int64_t* users, int64_t n_users, const int64_t* cand_off,
                      int64_t* out_users, int64_t* out_items, int threads) {
    if (n_users < 0 || !neg_off || !pos_off || !cand_off || !users || (n_users > 0 && (!alive || !out_users || !out_items))) {
        fr::set_error("fr_io_candidates: bad argument");
        return FR_EINVAL;
    }
    int n = user_threads(threads, n_users);
    run_threads(n, [&](int k) {
        int64_t u0 = n_users * k / n, u1 = n_users * (k + 1) / n;
        for (int64_t u = u0; u < u1; ++u) {
            int64_t o = cand_off[u];
            for (int64_t j = pos_off[u]; j < pos_off[u + 1]; ++j) out_items[o++] = pos[j];
            for (int64_t q = neg_off[u]; q < neg_off[u + 1]; ++q)
                if (alive[q]) out_items[o++] = neg[q];
            for (int64_t x = cand_off[u]; x < o; ++x) out_users[x] = users[u];
        }
    });
    return FR_OK;
}

}  // extern "C"
