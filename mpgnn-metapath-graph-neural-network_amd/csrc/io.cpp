// link.dat reader: `node_1 \t relation \t node_2` rows → the graph
// tensors the layers consume, laid out as get_edge_index_and_type_no_reverse builds them
// (main.py:366-372 ≡ main_rgcn.py:357-363: edge_index row 0 = node_1, row 1 = node_2,
// edge_type = relation, file order kept). The reference goes through pandas.read_csv
// (main.py:150-151) and Python lists; here the file is memory-mapped and parsed by a pool of
// threads over newline-aligned byte ranges (count pass, prefix sum, fill pass).
// node.dat / label.dat (main.py:140-147: `id \t value …` rows through pandas.read_csv) go
// through the same machinery as a numeric matrix (mpgnn_tsv_shape / mpgnn_tsv_parse_f64).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <charconv>
#include <cmath>
#include <limits>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mpgnn_rgcn.h"
#include "plan_internal.h"

namespace {

struct Mapped {
    const char* p = nullptr;
    size_t n = 0;
    int fd = -1;
    ~Mapped() {
        if (p && n) munmap(const_cast<char*>(p), n);
        if (fd >= 0) close(fd);
    }
};

int32_t map_file(const char* path, Mapped& m) {
    if (!path) {
        mpgnn::set_last_error("link file path is null");
        return MPGNN_ERR_ARG;
    }
    m.fd = open(path, O_RDONLY);
    if (m.fd < 0) {
        mpgnn::set_last_error(std::string("cannot open ") + path + ": " + strerror(errno));
        return MPGNN_ERR_ARG;
    }
    struct stat st;
    if (fstat(m.fd, &st) != 0) {
        mpgnn::set_last_error(std::string("cannot stat ") + path);
        return MPGNN_ERR_ARG;
    }
    m.n = (size_t)st.st_size;
    if (m.n == 0) return MPGNN_OK;
    void* p = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, m.fd, 0);
    if (p == MAP_FAILED) {
        mpgnn::set_last_error(std::string("cannot map ") + path);
        m.n = 0;
        return MPGNN_ERR_ALLOC;
    }
    madvise(p, m.n, MADV_SEQUENTIAL);
    m.p = (const char*)p;
    return MPGNN_OK;
}

inline bool is_blank(char c) { return c == ' ' || c == '\t' || c == '\r'; }

// A line holds a row when it has a non-blank character.
inline bool line_has_data(const char* b, const char* e) {
    for (; b < e; ++b)
        if (!is_blank(*b)) return true;
    return false;
}

// Byte ranges [cut[t], cut[t+1]) that start at a line start.
std::vector<size_t> split_lines(const Mapped& m, int parts) {
    std::vector<size_t> cut(parts + 1, m.n);
    cut[0] = 0;
    for (int t = 1; t < parts; ++t) {
        size_t pos = std::max(cut[t - 1], m.n * (size_t)t / (size_t)parts);
        if (pos > 0 && pos < m.n && m.p[pos - 1] != '\n') {
            const void* nl = memchr(m.p + pos, '\n', m.n - pos);
            pos = nl ? (size_t)((const char*)nl - m.p) + 1 : m.n;
        }
        cut[t] = pos;
    }
    return cut;
}

int64_t count_rows(const char* b, const char* e) {
    int64_t rows = 0;
    while (b < e) {
        const char* nl = (const char*)memchr(b, '\n', (size_t)(e - b));
        const char* le = nl ? nl : e;
        rows += line_has_data(b, le) ? 1 : 0;
        b = le + 1;
    }
    return rows;
}

inline bool parse_int(const char*& s, const char* e, int64_t& v) {
    while (s < e && is_blank(*s)) ++s;
    bool neg = false;
    if (s < e && (*s == '-' || *s == '+')) neg = (*s++ == '-');
    if (s >= e || *s < '0' || *s > '9') return false;
    uint64_t acc = 0;
    while (s < e && *s >= '0' && *s <= '9') acc = acc * 10 + (uint64_t)(*s++ - '0');
    // integral floats as pandas would read them ("3.0"): accept a zero fraction only
    if (s < e && *s == '.') {
        ++s;
        while (s < e && *s == '0') ++s;
        if (s < e && *s >= '1' && *s <= '9') return false;
    }
    if (s < e && !is_blank(*s)) return false;
    v = neg ? -(int64_t)acc : (int64_t)acc;
    return true;
}

// One numeric field (integer or decimal / exponent float, as pandas' C reader accepts them;
// also "nan"/"inf" through from_chars). Advances s past the field.
inline bool parse_double(const char*& s, const char* e, double& v) {
    while (s < e && is_blank(*s)) ++s;
    if (s >= e) return false;
    const char* b = s;
    if (*b == '+') ++b;  // from_chars rejects a leading '+'
    auto r = std::from_chars(b, e, v, std::chars_format::general);
    if (r.ec != std::errc() || r.ptr == b) return false;
    s = r.ptr;
    return s >= e || is_blank(*s);
}

// node.dat / label.dat fields as pandas.read_csv(sep='\t') cuts them: on every single '\t' (a
// trailing '\r' dropped), so an empty field ('1\t\t3', a trailing tab) is a field of its own
// (NaN) and a space never separates fields. 0 for a blank line.
inline const char* strip_cr(const char* b, const char* e) { return (e > b && e[-1] == '\r') ? e - 1 : e; }

inline int64_t count_fields(const char* b, const char* e) {
    if (!line_has_data(b, e)) return 0;
    e = strip_cr(b, e);
    int64_t n = 1;
    for (; b < e; ++b) n += *b == '\t';
    return n;
}

// One tab-separated field [b, e): surrounding spaces ignored (pandas' float parser skips them),
// empty -> NaN, otherwise it must be one number.
inline bool parse_field(const char* b, const char* e, double& v) {
    while (b < e && (*b == ' ' || *b == '\r')) ++b;
    while (e > b && (e[-1] == ' ' || e[-1] == '\r')) --e;
    if (b == e) {
        v = std::numeric_limits<double>::quiet_NaN();
        return true;
    }
    const char* s = b;
    return parse_double(s, e, v) && s == e;
}

int parse_threads(size_t bytes) {
    unsigned hw = std::thread::hardware_concurrency();
    int t = (int)std::min<size_t>(hw ? std::min(hw, 16u) : 1u, bytes / (1u << 20) + 1);
    return std::max(1, t);
}

}  // namespace

extern "C" {

int32_t mpgnn_links_count(const char* path, int64_t* rows) {
    if (!rows) {
        mpgnn::set_last_error("mpgnn_links_count: rows is null");
        return MPGNN_ERR_ARG;
    }
    Mapped m;
    int32_t st = map_file(path, m);
    if (st != MPGNN_OK) return st;
    const int parts = parse_threads(m.n);
    std::vector<size_t> cut = split_lines(m, parts);
    std::vector<int64_t> cnt(parts, 0);
    std::vector<std::thread> pool;
    for (int t = 0; t < parts; ++t)
        pool.emplace_back([&, t] { cnt[t] = count_rows(m.p + cut[t], m.p + cut[t + 1]); });
    for (auto& th : pool) th.join();
    int64_t total = 0;
    for (int64_t c : cnt) total += c;
    *rows = total;
    return MPGNN_OK;
}

int32_t mpgnn_links_parse(const char* path, int64_t* edge_index, int64_t* edge_type, int64_t rows) {
    if (rows < 0 || (rows > 0 && (!edge_index || !edge_type))) {
        mpgnn::set_last_error("mpgnn_links_parse: null output or negative row count");
        return MPGNN_ERR_ARG;
    }
    Mapped m;
    int32_t st = map_file(path, m);
    if (st != MPGNN_OK) return st;
    const int parts = parse_threads(m.n);
    std::vector<size_t> cut = split_lines(m, parts);
    std::vector<int64_t> cnt(parts, 0), first(parts + 1, 0);
    {
        std::vector<std::thread> pool;
        for (int t = 0; t < parts; ++t)
            pool.emplace_back([&, t] { cnt[t] = count_rows(m.p + cut[t], m.p + cut[t + 1]); });
        for (auto& th : pool) th.join();
    }
    for (int t = 0; t < parts; ++t) first[t + 1] = first[t] + cnt[t];
    if (first[parts] != rows) {
        mpgnn::set_last_error("mpgnn_links_parse: file has " + std::to_string(first[parts]) +
                              " rows, caller passed " + std::to_string(rows));
        return MPGNN_ERR_ARG;
    }
    std::vector<int64_t> bad(parts, -1);  // row index of the first malformed row per part
    std::vector<std::thread> pool;
    for (int t = 0; t < parts; ++t)
        pool.emplace_back([&, t] {
            const char* b = m.p + cut[t];
            const char* e = m.p + cut[t + 1];
            int64_t r = first[t];
            while (b < e) {
                const char* nl = (const char*)memchr(b, '\n', (size_t)(e - b));
                const char* le = nl ? nl : e;
                if (line_has_data(b, le)) {
                    const char* s = b;
                    int64_t n1, rel, n2;
                    bool ok = parse_int(s, le, n1) && parse_int(s, le, rel) && parse_int(s, le, n2);
                    if (ok) {
                        while (s < le && is_blank(*s)) ++s;
                        ok = s == le;  // exactly three columns
                    }
                    if (!ok) {
                        bad[t] = r;
                        return;
                    }
                    edge_index[r] = n1;
                    edge_index[rows + r] = n2;
                    edge_type[r] = rel;
                    ++r;
                }
                b = le + 1;
            }
        });
    for (auto& th : pool) th.join();
    for (int t = 0; t < parts; ++t)
        if (bad[t] >= 0) {
            mpgnn::set_last_error("mpgnn_links_parse: row " + std::to_string(bad[t]) +
                                  " is not three integer columns (node_1, relation, node_2)");
            return MPGNN_ERR_ARG;
        }
    return MPGNN_OK;
}

int32_t mpgnn_tsv_shape(const char* path, int64_t* rows, int64_t* cols) {
    if (!rows || !cols) {
        mpgnn::set_last_error("mpgnn_tsv_shape: rows / cols is null");
        return MPGNN_ERR_ARG;
    }
    Mapped m;
    int32_t st = map_file(path, m);
    if (st != MPGNN_OK) return st;
    const int parts = parse_threads(m.n);
    std::vector<size_t> cut = split_lines(m, parts);
    std::vector<int64_t> cnt(parts, 0), width(parts, 0);
    std::vector<std::thread> pool;
    for (int t = 0; t < parts; ++t)
        pool.emplace_back([&, t] {
            const char* b = m.p + cut[t];
            const char* e = m.p + cut[t + 1];
            while (b < e) {
                const char* nl = (const char*)memchr(b, '\n', (size_t)(e - b));
                const char* le = nl ? nl : e;
                int64_t f = count_fields(b, le);
                if (f > 0) {
                    ++cnt[t];
                    width[t] = std::max(width[t], f);
                }
                b = le + 1;
            }
        });
    for (auto& th : pool) th.join();
    int64_t r = 0, c = 0;
    for (int t = 0; t < parts; ++t) {
        r += cnt[t];
        c = std::max(c, width[t]);
    }
    *rows = r;
    *cols = c;
    return MPGNN_OK;
}

int32_t mpgnn_tsv_parse_f64(const char* path, double* out, int64_t rows, int64_t cols) {
    if (rows < 0 || cols < 0 || (rows > 0 && cols > 0 && !out)) {
        mpgnn::set_last_error("mpgnn_tsv_parse_f64: null output or negative shape");
        return MPGNN_ERR_ARG;
    }
    Mapped m;
    int32_t st = map_file(path, m);
    if (st != MPGNN_OK) return st;
    const int parts = parse_threads(m.n);
    std::vector<size_t> cut = split_lines(m, parts);
    std::vector<int64_t> cnt(parts, 0), first(parts + 1, 0);
    {
        std::vector<std::thread> pool;
        for (int t = 0; t < parts; ++t)
            pool.emplace_back([&, t] { cnt[t] = count_rows(m.p + cut[t], m.p + cut[t + 1]); });
        for (auto& th : pool) th.join();
    }
    for (int t = 0; t < parts; ++t) first[t + 1] = first[t] + cnt[t];
    if (first[parts] != rows) {
        mpgnn::set_last_error("mpgnn_tsv_parse_f64: file has " + std::to_string(first[parts]) +
                              " rows, caller passed " + std::to_string(rows));
        return MPGNN_ERR_ARG;
    }
    const double nan = std::numeric_limits<double>::quiet_NaN();
    std::vector<int64_t> bad(parts, -1);
    std::vector<std::thread> pool;
    for (int t = 0; t < parts; ++t)
        pool.emplace_back([&, t] {
            const char* b = m.p + cut[t];
            const char* e = m.p + cut[t + 1];
            int64_t r = first[t];
            while (b < e) {
                const char* nl = (const char*)memchr(b, '\n', (size_t)(e - b));
                const char* le = nl ? nl : e;
                if (line_has_data(b, le)) {
                    const char* s = b;
                    const char* lend = strip_cr(b, le);
                    double* row = out + r * cols;
                    int64_t c = 0;
                    for (;; ++c) {
                        const char* fe = (const char*)memchr(s, '\t', (size_t)(lend - s));
                        if (!fe) fe = lend;
                        if (c >= cols || !parse_field(s, fe, row[c])) {  // more fields than cols / not a number
                            bad[t] = r;
                            return;
                        }
                        if (fe == lend) break;
                        s = fe + 1;
                    }
                    for (++c; c < cols; ++c) row[c] = nan;  // ragged row: pandas fills NaN
                    ++r;
                }
                b = le + 1;
            }
        });
    for (auto& th : pool) th.join();
    for (int t = 0; t < parts; ++t)
        if (bad[t] >= 0) {
            mpgnn::set_last_error("mpgnn_tsv_parse_f64: row " + std::to_string(bad[t]) +
                                  " has a non-numeric field or more than " + std::to_string(cols) + " fields");
            return MPGNN_ERR_ARG;
        }
    return MPGNN_OK;
}

}  // extern "C"
