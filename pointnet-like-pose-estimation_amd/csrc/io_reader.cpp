// io_reader.cpp -- libpn2io.so: the dataset text reader (include/pn2io.h), host C++17.
//
// Replaces the per-item np.loadtxt(path, delimiter=",") of
// /root/reference/data_utils/ModelDataLoader.py:85-90 (the files data_build/*.py write with
// np.savetxt(fmt='%6f', delimiter=",")).  A file is read whole (one read() into a buffer),
// split into lines and fields in place, and every field converted correctly rounded, like
// numpy's PyOS_string_to_double, so the doubles are bit-identical to np.loadtxt's: plain
// decimals of <= 15 significant digits (all of '%6f') by Clinger's exact fast path, everything
// else by std::from_chars.  pn2io_read_many_f64 parses a batch of files on a small thread pool (one file
// per task, atomic work counter); nothing is shared between files but the output array.
#include "pn2io.h"

#include <atomic>
#include <cstdint>
#include <cerrno>
#include <charconv>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

namespace {

thread_local char g_err[512];

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int read_file(const char *path, std::string &buf) {
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return fail(PN2IO_EIO, "%s: %s", path, strerror(errno));
    struct stat st;
    if (fstat(fd, &st) != 0) {
        ::close(fd);
        return fail(PN2IO_EIO, "%s: %s", path, strerror(errno));
    }
    buf.resize((size_t)st.st_size);
    size_t got = 0;
    while (got < buf.size()) {
        const ssize_t r = ::read(fd, &buf[got], buf.size() - got);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
            ::close(fd);
            return fail(PN2IO_EIO, "%s: short read", path);
        }
        got += (size_t)r;
    }
    ::close(fd);
    return PN2IO_OK;
}

inline bool blank(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\f' || c == '\v'; }

// Exact powers of ten (every 10^k, k <= 22, is a double).
constexpr double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                               1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Clinger's fast path for plain decimals ("-0.123456", what np.savetxt(fmt='%6f') writes): with
// at most 15 significant digits the digit string m is an exact double, and so is 10^k for
// k <= 22, so m / 10^k (or m * 10^k) is ONE correctly rounded operation -- the same double a
// correctly rounded parser returns.  Anything else (exponents, more digits, inf/nan) -> false.
inline bool fast_decimal(const char *b, const char *e, double &v) {
    bool neg = false;
    if (b < e && (*b == '-' || *b == '+')) neg = *b++ == '-';
    uint64_t m = 0;
    int digits = 0, frac = 0;
    bool any = false, dot = false;
    for (; b < e; ++b) {
        const char c = *b;
        if (c >= '0' && c <= '9') {
            any = true;
            if (m == 0 && c == '0') {  // leading zeros are not significant
                if (dot) ++frac;
                continue;
            }
            if (++digits > 15) return false;
            m = m * 10 + (uint64_t)(c - '0');
            if (dot) ++frac;
        } else if (c == '.' && !dot) {
            dot = true;
        } else {
            return false;
        }
    }
    if (!any || frac > 22) return false;
    const double x = (double)m / kPow10[frac];
    v = neg ? -x : x;
    return true;
}

// One field [b, e) -> double, as float(field.strip()) in numpy's loadtxt converter.
bool parse_field(const char *b, const char *e, double &v) {
    while (b < e && blank(*b)) ++b;
    while (e > b && blank(e[-1])) --e;
    if (fast_decimal(b, e, v)) return true;
    if (b < e && *b == '+') {
        ++b;
        if (b < e && (*b == '+' || *b == '-')) return false;  // float("+-1") is an error
    }
    if (b == e) return false;
    auto r = std::from_chars(b, e, v, std::chars_format::general);
    if (r.ec == std::errc::result_out_of_range) {
        // from_chars reports overflow / underflow instead of rounding to inf / 0 (or a
        // subnormal); strtod rounds as Python does
        std::string s(b, e);
        char *end = nullptr;
        v = strtod(s.c_str(), &end);
        return end == s.c_str() + s.size();
    }
    return r.ec == std::errc() && r.ptr == e;
}

// Parse the rows of buf.  out may be null (shape only).  cols < 0: take the first row's count.
int parse(const char *path, const std::string &buf, char delim, int64_t &cols, int64_t max_rows,
          double *out, int64_t &rows) {
    rows = 0;
    const char *p = buf.data(), *end = p + buf.size();
    int64_t line = 0;
    while (p < end) {
        const char *eol = static_cast<const char *>(memchr(p, '\n', (size_t)(end - p)));
        if (!eol) eol = end;
        ++line;
        const char *lend = eol;
        const char *hash = static_cast<const char *>(memchr(p, '#', (size_t)(lend - p)));
        if (hash) lend = hash;
        const char *q = p;
        while (q < lend && blank(*q)) ++q;
        if (q < lend) {  // a data row
            if (out && rows >= max_rows)
                return fail(PN2IO_ESIZE, "%s: more than %lld rows", path, (long long)max_rows);
            int64_t c = 0;
            const char *f = p;
            while (true) {
                const char *d = static_cast<const char *>(memchr(f, delim, (size_t)(lend - f)));
                const char *fe = d ? d : lend;
                double v = 0.0;
                if (out && !parse_field(f, fe, v))  // the shape pass (out == null) only counts
                    return fail(PN2IO_EPARSE, "%s:%lld: could not convert '%.*s' to float", path,
                                (long long)line, (int)(fe - f), f);
                if (cols >= 0 && c >= cols)
                    return fail(PN2IO_EPARSE, "%s:%lld: more than %lld columns", path,
                                (long long)line, (long long)cols);
                if (out) out[rows * cols + c] = v;
                ++c;
                if (!d) break;
                f = d + 1;
            }
            if (cols < 0) cols = c;
            if (c != cols)
                return fail(PN2IO_EPARSE, "%s:%lld: %lld columns, expected %lld", path,
                            (long long)line, (long long)c, (long long)cols);
            ++rows;
        }
        p = eol + 1;
    }
    return PN2IO_OK;
}

}  // namespace

extern "C" {

int pn2io_abi_version(void) { return PN2IO_ABI_VERSION; }
const char *pn2io_last_error(void) { return g_err; }

int pn2io_shape(const char *path, char delim, int64_t *rows, int64_t *cols) {
    if (!path || !rows || !cols) return fail(PN2IO_EINVAL, "pn2io_shape: null pointer");
    std::string buf;
    int rc = read_file(path, buf);
    if (rc) return rc;
    int64_t c = -1, r = 0;
    rc = parse(path, buf, delim, c, 0, nullptr, r);
    if (rc) return rc;
    *rows = r;
    *cols = c < 0 ? 0 : c;
    return PN2IO_OK;
}

int pn2io_read_csv_f64(const char *path, char delim, int64_t cols, int64_t max_rows, double *out,
                       int64_t *rows_out) {
    if (!path || !out || !rows_out || cols <= 0 || max_rows < 0)
        return fail(PN2IO_EINVAL, "pn2io_read_csv_f64: bad argument");
    std::string buf;
    int rc = read_file(path, buf);
    if (rc) return rc;
    int64_t c = cols, r = 0;
    rc = parse(path, buf, delim, c, max_rows, out, r);
    *rows_out = r;
    return rc;
}

int pn2io_read_many_f64(const char *const *paths, int64_t n, char delim, int64_t cols,
                        int64_t max_rows, double *out, int64_t *rows_out, int threads) {
    if (n < 0 || (n > 0 && (!paths || !out || !rows_out)) || cols <= 0 || max_rows < 0)
        return fail(PN2IO_EINVAL, "pn2io_read_many_f64: bad argument");
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    if (threads < 1) threads = 1;
    if ((int64_t)threads > n) threads = (int)n;
    std::vector<int> codes((size_t)n, PN2IO_OK);
    std::vector<std::string> msgs((size_t)n);
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        std::string buf;
        for (int64_t i; (i = next.fetch_add(1)) < n;) {
            int64_t r = 0;
            int rc = paths[i] ? read_file(paths[i], buf) : fail(PN2IO_EINVAL, "null path %lld", (long long)i);
            if (rc == PN2IO_OK) {
                int64_t c = cols;
                rc = parse(paths[i], buf, delim, c, max_rows, out + i * max_rows * cols, r);
            }
            rows_out[i] = r;
            codes[(size_t)i] = rc;
            if (rc) msgs[(size_t)i] = g_err;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
    for (int64_t i = 0; i < n; ++i)
        if (codes[(size_t)i]) return fail(codes[(size_t)i], "%s", msgs[(size_t)i].c_str());
    return PN2IO_OK;
}

}  // extern "C"
