// PLINK .fam/.bim metadata parsing.
//
// The reference parses .fam (fid iid father mother sex pheno) and .bim (chrom sid cm bp a1 a2)
// in bed-reader's Python metadata layer (reached from snpreader/bed.py:137-194); at UK-Biobank
// shape (500k .fam lines, 1M .bim lines) that text parsing dominates Bed() open time.  Here the
// file is mmapped, cut at line boundaries into one range per thread, and each thread
// tokenises its lines on whitespace.  Strings come out as fixed-width NUL-padded byte rows
// (NumPy 'S<width>' arrays, no per-string Python objects); numbers are parsed to f64.
// Host-only code (no device work): it is the I/O side of the path, not a kernel.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <thread>
#include <vector>

#include "snpmi_internal.hpp"

namespace snpmi {
namespace {

struct TextMap {
    int fd = -1;
    const char* p = nullptr;
    size_t size = 0;
    ~TextMap() {
        if (p && size) munmap((void*)p, size);
        if (fd >= 0) close(fd);
    }
};

void open_text(TextMap& t, const char* path) {
    SNPMI_REQUIRE(path != nullptr, SNPMI_E_ARG, "path is NULL");
    t.fd = open(path, O_RDONLY);
    SNPMI_REQUIRE(t.fd >= 0, SNPMI_E_IO, std::string("cannot open ") + path);
    struct stat st;
    SNPMI_REQUIRE(fstat(t.fd, &st) == 0, SNPMI_E_IO, std::string("cannot stat ") + path);
    t.size = (size_t)st.st_size;
    if (t.size == 0) return;
    void* m = mmap(nullptr, t.size, PROT_READ, MAP_PRIVATE, t.fd, 0);
    SNPMI_REQUIRE(m != MAP_FAILED, SNPMI_E_IO, std::string("mmap failed: ") + path);
    t.p = (const char*)m;
    (void)madvise(m, t.size, MADV_SEQUENTIAL);
}

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// [begin, end) byte ranges, one per thread, each starting at a line start
std::vector<std::pair<size_t, size_t>> split_lines(const TextMap& t, int threads) {
    std::vector<std::pair<size_t, size_t>> r;
    const size_t per = std::max<size_t>(t.size / std::max(threads, 1), 1 << 16);
    size_t b = 0;
    while (b < t.size) {
        size_t e = std::min(t.size, b + per);
        while (e < t.size && t.p[e - 1] != '\n') e++;
        r.emplace_back(b, e);
        b = e;
    }
    return r;
}

// Visit every non-blank line of [b, e): fn(fields_begin[], fields_len[], n_fields, line_no_in_range)
template <class F>
void for_lines(const char* p, size_t b, size_t e, int max_fields, F&& fn) {
    const char* fb[16];
    uint32_t fl[16];
    size_t i = b;
    uint64_t row = 0;
    while (i < e) {
        int nf = 0;
        while (i < e && p[i] != '\n') {
            while (i < e && is_space(p[i])) i++;
            if (i >= e || p[i] == '\n') break;
            const size_t s = i;
            while (i < e && p[i] != '\n' && !is_space(p[i])) i++;
            if (nf < max_fields) {
                fb[nf] = p + s;
                fl[nf] = (uint32_t)(i - s);
            }
            nf++;
        }
        if (i < e) i++;  // '\n'
        if (nf == 0) continue;  // blank line
        fn(fb, fl, nf, row);
        row++;
    }
}

int n_threads(int num_threads) {
    if (num_threads > 0) return std::min(num_threads, 64);
    return (int)std::max(1u, std::min(std::thread::hardware_concurrency(), 16u));
}

template <class F>
void run_ranges(const std::vector<std::pair<size_t, size_t>>& ranges, F&& fn) {
    std::vector<std::thread> th;
    std::vector<std::string> errs(ranges.size());
    std::vector<int> codes(ranges.size(), 0);
    for (size_t k = 0; k < ranges.size(); k++)
        th.emplace_back([&, k] {
            try {
                fn(k);
            } catch (const Error& e) {
                codes[k] = e.code;
                errs[k] = e.what();
            } catch (const std::exception& e) {
                codes[k] = SNPMI_E_ARG;
                errs[k] = e.what();
            }
        });
    for (auto& t : th) t.join();
    for (size_t k = 0; k < ranges.size(); k++)
        if (codes[k]) throw Error(codes[k], errs[k]);
}

struct Scan {
    std::vector<std::pair<size_t, size_t>> ranges;
    std::vector<uint64_t> row0;  // first row of each range
    uint64_t rows = 0;
};

// Count rows per range (and the widest field per column), checking the field count.
Scan scan(const TextMap& t, int min_fields, int n_cols, uint64_t* widths, int threads, const char* path) {
    Scan s;
    if (t.size == 0) return s;
    s.ranges = split_lines(t, threads);
    const size_t R = s.ranges.size();
    std::vector<uint64_t> cnt(R, 0);
    std::vector<std::vector<uint64_t>> w(R, std::vector<uint64_t>(std::max(n_cols, 1), 0));
    run_ranges(s.ranges, [&](size_t k) {
        for_lines(t.p, s.ranges[k].first, s.ranges[k].second, 16,
                  [&](const char* const*, const uint32_t* fl, int nf, uint64_t) {
                      if (nf < min_fields)
                          throw Error(SNPMI_E_FORMAT, std::string("expected at least ") + std::to_string(min_fields) +
                                                          " fields per line in " + path);
                      for (int c = 0; c < n_cols && c < 16; c++) w[k][c] = std::max<uint64_t>(w[k][c], fl[c]);
                      cnt[k]++;
                  });
    });
    s.row0.resize(R);
    for (size_t k = 0; k < R; k++) {
        s.row0[k] = s.rows;
        s.rows += cnt[k];
        for (int c = 0; c < n_cols; c++) widths[c] = std::max(widths[c], w[k][c]);
    }
    return s;
}

}  // namespace
}  // namespace snpmi

using namespace snpmi;

extern "C" {

int snpmi_text_scan(const char* path, int min_fields, int n_cols, uint64_t* n_rows, uint64_t* widths,
                    int num_threads) {
    return guarded([&] {
        SNPMI_REQUIRE(n_rows != nullptr && n_cols >= 0 && n_cols <= 16 && (n_cols == 0 || widths != nullptr),
                      SNPMI_E_ARG, "bad text_scan arguments");
        for (int c = 0; c < n_cols; c++) widths[c] = 0;
        TextMap t;
        open_text(t, path);
        Scan s = scan(t, min_fields, n_cols, widths, n_threads(num_threads), path);
        *n_rows = s.rows;
    });
}

int snpmi_text_strings(const char* path, int col, uint64_t n_rows, uint64_t width, char* out, int num_threads) {
    return guarded([&] {
        SNPMI_REQUIRE(col >= 0 && col < 16 && (out != nullptr || n_rows == 0), SNPMI_E_ARG, "bad text_strings arguments");
        TextMap t;
        open_text(t, path);
        uint64_t wdummy[16] = {};
        Scan s = scan(t, col + 1, 0, wdummy, n_threads(num_threads), path);
        SNPMI_REQUIRE(s.rows == n_rows, SNPMI_E_FORMAT, std::string("line count changed while reading ") + path);
        run_ranges(s.ranges, [&](size_t k) {
            for_lines(t.p, s.ranges[k].first, s.ranges[k].second, col + 1,
                      [&](const char* const* fb, const uint32_t* fl, int, uint64_t r) {
                          char* dst = out + (s.row0[k] + r) * width;
                          const uint64_t len = std::min<uint64_t>(fl[col], width);
                          std::memcpy(dst, fb[col], len);
                          if (len < width) std::memset(dst + len, 0, width - len);
                      });
        });
    });
}

int snpmi_text_f64(const char* path, int col, uint64_t n_rows, double* out, int num_threads) {
    return guarded([&] {
        SNPMI_REQUIRE(col >= 0 && col < 16 && (out != nullptr || n_rows == 0), SNPMI_E_ARG, "bad text_f64 arguments");
        TextMap t;
        open_text(t, path);
        uint64_t wdummy[16] = {};
        Scan s = scan(t, col + 1, 0, wdummy, n_threads(num_threads), path);
        SNPMI_REQUIRE(s.rows == n_rows, SNPMI_E_FORMAT, std::string("line count changed while reading ") + path);
        run_ranges(s.ranges, [&](size_t k) {
            char buf[64];
            for_lines(t.p, s.ranges[k].first, s.ranges[k].second, col + 1,
                      [&](const char* const* fb, const uint32_t* fl, int, uint64_t r) {
                          const uint32_t len = fl[col];
                          if (len >= sizeof(buf))
                              throw Error(SNPMI_E_FORMAT, std::string("could not convert field to float in ") + path);
                          std::memcpy(buf, fb[col], len);
                          buf[len] = 0;
                          char* end = nullptr;
                          const double v = std::strtod(buf, &end);
                          if (end != buf + len)
                              throw Error(SNPMI_E_FORMAT, std::string("could not convert string to float: '") + buf +
                                                              "' in " + path);
                          out[s.row0[k] + r] = v;
                      });
        });
    });
}

}  // extern "C"
