// lsmck_formats.cpp -- the on-disk record of src/checksums.rs and small host
// utilities: error reporting, the checksum JSON file, synthetic lengths.
#include <errno.h>
#include <fcntl.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "lsmck.h"
#include "lsmck_internal.h"

namespace lsmck_host {

static thread_local std::string g_err;

int set_error(int rc, const char* msg) {
  g_err = msg ? msg : "";
  return rc;
}

int set_errno_error(int err, const char* what, const char* path) {
  g_err = std::string(what) + " " + (path ? path : "") + ": " + strerror(err);
  return -err;
}

static int write_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t k = write(fd, p, n);
    if (k < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    p += k;
    n -= (size_t)k;
  }
  return 0;
}

// serde_json::to_writer(checksum_file, &Checksums{index_checksum, data_checksum})
// with the file opened .write(true).create(true) -- no truncate (checksums.rs:75-79):
// a shorter JSON written over a longer old file leaves the old tail in place,
// exactly as the reference does.
int write_checksum_json(const char* path, const char* index_b64, const char* data_b64) {
  std::string s = std::string("{\"index_checksum\":\"") + index_b64 + "\",\"data_checksum\":\"" + data_b64 + "\"}";
  int fd = open(path, O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
  if (fd < 0) return set_errno_error(errno, "open", path);
  int rc = write_all(fd, s.data(), s.size());
  close(fd);
  if (rc) return set_errno_error(-rc, "write", path);
  return 0;
}

// Minimal JSON reader for the Checksums object: accepts whitespace, any field
// order, unknown fields (serde ignores them), standard string escapes; both
// fields are required (serde's "missing field" error).  Trailing non-space
// bytes after the object are an error, as serde_json::from_reader reports
// "trailing characters".
namespace {
struct P {
  const char* s;
  size_t n, i;
  void ws() {
    while (i < n && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) ++i;
  }
  bool lit(char c) {
    ws();
    if (i < n && s[i] == c) {
      ++i;
      return true;
    }
    return false;
  }
  bool str(std::string* out) {
    ws();
    if (i >= n || s[i] != '"') return false;
    ++i;
    out->clear();
    while (i < n && s[i] != '"') {
      char c = s[i++];
      if (c == '\\') {
        if (i >= n) return false;
        char e = s[i++];
        switch (e) {
          case '"': out->push_back('"'); break;
          case '\\': out->push_back('\\'); break;
          case '/': out->push_back('/'); break;
          case 'b': out->push_back('\b'); break;
          case 'f': out->push_back('\f'); break;
          case 'n': out->push_back('\n'); break;
          case 'r': out->push_back('\r'); break;
          case 't': out->push_back('\t'); break;
          case 'u': {
            if (i + 4 > n) return false;
            unsigned v = 0;
            for (int k = 0; k < 4; ++k) {
              char h = s[i++];
              v <<= 4;
              if (h >= '0' && h <= '9') v |= (unsigned)(h - '0');
              else if (h >= 'a' && h <= 'f') v |= (unsigned)(h - 'a' + 10);
              else if (h >= 'A' && h <= 'F') v |= (unsigned)(h - 'A' + 10);
              else return false;
            }
            if (v < 0x80) out->push_back((char)v);
            else if (v < 0x800) {
              out->push_back((char)(0xC0 | (v >> 6)));
              out->push_back((char)(0x80 | (v & 63)));
            } else {
              out->push_back((char)(0xE0 | (v >> 12)));
              out->push_back((char)(0x80 | ((v >> 6) & 63)));
              out->push_back((char)(0x80 | (v & 63)));
            }
            break;
          }
          default: return false;
        }
      } else if ((unsigned char)c < 0x20) {
        return false;
      } else {
        out->push_back(c);
      }
    }
    if (i >= n) return false;
    ++i;
    return true;
  }
  bool skip_value() {  // any JSON value (unknown field)
    ws();
    if (i >= n) return false;
    char c = s[i];
    if (c == '"') {
      std::string t;
      return str(&t);
    }
    if (c == '{' || c == '[') {
      char open = c, close = c == '{' ? '}' : ']';
      int depth = 0;
      while (i < n) {
        char d = s[i];
        if (d == '"') {
          std::string t;
          if (!str(&t)) return false;
          continue;
        }
        ++i;
        if (d == open) ++depth;
        else if (d == close && --depth == 0) return true;
      }
      return false;
    }
    size_t st = i;
    while (i < n && s[i] != ',' && s[i] != '}' && s[i] != ']' && s[i] != ' ' && s[i] != '\n' && s[i] != '\t' &&
           s[i] != '\r')
      ++i;
    return i > st;
  }
};
}  // namespace

// Small JSON files (a few hundred bytes): one read(2) normally suffices.  A
// read that returns less than asked is taken as end of file -- what a regular
// file's read does -- which saves the extra read(2) that would return 0: a
// whole-tree verify opens ~230k such files, and the system calls are its cost
// (DESIGN.md 7a).
// open_code != 0: the status when the file cannot be opened (a panic site of
// the reference) instead of -errno
static int read_file(const char* path, std::string* buf, int open_code = 0) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    if (open_code) {
      int e = errno;
      std::string m = std::string("Can't open checksum file ") + path + ": " + strerror(e);
      return set_error(open_code, m.c_str());
    }
    return set_errno_error(errno, "open", path);
  }
  buf->clear();
  char tmp[16384];
  for (;;) {
    ssize_t k = read(fd, tmp, sizeof tmp);
    if (k < 0) {
      if (errno == EINTR) continue;
      int e = errno;
      close(fd);
      return set_errno_error(e, "read", path);
    }
    buf->append(tmp, (size_t)k);
    if ((size_t)k < sizeof tmp) break;
  }
  close(fd);
  return 0;
}

int read_checksum_json(const char* path, std::string* index_b64, std::string* data_b64) {
  std::string buf;
  if (int rc = read_file(path, &buf, LSMCK_PANIC_OPEN_CHECKSUM)) return rc;  // checksums.rs:43-46
  P p{buf.data(), buf.size(), 0};
  bool have_i = false, have_d = false;
  if (!p.lit('{')) return set_error(LSMCK_EJSON, "checksum file: expected '{'");
  if (!p.lit('}')) {
    for (;;) {
      std::string key;
      if (!p.str(&key) || !p.lit(':')) return set_error(LSMCK_EJSON, "checksum file: bad member");
      if (key == "index_checksum") {
        if (have_i) return set_error(LSMCK_EJSON, "checksum file: duplicate field `index_checksum`");
        if (!p.str(index_b64)) return set_error(LSMCK_EJSON, "checksum file: index_checksum not a string");
        have_i = true;
      } else if (key == "data_checksum") {
        if (have_d) return set_error(LSMCK_EJSON, "checksum file: duplicate field `data_checksum`");
        if (!p.str(data_b64)) return set_error(LSMCK_EJSON, "checksum file: data_checksum not a string");
        have_d = true;
      } else if (!p.skip_value()) {
        return set_error(LSMCK_EJSON, "checksum file: bad value");
      }
      if (p.lit(',')) continue;
      if (p.lit('}')) break;
      return set_error(LSMCK_EJSON, "checksum file: expected ',' or '}'");
    }
  }
  p.ws();
  if (p.i != p.n) return set_error(LSMCK_EJSON, "checksum file: trailing characters");
  if (!have_i) return set_error(LSMCK_EJSON, "checksum file: missing field `index_checksum`");
  if (!have_d) return set_error(LSMCK_EJSON, "checksum file: missing field `data_checksum`");
  return 0;
}

static uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void gen_zipf_lengths(uint64_t seed, double s, int kmax, uint32_t lmin, uint64_t first, size_t n, uint32_t* out) {
  std::vector<double> cdf((size_t)kmax);
  double tot = 0.0;
  for (int k = 1; k <= kmax; ++k) tot += pow((double)k, -s);
  double acc = 0.0;
  for (int k = 1; k <= kmax; ++k) {
    acc += pow((double)k, -s);
    cdf[(size_t)k - 1] = acc / tot;
  }
  cdf[(size_t)kmax - 1] = 1.0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t r = first + i;  // counter-based: record r's length depends on (seed, r) alone
    uint64_t u1 = splitmix64(seed ^ (2 * r));
    uint64_t u2 = splitmix64(seed ^ (2 * r + 1));
    double u = (double)(u1 >> 11) * 0x1.0p-53;
    int lo = 0, hi = kmax - 1;
    while (lo < hi) {
      int mid = (lo + hi) / 2;
      if (u < cdf[(size_t)mid]) hi = mid;
      else lo = mid + 1;
    }
    int64_t L = 64 * (int64_t)(lo + 1) - (int64_t)(u2 & 63);
    out[i] = L < (int64_t)lmin ? lmin : (uint32_t)L;
  }
}

// serde_json::from_reader::<SsTableMetadata> (sstable_metadata.rs:7-17, 76-83):
// all eight fields required, unknown fields ignored, duplicates rejected; `id`
// must be a JSON integer that fits u128 and `level` one that fits u8 (serde's
// invalid-type / out-of-range errors otherwise).
static bool parse_uint(P& p, unsigned digits_max, const char* max_dec) {
  p.ws();
  size_t st = p.i;
  while (p.i < p.n && p.s[p.i] >= '0' && p.s[p.i] <= '9') ++p.i;
  size_t nd = p.i - st;
  if (nd == 0 || (nd > 1 && p.s[st] == '0')) return false;
  if (p.i < p.n && (p.s[p.i] == '.' || p.s[p.i] == 'e' || p.s[p.i] == 'E')) return false;
  if (nd > digits_max) return false;
  if (nd == digits_max && memcmp(p.s + st, max_dec, nd) > 0) return false;
  return true;
}

int read_metadata_json(const char* path, TableMeta* m) {
  std::string buf;
  if (int rc = read_file(path, &buf)) return rc;
  P p{buf.data(), buf.size(), 0};
  static const char* const kNames[8] = {"base_path",     "id",             "level",          "metadata_filename",
                                        "checksum_filename", "data_filename", "index_filename", "bloom_filter_filename"};
  std::string* strs[8] = {&m->base_path, nullptr, nullptr, &m->metadata_filename, &m->checksum_filename,
                          &m->data_filename, &m->index_filename, &m->bloom_filter_filename};
  bool have[8] = {};
  if (!p.lit('{')) return set_error(LSMCK_EJSON, "metadata file: expected '{'");
  if (!p.lit('}')) {
    for (;;) {
      std::string key;
      if (!p.str(&key) || !p.lit(':')) return set_error(LSMCK_EJSON, "metadata file: bad member");
      int f = -1;
      for (int k = 0; k < 8; ++k)
        if (key == kNames[k]) f = k;
      if (f >= 0 && have[f]) return set_error(LSMCK_EJSON, "metadata file: duplicate field");
      if (f == 1) {
        p.ws();
        const size_t st = p.i;
        if (!parse_uint(p, 39, "340282366920938463463374607431768211455"))
          return set_error(LSMCK_EJSON, "metadata file: id is not a u128");
        m->id.assign(p.s + st, p.i - st);
      } else if (f == 2) {
        p.ws();
        size_t st = p.i;
        if (!parse_uint(p, 3, "255")) return set_error(LSMCK_EJSON, "metadata file: level is not a u8");
        m->level = (unsigned)atoi(std::string(p.s + st, p.i - st).c_str());
      } else if (f >= 0) {
        if (!p.str(strs[f])) return set_error(LSMCK_EJSON, "metadata file: expected a string");
      } else if (!p.skip_value()) {
        return set_error(LSMCK_EJSON, "metadata file: bad value");
      }
      if (f >= 0) have[f] = true;
      if (p.lit(',')) continue;
      if (p.lit('}')) break;
      return set_error(LSMCK_EJSON, "metadata file: expected ',' or '}'");
    }
  }
  p.ws();
  if (p.i != p.n) return set_error(LSMCK_EJSON, "metadata file: trailing characters");
  for (int k = 0; k < 8; ++k)
    if (!have[k]) return set_error(LSMCK_EJSON, (std::string("metadata file: missing field `") + kNames[k] + "`").c_str());
  return 0;
}

// PathBuf::push: an absolute component replaces the path, otherwise joins with '/'
std::string path_push(const std::string& a, const std::string& b) {
  if (!b.empty() && b[0] == '/') return b;
  if (a.empty() || a.back() == '/') return a + b;
  return a + "/" + b;
}

}  // namespace lsmck_host

extern "C" const char* lsmck_last_error(void) { return lsmck_host::g_err.c_str(); }
