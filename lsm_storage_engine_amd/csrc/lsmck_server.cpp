// lsmck_server -- the loopback line-protocol server of the reference
// (src/server.rs, protocol src/command.rs), the front end that drives the
// checksum path end to end (BASELINE config 5):
//
//   * start-up is Db::load (src/tokio/db.rs:37-73): every SSTable of the tree
//     verified in one GPU batch (lsmck_tree_verify: Checksums::verify of every
//     table, checksums.rs:40-62), then the WAL replayed with its payload CRCs
//     checked in one GPU batch (lsmck_wal_replay_verify: CommandLog iterator +
//     MemTable::from_log, wal.rs:68-163, memtable.rs:28-47).  The replay runs
//     on its own thread and context while the tree is verified; its outcome is
//     acted on after the tree's, so a failing start-up reports what the
//     reference reports;
//   * every insert / update / delete is appended to the WAL with its CRC-32
//     from lsmck_crc32_ieee (through lsmck_wal_encode_*: CommandLog::log,
//     wal.rs:165-196), one write(2) per record as the reference's flushed
//     BufWriter does;
//   * a memtable over memtable_limit_bytes is flushed to a level-0 SSTable in
//     the reference's on-disk layout, its checksum file written by
//     lsmck_checksums_write (Checksums::write_checksums, checksums.rs:64-80)
//     (db.rs:73-123).  One deliberate difference: the reference deletes and
//     recreates the WAL after the flush completes (db.rs:109-114), so records
//     appended between the memtable swap and the delete are lost from the log
//     (a crash loses them).  Here the log is rotated AT the swap (wal.log ->
//     wal.log.flushing, a fresh wal.log for the new memtable) and the rotated
//     log is deleted when its table is written; a start-up that finds one
//     replays it before wal.log and merges the two;
//   * get reads the memtable, the memtable being flushed, then the SSTables
//     (level 0 first, newest table first) through their sparse index and data
//     file (tokio/sstable.rs:63-86, datafile.rs:70-112).  Bloom filters are not
//     read (their probabilistic-collections encoding is not reproduced; the
//     flush writes an empty bloom file); in their place a table is skipped when
//     the key lies outside its key range (first index key .. last record's
//     key, the latter read once per table on first use).
//
// Responses are the reference's: "ok", the value, "<key> not found",
// "Supported commands: get, insert, update, delete" (server.rs:42-67).  A
// command with a missing argument makes the reference's connection task panic
// (command.rs:27 indexes args[1]); here the connection is closed.  At EOF the
// reference's read_line loop spins on Ok(0) (server.rs:20); here the
// connection is closed.
//
// The compaction tick (server.rs:93-99: tokio interval of 10 s, its first
// tick at once) runs Db::compact (tokio/db.rs:191-228), whose checksum work
// is the re-verify: every table of levels 0..3 it keeps is cloned, and
// SsTable's Clone is SsTable::load (tokio/sstable.rs:274-277), which runs
// Checksums::verify (checksums.rs:40-62) on it.  Here each tick verifies
// those tables in one GPU batch (lsmck_checksums_verify_many) while the
// server serves.  The merge of a level at sstable_level_limit tables is not
// run (compaction proper is not on the checksum path): such a level keeps its
// tables and they are re-verified like the clones; the reference's quirk of
// dropping level 4 from the new levels (db.rs:221-222) is not reproduced.  A
// table that fails the verify panics the tick as the reference's does (its
// message, then "Compact failed"): ticks stop, serving goes on (a panicked
// tokio task does not end the process).
//
// Usage: lsmck_server [--base DIR] [--port P] [--bind ADDR] [--device D]
//                     [--memtable-limit BYTES] [--compact-interval MS]
//                     [--exit-after-load]
// Prints one JSON line when loaded ({"event":"loaded",...}), one when it
// listens ({"event":"listening","port":P}), and one per compaction tick
// ({"event":"compact",...}; {"event":"compact_failed",...}).
#include <arpa/inet.h>
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "lsmck.h"

namespace {

constexpr int kMaxLevel = LSMCK_SSTABLE_MAX_LEVEL;  // db.rs:17
constexpr size_t kIndexStep = 100;                  // tokio/sstable.rs:17

double now_s() {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

[[noreturn]] void panic_exit(const std::string& msg) {
  // a Rust panic in main: the message on stderr, exit status 101
  fprintf(stderr, "thread 'main' panicked at '%s'\n", msg.c_str());
  fflush(stderr);
  _exit(101);
}

std::string join(const std::string& a, const std::string& b) {
  if (a.empty()) return b;
  return a.back() == '/' ? a + b : a + "/" + b;
}

int mkdir_p(const std::string& p) {
  struct stat st;
  if (stat(p.c_str(), &st) == 0) return S_ISDIR(st.st_mode) ? 0 : -EEXIST;
  size_t cut = p.find_last_of('/');
  if (cut != std::string::npos && cut > 0) {
    int rc = mkdir_p(p.substr(0, cut));
    if (rc) return rc;
  }
  if (mkdir(p.c_str(), 0777) != 0 && errno != EEXIST) return -errno;
  return 0;
}

bool read_file(const std::string& path, std::string* out) {
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  out->clear();
  char buf[1 << 16];
  for (;;) {
    ssize_t k = read(fd, buf, sizeof buf);
    if (k < 0) {
      if (errno == EINTR) continue;
      close(fd);
      return false;
    }
    if (k == 0) break;
    out->append(buf, (size_t)k);
  }
  close(fd);
  return true;
}

bool write_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t k = write(fd, c, n);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= (size_t)k;
  }
  return true;
}

void put_u32(std::string& s, uint32_t v) {
  for (int i = 0; i < 4; ++i) s.push_back((char)(v >> (8 * i)));
}
void put_u64(std::string& s, uint64_t v) {
  for (int i = 0; i < 8; ++i) s.push_back((char)(v >> (8 * i)));
}
uint32_t get_u32(const unsigned char* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
uint64_t get_u64(const unsigned char* p) { return (uint64_t)get_u32(p) | ((uint64_t)get_u32(p + 4) << 32); }

// serde_json string escaping (the metadata's file names and base path)
std::string json_str(const std::string& s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o.push_back('\\');
      o.push_back((char)c);
    } else if (c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      o += b;
    } else {
      o.push_back((char)c);
    }
  }
  return o + "\"";
}

// the few fields of a SsTableMetadata JSON record the read path needs
// (sstable_metadata.rs:8-17); the file was verified by lsmck_tree_verify's
// serde-rules parser already
bool json_field(const std::string& j, const char* key, std::string* out) {
  const std::string k = std::string("\"") + key + "\"";
  size_t i = j.find(k);
  if (i == std::string::npos) return false;
  i = j.find(':', i + k.size());
  if (i == std::string::npos) return false;
  ++i;
  while (i < j.size() && isspace((unsigned char)j[i])) ++i;
  if (i < j.size() && j[i] == '"') {
    std::string v;
    for (++i; i < j.size() && j[i] != '"'; ++i) {
      if (j[i] == '\\' && i + 1 < j.size()) ++i;
      v.push_back(j[i]);
    }
    *out = v;
    return true;
  }
  size_t e = i;
  while (e < j.size() && (isdigit((unsigned char)j[e]) || j[e] == '-')) ++e;
  *out = j.substr(i, e - i);
  return e > i;
}

// ---------------------------------------------------------------------------
// MemTable (src/memtable.rs): BTreeMap + byte count
struct MemTable {
  std::map<std::string, std::string> data;
  size_t bytes = 0;
  void insert(const std::string& k, const std::string& v) {  // memtable.rs:67-74
    auto it = data.find(k);
    size_t prev = it != data.end() ? it->second.size() + k.size() : 0;
    bytes = bytes + k.size() + v.size() - prev;
    data[k] = v;
  }
  void remove(const std::string& k) {  // memtable.rs:76-81
    auto it = data.find(k);
    if (it == data.end()) return;
    bytes -= it->second.size() + k.size();
    data.erase(it);
  }
  const std::string* get(const std::string& k) const {
    auto it = data.find(k);
    return it == data.end() ? nullptr : &it->second;
  }
};

// ---------------------------------------------------------------------------
// SSTable read path: sparse index (bincode BTreeMap<Vec<u8>, u64>,
// sstable_index.rs) + data file ([u32 klen][u32 vlen][key][val], datafile.rs)
struct SsTable {
  uint64_t id = 0;
  int level = 0;
  std::string data_path, index_path, checksum_path;
  std::map<std::string, uint64_t> index;
  mutable std::once_flag last_once;
  mutable std::string last_key;  // the table's largest key (read on first use)

  bool load_index(const std::string& index_path) {
    std::string b;
    if (!read_file(index_path, &b) || b.size() < 8) return false;
    const unsigned char* p = (const unsigned char*)b.data();
    size_t n = b.size(), pos = 8;
    const uint64_t cnt = get_u64(p);
    for (uint64_t i = 0; i < cnt; ++i) {
      if (pos + 8 > n) return false;
      const uint64_t kl = get_u64(p + pos);
      pos += 8;
      if (pos + kl + 8 > n) return false;
      std::string k((const char*)p + pos, (size_t)kl);
      pos += kl;
      // bincode writes a BTreeMap in key order, so the end is the hint (a
      // repeated key keeps its last value, as the map's deserializer does)
      const uint64_t v = get_u64(p + pos);
      index.emplace_hint(index.end(), std::move(k), v)->second = v;
      pos += 8;
    }
    return true;
  }

  // read_record at pos: false at EOF (UnexpectedEof -> None, datafile.rs:59-67)
  static bool read_record(int fd, uint64_t pos, std::string* k, std::string* v, uint64_t* len) {
    unsigned char h[8];
    if (pread(fd, h, 8, (off_t)pos) != 8) return false;
    const uint32_t kl = get_u32(h), vl = get_u32(h + 4);
    std::string buf((size_t)kl + vl, '\0');
    if (kl + (size_t)vl && pread(fd, &buf[0], buf.size(), (off_t)(pos + 8)) != (ssize_t)buf.size()) return false;
    *k = buf.substr(0, kl);
    *v = buf.substr(kl);
    *len = 8ull + kl + vl;
    return true;
  }

  // the largest key: the records after the last index entry, read once
  const std::string& last() const {
    std::call_once(last_once, [this] {
      if (index.empty()) return;
      int fd = open(data_path.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) return;
      std::string k, v;
      uint64_t len = 0;
      for (uint64_t pos = index.rbegin()->second; read_record(fd, pos, &k, &v, &len); pos += len) last_key = k;
      close(fd);
    });
    return last_key;
  }
  void set_last(const std::string& k) {  // a table written here: its last key is known
    std::call_once(last_once, [&] { last_key = k; });
  }
  const std::string& first() const { return index.begin()->first; }

  // tokio/sstable.rs:63-86: exact index hit -> read_record, else scan the
  // index range that can hold the key
  bool get(const std::string& key, std::string* val) const {
    // key range filter (in place of the bloom filter, tokio/sstable.rs:64)
    if (index.empty() || key < first() || key > last()) return false;
    int fd = open(data_path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return false;
    std::string k, v;
    uint64_t len = 0;
    bool found = false;
    auto hit = index.find(key);
    if (hit != index.end()) {
      found = read_record(fd, hit->second, &k, &v, &len) && k == key;
    } else {
      auto hi = index.lower_bound(key);  // first entry >= key
      // (past the last entry: to EOF, where read_record stops -- the records fill the file)
      const uint64_t end = hi == index.end() ? UINT64_MAX : hi->second;
      uint64_t start = 0;
      if (hi != index.begin()) start = std::prev(hi)->second;
      for (uint64_t pos = start; read_record(fd, pos, &k, &v, &len);) {  // datafile.rs:87-106
        if (k == key) {
          found = true;
          break;
        }
        pos += len;
        if (pos >= end) break;
      }
    }
    close(fd);
    if (found) *val = v;
    return found;
  }
};

// One level's tables by key range, for Db::get: the reference asks every
// table of a level (its bloom filter, tokio/db.rs:160-181); a 100 GiB tree has
// ~230k tables, so the tables whose [first, last] key range can hold the key
// are found by binary search over the first keys and a running maximum of the
// last keys, then asked newest first as the reference does.
struct LevelIndex {
  bool built = false;
  std::vector<std::shared_ptr<SsTable>> by_first;  // non-empty tables, ascending first key
  std::vector<const std::string*> max_last;        // max_last[i] = max last key of by_first[0..i]

  void build(const std::vector<std::shared_ptr<SsTable>>& tables) {
    by_first.clear();
    for (const auto& t : tables)
      if (!t->index.empty()) by_first.push_back(t);
    std::sort(by_first.begin(), by_first.end(),
              [](const std::shared_ptr<SsTable>& a, const std::shared_ptr<SsTable>& b) { return a->first() < b->first(); });
    max_last.resize(by_first.size());
    for (size_t i = 0; i < by_first.size(); ++i) {
      const std::string& l = by_first[i]->last();
      max_last[i] = (i && *max_last[i - 1] > l) ? max_last[i - 1] : &l;
    }
    built = true;
  }
  // the tables that may hold k, newest (largest id) first
  void candidates(const std::string& k, std::vector<SsTable*>* out) const {
    out->clear();
    size_t p = std::upper_bound(by_first.begin(), by_first.end(), k,
                                [](const std::string& key, const std::shared_ptr<SsTable>& t) { return key < t->first(); }) -
               by_first.begin();
    while (p > 0 && !(*max_last[p - 1] < k)) {
      --p;
      if (!(by_first[p]->last() < k)) out->push_back(by_first[p].get());
    }
    std::sort(out->begin(), out->end(), [](const SsTable* a, const SsTable* b) { return a->id > b->id; });
  }
};

struct Config {
  std::string base = "./data";
  size_t memtable_limit = 4096;  // config/default: memtable_limit_bytes
  int port = 3333;
  std::string bind = "127.0.0.1";
  int device = 0;
  bool exit_after_load = false;
  long compact_interval_ms = 10000;  // server.rs:94 (0: no tick)
  // Db::load: threads loading the tables' sparse indexes beside the verify.
  // Two: small-file system calls contend in the kernel, so two load the 229k
  // indexes of the 100 GiB tree as fast as eight (0.78-0.92 s either way)
  // while taking less from the verify's readers (Db::load 3.26-3.48 s against
  // 3.51-3.61 s with eight; profiles/r05/srv2)
  int index_threads = 2;
};

// the name a panic of Checksums::verify (checksums.rs:49-60) gives: the
// metadata's data_filename / index_filename (the file name in the table's
// level directory)
std::string base_name(const std::string& p) {
  const size_t s = p.rfind('/');
  return s == std::string::npos ? p : p.substr(s + 1);
}

// the reference's panic message for a table whose verify returned `status`
// (lsmck_checksums_verify_many), or "" for an io::Error (the caller's
// expect() names it)
std::string verify_panic(int status, const std::string& data_path, const std::string& index_path) {
  switch (status) {
    case LSMCK_DATA_MISMATCH: return "Can't load SSTable from " + base_name(data_path) + ". Checksum is not correct";
    case LSMCK_INDEX_MISMATCH: return "Can't load SSTable from " + base_name(index_path) + ". Checksum is not correct";
    case LSMCK_PANIC_OPEN_FILE:
    case LSMCK_PANIC_OPEN_INDEX: return "Can't open file to calculate checksum";
    case LSMCK_PANIC_OPEN_CHECKSUM: return "Can't open checksum file";
    default: return "";
  }
}

// ---------------------------------------------------------------------------
struct Db {
  Config cfg;
  lsmck_ctx* ctx = nullptr;
  std::mutex wal_mu;
  int wal_fd = -1;
  std::mutex mem_mu;
  MemTable mem;
  std::shared_ptr<const MemTable> old;  // being flushed (db.rs:28)
  std::shared_mutex lv_mu;
  std::vector<std::vector<std::shared_ptr<SsTable>>> levels{(size_t)kMaxLevel};
  std::vector<LevelIndex> lindex{(size_t)kMaxLevel};  // built at a level's first table read
  uint64_t last_id = 0;

  std::string wal_path() const { return join(join(cfg.base, "wal"), "wal.log"); }
  std::string flushing_path() const { return wal_path() + ".flushing"; }

  int open_wal() {  // CommandLog::new (wal.rs:86-101): create dirs, read + append
    mkdir_p(join(cfg.base, "wal"));
    return open(wal_path().c_str(), O_RDWR | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
  }

  // Db::load (db.rs:37-73)
  void load() {
    const double t0 = now_s();
    // The tables' read-path state (their sparse indexes) is loaded on its own
    // threads while the tree is verified, from the verify's own listing
    // (lsmck_tree_verify_listed): every metadata file is opened once.  The
    // server serves nothing before both are done.
    int idx_err = 0;
    double t_index = 0;
    struct Listed {
      Db* db;
      int threads;
      std::vector<std::string> data, index, checksum;
      std::vector<uint64_t> id;
      std::vector<int> level;
      std::thread th;
      int* err;
      double* secs;
    } L{this, cfg.index_threads, {}, {}, {}, {}, {}, {}, &idx_err, &t_index};
    auto on_listed = [](void* user, const lsmck_table_entry* e, size_t n) {
      Listed& L = *(Listed*)user;
      const double t_idx0 = now_s();
      for (size_t i = 0; i < n; ++i) {  // copies: the entries die with the verify call
        if (e[i].status) continue;  // a bad metadata file: the verify reports it (the reference panics)
        L.data.emplace_back(e[i].data_path);
        L.index.emplace_back(e[i].index_path);
        L.checksum.emplace_back(e[i].checksum_path);
        L.id.push_back(strtoull(e[i].id, nullptr, 10));
        L.level.push_back((int)e[i].level);
      }
      L.th = std::thread([&L, t_idx0]() {
        const size_t m = L.data.size();
        std::vector<std::shared_ptr<SsTable>> tabs(m);
        std::atomic<size_t> next{0};
        std::atomic<bool> bad{false};
        auto work = [&]() {
          for (size_t i; (i = next.fetch_add(1)) < m;) {
            auto t = std::make_shared<SsTable>();
            t->id = L.id[i];
            t->level = L.level[i];
            t->data_path = L.data[i];
            t->index_path = L.index[i];
            t->checksum_path = L.checksum[i];
            if (!t->load_index(L.index[i])) bad = true;
            tabs[i] = t;
          }
        };
        std::vector<std::thread> th;
        for (size_t k = 1; k < std::min<size_t>((size_t)std::max(1, L.threads), m); ++k) th.emplace_back(work);
        work();
        for (auto& x : th) x.join();
        if (bad) {
          *L.err = 2;
          return;
        }
        for (auto& t : tabs) {
          if (t->level < 0 || t->level >= kMaxLevel) continue;
          L.db->last_id = std::max(L.db->last_id, t->id);
          L.db->levels[t->level].push_back(t);
        }
        for (auto& lv : L.db->levels)  // load order: per level, sorted by id
          std::sort(lv.begin(), lv.end(),
                    [](const std::shared_ptr<SsTable>& a, const std::shared_ptr<SsTable>& b) { return a->id < b->id; });
        *L.secs = now_s() - t_idx0;
      });
    };
    // The WAL is replayed on its own thread (and its own context on the same
    // GPU) while the tree is verified: the two read different files and
    // neither result depends on the other.  Its outcome is acted on only after
    // the tree's, in Db::load's order (db.rs:37-73: the tables, then
    // MemTable::from_log), so a start-up that fails reports what the
    // reference reports.  Nothing on disk changes before the tree is verified:
    // a rotated log (wal.log.flushing) is replayed from memory in front of
    // wal.log, and merged on disk afterwards.
    struct WalLoad {
      int rc = 0;                // lsmck_wal_replay_verify's result, or -1: see err
      std::string err;           // a message for exit(1) (rc < 0)
      std::string panic;         // a panic message (the replayed payloads)
      bool have_older = false;   // a rotated log was found
      std::string older, newer;  // its bytes and wal.log's (only when have_older)
      size_t n = 0, nrec = 0;
      double t_verify = 0, t_wal = 0;
    } W;
    // own_ctx: the replay's own context (beside the tree verify); otherwise
    // the given one (the sequential retry below)
    auto run_wal = [this, &W](lsmck_ctx* use_ctx) {
      const double t1 = now_s();
      const uint8_t* img = nullptr;
      void* map = nullptr;
      size_t n = 0;
      int rfd = -1;
      if (read_file(flushing_path(), &W.older)) {
        W.have_older = true;
        read_file(wal_path(), &W.newer);
        W.older += W.newer;
        img = (const uint8_t*)W.older.data();
        n = W.older.size();
      } else if ((rfd = open(wal_path().c_str(), O_RDONLY | O_CLOEXEC)) >= 0) {
        struct stat st;
        fstat(rfd, &st);
        n = (size_t)st.st_size;
        if (n) {
          map = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, rfd, 0);
          if (map == MAP_FAILED) {
            W.rc = -1;
            W.err = std::string("mmap wal: ") + strerror(errno);
            close(rfd);
            return;
          }
          img = (const uint8_t*)map;
        }
      }
      W.n = n;
      lsmck_ctx* wctx = use_ctx ? use_ctx : lsmck_ctx_create(cfg.device);
      if (!wctx) {
        W.rc = -1;
        W.err = std::string("lsmck_ctx_create: ") + lsmck_last_error();
      }
      const size_t cap = n / 9 + 1;  // a record is at least 9 bytes
      // uninitialised: only the records found are written (a zeroed vector of
      // 32 B per 9 log bytes cost more than the replay itself)
      std::unique_ptr<lsmck_wal_rec[]> recs(new lsmck_wal_rec[cap]);
      size_t nrec = 0;
      uint64_t bad_index = 0;
      uint32_t bad_crc = 0, bad_expected = 0;
      char msg[256];
      if (wctx) {
        W.rc = lsmck_wal_replay_verify(wctx, img, n, LSMCK_HOST, recs.get(), cap, &nrec, &bad_index, &bad_crc,
                                       &bad_expected);
        if (W.rc < 0) W.err = std::string("lsmck_wal_replay_verify: ") + lsmck_last_error();
        if (!use_ctx) lsmck_ctx_destroy(wctx);
      }
      W.t_verify = now_s() - t1;
      W.nrec = nrec;
      if (W.rc == LSMCK_WAL_CORRUPTED) {  // MemTable::from_log(..).expect(..) on Err (db.rs:61-62)
        snprintf(msg, sizeof msg, "Can't restore memtable from a log: CorruptedData { checksum: %u, expected: %u }",
                 bad_crc, bad_expected);
        W.panic = msg;
      } else if (W.rc == LSMCK_WAL_REMOVE_PANIC) {  // wal.rs:154-159
        snprintf(msg, sizeof msg, "data corruption encountered (%08x) != %08x", bad_crc, bad_expected);
        W.panic = msg;
      } else if (W.rc == LSMCK_WAL_BAD_TYPE) {
        snprintf(msg, sizeof msg, "Can't restore memtable from a log: InvalidCommandType(%u)", bad_crc);
        W.panic = msg;
      }
      if (W.rc < 0 || !W.panic.empty()) {
        if (map) munmap(map, n);
        if (rfd >= 0) close(rfd);
        return;
      }
      // MemTable::from_log (memtable.rs:28-47), on the payload actually read
      // (short at EOF).  The records are grouped by key (a stable sort keeps log
      // order inside a key); each key's final state and its share of the
      // reference's byte count are replayed per key, and the table is built in
      // key order with an end hint.  Same table and count as inserting record by
      // record, which took 0.48 s for 500k records (std::map comparisons and
      // rebalancing).  The count is from_log's: an Insert adds key + value even
      // over an existing key, a Remove of a present key subtracts its entry.
      struct KeyRec {
        std::string_view k;
        uint32_t i;
      };
      std::vector<KeyRec> kr(nrec);
      auto payload = [&](size_t i, size_t* klen, size_t* got) {
        const lsmck_wal_rec& r = recs[i];
        const uint64_t want = (uint64_t)(uint32_t)(r.klen + r.vlen);
        *got = (size_t)std::min<uint64_t>(want, n - r.payload_off);
        *klen = r.type == 1 ? (size_t)std::min<uint64_t>(r.klen, *got) : *got;
        return (const char*)img + r.payload_off;
      };
      for (size_t i = 0; i < nrec; ++i) {
        size_t kl, got;
        const char* p = payload(i, &kl, &got);
        if (recs[i].type == 1 && got < recs[i].klen) {
          // an Insert cut at EOF inside its key whose CRC matches the short
          // bytes: data.split_off(key_len) panics (wal.rs:142)
          snprintf(msg, sizeof msg, "`at` split index (is %u) should be <= len (is %zu)", recs[i].klen, got);
          W.panic = msg;
          if (map) munmap(map, n);
          if (rfd >= 0) close(rfd);
          return;
        }
        kr[i] = {std::string_view(p, kl), (uint32_t)i};
      }
      std::stable_sort(kr.begin(), kr.end(), [](const KeyRec& a, const KeyRec& b) { return a.k < b.k; });
      size_t bytes = 0;
      for (size_t a = 0; a < nrec;) {
        size_t b = a + 1;
        while (b < nrec && kr[b].k == kr[a].k) ++b;
        bool present = false;
        size_t vlen = 0, last = 0;
        for (size_t x = a; x < b; ++x) {
          size_t kl, got;
          payload(kr[x].i, &kl, &got);
          if (recs[kr[x].i].type == 1) {
            bytes += got;  // key + value
            present = true;
            vlen = got - kl;
            last = kr[x].i;
          } else if (present) {
            bytes -= vlen + kr[a].k.size();
            present = false;
          }
        }
        if (present) {
          size_t kl, got;
          const char* p = payload(last, &kl, &got);
          mem.data.emplace_hint(mem.data.end(), std::string(kr[a].k), std::string(p + kl, got - kl));
        }
        a = b;
      }
      mem.bytes = bytes;
      if (map) munmap(map, n);
      if (rfd >= 0) close(rfd);
      W.t_wal = now_s() - t1;
    };
    std::thread wal_th(run_wal, nullptr);
    lsmck_tree_report rep;
    int rc = lsmck_tree_verify_listed(ctx, cfg.base.c_str(), &rep, on_listed, &L);
    if (L.th.joinable()) L.th.join();
    wal_th.join();
    if (rc < 0) {
      fprintf(stderr, "lsmck_tree_verify: %s\n", lsmck_last_error());
      exit(1);
    }
    if (rc == 1) {  // the reference panics at its first bad table (SsTable::load)
      switch (rep.first_status) {
        case LSMCK_META_PANIC: panic_exit("Can't read metadata file, file with unknown format");
        case LSMCK_DATA_MISMATCH:
        case LSMCK_INDEX_MISMATCH: {  // checksums.rs:49-60 names the data / index file
          std::string j, fn;
          read_file(rep.first_metadata_path, &j);
          json_field(j, rep.first_status == LSMCK_DATA_MISMATCH ? "data_filename" : "index_filename", &fn);
          panic_exit(verify_panic(rep.first_status, fn, fn));
        }
        case LSMCK_PANIC_OPEN_FILE:
        case LSMCK_PANIC_OPEN_INDEX: panic_exit("Can't open file to calculate checksum");
        case LSMCK_PANIC_OPEN_CHECKSUM: panic_exit("Can't open checksum file");
        default:  // io::Error from SsTable::load -> `?` in Db::load -> .expect in main
          panic_exit(std::string("unable run storage: ") + rep.first_metadata_path + " (" +
                     std::to_string(rep.first_status) + ")");
      }
    }
    const double t_tree = now_s() - t0;
    if (idx_err == 2) panic_exit("Can't open index file");
    if (W.rc < 0) {
      // the concurrent replay failed as a call (its context or device memory
      // beside the tree verify's, not the log's contents): once more, alone,
      // on the server's context, as a sequential Db::load would have run it
      fprintf(stderr, "WAL replay beside the tree verify failed (%s); replaying alone\n", W.err.c_str());
      W = WalLoad();
      run_wal(ctx);
    }
    // the WAL's outcome, in from_log's place
    if (W.rc < 0) {
      fprintf(stderr, "%s\n", W.err.c_str());
      exit(1);
    }
    if (!W.panic.empty()) panic_exit(W.panic);
    if (W.have_older) {
      // a log rotated at a memtable swap whose flush did not complete: its
      // records came first in the replay; merge it in front of wal.log (see
      // the header)
      const std::string tmp = wal_path() + ".merge";
      int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
      if (fd < 0 || !write_all(fd, W.older.data(), W.older.size()) || fsync(fd) != 0 || close(fd) != 0 ||
          rename(tmp.c_str(), wal_path().c_str()) != 0)
        panic_exit("Can't merge the rotated WAL");
      unlink(flushing_path().c_str());
      std::string().swap(W.older);
    }
    wal_fd = open_wal();
    if (wal_fd < 0) {
      fprintf(stderr, "Can't create WAL file: %s\n", strerror(errno));
      exit(1);
    }
    const size_t n = W.n, nrec = W.nrec;
    const double t_verify = W.t_verify, t_wal = W.t_wal;
    uint64_t ntab = 0;
    for (auto& l : levels) ntab += l.size();
    printf("{\"event\": \"loaded\", \"tables\": %llu, \"table_bytes\": %llu, \"tree_verify_s\": %.6f, "
           "\"tree_list_s\": %.6f, \"wal_bytes\": %zu, \"wal_records\": %zu, \"wal_replay_s\": %.6f, "
           "\"wal_verify_s\": %.6f, \"memtable_entries\": %zu, \"memtable_bytes\": %zu, \"load_s\": %.6f, "
           "\"tree_phases\": {\"stat_s\": %.6f, \"read_s\": %.6f, \"gpu_wait_s\": %.6f, \"compare_s\": %.6f, "
           "\"rounds\": %llu}, \"index_load_s\": %.6f}\n",
           (unsigned long long)ntab, (unsigned long long)rep.table_bytes, t_tree, rep.list_seconds, n, nrec, t_wal,
           t_verify, mem.data.size(), mem.bytes, now_s() - t0, rep.stat_seconds, rep.read_seconds,
           rep.gpu_wait_seconds, rep.compare_seconds, (unsigned long long)rep.rounds, t_index);
    fflush(stdout);
  }

  int wal_append(const std::string& rec) {
    std::lock_guard<std::mutex> lk(wal_mu);
    return write_all(wal_fd, rec.data(), rec.size()) ? 0 : -errno;
  }

  // Db::insert (db.rs:76-124)
  int insert(const std::string& k, const std::string& v) {
    std::string rec(13 + k.size() + v.size(), '\0');
    lsmck_wal_encode_insert((const uint8_t*)k.data(), (uint32_t)k.size(), (const uint8_t*)v.data(),
                            (uint32_t)v.size(), (uint8_t*)&rec[0]);
    std::shared_ptr<const MemTable> to_flush;
    {
      // the log record and the memtable entry change together with respect to
      // a swap (a record never lands in one memtable's log and the other table)
      std::lock_guard<std::mutex> lk(mem_mu);
      int rc = wal_append(rec);
      if (rc) return rc;
      mem.insert(k, v);
      if (mem.bytes > cfg.memtable_limit && !old) {
        old = std::make_shared<const MemTable>(std::move(mem));
        mem = MemTable();
        to_flush = old;
        // rotate the log with the memtable (the reference recreates it only
        // after the flush, db.rs:109-114, and loses what came in between)
        std::lock_guard<std::mutex> wl(wal_mu);
        close(wal_fd);
        if (rename(wal_path().c_str(), flushing_path().c_str()) != 0) panic_exit("Can't rotate WAL file");
        wal_fd = open_wal();
        if (wal_fd < 0) panic_exit("Can't create WAL file");
      }
    }
    if (to_flush) std::thread([this, to_flush] { flush(to_flush); }).detach();
    return 0;
  }

  // Db::delete (db.rs:131-143): WAL Remove, memtable tombstone vec![0]
  int remove(const std::string& k) {
    std::string rec(9 + k.size(), '\0');
    lsmck_wal_encode_remove((const uint8_t*)k.data(), (uint32_t)k.size(), (uint8_t*)&rec[0]);
    std::lock_guard<std::mutex> lk(mem_mu);
    int rc = wal_append(rec);
    if (rc) return rc;
    mem.insert(k, std::string(1, '\0'));
    return 0;
  }

  // Db::get (db.rs:144-186); a tombstone [0] reads as not found
  bool get(const std::string& k, std::string* v) {
    bool found = false;
    {
      std::lock_guard<std::mutex> lk(mem_mu);
      if (const std::string* p = mem.get(k)) {
        *v = *p;
        found = true;
      } else if (old) {
        if (const std::string* q = old->get(k)) {
          *v = *q;
          found = true;
        }
      }
    }
    for (int lv = 0; lv < kMaxLevel && !found; ++lv) {
      std::shared_lock<std::shared_mutex> lk(lv_mu);
      if (!lindex[lv].built) {
        lk.unlock();
        {
          std::unique_lock<std::shared_mutex> ul(lv_mu);
          if (!lindex[lv].built) lindex[lv].build(levels[lv]);
        }
        lk.lock();
      }
      thread_local std::vector<SsTable*> cand;
      lindex[lv].candidates(k, &cand);
      for (SsTable* t : cand)
        if ((found = t->get(k, v))) break;
    }
    return found && !(v->size() == 1 && (*v)[0] == '\0');
  }

  // One compaction tick's checksum work (Db::compact, tokio/db.rs:191-228):
  // the tables of levels 0..3, each verified as its clone's SsTable::load
  // would (tokio/sstable.rs:274-277 -> checksums.rs:40-62), in one GPU batch.
  // Returns false when one fails: the reference's panic is printed and the
  // tick task is over.
  bool compact_tick(uint64_t tick) {
    std::vector<std::shared_ptr<SsTable>> tabs;
    {
      std::shared_lock<std::shared_mutex> lk(lv_mu);
      for (int lv = 0; lv < kMaxLevel - 1; ++lv) tabs.insert(tabs.end(), levels[lv].begin(), levels[lv].end());
    }
    const size_t n = tabs.size();
    std::vector<const char*> d(n), ix(n), c(n);
    uint64_t bytes = 0;
    for (size_t i = 0; i < n; ++i) {
      d[i] = tabs[i]->data_path.c_str();
      ix[i] = tabs[i]->index_path.c_str();
      c[i] = tabs[i]->checksum_path.c_str();
      struct stat st;
      if (stat(d[i], &st) == 0) bytes += (uint64_t)st.st_size;
      if (stat(ix[i], &st) == 0) bytes += (uint64_t)st.st_size;
    }
    std::vector<int> status(std::max<size_t>(n, 1), 0);
    const double t0 = now_s();
    const int rc = n ? lsmck_checksums_verify_many(ctx, d.data(), ix.data(), c.data(), n, status.data()) : 0;
    const double dt = now_s() - t0;
    if (rc < 0) {
      fprintf(stderr, "lsmck_checksums_verify_many: %s\n", lsmck_last_error());
      return false;
    }
    size_t bad = n;
    for (size_t i = 0; i < n && bad == n; ++i)
      if (status[i]) bad = i;  // the clone loop's first failing table (level, then id order)
    if (bad < n) {
      std::string msg = verify_panic(status[bad], tabs[bad]->data_path, tabs[bad]->index_path);
      if (msg.empty()) msg = "Can't load sstable file: status " + std::to_string(status[bad]);  // expect() on Err
      fprintf(stderr, "thread 'tokio-runtime-worker' panicked at '%s'\n", msg.c_str());
      fprintf(stderr, "thread 'tokio-runtime-worker' panicked at 'Compact failed: JoinError::Panic(...)'\n");
      fflush(stderr);
      printf("{\"event\": \"compact_failed\", \"tick\": %llu, \"panic\": %s}\n", (unsigned long long)tick,
             json_str(msg).c_str());
      fflush(stdout);
      return false;
    }
    printf("{\"event\": \"compact\", \"tick\": %llu, \"tables\": %zu, \"table_bytes\": %llu, "
           "\"verify_s\": %.6f, \"GiBps\": %.3f}\n",
           (unsigned long long)tick, n, (unsigned long long)bytes, dt, dt > 0 ? (double)bytes / dt / 1073741824.0 : 0.0);
    fflush(stdout);
    return true;
  }

  // server.rs:93-99: tokio::time::interval -- the first tick at once, then one
  // per period (a late tick is not made up twice here: the next waits a period)
  void compact_loop() {
    const auto period = std::chrono::milliseconds(cfg.compact_interval_ms);
    auto next = std::chrono::steady_clock::now();
    for (uint64_t tick = 0;; ++tick) {
      std::this_thread::sleep_until(next);
      if (!compact_tick(tick)) return;
      next = std::max(next + period, std::chrono::steady_clock::now());
    }
  }

  // SsTable::from_memtable (tokio/sstable.rs:88-111) + the WAL swap (db.rs:100-121)
  void flush(std::shared_ptr<const MemTable> m) {
    uint64_t id;
    {
      std::unique_lock<std::shared_mutex> lk(lv_mu);
      struct timespec ts;
      clock_gettime(CLOCK_REALTIME, &ts);
      id = (uint64_t)ts.tv_sec * 1000ull + (uint64_t)ts.tv_nsec / 1000000ull;  // ms ids (sstable_metadata.rs:21-27)
      if (id <= last_id) id = last_id + 1;  // two flushes in one ms would share file names
      last_id = id;
    }
    const std::string ids = std::to_string(id), dir = join(cfg.base, "level-0");
    mkdir_p(dir);
    const std::string data_fn = "data_" + ids + ".db", index_fn = "index_" + ids + ".db",
                      checksum_fn = "checksum_" + ids + ".db", bloom_fn = "bloom_" + ids + ".db",
                      meta_fn = "metadata_" + ids + ".db";
    auto t = std::make_shared<SsTable>();
    t->id = id;
    t->data_path = join(dir, data_fn);
    t->index_path = join(dir, index_fn);
    t->checksum_path = join(dir, checksum_fn);
    std::string data, index;
    uint64_t i = 0;
    if (!m->data.empty()) t->set_last(m->data.rbegin()->first);
    for (const auto& kv : m->data) {  // write_data_file (tokio/sstable.rs:113-135)
      if (i++ % kIndexStep == 0) t->index[kv.first] = data.size();
      put_u32(data, (uint32_t)kv.first.size());
      put_u32(data, (uint32_t)kv.second.size());
      data += kv.first;
      data += kv.second;
    }
    put_u64(index, t->index.size());  // bincode 1.x fixint BTreeMap<Vec<u8>, u64>
    for (const auto& e : t->index) {
      put_u64(index, e.first.size());
      index += e.first;
      put_u64(index, e.second);
    }
    auto write_file = [](const std::string& p, const std::string& b) {
      int fd = open(p.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
      if (fd < 0) return false;
      bool ok = write_all(fd, b.data(), b.size());
      close(fd);
      return ok;
    };
    std::string meta = "{\"base_path\":" + json_str(cfg.base) + ",\"id\":" + ids +
                       ",\"level\":0,\"metadata_filename\":" + json_str(meta_fn) +
                       ",\"checksum_filename\":" + json_str(checksum_fn) + ",\"data_filename\":" + json_str(data_fn) +
                       ",\"index_filename\":" + json_str(index_fn) +
                       ",\"bloom_filter_filename\":" + json_str(bloom_fn) + "}";
    if (!write_file(t->data_path, data) || !write_file(join(dir, index_fn), index))
      panic_exit("Can't create new sstable");
    int rc = lsmck_checksums_write(t->data_path.c_str(), join(dir, index_fn).c_str(), join(dir, checksum_fn).c_str());
    if (rc) panic_exit(std::string("Can't create new sstable: ") + lsmck_last_error());
    if (!write_file(join(dir, bloom_fn), "") || !write_file(join(dir, meta_fn), meta))
      panic_exit("Can't create new sstable");
    {
      std::unique_lock<std::shared_mutex> lk(lv_mu);
      levels[0].push_back(t);
      if (lindex[0].built) lindex[0].build(levels[0]);  // flushes are rare: rebuild
    }
    // the flushed memtable's log is no longer needed (wal.close(), db.rs:110)
    unlink(flushing_path().c_str());
    std::lock_guard<std::mutex> lk(mem_mu);
    old.reset();
  }
};

// String::from_utf8_lossy (server.rs:47): each maximal invalid subpart -> U+FFFD
std::string utf8_lossy(const std::string& in) {
  static const char kRep[] = "\xEF\xBF\xBD";
  std::string o;
  const unsigned char* s = (const unsigned char*)in.data();
  const size_t n = in.size();
  for (size_t i = 0; i < n;) {
    const unsigned c = s[i];
    if (c < 0x80) {
      o.push_back((char)c);
      ++i;
      continue;
    }
    size_t need;
    unsigned lo = 0x80, hi = 0xBF;  // bounds of the second byte
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) need = 2, lo = 0xA0;
    else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) need = 2;
    else if (c == 0xED) need = 2, hi = 0x9F;
    else if (c == 0xF0) need = 3, lo = 0x90;
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) need = 3, hi = 0x8F;
    else {
      o += kRep;
      ++i;
      continue;
    }
    size_t k = 1;
    for (; k <= need && i + k < n; ++k) {
      const unsigned b = s[i + k];
      if (k == 1 ? (b < lo || b > hi) : (b < 0x80 || b > 0xBF)) break;
    }
    if (k == need + 1) {
      o.append((const char*)s + i, need + 1);
      i += need + 1;
    } else {
      o += kRep;
      i += k;  // the valid prefix of the sequence is one maximal subpart
    }
  }
  return o;
}

// read_line into a String (server.rs:18-20): a line that is not valid UTF-8
// is an Err, and the reference shuts the connection down (server.rs:70-81)
bool valid_utf8_line(const std::string& in) {
  const unsigned char* s = (const unsigned char*)in.data();
  const size_t n = in.size();
  for (size_t i = 0; i < n;) {
    const unsigned c = s[i];
    if (c < 0x80) {
      ++i;
      continue;
    }
    size_t need;
    unsigned lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) need = 2, lo = 0xA0;
    else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) need = 2;
    else if (c == 0xED) need = 2, hi = 0x9F;
    else if (c == 0xF0) need = 3, lo = 0x90;
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) need = 3, hi = 0x8F;
    else return false;
    for (size_t k = 1; k <= need; ++k) {
      if (i + k >= n) return false;
      const unsigned b = s[i + k];
      if (k == 1 ? (b < lo || b > hi) : (b < 0x80 || b > 0xBF)) return false;
    }
    i += need + 1;
  }
  return true;
}

// Rust's char::is_whitespace (Unicode White_Space) at s[i] of a valid UTF-8
// string: returns the encoded length of the whitespace character, 0 if none
size_t ws_len(const std::string& s, size_t i) {
  const unsigned char c = (unsigned char)s[i];
  if (c == ' ' || (c >= 0x09 && c <= 0x0D)) return 1;
  if (c < 0xC2) return 0;
  const unsigned char c1 = i + 1 < s.size() ? (unsigned char)s[i + 1] : 0;
  if (c == 0xC2) return (c1 == 0x85 || c1 == 0xA0) ? 2 : 0;  // U+0085, U+00A0
  const unsigned char c2 = i + 2 < s.size() ? (unsigned char)s[i + 2] : 0;
  if (c == 0xE1) return (c1 == 0x9A && c2 == 0x80) ? 3 : 0;  // U+1680
  if (c == 0xE2 && c1 == 0x80) return ((c2 >= 0x80 && c2 <= 0x8A) || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF) ? 3 : 0;
  if (c == 0xE2 && c1 == 0x81) return c2 == 0x9F ? 3 : 0;    // U+205F
  if (c == 0xE3) return (c1 == 0x80 && c2 == 0x80) ? 3 : 0;  // U+3000
  return 0;
}

// split_whitespace (command.rs:17) on a valid UTF-8 line
std::vector<std::string> split_ws(const std::string& s) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < s.size()) {
    for (size_t w; i < s.size() && (w = ws_len(s, i)) != 0;) i += w;
    size_t j = i;
    while (j < s.size() && ws_len(s, j) == 0) ++j;
    if (j > i) out.push_back(s.substr(i, j - i));
    i = j;
  }
  return out;
}

// handle_client (server.rs:16-84); false ends the connection
bool handle_line(Db& db, const std::string& line, std::string* resp) {
  if (!valid_utf8_line(line)) return false;  // read_line's Err: the connection is shut down
  const std::vector<std::string> a = split_ws(line);
  if (a.empty()) {
    *resp = "Supported commands: get, insert, update, delete\n";
    return true;
  }
  const std::string& c = a[0];
  const bool known = c == "get" || c == "insert" || c == "update" || c == "delete";
  if (!known) {
    *resp = "Supported commands: get, insert, update, delete\n";
    return true;
  }
  const size_t need = (c == "insert" || c == "update") ? 3 : 2;
  if (a.size() < need) return false;  // the reference's args[i] panics its connection task
  if (c == "get") {
    std::string v;
    if (db.get(a[1], &v)) *resp = utf8_lossy(v) + "\n";
    else *resp = utf8_lossy(a[1]) + " not found\n";
    return true;
  }
  int rc = c == "delete" ? db.remove(a[1]) : db.insert(a[1], a[2]);
  if (rc) return false;  // db.*().await.unwrap() panics the task
  *resp = "ok\n";
  return true;
}

void serve_client(Db* db, int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  std::string buf, out;
  char tmp[65536];
  bool alive = true;
  while (alive) {
    ssize_t k = recv(fd, tmp, sizeof tmp, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) break;
    buf.append(tmp, (size_t)k);
    size_t start = 0;
    out.clear();
    for (size_t nl; (nl = buf.find('\n', start)) != std::string::npos; start = nl + 1) {
      std::string resp;
      if (!handle_line(*db, buf.substr(start, nl + 1 - start), &resp)) {
        alive = false;
        break;
      }
      out += resp;
    }
    buf.erase(0, start);
    if (!out.empty() && !write_all(fd, out.data(), out.size())) break;
  }
  close(fd);
}

}  // namespace

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);
  Config cfg;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> const char* {
      if (i + 1 >= argc) {
        fprintf(stderr, "missing value for %s\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--base") cfg.base = val();
    else if (a == "--port") cfg.port = atoi(val());
    else if (a == "--bind") cfg.bind = val();
    else if (a == "--device") cfg.device = atoi(val());
    else if (a == "--memtable-limit") cfg.memtable_limit = strtoull(val(), nullptr, 10);
    else if (a == "--compact-interval") cfg.compact_interval_ms = atol(val());
    else if (a == "--exit-after-load") cfg.exit_after_load = true;
    else if (a == "--index-threads") cfg.index_threads = atoi(val());
    else {
      fprintf(stderr, "usage: %s [--base DIR] [--port P] [--bind ADDR] [--device D] [--memtable-limit B] "
                      "[--compact-interval MS] [--exit-after-load] [--index-threads N]\n", argv[0]);
      return 2;
    }
  }
  Db db;
  db.cfg = cfg;
  db.ctx = lsmck_ctx_create(cfg.device);
  if (!db.ctx) {  // the batch paths have no CPU fallback
    fprintf(stderr, "lsmck_ctx_create(%d): %s\n", cfg.device, lsmck_last_error());
    return 1;
  }
  db.load();
  if (cfg.exit_after_load) {
    lsmck_ctx_destroy(db.ctx);
    return 0;
  }
  int ls = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  struct sockaddr_in sa;
  memset(&sa, 0, sizeof sa);
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)cfg.port);
  if (inet_pton(AF_INET, cfg.bind.c_str(), &sa.sin_addr) != 1 || bind(ls, (struct sockaddr*)&sa, sizeof sa) != 0 ||
      listen(ls, 128) != 0) {
    fprintf(stderr, "bind %s:%d: %s\n", cfg.bind.c_str(), cfg.port, strerror(errno));
    return 1;
  }
  socklen_t sl = sizeof sa;
  getsockname(ls, (struct sockaddr*)&sa, &sl);
  printf("{\"event\": \"listening\", \"port\": %d}\n", ntohs(sa.sin_port));
  fflush(stdout);
  if (cfg.compact_interval_ms > 0) std::thread(&Db::compact_loop, &db).detach();
  for (;;) {
    int fd = accept4(ls, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR || errno == ECONNABORTED) continue;
      break;
    }
    std::thread(serve_client, &db, fd).detach();
  }
  return 0;
}
