// lsmck_internal.h -- helpers shared by the host translation units of liblsmck.so.
#ifndef LSMCK_INTERNAL_H
#define LSMCK_INTERNAL_H
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace lsmck_host {
// thread-local error text; returns rc
int set_error(int rc, const char* msg);
int set_errno_error(int err, const char* what, const char* path);

// GF(2) arithmetic modulo the reflected CRC-32 polynomial (zlib conventions)
uint32_t gf2_mulmod(uint32_t a, uint32_t b);
uint32_t x_pow_8n(uint64_t n);
const uint32_t* crc_tables();  // [8][256] slicing tables, T0 first

// checksum_<ts>.db JSON (src/checksums.rs:13-17, 43-48, 75-79)
int write_checksum_json(const char* path, const char* index_b64, const char* data_b64);
int read_checksum_json(const char* path, std::string* index_b64, std::string* data_b64);

// metadata_<ts>.db JSON (src/sstable_metadata.rs:7-17, 76-83); id is validated, not kept
struct TableMeta {
  std::string base_path, metadata_filename, checksum_filename, data_filename, index_filename, bloom_filter_filename;
  std::string id;  // decimal u128
  unsigned level = 0;
};
int read_metadata_json(const char* path, TableMeta* m);
std::string path_push(const std::string& a, const std::string& b);

void gen_zipf_lengths(uint64_t seed, double s, int kmax, uint32_t lmin, uint64_t first, size_t n, uint32_t* out);
}  // namespace lsmck_host
#endif
