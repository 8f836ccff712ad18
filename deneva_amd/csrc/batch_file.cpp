// Versioned epoch batch files (.dccb), SURVEY.md §8(f) rank 2: the on-disk
// form of one captured epoch — the CSR access lists the reference keeps in
// TxnManager (system/txn.h:39-70), the per-txn timestamps OptCC reads
// (occ.cpp:142, worker_thread.cpp:500-502), the sequencer order for Calvin
// (sequencer.cpp:207) and, optionally, the decisions.  Capture (the host shim)
// and validation (the engine, the tests, the bench) meet at this format.
//
// Layout (little-endian, every section 8-byte aligned, in this order):
//   header   64 B   magic "DCCB", version, kind, section bits, n_txn, nnz,
//                   seed, epoch, tnc_before, FNV-1a 64 checksum (version 2:
//                   of the header's first 56 bytes and the payload; version
//                   1, still read: of the payload only)
//   offsets  u32[n_txn+1]
//   keys     u64[nnz]
//   acctype  u8[nnz]
//   start_tn, finish_tn  u64[n_txn] each        (DCC_FILE_HAS_TN)
//   order    u64[n_txn]                          (DCC_FILE_HAS_ORDER)
//   rc       u8[n_txn]                           (DCC_FILE_HAS_RC)
//   commit_tn u64[n_txn]                         (DCC_FILE_HAS_COMMIT_TN)
//   group    u32[nnz]                            (DCC_FILE_HAS_GROUP)
//   wave     u32[n_txn]                          (DCC_FILE_HAS_WAVE)
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <vector>

#include "dcc.h"

namespace {

constexpr uint32_t kMagic = 0x42434344u;  // "DCCB"

struct Header {
  uint32_t magic;
  uint16_t version;
  uint16_t kind;
  uint32_t sections;
  uint32_t header_bytes;
  uint64_t n_txn;
  uint64_t nnz;
  uint64_t seed;
  uint64_t epoch;
  uint64_t tnc_before;
  uint64_t checksum;
};
static_assert(sizeof(Header) == 64, "dccb header is 64 bytes");

struct Fnv {
  uint64_t h = 1469598103934665603ull;
  void add(const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; i++) {
      h ^= b[i];
      h *= 1099511628211ull;
    }
  }
};

size_t pad8(size_t n) { return (n + 7) & ~(size_t)7; }

struct Section {
  const void* src;
  void* dst;
  size_t bytes;
};

// The section list of a file, in order (sources for writing, destinations
// for reading; either may be null).
std::vector<Section> sections(uint32_t bits, uint64_t n, uint64_t nnz, const void* const* src,
                              void* const* dst) {
  std::vector<Section> v;
  auto add = [&](int idx, size_t bytes) {
    v.push_back(Section{src ? src[idx] : nullptr, dst ? dst[idx] : nullptr, bytes});
  };
  add(0, (n + 1) * 4);
  add(1, nnz * 8);
  add(2, nnz);
  if (bits & DCC_FILE_HAS_TN) {
    add(3, n * 8);
    add(4, n * 8);
  }
  if (bits & DCC_FILE_HAS_ORDER) add(5, n * 8);
  if (bits & DCC_FILE_HAS_RC) add(6, n);
  if (bits & DCC_FILE_HAS_COMMIT_TN) add(7, n * 8);
  if (bits & DCC_FILE_HAS_GROUP) add(8, nnz * 4);
  if (bits & DCC_FILE_HAS_WAVE) add(9, n * 4);
  return v;
}

constexpr uint32_t kKnownSections = DCC_FILE_HAS_TN | DCC_FILE_HAS_ORDER | DCC_FILE_HAS_RC |
                                    DCC_FILE_HAS_COMMIT_TN | DCC_FILE_HAS_GROUP | DCC_FILE_HAS_WAVE;

int read_header(FILE* f, Header& h) {
  if (fread(&h, sizeof h, 1, f) != 1) return DCC_EINVAL;
  if (h.magic != kMagic || h.header_bytes != sizeof(Header)) return DCC_EINVAL;
  if (h.version != 1 && h.version != DCC_FILE_VERSION) return DCC_ENOTSUP;
  if (h.kind > DCC_FILE_CALVIN || (h.sections & ~kKnownSections)) return DCC_EINVAL;
  if (h.nnz >= 0xFFFFFFFFull || h.n_txn >= 0xFFFFFFFFull) return DCC_ERANGE;
  return DCC_OK;
}

// the checksum's start: version 2 covers the header (all but its checksum)
void checksum_header(Fnv& fnv, const Header& h) {
  if (h.version >= 2) fnv.add(&h, offsetof(Header, checksum));
}

}  // namespace

extern "C" int dcc_file_write(const char* path, const dcc_file_info* info, const dcc_batch* b,
                              const uint8_t* rc, const uint64_t* commit_tn, const uint32_t* group,
                              const uint32_t* wave) {
  if (!path || !info || !b || (b->flags & DCC_DEVICE_PTRS)) return DCC_EINVAL;
  // the file holds the full-width form (u64 keys and timestamps, one access
  // type per byte): a compact batch must be widened by the caller first
  if (b->flags & DCC_COMPACT_FLAGS) return DCC_EINVAL;
  if (b->n_txn && !b->offsets) return DCC_EINVAL;
  const uint64_t n = b->n_txn, nnz = b->nnz;
  if (n && (b->offsets[0] != 0 || b->offsets[n] != nnz)) return DCC_EINVAL;
  uint32_t bits = 0;
  if (b->start_tn && b->finish_tn) bits |= DCC_FILE_HAS_TN;
  if (b->order) bits |= DCC_FILE_HAS_ORDER;
  if (rc) bits |= DCC_FILE_HAS_RC;
  if (commit_tn) bits |= DCC_FILE_HAS_COMMIT_TN;
  if (group) bits |= DCC_FILE_HAS_GROUP;
  if (wave) bits |= DCC_FILE_HAS_WAVE;
  static const uint32_t zero_off = 0;
  const void* src[10] = {n ? (const void*)b->offsets : (const void*)&zero_off,
                         b->keys, b->acctype, b->start_tn, b->finish_tn, b->order,
                         rc, commit_tn, group, wave};
  const std::vector<Section> secs = sections(bits, n, nnz, src, nullptr);
  static const uint8_t zeros[8] = {0};
  for (const Section& s : secs)
    if (s.bytes && !s.src) return DCC_EINVAL;
  Header h{};
  h.magic = kMagic;
  h.version = DCC_FILE_VERSION;
  h.kind = (uint16_t)info->kind;
  h.sections = bits;
  h.header_bytes = sizeof(Header);
  h.n_txn = n;
  h.nnz = nnz;
  h.seed = info->seed;
  h.epoch = info->epoch;
  h.tnc_before = info->tnc_before;
  Fnv fnv;
  checksum_header(fnv, h);
  for (const Section& s : secs) {
    fnv.add(s.src, s.bytes);
    fnv.add(zeros, pad8(s.bytes) - s.bytes);
  }
  h.checksum = fnv.h;
  FILE* f = fopen(path, "wb");
  if (!f) return DCC_EIO;
  bool ok = fwrite(&h, sizeof h, 1, f) == 1;
  for (const Section& s : secs) {
    if (!ok) break;
    if (s.bytes) ok = fwrite(s.src, 1, s.bytes, f) == s.bytes;
    const size_t p = pad8(s.bytes) - s.bytes;
    if (ok && p) ok = fwrite(zeros, 1, p, f) == p;
  }
  if (fclose(f) != 0) ok = false;
  return ok ? DCC_OK : DCC_EIO;
}

extern "C" int dcc_file_read_info(const char* path, dcc_file_info* info) {
  if (!path || !info) return DCC_EINVAL;
  FILE* f = fopen(path, "rb");
  if (!f) return DCC_EIO;
  Header h;
  const int r = read_header(f, h);
  fclose(f);
  if (r != DCC_OK) return r;
  info->version = h.version;
  info->kind = h.kind;
  info->sections = h.sections;
  info->reserved = 0;
  info->n_txn = h.n_txn;
  info->nnz = h.nnz;
  info->seed = h.seed;
  info->epoch = h.epoch;
  info->tnc_before = h.tnc_before;
  return DCC_OK;
}

extern "C" int dcc_file_read(const char* path, uint32_t* offsets, uint64_t* keys,
                             uint8_t* acctype, uint64_t* start_tn, uint64_t* finish_tn,
                             uint64_t* order, uint8_t* rc, uint64_t* commit_tn, uint32_t* group,
                             uint32_t* wave) {
  if (!path) return DCC_EINVAL;
  FILE* f = fopen(path, "rb");
  if (!f) return DCC_EIO;
  Header h;
  int r = read_header(f, h);
  if (r != DCC_OK) {
    fclose(f);
    return r;
  }
  void* dst[10] = {offsets, keys, acctype, start_tn, finish_tn, order, rc, commit_tn, group, wave};
  const std::vector<Section> secs = sections(h.sections, h.n_txn, h.nnz, nullptr, dst);
  Fnv fnv;
  checksum_header(fnv, h);
  std::vector<uint8_t> buf;
  r = DCC_OK;
  for (const Section& s : secs) {
    const size_t total = pad8(s.bytes);
    buf.resize(total);
    if (total && fread(buf.data(), 1, total, f) != total) {
      r = DCC_EINVAL;  // truncated
      break;
    }
    fnv.add(buf.data(), total);
    if (s.dst && s.bytes) memcpy(s.dst, buf.data(), s.bytes);
  }
  if (r == DCC_OK && fgetc(f) != EOF) r = DCC_EINVAL;  // trailing bytes
  fclose(f);
  if (r != DCC_OK) return r;
  if (fnv.h != h.checksum) return DCC_EINVAL;  // corrupted payload
  if (offsets && h.n_txn) {
    if (offsets[0] != 0 || offsets[h.n_txn] != h.nnz) return DCC_EINVAL;
    for (uint64_t t = 0; t < h.n_txn; t++)
      if (offsets[t + 1] < offsets[t]) return DCC_EINVAL;
  }
  return DCC_OK;
}
