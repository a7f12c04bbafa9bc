// tario.cpp — host-side shard ingest feeding the device path.
//
// * dino_tar_index: one pass over a WebDataset tar shard held in memory (an mmap of
//   the /dev/shm shard-cache file, reference shard_cache.py:584-609), grouping the
//   members into samples by key and reporting where each sample's JPEG and JSON
//   sidecar bytes lie.  It replaces the per-member Python work of the reference's
//   extraction worker (hpc_source.py:405-478, which calls the absent
//   dino_loader.datasets.utils._extract_jpegs_with_meta on memoryview(data) and then
//   copies every JPEG with bytes(mv)).
// * dino_gather: packs a batch's JPEG byte ranges (from any number of mapped shards)
//   into one pinned host buffer + int64 offsets[B+1] with a few threads, ready for a
//   single H2D copy (the packed layout dino_run_batch reads).
//
// Tar semantics follow Python's tarfile (POSIX ustar, GNU 'L' long names, pax 'x'
// path/size records, base-256 sizes, header checksum): a bad header at offset 0 is
// an error, a bad header later ends the archive, a member whose data runs past the
// buffer ends it with a truncation status.  Sample grouping follows WebDataset's
// base_plus_ext + group_by_keys: key = path up to the first '.' of the basename,
// extension = the rest, lower-cased; consecutive members with one key form a sample.
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dino_ingest.h"
#include "hostcopy.hpp"

namespace {

thread_local std::string g_tar_err;

int tar_fail(int code, const std::string& msg) {
  g_tar_err = msg;
  return code;
}

bool is_zero_block(const uint8_t* h) {
  for (int i = 0; i < 512; ++i)
    if (h[i]) return false;
  return true;
}

// tarfile.nti: octal (NUL/space padded) or GNU base-256 (first byte 0x80 / 0xFF).
bool parse_number(const uint8_t* f, int n, int64_t* out) {
  if (f[0] == 0x80 || f[0] == 0xFF) {
    // base-256: a value needing more than 63 bits (or a negative one) is rejected
    // instead of wrapping; tar sizes and checksums are never that large
    if (f[0] == 0xFF) return false;
    uint64_t v = 0;
    for (int i = 1; i < n; ++i) {
      if (v >> 55) return false;
      v = (v << 8) | f[i];
    }
    *out = (int64_t)v;
    return true;
  }
  int i = 0;
  while (i < n && (f[i] == ' ' || f[i] == 0)) ++i;  // leading padding
  int64_t v = 0;
  bool any = false;
  for (; i < n && f[i] >= '0' && f[i] <= '7'; ++i) {
    if (v >> 59) return false;
    v = v * 8 + (f[i] - '0');
    any = true;
  }
  for (; i < n; ++i)
    if (f[i] != ' ' && f[i] != 0) return false;
  *out = any ? v : 0;
  return true;
}

bool checksum_ok(const uint8_t* h) {
  int64_t stored;
  if (!parse_number(h + 148, 8, &stored)) return false;
  uint32_t u = 0;
  int32_t s = 0;
  for (int i = 0; i < 512; ++i) {
    const uint8_t b = (i >= 148 && i < 156) ? (uint8_t)' ' : h[i];
    u += b;
    s += (int8_t)b;
  }
  return stored == (int64_t)u || stored == (int64_t)s;
}

std::string cstr(const uint8_t* f, int n) {
  int l = 0;
  while (l < n && f[l]) ++l;
  return std::string((const char*)f, (size_t)l);
}

// pax records "len key=value\n": returns path / size overrides.
void parse_pax(const uint8_t* p, int64_t n, std::string* path, int64_t* size) {
  int64_t i = 0;
  while (i < n) {
    int64_t len = 0, j = i;
    while (j < n && p[j] >= '0' && p[j] <= '9') len = len * 10 + (p[j++] - '0');
    if (j >= n || p[j] != ' ' || len <= 0 || i + len > n) return;
    const std::string rec((const char*)p + j + 1, (size_t)(i + len - j - 1));
    const size_t eq = rec.find('=');
    if (eq != std::string::npos) {
      std::string key = rec.substr(0, eq), val = rec.substr(eq + 1);
      if (!val.empty() && val.back() == '\n') val.pop_back();
      if (key == "path") *path = val;
      if (key == "size") {
        // a size that is not a plain non-negative decimal below 2^62 is ignored
        int64_t v = 0;
        bool okv = !val.empty() && val.size() <= 18;
        for (char ch : val) okv = okv && ch >= '0' && ch <= '9';
        if (okv) {
          for (char ch : val) v = v * 10 + (ch - '0');
          *size = v;
        }
      }
    }
    i += len;
  }
}

// WebDataset base_plus_ext: ^((?:.*/|)[^.]+)[.]([^/]*)$
bool split_key(const std::string& name, std::string* key, std::string* ext) {
  const size_t slash = name.rfind('/');
  const size_t b0 = slash == std::string::npos ? 0 : slash + 1;
  const size_t dot = name.find('.', b0);
  if (dot == std::string::npos || dot == b0) return false;
  *key = name.substr(0, dot);
  *ext = name.substr(dot + 1);
  for (auto& ch : *ext) ch = (char)std::tolower((unsigned char)ch);
  return true;
}

// The tar walk over any byte source.  Src::at(pos, n): a pointer to n bytes at pos (n <=
// the bytes left), valid until the next call.  Memory: the mapped shard itself; file
// (dino_tar_index_fd): pread of the 512-byte headers and of pax / long-name data only, so that
// an index never touches (faults in) the members' data.
struct MemSrc {
  const uint8_t* tar;
  const uint8_t* at(int64_t pos, int64_t) { return tar + pos; }
};
struct FdSrc {
  int fd;
  int64_t base;
  std::vector<uint8_t> buf;
  bool ok = true;
  const uint8_t* at(int64_t pos, int64_t n) {
    if ((int64_t)buf.size() < n) buf.resize((size_t)n);
    int64_t got = 0;
    while (got < n) {
      const ssize_t r = pread(fd, buf.data() + got, (size_t)(n - got), (off_t)(base + pos + got));
      if (r <= 0) {
        ok = false;
        memset(buf.data() + got, 0, (size_t)(n - got));  // read as an end-of-archive block
        break;
      }
      got += r;
    }
    return buf.data();
  }
};

template <typename Src>
int tar_index(Src& src, int64_t len, dino_tar_sample* out, int64_t cap, char* keys, int64_t keys_cap,
              int64_t* n_samples, int64_t* n_members) {
  *n_samples = 0;
  if (n_members) *n_members = 0;
  int64_t pos = 0, ns = 0, nm = 0, kpos = 0;
  int status = DINO_OK;
  std::string long_name, pax_path, cur_key;
  int64_t pax_size = -1;
  bool have_cur = false;
  dino_tar_sample cur{};
  auto flush = [&]() -> int {
    if (!have_cur) return DINO_OK;
    have_cur = false;
    if (cur.img_off < 0) return DINO_OK;  // a sample without an image is skipped
    if (ns >= cap) return tar_fail(DINO_ERANGE, "dino_tar_index: sample capacity exceeded");
    const int64_t kl = (int64_t)cur_key.size();
    if (keys && kpos + kl <= keys_cap) {
      memcpy(keys + kpos, cur_key.data(), (size_t)kl);
      cur.key_off = kpos;
      cur.key_len = (int32_t)kl;
      kpos += kl;
    } else {
      cur.key_off = -1;
      cur.key_len = (int32_t)kl;
    }
    out[ns++] = cur;
    return DINO_OK;
  };
  uint8_t h[512];
  while (pos + 512 <= len) {
    memcpy(h, src.at(pos, 512), 512);
    if (is_zero_block(h)) break;  // end-of-archive marker
    if (!checksum_ok(h)) {
      if (pos == 0) return tar_fail(DINO_EFORMAT, "dino_tar_index: invalid tar header at offset 0");
      status = DINO_TAR_BAD_HEADER;  // tarfile stops iterating silently
      break;
    }
    int64_t size;
    if (!parse_number(h + 124, 12, &size) || size < 0) {
      if (pos == 0) return tar_fail(DINO_EFORMAT, "dino_tar_index: invalid size field at offset 0");
      status = DINO_TAR_BAD_HEADER;
      break;
    }
    const char type = (char)h[156];
    if (pax_size >= 0 && type != 'x' && type != 'g' && type != 'L' && type != 'K') size = pax_size;
    const int64_t data = pos + 512;
    if (size > len - data) {  // (no overflow: 0 <= size, data <= len)
      status = DINO_TAR_TRUNCATED;
      break;
    }
    const int64_t next = data + ((size + 511) / 512) * 512;
    if (type == 'L') {
      const int64_t n = std::min<int64_t>(size, 1 << 20);
      long_name = cstr(src.at(data, n), (int)n);
    } else if (type == 'x') {
      parse_pax(src.at(data, size), size, &pax_path, &pax_size);
    } else if (type == 'g' || type == 'K') {
      // global pax header / GNU long link name: nothing per member
    } else {
      std::string name;
      if (!long_name.empty()) {
        name = long_name;
      } else if (!pax_path.empty()) {
        name = pax_path;
      } else {
        name = cstr(h, 100);
        if (memcmp(h + 257, "ustar", 5) == 0) {
          const std::string prefix = cstr(h + 345, 155);
          if (!prefix.empty()) name = prefix + "/" + name;
        }
      }
      long_name.clear();
      pax_path.clear();
      pax_size = -1;
      if (type == '0' || type == '\0' || type == '7') {
        ++nm;
        std::string key, ext;
        if (split_key(name, &key, &ext)) {
          if (!have_cur || key != cur_key) {
            const int e = flush();
            if (e) return e;
            cur_key = key;
            cur = dino_tar_sample{-1, 0, -1, 0, -1, 0, 0};
            have_cur = true;
          }
          if (ext == "jpg" || ext == "jpeg") {
            cur.img_off = data;
            cur.img_len = size;
          } else if (ext == "json") {
            cur.meta_off = data;
            cur.meta_len = size;
          }
        }
      }
    }
    pos = next;
  }
  const int e = flush();
  if (e) return e;
  *n_samples = ns;
  if (n_members) *n_members = nm;
  if (status != DINO_OK) g_tar_err = status == DINO_TAR_TRUNCATED ? "truncated member" : "bad header after offset 0";
  return status;
}

}  // namespace

extern "C" {

const char* dino_tar_last_error(void) { return g_tar_err.c_str(); }

int dino_tar_index(const uint8_t* tar, int64_t len, dino_tar_sample* out, int64_t cap, char* keys, int64_t keys_cap,
                   int64_t* n_samples, int64_t* n_members) {
  if ((!tar && len > 0) || len < 0 || !n_samples || (cap > 0 && !out)) return tar_fail(DINO_EINVAL, "dino_tar_index: bad args");
  MemSrc src{tar};
  return tar_index(src, len, out, cap, keys, keys_cap, n_samples, n_members);
}

int dino_tar_index_fd(int32_t fd, int64_t base, int64_t len, dino_tar_sample* out, int64_t cap, char* keys,
                      int64_t keys_cap, int64_t* n_samples, int64_t* n_members) {
  if (fd < 0 || base < 0 || len < 0 || !n_samples || (cap > 0 && !out)) return tar_fail(DINO_EINVAL, "dino_tar_index_fd: bad args");
  FdSrc src{fd, base, {}};
  const int rc = tar_index(src, len, out, cap, keys, keys_cap, n_samples, n_members);
  if (!src.ok && rc >= 0) return tar_fail(DINO_EFORMAT, "dino_tar_index_fd: read error");
  return rc;
}

int dino_gather(const uint64_t* src_ptrs, const int64_t* lens, int64_t n, uint8_t* dst, int64_t dst_cap,
                int64_t* dst_offsets, int32_t nthreads) {
  if (n < 0 || (n > 0 && (!src_ptrs || !lens || !dst)) || !dst_offsets)
    return tar_fail(DINO_EINVAL, "dino_gather: bad args");
  dst_offsets[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (lens[i] < 0) return tar_fail(DINO_EINVAL, "dino_gather: negative length");
    dst_offsets[i + 1] = dst_offsets[i] + lens[i];
  }
  if (dst_offsets[n] > dst_cap) return tar_fail(DINO_ERANGE, "dino_gather: destination too small");
  const int64_t total = dst_offsets[n];
  int nt = nthreads > 0 ? nthreads : 1;
  if (total < ((int64_t)1 << 20)) nt = 1;
  nt = (int)std::min<int64_t>(nt, std::max<int64_t>(n, 1));
  // split by bytes: thread k copies the images whose start lies in [k*total/nt, (k+1)*total/nt)
  auto work = [&](int k) {
    const int64_t lo = total * k / nt, hi = total * (k + 1) / nt;
    int64_t i = std::upper_bound(dst_offsets, dst_offsets + n + 1, lo) - dst_offsets - 1;
    if (i < 0) i = 0;
    if (k > 0 && dst_offsets[i] < lo) ++i;
    for (; i < n && dst_offsets[i] < hi; ++i)
      if (lens[i]) dino::stream_copy(dst + dst_offsets[i], (const uint8_t*)(uintptr_t)src_ptrs[i], lens[i]);
    dino::stream_fence();
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    for (int k = 1; k < nt; ++k) th.emplace_back(work, k);
    work(0);
    for (auto& t : th) t.join();
  }
  return DINO_OK;
}

}  // extern "C"
