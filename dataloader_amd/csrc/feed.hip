// feed.hip — the native host half of the /dev/shm shard feed (dino_feed_*).
//
// Replaces, for the device backend, the per-batch Python work between the node-local
// shard cache and Stage 3: reference ShardIterator / MixingSource
// (sources/hpc_source.py:329-385 I/O + :405-478 extraction, bytes(mv) copies at :360) and
// _ReaderAdapter.__call__ (shard_reader.py:346-376) hand Stage 3 a Python list of JPEG
// arrays per batch; here a batch never becomes Python objects:
//
//   opener threads  mmap a shard-cache file ([data_len:u64][magic:u64] + tar, reference
//                   shard_cache.py:83-85, 584-609), index the tar
//                   (dino_tar_index), up to `lookahead` shards ahead of the packer; one
//                   thread per shard of the look-ahead (at most kMaxOpeners), so that two
//                   shards' page population overlaps (measured at 8 ranks per node: the
//                   single opener held a feed to 0.82-0.9x the device rate);
//                   the shards reach the packer in push order whatever order they finish in;
//   packer thread   takes the next B samples (a batch may straddle shards; the last partial
//                   batch of an epoch is dropped, dali_backend.py:187), packs them into a
//                   pinned slot with `nthreads` copier threads and probes each image right
//                   after its copy (status, kind, workspace bytes), hands consumed shards to
//                   the openers, which unmap them outside the feed's lock;
//   caller          dino_feed_next (blocks with the GIL released: ctypes), then
//                   dino_feed_copy (H2D of the slot on the caller's stream; the slot returns
//                   to the packer when that copy retires) or dino_feed_release.
//
// All of it runs without the Python interpreter, so the host half no longer waits for the
// GIL behind the thread that launches the kernels (measured: the same pack + probe work
// took 0.9 ms per 512-image batch alone and 16 ms next to a Python-busy thread).
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <stdio.h>
#include <string.h>
#include <sys/inotify.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dino_ingest.h"
#include "hostcopy.hpp"
#include "probe.hpp"

using namespace dino;

namespace {

thread_local std::string g_feed_err;

int feed_fail(int code, const std::string& msg) {
  g_feed_err = msg;
  return code;
}

constexpr uint64_t kShardMagic = 0xDEADBEEFCAFEF00Dull;
constexpr int kMaxOpeners = 4;
#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// How the feed reads a shard-cache file (DINO_FEED_IO):
//   "mmap" (default)  index and copies over a mapping of the file;
//   "index"           the tar index reads only the 512-byte headers (dino_tar_index_fd: the
//                     openers never fault a shard in), copies from the mapping;
//   "pread"           header-only index, and the copier threads pread each JPEG straight into
//                     the pinned slot (no mapping: no faults, no unmap per shard).
// At 8 ranks on one node (scripts/gpu_host_feed.sh, profiles/r06_host/): the openers' time fell
// 6.3 -> 3.2 (index) / 2.2 s (pread) of 8, but the slowest feed stayed 108-109k (index) or fell
// to 100-105k img/s (pread) against 107-115k (mmap): the node's copy bandwidth, not the
// openers, bounds 8 feeds (~85 GB/s of /dev/shm reads in all).
enum FeedIo { kIoMmap = 0, kIoIndex = 1, kIoPread = 2 };
FeedIo feed_io_mode() {
  static const FeedIo m = [] {
    const char* e = getenv("DINO_FEED_IO");
    if (e && !strcmp(e, "pread")) return kIoPread;
    return e && !strcmp(e, "index") ? kIoIndex : kIoMmap;
  }();
  return m;
}

struct Shard {
  std::string path;
  void* map = nullptr;
  size_t map_len = 0;
  int fd = -1;       // pread mode: the file stays open while its samples are packed
  const uint8_t* tar = nullptr;
  int64_t tar_len = 0;
  std::vector<dino_tar_sample> samples;
  size_t next = 0;   // next sample the packer takes
  ~Shard() {
    if (map) munmap(map, map_len);
    if (fd >= 0) close(fd);
  }
};

// The reference's _is_ready (shard_cache.py:331-340): the file exists and its header carries
// the ready magic (written last by the node master, then tmp -> rename, :689-703).
bool shard_ready(const std::string& path) {
  const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  uint64_t hdr[2] = {0, 0};
  const ssize_t n = pread(fd, hdr, sizeof hdr, 0);
  close(fd);
  return n == (ssize_t)sizeof hdr && hdr[1] == kShardMagic;
}

// A non-master rank's wait for the node master's write (reference _inotify_wait,
// shard_cache.py:373-449): check, watch the cache directory for IN_CLOSE_WRITE | IN_MOVED_TO,
// check again (the rename may land between the check and the watch), then wake on events
// until the file is ready or the timeout passes; stat-polls every 50 ms where inotify is
// unavailable.  Wakes at least every 100 ms to observe `cancelled` (feed reset / destroy).
// "" when ready, else the reason.
std::string wait_shard(const std::string& path, int32_t timeout_ms, const std::function<bool()>& cancelled) {
  if (shard_ready(path)) return "";
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  const size_t slash = path.rfind('/');
  const std::string dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : path.substr(0, slash));
  int ifd = inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
  int wd = ifd >= 0 ? inotify_add_watch(ifd, dir.c_str(), IN_CLOSE_WRITE | IN_MOVED_TO) : -1;
  std::string err;
  for (;;) {
    if (shard_ready(path)) break;
    if (cancelled()) {
      err = "shard " + path + ": wait cancelled";
      break;
    }
    const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now());
    if (left.count() <= 0) {
      char t[64];
      snprintf(t, sizeof t, "%.0f", timeout_ms / 1000.0);
      err = std::string("Timed out (") + t + "s) waiting for shard: " + path;
      break;
    }
    if (wd >= 0) {
      struct pollfd pf = {ifd, POLLIN, 0};
      if (poll(&pf, 1, (int)std::min<int64_t>(left.count(), 100)) > 0) {
        char buf[4096];
        while (read(ifd, buf, sizeof buf) > 0) {
        }
      }
    } else {
      usleep((useconds_t)std::min<int64_t>(left.count(), 50) * 1000);
    }
  }
  if (wd >= 0) inotify_rm_watch(ifd, wd);
  if (ifd >= 0) close(ifd);
  return err;
}

// Seeded in-shard sample order (the shuffle buffer of the extraction step, reference
// hpc_source.py:461-467 -> _extract_jpegs_with_meta(shuffle_buffer=512, rng)): Fisher-Yates
// over the shard's samples, keyed by (seed, epoch, shard path) with splitmix64.
uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
void shuffle_samples(std::vector<dino_tar_sample>& v, uint64_t seed, uint64_t epoch, const std::string& path) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a of the path
  for (unsigned char c : path) h = (h ^ c) * 1099511628211ull;
  uint64_t st = seed ^ (epoch * 0xD1B54A32D192ED03ull) ^ h;
  for (size_t i = v.size(); i > 1; --i) {
    const size_t j = (size_t)(splitmix64(st) % i);
    std::swap(v[i - 1], v[j]);
  }
}

// Opens and indexes one shard-cache file (feed_io_mode); "" on success, else the reason.
std::string open_shard(Shard& s) {
  const int fd = open(s.path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return "open " + s.path + ": " + strerror(errno);
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < 16) {
    close(fd);
    return "shard " + s.path + ": too short";
  }
  const FeedIo io = feed_io_mode();
  if (io != kIoMmap) {
    uint64_t hdr[2] = {0, 0};
    if (pread(fd, hdr, 16, 0) != 16 || hdr[1] != kShardMagic) {
      close(fd);
      return "shard " + s.path + ": corrupt header (not ready)";  // reference shard_cache.py:331-340
    }
    if ((int64_t)hdr[0] > st.st_size - 16) {
      close(fd);
      return "shard " + s.path + ": data length past the file";
    }
    s.tar_len = (int64_t)hdr[0];
    const int64_t cap = s.tar_len / 1024 + 16;  // a sample's member takes >= 1024 bytes
    s.samples.resize((size_t)cap);
    int64_t ns = 0, nm = 0;
    const int rc = dino_tar_index_fd(fd, 16, s.tar_len, s.samples.data(), cap, nullptr, 0, &ns, &nm);
    if (rc < 0) {
      close(fd);
      return "shard " + s.path + ": " + dino_tar_last_error();
    }
    s.samples.resize((size_t)ns);
    if (io == kIoPread) {
      s.fd = fd;
      return "";
    }
    void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);  // copies fault it in
    close(fd);
    if (m == MAP_FAILED) return "mmap " + s.path + ": " + strerror(errno);
    s.map = m;
    s.map_len = (size_t)st.st_size;
    s.tar = (const uint8_t*)m + 16;
    return "";
  }
  void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return "mmap " + s.path + ": " + strerror(errno);
  s.map = m;
  s.map_len = (size_t)st.st_size;
  uint64_t hdr[2];
  memcpy(hdr, m, 16);
  if (hdr[1] != kShardMagic) return "shard " + s.path + ": corrupt header (not ready)";  // reference shard_cache.py:331-340
  if ((int64_t)hdr[0] > st.st_size - 16) return "shard " + s.path + ": data length past the file";
  s.tar = (const uint8_t*)m + 16;
  s.tar_len = (int64_t)hdr[0];
  // No pre-fault by default: the copier threads fault the pages in as they pack (the kernel
  // maps 16 pages per fault around the address), spread over `nthreads` threads, where the
  // openers' MADV_POPULATE_READ of every page of a shard made them the feed's bottleneck
  // (e2e, same box, alternated: 151.0k / 172.0k / 168.9k img/s with it, 173.5k / 174.3k /
  // 175.4k without; scripts/populate_study.sh).  DINO_FEED_POPULATE=1 restores it.
  static const bool populate = getenv("DINO_FEED_POPULATE") && getenv("DINO_FEED_POPULATE")[0] == '1';
  if (populate && madvise(m, s.map_len, MADV_POPULATE_READ) != 0) {  // Linux >= 5.14; else touch every page
    volatile uint8_t sink = 0;
    for (size_t o = 0; o < s.map_len; o += 4096) sink ^= ((const uint8_t*)m)[o];
    (void)sink;
  }
  const int64_t cap = s.tar_len / 1024 + 16;  // a sample's member takes >= 1024 bytes
  s.samples.resize((size_t)cap);
  int64_t ns = 0, nm = 0;
  const int rc = dino_tar_index(s.tar, s.tar_len, s.samples.data(), cap, nullptr, 0, &ns, &nm);
  if (rc < 0) return "shard " + s.path + ": " + dino_tar_last_error();
  s.samples.resize((size_t)ns);  // a truncated / bad later header keeps the samples before it (tarfile)
  return "";
}

// Persistent copier threads: thread k packs + probes images [first(k), first(k+1)).
class CopyPool {
 public:
  explicit CopyPool(int n) : n_(std::max(1, n)), ws_(n_), aws_(n_) {
    for (int k = 1; k < n_; ++k) th_.emplace_back([this, k] { loop(k); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // Pack n images into dst at offs (offs[n] = total) and probe them; returns ws / aws sums.
  // fds (nullable): image i is read with pread(fds[i], ..., offset ptrs[i]) instead of copied
  // from address ptrs[i]
  void run(const uint64_t* ptrs, const int32_t* fds, const int64_t* lens, const int64_t* offs, int32_t n, uint8_t* dst,
           int32_t max_dim, const dino_aug_config* cfg, int32_t* info, int64_t* ws, int64_t* aws) {
    {
      std::lock_guard<std::mutex> g(m_);
      ptrs_ = ptrs, fds_ = fds, lens_ = lens, offs_ = offs, n_img_ = n, dst_ = dst, max_dim_ = max_dim, cfg_ = cfg,
      info_ = info;
      left_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    part(0);
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [this] { return left_ == 0; });
    int64_t w = 0, a = 0;
    for (int k = 0; k < n_; ++k) w += ws_[k], a += aws_[k];
    *ws = w;
    *aws = a;
  }

 private:
  void loop(int k) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      part(k);
      {
        std::lock_guard<std::mutex> g(m_);
        --left_;
      }
      done_cv_.notify_one();
    }
  }
  void part(int k) {
    std::vector<ScanRec>& scans = scans_[k % kScanSets];
    if (scans.empty()) scans.resize(kMaxScans);
    const int64_t total = offs_[n_img_];
    auto first = [&](int j) -> int32_t {
      if (j <= 0) return 0;
      if (j >= n_) return n_img_;
      return (int32_t)(std::lower_bound(offs_, offs_ + n_img_, total * j / n_) - offs_);
    };
    int64_t w = 0, a = 0;
    for (int32_t i = first(k), e = first(k + 1); i < e; ++i) {
      int64_t len = lens_[i];
      if (fds_) {  // pread into the slot, then probe the slot's copy
        int64_t got = 0;
        while (got < len) {
          const ssize_t r = pread(fds_[i], dst_ + offs_[i] + got, (size_t)(len - got), (off_t)(ptrs_[i] + got));
          if (r <= 0) break;
          got += r;
        }
        if (got < len) memset(dst_ + offs_[i] + got, 0, (size_t)(len - got));  // (a shard truncated under us)
        probe_one(dst_ + offs_[i], len, false, max_dim_, cfg_, scans.data(), info_ + 4 * i, &w, &a);
        continue;
      }
      const uint8_t* src = (const uint8_t*)(uintptr_t)ptrs_[i];
      if (len) stream_copy(dst_ + offs_[i], src, len);
      probe_one(src, len, false, max_dim_, cfg_, scans.data(), info_ + 4 * i, &w, &a);
    }
    stream_fence();
    ws_[k] = w;
    aws_[k] = a;
  }
  static constexpr int kScanSets = 64;
  int n_;
  std::vector<int64_t> ws_, aws_;
  std::vector<std::thread> th_;
  std::vector<ScanRec> scans_[kScanSets];
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  uint64_t gen_ = 0;
  bool stop_ = false;
  int left_ = 0;
  const uint64_t* ptrs_ = nullptr;
  const int32_t* fds_ = nullptr;
  const int64_t* lens_ = nullptr;
  const int64_t* offs_ = nullptr;
  int32_t n_img_ = 0;
  uint8_t* dst_ = nullptr;
  int32_t max_dim_ = 0;
  const dino_aug_config* cfg_ = nullptr;
  int32_t* info_ = nullptr;
};

enum SlotState { kFree = 0, kFilling, kReady, kHanded, kCopying };

struct Slot {
  SlotState state = kFree;
  uint8_t* host = nullptr;  // pinned (hipHostMalloc)
  int64_t cap = 0;
  int64_t nbytes = 0;
  std::vector<int64_t> offs;
  int64_t* offs_pinned = nullptr;  // offsets for the H2D copy
  std::vector<int32_t> info;
  int64_t ws = 0, aws = 0, seq = -1;
  hipEvent_t ev = nullptr;
};

}  // namespace

// Slot memory: pinned (hipHostMalloc) on a GPU host; plain memory where there is no device
// (the packing / epoch logic then runs and is tested on CPU; dino_feed_copy refuses).
void* slot_alloc(bool gpu, size_t n) {
  void* p = nullptr;
  if (gpu) return hipHostMalloc(&p, n, hipHostMallocDefault) == hipSuccess ? p : nullptr;
  return aligned_alloc(64, (n + 63) & ~(size_t)63);
}
void slot_free(bool gpu, void* p) {
  if (!p) return;
  if (gpu) (void)hipHostFree(p);
  else free(p);
}

struct dino_feed {
  bool gpu = true;
  int32_t batch = 0, max_dim = 0, lookahead = 2;
  dino_aug_config cfg{};
  bool have_cfg = false;
  int32_t wait_ms = 0;                 // > 0: wait that long for a shard the node master has not written yet
  bool shuffle = false;                // seeded in-shard sample order
  uint64_t shuffle_seed = 0;
  uint64_t epoch = 0;                  // the shuffle key: epochs since create, or dino_feed_set_epoch's
  std::unique_ptr<CopyPool> pool;
  std::vector<Slot> slots;
  std::mutex m;
  std::condition_variable cv;          // any state change
  std::deque<std::string> pending;     // paths pushed, not yet opened
  std::deque<std::shared_ptr<Shard>> opened;  // opened shards, in order (front: being consumed)
  int opening = 0;                     // shards the openers are working on
  int64_t open_next = 0;               // push-order ticket of the next shard an opener takes
  int64_t open_done = 0;               // ticket of the next shard to append to `opened`
  std::map<int64_t, std::shared_ptr<Shard>> parked;  // finished out of order (null: failed)
  // packed shards whose mappings the openers unmap: an unmap of a populated shard (a TLB
  // shootdown across the process's threads) ran on the packer under this feed's lock, where
  // the caller's dino_feed_next waits; the openers do it outside the lock
  std::vector<std::shared_ptr<Shard>> retired;
  bool epoch_end = false;              // no more pushes this epoch
  bool epoch_done = false;             // the packer found fewer than B samples left after epoch_end
  bool stop = false;
  int64_t generation = 0;              // bumped by dino_feed_reset (work of older epochs is dropped)
  int64_t next_seq = 0, next_out = 0;
  std::string error;                   // first shard error of the epoch (reported once by next)
  int64_t shards_failed = 0, shards_done = 0, batches = 0;
  double t_open = 0, t_pack = 0, t_slot_wait = 0, t_sample_wait = 0;
  std::vector<std::thread> openers;
  std::thread packer;
  // study trace (DINO_FEED_TRACE=path, written at destroy): per packed batch the packer's
  // loop start / slot / samples / pack end / ready stamps, per dino_feed_next its entry / return
  std::vector<std::array<double, 6>> trace_pack, trace_next;
  bool trace = getenv("DINO_FEED_TRACE") != nullptr;

  void opener_loop();
  void packer_loop();
  int free_slot_locked(std::unique_lock<std::mutex>& lk);
};

void dino_feed::opener_loop() {
  std::unique_lock<std::mutex> lk(m);
  for (;;) {
    cv.wait(lk, [&] {
      return stop || !retired.empty() ||
             (!pending.empty() && (int)(opened.size() + parked.size()) + opening < lookahead + 1);
    });
    if (stop) return;
    if (!retired.empty()) {
      std::vector<std::shared_ptr<Shard>> done;
      done.swap(retired);
      lk.unlock();
      done.clear();  // munmap, outside the lock
      lk.lock();
      continue;
    }
    auto sh = std::make_shared<Shard>();
    sh->path = pending.front();
    pending.pop_front();
    ++opening;
    const int64_t ticket = open_next++;
    const int64_t gen = generation;
    const int32_t wait = wait_ms;
    const bool shuf = shuffle;
    const uint64_t seed = shuffle_seed, ep = epoch;
    lk.unlock();
    const double t0 = now_s();
    std::string err;
    if (wait > 0)
      err = wait_shard(sh->path, wait, [&] {
        std::lock_guard<std::mutex> g(m);
        return stop || gen != generation;
      });
    if (err.empty()) err = open_shard(*sh);
    if (err.empty() && shuf) shuffle_samples(sh->samples, seed, ep, sh->path);
    const double dt = now_s() - t0;
    lk.lock();
    --opening;
    t_open += dt;
    if (gen == generation) {
      if (!err.empty()) {  // reference hpc_source.py:358-366: a shard I/O error is logged and skipped
        ++shards_failed;
        if (error.empty()) error = err;
        sh.reset();
      }
      parked.emplace(ticket, std::move(sh));
      // hand the shards on in push order
      for (auto it = parked.find(open_done); it != parked.end(); it = parked.find(open_done)) {
        if (it->second) opened.push_back(std::move(it->second));
        parked.erase(it);
        ++open_done;
      }
    }
    cv.notify_all();
  }
}

// A slot the packer may fill (waits for retired copies); -1 when stopping.  Called locked.
int dino_feed::free_slot_locked(std::unique_lock<std::mutex>& lk) {
  for (;;) {
    if (stop) return -1;
    for (size_t k = 0; k < slots.size(); ++k)
      if (slots[k].state == kFree) return (int)k;
    // the oldest copying slot: wait for its H2D copy outside the lock
    int best = -1;
    for (size_t k = 0; k < slots.size(); ++k)
      if (slots[k].state == kCopying && (best < 0 || slots[k].seq < slots[best].seq)) best = (int)k;
    if (best >= 0) {
      hipEvent_t ev = slots[best].ev;
      lk.unlock();
      (void)hipEventSynchronize(ev);
      lk.lock();
      if (slots[best].state == kCopying) slots[best].state = kFree;
      continue;
    }
    cv.wait(lk);  // every slot is ready or held by the caller
  }
}

void dino_feed::packer_loop() {
  std::vector<uint64_t> ptrs;
  std::vector<int32_t> fds;
  std::vector<int64_t> lens;
  std::vector<std::shared_ptr<Shard>> used;  // keeps the batch's mappings alive while it is packed
  std::unique_lock<std::mutex> lk(m);
  for (;;) {
    double t0 = now_s();
    std::array<double, 6> tr{t0, 0, 0, 0, 0, 0};
    const int k = free_slot_locked(lk);
    if (k < 0) return;
    t_slot_wait += now_s() - t0;
    tr[1] = now_s();
    // wait for B samples (or the end of the epoch)
    t0 = now_s();
    int64_t avail = 0;
    for (;;) {
      if (stop) return;
      avail = 0;
      for (auto& s : opened) avail += (int64_t)(s->samples.size() - s->next);
      const bool more = !pending.empty() || opening > 0;
      if (avail >= batch) break;
      if (!more && epoch_end && !epoch_done) {
        epoch_done = true;  // the last partial batch is dropped
        opened.clear();
        cv.notify_all();
      }
      cv.wait(lk);
    }
    t_sample_wait += now_s() - t0;
    tr[2] = now_s();
    const int64_t gen = generation;
    Slot& sl = slots[k];
    sl.state = kFilling;
    ptrs.resize(batch);
    fds.resize(batch);
    lens.resize(batch);
    bool by_fd = false;
    sl.offs.resize(batch + 1);
    sl.info.assign((size_t)batch * 4, 0);
    int32_t i = 0;
    sl.offs[0] = 0;
    used.clear();
    for (auto& s : opened) {
      if (i < batch && s->next < s->samples.size()) used.push_back(s);
      while (i < batch && s->next < s->samples.size()) {
        const dino_tar_sample& r = s->samples[s->next++];
        if (s->fd >= 0) {  // pread mode: file offset of the image
          ptrs[i] = (uint64_t)(16 + r.img_off);
          by_fd = true;
        } else {
          ptrs[i] = (uint64_t)(uintptr_t)(s->tar + r.img_off);
        }
        fds[i] = s->fd;
        lens[i] = r.img_len;
        sl.offs[i + 1] = sl.offs[i] + r.img_len;
        ++i;
      }
      if (i == batch) break;
    }
    const int64_t need = sl.offs[batch];
    const dino_aug_config* cfgp = have_cfg ? &cfg : nullptr;
    dino_aug_config cfg_copy = cfg;
    if (cfgp) cfgp = &cfg_copy;
    lk.unlock();
    t0 = now_s();
    bool ok = true;
    if (sl.cap < need) {
      slot_free(gpu, sl.host);
      sl.cap = 0;
      const int64_t c = need + need / 4 + 4096;
      sl.host = (uint8_t*)slot_alloc(gpu, (size_t)c);
      if (sl.host) sl.cap = c;
      else ok = false;
    }
    if (ok) {
      pool->run(ptrs.data(), by_fd ? fds.data() : nullptr, lens.data(), sl.offs.data(), batch, sl.host, max_dim, cfgp,
                sl.info.data(), &sl.ws, &sl.aws);
      memcpy(sl.offs_pinned, sl.offs.data(), sizeof(int64_t) * (batch + 1));
    }
    const double dt = now_s() - t0;
    tr[3] = now_s();
    lk.lock();
    tr[4] = now_s();
    t_pack += dt;
    // the shards every sample of which is packed (their bytes now live in slots) go to the
    // openers to unmap
    while (!opened.empty() && opened.front()->next >= opened.front()->samples.size()) {
      retired.push_back(std::move(opened.front()));
      opened.pop_front();
      ++shards_done;
    }
    for (auto& u : used)
      if (u.use_count() == 1) retired.push_back(std::move(u));  // a shard reset() dropped meanwhile
    used.clear();
    if (!ok) {
      sl.state = kFree;
      if (error.empty()) error = "dino_feed: allocation of a pinned slot failed";
      stop = true;
      cv.notify_all();
      return;
    }
    if (gen != generation) {  // reset while packing: the batch belongs to the dropped epoch
      sl.state = kFree;
      continue;
    }
    sl.nbytes = need;
    sl.seq = next_seq++;
    sl.state = kReady;
    ++batches;
    if (trace) {
      tr[5] = now_s();
      trace_pack.push_back(tr);
    }
    cv.notify_all();
  }
}

extern "C" {

const char* dino_feed_last_error(void) { return g_feed_err.c_str(); }

int dino_feed_create(int32_t batch, int32_t nthreads, int32_t nslots, int32_t lookahead, int32_t max_image_dim,
                     const dino_aug_config* cfg, dino_feed** out) {
  if (!out || batch <= 0 || nslots < 1) return feed_fail(DINO_EINVAL, "dino_feed_create: bad arguments");
  *out = nullptr;
  auto f = std::make_unique<dino_feed>();
  f->batch = batch;
  f->max_dim = (max_image_dim <= 0 || max_image_dim > kMaxImageDim) ? kMaxImageDim : max_image_dim;
  f->lookahead = std::max(1, lookahead);
  if (cfg) {
    f->cfg = *cfg;
    f->have_cfg = true;
  }
  f->pool = std::make_unique<CopyPool>(std::min(64, std::max(1, nthreads)));
  int ndev = 0;
  f->gpu = hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0;
  if (!f->gpu) (void)hipGetLastError();
  f->slots.resize((size_t)nslots);
  for (auto& s : f->slots) {
    s.offs_pinned = (int64_t*)slot_alloc(f->gpu, sizeof(int64_t) * (batch + 1));
    if (!s.offs_pinned || (f->gpu && hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess)) {
      for (auto& t : f->slots) {
        if (t.ev) (void)hipEventDestroy(t.ev);
        slot_free(f->gpu, t.offs_pinned);
      }
      return feed_fail(DINO_EHIP, "dino_feed_create: HIP event / pinned allocation failed");
    }
  }
  dino_feed* p = f.release();
  for (int k = 0; k < std::min(p->lookahead, kMaxOpeners); ++k) p->openers.emplace_back([p] { p->opener_loop(); });
  p->packer = std::thread([p] { p->packer_loop(); });
  *out = p;
  return DINO_OK;
}

int dino_feed_destroy(dino_feed* f) {
  if (!f) return DINO_OK;
  {
    std::lock_guard<std::mutex> g(f->m);
    f->stop = true;
  }
  f->cv.notify_all();
  for (auto& t : f->openers)
    if (t.joinable()) t.join();
  if (f->packer.joinable()) f->packer.join();
  if (f->trace) {
    if (FILE* fp = fopen(getenv("DINO_FEED_TRACE"), "w")) {
      for (auto& r : f->trace_pack) fprintf(fp, "P %.6f %.6f %.6f %.6f %.6f %.6f\n", r[0], r[1], r[2], r[3], r[4], r[5]);
      for (auto& r : f->trace_next) fprintf(fp, "N %.6f %.6f %.6f %.0f %.0f\n", r[0], r[1], r[2], r[3], r[4]);
      fclose(fp);
    }
  }
  for (auto& s : f->slots) {  // copies still reading a slot finish first
    if (s.state == kCopying) (void)hipEventSynchronize(s.ev);
    if (s.ev) (void)hipEventDestroy(s.ev);
    slot_free(f->gpu, s.host);
    slot_free(f->gpu, s.offs_pinned);
  }
  delete f;
  return DINO_OK;
}

int dino_feed_push(dino_feed* f, const char* path) {
  if (!f || !path) return feed_fail(DINO_EINVAL, "dino_feed_push: bad arguments");
  {
    std::lock_guard<std::mutex> g(f->m);
    if (f->epoch_end) return feed_fail(DINO_EINVAL, "dino_feed_push: the epoch was ended (dino_feed_reset first)");
    f->pending.emplace_back(path);
  }
  f->cv.notify_all();
  return DINO_OK;
}

int dino_feed_end_epoch(dino_feed* f) {
  if (!f) return feed_fail(DINO_EINVAL, "dino_feed_end_epoch: null feed");
  {
    std::lock_guard<std::mutex> g(f->m);
    f->epoch_end = true;
  }
  f->cv.notify_all();
  return DINO_OK;
}

int dino_feed_set_cfg(dino_feed* f, const dino_aug_config* cfg) {
  if (!f) return feed_fail(DINO_EINVAL, "dino_feed_set_cfg: null feed");
  std::lock_guard<std::mutex> g(f->m);
  if (cfg) f->cfg = *cfg;
  f->have_cfg = cfg != nullptr;
  return DINO_OK;
}

int dino_feed_set_shard_wait(dino_feed* f, int32_t timeout_ms) {
  if (!f) return feed_fail(DINO_EINVAL, "dino_feed_set_shard_wait: null feed");
  std::lock_guard<std::mutex> g(f->m);
  f->wait_ms = std::max(0, timeout_ms);
  return DINO_OK;
}

int dino_feed_set_shuffle(dino_feed* f, int32_t enable, uint64_t seed) {
  if (!f) return feed_fail(DINO_EINVAL, "dino_feed_set_shuffle: null feed");
  std::lock_guard<std::mutex> g(f->m);
  f->shuffle = enable != 0;
  f->shuffle_seed = seed;
  return DINO_OK;
}

int dino_feed_set_epoch(dino_feed* f, uint64_t epoch) {
  if (!f) return feed_fail(DINO_EINVAL, "dino_feed_set_epoch: null feed");
  std::lock_guard<std::mutex> g(f->m);
  f->epoch = epoch;
  return DINO_OK;
}

int dino_feed_next(dino_feed* f, int32_t timeout_ms, dino_feed_batch* out) {
  if (!f || !out) return feed_fail(DINO_EINVAL, "dino_feed_next: bad arguments");
  const double t_in = now_s();
  std::unique_lock<std::mutex> lk(f->m);
  const double t_lock = now_s();
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
  for (;;) {
    if (!f->error.empty()) {  // one shard failed: report it once, the feed goes on without it
      std::string e;
      e.swap(f->error);
      g_feed_err = e;
      return DINO_FEED_SHARD_ERROR;
    }
    for (size_t k = 0; k < f->slots.size(); ++k) {
      Slot& s = f->slots[k];
      if (s.state == kReady && s.seq == f->next_out) {
        s.state = kHanded;
        ++f->next_out;
        out->slot = (int32_t)k;
        out->n = f->batch;
        out->nbytes = s.nbytes;
        out->host = s.host;
        out->offsets = s.offs_pinned;
        out->info = s.info.data();
        out->ws_need = s.ws;
        out->aws_need = s.aws;
        out->seq = s.seq;
        if (f->trace) f->trace_next.push_back({t_in, t_lock, now_s(), (double)s.seq, (double)timeout_ms, 0});
        return DINO_OK;
      }
    }
    if (f->epoch_done) {
      bool any_ready = false;
      for (auto& s : f->slots) any_ready |= s.state == kReady || s.state == kFilling;
      if (!any_ready) return DINO_FEED_END;
    }
    if (f->stop) return feed_fail(DINO_EINVAL, "dino_feed_next: the feed stopped");
    if (timeout_ms < 0) {
      f->cv.wait(lk);
    } else if (f->cv.wait_until(lk, deadline) == std::cv_status::timeout) {
      return DINO_FEED_TIMEOUT;
    }
  }
}

int dino_feed_copy(dino_feed* f, int32_t slot, uint8_t* d_bytes, int64_t* d_offsets, void* stream) {
  if (!f || slot < 0 || slot >= (int32_t)f->slots.size() || !d_bytes || !d_offsets)
    return feed_fail(DINO_EINVAL, "dino_feed_copy: bad arguments");
  Slot& s = f->slots[slot];
  if (!f->gpu) return feed_fail(DINO_EINVAL, "dino_feed_copy: no GPU (host-only feed)");
  {
    std::lock_guard<std::mutex> g(f->m);
    if (s.state != kHanded) return feed_fail(DINO_EINVAL, "dino_feed_copy: slot not handed out");
  }
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemcpyAsync(d_bytes, s.host, (size_t)std::max<int64_t>(s.nbytes, 1), hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    e = hipMemcpyAsync(d_offsets, s.offs_pinned, sizeof(int64_t) * (f->batch + 1), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipEventRecord(s.ev, st);
  {
    std::lock_guard<std::mutex> g(f->m);
    s.state = e == hipSuccess ? kCopying : kFree;
  }
  f->cv.notify_all();
  if (e != hipSuccess) return feed_fail(DINO_EHIP, std::string("dino_feed_copy: ") + hipGetErrorString(e));
  return DINO_OK;
}

int dino_feed_release(dino_feed* f, int32_t slot) {
  if (!f || slot < 0 || slot >= (int32_t)f->slots.size()) return feed_fail(DINO_EINVAL, "dino_feed_release: bad slot");
  {
    std::lock_guard<std::mutex> g(f->m);
    if (f->slots[slot].state == kHanded) f->slots[slot].state = kFree;
  }
  f->cv.notify_all();
  return DINO_OK;
}

int dino_feed_reset(dino_feed* f) {
  if (!f) return feed_fail(DINO_EINVAL, "dino_feed_reset: null feed");
  {
    std::lock_guard<std::mutex> g(f->m);
    ++f->generation;
    ++f->epoch;
    f->pending.clear();
    f->opened.clear();
    f->parked.clear();
    f->open_done = f->open_next;  // shards still being opened belong to the old generation
    f->epoch_end = f->epoch_done = false;
    f->error.clear();
    for (auto& s : f->slots)
      if (s.state == kReady) s.state = kFree;  // filled for the old epoch, never handed out
    // renumber: batches of the new epoch start after everything handed out so far
    f->next_seq = f->next_out;
  }
  f->cv.notify_all();
  return DINO_OK;
}

int dino_feed_stats(dino_feed* f, double* seconds, int64_t* counts) {
  if (!f || !seconds || !counts) return feed_fail(DINO_EINVAL, "dino_feed_stats: bad arguments");
  std::lock_guard<std::mutex> g(f->m);
  seconds[0] = f->t_open;
  seconds[1] = f->t_pack;
  seconds[2] = f->t_slot_wait;
  seconds[3] = f->t_sample_wait;
  counts[0] = f->batches;
  counts[1] = f->shards_done;
  counts[2] = f->shards_failed;
  return DINO_OK;
}

}  // extern "C"
