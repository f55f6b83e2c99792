#include "memcap/usage.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>

#include "common/log.h"
#include "memcap_area.h"

namespace adp::memcap {
namespace {

namespace area = adp_memcap;
constexpr const char* kSuffix = ".memcap";

// Creation and collection take turns: a file collected between its age check
// and its unlink could otherwise be a grant created in between.
std::mutex g_mu;

bool IsKeyName(std::string_view name, std::string* key) {
  size_t n = strlen(kSuffix);
  if (name.size() != 16 + n || name.substr(16) != kSuffix) return false;
  for (char c : name.substr(0, 16))
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
  if (key) *key = std::string(name.substr(0, 16));
  return true;
}

template <typename T>
T Field(const unsigned char* hdr, size_t off) {
  T v;
  memcpy(&v, hdr + off, sizeof(v));
  return v;
}

std::vector<uint64_t> Column(const unsigned char* hdr, size_t off, uint32_t n) {
  std::vector<uint64_t> v(n);
  if (n) memcpy(v.data(), hdr + off, n * sizeof(uint64_t));
  return v;
}

}  // namespace

std::string AllocationKey(std::vector<std::string_view> ids) {
  std::sort(ids.begin(), ids.end());
  return AllocationKeySorted(ids);
}

std::string AllocationKeySorted(const std::vector<std::string_view>& sorted_ids) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a
  for (size_t i = 0; i < sorted_ids.size(); ++i) {
    if (i) h = (h ^ ',') * 1099511628211ull;
    for (unsigned char c : sorted_ids[i]) h = (h ^ c) * 1099511628211ull;
  }
  std::string key(16, '0');
  for (int i = 15; i >= 0; --i, h >>= 4) key[static_cast<size_t>(i)] = "0123456789abcdef"[h & 15];
  return key;
}

Status CreateGrantFile(const std::string& dir, const std::string& key, const std::vector<uint64_t>& cap_bytes,
                       std::string_view ids_joined) {
  if (cap_bytes.size() > static_cast<size_t>(area::kMaxDevices)) return InvalidArgument("too many devices");
  // Only up to the IDs: the rest of the file is sparse zeros.
  std::vector<unsigned char> hdr(offsetof(area::Area, ids) + std::min<size_t>(ids_joined.size(), area::kIdsBytes), 0);
  auto put = [&](size_t off, const void* p, size_t n) { memcpy(hdr.data() + off, p, n); };
  uint32_t magic = area::kMagic, version = area::kVersion, devices = static_cast<uint32_t>(cap_bytes.size());
  uint32_t ids_len = static_cast<uint32_t>(std::min<size_t>(ids_joined.size(), area::kIdsBytes));
  put(offsetof(area::Area, magic), &magic, 4);
  put(offsetof(area::Area, version), &version, 4);
  put(offsetof(area::Area, devices), &devices, 4);
  put(offsetof(area::Area, ids_len), &ids_len, 4);
  if (devices) put(offsetof(area::Area, cap), cap_bytes.data(), devices * sizeof(uint64_t));
  put(offsetof(area::Area, ids), ids_joined.data(), ids_len);

  std::string path = dir + "/" + key + kSuffix, tmp = path + ".tmp";
  std::lock_guard<std::mutex> lk(g_mu);
  int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_NOFOLLOW | O_CLOEXEC, 0666);
  if (fd < 0 && errno == ENOENT) {
    // The directory went with a kubelet cleaning its plugin directory (or was never made).
    size_t slash = dir.rfind('/');
    if (slash != std::string::npos && slash > 0) mkdir(dir.substr(0, slash).c_str(), 0755);
    mkdir(dir.c_str(), 0755);
    fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_NOFOLLOW | O_CLOEXEC, 0666);
  }
  if (fd < 0) return Internal("open " + tmp + ": " + strerror(errno));
  // Any uid in the container writes its counters (the directory stays the daemon's).
  bool ok = fchmod(fd, 0666) == 0 && ftruncate(fd, sizeof(area::Area)) == 0 &&
            pwrite(fd, hdr.data(), hdr.size(), 0) == static_cast<ssize_t>(hdr.size());
  int err = errno;
  close(fd);
  if (!ok || rename(tmp.c_str(), path.c_str()) != 0) {
    if (ok) err = errno;
    unlink(tmp.c_str());
    return Internal("create " + path + ": " + strerror(err));
  }
  return Status::Ok();
}

namespace {

struct Job {
  std::string dir, key, ids;
  std::vector<uint64_t> caps;
};

// One writer per process, never destroyed (its thread outlives every plugin).
struct Writer {
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::deque<Job> jobs;
  uint64_t queued = 0, done = 0;
  bool warned = false;
  std::atomic<bool> wake_pending{false};  // a job was queued without waking the writer

  Writer() { std::thread([this] { Run(); }).detach(); }
  void Run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      // Every job queued without a wake is followed by WakeWriter() once the
      // gRPC loop has written the Allocate response; the bounded wait is only a
      // backstop (an idle daemon wakes twice a second here, not 50 times).
      // system_clock: see Flush().
      while (jobs.empty()) cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(500));
      Job j = std::move(jobs.front());
      jobs.pop_front();
      lk.unlock();
      Status st = CreateGrantFile(j.dir, j.key, j.caps, j.ids);
      lk.lock();
      if (!st.ok() && !warned) {
        warned = true;
        LOG_WARN("memcap", "%s; containers' HBM use is not reported", st.ToString().c_str());
      }
      ++done;
      done_cv.notify_all();
    }
  }
};

Writer& TheWriter() {
  static Writer* w = new Writer;
  return *w;
}

constexpr size_t kMaxPending = 4096;

}  // namespace

void CreateGrantFileAsync(std::string dir, std::string key, std::vector<uint64_t> cap_bytes, std::string ids_joined,
                          bool wake) {
  Writer& w = TheWriter();
  std::lock_guard<std::mutex> lk(w.mu);
  if (w.jobs.size() >= kMaxPending) {  // the filesystem is stuck: the shim falls back to /dev/shm
    if (!w.warned) {
      w.warned = true;
      LOG_WARN("memcap", "%zu grant files waiting to be written; dropping new ones (HBM use not reported)",
               w.jobs.size());
    }
    return;
  }
  w.jobs.push_back({std::move(dir), std::move(key), std::move(ids_joined), std::move(cap_bytes)});
  ++w.queued;
  if (wake) w.cv.notify_one();
  else w.wake_pending.store(true, std::memory_order_release);
}

void WakeWriter() {
  Writer& w = TheWriter();
  // The job was queued under the mutex before the flag was set: the writer's
  // wait re-checks the queue, so notifying without the lock cannot be missed.
  if (w.wake_pending.load(std::memory_order_relaxed) && w.wake_pending.exchange(false, std::memory_order_acq_rel))
    w.cv.notify_one();
}

bool Flush(int timeout_ms) {
  WakeWriter();
  Writer& w = TheWriter();
  std::unique_lock<std::mutex> lk(w.mu);
  uint64_t target = w.queued;
  // system_clock: pthread_cond_timedwait (a steady_clock wait is
  // pthread_cond_clockwait, which this toolchain's TSan does not intercept).
  return w.done_cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms),
                              [&] { return w.done >= target; });
}

Result<Usage> ReadGrant(const std::string& dir, const std::string& key) {
  std::string path = dir + "/" + key + kSuffix;
  // Read-write only to trim a file the container grew; never follows a link,
  // never blocks on something that is not a regular file.
  int fd = open(path.c_str(), O_RDWR | O_NOFOLLOW | O_NONBLOCK | O_CLOEXEC);
  if (fd < 0) {
    if (errno == ENOENT) return NotFound(path);
    return InvalidArgument(path + ": " + strerror(errno));
  }
  struct stat st;
  std::vector<unsigned char> hdr(area::kHeaderBytes);
  bool regular = fstat(fd, &st) == 0 && S_ISREG(st.st_mode);
  if (regular && st.st_size > static_cast<off_t>(2 * sizeof(area::Area))) {
    int r = ftruncate(fd, sizeof(area::Area));
    (void)r;
  }
  bool got = regular && pread(fd, hdr.data(), hdr.size(), 0) == static_cast<ssize_t>(hdr.size());
  close(fd);
  if (!got) return InvalidArgument(path + ": not a grant file");
  const unsigned char* h = hdr.data();
  uint32_t devices = Field<uint32_t>(h, offsetof(area::Area, devices));
  uint32_t ids_len = Field<uint32_t>(h, offsetof(area::Area, ids_len));
  if (Field<uint32_t>(h, offsetof(area::Area, magic)) != area::kMagic ||
      Field<uint32_t>(h, offsetof(area::Area, version)) != area::kVersion ||
      devices > static_cast<uint32_t>(area::kMaxDevices) || ids_len > static_cast<uint32_t>(area::kIdsBytes))
    return InvalidArgument(path + ": bad header");
  Usage u;
  u.key = key;
  u.mtime_s = static_cast<int64_t>(st.st_mtime);
  u.used = Column(h, offsetof(area::Area, used), devices);
  u.cap = Column(h, offsetof(area::Area, cap), devices);
  u.peak = Column(h, offsetof(area::Area, peak), devices);
  u.refused = Column(h, offsetof(area::Area, refused), devices);
  u.processes = std::min<uint32_t>(Field<uint32_t>(h, offsetof(area::Area, processes)), area::kSlots);
  // The container may have rewritten the IDs: kept only if they still name this file.
  std::string ids(reinterpret_cast<const char*>(h + offsetof(area::Area, ids)), ids_len);
  std::vector<std::string_view> parts;
  for (size_t b = 0; b <= ids.size();) {
    size_t e = ids.find(',', b);
    if (e == std::string::npos) e = ids.size();
    parts.emplace_back(std::string_view(ids).substr(b, e - b));
    b = e + 1;
  }
  if (!ids.empty() && AllocationKey(parts) == key) u.ids = std::move(ids);
  return u;
}

std::vector<Usage> ReadAll(const std::string& dir) {
  std::vector<std::string> keys;
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) {
      std::string key;
      if (IsKeyName(e->d_name, &key)) keys.push_back(std::move(key));
    }
    closedir(d);
  }
  std::sort(keys.begin(), keys.end());
  std::vector<Usage> out;
  for (const auto& k : keys)
    if (auto u = ReadGrant(dir, k); u.ok()) out.push_back(std::move(*u));
  return out;
}

size_t Collect(const std::string& dir, const std::set<std::string>* live, int64_t min_age_s, size_t max_files) {
  std::lock_guard<std::mutex> lk(g_mu);
  DIR* d = opendir(dir.c_str());
  if (!d) return 0;
  int dfd = dirfd(d);
  time_t now = time(nullptr);
  std::vector<std::pair<int64_t, std::string>> kept;  // (mtime, name)
  size_t removed = 0;
  while (dirent* e = readdir(d)) {
    std::string name = e->d_name, key;
    bool grant = IsKeyName(name, &key);
    bool tmp = name.size() > 4 && name.compare(name.size() - 4, 4, ".tmp") == 0;
    struct stat st;
    if ((!grant && !tmp) || fstatat(dfd, name.c_str(), &st, AT_SYMLINK_NOFOLLOW) != 0) continue;
    bool old = now - st.st_mtime >= min_age_s;
    if ((tmp && old) || (grant && live && old && !live->count(key))) {
      // A directory: a runtime that mounted the path before the writer got to
      // it creates one (the shim then counts in /dev/shm); removed once empty.
      removed += unlinkat(dfd, name.c_str(), S_ISDIR(st.st_mode) ? AT_REMOVEDIR : 0) == 0;
      continue;
    }
    if (grant) kept.emplace_back(static_cast<int64_t>(st.st_mtime), name);
  }
  if (kept.size() > max_files) {
    std::sort(kept.begin(), kept.end());
    for (size_t i = 0; i + max_files < kept.size(); ++i)
      removed += unlinkat(dfd, kept[i].second.c_str(), 0) == 0 ||
                 unlinkat(dfd, kept[i].second.c_str(), AT_REMOVEDIR) == 0;
  }
  closedir(d);
  return removed;
}

}  // namespace adp::memcap
