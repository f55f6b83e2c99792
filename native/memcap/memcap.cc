// libadp_memcap.so: HBM caps for memory-unit sharing, enforced in the container.
//
// With `gpu-mem-gb` style resources (resourceConfig replicas = -1) a pod is
// granted N memory units of a GPU; the reference only counts them (server.go:
// 99-111: replicas = MiB/1000) and nothing stops a pod from using the whole
// GPU. When the plugin runs with --enforce-memory-units, Allocate() mounts this
// library into the container and preloads it (LD_PRELOAD). It interposes the
// HIP allocation entry points the frameworks call through the PLT, keeps a
// per-device byte count, and refuses (hipErrorOutOfMemory) an allocation that
// would take a device past its cap. hipMemGetInfo / hipDeviceTotalMem /
// hipGetDeviceProperties report the cap as the device's memory, so frameworks
// that size themselves from free memory (PyTorch's mem_get_info, vLLM's
// gpu_memory_utilization) stay inside the grant.
//
// Caps: the grant files the daemon mounts read-only under /run/amdgpu-dp/grant/
// (memcap_area.h kGrantDir: "<hip ordinal>" -> MiB) are authoritative; the
// pod's AMD_GPU_MEMORY_LIMIT_MIB="<mib>[,<mib>...]" (one per device in HIP
// order) can only lower them -- empty, missing or larger values change nothing
// -- and is the whole cap only where no grant file is mounted. Devices past
// both lists are not capped. The grant is the container's: its processes share
// the counters (a shared-memory segment, see AttachShared). ADP_MEMCAP_VERBOSE=1
// logs every decision to stderr.
//
// Stream-ordered pools: hipFreeAsync returns a block to its pool, which keeps
// the memory reserved (release threshold) -- the bytes stay counted until a
// refusal (or hipMemGetInfo) trims the pools and reads back what they still
// reserve (ReconcilePools), so the pool can never hold memory past the cap.
//
// It has to load into whatever the workload's image is -- PyTorch-ROCm wheels
// target glibc 2.28 -- so it needs nothing but old libc symbols: no libstdc++
// runtime (no allocation through operator new, no std::mutex / std::string /
// containers, no guarded statics), libc entry points pinned to their
// GLIBC_2.2.5 versions where newer glibc re-versioned them, and no link-time
// dependency on libamdhip64 (the real entry points are resolved lazily:
// RTLD_NEXT, else the already-loaded libamdhip64). The exported symbols carry
// libamdhip64's version nodes (memcap.map). tests/test_memcap.py checks the
// imported symbol versions.
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <hip/hip_deprecated.h>
#include <pthread.h>
#include <signal.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>

#include "memcap_area.h"

// glibc 2.34 moved these into libc under new default versions; bind the
// original ones, which every glibc since 2.2.5 exports.
__asm__(".symver dlsym,dlsym@GLIBC_2.2.5");
__asm__(".symver dlopen,dlopen@GLIBC_2.2.5");
__asm__(".symver pthread_once,pthread_once@GLIBC_2.2.5");

namespace {

using adp_memcap::kMaxDevices;

template <typename T>
T Min(T a, T b) {
  return a < b ? a : b;
}

// ---- the process-local table: device pointer / VMM handle -> owner ---------
// Open addressing over calloc'd memory (no operator new: see the file comment).
struct Entry {
  const void* key;  // nullptr = empty, Tomb() = erased
  int32_t device;
  int32_t pooled;  // 1: a stream-ordered (pool) allocation
  uint64_t bytes;
};
inline const void* Tomb() { return reinterpret_cast<const void*>(uintptr_t{1}); }  // not a constant expression

struct Table {
  Entry* e = nullptr;
  size_t cap = 0, used = 0, tombs = 0;  // used counts live entries

  static size_t Hash(const void* k, size_t cap) {
    return static_cast<size_t>((reinterpret_cast<uintptr_t>(k) >> 4) * 0x9E3779B97F4A7C15ull) & (cap - 1);
  }
  Entry* Find(const void* k) {
    if (!cap) return nullptr;
    for (size_t i = Hash(k, cap), n = 0; n < cap; i = (i + 1) & (cap - 1), ++n) {
      if (e[i].key == k) return &e[i];
      if (!e[i].key) return nullptr;
    }
    return nullptr;
  }
  bool Grow() {
    size_t ncap = cap ? cap * 2 : 1024;
    Entry* ne = static_cast<Entry*>(calloc(ncap, sizeof(Entry)));
    if (!ne) return false;
    for (size_t i = 0; i < cap; ++i) {
      if (!e[i].key || e[i].key == Tomb()) continue;
      size_t j = Hash(e[i].key, ncap);
      while (ne[j].key) j = (j + 1) & (ncap - 1);
      ne[j] = e[i];
    }
    free(e);
    e = ne;
    cap = ncap;
    tombs = 0;
    return true;
  }
  // Inserts or overwrites; false only when memory is exhausted.
  bool Put(const void* k, int32_t device, uint64_t bytes) {
    if (Entry* x = Find(k)) {
      x->device = device;
      x->bytes = bytes;
      return true;
    }
    if ((used + tombs + 1) * 2 > cap && !Grow()) return false;
    size_t i = Hash(k, cap);
    while (e[i].key && e[i].key != Tomb()) i = (i + 1) & (cap - 1);
    if (e[i].key == Tomb()) --tombs;
    e[i] = {k, device, 0, bytes};
    ++used;
    return true;
  }
  void Erase(Entry* x) {
    x->key = Tomb();
    --used;
    ++tombs;
  }
  void Clear() {
    if (cap) memset(e, 0, cap * sizeof(Entry));
    used = tombs = 0;
  }
};

// ---- container-wide accounting ------------------------------------------
// Every process of the container draws on one grant: the counters live in a
// shared file (memcap_area.h) -- the one the daemon bind-mounted for this
// allocation (ADP_MEMCAP_FILE), else a segment in /dev/shm named after the
// container (its cgroup, or ADP_MEMCAP_KEY). Each process owns a slot
// recording what it holds, so the bytes of a process that exits -- or is
// killed -- are given back: at exit by the process itself, otherwise by the
// next process that would be refused, asks for free memory or attaches.
// Without either file the accounting is per process.
using adp_memcap::kMagic;
using adp_memcap::kSlots;
using adp_memcap::kVersion;
using SharedArea = adp_memcap::Area;
using SharedSlot = adp_memcap::Slot;

struct State {
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  Table allocs;                               // this process's allocations
  uint64_t local_used[kMaxDevices] = {};      // used when there is no shared segment
  uint64_t cap[kMaxDevices] = {};             // 0 = not capped
  uint64_t pool_live[kMaxDevices] = {};       // bytes of live stream-ordered allocations (this process)
  uint64_t pool_held[kMaxDevices] = {};       // bytes freed to a pool, still counted (this process)
  hipMemPool_t pools[kMaxDevices][4] = {};    // pools allocated from (explicit, and current at hipMallocAsync)
  bool pools_overflow[kMaxDevices] = {};      // more pools than `pools` holds: their reserve is unknown
  // Bumped by every change of pool_live: ReconcilePools reads the pools'
  // reserve without the lock and applies it only if nothing moved meanwhile.
  uint64_t pool_gen[kMaxDevices] = {};
  int devices = 0;                            // devices with a cap entry (grant or env)
  int granted = 0;                            // devices with a daemon grant file
  bool verbose = false;
  bool any_cap = false;
  std::atomic<bool> warned[kMaxDevices] = {};
  SharedArea* area = nullptr;
  int slot = -1;
  pid_t slot_pid = 0;
  bool released = false;  // this process's slot was handed back (exit): stop touching the counters
  char shm_path[160] = {0};
  char file_path[256] = {0};  // the daemon's accounting file (ADP_MEMCAP_FILE), "" if none
};

State g_state;  // constant-initialised: no constructor runs at load time
pthread_once_t g_once = PTHREAD_ONCE_INIT;

struct Locked {
  explicit Locked(State& s) : s_(s) { pthread_mutex_lock(&s_.mu); }
  ~Locked() { pthread_mutex_unlock(&s_.mu); }
  Locked(const Locked&) = delete;
  Locked& operator=(const Locked&) = delete;
  State& s_;
};

void Log(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  fprintf(stderr, "amdgpu-dp memcap: %s\n", buf);
}

uint64_t StartTime(pid_t pid) {
  char path[64];
  snprintf(path, sizeof(path), "/proc/%d/stat", static_cast<int>(pid));
  FILE* f = fopen(path, "r");
  if (!f) return 0;
  char buf[1024];
  size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* p = strrchr(buf, ')');  // comm may contain spaces
  if (!p) return 0;
  int field = 2;  // fields after ")": 3 state ... 22 starttime
  for (const char* q = p + 1; *q; ++q)
    if (*q == ' ' && ++field == 22) return strtoull(q + 1, nullptr, 10);
  return 0;
}

bool Alive(pid_t pid, uint64_t start) {
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  uint64_t now = StartTime(pid);
  return !(start && now && now != start);  // a recycled pid is a different process
}

void SubSat(std::atomic<uint64_t>& a, uint64_t v) {
  uint64_t cur = a.load();
  while (!a.compare_exchange_weak(cur, cur - Min(cur, v))) {
  }
}

void RaisePeak(std::atomic<uint64_t>& peak, uint64_t v) {
  uint64_t cur = peak.load();
  while (cur < v && !peak.compare_exchange_weak(cur, v)) {
  }
}

// Hands the bytes of dead owners back (and frees their slots). `full` also
// catches a recycled pid (one /proc read per live slot); otherwise only
// owners that are gone (kill(2): ESRCH) are reclaimed -- cheap enough for
// every hipMemGetInfo.
void ReclaimDead(SharedArea* a, int mine, bool full = true) {
  for (int i = 0; i < kSlots; ++i) {
    if (i == mine) continue;
    SharedSlot& sl = a->slots[i];
    int32_t pid = sl.pid.load();
    if (pid <= 0) continue;
    bool dead = full ? !Alive(pid, sl.start.load()) : kill(pid, 0) != 0 && errno == ESRCH;
    if (!dead) continue;
    if (!sl.pid.compare_exchange_strong(pid, -1)) continue;  // someone else reclaims it
    for (int d = 0; d < kMaxDevices; ++d) SubSat(a->used[d], sl.bytes[d].exchange(0));
    sl.start.store(0);
    sl.pid.store(0);
    a->processes.fetch_sub(1);
  }
}

void ReleaseSlot() {
  State& s = g_state;
  Locked lk(s);
  if (!s.area || s.slot < 0 || s.slot_pid != getpid() || s.released) return;
  SharedSlot& sl = s.area->slots[s.slot];
  for (int d = 0; d < kMaxDevices; ++d) SubSat(s.area->used[d], sl.bytes[d].exchange(0));
  sl.start.store(0);
  sl.pid.store(0);
  s.area->processes.fetch_sub(1);
  s.released = true;
}

// Maps the daemon's accounting file for this grant: created and filled in by
// the daemon (grant, IDs); nullptr if it is absent or not a valid file.
SharedArea* MapDaemonFile(State& s) {
  int fd = open(s.file_path, O_RDWR | O_CLOEXEC | O_NOFOLLOW);
  if (fd < 0) {
    if (s.verbose) Log("no accounting file %s (%s)", s.file_path, strerror(errno));
    return nullptr;
  }
  off_t size = lseek(fd, 0, SEEK_END);
  void* m = size >= static_cast<off_t>(sizeof(SharedArea))
                ? mmap(nullptr, sizeof(SharedArea), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0)
                : MAP_FAILED;
  close(fd);
  if (m == MAP_FAILED) {
    Log("accounting file %s unusable (size %lld)", s.file_path, static_cast<long long>(size));
    return nullptr;
  }
  auto* a = static_cast<SharedArea*>(m);
  if (a->magic.load(std::memory_order_acquire) != kMagic || a->version != kVersion) {
    Log("accounting file %s has no valid header", s.file_path);
    munmap(m, sizeof(SharedArea));
    return nullptr;
  }
  return a;
}

// Maps (creating it if this process is first) the container's segment in /dev/shm.
SharedArea* MapShmSegment(State& s, bool* creator_out) {
  // shm_open(3) is open(2) under /dev/shm, and moved libraries across glibc versions.
  int fd = open(s.shm_path, O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC | O_NOFOLLOW, 0600);
  bool creator = fd >= 0;
  if (!creator) fd = open(s.shm_path, O_RDWR | O_CLOEXEC | O_NOFOLLOW);
  if (fd < 0) {
    if (s.verbose) Log("no shared segment %s (%s): accounting per process", s.shm_path, strerror(errno));
    return nullptr;
  }
  bool ok = true;
  if (creator) {
    ok = ftruncate(fd, sizeof(SharedArea)) == 0;
  } else {
    for (int i = 0; i < 1000 && ok; ++i) {  // the creator may still be sizing it
      off_t size = lseek(fd, 0, SEEK_END);
      if (size < 0) ok = false;
      else if (static_cast<size_t>(size) >= sizeof(SharedArea)) break;
      usleep(1000);
    }
  }
  void* m = ok ? mmap(nullptr, sizeof(SharedArea), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0) : MAP_FAILED;
  close(fd);
  if (m == MAP_FAILED) {
    if (s.verbose) Log("cannot map %s: accounting per process", s.shm_path);
    return nullptr;
  }
  auto* a = static_cast<SharedArea*>(m);
  if (creator) {
    a->version = kVersion;
    a->devices = static_cast<uint32_t>(s.devices);
    for (int d = 0; d < kMaxDevices; ++d) a->cap[d].store(s.cap[d]);
    a->magic.store(kMagic, std::memory_order_release);
  } else {
    for (int i = 0; i < 1000 && a->magic.load(std::memory_order_acquire) != kMagic; ++i) usleep(1000);
    if (a->magic.load(std::memory_order_acquire) != kMagic || a->version != kVersion) {
      munmap(m, sizeof(SharedArea));
      Log("shared segment %s not initialised: accounting per process", s.shm_path);
      return nullptr;
    }
  }
  *creator_out = creator;
  return a;
}

// Maps the container's accounting file and claims a slot for this process
// (called with the lock held, at initialisation and again in a forked child).
void AttachShared(State& s) {
  s.slot = -1;
  s.slot_pid = getpid();
  if (!s.area) {
    bool creator = false;
    if (s.file_path[0]) s.area = MapDaemonFile(s);
    if (!s.area) s.area = MapShmSegment(s, &creator);
    if (!s.area) return;
    // A restarted container finds its predecessor's processes still counted.
    if (!creator) ReclaimDead(s.area, -1);
  }
  uint64_t start = StartTime(s.slot_pid);
  for (int pass = 0; pass < 2 && s.slot < 0; ++pass) {
    if (pass) ReclaimDead(s.area, -1);
    for (int i = 0; i < kSlots; ++i) {
      int32_t zero = 0;
      if (s.area->slots[i].pid.compare_exchange_strong(zero, static_cast<int32_t>(s.slot_pid))) {
        s.area->slots[i].start.store(start);
        s.area->processes.fetch_add(1);
        s.slot = i;
        break;
      }
    }
  }
  if (s.slot < 0) {
    Log("no free slot in the shared segment: accounting per process");
    munmap(s.area, sizeof(SharedArea));
    s.area = nullptr;
  }
}

// fork(): the state is locked across it, so the child never sees the table or
// the counters half-updated by another thread.
void AtForkPrepare() { pthread_mutex_lock(&g_state.mu); }
void AtForkParent() { pthread_mutex_unlock(&g_state.mu); }
void AtForkChild() {
  // The child holds no device memory of its own yet: fresh local state, own slot.
  State& s = g_state;
  pthread_mutex_unlock(&s.mu);
  Locked lk(s);
  s.allocs.Clear();
  for (auto& u : s.local_used) u = 0;
  s.released = false;
  if (s.area) AttachShared(s);
}

// Reads "<dir>/<i>" grant files (i = 0, 1, ... until one is missing) into
// `mib`; returns how many were read. A file that exists but is not a plain
// number stops the list there (and is logged).
int ReadGrantFiles(const char* dir, uint64_t* mib, int max) {
  int n = 0;
  for (; n < max; ++n) {
    char path[256];
    snprintf(path, sizeof(path), "%s/%d", dir, n);
    int fd = open(path, O_RDONLY | O_CLOEXEC | O_NOFOLLOW | O_NONBLOCK);
    if (fd < 0) break;
    char buf[32];
    ssize_t r = read(fd, buf, sizeof(buf) - 1);
    close(fd);
    if (r <= 0) break;
    buf[r] = 0;
    char* end = nullptr;
    unsigned long long v = strtoull(buf, &end, 10);
    if (end == buf || (*end && *end != '\n') || v == 0 || v > (uint64_t{1} << 43)) {
      Log("grant file %s is not a MiB count; devices from %d on are capped by AMD_GPU_MEMORY_LIMIT_MIB only", path, n);
      break;
    }
    mib[n] = v;
  }
  return n;
}

// The grant directory: the daemon's read-only mount; ADP_MEMCAP_GRANT_DIR only
// where nothing is mounted there (tests), so a pod cannot point it elsewhere.
const char* GrantDir() {
  // access(2), not stat(2): stat is a GLIBC_2.33 symbol (see the file comment).
  if (access(adp_memcap::kGrantDir, F_OK) == 0) return adp_memcap::kGrantDir;
  const char* env = getenv("ADP_MEMCAP_GRANT_DIR");
  return env && env[0] == '/' ? env : nullptr;
}

void Init() {
  State& s = g_state;
  const char* v = getenv("ADP_MEMCAP_VERBOSE");
  s.verbose = v && *v && *v != '0';
  // The daemon's grant first: authoritative.
  uint64_t grant_mib[kMaxDevices] = {};
  const char* gdir = GrantDir();
  s.granted = gdir ? ReadGrantFiles(gdir, grant_mib, kMaxDevices) : 0;
  for (int d = 0; d < s.granted; ++d) s.cap[d] = grant_mib[d] << 20;
  // Then the environment: a lower value wins; never raises or removes a grant.
  const char* lim = getenv("AMD_GPU_MEMORY_LIMIT_MIB");
  int dev = 0;
  for (const char* p = lim; p && *p && dev < kMaxDevices; ++dev) {
    char* end = nullptr;
    unsigned long long mib = strtoull(p, &end, 10);
    if (end != p && mib > 0 && mib < (uint64_t{1} << 43)) {
      uint64_t b = static_cast<uint64_t>(mib) << 20;
      if (!s.cap[dev] || b < s.cap[dev]) s.cap[dev] = b;
    }
    p = strchr(p, ',');
    if (p) ++p;
  }
  s.devices = dev > s.granted ? dev : s.granted;
  for (int d = 0; d < s.devices; ++d) s.any_cap = s.any_cap || s.cap[d];
  if (s.verbose)
    Log("%d device(s) granted by %s, AMD_GPU_MEMORY_LIMIT_MIB=%s", s.granted, gdir ? gdir : "(no grant files)",
        lim ? lim : "(unset)");
  if (!s.any_cap) return;
  const char* file = getenv("ADP_MEMCAP_FILE");
  if (file && file[0] == '/' && strlen(file) < sizeof(s.file_path)) strcpy(s.file_path, file);
  // The container: its cgroup (shared by all its processes), unless named; and
  // the grant (a different grant is a different budget).
  uint64_t h = 1469598103934665603ull;  // FNV-1a
  auto mix = [&h](const char* b, size_t n) {
    for (size_t i = 0; i < n; ++i) h = (h ^ static_cast<unsigned char>(b[i])) * 1099511628211ull;
  };
  const char* k = getenv("ADP_MEMCAP_KEY");
  if (k && *k) {
    mix(k, strlen(k));
  } else if (FILE* f = fopen("/proc/self/cgroup", "r")) {
    char buf[4096];
    size_t n = fread(buf, 1, sizeof(buf), f);
    fclose(f);
    mix(buf, n);
  }
  mix("|", 1);
  for (int d = 0; d < s.devices; ++d) mix(reinterpret_cast<const char*>(&s.cap[d]), sizeof(s.cap[d]));
  const char* safe = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_.-";
  if (k && *k && strlen(k) <= 64 && strspn(k, safe) == strlen(k))  // a named budget, findable in /dev/shm
    snprintf(s.shm_path, sizeof(s.shm_path), "/dev/shm/adp-memcap-key-%s-%08llx", k,
             static_cast<unsigned long long>(h >> 32));
  else
    snprintf(s.shm_path, sizeof(s.shm_path), "/dev/shm/adp-memcap-%016llx", static_cast<unsigned long long>(h));
  {
    Locked lk(s);
    AttachShared(s);
  }
  pthread_atfork(AtForkPrepare, AtForkParent, AtForkChild);
  atexit(ReleaseSlot);
}

State& S() {
  pthread_once(&g_once, Init);
  return g_state;
}

uint64_t UsedLocked(State& s, int dev) { return s.area ? s.area->used[dev].load() : s.local_used[dev]; }

// Resolved entry points are cached in constant-initialised atomics (no guard
// variables): racing first callers store the same pointer.
void* HipLibrary() {
  static std::atomic<void*> lib{nullptr};
  void* h = lib.load(std::memory_order_acquire);
  if (h) return h;
  const char* env = getenv("ADP_MEMCAP_HIP_LIB");
  const char* names[] = {env, "libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"};
  for (const char* n : names)
    if (!h && n && *n) h = dlopen(n, RTLD_LAZY | RTLD_NOLOAD);
  for (const char* n : names)
    if (!h && n && *n) h = dlopen(n, RTLD_LAZY);
  if (h) lib.store(h, std::memory_order_release);
  return h;
}

void* RealSym(const char* name) {
  if (void* f = dlsym(RTLD_NEXT, name)) return f;
  // libamdhip64 pulled in by a library dlopen'ed RTLD_LOCAL is not in the
  // global scope RTLD_NEXT searches: take it by name (already loaded).
  void* lib = HipLibrary();
  return lib ? dlsym(lib, name) : nullptr;
}

void* Cached(std::atomic<void*>& slot, const char* name) {
  void* p = slot.load(std::memory_order_acquire);
  if (!p) {
    p = RealSym(name);
    if (p) slot.store(p, std::memory_order_release);
  }
  return p;
}

// The header also declares C++ template overloads of several entry points, so
// the real function's type is spelled out at each use.
#define REAL(fn, type)                         \
  static std::atomic<void*> real_slot{nullptr}; \
  auto real = reinterpret_cast<type>(Cached(real_slot, #fn))

int CurrentDevice() {
  static std::atomic<void*> slot{nullptr};
  auto get = reinterpret_cast<hipError_t (*)(int*)>(Cached(slot, "hipGetDevice"));
  int d = 0;
  if (!get || get(&d) != hipSuccess || d < 0 || d >= kMaxDevices) return 0;
  return d;
}

int StreamDevice(hipStream_t stream) {
  static std::atomic<void*> slot{nullptr};
  auto get = reinterpret_cast<hipError_t (*)(hipStream_t, hipDevice_t*)>(Cached(slot, "hipStreamGetDevice"));
  hipDevice_t d = 0;
  if (stream && get && get(stream, &d) == hipSuccess && d >= 0 && d < kMaxDevices) return d;
  return CurrentDevice();
}

// Reserves `bytes` on `dev` for this process (lock held); false if that would
// take the container past the cap.
bool TryReserveLocked(State& s, int dev, uint64_t bytes) {
  if (s.area && s.slot_pid != getpid()) AttachShared(s);  // a child forked around pthread_atfork
  if (s.area && !s.released) {
    for (int attempt = 0; attempt < 2; ++attempt) {
      uint64_t cur = s.area->used[dev].load();
      // cur + bytes <= cap without wrapping: a request near SIZE_MAX (an OOM
      // probe, an overflowed size) must be refused, not wrapped under the cap.
      while (bytes <= s.cap[dev] && cur <= s.cap[dev] - bytes) {
        if (s.area->used[dev].compare_exchange_weak(cur, cur + bytes)) {
          s.area->slots[s.slot].bytes[dev].fetch_add(bytes);
          RaisePeak(s.area->peak[dev], cur + bytes);
          return true;
        }
      }
      if (attempt == 0) ReclaimDead(s.area, s.slot);  // a dead process may still be counted
    }
    return false;
  }
  if (bytes <= s.cap[dev] && s.local_used[dev] <= s.cap[dev] - bytes) {
    s.local_used[dev] += bytes;
    return true;
  }
  return false;
}

bool ReconcilePools(int dev);

bool Reserve(int dev, uint64_t bytes) {
  State& s = S();
  if (!s.cap[dev]) return true;
  int reconciles = 0;
  for (;;) {
    {
      Locked lk(s);
      if (TryReserveLocked(s, dev, bytes)) return true;
      // Blocks freed to a stream-ordered pool are still counted: trim the
      // pools and count only what they still hold, then try once more (a few
      // times when other threads' stream-ordered calls keep racing the read).
      if (reconciles < 4 && s.pool_held[dev] && bytes <= s.cap[dev]) goto reconcile;
      if (s.area && !s.released) s.area->refused[dev].fetch_add(1);
      if (s.verbose || !s.warned[dev].exchange(true))
        Log("device %d: refused %.1f MiB (%.1f of %.1f MiB in use%s; the grant)", dev, bytes / 1048576.0,
            UsedLocked(s, dev) / 1048576.0, s.cap[dev] / 1048576.0, s.area ? " by the container" : "");
      return false;
    }
  reconcile:
    // Without the lock: it calls into HIP. A settled pass is the last one.
    reconciles = ReconcilePools(dev) ? 4 : reconciles + 1;
  }
}

void AddLocked(State& s, int dev, uint64_t bytes) {
  if (!s.area) {
    s.local_used[dev] += bytes;
  } else if (!s.released && s.slot_pid == getpid()) {
    RaisePeak(s.area->peak[dev], s.area->used[dev].fetch_add(bytes) + bytes);
    s.area->slots[s.slot].bytes[dev].fetch_add(bytes);
  }
}

void UnreserveLocked(State& s, int dev, uint64_t bytes) {
  if (s.area) {
    if (s.released || s.slot_pid != getpid()) return;
    SubSat(s.area->slots[s.slot].bytes[dev], bytes);
    SubSat(s.area->used[dev], bytes);
  } else {
    s.local_used[dev] -= Min(bytes, s.local_used[dev]);
  }
}

void Unreserve(int dev, uint64_t bytes) {
  State& s = S();
  if (!s.cap[dev]) return;
  Locked lk(s);
  UnreserveLocked(s, dev, bytes);
}

void Track(const void* key, int dev, uint64_t bytes) {
  State& s = S();
  if (!s.cap[dev] || !key) return;
  Locked lk(s);
  if (!s.allocs.Put(key, dev, bytes)) {
    UnreserveLocked(s, dev, bytes);  // out of host memory: cannot follow it, so do not count it
    return;
  }
  if (s.verbose) Log("device %d: +%llu bytes (%llu in use)", dev, static_cast<unsigned long long>(bytes),
                     static_cast<unsigned long long>(UsedLocked(s, dev)));
}

void Untrack(const void* key) {
  State& s = S();
  if (!key || !s.any_cap) return;
  Locked lk(s);
  Entry* x = s.allocs.Find(key);
  if (!x) return;  // not ours (uncapped device, or before a cap)
  int dev = x->device;
  uint64_t bytes = x->bytes;
  if (x->pooled) {
    // Back to its pool, which may keep it reserved: still counted (ReconcilePools).
    s.pool_live[dev] -= Min(bytes, s.pool_live[dev]);
    s.pool_held[dev] += bytes;
    ++s.pool_gen[dev];
  } else {
    UnreserveLocked(s, dev, bytes);
  }
  s.allocs.Erase(x);
  if (s.verbose) Log("device %d: -%llu bytes (%llu in use)", dev, static_cast<unsigned long long>(bytes),
                     static_cast<unsigned long long>(UsedLocked(s, dev)));
}

// Depth of interposed allocator calls on this thread: an entry point the HIP
// library implements by calling another exported one (hipMallocPitch ->
// hipMalloc, say) reaches this library again; only the outermost call counts.
thread_local int t_depth = 0;

// Common path of every allocator: reserve, call the real one, track or roll back.
template <typename Call>
hipError_t Capped(int dev, uint64_t bytes, void** out, Call call) {
  if (t_depth > 0) return call();
  if (!Reserve(dev, bytes)) {
    if (out) *out = nullptr;
    return hipErrorOutOfMemory;
  }
  ++t_depth;
  hipError_t e = call();
  --t_depth;
  if (e != hipSuccess || !out || !*out) {
    Unreserve(dev, bytes);
    return e;
  }
  Track(*out, dev, bytes);
  return e;
}

// A stream-ordered allocation just tracked: from `pool` (nullptr: the
// device's current pool).
void MarkPooled(const void* key, int dev, hipMemPool_t pool) {
  State& s = S();
  if (!s.cap[dev] || !key) return;
  Locked lk(s);
  Entry* x = s.allocs.Find(key);
  if (!x || x->pooled) return;
  x->pooled = 1;
  s.pool_live[dev] += x->bytes;
  ++s.pool_gen[dev];
  if (!pool) return;
  for (auto& p : s.pools[dev]) {
    if (p == pool) return;
    if (!p) {
      p = pool;
      return;
    }
  }
  s.pools_overflow[dev] = true;
}

// The pool hipMallocAsync on `dev` draws from now (hipDeviceSetMemPool may have
// replaced the default): recorded so a later trim covers it too.
hipMemPool_t CurrentPool(int dev) {
  static std::atomic<void*> s_cur{nullptr};
  auto get_current = reinterpret_cast<hipError_t (*)(hipMemPool_t*, int)>(Cached(s_cur, "hipDeviceGetMemPool"));
  hipMemPool_t p = nullptr;
  if (!get_current) return nullptr;
  ++t_depth;
  if (get_current(&p, dev) != hipSuccess) p = nullptr;
  --t_depth;
  return p;
}

// Trims every pool of `dev` this process allocated from and counts only what
// they still reserve beyond the live allocations (hipMemPoolAttrReservedMemCurrent);
// the rest of pool_held is given back to the grant. The reserve is read without
// the lock; if another thread's stream-ordered allocation or free moved
// pool_live meanwhile, reserve and pool_live no longer describe one moment and
// nothing is given back (returns false: the caller may try again).
bool ReconcilePools(int dev) {
  static std::atomic<void*> s_def{nullptr}, s_cur{nullptr}, s_trim{nullptr}, s_attr{nullptr};
  auto get_default = reinterpret_cast<hipError_t (*)(hipMemPool_t*, int)>(Cached(s_def, "hipDeviceGetDefaultMemPool"));
  auto get_current = reinterpret_cast<hipError_t (*)(hipMemPool_t*, int)>(Cached(s_cur, "hipDeviceGetMemPool"));
  auto trim = reinterpret_cast<hipError_t (*)(hipMemPool_t, size_t)>(Cached(s_trim, "hipMemPoolTrimTo"));
  auto attr = reinterpret_cast<hipError_t (*)(hipMemPool_t, hipMemPoolAttr, void*)>(
      Cached(s_attr, "hipMemPoolGetAttribute"));
  if (!trim || !attr) return true;
  State& s = g_state;
  hipMemPool_t pools[6] = {};
  int n = 0;
  uint64_t gen = 0;
  {
    Locked lk(s);
    if (s.pools_overflow[dev]) return true;  // a pool we cannot name: everything stays counted
    for (auto p : s.pools[dev])
      if (p) pools[n++] = p;
    gen = s.pool_gen[dev];
  }
  hipMemPool_t p = nullptr;
  if (get_default && get_default(&p, dev) == hipSuccess && p) pools[n++] = p;
  p = nullptr;
  if (get_current && get_current(&p, dev) == hipSuccess && p) pools[n++] = p;
  uint64_t reserved = 0;
  ++t_depth;  // whatever HIP calls back into this library passes through
  for (int i = 0; i < n; ++i) {
    bool dup = false;
    for (int j = 0; j < i; ++j) dup = dup || pools[j] == pools[i];
    if (dup) continue;
    (void)trim(pools[i], 0);
    uint64_t r = 0;
    if (attr(pools[i], hipMemPoolAttrReservedMemCurrent, &r) != hipSuccess) {
      --t_depth;
      return true;  // cannot tell: everything stays counted
    }
    reserved += r;
  }
  --t_depth;
  Locked lk(s);
  if (s.pool_gen[dev] != gen) return false;  // raced: the reserve may not cover pool_live's newest bytes
  uint64_t held = reserved > s.pool_live[dev] ? reserved - s.pool_live[dev] : 0;
  if (held < s.pool_held[dev]) {
    if (s.verbose)
      Log("device %d: pools hold %.1f MiB of %.1f MiB freed to them", dev, held / 1048576.0,
          s.pool_held[dev] / 1048576.0);
    UnreserveLocked(s, dev, s.pool_held[dev] - held);
    s.pool_held[dev] = held;
  }
  return true;
}

// Saturating size arithmetic: an overflowing size is refused at the cap.
uint64_t Mul(uint64_t a, uint64_t b) {
  if (a && b > UINT64_MAX / a) return UINT64_MAX;
  return a * b;
}
uint64_t Dim(size_t v) { return v ? v : 1; }

// Bytes of one element of a channel format (bits of x, y, z, w).
uint64_t ChannelBytes(const hipChannelFormatDesc* d) {
  if (!d) return 0;
  int bits = (d->x > 0 ? d->x : 0) + (d->y > 0 ? d->y : 0) + (d->z > 0 ? d->z : 0) + (d->w > 0 ? d->w : 0);
  return static_cast<uint64_t>((bits + 7) / 8);
}

uint64_t FormatBytes(hipArray_Format f) {
  switch (f) {
    case HIP_AD_FORMAT_UNSIGNED_INT8:
    case HIP_AD_FORMAT_SIGNED_INT8:
      return 1;
    case HIP_AD_FORMAT_UNSIGNED_INT16:
    case HIP_AD_FORMAT_SIGNED_INT16:
    case HIP_AD_FORMAT_HALF:
      return 2;
    default:
      return 4;
  }
}

// Bytes of a mipmapped array: every level, each half the previous (at least 1).
uint64_t MipmapBytes(uint64_t elem, size_t w, size_t h, size_t d, unsigned levels) {
  uint64_t total = 0;
  for (unsigned l = 0; l < (levels ? levels : 1); ++l) {
    uint64_t b = Mul(Mul(Mul(elem, Dim(w)), Dim(h)), Dim(d));
    total = b > UINT64_MAX - total ? UINT64_MAX : total + b;
    w = w > 1 ? w / 2 : w;
    h = h > 1 ? h / 2 : h;
    d = d > 1 ? d / 2 : d;
  }
  return total;
}

// Padding of a pitched allocation, counted once the pitch is known.
void AddPitchPadding(int dev, const void* key, uint64_t bytes_now) {
  State& s = S();
  if (!key || !s.cap[dev]) return;
  Locked lk(s);
  if (Entry* x = s.allocs.Find(key)) {
    if (bytes_now > x->bytes) {
      AddLocked(s, dev, bytes_now - x->bytes);
      x->bytes = bytes_now;
    }
  }
}

}  // namespace

extern "C" {

hipError_t hipMalloc(void** ptr, size_t size) {
  REAL(hipMalloc, hipError_t (*)(void**, size_t));
  if (!real) return hipErrorNotInitialized;
  return Capped(CurrentDevice(), size, ptr, [&] { return real(ptr, size); });
}

hipError_t hipExtMallocWithFlags(void** ptr, size_t size, unsigned int flags) {
  REAL(hipExtMallocWithFlags, hipError_t (*)(void**, size_t, unsigned int));
  if (!real) return hipErrorNotInitialized;
  return Capped(CurrentDevice(), size, ptr, [&] { return real(ptr, size, flags); });
}

hipError_t hipMallocManaged(void** ptr, size_t size, unsigned int flags) {
  REAL(hipMallocManaged, hipError_t (*)(void**, size_t, unsigned int));
  if (!real) return hipErrorNotInitialized;
  return Capped(CurrentDevice(), size, ptr, [&] { return real(ptr, size, flags); });
}

hipError_t hipMallocPitch(void** ptr, size_t* pitch, size_t width, size_t height) {
  REAL(hipMallocPitch, hipError_t (*)(void**, size_t*, size_t, size_t));
  if (!real) return hipErrorNotInitialized;
  // The pitch is only known afterwards: reserve the unpadded size, then count
  // the padding too (without a second check) and track what was allocated.
  int dev = CurrentDevice();
  bool outer = t_depth == 0;
  hipError_t e = Capped(dev, Mul(width, height), ptr, [&] { return real(ptr, pitch, width, height); });
  if (outer && e == hipSuccess && ptr && *ptr && pitch && *pitch > width) AddPitchPadding(dev, *ptr, Mul(*pitch, height));
  return e;
}

hipError_t hipMallocAsync(void** ptr, size_t size, hipStream_t stream) {
  REAL(hipMallocAsync, hipError_t (*)(void**, size_t, hipStream_t));
  if (!real) return hipErrorNotInitialized;
  int dev = StreamDevice(stream);
  bool outer = t_depth == 0;
  hipError_t e = Capped(dev, size, ptr, [&] { return real(ptr, size, stream); });
  if (outer && e == hipSuccess && ptr && *ptr) MarkPooled(*ptr, dev, CurrentPool(dev));
  return e;
}

hipError_t hipMallocFromPoolAsync(void** ptr, size_t size, hipMemPool_t pool, hipStream_t stream) {
  REAL(hipMallocFromPoolAsync, hipError_t (*)(void**, size_t, hipMemPool_t, hipStream_t));
  if (!real) return hipErrorNotInitialized;
  int dev = StreamDevice(stream);
  bool outer = t_depth == 0;
  hipError_t e = Capped(dev, size, ptr, [&] { return real(ptr, size, pool, stream); });
  if (outer && e == hipSuccess && ptr && *ptr) MarkPooled(*ptr, dev, pool);
  return e;
}

hipError_t hipFree(void* ptr) {
  REAL(hipFree, hipError_t (*)(void*));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(ptr);
  if (e == hipSuccess) Untrack(ptr);
  return e;
}

hipError_t hipFreeAsync(void* ptr, hipStream_t stream) {
  REAL(hipFreeAsync, hipError_t (*)(void*, hipStream_t));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(ptr, stream);
  if (e == hipSuccess) Untrack(ptr);  // a pool block: counted until the pool gives it back
  return e;
}

// 3D, array and mipmap allocations: device memory like any other. Sizes are
// computed saturating (an overflowing extent is refused at the cap), pitched
// ones counted at the padded pitch once it is known.
hipError_t hipMalloc3D(hipPitchedPtr* pitched, hipExtent extent) {
  REAL(hipMalloc3D, hipError_t (*)(hipPitchedPtr*, hipExtent));
  if (!real) return hipErrorNotInitialized;
  if (!pitched) return real(pitched, extent);
  int dev = CurrentDevice();
  bool outer = t_depth == 0;
  uint64_t rows = Mul(Dim(extent.height), Dim(extent.depth));
  hipError_t e = Capped(dev, Mul(extent.width, rows), &pitched->ptr, [&] { return real(pitched, extent); });
  if (outer && e == hipSuccess && pitched->ptr && pitched->pitch > extent.width)
    AddPitchPadding(dev, pitched->ptr, Mul(pitched->pitch, rows));
  return e;
}

hipError_t hipMemAllocPitch(hipDeviceptr_t* dptr, size_t* pitch, size_t width, size_t height, unsigned int elem) {
  REAL(hipMemAllocPitch, hipError_t (*)(hipDeviceptr_t*, size_t*, size_t, size_t, unsigned int));
  if (!real) return hipErrorNotInitialized;
  int dev = CurrentDevice();
  bool outer = t_depth == 0;
  hipError_t e = Capped(dev, Mul(width, height), reinterpret_cast<void**>(dptr),
                        [&] { return real(dptr, pitch, width, height, elem); });
  if (outer && e == hipSuccess && dptr && *dptr && pitch && *pitch > width)
    AddPitchPadding(dev, *dptr, Mul(*pitch, height));
  return e;
}

hipError_t hipMallocArray(hipArray_t* array, const hipChannelFormatDesc* desc, size_t width, size_t height,
                          unsigned int flags) {
  REAL(hipMallocArray, hipError_t (*)(hipArray_t*, const hipChannelFormatDesc*, size_t, size_t, unsigned int));
  if (!real) return hipErrorNotInitialized;
  uint64_t bytes = Mul(Mul(ChannelBytes(desc), Dim(width)), Dim(height));
  return Capped(CurrentDevice(), bytes, reinterpret_cast<void**>(array),
                [&] { return real(array, desc, width, height, flags); });
}

hipError_t hipMalloc3DArray(hipArray_t* array, const hipChannelFormatDesc* desc, hipExtent extent,
                            unsigned int flags) {
  REAL(hipMalloc3DArray, hipError_t (*)(hipArray_t*, const hipChannelFormatDesc*, hipExtent, unsigned int));
  if (!real) return hipErrorNotInitialized;
  uint64_t bytes = Mul(Mul(Mul(ChannelBytes(desc), Dim(extent.width)), Dim(extent.height)), Dim(extent.depth));
  return Capped(CurrentDevice(), bytes, reinterpret_cast<void**>(array),
                [&] { return real(array, desc, extent, flags); });
}

hipError_t hipArrayCreate(hipArray_t* array, const HIP_ARRAY_DESCRIPTOR* d) {
  REAL(hipArrayCreate, hipError_t (*)(hipArray_t*, const HIP_ARRAY_DESCRIPTOR*));
  if (!real) return hipErrorNotInitialized;
  if (!d) return real(array, d);
  uint64_t bytes = Mul(Mul(Mul(FormatBytes(d->Format), Dim(d->NumChannels)), Dim(d->Width)), Dim(d->Height));
  return Capped(CurrentDevice(), bytes, reinterpret_cast<void**>(array), [&] { return real(array, d); });
}

hipError_t hipArray3DCreate(hipArray_t* array, const HIP_ARRAY3D_DESCRIPTOR* d) {
  REAL(hipArray3DCreate, hipError_t (*)(hipArray_t*, const HIP_ARRAY3D_DESCRIPTOR*));
  if (!real) return hipErrorNotInitialized;
  if (!d) return real(array, d);
  uint64_t bytes = Mul(Mul(Mul(Mul(FormatBytes(d->Format), Dim(d->NumChannels)), Dim(d->Width)), Dim(d->Height)),
                       Dim(d->Depth));
  return Capped(CurrentDevice(), bytes, reinterpret_cast<void**>(array), [&] { return real(array, d); });
}

hipError_t hipMallocMipmappedArray(hipMipmappedArray_t* mm, const hipChannelFormatDesc* desc, hipExtent extent,
                                   unsigned int levels, unsigned int flags) {
  REAL(hipMallocMipmappedArray,
       hipError_t (*)(hipMipmappedArray_t*, const hipChannelFormatDesc*, hipExtent, unsigned int, unsigned int));
  if (!real) return hipErrorNotInitialized;
  uint64_t bytes = MipmapBytes(ChannelBytes(desc), extent.width, extent.height, extent.depth, levels);
  return Capped(CurrentDevice(), bytes, reinterpret_cast<void**>(mm),
                [&] { return real(mm, desc, extent, levels, flags); });
}

hipError_t hipMipmappedArrayCreate(hipMipmappedArray_t* mm, HIP_ARRAY3D_DESCRIPTOR* d, unsigned int levels) {
  REAL(hipMipmappedArrayCreate, hipError_t (*)(hipMipmappedArray_t*, HIP_ARRAY3D_DESCRIPTOR*, unsigned int));
  if (!real) return hipErrorNotInitialized;
  if (!d) return real(mm, d, levels);
  uint64_t bytes = MipmapBytes(Mul(FormatBytes(d->Format), Dim(d->NumChannels)), d->Width, d->Height, d->Depth,
                               levels);
  return Capped(CurrentDevice(), bytes, reinterpret_cast<void**>(mm), [&] { return real(mm, d, levels); });
}

hipError_t hipFreeArray(hipArray_t array) {
  REAL(hipFreeArray, hipError_t (*)(hipArray_t));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(array);
  if (e == hipSuccess) Untrack(array);
  return e;
}

hipError_t hipArrayDestroy(hipArray_t array) {
  REAL(hipArrayDestroy, hipError_t (*)(hipArray_t));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(array);
  if (e == hipSuccess) Untrack(array);
  return e;
}

hipError_t hipFreeMipmappedArray(hipMipmappedArray_t mm) {
  REAL(hipFreeMipmappedArray, hipError_t (*)(hipMipmappedArray_t));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(mm);
  if (e == hipSuccess) Untrack(mm);
  return e;
}

hipError_t hipMipmappedArrayDestroy(hipMipmappedArray_t mm) {
  REAL(hipMipmappedArrayDestroy, hipError_t (*)(hipMipmappedArray_t));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(mm);
  if (e == hipSuccess) Untrack(mm);
  return e;
}

// Virtual memory management (PyTorch's expandable segments): physical memory
// is created per handle.
hipError_t hipMemCreate(hipMemGenericAllocationHandle_t* handle, size_t size, const hipMemAllocationProp* prop,
                        unsigned long long flags) {
  REAL(hipMemCreate,
       hipError_t (*)(hipMemGenericAllocationHandle_t*, size_t, const hipMemAllocationProp*, unsigned long long));
  if (!real) return hipErrorNotInitialized;
  int dev = (prop && prop->location.type == hipMemLocationTypeDevice && prop->location.id >= 0 &&
             prop->location.id < kMaxDevices)
                ? prop->location.id
                : CurrentDevice();
  return Capped(dev, size, reinterpret_cast<void**>(handle), [&] { return real(handle, size, prop, flags); });
}

hipError_t hipMemRelease(hipMemGenericAllocationHandle_t handle) {
  REAL(hipMemRelease, hipError_t (*)(hipMemGenericAllocationHandle_t));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(handle);
  if (e == hipSuccess) Untrack(handle);
  return e;
}

// What the device "has": the cap, and what is left of it.
hipError_t hipMemGetInfo(size_t* free_bytes, size_t* total_bytes) {
  REAL(hipMemGetInfo, hipError_t (*)(size_t*, size_t*));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(free_bytes, total_bytes);
  int dev = CurrentDevice();
  State& s = S();
  if (e != hipSuccess || !s.cap[dev]) return e;
  Locked lk(s);
  if (s.area) ReclaimDead(s.area, s.slot, false);  // what died without saying so is free again
  // Blocks freed to a stream-ordered pool count as free here: an allocation
  // that needs them trims the pools first (Reserve -> ReconcilePools).
  uint64_t used = UsedLocked(s, dev);
  used -= Min(used, s.pool_held[dev]);
  uint64_t left = s.cap[dev] - Min(used, s.cap[dev]);
  if (free_bytes) *free_bytes = Min<uint64_t>(*free_bytes, left);
  if (total_bytes) *total_bytes = Min<uint64_t>(*total_bytes, s.cap[dev]);
  return e;
}

hipError_t hipDeviceTotalMem(size_t* bytes, hipDevice_t device) {
  REAL(hipDeviceTotalMem, hipError_t (*)(size_t*, hipDevice_t));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(bytes, device);
  if (e == hipSuccess && bytes && device >= 0 && device < kMaxDevices && S().cap[device])
    *bytes = Min<uint64_t>(*bytes, S().cap[device]);
  return e;
}

hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* prop, int device) {
  REAL(hipGetDevicePropertiesR0600, hipError_t (*)(hipDeviceProp_tR0600*, int));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(prop, device);
  if (e == hipSuccess && prop && device >= 0 && device < kMaxDevices && S().cap[device])
    prop->totalGlobalMem = Min<uint64_t>(prop->totalGlobalMem, S().cap[device]);
  return e;
}

// The pre-R0600 symbol binaries built with HIP 5 import (hipDeviceProp_tR0000).
hipError_t LegacyGetDeviceProperties(hipDeviceProp_tR0000* prop, int device) __asm__("hipGetDeviceProperties");
hipError_t LegacyGetDeviceProperties(hipDeviceProp_tR0000* prop, int device) {
  static std::atomic<void*> slot{nullptr};
  auto real = reinterpret_cast<hipError_t (*)(hipDeviceProp_tR0000*, int)>(Cached(slot, "hipGetDeviceProperties"));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(prop, device);
  if (e == hipSuccess && prop && device >= 0 && device < kMaxDevices && S().cap[device])
    prop->totalGlobalMem = Min<uint64_t>(prop->totalGlobalMem, S().cap[device]);
  return e;
}

}  // extern "C"
