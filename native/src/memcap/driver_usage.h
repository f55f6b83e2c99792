// Driver-side truth for HBM grants: what every process holds on every GPU as
// the amdgpu driver accounts it, attributed to the memory-unit grants.
//
// The HBM-cap shim (native/memcap/memcap.cc) counts inside the container, so
// it cannot see a process that goes around it: a dlsym()/ctypes call into
// libamdhip64, HSA-direct allocations, a forged used[] in the (container-
// writable) accounting file, a process started without the shim. The driver
// sees all of them. The source is DRM fdinfo (/proc/<pid>/fdinfo/<fd> of each
// render-node descriptor: drm-pdev, drm-client-id, drm-resident-vram): it is
// per process, counts the KFD (HIP) allocations of the process's GPU VM, and --
// unlike amdsmi_get_gpu_process_list, whose PIDs are the host's (measured:
// profiles/r3/driver/driver_usage.json) -- it is read in the PID namespace of
// the /proc it comes from, so it attributes correctly wherever that /proc is
// mounted from (hostPID, or the host's /proc at --host-proc).
//
// Attribution: a process that has its grant's accounting file mapped (the shim
// maps it; /proc/<pid>/maps device + inode equal the daemon's file) belongs to
// that grant; a process without the shim belongs to the grant of a process in
// the same cgroup (the same container), unless that cgroup is the daemon's
// own. Everything else on a GPU is "unattributed".
//
// The reference has nothing of the kind: it counts memory units and never
// looks at what a pod uses (/root/reference/cmd/nvidia-device-plugin/
// server.go:99-111).
#pragma once

#include <stdint.h>
#include <sys/types.h>

#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <string_view>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "common/status.h"

namespace adp::memcap {

// One process's HBM on one GPU.
struct ProcessHbm {
  int pid = 0;
  std::string bdf;       // drm-pdev
  uint64_t bytes = 0;    // drm-resident-vram (drm-memory-vram on older kernels)
  std::string cgroup;    // /proc/<pid>/cgroup (first line)
  std::string grant;     // grant key ("" = unattributed)
  bool via_cgroup = false;  // attributed through a cgroup sibling, not its own mapping
};

struct DriverScan {
  std::vector<ProcessHbm> procs;
  std::map<std::pair<std::string, std::string>, uint64_t> by_grant;  // (key, bdf) -> bytes
  std::map<std::pair<std::string, std::string>, int> grant_procs;    // (key, bdf) -> processes
  std::map<std::string, uint64_t> total;         // bdf -> bytes of every client seen
  std::map<std::string, uint64_t> unattributed;  // bdf -> bytes outside every grant
  size_t pids_scanned = 0;
  size_t fd_dirs_unreadable = 0;  // processes whose fds this daemon may not read (privileges)
  size_t fd_entries = 0;          // descriptor links examined (the scan's cost)
  // Where the candidate PIDs came from: "kfd" (the driver's list of GPU
  // processes, /sys/class/kfd/kfd/proc) or "proc" (every process).
  std::string pid_source = "proc";
  // Processes holding VRAM through a render node without /dev/kfd open (Mesa,
  // Vulkan, VA-API, a child that inherited the fd, raw amdgpu GEM ioctls): in
  // no KFD list, so only a full walk finds them (ScanState).
  size_t render_only = 0;
};

// What one scanner carries from scan to scan. KFD lists only the processes
// that opened /dev/kfd; a render-node-only VRAM holder is in no such list and
// the fast path alone would never see it -- a bypass of the in-process cap.
// So the first scan, and one every `full_walk_ms`, walks every process; the
// render-only holders it finds are read on every fast-path scan in between
// (their bytes do not vanish and reappear), and a new one is found within
// `full_walk_ms`.
struct ScanState {
  int64_t full_walk_ms = 60000;  // 0: only the first scan walks everything
  int64_t last_full_ms = -1;     // steady clock of the last full walk (-1: none yet)
  std::vector<std::string> render_only_pids;
  uint64_t full_walks = 0;
};
// ADP_DRIVER_FULL_WALK_MS, else 60000.
int64_t FullWalkMsFromEnv();

// A grant's accounting file as the daemon sees it: processes that mapped it
// show the same device and inode in /proc/<pid>/maps.
struct GrantFile {
  std::string key;
  unsigned dev_major = 0, dev_minor = 0;
  uint64_t ino = 0;
};
std::vector<GrantFile> ListGrantFiles(const std::string& usage_dir);

// "1195280 KiB" -> bytes; bare numbers are bytes.
uint64_t ParseFdinfoSize(const std::string& value);

// One pass over <proc_root>/<pid>/fd. `self_cgroup`: the daemon's own cgroup,
// never used for sibling attribution. With `kfd_proc_dir` (KFD's sysfs list of
// the processes that opened /dev/kfd, named by host PID) only those PIDs are
// read, so the cost follows the GPU processes, not every descriptor on the
// node; the full walk remains when that directory is absent or none of its
// PIDs is under `proc_root` (a /proc of another PID namespace).
// `state` (may be null: then the KFD list alone, as before) makes the fast
// path periodic full walks plus the render-only holders they found.
DriverScan ScanDriverHbm(const std::string& proc_root, const std::vector<GrantFile>& grants,
                         const std::string& self_cgroup, const std::string& kfd_proc_dir = "",
                         ScanState* state = nullptr);

// The cgroup line of the calling process ("" if unreadable).
std::string SelfCgroup();

// Recomputes a scan's per-GPU and per-grant sums from its process rows.
void Aggregate(DriverScan* s);

// The scan as the event relay sends it (health/relay.h): a header line
// "scan\t<pid source>\t<pids>\t<fds>\t<unreadable>\t<n>\t<render only>" and n lines
// "p\t<pid>\t<bdf>\t<bytes>\t<grant>\t<via cgroup 0|1>\t<cgroup>".
std::string SerializeScan(const DriverScan& s);
// Parses one complete reply at the start of `text`; `consumed` gets its length.
// kIncomplete: a prefix of a reply (wait for more bytes); kMalformed: no reply
// can start this way (fail at once). A relay of the previous version (no
// render-only field) is read too.
enum class ParseResult { kOk, kIncomplete, kMalformed };
ParseResult ParseScanReply(std::string_view text, DriverScan* out, size_t* consumed);
// ParseScanReply == kOk.
bool ParseScan(std::string_view text, DriverScan* out, size_t* consumed);
// Asks the event relay connected on `fd` for a scan (the relay holds the
// privilege to read other containers' /proc/<pid>/fd): usage_dir and the
// daemon's own cgroup as the relay should use them. A readable `cancel_fd`
// (>= 0) ends the wait early (the monitor's stop).
Result<DriverScan> RemoteScan(int fd, const std::string& usage_dir, const std::string& self_cgroup, int timeout_ms,
                              int cancel_fd = -1);

// Polls ScanDriverHbm and checks every grant against the driver: a grant is
// over when its processes hold more on a GPU than granted there plus `slack`
// per process (the HIP runtime's own allocations -- code objects, queues,
// scratch -- never pass through hipMalloc; about 0.1 GiB per process measured
// on MI355X). Transitions into "over" are counted.
class DriverHbmMonitor {
 public:
  struct Options {
    std::string proc_root = "/proc";
    std::string kfd_proc_dir = "/sys/class/kfd/kfd/proc";  // "" = always walk every process
    std::string usage_dir;
    // Non-empty: the event relay's socket; scans run there (RemoteScan), with
    // the relay's own /proc and KFD list, and proc_root/kfd_proc_dir are unused.
    std::string relay_socket;
    int poll_ms = 10000;
    uint64_t slack_bytes = 512ull << 20;
  };
  // key -> bdf -> granted bytes, for every live grant (called on the poll thread).
  using GrantFn = std::function<std::map<std::string, std::map<std::string, uint64_t>>()>;

  struct GrantState {
    uint64_t driver_bytes = 0;
    uint64_t granted_bytes = 0;
    int processes = 0;
    bool over = false;
    uint64_t over_transitions = 0;
  };
  struct Snapshot {
    DriverScan scan;
    std::map<std::pair<std::string, std::string>, GrantState> grants;  // (key, bdf)
    uint64_t polls = 0;
    uint64_t over_total = 0;  // every transition into "over", all grants
    uint64_t slack_bytes = 0;
    uint64_t last_scan_ns = 0;   // wall time of the last scan
    uint64_t scan_ns_total = 0;  // all scans
    uint64_t scan_failures = 0;  // relay scans that failed (the previous scan stays)
    std::string scan_error;      // the last failure's reason, "" once a scan succeeds again
    bool remote = false;         // scans run in the event relay
    size_t render_only = 0;      // render-node-only VRAM holders at the last full walk
    bool render_only_logged = false;
    uint64_t full_walks = 0;     // scans that walked every process (local scans)
  };

  DriverHbmMonitor(Options opts, GrantFn grants);
  ~DriverHbmMonitor();
  void Start();
  void Stop();
  void PollOnce();
  Snapshot Get() const;

 private:
  Options opts_;
  GrantFn grants_;
  std::string self_cgroup_;
  mutable std::mutex mu_;
  Snapshot snap_;
  std::map<std::pair<std::string, std::string>, uint64_t> transitions_;
  ScanState scan_state_;  // local scans (the relay keeps its own)
  std::atomic<bool> stop_{false};
  int wake_fd_ = -1;
  std::thread thread_;
};

}  // namespace adp::memcap
