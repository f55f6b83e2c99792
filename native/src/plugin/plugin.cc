#include "plugin/plugin.h"

#include <errno.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <tuple>
#include <set>
#include <map>
#include <chrono>
#include <cstring>
#include <future>
#include <thread>

#include "common/log.h"
#include "common/strings.h"
#include "memcap/usage.h"
#include "memcap_area.h"
#include "proto/messages.h"
#include "proto/wire.h"

namespace adp::plugin {
namespace {

constexpr const char* kComp = "plugin";
constexpr const char* kSvc = "/v1beta1.DevicePlugin/";


}  // namespace

bool ParseDeviceListStrategy(std::string_view s, DeviceListStrategy* out) {
  if (s == "envvar") { *out = DeviceListStrategy::kEnvvar; return true; }
  if (s == "volume-mounts") { *out = DeviceListStrategy::kVolumeMounts; return true; }
  if (s == "cdi-annotations") { *out = DeviceListStrategy::kCdiAnnotations; return true; }
  if (s == "cdi-cri") { *out = DeviceListStrategy::kCdiCri; return true; }
  return false;
}

bool ParseDeviceIdStrategy(std::string_view s, DeviceIdStrategy* out) {
  if (s == "uuid") { *out = DeviceIdStrategy::kUuid; return true; }
  if (s == "index") { *out = DeviceIdStrategy::kIndex; return true; }
  return false;
}

std::vector<std::pair<uint32_t, uint32_t>> ReplicaCuRanges(uint32_t cus, uint32_t xcds, unsigned replicas) {
  std::vector<std::pair<uint32_t, uint32_t>> out;
  if (replicas < 2 || cus == 0 || xcds == 0 || cus % xcds != 0) return out;
  const uint32_t per = cus / xcds;  // CUs per XCD
  if (replicas > per) return out;
  for (unsigned r = 0; r < replicas; ++r) {
    uint32_t lo = static_cast<uint32_t>(uint64_t(r) * per / replicas) * xcds;
    uint32_t hi = static_cast<uint32_t>(uint64_t(r + 1) * per / replicas) * xcds - 1;
    out.emplace_back(lo, hi);
  }
  return out;
}

std::vector<std::pair<uint32_t, uint32_t>> MemoryUnitCuRanges(uint32_t cus, uint32_t xcds, unsigned units) {
  std::vector<std::pair<uint32_t, uint32_t>> out;
  if (units < 2 || cus == 0 || xcds == 0 || cus % xcds != 0) return out;
  const uint32_t per = cus / xcds;
  // Slots follow the IDs' lexicographic order ("-replica-0" < "-replica-1" <
  // "-replica-10" < ...), the order the replica prioritizer takes free IDs in:
  // a pack request gets consecutive ranks, hence contiguous slots.
  std::vector<unsigned> by_name(units);
  for (unsigned r = 0; r < units; ++r) by_name[r] = r;
  std::sort(by_name.begin(), by_name.end(),
            [](unsigned a, unsigned b) { return std::to_string(a) < std::to_string(b); });
  out.resize(units);
  for (unsigned rank = 0; rank < units; ++rank) {
    uint32_t slot = static_cast<uint32_t>(uint64_t(rank) * per / units);
    out[by_name[rank]] = {slot * xcds, slot * xcds + xcds - 1};
  }
  return out;
}

double CpuBudget() {
  // The affinity mask first (taskset, cpuset cgroups)...
  cpu_set_t set;
  double cpus = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set)
                                                              : std::max(1u, std::thread::hardware_concurrency());
  // ... then a CFS quota: a DaemonSet with resources.limits.cpu. cgroup v2
  // "cpu.max" is "<quota> <period>" or "max <period>"; v1 splits it in two files.
  const char* env = getenv("ADP_CGROUP_ROOT");  // tests point this at a fake tree
  std::string root = env && *env ? env : "/sys/fs/cgroup";
  double quota = 0;
  if (FILE* f = fopen((root + "/cpu.max").c_str(), "r")) {
    char q[32] = {0};
    unsigned long long period = 0;
    if (fscanf(f, "%31s %llu", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
      quota = strtod(q, nullptr) / static_cast<double>(period);
    fclose(f);
  } else if (FILE* fq = fopen((root + "/cpu/cpu.cfs_quota_us").c_str(), "r")) {
    long long q = -1, period = 0;
    if (fscanf(fq, "%lld", &q) != 1) q = -1;
    fclose(fq);
    if (FILE* fp = fopen((root + "/cpu/cpu.cfs_period_us").c_str(), "r")) {
      if (fscanf(fp, "%lld", &period) != 1) period = 0;
      fclose(fp);
    }
    if (q > 0 && period > 0) quota = static_cast<double>(q) / static_cast<double>(period);
  }
  return quota > 0 ? std::min(cpus, quota) : cpus;
}

int DefaultServerThreads() {
  double budget = CpuBudget();
  return static_cast<int>(std::clamp(std::ceil(budget), 1.0, 8.0));
}

Plugin::Plugin(std::shared_ptr<const inventory::Snapshot> snap, strategy::PluginSpec spec,
               PluginOptions opts)
    : snap_(std::move(snap)), spec_(std::move(spec)), opts_(std::move(opts)) {
  if (opts_.kubelet_socket.empty()) opts_.kubelet_socket = PathJoin(opts_.plugin_dir, "kubelet.sock");
  if (opts_.quiet) {
    QuietLogs q;
    BuildUnits();
  } else {
    BuildUnits();
  }
}

Plugin::~Plugin() { Stop(); }

std::string Plugin::socket_path() const { return PathJoin(opts_.plugin_dir, spec_.socket_name); }

bool Plugin::owns_socket() const {
  std::lock_guard<std::mutex> lk(server_mu_);
  return server_ && server_->OwnsSocketPath();
}

static bool OrderForHip(const inventory::Snapshot& snap, std::vector<alloc::DeviceRef>* devices) {
  // ROCr creates one agent per KFD topology node whose render node the process
  // can open, in node order, and HIP numbers its devices after the agents: a
  // container given these devices sees them in KFD-node order, whatever order
  // amdsmi enumerated them in. Unit order is that order, so every per-device
  // list a container gets (HSA_CU_MASK agent numbers, AMD_GPU_MEMORY_* lists,
  // grant/<ordinal> mounts) lines up with its HIP ordinals.
  auto node = [&](const alloc::DeviceRef& r) {
    const auto& g = snap.gpus[r.gpu];
    return r.partition < 0 ? g.kfd_node : g.partitions[r.partition].kfd_node;
  };
  for (const auto& r : *devices)
    if (node(r) == inventory::kNoKfdNode) return false;  // unknown: amdsmi order, the best guess left
  std::stable_sort(devices->begin(), devices->end(),
                   [&](const alloc::DeviceRef& a, const alloc::DeviceRef& b) { return node(a) < node(b); });
  return true;
}

void Plugin::BuildUnits() {
  const auto& v = spec_.variant;
  std::vector<alloc::DeviceRef> amdsmi_order = spec_.devices;
  hip_order_known_ = OrderForHip(*snap_, &spec_.devices);
  if (!hip_order_known_ && spec_.devices.size() > 1)
    LOG_WARN(kComp, "'%s': amdsmi does not report KFD topology nodes; per-device container lists (HSA_CU_MASK, "
             "AMD_GPU_MEMORY_*) assume HIP numbers devices in amdsmi order", spec_.resource_name.c_str());
  else if (!std::equal(amdsmi_order.begin(), amdsmi_order.end(), spec_.devices.begin(),
                       [](const alloc::DeviceRef& a, const alloc::DeviceRef& b) {
                         return a.gpu == b.gpu && a.partition == b.partition;
                       }))
    LOG_INFO(kComp, "'%s': KFD topology order differs from amdsmi order; containers' devices are listed in KFD "
             "(HIP) order", spec_.resource_name.c_str());
  replicated_ = v.replicas > 1 || v.auto_replicas;
  memory_units_ = v.auto_replicas;
  // Per resource: the resource-config entry's own policy, else --replica-policy,
  // else (auto) pack for memory units -- a grant's HBM must come from as few
  // devices as possible -- and the reference's spread for time-slice replicas
  // (replica.go:149-190).
  replica_policy_ = v.policy != alloc::ReplicaPolicy::kAuto             ? v.policy
                    : opts_.replica_policy != alloc::ReplicaPolicy::kAuto ? opts_.replica_policy
                    : memory_units_                                     ? alloc::ReplicaPolicy::kPack
                                                                        : alloc::ReplicaPolicy::kSpread;
  hbm_grants_ = memory_units_ || (opts_.replica_hbm_share && replicated_);
  for (const auto& ref : spec_.devices) units_.push_back(MakeUnit(ref));
  if (memory_units_) CheckMemoryUnitName();
  if (replicated_)
    LOG_INFO(kComp, "'%s': preferred allocation %s replicas (%s)", spec_.resource_name.c_str(),
             replica_policy_ == alloc::ReplicaPolicy::kPack ? "packs" : "spreads",
             v.policy != alloc::ReplicaPolicy::kAuto             ? "resource-config entry"
             : opts_.replica_policy != alloc::ReplicaPolicy::kAuto ? "--replica-policy"
             : memory_units_                                     ? "auto: memory units"
                                                                 : "auto: time-slice replicas");
  BuildAdvertised();
  if (hbm_grants_ && !opts_.memcap_host_path.empty()) BuildMemcapBytes();
  pb::DeviceSpec kfd{"/dev/kfd", PathJoin(opts_.driver_root, "/dev/kfd"), "rw"};
  std::string kb;
  pb::Encode(kfd, &kb);
  pb::PutLen(&kfd_spec_bytes_, 3, kb);
  graph_ = alloc::DeviceGraph(*snap_, spec_.devices);
  if (!replicated_ && units_.size() <= 8) {
    // Anonymous zero pages: only the pages of entries actually used get memory.
    void* p = mmap(nullptr, kBestEffortCacheBytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p != MAP_FAILED) best_effort_cache_.reset(static_cast<std::atomic<uint16_t>*>(p));
  }
  healthy_.assign(units_.size(), 1);
  warned_law_.reset(new std::atomic<uint64_t>[units_.size()]());
  RebuildListAndWatch();
  // grpc-go clients -- the kubelet's device manager dials without raising it --
  // refuse messages above 4 MiB, so a larger device list never reaches the
  // kubelet and the resource stays at 0 allocatable.
  constexpr size_t kKubeletMaxRecv = 4u << 20;
  if (law_bytes_size_.load() + 5 > kKubeletMaxRecv)
    LOG_ERROR(kComp, "'%s': the ListAndWatch device list is %zu bytes (%zu IDs), above the 4 MiB a kubelet's gRPC "
              "client accepts; the kubelet will not see these devices. Lower the replica count (resource-config) "
              "or raise the memory unit (--auto-replica-unit-mib)", spec_.resource_name.c_str(),
              law_bytes_size_.load(), advertised_.size());
}

// One advertised device (a whole GPU or a partition) with everything Allocate
// hands out for it encoded once.
Unit Plugin::MakeUnit(const alloc::DeviceRef& ref) const {
  const auto& v = spec_.variant;
  const auto& g = snap_->gpus[ref.gpu];
  Unit u;
  u.gpu = ref.gpu;
  if (ref.partition < 0) {
    u.id = g.uuid;
    u.index = std::to_string(g.node_index);
    u.numa = g.numa;
    u.vram_mib = g.vram_mib;
    for (const auto& p : g.partitions) {
      if (!p.render_path.empty()) u.paths.push_back(p.render_path);
      if (!p.card_path.empty()) u.paths.push_back(p.card_path);
      u.handles.push_back(p.handle);
    }
  } else {
    const auto& p = g.partitions[ref.partition];
    u.id = p.uuid;
    u.index = std::to_string(g.node_index) + ":" + std::to_string(ref.partition);
    u.numa = p.numa >= 0 ? p.numa : g.numa;
    u.vram_mib = p.vram_mib;
    if (!p.render_path.empty()) u.paths.push_back(p.render_path);
    if (!p.card_path.empty()) u.paths.push_back(p.card_path);
    u.handles.push_back(p.handle);
  }
  // Auto replicas: one per `auto_replica_unit_mib` of this device's own memory
  // (server.go:100-103; per-partition memory fixes B4). At least one.
  u.replicas = v.auto_replicas
                   ? static_cast<unsigned>(std::max<uint64_t>(1, u.vram_mib / opts_.auto_replica_unit_mib))
                   : std::max(1u, v.replicas);
  if (hbm_grants_) u.grant_mib = memory_units_ ? opts_.auto_replica_unit_mib : u.vram_mib / u.replicas;
  u.cus = ref.partition < 0 ? g.cus : g.partitions[ref.partition].cus;
  u.xcds = ref.partition < 0 ? g.xcds : g.partitions[ref.partition].xcds;
  if (memory_units_ && opts_.cu_slot_units) {
    // One unit = one CU slot (one CU on every XCD) and that slot's share of
    // the HBM: 32 units of 9,215 MiB on an SPX MI355X. Every grant is then a
    // whole number of slots -- no slot is shared, none left idle.
    const uint32_t per = u.xcds && u.cus % u.xcds == 0 ? u.cus / u.xcds : 0;
    if (per >= 2 && u.vram_mib / per > 0) {
      u.replicas = per;
      u.grant_mib = u.vram_mib / per;
    } else {
      LOG_WARN(kComp, "device %s: %u CUs over %u XCDs give no CU slots; its memory units are %llu MiB",
               u.id.c_str(), u.cus, u.xcds, static_cast<unsigned long long>(opts_.auto_replica_unit_mib));
    }
  }
  if (opts_.replica_cu_mask && replicated_) {
    u.replica_cus = memory_units_ ? MemoryUnitCuRanges(u.cus, u.xcds, u.replicas)
                                  : ReplicaCuRanges(u.cus, u.xcds, u.replicas);
    if (memory_units_ && opts_.whole_cu_slots && !u.replica_cus.empty()) {
      u.slot_units.assign(u.cus / u.xcds, 0);
      for (const auto& rg : u.replica_cus) ++u.slot_units[rg.first / u.xcds];
    }
    if (u.replica_cus.empty() && u.replicas > 1)
      LOG_WARN(kComp, "device %s: %u CUs over %u XCDs cannot be split into %u CU shares; its replicas "
               "share all CUs", u.id.c_str(), u.cus, u.xcds, u.replicas);
  }
  u.visible_id = opts_.id_strategy == DeviceIdStrategy::kIndex ? u.index : u.id;
  for (const auto& path : u.paths) {
    pb::DeviceSpec ds{path, PathJoin(opts_.driver_root, path), "rw"};
    std::string b;
    pb::Encode(ds, &b);
    pb::PutLen(&u.spec_bytes, 3, b);
  }
  pb::Mount m{PathJoin(kVolumeMountRoot, u.visible_id), kVolumeMountHostPath, false};
  std::string mb;
  pb::Encode(m, &mb);
  pb::PutLen(&u.mount_bytes, 2, mb);
  return u;
}

// The advertised IDs: one per device, or its replicas' IDs (replicas.cc).
void Plugin::BuildAdvertised() {
  for (size_t i = 0; i < units_.size(); ++i) {
    const auto& u = units_[i];
    unit_by_id_[u.id] = static_cast<int>(i);
    unit_index_by_id_[u.id] = static_cast<int>(i);  // view into units_[i].id (never modified)
    if (replicated_) {
      if (memory_units_)
        LOG_INFO(kComp, "replicating device %s (%s, %llu MiB) %u times: '%s' units of %llu MiB (%s)", u.id.c_str(),
                 u.index.c_str(), static_cast<unsigned long long>(u.vram_mib), u.replicas,
                 spec_.resource_name.c_str(), static_cast<unsigned long long>(u.grant_mib),
                 UnitIsCuSlot(u) ? "cu-slot" : "mib");
      else
        LOG_INFO(kComp, "replicating device %s (%s, %llu MiB) %u times", u.id.c_str(), u.index.c_str(),
                 static_cast<unsigned long long>(u.vram_mib), u.replicas);
      for (unsigned r = 0; r < u.replicas; ++r) {
        advertised_.push_back(alloc::ReplicaId(u.id, r));
        advertised_unit_.push_back(static_cast<int>(i));
      }
    } else {
      advertised_.push_back(u.id);
      advertised_unit_.push_back(static_cast<int>(i));
    }
  }
  advertised_index_.reserve(advertised_.size() * 2);
  for (size_t i = 0; i < advertised_.size(); ++i) {
    if (advertised_[i].size() > 63)
      LOG_WARN(kComp, "device ID '%s' exceeds 63 characters", advertised_[i].c_str());
    advertised_index_[advertised_[i]] = advertised_unit_[i];
  }
}

// What every memory-unit container of an --enforce-memory-units plugin gets:
// the HBM-cap shim, preloaded (and pinned by /etc/ld.so.preload if asked).
void Plugin::BuildMemcapBytes() {
  grant_dir_prefix_ = GrantDir();
  if (grant_dir_prefix_.empty() || grant_dir_prefix_.back() != '/') grant_dir_prefix_ += '/';
  pb::PutMapEntry(&memcap_bytes_, 1, "LD_PRELOAD", kMemcapContainerPath);
  pb::Mount m{kMemcapContainerPath, opts_.memcap_host_path, true};
  std::string mb;
  pb::Encode(m, &mb);
  pb::PutLen(&memcap_bytes_, 2, mb);
  if (!opts_.memcap_preload_list.empty()) {
    pb::Mount pl{"/etc/ld.so.preload", opts_.memcap_preload_list, true};
    std::string pb_;
    pb::Encode(pl, &pb_);
    pb::PutLen(&memcap_bytes_, 2, pb_);
  }
}

bool Plugin::UnitIsCuSlot(const Unit& u) const {
  return memory_units_ && opts_.cu_slot_units && u.grant_mib != opts_.auto_replica_unit_mib;
}

// A resource named for gigabytes whose unit is not about one: with CU-slot
// units (--replica-cu-mask, --auto-replica-unit auto) one "gpu-mem-gb" is
// ~9 GiB on an MI355X, and a pod asking for 16 of them gets half the GPU.
void Plugin::CheckMemoryUnitName() {
  uint64_t common = units_.empty() ? 0 : units_[0].grant_mib;
  bool cu_slot = !units_.empty() && UnitIsCuSlot(units_[0]);
  for (const auto& u : units_) {
    if (u.grant_mib != common) common = 0;
    cu_slot = cu_slot && UnitIsCuSlot(u);
  }
  memory_unit_mib_ = common;
  memory_unit_kind_ = cu_slot ? "cu-slot" : "mib";
  std::string name = ToLower(spec_.resource_name);
  size_t slash = name.rfind('/');
  if (slash != std::string::npos) name = name.substr(slash + 1);
  const bool says_gb = name.find("gb") != std::string::npos || name.find("gib") != std::string::npos ||
                       name.find("mem") != std::string::npos;
  uint64_t lo = units_.empty() ? 0 : units_[0].grant_mib, hi = lo;
  for (const auto& u : units_) {
    lo = std::min(lo, u.grant_mib);
    hi = std::max(hi, u.grant_mib);
  }
  if (says_gb && (lo < 900 || hi > 1100))
    LOG_WARN(kComp, "'%s' is named for gigabytes but one unit is %llu%s MiB (%s units%s): a pod requesting N of it "
             "gets N x that. Name it for what it is (e.g. resourceConfig gpu:gpu-slot:-1) or use 1 GiB units "
             "(--auto-replica-unit mib). The node label amd.com/%s.memory-unit-mib says the size",
             spec_.resource_name.c_str(), static_cast<unsigned long long>(lo),
             hi != lo ? (".." + std::to_string(hi)).c_str() : "", memory_unit_kind_,
             cu_slot ? ": one CU on every XCD each, --replica-cu-mask" : "", name.c_str());
}

std::string Plugin::ReplicaLayout() const {
  if (!replicated_) return "";
  std::string out = memory_units_ ? std::string("memory-units ") + memory_unit_kind_ : std::string("time-slice");
  for (const auto& u : units_)
    out += " " + u.id + "=" + std::to_string(u.replicas) + "x" + std::to_string(u.grant_mib) + "MiB";
  return out;
}

void Plugin::RebuildListAndWatch() {
  // Encode every advertised ID once per health transition; sends reuse the bytes.
  std::string out;
  out.reserve(advertised_.size() * 72);
  std::string dev;
  for (size_t i = 0; i < advertised_.size(); ++i) {
    const Unit& u = units_[advertised_unit_[i]];
    pb::Device d;
    d.id = advertised_[i];
    d.health = healthy_[advertised_unit_[i]] ? pb::kHealthy : pb::kUnhealthy;
    if (u.numa >= 0) {
      d.has_topology = true;
      d.numa_nodes.push_back(u.numa);
    }
    dev.clear();
    pb::Encode(d, &dev);
    pb::PutLen(&out, 1, dev);
  }
  auto snap = std::make_shared<LawSnapshot>();
  snap->version = ++law_version_;
  snap->bytes = std::move(out);
  snap->healthy = healthy_;
  law_bytes_size_.store(snap->bytes.size(), std::memory_order_relaxed);
  size_t unhealthy = 0;
  for (uint8_t h : healthy_) unhealthy += !h;
  unhealthy_units_.store(unhealthy, std::memory_order_relaxed);
  std::lock_guard<std::mutex> lk(law_mu_);
  law_ = std::move(snap);
}

std::shared_ptr<const Plugin::LawSnapshot> Plugin::CurrentLaw() const {
  std::lock_guard<std::mutex> lk(law_mu_);
  return law_;
}

void Plugin::BroadcastLaw(int loop) {
  // Always the newest snapshot (latest wins); a stream that already carries it
  // -- e.g. it opened after the transition -- is not sent a duplicate.
  auto law = CurrentLaw();
  auto& streams = law_streams_[loop];
  size_t keep = 0;
  for (auto& ls : streams) {
    if (ls.stream->closed()) continue;
    if (ls.sent_version != law->version) {
      if (ls.stream->Send(law->bytes)) stats_.law_sends.Add(1);
      ls.sent_version = law->version;
    }
    streams[keep++] = std::move(ls);
  }
  streams.resize(keep);
}

Status Plugin::Register() {
  auto ch = grpc::Channel::Dial(opts_.kubelet_socket, opts_.dial_timeout_ms);
  if (!ch.ok()) return ch.status();
  pb::RegisterRequest rr;
  rr.version = pb::kApiVersion;
  rr.endpoint = BaseName(socket_path());
  rr.resource_name = spec_.resource_name;
  rr.has_options = true;
  rr.options.get_preferred_allocation_available = true;
  rr.options.pre_start_required = opts_.prestart_health_check;
  std::string resp;
  return (*ch)->Unary("/v1beta1.Registration/Register", pb::Encode(rr), &resp,
                      opts_.dial_timeout_ms);
}

std::string GrantFileName(uint64_t mib) { return std::to_string(mib) + ".mib"; }

std::string Plugin::GrantDir() const { return PathJoin(opts_.plugin_dir, "amdgpu-dp/grants"); }

Status Plugin::InstallGrantFiles() const {
  if (memcap_bytes_.empty()) return Status::Ok();
  std::string dir = GrantDir();
  mkdir(PathJoin(opts_.plugin_dir, "amdgpu-dp").c_str(), 0755);
  mkdir(dir.c_str(), 0755);
  std::set<uint64_t> sizes;
  for (const auto& u : units_)
    for (unsigned k = 1; k <= u.replicas && u.grant_mib; ++k) sizes.insert(uint64_t{k} * u.grant_mib);
  for (uint64_t mib : sizes) {
    std::string path = PathJoin(dir, GrantFileName(mib)), want = std::to_string(mib) + "\n";
    if (FILE* f = fopen(path.c_str(), "rb")) {  // present and right: keep the inode running containers mounted
      char buf[32];
      size_t n = fread(buf, 1, sizeof(buf), f);
      fclose(f);
      if (std::string(buf, n) == want) continue;
    }
    std::string tmp = path + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    bool ok = f && fwrite(want.data(), 1, want.size(), f) == want.size();
    if (f) ok = (fclose(f) == 0) && ok;
    if (!ok || chmod(tmp.c_str(), 0444) != 0 || rename(tmp.c_str(), path.c_str()) != 0) {
      int err = errno;
      unlink(tmp.c_str());
      return Internal("cannot write grant file " + path + ": " + strerror(err));
    }
  }
  return Status::Ok();
}

Status Plugin::Start(std::function<void()> on_fatal) {
  if (running()) return FailedPrecondition("plugin already started");
  if (Status gs = InstallGrantFiles(); !gs.ok()) {
    // Without them a container would start with only its (pod-overridable) env caps.
    LOG_ERROR(kComp, "'%s': %s", spec_.resource_name.c_str(), gs.ToString().c_str());
    return gs;
  }
  if (opts_.list_strategy == DeviceListStrategy::kCdiAnnotations ||
      opts_.list_strategy == DeviceListStrategy::kCdiCri) {
    Status cs = WriteCdiSpec();
    if (!cs.ok()) return cs;
  }
  int threads = opts_.server_threads > 0 ? opts_.server_threads : DefaultServerThreads();
  auto srv = std::make_unique<grpc::Server>(spec_.resource_name, threads);
  law_streams_.assign(threads, {});
  srv->set_trace(opts_.trace);
  int spin = opts_.busy_poll_us;
  if (double budget = CpuBudget(); budget < 2 && spin > 0) {
    // Under a CPU quota below two CPUs a spinning loop only burns the quota
    // and gets the process throttled: block in epoll_wait instead.
    static std::atomic<bool> logged{false};
    if (!logged.exchange(true))
      LOG_INFO(kComp, "CPU budget %.2f CPUs: busy-poll off, %d gRPC loop(s) per socket", budget, threads);
    spin = 0;
  }
  srv->set_busy_poll_us(spin);
  srv->set_native_http2(opts_.native_http2);
  srv->set_follow_peer_l3(opts_.follow_peer_l3);
  // Grant accounting files are queued by Allocate(); their writer is woken
  // once the response is on the wire.
  if (!memcap_bytes_.empty() && !opts_.memcap_usage_dir.empty()) srv->set_after_flush([] { memcap::WakeWriter(); });
  srv->AddUnary(std::string(kSvc) + "GetDevicePluginOptions",
                [this](std::string_view q, std::string* r) { return HandleGetOptions(q, r); });
  srv->AddUnary(std::string(kSvc) + "Allocate",
                [this](std::string_view q, std::string* r) { return HandleAllocate(q, r); });
  srv->AddUnary(std::string(kSvc) + "GetPreferredAllocation",
                [this](std::string_view q, std::string* r) { return HandlePreferred(q, r); });
  srv->AddUnary(std::string(kSvc) + "PreStartContainer",
                [this](std::string_view q, std::string* r) { return HandlePreStart(q, r); });
  srv->AddServerStream(std::string(kSvc) + "ListAndWatch",
                       [this](std::string_view, std::shared_ptr<grpc::ServerStream> s) {
                         auto law = CurrentLaw();
                         s->Send(law->bytes);
                         stats_.law_sends.Add(1);
                         law_streams_[s->loop()].push_back({s, law->version});
                         return Status::Ok();
                       });
  // Publish before the loop starts: from here on health updates are posted to the
  // loop (queued until it runs) instead of being applied on the caller's thread.
  grpc::Server* raw = srv.get();
  {
    std::lock_guard<std::mutex> lk(server_mu_);
    server_ = std::move(srv);
  }
  Status st = raw->Listen(socket_path());
  if (st.ok()) st = raw->Start(std::move(on_fatal));
  if (st.ok()) {
    // Block until the server answers, like the reference's self-dial (server.go:207-213).
    auto probe = grpc::Channel::Dial(socket_path(), opts_.dial_timeout_ms);
    if (!probe.ok()) st = probe.status();
  }
  if (!st.ok()) {
    LOG_ERROR(kComp, "could not start device plugin for '%s': %s", spec_.resource_name.c_str(),
              st.ToString().c_str());
    Stop();
    return st;
  }
  LOG_INFO(kComp, "serving '%s' on %s (%zu devices, %zu advertised)", spec_.resource_name.c_str(),
           socket_path().c_str(), units_.size(), advertised_.size());
  if (opts_.register_with_kubelet) {
    st = Register();
    if (!st.ok()) {
      LOG_ERROR(kComp, "could not register device plugin '%s' with kubelet at %s: %s",
                spec_.resource_name.c_str(), opts_.kubelet_socket.c_str(), st.ToString().c_str());
      Stop();
      return st;
    }
    LOG_INFO(kComp, "registered device plugin for '%s' with kubelet", spec_.resource_name.c_str());
    registered_.store(true);
  }
  return Status::Ok();
}

void Plugin::Stop() {
  // Held throughout: the loop thread never takes server_mu_, and a concurrent
  // PostHealth must not fall back to a direct ApplyHealth while the loop still runs.
  std::lock_guard<std::mutex> lk(server_mu_);
  std::unique_ptr<grpc::Server> srv = std::move(server_);
  if (!srv) return;
  registered_.store(false);
  LOG_INFO(kComp, "stopping '%s' on %s", spec_.resource_name.c_str(), socket_path().c_str());
  // End open ListAndWatch streams cleanly (the reference returns nil on stop);
  // each loop finishes the streams it owns.
  struct Pending {
    std::atomic<int> left;
    std::promise<void> done;
  };
  auto pending = std::make_shared<Pending>();
  pending->left.store(srv->loops());
  auto fut = pending->done.get_future();
  srv->PostAll([this, pending](int loop) {
    for (auto& ls : law_streams_[loop]) ls.stream->Finish(Status::Ok());
    law_streams_[loop].clear();
    if (pending->left.fetch_sub(1) == 1) pending->done.set_value();
  });
  fut.wait_for(std::chrono::milliseconds(500));
  srv->Stop();
  for (auto& v : law_streams_) v.clear();
}

bool Plugin::ApplyHealth(const std::vector<int>& us, bool healthy, const std::string& reason) {
  bool changed = false;
  for (int u : us) {
    if (static_cast<bool>(healthy_[u]) == healthy) continue;
    healthy_[u] = healthy ? 1 : 0;
    changed = true;
    LOG_INFO(kComp, "'%s' device %s marked %s: %s", spec_.resource_name.c_str(), units_[u].id.c_str(),
             healthy ? "healthy" : "unhealthy", reason.c_str());
  }
  if (changed) RebuildListAndWatch();
  return changed;
}

void Plugin::SetGpuHealth(int gpu, bool healthy, const std::string& reason) {
  std::vector<int> us;
  for (size_t i = 0; i < units_.size(); ++i)
    if (units_[i].gpu == gpu) us.push_back(static_cast<int>(i));
  PostHealth(std::move(us), healthy, reason);
}

void Plugin::PostHealth(std::vector<int> us, bool healthy, const std::string& reason) {
  if (us.empty()) return;
  std::lock_guard<std::mutex> lk(server_mu_);
  if (server_) {
    // Loops outlive every task they run, so the raw pointer stays valid.
    grpc::Server* srv = server_.get();
    srv->Post([this, srv, us, healthy, reason] {
      if (ApplyHealth(us, healthy, reason)) srv->PostAll([this](int loop) { BroadcastLaw(loop); });
    });
  } else {
    ApplyHealth(us, healthy, reason);  // not serving: the lock serialises callers
  }
}

std::string Plugin::CdiSpecPath() const {
  std::string name = spec_.resource_name;
  for (auto& ch : name)
    if (ch == '/') ch = '-';
  return PathJoin(opts_.cdi_spec_dir, name + ".json");
}

std::string Plugin::CdiSpecJson() const {
  auto node = [&](const std::string& path) {
    return "{\"path\": \"" + JsonEscape(path) + "\", \"hostPath\": \"" +
           JsonEscape(PathJoin(opts_.driver_root, path)) + "\", \"permissions\": \"rw\"}";
  };
  std::string out = "{\n  \"cdiVersion\": \"0.5.0\",\n  \"kind\": \"" + std::string(kCdiVendorClass) +
                    "\",\n  \"containerEdits\": {\"deviceNodes\": [" + node("/dev/kfd") + "]},\n  \"devices\": [";
  for (size_t i = 0; i < units_.size(); ++i) {
    const Unit& u = units_[i];
    out += i ? ",\n    " : "\n    ";
    out += "{\"name\": \"" + JsonEscape(u.visible_id) + "\", \"containerEdits\": {\"deviceNodes\": [";
    for (size_t p = 0; p < u.paths.size(); ++p) out += (p ? ", " : "") + node(u.paths[p]);
    out += "]}}";
  }
  return out + "\n  ]\n}\n";
}

Status Plugin::WriteCdiSpec() const {
  std::string path = CdiSpecPath();
  std::string tmp = path + ".tmp";
  mkdir(opts_.cdi_spec_dir.c_str(), 0755);
  FILE* f = fopen(tmp.c_str(), "w");
  if (!f) return Unavailable("cannot write CDI spec " + tmp + ": " + strerror(errno));
  std::string body = CdiSpecJson();
  bool ok = fwrite(body.data(), 1, body.size(), f) == body.size();
  ok = (fclose(f) == 0) && ok;
  if (!ok || rename(tmp.c_str(), path.c_str()) != 0)
    return Unavailable("cannot write CDI spec " + path + ": " + strerror(errno));
  LOG_INFO(kComp, "wrote CDI spec %s (%zu devices)", path.c_str(), units_.size());
  return Status::Ok();
}

}  // namespace adp::plugin
