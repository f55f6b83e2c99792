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

uint64_t NowNs() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Whether an ID occurs twice (a pod's k is small: pairwise up to 16, else sorted).
bool HasDuplicate(const std::vector<std::string>& ids) {
  if (ids.size() <= 16) {
    for (size_t i = 1; i < ids.size(); ++i)
      for (size_t j = 0; j < i; ++j)
        if (ids[i] == ids[j]) return true;
    return false;
  }
  std::vector<std::string_view> v(ids.begin(), ids.end());
  std::sort(v.begin(), v.end());
  return std::adjacent_find(v.begin(), v.end()) != v.end();
}

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

const char* DeviceListStrategyName(DeviceListStrategy s) {
  switch (s) {
    case DeviceListStrategy::kEnvvar: return "envvar";
    case DeviceListStrategy::kVolumeMounts: return "volume-mounts";
    case DeviceListStrategy::kCdiAnnotations: return "cdi-annotations";
    case DeviceListStrategy::kCdiCri: return "cdi-cri";
  }
  return "?";
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

const char* DeviceIdStrategyName(DeviceIdStrategy s) {
  return s == DeviceIdStrategy::kIndex ? "index" : "uuid";
}

Plugin::Plugin(std::shared_ptr<const inventory::Snapshot> snap, strategy::PluginSpec spec,
               PluginOptions opts)
    : snap_(std::move(snap)), spec_(std::move(spec)), opts_(std::move(opts)) {
  if (opts_.kubelet_socket.empty()) opts_.kubelet_socket = PathJoin(opts_.plugin_dir, "kubelet.sock");
  BuildUnits();
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

Status Plugin::HandleGetOptions(std::string_view, std::string* resp) {
  // Preferred allocation is always offered: replicas use the prioritizer, whole
  // GPUs and partitions use the topology policy (server.go:243-248 offered it
  // only with a policy or replicas).
  pb::DevicePluginOptions o;
  o.pre_start_required = opts_.prestart_health_check;
  o.get_preferred_allocation_available = true;
  pb::Encode(o, resp);
  return Status::Ok();
}

Status Plugin::HandlePreStart(std::string_view req, std::string*) {
  pb::PreStartContainerRequest r;
  ADP_RETURN_IF_ERROR(pb::Decode(req, &r));
  if (!opts_.prestart_health_check) return Status::Ok();  // the reference's no-op (server.go:356-358)
  // --prestart-health-check: the kubelet asks right before it starts each
  // container; a device that went Unhealthy since admission stops the start
  // (the kubelet retries the container) instead of handing the workload a
  // resetting or failed GPU.
  auto law = CurrentLaw();
  for (const auto& id : r.device_ids) {
    auto it = advertised_index_.find(id);
    if (it == advertised_index_.end())
      return InvalidArgument("PreStartContainer for '" + spec_.resource_name + "': unknown device: " + id);
    if (law->healthy[it->second]) continue;
    stats_.prestart_refusals.Add(1);
    LOG_WARN(kComp, "PreStartContainer '%s': device %s is Unhealthy; container start refused",
             spec_.resource_name.c_str(), units_[it->second].id.c_str());
    return FailedPrecondition("device " + units_[it->second].id + " of '" + spec_.resource_name +
                              "' is Unhealthy; not starting the container on it");
  }
  return Status::Ok();
}

Status Plugin::HandleAllocate(std::string_view req, std::string* resp) {
  uint64_t t0 = NowNs();
  std::vector<std::vector<std::string_view>> containers;
  ADP_RETURN_IF_ERROR(pb::DecodeView(req, &containers));
  std::vector<int> us, units_per;
  // The index entry of each requested ID: one node per advertised ID, so equal
  // addresses are the same ID (distinct IDs counted without comparing strings).
  std::vector<const std::pair<const std::string_view, int>*> entries;
  std::vector<std::pair<int, uint32_t>> shares;  // (unit, replica) of CU-partitioned units
  std::string c, joined, cu_mask;
  MemoryGrant grant;
  for (const auto& ids : containers) {
    us.clear();
    shares.clear();
    entries.clear();
    for (std::string_view id : ids) {
      auto it = advertised_index_.find(id);
      if (it == advertised_index_.end())
        return InvalidArgument("invalid allocation request for '" + spec_.resource_name +
                               "': unknown device: " + std::string(id));
      us.push_back(it->second);
      if (hbm_grants_) entries.push_back(&*it);
      if (!units_[it->second].replica_cus.empty()) {
        // An advertised replica ID ends in "<join><r>" (alloc::ReplicaId).
        uint32_t r = 0, scale = 1;
        for (size_t k = id.size(); k > 0 && id[k - 1] >= '0' && id[k - 1] <= '9'; --k, scale *= 10)
          r += static_cast<uint32_t>(id[k - 1] - '0') * scale;
        shares.emplace_back(it->second, r);
      }
    }
    // Unique physical devices. uuid strategy: sorted by ID (stripReplicas order,
    // server.go:325); index strategy: enumeration order (server.go:406-411),
    // which here is unit order = KFD-node order = the container's HIP order.
    std::sort(us.begin(), us.end());
    if (hbm_grants_) {
      // Replicas (memory units / HBM shares) granted per device: distinct IDs
      // only (an ID listed twice is one unit, never twice the HBM).
      units_per.assign(units_.size(), 0);
      std::sort(entries.begin(), entries.end());
      entries.erase(std::unique(entries.begin(), entries.end()), entries.end());
      for (const auto* e : entries) ++units_per[e->second];
    }
    us.erase(std::unique(us.begin(), us.end()), us.end());
    if (unhealthy_units_.load(std::memory_order_relaxed) != 0) ADP_RETURN_IF_ERROR(CheckAllocatedHealth(us));
    grant.Clear();
    if (hbm_grants_) BuildMemoryGrant(us, units_per, &grant);
    cu_mask.clear();
    if (!shares.empty()) BuildCuMask(us, &shares, &cu_mask);
    if (opts_.id_strategy == DeviceIdStrategy::kUuid)
      std::sort(us.begin(), us.end(), [&](int a, int b) { return units_[a].id < units_[b].id; });

    c.clear();
    joined.clear();
    for (size_t i = 0; i < us.size(); ++i) {
      if (i) joined += ',';
      joined += units_[us[i]].visible_id;
    }
    AppendDeviceList(us, joined, &c);
    if (!grant.mib.empty()) {
      pb::PutMapEntry(&c, 1, kMemoryLimitEnv, grant.mib);
      pb::PutMapEntry(&c, 1, kMemoryFractionEnv, grant.frac);
      pb::PutMapEntry(&c, 1, kMemoryDevicesEnv, grant.devs);
      c += memcap_bytes_;  // the container enforces the grant (empty unless --enforce-memory-units)
      if (!memcap_bytes_.empty()) AppendGrantMounts(grant.bytes, &c);
      if (!memcap_bytes_.empty() && !opts_.memcap_usage_dir.empty()) AddUsageFile(ids, grant.bytes, &c);
    }
    if (!cu_mask.empty()) pb::PutMapEntry(&c, 1, kCuMaskEnv, cu_mask);
    if (opts_.pass_device_specs) {
      c += kfd_spec_bytes_;
      for (int u : us) c += units_[u].spec_bytes;
    }
    pb::PutLen(resp, 1, c);
    LOG_DEBUG(kComp, "allocate '%s': %zu IDs -> [%s]", spec_.resource_name.c_str(), ids.size(),
              joined.c_str());
  }
  uint64_t dt = NowNs() - t0;
  stats_.allocate_hist.Observe(dt);
  stats_.allocate_calls.Add(1);
  stats_.allocate_ns_total.Add(dt);
  stats_.allocate_ns_max.Observe(dt);
  return Status::Ok();
}

// A kubelet racing a health transition (or holding a stale device list) can
// name a device that is Unhealthy right now.
Status Plugin::CheckAllocatedHealth(const std::vector<int>& us) {
  auto law = CurrentLaw();
  for (int u : us) {
    if (law->healthy[u]) continue;
    stats_.unhealthy_allocations.Add(1);
    if (opts_.reject_unhealthy)
      return FailedPrecondition("allocation request for '" + spec_.resource_name + "': device " + units_[u].id +
                                " is Unhealthy");
    if (warned_law_[u].exchange(law->version, std::memory_order_relaxed) != law->version)
      LOG_WARN(kComp, "allocate '%s': device %s is Unhealthy (allocated anyway; --reject-unhealthy refuses)",
               spec_.resource_name.c_str(), units_[u].id.c_str());
  }
  return Status::Ok();
}

// Memory-unit resources (replicas = -1): tell the container how much HBM it
// was granted on each device so frameworks can cap themselves (e.g.
// torch.cuda.set_per_process_memory_fraction). Listed in enumeration order
// (us sorted by unit) -- the order HIP numbers the container's devices and
// HSA_CU_MASK uses -- whatever order the ID strategy gives AMD_VISIBLE_DEVICES.
// The reference hands out memory units without telling the workload.
void Plugin::BuildMemoryGrant(const std::vector<int>& us, const std::vector<int>& units_per,
                              MemoryGrant* g) const {
  char buf[32];
  for (size_t i = 0; i < us.size(); ++i) {
    const Unit& u = units_[us[i]];
    uint64_t granted = static_cast<uint64_t>(units_per[us[i]]) * u.grant_mib;
    if (i) { g->mib += ','; g->frac += ','; g->devs += ','; }
    g->devs += u.visible_id;
    g->mib += std::to_string(granted);
    g->bytes.push_back(granted << 20);
    // Under the HBM-cap shim the device reports the grant as its memory, so
    // the grant is all of what the workload sees.
    double frac = !memcap_bytes_.empty() ? 1.0 : u.vram_mib ? std::min(1.0, double(granted) / u.vram_mib) : 0.0;
    snprintf(buf, sizeof(buf), "%.4f", frac);
    g->frac += buf;
  }
}

// HSA_CU_MASK="<agent>:<first>-<last>,...;...": agents are numbered in the
// container in KFD-node order (= unit order, us is sorted by unit), and
// devices without an entry keep all their CUs. Adjacent replica shares merge.
void Plugin::BuildCuMask(const std::vector<int>& us, std::vector<std::pair<int, uint32_t>>* shares_in,
                         std::string* cu_mask) {
  auto& shares = *shares_in;
  // By unit, then by where the replica's range starts (memory-unit ranges
  // follow the IDs' lexicographic order, not the replica number).
  std::sort(shares.begin(), shares.end(), [&](const auto& a, const auto& b) {
    if (a.first != b.first) return a.first < b.first;
    const auto& ra = units_[a.first].replica_cus[a.second];
    const auto& rb = units_[b.first].replica_cus[b.second];
    return ra != rb ? ra < rb : a.second < b.second;
  });
  shares.erase(std::unique(shares.begin(), shares.end()), shares.end());
  size_t k = 0;
  for (size_t ord = 0; ord < us.size(); ++ord) {
    while (k < shares.size() && shares[k].first < us[ord]) ++k;
    if (k == shares.size() || shares[k].first != us[ord]) continue;
    const Unit& unit = units_[us[ord]];
    const auto& ranges = unit.replica_cus;
    size_t end = k;
    while (end < shares.size() && shares[end].first == us[ord]) ++end;
    // Shares are sorted by range and distinct; memory units share slots, so a
    // run of equal ranges is the units of one slot this container holds.
    auto run_end = [&](size_t g) {
      size_t h = g + 1;
      while (h < end && ranges[shares[h].second] == ranges[shares[g].second]) ++h;
      return h;
    };
    auto filled = [&](size_t g, size_t h) {
      return h - g == unit.slot_units[ranges[shares[g].second].first / unit.xcds];
    };
    // --memory-unit-cu-slots whole: keep only the slots whose units are all
    // this container's, so no neighbour runs on them. A container filling no
    // slot keeps its partial ones (it needs some CUs) and is counted.
    bool whole_only = false;
    if (!unit.slot_units.empty()) {
      for (size_t g = k; g < end && !whole_only;) {
        size_t h = run_end(g);
        whole_only = filled(g, h);
        g = h;
      }
      if (!whole_only) stats_.partial_cu_slot_allocations.Add(1);
    }
    if (!cu_mask->empty()) *cu_mask += ';';
    *cu_mask += std::to_string(ord);
    char sep = ':';
    bool open = false;
    uint32_t lo = 0, hi = 0;
    auto emit = [&] {
      *cu_mask += sep;
      *cu_mask += std::to_string(lo) + "-" + std::to_string(hi);
      sep = ',';
    };
    for (size_t g = k; g < end;) {
      size_t h = run_end(g);
      const auto& rg = ranges[shares[g].second];
      bool keep = !whole_only || filled(g, h);
      g = h;
      if (!keep) continue;
      if (open && rg.first <= hi + 1) {  // equal and adjacent ranges merge
        hi = std::max(hi, rg.second);
        continue;
      }
      if (open) emit();
      lo = rg.first;
      hi = rg.second;
      open = true;
    }
    if (open) emit();
    k = end;
  }
}

// The device list in the --device-list-strategy's form (server.go:338-346, apiEnvs/apiMounts at
// server.go:423-441; the CDI forms are this plugin's own).
void Plugin::AppendDeviceList(const std::vector<int>& us, const std::string& joined, std::string* c) const {
  switch (opts_.list_strategy) {
    case DeviceListStrategy::kEnvvar:
      pb::PutMapEntry(c, 1, opts_.envvar, joined);
      break;
    case DeviceListStrategy::kVolumeMounts:
      pb::PutMapEntry(c, 1, opts_.envvar, kVolumeMountRoot);
      for (int u : us) *c += units_[u].mount_bytes;
      break;
    case DeviceListStrategy::kCdiAnnotations: {
      if (us.empty()) break;
      std::string names;
      for (size_t i = 0; i < us.size(); ++i) {
        if (i) names += ',';
        names += std::string(kCdiVendorClass) + "=" + units_[us[i]].visible_id;
      }
      pb::PutMapEntry(c, 4, "cdi.k8s.io/amd-gpu-device-plugin_" + units_[us[0]].visible_id, names);
      break;
    }
    case DeviceListStrategy::kCdiCri:
      for (int u : us) {
        std::string n;
        pb::PutStr(&n, 1, std::string(kCdiVendorClass) + "=" + units_[u].visible_id);
        pb::PutLen(c, 5, n);
      }
      break;
  }
}

// The grant itself, read-only: the shim's caps (the env can only lower them).
// Encoded in place (a Mount: container path, host path, read-only).
void Plugin::AppendGrantMounts(const std::vector<uint64_t>& grant_bytes, std::string* c) const {
  static thread_local std::string gm, cpath, hpath;
  for (size_t i = 0; i < grant_bytes.size(); ++i) {
    char num[24];
    cpath.assign(adp_memcap::kGrantDir).push_back('/');
    cpath.append(num, static_cast<size_t>(std::to_chars(num, num + sizeof(num), i).ptr - num));
    hpath.assign(grant_dir_prefix_);
    hpath.append(num, static_cast<size_t>(std::to_chars(num, num + sizeof(num), grant_bytes[i] >> 20).ptr - num));
    hpath.append(".mib");
    gm.clear();
    pb::PutStr(&gm, 1, cpath);
    pb::PutStr(&gm, 2, hpath);
    pb::PutBool(&gm, 3, true);
    pb::PutLen(c, 2, gm);
  }
}

// The grant's accounting file (memcap/usage.h), mounted read-write where the
// shim looks for it; written by a background thread, long before the runtime
// mounts it. Without it the shim counts in the pod's /dev/shm: the cap holds
// either way, only /metrics does not see the container's use.
void Plugin::AddUsageFile(const std::vector<std::string_view>& ids, const std::vector<uint64_t>& grant_bytes,
                          std::string* c) {
  std::vector<std::string_view> sorted(ids);
  std::sort(sorted.begin(), sorted.end());
  std::string key = memcap::AllocationKeySorted(sorted);
  size_t len = sorted.size();
  for (std::string_view id : sorted) len += id.size();
  std::string joined;
  joined.reserve(len);
  for (size_t i = 0; i < sorted.size(); ++i) {
    if (i) joined += ',';
    joined += sorted[i];
  }
  std::string host;
  host.reserve(opts_.memcap_usage_dir.size() + 24);
  host.append(opts_.memcap_usage_dir).append("/").append(key).append(".memcap");
  memcap::CreateGrantFileAsync(opts_.memcap_usage_dir, std::move(key), grant_bytes, std::move(joined),
                               /*wake=*/false);  // WakeWriter() after the response is written
  pb::PutMapEntry(c, 1, kMemcapFileEnv, kMemcapUsageContainerPath);
  pb::Mount m{kMemcapUsageContainerPath, std::move(host), false};
  std::string mb;
  pb::Encode(m, &mb);
  pb::PutLen(c, 2, mb);
}

Status Plugin::HandlePreferred(std::string_view req, std::string* resp) {
  uint64_t t0 = NowNs();
  Status st = PreferredImpl(req, resp);
  uint64_t dt = NowNs() - t0;
  stats_.preferred_hist.Observe(dt);
  stats_.preferred_ns_total.Add(dt);
  stats_.preferred_ns_max.Observe(dt);
  return st;
}

Status Plugin::PreferredImpl(std::string_view req, std::string* resp) {
  // Per loop thread, kept across calls: a memory-unit request names every free
  // unit of the node (2,352 IDs on 8 MI355X), decoded into reused capacity.
  static thread_local std::vector<pb::ContainerPreferredAllocationRequestView> reqs;
  ADP_RETURN_IF_ERROR(pb::DecodeView(req, &reqs));
  pb::PreferredAllocationResponse out;
  stats_.preferred_calls.Add(1);
  for (const auto& cr : reqs) {
    if (replicated_) {
      // Multi-device pack requests grow towards the devices already chosen
      // (same NUMA node / xGMI score), the memory-unit analogue of the
      // best-effort policy below.
      alloc::DeviceAffinity affinity = [this](std::string_view a, std::string_view b) -> long {
        auto ia = unit_index_by_id_.find(a), ib = unit_index_by_id_.find(b);
        if (ia == unit_index_by_id_.end() || ib == unit_index_by_id_.end()) return 0;
        return graph_.Score(ia->second, ib->second);
      };
      auto res = alloc::PrioritizeDeviceViews(cr.available, cr.must_include, cr.allocation_size,
                                              replica_policy_, alloc::kReplicaJoin, &affinity);
      if (!res.ok()) return res.status();
      if (HasDuplicate(res->ids)) {
        // An ID listed twice in availableDeviceIDs was chosen twice: choose
        // again from the de-duplicated list (off the common path).
        std::vector<std::string_view> avail(cr.available.begin(), cr.available.end());
        std::sort(avail.begin(), avail.end());
        avail.erase(std::unique(avail.begin(), avail.end()), avail.end());
        res = alloc::PrioritizeDeviceViews(avail, cr.must_include, cr.allocation_size, replica_policy_,
                                           alloc::kReplicaJoin, &affinity);
        if (!res.ok()) return res.status();
      }
      // Physical devices must be ours (reference: NewDevicesFrom fails on an
      // unknown UUID, server.go:274-278) -- one lookup per device, not per
      // replica -- and so must every ID handed back (of the final choice: an
      // ID the kubelet made up, e.g. "<uuid>-replica-1x", names a device of
      // ours but was never advertised).
      for (const auto& dev : res->devices)
        if (!unit_index_by_id_.count(dev))
          return InvalidArgument("unable to retrieve list of available devices: unknown device " + dev);
      for (const auto& id : res->ids)
        if (!advertised_index_.count(id))
          return InvalidArgument("unable to retrieve list of available devices: unknown device " + id);
      if (res->non_unique) LOG_DEBUG(kComp, "ignoring: %s", alloc::kNonUniqueMessage);
      out.container_responses.push_back(std::move(res->ids));
      continue;
    }
    std::vector<int> avail, must;
    for (std::string_view id : cr.available) {
      auto it = advertised_index_.find(id);
      if (it == advertised_index_.end())
        return InvalidArgument("unable to retrieve list of available devices: unknown device " +
                               std::string(id));
      avail.push_back(it->second);
    }
    for (std::string_view id : cr.must_include) {
      auto it = advertised_index_.find(id);
      if (it == advertised_index_.end())
        return InvalidArgument("unable to retrieve list of required devices: unknown device " +
                               std::string(id));
      must.push_back(it->second);
    }
    std::vector<std::string> ids;
    for (int u : CachedBestEffort(avail, must, cr.allocation_size))
      ids.push_back(units_[u].id);  // advertised ID (no replica suffix here), fixes B6
    out.container_responses.push_back(std::move(ids));
  }
  pb::Encode(out, resp);
  return Status::Ok();
}

void Plugin::Unmap::operator()(std::atomic<uint16_t>* p) const { munmap(p, kBestEffortCacheBytes); }

std::vector<int> Plugin::CachedBestEffort(const std::vector<int>& avail, const std::vector<int>& must,
                                          int size) {
  // Up to 8 devices the answer is a pure function of (available set, required
  // set, size) over an immutable graph: 256 x 256 x 9 entries of 16 bits,
  // filled lazily (0 = not computed, else 1 + result mask, kEmpty = no answer).
  constexpr int kMax = 8;
  constexpr uint16_t kEmpty = 0x200;
  const int n = static_cast<int>(units_.size());
  if (n > kMax || size < 0 || size > kMax || !best_effort_cache_)
    return alloc::BestEffortAllocate(graph_, avail, must, size);
  uint32_t am = 0, rm = 0;
  for (int u : avail) am |= 1u << u;
  for (int u : must) rm |= 1u << u;
  if ((rm & ~am) != 0) return {};
  std::atomic<uint16_t>& slot =
      best_effort_cache_.get()[(am * 256u + rm) * (kMax + 1) + static_cast<uint32_t>(size)];
  uint16_t v = slot.load(std::memory_order_relaxed);
  if (v == 0) {
    std::vector<int> r = alloc::BestEffortAllocate(graph_, avail, must, size);
    uint32_t mask = 0;
    for (int u : r) mask |= 1u << u;
    v = r.empty() ? kEmpty : static_cast<uint16_t>(1 + mask);
    slot.store(v, std::memory_order_relaxed);  // racing writers store the same value
  }
  std::vector<int> out;
  if (v == kEmpty) return out;
  for (uint32_t m = v - 1u; m; m &= m - 1) out.push_back(__builtin_ctz(m));
  return out;
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

void Plugin::SetHandleHealth(int handle, bool healthy, const std::string& reason) {
  std::vector<int> us;
  for (size_t i = 0; i < units_.size(); ++i)
    for (int h : units_[i].handles)
      if (h == handle) us.push_back(static_cast<int>(i));
  PostHealth(std::move(us), healthy, reason);
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
