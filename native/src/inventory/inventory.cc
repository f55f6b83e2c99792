#include "inventory/inventory.h"

#include <errno.h>
#include <fcntl.h>
#include <unistd.h>

#include <cctype>
#include <cstring>

#include <algorithm>
#include <map>
#include <set>
#include <sys/stat.h>

#include "common/log.h"
#include "common/strings.h"

namespace adp::inventory {
namespace {

constexpr const char* kComp = "inventory";

std::string Upper(std::string s) {
  for (auto& c : s) c = static_cast<char>(toupper(static_cast<unsigned char>(c)));
  return s;
}

std::string ModeForCount(size_t n) {
  switch (n) {
    case 1: return "SPX";
    case 2: return "DPX";
    case 3: return "TPX";
    case 4: return "QPX";
    default: return "CPX";
  }
}

// MI355X: 32 CUs per XCD. Used only when amdsmi cannot report XCD counts.
constexpr uint32_t kCusPerXcd = 32;

std::string ModeForProfile(const std::string& compute, const std::string& profile, size_t handles) {
  if (!compute.empty()) return compute;
  if (!profile.empty()) return profile;
  return ModeForCount(handles);
}

bool Near(uint64_t a, uint64_t b) {  // within 3 %
  uint64_t hi = std::max(a, b), lo = std::min(a, b);
  return hi - lo <= hi * 3 / 100;
}

int NpsCount(const std::string& memory_mode) {
  if (memory_mode.size() > 3 && memory_mode.compare(0, 3, "NPS") == 0) {
    int k = atoi(memory_mode.c_str() + 3);
    return k > 0 ? k : 1;
  }
  return 1;
}

}  // namespace

uint64_t ModelHbmMib(const std::string& market_name) {
  std::string m = Upper(market_name);
  if (m.find("MI355") != std::string::npos || m.find("MI350") != std::string::npos) return 294896;
  if (m.find("MI325") != std::string::npos) return 262144;
  if (m.find("MI300X") != std::string::npos || m.find("MI308") != std::string::npos) return 196608;
  return 0;
}

std::string RenderPath(uint32_t minor) { return "/dev/dri/renderD" + std::to_string(minor); }
std::string CardPath(uint32_t minor) { return "/dev/dri/card" + std::to_string(minor); }
uint64_t GbCeil(uint64_t mib) { return (mib + 1023) / 1024; }

std::string PhysicalGpu::PartitionProfile() const {
  if (compute_mode == "SPX" || partitions.empty()) return "";
  const Partition& p = partitions.front();
  uint32_t x = p.xcds;
  if (!x && xcds && !partitions.empty()) x = xcds / static_cast<uint32_t>(partitions.size());
  if (!x && p.cus) x = std::max<uint32_t>(1, p.cus / kCusPerXcd);
  if (!x) x = 1;
  return ToLower(compute_mode) + "-" + std::to_string(x) + "xcd." + std::to_string(GbCeil(p.vram_mib)) +
         "gb";
}

int Snapshot::GpuOfHandle(int h) const {
  for (const auto& g : gpus)
    for (const auto& p : g.partitions)
      if (p.handle == h) return g.index;
  return -1;
}

uint32_t KfdTopologyCus(const std::string& topology_dir, uint32_t node) {
  std::string path = topology_dir + "/" + std::to_string(node) + "/properties";
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return 0;
  std::string text;
  char buf[4096];
  ssize_t n;
  while ((n = read(fd, buf, sizeof(buf))) > 0 && text.size() < 65536) text.append(buf, static_cast<size_t>(n));
  close(fd);
  uint64_t simds = 0, per_cu = 0;
  for (size_t b = 0; b < text.size();) {
    size_t e = text.find('\n', b);
    if (e == std::string::npos) e = text.size();
    std::string line = text.substr(b, e - b);
    b = e + 1;
    size_t sp = line.find(' ');
    if (sp == std::string::npos) continue;
    std::string key = line.substr(0, sp);
    auto v = ParseUint(Trim(line.substr(sp + 1)));
    if (!v) continue;
    if (key == "simd_count") simds = *v;
    else if (key == "simd_per_cu") per_cu = *v;
  }
  if (simds == 0 || per_cu == 0 || simds % per_cu != 0 || simds / per_cu > 0xffffu) return 0;
  return static_cast<uint32_t>(simds / per_cu);
}

std::string PciProductName(const std::string& sysfs_root, const std::string& bdf) {
  // Compute partitions report their own function numbers; the board is function 0.
  size_t dot = bdf.rfind('.');
  if (dot == std::string::npos || bdf.find('/') != std::string::npos) return "";
  std::string path = sysfs_root + "/bus/pci/devices/" + bdf.substr(0, dot) + ".0/product_name";
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return "";
  char buf[256];
  ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0) return "";
  std::string v = Trim(std::string_view(buf, static_cast<size_t>(n)));
  for (char c : v)
    if (static_cast<unsigned char>(c) < 0x20) return "";  // not a name
  return v;
}

Result<std::shared_ptr<Snapshot>> GroupProcessors(std::vector<smi::ProcessorInfo> procs,
                                                  const BuildOptions& opt) {
  auto snap = std::make_shared<Snapshot>();
  snap->procs = std::move(procs);
  // Without the render node asic_info fails and the CU count (what CU shares
  // are cut from) is unknown; KFD's topology has it, readable unprivileged.
  // The board's FRU product name (PCI sysfs) names the model where asic_info
  // says "AMD Radeon Graphics" -- and answers without the render node too.
  if (!opt.sysfs_root.empty()) {
    const std::string topo = opt.sysfs_root + "/class/kfd/kfd/topology/nodes";
    size_t filled = 0, missing = 0, named = 0;
    for (auto& p : snap->procs) {
      std::string product = PciProductName(opt.sysfs_root, p.bdf);
      if (!product.empty() && product != p.market_name) {
        p.market_name = product;
        ++named;
      }
      if (p.num_cu != 0) continue;
      uint32_t cus = p.kfd_node == kNoKfdNode ? 0 : KfdTopologyCus(topo, p.kfd_node);
      if (cus) {
        p.num_cu = cus;
        ++filled;
      } else {
        ++missing;
      }
    }
    snap->cus_from_topology = filled;
    snap->cus_unknown = missing;
    if (filled)
      LOG_INFO(kComp, "CU counts of %zu processor(s) from KFD topology (%s): amdsmi's asic_info did not answer",
               filled, topo.c_str());
    if (named)
      LOG_INFO(kComp, "product names of %zu processor(s) from PCI sysfs (the board's FRU name)", named);
    if (missing)
      LOG_WARN(kComp, "CU count of %zu processor(s) unknown (asic_info and KFD topology): no CU shares on them",
               missing);
  }
  // Group handles into physical GPUs. Compute partitions of one GPU report the
  // same ASIC serial; without one, group by PCI domain:bus:device (partitions
  // differ only in the function number); last resort, the UUID.
  std::vector<std::string> order;
  std::map<std::string, std::vector<int>> groups;
  for (size_t i = 0; i < snap->procs.size(); ++i) {
    const auto& p = snap->procs[i];
    std::string key = !p.asic_serial.empty() ? "serial:" + p.asic_serial
                      : p.bdf_id             ? "bdf:" + std::to_string(p.bdf_id & ~uint64_t{7})
                                             : "uuid:" + p.uuid;
    if (!groups.count(key)) order.push_back(key);
    groups[key].push_back(static_cast<int>(i));
  }

  // Per-partition HBM, pinned to the driver: a partition handle's vram_info may
  // report its own share, its memory partition's pool, or the whole GPU
  // depending on the amdsmi/driver version. The GPU's physical HBM is taken
  // from the most authoritative source available and every partition gets
  // its share, physical / partitions, so resources named "...36gb" and memory
  // units always add up to the HBM that exists.
  auto PinPartitionVram = [](PhysicalGpu* g, const std::vector<int>& handles, const Snapshot& s) -> bool {
    const auto& first = s.procs[handles.front()];
    size_t n = handles.size();
    int k = NpsCount(g->memory_mode);
    uint64_t model = ModelHbmMib(first.market_name);
    uint64_t sum = 0, lo = UINT64_MAX, hi = 0, ranges_mib = 0;
    uint32_t ranges = 0;
    for (int h : handles) {
      uint64_t v = s.procs[h].vram_mib;
      sum += v;
      lo = std::min(lo, v);
      hi = std::max(hi, v);
      if (s.procs[h].mem_ranges_mib > ranges_mib) {
        ranges_mib = s.procs[h].mem_ranges_mib;
        ranges = s.procs[h].mem_ranges;
      }
    }
    uint64_t phys = 0;
    if (ranges_mib && (static_cast<int>(ranges) == k || g->memory_mode.empty())) {
      if (!model || Near(ranges_mib, model)) {
        phys = ranges_mib;
        g->vram_source = "memory-partition-config";
      } else {
        LOG_WARN(kComp, "GPU %s (%s): memory-partition ranges add up to %llu MiB, not the model's %llu; ignored",
                 g->bdf.c_str(), first.market_name.c_str(), static_cast<unsigned long long>(ranges_mib),
                 static_cast<unsigned long long>(model));
      }
    }
    if (phys) {
      // pinned by the driver's memory ranges
    } else if (n == 1) {
      phys = hi;  // SPX: the handle is the whole GPU, whatever the model table says
      g->vram_source = "spx";
    } else if (lo == hi) {
      struct Cand { uint64_t mib; const char* what; };
      std::vector<Cand> cands = {{hi * n, "share"}};
      if (k > 1 && static_cast<size_t>(k) < n) cands.push_back({hi * static_cast<uint64_t>(k), "pool"});
      cands.push_back({hi, "whole"});
      if (model) {
        for (const auto& c : cands)
          if (Near(c.mib, model)) {
            phys = c.mib;
            g->vram_source = c.what;
            break;
          }
      } else {
        phys = hi * n;
        g->vram_source = "share-unpinned";
        LOG_WARN(kComp, "GPU %s (%s): partitions each report %llu MiB and the model's HBM is unknown; "
                 "assuming that is each partition's share", g->bdf.c_str(), first.market_name.c_str(),
                 static_cast<unsigned long long>(hi));
      }
    } else if (!model || Near(sum, model)) {
      phys = sum;  // uneven shares that add up
      g->vram_source = model ? "share" : "share-unpinned";
    }
    if (!phys) {
      std::string got;
      for (int h : handles) got += (got.empty() ? "" : ",") + std::to_string(s.procs[h].vram_mib);
      LOG_ERROR(kComp, "GPU %s (%s, %s/%s): partition VRAM [%s] MiB is inconsistent with the model's %llu MiB "
                "of HBM under every reading (share / memory-partition pool / whole GPU); the GPU is not served",
                g->bdf.c_str(), first.market_name.c_str(), g->compute_mode.c_str(), g->memory_mode.c_str(),
                got.c_str(), static_cast<unsigned long long>(model));
      return false;
    }
    g->vram_mib = phys;
    bool keep_reported = g->vram_source == "share" && lo != hi;  // uneven split, reported as such
    for (auto& part : g->partitions)
      if (!keep_reported) part.vram_mib = phys / n;
    return true;
  };

  std::set<int> only(opt.only_gpus.begin(), opt.only_gpus.end());
  int index = 0;
  for (size_t gi = 0; gi < order.size(); ++gi) {
    auto& handles = groups[order[gi]];
    std::sort(handles.begin(), handles.end(), [&](int a, int b) {
      return snap->procs[a].partition_id < snap->procs[b].partition_id;
    });
    const auto& first = snap->procs[handles.front()];
    if (!only.empty() || !opt.only_ids.empty()) {
      bool keep = only.count(static_cast<int>(gi)) > 0;
      std::string bdf = smi::FormatBdf(first.bdf_id & ~uint64_t{7});
      std::string bus = bdf.substr(0, bdf.rfind('.'));  // "dddd:bb:dd"
      for (const auto& id : opt.only_ids) {
        std::string want = ToLower(id);
        if (want == ToLower(first.uuid)) keep = true;
        if (want.find(':') == std::string::npos) continue;
        if (size_t dot = want.rfind('.'); dot != std::string::npos) want.resize(dot);  // function ignored
        if (std::count(want.begin(), want.end(), ':') == 1) want = "0000:" + want;    // domain optional
        if (want == bus) keep = true;
      }
      if (!keep) continue;
    }
    PhysicalGpu g;
    g.index = index;
    g.node_index = static_cast<int>(gi);
    g.uuid = first.uuid;
    g.bdf = smi::FormatBdf(first.bdf_id & ~uint64_t{7});
    g.numa = first.numa_node;
    g.market_name = first.market_name;
    g.reported_compute = Upper(first.compute_partition);
    g.reported_memory = Upper(first.memory_partition);
    g.driver_profile = first.profile_type;
    g.compute_mode = ModeForProfile(g.reported_compute, g.driver_profile, handles.size());
    g.memory_mode = g.reported_memory;
    if (!g.driver_profile.empty() && !g.reported_compute.empty() && g.driver_profile != g.reported_compute)
      LOG_WARN(kComp, "GPU %s: compute partition %s but accelerator partition profile %s", g.bdf.c_str(),
               g.reported_compute.c_str(), g.driver_profile.c_str());
    if (first.profile_partitions && first.profile_partitions != handles.size())
      LOG_WARN(kComp, "GPU %s: the partition profile has %u partitions, amdsmi lists %zu handles", g.bdf.c_str(),
               first.profile_partitions, handles.size());

    // Partition IDs must be unique and stable across restarts: the handle UUID
    // when amdsmi reports distinct ones, else "<uuid>-p<partition>".
    std::set<std::string> seen;
    bool unique = true;
    for (int h : handles)
      if (!seen.insert(snap->procs[h].uuid).second) unique = false;
    for (int h : handles) {
      const auto& p = snap->procs[h];
      Partition part;
      part.handle = h;
      part.partition_id = p.partition_id;
      part.uuid = (unique || handles.size() == 1) ? p.uuid
                                                   : p.uuid + "-p" + std::to_string(p.partition_id);
      part.bdf = p.bdf;
      part.render_path = p.render_minor ? RenderPath(p.render_minor) : "";
      if (opt.include_card_nodes && p.card_minor != 0xffffffffu) part.card_path = CardPath(p.card_minor);
      part.numa = p.numa_node;
      part.vram_mib = p.vram_mib;
      part.xcds = p.profile_xccs ? p.profile_xccs : p.xcd_count;
      part.cus = p.num_cu;
      part.kfd_node = p.kfd_node;
      g.kfd_node = std::min(g.kfd_node, p.kfd_node);
      g.xcds += part.xcds;
      g.cus += p.num_cu;
      g.partitions.push_back(std::move(part));
    }
    if (!PinPartitionVram(&g, handles, *snap)) continue;  // inconsistent: not served (logged)
    if (g.compute_mode == "SPX" && handles.size() > 1) {
      LOG_WARN(kComp, "GPU %s reports SPX but has %zu handles; treating as %s", g.bdf.c_str(),
               handles.size(), ModeForCount(handles.size()).c_str());
      g.compute_mode = ModeForCount(handles.size());
    }
    snap->gpus.push_back(std::move(g));
    ++index;
  }
  size_t n = snap->gpus.size();
  snap->gpu_links.assign(n * n, LinkClass::kUnknown);
  snap->gpu_hops.assign(n * n, 0);
  snap->gpu_weights.assign(n * n, 0);
  snap->gpu_link_types.assign(n * n, -1);
  for (size_t a = 0; a < n; ++a) snap->gpu_links[a * n + a] = LinkClass::kSame;
  return snap;
}

Result<std::shared_ptr<const Snapshot>> BuildSnapshot(smi::Library* lib, const BuildOptions& opt) {
  auto procs = lib->Enumerate();
  if (!procs.ok()) return procs.status();
  auto grouped = GroupProcessors(std::move(*procs), opt);
  if (!grouped.ok()) return grouped.status();
  std::shared_ptr<Snapshot> snap = std::move(*grouped);
  snap->smi_path = lib->path();
  snap->smi_version = lib->Version();
  size_t n = snap->gpus.size();
  for (size_t a = 0; a < n; ++a) {
    auto& ga = snap->gpus[a];
    void* ha = snap->procs[ga.partitions.front().handle].handle;
    ga.xgmi_links_down = lib->XgmiLinksDown(ha);
    for (size_t b = 0; b < n; ++b) {
      if (a == b) continue;
      void* hb = snap->procs[snap->gpus[b].partitions.front().handle].handle;
      smi::Link l = lib->GetLink(ha, hb);
      LinkClass c = LinkClass::kUnknown;
      if (l.valid) {
        if (l.type == smi::LinkType::kXgmi) c = LinkClass::kXgmi;
        else if (l.type == smi::LinkType::kInternal) c = LinkClass::kSame;
        else if (l.type == smi::LinkType::kPcie)
          c = (ga.numa >= 0 && ga.numa == snap->gpus[b].numa) ? LinkClass::kPcieSameNuma
                                                               : LinkClass::kPcieCrossNuma;
      }
      snap->gpu_links[a * n + b] = c;
      snap->gpu_hops[a * n + b] = l.hops;
      snap->gpu_weights[a * n + b] = l.weight;
      snap->gpu_link_types[a * n + b] = l.valid ? static_cast<int>(l.type) : -1;
    }
  }
  struct stat st;
  std::string kfd = PathJoin(opt.driver_root, "/dev/kfd");
  if (stat(kfd.c_str(), &st) != 0)
    LOG_WARN(kComp, "%s is not visible to the plugin; it is still passed to containers", kfd.c_str());
  for (const auto& g : snap->gpus) {
    LOG_INFO(kComp,
             "GPU %d: %s bdf=%s numa=%d kfd_node=%s vram=%llu MiB (%s) mode=%s/%s partitions=%zu profile=%s "
             "render=%s",
             g.index, g.uuid.c_str(), g.bdf.c_str(), g.numa,
             g.kfd_node == kNoKfdNode ? "?" : std::to_string(g.kfd_node).c_str(),
             static_cast<unsigned long long>(g.vram_mib), g.vram_source.c_str(), g.compute_mode.c_str(),
             g.memory_mode.empty() ? "?" : g.memory_mode.c_str(), g.partitions.size(),
             g.PartitionProfile().empty() ? "-" : g.PartitionProfile().c_str(),
             g.partitions.front().render_path.c_str());
  }
  return std::shared_ptr<const Snapshot>(snap);
}

namespace {

std::string LabelSafe(std::string v) {
  for (auto& c : v)
    if (!isalnum(static_cast<unsigned char>(c)) && c != '.' && c != '_' && c != '-') c = '-';
  while (!v.empty() && !isalnum(static_cast<unsigned char>(v.front()))) v.erase(v.begin());
  while (!v.empty() && !isalnum(static_cast<unsigned char>(v.back()))) v.pop_back();
  if (v.size() > 63) v.resize(63);
  return v;
}

}  // namespace

std::vector<std::pair<std::string, std::string>> NodeLabels(const Snapshot& snap) {
  std::vector<std::pair<std::string, std::string>> out;
  const size_t n = snap.gpus.size();
  out.emplace_back("amd.com/gpu.present", n ? "true" : "false");
  out.emplace_back("amd.com/gpu.count", std::to_string(n));
  if (n == 0) return out;
  auto uniform = [&](auto get) {
    std::string v = get(snap.gpus[0]);
    for (const auto& g : snap.gpus)
      if (get(g) != v) return std::string("mixed");
    return v;
  };
  out.emplace_back("amd.com/gpu.product", LabelSafe(uniform([](const PhysicalGpu& g) { return g.market_name; })));
  uint64_t vram = snap.gpus[0].vram_mib;
  size_t parts = 0;
  for (const auto& g : snap.gpus) {
    vram = std::min(vram, g.vram_mib);
    parts += g.partitions.size();
  }
  out.emplace_back("amd.com/gpu.memory-mib", std::to_string(vram));
  out.emplace_back("amd.com/gpu.compute-partition", LabelSafe(uniform([](const PhysicalGpu& g) { return g.compute_mode; })));
  out.emplace_back("amd.com/gpu.memory-partition",
                   LabelSafe(uniform([](const PhysicalGpu& g) { return g.memory_mode.empty() ? std::string("unknown") : g.memory_mode; })));
  out.emplace_back("amd.com/gpu.partitions", std::to_string(parts));
  std::string profile = uniform([](const PhysicalGpu& g) { return g.PartitionProfile(); });
  if (!profile.empty()) out.emplace_back("amd.com/gpu.partition-profile", LabelSafe(profile));
  // Interconnect: every distinct pair over xGMI -> "xgmi-full-mesh".
  bool all_xgmi = n > 1, any_xgmi = false;
  for (size_t a = 0; a < n; ++a)
    for (size_t b = 0; b < n; ++b) {
      if (a == b) continue;
      bool x = snap.Link(static_cast<int>(a), static_cast<int>(b)) == LinkClass::kXgmi;
      all_xgmi = all_xgmi && x;
      any_xgmi = any_xgmi || x;
    }
  out.emplace_back("amd.com/gpu.interconnect", n == 1 ? "single" : all_xgmi ? "xgmi-full-mesh" : any_xgmi ? "xgmi-partial" : "pcie");
  int down = 0;
  for (const auto& g : snap.gpus) down += g.xgmi_links_down;
  out.emplace_back("amd.com/gpu.xgmi-links-down", std::to_string(down));
  return out;
}

int KfdAccessErrno(const std::string& driver_root) {
  std::string kfd = PathJoin(driver_root, "/dev/kfd");
  int fd = open(kfd.c_str(), O_RDWR | O_CLOEXEC | O_NONBLOCK);
  if (fd < 0) return errno;
  close(fd);
  return 0;
}

std::vector<NodeAccess> ProbeDeviceAccess(const Snapshot& snap, const std::string& driver_root) {
  std::vector<NodeAccess> out;
  out.push_back({PathJoin(driver_root, "/dev/kfd"), KfdAccessErrno(driver_root)});
  for (const auto& g : snap.gpus)
    for (const auto& p : g.partitions) {
      if (p.render_path.empty()) continue;
      std::string path = PathJoin(driver_root, p.render_path);
      int fd = open(path.c_str(), O_RDWR | O_CLOEXEC | O_NONBLOCK);
      out.push_back({path, fd < 0 ? errno : 0});
      if (fd >= 0) close(fd);
    }
  return out;
}

std::string DescribeAccess(const std::vector<NodeAccess>& access) {
  std::string denied;
  int err = 0;
  for (const auto& a : access)
    if (a.err) {
      denied += (denied.empty() ? "" : ", ") + a.path;
      err = a.err;
    }
  if (denied.empty()) return "ok";
  std::string why = std::string(strerror(err)) + ": " + denied;
  if (err == EPERM)
    why += " (the container's device cgroup does not allow them -- an unprivileged pod that only "
           "hostPath-mounts /dev; the plugin does not need them, amdsmi health events do: helm healthEvents: "
           "true registers those in its privileged event-relay container)";
  else if (err == ENOENT)
    why += " (not present: is /dev mounted from the host, and the driver root right?)";
  else if (err == EACCES)
    why += " (file permissions: run the plugin as root or in the render group)";
  return why;
}

}  // namespace adp::inventory
