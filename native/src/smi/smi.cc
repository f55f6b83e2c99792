#include "smi/smi.h"

#include <amd_smi/amdsmi.h>
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>

#include "common/log.h"

namespace adp::smi {

namespace {
constexpr const char* kComp = "smi";
}

// Function table resolved with dlsym. Required entries fail Open(); optional ones
// degrade a feature (e.g. no topology -> flat link matrix).
struct Library::Fns {
  decltype(&amdsmi_init) init = nullptr;
  decltype(&amdsmi_shut_down) shut_down = nullptr;
  decltype(&amdsmi_get_socket_handles) socket_handles = nullptr;
  decltype(&amdsmi_get_processor_handles) processor_handles = nullptr;
  decltype(&amdsmi_get_processor_type) processor_type = nullptr;
  decltype(&amdsmi_get_gpu_device_uuid) uuid = nullptr;
  decltype(&amdsmi_get_gpu_device_bdf) bdf = nullptr;
  decltype(&amdsmi_get_gpu_enumeration_info) enum_info = nullptr;
  decltype(&amdsmi_get_gpu_topo_numa_affinity) numa = nullptr;
  decltype(&amdsmi_get_gpu_vram_info) vram_info = nullptr;
  decltype(&amdsmi_get_gpu_memory_total) memory_total = nullptr;
  decltype(&amdsmi_get_gpu_memory_usage) memory_usage = nullptr;
  decltype(&amdsmi_get_gpu_activity) activity = nullptr;
  decltype(&amdsmi_get_gpu_compute_partition) compute_partition = nullptr;
  decltype(&amdsmi_get_gpu_memory_partition) memory_partition = nullptr;
  decltype(&amdsmi_get_gpu_kfd_info) kfd_info = nullptr;
  decltype(&amdsmi_get_gpu_asic_info) asic_info = nullptr;
  decltype(&amdsmi_get_gpu_xcd_counter) xcd_counter = nullptr;
  decltype(&amdsmi_get_gpu_accelerator_partition_profile) accel_profile = nullptr;
  decltype(&amdsmi_get_gpu_accelerator_partition_profile_config) accel_profile_config = nullptr;
  decltype(&amdsmi_get_gpu_memory_partition_config) memory_partition_config = nullptr;
  decltype(&amdsmi_topo_get_link_type) link_type = nullptr;
  decltype(&amdsmi_topo_get_link_weight) link_weight = nullptr;
  decltype(&amdsmi_get_gpu_xgmi_link_status) xgmi_link_status = nullptr;
  decltype(&amdsmi_init_gpu_event_notification) evt_init = nullptr;
  decltype(&amdsmi_set_gpu_event_notification_mask) evt_mask = nullptr;
  decltype(&amdsmi_get_gpu_event_notification) evt_get = nullptr;
  decltype(&amdsmi_stop_gpu_event_notification) evt_stop = nullptr;
  decltype(&amdsmi_get_gpu_total_ecc_count) ecc_total = nullptr;
  decltype(&amdsmi_get_gpu_bad_page_info) bad_pages = nullptr;
  decltype(&amdsmi_get_gpu_bad_page_threshold) bad_page_threshold = nullptr;
  decltype(&amdsmi_get_gpu_process_list) process_list = nullptr;
  decltype(&amdsmi_status_code_to_string) status_string = nullptr;
  decltype(&amdsmi_get_lib_version) lib_version = nullptr;
};

namespace {

template <typename T>
void Resolve(void* dl, const char* name, T* out) {
  *out = reinterpret_cast<T>(dlsym(dl, name));
}

}  // namespace

std::string FormatBdf(uint64_t bdf_id) {
  amdsmi_bdf_t b;
  b.as_uint = bdf_id;
  char buf[32];
  snprintf(buf, sizeof(buf), "%04llx:%02x:%02x.%x",
           static_cast<unsigned long long>(b.domain_number), static_cast<unsigned>(b.bus_number),
           static_cast<unsigned>(b.device_number), static_cast<unsigned>(b.function_number));
  return buf;
}

uint64_t EventMask(uint32_t event_type) { return AMDSMI_EVENT_MASK_FROM_INDEX(event_type); }

std::string EventTypeName(uint32_t type) {
  static const char* const kNames[] = {
      "NONE",           "VMFAULT",       "THERMAL_THROTTLE", "GPU_PRE_RESET", "GPU_POST_RESET",
      "MIGRATE_START",  "MIGRATE_END",   "PAGE_FAULT_START", "PAGE_FAULT_END", "QUEUE_EVICTION",
      "QUEUE_RESTORE",  "UNMAP_FROM_GPU", "PROCESS_START",   "PROCESS_END"};
  static_assert(sizeof(kNames) / sizeof(kNames[0]) == AMDSMI_EVT_NOTIF_LAST + 1, "amdsmi event types changed");
  if (type >= 1 && type <= AMDSMI_EVT_NOTIF_LAST) return kNames[type];
  return "EVENT_" + std::to_string(type);
}

Library::Library() = default;

Library::~Library() {
  if (f_) EventsStopAll();
  if (initialized_ && f_ && f_->shut_down) f_->shut_down();
  // Not dlclose'd: a library's thread-local destructors and atexit handlers
  // may still point into it (the process either exits next or, in the GPU
  // tests, goes on to load the HIP runtime, which crashed on an unmapped mock).
}

Result<std::unique_ptr<Library>> Library::Open(const std::string& path,
                                               const std::string& rocm_root) {
  std::vector<std::string> candidates;
  if (!path.empty()) {
    candidates.push_back(path);
  } else {
    if (const char* e = std::getenv("AMD_SMI_LIB"); e && *e) candidates.push_back(e);
    candidates.push_back("libamd_smi.so");
    candidates.push_back("libamd_smi.so.26");
    candidates.push_back(rocm_root + "/lib/libamd_smi.so");
  }
  std::unique_ptr<Library> lib(new Library());
  std::string errors;
  for (const auto& c : candidates) {
    lib->dl_ = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (lib->dl_) { lib->path_ = c; break; }
    const char* e = dlerror();
    errors += (errors.empty() ? "" : "; ") + std::string(e ? e : c);
    if (!path.empty()) break;
  }
  if (!lib->dl_) return Unavailable("cannot load libamd_smi: " + errors);

  auto f = std::make_unique<Fns>();
  void* dl = lib->dl_;
  Resolve(dl, "amdsmi_init", &f->init);
  Resolve(dl, "amdsmi_shut_down", &f->shut_down);
  Resolve(dl, "amdsmi_get_socket_handles", &f->socket_handles);
  Resolve(dl, "amdsmi_get_processor_handles", &f->processor_handles);
  Resolve(dl, "amdsmi_get_processor_type", &f->processor_type);
  Resolve(dl, "amdsmi_get_gpu_device_uuid", &f->uuid);
  Resolve(dl, "amdsmi_get_gpu_device_bdf", &f->bdf);
  Resolve(dl, "amdsmi_get_gpu_enumeration_info", &f->enum_info);
  Resolve(dl, "amdsmi_get_gpu_topo_numa_affinity", &f->numa);
  Resolve(dl, "amdsmi_get_gpu_vram_info", &f->vram_info);
  Resolve(dl, "amdsmi_get_gpu_memory_total", &f->memory_total);
  Resolve(dl, "amdsmi_get_gpu_memory_usage", &f->memory_usage);
  Resolve(dl, "amdsmi_get_gpu_activity", &f->activity);
  Resolve(dl, "amdsmi_get_gpu_compute_partition", &f->compute_partition);
  Resolve(dl, "amdsmi_get_gpu_memory_partition", &f->memory_partition);
  Resolve(dl, "amdsmi_get_gpu_kfd_info", &f->kfd_info);
  Resolve(dl, "amdsmi_get_gpu_asic_info", &f->asic_info);
  Resolve(dl, "amdsmi_get_gpu_xcd_counter", &f->xcd_counter);
  Resolve(dl, "amdsmi_get_gpu_accelerator_partition_profile", &f->accel_profile);
  Resolve(dl, "amdsmi_get_gpu_accelerator_partition_profile_config", &f->accel_profile_config);
  Resolve(dl, "amdsmi_get_gpu_memory_partition_config", &f->memory_partition_config);
  Resolve(dl, "amdsmi_topo_get_link_type", &f->link_type);
  Resolve(dl, "amdsmi_topo_get_link_weight", &f->link_weight);
  Resolve(dl, "amdsmi_get_gpu_xgmi_link_status", &f->xgmi_link_status);
  Resolve(dl, "amdsmi_init_gpu_event_notification", &f->evt_init);
  Resolve(dl, "amdsmi_set_gpu_event_notification_mask", &f->evt_mask);
  Resolve(dl, "amdsmi_get_gpu_event_notification", &f->evt_get);
  Resolve(dl, "amdsmi_stop_gpu_event_notification", &f->evt_stop);
  Resolve(dl, "amdsmi_get_gpu_total_ecc_count", &f->ecc_total);
  Resolve(dl, "amdsmi_get_gpu_bad_page_info", &f->bad_pages);
  Resolve(dl, "amdsmi_get_gpu_bad_page_threshold", &f->bad_page_threshold);
  Resolve(dl, "amdsmi_get_gpu_process_list", &f->process_list);
  Resolve(dl, "amdsmi_status_code_to_string", &f->status_string);
  Resolve(dl, "amdsmi_get_lib_version", &f->lib_version);
  if (!f->init || !f->shut_down || !f->socket_handles || !f->processor_handles || !f->uuid ||
      !f->bdf) {
    return Unavailable(lib->path_ + " lacks required amdsmi symbols");
  }
  lib->f_ = std::move(f);
  amdsmi_status_t st = lib->f_->init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    const char* s = nullptr;
    if (lib->f_->status_string) lib->f_->status_string(st, &s);
    return Unavailable("amdsmi_init failed: " + std::string(s ? s : std::to_string(st)));
  }
  lib->initialized_ = true;
  return lib;
}

std::string Library::Version() const {
  if (!f_->lib_version) return "unknown";
  amdsmi_version_t v{};
  if (f_->lib_version(&v) != AMDSMI_STATUS_SUCCESS) return "unknown";
  char buf[64];
  snprintf(buf, sizeof(buf), "%u.%u.%u", v.major, v.minor, v.release);
  return buf;
}

Result<std::vector<ProcessorInfo>> Library::Enumerate() {
  uint32_t nsock = 0;
  if (f_->socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS)
    return Unavailable("amdsmi_get_socket_handles(count) failed");
  std::vector<amdsmi_socket_handle> sockets(nsock);
  if (nsock && f_->socket_handles(&nsock, sockets.data()) != AMDSMI_STATUS_SUCCESS)
    return Unavailable("amdsmi_get_socket_handles failed");
  sockets.resize(nsock);

  std::vector<ProcessorInfo> out;
  for (auto sock : sockets) {
    uint32_t np = 0;
    if (f_->processor_handles(sock, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> procs(np);
    if (np && f_->processor_handles(sock, &np, procs.data()) != AMDSMI_STATUS_SUCCESS) continue;
    procs.resize(np);
    for (auto h : procs) {
      if (f_->processor_type) {
        processor_type_t t = AMDSMI_PROCESSOR_TYPE_UNKNOWN;
        if (f_->processor_type(h, &t) == AMDSMI_STATUS_SUCCESS && t != AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          continue;
      }
      ProcessorInfo p;
      p.handle = h;
      char uuid[AMDSMI_GPU_UUID_SIZE + 16] = {0};
      unsigned int ulen = sizeof(uuid);
      if (f_->uuid(h, &ulen, uuid) != AMDSMI_STATUS_SUCCESS) {
        LOG_WARN(kComp, "skipping processor: uuid query failed");
        continue;
      }
      p.uuid = uuid;
      amdsmi_bdf_t bdf{};
      if (f_->bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) {
        p.bdf_id = bdf.as_uint;
        p.bdf = FormatBdf(bdf.as_uint);
      }
      if (f_->enum_info) {
        amdsmi_enumeration_info_t ei{};
        if (f_->enum_info(h, &ei) == AMDSMI_STATUS_SUCCESS) {
          p.render_minor = ei.drm_render;
          p.card_minor = ei.drm_card;
          p.hip_id = ei.hip_id;
        }
      }
      if (f_->numa) {
        int32_t n = -1;
        if (f_->numa(h, &n) == AMDSMI_STATUS_SUCCESS) p.numa_node = n;
      }
      if (f_->vram_info) {
        amdsmi_vram_info_t vi{};
        if (f_->vram_info(h, &vi) == AMDSMI_STATUS_SUCCESS) p.vram_mib = vi.vram_size;
      }
      if (!p.vram_mib && f_->memory_total) {
        uint64_t total = 0;
        if (f_->memory_total(h, AMDSMI_MEM_TYPE_VRAM, &total) == AMDSMI_STATUS_SUCCESS)
          p.vram_mib = total >> 20;
      }
      if (f_->compute_partition) {
        char buf[64] = {0};
        if (f_->compute_partition(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS)
          p.compute_partition = buf;
      }
      if (f_->memory_partition) {
        char buf[64] = {0};
        if (f_->memory_partition(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS)
          p.memory_partition = buf;
      }
      if (f_->kfd_info) {
        amdsmi_kfd_info_t ki{};
        if (f_->kfd_info(h, &ki) == AMDSMI_STATUS_SUCCESS) {
          if (ki.current_partition_id != 0xffffffffu) p.partition_id = ki.current_partition_id;
          p.kfd_node = ki.node_id;
        }
      }
      if (f_->asic_info) {
        amdsmi_asic_info_t ai{};
        if (f_->asic_info(h, &ai) == AMDSMI_STATUS_SUCCESS) {
          p.market_name = ai.market_name;
          p.asic_serial.assign(ai.asic_serial, strnlen(ai.asic_serial, sizeof(ai.asic_serial)));
          if (p.asic_serial == "N/A" || p.asic_serial == "0" || p.asic_serial == "0x0") p.asic_serial.clear();
          if (ai.num_of_compute_units != 0xffffffffu) p.num_cu = ai.num_of_compute_units;
        }
      }
      if (f_->xcd_counter) {
        uint16_t x = 0;
        if (f_->xcd_counter(h, &x) == AMDSMI_STATUS_SUCCESS) p.xcd_count = x;
      }
      ReadPartitionProfile(h, &p);
      out.push_back(std::move(p));
    }
  }
  return out;
}

void Library::ReadPartitionProfile(void* h, ProcessorInfo* p) {
  if (f_->accel_profile) {
    // Both structs are large (the config is ~10 KiB): heap, not the stack.
    auto prof = std::make_unique<amdsmi_accelerator_partition_profile_t>();
    uint32_t pid = 0;
    if (f_->accel_profile(h, prof.get(), &pid) == AMDSMI_STATUS_SUCCESS) {
      static const char* names[] = {"", "SPX", "DPX", "TPX", "QPX", "CPX"};
      unsigned t = static_cast<unsigned>(prof->profile_type);
      if (t >= 1 && t <= 5) p->profile_type = names[t];
      p->profile_partitions = prof->num_partitions;
      if (f_->accel_profile_config) {
        auto cfg = std::make_unique<amdsmi_accelerator_partition_profile_config_t>();
        amdsmi_status_t cs = f_->accel_profile_config(h, cfg.get());
        if (cs == AMDSMI_STATUS_SUCCESS) {
          uint32_t n = std::min<uint32_t>(cfg->num_resource_profiles, AMDSMI_MAX_CP_PROFILE_RESOURCES);
          for (uint32_t i = 0; i < n; ++i) {
            const auto& r = cfg->resource_profiles[i];
            LOG_DEBUG(kComp, "%s: partition resource profile %u: profile_index=%u type=%d resource=%u shared_by=%u",
                      p->bdf.c_str(), i, r.profile_index, static_cast<int>(r.resource_type), r.partition_resource,
                      r.num_partitions_share_resource);
            if (r.profile_index == prof->profile_index && r.resource_type == AMDSMI_ACCELERATOR_XCC)
              p->profile_xccs = r.partition_resource;
          }
        } else {
          LOG_DEBUG(kComp, "%s: accelerator partition profile config unavailable (status %d)", p->bdf.c_str(),
                    static_cast<int>(cs));
        }
        LOG_DEBUG(kComp, "%s: accelerator partition profile type=%s partitions=%u index=%u resources=%u xccs=%u",
                  p->bdf.c_str(), p->profile_type.c_str(), prof->num_partitions, prof->profile_index,
                  prof->num_resources, p->profile_xccs);
      }
    }
  }
  if (f_->memory_partition_config) {
    auto mc = std::make_unique<amdsmi_memory_partition_config_t>();
    amdsmi_status_t ms = f_->memory_partition_config(h, mc.get());
    if (ms != AMDSMI_STATUS_SUCCESS)
      LOG_DEBUG(kComp, "%s: memory partition config unavailable (status %d)", p->bdf.c_str(), static_cast<int>(ms));
    if (ms == AMDSMI_STATUS_SUCCESS) {
      uint32_t n = std::min<uint32_t>(mc->num_numa_ranges, AMDSMI_MAX_NUM_NUMA_NODES);
      uint64_t bytes = 0;
      for (uint32_t i = 0; i < n; ++i)
        if (mc->numa_range[i].end > mc->numa_range[i].start)
          bytes += mc->numa_range[i].end - mc->numa_range[i].start + 1;
      p->mem_ranges = n;
      p->mem_ranges_mib = bytes >> 20;
    }
  }
}

Link Library::GetLink(void* src, void* dst) {
  Link l;
  if (!f_->link_type) return l;
  uint64_t hops = 0;
  amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
  if (f_->link_type(src, dst, &hops, &t) != AMDSMI_STATUS_SUCCESS) return l;
  l.valid = true;
  l.hops = hops;
  l.type = static_cast<LinkType>(t);
  if (f_->link_weight) {
    uint64_t w = 0;
    if (f_->link_weight(src, dst, &w) == AMDSMI_STATUS_SUCCESS) l.weight = w;
  }
  return l;
}

int Library::XgmiLinksDown(void* h) {
  if (!f_->xgmi_link_status) return 0;
  amdsmi_xgmi_link_status_t s{};
  if (f_->xgmi_link_status(h, &s) != AMDSMI_STATUS_SUCCESS) return 0;
  int down = 0;
  for (uint32_t i = 0; i < s.total_links && i < AMDSMI_MAX_NUM_XGMI_LINKS; ++i)
    if (s.status[i] == AMDSMI_XGMI_LINK_DOWN) ++down;
  return down;
}

Status Library::EventsInit(const std::vector<void*>& handles, uint64_t mask) {
  if (!f_->evt_init || !f_->evt_mask || !f_->evt_get)
    return NotSupported("event notification API not present");
  std::lock_guard<std::mutex> lk(evt_mu_);
  std::vector<void*> fresh;  // registered by this call: undone if a later handle fails
  auto rollback = [&](size_t failed_at, const Status& why) {
    if (!fresh.empty() && !f_->evt_stop)
      LOG_WARN(kComp, "%zu event registration(s) cannot be undone: amdsmi_stop_gpu_event_notification missing",
               fresh.size());
    else if (!fresh.empty())
      LOG_WARN(kComp, "event registration failed on processor %zu of %zu: undoing the %zu made before it", failed_at,
               handles.size(), fresh.size());
    if (f_->evt_stop)
      for (void* r : fresh) f_->evt_stop(r);
    else  // still registered: remembered, so the next call does not initialise them twice
      evt_live_.insert(evt_live_.end(), fresh.begin(), fresh.end());
    return why;
  };
  for (size_t i = 0; i < handles.size(); ++i) {
    void* h = handles[i];
    const bool live = std::find(evt_live_.begin(), evt_live_.end(), h) != evt_live_.end();
    amdsmi_status_t st = AMDSMI_STATUS_SUCCESS;
    if (!live) {
      st = f_->evt_init(h);
      if (st != AMDSMI_STATUS_SUCCESS)
        return rollback(i, Status(st == AMDSMI_STATUS_NOT_SUPPORTED ? Code::kNotSupported : Code::kUnavailable,
                                  "amdsmi_init_gpu_event_notification failed (" + std::to_string(st) + ") on processor " +
                                      std::to_string(i)));
      fresh.push_back(h);  // initialised: stopped again if anything below fails
    }
    st = f_->evt_mask(h, mask);
    if (st != AMDSMI_STATUS_SUCCESS)
      return rollback(i, Unavailable("amdsmi_set_gpu_event_notification_mask failed (" + std::to_string(st) +
                                     ") on processor " + std::to_string(i)));
  }
  evt_live_.insert(evt_live_.end(), fresh.begin(), fresh.end());
  return Status::Ok();
}

Status Library::EventsWait(int timeout_ms, std::vector<Event>* out) {
  amdsmi_evt_notification_data_t data[16];
  uint32_t n = 16;
  amdsmi_status_t st = f_->evt_get(timeout_ms, &n, data);
  if (st == AMDSMI_STATUS_NO_DATA) return Status::Ok();
  if (st != AMDSMI_STATUS_SUCCESS)
    return Unavailable("amdsmi_get_gpu_event_notification failed (" + std::to_string(st) + ")");
  for (uint32_t i = 0; i < n && i < 16; ++i) {
    Event e;
    e.handle = data[i].processor_handle;
    e.type = static_cast<uint32_t>(data[i].event);
    e.message.assign(data[i].message, strnlen(data[i].message, sizeof(data[i].message)));
    out->push_back(std::move(e));
  }
  return Status::Ok();
}

void Library::EventsStop(const std::vector<void*>& handles) {
  std::lock_guard<std::mutex> lk(evt_mu_);
  for (void* h : handles) {
    auto it = std::find(evt_live_.begin(), evt_live_.end(), h);
    if (it == evt_live_.end()) continue;
    if (f_->evt_stop) f_->evt_stop(h);
    evt_live_.erase(it);
  }
}

void Library::EventsStopAll() {
  std::lock_guard<std::mutex> lk(evt_mu_);
  if (f_->evt_stop)
    for (void* h : evt_live_) f_->evt_stop(h);
  evt_live_.clear();
}

size_t Library::EventsRegistered() const {
  std::lock_guard<std::mutex> lk(evt_mu_);
  return evt_live_.size();
}

Result<uint64_t> Library::UncorrectableErrors(void* h) {
  if (!f_->ecc_total) return NotSupported("ecc query not present");
  amdsmi_error_count_t ec{};
  amdsmi_status_t st = f_->ecc_total(h, &ec);
  if (st != AMDSMI_STATUS_SUCCESS) return Unavailable("ecc query failed (" + std::to_string(st) + ")");
  return static_cast<uint64_t>(ec.uncorrectable_count);
}

Result<uint32_t> Library::RetiredPages(void* h) {
  if (!f_->bad_pages) return NotSupported("bad page query not present");
  uint32_t n = 0;
  amdsmi_status_t st = f_->bad_pages(h, &n, nullptr);  // count only
  if (st != AMDSMI_STATUS_SUCCESS) return Unavailable("bad page query failed (" + std::to_string(st) + ")");
  return n;
}

Result<uint64_t> Library::VramUsed(void* h) {
  if (!f_->memory_usage) return NotSupported("memory usage query not present");
  uint64_t used = 0;
  amdsmi_status_t st = f_->memory_usage(h, AMDSMI_MEM_TYPE_VRAM, &used);
  if (st != AMDSMI_STATUS_SUCCESS) return Unavailable("memory usage query failed (" + std::to_string(st) + ")");
  return used;
}

Result<uint32_t> Library::Activity(void* h) {
  if (!f_->activity) return NotSupported("activity query not present");
  amdsmi_engine_usage_t u{};
  amdsmi_status_t st = f_->activity(h, &u);
  if (st != AMDSMI_STATUS_SUCCESS) return Unavailable("activity query failed (" + std::to_string(st) + ")");
  return u.gfx_activity;
}

Result<uint32_t> Library::RetiredPageThreshold(void* h) {
  if (!f_->bad_page_threshold) return NotSupported("bad page threshold query not present");
  uint32_t t = 0;
  amdsmi_status_t st = f_->bad_page_threshold(h, &t);  // root only on current drivers
  if (st != AMDSMI_STATUS_SUCCESS) return Unavailable("bad page threshold query failed (" + std::to_string(st) + ")");
  return t;
}

std::pair<std::string, std::string> Library::PartitionModes(void* h) {
  std::pair<std::string, std::string> out;
  char buf[64];
  if (f_->compute_partition) {
    memset(buf, 0, sizeof(buf));
    if (f_->compute_partition(h, buf, sizeof(buf) - 1) == AMDSMI_STATUS_SUCCESS) out.first = buf;
  }
  if (f_->memory_partition) {
    memset(buf, 0, sizeof(buf));
    if (f_->memory_partition(h, buf, sizeof(buf) - 1) == AMDSMI_STATUS_SUCCESS) out.second = buf;
  }
  return out;
}

Status Library::Reinit() {
  EventsStopAll();  // the handles die with the shut-down; their registrations must not outlive them unstopped
  if (initialized_) f_->shut_down();
  initialized_ = false;
  amdsmi_status_t st = f_->init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    const char* s = nullptr;
    if (f_->status_string) f_->status_string(st, &s);
    return Unavailable("amdsmi_init failed: " + std::string(s ? s : std::to_string(st)));
  }
  initialized_ = true;
  return Status::Ok();
}

std::string Library::QueryReport() {
  std::string out = "{\"amdsmi\": \"" + Version() + "\", \"path\": \"" + path_ + "\", \"processors\": [";
  uint32_t nsock = 0;
  std::vector<amdsmi_processor_handle> all;
  if (f_->socket_handles(&nsock, nullptr) == AMDSMI_STATUS_SUCCESS && nsock) {
    std::vector<amdsmi_socket_handle> socks(nsock);
    if (f_->socket_handles(&nsock, socks.data()) == AMDSMI_STATUS_SUCCESS)
      for (uint32_t i = 0; i < nsock && i < socks.size(); ++i) {
        uint32_t np = 0;
        if (f_->processor_handles(socks[i], &np, nullptr) != AMDSMI_STATUS_SUCCESS || !np) continue;
        std::vector<amdsmi_processor_handle> ps(np);
        if (f_->processor_handles(socks[i], &np, ps.data()) == AMDSMI_STATUS_SUCCESS)
          all.insert(all.end(), ps.begin(), ps.begin() + std::min<size_t>(np, ps.size()));
      }
  }
  bool first = true;
  for (auto h : all) {
    std::string row;
    auto add = [&row](const char* name, int st, const std::string& value = "") {
      row += std::string(row.empty() ? "" : ", ") + "\"" + name + "\": {\"status\": " + std::to_string(st);
      if (!value.empty()) row += ", \"value\": " + value;
      row += "}";
    };
    auto q = [](const std::string& v) { return "\"" + v + "\""; };
    const int kMissing = -1;  // symbol not in this libamd_smi
    {
      char uuid[AMDSMI_GPU_UUID_SIZE + 16] = {0};
      unsigned int ulen = sizeof(uuid);
      int st = f_->uuid(h, &ulen, uuid);
      add("uuid", st, st == 0 ? q(uuid) : "");
    }
    {
      amdsmi_bdf_t b{};
      int st = f_->bdf(h, &b);
      add("bdf", st, st == 0 ? q(FormatBdf(b.as_uint)) : "");
    }
    if (f_->enum_info) {
      amdsmi_enumeration_info_t ei{};
      int st = f_->enum_info(h, &ei);
      add("enumeration_info", st, st == 0 ? std::to_string(ei.drm_render) : "");
    } else add("enumeration_info", kMissing);
    if (f_->numa) { int32_t n = -1; int st = f_->numa(h, &n); add("numa_affinity", st, st == 0 ? std::to_string(n) : ""); }
    else add("numa_affinity", kMissing);
    if (f_->vram_info) { amdsmi_vram_info_t vi{}; int st = f_->vram_info(h, &vi); add("vram_info", st, st == 0 ? std::to_string(vi.vram_size) : ""); }
    else add("vram_info", kMissing);
    if (f_->memory_usage) { uint64_t u = 0; int st = f_->memory_usage(h, AMDSMI_MEM_TYPE_VRAM, &u); add("memory_usage", st, st == 0 ? std::to_string(u) : ""); }
    else add("memory_usage", kMissing);
    if (f_->activity) { amdsmi_engine_usage_t u{}; int st = f_->activity(h, &u); add("activity", st, st == 0 ? std::to_string(u.gfx_activity) : ""); }
    else add("activity", kMissing);
    if (f_->compute_partition) { char b[64] = {0}; int st = f_->compute_partition(h, b, sizeof(b) - 1); add("compute_partition", st, st == 0 ? q(b) : ""); }
    else add("compute_partition", kMissing);
    if (f_->memory_partition) { char b[64] = {0}; int st = f_->memory_partition(h, b, sizeof(b) - 1); add("memory_partition", st, st == 0 ? q(b) : ""); }
    else add("memory_partition", kMissing);
    if (f_->kfd_info) { amdsmi_kfd_info_t ki{}; int st = f_->kfd_info(h, &ki); add("kfd_info", st, st == 0 ? std::to_string(ki.kfd_id) : ""); }
    else add("kfd_info", kMissing);
    if (f_->asic_info) { amdsmi_asic_info_t ai{}; int st = f_->asic_info(h, &ai); add("asic_info", st, st == 0 ? std::to_string(ai.num_of_compute_units) : ""); }
    else add("asic_info", kMissing);
    if (f_->xcd_counter) { uint16_t x = 0; int st = f_->xcd_counter(h, &x); add("xcd_counter", st, st == 0 ? std::to_string(x) : ""); }
    else add("xcd_counter", kMissing);
    if (f_->accel_profile) {
      auto prof = std::make_unique<amdsmi_accelerator_partition_profile_t>();
      uint32_t pid = 0;
      add("accelerator_partition_profile", f_->accel_profile(h, prof.get(), &pid));
    } else add("accelerator_partition_profile", kMissing);
    if (f_->memory_partition_config) {
      auto mc = std::make_unique<amdsmi_memory_partition_config_t>();
      add("memory_partition_config", f_->memory_partition_config(h, mc.get()));
    } else add("memory_partition_config", kMissing);
    if (f_->ecc_total) { amdsmi_error_count_t ec{}; int st = f_->ecc_total(h, &ec); add("total_ecc_count", st, st == 0 ? std::to_string(ec.uncorrectable_count) : ""); }
    else add("total_ecc_count", kMissing);
    if (f_->bad_pages) { uint32_t n = 0; int st = f_->bad_pages(h, &n, nullptr); add("bad_page_info", st, st == 0 ? std::to_string(n) : ""); }
    else add("bad_page_info", kMissing);
    if (f_->bad_page_threshold) { uint32_t t = 0; int st = f_->bad_page_threshold(h, &t); add("bad_page_threshold", st, st == 0 ? std::to_string(t) : ""); }
    else add("bad_page_threshold", kMissing);
    if (f_->xgmi_link_status) { amdsmi_xgmi_link_status_t xs{}; int st = f_->xgmi_link_status(h, &xs); add("xgmi_link_status", st, st == 0 ? std::to_string(xs.total_links) : ""); }
    else add("xgmi_link_status", kMissing);
    if (f_->process_list) {
      std::vector<amdsmi_proc_info_t> buf(64);
      uint32_t n = static_cast<uint32_t>(buf.size());
      int st = f_->process_list(h, &n, buf.data());
      add("process_list", st, st == 0 ? std::to_string(n) : "");
    } else add("process_list", kMissing);
    bool live;
    {
      std::lock_guard<std::mutex> lk(evt_mu_);
      live = std::find(evt_live_.begin(), evt_live_.end(), h) != evt_live_.end();
    }
    if (live) {
      add("event_notification_init", 0, "\"registered by this process\"");  // not re-registered: no double init
    } else if (f_->evt_init && f_->evt_mask && f_->evt_stop) {
      int st = f_->evt_init(h);
      add("event_notification_init", st);
      if (st == 0) {
        add("event_notification_mask", f_->evt_mask(h, EventMask(kEvtGpuPreReset) | EventMask(kEvtGpuPostReset)));
        add("event_notification_stop", f_->evt_stop(h));
      }
    } else add("event_notification_init", kMissing);
    out += std::string(first ? "" : ",") + "\n  {" + row + "}";
    first = false;
  }
  out += first ? "]}" : "\n]}";
  return out;
}

bool Library::Responsive(void* h) {
  char uuid[AMDSMI_GPU_UUID_SIZE + 16] = {0};
  unsigned int ulen = sizeof(uuid);
  return f_->uuid(h, &ulen, uuid) == AMDSMI_STATUS_SUCCESS;
}

}  // namespace adp::smi
