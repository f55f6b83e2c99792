// libamdsmi_mock.so -- a stand-in for libamd_smi.so driven by a JSON fixture.
//
// It exports the subset of the amdsmi C ABI that native/src/smi/smi.cc resolves,
// compiled against the real /opt/rocm/include/amd_smi/amdsmi.h so the struct
// layouts match. It lets every plugin path (partition strategies on SPX/DPX/QPX/
// CPX x NPS nodes, 1..8 GPU xGMI meshes, health events, RAS errors, init failure)
// run on a machine without a GPU -- the reference has no device mock at all
// (SURVEY §4.1), so this is the backbone of the CPU test matrix.
//
// Fixture: $AMDSMI_MOCK_FIXTURE (JSON). Schema (all keys optional except gpus):
//   { "init_status": 0, "events_supported": true, "lib_version": [26,2,1],
//     "events_open_kfd": false,  event registration opens /dev/kfd (EPERM -> NO_PERM)
//     "evt_init_fail_on": [1],   amdsmi_init_gpu_event_notification fails (API_FAILED) on
//                                these processors (global enumeration index)
//     "event_fifo": "<path>", "state_dir": "<path>", "topology": "xgmi"|"pcie",
//     "numa_bw_penalty": false,
//     "gpus": [ { "uuid": "...", "bdf": "0000:0c:00.0", "numa": 0, "vram_mib": 294896,
//                 "num_cu": 256, "xcd": 8, "market_name": "...",
//                 "compute_partition": "SPX"|"DPX"|"QPX"|"CPX", "memory_partition": "NPS1",
//                 "partitions": N, "partition_uuids": "distinct"|"shared",
//                 "render_minor": 128, "card_minor": 0, "xgmi_links_down": 0,
//                 -- how a partitioned GPU reports itself (real amdsmi shapes differ):
//                 "partition_vram": "share"|"pool"|"whole",  per-handle vram_info =
//                     GPU/partitions (default) | the handle's NPS pool | the whole GPU
//                 "partition_vram_mib": [..],  explicit per-partition values
//                 "asic_serial": "",            no ASIC serial (grouped by BDF)
//                 "partition_numa": "gpu"|"memory",  NUMA node of the GPU (default) or
//                     one node per memory partition (numa*NPS + pool index)
//                 "report_profile": true,       amdsmi_get_gpu_accelerator_partition_profile
//                 "report_numa_ranges": true,   amdsmi_get_gpu_memory_partition_config
//                 "kfd_node": 2 + 8*i,          KFD topology node of partition 0 (partition p
//                     is kfd_node + p): the order ROCr/HIP number the GPUs in, which
//                     need not be amdsmi's enumeration order ("kfd_node": null =
//                     amdsmi_get_gpu_kfd_info reports node_id unsupported)
//                 "render_denied": true,        asic_info and vram_info fail (FILE_ERROR), as
//                     with the render node denied by a device cgroup
//               } ] }
// Runtime injection:
//   event FIFO lines: "<gpu>[:<partition>] <event-type> [message]",
//                     "foreign <event-type> [message]" (on a processor handle
//                     that was never enumerated: amdsmi's handles not being
//                     the ones it handed out),
//                     "hang <ms>" (that event wait then returns only after <ms>),
//                     "fail <n>" (the next n event waits fail)
//   state_dir files:  gpu<i>.ecc (uncorrectable count; not a number = query fails),
//                     gpu<i>.dead (device gone),
//                     gpu<i>.partition ("CPX NPS2": live partition-mode override),
//                     gpu<i>.xgmi_down (number of xGMI links reported down),
//                     gpu<i>.badpages (retired HBM pages; not a number = query fails),
//                     gpu<i>.badpage_threshold (absent = the query needs root, as unprivileged),
//                     enumerate_fail (amdsmi_get_socket_handles answers BUSY)
//   amdsmi_shut_down + amdsmi_init re-reads the fixture (re-enumeration after a
//   re-partition).
// Registration accounting (tests of the rollback of a partial registration):
//   $AMDSMI_MOCK_EVT_FILE, when set, holds "live=<n> double_init=<n>
//   leaked_at_shutdown=<n> inits=<n> stops=<n>" after every change: live
//   registrations, inits of a handle already registered (the real library
//   would leak its KFD event file), handles still registered at
//   amdsmi_shut_down.
#include <amd_smi/amdsmi.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <json.hpp>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

namespace {

using nlohmann::json;

struct MockProc {
  int gpu = 0;
  int part = 0;
  std::string uuid;
  uint64_t bdf = 0;
  uint32_t render = 0;
  uint32_t card = 0;
  int numa = -1;
  uint64_t vram_mib = 0;
  uint32_t num_cu = 0;
  uint16_t xcd = 0;
  std::string market;
  std::string serial;
  std::string cmode, mmode;
  int nparts = 1;
  int nmem = 1;                 // memory partitions (NPS count)
  uint64_t gpu_vram_mib = 0;    // physical HBM of the whole GPU
  uint16_t gpu_xcd = 0;
  bool report_profile = true;
  bool report_numa_ranges = true;
  int links_down = 0;
  int64_t kfd_node = 0;         // -1: node_id not reported
  bool render_denied = false;   // asic_info / vram_info fail as without render-node access
  bool evt_init = false;
  uint64_t evt_mask = 0;
};

struct MockGpu {
  std::vector<MockProc*> procs;
};

struct State {
  bool loaded = false;
  int init_status = 0;
  bool events_supported = true;
  // Like the real library: event notification opens /dev/kfd, so a device
  // cgroup that denies it fails the registration (libadp_devcgroup_sim.so).
  bool events_open_kfd = false;
  uint32_t ver[3] = {26, 2, 1};
  std::string topology = "xgmi";
  std::string event_fifo, state_dir;
  int fifo_fd = -1;
  std::string fifo_buf;
  int fail_waits = 0;  // "fail <n>": the next n event waits fail
  std::vector<int> evt_init_fail_on;  // global processor indices whose registration fails
  std::vector<std::unique_ptr<MockProc>> procs;
  std::vector<MockGpu> gpus;
};

State* g = nullptr;
std::mutex g_mu;

uint64_t ParseBdf(const std::string& s) {
  unsigned dom = 0, bus = 0, dev = 0, fn = 0;
  sscanf(s.c_str(), "%x:%x:%x.%x", &dom, &bus, &dev, &fn);
  amdsmi_bdf_t b;
  b.as_uint = 0;
  b.domain_number = dom;
  b.bus_number = bus;
  b.device_number = dev;
  b.function_number = fn;
  return b.as_uint;
}

int DefaultPartitions(const std::string& mode) {
  if (mode == "DPX") return 2;
  if (mode == "TPX") return 3;
  if (mode == "QPX") return 4;
  if (mode == "CPX") return 8;
  return 1;
}

bool Load() {
  if (g && g->loaded) return true;
  if (!g) g = new State();
  const char* path = getenv("AMDSMI_MOCK_FIXTURE");
  if (!path) {
    fprintf(stderr, "amdsmi_mock: AMDSMI_MOCK_FIXTURE not set\n");
    return false;
  }
  std::ifstream in(path);
  if (!in) {
    fprintf(stderr, "amdsmi_mock: cannot open %s\n", path);
    return false;
  }
  json j;
  try {
    in >> j;
  } catch (const std::exception& e) {
    fprintf(stderr, "amdsmi_mock: bad fixture %s: %s\n", path, e.what());
    return false;
  }
  g->init_status = j.value("init_status", 0);
  g->events_supported = j.value("events_supported", true);
  g->events_open_kfd = j.value("events_open_kfd", false);
  g->topology = j.value("topology", std::string("xgmi"));
  g->event_fifo = j.value("event_fifo", std::string());
  g->state_dir = j.value("state_dir", std::string());
  if (const char* e = getenv("AMDSMI_MOCK_EVENT_FIFO")) g->event_fifo = e;
  if (const char* e = getenv("AMDSMI_MOCK_STATE_DIR")) g->state_dir = e;
  if (j.count("evt_init_fail_on"))
    for (const auto& v : j["evt_init_fail_on"]) g->evt_init_fail_on.push_back(v.get<int>());
  if (j.count("lib_version")) {
    for (int i = 0; i < 3; ++i) g->ver[i] = j["lib_version"][i].get<uint32_t>();
  }
  int gi = 0;
  for (const auto& jg : j["gpus"]) {
    MockGpu mg;
    std::string cmode = jg.value("compute_partition", std::string("SPX"));
    std::string mmode = jg.value("memory_partition", std::string("NPS1"));
    int nparts = jg.value("partitions", DefaultPartitions(cmode));
    if (nparts < 1) nparts = 1;
    char defuuid[64];
    snprintf(defuuid, sizeof(defuuid), "%08x-0000-1000-80c0-%012llx", 0x75a30000u + gi,
             static_cast<unsigned long long>(0xbf9907890000ull + gi));
    std::string uuid = jg.value("uuid", std::string(defuuid));
    char defbdf[32];
    snprintf(defbdf, sizeof(defbdf), "0000:%02x:00.0", 0x0c + 0x20 * gi);
    uint64_t bdf = ParseBdf(jg.value("bdf", std::string(defbdf)));
    uint32_t render = jg.value("render_minor", 128u + 8u * gi);
    uint32_t card = jg.value("card_minor", 8u * gi);
    uint64_t vram = jg.value("vram_mib", static_cast<uint64_t>(294896));
    uint32_t ncu = jg.value("num_cu", 256u);
    uint16_t xcd = static_cast<uint16_t>(jg.value("xcd", 8));
    bool shared = jg.value("partition_uuids", std::string("distinct")) == "shared";
    int nmem = 1;
    if (mmode.size() > 3 && mmode.compare(0, 3, "NPS") == 0) nmem = atoi(mmode.c_str() + 3);
    if (nmem < 1) nmem = 1;
    std::string vram_shape = jg.value("partition_vram", std::string("share"));
    std::vector<uint64_t> explicit_vram;
    if (jg.count("partition_vram_mib"))
      for (const auto& v : jg["partition_vram_mib"]) explicit_vram.push_back(v.get<uint64_t>());
    bool numa_per_memory = jg.value("partition_numa", std::string("gpu")) == "memory";
    for (int p = 0; p < nparts; ++p) {
      auto mp = std::make_unique<MockProc>();
      mp->gpu = gi;
      mp->part = p;
      mp->uuid = uuid;
      if (p > 0 && !shared) {
        // Distinct per-partition UUID: encode the partition in the 3rd group.
        char buf[16];
        snprintf(buf, sizeof(buf), "%x", p);
        if (mp->uuid.size() > 15) mp->uuid[15] = buf[0];
      }
      amdsmi_bdf_t b;
      b.as_uint = bdf;
      b.function_number = p & 7;
      mp->bdf = b.as_uint;
      mp->render = render + p;
      mp->card = card + p;
      mp->numa = jg.value("numa", gi < 4 ? 0 : 1);
      int pool = nparts >= nmem ? p * nmem / nparts : 0;
      if (numa_per_memory) mp->numa = mp->numa * nmem + pool;
      // What a partition handle's vram_info reports (see the schema above).
      if (static_cast<size_t>(p) < explicit_vram.size()) mp->vram_mib = explicit_vram[p];
      else if (nparts == 1 || vram_shape == "whole") mp->vram_mib = vram;
      else if (vram_shape == "pool") mp->vram_mib = vram / nmem;
      else mp->vram_mib = vram / nparts;
      mp->nparts = nparts;
      mp->nmem = nmem;
      mp->gpu_vram_mib = vram;
      mp->gpu_xcd = xcd;
      mp->report_profile = jg.value("report_profile", true);
      mp->report_numa_ranges = jg.value("report_numa_ranges", true);
      mp->num_cu = nparts > 1 ? ncu / nparts : ncu;
      mp->xcd = nparts > 1 ? static_cast<uint16_t>(xcd / nparts ? xcd / nparts : 1) : xcd;
      mp->market = jg.value("market_name", std::string("AMD Instinct MI355X"));
      char defserial[32];
      snprintf(defserial, sizeof(defserial), "0x09C0BF99078973%02X", gi);
      mp->serial = jg.value("asic_serial", std::string(defserial));
      mp->cmode = cmode;
      mp->mmode = mmode;
      mp->links_down = jg.value("xgmi_links_down", 0);
      mp->render_denied = jg.value("render_denied", false);
      if (jg.count("kfd_node") && jg["kfd_node"].is_null()) mp->kfd_node = -1;
      else mp->kfd_node = jg.value("kfd_node", static_cast<int64_t>(2 + gi * 8)) + p;
      mg.procs.push_back(mp.get());
      g->procs.push_back(std::move(mp));
    }
    g->gpus.push_back(mg);
    ++gi;
  }
  g->loaded = true;
  return true;
}

MockProc* P(amdsmi_processor_handle h) {
  if (!g) return nullptr;
  for (auto& p : g->procs)
    if (p.get() == h) return p.get();
  return nullptr;
}

bool Dead(const MockProc* p) {
  if (!g || g->state_dir.empty()) return false;
  struct stat st;
  std::string f = g->state_dir + "/gpu" + std::to_string(p->gpu) + ".dead";
  return stat(f.c_str(), &st) == 0;
}

// Call accounting for tests that pin "no device-library calls on the RPC path"
// (reference defect B5): every query bumps a counter that is mirrored into
// $AMDSMI_MOCK_CALL_COUNT_FILE when set.
unsigned long long g_calls = 0;
void CountCall() {
  ++g_calls;
  const char* f = getenv("AMDSMI_MOCK_CALL_COUNT_FILE");
  if (!f) return;
  FILE* fp = fopen(f, "w");
  if (!fp) return;
  fprintf(fp, "%llu\n", g_calls);
  fclose(fp);
}

// Event registration accounting (outlives amdsmi_shut_down: process-wide).
struct EvtStats {
  long live = 0, double_init = 0, leaked_at_shutdown = 0, inits = 0, stops = 0;
} g_evt;
void WriteEvtStats() {
  const char* f = getenv("AMDSMI_MOCK_EVT_FILE");
  if (!f) return;
  FILE* fp = fopen(f, "w");
  if (!fp) return;
  fprintf(fp, "live=%ld double_init=%ld leaked_at_shutdown=%ld inits=%ld stops=%ld\n", g_evt.live,
          g_evt.double_init, g_evt.leaked_at_shutdown, g_evt.inits, g_evt.stops);
  fclose(fp);
}
void ForgetRegistrations() {  // amdsmi_shut_down: handles still registered were never stopped
  if (!g) return;
  for (auto& p : g->procs)
    if (p->evt_init) {
      ++g_evt.leaked_at_shutdown;
      --g_evt.live;
    }
  WriteEvtStats();
}

// A processor handle amdsmi never enumerated ("foreign" FIFO lines).
char g_foreign_handle;

#define GET_PROC(h)                                   \
  std::lock_guard<std::mutex> lk(g_mu);               \
  CountCall();                                        \
  MockProc* p = P(h);                                 \
  if (!p) return AMDSMI_STATUS_INVAL;                 \
  if (Dead(p)) return AMDSMI_STATUS_NOT_FOUND;

void CopyStr(char* dst, size_t len, const std::string& s) {
  if (!len) return;
  size_t n = s.size() < len - 1 ? s.size() : len - 1;
  memcpy(dst, s.data(), n);
  dst[n] = 0;
}

}  // namespace

extern "C" {

amdsmi_status_t amdsmi_init(uint64_t) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!Load()) return AMDSMI_STATUS_INIT_ERROR;
  auto st = static_cast<amdsmi_status_t>(g->init_status);
  if (st != AMDSMI_STATUS_SUCCESS) {  // a failed init leaves nothing to shut down
    if (g->fifo_fd >= 0) close(g->fifo_fd);
    delete g;
    g = nullptr;
  }
  return st;
}

amdsmi_status_t amdsmi_shut_down(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  ForgetRegistrations();
  if (g) {
    if (g->fifo_fd >= 0) close(g->fifo_fd);
    delete g;
    g = nullptr;
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_lib_version(amdsmi_version_t* v) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g || !v) return AMDSMI_STATUS_INVAL;
  v->major = g->ver[0];
  v->minor = g->ver[1];
  v->release = g->ver[2];
  v->build = "mock";
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_status_code_to_string(amdsmi_status_t status, const char** s) {
  static thread_local char buf[64];
  snprintf(buf, sizeof(buf), "AMDSMI_MOCK_STATUS_%d", static_cast<int>(status));
  *s = buf;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_socket_handles(uint32_t* count, amdsmi_socket_handle* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  CountCall();
  if (!g || !count) return AMDSMI_STATUS_INVAL;
  // state_dir/enumerate_fail: enumeration refused (a driver mid-reload).
  if (!g->state_dir.empty() && access((g->state_dir + "/enumerate_fail").c_str(), F_OK) == 0)
    return AMDSMI_STATUS_BUSY;
  uint32_t n = static_cast<uint32_t>(g->gpus.size());
  if (!out) { *count = n; return AMDSMI_STATUS_SUCCESS; }
  uint32_t m = *count < n ? *count : n;
  for (uint32_t i = 0; i < m; ++i) out[i] = &g->gpus[i];
  *count = m;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle sock, uint32_t* count,
                                             amdsmi_processor_handle* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  CountCall();
  if (!g || !count) return AMDSMI_STATUS_INVAL;
  MockGpu* mg = static_cast<MockGpu*>(sock);
  uint32_t n = static_cast<uint32_t>(mg->procs.size());
  if (!out) { *count = n; return AMDSMI_STATUS_SUCCESS; }
  uint32_t m = *count < n ? *count : n;
  for (uint32_t i = 0; i < m; ++i) out[i] = mg->procs[i];
  *count = m;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_type(amdsmi_processor_handle h, processor_type_t* t) {
  GET_PROC(h);
  *t = AMDSMI_PROCESSOR_TYPE_AMD_GPU;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_uuid(amdsmi_processor_handle h, unsigned int* len,
                                           char* uuid) {
  GET_PROC(h);
  if (*len < p->uuid.size() + 1) return AMDSMI_STATUS_INSUFFICIENT_SIZE;
  CopyStr(uuid, *len, p->uuid);
  *len = static_cast<unsigned>(p->uuid.size());
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_bdf(amdsmi_processor_handle h, amdsmi_bdf_t* bdf) {
  GET_PROC(h);
  bdf->as_uint = p->bdf;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_enumeration_info(amdsmi_processor_handle h,
                                                amdsmi_enumeration_info_t* info) {
  GET_PROC(h);
  memset(info, 0, sizeof(*info));
  info->drm_render = p->render;
  info->drm_card = p->card;
  // HIP/HSA number GPUs in KFD topology-node order, not amdsmi's: the rank of
  // this processor's node among all nodes (amdsmi order when none is reported).
  uint32_t idx = 0, rank = 0;
  for (auto& q : g->procs) {
    if (q.get() == p) break;
    ++idx;
  }
  if (p->kfd_node < 0) rank = idx;
  else
    for (auto& q : g->procs) rank += q->kfd_node >= 0 && q->kfd_node < p->kfd_node;
  info->hsa_id = rank + 1;
  info->hip_id = rank;
  CopyStr(info->hip_uuid, sizeof(info->hip_uuid), "GPU-" + p->uuid);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_topo_numa_affinity(amdsmi_processor_handle h, int32_t* numa) {
  GET_PROC(h);
  *numa = p->numa;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_vram_info(amdsmi_processor_handle h, amdsmi_vram_info_t* info) {
  GET_PROC(h);
  memset(info, 0, sizeof(*info));
  if (p->render_denied) return AMDSMI_STATUS_FILE_ERROR;  // libdrm could not open the render node
  info->vram_type = AMDSMI_VRAM_TYPE_HBM3E;
  CopyStr(info->vram_vendor, sizeof(info->vram_vendor), "MOCK");
  info->vram_size = p->vram_mib;
  info->vram_bit_width = 8192;
  info->vram_max_bandwidth = 8192;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_total(amdsmi_processor_handle h, amdsmi_memory_type_t,
                                            uint64_t* total) {
  GET_PROC(h);
  *total = p->vram_mib << 20;
  return AMDSMI_STATUS_SUCCESS;
}

// state_dir/gpu<i>.vram_used: MiB in use (default 0).
amdsmi_status_t amdsmi_get_gpu_memory_usage(amdsmi_processor_handle h, amdsmi_memory_type_t, uint64_t* used) {
  GET_PROC(h);
  uint64_t mib = 0;
  if (!g->state_dir.empty()) {
    std::ifstream f(g->state_dir + "/gpu" + std::to_string(p->gpu) + ".vram_used");
    if (!(f >> mib) && f.is_open()) return AMDSMI_STATUS_NOT_SUPPORTED;
  }
  *used = mib << 20;
  return AMDSMI_STATUS_SUCCESS;
}

// state_dir/gpu<i>.activity: the graphics activity in percent, or anything
// else for the driver's refusal while the GPU is in reset (AMDSMI_STATUS_BUSY).
amdsmi_status_t amdsmi_get_gpu_activity(amdsmi_processor_handle h, amdsmi_engine_usage_t* info) {
  GET_PROC(h);
  if (!info) return AMDSMI_STATUS_INVAL;
  memset(info, 0, sizeof(*info));
  if (!g->state_dir.empty()) {
    std::ifstream f(g->state_dir + "/gpu" + std::to_string(p->gpu) + ".activity");
    uint32_t pct = 0;
    if (f.is_open() && !(f >> pct)) return AMDSMI_STATUS_BUSY;
    info->gfx_activity = pct;
  }
  return AMDSMI_STATUS_SUCCESS;
}

// state_dir/gpu<i>.partition ("CPX NPS2") overrides the fixture's modes: an
// operator re-partitioning the GPU behind the daemon's back.
static bool PartitionOverride(const MockProc* p, std::string* cmode, std::string* mmode) {
  if (!g || g->state_dir.empty()) return false;
  std::ifstream f(g->state_dir + "/gpu" + std::to_string(p->gpu) + ".partition");
  return f && (f >> *cmode >> *mmode);
}

amdsmi_status_t amdsmi_get_gpu_compute_partition(amdsmi_processor_handle h, char* buf,
                                                 uint32_t len) {
  GET_PROC(h);
  std::string c, m;
  CopyStr(buf, len, PartitionOverride(p, &c, &m) ? c : p->cmode);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_partition(amdsmi_processor_handle h, char* buf,
                                                uint32_t len) {
  GET_PROC(h);
  std::string c, m;
  CopyStr(buf, len, PartitionOverride(p, &c, &m) ? m : p->mmode);
  return AMDSMI_STATUS_SUCCESS;
}

namespace {
amdsmi_accelerator_partition_type_t ProfileType(const std::string& mode) {
  if (mode == "SPX") return AMDSMI_ACCELERATOR_PARTITION_SPX;
  if (mode == "DPX") return AMDSMI_ACCELERATOR_PARTITION_DPX;
  if (mode == "TPX") return AMDSMI_ACCELERATOR_PARTITION_TPX;
  if (mode == "QPX") return AMDSMI_ACCELERATOR_PARTITION_QPX;
  if (mode == "CPX") return AMDSMI_ACCELERATOR_PARTITION_CPX;
  return AMDSMI_ACCELERATOR_PARTITION_INVALID;
}
}  // namespace

// The current accelerator partition profile: type, partition count and, per
// partition, the index of its XCC resource profile (profile_config below).
amdsmi_status_t amdsmi_get_gpu_accelerator_partition_profile(amdsmi_processor_handle h,
                                                             amdsmi_accelerator_partition_profile_t* prof,
                                                             uint32_t* partition_id) {
  GET_PROC(h);
  if (!p->report_profile) return AMDSMI_STATUS_NOT_SUPPORTED;
  memset(prof, 0, sizeof(*prof));
  prof->profile_type = ProfileType(p->cmode);
  prof->num_partitions = static_cast<uint32_t>(p->nparts);
  prof->memory_caps.nps_cap_mask = 0x3;  // NPS1 | NPS2
  prof->profile_index = static_cast<uint32_t>(prof->profile_type) - 1;
  prof->num_resources = 1;
  for (int i = 0; i < p->nparts && i < AMDSMI_MAX_ACCELERATOR_PARTITIONS; ++i) prof->resources[i][0] = prof->profile_index;
  if (partition_id) *partition_id = static_cast<uint32_t>(p->part);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_accelerator_partition_profile_config(
    amdsmi_processor_handle h, amdsmi_accelerator_partition_profile_config_t* cfg) {
  GET_PROC(h);
  if (!p->report_profile) return AMDSMI_STATUS_NOT_SUPPORTED;
  memset(cfg, 0, sizeof(*cfg));
  static const char* modes[] = {"SPX", "DPX", "QPX", "CPX"};
  static const int parts[] = {1, 2, 4, 8};
  cfg->num_profiles = 4;
  cfg->num_resource_profiles = 4;
  for (int i = 0; i < 4; ++i) {
    auto t = ProfileType(modes[i]);
    cfg->profiles[i].profile_type = t;
    cfg->profiles[i].num_partitions = static_cast<uint32_t>(parts[i]);
    cfg->profiles[i].profile_index = static_cast<uint32_t>(t) - 1;
    cfg->resource_profiles[i].profile_index = static_cast<uint32_t>(t) - 1;
    cfg->resource_profiles[i].resource_type = AMDSMI_ACCELERATOR_XCC;
    cfg->resource_profiles[i].partition_resource = static_cast<uint32_t>(p->gpu_xcd / parts[i]);
    cfg->resource_profiles[i].num_partitions_share_resource = 1;
  }
  return AMDSMI_STATUS_SUCCESS;
}

// NUMA memory ranges of the GPU (one per memory partition), whichever handle asks.
amdsmi_status_t amdsmi_get_gpu_memory_partition_config(amdsmi_processor_handle h,
                                                       amdsmi_memory_partition_config_t* cfg) {
  GET_PROC(h);
  if (!p->report_numa_ranges) return AMDSMI_STATUS_NOT_SUPPORTED;
  memset(cfg, 0, sizeof(*cfg));
  cfg->partition_caps.nps_cap_mask = 0x3;
  cfg->mp_mode = p->nmem == 1 ? AMDSMI_MEMORY_PARTITION_NPS1
                : p->nmem == 2 ? AMDSMI_MEMORY_PARTITION_NPS2
                : p->nmem == 4 ? AMDSMI_MEMORY_PARTITION_NPS4 : AMDSMI_MEMORY_PARTITION_NPS8;
  cfg->num_numa_ranges = static_cast<uint32_t>(p->nmem);
  uint64_t per = (p->gpu_vram_mib << 20) / static_cast<uint64_t>(p->nmem);
  for (int i = 0; i < p->nmem && i < AMDSMI_MAX_NUM_NUMA_NODES; ++i) {
    cfg->numa_range[i].memory_type = AMDSMI_VRAM_TYPE_HBM3E;
    cfg->numa_range[i].start = per * static_cast<uint64_t>(i);
    cfg->numa_range[i].end = per * static_cast<uint64_t>(i + 1) - 1;
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_kfd_info(amdsmi_processor_handle h, amdsmi_kfd_info_t* info) {
  GET_PROC(h);
  memset(info, 0, sizeof(*info));
  info->kfd_id = 1000 + p->gpu * 16 + p->part;
  info->node_id = p->kfd_node < 0 ? 0xffffffffu : static_cast<uint32_t>(p->kfd_node);
  info->current_partition_id = p->part;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_asic_info(amdsmi_processor_handle h, amdsmi_asic_info_t* info) {
  GET_PROC(h);
  memset(info, 0, sizeof(*info));
  if (p->render_denied) return AMDSMI_STATUS_FILE_ERROR;
  CopyStr(info->market_name, sizeof(info->market_name), p->market);
  CopyStr(info->asic_serial, sizeof(info->asic_serial), p->serial);
  info->vendor_id = 0x1002;
  info->device_id = 0x75a3;
  info->num_of_compute_units = p->num_cu;
  info->oam_id = p->gpu;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_xcd_counter(amdsmi_processor_handle h, uint16_t* xcd) {
  GET_PROC(h);
  *xcd = p->xcd;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_topo_get_link_type(amdsmi_processor_handle a, amdsmi_processor_handle b,
                                          uint64_t* hops, amdsmi_link_type_t* type) {
  std::lock_guard<std::mutex> lk(g_mu);
  CountCall();
  MockProc* pa = P(a);
  MockProc* pb = P(b);
  if (!pa || !pb) return AMDSMI_STATUS_INVAL;
  if (pa->gpu == pb->gpu) {
    *hops = 0;
    *type = AMDSMI_LINK_TYPE_INTERNAL;
  } else if (g->topology == "pcie") {
    *hops = pa->numa == pb->numa ? 2 : 3;
    *type = AMDSMI_LINK_TYPE_PCIE;
  } else {
    *hops = 1;
    *type = AMDSMI_LINK_TYPE_XGMI;
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_topo_get_link_weight(amdsmi_processor_handle a, amdsmi_processor_handle b,
                                            uint64_t* w) {
  std::lock_guard<std::mutex> lk(g_mu);
  CountCall();
  MockProc* pa = P(a);
  MockProc* pb = P(b);
  if (!pa || !pb) return AMDSMI_STATUS_INVAL;
  if (pa->gpu == pb->gpu) *w = 0;
  else if (g->topology == "pcie") *w = pa->numa == pb->numa ? 20 : 40;
  else *w = 15;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_xgmi_link_status(amdsmi_processor_handle h,
                                                amdsmi_xgmi_link_status_t* s) {
  GET_PROC(h);
  memset(s, 0, sizeof(*s));
  s->total_links = 8;
  int down = p->links_down;
  if (!g->state_dir.empty()) {  // gpu<i>.xgmi_down: live override (a link failing)
    std::ifstream f(g->state_dir + "/gpu" + std::to_string(p->gpu) + ".xgmi_down");
    int v;
    if (f >> v) down = v;
  }
  for (int i = 0; i < 8; ++i)
    s->status[i] = i < down ? AMDSMI_XGMI_LINK_DOWN : AMDSMI_XGMI_LINK_UP;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_total_ecc_count(amdsmi_processor_handle h,
                                               amdsmi_error_count_t* ec) {
  GET_PROC(h);
  memset(ec, 0, sizeof(*ec));
  if (!g->state_dir.empty()) {
    std::ifstream f(g->state_dir + "/gpu" + std::to_string(p->gpu) + ".ecc");
    uint64_t v = 0;
    if (f >> v) ec->uncorrectable_count = v;
    else if (f.is_open()) return AMDSMI_STATUS_NOT_SUPPORTED;  // e.g. "unsupported": the query fails
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_bad_page_info(amdsmi_processor_handle h, uint32_t* num_pages,
                                             amdsmi_retired_page_record_t* info) {
  GET_PROC(h);
  uint32_t n = 0;
  if (!g->state_dir.empty()) {
    std::ifstream f(g->state_dir + "/gpu" + std::to_string(p->gpu) + ".badpages");
    if (!(f >> n) && f.is_open()) return AMDSMI_STATUS_NOT_SUPPORTED;
  }
  if (info)
    for (uint32_t i = 0; i < std::min(n, *num_pages); ++i)
      info[i] = {0x100000000ull + i * 4096ull, 4096, AMDSMI_MEM_PAGE_STATUS_RESERVED};
  *num_pages = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_bad_page_threshold(amdsmi_processor_handle h, uint32_t* threshold) {
  GET_PROC(h);
  if (g->state_dir.empty()) return AMDSMI_STATUS_NO_PERM;
  std::ifstream f(g->state_dir + "/gpu" + std::to_string(p->gpu) + ".badpage_threshold");
  if (!(f >> *threshold)) return AMDSMI_STATUS_NO_PERM;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_init_gpu_event_notification(amdsmi_processor_handle h) {
  GET_PROC(h);
  if (!g->events_supported) return AMDSMI_STATUS_NOT_SUPPORTED;
  if (g->events_open_kfd) {
    int fd = open("/dev/kfd", O_RDWR | O_CLOEXEC);
    if (fd < 0 && errno == EPERM) return AMDSMI_STATUS_NO_PERM;
    if (fd >= 0) close(fd);
  }
  size_t index = 0;
  while (index < g->procs.size() && g->procs[index].get() != p) ++index;
  if (std::find(g->evt_init_fail_on.begin(), g->evt_init_fail_on.end(), static_cast<int>(index)) !=
      g->evt_init_fail_on.end())
    return AMDSMI_STATUS_API_FAILED;
  ++g_evt.inits;
  if (p->evt_init) ++g_evt.double_init;
  else ++g_evt.live;
  p->evt_init = true;
  WriteEvtStats();
  if (g->fifo_fd < 0 && !g->event_fifo.empty()) {
    // O_RDWR keeps a writer open so poll() blocks instead of reporting HUP.
    g->fifo_fd = open(g->event_fifo.c_str(), O_RDWR | O_NONBLOCK | O_CLOEXEC);
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_set_gpu_event_notification_mask(amdsmi_processor_handle h, uint64_t mask) {
  GET_PROC(h);
  if (!p->evt_init) return AMDSMI_STATUS_INIT_ERROR;
  p->evt_mask = mask;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_stop_gpu_event_notification(amdsmi_processor_handle h) {
  GET_PROC(h);
  ++g_evt.stops;
  if (p->evt_init) --g_evt.live;
  p->evt_init = false;
  WriteEvtStats();
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_event_notification(int timeout_ms, uint32_t* num,
                                                  amdsmi_evt_notification_data_t* data) {
  int fd;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g) return AMDSMI_STATUS_INIT_ERROR;
    fd = g->fifo_fd;
  }
  if (fd < 0) {
    if (timeout_ms > 0) usleep(static_cast<useconds_t>(timeout_ms) * 1000);
    *num = 0;
    return AMDSMI_STATUS_NO_DATA;
  }
  bool queued = false;  // lines read before and not yet handed out: return at once, as the library does
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g && g->fail_waits > 0) {
      --g->fail_waits;
      return AMDSMI_STATUS_API_FAILED;
    }
    queued = g && g->fifo_buf.find('\n') != std::string::npos;
  }
  pollfd pfd{fd, POLLIN, 0};
  int r = poll(&pfd, 1, queued ? 0 : timeout_ms);
  std::unique_lock<std::mutex> lk(g_mu);
  if (!g) return AMDSMI_STATUS_INIT_ERROR;
  int hang_ms = 0;
  if (r > 0) {
    char buf[4096];
    ssize_t n;
    while ((n = read(fd, buf, sizeof(buf))) > 0) g->fifo_buf.append(buf, n);
  }
  uint32_t cap = *num, got = 0;
  size_t nl;
  while (got < cap && (nl = g->fifo_buf.find('\n')) != std::string::npos) {
    std::string line = g->fifo_buf.substr(0, nl);
    g->fifo_buf.erase(0, nl + 1);
    std::istringstream ls(line);
    std::string target;
    int type = 0;
    if (!(ls >> target >> type)) continue;
    if (target == "hang") {  // fault injection: "hang <ms>" -- this wait does not return for that long
      hang_ms = type;
      continue;
    }
    if (target == "fail") {  // "fail <n>": the next n waits return AMDSMI_STATUS_API_FAILED
      g->fail_waits = type;
      continue;
    }
    std::string msg;
    std::getline(ls >> std::ws, msg);  // (the separator is not part of the message)
    if (target == "foreign") {  // a handle amdsmi never enumerated, while anything is registered
      bool any = false;
      for (auto& p : g->procs) any = any || p->evt_init;
      if (!any) continue;
      memset(&data[got], 0, sizeof(data[got]));
      data[got].processor_handle = &g_foreign_handle;
      data[got].event = static_cast<amdsmi_evt_notification_type_t>(type);
      CopyStr(data[got].message, sizeof(data[got].message), msg.empty() ? "mock event" : msg);
      ++got;
      continue;
    }
    int gpu = atoi(target.c_str());
    int part = 0;
    size_t colon = target.find(':');
    if (colon != std::string::npos) part = atoi(target.c_str() + colon + 1);
    MockProc* hit = nullptr;
    for (auto& p : g->procs)
      if (p->gpu == gpu && p->part == part) hit = p.get();
    if (!hit || !hit->evt_init) continue;
    if (!(hit->evt_mask & AMDSMI_EVENT_MASK_FROM_INDEX(type))) continue;
    memset(&data[got], 0, sizeof(data[got]));
    data[got].processor_handle = hit;
    data[got].event = static_cast<amdsmi_evt_notification_type_t>(type);
    CopyStr(data[got].message, sizeof(data[got].message), msg.empty() ? "mock event" : msg);
    ++got;
  }
  *num = got;
  if (hang_ms > 0) {
    lk.unlock();
    usleep(static_cast<useconds_t>(hang_ms) * 1000);
  }
  return got ? AMDSMI_STATUS_SUCCESS : AMDSMI_STATUS_NO_DATA;
}

}  // extern "C"
