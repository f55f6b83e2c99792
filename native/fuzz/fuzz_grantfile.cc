// Coverage-guided fuzzing (libFuzzer) of what a container can write and the
// daemon reads back: a memory-unit grant's accounting file (mounted
// read-write into the pod, memcap/usage.h) and the /metrics exposition built
// from it and from the kubelet's PodResources names (namespace, pod and
// container names are the users'). Whatever the file and the names hold, the
// daemon must not crash, and every line of the exposition must stay valid
// Prometheus text -- one container cannot break the scrape of the node.
#include <fcntl.h>
#include <fuzzer/FuzzedDataProvider.h>
#include <unistd.h>

#include <cstddef>
#include <cstring>
#include <string>
#include <vector>

#include "../tools/node_model.h"
#include "common/log.h"
#include "memcap_area.h"
#include "memcap/usage.h"
#include "plugin/plugin.h"
#include "podresources/podresources.h"
#include "strategy/strategy.h"

using namespace adp;
namespace area = adp_memcap;

namespace {

[[noreturn]] void Fail(const char* what, const std::string& line) {
  fprintf(stderr, "invariant violated: %s: %s\n", what, line.c_str());
  abort();
}

// One exposition line: "# HELP|TYPE ...", or name{l="v",...} number.
void CheckLine(const std::string& ln) {
  if (ln.rfind("# HELP ", 0) == 0 || ln.rfind("# TYPE ", 0) == 0) return;
  size_t i = 0;
  auto name_char = [](char c, bool first) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_' || c == ':' || (!first && c >= '0' && c <= '9');
  };
  if (i >= ln.size() || !name_char(ln[i], true)) Fail("metric name", ln);
  while (i < ln.size() && name_char(ln[i], false)) ++i;
  if (i < ln.size() && ln[i] == '{') {
    ++i;
    while (true) {
      if (i < ln.size() && ln[i] == '}') { ++i; break; }
      if (i >= ln.size() || !name_char(ln[i], true)) Fail("label name", ln);
      while (i < ln.size() && name_char(ln[i], false)) ++i;
      if (ln.compare(i, 2, "=\"") != 0) Fail("label =\"", ln);
      i += 2;
      while (i < ln.size() && ln[i] != '"') {
        if (ln[i] == '\\') {
          if (i + 1 >= ln.size() || (ln[i + 1] != '\\' && ln[i + 1] != '"' && ln[i + 1] != 'n')) Fail("escape", ln);
          ++i;
        }
        ++i;
      }
      if (i >= ln.size()) Fail("unterminated label value", ln);
      ++i;
      if (i < ln.size() && ln[i] == ',') ++i;
    }
  }
  if (i >= ln.size() || ln[i] != ' ') Fail("space before the value", ln);
  std::string v = ln.substr(i + 1);
  char* end = nullptr;
  strtod(v.c_str(), &end);
  if (v.empty() || *end) Fail("value", ln);
}

struct Fixture {
  std::unique_ptr<plugin::Plugin> p;
  std::string dir;
};

Fixture& Fx() {
  static Fixture* f = [] {
    SetLogLevel(LogLevel::kError);
    auto* fx = new Fixture();
    char tmpl[] = "/dev/shm/adp-fuzz-grant-XXXXXX";
    fx->dir = mkdtemp(tmpl);
    auto snap = testing::NodeModel(2, 1);
    auto rc = strategy::ResourceConfig::Parse("gpu:gpu-mem-gb:-1");
    auto specs = strategy::BuildPluginSpecs(*snap, strategy::PartitionStrategy::kNone, *rc);
    plugin::PluginOptions po;
    po.register_with_kubelet = false;
    po.replica_policy = alloc::ReplicaPolicy::kPack;
    po.memcap_host_path = "/nonexistent/libadp_memcap.so";  // the shim is never loaded here
    po.memcap_usage_dir = fx->dir;
    fx->p = std::make_unique<plugin::Plugin>(snap, (*specs)[0], po);
    return fx;
  }();
  return *f;
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  Fixture& fx = Fx();
  FuzzedDataProvider in(data, size);
  const auto& ids = fx.p->advertised_ids();
  // The grant: 1-6 of the plugin's memory units (the file is named after them).
  std::vector<std::string_view> grant;
  size_t n = in.ConsumeIntegralInRange<size_t>(1, 6);
  size_t first = in.ConsumeIntegralInRange<size_t>(0, ids.size() - n);
  for (size_t i = 0; i < n; ++i) grant.push_back(ids[first + i]);
  std::string key = memcap::AllocationKey(grant);
  // The header as the container left it: raw bytes, usually with a valid
  // magic/version and the grant's own IDs, sometimes rewritten.
  std::vector<unsigned char> hdr(area::kHeaderBytes, 0);
  std::vector<uint8_t> raw = in.ConsumeBytes<uint8_t>(in.ConsumeIntegralInRange<size_t>(0, 1200));
  uint8_t mode = in.ConsumeIntegral<uint8_t>();
  if (!raw.empty()) memcpy(hdr.data(), raw.data(), std::min(raw.size(), hdr.size()));
  auto put32 = [&](size_t off, uint32_t v) { memcpy(hdr.data() + off, &v, 4); };
  if (mode & 1) {
    put32(offsetof(area::Area, magic), area::kMagic);
    put32(offsetof(area::Area, version), area::kVersion);
  }
  if (mode & 2) {
    std::string joined;
    for (auto id : grant) joined += (joined.empty() ? "" : ",") + std::string(id);
    if (mode & 4) joined += in.ConsumeRandomLengthString(64);  // rewritten by the container
    joined.resize(std::min<size_t>(joined.size(), area::kIdsBytes));
    put32(offsetof(area::Area, ids_len), static_cast<uint32_t>(joined.size()));
    memcpy(hdr.data() + offsetof(area::Area, ids), joined.data(), joined.size());
  }
  if (mode & 8) put32(offsetof(area::Area, devices), in.ConsumeIntegralInRange<uint32_t>(0, 80));
  std::string path = fx.dir + "/" + key + ".memcap";
  int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
  if (fd < 0) return 0;
  size_t len = (mode & 16) ? in.ConsumeIntegralInRange<size_t>(0, hdr.size()) : hdr.size();
  ssize_t w = write(fd, hdr.data(), len);
  (void)w;
  close(fd);

  std::vector<memcap::Usage> files;
  if (auto u = memcap::ReadGrant(fx.dir, key); u.ok()) files.push_back(std::move(*u));
  // PodResources rows naming the grant's devices, with names from the input.
  std::vector<podresources::Assignment> asg;
  bool with_pods = mode & 32;
  if (with_pods) {
    std::string ns = in.ConsumeRandomLengthString(40), pod = in.ConsumeRandomLengthString(300),
                ctr = in.ConsumeRandomLengthString(40);
    for (auto id : grant) asg.push_back({pod, ns, ctr, fx.p->resource_name(), std::string(id)});
  }
  std::string out;
  plugin::Plugin::AppendPrometheus({fx.p.get()}, &out, with_pods ? &asg : nullptr, nullptr, &files);
  size_t b = 0;
  while (b < out.size()) {
    size_t e = out.find('\n', b);
    if (e == std::string::npos) Fail("exposition does not end with a newline", out.substr(b));
    CheckLine(out.substr(b, e - b));
    b = e + 1;
  }
  unlink(path.c_str());
  return 0;
}
