// Coverage-guided fuzzing (libFuzzer) of the driver-side HBM scan
// (memcap/driver_usage.cc) over a synthetic /proc: two processes, each with a
// render-node descriptor whose fdinfo, /proc/<pid>/maps and cgroup come from
// the input. Processes in pods write none of these directly, but their maps
// name files they create (any path, any length) and their cgroup paths follow
// pod names, so the parsers see arbitrary text. Checks: no crash, and the
// bytes add up -- per GPU, what is attributed to grants plus what is not
// equals the total, and a grant's process count never exceeds the processes.
#include <fcntl.h>
#include <fuzzer/FuzzedDataProvider.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <string>

#include "common/log.h"
#include "memcap/driver_usage.h"

using namespace adp;

namespace {

std::string& Root() {
  static std::string* r = [] {
    SetLogLevel(LogLevel::kError);
    char tmpl[] = "/dev/shm/adp-fuzz-proc-XXXXXX";
    auto* s = new std::string(mkdtemp(tmpl));
    for (const char* pid : {"/100", "/101"}) {
      std::string p = *s + pid;
      mkdir(p.c_str(), 0700);
      mkdir((p + "/fd").c_str(), 0700);
      mkdir((p + "/fdinfo").c_str(), 0700);
      int rc = symlink("/dev/dri/renderD128", (p + "/fd/5").c_str());  // dangling is fine: readlink only
      (void)rc;
    }
    mkdir((*s + "/usage").c_str(), 0700);
    int fd = open((*s + "/usage/0123456789abcdef.memcap").c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0600);
    if (fd >= 0) close(fd);
    return s;
  }();
  return *r;
}

void Put(const std::string& path, const std::string& body) {
  int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
  if (fd < 0) return;
  ssize_t w = write(fd, body.data(), body.size());
  (void)w;
  close(fd);
}

[[noreturn]] void Fail(const char* what) {
  fprintf(stderr, "invariant violated: %s\n", what);
  abort();
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  const std::string& root = Root();
  FuzzedDataProvider in(data, size);
  auto grants = memcap::ListGrantFiles(root + "/usage");
  for (const char* pid : {"/100", "/101"}) {
    std::string p = root + pid;
    std::string info = in.ConsumeRandomLengthString(400);
    if (in.ConsumeBool()) info = "drm-pdev:\t0000:0c:00.0\ndrm-client-id:\t" + std::to_string(in.ConsumeIntegral<uint8_t>()) +
                                 "\ndrm-resident-vram:\t" + in.ConsumeRandomLengthString(24) + "\n" + info;
    Put(p + "/fdinfo/5", info);
    std::string maps = in.ConsumeRandomLengthString(1500);
    if (in.ConsumeBool() && !grants.empty()) {
      char line[256];
      snprintf(line, sizeof(line), "7f00-7f10 rw-s 00000000 %02x:%02x %llu %s\n", grants[0].dev_major,
               grants[0].dev_minor, static_cast<unsigned long long>(grants[0].ino),
               in.ConsumeBool() ? "/run/amdgpu-dp/memcap" : "/x/0123456789abcdef.memcap");
      maps = line + maps;
    }
    Put(p + "/maps", maps);
    Put(p + "/cgroup", in.ConsumeRandomLengthString(200));
  }
  auto scan = memcap::ScanDriverHbm(root, grants, in.ConsumeRandomLengthString(40));
  std::map<std::string, uint64_t> sum;
  for (const auto& [kb, bytes] : scan.by_grant) sum[kb.second] += bytes;
  for (const auto& [bdf, bytes] : scan.unattributed) sum[bdf] += bytes;
  for (const auto& [bdf, total] : scan.total)
    if (sum[bdf] != total) Fail("grant + unattributed bytes != total");
  for (const auto& [kb, n] : scan.grant_procs)
    if (n < 0 || static_cast<size_t>(n) > scan.procs.size()) Fail("more grant processes than processes");
  (void)memcap::ParseFdinfoSize(in.ConsumeRemainingBytesAsString());
  return 0;
}
