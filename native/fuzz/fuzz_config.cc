// Coverage-guided fuzzing (libFuzzer) of the configuration front end: the
// versioned config file (YAML through libyaml, and the strict subset parser
// used when libyaml is absent), the resource-config grammar
// (<original>:<new>:<replicas>,...) and the command line + environment
// (LoadConfig with an injected environment, no config file). Operators write
// these, but a DaemonSet's values come from templating and typos: anything
// must be either accepted or refused with a message, never crash. A
// resource-config that parses must name valid resources only. Also the two
// files operators edit by hand next to the daemon: the health state file
// (what parses must survive a write and a re-read unchanged) and a drain-file
// line (undraining names removes exactly those names).
#include <map>
#include <set>
#include <string>
#include <vector>

#include "common/log.h"
#include "daemon/config.h"
#include "daemon/yaml.h"
#include "health/health.h"
#include "strategy/strategy.h"

using namespace adp;

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size < 1) return 0;
  static bool quiet = (SetLogLevel(LogLevel::kError), true);
  (void)quiet;
  std::string body(reinterpret_cast<const char*>(data + 1), size - 1);
  switch (data[0] % 6) {
    case 4: {
      auto recs = health::Ledger::Parse(body);
      auto again = health::Ledger::Parse(health::Ledger::Serialize(recs));
      bool same = again.size() == recs.size();
      for (const auto& [k, r] : recs) {
        auto it = again.find(k);
        same = same && it != again.end() && it->second.fail == r.fail && it->second.reason == r.reason &&
               it->second.has_baseline == r.has_baseline && it->second.ecc_baseline == r.ecc_baseline &&
               it->second.ecc_seen == r.ecc_seen && it->second.resets == r.resets && it->second.gap == r.gap;
      }
      if (!same) {
        fprintf(stderr, "invariant violated: the health state does not survive a write and a re-read\n");
        abort();
      }
      break;
    }
    case 5: {
      // "<line>\n<names, comma separated>"
      size_t nl = body.find('\n');
      if (nl == std::string::npos) return 0;
      std::string line = body.substr(0, nl);
      if (line.find('\r') != std::string::npos) return 0;
      std::set<std::string> names = health::DrainTokens(body.substr(nl + 1));
      std::string rest = health::RemoveDrainNames(line, names);
      auto before = health::DrainTokens(line), after = health::DrainTokens(rest);
      for (const auto& t : before)
        if (names.count(t) == after.count(t)) {  // a name removed stays; any other stays
          fprintf(stderr, "invariant violated: '%s' after undraining from '%s'\n", t.c_str(), line.c_str());
          abort();
        }
      for (const auto& t : after)
        if (!before.count(t)) {
          fprintf(stderr, "invariant violated: '%s' appeared undraining '%s'\n", t.c_str(), line.c_str());
          abort();
        }
      break;
    }
    case 0: (void)daemon::ParseConfigFile(body); break;
    case 1: (void)yaml::ParseSubset(body); break;
    case 2: {
      auto rc = strategy::ResourceConfig::Parse(body);
      if (rc.ok())
        for (const auto& [orig, v] : rc->entries())
          if (!strategy::ValidResourceName(v.name)) {
            fprintf(stderr, "invariant violated: accepted resource name '%s'\n", v.name.c_str());
            abort();
          }
      break;
    }
    default: {
      // NUL-separated argv; flags that name files are refused by the kernel
      // (ENOENT) rather than read.
      std::vector<std::string> args{"amdgpu-device-plugin"};
      size_t b = 0;
      for (size_t i = 0; i <= body.size() && args.size() < 32; ++i)
        if (i == body.size() || body[i] == '\0') {
          args.push_back(body.substr(b, i - b));
          b = i + 1;
        }
      std::vector<const char*> argv;
      for (const auto& a : args) {
        if (a.rfind("--config", 0) == 0) return 0;  // would read a file of the input's choosing
        argv.push_back(a.c_str());
      }
      std::map<std::string, std::string> env;
      (void)daemon::LoadConfig(static_cast<int>(argv.size()), argv.data(), &env);
      break;
    }
  }
  return 0;
}
