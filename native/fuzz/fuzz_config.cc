// Coverage-guided fuzzing (libFuzzer) of the configuration front end: the
// versioned config file (YAML through libyaml, and the strict subset parser
// used when libyaml is absent), the resource-config grammar
// (<original>:<new>:<replicas>,...) and the command line + environment
// (LoadConfig with an injected environment, no config file). Operators write
// these, but a DaemonSet's values come from templating and typos: anything
// must be either accepted or refused with a message, never crash. A
// resource-config that parses must name valid resources only.
#include <map>
#include <string>
#include <vector>

#include "common/log.h"
#include "daemon/config.h"
#include "daemon/yaml.h"
#include "strategy/strategy.h"

using namespace adp;

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size < 1) return 0;
  static bool quiet = (SetLogLevel(LogLevel::kError), true);
  (void)quiet;
  std::string body(reinterpret_cast<const char*>(data + 1), size - 1);
  switch (data[0] % 4) {
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
