// Flag validation: the daemon's Config checked and turned into the options of
// each layer (partition strategy, plugin options, resource config, snapshot
// options). Parity: reference cmd/nvidia-device-plugin/main.go:140-169
// (validateFlags + setup).
#pragma once

#include <set>

#include <string>

#include "common/status.h"
#include "daemon/config.h"
#include "inventory/inventory.h"
#include "plugin/plugin.h"
#include "strategy/strategy.h"

namespace adp::daemon {

struct Validated {
  strategy::PartitionStrategy partition;
  plugin::PluginOptions popts;
  strategy::ResourceConfig rc;
  inventory::BuildOptions bopts;
  std::set<uint32_t> extra_event_types;  // --health-event-extra-types
};

Result<Validated> Validate(const Config& cfg);

// The HBM-cap shim shipped with the daemon: --memcap-lib, else next to the
// binary, else the image's library directory. "" if none exists.
std::string MemcapSource(const Flags& f);

}  // namespace adp::daemon
