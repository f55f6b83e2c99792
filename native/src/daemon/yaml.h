// YAML documents for the versioned config file.
//
// Parity: the reference reads its config file with sigs.k8s.io/yaml
// (api/config/v1/config.go:70-94): go-yaml v2 turns any YAML 1.1 document --
// block or flow style, quoted/folded/literal scalars, anchors, aliases, merge
// keys -- into JSON, which is then unmarshalled into typed fields. Here the
// same documents are parsed by libyaml (dlopen'ed "libyaml-0.so.2", the
// Ubuntu/UBI package the image installs; the reference vendors its Go parser)
// into a Node tree, and plain scalars are resolved with go-yaml v2's rules
// (null ~, bools y/yes/on/true/..., ints incl. 0x/0o/0b, floats).
//
// Without libyaml a strict block-style subset parser is used: every construct
// it does not understand (flow collections, block scalars, anchors, tags,
// sequences, several documents) is an error that names the line and says
// libyaml is needed -- never a silent misreading.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "common/status.h"

namespace adp::yaml {

struct Node {
  enum Kind { kNull, kScalar, kMap, kSeq };
  Kind kind = kNull;
  std::string value;  // scalar text (after unquoting / folding)
  bool plain = false;  // plain scalar without an explicit tag: its type is resolved
  std::string tag;     // explicit tag, e.g. "tag:yaml.org,2002:str" ("" = none)
  std::vector<std::pair<std::string, Node>> map;  // document order, merge keys applied
  std::vector<Node> seq;
  int line = 0;  // 1-based line of the node's start
  const Node* Get(const std::string& key) const;
};

enum class ScalarType { kNull, kBool, kInt, kFloat, kString };

// go-yaml v2 resolution of a scalar node; `canonical` receives "true"/"false"
// for bools, the decimal value for ints, and the text otherwise.
ScalarType Resolve(const Node& n, std::string* canonical);
const char* TypeName(ScalarType t);

// True if libyaml could be loaded (once per process; ADP_LIBYAML overrides
// the library path).
bool Available();
std::string LibraryVersion();  // "" when unavailable

// Parses the first document of `body` (later documents are ignored, as
// go-yaml's Unmarshal does; `*extra_docs` reports them). An empty document is
// a kNull node. Uses libyaml when available, else the strict subset parser.
Result<Node> Parse(const std::string& body, bool* extra_docs = nullptr);
// The subset parser alone (exposed for tests).
Result<Node> ParseSubset(const std::string& body);

}  // namespace adp::yaml
