#include "daemon/yaml.h"

#include <dlfcn.h>
#include <yaml.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>

#include "common/strings.h"

namespace adp::yaml {
namespace {

constexpr int kMaxDepth = 64;
constexpr size_t kMaxNodes = 100000;  // aliases included: no "billion laughs"

struct Api {
  void* handle = nullptr;
  int (*parser_initialize)(yaml_parser_t*) = nullptr;
  void (*parser_delete)(yaml_parser_t*) = nullptr;
  void (*parser_set_input_string)(yaml_parser_t*, const unsigned char*, size_t) = nullptr;
  int (*parser_parse)(yaml_parser_t*, yaml_event_t*) = nullptr;
  void (*event_delete)(yaml_event_t*) = nullptr;
  const char* (*get_version_string)() = nullptr;
};

const Api* LoadApi() {
  static std::once_flag once;
  static Api api;
  static bool ok = false;
  std::call_once(once, [] {
    std::vector<std::string> candidates;
    if (const char* env = std::getenv("ADP_LIBYAML"); env && *env) {
      candidates.push_back(env);
    } else {
      candidates = {"libyaml-0.so.2", "/usr/lib64/libyaml-0.so.2", "/opt/conda/lib/libyaml-0.so.2"};
    }
    for (const auto& c : candidates) {
      api.handle = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL);
      if (api.handle) break;
    }
    if (!api.handle) return;
    auto sym = [&](const char* name) { return dlsym(api.handle, name); };
    api.parser_initialize = reinterpret_cast<decltype(api.parser_initialize)>(sym("yaml_parser_initialize"));
    api.parser_delete = reinterpret_cast<decltype(api.parser_delete)>(sym("yaml_parser_delete"));
    api.parser_set_input_string =
        reinterpret_cast<decltype(api.parser_set_input_string)>(sym("yaml_parser_set_input_string"));
    api.parser_parse = reinterpret_cast<decltype(api.parser_parse)>(sym("yaml_parser_parse"));
    api.event_delete = reinterpret_cast<decltype(api.event_delete)>(sym("yaml_event_delete"));
    api.get_version_string = reinterpret_cast<decltype(api.get_version_string)>(sym("yaml_get_version_string"));
    ok = api.parser_initialize && api.parser_delete && api.parser_set_input_string && api.parser_parse &&
         api.event_delete && api.get_version_string;
  });
  return ok ? &api : nullptr;
}

// One libyaml event, copied out so the libyaml event can be freed at once.
struct Ev {
  yaml_event_type_t type = YAML_NO_EVENT;
  std::string anchor, tag, value;
  bool plain = false;
  int line = 0;
};

class Reader {
 public:
  Reader(const Api* api, const std::string& body) : api_(api) {
    api_->parser_initialize(&parser_);
    api_->parser_set_input_string(&parser_, reinterpret_cast<const unsigned char*>(body.data()), body.size());
  }
  ~Reader() { api_->parser_delete(&parser_); }
  Reader(const Reader&) = delete;
  Reader& operator=(const Reader&) = delete;

  Status Next(Ev* out) {
    yaml_event_t e;
    if (!api_->parser_parse(&parser_, &e)) {
      std::string msg = parser_.problem ? parser_.problem : "syntax error";
      if (parser_.context) msg = std::string(parser_.context) + ": " + msg;
      return InvalidArgument("yaml: line " + std::to_string(parser_.problem_mark.line + 1) + ": " + msg);
    }
    *out = Ev{};
    out->type = e.type;
    out->line = static_cast<int>(e.start_mark.line) + 1;
    auto str = [](const yaml_char_t* s) { return s ? std::string(reinterpret_cast<const char*>(s)) : std::string(); };
    switch (e.type) {
      case YAML_SCALAR_EVENT:
        out->anchor = str(e.data.scalar.anchor);
        out->tag = str(e.data.scalar.tag);
        out->value.assign(reinterpret_cast<const char*>(e.data.scalar.value), e.data.scalar.length);
        out->plain = e.data.scalar.style == YAML_PLAIN_SCALAR_STYLE && out->tag.empty();
        break;
      case YAML_ALIAS_EVENT:
        out->anchor = str(e.data.alias.anchor);
        break;
      case YAML_MAPPING_START_EVENT:
        out->anchor = str(e.data.mapping_start.anchor);
        out->tag = str(e.data.mapping_start.tag);
        break;
      case YAML_SEQUENCE_START_EVENT:
        out->anchor = str(e.data.sequence_start.anchor);
        out->tag = str(e.data.sequence_start.tag);
        break;
      default:
        break;
    }
    api_->event_delete(&e);
    return Status::Ok();
  }

 private:
  const Api* api_;
  yaml_parser_t parser_;
};

size_t CountNodes(const Node& n) {
  size_t c = 1;
  for (const auto& [_, v] : n.map) c += CountNodes(v);
  for (const auto& v : n.seq) c += CountNodes(v);
  return c;
}

bool IsMergeKey(const Node& k) { return k.kind == Node::kScalar && k.plain && k.value == "<<"; }

class Builder {
 public:
  explicit Builder(Reader* r) : r_(r) {}

  // Builds the node that starts with event `ev`.
  Status Build(const Ev& ev, Node* out, int depth) {
    if (depth > kMaxDepth) return InvalidArgument("yaml: line " + std::to_string(ev.line) + ": nesting too deep");
    if (++nodes_ > kMaxNodes) return InvalidArgument("yaml: document too large");
    out->line = ev.line;
    switch (ev.type) {
      case YAML_SCALAR_EVENT:
        out->kind = Node::kScalar;
        out->value = ev.value;
        out->plain = ev.plain;
        out->tag = ev.tag;
        if (ResolveTag(*out) == ScalarType::kNull && (ev.plain || ev.tag == YAML_NULL_TAG)) out->kind = Node::kNull;
        break;
      case YAML_ALIAS_EVENT: {
        auto it = anchors_.find(ev.anchor);
        if (it == anchors_.end())
          return InvalidArgument("yaml: line " + std::to_string(ev.line) + ": unknown anchor '" + ev.anchor +
                                 "' referenced");
        nodes_ += CountNodes(it->second);
        if (nodes_ > kMaxNodes) return InvalidArgument("yaml: document too large (alias expansion)");
        int line = out->line;
        *out = it->second;
        out->line = line;
        return Status::Ok();
      }
      case YAML_SEQUENCE_START_EVENT: {
        out->kind = Node::kSeq;
        out->tag = ev.tag;
        while (true) {
          Ev child;
          ADP_RETURN_IF_ERROR(r_->Next(&child));
          if (child.type == YAML_SEQUENCE_END_EVENT) break;
          out->seq.emplace_back();
          ADP_RETURN_IF_ERROR(Build(child, &out->seq.back(), depth + 1));
        }
        break;
      }
      case YAML_MAPPING_START_EVENT: {
        out->kind = Node::kMap;
        out->tag = ev.tag;
        std::vector<Node> merges;
        while (true) {
          Ev kev;
          ADP_RETURN_IF_ERROR(r_->Next(&kev));
          if (kev.type == YAML_MAPPING_END_EVENT) break;
          Node key, val;
          ADP_RETURN_IF_ERROR(Build(kev, &key, depth + 1));
          Ev vev;
          ADP_RETURN_IF_ERROR(r_->Next(&vev));
          ADP_RETURN_IF_ERROR(Build(vev, &val, depth + 1));
          if (key.kind == Node::kMap || key.kind == Node::kSeq)
            return InvalidArgument("yaml: line " + std::to_string(key.line) + ": a mapping key must be a scalar");
          if (IsMergeKey(key)) {
            merges.push_back(std::move(val));
            continue;
          }
          std::string k = key.kind == Node::kNull ? "null" : key.value;
          bool replaced = false;
          for (auto& [ek, ev2] : out->map)
            if (ek == k) {
              ev2 = std::move(val);  // last one wins, as in the JSON the reference builds
              replaced = true;
              break;  // keys are unique in out->map
            }
          if (!replaced) out->map.emplace_back(std::move(k), std::move(val));
        }
        // Merge keys: explicit keys win, then earlier merge sources win.
        for (const auto& m : merges) {
          std::vector<const Node*> sources;
          if (m.kind == Node::kMap) sources.push_back(&m);
          else if (m.kind == Node::kSeq)
            for (const auto& s : m.seq) sources.push_back(&s);
          else
            sources.push_back(&m);  // rejected below
          for (const Node* s : sources) {
            if (s->kind != Node::kMap)
              return InvalidArgument("yaml: line " + std::to_string(s->line) +
                                     ": map merge requires map or sequence of maps as the value");
            for (const auto& [k, v] : s->map)
              if (!out->Get(k)) out->map.emplace_back(k, v);
          }
        }
        break;
      }
      default:
        return InvalidArgument("yaml: line " + std::to_string(ev.line) + ": unexpected event");
    }
    if (!ev.anchor.empty()) anchors_[ev.anchor] = *out;
    return Status::Ok();
  }

  static ScalarType ResolveTag(const Node& n) {
    std::string canon;
    return Resolve(n, &canon);
  }

 private:
  Reader* r_;
  std::map<std::string, Node> anchors_;
  size_t nodes_ = 0;
};

bool ParseGoInt(std::string s, std::string* canonical) {
  s.erase(std::remove(s.begin(), s.end(), '_'), s.end());
  if (s.empty()) return false;
  bool neg = false;
  size_t i = 0;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  int base = 10;
  if (s.size() > i + 1 && s[i] == '0' && (s[i + 1] == 'x' || s[i + 1] == 'X')) {
    base = 16;
    i += 2;
  } else if (s.size() > i + 1 && s[i] == '0' && (s[i + 1] == 'b' || s[i + 1] == 'B')) {
    base = 2;
    i += 2;
  } else if (s.size() > i + 1 && s[i] == '0' && (s[i + 1] == 'o' || s[i + 1] == 'O')) {
    base = 8;
    i += 2;
  } else if (s.size() > i + 1 && s[i] == '0') {
    base = 8;
    i += 1;
  }
  if (i >= s.size()) return false;
  unsigned __int128 v = 0;
  for (; i < s.size(); ++i) {
    int d;
    char c = s[i];
    if (c >= '0' && c <= '9') d = c - '0';
    else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
    else return false;
    if (d >= base) return false;
    v = v * base + d;
    if (v > static_cast<unsigned __int128>(UINT64_MAX)) return false;
  }
  if (neg) {
    if (v > static_cast<unsigned __int128>(INT64_MAX) + 1) return false;
    *canonical = v == 0 ? "0" : "-" + std::to_string(static_cast<uint64_t>(v));
  } else {
    *canonical = std::to_string(static_cast<uint64_t>(v));
  }
  return true;
}

bool IsYamlFloat(const std::string& s) {
  // go-yaml v2: ^[-+]?(\.[0-9]+|[0-9]+(\.[0-9]*)?)([eE][-+]?[0-9]+)?$ and .inf/.nan forms.
  static const char* specials[] = {".inf", ".Inf", ".INF", "+.inf", "+.Inf", "+.INF", "-.inf",
                                   "-.Inf", "-.INF", ".nan", ".NaN", ".NAN"};
  for (const char* sp : specials)
    if (s == sp) return true;
  size_t i = 0, n = s.size();
  if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
  size_t digits = 0;
  while (i < n && isdigit(static_cast<unsigned char>(s[i]))) ++i, ++digits;
  if (i < n && s[i] == '.') {
    ++i;
    size_t frac = 0;
    while (i < n && isdigit(static_cast<unsigned char>(s[i]))) ++i, ++frac;
    if (digits == 0 && frac == 0) return false;
  } else if (digits == 0) {
    return false;
  }
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
    size_t exp = 0;
    while (i < n && isdigit(static_cast<unsigned char>(s[i]))) ++i, ++exp;
    if (exp == 0) return false;
  }
  return i == n;
}

// ---- strict block-style subset (no libyaml) --------------------------------

Status NeedsLibyaml(int line, const std::string& what) {
  return InvalidArgument("yaml: line " + std::to_string(line) + ": " + what +
                         " needs libyaml (libyaml-0.so.2), which could not be loaded; install the libyaml "
                         "package or write the file in plain block style");
}

std::string UnquoteSubset(const std::string& v, int line, Status* st) {
  if (v.size() >= 2 && v.front() == '\'' && v.back() == '\'') {
    std::string out;
    for (size_t i = 1; i + 1 < v.size(); ++i) {
      out += v[i];
      if (v[i] == '\'' && i + 2 < v.size() && v[i + 1] == '\'') ++i;  // '' -> '
    }
    return out;
  }
  if (v.size() >= 2 && v.front() == '"' && v.back() == '"') {
    std::string out;
    for (size_t i = 1; i + 1 < v.size(); ++i) {
      if (v[i] != '\\') {
        out += v[i];
        continue;
      }
      if (i + 2 >= v.size()) break;
      char e = v[++i];
      switch (e) {
        case 'n': out += '\n'; break;
        case 't': out += '\t'; break;
        case '\\': out += '\\'; break;
        case '"': out += '"'; break;
        case '/': out += '/'; break;
        default: *st = NeedsLibyaml(line, std::string("the escape \\") + e);
      }
    }
    return out;
  }
  return v;
}

}  // namespace

const Node* Node::Get(const std::string& key) const {
  for (const auto& [k, v] : map)
    if (k == key) return &v;
  return nullptr;
}

ScalarType Resolve(const Node& n, std::string* canonical) {
  *canonical = n.value;
  if (n.kind == Node::kNull) return ScalarType::kNull;
  if (!n.tag.empty()) {
    const std::string& t = n.tag;
    if (t == YAML_NULL_TAG) return ScalarType::kNull;
    if (t == YAML_BOOL_TAG) {
      Node plain = n;
      plain.tag.clear();
      plain.plain = true;
      std::string c;
      if (Resolve(plain, &c) == ScalarType::kBool) {
        *canonical = c;
        return ScalarType::kBool;
      }
      return ScalarType::kString;
    }
    if (t == YAML_INT_TAG && ParseGoInt(n.value, canonical)) return ScalarType::kInt;
    if (t == YAML_FLOAT_TAG && IsYamlFloat(n.value)) return ScalarType::kFloat;
    *canonical = n.value;
    return ScalarType::kString;  // !!str and unknown tags
  }
  if (!n.plain) return ScalarType::kString;
  const std::string& s = n.value;
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return ScalarType::kNull;
  static const char* yes[] = {"y", "Y", "yes", "Yes", "YES", "true", "True", "TRUE", "on", "On", "ON"};
  static const char* no[] = {"n", "N", "no", "No", "NO", "false", "False", "FALSE", "off", "Off", "OFF"};
  for (const char* v : yes)
    if (s == v) {
      *canonical = "true";
      return ScalarType::kBool;
    }
  for (const char* v : no)
    if (s == v) {
      *canonical = "false";
      return ScalarType::kBool;
    }
  char c0 = s[0];
  if (isdigit(static_cast<unsigned char>(c0)) || c0 == '+' || c0 == '-' || c0 == '.') {
    std::string c;
    if (ParseGoInt(s, &c)) {
      *canonical = c;
      return ScalarType::kInt;
    }
    if (IsYamlFloat(s)) return ScalarType::kFloat;
  }
  return ScalarType::kString;
}

const char* TypeName(ScalarType t) {
  switch (t) {
    case ScalarType::kNull: return "null";
    case ScalarType::kBool: return "bool";
    case ScalarType::kInt: return "number";
    case ScalarType::kFloat: return "number";
    case ScalarType::kString: return "string";
  }
  return "?";
}

bool Available() { return LoadApi() != nullptr; }

std::string LibraryVersion() {
  const Api* api = LoadApi();
  return api ? api->get_version_string() : "";
}

Result<Node> Parse(const std::string& body, bool* extra_docs) {
  if (extra_docs) *extra_docs = false;
  const Api* api = LoadApi();
  if (!api) return ParseSubset(body);
  Reader r(api, body);
  Builder b(&r);
  Node root;
  bool have_doc = false;
  while (true) {
    Ev ev;
    ADP_RETURN_IF_ERROR(r.Next(&ev));
    if (ev.type == YAML_STREAM_END_EVENT || ev.type == YAML_NO_EVENT) break;
    if (ev.type == YAML_STREAM_START_EVENT || ev.type == YAML_DOCUMENT_END_EVENT) continue;
    if (ev.type == YAML_DOCUMENT_START_EVENT) {
      if (have_doc) {
        if (extra_docs) *extra_docs = true;
        break;  // go-yaml's Unmarshal reads the first document only
      }
      have_doc = true;
      Ev first;
      ADP_RETURN_IF_ERROR(r.Next(&first));
      if (first.type == YAML_DOCUMENT_END_EVENT) continue;  // empty document
      ADP_RETURN_IF_ERROR(b.Build(first, &root, 0));
      continue;
    }
    return InvalidArgument("yaml: line " + std::to_string(ev.line) + ": unexpected event");
  }
  return root;
}

Result<Node> ParseSubset(const std::string& body) {
  Node root;
  // Open mappings: (indent of their keys, node).
  std::vector<std::pair<int, Node*>> stack;
  std::istringstream in(body);
  std::string line;
  int lineno = 0;
  bool seen_content = false;
  // A key whose value is on the following lines: its mapping is created by the
  // first more-indented key (or stays null).
  Node* pending = nullptr;
  int pending_indent = -1;
  while (std::getline(in, line)) {
    ++lineno;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    // Strip comments outside quotes.
    char quote = 0;
    for (size_t i = 0; i < line.size(); ++i) {
      char c = line[i];
      if (quote) {
        if (c == quote) quote = 0;
        continue;
      }
      if (c == '"' || c == '\'') quote = c;
      else if (c == '#' && (i == 0 || isspace(static_cast<unsigned char>(line[i - 1])))) {
        line.resize(i);
        break;
      }
    }
    if (line.find('\t') != std::string::npos && Trim(line).size() && line.find_first_not_of(" \t") > 0 &&
        line.find('\t') < line.find_first_not_of(" \t"))
      return InvalidArgument("yaml: line " + std::to_string(lineno) + ": found a tab character in indentation");
    std::string t = Trim(line);
    if (t.empty()) continue;
    if (t == "---" || StartsWith(t, "--- ")) {
      if (seen_content) return NeedsLibyaml(lineno, "a second document");
      if (t != "---") return NeedsLibyaml(lineno, "content after '---'");
      continue;
    }
    if (t == "...") continue;
    if (t[0] == '%') return NeedsLibyaml(lineno, "a directive");
    seen_content = true;
    if (t[0] == '-' && (t.size() == 1 || t[1] == ' ')) return NeedsLibyaml(lineno, "a sequence");
    if (t[0] == '{' || t[0] == '[') return NeedsLibyaml(lineno, "a flow collection");
    if (t[0] == '?') return NeedsLibyaml(lineno, "a complex key");
    int indent = 0;
    while (indent < static_cast<int>(line.size()) && line[indent] == ' ') ++indent;
    size_t colon = std::string::npos;
    quote = 0;
    for (size_t i = 0; i < t.size(); ++i) {
      char c = t[i];
      if (quote) {
        if (c == quote) quote = 0;
        continue;
      }
      if (c == '"' || c == '\'') quote = c;
      else if (c == ':' && (i + 1 == t.size() || t[i + 1] == ' ')) {
        colon = i;
        break;
      }
    }
    if (colon == std::string::npos)
      return InvalidArgument("yaml: line " + std::to_string(lineno) + ": could not find expected ':'");
    Status st;
    std::string rawkey = Trim(t.substr(0, colon));
    if (!rawkey.empty() && (rawkey[0] == '&' || rawkey[0] == '*' || rawkey[0] == '!'))
      return NeedsLibyaml(lineno, "an anchor, alias or tag");
    std::string key = UnquoteSubset(rawkey, lineno, &st);
    ADP_RETURN_IF_ERROR(st);
    if (key == "<<") return NeedsLibyaml(lineno, "a merge key");
    std::string val = Trim(t.substr(colon + 1));

    // Find the mapping this key belongs to.
    Node* parent = nullptr;
    if (pending && indent > pending_indent) {
      pending->kind = Node::kMap;
      stack.emplace_back(indent, pending);
      parent = pending;
    } else {
      while (!stack.empty() && stack.back().first > indent) stack.pop_back();
      if (stack.empty()) {
        if (root.kind == Node::kNull && indent == 0) {
          root.kind = Node::kMap;
          root.line = lineno;
          stack.emplace_back(0, &root);
        } else {
          return InvalidArgument("yaml: line " + std::to_string(lineno) + ": did not find expected key");
        }
      }
      if (stack.back().first != indent)
        return InvalidArgument("yaml: line " + std::to_string(lineno) + ": mapping values are not allowed here");
      parent = stack.back().second;
    }
    pending = nullptr;
    if (parent->Get(key))
      return InvalidArgument("yaml: line " + std::to_string(lineno) + ": duplicate key '" + key + "'");
    parent->map.emplace_back(key, Node{});
    Node& v = parent->map.back().second;
    v.line = lineno;
    if (val.empty()) {
      pending = &v;  // null unless a nested mapping follows
      pending_indent = indent;
      continue;
    }
    char c0 = val[0];
    if (c0 == '{' || c0 == '[') return NeedsLibyaml(lineno, "a flow collection");
    if (c0 == '|' || c0 == '>') return NeedsLibyaml(lineno, "a block scalar");
    if (c0 == '&' || c0 == '*' || c0 == '!') return NeedsLibyaml(lineno, "an anchor, alias or tag");
    if (c0 == '@' || c0 == '`')
      return InvalidArgument("yaml: line " + std::to_string(lineno) + ": found character that cannot start any token");
    if ((c0 == '"' || c0 == '\'') && (val.size() < 2 || val.back() != c0))
      return NeedsLibyaml(lineno, "a multi-line quoted scalar");
    v.kind = Node::kScalar;
    v.plain = !(c0 == '"' || c0 == '\'');
    v.value = UnquoteSubset(val, lineno, &st);
    ADP_RETURN_IF_ERROR(st);
    if (v.plain) {
      std::string canon;
      if (Resolve(v, &canon) == ScalarType::kNull) v.kind = Node::kNull;
    }
  }
  return root;
}

}  // namespace adp::yaml
