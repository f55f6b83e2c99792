#include "proto/messages.h"

#include <algorithm>

#include "proto/wire.h"

namespace adp::pb {
namespace {

Status Malformed(const char* what) {
  return InvalidArgument(std::string("malformed protobuf message: ") + what);
}

// Sub-message helper: encode into a scratch string, then emit as field.
template <typename M>
void PutMsg(std::string* o, uint32_t field, const M& m) {
  std::string tmp;
  Encode(m, &tmp);
  PutLen(o, field, tmp);
}

// Iterate fields; `fn(field, wt, reader)` returns false to signal a decode error.
template <typename Fn>
Status ForEachField(std::string_view b, const char* what, Fn fn) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.Next(&f, &wt)) {
    if (!fn(f, wt, r)) return Malformed(what);
  }
  if (!r.ok()) return Malformed(what);
  return Status::Ok();
}

bool ReadString(Reader& r, WireType wt, std::string* s) {
  if (wt != kLen) return false;
  std::string_view v;
  if (!r.ReadLen(&v)) return false;
  s->assign(v.data(), v.size());
  return true;
}
bool ReadAppend(Reader& r, WireType wt, std::vector<std::string>* v) {
  v->emplace_back();
  return ReadString(r, wt, &v->back());
}
bool ReadBool(Reader& r, WireType wt, bool* b) {
  if (wt != kVarint) return false;
  uint64_t x;
  if (!r.ReadVarint(&x)) return false;
  *b = x != 0;
  return true;
}
template <typename M>
bool ReadMsg(Reader& r, WireType wt, M* m) {
  if (wt != kLen) return false;
  std::string_view v;
  if (!r.ReadLen(&v)) return false;
  return Decode(v, m).ok();
}
bool ReadMapEntry(Reader& r, WireType wt, StrMap* m) {
  if (wt != kLen) return false;
  std::string_view v;
  if (!r.ReadLen(&v)) return false;
  std::string k, val;
  Status st = ForEachField(v, "map entry", [&](uint32_t f, WireType w, Reader& rr) {
    if (f == 1) return ReadString(rr, w, &k);
    if (f == 2) return ReadString(rr, w, &val);
    return rr.Skip(w);
  });
  if (!st.ok()) return false;
  m->emplace_back(std::move(k), std::move(val));
  return true;
}

}  // namespace

// ---------------- encoders ----------------

void Encode(const DevicePluginOptions& m, std::string* o) {
  PutBool(o, 1, m.pre_start_required);
  PutBool(o, 2, m.get_preferred_allocation_available);
}

void Encode(const RegisterRequest& m, std::string* o) {
  PutStr(o, 1, m.version);
  PutStr(o, 2, m.endpoint);
  PutStr(o, 3, m.resource_name);
  if (m.has_options) PutMsg(o, 4, m.options);
}

void Encode(const Device& m, std::string* o) {
  PutStr(o, 1, m.id);
  PutStr(o, 2, m.health);
  if (m.has_topology) {
    std::string topo;
    for (int64_t n : m.numa_nodes) {
      std::string node;
      PutInt64(&node, 1, n);
      PutLen(&topo, 1, node);
    }
    PutLen(o, 3, topo);
  }
}

void Encode(const ListAndWatchResponse& m, std::string* o) {
  for (const auto& d : m.devices) PutMsg(o, 1, d);
}

void Encode(const ContainerPreferredAllocationRequest& m, std::string* o) {
  for (const auto& s : m.available) PutLen(o, 1, s);
  for (const auto& s : m.must_include) PutLen(o, 2, s);
  PutInt32(o, 3, m.allocation_size);
}

void Encode(const PreferredAllocationRequest& m, std::string* o) {
  for (const auto& r : m.container_requests) PutMsg(o, 1, r);
}

void Encode(const PreferredAllocationResponse& m, std::string* o) {
  for (const auto& ids : m.container_responses) {
    std::string c;
    for (const auto& s : ids) PutLen(&c, 1, s);
    PutLen(o, 1, c);
  }
}

void Encode(const AllocateRequest& m, std::string* o) {
  for (const auto& ids : m.container_requests) {
    std::string c;
    for (const auto& s : ids) PutLen(&c, 1, s);
    PutLen(o, 1, c);
  }
}

void Encode(const Mount& m, std::string* o) {
  PutStr(o, 1, m.container_path);
  PutStr(o, 2, m.host_path);
  PutBool(o, 3, m.read_only);
}

void Encode(const DeviceSpec& m, std::string* o) {
  PutStr(o, 1, m.container_path);
  PutStr(o, 2, m.host_path);
  PutStr(o, 3, m.permissions);
}

void Encode(const ContainerAllocateResponse& m, std::string* o) {
  for (const auto& [k, v] : m.envs) PutMapEntry(o, 1, k, v);
  for (const auto& x : m.mounts) PutMsg(o, 2, x);
  for (const auto& x : m.devices) PutMsg(o, 3, x);
  for (const auto& [k, v] : m.annotations) PutMapEntry(o, 4, k, v);
  for (const auto& n : m.cdi_devices) {
    std::string c;
    PutStr(&c, 1, n);
    PutLen(o, 5, c);
  }
}

void Encode(const AllocateResponse& m, std::string* o) {
  for (const auto& r : m.container_responses) PutMsg(o, 1, r);
}

void Encode(const PreStartContainerRequest& m, std::string* o) {
  for (const auto& s : m.device_ids) PutLen(o, 1, s);
}

// ---------------- decoders ----------------

Status Decode(std::string_view b, DevicePluginOptions* m) {
  *m = {};
  return ForEachField(b, "DevicePluginOptions", [&](uint32_t f, WireType wt, Reader& r) {
    if (f == 1) return ReadBool(r, wt, &m->pre_start_required);
    if (f == 2) return ReadBool(r, wt, &m->get_preferred_allocation_available);
    return r.Skip(wt);
  });
}

Status Decode(std::string_view b, RegisterRequest* m) {
  *m = {};
  return ForEachField(b, "RegisterRequest", [&](uint32_t f, WireType wt, Reader& r) {
    if (f == 1) return ReadString(r, wt, &m->version);
    if (f == 2) return ReadString(r, wt, &m->endpoint);
    if (f == 3) return ReadString(r, wt, &m->resource_name);
    if (f == 4) { m->has_options = true; return ReadMsg(r, wt, &m->options); }
    return r.Skip(wt);
  });
}

Status Decode(std::string_view b, Device* m) {
  *m = {};
  return ForEachField(b, "Device", [&](uint32_t f, WireType wt, Reader& r) {
    if (f == 1) return ReadString(r, wt, &m->id);
    if (f == 2) return ReadString(r, wt, &m->health);
    if (f == 3) {
      if (wt != kLen) return false;
      std::string_view topo;
      if (!r.ReadLen(&topo)) return false;
      m->has_topology = true;
      return ForEachField(topo, "TopologyInfo", [&](uint32_t tf, WireType twt, Reader& tr) {
               if (tf != 1) return tr.Skip(twt);
               if (twt != kLen) return false;
               std::string_view node;
               if (!tr.ReadLen(&node)) return false;
               int64_t id = 0;
               Status st = ForEachField(node, "NUMANode", [&](uint32_t nf, WireType nwt, Reader& nr) {
                 if (nf != 1) return nr.Skip(nwt);
                 if (nwt != kVarint) return false;
                 uint64_t v;
                 if (!nr.ReadVarint(&v)) return false;
                 id = static_cast<int64_t>(v);
                 return true;
               });
               if (!st.ok()) return false;
               m->numa_nodes.push_back(id);
               return true;
             }).ok();
    }
    return r.Skip(wt);
  });
}

Status Decode(std::string_view b, ListAndWatchResponse* m) {
  *m = {};
  return ForEachField(b, "ListAndWatchResponse", [&](uint32_t f, WireType wt, Reader& r) {
    if (f == 1) { m->devices.emplace_back(); return ReadMsg(r, wt, &m->devices.back()); }
    return r.Skip(wt);
  });
}

Status Decode(std::string_view b, ContainerPreferredAllocationRequest* m) {
  *m = {};
  return ForEachField(b, "ContainerPreferredAllocationRequest",
                      [&](uint32_t f, WireType wt, Reader& r) {
    if (f == 1) return ReadAppend(r, wt, &m->available);
    if (f == 2) return ReadAppend(r, wt, &m->must_include);
    if (f == 3) {
      if (wt != kVarint) return false;
      uint64_t v;
      if (!r.ReadVarint(&v)) return false;
      m->allocation_size = static_cast<int32_t>(static_cast<int64_t>(v));
      return true;
    }
    return r.Skip(wt);
  });
}

Status Decode(std::string_view b, PreferredAllocationRequest* m) {
  *m = {};
  return ForEachField(b, "PreferredAllocationRequest", [&](uint32_t f, WireType wt, Reader& r) {
    if (f == 1) {
      m->container_requests.emplace_back();
      return ReadMsg(r, wt, &m->container_requests.back());
    }
    return r.Skip(wt);
  });
}

namespace {
Status DecodeIdList(std::string_view b, const char* what, std::vector<std::string>* ids) {
  return ForEachField(b, what, [&](uint32_t f, WireType wt, Reader& r) {
    if (f == 1) return ReadAppend(r, wt, ids);
    return r.Skip(wt);
  });
}
}  // namespace

Status Decode(std::string_view b, PreferredAllocationResponse* m) {
  *m = {};
  return ForEachField(b, "PreferredAllocationResponse", [&](uint32_t f, WireType wt, Reader& r) {
    if (f != 1) return r.Skip(wt);
    if (wt != kLen) return false;
    std::string_view c;
    if (!r.ReadLen(&c)) return false;
    m->container_responses.emplace_back();
    return DecodeIdList(c, "ContainerPreferredAllocationResponse", &m->container_responses.back()).ok();
  });
}

Status Decode(std::string_view b, AllocateRequest* m) {
  *m = {};
  return ForEachField(b, "AllocateRequest", [&](uint32_t f, WireType wt, Reader& r) {
    if (f != 1) return r.Skip(wt);
    if (wt != kLen) return false;
    std::string_view c;
    if (!r.ReadLen(&c)) return false;
    m->container_requests.emplace_back();
    return DecodeIdList(c, "ContainerAllocateRequest", &m->container_requests.back()).ok();
  });
}

Status Decode(std::string_view b, Mount* m) {
  *m = {};
  return ForEachField(b, "Mount", [&](uint32_t f, WireType wt, Reader& r) {
    if (f == 1) return ReadString(r, wt, &m->container_path);
    if (f == 2) return ReadString(r, wt, &m->host_path);
    if (f == 3) return ReadBool(r, wt, &m->read_only);
    return r.Skip(wt);
  });
}

Status Decode(std::string_view b, DeviceSpec* m) {
  *m = {};
  return ForEachField(b, "DeviceSpec", [&](uint32_t f, WireType wt, Reader& r) {
    if (f == 1) return ReadString(r, wt, &m->container_path);
    if (f == 2) return ReadString(r, wt, &m->host_path);
    if (f == 3) return ReadString(r, wt, &m->permissions);
    return r.Skip(wt);
  });
}

Status Decode(std::string_view b, ContainerAllocateResponse* m) {
  *m = {};
  return ForEachField(b, "ContainerAllocateResponse", [&](uint32_t f, WireType wt, Reader& r) {
    switch (f) {
      case 1: return ReadMapEntry(r, wt, &m->envs);
      case 2: m->mounts.emplace_back(); return ReadMsg(r, wt, &m->mounts.back());
      case 3: m->devices.emplace_back(); return ReadMsg(r, wt, &m->devices.back());
      case 4: return ReadMapEntry(r, wt, &m->annotations);
      case 5: {
        if (wt != kLen) return false;
        std::string_view c;
        if (!r.ReadLen(&c)) return false;
        std::string name;
        Status st = ForEachField(c, "CDIDevice", [&](uint32_t cf, WireType cwt, Reader& cr) {
          if (cf == 1) return ReadString(cr, cwt, &name);
          return cr.Skip(cwt);
        });
        if (!st.ok()) return false;
        m->cdi_devices.push_back(std::move(name));
        return true;
      }
      default: return r.Skip(wt);
    }
  });
}

Status Decode(std::string_view b, AllocateResponse* m) {
  *m = {};
  return ForEachField(b, "AllocateResponse", [&](uint32_t f, WireType wt, Reader& r) {
    if (f == 1) {
      m->container_responses.emplace_back();
      return ReadMsg(r, wt, &m->container_responses.back());
    }
    return r.Skip(wt);
  });
}

namespace {
bool ReadView(Reader& r, WireType wt, std::vector<std::string_view>* v) {
  if (wt != kLen) return false;
  std::string_view s;
  if (!r.ReadLen(&s)) return false;
  v->push_back(s);
  return true;
}
}  // namespace

Status DecodeView(std::string_view b, std::vector<ContainerPreferredAllocationRequestView>* m) {
  // Elements already in *m are reused with their capacity (a caller that keeps
  // the vector across calls decodes 2,352-ID requests without touching malloc).
  size_t n = 0;
  Status st = ForEachField(b, "PreferredAllocationRequest", [&](uint32_t f, WireType wt, Reader& r) {
    if (f != 1) return r.Skip(wt);
    if (wt != kLen) return false;
    std::string_view c;
    if (!r.ReadLen(&c)) return false;
    if (n == m->size()) m->emplace_back();
    auto& cr = (*m)[n++];
    cr.available.clear();
    cr.must_include.clear();
    cr.allocation_size = 0;
    // One growth step up front, sized from the first entry (tag + length + ID;
    // the kubelet's IDs of one resource have one shape).
    size_t first = c.size() >= 2 ? static_cast<uint8_t>(c[1]) : 0;
    if (c.size() >= 2 && c[0] == 0x0a && first < 0x80)  // bounded: a tiny first ID must not pin megabytes
      cr.available.reserve(std::min<size_t>(c.size() / (2 + first + (first == 0)) + 1, 16384));
    // Fast path: the run of available_deviceIDs (field 1, length < 128) the
    // kubelet writes first -- two header bytes per ID, no varint loop.
    const char* p = c.data();
    const char* end = p + c.size();
    while (end - p >= 2 && p[0] == 0x0a && !(static_cast<uint8_t>(p[1]) & 0x80)) {
      size_t len = static_cast<uint8_t>(p[1]);
      if (static_cast<size_t>(end - p - 2) < len) return false;
      cr.available.emplace_back(p + 2, len);
      p += 2 + len;
    }
    c.remove_prefix(static_cast<size_t>(p - c.data()));
    return ForEachField(c, "ContainerPreferredAllocationRequest", [&](uint32_t cf, WireType cwt, Reader& cr_r) {
             if (cf == 1) return ReadView(cr_r, cwt, &cr.available);
             if (cf == 2) return ReadView(cr_r, cwt, &cr.must_include);
             if (cf == 3) {
               if (cwt != kVarint) return false;
               uint64_t v;
               if (!cr_r.ReadVarint(&v)) return false;
               cr.allocation_size = static_cast<int32_t>(static_cast<int64_t>(v));
               return true;
             }
             return cr_r.Skip(cwt);
           }).ok();
  });
  m->resize(n);
  return st;
}

Status DecodeView(std::string_view b, std::vector<std::vector<std::string_view>>* m) {
  m->clear();
  return ForEachField(b, "AllocateRequest", [&](uint32_t f, WireType wt, Reader& r) {
    if (f != 1) return r.Skip(wt);
    if (wt != kLen) return false;
    std::string_view c;
    if (!r.ReadLen(&c)) return false;
    m->emplace_back();
    auto& ids = m->back();
    return ForEachField(c, "ContainerAllocateRequest", [&](uint32_t cf, WireType cwt, Reader& cr) {
             if (cf == 1) return ReadView(cr, cwt, &ids);
             return cr.Skip(cwt);
           }).ok();
  });
}

Status Decode(std::string_view b, PreStartContainerRequest* m) {
  *m = {};
  return DecodeIdList(b, "PreStartContainerRequest", &m->device_ids);
}

}  // namespace adp::pb
