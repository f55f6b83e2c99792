#include "podresources/podresources.h"

#include "grpc/grpc.h"
#include "proto/wire.h"

namespace adp::podresources {
namespace {

Status Bad(const char* what) { return InvalidArgument(std::string("malformed ListPodResourcesResponse: ") + what); }

Status DecodeDevices(std::string_view b, const std::string& pod, const std::string& ns, const std::string& ctr,
                     std::vector<Assignment>* out) {
  pb::Reader r(b);
  uint32_t f;
  pb::WireType wt;
  std::string resource;
  std::vector<std::string> ids;
  while (r.Next(&f, &wt)) {
    std::string_view v;
    if (f == 1 && wt == pb::kLen) {
      if (!r.ReadLen(&v)) return Bad("resource_name");
      resource.assign(v);
    } else if (f == 2 && wt == pb::kLen) {
      if (!r.ReadLen(&v)) return Bad("device_ids");
      ids.emplace_back(v);
    } else if (!r.Skip(wt)) {
      return Bad("devices");
    }
  }
  if (!r.ok()) return Bad("devices");
  for (auto& id : ids) out->push_back({pod, ns, ctr, resource, std::move(id)});
  return Status::Ok();
}

Status DecodeContainer(std::string_view b, const std::string& pod, const std::string& ns,
                       std::vector<Assignment>* out) {
  pb::Reader r(b);
  uint32_t f;
  pb::WireType wt;
  std::string name;
  std::vector<std::string_view> devices;
  while (r.Next(&f, &wt)) {
    std::string_view v;
    if (f == 1 && wt == pb::kLen) {
      if (!r.ReadLen(&v)) return Bad("container name");
      name.assign(v);
    } else if (f == 2 && wt == pb::kLen) {
      if (!r.ReadLen(&v)) return Bad("container devices");
      devices.push_back(v);
    } else if (!r.Skip(wt)) {
      return Bad("container");
    }
  }
  if (!r.ok()) return Bad("container");
  for (auto d : devices) {
    Status st = DecodeDevices(d, pod, ns, name, out);
    if (!st.ok()) return st;
  }
  return Status::Ok();
}

Status DecodePod(std::string_view b, std::vector<Assignment>* out) {
  pb::Reader r(b);
  uint32_t f;
  pb::WireType wt;
  std::string name, ns;
  std::vector<std::string_view> containers;
  while (r.Next(&f, &wt)) {
    std::string_view v;
    if ((f == 1 || f == 2) && wt == pb::kLen) {
      if (!r.ReadLen(&v)) return Bad("pod");
      (f == 1 ? name : ns).assign(v);
    } else if (f == 3 && wt == pb::kLen) {
      if (!r.ReadLen(&v)) return Bad("containers");
      containers.push_back(v);
    } else if (!r.Skip(wt)) {
      return Bad("pod");
    }
  }
  if (!r.ok()) return Bad("pod");
  for (auto c : containers) {
    Status st = DecodeContainer(c, name, ns, out);
    if (!st.ok()) return st;
  }
  return Status::Ok();
}

}  // namespace

Status DecodeList(std::string_view bytes, std::vector<Assignment>* out) {
  pb::Reader r(bytes);
  uint32_t f;
  pb::WireType wt;
  while (r.Next(&f, &wt)) {
    if (f == 1 && wt == pb::kLen) {
      std::string_view v;
      if (!r.ReadLen(&v)) return Bad("pod_resources");
      Status st = DecodePod(v, out);
      if (!st.ok()) return st;
    } else if (!r.Skip(wt)) {
      return Bad("response");
    }
  }
  return r.ok() ? Status::Ok() : Bad("response");
}

Result<std::vector<Assignment>> List(const std::string& socket, int timeout_ms) {
  auto ch = grpc::Channel::Dial(socket, timeout_ms);
  if (!ch.ok()) return ch.status();
  std::string resp;
  Status st = (*ch)->Unary("/v1.PodResourcesLister/List", "", &resp, timeout_ms);
  if (!st.ok()) return st;
  std::vector<Assignment> out;
  st = DecodeList(resp, &out);
  if (!st.ok()) return st;
  return out;
}

Result<std::vector<Assignment>> CachedLister::Get() {
  std::lock_guard<std::mutex> lk(mu_);
  auto now = std::chrono::steady_clock::now();
  if (have_ && now - fetched_ < max_age_) return cached_;
  auto r = List(socket_, 1000);
  if (!r.ok()) return r.status();
  cached_ = std::move(*r);
  fetched_ = now;
  have_ = true;
  return cached_;
}

}  // namespace adp::podresources
