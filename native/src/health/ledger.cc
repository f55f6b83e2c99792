// Ledger: per-GPU health verdicts kept across monitor generations and (with
// --health-state-file) container restarts; event-gap marks and reset history
// (memory only); the operator's drain file.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "common/log.h"
#include "common/strings.h"
#include "health/health.h"

namespace adp::health {
namespace {
constexpr const char* kComp = "health";
// A node's verdicts take a few hundred bytes a GPU: anything past this is not
// a state file this daemon wrote, and is not read whole into memory.
constexpr size_t kMaxStateBytes = 1 << 20;

// The state file's text (at most kMaxStateBytes); false when it cannot be read
// (errno says why; ENOENT: there is none yet).
bool ReadState(const std::string& path, std::string* out) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return false;
  out->resize(kMaxStateBytes);
  in.read(out->data(), static_cast<std::streamsize>(kMaxStateBytes));
  out->resize(static_cast<size_t>(in.gcount()));
  if (out->size() == kMaxStateBytes && in.peek() != std::ifstream::traits_type::eof()) {
    LOG_WARN(kComp, "health state %s is larger than %zu bytes: only its start is read", path.c_str(),
             kMaxStateBytes);
    if (size_t nl = out->rfind('\n'); nl != std::string::npos) out->resize(nl + 1);  // whole lines only
  }
  return true;
}
}  // namespace

Ledger::Ledger(std::string path) : path_(std::move(path)) {
  if (path_.empty()) return;
  std::string body;
  if (!ReadState(path_, &body)) {
    if (errno != ENOENT)
      LOG_WARN(kComp, "cannot read health state %s: %s; starting empty", path_.c_str(), strerror(errno));
    return;
  }
  recs_ = Parse(body);
  size_t failed = 0;
  for (const auto& [_, r] : recs_) failed += r.fail != 0;
  LOG_INFO(kComp, "health state %s: %zu GPU record(s), %zu unhealthy", path_.c_str(), recs_.size(), failed);
}

void Ledger::Reload() {
  if (path_.empty()) return;
  std::string body;
  std::map<std::string, GpuRecord> next;
  if (ReadState(path_, &body)) {
    next = Parse(body);
  } else if (errno != ENOENT) {
    LOG_WARN(kComp, "cannot re-read health state %s: %s; keeping the current state", path_.c_str(), strerror(errno));
    return;
  }
  std::lock_guard<std::mutex> lk(mu_);
  for (const auto& [k, r] : recs_)
    if (r.fail && (!next.count(k) || !next[k].fail))
      LOG_INFO(kComp, "health state %s: GPU %s cleared by the operator (was: %s)", path_.c_str(), k.c_str(),
               r.reason.c_str());
  recs_ = std::move(next);
}

std::string Ledger::Serialize(const std::map<std::string, GpuRecord>& m) {
  std::string out = "adp-health v1\n";
  for (const auto& [k, r] : m) {
    std::string reason = r.reason;
    for (auto& c : reason)
      if (c == '\t' || c == '\n' || c == '\r') c = ' ';
    out += k + "\t" + (r.has_baseline ? std::to_string(r.ecc_baseline) : "-") + "\t" +
           std::to_string(r.ecc_seen) + "\t" + std::to_string(r.fail) + "\t" + reason;
    if (!r.resets.empty()) {
      out += "\tresets=";
      for (size_t i = 0; i < r.resets.size(); ++i) out += (i ? "," : "") + std::to_string(r.resets[i]);
    }
    if (!r.gap.empty()) {
      std::string gap = r.gap;
      for (auto& c : gap)
        if (c == '\t' || c == '\n' || c == '\r') c = ' ';
      out += "\tgap=" + gap;
    }
    if (!r.last_reset_event.empty() && r.last_reset_event.find_first_of("\t\n\r ") == std::string::npos)
      out += "\treset_event=" + r.last_reset_event;
    out += "\n";
  }
  return out;
}

std::map<std::string, GpuRecord> Ledger::Parse(const std::string& body) {
  std::map<std::string, GpuRecord> out;
  std::istringstream in(body);
  std::string line;
  bool header = false;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();  // CRLF (a file edited elsewhere)
    if (!header) {
      if (Trim(line) != "adp-health v1") {
        LOG_WARN(kComp, "health state: unknown format '%s'; ignored", line.c_str());
        return {};
      }
      header = true;
      continue;
    }
    if (Trim(line).empty()) continue;
    auto f = Split(line, '\t');
    if (f.size() < 4 || f[0].empty()) {
      LOG_WARN(kComp, "health state: malformed line '%s' skipped", line.c_str());
      continue;
    }
    GpuRecord r;
    auto seen = ParseUint(f[2]);
    auto fail = ParseUint(f[3]);
    if (f[1] != "-") {
      auto b = ParseUint(f[1]);
      if (!b) { LOG_WARN(kComp, "health state: malformed line '%s' skipped", line.c_str()); continue; }
      r.has_baseline = true;
      r.ecc_baseline = *b;
    }
    if (!seen || !fail) {
      LOG_WARN(kComp, "health state: malformed line '%s' skipped", line.c_str());
      continue;
    }
    r.ecc_seen = *seen;
    r.fail = static_cast<uint32_t>(*fail) &
             (kFailEcc | kFailUnresponsive | kFailResetPending | kFailEvent | kFailRetiredPages | kFailFlapping);
    if (f.size() > 4) r.reason = f[4];
    for (auto& c : r.reason)
      if (c == '\r') c = ' ';  // as Serialize writes it
    // Extension fields ("name=value"), each at most once; unknown ones ignored.
    for (size_t i = 5; i < f.size(); ++i) {
      if (f[i].rfind("resets=", 0) == 0 && r.resets.empty()) {
        for (const auto& t : Split(std::string_view(f[i]).substr(7), ',')) {
          auto v = ParseUint(t);
          if (!v) {
            LOG_WARN(kComp, "health state: reset history of %s malformed; ignored", f[0].c_str());
            r.resets.clear();
            break;
          }
          r.resets.push_back(static_cast<int64_t>(*v));
        }
        // A longer history (an older version kept every one): the newest count.
        std::sort(r.resets.begin(), r.resets.end());
        if (r.resets.size() > kMaxResetHistory) r.resets.erase(r.resets.begin(), r.resets.end() - kMaxResetHistory);
      } else if (f[i].rfind("reset_event=", 0) == 0 && r.last_reset_event.empty() && f[i].size() > 12) {
        r.last_reset_event = f[i].substr(12);
      } else if (f[i].rfind("gap=", 0) == 0 && r.gap.empty() && f[i].size() > 4) {
        r.gap = f[i].substr(4);
      }
    }
    out[f[0]] = std::move(r);
  }
  return out;
}

GpuRecord Ledger::Get(const std::string& key) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = recs_.find(key);
  return it == recs_.end() ? GpuRecord{} : it->second;
}

std::map<std::string, GpuRecord> Ledger::All() const {
  std::lock_guard<std::mutex> lk(mu_);
  return recs_;
}

void Ledger::Put(const std::string& key, const GpuRecord& r) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = recs_.find(key);
  if (it != recs_.end() && it->second.has_baseline == r.has_baseline && it->second.ecc_baseline == r.ecc_baseline &&
      it->second.ecc_seen == r.ecc_seen && it->second.fail == r.fail && it->second.reason == r.reason)
    return;
  // The reset history and the gap are the ledger's own (RecordReset,
  // MarkGap): a record read earlier does not roll them back.
  std::vector<int64_t> resets = it != recs_.end() ? std::move(it->second.resets) : std::vector<int64_t>{};
  std::string gap = it != recs_.end() ? std::move(it->second.gap) : std::string();
  std::string last_event = it != recs_.end() ? std::move(it->second.last_reset_event) : std::string();
  recs_[key] = r;
  recs_[key].resets = std::move(resets);
  recs_[key].gap = std::move(gap);
  recs_[key].last_reset_event = std::move(last_event);
  SaveLocked();
}

void Ledger::SaveLocked() const {
  if (path_.empty()) return;
  std::string body = Serialize(recs_);
  std::string tmp = path_ + ".tmp";
  FILE* f = fopen(tmp.c_str(), "w");
  bool ok = f && fwrite(body.data(), 1, body.size(), f) == body.size();
  if (f) ok = (fflush(f) == 0) && (fsync(fileno(f)) == 0) && ok;
  if (f) ok = (fclose(f) == 0) && ok;
  if (!ok || rename(tmp.c_str(), path_.c_str()) != 0) {
    LOG_WARN(kComp, "cannot write health state %s: %s", path_.c_str(), strerror(errno));
    unlink(tmp.c_str());
  }
}

bool Ledger::MarkGap(const std::string& key, const std::string& why, bool tentative, int64_t now_ms) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = gaps_.find(key);
  bool marked = false;
  if (it == gaps_.end()) {
    gaps_[key] = GapMark{now_ms, why, tentative, 0};
    marked = true;
  } else if (it->second.tentative && !tentative) {  // confirmed: the relay could not replay what was missed
    it->second.tentative = false;
    it->second.why = why;
    marked = true;
  }
  if (auto r = recs_.find(key); marked && !tentative && r != recs_.end()) {
    r->second.gap = why;  // a confirmed gap outlives this process (GpuRecord::gap)
    SaveLocked();
  }
  return marked;
}

std::vector<std::string> Ledger::CancelTentativeGaps() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> out;
  for (auto it = gaps_.begin(); it != gaps_.end();) {
    if (it->second.tentative) {
      out.push_back(it->first);
      it = gaps_.erase(it);
    } else {
      ++it;
    }
  }
  return out;
}

void Ledger::ClearGap(const std::string& key) {
  std::lock_guard<std::mutex> lk(mu_);
  gaps_.erase(key);
  if (auto it = recs_.find(key); it != recs_.end() && !it->second.gap.empty()) {
    it->second.gap.clear();
    SaveLocked();
  }
}

bool Ledger::Gap(const std::string& key, GapMark* out) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = gaps_.find(key);
  if (it == gaps_.end()) return false;
  if (out) *out = it->second;
  return true;
}

namespace {
// "<relay>:<seq>" -> (relay, seq); false when not that shape.
bool SplitEventId(const std::string& id, std::string* relay, uint64_t* seq) {
  size_t colon = id.rfind(':');
  if (colon == std::string::npos || colon == 0) return false;
  auto v = ParseUint(id.substr(colon + 1));
  if (!v) return false;
  *relay = id.substr(0, colon);
  *seq = *v;
  return true;
}
}  // namespace

int Ledger::RecordReset(const std::string& key, int64_t now_ms, int64_t window_ms, const std::string& event_id) {
  std::lock_guard<std::mutex> lk(mu_);
  GpuRecord& r = recs_[key];
  auto& v = r.resets;
  auto in_window = [&] {
    v.erase(std::remove_if(v.begin(), v.end(), [&](int64_t t) { return now_ms - t >= window_ms; }), v.end());
    return static_cast<int>(v.size());
  };
  std::string relay, last_relay;
  uint64_t seq = 0, last_seq = 0;
  if (SplitEventId(event_id, &relay, &seq) && SplitEventId(r.last_reset_event, &last_relay, &last_seq) &&
      relay == last_relay && seq <= last_seq) {
    LOG_INFO(kComp, "GPU %s: GPU_PRE_RESET #%llu replayed by the event relay was counted before; not counted again",
             key.c_str(), static_cast<unsigned long long>(seq));
    return in_window();
  }
  v.push_back(now_ms);
  if (v.size() > kMaxResetHistory) v.erase(v.begin(), v.end() - kMaxResetHistory);  // the newest
  if (!event_id.empty()) r.last_reset_event = event_id;
  const int n = in_window();
  SaveLocked();
  return n;
}

int64_t Ledger::LastReset(const std::string& key, int64_t now_ms) {
  std::lock_guard<std::mutex> lk(mu_);
  auto& v = recs_[key].resets;
  if (v.empty()) {
    v.push_back(now_ms);
    SaveLocked();
  }
  return *std::max_element(v.begin(), v.end());
}

void Ledger::ClearResets(const std::string& key) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = recs_.find(key);
  if (it == recs_.end() || it->second.resets.empty()) return;
  it->second.resets.clear();
  SaveLocked();
}

void Ledger::SetResponsiveSince(const std::string& key, int64_t ms) {
  std::lock_guard<std::mutex> lk(mu_);
  if (auto it = gaps_.find(key); it != gaps_.end()) it->second.responsive_since_ms = ms;
}

std::vector<std::pair<int, std::string>> Ledger::Failed(const inventory::Snapshot& snap) const {
  std::vector<std::pair<int, std::string>> out;
  std::lock_guard<std::mutex> lk(mu_);
  for (const auto& g : snap.gpus) {
    auto it = recs_.find(KeyOf(g));
    if (it != recs_.end() && it->second.fail) out.emplace_back(g.index, it->second.reason);
  }
  return out;
}

std::set<std::string> DrainTokens(std::string_view text) {
  std::set<std::string> names;
  for (size_t b = 0; b < text.size();) {
    size_t e = text.find('\n', b);
    if (e == std::string_view::npos) e = text.size();
    std::string line(text.substr(b, e - b));
    b = e + 1;
    if (size_t hash = line.find('#'); hash != std::string::npos) line.resize(hash);
    for (char& c : line)
      if (c == ',' || c == '\t' || c == '\r') c = ' ';
    for (size_t p = 0; p < line.size();) {
      size_t q = line.find(' ', p);
      if (q == std::string::npos) q = line.size();
      if (q > p) names.insert(line.substr(p, q - p));
      p = q + 1;
    }
  }
  return names;
}

std::string RemoveDrainNames(std::string_view line, const std::set<std::string>& names) {
  std::string_view body = line, comment;
  if (size_t hash = line.find('#'); hash != std::string_view::npos) {
    body = line.substr(0, hash);
    comment = line.substr(hash);
  }
  bool commas = body.find(',') != std::string_view::npos;
  std::vector<std::string> keep;
  bool removed = false;
  for (size_t p = 0; p < body.size();) {
    size_t q = body.find_first_of(" \t,\r", p);
    if (q == std::string_view::npos) q = body.size();
    if (q > p) {
      std::string tok(body.substr(p, q - p));
      if (names.count(tok)) removed = true;
      else keep.push_back(std::move(tok));
    }
    p = q + 1;
  }
  if (!removed) return std::string(line);
  if (keep.empty()) return "";
  std::string out;
  for (const auto& t : keep) out += (out.empty() ? "" : commas ? "," : " ") + t;
  if (!comment.empty()) out += "  " + std::string(comment);
  return out;
}

std::set<std::string> DrainNames(const inventory::PhysicalGpu& g) {
  std::set<std::string> n = {g.uuid, g.bdf, std::to_string(g.node_index)};
  if (size_t dot = g.bdf.rfind('.'); dot != std::string::npos) n.insert(g.bdf.substr(0, dot));
  // A partitioned GPU's compute partitions have PCI addresses of their own
  // (functions of the GPU's: 0000:0c:00.0 .. .7 on a CPX MI355X, as amd-smi
  // lists them): naming one names the GPU -- a drain holds the whole GPU, as a
  // reset does.
  for (const auto& p : g.partitions) {
    n.insert(p.uuid);
    n.insert(p.bdf);
  }
  n.erase("");
  return n;
}

}  // namespace adp::health
