// HealthCounters: what the health monitor has seen, for /metrics, /stats and
// the relay cursor that outlives monitor generations (and, persisted, the
// container).
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>

#include "common/log.h"
#include "common/strings.h"
#include "health/health.h"

namespace adp::health {
namespace {
constexpr const char* kComp = "health";

int64_t NowMs() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

void HealthCounters::SetRetiredPages(const std::string& bdf, uint32_t n) {
  std::lock_guard<std::mutex> lk(mu_);
  retired_[bdf] = n;
}

std::map<std::string, uint32_t> HealthCounters::RetiredPages() const {
  std::lock_guard<std::mutex> lk(mu_);
  return retired_;
}

void HealthCounters::SetVramUsed(const std::string& bdf, uint64_t bytes) {
  std::lock_guard<std::mutex> lk(mu_);
  vram_used_[bdf] = bytes;
}

void HealthCounters::MarkQueryOk(const std::string& bdf, const std::string& query) {
  std::lock_guard<std::mutex> lk(mu_);
  queries_ok_.insert({bdf, query});
}

bool HealthCounters::QueryEverOk(const std::string& bdf, const std::string& query) const {
  std::lock_guard<std::mutex> lk(mu_);
  return queries_ok_.count({bdf, query}) != 0;
}

bool HealthCounters::HasVramUsed(const std::string& bdf) const {
  std::lock_guard<std::mutex> lk(mu_);
  return vram_used_.count(bdf) != 0;
}

std::map<std::string, uint64_t> HealthCounters::VramUsed() const {
  std::lock_guard<std::mutex> lk(mu_);
  return vram_used_;
}

void HealthCounters::SetVramTotal(const std::string& bdf, uint64_t bytes) {
  std::lock_guard<std::mutex> lk(mu_);
  vram_total_[bdf] = bytes;
}

std::map<std::string, uint64_t> HealthCounters::VramTotal() const {
  std::lock_guard<std::mutex> lk(mu_);
  return vram_total_;
}

void HealthCounters::CountEvent(const std::string& bdf, const std::string& type) {
  std::lock_guard<std::mutex> lk(mu_);
  ++events_[{bdf, type}];
}

std::map<std::pair<std::string, std::string>, uint64_t> HealthCounters::EventCounts() const {
  std::lock_guard<std::mutex> lk(mu_);
  return events_;
}

void HealthCounters::CountUnmatched(const std::string& type) {
  std::lock_guard<std::mutex> lk(mu_);
  ++unmatched_[type];
}

std::map<std::string, uint64_t> HealthCounters::Unmatched() const {
  std::lock_guard<std::mutex> lk(mu_);
  return unmatched_;
}

void HealthCounters::CountRecovered(const std::string& bdf) {
  std::lock_guard<std::mutex> lk(mu_);
  ++recovered_[bdf];
}

std::map<std::string, uint64_t> HealthCounters::Recovered() const {
  std::lock_guard<std::mutex> lk(mu_);
  return recovered_;
}

HealthCounters::RelayCursor HealthCounters::GetRelayCursor() const {
  std::lock_guard<std::mutex> lk(mu_);
  return cursor_;
}

void HealthCounters::SetRelayCursor(const RelayCursor& c) {
  std::lock_guard<std::mutex> lk(mu_);
  cursor_ = c;
  cursor_dirty_ = true;
  SaveCursorLocked();
}

void HealthCounters::AdvanceRelaySeq(uint64_t seq) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!cursor_.valid || seq <= cursor_.seq) return;
  cursor_.seq = seq;
  cursor_dirty_ = true;
  if (clock_->SteadyMs() - cursor_saved_ms_ >= 1000) SaveCursorLocked();
}

void HealthCounters::PersistRelayCursor(const std::string& path) {
  std::lock_guard<std::mutex> lk(mu_);
  cursor_path_ = path;
  // Two short lines; at most 4 KiB of whatever is there is looked at.
  std::ifstream in(path, std::ios::binary);
  if (!in) return;
  std::string body(4096, '\0');
  in.read(body.data(), static_cast<std::streamsize>(body.size()));
  body.resize(static_cast<size_t>(in.gcount()));
  auto lines = Split(body, '\n');
  if (lines.size() < 2 || Trim(lines[0]) != "adp-relay-cursor v1") return;
  std::string line = lines[1];
  if (!line.empty() && line.back() == '\r') line.pop_back();
  auto f = Split(line, '\t');
  auto seq = f.size() == 3 ? ParseUint(f[1]) : std::nullopt;
  auto gen = f.size() == 3 ? ParseUint(f[2]) : std::nullopt;
  if (!seq || !gen || f[0].empty()) {
    LOG_WARN(kComp, "relay cursor %s: malformed; the relay will report a gap", path.c_str());
    return;
  }
  cursor_ = {true, f[0], *seq, *gen};
  LOG_INFO(kComp, "relay cursor %s: relay %s, event #%llu, generation %llu", path.c_str(), f[0].c_str(),
           static_cast<unsigned long long>(*seq), static_cast<unsigned long long>(*gen));
}

void HealthCounters::FlushRelayCursor() {
  std::lock_guard<std::mutex> lk(mu_);
  SaveCursorLocked();
}

void HealthCounters::SaveCursorLocked() {
  if (cursor_path_.empty() || !cursor_dirty_ || !cursor_.valid) return;
  cursor_saved_ms_ = clock_->SteadyMs();
  cursor_dirty_ = false;
  std::string body = "adp-relay-cursor v1\n" + cursor_.relay + "\t" + std::to_string(cursor_.seq) + "\t" +
                     std::to_string(cursor_.gen) + "\n";
  std::string tmp = cursor_path_ + ".tmp";
  FILE* f = fopen(tmp.c_str(), "w");
  bool ok = f && fwrite(body.data(), 1, body.size(), f) == body.size();
  if (f) ok = (fclose(f) == 0) && ok;
  if (!ok || rename(tmp.c_str(), cursor_path_.c_str()) != 0) {
    LOG_WARN(kComp, "cannot write relay cursor %s: %s", cursor_path_.c_str(), strerror(errno));
    unlink(tmp.c_str());
  }
}

std::string HealthCounters::Json() const {
  char buf[512];
  int e = events_enabled.load();
  uint64_t recovered = 0;
  for (const auto& [_, n] : Recovered()) recovered += n;
  snprintf(buf, sizeof(buf),
           "{\"events\": \"%s\", \"polls\": %llu, \"responsive\": %llu, \"ecc_reads_ok\": %llu, "
           "\"ecc_read_errors\": %llu, \"events_received\": %llu, \"retired_reads_ok\": %llu, "
           "\"retired_read_errors\": %llu, \"event_gaps\": %llu, \"recovered_without_event\": %llu}",
           e < 0 ? "not started" : e ? "on" : "off", static_cast<unsigned long long>(polls.load()),
           static_cast<unsigned long long>(responsive.load()), static_cast<unsigned long long>(ecc_reads_ok.load()),
           static_cast<unsigned long long>(ecc_read_errors.load()),
           static_cast<unsigned long long>(events_received.load()),
           static_cast<unsigned long long>(retired_reads_ok.load()),
           static_cast<unsigned long long>(retired_read_errors.load()),
           static_cast<unsigned long long>(event_gaps.load()), static_cast<unsigned long long>(recovered));
  return buf;
}

int64_t HealthCounters::HealthLoopAgeMs() const {
  int64_t beat = loop_beat_ms.load();
  return beat == 0 ? 0 : std::max<int64_t>(0, NowMs() - beat);
}

}  // namespace adp::health
