// Coverage-guided fuzzing (libFuzzer) of the event-relay wire lines
// (health/relay_protocol.cc): the daemon parses whatever arrives on its relay socket,
// and the privileged relay parses the daemon's request lines (a scan's
// directory is only accepted absolute and without "..").
// Checks: no crash; an accepted event line re-formatted from its fields parses
// back to the same fields (message newlines folded to spaces); a hello's
// verdict is exactly "events=ok" present before its reason; an accepted scan reply (the relay's
// answer to "scan", memcap/driver_usage.h) re-serialises to the bytes it was
// parsed from, and its sums match its rows.
#include <fuzzer/FuzzedDataProvider.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "common/log.h"
#include "health/relay.h"
#include "memcap/driver_usage.h"

using namespace adp;

namespace {
[[noreturn]] void Fail(const char* what) {
  fprintf(stderr, "invariant violated: %s\n", what);
  abort();
}
}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  static bool quiet = (SetLogLevel(LogLevel::kError), true);
  (void)quiet;
  std::string line(reinterpret_cast<const char*>(data), size);
  health::RelayLine r = health::ParseRelayLine(line);
  if (r.kind == "event") {
    if (r.bdf.find(' ') != std::string::npos) Fail("bdf with a space");
    smi::ProcessorInfo p;
    p.kfd_node = r.node;
    p.bdf = r.bdf == "-" ? "" : r.bdf;
    p.partition_id = r.part;
    health::RelayLine back = health::ParseRelayLine(health::FormatRelayEvent(p, r.type, r.message));
    std::string folded = r.message;
    for (char& c : folded)
      if (c == '\n' || c == '\r') c = ' ';
    while (!folded.empty() && (folded.back() == '\n' || folded.back() == '\r' || folded.back() == ' ')) folded.pop_back();
    std::string got = back.message;
    while (!got.empty() && got.back() == ' ') got.pop_back();
    if (back.kind != "event" || back.node != r.node || back.part != r.part || back.type != r.type) Fail("round trip");
    if (!r.bdf.empty() && r.bdf != "-" && back.bdf != r.bdf) Fail("bdf round trip");
    if (got != folded) Fail("message round trip");
  } else if (r.kind == "hello") {
    // ok iff the first "events=" token before the free-text reason is exactly "events=ok"
    std::string first;
    std::string body = line;
    while (!body.empty() && (body.back() == '\n' || body.back() == '\r')) body.pop_back();
    if (size_t at = body.find(" reason="); at != std::string::npos) body.resize(at);
    if (r.gap < -1 || r.gap > 1) Fail("gap");
    for (size_t b = 0; b <= body.size() && first.empty();) {
      size_t e = body.find(' ', b);
      if (e == std::string::npos) e = body.size();
      std::string tok = body.substr(b, e - b);
      if (tok.size() >= 7 && tok.compare(0, 7, "events=") == 0) first = tok;
      b = e + 1;
    }
    if (r.events_ok != (first == "events=ok")) Fail("hello verdict");
  } else if (!r.kind.empty()) {
    Fail("unknown kind");
  }
  // The privileged side: the relay's reading of a daemon's request line.
  health::RelayRequest q = health::ParseRelayRequest(line);
  if (q.kind == "reinit") {
    if (!q.fp.empty() && q.fp.size() != 16) Fail("fingerprint shape");
    if (q.has_since && (q.since_relay.empty() || q.since_relay.size() > 32)) Fail("cursor shape");
    if (!q.usage_dir.empty() || q.malformed) Fail("reinit with scan fields");
  } else if (q.kind == "scan") {
    if (!q.malformed && (q.usage_dir.empty() || q.usage_dir[0] != '/' ||
                         q.usage_dir.find("/..") != std::string::npos || q.usage_dir.find('\t') != std::string::npos))
      Fail("scan directory accepted");
  } else if (!q.kind.empty()) {
    Fail("unknown request kind");
  }
  memcap::DriverScan s;
  size_t used = 0;
  if (memcap::ParseScan(line, &s, &used)) {
    if (used > line.size()) Fail("scan consumed past the input");
    // (a previous-version header without the render-only field reads as 0)
    std::string expect = line.substr(0, used);
    size_t nl = expect.find('\n');
    if (std::count(expect.begin(), expect.begin() + nl, '\t') == 5) expect.insert(nl, "\t0");
    if (memcap::SerializeScan(s) != expect) Fail("scan round trip");
    uint64_t sum = 0, total = 0;
    for (const auto& p : s.procs) sum += p.bytes;
    for (const auto& [bdf, b] : s.total) total += b;
    if (sum != total) Fail("scan totals");
  }
  return 0;
}
