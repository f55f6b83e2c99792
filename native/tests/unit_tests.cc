// Native unit tests (no GPU, no kubelet). Run: build/native/adp_unit_tests
// Pins the reference's test vectors:
//   cmd/nvidia-device-plugin/replica_test.go:37-96   (15 prioritizeDevices cases)
//   cmd/nvidia-device-plugin/replica_test.go:120-122 (3 stripReplicas cases)
//   cmd/nvidia-device-plugin/nvidia_test.go:31-64    (10 getAdditionalXids cases)
// plus codec, config, resource-config, topology and gRPC loopback tests.
#include <fcntl.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdio>
#include <functional>
#include <climits>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include <json.hpp>

#include "alloc/replicas.h"
#include "alloc/topology.h"
#include "common/log.h"
#include "common/strings.h"
#include "daemon/config.h"
#include "daemon/yaml.h"
#include "grpc/grpc.h"
#include "grpc/server_conn.h"
#include "health/health.h"
#include "health/relay.h"
#include "memcap/driver_usage.h"
#include "memcap/usage.h"
#include "metrics/metrics.h"
#include "plugin/plugin.h"
#include "podresources/podresources.h"
#include "proto/wire.h"
#include "proto/messages.h"
#include "strategy/strategy.h"

using namespace adp;
using V = std::vector<std::string>;

static int g_failed = 0, g_checks = 0;
static std::string g_case;

#define CHECK(cond)                                                                \
  do {                                                                             \
    ++g_checks;                                                                    \
    if (!(cond)) {                                                                 \
      ++g_failed;                                                                  \
      fprintf(stderr, "FAIL [%s] %s:%d: %s\n", g_case.c_str(), __FILE__, __LINE__, #cond); \
    }                                                                              \
  } while (0)

static std::string Str(const V& v) { return "[" + Join(v, ",") + "]"; }

static void TestPrioritize() {
  struct Case {
    const char* name;
    V avail, must;
    int size;
    bool ok;
    V want;
    bool non_unique;
    std::string err;
  };
  const std::string missing = "in mustIncludeDeviceIDs is missing from availableDeviceIDs";
  std::vector<Case> cases = {
      {"Basic", {"a-replica-0", "a-replica-1", "b-replica-1"}, {}, 1, true, {"a-replica-0"}, false, ""},
      {"Multiple Unique", {"a-replica-0", "a-replica-1", "b-replica-1"}, {}, 2, true, {"a-replica-0", "b-replica-1"}, false, ""},
      {"NonuniqueError", {"a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"}, {}, 3, true,
       {"a-replica-0", "a-replica-1", "b-replica-1"}, true, ""},
      {"Must Include Greater Utilized", {"a-replica-0", "a-replica-1", "b-replica-1"}, {"b-replica-1"}, 1, true, {"b-replica-1"}, false, ""},
      {"Must Include Least Utilized", {"a-replica-0", "a-replica-1", "b-replica-1"}, {"a-replica-1"}, 1, true, {"a-replica-1"}, false, ""},
      {"Must Include Two", {"a-replica-0", "a-replica-1", "b-replica-1"}, {"a-replica-1"}, 2, true, {"a-replica-1", "b-replica-1"}, false, ""},
      {"NonuniqueError Must Include", {"a-replica-0", "a-replica-1", "a-replica-2", "b-replica-2", "b-replica-1"}, {"a-replica-2"}, 3, true,
       {"a-replica-0", "a-replica-2", "b-replica-1"}, true, ""},
      {"Must Include", {"a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1", "c-replica-0"}, {"a-replica-2"}, 3, true,
       {"a-replica-2", "b-replica-1", "c-replica-0"}, false, ""},
      {"Must Include Entire Allocated", {"a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"},
       {"a-replica-2", "b-replica-1", "a-replica-1"}, 3, true, {"a-replica-1", "a-replica-2", "b-replica-1"}, true, ""},
      {"Deterministic", {"a-replica-1", "b-replica-1", "c-replica-1", "d-replica-1", "e-replica-1", "f-replica-1", "g-replica-1", "h-replica-1"},
       {}, 1, true, {"a-replica-1"}, false, ""},
      {"OversizedRequest", {"a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"}, {}, 5, false, {}, false, "no devices left to allocate"},
      {"Undersized", {"a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"}, {}, 0, true, {}, false, ""},
      {"NoneAvailable", {}, {}, 1, false, {}, false, "no devices left to allocate"},
      {"SubsetSame", {"a-replica-0", "a-replica-1"}, {"a-replica-2"}, 1, false, {}, false, "device 'a-replica-2' " + missing},
      {"SubsetDifferent", {"a-replica-0", "a-replica-1"}, {"b-replica-2"}, 1, false, {}, false, "device 'b-replica-2' " + missing},
  };
  for (const auto& c : cases) {
    g_case = std::string("prioritize/") + c.name;
    auto r = alloc::PrioritizeDevices(c.avail, c.must, c.size);
    CHECK(r.ok() == c.ok);
    if (c.ok && r.ok()) {
      if (r->ids != c.want) fprintf(stderr, "  got %s want %s\n", Str(r->ids).c_str(), Str(c.want).c_str());
      CHECK(r->ids == c.want);
      CHECK(r->non_unique == c.non_unique);
    }
    if (!c.ok && !r.ok()) CHECK(r.status().message() == c.err);
  }
  g_case = "prioritize/B12-must-exceeds-size";
  CHECK(!alloc::PrioritizeDevices({"a-replica-0", "b-replica-0"}, {"a-replica-0", "b-replica-0"}, 1).ok());

  g_case = "prioritize/pack";
  auto p = alloc::PrioritizeDevices({"a-replica-0", "a-replica-1", "a-replica-2", "b-replica-0", "b-replica-1",
                                     "c-replica-0", "c-replica-1", "c-replica-2", "c-replica-3"},
                                    {}, 2, alloc::ReplicaPolicy::kPack);
  CHECK(p.ok());
  if (p.ok()) CHECK(p->ids == V({"b-replica-0", "b-replica-1"}));  // best fit: tightest GPU
  auto p2 = alloc::PrioritizeDevices({"a-replica-0", "a-replica-1", "b-replica-0", "b-replica-1", "b-replica-2"},
                                     {"a-replica-1"}, 3, alloc::ReplicaPolicy::kPack);
  CHECK(p2.ok());
  if (p2.ok()) CHECK(p2->ids == V({"a-replica-0", "a-replica-1", "b-replica-0"}));
}

static void TestStrip() {
  g_case = "strip";
  CHECK(alloc::StripReplicas({"b-replica-5", "a-replica-1", "a-replica-0"}) == V({"a", "b"}));
  CHECK(alloc::StripReplicas({"b-replica-0", "a-replica-1", "a-replica-2", "c-replica-2"}) == V({"a", "b", "c"}));
  CHECK(alloc::StripReplicas({}).empty());
  CHECK(alloc::StripReplica("plain-uuid") == "plain-uuid");
  CHECK(alloc::ReplicaId("u", 7) == "u-replica-7");
}

static void TestAdditionalIds() {
  g_case = "additional-ids";
  using U = std::vector<uint64_t>;
  CHECK(health::ParseAdditionalIds("") == U{});
  CHECK(health::ParseAdditionalIds(",") == U{});
  CHECK(health::ParseAdditionalIds("not-an-int") == U{});
  CHECK(health::ParseAdditionalIds("68") == U{68});
  CHECK(health::ParseAdditionalIds("-68") == U{});
  CHECK(health::ParseAdditionalIds("68  ") == U{68});
  CHECK(health::ParseAdditionalIds("68,") == U{68});
  CHECK(health::ParseAdditionalIds(",68") == U{68});
  CHECK(health::ParseAdditionalIds("68,67") == (U{68, 67}));
  CHECK(health::ParseAdditionalIds("68,not-an-int,67") == (U{68, 67}));

  g_case = "health-config";
  auto c = health::HealthConfig::FromValues("all", nullptr);
  CHECK(c.disabled);
  c = health::HealthConfig::FromValues("XIDS", nullptr);
  CHECK(c.disabled);
  c = health::HealthConfig::FromValues("3", "0");
  CHECK(!c.disabled && c.ignored.count(3) && c.poll_interval_ms == 0);
  CHECK(health::Monitor::Classify(c, 3) == 0);
  c = health::HealthConfig::FromValues("", nullptr);
  CHECK(health::Monitor::Classify(c, 3) == -1);
  CHECK(health::Monitor::Classify(c, 4) == +1);
  CHECK(health::Monitor::Classify(c, 1) == 0);
}

static void TestResourceConfig() {
  g_case = "resource-config";
  auto rc = strategy::ResourceConfig::Parse("gpu:sharedgpu:4, cpx-1xcd.36gb:small:2,,");
  CHECK(rc.ok());
  if (rc.ok()) {
    CHECK(rc->Get("gpu").name == "sharedgpu" && rc->Get("gpu").replicas == 4);
    CHECK(rc->Get("cpx-1xcd.36gb").name == "small");
    CHECK(rc->Get("other").name == "other" && rc->Get("other").replicas == 1);  // B2 fixed
  }
  auto a = strategy::ResourceConfig::Parse("gpu:gpu-mem-gb:-1");
  CHECK(a.ok() && a->Get("gpu").auto_replicas && a->Get("gpu").replicas == 1);
  CHECK(!strategy::ResourceConfig::Parse("gpu:x").ok());
  CHECK(strategy::ResourceConfig::Parse("gpu:x").status().message().find("colon") != std::string::npos);
  CHECK(!strategy::ResourceConfig::Parse("gpu:x:-2").ok());  // B11
  CHECK(!strategy::ResourceConfig::Parse("gpu:x:0").ok());
  CHECK(!strategy::ResourceConfig::Parse("gpu:x:abc").ok());
  CHECK(!strategy::ResourceConfig::Parse("gpu:bad name:2").ok());
  CHECK(strategy::ResourceConfig::Parse("").ok());
  // optional 4th field: this resource's replica policy
  auto p = strategy::ResourceConfig::Parse("gpu:sharedgpu:4:pack,cpx-1xcd.36gb:s:2");
  CHECK(p.ok() && p->Get("gpu").policy == alloc::ReplicaPolicy::kPack);
  CHECK(p.ok() && p->Get("cpx-1xcd.36gb").policy == alloc::ReplicaPolicy::kAuto);
  CHECK(p.ok() && p->ToJson().find("\"Policy\": \"pack\"") != std::string::npos);
  CHECK(!strategy::ResourceConfig::Parse("gpu:x:2:tight").ok());
  CHECK(!strategy::ResourceConfig::Parse("gpu:x:2:pack:extra").ok());
  alloc::ReplicaPolicy pol;
  CHECK(alloc::ParseReplicaPolicy("auto", &pol) && pol == alloc::ReplicaPolicy::kAuto);
  CHECK(std::string(alloc::ReplicaPolicyName(alloc::ReplicaPolicy::kAuto)) == "auto");
}

// Round-5 advice: the reset history is capped at the newest 64 (recording and
// parsing), and a relayed GPU_PRE_RESET replayed after a restart is not
// counted twice (keyed by "<relay>:<seq>").
static void TestLedgerResetHistory() {
  g_case = "ledger-reset-history";
  health::Ledger l;
  CHECK(l.RecordReset("g", 1000, 10000, "aa:5") == 1);
  CHECK(l.RecordReset("g", 1100, 10000, "aa:5") == 1);  // the same event, replayed
  CHECK(l.RecordReset("g", 1200, 10000, "aa:4") == 1);  // an older one of that relay: replayed too
  CHECK(l.RecordReset("g", 1300, 10000, "bb:1") == 2);  // another relay instance: a new reset
  CHECK(l.RecordReset("g", 1400, 10000, "") == 3);      // in-process: no identity, always new
  CHECK(l.Get("g").last_reset_event == "bb:1");
  for (int i = 0; i < 100; ++i) l.RecordReset("h", 5000 + i, 1000000);
  auto h = l.Get("h").resets;
  CHECK(h.size() == health::Ledger::kMaxResetHistory);
  CHECK(!h.empty() && h.front() == 5000 + 100 - 64 && h.back() == 5099);  // the newest kept
  // A file from an older version with 100 entries: the newest 64, not none.
  std::string body = "adp-health v1\nk\t0\t0\t4\tflapping\tresets=";
  for (int i = 0; i < 100; ++i) body += (i ? "," : "") + std::to_string(7000 + i);
  body += "\treset_event=cc:9\n";
  auto m = health::Ledger::Parse(body);
  CHECK(m.count("k") && m["k"].resets.size() == 64 && m["k"].resets.front() == 7036 && m["k"].resets.back() == 7099);
  CHECK(m["k"].last_reset_event == "cc:9");
  auto back = health::Ledger::Parse(health::Ledger::Serialize(m));
  CHECK(back["k"].resets == m["k"].resets && back["k"].last_reset_event == "cc:9");
}

static void TestLedgerGaps() {
  g_case = "ledger-gaps";
  health::Ledger l;
  health::GapMark m;
  CHECK(!l.Gap("a", &m));
  CHECK(l.MarkGap("a", "relay dropped", true, 100));     // new: worth a log line
  CHECK(!l.MarkGap("a", "relay dropped", true, 200));    // again: not
  CHECK(l.Gap("a", &m) && m.tentative && m.since_ms == 100);
  CHECK(l.MarkGap("a", "relay renewed", false, 300));    // confirmed: logged, keeps its start
  CHECK(l.Gap("a", &m) && !m.tentative && m.since_ms == 100 && m.why == "relay renewed");
  CHECK(!l.MarkGap("a", "other", true, 400));            // a confirmed mark never goes back to tentative
  CHECK(l.MarkGap("b", "relay dropped", true, 500));
  l.SetResponsiveSince("b", 600);
  CHECK(l.Gap("b", &m) && m.responsive_since_ms == 600);
  auto cancelled = l.CancelTentativeGaps();              // the relay replayed what b missed
  CHECK(cancelled.size() == 1 && cancelled[0] == "b" && !l.Gap("b", nullptr) && l.Gap("a", nullptr));
  l.ClearGap("a");
  CHECK(!l.Gap("a", nullptr));
  // a confirmed gap is part of the state file (a tentative one is not)
  health::GpuRecord r;
  r.fail = health::kFailResetPending;
  l.Put("c", r);
  l.MarkGap("c", "x", false, 1);
  CHECK(health::Ledger::Serialize(l.All()) == "adp-health v1\nc\t-\t0\t4\t\tgap=x\n");
  l.ClearGap("c");
  CHECK(health::Ledger::Serialize(l.All()) == "adp-health v1\nc\t-\t0\t4\t\n");
  // reset history for flap damping: a sliding window
  CHECK(l.RecordReset("d", 1000, 500) == 1);
  CHECK(l.RecordReset("d", 1200, 500) == 2);
  CHECK(l.RecordReset("d", 1600, 500) == 2);  // 1000 fell out of the window
  CHECK(l.LastReset("d", 9999) == 1600);
  CHECK(l.LastReset("e", 5000) == 5000);      // none known: now (a loaded quarantine lasts a window)
  // the flapping bit survives the state file; drained never does (the drain file is its source)
  auto parsed = health::Ledger::Parse("adp-health v1\nf\t-\t0\t96\tx\n");
  CHECK(parsed["f"].fail == health::kFailFlapping);
  // the reset history is written with the verdicts and read back; a record
  // Put() from an earlier Get() does not roll it back
  health::GpuRecord before = l.Get("d");
  l.Put("d", before);
  CHECK(l.Get("d").resets == std::vector<int64_t>({1200, 1600}));
  std::string body = health::Ledger::Serialize(l.All());
  CHECK(body.find("\nd\t-\t0\t0\t\tresets=1200,1600\n") != std::string::npos);
  auto back = health::Ledger::Parse(body);
  CHECK(back["d"].resets == std::vector<int64_t>({1200, 1600}) && back["c"].resets.empty());
  // CRLF line endings (a file edited on another system) read as LF
  auto crlf = health::Ledger::Parse("adp-health v1\r\nh\t-\t0\t4\twhy\tresets=5,6\r\n");
  CHECK(crlf["h"].fail == 4 && crlf["h"].reason == "why" && crlf["h"].resets == std::vector<int64_t>({5, 6}));
  {
    // a state file far larger than any node's: its start is read, no more
    char tmpl[] = "/tmp/adp-ledger-XXXXXX";
    int fd = mkstemp(tmpl);
    std::string big = "adp-health v1\nbig\t-\t0\t4\tr\n" + std::string(3u << 20, '#') + "\ntail\t-\t0\t4\tr\n";
    CHECK(fd >= 0 && write(fd, big.data(), big.size()) == static_cast<ssize_t>(big.size()));
    close(fd);
    health::Ledger lb(tmpl);
    CHECK(lb.Get("big").fail == 4 && lb.All().count("tail") == 0);
    unlink(tmpl);
  }
  {
    // the relay cursor file: read back (CRLF too); malformed = no cursor (the relay reports a gap)
    char tmpl[] = "/tmp/adp-cursor-XXXXXX";
    int fd = mkstemp(tmpl);
    close(fd);
    auto cursor_from = [&](const std::string& text) {
      FILE* f = fopen(tmpl, "w");
      fputs(text.c_str(), f);
      fclose(f);
      health::HealthCounters hc;
      hc.PersistRelayCursor(tmpl);
      return hc.GetRelayCursor();
    };
    auto c1 = cursor_from("adp-relay-cursor v1\nab12\t7\t3\n");
    CHECK(c1.valid && c1.relay == "ab12" && c1.seq == 7 && c1.gen == 3);
    CHECK(cursor_from("adp-relay-cursor v1\r\nab12\t7\t3\r\n").valid);
    CHECK(!cursor_from("adp-relay-cursor v1\nab12\t7\n").valid);
    CHECK(!cursor_from("something else\nab12\t7\t3\n").valid);
    CHECK(!cursor_from("adp-relay-cursor v1\n" + std::string(10000, 'x') + "\t1\t1\n").valid);
    unlink(tmpl);
  }
  {
    // a confirmed gap is written with the verdict (a tentative one is not),
    // survives Put() of an earlier record, and goes with ClearGap
    health::Ledger lg;
    health::GpuRecord rp;
    rp.fail = health::kFailResetPending;
    lg.Put("p", rp);
    lg.MarkGap("p", "the relay restarted", true, 5);
    CHECK(lg.Get("p").gap.empty());
    lg.MarkGap("p", "the relay restarted", false, 6);  // confirmed
    CHECK(lg.Get("p").gap == "the relay restarted");
    lg.Put("p", rp);
    std::string persisted = health::Ledger::Serialize(lg.All());
    CHECK(persisted.find("\tgap=the relay restarted\n") != std::string::npos);
    CHECK(health::Ledger::Parse(persisted)["p"].gap == "the relay restarted");
    CHECK(health::Ledger::Parse("adp-health v1\nq\t-\t0\t4\tr\tgap=x\tresets=1,2\n")["q"].resets.size() == 2);
    CHECK(health::Ledger::Parse("adp-health v1\nq\t-\t0\t4\tr\tgap=x\tresets=1,2\n")["q"].gap == "x");
    lg.ClearGap("p");
    CHECK(lg.Get("p").gap.empty() && !lg.Gap("p", nullptr));
  }
  CHECK(health::DescribeFailures(health::kFailDrained) == "drained by the operator");
  CHECK(health::DescribeFailures(health::kFailEcc | health::kFailResetPending) ==
        "waiting for GPU_POST_RESET, uncorrectable ECC errors");
  CHECK(health::DescribeFailures(0).empty());
  l.ClearResets("d");  // --return-to-service
  CHECK(l.Get("d").resets.empty() && l.RecordReset("d", 1700, 500) == 1);
  // an older file (no field) and a malformed field: no history, the line kept
  CHECK(health::Ledger::Parse("adp-health v1\ng\t-\t0\t64\tx\tresets=1,y\n")["g"].fail == health::kFailFlapping);
  CHECK(health::Ledger::Parse("adp-health v1\ng\t-\t0\t64\tx\tresets=1,y\n")["g"].resets.empty());
  CHECK(health::Ledger::Parse("adp-health v1\ng\t-\t0\t64\tx\tfuture=1\n")["g"].resets.empty());
}

static void TestRemoveDrainNames() {
  g_case = "remove-drain-names";
  std::set<std::string> g0 = {"0000:0c:00.0", "0000:0c:00", "0", "GPU-a"};
  CHECK(health::RemoveDrainNames("0000:0c:00.0  # GPU-a", g0).empty());  // our own line goes
  CHECK(health::RemoveDrainNames("0,1 # maintenance", g0) == "1  # maintenance");
  CHECK(health::RemoveDrainNames("GPU-a GPU-b\tGPU-c", g0) == "GPU-b GPU-c");
  CHECK(health::RemoveDrainNames("# 0 is mentioned only in a comment", g0) == "# 0 is mentioned only in a comment");
  CHECK(health::RemoveDrainNames("1,2", g0) == "1,2");  // untouched: byte for byte
  CHECK(health::RemoveDrainNames("0000:0c:00,0000:0c:00.0", g0).empty());
}

static void TestRelayLines() {
  g_case = "relay-lines";
  smi::ProcessorInfo p;
  p.kfd_node = 10;
  p.bdf = "0000:0c:00.1";
  p.partition_id = 1;
  std::string line = health::FormatRelayEvent(p, 3, "mode1 reset\nsecond line");
  CHECK(line == "event node=10 bdf=0000:0c:00.1 part=1 type=3 mode1 reset second line\n");
  auto r = health::ParseRelayLine(line);
  CHECK(r.kind == "event" && r.node == 10 && r.bdf == "0000:0c:00.1" && r.part == 1 && r.type == 3);
  CHECK(r.message == "mode1 reset second line");
  p.kfd_node = 0xffffffffu;
  r = health::ParseRelayLine(health::FormatRelayEvent(p, 4, ""));
  CHECK(r.kind == "event" && r.node == 0xffffffffu && r.type == 4 && r.message.empty());
  r = health::ParseRelayLine("hello v1 events=ok processors=8");
  CHECK(r.kind == "hello" && r.events_ok && !r.after_reinit);
  r = health::ParseRelayLine("hello v1 reinit events=ok processors=8");
  CHECK(r.kind == "hello" && r.events_ok && r.after_reinit);
  r = health::ParseRelayLine("hello v1 events=off reason=NO_PERM: denied");
  CHECK(r.kind == "hello" && !r.events_ok && r.reason == "NO_PERM: denied");
  for (const char* bad : {"", "event", "event node=x bdf=a part=0 type=3", "event node=1 bdf=a part=0",
                          "event node=1 bdf=a part=-1 type=3", "event node=4294967295 bdf=a part=0 type=3",
                          "bogus line", "event node=1 bdf=a part=0 type=99999999999",
                          "event seq=x node=1 bdf=a part=0 type=3"})
    CHECK(health::ParseRelayLine(bad).kind.empty());
  // sequence numbers, the relay's cursor fields and gap
  r = health::ParseRelayLine("event seq=42 node=10 bdf=0000:0c:00.1 part=1 type=4 reset done");
  CHECK(r.kind == "event" && r.seq == 42 && r.node == 10 && r.type == 4 && r.message == "reset done");
  r = health::ParseRelayLine("hello v1 reinit events=ok processors=8 relay=00ff00ff00ff00ff gen=3 seq=17 gap=0");
  CHECK(r.kind == "hello" && r.after_reinit && r.events_ok && r.relay == "00ff00ff00ff00ff" && r.gen == 3 &&
        r.seq == 17 && r.gap == 0);
  // keys inside the reason are not the hello's
  r = health::ParseRelayLine("hello v1 reinit events=off relay=ab gen=2 seq=5 gap=1 reason=x gap=0 events=ok");
  CHECK(!r.events_ok && r.gap == 1 && r.reason == "x gap=0 events=ok" && r.seq == 5);
  r = health::ParseRelayLine("hello v1 events=ok processors=8");  // an older relay: no gap said
  CHECK(r.gap == -1 && r.relay.empty());

  // the relay's reading of a daemon's requests
  auto rq = health::ParseRelayRequest("reinit fp=0123456789abcdef since=00ff00ff00ff00ff:17:3\n");
  CHECK(rq.kind == "reinit" && rq.fp == "0123456789abcdef" && rq.has_since && rq.since_relay == "00ff00ff00ff00ff" &&
        rq.since_seq == 17 && rq.since_gen == 3);
  rq = health::ParseRelayRequest("reinit");
  CHECK(rq.kind == "reinit" && rq.fp.empty() && !rq.has_since);
  rq = health::ParseRelayRequest("reinit fp=XYZ since=-");
  CHECK(rq.kind == "reinit" && rq.fp.empty() && !rq.has_since);
  rq = health::ParseRelayRequest("reinit since=zz:1:2");  // not a relay ID
  CHECK(!rq.has_since);
  rq = health::ParseRelayRequest("reinitx");
  CHECK(rq.kind.empty());
  rq = health::ParseRelayRequest("scan\t/var/lib/kubelet/device-plugins/amdgpu-dp/usage\t0::/kubepods/x");
  CHECK(rq.kind == "scan" && !rq.malformed && rq.usage_dir == "/var/lib/kubelet/device-plugins/amdgpu-dp/usage" &&
        rq.cgroup == "0::/kubepods/x");
  for (const char* bad : {"scan\trelative\tx", "scan\t/a/../etc\tx", "scan\tnotab", "scan\t\tx"})
    CHECK(health::ParseRelayRequest(bad).kind == "scan" && health::ParseRelayRequest(bad).malformed);

  // processor fingerprints: order-independent, sensitive to every field
  smi::ProcessorInfo q = p;
  q.bdf = "0000:0d:00.0";
  q.kfd_node = 11;
  std::string fp = health::ProcessorFingerprint({p, q});
  CHECK(fp.size() == 16 && fp == health::ProcessorFingerprint({q, p}));
  CHECK(fp != health::ProcessorFingerprint({p}));
  smi::ProcessorInfo q2 = q;
  q2.compute_partition = "CPX";
  CHECK(fp != health::ProcessorFingerprint({p, q2}));
  q2 = q;
  q2.kfd_node = 12;
  CHECK(fp != health::ProcessorFingerprint({p, q2}));
  q2 = q;
  q2.partition_id = 2;
  CHECK(fp != health::ProcessorFingerprint({p, q2}));

  // the relay's scan reply
  memcap::DriverScan scan;
  scan.pid_source = "kfd";
  scan.pids_scanned = 3;
  scan.fd_entries = 7;
  scan.procs = {{11, "0000:0c:00.0", 3u << 20, "0::/pod/a", "k1", false},
                {12, "0000:0c:00.0", 5u << 20, "0::/pod/a\tx", "k1", true},
                {13, "0000:0d:00.0", 1u << 20, "0::/", "", false}};
  memcap::Aggregate(&scan);
  std::string text = memcap::SerializeScan(scan);
  memcap::DriverScan back;
  size_t used = 0;
  CHECK(memcap::ParseScan(text + "trailing", &back, &used) && used == text.size());
  CHECK(back.pid_source == "kfd" && back.pids_scanned == 3 && back.fd_entries == 7 && back.procs.size() == 3);
  CHECK(back.procs[1].cgroup == "0::/pod/a x" && back.procs[1].via_cgroup && back.procs[1].pid == 12);
  CHECK((back.by_grant[{"k1", "0000:0c:00.0"}] == 8u << 20) && back.unattributed["0000:0d:00.0"] == 1u << 20);
  CHECK((back.grant_procs[{"k1", "0000:0c:00.0"}] == 2));
  CHECK(!memcap::ParseScan(text.substr(0, text.size() - 1), &back, &used));  // incomplete
  for (const char* bad : {"scan\tproc\t1\t1\t0\t1\np\tx\tb\t1\tk\t0\tc\n",
                          "scan\tproc\t1\t1\t0\n", "scan\tproc\t1\t1\t0\t1\np\t1\tb\t1\tk\t2\tc\n",
                          "scan\tproc\t1\t1\t0\t99999999999999999999999\n"})
    CHECK(!memcap::ParseScan(bad, &back, &used));

  // incomplete vs malformed: a prefix of a reply waits, anything else fails at once
  using PR = memcap::ParseResult;
  for (std::string part : {std::string(""), std::string("sc"), std::string("scan\t"), std::string("scan\tproc\t1"),
                           text.substr(0, text.size() - 1), text.substr(0, text.find('\n') + 2)})
    CHECK(memcap::ParseScanReply(part, &back, &used) == PR::kIncomplete);
  for (const char* bad : {"scab", "hello v1", "scan\tproc\t1\r", "scan\tproc\t1\t1\t0\t1\nq",
                          "scan\tproc\t1\t1\t0\t1\np\tx\tb\t1\tk\t0\tc\n", "scan\tproc\t1\t1\t0\t1\t-3\n"})
    CHECK(memcap::ParseScanReply(bad, &back, &used) == PR::kMalformed);
  // the render-only count travels; a relay of the previous version (6 header fields) is read too
  scan.render_only = 2;
  CHECK(memcap::ParseScanReply(memcap::SerializeScan(scan), &back, &used) == PR::kOk && back.render_only == 2);
  CHECK(memcap::ParseScanReply("scan\tproc\t1\t1\t0\t0\n", &back, &used) == PR::kOk && back.render_only == 0);
}

static void TestRemoteScan() {
  g_case = "remote-scan";
  memcap::DriverScan scan;
  scan.pid_source = "kfd";
  scan.pids_scanned = 1;
  scan.procs = {{42, "0000:0c:00.0", 7u << 20, "0::/pod/a", "k", false}};
  memcap::Aggregate(&scan);
  int sv[2];
  CHECK(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
  // the relay's greeting, then (after the request) the reply in two pieces
  std::thread relay([&] {
    std::string hello = "hello v1 events=ok processors=1\n";
    CHECK(write(sv[1], hello.data(), hello.size()) == static_cast<ssize_t>(hello.size()));
    char req[512];
    ssize_t n = read(sv[1], req, sizeof(req));
    CHECK(n > 0 && std::string(req, static_cast<size_t>(n)) == "scan\t/usage\t0::/self\n");
    std::string reply = memcap::SerializeScan(scan);
    CHECK(write(sv[1], reply.data(), 7) == 7);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    CHECK(write(sv[1], reply.data() + 7, reply.size() - 7) == static_cast<ssize_t>(reply.size() - 7));
  });
  auto r = memcap::RemoteScan(sv[0], "/usage", "0::/self", 5000);
  relay.join();
  CHECK(r.ok() && r->pid_source == "kfd" && r->procs.size() == 1 && r->procs[0].pid == 42);
  CHECK((r->by_grant[{"k", "0000:0c:00.0"}] == 7u << 20));
  close(sv[1]);
  // a closed connection before a full reply is an error, not a partial scan
  r = memcap::RemoteScan(sv[0], "/usage", "0::/self", 5000);
  CHECK(!r.ok());
  close(sv[0]);
  // a tab in the directory never reaches the wire
  CHECK(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
  CHECK(!memcap::RemoteScan(sv[0], "/us\tage", "c", 100).ok());
  close(sv[0]);
  close(sv[1]);
}

static void TestDrainSyntax() {
  g_case = "drain-syntax";
  auto t = health::DrainTokens("# maintenance\n0000:0c:00.0  # fan\r\nGPU-a,GPU-b\t3\n\n#0000:0d:00.0\n");
  CHECK((t == std::set<std::string>{"0000:0c:00.0", "GPU-a", "GPU-b", "3"}));
  inventory::PhysicalGpu g;
  g.uuid = "GPU-a";
  g.bdf = "0000:0c:00.0";
  g.node_index = 3;
  inventory::Partition p;
  p.uuid = "GPU-a-p1";
  g.partitions.push_back(p);
  auto n = health::DrainNames(g);
  CHECK((n == std::set<std::string>{"GPU-a", "0000:0c:00.0", "0000:0c:00", "3", "GPU-a-p1"}));
  p.uuid = "GPU-a-p2";
  p.bdf = "0000:0c:00.1";
  g.partitions.push_back(p);  // two partitions: the second one's PCI function names the GPU too
  n = health::DrainNames(g);
  CHECK((n == std::set<std::string>{"GPU-a", "0000:0c:00.0", "0000:0c:00", "0000:0c:00.1", "3", "GPU-a-p1",
                                    "GPU-a-p2"}));
  CHECK(health::DrainTokens("").empty() && health::DrainTokens("# only a comment").empty());
}

static void TestProto() {
  g_case = "proto";
  pb::AllocateResponse r;
  r.container_responses.emplace_back();
  auto& c = r.container_responses[0];
  c.envs = {{"AMD_VISIBLE_DEVICES", "u1,u2"}};
  c.mounts.push_back({"/var/run/amd-container-devices/u1", "/dev/null", true});
  c.devices.push_back({"/dev/kfd", "/dev/kfd", "rw"});
  c.devices.push_back({"/dev/dri/renderD128", "/dev/dri/renderD128", "rw"});
  c.annotations = {{"k", ""}};
  c.cdi_devices = {"amd.com/gpu=u1"};
  std::string b = pb::Encode(r);
  pb::AllocateResponse d;
  CHECK(pb::Decode(b, &d).ok());
  CHECK(d.container_responses.size() == 1);
  const auto& e = d.container_responses[0];
  CHECK(e.envs == c.envs && e.annotations == c.annotations && e.cdi_devices == c.cdi_devices);
  CHECK(e.mounts.size() == 1 && e.mounts[0].read_only && e.mounts[0].host_path == "/dev/null");
  CHECK(e.devices.size() == 2 && e.devices[1].container_path == "/dev/dri/renderD128");
  CHECK(pb::Encode(d) == b);

  pb::ListAndWatchResponse law;
  law.devices.push_back({"id0", pb::kHealthy, true, {1}});
  law.devices.push_back({"id1", pb::kUnhealthy, false, {}});
  pb::ListAndWatchResponse law2;
  CHECK(pb::Decode(pb::Encode(law), &law2).ok());
  CHECK(law2.devices.size() == 2 && law2.devices[0].numa_nodes == std::vector<int64_t>{1} &&
        !law2.devices[1].has_topology && law2.devices[1].health == pb::kUnhealthy);

  pb::PreferredAllocationRequest pr;
  pr.container_requests.push_back({{"a", "b"}, {"a"}, -1});
  pb::PreferredAllocationRequest pr2;
  CHECK(pb::Decode(pb::Encode(pr), &pr2).ok());
  CHECK(pr2.container_requests[0].allocation_size == -1 && pr2.container_requests[0].must_include == V({"a"}));

  pb::AllocateRequest bad;
  CHECK(!pb::Decode(std::string("\x0a\x05\x0a\x09", 4), &bad).ok());  // truncated
}

// DecodeView (zero-copy, fast path over the run of available IDs, reused
// capacity) against the owning Decode: random requests -- IDs of 0..200 bytes
// (two-byte and three-byte headers), must_include before or after, several
// container requests -- and random corruptions of them.
static void TestPreferredViewFuzz() {
  g_case = "proto/preferred-view-differential";
  uint64_t seed = 0x2545f4914f6cdd1dull;
  auto rnd = [&](uint64_t n) {
    seed ^= seed << 13;
    seed ^= seed >> 7;
    seed ^= seed << 17;
    return n ? seed % n : 0;
  };
  std::vector<pb::ContainerPreferredAllocationRequestView> views;  // reused across iterations
  int agreed = 0, rejected = 0;
  for (int it = 0; it < 4000; ++it) {
    pb::PreferredAllocationRequest pr;
    int ncr = 1 + static_cast<int>(rnd(3));
    for (int c = 0; c < ncr; ++c) {
      pb::ContainerPreferredAllocationRequest cr;
      int n = static_cast<int>(rnd(60));
      for (int i = 0; i < n; ++i) cr.available.push_back(std::string(rnd(8) ? 20 + rnd(60) : rnd(201), 'a' + rnd(26)));
      for (int i = 0, m = static_cast<int>(rnd(3)); i < m; ++i) cr.must_include.push_back(std::string(1 + rnd(40), 'x'));
      cr.allocation_size = static_cast<int32_t>(rnd(9)) - 1;
      pr.container_requests.push_back(std::move(cr));
    }
    std::string b = pb::Encode(pr);
    if (rnd(4) == 0) {  // must_include first: re-encode the fields of the first request in the other order
      std::string c0, rest;
      for (const auto& id : pr.container_requests[0].must_include) pb::PutLen(&c0, 2, id);
      for (const auto& id : pr.container_requests[0].available) pb::PutLen(&c0, 1, id);
      pb::PutInt32(&c0, 3, pr.container_requests[0].allocation_size);
      pb::PutLen(&rest, 1, c0);
      for (size_t c = 1; c < pr.container_requests.size(); ++c) {
        pb::PreferredAllocationRequest one;
        one.container_requests.push_back(pr.container_requests[c]);
        rest += pb::Encode(one);
      }
      b = rest;
    }
    if (rnd(3) == 0 && !b.empty()) {  // corrupt: flip, truncate or extend
      switch (rnd(3)) {
        case 0: b[rnd(b.size())] ^= static_cast<char>(1 + rnd(255)); break;
        case 1: b.resize(rnd(b.size())); break;
        default: b += std::string(1 + rnd(4), static_cast<char>(rnd(256)));
      }
    }
    pb::PreferredAllocationRequest owned;
    bool ok_owned = pb::Decode(b, &owned).ok();
    bool ok_view = pb::DecodeView(b, &views).ok();
    CHECK(ok_owned == ok_view);
    if (!ok_owned) { ++rejected; continue; }
    CHECK(views.size() == owned.container_requests.size());
    for (size_t c = 0; c < views.size() && c < owned.container_requests.size(); ++c) {
      const auto& o = owned.container_requests[c];
      const auto& v = views[c];
      CHECK(v.allocation_size == o.allocation_size);
      CHECK(std::vector<std::string>(v.available.begin(), v.available.end()) == o.available);
      CHECK(std::vector<std::string>(v.must_include.begin(), v.must_include.end()) == o.must_include);
    }
    ++agreed;
  }
  CHECK(agreed > 1000 && rejected > 100);
}

// The original map/set implementation of the hierarchical (partition) policy,
// kept as the oracle for the flat-array one in alloc/topology.cc.
static std::vector<int> OracleHierarchical(const alloc::DeviceGraph& g, const std::vector<int>& avail,
                              const std::vector<int>& required, int size) {
  std::set<int> chosen(required.begin(), required.end());
  std::map<int, std::vector<int>> remaining;  // parent -> unchosen available devices
  std::map<int, int> rep;                     // parent -> representative device
  for (int d : avail) {
    rep.emplace(g.parent(d), d);
    if (!chosen.count(d)) remaining[g.parent(d)].push_back(d);
  }
  std::set<int> parents;
  for (int d : required) parents.insert(g.parent(d));
  int need = size - static_cast<int>(chosen.size());

  auto take = [&](int p) {
    auto& v = remaining[p];
    while (need > 0 && !v.empty()) {
      chosen.insert(v.front());
      v.erase(v.begin());
      --need;
    }
    parents.insert(p);
  };

  // 1. Finish on the GPUs the required devices already occupy (most room first).
  std::vector<int> req_parents(parents.begin(), parents.end());
  std::stable_sort(req_parents.begin(), req_parents.end(),
                   [&](int a, int b) { return remaining[a].size() > remaining[b].size(); });
  for (int p : req_parents) take(p);

  // 2. Grow: affinity to the GPUs already chosen, then best fit, then index.
  while (need > 0) {
    int best = -1;
    long best_aff = LONG_MIN;
    bool best_fits = false;
    size_t best_room = 0;
    for (auto& [p, v] : remaining) {
      if (v.empty() || parents.count(p)) continue;
      long aff = 0;
      for (int q : parents) aff += g.Score(rep[p], rep[q]);
      bool fits = v.size() >= static_cast<size_t>(need);
      bool better;
      if (best < 0) better = true;
      else if (aff != best_aff) better = aff > best_aff;
      else if (fits != best_fits) better = fits;
      else if (fits) better = v.size() < best_room;   // best fit: tightest hole
      else better = v.size() > best_room;             // else: biggest chunk first
      if (better) {
        best = p;
        best_aff = aff;
        best_fits = fits;
        best_room = v.size();
      }
    }
    if (best < 0) return {};
    take(best);
  }
  return std::vector<int>(chosen.begin(), chosen.end());
}

// Randomised differential test: partition graphs always take the hierarchical
// path; every result must equal the oracle's.
static void TestHierarchicalMatchesOracle() {
  g_case = "topology/hierarchical-differential";
  uint64_t seed = 0x9e3779b97f4a7c15ull;
  auto rnd = [&](int n) {
    seed ^= seed << 13; seed ^= seed >> 7; seed ^= seed << 17;
    return static_cast<int>(seed % static_cast<uint64_t>(n));
  };
  int mismatches = 0, cases = 0;
  for (int iter = 0; iter < 3000; ++iter) {
    int gpus = 1 + rnd(8), per = 1 + rnd(8), n = gpus * per;
    std::vector<int> parent(n), score(n * n);
    for (int i = 0; i < n; ++i) parent[i] = i / per;
    std::vector<int> gscore(gpus * gpus);
    for (int a = 0; a < gpus; ++a)
      for (int b = a; b < gpus; ++b) gscore[a * gpus + b] = gscore[b * gpus + a] = 100 + 10 * rnd(3);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j)
        score[i * n + j] = i == j ? 0 : parent[i] == parent[j] ? 1000 : gscore[parent[i] * gpus + parent[j]];
    alloc::DeviceGraph g(parent, score);
    std::vector<int> avail, req;
    for (int i = 0; i < n; ++i)
      if (rnd(4)) avail.push_back(i);
    if (avail.empty()) continue;
    for (int d : avail)
      if (rnd(10) == 0) req.push_back(d);
    int size = static_cast<int>(req.size()) + rnd(static_cast<int>(avail.size() - req.size()) + 1);
    if (size <= 0) continue;
    bool distinct = per == 1;
    if (distinct && avail.size() <= 12) continue;  // exact path, covered elsewhere
    ++cases;
    auto got = alloc::BestEffortAllocate(g, avail, req, size);
    auto want = OracleHierarchical(g, avail, req, size);
    if (got != want) ++mismatches;
  }
  CHECK(cases > 1000);
  CHECK(mismatches == 0);
}

static void TestTopology() {
  g_case = "topology";
  // 4 GPUs: 0,1 on NUMA 0 and 2,3 on NUMA 1, full xGMI. Scores: same NUMA 120, cross 110.
  std::vector<int> parent = {0, 1, 2, 3};
  auto score = [](int a, int b) { return (a / 2 == b / 2) ? 120 : 110; };
  std::vector<int> s(16);
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) s[a * 4 + b] = a == b ? 0 : score(a, b);
  alloc::DeviceGraph g(parent, s);
  CHECK(alloc::BestEffortAllocate(g, {0, 1, 2, 3}, {}, 2) == std::vector<int>({0, 1}));
  CHECK(alloc::BestEffortAllocate(g, {0, 1, 2, 3}, {2}, 2) == std::vector<int>({2, 3}));
  CHECK(alloc::BestEffortAllocate(g, {0, 2, 3}, {}, 2) == std::vector<int>({2, 3}));
  CHECK(alloc::BestEffortAllocate(g, {0, 1}, {}, 3).empty());
  CHECK(alloc::BestEffortAllocate(g, {0, 1, 2, 3}, {}, 0).empty());
  CHECK(alloc::BestEffortAllocate(g, {0, 1, 2, 3}, {0, 1, 2}, 2).empty());
  // Partitions: 2 GPUs x 4 partitions; GPU 0 has 1 free, GPU 1 has 4 free.
  std::vector<int> pp = {0, 1, 1, 1, 1};
  std::vector<int> ps(25);
  for (int a = 0; a < 5; ++a)
    for (int b = 0; b < 5; ++b) ps[a * 5 + b] = a == b ? 0 : (pp[a] == pp[b] ? 1000 : 110);
  alloc::DeviceGraph pg(pp, ps);
  CHECK(alloc::BestEffortAllocate(pg, {0, 1, 2, 3, 4}, {}, 1) == std::vector<int>({0}));   // best fit
  CHECK(alloc::BestEffortAllocate(pg, {0, 1, 2, 3, 4}, {}, 2) == std::vector<int>({1, 2})); // one die
  CHECK(alloc::BestEffortAllocate(pg, {0, 1, 2, 3, 4}, {0}, 2).size() == 2);
}

static void TestConfig() {
  g_case = "config";
  std::map<std::string, std::string> env = {{"FAIL_ON_INIT_ERROR", "false"}, {"DEVICE_ID_STRATEGY", "index"}};
  const char* argv[] = {"x", "--device-id-strategy=uuid", "--pass-device-specs", "--partition-strategy", "mixed"};
  auto c = daemon::LoadConfig(5, argv, &env);
  CHECK(c.ok());
  if (c.ok()) {
    CHECK(!c->flags.fail_on_init_error);
    CHECK(c->flags.device_id_strategy == "uuid");
    CHECK(c->flags.partition_strategy == "mixed");
  }
  auto f = daemon::ParseConfigFile("version: v1\nflags:\n  failOnInitError: false # comment\n  resourceConfig: 'gpu:g:2'\n");
  CHECK(f.ok());
  if (f.ok()) {
    CHECK(f->values["flags.failOnInitError"].text == "false" && f->values["flags.failOnInitError"].type == 'b');
    CHECK(f->values["flags.resourceConfig"].text == "gpu:g:2" && f->values["flags.resourceConfig"].type == 's');
  }
  CHECK(!daemon::ParseConfigFile("flags:\n  a: b\n").ok());
  CHECK(!daemon::ParseConfigFile("version: v2\n").ok());
  auto j = daemon::ParseConfigFile("{\"version\": \"v1\", \"flags\": {\"passDeviceSpecs\": false}}");
  CHECK(j.ok() && j->values["flags.passDeviceSpecs"].text == "false");
  // Flow style, as sigs.k8s.io/yaml accepts it (the round-1 parser dropped it).
  auto flow = daemon::ParseConfigFile("version: v1\nflags: {migStrategy: single, failOnInitError: no}\n");
  CHECK(flow.ok() && flow->values["flags.migStrategy"].text == "single" &&
        flow->values["flags.failOnInitError"].text == "false");
  CHECK(!daemon::ParseConfigFile("version: v1\nflags: [a, b]\n").ok());
  CHECK(!daemon::ParseConfigFile("version: v1\nflags: single\n").ok());
  auto unknown = daemon::ParseConfigFile("version: v1\nflags:\n  migStrategi: single\nextra: 1\n");
  CHECK(unknown.ok() && unknown->warnings.size() == 2 && unknown->values.count("flags.migStrategi") == 0);
  const char* bad[] = {"x", "--no-such-flag"};
  CHECK(!daemon::LoadConfig(2, bad, &env).ok());
}

// Precedence, property-tested over every setting: each one randomly given on
// the command line, in the environment and in the config file, each by its
// canonical name and by its compatibility alias where it has one; the value
// that wins is the highest source's -- command line > environment > file >
// default, the canonical name before the alias at each level (config.cc
// LoadConfig; the reference's order, main.go:62-130 + config.go:30-144, with
// its quirk fixed: a `false` in the file turns a default-on flag off).
static void TestConfigPrecedenceProperty() {
  g_case = "config precedence";
  const std::vector<daemon::FlagInfo> flags = daemon::FlagTable();
  CHECK(flags.size() > 50);
  std::mt19937_64 rng(20261018);
  char path[] = "/tmp/adp-precedence-XXXXXX";
  int fd = mkstemp(path);
  CHECK(fd >= 0);
  if (fd < 0) return;
  close(fd);
  const daemon::Config defaults;
  const nlohmann::json dflt = nlohmann::json::parse(defaults.ToJson())["flags"];
  int from_level[7] = {0};
  for (int trial = 0; trial < 300; ++trial) {
    std::vector<std::string> args = {"x", "--config-file", path};
    std::map<std::string, std::string> env;
    std::string file = "version: v1\nflags:\n";
    std::vector<nlohmann::json> want(flags.size());
    std::vector<int> won(flags.size(), 6);
    for (size_t i = 0; i < flags.size(); ++i) {
      const daemon::FlagInfo& f = flags[i];
      const std::string names[6] = {f.name, f.alias_name, f.env, f.alias_env, f.file_key, f.alias_file_key};
      const std::string key = f.file_key.empty() ? f.name : f.file_key;
      want[i] = dflt[key];
      for (int src = 0; src < 6; ++src) {
        if (names[src].empty() || rng() % 3 != 0) continue;
        // A value of the setting's type: JSON (what ToJson shows) + its text.
        nlohmann::json v;
        std::string text;
        if (f.kind == 'b') {
          v = static_cast<bool>(rng() % 2);
          text = v.get<bool>() ? "true" : "false";
        } else if (f.kind == 'u') {
          uint64_t n = (f.allow_zero ? 0 : 1) + rng() % 5000;
          v = n;
          text = std::to_string(n);
        } else {
          text = rng() % 4 == 0 ? std::to_string(1000 + rng() % 9000)  // a number where a string belongs
                                : "v" + std::to_string(trial) + "-" + std::to_string(i) + "-" + std::to_string(src);
          v = text;
        }
        if (src <= 1) {
          if (f.kind == 'b' && text == "true" && rng() % 2) args.push_back("--" + names[src]);  // bare bool
          else if (rng() % 2) args.push_back("--" + names[src] + "=" + text);
          else if (f.kind != 'b') args.insert(args.end(), {"--" + names[src], text});
          else args.push_back("--" + names[src] + "=" + text);
        } else if (src <= 3) {
          env[names[src]] = text;
        } else {
          // Plain or quoted: a quoted "true" / "12" is accepted for a bool / integer too.
          const bool quote = f.kind == 's' ? !std::all_of(text.begin(), text.end(), ::isdigit) || rng() % 2
                                           : rng() % 3 == 0;
          file += "  " + names[src] + ": " + (quote ? "'" + text + "'" : text) + "\n";
        }
        if (src < won[i]) {
          won[i] = src;
          want[i] = v;
        }
      }
    }
    FILE* out = fopen(path, "w");
    CHECK(out != nullptr);
    if (!out) break;
    fputs(file.c_str(), out);
    fclose(out);
    std::vector<const char*> argv;
    for (const auto& a : args) argv.push_back(a.c_str());
    auto c = daemon::LoadConfig(static_cast<int>(argv.size()), argv.data(), &env);
    CHECK(c.ok());
    if (!c.ok()) {
      fprintf(stderr, "trial %d: %s\n", trial, c.status().ToString().c_str());
      continue;
    }
    const nlohmann::json got = nlohmann::json::parse(c->ToJson())["flags"];
    for (size_t i = 0; i < flags.size(); ++i) {
      const std::string key = flags[i].file_key.empty() ? flags[i].name : flags[i].file_key;
      ++from_level[won[i]];
      if (got[key] != want[i]) {
        CHECK(got[key] == want[i]);
        fprintf(stderr, "trial %d: %s = %s, want %s (from source %d)\n", trial, key.c_str(), got[key].dump().c_str(),
                want[i].dump().c_str(), won[i]);
      }
    }
  }
  unlink(path);
  // Every level decided some settings (the aliases are few: fewer wins there).
  for (int l = 0; l < 7; ++l) CHECK(from_level[l] > 0);
}

static void TestGrpcLoopback(bool native_http2) {
  g_case = native_http2 ? "grpc" : "grpc/nghttp2";
  std::string dir = "/tmp/adp-unit-" + std::to_string(getpid());
  mkdir(dir.c_str(), 0755);
  std::string sock = dir + "/t.sock";
  grpc::Server srv("test");
  srv.set_native_http2(native_http2);
  srv.AddUnary("/t.S/Echo", [](std::string_view q, std::string* r) {
    r->assign(q);
    return Status::Ok();
  });
  srv.AddUnary("/t.S/Fail", [](std::string_view, std::string*) { return InvalidArgument("bad thing: 100%"); });
  std::shared_ptr<grpc::ServerStream> keep;
  srv.AddServerStream("/t.S/Watch", [&](std::string_view, std::shared_ptr<grpc::ServerStream> s) {
    keep = s;
    s->Send("first");
    return Status::Ok();
  });
  CHECK(srv.Listen(sock).ok());
  CHECK(srv.Start().ok());
  auto ch = grpc::Channel::Dial(sock, 2000);
  CHECK(ch.ok());
  if (ch.ok()) {
    std::string resp;
    std::string big(300000, 'x');
    CHECK((*ch)->Unary("/t.S/Echo", big, &resp, 2000).ok() && resp == big);
    Status st = (*ch)->Unary("/t.S/Fail", "", &resp, 2000);
    CHECK(st.code() == Code::kInvalidArgument && st.message() == "bad thing: 100%");
    CHECK((*ch)->Unary("/t.S/Nope", "", &resp, 2000).code() == Code::kUnimplemented);
    auto sid = (*ch)->StartStream("/t.S/Watch", "");
    CHECK(sid.ok());
    std::string m;
    CHECK((*ch)->Recv(*sid, &m, 2000).ok() && m == "first");
    // A client that stops reading: 300 x 100 KB snapshots (30 MB >> flow-control
    // windows) are coalesced server-side; the client still ends on the newest.
    g_case = "grpc/stream-coalescing";
    srv.Post([&] {
      for (int i = 0; i < 300; ++i) keep->Send(std::string(100000, static_cast<char>('a' + i % 26)) + std::to_string(i));
    });
    usleep(200 * 1000);
    int received = 0;
    std::string last;
    // Read until the newest snapshot arrives (a sanitizer build produces the 30 MB
    // slowly: no fixed per-message timeout), within a generous overall deadline.
    auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(20);
    while (!EndsWith(last, "299") && std::chrono::steady_clock::now() < deadline) {
      if ((*ch)->Recv(*sid, &m, 1000).ok()) {
        ++received;
        last = m;
      }
    }
    CHECK(received >= 1 && received < 300);
    CHECK(EndsWith(last, "299"));
    srv.Post([&] { keep->Send(std::string(100000, 'y')); keep->Finish(Status::Ok()); });
    CHECK((*ch)->Recv(*sid, &m, 2000).ok() && m.size() == 100000);
    CHECK((*ch)->Recv(*sid, &m, 2000).code() == Code::kNotFound);
    g_case = native_http2 ? "grpc" : "grpc/nghttp2";
  }
  srv.Stop();
  unlink(sock.c_str());
  if (!native_http2) {
    rmdir(dir.c_str());
    return;
  }

  // Crash budget (server.go:177-205): a loop that keeps failing within the hour
  // is fatal on the 7th failure; it keeps serving until then.
  g_case = "grpc/crash-budget";
  grpc::Server flaky("flaky");
  flaky.AddUnary("/t.S/Echo", [](std::string_view q, std::string* r) { r->assign(q); return Status::Ok(); });
  std::atomic<int> fatal{0};
  CHECK(flaky.Listen(sock).ok());
  CHECK(flaky.Start([&] { fatal.fetch_add(1); }).ok());
  for (int i = 0; i < 6; ++i) {
    flaky.InjectLoopFailureForTest();
    flaky.Post([] {});
    usleep(20 * 1000);
  }
  CHECK(fatal.load() == 0);
  auto ch2 = grpc::Channel::Dial(sock, 2000);
  std::string r2;
  CHECK(ch2.ok() && (*ch2)->Unary("/t.S/Echo", "still", &r2, 2000).ok() && r2 == "still");
  flaky.InjectLoopFailureForTest();
  flaky.Post([] {});
  for (int i = 0; i < 100 && fatal.load() == 0; ++i) usleep(10 * 1000);
  CHECK(fatal.load() == 1);
  flaky.Stop();
  unlink(sock.c_str());
  rmdir(dir.c_str());
}

// The native HTTP/2 parser on hostile input (run under ASan/UBSan by `make
// asan`): a valid preface and SETTINGS, then random mixes of well-formed
// requests and random frames (types, flags, stream ids, lengths, payloads),
// delivered in random-sized chunks. The connection may end at any point, but
// must never crash, read out of bounds or leak.
static void TestH2Fuzz() {
  g_case = "h2-fuzz";
  grpc::Server srv("fuzz");
  srv.AddUnary("/t.S/Echo", [](std::string_view q, std::string* r) { r->assign(q); return Status::Ok(); });
  srv.AddServerStream("/t.S/Watch", [](std::string_view, std::shared_ptr<grpc::ServerStream> s) {
    s->Send(std::string(70000, 'w'));
    return Status::Ok();
  });
  uint64_t rng = 0x9e3779b97f4a7c15ull;
  auto next = [&] {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  auto frame = [](uint8_t type, uint8_t flags, uint32_t sid, const std::string& p) {
    std::string f;
    f.push_back(static_cast<char>(p.size() >> 16));
    f.push_back(static_cast<char>(p.size() >> 8));
    f.push_back(static_cast<char>(p.size()));
    f.push_back(static_cast<char>(type));
    f.push_back(static_cast<char>(flags));
    for (int i = 3; i >= 0; --i) f.push_back(static_cast<char>(sid >> (8 * i)));
    return f + p;
  };
  auto lit = [](const std::string& n, const std::string& v) {
    return std::string(1, '\0') + static_cast<char>(n.size()) + n + static_cast<char>(v.size()) + v;
  };
  int survived = 0, conns = 0;
  for (int round = 0; round < 1500; ++round) {
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK, 0, sv) != 0) break;
    auto conn = grpc::MakeH2Conn(&srv, 0, sv[1]);  // owns sv[1]
    if (!conn->Init()) { close(sv[0]); continue; }
    ++conns;
    std::string in = std::string("PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n") + frame(4, 0, 0, "");
    uint32_t sid = 1;
    int nframes = 1 + static_cast<int>(next() % 24);
    for (int i = 0; i < nframes; ++i) {
      uint64_t r = next();
      if (r % 3 == 0) {  // a well-formed call, sometimes split or padded
        std::string path = (r & 8) ? "/t.S/Watch" : "/t.S/Echo";
        std::string hb = lit(":method", "POST") + lit(":path", path) + lit("content-type", "application/grpc");
        std::string msg = std::string(1, '\0') + std::string("\0\0\0\3", 4) + "abc";
        if (r & 16) {
          in += frame(1, 0, sid, hb.substr(0, 5)) + frame(9, 4, sid, hb.substr(5));
        } else {
          in += frame(1, 4, sid, hb);
        }
        in += frame(0, 1 | ((r & 32) ? 8 : 0), sid, (r & 32) ? std::string(1, '\2') + msg + "xx" : msg);
        sid += 2;
      } else {  // a random frame
        std::string payload;
        size_t len = next() % ((r & 64) ? 70000 : 40);
        for (size_t k = 0; k < len; ++k) payload.push_back(static_cast<char>(next()));
        uint32_t fsid = (r & 128) ? 0 : static_cast<uint32_t>(next() % 16);
        in += frame(static_cast<uint8_t>(next() % 12), static_cast<uint8_t>(next()), fsid, payload);
      }
    }
    if (next() % 4 == 0) in.resize(next() % (in.size() + 1));  // truncated mid-frame
    bool alive = true;
    size_t off = 0;
    char sink[65536];
    while (alive && off < in.size()) {
      size_t chunk = std::min<size_t>(in.size() - off, 1 + next() % 9000);
      ssize_t w = write(sv[0], in.data() + off, chunk);
      if (w > 0) off += static_cast<size_t>(w);
      alive = conn->OnReadable() && !conn->Done();
      while (read(sv[0], sink, sizeof(sink)) > 0) {
      }
      if (w <= 0) alive = alive && conn->Flush();
    }
    if (alive) ++survived;
    conn.reset();
    close(sv[0]);
  }
  CHECK(conns == 1500);
  CHECK(survived > 0 && survived < conns);  // both outcomes were exercised
}

// N loops: connections are dealt round-robin, handlers of different connections
// run on different threads, PostAll reaches every loop, and each stream is
// only touched by the loop that owns it.
static void TestGrpcMultiLoop() {
  g_case = "grpc/multi-loop";
  std::string dir = "/tmp/adp-unit-ml-" + std::to_string(getpid());
  mkdir(dir.c_str(), 0755);
  std::string sock = dir + "/m.sock";
  constexpr int kLoops = 4, kClients = 8;
  grpc::Server srv("multi", kLoops);
  CHECK(srv.loops() == kLoops);
  std::mutex mu;
  std::set<std::thread::id> threads;
  std::vector<std::vector<std::shared_ptr<grpc::ServerStream>>> per_loop(kLoops);
  std::atomic<int> early{0}, off_loop{0};
  srv.Post([&] { early.fetch_add(1); });  // queued before Start()
  srv.AddUnary("/t.S/Who", [&](std::string_view q, std::string* r) {
    std::lock_guard<std::mutex> lk(mu);
    threads.insert(std::this_thread::get_id());
    r->assign(q);
    return Status::Ok();
  });
  srv.AddServerStream("/t.S/Watch", [&](std::string_view, std::shared_ptr<grpc::ServerStream> s) {
    if (!srv.OnLoopThread()) off_loop.fetch_add(1);
    per_loop[s->loop()].push_back(s);  // confined to loop s->loop()
    s->Send("hello");
    return Status::Ok();
  });
  CHECK(srv.Listen(sock).ok());
  CHECK(srv.Start().ok());
  std::vector<std::unique_ptr<grpc::Channel>> chans;
  std::vector<int32_t> sids;
  for (int i = 0; i < kClients; ++i) {
    auto ch = grpc::Channel::Dial(sock, 2000);
    CHECK(ch.ok());
    if (!ch.ok()) break;
    chans.push_back(std::move(*ch));
  }
  for (auto& ch : chans) {
    std::string r;
    CHECK(ch->Unary("/t.S/Who", "x", &r, 2000).ok() && r == "x");
    auto sid = ch->StartStream("/t.S/Watch", "");
    CHECK(sid.ok());
    std::string m;
    CHECK(sid.ok() && ch->Recv(*sid, &m, 2000).ok() && m == "hello");
    sids.push_back(sid.ok() ? *sid : 0);
  }
  CHECK(early.load() == 1);
  CHECK(off_loop.load() == 0);
  {
    std::lock_guard<std::mutex> lk(mu);
    CHECK(static_cast<int>(threads.size()) == kLoops);
  }
  std::atomic<int> reached{0};
  srv.PostAll([&](int loop) {
    reached.fetch_add(1);
    for (auto& s : per_loop[loop]) s->Send("update-" + std::to_string(loop));
  });
  for (size_t i = 0; i < chans.size(); ++i) {
    std::string m;
    CHECK(chans[i]->Recv(sids[i], &m, 2000).ok() && StartsWith(m, "update-"));
  }
  CHECK(reached.load() == kLoops);
  int streams = 0;
  for (auto& v : per_loop) streams += static_cast<int>(v.size());
  CHECK(streams == kClients);
  for (auto& v : per_loop) CHECK(v.size() == kClients / kLoops);  // round-robin
  srv.PostAll([&](int loop) {
    for (auto& s : per_loop[loop]) s->Finish(Status::Ok());
  });
  for (size_t i = 0; i < chans.size(); ++i) {
    std::string m;
    CHECK(chans[i]->Recv(sids[i], &m, 2000).code() == Code::kNotFound);
  }
  srv.Stop();
  srv.Stop();  // idempotent
  srv.Post([] {});  // dropped after Stop
  chans.clear();
  for (auto& v : per_loop) v.clear();
  rmdir(dir.c_str());
}

// Sharded counters/histograms: exact totals from many writer threads.
static void TestMetrics() {
  g_case = "metrics";
  metrics::Counter c;
  metrics::MaxGauge m;
  metrics::Histogram h;
  std::vector<std::thread> ts;
  for (int t = 0; t < 20; ++t)
    ts.emplace_back([&, t] {
      for (int i = 0; i < 10000; ++i) {
        c.Add(1);
        m.Observe(static_cast<uint64_t>(t) * 1000 + i % 7);
        h.Observe(i % 2 ? 300 : 3000);  // 500 ns and 5 us buckets
      }
    });
  for (auto& t : ts) t.join();
  CHECK(c.Value() == 200000);
  CHECK(m.Value() == 19 * 1000 + 6);
  CHECK(h.count() == 200000);
  CHECK(h.QuantileUs(0.25) == 0.5);
  CHECK(h.QuantileUs(0.99) == 5.0);
  std::string text;
  h.AppendPrometheus("x_seconds", "a=\"b\"", &text);
  CHECK(text.find("x_seconds_bucket{a=\"b\",le=\"+Inf\"} 200000\n") != std::string::npos);
  CHECK(text.find("x_seconds_count{a=\"b\"} 200000\n") != std::string::npos);
  CHECK(metrics::LabelValue("a\"b\\c\n") == "a\\\"b\\\\c\\n");

  // 100 ns bins: 3,000 x 2.35 us, 1,000 x 7.05 us, 10 beyond the last bin.
  metrics::FineHistogram f;
  std::vector<std::thread> fs;
  for (int t = 0; t < 4; ++t)
    fs.emplace_back([&, t] {
      for (int i = 0; i < 1000; ++i) f.Observe(t == 3 ? 7050 : 2350);
      if (t == 0)
        for (int i = 0; i < 10; ++i) f.Observe(5000000);
    });
  for (auto& t : fs) t.join();
  std::vector<uint64_t> fc = f.Counts();
  CHECK(fc.size() == metrics::FineHistogram::kBins + 1);
  CHECK(fc[23] == 3000 && fc[70] == 1000 && fc[metrics::FineHistogram::kBins] == 10);
  CHECK(metrics::FineHistogram::QuantileUs(fc, 0.5) == 2.4);
  CHECK(metrics::FineHistogram::QuantileUs(fc, 0.9) == 7.1);
  CHECK(metrics::FineHistogram::QuantileUs({}, 0.5) == 0.0);
  CHECK(f.SparseJson() == "[[23, 3000], [70, 1000], [1024, 10]]");
  CHECK(f.sum_ns() == 3000ull * 2350 + 1000ull * 7050 + 10ull * 5000000);
  text.clear();
  f.AppendPrometheus("r_seconds", "", &text);
  CHECK(text.find("r_seconds_bucket{le=\"2e-06\"} 0\n") != std::string::npos);
  CHECK(text.find("r_seconds_bucket{le=\"5e-06\"} 3000\n") != std::string::npos);
  CHECK(text.find("r_seconds_bucket{le=\"1e-05\"} 4000\n") != std::string::npos);
  CHECK(text.find("r_seconds_bucket{le=\"0.0001\"} 4000\n") != std::string::npos);
  CHECK(text.find("r_seconds_bucket{le=\"+Inf\"} 4010\n") != std::string::npos);
  CHECK(text.find("r_seconds_count{} 4010\n") != std::string::npos);
}

// Log lines longer than the 4 KiB stack buffer come out whole.
static void TestLongLogLine() {
  g_case = "long log line";
  char path[] = "/tmp/adp_log_XXXXXX";
  int fd = mkstemp(path);
  CHECK(fd >= 0);
  fflush(stderr);
  int saved = dup(2);
  dup2(fd, 2);
  std::string big(10000, 'x');
  Logf(LogLevel::kError, "test", "head %s tail", big.c_str());
  fflush(stderr);
  dup2(saved, 2);
  close(saved);
  std::string text;
  char buf[4096];
  lseek(fd, 0, SEEK_SET);
  for (ssize_t n; (n = read(fd, buf, sizeof(buf))) > 0;) text.append(buf, static_cast<size_t>(n));
  close(fd);
  unlink(path);
  CHECK(text.find("head " + big + " tail\n") != std::string::npos);
}

static void TestPodResources() {
  g_case = "podresources";
  // pod_resources { name: "p" namespace: "n" containers { name: "c"
  //   devices { resource_name: "amd.com/gpu" device_ids: "a" device_ids: "b" } } }
  std::string devs, ctr, pod, resp;
  pb::PutStr(&devs, 1, "amd.com/gpu");
  pb::PutLen(&devs, 2, "a");
  pb::PutLen(&devs, 2, "b");
  pb::PutInt64(&devs, 7, 42);  // unknown field: skipped
  pb::PutStr(&ctr, 1, "c");
  pb::PutLen(&ctr, 2, devs);
  pb::PutStr(&pod, 1, "p");
  pb::PutStr(&pod, 2, "n");
  pb::PutLen(&pod, 3, ctr);
  pb::PutLen(&resp, 1, pod);
  std::vector<podresources::Assignment> out;
  CHECK(podresources::DecodeList(resp, &out).ok());
  CHECK(out.size() == 2);
  if (out.size() == 2)
    CHECK(out[1].pod == "p" && out[1].ns == "n" && out[1].container == "c" && out[1].resource == "amd.com/gpu" &&
          out[1].device_id == "b");
  out.clear();
  CHECK(!podresources::DecodeList(resp.substr(0, resp.size() - 3), &out).ok());
  CHECK(!podresources::DecodeList("\x0a\xff\xff\xff\xff\x0f", &out).ok());
}

static void TestReplicaCuRanges() {
  g_case = "replica-cu-ranges";
  using R = std::vector<std::pair<uint32_t, uint32_t>>;
  // MI355X SPX: 256 CUs over 8 XCDs; mask bit i lands on XCD i % 8.
  CHECK((plugin::ReplicaCuRanges(256, 8, 4) == R{{0, 63}, {64, 127}, {128, 191}, {192, 255}}));
  CHECK((plugin::ReplicaCuRanges(256, 8, 2) == R{{0, 127}, {128, 255}}));
  // Uneven split: every share still ends on an XCD boundary and is non-empty.
  R three = plugin::ReplicaCuRanges(256, 8, 3);
  CHECK((three == R{{0, 79}, {80, 167}, {168, 255}}));
  for (auto [lo, hi] : three) CHECK(lo % 8 == 0 && (hi + 1) % 8 == 0 && hi > lo);
  R r32 = plugin::ReplicaCuRanges(256, 8, 32);
  CHECK(r32.size() == 32 && r32[31] == std::make_pair(248u, 255u));
  for (size_t i = 0; i < r32.size(); ++i) CHECK(r32[i].first == 8 * i && r32[i].second == 8 * i + 7);
  // CPX partition: 32 CUs on one XCD.
  CHECK((plugin::ReplicaCuRanges(32, 1, 4) == R{{0, 7}, {8, 15}, {16, 23}, {24, 31}}));
  // Impossible or pointless splits.
  CHECK(plugin::ReplicaCuRanges(256, 8, 33).empty());  // < 1 CU per XCD per replica
  CHECK(plugin::ReplicaCuRanges(256, 8, 1).empty());
  CHECK(plugin::ReplicaCuRanges(0, 8, 4).empty());
  CHECK(plugin::ReplicaCuRanges(256, 0, 4).empty());
  CHECK(plugin::ReplicaCuRanges(250, 8, 4).empty());  // CUs not uniform over XCDs
  // Memory units: 294 x 1000 MiB of an MI355X over 32 CU slots (8 CUs each).
  R mu = plugin::MemoryUnitCuRanges(256, 8, 294);
  CHECK(mu.size() == 294);
  // replica 0 is first by name, replica 99 last ("99" > "293" > ... lexicographically)
  CHECK(mu[0] == std::make_pair(0u, 7u) && mu[99] == std::make_pair(248u, 255u));
  std::vector<unsigned> by_name(294);
  for (unsigned r = 0; r < 294; ++r) by_name[r] = r;
  std::sort(by_name.begin(), by_name.end(),
            [](unsigned a, unsigned b) { return std::to_string(a) < std::to_string(b); });
  size_t prev = 0;
  std::set<uint32_t> slots;
  for (unsigned r : by_name) {
    CHECK(mu[r].first % 8 == 0 && mu[r].second == mu[r].first + 7);
    CHECK(mu[r].first >= prev);  // monotonic in the IDs' name order
    prev = mu[r].first;
    slots.insert(mu[r].first);
  }
  CHECK(slots.size() == 32);  // every slot is owned by some unit
  CHECK(plugin::MemoryUnitCuRanges(256, 0, 294).empty());
}


static void TestYaml() {
  using adp::yaml::Node;
  using adp::yaml::ScalarType;
  auto plain = [](const char* v) {
    Node n;
    n.kind = Node::kScalar;
    n.plain = true;
    n.value = v;
    return n;
  };
  std::string c;
  // go-yaml v2 resolution
  CHECK(adp::yaml::Resolve(plain("yes"), &c) == ScalarType::kBool && c == "true");
  CHECK(adp::yaml::Resolve(plain("Off"), &c) == ScalarType::kBool && c == "false");
  CHECK(adp::yaml::Resolve(plain("n"), &c) == ScalarType::kBool && c == "false");
  CHECK(adp::yaml::Resolve(plain("0x1F"), &c) == ScalarType::kInt && c == "31");
  CHECK(adp::yaml::Resolve(plain("0o17"), &c) == ScalarType::kInt && c == "15");
  CHECK(adp::yaml::Resolve(plain("017"), &c) == ScalarType::kInt && c == "15");
  CHECK(adp::yaml::Resolve(plain("0b101"), &c) == ScalarType::kInt && c == "5");
  CHECK(adp::yaml::Resolve(plain("1_000"), &c) == ScalarType::kInt && c == "1000");
  CHECK(adp::yaml::Resolve(plain("-42"), &c) == ScalarType::kInt && c == "-42");
  CHECK(adp::yaml::Resolve(plain("99999999999999999999"), &c) == ScalarType::kFloat);
  CHECK(adp::yaml::Resolve(plain("1.5e3"), &c) == ScalarType::kFloat);
  CHECK(adp::yaml::Resolve(plain(".inf"), &c) == ScalarType::kFloat);
  CHECK(adp::yaml::Resolve(plain("~"), &c) == ScalarType::kNull);
  CHECK(adp::yaml::Resolve(plain("gpu:sharedgpu:4"), &c) == ScalarType::kString);
  CHECK(adp::yaml::Resolve(plain("1.2.3"), &c) == ScalarType::kString);
  Node quoted = plain("true");
  quoted.plain = false;
  CHECK(adp::yaml::Resolve(quoted, &c) == ScalarType::kString);
  Node tagged = plain("12");
  tagged.plain = false;
  tagged.tag = "tag:yaml.org,2002:str";
  CHECK(adp::yaml::Resolve(tagged, &c) == ScalarType::kString);
  tagged.tag = "tag:yaml.org,2002:int";
  CHECK(adp::yaml::Resolve(tagged, &c) == ScalarType::kInt && c == "12");

  if (adp::yaml::Available()) {
    CHECK(!adp::yaml::LibraryVersion().empty());
    auto doc = adp::yaml::Parse("a: &x {b: 1, c: [1, 2]}\nd: *x\ne:\n  <<: [*x, {f: 2}]\n  b: 9\n");
    CHECK(doc.ok());
    if (doc.ok()) {
      const Node* d = doc->Get("d");
      CHECK(d && d->kind == Node::kMap && d->Get("c") && d->Get("c")->seq.size() == 2);
      const Node* e = doc->Get("e");
      CHECK(e && e->Get("b") && e->Get("b")->value == "9" && e->Get("f") && e->Get("c"));
    }
    CHECK(!adp::yaml::Parse("a: *nope\n").ok());
    CHECK(!adp::yaml::Parse("a: [1, 2\n").ok());
    CHECK(!adp::yaml::Parse("{[1]: 2}\n").ok());  // non-scalar key
    CHECK(!adp::yaml::Parse("a: {<<: 3}\n").ok());  // merge of a scalar
    // billion laughs: alias expansion is bounded
    std::string bomb = "a: &a [x, x, x, x, x, x, x, x, x, x]\n";
    for (char k = 'b'; k <= 'j'; ++k)
      bomb += std::string(1, k) + ": &" + k + " [*" + char(k - 1) + ", *" + char(k - 1) + ", *" + char(k - 1) +
              ", *" + char(k - 1) + ", *" + char(k - 1) + ", *" + char(k - 1) + ", *" + char(k - 1) + ", *" +
              char(k - 1) + ", *" + char(k - 1) + ", *" + char(k - 1) + "]\n";
    auto b = adp::yaml::Parse(bomb);
    CHECK(!b.ok() && b.status().message().find("too large") != std::string::npos);
    bool extra = false;
    auto two = adp::yaml::Parse("a: 1\n---\nb: 2\n", &extra);
    CHECK(two.ok() && extra && two->Get("a") && !two->Get("b"));
    auto empty = adp::yaml::Parse("");
    CHECK(empty.ok() && empty->kind == Node::kNull);
  }

  // The strict subset parser (no libyaml).
  auto ok = adp::yaml::ParseSubset("# c\nversion: v1\nflags:\n  a: 'it''s'  # c\n  b: \"x\\ty\"\n  c:\n  d: ~\ntop: 1\n");
  CHECK(ok.ok());
  if (ok.ok()) {
    const Node* f = ok->Get("flags");
    CHECK(f && f->kind == Node::kMap && f->Get("a")->value == "it's" && f->Get("b")->value == "x\ty");
    CHECK(f->Get("c")->kind == Node::kNull && f->Get("d")->kind == Node::kNull && ok->Get("top")->value == "1");
  }
  const char* refused[] = {"a: {b: 1}\n", "a: [1]\n", "a: |\n  x\n", "a: >\n  x\n", "a: &x 1\n", "a: *x\n",
                           "a: !!str 1\n", "- a\n", "a: 1\n---\nb: 2\n", "%YAML 1.1\n---\na: 1\n",
                           "? a\n: b\n", "a:\n  <<: x\n", "a: \"open\n", "a: \"\\x41\"\n"};
  for (const char* r : refused) {
    auto st = adp::yaml::ParseSubset(r);
    CHECK(!st.ok() && st.status().message().find("libyaml") != std::string::npos);
  }
  const char* bad[] = {"a: 1\n b: 2\n", "a: 1\na: 2\n", "just text\n", "a: @x\n", "  a: 1\nb: 2\n"};
  for (const char* r : bad) CHECK(!adp::yaml::ParseSubset(r).ok());
}

// Random mutations of valid config documents: ParseConfigFile (libyaml and the
// subset parser) must return a Status, never crash or hang (run under ASan).
static void TestConfigFuzz() {
  const char* seeds[] = {
      "version: v1\nflags:\n  migStrategy: single\n  failOnInitError: false\n",
      "version: v1\nflags: {migStrategy: mixed, resourceConfig: 'gpu:a:2', serverThreads: 4}\n",
      "version: v1\nd: &d {deviceIDStrategy: index}\nflags:\n  <<: *d\n  resourceConfig: >-\n    gpu:a:2,\n    gpu:b:3\n",
      "{\"version\": \"v1\", \"flags\": {\"passDeviceSpecs\": false, \"devices\": \"0,1\"}}\n",
  };
  const char alphabet[] = "{}[]:,-&*!|>'\"#\n \t?%@`<~.0123456789abcxyzv";
  uint64_t x = 0x9E3779B97F4A7C15ull;
  auto rnd = [&x]() {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  };
  int ok = 0, failed = 0;
  for (int i = 0; i < 20000; ++i) {
    std::string doc = seeds[rnd() % 4];
    int edits = 1 + static_cast<int>(rnd() % 6);
    for (int e = 0; e < edits && !doc.empty(); ++e) {
      size_t pos = rnd() % (doc.size() + 1);
      switch (rnd() % 4) {
        case 0: doc.insert(pos, 1, alphabet[rnd() % (sizeof(alphabet) - 1)]); break;
        case 1: if (pos < doc.size()) doc.erase(pos, 1 + rnd() % 4); break;
        case 2: if (pos < doc.size()) doc[pos] = alphabet[rnd() % (sizeof(alphabet) - 1)]; break;
        case 3: doc.insert(pos, doc.substr(rnd() % doc.size(), rnd() % 12)); break;
      }
    }
    auto r = adp::daemon::ParseConfigFile(doc);
    (r.ok() ? ok : failed)++;
    auto sub = adp::yaml::ParseSubset(doc);
    (void)sub;
  }
  CHECK(ok > 0 && failed > 0);
}

// Grant accounting files: written by the background writer from several
// threads at once (Allocate() runs on every gRPC loop), read back, collected.
void TestMemcapUsage() {
  char tmpl[] = "/tmp/adp-usage-XXXXXX";
  char* root = mkdtemp(tmpl);
  CHECK(root != nullptr);
  if (!root) return;
  std::string dir = std::string(root) + "/amdgpu-dp/usage";  // created on first use
  CHECK(memcap::AllocationKey({"b", "a"}) == memcap::AllocationKey({"a", "b"}));
  CHECK(memcap::AllocationKey({"a", "b"}).size() == 16);
  std::vector<std::thread> ts;
  for (int t = 0; t < 4; ++t)
    ts.emplace_back([&, t] {
      for (int i = 0; i < 50; ++i) {
        std::string id = "gpu" + std::to_string(t) + "-replica-" + std::to_string(i);
        memcap::CreateGrantFileAsync(dir, memcap::AllocationKey({id}), {uint64_t(i + 1) << 20}, id);
      }
    });
  for (auto& t : ts) t.join();
  memcap::Flush();
  auto all = memcap::ReadAll(dir);
  CHECK(all.size() == 200);
  auto one = memcap::ReadGrant(dir, memcap::AllocationKey({"gpu2-replica-7"}));
  CHECK(one.ok());
  if (one.ok()) {
    CHECK(one->ids == "gpu2-replica-7");
    CHECK(one->cap.size() == 1 && one->cap[0] == (uint64_t(8) << 20));
    CHECK(one->used.size() == 1 && one->used[0] == 0 && one->peak[0] == 0 && one->refused[0] == 0);
  }
  CHECK(memcap::ReadGrant(dir, "0123456789abcdef").status().code() == Code::kNotFound);
  // Live: the gpu0 grants; everything else is too young to collect ...
  std::set<std::string> live;
  for (int i = 0; i < 50; ++i) live.insert(memcap::AllocationKey({"gpu0-replica-" + std::to_string(i)}));
  // (a runtime that mounted a path before it was written leaves a directory)
  CHECK(mkdir((dir + "/00000000000000aa.memcap").c_str(), 0755) == 0);
  CHECK(memcap::Collect(dir, &live, 120, 4096) == 0);
  // ... until it is not; and without a live set only the newest max_files stay.
  CHECK(memcap::Collect(dir, &live, 0, 4096) == 151);
  CHECK(memcap::ReadAll(dir).size() == 50);
  CHECK(memcap::Collect(dir, nullptr, 0, 10) == 40);
  CHECK(memcap::Collect(dir, nullptr, 0, 0) == 10);
  // Whatever a container writes into its file: a bounded result or an error.
  std::mt19937 rng(7);
  std::string key = memcap::AllocationKey({"fuzz"});
  CHECK(memcap::CreateGrantFile(dir, key, {1u << 20}, "fuzz").ok());
  std::string path = dir + "/" + key + ".memcap";
  for (int it = 0; it < 300; ++it) {
    int fd = open(path.c_str(), O_RDWR);
    CHECK(fd >= 0);
    if (fd < 0) break;
    if (it % 3 == 0) {  // a short or grown file
      int r = ftruncate(fd, static_cast<off_t>(rng() % (300 * 1024)));
      (void)r;
    }
    for (int k = 0; k < 8; ++k) {  // scribble over the header (magic/version kept half the time)
      uint32_t off = rng() % 6200, v = rng();
      if (it % 2 == 0 && off < 8) continue;
      ssize_t w = pwrite(fd, &v, sizeof(v), off);
      (void)w;
    }
    close(fd);
    auto u = memcap::ReadGrant(dir, key);
    if (u.ok()) {
      CHECK(u->used.size() <= 64 && u->cap.size() == u->used.size() && u->peak.size() == u->used.size());
      CHECK(u->ids.empty() || memcap::AllocationKey({u->ids}) == key);
    }
    struct stat st;
    CHECK(stat(path.c_str(), &st) == 0 && st.st_size <= 2 * 150000);  // trimmed when grown
  }
  unlink(path.c_str());
  rmdir(dir.c_str());
  rmdir((std::string(root) + "/amdgpu-dp").c_str());
  rmdir(root);
}

static void TestStringHelpers() {
  g_case = "strings";
  CHECK(Split("a,,b", ',') == std::vector<std::string>({"a", "", "b"}));
  CHECK(Split("", ',') == std::vector<std::string>({""}));
  CHECK(SplitOn("a::b::", "::") == std::vector<std::string>({"a", "b", ""}));
  CHECK(SplitOn("abc", "") == std::vector<std::string>({"abc"}));
  CHECK(Trim(" \t x y \n") == "x y" && Trim("   ").empty());
  CHECK(Join({"a", "b", "c"}, ", ") == "a, b, c" && Join({}, ",").empty());
  CHECK(ToLower("MiXeD-1") == "mixed-1");
  CHECK(StartsWith("abc", "ab") && !StartsWith("a", "ab") && EndsWith("abc", "bc") && !EndsWith("c", "bc"));
  CHECK(ParseInt("-42") == -42 && !ParseInt("") && !ParseInt(" 1") && !ParseInt("1x") &&
        !ParseInt("99999999999999999999"));
  CHECK(ParseUint("18446744073709551615") == UINT64_MAX && !ParseUint("18446744073709551616") &&
        !ParseUint("-1") && !ParseUint("+1") && !ParseUint(""));
  CHECK(ParseBool(" Yes ") == true && ParseBool("off") == false && ParseBool("t") == true && !ParseBool("maybe"));
  CHECK(JsonEscape("a\"b\\c\nd\re\tf") == "a\\\"b\\\\c\\nd\\re\\tf");
  CHECK(JsonEscape(std::string("\x01z", 2)) == "\\u0001z");
  CHECK(PathJoin("/a/", "/b//c/") == "/a/b/c" && PathJoin("", "x") == "x" && PathJoin("/", "") == "/");
  CHECK(BaseName("/a/b/") == "b" && BaseName("c") == "c" && BaseName("/").empty());  // "/": no file name
}

static void TestGrpcCommon() {
  g_case = "grpc-common";
  using adp::grpc::FromGrpcCode;
  using adp::grpc::ToGrpcCode;
  // every status code maps to its gRPC code and back (kNotSupported is
  // UNIMPLEMENTED on the wire)
  for (Code c : {Code::kOk, Code::kInvalidArgument, Code::kNotFound, Code::kAlreadyExists,
                 Code::kFailedPrecondition, Code::kUnavailable, Code::kUnimplemented, Code::kInternal,
                 Code::kDeadlineExceeded, Code::kPermissionDenied})
    CHECK(FromGrpcCode(ToGrpcCode(c)) == c);
  CHECK(ToGrpcCode(Code::kNotSupported) == adp::grpc::kGrpcUnimplemented);
  CHECK(FromGrpcCode(adp::grpc::kGrpcResourceExhausted) == Code::kInternal);  // codes we never send
  std::string framed;
  adp::grpc::FrameMessage(std::string(300, 'x'), &framed);
  CHECK(framed.size() == 305 && framed[0] == 0 && framed[3] == 1 && static_cast<unsigned char>(framed[4]) == 44);
  // grpc-message percent-encoding: printable ASCII but '%' passes; round trip
  std::string msg = "100% done\n\xc3\xa9";
  std::string enc = adp::grpc::PercentEncode(msg);
  CHECK(enc == "100%25 done%0A%C3%A9");
  CHECK(adp::grpc::PercentDecode(enc) == msg);
  CHECK(adp::grpc::PercentDecode("%4") == "%4" && adp::grpc::PercentDecode("%zz") == "%zz" &&
        adp::grpc::PercentDecode("a%41") == "aA");
}

int main() {
  TestLongLogLine();
  TestStringHelpers();
  TestGrpcCommon();
  TestYaml();
  TestConfigFuzz();
  TestReplicaCuRanges();
  TestPodResources();
  TestMemcapUsage();
  TestMetrics();
  TestPrioritize();
  TestStrip();
  TestAdditionalIds();
  TestResourceConfig();
  TestRelayLines();
  TestLedgerGaps();
  TestLedgerResetHistory();
  TestRemoveDrainNames();
  TestDrainSyntax();
  TestRemoteScan();
  TestProto();
  TestTopology();
  TestHierarchicalMatchesOracle();
  TestConfig();
  TestConfigPrecedenceProperty();
  TestGrpcLoopback(true);
  TestGrpcLoopback(false);
  TestH2Fuzz();
  TestPreferredViewFuzz();
  TestGrpcMultiLoop();
  printf("%d checks, %d failed\n", g_checks, g_failed);
  return g_failed ? 1 : 0;
}
