// amdgpu-dp-probe: validate the GPU(s) a container was given.
//
//   amdgpu-dp-probe [--list] [--device N] [--bytes B] [--iters I]
//                   [--expect-xcds X] [--expect-cus C] [--min-gbps G]
//                   [--p2p [--min-p2p-gbps P]] [--mfma [--min-tflops T]]
//                   [--census [--expect-cus-seen C]] [--latency N] [--aggressor SECONDS]
//                   [--check-grant]
//
// Runs the visibility probe (visibility_probe.hip) on every visible HIP device
// (or one) and prints one JSON line per device. Exits non-zero when a device
// fails its checksum or does not have the expected shape -- e.g. a pod that
// requested one CPX partition must see exactly 1 XCD / 32 CUs:
//   amdgpu-dp-probe --expect-xcds 1 --expect-cus 32
// See examples/pods/pod-validate.yml. --p2p additionally measures xGMI peer-read
// bandwidth between every pair of the pod's GPUs (a multi-GPU pod placed by the
// xGMI-aware preferred allocation should see every pair connected); it fails if a
// pair has no peer access or is below --min-p2p-gbps. --mfma runs the bf16
// matrix cores flat out (v_mfma_f32_32x32x16_bf16) and checks every result is
// exact; it fails on a wrong element or a rate below --min-tflops. --census
// prints which XCDs/CUs the process's queues can use (the CU share of a
// CU-partitioned replica, HSA_CU_MASK); --expect-cus-seen checks that count.
// --latency N times N launches of a small kernel (what a latency-sensitive pod
// sees); --aggressor S saturates the GPU for S seconds (a noisy neighbour).
// --check-grant checks an enforced memory-unit grant (AMD_GPU_MEMORY_LIMIT_MIB,
// --enforce-memory-units): each device reports its grant as its memory,
// refuses an allocation past it and allows one of half of it.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

extern "C" int adp_probe_device_count();
extern "C" int adp_probe_list(char* out, int len);
extern "C" int adp_probe_run(int device, unsigned long long bytes, int iters, char* out, int len);
extern "C" int adp_probe_p2p(int ndev, unsigned long long bytes, int iters, char* out, int len);
extern "C" int adp_probe_mfma(int device, int iters, char* out, int len);
extern "C" int adp_probe_census(int device, char* out, int len);
extern "C" int adp_probe_latency(int device, int n, char* out, int len);
extern "C" int adp_probe_aggressor(int device, double seconds, char* out, int len);
extern "C" int adp_probe_grant(int device, unsigned long long grant_mib, char* out, int len);

namespace {

long JsonInt(const char* json, const char* key) {
  std::string k = std::string("\"") + key + "\": ";
  const char* p = strstr(json, k.c_str());
  return p ? strtol(p + k.size(), nullptr, 10) : -1;
}

double JsonDouble(const char* json, const char* key) {
  std::string k = std::string("\"") + key + "\": ";
  const char* p = strstr(json, k.c_str());
  return p ? strtod(p + k.size(), nullptr) : -1.0;
}

}  // namespace

int main(int argc, char** argv) {
  int device = -1, iters = 5;
  unsigned long long bytes = 256ull << 20;
  long expect_xcds = -1, expect_cus = -1;
  double min_gbps = -1, min_p2p_gbps = -1, min_tflops = -1;
  long expect_cus_seen = -1;
  int latency = 0;
  double aggressor = 0;
  bool list = false, p2p = false, mfma = false, census = false, check_grant = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* { return i + 1 < argc ? argv[++i] : "0"; };
    if (a == "--list") list = true;
    else if (a == "--device") device = atoi(next());
    else if (a == "--bytes") bytes = strtoull(next(), nullptr, 10);
    else if (a == "--iters") iters = atoi(next());
    else if (a == "--expect-xcds") expect_xcds = atol(next());
    else if (a == "--expect-cus") expect_cus = atol(next());
    else if (a == "--min-gbps") min_gbps = atof(next());
    else if (a == "--p2p") p2p = true;
    else if (a == "--min-p2p-gbps") min_p2p_gbps = atof(next());
    else if (a == "--mfma") mfma = true;
    else if (a == "--min-tflops") min_tflops = atof(next());
    else if (a == "--census") census = true;
    else if (a == "--expect-cus-seen") expect_cus_seen = atol(next());
    else if (a == "--latency") latency = atoi(next());
    else if (a == "--aggressor") aggressor = atof(next());
    else if (a == "--check-grant") check_grant = true;
    else {
      fprintf(stderr, "usage: %s [--list] [--device N] [--bytes B] [--iters I] [--expect-xcds X] "
                      "[--expect-cus C] [--min-gbps G] [--p2p [--min-p2p-gbps P]] [--mfma [--min-tflops T]] "
                      "[--census [--expect-cus-seen C]] [--latency N] [--aggressor SECONDS] [--check-grant]\n",
              argv[0]);
      return 2;
    }
  }
  static char buf[1 << 16];
  if (list) {
    int rc = adp_probe_list(buf, sizeof(buf));
    printf("%s\n", buf);
    return rc ? 1 : 0;
  }
  int n = adp_probe_device_count();
  if (n <= 0) {
    fprintf(stderr, "no HIP devices visible (is /dev/kfd + a render node mounted?)\n");
    return 1;
  }
  int failures = 0;
  for (int d = (device < 0 ? 0 : device); d < (device < 0 ? n : device + 1); ++d) {
    if (aggressor > 0 || latency > 0) {
      int arc = aggressor > 0 ? adp_probe_aggressor(d, aggressor, buf, sizeof(buf))
                              : adp_probe_latency(d, latency, buf, sizeof(buf));
      printf("%s\n", buf);
      if (arc != 0) ++failures;
      continue;
    }
    if (check_grant) {
      // The grant of the d-th device of the container: AMD_GPU_MEMORY_LIMIT_MIB, in HIP order.
      const char* lim = getenv("AMD_GPU_MEMORY_LIMIT_MIB");
      const char* p = lim;
      for (int k = 0; p && k < d; ++k) {
        p = strchr(p, ',');
        if (p) ++p;
      }
      unsigned long long grant = p ? strtoull(p, nullptr, 10) : 0;
      if (!grant) {
        printf("{\"device\": %d, \"error\": \"no AMD_GPU_MEMORY_LIMIT_MIB entry for this device\"}\n", d);
        ++failures;
        continue;
      }
      int grc = adp_probe_grant(d, grant, buf, sizeof(buf));
      printf("%s\n", buf);
      if (grc != 0) ++failures;
      continue;
    }
    if (census) {
      int crc = adp_probe_census(d, buf, sizeof(buf));
      printf("%s\n", buf);
      if (crc != 0) ++failures;
      else if (expect_cus_seen >= 0 && JsonInt(buf, "cus_seen") != expect_cus_seen) ++failures;
      continue;
    }
    int rc = adp_probe_run(d, bytes, iters, buf, sizeof(buf));
    printf("%s\n", buf);
    if (rc != 0) { ++failures; continue; }
    if (expect_xcds >= 0 && JsonInt(buf, "xccs_seen") != expect_xcds) ++failures;
    if (expect_cus >= 0 && JsonInt(buf, "cus") != expect_cus) ++failures;
    if (min_gbps >= 0 && JsonDouble(buf, "hbm_copy_gbps") < min_gbps) ++failures;
    if (mfma) {
      int mrc = adp_probe_mfma(d, 1 << 14, buf, sizeof(buf));
      printf("%s\n", buf);
      if (mrc != 0) ++failures;
      if (min_tflops >= 0 && JsonDouble(buf, "bf16_tflops") < min_tflops) ++failures;
    }
  }
  if (p2p) {
    int rc = adp_probe_p2p(n, bytes, iters, buf, sizeof(buf));
    printf("%s\n", buf);
    if (rc != 0 || strstr(buf, "no-peer-access")) ++failures;
    if (min_p2p_gbps >= 0) {
      for (const char* q = strstr(buf, "\"gbps\": "); q; q = strstr(q + 1, "\"gbps\": "))
        if (strtod(q + 8, nullptr) < min_p2p_gbps) ++failures;
    }
  }
  fflush(stdout);
  return failures ? 1 : 0;
}
