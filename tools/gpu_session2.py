"""GPU session 2: probe bandwidth sweep, real-hardware daemon log (health events),
cold-start registration latency, bench configs. Writes gpurun_out/s2/*."""
import json, os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "gpurun_out", "s2")
os.makedirs(OUT, exist_ok=True)
from k8s_gpu_sharing_plugin_amd.ops import probe
from k8s_gpu_sharing_plugin_amd.utils import harness

def dump(name, obj):
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(obj, f, indent=1)
    print(name, "written", flush=True)

step = sys.argv[1]
if step == "sweep":
    res = probe.bw_sweep(0, 1 << 30, 10)
    res.sort(key=lambda r: -r["gbps"])
    dump("bw_sweep.json", res)
    print(res[:5])
elif step == "daemon":
    # cold start: exec -> registration seen by the stub kubelet, 5 runs
    lat = []
    for i in range(5):
        d = harness.scratch_dir("adps2")
        k = harness.NativeKubelet(os.path.join(d, "kubelet.sock")).start()
        t0 = time.perf_counter()
        dm = harness.Daemon(d, real_smi=True, env={"DP_HEALTH_POLL_MS": "500"}).start()
        k.wait(lambda e: e.get("event") == "register", 30)
        t1 = time.perf_counter()
        k.wait(lambda e: e.get("event") == "devices", 30)
        t2 = time.perf_counter()
        lat.append({"register_ms": (t1 - t0) * 1e3, "first_law_ms": (t2 - t0) * 1e3})
        time.sleep(1.5 if i == 0 else 0.1)
        dm.stop(); k.stop()
        if i == 0:
            with open(os.path.join(OUT, "daemon_real.log"), "w") as f:
                f.write(dm.log())
    dump("cold_start.json", lat)
    print(lat)
