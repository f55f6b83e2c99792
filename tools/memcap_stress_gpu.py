#!/usr/bin/env python3
"""The HBM-cap shim under concurrency on real HIP: N PyTorch processes of one
"container" share one daemon-style grant (a read-only grant file) and churn
random tensors (allocate 64-1024 MiB, free at random, PyTorch's caching
allocator on) for --seconds. Meanwhile this process samples what the amdgpu
driver says each worker holds (DRM fdinfo `drm-resident-vram` of its render
descriptors, the source of the daemon's driver-side check) every 20 ms.

The grant holds if the driver's sum over the workers never exceeds the grant
plus the HIP runtime's own per-process allocations (code objects, queues,
scratch -- never requested through hipMalloc), measured per worker after it
loaded its kernels and before its first tensor, plus --slack-mib per process
for what the runtime adds later and for blocks PyTorch freed (the shim gives
their bytes back at hipFree) that the driver has not released yet: on a
refusal PyTorch empties its cache and retries at once. --compare-uncapped runs
the same churn without the shim, whose peak must pass that bound. Prints one JSON object; exit 1 if the grant was exceeded or no
allocation was ever refused (then the test did not reach the cap).

  python tools/memcap_stress_gpu.py [--workers 4] [--grant-mib 8000] [--seconds 30]
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

WORKER = r"""
import json, os, random, sys, time
import torch
seed, seconds = int(sys.argv[1]), float(sys.argv[2])
rng = random.Random(seed)
torch.cuda.init()
w = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")  # load the kernels this loop uses
w.fill_(1)
w[:: 1 << 10].fill_(2)
torch.cuda.synchronize()
del w
torch.cuda.empty_cache()
print("ready", flush=True)
sys.stdin.readline()  # start together
held, granted, refused, freed = [], 0, 0, 0
t_end = time.time() + seconds
while time.time() < t_end:
    if held and (rng.random() < 0.45 or len(held) > 24):
        held.pop(rng.randrange(len(held)))
        freed += 1
        continue
    mib = rng.choice((64, 128, 256, 512, 1024))
    try:
        t = torch.empty(mib << 20, dtype=torch.uint8, device="cuda")
        t[:: 1 << 20].fill_(1)  # touch it
        held.append(t)
        granted += 1
    except torch.OutOfMemoryError:
        refused += 1
        if held:
            held.pop(rng.randrange(len(held)))
torch.cuda.synchronize()
print(json.dumps({"granted": granted, "refused": refused, "freed": freed,
                  "reserved_mib_end": torch.cuda.memory_reserved() >> 20,
                  "total_mib": torch.cuda.get_device_properties(0).total_memory >> 20}), flush=True)
"""


def driver_bytes(pid):
    """HBM the driver counts for `pid` (sum over its render-node clients)."""
    total, seen = 0, set()
    for fd in glob.glob(f"/proc/{pid}/fd/*"):
        try:
            if not os.readlink(fd).startswith("/dev/dri/renderD"):
                continue
            info = open(f"/proc/{pid}/fdinfo/{os.path.basename(fd)}").read()
        except OSError:
            continue
        fields = dict(ln.split(":", 1) for ln in info.splitlines() if ":" in ln)
        client = (fields.get("drm-pdev", "").strip(), fields.get("drm-client-id", "").strip())
        if client in seen:
            continue
        seen.add(client)
        v = (fields.get("drm-resident-vram") or fields.get("drm-memory-vram") or "0").split()
        mul = {"KiB": 1 << 10, "MiB": 1 << 20, "GiB": 1 << 30}.get(v[1] if len(v) > 1 else "", 1)
        total += int(v[0]) * mul
    return total


def run_workers(a, env):
    """Starts the workers, samples the driver's count for them while they
    churn; returns (peak bytes, runtime baseline per pid, worker results, samples)."""
    procs = [subprocess.Popen([sys.executable, "-c", WORKER, str(i), str(a.seconds)], env=env, stdin=subprocess.PIPE,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for i in range(a.workers)]
    try:
        for p in procs:
            line = p.stdout.readline().strip()
            if line != "ready":
                raise SystemExit("worker failed to start: " + p.stderr.read()[-2000:])
        base = {p.pid: driver_bytes(p.pid) for p in procs}  # runtime allocations before any tensor
        for p in procs:
            p.stdin.write("go\n")
            p.stdin.flush()
        samples, peak, t0 = 0, 0, time.time()
        while any(p.poll() is None for p in procs) and time.time() - t0 < a.seconds + 120:
            s = sum(driver_bytes(p.pid) for p in procs if p.poll() is None)
            peak = max(peak, s)
            samples += 1
            time.sleep(0.02)
        outs = []
        for p in procs:
            out, err = p.communicate(timeout=120)
            if p.returncode != 0:
                raise SystemExit(f"worker exited {p.returncode}: {err[-2000:]}")
            outs.append(json.loads(out.strip().splitlines()[-1]))
        return peak, base, outs, samples
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--grant-mib", type=int, default=8000)
    ap.add_argument("--seconds", type=float, default=30)
    ap.add_argument("--slack-mib", type=int, default=256)
    ap.add_argument("--compare-uncapped", action="store_true",
                    help="also run the same workers without the shim (their peak must pass the bound)")
    a = ap.parse_args()
    from k8s_gpu_sharing_plugin_amd import BUILD_DIR
    gdir = tempfile.mkdtemp(prefix="adpgrant")
    with open(os.path.join(gdir, "0"), "w") as f:
        f.write(f"{a.grant_mib}\n")
    os.chmod(os.path.join(gdir, "0"), 0o444)
    key = f"stress-{os.getpid()}"
    preload = " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), os.path.join(BUILD_DIR, "libadp_memcap.so")) if x)
    env = {**os.environ, "LD_PRELOAD": preload, "ADP_MEMCAP_GRANT_DIR": gdir, "ADP_MEMCAP_KEY": key}
    env.pop("AMD_GPU_MEMORY_LIMIT_MIB", None)
    result = {"workers": a.workers, "grant_mib": a.grant_mib, "seconds": a.seconds, "slack_mib_per_process": a.slack_mib}
    try:
        peak, base, outs, samples = run_workers(a, env)
    finally:
        for f in glob.glob(f"/dev/shm/adp-memcap-key-{key}-*"):
            os.unlink(f)
    bound = (a.grant_mib << 20) + sum(base.values()) + (a.workers * a.slack_mib << 20)
    result.update({
        "driver_samples": samples,
        "driver_peak_mib": round(peak / 1048576, 1),
        "runtime_baseline_mib": {str(k): round(v / 1048576, 1) for k, v in base.items()},
        "bound_mib": bound >> 20,
        "peak_over_grant_mib": round(peak / 1048576 - a.grant_mib, 1),
        "per_worker": outs,
        "granted": sum(o["granted"] for o in outs),
        "refused": sum(o["refused"] for o in outs),
        "reported_total_mib": sorted({o["total_mib"] for o in outs}),
    })
    result["held"] = peak <= bound
    result["ok"] = result["held"] and result["refused"] > 0 and result["reported_total_mib"] == [a.grant_mib]
    if a.compare_uncapped:
        plain = {k: v for k, v in os.environ.items() if k not in ("AMD_GPU_MEMORY_LIMIT_MIB",)}
        upeak, _, uouts, _ = run_workers(a, plain)
        result["uncapped_peak_mib"] = round(upeak / 1048576, 1)
        result["uncapped_refused"] = sum(o["refused"] for o in uouts)
        result["ok"] = result["ok"] and upeak > bound  # the same churn does pass the bound without the shim
    print(json.dumps(result), flush=True)
    return 0 if result["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
