"""Multi-rank pod-churn benchmark of the device plugin.

One process per GPU. ``python bench.py --gpus N`` with N > 1 and no launcher
starts the N ranks itself (``torch.distributed.run`` as a child process,
before this process touches the GPU) and exits with the job's status; under a
launcher every rank runs ``run()``.

Every rank names its own GPU by PCI address (HIP device ``LOCAL_RANK`` on a
GPU box; GPU ``LOCAL_RANK`` of the 8-GPU node model on the mock), the addresses
are all-gathered, and rank 0 starts the native stub kubelet and the real
``amdgpu-device-plugin`` daemon serving exactly those GPUs (``--devices
<bdf>,...``: amdsmi's enumeration order and HIP's can differ, and amdsmi ignores
``HIP_VISIBLE_DEVICES``). Rank 0 records the node as the daemon's inventory code
sees it -- compute/memory mode and xGMI links down per GPU, the N x N link
type / hops / weight matrix -- and one real GetPreferredAllocation(k=min(4,N))
answer over the whole served set. Then each rank plays kubelet for the devices
of its own GPU: a "pod" is GetPreferredAllocation(free, 1) + Allocate(chosen)
on one persistent gRPC connection, retiring the oldest pod when its share of
the node is full. One step = ``pods_per_step`` pods per rank. The K timed steps
run between barrier + device-synchronize brackets; the job reports the max
over ranks.

After the timed region each rank runs the HIP probe on the GPU its kubelet
client admitted (real hardware only) to show the allocated device is usable
and has the advertised shape. The JSON records the RCCL world as
torch.distributed saw it, the backend, and per rank the BDF it owns, the BDFs
it admitted and the BDF the probe ran on.

Reference: the kubelet-facing calls timed here are
/root/reference/cmd/nvidia-device-plugin/server.go:268-353.
"""

import json
import os
import time

METRIC = "allocatable amd.com/gpu count + Allocate() p50 latency at 1/2/4/8 MI355X"

# name -> (partition strategy, resource config, description)
CONFIGS = {
    "spx-none": ("none", "", "{n}xMI355X SPX, partitionStrategy=none, one amd.com/gpu:1 pod per GPU"),
    "timeslice4": ("none", "gpu:gpu:4", "{n}xMI355X SPX, time-slice sharing 4 replicas/GPU ({p} concurrent pods)"),
    "auto-mem": ("none", "gpu:gpu-mem-gb:-1", "{n}xMI355X SPX, auto memory replicas (gpu-mem-gb)"),
    # auto-mem with the grant enforced in the pod and reported on /metrics: each
    # Allocate() also writes the grant's accounting file (memcap/usage.h).
    "auto-mem-enforced": ("none", "gpu:gpu-mem-gb:-1",
                          "{n}xMI355X SPX, auto memory replicas, HBM-cap shim + per-grant accounting files"),
    "cpx-single": ("single", "", "{n}xMI355X CPX, partitionStrategy=single, 8 partitions/GPU"),
    # BASELINE config 5: always an 8-GPU node (6 SPX + 2 CPX, node model); one
    # kubelet client admits amd.com/gpu:4 pods, so every admission runs the
    # xGMI/NUMA-aware GetPreferredAllocation over the free SPX GPUs.
    "mixed-gpu4": ("mixed", "", "8xMI355X mixed 6 SPX + 2 CPX, xGMI-aware GetPreferredAllocation for amd.com/gpu:4 pods"),
}
POD_SIZE = {"mixed-gpu4": 4}


def _env_int(name, default):
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


def _sync(torch_mod):
    if torch_mod is not None and torch_mod.cuda.is_available():
        torch_mod.cuda.synchronize()


def _server_stats(daemon):
    """Asks the daemon for its RPC counters (SIGUSR1) and parses the log line."""
    import signal
    if daemon is None:
        return {}
    try:
        before = daemon.log().count("stats: {")
        daemon.signal(signal.SIGUSR1)
        text = daemon.wait_log("stats: {", timeout=5, count=before + 1)
        line = [ln for ln in text.splitlines() if "stats: {" in ln][-1]
        return json.loads(line.split("stats: ", 1)[1])
    except Exception:
        return {}


def _grpcio_allocate_p50(socket_path, device=None, calls=300):
    """Allocate p50 through grpcio (gRPC C-core + Python): an independent gRPC
    client stack, next to the native client's number."""
    try:
        from ..utils import kubelet
        c = kubelet.PluginClient(socket_path)
        q, call = c.watch()
        devs = q.get(timeout=5).devices
        call.cancel()
        ids = [d.ID for d in devs]
        dev = next((i for i in ids if device and i.startswith(device)), ids[0])
        lat = []
        for i in range(calls + 50):
            t = time.perf_counter()
            c.allocate([dev])
            if i >= 50:
                lat.append((time.perf_counter() - t) * 1e6)
        c.close()
        lat.sort()
        return round(lat[len(lat) // 2], 2)
    except Exception:
        return None


def _residency(before, after):
    """The daemon's read -> reply-written time (gRPC loop residency, 100 ns bins
    from the SIGUSR1 stats) of the unary calls served between two stats
    snapshots: p50/p99 in us, or None without samples."""
    if not after or "residency_100ns" not in after:
        return None
    b = {k: v for k, v in (before or {}).get("residency_100ns", [])}
    counts = sorted((k, v - b.get(k, 0)) for k, v in after["residency_100ns"] if v > b.get(k, 0))
    total = sum(v for _, v in counts)
    if not total:
        return None

    def q(x):
        rank, seen = int(x * (total - 1)) + 1, 0
        for k, v in counts:
            seen += v
            if seen >= rank:
                return round((k + 1) / 10, 1)

    return {"samples": total, "p50_us": q(0.5), "p99_us": q(0.99)}


def _cpu_group(cpu, rel):
    """First CPU of `cpu`'s sysfs group (cache/index3/shared_cpu_list: its L3;
    topology/thread_siblings_list: its core), -1 if unknown."""
    try:
        with open(f"/sys/devices/system/cpu/cpu{cpu}/{rel}") as f:
            first = f.read().strip().split(",")[0]
        return int(first.split("-")[0])
    except (OSError, ValueError):
        return -1


def _placement(client_cpus, loops_before, loops_after):
    """Where the timed client and the gRPC loop that served it ran (diagnosis
    of the run's latency mode): the client's CPUs, the loop busiest during the
    timed region (busy-iteration counts before/after it) and its last CPU, and
    whether the two shared a core, an L3, or neither."""
    cpus = {int(c): n for c, n in (client_cpus or {}).items()}
    before = [b for _, b in (loops_before or [])]
    loops = [(c, b - (before[i] if i < len(before) else 0)) for i, (c, b) in enumerate(loops_after or [])]
    out = {"client_cpus": cpus, "loops_during_timed": loops}
    if cpus and loops and max(b for _, b in loops) > 0:
        client = max(cpus, key=cpus.get)
        loop = max(loops, key=lambda x: x[1])[0]
        same_core = _cpu_group(client, "topology/thread_siblings_list") == _cpu_group(loop, "topology/thread_siblings_list")
        same_l3 = _cpu_group(client, "cache/index3/shared_cpu_list") == _cpu_group(loop, "cache/index3/shared_cpu_list")
        out.update({"client_cpu": client, "busiest_loop_cpu": loop,
                    "relation": "same-core" if same_core else "same-l3" if same_l3 else "other-l3"})
    return out


def _grpc_go_shaped(socket_path, pod_size, rank, world, warm, pods, owned=None):
    """Allocate / GetPreferredAllocation latency with the client frame pattern of
    the kubelet's grpc-go transport (grpc::Channel::EmulateGrpcGo): what the
    plugin costs a real kubelet, next to the plain native-client headline."""
    from ..utils import native
    try:
        c = native.ChurnClient(socket_path, pod_size=pod_size, rank=rank, world=world, grpc_go=True, owned=owned)
        c.run(warm, record=False)
        c.reset()
        c.run(pods, record=True)
        s = c.stats()
        c.close()
        return {"pods": s["pods"], "bdp_pings": s["bdp_pings"], "allocate": s["allocate"],
                "preferred": s["preferred"], "cpus": s.get("cpus")}
    except Exception as e:  # reported, not fatal for the headline
        return {"error": str(e)}


def _node_snapshot(real, fixture, devices=None):
    """The served GPUs as the daemon's inventory code enumerates them (the same
    BuildSnapshot, through libadp_capi), or {} when enumeration fails."""
    from .. import MOCK_LIB
    from ..utils import native
    try:
        if real:
            return native.snapshot(devices=devices)
        import tempfile
        from ..models import fixtures
        os.environ["AMDSMI_MOCK_FIXTURE"] = fixtures.write(fixture, tempfile.mkdtemp(prefix="adpbdf"))
        return native.snapshot(MOCK_LIB, devices=devices)
    except Exception:
        return {}


def _bdf_map(snap):
    """Device ID (GPU or partition UUID) -> PCI address of its GPU."""
    out = {}
    for g in snap.get("gpus", []):
        out[g["uuid"]] = g["bdf"]
        for p in g["partitions"]:
            out[p["uuid"]] = g["bdf"]
    return out


def _device_order(snap, rank_bdfs):
    """The three orders of the served GPUs: amdsmi's enumeration, KFD topology
    node (what the plugin orders every per-device container list by: HSA_CU_MASK
    agents, AMD_GPU_MEMORY_* and grant/<i>) and HIP's -- rank r binds HIP device
    r, so rank_bdfs is HIP's order of the first N devices. On a multi-GPU node
    this records whether HIP really follows KFD node order."""
    gpus = snap["gpus"]
    amdsmi = [g["bdf"] for g in gpus]
    known = all(g.get("kfd_node") is not None for g in gpus)
    kfd = [g["bdf"] for g in sorted(gpus, key=lambda g: g["kfd_node"])] if known else None
    hip = list(dict.fromkeys(rank_bdfs))
    out = {"amdsmi_order": amdsmi, "kfd_order": kfd, "hip_order": hip,
           "kfd_order_differs_from_amdsmi": None if kfd is None else kfd != amdsmi}
    if sorted(hip) == sorted(amdsmi):  # HIP's view of exactly the served set
        out["hip_order_is_kfd_order"] = None if kfd is None else hip == kfd
        out["hip_order_is_amdsmi_order"] = hip == amdsmi
    return out


def _container_view(snap):
    """HIP's numbering as a container sees it, on real GPUs: a process that may
    open only some render nodes (libadp_devcgroup_sim.so returns EPERM for the
    others, as a container's device cgroup does) lists its HIP devices. For
    every served GPU together, and for the last and first GPU requested in
    reverse order, the listed PCI addresses must come in KFD-node order -- the
    order the plugin gives every per-device container list in. Reported, never
    fatal."""
    import subprocess
    from .. import BUILD_DIR
    from ..utils.build import PROBE_EXE
    sim = os.path.join(BUILD_DIR, "libadp_devcgroup_sim.so")
    gpus = snap.get("gpus") or []
    if not gpus or any(g.get("kfd_node") is None for g in gpus) or not os.path.exists(PROBE_EXE):
        return {"skipped": "no KFD nodes or probe"}
    render = {g["bdf"]: [p["render"] for p in g["partitions"] if p.get("render")] for g in gpus}
    kfd = [g["bdf"] for g in sorted(gpus, key=lambda g: g["kfd_node"])]

    def hip_list(bdfs):
        env = {k: v for k, v in os.environ.items() if k not in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                                  "CUDA_VISIBLE_DEVICES")}
        env["LD_PRELOAD"] = " ".join(x for x in (env.get("LD_PRELOAD", ""), sim) if x)
        env["ADP_DEVCGROUP_ALLOW"] = ":".join(["/dev/kfd"] + [r for b in bdfs for r in render[b]])
        r = subprocess.run([PROBE_EXE, "--list"], env=env, capture_output=True, text=True, timeout=120)
        devs = json.loads(r.stdout.strip().splitlines()[-1])
        return [d["pci"] for d in devs] if isinstance(devs, list) else devs

    cases = [kfd] + ([[kfd[-1], kfd[0]]] if len(kfd) >= 2 else [])
    out = {"cases": []}
    try:
        for req in cases:
            want = [b for b in kfd if b in req]
            out["cases"].append({"granted": req, "kfd_order": want, "hip": hip_list(req)})
        out["hip_order_is_kfd_order"] = all(c["hip"] == c["kfd_order"] for c in out["cases"])
    except Exception as e:  # diagnostic only
        out["error"] = str(e)
    return out


def _topology(snap, rank_bdfs):
    """The node block of the JSON: what GetPreferredAllocation scores against."""
    if not snap:
        return {"error": "enumeration failed"}
    return {
        "amdsmi": snap.get("smi_version"),
        "rank_bdfs": rank_bdfs,
        "served_bdfs": [g["bdf"] for g in snap["gpus"]],
        "device_order": _device_order(snap, rank_bdfs),
        "gpus": [{"bdf": g["bdf"], "uuid": g["uuid"], "product": g.get("market_name"),
                  "compute_mode": g["compute_mode"], "memory_mode": g["memory_mode"],
                  "partitions": len(g["partitions"]), "numa": g["numa"], "vram_mib": g["vram_mib"],
                  "kfd_node": g.get("kfd_node"),
                  "hip_id": (g["partitions"][0].get("hip_id") if g["partitions"] else None),
                  "xgmi_links_down": g["xgmi_links_down"]} for g in snap["gpus"]],
        # rows/columns in served_bdfs order
        "link_types": snap.get("link_types"),
        "hops": snap.get("hops"),
        "weights": snap.get("weights"),
        "link_class": snap.get("links"),  # inventory::LinkClass the allocator scores
    }


def _rank_bdf(real, torch_mod, local_rank, fixture):
    """PCI address of this rank's GPU: HIP device `local_rank` on a GPU box
    (what torch.cuda.set_device binds), GPU `local_rank` of the node model on the mock."""
    if real:
        p = torch_mod.cuda.get_device_properties(local_rank)
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    # ADP_BENCH_MOCK_GPUS="5,2": rank r owns node GPU list[r] -- a job that was
    # given some of the node's GPUs, in an order that is not amdsmi's.
    order = [int(x) for x in os.environ.get("ADP_BENCH_MOCK_GPUS", "").split(",") if x.strip()]
    return fixture["gpus"][order[local_rank] if order else local_rank]["bdf"]


def _preferred_probe(socket_path, k, bdf_of):
    """One GetPreferredAllocation(k) over every advertised device, all free,
    through grpcio (an independent gRPC stack): the placement a k-GPU pod gets."""
    try:
        from ..utils import kubelet
        c = kubelet.PluginClient(socket_path)
        q, call = c.watch()
        ids = [d.ID for d in q.get(timeout=5).devices if d.health == "Healthy"]
        call.cancel()
        k = min(k, len(ids))
        resp = c.preferred(ids, (), k)
        c.close()
        got = list(resp.container_responses[0].deviceIDs)
        from ..utils import native
        return {"k": k, "available": len(ids), "device_ids": got,
                "bdfs": [bdf_of.get(i, bdf_of.get(native.strip_replicas([i])[0], "?")) for i in got]}
    except Exception as e:  # reported, not fatal for the headline
        return {"error": str(e)}


def run(gpus=1, steps=20, warmup=2, pods_per_step=100, config="spx-none", force_mock=False,
        probe=True, log=print):
    try:
        import torch
        import torch.distributed as dist
    except ImportError:  # pragma: no cover - torch is part of the image
        torch, dist = None, None
    from ..models import fixtures
    from ..utils import harness, native

    rank = _env_int("RANK", 0)
    world = _env_int("WORLD_SIZE", 1)
    local_rank = _env_int("LOCAL_RANK", 0)
    if world != gpus:
        raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={world}")
    have_gpu = torch is not None and torch.cuda.is_available()
    real = have_gpu and not force_mock
    if real and torch.cuda.device_count() < gpus:
        raise SystemExit(f"--gpus {gpus} but only {torch.cuda.device_count()} GPU(s) are visible to HIP")
    # A process group whenever a launcher started us (torchrun sets MASTER_ADDR),
    # even with one rank: the 1-rank torchrun run then exercises the same RCCL
    # init + object collectives the driver's multi-GPU run uses.
    use_dist = dist is not None and (world > 1 or ("MASTER_ADDR" in os.environ and "RANK" in os.environ))
    if use_dist:
        # RCCL between GPU ranks; gloo when the run is on the mock (no GPU, or
        # --mock on a GPU box: then no rank touches the device at all).
        backend = "nccl" if real else "gloo"
        if real:
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend=backend)
    sync = _sync if real else (lambda _t: None)

    strategy, rc, desc = CONFIGS[config]
    mode = "CPX" if config == "cpx-single" else "SPX"
    # The mock plays a whole 8-GPU node (as on the driver's node, the job may
    # own only some of its GPUs); mixed-gpu4 is BASELINE config 5's fixed node.
    if config == "mixed-gpu4":
        if real or world != 1:
            raise SystemExit("mixed-gpu4 runs on the 8-GPU node model with one client (--mock, 1 rank)")
        fx = fixtures.node(8, ["SPX"] * 6 + ["CPX"] * 2, memory="NPS1")
    else:
        fx = None if real else fixtures.node(max(8, gpus), mode, memory="NPS2" if mode == "CPX" else "NPS1")
    my_bdf = _rank_bdf(real, torch, local_rank, fx)
    rank_bdfs = [my_bdf]
    if use_dist:
        rank_bdfs = [None] * world
        dist.all_gather_object(rank_bdfs, my_bdf)
    daemon = kub = None
    info = {}
    info_snap = {}
    try:
        if rank == 0:
            d = harness.scratch_dir("adpbench")
            kub = harness.NativeKubelet(os.path.join(d, "kubelet.sock")).start()
            # (ranks on compute partitions of one GPU share its address: served once)
            served = None if config == "mixed-gpu4" else list(dict.fromkeys(rank_bdfs))
            args = ["--partition-strategy", strategy]
            if served:
                args += ["--devices", ",".join(served)]
            if rc:
                args += ["--resource-config", rc]
            if config == "auto-mem-enforced":
                from .. import BUILD_DIR
                args += ["--enforce-memory-units", "--memcap-lib", os.path.join(BUILD_DIR, "libadp_memcap.so"),
                         "--metrics-addr", "127.0.0.1:0"]
            daemon = harness.Daemon(d, fx, args=args, real_smi=real,
                                    env={"DP_HEALTH_POLL_MS": "0", "ADP_LOG_LEVEL": "warn"}).start()
            # The measured resource is amd.com/gpu (mixed registers partition resources too).
            reg = kub.wait(lambda e: e.get("event") == "register" and
                           (config not in POD_SIZE or e.get("resource", "").endswith("/gpu")), 20)
            devs = kub.wait(lambda e: e.get("event") == "devices" and e.get("resource") == reg["resource"], 20)
            snap = _node_snapshot(real, fx, served)
            info_snap = snap
            bdf_of = _bdf_map(snap)
            sock = os.path.join(d, reg["endpoint"])
            info = {"socket": sock, "resource": reg["resource"],
                    "allocatable": devs["healthy"], "advertised": devs["total"], "scratch": d,
                    "bdf_of": bdf_of, "topology": _topology(snap, rank_bdfs),
                    "preferred_k": _preferred_probe(sock, min(4, len(snap.get("gpus", [])) or 1), bdf_of)}
        if use_dist:
            box = [info]
            dist.broadcast_object_list(box, src=0)
            info = box[0]

        # This rank churns the devices of its own GPU (every device when one
        # client serves a multi-GPU pod size).
        owned = None
        if config not in POD_SIZE:
            owned = sorted(i for i, b in info["bdf_of"].items() if b == my_bdf)
            if not owned:
                raise SystemExit(f"rank {rank}: the daemon serves no device on {my_bdf}")
        # Diagnostic (ADP_BENCH_PRE_CLIENT=native|grpc-go): a throw-away churn of
        # 2000 pods on another connection before the timed client's, to tell
        # "the first client of a run is slower" from "this client kind is slower".
        pre = os.environ.get("ADP_BENCH_PRE_CLIENT")
        if pre:
            pc = native.ChurnClient(info["socket"], pod_size=POD_SIZE.get(config, 1), rank=rank, world=world,
                                    owned=owned, grpc_go=pre == "grpc-go")
            pc.run(2000, record=False)
            pc.close()
        client = native.ChurnClient(info["socket"], pod_size=POD_SIZE.get(config, 1), rank=rank, world=world,
                                    owned=owned)
        client.run(max(1, warmup) * pods_per_step, record=False)
        client.reset()

        # (1 rank: the loops' placement counters before the timed region, to
        # find the loop that serves it; outside the timing)
        st_before = _server_stats(daemon) if world == 1 else {}
        loops_before = st_before.get("loop_cpus")
        if use_dist:
            dist.barrier()
        sync(torch)
        t0 = time.perf_counter()
        for _ in range(steps):
            client.run(pods_per_step, record=True)
        sync(torch)
        if use_dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        st_timed = _server_stats(daemon) if world == 1 else {}
        loops_after = st_timed.get("loop_cpus")
        stats = client.stats()
        stats["elapsed_s"] = elapsed
        client.close()
        # After the timed region: the same churn with the kubelet's grpc-go frame
        # pattern (a BDP PING per response, grpc-go user-agent) ...
        stats["grpc_go_shaped"] = _grpc_go_shaped(info["socket"], POD_SIZE.get(config, 1), rank, world,
                                                  max(1, warmup) * pods_per_step,
                                                  min(steps * pods_per_step, 2000), owned)
        st_gg = _server_stats(daemon) if world == 1 else {}
        # ... and every rank times its own device through grpcio.
        stats["grpcio_allocate_p50_us"] = _grpcio_allocate_p50(
            info["socket"], (stats.get("device_ids") or [None])[0])
        st_grpcio = _server_stats(daemon) if world == 1 else {}

        bdf_of = info.get("bdf_of") or {}
        stats["admitted_bdfs"] = sorted({bdf_of.get(i, "?") for i in stats.get("device_ids", [])})
        stats["rank_bdf"] = my_bdf
        if real and probe:
            from ..ops import probe as hip_probe
            try:
                # The GPU this rank's client admitted, by PCI address (not local_rank).
                bdf = stats["admitted_bdfs"][0] if stats["admitted_bdfs"] else None
                dev = hip_probe.device_for_bdf(bdf) if bdf and bdf != "?" else local_rank
                stats["probe"] = hip_probe.run(dev, 256 << 20, 5)
                stats["probe_bdf"] = stats["probe"].get("pci")
            except Exception as e:  # reported, not fatal for the latency metric
                stats["probe"] = {"error": str(e)}
            # The probe may have run on another HIP device than this rank's (amdsmi
            # and HIP orders can differ); the collectives below use the rank's own.
            # (The probe restores the caller's device itself; this is the backstop.)
            torch.cuda.set_device(local_rank)

        everyone = [stats]
        if use_dist:
            everyone = [None] * world
            dist.all_gather_object(everyone, stats)
        if rank == 0:
            server = _server_stats(daemon)
            grpcio = [s.get("grpcio_allocate_p50_us") for s in everyone]
            grpcio = max(grpcio) if all(g is not None for g in grpcio) else None
            gg = [s.get("grpc_go_shaped") or {} for s in everyone]
            gg_ok = all("allocate" in g for g in gg)
            ms_per_step = max(s["elapsed_s"] for s in everyone) / steps * 1e3
            p50 = max(s["allocate"]["p50_us"] for s in everyone)
            total_pods = sum(s["pods"] for s in everyone)
            result = {
                "metric": METRIC,
                "value": round(p50, 2),
                "unit": "us",
                "n_gpus": gpus,
                "steps": steps,
                "warmup": warmup,
                "ms_per_step": round(ms_per_step, 4),
                "higher_is_better": False,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": "n/a",
                "data": ("synthetic pod churn; real libamd_smi on MI355X" if real
                         else "synthetic pod churn; amdsmi mock node model (no GPU)"),
                "config": {
                    "model": desc.format(n=gpus, p=info.get("advertised")),
                    "global_batch": pods_per_step * world,
                    "seq_len": None,
                    "parallelism": f"ranks{world} (one kubelet client per GPU)",
                    "partition_strategy": strategy,
                    "resource_config": rc,
                    "server_threads": server.get("server_threads"),
                },
                "allocatable": info["allocatable"],
                "advertised": info["advertised"],
                "resource": info["resource"],
                "allocate_p99_us": round(max(s["allocate"]["p99_us"] for s in everyone), 2),
                "preferred_p50_us": round(max(s["preferred"]["p50_us"] for s in everyone), 2),
                "pod_p50_us": round(max(s["pod"]["p50_us"] for s in everyone), 2),
                "pods_per_s": round(total_pods / (max(s["elapsed_s"] for s in everyone)), 1),
                # in-daemon time of the Allocate handler (decode + lookup + encode), from SIGUSR1 stats
                "server_allocate_handler_avg_us": server.get("allocate_handler_avg_us"),
                # the same Allocate through grpcio (gRPC C-core + Python), i.e. what a
                # heavyweight gRPC client stack adds on top of the plugin (max over ranks)
                "grpcio_client_allocate_p50_us": grpcio,
                # the same churn with the kubelet's grpc-go client frame pattern (BDP
                # PING per response, grpc-go user-agent), max over ranks
                "grpc_go_shaped_allocate_p50_us": (round(max(g["allocate"]["p50_us"] for g in gg), 2)
                                                   if gg_ok else None),
                "grpc_go_shaped_allocate_p99_us": (round(max(g["allocate"]["p99_us"] for g in gg), 2)
                                                   if gg_ok else None),
                # what torch.distributed actually ran with (RCCL on the GPU box)
                "rccl_world": dist.get_world_size() if use_dist else 1,
                "backend": dist.get_backend() if use_dist else "none",
                "per_rank": [{**{k: s[k] for k in ("rank", "rank_devices", "pods", "allocate", "preferred")},
                              "rank_bdf": s.get("rank_bdf"),
                              "admitted_bdfs": s.get("admitted_bdfs"), "probe_bdf": s.get("probe_bdf"),
                              "grpcio_allocate_p50_us": s.get("grpcio_allocate_p50_us"),
                              "grpc_go_shaped": s.get("grpc_go_shaped"),
                              "client_cpus": s.get("cpus")}
                             for s in everyone],
            }
            # CPU placement of the timed client vs the gRPC loops (1 rank: directly comparable).
            if world == 1:
                result["placement"] = _placement(everyone[0].get("cpus"), loops_before, loops_after)
            # The daemon's own share of each client's latency: unary calls from the
            # socket read that carried them to the reply written (the headline and
            # grpc-go-shaped phases mix Allocate and GetPreferredAllocation; the
            # grpcio phase is Allocate only). Whatever the client stack costs, this
            # is what the plugin adds to it.
            if world == 1:
                result["server_residency"] = {"native_client": _residency(st_before, st_timed),
                                              "grpc_go_shaped": _residency(st_timed, st_gg),
                                              "grpcio": _residency(st_gg, st_grpcio)}
            else:
                result["server_residency"] = {"all_calls": _residency({}, server)}
            # The node the daemon served, and a k-GPU pod's placement on it.
            result["topology"] = info.get("topology")
            result["preferred_k"] = info.get("preferred_k")
            if real and probe and isinstance(result["topology"], dict) and "device_order" in result["topology"]:
                result["topology"]["device_order"]["container_view"] = _container_view(info_snap)
            probes = [s.get("probe") for s in everyone if s.get("probe")]
            if probes:
                result["probe"] = probes
            # Last: how long a node is without the resource when the kubelet restarts
            # (reported, never fatal for the headline).
            try:
                kub, result["kubelet_restart"] = _kubelet_restart(kub, info["resource"])
            except Exception as e:
                result["kubelet_restart"] = {"error": str(e)}
            return result
        return None
    finally:
        if rank == 0:
            if daemon is not None:
                code = daemon.stop()
                if code not in (0, None):
                    log(f"daemon exited with {code}:\n{daemon.log()[-3000:]}")
            if kub is not None:
                kub.stop()
        if use_dist and dist.is_initialized():
            dist.destroy_process_group()


def _kubelet_restart(kub, resource, rounds=5):
    """Restarts the stub kubelet `rounds` times (its socket re-created, as a
    kubelet restart does) and times, on the stub's monotonic clock, from its
    socket listening to the plugin's Register() and to the first device list
    (the node can schedule the resource again). Returns the running stub and
    the medians in ms."""
    import statistics
    from ..utils import harness
    reg, devs = [], []
    for _ in range(rounds):
        kub.stop()
        kub = harness.NativeKubelet(kub.socket_path)
        try:
            kub.start()
        except Exception as e:  # the caller stops `kub` whatever happened
            return kub, {"error": str(e)}
        t0 = next((e["t_us"] for e in kub.events if e.get("event") == "listening"), None)
        if t0 is None:
            return kub, None
        r = kub.wait(lambda e: e.get("event") == "register" and e.get("resource") == resource, 20)
        d = kub.wait(lambda e: e.get("event") == "devices" and e.get("resource") == resource, 20)
        if r is None or d is None:
            return kub, None
        reg.append((r["t_us"] - t0) / 1e3)
        devs.append((d["t_us"] - t0) / 1e3)
    return kub, {"rounds": rounds, "register_ms": round(statistics.median(reg), 3),
                 "devices_ms": round(statistics.median(devs), 3), "devices_ms_max": round(max(devs), 3)}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(gpus, argv):
    """Runs this benchmark as a `gpus`-rank job: torch.distributed.run as a
    child process (one rank per GPU, rendezvous on 127.0.0.1) and returns its
    exit status. Called before anything in this process touches the GPU, so
    the parent never holds a device while the ranks run."""
    import subprocess
    import sys
    from .. import REPO_ROOT
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO_ROOT, "bench.py"), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL between ranks
    return subprocess.call(cmd, env=env)


def main(argv=None):
    import argparse
    import sys
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pods-per-step", type=int, default=100)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="spx-none")
    ap.add_argument("--mock", action="store_true", help="use the amdsmi mock even on a GPU box")
    ap.add_argument("--no-probe", action="store_true")
    a = ap.parse_args(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # No launcher: start the ranks ourselves (rank 0 prints the JSON line).
        raise SystemExit(launch_ranks(a.gpus, argv))
    res = run(a.gpus, a.steps, a.warmup, a.pods_per_step, a.config, a.mock, not a.no_probe)
    if res is not None:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
