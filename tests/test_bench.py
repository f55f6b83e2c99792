"""bench.py contract on CPU: single process, launcher-less multi-rank runs and a
2-rank torchrun (gloo) job on the mock."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _last_json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_single_process_contract():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--mock"],
                       cwd=ROOT, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    res = _last_json(r.stdout)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in res
    assert res["n_gpus"] == 1 and res["steps"] == 3 and res["warmup"] == 1
    assert res["higher_is_better"] is False and res["unit"] == "us"
    assert res["allocatable"] == 1
    assert 0 < res["value"] < 5000
    assert res["per_rank"][0]["allocate"]["n"] == 300
    assert res["rccl_world"] == 1 and res["backend"] == "none"
    assert res["per_rank"][0]["admitted_bdfs"] == ["0000:0c:00.0"]  # GPU 0 of the node model
    # the daemon serves exactly the rank's GPU of the 8-GPU node model
    topo = res["topology"]
    assert topo["served_bdfs"] == topo["rank_bdfs"] == ["0000:0c:00.0"]
    assert res["preferred_k"]["k"] == 1 and res["preferred_k"]["bdfs"] == ["0000:0c:00.0"]
    # the kubelet's grpc-go frame pattern: a BDP PING after (about) every response
    gg = res["per_rank"][0]["grpc_go_shaped"]
    assert gg["allocate"]["n"] == 300 and gg["bdp_pings"] >= gg["pods"]
    assert res["grpc_go_shaped_allocate_p50_us"] == gg["allocate"]["p50_us"] > 0
    # kubelet restarts: re-registered without re-enumeration or a health-monitor
    # restart (whose amdsmi event wait took up to 500 ms to stop)
    kr = res["kubelet_restart"]
    assert kr["rounds"] == 5 and 0 < kr["register_ms"] <= kr["devices_ms"] < 150, kr
    # where the timed client and the loop that served it ran: exactly one loop
    # was busy during the timed region (its 300 pods = 600 calls)
    pl = res["placement"]
    assert pl["relation"] in ("same-core", "same-l3", "other-l3") and pl["client_cpus"], pl
    # (another loop may wake a few times meanwhile: a health broadcast to the
    # ListAndWatch stream it serves)
    busy = [b for _, b in pl["loops_during_timed"] if b >= 300]
    idle = [b for _, b in pl["loops_during_timed"] if b < 300]
    assert len(busy) == 1 and all(b <= 10 for b in idle), pl
    # the daemon's own share of each client's latency (read -> reply handed to
    # send()): one sample per call, the timed 300 pods being 600 calls
    sr = res["server_residency"]
    assert sr["native_client"]["samples"] == 600, sr
    assert 0 < sr["native_client"]["p50_us"] <= sr["native_client"]["p99_us"]
    assert sr["native_client"]["p50_us"] < res["pod_p50_us"], (sr, res["pod_p50_us"])
    assert sr["grpc_go_shaped"]["samples"] >= 600 and 300 <= sr["grpcio"]["samples"] <= 350, sr


@pytest.mark.slow
def test_bench_two_ranks_gloo():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29561", "bench.py", "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--mock"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = _last_json(r.stdout)
    assert res["n_gpus"] == 2 and res["allocatable"] == 2
    assert sorted(p["rank"] for p in res["per_rank"]) == [0, 1]
    assert all(p["rank_devices"] == 1 for p in res["per_rank"])
    assert res["rccl_world"] == 2 and res["backend"] == "gloo"  # nccl (RCCL) on the GPU box
    bdfs = {p["rank"]: p["admitted_bdfs"] for p in res["per_rank"]}
    assert bdfs == {0: ["0000:0c:00.0"], 1: ["0000:2c:00.0"]}  # each rank admits its own GPU
    # an independent gRPC stack (grpcio) per rank, max over ranks at the top
    per = [p["grpcio_allocate_p50_us"] for p in res["per_rank"]]
    assert all(v and v > 0 for v in per) and res["grpcio_client_allocate_p50_us"] == max(per)
    gg = [p["grpc_go_shaped"]["allocate"]["p50_us"] for p in res["per_rank"]]
    assert res["grpc_go_shaped_allocate_p50_us"] == max(gg)
    assert res["server_residency"]["all_calls"]["samples"] > 0


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_multi_gpu_without_launcher(n):
    """`python bench.py --gpus N` starts its N ranks itself (the driver's 1-GPU
    invocation, N > 1): one process group of N ranks, the daemon serving
    exactly the ranks' GPUs by PCI address, the node's link matrix and a
    k=min(4,N) preferred allocation in the JSON."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--steps", "2", "--warmup", "1", "--mock",
                        "--pods-per-step", "20"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = _last_json(r.stdout)
    assert res["n_gpus"] == n and res["rccl_world"] == n and res["backend"] == "gloo"
    assert res["allocatable"] == n
    topo = res["topology"]
    assert topo["served_bdfs"] == topo["rank_bdfs"] and len(topo["rank_bdfs"]) == n
    for key in ("link_types", "hops", "weights", "link_class"):
        assert len(topo[key]) == n and all(len(row) == n for row in topo[key])
    assert all(topo["link_types"][i][j] == ("self" if i == j else "xgmi") for i in range(n) for j in range(n))
    assert [g["xgmi_links_down"] for g in topo["gpus"]] == [0] * n
    pk = res["preferred_k"]
    assert pk["k"] == min(4, n) and len(set(pk["bdfs"])) == pk["k"] and set(pk["bdfs"]) <= set(topo["served_bdfs"])
    for p in res["per_rank"]:
        assert p["admitted_bdfs"] == [p["rank_bdf"]] and p["allocate"]["n"] == 40
    assert sorted(p["rank_bdf"] for p in res["per_rank"]) == sorted(topo["served_bdfs"])
    # container lists follow KFD order; on the node model HIP order is the same
    order = topo["device_order"]
    assert order["hip_order"] == topo["rank_bdfs"] and order["hip_order_is_kfd_order"] is True
    assert sorted(order["kfd_order"]) == sorted(topo["served_bdfs"])
    # a k=4 pod on the 8-GPU mesh stays on one NUMA node (GPUs 0-3 and 4-7 share one each)
    numa = {g["bdf"]: g["numa"] for g in topo["gpus"]}
    if n >= 4:
        assert len({numa[b] for b in pk["bdfs"]}) == 1, (pk, numa)


def test_bench_serves_the_ranks_gpus_not_amdsmi_order():
    """A job given GPUs 5 and 2 of the node (HIP order != amdsmi order): the
    daemon serves exactly those two, and each rank admits its own."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR")}
    env["ADP_BENCH_MOCK_GPUS"] = "5,2"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1", "--mock",
                        "--pods-per-step", "10", "--config", "timeslice4"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = _last_json(r.stdout)
    topo = res["topology"]
    assert topo["rank_bdfs"] == ["0000:ac:00.0", "0000:4c:00.0"]
    assert sorted(topo["served_bdfs"]) == sorted(topo["rank_bdfs"])
    assert res["advertised"] == 8  # 2 GPUs x 4 replicas, not 8 GPUs x 4
    bdfs = {p["rank"]: (p["rank_bdf"], p["admitted_bdfs"]) for p in res["per_rank"]}
    assert bdfs == {0: ("0000:ac:00.0", ["0000:ac:00.0"]), 1: ("0000:4c:00.0", ["0000:4c:00.0"])}
    assert all(p["rank_devices"] == 4 for p in res["per_rank"])
    # the three device orders: amdsmi's, KFD node order (what container lists
    # follow) and HIP's (rank r = HIP device r), with the per-GPU KFD node
    order = topo["device_order"]
    assert order["amdsmi_order"] == ["0000:4c:00.0", "0000:ac:00.0"] == order["kfd_order"]
    assert order["hip_order"] == topo["rank_bdfs"]
    assert order["hip_order_is_kfd_order"] is False and order["hip_order_is_amdsmi_order"] is False
    assert [g["kfd_node"] for g in topo["gpus"]] == [2 + 8 * 2, 2 + 8 * 5]


@pytest.mark.parametrize("config,advertised", [("timeslice4", 4), ("cpx-single", 8), ("auto-mem", 294),
                                               ("mixed-gpu4", 6)])
def test_bench_configs_on_mock(config, advertised, monkeypatch):
    sys.path.insert(0, ROOT)
    from k8s_gpu_sharing_plugin_amd.parallel import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    res = bench.run(gpus=1, steps=1, warmup=1, pods_per_step=50, config=config, force_mock=True, probe=False)
    assert res["advertised"] == advertised
    assert res["allocatable"] == advertised
    assert res["per_rank"][0]["allocate"]["n"] == 50


def test_bench_mixed_gpu4_admits_four_gpu_pods(monkeypatch):
    """BASELINE config 5: every admission is a 4-GPU preferred allocation on the SPX part."""
    sys.path.insert(0, ROOT)
    from k8s_gpu_sharing_plugin_amd.parallel import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    res = bench.run(gpus=1, steps=1, warmup=1, pods_per_step=20, config="mixed-gpu4", force_mock=True, probe=False)
    assert res["resource"] == "amd.com/gpu" and res["advertised"] == 6
    assert res["per_rank"][0]["preferred"]["n"] == 20


def test_bench_one_rank_under_torchrun_uses_a_process_group():
    """torchrun with one rank runs the same collectives as the multi-GPU job
    (gloo here on the mock; RCCL on the GPU box, tests/test_gpu.py)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", "29563", "bench.py", "--gpus", "1",
                        "--steps", "2", "--warmup", "1", "--mock"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = _last_json(r.stdout)
    assert res["rccl_world"] == 1 and res["backend"] == "gloo"


@pytest.mark.parametrize("config,advertised", [("timeslice4", 32), ("cpx-single", 64)])
def test_bench_eight_ranks_advertise_the_baseline_counts(config, advertised):
    """BASELINE configs 3 and 4 at N=8 -- the path the driver's 8-GPU scaling run
    takes: 8 ranks (gloo here, RCCL there), one daemon serving all 8 GPUs.
    Time-slice sharing advertises 4 replicas x 8 GPUs = 32; CPX with
    partitionStrategy=single advertises 8 partitions x 8 GPUs = 64. Every rank
    admits pods on its own GPU only, and a k=4 pod's preferred placement stays
    on one GPU's partitions (CPX) or one NUMA node (SPX)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--steps", "2", "--warmup", "1", "--mock",
                        "--pods-per-step", "20", "--config", config],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = _last_json(r.stdout)
    assert res["n_gpus"] == 8 and res["rccl_world"] == 8
    assert res["allocatable"] == advertised and res["advertised"] == advertised
    assert res["value"] > 0 and res["allocate_p99_us"] >= res["value"]
    per = res["per_rank"]
    assert sorted(p["rank"] for p in per) == list(range(8))
    assert all(p["rank_devices"] == advertised // 8 for p in per)
    assert all(p["admitted_bdfs"] == [p["rank_bdf"]] for p in per)
    topo = res["topology"]
    pk = res["preferred_k"]
    assert pk["k"] == 4 and pk["available"] == advertised
    numa = {g["bdf"]: g["numa"] for g in topo["gpus"]}
    if config == "cpx-single":
        assert len(set(pk["bdfs"])) == 1  # four partitions of one GPU
    else:
        assert len(set(pk["bdfs"])) == 4 and len({numa[b] for b in pk["bdfs"]}) == 1
