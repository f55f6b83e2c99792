"""CU counts and product names from sysfs when amdsmi's asic_info cannot answer.

asic_info (market name, CU count) goes through libdrm and needs the GPU's
render node; an unprivileged pod's device cgroup denies it (measured on the
MI355X: profiles/r3/access/). Without a CU count there are no CU shares
(--replica-cu-mask) and no CU-slot memory units, so the chart's drop-ALL
plugin container would silently lose them. KFD's topology
(/sys/class/kfd/kfd/topology/nodes/<n>/properties: simd_count / simd_per_cu),
readable unprivileged, gives the count per KFD node -- per GPU in SPX, per
partition in CPX. The board's FRU name (/sys/bus/pci/devices/<bdf>/
product_name: "AMD Instinct MI355 OAM" on the MI355X box, where asic_info says
"AMD Radeon Graphics") names the product, with or without the render node.
Both live under --sysfs-root. The mock's "render_denied" makes asic_info and
vram_info fail as the denial does. The real-hardware check is
tests/test_gpu_isolation.py::test_kfd_topology_cus_match_asic_info.
"""

import json
import os
import subprocess

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, native
from k8s_gpu_sharing_plugin_amd import MOCK_LIB


def _topology(root, nodes):
    """A sysfs root whose KFD topology has nodes {kfd node: CUs}, in the
    properties layout the amdgpu driver writes."""
    for n, cus in nodes.items():
        d = os.path.join(root, "class/kfd/kfd/topology/nodes", str(n))
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "properties"), "w") as f:
            f.write(f"cpu_cores_count 0\nsimd_count {cus * 4}\nmem_banks_count 1\nsimd_per_cu 4\n"
                    f"max_waves_per_simd 8\nnum_xcc {8 if cus == 256 else 1}\nlocation_id 3072\n")
    return root


def _dry_run(scratch, fx, *args):
    env = harness.Daemon(scratch, fx).env
    r = subprocess.run([harness.DAEMON, "--device-plugin-path", scratch, "--dry-run", *args], capture_output=True,
                       text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout), r.stderr


def test_cu_slots_survive_a_denied_render_node(scratch, tmp_path):
    fx = fixtures.node(2)
    for g in fx["gpus"]:
        g["render_denied"] = True
    topo = _topology(str(tmp_path / "nodes"), {2: 256, 10: 256})  # the mock's KFD nodes: 2 + 8*i
    out, log = _dry_run(scratch, fx, "--replica-cu-mask", "--resource-config", "gpu:gpu-mem-gb:-1",
                        "--sysfs-root", topo)
    assert [g["cus"] for g in out["gpus"]] == [256, 256]
    (res,) = out["resources"]
    assert res["allocatable"] == 2 * 32  # CU-slot units: 32 per GPU, as with asic_info
    assert "CU counts of 2 processor(s) from KFD topology" in log
    # no topology: the CU count is unknown, and the daemon says what that costs
    out, log = _dry_run(scratch, fx, "--replica-cu-mask", "--resource-config", "gpu:gpu-mem-gb:-1",
                        "--sysfs-root", str(tmp_path / "absent"))
    assert out["resources"][0]["allocatable"] == 2 * 294
    assert "CU count of 2 processor(s) unknown" in log and "no CU slots" in log


def test_asic_info_wins_and_partitions_read_their_own_nodes(scratch, tmp_path, monkeypatch):
    """asic_info, when it answers, is used as is (the topology is not read);
    CPX partitions are KFD nodes of their own, 32 CUs each."""
    fx = fixtures.node(1)
    out, log = _dry_run(scratch, fx, "--sysfs-root", _topology(str(tmp_path / "wrong"), {2: 100}))
    assert out["gpus"][0]["cus"] == 256 and "from KFD topology" not in log
    cpx = fixtures.node(1, ["CPX"], memory="NPS2")
    cpx["gpus"][0]["render_denied"] = True
    topo = _topology(str(tmp_path / "cpx"), {2 + p: 32 for p in range(8)})
    monkeypatch.setenv("AMDSMI_MOCK_FIXTURE", fixtures.write(cpx, str(tmp_path / "fx")))
    snap = native.snapshot(MOCK_LIB, sysfs_root=topo)
    assert [p["cus"] for p in snap["gpus"][0]["partitions"]] == [32] * 8
    assert snap["gpus"][0]["cus"] == 256


def test_pci_product_name_names_the_board(scratch, tmp_path):
    """The FRU name wins over asic_info's market name (label and HBM model
    table), for every partition of the board (function 0)."""
    root = str(tmp_path / "sys")
    fx = fixtures.node(1, ["CPX"], memory="NPS2")
    bdf = fx["gpus"][0]["bdf"]
    d = os.path.join(root, "bus/pci/devices", bdf.rsplit(".", 1)[0] + ".0")
    os.makedirs(d)
    with open(os.path.join(d, "product_name"), "w") as f:
        f.write("AMD Instinct MI355 OAM\n")
    out, log = _dry_run(scratch, fx, "--sysfs-root", root)
    assert out["labels"]["amd.com/gpu.product"] == "AMD-Instinct-MI355-OAM"
    assert "product names of 8 processor(s) from PCI sysfs" in log
    out, _ = _dry_run(scratch, fx, "--sysfs-root", str(tmp_path / "empty"))
    assert out["labels"]["amd.com/gpu.product"] != "AMD-Instinct-MI355-OAM"


def test_topology_parser_edge_cases(tmp_path):
    root = str(tmp_path / "n")
    for node, text in (("1", "simd_count 1024\nsimd_per_cu 4\n"), ("2", "simd_count 0\nsimd_per_cu 4\n"),
                       ("3", "simd_count 1023\nsimd_per_cu 4\n"), ("4", "simd_per_cu 4\n"),
                       ("5", "simd_count x\nsimd_per_cu 4\n")):
        os.makedirs(os.path.join(root, node))
        with open(os.path.join(root, node, "properties"), "w") as f:
            f.write(text)
    assert [native.kfd_topology_cus(root, n) for n in (1, 2, 3, 4, 5, 6)] == [256, 0, 0, 0, 0, 0]


def test_doctor_names_the_cu_count_source(tmp_path):
    from test_doctor import _doctor, _find
    fx = fixtures.node(1)
    fx["gpus"][0]["render_denied"] = True
    topo = _topology(str(tmp_path / "nodes"), {2: 256})
    _, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), "--sysfs-root", topo, fx=fx)
    assert _find(lines, "CU counts:").startswith("ok") and "from KFD topology on 1" in _find(lines, "CU counts:")
    rc, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), "--sysfs-root", str(tmp_path / "x"),
                        "--replica-cu-mask", fx=fx)
    line = _find(lines, "CU counts:")
    assert rc == 1 and line.startswith("FAIL") and "no CU shares" in line, lines
    _, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), fx=fixtures.node(1))
    assert _find(lines, "CU counts:") is None  # asic_info answered: nothing to say


def test_smi_report_lists_the_sysfs_fallbacks(tmp_path):
    sysfs = _topology(str(tmp_path / "sys"), {2: 256})
    fx = fixtures.node(1)
    d = os.path.join(sysfs, "bus/pci/devices", fx["gpus"][0]["bdf"])
    os.makedirs(d)
    with open(os.path.join(d, "product_name"), "w") as f:
        f.write("AMD Instinct MI355 OAM\n")
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=fixtures.write(fx, str(tmp_path / "fx")))
    r = subprocess.run([harness.DAEMON, "--device-plugin-path", str(tmp_path), "--smi-report", "--sysfs-root", sysfs],
                       capture_output=True, text=True, timeout=60, env=env)
    rep = json.loads(r.stdout)
    assert rep["sysfs"] == [{"bdf": fx["gpus"][0]["bdf"], "kfd_node": 2, "topology_cus": 256,
                             "pci_product_name": "AMD Instinct MI355 OAM"}], rep["sysfs"]
