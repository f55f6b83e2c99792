"""partitionStrategy none|single|mixed and resourceConfig over MI355X node models.

Parity: reference mig-strategy.go:94-278 (none/single/mixed), main.go:171-203
(resource config), server.go:95-111 (replicas, auto = MiB/1000). Runs the daemon's
own strategy code in-process (libadp_capi) against the amdsmi mock.
"""

import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import native

VRAM = fixtures.MI355X_VRAM_MIB


def specs(mock_env, fx, **kw):
    return native.plugin_specs(mock_env(fx), **kw)


def by_resource(out):
    return {s["resource"]: s for s in out}


def test_none_spx8_one_device_per_gpu(mock_env):
    out = specs(mock_env, fixtures.node(8))
    assert len(out) == 1
    s = out[0]
    assert s["resource"] == "amd.com/gpu" and s["socket"] == "amd-gpu.sock"
    assert s["advertised"] == 8 and not s["replicated"]
    assert [d["index"] for d in s["devices"]] == [str(i) for i in range(8)]
    assert [d["paths"] for d in s["devices"]] == [[f"/dev/dri/renderD{128 + 8 * i}"] for i in range(8)]
    assert [d["numa"] for d in s["devices"]] == [0, 0, 0, 0, 1, 1, 1, 1]


def test_none_on_cpx_gpu_hands_out_the_whole_chip(mock_env):
    out = specs(mock_env, fixtures.node(2, "CPX", memory="NPS2"))
    d0 = out[0]["devices"][0]
    assert d0["paths"] == [f"/dev/dri/renderD{128 + p}" for p in range(8)]
    assert d0["vram_mib"] == (VRAM // 8) * 8


def test_single_cpx8_advertises_64_partitions(mock_env):
    out = specs(mock_env, fixtures.node(8, "CPX", memory="NPS2"), strategy="single")
    assert len(out) == 1
    s = out[0]
    assert s["resource"] == "amd.com/gpu"
    assert s["advertised"] == 64
    assert s["devices"][9]["index"] == "1:1"
    assert s["devices"][9]["paths"] == ["/dev/dri/renderD137"]
    assert len({d["id"] for d in s["devices"]}) == 64  # distinct, stable partition IDs
    assert all(d["vram_mib"] == VRAM // 8 for d in s["devices"])


def test_single_falls_back_to_none_without_partitions(mock_env):
    out = specs(mock_env, fixtures.node(2), strategy="single")
    assert out[0]["resource"] == "amd.com/gpu" and out[0]["advertised"] == 2


def test_single_rejects_mixed_modes(mock_env):
    with pytest.raises(native.NativeError, match="same compute partition mode"):
        specs(mock_env, fixtures.node(2, ["SPX", "CPX"], memory="NPS2"), strategy="single")


def test_single_rejects_two_profiles(mock_env):
    with pytest.raises(native.NativeError, match="more than one partition profile"):
        specs(mock_env, fixtures.node(2, ["DPX", "CPX"]), strategy="single")


def test_single_rejects_invalid_memory_layout(mock_env):
    # NPS4 memory partitions cannot split over 2 (DPX) compute partitions
    with pytest.raises(native.NativeError, match="incompatible"):
        specs(mock_env, fixtures.node(1, "DPX", memory="NPS4"), strategy="single")


def test_mixed_spx_plus_cpx(mock_env):
    out = by_resource(specs(mock_env, fixtures.CONFIGS["mixed8"](), strategy="mixed"))
    assert set(out) == {"amd.com/gpu", "amd.com/cpx-1xcd.36gb"}
    assert out["amd.com/gpu"]["advertised"] == 4
    assert out["amd.com/cpx-1xcd.36gb"]["advertised"] == 32
    assert out["amd.com/cpx-1xcd.36gb"]["socket"] == "amd-cpx-1xcd.36gb.sock"
    assert {d["gpu"] for d in out["amd.com/cpx-1xcd.36gb"]["devices"]} == {4, 5, 6, 7}


def test_mixed_skips_invalid_partitions(mock_env):
    out = by_resource(specs(mock_env, fixtures.node(2, ["SPX", "DPX"], memory="NPS4"), strategy="mixed"))
    assert set(out) == {"amd.com/gpu"}


def test_mixed_rename_applies_to_partition_resources(mock_env):
    # Reference defect B3: mixed mode ignored renames of MIG resources.
    out = by_resource(specs(mock_env, fixtures.CONFIGS["mixed8"](), strategy="mixed",
                            resource_config="gpu:fullgpu:1,cpx-1xcd.36gb:slice:2"))
    assert set(out) == {"amd.com/fullgpu", "amd.com/slice"}
    assert out["amd.com/slice"]["advertised"] == 64 and out["amd.com/slice"]["replicated"]


def test_timeslice_replicas(mock_env):
    s = specs(mock_env, fixtures.node(8), resource_config="gpu:sharedgpu:4")[0]
    assert s["resource"] == "amd.com/sharedgpu"
    assert s["advertised"] == 32 and s["replicated"]
    ids = s["advertised_ids"]
    assert ids[0] == s["devices"][0]["id"] + "-replica-0"
    assert ids[3] == s["devices"][0]["id"] + "-replica-3"
    assert max(len(i) for i in ids) <= 63


def test_auto_memory_replicas_per_gpu_and_per_partition(mock_env):
    s = specs(mock_env, fixtures.node(8), resource_config="gpu:gpu-mem-gb:-1")[0]
    assert s["resource"] == "amd.com/gpu-mem-gb"
    assert all(d["replicas"] == VRAM // 1000 for d in s["devices"])  # 294
    assert s["advertised"] == 8 * (VRAM // 1000)  # 2352
    # B4: partitions use their own share, not the parent's memory
    p = specs(mock_env, fixtures.node(8, "CPX", memory="NPS2"), strategy="single",
              resource_config="gpu:gpu-mem-gb:-1")[0]
    assert all(d["replicas"] == (VRAM // 8) // 1000 for d in p["devices"])  # 36
    assert p["advertised"] == 64 * ((VRAM // 8) // 1000)


def test_no_entry_means_one_replica_not_zero(mock_env):
    # Reference defect B2: a missing resourceConfig entry advertised zero devices.
    s = specs(mock_env, fixtures.node(2), resource_config="cpx-1xcd.36gb:other:2")[0]
    assert s["advertised"] == 2


def test_devices_filter_and_index_strategy(mock_env):
    s = specs(mock_env, fixtures.node(8), devices=[4, 6], id_strategy="index")[0]
    assert [d["index"] for d in s["devices"]] == ["4", "6"]


def test_partition_ids_when_amdsmi_reports_shared_uuids(mock_env):
    fx = fixtures.node(1, "QPX", memory="NPS1")
    fx["gpus"][0]["partition_uuids"] = "shared"
    s = specs(mock_env, fx, strategy="single")[0]
    ids = [d["id"] for d in s["devices"]]
    assert ids == [fx["gpus"][0]["uuid"] + f"-p{i}" for i in range(4)]


def test_partitions_grouped_by_asic_serial_even_across_pci_functions(mock_env):
    # Partitions of one GPU may not share a PCI bus/device; the ASIC serial still groups them.
    fx = fixtures.node(2, "QPX", memory="NPS1")
    out = specs(mock_env, fx, strategy="single")[0]
    assert out["advertised"] == 8 and {d["gpu"] for d in out["devices"]} == {0, 1}
    # Without serials, fall back to the PCI bus/device grouping: same answer.
    for g in fx["gpus"]:
        g["asic_serial"] = ""
    out2 = specs(mock_env, fx, strategy="single")[0]
    assert [d["id"] for d in out2["devices"]] == [d["id"] for d in out["devices"]]


@pytest.mark.parametrize("text,err", [
    ("gpu:x", "colon"), ("gpu:x:-2", "positive"), ("gpu:x:0", "positive"), ("gpu:x:y", "integer"),
    ("gpu::1", "invalid new resource name"),
])
def test_resource_config_errors(text, err):
    with pytest.raises(native.NativeError, match=err):
        native.parse_resource_config(text)


def test_resource_config_grammar():
    rc = native.parse_resource_config(" gpu:sharedgpu:4 , cpx-1xcd.36gb:small:2,, gpu2:m:-1 ")
    assert rc == {"gpu": {"name": "sharedgpu", "replicas": 4, "auto": False},
                  "cpx-1xcd.36gb": {"name": "small", "replicas": 2, "auto": False},
                  "gpu2": {"name": "m", "replicas": 1, "auto": True}}
