"""Flags / env / versioned config file precedence.

Parity: api/config/v1/config.go:30-144 (version v1, CLI > env > file) and
main.go:62-130 (flags + env). Fixes pinned: B7 (false booleans from the file
are honoured), B8 (resourceConfig can come from the file).
"""

import json
import os

import pytest

from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet


def effective_config(scratch, args=(), env=None, file_body=None, expect_exit=None):
    if file_body is not None:
        path = os.path.join(scratch, "config.yaml")
        with open(path, "w") as f:
            f.write(file_body)
        args = ["--config-file", path, *args]
    d = harness.Daemon(scratch, args=args, env=env).start()
    if expect_exit is not None:
        assert d.proc.wait(10) == expect_exit
        return d.log()
    text = d.wait_log("running with resource config")
    d.stop()
    start = text.index("running with config:\n") + len("running with config:\n")
    end = text.index("\n}\n", start) + 2
    return json.loads(text[start:end])["flags"]


def test_defaults(scratch):
    f = effective_config(scratch)
    assert f["partitionStrategy"] == "none"
    assert f["failOnInitError"] is True
    assert f["passDeviceSpecs"] is True
    assert f["deviceListStrategy"] == "envvar"
    assert f["deviceIDStrategy"] == "uuid"
    assert f["driverRoot"] == "/"
    assert f["resourceConfig"] == ""
    # round 3: loop placement is opt-in (peer-l3 only acts on a visible, single-threaded caller)
    assert f["loopAffinity"] == "none"
    assert f["healthEvents"] is True


def test_file_values_apply(scratch):
    body = """
version: v1
flags:
  partitionStrategy: mixed
  failOnInitError: false      # B7: false from the file is honoured
  passDeviceSpecs: false
  deviceListStrategy: volume-mounts
  deviceIDStrategy: index
  driverRoot: /run/amd/driver
  resourceConfig: "gpu:sharedgpu:4"   # B8: resourceConfig from the file
"""
    f = effective_config(scratch, file_body=body)
    assert f["partitionStrategy"] == "mixed"
    assert f["failOnInitError"] is False
    assert f["passDeviceSpecs"] is False
    assert f["deviceListStrategy"] == "volume-mounts"
    assert f["deviceIDStrategy"] == "index"
    assert f["driverRoot"] == "/run/amd/driver"
    assert f["resourceConfig"] == "gpu:sharedgpu:4"


def test_precedence_cli_over_env_over_file(scratch):
    body = "version: v1\nflags:\n  deviceIDStrategy: index\n  deviceListStrategy: volume-mounts\n  driverRoot: /file\n"
    f = effective_config(scratch, args=["--device-id-strategy", "uuid"],
                         env={"DEVICE_LIST_STRATEGY": "envvar", "DEVICE_ID_STRATEGY": "index"},
                         file_body=body)
    assert f["deviceIDStrategy"] == "uuid"          # CLI beats env and file
    assert f["deviceListStrategy"] == "envvar"      # env beats file
    assert f["driverRoot"] == "/file"               # file beats default


def test_json_config_file(scratch):
    body = json.dumps({"version": "v1", "flags": {"passDeviceSpecs": False, "resourceConfig": "gpu:g:2"}})
    f = effective_config(scratch, file_body=body)
    assert f["passDeviceSpecs"] is False and f["resourceConfig"] == "gpu:g:2"


def test_config_file_from_env(scratch):
    path = os.path.join(scratch, "c.yaml")
    with open(path, "w") as fh:
        fh.write("version: v1\nflags:\n  deviceIDStrategy: index\n")
    f = effective_config(scratch, env={"CONFIG_FILE": path})
    assert f["deviceIDStrategy"] == "index"


@pytest.mark.parametrize("body,msg", [
    ("flags:\n  deviceIDStrategy: index\n", "missing version field"),
    ("version: v2\n", "unknown version: v2"),
    ("version: v1\nflags:\n  failOnInitError: maybe\n", "invalid boolean 'maybe'"),
    ("version: v1\nflags:\n  - a\n", "flags must be a mapping"),
    ("version: v1\nflags: single\n", "flags must be a mapping"),
    ("version: v1\nflags: {migStrategy: [a, b]}\n", "flags.migStrategy must be a scalar, not a sequence"),
    # typed fields, as the reference's json.Unmarshal into Go structs
    ("version: v1\nflags:\n  migStrategy: yes\n", "cannot unmarshal bool into flags.migStrategy of type string"),
    ("version: v1\nflags:\n  passDeviceSpecs: 3\n", "cannot unmarshal number into flags.passDeviceSpecs of type bool"),
    ("version: 1\n", "unknown version: 1"),
    ("version: v1\nflags: {a: b\n", "unmarshal error: yaml: line"),
    ("- version: v1\n", "must be a mapping"),
])
def test_bad_config_files(scratch, body, msg):
    log = effective_config(scratch, file_body=body, expect_exit=1)
    assert msg in log


def test_missing_config_file(scratch):
    d = harness.Daemon(scratch, args=["--config-file", "/nonexistent.yaml"]).start()
    assert d.proc.wait(10) == 1
    assert "error opening config file" in d.log()


def test_resource_config_env_renames_resource(scratch):
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, env={"RESOURCE_CONFIG": "gpu:sharedgpu:3"}).start()
    reg = k.wait_registration()
    assert reg.resource_name == "amd.com/sharedgpu"
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    assert len(c.watch()[0].get(timeout=5).devices) == 6
    c.close()
    d.stop()
    k.stop()


def test_reference_flag_names_are_accepted(scratch):
    """A reference DaemonSet/config (mig-strategy, nvidia-driver-root,
    NVIDIA_DRIVER_RESOURCE_CONFIG; main.go:63-129) keeps working unchanged."""
    body = "version: v1\nflags:\n  migStrategy: mixed\n  nvidiaDriverRoot: /run/nvidia/driver\n"
    f = effective_config(scratch, file_body=body,
                         env={"NVIDIA_DRIVER_RESOURCE_CONFIG": "gpu:sharedgpu:2"})
    assert f["partitionStrategy"] == "mixed"
    assert f["driverRoot"] == "/run/nvidia/driver"
    assert f["resourceConfig"] == "gpu:sharedgpu:2"
    f = effective_config(scratch, args=["--mig-strategy", "single", "--nvidia-driver-root=/x"],
                         env={"MIG_STRATEGY": "mixed"})
    assert f["partitionStrategy"] == "single" and f["driverRoot"] == "/x"
    f = effective_config(scratch, env={"MIG_STRATEGY": "single"})
    assert f["partitionStrategy"] == "single"


def test_canonical_name_beats_alias(scratch):
    f = effective_config(scratch, args=["--mig-strategy", "mixed", "--partition-strategy", "single"],
                         env={"MIG_STRATEGY": "mixed", "NVIDIA_DRIVER_RESOURCE_CONFIG": "gpu:a:2",
                              "RESOURCE_CONFIG": "gpu:b:3"})
    assert f["partitionStrategy"] == "single"
    assert f["resourceConfig"] == "gpu:b:3"


def test_alias_use_is_logged(scratch):
    d = harness.Daemon(scratch, args=["--mig-strategy", "none"]).start()
    text = d.wait_log("running with resource config")
    d.stop()
    assert "--mig-strategy is accepted for compatibility; use --partition-strategy" in text


def test_server_threads_zero_means_auto(scratch):
    f = effective_config(scratch, args=["--server-threads", "0"])
    assert f["serverThreads"] == 0
    f = effective_config(scratch, env={"DP_SERVER_THREADS": "3"})
    assert f["serverThreads"] == 3


# --- YAML as the reference's sigs.k8s.io/yaml reads it (config.go:70-94) ---

def test_flow_mapping_flags(scratch):
    """The round-1 line parser silently ignored this; go-yaml reads it."""
    body = "version: v1\nflags: {migStrategy: single, failOnInitError: false}\n"
    f = effective_config(scratch, file_body=body)
    assert f["partitionStrategy"] == "single" and f["failOnInitError"] is False


def test_block_scalars_quotes_and_yaml11_bools(scratch):
    body = """version: "v1"
flags:
  resourceConfig: >-
    gpu:sharedgpu:4,
    cpx-1xcd.36gb:small:2
  driverRoot: '/run/it''s'
  deviceIDStrategy: "ind\\x65x"
  passDeviceSpecs: off
  failOnInitError: No
  includeCardNodes: "true"
  serverThreads: 0x4
"""
    f = effective_config(scratch, file_body=body)
    assert f["resourceConfig"] == "gpu:sharedgpu:4, cpx-1xcd.36gb:small:2"
    assert f["driverRoot"] == "/run/it's"
    assert f["deviceIDStrategy"] == "index"
    assert f["passDeviceSpecs"] is False and f["failOnInitError"] is False
    assert f["includeCardNodes"] is True  # quoted bool accepted (lenient)
    assert f["serverThreads"] == 4


def test_literal_block_scalar(scratch):
    body = "version: v1\nflags:\n  resourceConfig: |-\n    gpu:sharedgpu:3\n"
    assert effective_config(scratch, file_body=body)["resourceConfig"] == "gpu:sharedgpu:3"


def test_anchors_aliases_and_merge_keys(scratch):
    body = """version: v1
defaults: &d
  deviceIDStrategy: index
  passDeviceSpecs: false
flags:
  <<: *d
  passDeviceSpecs: true
  resourceConfig: &rc gpu:sharedgpu:2
"""
    text = effective_config(scratch, file_body=body + "", expect_exit=None)
    assert text["deviceIDStrategy"] == "index"      # merged
    assert text["passDeviceSpecs"] is True          # explicit key wins over the merge
    assert text["resourceConfig"] == "gpu:sharedgpu:2"


def test_null_values_leave_defaults(scratch):
    f = effective_config(scratch, file_body="version: v1\nflags:\n  migStrategy: ~\n  driverRoot:\n")
    assert f["partitionStrategy"] == "none" and f["driverRoot"] == "/"


def test_unknown_keys_are_warned_about(scratch):
    body = "version: v1\nflags:\n  migStrategi: single\n  deviceIDStrategy: index\nsharing: {}\n"
    d = harness.Daemon(scratch, args=["--config-file", _write(scratch, body)]).start()
    text = d.wait_log("running with resource config")
    d.stop()
    assert "unknown key flags.migStrategi (ignored)" in text
    assert "unknown key sharing (ignored)" in text
    assert '"deviceIDStrategy": "index"' in text


def test_only_the_first_document_is_read(scratch):
    body = "version: v1\nflags: {deviceIDStrategy: index}\n---\nversion: v2\n"
    assert effective_config(scratch, file_body=body)["deviceIDStrategy"] == "index"


def test_json_with_yaml_types(scratch):
    body = '{"version": "v1", "flags": {"failOnInitError": false, "serverThreads": 2, "migStrategy": null}}'
    f = effective_config(scratch, file_body=body)
    assert f["failOnInitError"] is False and f["serverThreads"] == 2 and f["partitionStrategy"] == "none"


def test_without_libyaml_unsupported_yaml_is_an_error_not_ignored(scratch):
    """The strict fallback parser (libyaml missing) refuses what it cannot read."""
    env = {"ADP_LIBYAML": "/nonexistent/libyaml.so"}
    log = effective_config(scratch, env=env, expect_exit=1,
                           file_body="version: v1\nflags: {migStrategy: single}\n")
    assert "a flow collection needs libyaml" in log
    log = effective_config(scratch, env=env, expect_exit=1,
                           file_body="version: v1\nflags:\n  resourceConfig: >-\n    gpu:a:2\n")
    assert "a block scalar needs libyaml" in log
    # plain block style still works without it
    f = effective_config(scratch, env=env,
                         file_body="version: v1\nflags:\n  migStrategy: single\n  failOnInitError: no\n")
    assert f["partitionStrategy"] == "single" and f["failOnInitError"] is False
    f = effective_config(scratch, env=env, file_body='{"version": "v1", "flags": {"migStrategy": "mixed"}}')
    assert f["partitionStrategy"] == "mixed"


def _write(scratch, body):
    path = os.path.join(scratch, "config.yaml")
    with open(path, "w") as f:
        f.write(body)
    return path


def test_numbers_are_accepted_for_string_settings(scratch):
    f = effective_config(scratch, file_body="version: v1\nflags:\n  devices: 0\n  resourcePrefix: 1.5\n")
    assert f["devices"] == "0" and f["resourcePrefix"] == "1.5"


def test_sharing_and_health_gate_settings_from_file_and_env(scratch):
    """The round-2 settings have file keys and env names like every other flag
    (the memcap library must exist for enforcement to validate)."""
    from k8s_gpu_sharing_plugin_amd import BUILD_DIR
    shim = os.path.join(BUILD_DIR, "libadp_memcap.so")
    body = f"""
version: v1
flags: {{enforceMemoryUnits: true, memcapLib: "{shim}", replicaHbmShare: yes, prestartHealthCheck: true}}
"""
    f = effective_config(scratch, file_body=body)
    assert f["enforceMemoryUnits"] is True and f["memcapLib"] == shim
    assert f["replicaHbmShare"] is True and f["prestartHealthCheck"] is True
    f = effective_config(scratch, env={"DP_PRESTART_HEALTH_CHECK": "true", "DP_REPLICA_HBM_SHARE": "false"})
    assert f["prestartHealthCheck"] is True and f["replicaHbmShare"] is False and f["enforceMemoryUnits"] is False
