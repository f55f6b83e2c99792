"""Hand-written protobuf codec vs. the protobuf library (independent implementation).

Messages are built and serialized by google.protobuf (classes from
proto/deviceplugin/v1beta1/api.proto via protoc), decoded and re-encoded by the
daemon's C++ codec, and parsed back by protobuf.
"""

from hypothesis import given, settings, strategies as st

from k8s_gpu_sharing_plugin_amd.utils import kubelet, native

M = kubelet.messages()
ids = st.lists(st.text(alphabet="abcdef0123456789-", min_size=0, max_size=40), max_size=12)
text = st.text(max_size=30)


def roundtrip(kind, msg):
    data = msg.SerializeToString()
    out = native.proto_roundtrip(kind, data)
    back = type(msg).FromString(out)
    assert back == msg
    return data, out


def test_allocate_response_bytes_identical():
    r = M["AllocateResponse"]()
    c = r.container_responses.add()
    c.envs["AMD_VISIBLE_DEVICES"] = "a,b"
    m = c.mounts.add(container_path="/var/run/amd-container-devices/a", host_path="/dev/null", read_only=True)
    assert m.read_only
    c.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
    c.devices.add(container_path="/dev/dri/renderD128", host_path="/dev/dri/renderD128", permissions="rw")
    c.annotations["k"] = "v"
    c.cdi_devices.add(name="amd.com/gpu=a")
    data, out = roundtrip("allocate_response", r)
    assert data == out  # canonical field order, single-entry maps


def test_law_register_options_prestart():
    law = M["ListAndWatchResponse"]()
    d = law.devices.add(ID="id-0", health="Healthy")
    d.topology.nodes.add(ID=1)
    law.devices.add(ID="id-1", health="Unhealthy")
    data, out = roundtrip("law_response", law)
    assert data == out
    reg = M["RegisterRequest"](version="v1beta1", endpoint="amd-gpu.sock", resource_name="amd.com/gpu")
    reg.options.get_preferred_allocation_available = True
    assert roundtrip("register_request", reg)[1] == reg.SerializeToString()
    o = M["DevicePluginOptions"](pre_start_required=True, get_preferred_allocation_available=True)
    roundtrip("options", o)
    roundtrip("prestart_request", M["PreStartContainerRequest"](devicesIDs=["a", "b"]))


def test_empty_messages():
    assert native.proto_roundtrip("allocate_request", b"") == b""
    assert native.proto_roundtrip("law_response", b"") == b""


def test_unknown_fields_are_skipped():
    # field 15 varint + field 16 fixed64 + field 17 fixed32 ahead of a known field
    data = bytes([0x78, 0x05, 0x81, 0x01]) + b"\x00" * 8 + bytes([0x8d, 0x01]) + b"\x00" * 4
    data += M["AllocateRequest"](container_requests=[M["ContainerAllocateRequest"](devicesIDs=["x"])]).SerializeToString()
    out = native.proto_roundtrip("allocate_request", data)
    assert M["AllocateRequest"].FromString(out).container_requests[0].devicesIDs == ["x"]


@settings(max_examples=150, deadline=None)
@given(st.lists(ids, max_size=4))
def test_fuzz_allocate_request(containers):
    r = M["AllocateRequest"]()
    for c in containers:
        r.container_requests.add().devicesIDs.extend(c)
    roundtrip("allocate_request", r)


@settings(max_examples=150, deadline=None)
@given(st.lists(st.tuples(ids, ids, st.integers(-2**31, 2**31 - 1)), max_size=3))
def test_fuzz_preferred_request(reqs):
    r = M["PreferredAllocationRequest"]()
    for avail, must, size in reqs:
        c = r.container_requests.add(allocation_size=size)
        c.available_deviceIDs.extend(avail)
        c.must_include_deviceIDs.extend(must)
    roundtrip("preferred_request", r)


@settings(max_examples=100, deadline=None)
@given(st.lists(st.tuples(st.dictionaries(text, text, max_size=3), ids), max_size=3))
def test_fuzz_allocate_response(items):
    r = M["AllocateResponse"]()
    for envs, paths in items:
        c = r.container_responses.add()
        for k, v in envs.items():
            c.envs[k] = v
        for p in paths:
            c.devices.add(container_path=p, host_path=p, permissions="rw")
    roundtrip("allocate_response", r)


@settings(max_examples=300, deadline=None)
@given(st.binary(max_size=64))
def test_garbage_never_crashes(blob):
    for kind in ("allocate_request", "preferred_request", "law_response", "allocate_response"):
        try:
            native.proto_roundtrip(kind, blob)
        except native.NativeError:
            pass
