"""Hostile and broken peers on the plugin socket: the daemon keeps serving.

The reference relies on grpc-go for all of this; our gRPC layer is our own
(nghttp2 + hand-written framing), so it gets its own abuse tests: garbage bytes,
truncated HTTP/2, random frames after a valid preface, malformed protobuf and
gRPC framing, connection storms and peers vanishing mid-stream. After each, a
normal Allocate must still succeed and the process must still be alive.
"""

import os
import socket
import struct
import threading

import grpc
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"


@pytest.fixture(scope="module")
def plugin(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("robust") / "dp")
    os.makedirs(d)
    k = kubelet.StubKubelet(os.path.join(d, "kubelet.sock")).start()
    dm = harness.Daemon(d).start()
    reg = k.wait_registration()
    sock = os.path.join(d, reg.endpoint)
    c = kubelet.PluginClient(sock)
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    yield dm, sock, c, ids
    c.close()
    dm.stop()
    k.stop()


def _still_serving(dm, c, ids):
    assert dm.proc.poll() is None, "daemon died"
    r = c.allocate([ids[0]], timeout=5)
    assert r.container_responses[0].devices


def _raw(sock_path, payload, read=True, timeout=2.0):
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.settimeout(timeout)
    s.connect(sock_path)
    try:
        s.sendall(payload)
        if read:
            try:
                while s.recv(65536):
                    pass
            except (socket.timeout, ConnectionResetError):
                pass
    except (BrokenPipeError, ConnectionResetError):
        pass
    finally:
        s.close()


def _frame(ftype, flags, sid, payload):
    return struct.pack(">I", len(payload))[1:] + bytes([ftype, flags]) + struct.pack(">I", sid) + payload


def test_garbage_and_truncated_prefaces(plugin):
    dm, sock, c, ids = plugin
    for payload in (b"GET / HTTP/1.1\r\nHost: x\r\n\r\n", b"\x00" * 1000, PREFACE[:10], PREFACE + b"\xff" * 9,
                    os.urandom(4096)):
        _raw(sock, payload)
    _still_serving(dm, c, ids)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(frames=st.lists(st.tuples(st.integers(0, 12), st.integers(0, 255), st.integers(0, 9),
                                 st.binary(max_size=64)), max_size=8))
def test_random_frames_after_preface(plugin, frames):
    dm, sock, c, ids = plugin
    data = PREFACE + _frame(4, 0, 0, b"")  # SETTINGS
    for ftype, flags, sid, payload in frames:
        data += _frame(ftype, flags, sid, payload)
    _raw(sock, data, timeout=0.2)
    assert dm.proc.poll() is None


def test_malformed_grpc_and_protobuf(plugin):
    dm, sock, c, ids = plugin
    ch = grpc.insecure_channel("unix:" + sock)
    raw = ch.unary_unary("/v1beta1.DevicePlugin/Allocate")  # bytes in, bytes out
    for body in (b"\xff\xff\xff", b"\x0a\xff\xff\xff\xff\x0f", b"\x0a\x05\x0a\x03abc", os.urandom(64)):
        with pytest.raises(grpc.RpcError) as e:
            raw(body, timeout=5)
        assert e.value.code() in (grpc.StatusCode.INVALID_ARGUMENT, grpc.StatusCode.INTERNAL)
    with pytest.raises(grpc.RpcError) as e:
        ch.unary_unary("/v1beta1.DevicePlugin/NoSuchMethod")(b"", timeout=5)
    assert e.value.code() == grpc.StatusCode.UNIMPLEMENTED
    ch.close()
    _still_serving(dm, c, ids)


def test_connection_storm_and_abrupt_closes(plugin):
    dm, sock, c, ids = plugin

    def churn():
        for _ in range(25):
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            s.connect(sock)
            s.sendall(PREFACE + _frame(4, 0, 0, b""))
            s.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))  # RST on close
            s.close()
    ts = [threading.Thread(target=churn) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    _still_serving(dm, c, ids)


def test_watchers_vanishing_mid_stream(plugin):
    dm, sock, c, ids = plugin
    for _ in range(20):
        w = kubelet.PluginClient(sock)
        q, call = w.watch()
        q.get(timeout=5)
        w.close()  # drop the connection with the stream open
    _still_serving(dm, c, ids)


def test_oversized_request_is_refused(plugin):
    dm, sock, c, ids = plugin
    ch = grpc.insecure_channel("unix:" + sock, options=[("grpc.max_send_message_length", 64 << 20)])
    raw = ch.unary_unary("/v1beta1.DevicePlugin/Allocate")
    with pytest.raises(grpc.RpcError):
        raw(b"\x0a" + b"\xff" * (17 << 20), timeout=20)
    ch.close()
    _still_serving(dm, c, ids)


def test_descriptor_exhaustion_sheds_connections_without_spinning(tmp_path):
    """At the open-files limit the listener stays readable while connections
    are pending; the daemon sheds them with a reserve descriptor (warning +
    amdgpu_dp_grpc_connections_shed_total) instead of spinning on accept, and
    serves normally once descriptors are free again."""
    import time
    d = str(tmp_path / "dp")
    os.makedirs(d)
    k = kubelet.StubKubelet(os.path.join(d, "kubelet.sock")).start()
    dm = harness.Daemon(d, args=["--server-threads", "1"], nofile=64).start()
    try:
        reg = k.wait_registration()
        path = os.path.join(d, reg.endpoint)
        socks = []
        for _ in range(120):
            s = socket.socket(socket.AF_UNIX)
            s.connect(path)
            socks.append(s)

        def cpu_s():
            f = open(f"/proc/{dm.proc.pid}/stat").read().rsplit(")", 1)[1].split()
            return (int(f[11]) + int(f[12])) / os.sysconf("SC_CLK_TCK")
        time.sleep(0.5)
        c0 = cpu_s()
        time.sleep(1.5)
        assert cpu_s() - c0 < 0.5  # a spinning accept loop burns the whole 1.5 s
        dm.wait_log("out of file descriptors; refused connection #1")
        for s in socks:
            s.close()
        time.sleep(0.3)
        c = kubelet.PluginClient(path)
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        assert len(c.allocate(ids[:1]).container_responses) == 1
        c.close()
        assert dm.proc.poll() is None
    finally:
        dm.stop()
        k.stop()
