"""grpc-go-shaped HTTP/2 clients against both plugin engines.

The kubelet talks to a device plugin with grpc-go (reference server.go:168-240,
vendor/google.golang.org/grpc). Go is not in this image, so this scripts, at
the frame level, what grpc-go's transport does and the other suites do not:

* its preface: SETTINGS immediately followed by a connection WINDOW_UPDATE,
  before the server's SETTINGS has been acknowledged;
* BDP estimation: a PING with grpc-go's payload after DATA, interleaved with
  WINDOW_UPDATEs (connection updates as data arrives, stream updates as the
  application reads);
* request headers as grpc-go's HPACK encoder writes them -- Huffman strings,
  incremental indexing, `te: trailers`, `grpc-timeout`, `user-agent: grpc-go/...`
  -- produced here by nghttp2's deflater (same encoding rules), so the dynamic
  table is reused over 10,000 calls on one connection;
* a 2,352-ID ListAndWatch read through grpc-go's default 64 KiB stream window
  with stream credit withheld for a while (a slow reader), during which unary
  calls on the same connection must still complete;
* GOAWAY from the client when the kubelet shuts down, with a watch still open.

Every case runs on both engines (--http2-server native | nghttp2). Server
header blocks are decoded with nghttp2's inflater. Parity for grpc-go itself
stays unpinned (no Go toolchain); this pins its observable wire behaviour.
"""

import ctypes
import os
import socket
import struct
import threading
import time

import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

from test_h2_native import (ACK, CONTINUATION, DATA, END_HEADERS, END_STREAM, GOAWAY, HEADERS, PING, PREFACE,
                            RST_STREAM, SETTINGS, SVC, WINDOW_UPDATE, allocate_msg, frame)

BDP_PING = bytes([2, 4, 16, 16, 9, 14, 7, 7])  # grpc-go's bdpPing payload
GO_UA = "grpc-go/1.50.1"
DEFAULT_WINDOW = 65535


class _NV(ctypes.Structure):
    _fields_ = [("name", ctypes.c_void_p), ("value", ctypes.c_void_p), ("namelen", ctypes.c_size_t),
                ("valuelen", ctypes.c_size_t), ("flags", ctypes.c_uint8)]


_ng = ctypes.CDLL("libnghttp2.so.14")
_ng.nghttp2_hd_deflate_new.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
_ng.nghttp2_hd_deflate_hd.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_NV),
                                      ctypes.c_size_t]
_ng.nghttp2_hd_deflate_hd.restype = ctypes.c_ssize_t
_ng.nghttp2_hd_deflate_del.argtypes = [ctypes.c_void_p]
_ng.nghttp2_hd_inflate_new.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
_ng.nghttp2_hd_inflate_hd2.argtypes = [ctypes.c_void_p, ctypes.POINTER(_NV), ctypes.POINTER(ctypes.c_int),
                                       ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
_ng.nghttp2_hd_inflate_hd2.restype = ctypes.c_ssize_t
_ng.nghttp2_hd_inflate_end_headers.argtypes = [ctypes.c_void_p]
_ng.nghttp2_hd_inflate_del.argtypes = [ctypes.c_void_p]


class Hpack:
    """nghttp2's HPACK deflater (Huffman + incremental indexing, like
    golang.org/x/net/http2/hpack's Encoder) and inflater for server blocks."""

    def __init__(self):
        self.d, self.i = ctypes.c_void_p(), ctypes.c_void_p()
        assert _ng.nghttp2_hd_deflate_new(ctypes.byref(self.d), 4096) == 0
        assert _ng.nghttp2_hd_inflate_new(ctypes.byref(self.i)) == 0

    def encode(self, fields):
        bufs = [(k.encode(), v.encode()) for k, v in fields]
        nva = (_NV * len(bufs))()
        keep = []
        for j, (k, v) in enumerate(bufs):
            kb, vb = ctypes.create_string_buffer(k, len(k)), ctypes.create_string_buffer(v, len(v))
            keep += [kb, vb]
            nva[j] = _NV(ctypes.cast(kb, ctypes.c_void_p), ctypes.cast(vb, ctypes.c_void_p), len(k), len(v), 0)
        out = ctypes.create_string_buffer(4096)
        n = _ng.nghttp2_hd_deflate_hd(self.d, out, 4096, nva, len(bufs))
        assert n > 0, n
        return out.raw[:n]

    def decode(self, block):
        fields, pos = [], 0
        nv, flags = _NV(), ctypes.c_int(0)
        while True:
            rest = block[pos:]
            n = _ng.nghttp2_hd_inflate_hd2(self.i, ctypes.byref(nv), ctypes.byref(flags), rest, len(rest), 1)
            assert n >= 0, f"server header block does not decode ({n})"
            pos += n
            if flags.value & 0x02:  # NGHTTP2_HD_INFLATE_EMIT
                fields.append((ctypes.string_at(nv.name, nv.namelen).decode(),
                               ctypes.string_at(nv.value, nv.valuelen).decode()))
            if flags.value & 0x01:  # NGHTTP2_HD_INFLATE_FINAL
                _ng.nghttp2_hd_inflate_end_headers(self.i)
                return fields
            if n == 0 and not flags.value & 0x02:
                raise AssertionError("inflater made no progress")

    def close(self):
        _ng.nghttp2_hd_deflate_del(self.d)
        _ng.nghttp2_hd_inflate_del(self.i)


def go_request(method, timeout="9999863u"):
    return [(":method", "POST"), (":scheme", "http"), (":path", SVC + method), (":authority", "localhost"),
            ("content-type", "application/grpc"), ("user-agent", GO_UA), ("te", "trailers"),
            ("grpc-timeout", timeout)]


class GoConn:
    """A raw HTTP/2 connection that behaves like grpc-go's client transport."""

    def __init__(self, path, conn_window_delta=(1 << 20) - DEFAULT_WINDOW, settings=b""):
        self.s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.s.settimeout(10)
        self.s.connect(path)
        self.buf = b""
        self.hp = Hpack()
        self.next_sid = 1
        self.pings_acked = 0
        self.pings_sent = 0
        self.server_settings_seen = False
        self.lock = threading.Lock()
        first = PREFACE + frame(SETTINGS, 0, 0, settings)
        if conn_window_delta:  # before the server's SETTINGS is even read
            first += frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", conn_window_delta))
        self.s.sendall(first)

    def send(self, *frames):
        with self.lock:
            self.s.sendall(b"".join(frames))

    def read_frame(self):
        while len(self.buf) < 9 or len(self.buf) < 9 + int.from_bytes(self.buf[:3], "big"):
            chunk = self.s.recv(1 << 20)
            if not chunk:
                raise ConnectionError("closed")
            self.buf += chunk
        n = int.from_bytes(self.buf[:3], "big")
        f = (self.buf[3], self.buf[4], int.from_bytes(self.buf[5:9], "big") & 0x7FFFFFFF, self.buf[9:9 + n])
        self.buf = self.buf[9 + n:]
        return f

    def handle_control(self, ftype, flags, payload):
        """What grpc-go's reader does for connection-level frames."""
        if ftype == SETTINGS and not flags & ACK:
            self.server_settings_seen = True
            self.send(frame(SETTINGS, ACK, 0))
        elif ftype == PING and flags & ACK:
            assert payload == BDP_PING, payload
            self.pings_acked += 1
        elif ftype == PING:
            self.send(frame(PING, ACK, 0, payload))

    def open(self, method, msg, end=True):
        sid = self.next_sid
        self.next_sid += 2
        block = self.hp.encode(go_request(method))
        # grpc-go splits header blocks larger than the peer's max frame size; ours are small.
        self.send(frame(HEADERS, END_HEADERS, sid, block),
                  frame(DATA, END_STREAM if end else 0, sid, msg))
        return sid

    def unary(self, method, msg, bdp=True):
        sid = self.open(method, msg)
        return self.finish(sid, bdp)

    def finish(self, sid, bdp=True):
        heads, data = [], b""
        while True:
            ftype, flags, fsid, payload = self.read_frame()
            if fsid == 0:
                self.handle_control(ftype, flags, payload)
                continue
            if ftype == HEADERS:
                assert flags & END_HEADERS  # servers here never need CONTINUATION for these
                fields = self.hp.decode(payload)
                if fsid == sid:
                    heads.append(fields)
            elif ftype == DATA and fsid == sid:
                data += payload
                if payload:
                    upd = frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", len(payload))) + \
                        frame(WINDOW_UPDATE, 0, sid, struct.pack(">I", len(payload)))
                    if bdp:
                        self.pings_sent += 1
                        upd += frame(PING, 0, 0, BDP_PING)
                    self.send(upd)
            elif ftype == RST_STREAM and fsid == sid:
                raise AssertionError(f"stream {sid} reset: {payload.hex()}")
            if fsid == sid and flags & END_STREAM and ftype in (HEADERS, DATA):
                return heads, data

    def close(self):
        self.s.close()
        self.hp.close()


ENGINES = ["native", "nghttp2"]


@pytest.fixture
def plugin(scratch):
    started = []

    def start(engine, fx=None, args=()):
        k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        d = harness.Daemon(scratch, fx or fixtures.node(2), args=["--http2-server", engine, *args]).start()
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        c.close()
        started.append((d, k))
        return d, os.path.join(scratch, reg.endpoint), ids
    yield start
    for d, k in started:
        assert d.stop() == 0, d.log()[-3000:]
        k.stop()


def status_of(heads):
    trailers = dict(heads[-1])
    return trailers.get("grpc-status"), trailers.get("grpc-message")


@pytest.mark.parametrize("engine", ENGINES)
def test_preface_window_update_and_bdp_pings(plugin, engine):
    d, path, ids = plugin(engine)
    c = GoConn(path)
    # The first call goes out before the server's SETTINGS was read or acked.
    heads, data = c.unary("Allocate", allocate_msg([ids[0]]))
    assert status_of(heads) == ("0", None)
    assert (":status", "200") in heads[0] and ("content-type", "application/grpc") in heads[0]
    assert b"/dev/kfd" in data
    heads, data = c.unary("GetDevicePluginOptions", b"\x00\x00\x00\x00\x00")
    assert status_of(heads)[0] == "0"
    # Drain: every BDP ping is acknowledged with its payload.
    deadline = time.monotonic() + 5
    c.s.settimeout(0.5)
    while c.pings_acked < c.pings_sent and time.monotonic() < deadline:
        try:
            ftype, flags, sid, payload = c.read_frame()
        except socket.timeout:
            continue
        if sid == 0:
            c.handle_control(ftype, flags, payload)
    assert c.server_settings_seen and c.pings_sent >= 2 and c.pings_acked == c.pings_sent
    c.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_hpack_dynamic_table_reuse_over_10k_calls(plugin, engine):
    d, path, ids = plugin(engine)
    c = GoConn(path)
    sizes = []
    for i in range(10_000):
        sid = c.next_sid
        # grpc-go sends the remaining deadline, a new value per call: with
        # incremental indexing every call adds a table entry and evicts old ones.
        block = c.hp.encode(go_request("Allocate", timeout=f"{9_999_999 - 7 * i}u"))
        sizes.append(len(block))
        c.next_sid += 2
        c.send(frame(HEADERS, END_HEADERS, sid, block), frame(DATA, END_STREAM, sid, allocate_msg([ids[i % 2]])))
        heads, data = c.finish(sid, bdp=(i % 1000 == 0))
        assert status_of(heads) == ("0", None), (i, heads)
        assert data.count(b"/dev/kfd") == 2  # container path + host path
    # Huffman + indexing: the first block carries every string; later ones are
    # indexed fields plus the (Huffman) :path and grpc-timeout literals -- the
    # server's decoder tracks the table through ~10k insertions and evictions.
    # (Evicted entries are re-sent as literals now and then.)
    later = sorted(sizes[1:])
    assert sizes[0] > 80 and later[len(later) // 2] <= 40 and later[-1] <= sizes[0], (sizes[0], later[-1])
    assert sum(1 for n in sizes if n > 60) < 200  # re-sends are rare
    c.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_concurrent_streams_on_one_connection(plugin, engine):
    """grpc-go multiplexes concurrent unary calls: 64 streams in flight."""
    d, path, ids = plugin(engine)
    c = GoConn(path)
    sids = [c.open("Allocate", allocate_msg([ids[j % 2]])) for j in range(64)]
    done, heads_of = set(), {}
    while len(done) < len(sids):
        ftype, flags, sid, payload = c.read_frame()
        if sid == 0:
            c.handle_control(ftype, flags, payload)
            continue
        if ftype == HEADERS:
            heads_of.setdefault(sid, []).append(c.hp.decode(payload))
        elif ftype == DATA and payload:
            c.send(frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", len(payload))))
        if flags & END_STREAM:
            done.add(sid)
    assert all(status_of(heads_of[s]) == ("0", None) for s in sids)
    c.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_large_watch_through_64k_window_with_a_slow_reader(plugin, engine):
    """2,352 IDs (~154 KB) through grpc-go's default 65,535-byte stream window.
    The reader withholds stream credit for 0.4 s after the window fills (the
    connection credit flows as data arrives); unary calls on other streams of
    the same connection complete meanwhile; then the watch completes."""
    d, path, ids = plugin(engine, fixtures.node(8), ["--resource-config", "gpu:gpu-mem-gb:-1"])
    assert len(ids) == 2352
    c = GoConn(path, conn_window_delta=0)
    law = c.open("ListAndWatch", b"", end=True)
    got, stalled_at, unary_done, law_heads = b"", None, 0, []
    stream_credit_owed = 0
    while len(got) < 5 or len(got) < 5 + int.from_bytes(got[1:5], "big"):
        if stalled_at is not None and time.monotonic() - stalled_at > 0.4 and stream_credit_owed:
            c.send(frame(WINDOW_UPDATE, 0, law, struct.pack(">I", stream_credit_owed)))
            stream_credit_owed = 0
        c.s.settimeout(0.05)
        try:
            ftype, flags, sid, payload = c.read_frame()
        except socket.timeout:
            if stalled_at is None and len(got) >= DEFAULT_WINDOW - 5:
                stalled_at = time.monotonic()
                # the stream is stalled on its window: unary calls still get through
                for j in range(20):
                    heads, data = c.unary("Allocate", allocate_msg([ids[j]]), bdp=False)
                    assert status_of(heads) == ("0", None)
                    unary_done += 1
            continue
        finally:
            c.s.settimeout(10)
        if sid == 0:
            c.handle_control(ftype, flags, payload)
        elif ftype == HEADERS and sid == law:
            law_heads.append(c.hp.decode(payload))
        elif ftype == DATA and sid == law:
            assert len(got) + len(payload) <= DEFAULT_WINDOW or stalled_at is not None, \
                "DATA beyond the stream window"
            got += payload
            # connection credit right away, stream credit only after the stall
            c.send(frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", len(payload))))
            if stalled_at is None:
                stream_credit_owed += len(payload)
            else:
                c.send(frame(WINDOW_UPDATE, 0, law, struct.pack(">I", len(payload))))
    assert stalled_at is not None and unary_done == 20
    assert (":status", "200") in law_heads[0]
    assert got.count(b"-replica-") == 2352
    c.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_goaway_from_a_shutting_down_kubelet(plugin, engine):
    d, path, ids = plugin(engine)
    c = GoConn(path)
    law = c.open("ListAndWatch", b"", end=True)
    # first ListAndWatch response arrives
    while True:
        ftype, flags, sid, payload = c.read_frame()
        if sid == 0:
            c.handle_control(ftype, flags, payload)
        elif ftype == DATA and sid == law and payload:
            break
    # grpc-go's Close(): GOAWAY(NO_ERROR, last stream 0), then the socket closes
    c.send(frame(GOAWAY, 0, 0, struct.pack(">II", 0, 0) + b"client shutdown"))
    c.close()
    time.sleep(0.2)
    assert d.proc.poll() is None, "daemon died on a client GOAWAY"
    c2 = GoConn(path)
    heads, data = c2.unary("Allocate", allocate_msg([ids[1]]))
    assert status_of(heads) == ("0", None)
    c2.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_header_block_split_over_continuation_with_huffman(plugin, engine):
    """A header block split across HEADERS + CONTINUATION mid-Huffman-string."""
    d, path, ids = plugin(engine)
    c = GoConn(path)
    block = c.hp.encode(go_request("Allocate") + [("x-padding", "p" * 300)])
    cut = len(block) // 2
    c.send(frame(HEADERS, 0, 1, block[:cut]), frame(CONTINUATION, END_HEADERS, 1, block[cut:]),
           frame(DATA, END_STREAM, 1, allocate_msg([ids[0]])))
    c.next_sid = 3
    heads, data = c.finish(1)
    assert status_of(heads) == ("0", None) and b"/dev/kfd" in data
    c.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_request_trailers_do_not_change_the_call(plugin, engine):
    """A client trailer block (HEADERS + END_STREAM after the DATA) that names
    :path or content-type again does not re-route or re-type the call: the
    nghttp2 engine used to take the trailers' :path (found by
    native/fuzz/fuzz_h2_diff.cc, where the two engines disagreed)."""
    d, path, ids = plugin(engine)
    c = GoConn(path)
    block = c.hp.encode(go_request("Allocate"))
    trailers = c.hp.encode([(":path", SVC + "NoSuchMethod"), ("content-type", "text/plain")])
    c.send(frame(HEADERS, END_HEADERS, 1, block), frame(DATA, 0, 1, allocate_msg([ids[0]])),
           frame(HEADERS, END_HEADERS | END_STREAM, 1, trailers))
    c.next_sid = 3
    heads, data = c.finish(1)
    assert status_of(heads) == ("0", None) and b"/dev/kfd" in data
    c.close()
