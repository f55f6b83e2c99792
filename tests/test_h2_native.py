"""The native HTTP/2 engine (native/src/grpc/h2_conn.cc) at the frame level.

A raw-socket HTTP/2 client drives the protocol corners that gRPC peers (grpc-go
in the kubelet, grpcio here) may use but the end-to-end suites do not force:
CONTINUATION, padding and priority fields, PING and SETTINGS acknowledgements,
a peer that shrinks the stream window to a few bytes and the HPACK table to 0
(server DATA must follow the windows; its next header block must start with a
table size update and must not index), and connection errors answered with
GOAWAY. The server's header blocks use static indices, raw literals and at most
two dynamic-table entries, so a small decoder here follows them exactly.
"""

import os
import socket
import struct

import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"
DATA, HEADERS, PRIORITY, RST_STREAM, SETTINGS, PUSH_PROMISE, PING, GOAWAY, WINDOW_UPDATE, CONTINUATION = range(10)
END_STREAM, ACK, END_HEADERS, PADDED, PRIO = 0x1, 0x1, 0x4, 0x8, 0x20
SVC = "/v1beta1.DevicePlugin/"


def frame(ftype, flags, sid, payload=b""):
    return struct.pack(">I", len(payload))[1:] + bytes([ftype, flags]) + struct.pack(">I", sid) + payload


def hpack_int(v, prefix, first=0):
    mx = (1 << prefix) - 1
    if v < mx:
        return bytes([first | v])
    out = [first | mx]
    v -= mx
    while v >= 128:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    return bytes(out + [v])


def literal(name, value):
    n, v = name.encode(), value.encode()
    return b"\x00" + hpack_int(len(n), 7) + n + hpack_int(len(v), 7) + v


def request_block(method):
    return b"".join(literal(k, v) for k, v in [
        (":method", "POST"), (":scheme", "http"), (":path", SVC + method), (":authority", "localhost"),
        ("content-type", "application/grpc"), ("te", "trailers")])


def pb_len(field, payload):
    return hpack_varint(field << 3 | 2) + hpack_varint(len(payload)) + payload


def hpack_varint(v):
    out = b""
    while v >= 0x80:
        out += bytes([(v & 0x7F) | 0x80])
        v >>= 7
    return out + bytes([v])


def grpc_frame(msg):
    return b"\x00" + struct.pack(">I", len(msg)) + msg


STATIC = {8: (":status", "200"), 31: ("content-type", "")}


def decode_block(b, dyn=None):
    """Server header blocks: indexed fields (static or dynamic), literals with or
    without indexing, size updates. `dyn` is the connection's dynamic table
    (newest first), updated in place."""
    dyn = [] if dyn is None else dyn
    out, i, updates = [], 0, []

    def integer(prefix):
        nonlocal i
        mx = (1 << prefix) - 1
        v = b[i] & mx
        i += 1
        if v < mx:
            return v
        m = 0
        while True:
            c = b[i]
            i += 1
            v += (c & 0x7F) << m
            m += 7
            if not c & 0x80:
                return v

    def string():
        nonlocal i
        assert not b[i] & 0x80, "server header strings are never Huffman-coded"
        n = integer(7)
        s = b[i:i + n].decode()
        i += n
        return s

    def entry(idx):
        return STATIC[idx] if idx < 62 else dyn[idx - 62]
    while i < len(b):
        c = b[i]
        if c & 0x80:
            out.append(entry(integer(7)))
        elif c & 0xC0 == 0x40:  # literal with incremental indexing
            idx = integer(6)
            name = entry(idx)[0] if idx else string()
            field = (name, string())
            dyn.insert(0, field)
            out.append(field)
        elif c & 0xE0 == 0x20:
            size = integer(5)
            updates.append(size)
            if size == 0:
                dyn.clear()
        else:
            assert c & 0xE0 == 0x00, f"unexpected HPACK representation {c:#x}"
            idx = integer(4)
            name = entry(idx)[0] if idx else string()
            out.append((name, string()))
    return out, updates


class Conn:
    def __init__(self, path, settings=b""):
        self.s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.s.settimeout(5)
        self.s.connect(path)
        self.buf = b""
        self.dyn = []  # the server encoder's HPACK dynamic table, as this decoder sees it
        self.s.sendall(PREFACE + frame(SETTINGS, 0, 0, settings))

    def decode(self, block):
        return decode_block(block, self.dyn)

    def send(self, *frames):
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

    def call(self, sid, on_frame=None):
        """Frames of stream `sid` until END_STREAM: (decoded header blocks as
        (fields, size updates), data, all frames). Every HEADERS block is decoded
        in arrival order so the dynamic table stays in step with the server's."""
        blocks, data, seen = [], b"", []
        while True:
            ftype, flags, fsid, payload = self.read_frame()
            seen.append((ftype, flags, fsid, len(payload)))
            if on_frame:
                on_frame(ftype, flags, fsid, payload)
            if ftype == HEADERS:
                decoded = self.decode(payload)
                if fsid == sid:
                    blocks.append(decoded)
            if fsid != sid:
                continue
            elif ftype == DATA:
                data += payload
            if flags & END_STREAM and ftype in (HEADERS, DATA):
                return blocks, data, seen

    def close(self):
        self.s.close()


@pytest.fixture
def plugin(scratch):
    started = []

    def start(fx=None, args=()):
        k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        d = harness.Daemon(scratch, fx or fixtures.node(2), args=list(args)).start()
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        started.append((d, k, c))
        return d, os.path.join(scratch, reg.endpoint), ids
    yield start
    for d, k, c in started:
        c.close()
        d.stop()
        k.stop()


def allocate_msg(ids):
    return grpc_frame(pb_len(1, b"".join(pb_len(1, i.encode()) for i in ids)))


def test_continuation_padding_priority_and_split_data(plugin):
    d, path, ids = plugin()
    c = Conn(path)
    block = request_block("Allocate")
    # HEADERS: padded (3 bytes) + priority fields, first half of the block; CONTINUATION: the rest.
    h = bytes([3]) + struct.pack(">IB", 0, 15) + block[:20] + b"\x00" * 3
    msg = allocate_msg([ids[1]])
    c.send(frame(HEADERS, PADDED | PRIO, 1, h), frame(CONTINUATION, END_HEADERS, 1, block[20:]),
           frame(DATA, PADDED, 1, bytes([4]) + msg[:7] + b"\x00" * 4),
           frame(DATA, END_STREAM, 1, msg[7:]))
    blocks, data, _ = c.call(1)
    heads, _ = blocks[0]
    assert (":status", "200") in heads and ("content-type", "application/grpc") in heads
    trailers, _ = blocks[-1]
    assert ("grpc-status", "0") in trailers
    assert data[0] == 0 and int.from_bytes(data[1:5], "big") == len(data) - 5
    assert b"/dev/kfd" in data and b"renderD136" in data  # GPU 1's render node
    c.close()


def test_ping_settings_ack_and_unknown_frames(plugin):
    d, path, ids = plugin()
    c = Conn(path)
    c.send(frame(0xEE, 0, 0, b"ignored extension frame"), frame(PING, 0, 0, b"12345678"))
    got = set()
    while not {"settings", "settings-ack", "ping"} <= got:
        ftype, flags, sid, payload = c.read_frame()
        if ftype == SETTINGS and not flags & ACK:
            got.add("settings")
            params = {struct.unpack(">H", payload[i:i + 2])[0]: struct.unpack(">I", payload[i + 2:i + 6])[0]
                      for i in range(0, len(payload), 6)}
            assert params[0x3] == 1024 and params[0x4] == 1 << 20  # MAX_CONCURRENT_STREAMS, INITIAL_WINDOW_SIZE
        elif ftype == SETTINGS:
            got.add("settings-ack")
        elif ftype == PING:
            assert flags & ACK and payload == b"12345678"
            got.add("ping")
    # Unknown method and bad content-type: trailers-only gRPC errors, connection stays up.
    c.send(frame(HEADERS, END_HEADERS | END_STREAM, 1, request_block("Nope")))
    blocks, _, _ = c.call(1)
    fields = dict(blocks[0][0])
    assert fields["grpc-status"] == "12" and "unknown method" in fields["grpc-message"]
    c.send(frame(HEADERS, END_HEADERS, 3, request_block("Allocate")),
           frame(DATA, END_STREAM, 3, allocate_msg([ids[0]])))
    blocks, data, _ = c.call(3)
    assert ("grpc-status", "0") in blocks[-1][0] and b"/dev/kfd" in data
    # From now on both repeated fields come from the dynamic table: 2 + 1 bytes of headers.
    c.send(frame(HEADERS, END_HEADERS, 5, request_block("Allocate")),
           frame(DATA, END_STREAM, 5, allocate_msg([ids[1]])))
    blocks, data, seen = c.call(5)
    assert [n for t, f, sid, n in seen if t == HEADERS and sid == 5] == [2, 1]
    assert (":status", "200") in blocks[0][0] and ("content-type", "application/grpc") in blocks[0][0]
    assert blocks[-1][0] == [("grpc-status", "0")]
    c.close()


def test_tiny_windows_and_zero_header_table(plugin):
    """A peer with a 1000-byte stream window and an HPACK table of 0: the 154 KB
    ListAndWatch of a 2,352-unit node arrives in window-sized DATA frames as the
    peer grants credit, and the response header block opens with a size update."""
    d, path, ids = plugin(fixtures.node(8), ["--resource-config", "gpu:gpu-mem-gb:-1"])
    assert len(ids) == 2352
    win = 1000
    c = Conn(path, struct.pack(">HI", 0x1, 0) + struct.pack(">HI", 0x4, win))
    c.send(frame(HEADERS, END_HEADERS, 1, request_block("ListAndWatch")), frame(DATA, END_STREAM, 1, b""))
    blocks, data, frames = [], b"", 0
    while len(data) < 5 or len(data) < 5 + int.from_bytes(data[1:5], "big"):
        ftype, flags, sid, payload = c.read_frame()
        if sid != 1:
            continue
        if ftype == HEADERS:
            blocks.append(c.decode(payload))
        elif ftype == DATA:
            assert len(payload) <= win, "DATA beyond the stream window"
            data += payload
            frames += 1
            # grant exactly what was consumed, on the stream and the connection
            c.send(frame(WINDOW_UPDATE, 0, 1, struct.pack(">I", len(payload))),
                   frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", len(payload))))
    heads, updates = blocks[0]
    assert updates == [0] and (":status", "200") in heads
    assert frames >= len(data) // win and len(data) > 150_000
    assert data.count(b"-replica-") == 2352
    c.close()


@pytest.mark.parametrize("bad", [
    frame(DATA, 0, 0, b"x"),                               # DATA on stream 0
    frame(HEADERS, END_HEADERS, 2, b""),                   # even (server-initiated) stream id
    frame(PUSH_PROMISE, END_HEADERS, 1, b"\x00" * 4),      # clients never push
    frame(SETTINGS, 0, 0, b"\x00\x04\x80\x00\x00\x00"),    # INITIAL_WINDOW_SIZE > 2^31-1
    frame(HEADERS, 0, 1, b"\x82") + frame(PING, 0, 0, b"8 bytes!"),  # CONTINUATION expected
    frame(PING, 0, 0, b"short"),                           # PING length
    frame(HEADERS, END_HEADERS, 1, b"\xff\xff\xff\xff\x0f"),  # undecodable HPACK
])
def test_connection_errors_are_answered_with_goaway(plugin, bad):
    d, path, ids = plugin()
    c = Conn(path)
    c.send(bad)
    while True:
        try:
            ftype, flags, sid, payload = c.read_frame()
        except (ConnectionError, socket.timeout, ConnectionResetError):
            pytest.fail("connection closed without GOAWAY")
        if ftype == GOAWAY:
            assert struct.unpack(">I", payload[4:8])[0] != 0  # an error code, not NO_ERROR
            break
    c.close()
    # the daemon keeps serving
    c2 = Conn(path)
    c2.send(frame(HEADERS, END_HEADERS, 1, request_block("Allocate")), frame(DATA, END_STREAM, 1, allocate_msg(ids[:1])))
    blocks, data, _ = c2.call(1)
    assert ("grpc-status", "0") in blocks[-1][0]
    c2.close()


def test_rst_stream_cancels_a_watch(plugin):
    d, path, ids = plugin()
    c = Conn(path)
    c.send(frame(HEADERS, END_HEADERS, 1, request_block("ListAndWatch")), frame(DATA, END_STREAM, 1, b""))
    while True:
        ftype, flags, sid, payload = c.read_frame()
        if ftype == HEADERS:
            c.decode(payload)
        if sid == 1 and ftype == DATA:
            break
    c.send(frame(RST_STREAM, 0, 1, struct.pack(">I", 8)),  # CANCEL
           frame(HEADERS, END_HEADERS, 3, request_block("Allocate")), frame(DATA, END_STREAM, 3, allocate_msg(ids[:1])))
    blocks, data, _ = c.call(3)
    assert ("grpc-status", "0") in blocks[-1][0]
    c.close()


def test_ping_flood_without_reading_is_cut_off(plugin):
    """A peer that floods PINGs and never reads the ACKs is disconnected once the
    queued output passes the cap; the daemon keeps serving others."""
    d, path, ids = plugin()
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
    s.settimeout(10)
    s.connect(path)
    s.sendall(PREFACE + frame(SETTINGS, 0, 0))
    burst = frame(PING, 0, 0, b"flooding") * 4096
    sent = 0
    try:
        while sent < (200 << 20):  # far more ACK bytes than the cap
            s.sendall(burst)
            sent += len(burst)
    except (BrokenPipeError, ConnectionResetError):
        pass
    s.close()
    assert sent < (200 << 20), "the flooding peer was never disconnected"
    assert d.proc.poll() is None
    c2 = Conn(path)
    c2.send(frame(HEADERS, END_HEADERS, 1, request_block("Allocate")), frame(DATA, END_STREAM, 1, allocate_msg(ids[:1])))
    blocks, data, _ = c2.call(1)
    assert ("grpc-status", "0") in blocks[-1][0]
    c2.close()


def test_a_peer_that_keeps_sending_after_a_connection_error_is_cut_off(plugin):
    """After a connection error the daemon drops what the peer sends until it
    stops, then writes its GOAWAY and closes; a peer that never stops is cut
    off after 64 MiB. Before the bound, a peer faster than the daemon kept its
    loop reading and dropping for ever (it never saw EAGAIN) -- a TSan run,
    where the daemon is the slower side, caught that through the PING-flood
    test; on a fast machine the daemon usually sees EAGAIN first. Either way
    the peer is disconnected and the daemon keeps serving others."""
    d, path, ids = plugin()
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.settimeout(20)
    s.connect(path)
    s.sendall(PREFACE + frame(SETTINGS, 0, 0) + frame(PING, 0, 1, b"onstream"))  # PING on a stream: error
    junk = b"\x00" * (1 << 20)
    sent = 0
    try:
        while sent < (256 << 20):
            s.sendall(junk)
            sent += len(junk)
    except (BrokenPipeError, ConnectionResetError):
        pass
    s.close()
    assert sent < (256 << 20), "the peer was never cut off"
    assert d.proc.poll() is None
    c2 = Conn(path)
    c2.send(frame(HEADERS, END_HEADERS, 1, request_block("Allocate")), frame(DATA, END_STREAM, 1, allocate_msg(ids[:1])))
    blocks, data, _ = c2.call(1)
    assert ("grpc-status", "0") in blocks[-1][0]
    c2.close()


def test_buffered_request_bytes_are_capped(plugin):
    """Streams that keep sending request bytes without ever ending are cut off at
    64 MiB buffered per connection (GOAWAY ENHANCE_YOUR_CALM)."""
    d, path, ids = plugin()
    c = Conn(path)
    payload = b"\x00" * 60000
    got_goaway = None
    try:
        for n in range(80):
            sid = 1 + 2 * n
            c.send(frame(HEADERS, END_HEADERS, sid, request_block("Allocate")),
                   *[frame(DATA, 0, sid, payload) for _ in range(18)])  # ~1 MiB, stream left open
    except (BrokenPipeError, ConnectionResetError):
        pass
    try:
        while got_goaway is None:
            ftype, flags, sid, p = c.read_frame()
            if ftype == GOAWAY:
                got_goaway = struct.unpack(">I", p[4:8])[0]
    except (ConnectionError, socket.timeout, ConnectionResetError):
        pass
    assert got_goaway == 11
    c.close()
    assert d.proc.poll() is None
