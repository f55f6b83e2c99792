#!/usr/bin/env python3
"""Seed inputs for native/fuzz/fuzz_h2.cc and fuzz_h2_diff.cc (and, for a
directory named h2_client, native/fuzz/fuzz_h2_client.cc): well-formed gRPC exchanges the
fuzzer mutates from, so it starts inside the HTTP/2 state machine instead of
at the frame-header checks. Written to each <dir> given (default
build/fuzz/corpus/h2).

Input layout (fuzz_h2.cc): byte 0 = log2 of the write chunk size, then the
client's frames after the preface and an empty SETTINGS frame."""

import os
import struct
import sys

DATA, HEADERS, PRIORITY, RST, SETTINGS, PING, GOAWAY, WINDOW, CONT = 0, 1, 2, 3, 4, 6, 7, 8, 9
END_STREAM, END_HEADERS, PADDED, PRIO = 1, 4, 8, 0x20


def frame(ftype, flags, sid, payload=b""):
    return struct.pack(">I", len(payload))[1:] + bytes([ftype, flags]) + struct.pack(">I", sid) + payload


def lit(name, value):
    """HPACK literal header field without indexing, new name (0x00)."""
    n, v = name.encode(), value.encode()
    return b"\x00" + bytes([len(n)]) + n + bytes([len(v)]) + v


def request_headers(path):
    return (lit(":method", "POST") + lit(":scheme", "http") + lit(":path", path) +
            lit(":authority", "localhost") + lit("content-type", "application/grpc") + lit("te", "trailers") +
            lit("user-agent", "grpc-go/1.59.0"))


def grpc_msg(body):
    return b"\x00" + struct.pack(">I", len(body)) + body


def seeds():
    echo = request_headers("/t.S/Echo")
    yield "unary", bytes([3]) + frame(HEADERS, END_HEADERS, 1, echo) + frame(DATA, END_STREAM, 1, grpc_msg(b"abc"))
    yield "unary_bytewise", bytes([0]) + frame(HEADERS, END_HEADERS, 1, echo) + frame(DATA, END_STREAM, 1, grpc_msg(b"x"))
    yield "two_calls_ping", (bytes([12]) + frame(HEADERS, END_HEADERS, 1, echo) + frame(DATA, END_STREAM, 1, grpc_msg(b"1")) +
                             frame(PING, 0, 0, b"\x01" * 8) + frame(HEADERS, END_HEADERS, 3, echo) +
                             frame(DATA, END_STREAM, 3, grpc_msg(b"2")))
    yield "continuation", (bytes([5]) + frame(HEADERS, 0, 1, echo[:9]) + frame(CONT, END_HEADERS, 1, echo[9:]) +
                           frame(DATA, END_STREAM, 1, grpc_msg(b"abc")))
    yield "padded_priority", (bytes([15]) + frame(HEADERS, END_HEADERS | PADDED | PRIO, 1,
                                                  b"\x02" + b"\x00\x00\x00\x00\x10" + echo + b"\x00\x00") +
                              frame(DATA, END_STREAM | PADDED, 1, b"\x03" + grpc_msg(b"abc") + b"\x00" * 3))
    watch = request_headers("/t.S/Watch")
    yield "stream_window", (bytes([10]) + frame(HEADERS, END_HEADERS, 1, watch) + frame(DATA, END_STREAM, 1, grpc_msg(b"")) +
                            frame(WINDOW, 0, 0, struct.pack(">I", 1 << 20)) + frame(WINDOW, 0, 1, struct.pack(">I", 1 << 20)))
    yield "settings_rst", (bytes([8]) + frame(SETTINGS, 0, 0, struct.pack(">HI", 4, 1 << 16) + struct.pack(">HI", 5, 1 << 14)) +
                           frame(HEADERS, END_HEADERS, 1, watch) + frame(RST, 0, 1, struct.pack(">I", 8)) +
                           frame(GOAWAY, 0, 0, struct.pack(">II", 1, 0)))
    yield "fail_status", bytes([9]) + frame(HEADERS, END_HEADERS, 1, request_headers("/t.S/Fail")) + frame(DATA, END_STREAM, 1, grpc_msg(b""))
    yield "unknown_path", bytes([9]) + frame(HEADERS, END_HEADERS | END_STREAM, 1, request_headers("/t.S/Nope"))


def client_seeds():
    """fuzz_h2_client.cc: byte 0 = mode (even: a unary call, odd: a server
    stream), then the server's frames after its empty SETTINGS frame."""
    ok = lit(":status", "200") + lit("content-type", "application/grpc")
    trailers = lit("grpc-status", "0")
    yield "unary", (bytes([0]) + frame(SETTINGS, 1, 0) + frame(HEADERS, END_HEADERS, 1, ok) +
                    frame(DATA, 0, 1, grpc_msg(b"pong")) + frame(HEADERS, END_HEADERS | END_STREAM, 1, trailers))
    yield "unary_error", (bytes([0]) + frame(HEADERS, END_HEADERS | END_STREAM, 1,
                                             ok + lit("grpc-status", "3") + lit("grpc-message", "bad%20x")))
    msg = grpc_msg(b"split across frames")
    yield "unary_split", (bytes([2]) + frame(HEADERS, END_HEADERS, 1, ok) + frame(DATA, 0, 1, msg[:3]) +
                          frame(DATA, PADDED, 1, b"\x02" + msg[3:] + b"\x00\x00") +
                          frame(HEADERS, END_HEADERS | END_STREAM, 1, trailers))
    yield "unary_too_large", (bytes([0]) + frame(HEADERS, END_HEADERS, 1, ok) +
                              frame(DATA, 0, 1, b"\x00\x7f\xff\xff\xff" + b"x" * 64))
    yield "stream", (bytes([1]) + frame(HEADERS, END_HEADERS, 1, ok) +
                     b"".join(frame(DATA, 0, 1, grpc_msg(b"m%d" % i)) for i in range(4)) +
                     frame(HEADERS, END_HEADERS | END_STREAM, 1, trailers))
    yield "stream_ping_goaway", (bytes([1]) + frame(PING, 0, 0, b"\x02" * 8) + frame(HEADERS, END_HEADERS, 1, ok) +
                                 frame(DATA, 0, 1, grpc_msg(b"one")) + frame(RST, 0, 1, struct.pack(">I", 8)) +
                                 frame(GOAWAY, 0, 0, struct.pack(">II", 1, 0)))


def main():
    for out in sys.argv[1:] or ["build/fuzz/corpus/h2"]:
        os.makedirs(out, exist_ok=True)
        for name, data in (client_seeds() if os.path.basename(out.rstrip("/")) == "h2_client" else seeds()):
            with open(os.path.join(out, "seed_" + name), "wb") as f:
                f.write(data)


if __name__ == "__main__":
    main()
