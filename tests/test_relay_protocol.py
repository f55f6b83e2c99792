"""The event relay's replay contract, spoken to the real relay by a raw client.

A daemon that (re)connects sends "reinit fp=<fp> since=<relay>:<seq>:<gen>"
with the cursor of the last event it handled. The relay (relay.cc Subscribe)
replays every event it still holds after that cursor, then answers with a
"hello v1 reinit ... gap=<0|1>": gap=0 only when nothing can have been missed --
the same relay instance, the same registration generation, a cursor it has not
passed beyond its ring (kRelayRingSize = 1024 events) and no event lost after
it. The daemon-level tests (test_event_relay.py) and the model checker
(native/tests/health_model.cc, whose relay is a model of Subscribe with a ring
that never overflows) cover what the daemon does with the answer; these pin the
relay's side of the wire exactly, fence posts included: ring overflow, a lost
event, a cursor from another relay / generation / the future, a malformed or
over-long request, an unplaceable event's line.

Reference: the reference has no relay -- its plugin registers NVML events
itself (/root/reference/cmd/nvidia-device-plugin/nvidia.go:181-269).
"""

import os
import re
import socket
import time

import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness

RING = 1024  # kRelayRingSize (native/src/health/relay.h)
HELLO = re.compile(r"hello v1 (reinit )?(events=\S+)(?: processors=(\d+))? relay=(\w+) gen=(\d+) seq=(\d+) fp=(\S+)"
                   r" renew_ms=\d+(?: gap=(\d))?(?: reason=(.*))?")
EVENT = re.compile(r"event seq=(\d+) node=(\S+) bdf=(\S+) part=(\d+) type=(\d+) ?(.*)")


class Relay:
    """The relay alone (no daemon) on the mock, events injected through its FIFO."""

    def __init__(self, scratch, env=None):
        fdir = scratch + ".fixture"
        os.makedirs(fdir, exist_ok=True)
        self.state = os.path.join(fdir, "state")  # the mock's runtime knobs
        os.makedirs(self.state, exist_ok=True)
        self.fifo = os.path.join(fdir, "events")
        os.mkfifo(self.fifo)
        self.sock = os.path.join(fdir, "events.sock")
        self.fx = dict(fixtures.node(2), events_open_kfd=True)
        self.d = harness.Daemon(scratch, self.fx, args=["--event-relay", "--health-event-socket", self.sock],
                                env=env, event_fifo=self.fifo, state_dir=self.state).start()
        self.clients = []
        try:
            self.d.wait_log("event notification registered on")
        except BaseException:
            self.d.stop()
            raise

    def inject(self, lines):
        fd = os.open(self.fifo, os.O_WRONLY | os.O_NONBLOCK)
        try:
            os.write(fd, "".join(ln + "\n" for ln in lines).encode())
        finally:
            os.close(fd)

    def events(self, n, prefix="e"):
        """n events (GPU 0 / GPU 1 alternating, a VM fault: no verdict anywhere),
        in chunks the relay's pipes keep up with; waits until all are numbered."""
        seq0, log0 = self.hello()["seq"], len(self.d.log())
        chunk = 200  # (~22 KB of lines: well inside the relay's 64 KiB event pipe)
        for i in range(0, n, chunk):
            self.inject([f"{(i + j) % 2} 1 {prefix}{i + j}" for j in range(min(chunk, n - i))])
            deadline = time.time() + 10
            while self.hello()["seq"] < seq0 + min(n, i + chunk):
                assert time.time() < deadline, self.d.log()[-3000:]
                time.sleep(0.01)
        assert "lost after" not in self.d.log()[log0:]

    def connect(self):
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(10)
        s.connect(self.sock)
        self.clients.append(s)
        return s, s.makefile("r", encoding="utf-8", newline="\n")

    def hello(self):
        """The greeting a fresh connection gets: relay id, generation, last seq."""
        s, f = self.connect()
        m = HELLO.fullmatch(f.readline().rstrip("\n"))
        s.close()
        self.clients.remove(s)
        assert m and not m.group(1), m
        return {"events": m.group(2), "relay": m.group(4), "gen": int(m.group(5)), "seq": int(m.group(6))}

    def subscribe(self, since=None, raw=None):
        """Sends a reinit; returns (replayed event lines, the reinit hello's
        fields) -- everything up to and including the registrar's answer."""
        s, f = self.connect()
        greeting = f.readline()
        g = HELLO.fullmatch(greeting.rstrip("\n"))
        assert g, greeting
        # The daemon's processor fingerprint, as it would send it (the
        # registration's: no renewal, so the generation stays).
        fp = g.group(7)
        line = (raw if raw is not None else "reinit fp={fp}" + (f" since={since}" if since else "")).format(fp=fp)
        s.sendall((line + "\n").encode())
        replay = []
        while True:
            ln = f.readline().rstrip("\n")
            assert ln, "connection closed before the reinit hello"
            m = HELLO.fullmatch(ln)
            if m and m.group(1):
                return replay, {"events": m.group(2), "gen": int(m.group(5)), "seq": int(m.group(6)),
                                "gap": int(m.group(8)) if m.group(8) is not None else None, "reason": m.group(9)}
            replay.append(ln)

    def stop(self):
        for s in self.clients:
            s.close()
        assert self.d.stop() == 0


@pytest.fixture
def relay(scratch):
    r = Relay(scratch)
    yield r
    r.stop()


def _seqs(lines):
    out = []
    for ln in lines:
        m = EVENT.fullmatch(ln)
        assert m, ln
        out.append(int(m.group(1)))
    return out


def test_replay_is_exactly_what_follows_the_cursor(relay):
    relay.events(5)
    h = relay.hello()
    assert h["seq"] == 5 and h["events"] == "events=ok"
    cur = lambda seq, gen=h["gen"], rid=h["relay"]: f"{rid}:{seq}:{gen}"  # noqa: E731
    for since, want in [(0, [1, 2, 3, 4, 5]), (2, [3, 4, 5]), (4, [5]), (5, [])]:
        replay, r = relay.subscribe(cur(since))
        assert _seqs(replay) == want and r["gap"] == 0 and r["seq"] == 5, (since, replay, r)
    # every replayed line is the line a live subscriber got, byte for byte
    s, f = relay.connect()
    fp = HELLO.fullmatch(f.readline().rstrip("\n")).group(7)
    s.sendall(f"reinit fp={fp}\n".encode())
    while not f.readline().startswith("hello v1 reinit"):
        pass
    relay.events(2, prefix="live")
    live = [f.readline().rstrip("\n") for _ in range(2)]
    replay, r = relay.subscribe(cur(5))
    assert replay == live and _seqs(live) == [6, 7] and r["gap"] == 0, (live, replay)
    assert EVENT.fullmatch(live[0]).group(3) == relay.fx["gpus"][0]["bdf"]
    assert EVENT.fullmatch(live[1]).group(3) == relay.fx["gpus"][1]["bdf"]


def test_a_cursor_the_relay_cannot_vouch_for_is_a_gap(relay):
    relay.events(3)
    h = relay.hello()
    other = "f" * len(h["relay"]) if h["relay"] != "f" * len(h["relay"]) else "e" * len(h["relay"])
    cases = {
        "no cursor (a new daemon)": (None, [], 1),
        "another relay instance": (f"{other}:2:{h['gen']}", [], 1),
        "another registration generation: replayed, yet a gap": (f"{h['relay']}:1:{h['gen'] + 1}", [2, 3], 1),
        "a cursor from the future": (f"{h['relay']}:9:{h['gen']}", [], 1),
    }
    for what, (since, want, gap) in cases.items():
        replay, r = relay.subscribe(since)
        assert _seqs(replay) == want and r["gap"] == gap, (what, replay, r)


@pytest.mark.parametrize("line", [
    "reinit fp={fp} since=zz:1:1",   # relay id not hex
    "reinit fp={fp} since=abc:x:1",  # seq not a number
    "reinit fp={fp} since=abc:1",    # two fields
    "reinit fp={fp} since=",         # empty
])
def test_a_malformed_cursor_is_no_cursor(relay, line):
    relay.events(2)
    replay, r = relay.subscribe(raw=line)
    assert replay == [] and r["gap"] == 1, (line, replay, r)


def test_an_overlong_request_closes_the_connection(relay):
    s, f = relay.connect()
    f.readline()
    s.sendall(b"reinit " + b"x" * 5000)  # no newline, past the relay's 4096-byte bound
    try:
        assert f.readline() == ""  # closed, nothing more sent
    except ConnectionResetError:  # closed with the request unread
        pass
    assert relay.hello()["events"] == "events=ok"  # the relay goes on


def test_ring_overflow_fence_post(relay):
    """The ring holds the last 1024 events: a cursor whose next event is still
    held is replayed without a gap; one event further back is a gap (the
    replay is still everything held)."""
    n = RING + 6
    relay.events(n)
    h = relay.hello()
    assert h["seq"] == n
    first_held = n - RING + 1  # 7
    for since, gap in [(first_held - 1, 0), (first_held - 2, 1), (0, 1), (n - 1, 0)]:
        replay, r = relay.subscribe(f"{h['relay']}:{since}:{h['gen']}")
        want = list(range(max(since, first_held - 1) + 1, n + 1))
        assert _seqs(replay) == want and r["gap"] == gap, (since, len(replay), r)
    # its log: the first hundred event batches, then every thousandth -- every reset line
    logged = [ln for ln in relay.d.log().splitlines() if "I event-relay: event seq=" in ln]
    assert len(logged) <= 101, len(logged)
    relay.inject(["0 3 a reset"])
    assert " type=3 a reset" in relay.d.wait_log(" type=3 a reset")


def test_an_event_the_relay_lost_is_a_gap_for_every_cursor_before_it(scratch):
    """An event the relay could not number (its loop behind: here the test
    hook refuses it) is in no stream and no replay: a cursor at or before the
    loss is answered gap=1, a cursor past it gap=0."""
    r = Relay(scratch, env={"ADP_DEBUG_RELAY_REFUSE_EVENT": "refuseme"})
    try:
        r.events(3)
        r.inject(["0 1 refuseme"])
        r.d.wait_log("lost after #3")
        r.events(2)
        h = r.hello()
        assert h["seq"] == 5
        for since, want, gap in [(2, [3, 4, 5], 1), (3, [4, 5], 1), (4, [5], 0), (5, [], 0)]:
            replay, a = r.subscribe(f"{h['relay']}:{since}:{h['gen']}")
            assert _seqs(replay) == want and a["gap"] == gap, (since, replay, a)
    finally:
        r.stop()


def test_an_unplaceable_event_is_numbered_and_replayed_unplaced(relay):
    relay.events(1)
    relay.inject(["foreign 3 from nowhere"])
    relay.d.wait_log("forwarded unplaced")
    deadline = time.time() + 5
    while relay.hello()["seq"] < 2:
        assert time.time() < deadline
        time.sleep(0.02)
    h = relay.hello()
    replay, r = relay.subscribe(f"{h['relay']}:1:{h['gen']}")
    assert len(replay) == 1 and r["gap"] == 0, replay
    m = EVENT.fullmatch(replay[0])
    assert m.group(1, 2, 3, 5, 6) == ("2", "-", "-", "3", "from nowhere"), replay


class SubscribeModel:
    """relay.cc Subscribe in a few lines: what a cursor is replayed and
    whether nothing can have been missed."""

    def __init__(self, relay_id, gen):
        self.id, self.gen, self.seq, self.ring = relay_id, gen, 0, []
        self.lost, self.lost_seq = False, 0

    def event(self):
        self.seq += 1
        self.ring = (self.ring + [self.seq])[-RING:]

    def lose(self):
        self.lost, self.lost_seq = True, self.seq

    def subscribe(self, rid, seq, gen):
        if rid != self.id or seq > self.seq:
            return [], 1
        held = seq == self.seq or (bool(self.ring) and self.ring[0] <= seq + 1)
        if self.lost and seq <= self.lost_seq:
            held = False
        return [q for q in self.ring if q > seq], 0 if held and gen == self.gen else 1


@pytest.mark.parametrize("seed", [int(x) for x in os.environ.get("ADP_RELAY_SEEDS", "1,2,3,4").split(",")])
def test_random_histories_match_the_subscribe_model(scratch, seed):
    """Seeded random histories -- events, events the relay loses, renewals
    (new generations), daemons reconnecting with cursors of this relay or
    another, this generation or another, behind, current or from the future --
    answered by the real relay exactly as the model of its Subscribe says (the
    model the health model check's relay follows)."""
    import random
    rnd = random.Random(seed)
    r = Relay(scratch, env={"ADP_DEBUG_RELAY_REFUSE_EVENT": "refuseme"})
    try:
        h = r.hello()
        m = SubscribeModel(h["relay"], h["gen"])
        other = "0" * len(h["relay"]) if h["relay"] != "0" * len(h["relay"]) else "1" * len(h["relay"])
        losses = 0
        for step in range(30):
            what = rnd.random()
            if what < 0.35:
                k = rnd.randint(1, 4)
                r.events(k, prefix=f"s{step}-")
                for _ in range(k):
                    m.event()
            elif what < 0.45:
                losses += 1
                r.inject([f"{rnd.randint(0, 1)} 1 refuseme {step}"])
                r.d.wait_log("lost after", count=losses)
                m.lose()
            elif what < 0.52:
                # a daemon whose processors differ: the relay renews its
                # registration -- a new generation, and every subscriber is
                # told it may have missed events (the replay is still made)
                seq = rnd.randint(0, m.seq)
                replay, a = r.subscribe(raw=f"reinit fp=0123456789abcdef since={h['relay']}:{seq}:{m.gen}")
                want_replay, _ = m.subscribe(h["relay"], seq, m.gen)
                assert _seqs(replay) == want_replay and a["gap"] == 1 and a["gen"] == m.gen + 1, (step, a)
                m.gen += 1
            else:
                rid = h["relay"] if rnd.random() < 0.85 else other
                seq = rnd.randint(0, m.seq + 2)
                gen = m.gen if rnd.random() < 0.85 else rnd.choice([m.gen - 1, m.gen + 1])
                replay, a = r.subscribe(f"{rid}:{seq}:{gen}")
                want = m.subscribe(rid, seq, gen)
                assert (_seqs(replay), a["gap"]) == want, (step, rid == h["relay"], seq, gen, m.seq, m.lost_seq)
        assert r.hello()["seq"] == m.seq
    finally:
        r.stop()


def test_a_failed_renewal_is_events_off_until_one_succeeds(relay):
    """A daemon whose processors differ from the registration makes the relay
    renew it; when amdsmi cannot enumerate then, every daemon is told events
    are off (with why) in a new generation -- and the next daemon that
    subscribes while they are off makes the relay try again."""
    relay.events(2)
    h = relay.hello()
    open(os.path.join(relay.state, "enumerate_fail"), "w").close()
    replay, r = relay.subscribe(raw="reinit fp=0123456789abcdef since=%s:2:%d" % (h["relay"], h["gen"]))
    assert r["events"] == "events=off" and r["gen"] == h["gen"] + 1 and r["gap"] == 1, r
    assert "enumeration failed" in r["reason"], r
    assert _seqs(replay) == [], replay
    assert "enumeration failed" in relay.d.wait_log("enumeration failed")
    g = relay.hello()
    assert g["events"] == "events=off" and g["gen"] == h["gen"] + 1
    os.unlink(os.path.join(relay.state, "enumerate_fail"))
    replay, r = relay.subscribe(f"{h['relay']}:2:{g['gen']}")  # its own fingerprint: still renewed (events off)
    assert r["events"] == "events=ok" and r["gen"] == g["gen"] + 1 and r["gap"] == 1, r
    relay.events(1)
    replay, r = relay.subscribe(f"{h['relay']}:2:{r['gen']}")
    assert _seqs(replay) == [3] and r["gap"] == 0, (replay, r)


def test_a_renewal_asked_for_under_a_stuck_wait_is_skipped(scratch):
    """amdsmi cannot be re-initialised under an event wait that does not
    return: a daemon whose processors differ from the registration, arriving
    while the watchdog says events are off, gets the current state (events
    off, the same generation, why) at once instead of a registrar hung behind
    the wait -- and events come back on when the wait returns."""
    r = Relay(scratch, env={"ADP_RELAY_STUCK_MS": "300"})
    try:
        h = r.hello()
        r.inject(["hang 5000"])
        r.d.wait_log("daemons fall back to polling")
        t0 = time.monotonic()
        replay, a = r.subscribe(raw="reinit fp=0123456789abcdef since=%s:0:%d" % (h["relay"], h["gen"]))
        assert time.monotonic() - t0 < 1.5, "the answer waited for the stuck wait"
        assert a["events"] == "events=off" and a["gen"] == h["gen"] and a["gap"] == 1, a
        assert "has not returned" in a["reason"], a
        r.d.wait_log("re-enumeration a daemon asked for skipped: the event wait is stuck")  # (the registrar's)
        r.d.wait_log("the amdsmi event wait returned again", timeout=10)
        assert r.hello()["events"] == "events=ok"
    finally:
        r.stop()


def test_a_daemon_that_stops_reading_is_dropped_not_waited_for(relay):
    """A subscriber whose socket buffer fills (it stopped reading) is dropped
    -- never waited for: the relay keeps numbering and serving others, and
    what the dropped one missed is in the ring for its reconnection."""
    h = relay.hello()
    s, f = relay.connect()
    fp = HELLO.fullmatch(f.readline().rstrip("\n")).group(7)
    s.sendall(f"reinit fp={fp}\n".encode())
    while not f.readline().startswith("hello v1 reinit"):
        pass
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)  # (and now it reads nothing)
    relay.events(3000, prefix="y" * 50)  # ~330 KB of lines: far past what its socket holds
    assert relay.hello()["seq"] == 3000  # the relay went on
    # the stalled subscriber was cut: reading what was buffered ends in EOF
    s.settimeout(10)
    got = b""
    while True:
        chunk = s.recv(1 << 16)
        if not chunk:
            break
        got += chunk
    assert got.count(b"\n") < 3000, len(got)
    # reconnecting from where it got to, it is replayed what the ring holds
    last = max([int(m) for m in re.findall(rb"event seq=(\d+)", got)] or [0])
    replay, a = relay.subscribe(f"{h['relay']}:{last}:{h['gen']}")
    assert _seqs(replay) == list(range(max(last, 3000 - RING) + 1, 3001)), (last, len(replay))
    assert a["gap"] == (0 if last >= 3000 - RING else 1), (last, a)
