"""The daemon's side of the relay socket against a relay that misbehaves.

The relay is the daemon's own privileged sidecar, but a bug in it (or a
truncated write when it is killed) must not take the plugin down or poison
its health state. A scripted relay here -- a plain Unix socket server -- greets
the daemon, answers its reinit, then sends garbage: lines that are not
protocol, event lines with broken fields, binary bytes, a line longer than the
daemon's 64 KiB buffer, 16 MiB without a newline, a connection cut in the
middle of a line. The daemon
keeps serving, ignores what it cannot parse, acts on the valid events after
it, and reconnects after the cut. (The parser itself is fuzzed: fuzz_relay.)
"""

import os
import queue
import re
import socket
import threading
import time

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

from test_metrics import _get, _parse, _value


class ScriptedRelay:
    """Accepts daemon connections; each is greeted, its reinit answered, then
    handed to `script(conn)`."""

    def __init__(self, path, script):
        self.path, self.script = path, script
        self.srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.srv.bind(path)
        self.srv.listen(4)
        self.connections = 0
        self.requests = []
        self.errors = []
        threading.Thread(target=self._serve, daemon=True).start()

    def _serve(self):
        while True:
            try:
                c, _ = self.srv.accept()
            except OSError:
                return
            self.connections += 1
            hello = "hello v1 events=ok processors=2 relay=abc123 gen=1 seq=0 fp=- renew_ms=0\n"
            try:
                c.sendall(hello.encode())
                f = c.makefile("r")
                self.requests.append(f.readline().strip())
                c.sendall(b"hello v1 reinit events=ok processors=2 relay=abc123 gen=1 seq=0 fp=- renew_ms=0 gap=0\n")
                self.script(c, self.connections)
            except OSError as e:
                self.errors.append(repr(e))

    def close(self):
        self.srv.close()


def test_a_misbehaving_relay_does_not_take_the_daemon_down(scratch, tmp_path):
    sock = str(tmp_path / "events.sock")
    bdf0 = fixtures.node(2)["gpus"][0]["bdf"]
    done = threading.Event()

    def script(c, n):
        if n == 1:
            for junk in (b"not the protocol\n", b"event seq=x node=2 bdf=" + bdf0.encode() + b" part=0 type=3 bad\n",
                         b"event seq=1 node=2 bdf=" + bdf0.encode() + b" part=zz type=3\n",
                         b"event seq=2 node=99999999999 bdf=- part=0 type=3\n",
                         b"\x00\xff\xfe binary \x01\n", b"hello\n", b"x" * 70000 + b"\n"):
                c.sendall(junk)
            for _ in range(16):  # 16 MiB without a newline: the daemon's buffer stays bounded
                c.sendall(b"y" * (1 << 20))
            c.sendall(b"\n")
            # then a valid reset of GPU 0, and the connection cut mid-line
            c.sendall(f"event seq=3 node=2 bdf={bdf0} part=0 type=3 a real reset\n".encode())
            time.sleep(0.5)
            c.sendall(b"event seq=4 node=2 bdf=")
            c.shutdown(socket.SHUT_RDWR)  # (the reader's file object still holds the descriptor)
            c.close()
        else:
            # the daemon came back: the reset completes
            c.sendall(f"event seq=4 node=2 bdf={bdf0} part=0 type=4 reset done\n".encode())
            done.wait(30)
            c.shutdown(socket.SHUT_RDWR)
            c.close()

    relay = ScriptedRelay(sock, script)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=["--health-event-socket", sock, "--metrics-addr",
                                                        "127.0.0.1:0"],
                       env={"DP_HEALTH_POLL_MS": "100"}).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        q, call = c.watch()
        seen = []
        deadline = time.time() + 15
        while not (["Unhealthy", "Healthy"] in seen and seen[-1] == ["Healthy", "Healthy"]):
            assert time.time() < deadline, (seen, relay.connections, relay.errors, d.log()[-3000:])
            try:
                seen.append([x.health for x in q.get(timeout=0.2).devices])
            except queue.Empty:
                pass
        # Healthy -> GPU 0 held by the valid PRE (the garbage before it ignored) -> back on the POST
        assert ["Unhealthy", "Healthy"] in seen, seen
        call.cancel()
        c.close()
        log = d.log()
        assert "event relay: malformed line ignored" in log
        assert relay.connections >= 2 and all(r.startswith("reinit ") for r in relay.requests), relay.requests
        m = _parse(_get(port, "/metrics")[1])
        assert _value(m, "amdgpu_dp_gpu_events_total", bdf=bdf0, type="GPU_PRE_RESET") == 1
        assert _value(m, "amdgpu_dp_gpu_events_total", bdf=bdf0, type="GPU_POST_RESET") == 1
        assert d.proc.poll() is None
    finally:
        done.set()
        assert d.stop() == 0
        k.stop()
        relay.close()
