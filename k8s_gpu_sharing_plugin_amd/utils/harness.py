"""Run the real daemon binary against a scratch kubelet directory.

The daemon under test is always the native ``amdgpu-device-plugin`` process;
the device library is either the real libamd_smi (GPU box) or libamdsmi_mock
with a node fixture (CPU).
"""

import os
import signal
import subprocess
import tempfile
import time

from .. import DAEMON, KUBELET_STUB, MOCK_LIB
from ..models import fixtures


class Daemon:
    def __init__(self, plugin_dir: str, fixture: dict = None, args=(), env=None, real_smi=False,
                 event_fifo: str = None, state_dir: str = None, nofile: int = None, launch=None,
                 log_path: str = None):
        self.plugin_dir = plugin_dir
        self.args = list(args)
        self.env = dict(os.environ)
        self.env.setdefault("ADP_LOG_LEVEL", "info")
        if not real_smi:
            fx = dict(fixture or fixtures.node(2))
            if event_fifo:
                fx["event_fifo"] = event_fifo
            if state_dir:
                fx["state_dir"] = state_dir
            self.fixture_path = fixtures.write(fx, plugin_dir + ".fixture")
            self.env["AMD_SMI_LIB"] = MOCK_LIB
            self.env["AMDSMI_MOCK_FIXTURE"] = self.fixture_path
        else:
            self.env.pop("AMD_SMI_LIB", None)
        self.env.update(env or {})
        self.log_path = log_path or plugin_dir + ".daemon.log"
        self.proc = None
        self.nofile = nofile  # RLIMIT_NOFILE for the daemon (descriptor exhaustion tests)
        # argv -> argv: how the daemon binary is started (e.g. inside an
        # assembled container image, utils/image.py); the result must exec the
        # daemon in place so signals reach it.
        self.launch = launch

    def start(self):
        self._log = open(self.log_path, "w")
        argv = [DAEMON, "--device-plugin-path", self.plugin_dir, *self.args]
        if self.launch:
            argv = self.launch(argv)
        if self.nofile:
            # The limit is set by a shell that then execs the daemon (same pid).
            # A preexec_fn would run Python between fork and exec, which can
            # deadlock on a lock another thread (the stub kubelet's gRPC
            # threads, the import lock) held at fork time.
            argv = ["/bin/sh", "-c", 'ulimit -n %d && exec "$0" "$@"' % int(self.nofile), *argv]
        self.proc = subprocess.Popen(argv, env=self.env, stdout=self._log, stderr=subprocess.STDOUT)
        return self

    def log(self) -> str:
        with open(self.log_path) as f:
            return f.read()

    def wait_log(self, needle: str, timeout: float = 10.0, count: int = 1) -> str:
        deadline = time.time() + timeout
        while time.time() < deadline:
            text = self.log()
            if text.count(needle) >= count:
                return text
            if self.proc.poll() is not None:
                break
            time.sleep(0.02)
        raise TimeoutError(f"'{needle}' x{count} not seen in daemon log:\n{self.log()[-4000:]}")

    def signal(self, sig=signal.SIGHUP):
        self.proc.send_signal(sig)

    def stop(self, timeout: float = 10.0) -> int:
        if self.proc is None:
            return 0
        if self.proc.poll() is None:
            self.proc.send_signal(signal.SIGTERM)
            try:
                self.proc.wait(timeout)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        self._log.close()
        return self.proc.returncode


class NativeKubelet:
    """The native stub kubelet (`amdgpu-dp-kubelet serve`), JSON events on stdout."""

    def __init__(self, socket_path: str):
        self.socket_path = socket_path
        self.proc = None
        self.events = []

    def start(self):
        self.proc = subprocess.Popen([KUBELET_STUB, "serve", "--kubelet-socket", self.socket_path],
                                     stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        self.wait(lambda e: e.get("event") == "listening", 10)
        return self

    def wait(self, pred, timeout=10.0, since=0):
        """Returns the first event (old or new, from index `since` on) matching `pred`.

        Reads the pipe with os.read on the raw fd: a buffered readline() after
        select() can strand a second line in Python's buffer where select() no
        longer sees it.
        """
        import json
        import select
        deadline = time.time() + timeout
        for e in self.events[since:]:
            if pred(e):
                return e
        fd = self.proc.stdout.fileno()
        if not hasattr(self, "_pending"):
            self._pending = b""
        while time.time() < deadline:
            r, _, _ = select.select([fd], [], [], 0.1)
            if not r:
                continue
            chunk = os.read(fd, 65536)
            if not chunk:
                break
            self._pending += chunk
            *lines, self._pending = self._pending.split(b"\n")
            hit = None
            for line in lines:
                try:
                    e = json.loads(line)
                except ValueError:
                    continue
                self.events.append(e)
                if hit is None and pred(e):
                    hit = e
            if hit is not None:
                return hit
        raise TimeoutError(f"event not seen; got {self.events[-5:]}")

    def stop(self):
        if self.proc and self.proc.poll() is None:
            self.proc.send_signal(signal.SIGTERM)
            try:
                self.proc.wait(10)
            except subprocess.TimeoutExpired:
                self.proc.kill()


def scratch_dir(prefix="adp") -> str:
    # Unix socket paths are limited to 107 bytes: keep scratch dirs short.
    return tempfile.mkdtemp(prefix=prefix + "-", dir="/tmp")
