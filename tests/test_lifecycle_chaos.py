"""Seeded random lifecycles: everything that restarts or re-registers the
plugins, interleaved, against one running daemon.

Each step is one of: SIGHUP, or three at once; the kubelet restarting (its
socket re-created), or going away for a few steps; the plugin's own socket
deleted; a config-file edit (resource renamed and/or replica count changed,
applied live), or a broken one (ignored: the running config stays, across a
SIGHUP too); GPU 1 drained or undrained by the operator's drain file; SIGUSR1;
a GPU reset (every partition's GPU_PRE_RESET, then every GPU_POST_RESET);
in the chart's layout also the event relay stopped or killed and started
again (events must be back on through it at every settle).
After every step (the kubelet's absence aside) the daemon must come back
to the expected state on its own: registered with the current kubelet for the
expected resource, and that resource's ListAndWatch listing 2 GPUs x R
replicas with exactly GPU 1's replicas Unhealthy while it is drained. At the
end its descriptors and threads are where they started and SIGTERM exits 0
with its sockets removed. The single triggers are pinned one by one in
test_lifecycle.py; this is their interleavings (the reference restarts on
kubelet.sock re-creation and SIGHUP only: main.go:283-326).
"""

import os
import queue
import random
import signal
import time

import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

SEEDS = [int(s) for s in os.environ.get("ADP_LIFECYCLE_SEEDS", "1,2,3").split(",")]
RELAY_SEEDS = [int(s) for s in os.environ.get("ADP_LIFECYCLE_RELAY_SEEDS", "1,2").split(",")]
CPX_SEEDS = [int(s) for s in os.environ.get("ADP_LIFECYCLE_CPX_SEEDS", "1").split(",")]
STEPS = int(os.environ.get("ADP_LIFECYCLE_STEPS", "12"))


def _count(pid, what):
    if what == "fds":
        return len(os.listdir(f"/proc/{pid}/fd"))
    return len(os.listdir(f"/proc/{pid}/task"))


class Life:
    def __init__(self, scratch, tmp_path, relay=False, cpx=False):
        self.scratch = scratch
        self.ksock = os.path.join(scratch, "kubelet.sock")
        # cpx: both GPUs in CPX, every partition a device (--partition-strategy single)
        self.fx = fixtures.node(2, modes="CPX") if cpx else fixtures.node(2)
        self.per_gpu = 8 if cpx else 1
        self.cfg = str(tmp_path / "config.yaml")
        self.drain = str(tmp_path / "drain")
        self.replicas, self.name, self.drained = 2, "sharedgpu", False
        self.write_config()
        self.k = kubelet.StubKubelet(self.ksock).start()
        # GPU resets (every partition's GPU_PRE_RESET, then every GPU_POST_RESET)
        # come through the mock's event FIFO; a POST lost to a restart is a gap
        # the polled check closes within the short hold. Flap damping off: the
        # random resets are not a flapping GPU.
        self.fifo = str(tmp_path / "events")
        os.mkfifo(self.fifo)
        args = ["--config-file", self.cfg, "--drain-file", self.drain, "--reset-flap-limit", "0",
                "--reset-recovery-hold-ms", "500"]
        if cpx:
            args += ["--partition-strategy", "single"]
        env = {"DP_HEALTH_POLL_MS": "100"}
        self.relay, self.relays = None, 0
        if relay:
            # the chart's layout: events through the relay, the daemon denied
            # /dev/kfd and the render nodes like an unprivileged pod
            from k8s_gpu_sharing_plugin_amd import BUILD_DIR
            self.fx = dict(self.fx, events_open_kfd=True)
            self.rsock = str(tmp_path / "events.sock")
            self.start_relay()
            sim = os.path.join(BUILD_DIR, "libadp_devcgroup_sim.so")
            args += ["--health-event-socket", self.rsock, "--metrics-addr", "127.0.0.1:0"]
            env["LD_PRELOAD"] = " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), sim) if x)
        self.d = harness.Daemon(scratch, self.fx, args=args, env=env,
                                event_fifo=None if relay else self.fifo).start()
        self.reg = None
        self.history = []
        self.kubelet_down = False

    def start_relay(self):
        self.relays += 1
        rdir = f"{self.scratch}-relay{self.relays}"
        os.makedirs(rdir, exist_ok=True)
        self.relay = harness.Daemon(rdir, self.fx, args=["--event-relay", "--health-event-socket", self.rsock],
                                    event_fifo=self.fifo).start()
        self.relay.wait_log("relaying amdsmi events on")

    def events_on(self):
        import re
        from test_metrics import _get, _parse, _value
        port = int(re.search(r"on port (\d+)", self.d.wait_log("serving /metrics")).group(1))
        try:
            return _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_health_events_enabled") == 1
        except OSError:  # /metrics restarting with a generation
            return False

    def write_config(self):
        tmp = self.cfg + ".tmp"
        with open(tmp, "w") as f:
            f.write(f"version: v1\nflags:\n  resourceConfig: gpu:{self.name}:{self.replicas}\n")
        os.rename(tmp, self.cfg)

    def step(self, rnd):
        what = rnd.choice(["sighup", "storm", "kubelet", "kubelet-away", "socket", "config", "config", "broken",
                           "drain", "usr1", "reset", "reset"] + (["relay-restart", "relay-kill"] if self.relay else []))
        if self.kubelet_down and what in ("kubelet", "kubelet-away"):
            what = "kubelet-back"
        if what == "sighup":
            self.d.signal(signal.SIGHUP)
        elif what == "storm":
            for _ in range(3):
                self.d.signal(signal.SIGHUP)
        elif what == "kubelet-away":
            self.k.stop()
            if os.path.exists(self.ksock):
                os.unlink(self.ksock)
            self.kubelet_down = True
            self.reg = None
        elif what == "kubelet-back":
            self.k = kubelet.StubKubelet(self.ksock).start()
            self.kubelet_down = False
            self.reg = None
        elif what == "usr1":
            self.d.signal(signal.SIGUSR1)
        elif what == "reset":
            g = rnd.randint(0, 1)
            parts = range(self.per_gpu)
            lines = [f"{g}:{p} 3 chaos pre" for p in parts] + [f"{g}:{p} 4 chaos post" for p in parts]
            try:
                fd = os.open(self.fifo, os.O_WRONLY | os.O_NONBLOCK)
                os.write(fd, "".join(ln + "\n" for ln in lines).encode())
                os.close(fd)
                what += f" gpu {g}"
            except OSError:  # no reader right now (a restart): nothing reset
                what += " (no reader)"
        elif what in ("relay-restart", "relay-kill"):
            if what == "relay-kill":
                self.relay.proc.kill()
                self.relay.proc.wait()
            self.relay.stop()
            self.start_relay()
        elif what == "broken":
            # A valid edit replaced at once by a broken one may never be read
            # (then the daemon rightly keeps what it ran): the valid one is
            # let settle first.
            if self.history and self.history[-1].startswith("config"):
                self.settle()
            with open(self.cfg + ".tmp", "w") as f:
                f.write("version: v2\n")
            os.rename(self.cfg + ".tmp", self.cfg)
        elif what == "kubelet":
            self.k.stop()
            if os.path.exists(self.ksock):
                os.unlink(self.ksock)
            self.k = kubelet.StubKubelet(self.ksock).start()
            self.reg = None  # the new kubelet knows no plugin yet
        elif what == "socket":
            if self.reg is not None:
                try:
                    os.unlink(os.path.join(self.scratch, self.reg.endpoint))
                except FileNotFoundError:
                    pass
        elif what == "config":
            self.replicas = rnd.choice([1, 2, 3])
            self.name = rnd.choice(["sharedgpu", "timeshared"])
            self.write_config()
            what += f" gpu:{self.name}:{self.replicas}"
        elif what == "drain":
            self.drained = not self.drained
            with open(self.drain + ".tmp", "w") as f:
                f.write(f"{self.fx['gpus'][1]['bdf']}\n" if self.drained else "# none\n")
            os.rename(self.drain + ".tmp", self.drain)
            what += " on" if self.drained else " off"
        self.history.append(what)

    def step_kubelet_back(self):
        self.k = kubelet.StubKubelet(self.ksock).start()
        self.kubelet_down = False
        self.reg = None
        self.history.append("kubelet-back")

    def settle(self, timeout=20.0):
        """Until the kubelet's latest registration is the expected resource and
        its ListAndWatch shows the expected devices and health."""
        if self.kubelet_down:  # nothing to register with: alive, that is all
            time.sleep(0.3)
            assert self.d.proc.poll() is None, (self.history, self.d.log()[-4000:])
            return
        want_name = f"amd.com/{self.name}"
        want = (2 * self.per_gpu * self.replicas, self.per_gpu * self.replicas if self.drained else 0)
        deadline = time.monotonic() + timeout
        seen = None
        while True:
            assert self.d.proc.poll() is None, (self.history, self.d.log()[-4000:])
            try:
                while True:
                    self.reg = self.k.registrations.get_nowait()
            except queue.Empty:
                pass
            if self.reg is not None and self.reg.resource_name == want_name:
                c = kubelet.PluginClient(os.path.join(self.scratch, self.reg.endpoint))
                try:
                    q, call = c.watch()
                    first = q.get(timeout=2)
                    call.cancel()
                    if hasattr(first, "devices"):
                        # ... and no other resource's socket left behind (a renamed one is gone)
                        socks = sorted(e for e in os.listdir(self.scratch)
                                       if e.endswith(".sock") and e != "kubelet.sock")
                        seen = (len(first.devices), sum(x.health != "Healthy" for x in first.devices), socks)
                        if seen == want + ([self.reg.endpoint],):
                            if self.relay is None or self.events_on():
                                return
                            seen = "events not on through the relay"
                    else:  # the endpoint is being restarted: the call failed
                        seen = repr(first)[:200]
                except queue.Empty:
                    seen = "no ListAndWatch answer"
                finally:
                    c.close()
            else:
                seen = self.reg.resource_name if self.reg is not None else "no registration"
            assert time.monotonic() < deadline, (self.history, want_name, want, seen, self.d.log()[-4000:])
            time.sleep(0.1)

    def close(self):
        rc = self.d.stop()
        if not self.kubelet_down:
            self.k.stop()
        if self.relay is not None:
            self.relay.stop()
        return rc


@pytest.mark.parametrize("seed,relay,cpx", [(s, False, False) for s in SEEDS] + [(s, True, False) for s in RELAY_SEEDS]
                         + [(s, True, True) for s in CPX_SEEDS])
def test_interleaved_restarts_reloads_and_drains_settle(scratch, tmp_path, seed, relay, cpx):
    """(relay: the chart's layout, with the relay also stopped or killed and
    started again, and events required back on through it at every settle;
    cpx: a node of CPX GPUs, every partition a device)"""
    rnd = random.Random(seed)
    life = Life(scratch, tmp_path, relay=relay, cpx=cpx)
    try:
        life.settle()
        life.d.wait_log("health monitor watching")  # (its thread starts after the registration)
        pid = life.d.proc.pid
        fds0, threads0 = _count(pid, "fds"), _count(pid, "threads")
        for _ in range(STEPS):
            life.step(rnd)
            if rnd.random() < 0.3:  # sometimes a second trigger before the first settled
                life.step(rnd)
            life.settle()
        if life.kubelet_down:
            life.step_kubelet_back()
            life.settle()
        fds, threads = _count(pid, "fds"), _count(pid, "threads")
        # (a restart may be mid-way: a few descriptors of slack, none per step)
        assert fds <= fds0 + 6 and threads <= threads0 + 2, (fds0, fds, threads0, threads, life.history)
        endpoints = [e for e in os.listdir(scratch) if e.endswith(".sock") and e != "kubelet.sock"]
    finally:
        rc = life.close()
    assert rc == 0, life.d.log()[-3000:]
    assert all(not os.path.exists(os.path.join(scratch, e)) for e in endpoints), endpoints
