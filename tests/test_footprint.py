"""The daemon's idle footprint (tools/idle_footprint.py): registered, health
monitoring on, /metrics scraped, no pods. An idle DaemonSet must not spin:
its wake-ups come from the health monitor's 100 ms event-wait slices and the
grant writer's backstop, not from polling loops."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import idle_footprint  # noqa: E402


@pytest.mark.parametrize("enforce", [False, True])
def test_idle_daemon_sleeps(enforce, capsys):
    args = ["--seconds", "4", "--scrape-s", "1", "--settle-s", "1"] + (["--enforce"] if enforce else [])
    assert idle_footprint.main(args) == 0
    import json
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert res["daemon_alive"] and res["scrapes"] >= 4
    # ~10/s from the event-wait slices (+2/s from the grant writer when enforcing)
    assert res["context_switches_per_s"] < 40, res
    assert res["cpu_pct_of_a_core"] < 5, res
    assert res["threads"] < 20 and res["rss_mib"] < 64, res


def test_idle_daemon_behind_the_relay_sleeps_between_polls(capsys):
    """The chart's layout: events come from the relay, so the monitor waits on
    sockets the wake eventfd interrupts, not in amdsmi, and sleeps until its
    next poll -- a few wake-ups a second (the relay's own waiter keeps its
    100 ms slices)."""
    args = ["--seconds", "4", "--scrape-s", "1", "--settle-s", "1", "--relay"]
    assert idle_footprint.main(args) == 0
    import json
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert res["daemon_alive"] and res["relay"]["alive"], res
    assert res["context_switches_per_s"] < 10, res  # ~3/s idle (was ~12/s with 100 ms slices)


def test_health_event_reaches_the_kubelet_fast(capsys):
    """tools/health_latency.py: a GPU_PRE_RESET on one of 8 GPUs reaches the
    kubelet as an Unhealthy device list, and GPU_POST_RESET as Healthy, within
    milliseconds (the event path: amdsmi wait -> ledger -> ListAndWatch)."""
    import json
    import health_latency
    assert health_latency.main(["--rounds", "8"]) == 0
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert res["advertised"] == 32
    for k in ("event_to_unhealthy", "event_to_healthy"):
        assert res[k]["n"] == 8 and res[k]["median_ms"] < 50 and res[k]["max_ms"] < 1000, res
