"""Command-line front end for the tooling around the native daemon.

  python -m k8s_gpu_sharing_plugin_amd build              # native tree + gfx950 probe
  python -m k8s_gpu_sharing_plugin_amd report [daemon flags...]
                                                          # what this node would advertise
  python -m k8s_gpu_sharing_plugin_amd validate [--mfma] [--p2p]
                                                          # probe every visible GPU
  python -m k8s_gpu_sharing_plugin_amd bench [bench.py flags...]
  python -m k8s_gpu_sharing_plugin_amd hbm [daemon flags...]  # HBM use of enforced grants
  python -m k8s_gpu_sharing_plugin_amd doctor [daemon flags...]
                                                          # deployment checks, what to change
  python -m k8s_gpu_sharing_plugin_amd status [URL]       # a running daemon, from its /metrics

`report` runs `amdgpu-device-plugin --dry-run` (real libamd_smi unless
AMD_SMI_LIB points elsewhere) and prints a table; `validate` runs
`amdgpu-dp-probe`; `bench` is the headline benchmark (see bench.py); `hbm`
runs `amdgpu-device-plugin --list-grants` (the accounting files of
--enforce-memory-units with /metrics under <device-plugin dir>/amdgpu-dp/usage)
and prints a table; `doctor` runs `amdgpu-device-plugin --doctor` (exit 1 on a
failure); `status` reads a running daemon's /metrics (default
http://127.0.0.1:9400/metrics) and prints its resources, device health (why a
GPU is out of service, whether it awaits the polled recovery after an event
gap), what one memory unit is, RPC counts with the loops' residency, and the
containers' HBM against their grants; exit 1 on an Unhealthy device, a
container over its grant, or IDs running pods hold that are no longer
advertised.
"""

import json
import subprocess
import sys

from . import DAEMON


def _report(args) -> int:
    r = subprocess.run([DAEMON, "--dry-run", *args], capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stderr)
        return r.returncode
    rep = json.loads(r.stdout)
    print(f"amdsmi {rep['amdsmi']}")
    print(f"{'gpu':>3}  {'bdf':<13} {'mode':<10} {'parts':>5} {'HBM MiB':>9} {'numa':>4}  uuid")
    for g in rep["gpus"]:
        print(f"{g['index']:>3}  {g['bdf']:<13} {g['mode']:<10} {g['partitions']:>5} {g['vram_mib']:>9} "
              f"{g['numa']:>4}  {g['uuid']}")
    print()
    print(f"{'resource':<28} {'devices':>7} {'allocatable':>11}  socket")
    for res in rep["resources"]:
        print(f"{res['resource']:<28} {res['devices']:>7} {res['allocatable']:>11}  {res['socket']}")
    print()
    for k, v in rep.get("labels", {}).items():
        print(f"{k}={v}")
    return 0


def _validate(args) -> int:
    from .utils.build import PROBE_EXE, build_probe
    build_probe()
    return subprocess.run([PROBE_EXE, *args]).returncode


def _hbm(args) -> int:
    r = subprocess.run([DAEMON, "--list-grants", *args], capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stderr)
        return r.returncode
    rep = json.loads(r.stdout)
    mib = 1 << 20
    print(f"{'grant':<16} {'dev':>3} {'used MiB':>9} {'granted MiB':>11} {'peak MiB':>9} {'refused':>7}  ids")
    for g in rep["grants"]:
        for i in range(len(g["used"])):
            print(f"{g['key']:<16} {i:>3} {g['used'][i] // mib:>9} {g['granted'][i] // mib:>11} "
                  f"{g['peak'][i] // mib:>9} {g['refused'][i]:>7}  {g['ids'] if i == 0 else ''}")
    return 0


def parse_prometheus(text):
    """[(name, {label: value}, float)] of a Prometheus text exposition."""
    import re
    out = []
    for line in text.splitlines():
        if not line or line.startswith("#"):
            continue
        m = re.match(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(?:\{(.*)\})? (\S+)$', line)
        if not m:
            continue
        labels = {k: bytes(v, "utf-8").decode("unicode_escape")
                  for k, v in re.findall(r'(\w+)="((?:[^"\\]|\\.)*)"', m.group(2) or "")}
        out.append((m.group(1), labels, float(m.group(3))))
    return out


def _quantile(buckets, q):
    """Upper bound of the bucket holding quantile q of cumulative (le, count) pairs."""
    buckets = sorted(buckets)
    total = buckets[-1][1] if buckets else 0
    if not total:
        return None
    for le, c in buckets:
        if c >= q * total:
            return le
    return buckets[-1][0]


def _status(args) -> int:
    import urllib.request
    url = args[0] if args else "http://127.0.0.1:9400/metrics"
    try:
        with urllib.request.urlopen(url, timeout=5) as r:
            samples = parse_prometheus(r.read().decode())
    except OSError as e:
        print(f"cannot read {url}: {e}", file=sys.stderr)
        return 1

    def by(name):
        return [(ls, v) for n, ls, v in samples if n == name]

    # /stats on the same port has the residency at 100 ns resolution
    fine = {}
    try:
        with urllib.request.urlopen(url.rsplit("/", 1)[0] + "/stats", timeout=5) as r:
            for p in json.loads(r.read()).get("plugins", []):
                fine[p["resource"]] = sorted((int(b), int(n)) for b, n in p.get("residency_100ns", []))
    except (OSError, ValueError):
        pass

    def fine_q(bins, q):
        total = sum(n for _, n in bins)
        seen = 0
        for b, n in bins:
            seen += n
            if seen >= q * total:
                return (b + 1) / 10
        return None

    build = by("amdgpu_dp_build_info")
    if build:
        print("amdgpu-device-plugin " + " ".join(f"{k}={v}" for k, v in sorted(build[0][0].items())))
    print(f"{'resource':<28} {'devices':>7} {'healthy':>7} {'allocatable':>11} {'registered':>10} "
          f"{'Allocate':>9} {'Preferred':>9} {'residency p50/p99 us':>21}")
    for ls, n in by("amdgpu_dp_devices"):
        res = ls.get("resource")

        def one(name, extra=None):
            return next((v for l2, v in by(name) if l2.get("resource") == res and
                         all(l2.get(k) == x for k, x in (extra or {}).items())), 0)
        buckets = [(float("inf") if l2["le"] == "+Inf" else float(l2["le"]), v)
                   for l2, v in by("amdgpu_dp_rpc_residency_seconds_bucket") if l2.get("resource") == res]
        p50, p99 = _quantile(buckets, 0.5), _quantile(buckets, 0.99)
        resid = "-" if p50 is None else f"<={p50 * 1e6:g} / <={p99 * 1e6:g}"
        if fine.get(res):
            resid = f"{fine_q(fine[res], 0.5):.1f} / {fine_q(fine[res], 0.99):.1f}"
        print(f"{res:<28} {int(n):>7} {int(one('amdgpu_dp_healthy_devices')):>7} "
              f"{int(one('amdgpu_dp_allocatable')):>11} {'yes' if one('amdgpu_dp_registered') else 'no':>10} "
              f"{int(one('amdgpu_dp_rpc_total', {'method': 'Allocate'})):>9} "
              f"{int(one('amdgpu_dp_rpc_total', {'method': 'GetPreferredAllocation'})):>9} {resid:>21}")
    def scalar(name):
        got = by(name)
        return got[0][1] if got else None
    ev = scalar("amdgpu_dp_health_events_enabled")
    age = scalar("amdgpu_dp_health_loop_age_seconds")
    line = "health: events " + {1: "on", 0: "off (polling)", -1: "not started", None: "?"}.get(
        None if ev is None else int(ev), "?")
    if age is not None:
        line += f", monitor loop {age:.1f} s ago"
    polls = scalar("amdgpu_dp_driver_hbm_polls_total")
    if polls is not None:
        failures = scalar("amdgpu_dp_driver_hbm_scan_failures_total") or 0
        secs = scalar("amdgpu_dp_driver_hbm_scan_seconds") or 0
        line += f"; driver-side scans {int(polls)} (last {secs * 1e3:.2f} ms, {int(failures)} failed)"
    relay = scalar("amdgpu_dp_event_relay_connected")
    if relay is not None:
        lost = int(scalar("amdgpu_dp_event_relay_disconnects_total") or 0)
        line += "; event relay " + ("connected" if relay == 1 else "NOT connected") + (
            f" ({lost} connection(s) lost)" if lost else "")
    gaps = scalar("amdgpu_dp_health_event_gaps_total")
    if gaps:
        line += f"; {int(gaps)} event gap(s)"
    recovered = sum(v for _, v in by("amdgpu_dp_gpu_recovered_without_event_total"))
    if recovered:
        line += f", {int(recovered)} GPU(s) recovered without GPU_POST_RESET"
    print(line)
    # memory-unit resources: what one unit is (a pod asking for N gets N x this)
    units = {}
    for ls, v in by("amdgpu_dp_memory_unit_mib"):
        units.setdefault(ls.get("resource"), set()).add((int(v), ls.get("kind")))
    for res, us in sorted(units.items()):
        sizes = sorted(us)
        size = (f"{sizes[0][0]} MiB" if len(sizes) == 1 else
                f"{sizes[0][0]}..{sizes[-1][0]} MiB")
        print(f"{res}: one unit = {size} ({', '.join(sorted({k for _, k in sizes}))})")
    unmatched = sorted((ls.get("type"), int(v)) for ls, v in by("amdgpu_dp_unmatched_events_total") if v)
    if unmatched:
        print("UNMATCHED events (amdsmi named a processor no GPU of this node is): " +
              ", ".join(f"{t} x{n}" for t, n in unmatched))
    for ls, v in by("amdgpu_dp_deferred_layout_change"):
        if v:
            print(f"DEFERRED {ls.get('resource')}: a config change waits for the running pods holding its IDs")
    stale = [(ls.get("resource"), v) for ls, v in by("amdgpu_dp_stale_allocated_ids") if v]
    for res, v in stale:
        print(f"STALE {res}: {int(v)} ID(s) running pods hold are no longer advertised (the layout changed "
              "under them: drain the node)")
    awaiting = {ls.get("bdf") for ls, v in by("amdgpu_dp_gpu_awaiting_polled_recovery") if v}
    causes = {}
    for ls, v in by("amdgpu_dp_gpu_failure"):
        if v:
            causes.setdefault(ls.get("bdf"), []).append(ls.get("cause"))
    for bdf, cs in sorted(causes.items()):
        print(f"GPU {bdf}: " + ", ".join(sorted(cs)) +
              (" (awaiting polled recovery after an event gap)" if bdf in awaiting else ""))
    bad = [ls for ls, v in by("amdgpu_dp_device_healthy") if v == 0]
    for ls in bad:
        print(f"UNHEALTHY {ls.get('resource')} {ls.get('device')} (index {ls.get('index')})")
    used = {tuple(sorted(ls.items())): v for ls, v in by("amdgpu_dp_container_hbm_used_bytes")}
    granted = {tuple(sorted(ls.items())): v for ls, v in by("amdgpu_dp_container_hbm_granted_bytes")}
    if granted:
        print()
        print(f"{'namespace/pod/container':<48} {'device':>6} {'used MiB':>9} {'granted MiB':>11}")
        for key, g in sorted(granted.items()):
            ls = dict(key)
            who = "/".join(ls.get(k, "?") for k in ("namespace", "pod", "container"))
            print(f"{who:<48} {ls.get('index', ls.get('device', '?')):>6} {int(used.get(key, 0)) >> 20:>9} "
                  f"{int(g) >> 20:>11}")
    over = [ls for ls, v in by("amdgpu_dp_container_hbm_over_grant") if v]
    for ls in over:
        print(f"OVER GRANT {ls.get('namespace')}/{ls.get('pod')}/{ls.get('container')} on {ls.get('bdf')}")
    return 1 if bad or over or stale else 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    cmd, rest = argv[0], argv[1:]
    if cmd == "build":
        from .utils import build
        build.build_all(probe="--no-probe" not in rest)
        return 0
    if cmd == "report":
        return _report(rest)
    if cmd == "validate":
        return _validate(rest)
    if cmd == "hbm":
        return _hbm(rest)
    if cmd == "status":
        return _status(rest)
    if cmd == "doctor":
        return subprocess.run([DAEMON, "--doctor", *rest]).returncode
    if cmd == "bench":
        from .parallel import bench
        bench.main(rest)
        return 0
    print(f"unknown command {cmd!r}\n{__doc__}", file=sys.stderr)
    return 2


if __name__ == "__main__":
    sys.exit(main())
