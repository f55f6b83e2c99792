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

`report` runs `amdgpu-device-plugin --dry-run` (real libamd_smi unless
AMD_SMI_LIB points elsewhere) and prints a table; `validate` runs
`amdgpu-dp-probe`; `bench` is the headline benchmark (see bench.py); `hbm`
runs `amdgpu-device-plugin --list-grants` (the accounting files of
--enforce-memory-units with /metrics under <device-plugin dir>/amdgpu-dp/usage)
and prints a table; `doctor` runs `amdgpu-device-plugin --doctor` (exit 1 on a
failure).
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
