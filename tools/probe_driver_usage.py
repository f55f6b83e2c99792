#!/usr/bin/env python3
"""What the driver tells an unprivileged process about per-process HBM use
(for the daemon's driver-side grant check): the KFD sysfs process tree, the
KFD topology's gpu_id <-> PCI address map, and amdsmi_get_gpu_process_list,
before and while this process (PyTorch) holds 1 GiB on GPU 0. JSON on stdout.
Run on the GPU box: python tools/probe_driver_usage.py > gpurun_out/x.json
"""
import ctypes
import glob
import json
import os
import sys
import time


def kfd_procs():
    out = {}
    for d in sorted(glob.glob("/sys/class/kfd/kfd/proc/*")):
        ent = {}
        for f in sorted(os.listdir(d)) if os.path.isdir(d) else []:
            p = os.path.join(d, f)
            if os.path.isfile(p):
                try:
                    ent[f] = open(p).read().strip()[:200]
                except OSError as e:
                    ent[f] = f"<{e.strerror}>"
            else:
                ent[f] = "<dir>"
        out[os.path.basename(d)] = ent
    return out


def kfd_nodes():
    out = []
    for d in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*")):
        props = {}
        try:
            for ln in open(os.path.join(d, "properties")):
                k, _, v = ln.strip().partition(" ")
                if k in ("gpu_id", "location_id", "domain", "simd_count", "drm_render_minor", "unique_id"):
                    props[k] = v
            props["gpu_id_file"] = open(os.path.join(d, "gpu_id")).read().strip()
        except OSError as e:
            props["error"] = e.strerror
        out.append({"node": os.path.basename(d), **props})
    return out


class ProcInfo(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 256), ("pid", ctypes.c_uint32), ("mem", ctypes.c_uint64),
                ("gfx", ctypes.c_uint64), ("enc", ctypes.c_uint64), ("eres", ctypes.c_uint32 * 12),
                ("gtt_mem", ctypes.c_uint64), ("cpu_mem", ctypes.c_uint64), ("vram_mem", ctypes.c_uint64),
                ("mres", ctypes.c_uint32 * 10), ("container_name", ctypes.c_char * 256),
                ("cu_occupancy", ctypes.c_uint32), ("evicted_time", ctypes.c_uint32), ("res", ctypes.c_uint32 * 10)]


def smi_process_list():
    try:
        lib = ctypes.CDLL("libamd_smi.so")
    except OSError:
        lib = ctypes.CDLL("/opt/rocm/lib/libamd_smi.so")
    rc = lib.amdsmi_init(ctypes.c_uint64(2))  # AMDSMI_INIT_AMD_GPUS
    if rc:
        return {"init": rc}
    n = ctypes.c_uint32(0)
    lib.amdsmi_get_socket_handles(ctypes.byref(n), None)
    socks = (ctypes.c_void_p * n.value)()
    lib.amdsmi_get_socket_handles(ctypes.byref(n), socks)
    res = []
    for s in socks:
        m = ctypes.c_uint32(0)
        lib.amdsmi_get_processor_handles(ctypes.c_void_p(s), ctypes.byref(m), None)
        hs = (ctypes.c_void_p * m.value)()
        lib.amdsmi_get_processor_handles(ctypes.c_void_p(s), ctypes.byref(m), hs)
        for h in hs:
            cnt = ctypes.c_uint32(64)
            buf = (ProcInfo * 64)()
            rc = lib.amdsmi_get_gpu_process_list(ctypes.c_void_p(h), ctypes.byref(cnt), buf)
            res.append({"rc": rc, "count": cnt.value,
                        "procs": [{"pid": buf[i].pid, "name": buf[i].name.decode(errors="replace"),
                                   "mem": buf[i].mem, "vram": buf[i].vram_mem,
                                   "container": buf[i].container_name.decode(errors="replace")}
                                  for i in range(min(cnt.value, 64))]})
    lib.amdsmi_shut_down()
    return res


def fdinfo(pid="self"):
    """DRM fdinfo of every render-node / kfd fd of `pid` (per-client VRAM)."""
    out = []
    base = f"/proc/{pid}/fd"
    try:
        fds = os.listdir(base)
    except OSError as e:
        return {"error": e.strerror}
    for fd in fds:
        try:
            target = os.readlink(os.path.join(base, fd))
        except OSError:
            continue
        if not (target.startswith("/dev/dri/") or target == "/dev/kfd"):
            continue
        try:
            info = open(f"/proc/{pid}/fdinfo/{fd}").read()
        except OSError as e:
            info = f"<{e.strerror}>"
        out.append({"fd": fd, "target": target,
                    "fdinfo": [ln for ln in info.splitlines() if ln.startswith("drm-") or ln.startswith("pos")]})
    return out


CHILD = """
import sys, time, torch
x = torch.empty(2 << 30, dtype=torch.uint8, device="cuda:0"); x.fill_(2); torch.cuda.synchronize()
print("ready", flush=True); sys.stdin.read()
"""


def main():
    rep = {"uid": os.getuid(), "pid": os.getpid(), "before": {"kfd_procs": kfd_procs()}, "nodes": kfd_nodes()}
    rep["before"]["smi"] = smi_process_list()
    import torch
    x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda:0")
    x.fill_(1)
    torch.cuda.synchronize()
    time.sleep(1.2)  # amdsmi asks for >= 1 s between process-list reads
    rep["holding_1gib"] = {"kfd_procs": kfd_procs(), "smi": smi_process_list()}
    rep["self_fdinfo"] = fdinfo()
    import subprocess
    child = subprocess.Popen([sys.executable, "-c", CHILD], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    child.stdout.readline()
    rep["child"] = {"pid": child.pid, "fdinfo": fdinfo(child.pid)}
    try:
        rep["child"]["cgroup"] = open(f"/proc/{child.pid}/cgroup").read()
        rep["child"]["maps_lines"] = sum(1 for _ in open(f"/proc/{child.pid}/maps"))
    except OSError as e:
        rep["child"]["proc_error"] = e.strerror
    time.sleep(1.1)
    rep["child"]["smi"] = smi_process_list()
    child.stdin.close()
    child.wait(30)
    try:
        rep["self_maps_has_kfd"] = sum(1 for ln in open("/proc/self/maps") if "kfd" in ln or "renderD" in ln)
    except OSError:
        pass
    json.dump(rep, sys.stdout, indent=1)
    del x


if __name__ == "__main__":
    main()
