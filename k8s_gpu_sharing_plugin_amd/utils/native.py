"""ctypes binding to libadp_capi.so: the daemon's own C++ core, called in-process.

Used by the tests to pin the reference's test vectors against the exact code the
daemon runs, and by the GPU tests to enumerate real hardware through libamd_smi.
Fails loudly if the library has not been built.
"""

import ctypes
import json
import os
from functools import lru_cache

from .. import CAPI_LIB


class NativeError(RuntimeError):
    pass


@lru_cache(maxsize=1)
def lib() -> ctypes.CDLL:
    if not os.path.exists(CAPI_LIB):
        raise NativeError(f"{CAPI_LIB} not built; run `python -m k8s_gpu_sharing_plugin_amd.utils.build`")
    so = ctypes.CDLL(CAPI_LIB)
    for name in ("adp_prioritize", "adp_strip_replicas", "adp_parse_additional_ids",
                 "adp_parse_resource_config", "adp_best_effort", "adp_snapshot", "adp_plugin_specs",
                 "adp_driver_scan", "adp_kfd_topology_cus"):
        fn = getattr(so, name)
        fn.argtypes = [ctypes.c_char_p]
        fn.restype = ctypes.c_void_p
    so.adp_health_config.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    so.adp_health_config.restype = ctypes.c_void_p
    so.adp_proto_roundtrip.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    so.adp_proto_roundtrip.restype = ctypes.c_void_p
    so.adp_free.argtypes = [ctypes.c_void_p]
    so.adp_version.restype = ctypes.c_char_p
    return so


def _take(ptr) -> object:
    so = lib()
    try:
        text = ctypes.string_at(ptr).decode()
    finally:
        so.adp_free(ptr)
    return json.loads(text)


def _call(name: str, payload) -> object:
    arg = payload if isinstance(payload, str) else json.dumps(payload)
    return _take(getattr(lib(), name)(arg.encode()))


def _check(res):
    if isinstance(res, dict) and "error" in res:
        raise NativeError(res["error"])
    return res


def version() -> str:
    return lib().adp_version().decode()


def prioritize(available, must_include, size, policy="spread"):
    """Returns (ids, non_unique) or raises NativeError with the reference's message."""
    res = _check(_call("adp_prioritize", {"available": list(available), "must_include": list(must_include),
                                           "size": size, "policy": policy}))
    return res["ids"], res["non_unique"]


def driver_scan(proc_root, kfd_proc_dir="", usage_dir="", self_cgroup=""):
    """One driver-side HBM scan (memcap::ScanDriverHbm) of a /proc tree."""
    return _check(_call("adp_driver_scan", {"proc_root": proc_root, "kfd_proc_dir": kfd_proc_dir,
                                            "usage_dir": usage_dir, "self_cgroup": self_cgroup}))


def kfd_topology_cus(topology_dir, node):
    """CUs of a KFD topology node (inventory::KfdTopologyCus), 0 when unreadable."""
    return _check(_call("adp_kfd_topology_cus", {"dir": topology_dir, "node": int(node)}))["cus"]


def strip_replicas(ids):
    return _call("adp_strip_replicas", list(ids))


def parse_additional_ids(text: str):
    return _call("adp_parse_additional_ids", text)


def health_config(disable_value: str = "", poll_ms: str = ""):
    return _take(lib().adp_health_config(disable_value.encode(), poll_ms.encode()))


def parse_resource_config(text: str):
    return _check(_call("adp_parse_resource_config", text))


def best_effort(parent, scores, available, required, size):
    return _call("adp_best_effort", {"parent": parent, "scores": scores, "available": available,
                                      "required": required, "size": size})


def snapshot(lib_path: str = "", devices=None, include_card_nodes=False, sysfs_root=None):
    req = {"lib": lib_path, "include_card_nodes": include_card_nodes}
    if sysfs_root is not None:
        req["sysfs_root"] = sysfs_root
    if devices is not None:
        req["devices"] = list(devices)
    return _check(_call("adp_snapshot", req))


def plugin_specs(lib_path: str = "", strategy="none", resource_config="", devices=None,
                 auto_unit_mib=1000, id_strategy="uuid"):
    req = {"lib": lib_path, "strategy": strategy, "resource_config": resource_config,
           "auto_unit_mib": auto_unit_mib, "id_strategy": id_strategy}
    if devices is not None:
        req["devices"] = list(devices)
    return _check(_call("adp_plugin_specs", req))


class ChurnClient:
    """In-process pod-churn client (native/src/bench/churn.cc) on one plugin socket."""

    def __init__(self, socket_path: str, pod_size=1, rank=0, world=1, preferred=True, grpc_go=False,
                 owned=None):
        so = lib()
        so.adp_bench_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
        so.adp_bench_open.restype = ctypes.c_void_p
        so.adp_bench_run.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        so.adp_bench_run.restype = ctypes.c_void_p
        so.adp_bench_stats.argtypes = [ctypes.c_void_p]
        so.adp_bench_stats.restype = ctypes.c_void_p
        so.adp_bench_reset.argtypes = [ctypes.c_void_p]
        so.adp_bench_close.argtypes = [ctypes.c_void_p]
        err = ctypes.c_void_p()
        cfg = json.dumps({"socket": socket_path, "pod_size": pod_size, "rank": rank, "world": world,
                          "preferred": preferred, "grpc_go": grpc_go,
                          **({"owned": list(owned)} if owned else {})}).encode()
        self._h = so.adp_bench_open(cfg, ctypes.byref(err))
        if not self._h:
            msg = ctypes.string_at(err.value).decode() if err.value else "unknown error"
            so.adp_free(err.value)
            raise NativeError(msg)

    def run(self, pods: int, record: bool = True) -> None:
        err = lib().adp_bench_run(self._h, pods, 1 if record else 0)
        if err:
            msg = ctypes.string_at(err).decode()
            lib().adp_free(err)
            raise NativeError(msg)

    def stats(self) -> dict:
        return _take(lib().adp_bench_stats(self._h))

    def reset(self) -> None:
        lib().adp_bench_reset(self._h)

    def close(self) -> None:
        if self._h:
            lib().adp_bench_close(self._h)
            self._h = None


def proto_roundtrip(msg_type: str, data: bytes) -> bytes:
    res = _check(_take(lib().adp_proto_roundtrip(msg_type.encode(), data, len(data))))
    return bytes.fromhex(res["hex"])


def _open(fn_name: str, cfg: dict):
    so = lib()
    fn = getattr(so, fn_name)
    fn.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
    fn.restype = ctypes.c_void_p
    err = ctypes.c_void_p()
    h = fn(json.dumps(cfg).encode(), ctypes.byref(err))
    if not h:
        msg = ctypes.string_at(err.value).decode() if err.value else "unknown error"
        if err.value:
            so.adp_free(err.value)
        raise NativeError(msg)
    return h


class HostedMonitor:
    """The daemon's health monitor (health::Monitor) running in this process,
    on the real libamd_smi by default: KFD hands an unprivileged registration
    only its own process's per-process events, so a test that then opens the
    GPU from this same process sees real events reach the monitor."""

    def __init__(self, lib_path: str = "", devices=(0,), extra_types: str = "", poll_ms: int = 200):
        self._h = _open("adp_monitor_open", {"lib": lib_path, "devices": list(devices),
                                              "extra_types": extra_types, "poll_ms": poll_ms})
        so = lib()
        so.adp_monitor_state.argtypes = [ctypes.c_void_p]
        so.adp_monitor_state.restype = ctypes.c_void_p
        so.adp_monitor_close.argtypes = [ctypes.c_void_p]

    def state(self) -> dict:
        return _check(_take(lib().adp_monitor_state(self._h)))

    def close(self) -> None:
        if self._h:
            lib().adp_monitor_close(self._h)
            self._h = None


class HostedRelay:
    """The event relay (health::RunEventRelay) serving `socket_path` from a
    thread of this process (see HostedMonitor for why)."""

    def __init__(self, socket_path: str, lib_path: str = "", extra_types: str = ""):
        self._h = _open("adp_relay_open", {"lib": lib_path, "socket": socket_path, "extra_types": extra_types})
        lib().adp_relay_close.argtypes = [ctypes.c_void_p]
        lib().adp_relay_close.restype = ctypes.c_int

    def close(self) -> int:
        rc = 0
        if self._h:
            rc = lib().adp_relay_close(self._h)
            self._h = None
        return rc
