"""Python binding of the HIP visibility/partition probe (native/probe/visibility_probe.hip).

``run(device)`` launches the probe's census, HBM-copy and checksum kernels on a
HIP device and returns its JSON report. ``device_for_bdf`` maps an allocated
device's PCI address (from the plugin's snapshot) to the HIP device ordinal.
Raises if the probe library is missing -- there is no Python fallback.
"""

import ctypes
import json
import os
from functools import lru_cache

from .. import PROBE_LIB


class ProbeError(RuntimeError):
    pass


@lru_cache(maxsize=1)
def _lib():
    if not os.path.exists(PROBE_LIB):
        raise ProbeError(f"{PROBE_LIB} not built (python -m k8s_gpu_sharing_plugin_amd.utils.build)")
    so = ctypes.CDLL(PROBE_LIB)
    so.adp_probe_device_count.restype = ctypes.c_int
    so.adp_probe_list.argtypes = [ctypes.c_char_p, ctypes.c_int]
    so.adp_probe_run.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    return so


def device_count() -> int:
    return _lib().adp_probe_device_count()


def devices() -> list:
    buf = ctypes.create_string_buffer(1 << 16)
    rc = _lib().adp_probe_list(buf, len(buf))
    res = json.loads(buf.value.decode())
    if rc != 0:
        raise ProbeError(res)
    return res


def run(device: int = 0, nbytes: int = 1 << 30, iters: int = 10) -> dict:
    buf = ctypes.create_string_buffer(1 << 14)
    rc = _lib().adp_probe_run(device, nbytes, iters, buf, len(buf))
    res = json.loads(buf.value.decode())
    if rc != 0:
        raise ProbeError(f"probe failed (rc={rc}): {res}")
    return res


def bw_sweep(device: int = 0, nbytes: int = 1 << 30, iters: int = 10) -> list:
    """HBM copy bandwidth of each copy-kernel variant (unroll x NT stores x grid)."""
    so = _lib()
    so.adp_probe_bw_sweep.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_char_p,
                                      ctypes.c_int]
    buf = ctypes.create_string_buffer(1 << 16)
    rc = so.adp_probe_bw_sweep(device, nbytes, iters, buf, len(buf))
    res = json.loads(buf.value.decode())
    if rc != 0:
        raise ProbeError(res)
    return res


def p2p(ndev: int = 0, nbytes: int = 256 << 20, iters: int = 5) -> dict:
    """xGMI peer-read GB/s for every ordered pair of the first `ndev` devices (0 = all)."""
    so = _lib()
    so.adp_probe_p2p.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    buf = ctypes.create_string_buffer(1 << 16)
    rc = so.adp_probe_p2p(ndev, nbytes, iters, buf, len(buf))
    res = json.loads(buf.value.decode())
    if rc != 0:
        raise ProbeError(res)
    return res


def mfma(device: int = 0, iters: int = 1 << 14) -> dict:
    """bf16 MFMA rate (TFLOP/s) and exactness of every accumulator on `device`."""
    so = _lib()
    so.adp_probe_mfma.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    buf = ctypes.create_string_buffer(1 << 12)
    rc = so.adp_probe_mfma(device, iters, buf, len(buf))
    res = json.loads(buf.value.decode())
    if rc != 0:
        raise ProbeError(res)
    return res


def device_for_bdf(bdf: str) -> int:
    """HIP ordinal of the GPU at PCI address `bdf` ("dddd:bb:dd.f"), function ignored."""
    want = bdf.lower().rsplit(".", 1)[0]
    for d in devices():
        if d["pci"].lower().rsplit(".", 1)[0] == want:
            return d["device"]
    raise ProbeError(f"no HIP device at {bdf}; visible: {devices()}")
