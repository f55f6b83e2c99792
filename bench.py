#!/usr/bin/env python3
"""Headline benchmark: Allocate() p50 latency + allocatable amd.com/gpu count.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Starts the native amdgpu-device-plugin daemon against a native stub kubelet
and drives synthetic pod churn from one client per GPU; see
k8s_gpu_sharing_plugin_amd/parallel/bench.py. Rank 0 prints one JSON line.
Builds the native tree first if it is missing.
"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from k8s_gpu_sharing_plugin_amd import DAEMON, CAPI_LIB, PROBE_LIB  # noqa: E402


def _ensure_built():
    if os.environ.get("RANK", "0") != "0":
        # Other ranks wait for rank 0's build by polling for the artefacts.
        import time
        for _ in range(600):
            if os.path.exists(DAEMON) and os.path.exists(CAPI_LIB):
                return
            time.sleep(0.5)
        return
    if not (os.path.exists(DAEMON) and os.path.exists(CAPI_LIB)):
        from k8s_gpu_sharing_plugin_amd.utils import build
        build.build_native()
    if not os.path.exists(PROBE_LIB):
        try:
            from k8s_gpu_sharing_plugin_amd.utils import build
            build.build_probe()
        except Exception as e:  # probe is reported, not required for the metric
            print(f"warning: HIP probe not built: {e}", file=sys.stderr)


if __name__ == "__main__":
    _ensure_built()
    from k8s_gpu_sharing_plugin_amd.parallel import bench
    bench.main()
