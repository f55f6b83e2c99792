"""Runs the HIP probe once on device 0 (used under rocprofv3)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_sharing_plugin_amd.ops import probe
print(json.dumps(probe.run(0, 1 << 30, 20)))
