"""PyTorch under the HBM-cap shim with each allocator configuration
(PYTORCH_CUDA_ALLOC_CONF=backend:native | backend:cudaMallocAsync, the latter
hipMallocAsync / hipFreeAsync on ROCm, whose freed blocks stay in the
stream-ordered pool; expandable_segments:True is reported unsupported by
PyTorch 2.10 on ROCm 7 and falls back to the native allocator): the grant is the device's memory, a freed 3 GiB can be
allocated again, 2 GiB more past a 4000 MiB grant are refused, and 200 rounds
of 512 MiB allocate/free all succeed. One JSON line; run with the shim
preloaded and a grant (tests/test_gpu.py::test_memcap_with_pytorch_allocator_configs).
"""
import json, os, torch
torch.cuda.init()
res = {"backend": torch.cuda.get_allocator_backend(), "conf": os.environ.get("PYTORCH_CUDA_ALLOC_CONF", "")}
free, total = torch.cuda.mem_get_info()
res["total_mib"] = total >> 20
def alloc(gib):
    try:
        return torch.empty(int(gib * (1 << 30)), dtype=torch.uint8, device="cuda")
    except torch.OutOfMemoryError:
        return None
a = alloc(3); res["first_3g"] = a is not None
del a; torch.cuda.synchronize()
b = alloc(3); res["second_3g_after_free"] = b is not None
c = alloc(2); res["extra_2g_while_holding_3g"] = c is not None
del b, c; torch.cuda.synchronize()
ok = 0
for i in range(200):
    t = alloc(0.5)
    if t is not None:
        ok += 1
    del t
res["churn_500m_ok"] = ok
print(json.dumps(res))
