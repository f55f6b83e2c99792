"""MI355X node models rendered as libamdsmi_mock fixtures.

An 8x MI355X OAM node: 8 GPUs, each 256 CUs in 8 XCDs with 288 GB HBM3E
(amdsmi reports 294,896 MiB on the real box, see profiles/discovery.md), a fully
connected xGMI mesh (one hop between any two GPUs), GPUs 0-3 on NUMA node 0 and
4-7 on NUMA node 1. Compute partition modes SPX/DPX/QPX/CPX split each GPU into
1/2/4/8 partitions, each with its own render node and share of HBM; memory
partition modes NPS1/NPS2 decide which combinations are valid.

These models drive every CPU test and the multi-GPU/partition benchmark
configurations that a 1-GPU box cannot exercise (BASELINE.json configs 1, 3-5).
"""

import json
import os

MI355X_VRAM_MIB = 294896  # measured: amd-smi static on the gpurun box
MI355X_CUS = 256
MI355X_XCDS = 8
PARTITIONS = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}


def gpu(index: int, mode: str = "SPX", memory: str = "NPS1", numa=None, **extra) -> dict:
    g = {
        "uuid": f"{0x75a30000 + index:08x}-0000-1000-80c0-{0xbf9907890000 + index:012x}",
        "bdf": f"0000:{0x0c + 0x20 * index:02x}:00.0",
        "numa": (0 if index < 4 else 1) if numa is None else numa,
        "vram_mib": MI355X_VRAM_MIB,
        "num_cu": MI355X_CUS,
        "xcd": MI355X_XCDS,
        "market_name": "AMD Instinct MI355X",
        "compute_partition": mode,
        "memory_partition": memory,
        "partitions": PARTITIONS[mode],
        "render_minor": 128 + 8 * index,
        "card_minor": 8 * index,
    }
    g.update(extra)
    return g


def node(n_gpus: int = 8, modes=None, memory="NPS1", topology="xgmi", **kw) -> dict:
    """A node of `n_gpus` MI355X. `modes` is one mode for all GPUs or a list per GPU."""
    if modes is None:
        modes = "SPX"
    if isinstance(modes, str):
        modes = [modes] * n_gpus
    fx = {"topology": topology, "gpus": [gpu(i, modes[i], memory) for i in range(n_gpus)]}
    fx.update(kw)
    return fx


def write(fixture: dict, directory: str, name: str = "fixture.json") -> str:
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, name)
    with open(path, "w") as f:
        json.dump(fixture, f, indent=1)
    return path


# Named configurations of BASELINE.json.
CONFIGS = {
    # 1: "plugin against stub kubelet on CPU, 2 fake devices via amdsmi mock"
    "mock2": lambda: node(2),
    # 2: "8xMI355X SPX, partitionStrategy=none, one amd.com/gpu:1 pod per GPU"
    "spx8": lambda: node(8),
    # 4: "partitionStrategy=single: CPX mode, 8 compute partitions/GPU -> 64 amd.com/gpu"
    "cpx8": lambda: node(8, "CPX", memory="NPS2"),
    # 5: "partitionStrategy=mixed SPX+CPX node"
    "mixed8": lambda: node(8, ["SPX"] * 4 + ["CPX"] * 4, memory="NPS2"),
}
