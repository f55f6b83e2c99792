"""Reference test vectors, run against the daemon's own C++ code via libadp_capi.

cmd/nvidia-device-plugin/replica_test.go:37-96   Test_prioritizeDevices (15 cases)
cmd/nvidia-device-plugin/replica_test.go:120-122 Test_stripReplicas (3 cases)
"""

import pytest

from k8s_gpu_sharing_plugin_amd.utils import native

MISSING = "device '{}' in mustIncludeDeviceIDs is missing from availableDeviceIDs"
NO_DEVICES = "no devices left to allocate"

# name, available, must_include, size, want ids (None = error), want non_unique, want error
CASES = [
    ("Basic", ["a-replica-0", "a-replica-1", "b-replica-1"], [], 1, ["a-replica-0"], False, None),
    ("Multiple Unique", ["a-replica-0", "a-replica-1", "b-replica-1"], [], 2,
     ["a-replica-0", "b-replica-1"], False, None),
    ("NonuniqueError", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"], [], 3,
     ["a-replica-0", "a-replica-1", "b-replica-1"], True, None),
    ("Must Include Greater Utilized", ["a-replica-0", "a-replica-1", "b-replica-1"], ["b-replica-1"], 1,
     ["b-replica-1"], False, None),
    ("Must Include Least Utilized", ["a-replica-0", "a-replica-1", "b-replica-1"], ["a-replica-1"], 1,
     ["a-replica-1"], False, None),
    ("Must Include Two", ["a-replica-0", "a-replica-1", "b-replica-1"], ["a-replica-1"], 2,
     ["a-replica-1", "b-replica-1"], False, None),
    ("NonuniqueError Must Include", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-2", "b-replica-1"],
     ["a-replica-2"], 3, ["a-replica-0", "a-replica-2", "b-replica-1"], True, None),
    ("Must Include", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1", "c-replica-0"],
     ["a-replica-2"], 3, ["a-replica-2", "b-replica-1", "c-replica-0"], False, None),
    ("Must Include Entire Allocated", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"],
     ["a-replica-2", "b-replica-1", "a-replica-1"], 3, ["a-replica-1", "a-replica-2", "b-replica-1"], True, None),
    ("Deterministic", [f"{c}-replica-1" for c in "abcdefgh"], [], 1, ["a-replica-1"], False, None),
    ("OversizedRequest", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"], [], 5, None, False,
     NO_DEVICES),
    ("Undersized", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"], [], 0, [], False, None),
    ("NoneAvailable", [], [], 1, None, False, NO_DEVICES),
    ("SubsetSame", ["a-replica-0", "a-replica-1"], ["a-replica-2"], 1, None, False, MISSING.format("a-replica-2")),
    ("SubsetDifferent", ["a-replica-0", "a-replica-1"], ["b-replica-2"], 1, None, False,
     MISSING.format("b-replica-2")),
]


# "auto" is the daemon's default: a time-slice resource resolves it to spread,
# so the reference's vectors hold under it unchanged.
@pytest.mark.parametrize("policy", ["spread", "auto"])
@pytest.mark.parametrize("name,avail,must,size,want,non_unique,err", CASES, ids=[c[0] for c in CASES])
def test_prioritize_devices_reference_vectors(name, avail, must, size, want, non_unique, err, policy):
    if err is not None:
        with pytest.raises(native.NativeError) as e:
            native.prioritize(avail, must, size, policy=policy)
        assert str(e.value) == err
        return
    ids, nu = native.prioritize(avail, must, size, policy=policy)
    assert ids == want
    assert nu == non_unique


@pytest.mark.parametrize("ids,want", [
    (["b-replica-5", "a-replica-1", "a-replica-0"], ["a", "b"]),
    (["b-replica-0", "a-replica-1", "a-replica-2", "c-replica-2"], ["a", "b", "c"]),
    ([], []),
])
def test_strip_replicas_reference_vectors(ids, want):
    assert native.strip_replicas(ids) == want


def test_must_include_larger_than_size_is_an_error_not_a_panic():
    # Reference defect B12: make([]string, len(must), size) panics.
    with pytest.raises(native.NativeError):
        native.prioritize(["a-replica-0", "b-replica-0"], ["a-replica-0", "b-replica-0"], 1)


def test_pack_policy_keeps_memory_units_on_one_gpu():
    # B19: a 20-unit gpu-mem-gb request must come from one GPU.
    avail = [f"g{g}-replica-{i}" for g in range(4) for i in range(30 if g else 10)]
    ids, nu = native.prioritize(avail, [], 20, policy="pack")
    assert len(ids) == 20 and not nu
    assert len({i.split("-replica-")[0] for i in ids}) == 1
    # best fit: a GPU with exactly enough room beats a bigger one
    avail = [f"big-replica-{i}" for i in range(40)] + [f"fit-replica-{i}" for i in range(20)]
    ids, _ = native.prioritize(avail, [], 20, policy="pack")
    assert {i.split("-replica-")[0] for i in ids} == {"fit"}


def test_spread_vs_pack_on_the_same_input():
    avail = [f"{g}-replica-{i}" for g in "ab" for i in range(4)]
    spread, nu = native.prioritize(avail, [], 2)
    assert {i.split("-replica-")[0] for i in spread} == {"a", "b"} and not nu
    pack, _ = native.prioritize(avail, [], 2, policy="pack")
    assert len({i.split("-replica-")[0] for i in pack}) == 1


def _reference_prioritize(avail, must, size, join="-replica-"):
    """Executable model of the reference's prioritizeDevices
    (cmd/nvidia-device-plugin/replica.go:95-198): group by the text before the
    first join, sort each group, take must-includes by swap-remove, then pick
    the unallocated device with the most replicas left (ties: first in sorted
    key order), else the allocated one with the most left."""
    pools = {}
    for i in avail:
        pools.setdefault(i.split(join)[0], []).append(i)
    for v in pools.values():
        v.sort()
    used = set()
    out = list(must)
    unique = True
    for m in must:
        dev = m.split(join)[0]
        if dev not in pools or m not in pools[dev]:
            return None, None
        if dev in used:
            unique = False
        lst = pools[dev]
        k = lst.index(m)
        lst[k] = lst[-1]
        lst.pop()
        used.add(dev)
    for _ in range(len(out), size):
        best_u = best_a = None
        hi_u = hi_a = 0
        for dev in sorted(pools):
            n = len(pools[dev])
            if dev in used:
                if n > hi_a:
                    best_a, hi_a = dev, n
            elif n > hi_u:
                best_u, hi_u = dev, n
        pick = best_u if best_u is not None else best_a
        if pick is None:
            return None, None
        if pick in used:
            unique = False
        out.append(pools[pick].pop(0))
        used.add(pick)
    return sorted(out), not unique


def test_prioritize_matches_reference_model_on_random_and_adversarial_ids():
    """Randomised differential test of the C++ prioritizer against the model
    above, including IDs where the join overlaps the device prefix
    ("x-replica" + "-replica-0"), IDs without a join and unsorted lists."""
    import random
    rng = random.Random(7)
    stems = ["a", "b", "x-replica", "x", "gpu-7-replica", "75a30000-0000-1000-80c0-bf9907890000", "-", "r-"]
    for trial in range(400):
        avail = []
        for s in rng.sample(stems, rng.randint(1, len(stems))):
            n = rng.randint(0, 6)
            avail += [f"{s}-replica-{i}" for i in rng.sample(range(20), n)]
            if rng.random() < 0.2:
                avail.append(s)  # a non-replicated ID
        avail = list(dict.fromkeys(avail))
        if rng.random() < 0.5:
            avail.sort()
        else:
            rng.shuffle(avail)
        must = rng.sample(avail, min(len(avail), rng.randint(0, 2)))
        size = rng.randint(len(must), len(must) + 4)
        want, want_nu = _reference_prioritize(avail, must, size)
        if want is None:
            with pytest.raises(native.NativeError):
                native.prioritize(avail, must, size)
            continue
        ids, nu = native.prioritize(avail, must, size)
        assert (ids, nu) == (want, want_nu), (trial, avail, must, size)


def _pack_model(avail, must, size, join="-replica-"):
    """Executable model of the pack policy (no topology affinity): must-includes
    as in the reference, then finish on the devices the request already touches
    (sorted key order), then best fit -- the smallest untouched device that
    holds the rest, else the largest -- taking each device's smallest IDs."""
    pools = {}
    for i in avail:
        pools.setdefault(i.split(join)[0], []).append(i)
    for v in pools.values():
        v.sort()
    used, out = set(), list(must)
    for m in must:
        dev = m.split(join)[0]
        if dev not in pools or m not in pools[dev]:
            return None
        lst = pools[dev]
        k = lst.index(m)
        lst[k] = lst[-1]
        lst.pop()
        used.add(dev)
    need = size - len(out)

    def take(dev, n):
        got = pools[dev][:n]
        del pools[dev][:n]
        out.extend(got)
        used.add(dev)
        return len(got)
    for dev in sorted(pools):
        if need > 0 and dev in used:
            need -= take(dev, need)
    while need > 0:
        fit = largest = None
        for dev in sorted(pools):
            n = len(pools[dev])
            if dev in used or n == 0:
                continue
            if n >= need and (fit is None or n < len(pools[fit])):
                fit = dev
            if largest is None or n > len(pools[largest]):
                largest = dev
        pick = fit if fit is not None else largest
        if pick is None:
            return None
        need -= take(pick, need)
    return sorted(out)


def test_pack_matches_its_model_on_random_ids():
    """Randomised differential test of the pack policy (one partial sort per
    device taken from) against the model above."""
    import random
    rng = random.Random(11)
    stems = ["a", "b", "c", "x-replica", "75a30000-0000-1000-80c0-bf9907890000", "r-"]
    for trial in range(400):
        avail = []
        for s in rng.sample(stems, rng.randint(1, len(stems))):
            avail += [f"{s}-replica-{i}" for i in rng.sample(range(40), rng.randint(0, 12))]
        avail = list(dict.fromkeys(avail))
        rng.shuffle(avail)
        must = rng.sample(avail, min(len(avail), rng.randint(0, 2)))
        size = rng.randint(len(must), len(must) + 20)
        want = _pack_model(avail, must, size)
        if want is None:
            with pytest.raises(native.NativeError):
                native.prioritize(avail, must, size, policy="pack")
            continue
        ids, _ = native.prioritize(avail, must, size, policy="pack")
        assert ids == want, (trial, avail, must, size)
