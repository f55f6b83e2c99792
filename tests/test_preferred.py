"""GetPreferredAllocation over the wire: xGMI/NUMA/partition-aware and replica-aware.

Parity: reference server.go:268-313 and go-gpuallocator besteffort_policy.go
(objective: best total split of the available devices, then the best set that
holds the required ones). Fixes pinned: B5 (no device-library calls per RPC,
partitions supported), B6 (returned IDs are advertised IDs).
"""

import os

import grpc
import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet, native


@pytest.fixture
def plugin(scratch):
    made = []

    def make(fx, args=()):
        k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        d = harness.Daemon(scratch, fx, args=args).start()
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        made.append((k, d, c))
        return c, ids
    yield make
    for k, d, c in made:
        c.close()
        d.stop()
        k.stop()


def pref(c, available, must=(), size=1):
    return list(c.preferred(available, must, size).container_responses[0].deviceIDs)


def idx(ids, chosen):
    return sorted(ids.index(x) for x in chosen)


def test_numa_local_pairs_on_xgmi_mesh(plugin):
    c, ids = plugin(fixtures.node(8))
    assert idx(ids, pref(c, ids, size=2)) == [0, 1]
    assert idx(ids, pref(c, ids, size=4)) == [0, 1, 2, 3]
    assert idx(ids, pref(c, ids, [ids[5]], size=2)) == [4, 5]
    assert idx(ids, pref(c, [ids[i] for i in (0, 4, 5, 6)], size=2)) == [4, 5]
    assert idx(ids, pref(c, ids, size=8)) == list(range(8))


def test_degraded_xgmi_links_are_avoided(plugin):
    fx = fixtures.node(4)
    fx["gpus"][1]["xgmi_links_down"] = 3
    c, ids = plugin(fx)
    assert idx(ids, pref(c, ids, size=2)) == [0, 2]


def test_pcie_only_node_prefers_same_numa(plugin):
    c, ids = plugin(fixtures.node(8, topology="pcie"))
    got = idx(ids, pref(c, [ids[i] for i in (0, 5, 6)], size=2))
    assert got == [5, 6]


def test_unsatisfiable_requests_return_empty(plugin):
    c, ids = plugin(fixtures.node(2))
    assert pref(c, ids[:1], size=2) == []
    assert pref(c, ids, ids, size=1) == []  # must-include larger than the request


def test_unknown_available_device_is_an_error(plugin):
    c, ids = plugin(fixtures.node(2))
    with pytest.raises(grpc.RpcError) as e:
        pref(c, ids + ["ghost"], size=1)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_partitions_stay_on_one_die_and_best_fit(plugin):
    c, ids = plugin(fixtures.node(2, "CPX", memory="NPS2"), args=["--partition-strategy", "single"])
    assert len(ids) == 16
    four = pref(c, ids, size=4)
    assert idx(ids, four) == [0, 1, 2, 3]
    # GPU 0 has exactly 2 free partitions: best fit keeps GPU 1 whole
    avail = [ids[0], ids[1]] + ids[8:]
    assert idx(ids, pref(c, avail, size=2)) == [0, 1]
    # must-include on GPU 1 pulls the rest onto GPU 1
    assert idx(ids, pref(c, avail, [ids[12]], size=3)) == [8, 9, 12]
    # more than one die: fill the die with most room, then the nearest
    assert len(set(i // 8 for i in idx(ids, pref(c, ids, size=10)))) == 2


def test_replicated_resource_uses_prioritizer_and_advertised_ids(plugin):
    c, ids = plugin(fixtures.node(2), args=["--resource-config", "gpu:sharedgpu:4"])
    assert len(ids) == 8
    got = pref(c, ids, size=2)
    assert set(got) <= set(ids)  # B6: suffixed, advertised IDs
    assert len({g.split("-replica-")[0] for g in got}) == 2  # spread over both GPUs


def test_replicated_request_names_only_our_devices_and_no_id_twice(plugin):
    """Replicated resources: a physical device we do not serve is an error (the
    reference's NewDevicesFrom check, server.go:274-278), and an ID listed twice
    in availableDeviceIDs is never handed back twice."""
    c, ids = plugin(fixtures.node(2), args=["--resource-config", "gpu:gpu:3"])
    with pytest.raises(grpc.RpcError) as e:
        c.preferred(["x-replica-0"] + ids, size=1)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT and "unknown device x" in e.value.details()
    with pytest.raises(grpc.RpcError) as e:  # our GPU, a replica number we never advertised
        c.preferred([ids[0].rsplit("-replica-", 1)[0] + "-replica-99"], size=1)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    got = pref(c, [ids[0], ids[0], ids[1]], size=2)
    assert sorted(got) == sorted({ids[0], ids[1]})


def test_rechosen_replicas_are_checked_too(plugin):
    """Found by native/fuzz/fuzz_plugin.cc: an ID listed twice made the handler
    choose again from the de-duplicated list without checking that choice, so
    a made-up replica of one of our GPUs ("<uuid>-replica-1x") came back."""
    c, ids = plugin(fixtures.node(2), args=["--resource-config", "gpu:gpu:3", "--replica-policy", "pack"])
    g0, g1 = ids[:3], ids[3:]
    avail = [g0[1], g1[0], g1[1], g1[1] + "x", g0[0] + "x", g1[1]]
    try:
        got = pref(c, avail, size=3)
    except grpc.RpcError as e:
        assert e.code() == grpc.StatusCode.INVALID_ARGUMENT
    else:
        assert len(set(got)) == 3 and set(got) <= set(ids), got


def test_pack_policy_over_the_wire(plugin):
    c, ids = plugin(fixtures.node(2), args=["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack"])
    assert len(ids) == 2 * (fixtures.MI355X_VRAM_MIB // 1000)
    got = pref(c, ids, size=40)
    assert len(got) == 40 and len({g.split("-replica-")[0] for g in got}) == 1


def test_exact_search_matches_bruteforce_objective():
    """The DP search gives the reference objective's optimum on random score matrices."""
    import itertools
    import random

    rnd = random.Random(7)

    def partitions(items, k):
        if not items:
            yield []
            return
        first, rest = items[0], items[1:]
        size = k if len(items) % k == 0 else len(items) % k
        for combo in itertools.combinations(rest, size - 1):
            group = (first,) + combo
            remaining = [x for x in rest if x not in combo]
            for p in partitions(remaining, k):
                yield [group] + p
        if len(items) % k != 0 and len(items) > k:  # first item in a full group instead
            for combo in itertools.combinations(rest, k - 1):
                group = (first,) + combo
                remaining = [x for x in rest if x not in combo]
                for p in partitions(remaining, k):
                    yield [group] + p

    for trial in range(40):
        n = rnd.randint(2, 8)
        k = rnd.randint(1, n)
        s = [[0] * n for _ in range(n)]
        for a in range(n):
            for b in range(a + 1, n):
                s[a][b] = s[b][a] = rnd.choice([110, 120, 90, 100])
        req = rnd.sample(range(n), rnd.randint(0, min(2, k)))
        flat = [s[a][b] for a in range(n) for b in range(n)]
        got = native.best_effort(list(range(n)), flat, list(range(n)), req, k)

        def score(g):
            return sum(s[a][b] for a, b in itertools.combinations(g, 2))

        best = None
        for p in partitions(list(range(n)), k):
            for g in p:
                if len(g) == k and set(req) <= set(g):
                    key = (sum(score(x) for x in p), score(g))
                    if best is None or key > best:
                        best = key
        assert len(got) == k and set(req) <= set(got)
        total_got = None
        rest = [x for x in range(n) if x not in got]
        for p in partitions(rest, k) if rest else [[]]:
            t = score(got) + sum(score(x) for x in p)
            total_got = t if total_got is None else max(total_got, t)
        assert (total_got, score(got)) == best, (n, k, req, got, best)


def test_pack_spanning_gpus_stays_numa_local(plugin):
    """A memory-unit request larger than one GPU: after the first GPU, the pack
    policy continues on a GPU of the same NUMA node (not simply the best fit)."""
    c, ids = plugin(fixtures.node(8), args=["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack"])
    per = fixtures.MI355X_VRAM_MIB // 1000

    def units(gpu, n):
        prefix = ids[gpu * per].split("-replica-")[0]
        return [i for i in ids if i.startswith(prefix + "-")][:n]
    avail = units(0, per) + units(1, 150) + units(5, 120)   # GPU 0,1 on NUMA 0; GPU 5 on NUMA 1
    got = pref(c, avail, size=per + 106)
    by_gpu = {}
    for g in got:
        by_gpu.setdefault(g.split("-replica-")[0], 0)
        by_gpu[g.split("-replica-")[0]] += 1
    gpu1 = ids[1 * per].split("-replica-")[0]
    gpu5 = ids[5 * per].split("-replica-")[0]
    assert len(got) == per + 106
    assert by_gpu.get(gpu1) == 106 and gpu5 not in by_gpu, by_gpu


def test_memoised_answers_match_fresh_computation(plugin, scratch):
    """<= 8 whole GPUs: answers are memoised per (available, required, size).
    Replayed requests, and the same requests to a fresh daemon (empty cache),
    must give identical answers."""
    import random
    fx = fixtures.node(8)
    fx["gpus"][2]["xgmi_links_down"] = 2
    fx["gpus"][6]["xgmi_links_down"] = 1
    rnd = random.Random(11)
    c, ids = plugin(fx)
    reqs = []
    for _ in range(40):
        avail = sorted(rnd.sample(ids, rnd.randint(1, 8)))
        k = rnd.randint(1, len(avail))
        must = rnd.sample(avail, rnd.randint(0, min(2, k)))
        reqs.append((avail, must, k))
    first = [pref(c, a, m, k) for a, m, k in reqs]
    again = [pref(c, a, m, k) for a, m, k in reqs]
    assert first == again
    # a fresh daemon (empty cache, own plugin directory) computes every answer anew
    d2dir = scratch + ".second"
    os.makedirs(d2dir)
    k2 = kubelet.StubKubelet(os.path.join(d2dir, "kubelet.sock")).start()
    d2 = harness.Daemon(d2dir, fx).start()
    try:
        reg = k2.wait_registration()
        c2 = kubelet.PluginClient(os.path.join(d2dir, reg.endpoint))
        assert [x.ID for x in c2.watch()[0].get(timeout=5).devices] == ids
        fresh = [pref(c2, a, m, k) for a, m, k in reqs]
        c2.close()
    finally:
        d2.stop()
        k2.stop()
    assert fresh == first
    for (a, m, k), got in zip(reqs, first):
        assert len(got) == k and set(m) <= set(got) <= set(a)
