"""`kgs create --gpus N`: which N GPUs get advertised (kgs.cluster.select_gpus).

Properties over random host topologies (hypothesis): exactly N distinct GPUs
out of the healthy ones, deterministic, one xGMI island whenever one of size N
exists, and the fewest NUMA nodes among such islands. Plus the cross-check
that the cluster-level choice is the device plugin's own GetPreferredAllocation
answer over real gRPC, so `create --gpus N` and a pod asking the full plugin
for N land on the same GPUs.
"""
import itertools
import os
import tempfile
from dataclasses import dataclass, field

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from kgs.cluster import ProvisionError, select_gpus


@dataclass
class G:
    index: int
    render_minor: int
    numa_node: int
    node_id: int
    peers: set = field(default_factory=set)

    def xgmi_peers(self):
        return set(self.peers)


@st.composite
def hosts(draw):
    n = draw(st.integers(1, 8))
    gpus = [G(i, 128 + 8 * i, draw(st.integers(0, 1)), 2 + i) for i in range(n)]
    for a, b in itertools.combinations(range(n), 2):
        if draw(st.booleans()):
            gpus[a].peers.add(gpus[b].node_id)
            gpus[b].peers.add(gpus[a].node_id)
    k = draw(st.integers(1, n))
    return gpus, k


def _island(gs):
    return all(b.node_id in a.peers for a, b in itertools.combinations(gs, 2))


@settings(max_examples=300, deadline=None)
@given(hosts())
def test_selection_properties(host):
    gpus, k = host
    pick = select_gpus(gpus, k)
    assert len(pick) == k and len({g.render_minor for g in pick}) == k
    assert all(g in gpus for g in pick)
    assert [g.index for g in pick] == sorted(g.index for g in pick)
    assert select_gpus(gpus, k) == pick  # deterministic
    islands = [c for c in itertools.combinations(gpus, k) if _island(c)]
    if islands:
        assert _island(pick)
        assert len({g.numa_node for g in pick}) == min(len({g.numa_node for g in c}) for c in islands)


def test_selection_bounds():
    gpus = [G(i, 128 + 8 * i, 0, 2 + i) for i in range(4)]
    assert select_gpus(gpus, None) == gpus
    with pytest.raises(ProvisionError):
        select_gpus(gpus, 5)
    with pytest.raises(ProvisionError):
        select_gpus(gpus, 0)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 6])
def test_cluster_choice_is_the_plugins_preferred_allocation(n):
    """Over real gRPC: the plugin serving all 8 fake GPUs answers
    GetPreferredAllocation(size n) with exactly the GPUs select_gpus picks."""
    from kgs import gpuinfo
    from kgs.deviceplugin.fake_kubelet import FakeKubelet
    from kgs.deviceplugin.server import AmdGpuDevicePlugin, RealSource
    from kgs.gpuinfo.fake import make_fake_mi355x

    d = tempfile.mkdtemp(prefix="kgs-sel", dir="/tmp")
    root = str(make_fake_mi355x(os.path.join(d, "host")))
    gpus = [g for g in gpuinfo.discover(root, use_amdsmi=False).gpus if g.healthy]
    want = sorted(g.render_minor for g in select_gpus(gpus, n))
    kub = FakeKubelet(d)
    kub.start()
    src = RealSource(root, None, use_amdsmi=False)
    plug = AmdGpuDevicePlugin(src, plugin_dir=d)
    try:
        plug.start()
        plug.register()
        plug.notify()
        assert kub.wait(lambda: kub.capacity() == 8, timeout=10)
        ids = [i for i, h, _ in kub.latest_devices() if h == "Healthy"]
        got_ids = kub.preferred(ids, [], n)
        minor_of = {dv.id: dv.render_minor for dv in src.devices()}
        assert sorted(minor_of[i] for i in got_ids) == want
    finally:
        plug.stop()
        kub.stop()
