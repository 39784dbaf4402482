"""Wire-format pins for the hand-built v1beta1 descriptors + allocator properties."""
import itertools

from hypothesis import given, settings
from hypothesis import strategies as st

from kgs.deviceplugin import api
from kgs.deviceplugin.allocator import DevInfo, preferred


def test_register_request_golden_bytes():
    r = api.RegisterRequest(version="v1beta1", endpoint="x.sock", resource_name="amd.com/gpu",
                            options=api.DevicePluginOptions(get_preferred_allocation_available=True))
    # field 1 "v1beta1", field 2 "x.sock", field 3 "amd.com/gpu", field 4 {field 2: true}
    assert r.SerializeToString().hex() == (
        "0a07763162657461311206782e736f636b1a0b616d642e636f6d2f67707522021001"
    )


def test_container_allocate_response_golden_bytes():
    c = api.ContainerAllocateResponse(envs={"A": "1"}, devices=[
        api.DeviceSpec(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")])
    assert c.SerializeToString().hex() == (
        "0a060a01411201311a180a082f6465762f6b666412082f6465762f6b66641a027277"
    )


def test_device_with_topology_roundtrip():
    d = api.Device(ID="0000:05:00.0", health=api.HEALTHY)
    d.topology.nodes.add(ID=1)
    b = api.ListAndWatchResponse(devices=[d]).SerializeToString()
    back = api.ListAndWatchResponse.FromString(b)
    assert back.devices[0].ID == "0000:05:00.0" and back.devices[0].topology.nodes[0].ID == 1
    # Device{ID=1 string, health=2 string, topology=3 {nodes=1 {ID=1 int64}}}
    # ListAndWatchResponse{devices=1 {ID=1 "0000:05:00.0", health=2 "Healthy", topology=3 {nodes=1 {ID=1: 1}}}}
    assert b.hex() == "0a1d0a0c303030303a30353a30302e3012074865616c7468791a040a020801"


def test_method_paths():
    assert api.method_path("Registration", "Register") == "/v1beta1.Registration/Register"
    assert api.method_path("DevicePlugin", "ListAndWatch") == "/v1beta1.DevicePlugin/ListAndWatch"
    svc = api.FILE_DESCRIPTOR.services_by_name["DevicePlugin"]
    assert [m.name for m in svc.methods] == ["GetDevicePluginOptions", "ListAndWatch", "GetPreferredAllocation",
                                             "Allocate", "PreStartContainer"]
    assert svc.methods_by_name["ListAndWatch"].server_streaming
    assert not svc.methods_by_name["Allocate"].server_streaming


def test_field_numbers_match_upstream():
    m = api.ContainerAllocateResponse.DESCRIPTOR
    assert {f.name: f.number for f in m.fields} == {"envs": 1, "mounts": 2, "devices": 3, "annotations": 4,
                                                     "cdi_devices": 5}
    assert m.fields_by_name["envs"].message_type.GetOptions().map_entry
    p = api.ContainerPreferredAllocationRequest.DESCRIPTOR
    assert {f.name: f.number for f in p.fields} == {"available_deviceIDs": 1, "must_include_deviceIDs": 2,
                                                    "allocation_size": 3}


def _mesh(n, numa_split=2, missing=()):
    devs = {}
    for i in range(n):
        peers = frozenset(j + 10 for j in range(n) if j != i and frozenset((i, j)) not in missing)
        devs[f"g{i}"] = DevInfo(f"g{i}", i, (i * numa_split) // n, i + 10, peers)
    return devs


@settings(max_examples=200, deadline=None)
@given(n=st.integers(1, 8), data=st.data())
def test_preferred_invariants(n, data):
    devs = _mesh(n)
    ids = list(devs)
    avail = data.draw(st.lists(st.sampled_from(ids), min_size=1, max_size=n, unique=True))
    must = data.draw(st.lists(st.sampled_from(avail), max_size=len(avail), unique=True))
    size = data.draw(st.integers(len(must) if must else 1, len(avail)))
    got = preferred(avail, must, size, devs)
    assert len(got) == size
    assert len(set(got)) == size
    assert set(got) <= set(avail)
    assert set(must) <= set(got)
    assert got == preferred(avail, must, size, devs)  # deterministic


def test_preferred_avoids_broken_xgmi_pair():
    # 4 GPUs, link 0<->1 missing: a 2-GPU request must not pick {0,1}
    devs = _mesh(4, numa_split=1, missing={frozenset((0, 1))})
    got = preferred(list(devs), [], 2, devs)
    assert set(got) != {"g0", "g1"}
    # 3 GPUs: best all-xGMI triple excludes one of 0/1
    got3 = preferred(list(devs), [], 3, devs)
    assert not {"g0", "g1"} <= set(got3)


def test_preferred_greedy_large():
    devs = _mesh(32, numa_split=4)
    got = preferred(list(devs), [], 16, devs)
    assert len(got) == 16
    assert len({devs[i].numa for i in got}) == 2  # 16 GPUs fill 2 of the 4 NUMA groups
    for a, b in itertools.combinations(got, 2):
        assert devs[a].index != devs[b].index
