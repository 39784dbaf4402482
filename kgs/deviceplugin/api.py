"""Kubelet device-plugin API ``v1beta1``, built at import time (no protoc).

There is no protoc / grpc_tools in this environment, so the
``k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1`` messages are declared here as a
``FileDescriptorProto`` and turned into message classes with
``message_factory.GetMessageClass``. Wire compatibility with the kubelet depends
only on the package name, service/method names, field numbers and field types,
all of which follow the upstream ``api.proto``; ``tests/test_deviceplugin_api.py``
pins the encoded bytes.

The reference never speaks this API itself: its upstream Go plugins do, and the
ROCm one is deployed without the kubelet socket mount so it can never register
(kind-gpu-sim.sh:248-276).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "v1beta1"
VERSION = "v1beta1"
KUBELET_SOCKET = "kubelet.sock"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

_F = descriptor_pb2.FieldDescriptorProto
_STR, _BOOL, _I32, _I64, _MSG = _F.TYPE_STRING, _F.TYPE_BOOL, _F.TYPE_INT32, _F.TYPE_INT64, _F.TYPE_MESSAGE
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED

# (message name, [(field name, number, type, label, type_name or None)])
_MESSAGES = [
    ("DevicePluginOptions", [("pre_start_required", 1, _BOOL, _OPT, None),
                             ("get_preferred_allocation_available", 2, _BOOL, _OPT, None)]),
    ("RegisterRequest", [("version", 1, _STR, _OPT, None),
                         ("endpoint", 2, _STR, _OPT, None),
                         ("resource_name", 3, _STR, _OPT, None),
                         ("options", 4, _MSG, _OPT, "DevicePluginOptions")]),
    ("Empty", []),
    ("ListAndWatchResponse", [("devices", 1, _MSG, _REP, "Device")]),
    ("TopologyInfo", [("nodes", 1, _MSG, _REP, "NUMANode")]),
    ("NUMANode", [("ID", 1, _I64, _OPT, None)]),
    ("Device", [("ID", 1, _STR, _OPT, None),
                ("health", 2, _STR, _OPT, None),
                ("topology", 3, _MSG, _OPT, "TopologyInfo")]),
    ("PreStartContainerRequest", [("devices_ids", 1, _STR, _REP, None)]),
    ("PreStartContainerResponse", []),
    ("PreferredAllocationRequest", [("container_requests", 1, _MSG, _REP, "ContainerPreferredAllocationRequest")]),
    ("ContainerPreferredAllocationRequest", [("available_deviceIDs", 1, _STR, _REP, None),
                                             ("must_include_deviceIDs", 2, _STR, _REP, None),
                                             ("allocation_size", 3, _I32, _OPT, None)]),
    ("PreferredAllocationResponse", [("container_responses", 1, _MSG, _REP, "ContainerPreferredAllocationResponse")]),
    ("ContainerPreferredAllocationResponse", [("deviceIDs", 1, _STR, _REP, None)]),
    ("AllocateRequest", [("container_requests", 1, _MSG, _REP, "ContainerAllocateRequest")]),
    ("ContainerAllocateRequest", [("devices_ids", 1, _STR, _REP, None)]),
    ("CDIDevice", [("name", 1, _STR, _OPT, None)]),
    ("AllocateResponse", [("container_responses", 1, _MSG, _REP, "ContainerAllocateResponse")]),
    ("ContainerAllocateResponse", [("envs", 1, _MSG, _REP, "ContainerAllocateResponse.EnvsEntry"),
                                   ("mounts", 2, _MSG, _REP, "Mount"),
                                   ("devices", 3, _MSG, _REP, "DeviceSpec"),
                                   ("annotations", 4, _MSG, _REP, "ContainerAllocateResponse.AnnotationsEntry"),
                                   ("cdi_devices", 5, _MSG, _REP, "CDIDevice")]),
    ("Mount", [("container_path", 1, _STR, _OPT, None),
               ("host_path", 2, _STR, _OPT, None),
               ("read_only", 3, _BOOL, _OPT, None)]),
    ("DeviceSpec", [("container_path", 1, _STR, _OPT, None),
                    ("host_path", 2, _STR, _OPT, None),
                    ("permissions", 3, _STR, _OPT, None)]),
]

# map<string,string> fields are repeated nested *Entry messages with map_entry=true
_MAP_ENTRIES = {"ContainerAllocateResponse": ["EnvsEntry", "AnnotationsEntry"]}

SERVICES = {
    "Registration": [("Register", "RegisterRequest", "Empty", False)],
    "DevicePlugin": [
        ("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
        ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
        ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
        ("Allocate", "AllocateRequest", "AllocateResponse", False),
        ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False),
    ],
}


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "kgs/deviceplugin/v1beta1/api.proto"
    fd.package = PACKAGE
    fd.syntax = "proto3"
    for name, fields in _MESSAGES:
        m = fd.message_type.add()
        m.name = name
        for fname, num, ftype, label, tname in fields:
            f = m.field.add()
            f.name, f.number, f.type, f.label = fname, num, ftype, label
            f.json_name = fname
            if tname:
                f.type_name = f".{PACKAGE}.{tname}"
        for entry in _MAP_ENTRIES.get(name, []):
            e = m.nested_type.add()
            e.name = entry
            e.options.map_entry = True
            for fname, num in (("key", 1), ("value", 2)):
                f = e.field.add()
                f.name, f.number, f.type, f.label = fname, num, _STR, _OPT
                f.json_name = fname
    for sname, methods in SERVICES.items():
        s = fd.service.add()
        s.name = sname
        for mname, req, resp, stream in methods:
            mm = s.method.add()
            mm.name = mname
            mm.input_type = f".{PACKAGE}.{req}"
            mm.output_type = f".{PACKAGE}.{resp}"
            mm.server_streaming = stream
    return fd


_POOL = descriptor_pool.DescriptorPool()
FILE_DESCRIPTOR = _POOL.Add(_build_file())
_FILE = _POOL.FindFileByName("kgs/deviceplugin/v1beta1/api.proto")

_classes = {}
for _name, _ in _MESSAGES:
    _classes[_name] = message_factory.GetMessageClass(_POOL.FindMessageTypeByName(f"{PACKAGE}.{_name}"))
globals().update(_classes)

DevicePluginOptions = _classes["DevicePluginOptions"]
RegisterRequest = _classes["RegisterRequest"]
Empty = _classes["Empty"]
ListAndWatchResponse = _classes["ListAndWatchResponse"]
TopologyInfo = _classes["TopologyInfo"]
NUMANode = _classes["NUMANode"]
Device = _classes["Device"]
PreStartContainerRequest = _classes["PreStartContainerRequest"]
PreStartContainerResponse = _classes["PreStartContainerResponse"]
PreferredAllocationRequest = _classes["PreferredAllocationRequest"]
ContainerPreferredAllocationRequest = _classes["ContainerPreferredAllocationRequest"]
PreferredAllocationResponse = _classes["PreferredAllocationResponse"]
ContainerPreferredAllocationResponse = _classes["ContainerPreferredAllocationResponse"]
AllocateRequest = _classes["AllocateRequest"]
ContainerAllocateRequest = _classes["ContainerAllocateRequest"]
CDIDevice = _classes["CDIDevice"]
AllocateResponse = _classes["AllocateResponse"]
ContainerAllocateResponse = _classes["ContainerAllocateResponse"]
Mount = _classes["Mount"]
DeviceSpec = _classes["DeviceSpec"]


def method_path(service: str, method: str) -> str:
    return f"/{PACKAGE}.{service}/{method}"


def message(name: str):
    return _classes[name]
