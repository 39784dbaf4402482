"""What a captured hipGraph contains: node types, and the memset nodes' targets.

Round 5 traced the serving fault to a memset node (a captured
``hipMemsetAsync``) that left garbage in a ticket slot instead of zeros
(profiles/r5/fault/README.md). Every memset path of ours that can be captured
was replaced by a kernel node, but torch or a library could put memset nodes
into the graphs the serving engine captures. This walks a graph -- child
graphs included -- through the HIP graph API (ctypes on the HIP runtime the
process already has loaded: torch's), so a test can assert that the serving
graphs hold no memset node, or check each one's target after a replay.

    g = torch.cuda.CUDAGraph(keep_graph=True)   # the hipGraph_t must be kept
    ...capture...
    audit(g)  -> {"nodes": 412, "types": {"kernel": 410, "memcpy": 2}, "memsets": []}
"""
from __future__ import annotations

import ctypes
import os

NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
              7: "event_record", 8: "ext_semaphore_signal", 9: "ext_semaphore_wait", 10: "mem_alloc",
              11: "mem_free", 12: "memcpy_from_symbol", 13: "memcpy_to_symbol", 14: "batch_mem_op"}
MEMSET = 2
GRAPH = 4


class MemsetParams(ctypes.Structure):  # hipMemsetParams (hip_runtime_api.h)
    _fields_ = [("dst", ctypes.c_void_p), ("elementSize", ctypes.c_uint), ("height", ctypes.c_size_t),
                ("pitch", ctypes.c_size_t), ("value", ctypes.c_uint), ("width", ctypes.c_size_t)]


_HIP = None


def hip_runtime() -> ctypes.CDLL:
    """The HIP runtime this process already uses (torch's bundled
    libamdhip64.so when torch loaded one): a second runtime in one process
    would have its own device state."""
    global _HIP
    if _HIP is None:
        path = None
        try:
            with open("/proc/self/maps") as f:
                for ln in f:
                    if "libamdhip64.so" in ln:
                        path = ln.split()[-1]
                        break
        except OSError:
            pass
        lib = ctypes.CDLL(path or "libamdhip64.so")
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.hipGraphGetNodes.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(sz)]
        lib.hipGraphNodeGetType.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
        lib.hipGraphChildGraphNodeGetGraph.argtypes = [vp, ctypes.POINTER(vp)]
        lib.hipGraphMemsetNodeGetParams.argtypes = [vp, ctypes.POINTER(MemsetParams)]
        for fn in ("hipGraphGetNodes", "hipGraphNodeGetType", "hipGraphChildGraphNodeGetGraph",
                   "hipGraphMemsetNodeGetParams"):
            getattr(lib, fn).restype = ctypes.c_int
        _HIP = lib
    return _HIP


def _ck(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: hipError {rc}")


def nodes(raw_graph: int) -> list:
    """(node handle, type) of every node of ``raw_graph`` (a hipGraph_t as int),
    child graphs expanded in place."""
    hip = hip_runtime()
    n = ctypes.c_size_t(0)
    _ck(hip.hipGraphGetNodes(ctypes.c_void_p(raw_graph), None, ctypes.byref(n)), "hipGraphGetNodes")
    arr = (ctypes.c_void_p * max(1, n.value))()
    _ck(hip.hipGraphGetNodes(ctypes.c_void_p(raw_graph), arr, ctypes.byref(n)), "hipGraphGetNodes")
    out = []
    for i in range(n.value):
        t = ctypes.c_int(-1)
        _ck(hip.hipGraphNodeGetType(ctypes.c_void_p(arr[i]), ctypes.byref(t)), "hipGraphNodeGetType")
        if t.value == GRAPH:
            child = ctypes.c_void_p()
            _ck(hip.hipGraphChildGraphNodeGetGraph(ctypes.c_void_p(arr[i]), ctypes.byref(child)),
                "hipGraphChildGraphNodeGetGraph")
            out.extend(nodes(child.value))
        else:
            out.append((arr[i], t.value))
    return out


def audit_raw(raw_graph: int) -> dict:
    """Node count, count per type, and every memset node's parameters."""
    types: dict = {}
    memsets = []
    hip = hip_runtime()
    for node, t in nodes(raw_graph):
        name = NODE_TYPES.get(t, f"type{t}")
        types[name] = types.get(name, 0) + 1
        if t == MEMSET:
            p = MemsetParams()
            _ck(hip.hipGraphMemsetNodeGetParams(ctypes.c_void_p(node), ctypes.byref(p)),
                "hipGraphMemsetNodeGetParams")
            memsets.append({"dst": p.dst or 0, "element_size": p.elementSize, "width": p.width,
                            "height": p.height, "pitch": p.pitch, "value": p.value})
    return {"nodes": sum(types.values()), "types": types, "memsets": memsets}


def audit(graph) -> dict:
    """:func:`audit_raw` of a ``torch.cuda.CUDAGraph`` made with ``keep_graph=True``."""
    return audit_raw(int(graph.raw_cuda_graph()))


def enabled() -> bool:
    """``KGS_GRAPH_AUDIT=1``: the serving engine keeps its hipGraphs and audits each capture."""
    return os.environ.get("KGS_GRAPH_AUDIT", "0") == "1"
