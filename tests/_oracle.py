"""ctypes handle on the CPU oracle (oracle/lib/libksg_oracle.so).

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use this module.
"""
import ctypes
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "lib", "libksg_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB)
        L.ksg_oracle_load.restype = ctypes.c_void_p
        L.ksg_oracle_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.ksg_oracle_free.argtypes = [ctypes.c_void_p]
        L.ksg_oracle_num_nodes.argtypes = [ctypes.c_void_p]
        L.ksg_oracle_num_queue.argtypes = [ctypes.c_void_p]
        L.ksg_oracle_schedule.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.ksg_oracle_whatif.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.ksg_oracle_result.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.POINTER(ctypes.c_int)] * 3
        L.ksg_oracle_digest.restype = ctypes.c_ulonglong
        L.ksg_oracle_digest.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ksg_oracle_nominated.restype = ctypes.c_int
        L.ksg_oracle_nominated.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_size_t)]
        L.ksg_oracle_annotations.restype = ctypes.c_void_p
        L.ksg_oracle_annotations.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]
        L.ksg_oracle_queue_pod.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_size_t)]
        L.ksg_oracle_num_gated.argtypes = [ctypes.c_void_p]
        L.ksg_oracle_go_log.restype = ctypes.c_double
        L.ksg_oracle_go_log.argtypes = [ctypes.c_double]
        L.ksg_oracle_pack_key.restype = ctypes.c_ulonglong
        L.ksg_oracle_pack_key.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int]
        _lib = L
    return _lib


class Oracle:
    def __init__(self, doc):
        s = doc if isinstance(doc, (bytes, str)) else json.dumps(doc)
        b = s.encode() if isinstance(s, str) else s
        err = ctypes.create_string_buffer(512)
        self.h = lib().ksg_oracle_load(b, len(b), err, 512)
        if not self.h:
            raise ValueError(err.value.decode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().ksg_oracle_free(self.h)
            self.h = None

    @property
    def n_queue(self):
        return lib().ksg_oracle_num_queue(self.h)

    def _pod_name(self, q):
        n = ctypes.c_size_t()
        buf = ctypes.create_string_buffer(1024)
        if lib().ksg_oracle_queue_pod(self.h, q, buf, 1024, ctypes.byref(n)) != 0:
            raise IndexError(q)
        return buf.raw[:n.value].decode()

    def queue_names(self):
        """"namespace/name" of every queue pod, in scheduling order (PrioritySort)."""
        return [self._pod_name(q) for q in range(self.n_queue)]

    def gated_names(self):
        """"namespace/name" of the pods SchedulingGates' PreEnqueue keeps out of the queue."""
        return [self._pod_name(-1 - i) for i in range(lib().ksg_oracle_num_gated(self.h))]

    def ordered_queue(self, doc):
        """The document's pending pod objects in the oracle's scheduling order (what the
        framework would run through the drop-in cycle API one by one)."""
        pend = doc["queue"] if "queue" in doc else [p for p in doc["pods"] if not p["spec"].get("nodeName")]
        by = {(p["metadata"].get("namespace") or "default") + "/" + p["metadata"]["name"]: p for p in pend}
        return [by[n] for n in self.queue_names()]

    def schedule(self, n=None, workers=1, record=3):
        n = self.n_queue if n is None else n
        return lib().ksg_oracle_schedule(self.h, n, workers, record)

    def whatif(self, n, workers=1, record=0):
        """What-if step: n pods against one snapshot, placements bound afterwards."""
        return lib().ksg_oracle_whatif(self.h, n, workers, record)

    def result(self, q):
        s, f, st = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        lib().ksg_oracle_result(self.h, q, ctypes.byref(s), ctypes.byref(f), ctypes.byref(st))
        return s.value, f.value, st.value

    def digest(self, q):
        return lib().ksg_oracle_digest(self.h, q)

    def nominated(self, q):
        """DefaultPreemption dry run of queue pod q: (nominated node index or -1, victims)."""
        n = ctypes.c_size_t()
        lib().ksg_oracle_nominated(self.h, q, None, 0, ctypes.byref(n))
        buf = ctypes.create_string_buffer(n.value + 1)
        idx = lib().ksg_oracle_nominated(self.h, q, buf, n.value + 1, ctypes.byref(n))
        return idx, [x for x in buf.raw[:n.value].decode().split("\n") if x]

    def annotations(self, q):
        n = ctypes.c_size_t()
        p = lib().ksg_oracle_annotations(self.h, q, ctypes.byref(n))
        return json.loads(ctypes.string_at(p, n.value).decode()) if n.value else {}


def go_log(x):
    return lib().ksg_oracle_go_log(x)
