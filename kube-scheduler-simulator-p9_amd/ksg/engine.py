"""ctypes binding of libksg.so (include/ksg.h).  No fallback path."""
from __future__ import annotations

import ctypes
import json
import os
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
_lib = None

FILTER_PASSED = 0xFFFFFFFF
FILTER_NOT_EVALUATED = 0xFFFFFFFE


def lib_path() -> str:
    # KSG_LIB: diagnostic override (A/B builds of the same sources)
    return os.environ.get("KSG_LIB") or os.path.join(_PKG, "libksg.so")


class _PodResult(ctypes.Structure):
    _fields_ = [("selected", ctypes.c_int32), ("feasible", ctypes.c_int32), ("status", ctypes.c_int32),
                ("skip_filter", ctypes.c_uint32), ("skip_score", ctypes.c_uint32), ("total", ctypes.c_int32)]


class _Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("stream", ctypes.c_void_p), ("shard_rank", ctypes.c_uint32),
                ("shard_count", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class _CycleView(ctypes.Structure):
    _fields_ = [("q", ctypes.c_uint32), ("n_positions", ctypes.c_uint32), ("node_offset", ctypes.c_uint32),
                ("n_nodes", ctypes.c_uint32), ("result", _PodResult),
                ("filter_called", ctypes.POINTER(ctypes.c_uint8)),
                ("fail_pos", ctypes.POINTER(ctypes.c_int8)), ("fail_code", ctypes.POINTER(ctypes.c_int8)),
                ("fail_msg", ctypes.POINTER(ctypes.c_uint16)),
                ("score", ctypes.POINTER(ctypes.c_void_p)), ("normalized", ctypes.POINTER(ctypes.c_void_p)),
                ("score_bytes", ctypes.POINTER(ctypes.c_uint8)), ("normalized_bytes", ctypes.POINTER(ctypes.c_uint8)),
                ("prefilter_code", ctypes.POINTER(ctypes.c_int8)), ("prefilter_msg", ctypes.POINTER(ctypes.c_uint16)),
                ("prescore_code", ctypes.POINTER(ctypes.c_int8)), ("prescore_msg", ctypes.POINTER(ctypes.c_uint16)),
                ("messages", ctypes.POINTER(ctypes.c_char_p)), ("n_messages", ctypes.c_uint32),
                ("owner", ctypes.c_void_p)]


class CycleView:
    """ksg_cycle_view: one cycle's per-node results as immutable arrays, read
    without calling into the library (what the framework's parallel Filter / Score
    workers do); released with release() or when garbage-collected."""

    def __init__(self, L, ptr):
        self._L, self._p = L, ptr
        v = ptr.contents
        self.q, self.P, self.N, self.node_offset = v.q, v.n_positions, v.n_nodes, v.node_offset
        r = v.result
        self.result = PodResult(r.selected, r.feasible, r.status, r.total)
        self._v = v
        self._msgs = None  # (decoded on first use: most of the slots are empty)

    @property
    def messages(self):
        if self._msgs is None:
            v = self._v
            self._msgs = [v.messages[i].decode() for i in range(v.n_messages)]
        return self._msgs

    def message(self, k):
        return self._v.messages[k].decode() if self._msgs is None else self._msgs[k]

    def release(self):
        if self._p:
            self._L.ksg_cycle_view_release(self._p)
            self._p = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass

    def filter_status(self, pos, i):
        """What Filter of profile position pos returns on local node i (ksg.h rule)."""
        v = self._v
        if not v.filter_called[pos]:
            return -1, ""
        fp = v.fail_pos[i]
        if fp < 0 or pos > fp:
            return -1, ""
        if pos < fp:
            return 0, ""
        return v.fail_code[i], self.message(v.fail_msg[i])

    def prefilter_status(self, pos):
        return self._v.prefilter_code[pos], self.message(self._v.prefilter_msg[pos])

    def prescore_status(self, pos):
        return self._v.prescore_code[pos], self.message(self._v.prescore_msg[pos])

    _WIDTH = {1: ctypes.c_int8, 2: ctypes.c_int16, 4: ctypes.c_int32}

    def _row(self, p, w):
        if not p:
            return [0] * self.N
        return list(ctypes.cast(p, ctypes.POINTER(self._WIDTH[w] * self.N)).contents)

    def scores(self, pos):
        """Raw scores of position pos (ksg_view_score: rows as narrow as their values)."""
        return self._row(self._v.score[pos], self._v.score_bytes[pos])

    def normalized_scores(self, pos):
        return self._row(self._v.normalized[pos], self._v.normalized_bytes[pos])


@dataclass
class PodResult:
    selected: int
    feasible: int
    status: int
    total: int


def load_library():
    """Load libksg.so; raises OSError when the HIP build is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    p = lib_path()
    if not os.path.exists(p):
        raise OSError(f"libksg.so not built at {p}: run __graft_entry__.build() (hipcc gfx950)")
    L = ctypes.CDLL(p)
    vp, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int32
    L.ksg_create.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(_Opts), ctypes.POINTER(vp)]
    L.ksg_destroy.argtypes = [vp]
    L.ksg_last_error.restype = ctypes.c_char_p
    L.ksg_last_error.argtypes = [vp]
    L.ksg_load_cluster.argtypes = [vp, ctypes.c_char_p, sz]
    L.ksg_num_nodes.argtypes = [vp]
    L.ksg_queue_len.argtypes = [vp]
    L.ksg_schedule_queue.argtypes = [vp, u32, u32]
    L.ksg_wait.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    L.ksg_pod_results.argtypes = [vp, u32, u32, ctypes.POINTER(_PodResult)]
    L.ksg_keep_outputs.argtypes = [vp, u32, u32]
    L.ksg_filter_codes.argtypes = [vp, u32, ctypes.POINTER(u32), u32]
    L.ksg_scores.argtypes = [vp, u32, u32, ctypes.POINTER(i32), u32]
    L.ksg_annotations.argtypes = [vp, u32, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.ksg_reset.argtypes = [vp]
    L.ksg_sample_kernel.argtypes = [vp, u32]
    L.ksg_nccl_unique_id.argtypes = [ctypes.c_void_p]
    L.ksg_set_exchange.argtypes = [vp, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.ksg_set_path.argtypes = [vp, ctypes.c_int]
    L.ksg_batch_path.argtypes = [vp]
    L.ksg_kernel_time.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(u32)]
    L.ksg_node_requested.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(i32), u32, u32]
    L.ksg_whatif.argtypes = [vp, u32, u32]
    L.ksg_cycle.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_int, ctypes.c_void_p]
    L.ksg_reserve.argtypes = [vp, u32, i32]
    L.ksg_unreserve.argtypes = [vp, u32]
    L.ksg_apply_events.argtypes = [vp, ctypes.c_char_p, sz]
    i64 = ctypes.c_int64
    L.ksg_node_nonzero.argtypes = [vp, ctypes.POINTER(i64), u32]
    cp = ctypes.c_char_p
    L.ksg_plugin_position.argtypes = [vp, cp, sz]
    L.ksg_node_index.argtypes = [vp, cp, sz]
    L.ksg_plugin_weights.argtypes = [vp, u32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.ksg_compact.argtypes = [vp, u32]
    L.ksg_prefilter_status.argtypes = [vp, u32, u32, ctypes.POINTER(i32), cp, sz, ctypes.POINTER(sz)]
    L.ksg_prefilter_result.argtypes = [vp, u32, cp, sz, ctypes.POINTER(sz)]
    L.ksg_prefilter_result_pos.argtypes = [vp, u32, u32, cp, sz, ctypes.POINTER(sz)]
    L.ksg_postfilter_result.argtypes = [vp, u32, ctypes.POINTER(ctypes.c_int32), cp, sz, ctypes.POINTER(sz)]
    L.ksg_filter_status.argtypes = [vp, u32, u32, u32, ctypes.POINTER(i32), cp, sz, ctypes.POINTER(sz)]
    L.ksg_prescore_status.argtypes = [vp, u32, u32, ctypes.POINTER(i32), cp, sz, ctypes.POINTER(sz)]
    L.ksg_normalized_scores.argtypes = [vp, u32, u32, ctypes.POINTER(i64), u32]
    L.ksg_cycle_view_acquire.argtypes = [vp, u32, ctypes.POINTER(ctypes.POINTER(_CycleView))]
    L.ksg_cycle_view_release.argtypes = [ctypes.POINTER(_CycleView)]
    L.ksg_cycle_view_release.restype = None
    L.ksg_debug_path_counts.argtypes = [vp, ctypes.c_void_p]
    L.ksg_queue_pod.argtypes = [vp, u32, cp, sz, ctypes.POINTER(sz)]
    L.ksg_gated_pods.argtypes = [vp, cp, sz, ctypes.POINTER(sz)]
    L.ksg_synth_cluster.argtypes = [ctypes.c_int, i64, i64, i64, i64, ctypes.c_uint64, ctypes.POINTER(vp),
                                    ctypes.POINTER(sz)]
    L.ksg_free.argtypes = [vp]
    _lib = L
    return L


class KsgError(RuntimeError):
    pass


class Scheduler:
    """One engine context (one profile, one GPU, optionally one node shard)."""

    def __init__(self, profile: dict, device: int = 0, stream: int | None = None, shard_rank=0, shard_count=1):
        self.L = load_library()
        self.h = ctypes.c_void_p()
        prof = json.dumps(profile).encode()
        opts = _Opts(device, stream, shard_rank, shard_count, 0)
        rc = self.L.ksg_create(prof, len(prof), ctypes.byref(opts), ctypes.byref(self.h))
        if rc != 0:
            raise KsgError(f"ksg_create failed ({rc})")

    def _chk(self, rc, what):
        if rc != 0:
            raise KsgError(f"{what}: {rc} {self.L.ksg_last_error(self.h).decode()}")

    def close(self):
        if self.h:
            self.L.ksg_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_cluster(self, doc):
        s = doc if isinstance(doc, (bytes, str)) else json.dumps(doc)
        b = s.encode() if isinstance(s, str) else s
        self._chk(self.L.ksg_load_cluster(self.h, b, len(b)), "ksg_load_cluster")

    @property
    def n_nodes(self):
        return self.L.ksg_num_nodes(self.h)

    @property
    def queue_len(self):
        return self.L.ksg_queue_len(self.h)

    def queue_pod(self, q):
        """"namespace/name" of queue pod q (the queue is in scheduling order: PrioritySort)."""
        n = ctypes.c_size_t()
        buf = ctypes.create_string_buffer(1024)
        self._chk(self.L.ksg_queue_pod(self.h, q, buf, 1024, ctypes.byref(n)), "ksg_queue_pod")
        return buf.raw[:n.value].decode()

    def gated_pods(self):
        """Pods SchedulingGates' PreEnqueue keeps out of the queue ("namespace/name")."""
        n = ctypes.c_size_t()
        self.L.ksg_gated_pods(self.h, None, 0, ctypes.byref(n))
        buf = ctypes.create_string_buffer(n.value + 1)
        self._chk(self.L.ksg_gated_pods(self.h, buf, n.value + 1, ctypes.byref(n)), "ksg_gated_pods")
        return [x for x in buf.raw[:n.value].decode().split("\n") if x]

    def keep_outputs(self, first, count):
        self._chk(self.L.ksg_keep_outputs(self.h, first, count), "ksg_keep_outputs")

    def schedule(self, first=0, count=None, wait=True):
        count = self.queue_len - first if count is None else count
        self._chk(self.L.ksg_schedule_queue(self.h, first, count), "ksg_schedule_queue")
        return self.wait() if wait else None

    def whatif(self, first=0, count=None, wait=True):
        """What-if step: pods [first, first+count) against one snapshot, then bound."""
        count = self.queue_len - first if count is None else count
        self._chk(self.L.ksg_whatif(self.h, first, count), "ksg_whatif")
        return self.wait() if wait else None

    def wait(self):
        ms = ctypes.c_float()
        self._chk(self.L.ksg_wait(self.h, ctypes.byref(ms)), "ksg_wait")
        return ms.value

    def results(self, first=0, count=None):
        count = self.queue_len - first if count is None else count
        arr = (_PodResult * max(count, 1))()
        self._chk(self.L.ksg_pod_results(self.h, first, count, arr), "ksg_pod_results")
        return [PodResult(a.selected, a.feasible, a.status, a.total) for a in arr[:count]]

    def filter_codes(self, q):
        n = self.n_nodes
        arr = (ctypes.c_uint32 * n)()
        self._chk(self.L.ksg_filter_codes(self.h, q, arr, n), "ksg_filter_codes")
        return list(arr)

    def scores(self, q, pos):
        n = self.n_nodes
        arr = (ctypes.c_int32 * n)()
        self._chk(self.L.ksg_scores(self.h, q, pos, arr, n), "ksg_scores")
        return list(arr)

    def annotations(self, q) -> dict:
        n = ctypes.c_size_t()
        self.L.ksg_annotations(self.h, q, None, 0, ctypes.byref(n))
        buf = ctypes.create_string_buffer(n.value + 1)
        self._chk(self.L.ksg_annotations(self.h, q, buf, n.value + 1, ctypes.byref(n)), "ksg_annotations")
        return json.loads(buf.raw[:n.value].decode())

    def reset(self):
        self._chk(self.L.ksg_reset(self.h), "ksg_reset")

    def cycle(self, pod, commit=True):
        """One drop-in scheduling cycle for a new pod (v1.Pod dict); returns
        (queue index, PodResult).  commit=False leaves the assume to reserve()."""
        b = (pod if isinstance(pod, (bytes, str)) else json.dumps(pod))
        b = b.encode() if isinstance(b, str) else b
        r = _PodResult()
        self._chk(self.L.ksg_cycle(self.h, b, len(b), 1 if commit else 0, ctypes.byref(r)), "ksg_cycle")
        return self.queue_len - 1, PodResult(r.selected, r.feasible, r.status, r.total)

    def reserve(self, q, node):
        self._chk(self.L.ksg_reserve(self.h, q, node), "ksg_reserve")

    def unreserve(self, q):
        self._chk(self.L.ksg_unreserve(self.h, q), "ksg_unreserve")

    def apply_events(self, events, reencode=False):
        """Scheduler-cache events (addNode/updateNode/removeNode/addPod/updatePod/
        removePod dicts, see ksg.h) applied as one all-or-nothing batch;
        reencode=True skips the in-place path for bound-pod batches."""
        b = json.dumps({"events": list(events), "reencode": bool(reencode)}).encode()
        self._chk(self.L.ksg_apply_events(self.h, b, len(b)), "ksg_apply_events")

    def sample_kernel(self, every):
        self._chk(self.L.ksg_sample_kernel(self.h, every), "ksg_sample_kernel")

    def set_exchange_rccl(self, unique_id: bytes):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        self._chk(self.L.ksg_set_exchange(self.h, 1, buf, None, None), "ksg_set_exchange")

    def set_exchange_host(self, world: int):
        from .distributed import make_host_exchange
        self._xfn = make_host_exchange(world)  # keep alive
        self._chk(self.L.ksg_set_exchange(self.h, 2, None, ctypes.cast(self._xfn, ctypes.c_void_p), None),
                  "ksg_set_exchange")

    def cycle_view(self, q) -> CycleView:
        """ksg_cycle_view_acquire: the kept outputs of queue pod q as a read-only view."""
        p = ctypes.POINTER(_CycleView)()
        self._chk(self.L.ksg_cycle_view_acquire(self.h, q, ctypes.byref(p)), "ksg_cycle_view_acquire")
        return CycleView(self.L, p)

    def path_counts(self, solo=False):
        """Diagnostic: (pods through the table chain, pods through the scanning chain) so far
        (+ of the first, the one-launch cycles when solo)."""
        out = (ctypes.c_uint64 * 8)()
        self._chk(self.L.ksg_debug_path_counts(self.h, out), "ksg_debug_path_counts")
        return (out[0], out[1], out[2]) if solo else (out[0], out[1])

    def whatif_class_chunks(self):
        """Diagnostic: what-if pod chunks that ran the class path (k_whatif_cls1/2)."""
        out = (ctypes.c_uint64 * 8)()
        self._chk(self.L.ksg_debug_path_counts(self.h, out), "ksg_debug_path_counts")
        return out[3]

    def run_counts(self):
        """Diagnostic: (table-chain pods of persistent segments, segments) so far (k_chain_run)."""
        out = (ctypes.c_uint64 * 8)()
        self._chk(self.L.ksg_debug_path_counts(self.h, out), "ksg_debug_path_counts")
        return out[4], out[5]

    def views_fused(self):
        """Diagnostic: cycle views written by the cycle's k_eval itself (no k_view launch)."""
        out = ctypes.c_uint64()
        self.L.ksg_debug_views_fused.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self._chk(self.L.ksg_debug_views_fused(self.h, ctypes.byref(out)), "ksg_debug_views_fused")
        return out.value

    def run_fallbacks(self):
        """Diagnostic: persistent segments whose blocks were not all resident and ran on
        the two-launch chain instead."""
        out = (ctypes.c_uint64 * 8)()
        self._chk(self.L.ksg_debug_path_counts(self.h, out), "ksg_debug_path_counts")
        return out[6]

    def set_path(self, per_pod: bool):
        self._chk(self.L.ksg_set_path(self.h, 1 if per_pod else 0), "ksg_set_path")

    @property
    def batch_path(self) -> bool:
        return self.L.ksg_batch_path(self.h) == 1

    def static_dec_chunks(self):
        """Diagnostic: static-record chunks computed from decoded pods (k_static_dec)."""
        out = ctypes.c_uint64()
        self.L.ksg_debug_static_dec_chunks.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self._chk(self.L.ksg_debug_static_dec_chunks(self.h, ctypes.byref(out)), "ksg_debug_static_dec_chunks")
        return out.value

    def static_overlaps(self):
        """Diagnostic: persistent window runs whose static records k_static_dec
        computed beside the loop (KSG_STATIC_OVERLAP)."""
        out = ctypes.c_uint64()
        self.L.ksg_debug_static_overlaps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self._chk(self.L.ksg_debug_static_overlaps(self.h, ctypes.byref(out)), "ksg_debug_static_overlaps")
        return out.value

    def static_time(self):
        """Diagnostic: (total ms, launches, pods) of the sampled run's k_static launches."""
        ms, n, pods = ctypes.c_float(), ctypes.c_uint32(), ctypes.c_uint64()
        self.L.ksg_debug_static_time.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        self._chk(self.L.ksg_debug_static_time(self.h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(pods)),
                  "ksg_debug_static_time")
        return ms.value, n.value, pods.value

    def preempt_batched(self):
        """Diagnostic: DefaultPreemption dry runs that took the batched victim search."""
        out = ctypes.c_uint64()
        self.L.ksg_debug_preempt_batched.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self._chk(self.L.ksg_debug_preempt_batched(self.h, ctypes.byref(out)), "ksg_debug_preempt_batched")
        return out.value

    def window_runs(self):
        """Diagnostic: persistent window launches (k_window_run) so far."""
        out = (ctypes.c_uint64 * 8)()
        self._chk(self.L.ksg_debug_path_counts(self.h, out), "ksg_debug_path_counts")
        return out[7]

    def kernel_time(self):
        ms, n = ctypes.c_float(), ctypes.c_uint32()
        self._chk(self.L.ksg_kernel_time(self.h, ctypes.byref(ms), ctypes.byref(n)), "ksg_kernel_time")
        return ms.value, n.value

    def node_requested(self, n_res=8):
        n = self.n_nodes
        req = (ctypes.c_int64 * (n_res * n))()
        pc = (ctypes.c_int32 * n)()
        self._chk(self.L.ksg_node_requested(self.h, req, pc, n_res, n), "ksg_node_requested")
        return [list(req[r * n:(r + 1) * n]) for r in range(n_res)], list(pc)

    # ---- the Go plugin's per-extension-point calls (ksg.h)
    def plugin_position(self, name):
        b = name.encode()
        r = self.L.ksg_plugin_position(self.h, b, len(b))
        return None if r < 0 else r

    def compact(self, keep_from=None):
        """Drop queue pods [0, keep_from) (placed ones become bound pods); the rest are re-indexed from 0."""
        self._chk(self.L.ksg_compact(self.h, self.queue_len if keep_from is None else keep_from), "ksg_compact")

    def plugin_weights(self, pos):
        """(framework weight, store weight) the profile resolved for position pos."""
        w, sw = ctypes.c_int64(), ctypes.c_int64()
        self._chk(self.L.ksg_plugin_weights(self.h, pos, ctypes.byref(w), ctypes.byref(sw)), "plugin_weights")
        return w.value, sw.value

    def node_index(self, name):
        b = name.encode()
        r = self.L.ksg_node_index(self.h, b, len(b))
        return None if r < 0 else r

    def _status(self, fn, *args):
        code, n = ctypes.c_int32(), ctypes.c_size_t()
        buf = ctypes.create_string_buffer(4096)
        self._chk(fn(self.h, *args, ctypes.byref(code), buf, 4096, ctypes.byref(n)), fn.__name__)
        return code.value, buf.raw[:n.value].decode()

    def prefilter_status(self, q, pos):
        """(framework.Code, message) of PreFilter at profile position pos; code -1: not run."""
        return self._status(self.L.ksg_prefilter_status, q, pos)

    def prefilter_result(self, q):
        n = ctypes.c_size_t()
        self.L.ksg_prefilter_result(self.h, q, None, 0, ctypes.byref(n))
        buf = ctypes.create_string_buffer(n.value + 1)
        self._chk(self.L.ksg_prefilter_result(self.h, q, buf, n.value + 1, ctypes.byref(n)), "ksg_prefilter_result")
        return json.loads(buf.raw[:n.value].decode())

    def prefilter_result_pos(self, q, pos):
        """PreFilterResult of the plugin at profile position pos (None: every node)."""
        n = ctypes.c_size_t()
        self.L.ksg_prefilter_result_pos(self.h, q, pos, None, 0, ctypes.byref(n))
        buf = ctypes.create_string_buffer(n.value + 1)
        self._chk(self.L.ksg_prefilter_result_pos(self.h, q, pos, buf, n.value + 1, ctypes.byref(n)),
                  "ksg_prefilter_result_pos")
        return json.loads(buf.raw[:n.value].decode())

    def postfilter_result(self, q):
        """DefaultPreemption dry run of pod q: (nominated global node index or -1, ["ns/name", ...] victims)."""
        n, node = ctypes.c_size_t(), ctypes.c_int32()
        self.L.ksg_postfilter_result(self.h, q, ctypes.byref(node), None, 0, ctypes.byref(n))
        buf = ctypes.create_string_buffer(n.value + 1)
        self._chk(self.L.ksg_postfilter_result(self.h, q, ctypes.byref(node), buf, n.value + 1, ctypes.byref(n)),
                  "ksg_postfilter_result")
        return node.value, [x for x in buf.raw[:n.value].decode().split("\n") if x]

    def filter_status(self, q, pos, node):
        """(framework.Code, Status.Message()) of Filter on a node; code -1: not called."""
        return self._status(self.L.ksg_filter_status, q, pos, node)

    def prescore_status(self, q, pos):
        """(framework.Code, message) of PreScore at profile position pos; code -1: not run."""
        return self._status(self.L.ksg_prescore_status, q, pos)

    def normalized_scores(self, q, pos):
        n = self.n_nodes
        arr = (ctypes.c_int64 * n)()
        self._chk(self.L.ksg_normalized_scores(self.h, q, pos, arr, n), "ksg_normalized_scores")
        return list(arr)

    def node_nonzero(self):
        """NonZeroRequested (cpu milli, memory bytes) rows of every local node."""
        n = self.n_nodes
        nz = (ctypes.c_int64 * (2 * n))()
        self._chk(self.L.ksg_node_nonzero(self.h, nz, n), "ksg_node_nonzero")
        return list(nz[:n]), list(nz[n:])
