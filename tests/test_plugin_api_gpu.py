"""The Go-plugin view of the boundary: every scheduling-result annotation the
simulator's wrapped plugins record, rebuilt from the per-extension-point ABI
calls alone (ksg_prefilter_status / ksg_prefilter_result / ksg_filter_status /
ksg_prescore_status / ksg_scores / ksg_normalized_scores), must equal the
engine's own annotations and the oracle's byte for byte.

This is the recording a wrapped plugin does (simulator/scheduler/plugin/
wrappedplugin.go: PreFilter :491-518 stores Status.Message() or "success" and
the PreFilterResult; Filter :535 "passed" or the message; PreScore :472;
Score :419 the raw score; NormalizeScore :400 the normalized score, which the
result store multiplies by the plugin's weight, resultstore/store.go:504-507)
and the serialisation the store does (encoding/json: sorted keys, no spaces).
"""
import json

import pytest

from _oracle import Oracle
from ksg import Scheduler, generator as g

P = "kube-scheduler-simulator.sigs.k8s.io/"
SCORERS = {"NodeResourcesFit", "NodeResourcesBalancedAllocation", "TaintToleration", "NodeAffinity",
           "PodTopologySpread", "InterPodAffinity", "ImageLocality"}
C_SUCCESS, C_SKIP, C_NOT_RUN = 0, 5, -1

CASES = [
    ("cfg1", 1, dict(n_nodes=60, n_pods=90)),
    ("cfg2", 2, dict(n_nodes=120, n_pods=60)),
    ("cfg3", 3, dict(n_nodes=150, n_pods=60)),
    ("cfg4", 4, dict(n_nodes=120, n_existing=500, n_pods=60, n_zones=5)),
]


def _js(v):
    return json.dumps(v, separators=(",", ":"), sort_keys=True, ensure_ascii=False)


def _store_weight(prof, name):
    sw = prof.get("storeWeights", {})
    if name not in sw:
        return 0
    return 1 if sw[name] == 0 else sw[name]


def rebuild(s, q, prof, names, status):
    plugins = prof["plugins"]
    pre_status, pre_result = {}, {}
    aborted = False
    for pos, name in enumerate(plugins):
        code, msg = s.prefilter_status(q, pos)
        if code == C_NOT_RUN:
            continue
        pre_status[name] = "success" if code == C_SUCCESS else msg
        aborted |= code not in (C_SUCCESS, C_SKIP)
        if name in ("NodeAffinity", "VolumeBinding") and code == C_SUCCESS:
            r = s.prefilter_result_pos(q, pos)
            if r is not None:
                pre_result[name] = r
            if name == "NodeAffinity":
                assert r == s.prefilter_result(q)
    filt, feasible = {}, []
    for i, nm in enumerate(names):
        row = {}
        for pos, name in enumerate(plugins):
            code, msg = s.filter_status(q, pos, i)
            if code != C_NOT_RUN:
                row[name] = "passed" if code == C_SUCCESS else msg
        if row:
            filt[nm] = row
            if all(v == "passed" for v in row.values()):
                feasible.append(i)
    pre_score, score, fin = {}, {}, {}
    if not aborted and len(feasible) > 1 and status != 2:
        skipped = set()
        for pos, name in enumerate(plugins):
            code, _ = s.prescore_status(q, pos)
            if code == C_NOT_RUN:
                continue
            pre_score[name] = "success" if code == C_SUCCESS else ""
            if code == C_SKIP:
                skipped.add(name)
        for pos, name in enumerate(plugins):
            if name not in SCORERS or name in skipped:
                continue
            raw, norm, w = s.scores(q, pos), s.normalized_scores(q, pos), _store_weight(prof, name)
            for i in feasible:
                score.setdefault(names[i], {})[name] = str(raw[i])
                fin.setdefault(names[i], {})[name] = str(norm[i] * w)
    elif aborted:
        filt = {}
    elif len(feasible) > 1 and status == 2:  # a PreScore failed: the statuses up to it
        for pos, name in enumerate(plugins):
            code, msg = s.prescore_status(q, pos)
            if code != C_NOT_RUN:
                pre_score[name] = "success" if code == C_SUCCESS else msg
    post = {}  # PostFilter: DefaultPreemption records every node, the nominated one with its message
    if status == 1 and "DefaultPreemption" in plugins:
        post = {nm: {} for nm in names}
        node, _victims = s.postfilter_result(q)
        if node >= 0:
            post[names[node]] = {"DefaultPreemption": "preemption victim"}
    return {P + "prefilter-result-status": _js(pre_status), P + "prefilter-result": _js(pre_result),
            P + "filter-result": _js(filt), P + "prescore-result": _js(pre_score),
            P + "score-result": _js(score), P + "finalscore-result": _js(fin), P + "postfilter-result": _js(post)}


@pytest.mark.gpu
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
def test_annotations_from_extension_point_calls(name, c, sizes):
    doc = g.generate(c, **sizes)
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    d = dict(doc)
    d["queue"] = []
    s.load_cluster(d)
    names = [n["metadata"]["name"] for n in doc["nodes"]]
    for i, nm in enumerate(names):
        assert s.node_index(nm) == i
    assert s.node_index("no-such-node") is None
    for pos, pl in enumerate(doc["profile"]["plugins"]):
        assert s.plugin_position(pl) == pos
    checked = 0
    for i, pod in enumerate(doc["queue"]):
        q, r = s.cycle(pod, commit=True)
        assert (r.selected, r.feasible, r.status) == o.result(i), (name, i)
        if i % 3:
            continue
        got = rebuild(s, q, doc["profile"], names, r.status)
        eng, ora = s.annotations(q), o.annotations(i)
        for k, v in got.items():
            assert v == eng[k], (name, i, k)
            assert v == ora[k], (name, i, k)
        # Σ normalized × framework weight is the total the selection used
        if r.selected >= 0 and r.feasible > 1:
            tot = 0
            for pos, pl in enumerate(doc["profile"]["plugins"]):
                if pl in SCORERS and s.prescore_status(q, pos)[0] == C_SUCCESS or pl == "ImageLocality":
                    tot += s.normalized_scores(q, pos)[r.selected] * doc["profile"]["weights"][pl]
            assert tot == r.total, (name, i)
        checked += 1
    assert checked >= 20


@pytest.mark.gpu
def test_scheduler_configuration_profile():
    """A KubeSchedulerConfiguration profile (scheduler_test.go:344-407 shape: Score.Enabled
    re-weights MultiPoint plugins): the engine's selections use the framework weights
    (Score wins), the recorded finalscore the store weights (MultiPoint wins,
    plugins.go:289-304) — every pod and every annotation equal to the oracle's, and
    Σ normalized × framework weight is the selected node's total."""
    doc = g.generate(1, n_nodes=60, n_pods=80)
    mp = [(n, 2 if n == "NodeResourcesFit" else (3 if n == "NodeResourcesBalancedAllocation" else w))
          for n, w in g.DEFAULT_PROFILE]
    cfg = g.config_profile(mp, doc["profile"]["seed"], score=[("NodeResourcesFit", 5), ("ImageLocality", 4)])
    doc = dict(doc, profile=cfg)
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(cfg)
    s.load_cluster(doc)
    s.keep_outputs(0, len(doc["queue"]))
    s.schedule()
    fw = {}
    for n, _ in g.DEFAULT_PROFILE:
        pos = s.plugin_position(n)
        assert pos == s.plugin_position(n + "Wrapped")
        fw[n] = s.plugin_weights(pos)
    assert fw["NodeResourcesFit"] == (5, 2) and fw["ImageLocality"] == (4, 1)
    assert fw["NodeResourcesBalancedAllocation"] == (3, 3) and fw["TaintToleration"] == (3, 3)
    for q, r in enumerate(s.results()):
        assert (r.selected, r.feasible, r.status) == o.result(q), q
        assert s.annotations(q) == o.annotations(q), q
        if r.selected >= 0 and r.feasible > 1:
            tot = sum(s.normalized_scores(q, s.plugin_position(n))[r.selected] * fw[n][0]
                      for n in SCORERS if s.prescore_status(q, s.plugin_position(n))[0] == C_SUCCESS
                      or n == "ImageLocality")
            assert tot == r.total, q


class _ViewCalls:
    """rebuild()'s per-node calls answered from a ksg_cycle_view (no library call);
    the once-per-cycle PreFilterResult / PostFilter calls go to the context."""

    def __init__(self, s, v):
        self.s, self.v = s, v

    def prefilter_status(self, q, pos):
        return self.v.prefilter_status(pos)

    def filter_status(self, q, pos, i):
        return self.v.filter_status(pos, i)

    def prescore_status(self, q, pos):
        return self.v.prescore_status(pos)

    def scores(self, q, pos):
        return self.v.scores(pos)

    def normalized_scores(self, q, pos):
        return self.v.normalized_scores(pos)

    def prefilter_result(self, q):
        return self.s.prefilter_result(q)

    def prefilter_result_pos(self, q, pos):
        return self.s.prefilter_result_pos(q, pos)

    def postfilter_result(self, q):
        return self.s.postfilter_result(q)


@pytest.mark.gpu
@pytest.mark.parametrize("copy", ["0", "1", "r"], ids=["direct", "copy", "reserve"])
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
def test_cycle_view_matches_extension_point_calls(monkeypatch, name, c, sizes, copy):
    """ksg_cycle_view (include/ksg.h): the arrays the framework's 16 parallel
    Filter / Score workers index instead of calling the library per node.  Every
    annotation rebuilt from a view equals the oracle's; 16 threads rebuilding from
    one view agree; a view is unchanged by the cycles that follow it.  Per-node
    arrays written by the view kernel into the pinned block, or copied after it
    (KSG_VIEW_COPY=1).  "reserve": the drop-in's own order -- a cycle without the
    assume, its view, then Reserve on the node the framework picked -- where a
    profile without ScoreExtensions (cfg2) has the cycle's k_eval write the view
    itself (the fused view, no k_view launch)."""
    from concurrent.futures import ThreadPoolExecutor
    monkeypatch.setenv("KSG_VIEW_COPY", "1" if copy == "1" else "0")
    doc = g.generate(c, **sizes)
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    d = dict(doc)
    d["queue"] = []
    s.load_cluster(d)
    names = [n["metadata"]["name"] for n in doc["nodes"]]
    held = []
    widths = set()  # PodTopologySpread / InterPodAffinity raw rows: as narrow as the cycle's range
    plugins = doc["profile"]["plugins"]
    for i, pod in enumerate(doc["queue"][:30]):
        q, r = s.cycle(pod, commit=copy != "r")
        v = s.cycle_view(q)
        for pos, pl in enumerate(plugins):
            if pl in ("PodTopologySpread", "InterPodAffinity") and v._v.score[pos] and r.status == 0:
                widths.add(v._v.score_bytes[pos])
        assert (v.result.selected, v.result.feasible, v.result.status) == o.result(i), (name, i)
        nodes = range(len(names)) if i < 8 else (0, len(names) // 2, len(names) - 1)
        for pos in range(len(doc["profile"]["plugins"])):  # the view holds what the per-node calls return
            for k in nodes:
                assert v.filter_status(pos, k) == tuple(s.filter_status(q, pos, k)), (name, i, pos, k)
            if i < 8 and r.feasible > 1 and v._v.score[pos]:  # raw / normalized on every feasible node
                raw, norm = s.scores(q, pos), s.normalized_scores(q, pos)
                vr, vn = v.scores(pos), v.normalized_scores(pos)
                for k in range(len(names)):
                    if v._v.fail_pos[k] == len(doc["profile"]["plugins"]):
                        assert (vr[k], vn[k]) == (raw[k], norm[k]), (name, i, pos, k)
        vc = _ViewCalls(s, v)
        with ThreadPoolExecutor(16) as ex:
            outs = list(ex.map(lambda _: rebuild(vc, q, doc["profile"], names, r.status), range(16)))
        ora = o.annotations(i)
        for got in outs:
            for k, val in got.items():
                assert val == ora[k], (name, i, k)
        if i % 10 == 0:
            held.append((i, q, v, outs[0]))
        if copy == "r" and r.selected >= 0:
            s.reserve(q, r.selected)
    assert widths <= {1, 2, 4}, widths
    if name == "cfg4":
        assert widths and min(widths) < 4, widths
    if copy == "r" and name == "cfg2":  # no ScoreExtensions: the cycle's k_eval wrote the view
        assert s.views_fused() > 0
    for i, q, v, first in held:  # views stay valid and unchanged after later cycles
        assert rebuild(_ViewCalls(s, v), q, doc["profile"], names, v.result.status) == first, (name, i)
        v.release()
