"""Edge-case cluster family: the plugin arguments and pod / node shapes the five
BASELINE configs never produce, so that the device path and the oracle meet on
them (VERDICT r1 parity holes; SURVEY.md §4 test strategy).

Variants (each a small seeded cluster, same document shape as ``generator``):

* ``fit_most``  NodeResourcesFit MostAllocated over cpu / memory /
  ephemeral-storage / a scalar resource with unequal weights, BalancedAllocation
  over four resources; init containers (restartPolicy Always sidecars and plain
  ones), pod overhead, requests of ephemeral-storage and the scalar, empty
  requests (the non-zero defaults), pods in several namespaces.
* ``fit_rtc``   the same cluster shape under RequestedToCapacityRatio (a
  three-point shape) over cpu / memory / the scalar.
* ``na``        TaintToleration + NodeAffinity + Fit + BA: nodeSelector,
  required terms with In / NotIn / Exists / DoesNotExist / Gt / Lt (numeric and
  non-numeric values), matchFields metadata.name In / NotIn, preferred terms,
  tolerations with Exists / Equal / empty keys / empty effects, PreferNoSchedule
  and NoExecute taints, nodes without the labels.
* ``pts``       Fit + PodTopologySpread + BA: minDomains, nodeAffinityPolicy
  Honor / Ignore, nodeTaintsPolicy Honor / Ignore, matchLabelKeys, several
  DoNotSchedule / ScheduleAnyway constraints, nodes without the zone label,
  terminating bound pods, namespaces.
* ``ipa``       Fit + InterPodAffinity + BA with hardPodAffinityWeight 3:
  namespaces lists, namespaceSelector {} (every namespace) and a selector no
  namespace matches, matchExpressions, required / preferred terms on bound pods
  in several namespaces.
* ``ipa_ignore`` the ``ipa`` cluster with ignorePreferredTermsOfExistingPods and
  hardPodAffinityWeight 0.
* ``preempt``   DefaultPreemption: a nearly full cluster of bound pods at mixed
  priorities (status.startTime set on most of them), queue pods at mixed
  priorities (some preemptionPolicy Never), host ports, pod-count limits,
  spread constraints, required anti-affinity, taints and node selectors, so that
  unschedulable pods meet both Unschedulable nodes (preemption may help) and
  UnschedulableAndUnresolvable ones.  The queue pops in PrioritySort order;
  with ``queue_sort=False`` (document key ``"queueSort": false``: pods arriving
  one at a time) it keeps document order, so earlier queue pods can be victims
  of later ones.
* ``volumes``   the whole default profile over pods with PersistentVolumeClaims
  (ResourcesForSnap pvs / pvcs / storageClasses): claims bound to local PVs
  (hostname node affinity: VolumeBinding's PreFilterResult), to zonal PVs
  (VolumeZone labels, multi-zone "__" values, a malformed one; node affinity by
  zone), to a PV with an empty or a matchFields-only affinity, to a missing PV;
  WaitForFirstConsumer claims to provision (allowedTopologies, a selected-node
  annotation, a class without a provisioner), immediate and pre-bound unbound
  claims, deleting / lost / missing claims, ReadWriteOncePod claims used by a
  bound pod or shared by two queue pods; nodes with and without zone / region
  labels; CSI attach limits from CSINode counts or the legacy allocatable key.
* ``queue``     queue entry of the default profile, as a ResourcesForSnap
  document (pending pods mixed into "pods", no "queue" key): pods carrying
  spec.schedulingGates (SchedulingGates' PreEnqueue keeps them out: never
  scheduled, no annotations), pending pods at mixed priorities (PrioritySort:
  higher priority first, then document order) on a nearly full cluster, so
  that the order decides placements and DefaultPreemption nominations.
"""
from __future__ import annotations

import json

from .generator import (HOSTNAME, ZONE, Gi, Mi, Rng, make_profile, node_obj, pod_obj, req)

GPU = "example.com/gpu"
EPH = "ephemeral-storage"
NAMESPACES = ["default", "ns-a", "ns-b", "team-x"]
EDGE_VARIANTS = ("fit_most", "fit_rtc", "na", "pts", "ipa", "ipa_ignore", "preempt", "volumes", "queue")


def edge_seed(variant: str) -> int:
    return 20250131 * 100 + 50 + EDGE_VARIANTS.index(variant)


def _containers(r, scalar=True):
    cs = []
    for _ in range(1 + r.below(2)):
        p = r.pct()
        if p < 12:
            cs.append({})  # no requests: the non-zero defaults (scoring) and zero (filter)
            continue
        extra = {}
        if r.pct() < 40:
            extra[EPH] = f"{1 + r.below(20)}Gi"
        if scalar and r.pct() < 25:
            extra[GPU] = str(1 + r.below(2))
        cs.append(req(100 * (1 + r.below(20)), 128 * Mi * (1 + r.below(24)), extra))
    return cs


def _init_containers(r):
    out = []
    for i in range(r.below(3)):
        c = {"name": f"init{i}", "image": "registry.k8s.io/pause:3.5",
             "resources": req(100 * (1 + r.below(30)), 64 * Mi * (1 + r.below(40)))}
        if r.pct() < 50:
            c["restartPolicy"] = "Always"  # a sidecar: its requests add to the containers'
        out.append(c)
    return out


def _fit_cluster(r, n_nodes, n_pods):
    nodes = []
    for i in range(n_nodes):
        scal = {GPU: r.pick([0, 0, 2, 4, 8])} if r.pct() < 70 else {}
        nodes.append(node_obj(f"node-{i:07d}", 1000 * r.pick([4, 8, 16, 32]), Gi * r.pick([16, 32, 64, 128]),
                              pods=r.pick([8, 16, 110]), eph=Gi * r.pick([50, 100, 400]) if r.pct() < 85 else None,
                              scalars=scal))
    queue = []
    for j in range(n_pods):
        spec = {}
        ic = _init_containers(r)
        if ic:
            spec["initContainers"] = ic
        if r.pct() < 30:
            spec["overhead"] = {"cpu": f"{50 * (1 + r.below(4))}m", "memory": f"{32 * (1 + r.below(4))}Mi"}
        queue.append(pod_obj(f"pod-{j:07d}", _containers(r), ns=r.pick(NAMESPACES), **spec))
    return nodes, queue


def gen_fit(variant, n_nodes=60, n_pods=160, seed=None):
    seed = edge_seed(variant) if seed is None else seed
    r = Rng(seed)
    nodes, queue = _fit_cluster(r, n_nodes, n_pods)
    prof = make_profile([("NodeResourcesFit", 1), ("NodeResourcesBalancedAllocation", 1)], seed)
    pc = prof["pluginConfig"]
    if variant == "fit_most":
        pc["NodeResourcesFit"] = {"scoringStrategy": {"type": "MostAllocated", "resources": [
            {"name": "cpu", "weight": 1}, {"name": "memory", "weight": 2}, {"name": EPH, "weight": 1},
            {"name": GPU, "weight": 3}]}}
    else:
        pc["NodeResourcesFit"] = {"scoringStrategy": {"type": "RequestedToCapacityRatio", "resources": [
            {"name": "cpu", "weight": 2}, {"name": "memory", "weight": 1}, {"name": GPU, "weight": 1}],
            "requestedToCapacityRatio": {"shape": [{"utilization": 0, "score": 0}, {"utilization": 40, "score": 8},
                                                   {"utilization": 100, "score": 3}]}}}
    pc["NodeResourcesBalancedAllocation"] = {"resources": [
        {"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1}, {"name": EPH, "weight": 1},
        {"name": GPU, "weight": 1}]}
    return {"profile": prof, "nodes": nodes, "pods": [], "queue": queue}


NA_TAINTS = [{"key": "dedicated", "value": "infra", "effect": "NoSchedule"},
             {"key": "dedicated", "value": "gpu", "effect": "NoExecute"},
             {"key": "spot", "value": "", "effect": "PreferNoSchedule"},
             {"key": "maint", "value": "soon", "effect": "PreferNoSchedule"},
             {"key": "flaky", "value": "yes", "effect": "NoSchedule"}]


def _na_expr(r, n_nodes):
    k = r.below(8)
    if k == 0:
        return {"key": "disk", "operator": "In", "values": sorted({r.pick(["ssd", "hdd", "nvme"]) for _ in range(2)})}
    if k == 1:
        return {"key": "disk", "operator": "NotIn", "values": [r.pick(["ssd", "hdd"])]}
    if k == 2:
        return {"key": "gpu-model", "operator": "Exists"}
    if k == 3:
        return {"key": "gpu-model", "operator": "DoesNotExist"}
    if k == 4:
        return {"key": "gen", "operator": "Gt", "values": [str(r.below(6))]}
    if k == 5:
        return {"key": "gen", "operator": "Lt", "values": [str(2 + r.below(7))]}
    if k == 6:
        return {"key": ZONE, "operator": "In", "values": [f"zone-{r.below(4)}"]}
    return {"key": "disk", "operator": "Exists"}


def _na_fields(r, n_nodes):
    names = sorted({f"node-{r.below(n_nodes):07d}" for _ in range(1 + r.below(6))})
    return {"key": "metadata.name", "operator": r.pick(["In", "In", "NotIn"]), "values": names}


def gen_na(n_nodes=80, n_pods=160, seed=None):
    seed = edge_seed("na") if seed is None else seed
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        labels = {}
        if r.pct() < 85:
            labels[ZONE] = f"zone-{r.below(4)}"
        if r.pct() < 70:
            labels["disk"] = r.pick(["ssd", "hdd", "nvme"])
        if r.pct() < 30:
            labels["gpu-model"] = r.pick(["a", "b"])
        if r.pct() < 80:
            labels["gen"] = r.pick([str(g) for g in range(1, 9)] + ["x9"])  # "x9": not an integer (Gt/Lt fail)
        taints = []
        for t in NA_TAINTS:
            if r.pct() < 15:
                taints.append(dict(t))
        nodes.append(node_obj(f"node-{i:07d}", 1000 * r.pick([4, 8, 16]), Gi * r.pick([16, 32, 64]), labels=labels,
                              taints=taints))
    queue = []
    for j in range(n_pods):
        spec = {}
        tols = []
        for _ in range(r.below(4)):
            t = r.pick(NA_TAINTS)
            k = r.below(5)
            if k == 0:
                tols.append({"operator": "Exists"})  # empty key + Exists: every taint
            elif k == 1:
                tols.append({"key": t["key"], "operator": "Exists"})
            elif k == 2:
                tols.append({"key": t["key"], "operator": "Equal", "value": t["value"], "effect": t["effect"]})
            elif k == 3:
                tols.append({"key": t["key"], "value": t["value"]})  # operator defaults to Equal, any effect
            else:
                tols.append({"key": t["key"], "operator": "Exists", "effect": r.pick(["NoSchedule", "NoExecute"])})
        if tols:
            spec["tolerations"] = tols
        if r.pct() < 20:
            spec["nodeSelector"] = {"disk": r.pick(["ssd", "hdd"])}
        na = {}
        if r.pct() < 60:
            terms = []
            for _ in range(1 + r.below(3)):
                t = {}
                if r.pct() < 75:
                    t["matchExpressions"] = [_na_expr(r, n_nodes) for _ in range(1 + r.below(3))]
                if r.pct() < 35:
                    t["matchFields"] = [_na_fields(r, n_nodes)]
                terms.append(t)
            na["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": terms}
        if r.pct() < 60:
            pref = []
            for _ in range(1 + r.below(3)):
                p = {}
                if r.pct() < 80:
                    p["matchExpressions"] = [_na_expr(r, n_nodes)]
                else:
                    p["matchFields"] = [_na_fields(r, n_nodes)]
                pref.append({"weight": 1 + r.below(100), "preference": p})
            na["preferredDuringSchedulingIgnoredDuringExecution"] = pref
        if na:
            spec["affinity"] = {"nodeAffinity": na}
        queue.append(pod_obj(f"pod-{j:07d}", _containers(r, scalar=False), ns=r.pick(NAMESPACES), **spec))
    prof = make_profile([("TaintToleration", 3), ("NodeAffinity", 2), ("NodeResourcesFit", 1),
                         ("NodeResourcesBalancedAllocation", 1)], seed)
    return {"profile": prof, "nodes": nodes, "pods": [], "queue": queue}


APPS = [f"app-{k}" for k in range(6)]


def _sel(r, key="app"):
    if r.pct() < 75:
        return {"matchLabels": {key: r.pick(APPS)}}
    return {"matchExpressions": [{"key": key, "operator": r.pick(["In", "NotIn"]),
                                  "values": sorted({r.pick(APPS) for _ in range(2)})}]}


def _labels(r):
    lab = {"app": r.pick(APPS), "tier": r.pick(["web", "db"])}
    if r.pct() < 50:
        lab["pod-template-hash"] = r.pick(["h1", "h2", "h3"])
    return lab


def _topo_nodes(r, n_nodes, taints=True):
    nodes = []
    for i in range(n_nodes):
        labels = {}
        if r.pct() < 88:
            labels[ZONE] = f"zone-{r.below(5)}"
        if r.pct() < 60:
            labels["disk"] = r.pick(["ssd", "hdd"])
        tl = [dict(NA_TAINTS[0])] if taints and r.pct() < 15 else []
        nodes.append(node_obj(f"node-{i:07d}", 1000 * r.pick([8, 16, 32]), Gi * r.pick([32, 64]), labels=labels,
                              taints=tl))
    return nodes


def _bound(r, nodes, n, terms_fn=None):
    pods = []
    for e in range(n):
        spec = {}
        if terms_fn:
            aff = terms_fn(r)
            if aff:
                spec["affinity"] = aff
        p = pod_obj(f"ex-{e:07d}", [req(100 * (1 + r.below(8)), 128 * Mi * (1 + r.below(8)))], labels=_labels(r),
                    node=nodes[r.below(len(nodes))]["metadata"]["name"], ns=r.pick(NAMESPACES), **spec)
        if r.pct() < 6:
            p["metadata"]["deletionTimestamp"] = "2025-01-01T00:00:00Z"  # terminating: PodTopologySpread skips it
        pods.append(p)
    return pods


def gen_pts(n_nodes=70, n_existing=160, n_pods=140, seed=None):
    seed = edge_seed("pts") if seed is None else seed
    r = Rng(seed)
    nodes = _topo_nodes(r, n_nodes)
    bound = _bound(r, nodes, n_existing)
    queue = []
    for j in range(n_pods):
        spec = {}
        tsc = []
        for _ in range(1 + r.below(3)):
            c = {"maxSkew": 1 + r.below(3), "topologyKey": r.pick([ZONE, ZONE, HOSTNAME, "disk"]),
                 "whenUnsatisfiable": r.pick(["DoNotSchedule", "ScheduleAnyway"]), "labelSelector": _sel(r)}
            if c["whenUnsatisfiable"] == "DoNotSchedule" and r.pct() < 35:
                c["minDomains"] = 2 + r.below(5)
            if r.pct() < 30:
                c["nodeAffinityPolicy"] = r.pick(["Honor", "Ignore"])
            if r.pct() < 30:
                c["nodeTaintsPolicy"] = r.pick(["Honor", "Ignore"])
            if r.pct() < 25:
                c["matchLabelKeys"] = [r.pick(["pod-template-hash", "tier", "missing-key"])]
            tsc.append(c)
        spec["topologySpreadConstraints"] = tsc
        if r.pct() < 25:
            spec["nodeSelector"] = {"disk": r.pick(["ssd", "hdd"])}
        if r.pct() < 20:
            spec["tolerations"] = [{"key": "dedicated", "operator": "Exists"}]
        queue.append(pod_obj(f"pod-{j:07d}", [req(100 * (1 + r.below(10)), 128 * Mi * (1 + r.below(10)))],
                             labels=_labels(r), ns=r.pick(NAMESPACES), **spec))
    prof = make_profile([("NodeResourcesFit", 1), ("PodTopologySpread", 2), ("NodeResourcesBalancedAllocation", 1)],
                        seed)
    return {"profile": prof, "nodes": nodes, "pods": bound, "queue": queue}


def _aff_term(r, topo=None):
    t = {"labelSelector": _sel(r), "topologyKey": topo or r.pick([ZONE, HOSTNAME, ZONE])}
    k = r.below(5)
    if k == 1:
        t["namespaces"] = sorted({r.pick(NAMESPACES) for _ in range(2)})
    elif k == 2:
        t["namespaceSelector"] = {}  # every namespace
    elif k == 3:
        t["namespaceSelector"] = {"matchLabels": {"team": "x"}}  # namespaces carry no labels: none
    return t


def _ipa_affinity(r, p_req_aff, p_req_anti, p_pref):
    aff, anti = {}, {}
    if r.pct() < p_req_aff:
        aff["requiredDuringSchedulingIgnoredDuringExecution"] = [_aff_term(r) for _ in range(1 + r.below(2))]
    if r.pct() < p_req_anti:
        anti["requiredDuringSchedulingIgnoredDuringExecution"] = [_aff_term(r, HOSTNAME)]
    if r.pct() < p_pref:
        aff["preferredDuringSchedulingIgnoredDuringExecution"] = [
            {"weight": 1 + r.below(100), "podAffinityTerm": _aff_term(r)} for _ in range(1 + r.below(2))]
    if r.pct() < p_pref // 2:
        anti["preferredDuringSchedulingIgnoredDuringExecution"] = [
            {"weight": 1 + r.below(100), "podAffinityTerm": _aff_term(r)}]
    out = {}
    if aff:
        out["podAffinity"] = aff
    if anti:
        out["podAntiAffinity"] = anti
    return out


def gen_ipa(variant="ipa", n_nodes=60, n_existing=150, n_pods=140, seed=None):
    seed = edge_seed(variant) if seed is None else seed
    r = Rng(seed)
    nodes = _topo_nodes(r, n_nodes, taints=False)
    bound = _bound(r, nodes, n_existing, lambda rr: _ipa_affinity(rr, 6, 8, 20))
    queue = []
    for j in range(n_pods):
        spec = {}
        aff = _ipa_affinity(r, 15, 25, 40)
        if aff:
            spec["affinity"] = aff
        queue.append(pod_obj(f"pod-{j:07d}", [req(100 * (1 + r.below(10)), 128 * Mi * (1 + r.below(10)))],
                             labels=_labels(r), ns=r.pick(NAMESPACES), **spec))
    prof = make_profile([("NodeResourcesFit", 1), ("InterPodAffinity", 2), ("NodeResourcesBalancedAllocation", 1)],
                        seed)
    ipa = prof["pluginConfig"]["InterPodAffinity"]
    if variant == "ipa_ignore":
        ipa["hardPodAffinityWeight"] = 0
        ipa["ignorePreferredTermsOfExistingPods"] = True
    else:
        ipa["hardPodAffinityWeight"] = 3
    return {"profile": prof, "nodes": nodes, "pods": bound, "queue": queue}


PRIORITIES = [0, 0, 10, 100, 1000]
PORT = {"containerPort": 8080, "hostPort": 8080, "protocol": "TCP"}


def _start(r):
    if r.pct() < 12:
        return None  # no status.startTime: started last
    return f"2025-01-{1 + r.below(28):02d}T{r.below(24):02d}:{r.pick([0, 30]):02d}:00Z"


def gen_preempt(n_nodes=24, n_existing=120, n_pods=90, seed=None, queue_sort=True):
    seed = edge_seed("preempt") if seed is None else seed
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        labels = {}
        if r.pct() < 85:
            labels[ZONE] = f"zone-{r.below(3)}"
        if r.pct() < 60:
            labels["disk"] = r.pick(["ssd", "hdd"])
        tl = [dict(NA_TAINTS[0])] if r.pct() < 12 else []
        nodes.append(node_obj(f"node-{i:07d}", 1000 * r.pick([4, 8]), Gi * r.pick([16, 32]),
                              pods=r.pick([110, 110, 110, 6]), labels=labels, taints=tl))
    bound = []
    for e in range(n_existing):
        spec = {"priority": r.pick(PRIORITIES)}
        if r.pct() < 8:
            spec["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": _sel(r), "topologyKey": HOSTNAME}]}}
        p = pod_obj(f"ex-{e:07d}", [req(250 * (1 + r.below(8)), 512 * Mi * (1 + r.below(6)))], labels=_labels(r),
                    node=nodes[r.below(n_nodes)]["metadata"]["name"], ns=r.pick(NAMESPACES),
                    ports={0: [dict(PORT)]} if r.pct() < 10 else None, **spec)
        st = _start(r)
        if st:
            p["status"] = {"startTime": st}
        bound.append(p)
    queue = []
    for j in range(n_pods):
        spec = {"priority": r.pick(PRIORITIES + [5000, 5000])}
        if r.pct() < 15:
            spec["preemptionPolicy"] = "Never"
        if r.pct() < 20:
            spec["topologySpreadConstraints"] = [{
                "maxSkew": 1, "topologyKey": r.pick([ZONE, HOSTNAME, "disk"]), "whenUnsatisfiable": "DoNotSchedule",
                "labelSelector": _sel(r)}]
        if r.pct() < 15:
            spec["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": _sel(r), "topologyKey": HOSTNAME}]}}
        if r.pct() < 15:
            spec["tolerations"] = [{"key": "dedicated", "operator": "Exists"}]
        if r.pct() < 10:
            spec["nodeSelector"] = {"disk": r.pick(["ssd", "hdd"])}
        cpu = 500 * (1 + r.below(8)) if r.pct() < 90 else 10000  # 10 cores: above every allocatable
        queue.append(pod_obj(f"pod-{j:07d}", [req(cpu, 512 * Mi * (1 + r.below(10)))], labels=_labels(r),
                             ns=r.pick(NAMESPACES), ports={0: [dict(PORT)]} if r.pct() < 12 else None, **spec))
    prof = make_profile([("TaintToleration", 3), ("NodeAffinity", 2), ("NodePorts", 1), ("NodeResourcesFit", 1),
                         ("PodTopologySpread", 2), ("InterPodAffinity", 2), ("DefaultPreemption", 1),
                         ("NodeResourcesBalancedAllocation", 1)], seed)
    doc = {"profile": prof, "nodes": nodes, "pods": bound, "queue": queue}
    if not queue_sort:
        doc["queueSort"] = False
    return doc


REGION = "topology.kubernetes.io/region"
BETA_ZONE = "failure-domain.beta.kubernetes.io/zone"
CSI = "csi.example.com"


def _pvc(name, ns, volume=None, cls=None, bound=False, modes=("ReadWriteOnce",), ann=None, **extra):
    md = {"name": name, "namespace": ns}
    a = dict(ann or {})
    if bound:
        a["pv.kubernetes.io/bind-completed"] = "yes"
    if a:
        md["annotations"] = a
    md.update(extra.pop("metadata", {}))
    spec = {"accessModes": list(modes), "resources": {"requests": {"storage": "1Gi"}}}
    if volume:
        spec["volumeName"] = volume
    if cls is not None:
        spec["storageClassName"] = cls
    o = {"metadata": md, "spec": spec}
    o.update(extra)
    return o


def _pv(name, cls, claim=None, labels=None, affinity=None, csi=True):
    spec = {"capacity": {"storage": "10Gi"}, "accessModes": ["ReadWriteOnce"], "storageClassName": cls}
    if csi:
        spec["csi"] = {"driver": CSI, "volumeHandle": name}
    if claim:
        spec["claimRef"] = {"namespace": claim[0], "name": claim[1]}
    if affinity is not None:
        spec["nodeAffinity"] = {"required": affinity}
    return {"metadata": {"name": name, "labels": dict(labels or {})}, "spec": spec}


def gen_volumes(n_nodes=40, n_existing=60, n_pods=120, seed=None):
    seed = edge_seed("volumes") if seed is None else seed
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        labels = {}
        if r.pct() < 80:
            z = r.below(3)
            labels[ZONE] = f"zone-{z}"
            if r.pct() < 70:
                labels[REGION] = "region-a" if z < 2 else "region-b"
        if r.pct() < 15:
            labels[BETA_ZONE] = f"zone-{r.below(3)}"
        nodes.append(node_obj(f"node-{i:07d}", 1000 * r.pick([8, 16]), Gi * r.pick([32, 64]), labels=labels))
    names = [n["metadata"]["name"] for n in nodes]
    classes = [
        {"metadata": {"name": "wffc-any"}, "provisioner": CSI, "volumeBindingMode": "WaitForFirstConsumer"},
        {"metadata": {"name": "wffc-zone"}, "provisioner": CSI, "volumeBindingMode": "WaitForFirstConsumer",
         "allowedTopologies": [{"matchLabelExpressions": [{"key": ZONE, "values": ["zone-0", "zone-1"]}]},
                               {"matchLabelExpressions": []}]},
        {"metadata": {"name": "wffc-region"}, "provisioner": CSI, "volumeBindingMode": "WaitForFirstConsumer",
         "allowedTopologies": [{"matchLabelExpressions": [{"key": REGION, "values": ["region-b"]},
                                                          {"key": ZONE, "values": ["zone-2"]}]}]},
        {"metadata": {"name": "wffc-static"}, "provisioner": "kubernetes.io/no-provisioner",
         "volumeBindingMode": "WaitForFirstConsumer"},
        {"metadata": {"name": "immediate"}, "provisioner": CSI, "volumeBindingMode": "Immediate"},
    ]
    pvs, pvcs = [], []
    ns_of = {}

    def claim(name, ns, **kw):
        pvcs.append(_pvc(name, ns, **kw))
        ns_of[name] = ns
        return name
    # bound claims (a pool several pods may use) and their PVs
    pool = []
    for k in range(14):
        ns = r.pick(NAMESPACES)
        cn, pn = f"data-{k:03d}", f"pv-{k:03d}"
        kind = k % 7
        labels, aff = {}, None
        if kind == 0:  # local PV: hostname affinity (VolumeBinding PreFilterResult)
            aff = {"nodeSelectorTerms": [{"matchExpressions": [
                {"key": HOSTNAME, "operator": "In", "values": [r.pick(names), r.pick(names)]}]}]}
        elif kind == 1:  # zonal PV by labels (VolumeZone)
            labels = {ZONE: r.pick(["zone-0", "zone-1", "zone-2", "zone-0__zone-2"])}
            if r.pct() < 50:
                labels[REGION] = r.pick(["region-a", "region-b"])
        elif kind == 2:  # zonal PV by node affinity
            aff = {"nodeSelectorTerms": [{"matchExpressions": [
                {"key": ZONE, "operator": "In", "values": [r.pick(["zone-0", "zone-1", "zone-2"])]}]},
                {"matchExpressions": [{"key": BETA_ZONE, "operator": "Exists"}]}]}
        elif kind == 3:  # labels + affinity; a malformed zone list is ignored by VolumeZone
            labels = {BETA_ZONE: "zone-1__", REGION: "region-a"}
            aff = {"nodeSelectorTerms": [{"matchExpressions": [{"key": REGION, "operator": "NotIn", "values": ["region-b"]}]}]}
        elif kind == 4:  # an affinity no node matches: empty terms / matchFields against a labels-only node
            aff = r.pick([{"nodeSelectorTerms": []},
                          {"nodeSelectorTerms": [{"matchFields": [
                              {"key": "metadata.name", "operator": "In", "values": [names[0]]}]}]},
                          {"nodeSelectorTerms": [{}]}])
        elif kind == 5:  # no constraints
            pass
        else:  # local PV on two nodes, several hostname terms (union)
            aff = {"nodeSelectorTerms": [
                {"matchExpressions": [{"key": HOSTNAME, "operator": "In", "values": names[k % n_nodes: k % n_nodes + 3]},
                                      {"key": HOSTNAME, "operator": "In", "values": names[k % n_nodes + 1: k % n_nodes + 2]}]},
                {"matchExpressions": [{"key": HOSTNAME, "operator": "In", "values": [names[(3 * k) % n_nodes]]}]}]}
        cls = r.pick(["wffc-any", "immediate", "wffc-zone"])
        pvs.append(_pv(pn, cls, claim=(ns, cn), labels=labels, affinity=aff))
        pool.append(claim(cn, ns, volume=pn, cls=cls, bound=True))
    gone = claim("data-gone", "default", volume="pv-gone", cls="wffc-any", bound=True)  # PV missing
    rwop_used = claim("rwop-used", "ns-a", volume="pv-rwop-1", cls="wffc-any", bound=True, modes=("ReadWriteOncePod",))
    pvs.append(_pv("pv-rwop-1", "wffc-any", claim=("ns-a", "rwop-used")))
    rwop_free = claim("rwop-free", "ns-b", volume="pv-rwop-2", cls="wffc-any", bound=True, modes=("ReadWriteOncePod",))
    pvs.append(_pv("pv-rwop-2", "wffc-any", claim=("ns-b", "rwop-free"),
                   affinity={"nodeSelectorTerms": [{"matchExpressions": [
                       {"key": ZONE, "operator": "In", "values": ["zone-1", "zone-2"]}]}]}))
    immediate = claim("data-immediate", "default", cls="immediate")
    prebound = claim("data-prebound", "default", volume="pv-005", cls="wffc-any")  # no bind-completed
    deleting = claim("data-deleting", "team-x", volume="pv-gone", cls="wffc-any", bound=True,
                     metadata={"deletionTimestamp": "2025-01-01T00:00:00Z"})
    lost = claim("data-lost", "ns-a", volume="pv-lost", cls="wffc-any", bound=True, status={"phase": "Lost"})
    bound = []
    for e in range(n_existing):
        ns = r.pick(NAMESPACES)
        spec = {}
        mine = [c for c in pool if ns_of[c] == ns]
        vols = []
        if mine and r.pct() < 40:
            vols.append(r.pick(mine))
        if e == 3:
            ns, vols = "ns-a", [rwop_used]
        if vols:
            spec["volumes"] = [{"name": f"v{i}", "persistentVolumeClaim": {"claimName": c}} for i, c in enumerate(vols)]
        bound.append(pod_obj(f"ex-{e:07d}", [req(100 * (1 + r.below(6)), 256 * Mi * (1 + r.below(6)))],
                             node=r.pick(names), ns=ns, **spec))
    queue = []
    for j in range(n_pods):
        ns = r.pick(NAMESPACES)
        vols = []
        k = r.pct()
        if k < 15:
            pass  # no volumes: every volume plugin Skips
        elif k < 50:
            mine = [c for c in pool if ns_of[c] == ns]
            if mine:
                vols = [r.pick(mine) for _ in range(1 + r.below(2))]
        elif k < 72:  # a fresh WaitForFirstConsumer claim of its own
            cls = r.pick(["wffc-any", "wffc-zone", "wffc-region", "wffc-static"])
            ann = {"volume.kubernetes.io/selected-node": r.pick(names + ["node-gone"])} if r.pct() < 20 else None
            vols = [claim(f"new-{j:04d}", ns, cls=cls, ann=ann)]
            mine = [c for c in pool if ns_of[c] == ns]
            if mine and r.pct() < 40:
                vols.append(r.pick(mine))
        elif k < 80:
            ns = "default"
            vols = [r.pick([immediate, prebound, gone, "no-such-claim", ""])]
        elif k < 86:
            ns, vols = r.pick([("team-x", [deleting]), ("ns-a", [lost])])
        else:
            ns, vols = r.pick([("ns-a", [rwop_used]), ("ns-b", [rwop_free])])
        spec = {}
        if vols:
            spec["volumes"] = [{"name": f"v{i}", "persistentVolumeClaim": {"claimName": c}} for i, c in enumerate(vols)]
        if r.pct() < 10:
            spec["nodeSelector"] = {ZONE: r.pick(["zone-0", "zone-1"])}
        queue.append(pod_obj(f"pod-{j:07d}", [req(100 * (1 + r.below(10)), 256 * Mi * (1 + r.below(8)))],
                             ns=ns, **spec))
    # NodeVolumeLimits: CSINode driver counts on some nodes, the legacy allocatable key on others
    csi_nodes = []
    for i, n in enumerate(nodes):
        k = r.pct()
        if k < 35:
            csi_nodes.append({"metadata": {"name": n["metadata"]["name"]},
                              "spec": {"drivers": [{"name": CSI, "nodeID": n["metadata"]["name"],
                                                    "allocatable": {"count": 1 + r.below(3)}}]}})
        elif k < 50:
            n["status"]["allocatable"]["attachable-volumes-csi-" + CSI] = str(1 + r.below(3))
        elif k < 55:
            csi_nodes.append({"metadata": {"name": n["metadata"]["name"]},
                              "spec": {"drivers": [{"name": CSI, "nodeID": n["metadata"]["name"]}]}})  # no count
    from .generator import DEFAULT_PROFILE
    prof = make_profile(DEFAULT_PROFILE, seed)
    return {"profile": prof, "nodes": nodes, "pods": bound, "queue": queue, "pvs": pvs, "pvcs": pvcs,
            "storageClasses": classes, "csiNodes": csi_nodes}


def gen_queue(n_nodes=16, n_existing=60, n_pods=70, seed=None):
    seed = edge_seed("queue") if seed is None else seed
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        labels = {ZONE: f"zone-{r.below(3)}"} if r.pct() < 90 else {}
        nodes.append(node_obj(f"node-{i:07d}", 1000 * r.pick([4, 8]), Gi * r.pick([16, 32]),
                              pods=r.pick([110, 110, 8]), labels=labels))
    pods = []
    for e in range(n_existing):
        p = pod_obj(f"ex-{e:07d}", [req(250 * (1 + r.below(8)), 512 * Mi * (1 + r.below(6)))], labels=_labels(r),
                    node=nodes[r.below(n_nodes)]["metadata"]["name"], ns=r.pick(NAMESPACES),
                    priority=r.pick(PRIORITIES))
        st = _start(r)
        if st:
            p["status"] = {"startTime": st}
        pods.append(p)
    for j in range(n_pods):
        spec = {"priority": r.pick(PRIORITIES + [5000, 20000])}
        if r.pct() < 18:
            spec["schedulingGates"] = [{"name": r.pick(["example.com/quota", "example.com/storage"])}]
        if r.pct() < 10:
            spec["preemptionPolicy"] = "Never"
        if r.pct() < 20:
            spec["topologySpreadConstraints"] = [{
                "maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": r.pick(["DoNotSchedule", "ScheduleAnyway"]),
                "labelSelector": _sel(r)}]
        cpu = 500 * (1 + r.below(8)) if r.pct() < 92 else 10000
        p = pod_obj(f"pod-{j:07d}", [req(cpu, 512 * Mi * (1 + r.below(10)))], labels=_labels(r),
                    ns=r.pick(NAMESPACES), **spec)
        pods.insert(r.below(len(pods) + 1), p)  # pending pods anywhere in the document
    from .generator import DEFAULT_PROFILE
    prof = make_profile(DEFAULT_PROFILE, seed)
    return {"profile": prof, "nodes": nodes, "pods": pods, "pvs": [], "pvcs": [], "storageClasses": [],
            "priorityClasses": [], "namespaces": []}


def generate_edge(variant: str, **sizes) -> dict:
    if variant in ("fit_most", "fit_rtc"):
        return gen_fit(variant, **sizes)
    if variant == "na":
        return gen_na(**sizes)
    if variant == "pts":
        return gen_pts(**sizes)
    if variant in ("ipa", "ipa_ignore"):
        return gen_ipa(variant, **sizes)
    if variant == "preempt":
        return gen_preempt(**sizes)
    if variant == "volumes":
        return gen_volumes(**sizes)
    if variant == "queue":
        return gen_queue(**sizes)
    raise ValueError(variant)


def dumps(doc) -> str:
    return json.dumps(doc, separators=(",", ":"), sort_keys=False)
