"""Synthetic cluster generator for the five BASELINE.json configs.

Every draw comes from one splitmix64 stream seeded with ``20250131*100 + c`` so a
cluster is a pure function of (config, sizes, seed).  The output is a
Kubernetes-shaped JSON document (``metadata``/``spec``/``status`` with quantity
strings) that both the CPU oracle (``oracle/``) and the product host encoder
(``csrc/host``) parse independently:

    {"profile": {...}, "nodes": [Node...], "pods": [bound Pod...], "queue": [Pod...]}

``pods`` are already bound (``spec.nodeName`` set; they make up the NodeInfo of
each node, upstream ``framework.NodeInfo.AddPod``), ``queue`` is the scheduling
queue in PrioritySort order (all priorities equal => FIFO).

The profile mirrors a KubeSchedulerConfiguration MultiPoint plugin list, the
shape the reference pins in ``simulator/scheduler/scheduler_test.go:531-557``.
Names are zero padded (``node-%07d``) so Go's sorted JSON map order equals index
order.
"""
from __future__ import annotations

import json

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15

HOSTNAME = "kubernetes.io/hostname"
ZONE = "topology.kubernetes.io/zone"
Mi = 1 << 20
Gi = 1 << 30


def splitmix64(x: int) -> int:
    """One splitmix64 output for state ``x`` (state is advanced by GOLDEN first)."""
    z = (x + GOLDEN) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def tiebreak_h20(seed: int, pod_idx: int, node_idx: int) -> int:
    """20-bit tie-break hash shared by GPU and oracle."""
    return splitmix64((seed ^ ((pod_idx * GOLDEN) & M64) ^ node_idx) & M64) >> 44


class Rng:
    def __init__(self, seed: int):
        self.s = seed & M64

    def next(self) -> int:
        self.s = (self.s + GOLDEN) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    def below(self, n: int) -> int:
        return self.next() % n

    def pct(self) -> int:
        return self.next() % 100

    def pick(self, seq):
        return seq[self.next() % len(seq)]


def config_seed(c: int) -> int:
    return 20250131 * 100 + c


# --------------------------------------------------------------------------- profiles
# weights: framework weights (used for the total/selectHost).  storeWeights:
# the result store's map (plugins.go:289-304 getScorePluginWeight); identical
# unless a test exercises the MultiPoint/Score quirk (scheduler_test.go:344-407).
DEFAULT_ARGS = {
    "NodeResourcesFit": {"scoringStrategy": {"type": "LeastAllocated",
                                             "resources": [{"name": "cpu", "weight": 1},
                                                           {"name": "memory", "weight": 1}]}},
    "NodeResourcesBalancedAllocation": {"resources": [{"name": "cpu", "weight": 1},
                                                      {"name": "memory", "weight": 1}]},
    "InterPodAffinity": {"hardPodAffinityWeight": 1, "ignorePreferredTermsOfExistingPods": False},
    "PodTopologySpread": {"defaultingType": "System"},
}


def make_profile(plugins, seed):
    """plugins: list of (name, weight) in MultiPoint order."""
    return {
        "plugins": [p for p, _ in plugins],
        "weights": {p: w for p, w in plugins},
        "storeWeights": {p: w for p, w in plugins},
        "pluginConfig": json.loads(json.dumps(DEFAULT_ARGS)),
        "seed": seed,
    }


def config_profile(plugins, seed, score=None):
    """The same profile as a KubeSchedulerConfiguration after the simulator's
    ConvertForSimulator (scheduler_test.go:344-407 "want"): MultiPoint lists every
    plugin as "<name>Wrapped" (default MultiPoint disabled "*"), `score` adds
    Score.Enabled entries [(name, weight)] that re-weight MultiPoint plugins.
    ksg_create resolves it like the framework (weights) and the store
    (storeWeights) do; see include/ksg.h ksg_plugin_weights."""
    def ent(n, w):
        e = {"name": n + "Wrapped"}
        if w is not None:
            e["weight"] = w
        return e
    return {"profiles": [{
        "schedulerName": "default-scheduler",
        "plugins": {"multiPoint": {"enabled": [ent(p, w) for p, w in plugins], "disabled": [{"name": "*"}]},
                    "score": {"enabled": [ent(p, w) for p, w in (score or [])]}},
        "pluginConfig": [{"name": k + "Wrapped", "args": v} for k, v in json.loads(json.dumps(DEFAULT_ARGS)).items()],
        "seed": seed}]}


# default profile order/weights for the hot-path plugins (scheduler_test.go:535-557)
DEFAULT_HOT_PROFILE = [("TaintToleration", 3), ("NodeAffinity", 2), ("NodeResourcesFit", 1),
                       ("PodTopologySpread", 2), ("InterPodAffinity", 2),
                       ("NodeResourcesBalancedAllocation", 1)]


# the whole default profile (scheduler_test.go:531-557 configGeneratedFromDefault):
# MultiPoint order; plugins without an explicit weight get 1 (plugins.go:289-304)
DEFAULT_PROFILE = [("SchedulingGates", 1), ("PrioritySort", 1), ("NodeUnschedulable", 1), ("NodeName", 1),
                   ("TaintToleration", 3), ("NodeAffinity", 2), ("NodePorts", 1), ("NodeResourcesFit", 1),
                   ("VolumeRestrictions", 1), ("EBSLimits", 1), ("GCEPDLimits", 1), ("NodeVolumeLimits", 1),
                   ("AzureDiskLimits", 1), ("VolumeBinding", 1), ("VolumeZone", 1), ("PodTopologySpread", 2),
                   ("InterPodAffinity", 2), ("DefaultPreemption", 1), ("NodeResourcesBalancedAllocation", 1),
                   ("ImageLocality", 1), ("DefaultBinder", 1)]


# --------------------------------------------------------------------------- builders
def node_obj(name, cpu_milli, mem, pods=110, labels=None, taints=None, eph=None, scalars=None, images=None,
             unschedulable=False):
    alloc = {"cpu": f"{cpu_milli}m" if cpu_milli % 1000 else str(cpu_milli // 1000),
             "memory": f"{mem // Gi}Gi" if mem % Gi == 0 else str(mem),
             "pods": str(pods)}
    if eph is not None:
        alloc["ephemeral-storage"] = str(eph)
    for k, v in (scalars or {}).items():
        alloc[k] = str(v)
    lab = {HOSTNAME: name}
    lab.update(labels or {})
    spec = {}
    if taints:
        spec["taints"] = taints
    if unschedulable:
        spec["unschedulable"] = True
    status = {"allocatable": alloc, "capacity": dict(alloc)}
    if images:
        status["images"] = [{"names": list(n), "sizeBytes": sz} for n, sz in images]
    return {"metadata": {"name": name, "labels": lab}, "spec": spec, "status": status}


def req(cpu_milli=None, mem=None, extra=None):
    r = {}
    if cpu_milli is not None:
        r["cpu"] = f"{cpu_milli}m"
    if mem is not None:
        r["memory"] = f"{mem // Mi}Mi" if mem % Mi == 0 else str(mem)
    r.update(extra or {})
    return {"requests": r} if r else {}


def pod_obj(name, containers, labels=None, node=None, ns="default", images=None, ports=None, **spec_extra):
    """images / ports: per container (image name, list of v1.ContainerPort dicts)."""
    spec = {"containers": [{"name": f"c{i}", "image": (images or {}).get(i, "registry.k8s.io/pause:3.5"),
                            "resources": c} for i, c in enumerate(containers)]}
    for i, ps in (ports or {}).items():
        spec["containers"][i]["ports"] = ps
    if node is not None:
        spec["nodeName"] = node
    spec.update(spec_extra)
    return {"metadata": {"name": name, "namespace": ns, "labels": dict(labels or {})},
            "spec": spec}


def filler_pod(name, node, cpu, mem):
    """Pre-utilisation: one bound pod carrying the node's initial requests."""
    return pod_obj(name, [req(cpu, mem)], labels={"role": "filler"}, node=node)


# --------------------------------------------------------------------------- config 1
# image vocabulary of cfg1: (names as listed in node.status.images, sizeBytes)
CFG1_IMAGES = [((f"registry.k8s.io/app-{k}:1.{k}", f"registry.k8s.io/app-{k}@sha256:{k:064x}"), (40 + 110 * k) * Mi)
               for k in range(8)] + [(("docker.io/library/busybox:latest",), 4 * Mi),
                                     (("quay.io/big/model:latest",), 1800 * Mi)]
CFG1_POD_IMAGES = [f"registry.k8s.io/app-{k}:1.{k}" for k in range(8)] + [
    "docker.io/library/busybox", "quay.io/big/model", "registry.k8s.io/pause:3.5", "example.com:5000/tool"]


def gen_cfg1(n_nodes=100, n_pods=1000, seed=None):
    """Default KubeSchedulerConfiguration (all 21 MultiPoint plugins).  Besides the
    hot-path plugins' inputs the cluster carries what the rest of the default
    profile reads: cordoned nodes (NodeUnschedulable), node images (ImageLocality),
    host ports on bound and queued pods (NodePorts)."""
    seed = config_seed(1) if seed is None else seed
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        imgs = [CFG1_IMAGES[r.below(len(CFG1_IMAGES))] for _ in range(r.below(5))]
        imgs = list({n[0]: (n, sz) for n, sz in imgs}.values())
        nodes.append(node_obj(f"node-{i:07d}", 16000, 64 * Gi, labels={ZONE: f"zone-{i % 4}"}, images=imgs,
                              unschedulable=r.pct() < 8))
    bound = []
    for i in range(0, n_nodes, 5):  # a host-port daemon on every fifth node
        ports = [{"containerPort": 9100, "hostPort": 9100, "protocol": "TCP"}]
        if i % 10 == 0:
            ports.append({"containerPort": 53, "hostPort": 5353, "protocol": "UDP", "hostIP": "10.0.0.1"})
        bound.append(pod_obj(f"daemon-{i:07d}", [req(100, 128 * Mi)], labels={"app": "daemon"},
                             node=nodes[i]["metadata"]["name"], ports={0: ports}))
    queue = []
    for j in range(n_pods):
        nc = 2 if r.pct() < 10 else 1
        if r.pct() < 10:
            c = [{}] * nc
        else:
            c = [req(100 * (1 + r.below(10)), 256 * Mi * (1 + r.below(8))) for _ in range(nc)]
        images = {k: CFG1_POD_IMAGES[r.below(len(CFG1_POD_IMAGES))] for k in range(nc)}
        ports = None
        u = r.pct()
        if u < 4:
            ports = {0: [{"containerPort": 8080, "hostPort": 8080 + r.below(3)}]}
        elif u < 6:
            ports = {0: [{"containerPort": 9100, "hostPort": 9100, "protocol": "TCP", "hostIP": "10.0.0.2"}]}
        elif u < 7:
            ports = {0: [{"containerPort": 53, "hostPort": 5353, "protocol": "UDP"}]}
        extra = {}
        if r.pct() < 10:
            extra["tolerations"] = [{"key": "node.kubernetes.io/unschedulable", "operator": "Exists",
                                     "effect": "NoSchedule"}]
        queue.append(pod_obj(f"pod-{j:07d}", c, labels={"app": f"app-{r.below(10)}"}, images=images, ports=ports,
                             **extra))
    return {"profile": make_profile(DEFAULT_PROFILE, seed), "nodes": nodes, "pods": bound, "queue": queue}


# --------------------------------------------------------------------------- config 2
CFG2_SHAPES = [(8000, 32 * Gi), (16000, 64 * Gi), (32000, 128 * Gi), (64000, 256 * Gi)]


def _cfg2_pod(r, name):
    if r.pct() < 10:                     # BestEffort
        return pod_obj(name, [{}])
    cs = [req(50 * (1 + r.below(40)), 64 * Mi * (1 + r.below(64)))]
    if r.pct() < 5:                      # two-container pod
        cs.append(req(50 * (1 + r.below(40)), 64 * Mi * (1 + r.below(64))))
    return pod_obj(name, cs)


def gen_cfg2(n_nodes=5000, n_pods=10000, seed=None):
    seed = config_seed(2) if seed is None else seed
    r = Rng(seed)
    nodes, bound = [], []
    for i in range(n_nodes):
        cpu, mem = CFG2_SHAPES[r.below(4)]
        name = f"node-{i:07d}"
        nodes.append(node_obj(name, cpu, mem))
        uc, um = r.below(51), r.below(51)
        if uc or um:
            bound.append(filler_pod(f"fill-{i:07d}", name, cpu * uc // 100, mem * um // 100))
    queue = [_cfg2_pod(r, f"pod-{j:07d}") for j in range(n_pods)]
    prof = make_profile([("NodeResourcesFit", 1), ("NodeResourcesBalancedAllocation", 1)], seed)
    return {"profile": prof, "nodes": nodes, "pods": bound, "queue": queue}


# --------------------------------------------------------------------------- config 3
CFG3_EFFECTS = ["NoSchedule"] * 12 + ["PreferNoSchedule"] * 12 + ["NoExecute"] * 8
CFG3_TAINTS = [{"key": f"taint-{t:02d}", "value": f"v{t % 3}", "effect": CFG3_EFFECTS[t]}
               for t in range(32)]
CFG3_LABELS = {
    ZONE: [f"zone-{z:02d}" for z in range(20)],
    "node.kubernetes.io/instance-type": [f"it-{t:02d}" for t in range(16)],
    "kubernetes.io/arch": ["amd64", "arm64"],
    "tier": ["a", "b", "c"],
    "gen": [str(g) for g in range(1, 9)],
}


def _cfg3_node(r, i):
    name = f"node-{i:07d}"
    cpu, mem = CFG2_SHAPES[r.below(4)]
    labels = {k: r.pick(v) for k, v in CFG3_LABELS.items()}
    for f in range(48):
        if r.below(4) == 0:
            labels[f"feat-{f:02d}"] = "true"
    p = r.pct()
    nt = 0 if p < 40 else 1 if p < 70 else 2 if p < 90 else 3 + r.below(2)
    taints, seen = [], set()
    for _ in range(nt):
        t = r.below(32)
        if t not in seen:
            seen.add(t)
            taints.append(dict(CFG3_TAINTS[t]))
    return node_obj(name, cpu, mem, labels=labels, taints=taints), (cpu, mem)


def _cfg3_req_expr(r):
    kind = r.below(4)
    if kind == 0:   # In
        k = r.pick(list(CFG3_LABELS.keys()))
        vals = sorted({r.pick(CFG3_LABELS[k]) for _ in range(1 + r.below(3))})
        return {"key": k, "operator": "In", "values": vals}
    if kind == 1:   # NotIn
        k = r.pick(list(CFG3_LABELS.keys()))
        vals = sorted({r.pick(CFG3_LABELS[k]) for _ in range(1 + r.below(2))})
        return {"key": k, "operator": "NotIn", "values": vals}
    if kind == 2:   # Exists on a feature label
        return {"key": f"feat-{r.below(48):02d}", "operator": "Exists"}
    return {"key": "gen", "operator": "Gt", "values": [str(1 + r.below(6))]}


def _cfg3_pod(r, name):
    p = r.pct()
    cs = [{}] if p < 10 else [req(50 * (1 + r.below(40)), 64 * Mi * (1 + r.below(64)))]
    spec = {}
    tols = []
    for _ in range(r.below(5)):
        t = CFG3_TAINTS[r.below(32)]
        tol = {"key": t["key"]}
        if r.pct() < 70:
            tol["operator"] = "Equal"
            tol["value"] = t["value"]
        else:
            tol["operator"] = "Exists"
        if r.pct() >= 20:
            tol["effect"] = t["effect"]
        tols.append(tol)
    if tols:
        spec["tolerations"] = tols
    na = {}
    if r.pct() < 50:
        terms = []
        for _ in range(1 + r.below(2)):
            terms.append({"matchExpressions": [_cfg3_req_expr(r) for _ in range(1 + r.below(3))]})
        na["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": terms}
    if r.pct() < 20:
        k = r.pick(["tier", "kubernetes.io/arch", ZONE])
        spec["nodeSelector"] = {k: r.pick(CFG3_LABELS[k])}
    if r.pct() < 60:
        pref = []
        for _ in range(1 + r.below(4)):
            pref.append({"weight": 1 + r.below(100),
                         "preference": {"matchExpressions": [_cfg3_req_expr(r)]}})
        na["preferredDuringSchedulingIgnoredDuringExecution"] = pref
    if na:
        spec["affinity"] = {"nodeAffinity": na}
    return pod_obj(name, cs, **spec)


def gen_cfg3(n_nodes=15000, n_pods=10000, seed=None, feasible_check=True):
    seed = config_seed(3) if seed is None else seed
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        n, _ = _cfg3_node(r, i)
        nodes.append(n)
    queue = []
    for j in range(n_pods):
        for _attempt in range(64):
            p = _cfg3_pod(r, f"pod-{j:07d}")
            if not feasible_check or _cfg3_feasible_somewhere(p, nodes):
                break
        queue.append(p)
    prof = make_profile([("TaintToleration", 3), ("NodeAffinity", 2), ("NodeResourcesFit", 1),
                         ("NodeResourcesBalancedAllocation", 1)], seed)
    return {"profile": prof, "nodes": nodes, "pods": [], "queue": queue}


def _tolerates(tols, taint):
    for t in tols:
        if t.get("effect") and t["effect"] != taint["effect"]:
            continue
        if t.get("key") and t["key"] != taint["key"]:
            continue
        op = t.get("operator", "")
        if op in ("", "Equal") and t.get("value", "") == taint.get("value", ""):
            return True
        if op == "Exists":
            return True
    return False


def _expr_ok(e, labels):
    k, op, vals = e["key"], e["operator"], e.get("values", [])
    has = k in labels
    if op == "In":
        return has and labels[k] in vals
    if op == "NotIn":
        return not has or labels[k] not in vals
    if op == "Exists":
        return has
    if op == "DoesNotExist":
        return not has
    if op in ("Gt", "Lt"):
        try:
            a, b = int(labels[k]), int(vals[0])
        except (KeyError, ValueError, IndexError):
            return False
        return a > b if op == "Gt" else a < b
    return False


def _cfg3_feasible_somewhere(p, nodes):
    """Cheap generator-side screen (not the oracle): some node tolerates+matches."""
    spec = p["spec"]
    tols = spec.get("tolerations", [])
    sel = spec.get("nodeSelector", {})
    req_terms = (spec.get("affinity", {}).get("nodeAffinity", {})
                 .get("requiredDuringSchedulingIgnoredDuringExecution", {})
                 .get("nodeSelectorTerms"))
    for n in nodes:
        lab = n["metadata"]["labels"]
        if any(t["effect"] in ("NoSchedule", "NoExecute") and not _tolerates(tols, t)
               for t in n["spec"].get("taints", [])):
            continue
        if any(lab.get(k) != v for k, v in sel.items()):
            continue
        if req_terms is not None and not any(
                all(_expr_ok(e, lab) for e in t.get("matchExpressions", [])) for t in req_terms):
            continue
        return True
    return False


# --------------------------------------------------------------------------- config 4
def _sel(labels):
    return {"matchLabels": dict(labels)}


def gen_cfg4(n_nodes=50000, n_existing=200000, n_pods=10000, n_zones=20, seed=None):
    seed = config_seed(4) if seed is None else seed
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        name = f"node-{i:07d}"
        nodes.append(node_obj(name, 32000, 128 * Gi,
                              labels={ZONE: f"zone-{(i * n_zones) // n_nodes:02d}"}))
    n_apps = 200
    bound = []
    for e in range(n_existing):
        app, team = f"app-{r.below(n_apps):03d}", f"team-{r.below(10)}"
        node = f"node-{r.below(n_nodes):07d}"
        spec = {}
        p = r.pct()
        aff = {}
        if p < 5:
            aff["podAntiAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": _sel({"app": app}), "topologyKey": HOSTNAME}]}
        elif p < 15:
            aff["podAffinity"] = {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 1 + r.below(100),
                 "podAffinityTerm": {"labelSelector": _sel({"team": team}), "topologyKey": ZONE}}]}
        elif p < 20:
            aff["podAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": _sel({"team": team}), "topologyKey": ZONE}]}
        if aff:
            spec["affinity"] = aff
        bound.append(pod_obj(f"ex-{e:07d}", [req(100 * (1 + r.below(5)), 128 * Mi * (1 + r.below(8)))],
                             labels={"app": app, "team": team}, node=node, **spec))
    queue = []
    for j in range(n_pods):
        app, team = f"app-{r.below(n_apps):03d}", f"team-{r.below(10)}"
        spec = {}
        tsc = []
        if r.pct() < 70:
            tsc.append({"maxSkew": 1 + r.below(3), "topologyKey": ZONE,
                        "whenUnsatisfiable": "DoNotSchedule", "labelSelector": _sel({"app": app})})
        if r.pct() < 50:
            tsc.append({"maxSkew": 1 + r.below(5), "topologyKey": HOSTNAME,
                        "whenUnsatisfiable": "ScheduleAnyway", "labelSelector": _sel({"app": app})})
        if tsc:
            spec["topologySpreadConstraints"] = tsc
        aff = {}
        if r.pct() < 20:
            aff.setdefault("podAntiAffinity", {})["requiredDuringSchedulingIgnoredDuringExecution"] = [
                {"labelSelector": _sel({"app": app}), "topologyKey": HOSTNAME}]
        if r.pct() < 20:
            aff.setdefault("podAffinity", {})["preferredDuringSchedulingIgnoredDuringExecution"] = [
                {"weight": 1 + r.below(100),
                 "podAffinityTerm": {"labelSelector": _sel({"team": team}), "topologyKey": ZONE}}]
        if r.pct() < 10:
            aff.setdefault("podAntiAffinity", {})["preferredDuringSchedulingIgnoredDuringExecution"] = [
                {"weight": 1 + r.below(100),
                 "podAffinityTerm": {"labelSelector": _sel({"app": app}), "topologyKey": ZONE}}]
        if aff:
            spec["affinity"] = aff
        queue.append(pod_obj(f"pod-{j:07d}", [req(100 * (1 + r.below(10)), 128 * Mi * (1 + r.below(16)))],
                             labels={"app": app, "team": team}, **spec))
    prof = make_profile([("NodeResourcesFit", 1), ("PodTopologySpread", 2), ("InterPodAffinity", 2),
                         ("NodeResourcesBalancedAllocation", 1)], seed)
    return {"profile": prof, "nodes": nodes, "pods": bound, "queue": queue}


# --------------------------------------------------------------------------- config 5
def gen_cfg5(n_nodes=1_000_000, n_pods=4096, seed=None):
    """What-if batch: cfg3 node distribution, Fit+BA+Taint+NodeAffinity."""
    seed = config_seed(5) if seed is None else seed
    doc = gen_cfg3(n_nodes=n_nodes, n_pods=n_pods, seed=seed, feasible_check=False)
    doc["profile"]["seed"] = seed
    return doc


GENERATORS = {1: gen_cfg1, 2: gen_cfg2, 3: gen_cfg3, 4: gen_cfg4, 5: gen_cfg5}


def generate(c: int, **sizes) -> dict:
    return GENERATORS[c](**sizes)


def dumps(doc) -> str:
    return json.dumps(doc, separators=(",", ":"), sort_keys=False)


def generate_native(c: int, n_nodes=-1, n_pods=-1, n_existing=-1, n_zones=-1, seed=0) -> bytes:
    """The same document as generate(c, ...) as JSON bytes, built by the native twin
    (libksg.so ksg_synth_cluster, csrc/synth.cpp): configs 2..5 at full size in
    seconds.  tests/test_synth.py checks the two agree."""
    import ctypes
    from .engine import load_library
    L = load_library()
    out, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = L.ksg_synth_cluster(c, n_nodes, n_pods, n_existing, n_zones, seed, ctypes.byref(out), ctypes.byref(n))
    if rc != 0:
        raise ValueError(f"ksg_synth_cluster({c}) failed ({rc})")
    try:
        return ctypes.string_at(out, n.value)
    finally:
        L.ksg_free(out)
