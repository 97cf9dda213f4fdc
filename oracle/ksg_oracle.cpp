// ksg_oracle — CPU restatement of the reference's scheduling-cycle hot path.
//
// TEST INFRASTRUCTURE ONLY.  Nothing in the product (kube-scheduler-simulator-p9_amd/)
// may link, load or call this file; only tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py use it, as the checker / timed CPU baseline.
//
// What it restates.  The arithmetic of the path
// lives in k8s.io/kubernetes v1.30.4 and k8s.io/component-helpers v0.30.4
// (pinned at /root/reference/simulator/go.mod:55, go.sum:410/434), which are NOT
// vendored in /root/reference; those upstream algorithms are restated here from
// their published source, and the reference's own call sites are followed for
// how results are recorded:
//   * framework cycle: schedulePod / findNodesThatPassFilters / RunFilterPlugins
//     (first failure stops), RunPreScorePlugins (Skip), RunScorePlugins (score,
//     NormalizeScore, [0,100] check, x weight) [upstream schedule_one.go,
//     framework/runtime/framework.go]; selectHost replaced by the seeded
//     deterministic rule of SURVEY.md §8(e).
//   * plugins: NodeResourcesFit (fit.go, resource_allocation.go,
//     least_allocated.go, most_allocated.go), NodeResourcesBalancedAllocation
//     (balanced_allocation.go), TaintToleration (taint_toleration.go),
//     NodeAffinity (node_affinity.go + component-helpers nodeaffinity),
//     PodTopologySpread (filtering.go, scoring.go, common.go), InterPodAffinity
//     (filtering.go, scoring.go), helper.DefaultNormalizeScore; the rest of
//     the default profile (scheduler_test.go:531-557): NodeUnschedulable
//     (node_unschedulable.go), NodeName (node_name.go), NodePorts
//     (node_ports.go + framework HostPortInfo), ImageLocality
//     (image_locality.go + ImageStateSummary.Snapshot), the volume plugins'
//     PreFilter/PreScore Skip for pods without volumes they act on
//     (VolumeRestrictions, EBSLimits, GCEPDLimits, NodeVolumeLimits,
//     AzureDiskLimits, VolumeBinding, VolumeZone), and the plugins with no
//     PreFilter/Filter/PreScore/Score extension (PrioritySort, SchedulingGates,
//     DefaultPreemption, DefaultBinder: the wrapper records nothing for them).
//   * recording: simulator/scheduler/plugin/wrappedplugin.go:388-548,616-645
//     (what is recorded per extension point) and resultstore/store.go:133-507
//     (maps, finalscore = score x weight, GetStoredResult JSON).
//
// Parity pins: the README / debuggable-scheduler.md example
// (Fit 73, BA 76, Taint final 300) and store/weight semantics from
// resultstore/store_test.go:284-833.  Everything else is "parity unpinned"
// against the real Go code (no Go toolchain / module cache in this container) and
// is pinned to this restatement instead; see DESIGN.md.
//
// Float64 work follows the reference operation order with no contraction
// (build with -ffp-contract=off); PodTopologySpread uses a restatement of Go's
// math.Log (go_log below), never libm.

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "ojson.hpp"

namespace oracle {

using std::map;
using std::set;
using std::string;
using std::vector;
typedef long long i64;
typedef __int128 i128;

static const i64 kMaxNodeScore = 100;
static const i64 kDefaultMilliCPU = 100;               // schedutil.DefaultMilliCPURequest
static const i64 kDefaultMemory = 200LL * 1024 * 1024;  // schedutil.DefaultMemoryRequest

// ============================================================ Go math restatements
// Go math.Log (src/math/log.go; the amd64 assembly follows the same formula).
static double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
               L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
               L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
               L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (std::isnan(x) || (std::isinf(x) && x > 0)) return x;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = std::frexp(x, &ki);
  if (f1 < M_SQRT2 / 2) {
    f1 *= 2;
    ki--;
  }
  double f = f1 - 1;
  double k = double(ki);
  double s = f / (2 + f);
  double s2 = s * s;
  double s4 = s2 * s2;
  double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  double R = t1 + t2;
  double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

// Go math.Round: half away from zero (same as C round()).
static double go_round(double x) { return std::round(x); }

// strconv.ParseInt(s, 10, 64)
static bool go_parse_int64(const string& s, i64& out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
    if (s.size() == 1) return false;
  }
  unsigned long long v = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    unsigned d = s[i] - '0';
    if (v > (18446744073709551615ULL - d) / 10) return false;
    v = v * 10 + d;
  }
  if (!neg && v > 9223372036854775807ULL) return false;
  if (neg && v > 9223372036854775808ULL) return false;
  out = neg ? (i64)(0 - v) : (i64)v;
  return true;
}

// ============================================================ quantities
// resource.Quantity held exactly in nano units (enough for every suffix we accept).
static bool parse_quantity(const string& s, i128& nano) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[i] == '+' || s[i] == '-') { neg = s[i] == '-'; ++i; }
  i128 mant = 0;
  int frac_digits = 0;
  bool any = false, dot = false;
  for (; i < s.size(); ++i) {
    char c = s[i];
    if (c >= '0' && c <= '9') {
      mant = mant * 10 + (c - '0');
      if (dot) frac_digits++;
      any = true;
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (!any) return false;
  string suf = s.substr(i);
  // value = mant * 10^-frac * mult
  i128 num = mant * 1000000000;  // nano
  i128 den = 1;
  for (int k = 0; k < frac_digits; ++k) den *= 10;
  auto mulpow = [&](int base, int e) { for (int k = 0; k < e; ++k) num *= base; };
  auto divpow = [&](int base, int e) { for (int k = 0; k < e; ++k) den *= base; };
  if (suf.empty()) {
  } else if (suf == "n") divpow(10, 9);
  else if (suf == "u") divpow(10, 6);
  else if (suf == "m") divpow(10, 3);
  else if (suf == "k") mulpow(10, 3);
  else if (suf == "M") mulpow(10, 6);
  else if (suf == "G") mulpow(10, 9);
  else if (suf == "T") mulpow(10, 12);
  else if (suf == "P") mulpow(10, 15);
  else if (suf == "E") mulpow(10, 18);
  else if (suf == "Ki") mulpow(2, 10);
  else if (suf == "Mi") mulpow(2, 20);
  else if (suf == "Gi") mulpow(2, 30);
  else if (suf == "Ti") mulpow(2, 40);
  else if (suf == "Pi") mulpow(2, 50);
  else if (suf == "Ei") mulpow(2, 60);
  else if (suf[0] == 'e' || suf[0] == 'E') {
    i64 e;
    if (!go_parse_int64(suf.substr(1), e)) return false;
    if (e >= 0) mulpow(10, (int)e); else divpow(10, (int)-e);
  } else return false;
  // round up to nano (Quantity keeps at most nano precision; rounding up)
  i128 q = num / den;
  if (q * den != num) q += 1;
  nano = neg ? -q : q;
  return true;
}
static i64 ceil_div(i128 a, i64 b) {
  i128 q = a / b;
  if (q * b != a && a > 0) q += 1;
  return (i64)q;
}
static i64 q_value(i128 nano) { return ceil_div(nano, 1000000000LL); }
static i64 q_milli(i128 nano) { return ceil_div(nano, 1000000LL); }

typedef map<string, i128> ResourceList;  // presence matters (applyNonMissing)

// ============================================================ label selectors
enum Op { OpIn, OpNotIn, OpExists, OpDoesNotExist, OpGt, OpLt };
struct Req {
  string key;
  Op op;
  set<string> vals;
  i64 num = 0;  // Gt/Lt
};
typedef map<string, string> Labels;

static bool req_matches(const Req& r, const Labels& ls) {
  auto it = ls.find(r.key);
  bool has = it != ls.end();
  switch (r.op) {
    case OpIn: return has && r.vals.count(it->second);
    case OpNotIn: return !has || !r.vals.count(it->second);
    case OpExists: return has;
    case OpDoesNotExist: return !has;
    case OpGt:
    case OpLt: {
      if (!has) return false;
      i64 v;
      if (!go_parse_int64(it->second, v)) return false;
      return r.op == OpGt ? v > r.num : v < r.num;
    }
  }
  return false;
}

// labels.Selector: Nothing (nil LabelSelector) or a requirement list (empty = Everything).
struct Selector {
  bool nothing = true;
  vector<Req> reqs;
  bool empty() const { return !nothing && reqs.empty(); }
  bool matches(const Labels& ls) const {
    if (nothing) return false;
    for (auto& r : reqs)
      if (!req_matches(r, ls)) return false;
    return true;
  }
};

// labels.NewRequirement validation (value-count rules + Gt/Lt integer parse).
static bool make_req(const string& key, const string& op, const vector<string>& vals, Req& out) {
  out.key = key;
  if (key.empty()) return false;
  if (op == "In" || op == "NotIn") {
    if (vals.empty()) return false;
    out.op = op == "In" ? OpIn : OpNotIn;
  } else if (op == "Exists" || op == "DoesNotExist") {
    if (!vals.empty()) return false;
    out.op = op == "Exists" ? OpExists : OpDoesNotExist;
  } else if (op == "Gt" || op == "Lt") {
    if (vals.size() != 1) return false;
    if (!go_parse_int64(vals[0], out.num)) return false;
    out.op = op == "Gt" ? OpGt : OpLt;
  } else {
    return false;
  }
  out.vals.insert(vals.begin(), vals.end());
  return true;
}

static vector<string> str_list(const ojson::Value* v) {
  vector<string> o;
  if (v && v->kind == ojson::Value::Arr)
    for (auto& e : v->arr) o.push_back(e.str());
  return o;
}
static Labels str_map(const ojson::Value* v) {
  Labels o;
  if (v && v->kind == ojson::Value::Obj)
    for (auto& kv : v->obj) o[kv.first] = kv.second.str();
  return o;
}

// metav1.LabelSelectorAsSelector
static bool label_selector(const ojson::Value* v, Selector& out) {
  out = Selector();
  if (!v || v->is_null()) return true;  // Nothing
  out.nothing = false;
  Labels ml = str_map(v->get("matchLabels"));
  for (auto& kv : ml) {
    Req r;
    if (!make_req(kv.first, "In", {kv.second}, r)) return false;
    out.reqs.push_back(r);
  }
  if (auto* ex = v->get("matchExpressions")) {
    for (auto& e : ex->arr) {
      string op = e.get("operator") ? e.get("operator")->str() : "";
      if (op != "In" && op != "NotIn" && op != "Exists" && op != "DoesNotExist") return false;
      Req r;
      if (!make_req(e.get("key") ? e.get("key")->str() : "", op, str_list(e.get("values")), r)) return false;
      out.reqs.push_back(r);
    }
  }
  return true;
}

// ============================================================ node affinity (component-helpers)
struct FieldReq {
  string key;
  bool eq;
  string val;
};
struct NodeSelTerm {
  bool err = false;
  bool has_labels = false;  // matchLabels != nil (len(MatchExpressions) != 0)
  Selector labels;
  bool has_fields = false;
  vector<FieldReq> fields;
  bool match(const Labels& ls, const string& node_name) const {
    if (has_labels && !labels.matches(ls)) return false;
    if (has_fields) {
      for (auto& f : fields) {
        string v = f.key == "metadata.name" ? node_name : "";
        if (f.eq ? v != f.val : v == f.val) return false;
      }
    }
    return true;
  }
};

static bool term_is_empty(const ojson::Value& t) {
  auto* me = t.get("matchExpressions");
  auto* mf = t.get("matchFields");
  return (!me || me->arr.empty()) && (!mf || mf->arr.empty());
}

static NodeSelTerm parse_node_term(const ojson::Value& t) {
  NodeSelTerm o;
  auto* me = t.get("matchExpressions");
  if (me && !me->arr.empty()) {
    o.has_labels = true;
    o.labels.nothing = false;
    for (auto& e : me->arr) {
      Req r;
      string op = e.get("operator") ? e.get("operator")->str() : "";
      if (!make_req(e.get("key") ? e.get("key")->str() : "", op, str_list(e.get("values")), r)) {
        o.err = true;
        continue;
      }
      o.labels.reqs.push_back(r);
    }
  }
  auto* mf = t.get("matchFields");
  if (mf && !mf->arr.empty()) {
    o.has_fields = true;
    for (auto& e : mf->arr) {
      string op = e.get("operator") ? e.get("operator")->str() : "";
      vector<string> vals = str_list(e.get("values"));
      if ((op != "In" && op != "NotIn") || vals.size() != 1) {
        o.err = true;
        continue;
      }
      o.fields.push_back({e.get("key") ? e.get("key")->str() : "", op == "In", vals[0]});
    }
  }
  return o;
}

struct RequiredNodeAffinity {
  bool has_label_sel = false;
  Selector label_sel;
  bool has_node_sel = false;
  vector<NodeSelTerm> terms;
  bool match(const Labels& ls, const string& name) const {
    if (has_label_sel && !label_sel.matches(ls)) return false;
    if (has_node_sel) {
      for (auto& t : terms) {
        if (t.err) continue;
        if (t.match(ls, name)) return true;
      }
      return false;
    }
    return true;
  }
};

struct PrefTerm {
  NodeSelTerm term;
  i64 weight;
};

// ============================================================ API objects
struct Taint {
  string key, value, effect;
};
struct Toleration {
  string key, op, value, effect;
  bool tolerates(const Taint& t) const {  // k8s.io/api core/v1 toleration.go ToleratesTaint
    if (!effect.empty() && effect != t.effect) return false;
    if (!key.empty() && key != t.key) return false;
    if (op.empty() || op == "Equal") return value == t.value;
    if (op == "Exists") return true;
    return false;
  }
};
static bool tolerations_tolerate(const vector<Toleration>& tols, const Taint& t) {
  for (auto& x : tols)
    if (x.tolerates(t)) return true;
  return false;
}

struct Resource {
  i64 milli_cpu = 0, memory = 0, eph = 0, allowed_pods = 0;
  map<string, i64> scalar;
};
static bool is_scalar_name(const string& n) {
  return n.find('/') != string::npos || n.rfind("hugepages-", 0) == 0;
}
static void resource_add(Resource& r, const ResourceList& rl) {  // framework.Resource.Add
  for (auto& kv : rl) {
    if (kv.first == "cpu") r.milli_cpu += q_milli(kv.second);
    else if (kv.first == "memory") r.memory += q_value(kv.second);
    else if (kv.first == "pods") r.allowed_pods += q_value(kv.second);
    else if (kv.first == "ephemeral-storage") r.eph += q_value(kv.second);
    else if (is_scalar_name(kv.first)) r.scalar[kv.first] += q_value(kv.second);
  }
}

struct AffTerm {
  set<string> namespaces;
  Selector ns_selector;
  Selector selector;
  string topology_key;
  bool matches(const Labels& pod_labels, const string& pod_ns, const Labels* ns_labels) const {
    static const Labels kEmpty;
    if (namespaces.count(pod_ns) || ns_selector.matches(ns_labels ? *ns_labels : kEmpty))
      return selector.matches(pod_labels);
    return false;
  }
};
struct WAffTerm {
  AffTerm t;
  int32_t weight;
};

struct TSC {
  int32_t max_skew;
  string key;
  string when;
  const ojson::Value* selector_json = nullptr;
  bool has_min_domains = false;
  int32_t min_domains = 1;
  string node_affinity_policy, node_taints_policy;
  vector<string> match_label_keys;
};

struct HostPort {  // v1.ContainerPort with hostPort > 0, sanitised (HostPortInfo.sanitize)
  string ip, proto;
  int32_t port;
};
struct Container {
  ResourceList requests;
  bool restart_always = false;
  string image;
  vector<HostPort> ports;
};

struct Pod {
  string name, ns;
  Labels labels;
  string node_name;
  bool terminating = false;
  vector<Container> containers, init_containers;
  ResourceList overhead;
  bool has_node_selector = false;
  Labels node_selector;
  vector<Toleration> tolerations;
  // node affinity
  bool has_required_na = false;
  vector<const ojson::Value*> required_terms;
  bool has_preferred_na = false;
  vector<const ojson::Value*> preferred_terms;
  // pod (anti)affinity
  bool has_pod_affinity = false, has_pod_anti_affinity = false;
  vector<AffTerm> req_aff, req_anti;
  vector<WAffTerm> pref_aff, pref_anti;
  bool pref_aff_present = false, pref_anti_present = false;  // for hasConstraints
  vector<TSC> tsc;
  bool volume_plugins_act = false;  // a volume other than a PVC the volume plugins act on (unsupported)
  vector<string> claims;            // persistentVolumeClaim.claimName of spec.volumes, in order
  i64 priority = 0;
  bool gated = false;               // spec.schedulingGates non-empty (SchedulingGates PreEnqueue)
  bool preempt_never = false;       // spec.preemptionPolicy: Never
  i64 start_time = INT64_MAX;       // status.startTime (epoch s); none: later than any (util.GetPodStartTime: now)
};

struct NodeImage {
  vector<string> names;
  i64 size = 0;
};
struct Node {
  string name;
  Labels labels;
  vector<Taint> taints;
  Resource alloc;
  vector<string> alloc_raw;  // allocatable resource names
  map<string, i64> attach_alloc;  // attachable-volumes-* allocatable (volume attach limits)
  bool unschedulable = false;
  vector<NodeImage> images;
};

// ============================================================ parsing
static ResourceList parse_rl(const ojson::Value* v) {
  ResourceList rl;
  if (v && v->kind == ojson::Value::Obj)
    for (auto& kv : v->obj) {
      i128 q;
      if (parse_quantity(kv.second.str(), q)) rl[kv.first] = q;
    }
  return rl;
}

static AffTerm parse_aff_term(const ojson::Value& t, const string& owner_ns, bool& err) {
  AffTerm a;
  if (!label_selector(t.get("labelSelector"), a.selector)) err = true;
  vector<string> nss = str_list(t.get("namespaces"));
  auto* nsSel = t.get("namespaceSelector");
  bool ns_sel_nil = !nsSel || nsSel->is_null();
  if (nss.empty() && ns_sel_nil) a.namespaces.insert(owner_ns);
  else a.namespaces.insert(nss.begin(), nss.end());
  if (!label_selector(nsSel, a.ns_selector)) err = true;
  a.topology_key = t.get("topologyKey") ? t.get("topologyKey")->str() : "";
  return a;
}

// "YYYY-MM-DDTHH:MM:SSZ" -> seconds since the epoch (days from civil, proleptic Gregorian)
static i64 parse_rfc3339(const string& s) {
  int Y, M, D, h, m, sec;
  if (std::sscanf(s.c_str(), "%d-%d-%dT%d:%d:%d", &Y, &M, &D, &h, &m, &sec) != 6) return INT64_MAX;
  Y -= M <= 2;
  const i64 era = (Y >= 0 ? Y : Y - 399) / 400;
  const i64 yoe = Y - era * 400;
  const i64 doy = (153 * (M + (M > 2 ? -3 : 9)) + 2) / 5 + D - 1;
  const i64 doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return (era * 146097 + doe - 719468) * 86400 + h * 3600 + m * 60 + sec;
}

static bool parse_pod(const ojson::Value& v, Pod& p) {
  bool err = false;
  auto* md = v.get("metadata");
  auto* sp = v.get("spec");
  p.name = md && md->get("name") ? md->get("name")->str() : "";
  p.ns = md && md->get("namespace") ? md->get("namespace")->str() : "default";
  if (p.ns.empty()) p.ns = "default";
  p.labels = str_map(md ? md->get("labels") : nullptr);
  p.terminating = md && md->get("deletionTimestamp") && !md->get("deletionTimestamp")->is_null();
  if (!sp) return true;
  p.node_name = sp->get("nodeName") ? sp->get("nodeName")->str() : "";
  if (auto* pr = sp->get("priority"); pr && !pr->is_null()) p.priority = pr->i64();
  if (auto* g = sp->get("schedulingGates"); g && !g->is_null() && !g->arr.empty()) p.gated = true;
  if (auto* pp = sp->get("preemptionPolicy"); pp && !pp->is_null()) p.preempt_never = pp->str() == "Never";
  if (auto* st = v.get("status"))
    if (auto* t = st->get("startTime"); t && !t->is_null()) p.start_time = parse_rfc3339(t->str());
  auto conts = [](const ojson::Value* a, vector<Container>& out) {
    if (!a) return;
    for (auto& c : a->arr) {
      Container k;
      auto* res = c.get("resources");
      k.requests = parse_rl(res ? res->get("requests") : nullptr);
      k.restart_always = c.get("restartPolicy") && c.get("restartPolicy")->str() == "Always";
      k.image = c.get("image") ? c.get("image")->str() : "";
      if (auto* ps = c.get("ports"))
        for (auto& x : ps->arr) {
          i64 hp = x.get("hostPort") ? x.get("hostPort")->i64() : 0;
          if (hp <= 0) continue;  // node_ports.go getContainerPorts: host ports only
          HostPort h{x.get("hostIP") ? x.get("hostIP")->str() : "", x.get("protocol") ? x.get("protocol")->str() : "",
                     (int32_t)hp};
          if (h.ip.empty()) h.ip = "0.0.0.0";  // HostPortInfo.sanitize
          if (h.proto.empty()) h.proto = "TCP";
          k.ports.push_back(h);
        }
      out.push_back(k);
    }
  };
  conts(sp->get("containers"), p.containers);
  conts(sp->get("initContainers"), p.init_containers);
  for (auto& c : p.init_containers) c.ports.clear();  // v1.30: Spec.Containers only (getContainerPorts, updateUsedPorts)
  if (auto* vs = sp->get("volumes"))
    for (auto& v : vs->arr) {
      auto* pvc = v.get("persistentVolumeClaim");
      if (pvc && !pvc->is_null()) p.claims.push_back(pvc->get("claimName") ? pvc->get("claimName")->str() : "");
      for (const char* k : {"ephemeral", "gcePersistentDisk", "awsElasticBlockStore", "rbd", "iscsi", "azureDisk",
                            "cinder", "csi"})
        if (v.get(k) && !v.get(k)->is_null()) p.volume_plugins_act = true;
    }
  p.overhead = parse_rl(sp->get("overhead"));
  if (auto* ns = sp->get("nodeSelector"); ns && !ns->is_null()) {
    p.has_node_selector = true;
    p.node_selector = str_map(ns);
  }
  if (auto* tl = sp->get("tolerations"))
    for (auto& t : tl->arr) {
      Toleration x;
      x.key = t.get("key") ? t.get("key")->str() : "";
      x.op = t.get("operator") ? t.get("operator")->str() : "";
      x.value = t.get("value") ? t.get("value")->str() : "";
      x.effect = t.get("effect") ? t.get("effect")->str() : "";
      p.tolerations.push_back(x);
    }
  if (auto* aff = sp->get("affinity"); aff && !aff->is_null()) {
    if (auto* na = aff->get("nodeAffinity"); na && !na->is_null()) {
      if (auto* rq = na->get("requiredDuringSchedulingIgnoredDuringExecution"); rq && !rq->is_null()) {
        p.has_required_na = true;
        if (auto* terms = rq->get("nodeSelectorTerms"))
          for (auto& t : terms->arr) p.required_terms.push_back(&t);
      }
      if (auto* pf = na->get("preferredDuringSchedulingIgnoredDuringExecution"); pf && !pf->is_null()) {
        p.has_preferred_na = true;
        for (auto& t : pf->arr) p.preferred_terms.push_back(&t);
      }
    }
    auto pa = [&](const char* k, bool& present, vector<AffTerm>& req, vector<WAffTerm>& pref, bool& pref_present) {
      auto* x = aff->get(k);
      if (!x || x->is_null()) return;
      present = true;
      if (auto* rq = x->get("requiredDuringSchedulingIgnoredDuringExecution"))
        for (auto& t : rq->arr) req.push_back(parse_aff_term(t, p.ns, err));
      if (auto* pf = x->get("preferredDuringSchedulingIgnoredDuringExecution"); pf && !pf->is_null()) {
        pref_present = !pf->arr.empty();
        for (auto& t : pf->arr) {
          WAffTerm w;
          w.weight = (int32_t)(t.get("weight") ? t.get("weight")->i64() : 0);
          auto* pt = t.get("podAffinityTerm");
          if (pt) w.t = parse_aff_term(*pt, p.ns, err);
          pref.push_back(w);
        }
      }
    };
    pa("podAffinity", p.has_pod_affinity, p.req_aff, p.pref_aff, p.pref_aff_present);
    pa("podAntiAffinity", p.has_pod_anti_affinity, p.req_anti, p.pref_anti, p.pref_anti_present);
  }
  if (auto* ts = sp->get("topologySpreadConstraints"))
    for (auto& c : ts->arr) {
      TSC t;
      t.max_skew = (int32_t)(c.get("maxSkew") ? c.get("maxSkew")->i64() : 0);
      t.key = c.get("topologyKey") ? c.get("topologyKey")->str() : "";
      t.when = c.get("whenUnsatisfiable") ? c.get("whenUnsatisfiable")->str() : "";
      t.selector_json = c.get("labelSelector");
      if (auto* md2 = c.get("minDomains"); md2 && !md2->is_null()) {
        t.has_min_domains = true;
        t.min_domains = (int32_t)md2->i64();
      }
      t.node_affinity_policy = c.get("nodeAffinityPolicy") ? c.get("nodeAffinityPolicy")->str() : "";
      t.node_taints_policy = c.get("nodeTaintsPolicy") ? c.get("nodeTaintsPolicy")->str() : "";
      t.match_label_keys = str_list(c.get("matchLabelKeys"));
      p.tsc.push_back(t);
    }
  return !err;
}

static void parse_node(const ojson::Value& v, Node& n) {
  auto* md = v.get("metadata");
  n.name = md && md->get("name") ? md->get("name")->str() : "";
  n.labels = str_map(md ? md->get("labels") : nullptr);
  if (auto* sp = v.get("spec"))
    if (auto* ts = sp->get("taints"))
      for (auto& t : ts->arr)
        n.taints.push_back({t.get("key") ? t.get("key")->str() : "", t.get("value") ? t.get("value")->str() : "",
                            t.get("effect") ? t.get("effect")->str() : ""});
  if (auto* sp = v.get("spec"))
    if (auto* u = sp->get("unschedulable")) n.unschedulable = u->b;
  auto* st = v.get("status");
  resource_add(n.alloc, parse_rl(st ? st->get("allocatable") : nullptr));
  if (auto* al = st ? st->get("allocatable") : nullptr)
    for (auto& kv : al->obj) {
      n.alloc_raw.push_back(kv.first);
      i128 q;
      if (kv.first.rfind("attachable-volumes-", 0) == 0 && parse_quantity(kv.second.str(), q))
        n.attach_alloc[kv.first] = (i64)(q / 1000000000);  // (quantity in nano units)
    }
  if (st)
    if (auto* im = st->get("images"))
      for (auto& x : im->arr) {
        NodeImage ni;
        ni.names = str_list(x.get("names"));
        ni.size = x.get("sizeBytes") ? x.get("sizeBytes")->i64() : 0;
        n.images.push_back(ni);
      }
}

// ============================================================ resource helpers (PodRequests)
static void add_rl(ResourceList& a, const ResourceList& b) {
  for (auto& kv : b) a[kv.first] += kv.second;
}
static void max_rl(ResourceList& a, const ResourceList& b) {
  for (auto& kv : b) {
    auto it = a.find(kv.first);
    if (it == a.end() || kv.second > it->second) a[kv.first] = kv.second;
  }
}
static ResourceList apply_non_missing(const ResourceList& r, bool nonzero) {
  ResourceList o = r;
  if (nonzero) {
    if (!o.count("cpu")) o["cpu"] = (i128)kDefaultMilliCPU * 1000000;
    if (!o.count("memory")) o["memory"] = (i128)kDefaultMemory * 1000000000;
  }
  return o;
}
// resourcehelper.PodRequests (pkg/api/v1/resource/helpers.go) with optional
// NonMissingContainerRequests = {cpu: 100m, memory: 200Mi}.
static ResourceList pod_requests(const Pod& p, bool nonzero) {
  ResourceList reqs;
  for (auto& c : p.containers) add_rl(reqs, apply_non_missing(c.requests, nonzero));
  ResourceList restartable, init;
  for (auto& c : p.init_containers) {
    ResourceList cr = apply_non_missing(c.requests, nonzero);
    if (c.restart_always) {
      add_rl(reqs, cr);
      add_rl(restartable, cr);
      cr = restartable;
    } else {
      ResourceList tmp;
      add_rl(tmp, cr);
      add_rl(tmp, restartable);
      cr = tmp;
    }
    max_rl(init, cr);
  }
  max_rl(reqs, init);
  add_rl(reqs, p.overhead);
  return reqs;
}

// ============================================================ parallelize.Until
// Persistent worker pool (goroutines are cheap in Go; spawning OS threads per
// call would penalise the CPU baseline).  chunk = max(1, min(sqrt(n), n/workers+1))
// (framework/parallelize/parallelism.go chunkSizeFor).
struct Pool {
  int workers;
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  const std::function<void(int)>* fn = nullptr;
  int n = 0, chunk = 1;
  std::atomic<int> next{0};
  int active = 0;
  unsigned long long gen = 0;
  bool stop = false;
  explicit Pool(int w) : workers(w < 1 ? 1 : w) {
    for (int t = 1; t < workers; ++t) th.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  void work() {
    for (;;) {
      int s = next.fetch_add(chunk);
      if (s >= n) return;
      int e = std::min(n, s + chunk);
      for (int i = s; i < e; ++i) (*fn)(i);
    }
  }
  void loop() {
    unsigned long long seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
      }
      work();
      {
        std::lock_guard<std::mutex> g(mu);
        if (--active == 0) done_cv.notify_one();
      }
    }
  }
  void until(int count, const std::function<void(int)>& f) {
    if (count <= 0) return;
    if (workers == 1) {
      for (int i = 0; i < count; ++i) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu);
      fn = &f;
      n = count;
      chunk = std::max(1, std::min((int)std::sqrt((double)count), count / workers + 1));
      next = 0;
      active = workers - 1;
      ++gen;
    }
    cv.notify_all();
    work();
    std::unique_lock<std::mutex> g(mu);
    done_cv.wait(g, [&] { return active == 0; });
  }
};

// ============================================================ scheduler state
struct PodRecord {
  Pod pod;
  bool parse_ok = true;
  bool has_required_anti = false;
  bool with_affinity = false;
};

struct NodeInfo {
  Resource requested;
  i64 nz_cpu = 0, nz_mem = 0;
  vector<int> pods, pods_with_affinity, pods_with_req_anti;
  map<string, map<std::pair<string, int32_t>, int>> used_ports;  // HostPortInfo: ip -> (protocol, port)
};

struct ScoreSpec {
  string name;
  i64 weight;
};

// Volume plugins (PreFilter + Filter): P_VOLRESTRICT VolumeRestrictions,
// P_NONCSI EBSLimits / GCEPDLimits / AzureDiskLimits, P_CSILIMITS NodeVolumeLimits,
// P_VOLZONE VolumeZone, P_VOLBIND VolumeBinding (also PreScore, Skip with the
// default feature gates: no scorer).  P_NOOP: plugins with none of the recorded
// extension points.
enum PluginId { P_FIT, P_BA, P_TAINT, P_NA, P_PTS, P_IPA, P_UNSCHED, P_NODENAME, P_PORTS, P_IMAGE,
                P_VOLRESTRICT, P_NONCSI, P_CSILIMITS, P_VOLZONE, P_VOLBIND, P_NOOP, P_UNKNOWN };
static bool is_volume_plugin(PluginId p) { return p >= P_VOLRESTRICT && p <= P_VOLBIND; }
static PluginId plugin_id(const string& n) {
  if (n == "NodeResourcesFit") return P_FIT;
  if (n == "NodeResourcesBalancedAllocation") return P_BA;
  if (n == "TaintToleration") return P_TAINT;
  if (n == "NodeAffinity") return P_NA;
  if (n == "PodTopologySpread") return P_PTS;
  if (n == "InterPodAffinity") return P_IPA;
  if (n == "NodeUnschedulable") return P_UNSCHED;
  if (n == "NodeName") return P_NODENAME;
  if (n == "NodePorts") return P_PORTS;
  if (n == "ImageLocality") return P_IMAGE;
  if (n == "VolumeRestrictions") return P_VOLRESTRICT;
  if (n == "EBSLimits" || n == "GCEPDLimits" || n == "AzureDiskLimits") return P_NONCSI;
  if (n == "NodeVolumeLimits") return P_CSILIMITS;
  if (n == "VolumeZone") return P_VOLZONE;
  if (n == "VolumeBinding") return P_VOLBIND;
  if (n == "PrioritySort" || n == "SchedulingGates" || n == "DefaultPreemption" || n == "DefaultBinder") return P_NOOP;
  return P_UNKNOWN;
}
static bool has_prefilter(PluginId p) {
  return p == P_FIT || p == P_NA || p == P_PTS || p == P_IPA || p == P_PORTS || is_volume_plugin(p);
}
static bool has_filter(PluginId p) {
  return p == P_FIT || p == P_TAINT || p == P_NA || p == P_PTS || p == P_IPA || p == P_UNSCHED || p == P_NODENAME ||
         p == P_PORTS || is_volume_plugin(p);
}
static bool has_prescore(PluginId p) { return p <= P_IPA || p == P_VOLBIND; }
static bool has_score(PluginId p) { return p <= P_IPA || p == P_IMAGE || p == P_VOLBIND; }
static bool has_score_ext(PluginId p) { return p == P_TAINT || p == P_NA || p == P_PTS || p == P_IPA; }

struct ResSpec {
  string name;
  i64 weight;
};

struct Status {
  enum Code { Success, Error, Unschedulable, UnschedulableAndUnresolvable, Skip } code = Success;
  string msg;
  bool ok() const { return code == Success; }
  static Status skip() { return {Skip, ""}; }
};

struct PodResult {
  string selected;
  int selected_idx = -1;
  int feasible = 0;
  int status = 0;  // 0 scheduled, 1 unschedulable, 2 error
  // store maps (resultstore/store.go result)
  map<string, string> pre_filter_status, pre_score;
  vector<string> post_filter_nodes;  // DefaultPreemption: nodes of the NodeToStatusMap
  string nominated, preempt_plugin;  // DefaultPreemption dry run: the nominated node, and the plugin's name
  int nominated_idx = -1;
  vector<string> victims;            // ... and its victims ("namespace/name", most important first)
  map<string, string> reserve, prebind, bind;  // binding cycle of a scheduled pod (bind assumed to succeed)
  map<string, vector<string>> pre_filter_result;
  std::unordered_map<string, std::unordered_map<string, string>> filter, score, final_score;
};

// ============================================================ JSON rendering (Go encoding/json)
static void go_json_string(string& o, const string& s) {
  static const char* hex = "0123456789abcdef";
  o += '"';
  for (size_t i = 0; i < s.size(); ++i) {
    unsigned char c = s[i];
    if (c == '"') o += "\\\"";
    else if (c == '\\') o += "\\\\";
    else if (c == '\n') o += "\\n";
    else if (c == '\r') o += "\\r";
    else if (c == '\t') o += "\\t";
    else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
      o += "\\u00";
      o += hex[c >> 4];
      o += hex[c & 15];
    } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
               ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
      o += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
      i += 2;
    } else o += (char)c;
  }
  o += '"';
}
static string json_map(const map<string, string>& m) {
  string o = "{";
  bool first = true;
  for (auto& kv : m) {
    if (!first) o += ',';
    first = false;
    go_json_string(o, kv.first);
    o += ':';
    go_json_string(o, kv.second);
  }
  return o + "}";
}
static string json_map2(const std::unordered_map<string, std::unordered_map<string, string>>& um) {
  map<string, map<string, string>> m;  // encoding/json sorts map keys
  for (auto& kv : um) m[kv.first] = map<string, string>(kv.second.begin(), kv.second.end());
  string o = "{";
  bool first = true;
  for (auto& kv : m) {
    if (!first) o += ',';
    first = false;
    go_json_string(o, kv.first);
    o += ':';
    o += json_map(kv.second);
  }
  return o + "}";
}
static string json_map_list(const map<string, vector<string>>& m) {
  string o = "{";
  bool first = true;
  for (auto& kv : m) {
    if (!first) o += ',';
    first = false;
    go_json_string(o, kv.first);
    o += ":[";
    vector<string> v = kv.second;
    std::sort(v.begin(), v.end());  // UnsortedList(): order is random upstream; compared as a set
    for (size_t i = 0; i < v.size(); ++i) {
      if (i) o += ',';
      go_json_string(o, v[i]);
    }
    o += ']';
  }
  return o + "}";
}

static const char* kAnnPrefix = "kube-scheduler-simulator.sigs.k8s.io/";

// Store.GetStoredResult (resultstore/store.go:133-198): every key, "{}" when empty.
static string render_annotations(const PodResult& r) {
  map<string, string> ann;
  auto k = [](const char* s) { return string(kAnnPrefix) + s; };
  ann[k("prefilter-result")] = json_map_list(r.pre_filter_result);
  ann[k("prefilter-result-status")] = json_map(r.pre_filter_status);
  ann[k("filter-result")] = json_map2(r.filter);
  {  // Store.AddPostFilterResult: every node of the status map gets an (empty) entry
    map<string, map<string, string>> pf;
    for (auto& n : r.post_filter_nodes) pf[n];
    if (!r.nominated.empty()) pf[r.nominated][r.preempt_plugin] = "preemption victim";  // PostFilterNominatedMessage
    string o = "{";
    for (auto& kv : pf) {
      if (o.size() > 1) o += ',';
      go_json_string(o, kv.first);
      o += ':';
      o += json_map(kv.second);
    }
    ann[k("postfilter-result")] = o + "}";
  }
  ann[k("prescore-result")] = json_map(r.pre_score);
  ann[k("score-result")] = json_map2(r.score);
  ann[k("finalscore-result")] = json_map2(r.final_score);
  ann[k("reserve-result")] = json_map(r.reserve);
  ann[k("permit-result")] = "{}";
  ann[k("permit-result-timeout")] = "{}";
  ann[k("prebind-result")] = json_map(r.prebind);
  ann[k("bind-result")] = json_map(r.bind);
  ann[k("selected-node")] = r.selected;
  return json_map(ann);
}

// ============================================================ storage (volume plugins)
// ResourcesForSnap pvs / pvcs / storageClasses as v1.30.4's volume plugins read
// them (GetPersistentVolumeClaimClass / GetPersistentVolumeClass: the beta
// annotation wins over spec.storageClassName).
struct ClaimObj {
  string ns, name, volume_name, class_name;
  bool bind_completed = false, deleting = false, lost = false, rwop = false;
  bool has_selected_node = false;
  string selected_node;
};
struct VolumeObj {
  string name, class_name;
  Labels labels;
  bool has_required = false;       // spec.nodeAffinity.required
  vector<NodeSelTerm> required;    // its terms (empty / invalid ones never match)
  vector<bool> required_empty;
  bool claim_ref = false;
  string ref_ns, ref_name;
  bool intree = false;
  bool csi = false;                // spec.csi
  string csi_driver, csi_handle;
  const ojson::Value* required_json = nullptr;
};
struct ClassObj {
  string name, provisioner;
  bool mode_set = false, wait_for_consumer = false;
  vector<vector<std::pair<string, vector<string>>>> topology;  // allowedTopologies terms (label expressions)
};
static const char* kVolumeZoneLabels[4] = {"failure-domain.beta.kubernetes.io/zone",
                                           "failure-domain.beta.kubernetes.io/region",
                                           "topology.kubernetes.io/zone", "topology.kubernetes.io/region"};

// ============================================================ the simulator
struct Cluster;

struct CycleState {
  // NodeResourcesFit
  ResourceList fit_req;  // preFilterState (PodRequests)
  Resource fit_req_res;
  vector<i64> fit_score_req;  // preScoreState.podRequests per scoring resource
  vector<i64> ba_req;
  // NodeAffinity
  RequiredNodeAffinity na_required;
  vector<PrefTerm> na_pref;
  bool na_pref_err = false;
  // TaintToleration
  vector<Toleration> taint_prefer_tols;
  // PodTopologySpread filter
  struct TsConstraint {
    int32_t max_skew;
    string key;
    Selector sel;
    int32_t min_domains;
    bool honor_affinity, honor_taints;
  };
  vector<TsConstraint> pts_filter;
  map<std::pair<string, string>, i64> pts_pair_num;
  map<string, i64> pts_key_domains;
  map<string, i64> pts_key_min;
  // PodTopologySpread score
  vector<TsConstraint> pts_score;
  set<string> pts_ignored;
  map<std::pair<string, string>, i64> pts_pair_counts;
  vector<double> pts_weight;
  // InterPodAffinity
  vector<AffTerm> ipa_req_aff, ipa_req_anti;
  map<std::pair<string, string>, i64> ipa_existing_anti, ipa_aff_counts, ipa_anti_counts;
  vector<WAffTerm> ipa_pref_aff, ipa_pref_anti;
  map<string, map<string, i64>> ipa_topo_score;
  // NodePorts preFilterState (getContainerPorts)
  vector<HostPort> ports_want;
  // VolumeRestrictions preFilterState.conflictingPVCRefCount
  int vr_conflicts = 0;
  // VolumeBinding stateData.podVolumeClaims
  vector<const ClaimObj*> vb_bound, vb_delayed;
  // VolumeZone stateData.podPVTopologies
  vector<std::pair<string, set<string>>> vz_topologies;
};

static const i64 kMB = 1024 * 1024;
static const i64 kImgMinThreshold = 23 * kMB;            // image_locality.go minThreshold
static const i64 kImgMaxContainerThreshold = 1000 * kMB;  // maxContainerThreshold
// image_locality.go normalizedImageName
static string normalized_image_name(const string& n) {
  size_t c = n.rfind(':'), sl = n.rfind('/');
  long ci = c == string::npos ? -1 : (long)c, si = sl == string::npos ? -1 : (long)sl;
  return ci <= si ? n + ":latest" : n;
}

struct Cluster {
  std::unique_ptr<ojson::Value> doc;
  vector<Node> nodes;
  std::unordered_map<string, int> node_index;
  vector<NodeInfo> infos;
  vector<PodRecord> pods;  // bound + queue
  vector<int> queue;       // scheduling order (PrioritySort)
  vector<int> gated;       // held back by SchedulingGates' PreEnqueue
  set<string> namespaces;
  // profile
  vector<PluginId> profile;  // MultiPoint order
  vector<string> profile_names;
  map<string, i64> fw_weight, store_weight;
  string fit_strategy = "LeastAllocated";
  vector<ResSpec> fit_res{{"cpu", 1}, {"memory", 1}};
  vector<std::pair<i64, i64>> rtc_shape;  // (utilization, score)
  vector<ResSpec> ba_res{{"cpu", 1}, {"memory", 1}};
  i64 ipa_hard_weight = 1;
  bool ipa_ignore_existing_pref = false;
  unsigned long long seed = 0;
  // ImageStateSummary per image name (size of the first node listing it, node count)
  std::unordered_map<string, std::pair<i64, int>> image_states;
  // storage objects (volume plugins) and NodeInfo.PVCRefCounts summed over the nodes
  map<string, ClaimObj> claims;  // "namespace/name"
  map<string, VolumeObj> volumes;
  map<string, ClassObj> classes;
  map<string, int> pvc_refs;
  map<string, map<string, i64>> csi_counts;  // CSINode: node -> driver -> spec.drivers[].allocatable.count
  // results
  vector<PodResult> results;
  std::mutex store_mu;

  // ---------------------------------------------------------------- assume
  // What-if batches (BASELINE cfg5): every pod of a step is scheduled against the
  // same snapshot; the step's placements are bound together afterwards.
  bool defer_assume = false;
  vector<std::pair<int, int>> deferred;
  void add_pod(int pi, int ni) {  // framework.NodeInfo.AddPod (+ calculateResource)
    NodeInfo& n = infos[ni];
    PodRecord& r = pods[pi];
    Resource res;
    resource_add(res, pod_requests(r.pod, false));
    ResourceList nz = pod_requests(r.pod, true);
    n.requested.milli_cpu += res.milli_cpu;
    n.requested.memory += res.memory;
    n.requested.eph += res.eph;
    for (auto& kv : res.scalar) n.requested.scalar[kv.first] += kv.second;
    n.nz_cpu += nz.count("cpu") ? q_milli(nz["cpu"]) : 0;
    n.nz_mem += nz.count("memory") ? q_value(nz["memory"]) : 0;
    n.pods.push_back(pi);
    for (auto& c : r.pod.containers)  // NodeInfo.updateUsedPorts
      for (auto& h : c.ports) n.used_ports[h.ip][{h.proto, h.port}]++;
    if (r.with_affinity) n.pods_with_affinity.push_back(pi);
    if (r.has_required_anti) n.pods_with_req_anti.push_back(pi);
    for (auto& c : r.pod.claims) pvc_refs[r.pod.ns + "/" + c] += 1;  // updatePVCRefCounts
  }

  void remove_pod(int pi, int ni) {  // framework.NodeInfo.RemovePod
    NodeInfo& n = infos[ni];
    PodRecord& r = pods[pi];
    Resource res;
    resource_add(res, pod_requests(r.pod, false));
    ResourceList nz = pod_requests(r.pod, true);
    n.requested.milli_cpu -= res.milli_cpu;
    n.requested.memory -= res.memory;
    n.requested.eph -= res.eph;
    for (auto& kv : res.scalar) n.requested.scalar[kv.first] -= kv.second;
    n.nz_cpu -= nz.count("cpu") ? q_milli(nz["cpu"]) : 0;
    n.nz_mem -= nz.count("memory") ? q_value(nz["memory"]) : 0;
    auto drop = [pi](vector<int>& v) {
      auto it = std::find(v.begin(), v.end(), pi);
      if (it != v.end()) v.erase(it);
    };
    drop(n.pods);
    drop(n.pods_with_affinity);
    drop(n.pods_with_req_anti);
    for (auto& c : r.pod.containers)
      for (auto& h : c.ports) {
        auto& m = n.used_ports[h.ip];
        if (--m[{h.proto, h.port}] <= 0) m.erase({h.proto, h.port});
        if (m.empty()) n.used_ports.erase(h.ip);
      }
    for (auto& c : r.pod.claims) {
      const string key = r.pod.ns + "/" + c;
      if (--pvc_refs[key] <= 0) pvc_refs.erase(key);
    }
  }

  // ---------------------------------------------------------------- volume plugins (v1.30.4)
  const ClaimObj* find_claim(const string& ns, const string& name) const {
    auto it = claims.find(ns + "/" + name);
    return it == claims.end() ? nullptr : &it->second;
  }
  static Status unresolvable(const string& m) { return {Status::UnschedulableAndUnresolvable, m}; }
  // volumerestrictions PreFilter: readWriteOncePodPVCsForPod + calPreFilterState
  // (needsRestrictionsCheck: any PVC volume; inline disks are refused at load)
  Status vr_prefilter(const Pod& p, CycleState& cs) const {
    set<string> rwop;
    for (auto& cn : p.claims) {
      const ClaimObj* c = find_claim(p.ns, cn);
      if (!c) return unresolvable("persistentvolumeclaim \"" + cn + "\" not found");
      if (c->rwop) rwop.insert(c->name);
    }
    int conflicts = 0;
    for (auto& n : rwop)
      if (pvc_refs.count(p.ns + "/" + n)) conflicts++;  // StorageInfos().IsPVCUsedByPods
    if (p.claims.empty() && conflicts == 0) return Status::skip();
    cs.vr_conflicts = conflicts;
    return {};
  }
  Status vr_filter(const CycleState& cs) const {  // satisfyReadWriteOncePod
    if (cs.vr_conflicts != 0)
      return {Status::Unschedulable,
              "node has pod using PersistentVolumeClaim with the same name and ReadWriteOncePod access mode"};
    return {};
  }
  // nodevolumelimits non_csi.go / csi.go PreFilter: Skip without a PVC (the claims
  // accepted at load bring no volume either counts against a limit: Filter passes)
  static Status limits_prefilter(const Pod& p) { return p.claims.empty() ? Status::skip() : Status{}; }
  // nodevolumelimits csi.go: volumeutil.GetCSIAttachLimitKey (keys of 63+ characters,
  // which it hashes, are refused at load)
  static string csi_limit_key(const string& driver) { return "attachable-volumes-csi-" + driver; }
  // filterAttachableVolumes: unique volume name (driver/handle) -> limit key of the pod's
  // CSI volumes; an unbound claim (or one whose PV is missing) counts by its class's
  // provisioner and the claim's name (getCSIDriverInfoFromSC's handle)
  void attachable_volumes(const Pod& p, map<string, string>& out) const {
    for (auto& cn : p.claims) {
      const ClaimObj* c = find_claim(p.ns, cn);
      if (!c) continue;
      string driver, handle;
      auto from_class = [&] {
        if (c->class_name.empty()) return;
        auto k = classes.find(c->class_name);
        if (k == classes.end()) return;
        driver = k->second.provisioner;
        handle = "ksg-" + c->ns + "/" + c->name;
      };
      auto v = c->volume_name.empty() ? volumes.end() : volumes.find(c->volume_name);
      if (c->volume_name.empty() || v == volumes.end()) from_class();
      else if (v->second.csi) {
        driver = v->second.csi_driver;
        handle = v->second.csi_handle;
      }
      if (driver.empty() || handle.empty()) continue;
      out[driver + "/" + handle] = csi_limit_key(driver);
    }
  }
  // getVolumeLimits: attachable-volumes-* of the node's allocatable, CSINode counts over them
  map<string, i64> volume_limits(int ni) const {
    map<string, i64> lim = nodes[ni].attach_alloc;
    auto it = csi_counts.find(nodes[ni].name);
    if (it != csi_counts.end())
      for (auto& kv : it->second) lim[csi_limit_key(kv.first)] = kv.second;
    return lim;
  }
  Status csi_filter(const Pod& p, int ni) const {
    map<string, string> fresh, attached;
    attachable_volumes(p, fresh);
    if (fresh.empty()) return {};
    const map<string, i64> lim = volume_limits(ni);
    if (lim.empty()) return {};
    for (int pi : infos[ni].pods) attachable_volumes(pods[pi].pod, attached);
    map<string, int> have, want;
    for (auto& kv : attached) {
      fresh.erase(kv.first);  // a volume already attached is not counted twice
      have[kv.second]++;
    }
    for (auto& kv : fresh) want[kv.second]++;
    for (auto& kv : want) {
      auto l = lim.find(kv.first);
      if (l != lim.end() && have[kv.first] + kv.second > l->second)
        return {Status::Unschedulable, "node(s) exceed max volume count"};
    }
    return {};
  }
  // volume.GetLocalPersistentVolumeNodeNames
  static set<string> local_pv_nodes(const VolumeObj& v) {
    set<string> out;
    if (!v.has_required || !v.required_json) return out;
    if (auto* ts = v.required_json->get("nodeSelectorTerms"))
      for (auto& t : ts->arr) {
        std::unique_ptr<set<string>> nodes;
        if (auto* me = t.get("matchExpressions"))
          for (auto& e : me->arr) {
            if (!e.get("key") || e.get("key")->str() != "kubernetes.io/hostname") continue;
            if (!e.get("operator") || e.get("operator")->str() != "In") continue;
            vector<string> vs = str_list(e.get("values"));
            set<string> x(vs.begin(), vs.end());
            if (!nodes) nodes.reset(new set<string>(x));
            else {
              set<string> y;
              std::set_intersection(nodes->begin(), nodes->end(), x.begin(), x.end(), std::inserter(y, y.begin()));
              *nodes = y;
            }
          }
        if (nodes) out.insert(nodes->begin(), nodes->end());
      }
    return out;
  }
  // volume.CheckNodeAffinity: the node object carries only its labels
  static bool pv_affinity_match(const VolumeObj& v, const Labels& node_labels) {
    if (!v.has_required) return true;
    for (size_t i = 0; i < v.required.size(); ++i) {
      if (v.required_empty[i] || v.required[i].err) continue;
      if (v.required[i].match(node_labels, "")) return true;
    }
    return false;
  }
  // v1helper.MatchTopologySelectorTerms
  static bool topology_match(const ClassObj& k, const Labels& ls) {
    if (k.topology.empty()) return true;
    for (auto& term : k.topology) {
      if (term.empty()) continue;
      bool ok = true;
      for (auto& e : term) {
        auto it = ls.find(e.first);
        if (e.second.empty() || it == ls.end() || std::find(e.second.begin(), e.second.end(), it->second) == e.second.end()) {
          ok = false;
          break;
        }
      }
      if (ok) return true;
    }
    return false;
  }
  // volumebinding PreFilter: podHasPVCs, GetPodVolumeClaims, GetEligibleNodes
  Status vb_prefilter(const Pod& p, CycleState& cs, bool& has_res, vector<string>& res) const {
    if (p.claims.empty()) return Status::skip();
    for (auto& cn : p.claims) {
      const ClaimObj* c = find_claim(p.ns, cn);
      if (!c) return unresolvable("persistentvolumeclaim \"" + cn + "\" not found");
      if (c->lost)
        return unresolvable("persistentvolumeclaim \"" + c->name + "\" bound to non-existent persistentvolume \"" +
                            c->volume_name + "\"");
      if (c->deleting) return unresolvable("persistentvolumeclaim \"" + c->name + "\" is being deleted");
    }
    bool immediate = false;
    for (auto& cn : p.claims) {
      const ClaimObj* c = find_claim(p.ns, cn);
      if (!c->volume_name.empty() && c->bind_completed) {
        cs.vb_bound.push_back(c);
        continue;
      }
      bool delay = false;  // IsDelayBindingMode
      if (!c->class_name.empty()) {
        auto k = classes.find(c->class_name);
        delay = k != classes.end() && k->second.wait_for_consumer;
      }
      if (delay && c->volume_name.empty()) cs.vb_delayed.push_back(c);
      else immediate = true;
    }
    if (immediate) return unresolvable("pod has unbound immediate PersistentVolumeClaims");
    bool any = false, missing = false;
    set<string> elig;
    for (auto* c : cs.vb_bound) {
      auto it = volumes.find(c->volume_name);
      if (it == volumes.end()) { missing = true; continue; }
      set<string> nn = local_pv_nodes(it->second);
      if (nn.empty()) continue;
      if (!any) { elig = nn; any = true; continue; }
      set<string> y;
      std::set_intersection(elig.begin(), elig.end(), nn.begin(), nn.end(), std::inserter(y, y.begin()));
      elig = y;
    }
    if (any && !missing) {
      has_res = true;
      res.assign(elig.begin(), elig.end());
    }
    return {};
  }
  // volumebinding Filter -> binder.FindPodVolumes (static PV matching never applies:
  // refused at load; provisioning capacity: no CSIDriver objects, sufficient)
  Status vb_filter(const CycleState& cs, int ni) const {
    const Node& n = nodes[ni];
    bool bound_ok = true, found = true, unbound_ok = true;
    for (auto* c : cs.vb_bound) {  // checkBoundClaims
      auto it = volumes.find(c->volume_name);
      if (it == volumes.end()) { found = false; break; }
      if (!pv_affinity_match(it->second, n.labels)) { bound_ok = false; break; }
    }
    if (!cs.vb_delayed.empty()) {
      vector<const ClaimObj*> provision;
      for (auto* c : cs.vb_delayed)
        if (c->has_selected_node) {
          if (c->selected_node != n.name) { unbound_ok = false; break; }
          provision.push_back(c);
        }
      if (unbound_ok) {
        for (auto* c : cs.vb_delayed)
          if (!c->has_selected_node) provision.push_back(c);
        for (auto* c : provision) {  // checkVolumeProvisions
          const ClassObj& k = classes.at(c->class_name);
          if (k.provisioner.empty() || k.provisioner == "kubernetes.io/no-provisioner" || !topology_match(k, n.labels)) {
            unbound_ok = false;
            break;
          }
        }
      }
    }
    string m;
    auto reason = [&](const char* r) { m += (m.empty() ? "" : ", ") + string(r); };
    if (!bound_ok) reason("node(s) had volume node affinity conflict");
    if (!unbound_ok) reason("node(s) didn't find available persistent volumes to bind");
    if (!found) reason("node(s) unavailable due to one or more pvc(s) bound to non-existent pv(s)");
    if (m.empty()) return {};
    return unresolvable(m);
  }
  // volumezone PreFilter (getPVbyPod, getPVTopologies / LabelZonesToSet) and Filter
  Status vz_prefilter(const Pod& p, CycleState& cs) const {
    for (auto& cn : p.claims) {
      if (cn.empty()) return unresolvable("PersistentVolumeClaim had no name");
      const ClaimObj* c = find_claim(p.ns, cn);
      if (!c) return unresolvable("persistentvolumeclaim \"" + cn + "\" not found");
      if (c->volume_name.empty()) {
        if (c->class_name.empty()) return unresolvable("PersistentVolumeClaim had no pv name and storageClass name");
        auto k = classes.find(c->class_name);
        if (k == classes.end()) return unresolvable("storageclass.storage.k8s.io \"" + c->class_name + "\" not found");
        if (!k->second.mode_set) return unresolvable("VolumeBindingMode not set for StorageClass \"" + c->class_name + "\"");
        if (k->second.wait_for_consumer) continue;
        return unresolvable("PersistentVolume had no name");
      }
      auto v = volumes.find(c->volume_name);
      if (v == volumes.end()) return unresolvable("persistentvolume \"" + c->volume_name + "\" not found");
      for (const char* key : kVolumeZoneLabels) {
        auto it = v->second.labels.find(key);
        if (it == v->second.labels.end()) continue;
        set<string> zones;
        bool bad = false;
        string rest = it->second;
        for (;;) {
          size_t cut = rest.find("__");
          string z = rest.substr(0, cut);
          const char* ws = " \t\n\r\v\f";
          size_t a = z.find_first_not_of(ws);
          z = a == string::npos ? string() : z.substr(a, z.find_last_not_of(ws) - a + 1);
          if (z.empty()) { bad = true; break; }
          zones.insert(z);
          if (cut == string::npos) break;
          rest = rest.substr(cut + 2);
        }
        if (!bad) cs.vz_topologies.push_back({key, zones});
      }
    }
    if (cs.vz_topologies.empty()) return Status::skip();
    return {};
  }
  Status vz_filter(const CycleState& cs, int ni) const {
    const Labels& ls = nodes[ni].labels;
    bool constrained = false;
    for (const char* key : kVolumeZoneLabels) constrained |= ls.count(key) > 0;
    if (!constrained) return {};
    for (auto& t : cs.vz_topologies) {
      auto it = ls.find(t.first);
      if (it == ls.end() || !t.second.count(it->second)) return unresolvable("node(s) had no available volume zone");
    }
    return {};
  }

  // ---------------------------------------------------------------- DefaultPreemption (dry run)
  // The PostFilter of an unschedulable pod (default_preemption.go, framework/
  // preemption/preemption.go; v1.30.4), run without its side effects: victims are
  // chosen and a node nominated on the current snapshot, nothing is evicted.
  // Deliberate, documented choices: every potential node is examined
  // (upstream examines max(10%, 100) of them from a random offset and stops
  // early), ties of pickOneNodeForPreemption go to the seeded selectHost rule
  // (upstream: the first of a map iteration), pods without status.startTime
  // count as started last (upstream: time.Now()).  No PodDisruptionBudgets exist
  // in this model, so every victim is non-violating.
  // Does pod p pass every Filter on node ni of the current snapshot
  // (SelectVictimsOnNode -> RunFilterPluginsWithNominatedPods; the PreFilter
  // state is recomputed on the snapshot, which is what RemovePod / AddPod keep
  // it equal to).
  bool fits_on(const Pod& p, int ni, Pool& pool) {
    CycleState cs;
    set<PluginId> skip;
    for (size_t k = 0; k < profile.size(); ++k) {
      PluginId id = profile[k];
      if (!has_prefilter(id)) continue;
      Status s;
      bool has_res = false;
      if (id == P_FIT) s = fit_prefilter(p, cs);
      else if (id == P_NA) s = na_prefilter(p, cs, has_res).first;
      else if (id == P_PTS) s = pts_prefilter(p, cs, pool);
      else if (id == P_IPA) s = ipa_prefilter(p, cs, pool);
      else if (id == P_PORTS) s = ports_prefilter(p, cs);
      else if (id == P_VOLRESTRICT) s = vr_prefilter(p, cs);
      else if (id == P_NONCSI || id == P_CSILIMITS) s = limits_prefilter(p);
      else if (id == P_VOLBIND) { vector<string> res; s = vb_prefilter(p, cs, has_res, res); }
      else if (id == P_VOLZONE) s = vz_prefilter(p, cs);
      if (s.code == Status::Skip) { skip.insert(id); continue; }
      if (!s.ok()) return false;
    }
    for (size_t k = 0; k < profile.size(); ++k) {
      PluginId id = profile[k];
      if (!has_filter(id) || skip.count(id)) continue;
      Status s;
      if (id == P_FIT) s = fit_filter(cs, ni);
      else if (id == P_TAINT) s = taint_filter(p, ni);
      else if (id == P_NA) s = na_filter(cs, ni);
      else if (id == P_PTS) s = pts_filter(p, cs, ni);
      else if (id == P_IPA) s = ipa_filter(p, cs, ni);
      else if (id == P_UNSCHED) s = unsched_filter(p, ni);
      else if (id == P_NODENAME) s = nodename_filter(p, ni);
      else if (id == P_PORTS) s = ports_filter(cs, ni);
      else if (id == P_VOLRESTRICT) s = vr_filter(cs);
      else if (id == P_CSILIMITS) s = csi_filter(p, ni);
      else if (id == P_VOLBIND) s = vb_filter(cs, ni);
      else if (id == P_VOLZONE) s = vz_filter(cs, ni);
      if (!s.ok()) return false;
    }
    return true;
  }
  // util.MoreImportantPod: higher priority, then the earlier start
  bool more_important(int a, int b) const {
    const Pod& x = pods[a].pod;
    const Pod& y = pods[b].pod;
    if (x.priority != y.priority) return x.priority > y.priority;
    if (x.start_time != y.start_time) return x.start_time < y.start_time;
    return a < b;
  }
  void preempt(int qidx, int pi, const vector<int>& potential, PodResult& r, Pool& pool) {
    int pk = -1;
    for (size_t k = 0; k < profile.size(); ++k)
      if (profile_names[k] == "DefaultPreemption") pk = (int)k;
    if (pk < 0) return;
    const Pod& p = pods[pi].pod;
    if (p.preempt_never) return;  // PodEligibleToPreemptOthers
    struct Cand { int node; vector<int> victims; };
    vector<Cand> cands;
    for (int ni : potential) {  // DryRunPreemption -> SelectVictimsOnNode
      vector<int> pv;
      for (int v : infos[ni].pods)
        if (pods[v].pod.priority < p.priority) pv.push_back(v);
      if (pv.empty()) continue;  // "No preemption victims found for incoming pod"
      for (int v : pv) remove_pod(v, ni);
      if (!fits_on(p, ni, pool)) {
        for (int v : pv) add_pod(v, ni);
        continue;
      }
      std::sort(pv.begin(), pv.end(), [&](int a, int b) { return more_important(a, b); });
      vector<int> victims;
      for (int v : pv) {  // reprieve, most important first
        add_pod(v, ni);
        if (!fits_on(p, ni, pool)) {
          remove_pod(v, ni);
          victims.push_back(v);
        }
      }
      for (int v : victims) add_pod(v, ni);  // dry run: the snapshot is left as it was
      if (!victims.empty()) cands.push_back({ni, victims});
    }
    if (cands.empty()) return;
    // pickOneNodeForPreemption: min PDB violations (none), min highest victim
    // priority, min sum of (priority + 2^31), fewest victims, latest start of the
    // highest-priority victims; then the seeded tie-break
    auto key = [&](const Cand& c, int f) -> i64 {
      const vector<int>& v = c.victims;
      switch (f) {
        case 0: return -(i64)pods[v[0]].pod.priority;
        case 1: {
          i64 s = 0;
          for (int x : v) s += pods[x].pod.priority + (i64)2147483648LL;
          return -s;
        }
        case 2: return -(i64)v.size();
        default: {
          const i64 hp = pods[v[0]].pod.priority;
          i64 e = pods[v[0]].pod.start_time;
          for (int x : v)
            if (pods[x].pod.priority == hp && pods[x].pod.start_time < e) e = pods[x].pod.start_time;
          return e;
        }
      }
    };
    vector<size_t> all(cands.size());
    for (size_t i = 0; i < all.size(); ++i) all[i] = i;
    for (int f = 0; f < 4 && all.size() > 1; ++f) {
      i64 best = INT64_MIN;
      vector<size_t> sel;
      for (size_t i : all) {
        const i64 k = key(cands[i], f);
        if (k > best) { best = k; sel.clear(); }
        if (k == best) sel.push_back(i);
      }
      all = sel;
    }
    size_t pick = all[0];
    unsigned long long bk = 0;
    for (size_t i : all) {
      const unsigned long long k = pack_key(0, qidx, cands[i].node);
      if (k > bk) { bk = k; pick = i; }
    }
    r.nominated = nodes[cands[pick].node].name;
    r.nominated_idx = cands[pick].node;
    r.preempt_plugin = profile_names[pk];
    for (int v : cands[pick].victims) r.victims.push_back(pods[v].pod.ns + "/" + pods[v].pod.name);
  }

  // ---------------------------------------------------------------- NodeResourcesFit
  Status fit_prefilter(const Pod& p, CycleState& cs) {
    cs.fit_req = pod_requests(p, false);
    cs.fit_req_res = Resource();
    resource_add(cs.fit_req_res, cs.fit_req);
    return {};
  }
  Status fit_filter(CycleState& cs, int ni) {  // fit.go fitsRequest
    const Resource& pr = cs.fit_req_res;
    const NodeInfo& n = infos[ni];
    const Resource& a = nodes[ni].alloc;
    vector<string> reasons;
    bool unres = false;
    if ((i64)n.pods.size() + 1 > a.allowed_pods) reasons.push_back("Too many pods");
    bool any_scalar = false;
    for (auto& kv : pr.scalar) any_scalar = true, (void)kv;
    if (pr.milli_cpu == 0 && pr.memory == 0 && pr.eph == 0 && !any_scalar) goto done;
    // InsufficientResource.Unresolvable: the request exceeds the allocatable itself
    // (the Filter then returns UnschedulableAndUnresolvable; preemption cannot help)
    if (pr.milli_cpu > 0 && pr.milli_cpu > a.milli_cpu - n.requested.milli_cpu) {
      reasons.push_back("Insufficient cpu");
      unres |= pr.milli_cpu > a.milli_cpu;
    }
    if (pr.memory > 0 && pr.memory > a.memory - n.requested.memory) {
      reasons.push_back("Insufficient memory");
      unres |= pr.memory > a.memory;
    }
    if (pr.eph > 0 && pr.eph > a.eph - n.requested.eph) {
      reasons.push_back("Insufficient ephemeral-storage");
      unres |= pr.eph > a.eph;
    }
    for (auto& kv : pr.scalar) {  // map order upstream; sorted here
      if (kv.second == 0) continue;
      i64 al = a.scalar.count(kv.first) ? a.scalar.at(kv.first) : 0;
      i64 rq = n.requested.scalar.count(kv.first) ? n.requested.scalar.at(kv.first) : 0;
      if (kv.second > al - rq) {
        reasons.push_back("Insufficient " + kv.first);
        unres |= kv.second > al;
      }
    }
  done:
    if (reasons.empty()) return {};
    string m;
    for (size_t i = 0; i < reasons.size(); ++i) m += (i ? ", " : "") + reasons[i];
    return {unres ? Status::UnschedulableAndUnresolvable : Status::Unschedulable, m};
  }
  // resourceAllocationScorer.calculatePodResourceRequest
  static i64 pod_res_request(const Pod& p, const string& name, bool use_requested) {
    ResourceList r = pod_requests(p, !use_requested);
    auto it = r.find(name);
    if (it == r.end()) return 0;
    return name == "cpu" ? q_milli(it->second) : q_value(it->second);
  }
  // calculateResourceAllocatableRequest -> (alloc, req)
  std::pair<i64, i64> alloc_req(int ni, const string& res, i64 pod_req, bool use_requested) {
    const NodeInfo& n = infos[ni];
    const Resource& a = nodes[ni].alloc;
    if (pod_req == 0 && is_scalar_name(res)) return {0, 0};
    if (res == "cpu") return {a.milli_cpu, (use_requested ? n.requested.milli_cpu : n.nz_cpu) + pod_req};
    if (res == "memory") return {a.memory, (use_requested ? n.requested.memory : n.nz_mem) + pod_req};
    if (res == "ephemeral-storage") return {a.eph, n.requested.eph + pod_req};
    auto it = a.scalar.find(res);
    if (it != a.scalar.end()) {
      i64 rq = n.requested.scalar.count(res) ? n.requested.scalar.at(res) : 0;
      return {it->second, rq + pod_req};
    }
    return {0, 0};
  }
  i64 rtc_fn(i64 p) {  // helper.BuildBrokenLinearFunction over the scaled shape
    for (size_t i = 0; i < rtc_shape.size(); ++i) {
      if (p <= rtc_shape[i].first) {
        if (i == 0) return rtc_shape[0].second;
        return rtc_shape[i - 1].second + (rtc_shape[i].second - rtc_shape[i - 1].second) *
                                             (p - rtc_shape[i - 1].first) /
                                             (rtc_shape[i].first - rtc_shape[i - 1].first);
      }
    }
    return rtc_shape.back().second;
  }
  i64 fit_score(CycleState& cs, int ni) {
    vector<i64> req(fit_res.size(), 0), al(fit_res.size(), 0);
    for (size_t i = 0; i < fit_res.size(); ++i) {
      auto ar = alloc_req(ni, fit_res[i].name, cs.fit_score_req[i], false);
      if (ar.first == 0) continue;
      al[i] = ar.first;
      req[i] = ar.second;
    }
    i64 node_score = 0, wsum = 0;
    if (fit_strategy == "RequestedToCapacityRatio") {
      for (size_t i = 0; i < req.size(); ++i) {
        if (al[i] == 0) continue;
        i64 s = (al[i] == 0 || req[i] > al[i]) ? rtc_fn(100) : rtc_fn(req[i] * 100 / al[i]);
        if (s > 0) {
          node_score += s * fit_res[i].weight;
          wsum += fit_res[i].weight;
        }
      }
      if (wsum == 0) return 0;
      return (i64)go_round((double)node_score / (double)wsum);
    }
    for (size_t i = 0; i < req.size(); ++i) {
      if (al[i] == 0) continue;
      i64 s;
      if (fit_strategy == "MostAllocated") {
        i64 r = req[i] > al[i] ? al[i] : req[i];
        s = r * kMaxNodeScore / al[i];
      } else {
        s = req[i] > al[i] ? 0 : (al[i] - req[i]) * kMaxNodeScore / al[i];
      }
      node_score += s * fit_res[i].weight;
      wsum += fit_res[i].weight;
    }
    if (wsum == 0) return 0;
    return node_score / wsum;
  }
  // ---------------------------------------------------------------- BalancedAllocation
  i64 ba_score(CycleState& cs, int ni) {
    vector<double> fr;
    double total = 0;
    for (size_t i = 0; i < ba_res.size(); ++i) {
      auto ar = alloc_req(ni, ba_res[i].name, cs.ba_req[i], true);
      if (ar.first == 0) continue;
      double f = (double)ar.second / (double)ar.first;
      if (f > 1) f = 1;
      total += f;
      fr.push_back(f);
    }
    double std_ = 0.0;
    if (fr.size() == 2) {
      std_ = std::fabs((fr[0] - fr[1]) / 2);
    } else if (fr.size() > 2) {
      double mean = total / (double)fr.size();
      double sum = 0;
      for (double f : fr) sum = sum + (f - mean) * (f - mean);
      std_ = std::sqrt(sum / (double)fr.size());
    }
    return (i64)((1 - std_) * (double)kMaxNodeScore);
  }
  // ---------------------------------------------------------------- NodeUnschedulable / NodeName
  Status unsched_filter(const Pod& p, int ni) {  // node_unschedulable.go Filter
    if (!nodes[ni].unschedulable) return {};
    if (tolerations_tolerate(p.tolerations, Taint{"node.kubernetes.io/unschedulable", "", "NoSchedule"})) return {};
    return {Status::UnschedulableAndUnresolvable, "node(s) were unschedulable"};
  }
  Status nodename_filter(const Pod& p, int ni) {  // node_name.go Fits
    if (p.node_name.empty() || p.node_name == nodes[ni].name) return {};
    return {Status::UnschedulableAndUnresolvable, "node(s) didn't match the requested node name"};
  }
  // ---------------------------------------------------------------- NodePorts
  Status ports_prefilter(const Pod& p, CycleState& cs) {
    cs.ports_want.clear();
    for (auto& c : p.containers) cs.ports_want.insert(cs.ports_want.end(), c.ports.begin(), c.ports.end());
    if (cs.ports_want.empty()) return Status::skip();
    return {};
  }
  Status ports_filter(CycleState& cs, int ni) {  // fitsPorts -> HostPortInfo.CheckConflict
    const auto& used = infos[ni].used_ports;
    for (auto& w : cs.ports_want) {
      std::pair<string, int32_t> pp{w.proto, w.port};
      bool conflict = false;
      if (w.ip == "0.0.0.0") {
        for (auto& kv : used)
          if (kv.second.count(pp)) conflict = true;
      } else {
        for (const string& k : {string("0.0.0.0"), w.ip}) {
          auto it = used.find(k);
          if (it != used.end() && it->second.count(pp)) conflict = true;
        }
      }
      if (conflict) return {Status::Unschedulable, "node(s) didn't have free ports for the requested pod ports"};
    }
    return {};
  }
  // ---------------------------------------------------------------- ImageLocality
  i64 image_score(const Pod& p, int ni) {  // image_locality.go Score
    const Node& n = nodes[ni];
    i64 sum = 0;
    auto add = [&](const vector<Container>& cs) {
      for (auto& c : cs) {
        string nm = normalized_image_name(c.image);
        bool has = false;
        for (auto& im : n.images)
          for (auto& x : im.names) has |= x == nm;
        if (!has) continue;
        auto& st = image_states[nm];
        double spread = (double)st.second / (double)nodes.size();  // scaledImageScore
        sum += (i64)((double)st.first * spread);
      }
    };
    add(p.init_containers);
    add(p.containers);
    i64 maxT = kImgMaxContainerThreshold * (i64)(p.init_containers.size() + p.containers.size());
    if (sum < kImgMinThreshold) sum = kImgMinThreshold;
    else if (sum > maxT) sum = maxT;
    return kMaxNodeScore * (sum - kImgMinThreshold) / (maxT - kImgMinThreshold);
  }
  // ---------------------------------------------------------------- TaintToleration
  Status taint_filter(const Pod& p, int ni) {
    for (auto& t : nodes[ni].taints) {
      if (t.effect != "NoSchedule" && t.effect != "NoExecute") continue;
      if (!tolerations_tolerate(p.tolerations, t))
        return {Status::UnschedulableAndUnresolvable,
                "node(s) had untolerated taint {" + t.key + ": " + t.value + "}"};
    }
    return {};
  }
  i64 taint_score(CycleState& cs, int ni) {
    i64 c = 0;
    for (auto& t : nodes[ni].taints) {
      if (t.effect != "PreferNoSchedule") continue;
      if (!tolerations_tolerate(cs.taint_prefer_tols, t)) c++;
    }
    return c;
  }
  // ---------------------------------------------------------------- NodeAffinity
  RequiredNodeAffinity get_required(const Pod& p) {  // nodeaffinity.GetRequiredNodeAffinity
    RequiredNodeAffinity r;
    if (!p.node_selector.empty()) {
      r.has_label_sel = true;
      r.label_sel.nothing = false;
      for (auto& kv : p.node_selector) {
        Req q;
        make_req(kv.first, "In", {kv.second}, q);
        r.label_sel.reqs.push_back(q);
      }
    }
    if (p.has_required_na) {
      r.has_node_sel = true;
      for (auto* t : p.required_terms) {
        if (term_is_empty(*t)) continue;
        r.terms.push_back(parse_node_term(*t));
      }
    }
    return r;
  }
  std::pair<Status, vector<string>> na_prefilter(const Pod& p, CycleState& cs, bool& has_result) {
    has_result = false;
    bool no_na = !p.has_required_na;
    if (no_na && !p.has_node_selector) return {Status::skip(), {}};
    cs.na_required = get_required(p);
    if (no_na || p.required_terms.empty()) return {{}, {}};
    set<string> node_names;
    bool names_nil = true;
    for (auto* t : p.required_terms) {
      bool term_nil = true;
      set<string> tn;
      if (auto* mf = t->get("matchFields"))
        for (auto& r : mf->arr) {
          if ((r.get("key") ? r.get("key")->str() : "") == "metadata.name" &&
              (r.get("operator") ? r.get("operator")->str() : "") == "In") {
            vector<string> v = str_list(r.get("values"));
            set<string> s(v.begin(), v.end());
            if (term_nil) tn = s, term_nil = false;
            else {
              set<string> x;
              for (auto& a : tn)
                if (s.count(a)) x.insert(a);
              tn = x;
            }
          }
        }
      if (term_nil) return {{}, {}};
      names_nil = false;
      node_names.insert(tn.begin(), tn.end());
    }
    if (!names_nil && node_names.empty())
      return {{Status::UnschedulableAndUnresolvable, "pod affinity terms conflict"}, {}};
    if (!node_names.empty()) {
      has_result = true;
      return {{}, vector<string>(node_names.begin(), node_names.end())};
    }
    return {{}, {}};
  }
  Status na_filter(CycleState& cs, int ni) {
    if (!cs.na_required.match(nodes[ni].labels, nodes[ni].name))
      return {Status::UnschedulableAndUnresolvable, "node(s) didn't match Pod's node affinity/selector"};
    return {};
  }
  Status na_prescore(const Pod& p, CycleState& cs, int n_nodes) {
    if (n_nodes == 0) return {};
    if (!p.has_preferred_na) return Status::skip();
    cs.na_pref.clear();
    for (auto* t : p.preferred_terms) {  // NewPreferredSchedulingTerms
      i64 w = t->get("weight") ? t->get("weight")->i64() : 0;
      auto* pref = t->get("preference");
      static const ojson::Value kEmptyObj = [] { ojson::Value v; v.kind = ojson::Value::Obj; return v; }();
      const ojson::Value& pv = pref ? *pref : kEmptyObj;
      if (w == 0 || term_is_empty(pv)) continue;
      NodeSelTerm nt = parse_node_term(pv);
      if (nt.err) return {Status::Error, "invalid preferred node affinity term"};
      cs.na_pref.push_back({nt, w});
    }
    return {};
  }
  i64 na_score(CycleState& cs, int ni) {
    i64 s = 0;
    for (auto& t : cs.na_pref)
      if (t.term.match(nodes[ni].labels, nodes[ni].name)) s += t.weight;
    return s;
  }
  // ---------------------------------------------------------------- PodTopologySpread
  bool filter_tsc(const Pod& p, const string& action, vector<CycleState::TsConstraint>& out) {
    out.clear();
    for (auto& c : p.tsc) {
      if (c.when != action) continue;
      CycleState::TsConstraint t;
      if (!label_selector(c.selector_json, t.sel)) return false;
      if (!c.match_label_keys.empty()) {  // MatchLabelKeysInPodTopologySpread (beta, on)
        Labels ml;
        for (auto& k : c.match_label_keys) {
          auto it = p.labels.find(k);
          if (it != p.labels.end()) ml[k] = it->second;
        }
        if (!ml.empty() && !t.sel.nothing)
          for (auto& kv : ml) {
            Req q;
            make_req(kv.first, "In", {kv.second}, q);
            t.sel.reqs.push_back(q);
          }
      }
      t.max_skew = c.max_skew;
      t.key = c.key;
      t.min_domains = c.has_min_domains ? c.min_domains : 1;
      t.honor_affinity = c.node_affinity_policy.empty() || c.node_affinity_policy == "Honor";
      t.honor_taints = c.node_taints_policy == "Honor";
      out.push_back(t);
    }
    return true;
  }
  bool node_has_keys(int ni, const vector<CycleState::TsConstraint>& cs) {
    for (auto& c : cs)
      if (!nodes[ni].labels.count(c.key)) return false;
    return true;
  }
  bool match_inclusion(const Pod& p, const CycleState::TsConstraint& c, int ni, const RequiredNodeAffinity& ra) {
    if (c.honor_affinity && !ra.match(nodes[ni].labels, nodes[ni].name)) return false;
    if (c.honor_taints)
      for (auto& t : nodes[ni].taints)
        if ((t.effect == "NoSchedule" || t.effect == "NoExecute") && !tolerations_tolerate(p.tolerations, t))
          return false;
    return true;
  }
  i64 count_match(int ni, const Selector& sel, const string& ns) {  // countPodsMatchSelector
    if (sel.empty()) return 0;
    i64 c = 0;
    for (int pi : infos[ni].pods) {
      const Pod& q = pods[pi].pod;
      if (q.terminating || q.ns != ns) continue;
      if (sel.matches(q.labels)) c++;
    }
    return c;
  }
  Status pts_prefilter(const Pod& p, CycleState& cs, Pool& pool) {
    if (!filter_tsc(p, "DoNotSchedule", cs.pts_filter)) return {Status::Error, "invalid topology spread constraint"};
    // system-default constraints need a Service/RC/RS/SS selector; none are modelled => empty.
    if (cs.pts_filter.empty()) return Status::skip();
    RequiredNodeAffinity ra = get_required(p);
    int N = (int)nodes.size();
    vector<vector<std::pair<std::pair<string, string>, i64>>> per_node(N);
    pool.until(N, [&](int ni) {
      if (!node_has_keys(ni, cs.pts_filter)) return;
      map<std::pair<string, string>, i64> tp;
      for (auto& c : cs.pts_filter) {
        if (!match_inclusion(p, c, ni, ra)) continue;
        tp[{c.key, nodes[ni].labels.at(c.key)}] = count_match(ni, c.sel, p.ns);  // overwrite (upstream)
      }
      per_node[ni].assign(tp.begin(), tp.end());
    });
    cs.pts_pair_num.clear();
    for (auto& v : per_node)
      for (auto& kv : v) cs.pts_pair_num[kv.first] += kv.second;
    cs.pts_key_domains.clear();
    cs.pts_key_min.clear();
    for (auto& c : cs.pts_filter) cs.pts_key_min[c.key] = 2147483647;  // newCriticalPaths
    for (auto& kv : cs.pts_pair_num) {
      cs.pts_key_domains[kv.first.first]++;
      auto& m = cs.pts_key_min[kv.first.first];
      if (kv.second < m) m = kv.second;
    }
    return {};
  }
  Status pts_filter(const Pod& p, CycleState& cs, int ni) {
    for (auto& c : cs.pts_filter) {
      auto it = nodes[ni].labels.find(c.key);
      if (it == nodes[ni].labels.end())
        return {Status::UnschedulableAndUnresolvable,
                "node(s) didn't match pod topology spread constraints (missing required label)"};
      auto dn = cs.pts_key_domains.find(c.key);
      if (dn == cs.pts_key_domains.end()) return {Status::Error, "internal error: get domains num"};
      i64 min_match = cs.pts_key_min[c.key];
      if (dn->second < c.min_domains) min_match = 0;
      i64 self = c.sel.matches(p.labels) ? 1 : 0;
      auto pn = cs.pts_pair_num.find({c.key, it->second});
      i64 match = pn == cs.pts_pair_num.end() ? 0 : pn->second;
      if (match + self - min_match > c.max_skew)
        return {Status::Unschedulable, "node(s) didn't match pod topology spread constraints"};
    }
    return {};
  }
  Status pts_prescore(const Pod& p, CycleState& cs, const vector<int>& filtered, Pool& pool) {
    if (filtered.empty() || nodes.empty()) return Status::skip();
    if (!filter_tsc(p, "ScheduleAnyway", cs.pts_score)) return {Status::Error, "invalid topology spread constraint"};
    bool require_all = true;  // explicit constraints, or systemDefaulted == false
    if (cs.pts_score.empty()) return Status::skip();
    cs.pts_ignored.clear();
    cs.pts_pair_counts.clear();
    vector<i64> topo_size(cs.pts_score.size(), 0);
    for (int ni : filtered) {
      if (require_all && !node_has_keys(ni, cs.pts_score)) {
        cs.pts_ignored.insert(nodes[ni].name);
        continue;
      }
      for (size_t i = 0; i < cs.pts_score.size(); ++i) {
        auto& c = cs.pts_score[i];
        if (c.key == "kubernetes.io/hostname") continue;
        std::pair<string, string> pr{c.key, nodes[ni].labels.count(c.key) ? nodes[ni].labels.at(c.key) : ""};
        if (!cs.pts_pair_counts.count(pr)) {
          cs.pts_pair_counts[pr] = 0;
          topo_size[i]++;
        }
      }
    }
    cs.pts_weight.assign(cs.pts_score.size(), 0);
    for (size_t i = 0; i < cs.pts_score.size(); ++i) {
      i64 sz = topo_size[i];
      if (cs.pts_score[i].key == "kubernetes.io/hostname") sz = (i64)filtered.size() - (i64)cs.pts_ignored.size();
      cs.pts_weight[i] = go_log((double)(sz + 2));
    }
    RequiredNodeAffinity ra = get_required(p);
    int N = (int)nodes.size();
    std::mutex mu;
    pool.until(N, [&](int ni) {
      if (require_all && !node_has_keys(ni, cs.pts_score)) return;
      for (auto& c : cs.pts_score) {
        if (!match_inclusion(p, c, ni, ra)) continue;
        std::pair<string, string> pr{c.key, nodes[ni].labels.count(c.key) ? nodes[ni].labels.at(c.key) : ""};
        auto it = cs.pts_pair_counts.find(pr);  // map structure is frozen; values updated
        if (it == cs.pts_pair_counts.end()) continue;
        i64 cnt = count_match(ni, c.sel, p.ns);
        std::lock_guard<std::mutex> g(mu);
        it->second += cnt;
      }
    });
    return {};
  }
  i64 pts_score(const Pod& p, CycleState& cs, int ni) {
    if (cs.pts_ignored.count(nodes[ni].name)) return 0;
    double score = 0;
    for (size_t i = 0; i < cs.pts_score.size(); ++i) {
      auto& c = cs.pts_score[i];
      auto it = nodes[ni].labels.find(c.key);
      if (it == nodes[ni].labels.end()) continue;
      i64 cnt;
      if (c.key == "kubernetes.io/hostname") cnt = count_match(ni, c.sel, p.ns);
      else cnt = cs.pts_pair_counts.at({c.key, it->second});
      score += (double)cnt * cs.pts_weight[i] + (double)(c.max_skew - 1);  // scoreForCount
    }
    return (i64)go_round(score);
  }
  // ---------------------------------------------------------------- InterPodAffinity
  void merge_ns(AffTerm& t) {  // mergeAffinityTermNamespacesIfNotEmpty (namespaces carry no labels)
    if (t.ns_selector.empty()) return;
    static const Labels kEmpty;
    for (auto& ns : namespaces)
      if (t.ns_selector.matches(kEmpty)) t.namespaces.insert(ns);
    t.ns_selector = Selector();  // Nothing
  }
  static void tm_update(map<std::pair<string, string>, i64>& m, const Labels& nl, const string& key, i64 v) {
    auto it = nl.find(key);
    if (it == nl.end()) return;
    auto& x = m[{key, it->second}];
    x += v;
    if (x == 0) m.erase({key, it->second});
  }
  static bool matches_all(const vector<AffTerm>& terms, const Pod& q) {
    if (terms.empty()) return false;
    for (auto& t : terms)
      if (!t.matches(q.labels, q.ns, nullptr)) return false;
    return true;
  }
  Status ipa_prefilter(const Pod& p, CycleState& cs, Pool& pool) {
    cs.ipa_req_aff = p.req_aff;
    cs.ipa_req_anti = p.req_anti;
    for (auto& t : cs.ipa_req_aff) merge_ns(t);
    for (auto& t : cs.ipa_req_anti) merge_ns(t);
    static const Labels kNsLabels;  // namespace labels are not modelled (empty)
    int N = (int)nodes.size();
    vector<map<std::pair<string, string>, i64>> ex(N), af(N), an(N);
    pool.until(N, [&](int ni) {
      const Labels& nl = nodes[ni].labels;
      for (int pi : infos[ni].pods_with_req_anti)
        for (auto& t : pods[pi].pod.req_anti)
          if (t.matches(p.labels, p.ns, &kNsLabels)) tm_update(ex[ni], nl, t.topology_key, 1);
      if (cs.ipa_req_aff.empty() && cs.ipa_req_anti.empty()) return;
      for (int pi : infos[ni].pods) {
        const Pod& q = pods[pi].pod;
        if (matches_all(cs.ipa_req_aff, q))
          for (auto& t : cs.ipa_req_aff) tm_update(af[ni], nl, t.topology_key, 1);
        for (auto& t : cs.ipa_req_anti)
          if (t.matches(q.labels, q.ns, nullptr)) tm_update(an[ni], nl, t.topology_key, 1);
      }
    });
    cs.ipa_existing_anti.clear();
    cs.ipa_aff_counts.clear();
    cs.ipa_anti_counts.clear();
    auto append = [](map<std::pair<string, string>, i64>& dst, const map<std::pair<string, string>, i64>& src) {
      for (auto& kv : src) {
        auto& x = dst[kv.first];
        x += kv.second;
        if (x == 0) dst.erase(kv.first);
      }
    };
    for (int ni = 0; ni < N; ++ni) {
      append(cs.ipa_existing_anti, ex[ni]);
      append(cs.ipa_aff_counts, af[ni]);
      append(cs.ipa_anti_counts, an[ni]);
    }
    if (cs.ipa_existing_anti.empty() && cs.ipa_req_aff.empty() && cs.ipa_req_anti.empty()) return Status::skip();
    return {};
  }
  Status ipa_filter(const Pod& p, CycleState& cs, int ni) {
    const Labels& nl = nodes[ni].labels;
    // satisfyPodAffinity
    bool pods_exist = true, aff_ok = true;
    for (auto& t : cs.ipa_req_aff) {
      auto it = nl.find(t.topology_key);
      if (it == nl.end()) {
        aff_ok = false;
        break;
      }
      auto c = cs.ipa_aff_counts.find({t.topology_key, it->second});
      if (c == cs.ipa_aff_counts.end() || c->second <= 0) pods_exist = false;
    }
    if (aff_ok && !pods_exist)
      aff_ok = cs.ipa_aff_counts.empty() && matches_all(cs.ipa_req_aff, p);
    if (!aff_ok) return {Status::UnschedulableAndUnresolvable, "node(s) didn't match pod affinity rules"};
    // satisfyPodAntiAffinity
    if (!cs.ipa_anti_counts.empty())
      for (auto& t : cs.ipa_req_anti) {
        auto it = nl.find(t.topology_key);
        if (it == nl.end()) continue;
        auto c = cs.ipa_anti_counts.find({t.topology_key, it->second});
        if (c != cs.ipa_anti_counts.end() && c->second > 0)
          return {Status::Unschedulable, "node(s) didn't match pod anti-affinity rules"};
      }
    // satisfyExistingPodsAntiAffinity
    if (!cs.ipa_existing_anti.empty())
      for (auto& kv : nl) {
        auto c = cs.ipa_existing_anti.find({kv.first, kv.second});
        if (c != cs.ipa_existing_anti.end() && c->second > 0)
          return {Status::Unschedulable, "node(s) didn't satisfy existing pods anti-affinity rules"};
      }
    return {};
  }
  Status ipa_prescore(const Pod& p, CycleState& cs, const vector<int>& filtered, Pool& pool) {
    if (filtered.empty()) return Status::skip();
    bool has_constraints = p.pref_aff_present || p.pref_anti_present;
    if (ipa_ignore_existing_pref && !has_constraints) return Status::skip();
    cs.ipa_pref_aff = p.pref_aff;
    cs.ipa_pref_anti = p.pref_anti;
    for (auto& t : cs.ipa_pref_aff) merge_ns(t.t);
    for (auto& t : cs.ipa_pref_anti) merge_ns(t.t);
    static const Labels kNsLabels;
    int N = (int)nodes.size();
    vector<map<string, map<string, i64>>> per(N);
    pool.until(N, [&](int ni) {
      const Labels& nl = nodes[ni].labels;
      const vector<int>& podsv = has_constraints ? infos[ni].pods : infos[ni].pods_with_affinity;
      if (!has_constraints && podsv.empty()) return;
      auto& m = per[ni];
      auto term = [&](const AffTerm& t, int32_t w, const Labels& ql, const string& qns, const Labels* nsl, int32_t mul) {
        if (!t.matches(ql, qns, nsl)) return;
        auto it = nl.find(t.topology_key);
        if (it == nl.end()) return;
        m[t.topology_key][it->second] += (i64)(int32_t)(w * mul);
      };
      for (int pi : podsv) {
        const Pod& q = pods[pi].pod;
        if (nl.empty()) continue;  // processExistingPod: node without labels
        for (auto& t : cs.ipa_pref_aff) term(t.t, t.weight, q.labels, q.ns, nullptr, 1);
        for (auto& t : cs.ipa_pref_anti) term(t.t, t.weight, q.labels, q.ns, nullptr, -1);
        if (ipa_hard_weight > 0)
          for (auto& t : q.req_aff) term(t, (int32_t)ipa_hard_weight, p.labels, p.ns, &kNsLabels, 1);
        for (auto& t : q.pref_aff) term(t.t, t.weight, p.labels, p.ns, &kNsLabels, 1);
        for (auto& t : q.pref_anti) term(t.t, t.weight, p.labels, p.ns, &kNsLabels, -1);
      }
    });
    cs.ipa_topo_score.clear();
    for (auto& m : per)
      for (auto& kv : m)
        for (auto& v : kv.second) cs.ipa_topo_score[kv.first][v.first] += v.second;
    if (cs.ipa_topo_score.empty()) return Status::skip();
    return {};
  }
  i64 ipa_score(CycleState& cs, int ni) {
    i64 s = 0;
    for (auto& kv : cs.ipa_topo_score) {
      auto it = nodes[ni].labels.find(kv.first);
      if (it == nodes[ni].labels.end()) continue;
      auto v = kv.second.find(it->second);
      if (v != kv.second.end()) s += v->second;
    }
    return s;
  }

  // ---------------------------------------------------------------- normalizers
  static void default_normalize(vector<i64>& s, bool reverse) {  // helper.DefaultNormalizeScore
    i64 mx = 0;
    for (i64 x : s)
      if (x > mx) mx = x;
    if (mx == 0) {
      if (reverse)
        for (auto& x : s) x = kMaxNodeScore;
      return;
    }
    for (auto& x : s) {
      i64 v = kMaxNodeScore * x / mx;
      if (reverse) v = kMaxNodeScore - v;
      x = v;
    }
  }
  void pts_normalize(CycleState& cs, const vector<int>& nodes_idx, vector<i64>& s) {
    i64 mn = INT64_MAX, mx = 0;
    vector<bool> inv(s.size(), false);
    for (size_t i = 0; i < s.size(); ++i) {
      if (cs.pts_ignored.count(nodes[nodes_idx[i]].name)) {
        inv[i] = true;
        continue;
      }
      if (s[i] < mn) mn = s[i];
      if (s[i] > mx) mx = s[i];
    }
    for (size_t i = 0; i < s.size(); ++i) {
      if (inv[i]) { s[i] = 0; continue; }
      if (mx == 0) { s[i] = kMaxNodeScore; continue; }
      s[i] = kMaxNodeScore * (mx + mn - s[i]) / mx;
    }
  }
  static void ipa_normalize(CycleState& cs, vector<i64>& s) {
    if (cs.ipa_topo_score.empty()) return;
    i64 mn = INT64_MAX, mx = INT64_MIN;
    for (i64 x : s) {
      if (x > mx) mx = x;
      if (x < mn) mn = x;
    }
    i64 diff = mx - mn;
    for (auto& x : s) {
      double f = 0;
      if (diff > 0) f = (double)kMaxNodeScore * ((double)(x - mn) / (double)diff);
      x = (i64)f;
    }
  }

  // ---------------------------------------------------------------- one scheduling cycle
  void schedule_one(int qidx, int pi, Pool& pool, int record) {
    Pod& p = pods[pi].pod;
    PodResult r;
    CycleState cs;
    auto rec = [&](auto fn) {
      if (!record) return;
      std::lock_guard<std::mutex> g(store_mu);
      fn();
    };
    // ---- PreFilter (RunPreFilterPlugins)
    set<PluginId> skip_filter;
    bool have_names = false;
    set<string> names;
    bool aborted = false;
    for (size_t k = 0; k < profile.size(); ++k) {
      PluginId id = profile[k];
      if (!has_prefilter(id)) continue;
      Status s;
      vector<string> res;
      bool has_res = false;
      if (id == P_FIT) s = fit_prefilter(p, cs);
      else if (id == P_NA) { auto x = na_prefilter(p, cs, has_res); s = x.first; res = x.second; }
      else if (id == P_PTS) s = pts_prefilter(p, cs, pool);
      else if (id == P_IPA) s = ipa_prefilter(p, cs, pool);
      else if (id == P_PORTS) s = ports_prefilter(p, cs);
      else if (id == P_VOLRESTRICT) s = vr_prefilter(p, cs);
      else if (id == P_NONCSI || id == P_CSILIMITS) s = limits_prefilter(p);
      else if (id == P_VOLBIND) s = vb_prefilter(p, cs, has_res, res);
      else if (id == P_VOLZONE) s = vz_prefilter(p, cs);
      const string& nm = profile_names[k];
      rec([&] {
        r.pre_filter_status[nm] = s.ok() ? "success" : s.msg;
        if (has_res) r.pre_filter_result[nm] = res;
      });
      if (s.code == Status::Skip) { skip_filter.insert(id); continue; }
      if (!s.ok()) { aborted = true; r.status = s.code == Status::Error ? 2 : 1; break; }
      if (has_res) {
        if (!have_names) { names.insert(res.begin(), res.end()); have_names = true; }
        else { set<string> x; for (auto& a : names) if (std::count(res.begin(), res.end(), a)) x.insert(a); names = x; }
        if (names.empty()) { aborted = true; r.status = 1; break; }
      }
    }
    if (aborted) { finish(qidx, pi, r, record); return; }
    // ---- Filter (findNodesThatPassFilters / RunFilterPlugins)
    vector<int> cand;
    for (int ni = 0; ni < (int)nodes.size(); ++ni)
      if (!have_names || names.count(nodes[ni].name)) cand.push_back(ni);
    vector<char> pass(cand.size(), 0), fcode(cand.size(), 0);  // fcode: 1 Unschedulable, 2 ...AndUnresolvable
    std::atomic<bool> err{false};
    pool.until((int)cand.size(), [&](int i) {
      int ni = cand[i];
      for (size_t k = 0; k < profile.size(); ++k) {
        PluginId id = profile[k];
        if (!has_filter(id) || skip_filter.count(id)) continue;
        Status s;
        if (id == P_FIT) s = fit_filter(cs, ni);
        else if (id == P_TAINT) s = taint_filter(p, ni);
        else if (id == P_NA) s = na_filter(cs, ni);
        else if (id == P_PTS) s = pts_filter(p, cs, ni);
        else if (id == P_IPA) s = ipa_filter(p, cs, ni);
        else if (id == P_UNSCHED) s = unsched_filter(p, ni);
        else if (id == P_NODENAME) s = nodename_filter(p, ni);
        else if (id == P_PORTS) s = ports_filter(cs, ni);
        else if (id == P_VOLRESTRICT) s = vr_filter(cs);
        else if (id == P_CSILIMITS) s = csi_filter(p, ni);
        else if (id == P_VOLBIND) s = vb_filter(cs, ni);
        else if (id == P_VOLZONE) s = vz_filter(cs, ni);
        rec([&] { r.filter[nodes[ni].name][profile_names[k]] = s.ok() ? "passed" : s.msg; });
        if (!s.ok()) {
          if (s.code == Status::Error) err = true;
          fcode[i] = s.code == Status::Unschedulable ? 1 : 2;
          return;
        }
      }
      pass[i] = 1;
    });
    vector<int> feasible;
    for (size_t i = 0; i < cand.size(); ++i)
      if (pass[i]) feasible.push_back(cand[i]);
    r.feasible = (int)feasible.size();
    if (err) { r.status = 2; finish(qidx, pi, r, record); return; }
    if (feasible.empty()) {
      r.status = 1;
      if (record) {  // PostFilter: DefaultPreemption dry run
        vector<int> potential;  // nodesWherePreemptionMightHelp: not UnschedulableAndUnresolvable
        for (size_t i = 0; i < cand.size(); ++i)
          if (fcode[i] == 1) potential.push_back(cand[i]);
        preempt(qidx, pi, potential, r, pool);
      }
      finish(qidx, pi, r, record);
      return;
    }
    int chosen = -1;
    if (feasible.size() == 1) {
      chosen = feasible[0];
    } else {
      // ---- PreScore
      set<PluginId> skip_score;
      for (size_t k = 0; k < profile.size(); ++k) {
        PluginId id = profile[k];
        if (!has_prescore(id)) continue;
        Status s;
        if (id == P_FIT) { cs.fit_score_req.clear(); for (auto& rs : fit_res) cs.fit_score_req.push_back(pod_res_request(p, rs.name, false)); }
        else if (id == P_BA) { cs.ba_req.clear(); for (auto& rs : ba_res) cs.ba_req.push_back(pod_res_request(p, rs.name, true)); }
        else if (id == P_TAINT) { cs.taint_prefer_tols.clear(); for (auto& t : p.tolerations) if (t.effect.empty() || t.effect == "PreferNoSchedule") cs.taint_prefer_tols.push_back(t); }
        else if (id == P_NA) s = na_prescore(p, cs, (int)feasible.size());
        else if (id == P_PTS) s = pts_prescore(p, cs, feasible, pool);
        else if (id == P_IPA) s = ipa_prescore(p, cs, feasible, pool);
        else if (id == P_VOLBIND) s = Status::skip();  // PreScore: no scorer (VolumeCapacityPriority off)
        rec([&] { r.pre_score[profile_names[k]] = s.ok() ? "success" : s.msg; });
        if (s.code == Status::Skip) { skip_score.insert(id); continue; }
        if (!s.ok()) { r.status = 2; finish(qidx, pi, r, record); return; }
      }
      // ---- Score
      vector<size_t> sp;
      for (size_t k = 0; k < profile.size(); ++k)
        if (has_score(profile[k]) && !skip_score.count(profile[k])) sp.push_back(k);
      size_t F = feasible.size();
      vector<vector<i64>> scores(sp.size(), vector<i64>(F, 0));
      pool.until((int)F, [&](int i) {
        int ni = feasible[i];
        for (size_t j = 0; j < sp.size(); ++j) {
          PluginId id = profile[sp[j]];
          i64 s = 0;
          if (id == P_FIT) s = fit_score(cs, ni);
          else if (id == P_BA) s = ba_score(cs, ni);
          else if (id == P_TAINT) s = taint_score(cs, ni);
          else if (id == P_NA) s = na_score(cs, ni);
          else if (id == P_PTS) s = pts_score(p, cs, ni);
          else if (id == P_IPA) s = ipa_score(cs, ni);
          else if (id == P_IMAGE) s = image_score(p, ni);
          scores[j][i] = s;
          const string& nm = profile_names[sp[j]];
          rec([&] {  // Store.AddScoreResult: raw + provisional final = raw x weight
            r.score[nodes[ni].name][nm] = std::to_string(s);
            r.final_score[nodes[ni].name][nm] = std::to_string(s * store_weight_of(nm));
          });
        }
      });
      // ---- NormalizeScore
      for (size_t j = 0; j < sp.size(); ++j) {
        PluginId id = profile[sp[j]];
        if (!has_score_ext(id)) continue;
        if (id == P_TAINT) default_normalize(scores[j], true);
        else if (id == P_NA) default_normalize(scores[j], false);
        else if (id == P_PTS) pts_normalize(cs, feasible, scores[j]);
        else if (id == P_IPA) ipa_normalize(cs, scores[j]);
        const string& nm = profile_names[sp[j]];
        rec([&] {
          for (size_t i = 0; i < F; ++i)
            r.final_score[nodes[feasible[i]].name][nm] = std::to_string(scores[j][i] * store_weight_of(nm));
        });
      }
      // ---- weights + selectHost (seeded deterministic rule)
      bool any_score_plugin = false;
      for (PluginId id : profile) any_score_plugin |= has_score(id);
      unsigned long long best = 0;
      for (size_t i = 0; i < F; ++i) {
        i64 total = 0;
        if (!any_score_plugin) total = 1;
        for (size_t j = 0; j < sp.size(); ++j) {
          i64 s = scores[j][i];
          if (s > kMaxNodeScore || s < 0) { r.status = 2; finish(qidx, pi, r, record); return; }
          total += s * fw_weight_of(profile_names[sp[j]]);
        }
        unsigned long long key = pack_key(total, qidx, feasible[i]);
        if (key > best || chosen < 0) { best = key; chosen = feasible[i]; }
      }
    }
    r.selected = nodes[chosen].name;
    r.selected_idx = chosen;
    rec([&] {  // wrappedplugin.go Reserve/PreBind/Bind: VolumeBinding (allBound), DefaultBinder
      for (size_t k = 0; k < profile.size(); ++k) {
        if (profile[k] == P_VOLBIND) r.reserve[profile_names[k]] = r.prebind[profile_names[k]] = "success";
        if (profile_names[k] == "DefaultBinder") r.bind[profile_names[k]] = "success";
      }
    });
    if (defer_assume) deferred.emplace_back(pi, chosen);  // what-if batch: bound after the step
    else add_pod(pi, chosen);  // assume
    finish(qidx, pi, r, record);
  }
  unsigned long long pack_key(i64 total, int qidx, int ni) const {
    unsigned long long z = seed ^ ((unsigned long long)qidx * 0x9E3779B97F4A7C15ULL) ^ (unsigned long long)ni;
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    unsigned long long h20 = z >> 44;
    return ((unsigned long long)total << 40) | ((0xFFFFFULL - h20) << 20) | (unsigned long long)ni;
  }
  i64 store_weight_of(const string& n) const {
    auto it = store_weight.find(n);
    return it == store_weight.end() ? 0 : it->second;
  }
  i64 fw_weight_of(const string& n) const {
    auto it = fw_weight.find(n);
    return it == fw_weight.end() ? 1 : it->second;
  }
  vector<string> rendered;
  vector<unsigned long long> digests;
  int keep_annotations = 0;
  void finish(int qidx, int pi, PodResult& r, int record) {
    (void)pi;
    // PostFilter (schedule_one.go: unschedulable pods only).  DefaultPreemption with
    // every pod at the same priority finds no victims (SelectVictimsOnNode removes
    // only lower-priority pods), so nothing is nominated; the wrapper still records
    // every node of the status map, which holds every node (failed Filter, outside
    // the PreFilterResult, or a rejecting PreFilter).
    if (record && r.status == 1)
      for (size_t k = 0; k < profile.size(); ++k)
        if (profile_names[k] == "DefaultPreemption")
          for (auto& n : nodes) r.post_filter_nodes.push_back(n.name);
    if (record >= 2) {
      string a = render_annotations(r);
      unsigned long long h = 1469598103934665603ULL;  // FNV-1a 64
      for (unsigned char c : a) h = (h ^ c) * 1099511628211ULL;
      digests[qidx] = h;
      if (record >= 3) rendered[qidx] = a;
    }
    r.filter.clear();
    r.score.clear();
    r.final_score.clear();
    results[qidx] = std::move(r);
  }
};

// Scheduler configuration → flat profile.  Restates, for one profile:
//  * simulator/scheduler/plugin/plugins.go:289-304 getScorePluginWeight — store
//    weights over Score.Enabled ++ MultiPoint.Enabled, later entries overwrite,
//    weight 0 → 1, the "Wrapped" suffix trimmed;
//  * upstream v1.30.4 pkg/scheduler/framework/runtime/framework.go getScoreWeights
//    — framework weights over the same concatenation, but a name already seen is
//    skipped ("let the individual Score weight take precedence"), 0 → 1;
//  * expandMultiPointPlugins — MultiPoint order is the extension-point order when
//    no extension point lists plugins of its own; a MultiPoint name twice is an error.
// Pinned by scheduler_test.go:344-407 (Score w3 + MultiPoint w2 → store 2).
static std::string trim_wrapped(std::string n) {
  const std::string suffix = "Wrapped";
  if (n.size() > suffix.size() && n.substr(n.size() - suffix.size()) == suffix) n.resize(n.size() - suffix.size());
  return n;
}
static bool flatten_config(const ojson::Value& cfg, ojson::Value& flat, string& err) {
  const ojson::Value* prof = &cfg;
  if (auto* ps = cfg.get("profiles")) {
    if (ps->kind != ojson::Value::Arr || ps->arr.empty()) {
      err = "profiles: empty";
      return false;
    }
    prof = &ps->arr[0];
  }
  const ojson::Value* plugins = prof->get("plugins");
  if (!plugins || plugins->kind != ojson::Value::Obj) {
    err = "plugins: not an object";
    return false;
  }
  struct Entry {
    std::string name;
    long long weight;
  };
  std::vector<Entry> multi, score;
  for (auto& ext : plugins->obj) {
    const ojson::Value* en = ext.second.get("enabled");
    const ojson::Value* dis = ext.second.get("disabled");
    std::vector<Entry>* dst = ext.first == "multiPoint" ? &multi : ext.first == "score" ? &score : nullptr;
    if (!dst) {
      if ((en && !en->arr.empty()) || (dis && !dis->arr.empty())) {
        err = ext.first + ": per-extension-point sets unsupported";
        return false;
      }
      continue;
    }
    if (ext.first == "score" && dis && !dis->arr.empty()) {
      err = "score.disabled unsupported";
      return false;
    }
    if (en)
      for (auto& p : en->arr) {
        auto* w = p.get("weight");
        dst->push_back({trim_wrapped(p.get("name") ? p.get("name")->str() : ""), w ? w->i64() : 0});
      }
  }
  ojson::Value list, fw, sw;
  list.kind = ojson::Value::Arr;
  fw.kind = sw.kind = ojson::Value::Obj;
  std::set<std::string> in_multi;
  for (auto& e : multi) {
    if (!in_multi.insert(e.name).second) {
      err = "plugin " + e.name + " already registered";
      return false;
    }
    ojson::Value s;
    s.kind = ojson::Value::Str;
    s.raw = e.name;
    list.arr.push_back(s);
  }
  for (auto& e : score)
    if (!in_multi.count(e.name)) {
      err = "score plugin " + e.name + " outside multiPoint";
      return false;
    }
  std::vector<Entry> order = score;
  order.insert(order.end(), multi.begin(), multi.end());
  std::map<std::string, long long> fwm, swm;
  for (auto& e : order) {  // getScoreWeights: first one kept
    if (fwm.count(e.name)) continue;
    fwm[e.name] = e.weight == 0 ? 1 : e.weight;
  }
  for (auto& e : order) swm[e.name] = e.weight != 0 ? e.weight : 1;  // getScorePluginWeight: overwrite
  auto num = [](long long v) {
    ojson::Value n;
    n.kind = ojson::Value::Num;
    n.raw = std::to_string(v);
    return n;
  };
  for (auto& kv : fwm) fw.obj.push_back({kv.first, num(kv.second)});
  for (auto& kv : swm) sw.obj.push_back({kv.first, num(kv.second)});
  flat.kind = ojson::Value::Obj;
  flat.obj.push_back({"plugins", list});
  flat.obj.push_back({"weights", fw});
  flat.obj.push_back({"storeWeights", sw});
  if (auto* pc = prof->get("pluginConfig")) {
    ojson::Value m;
    m.kind = ojson::Value::Obj;
    if (pc->kind == ojson::Value::Arr) {
      for (auto& e : pc->arr)
        if (e.get("args")) m.obj.push_back({trim_wrapped(e.get("name") ? e.get("name")->str() : ""), *e.get("args")});
    } else {
      m = *pc;
    }
    flat.obj.push_back({"pluginConfig", m});
  }
  if (auto* s = prof->get("seed") ? prof->get("seed") : cfg.get("seed")) flat.obj.push_back({"seed", *s});
  return true;
}

static bool load_cluster(const char* js, size_t len, Cluster& c, string& err) {
  ojson::Value doc;
  try {
    doc = ojson::parse(js, len);
  } catch (std::exception& e) {
    err = e.what();
    return false;
  }
  c.doc.reset(new ojson::Value(std::move(doc)));  // pods reference JSON nodes (terms)
  const ojson::Value& d = *c.doc;
  ojson::Value flat;
  const ojson::Value* pr = d.get("profile");
  if (pr && (pr->get("profiles") || (pr->get("plugins") && pr->get("plugins")->kind == ojson::Value::Obj))) {
    if (!flatten_config(*pr, flat, err)) return false;
    pr = &flat;
  }
  if (pr) {
    for (auto& n : pr->get("plugins")->arr) {
      PluginId id = plugin_id(n.str());
      if (id == P_UNKNOWN) {
        err = "unsupported plugin " + n.str();
        return false;
      }
      c.profile.push_back(id);
      c.profile_names.push_back(n.str());
    }
    if (auto* w = pr->get("weights"))
      for (auto& kv : w->obj) c.fw_weight[kv.first] = kv.second.i64() == 0 ? 1 : kv.second.i64();
    if (auto* w = pr->get("storeWeights"))
      for (auto& kv : w->obj) c.store_weight[kv.first] = kv.second.i64() == 0 ? 1 : kv.second.i64();
    if (auto* s = pr->get("seed")) c.seed = std::strtoull(s->raw.c_str(), nullptr, 10);
    if (auto* pc = pr->get("pluginConfig")) {
      if (auto* fit = pc->get("NodeResourcesFit"))
        if (auto* ss = fit->get("scoringStrategy")) {
          if (auto* t = ss->get("type")) c.fit_strategy = t->str();
          if (auto* rs = ss->get("resources")) {
            c.fit_res.clear();
            for (auto& x : rs->arr) c.fit_res.push_back({x.get("name")->str(), x.get("weight") ? x.get("weight")->i64() : 1});
          }
          if (auto* sh = ss->get("requestedToCapacityRatio"))
            if (auto* pts = sh->get("shape"))
              for (auto& x : pts->arr)
                c.rtc_shape.push_back({x.get("utilization")->i64(), x.get("score")->i64() * (kMaxNodeScore / 10)});
        }
      if (auto* ba = pc->get("NodeResourcesBalancedAllocation"))
        if (auto* rs = ba->get("resources")) {
          c.ba_res.clear();
          for (auto& x : rs->arr) c.ba_res.push_back({x.get("name")->str(), x.get("weight") ? x.get("weight")->i64() : 1});
        }
      if (auto* ipa = pc->get("InterPodAffinity")) {
        if (auto* h = ipa->get("hardPodAffinityWeight")) c.ipa_hard_weight = h->i64();
        if (auto* ig = ipa->get("ignorePreferredTermsOfExistingPods")) c.ipa_ignore_existing_pref = ig->b;
      }
    }
  }
  if (auto* ns = d.get("nodes"))
    for (auto& n : ns->arr) {
      Node x;
      parse_node(n, x);
      c.node_index[x.name] = (int)c.nodes.size();
      c.nodes.push_back(std::move(x));
    }
  c.infos.assign(c.nodes.size(), NodeInfo());
  for (auto& n : c.nodes) {  // ImageStateSummary: Size from the first node listing the name, NumNodes
    set<string> seen;
    for (auto& im : n.images)
      for (auto& nm : im.names) {
        auto it = c.image_states.find(nm);
        if (it == c.image_states.end()) c.image_states[nm] = {im.size, 0};
        if (seen.insert(nm).second) c.image_states[nm].second++;
      }
  }
  auto add = [&](const ojson::Value& v) {
    PodRecord r;
    r.parse_ok = parse_pod(v, r.pod);
    r.has_required_anti = !r.pod.req_anti.empty();
    r.with_affinity = r.pod.has_pod_affinity || r.pod.has_pod_anti_affinity;
    c.namespaces.insert(r.pod.ns);
    c.pods.push_back(std::move(r));
    return (int)c.pods.size() - 1;
  };
  // {"pods": bound, "queue": pending}, or the simulator's snapshot document
  // (ResourcesForSnap, simulator/snapshot/snapshot.go:33-42): pending pods (no
  // spec.nodeName) in "pods" are the queue, in document order
  const ojson::Value* qdoc = d.get("queue");
  if (auto* ps = d.get("pods"))
    for (auto& p : ps->arr) {
      int pi = add(p);
      auto it = c.node_index.find(c.pods[pi].pod.node_name);
      if (it != c.node_index.end()) c.add_pod(pi, it->second);
      else if (!qdoc && c.pods[pi].pod.node_name.empty()) c.queue.push_back(pi);
    }
  if (qdoc)
    for (auto& p : qdoc->arr) c.queue.push_back(add(p));
  // the scheduling queue (upstream v1.30.4 internal/queue/scheduling_queue.go):
  // SchedulingGates' PreEnqueue (plugins/schedulinggates/scheduling_gates.go)
  // keeps pods with spec.schedulingGates out of activeQ — never scheduled,
  // nothing recorded — and activeQ pops in PrioritySort order
  // (plugins/queuesort/priority_sort.go Less: higher priority first, then the
  // earlier queue timestamp = document order)
  if (std::find(c.profile_names.begin(), c.profile_names.end(), "SchedulingGates") != c.profile_names.end()) {
    vector<int> keep;
    for (int qi : c.queue) (c.pods[qi].pod.gated ? c.gated : keep).push_back(qi);
    c.queue = std::move(keep);
  }
  // ("queueSort": false — pods arriving one at a time at an idle scheduler — keeps arrival order)
  auto* qs = d.get("queueSort");
  if (!(qs && qs->kind == ojson::Value::Bool && !qs->b))
    std::stable_sort(c.queue.begin(), c.queue.end(),
                     [&](int a, int b) { return c.pods[a].pod.priority > c.pods[b].pod.priority; });
  // storage objects
  auto beta_class = [](const ojson::Value* md, string& cls) {
    auto* ann = md ? md->get("annotations") : nullptr;
    if (auto* b = ann ? ann->get("volume.beta.kubernetes.io/storage-class") : nullptr) cls = b->str();
  };
  if (auto* a = d.get("pvcs"))
    for (auto& v : a->arr) {
      ClaimObj o;
      auto* md = v.get("metadata");
      auto* sp = v.get("spec");
      o.name = md && md->get("name") ? md->get("name")->str() : "";
      o.ns = md && md->get("namespace") ? md->get("namespace")->str() : "";
      if (o.ns.empty()) o.ns = "default";
      o.deleting = md && md->get("deletionTimestamp") && !md->get("deletionTimestamp")->is_null();
      if (sp) {
        o.volume_name = sp->get("volumeName") ? sp->get("volumeName")->str() : "";
        if (auto* sc = sp->get("storageClassName"); sc && !sc->is_null()) o.class_name = sc->str();
        for (auto& m : str_list(sp->get("accessModes"))) o.rwop = o.rwop || m == "ReadWriteOncePod";
      }
      beta_class(md, o.class_name);
      auto* ann = md ? md->get("annotations") : nullptr;
      o.bind_completed = ann && ann->get("pv.kubernetes.io/bind-completed");
      if (auto* sn = ann ? ann->get("volume.kubernetes.io/selected-node") : nullptr) {
        o.has_selected_node = true;
        o.selected_node = sn->str();
      }
      if (auto* st = v.get("status")) o.lost = st->get("phase") && st->get("phase")->str() == "Lost";
      c.claims[o.ns + "/" + o.name] = o;
    }
  if (auto* a = d.get("pvs"))
    for (auto& v : a->arr) {
      VolumeObj o;
      auto* md = v.get("metadata");
      auto* sp = v.get("spec");
      o.name = md && md->get("name") ? md->get("name")->str() : "";
      o.labels = str_map(md ? md->get("labels") : nullptr);
      if (sp) {
        o.class_name = sp->get("storageClassName") ? sp->get("storageClassName")->str() : "";
        auto* na = sp->get("nodeAffinity");
        auto* rq = na && !na->is_null() ? na->get("required") : nullptr;
        if (rq && !rq->is_null()) {
          o.has_required = true;
          o.required_json = rq;
          if (auto* ts = rq->get("nodeSelectorTerms"))
            for (auto& t : ts->arr) {
              o.required.push_back(parse_node_term(t));
              o.required_empty.push_back(term_is_empty(t));
            }
        }
        if (auto* cr = sp->get("claimRef"); cr && !cr->is_null()) {
          o.claim_ref = true;
          o.ref_ns = cr->get("namespace") ? cr->get("namespace")->str() : "";
          o.ref_name = cr->get("name") ? cr->get("name")->str() : "";
        }
        for (const char* k : {"awsElasticBlockStore", "gcePersistentDisk", "azureDisk", "cinder"})
          o.intree = o.intree || (sp->get(k) && !sp->get(k)->is_null());
        if (auto* cs = sp->get("csi"); cs && !cs->is_null()) {
          o.csi = true;
          o.csi_driver = cs->get("driver") ? cs->get("driver")->str() : "";
          o.csi_handle = cs->get("volumeHandle") ? cs->get("volumeHandle")->str() : "";
        }
      }
      beta_class(md, o.class_name);
      c.volumes[o.name] = o;
    }
  if (auto* a = d.get("storageClasses"))
    for (auto& v : a->arr) {
      ClassObj o;
      auto* md = v.get("metadata");
      o.name = md && md->get("name") ? md->get("name")->str() : "";
      o.provisioner = v.get("provisioner") ? v.get("provisioner")->str() : "";
      if (auto* m = v.get("volumeBindingMode"); m && !m->is_null()) {
        o.mode_set = true;
        o.wait_for_consumer = m->str() == "WaitForFirstConsumer";
      }
      if (auto* at = v.get("allowedTopologies"))
        for (auto& t : at->arr) {
          vector<std::pair<string, vector<string>>> term;
          if (auto* me = t.get("matchLabelExpressions"))
            for (auto& e : me->arr) term.push_back({e.get("key") ? e.get("key")->str() : "", str_list(e.get("values"))});
          o.topology.push_back(term);
        }
      c.classes[o.name] = o;
    }
  if (auto* a = d.get("csiNodes"))
    for (auto& v : a->arr) {
      auto* md = v.get("metadata");
      const string node = md && md->get("name") ? md->get("name")->str() : "";
      auto* sp = v.get("spec");
      if (auto* ds = sp ? sp->get("drivers") : nullptr)
        for (auto& dr : ds->arr) {
          auto* al = dr.get("allocatable");
          auto* cnt = al && !al->is_null() ? al->get("count") : nullptr;
          if (cnt && !cnt->is_null()) c.csi_counts[node][dr.get("name") ? dr.get("name")->str() : ""] = cnt->i64();
        }
    }
  // Volume inputs outside the model are refused, never approximated
  auto in_profile = [&](PluginId id) { return std::find(c.profile.begin(), c.profile.end(), id) != c.profile.end(); };
  bool vol = false;
  for (PluginId id : c.profile) vol = vol || is_volume_plugin(id);
  bool preemption = std::find(c.profile_names.begin(), c.profile_names.end(), "DefaultPreemption") != c.profile_names.end();
  if (vol)
    for (int qi : c.queue) {
      const Pod& p = c.pods[qi].pod;
      auto refuse = [&](const string& why) {
        err = "pod " + p.name + ": " + why + " (not modelled)";
        return false;
      };
      if (p.volume_plugins_act) return refuse("volumes other than persistentVolumeClaim");
      if (p.claims.empty()) continue;
      if (in_profile(P_CSILIMITS)) {
        map<string, string> mine;
        c.attachable_volumes(p, mine);
        for (auto& kv : mine)
          if (kv.second.size() >= 63) return refuse("a CSI driver name whose attach-limit key is hashed");
      }
      auto count_users = [&](const string& ns, const string& name, bool with_queue) {
        int u = 0;
        for (size_t i = 0; i < c.pods.size(); ++i) {
          const Pod& o = c.pods[i].pod;
          const bool queued = std::find(c.queue.begin(), c.queue.end(), (int)i) != c.queue.end();
          if (std::find(c.gated.begin(), c.gated.end(), (int)i) != c.gated.end()) continue;  // never assigned
          if (queued && !with_queue) continue;
          u += (int)std::count(o.claims.begin(), o.claims.end(), name) * (o.ns == ns);
        }
        return u;
      };
      for (auto& cn : p.claims) {
        const ClaimObj* cl = c.find_claim(p.ns, cn);
        if (!cl) {
          if (!in_profile(P_VOLRESTRICT) && !in_profile(P_VOLBIND) && !in_profile(P_VOLZONE))
            return refuse("a missing claim no PreFilter rejects");
          continue;
        }
        if (!cl->volume_name.empty()) {
          auto v = c.volumes.find(cl->volume_name);
          if (v != c.volumes.end() && v->second.intree) return refuse("an in-tree cloud disk persistent volume");
        }
        if (cl->rwop && preemption) {
          if (count_users(p.ns, cn, false) > 1) return refuse("a ReadWriteOncePod claim used by several bound pods");
          for (auto& pr : c.pods)
            if (pr.pod.ns != p.ns && std::count(pr.pod.claims.begin(), pr.pod.claims.end(), cn))
              return refuse("a ReadWriteOncePod claim name used in several namespaces");
        }
        if (!cl->volume_name.empty() && cl->bind_completed) continue;
        auto k = cl->class_name.empty() ? c.classes.end() : c.classes.find(cl->class_name);
        if (k != c.classes.end() && !k->second.mode_set && in_profile(P_VOLBIND))
          return refuse("a storage class without volumeBindingMode");
        if (k == c.classes.end() || !k->second.wait_for_consumer || !cl->volume_name.empty()) continue;
        const string& prov = k->second.provisioner;
        if ((prov == "kubernetes.io/aws-ebs" || prov == "kubernetes.io/gce-pd" || prov == "kubernetes.io/azure-disk" ||
             prov == "kubernetes.io/cinder") && in_profile(P_NONCSI))
          return refuse("an in-tree provisioner");
        for (auto& kv : c.volumes) {
          const VolumeObj& v = kv.second;
          if (v.class_name == cl->class_name && (!v.claim_ref || (v.ref_ns == cl->ns && v.ref_name == cl->name)))
            return refuse("static persistent volumes a WaitForFirstConsumer claim could bind");
        }
        if (count_users(p.ns, cn, true) > 1) return refuse("a WaitForFirstConsumer claim shared by several pods");
      }
    }
  c.results.assign(c.queue.size(), PodResult());
  c.rendered.assign(c.queue.size(), string());
  c.digests.assign(c.queue.size(), 0);
  return true;
}

}  // namespace oracle

// ============================================================ C ABI (tests / bench cpu_baseline only)
extern "C" {

struct ksg_oracle {
  oracle::Cluster c;
  std::string err;
  int next = 0;
  std::unique_ptr<oracle::Pool> pool;
};

ksg_oracle* ksg_oracle_load(const char* json, size_t len, char* err, size_t errlen) {
  auto* h = new ksg_oracle();
  std::string e;
  if (!oracle::load_cluster(json, len, h->c, e)) {
    if (err && errlen) std::snprintf(err, errlen, "%s", e.c_str());
    delete h;
    return nullptr;
  }
  return h;
}

void ksg_oracle_free(ksg_oracle* h) { delete h; }

int ksg_oracle_num_nodes(ksg_oracle* h) { return (int)h->c.nodes.size(); }
int ksg_oracle_num_queue(ksg_oracle* h) { return (int)h->c.queue.size(); }

// "namespace/name" of queue pod q (scheduling order), or of gated pod -1-q (q < 0)
int ksg_oracle_queue_pod(ksg_oracle* h, int q, char* buf, size_t cap, size_t* len) {
  int pi = -1;
  if (q >= 0 && q < (int)h->c.queue.size()) pi = h->c.queue[q];
  if (q < 0 && -1 - q < (int)h->c.gated.size()) pi = h->c.gated[-1 - q];
  if (pi < 0) return -1;
  const std::string s = h->c.pods[pi].pod.ns + "/" + h->c.pods[pi].pod.name;
  *len = s.size();
  if (buf && cap >= s.size()) std::memcpy(buf, s.data(), s.size());
  return 0;
}
int ksg_oracle_num_gated(ksg_oracle* h) { return (int)h->c.gated.size(); }

// Schedule the next n queue pods.  record: 0 = plugins only, 1 = store emulation
// (global mutex + map insert + FormatInt per (node, plugin), as the debuggable
// scheduler does), 2 = also digest the rendered annotations, 3 = also keep them.
// Returns pods processed.
int ksg_oracle_schedule(ksg_oracle* h, int n, int workers, int record) {
  if (!h->pool || h->pool->workers != (workers < 1 ? 1 : workers)) h->pool.reset(new oracle::Pool(workers));
  int done = 0;
  while (done < n && h->next < (int)h->c.queue.size()) {
    int q = h->next++;
    h->c.schedule_one(q, h->c.queue[q], *h->pool, record);
    ++done;
  }
  return done;
}

// What-if step: the next n queue pods each scheduled against the current
// snapshot (no assume between them), then all their placements bound in queue
// order.  Returns pods processed.
int ksg_oracle_whatif(ksg_oracle* h, int n, int workers, int record) {
  h->c.defer_assume = true;
  h->c.deferred.clear();
  int done = ksg_oracle_schedule(h, n, workers, record);
  h->c.defer_assume = false;
  for (auto& pn : h->c.deferred) h->c.add_pod(pn.first, pn.second);
  h->c.deferred.clear();
  return done;
}

// per queue pod: selected node index (-1 none), feasible count, status
int ksg_oracle_result(ksg_oracle* h, int q, int* selected, int* feasible, int* status) {
  if (q < 0 || q >= (int)h->c.results.size()) return -1;
  *selected = h->c.results[q].selected_idx;
  *feasible = h->c.results[q].feasible;
  *status = h->c.results[q].status;
  return 0;
}

unsigned long long ksg_oracle_digest(ksg_oracle* h, int q) { return h->c.digests[q]; }

// DefaultPreemption dry run of queue pod q (record >= 1): nominated node index or -1;
// its victims as "namespace/name" lines (most important first) into buf.
int ksg_oracle_nominated(ksg_oracle* h, int q, char* buf, size_t cap, size_t* len) {
  if (q < 0 || q >= (int)h->c.results.size()) return -2;
  const oracle::PodResult& r = h->c.results[q];
  std::string v;
  for (auto& x : r.victims) v += x + "\n";
  if (len) *len = v.size();
  if (buf && cap >= v.size()) std::memcpy(buf, v.data(), v.size());
  return r.nominated_idx;
}

// Rendered GetStoredResult map (JSON object of annotation key -> value); record >= 3.
const char* ksg_oracle_annotations(ksg_oracle* h, int q, size_t* len) {
  *len = h->c.rendered[q].size();
  return h->c.rendered[q].data();
}

double ksg_oracle_go_log(double x) { return oracle::go_log(x); }

unsigned long long ksg_oracle_pack_key(ksg_oracle* h, long long total, int qidx, int ni) {
  return h->c.pack_key(total, qidx, ni);
}
}
