// Host side of the drop-in: Kubernetes objects (JSON) -> interned device
// snapshot + per-pod programs, result-store rendering, and the C ABI (ksg.h).
//
// What the Go cgo package would do natively lives here in C++ (no Go toolchain
// in this image):  the plugin-facing semantics that are host-known per pod
// (PreFilter Skip rules, PreFilterResult, PodRequests, toleration sets,
// selector compilation) are decided here; everything per (pod, node) runs on
// the GPU (engine.hip).  Recording follows the simulator's wrapper
// (simulator/scheduler/plugin/wrappedplugin.go:388-548, 616-645) and store
// (resultstore/store.go:133-507): filter[node][plugin] = "passed" | message
// up to the first failure, score = raw, finalscore = normalized x store weight
// (raw x weight for plugins without ScoreExtensions), selected node on Reserve.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <thread>
#include <vector>

#include <dlfcn.h>

#include "../../include/ksg.h"
#include "engine.h"
#include "json.hpp"

// ROCTx ranges (KSG_ROCTX=1): the C entry points and ksg_cycle's host phases as
// named ranges for `rocprofv3 --marker-trace`, beside the kernels they launch.
// The ROCTx library is opened at run time, so nothing links against it and a
// run without the variable (or without the library) pays one branch per range.
namespace rtx {
struct Api {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
};
inline const Api& api() {
  static const Api a = [] {
    Api x;
    const char* e = std::getenv("KSG_ROCTX");
    if (!e || std::strtol(e, nullptr, 10) == 0) return x;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return x;
    x.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
    x.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    if (!x.push || !x.pop) x = Api{};
    return x;
  }();
  return a;
}
struct Range {  // one range for the scope
  bool on;
  explicit Range(const char* name) : on(api().push != nullptr) {
    if (on) api().push(name);
  }
  ~Range() {
    if (on) api().pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};
struct Phases {  // consecutive ranges within a scope: next() ends one and starts the next
  bool on, open = false;
  Phases() : on(api().push != nullptr) {}
  void next(const char* name) {
    if (!on) return;
    if (open) api().pop();
    api().push(name);
    open = true;
  }
  ~Phases() {
    if (on && open) api().pop();
  }
};
}  // namespace rtx

namespace ksg {
namespace host {

using std::map;
using std::set;
using std::string;
using std::unordered_map;
using std::vector;
typedef long long i64;
typedef __int128 i128;
typedef json::Node J;

static const char* kHostname = "kubernetes.io/hostname";

// ---------------------------------------------------------------- small helpers
static string str_of(const J* n) { return n ? n->text() : string(); }
static map<string, string> smap(const J* n) {
  map<string, string> m;
  if (n && n->t == J::OBJ)
    for (size_t i = 0; i < n->keys.size(); ++i) m[n->keys[i]] = n->items[i].text();
  return m;
}
static vector<string> slist(const J* n) {
  vector<string> v;
  if (n && n->t == J::ARR)
    for (auto& x : n->items) v.push_back(x.text());
  return v;
}

// strconv.ParseInt(s, 10, 64)
static bool parse_i64(const string& s, i64& out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    if (s.size() == 1) return false;
    i = 1;
  }
  unsigned __int128 v = 0;
  for (; i < s.size(); ++i) {
    if (!std::isdigit((unsigned char)s[i])) return false;
    v = v * 10 + (unsigned)(s[i] - '0');
    if (v > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  out = neg ? (i64)(-(i128)v) : (i64)v;
  return true;
}

// resource.Quantity -> exact nano units; Value()/MilliValue() round up.
// Quantities beyond 10^30 or with exponents beyond +-40 (no Kubernetes object
// carries them) are rejected rather than overflowing.
static bool mul_i128(i128& x, i128 f) {
  static const i128 kMax = (i128)(((unsigned __int128)1 << 126) - 1);
  if (x > kMax / f) return false;
  x *= f;
  return true;
}
static bool quantity(const string& s, i128& nano) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  i128 m = 0;
  int frac = 0, nd = 0;
  bool digits = false, dot = false;
  for (; i < s.size(); ++i) {
    char c = s[i];
    if (std::isdigit((unsigned char)c)) {
      if (m == 0 && c == '0' && !dot) {  // leading zeros
        digits = true;
        continue;
      }
      if (++nd > 30) return false;
      m = m * 10 + (c - '0');
      digits = true;
      if (dot) ++frac;
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (!digits) return false;
  string suf = s.substr(i);
  i128 num = m * 1000000000, den = 1;
  for (int k = 0; k < frac; ++k) den *= 10;  // <= 10^30
  static const char* dec[] = {"n", "u", "m", "", "k", "M", "G", "T", "P", "E"};
  static const int dexp[] = {-9, -6, -3, 0, 3, 6, 9, 12, 15, 18};
  static const char* bin[] = {"Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  bool ok = false;
  for (int k = 0; k < 10 && !ok; ++k)
    if (suf == dec[k]) {
      int e = dexp[k];
      for (; e > 0; --e)
        if (!mul_i128(num, 10)) return false;
      for (; e < 0; ++e)
        if (!mul_i128(den, 10)) return false;
      ok = true;
    }
  for (int k = 0; k < 6 && !ok; ++k)
    if (suf == bin[k]) {
      if (!mul_i128(num, (i128)1 << (10 * (k + 1)))) return false;
      ok = true;
    }
  if (!ok && !suf.empty() && (suf[0] == 'e' || suf[0] == 'E')) {
    i64 e;
    if (!parse_i64(suf.substr(1), e) || e > 40 || e < -40) return false;
    for (; e > 0; --e)
      if (!mul_i128(num, 10)) return false;
    for (; e < 0; ++e)
      if (!mul_i128(den, 10)) return false;
    ok = true;
  }
  if (!ok) return false;
  i128 q = num / den;
  if (q * den != num) q += 1;
  nano = neg ? -q : q;
  return true;
}
static i64 up_div(i128 a, i64 b) {
  i128 q = a / b;
  if (q * b != a && a > 0) ++q;
  if (q > (i128)INT64_MAX) return INT64_MAX;
  if (q < (i128)INT64_MIN) return INT64_MIN;
  return (i64)q;
}
static i64 as_value(i128 nano) { return up_div(nano, 1000000000LL); }
// int64 addition with Go's wrap-around (NodeInfo sums; the device adds the same way)
static inline i64 wadd(i64 a, i64 b) { return (i64)((uint64_t)a + (uint64_t)b); }
static i64 as_milli(i128 nano) { return up_div(nano, 1000000LL); }

typedef map<string, i128> RList;
static RList rlist(const J* n) {
  RList r;
  if (n && n->t == J::OBJ)
    for (size_t i = 0; i < n->keys.size(); ++i) {
      i128 q;
      if (quantity(n->items[i].text(), q)) r[n->keys[i]] = q;
    }
  return r;
}
static bool scalar_name(const string& n) { return n.find('/') != string::npos || n.rfind("hugepages-", 0) == 0; }

// ---------------------------------------------------------------- API objects
struct Taint { string key, value, effect; };
struct Tol {
  string key, op, value, effect;
  bool tolerates(const Taint& t) const {
    if (!effect.empty() && effect != t.effect) return false;
    if (!key.empty() && key != t.key) return false;
    if (op.empty() || op == "Equal") return value == t.value;
    return op == "Exists";
  }
};
static bool tolerated(const vector<Tol>& ts, const Taint& t) {
  for (auto& x : ts)
    if (x.tolerates(t)) return true;
  return false;
}

struct SelReq { string key, op; vector<string> vals; };
struct LSel {             // metav1.LabelSelector after LabelSelectorAsSelector
  bool nothing = true;    // nil selector
  bool err = false;
  vector<SelReq> reqs;    // matchLabels as In, then matchExpressions
  bool matches(const map<string, string>& l) const {
    if (nothing || err) return false;
    for (auto& r : reqs) {
      auto it = l.find(r.key);
      bool has = it != l.end();
      bool in = has && std::find(r.vals.begin(), r.vals.end(), it->second) != r.vals.end();
      bool ok = r.op == "In" ? in : r.op == "NotIn" ? !in : r.op == "Exists" ? has : !has;
      if (!ok) return false;
    }
    return true;
  }
};
static LSel lsel(const J* n) {
  LSel s;
  if (!n || n->null()) return s;
  s.nothing = false;
  for (auto& kv : smap((*n)["matchLabels"])) s.reqs.push_back({kv.first, "In", {kv.second}});
  if (auto* ex = (*n)["matchExpressions"])
    for (auto& e : ex->items) {
      SelReq r{str_of(e["key"]), str_of(e["operator"]), slist(e["values"])};
      bool setop = r.op == "In" || r.op == "NotIn";
      bool exop = r.op == "Exists" || r.op == "DoesNotExist";
      if (r.key.empty() || (!setop && !exop) || (setop && r.vals.empty()) || (exop && !r.vals.empty())) s.err = true;
      s.reqs.push_back(r);
    }
  return s;
}

struct ATerm {  // framework.AffinityTerm
  LSel sel;
  set<string> namespaces;
  bool ns_all = false;  // namespaceSelector matches the (label-less) namespaces
  string topo;
  int32_t weight = 0;
};
static ATerm aterm(const J& t, const string& owner_ns) {
  ATerm a;
  a.sel = lsel(t["labelSelector"]);
  vector<string> nss = slist(t["namespaces"]);
  const J* nsSel = t["namespaceSelector"];
  if (nss.empty() && (!nsSel || nsSel->null())) a.namespaces.insert(owner_ns);
  else a.namespaces.insert(nss.begin(), nss.end());
  LSel ns = lsel(nsSel);
  a.ns_all = ns.matches({});  // namespaces carry no labels in this model
  a.topo = str_of(t["topologyKey"]);
  return a;
}

struct TSC {
  int32_t max_skew = 0;
  string key, when;
  const J* sel = nullptr;
  int32_t min_domains = 1;
  string aff_policy, taint_policy;
  vector<string> match_label_keys;
};

struct Pod {
  string name, ns;
  map<string, string> labels;
  string node;
  bool terminating = false;
  RList req, req_nz;  // PodRequests without / with NonMissingContainerRequests
  bool has_node_sel = false;
  map<string, string> node_sel;
  vector<Tol> tols;
  bool has_req_na = false, has_pref_na = false;
  vector<const J*> req_terms, pref_terms;
  bool pod_aff = false, pod_anti = false, pref_aff_present = false, pref_anti_present = false;
  vector<ATerm> req_aff, req_anti, pref_aff, pref_anti;
  vector<TSC> tsc;
  // rest of the default profile
  vector<string> images;  // init containers then containers (ImageLocality sumImageScores order)
  int n_containers = 0;   // init + regular
  struct HostPort { string ip, proto; int32_t port; };
  vector<HostPort> ports; // Spec.Containers host ports (hostPort > 0), sanitised
  bool volume_plugins_act = false;  // a volume other than a PVC the volume plugins act on (not modelled)
  vector<string> claims;            // spec.volumes[].persistentVolumeClaim.claimName, in volume order
  int32_t doc = -1;                 // index of a JSON document only this pod references (ksg_cycle), or -1
  i64 priority = 0;                 // spec.priority (PrioritySort queue order; DefaultPreemption)
  bool gated = false;               // spec.schedulingGates non-empty (SchedulingGates PreEnqueue)
  bool preempt_never = false;       // spec.preemptionPolicy Never (PodEligibleToPreemptOthers)
  i64 start_time = INT64_MAX;       // status.startTime, epoch seconds; none: started last (GetPodStartTime: now)
};

// RFC 3339 date-time -> seconds since the epoch (the date and time fields; a
// fraction and the offset are ignored: the simulator's objects carry "Z").
// INT64_MAX when the text is not a date-time.
static i64 rfc3339_seconds(const string& t) {
  int f[6] = {0, 0, 0, 0, 0, 0};
  size_t at = 0;
  const char sep[6] = {'-', '-', 'T', ':', ':', 0};
  for (int k = 0; k < 6; ++k) {
    size_t b = at;
    while (at < t.size() && at - b < 9 && t[at] >= '0' && t[at] <= '9') f[k] = f[k] * 10 + (t[at++] - '0');
    if (at == b) return INT64_MAX;
    if (k < 5) {
      if (at >= t.size() || (t[at] != sep[k] && !(k == 2 && t[at] == 't'))) return INT64_MAX;
      ++at;
    }
  }
  // days from 1970-01-01 of the proleptic Gregorian date (era arithmetic, March-based years)
  const i64 y = (i64)f[0] - (f[1] <= 2 ? 1 : 0);
  const i64 era = (y >= 0 ? y : y - 399) / 400;
  const i64 yoe = y - era * 400;
  const i64 mp = (f[1] + 9) % 12;
  const i64 doy = (153 * mp + 2) / 5 + f[2] - 1;
  const i64 days = era * 146097 + yoe * 365 + yoe / 4 - yoe / 100 + doy - 719468;
  return days * 86400 + (i64)f[3] * 3600 + (i64)f[4] * 60 + f[5];
}

static RList pod_requests(const J* spec, bool nonzero) {
  auto fill = [&](RList r) {
    if (nonzero) {
      if (!r.count("cpu")) r["cpu"] = (i128)100 * 1000000;                      // DefaultMilliCPURequest
      if (!r.count("memory")) r["memory"] = (i128)(200LL << 20) * 1000000000;  // DefaultMemoryRequest
    }
    return r;
  };
  auto add = [](RList& a, const RList& b) {
    for (auto& kv : b) a[kv.first] += kv.second;
  };
  auto mx = [](RList& a, const RList& b) {
    for (auto& kv : b) {
      auto it = a.find(kv.first);
      if (it == a.end() || kv.second > it->second) a[kv.first] = kv.second;
    }
  };
  RList reqs, restartable, init;
  if (!spec) return reqs;
  if (auto* cs = (*spec)["containers"])
    for (auto& c : cs->items) {
      const J* res = c["resources"];
      add(reqs, fill(rlist(res ? (*res)["requests"] : nullptr)));
    }
  if (auto* cs = (*spec)["initContainers"])
    for (auto& c : cs->items) {
      const J* res = c["resources"];
      RList cr = fill(rlist(res ? (*res)["requests"] : nullptr));
      if (str_of(c["restartPolicy"]) == "Always") {
        add(reqs, cr);
        add(restartable, cr);
        cr = restartable;
      } else {
        RList t;
        add(t, cr);
        add(t, restartable);
        cr = t;
      }
      mx(init, cr);
    }
  mx(reqs, init);
  add(reqs, rlist((*spec)["overhead"]));
  return reqs;
}

static Pod parse_pod(const J& v) {
  Pod p;
  const J* md = v["metadata"];
  const J* sp = v["spec"];
  p.name = md ? str_of((*md)["name"]) : "";
  p.ns = md ? str_of((*md)["namespace"]) : "";
  if (p.ns.empty()) p.ns = "default";
  p.labels = smap(md ? (*md)["labels"] : nullptr);
  p.terminating = md && (*md)["deletionTimestamp"] && !(*md)["deletionTimestamp"]->null();
  p.req = pod_requests(sp, false);
  p.req_nz = pod_requests(sp, true);
  if (!sp) return p;
  p.node = str_of((*sp)["nodeName"]);
  if (auto* pr = (*sp)["priority"]; pr && !pr->null()) p.priority = (i64)pr->num();
  if (auto* g = (*sp)["schedulingGates"]; g && !g->items.empty()) p.gated = true;
  p.preempt_never = str_of((*sp)["preemptionPolicy"]) == "Never";
  if (const J* st = v["status"])
    if (const J* t = (*st)["startTime"]; t && !t->null()) p.start_time = rfc3339_seconds(str_of(t));
  for (const char* k : {"initContainers", "containers"})
    if (auto* cs = (*sp)[k])
      for (auto& c : cs->items) {
        p.images.push_back(str_of(c["image"]));
        p.n_containers++;
        if (string(k) != "containers") continue;  // v1.30 getContainerPorts / updateUsedPorts: Spec.Containers
        if (auto* ps = c["ports"])
          for (auto& x : ps->items) {
            i64 hp = x["hostPort"] ? (i64)x["hostPort"]->num() : 0;
            if (hp <= 0) continue;
            Pod::HostPort h{str_of(x["hostIP"]), str_of(x["protocol"]), (int32_t)hp};
            if (h.ip.empty()) h.ip = "0.0.0.0";  // HostPortInfo.sanitize
            if (h.proto.empty()) h.proto = "TCP";
            p.ports.push_back(h);
          }
      }
  if (auto* vs = (*sp)["volumes"])
    for (auto& v : vs->items) {
      if (const J* c = v["persistentVolumeClaim"]; c && !c->null()) p.claims.push_back(str_of((*c)["claimName"]));
      for (const char* k : {"ephemeral", "gcePersistentDisk", "awsElasticBlockStore", "rbd", "iscsi", "azureDisk",
                            "cinder", "csi"})
        if (v[k] && !v[k]->null()) p.volume_plugins_act = true;
    }
  if (auto* ns = (*sp)["nodeSelector"]; ns && !ns->null()) {
    p.has_node_sel = true;
    p.node_sel = smap(ns);
  }
  if (auto* ts = (*sp)["tolerations"])
    for (auto& t : ts->items) p.tols.push_back({str_of(t["key"]), str_of(t["operator"]), str_of(t["value"]), str_of(t["effect"])});
  if (auto* aff = (*sp)["affinity"]; aff && !aff->null()) {
    if (auto* na = (*aff)["nodeAffinity"]; na && !na->null()) {
      if (auto* rq = (*na)["requiredDuringSchedulingIgnoredDuringExecution"]; rq && !rq->null()) {
        p.has_req_na = true;
        if (auto* ts = (*rq)["nodeSelectorTerms"])
          for (auto& t : ts->items) p.req_terms.push_back(&t);
      }
      if (auto* pf = (*na)["preferredDuringSchedulingIgnoredDuringExecution"]; pf && !pf->null()) {
        p.has_pref_na = true;
        for (auto& t : pf->items) p.pref_terms.push_back(&t);
      }
    }
    auto pa = [&](const char* k, bool& present, vector<ATerm>& rq, vector<ATerm>& pf, bool& pf_present) {
      const J* x = (*aff)[k];
      if (!x || x->null()) return;
      present = true;
      if (auto* r = (*x)["requiredDuringSchedulingIgnoredDuringExecution"])
        for (auto& t : r->items) rq.push_back(aterm(t, p.ns));
      if (auto* f = (*x)["preferredDuringSchedulingIgnoredDuringExecution"]; f && !f->null()) {
        pf_present = f->size() > 0;
        for (auto& t : f->items) {
          const J* pt = t["podAffinityTerm"];
          ATerm a = pt ? aterm(*pt, p.ns) : ATerm();
          a.weight = (int32_t)(t["weight"] ? t["weight"]->num() : 0);
          pf.push_back(a);
        }
      }
    };
    pa("podAffinity", p.pod_aff, p.req_aff, p.pref_aff, p.pref_aff_present);
    pa("podAntiAffinity", p.pod_anti, p.req_anti, p.pref_anti, p.pref_anti_present);
  }
  if (auto* ts = (*sp)["topologySpreadConstraints"])
    for (auto& c : ts->items) {
      TSC t;
      t.max_skew = (int32_t)(c["maxSkew"] ? c["maxSkew"]->num() : 0);
      t.key = str_of(c["topologyKey"]);
      t.when = str_of(c["whenUnsatisfiable"]);
      t.sel = c["labelSelector"];
      if (c["minDomains"] && !c["minDomains"]->null()) t.min_domains = (int32_t)c["minDomains"]->num();
      t.aff_policy = str_of(c["nodeAffinityPolicy"]);
      t.taint_policy = str_of(c["nodeTaintsPolicy"]);
      t.match_label_keys = slist(c["matchLabelKeys"]);
      p.tsc.push_back(t);
    }
  return p;
}

struct Node {
  string name;
  map<string, string> labels;
  vector<Taint> taints;
  RList alloc;
  bool unschedulable = false;
  vector<std::pair<vector<string>, i64>> images;  // status.images: names, sizeBytes
};
static Node parse_node(const J& v) {
  Node n;
  const J* md = v["metadata"];
  n.name = md ? str_of((*md)["name"]) : "";
  n.labels = smap(md ? (*md)["labels"] : nullptr);
  if (auto* sp = v["spec"])
    if (auto* ts = (*sp)["taints"])
      for (auto& t : ts->items) n.taints.push_back({str_of(t["key"]), str_of(t["value"]), str_of(t["effect"])});
  if (auto* sp = v["spec"])
    if (auto* u = (*sp)["unschedulable"]) n.unschedulable = u->b;
  const J* st = v["status"];
  n.alloc = rlist(st ? (*st)["allocatable"] : nullptr);
  if (st)
    if (auto* im = (*st)["images"])
      for (auto& x : im->items) n.images.push_back({slist(x["names"]), x["sizeBytes"] ? (i64)x["sizeBytes"]->num() : 0});
  return n;
}

// ---------------------------------------------------------------- interning
struct Dict {
  unordered_map<string, int32_t> id;
  vector<string> names;
  int32_t get(const string& s) const {
    auto it = id.find(s);
    return it == id.end() ? -1 : it->second;
  }
  int32_t add(const string& s) {
    auto it = id.find(s);
    if (it != id.end()) return it->second;
    id.emplace(s, (int32_t)names.size());
    names.push_back(s);
    return (int32_t)names.size() - 1;
  }
};

enum { P_FIT = KP_FIT, P_BA = KP_BA, P_TAINT = KP_TAINT, P_NA = KP_NA, P_PTS = KP_PTS, P_IPA = KP_IPA,
       P_UNSCHED = KP_UNSCHED, P_NODENAME = KP_NODENAME, P_PORTS = KP_PORTS, P_IMAGE = KP_IMAGE,
       P_VOLUME = KP_VOLUME, P_VOLBIND = KP_VOLBIND, P_NOOP = KP_NOOP };
// The default profile's plugins (scheduler_test.go:531-557) by original name.
static int plugin_id(const string& n) {
  static const std::pair<const char*, int> tab[] = {
      {"NodeResourcesFit", P_FIT}, {"NodeResourcesBalancedAllocation", P_BA}, {"TaintToleration", P_TAINT},
      {"NodeAffinity", P_NA}, {"PodTopologySpread", P_PTS}, {"InterPodAffinity", P_IPA},
      {"NodeUnschedulable", P_UNSCHED}, {"NodeName", P_NODENAME}, {"NodePorts", P_PORTS}, {"ImageLocality", P_IMAGE},
      {"VolumeRestrictions", P_VOLUME}, {"EBSLimits", P_VOLUME}, {"GCEPDLimits", P_VOLUME},
      {"NodeVolumeLimits", P_VOLUME}, {"AzureDiskLimits", P_VOLUME}, {"VolumeZone", P_VOLUME},
      {"VolumeBinding", P_VOLBIND}, {"SchedulingGates", P_NOOP}, {"PrioritySort", P_NOOP},
      {"DefaultPreemption", P_NOOP}, {"DefaultBinder", P_NOOP}};
  for (auto& t : tab)
    if (n == t.first) return t.second;
  return -1;
}
// ---------------------------------------------------------------- scheduler configuration
// A KubeSchedulerConfiguration / KubeSchedulerProfile (what the simulator's
// ConvertForSimulator hands the framework, plugins.go) → the flat profile
// {plugins, weights, storeWeights, pluginConfig} the engine takes.
//  * plugin order: multiPoint.enabled (the filter order; scores are order-free);
//  * framework weights: upstream v1.30.4 framework.go getScoreWeights over
//    score.enabled ++ multiPoint.enabled — the first entry of a name wins (an
//    explicit Score weight overrides MultiPoint's), 0 → 1;
//  * store weights: getScorePluginWeight (plugins.go:289-304) over the same list —
//    the last entry wins (MultiPoint overwrites), 0 → 1, "Wrapped" suffix stripped.
// The two differ exactly in the quirk of scheduler_test.go:344-407.  Per-extension-
// point sets other than score weights of MultiPoint plugins are refused.
static J jnum(i64 v) {
  J n;
  n.t = J::NUM;
  n.s = std::to_string(v);
  return n;
}
static void jput(J& o, const string& k, J v) {
  for (size_t i = 0; i < o.keys.size(); ++i)
    if (o.keys[i] == k) { o.items[i] = std::move(v); return; }
  o.keys.push_back(k);
  o.items.push_back(std::move(v));
}
static string unwrapped(const string& n) {
  static const string suf = "Wrapped";
  return n.size() > suf.size() && n.compare(n.size() - suf.size(), suf.size(), suf) == 0
             ? n.substr(0, n.size() - suf.size()) : n;
}
static bool profile_from_config(const J& in, J& out, string& err) {
  const J* prof = &in;
  if (const J* ps = in["profiles"]) {
    if (ps->t != J::ARR || ps->items.empty()) { err = "profiles: expected a non-empty list"; return false; }
    prof = &ps->items[0];  // one profile (getScorePluginWeight reads Profiles[0])
  }
  const J* pl = (*prof)["plugins"];
  if (!pl || pl->t != J::OBJ) { err = "profile.plugins: expected an object"; return false; }
  vector<std::pair<string, i64>> mp, sc;  // (name, weight) in order
  auto entries = [&](const J* set, const char* what, vector<std::pair<string, i64>>& dst) -> bool {
    if (!set) return true;
    if (const J* en = (*set)["enabled"]) {
      if (en->t != J::ARR) { err = string(what) + ".enabled: expected a list"; return false; }
      for (auto& e : en->items) {
        const string nm = unwrapped(str_of(e["name"]));
        if (nm.empty()) { err = string(what) + ".enabled: plugin without a name"; return false; }
        const i64 w = e["weight"] ? e["weight"]->num() : 0;
        if (w < 0 || w > INT32_MAX) { err = string(what) + ": weight of " + nm + " out of range"; return false; }
        dst.push_back({nm, w});
      }
    }
    return true;
  };
  for (size_t i = 0; i < pl->keys.size(); ++i) {
    const string& ext = pl->keys[i];
    const J& set = pl->items[i];
    if (ext == "multiPoint") {
      if (!entries(&set, "multiPoint", mp)) return false;
    } else if (ext == "score") {
      if (!entries(&set, "score", sc)) return false;
      if (const J* d = set["disabled"])
        if (!d->items.empty()) { err = "score.disabled: per-extension-point disabling is not supported"; return false; }
    } else {
      for (const char* k : {"enabled", "disabled"})
        if (const J* l = set[k])
          if (!l->items.empty()) {
            err = ext + "." + k + ": per-extension-point plugin sets are not supported (use multiPoint)";
            return false;
          }
    }
  }
  J names;
  names.t = J::ARR;
  set<string> seen;
  for (auto& e : mp) {
    if (plugin_id(e.first) < 0) { err = "unsupported plugin " + e.first; return false; }
    if (!seen.insert(e.first).second) { err = "plugin " + e.first + " already registered"; return false; }
    J s;
    s.t = J::STR;
    s.s = e.first;
    names.items.push_back(s);
  }
  for (auto& e : sc)
    if (!seen.count(e.first)) { err = "score.enabled: " + e.first + " is not a multiPoint plugin"; return false; }
  J fw, sw;
  fw.t = sw.t = J::OBJ;
  vector<std::pair<string, i64>> all(sc);
  all.insert(all.end(), mp.begin(), mp.end());
  for (auto& e : all) {
    const i64 w = e.second == 0 ? 1 : e.second;
    if (!fw[e.first.c_str()]) jput(fw, e.first, jnum(w));  // first wins (framework)
    jput(sw, e.first, jnum(w));                            // last wins (store)
  }
  out = J();
  out.t = J::OBJ;
  jput(out, "plugins", names);
  jput(out, "weights", fw);
  jput(out, "storeWeights", sw);
  if (const J* pc = (*prof)["pluginConfig"]) {
    J m;
    m.t = J::OBJ;
    if (pc->t == J::ARR) {
      for (auto& e : pc->items)
        if (const J* a = e["args"]) jput(m, unwrapped(str_of(e["name"])), *a);
    } else if (pc->t == J::OBJ) {
      m = *pc;
    }
    jput(out, "pluginConfig", m);
  }
  if (const J* s = (*prof)["seed"] ? (*prof)["seed"] : in["seed"]) jput(out, "seed", *s);
  return true;
}

static bool host_only(int p) { return p == P_NOOP; }
static bool is_volume(int p) { return p == P_VOLUME || p == P_VOLBIND; }
// the volume plugins by behaviour (v1.30.4 plugins/volumerestrictions, nodevolumelimits
// non_csi.go / csi.go, volumebinding, volumezone)
enum { VK_NONE = 0, VK_RESTRICT, VK_NONCSI, VK_CSI, VK_ZONE, VK_BIND };
static int volume_kind(const string& n) {
  if (n == "VolumeRestrictions") return VK_RESTRICT;
  if (n == "EBSLimits" || n == "GCEPDLimits" || n == "AzureDiskLimits") return VK_NONCSI;
  if (n == "NodeVolumeLimits") return VK_CSI;
  if (n == "VolumeZone") return VK_ZONE;
  if (n == "VolumeBinding") return VK_BIND;
  return VK_NONE;
}
// extension points the original plugin implements (the wrapper records only those)
static bool has_prefilter(int p) {
  return p == P_FIT || p == P_NA || p == P_PTS || p == P_IPA || p == P_PORTS || p == P_VOLUME || p == P_VOLBIND;
}
static bool has_filter(int p) { return p != P_BA && p != P_IMAGE && p != P_NOOP; }
static bool has_prescore(int p) { return p <= P_IPA || p == P_VOLBIND; }
static bool has_score(int p) { return p <= P_IPA || p == P_IMAGE; }  // VolumeBinding: PreScore Skip (no scorer)

// Per-pod host-known facts the renderer needs besides the device outputs.
struct PodMeta {
  uint32_t flags = 0;
  string prefilter_fail_msg;  // PreFilter rejection (NodeAffinity conflict)
  int prefilter_fail_pos = -1;
  bool prefilter_error = false;
  bool restricted = false;
  vector<string> prefilter_names;  // NodeAffinity PreFilterResult
  bool ipa_no_req_terms = true;
  bool ipa_prescore_skip_static = false;
  bool na_prescore_error = false;
  // volume plugins
  uint32_t vol_skip = 0;           // bit = profile position: PreFilter returned Skip
  bool vb_restricted = false;      // VolumeBinding PreFilterResult (GetEligibleNodes)
  vector<string> vb_names;
  bool merge_reject = false;       // the framework's PreFilterResult merge came out empty at prefilter_fail_pos
};

// ---------------------------------------------------------------- storage objects
// ResourcesForSnap pvs / pvcs / storageClasses (snapshot.go:33-42), as the volume
// plugins of v1.30.4 read them.
struct PVC {
  string ns, name, volume_name, cls;  // cls: storagehelpers.GetPersistentVolumeClaimClass
  bool bind_completed = false;        // pv.kubernetes.io/bind-completed present (isPVCFullyBound)
  bool deleting = false, lost = false, rwop = false;
  bool has_selected = false;          // volume.kubernetes.io/selected-node
  string selected;
};
struct PV {
  string name, cls;                   // cls: GetPersistentVolumeClass
  map<string, string> labels;
  const J* required = nullptr;        // spec.nodeAffinity.required (NodeSelector)
  bool claimed = false;               // spec.claimRef
  string cref_ns, cref_name;
  bool csi = false, intree = false;   // spec.csi / an in-tree cloud disk source
  string csi_driver, csi_handle;
};
struct SClass {
  string name, provisioner;
  bool has_mode = false, wffc = false;  // volumeBindingMode set / WaitForFirstConsumer
  const J* allowed = nullptr;           // allowedTopologies
};
static const char* kBetaClassAnn = "volume.beta.kubernetes.io/storage-class";
static PVC parse_pvc(const J& v) {
  PVC c;
  const J* md = v["metadata"];
  const J* sp = v["spec"];
  c.name = md ? str_of((*md)["name"]) : "";
  c.ns = md ? str_of((*md)["namespace"]) : "";
  if (c.ns.empty()) c.ns = "default";
  const J* ann = md ? (*md)["annotations"] : nullptr;
  c.deleting = md && (*md)["deletionTimestamp"] && !(*md)["deletionTimestamp"]->null();
  if (sp) {
    c.volume_name = str_of((*sp)["volumeName"]);
    if (const J* sc = (*sp)["storageClassName"]; sc && !sc->null()) c.cls = sc->text();
    for (auto& m : slist((*sp)["accessModes"])) c.rwop |= m == "ReadWriteOncePod";
  }
  if (ann && (*ann)[kBetaClassAnn]) c.cls = str_of((*ann)[kBetaClassAnn]);
  c.bind_completed = ann && (*ann)["pv.kubernetes.io/bind-completed"];
  if (ann && (*ann)["volume.kubernetes.io/selected-node"]) {
    c.has_selected = true;
    c.selected = str_of((*ann)["volume.kubernetes.io/selected-node"]);
  }
  if (const J* st = v["status"]) c.lost = str_of((*st)["phase"]) == "Lost";
  return c;
}
static PV parse_pv(const J& v) {
  PV p;
  const J* md = v["metadata"];
  const J* sp = v["spec"];
  p.name = md ? str_of((*md)["name"]) : "";
  p.labels = smap(md ? (*md)["labels"] : nullptr);
  const J* ann = md ? (*md)["annotations"] : nullptr;
  if (sp) {
    p.cls = str_of((*sp)["storageClassName"]);
    if (const J* na = (*sp)["nodeAffinity"]; na && !na->null())
      if (const J* rq = (*na)["required"]; rq && !rq->null()) p.required = rq;
    if (const J* cr = (*sp)["claimRef"]; cr && !cr->null()) {
      p.claimed = true;
      p.cref_ns = str_of((*cr)["namespace"]);
      p.cref_name = str_of((*cr)["name"]);
    }
    p.csi = (*sp)["csi"] && !(*sp)["csi"]->null();
    if (p.csi) {
      p.csi_driver = str_of((*(*sp)["csi"])["driver"]);
      p.csi_handle = str_of((*(*sp)["csi"])["volumeHandle"]);
    }
    for (const char* k : {"awsElasticBlockStore", "gcePersistentDisk", "azureDisk", "cinder"})
      if ((*sp)[k] && !(*sp)[k]->null()) p.intree = true;
  }
  if (ann && (*ann)[kBetaClassAnn]) p.cls = str_of((*ann)[kBetaClassAnn]);
  return p;
}
static SClass parse_sc(const J& v) {
  SClass c;
  const J* md = v["metadata"];
  c.name = md ? str_of((*md)["name"]) : "";
  c.provisioner = str_of(v["provisioner"]);
  if (const J* m = v["volumeBindingMode"]; m && !m->null()) {
    c.has_mode = true;
    c.wffc = m->text() == "WaitForFirstConsumer";
  }
  if (const J* a = v["allowedTopologies"]; a && !a->null()) c.allowed = a;
  return c;
}
// in-tree provisioners the non-CSI limits plugins count (non_csi.go matchProvisioner)
static bool intree_provisioner(const string& p) {
  return p == "kubernetes.io/aws-ebs" || p == "kubernetes.io/gce-pd" || p == "kubernetes.io/azure-disk" ||
         p == "kubernetes.io/cinder";
}

struct Cluster {
  // profile
  int n_plugins = 0;  // whole profile (host-only plugins included)
  int plugins[KSG_MAX_PROFILE] = {};
  string names[KSG_MAX_PROFILE];
  i64 fw_w[KSG_MAX_PROFILE] = {}, store_w[KSG_MAX_PROFILE] = {};
  int dpos[KSG_MAX_PROFILE] = {};  // device profile position of each plugin (-1: host-only)
  int fpos[KSG_MAX_PLUGINS] = {};  // profile position of each device position (a volume run: its first plugin)
  int vkind[KSG_MAX_PROFILE] = {};  // VK_* of each profile position
  int n_dev = 0;
  bool has_volume_plugins = false;
  Dict images;  // ImageLocality: every image name some node lists
  vector<std::pair<i64, int32_t>> image_state;  // per image: Size (first node listing it), NumNodes
  std::map<std::tuple<string, string, int32_t>, int32_t> port_id;  // host-port triples (ip, protocol, port)
  EngineConfig ecfg;
  vector<string> fit_res_names{"cpu", "memory"}, ba_res_names{"cpu", "memory"};
  i64 ipa_hard = 1;
  bool ipa_ignore = false;
  // objects
  vector<Node> nodes;
  Dict node_names;
  vector<Pod> bound;
  vector<int32_t> bound_row;  // per bound pod: its existing-pod table row on this shard's device (-1 none)
  bool inplace_dirty = false;  // cluster events applied in place since the last encode
  std::unordered_map<string, uint32_t> bound_at;  // "ns\x1fname" -> index in bound (in-place events)
  bool bound_at_valid = false;
  vector<Pod> queue;
  // storage (volume plugins)
  std::map<string, PVC> pvcs;  // "ns/name"
  std::map<string, PV> pvs;
  std::map<string, SClass> classes;
  map<string, map<string, i64>> csi_counts;  // CSINode: node -> driver -> allocatable count
  Dict pvc_ids;                // PVC keys "ns/name" the pods use (device use counts)
  Dict lkeys;                  // NodeVolumeLimits limit keys (attachable-volumes-csi-<driver>)
  Dict vols;                   // CSI volumes (driver/handle) the pods use
  // vocabularies
  Dict res;  // resource columns
  Dict nkeys;
  vector<Dict> nvals;
  Dict pkeys;
  vector<Dict> pvals;
  Dict nss;
  std::map<std::tuple<string, string, string>, int32_t> taint_id;
  vector<Taint> taints;
  Dict topo;  // topology key name -> slot
  // shard
  uint32_t rank = 0, shards = 1, lo = 0, hi = 0;
  // device
  std::unique_ptr<Engine> eng;
  vector<PodMeta> meta;
  bool compiled = false;
  uint32_t keep_first = 0, keep_n = 0;
  string err;
  bool broken = false;  // a device error left the snapshot half-updated: refuse calls until reload

  // ------------------------------------------------------------ profile
  bool load_profile(const J& pr) {
    vcfg_ok_ = false;
    if (pr["profiles"] || (pr["plugins"] && pr["plugins"]->t == J::OBJ)) {  // scheduler configuration form
      J flat;
      if (!profile_from_config(pr, flat, err)) return false;
      return load_profile(flat);
    }
    const J* pl = pr["plugins"];
    if (!pl) { err = "profile.plugins missing"; return false; }
    for (auto& x : pl->items) {
      int id = plugin_id(x.text());
      if (id < 0) { err = "unsupported plugin " + x.text(); return false; }
      if (n_plugins >= KSG_MAX_PROFILE) { err = "too many plugins"; return false; }
      names[n_plugins] = x.text();
      plugins[n_plugins++] = id;
    }
    auto weights = smap(pr["weights"]), sw = smap(pr["storeWeights"]);
    for (int i = 0; i < n_plugins; ++i) {
      i64 w = 0, s = 0;
      if (weights.count(names[i])) parse_i64(weights[names[i]], w);
      if (sw.count(names[i])) parse_i64(sw[names[i]], s);
      fw_w[i] = w == 0 ? 1 : w;
      store_w[i] = sw.count(names[i]) ? (s == 0 ? 1 : s) : 0;
    }
    {  // the selection key (pack_key) holds the weighted total in 24 bits: a node's total is at
       // most 100 (MaxNodeScore) x the sum of the weights, so that sum is bounded here, loudly
      i64 wsum = 0;
      for (int i = 0; i < n_plugins; ++i) {
        if (fw_w[i] < 0) { err = "profile: negative weight of " + names[i]; return false; }
        wsum += fw_w[i] < ((i64)1 << 24) ? fw_w[i] : ((i64)1 << 24);
      }
      if (100 * wsum >= ((i64)1 << 24)) {
        err = "profile: 100 x the sum of the plugin weights must be below 2^24 (the selection key's score field)";
        return false;
      }
    }
    if (const J* s = pr["seed"]) ecfg.seed = std::strtoull(s->text().c_str(), nullptr, 10);
    if (const J* pc = pr["pluginConfig"]) {
      if (const J* fit = (*pc)["NodeResourcesFit"])
        if (const J* ss = (*fit)["scoringStrategy"]) {
          string t = str_of((*ss)["type"]);
          ecfg.fit_strategy = t == "MostAllocated" ? 1 : t == "RequestedToCapacityRatio" ? 2 : 0;
          if (const J* rs = (*ss)["resources"]) {
            fit_res_names.clear();
            ecfg.fit_n = 0;
            for (auto& r : rs->items) {
              if (ecfg.fit_n >= KSG_MAX_SCORE_RES) break;
              fit_res_names.push_back(str_of(r["name"]));
              ecfg.fit_w[ecfg.fit_n++] = r["weight"] ? r["weight"]->num() : 1;
              if (ecfg.fit_w[ecfg.fit_n - 1] < 1 || ecfg.fit_w[ecfg.fit_n - 1] > 100) {  // validation.go
                err = "NodeResourcesFit: resource weight out of 1..100";
                return false;
              }
            }
          }
          if (const J* rtc = (*ss)["requestedToCapacityRatio"])
            if (const J* sh = (*rtc)["shape"])
              for (auto& pt : sh->items) {  // validation.go: utilization 0..100 increasing, score 0..10
                if (ecfg.rtc_n >= KSG_MAX_RTC || !pt["utilization"] || !pt["score"]) {
                  err = "requestedToCapacityRatio: invalid shape";
                  return false;
                }
                const i64 u = pt["utilization"]->num(-1), sc = pt["score"]->num(-1);
                if (u < 0 || u > 100 || sc < 0 || sc > 10 || (ecfg.rtc_n > 0 && u <= ecfg.rtc_util[ecfg.rtc_n - 1])) {
                  err = "requestedToCapacityRatio: invalid shape";
                  return false;
                }
                ecfg.rtc_util[ecfg.rtc_n] = u;
                ecfg.rtc_score[ecfg.rtc_n++] = sc * (100 / 10);  // MaxNodeScore / MaxCustomPriorityScore
              }
        }
      if (ecfg.fit_strategy == 2 && ecfg.rtc_n == 0) {
        err = "requestedToCapacityRatio: shape required";
        return false;
      }
      if (const J* ba = (*pc)["NodeResourcesBalancedAllocation"])
        if (const J* rs = (*ba)["resources"]) {
          ba_res_names.clear();
          for (auto& r : rs->items)
            if (ba_res_names.size() < KSG_MAX_SCORE_RES) ba_res_names.push_back(str_of(r["name"]));
        }
      if (const J* ipa = (*pc)["InterPodAffinity"]) {
        if (const J* h = (*ipa)["hardPodAffinityWeight"]) ipa_hard = h->num();
        if (const J* ig = (*ipa)["ignorePreferredTermsOfExistingPods"]) ipa_ignore = ig->b;
      }
    }
    n_dev = 0;
    for (int i = 0; i < n_plugins; ++i) {
      const bool vol = is_volume(plugins[i]);
      has_volume_plugins |= vol;
      vkind[i] = volume_kind(names[i]);
      dpos[i] = -1;
      if (host_only(plugins[i])) continue;
      if (vol && i > 0 && is_volume(plugins[i - 1])) {  // consecutive volume plugins share one KP_VOLUMES position
        dpos[i] = dpos[i - 1];
        continue;
      }
      if (n_dev >= KSG_MAX_PLUGINS) { err = "too many plugins with device work"; return false; }
      dpos[i] = n_dev;
      fpos[n_dev] = i;
      ecfg.plugins[n_dev] = vol ? KP_VOLUMES : plugins[i];
      ecfg.weight[n_dev] = fw_w[i];
      n_dev++;
    }
    ecfg.n_plugins = n_dev;
    ecfg.ba_n = (int)ba_res_names.size();
    ecfg.ipa_hard_weight = ipa_hard;
    ecfg.ipa_ignore_existing_pref = ipa_ignore;
    return true;
  }

  int pos_of(int plugin) const {
    for (int i = 0; i < n_plugins; ++i)
      if (plugins[i] == plugin) return i;
    return -1;
  }

  // ------------------------------------------------------------ class tables
  // Registry of the pod classes and term classes the device keeps counts for
  // (ksg_types.h "class tables"; engine add_classes).  Class ids are stable
  // until the next encode; a program lists the classes it belongs to / that
  // apply to it, refreshed when classes are added after it was compiled.
  struct PClass {
    bool excl = false;     // terminating pods never match (PodTopologySpread)
    vector<ATerm> terms;   // conjunction
  };
  struct TClass {
    int group = 0;         // KSG_TC_*
    string topo;           // topology key
    int32_t slot = -1;
    uint32_t off = 0;      // offset of its values in the device pool (per pair, or per node)
    ATerm term;
  };
  vector<PClass> pcls;
  vector<TClass> tcls;
  // Candidate index over the registry's selector conjunctions: every class is
  // filed under one necessary condition of its selectors -- an In requirement's
  // (key, value) pairs, else an Exists key -- or, with neither, checked for every
  // pod.  A pod's candidates are the classes filed under its labels plus the
  // unfiled ones, in id order; pclass_matches / term_matches then decide exactly.
  // compile() lists a pod's class memberships through it: O(matching classes)
  // instead of a scan of the registry per pod (250,000 bound pods' victim
  // programs, the drop-in cycle's compile).
  struct SelIndex {
    size_t n = 0;  // classes filed
    std::unordered_map<string, vector<int32_t>> kv, key;
    vector<int32_t> always;
    void add(const vector<const LSel*>& sels, int32_t id) {
      const SelReq* best = nullptr;
      for (auto* sl : sels)
        for (auto& r : sl->reqs) {
          if (r.op == "In" && !r.vals.empty() &&
              (!best || best->op != "In" || r.vals.size() < best->vals.size()))
            best = &r;
          else if (r.op == "Exists" && !best)
            best = &r;
        }
      if (!best) {
        always.push_back(id);
      } else if (best->op == "In") {
        vector<string> v(best->vals);
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        for (auto& x : v) kv[best->key + '\x1f' + x].push_back(id);
      } else {
        key[best->key].push_back(id);
      }
    }
    void candidates(const map<string, string>& labels, vector<int32_t>& out) const {
      out = always;
      for (auto& l : labels) {
        auto it = kv.find(l.first + '\x1f' + l.second);
        if (it != kv.end()) out.insert(out.end(), it->second.begin(), it->second.end());
        auto jt = key.find(l.first);
        if (jt != key.end()) out.insert(out.end(), jt->second.begin(), jt->second.end());
      }
      std::sort(out.begin(), out.end());
    }
  };
  SelIndex pidx, tidx;
  void sync_index() {
    for (; pidx.n < pcls.size(); ++pidx.n) {
      vector<const LSel*> v;
      for (auto& t : pcls[pidx.n].terms) v.push_back(&t.sel);
      pidx.add(v, (int32_t)pidx.n);
    }
    for (; tidx.n < tcls.size(); ++tidx.n) tidx.add({&tcls[tidx.n].term.sel}, (int32_t)tidx.n);
  }
  unordered_map<string, int32_t> pcls_id, tcls_id;
  // node topology keys (class-table path eligibility), this shard's nodes
  vector<uint32_t> node_slots;             // per node: bit s = carries topology slot s's key
  vector<uint32_t> slot_nodes;             // per slot: nodes carrying its key
  std::unordered_map<uint32_t, uint32_t> keyset_nodes;  // slot mask -> nodes carrying every key of it
  vector<uint32_t> enc_topo_count;
  vector<uint8_t> enc_topo_unique;
  vector<uint32_t> enc_nu_base;  // per slot: base among the shared-key pairs (UINT32_MAX: one node per value)
  vector<uint32_t> enc_topo_base;
  vector<int32_t> enc_slot_dom;  // per slot: values present on this shard's nodes
  uint32_t enc_N = 0, enc_NU = 0;
  uint32_t tc_total = 0;         // term-class value pool entries assigned (offsets follow class order)
  // a class-table count reference for topology slot `slot`: the key's base among
  // the shared-key pairs, -1 for a key with one node per value (the node's count)
  int32_t nub_of(int32_t slot) const {
    if (slot < 0 || (size_t)slot >= enc_nu_base.size() || enc_nu_base[slot] == 0xFFFFFFFFu) return -1;
    return (int32_t)enc_nu_base[slot];
  }

  static void key_sel(string& k, const LSel& s) {
    k += s.nothing ? 'N' : (s.err ? 'E' : 'S');
    for (auto& r : s.reqs) {
      k += '\x1e';
      k += r.key;
      k += '\x1d';
      k += r.op;
      for (auto& v : r.vals) {
        k += '\x1c';
        k += v;
      }
    }
  }
  static void key_term(string& k, const ATerm& a) {
    k += a.ns_all ? 'A' : 'L';
    for (auto& n : a.namespaces) {
      k += '\x1f';
      k += n;
    }
    k += '|';
    key_sel(k, a.sel);
  }
  // pod class of the conjunction `terms` (-1: matches no pod)
  int32_t pclass(bool excl, const vector<ATerm>& terms) {
    if (terms.empty()) return -1;
    for (auto& t : terms)
      if (t.sel.nothing || t.sel.err) return -1;
    string k(excl ? "X" : "I");
    for (auto& t : terms) {
      k += '#';
      key_term(k, t);
    }
    auto it = pcls_id.find(k);
    if (it != pcls_id.end()) return it->second;
    const int32_t id = (int32_t)pcls.size();
    PClass c;
    c.excl = excl;
    for (auto& t : terms) {
      ATerm a;
      a.sel = t.sel;
      a.namespaces = t.namespaces;
      a.ns_all = t.ns_all;
      c.terms.push_back(std::move(a));
    }
    pcls.push_back(std::move(c));
    pcls_id.emplace(std::move(k), id);
    return id;
  }
  // term class of an existing pod's term of `kind` (0 required affinity, 1 required
  // anti, 2/3 preferred); -1 matches nothing / no topology slot
  int32_t tclass(int kind, const ATerm& a) {
    if (a.sel.nothing || a.sel.err || topo.get(a.topo) < 0) return -1;
    const int group = kind == 0 ? KSG_TC_HARD : kind == 1 ? KSG_TC_ANTI : KSG_TC_PREF;
    string k = std::to_string(group) + '@' + a.topo + '@';
    key_term(k, a);
    auto it = tcls_id.find(k);
    if (it != tcls_id.end()) return it->second;
    const int32_t id = (int32_t)tcls.size();
    TClass c;
    c.group = group;
    c.topo = a.topo;
    c.slot = topo.get(a.topo);
    c.off = tc_total;
    const bool one = (size_t)c.slot < enc_topo_unique.size() && enc_topo_unique[c.slot];
    tc_total += std::max<uint32_t>(one ? enc_N : ((size_t)c.slot < enc_topo_count.size() ? enc_topo_count[c.slot] : 0), 1);
    c.term.sel = a.sel;
    c.term.namespaces = a.namespaces;
    c.term.ns_all = a.ns_all;
    tcls.push_back(std::move(c));
    tcls_id.emplace(std::move(k), id);
    return id;
  }
  static bool term_matches(const ATerm& t, const Pod& p) {
    return (t.ns_all || t.namespaces.count(p.ns)) && t.sel.matches(p.labels);
  }
  static bool pclass_matches(const PClass& c, const Pod& p) {
    if (c.excl && p.terminating) return false;
    for (auto& t : c.terms)
      if (!term_matches(t, p)) return false;
    return true;
  }
  // PodTopologySpread constraint selector with matchLabelKeys merged (v1.30 PreFilter)
  static LSel tsc_selector(const Pod& p, const TSC& c) {
    LSel s = lsel(c.sel);
    if (!c.match_label_keys.empty() && !s.nothing)
      for (auto& k : c.match_label_keys) {
        auto it = p.labels.find(k);
        if (it != p.labels.end()) s.reqs.push_back({k, "In", {it->second}});
      }
    return s;
  }
  int32_t tsc_class(const Pod& p, const LSel& s) {  // countPodsMatchSelector: Empty() counts nothing
    if (s.nothing || s.err || s.reqs.empty()) return -1;
    ATerm a;
    a.sel = s;
    a.namespaces.insert(p.ns);
    return pclass(true, {a});
  }
  // Register every class pod p's program refers to (compile_queue's first pass).
  void register_classes(const Pod& p) {
    if (!tables_on()) return;
    for (auto& c : p.tsc) tsc_class(p, tsc_selector(p, c));
    for (auto* v : {&p.req_aff, &p.req_anti, &p.pref_aff, &p.pref_anti})
      for (auto& a : *v) pclass(false, {a});
    if (!p.req_aff.empty()) pclass(false, p.req_aff);
    for (auto& a : p.req_aff) tclass(0, a);
    for (auto& a : p.req_anti) tclass(1, a);
    for (auto& a : p.pref_aff) tclass(2, a);
    for (auto& a : p.pref_anti) tclass(3, a);
  }
  // Upload the classes the device has no tables for yet (and build them); prog:
  // the cycle's program, placed in the same upload when *placed comes back true.
  bool sync_classes(const vector<uint8_t>* prog = nullptr, bool* placed = nullptr) {
    if (placed) *placed = false;
    if (!tables_on()) return true;
    ClassUpload u;
    for (uint32_t c = eng->pod_classes(); c < pcls.size(); ++c) {
      ksg_pclass pc{};
      pc.n_terms = (int32_t)pcls[c].terms.size();
      pc.term_off = (int32_t)u.ct.size();
      pc.excl_term = pcls[c].excl ? 1 : 0;
      for (auto& t : pcls[c].terms) {
        ksg_cterm ct{};
        compile_lsel(t.sel, ct.sel, u.creq, u.cval);
        ct.ns_all = t.ns_all ? 1 : 0;
        ct.ns_off = (int32_t)u.cval.size();
        for (auto& ns : t.namespaces) u.cval.push_back(nss.get(ns) < 0 ? -2 : nss.get(ns));
        ct.ns_cnt = (int32_t)t.namespaces.size();
        u.ct.push_back(ct);
      }
      u.pc.push_back(pc);
    }
    for (uint32_t k = eng->term_classes(); k < tcls.size(); ++k) {
      u.tc_slot.push_back(tcls[k].slot);
      u.tc_off.push_back(tcls[k].off);
    }
    return eng->add_classes(u, err, prog, placed);
  }
  // nodes carrying every key of slot mask m
  uint32_t nodes_with_all(uint32_t m) {
    auto it = keyset_nodes.find(m);
    if (it != keyset_nodes.end()) return it->second;
    uint32_t c = 0;
    for (uint32_t x : node_slots) c += (x & m) == m;
    keyset_nodes.emplace(m, c);
    return c;
  }
  // every node with one of the keys of mask m carries all of them
  bool keys_together(uint32_t m) {
    const uint32_t all = nodes_with_all(m);
    for (size_t s = 0; s < slot_nodes.size(); ++s)
      if (((m >> s) & 1u) && slot_nodes[s] != all) return false;
    return true;
  }
  // Class counts each program's lists were computed against (stale-list refresh).
  vector<std::pair<uint32_t, uint32_t>> prog_cls;

  // Can the pod's PodTopologySpread / InterPodAffinity inputs be read from the
  // class tables (the table chain)?  Unsharded; for PodTopologySpread, counting
  // that excludes no node for this pod (no node-inclusion policy narrows it, and
  // every node carrying one of the constraints' keys carries them all), filter
  // keys with at most KSG_TAB_MAXV values shared by several nodes (minMatchNum
  // per block), score keys whose registered values fit a 64-bit mask or sit one
  // per node.  Every other pod runs the scanning chain (k_scan_pods ...).
  bool table_path(const ksg_prog& h) {
    if (pos_of(P_PTS) < 0) return true;
    const bool na_restrict = (h.flags & (KPF_HAS_NODE_SEL | KPF_HAS_REQ_NA)) != 0;
    const int nf = h.n_tsc_filter, ns = h.n_tsc_score;
    auto policy_ok = [&](const ksg_tsc& t) { return !(t.honor_affinity && na_restrict) && !t.honor_taints; };
    if (!(h.flags & KPF_SKIP_PTS_FILTER)) {
      uint32_t m = 0;
      for (int c = 0; c < nf; ++c) {
        const ksg_tsc& t = h.tsc[c];
        if (!policy_ok(t) || enc_topo_unique[t.topo] || enc_topo_count[t.topo] > KSG_TAB_MAXV) return false;
        m |= 1u << t.topo;
      }
      if (!keys_together(m)) return false;
    }
    if (!(h.flags & KPF_SKIP_PTS_SCORE)) {
      uint32_t m = 0;
      for (int c = nf; c < nf + ns; ++c) {
        const ksg_tsc& t = h.tsc[c];
        if (!policy_ok(t)) return false;
        if (!t.is_hostname && t.first_of_key && !enc_topo_unique[t.topo] && enc_topo_count[t.topo] > KSG_TAB_REGV)
          return false;
        m |= 1u << t.topo;
      }
      if (!keys_together(m)) return false;
    }
    return true;
  }
  // The table chain's lookup plan of a compiled program (ksg_look / ksg_ubit):
  // k_eval's per-node class-table counts and the pod-uniform InterPodAffinity
  // map totals, in the order k_eval's reads had them.  False: does not fit.
  template <class Pools>
  bool lookup_plan(ksg_prog& h, const Pools& P) const {
    h.n_lk = h.n_ub = 0;
    bool ok = true;
    auto look = [&](int kind, uint64_t base, int slot, int use, int64_t weight, int aux) {
      if (h.n_lk >= KSG_LK_MAX || base > 0x7FFFFFFFull || weight > INT32_MAX || weight < INT32_MIN || slot < -1 ||
          slot > 254 || kind < 0 || kind > 255 || use < 0 || use > 255 || aux < 0 || aux > 255) {
        ok = false;
        return;
      }
      ksg_look& e = h.lk[h.n_lk++];
      e = ksg_look{};
      e.base = (int32_t)base;
      e.weight = (int32_t)weight;
      e.sku = (uint32_t)(slot + 1) | (uint32_t)kind << 8 | (uint32_t)use << 16 | (uint32_t)aux << 24;
    };
    auto pc_look = [&](int32_t cls, int32_t nub, int slot, int use, int64_t weight, int aux) {
      if (cls < 0) {
        if (use == KLU_AFF) look(KLK_NONE, 0, slot, use, 0, aux);  // a missing value still fails
        return;
      }
      if (nub < 0) look(KLK_PC_NODE, (uint64_t)cls * enc_N, slot, use, weight, aux);
      else look(KLK_PC_DOM, (uint64_t)cls * enc_NU + (uint32_t)nub, slot, use, weight, aux);
    };
    auto ub = [&](int kind, uint64_t idx, int bit) {
      if (!bit) return;
      if (h.n_ub >= KSG_UB_MAX || idx > 0x7FFFFFFFull) { ok = false; return; }
      ksg_ubit& u = h.ub[h.n_ub++];
      u.idx = (int32_t)idx;
      u.kind = (int32_t)kind;
      u.bit = (int32_t)bit;
    };
    const int nf = h.n_tsc_filter, ns = h.n_tsc_score;
    if (pos_of(P_PTS) >= 0) {
      if (!(h.flags & KPF_SKIP_PTS_FILTER))
        for (int c = 0; c < nf; ++c) pc_look(h.tsc[c].eff_cls, h.tsc[c].nub, h.tsc[c].topo, KLU_PTSF, 0, c);
      if (ns > 0 && !(h.flags & KPF_SKIP_PTS_SCORE) && !(h.tab & KTAB_PTS_MULTI)) {
        const ksg_tsc& t = h.tsc[nf];  // pts_count_tab: the constraint's pair count
        if (t.is_hostname) {
          if (t.cls >= 0) look(KLK_PC_NODE, (uint64_t)t.cls * enc_N, t.topo, KLU_PTSS, 0, 0);
        } else {
          for (int k = 0; k < t.sc_n; ++k) pc_look(P.i32[(size_t)t.sc_off + k], t.nub, t.topo, KLU_PTSS, 0, 0);
        }
      }
    }
    if (pos_of(P_IPA) >= 0) {
      const ksg_aterm* aff = P.at.data() + h.aterm_off;
      const ksg_aterm* anti = aff + h.n_req_aff;
      const ksg_aterm* pref = anti + h.n_req_anti;
      const bool has_c = (h.flags & KPF_IPA_HAS_CONSTRAINTS) != 0;
      const bool score_on = !(ipa_ignore && !has_c);
      for (int i = 0; i < h.n_req_aff; ++i) {
        pc_look(h.aff_cls, aff[i].nub, aff[i].topo, KLU_AFF, 0, 0);
        if (h.aff_cls >= 0) ub(1, (uint64_t)h.aff_cls * KSG_MAX_TOPO + aff[i].topo, 1);
      }
      for (int i = 0; i < h.n_req_anti; ++i) pc_look(anti[i].cls, anti[i].nub, anti[i].topo, KLU_ANTI, 0, 0);
      if (has_c)
        for (int i = 0; i < h.n_pref_aff + h.n_pref_anti; ++i) {
          const ksg_aterm& t = pref[i];
          pc_look(t.cls, t.nub, t.topo, KLU_RAW, i < h.n_pref_aff ? (int64_t)t.weight : -(int64_t)t.weight, 0);
          if (t.cls >= 0) ub(1, (uint64_t)t.cls * KSG_MAX_TOPO + t.topo, 8);
        }
      for (int i = 0; i < h.n_tc_match; ++i) {
        const int32_t* e = P.i32.data() + h.tc_match_off + 4 * i;  // (class, offset, slot, group)
        const bool one = (size_t)e[2] < enc_topo_unique.size() && enc_topo_unique[e[2]];
        const int kind = one ? KLK_TC_NODE : KLK_TC_DOM;
        if (e[3] == KSG_TC_ANTI) {
          look(kind, (uint32_t)e[1], e[2], KLU_EXANTI, 0, 0);
          ub(2, (uint32_t)e[0], 4);
        } else if (score_on && (e[3] == KSG_TC_PREF || ipa_hard > 0)) {
          look(kind, (uint32_t)e[1], e[2], KLU_RAW, e[3] == KSG_TC_HARD ? ipa_hard : 1, 0);
          ub(2, (uint32_t)e[0], 8);
        }
      }
    }
    return ok;
  }
  // The pair-level class-table entries the program's evaluation reads and its
  // assume writes, as Bloom filters (ksg_prog tab_rd / tab_md).
  template <class Pools>
  void tab_blooms(ksg_prog& h, const Pools& P) const {
    h.tab_rd = h.tab_md = ~0ull;
    h.nd_rd = h.nd_md = ~0ull;
    if (!(h.tab & KTAB_ON) || enc_NU == 0 || enc_N == 0) return;
    uint64_t rd = 0, md = 0, nrd = 0, nmd = 0;
    for (int i = 0; i < h.n_lk; ++i) {  // (PC_NODE / TC_NODE entries are node-level: nd_rd)
      const ksg_look& e = h.lk[i];
      const int32_t kind = ksg_lk_kind(e.sku);
      if (kind == KLK_PC_DOM) rd |= ksg_tab_bloom(1, (uint32_t)e.base / (uint32_t)enc_NU);
      else if (kind == KLK_TC_DOM) rd |= ksg_tab_bloom(2, (uint32_t)e.base);
      else if (kind == KLK_PC_NODE) nrd |= ksg_tab_bloom(4, (uint32_t)(e.base / (uint64_t)enc_N));
      else if (kind == KLK_TC_NODE) nrd |= ksg_tab_bloom(5, (uint32_t)e.base);
    }
    for (int c = 0; c < h.n_tsc_filter; ++c)  // minMatchNum candidates (pc_dom)
      if (h.tsc[c].eff_cls >= 0) rd |= ksg_tab_bloom(1, (uint32_t)h.tsc[c].eff_cls);
    for (int i = 0; i < h.n_ub; ++i)
      rd |= h.ub[i].kind == 1 ? ksg_tab_bloom(1, (uint32_t)h.ub[i].idx / KSG_MAX_TOPO) : ksg_tab_bloom(3, (uint32_t)h.ub[i].idx);
    for (int i = 0; i < h.n_pc_match; ++i) {
      const uint32_t c = (uint32_t)P.i32[(size_t)h.pc_match_off + i];
      md |= ksg_tab_bloom(1, c);
      nmd |= ksg_tab_bloom(4, c);  // (its pc_cnt entry at the node)
    }
    for (int i = 0; i < h.n_exist_terms; ++i) {
      const ksg_exist_term& e = P.et[(size_t)h.exist_terms_off + i];
      if (e.cls < 0) continue;  // (no class: tc_add writes nothing)
      md |= ksg_tab_bloom(2, (uint32_t)e.toff) | ksg_tab_bloom(3, (uint32_t)e.cls);
      nmd |= ksg_tab_bloom(5, (uint32_t)e.toff);  // (a one-node-per-value key's entry at the node)
    }
    h.tab_rd = rd;
    h.tab_md = md;
    h.nd_rd = nrd;
    h.nd_md = nmd;
  }
  // Recompile queue pod q when classes added since its compile apply to it (its
  // pod-class list must hold every class whose table counts it; its term-class
  // list every term class that applies to it).
  bool refresh_program(uint32_t q) {
    if (!tables_on() || q >= progs.size() || q >= prog_cls.size()) return true;
    const auto at = prog_cls[q];
    if (at.first == pcls.size() && at.second == tcls.size()) return true;
    bool stale = false;
    for (size_t c = at.first; c < pcls.size() && !stale; ++c) stale = pclass_matches(pcls[c], queue[q]);
    for (size_t k = at.second; k < tcls.size() && !stale; ++k) stale = term_matches(tcls[k].term, queue[q]);
    if (!stale) {
      prog_cls[q] = {(uint32_t)pcls.size(), (uint32_t)tcls.size()};
      return true;
    }
    vector<uint8_t> blob;
    PodMeta m;
    if (!compile(queue[q], (int32_t)(seq_base + q), blob, m)) return false;
    if (!sync_classes()) return false;  // (no new classes: the pod's own were registered)
    if (!eng->replace_program(q, blob, err)) return false;
    progs[q] = std::move(blob);
    meta[q] = std::move(m);
    return true;
  }
  bool refresh_programs(uint32_t first, uint32_t count) {
    if (!tables_on()) return true;  // (no class tables: no program to refresh)
    for (uint32_t q = first; q < first + count; ++q)
      if (!refresh_program(q)) return false;
    return true;
  }

  // ------------------------------------------------------------ vocabularies
  // Pod-label space: the pod's namespace, label keys and values, and every key,
  // value and namespace its selectors name.  Interning what selectors name (not
  // only what pods carry) keeps every compiled selector exact when a later pod
  // brings a new label value, key or namespace: the vocabulary then grows in
  // place (grow_vocab) instead of re-encoding the snapshot.
  void intern_pod_labels(const Pod& p) {
    nss.add(p.ns);
    auto val = [&](const string& key, const string* v) {
      int32_t k = pkeys.add(key);
      if ((int32_t)pvals.size() <= k) pvals.resize(k + 1);
      if (v) pvals[k].add(*v);
    };
    for (auto& kv : p.labels) val(kv.first, &kv.second);
    auto sel = [&](const LSel& s) {
      for (auto& r : s.reqs) {
        val(r.key, nullptr);
        for (auto& v : r.vals) val(r.key, &v);
      }
    };
    auto topo_of = [&](const string& key) { topo.add(key); nkeys.add(key); };
    for (auto* v : {&p.req_aff, &p.req_anti, &p.pref_aff, &p.pref_anti})
      for (auto& t : *v) {
        topo_of(t.topo);
        sel(t.sel);
        for (auto& ns : t.namespaces) nss.add(ns);
      }
    for (auto& c : p.tsc) {
      topo_of(c.key);
      sel(tsc_selector(p, c));
    }
  }
  // Could the vocabulary take pod p in place (its topology keys, scalar
  // resources and host ports are known: only pod-label space grows)?
  bool vocab_grows_in_place(const Pod& p) const {
    for (auto* v : {&p.req_aff, &p.req_anti, &p.pref_aff, &p.pref_anti})
      for (auto& t : *v)
        if (topo.get(t.topo) < 0) return false;
    for (auto& c : p.tsc)
      if (topo.get(c.key) < 0) return false;
    for (auto& kv : p.req)
      if (scalar_name(kv.first) && res.get(kv.first) < 0) return false;
    for (auto& h : p.ports)
      if (!port_id.count(std::make_tuple(h.ip, h.proto, h.port))) return false;
    for (auto& c : p.claims)
      if (pvc_ids.get(p.ns + "/" + c) < 0) return false;  // the device PVC use counts: re-encode
    if (has_volume_plugins) {
      vector<std::pair<string, string>> av;
      attachable(p, av);
      for (auto& x : av)
        if (vols.get(x.first) < 0 || lkeys.get(x.second) < 0) return false;
    }
    return true;
  }
  // Intern pod p's label space in place; new label keys widen the device's
  // existing-pod label columns (Engine::grow_table).
  bool grow_vocab(const Pod& p) {
    ++bprog_gen;
    const size_t k0 = pkeys.names.size();
    intern_pod_labels(p);
    if (pkeys.names.size() == k0) return true;
    return eng->grow_table(0, 0, 0, 0, (uint32_t)pkeys.names.size(), err);
  }

  bool build_vocab() {
    pvc_ids = Dict();
    lkeys = Dict();
    vols = Dict();
    for (auto* v : {&bound, &queue})
      for (auto& p : *v)
        for (auto& c : p.claims) pvc_ids.add(p.ns + "/" + c);
    if (has_volume_plugins) {  // NodeVolumeLimits: limit keys and CSI volumes
      for (auto& n : nodes)
        for (auto& kv : n.alloc)
          if (kv.first.rfind("attachable-volumes-", 0) == 0) lkeys.add(kv.first);
      for (auto& kv : csi_counts)
        for (auto& d : kv.second) lkeys.add("attachable-volumes-csi-" + d.first);
      vector<std::pair<string, string>> av;
      for (auto* v : {&bound, &queue})
        for (auto& p : *v) {
          attachable(p, av);
          for (auto& x : av) {
            vols.add(x.first);
            lkeys.add(x.second);
          }
        }
    }
    res = Dict();
    res.add("cpu");
    res.add("memory");
    res.add("ephemeral-storage");
    set<string> scal;
    for (auto& n : nodes)
      for (auto& kv : n.alloc)
        if (scalar_name(kv.first)) scal.insert(kv.first);
    for (auto* v : {&bound, &queue})
      for (auto& p : *v)
        for (auto& kv : p.req)
          if (scalar_name(kv.first)) scal.insert(kv.first);
    for (auto& s : scal) res.add(s);  // sorted: Fit reasons come out in name order
    if (res.names.size() > KSG_MAX_RES) { err = "too many scalar resources"; return false; }
    for (auto& n : nodes)
      for (auto& kv : n.labels) {
        int32_t k = nkeys.add(kv.first);
        if ((int32_t)nvals.size() <= k) nvals.resize(k + 1);
        nvals[k].add(kv.second);
      }
    for (auto& n : nodes)
      for (auto& t : n.taints) {
        auto key = std::make_tuple(t.key, t.value, t.effect);
        if (!taint_id.count(key)) {
          taint_id[key] = (int32_t)taints.size();
          taints.push_back(t);
        }
      }
    for (auto* v : {&bound, &queue})
      for (auto& p : *v) intern_pod_labels(p);
    if (nvals.size() < nkeys.names.size()) nvals.resize(nkeys.names.size());
    // ImageLocality: ImageStateSummary per name (cache addNodeImageStates; NumNodes as in
    // ImageStateSummary.Snapshot: the nodes listing the name)
    images = Dict();
    image_state.clear();
    for (auto& n : nodes) {
      set<int32_t> seen;
      for (auto& im : n.images)
        for (auto& nm : im.first) {
          int32_t id = images.add(nm);
          if ((size_t)id == image_state.size()) image_state.push_back({im.second, 0});
          if (seen.insert(id).second) image_state[id].second++;
        }
    }
    // NodePorts: every host-port triple a bound or queued pod uses
    port_id.clear();
    for (auto* v : {&bound, &queue})
      for (auto& p : *v)
        for (auto& h : p.ports) port_id.emplace(std::make_tuple(h.ip, h.proto, h.port), (int32_t)port_id.size());
    if (port_id.size() > 4096) { err = "too many distinct host ports"; return false; }
    if (topo.names.size() > KSG_MAX_TOPO) { err = "too many topology keys"; return false; }
    if (fit_res_names.size() > KSG_MAX_SCORE_RES || ba_res_names.size() > KSG_MAX_SCORE_RES) {
      err = "too many scoring resources";
      return false;
    }
    for (size_t i = 0; i < fit_res_names.size(); ++i) ecfg.fit_res[i] = res.get(fit_res_names[i]);
    for (size_t i = 0; i < ba_res_names.size(); ++i) ecfg.ba_res[i] = res.get(ba_res_names[i]);
    return true;
  }

  // ------------------------------------------------------------ snapshot encode
  void add_requests(const Pod& p, vector<i64>& out_req, i64& nzc, i64& nzm) {
    out_req.assign(res.names.size(), 0);
    for (auto& kv : p.req) {
      int32_t r = res.get(kv.first);
      if (r < 0) continue;
      out_req[r] = wadd(out_req[r], r == 0 ? as_milli(kv.second) : as_value(kv.second));
    }
    auto c = p.req_nz.find("cpu");
    auto m = p.req_nz.find("memory");
    nzc = c == p.req_nz.end() ? 0 : as_milli(c->second);
    nzm = m == p.req_nz.end() ? 0 : as_value(m->second);
  }

  int32_t pkey_vid(int32_t key, const string& v) const {
    if (key < 0 || key >= (int32_t)pvals.size()) return -2;
    int32_t x = pvals[key].get(v);
    return x < 0 ? -2 : x;
  }

  // label selector -> reqs over pod-label space into (reqs, vals)
  void compile_lsel(const LSel& s, ksg_sel& out, vector<ksg_req>& reqs, vector<int32_t>& vals) {
    out.kind = s.nothing ? 0 : 1;
    out.req_off = (int32_t)reqs.size();
    out.req_cnt = 0;
    out.pad = 0;
    if (s.nothing) return;
    if (s.err) {  // unparsable selector never matches
      out.kind = 0;
      return;
    }
    for (auto& r : s.reqs) {
      ksg_req q{};
      q.key = pkeys.get(r.key);
      q.op = r.op == "In" ? KR_IN : r.op == "NotIn" ? KR_NOT_IN : r.op == "Exists" ? KR_EXISTS : KR_NOT_EXISTS;
      q.val_off = (int32_t)vals.size();
      for (auto& v : r.vals) vals.push_back(pkey_vid(q.key, v));
      q.nvals = (int32_t)r.vals.size();
      if (q.key < 0) q.key = -1;
      reqs.push_back(q);
      out.req_cnt++;
    }
  }

  // The sharded Taint / NodeAffinity window keeps every node's labels and taints
  // on every rank.
  bool global_statics() const { return shards > 1 && (has_plugin("TaintToleration") || has_plugin("NodeAffinity")); }
  // Taint lists of nodes [a, b) as CSR over the taint vocabulary (node order kept:
  // the first untolerated taint names the Filter failure).
  void taint_lists(uint32_t a, uint32_t b, vector<uint32_t>& off, vector<int32_t>& ids) const {
    off.assign(b - a + 1, 0);
    ids.clear();
    for (uint32_t i = a; i < b; ++i) {
      for (auto& t : nodes[i].taints) ids.push_back(taint_id.at(std::make_tuple(t.key, t.value, t.effect)));
      off[i - a + 1] = (uint32_t)ids.size();
    }
  }
  // Can node labels `from` become `to` by rewriting label columns alone?  Every
  // key and value is in the node-label vocabulary (selectors were compiled
  // against it) and no topology key changes value (topology slots, class
  // tables and spread domains stay valid).
  bool labels_in_place(const map<string, string>& from, const map<string, string>& to) const {
    auto ok = [&](const string& key, const string* v) {
      const int32_t k = nkeys.get(key);
      if (k < 0 || topo.get(key) >= 0) return false;
      return !v || nvals[k].get(*v) >= 0;
    };
    for (auto& kv : to) {
      auto it = from.find(kv.first);
      if ((it == from.end() || it->second != kv.second) && !ok(kv.first, &kv.second)) return false;
    }
    for (auto& kv : from)
      if (!to.count(kv.first) && !ok(kv.first, nullptr)) return false;
    return true;
  }

  // Compiled programs of bound pods for the preemption search (DefaultPreemption
  // toggles candidate victims with them), cached by bound index: valid while
  // bprog_gen holds (bumped by every encode, vocabulary growth, node change and
  // event batch: bound indices, vocabulary ids and node columns are then stable)
  // and refreshed like refresh_program when classes were added since.
  struct BProg {
    vector<uint8_t> blob;
    uint32_t npc = 0, ntc = 0;
    uint64_t gen = 0;  // bprog_gen + 1 when valid
  };
  vector<BProg> bprog_cache;
  uint64_t bprog_gen = 0;
  uint64_t node_gen = 0;  // node list / allocatable changes (alloc_cache)
  const vector<uint8_t>* bound_prog(int32_t b) {
    if (bprog_cache.size() < bound.size()) bprog_cache.resize(bound.size());
    BProg& e = bprog_cache[(size_t)b];
    if (e.gen == bprog_gen + 1) {
      if (e.npc == pcls.size() && e.ntc == tcls.size()) return &e.blob;
      bool stale = false;
      for (size_t c = e.npc; c < pcls.size() && !stale; ++c) stale = pclass_matches(pcls[c], bound[b]);
      for (size_t k = e.ntc; k < tcls.size() && !stale; ++k) stale = term_matches(tcls[k].term, bound[b]);
      if (!stale) {
        e.npc = (uint32_t)pcls.size();
        e.ntc = (uint32_t)tcls.size();
        return &e.blob;
      }
    }
    PodMeta m;
    e.blob.clear();
    if (!compile(bound[b], 0, e.blob, m)) return nullptr;
    e.npc = (uint32_t)pcls.size();
    e.ntc = (uint32_t)tcls.size();
    e.gen = bprog_gen + 1;
    return &e.blob;
  }
  // allocatable per resource column and local node (Fit's Filter code rule),
  // rebuilt when node_gen moves
  vector<i64> alloc_cache;
  uint64_t alloc_cache_gen = ~0ull;
  const vector<i64>& node_allocs() {
    if (alloc_cache_gen == node_gen && alloc_cache.size() == res.names.size() * (size_t)(hi - lo)) return alloc_cache;
    const size_t R = res.names.size(), n = hi - lo;
    alloc_cache.assign(R * n, 0);
    for (size_t i = 0; i < n; ++i)
      for (auto& kv : nodes[lo + i].alloc) {
        const int32_t r = res.get(kv.first);
        if (r >= 0) alloc_cache[(size_t)r * n + i] = r == 0 ? as_milli(kv.second) : as_value(kv.second);
      }
    alloc_cache_gen = node_gen;
    return alloc_cache;
  }
  // bound pods grouped by local node (bcsr_idx[boff[i] .. boff[i + 1]), load order),
  // rebuilt when bprog_gen moves
  vector<uint32_t> bcsr_off;
  vector<int32_t> bcsr_idx;
  uint64_t bcsr_gen = ~0ull;
  const vector<uint32_t>& bound_by_node() {
    const uint32_t n = hi - lo;
    if (bcsr_gen == bprog_gen && bcsr_off.size() == (size_t)n + 1 && bcsr_idx.size() <= bound.size()) return bcsr_off;
    vector<int32_t> at(bound.size(), -1);
    bcsr_off.assign((size_t)n + 1, 0);
    for (size_t b = 0; b < bound.size(); ++b) {
      const int32_t g = node_names.get(bound[b].node);
      if (g < (int32_t)lo || g >= (int32_t)hi) continue;
      at[b] = g - (int32_t)lo;
      ++bcsr_off[at[b] + 1];
    }
    for (uint32_t i = 0; i < n; ++i) bcsr_off[i + 1] += bcsr_off[i];
    bcsr_idx.assign(bcsr_off[n], 0);
    vector<uint32_t> fill(bcsr_off.begin(), bcsr_off.end() - 1);
    for (size_t b = 0; b < bound.size(); ++b)
      if (at[b] >= 0) bcsr_idx[fill[at[b]]++] = (int32_t)b;
    bcsr_gen = bprog_gen;
    return bcsr_off;
  }
  // The device-resident victim store (Engine::victim_store): every bound pod's
  // program, current while bprog_gen and the class registry hold.
  // bound victims that make a search upload the store (KSG_VICTIM_STORE_MIN: tests force it)
  size_t victim_store_min = std::getenv("KSG_VICTIM_STORE_MIN") ? std::strtoull(std::getenv("KSG_VICTIM_STORE_MIN"), nullptr, 10) : 2048;
  uint64_t vstore_gen = ~0ull;
  size_t vstore_n = 0, vstore_npc = 0, vstore_ntc = 0;
  const void* vstore_eng = nullptr;
  bool victim_store_current() const {
    return vstore_eng == eng.get() && vstore_gen == bprog_gen && vstore_n == bound.size() && vstore_npc == pcls.size() &&
           vstore_ntc == tcls.size();
  }
  // Background warm-up of the victim store after a load (round 6): a thread of the
  // context (ksg_ctx::warm) compiles the bound pods' programs in slices under the
  // context lock and uploads the store, so the first DefaultPreemption search of a
  // snapshot finds it current instead of compiling 250,000 programs itself.  A
  // slice stops the warm-up when the state moved (events, vocabulary growth,
  // another load): the search then builds what it needs, as before.
  size_t warm_next = 0;
  uint64_t warm_gen = 0;
  bool warm_started = false, warm_done = false, warm_running = false;
  double warm_t0 = 0, warm_ms = -1;  // diagnostic: wall time from the load to the store being current
  bool warm_wanted() const {
    const char* e = std::getenv("KSG_VICTIM_WARM");
    if (e && std::strtol(e, nullptr, 10) == 0) return false;
    return has_preemption() && shards == 1 && tables_on() && bound.size() >= std::max<size_t>(victim_store_min, 1);
  }
  // one slice of up to n programs; true when the warm-up is over
  bool warm_step(size_t n) {
    if (!warm_started) {
      if (!compile_queue()) return true;  // (the queue's classes first: the store is built against them)
      warm_started = true;
      warm_gen = bprog_gen;
      warm_next = 0;
    }
    if (warm_gen != bprog_gen || broken) return true;
    const size_t end = std::min(bound.size(), warm_next + n);
    for (; warm_next < end; ++warm_next)
      if (!bound_prog((int32_t)warm_next)) return true;
    if (warm_next < bound.size()) return false;
    warm_done = ensure_victim_store();
    if (warm_done) warm_ms = (now_us() - warm_t0) / 1e3;
    return true;
  }
  bool ensure_victim_store() {
    if (victim_store_current()) return true;
    vector<const vector<uint8_t>*> pp(bound.size());
    const double t0 = now_us();
    for (size_t b = 0; b < bound.size(); ++b)
      if (!(pp[b] = bound_prog((int32_t)b))) return false;
    const double t1 = now_us();
    if (!eng->victim_store(pp, err)) return false;
    if (std::getenv("KSG_PREEMPT_TRACE"))
      std::fprintf(stderr, "victim store: %zu programs compiled in %.1f ms, uploaded in %.1f ms\n", pp.size(),
                   (t1 - t0) / 1e3, (now_us() - t1) / 1e3);
    vstore_eng = eng.get();
    vstore_gen = bprog_gen;
    vstore_n = bound.size();
    vstore_npc = pcls.size();
    vstore_ntc = tcls.size();
    return true;
  }
  bool encode_snapshot(NodeSoA& S, PodTableSoA& T) {
    ++bprog_gen;
    ++node_gen;
    // a new snapshot: the class registry restarts (the bound pods' terms register first)
    pcls.clear();
    tcls.clear();
    pidx = SelIndex();
    tidx = SelIndex();
    pcls_id.clear();
    tcls_id.clear();
    prog_cls.clear();
    uint32_t G = (uint32_t)nodes.size();
    lo = (uint32_t)((uint64_t)G * rank / shards);
    hi = (uint32_t)((uint64_t)G * (rank + 1) / shards);
    uint32_t n = hi - lo, R = (uint32_t)res.names.size(), K = (uint32_t)nkeys.names.size();
    S = NodeSoA();
    S.n = n;
    S.global_offset = lo;
    S.global_n = G;
    S.n_res = R;
    S.n_keys = K;
    S.alloc.assign((size_t)R * n, 0);
    S.requested.assign((size_t)R * n, 0);
    S.nz_cpu.assign(n, 0);
    S.nz_mem.assign(n, 0);
    S.allowed_pods.assign(n, 0);
    S.pod_count.assign(n, 0);
    S.label_vid.assign((size_t)K * n, -1);
    S.has_labels.assign(n, 0);
    S.node_flags.assign(n, 0);
    S.img_words = ((uint32_t)images.names.size() + 31) / 32;
    S.img_bits.assign((size_t)S.img_words * n, 0);
    S.n_ports = (uint32_t)port_id.size();
    S.port_count.assign((size_t)S.n_ports * n, 0);
    // PVCRefCounts of the bound pods, summed over the whole cluster (IsPVCUsedByPods)
    S.pvc_use.assign(pvc_ids.names.size(), 0);
    for (auto& p : bound)
      if (node_names.get(p.node) >= 0)
        for (auto& c : p.claims) S.pvc_use[pvc_ids.get(p.ns + "/" + c)] += 1;
    // NodeVolumeLimits (csi.go getVolumeLimits: attachable-volumes-* allocatable,
    // CSINode counts over them; attached volumes of the bound pods, each once per node)
    S.n_lkeys = (uint32_t)lkeys.names.size();
    S.n_vols = (uint32_t)vols.names.size();
    S.vol_limit.assign((size_t)S.n_lkeys * n, -1);
    S.vol_attached.assign((size_t)S.n_lkeys * n, 0);
    S.vol_node.assign((size_t)S.n_vols * KSG_VOL_NODES, -1);
    S.vol_ref.assign((size_t)S.n_vols * KSG_VOL_NODES, 0);
    for (uint32_t i = 0; i < n; ++i) {
      const Node& nd = nodes[lo + i];
      for (auto& kv : nd.alloc) {
        const int32_t k = lkeys.get(kv.first);
        if (k >= 0) S.vol_limit[(size_t)k * n + i] = (int32_t)as_value(kv.second);
      }
      auto it = csi_counts.find(nd.name);
      if (it != csi_counts.end())
        for (auto& d : it->second) S.vol_limit[(size_t)lkeys.get("attachable-volumes-csi-" + d.first) * n + i] = (int32_t)d.second;
    }
    if (S.n_vols) {
      vector<std::pair<string, string>> av;
      for (auto& p : bound) {
        const int32_t g = node_names.get(p.node);
        if (g < 0 || (uint32_t)g < lo || (uint32_t)g >= hi) continue;
        const int32_t i = g - (int32_t)lo;
        attachable(p, av);
        for (auto& x : av) {
          const int32_t v = vols.get(x.first);
          int32_t* vn = &S.vol_node[(size_t)v * KSG_VOL_NODES];
          int32_t* vr = &S.vol_ref[(size_t)v * KSG_VOL_NODES];
          int at = -1, empty = -1;
          for (int k = 0; k < KSG_VOL_NODES; ++k) {
            if (vn[k] == i) at = k;
            if (vn[k] < 0 && empty < 0) empty = k;
          }
          if (at < 0) {
            if (empty < 0) { err = "CSI volume " + x.first + " attached to more than 16 nodes (not modelled)"; return false; }
            at = empty;
            vn[at] = i;
            S.vol_attached[(size_t)lkeys.get(x.second) * n + i] += 1;
          }
          vr[at] += 1;
        }
      }
    }
    if (global_statics()) {
      // every node's labels and taints (the sharded Taint / NodeAffinity window's
      // static records cover the whole cluster on every rank)
      S.g_label_vid.assign((size_t)K * G, -1);
      for (uint32_t g = 0; g < G; ++g)
        for (auto& kv : nodes[g].labels)
          S.g_label_vid[(size_t)nkeys.get(kv.first) * G + g] = nvals[nkeys.get(kv.first)].get(kv.second);
      taint_lists(0, G, S.g_taint_off, S.g_taint_id);
    }
    taint_lists(lo, hi, S.taint_off, S.taint_id);
    for (uint32_t i = 0; i < n; ++i) {
      const Node& nd = nodes[lo + i];
      for (auto& kv : nd.alloc) {
        if (kv.first == "pods") S.allowed_pods[i] = (int32_t)as_value(kv.second);
        int32_t r = res.get(kv.first);
        if (r >= 0) S.alloc[(size_t)r * n + i] = r == 0 ? as_milli(kv.second) : as_value(kv.second);
      }
      for (auto& kv : nd.labels) S.label_vid[(size_t)nkeys.get(kv.first) * n + i] = nvals[nkeys.get(kv.first)].get(kv.second);
      S.has_labels[i] = !nd.labels.empty();
      if (nd.unschedulable) S.node_flags[i] |= KSG_NODE_UNSCHEDULABLE;
      for (auto& im : nd.images)
        for (auto& nm : im.first) {
          int32_t id = images.get(nm);
          S.img_bits[(size_t)(id >> 5) * n + i] |= 1u << (id & 31);
        }
    }
    S.key_val_off.assign(K + 1, 0);
    for (uint32_t k = 0; k < K; ++k) {
      S.key_val_off[k + 1] = S.key_val_off[k] + (uint32_t)nvals[k].names.size();
      for (auto& v : nvals[k].names) {
        i64 x = 0;
        bool ok = parse_i64(v, x);
        S.val_num.push_back(ok ? x : 0);
        S.val_num_ok.push_back(ok ? 1 : 0);
      }
    }
    uint32_t pairs = 0;
    for (auto& tk : topo.names) {
      int32_t k = nkeys.get(tk);
      S.topo_key.push_back(k);
      S.topo_base.push_back(pairs);
      uint32_t c = k < 0 ? 0 : (uint32_t)nvals[k].names.size();
      S.topo_count.push_back(c);
      pairs += c;
      // one node per value (e.g. kubernetes.io/hostname): a shard's domains of
      // this key are its own (no exchange of their histograms)
      bool uniq = true;
      if (k >= 0) {
        std::vector<uint8_t> seen(c, 0);
        for (auto& nd : nodes) {
          auto it = nd.labels.find(tk);
          if (it == nd.labels.end()) continue;
          int32_t v = nvals[k].get(it->second);
          if (v < 0) continue;
          if (seen[(size_t)v]++) { uniq = false; break; }
        }
      }
      S.topo_unique.push_back(uniq ? 1 : 0);
    }
    S.topo_pairs = pairs;
    // class tables: pair index space of the keys whose values span nodes, the
    // values present on some node of the cluster, and every node's topology keys
    // and values (the whole cluster: a sharded context's class tables are global,
    // every rank applies the same pair-level deltas, SURVEY §8(e) "Bind delta")
    S.shards = shards;
    S.nu_base.assign(topo.names.size(), 0xFFFFFFFFu);
    S.slot_dom.assign(topo.names.size(), 0);
    S.pair_node.assign(pairs, 0);
    S.nu_pairs = 0;
    for (size_t t = 0; t < topo.names.size(); ++t)
      if (!S.topo_unique[t]) {
        S.nu_base[t] = S.nu_pairs;
        S.nu_pairs += S.topo_count[t];
      }
    S.gtopo.assign(topo.names.size() * (size_t)G, -1);
    node_slots.assign(G, 0);
    slot_nodes.assign(topo.names.size(), 0);
    keyset_nodes.clear();
    for (size_t t = 0; t < topo.names.size(); ++t) {
      const int32_t k = S.topo_key[t];
      if (k < 0) continue;
      for (uint32_t g = 0; g < G; ++g) {
        auto it = nodes[g].labels.find(topo.names[t]);
        if (it == nodes[g].labels.end()) continue;
        const int32_t v = nvals[k].get(it->second);
        if (v < 0) continue;
        S.gtopo[t * (size_t)G + g] = v;
        node_slots[g] |= 1u << t;
        slot_nodes[t]++;
        if (!S.pair_node[S.topo_base[t] + v]) {
          S.pair_node[S.topo_base[t] + v] = 1;
          S.slot_dom[t]++;
        }
      }
    }
    enc_topo_count = S.topo_count;
    enc_topo_unique = S.topo_unique;
    enc_nu_base = S.nu_base;
    enc_topo_base = S.topo_base;
    enc_slot_dom = S.slot_dom;
    enc_N = n;
    enc_NU = S.nu_pairs;
    tc_total = 0;
    // bound pods: NodeInfo aggregates + existing-pod table (this shard's nodes)
    T = PodTableSoA();
    T.n_keys = (uint32_t)pkeys.names.size();
    vector<i64> rq;
    vector<vector<int32_t>> lab;
    bound_row.assign(bound.size(), -1);
    if (tables_on())  // term classes in the order of the whole cluster's bound pods: the same ids on every rank
      for (auto& p : bound)
        if (node_names.get(p.node) >= 0) {
          for (auto& t : p.req_aff) tclass(0, t);
          for (auto& t : p.req_anti) tclass(1, t);
          for (auto& t : p.pref_aff) tclass(2, t);
          for (auto& t : p.pref_anti) tclass(3, t);
        }
    for (size_t bi = 0; bi < bound.size(); ++bi) {
      const Pod& p = bound[bi];
      int32_t g = node_names.get(p.node);
      if (g < 0 || (uint32_t)g < lo || (uint32_t)g >= hi) continue;
      uint32_t i = (uint32_t)g - lo;
      i64 nzc, nzm;
      add_requests(p, rq, nzc, nzm);
      for (uint32_t r = 0; r < R; ++r) S.requested[(size_t)r * n + i] = wadd(S.requested[(size_t)r * n + i], rq[r]);
      S.nz_cpu[i] = wadd(S.nz_cpu[i], nzc);
      S.nz_mem[i] = wadd(S.nz_mem[i], nzm);
      S.pod_count[i] += 1;
      for (auto& h : p.ports) S.port_count[(size_t)port_id[std::make_tuple(h.ip, h.proto, h.port)] * n + i] += 1;
      bound_row[bi] = (int32_t)T.n;
      T.node.push_back((int32_t)i);
      T.ns.push_back(nss.get(p.ns));
      T.flags.push_back(exist_flags(p));
      vector<int32_t> l(T.n_keys, -1);
      for (auto& kv : p.labels) l[pkeys.get(kv.first)] = pvals[pkeys.get(kv.first)].get(kv.second);
      lab.push_back(l);
      append_terms(p, (int32_t)T.n, T.terms, T.term_pod, T.reqs, T.vals);
      T.n++;
    }
    T.label_vid.assign((size_t)T.n_keys * T.n, -1);
    for (uint32_t r = 0; r < T.n; ++r)
      for (uint32_t k = 0; k < T.n_keys; ++k) T.label_vid[(size_t)k * T.n + r] = lab[r][k];
    return true;
  }

  static uint32_t exist_flags(const Pod& p) {
    uint32_t f = 0;
    if (p.terminating) f |= KEF_TERMINATING;
    if (p.pod_aff || p.pod_anti) f |= KEF_WITH_AFFINITY;
    if (!p.req_anti.empty()) f |= KEF_REQ_ANTI;
    return f;
  }

  // existing pod's terms (PodInfo.RequiredAffinityTerms etc., not namespace-merged)
  void append_terms(const Pod& p, int32_t row, vector<ksg_exist_term>& terms, vector<int32_t>* term_pod_v,
                    vector<ksg_req>& reqs, vector<int32_t>& vals) {
    auto add = [&](const ATerm& a, int kind) {
      ksg_exist_term e{};
      e.kind = kind;
      e.weight = a.weight;
      e.topo = topo.get(a.topo);
      e.topo_key = nkeys.get(a.topo);
      compile_lsel(a.sel, e.sel, reqs, vals);
      e.ns_all = a.ns_all ? 1 : 0;
      e.ns_off = (int32_t)vals.size();
      for (auto& ns : a.namespaces) vals.push_back(nss.get(ns) < 0 ? -2 : nss.get(ns));
      e.ns_cnt = (int32_t)a.namespaces.size();
      e.cls = tables_on() ? tclass(kind, a) : -1;
      e.toff = e.cls >= 0 ? (int32_t)tcls[e.cls].off : 0;
      terms.push_back(e);
      if (term_pod_v) term_pod_v->push_back(row);
    };
    for (auto& t : p.req_aff) add(t, 0);
    for (auto& t : p.req_anti) add(t, 1);
    for (auto& t : p.pref_aff) add(t, 2);
    for (auto& t : p.pref_anti) add(t, 3);
  }
  void append_terms(const Pod& p, int32_t row, vector<ksg_exist_term>& terms, vector<int32_t>& term_pod,
                    vector<ksg_req>& reqs, vector<int32_t>& vals) {
    append_terms(p, row, terms, &term_pod, reqs, vals);
  }

  // ------------------------------------------------------------ pod program
  struct Prog {
    ksg_prog h{};
    vector<int32_t> i32;
    vector<uint32_t> u32;
    vector<ksg_req> req;
    vector<ksg_sel> sel;
    vector<ksg_aterm> at;
    vector<ksg_exist_term> et;
    vector<ksg_freq> freq;  // flattened node-label requirements, by req index (KPF_FLAT_NA)
    bool flat_ok = true;
  };
  // The flattened form of node-label requirement P.req[idx] (ksg_types.h ksg_freq);
  // a key with more than 64 values keeps the program on the value-list path.
  void flatten_req(Prog& P, size_t idx) {
    if (P.freq.size() <= idx) P.freq.resize(idx + 1, ksg_freq{-1, KFR_FALSE, 0});  // (in req order)
    const ksg_req& q = P.req[idx];
    ksg_freq& f = P.freq[idx];
    f = ksg_freq{q.key, KFR_FALSE, 0};
    if (q.op == KR_NAME_EQ || q.op == KR_NAME_NE) {
      f.mode = q.op == KR_NAME_EQ ? KFR_NAME_EQ : KFR_NAME_NE;
      f.arg = (uint64_t)q.num;
      return;
    }
    if (q.op == KR_FALSE) return;
    const size_t nv = (q.key >= 0 && (size_t)q.key < nvals.size()) ? nvals[q.key].names.size() : 0;
    if (nv > 64) { P.flat_ok = false; return; }
    const uint64_t all = nv == 64 ? ~0ull : ((1ull << nv) - 1);
    uint64_t m = 0;
    switch (q.op) {
      case KR_IN:
      case KR_NOT_IN:
        for (int i = 0; i < q.nvals; ++i) {
          const int32_t v = P.i32[(size_t)q.val_off + i];
          if (v >= 0 && (size_t)v < nv) m |= 1ull << v;
        }
        f.mode = q.op == KR_IN ? KFR_ANY : KFR_NONE;
        break;
      case KR_EXISTS: m = all; f.mode = KFR_ANY; break;
      case KR_NOT_EXISTS: m = all; f.mode = KFR_NONE; break;
      case KR_GT:
      case KR_LT:
        for (size_t v = 0; v < nv; ++v) {
          i64 x = 0;
          if (!parse_i64(nvals[q.key].names[v], x)) continue;  // (the numeric view: strconv.ParseInt)
          if (q.op == KR_GT ? x > q.num : x < q.num) m |= 1ull << v;
        }
        f.mode = KFR_ANY;
        break;
      default: P.flat_ok = false; return;
    }
    f.arg = m;
  }

  int32_t nval(int32_t key, const string& v) const {
    if (key < 0 || key >= (int32_t)nvals.size()) return -2;
    int32_t x = nvals[key].get(v);
    return x < 0 ? -2 : x;
  }

  // node selector term (component-helpers nodeSelectorTerm); false on parse error
  // labels_only: the node carries only its labels (volume.CheckNodeAffinity): fields read ""
  bool compile_node_term(const J& t, Prog& P, ksg_sel& out, bool labels_only = false) {
    out = ksg_sel{1, (int32_t)P.req.size(), 0, 0};
    vector<ksg_req> rs;
    if (const J* me = t["matchExpressions"])
      for (auto& e : me->items) {
        string op = str_of(e["operator"]), key = str_of(e["key"]);
        vector<string> vals = slist(e["values"]);
        ksg_req q{};
        q.key = nkeys.get(key);
        if (op == "In" || op == "NotIn") {
          if (vals.empty()) return false;
          q.op = op == "In" ? KR_IN : KR_NOT_IN;
          q.val_off = (int32_t)P.i32.size();
          for (auto& v : vals) P.i32.push_back(nval(q.key, v));
          q.nvals = (int32_t)vals.size();
        } else if (op == "Exists" || op == "DoesNotExist") {
          if (!vals.empty()) return false;
          q.op = op == "Exists" ? KR_EXISTS : KR_NOT_EXISTS;
        } else if (op == "Gt" || op == "Lt") {
          i64 thr = 0;
          if (vals.size() != 1 || !parse_i64(vals[0], thr)) return false;
          q.num = thr;
          q.op = op == "Gt" ? KR_GT : KR_LT;
        } else {
          return false;
        }
        if (key.empty()) return false;
        rs.push_back(q);
      }
    if (const J* mf = t["matchFields"])
      for (auto& e : mf->items) {
        string op = str_of(e["operator"]), key = str_of(e["key"]);
        vector<string> vals = slist(e["values"]);
        if ((op != "In" && op != "NotIn") || vals.size() != 1) return false;
        ksg_req q{};
        q.key = -1;
        if (key == "metadata.name" && !labels_only) {
          q.op = op == "In" ? KR_NAME_EQ : KR_NAME_NE;
          q.num = node_names.get(vals[0]);  // -1: no such node
        } else {  // other fields read "" on a node
          bool eq = vals[0].empty();
          bool match = op == "In" ? eq : !eq;
          q.op = match ? KR_NAME_NE : KR_FALSE;
          q.num = -1;
        }
        rs.push_back(q);
      }
    for (auto& q : rs) P.req.push_back(q);
    out.req_cnt = (int32_t)rs.size();
    return true;
  }

  static bool term_empty(const J& t) {
    const J* me = t["matchExpressions"];
    const J* mf = t["matchFields"];
    return (!me || me->size() == 0) && (!mf || mf->size() == 0);
  }

  void fill_aterm(const ATerm& a, Prog& P, ksg_aterm& t) {
    t = ksg_aterm{};
    compile_lsel(a.sel, t.sel, P.req, P.i32);
    t.topo = topo.get(a.topo);
    t.topo_key = nkeys.get(a.topo);
    t.ns_all = a.ns_all ? 1 : 0;
    t.ns_off = (int32_t)P.i32.size();
    for (auto& ns : a.namespaces) P.i32.push_back(nss.get(ns) < 0 ? -2 : nss.get(ns));
    t.ns_cnt = (int32_t)a.namespaces.size();
    t.weight = a.weight;
    t.cls = tables_on() ? pclass(false, {a}) : -1;
    t.nub = nub_of(t.topo);
  }

  // ------------------------------------------------------------ volume plugins
  // Upstream v1.30.4 plugins/volumerestrictions, nodevolumelimits (non_csi.go,
  // csi.go), volumebinding (volume_binding.go, binder.go FindPodVolumes) and
  // volumezone: their PreFilter runs here on the storage objects; each Filter
  // becomes device checks on the node's labels / name (KP_VOLUMES) and, for
  // ReadWriteOncePod claims, on the device's PVC use counts.
  bool has_vkind(int k) const {
    for (int i = 0; i < n_plugins; ++i)
      if (vkind[i] == k) return true;
    return false;
  }
  const PVC* pvc_of(const string& ns, const string& name) const {
    auto it = pvcs.find(ns + "/" + name);
    return it == pvcs.end() ? nullptr : &it->second;
  }
  const PV* pv_of(const string& n) const {
    auto it = pvs.find(n);
    return it == pvs.end() ? nullptr : &it->second;
  }
  const SClass* class_of(const string& n) const {
    auto it = classes.find(n);
    return it == classes.end() ? nullptr : &it->second;
  }
  static bool fully_bound(const PVC& c) { return !c.volume_name.empty() && c.bind_completed; }  // isPVCFullyBound
  bool delay_binding(const PVC& c) const {  // volume.IsDelayBindingMode (a class without a mode is refused)
    if (c.cls.empty()) return false;
    const SClass* sc = class_of(c.cls);
    return sc && sc->has_mode && sc->wffc;
  }
  // nodevolumelimits csi.go filterAttachableVolumes: the pod's CSI volumes as
  // (driver/handle, limit key) — an unbound claim, or one whose PV is missing,
  // counts by its class's provisioner and the claim (getCSIDriverInfoFromSC)
  void attachable(const Pod& p, vector<std::pair<string, string>>& out) const {
    out.clear();
    set<string> seen;
    for (auto& cn : p.claims) {
      const PVC* c = pvc_of(p.ns, cn);
      if (!c) continue;
      string driver, handle;
      const PV* v = c->volume_name.empty() ? nullptr : pv_of(c->volume_name);
      if (!v) {
        const SClass* sc = c->cls.empty() ? nullptr : class_of(c->cls);
        if (sc) {
          driver = sc->provisioner;
          handle = "ksg-" + c->ns + "/" + c->name;
        }
      } else if (v->csi) {
        driver = v->csi_driver;
        handle = v->csi_handle;
      }
      if (driver.empty() || handle.empty() || !seen.insert(driver + "/" + handle).second) continue;
      out.push_back({driver + "/" + handle, "attachable-volumes-csi-" + driver});  // GetCSIAttachLimitKey
    }
  }
  // Inputs whose volume-plugin results this build does not model are refused
  // with an error, never approximated.
  bool volumes_modelled(const Pod& p) {
    if (!has_volume_plugins) return true;
    auto no = [&](const string& why) {
      err = "pod " + p.name + ": " + why + " (not modelled)";
      return false;
    };
    if (p.volume_plugins_act) return no("volumes other than persistentVolumeClaim");
    if (p.claims.empty()) return true;
    if (shards != 1) return no("persistent volume claims on a sharded context");
    if (has_vkind(VK_CSI)) {
      vector<std::pair<string, string>> mine;
      attachable(p, mine);
      for (auto& v : mine) {
        if (v.second.size() >= 63) return no("a CSI driver name whose attach-limit key is hashed");
        set<string> at;  // nodes the volume may be attached to: its bound users' nodes + every queue user
        size_t queued = 0;
        for (auto* list : {&bound, &queue})
          for (auto& o : *list) {
            vector<std::pair<string, string>> theirs;
            attachable(o, theirs);
            for (auto& t : theirs)
              if (t.first == v.first) {
                if (list == &bound) at.insert(o.node);
                else queued++;
              }
          }
        if (at.size() + queued > KSG_VOL_NODES) return no("a CSI volume used on more than 16 nodes");
      }
    }
    const bool rejecting = has_vkind(VK_RESTRICT) || has_vkind(VK_BIND) || has_vkind(VK_ZONE);
    auto users = [&](const string& ns, const string& cn, bool queue_too) {
      int u = 0;
      for (auto* v : {&bound, &queue}) {
        if (v == &queue && !queue_too) continue;
        for (auto& o : *v)
          for (auto& x : o.claims) u += o.ns == ns && x == cn;
      }
      return u;
    };
    for (auto& cn : p.claims) {
      const PVC* c = pvc_of(p.ns, cn);
      if (!c) {
        if (!rejecting) return no("a missing claim no PreFilter rejects");
        continue;
      }
      if (const PV* v = c->volume_name.empty() ? nullptr : pv_of(c->volume_name); v && v->intree)
        return no("an in-tree cloud disk persistent volume");
      if (c->rwop && has_preemption()) {  // RemovePod counts by claim name (volume_restrictions.go)
        if (users(p.ns, cn, false) > 1) return no("a ReadWriteOncePod claim used by several bound pods");
        for (auto* v : {&bound, &queue})
          for (auto& o : *v)
            for (auto& x : o.claims)
              if (x == cn && o.ns != p.ns) return no("a ReadWriteOncePod claim name used in several namespaces");
      }
      if (fully_bound(*c)) continue;
      const SClass* sc = c->cls.empty() ? nullptr : class_of(c->cls);
      if (sc && !sc->has_mode && has_vkind(VK_BIND)) return no("a storage class without volumeBindingMode");
      if (!delay_binding(*c) || !c->volume_name.empty()) continue;
      // a WaitForFirstConsumer claim the scheduler provisions for
      if (intree_provisioner(sc->provisioner) && has_vkind(VK_NONCSI)) return no("an in-tree provisioner");
      for (auto& kv : pvs)
        if (kv.second.cls == c->cls && (!kv.second.claimed || (kv.second.cref_ns == c->ns && kv.second.cref_name == c->name)))
          return no("static persistent volumes a WaitForFirstConsumer claim could bind");
      if (users(p.ns, cn, true) > 1) return no("a WaitForFirstConsumer claim shared by several pods");
    }
    return true;
  }
  // volume.GetLocalPersistentVolumeNodeNames
  static set<string> local_pv_nodes(const PV& v) {
    set<string> out;
    if (!v.required) return out;
    if (const J* ts = (*v.required)["nodeSelectorTerms"])
      for (auto& t : ts->items) {
        bool have = false;
        set<string> nodes;
        if (const J* me = t["matchExpressions"])
          for (auto& e : me->items) {
            if (str_of(e["key"]) != kHostname || str_of(e["operator"]) != "In") continue;
            vector<string> vs = slist(e["values"]);
            set<string> x(vs.begin(), vs.end());
            if (!have) { nodes = x; have = true; }
            else {
              set<string> y;
              for (auto& a : nodes)
                if (x.count(a)) y.insert(a);
              nodes = y;
            }
          }
        out.insert(nodes.begin(), nodes.end());
      }
    return out;
  }
  // A NodeSelector matched against a node carrying only its labels
  // (volume.CheckNodeAffinity): terms into the sel pool; empty or invalid terms
  // never match.
  void pv_affinity_terms(const J& required, Prog& P, int32_t& off, int32_t& cnt) {
    vector<ksg_sel> terms;
    if (const J* ts = required["nodeSelectorTerms"])
      for (auto& t : ts->items) {
        if (term_empty(t)) continue;
        ksg_sel s;
        const size_t r0 = P.req.size(), v0 = P.i32.size();
        if (compile_node_term(t, P, s, true)) terms.push_back(s);
        else { P.req.resize(r0); P.i32.resize(v0); }
      }
    off = (int32_t)P.sel.size();
    cnt = (int32_t)terms.size();
    for (auto& s : terms) P.sel.push_back(s);
  }
  // v1helper.MatchTopologySelectorTerms over a class's allowedTopologies: terms
  // with no expressions or an empty value list select nothing
  void topology_terms(const J& allowed, Prog& P, int32_t& off, int32_t& cnt) {
    vector<ksg_sel> terms;
    for (auto& t : allowed.items) {
      const J* me = t["matchLabelExpressions"];
      if (!me || me->size() == 0) continue;
      ksg_sel s{1, (int32_t)P.req.size(), 0, 0};
      bool ok = true;
      vector<ksg_req> rs;
      for (auto& e : me->items) {
        vector<string> vals = slist(e["values"]);
        if (vals.empty()) { ok = false; break; }
        ksg_req q{};
        q.key = nkeys.get(str_of(e["key"]));
        q.op = KR_IN;
        q.val_off = (int32_t)P.i32.size();
        for (auto& v : vals) P.i32.push_back(nval(q.key, v));
        q.nvals = (int32_t)vals.size();
        rs.push_back(q);
      }
      if (!ok) continue;
      for (auto& q : rs) P.req.push_back(q);
      s.req_cnt = (int32_t)rs.size();
      terms.push_back(s);
    }
    off = (int32_t)P.sel.size();
    cnt = (int32_t)terms.size();
    for (auto& s : terms) P.sel.push_back(s);
  }
  static constexpr const char* kZoneKeys[4] = {"failure-domain.beta.kubernetes.io/zone",
                                               "failure-domain.beta.kubernetes.io/region",
                                               "topology.kubernetes.io/zone", "topology.kubernetes.io/region"};
  bool compile_volumes(const Pod& p, Prog& P, PodMeta& m) {
    ksg_prog& h = P.h;
    h.pvc_off = (int32_t)P.i32.size();  // NodeInfo.PVCRefCounts delta of the pod's assume
    for (auto& cn : p.claims) {
      const int32_t id = pvc_ids.get(p.ns + "/" + cn);
      if (id < 0) { err = "internal: PVC " + cn + " not interned"; return false; }
      P.i32.push_back(id);
    }
    h.n_pvc = (int32_t)p.claims.size();
    if (!has_volume_plugins) return true;
    vector<std::pair<string, string>> av;  // NodeVolumeLimits: attached-volume delta of the assume
    attachable(p, av);
    h.csi_off = (int32_t)P.i32.size();
    for (auto& x : av) {
      const int32_t v = vols.get(x.first), k = lkeys.get(x.second);
      if (v < 0 || k < 0) { err = "internal: CSI volume " + x.first + " not interned"; return false; }
      P.i32.push_back(v);
      P.i32.push_back(k);
    }
    h.n_csi = (int32_t)av.size();
    vector<ksg_vchk> chk;
    int vb_pos = -1;
    for (int pos = 0; pos < n_plugins; ++pos) {
      const int vk = vkind[pos];
      if (vk == VK_NONE) continue;
      if (m.prefilter_fail_pos >= 0 && m.prefilter_fail_pos < pos) break;  // an earlier PreFilter rejected the pod
      const int d = dpos[pos], sub = pos - fpos[d];
      auto add = [&](int kind, uint32_t bits, uint32_t unless, int32_t off, int32_t cnt) {
        chk.push_back(ksg_vchk{d, sub, kind, (int32_t)bits, (int32_t)unless, off, cnt, 0});
      };
      string fail;  // PreFilter UnschedulableAndUnresolvable message
      bool skip = p.claims.empty();
      if (vk == VK_RESTRICT && !skip) {  // readWriteOncePodPVCsForPod + calPreFilterState; Filter satisfyReadWriteOncePod
        vector<int32_t> rw;
        for (auto& cn : p.claims) {
          const PVC* c = pvc_of(p.ns, cn);
          if (!c) { fail = "persistentvolumeclaim \"" + cn + "\" not found"; break; }
          if (c->rwop) rw.push_back(pvc_ids.get(p.ns + "/" + cn));
        }
        if (fail.empty() && !rw.empty()) {
          add(KSG_VCHK_USED, KSG_VOL_RWOP, 0, (int32_t)P.i32.size(), (int32_t)rw.size());
          P.i32.insert(P.i32.end(), rw.begin(), rw.end());
        }
      } else if (vk == VK_BIND && !skip) {
        vb_pos = pos;
        for (auto& cn : p.claims) {  // podHasPVCs
          const PVC* c = pvc_of(p.ns, cn);
          if (!c) fail = "persistentvolumeclaim \"" + cn + "\" not found";
          else if (c->lost)
            fail = "persistentvolumeclaim \"" + c->name + "\" bound to non-existent persistentvolume \"" + c->volume_name + "\"";
          else if (c->deleting) fail = "persistentvolumeclaim \"" + c->name + "\" is being deleted";
          if (!fail.empty()) break;
        }
        vector<const PVC*> bnd, dly;
        bool immediate = false;
        if (fail.empty()) {
          for (auto& cn : p.claims) {  // GetPodVolumeClaims
            const PVC* c = pvc_of(p.ns, cn);
            if (fully_bound(*c)) bnd.push_back(c);
            else if (delay_binding(*c) && c->volume_name.empty()) dly.push_back(c);
            else immediate = true;
          }
          if (immediate) fail = "pod has unbound immediate PersistentVolumeClaims";
        }
        if (fail.empty()) {
          bool have = false, missing = false;  // GetEligibleNodes
          set<string> elig;
          for (auto* c : bnd) {
            const PV* v = pv_of(c->volume_name);
            if (!v) { missing = true; continue; }
            set<string> nn = local_pv_nodes(*v);
            if (nn.empty()) continue;
            if (!have) { elig = nn; have = true; }
            else {
              set<string> y;
              for (auto& a : elig)
                if (nn.count(a)) y.insert(a);
              elig = y;
            }
          }
          if (have && !missing) {
            m.vb_restricted = true;
            m.vb_names.assign(elig.begin(), elig.end());
          }
          for (auto* c : bnd) {  // checkBoundClaims: stops at a missing PV or a mismatch
            const PV* v = pv_of(c->volume_name);
            if (!v) { add(KSG_VCHK_FAIL, KSG_VOL_PV_NOT_EXIST, KSG_VOL_NODE_CONFLICT, 0, 0); break; }
            if (!v->required) continue;
            int32_t off, cnt;
            pv_affinity_terms(*v->required, P, off, cnt);
            add(KSG_VCHK_SELS, KSG_VOL_NODE_CONFLICT, 0, off, cnt);
          }
          vector<const PVC*> prov;  // FindPodVolumes: selected-node claims, then those no static PV matches
          for (auto* c : dly)
            if (c->has_selected) {
              ksg_sel s{1, (int32_t)P.req.size(), 1, 0};
              ksg_req q{};
              q.key = -1;
              const int32_t g = node_names.get(c->selected);
              q.op = g >= 0 ? KR_NAME_EQ : KR_FALSE;
              q.num = g;
              P.req.push_back(q);
              add(KSG_VCHK_SELS, KSG_VOL_BIND_CONFLICT, 0, (int32_t)P.sel.size(), 1);
              P.sel.push_back(s);
              prov.push_back(c);
            }
          for (auto* c : dly)
            if (!c->has_selected) prov.push_back(c);
          for (auto* c : prov) {  // checkVolumeProvisions (capacity: no CSIDriver objects, sufficient)
            const SClass* sc = class_of(c->cls);
            if (sc->provisioner.empty() || sc->provisioner == "kubernetes.io/no-provisioner") {
              add(KSG_VCHK_FAIL, KSG_VOL_BIND_CONFLICT, 0, 0, 0);
              break;
            }
            if (sc->allowed && sc->allowed->size() > 0) {
              int32_t off, cnt;
              topology_terms(*sc->allowed, P, off, cnt);
              add(KSG_VCHK_SELS, KSG_VOL_BIND_CONFLICT, 0, off, cnt);
            }
          }
        }
      } else if (vk == VK_ZONE) {  // getPVbyPod; Filter
        vector<std::pair<int32_t, vector<string>>> topo;  // (node key, zones)
        for (auto& cn : p.claims) {
          if (cn.empty()) { fail = "PersistentVolumeClaim had no name"; break; }
          const PVC* c = pvc_of(p.ns, cn);
          if (!c) { fail = "persistentvolumeclaim \"" + cn + "\" not found"; break; }
          if (c->volume_name.empty()) {
            if (c->cls.empty()) { fail = "PersistentVolumeClaim had no pv name and storageClass name"; break; }
            const SClass* sc = class_of(c->cls);
            if (!sc) { fail = "storageclass.storage.k8s.io \"" + c->cls + "\" not found"; break; }
            if (!sc->has_mode) { fail = "VolumeBindingMode not set for StorageClass \"" + c->cls + "\""; break; }
            if (sc->wffc) continue;
            fail = "PersistentVolume had no name";
            break;
          }
          const PV* v = pv_of(c->volume_name);
          if (!v) { fail = "persistentvolume \"" + c->volume_name + "\" not found"; break; }
          for (const char* key : kZoneKeys) {  // getPVTopologies, volumehelpers.LabelZonesToSet
            auto it = v->labels.find(key);
            if (it == v->labels.end()) continue;
            vector<string> zs;
            bool bad = false;
            size_t at = 0;
            for (;;) {
              size_t k = it->second.find("__", at);
              string z = it->second.substr(at, k == string::npos ? string::npos : k - at);
              size_t b = z.find_first_not_of(" \t\n\r\v\f"), e = z.find_last_not_of(" \t\n\r\v\f");
              z = b == string::npos ? "" : z.substr(b, e - b + 1);
              if (z.empty()) { bad = true; break; }
              zs.push_back(z);
              if (k == string::npos) break;
              at = k + 2;
            }
            if (!bad) topo.push_back({nkeys.get(key), zs});
          }
        }
        skip = fail.empty() && topo.empty();
        if (fail.empty() && !skip) {
          // node without any zone / region label passes; else every PV topology label must match
          ksg_sel none{1, (int32_t)P.req.size(), 4, 0};
          for (const char* key : kZoneKeys) {
            ksg_req q{};
            q.key = nkeys.get(key);
            q.op = KR_NOT_EXISTS;
            P.req.push_back(q);
          }
          ksg_sel all{1, (int32_t)P.req.size(), (int32_t)topo.size(), 0};
          for (auto& t : topo) {
            ksg_req q{};
            q.key = t.first;
            q.op = KR_IN;
            q.val_off = (int32_t)P.i32.size();
            for (auto& z : t.second) P.i32.push_back(nval(q.key, z));
            q.nvals = (int32_t)t.second.size();
            P.req.push_back(q);
          }
          add(KSG_VCHK_SELS, KSG_VOL_ZONE_CONFLICT, 0, (int32_t)P.sel.size(), 2);
          P.sel.push_back(none);
          P.sel.push_back(all);
        }
      }
      if (vk == VK_CSI && !skip && h.n_csi > 0)  // csi.go Filter: attached + new volumes per limit key
        add(KSG_VCHK_LIMIT, KSG_VOL_MAX_COUNT, 0, h.csi_off, h.n_csi);
      // (EBS / GCE / Azure limits: the claims bring no in-tree volume they count,
      // volumes_modelled: every node passes)
      if (skip) m.vol_skip |= 1u << pos;
      if (!fail.empty()) {
        if (m.prefilter_fail_pos < 0 || pos < m.prefilter_fail_pos) {
          m.prefilter_fail_pos = pos;
          m.prefilter_fail_msg = fail;
          h.flags |= KPF_PREFILTER_REJECT;
        }
        break;
      }
    }
    // RunPreFilterPlugins merges the PreFilterResults (NodeAffinity's, VolumeBinding's)
    if (m.vb_restricted && (m.prefilter_fail_pos < 0 || m.prefilter_fail_pos > vb_pos)) {
      vector<string> names = m.vb_names;
      if (m.restricted) {
        vector<string> x;
        for (auto& a : m.prefilter_names)
          if (std::binary_search(m.vb_names.begin(), m.vb_names.end(), a)) x.push_back(a);
        names = x;
      }
      const int at = m.restricted ? std::max(vb_pos, pos_of(P_NA)) : vb_pos;
      if (names.empty()) {  // "node(s) didn't satisfy plugin(s) ..." after the later plugin's PreFilter
        if (m.prefilter_fail_pos < 0 || at < m.prefilter_fail_pos) {
          m.prefilter_fail_pos = at;
          m.prefilter_fail_msg = "success";
          m.merge_reject = true;
          h.flags |= KPF_PREFILTER_REJECT;
        }
      } else {
        h.flags |= KPF_RESTRICT;
        const uint32_t n = hi - lo, w = (n + 31) / 32;
        h.restrict_words = (int32_t)w;
        h.restrict_off = (int32_t)P.u32.size();
        P.u32.resize(P.u32.size() + w, 0);
        for (auto& nm : names) {
          int32_t g = node_names.get(nm);
          if (g >= (int32_t)lo && g < (int32_t)hi) P.u32[h.restrict_off + (g - lo) / 32] |= 1u << ((g - lo) % 32);
        }
      }
    }
    h.vchk_off = (int32_t)P.i32.size();
    h.n_vchk = (int32_t)chk.size();
    for (auto& c : chk) {
      const int32_t* w = reinterpret_cast<const int32_t*>(&c);
      P.i32.insert(P.i32.end(), w, w + 8);
    }
    return true;
  }

  bool compile(const Pod& p, int32_t qidx, vector<uint8_t>& blob, PodMeta& m) {
    Prog P;
    ksg_prog& h = P.h;
    h.queue_idx = qidx;
    h.ns_id = nss.get(p.ns);
    uint32_t R = (uint32_t)res.names.size();
    // incoming pod labels (pod-label space)
    h.n_pod_label_keys = (int32_t)pkeys.names.size();
    h.labels_off = 0;
    P.i32.assign(pkeys.names.size(), -1);
    for (auto& kv : p.labels) P.i32[pkeys.get(kv.first)] = pvals[pkeys.get(kv.first)].get(kv.second);
    // ---- resources
    vector<i64> rq;
    i64 nzc = 0, nzm = 0;
    add_requests(p, rq, nzc, nzm);
    h.nz_cpu = nzc;
    h.nz_mem = nzm;
    bool any_scalar = false;
    for (auto& kv : p.req)
      if (scalar_name(kv.first)) any_scalar = true;
    bool zero = !any_scalar;
    for (uint32_t r = 0; r < R && r < 3; ++r) zero &= rq[r] == 0;
    for (uint32_t r = 0; r < R; ++r) h.req[r] = rq[r];
    if (zero) h.flags |= KPF_ZERO_REQUEST;
    auto res_req = [&](const string& name, bool nonzero) -> i64 {
      const RList& l = nonzero ? p.req_nz : p.req;
      auto it = l.find(name);
      if (it == l.end()) return 0;
      return name == "cpu" ? as_milli(it->second) : as_value(it->second);
    };
    for (size_t i = 0; i < fit_res_names.size(); ++i) h.fit_score_req[i] = res_req(fit_res_names[i], true);
    for (size_t i = 0; i < ba_res_names.size(); ++i) h.ba_req[i] = res_req(ba_res_names[i], false);
    // ---- TaintToleration
    uint32_t words = ((uint32_t)taints.size() + 31) / 32;
    h.taint_words = (int32_t)words;
    h.taint_hard_off = (int32_t)P.u32.size();
    P.u32.resize(P.u32.size() + words, 0);
    h.taint_pref_off = (int32_t)P.u32.size();
    P.u32.resize(P.u32.size() + words, 0);
    vector<Tol> pref_tols;
    for (auto& t : p.tols)
      if (t.effect.empty() || t.effect == "PreferNoSchedule") pref_tols.push_back(t);
    for (size_t t = 0; t < taints.size(); ++t) {
      const Taint& tt = taints[t];
      if ((tt.effect == "NoSchedule" || tt.effect == "NoExecute") && !tolerated(p.tols, tt))
        P.u32[h.taint_hard_off + t / 32] |= 1u << (t % 32);
      if (tt.effect == "PreferNoSchedule" && !tolerated(pref_tols, tt))
        P.u32[h.taint_pref_off + t / 32] |= 1u << (t % 32);
    }
    // ---- NodeAffinity
    if (!p.has_req_na && !p.has_node_sel) h.flags |= KPF_SKIP_NA_FILTER;
    if (!p.node_sel.empty()) {
      h.flags |= KPF_HAS_NODE_SEL;
      h.node_sel = ksg_sel{1, (int32_t)P.req.size(), 0, 0};
      for (auto& kv : p.node_sel) {
        ksg_req q{};
        q.key = nkeys.get(kv.first);
        q.op = KR_IN;
        q.val_off = (int32_t)P.i32.size();
        P.i32.push_back(nval(q.key, kv.second));
        q.nvals = 1;
        P.req.push_back(q);
        h.node_sel.req_cnt++;
      }
    }
    if (p.has_req_na) {
      h.flags |= KPF_HAS_REQ_NA;
      vector<ksg_sel> terms;
      for (auto* t : p.req_terms) {
        if (term_empty(*t)) continue;
        ksg_sel s;
        size_t r0 = P.req.size(), v0 = P.i32.size();
        if (compile_node_term(*t, P, s)) terms.push_back(s);
        else {  // parse error: term never matches
          P.req.resize(r0);
          P.i32.resize(v0);
        }
      }
      h.req_terms_off = (int32_t)P.sel.size();
      h.n_req_terms = (int32_t)terms.size();
      for (auto& s : terms) P.sel.push_back(s);
      // PreFilterResult from matchFields metadata.name In (node_affinity.go PreFilter)
      if (!p.req_terms.empty()) {
        bool names_nil = true, all_named = true;
        set<string> names;
        for (auto* t : p.req_terms) {
          bool tnil = true;
          set<string> tn;
          if (const J* mf = (*t)["matchFields"])
            for (auto& r : mf->items)
              if (str_of(r["key"]) == "metadata.name" && str_of(r["operator"]) == "In") {
                vector<string> v = slist(r["values"]);
                set<string> s(v.begin(), v.end());
                if (tnil) { tn = s; tnil = false; }
                else {
                  set<string> x;
                  for (auto& a : tn)
                    if (s.count(a)) x.insert(a);
                  tn = x;
                }
              }
          if (tnil) { all_named = false; break; }
          names_nil = false;
          names.insert(tn.begin(), tn.end());
        }
        if (all_named && !names_nil) {
          if (names.empty()) {
            m.prefilter_fail_pos = pos_of(P_NA);
            m.prefilter_fail_msg = "pod affinity terms conflict";
            h.flags |= KPF_PREFILTER_REJECT;
          } else {
            m.restricted = true;
            m.prefilter_names.assign(names.begin(), names.end());
            h.flags |= KPF_RESTRICT;
            uint32_t n = hi - lo, w = (n + 31) / 32;
            h.restrict_words = (int32_t)w;
            h.restrict_off = (int32_t)P.u32.size();
            P.u32.resize(P.u32.size() + w, 0);
            for (auto& nm : names) {
              int32_t g = node_names.get(nm);
              if (g >= (int32_t)lo && g < (int32_t)hi) P.u32[h.restrict_off + (g - lo) / 32] |= 1u << ((g - lo) % 32);
            }
            if (shards > 1) {  // (the sharded static records cover every node)
              const uint32_t G = (uint32_t)nodes.size(), wg = (G + 31) / 32;
              h.restrict_g_words = (int32_t)wg;
              h.restrict_g_off = (int32_t)P.u32.size();
              P.u32.resize(P.u32.size() + wg, 0);
              for (auto& nm : names) {
                const int32_t g = node_names.get(nm);
                if (g >= 0) P.u32[h.restrict_g_off + g / 32] |= 1u << (g % 32);
              }
            }
          }
        }
      }
    }
    if (!p.has_pref_na) h.flags |= KPF_SKIP_NA_SCORE;
    else {
      h.pref_terms_off = (int32_t)P.sel.size();
      vector<std::pair<ksg_sel, int32_t>> pts;
      bool bad = false;
      for (auto* t : p.pref_terms) {
        i64 w = (*t)["weight"] ? (*t)["weight"]->num() : 0;
        const J* pref = (*t)["preference"];
        if (w == 0 || !pref || term_empty(*pref)) continue;
        ksg_sel s;
        if (!compile_node_term(*pref, P, s)) { bad = true; continue; }
        pts.push_back({s, (int32_t)w});
      }
      if (bad && pos_of(P_NA) >= 0) { m.na_prescore_error = true; h.flags |= KPF_NA_PREF_ERROR; }
      h.n_pref_terms = (int32_t)pts.size();
      h.pref_w_off = (int32_t)P.i32.size();
      for (auto& x : pts) { P.sel.push_back(x.first); P.i32.push_back(x.second); }
    }
    // ---- volume plugins (their PreFilter state on the host, their Filters as device checks)
    if (!compile_volumes(p, P, m)) return false;
    // ---- PodTopologySpread
    auto build_tsc = [&](const string& when, int& count) -> bool {
      count = 0;
      for (auto& c : p.tsc) {
        if (c.when != when) continue;
        int idx = h.n_tsc_filter + h.n_tsc_score + count;
        if (idx >= KSG_MAX_TSC) { err = "too many topology spread constraints"; return false; }
        ksg_tsc& t = h.tsc[idx];
        t = ksg_tsc{};
        const LSel s = tsc_selector(p, c);
        if (s.err) m.prefilter_error = true;
        compile_lsel(s, t.sel, P.req, P.i32);
        t.cls = tables_on() ? tsc_class(p, s) : -1;
        t.nub = -1;
        t.pair_base = t.nvals = 0;
        t.topo = topo.get(c.key);
        t.topo_key = nkeys.get(c.key);
        t.max_skew = c.max_skew;
        t.min_domains = c.min_domains;
        t.honor_affinity = c.aff_policy.empty() || c.aff_policy == "Honor";
        t.honor_taints = c.taint_policy == "Honor";
        t.self_match = s.matches(p.labels) ? 1 : 0;
        t.is_hostname = c.key == kHostname;
        count++;
      }
      return true;
    };
    int nf = 0, ns = 0;
    if (!build_tsc("DoNotSchedule", nf)) return false;
    h.n_tsc_filter = nf;
    if (!build_tsc("ScheduleAnyway", ns)) return false;
    h.n_tsc_score = ns;
    for (int i = nf; i < nf + ns; ++i) {
      ksg_tsc& t = h.tsc[i];
      t.first_of_key = 1;
      for (int j = nf; j < i; ++j)
        if (h.tsc[j].topo_key == t.topo_key && !h.tsc[j].is_hostname) t.first_of_key = 0;
    }
    if (nf == 0) h.flags |= KPF_SKIP_PTS_FILTER;
    if (ns == 0) h.flags |= KPF_SKIP_PTS_SCORE;
    // class tables: the filter pair count is the LAST filter constraint's on the key
    // (calPreFilterState keeps one count per pair); a score pair sums every
    // non-hostname score constraint on the key (TopologyPairToPodCounts)
    for (int i = 0; i < nf + ns; ++i) {
      ksg_tsc& t = h.tsc[i];
      t.nub = nub_of(t.topo);
      const bool known = t.topo >= 0 && (size_t)t.topo < enc_topo_base.size();
      t.pair_base = known ? (int32_t)enc_topo_base[t.topo] : 0;
      t.nvals = known ? (int32_t)enc_topo_count[t.topo] : 0;
      t.dom = known && (size_t)t.topo < enc_slot_dom.size() ? enc_slot_dom[t.topo] : 0;
    }
    for (int i = 0; i < nf; ++i) {
      h.tsc[i].eff_cls = h.tsc[i].cls;
      for (int j = i + 1; j < nf; ++j)
        if (h.tsc[j].topo == h.tsc[i].topo) h.tsc[i].eff_cls = h.tsc[j].cls;
    }
    for (int i = nf; i < nf + ns; ++i) {
      ksg_tsc& t = h.tsc[i];
      t.eff_cls = t.cls;
      t.sc_off = (int32_t)P.i32.size();
      t.sc_n = 0;
      if (t.is_hostname) continue;
      for (int j = nf; j < nf + ns; ++j)
        if (h.tsc[j].topo == t.topo && !h.tsc[j].is_hostname && h.tsc[j].cls >= 0) {
          P.i32.push_back(h.tsc[j].cls);
          t.sc_n++;
        }
    }
    // ---- InterPodAffinity (incoming terms; namespaceSelector merged)
    h.aterm_off = (int32_t)P.at.size();
    for (auto* v : {&p.req_aff, &p.req_anti, &p.pref_aff, &p.pref_anti})
      for (auto& a : *v) {
        ksg_aterm t;
        fill_aterm(a, P, t);
        P.at.push_back(t);
        if (a.sel.err) m.prefilter_error = true;
      }
    h.n_req_aff = (int32_t)p.req_aff.size();
    h.n_req_anti = (int32_t)p.req_anti.size();
    h.n_pref_aff = (int32_t)p.pref_aff.size();
    h.n_pref_anti = (int32_t)p.pref_anti.size();
    bool self_all = !p.req_aff.empty();
    for (auto& a : p.req_aff)
      self_all = self_all && (a.namespaces.count(p.ns) || a.ns_all) && a.sel.matches(p.labels);
    h.self_matches_all = self_all ? 1 : 0;
    h.aff_cls = tables_on() && !p.req_aff.empty() ? pclass(false, p.req_aff) : -1;
    if (p.pref_aff_present || p.pref_anti_present) h.flags |= KPF_IPA_HAS_CONSTRAINTS;
    m.ipa_no_req_terms = p.req_aff.empty() && p.req_anti.empty();
    m.ipa_prescore_skip_static = ipa_ignore && !(p.pref_aff_present || p.pref_anti_present);
    if (m.prefilter_error) h.flags |= KPF_PREFILTER_ERROR;
    // ---- NodeUnschedulable / NodeName / NodePorts / ImageLocality
    {
      Taint unsched{"node.kubernetes.io/unschedulable", "", "NoSchedule"};
      if (tolerated(p.tols, unsched)) h.flags |= KPF_TOL_UNSCHED;
      h.node_name_gid = p.node.empty() ? -1 : (node_names.get(p.node) < 0 ? -2 : node_names.get(p.node));
      if (p.ports.empty()) h.flags |= KPF_SKIP_PORTS;
      set<int32_t> check;  // CheckConflict: 0.0.0.0 wants every ip of (protocol, port); an ip wants itself and 0.0.0.0
      for (auto& w : p.ports)
        for (auto& kv : port_id)
          if (std::get<1>(kv.first) == w.proto && std::get<2>(kv.first) == w.port &&
              (w.ip == "0.0.0.0" || std::get<0>(kv.first) == "0.0.0.0" || std::get<0>(kv.first) == w.ip))
            check.insert(kv.second);
      h.port_check_off = (int32_t)P.i32.size();
      h.n_port_check = (int32_t)check.size();
      P.i32.insert(P.i32.end(), check.begin(), check.end());
      h.port_own_off = (int32_t)P.i32.size();
      h.n_port_own = 0;
      for (auto& w : p.ports) {
        auto it = port_id.find(std::make_tuple(w.ip, w.proto, w.port));
        if (it == port_id.end()) { err = "pod " + p.name + ": host port outside the vocabulary"; return false; }
        P.i32.push_back(it->second);
        h.n_port_own++;
      }
      // image_locality.go: normalizedImageName, scaledImageScore (spread = NumNodes / totalNumNodes)
      std::map<int32_t, i64> sc;
      for (auto& im : p.images) {
        string nm = im;
        size_t c = nm.rfind(':'), sl = nm.rfind('/');
        if ((c == string::npos ? -1L : (long)c) <= (sl == string::npos ? -1L : (long)sl)) nm += ":latest";
        int32_t id = images.get(nm);
        if (id < 0) continue;
        double spread = (double)image_state[id].second / (double)nodes.size();
        sc[id] += (i64)((double)image_state[id].first * spread);
      }
      if (sc.size() > KSG_MAX_IMG) { err = "pod " + p.name + ": too many node-listed images"; return false; }
      h.n_img = 0;
      for (auto& kv : sc) {
        h.img_id[h.n_img] = kv.first;
        h.img_scaled[h.n_img++] = kv.second;
      }
      h.img_max_threshold = (1000LL << 20) * (i64)p.n_containers;
      if (h.img_max_threshold <= (23LL << 20)) h.n_img = 0, h.img_max_threshold = (23LL << 20) + 1;  // no containers
    }
    // ---- as-existing record
    h.exist_flags = exist_flags(p);
    h.exist_terms_off = (int32_t)P.et.size();
    vector<int32_t>* none = nullptr;
    append_terms(p, 0, P.et, none, P.req, P.i32);
    h.n_exist_terms = (int32_t)P.et.size();
    // ---- class tables: the classes this pod belongs to (its assume's deltas) and
    // the existing pods' term classes that match it (their groups follow the ids)
    h.pc_match_off = (int32_t)P.i32.size();
    h.n_pc_match = 0;
    h.tc_match_off = h.pc_match_off;
    h.n_tc_match = 0;
    if (tables_on()) {
      sync_index();
      vector<int32_t> cand;
      pidx.candidates(p.labels, cand);  // (ascending ids: the order of a scan of the registry)
      for (const int32_t c : cand)
        if (pclass_matches(pcls[c], p)) {
          P.i32.push_back(c);
          h.n_pc_match++;
        }
      h.tc_match_off = (int32_t)P.i32.size();
      tidx.candidates(p.labels, cand);
      for (const int32_t k : cand)  // (class, value offset, topology slot, group)
        if (term_matches(tcls[k].term, p)) {
          P.i32.push_back((int32_t)k);
          P.i32.push_back((int32_t)tcls[k].off);
          P.i32.push_back(tcls[k].slot);
          P.i32.push_back(tcls[k].group);
          h.n_tc_match++;
        }
      h.tab = table_path(h) ? KTAB_ON : 0;
      if ((h.tab & KTAB_ON) && pos_of(P_PTS) >= 0 && h.n_tsc_score > 1 && !(h.flags & KPF_SKIP_PTS_SCORE))
        h.tab |= KTAB_PTS_MULTI;
      if ((h.tab & KTAB_ON) && !lookup_plan(h, P)) h.tab = 0;  // more lookups than the plan holds
      tab_blooms(h, P);
    } else {
      h.tab = KTAB_ON;  // profiles without PTS / IPA: the chain needs no tables
      h.tab_rd = h.tab_md = 0;
      h.nd_rd = h.nd_md = 0;
    }
    // every requirement of the pool (NodeAffinity, node selector, volume and
    // topology terms alike) in its flattened form
    P.freq.clear();
    P.flat_ok = true;
    for (size_t i = 0; i < P.req.size(); ++i) flatten_req(P, i);
    if (P.flat_ok) h.flags |= KPF_FLAT_NA;
    m.flags = h.flags;
    // ---- lay out the blob
    auto align = [](uint32_t x) { return (x + 15u) & ~15u; };
    uint32_t off = align(sizeof(ksg_prog));
    h.off_i32 = off; h.n_i32 = (uint32_t)P.i32.size(); off = align(off + h.n_i32 * 4);
    h.off_u32 = off; h.n_u32 = (uint32_t)P.u32.size(); off = align(off + h.n_u32 * 4);
    h.off_req = off; h.n_req = (uint32_t)P.req.size(); off = align(off + h.n_req * sizeof(ksg_req));
    h.off_sel = off; h.n_sel = (uint32_t)P.sel.size(); off = align(off + h.n_sel * sizeof(ksg_sel));
    h.off_aterm = off; h.n_aterm = (uint32_t)P.at.size(); off = align(off + h.n_aterm * sizeof(ksg_aterm));
    h.off_eterm = off; h.n_eterm = (uint32_t)P.et.size(); off = align(off + h.n_eterm * sizeof(ksg_exist_term));
    h.off_freq = off; h.n_freq = (uint32_t)P.freq.size(); off = align(off + h.n_freq * sizeof(ksg_freq));
    h.total_bytes = off;
    blob.assign(off, 0);
    std::memcpy(blob.data(), &h, sizeof(h));
    if (h.n_i32) std::memcpy(blob.data() + h.off_i32, P.i32.data(), h.n_i32 * 4);
    if (h.n_u32) std::memcpy(blob.data() + h.off_u32, P.u32.data(), h.n_u32 * 4);
    if (h.n_req) std::memcpy(blob.data() + h.off_req, P.req.data(), h.n_req * sizeof(ksg_req));
    if (h.n_sel) std::memcpy(blob.data() + h.off_sel, P.sel.data(), h.n_sel * sizeof(ksg_sel));
    if (h.n_aterm) std::memcpy(blob.data() + h.off_aterm, P.at.data(), h.n_aterm * sizeof(ksg_aterm));
    if (h.n_eterm) std::memcpy(blob.data() + h.off_eterm, P.et.data(), h.n_eterm * sizeof(ksg_exist_term));
    if (h.n_freq) std::memcpy(blob.data() + h.off_freq, P.freq.data(), h.n_freq * sizeof(ksg_freq));
    return true;
  }

  // ------------------------------------------------------------ load / run
  bool load(const char* js, size_t len) {
    J doc;
    try {
      doc = json::parse(js, len);
    } catch (std::exception& e) {
      err = e.what();
      return false;
    }
    docs.emplace_back(new J(std::move(doc)));
    const J& d = *docs.back();
    nodes.clear();
    ++node_gen;
    ++bprog_gen;
    node_names = Dict();
    bound.clear();
    queue.clear();
    nkeys = Dict(); nvals.clear(); pkeys = Dict(); pvals.clear(); nss = Dict();
    taint_id.clear(); taints.clear(); topo = Dict();
    if (const J* ns = d["nodes"])
      for (auto& n : ns->items) {
        nodes.push_back(parse_node(n));
        node_names.add(nodes.back().name);
      }
    // {"nodes", "pods" (bound), "queue"}; or the simulator's snapshot document
    // (ResourcesForSnap, simulator/snapshot/snapshot.go:33-42: no "queue") —
    // then pods without spec.nodeName are the queue, in document order, and
    // pvs / pvcs / storageClasses / priorityClasses / schedulerConfig /
    // namespaces are not read (no plugin on the path uses them)
    const J* qd = d["queue"];
    if (const J* ps = d["pods"])
      for (auto& p : ps->items) {
        Pod pod = parse_pod(p);
        if (!qd && pod.node.empty()) queue.push_back(std::move(pod));
        else bound.push_back(std::move(pod));
      }
    if (qd)
      for (auto& p : qd->items) queue.push_back(parse_pod(p));
    const J* qs = d["queueSort"];  // false: pods arrive one at a time (arrival order, no PrioritySort reordering)
    order_queue(!(qs && qs->t == J::BOOL && !qs->b));
    pvcs.clear(); pvs.clear(); classes.clear();
    if (const J* a = d["pvcs"])
      for (auto& x : a->items) { PVC c = parse_pvc(x); pvcs[c.ns + "/" + c.name] = c; }
    if (const J* a = d["pvs"])
      for (auto& x : a->items) { PV v = parse_pv(x); pvs[v.name] = v; }
    if (const J* a = d["storageClasses"])
      for (auto& x : a->items) { SClass c = parse_sc(x); classes[c.name] = c; }
    csi_counts.clear();
    if (const J* a = d["csiNodes"])
      for (auto& x : a->items) {
        const string node = (x["metadata"] ? str_of((*x["metadata"])["name"]) : "");
        if (const J* sp = x["spec"])
          if (const J* ds = (*sp)["drivers"])
            for (auto& dr : ds->items)
              if (const J* al = dr["allocatable"]; al && !al->null())
                if (const J* c = (*al)["count"]; c && !c->null()) csi_counts[node][str_of(dr["name"])] = c->num();
      }
    index_queue();
    qneed.clear();
    broken = false;
    eng->clear_lost();
    for (auto& p : queue)
      if (!volumes_modelled(p)) return false;
    if (!equal_priorities()) return false;
    if (!build_vocab() || !eng->set_score_resources(ecfg.fit_res, ecfg.ba_res, err)) return false;
    eng->release_scratch();
    NodeSoA S;
    PodTableSoA T;
    if (!encode_snapshot(S, T)) return false;
    // capacity for device-side appends of the whole queue
    uint32_t qn = (uint32_t)queue.size();
    size_t qterms = 0, qreqs = 0, qvals = 0;
    for (auto& p : queue) {
      vector<ksg_exist_term> et;
      vector<ksg_req> rq;
      vector<int32_t> vl, tp;
      append_terms(p, 0, et, tp, rq, vl);
      qterms += et.size();
      qreqs += rq.size();
      qvals += vl.size();
    }
    const uint32_t slack = 1024;  // room for drop-in cycle pods (ksg_cycle) before a re-encode
    if (!eng->upload(S, T, T.n + qn + slack, (uint32_t)(T.terms.size() + qterms + 4 * slack),
                     (uint32_t)(T.reqs.size() + qreqs + 8 * slack), (uint32_t)(T.vals.size() + qvals + 16 * slack),
                     err))
      return false;
    compiled = false;
    inplace_dirty = false;
    bound_at_valid = false;
    seq_base = 0;
    progs.clear();
    meta.clear();
    qmode.clear();
    placed.clear();
    assumed_in.clear();
    epoch = 0;
    return true;
  }

  // The pending pods of a loaded document enter the scheduling queue together
  // (upstream v1.30.4 internal/queue/scheduling_queue.go): PreEnqueue of
  // SchedulingGates (plugins/schedulinggates, in the default MultiPoint list,
  // scheduler_test.go:536) keeps a pod with spec.schedulingGates out of activeQ —
  // it is never scheduled and no plugin records anything for it — and activeQ
  // pops in PrioritySort order (plugins/queuesort/priority_sort.go Less: higher
  // spec.priority first, then the earlier queue timestamp = document order).
  // Queue index q is the position in that order; gated pods are listed apart.
  // sort == false (document key "queueSort": false): the pods arrive one at a
  // time at an idle scheduler, each popped before the next arrives (arrival order).
  vector<Pod> gated;
  bool has_plugin(const char* n) const {
    for (int i = 0; i < n_plugins; ++i)
      if (names[i] == n) return true;
    return false;
  }
  void order_queue(bool sort) {
    gated.clear();
    if (has_plugin("SchedulingGates")) {
      vector<Pod> keep;
      keep.reserve(queue.size());
      for (auto& p : queue) (p.gated ? gated : keep).push_back(std::move(p));
      queue = std::move(keep);
    }
    if (sort)
      std::stable_sort(queue.begin(), queue.end(), [](const Pod& a, const Pod& b) { return a.priority > b.priority; });
  }

  // DefaultPreemption's dry run (preempt()) runs on unsharded contexts; a sharded
  // one takes queues whose pods all share one priority (no victims can exist),
  // other clusters are refused, not approximated.
  bool has_preemption() const {
    for (int i = 0; i < n_plugins; ++i)
      if (names[i] == "DefaultPreemption") return true;
    return false;
  }
  bool equal_priorities() {
    prio_dirty = true;
    if (!has_preemption() || shards == 1) return true;
    set<i64> pr;
    for (auto* v : {&bound, &queue})
      for (auto& p : *v) pr.insert(p.priority);
    if (pr.size() > 1) { err = "pods of different priorities: DefaultPreemption victims are not modelled"; return false; }
    return true;
  }

  vector<std::unique_ptr<J>> docs;
  vector<vector<uint8_t>> progs;

  // ------------------------------------------------------------ drop-in cycles
  // Host mirror of what the device has assumed, so the snapshot can be rebuilt
  // (a pod bringing new vocabulary, an Unreserve the device cannot undo).
  vector<int8_t> qmode;         // per queue pod: 0 not run, 1 queue mode (placement = summary), 2 cycle mode
  vector<int32_t> placed;       // cycle mode: node the pod is assumed on (-1 none)
  vector<uint32_t> assumed_in;  // rebuild epoch in which the device assumed the pod
  uint32_t epoch = 0;

  void track_queue() {
    qmode.resize(queue.size(), 0);
    placed.resize(queue.size(), -1);
    assumed_in.resize(queue.size(), 0);
  }
  // (namespace, name) -> every queue index holding that pod, in queue order (a
  // pod the framework retries is cycled again under the same name), for the
  // events' name lookups
  std::unordered_map<string, vector<uint32_t>> queue_idx;
  static string pod_key(const string& ns, const string& name) { return ns + '\x1f' + name; }
  void index_queue() {
    queue_idx.clear();
    for (size_t q = 0; q < queue.size(); ++q) queue_idx[pod_key(queue[q].ns, queue[q].name)].push_back((uint32_t)q);
  }
  // the latest queue index of the pod (-1 none)
  int32_t queue_find(const string& ns, const string& name) const {
    auto it = queue_idx.find(pod_key(ns, name));
    return it == queue_idx.end() || it->second.empty() ? -1 : (int32_t)it->second.back();
  }
  const vector<uint32_t>* queue_all(const string& ns, const string& name) const {
    auto it = queue_idx.find(pod_key(ns, name));
    return it == queue_idx.end() ? nullptr : &it->second;
  }
  // Existing-pod table entries one assume of p appends (rows, terms, reqs, vals;
  // engine assume_pod), cached per queue pod.
  bool tables_on() const { return pos_of(P_PTS) >= 0 || pos_of(P_IPA) >= 0; }
  void table_need(const Pod& p, uint64_t need[4]) {
    vector<ksg_exist_term> et;
    vector<ksg_req> rq;
    vector<int32_t> vl, tp;
    append_terms(p, 0, et, tp, rq, vl);
    need[0] += 1;
    need[1] += et.size();
    need[2] += rq.size();
    need[3] += vl.size();
  }
  vector<std::array<uint32_t, 4>> qneed;
  void queue_need(uint32_t q, uint64_t need[4]) {
    if (qneed.size() < queue.size()) {
      size_t q0 = qneed.size();
      qneed.resize(queue.size());
      for (size_t j = q0; j < queue.size(); ++j) {
        uint64_t n[4] = {0, 0, 0, 0};
        table_need(queue[j], n);
        for (int i = 0; i < 4; ++i) qneed[j][i] = (uint32_t)n[i];
      }
    }
    for (int i = 0; i < 4; ++i) need[i] += qneed[q][i];
  }
  // Queue pods that may still be assumed: not run, or cycle pods without a placement.
  bool may_assume(uint32_t q) const { return qmode[q] == 0 || (qmode[q] == 2 && placed[q] < 0); }
  void mark_run(uint32_t first, uint32_t count) {
    track_queue();
    for (uint32_t q = first; q < first + count; ++q) {
      qmode[q] = 1;
      assumed_in[q] = epoch;
    }
  }
  // Current placement of queue pod q (-1 none), from the mirror or the device summary.
  int32_t placement(uint32_t q, const ksg_pod_summary* sum) const {
    if (qmode[q] == 2) return placed[q];
    if (qmode[q] == 1 && sum) return sum->status == 0 ? sum->selected : -1;
    return -1;
  }
  bool vocab_grows(const Pod& p) const {
    if (nss.get(p.ns) < 0) return true;
    for (auto& c : p.claims)
      if (pvc_ids.get(p.ns + "/" + c) < 0) return true;  // a PVC the device use counts do not cover
    if (has_volume_plugins) {
      vector<std::pair<string, string>> av;
      attachable(p, av);
      for (auto& x : av)
        if (vols.get(x.first) < 0 || lkeys.get(x.second) < 0) return true;  // NodeVolumeLimits tables
    }
    auto known = [&](const string& key, const string* v) {
      int32_t k = pkeys.get(key);
      return k >= 0 && k < (int32_t)pvals.size() && (!v || pvals[k].get(*v) >= 0);
    };
    auto sel_known = [&](const LSel& s) {
      for (auto& r : s.reqs) {
        if (!known(r.key, nullptr)) return false;
        for (auto& v : r.vals)
          if (!known(r.key, &v)) return false;
      }
      return true;
    };
    for (auto& kv : p.labels)
      if (!known(kv.first, &kv.second)) return true;
    for (auto* v : {&p.req_aff, &p.req_anti, &p.pref_aff, &p.pref_anti})
      for (auto& t : *v) {
        if (topo.get(t.topo) < 0 || !sel_known(t.sel)) return true;
        for (auto& ns : t.namespaces)
          if (nss.get(ns) < 0) return true;
      }
    for (auto& c : p.tsc)
      if (topo.get(c.key) < 0 || !sel_known(tsc_selector(p, c))) return true;
    for (auto& kv : p.req)
      if (scalar_name(kv.first) && res.get(kv.first) < 0) return true;
    for (auto& h : p.ports)
      if (!port_id.count(std::make_tuple(h.ip, h.proto, h.port))) return true;
    return false;
  }
  // Re-encode and re-upload the snapshot with every assumed queue pod as a bound
  // pod, recompile the queue, and restore the per-pod summaries.
  // remap: old node index -> new index, when nodes were removed (cluster events).
  // given: the queue's summaries (compaction re-indexes the queue), else read from the device
  bool rebuild(const vector<int32_t>* remap = nullptr, const vector<ksg_pod_summary>* given = nullptr) {
    room_ok = false;
    track_queue();
    size_t nq = queue.size();
    const size_t ns = given ? given->size() : compiled ? progs.size() : 0;  // pods with summaries on the device
    vector<ksg_pod_summary> sum(nq);
    if (given) std::copy(given->begin(), given->end(), sum.begin());
    else if (ns && !eng->summaries(0, (uint32_t)ns, sum.data(), err)) return false;
    if (remap)
      for (size_t q = 0; q < ns; ++q)
        if (sum[q].selected >= 0 && sum[q].selected < (int32_t)remap->size()) {
          int32_t to = (*remap)[sum[q].selected];
          sum[q].selected = to;
          sum[q].best_key = (sum[q].best_key & ~0xFFFFFull) | (uint64_t)(to < 0 ? 0 : to);
        }
    vector<Pod> saved = bound;
    vector<uint32_t> as_bound;  // queue pods encoded as bound pods, in order
    for (size_t q = 0; q < nq; ++q) {
      int32_t at = placement((uint32_t)q, q < ns ? &sum[q] : nullptr);
      if (at < 0 || at >= (int32_t)nodes.size()) continue;
      Pod x = queue[q];
      x.node = nodes[at].name;
      bound.push_back(x);
      as_bound.push_back((uint32_t)q);
    }
    nkeys = Dict(); nvals.clear(); pkeys = Dict(); pvals.clear(); nss = Dict();
    taint_id.clear(); taints.clear(); topo = Dict();
    bool ok = build_vocab() && eng->set_score_resources(ecfg.fit_res, ecfg.ba_res, err);
    NodeSoA S;
    PodTableSoA T;
    ok = ok && encode_snapshot(S, T);
    if (ok) {
      size_t qterms = 0, qreqs = 0, qvals = 0;
      for (auto& p : queue) {
        vector<ksg_exist_term> et;
        vector<ksg_req> rq;
        vector<int32_t> vl, tp;
        append_terms(p, 0, et, tp, rq, vl);
        qterms += et.size();
        qreqs += rq.size();
        qvals += vl.size();
      }
      const uint32_t slack = 1024;  // room for cycle pods assumed before the next rebuild
      ok = eng->upload(S, T, T.n + (uint32_t)nq + slack, (uint32_t)(T.terms.size() + qterms + 4 * slack),
                       (uint32_t)(T.reqs.size() + qreqs + 8 * slack), (uint32_t)(T.vals.size() + qvals + 16 * slack), err);
    }
    bound.swap(saved);
    qrow.assign(nq, -1);
    if (ok && bound_row.size() == bound.size() + as_bound.size())
      for (size_t k = 0; k < as_bound.size(); ++k) qrow[as_bound[k]] = bound_row[bound.size() + k];
    bound_row.resize(bound.size());  // placements were encoded after the bound pods
    if (!ok) return false;
    inplace_dirty = false;
    compiled = false;
    if (!compile_queue()) return false;
    if (ns && !eng->set_summaries(0, (uint32_t)ns, sum.data(), err)) return false;
    ++epoch;
    return true;
  }
  // Bounded memory in plugin mode (ksg_compact): queue pods [0, keep_from) leave
  // the queue — those placed become bound pods of the snapshot, the JSON documents
  // of the others are released — and the rest are re-indexed from 0 (their
  // results kept); one re-encode.
  // Queue position of queue pod 0 in the sequence of every pod this context has
  // queued since the load: the tie-break hash (pack_key) takes seq_base + q, so a
  // compaction does not move later pods' ties.
  uint32_t seq_base = 0;
  bool compact(uint32_t keep_from) {
    if (shards != 1) { err = "compaction needs an unsharded context"; return false; }
    if (keep_from > queue.size()) { err = "compact: queue range"; return false; }
    if (!compile_queue()) return false;
    track_queue();
    const size_t nq = queue.size(), ns = progs.size();
    vector<ksg_pod_summary> sum(nq);
    if (ns && !eng->summaries(0, (uint32_t)ns, sum.data(), err)) return false;
    for (uint32_t q = 0; q < keep_from; ++q) {
      const int32_t at = placement(q, q < ns ? &sum[q] : nullptr);
      if (at >= 0 && at < (int32_t)nodes.size()) {
        Pod x = queue[q];
        x.node = nodes[at].name;
        bound.push_back(std::move(x));
      } else if (queue[q].doc >= 0 && (size_t)queue[q].doc < docs.size()) {
        docs[queue[q].doc].reset();  // its own document: nothing else points into it
      }
    }
    auto cut = [&](auto& v) {
      if (v.size() > keep_from) v.erase(v.begin(), v.begin() + keep_from);
      else v.clear();
    };
    cut(queue);
    cut(qmode);
    cut(placed);
    cut(assumed_in);
    cut(nom);
    cut(qneed);
    cut(sum);
    if (ns > keep_from) sum.resize(ns - keep_from);
    else sum.clear();
    bound_at_valid = false;
    index_queue();
    keep_first = keep_n = 0;
    if (!eng->keep_outputs(0, 0, err)) return false;
    oc_q = -1;
    compiled = false;
    seq_base += keep_from;
    eng->release_scratch();
    if (!rebuild(nullptr, &sum)) {  // the host state moved on: the device would hold the old one
      broken = true;
      return false;
    }
    return true;
  }

  // One scheduling cycle of a new pod (appended to the queue).
  // Host wall time per phase of the drop-in cycle (diagnostic: ksg_debug_cycle_times):
  // [0] JSON parse + pod decode, [1] queue checks + vocabulary, [2] compile,
  // [3] program append (+ classes), [4] launch, [5] summary wait, [6] PostFilter,
  // [7] cycles; microseconds summed.
  double ctimes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // The cycle view of the last ksg_cycle(commit = 0), filled by a k_view queued
  // behind the cycle's own run (the cycle's one sync completes it), so that the
  // plugin's ksg_cycle_view_acquire for that pod needs no launch and no sync.
  // Valid while out_gen is unchanged (any later state-changing call drops it).
  struct PreView {
    uint8_t* block = nullptr;
    size_t cap = 0;
    int64_t q = -1;
    uint64_t gen = 0;
    ksg::Engine::ViewLayout lay;
    void drop() {
      if (block) ksg::Engine::pinned_put(block, cap);
      block = nullptr;
      cap = 0;
      q = -1;
    }
    ~PreView() { drop(); }
  } pview;
  bool classes_early = std::getenv("KSG_CLASSES_EARLY") && std::strtol(std::getenv("KSG_CLASSES_EARLY"), nullptr, 10) != 0;
  bool view_prefetch = !(std::getenv("KSG_VIEW_PREFETCH") && std::strtol(std::getenv("KSG_VIEW_PREFETCH"), nullptr, 10) == 0);
  // arm: prepared before the cycle's run (Engine::view_arm), so that the run's k_eval
  // can write it itself (a profile without ScoreExtensions); the run's caller then
  // calls Engine::view_arm_finish
  bool prefetch_view(uint32_t q, bool arm = false) {
    pview.drop();
    eng->view_layout(pview.lay);
    pview.block = ksg::Engine::pinned_get(pview.lay.bytes, pview.cap);
    if (!pview.block) return true;  // (no pinned memory: acquire builds it)
    if (arm && pview.lay.N && ksg::Engine::pinned_dev(pview.block)) {
      if (!eng->view_arm(q, view_cfg(), pview.lay, pview.block, err)) return false;
    } else if (!eng->view(q, view_cfg(), pview.lay, pview.block, err, false)) {
      return false;
    }
    pview.q = q;
    pview.gen = out_gen;
    return true;
  }
  static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  bool cycle(const char* js, size_t len, bool commit, ksg_pod_summary& out) {
    if (shards != 1) { err = "the cycle API needs an unsharded context"; return false; }
    if (!compile_queue()) return false;
    static const char* const kPhase[8] = {"parse", "checks_vocab", "compile", "append", "launch", "wait", "postfilter", ""};
    rtx::Phases ph;
    ph.next(kPhase[0]);
    double t = now_us();
    auto lap = [&](int k) {
      const double u = now_us();
      ctimes[k] += u - t;
      t = u;
      if (k < 6) ph.next(kPhase[k + 1]);
    };
    try {
      docs.emplace_back(new J(json::parse(js, len)));
    } catch (std::exception& e) {
      err = e.what();
      return false;
    }
    const J& d = *docs.back();
    queue.push_back(parse_pod(d["pod"] ? *d["pod"] : d));
    lap(0);
    queue.back().doc = (int32_t)docs.size() - 1;
    if (!volumes_modelled(queue.back())) {
      queue.pop_back();
      return false;
    }
    if (!equal_priorities()) {
      queue.pop_back();
      return false;
    }
    track_queue();
    uint32_t q = (uint32_t)queue.size() - 1;
    queue_idx[pod_key(queue[q].ns, queue[q].name)].push_back(q);
    qmode[q] = 2;
    bool in_place = !vocab_grows(queue[q]);
    if (!in_place && vocab_grows_in_place(queue[q])) {  // new label values / keys / namespaces only
      if (!grow_vocab(queue[q])) return false;
      in_place = true;
    }
    lap(1);
    if (!in_place) {
      if (!rebuild()) return false;
    } else {
      vector<uint8_t> blob;
      PodMeta m;
      // classes_early: the pod's new classes registered and their tables built
      // (one upload + k_pc_build on the engine stream) before its program is
      // compiled, so the device builds them while the host compiles; the program
      // then goes out on its own (k_place_program).  Otherwise the program rides
      // in the class upload after the compile.
      if (classes_early) {
        register_classes(queue[q]);
        if (!sync_classes()) return false;
      }
      if (!compile(queue[q], (int32_t)(seq_base + q), blob, m)) return false;
      lap(2);
      bool placed = false;  // (with the classes it brought, in one upload)
      if (!sync_classes(&blob, &placed) || (!placed && !eng->append_program(blob, err))) return false;
      progs.push_back(std::move(blob));
      meta.push_back(std::move(m));
      prog_cls.resize(progs.size(), {(uint32_t)pcls.size(), (uint32_t)tcls.size()});
    }
    lap(3);
    if (commit) room_ok = false;
    if (commit && !room_for(q)) return false;
    // (the summary's copy waits for the run; sync then only checks the run's state)
    if (!eng->keep_outputs(q, 1, err)) return false;
    if (!commit && view_prefetch && !prefetch_view(q, true)) return false;  // (armed: the run may write it)
    if (!eng->run_queue(q, 1, commit, err) || !eng->view_arm_finish(err)) return false;
    lap(4);
    if (!commit && pview.block && pview.q == (int64_t)q) {  // (the prefetched view carries the summary)
      if (!eng->sync(err)) return false;
      std::memcpy(&out, pview.block + pview.lay.off_sum, sizeof(out));
      if (out.status == 2 && eng->view_fused()) {  // (a Score error: its rows at 4 bytes, rebuilt)
        if (!eng->view(q, view_cfg(), pview.lay, pview.block, err, true)) return false;
        std::memcpy(&out, pview.block + pview.lay.off_sum, sizeof(out));
      }
    } else if (!eng->summaries(q, 1, &out, err) || !eng->sync(err)) {
      return false;
    }
    lap(5);
    if (!preempt(q, out)) return false;  // PostFilter of an unschedulable pod
    lap(6);
    ctimes[7] += 1;
    if (commit && out.status == 0) {
      placed[q] = out.selected;
      assumed_in[q] = epoch;
    }
    return true;
  }
  // The device appends assumed pods to its existing-pod table: before an assume,
  // make room for queue pod q's row in place (capacities doubled, contents kept).
  // room_ok: the device's table use is known on the host (room_used, an upper
  // bound) — set by a query from the drop-in Reserve path, whose own appends it
  // counts, and cleared by every other entry point that may append or re-upload
  // (the C API calls and rebuild()), so back-to-back Reserves skip the read-back.
  bool room_ok = false;
  uint64_t room_used[4] = {0, 0, 0, 0}, room_cap[4] = {0, 0, 0, 0};
  bool room_for(uint32_t q, bool cached = false) {
    if (!tables_on()) return true;
    uint64_t need[4] = {0, 0, 0, 0};
    queue_need(q, need);
    return ensure_room(need, cached);
  }
  bool ensure_room(const uint64_t need[4], bool cached = false) {
    if (cached && room_ok) {
      bool fits = true;
      for (int i = 0; i < 4; ++i) fits &= room_used[i] + need[i] <= room_cap[i];
      if (fits) {
        for (int i = 0; i < 4; ++i) room_used[i] += need[i];
        return true;
      }
    }
    room_ok = false;
    uint32_t used[4], cap[4];
    if (!eng->table_room(used, cap, err)) return false;
    bool fits = true;
    uint32_t nc[4];
    for (int i = 0; i < 4; ++i) {
      const uint64_t want = (uint64_t)used[i] + need[i];
      fits &= want <= cap[i];
      nc[i] = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(2ull * cap[i], want + 1024), UINT32_MAX);
    }
    if (!fits) return eng->grow_table(nc[0], nc[1], nc[2], nc[3], 0, err);
    if (cached) {
      for (int i = 0; i < 4; ++i) {
        room_used[i] = (uint64_t)used[i] + need[i];
        room_cap[i] = cap[i];
      }
      room_ok = true;
    }
    return true;
  }
  // ------------------------------------------------------------ DefaultPreemption
  // PostFilter of an unschedulable pod, as a dry run on the device state of the
  // pod's own cycle (v1.30.4 plugins/defaultpreemption/default_preemption.go,
  // framework/preemption/preemption.go; the oracle's preempt() restates it):
  // PodEligibleToPreemptOthers (preemptionPolicy Never), nodesWherePreemptionMightHelp
  // (nodes whose Filter status is Unschedulable, not UnschedulableAndUnresolvable),
  // SelectVictimsOnNode per such node (every lower-priority pod taken off, the
  // pod's cycle re-run on the device, then the victims reprieved most important
  // first while the pod still fits), pickOneNodeForPreemption.  Nothing is
  // evicted: the device state is restored exactly (rows revived in place) and the
  // result is the nominated node and its victims (the store's postfilter-result
  // entry, store.go:442-458).  Deviations: every potential node is
  // examined (upstream: a random-offset sample of max(10%, 100)), the seeded
  // selectHost rule breaks the last tie, no PodDisruptionBudgets exist.
  struct Nomination {
    int32_t node = -1;        // global node index
    vector<string> victims;   // "namespace/name"
  };
  vector<Nomination> nom;
  vector<int32_t> qrow;  // queue pods the last rebuild encoded as bound pods: their table rows
  bool prio_dirty = true;
  i64 low_prio = INT64_MAX;
  // Can queue pod q preempt anything (some pod of a lower priority exists)?
  bool may_preempt(uint32_t q) {
    if (!has_preemption() || shards != 1 || queue[q].preempt_never) return false;
    if (prio_dirty) {
      low_prio = INT64_MAX;
      for (auto* v : {&bound, &queue})
        for (auto& p : *v) low_prio = std::min(low_prio, p.priority);
      prio_dirty = false;
    }
    return queue[q].priority > low_prio;
  }
  uint64_t tie_key(uint32_t q, uint32_t g) const {  // engine pack_key with total 0
    uint64_t z = ecfg.seed ^ ((uint64_t)(seq_base + q) * 0x9E3779B97F4A7C15ull) ^ (uint64_t)g;
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return ((0xFFFFFull - (z >> 44)) << 20) | (uint64_t)g;
  }
  // The batched victim search applies (see preempt): removing pods changes
  // nothing the pod's filters read but the node they are removed from.
  uint64_t preempt_batched_runs = 0;  // diagnostic: pods whose dry run took the batched search
  bool preempt_no_batch = std::getenv("KSG_PREEMPT_BATCH") && std::strtol(std::getenv("KSG_PREEMPT_BATCH"), nullptr, 10) == 0;
  // Is every node's value of label key `key` its own (no two nodes share one)?  A
  // required anti-affinity term over such a key reads only the pods of the node it
  // filters (upstream satisfyPodAntiAffinity: counts per (key, value) domain).
  mutable std::unordered_map<string, std::pair<uint64_t, bool>> topo_uniq_cache;
  bool topo_unique_now(const string& key) const {
    auto it = topo_uniq_cache.find(key);
    if (it != topo_uniq_cache.end() && it->second.first == node_gen) return it->second.second;
    std::unordered_set<string> seen;
    bool u = !key.empty();
    for (size_t i = 0; u && i < nodes.size(); ++i) {
      auto l = nodes[i].labels.find(key);
      if (l != nodes[i].labels.end() && !seen.insert(l->second).second) u = false;
    }
    topo_uniq_cache[key] = {node_gen, u};
    return u;
  }
  bool preempt_batched(const Pod& p, const ksg_pod_summary& S) const {
    if (preempt_no_batch) return false;
    if (!p.req_aff.empty() || (S.ipa_flags & 4u)) return false;
    // (required anti-affinity over one-node-per-value keys, e.g. kubernetes.io/hostname:
    // a node's removals change only its own domain)
    for (auto& t : p.req_anti)
      if (!topo_unique_now(t.topo)) return false;
    // (ScheduleAnyway constraints only score: PodTopologySpread's PreFilter state
    // holds the DoNotSchedule ones, so a pod with no other reads no spread counts)
    for (auto& t : p.tsc)
      if (t.when != "ScheduleAnyway") return false;
    for (auto& cn : p.claims) {
      const PVC* c = pvc_of(p.ns, cn);
      if (c && c->rwop) return false;
    }
    return true;
  }
  // Host wall time per phase of the DefaultPreemption dry runs (diagnostic:
  // ksg_debug_preempt_times): [0] the pod's dry run + potential nodes, [1] candidate
  // victims and their programs, [2] the victim search (toggles, dry runs), [3] searches.
  double ptimes[4] = {0, 0, 0, 0};
  bool preempt(uint32_t q, const ksg_pod_summary& S) {
    if (nom.size() < queue.size()) nom.resize(queue.size());
    nom[q] = Nomination();
    if (S.status != 1 || q >= meta.size() || meta[q].prefilter_fail_pos >= 0 || !may_preempt(q)) return true;
    double pt = now_us();
    auto plap = [&](int k) {
      const double u = now_us();
      ptimes[k] += u - pt;
      pt = u;
    };
    struct PCount {
      double* c;
      ~PCount() { *c += 1; }
    } pcount{&ptimes[3]};
    const Pod& p = queue[q];
    const uint32_t n = hi - lo;
    PodOutputs o;
    o.summary = S;
    if (!refresh_program(q) || !eng->dry_filter(q, -1, o.filter, err)) return false;
    // victims' candidates per potential node: bound pods, then assumed queue pods
    struct Vic {
      int32_t bound = -1, qpod = -1;
      i64 prio, start;
      uint64_t order;  // load order (MoreImportantPod's last tie, as the oracle's)
    };
    vector<int32_t> potential;
    vector<char> is_pot(n, 0);
    {  // nodesWherePreemptionMightHelp: the framework code of each node's failure
      // (filter_status without its message; Fit's rule on the cached allocatable)
      vector<i64> rq;
      i64 nzc = 0, nzm = 0;
      add_requests_const(p, rq, nzc, nzm);
      const vector<i64>& al = node_allocs();
      const uint32_t skip = skip_filter_mask(meta[q], o.summary);
      for (uint32_t i = 0; i < n; ++i) {
        const uint32_t c = o.filter[i];
        if (c == KSG_FILTER_PASS || c >= KSG_FILTER_NOT_EVALUATED || (c >> 24) >= (uint32_t)n_dev) continue;
        const int pos = code_pos(c);
        if (pos < 0 || pos >= n_plugins || !has_filter(plugins[pos]) || filter_skipped(meta[q], skip, pos)) continue;
        const int fc = plugins[pos] == P_FIT
                           ? fit_fail_code(rq, code_detail(c), res.names.size(), [&](size_t r) { return al[r * n + i]; })
                           : filter_fail_code(q, pos, i, code_detail(c));
        if (fc == C_UNSCHED) {
          potential.push_back((int32_t)i);
          is_pot[i] = 1;
        }
      }
    }
    plap(0);
    if (potential.empty()) return true;
    // candidate victims per potential node k (flat: vic[voff[k] .. voff[k + 1])):
    // its lower-priority bound pods in load order, then its assumed queue pods
    const vector<uint32_t>& boff = bound_by_node();
    vector<std::pair<int32_t, Vic>> qvic;  // queue pods placed on potential nodes, by node
    vector<ksg_pod_summary> sum(progs.size());
    if (!sum.empty() && !eng->summaries(0, (uint32_t)sum.size(), sum.data(), err)) return false;
    for (uint32_t j = 0; j < queue.size() && j < progs.size(); ++j) {
      if (j == q || queue[j].priority >= p.priority) continue;
      const int32_t g = placement(j, &sum[j]);
      if (g < 0 || g >= (int32_t)n || !is_pot[g]) continue;
      qvic.push_back({g, Vic{-1, (int32_t)j, queue[j].priority, queue[j].start_time, (uint64_t)bound.size() + j}});
    }
    std::stable_sort(qvic.begin(), qvic.end(), [](const std::pair<int32_t, Vic>& a, const std::pair<int32_t, Vic>& b) {
      return a.first < b.first;
    });
    vector<Vic> vic;
    vector<uint32_t> voff(potential.size() + 1, 0);
    size_t n_bound_vic = 0;
    for (size_t k = 0, qi = 0; k < potential.size(); ++k) {
      const int32_t g = potential[k];
      voff[k] = (uint32_t)vic.size();
      for (uint32_t e = boff[g]; e < boff[g + 1]; ++e) {
        const int32_t b = bcsr_idx[e];
        if (bound[b].priority >= p.priority) continue;
        vic.push_back({b, -1, bound[b].priority, bound[b].start_time, (uint64_t)b});
      }
      n_bound_vic += vic.size() - voff[k];
      while (qi < qvic.size() && qvic[qi].first < g) ++qi;
      for (; qi < qvic.size() && qvic[qi].first == g; ++qi) vic.push_back(qvic[qi].second);
    }
    voff[potential.size()] = (uint32_t)vic.size();
    // bound victims' programs: the device-resident victim store (every bound pod,
    // uploaded once per cache generation) once the search is large or the store is
    // current; small searches stage copies of the victims' programs
    const bool by_ref = preempt_batched(p, S) && (victim_store_current() || n_bound_vic >= victim_store_min);
    std::unordered_map<int32_t, const vector<uint8_t>*> bprog;
    std::map<int32_t, int32_t> qrows;
    for (const Vic& v : vic) {
      if (v.bound >= 0) {
        if (by_ref) continue;
        const vector<uint8_t>* bp = bound_prog(v.bound);
        if (!bp) return false;
        bprog[v.bound] = bp;
      } else {
        int32_t row = -1;
        if (tables_on()) {
          if (assumed_in[v.qpod] == epoch) {
            if (!eng->pod_row((uint32_t)v.qpod, row, err)) return false;
          } else if ((size_t)v.qpod < qrow.size()) {
            row = qrow[v.qpod];
          }
        }
        qrows[v.qpod] = row;
      }
    }
    if (!sync_classes() || !refresh_program(q)) return false;
    for (auto& kv : qrows)
      if (!refresh_program((uint32_t)kv.first)) return false;
    if (by_ref && !ensure_victim_store()) return false;
    plap(1);
    struct PLap {  // the search's time, whichever way it returns
      std::function<void()> f;
      ~PLap() { f(); }
    } psearch{[&]() { plap(2); }};
    auto toggle = [&](const vector<Vic>& vs, int32_t g, int sign) {
      vector<const vector<uint8_t>*> pp;
      vector<int32_t> gn, rows;
      for (auto& v : vs) {
        pp.push_back(v.bound >= 0 ? bprog[v.bound] : &progs[v.qpod]);
        gn.push_back(g + (int32_t)lo);
        rows.push_back(v.bound >= 0 ? (tables_on() ? bound_row[v.bound] : -1) : qrows[v.qpod]);
      }
      return eng->toggle_pods(pp, gn, rows, sign, err);
    };
    vector<uint32_t> code;
    auto fits = [&](int32_t g, bool& ok) {
      if (!eng->dry_filter(q, g + (int32_t)lo, code, err)) return false;
      ok = code[0] == KSG_FILTER_PASS;
      return true;
    };
    struct Cand {
      int32_t node;
      vector<Vic> victims;
    };
    vector<Cand> cands;
    auto more_important = [](const Vic& a, const Vic& b) {  // util.MoreImportantPod
      if (a.prio != b.prio) return a.prio > b.prio;
      if (a.start != b.start) return a.start < b.start;
      return a.order < b.order;
    };
    if (preempt_batched(p, S)) {
      // Batched search (every potential node at once).  Removing a node's victims
      // changes only that node (its row, host ports, attached volumes): the pod
      // has no DoNotSchedule spread constraint, no required affinity term, required
      // anti-affinity only over one-node-per-value keys, no existing pod's
      // anti-affinity applies to it and it holds no ReadWriteOncePod claim, so its
      // PreFilter state is the same whatever is removed, and the victim sets of
      // different nodes are disjoint.  One dry run with every potential node's
      // victims removed answers SelectVictimsOnNode's first question for all of
      // them; the reprieve then runs in lockstep over the candidates, one dry run
      // per round (its i-th most important victim re-added on every candidate).
      // every candidate victim staged on the device once (entry i = vic[i]); the
      // toggles below name entries (one launch each, a thread per node)
      // (entry i = vic[i]: node by node, so every list below comes grouped by node)
      if (vic.empty()) return true;
      {
        vector<int32_t> gn(vic.size()), rows(vic.size());
        for (size_t k = 0; k < potential.size(); ++k)
          for (uint32_t i = voff[k]; i < voff[k + 1]; ++i) {
            const Vic& v = vic[i];
            gn[i] = potential[k] + (int32_t)lo;
            rows[i] = v.bound >= 0 ? (tables_on() ? bound_row[v.bound] : -1) : qrows[v.qpod];
          }
        if (by_ref) {
          vector<int64_t> ref(vic.size());
          vector<uint8_t> qcsi(progs.size(), 0);
          for (size_t i = 0; i < vic.size(); ++i) {
            const Vic& v = vic[i];
            if (v.bound >= 0) {
              ref[i] = v.bound;
            } else {
              ref[i] = -1 - (int64_t)v.qpod;
              qcsi[v.qpod] = reinterpret_cast<const ksg_prog*>(progs[v.qpod].data())->n_csi > 0 ? 1 : 0;
            }
          }
          if (!eng->toggle_stage_refs(ref, gn, rows, qcsi, err)) return false;
        } else {
          vector<const vector<uint8_t>*> pp(vic.size());
          for (size_t i = 0; i < vic.size(); ++i) pp[i] = vic[i].bound >= 0 ? bprog[vic[i].bound] : &progs[vic[i].qpod];
          if (!eng->toggle_stage(pp, gn, rows, err)) return false;
        }
      }
      auto all_vic = [&](uint32_t e) -> const Vic& { return vic[e]; };
      vector<uint32_t> every(vic.size());
      for (size_t i = 0; i < vic.size(); ++i) every[i] = (uint32_t)i;
      vector<uint32_t> codes;
      if (!eng->toggle_staged(every, -1, err) || !eng->dry_filter(q, -1, codes, err) ||
          !eng->toggle_staged(every, +1, err))
        return false;
      vector<vector<uint32_t>> pv;  // per candidate: its victims (entries), most important first
      {
        for (size_t k = 0; k < potential.size(); ++k) {
          const int32_t g = potential[k];
          if (voff[k] == voff[k + 1] || codes[g] != KSG_FILTER_PASS) continue;
          cands.push_back(Cand{g, {}});
          pv.emplace_back();
          for (uint32_t i = voff[k]; i < voff[k + 1]; ++i) pv.back().push_back(i);
          std::sort(pv.back().begin(), pv.back().end(),
                    [&](uint32_t a, uint32_t b) { return more_important(all_vic(a), all_vic(b)); });
        }
      }
      vector<uint32_t> off;  // every candidate's victims off, then reprieve round by round
      size_t rounds = 0;
      for (size_t c = 0; c < cands.size(); ++c) {
        off.insert(off.end(), pv[c].begin(), pv[c].end());
        rounds = std::max(rounds, pv[c].size());
      }
      if (!eng->toggle_staged(off, -1, err)) return false;
      ++preempt_batched_runs;
      vector<vector<uint32_t>> vict(cands.size());
      for (size_t r = 0; r < rounds; ++r) {
        vector<uint32_t> back, keep_off;
        vector<size_t> who;
        for (size_t c = 0; c < cands.size(); ++c)
          if (r < pv[c].size()) {
            back.push_back(pv[c][r]);
            who.push_back(c);
          }
        if (!eng->toggle_staged(back, +1, err) || !eng->dry_filter(q, -1, codes, err)) return false;
        for (size_t i = 0; i < who.size(); ++i)
          if (codes[cands[who[i]].node] != KSG_FILTER_PASS) {  // it must go: a victim
            keep_off.push_back(back[i]);
            vict[who[i]].push_back(back[i]);
          }
        if (!eng->toggle_staged(keep_off, -1, err)) return false;
      }
      vector<uint32_t> restore;  // the dry run leaves the state as it was
      for (size_t c = 0; c < cands.size(); ++c) {
        restore.insert(restore.end(), vict[c].begin(), vict[c].end());
        for (uint32_t e : vict[c]) cands[c].victims.push_back(all_vic(e));
      }
      if (!eng->toggle_staged(restore, +1, err)) return false;
      vector<Cand> kept;
      for (auto& c : cands)
        if (!c.victims.empty()) kept.push_back(std::move(c));
      cands.swap(kept);
    } else {
      for (size_t k = 0; k < potential.size(); ++k) {
        const int32_t g = potential[k];
        vector<Vic> pvg(vic.begin() + voff[k], vic.begin() + voff[k + 1]);
        if (pvg.empty()) continue;  // "No preemption victims found for incoming pod"
        bool ok = false;
        if (!toggle(pvg, g, -1) || !fits(g, ok)) return false;
        if (!ok) {
          if (!toggle(pvg, g, +1)) return false;
          continue;
        }
        std::sort(pvg.begin(), pvg.end(), more_important);
        Cand c{g, {}};
        for (auto& v : pvg) {  // reprieve: most important first
          if (!toggle({v}, g, +1) || !fits(g, ok)) return false;
          if (!ok) {
            if (!toggle({v}, g, -1)) return false;
            c.victims.push_back(v);
          }
        }
        if (!toggle(c.victims, g, +1)) return false;  // the dry run leaves the state as it was
        if (!c.victims.empty()) cands.push_back(std::move(c));
      }
    }
    if (cands.empty()) return true;
    // pickOneNodeForPreemption: fewest PDB violations (none here), lowest highest
    // victim priority, lowest sum of (priority + 2^31), fewest victims, latest
    // earliest start among the highest-priority victims; then the seeded rule
    auto crit = [](const Cand& c, int f) -> i64 {
      const vector<Vic>& v = c.victims;  // most important first
      if (f == 0) return -v[0].prio;
      if (f == 1) {
        i64 t = 0;
        for (auto& x : v) t += x.prio + ((i64)1 << 31);
        return -t;
      }
      if (f == 2) return -(i64)v.size();
      i64 e = v[0].start;
      for (auto& x : v)
        if (x.prio == v[0].prio) e = std::min(e, x.start);
      return e;
    };
    vector<size_t> keep(cands.size());
    for (size_t i = 0; i < keep.size(); ++i) keep[i] = i;
    for (int f = 0; f < 4 && keep.size() > 1; ++f) {
      i64 best = INT64_MIN;
      for (size_t i : keep) best = std::max(best, crit(cands[i], f));
      vector<size_t> next;
      for (size_t i : keep)
        if (crit(cands[i], f) == best) next.push_back(i);
      keep.swap(next);
    }
    size_t pick = keep[0];
    for (size_t i : keep)
      if (tie_key(q, cands[i].node + lo) > tie_key(q, cands[pick].node + lo)) pick = i;
    Nomination& r = nom[q];
    r.node = cands[pick].node + (int32_t)lo;
    for (auto& v : cands[pick].victims) {
      const Pod& x = v.bound >= 0 ? bound[v.bound] : queue[v.qpod];
      r.victims.push_back(x.ns + "/" + x.name);
    }
    return true;
  }

  // The device went back to the last upload (ksg_reset): pods it assumed since
  // are no longer placed (their results stay).
  void forget_epoch() {
    track_queue();
    for (size_t q = 0; q < queue.size(); ++q)
      if (assumed_in[q] == epoch && qmode[q] != 0) {
        if (qmode[q] == 1) qmode[q] = 0;
        placed[q] = -1;
      }
  }

  bool reserve(uint32_t q, int32_t node) {
    track_queue();
    if (q >= queue.size() || qmode[q] != 2 || placed[q] >= 0) { err = "reserve: pod not in an uncommitted cycle"; return false; }
    if (node < 0 || node >= (int32_t)nodes.size()) { err = "reserve: node out of range"; return false; }
    // (no wait for the assume: every later call is ordered behind it on the stream)
    if (!refresh_program(q) || !room_for(q, true) || !eng->assume(q, node, +1, err, false)) return false;
    placed[q] = node;
    assumed_in[q] = epoch;
    return true;
  }
  bool unreserve(uint32_t q) {
    track_queue();
    if (q >= queue.size()) { err = "unreserve: pod out of range"; return false; }
    ksg_pod_summary sm;
    if (qmode[q] == 1 && !eng->summaries(q, 1, &sm, err)) return false;
    int32_t at = placement(q, qmode[q] == 1 ? &sm : nullptr);
    if (at < 0) { err = "unreserve: pod is not assumed"; return false; }
    qmode[q] = 2;
    placed[q] = -1;
    if (assumed_in[q] == epoch) return refresh_program(q) && eng->assume(q, at, -1, err);
    return rebuild();  // assumed before the last rebuild: it is a bound pod of the snapshot now
  }

  // ------------------------------------------------------------ cluster events
  // Scheduler-cache events between cycles: upstream Cache.AddNode / UpdateNode /
  // RemoveNode / AddPod / UpdatePod / RemovePod (v1.30.4 pkg/scheduler/internal/
  // cache/cache.go, fed by eventhandlers.go; in the simulator the events come from
  // its apiserver, e.g. resources applied by simulator/resourceapplier or the
  // snapshot service).  A batch is applied to the host mirror, then the snapshot
  // is re-encoded once with every placement kept (queue pods already scheduled
  // stay bound where they were).  A batch that fails leaves the mirror unchanged.
  static string obj_name(const J& e, const char* field, string* ns) {
    const J* o = e[field];
    const J* md = o ? (*o)["metadata"] : nullptr;
    if (ns) *ns = md && (*md)["namespace"] ? str_of((*md)["namespace"]) : (e["namespace"] ? str_of(e["namespace"]) : "default");
    return md ? str_of((*md)["name"]) : str_of(e["name"]);
  }
  // In-place path for batches of bound-pod additions / removals on known nodes
  // that bring no new vocabulary: the device applies each as the assume delta
  // (rows +- requests, host ports; existing-pod table append or tombstone), the
  // same k_assume Reserve/Unreserve use, instead of a re-encode.  Returns 1
  // applied, 0 not eligible (nothing changed), -1 error.
  int inplace_events(const J& ev) {
    struct Op {
      bool add;
      Pod pod;
      vector<uint8_t> blob;
      string key;
      int32_t node = -1;
      Node nd;
      int32_t qpod = -1, qat = -1;
      bool statics = false, taints = false;  // node update: label / flag columns, taint lists rewritten
    };
    auto pkey = [](const string& ns, const string& name) { return ns + '\x1f' + name; };
    track_queue();
    prio_dirty = true;
    if (!bound_at_valid) {
      bound_at.clear();
      for (size_t i = 0; i < bound.size(); ++i) bound_at[pkey(bound[i].ns, bound[i].name)] = (uint32_t)i;
      bound_at_valid = true;
    }
    vector<Op> ops;
    std::unordered_set<string> added, removed;  // the batch on top of bound_at, simulated
    std::set<int32_t> gone_q;                    // scheduled queue pods the batch deletes
    auto present = [&](const string& k) { return added.count(k) || (bound_at.count(k) && !removed.count(k)); };
    std::set<i64> prios;  // a sharded context keeps one priority (equal_priorities)
    if (has_preemption() && shards != 1)
      for (auto* v : {&bound, &queue})
        for (auto& p : *v) prios.insert(p.priority);
    for (auto& e : ev.items) {
      const string op = str_of(e["op"]);
      if (op == "addPod") {
        if (!e["pod"]) return 0;
        Pod p = parse_pod(*e["pod"]);
        if (p.node.empty() || node_names.get(p.node) < 0) return 0;
        if (has_volume_plugins && !p.claims.empty()) return 0;  // claim users: the re-encode path re-checks the queue
        if (vocab_grows(p)) {  // new label values / keys / namespaces grow in place
          if (!vocab_grows_in_place(p)) return 0;
          if (!grow_vocab(p)) return -1;
        }
        string k = pkey(p.ns, p.name);
        if (present(k)) return 0;
        if (queue_find(p.ns, p.name) >= 0) return 0;
        if (has_preemption() && shards != 1) {
          prios.insert(p.priority);
          if (prios.size() > 1) return 0;
        }
        Op o{true, std::move(p), {}, k};
        PodMeta m;
        if (!compile(o.pod, 0, o.blob, m)) return 0;  // the re-encode path takes it
        added.insert(k);
        removed.erase(k);
        ops.push_back(std::move(o));
      } else if (op == "updateNode") {
        // allocatable, unschedulable, label and taint updates whose values the
        // vocabularies already hold (no topology key changes value: the class
        // tables and topology slots stay as they are); images unchanged
        if (!e["node"]) return 0;
        Node x = parse_node(*e["node"]);
        const int32_t at = node_names.get(x.name);
        if (at < 0) return 0;
        const Node& old = nodes[at];
        if (x.images != old.images) return 0;
        bool retaint = x.taints.size() != old.taints.size();
        for (size_t t = 0; t < x.taints.size() && !retaint; ++t)
          retaint = x.taints[t].key != old.taints[t].key || x.taints[t].value != old.taints[t].value ||
                    x.taints[t].effect != old.taints[t].effect;
        const bool relabel = x.labels != old.labels;
        if ((relabel || retaint) && has_volume_plugins) return 0;  // (volume topology is read from labels at encode)
        if (relabel && !labels_in_place(old.labels, x.labels)) return 0;
        if (retaint)
          for (auto& t : x.taints)
            if (!taint_id.count(std::make_tuple(t.key, t.value, t.effect))) return 0;
        for (auto& kv : x.alloc)
          if (kv.first != "pods" && res.get(kv.first) < 0) return 0;
        Op o{false, Pod(), {}, string()};
        o.node = at;
        o.statics = relabel || x.unschedulable != old.unschedulable;
        o.taints = retaint;
        o.nd = std::move(x);
        ops.push_back(std::move(o));
      } else if (op == "removePod") {
        string pns, name = obj_name(e, "pod", &pns);
        string k = pkey(pns, name);
        if (!present(k)) {
          // a queue pod this context scheduled (assumed since the last encode): Unreserve's delta
          const int32_t q = queue_find(pns, name);
          if (q < 0 || gone_q.count(q) || (size_t)q >= qmode.size() || assumed_in[q] != epoch) return 0;
          ksg_pod_summary sm;
          if (qmode[q] == 1 && !eng->summaries((uint32_t)q, 1, &sm, err)) return -1;
          const int32_t at = placement((uint32_t)q, qmode[q] == 1 ? &sm : nullptr);
          if (at < 0) return 0;
          gone_q.insert(q);
          Op o{false, Pod(), {}, k};
          o.qpod = q;
          o.qat = at;
          ops.push_back(std::move(o));
          continue;
        }
        Op o{false, Pod(), {}, k};
        if (added.count(k)) {  // added by this batch: the addition's program
          for (size_t j = ops.size(); j-- > 0;)
            if (ops[j].add && ops[j].key == k) { o.blob = ops[j].blob; break; }
        } else {
          PodMeta m;
          if (!compile(bound[bound_at.at(k)], 0, o.blob, m)) return 0;  // the re-encode path takes it
        }
        if (!added.erase(k)) removed.insert(k);
        ops.push_back(std::move(o));
      } else {
        return 0;
      }
    }
    // Room in the device existing-pod table (PTS/IPA profiles) for the batch's
    // additions, grown in place (queue pods get theirs before they are assumed).
    if (tables_on()) {
      uint64_t need[4] = {0, 0, 0, 0};
      for (auto& o : ops)
        if (o.add) table_need(o.pod, need);
      if (!ensure_room(need)) return -1;
    }
    // Host mirror first; device writes after (bound-pod deltas, then the queue
    // pods' Unreserve deltas and allocatable updates: row deltas commute).  A
    // device error part-way leaves the context unusable (broken): reload.
    vector<vector<uint8_t>> blobs;
    vector<int32_t> gn, sg, slot, rows;
    vector<std::pair<string, size_t>> adds;      // key, op slot of additions
    std::unordered_map<string, int32_t> add_slot;  // additions of this batch still present
    vector<std::pair<int32_t, int32_t>> unres;     // queue pod, node
    vector<std::tuple<int32_t, vector<int64_t>, int32_t>> allocs;  // node, allocatable, allowed pods
    vector<int32_t> restat;  // nodes whose label / flag columns are rewritten
    bool retaint = false;    // some node's taint list changed: the lists are re-uploaded
    for (auto& o : ops) {
      if (o.qpod >= 0) {
        unres.push_back({o.qpod, o.qat});
        qmode[o.qpod] = 2;  // deleted after it was scheduled: its result stays, its placement goes
        placed[o.qpod] = -1;
      } else if (o.node >= 0) {
        vector<int64_t> al(res.names.size(), 0);
        int32_t allowed = 0;
        for (auto& kv : o.nd.alloc) {  // as encode_snapshot
          if (kv.first == "pods") allowed = (int32_t)as_value(kv.second);
          int32_t r = res.get(kv.first);
          if (r >= 0) al[r] = r == 0 ? as_milli(kv.second) : as_value(kv.second);
        }
        allocs.emplace_back(o.node, std::move(al), allowed);
        if (o.statics) restat.push_back(o.node);
        retaint |= o.taints;
        nodes[o.node] = std::move(o.nd);
      } else if (o.add) {
        const int32_t k = (int32_t)blobs.size();
        gn.push_back(node_names.get(o.pod.node));
        sg.push_back(+1);
        slot.push_back(k);
        rows.push_back(-1);
        blobs.push_back(std::move(o.blob));
        add_slot[o.key] = k;
        adds.push_back({o.key, (size_t)k});
        bound_at[o.key] = (uint32_t)bound.size();
        bound.push_back(std::move(o.pod));
        bound_row.push_back(-1);  // known after the launches
      } else {
        const uint32_t i = bound_at.at(o.key);
        const int32_t k = (int32_t)blobs.size();
        auto it = add_slot.find(o.key);
        gn.push_back(node_names.get(bound[i].node));
        sg.push_back(-1);
        slot.push_back(it != add_slot.end() ? it->second : k);
        rows.push_back(bound_row[i]);
        blobs.push_back(std::move(o.blob));
        if (it != add_slot.end()) add_slot.erase(it);
        // swap with the last pod (bound-pod order does not enter any plugin's result)
        const uint32_t last = (uint32_t)bound.size() - 1;
        if (i != last) {
          std::swap(bound[i], bound[last]);
          std::swap(bound_row[i], bound_row[last]);
          bound_at[pkey(bound[i].ns, bound[i].name)] = i;
        }
        bound.pop_back();
        bound_row.pop_back();
        bound_at.erase(o.key);
      }
      inplace_dirty = true;
    }
    bool ok = sync_classes() && eng->bound_deltas(blobs, gn, sg, slot, rows, err);  // (term classes the added pods brought)
    for (size_t i = 0; ok && i < unres.size(); ++i)
      ok = refresh_program((uint32_t)unres[i].first) && eng->assume((uint32_t)unres[i].first, unres[i].second, -1, err);
    for (size_t i = 0; ok && i < allocs.size(); ++i)
      ok = eng->node_alloc(std::get<0>(allocs[i]), std::get<1>(allocs[i]), std::get<2>(allocs[i]), err);
    if (ok && !restat.empty()) {  // one batch, one synchronisation
      const size_t K = nkeys.names.size();
      vector<int32_t> gs, lv(restat.size() * K, -1);  // as encode_snapshot
      vector<uint8_t> hl, fl;
      for (size_t i = 0; i < restat.size(); ++i) {
        const Node& nd = nodes[restat[i]];
        gs.push_back((int32_t)restat[i]);
        for (auto& kv : nd.labels) lv[i * K + nkeys.get(kv.first)] = nvals[nkeys.get(kv.first)].get(kv.second);
        hl.push_back(nd.labels.empty() ? 0 : 1);
        fl.push_back(nd.unschedulable ? KSG_NODE_UNSCHEDULABLE : 0);
      }
      ok = eng->node_static(gs, lv, hl, fl, err);
    }
    if (ok && retaint) {
      vector<uint32_t> off, goff;
      vector<int32_t> ids, gids;
      taint_lists(lo, hi, off, ids);
      if (global_statics()) taint_lists(0, (uint32_t)nodes.size(), goff, gids);
      ok = eng->node_taints(off, ids, goff, gids, err);
    }
    if (!ok) {
      broken = true;
      return -1;
    }
    for (auto& a : adds)
      if (add_slot.count(a.first)) bound_row[bound_at.at(a.first)] = rows[a.second];
    bool full = false;  // (room was made above: a full table here re-encodes from the mirror)
    if (!eng->table_overflow(full, err)) return -1;
    return !full || rebuild() ? 1 : -1;
  }

  bool apply_events(const char* js, size_t len) {
    ++bprog_gen;
    ++node_gen;
    if (!compile_queue()) return false;
    try {
      docs.emplace_back(new J(json::parse(js, len)));
    } catch (std::exception& e) {
      err = e.what();
      return false;
    }
    const J& d = *docs.back();
    const J* ev = d["events"] ? d["events"] : &d;
    const J* re = d["reencode"];  // {"reencode": true}: skip the in-place path (A/B tests)
    if (!(re && re->b)) {
      int r = inplace_events(*ev);
      if (r != 0) return r > 0;
    }
    track_queue();
    const size_t ns = progs.size();
    vector<ksg_pod_summary> sum(ns);
    if (ns && !eng->summaries(0, (uint32_t)ns, sum.data(), err)) return false;
    vector<Node> nn = nodes;
    vector<Pod> bb = bound;
    vector<int8_t> qm = qmode;
    vector<int32_t> pl = placed;
    vector<int32_t> remap(nodes.size());  // original index -> current index (-1 removed)
    for (size_t i = 0; i < remap.size(); ++i) remap[i] = (int32_t)i;
    bool removed = false;
    auto node_at = [&](const string& name) -> int32_t {
      for (size_t i = 0; i < nn.size(); ++i)
        if (nn[i].name == name) return (int32_t)i;
      return -1;
    };
    auto pod_at = [&](const string& name, const string& pns) -> int32_t {
      for (size_t i = 0; i < bb.size(); ++i)
        if (bb[i].name == name && bb[i].ns == pns) return (int32_t)i;
      return -1;
    };
    // current node index of queue pod q's placement (-1 none)
    auto qplace = [&](size_t q) -> int32_t {
      int32_t at = qm[q] == 2 ? pl[q] : (qm[q] == 1 && q < ns && sum[q].status == 0 ? sum[q].selected : -1);
      if (at < 0) return -1;
      return qm[q] == 2 ? at : remap[at];  // summaries hold original indices until the rebuild
    };
    auto queue_at = [&](const string& name, const string& pns) -> int32_t {  // the first placed one
      if (const vector<uint32_t>* all = queue_all(pns, name))
        for (uint32_t q : *all)
          if (q < queue.size() && qplace(q) >= 0) return (int32_t)q;
      return -1;
    };
    for (auto& e : ev->items) {
      const string op = str_of(e["op"]);
      string pns;
      if (op == "addNode" || op == "updateNode") {
        if (!e["node"]) { err = op + ": no node object"; return false; }
        Node x = parse_node(*e["node"]);
        int32_t at = node_at(x.name);
        if (op == "addNode") {
          if (x.name.empty() || at >= 0) { err = "addNode: node '" + x.name + "' exists or has no name"; return false; }
          nn.push_back(std::move(x));
        } else {
          if (at < 0) { err = "updateNode: no node '" + x.name + "'"; return false; }
          nn[at] = std::move(x);
        }
      } else if (op == "removeNode") {
        string name = obj_name(e, "node", nullptr);
        int32_t at = node_at(name);
        if (at < 0) { err = "removeNode: no node '" + name + "'"; return false; }
        for (auto& p : bb)
          if (p.node == name) { err = "removeNode: pod " + p.ns + "/" + p.name + " is still bound to " + name; return false; }
        for (size_t q = 0; q < queue.size(); ++q)
          if (qplace(q) == at) { err = "removeNode: queue pod " + queue[q].name + " is assumed on " + name; return false; }
        nn.erase(nn.begin() + at);
        for (auto& r : remap)
          if (r == at) r = -1;
          else if (r > at) --r;
        for (size_t q = 0; q < queue.size(); ++q)
          if (qm[q] == 2 && pl[q] > at) --pl[q];
        removed = true;
      } else if (op == "addPod" || op == "updatePod") {
        if (!e["pod"]) { err = op + ": no pod object"; return false; }
        Pod p = parse_pod(*e["pod"]);
        if (p.node.empty()) { err = op + ": pod " + p.name + " has no spec.nodeName (pending pods enter through ksg_cycle)"; return false; }
        if (node_at(p.node) < 0) { err = op + ": pod " + p.name + " is bound to unknown node '" + p.node + "'"; return false; }
        int32_t at = pod_at(p.name, p.ns);
        if (op == "addPod") {
          if (at >= 0 || queue_at(p.name, p.ns) >= 0) { err = "addPod: pod " + p.ns + "/" + p.name + " exists"; return false; }
          bb.push_back(std::move(p));
        } else {
          if (at < 0) { err = "updatePod: no bound pod " + p.ns + "/" + p.name; return false; }
          bb[at] = std::move(p);
        }
      } else if (op == "removePod") {
        string name = obj_name(e, "pod", &pns);
        int32_t at = pod_at(name, pns);
        if (at >= 0) {
          bb.erase(bb.begin() + at);
        } else {
          int32_t q = queue_at(name, pns);
          if (q < 0) { err = "removePod: no bound or assumed pod " + pns + "/" + name; return false; }
          qm[q] = 2;  // deleted after it was scheduled: its result stays, its placement goes
          pl[q] = -1;
        }
      } else {
        err = "unknown event op '" + op + "'";
        return false;
      }
    }
    std::swap(nodes, nn);
    std::swap(bound, bb);
    std::swap(qmode, qm);
    std::swap(placed, pl);
    bound_at_valid = false;
    bool vol_ok = true;  // the batch may change what the volume plugins see (claim users)
    if (has_volume_plugins)
      for (size_t q = 0; q < queue.size() && vol_ok; ++q)
        if (qmode.size() <= q || qmode[q] == 0) vol_ok = volumes_modelled(queue[q]);
    if (!vol_ok || !equal_priorities()) {
      std::swap(nodes, nn);
      std::swap(bound, bb);
      std::swap(qmode, qm);
      std::swap(placed, pl);
      return false;
    }
    node_names = Dict();
    for (auto& n : nodes) node_names.add(n.name);
    return rebuild(removed ? &remap : nullptr);
  }

  bool compile_queue() {
    if (compiled) return true;
    for (auto& p : queue) register_classes(p);  // every class first: complete lists in one pass
    progs.assign(queue.size(), {});
    meta.assign(queue.size(), PodMeta());
    for (size_t q = 0; q < queue.size(); ++q)
      if (!compile(queue[q], (int32_t)(seq_base + q), progs[q], meta[q])) return false;
    prog_cls.assign(queue.size(), {(uint32_t)pcls.size(), (uint32_t)tcls.size()});
    if (!eng->set_programs(progs, err) || !sync_classes()) return false;
    compiled = true;
    return true;
  }

  // ------------------------------------------------------------ rendering
  static void jstr(string& o, const string& s) {
    static const char* hx = "0123456789abcdef";
    o += '"';
    for (size_t i = 0; i < s.size(); ++i) {
      unsigned char c = (unsigned char)s[i];
      switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\r': o += "\\r"; break;
        case '\t': o += "\\t"; break;
        default:
          if (c < 0x20 || c == '<' || c == '>' || c == '&') {
            o += "\\u00";
            o += hx[c >> 4];
            o += hx[c & 15];
          } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
                     ((unsigned char)s[i + 2] & 0xFE) == 0xA8) {
            o += ((unsigned char)s[i + 2] == 0xA8) ? "\\u2028" : "\\u2029";
            i += 2;
          } else {
            o += (char)c;
          }
      }
    }
    o += '"';
  }
  static string jmap(const map<string, string>& m) {
    string o = "{";
    for (auto it = m.begin(); it != m.end(); ++it) {
      if (it != m.begin()) o += ',';
      jstr(o, it->first);
      o += ':';
      jstr(o, it->second);
    }
    return o + "}";
  }

  string filter_message(int pos, uint32_t detail) const {  // pos: profile position
    switch (plugins[pos]) {
      case P_UNSCHED: return "node(s) were unschedulable";
      case P_NODENAME: return "node(s) didn't match the requested node name";
      case P_PORTS: return "node(s) didn't have free ports for the requested pod ports";
      case P_FIT: {
        string m;
        auto add = [&](const string& s) { m += (m.empty() ? "" : ", ") + s; };
        if (detail & KSG_FIT_TOO_MANY_PODS) add("Too many pods");
        for (size_t r = 0; r < res.names.size(); ++r)
          if (detail & (1u << (1 + r))) add("Insufficient " + res.names[r]);
        return m;
      }
      case P_TAINT: {
        if (detail >= taints.size()) return "node(s) had untolerated taint";  // (not a device code)
        const Taint& t = taints[detail];
        return "node(s) had untolerated taint {" + t.key + ": " + t.value + "}";
      }
      case P_NA: return "node(s) didn't match Pod's node affinity/selector";
      case P_PTS:
        return detail == KSG_PTS_MISSING_LABEL ? "node(s) didn't match pod topology spread constraints (missing required label)"
                                               : "node(s) didn't match pod topology spread constraints";
      case P_IPA:
        return detail == KSG_IPA_AFFINITY ? "node(s) didn't match pod affinity rules"
               : detail == KSG_IPA_ANTI_AFFINITY ? "node(s) didn't match pod anti-affinity rules"
                                                 : "node(s) didn't satisfy existing pods anti-affinity rules";
      case P_VOLUME:
      case P_VOLBIND: {  // Status.Message(): the reasons joined (volume_binding.go Filter appends them in this order)
        if (vkind[pos] == VK_RESTRICT)
          return "node has pod using PersistentVolumeClaim with the same name and ReadWriteOncePod access mode";
        if (vkind[pos] == VK_ZONE) return "node(s) had no available volume zone";
        if (vkind[pos] == VK_CSI) return "node(s) exceed max volume count";
        string m;
        auto add = [&](const char* r) { m += (m.empty() ? "" : ", ") + string(r); };
        if (detail & KSG_VOL_NODE_CONFLICT) add("node(s) had volume node affinity conflict");
        if (detail & KSG_VOL_BIND_CONFLICT) add("node(s) didn't find available persistent volumes to bind");
        if (detail & KSG_VOL_PV_NOT_EXIST) add("node(s) unavailable due to one or more pvc(s) bound to non-existent pv(s)");
        return m;
      }
    }
    return "";
  }

  // ------------------------------------------------------------ per-plugin statuses
  // What each wrapped plugin's extension point returns for the cycle of queue pod
  // q (the Go plugin API of ksg.h; render() records the same into the store).
  // framework.Code (v1.30 pkg/scheduler/framework/interface.go)
  enum { C_SUCCESS = 0, C_ERROR = 1, C_UNSCHED = 2, C_UNRESOLVABLE = 3, C_SKIP = 5 };
  // PreFilter Skip per plugin id (PreFilter / the NodeAffinity, PTS, IPA, NodePorts Skip rules)
  uint32_t skip_filter_mask(const PodMeta& m, const ksg_pod_summary& S) const {
    uint32_t skip_f = 0;
    if (m.flags & KPF_SKIP_NA_FILTER) skip_f |= 1u << P_NA;
    if (m.flags & KPF_SKIP_PTS_FILTER) skip_f |= 1u << P_PTS;
    if (m.ipa_no_req_terms && !(S.ipa_flags & 4u)) skip_f |= 1u << P_IPA;
    if (m.flags & KPF_SKIP_PORTS) skip_f |= 1u << P_PORTS;
    return skip_f;
  }
  // PreFilter Skip of profile position pos (skip_f: skip_filter_mask; volume plugins per position)
  bool filter_skipped(const PodMeta& m, uint32_t skip_f, int pos) const {
    return is_volume(plugins[pos]) ? ((m.vol_skip >> pos) & 1u) != 0 : (skip_f & (1u << plugins[pos])) != 0;
  }
  // profile position / detail a device filter code names (a volume run: its failing plugin)
  int code_pos(uint32_t code) const {
    const int base = fpos[code >> 24];
    return is_volume(plugins[base]) ? base + (int)((code >> 16) & 0xFFu) : base;
  }
  uint32_t code_detail(uint32_t code) const {
    return is_volume(plugins[fpos[code >> 24]]) ? code & 0xFFFFu : code & 0xFFFFFFu;
  }
  uint32_t skip_score_mask(const PodMeta& m, const ksg_pod_summary& S) const {
    uint32_t skip_s = 0;
    if (m.flags & KPF_SKIP_NA_SCORE) skip_s |= 1u << P_NA;
    if (m.flags & KPF_SKIP_PTS_SCORE) skip_s |= 1u << P_PTS;
    if (m.ipa_prescore_skip_static || !(S.ipa_flags & 8u)) skip_s |= 1u << P_IPA;
    skip_s |= 1u << P_VOLBIND;  // PreScore: no scorer (VolumeCapacityPriority off)
    return skip_s;
  }
  // PreFilter of profile position pos: the status code (-1: the plugin has no
  // PreFilter, or an earlier PreFilter rejected the pod and it never ran).
  int prefilter_status(uint32_t q, int pos, const ksg_pod_summary& S, string& msg) const {
    const PodMeta& m = meta[q];
    const uint32_t skip_f = skip_filter_mask(m, S);
    for (int p = 0; p < n_plugins; ++p) {
      if (!has_prefilter(plugins[p])) continue;
      if (p == pos) {
        if (p == m.prefilter_fail_pos && !m.merge_reject) { msg = m.prefilter_fail_msg; return C_UNRESOLVABLE; }
        msg.clear();
        return filter_skipped(m, skip_f, p) ? C_SKIP : C_SUCCESS;
      }
      if (p == m.prefilter_fail_pos) break;
    }
    return -1;
  }
  // Filter of profile position pos on local node i: the status code and message
  // (-1: not called: no Filter, PreFilter Skip / rejection, outside the
  // PreFilterResult, or an earlier filter failed on the node).
  int filter_status(uint32_t q, int pos, uint32_t i, const PodOutputs& o, string& msg) const {
    const PodMeta& m = meta[q];
    msg.clear();
    if (pos < 0 || pos >= n_plugins || !has_filter(plugins[pos])) return -1;
    if (m.prefilter_fail_pos >= 0 || filter_skipped(m, skip_filter_mask(m, o.summary), pos)) return -1;
    const uint32_t code = o.filter[i];
    if (code == KSG_FILTER_NOT_EVALUATED) return -1;
    const int fail_pos = code == KSG_FILTER_PASS ? n_plugins : code_pos(code);
    if (pos < fail_pos) return C_SUCCESS;
    if (pos > fail_pos) return -1;
    const uint32_t detail = code_detail(code);
    msg = filter_message(pos, detail);
    return filter_fail_code(q, pos, i, detail);
  }
  // fit.go Filter's code: UnschedulableAndUnresolvable when a failing request
  // exceeds the node's allocatable, else Unschedulable -- the one rule behind the
  // status calls, the cycle view and DefaultPreemption's potential nodes
  // (alloc_of(r): the node's allocatable of resource column r)
  template <class AllocOf>
  static int fit_fail_code(const vector<i64>& rq, uint32_t detail, size_t R, AllocOf alloc_of) {
    for (size_t r = 0; r < R; ++r)
      if ((detail & (1u << (1 + r))) && rq[r] > alloc_of(r)) return C_UNRESOLVABLE;
    return C_UNSCHED;
  }
  // framework.Code of a Filter failure of profile position pos on local node i
  int filter_fail_code(uint32_t q, int pos, uint32_t i, uint32_t detail) const {
    if (is_volume(plugins[pos])) return vkind[pos] == VK_RESTRICT || vkind[pos] == VK_CSI ? C_UNSCHED : C_UNRESOLVABLE;
    switch (plugins[pos]) {
      case P_FIT: {
        vector<i64> rq;
        i64 nzc = 0, nzm = 0;
        add_requests_const(queue[q], rq, nzc, nzm);
        const Node& nd = nodes[lo + i];
        return fit_fail_code(rq, detail, res.names.size(), [&](size_t r) -> i64 {
          auto it = nd.alloc.find(res.names[r]);
          return it == nd.alloc.end() ? 0 : (r == 0 ? as_milli(it->second) : as_value(it->second));
        });
      }
      case P_PTS: return detail == KSG_PTS_MISSING_LABEL ? C_UNRESOLVABLE : C_UNSCHED;
      case P_IPA: return detail == KSG_IPA_AFFINITY ? C_UNRESOLVABLE : C_UNSCHED;
      case P_PORTS: return C_UNSCHED;
      default: return C_UNRESOLVABLE;  // TaintToleration, NodeAffinity, NodeUnschedulable, NodeName
    }
  }
  // The same rule per profile position, for the device view (Engine::view)
  ksg::Engine::ViewCfg vcfg_;
  bool vcfg_ok_ = false;
  const ksg::Engine::ViewCfg& view_cfg() {
    if (!vcfg_ok_) {
      ksg::Engine::ViewCfg v;
      v.n_profile = n_plugins;
      for (int d = 0; d < KSG_MAX_PLUGINS; ++d) {
        v.prof_of_dev[d] = fpos[d];
        v.dev_vol[d] = fpos[d] >= 0 && fpos[d] < n_plugins && is_volume(plugins[fpos[d]]);
      }
      for (int pos = 0; pos < n_plugins && pos < KSG_MAX_PROFILE; ++pos) {
        int k = 0;
        if (is_volume(plugins[pos])) k = vkind[pos] == VK_RESTRICT || vkind[pos] == VK_CSI ? 1 : 0;
        else if (plugins[pos] == P_FIT) k = 2;
        else if (plugins[pos] == P_PTS) k = 3;
        else if (plugins[pos] == P_IPA) k = 4;
        else if (plugins[pos] == P_PORTS) k = 1;
        v.kind[pos] = k;
      }
      vcfg_ = v;
      vcfg_ok_ = true;
    }
    return vcfg_;
  }
  // PreScore of profile position pos (-1: no PreScore, or no scoring: one feasible
  // node / none, or a PreScore before it failed).  NodeAffinity's PreScore fails
  // on an invalid preferred term (the cycle's Error: a status 2 with more than
  // one feasible node comes from there; node_affinity.go PreScore).
  static constexpr const char* kNaPrefErr = "invalid preferred node affinity term";
  int prescore_status(uint32_t q, int pos, const ksg_pod_summary& S, string& msg) const {
    msg.clear();
    if (pos < 0 || pos >= n_plugins || !has_prescore(plugins[pos])) return -1;
    const PodMeta& m = meta[q];
    if (m.prefilter_fail_pos >= 0 || S.feasible <= 1) return -1;
    if (S.status == 2) {
      if (!m.na_prescore_error) return -1;
      const int na = pos_of(P_NA);
      if (pos > na) return -1;
      if (pos == na) { msg = kNaPrefErr; return C_ERROR; }
    }
    return (skip_score_mask(m, S) & (1u << plugins[pos])) ? C_SKIP : C_SUCCESS;
  }
  void add_requests_const(const Pod& p, vector<i64>& out_req, i64& nzc, i64& nzm) const {
    out_req.assign(res.names.size(), 0);
    for (auto& kv : p.req) {
      const int32_t r = res.get(kv.first);
      if (r >= 0) out_req[r] = wadd(out_req[r], r == 0 ? as_milli(kv.second) : as_value(kv.second));
    }
    auto c = p.req_nz.find("cpu");
    auto mm = p.req_nz.find("memory");
    nzc = c == p.req_nz.end() ? 0 : as_milli(c->second);
    nzm = mm == p.req_nz.end() ? 0 : as_value(mm->second);
  }
  // Kept outputs of queue pod q, cached until the next run (ABI lookups per node).
  uint64_t out_gen = 0;
  int64_t oc_q = -1;
  uint64_t oc_gen = 0;
  PodOutputs oc;
  vector<int32_t> oc_norm;
  bool oc_norm_ok = false;
  const PodOutputs* outputs_of(uint32_t q) {
    if (oc_q != (int64_t)q || oc_gen != out_gen) {
      if (!eng->outputs(q, oc, err)) { oc_q = -1; return nullptr; }
      oc_q = q;
      oc_gen = out_gen;
      oc_norm_ok = false;
    }
    return &oc;
  }
  const vector<int32_t>* normalized_of(uint32_t q) {
    if (!outputs_of(q)) return nullptr;
    if (!oc_norm_ok) {
      if (!eng->normalized(q, oc_norm, err)) return nullptr;
      oc_norm_ok = true;
    }
    return &oc_norm;
  }

  bool render(uint32_t q, string& out) {
    PodOutputs o;
    if (!eng->outputs(q, o, err)) return false;
    const ksg_pod_summary& S = o.summary;
    const PodMeta& m = meta[q];
    uint32_t n = hi - lo;
    map<string, string> pre_status, pre_score;
    map<string, vector<string>> pre_result;
    map<string, map<string, string>> filt, score, fin;
    // skip sets
    const uint32_t skip_f = skip_filter_mask(m, S);
    uint32_t skip_s = 0;
    bool aborted = false;
    for (int pos = 0; pos < n_plugins && !aborted; ++pos) {
      int id = plugins[pos];
      if (!has_prefilter(id)) continue;
      string msg = "success";
      if (filter_skipped(m, skip_f, pos)) msg = "";
      if (pos == m.prefilter_fail_pos) {
        msg = m.prefilter_fail_msg;
        aborted = true;
      }
      pre_status[names[pos]] = msg;
      if (id == P_NA && m.restricted) pre_result[names[pos]] = m.prefilter_names;
      if (vkind[pos] == VK_BIND && m.vb_restricted) pre_result[names[pos]] = m.vb_names;
    }
    if (!aborted) {
      for (uint32_t i = 0; i < n; ++i) {
        uint32_t code = o.filter[i];
        if (code == KSG_FILTER_NOT_EVALUATED) continue;
        int fail_pos = code == KSG_FILTER_PASS ? n_plugins : code_pos(code);
        auto& row = filt[nodes[lo + i].name];
        for (int pos = 0; pos < n_plugins; ++pos) {
          int id = plugins[pos];
          if (!has_filter(id) || filter_skipped(m, skip_f, pos)) continue;
          if (pos < fail_pos) row[names[pos]] = "passed";
          else if (pos == fail_pos) { row[names[pos]] = filter_message(pos, code_detail(code)); break; }
        }
      }
      if (S.feasible > 1 && S.status == 2 && m.na_prescore_error)  // PreScore ran up to NodeAffinity's error
        for (int pos = 0; pos < n_plugins; ++pos) {
          string msg;
          const int code = prescore_status(q, pos, S, msg);
          if (code >= 0) pre_score[names[pos]] = code == C_SUCCESS ? "success" : msg;
        }
      if (S.feasible > 1 && S.status != 2) {
        skip_s = skip_score_mask(m, S);
        for (int pos = 0; pos < n_plugins; ++pos)
          if (has_prescore(plugins[pos])) pre_score[names[pos]] = (skip_s & (1u << plugins[pos])) ? "" : "success";
        vector<int32_t> norm;  // NormalizeScore on the device (k_norm_out: the selection's normalize_pos)
        if (!eng->normalized(q, norm, err)) return false;
        for (uint32_t i = 0; i < n; ++i) {
          if (o.filter[i] != KSG_FILTER_PASS) continue;
          const string& nm = nodes[lo + i].name;
          for (int pos = 0; pos < n_plugins; ++pos) {
            int id = plugins[pos];
            if (!has_score(id) || (skip_s & (1u << id))) continue;
            const i64 raw = o.score[(size_t)dpos[pos] * n + i];
            score[nm][names[pos]] = std::to_string(raw);
            // applyWeightOnScore (store.go:504-507): normalized x the store's weight
            fin[nm][names[pos]] = std::to_string((i64)norm[(size_t)dpos[pos] * n + i] * store_w[pos]);
          }
        }
      }
    }
    string sel = S.status == 0 && S.selected >= 0 ? nodes[S.selected].name : "";
    // PostFilter: DefaultPreemption records every node of the status map (all of
    // them), the nominated one with PostFilterNominatedMessage (store.go:442-458)
    string post = "{}";
    if (S.status == 1)
      for (int pos = 0; pos < n_plugins; ++pos)
        if (names[pos] == "DefaultPreemption") {
          const int32_t nominated = q < nom.size() ? nom[q].node : -1;
          vector<std::pair<string, bool>> nn;  // encoding/json: map keys sorted
          for (uint32_t i = 0; i < n; ++i) nn.push_back({nodes[lo + i].name, (int32_t)(lo + i) == nominated});
          std::sort(nn.begin(), nn.end());
          post = "{";
          for (size_t i = 0; i < nn.size(); ++i) {
            if (i) post += ',';
            jstr(post, nn[i].first);
            if (!nn[i].second) {
              post += ":{}";
              continue;
            }
            post += ":{";
            jstr(post, names[pos]);
            post += ":\"preemption victim\"}";
          }
          post += "}";
        }
    map<string, string> reserve, prebind, bind;  // binding cycle of a scheduled pod (the bind assumed to succeed)
    if (!sel.empty())
      for (int pos = 0; pos < n_plugins; ++pos) {
        if (plugins[pos] == P_VOLBIND) reserve[names[pos]] = prebind[names[pos]] = "success";
        if (names[pos] == "DefaultBinder") bind[names[pos]] = "success";
      }
    auto j2 = [&](const map<string, map<string, string>>& mm) {
      string s = "{";
      for (auto it = mm.begin(); it != mm.end(); ++it) {
        if (it != mm.begin()) s += ',';
        jstr(s, it->first);
        s += ':';
        s += jmap(it->second);
      }
      return s + "}";
    };
    string pr = "{";
    for (auto it = pre_result.begin(); it != pre_result.end(); ++it) {
      if (it != pre_result.begin()) pr += ',';
      jstr(pr, it->first);
      pr += ":[";
      for (size_t k = 0; k < it->second.size(); ++k) {
        if (k) pr += ',';
        jstr(pr, it->second[k]);
      }
      pr += ']';
    }
    pr += "}";
    const string P = "kube-scheduler-simulator.sigs.k8s.io/";
    map<string, string> ann{{P + "prefilter-result", pr},          {P + "prefilter-result-status", jmap(pre_status)},
                            {P + "filter-result", j2(filt)},       {P + "postfilter-result", post},
                            {P + "prescore-result", jmap(pre_score)}, {P + "score-result", j2(score)},
                            {P + "finalscore-result", j2(fin)},    {P + "reserve-result", jmap(reserve)},
                            {P + "permit-result", "{}"},           {P + "permit-result-timeout", "{}"},
                            {P + "prebind-result", jmap(prebind)}, {P + "bind-result", jmap(bind)},
                            {P + "selected-node", sel}};
    out = jmap(ann);
    return true;
  }

};

}  // namespace host
}  // namespace ksg

// ================================================================== C ABI
using ksg::host::Cluster;

// Every entry point that takes a context holds its (recursive) mutex for the
// call, so calls from several threads are serialised by the library; the
// per-node reads of the framework's parallel Filter / Score workers go through
// a ksg_cycle_view instead (no call, no lock).  last_error is also kept per
// thread: ksg_last_error returns the calling thread's last failure on ctx.
// The thread-local copy is tagged with the context's generation id (unique per
// ksg_create), so a context freed and reallocated at the same address never
// returns its predecessor's error.
static std::atomic<uint64_t> g_ctx_gen{0};
static thread_local const void* t_err_ctx = nullptr;
static thread_local uint64_t t_err_gen = 0;
static thread_local std::string t_err;
static thread_local bool t_err_own = false;  // t_err was set by this thread's own failing call
struct ksg_ctx {
  Cluster c;
  std::string last_error;
  mutable std::recursive_mutex mu;
  const uint64_t gen = ++g_ctx_gen;
  // the victim-store warm-up after a load (Cluster::warm_step), stopped and joined
  // before the next load and at destruction (never while holding mu: a slice takes it)
  std::thread warm;
  std::atomic<bool> warm_stop{false};
  void stop_warm() {
    warm_stop = true;
    if (warm.joinable()) warm.join();
    warm_stop = false;
  }
  void start_warm();
  ~ksg_ctx();
  int fail(const std::string& m, int code) {
    last_error = m;
    t_err_ctx = this;
    t_err_gen = gen;
    t_err = m;
    t_err_own = true;
    return code;
  }
};
namespace ksg {
bool rccl_selftest(int device, size_t bytes, std::string& err);  // engine.hip (diagnostic)
}
#define KSG_LOCK(ctx)                                 \
  std::unique_lock<std::recursive_mutex> ksg_lk_;    \
  if (ctx) ksg_lk_ = std::unique_lock<std::recursive_mutex>((ctx)->mu)

// A context whose device state a failed in-place update left half-applied
// refuses every call but ksg_load_cluster / ksg_destroy / ksg_last_error.
#define KSG_GUARD(ctx)                                                                                   \
  do {                                                                                                   \
    if (!(ctx)) return KSG_E_INVALID;                                                                    \
    if ((ctx)->c.eng && (ctx)->c.eng->lost()) (ctx)->c.broken = true;                                    \
    if ((ctx)->c.broken) return (ctx)->fail("context unusable after a device error: reload", KSG_E_STATE); \
  } while (0)

// Contexts with a running warm-up: joined at library teardown, before the HIP
// runtime's own (a thread still inside a HIP call at process exit would race it).
static std::mutex g_warm_mu;
static std::set<ksg_ctx*> g_warm_ctx;
static struct WarmTeardown {
  ~WarmTeardown() {
    std::lock_guard<std::mutex> g(g_warm_mu);
    for (ksg_ctx* c : g_warm_ctx) {
      c->warm_stop = true;
      if (c->warm.joinable()) c->warm.join();
    }
    g_warm_ctx.clear();
  }
} g_warm_teardown;
void ksg_ctx::start_warm() {
  {
    std::lock_guard<std::mutex> g(g_warm_mu);
    g_warm_ctx.insert(this);
  }
  c.warm_running = true;  // (under the load's lock)
  warm = std::thread([this] {
    for (;;) {
      {
        std::lock_guard<std::recursive_mutex> g(mu);
        if (warm_stop || c.warm_step(4096)) {
          c.warm_running = false;
          return;
        }
      }
      std::this_thread::yield();  // (a foreground call may take the lock between slices)
    }
  });
}
ksg_ctx::~ksg_ctx() {
  stop_warm();
  std::lock_guard<std::mutex> g(g_warm_mu);
  g_warm_ctx.erase(this);
}

extern "C" {

int ksg_abi_version(void) { return KSG_ABI_VERSION; }

int ksg_create(const char* profile_json, size_t len, const ksg_opts* opts, ksg_ctx** out) {
  if (!out || !profile_json) return KSG_E_INVALID;
  *out = nullptr;
  std::unique_ptr<ksg_ctx> ctx(new ksg_ctx());
  try {
    ksg::json::Node pr = ksg::json::parse(profile_json, len);
    const ksg::json::Node* p = pr["profile"] ? pr["profile"] : &pr;
    if (!ctx->c.load_profile(*p)) return KSG_E_INVALID;
  } catch (std::exception& e) {
    return KSG_E_INVALID;
  }
  if (opts) {
    ctx->c.ecfg.device = opts->device;
    ctx->c.ecfg.stream = opts->stream;
    ctx->c.rank = opts->shard_rank;
    ctx->c.shards = opts->shard_count ? opts->shard_count : 1;
    if (ctx->c.rank >= ctx->c.shards) return KSG_E_INVALID;
  }
  ctx->c.eng.reset(new ksg::Engine());
  std::string err;
  if (!ctx->c.eng->init(ctx->c.ecfg, err)) return KSG_E_DEVICE;
  *out = ctx.release();
  return KSG_OK;
}

void ksg_destroy(ksg_ctx* ctx) {
  if (ctx && t_err_ctx == ctx) t_err_ctx = nullptr;
  delete ctx;
}

// Always the calling thread's own copy: another thread's fail() can reassign
// ctx->last_error after the lock is released, so it is copied under the lock.
const char* ksg_last_error(const ksg_ctx* ctx) {
  if (!ctx) return "null context";
  // this thread's own failure on ctx; otherwise the context's current error,
  // copied under the lock on every call (a newer failure of another thread shows)
  if (t_err_own && t_err_ctx == ctx && t_err_gen == ctx->gen) return t_err.c_str();
  KSG_LOCK(ctx);
  t_err = ctx->last_error;
  t_err_ctx = ctx;
  t_err_gen = ctx->gen;
  t_err_own = false;
  return t_err.c_str();
}

int ksg_load_cluster(ksg_ctx* ctx, const char* json, size_t len) {
  if (ctx) ctx->stop_warm();  // (before the lock: a warm-up slice holds it)
  KSG_LOCK(ctx);
  if (!ctx || !json) return KSG_E_INVALID;
  ctx->c.out_gen++;
  ctx->c.room_ok = false;  // (room_ok: see Cluster::ensure_room)
  try {
    Cluster& c = ctx->c;
    // fix the engine's global node offset for this shard before upload
    if (!c.load(json, len)) return ctx->fail(c.err, KSG_E_INVALID);
    c.warm_started = c.warm_done = false;
    c.warm_ms = -1;
    c.warm_t0 = Cluster::now_us();
    if (c.warm_wanted()) ctx->start_warm();  // (it waits for this call's lock)
  } catch (std::exception& e) {
    return ctx->fail(e.what(), KSG_E_INVALID);
  }
  return KSG_OK;
}

int ksg_num_nodes(const ksg_ctx* ctx) {
  KSG_LOCK(ctx);
  return ctx ? (int)ctx->c.nodes.size() : KSG_E_INVALID;
}
int ksg_queue_len(const ksg_ctx* ctx) {
  KSG_LOCK(ctx);
  return ctx ? (int)ctx->c.queue.size() : KSG_E_INVALID;
}

int ksg_keep_outputs(ksg_ctx* ctx, uint32_t first, uint32_t count) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  ctx->c.out_gen++;
  if (!ctx->c.eng->keep_outputs(first, count, ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_DEVICE);
  return KSG_OK;
}

int ksg_schedule_queue(ksg_ctx* ctx, uint32_t first, uint32_t count) {
  rtx::Range rr("ksg_schedule_queue");
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  ctx->c.out_gen++;
  ctx->c.room_ok = false;  // (room_ok: see Cluster::ensure_room)
  Cluster& c = ctx->c;
  if (first + count > c.queue.size()) return ctx->fail("queue range", KSG_E_RANGE);
  if (c.shards != 1 && c.eng->exchange_ranks() != c.shards)
    return ctx->fail("sharded context: call ksg_set_exchange first", KSG_E_STATE);
  if (!c.compile_queue()) return ctx->fail(c.err, KSG_E_INVALID);
  if (!c.refresh_programs(first, count)) return ctx->fail(c.err, KSG_E_DEVICE);
  if (c.tables_on()) {  // the run appends every scheduled pod to the existing-pod table
    uint64_t need[4] = {0, 0, 0, 0};
    for (uint32_t q = first; q < first + count; ++q) c.queue_need(q, need);
    if (!c.ensure_room(need)) return ctx->fail(c.err, KSG_E_DEVICE);  // grown in place, contents kept
  }
  // Pods that may preempt end a segment: the run stops after each, and an
  // unschedulable one gets its DefaultPreemption dry run on the state of its own
  // cycle (Cluster::preempt); the call then returns with those segments done.
  if (c.nom.size() < c.queue.size()) c.nom.resize(c.queue.size());
  uint32_t j = first;
  // (without DefaultPreemption no pod is ever nominated: nothing to clear or stop for)
  const bool may_nominate = c.has_preemption();
  for (uint32_t q = first; may_nominate && q < first + count; ++q) {
    c.nom[q] = Cluster::Nomination();
    if (!c.may_preempt(q)) continue;
    ksg_pod_summary S;
    if (!c.eng->run_queue(j, q + 1 - j, true, c.err) || !c.eng->sync(c.err)) return ctx->fail(c.err, KSG_E_DEVICE);
    c.mark_run(j, q + 1 - j);
    if (!c.eng->summaries(q, 1, &S, c.err) || !c.preempt(q, S)) return ctx->fail(c.err, KSG_E_DEVICE);
    if (!c.refresh_programs(q + 1, first + count - q - 1)) return ctx->fail(c.err, KSG_E_DEVICE);
    j = q + 1;
  }
  if (j < first + count) {
    if (!c.eng->run_queue(j, first + count - j, true, c.err)) return ctx->fail(c.err, KSG_E_DEVICE);
    c.mark_run(j, first + count - j);
  }
  return KSG_OK;
}

int ksg_compact(ksg_ctx* ctx, uint32_t keep_from) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  ctx->c.out_gen++;
  ctx->c.room_ok = false;  // (room_ok: see Cluster::ensure_room)
  if (!ctx->c.compact(keep_from)) return ctx->fail(ctx->c.err, KSG_E_STATE);
  return KSG_OK;
}

int ksg_whatif(ksg_ctx* ctx, uint32_t first, uint32_t count) {
  rtx::Range rr("ksg_whatif");
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  ctx->c.out_gen++;
  ctx->c.room_ok = false;  // (room_ok: see Cluster::ensure_room)
  Cluster& c = ctx->c;
  if (first + count > c.queue.size()) return ctx->fail("queue range", KSG_E_RANGE);
  if (c.shards != 1 && c.eng->exchange_ranks() != c.shards)
    return ctx->fail("sharded context: call ksg_set_exchange first", KSG_E_STATE);
  if (!c.compile_queue()) return ctx->fail(c.err, KSG_E_INVALID);
  if (!c.refresh_programs(first, count)) return ctx->fail(c.err, KSG_E_DEVICE);
  if (c.tables_on()) {  // the step's binds append its pods to the existing-pod table
    uint64_t need[4] = {0, 0, 0, 0};
    for (uint32_t q = first; q < first + count; ++q) c.queue_need(q, need);
    if (!c.ensure_room(need)) return ctx->fail(c.err, KSG_E_DEVICE);
  }
  if (c.nom.size() < c.queue.size()) c.nom.resize(c.queue.size());
  if (c.has_preemption())  // (a what-if step runs no PostFilter; without DefaultPreemption none ever ran)
    for (uint32_t q = first; q < first + count; ++q) c.nom[q] = Cluster::Nomination();
  if (!c.eng->run_whatif(first, count, c.err)) return ctx->fail(c.err, KSG_E_STATE);
  c.mark_run(first, count);
  return KSG_OK;
}

int ksg_wait(ksg_ctx* ctx, float* ms) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  if (!ctx->c.eng->sync(ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_DEVICE);
  if (ms) *ms = ctx->c.eng->last_ms();
  if (ctx->c.tables_on()) {  // capacity is checked before every run; an overflow is a bug, not a state
    bool full = false;
    if (!ctx->c.eng->table_overflow(full, ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_DEVICE);
    if (full) {
      ctx->c.broken = true;
      return ctx->fail("existing-pod table overflow: results of this run are not valid; reload", KSG_E_STATE);
    }
  }
  return KSG_OK;
}

int ksg_pod_results(ksg_ctx* ctx, uint32_t first, uint32_t count, ksg_pod_result* out) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  if (!ctx || !out) return KSG_E_INVALID;
  Cluster& c = ctx->c;
  if (first + count > c.queue.size()) return ctx->fail("queue range", KSG_E_RANGE);
  std::vector<ksg_pod_summary> s(count);
  if (count && !c.eng->summaries(first, count, s.data(), c.err)) return ctx->fail(c.err, KSG_E_DEVICE);
  for (uint32_t i = 0; i < count; ++i) {
    out[i].selected = s[i].selected;
    out[i].feasible = s[i].feasible;
    out[i].status = s[i].status;
    out[i].skip_filter = s[i].skip_filter;
    out[i].skip_score = s[i].skip_score;
    out[i].total = (int32_t)(s[i].best_key >> 40);
  }
  return KSG_OK;
}

int ksg_filter_codes(ksg_ctx* ctx, uint32_t q, uint32_t* out, uint32_t n) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  if (!ctx || !out) return KSG_E_INVALID;
  ksg::PodOutputs o;
  if (!ctx->c.eng->outputs(q, o, ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_STATE);
  if (n < o.filter.size()) return KSG_E_NOBUF;
  for (size_t i = 0; i < o.filter.size(); ++i) {  // device position -> profile position
    uint32_t c = o.filter[i];
    out[i] = c >= KSG_FILTER_NOT_EVALUATED ? c : ((uint32_t)ctx->c.code_pos(c) << 24) | ctx->c.code_detail(c);
  }
  return KSG_OK;
}

int ksg_scores(ksg_ctx* ctx, uint32_t q, uint32_t pos, int32_t* out, uint32_t n) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  if (!ctx || !out) return KSG_E_INVALID;
  ksg::PodOutputs o;
  if (!ctx->c.eng->outputs(q, o, ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_STATE);
  size_t N = o.filter.size();
  if (n < N) return KSG_E_NOBUF;
  if (pos >= (uint32_t)ctx->c.n_plugins || ctx->c.dpos[pos] < 0) return ctx->fail("no device scores at this position", KSG_E_INVALID);
  const size_t d = (size_t)ctx->c.dpos[pos];
  std::copy(o.score.begin() + d * N, o.score.begin() + (d + 1) * N, out);
  return KSG_OK;
}

int ksg_annotations(ksg_ctx* ctx, uint32_t q, char* buf, size_t cap, size_t* len) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  if (!ctx || !len) return KSG_E_INVALID;
  std::string s;
  if (q >= ctx->c.queue.size()) return ctx->fail("queue range", KSG_E_RANGE);
  if (!ctx->c.render(q, s)) return ctx->fail(ctx->c.err, KSG_E_STATE);
  *len = s.size();
  if (!buf || cap < s.size()) return KSG_E_NOBUF;
  std::memcpy(buf, s.data(), s.size());
  return KSG_OK;
}

int ksg_reset(ksg_ctx* ctx) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  ctx->c.out_gen++;
  ctx->c.room_ok = false;  // (room_ok: see Cluster::ensure_room)
  if (ctx->c.inplace_dirty)
    return ctx->fail("reset after in-place cluster events: reload the cluster (ksg_load_cluster)", KSG_E_STATE);
  if (!ctx->c.compile_queue()) return ctx->fail(ctx->c.err, KSG_E_INVALID);
  if (!ctx->c.eng->reset(ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_DEVICE);
  ctx->c.forget_epoch();
  return KSG_OK;
}

int ksg_sample_kernel(ksg_ctx* ctx, uint32_t every) {
  KSG_LOCK(ctx);
  if (!ctx) return KSG_E_INVALID;
  ctx->c.eng->sample_kernel(every);
  return KSG_OK;
}

int ksg_set_path(ksg_ctx* ctx, int per_pod) {
  KSG_LOCK(ctx);
  if (!ctx) return KSG_E_INVALID;
  ctx->c.eng->set_path(per_pod);
  return KSG_OK;
}

// diagnostic (not in ksg.h): fixup-loop s_memtime stamps, 8 per pod
extern "C" int ksg_debug_fixup_stamps(ksg_ctx* ctx, uint32_t count, uint64_t* out) {
  KSG_LOCK(ctx);
  if (!ctx) return KSG_E_INVALID;
  std::vector<uint64_t> v;
  if (!ctx->c.eng->fixup_stamps(count, out ? &v : nullptr, ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_DEVICE);
  if (out) std::copy(v.begin(), v.end(), out);
  return KSG_OK;
}

extern "C" int ksg_debug_eval_stamps(ksg_ctx* ctx, int on, uint64_t* out, size_t* n) {
  KSG_LOCK(ctx);
  if (!ctx) return KSG_E_INVALID;
  std::vector<uint64_t> v;
  if (!ctx->c.eng->eval_stamps(on != 0, out ? &v : nullptr, ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_DEVICE);
  if (out) std::copy(v.begin(), v.end(), out);
  if (n) *n = v.size();
  return KSG_OK;
}

// diagnostic (not in ksg.h): out[6] = pods run through the table chain / the scanning
// chain so far, of the first those whose cycle was one launch, what-if pod chunks
// that ran the class path, table-chain pods of persistent segments (k_chain_run)
// and those segments, segments that fell back to the two-launch chain, 0
extern "C" int ksg_debug_path_counts(ksg_ctx* ctx, uint64_t* out) {
  KSG_LOCK(ctx);
  if (!ctx || !out) return KSG_E_INVALID;
  ctx->c.eng->path_counts(out);
  return KSG_OK;
}

// diagnostic (not in ksg.h): DefaultPreemption dry runs that took the batched search
extern "C" int ksg_debug_preempt_batched(ksg_ctx* ctx, uint64_t* out) {
  KSG_LOCK(ctx);
  if (!ctx || !out) return KSG_E_INVALID;
  *out = ctx->c.preempt_batched_runs;
  return KSG_OK;
}

int ksg_nccl_unique_id(uint8_t* out128) {
  std::string err;
  if (!out128) return KSG_E_INVALID;
  return ksg::Engine::nccl_unique_id(out128, err) ? KSG_OK : KSG_E_DEVICE;
}

int ksg_set_exchange(ksg_ctx* ctx, int mode, const uint8_t* nccl_id, ksg_exchange_fn fn, void* user) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  Cluster& c = ctx->c;
  if (!c.eng->set_exchange(mode, nccl_id, c.rank, c.shards, fn, user, c.err)) return ctx->fail(c.err, KSG_E_DEVICE);
  return KSG_OK;
}

int ksg_batch_path(const ksg_ctx* ctx) {
  KSG_LOCK(ctx);
  return ctx ? (ctx->c.eng->batch_path() ? 1 : 0) : KSG_E_INVALID;
}

// diagnostic (not in ksg.h): a one-rank RCCL communicator's all-gather on `device`
// (the calls the exchange's mode 1 makes; error text into err_buf)
extern "C" int ksg_debug_rccl_selftest(int device, size_t bytes, char* err_buf, size_t cap) {
  std::string err;
  const bool ok = ksg::rccl_selftest(device, bytes, err);
  if (err_buf && cap) {
    std::snprintf(err_buf, cap, "%s", err.c_str());
  }
  return ok ? KSG_OK : KSG_E_DEVICE;
}

// diagnostic (not in ksg.h): the drop-in cycle's host phases (Cluster::ctimes), 8
// doubles; reset = 1 clears them after the read
extern "C" int ksg_debug_cycle_times(ksg_ctx* ctx, double* out, int reset) {
  KSG_LOCK(ctx);
  if (!ctx) return KSG_E_INVALID;
  if (out) std::memcpy(out, ctx->c.ctimes, sizeof(ctx->c.ctimes));
  if (reset) std::memset(ctx->c.ctimes, 0, sizeof(ctx->c.ctimes));
  return KSG_OK;
}

// diagnostic (not in ksg.h): the preemption dry runs' host phases (Cluster::ptimes), 4
// doubles; reset = 1 clears them after the read
// Diagnostic: the victim-store warm-up after the last load: 1 done (*ms: load to
// current store), 0 running, -1 none (not wanted, stopped, or failed).
extern "C" int ksg_debug_victim_warm(ksg_ctx* ctx, double* ms) {
  if (!ctx) return KSG_E_INVALID;
  KSG_LOCK(ctx);
  if (ms) *ms = ctx->c.warm_ms;
  return ctx->c.warm_done ? 1 : ctx->c.warm_running ? 0 : -1;
}
extern "C" int ksg_debug_preempt_times(ksg_ctx* ctx, double* out, int reset) {
  KSG_LOCK(ctx);
  if (!ctx) return KSG_E_INVALID;
  if (out) std::memcpy(out, ctx->c.ptimes, sizeof(ctx->c.ptimes));
  if (reset) std::memset(ctx->c.ptimes, 0, sizeof(ctx->c.ptimes));
  return KSG_OK;
}

// diagnostic (not in ksg.h): static-record chunks computed from decoded pods (k_static_dec)
// diagnostic (not in ksg.h): cycle views k_eval wrote itself (the fused view, Engine::view_arm)
extern "C" int ksg_debug_views_fused(ksg_ctx* ctx, uint64_t* out) {
  KSG_LOCK(ctx);
  if (!ctx || !out) return KSG_E_INVALID;
  *out = ctx->c.eng->views_fused();
  return KSG_OK;
}
extern "C" int ksg_debug_static_dec_chunks(ksg_ctx* ctx, uint64_t* out) {
  KSG_LOCK(ctx);
  if (!ctx || !out) return KSG_E_INVALID;
  *out = ctx->c.eng->static_dec_chunks();
  return KSG_OK;
}
extern "C" int ksg_debug_static_overlaps(ksg_ctx* ctx, uint64_t* out) {
  KSG_LOCK(ctx);
  if (!ctx || !out) return KSG_E_INVALID;
  *out = ctx->c.eng->static_overlaps();
  return KSG_OK;
}

// diagnostic (not in ksg.h): the sampled run's k_static launches (cfg3 roofline)
extern "C" int ksg_debug_static_time(ksg_ctx* ctx, float* total_ms, uint32_t* launches, uint64_t* pods) {
  KSG_LOCK(ctx);
  if (!ctx || !total_ms || !launches || !pods) return KSG_E_INVALID;
  if (!ctx->c.eng->static_time(*total_ms, *launches, *pods, ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_DEVICE);
  return KSG_OK;
}

int ksg_kernel_time(ksg_ctx* ctx, float* avg_ms, uint32_t* samples) {
  KSG_LOCK(ctx);
  if (!ctx || !avg_ms || !samples) return KSG_E_INVALID;
  if (!ctx->c.eng->kernel_time(*avg_ms, *samples, ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_DEVICE);
  return KSG_OK;
}

int ksg_cycle(ksg_ctx* ctx, const char* pod_json, size_t len, int commit, ksg_pod_result* out) {
  rtx::Range rr("ksg_cycle");
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  ctx->c.out_gen++;
  if (!ctx || !pod_json) return KSG_E_INVALID;
  ksg_pod_summary s;
  try {
    if (!ctx->c.cycle(pod_json, len, commit != 0, s)) return ctx->fail(ctx->c.err, KSG_E_STATE);
  } catch (std::exception& e) {
    return ctx->fail(e.what(), KSG_E_INVALID);
  }
  if (out) {
    out->selected = s.selected;
    out->feasible = s.feasible;
    out->status = s.status;
    out->skip_filter = s.skip_filter;
    out->skip_score = s.skip_score;
    out->total = (int32_t)(s.best_key >> 40);
  }
  return KSG_OK;
}

int ksg_reserve(ksg_ctx* ctx, uint32_t q, int32_t node) {
  rtx::Range rr("ksg_reserve");
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  if (!ctx->c.reserve(q, node)) return ctx->fail(ctx->c.err, KSG_E_STATE);
  return KSG_OK;
}

int ksg_unreserve(ksg_ctx* ctx, uint32_t q) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  ctx->c.out_gen++;
  ctx->c.room_ok = false;  // (room_ok: see Cluster::ensure_room)
  if (!ctx->c.unreserve(q)) return ctx->fail(ctx->c.err, KSG_E_STATE);
  return KSG_OK;
}

int ksg_apply_events(ksg_ctx* ctx, const char* events_json, size_t len) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  ctx->c.out_gen++;
  ctx->c.room_ok = false;  // (room_ok: see Cluster::ensure_room)
  if (!ctx || !events_json) return KSG_E_INVALID;
  try {
    if (!ctx->c.apply_events(events_json, len)) return ctx->fail(ctx->c.err, KSG_E_STATE);
  } catch (std::exception& e) {
    return ctx->fail(e.what(), KSG_E_INVALID);
  }
  return KSG_OK;
}

int ksg_node_requested(ksg_ctx* ctx, int64_t* requested, int32_t* pod_count, uint32_t n_res, uint32_t n) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  std::vector<int64_t> r;
  std::vector<int32_t> pc;
  if (!ctx->c.eng->read_requested(r, pc, ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_DEVICE);
  uint32_t N = (uint32_t)pc.size(), R = N ? (uint32_t)(r.size() / N) : 0;
  if (n < N || n_res < R) return KSG_E_NOBUF;
  for (uint32_t k = 0; k < R; ++k)
    for (uint32_t i = 0; i < N; ++i) requested[(size_t)k * n + i] = r[(size_t)k * N + i];
  for (uint32_t i = 0; i < N; ++i) pod_count[i] = pc[i];
  return KSG_OK;
}

// ---- the Go plugin's per-extension-point calls
static int put_str(ksg_ctx* ctx, const std::string& s, char* buf, size_t cap, size_t* len) {
  (void)ctx;
  if (len) *len = s.size();
  if (!buf) return cap ? KSG_E_INVALID : KSG_OK;
  if (cap < s.size()) return KSG_E_NOBUF;
  std::memcpy(buf, s.data(), s.size());
  return KSG_OK;
}

int ksg_queue_pod(const ksg_ctx* ctx, uint32_t q, char* buf, size_t cap, size_t* len) {
  KSG_LOCK(ctx);
  if (!ctx) return KSG_E_INVALID;
  if (q >= ctx->c.queue.size()) return KSG_E_RANGE;
  return put_str(nullptr, ctx->c.queue[q].ns + "/" + ctx->c.queue[q].name, buf, cap, len);
}

int ksg_gated_pods(const ksg_ctx* ctx, char* buf, size_t cap, size_t* len) {
  KSG_LOCK(ctx);
  if (!ctx) return KSG_E_INVALID;
  std::string s;
  for (auto& p : ctx->c.gated) s += p.ns + "/" + p.name + "\n";
  return put_str(nullptr, s, buf, cap, len);
}

int ksg_plugin_position(const ksg_ctx* ctx, const char* name, size_t len) {
  KSG_LOCK(ctx);
  if (!ctx || !name) return KSG_E_INVALID;
  const std::string nm = ksg::host::unwrapped(std::string(name, len));
  for (int i = 0; i < ctx->c.n_plugins; ++i)
    if (ctx->c.names[i] == nm) return i;
  return KSG_E_RANGE;
}

int ksg_plugin_weights(const ksg_ctx* ctx, uint32_t pos, int64_t* weight, int64_t* store_weight) {
  KSG_LOCK(ctx);
  if (!ctx) return KSG_E_INVALID;
  if ((int)pos >= ctx->c.n_plugins) return KSG_E_RANGE;
  if (weight) *weight = ctx->c.fw_w[pos];
  if (store_weight) *store_weight = ctx->c.store_w[pos];
  return KSG_OK;
}

int ksg_node_index(const ksg_ctx* ctx, const char* name, size_t len) {
  KSG_LOCK(ctx);
  if (!ctx || !name) return KSG_E_INVALID;
  const int32_t g = ctx->c.node_names.get(std::string(name, len));
  return g < 0 ? KSG_E_RANGE : g;
}

int ksg_prefilter_status(ksg_ctx* ctx, uint32_t q, uint32_t pos, int32_t* code, char* msg, size_t cap, size_t* len) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  Cluster& c = ctx->c;
  if (!code || q >= c.meta.size() || (int)pos >= c.n_plugins) return ctx->fail("prefilter_status: range", KSG_E_RANGE);
  const ksg::PodOutputs* o = c.outputs_of(q);
  if (!o) return ctx->fail(c.err, KSG_E_STATE);
  std::string m;
  *code = c.prefilter_status(q, (int)pos, o->summary, m);
  return put_str(ctx, m, msg, cap, len);
}

int ksg_prefilter_result(ksg_ctx* ctx, uint32_t q, char* buf, size_t cap, size_t* len) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  Cluster& c = ctx->c;
  if (q >= c.meta.size()) return ctx->fail("prefilter_result: range", KSG_E_RANGE);
  std::string s = "null";  // PreFilterResult nil: every node
  if (c.meta[q].restricted) {
    s = "[";
    for (size_t i = 0; i < c.meta[q].prefilter_names.size(); ++i) {
      if (i) s += ',';
      Cluster::jstr(s, c.meta[q].prefilter_names[i]);
    }
    s += "]";
  }
  return put_str(ctx, s, buf, cap, len);
}

int ksg_prefilter_result_pos(ksg_ctx* ctx, uint32_t q, uint32_t pos, char* buf, size_t cap, size_t* len) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  Cluster& c = ctx->c;
  if (q >= c.meta.size() || (int)pos >= c.n_plugins) return ctx->fail("prefilter_result_pos: range", KSG_E_RANGE);
  const ksg::host::PodMeta& m = c.meta[q];
  const std::vector<std::string>* names = nullptr;  // PreFilterResult nil: every node
  if (c.plugins[pos] == ksg::host::P_NA && m.restricted) names = &m.prefilter_names;
  if (c.vkind[pos] == ksg::host::VK_BIND && m.vb_restricted) names = &m.vb_names;
  std::string s = "null";
  if (names) {
    s = "[";
    for (size_t i = 0; i < names->size(); ++i) {
      if (i) s += ',';
      Cluster::jstr(s, (*names)[i]);
    }
    s += "]";
  }
  return put_str(ctx, s, buf, cap, len);
}

int ksg_postfilter_result(ksg_ctx* ctx, uint32_t q, int32_t* nominated, char* buf, size_t cap, size_t* len) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  Cluster& c = ctx->c;
  if (!nominated || q >= c.queue.size()) return ctx->fail("postfilter_result: range", KSG_E_RANGE);
  *nominated = -1;
  std::string s;
  if (q < c.nom.size()) {
    *nominated = c.nom[q].node;
    for (auto& v : c.nom[q].victims) s += v + "\n";
  }
  return put_str(ctx, s, buf, cap, len);
}

int ksg_filter_status(ksg_ctx* ctx, uint32_t q, uint32_t pos, uint32_t node, int32_t* code, char* msg, size_t cap,
                      size_t* len) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  Cluster& c = ctx->c;
  if (!code || q >= c.meta.size() || (int)pos >= c.n_plugins) return ctx->fail("filter_status: range", KSG_E_RANGE);
  if (node < c.lo || node >= c.hi) return ctx->fail("filter_status: node outside this context's nodes", KSG_E_RANGE);
  const ksg::PodOutputs* o = c.outputs_of(q);
  if (!o) return ctx->fail(c.err, KSG_E_STATE);
  std::string m;
  *code = c.filter_status(q, (int)pos, node - c.lo, *o, m);
  return put_str(ctx, m, msg, cap, len);
}

int ksg_prescore_status(ksg_ctx* ctx, uint32_t q, uint32_t pos, int32_t* code, char* msg, size_t cap, size_t* len) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  Cluster& c = ctx->c;
  if (!code || q >= c.meta.size() || (int)pos >= c.n_plugins) return ctx->fail("prescore_status: range", KSG_E_RANGE);
  const ksg::PodOutputs* o = c.outputs_of(q);
  if (!o) return ctx->fail(c.err, KSG_E_STATE);
  std::string m;
  *code = c.prescore_status(q, (int)pos, o->summary, m);
  return put_str(ctx, m, msg, cap, len);
}

int ksg_normalized_scores(ksg_ctx* ctx, uint32_t q, uint32_t pos, int64_t* out, uint32_t n) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  Cluster& c = ctx->c;
  if (!out || q >= c.meta.size()) return ctx->fail("normalized_scores: range", KSG_E_RANGE);
  if ((int)pos >= c.n_plugins || c.dpos[pos] < 0) return ctx->fail("no device scores at this position", KSG_E_INVALID);
  const std::vector<int32_t>* nm = c.normalized_of(q);
  if (!nm) return ctx->fail(c.err, KSG_E_STATE);
  const uint32_t N = c.hi - c.lo;
  if (n < N) return KSG_E_NOBUF;
  const size_t d = (size_t)c.dpos[pos];
  for (uint32_t i = 0; i < N; ++i) out[i] = (*nm)[d * N + i];
  return KSG_OK;
}

// ---- ksg_cycle_view: one cycle's per-node results as immutable arrays (the
// Filter / Score / NormalizeScore calls of the framework's parallel workers read
// them without calling into the library).  The device fills the per-node arrays
// into a pinned block (Engine::view: one kernel, one copy); the host adds the
// pod-level statuses and renders one message per distinct failing code.
namespace {
struct CycleView {
  ksg_cycle_view pub;  // (first member: the pointer handed out)
  uint8_t* block = nullptr;  // pinned (Engine::pinned_get)
  size_t cap = 0;
  std::vector<int8_t> fpos_h, fcode_h;  // host-built arrays (slot-table overflow)
  std::vector<uint16_t> fmsg_h;
  std::vector<uint8_t> called;
  std::vector<int8_t> pfcode, pscode;
  std::vector<uint16_t> pfmsg, psmsg;
  std::vector<const void*> sptr, nptr;
  std::vector<uint8_t> sbytes, nbytes;
  std::vector<std::string> msgs;
  std::vector<const char*> mptr;
  std::unordered_map<std::string, uint16_t> mid;
  uint16_t intern(const std::string& m) {
    if (m.empty()) return 0;
    auto it = mid.find(m);
    if (it != mid.end()) return it->second;
    if (msgs.size() >= 0xFFFF) return 0;  // (never: a cycle has a few dozen distinct messages)
    const uint16_t k = (uint16_t)msgs.size();
    msgs.push_back(m);
    mid.emplace(m, k);
    return k;
  }
  ~CycleView() { ksg::Engine::pinned_put(block, cap); }
};
}  // namespace

int ksg_cycle_view_acquire(ksg_ctx* ctx, uint32_t q, const ksg_cycle_view** out) {
  rtx::Range rr("ksg_cycle_view_acquire");
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  Cluster& c = ctx->c;
  if (!out) return KSG_E_INVALID;
  *out = nullptr;
  if (q >= c.meta.size()) return ctx->fail("cycle_view: range", KSG_E_RANGE);
  ksg::Engine::ViewLayout lay;
  c.eng->view_layout(lay);
  std::unique_ptr<CycleView> v(new CycleView());
  auto& pv = c.pview;
  if (pv.block && pv.q == (int64_t)q && pv.gen == c.out_gen && pv.lay.bytes == lay.bytes && pv.lay.N == lay.N &&
      pv.lay.n_raw == lay.n_raw) {  // filled by q's own cycle
    lay = pv.lay;
    v->block = pv.block;
    v->cap = pv.cap;
    pv.block = nullptr;
    pv.drop();
  } else {
    v->block = ksg::Engine::pinned_get(lay.bytes, v->cap);
    if (!v->block) return ctx->fail("cycle_view: no host memory", KSG_E_DEVICE);
    if (!c.eng->view(q, c.view_cfg(), lay, v->block, c.err)) return ctx->fail(c.err, KSG_E_STATE);
  }
  const uint32_t P = (uint32_t)c.n_plugins, N = c.hi - c.lo;
  v->msgs.resize(lay.n_slots + 1);  // messages[s + 1]: the message of slot s's code
  const uint64_t* slots = reinterpret_cast<const uint64_t*>(v->block);
  const bool overflow = (uint32_t)(slots[lay.n_slots] >> 32) == lay.gen;
  ksg_pod_summary S;
  std::memcpy(&S, v->block + lay.off_sum, sizeof(S));
  const int8_t* fail_pos = reinterpret_cast<const int8_t*>(v->block + lay.off_fail_pos);
  const int8_t* fail_code = reinterpret_cast<const int8_t*>(v->block + lay.off_fail_code);
  const uint16_t* fail_msg = reinterpret_cast<const uint16_t*>(v->block + lay.off_fail_msg);
  if (!overflow) {
    for (uint32_t k = 0; k < lay.n_slots; ++k)
      if ((uint32_t)(slots[k] >> 32) == lay.gen) {
        const uint32_t code = (uint32_t)slots[k];
        v->msgs[k + 1] = c.filter_message(c.code_pos(code), c.code_detail(code));
      }
  } else {  // more distinct failing codes than slots (never seen): the per-node calls' answers
    const ksg::PodOutputs* o = c.outputs_of(q);
    if (!o) return ctx->fail(c.err, KSG_E_STATE);
    v->fpos_h.assign(N, -1);
    v->fcode_h.assign(N, 0);
    v->fmsg_h.assign(N, 0);
    std::string m;
    for (uint32_t i = 0; i < N; ++i) {
      const uint32_t code = o->filter[i];
      if (code == KSG_FILTER_NOT_EVALUATED) continue;
      if (code == KSG_FILTER_PASS) { v->fpos_h[i] = (int8_t)P; continue; }
      const int fp = c.code_pos(code);
      v->fpos_h[i] = (int8_t)fp;
      const uint32_t d = c.code_detail(code);
      m = c.filter_message(fp, d);
      v->fcode_h[i] = (int8_t)c.filter_fail_code(q, fp, i, d);
      v->fmsg_h[i] = v->intern(m);
    }
    fail_pos = v->fpos_h.data();
    fail_code = v->fcode_h.data();
    fail_msg = v->fmsg_h.data();
  }
  v->called.assign(P, 0);
  v->pfcode.assign(P, -1);
  v->pfmsg.assign(P, 0);
  v->pscode.assign(P, -1);
  v->psmsg.assign(P, 0);
  v->sptr.assign(P, nullptr);
  v->nptr.assign(P, nullptr);
  v->sbytes.assign(P, 4);
  v->nbytes.assign(P, 4);
  ksg::Engine::ViewRows rows;
  std::memcpy(&rows, v->block + lay.off_rows, sizeof(rows));
  std::string m;
  const ksg::host::PodMeta& pm = c.meta[q];
  const uint32_t skip_f = c.skip_filter_mask(pm, S);
  for (uint32_t pos = 0; pos < P; ++pos) {
    v->pfcode[pos] = (int8_t)c.prefilter_status(q, (int)pos, S, m);
    v->pfmsg[pos] = v->intern(m);
    v->pscode[pos] = (int8_t)c.prescore_status(q, (int)pos, S, m);
    v->psmsg[pos] = v->intern(m);
    v->called[pos] = ksg::host::has_filter(c.plugins[pos]) && pm.prefilter_fail_pos < 0 &&
                     !c.filter_skipped(pm, skip_f, (int)pos) ? 1 : 0;
    const int d = c.dpos[pos];
    if (d < 0 || !rows.bytes[d]) continue;
    v->sptr[pos] = v->block + rows.off[d];
    v->sbytes[pos] = rows.bytes[d];
    const int r = lay.norm_row[d];
    v->nptr[pos] = r >= 0 ? (const void*)(v->block + rows.off[KSG_MAX_PLUGINS + r]) : v->sptr[pos];
    v->nbytes[pos] = r >= 0 ? rows.bytes[KSG_MAX_PLUGINS + r] : v->sbytes[pos];
  }
  for (auto& x : v->msgs) v->mptr.push_back(x.c_str());
  ksg_cycle_view& p = v->pub;
  p.q = q;
  p.n_positions = P;
  p.node_offset = c.lo;
  p.n_nodes = N;
  p.result.selected = S.selected;
  p.result.feasible = S.feasible;
  p.result.status = S.status;
  p.result.skip_filter = S.skip_filter;
  p.result.skip_score = S.skip_score;
  p.result.total = (int32_t)(S.best_key >> 40);
  p.filter_called = v->called.data();
  p.fail_pos = fail_pos;
  p.fail_code = fail_code;
  p.fail_msg = fail_msg;
  p.score = v->sptr.data();
  p.normalized = v->nptr.data();
  p.score_bytes = v->sbytes.data();
  p.normalized_bytes = v->nbytes.data();
  p.prefilter_code = v->pfcode.data();
  p.prefilter_msg = v->pfmsg.data();
  p.prescore_code = v->pscode.data();
  p.prescore_msg = v->psmsg.data();
  p.messages = v->mptr.data();
  p.n_messages = (uint32_t)v->mptr.size();
  p.owner = v.get();
  *out = &v.release()->pub;
  return KSG_OK;
}

void ksg_cycle_view_release(const ksg_cycle_view* v) {
  if (v) delete static_cast<const CycleView*>(v->owner);
}

int ksg_node_nonzero(ksg_ctx* ctx, int64_t* nonzero, uint32_t n) {
  KSG_LOCK(ctx);
  KSG_GUARD(ctx);
  if (!nonzero) return KSG_E_INVALID;
  std::vector<int64_t> nz;
  if (!ctx->c.eng->read_nonzero(nz, ctx->c.err)) return ctx->fail(ctx->c.err, KSG_E_DEVICE);
  const uint32_t N = (uint32_t)(nz.size() / 2);
  if (n < N) return KSG_E_NOBUF;
  for (uint32_t i = 0; i < N; ++i) {
    nonzero[i] = nz[i];
    nonzero[(size_t)n + i] = nz[(size_t)N + i];
  }
  return KSG_OK;
}

}  // extern "C"
