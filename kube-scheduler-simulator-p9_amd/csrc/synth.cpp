// Synthetic clusters of BASELINE.json configs 2-5, native twin
// of ksg/generator.py: the same splitmix64 stream, the same draws in the same
// order, the same Kubernetes-shaped JSON document
//   {"profile": {...}, "nodes": [Node...], "pods": [bound Pod...], "queue": [Pod...]}
// (tests/test_synth.py checks json.loads(native) == the Python document).  Harness
// mode only: the benchmarks and the full-size parity tests build 50,000- and
// 1,000,000-node clusters with it in seconds instead of minutes of Python.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/ksg.h"

namespace ksg {
namespace synth {

using std::string;
using std::vector;
typedef long long i64;

static const uint64_t kGolden = 0x9E3779B97F4A7C15ull;
static const char* kHostname = "kubernetes.io/hostname";
static const char* kZone = "topology.kubernetes.io/zone";
static const i64 Mi = 1ll << 20, Gi = 1ll << 30;

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    s += kGolden;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t n) { return next() % n; }
  uint64_t pct() { return next() % 100; }
};

static uint64_t config_seed(int c) { return 20250131ull * 100 + (uint64_t)c; }

// ------------------------------------------------------------------ JSON writer
struct W {
  string o;
  void raw(const char* s) { o += s; }
  void raw(const string& s) { o += s; }
  void str(const string& s) {
    o += '"';
    for (char c : s) {
      if (c == '"' || c == '\\') o += '\\';
      o += c;
    }
    o += '"';
  }
  void key(const char* k) {
    str(k);
    o += ':';
  }
  void num(i64 v) { o += std::to_string(v); }
};

static string fmt(const char* f, i64 v) {
  char b[64];
  std::snprintf(b, sizeof b, f, v);
  return b;
}
static string cpu_q(i64 milli) { return milli % 1000 ? std::to_string(milli) + "m" : std::to_string(milli / 1000); }
static string mem_q(i64 b) { return b % Gi == 0 ? std::to_string(b / Gi) + "Gi" : std::to_string(b); }

typedef std::map<string, string> Labels;
struct Taint { string key, value, effect; };

// generator.node_obj (pods 110, allocatable == capacity)
static void node_obj(W& w, const string& name, i64 cpu, i64 mem, const vector<std::pair<string, string>>& labels,
                     const vector<Taint>& taints) {
  w.raw("{\"metadata\":{\"name\":");
  w.str(name);
  w.raw(",\"labels\":{");
  w.key(kHostname);
  w.str(name);
  for (auto& kv : labels) {
    w.raw(",");
    w.key(kv.first.c_str());
    w.str(kv.second);
  }
  w.raw("}},\"spec\":{");
  if (!taints.empty()) {
    w.raw("\"taints\":[");
    for (size_t i = 0; i < taints.size(); ++i) {
      if (i) w.raw(",");
      w.raw("{\"key\":");
      w.str(taints[i].key);
      w.raw(",\"value\":");
      w.str(taints[i].value);
      w.raw(",\"effect\":");
      w.str(taints[i].effect);
      w.raw("}");
    }
    w.raw("]");
  }
  string alloc = "{\"cpu\":\"" + cpu_q(cpu) + "\",\"memory\":\"" + mem_q(mem) + "\",\"pods\":\"110\"}";
  w.raw("},\"status\":{\"allocatable\":");
  w.raw(alloc);
  w.raw(",\"capacity\":");
  w.raw(alloc);
  w.raw("}}");
}

// generator.req: {"requests": {...}} or {} (cpu < 0 / mem < 0: not requested)
static string req(i64 cpu_milli, i64 mem) {
  string r;
  if (cpu_milli >= 0) r += "\"cpu\":\"" + std::to_string(cpu_milli) + "m\"";
  if (mem >= 0) {
    if (!r.empty()) r += ",";
    r += "\"memory\":\"" + (mem % Mi == 0 ? std::to_string(mem / Mi) + "Mi" : std::to_string(mem)) + "\"";
  }
  return r.empty() ? "{}" : "{\"requests\":{" + r + "}}";
}

// generator.pod_obj: containers = resources objects; extra = pre-rendered spec members
static void pod_obj(W& w, const string& name, const vector<string>& containers, const Labels& labels,
                    const string& node, const string& extra) {
  w.raw("{\"metadata\":{\"name\":");
  w.str(name);
  w.raw(",\"namespace\":\"default\",\"labels\":{");
  bool first = true;
  for (auto& kv : labels) {
    if (!first) w.raw(",");
    first = false;
    w.key(kv.first.c_str());
    w.str(kv.second);
  }
  w.raw("}},\"spec\":{\"containers\":[");
  for (size_t i = 0; i < containers.size(); ++i) {
    if (i) w.raw(",");
    w.raw("{\"name\":\"c" + std::to_string(i) + "\",\"image\":\"registry.k8s.io/pause:3.5\",\"resources\":");
    w.raw(containers[i]);
    w.raw("}");
  }
  w.raw("]");
  if (!node.empty()) {
    w.raw(",\"nodeName\":");
    w.str(node);
  }
  if (!extra.empty()) {
    w.raw(",");
    w.raw(extra);
  }
  w.raw("}}");
}

// generator.make_profile with DEFAULT_ARGS
static void profile(W& w, const vector<std::pair<string, int>>& plugins, uint64_t seed) {
  w.raw("{\"plugins\":[");
  for (size_t i = 0; i < plugins.size(); ++i) {
    if (i) w.raw(",");
    w.str(plugins[i].first);
  }
  w.raw("]");
  for (const char* m : {"weights", "storeWeights"}) {
    w.raw(",\"");
    w.raw(m);
    w.raw("\":{");
    for (size_t i = 0; i < plugins.size(); ++i) {
      if (i) w.raw(",");
      w.key(plugins[i].first.c_str());
      w.num(plugins[i].second);
    }
    w.raw("}");
  }
  w.raw(",\"pluginConfig\":{\"NodeResourcesFit\":{\"scoringStrategy\":{\"type\":\"LeastAllocated\",\"resources\":"
        "[{\"name\":\"cpu\",\"weight\":1},{\"name\":\"memory\",\"weight\":1}]}},"
        "\"NodeResourcesBalancedAllocation\":{\"resources\":[{\"name\":\"cpu\",\"weight\":1},{\"name\":\"memory\","
        "\"weight\":1}]},\"InterPodAffinity\":{\"hardPodAffinityWeight\":1,\"ignorePreferredTermsOfExistingPods\":"
        "false},\"PodTopologySpread\":{\"defaultingType\":\"System\"}},\"seed\":");
  w.raw(std::to_string(seed));
  w.raw("}");
}

static const i64 kShapes[4][2] = {{8000, 32 * Gi}, {16000, 64 * Gi}, {32000, 128 * Gi}, {64000, 256 * Gi}};

// ------------------------------------------------------------------ cfg2
static string gen_cfg2(i64 n_nodes, i64 n_pods, uint64_t seed) {
  Rng r(seed);
  W nodes, pods, queue;
  bool first_pod = true;
  for (i64 i = 0; i < n_nodes; ++i) {
    const i64* sh = kShapes[r.below(4)];
    string name = fmt("node-%07lld", i);
    if (i) nodes.raw(",");
    node_obj(nodes, name, sh[0], sh[1], {}, {});
    i64 uc = (i64)r.below(51), um = (i64)r.below(51);
    if (uc || um) {
      if (!first_pod) pods.raw(",");
      first_pod = false;
      pod_obj(pods, fmt("fill-%07lld", i), {req(sh[0] * uc / 100, sh[1] * um / 100)}, {{"role", "filler"}}, name, "");
    }
  }
  for (i64 j = 0; j < n_pods; ++j) {
    if (j) queue.raw(",");
    string name = fmt("pod-%07lld", j);
    vector<string> cs;
    if (r.pct() < 10) {
      cs.push_back("{}");
    } else {
      i64 c = 50 * (1 + (i64)r.below(40)), m = 64 * Mi * (1 + (i64)r.below(64));
      cs.push_back(req(c, m));
      if (r.pct() < 5) {
        i64 c2 = 50 * (1 + (i64)r.below(40)), m2 = 64 * Mi * (1 + (i64)r.below(64));
        cs.push_back(req(c2, m2));
      }
    }
    pod_obj(queue, name, cs, {}, "", "");
  }
  W d;
  d.raw("{\"profile\":");
  profile(d, {{"NodeResourcesFit", 1}, {"NodeResourcesBalancedAllocation", 1}}, seed);
  d.raw(",\"nodes\":[" + nodes.o + "],\"pods\":[" + pods.o + "],\"queue\":[" + queue.o + "]}");
  return d.o;
}

// ------------------------------------------------------------------ cfg3 / cfg5
static const char* kEffects(int t) { return t < 12 ? "NoSchedule" : t < 24 ? "PreferNoSchedule" : "NoExecute"; }
static Taint cfg3_taint(int t) { return {fmt("taint-%02lld", t), fmt("v%lld", t % 3), kEffects(t)}; }
struct LabelKey { string key; vector<string> vals; };
static const vector<LabelKey>& cfg3_labels() {
  static vector<LabelKey> L;
  if (L.empty()) {
    LabelKey z{kZone, {}}, it{"node.kubernetes.io/instance-type", {}}, ar{"kubernetes.io/arch", {"amd64", "arm64"}},
        ti{"tier", {"a", "b", "c"}}, ge{"gen", {}};
    for (int i = 0; i < 20; ++i) z.vals.push_back(fmt("zone-%02lld", i));
    for (int i = 0; i < 16; ++i) it.vals.push_back(fmt("it-%02lld", i));
    for (int i = 1; i <= 8; ++i) ge.vals.push_back(std::to_string(i));
    L = {z, it, ar, ti, ge};
  }
  return L;
}
static const LabelKey& cfg3_key(const string& k) {
  for (auto& x : cfg3_labels())
    if (x.key == k) return x;
  return cfg3_labels()[0];
}

struct Node3 {
  Labels labels;  // without the hostname
  vector<Taint> taints;
};
struct Expr { string key, op; vector<string> vals; };
struct Tol { string key, op, value, effect; bool has_op = false, has_value = false, has_effect = false; };
struct Pod3 {
  bool best_effort = false;
  i64 cpu = 0, mem = 0;
  vector<Tol> tols;
  bool has_req = false;
  vector<vector<Expr>> terms;
  bool has_sel = false;
  string sel_key, sel_val;
  bool has_pref = false;
  vector<std::pair<i64, Expr>> pref;
};

static Expr cfg3_req_expr(Rng& r) {
  const auto& L = cfg3_labels();
  uint64_t kind = r.below(4);
  if (kind == 0 || kind == 1) {
    const LabelKey& k = L[r.next() % L.size()];
    uint64_t n = 1 + r.below(kind == 0 ? 3 : 2);
    std::set<string> vs;
    for (uint64_t i = 0; i < n; ++i) vs.insert(k.vals[r.next() % k.vals.size()]);
    return {k.key, kind == 0 ? "In" : "NotIn", vector<string>(vs.begin(), vs.end())};
  }
  if (kind == 2) return {fmt("feat-%02lld", (i64)r.below(48)), "Exists", {}};
  return {"gen", "Gt", {std::to_string(1 + r.below(6))}};
}

static Pod3 cfg3_pod(Rng& r) {
  Pod3 p;
  uint64_t pc = r.pct();
  if (pc < 10) {
    p.best_effort = true;
  } else {
    p.cpu = 50 * (1 + (i64)r.below(40));
    p.mem = 64 * Mi * (1 + (i64)r.below(64));
  }
  uint64_t nt = r.below(5);
  for (uint64_t i = 0; i < nt; ++i) {
    Taint t = cfg3_taint((int)r.below(32));
    Tol tol;
    tol.key = t.key;
    tol.has_op = true;
    if (r.pct() < 70) {
      tol.op = "Equal";
      tol.value = t.value;
      tol.has_value = true;
    } else {
      tol.op = "Exists";
    }
    if (r.pct() >= 20) {
      tol.effect = t.effect;
      tol.has_effect = true;
    }
    p.tols.push_back(tol);
  }
  if (r.pct() < 50) {
    p.has_req = true;
    uint64_t n = 1 + r.below(2);
    for (uint64_t i = 0; i < n; ++i) {
      vector<Expr> t;
      uint64_t m = 1 + r.below(3);
      for (uint64_t j = 0; j < m; ++j) t.push_back(cfg3_req_expr(r));
      p.terms.push_back(t);
    }
  }
  if (r.pct() < 20) {
    static const char* keys[3] = {"tier", "kubernetes.io/arch", kZone};
    p.has_sel = true;
    p.sel_key = keys[r.next() % 3];
    const LabelKey& k = cfg3_key(p.sel_key);
    p.sel_val = k.vals[r.next() % k.vals.size()];
  }
  if (r.pct() < 60) {
    p.has_pref = true;
    uint64_t n = 1 + r.below(4);
    for (uint64_t i = 0; i < n; ++i) {
      i64 wgt = 1 + (i64)r.below(100);
      p.pref.push_back({wgt, cfg3_req_expr(r)});
    }
  }
  return p;
}

static bool tolerates(const vector<Tol>& tols, const Taint& t) {
  for (auto& x : tols) {
    if (x.has_effect && !x.effect.empty() && x.effect != t.effect) continue;
    if (!x.key.empty() && x.key != t.key) continue;
    if ((x.op.empty() || x.op == "Equal") && (x.has_value ? x.value : string()) == t.value) return true;
    if (x.op == "Exists") return true;
  }
  return false;
}
static bool expr_ok(const Expr& e, const string& name, const Node3& n) {
  auto it = n.labels.find(e.key);
  bool has = it != n.labels.end() || e.key == kHostname;
  string v = e.key == kHostname ? name : (it != n.labels.end() ? it->second : string());
  if (e.op == "In") return has && std::find(e.vals.begin(), e.vals.end(), v) != e.vals.end();
  if (e.op == "NotIn") return !has || std::find(e.vals.begin(), e.vals.end(), v) == e.vals.end();
  if (e.op == "Exists") return has;
  if (e.op == "DoesNotExist") return !has;
  if (e.op == "Gt" || e.op == "Lt") {
    if (!has || e.vals.empty()) return false;
    char* end = nullptr;
    long long a = std::strtoll(v.c_str(), &end, 10);
    if (v.empty() || *end) return false;
    long long b = std::strtoll(e.vals[0].c_str(), &end, 10);
    if (e.vals[0].empty() || *end) return false;
    return e.op == "Gt" ? a > b : a < b;
  }
  return false;
}
// generator._cfg3_feasible_somewhere (a cheap screen, not the oracle)
static bool feasible_somewhere(const Pod3& p, const vector<Node3>& nodes) {
  for (size_t i = 0; i < nodes.size(); ++i) {
    const Node3& n = nodes[i];
    bool bad = false;
    for (auto& t : n.taints)
      if ((t.effect == "NoSchedule" || t.effect == "NoExecute") && !tolerates(p.tols, t)) { bad = true; break; }
    if (bad) continue;
    string name = fmt("node-%07lld", (i64)i);
    if (p.has_sel) {
      auto it = n.labels.find(p.sel_key);
      if (it == n.labels.end() || it->second != p.sel_val) continue;
    }
    if (p.has_req) {
      bool any = false;
      for (auto& t : p.terms) {
        bool all = true;
        for (auto& e : t) all = all && expr_ok(e, name, n);
        if (all) { any = true; break; }
      }
      if (!any) continue;
    }
    return true;
  }
  return false;
}

static string expr_json(const Expr& e) {
  W w;
  w.raw("{\"key\":");
  w.str(e.key);
  w.raw(",\"operator\":");
  w.str(e.op);
  if (e.op != "Exists" && e.op != "DoesNotExist") {
    w.raw(",\"values\":[");
    for (size_t i = 0; i < e.vals.size(); ++i) {
      if (i) w.raw(",");
      w.str(e.vals[i]);
    }
    w.raw("]");
  }
  w.raw("}");
  return w.o;
}

static string pod3_spec(const Pod3& p) {
  W w;
  bool any = false;
  auto sep = [&]() { if (any) w.raw(","); any = true; };
  if (!p.tols.empty()) {
    sep();
    w.raw("\"tolerations\":[");
    for (size_t i = 0; i < p.tols.size(); ++i) {
      const Tol& t = p.tols[i];
      if (i) w.raw(",");
      w.raw("{\"key\":");
      w.str(t.key);
      w.raw(",\"operator\":");
      w.str(t.op);
      if (t.has_value) { w.raw(",\"value\":"); w.str(t.value); }
      if (t.has_effect) { w.raw(",\"effect\":"); w.str(t.effect); }
      w.raw("}");
    }
    w.raw("]");
  }
  if (p.has_sel) {
    sep();
    w.raw("\"nodeSelector\":{");
    w.key(p.sel_key.c_str());
    w.str(p.sel_val);
    w.raw("}");
  }
  if (p.has_req || p.has_pref) {
    sep();
    w.raw("\"affinity\":{\"nodeAffinity\":{");
    if (p.has_req) {
      w.raw("\"requiredDuringSchedulingIgnoredDuringExecution\":{\"nodeSelectorTerms\":[");
      for (size_t i = 0; i < p.terms.size(); ++i) {
        if (i) w.raw(",");
        w.raw("{\"matchExpressions\":[");
        for (size_t j = 0; j < p.terms[i].size(); ++j) {
          if (j) w.raw(",");
          w.raw(expr_json(p.terms[i][j]));
        }
        w.raw("]}");
      }
      w.raw("]}");
    }
    if (p.has_pref) {
      if (p.has_req) w.raw(",");
      w.raw("\"preferredDuringSchedulingIgnoredDuringExecution\":[");
      for (size_t i = 0; i < p.pref.size(); ++i) {
        if (i) w.raw(",");
        w.raw("{\"weight\":" + std::to_string(p.pref[i].first) + ",\"preference\":{\"matchExpressions\":[" +
              expr_json(p.pref[i].second) + "]}}");
      }
      w.raw("]");
    }
    w.raw("}}");
  }
  return w.o;
}

static string gen_cfg3(i64 n_nodes, i64 n_pods, uint64_t seed, bool feasible_check) {
  Rng r(seed);
  const auto& L = cfg3_labels();
  vector<Node3> nodes((size_t)n_nodes);
  W nw;
  for (i64 i = 0; i < n_nodes; ++i) {
    Node3& n = nodes[(size_t)i];
    string name = fmt("node-%07lld", i);
    const i64* sh = kShapes[r.below(4)];
    vector<std::pair<string, string>> lab;
    for (auto& k : L) {
      const string& v = k.vals[r.next() % k.vals.size()];
      n.labels[k.key] = v;
      lab.push_back({k.key, v});
    }
    for (int f = 0; f < 48; ++f)
      if (r.below(4) == 0) {
        string k = fmt("feat-%02lld", f);
        n.labels[k] = "true";
        lab.push_back({k, "true"});
      }
    uint64_t p = r.pct();
    uint64_t nt = p < 40 ? 0 : p < 70 ? 1 : p < 90 ? 2 : 3 + r.below(2);
    std::set<int> seen;
    for (uint64_t k = 0; k < nt; ++k) {
      int t = (int)r.below(32);
      if (seen.insert(t).second) n.taints.push_back(cfg3_taint(t));
    }
    if (i) nw.raw(",");
    node_obj(nw, name, sh[0], sh[1], lab, n.taints);
  }
  W qw;
  for (i64 j = 0; j < n_pods; ++j) {
    Pod3 p;
    for (int attempt = 0; attempt < 64; ++attempt) {
      p = cfg3_pod(r);
      if (!feasible_check || feasible_somewhere(p, nodes)) break;
    }
    if (j) qw.raw(",");
    pod_obj(qw, fmt("pod-%07lld", j), {p.best_effort ? string("{}") : req(p.cpu, p.mem)}, {}, "", pod3_spec(p));
  }
  W d;
  d.raw("{\"profile\":");
  profile(d, {{"TaintToleration", 3}, {"NodeAffinity", 2}, {"NodeResourcesFit", 1}, {"NodeResourcesBalancedAllocation", 1}},
          seed);
  d.raw(",\"nodes\":[" + nw.o + "],\"pods\":[],\"queue\":[" + qw.o + "]}");
  return d.o;
}

// ------------------------------------------------------------------ cfg4
static string sel_json(const char* k, const string& v) { return "{\"matchLabels\":{\"" + string(k) + "\":\"" + v + "\"}}"; }
static string term_json(const char* k, const string& v, const char* topo) {
  return "{\"labelSelector\":" + sel_json(k, v) + ",\"topologyKey\":\"" + topo + "\"}";
}

static string gen_cfg4(i64 n_nodes, i64 n_existing, i64 n_pods, i64 n_zones, uint64_t seed) {
  Rng r(seed);
  W nw;
  for (i64 i = 0; i < n_nodes; ++i) {
    if (i) nw.raw(",");
    node_obj(nw, fmt("node-%07lld", i), 32000, 128 * Gi, {{kZone, fmt("zone-%02lld", (i * n_zones) / n_nodes)}}, {});
  }
  W pw;
  for (i64 e = 0; e < n_existing; ++e) {
    string app = fmt("app-%03lld", (i64)r.below(200)), team = fmt("team-%lld", (i64)r.below(10));
    string node = fmt("node-%07lld", (i64)r.below((uint64_t)n_nodes));
    uint64_t p = r.pct();
    string aff;
    if (p < 5) {
      aff = "\"podAntiAffinity\":{\"requiredDuringSchedulingIgnoredDuringExecution\":[" + term_json("app", app, kHostname) + "]}";
    } else if (p < 15) {
      i64 wgt = 1 + (i64)r.below(100);
      aff = "\"podAffinity\":{\"preferredDuringSchedulingIgnoredDuringExecution\":[{\"weight\":" + std::to_string(wgt) +
            ",\"podAffinityTerm\":" + term_json("team", team, kZone) + "}]}";
    } else if (p < 20) {
      aff = "\"podAffinity\":{\"requiredDuringSchedulingIgnoredDuringExecution\":[" + term_json("team", team, kZone) + "]}";
    }
    i64 c = 100 * (1 + (i64)r.below(5)), m = 128 * Mi * (1 + (i64)r.below(8));
    if (e) pw.raw(",");
    pod_obj(pw, fmt("ex-%07lld", e), {req(c, m)}, {{"app", app}, {"team", team}}, node,
            aff.empty() ? "" : "\"affinity\":{" + aff + "}");
  }
  W qw;
  for (i64 j = 0; j < n_pods; ++j) {
    string app = fmt("app-%03lld", (i64)r.below(200)), team = fmt("team-%lld", (i64)r.below(10));
    vector<string> tsc;
    if (r.pct() < 70) {
      i64 ms = 1 + (i64)r.below(3);
      tsc.push_back("{\"maxSkew\":" + std::to_string(ms) + ",\"topologyKey\":\"" + kZone +
                    "\",\"whenUnsatisfiable\":\"DoNotSchedule\",\"labelSelector\":" + sel_json("app", app) + "}");
    }
    if (r.pct() < 50) {
      i64 ms = 1 + (i64)r.below(5);
      tsc.push_back("{\"maxSkew\":" + std::to_string(ms) + ",\"topologyKey\":\"" + kHostname +
                    "\",\"whenUnsatisfiable\":\"ScheduleAnyway\",\"labelSelector\":" + sel_json("app", app) + "}");
    }
    string anti_req, aff_pref, anti_pref;
    if (r.pct() < 20) anti_req = "\"requiredDuringSchedulingIgnoredDuringExecution\":[" + term_json("app", app, kHostname) + "]";
    if (r.pct() < 20) {
      i64 wgt = 1 + (i64)r.below(100);
      aff_pref = "\"preferredDuringSchedulingIgnoredDuringExecution\":[{\"weight\":" + std::to_string(wgt) +
                 ",\"podAffinityTerm\":" + term_json("team", team, kZone) + "}]";
    }
    if (r.pct() < 10) {
      i64 wgt = 1 + (i64)r.below(100);
      anti_pref = "\"preferredDuringSchedulingIgnoredDuringExecution\":[{\"weight\":" + std::to_string(wgt) +
                  ",\"podAffinityTerm\":" + term_json("app", app, kZone) + "}]";
    }
    string spec;
    if (!tsc.empty()) {
      spec = "\"topologySpreadConstraints\":[";
      for (size_t i = 0; i < tsc.size(); ++i) spec += (i ? "," : "") + tsc[i];
      spec += "]";
    }
    string aff;
    if (!anti_req.empty() || !anti_pref.empty())
      aff = "\"podAntiAffinity\":{" + anti_req + (anti_req.empty() || anti_pref.empty() ? "" : ",") + anti_pref + "}";
    if (!aff_pref.empty()) aff += (aff.empty() ? "" : ",") + string("\"podAffinity\":{") + aff_pref + "}";
    if (!aff.empty()) spec += (spec.empty() ? "" : ",") + string("\"affinity\":{") + aff + "}";
    i64 c = 100 * (1 + (i64)r.below(10)), m = 128 * Mi * (1 + (i64)r.below(16));
    if (j) qw.raw(",");
    pod_obj(qw, fmt("pod-%07lld", j), {req(c, m)}, {{"app", app}, {"team", team}}, "", spec);
  }
  W d;
  d.raw("{\"profile\":");
  profile(d, {{"NodeResourcesFit", 1}, {"PodTopologySpread", 2}, {"InterPodAffinity", 2}, {"NodeResourcesBalancedAllocation", 1}},
          seed);
  d.raw(",\"nodes\":[" + nw.o + "],\"pods\":[" + pw.o + "],\"queue\":[" + qw.o + "]}");
  return d.o;
}

}  // namespace synth
}  // namespace ksg

extern "C" {

// params: n_nodes, n_pods, n_existing, n_zones (< 0: the config's default), seed (0: config seed)
int ksg_synth_cluster(int config, int64_t n_nodes, int64_t n_pods, int64_t n_existing, int64_t n_zones, uint64_t seed,
                      char** out, size_t* len) {
  using namespace ksg::synth;
  if (!out || !len) return KSG_E_INVALID;
  *out = nullptr;
  *len = 0;
  std::string s;
  try {
    const uint64_t sd = seed ? seed : config_seed(config);
    switch (config) {
      case 2: s = gen_cfg2(n_nodes < 0 ? 5000 : n_nodes, n_pods < 0 ? 10000 : n_pods, sd); break;
      case 3: s = gen_cfg3(n_nodes < 0 ? 15000 : n_nodes, n_pods < 0 ? 10000 : n_pods, sd, true); break;
      case 4:
        s = gen_cfg4(n_nodes < 0 ? 50000 : n_nodes, n_existing < 0 ? 200000 : n_existing, n_pods < 0 ? 10000 : n_pods,
                     n_zones < 0 ? 20 : n_zones, sd);
        break;
      case 5: s = gen_cfg3(n_nodes < 0 ? 1000000 : n_nodes, n_pods < 0 ? 4096 : n_pods, sd, false); break;
      default: return KSG_E_INVALID;
    }
  } catch (...) {
    return KSG_E_INVALID;
  }
  char* b = static_cast<char*>(std::malloc(s.size() + 1));
  if (!b) return KSG_E_INVALID;
  std::memcpy(b, s.data(), s.size());
  b[s.size()] = 0;
  *out = b;
  *len = s.size();
  return KSG_OK;
}

void ksg_free(void* p) { std::free(p); }

}  // extern "C"
