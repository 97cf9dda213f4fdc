// Fuzz driver for the host layer's JSON entry points (built with ASan/UBSan
// against stub_engine.cpp; tests/test_fuzz_host.py).  Each input file holds
// four sections separated by "\n\x1e\n": profile, cluster document, one pod,
// one event batch.  Every ABI call must either succeed or return an error
// code with a message; the sanitizers turn any memory or UB fault into a
// non-zero exit.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/ksg.h"

static std::vector<std::string> sections(const std::string& s) {
  std::vector<std::string> out;
  const std::string sep = "\n\x1e\n";
  size_t at = 0;
  for (;;) {
    size_t k = s.find(sep, at);
    out.push_back(s.substr(at, k == std::string::npos ? std::string::npos : k - at));
    if (k == std::string::npos) break;
    at = k + sep.size();
  }
  while (out.size() < 4) out.push_back("");
  return out;
}

static void exercise(ksg_ctx* c) {
  const int qn = ksg_queue_len(c), nn = ksg_num_nodes(c);
  if (qn > 0) {
    ksg_keep_outputs(c, 0, (uint32_t)qn);
    if (ksg_schedule_queue(c, 0, (uint32_t)qn) == KSG_OK) ksg_wait(c, nullptr);
    std::vector<ksg_pod_result> r((size_t)qn);
    ksg_pod_results(c, 0, (uint32_t)qn, r.data());
  }
  std::vector<char> buf(1 << 16);
  std::vector<uint32_t> codes((size_t)(nn > 0 ? nn : 1));
  std::vector<int32_t> sc((size_t)(nn > 0 ? nn : 1));
  std::vector<int64_t> ns((size_t)(nn > 0 ? nn : 1));
  for (int q = 0; q < qn && q < 3; ++q) {
    size_t len = 0;
    ksg_annotations(c, (uint32_t)q, buf.data(), buf.size(), &len);
    ksg_annotations(c, (uint32_t)q, nullptr, 0, &len);
    ksg_prefilter_result(c, (uint32_t)q, buf.data(), buf.size(), &len);
    int32_t nominated = -1;
    ksg_postfilter_result(c, (uint32_t)q, &nominated, buf.data(), buf.size(), &len);
    ksg_postfilter_result(c, (uint32_t)q, &nominated, nullptr, 0, &len);
    if (nn > 0) {
      ksg_filter_codes(c, (uint32_t)q, codes.data(), (uint32_t)nn);
      for (uint32_t pos = 0; pos < 24; ++pos) {
        int32_t code = 0;
        ksg_prefilter_status(c, (uint32_t)q, pos, &code, buf.data(), buf.size(), &len);
        ksg_filter_status(c, (uint32_t)q, pos, 0, &code, buf.data(), buf.size(), &len);
        ksg_prescore_status(c, (uint32_t)q, pos, &code, buf.data(), buf.size(), &len);
        ksg_scores(c, (uint32_t)q, pos, sc.data(), (uint32_t)nn);
        ksg_normalized_scores(c, (uint32_t)q, pos, ns.data(), (uint32_t)nn);
      }
    }
  }
  ksg_filter_codes(c, 1u << 30, codes.data(), 1);
  ksg_annotations(c, 1u << 30, buf.data(), buf.size(), nullptr);
  const char* names[] = {"NodeResourcesFit", "node-0000000", "", "nope"};
  for (const char* s : names) {
    ksg_plugin_position(c, s, std::string(s).size());
    ksg_node_index(c, s, std::string(s).size());
  }
}

static int run_one(const std::string& text) {
  auto sec = sections(text);
  ksg_ctx* c = nullptr;
  ksg_opts o{};
  o.shard_count = 1;
  if (ksg_create(sec[0].data(), sec[0].size(), &o, &c) != KSG_OK) return 0;
  if (ksg_load_cluster(c, sec[1].data(), sec[1].size()) == KSG_OK) {
    exercise(c);
    ksg_pod_result r{};
    if (!sec[2].empty() && ksg_cycle(c, sec[2].data(), sec[2].size(), 0, &r) == KSG_OK) {
      const uint32_t q = (uint32_t)ksg_queue_len(c) - 1;
      ksg_reserve(c, q, r.selected >= 0 ? r.selected : 0);
      ksg_unreserve(c, q);
      ksg_cycle(c, sec[2].data(), sec[2].size(), 1, &r);
      ksg_compact(c, (uint32_t)ksg_queue_len(c) / 2);
      ksg_compact(c, 1u << 30);
    }
    if (!sec[3].empty()) ksg_apply_events(c, sec[3].data(), sec[3].size());
    exercise(c);
    ksg_whatif(c, 0, (uint32_t)ksg_queue_len(c));
    ksg_reset(c);
    ksg_apply_events(c, "{\"events\":[]}", 13);
  }
  ksg_last_error(c);
  ksg_destroy(c);
  return 0;
}

// --weights FILE: the profile's resolved plugin order and weights, one
// "position name weight store_weight" line per plugin (tests/test_fuzz_host.py).
static int print_weights(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string prof = ss.str();
  ksg_ctx* c = nullptr;
  ksg_opts o{};
  o.shard_count = 1;
  if (ksg_create(prof.data(), prof.size(), &o, &c) != KSG_OK) {
    std::printf("error\n");
    return 0;
  }
  static const char* kNames[] = {"SchedulingGates", "PrioritySort", "NodeUnschedulable", "NodeName",
                                 "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
                                 "VolumeRestrictions", "EBSLimits", "GCEPDLimits", "NodeVolumeLimits",
                                 "AzureDiskLimits", "VolumeBinding", "VolumeZone", "PodTopologySpread",
                                 "InterPodAffinity", "DefaultPreemption", "NodeResourcesBalancedAllocation",
                                 "ImageLocality", "DefaultBinder"};
  for (const char* nm : kNames) {
    const int pos = ksg_plugin_position(c, nm, std::string(nm).size());
    int64_t w = 0, sw = 0;
    if (pos >= 0 && ksg_plugin_weights(c, (uint32_t)pos, &w, &sw) == KSG_OK)
      std::printf("%d %s %lld %lld\n", pos, nm, (long long)w, (long long)sw);
  }
  ksg_destroy(c);
  return 0;
}

int main(int argc, char** argv) {
  if (argc == 3 && std::string(argv[1]) == "--weights") return print_weights(argv[2]);
  int n = 0;
  for (int i = 1; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    run_one(ss.str());
    ++n;
  }
  std::printf("fuzzed %d inputs\n", n);
  return 0;
}
