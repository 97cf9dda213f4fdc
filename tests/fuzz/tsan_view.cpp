// ThreadSanitizer driver for the boundary's thread model (include/ksg.h
// "Threads"; tests/test_fuzz_host.py): the framework's 16 parallelize.Until
// workers read one cycle's per-node results (Filter / Score / NormalizeScore,
// wrappedplugin.go:523-548, :420-445, :388-415) through a ksg_cycle_view while
// other goroutines keep calling into the same context (per-node status calls,
// new cycles, view acquire / release).  Built against stub_engine.cpp with
// -fsanitize=thread; any race report fails the run.  argv: profile.json cluster.json pod.json
#include <atomic>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ksg.h"

static std::string slurp(const char* p) {
  std::ifstream f(p, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// a digest of everything a view holds
static uint64_t digest(const ksg_cycle_view* v) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
  for (uint32_t i = 0; i < v->n_nodes; ++i) {
    mix((uint64_t)(int64_t)v->fail_pos[i]);
    mix((uint64_t)(int64_t)v->fail_code[i]);
    mix(v->fail_msg[i]);
    if (v->fail_msg[i] >= v->n_messages) return 0;
    for (const char* c = v->messages[v->fail_msg[i]]; *c; ++c) mix((uint64_t)*c);
  }
  for (uint32_t p = 0; p < v->n_positions; ++p) {
    mix(v->filter_called[p]);
    for (uint32_t i = 0; i < v->n_nodes; ++i) {
      if (v->score[p]) mix((uint64_t)ksg_view_score(v, p, i, 0));
      if (v->normalized[p]) mix((uint64_t)ksg_view_score(v, p, i, 1));
    }
  }
  for (uint32_t p = 0; p < v->n_positions; ++p) {
    mix((uint64_t)(int64_t)v->prefilter_code[p]);
    mix((uint64_t)(int64_t)v->prescore_code[p]);
  }
  mix((uint64_t)v->result.selected);
  mix((uint64_t)v->result.feasible);
  return h;
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const std::string prof = slurp(argv[1]), cl = slurp(argv[2]), pod = slurp(argv[3]);
  ksg_ctx* c = nullptr;
  if (ksg_create(prof.data(), prof.size(), nullptr, &c) != KSG_OK) return 3;
  if (ksg_load_cluster(c, cl.data(), cl.size()) != KSG_OK) { std::fprintf(stderr, "%s\n", ksg_last_error(c)); return 4; }
  const int qn = ksg_queue_len(c);
  if (qn <= 0) return 5;
  ksg_keep_outputs(c, 0, (uint32_t)qn);
  if (ksg_schedule_queue(c, 0, (uint32_t)qn) != KSG_OK || ksg_wait(c, nullptr) != KSG_OK) return 6;
  // reference digests, single-threaded
  std::vector<uint64_t> ref((size_t)qn);
  for (int q = 0; q < qn; ++q) {
    const ksg_cycle_view* v = nullptr;
    if (ksg_cycle_view_acquire(c, (uint32_t)q, &v) != KSG_OK) { std::fprintf(stderr, "%s\n", ksg_last_error(c)); return 7; }
    ref[(size_t)q] = digest(v);
    ksg_cycle_view_release(v);
  }
  const ksg_cycle_view* shared = nullptr;  // one cycle's view read by all the workers
  if (ksg_cycle_view_acquire(c, 0, &shared) != KSG_OK) return 8;
  const int nn = ksg_num_nodes(c);
  std::atomic<int> bad{0}, calls{0};
  std::vector<std::thread> th;
  // phase 1: views of every pod acquired / read / released concurrently (the
  // context unchanged: each equals its single-threaded digest); phase 2: a new
  // cycle now and then (later views show what is kept then, not checked), the
  // shared view unchanged throughout
  std::atomic<int> phase1_left{16};
  for (int t = 0; t < 16; ++t)
    th.emplace_back([&, t] {
      for (int it = 0; it < 40; ++it) {
        if (digest(shared) != ref[0]) bad++;  // Filter / Score reads: no call into the library
        const int q = (t + it) % qn;
        const bool p1 = it < 20;
        if (it == 20) phase1_left--;
        const ksg_cycle_view* v = nullptr;
        if (ksg_cycle_view_acquire(c, (uint32_t)q, &v) == KSG_OK) {
          if (p1 && digest(v) != ref[(size_t)q]) bad++;
          ksg_cycle_view_release(v);
        } else if (p1) {
          bad++;
        }
        int32_t code = 0;
        char msg[512];
        size_t len = 0;
        if (ksg_filter_status(c, (uint32_t)q, (uint32_t)(it % 3), (uint32_t)((t * 7 + it) % (nn > 0 ? nn : 1)), &code, msg,
                              sizeof msg, &len) == KSG_OK)
          calls++;
        ksg_prefilter_status(c, (uint32_t)q, 0, &code, msg, sizeof msg, &len);
        if (t == 0 && it >= 20 && it % 4 == 0) {  // the scheduling goroutine: a new cycle meanwhile
          while (phase1_left.load() > 0) std::this_thread::yield();
          ksg_pod_result r;
          ksg_cycle(c, pod.data(), pod.size(), 1, &r);
        }
        if (t == 1 && it == 20) (void)ksg_last_error(c);
      }
    });
  for (auto& x : th) x.join();
  const uint64_t again = digest(shared);
  ksg_cycle_view_release(shared);
  ksg_destroy(c);
  if (bad.load() || again != ref[0]) { std::fprintf(stderr, "views changed under concurrent use (%d)\n", bad.load()); return 9; }
  std::printf("tsan ok: %d status calls, %d pods\n", calls.load(), qn);
  return 0;
}
