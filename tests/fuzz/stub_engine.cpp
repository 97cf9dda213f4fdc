// Test-only stand-in for the HIP engine (csrc/engine.hip) so that the host
// layer (csrc/host.cpp: JSON parsing, vocabulary, snapshot encoding, program
// compilation, class registry, events, rendering, the C ABI) can be built on
// the CPU with AddressSanitizer / UndefinedBehaviorSanitizer and fuzzed.
// Nothing here is shipped or linked into libksg.so: every cycle ends
// "unschedulable" with no node evaluated; the shapes the host hands over are
// checked so that an encoder bug shows up as a failure here.
#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "../../kube-scheduler-simulator-p9_amd/csrc/engine.h"

namespace ksg {

struct Engine::Impl {
  EngineConfig cfg;
  uint32_t N = 0, R = 0;
  std::vector<std::vector<uint8_t>> progs;
  std::vector<ksg_pod_summary> sums;
  std::vector<int64_t> req;
  std::vector<int32_t> podcnt;
  uint32_t used[4] = {0, 0, 0, 0}, cap[4] = {0, 0, 0, 0};
  uint32_t npc = 0, ntc = 0;
  uint32_t keep_first = 0, keep_n = 0;
  size_t staged = 0, vstore = 0;
};

static bool check_prog(const std::vector<uint8_t>& p, std::string& err) {
  if (p.size() < sizeof(ksg_prog)) { err = "stub: short program"; return false; }
  ksg_prog h;
  std::memcpy(&h, p.data(), sizeof(h));
  if (h.total_bytes != p.size()) { err = "stub: program size"; return false; }
  const uint64_t ends[] = {(uint64_t)h.off_i32 + 4ull * h.n_i32, (uint64_t)h.off_u32 + 4ull * h.n_u32,
                           (uint64_t)h.off_req + sizeof(ksg_req) * (uint64_t)h.n_req,
                           (uint64_t)h.off_sel + sizeof(ksg_sel) * (uint64_t)h.n_sel,
                           (uint64_t)h.off_aterm + sizeof(ksg_aterm) * (uint64_t)h.n_aterm,
                           (uint64_t)h.off_eterm + sizeof(ksg_exist_term) * (uint64_t)h.n_eterm,
                           (uint64_t)h.off_freq + sizeof(ksg_freq) * (uint64_t)h.n_freq};
  for (uint64_t e : ends)
    if (e > p.size()) { err = "stub: pool outside the program"; return false; }
  if (h.n_lk < 0 || h.n_lk > KSG_LK_MAX || h.n_ub < 0 || h.n_ub > KSG_UB_MAX) { err = "stub: plan"; return false; }
  if (h.n_tsc_filter < 0 || h.n_tsc_score < 0 || h.n_tsc_filter + h.n_tsc_score > KSG_MAX_TSC) {
    err = "stub: constraints";
    return false;
  }
  return true;
}

Engine::Engine() : p_(new Impl) {}
Engine::~Engine() { delete p_; }
bool Engine::init(const EngineConfig& cfg, std::string&) {
  p_->cfg = cfg;
  return true;
}
bool Engine::upload(const NodeSoA& nodes, const PodTableSoA& pods, uint32_t pod_cap, uint32_t term_cap,
                    uint32_t req_cap, uint32_t val_cap, std::string& err) {
  Impl& I = *p_;
  if (nodes.alloc.size() != (size_t)nodes.n_res * nodes.n || nodes.requested.size() != nodes.alloc.size() ||
      nodes.label_vid.size() != (size_t)nodes.n_keys * nodes.n || nodes.taint_off.size() != (size_t)nodes.n + 1 ||
      pods.node.size() != pods.n || pods.label_vid.size() != (size_t)pods.n_keys * pods.n) {
    err = "stub: snapshot shapes";
    return false;
  }
  if (pod_cap < pods.n || term_cap < pods.terms.size()) { err = "stub: capacities"; return false; }
  I.N = nodes.n;
  I.R = nodes.n_res;
  I.req = nodes.requested;
  I.podcnt = nodes.pod_count;
  I.used[0] = pods.n;
  I.used[1] = (uint32_t)pods.terms.size();
  I.used[2] = (uint32_t)pods.reqs.size();
  I.used[3] = (uint32_t)pods.vals.size();
  I.cap[0] = pod_cap;
  I.cap[1] = term_cap;
  I.cap[2] = req_cap;
  I.cap[3] = val_cap;
  I.npc = I.ntc = 0;
  return true;
}
bool Engine::set_score_resources(const int32_t*, const int32_t*, std::string&) { return true; }
bool Engine::set_programs(const std::vector<std::vector<uint8_t>>& progs, std::string& err) {
  for (auto& p : progs)
    if (!check_prog(p, err)) return false;
  p_->progs = progs;
  p_->sums.assign(progs.size(), ksg_pod_summary{});
  return true;
}
bool Engine::append_program(const std::vector<uint8_t>& prog, std::string& err) {
  if (!check_prog(prog, err)) return false;
  p_->progs.push_back(prog);
  p_->sums.push_back(ksg_pod_summary{});
  return true;
}
bool Engine::assume(uint32_t q, int32_t gnode, int, std::string& err, bool) {
  if (q >= p_->progs.size() || gnode < 0) { err = "stub: assume range"; return false; }
  return true;
}
bool Engine::bound_deltas(const std::vector<std::vector<uint8_t>>& progs, const std::vector<int32_t>& gnode,
                          const std::vector<int32_t>& sign, const std::vector<int32_t>& slot, std::vector<int32_t>& rows,
                          std::string& err) {
  if (gnode.size() != progs.size() || sign.size() != progs.size() || slot.size() != progs.size()) {
    err = "stub: deltas";
    return false;
  }
  for (auto& p : progs)
    if (!check_prog(p, err)) return false;
  for (size_t i = 0; i < slot.size(); ++i) {
    if (slot[i] < 0 || (size_t)slot[i] >= rows.size()) { err = "stub: slot"; return false; }
    if (sign[i] > 0) rows[slot[i]] = -1;
  }
  return true;
}
bool Engine::toggle_pods(const std::vector<const std::vector<uint8_t>*>& progs, const std::vector<int32_t>& gnode,
                         const std::vector<int32_t>& rows, int sign, std::string& err) {
  if (gnode.size() != progs.size() || rows.size() != progs.size() || (sign != 1 && sign != -1)) {
    err = "stub: toggle";
    return false;
  }
  for (size_t i = 0; i < progs.size(); ++i) {
    if (!progs[i] || !check_prog(*progs[i], err)) return false;
    if (gnode[i] < 0 || (uint32_t)gnode[i] >= p_->N) { err = "stub: toggle node"; return false; }
  }
  return true;
}
bool Engine::toggle_stage(const std::vector<const std::vector<uint8_t>*>& progs, const std::vector<int32_t>& gnode,
                          const std::vector<int32_t>& rows, std::string& err) {
  if (gnode.size() != progs.size() || rows.size() != progs.size()) { err = "stub: toggle_stage"; return false; }
  for (size_t i = 0; i < progs.size(); ++i) {
    if (!progs[i] || !check_prog(*progs[i], err)) return false;
    if (gnode[i] < 0 || (uint32_t)gnode[i] >= p_->N) { err = "stub: toggle node"; return false; }
  }
  p_->staged = progs.size();
  return true;
}
bool Engine::victim_store(const std::vector<const std::vector<uint8_t>*>& progs, std::string& err) {
  for (auto* pr : progs)
    if (!pr || !check_prog(*pr, err)) return false;
  p_->vstore = progs.size();
  return true;
}
bool Engine::toggle_stage_refs(const std::vector<int64_t>& ref, const std::vector<int32_t>& gnode,
                               const std::vector<int32_t>& rows, const std::vector<uint8_t>& queue_csi, std::string& err) {
  if (gnode.size() != ref.size() || rows.size() != ref.size()) { err = "stub: toggle_stage_refs"; return false; }
  for (size_t i = 0; i < ref.size(); ++i) {
    if (ref[i] >= 0 ? (size_t)ref[i] >= p_->vstore : (size_t)(-1 - ref[i]) >= std::min(p_->progs.size(), queue_csi.size())) {
      err = "stub: toggle ref";
      return false;
    }
    if (gnode[i] < 0 || (uint32_t)gnode[i] >= p_->N) { err = "stub: toggle node"; return false; }
  }
  p_->staged = ref.size();
  return true;
}
bool Engine::toggle_staged(const std::vector<uint32_t>& idx, int sign, std::string& err) {
  if (sign != 1 && sign != -1) { err = "stub: toggle sign"; return false; }
  for (uint32_t i : idx)
    if (i >= p_->staged) { err = "stub: toggle index"; return false; }
  return true;
}
// Filter codes that walk the host's preemption paths: every node fails the
// device position (i mod n) with detail 1; single-node probes pass on odd nodes.
bool Engine::dry_filter(uint32_t q, int32_t gnode, std::vector<uint32_t>& codes, std::string& err) {
  if (q >= p_->progs.size()) { err = "stub: dry_filter range"; return false; }
  if (gnode >= (int32_t)p_->N) { err = "stub: dry_filter node"; return false; }
  const uint32_t nd = p_->cfg.n_plugins > 0 ? (uint32_t)p_->cfg.n_plugins : 1;
  if (gnode >= 0) {
    codes.assign(1, (gnode & 1) ? KSG_FILTER_PASS : ((uint32_t)(gnode % nd) << 24) | 1u);
    return true;
  }
  codes.resize(p_->N);
  for (uint32_t i = 0; i < p_->N; ++i) codes[i] = ((i % nd) << 24) | 1u;
  return true;
}
bool Engine::pod_row(uint32_t q, int32_t& row, std::string& err) {
  if (q >= p_->progs.size()) { err = "stub: pod_row range"; return false; }
  row = -1;
  return true;
}
bool Engine::grow_table(uint32_t pod_cap, uint32_t term_cap, uint32_t req_cap, uint32_t val_cap, uint32_t,
                        std::string&) {
  uint32_t c[4] = {pod_cap, term_cap, req_cap, val_cap};
  for (int i = 0; i < 4; ++i) p_->cap[i] = std::max(p_->cap[i], c[i]);
  return true;
}
bool Engine::node_alloc(int32_t gnode, const std::vector<int64_t>& alloc, int32_t, std::string& err) {
  if (gnode < 0 || alloc.size() < p_->R) { err = "stub: node_alloc"; return false; }
  return true;
}
bool Engine::node_static(const std::vector<int32_t>& gnodes, const std::vector<int32_t>&, const std::vector<uint8_t>& hl,
                         const std::vector<uint8_t>& fl, std::string& err) {
  if (hl.size() != gnodes.size() || fl.size() != gnodes.size()) { err = "stub: node_static sizes"; return false; }
  for (int32_t g : gnodes)
    if (g < 0) { err = "stub: node_static"; return false; }
  return true;
}
bool Engine::node_taints(const std::vector<uint32_t>& offs, const std::vector<int32_t>& ids,
                         const std::vector<uint32_t>&, const std::vector<int32_t>&, std::string& err) {
  if (offs.empty() || offs.back() != ids.size()) { err = "stub: node_taints"; return false; }
  return true;
}
bool Engine::set_summaries(uint32_t first, uint32_t count, const ksg_pod_summary* in, std::string& err) {
  if ((size_t)first + count > p_->sums.size()) { err = "stub: summaries range"; return false; }
  std::memcpy(p_->sums.data() + first, in, (size_t)count * sizeof(ksg_pod_summary));
  return true;
}
bool Engine::table_overflow(bool& overflow, std::string&) {
  overflow = false;
  return true;
}
bool Engine::table_room(uint32_t used[4], uint32_t cap[4], std::string&) {
  for (int k = 0; k < 4; ++k) {
    used[k] = p_->used[k];
    cap[k] = p_->cap[k];
  }
  return true;
}
bool Engine::add_classes(const ClassUpload& u, std::string& err, const std::vector<uint8_t>*, bool* placed) {
  if (placed) *placed = false;
  if (u.tc_off.size() != u.tc_slot.size()) { err = "stub: classes"; return false; }
  p_->npc += (uint32_t)u.pc.size();
  p_->ntc += (uint32_t)u.tc_slot.size();
  return true;
}
uint32_t Engine::pod_classes() const { return p_->npc; }
uint32_t Engine::term_classes() const { return p_->ntc; }
bool Engine::rebuild_class_tables(std::string&) { return true; }
bool Engine::replace_program(uint32_t q, const std::vector<uint8_t>& prog, std::string& err) {
  if (q >= p_->progs.size()) { err = "stub: replace range"; return false; }
  if (!check_prog(prog, err)) return false;
  p_->progs[q] = prog;
  return true;
}
bool Engine::normalized(uint32_t, std::vector<int32_t>& norm, std::string&) {
  norm.assign((size_t)p_->cfg.n_plugins * p_->N, 0);
  return true;
}
bool Engine::run_queue(uint32_t first, uint32_t count, bool, std::string& err) {
  if ((size_t)first + count > p_->progs.size()) { err = "stub: run range"; return false; }
  for (uint32_t j = first; j < first + count; ++j) {
    ksg_pod_summary& s = p_->sums[j];
    s = ksg_pod_summary{};
    s.selected = -1;
    s.status = 1;  // unschedulable: no node evaluated
  }
  return true;
}
bool Engine::run_whatif(uint32_t first, uint32_t count, std::string& err) { return run_queue(first, count, false, err); }
void Engine::release_scratch() {}
bool Engine::keep_outputs(uint32_t keep_first, uint32_t keep_n, std::string&) {
  p_->keep_first = keep_first;
  p_->keep_n = keep_n;
  return true;
}
bool Engine::summaries(uint32_t first, uint32_t count, ksg_pod_summary* out, std::string& err) {
  if ((size_t)first + count > p_->sums.size()) { err = "stub: summaries range"; return false; }
  std::memcpy(out, p_->sums.data() + first, (size_t)count * sizeof(ksg_pod_summary));
  return true;
}
bool Engine::outputs(uint32_t prog_idx, PodOutputs& out, std::string& err) {
  if (prog_idx >= p_->sums.size()) { err = "stub: outputs range"; return false; }
  // kept pods: every other node passed, raw scores a function of (pod, node, position)
  const bool kept = p_->keep_n && prog_idx >= p_->keep_first && prog_idx < p_->keep_first + p_->keep_n;
  out.filter.assign(p_->N, KSG_FILTER_NOT_EVALUATED);
  out.score.assign((size_t)p_->cfg.n_plugins * p_->N, 0);
  out.total.assign(p_->N, 0);
  if (kept)
    for (uint32_t i = 0; i < p_->N; ++i) {
      if ((i + prog_idx) % 2 == 0) out.filter[i] = KSG_FILTER_PASS;
      for (int d = 0; d < p_->cfg.n_plugins; ++d)
        out.score[(size_t)d * p_->N + i] = (int32_t)((i * 7 + prog_idx * 3 + (uint32_t)d) % 101);
    }
  out.summary = p_->sums[prog_idx];
  return true;
}
bool Engine::sync(std::string&) { return true; }
bool Engine::static_time(float& total_ms, uint32_t& launches, uint64_t& pods, std::string&) {
  total_ms = 0;
  launches = 0;
  pods = 0;
  return true;
}
bool Engine::reset(std::string&) { return true; }
void Engine::sample_kernel(uint32_t) {}
void Engine::set_path(int) {}
bool Engine::batch_path() const { return false; }
bool Engine::set_exchange(int, const void*, uint32_t, uint32_t, ExchangeFn, void*, std::string& err) {
  err = "stub: no exchange";
  return false;
}
uint32_t Engine::exchange_ranks() const { return 1; }
void Engine::path_counts(uint64_t out[8]) const {
  for (int i = 0; i < 8; ++i) out[i] = 0;
}
bool Engine::lost() const { return false; }
void Engine::clear_lost() {}
bool Engine::nccl_unique_id(void*, std::string& err) {
  err = "stub: no RCCL";
  return false;
}
bool Engine::fixup_stamps(uint32_t, std::vector<uint64_t>* out, std::string&) {
  if (out) out->clear();
  return true;
}
bool Engine::eval_stamps(bool, std::vector<uint64_t>* out, std::string&) {
  if (out) out->clear();
  return true;
}
bool Engine::kernel_time(float& avg_ms, uint32_t& samples, std::string&) {
  avg_ms = 0;
  samples = 0;
  return true;
}
bool Engine::read_requested(std::vector<int64_t>& requested, std::vector<int32_t>& pod_count, std::string&) {
  requested = p_->req;
  pod_count = p_->podcnt;
  return true;
}
bool Engine::read_nonzero(std::vector<int64_t>& nz, std::string&) {
  nz.assign(2 * (size_t)p_->N, 0);
  return true;
}
uint32_t Engine::n_nodes() const { return p_->N; }
void* Engine::stream() const { return nullptr; }
float Engine::last_ms() const { return 0; }
std::vector<Engine::KernelStat> Engine::kernel_stats() const { return {}; }

}  // namespace ksg

// device cycle view, stub: the synthetic outputs laid out as Engine::view does
namespace ksg {
static size_t al256s(size_t x) { return (x + 255) & ~(size_t)255; }
void Engine::view_layout(ViewLayout& lay) const {
  lay = ViewLayout{};
  lay.N = p_->N;
  lay.n_raw = (uint32_t)p_->cfg.n_plugins;
  lay.n_slots = 256;
  for (int d = 0; d < KSG_MAX_PLUGINS; ++d) lay.norm_row[d] = -1;
  const size_t N = p_->N ? p_->N : 1;
  lay.off_sum = al256s(257 * 8);
  lay.off_rows = lay.off_sum + al256s(sizeof(ksg_pod_summary));
  lay.off_fail_pos = lay.off_rows + al256s(sizeof(ViewRows));
  lay.off_fail_code = lay.off_fail_pos + al256s(N);
  lay.off_fail_msg = lay.off_fail_code + al256s(N);
  lay.off_raw = lay.off_fail_msg + al256s(2 * N);
  lay.off_norm = lay.off_raw + al256s(4 * N) * lay.n_raw;
  lay.bytes = lay.off_norm;
}
bool Engine::view_arm(uint32_t q, const ViewCfg& cfg, const ViewLayout& lay, uint8_t* host, std::string& err) {
  return view(q, cfg, lay, host, err, false);
}
bool Engine::view_arm_finish(std::string&) { return true; }
bool Engine::view_fused() const { return false; }
uint64_t Engine::views_fused() const { return 0; }
bool Engine::view(uint32_t q, const ViewCfg& cfg, const ViewLayout& lay, uint8_t* host, std::string& err, bool) {
  PodOutputs o;
  if (!(p_->keep_n && q >= p_->keep_first && q < p_->keep_first + p_->keep_n)) { err = "outputs not kept for this pod"; return false; }
  if (!outputs(q, o, err)) return false;
  std::memset(host, 0, lay.bytes);
  lay.gen = 1;
  std::memcpy(host + lay.off_sum, &o.summary, sizeof(o.summary));
  ViewRows rows{};
  for (uint32_t d = 0; d < lay.n_raw; ++d) {
    rows.off[d] = (uint32_t)(lay.off_raw + al256s(4 * (size_t)(p_->N ? p_->N : 1)) * d);
    rows.bytes[d] = 4;
  }
  std::memcpy(host + lay.off_rows, &rows, sizeof(rows));
  for (uint32_t i = 0; i < p_->N; ++i) {
    const uint32_t c = o.filter[i];
    reinterpret_cast<int8_t*>(host + lay.off_fail_pos)[i] =
        (int8_t)(c == KSG_FILTER_PASS ? cfg.n_profile : (c == KSG_FILTER_NOT_EVALUATED ? -1 : 0));
    for (uint32_t d = 0; d < lay.n_raw; ++d)
      reinterpret_cast<int32_t*>(host + rows.off[d])[i] = o.score[(size_t)d * p_->N + i];
  }
  return true;
}
uint8_t* Engine::pinned_get(size_t bytes, size_t& cap) {
  cap = bytes ? bytes : 1;
  return static_cast<uint8_t*>(std::malloc(cap));
}
void Engine::pinned_put(uint8_t* p, size_t) { std::free(p); }
uint8_t* Engine::pinned_dev(const uint8_t*) { return nullptr; }
uint64_t Engine::static_dec_chunks() const { return 0; }
uint64_t Engine::static_overlaps() const { return 0; }
bool rccl_selftest(int, size_t, std::string& err) {
  err = "stub: no RCCL";
  return false;
}
}  // namespace ksg
