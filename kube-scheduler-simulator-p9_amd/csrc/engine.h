// Engine: device-resident node snapshot + existing-pod table + the per-pod
// scheduling-cycle kernels.  Host-side C++ (host.cpp) owns the object model,
// interning and rendering; it talks to the engine only through this class.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "ksg_types.h"

namespace ksg {

struct EngineConfig {
  int device = 0;
  void* stream = nullptr;  // hipStream_t (nullptr: engine creates its own)
  int n_plugins = 0;
  int plugins[KSG_MAX_PLUGINS] = {};         // KP_* in MultiPoint (profile) order
  int64_t weight[KSG_MAX_PLUGINS] = {};      // framework score weights per profile position
  int fit_strategy = 0;                      // 0 LeastAllocated 1 MostAllocated 2 RequestedToCapacityRatio
  int fit_n = 2;
  int fit_res[KSG_MAX_SCORE_RES] = {0, 1};
  int64_t fit_w[KSG_MAX_SCORE_RES] = {1, 1};
  int rtc_n = 0;
  int64_t rtc_util[KSG_MAX_RTC] = {};
  int64_t rtc_score[KSG_MAX_RTC] = {};
  int ba_n = 2;
  int ba_res[KSG_MAX_SCORE_RES] = {0, 1};
  int64_t ipa_hard_weight = 1;
  int ipa_ignore_existing_pref = 0;
  uint64_t seed = 0;
  uint32_t global_node_offset = 0;  // shard: global index of local node 0
};

// Host-side SoA image of the node snapshot (one shard).
struct NodeSoA {
  uint32_t n = 0, n_res = 3, n_keys = 0;
  uint32_t global_offset = 0;             // global index of local node 0 (sharding)
  uint32_t global_n = 0;                  // nodes of the whole cluster (every shard)
  std::vector<int64_t> alloc, requested;  // [n_res][n]
  std::vector<int64_t> nz_cpu, nz_mem;    // [n]
  std::vector<int32_t> allowed_pods, pod_count;
  std::vector<int32_t> label_vid;         // [n_keys][n]
  std::vector<uint32_t> taint_off;        // [n+1]
  std::vector<int32_t> taint_id;
  std::vector<uint8_t> has_labels;        // [n]
  std::vector<uint8_t> node_flags;        // [n] KSG_NODE_*
  uint32_t img_words = 0;                 // ImageLocality: node image bitsets [img_words][n] over the image vocabulary
  std::vector<uint32_t> img_bits;
  uint32_t n_ports = 0;                   // NodePorts: used host-port triple counts [n_ports][n]
  std::vector<int32_t> port_count;
  std::vector<int32_t> pvc_use;           // VolumeRestrictions: pods using each PVC id (bound pods of the whole cluster)
  // NodeVolumeLimits: per limit key (attachable-volumes-csi-<driver>) the node's limit
  // (-1 none) and its attached unique volumes; per CSI volume the nodes it is
  // attached to (KSG_VOL_NODES slots, node -1 empty) and the pods using it there
  uint32_t n_lkeys = 0, n_vols = 0;
  std::vector<int32_t> vol_limit, vol_attached;  // [n_lkeys][n]
  std::vector<int32_t> vol_node, vol_ref;        // [n_vols][KSG_VOL_NODES]
  // node-label vocabulary numeric view (Gt/Lt): per key offset into value tables
  std::vector<uint32_t> key_val_off;      // [n_keys+1]
  std::vector<int64_t> val_num;
  std::vector<uint8_t> val_num_ok;
  // topology slots: node label key per slot and value count
  std::vector<int32_t> topo_key;
  std::vector<uint32_t> topo_base, topo_count;
  std::vector<uint8_t> topo_unique;  // per slot: every value of the key sits on one node (whole cluster)
  uint32_t topo_pairs = 0;
  // class tables: per slot the base of its values among the pairs of keys whose
  // values span nodes (UINT32_MAX for one-node keys) and its values present on
  // some node of this shard; per pair whether some node of this shard carries it
  std::vector<uint32_t> nu_base;
  uint32_t nu_pairs = 0;
  std::vector<int32_t> slot_dom;
  std::vector<uint8_t> pair_node;
  // node sharding: ranks of the context, and every node's topology values
  // [slot][global_n] (value id, -1 none) — the pair-level class-table deltas
  // of an assume on another rank's node (every rank keeps the global tables)
  uint32_t shards = 1;
  // node-sharded Taint / NodeAffinity windows: every node's static data (labels,
  // taints) on every rank, so that each rank holds every (pod, node) static record
  std::vector<int32_t> g_label_vid;   // [n_keys][global_n], empty when not needed
  std::vector<uint32_t> g_taint_off;  // [global_n + 1]
  std::vector<int32_t> g_taint_id;
  std::vector<int32_t> gtopo;
};

// Class definitions appended to the device (host.cpp registry; ksg_types.h
// "class tables").  Offsets are relative to this upload's own pools.
struct ClassUpload {
  std::vector<ksg_pclass> pc;    // new pod classes (term_off into ct)
  std::vector<ksg_cterm> ct;     // their terms (sel.req_off into creq, ns_off into cval)
  std::vector<ksg_req> creq;     // selector requirements (val_off into cval)
  std::vector<int32_t> cval;
  std::vector<int32_t> tc_slot;  // new term classes: their topology slot
  std::vector<uint32_t> tc_off;  // ... and the offset of their values in the pool (host-assigned, ascending)
};

// Existing pods (bound) on this shard's nodes, and their (anti)affinity terms.
struct PodTableSoA {
  uint32_t n = 0, n_keys = 0;
  std::vector<int32_t> node, ns;
  std::vector<uint32_t> flags;     // KEF_*
  std::vector<int32_t> label_vid;  // [n_keys][cap] (cap == n on upload)
  std::vector<ksg_exist_term> terms;
  std::vector<int32_t> term_pod;
  std::vector<ksg_req> reqs;
  std::vector<int32_t> vals;
};

struct PodOutputs {  // per-pair outputs of one pod, host copies
  std::vector<uint32_t> filter;  // [n]
  std::vector<int32_t> score;    // [n_plugins][n]
  std::vector<int32_t> total;    // [n]
  ksg_pod_summary summary;
};

class Engine {
 public:
  Engine();
  ~Engine();
  bool init(const EngineConfig& cfg, std::string& err);
  // capacities: pods/terms/reqs/vals of the existing-pod table (device appends on assume)
  bool upload(const NodeSoA& nodes, const PodTableSoA& pods, uint32_t pod_cap, uint32_t term_cap,
              uint32_t req_cap, uint32_t val_cap, std::string& err);
  // Resource columns of the Fit / BalancedAllocation scoring arguments (after a
  // vocabulary build: the columns the names resolve to).
  bool set_score_resources(const int32_t* fit_res, const int32_t* ba_res, std::string& err);
  // Queue programs: blobs laid out by the host encoder (ksg_prog + pools).
  bool set_programs(const std::vector<std::vector<uint8_t>>& progs, std::string& err);
  // Append one program (drop-in cycle API); its index is the previous count.
  bool append_program(const std::vector<uint8_t>& prog, std::string& err);
  // Reserve (sign +1) / Unreserve (sign -1) program q on global node gnode.
  // (wait = false: the launch is queued and the call returns; a later sync
  // reports any device error)
  bool assume(uint32_t q, int32_t gnode, int sign, std::string& err, bool wait = true);
  // Cluster events applied in place, one k_assume per op in stream order, one sync:
  // bound pod progs[i] added on (sign +1) / removed from (sign -1) global node
  // gnode[i] (nodes outside this shard are ignored).  rows[] holds one existing-pod
  // table row slot per op (in: the row a removal tombstones; out: the row an
  // addition appended, -1 none); op i reads/writes slot[i] (a removal of a pod
  // added by the same batch uses that addition's slot).
  bool bound_deltas(const std::vector<std::vector<uint8_t>>& progs, const std::vector<int32_t>& gnode,
                    const std::vector<int32_t>& sign, const std::vector<int32_t>& slot, std::vector<int32_t>& rows,
                    std::string& err);
  // DefaultPreemption dry run (host-orchestrated, SelectVictimsOnNode): pods
  // progs[i] leave (sign -1) / re-enter (sign +1) global node gnode[i]; rows[i]
  // is the existing-pod table row tombstoned / revived in place (-1 none).
  bool toggle_pods(const std::vector<const std::vector<uint8_t>*>& progs, const std::vector<int32_t>& gnode,
                   const std::vector<int32_t>& rows, int sign, std::string& err);
  // The batched victim search's form: the candidate victims are uploaded once
  // (entries 0..n-1: program, global node, table row), then subsets of them
  // toggled by index, one launch per subset (one thread per node: a node's
  // victims in sequence, different nodes in parallel).
  bool toggle_stage(const std::vector<const std::vector<uint8_t>*>& progs, const std::vector<int32_t>& gnode,
                    const std::vector<int32_t>& rows, std::string& err);
  bool toggle_staged(const std::vector<uint32_t>& idx, int sign, std::string& err);
  // The same staging by reference, without a program upload per search: the bound
  // pods' programs live on the device in the victim store (entry b = bound pod b,
  // uploaded by victim_store when the host's cache moves); entry i of the staging
  // is bound pod ref[i] (>= 0) or queue pod -1 - ref[i] (its program in the
  // queue's buffer; queue_csi[q]: it has CSI volumes).
  bool victim_store(const std::vector<const std::vector<uint8_t>*>& progs, std::string& err);
  bool toggle_stage_refs(const std::vector<int64_t>& ref, const std::vector<int32_t>& gnode,
                         const std::vector<int32_t>& rows, const std::vector<uint8_t>& queue_csi, std::string& err);
  // Filter codes of program q against the current device state (its whole cycle
  // re-run without commit; kept outputs and the pod's summary are left as they
  // were): global node gnode's code, or every node's when gnode is -1.
  bool dry_filter(uint32_t q, int32_t gnode, std::vector<uint32_t>& codes, std::string& err);
  // Existing-pod table row the device appended for queue pod q (-1 none).
  bool pod_row(uint32_t q, int32_t& row, std::string& err);
  // Cluster event applied in place: node gnode's allocatable [R] and allowed pod count.
  bool node_alloc(int32_t gnode, const std::vector<int64_t>& alloc, int32_t allowed, std::string& err);
  // Cluster events applied in place, one batch: node gnodes[i]'s label value per
  // node-label key (label_vid[i*K .. i*K+K), -1 none; vocabulary and topology
  // values unchanged), has-labels byte and KSG_NODE_* flags — into its columns when
  // it is on this shard, and into the every-node static columns when the context
  // keeps them.  One stream synchronisation for the whole batch.
  bool node_static(const std::vector<int32_t>& gnodes, const std::vector<int32_t>& label_vid,
                   const std::vector<uint8_t>& has_labels, const std::vector<uint8_t>& flags, std::string& err);
  // The node taint lists replaced (CSR over this shard's nodes; gofs/gids over
  // every node, used when the context keeps the every-node static columns).
  bool node_taints(const std::vector<uint32_t>& offs, const std::vector<int32_t>& ids,
                   const std::vector<uint32_t>& gofs, const std::vector<int32_t>& gids, std::string& err);
  bool set_summaries(uint32_t first, uint32_t count, const ksg_pod_summary* in, std::string& err);
  // An assume found the existing-pod table full (the pod was not appended).
  bool table_overflow(bool& overflow, std::string& err);
  // Grow the existing-pod table in place (contents kept): row / term / req / val
  // capacities and the pod-label key count (new keys' columns read "no label").
  bool grow_table(uint32_t pod_cap, uint32_t term_cap, uint32_t req_cap, uint32_t val_cap, uint32_t n_keys,
                  std::string& err);
  // Existing-pod table entries in use and capacity: rows, terms, reqs, vals.
  bool table_room(uint32_t used[4], uint32_t cap[4], std::string& err);
  // Class tables: append pod / term classes and build their tables from the
  // existing-pod table; counts of classes with tables; rebuild every table.
  // prog: the cycle's pod program, appended (as append_program) in the same
  // upload when the classes go out as one (*placed: it was; otherwise the caller
  // appends it).
  bool add_classes(const ClassUpload& u, std::string& err, const std::vector<uint8_t>* prog = nullptr,
                   bool* placed = nullptr);
  uint32_t pod_classes() const;
  uint32_t term_classes() const;
  bool rebuild_class_tables(std::string& err);
  // Replace program q (its class lists grew); summaries and placements stay.
  bool replace_program(uint32_t q, const std::vector<uint8_t>& prog, std::string& err);
  // Normalized scores of a kept pod, [n_plugins][n] (device NormalizeScore).
  bool normalized(uint32_t prog_idx, std::vector<int32_t>& norm, std::string& err);
  // Run pods [first, first+count) of the program list back to back on the device
  // (device-side assume).  keep: store per-pair outputs for pods [keep_first, keep_first+keep_n).
  bool run_queue(uint32_t first, uint32_t count, bool commit, std::string& err);
  // What-if step: pods [first, first+count) each against the current snapshot,
  // then all their placements bound (Fit/BA/Taint/NodeAffinity profiles).
  bool run_whatif(uint32_t first, uint32_t count, std::string& err);
  // Free the what-if record buffer (kept across steps: up to KSG_WHATIF_REC_MB).
  void release_scratch();
  bool keep_outputs(uint32_t keep_first, uint32_t keep_n, std::string& err);
  bool summaries(uint32_t first, uint32_t count, ksg_pod_summary* out, std::string& err);
  bool outputs(uint32_t prog_idx, PodOutputs& out, std::string& err);
  bool sync(std::string& err);
  // ksg_cycle_view on the device: profile facts the view kernel needs (host.cpp
  // fills them once per profile), the block layout for the current snapshot, and
  // the fill of a kept pod's view into a caller's (pinned) host block: one kernel,
  // one device-to-host copy.  Block: message-slot table (kViewSlots codes, 0xFFFFFFFF
  // empty, then an overflow word; 64-bit entries gen << 32 | code, live when gen is
  // this view's), the pod's summary, per node fail_pos / fail_code / fail_msg, raw
  // scores [device position][node], normalized [normalising row][node].
  struct ViewCfg {
    int n_profile = 0;
    int prof_of_dev[KSG_MAX_PLUGINS] = {};  // device position -> profile position
    bool dev_vol[KSG_MAX_PLUGINS] = {};     // the device position is a volume run
    int kind[KSG_MAX_PROFILE] = {};         // Filter failure code: 0 unresolvable, 1 unschedulable, 2 Fit, 3 PTS, 4 IPA
  };
  // the view block's score-row table (written by the view: offsets in the block,
  // value widths; index d: raw row of device position d, KSG_MAX_PLUGINS + r:
  // normalized row r)
  struct ViewRows {
    uint32_t off[2 * KSG_MAX_PLUGINS];
    uint8_t bytes[2 * KSG_MAX_PLUGINS];
  };
  struct ViewLayout {
    uint32_t N = 0, n_raw = 0, n_norm = 0, n_slots = 0;
    mutable uint32_t gen = 0;  // set by view(): live slot entries are gen << 32 | code
    size_t off_sum = 0;        // the pod's summary
    int norm_row[KSG_MAX_PLUGINS] = {};  // device position -> normalized row (-1: output == raw)
    size_t off_rows = 0;       // its ViewRows (score rows start at off_raw, packed, 256-B aligned)
    size_t off_fail_pos = 0, off_fail_code = 0, off_fail_msg = 0, off_raw = 0, off_norm = 0, bytes = 0;
  };
  void view_layout(ViewLayout& lay) const;
  // wait = false: only queued on the engine stream (the block is complete after the next sync)
  bool view(uint32_t q, const ViewCfg& cfg, const ViewLayout& lay, uint8_t* host, std::string& err, bool wait = true);
  // The fused view (round 6): view_arm prepares pod q's view like view() but launches
  // nothing; the next run_queue writes it from k_eval itself when the pod's cycle
  // is one k_eval (a profile without ScoreExtensions), and view_arm_finish launches
  // k_view otherwise.  view_fused(): the last armed view was written by k_eval (its
  // rows assume no Score error: a summary with status 2 needs a view() rebuild).
  bool view_arm(uint32_t q, const ViewCfg& cfg, const ViewLayout& lay, uint8_t* host, std::string& err);
  bool view_arm_finish(std::string& err);
  bool view_fused() const;
  uint64_t views_fused() const;  // diagnostic: views written by k_eval so far
  // pinned host blocks for views (process-wide pool: a view outlives its context)
  static uint8_t* pinned_get(size_t bytes, size_t& cap);
  static void pinned_put(uint8_t* p, size_t cap);
  static uint8_t* pinned_dev(const uint8_t* host);  // its device address (null: none / not pinned)
  // Restore the node rows / pod table to the state of the last upload (device copy).
  bool reset(std::string& err);
  // Sample the dominant kernel (k_filter_score) every `every` pods inside run_queue
  // with HIP events on the engine stream; 0 disables.
  void sample_kernel(uint32_t every);
  // 1: force the per-pod kernel chain even when the speculative batch path applies
  void set_path(int per_pod);
  bool batch_path() const;
  // Node-shard exchange for the batch path: mode 1 = RCCL all-gather on the engine
  // stream (nccl_id from nccl_unique_id on one rank), mode 2 = host callback
  // fn(user, send, recv, bytes_per_rank) returning 0 (tests: gloo).
  typedef int (*ExchangeFn)(void* user, const void* send, void* recv, size_t bytes_per_rank);
  bool set_exchange(int mode, const void* nccl_id, uint32_t rank, uint32_t ranks, ExchangeFn fn, void* user,
                    std::string& err);
  uint32_t exchange_ranks() const;
  // diagnostic: pods the per-pod runs sent down the table chain / the scanning chain /
  // of the table-chain pods, those whose cycle was one launch (k_eval_solo)
  // and persistent segments that fell back to the two-launch chain (out[6])
  void path_counts(uint64_t out[8]) const;
  // An aborted persistent launch left the device state half-updated: the context
  // must be reloaded (host.cpp marks it broken); cleared by a reload.
  bool lost() const;
  uint64_t static_dec_chunks() const;  // diagnostic: static-record chunks computed from decoded pods
  uint64_t static_overlaps() const;     // diagnostic: persistent runs whose static records were computed beside the loop
  void clear_lost();
  static bool nccl_unique_id(void* out128, std::string& err);
  // diagnostic: enable (out == nullptr, count pods) / read back s_memtime stamps of the fixup loop
  bool fixup_stamps(uint32_t count, std::vector<uint64_t>* out, std::string& err);
  bool eval_stamps(bool on, std::vector<uint64_t>* out, std::string& err);
  // Average duration (ms) and count of the sampled launches of the last run.
  bool kernel_time(float& avg_ms, uint32_t& samples, std::string& err);
  // The static-record launches (k_static) of the same sampled window run: their
  // total time, launches and pods.
  bool static_time(float& total_ms, uint32_t& launches, uint64_t& pods, std::string& err);
  // Read back the node resource rows (parity tests of the assume delta).
  bool read_requested(std::vector<int64_t>& requested, std::vector<int32_t>& pod_count, std::string& err);
  // NonZeroRequested cpu / memory rows [2][n] (Fit scoring input).
  bool read_nonzero(std::vector<int64_t>& nz, std::string& err);
  uint32_t n_nodes() const;
  void* stream() const;
  // timing of the last run_queue (device events), ms
  float last_ms() const;
  // per-kernel launch records for roofline accounting
  struct KernelStat {
    const char* name;
    double bytes;   // algorithmic bytes per launch
    uint32_t launches;
  };
  std::vector<KernelStat> kernel_stats() const;

  struct Impl;
  Impl* impl() { return p_; }

 private:
  bool view_impl(uint32_t q, const ViewCfg& cfg, const ViewLayout& lay, uint8_t* host, std::string& err, bool wait,
                 bool arm);
  Impl* p_;
};

}  // namespace ksg
