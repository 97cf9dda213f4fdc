// Device-visible data layout shared by the host encoder and the HIP kernels.
//
// Everything the kernels read about the cluster is interned to integers by the
// host (label keys, per-key label values, taints, namespaces, pod-label keys and
// values) and stored structure-of-arrays in HBM, one column per field, so a
// wavefront reading 64 consecutive nodes touches 64 consecutive elements.
// See DESIGN.md "Data layout in HBM" for sizes per config.
#pragma once
#include <stdint.h>

#define KSG_MAX_RES 8        // resource columns: 0 cpu(milli) 1 memory 2 ephemeral-storage 3.. scalar
#define KSG_MAX_PLUGINS 12   // plugins with device work in one profile (device profile positions)
#define KSG_MAX_PROFILE 32   // plugins in one profile (host; with the host-only ones)
#define KSG_MAX_IMG 16       // distinct node-listed images of one pod (ImageLocality)
#define KSG_MAX_SCORE_RES 8  // resources in a Fit/BA scoring config
#define KSG_MAX_TSC 8        // topology spread constraints per pod (filter + score)
#define KSG_MAX_TOPO 16      // distinct topology keys in one cluster
#define KSG_MAX_RTC 16       // RequestedToCapacityRatio shape points

#define KSG_RES_CPU 0
#define KSG_RES_MEM 1
#define KSG_RES_EPH 2

// plugin ids (ksg.h KSG_PLUGIN_*)
#define KP_FIT 0
#define KP_BA 1
#define KP_TAINT 2
#define KP_NA 3
#define KP_PTS 4
#define KP_IPA 5
#define KP_UNSCHED 6    // NodeUnschedulable
#define KP_NODENAME 7   // NodeName
#define KP_PORTS 8      // NodePorts
#define KP_IMAGE 9      // ImageLocality
#define KP_VOLUMES 10   // a run of consecutive volume plugins in the profile (one device position):
                        // the pod's volume checks (ksg_vchk) of that position, in plugin order
// host plugin kinds (the host records what the wrapper would; their Filters run on
// the device as KP_VOLUMES positions)
#define KP_VOLUME 16    // VolumeRestrictions, EBSLimits, GCEPDLimits, NodeVolumeLimits, AzureDiskLimits, VolumeZone
#define KP_VOLBIND 17   // VolumeBinding
#define KP_NOOP 18      // SchedulingGates, PrioritySort, DefaultPreemption, DefaultBinder

// node flags column
#define KSG_NODE_UNSCHEDULABLE 1u  // node.spec.unschedulable

// filter result code per (pod,node): 0xFFFFFFFF passed every filter plugin,
// 0xFFFFFFFE not evaluated (outside the NodeAffinity PreFilterResult), else
// (profile position << 24) | detail  (detail: Fit reason bits, taint id, PTS/IPA reason;
// KP_VOLUMES: plugin index within the run << 16 | KSG_VOL_* reason bits).
#define KSG_FILTER_PASS 0xFFFFFFFFu
#define KSG_FILTER_NOT_EVALUATED 0xFFFFFFFEu
#define KSG_FIT_TOO_MANY_PODS 1u   // Fit detail bit 0; bit (1 + r) = insufficient resource column r
#define KSG_PTS_MISSING_LABEL 0u
#define KSG_PTS_SKEW 1u
#define KSG_IPA_AFFINITY 0u
#define KSG_IPA_ANTI_AFFINITY 1u
#define KSG_IPA_EXISTING_ANTI 2u

// volume plugin reasons (KP_VOLUMES detail bits; messages rendered by the host)
#define KSG_VOL_RWOP (1u << 0)            // VolumeRestrictions ErrReasonReadWriteOncePodConflict
#define KSG_VOL_NODE_CONFLICT (1u << 1)   // VolumeBinding ErrReasonNodeConflict
#define KSG_VOL_BIND_CONFLICT (1u << 2)   // VolumeBinding ErrReasonBindConflict
#define KSG_VOL_PV_NOT_EXIST (1u << 3)    // VolumeBinding ErrReasonPVNotExist
#define KSG_VOL_ZONE_CONFLICT (1u << 4)   // VolumeZone ErrReasonConflict
#define KSG_VOL_MAX_COUNT (1u << 5)       // NodeVolumeLimits ErrReasonMaxVolumeCountExceeded
#define KSG_VOL_NODES 16                  // nodes one CSI volume may be attached to (host-checked)

// requirement operators (labels.Requirement / node selector requirement)
#define KR_IN 0          // present && value in vals
#define KR_NOT_IN 1      // !present || value not in vals
#define KR_EXISTS 2
#define KR_NOT_EXISTS 3
#define KR_GT 4          // present && numeric(value) > num
#define KR_LT 5
#define KR_FALSE 6       // parse error: never matches
#define KR_NAME_EQ 7     // matchFields metadata.name In: global node index == num
#define KR_NAME_NE 8     // matchFields metadata.name NotIn

typedef struct ksg_req {
  int32_t key;      // label key id (node-label space or pod-label space)
  int32_t op;       // KR_*
  int32_t nvals;    // values in the program's value pool
  int32_t val_off;
  int64_t num;      // KR_GT / KR_LT threshold
} ksg_req;          // 24 B

// A selector = AND of reqs. kind 0: labels.Nothing (matches nothing, Empty()==false);
// kind 1: requirement list (zero reqs = labels.Everything, Empty()==true).
typedef struct ksg_sel {
  int32_t kind;
  int32_t req_off;
  int32_t req_cnt;
  int32_t pad;
} ksg_sel;

// A node-label requirement flattened by the host (ksg_prog.off_freq, one entry
// per ksg_req of the program, same index; KPF_FLAT_NA): for keys with at most 64
// values every operator is a test of the node's value id against a 64-bit mask
// of the value ids that satisfy it (In: the listed values; Exists: every value;
// Gt / Lt: the values whose integer view compares true; NotIn / DoesNotExist
// the complement rule), so the evaluation has no value-list loop.
#define KFR_ANY 0     // matches when the node has the key and its value's bit is set
#define KFR_NONE 1    // matches when the node lacks the key or its value's bit is clear
#define KFR_NAME_EQ 2 // matchFields metadata.name In: global node index == arg
#define KFR_NAME_NE 3
#define KFR_FALSE 4
typedef struct ksg_freq {
  int32_t key;      // node label key id (-1: not in the vocabulary: no node has it)
  int32_t mode;     // KFR_*
  uint64_t arg;     // value-id mask (KFR_ANY / KFR_NONE) or the node index
} ksg_freq;         // 16 B

// one pod (anti-)affinity term of the incoming pod (framework.AffinityTerm)
typedef struct ksg_aterm {
  ksg_sel sel;
  int32_t topo;      // topology slot (index into pair_base)
  int32_t topo_key;  // node label key id
  int32_t ns_all;    // namespaceSelector matches every namespace
  int32_t ns_cnt;    // namespaces (ids) in the program's value pool
  int32_t ns_off;
  int32_t weight;    // preferred terms
  int32_t cls;       // pod class of the pods the term matches (class tables; -1 matches none)
  int32_t nub;       // its key's base among the shared-key pairs (pc_dom), -1: one node per value (pc_cnt)
} ksg_aterm;

typedef struct ksg_tsc {
  ksg_sel sel;
  int32_t topo;          // topology slot of the key
  int32_t topo_key;      // node label key id
  int32_t max_skew;
  int32_t min_domains;
  int32_t honor_affinity;
  int32_t honor_taints;
  int32_t self_match;    // selector matches the incoming pod's own labels
  int32_t is_hostname;
  int32_t first_of_key;  // first score constraint with this key (topoSize owner)
  int32_t cls;           // pod class counted (class tables; -1: the selector counts nothing)
  int32_t eff_cls;       // filter: class of the LAST filter constraint on this key (its count fills the pair)
  int32_t nub;           // the key's base among the shared-key pairs (pc_dom), -1: one node per value (pc_cnt)
  int32_t sc_n, sc_off;  // score: (class, nub) pairs whose counts share this constraint's pair (pool_i32)
  int32_t pair_base;     // the key's first (key, value) pair, and its values (minMatchNum per block)
  int32_t nvals;
  int32_t dom;           // values of the key present on some node of the shard (minMatchNum: none -> Error)
} ksg_tsc;

// One volume check of an incoming pod (host compile of the volume plugins'
// PreFilter state; evaluated at device position dpos, KP_VOLUMES).  The checks of
// one plugin (sub) are consecutive; a failing check ORs `bits` into that plugin's
// reasons unless one of `unless` is already there; the first plugin of the run
// with reasons fails the node.
#define KSG_VCHK_FAIL 0   // always fails (pod-uniform verdict)
#define KSG_VCHK_SELS 1   // fails unless one of the node selector terms pool_sel[off .. off+cnt) matches
#define KSG_VCHK_USED 2   // fails if a PVC of pool_i32[off .. off+cnt) is used by a pod (ReadWriteOncePod)
#define KSG_VCHK_LIMIT 3  // NodeVolumeLimits: (volume, limit key) pairs pool_i32[off .. off+2*cnt): attached + new
                          // volumes of a key above the node's limit for it fails
typedef struct ksg_vchk {
  int32_t dpos, sub, kind, bits, unless, off, cnt, pad;
} ksg_vchk;  // 32 B, in pool_i32 (8 words each)

// Table-chain lookup plan (host compile, table-path pods): every class-table
// count k_eval reads per node, issued together once the node's topology values
// are known, and what the count feeds.
typedef struct ksg_look {
  int32_t base;    // the table entry of value 0 / node 0 (kind)
  int32_t weight;  // KLU_RAW: signed multiplier
  // slot + 1 | kind << 8 | use << 16 | aux << 24 in ONE 32-bit word (ksg_lk_*):
  // the device reads the plan with scalar loads (which cannot fetch a byte at an
  // unaligned offset), and the unrolled plan's fields are live in SGPRs across
  // the evaluation — four words per entry there spilled to VGPR lanes.
  //   slot: topology slot whose value selects the entry (no value: count 0)
  //   kind: KLK_*; use: KLU_*; aux: KLU_PTSF's filter constraint
  uint32_t sku;
  int32_t pad;
} ksg_look;
#define KSG_LK_MAX 24
#ifdef __cplusplus  // (constexpr: host and device functions alike under hipcc)
constexpr int32_t ksg_lk_slot(uint32_t sku) { return (int32_t)(sku & 0xFFu) - 1; }
constexpr int32_t ksg_lk_kind(uint32_t sku) { return (int32_t)((sku >> 8) & 0xFFu); }
constexpr int32_t ksg_lk_use(uint32_t sku) { return (int32_t)((sku >> 16) & 0xFFu); }
constexpr int32_t ksg_lk_aux(uint32_t sku) { return (int32_t)(sku >> 24); }
#endif
#define KLK_NONE 0      // count 0 (class counts nothing)
#define KLK_PC_NODE 1   // pc_cnt[base + node]
#define KLK_PC_DOM 2    // pc_dom[base + value]
#define KLK_TC_NODE 3   // tc_val[base + node]
#define KLK_TC_DOM 4    // tc_val[base + value]
#define KLU_PTSF 1      // PodTopologySpread filter count of constraint aux
#define KLU_PTSS 2      // PodTopologySpread score count (summed)
#define KLU_AFF 3       // InterPodAffinity required affinity: count <= 0 or no value fails
#define KLU_ANTI 4      // required anti-affinity: a count > 0 fails
#define KLU_RAW 5       // InterPodAffinity raw score += count * weight
#define KLU_EXANTI 6    // existing pods' required anti-affinity: a count > 0 fails (when in force)
// InterPodAffinity map-emptiness bits (pod-uniform): bit set when the total is > 0
typedef struct ksg_ubit {
  int32_t idx;   // pc_tot / tc_tot index
  int32_t kind;  // 1 pc_tot, 2 tc_tot (32-bit fields: scalar loads, see ksg_look)
  int32_t bit;
} ksg_ubit;
#define KSG_UB_MAX 16
// ksg_prog tab_rd / tab_md bit of class-table key (space 1: pod class, 2: term
// class value offset, 3: term class) — one bit per key
static inline uint64_t ksg_tab_bloom(uint32_t space, uint32_t id) {
  const uint64_t x = (((uint64_t)space << 32) | id) * 0x9E3779B97F4A7C15ull;
  return 1ull << (x >> 58);
}

// Existing-pod record appended at assume time (Reserve -> NodeInfo.AddPod).
typedef struct ksg_exist_term {
  int32_t kind;      // 0 required affinity, 1 required anti, 2 preferred affinity, 3 preferred anti
  int32_t weight;
  int32_t topo;      // topology slot
  int32_t topo_key;  // node label key id
  ksg_sel sel;       // offsets into the TABLE's req pool once appended
  int32_t ns_all;
  int32_t ns_cnt;
  int32_t ns_off;    // into the table's value pool
  int32_t cls;       // term class (class tables), -1 none
  int32_t toff;      // its table's offset in the term-class value pool
  int32_t pad;
} ksg_exist_term;

// ---- class tables (PodTopologySpread / InterPodAffinity counts kept by the assume delta)
// A pod class is a conjunction of (namespaces, label selector) terms, optionally
// skipping terminating pods (PodTopologySpread's countPodsMatchSelector); per
// class the device keeps, per node, the matching existing pods, per (topology
// key, value) of keys whose values span several nodes their sum, and per key the
// pods on nodes carrying the key.  A term class groups existing pods' affinity
// terms (kind group, topology key, namespaces, selector): per (key, value) the
// terms there (anti / required) or their signed weights (preferred).
#define KSG_TC_HARD 0     // existing pods' required affinity terms (hardPodAffinityWeight)
#define KSG_TC_ANTI 1     // required anti-affinity (existing anti-affinity filter)
#define KSG_TC_PREF 2     // preferred affinity (+w) / anti-affinity (-w)
typedef struct ksg_cterm {
  ksg_sel sel;       // pod-label space, class pools
  int32_t ns_all, ns_cnt, ns_off, pad;
} ksg_cterm;
typedef struct ksg_pclass {
  int32_t n_terms, term_off;
  int32_t excl_term;  // terminating pods never match
  int32_t pad;
} ksg_pclass;

// Pod program: everything the kernels need about one incoming pod.  The
// program is a flat blob: this header followed by pools addressed by offsets
// (all offsets are element indices into the named pool, which start at the
// byte offsets given in the header).
typedef struct ksg_prog {
  int32_t queue_idx;        // scheduling-queue position (tie-break hash input)
  int32_t ns_id;
  uint32_t flags;           // KPF_*
  int32_t n_pod_label_keys; // incoming pod's label values: pool_i32[labels_off .. + n)
  int32_t labels_off;

  // ---- NodeResourcesFit / BalancedAllocation
  int64_t req[KSG_MAX_RES];               // PodRequests (Fit filter, Requested delta)
  int64_t fit_score_req[KSG_MAX_SCORE_RES];  // nonzero requests per Fit scoring resource
  int64_t ba_req[KSG_MAX_SCORE_RES];      // requests per BA resource
  int64_t nz_cpu, nz_mem;                 // NonZeroRequested delta

  // ---- TaintToleration: bitsets over the taint vocabulary in pool_u32
  int32_t taint_words;
  int32_t taint_hard_off;   // bit t: taint t is NoSchedule/NoExecute and NOT tolerated
  int32_t taint_pref_off;   // bit t: taint t is PreferNoSchedule and NOT tolerated by prefer-tolerations

  // ---- NodeAffinity (RequiredNodeAffinity + PreferredSchedulingTerms)
  ksg_sel node_sel;         // pod.spec.nodeSelector (kind 1 with reqs) when present
  int32_t n_req_terms;      // required terms (OR); terms with parse errors are dropped
  int32_t req_terms_off;    // pool_sel
  int32_t n_pref_terms;
  int32_t pref_terms_off;   // pool_sel; weight in pool_i32[pref_w_off + i]
  int32_t pref_w_off;
  int32_t restrict_words;   // PreFilterResult node bitmask (local nodes) in pool_u32
  int32_t restrict_off;
  int32_t restrict_g_words; // ... over every node of the cluster (node-sharded static records), or 0
  int32_t restrict_g_off;

  // ---- PodTopologySpread
  int32_t n_tsc_filter, n_tsc_score;
  ksg_tsc tsc[KSG_MAX_TSC];  // filter constraints first, then score constraints

  // ---- InterPodAffinity (incoming terms, namespaces merged)
  int32_t n_req_aff, n_req_anti, n_pref_aff, n_pref_anti;
  int32_t aterm_off;        // pool_aterm: req_aff, req_anti, pref_aff, pref_anti
  int32_t self_matches_all; // podMatchesAllAffinityTerms(required affinity, pod)

  // ---- NodeName / NodePorts / ImageLocality
  int32_t node_name_gid;    // spec.nodeName: -1 empty (fits every node), -2 names no node, else global node index
  int32_t n_port_check;     // pool_i32[port_check_off ..): host-port triples whose count > 0 on a node conflicts
  int32_t port_check_off;   //   (HostPortInfo.CheckConflict of every wanted port, folded on the host)
  int32_t n_port_own;       // pool_i32[port_own_off ..): the pod's own triples (NodeInfo.UsedPorts delta on assume)
  int32_t port_own_off;
  int32_t n_img;            // images some node lists, with the summed scaledImageScore of the containers using them
  int32_t img_id[KSG_MAX_IMG];
  int64_t img_scaled[KSG_MAX_IMG];
  int64_t img_max_threshold;  // maxContainerThreshold x (#init + #containers)

  // ---- as-existing record (committed on assume)
  uint32_t exist_flags;     // KEF_*
  int32_t n_exist_terms;
  int32_t exist_terms_off;  // pool_eterm (sel/ns offsets relative to this program's pools)

  // ---- class tables
  uint32_t tab;             // KTAB_*: PodTopologySpread / InterPodAffinity read the class tables
  int32_t aff_cls;          // required pod affinity: class of the pods matching every term (-1 none)
  int32_t n_pc_match, pc_match_off;  // pool_i32: pod classes this pod belongs to (its assume: +-1)
  int32_t n_tc_match, tc_match_off;  // pool_i32: term classes whose terms match this pod (id, value offset, slot, group)
  int32_t n_lk, n_ub;       // table chain: lookup plan and InterPodAffinity bits
  ksg_look lk[KSG_LK_MAX];
  ksg_ubit ub[KSG_UB_MAX];
  // 64-bit Bloom filters (ksg_tab_bloom) of the pair-level class-table entries —
  // pod classes' pc_dom / pc_tot, term classes' shared-value tc_val / tc_tot — the
  // pod's evaluation reads (tab_rd) and its assume writes (tab_md).  k_chain_run:
  // a pod whose reads miss the previous pod's writes does not wait for that assume
  // (node-level entries are read only by the block owning the node).  ~0: unknown.
  uint64_t tab_rd, tab_md;
  // the same for the node-level entries (pc_cnt of the pod's classes, one-node-per-value
  // tc_val): k_chain_run evaluates pod k+1 before pod k's assume only when pod k+1
  // reads none of the entries pod k writes at either level.  ~0: unknown.
  uint64_t nd_rd, nd_md;

  // ---- volume plugins
  int32_t n_vchk, vchk_off;  // pool_i32: ksg_vchk records (8 words each)
  int32_t n_pvc, pvc_off;    // pool_i32: PVC ids of the pod's volumes (NodeInfo PVCRefCounts delta on assume)
  int32_t n_csi, csi_off;    // pool_i32: (CSI volume, limit key) pairs of the pod (attached-volume delta on assume)

  // ---- pools (byte offsets from the start of the blob)
  uint32_t off_i32, n_i32;
  uint32_t off_u32, n_u32;
  uint32_t off_req, n_req;
  uint32_t off_sel, n_sel;
  uint32_t off_aterm, n_aterm;
  uint32_t off_eterm, n_eterm;
  uint32_t off_freq, n_freq;    // ksg_freq per ksg_req (KPF_FLAT_NA)
  uint32_t total_bytes;
  uint32_t pad;
} ksg_prog;

// KPF_* pod flags
#define KPF_ZERO_REQUEST (1u << 0)    // PodRequests all zero incl. scalars (fitsRequest early return)
#define KPF_HAS_NODE_SEL (1u << 1)    // RequiredNodeAffinity.labelSelector != nil
#define KPF_HAS_REQ_NA (1u << 2)      // RequiredNodeAffinity.nodeSelector != nil
#define KPF_RESTRICT (1u << 3)        // PreFilterResult restricts evaluated nodes
#define KPF_SKIP_NA_FILTER (1u << 4)  // PreFilter Skip (host-known)
#define KPF_SKIP_PTS_FILTER (1u << 5)
#define KPF_SKIP_NA_SCORE (1u << 6)   // PreScore Skip (host-known)
#define KPF_SKIP_PTS_SCORE (1u << 7)
#define KPF_IPA_HAS_CONSTRAINTS (1u << 8)  // incoming preferred (anti)affinity terms present
#define KPF_NA_PREF_ERROR (1u << 9)   // preferred terms failed to parse: PreScore error
#define KPF_HAS_SCALAR_REQ (1u << 10)
#define KPF_PREFILTER_REJECT (1u << 11)  // PreFilter Unschedulable (host-known): no node evaluated
#define KPF_PREFILTER_ERROR (1u << 12)   // PreFilter error status: cycle aborts
#define KPF_TOL_UNSCHED (1u << 13)       // tolerates node.kubernetes.io/unschedulable:NoSchedule
#define KPF_SKIP_PORTS (1u << 14)        // NodePorts PreFilter Skip (no host ports)
#define KPF_FLAT_NA (1u << 15)           // node selectors evaluate through the ksg_freq pool

// KTAB_* (ksg_prog.tab)
#define KTAB_ON (1u << 0)        // the pod runs the table chain (k_eval / k_final / k_select)
#define KTAB_PTS_MULTI (1u << 1) // several score constraints: PodTopologySpread raw scores need their own pass
#define KSG_TAB_MAXV 1024        // table chain: values of a filter key reduced per block (minMatchNum)
#define KSG_TAB_REGV 64          // table chain: values of a score key registered in a 64-bit mask

// KEF_* existing-pod flags
#define KEF_TERMINATING (1u << 0)
#define KEF_WITH_AFFINITY (1u << 1)
#define KEF_REQ_ANTI (1u << 2)
#define KEF_DELETED (1u << 3)      // unreserved: ignored by every scan

// per-pod cycle summary written by the device (read back by the host)
typedef struct ksg_pod_summary {
  uint64_t best_key;        // (total << 40) | ((0xFFFFF - h20) << 20) | global node index
  int32_t selected;         // global node index, -1 none
  int32_t feasible;
  int32_t status;           // 0 scheduled, 1 unschedulable, 2 error
  uint32_t skip_filter;     // bit = plugin id, PreFilter returned Skip
  uint32_t skip_score;      // bit = plugin id, PreScore returned Skip
  int32_t ignored;          // PodTopologySpread ignored nodes (feasible, missing keys)
  int64_t max_score[KSG_MAX_PLUGINS];  // per profile position, over feasible nodes
  int64_t min_score[KSG_MAX_PLUGINS];
  double pts_weight[KSG_MAX_TSC];
  uint32_t ipa_flags;       // bit0 affinity counts non-empty, bit1 anti counts, bit2 existing anti, bit3 topo score non-empty
  int32_t pad;
} ksg_pod_summary;
