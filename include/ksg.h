/* ksg.h — C ABI of the MI355X scheduling-cycle engine (drop-in boundary).
 *
 * This is the surface a cgo package behind the simulator's debuggable scheduler
 * binds.  It replaces, for the hot-path plugins
 * (NodeResourcesFit, NodeResourcesBalancedAllocation, TaintToleration,
 * NodeAffinity, PodTopologySpread, InterPodAffinity), the per-(pod, node)
 * plugin calls the framework makes through the simulator's wrapper:
 *
 *   PreFilter        simulator/scheduler/plugin/wrappedplugin.go:504
 *   Filter           wrappedplugin.go:535   (interface pinned: plugin/mock/framework.go:114)
 *   PreScore         wrappedplugin.go:472   (mock :233)
 *   Score            wrappedplugin.go:433   (mock :285)
 *   NormalizeScore   wrappedplugin.go:400   (mock :338, ScoreExtensions :300)
 *   Reserve          wrappedplugin.go:631   (mock :597)  -> assume delta on the device
 *   selectHost       upstream schedule_one.go (seeded deterministic tie-break)
 * and renders the result store's annotations (resultstore/store.go:133-198) for
 * the evaluated pod, so filter-result / score-result / finalscore-result /
 * selected-node are byte-identical to what the wrapper records.
 *
 * Objects cross the boundary as Kubernetes JSON (what json.Marshal of a *v1.Pod /
 * *v1.Node produces); the library interns them into the device SoA snapshot.
 * Conventions: every function returns 0 on success and a negative KSG_E* code on
 * failure (message in ksg_last_error: the calling thread's last failure on that
 * context); no exceptions or aborts cross the ABI; output buffers are
 * caller-owned; one context per scheduler profile and GPU.
 * Threads: every call that takes a context holds that context's lock for its
 * duration, so calls from several threads (goroutines) are safe and serialised;
 * the per-node lookups of the framework's parallel workers should read a
 * ksg_cycle_view (no call at all) instead of ksg_filter_status & co. per node.
 * ksg_destroy must not race with other calls on the same context.
 */
#ifndef KSG_H_
#define KSG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history.  1: round-1..2 surface.  2: ksg_load_cluster orders the queue by
 * PrioritySort and holds back pods with schedulingGates (queue index q is no
 * longer document order: ksg_queue_pod names it); ksg_queue_pod, ksg_gated_pods,
 * ksg_cycle_view_acquire / _release added; a context whose persistent launch
 * stalled refuses calls (KSG_E_STATE) until ksg_load_cluster.  Bindings check
 * ksg_abi_version() >= the version they were written against.  3: ksg_cycle_view
 * holds the Filter outcome once per node (fail_pos / fail_code / fail_msg) and
 * 32-bit scores per position, built on the device.  4: its score rows are as
 * narrow as their values allow (score_bytes / normalized_bytes; ksg_view_score). */
#define KSG_ABI_VERSION 4

#define KSG_OK 0
#define KSG_E_INVALID (-1)   /* bad argument / JSON */
#define KSG_E_DEVICE (-2)    /* HIP error */
#define KSG_E_STATE (-3)     /* call out of order */
#define KSG_E_RANGE (-4)     /* index out of range */
#define KSG_E_NOBUF (-5)     /* output buffer too small (*len holds the size) */

/* plugin ids (profile positions are reported in this order of the profile) */
#define KSG_PLUGIN_NODE_RESOURCES_FIT 0
#define KSG_PLUGIN_NODE_RESOURCES_BALANCED_ALLOCATION 1
#define KSG_PLUGIN_TAINT_TOLERATION 2
#define KSG_PLUGIN_NODE_AFFINITY 3
#define KSG_PLUGIN_POD_TOPOLOGY_SPREAD 4
#define KSG_PLUGIN_INTER_POD_AFFINITY 5

/* ksg_pod_result.status */
#define KSG_SCHEDULED 0
#define KSG_UNSCHEDULABLE 1
#define KSG_ERROR 2

/* filter code per (pod, node): see ksg_filter_codes */
#define KSG_FILTER_PASSED 0xFFFFFFFFu
#define KSG_FILTER_NOT_EVALUATED 0xFFFFFFFEu

typedef struct ksg_ctx ksg_ctx;

typedef struct ksg_opts {
  int32_t device;        /* HIP device ordinal */
  void* stream;          /* hipStream_t to run on; NULL = library-owned stream */
  uint32_t shard_rank;   /* node sharding across GPUs: this context owns nodes   */
  uint32_t shard_count;  /* [rank*N/count, (rank+1)*N/count) of the cluster      */
  uint32_t flags;        /* reserved, 0 */
} ksg_opts;

typedef struct ksg_pod_result {
  int32_t selected;      /* global node index, -1 when none */
  int32_t feasible;      /* nodes that passed every filter plugin */
  int32_t status;        /* KSG_SCHEDULED / KSG_UNSCHEDULABLE / KSG_ERROR */
  uint32_t skip_filter;  /* bit i: plugin id i returned Skip from PreFilter */
  uint32_t skip_score;   /* bit i: plugin id i returned Skip from PreScore */
  int32_t total;         /* weighted score of the selected node */
} ksg_pod_result;

/* Profile JSON: {"plugins": [names in MultiPoint order], "weights": {name: w},
 * "storeWeights": {name: w}, "pluginConfig": {name: args}, "seed": n}
 * (the shape of KubeSchedulerConfiguration.profiles[0] restricted to the hot path;
 * storeWeights is the result store's map, plugins.go:289-304). */
int ksg_create(const char* profile_json, size_t len, const ksg_opts* opts, ksg_ctx** out);
void ksg_destroy(ksg_ctx* ctx);
const char* ksg_last_error(const ksg_ctx* ctx);
int ksg_abi_version(void);

/* Snapshot: {"nodes": [v1.Node], "pods": [bound v1.Pod], "queue": [v1.Pod],
 * "pvs": [v1.PersistentVolume], "pvcs": [v1.PersistentVolumeClaim],
 * "storageClasses": [storagev1.StorageClass]} (ResourcesForSnap field names; the
 * storage objects feed the volume plugins).
 * Replaces the device snapshot (UpdateSnapshot) and the queue.
 * With DefaultPreemption in the profile and >= 2,048 bound pods, the call starts a
 * thread of the context that compiles the bound pods' programs and uploads the
 * victim store DefaultPreemption's search reads (slices under the context's lock;
 * KSG_VICTIM_WARM=0: off); it is joined by the next ksg_load_cluster and by
 * ksg_destroy.  No entry point waits for it. */
int ksg_load_cluster(ksg_ctx* ctx, const char* json, size_t len);
int ksg_num_nodes(const ksg_ctx* ctx);     /* global node count */
int ksg_queue_len(const ksg_ctx* ctx);
/* The queue a document loads is the scheduling queue's pop order (upstream
 * v1.30.4 internal/queue/scheduling_queue.go): with SchedulingGates in the
 * profile (its PreEnqueue; default MultiPoint, scheduler_test.go:536) pods
 * carrying spec.schedulingGates never enter it — no cycle, no annotations —
 * and the rest are ordered as PrioritySort's Less (queuesort/priority_sort.go):
 * higher spec.priority first, then document order.  Queue index q is that
 * position; ksg_queue_pod names it ("namespace/name"), ksg_gated_pods lists the
 * held-back pods ("namespace/name\n" lines).  ksg_cycle pods are appended in
 * the order the framework runs them. */
int ksg_queue_pod(const ksg_ctx* ctx, uint32_t q, char* buf, size_t cap, size_t* len);
int ksg_gated_pods(const ksg_ctx* ctx, char* buf, size_t cap, size_t* len);

/* Queue mode: schedule queue pods [first, first+count) back to back on the
 * device; every selection is assumed on the device before the next pod
 * (no host round trip per pod).  Runs of consecutive PodTopologySpread /
 * InterPodAffinity table-chain pods execute as one persistent launch each
 * (env KSG_RUN=0: one launch pair per pod).  A persistent launch starts with a
 * handshake: when its blocks are not all resident within a few ms (e.g. another
 * context's persistent launch holds part of the CUs) every block leaves before
 * touching any state and the segment's pods run on the two-launch chain; the
 * call blocks until each segment's handshake has decided.  A launch that stalls
 * after its handshake (a poll bound of seconds) fails the call (KSG_E_DEVICE
 * from this call or ksg_wait) instead of hanging, and the context then refuses
 * every call (KSG_E_STATE) until ksg_load_cluster.  Asynchronous: ksg_wait()
 * completes it.
 * Every queue pod gets exactly one scheduling cycle, in queue order: a pod that
 * is unschedulable stays so (upstream parks it in unschedulablePods and retries
 * it after cluster events such as AssignedPodAdd; here the caller re-submits it,
 * e.g. through ksg_cycle, as the framework does in plugin mode).  The oracle
 * follows the same rule, so long queues on a tight cluster can diverge from a
 * live scheduler's retry order, not from the per-cycle results. */
int ksg_schedule_queue(ksg_ctx* ctx, uint32_t first, uint32_t count);
int ksg_wait(ksg_ctx* ctx, float* device_ms);
/* What-if step (BASELINE cfg5): queue pods [first, first+count) are each
 * scheduled against the SAME snapshot (no assume between them: the question
 * "where would each of these pods go now?"), then all their placements are
 * bound together, in queue order.  Any profile: NodeResourcesFit /
 * BalancedAllocation / TaintToleration / NodeAffinity profiles run as two
 * pod-tile x node-tile passes, the first leaving a 4- or 8-byte record per
 * (pod, node) for the second (count x nodes x 4 B: 16 GB at 4,096 pods x 1M
 * nodes; env KSG_WHATIF_REC_MB caps it, default 40960, larger steps run in pod
 * chunks, 0 recomputes every pair in the second pass instead; the record
 * buffer stays allocated across steps until the next ksg_load_cluster or
 * ksg_compact); a what-if step runs no PostFilter (no nomination is reported for its pods); others (PodTopologySpread / InterPodAffinity on
 * frozen class tables, the default profile) run every pod's cycle without
 * assume.  Sharded contexts reduce the per-pod feasible counts, normaliser
 * max/min and argmax keys across ranks.
 * Asynchronous like ksg_schedule_queue; results via ksg_pod_results. */
int ksg_whatif(ksg_ctx* ctx, uint32_t first, uint32_t count);
int ksg_pod_results(ksg_ctx* ctx, uint32_t first, uint32_t count, ksg_pod_result* out);

/* Restore node rows and the existing-pod table to the loaded snapshot
 * (benchmark steps replay the same queue). */
int ksg_reset(ksg_ctx* ctx);
/* Time the dominant Filter/Score kernel with HIP events on the context stream
 * for every `every`-th pod of the following ksg_schedule_queue (0 = off). */
int ksg_sample_kernel(ksg_ctx* ctx, uint32_t every);
int ksg_kernel_time(ksg_ctx* ctx, float* avg_ms, uint32_t* samples);
/* Execution path: profiles made only of NodeResourcesFit / BalancedAllocation
 * run as exact speculative 32-pod windows (k_window: evaluation of window j+1
 * beside the exact replay of window j); every other profile runs the per-pod
 * kernel chain.  per_pod != 0 forces the chain. */
int ksg_set_path(ksg_ctx* ctx, int per_pod);
int ksg_batch_path(const ksg_ctx* ctx);  /* 1 when the batch path is active */

/* Node sharding across GPUs (ksg_opts.shard_rank / shard_count; existing pods
 * live with their node).  Fit/BalancedAllocation profiles: per window of 32
 * pods every rank all-gathers its per-pod top-64 candidates (with their node
 * rows) and local feasible counts, merges them, and runs the same deterministic
 * replay, applying only its own nodes' assume deltas.  Other profiles: the
 * table chain on every rank's nodes against global class tables (each rank sums
 * its pair-level counts with the others' when a class is built and applies every
 * assume's pair-level delta), two exchanges per cycle (counts and normalisers;
 * argmax key), three with several PodTopologySpread score constraints; pods
 * whose spread constraints the tables cannot answer run the scanning chain
 * (four exchanges).  Needs ksg_set_exchange before the first run.  What-if
 * steps: per-pod summaries merged after each pass.
 *   mode 1: RCCL all-gather on the context stream; nccl_id = 128 bytes from
 *           ksg_nccl_unique_id() on one rank, broadcast by the caller.
 *   mode 2: host callback fn(user, send, recv, bytes_per_rank) that all-gathers
 *           host buffers (recv = ranks x bytes, rank order); returns 0.        */
typedef int (*ksg_exchange_fn)(void* user, const void* send, void* recv, size_t bytes_per_rank);
int ksg_nccl_unique_id(uint8_t* out128);
int ksg_set_exchange(ksg_ctx* ctx, int mode, const uint8_t* nccl_id, ksg_exchange_fn fn, void* user);

/* Keep per-(pod, node) outputs for queue pods [first, first+count) (tests,
 * annotation rendering).  Must precede ksg_schedule_queue. */
int ksg_keep_outputs(ksg_ctx* ctx, uint32_t first, uint32_t count);
/* Filter code per local node: KSG_FILTER_PASSED, KSG_FILTER_NOT_EVALUATED or
 * (profile position << 24) | detail (volume plugins: KSG_VOL_* reason bits of
 * ksg_types.h in the low 16 bits). */
int ksg_filter_codes(ksg_ctx* ctx, uint32_t q, uint32_t* out, uint32_t n);
/* Raw Score of profile position pos per local node (valid where the filter passed). */
int ksg_scores(ksg_ctx* ctx, uint32_t q, uint32_t pos, int32_t* out, uint32_t n);
/* Store.GetStoredResult for queue pod q as a JSON object {annotation key: value}. */
int ksg_annotations(ksg_ctx* ctx, uint32_t q, char* buf, size_t cap, size_t* len);

/* Drop-in cycle (one pod, the framework's scheduleOne): PreFilter..Score..
 * NormalizeScore for a new pod (v1.Pod JSON, appended to the queue: its index
 * is ksg_queue_len() - 1), its per-node outputs kept for ksg_filter_codes /
 * ksg_scores / ksg_annotations.  commit != 0 also assumes it on the engine's
 * selectHost choice (harness mode); commit == 0 leaves the assume to
 * ksg_reserve with the framework's own choice (plugin mode).  New label keys,
 * label values and namespaces are interned in place; a pod bringing a topology
 * key, a scalar resource or a host port the snapshot has not seen triggers a
 * re-encode of the snapshot (placements kept). */
int ksg_cycle(ksg_ctx* ctx, const char* pod_json, size_t len, int commit, ksg_pod_result* out);
/* ReservePlugin.Reserve (wrappedplugin.go:631 -> scheduler cache assume):
 * assume queue pod q (run with commit == 0) on global node `node`.  The device
 * delta is queued without a wait: a device failure of it is reported late, by the
 * next call that synchronises (a cycle, a view, Unreserve ...), which then returns
 * KSG_E_DEVICE and leaves the context refusing calls (KSG_E_STATE) until
 * ksg_load_cluster, since the host already counts the pod as placed. */
int ksg_reserve(ksg_ctx* ctx, uint32_t q, int32_t node);
/* ReservePlugin.Unreserve (mock framework.go:611): undo the assume of queue
 * pod q (cycle or queue mode): node rows, and its existing-pod table entry. */
int ksg_unreserve(ksg_ctx* ctx, uint32_t q);
/* Bounded memory in plugin mode: queue pods [0, keep_from) leave the queue —
 * the placed ones become bound pods of the snapshot, the rest are forgotten
 * (their documents released) — and pod keep_from + i becomes queue pod i, its
 * results and placement kept.  One snapshot re-encode; call between cycles with
 * keep_from = the oldest pod whose Reserve / Unreserve / lookups may still come
 * (ksg_queue_len() when none). */
int ksg_compact(ksg_ctx* ctx, uint32_t keep_from);

/* ---- what each wrapped plugin's extension point returns (the Go plugin's calls,
 * INTEGRATION.md), for queue pod q whose per-node outputs are kept (the pod of the
 * last ksg_cycle, or a range given to ksg_keep_outputs).  `pos` is the profile
 * position (ksg_plugin_position); `node` a global node index (ksg_node_index).
 * Status codes are framework.Code values (v1.30 framework/interface.go):
 * 0 Success, 1 Error, 2 Unschedulable, 3 UnschedulableAndUnresolvable, 5 Skip;
 * -1 means the framework does not call this plugin there (an earlier filter
 * failed on the node, PreFilter Skip, outside the PreFilterResult, no scoring).
 * Messages are Status.Message() (what the wrapper records, wrappedplugin.go:542). */
int ksg_plugin_position(const ksg_ctx* ctx, const char* name, size_t len);  /* or KSG_E_RANGE; "…Wrapped" accepted */
/* The weights the profile resolved for position `pos`: *weight is the framework's
 * (upstream framework.go getScoreWeights: an explicit Score weight wins over
 * MultiPoint's; it scales the total selectHost uses), *store_weight the result
 * store's (plugins.go:289-304 getScorePluginWeight: MultiPoint overwrites; it
 * scales finalscore-result, store.go:504-507).  They differ only in the quirk of
 * scheduler_test.go:344-407.  ksg_create takes the flat profile
 * {plugins, weights, storeWeights, pluginConfig} or a KubeSchedulerConfiguration /
 * KubeSchedulerProfile (plugins.multiPoint / plugins.score, pluginConfig list). */
int ksg_plugin_weights(const ksg_ctx* ctx, uint32_t pos, int64_t* weight, int64_t* store_weight);
int ksg_node_index(const ksg_ctx* ctx, const char* name, size_t len);       /* or KSG_E_RANGE */
/* PreFilter (wrappedplugin.go:504, mock framework.go:61): status; and the
 * PreFilterResult node set as a JSON array of node names, "null" for all nodes. */
int ksg_prefilter_status(ksg_ctx* ctx, uint32_t q, uint32_t pos, int32_t* code, char* msg, size_t cap, size_t* len);
int ksg_prefilter_result(ksg_ctx* ctx, uint32_t q, char* buf, size_t cap, size_t* len);
/* The PreFilterResult of the plugin at profile position pos (NodeAffinity's, or
 * VolumeBinding's GetEligibleNodes for claims bound to local PVs): JSON array of
 * node names, "null" when the plugin returns none.  The framework intersects them;
 * an empty intersection rejects the pod after the later plugin's PreFilter, whose
 * own status stays Success (ksg_prefilter_status). */
int ksg_prefilter_result_pos(ksg_ctx* ctx, uint32_t q, uint32_t pos, char* buf, size_t cap, size_t* len);
/* Filter (wrappedplugin.go:535, mock framework.go:114) on one node. */
int ksg_filter_status(ksg_ctx* ctx, uint32_t q, uint32_t pos, uint32_t node, int32_t* code, char* msg, size_t cap,
                      size_t* len);
/* PreScore (wrappedplugin.go:472, mock framework.go:233): status and message. */
int ksg_prescore_status(ksg_ctx* ctx, uint32_t q, uint32_t pos, int32_t* code, char* msg, size_t cap, size_t* len);
/* NormalizeScore (wrappedplugin.go:400, mock framework.go:338): the plugin's
 * normalized score per local node (raw score for plugins without
 * ScoreExtensions), computed on the device by the NormalizeScore the selection
 * used; valid where the node passed every filter. */
int ksg_normalized_scores(ksg_ctx* ctx, uint32_t q, uint32_t pos, int64_t* out, uint32_t n);
/* PostFilter (wrappedplugin.go:550-577 -> store.go:442 AddPostFilterResult):
 * DefaultPreemption's dry run for an unschedulable pod q (PodEligibleToPreemptOthers,
 * nodesWherePreemptionMightHelp, SelectVictimsOnNode, pickOneNodeForPreemption of
 * upstream v1.30.4 default_preemption.go / preemption.go; nothing is evicted).
 * *nominated = the nominated global node index, -1 none; buf receives the
 * victims as "namespace/name\n" lines (most important first).  Unsharded
 * contexts with DefaultPreemption in the profile; queue runs stop after each
 * pod that may preempt (ksg_schedule_queue then returns with them done). */
int ksg_postfilter_result(ksg_ctx* ctx, uint32_t q, int32_t* nominated, char* buf, size_t cap, size_t* len);

/* ---- per-node results of one cycle for concurrent readers.  The framework
 * calls Filter (wrappedplugin.go:523-548) and Score (:420-445) from its 16
 * parallelize.Until workers and NormalizeScore (:388-415) per plugin; a Go
 * plugin acquires the cycle's view once (the cycle's first PreFilter, after
 * ksg_cycle; kept in CycleState) and its per-node calls index these immutable
 * arrays — no library call, no lock.  Local node i is global node
 * node_offset + i.  The device builds the view (one kernel, one copy into a
 * pinned host block): the per-node Filter outcome is stored once per node, not
 * per position.  Filter of profile position pos on node i returns
 *   -1 (not called)               if !filter_called[pos] or fail_pos[i] < 0 or pos > fail_pos[i]
 *   Success (0)                    if pos < fail_pos[i]  (fail_pos[i] == n_positions: passed every filter)
 *   fail_code[i], messages[fail_msg[i]]   if pos == fail_pos[i]
 * Codes are framework.Code values (as ksg_filter_status).  score[pos] /
 * normalized[pos] point at n_nodes signed little-endian integers of
 * score_bytes[pos] / normalized_bytes[pos] bytes each (1, 2 or 4: the narrowest
 * width the cycle's values need, so fewer bytes cross the host link; read them
 * with ksg_view_score), NULL when there is no device Score at pos; valid where
 * the node passed every filter; normalized[pos] == score[pos] for plugins
 * without ScoreExtensions.  A view stays valid, unchanged, until
 * ksg_cycle_view_release, whatever the context does meanwhile (later cycles,
 * Reserve, events, ksg_destroy); release needs no context and may run on any
 * thread. */
typedef struct ksg_cycle_view {
  uint32_t q;                          /* queue pod */
  uint32_t n_positions;                /* profile positions */
  uint32_t node_offset;                /* global index of local node 0 */
  uint32_t n_nodes;                    /* local nodes */
  ksg_pod_result result;               /* the cycle's outcome (engine selectHost) */
  const uint8_t* filter_called;        /* [pos] 1: the framework calls this position's Filter */
  const int8_t* fail_pos;              /* [node] first failing position; n_positions: passed; -1: not evaluated */
  const int8_t* fail_code;             /* [node] framework code of that failure */
  const uint16_t* fail_msg;            /* [node] its Status.Message(): index into messages */
  const void* const* score;            /* [pos] -> [node] raw Score (score_bytes[pos] each), or NULL */
  const void* const* normalized;       /* [pos] -> [node] NormalizeScore output, or NULL */
  const uint8_t* score_bytes;          /* [pos] width of score[pos]'s values: 1, 2 or 4 */
  const uint8_t* normalized_bytes;     /* [pos] width of normalized[pos]'s values */
  const int8_t* prefilter_code;        /* [pos] PreFilter code (ksg_prefilter_status) */
  const uint16_t* prefilter_msg;       /* [pos] its message index */
  const int8_t* prescore_code;         /* [pos] PreScore code (ksg_prescore_status) */
  const uint16_t* prescore_msg;        /* [pos] its message index */
  const char* const* messages;         /* message table; messages[0] == "" */
  uint32_t n_messages;
  const void* owner;                   /* library-private */
} ksg_cycle_view;
/* The raw (normalized == 0) or normalized score of position pos on local node i. */
static inline int64_t ksg_view_score(const ksg_cycle_view* v, uint32_t pos, uint32_t i, int normalized) {
  const void* row = normalized ? v->normalized[pos] : v->score[pos];
  const uint8_t w = normalized ? v->normalized_bytes[pos] : v->score_bytes[pos];
  if (!row) return 0;
  if (w == 1) return ((const int8_t*)row)[i];
  if (w == 2) return ((const int16_t*)row)[i];
  return ((const int32_t*)row)[i];
}
/* Snapshot the kept outputs of queue pod q (the pod of the last ksg_cycle, or a
 * ksg_keep_outputs range) into a view.  For the pod of the last ksg_cycle with
 * commit = 0, acquired before any other state-changing call, the view was filled
 * behind that cycle's own kernels and is returned without a device launch. */
int ksg_cycle_view_acquire(ksg_ctx* ctx, uint32_t q, const ksg_cycle_view** out);
void ksg_cycle_view_release(const ksg_cycle_view* view);

/* Scheduler-cache events between cycles (replaces the informer -> Cache path:
 * Cache.AddNode/UpdateNode/RemoveNode/AddPod/UpdatePod/RemovePod of upstream
 * v1.30.4 pkg/scheduler/internal/cache/cache.go, driven by eventhandlers.go;
 * the simulator raises them from its apiserver).  JSON:
 *   {"events": [{"op": "addNode"|"updateNode", "node": {v1.Node}},
 *               {"op": "removeNode", "name": "node-x"},
 *               {"op": "addPod"|"updatePod", "pod": {v1.Pod with spec.nodeName}},
 *               {"op": "removePod", "name": "p", "namespace": "ns"}, ...]}
 * applied in order; the batch is all-or-nothing.  removePod also takes a queue
 * pod that was scheduled (its placement is released, its result kept);
 * removeNode requires that no pod is bound or assumed on the node (upstream
 * deletes the node's pods first).  Batches of bound-pod add/remove events,
 * deletions of queue pods scheduled since the last encode, and node updates of
 * allocatable, spec.unschedulable, labels (keys and values some node already
 * carried, no topology key changing value) and taints (taints some node already
 * carried) with the same images, all bringing no new vocabulary, are applied in
 * place on the device; any other batch re-encodes the snapshot (after an in-place
 * batch ksg_reset is refused: reload).  Placements of scheduled queue pods are kept;
 * node indices after a removed node shift down by one.  Per-node outputs kept for
 * pods scheduled before the batch are not re-indexed. */
int ksg_apply_events(ksg_ctx* ctx, const char* events_json, size_t len);

/* Device node rows (assume parity): requested [n_res][n], pod count [n]. */
int ksg_node_requested(ksg_ctx* ctx, int64_t* requested, int32_t* pod_count, uint32_t n_res, uint32_t n);
/* NonZeroRequested rows (Fit scoring input): cpu in nonzero[0..n), memory in nonzero[n..2n). */
int ksg_node_nonzero(ksg_ctx* ctx, int64_t* nonzero, uint32_t n);

/* Harness mode (benchmarks, full-size tests; no context): the synthetic cluster
 * document of BASELINE.json config 2..5 — the document
 * ksg/generator.py builds, from the same seeded draws.  Sizes < 0: the config's
 * default; seed 0: the config's seed.  *out is malloc'd: release with ksg_free. */
int ksg_synth_cluster(int config, int64_t n_nodes, int64_t n_pods, int64_t n_existing, int64_t n_zones, uint64_t seed,
                      char** out, size_t* len);
void ksg_free(void* p);

#ifdef __cplusplus
}
#endif
#endif /* KSG_H_ */
