// HIP engine for the scheduling-cycle hot path (gfx950 / MI355X).
//
// One scheduling cycle of one pod = the reference's schedulePod
// (findNodesThatFitPod -> prioritizeNodes -> selectHost) plus the assume of
// scheduleOne, restated as a short chain of kernels over the device-resident
// node snapshot (SoA, one thread per node, coalesced columns):
//
//   k_begin        zero the per-pod topology histograms            (PTS/IPA only)
//   k_scan_pods    existing pods  x incoming selectors/terms       (PTS/IPA only)
//   k_scan_terms   existing terms x incoming pod                   (IPA only)
//   k_pts_prep     per-node eligibility -> domain histograms       (PTS only)
//   k_pts_reduce   minMatchNum / domain counts per topology key     (PTS only)
//   k_filter_score Filter chain (first failure stops) + raw Score + per-plugin
//                  max/min + feasible count  [+ total & argmax when no plugin
//                  of the profile has ScoreExtensions]
//   k_pts_weights  topologyNormalizingWeight (Go math.Log restated) (PTS only)
//   k_pts_score    PodTopologySpread raw score + min/max            (PTS only)
//   k_finalize     NormalizeScore, [0,100] check, x weight, packed-key argmax
//   k_commit       assume: NodeInfo.AddPod delta on the selected node, append the
//                  pod (and its affinity terms) to the existing-pod table
//
// Reference call sites replaced: wrappedplugin.go:504 (PreFilter), :535
// (Filter), :472 (PreScore), :433 (Score), :400 (NormalizeScore), :631
// (Reserve); upstream algorithms restated in oracle/ksg_oracle.cpp (the
// checker).  Float64 arithmetic is compiled with -ffp-contract=off and follows
// the reference operation order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>
#include <utility>
#include <deque>
#include <atomic>
#include <map>
#include <mutex>
#include <chrono>
#include <cstddef>
#include <thread>

#include "engine.h"
#include <rccl/rccl.h>

namespace ksg {

#define HIPCHK(x)                                                                 \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      err = std::string(#x) + ": " + hipGetErrorString(e_);                       \
      return false;                                                               \
    }                                                                             \
  } while (0)

static constexpr int kBlock = 256;

// ----------------------------------------------------------------- kernel args
// Class tables (ksg_types.h "class tables"): PodTopologySpread / InterPodAffinity
// counts kept up to date by every assume delta instead of rescanning the
// existing pods per incoming pod.
struct DevTables {
  int on;                    // profile with PodTopologySpread / InterPodAffinity: assumes update the tables
  uint32_t npc, ntc;         // pod classes / term classes with tables
  uint32_t NU;               // (key, value) pairs of the keys whose values span several nodes
  uint32_t uniq;             // topology slots whose every value sits on one node (pair == node)
  int32_t* pc_cnt;           // [npc][N] matching existing pods per node
  int32_t* pc_dom;           // [npc][NU] ... per (key, value) of the shared keys
  int32_t* pc_tot;           // [npc][KSG_MAX_TOPO] ... on nodes carrying the key
  const uint32_t* nu_base;   // [KSG_MAX_TOPO] slot base in NU space
  const int32_t* slot_dom;   // [KSG_MAX_TOPO] values of the key on some node
  const uint8_t* pair_node;  // [pairs] the (key, value) pair is on some node
  const ksg_pclass* pcls;
  const ksg_cterm* cterm;
  const ksg_req* creq;
  const int32_t* cval;
  int32_t* tc_val;           // term classes: per (key, value) (per node for one-node keys)
  const uint32_t* tc_off;    // [ntc]
  const int32_t* tc_slot;    // [ntc]
  int32_t* tc_tot;           // [ntc] terms on nodes carrying the key
  // node sharding: the node-level entries (pc_cnt, tc_val of one-node keys) are
  // the owner's, the pair-level ones (pc_dom, pc_tot, tc_val of shared keys,
  // tc_tot) are global on every rank — an assume on another rank's node applies
  // them too, with that node's topology values from gtv
  int sharded;
  uint32_t G;                // nodes of the whole cluster
  const int32_t* gtv;        // [n_topo][G] every node's topology values (-1 none), sharded contexts
};

struct DevCluster {
  uint32_t N, R, K, goff;
  const int64_t* alloc;
  int64_t* req;
  int64_t* nzc;
  int64_t* nzm;
  const int32_t* allowed;
  int32_t* podcnt;
  const int32_t* label;
  const uint32_t* toff;
  const int32_t* tid;
  const uint8_t* haslab;
  const uint32_t* kvo;
  const int64_t* vnum;
  const uint8_t* vok;
  uint32_t n_topo, pairs;
  const int32_t* tkey;     // [n_topo] node label key of each topology slot (device memory:
  const uint32_t* tbase;   // runtime-indexed kernel-argument arrays would spill to scratch)
  const uint32_t* tcount;
  // existing-pod table
  uint32_t pcap, pkeys, tcap, rcap, vcap;
  int32_t* ptnode;
  int32_t* ptns;
  uint32_t* ptflags;
  int32_t* ptlab;
  ksg_exist_term* terms;
  int32_t* tpod;
  ksg_req* treq;
  int32_t* tval;
  uint32_t* tcounts;  // [0] pods [1] terms [2] reqs [3] vals [4] overflow flag
  // rest of the default profile
  const uint8_t* nflags;   // [N] KSG_NODE_*
  uint32_t img_words;
  const uint32_t* img;     // [img_words][N]
  uint32_t n_ports;
  int32_t* ports;          // [n_ports][N] used host-port triple counts
  int32_t* pvcuse;         // [PVC ids] pods (bound + assumed) using the claim: NodeInfo PVCRefCounts summed
  int32_t* vlim;           // [limit keys][N] NodeVolumeLimits limit (-1 none)
  int32_t* vatt;           // [limit keys][N] attached unique CSI volumes
  int32_t* vnode;          // [CSI volumes][KSG_VOL_NODES] nodes (local index) the volume is attached to, -1 empty
  int32_t* vref;           // [CSI volumes][KSG_VOL_NODES] pods using it there
  DevTables T;
  // per topology slot, by value for fully unrolled loops (no load): its node
  // label key and its base among the shared-key pairs (-1: one node per value)
  int32_t tkeyv[KSG_MAX_TOPO];
  int32_t nubv[KSG_MAX_TOPO];
};

struct DevProfile {
  int n;
  int plugins[KSG_MAX_PLUGINS];
  int64_t weight[KSG_MAX_PLUGINS];
  int has_ext;  // any plugin with ScoreExtensions (or PTS)
  int fit_strategy, fit_n, ba_n, rtc_n;
  int fit_res[KSG_MAX_SCORE_RES];
  int64_t fit_w[KSG_MAX_SCORE_RES];
  int ba_res[KSG_MAX_SCORE_RES];
  int64_t rtc_util[KSG_MAX_RTC], rtc_score[KSG_MAX_RTC];
  int64_t ipa_hard_weight;
  int ipa_ignore_existing_pref;
  uint64_t seed;
  int pos_fit, pos_ba;  // profile positions (-1 absent)
  int pos_taint, pos_na;
  int64_t w_fit, w_ba, w_taint, w_na;  // their weights (0 absent)
  // copies in device memory for run-time indexed loops (kernel-argument arrays
  // indexed at run time would be copied to scratch)
  const int32_t* fit_res_d;
  const int64_t* fit_w_d;
  const int32_t* ba_res_d;
};

struct DevScratch {
  int32_t* cnt;        // [KSG_MAX_TSC][N]
  int32_t* hist_f;     // [pairs] PTS filter TpPairToMatchNum
  uint8_t* present_f;  // [pairs] pair registered
  int32_t* hist_s;     // [pairs] PTS score TopologyPairToPodCounts
  uint8_t* reg;        // [pairs] pair registered by a filtered node
  int32_t* ipa_aff;    // [pairs]
  int32_t* ipa_anti;   // [pairs]
  int32_t* ipa_exist;  // [pairs]
  int64_t* ipa_score;  // [pairs]
  int32_t* pts_min;    // [KSG_MAX_TOPO]
  int32_t* pts_dom;    // [KSG_MAX_TOPO]
  uint32_t* exist_any; // [1] bitmask over topology slots with existing anti counts
};

struct DevOut {
  uint32_t* filter;  // [N]
  int32_t* score;    // [n_plugins][N]
  int32_t* total;    // [N]
  ksg_pod_summary* sum;
  uint32_t* arrive;  // block arrivals of the cycle's last kernel (its last block commits), or null
  int mode;          // commit mode (k_commit)
  int32_t* prow;     // existing-pod table row of the assumed pod
};

// Programs are read through the constant address space: they never change
// during a launch (uploads and k_place_program run between launches), so every
// wave-uniform read of a header field is a scalar load (s_load, scalar cache),
// whatever stores, atomics, fences or asm memory clobbers the kernel holds.
// Through a generic pointer the compiler could prove that only for __restrict__
// kernel arguments with no clobber on the path: the persistent kernels read
// their programs with vector loads, each one waited for (round 5).
// (the host pass of this single-source file parses these device functions but
// never emits them: there the qualifier is left out, which its semantic checks need)
#if defined(__HIP_DEVICE_COMPILE__)
#define KSG_CONST __attribute__((address_space(4)))
#else
#define KSG_CONST
#endif
template <class T>
using cptr = const KSG_CONST T*;
using PH = cptr<ksg_prog>;
struct ProgView {
  PH h;
  cptr<int32_t> i32;
  cptr<uint32_t> u32;
  cptr<ksg_req> req;
  cptr<ksg_sel> sel;
  cptr<ksg_aterm> at;
  cptr<ksg_exist_term> et;
  cptr<ksg_vchk> vchk;
  cptr<ksg_freq> fq;
};

__device__ __forceinline__ ProgView view(const uint8_t* pg) {
  ProgView v;
  const KSG_CONST uint8_t* p = (const KSG_CONST uint8_t*)pg;
  v.h = (PH)p;
  v.i32 = (cptr<int32_t>)(p + v.h->off_i32);
  v.u32 = (cptr<uint32_t>)(p + v.h->off_u32);
  v.req = (cptr<ksg_req>)(p + v.h->off_req);
  v.sel = (cptr<ksg_sel>)(p + v.h->off_sel);
  v.at = (cptr<ksg_aterm>)(p + v.h->off_aterm);
  v.et = (cptr<ksg_exist_term>)(p + v.h->off_eterm);
  v.vchk = (cptr<ksg_vchk>)(v.i32 + v.h->vchk_off);
  v.fq = (cptr<ksg_freq>)(p + v.h->off_freq);
  return v;
}

// Scalar-cache warm-up: every 64-B line of [p + O, p + END) is requested at
// once by independent scalar loads, and one wait covers them all.  Without it
// the kernel's first scalar reads of its (1.5 KB) arguments and of the pod's
// program header arrive one dependent cache miss at a time.  Loads only (no
// scalar stores).  The loads land in one compiler-allocated SGPR threaded
// through every statement as an in/out operand up to the wait (warm_wait), so
// the register holds nothing else while they are in flight.
template <int O, int END>
struct KWarm {
  static __device__ __forceinline__ void run(const void* p, uint32_t& t) {
    asm volatile("s_load_dword %0, %1, %2" : "+s"(t) : "s"(p), "i"(O));
    KWarm<O + 64, END>::run(p, t);
  }
};
template <int END>
struct KWarm<END, END> {
  static __device__ __forceinline__ void run(const void*, uint32_t&) {}
};
__device__ __forceinline__ void warm_wait(uint32_t& t) { asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(t)::"memory"); }
// NodeAffinity PreScore error (an invalid preferred term; the host sets the
// flag only when the profile has NodeAffinity): the cycle ends in Error once
// PreScore runs, i.e. with more than one feasible node (schedule_one.go).
__device__ __forceinline__ bool na_prescore_error(uint32_t flags, int32_t feasible) {
  return (flags & KPF_NA_PREF_ERROR) && feasible > 1;
}

// ----------------------------------------------------------------- helpers
__device__ __forceinline__ bool in_list(int32_t v, const int32_t* vals, int cnt) {
  for (int i = 0; i < cnt; ++i)
    if (vals[i] == v) return true;
  return false;
}

// labels.Requirement.Matches over an interned label set (vid < 0: key absent).
template <class VidF>
__device__ __forceinline__ bool sel_eval(const ksg_sel& s, const ksg_req* reqs, const int32_t* vals, VidF vid_of) {
  if (s.kind == 0) return false;
  for (int i = 0; i < s.req_cnt; ++i) {
    const ksg_req& r = reqs[s.req_off + i];
    int32_t v = vid_of(r.key);
    bool ok;
    switch (r.op) {
      case KR_IN: ok = v >= 0 && in_list(v, vals + r.val_off, r.nvals); break;
      case KR_NOT_IN: ok = v < 0 || !in_list(v, vals + r.val_off, r.nvals); break;
      case KR_EXISTS: ok = v >= 0; break;
      case KR_NOT_EXISTS: ok = v < 0; break;
      default: ok = false;
    }
    if (!ok) return false;
  }
  return true;
}

__device__ __forceinline__ int32_t node_vid(const DevCluster& C, int32_t key, uint32_t n) {
  return (key >= 0 && (uint32_t)key < C.K) ? C.label[(size_t)key * C.N + n] : -1;
}

// node selector requirement incl. Gt/Lt (numeric view of the value) and
// matchFields metadata.name (KR_NAME_EQ / KR_NAME_NE on the global node index).
// v: the node's value id for r.key (loaded by the caller, so that the label
// loads of a whole selector are in flight together instead of one per
// requirement behind the previous one's compare).
__device__ __forceinline__ bool node_req_v(const DevCluster& C, const ksg_req& r, const int32_t* vals, uint32_t n,
                                           int32_t v) {
  if (r.op == KR_NAME_EQ) return (int64_t)(C.goff + n) == r.num;
  if (r.op == KR_NAME_NE) return (int64_t)(C.goff + n) != r.num;
  switch (r.op) {
    case KR_IN: return v >= 0 && in_list(v, vals + r.val_off, r.nvals);
    case KR_NOT_IN: return v < 0 || !in_list(v, vals + r.val_off, r.nvals);
    case KR_EXISTS: return v >= 0;
    case KR_NOT_EXISTS: return v < 0;
    case KR_GT:
    case KR_LT: {
      if (v < 0) return false;
      uint32_t o = C.kvo[r.key] + (uint32_t)v;
      if (!C.vok[o]) return false;
      return r.op == KR_GT ? C.vnum[o] > r.num : C.vnum[o] < r.num;
    }
    default: return false;
  }
}

__device__ __forceinline__ bool node_req(const DevCluster& C, const ksg_req& r, const int32_t* vals, uint32_t n) {
  return node_req_v(C, r, vals, n, node_vid(C, r.key, n));
}

// A flattened requirement (ksg_freq) on local node n, without branches on the
// (wave-uniform) mode: one 16-byte scalar load of the entry, the node's value
// for the key, the mask bit, the name compare, a select.
__device__ __forceinline__ bool freq_match(const DevCluster& C, const ksg_freq* fp, uint32_t n) {
  const uint4 w = *reinterpret_cast<const uint4*>(fp);
  const int32_t key = (int32_t)w.x, mode = (int32_t)w.y;
  const uint64_t arg = (uint64_t)w.z | ((uint64_t)w.w << 32);
  const bool kok = key >= 0 && (uint32_t)key < C.K;
  const int32_t v = C.label[(size_t)(kok ? (uint32_t)key : 0u) * C.N + n];  // (key 0's column when unknown)
  const bool inset = kok && v >= 0 && ((arg >> ((uint32_t)v & 63u)) & 1ull);
  const bool name = (uint64_t)(C.goff + n) == arg;
  const bool r = mode <= KFR_NONE ? inset : name;
  return mode == KFR_FALSE ? false : (r != (mode == KFR_NONE || mode == KFR_NAME_NE));
}
__device__ bool node_sel(const DevCluster& C, const ProgView& V, const ksg_sel& s, uint32_t n) {
  if (s.kind == 0) return false;
  if (V.h->flags & KPF_FLAT_NA) {  // (a wave-uniform loop: the entries stay scalar loads)
    bool ok = true;
    for (int i = 0; i < s.req_cnt; ++i) {
      ok &= freq_match(C, V.fq + s.req_off + i, n);
      if (!__ballot(ok)) break;
    }
    return ok;
  }
  for (int i = 0; i < s.req_cnt; ++i)
    if (!node_req(C, V.req[s.req_off + i], V.i32, n)) return false;
  return true;
}

// nodeaffinity.RequiredNodeAffinity.Match
__device__ bool required_na(const DevCluster& C, const ProgView& V, uint32_t n) {
  uint32_t f = V.h->flags;
  if (f & KPF_FLAT_NA) {  // wave-uniform loops (no per-lane early exit): scalar program reads
    bool ok = !(f & KPF_HAS_NODE_SEL) || node_sel(C, V, V.h->node_sel, n);
    if ((f & KPF_HAS_REQ_NA) && __ballot(ok)) {
      bool any = false;
      for (int t = 0; t < V.h->n_req_terms; ++t) {
        any |= node_sel(C, V, V.sel[V.h->req_terms_off + t], n);
        if (!__ballot(ok && !any)) break;
      }
      ok = ok && any;
    }
    return ok;
  }
  if ((f & KPF_HAS_NODE_SEL) && !node_sel(C, V, V.h->node_sel, n)) return false;
  if (f & KPF_HAS_REQ_NA) {
    for (int t = 0; t < V.h->n_req_terms; ++t)
      if (node_sel(C, V, V.sel[V.h->req_terms_off + t], n)) return true;
    return false;
  }
  return true;
}

__device__ __forceinline__ bool bit(const uint32_t* w, int nw, int32_t i) {
  return i >= 0 && (i >> 5) < nw && ((w[i >> 5] >> (i & 31)) & 1u);
}

// first untolerated NoSchedule/NoExecute taint in node.spec.taints order, or -1
__device__ __forceinline__ int32_t untolerated_taint(const DevCluster& C, const ProgView& V, uint32_t n) {
  const uint32_t* hard = V.u32 + V.h->taint_hard_off;
  for (uint32_t i = C.toff[n]; i < C.toff[n + 1]; ++i) {
    int32_t t = C.tid[i];
    if (bit(hard, V.h->taint_words, t)) return t;
  }
  return -1;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// highest total, then smallest h20, then largest node index.
__device__ __forceinline__ uint64_t pack_key(int64_t total, uint64_t seed, int32_t qidx, uint32_t gnode) {
  uint64_t h20 = splitmix64(seed ^ ((uint64_t)(uint32_t)qidx * 0x9E3779B97F4A7C15ull) ^ (uint64_t)gnode) >> 44;
  return ((uint64_t)total << 40) | ((0xFFFFFull - h20) << 20) | (uint64_t)gnode;
}

// Wave-wide reductions on DPP (ockl wfred): a 64-bit value is reduced as its
// high word, then the low word among the lanes holding the winning high word.
// (A 64-bit __shfl_xor lowers to two dependent ds_bpermute round trips per
// step through the LDS pipe.)  All reductions cover the active lanes.
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  uint32_t hi = (uint32_t)(v >> 32);
  uint32_t mh = __ockl_wfred_max_u32(hi);
  uint32_t ml = __ockl_wfred_max_u32(hi == mh ? (uint32_t)v : 0u);
  return ((uint64_t)mh << 32) | ml;
}
__device__ __forceinline__ uint64_t wave_max(uint64_t v) { return wave_max_u64(v); }
__device__ __forceinline__ int64_t wave_max(int64_t v) {  // order-preserving map to unsigned
  return (int64_t)(wave_max_u64((uint64_t)v ^ 0x8000000000000000ull) ^ 0x8000000000000000ull);
}
__device__ __forceinline__ int64_t wave_min(int64_t v) { return ~wave_max((int64_t)~v); }
__device__ __forceinline__ int32_t wave_min(int32_t v) { return __ockl_wfred_min_i32(v); }
__device__ __forceinline__ int32_t wave_max(int32_t v) { return __ockl_wfred_max_i32(v); }
__device__ __forceinline__ int32_t wave_sum(int32_t v) { return __ockl_wfred_add_i32(v); }
__device__ __noinline__ int64_t div_i64_slow(int64_t x, int64_t a) { return x / a; }
// floor(x / a) for 0 <= x, a > 0 — exact.  32-bit operands use the hardware
// 32-bit divide; otherwise an estimate from one v_rcp_f64 (relative error
// ~2^-50, so |estimate - quotient| < 1 for x < 2^52 with small quotients) is
// corrected with exact 64-bit products.  Only BalancedAllocation's fractions
// need an IEEE-rounded f64 division; integer quotients never do.
__device__ __forceinline__ int64_t div_small(int64_t x, int64_t a) {
  if ((uint64_t)x <= 0xFFFFFFFFull && (uint64_t)a <= 0xFFFFFFFFull) return (int64_t)((uint32_t)x / (uint32_t)a);
  if (x >= ((int64_t)1 << 52)) return div_i64_slow(x, a);
  int64_t q = (int64_t)((double)x * __builtin_amdgcn_rcp((double)a));
  if (q < 0) q = 0;
  if (q * a > x) q--;
  else if ((q + 1) * a <= x) q++;
  return q;
}
// floor(x / d) for x < 2^27, 1 <= d, quotient <= 128: one f32 reciprocal
// estimate (error well below 1) and one exact correction either way.
__device__ __forceinline__ uint32_t udiv_small(uint32_t x, uint32_t d) {
  uint32_t q = (uint32_t)((float)x * __builtin_amdgcn_rcpf((float)d));
  const int32_t r = (int32_t)(x - q * d);
  return r < 0 ? q - 1 : ((uint32_t)r >= d ? q + 1 : q);
}
__device__ __forceinline__ bool lane0() { return (threadIdx.x & 63) == 0; }

// Go math.Log restated (oracle/ksg_oracle.cpp go_log); no contraction.
__device__ double go_log(double x) {
#pragma clang fp contract(off)
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
               L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
               L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
               L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (!(x > 0)) return x == 0 ? -INFINITY : NAN;
  if (isinf(x)) return x;
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < 0.70710678118654752440) {  // Sqrt2/2
    f1 = __dmul_rn(f1, 2.0);
    ki--;
  }
  double f = __dsub_rn(f1, 1.0);
  double k = (double)ki;
  double s = __ddiv_rn(f, __dadd_rn(2.0, f));
  double s2 = __dmul_rn(s, s);
  double s4 = __dmul_rn(s2, s2);
  double t1 = __dmul_rn(s2, __dadd_rn(L1, __dmul_rn(s4, __dadd_rn(L3, __dmul_rn(s4, __dadd_rn(L5, __dmul_rn(s4, L7)))))));
  double t2 = __dmul_rn(s4, __dadd_rn(L2, __dmul_rn(s4, __dadd_rn(L4, __dmul_rn(s4, L6)))));
  double R = __dadd_rn(t1, t2);
  double hfsq = __dmul_rn(__dmul_rn(0.5, f), f);
  return __dsub_rn(__dmul_rn(k, Ln2Hi),
                   __dsub_rn(__dsub_rn(hfsq, __dadd_rn(__dmul_rn(s, __dadd_rn(hfsq, R)), __dmul_rn(k, Ln2Lo))), f));
}

// ----------------------------------------------------------------- plugins (per node)
// NodeResourcesFit Filter (fit.go fitsRequest): reason bits, 0 = fits.
// NodeUnschedulable Filter (node_unschedulable.go): a cordoned node fails unless the
// pod tolerates node.kubernetes.io/unschedulable:NoSchedule (decided on the host).
__device__ __forceinline__ bool unsched_fails(const DevCluster& C, const ProgView& V, uint32_t n) {
  return (C.nflags[n] & KSG_NODE_UNSCHEDULABLE) && !(V.h->flags & KPF_TOL_UNSCHED);
}
// NodeName Filter (node_name.go Fits): empty spec.nodeName or this node's name.
__device__ __forceinline__ bool nodename_fails(const DevCluster& C, const ProgView& V, uint32_t n) {
  const int32_t g = V.h->node_name_gid;
  return g != -1 && (g < 0 || (uint32_t)g != C.goff + n);
}
// NodePorts Filter (fitsPorts -> HostPortInfo.CheckConflict): the host folds every
// wanted (ip, protocol, port) into the used-port triples that conflict with it.
__device__ __forceinline__ bool ports_fail(const DevCluster& C, const ProgView& V, uint32_t n) {
  const int32_t k = V.h->n_port_check, o = V.h->port_check_off;
  for (int i = 0; i < k; ++i)
    if (C.ports[(size_t)V.i32[o + i] * C.N + n] > 0) return true;
  return false;
}
// ImageLocality Score (image_locality.go): sum of the containers' scaledImageScore
// over images the node lists, clamped to [minThreshold, maxThreshold], scaled to 0..100.
__device__ __forceinline__ int64_t image_score(const DevCluster& C, const ProgView& V, uint32_t n) {
  const ksg_prog* h = V.h;
  const int64_t kMin = 23ll << 20, kMax = h->img_max_threshold;
  int64_t sum = 0;
  for (int i = 0; i < h->n_img; ++i) {
    const int32_t id = h->img_id[i];
    if ((C.img[(size_t)(id >> 5) * C.N + n] >> (id & 31)) & 1u) sum += h->img_scaled[i];
  }
  sum = sum < kMin ? kMin : (sum > kMax ? kMax : sum);
  return 100 * (sum - kMin) / (kMax - kMin);
}

// Volume plugins of the run at device position pos (KP_VOLUMES): the pod's checks
// for that position, grouped by plugin in profile order (VolumeRestrictions'
// ReadWriteOncePod conflict, VolumeBinding's PV node affinity / provisioning
// topology / selected node, VolumeZone's PV zone labels, pod-uniform verdicts;
// compiled by the host from the PreFilter state, host.cpp compile_volumes).
// 0: every plugin passes; else (plugin index in the run << 16) | reason bits.
__device__ uint32_t volume_filter(const DevCluster& C, const ProgView& V, int pos, uint32_t n) {
  const int nv = V.h->n_vchk;
  int sub = -1;
  uint32_t bits = 0;
  for (int i = 0; i < nv; ++i) {
    const ksg_vchk c = V.vchk[i];
    if (c.dpos != pos) continue;
    if (c.sub != sub) {
      if (bits) break;
      sub = c.sub;
    }
    if (bits & (uint32_t)c.unless) continue;
    bool fail = true;
    if (c.kind == KSG_VCHK_SELS) {
      for (int t = 0; t < c.cnt && fail; ++t) fail = !node_sel(C, V, V.sel[c.off + t], n);
    } else if (c.kind == KSG_VCHK_USED) {
      fail = false;
      for (int t = 0; t < c.cnt && !fail; ++t) fail = C.pvcuse[V.i32[c.off + t]] > 0;
    } else if (c.kind == KSG_VCHK_LIMIT) {  // csi.go Filter: per limit key, attached + new > limit
      fail = false;
      for (int t = 0; t < c.cnt && !fail; ++t) {
        const int32_t key = V.i32[c.off + 2 * t + 1];
        bool first = true;  // count each key once, at its first pair
        for (int u = 0; u < t; ++u) first &= V.i32[c.off + 2 * u + 1] != key;
        if (!first) continue;
        const int32_t lim = C.vlim[(size_t)key * C.N + n];
        if (lim < 0) continue;
        int32_t fresh = 0;
        for (int u = t; u < c.cnt; ++u) {
          if (V.i32[c.off + 2 * u + 1] != key) continue;
          const int32_t* vn = C.vnode + (size_t)V.i32[c.off + 2 * u] * KSG_VOL_NODES;
          bool on = false;
          for (int k = 0; k < KSG_VOL_NODES; ++k) on |= vn[k] == (int32_t)n;
          fresh += on ? 0 : 1;
        }
        fail = fresh > 0 && C.vatt[(size_t)key * C.N + n] + fresh > lim;
      }
    }
    if (fail) bits |= (uint32_t)c.bits;
  }
  return bits ? ((uint32_t)sub << 16) | bits : 0u;
}

__device__ __forceinline__ uint32_t fit_filter(const DevCluster& C, const ProgView& V, uint32_t n) {
  uint32_t bits = 0;
  if (C.podcnt[n] + 1 > C.allowed[n]) bits |= KSG_FIT_TOO_MANY_PODS;
  if (V.h->flags & KPF_ZERO_REQUEST) return bits;
  for (uint32_t r = 0; r < C.R; ++r) {
    int64_t q = V.h->req[r];
    if (q <= 0) continue;  // cpu/mem/eph: "> 0" guard; scalars: zero skipped
    if (q > C.alloc[(size_t)r * C.N + n] - C.req[(size_t)r * C.N + n]) bits |= 1u << (1 + r);
  }
  return bits;
}

// resourceAllocationScorer.calculateResourceAllocatableRequest
__device__ __forceinline__ void alloc_req(const DevCluster& C, uint32_t n, int res, int64_t pod_req, bool use_requested,
                                          int64_t& a, int64_t& q) {
  if (res < 0 || (res >= KSG_RES_EPH + 1 && pod_req == 0)) { a = 0; q = 0; return; }  // unknown / scalar not requested
  a = C.alloc[(size_t)res * C.N + n];
  if (res == KSG_RES_CPU) q = (use_requested ? C.req[n] : C.nzc[n]) + pod_req;
  else if (res == KSG_RES_MEM) q = (use_requested ? C.req[(size_t)C.N + n] : C.nzm[n]) + pod_req;
  else q = C.req[(size_t)res * C.N + n] + pod_req;
}

__device__ int64_t rtc_fn(const DevProfile& F, int64_t p) {
  for (int i = 0; i < F.rtc_n; ++i) {
    if (p <= F.rtc_util[i]) {
      if (i == 0) return F.rtc_score[0];
      return F.rtc_score[i - 1] + (F.rtc_score[i] - F.rtc_score[i - 1]) * (p - F.rtc_util[i - 1]) /
                                      (F.rtc_util[i] - F.rtc_util[i - 1]);
    }
  }
  return F.rtc_score[F.rtc_n - 1];
}

__device__ int64_t fit_score(const DevCluster& C, const DevProfile& F, const ProgView& V, uint32_t n) {
  int64_t ns = 0, ws = 0;
#pragma unroll 1
  for (int i = 0; i < F.fit_n; ++i) {
    int64_t a, q;
    alloc_req(C, n, F.fit_res[i], V.h->fit_score_req[i], false, a, q);
    if (a == 0) continue;
    int64_t s;
    if (F.fit_strategy == 2) {
      s = q > a ? rtc_fn(F, 100) : rtc_fn(F, q * 100 / a);
      if (s <= 0) continue;
    } else if (F.fit_strategy == 1) {
      s = div_small((q > a ? a : q) * 100, a);
    } else {
      s = q > a ? 0 : div_small((a - q) * 100, a);
    }
    ns += s * F.fit_w[i];
    ws += F.fit_w[i];
  }
  if (ws == 0) return 0;
  if (F.fit_strategy == 2) return (int64_t)round((double)ns / (double)ws);
  return div_small(ns, ws);
}

__device__ int64_t ba_score(const DevCluster& C, const DevProfile& F, const ProgView& V, uint32_t n) {
#pragma clang fp contract(off)
  int m = 0;
  double total = 0, f0 = 0, f1 = 0, sd = 0.0;
#pragma unroll 1
  for (int i = 0; i < F.ba_n; ++i) {
    int64_t a, q;
    alloc_req(C, n, F.ba_res[i], V.h->ba_req[i], true, a, q);
    if (a == 0) continue;
    double f = (double)q / (double)a;
    if (f > 1) f = 1;
    total = total + f;
    if (m == 0) f0 = f;
    else if (m == 1) f1 = f;
    m++;
  }
  if (m == 2) {
    sd = fabs((f0 - f1) / 2);
  } else if (m > 2) {
    double mean = total / (double)m;
    double sum = 0;
#pragma unroll 1
    for (int i = 0; i < F.ba_n; ++i) {
      int64_t a, q;
      alloc_req(C, n, F.ba_res[i], V.h->ba_req[i], true, a, q);
      if (a == 0) continue;
      double f = (double)q / (double)a;
      if (f > 1) f = 1;
      sum = sum + (f - mean) * (f - mean);
    }
    sd = sqrt(sum / (double)m);
  }
  return (int64_t)((1 - sd) * 100.0);
}

__device__ __forceinline__ int64_t taint_score(const DevCluster& C, const ProgView& V, uint32_t n) {
  const uint32_t* pref = V.u32 + V.h->taint_pref_off;
  int64_t c = 0;
  for (uint32_t i = C.toff[n]; i < C.toff[n + 1]; ++i)
    if (bit(pref, V.h->taint_words, C.tid[i])) c++;
  return c;
}

__device__ __forceinline__ int64_t na_score(const DevCluster& C, const ProgView& V, uint32_t n) {
  int64_t s = 0;
  for (int t = 0; t < V.h->n_pref_terms; ++t)
    if (node_sel(C, V, V.sel[V.h->pref_terms_off + t], n)) s += V.i32[V.h->pref_w_off + t];
  return s;
}

__device__ __forceinline__ bool pts_has_keys(const DevCluster& C, const ProgView& V, int c0, int c1, uint32_t n) {
  for (int c = c0; c < c1; ++c)
    if (node_vid(C, V.h->tsc[c].topo_key, n) < 0) return false;
  return true;
}

// PodTopologySpread Filter
// Topology-slot value ids of this thread's node, loaded once per kernel into
// LDS (tv(s) = node_vid(C, C.tkey[s], n)): the cycle's histogram lookups then
// depend on one LDS read instead of a label load each.
struct SlotVids {
  const int32_t* base;  // [KSG_MAX_TOPO][kBlock] in LDS, this thread's column
  __device__ __forceinline__ int32_t operator()(int s) const { return base[s * kBlock]; }
};
__device__ __forceinline__ void load_slot_vids(const DevCluster& C, uint32_t n, bool active, int32_t* lds) {
  const uint32_t nt = C.n_topo < KSG_MAX_TOPO ? C.n_topo : KSG_MAX_TOPO;
  int32_t v[KSG_MAX_TOPO];
#pragma unroll
  for (int s = 0; s < KSG_MAX_TOPO; ++s) v[s] = ((uint32_t)s < nt && active) ? node_vid(C, C.tkeyv[s], n) : -1;
#pragma unroll
  for (int s = 0; s < KSG_MAX_TOPO; ++s)
    if ((uint32_t)s < nt) lds[s * kBlock + threadIdx.x] = v[s];
}
// pts_filter with the slot vids preloaded: every histogram load of the pod's
// constraints is issued before the first check (same verdict and order)
__device__ __forceinline__ int pts_filter_v(const DevCluster& C, const DevScratch& S, const ProgView& V,
                                            const SlotVids& tv, bool& error) {
  const int nf = V.h->n_tsc_filter;
  int32_t m[KSG_MAX_TSC];
#pragma unroll
  for (int c = 0; c < KSG_MAX_TSC; ++c) {
    m[c] = 0;
    if (c < nf) {
      const int32_t v = tv(V.h->tsc[c].topo);
      if (v >= 0) m[c] = S.hist_f[C.tbase[V.h->tsc[c].topo] + v];
    }
  }
  int r = 0;
  bool done = false;
#pragma unroll
  for (int c = 0; c < KSG_MAX_TSC; ++c) {
    if (c < nf && !done) {
      const ksg_tsc& t = V.h->tsc[c];
      const int32_t dom = S.pts_dom[t.topo];
      const int64_t mn = dom < t.min_domains ? 0 : S.pts_min[t.topo];
      if (tv(t.topo) < 0) { r = 1 + KSG_PTS_MISSING_LABEL; done = true; }
      else if (dom == 0) { error = true; done = true; }  // minMatchNum: no domains for key -> Error status
      else if ((int64_t)m[c] + t.self_match - mn > t.max_skew) { r = 1 + KSG_PTS_SKEW; done = true; }
    }
  }
  return r;
}
__device__ __forceinline__ int pts_filter(const DevCluster& C, const DevScratch& S, const ProgView& V, uint32_t n,
                                          bool& error) {
  for (int c = 0; c < V.h->n_tsc_filter; ++c) {
    const ksg_tsc& t = V.h->tsc[c];
    int32_t v = node_vid(C, t.topo_key, n);
    if (v < 0) return 1 + KSG_PTS_MISSING_LABEL;
    int32_t dom = S.pts_dom[t.topo];
    if (dom == 0) { error = true; return 0; }  // minMatchNum: no domains for key -> Error status
    int64_t mn = dom < t.min_domains ? 0 : S.pts_min[t.topo];
    int64_t match = S.hist_f[C.tbase[t.topo] + v];
    if (match + t.self_match - mn > t.max_skew) return 1 + KSG_PTS_SKEW;
  }
  return 0;
}

// InterPodAffinity Filter
__device__ __forceinline__ int ipa_filter(const DevCluster& C, const DevScratch& S, const ProgView& V, uint32_t n,
                                          uint32_t ipa_flags, uint32_t exist_any) {
  const ksg_prog* h = V.h;
  const ksg_aterm* aff = V.at + h->aterm_off;
  const ksg_aterm* anti = aff + h->n_req_aff;
  bool pods_exist = true;
  for (int i = 0; i < h->n_req_aff; ++i) {
    int32_t v = node_vid(C, aff[i].topo_key, n);
    if (v < 0) return 1 + KSG_IPA_AFFINITY;
    if (S.ipa_aff[C.tbase[aff[i].topo] + v] <= 0) pods_exist = false;
  }
  if (!pods_exist && !(!(ipa_flags & 1u) && h->self_matches_all)) return 1 + KSG_IPA_AFFINITY;
  if (ipa_flags & 2u)
    for (int i = 0; i < h->n_req_anti; ++i) {
      int32_t v = node_vid(C, anti[i].topo_key, n);
      if (v >= 0 && S.ipa_anti[C.tbase[anti[i].topo] + v] > 0) return 1 + KSG_IPA_ANTI_AFFINITY;
    }
  if (exist_any)
    for (uint32_t s = 0; s < C.n_topo; ++s) {
      if (!((exist_any >> s) & 1u)) continue;
      int32_t v = node_vid(C, C.tkey[s], n);
      if (v >= 0 && S.ipa_exist[C.tbase[s] + v] > 0) return 1 + KSG_IPA_EXISTING_ANTI;
    }
  return 0;
}

__device__ __forceinline__ int ipa_filter_v(const DevCluster& C, const DevScratch& S, const ProgView& V,
                                            const SlotVids& tv, uint32_t ipa_flags, uint32_t exist_any) {
  const ksg_prog* h = V.h;
  const ksg_aterm* aff = V.at + h->aterm_off;
  const ksg_aterm* anti = aff + h->n_req_aff;
  // existing pods' anti-affinity per slot: loaded up front (no early exit in between)
  int32_t ex[KSG_MAX_TOPO];
#pragma unroll
  for (int s = 0; s < KSG_MAX_TOPO; ++s) {
    ex[s] = 0;
    if ((exist_any >> s) & 1u) {
      const int32_t v = tv(s);
      if (v >= 0) ex[s] = S.ipa_exist[C.tbase[s] + v];
    }
  }
  bool pods_exist = true;
  for (int i = 0; i < h->n_req_aff; ++i) {
    int32_t v = tv(aff[i].topo);
    if (v < 0) return 1 + KSG_IPA_AFFINITY;
    if (S.ipa_aff[C.tbase[aff[i].topo] + v] <= 0) pods_exist = false;
  }
  if (!pods_exist && !(!(ipa_flags & 1u) && h->self_matches_all)) return 1 + KSG_IPA_AFFINITY;
  if (ipa_flags & 2u)
    for (int i = 0; i < h->n_req_anti; ++i) {
      int32_t v = tv(anti[i].topo);
      if (v >= 0 && S.ipa_anti[C.tbase[anti[i].topo] + v] > 0) return 1 + KSG_IPA_ANTI_AFFINITY;
    }
  bool hit = false;
#pragma unroll
  for (int s = 0; s < KSG_MAX_TOPO; ++s) hit |= ex[s] > 0;
  return hit ? 1 + KSG_IPA_EXISTING_ANTI : 0;
}
__device__ __forceinline__ int64_t ipa_score_v(const DevCluster& C, const DevScratch& S, const SlotVids& tv) {
  const uint32_t nt = C.n_topo < KSG_MAX_TOPO ? C.n_topo : KSG_MAX_TOPO;
  int64_t s = 0;
#pragma unroll
  for (int t = 0; t < KSG_MAX_TOPO; ++t) {
    if ((uint32_t)t >= nt) break;
    const int32_t v = tv(t);
    if (v >= 0) s += S.ipa_score[C.tbase[t] + v];
  }
  return s;
}
__device__ __forceinline__ int64_t ipa_score(const DevCluster& C, const DevScratch& S, uint32_t n) {
  int64_t s = 0;
  for (uint32_t t = 0; t < C.n_topo; ++t) {
    int32_t v = node_vid(C, C.tkey[t], n);
    if (v >= 0) s += S.ipa_score[C.tbase[t] + v];
  }
  return s;
}

// ----------------------------------------------------------------- kernels
__global__ void k_init_summaries(ksg_pod_summary* sum, uint32_t count, DevProfile F) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  ksg_pod_summary s = {};
  s.selected = -1;
  for (int p = 0; p < KSG_MAX_PLUGINS; ++p) {
    s.max_score[p] = (p < F.n && F.plugins[p] == KP_IPA) ? INT64_MIN : 0;
    s.min_score[p] = INT64_MAX;
  }
  sum[i] = s;
}

// append_program's placement of one staged [PodLite | program] block.
__global__ void k_place_program(const uint8_t* __restrict__ src, uint32_t bytes, uint8_t* dst, uint64_t* off_slot,
                                uint64_t off, void* plite_slot, int32_t* prow_slot, int32_t row, ksg_pod_summary* sum,
                                DevProfile F);

__global__ void k_begin(DevCluster C, DevScratch S, const uint8_t* __restrict__ prog) {
  ProgView V = view(prog);
  uint32_t ntsc = (uint32_t)(V.h->n_tsc_filter + V.h->n_tsc_score);
  size_t cnt_n = (size_t)ntsc * C.N;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt_n || i < C.pairs; i += stride) {
    if (i < cnt_n) S.cnt[i] = 0;
    if (i < C.pairs) {
      S.hist_f[i] = 0; S.present_f[i] = 0; S.hist_s[i] = 0; S.reg[i] = 0;
      S.ipa_aff[i] = 0; S.ipa_anti[i] = 0; S.ipa_exist[i] = 0; S.ipa_score[i] = 0;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < KSG_MAX_TOPO) {
    S.pts_min[threadIdx.x] = 0x7FFFFFFF;
    S.pts_dom[threadIdx.x] = 0;
    if (threadIdx.x == 0) S.exist_any[0] = 0;
  }
}

// existing pods x (PTS selectors, IPA incoming required terms, IPA incoming preferred terms)
__global__ void k_scan_pods(DevCluster C, DevProfile F, DevScratch S, DevOut O, const uint8_t* __restrict__ prog) {
  ProgView V = view(prog);
  const ksg_prog* h = V.h;
  uint32_t np = C.tcounts[0];
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t aff_hit = 0;
  if (p < np && !(C.ptflags[p] & KEF_DELETED)) {
    int32_t node = C.ptnode[p];
    int32_t ns = C.ptns[p];
    uint32_t fl = C.ptflags[p];
    auto vid = [&](int32_t k) -> int32_t {
      return (k >= 0 && (uint32_t)k < C.pkeys) ? C.ptlab[(size_t)k * C.pcap + p] : -1;
    };
    // PTS countPodsMatchSelector (Empty() selector counts nothing)
    int ntsc = h->n_tsc_filter + h->n_tsc_score;
    if (!(fl & KEF_TERMINATING) && ns == h->ns_id)
      for (int c = 0; c < ntsc; ++c) {
        const ksg_sel& s = h->tsc[c].sel;
        if (s.kind == 1 && s.req_cnt > 0 && sel_eval(s, V.req, V.i32, vid)) atomicAdd(&S.cnt[(size_t)c * C.N + node], 1);
      }
    const ksg_aterm* aff = V.at + h->aterm_off;
    const ksg_aterm* anti = aff + h->n_req_aff;
    const ksg_aterm* paff = anti + h->n_req_anti;  // preferred affinity, then preferred anti
    auto term_ok = [&](const ksg_aterm& t) {
      return (t.ns_all || in_list(ns, V.i32 + t.ns_off, t.ns_cnt)) && sel_eval(t.sel, V.req, V.i32, vid);
    };
    if (h->n_req_aff > 0) {
      bool all = true;
      for (int i = 0; i < h->n_req_aff && all; ++i) all = term_ok(aff[i]);
      if (all)
        for (int i = 0; i < h->n_req_aff; ++i) {
          int32_t v = node_vid(C, aff[i].topo_key, node);
          if (v >= 0) { atomicAdd(&S.ipa_aff[C.tbase[aff[i].topo] + v], 1); aff_hit |= 1u; }
        }
    }
    for (int i = 0; i < h->n_req_anti; ++i)
      if (term_ok(anti[i])) {
        int32_t v = node_vid(C, anti[i].topo_key, node);
        if (v >= 0) { atomicAdd(&S.ipa_anti[C.tbase[anti[i].topo] + v], 1); aff_hit |= 2u; }
      }
    if ((h->flags & KPF_IPA_HAS_CONSTRAINTS) && C.haslab[node]) {
      for (int i = 0; i < h->n_pref_aff + h->n_pref_anti; ++i) {
        const ksg_aterm& t = paff[i];
        if (!term_ok(t)) continue;
        int32_t v = node_vid(C, t.topo_key, node);
        if (v < 0) continue;
        int64_t w = i < h->n_pref_aff ? (int64_t)t.weight : -(int64_t)t.weight;
        atomicAdd((unsigned long long*)&S.ipa_score[C.tbase[t.topo] + v], (unsigned long long)w);
        aff_hit |= 8u;
      }
    }
  }
    uint32_t m = aff_hit;
  for (int o = 32; o > 0; o >>= 1) m |= __shfl_xor(m, o, 64);
  if (lane0() && m) atomicOr(&O.sum->ipa_flags, m);
}

// existing pods' terms x incoming pod (existing anti-affinity counts, IPA score terms)
__global__ void k_scan_terms(DevCluster C, DevProfile F, DevScratch S, DevOut O, const uint8_t* __restrict__ prog) {
  ProgView V = view(prog);
  const ksg_prog* h = V.h;
  uint32_t nt = C.tcounts[1];
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t hit = 0, slots = 0;
  if (t < nt && !(C.ptflags[C.tpod[t]] & KEF_DELETED)) {
    const ksg_exist_term& e = C.terms[t];
    int32_t p = C.tpod[t];
    int32_t node = C.ptnode[p];
    auto vid = [&](int32_t k) -> int32_t {
      return (k >= 0 && k < h->n_pod_label_keys) ? V.i32[h->labels_off + k] : -1;
    };
    bool ns_ok = e.ns_all || in_list(h->ns_id, C.tval + e.ns_off, e.ns_cnt);
    bool score_on = !(F.ipa_ignore_existing_pref && !(h->flags & KPF_IPA_HAS_CONSTRAINTS));
    if (ns_ok && sel_eval(e.sel, C.treq, C.tval, vid)) {
      int32_t v = node_vid(C, e.topo_key, node);
      if (v >= 0) {
        uint32_t pair = C.tbase[e.topo] + v;
        if (e.kind == 1) {
          atomicAdd(&S.ipa_exist[pair], 1);
          slots |= 1u << e.topo;
        } else if (score_on && C.haslab[node]) {
          int64_t w = e.kind == 0 ? (F.ipa_hard_weight > 0 ? F.ipa_hard_weight : 0)
                                  : (e.kind == 2 ? (int64_t)e.weight : -(int64_t)e.weight);
          if (e.kind != 0 || F.ipa_hard_weight > 0) {
            atomicAdd((unsigned long long*)&S.ipa_score[pair], (unsigned long long)w);
            hit |= 8u;
          }
        }
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    hit |= __shfl_xor(hit, o, 64);
    slots |= __shfl_xor(slots, o, 64);
  }
  if (lane0()) {
    if (hit) atomicOr(&O.sum->ipa_flags, hit);
    if (slots) { atomicOr(S.exist_any, slots); atomicOr(&O.sum->ipa_flags, 4u); }
  }
}

// PodTopologySpread PreFilter / PreScore per-node aggregation
__global__ void k_pts_prep(DevCluster C, DevScratch S, const uint8_t* __restrict__ prog) {
  ProgView V = view(prog);
  const ksg_prog* h = V.h;
  uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= C.N) return;
  int nf = h->n_tsc_filter, ns = h->n_tsc_score;
  bool na_ok = true, taint_ok = true;
  bool need_na = false, need_taint = false;
  for (int c = 0; c < nf + ns; ++c) {
    need_na |= h->tsc[c].honor_affinity != 0;
    need_taint |= h->tsc[c].honor_taints != 0;
  }
  if (need_na) na_ok = required_na(C, V, n);
  if (need_taint) taint_ok = untolerated_taint(C, V, n) < 0;
  if (nf > 0 && pts_has_keys(C, V, 0, nf, n)) {
    uint32_t done = 0;
    for (int c = nf - 1; c >= 0; --c) {  // last passing constraint per key wins (tpCounts[pair] = count)
      const ksg_tsc& t = h->tsc[c];
      if ((done >> t.topo) & 1u) continue;
      if ((t.honor_affinity && !na_ok) || (t.honor_taints && !taint_ok)) continue;
      done |= 1u << t.topo;
      uint32_t pair = C.tbase[t.topo] + node_vid(C, t.topo_key, n);
      int32_t cnt = S.cnt[(size_t)c * C.N + n];
      if (cnt) atomicAdd(&S.hist_f[pair], cnt);
      S.present_f[pair] = 1;
    }
  }
  if (ns > 0 && !(h->flags & KPF_SKIP_PTS_SCORE) && pts_has_keys(C, V, nf, nf + ns, n)) {
    for (int c = nf; c < nf + ns; ++c) {
      const ksg_tsc& t = h->tsc[c];
      if (t.is_hostname) continue;
      if ((t.honor_affinity && !na_ok) || (t.honor_taints && !taint_ok)) continue;
      uint32_t pair = C.tbase[t.topo] + node_vid(C, t.topo_key, n);
      int32_t cnt = S.cnt[(size_t)c * C.N + n];
      if (cnt) atomicAdd(&S.hist_s[pair], cnt);
    }
  }
}

// minMatchNum / TpKeyToDomainsNum per filter topology key
// slots: topology slots to reduce (sharded chain: the slots whose domains each
// sit on one node first, from local counts; the shared ones after the exchange)
__global__ void k_pts_reduce(DevCluster C, DevScratch S, const uint8_t* __restrict__ prog, uint32_t slots) {
  ProgView V = view(prog);
  const ksg_prog* h = V.h;
  uint32_t seen = 0;
  for (int c = 0; c < h->n_tsc_filter; ++c) {
    int slot = h->tsc[c].topo;
    if (!((slots >> slot) & 1u)) continue;
    if ((seen >> slot) & 1u) continue;
    seen |= 1u << slot;
    uint32_t base = C.tbase[slot], cnt = C.tcount[slot];
    int32_t mn = 0x7FFFFFFF;
    int32_t dom = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
      if (S.present_f[base + i]) {
        dom++;
        int32_t x = S.hist_f[base + i];
        mn = x < mn ? x : mn;
      }
    }
    mn = wave_min(mn);
    dom = wave_sum(dom);
    if (lane0()) {
      if (mn != 0x7FFFFFFF) atomicMin(&S.pts_min[slot], mn);
      if (dom) atomicAdd(&S.pts_dom[slot], dom);
    }
  }
}

__device__ void commit_cycle(DevCluster& C, const ProgView& V, ksg_pod_summary* s, int mode, int32_t* prow,
                             bool fresh);
// The cycle's last kernel: its last-arriving block resolves selectHost and the
// assume (what k_commit does as a launch of its own).  Every wave's atomics on
// the summary have completed (vmcnt(0) at the barrier) before its block
// arrives; the last block re-reads them with atomic RMWs (coherence point).
__device__ __forceinline__ void last_block_commit(DevCluster& C, const ProgView& V, const DevOut& O) {
  __shared__ uint32_t last;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t old = __hip_atomic_fetch_add(O.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __hip_atomic_store(O.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  commit_cycle(C, V, O.sum, O.mode, O.prow, true);
}

// Filter chain + raw scores (+ total/argmax when the profile has no ScoreExtensions).
// Position loops are run-time loops (one copy of each plugin's code: the
// instruction cache, not the loop overhead, is what limits this kernel); raw
// scores go straight to global memory, reductions run per position.
__global__ __launch_bounds__(kBlock) void k_filter_score(DevCluster C, DevProfile F, DevScratch S, DevOut O,
                                                         const uint8_t* __restrict__ prog) {
  ProgView V = view(prog);
  const ksg_prog* h = V.h;
  uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  bool active = n < C.N;
  uint32_t code = KSG_FILTER_NOT_EVALUATED;
  bool err = false;
  uint32_t ipa_flags = O.sum->ipa_flags;
  uint32_t exist_any = S.exist_any ? S.exist_any[0] : 0;
  __shared__ int32_t tvl[KSG_MAX_TOPO * kBlock];
  load_slot_vids(C, n, active, tvl);  // (each thread reads back only its own column)
  const SlotVids tv{tvl + threadIdx.x};
  if (active && !(h->flags & KPF_PREFILTER_REJECT) &&
      !((h->flags & KPF_RESTRICT) && !bit(V.u32 + h->restrict_off, h->restrict_words, (int32_t)n))) {
    code = KSG_FILTER_PASS;
#pragma unroll 1
    for (int pos = 0; pos < F.n; ++pos) {
      uint32_t detail = 0;
      bool fail = false;
      switch (F.plugins[pos]) {
        case KP_FIT: {
          uint32_t b = fit_filter(C, V, n);
          if (b) { fail = true; detail = b; }
          break;
        }
        case KP_TAINT: {
          int32_t t = untolerated_taint(C, V, n);
          if (t >= 0) { fail = true; detail = (uint32_t)t; }
          break;
        }
        case KP_NA:
          if (!(h->flags & KPF_SKIP_NA_FILTER) && !required_na(C, V, n)) fail = true;
          break;
        case KP_PTS:
          if (!(h->flags & KPF_SKIP_PTS_FILTER)) {
            int r = pts_filter_v(C, S, V, tv, err);
            if (r) { fail = true; detail = (uint32_t)(r - 1); }
          }
          break;
        case KP_IPA: {
          int r = ipa_filter_v(C, S, V, tv, ipa_flags, exist_any);
          if (r) { fail = true; detail = (uint32_t)(r - 1); }
          break;
        }
        case KP_UNSCHED: fail = unsched_fails(C, V, n); break;
        case KP_NODENAME: fail = nodename_fails(C, V, n); break;
        case KP_PORTS:
          if (!(h->flags & KPF_SKIP_PORTS)) fail = ports_fail(C, V, n);
          break;
        case KP_VOLUMES:
          detail = volume_filter(C, V, pos, n);
          fail = detail != 0;
          break;
        default: break;
      }
      if (fail) {
        code = ((uint32_t)pos << 24) | (detail & 0xFFFFFFu);
        break;
      }
    }
  }
  bool feasible = active && code == KSG_FILTER_PASS;
  if (active) O.filter[n] = code;
  unsigned long long bal = __ballot(feasible);
  if (lane0() && bal) atomicAdd(&O.sum->feasible, (int)__popcll(bal));
  if (__any(err) && lane0()) atomicOr((uint32_t*)&O.sum->status, 2u);
  if (!bal) {  // wave-uniform: no feasible node in this wave
    if (O.arrive && !F.has_ext) last_block_commit(C, V, O);
    return;
  }
  int64_t tot = 0;
  bool range_err = false;
#pragma unroll 1
  for (int pos = 0; pos < F.n; ++pos) {
    int p = F.plugins[pos];
    int64_t sc = 0;
    if (feasible) {
      switch (p) {
        case KP_FIT: sc = fit_score(C, F, V, n); break;
        case KP_BA: sc = ba_score(C, F, V, n); break;
        case KP_TAINT: sc = taint_score(C, V, n); break;
        case KP_NA: sc = (h->flags & KPF_SKIP_NA_SCORE) ? 0 : na_score(C, V, n); break;
        case KP_IPA: sc = ipa_score_v(C, S, tv); break;
        case KP_IMAGE: sc = image_score(C, V, n); break;
        default: break;
      }
      O.score[(size_t)pos * C.N + n] = (int32_t)sc;
      if (sc < 0 || sc > 100) range_err = true;
      tot += sc * F.weight[pos];
    }
    if (p == KP_TAINT || p == KP_NA || p == KP_IPA) {
      int64_t mx = wave_max(feasible ? sc : INT64_MIN);
      int64_t mn = wave_min(feasible ? sc : INT64_MAX);
      if (lane0()) {
        atomicMax((long long*)&O.sum->max_score[pos], (long long)mx);
        atomicMin((long long*)&O.sum->min_score[pos], (long long)mn);
      }
    }
  }
  if (feasible) {
    // PodTopologySpread PreScore registration (initPreScoreState)
    int nf = h->n_tsc_filter, ns = h->n_tsc_score;
    if (ns > 0 && !(h->flags & KPF_SKIP_PTS_SCORE)) {
      bool keys = true;
      for (int c = nf; c < nf + ns; ++c) keys &= tv(h->tsc[c].topo) >= 0;
      if (!keys) {
        atomicAdd(&O.sum->ignored, 1);
      } else {
        for (int c = nf; c < nf + ns; ++c)
          if (!h->tsc[c].is_hostname) S.reg[C.tbase[h->tsc[c].topo] + tv(h->tsc[c].topo)] = 1;
      }
    }
  }
  if (!F.has_ext) {
    uint64_t best = 0;
    if (feasible) {
      O.total[n] = (int32_t)tot;
      best = pack_key(tot, F.seed, h->queue_idx, C.goff + n);
    }
    uint64_t b = wave_max(best);
    if (lane0()) atomicMax((unsigned long long*)&O.sum->best_key, (unsigned long long)b);
    if (__any(range_err) && lane0()) atomicOr((uint32_t*)&O.sum->status, 2u);
  }
  if (O.arrive && !F.has_ext) last_block_commit(C, V, O);
}

// topologyNormalizingWeight per score constraint
// regcnt (sharded chain, or null): per score constraint, the global count of
// registered domains of a slot whose domains each sit on one node (uniq)
__global__ void k_pts_weights(DevCluster C, DevScratch S, DevOut O, const uint8_t* __restrict__ prog, const int64_t* regcnt,
                              uint32_t uniq) {
  ProgView V = view(prog);
  const ksg_prog* h = V.h;
  __shared__ int32_t red[kBlock / 64];
  int nf = h->n_tsc_filter, ns = h->n_tsc_score;
  for (int c = nf; c < nf + ns; ++c) {
    const ksg_tsc& t = h->tsc[c];
    int64_t size = 0;
    if (t.is_hostname) {
      size = (int64_t)O.sum->feasible - O.sum->ignored;
    } else if (t.first_of_key && regcnt && ((uniq >> t.topo) & 1u)) {
      size = regcnt[c - nf];
    } else if (t.first_of_key) {
      uint32_t base = C.tbase[t.topo], cnt = C.tcount[t.topo];
      int32_t x = 0;
      for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) x += S.reg[base + i];
      x = wave_sum(x);
      if (lane0()) red[threadIdx.x >> 6] = x;
      __syncthreads();
      if (threadIdx.x == 0)
        for (int w = 0; w < kBlock / 64; ++w) size += red[w];
      __syncthreads();
    }
    if (threadIdx.x == 0) O.sum->pts_weight[c - nf] = go_log((double)(size + 2));
  }
}

__global__ void k_pts_score(DevCluster C, DevScratch S, DevOut O, const uint8_t* __restrict__ prog, int pos) {
  ProgView V = view(prog);
  const ksg_prog* h = V.h;
  uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  bool feasible = n < C.N && O.filter[n] == KSG_FILTER_PASS;
  bool counted = false;
  int64_t s = 0;
  int nf = h->n_tsc_filter, ns = h->n_tsc_score;
  if (feasible && !(h->flags & KPF_SKIP_PTS_SCORE) && pts_has_keys(C, V, nf, nf + ns, n)) {
#pragma clang fp contract(off)
    counted = true;
    double score = 0;
    for (int c = nf; c < nf + ns; ++c) {
      const ksg_tsc& t = h->tsc[c];
      int32_t v = node_vid(C, t.topo_key, n);
      if (v < 0) continue;
      int64_t cnt = t.is_hostname ? S.cnt[(size_t)c * C.N + n] : S.hist_s[C.tbase[t.topo] + v];
      score = __dadd_rn(score, __dadd_rn(__dmul_rn((double)cnt, O.sum->pts_weight[c - nf]), (double)(t.max_skew - 1)));
    }
    s = (int64_t)round(score);
  }
  if (feasible) O.score[(size_t)pos * C.N + n] = (int32_t)s;
  int64_t mx = wave_max(counted ? s : INT64_MIN);
  int64_t mn = wave_min(counted ? s : INT64_MAX);
  bool any = __any(counted);  // every lane votes (no short-circuit around the wave op)
  if (any && lane0()) {
    atomicMax((long long*)&O.sum->max_score[pos], (long long)mx);
    atomicMin((long long*)&O.sum->min_score[pos], (long long)mn);
  }
}

// floor(x / mx) for NormalizeScore's 0 <= x <= 100 * mx: the f32-reciprocal
// divide (udiv_small: x < 2^27, quotient <= 128) for every normaliser below 2^20
// (pod-uniform branch), else div_small — not the 32-bit integer divide's
// ~40-instruction sequence per node
__device__ __forceinline__ int64_t norm_div(int64_t x, int64_t mx) {
  return mx < ((int64_t)1 << 20) && x >= 0 && x <= 100 * mx ? (int64_t)udiv_small((uint32_t)x, (uint32_t)mx)
                                                              : div_small(x, mx);
}
// NormalizeScore (wrappedplugin.go:400 -> the plugin's ScoreExtensions) of one
// feasible node's raw score at a profile position, given the pod's normaliser
// max / min over the feasible nodes: every path that selects (k_finalize, the
// table chain's k_final) and the normalized-score export (k_norm_out) use this.
// use = false: the plugin's PreScore returned Skip (no score, no weight).
// PM: the plugins compiled in (table_chain.hip eval_body); a plugin outside it
// is never met at run time
template <uint32_t PM = ~0u>
__device__ __forceinline__ int64_t normalize_pos(int plugin, const ksg_prog* h, int64_t s, int64_t mx, int64_t mn,
                                                 uint32_t ipa_flags, bool pts_keys, bool& use) {
  use = true;
  if (!((PM >> plugin) & 1u)) return s;
  switch (plugin) {
    case KP_TAINT:  // DefaultNormalizeScore(100, reverse); 0 <= s <= mx
      if constexpr (!((PM >> KP_TAINT) & 1u)) return s;
      return mx == 0 ? 100 : 100 - norm_div(100 * s, mx);
    case KP_NA:  // DefaultNormalizeScore(100, false)
      if constexpr (!((PM >> KP_NA) & 1u)) return s;
      if (h->flags & KPF_SKIP_NA_SCORE) { use = false; return s; }
      return mx == 0 ? s : norm_div(100 * s, mx);
    case KP_PTS:  // 0 <= mn <= s <= mx; nodes missing a key (IgnoredNodes) score 0
      if (h->flags & KPF_SKIP_PTS_SCORE) { use = false; return s; }
      if (!pts_keys) return 0;
      if (mx == 0) return 100;
      return norm_div(100 * (mx + mn - s), mx);
    case KP_IPA: {
#pragma clang fp contract(off)
      if (!(ipa_flags & 8u)) { use = false; return s; }  // PreScore Skip (empty topology score map)
      const int64_t diff = mx - mn;
      double f = 0;
      if (diff > 0) f = __dmul_rn(100.0, __ddiv_rn((double)(s - mn), (double)diff));
      return (int64_t)f;
    }
    default: return s;  // no ScoreExtensions: the raw score
  }
}

// NormalizeScore + [0,100] check + weights + packed-key argmax
__global__ void k_finalize(DevCluster C, DevProfile F, DevScratch S, DevOut O, const uint8_t* __restrict__ prog) {
  ProgView V = view(prog);
  const ksg_prog* h = V.h;
  uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  bool feasible = n < C.N && O.filter[n] == KSG_FILTER_PASS;
  uint64_t best = 0;
  bool range_err = false;
  if (feasible) {
    int nf = h->n_tsc_filter, ns = h->n_tsc_score;
    int64_t tot = 0;
    uint32_t ipa_flags = O.sum->ipa_flags;
    // every position's raw score and the PTS key check loaded up front
    int32_t raw[KSG_MAX_PLUGINS];
#pragma unroll
    for (int pos = 0; pos < KSG_MAX_PLUGINS; ++pos) raw[pos] = pos < F.n ? O.score[(size_t)pos * C.N + n] : 0;
    const bool pts_keys = ns > 0 && pts_has_keys(C, V, nf, nf + ns, n);
#pragma unroll
    for (int pos = 0; pos < KSG_MAX_PLUGINS; ++pos) {
      if (pos >= F.n) continue;
      bool use;  // false: the plugin's PreScore returned Skip (not scored)
      const int64_t s = normalize_pos(F.plugins[pos], h, raw[pos], O.sum->max_score[pos], O.sum->min_score[pos],
                                      ipa_flags, pts_keys, use);
      if (use) {
        if (s < 0 || s > 100) range_err = true;
        tot += s * F.weight[pos];
      }
    }
    if (O.sum->feasible == 1) tot = 0;  // single feasible node: no scoring
    O.total[n] = (int32_t)tot;
    best = pack_key(tot, F.seed, h->queue_idx, C.goff + n);
  }
  if (O.sum->feasible > 1 && __any(range_err) && lane0()) atomicOr((uint32_t*)&O.sum->status, 2u);
  uint64_t b = wave_max(best);
  if (lane0() && b) atomicMax((unsigned long long*)&O.sum->best_key, (unsigned long long)b);
  if (O.arrive) last_block_commit(C, V, O);
}

// ---- class tables: lookups and the assume delta
// Pods of class `cls` counted for topology pair (slot, v) of local node n: the
// node's own count for keys with one node per value, the pair's sum otherwise.
// nub: the key's base among the shared-key pairs (ksg_tsc / ksg_aterm .nub),
// -1 for a key with one node per value.
__device__ __forceinline__ int32_t pc_count(const DevCluster& C, int32_t cls, int32_t nub, uint32_t n, int32_t v) {
  if (cls < 0 || v < 0) return 0;
  if (nub < 0) return C.T.pc_cnt[(size_t)cls * C.N + n];
  return C.T.pc_dom[(size_t)cls * C.T.NU + (uint32_t)nub + v];
}
// A term class's value at local node n: its table at `off`, key in topology
// slot `slot` (v: n's value of that key).
__device__ __forceinline__ int32_t tc_value(const DevCluster& C, uint32_t off, int slot, uint32_t n, int32_t v) {
  if (v < 0) return 0;
  return C.T.tc_val[off + (((C.T.uniq >> slot) & 1u) ? n : (uint32_t)v)];
}
// v: node n's topology values (node_slot_vids)
// (the slot keys are read first, all together, so that the value loads issue back to back)
__device__ __forceinline__ void node_slot_vids(const DevCluster& C, uint32_t n, int32_t v[KSG_MAX_TOPO]) {
  int32_t key[KSG_MAX_TOPO];
#pragma unroll
  for (int s = 0; s < KSG_MAX_TOPO; ++s) key[s] = C.tkeyv[s];
#pragma unroll
  for (int s = 0; s < KSG_MAX_TOPO; ++s) v[s] = (uint32_t)s < C.n_topo ? node_vid(C, key[s], n) : -1;
}
// Class-table deltas come in two parts (DevTables: sharding): TP_NODE the
// node-level entries of local node n, TP_PAIR the pair-level ones.
enum { TP_NODE = 1, TP_PAIR = 2, TP_ALL = 3 };
__device__ __forceinline__ void pc_add(DevCluster& C, int32_t cls, uint32_t n, int sign, const int32_t v[KSG_MAX_TOPO],
                                       int part = TP_ALL) {
  const DevTables& T = C.T;
  if (cls < 0 || (uint32_t)cls >= T.npc) return;
  if (part & TP_NODE) atomicAdd(&T.pc_cnt[(size_t)cls * C.N + n], sign);
  if (!(part & TP_PAIR)) return;
#pragma unroll
  for (int s = 0; s < KSG_MAX_TOPO; ++s) {
    if (v[s] < 0) continue;
    atomicAdd(&T.pc_tot[(size_t)cls * KSG_MAX_TOPO + s], sign);
    if (C.nubv[s] >= 0) atomicAdd(&T.pc_dom[(size_t)cls * T.NU + (uint32_t)C.nubv[s] + v[s]], sign);
  }
}
// Topology values of global node g from the replicated table (sharded contexts).
__device__ __forceinline__ void global_slot_vids(const DevCluster& C, uint32_t g, int32_t v[KSG_MAX_TOPO]) {
#pragma unroll
  for (int s = 0; s < KSG_MAX_TOPO; ++s) v[s] = (uint32_t)s < C.n_topo ? C.T.gtv[(size_t)s * C.T.G + g] : -1;
}
// an existing pod's term: +1 (required terms) or its signed weight (preferred)
__device__ __forceinline__ int32_t eterm_inc(const ksg_exist_term& e) {
  return e.kind == 2 ? e.weight : (e.kind == 3 ? -e.weight : 1);
}
// an existing pod's term e (its term class, table offset and topology slot) on
// node n whose topology values are vs (null: read the term's key)
__device__ __forceinline__ void tc_add(DevCluster& C, const ksg_exist_term& e, uint32_t n, int sign,
                                       const int32_t* vs = nullptr, int part = TP_ALL) {
  if (e.cls < 0 || (uint32_t)e.cls >= C.T.ntc) return;
  int32_t v = -1;
  if (vs) {
#pragma unroll
    for (int s = 0; s < KSG_MAX_TOPO; ++s)
      if (s == e.topo) v = vs[s];
  } else {
    v = node_vid(C, e.topo_key, n);
  }
  if (v < 0) return;
  const bool one = ((C.T.uniq >> e.topo) & 1u) != 0;  // one node per value: a node-level entry
  if (part & (one ? TP_NODE : TP_PAIR)) atomicAdd(&C.T.tc_val[(uint32_t)e.toff + (one ? n : (uint32_t)v)], sign * eterm_inc(e));
  if (part & TP_PAIR) atomicAdd(&C.T.tc_tot[e.cls], sign);
}
// Every class-table delta of program V placed on (sign +1) / removed from
// (sign -1) a node with topology values v: its pod classes and its own affinity
// terms (part: TP_ALL on local node n; TP_PAIR for another rank's node, n
// unused).  Items i = lane, lane + lanes, ... (one thread: lane 0 of 1).
__device__ __forceinline__ void tables_assume_items(DevCluster& C, const ProgView& V, uint32_t n, const int32_t v[KSG_MAX_TOPO],
                                                    int sign, uint32_t lane, uint32_t lanes, int part) {
  const ksg_prog* h = V.h;
  const uint32_t npm = (uint32_t)h->n_pc_match, ne = (uint32_t)h->n_exist_terms;
  for (uint32_t i = lane; i < npm + ne; i += lanes) {
    if (i < npm) {
      pc_add(C, V.i32[h->pc_match_off + i], n, sign, v, part);
    } else {
      tc_add(C, V.et[h->exist_terms_off + (i - npm)], n, sign, v, part);
    }
  }
}
// (an out-of-line copy for the kernels that assume off their critical path; the
// persistent chain inlines tables_assume_items: a call spills its live registers
// and the cluster argument to scratch, microseconds on the pod's critical path)
__device__ void tables_assume_v(DevCluster& C, const ProgView& V, uint32_t n, const int32_t v[KSG_MAX_TOPO], int sign,
                                uint32_t lane, uint32_t lanes, int part) {
  tables_assume_items(C, V, n, v, sign, lane, lanes, part);
}
__device__ void tables_assume(DevCluster& C, const ProgView& V, uint32_t n, int sign, uint32_t lane, uint32_t lanes) {
  if (!C.T.on) return;
  const ksg_prog* h = V.h;
  if (lane >= (uint32_t)(h->n_pc_match + h->n_exist_terms)) return;
  int32_t v[KSG_MAX_TOPO];  // the node's topology values, loaded beside the items
  node_slot_vids(C, n, v);
  tables_assume_v(C, V, n, v, sign, lane, lanes, TP_ALL);
}
// A sharded context's assume on global node g another rank owns: the pair-level deltas.
__device__ void tables_assume_remote(DevCluster& C, const ProgView& V, uint32_t g, int sign, uint32_t lane,
                                     uint32_t lanes) {
  if (!C.T.on || !C.T.sharded || g >= C.T.G) return;
  const ksg_prog* h = V.h;
  if (lane >= (uint32_t)(h->n_pc_match + h->n_exist_terms)) return;
  int32_t v[KSG_MAX_TOPO];
  global_slot_vids(C, g, v);
  tables_assume_v(C, V, 0, v, sign, lane, lanes, TP_PAIR);
}

__device__ void table_need(const ProgView& V, uint32_t need[4]);
__device__ void table_write(DevCluster& C, const ProgView& V, uint32_t n, uint32_t row, uint32_t tb, uint32_t rb,
                            uint32_t vb);
// NodeVolumeLimits' attached volumes of node n: the pod's CSI volumes (one thread)
__device__ __forceinline__ void csi_assume(DevCluster& C, const ProgView& V, uint32_t n, int sign) {
  const ksg_prog* h = V.h;
  for (int i = 0; i < h->n_csi; ++i) {
    const int32_t v = V.i32[h->csi_off + 2 * i], key = V.i32[h->csi_off + 2 * i + 1];
    int32_t* vn = C.vnode + (size_t)v * KSG_VOL_NODES;
    int32_t* vr = C.vref + (size_t)v * KSG_VOL_NODES;
    int at = -1, empty = -1;
    for (int k = 0; k < KSG_VOL_NODES; ++k) {
      if (vn[k] == (int32_t)n) at = k;
      if (vn[k] < 0 && empty < 0) empty = k;
    }
    if (sign > 0) {
      if (at < 0) {
        if (empty < 0) continue;  // (the host bounds the nodes per volume)
        at = empty;
        vn[at] = (int32_t)n;
        vr[at] = 0;
        C.vatt[(size_t)key * C.N + n] += 1;
      }
      vr[at] += 1;
    } else if (at >= 0 && --vr[at] <= 0) {
      vn[at] = -1;
      C.vatt[(size_t)key * C.N + n] -= 1;
    }
  }
}

// assume (scheduleOne -> assume -> NodeInfo.AddPod, or its reversal for
// Unreserve) of program V on local node n: resource rows, the class tables, and
// for PTS/IPA profiles the existing-pod table (append; reversal marks the row
// deleted).  lanes > 1: the caller's other lanes apply the class-table deltas
// (tables_assume) themselves.
__device__ void assume_pod(DevCluster& C, const ProgView& V, uint32_t n, int sign, bool table, int32_t* prow,
                           uint32_t lanes = 1) {
  const ksg_prog* h = V.h;
  if (lanes == 1) tables_assume(C, V, n, sign, 0, 1);
  for (uint32_t r = 0; r < C.R; ++r) C.req[(size_t)r * C.N + n] += sign * h->req[r];
  C.nzc[n] += sign * h->nz_cpu;
  C.nzm[n] += sign * h->nz_mem;
  C.podcnt[n] += sign;
  for (int i = 0; i < h->n_port_own; ++i) C.ports[(size_t)V.i32[h->port_own_off + i] * C.N + n] += sign;
  for (int i = 0; i < h->n_pvc; ++i) atomicAdd(&C.pvcuse[V.i32[h->pvc_off + i]], sign);
  csi_assume(C, V, n, sign);
  if (sign < 0) {
    if (prow && *prow >= 0) {
      C.ptflags[*prow] |= KEF_DELETED;
      *prow = -1;
    }
    return;
  }
  if (!table) return;
  const uint32_t row = C.tcounts[0], tb = C.tcounts[1], rb = C.tcounts[2], vb = C.tcounts[3];
  uint32_t need[4];
  table_need(V, need);
  if (row + need[0] > C.pcap || tb + need[1] > C.tcap || rb + need[2] > C.rcap || vb + need[3] > C.vcap) {
    C.tcounts[4] = 1;  // overflow: host re-uploads the table from its mirror
    return;
  }
  table_write(C, V, n, row, tb, rb, vb);
  C.tcounts[0] = row + 1;
  C.tcounts[1] = tb + need[1];
  C.tcounts[2] = rb + need[2];
  C.tcounts[3] = vb + need[3];
  if (prow) *prow = (int32_t)row;
}

// Existing-pod table entries program V's row takes: rows, terms, reqs, vals.
__device__ void table_need(const ProgView& V, uint32_t need[4]) {
  const ksg_prog* h = V.h;
  const int ne = h->n_exist_terms;
  uint32_t need_r = 0, need_v = 0;
  for (int i = 0; i < ne; ++i) {
    const ksg_exist_term& e = V.et[h->exist_terms_off + i];
    need_r += e.sel.req_cnt;
    need_v += e.ns_cnt;
    for (int k = 0; k < e.sel.req_cnt; ++k) need_v += V.req[e.sel.req_off + k].nvals;
  }
  need[0] = 1;
  need[1] = (uint32_t)ne;
  need[2] = need_r;
  need[3] = need_v;
}
// Write program V's existing-pod row (on local node n) and its terms at the given offsets.
__device__ void table_write(DevCluster& C, const ProgView& V, uint32_t n, uint32_t row, uint32_t tb, uint32_t rb,
                            uint32_t vb) {
  const ksg_prog* h = V.h;
  const int ne = h->n_exist_terms;
  C.ptnode[row] = (int32_t)n;
  C.ptns[row] = h->ns_id;
  C.ptflags[row] = h->exist_flags;
  for (uint32_t k = 0; k < C.pkeys; ++k)
    C.ptlab[(size_t)k * C.pcap + row] = (int32_t)k < h->n_pod_label_keys ? V.i32[h->labels_off + k] : -1;
  for (int i = 0; i < ne; ++i) {
    ksg_exist_term e = V.et[h->exist_terms_off + i];
    for (int k = 0; k < e.ns_cnt; ++k) C.tval[vb + k] = V.i32[e.ns_off + k];
    e.ns_off = (int32_t)vb;
    vb += e.ns_cnt;
    int r0 = e.sel.req_off;
    e.sel.req_off = (int32_t)rb;
    for (int k = 0; k < e.sel.req_cnt; ++k) {
      ksg_req q = V.req[r0 + k];
      for (int j = 0; j < q.nvals; ++j) C.tval[vb + j] = V.i32[q.val_off + j];
      q.val_off = (int32_t)vb;
      vb += q.nvals;
      C.treq[rb++] = q;
    }
    C.terms[tb] = e;
    C.tpod[tb] = (int32_t)row;
    tb++;
  }
}

// selectHost result of the cycle; mode bit 0: assume on the selected node,
// bit 1: also append the pod to the existing-pod table.
// fresh: the summary was updated by atomics of other blocks of the running
// kernel — read it back through atomic RMWs (performed at the coherence point).
__device__ void commit_cycle(DevCluster& C, const ProgView& V, ksg_pod_summary* s, int mode, int32_t* prow,
                             bool fresh) {
  const ksg_prog* h = V.h;
  *prow = -1;
  int32_t status = fresh ? (int32_t)atomicOr((uint32_t*)&s->status, 0u) : s->status;
  int32_t feasible = fresh ? atomicAdd(&s->feasible, 0) : s->feasible;
  uint64_t best = fresh ? atomicMax((unsigned long long*)&s->best_key, 0ull) : s->best_key;
  if ((h->flags & KPF_PREFILTER_ERROR) || na_prescore_error(h->flags, feasible)) status |= 2;
  if (status & 2) { s->status = 2; s->selected = -1; return; }
  if (feasible == 0) { s->status = 1; s->selected = -1; return; }
  uint32_t g = (uint32_t)(best & 0xFFFFFull);
  s->selected = (int32_t)g;
  s->status = 0;
  uint32_t n = g - C.goff;
  if (!(mode & 1)) return;  // what-if
  if (g < C.goff || n >= C.N) {  // another shard owns the node: the global class tables only
    tables_assume_remote(C, V, g, +1, 0, 1);
    return;
  }
  assume_pod(C, V, n, +1, (mode & 2) != 0, prow);
}

__global__ void k_commit(DevCluster C, DevProfile F, DevOut O, const uint8_t* __restrict__ prog, int mode, int32_t* prow) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  ProgView V = view(prog);
  commit_cycle(C, V, O.sum, mode, prow, false);
}

// ---- sharded per-pod chain: every rank runs the cycle on its
// nodes and its existing pods (pods live with their node); at the cycle's
// global reductions the ranks all-gather an int64 vector and merge it:
//   X1 after the scans: the pair histograms of the topology slots whose
//      domains span nodes (SUM; presence: any), IPA flags / existing-anti slot
//      mask (OR), and per slot whose domains each sit on one node the local
//      (min, #domains) of PodTopologySpread's filter histogram (MIN, SUM);
//   X2 after Filter+Score: feasible (SUM), ignored (SUM), status (OR), the
//      normalisers' max / min per position (MAX / MIN), the PTS score
//      registration of shared pairs (any) and per score constraint on a
//      one-node-domain slot its registered-domain count (SUM);
//   X3 after the PTS score: max / min per position again;
//   X4 after NormalizeScore: the argmax key (MAX) and status (OR).
// Merging is rank-order independent, so every rank holds the same summary
// and the owner of the selected node applies the assume.
struct XLay {
  uint32_t nsp;          // shared pairs
  const uint32_t* spair; // [nsp] pair index
  uint32_t uniq;         // slot bitmask: every value on one node
};
__device__ __forceinline__ int64_t xmerge_op(const int64_t* recv, uint32_t ranks, size_t len, size_t i, int op) {
  int64_t v = recv[i];
  for (uint32_t r = 1; r < ranks; ++r) {
    const int64_t x = recv[(size_t)r * len + i];
    switch (op) {
      case 0: v += x; break;                      // sum
      case 1: v = x > v ? x : v; break;           // max
      case 2: v = x < v ? x : v; break;           // min
      case 3: v |= x; break;                      // or
      default: v = (uint64_t)x > (uint64_t)v ? x : v; break;  // unsigned max
    }
  }
  return v;
}
__device__ __forceinline__ size_t x1_len(const XLay& L) { return (size_t)7 * L.nsp + 2 + 2 * KSG_MAX_TOPO; }
__global__ void k_x1_pack(DevScratch S, DevOut O, XLay L, int64_t* out) {
  for (uint32_t i = threadIdx.x; i < L.nsp; i += blockDim.x) {
    const uint32_t p = L.spair[i];
    out[i] = S.hist_f[p];
    out[L.nsp + i] = S.present_f[p];
    out[2 * L.nsp + i] = S.hist_s[p];
    out[3 * L.nsp + i] = S.ipa_aff[p];
    out[4 * L.nsp + i] = S.ipa_anti[p];
    out[5 * L.nsp + i] = S.ipa_exist[p];
    out[6 * L.nsp + i] = S.ipa_score[p];
  }
  const size_t b = (size_t)7 * L.nsp;
  if (threadIdx.x == 0) {
    out[b] = S.exist_any[0];
    out[b + 1] = O.sum->ipa_flags;
  }
  if (threadIdx.x < KSG_MAX_TOPO) {
    out[b + 2 + threadIdx.x] = S.pts_min[threadIdx.x];
    out[b + 2 + KSG_MAX_TOPO + threadIdx.x] = S.pts_dom[threadIdx.x];
  }
}
__global__ void k_x1_merge(DevScratch S, DevOut O, XLay L, const int64_t* recv, uint32_t ranks) {
  const size_t len = x1_len(L);
  for (uint32_t i = threadIdx.x; i < L.nsp; i += blockDim.x) {
    const uint32_t p = L.spair[i];
    S.hist_f[p] = (int32_t)xmerge_op(recv, ranks, len, i, 0);
    S.present_f[p] = xmerge_op(recv, ranks, len, L.nsp + i, 0) > 0 ? 1 : 0;
    S.hist_s[p] = (int32_t)xmerge_op(recv, ranks, len, 2 * L.nsp + i, 0);
    S.ipa_aff[p] = (int32_t)xmerge_op(recv, ranks, len, 3 * L.nsp + i, 0);
    S.ipa_anti[p] = (int32_t)xmerge_op(recv, ranks, len, 4 * L.nsp + i, 0);
    S.ipa_exist[p] = (int32_t)xmerge_op(recv, ranks, len, 5 * L.nsp + i, 0);
    S.ipa_score[p] = xmerge_op(recv, ranks, len, 6 * L.nsp + i, 0);
  }
  const size_t b = (size_t)7 * L.nsp;
  if (threadIdx.x == 0) {
    S.exist_any[0] = (uint32_t)xmerge_op(recv, ranks, len, b, 3);
    O.sum->ipa_flags = (uint32_t)xmerge_op(recv, ranks, len, b + 1, 3);
  }
  if (threadIdx.x < KSG_MAX_TOPO && ((L.uniq >> threadIdx.x) & 1u)) {
    S.pts_min[threadIdx.x] = (int32_t)xmerge_op(recv, ranks, len, b + 2 + threadIdx.x, 2);
    S.pts_dom[threadIdx.x] = (int32_t)xmerge_op(recv, ranks, len, b + 2 + KSG_MAX_TOPO + threadIdx.x, 0);
  }
}
__device__ __forceinline__ size_t x2_len(const XLay& L) { return 3 + 2 * KSG_MAX_PLUGINS + (size_t)L.nsp + KSG_MAX_TSC; }
__global__ void k_x2_pack(DevCluster C, DevScratch S, DevOut O, const uint8_t* __restrict__ prog, XLay L, int64_t* out) {
  __shared__ int32_t red[kBlock / 64];
  const ksg_prog* h = view(prog).h;
  if (threadIdx.x == 0) {
    out[0] = O.sum->feasible;
    out[1] = O.sum->ignored;
    out[2] = O.sum->status;
  }
  if (threadIdx.x < KSG_MAX_PLUGINS) {
    out[3 + threadIdx.x] = O.sum->max_score[threadIdx.x];
    out[3 + KSG_MAX_PLUGINS + threadIdx.x] = O.sum->min_score[threadIdx.x];
  }
  const size_t b = 3 + 2 * KSG_MAX_PLUGINS;
  for (uint32_t i = threadIdx.x; i < L.nsp; i += blockDim.x) out[b + i] = S.reg[L.spair[i]];
  const int nf = h->n_tsc_filter, ns = h->n_tsc_score;
  for (int c = 0; c < KSG_MAX_TSC; ++c) {
    int64_t cnt = 0;
    if (c < ns) {
      const ksg_tsc& t = h->tsc[nf + c];
      if (!t.is_hostname && t.first_of_key && ((L.uniq >> t.topo) & 1u)) {
        const uint32_t base = C.tbase[t.topo], n = C.tcount[t.topo];
        int32_t x = 0;
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) x += S.reg[base + i];
        x = wave_sum(x);
        if (lane0()) red[threadIdx.x >> 6] = x;
        __syncthreads();
        for (int w = 0; w < (int)(blockDim.x / 64); ++w) cnt += red[w];
        __syncthreads();
      }
    }
    if (threadIdx.x == 0) out[b + L.nsp + c] = cnt;
  }
}
__global__ void k_x2_merge(DevScratch S, DevOut O, XLay L, const int64_t* recv, uint32_t ranks, int64_t* regcnt) {
  const size_t len = x2_len(L);
  if (threadIdx.x == 0) {
    O.sum->feasible = (int32_t)xmerge_op(recv, ranks, len, 0, 0);
    O.sum->ignored = (int32_t)xmerge_op(recv, ranks, len, 1, 0);
    O.sum->status = (int32_t)xmerge_op(recv, ranks, len, 2, 3);
  }
  if (threadIdx.x < KSG_MAX_PLUGINS) {
    O.sum->max_score[threadIdx.x] = xmerge_op(recv, ranks, len, 3 + threadIdx.x, 1);
    O.sum->min_score[threadIdx.x] = xmerge_op(recv, ranks, len, 3 + KSG_MAX_PLUGINS + threadIdx.x, 2);
  }
  const size_t b = 3 + 2 * KSG_MAX_PLUGINS;
  for (uint32_t i = threadIdx.x; i < L.nsp; i += blockDim.x)
    S.reg[L.spair[i]] = xmerge_op(recv, ranks, len, b + i, 0) > 0 ? 1 : 0;
  if (threadIdx.x < KSG_MAX_TSC) regcnt[threadIdx.x] = xmerge_op(recv, ranks, len, b + L.nsp + threadIdx.x, 0);
}
__global__ void k_x3_pack(DevOut O, int64_t* out) {
  if (threadIdx.x < KSG_MAX_PLUGINS) {
    out[threadIdx.x] = O.sum->max_score[threadIdx.x];
    out[KSG_MAX_PLUGINS + threadIdx.x] = O.sum->min_score[threadIdx.x];
  }
}
__global__ void k_x3_merge(DevOut O, const int64_t* recv, uint32_t ranks) {
  if (threadIdx.x < KSG_MAX_PLUGINS) {
    O.sum->max_score[threadIdx.x] = xmerge_op(recv, ranks, 2 * KSG_MAX_PLUGINS, threadIdx.x, 1);
    O.sum->min_score[threadIdx.x] = xmerge_op(recv, ranks, 2 * KSG_MAX_PLUGINS, KSG_MAX_PLUGINS + threadIdx.x, 2);
  }
}
__global__ void k_x4_pack(DevOut O, int64_t* out) {
  if (threadIdx.x == 0) {
    out[0] = (int64_t)O.sum->best_key;
    out[1] = O.sum->status;
  }
}
__global__ void k_x4_merge(DevOut O, const int64_t* recv, uint32_t ranks) {
  if (threadIdx.x == 0) {
    O.sum->best_key = (uint64_t)xmerge_op(recv, ranks, 2, 0, 4);
    O.sum->status = (int32_t)xmerge_op(recv, ranks, 2, 1, 3);
  }
}

// Reserve / Unreserve on an explicit node (the framework's selectHost choice).
// table 2: a DefaultPreemption dry-run toggle — the pod leaves (sign -1) or
// re-enters (+1) its node with its existing-pod table row *prow tombstoned or
// revived in place (the table neither grows nor reorders).
__global__ void k_assume(DevCluster C, const uint8_t* __restrict__ prog, int32_t gnode, int sign, int table, int32_t* prow) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  ProgView V = view(prog);
  uint32_t n = (uint32_t)gnode - C.goff;
  if (gnode < 0) return;
  if ((uint32_t)gnode < C.goff || n >= C.N) {  // another shard's node: the global class tables only
    if (table != 2) tables_assume_remote(C, V, (uint32_t)gnode, sign, 0, 1);
    return;
  }
  if (table == 2) {
    assume_pod(C, V, n, sign, false, nullptr);
    if (prow && *prow >= 0) {
      if (sign < 0) C.ptflags[*prow] |= KEF_DELETED;
      else C.ptflags[*prow] &= ~KEF_DELETED;
    }
    return;
  }
  assume_pod(C, V, n, sign, table != 0, prow);
}
// toggle_staged: thread g toggles group g's entries (sorted idx[gs[g] .. gs[g+1]),
// all on one node) in sequence: a node's row, ports and existing-pod flags are
// touched by one thread only; the class tables and claim counts take atomics.
// (Entries with CSI volumes, whose per-volume node lists are shared across
// nodes, never come here: the host toggles those one launch per pod.)
__global__ __launch_bounds__(256) void k_toggle_groups(DevCluster C, const uint64_t* __restrict__ addr,
                                                       const int32_t* __restrict__ gnode,
                                                       int32_t* rows, const uint32_t* __restrict__ idx,
                                                       const uint32_t* __restrict__ gs, uint32_t ngroups, int sign) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  if (g >= ngroups) return;
  for (uint32_t j = gs[g]; j < gs[g + 1]; ++j) {
    const uint32_t e = idx[j];
    const ProgView V = view(reinterpret_cast<const uint8_t*>(addr[e]));
    const uint32_t n = (uint32_t)gnode[e] - C.goff;
    if (gnode[e] < 0 || (uint32_t)gnode[e] < C.goff || n >= C.N) continue;
    assume_pod(C, V, n, sign, false, nullptr);
    const int32_t r = rows[e];
    if (r >= 0) {
      if (sign < 0) C.ptflags[r] |= KEF_DELETED;
      else C.ptflags[r] &= ~KEF_DELETED;
    }
  }
}


// ----------------------------------------------------------------- what-if batches (cfg5)
// A step of `count` queue pods is scheduled against ONE frozen snapshot (no
// assume between them), then all placements are bound together
// (BASELINE.json cfg5; oracle: ksg_oracle_whatif).  Profiles of NodeResourcesFit,
// BalancedAllocation, TaintToleration and NodeAffinity.  Two passes over the
// (pod tile x node tile) grid:
//   k_whatif<1>  filter chain + the raw scores of the normalised plugins:
//                per-pod feasible count and max/min (DefaultNormalizeScore input)
//   k_whatif<2>  filter chain + all scores, NormalizeScore, weights, packed key:
//                per-pod argmax (atomicMax of the 64-bit key)
// A block holds KSG_WI_PODS pods (program headers through the scalar cache) x
// KSG_WI_NPT * 256 nodes; every node row is read from HBM once per pod tile and
// served from L1/L2 for the tile's pods.  Per-pod reductions: wave DPP, then one
// atomic per wave.  Per-pair outputs are written only for the kept pods (the
// sampled parity subset).
#define KSG_WI_PODS 32
#define KSG_WI_NPT 4
struct WiArgs {
  const uint8_t* progs;
  const uint64_t* prog_off;
  uint32_t q0, count;
  ksg_pod_summary* sums;
  uint32_t keep_first, keep_n;
  uint32_t* kfilter;
  int32_t *kscore, *ktotal;
  // per-pair record of pass 1 for pass 2 (null: pass 2 recomputes), 4 or 8 bytes:
  // top bit feasible, next Fit/BA score out of range, then from bit 0 the raw
  // NodeAffinity score (bw_a bits), the raw Taint score (bw_t), the Fit/BA weighted
  // sum (bw_tot); row (q - q0) * N + n
  void* rec;
  uint32_t bw_a, bw_t, bw_tot;
  uint32_t small;  // 100 x the profile's weights < 2^31: every total fits 32 bits (k_whatif_rec2)
  uint32_t need_eph;  // resource columns 2..3 requested by some pod (RowV loads)
  // class path (k_whatif_cls1 / k_whatif_cls2): per (pod, tile) class rows and
  // feasible counts (bit 31: a Fit/BA score out of range); per pod the folded
  // class row and flag between the phases of a sharded step
  uint64_t* wc_part;
  uint32_t* wc_cnt;
  uint64_t* wc_cls;
  uint32_t* wc_flag;
};

// (programs as restrict parameters: their reads stay scalar loads beside the
// kernel's summary atomics and kept-output stores)
template <int PASS>
__global__ __launch_bounds__(256) void k_whatif(DevCluster C, DevProfile F, WiArgs A, const uint8_t* __restrict__ progs,
                                                const uint64_t* __restrict__ prog_off) {
  const uint32_t base = blockIdx.x * (256 * KSG_WI_NPT) + threadIdx.x;
#pragma unroll 1
  for (uint32_t pi = 0; pi < KSG_WI_PODS; ++pi) {
    const uint32_t j = blockIdx.y * KSG_WI_PODS + pi;
    if (j >= A.count) break;
    const uint32_t q = A.q0 + j;
    const ProgView V = view(progs + prog_off[q]);
    const ksg_prog* h = V.h;
    ksg_pod_summary* sm = A.sums + q;
    const bool kept = A.keep_n && q >= A.keep_first && q < A.keep_first + A.keep_n;
    const size_t slot = kept ? q - A.keep_first : 0;
    int32_t feas_all = 0;
    if (PASS == 2) feas_all = sm->feasible;
    int cnt = 0;
    uint64_t best = 0;
    bool range_err = false;
    int64_t mx[KSG_MAX_PLUGINS], mn[KSG_MAX_PLUGINS];
#pragma unroll
    for (int p = 0; p < KSG_MAX_PLUGINS; ++p) {
      mx[p] = INT64_MIN;
      mn[p] = INT64_MAX;
    }
    if (PASS == 2 && A.rec && !kept) continue;  // k_whatif_rec2
#pragma unroll 1
    for (int k = 0; k < KSG_WI_NPT; ++k) {
      const uint32_t n = base + k * 256;
      if (n >= C.N || (h->flags & KPF_PREFILTER_REJECT) ||
          ((h->flags & KPF_RESTRICT) && !bit(V.u32 + h->restrict_off, h->restrict_words, (int32_t)n))) {
        if (PASS == 2 && kept && n < C.N) A.kfilter[slot * C.N + n] = KSG_FILTER_NOT_EVALUATED;
        continue;
      }
      uint32_t code = KSG_FILTER_PASS;
#pragma unroll 1
      for (int pos = 0; pos < F.n && code == KSG_FILTER_PASS; ++pos) {
        switch (F.plugins[pos]) {
          case KP_FIT: {
            uint32_t b = fit_filter(C, V, n);
            if (b) code = ((uint32_t)pos << 24) | b;
            break;
          }
          case KP_TAINT: {
            int32_t t = untolerated_taint(C, V, n);
            if (t >= 0) code = ((uint32_t)pos << 24) | ((uint32_t)t & 0xFFFFFFu);
            break;
          }
          case KP_NA:
            if (!(h->flags & KPF_SKIP_NA_FILTER) && !required_na(C, V, n)) code = (uint32_t)pos << 24;
            break;
          default: break;
        }
      }
      if (PASS == 2 && kept) A.kfilter[slot * C.N + n] = code;
      if (code != KSG_FILTER_PASS) continue;
      ++cnt;
      int64_t tot = 0;
#pragma unroll 1
      for (int pos = 0; pos < F.n; ++pos) {
        const int p = F.plugins[pos];
        int64_t s = 0;
        if (PASS == 1 && p != KP_TAINT && p != KP_NA) continue;
        switch (p) {
          case KP_FIT: s = fit_score(C, F, V, n); break;
          case KP_BA: s = ba_score(C, F, V, n); break;
          case KP_TAINT: s = taint_score(C, V, n); break;
          case KP_NA: s = (h->flags & KPF_SKIP_NA_SCORE) ? 0 : na_score(C, V, n); break;
          default: break;
        }
        if (PASS == 1) {
          mx[pos] = s > mx[pos] ? s : mx[pos];
          mn[pos] = s < mn[pos] ? s : mn[pos];
          continue;
        }
        if (kept) A.kscore[(slot * KSG_MAX_PLUGINS + pos) * C.N + n] = (int32_t)s;
        const int64_t M = sm->max_score[pos];
        if (p == KP_TAINT) s = M == 0 ? 100 : 100 - 100 * s / M;  // DefaultNormalizeScore(reverse)
        else if (p == KP_NA) s = (h->flags & KPF_SKIP_NA_SCORE) ? 0 : (M == 0 ? s : 100 * s / M);
        if (s < 0 || s > 100) range_err = true;
        tot += s * F.weight[pos];
      }
      if (PASS == 2) {
        if (feas_all == 1) tot = 0;  // single feasible node: no scoring
        if (kept) A.ktotal[slot * C.N + n] = (int32_t)tot;
        uint64_t key = pack_key(tot, F.seed, h->queue_idx, C.goff + n);
        best = key > best ? key : best;
      }
    }
    if (PASS == 1) {
      int c = wave_sum(cnt);
      if (lane0() && c) atomicAdd(&sm->feasible, c);
#pragma unroll 1
      for (int pos = 0; pos < F.n; ++pos) {
        if (F.plugins[pos] != KP_TAINT && F.plugins[pos] != KP_NA) continue;
        int64_t a = wave_max(mx[pos]), b = wave_min(mn[pos]);
        if (lane0() && c) {
          atomicMax((long long*)&sm->max_score[pos], (long long)a);
          atomicMin((long long*)&sm->min_score[pos], (long long)b);
        }
      }
    } else {
      uint64_t b = wave_max(best);
      if (lane0() && b) atomicMax((unsigned long long*)&sm->best_key, (unsigned long long)b);
      if (feas_all > 1 && __any(range_err) && lane0()) atomicOr((uint32_t*)&sm->status, 2u);
    }
  }
}

// selectHost result per pod of the step (no assume yet)
__global__ void k_whatif_select(WiArgs A) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= A.count) return;
  const ksg_prog* h = reinterpret_cast<const ksg_prog*>(A.progs + A.prog_off[A.q0 + j]);
  ksg_pod_summary* s = A.sums + A.q0 + j;
  if ((h->flags & KPF_PREFILTER_ERROR) || na_prescore_error(h->flags, s->feasible)) s->status |= 2;
  if (s->status & 2) { s->status = 2; s->selected = -1; return; }
  if (s->feasible == 0) { s->status = 1; s->selected = -1; return; }
  s->selected = (int32_t)(s->best_key & 0xFFFFFull);
  s->status = 0;
}

// Bind the step's placements (resource rows; sums commute, so in parallel).
__global__ void k_whatif_bind(DevCluster C, WiArgs A) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= A.count) return;
  const ksg_pod_summary* s = A.sums + A.q0 + j;
  if (s->status != 0) return;
  const ksg_prog* h = reinterpret_cast<const ksg_prog*>(A.progs + A.prog_off[A.q0 + j]);
  uint32_t g = (uint32_t)s->selected, n = g - C.goff;
  if (g < C.goff || n >= C.N) return;  // another shard owns the node
  for (uint32_t r = 0; r < C.R; ++r)
    atomicAdd((unsigned long long*)&C.req[(size_t)r * C.N + n], (unsigned long long)h->req[r]);
  atomicAdd((unsigned long long*)&C.nzc[n], (unsigned long long)h->nz_cpu);
  atomicAdd((unsigned long long*)&C.nzm[n], (unsigned long long)h->nz_mem);
  atomicAdd(&C.podcnt[n], 1);
}

// Bind a step's placements one pod after another, in queue order (the order
// ksg_oracle_whatif applies its deferred AddPods): for profiles with class tables
// and an existing-pod table, whose appends must stay sequential.  One wave: the
// lanes apply a pod's class-table deltas, lane 0 its node row and table row.
__global__ __launch_bounds__(64) void k_whatif_bind_seq(DevCluster C, const uint8_t* __restrict__ progs,
                                                        const uint64_t* __restrict__ prog_off,
                                                        const ksg_pod_summary* sums, uint32_t q0, uint32_t count,
                                                        int table, int32_t* prow) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t j = q0; j < q0 + count; ++j) {
    const ksg_pod_summary& s = sums[j];
    const uint32_t g = (uint32_t)s.selected, n = g - C.goff;
    if (s.status != 0) continue;
    if (g < C.goff || n >= C.N) {  // another shard owns the node: the global class tables only
      tables_assume_remote(C, view(progs + prog_off[j]), g, +1, lane, 64);
      __syncthreads();
      continue;
    }
    const ProgView V = view(progs + prog_off[j]);
    tables_assume(C, V, n, +1, lane, 64);
    if (lane == 0) assume_pod(C, V, n, +1, table != 0, prow + j, 64);
    __syncthreads();
  }
}

// Sharded steps: merge the ranks' summaries of the step's pods
// (phase 1: feasible counts and score max/min; phase 2: argmax key, status bits).
__global__ void k_whatif_merge(const ksg_pod_summary* recv, uint32_t ranks, uint32_t count, ksg_pod_summary* sums,
                               int phase) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  ksg_pod_summary m = recv[j];
  for (uint32_t r = 1; r < ranks; ++r) {
    const ksg_pod_summary& o = recv[(size_t)r * count + j];
    if (phase == 1) {
      m.feasible += o.feasible;
      for (int p = 0; p < KSG_MAX_PLUGINS; ++p) {
        m.max_score[p] = o.max_score[p] > m.max_score[p] ? o.max_score[p] : m.max_score[p];
        m.min_score[p] = o.min_score[p] < m.min_score[p] ? o.min_score[p] : m.min_score[p];
      }
    } else {
      m.best_key = o.best_key > m.best_key ? o.best_key : m.best_key;
      m.status |= o.status;
    }
  }
  sums[j] = m;
}


// ----------------------------------------------------------------- static pre-pass (per-pod chain, Taint/NA profiles)
// TaintToleration's and NodeAffinity's Filter and raw Score of a (pod, node)
// pair depend only on the node's taints and labels, never on the pods assumed on
// it.  So a chunk of queue pods gets them in one wide pass (k_static, same tiling
// as the what-if kernels) and each pod's cycle is then ONE kernel (k_fs_static)
// that reads an 8-B record per node instead of walking taints and label columns
// through dependent loads.  NormalizeScore's max is taken over feasible nodes;
// k_static provides the max over the statically feasible nodes (M), which is
// the true max whenever one node reaching it is also Fit-feasible — counted per
// cycle; otherwise the cycle's last block recomputes it (exact fallback).
struct StaticRec {
  uint32_t code;  // KSG_FILTER_PASS, KSG_FILTER_NOT_EVALUATED, or (pos << 24) | detail of the first failing static filter
  uint32_t raw;   // raw TaintToleration score << 20 | raw NodeAffinity score
};
#define KSG_RAW_NA_MASK 0xFFFFFu

// Grid: node tiles of 256 x KSG_ST_NPT nodes x pod tiles of KSG_ST_PODS pods —
// small tiles, so that a chunk of pods gives every SIMD several waves to hide
// the label loads' latency behind (the work per pair is a few dependent loads).
#define KSG_ST_PODS 4
#define KSG_ST_NPT 1
// glob: C covers every node of a node-sharded cluster (the PreFilterResult's
// global bitmap applies)
__global__ __launch_bounds__(256) void k_static(DevCluster C, DevProfile F, const uint8_t* __restrict__ progs, const uint64_t* __restrict__ prog_off,
                                                uint32_t q0, uint32_t count, StaticRec* out, int64_t* mpred, int glob) {
  const uint32_t base = blockIdx.x * (256 * KSG_ST_NPT) + threadIdx.x;
#pragma unroll 1
  for (uint32_t pi = 0; pi < KSG_ST_PODS; ++pi) {
    const uint32_t j = blockIdx.y * KSG_ST_PODS + pi;
    if (j >= count) break;
    const ProgView V = view(progs + prog_off[q0 + j]);
    const ksg_prog* h = V.h;
    const bool skip_na_score = (h->flags & KPF_SKIP_NA_SCORE) != 0;
    int64_t mt = -1, ma = -1;
#pragma unroll 1
    for (int k = 0; k < KSG_ST_NPT; ++k) {
      const uint32_t n = base + k * 256;
      if (n >= C.N) continue;
      uint32_t code = KSG_FILTER_PASS, raw = 0;
      if ((h->flags & KPF_PREFILTER_REJECT) ||
          ((h->flags & KPF_RESTRICT) && !(glob ? bit(V.u32 + h->restrict_g_off, h->restrict_g_words, (int32_t)n)
                                               : bit(V.u32 + h->restrict_off, h->restrict_words, (int32_t)n)))) {
        code = KSG_FILTER_NOT_EVALUATED;
      } else {
#pragma unroll 1
        for (int pos = 0; pos < F.n && code == KSG_FILTER_PASS; ++pos) {
          if (F.plugins[pos] == KP_TAINT) {
            int32_t t = untolerated_taint(C, V, n);
            if (t >= 0) code = ((uint32_t)pos << 24) | ((uint32_t)t & 0xFFFFFFu);
          } else if (F.plugins[pos] == KP_NA) {
            if (!(h->flags & KPF_SKIP_NA_FILTER) && !required_na(C, V, n)) code = (uint32_t)pos << 24;
          }
        }
        if (code == KSG_FILTER_PASS) {
          int64_t t = F.pos_taint >= 0 ? taint_score(C, V, n) : 0;
          int64_t a = (F.pos_na >= 0 && !skip_na_score) ? na_score(C, V, n) : 0;
          raw = ((uint32_t)t << 20) | ((uint32_t)a & KSG_RAW_NA_MASK);
          mt = t > mt ? t : mt;
          ma = a > ma ? a : ma;
        }
      }
      out[(size_t)j * C.N + n] = StaticRec{code, raw};
    }
    int64_t a0 = wave_max(mt), a1 = wave_max(ma);
    if (lane0()) {
      if (a0 >= 0) atomicMax((long long*)&mpred[2 * j], (long long)a0);
      if (a1 >= 0) atomicMax((long long*)&mpred[2 * j + 1], (long long)a1);
    }
  }
}

__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(int32_t* p, int32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(int64_t* p, int64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int64_t ld_sc1(const int64_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int32_t ld_sc1(const int32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// DefaultNormalizeScore of the two static plugins, weighted; raw Fit/BA scores given.
__device__ __forceinline__ int64_t static_total(const DevProfile& F, bool skip_na_score, int64_t fit, int64_t ba,
                                                int64_t t, int64_t a, int64_t MT, int64_t MA, bool& range_err) {
  int64_t tot = 0;
  for (int pos = 0; pos < F.n; ++pos) {
    int64_t s = 0;
    switch (F.plugins[pos]) {
      case KP_FIT: s = fit; break;
      case KP_BA: s = ba; break;
      case KP_TAINT: s = MT == 0 ? 100 : 100 - div_small(100 * t, MT); break;  // reverse; 0 <= t <= MT
      case KP_NA:
        if (skip_na_score) continue;
        s = MA == 0 ? a : div_small(100 * a, MA);
        break;
      default: break;
    }
    if (s < 0 || s > 100) range_err = true;
    tot += s * F.weight[pos];
  }
  return tot;
}

// One scheduling cycle of one pod for a profile of Fit/BA/Taint/NA (any order):
// Filter chain in profile order, raw scores, NormalizeScore with the static max,
// weighted total, packed-key argmax; the last block checks the max, falls back
// to the exact max when no Fit-feasible node reaches it, and commits.
// Per-pair outputs are stored sc1 (the fallback re-reads them in this kernel).
__global__ __launch_bounds__(kBlock) void k_fs_static(DevCluster C, DevProfile F, DevOut O, const uint8_t* __restrict__ prog,
                                                     const StaticRec* st, const int64_t* mp, int32_t* aux) {
  // aux: [0] a feasible node reaches the static Taint max, [1] NodeAffinity, [2] a score out of range, [3] arrivals
  __shared__ uint64_t red64[kBlock / 64];
  __shared__ int64_t redm[2][kBlock / 64];
  __shared__ uint32_t last;
  const ProgView V = view(prog);
  const ksg_prog* h = V.h;
  const bool skip_na_score = (h->flags & KPF_SKIP_NA_SCORE) != 0;
  const int64_t MT = mp[0] < 0 ? 0 : mp[0], MA = mp[1] < 0 ? 0 : mp[1];
  const uint32_t N = C.N;
  // one node: Filter chain in profile order (static part from the record), raw scores, total with (mt, ma)
  auto eval = [&](uint32_t n, int64_t mt, int64_t ma, uint32_t& code, int64_t (&raw)[4], int64_t& tot, bool& re) {
    const StaticRec r = st[n];
    code = r.code;
    if (code != KSG_FILTER_NOT_EVALUATED && F.pos_fit >= 0) {
      const uint32_t spos = code == KSG_FILTER_PASS ? 0xFFu : code >> 24;
      if ((uint32_t)F.pos_fit < spos) {
        const uint32_t fb = fit_filter(C, V, n);
        if (fb) code = ((uint32_t)F.pos_fit << 24) | fb;
      }
    }
    if (code != KSG_FILTER_PASS) return;
    raw[0] = F.pos_fit >= 0 ? fit_score(C, F, V, n) : 0;
    raw[1] = F.pos_ba >= 0 ? ba_score(C, F, V, n) : 0;
    raw[2] = r.raw >> 20;
    raw[3] = skip_na_score ? 0 : (int64_t)(r.raw & KSG_RAW_NA_MASK);
    tot = static_total(F, skip_na_score, raw[0], raw[1], raw[2], raw[3], mt, ma, re);
  };
  auto store = [&](uint32_t n, uint32_t code, const int64_t (&raw)[4], int64_t tot) {
    O.filter[n] = code;
    if (code != KSG_FILTER_PASS) return;
    if (F.pos_fit >= 0) O.score[(size_t)F.pos_fit * N + n] = (int32_t)raw[0];
    if (F.pos_ba >= 0) O.score[(size_t)F.pos_ba * N + n] = (int32_t)raw[1];
    if (F.pos_taint >= 0) O.score[(size_t)F.pos_taint * N + n] = (int32_t)raw[2];
    if (F.pos_na >= 0) O.score[(size_t)F.pos_na * N + n] = (int32_t)raw[3];
    O.total[n] = (int32_t)tot;
  };
  const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t code = KSG_FILTER_NOT_EVALUATED;
  int64_t raw[4] = {0, 0, 0, 0}, tot = 0;
  bool range_err = false;
  if (n < N) eval(n, MT, MA, code, raw, tot, range_err);
  const bool feasible = n < N && code == KSG_FILTER_PASS;
  const uint64_t best = feasible ? pack_key(tot, F.seed, h->queue_idx, C.goff + n) : 0;
  // aggregates first (completed before this block arrives); the per-pair stores drain afterwards
  const unsigned long long bal = __ballot(feasible);
  const uint64_t bk = wave_max(best);
  const bool at = __any(feasible && raw[2] == MT), aa = __any(feasible && raw[3] == MA), re = __any(range_err);
  if (lane0()) {
    if (bal) atomicAdd(&O.sum->feasible, (int)__popcll(bal));
    if (bk) atomicMax((unsigned long long*)&O.sum->best_key, (unsigned long long)bk);
    if (at) atomicOr(&aux[0], 1);
    if (aa) atomicOr(&aux[1], 1);
    if (re) atomicOr(&aux[2], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add((uint32_t*)&aux[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  if (n < N) store(n, code, raw, tot);
  __syncthreads();
  if (!last) return;
  // ---- last block: the cycle's aggregates, read back in one round of atomic RMWs
  __shared__ int64_t agg[8];
  if (threadIdx.x < 6) {
    int64_t v = 0;
    switch (threadIdx.x) {
      case 0: v = atomicAdd(&O.sum->feasible, 0); break;
      case 1: v = atomicOr(&aux[0], 0); break;
      case 2: v = atomicOr(&aux[1], 0); break;
      case 3: v = atomicOr(&aux[2], 0); break;
      case 4: v = (int64_t)atomicOr((uint32_t*)&O.sum->status, 0u); break;
      case 5: v = (int64_t)atomicMax((unsigned long long*)&O.sum->best_key, 0ull); break;
    }
    agg[threadIdx.x] = v;
  }
  __syncthreads();
  const int32_t feas_all = (int32_t)agg[0];
  bool any_range = agg[3] != 0;
  uint64_t best_all = (uint64_t)agg[5];
  const bool need_t = F.pos_taint >= 0 && agg[1] == 0, need_a = F.pos_na >= 0 && !skip_na_score && agg[2] == 0;
  int64_t mt = MT, ma = MA;
  if (feas_all > 0 && (need_t || need_a)) {
    // exact fallback (no Fit-feasible node reaches the static max): recompute the
    // max over the feasible nodes, then every total and the argmax, from the rows
    int64_t lt = 0, la = 0;
    for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
      uint32_t c;
      int64_t rw[4] = {0, 0, 0, 0}, t2 = 0;
      bool e2 = false;
      eval(i, MT, MA, c, rw, t2, e2);
      if (c == KSG_FILTER_PASS) { lt = max(lt, rw[2]); la = max(la, rw[3]); }
    }
    lt = wave_max(lt);
    la = wave_max(la);
    if (lane0()) { redm[0][threadIdx.x >> 6] = lt; redm[1][threadIdx.x >> 6] = la; }
    __syncthreads();
    mt = ma = 0;
    for (int w = 0; w < kBlock / 64; ++w) { mt = max(mt, redm[0][w]); ma = max(ma, redm[1][w]); }
    uint64_t lb = 0;
    bool lre = false;
    for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
      uint32_t c;
      int64_t rw[4] = {0, 0, 0, 0}, t2 = 0;
      eval(i, mt, ma, c, rw, t2, lre);
      if (c == KSG_FILTER_PASS) {
        uint64_t key = pack_key(t2, F.seed, h->queue_idx, C.goff + i);
        lb = key > lb ? key : lb;
      }
    }
    lb = wave_max(lb);
    lre = __any(lre);
    if (lane0()) red64[threadIdx.x >> 6] = lb | (lre ? 0x8000000000000000ull : 0ull);
    __syncthreads();
    best_all = 0;
    any_range = false;
    for (int w = 0; w < kBlock / 64; ++w) {
      uint64_t x = red64[w] & 0x7FFFFFFFFFFFFFFFull;
      best_all = x > best_all ? x : best_all;
      any_range |= (red64[w] >> 63) != 0;
    }
  }
  if (threadIdx.x != 0) return;
  if (F.pos_taint >= 0) O.sum->max_score[F.pos_taint] = mt;
  if (F.pos_na >= 0) O.sum->max_score[F.pos_na] = skip_na_score ? 0 : ma;
  int32_t status = (int32_t)agg[4];
  if (feas_all > 1 && any_range) status |= 2;
  O.sum->best_key = feas_all == 1 ? (best_all & 0xFFFFFFFFFFull) : best_all;  // one feasible node: not scored
  O.sum->status = status;
  O.sum->feasible = feas_all;
  for (int i = 0; i < 4; ++i) aux[i] = 0;  // the next cycle's counters (ordered by the kernel boundary)
  commit_cycle(C, V, O.sum, O.mode, O.prow, false);
}

// ----------------------------------------------------------------- speculative window path
// For profiles whose plugins are all NodeResourcesFit / BalancedAllocation (no
// ScoreExtensions, no cross-node state) a pod's result on node n depends only on
// node n's row, so the queue runs as windows of KSG_BATCH pods, pipelined two
// deep: ONE launch of k_window per window j
//
//   block 0      replays window j exactly (k_window's fixup: Jacobi iteration
//                over the window's picks, see win_fixup), appends the window's
//                assume deltas to the pending list P_j and writes P_{j-1} back
//                into the node rows;
//   blocks 1..   evaluate window j+1 against the rows as of the end of window
//                j-1 (rows of P_{j-1} taken from the list, since block 0 is
//                rewriting them), write every per-pair output, keep each tile's
//                top-64 keys; the last tile block of each pod (arrival counter)
//                merges them into the pod's 64 candidates with their rows.
//
// The candidates of window j+1 are thus taken on a snapshot two windows old:
// at most 32 (window j) + 31 (earlier pods of window j+1) nodes can have
// changed since, so of 64 candidates at least one is unmodified, and the best
// unmodified node of a pod is always in its list.  Modified nodes are
// re-evaluated exactly on their current rows.  The result is the sequential
// schedule: same selections, same per-pair outputs, same assume deltas.
#define KSG_BATCH 32
#define KSG_CAND 64        // candidates per pod: >= 2*KSG_BATCH (see above)
#define KSG_TOPK 64
#ifndef KSG_WIN_THREADS
#define KSG_WIN_THREADS 1024  // (a build-time knob for A/B builds: 512 lifts the 128-VGPR cap)
#endif
#define KSG_TILE KSG_WIN_THREADS  // nodes per eval block
#define KSG_STASH_NPT 8    // eval tiles of up to this many nodes per thread hold their outputs in LDS
#ifndef KSG_STAGE
#define KSG_STAGE 4        // candidate ranks whose rows are staged in LDS (deeper ranks: global; 4 measured +4% over 16 on cfg2)
#endif
#define KSG_XHDR 512       // record header: per pod feasible count, static-max achievers (Taint, NodeAffinity): 3 x KSG_BATCH ints
#define KSG_NOT_PATCHED 0xFFFFFFFDu

struct RowV {  // one node row (resource columns 0..3)
  int64_t alloc[4], req[4];
  int64_t nzc, nzm;
  int32_t podcnt, allowed;
};
struct Pend {  // a node modified by a window: row before (base) and after it
  int32_t node, pad;  // global node index
  RowV base, after;
};
// Candidate record of a window: header, then the 32 x 64 candidate keys, then the
// rows the keys were computed on (structure of arrays: the replay stages every key
// but only the rows of its shallow ranks).
static constexpr size_t kRecKeys = (size_t)KSG_BATCH * KSG_CAND;
static constexpr size_t kRecBytes = KSG_XHDR + kRecKeys * 8 + kRecKeys * sizeof(RowV);
// Sharded windows exchange the header and the keys only (16.5 KiB per rank):
// every rank keeps a replica of every node's row (WinArgs::xrows), so the
// merged candidates' rows come from the local replica, not from the wire.
static constexpr size_t kXchgBytes = KSG_XHDR + kRecKeys * 8;
static_assert(sizeof(RowV) % 8 == 0, "RowV is staged as 64-bit words");
__device__ __forceinline__ uint64_t* rec_keys(uint8_t* rec) { return reinterpret_cast<uint64_t*>(rec + KSG_XHDR); }
__device__ __forceinline__ const uint64_t* rec_keys(const uint8_t* rec) {
  return reinterpret_cast<const uint64_t*>(rec + KSG_XHDR);
}
__device__ __forceinline__ RowV* rec_rows(uint8_t* rec) { return reinterpret_cast<RowV*>(rec + KSG_XHDR + kRecKeys * 8); }
__device__ __forceinline__ const RowV* rec_rows(const uint8_t* rec) {
  return reinterpret_cast<const RowV*>(rec + KSG_XHDR + kRecKeys * 8);
}


struct PodLite {  // the fields of ksg_prog the Fit/BA evaluation reads (LDS-staged)
  int64_t req[4];
  int64_t fit_score_req[KSG_MAX_SCORE_RES];
  int64_t ba_req[KSG_MAX_SCORE_RES];
  int64_t nz_cpu, nz_mem;
  int32_t queue_idx;
  uint32_t flags;
};

// staging block [PodLite | pad | program]: the program 16-byte aligned
constexpr size_t kPlOff = (sizeof(PodLite) + 15) & ~(size_t)15;
static_assert(sizeof(PodLite) % 4 == 0, "PodLite words");
__global__ void k_place_program(const uint8_t* __restrict__ src, uint32_t bytes, uint8_t* dst, uint64_t* off_slot,
                                uint64_t off, void* plite_slot, int32_t* prow_slot, int32_t row, ksg_pod_summary* sum,
                                DevProfile F) {
  const uint32_t t = threadIdx.x;
  const uint8_t* prog = src + kPlOff;
  // 16-byte pieces, all issued before any is stored (src may be pinned host
  // memory: one PCIe round trip, not one per byte-loop iteration)
  const uint32_t n16 = bytes / 16;
  for (uint32_t i = t; i < n16; i += blockDim.x)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(prog)[i];
  for (uint32_t i = n16 * 16 + t; i < bytes; i += blockDim.x) dst[i] = prog[i];
  for (uint32_t i = t; i < (uint32_t)(sizeof(PodLite) / 4); i += blockDim.x)
    reinterpret_cast<uint32_t*>(plite_slot)[i] = reinterpret_cast<const uint32_t*>(src)[i];
  if (t == 0) {
    *off_slot = off;
    *prow_slot = row;
    ksg_pod_summary z = {};
    z.selected = -1;
    for (int p = 0; p < KSG_MAX_PLUGINS; ++p) {
      z.max_score[p] = (p < F.n && F.plugins[p] == KP_IPA) ? INT64_MIN : 0;
      z.min_score[p] = INT64_MAX;
    }
    *sum = z;
  }
}

struct WinArgs {
  const PodLite* plite;  // Fit/BA fields of every queue pod (flat copy of the programs)
  uint32_t first, keep_first, keep_n, need_eph;
  uint32_t *kfilter, *sfilter;  // kept outputs / scratch ring of 2*KSG_BATCH pods
  int32_t *kscore, *sscore, *ktotal, *stotal;
  // eval part: window E = queue pods [e0, e0 + ne)
  uint32_t e0, ne, T, npt, tile_len;  // T tiles of tile_len <= KSG_TILE * npt nodes per pod
  uint64_t* tile_top;    // [KSG_BATCH][T][KSG_TOPK] (window E's buffer)
  int32_t* tile_feas;    // [KSG_BATCH][T][3]
  // defer: the eval blocks only store their tile lists; block 0 of the next
  // launch merges them (window W's buffers below) and loads the candidates'
  // rows from the node rows — the pod's merge leaves the evaluation's chain
  uint32_t defer;
  uint32_t stash_npt;  // eval tiles of up to this many nodes per thread hold all outputs in LDS
  const uint64_t* wtile_top;
  const int32_t* wtile_feas;
  uint32_t* arrive;      // [KSG_BATCH] tile arrivals (reset by the last block)
  uint8_t* erec;         // candidate record of window E (kRecBytes)
  // fixup part: window W = queue pods [w0, w0 + nw)
  uint32_t w0, nw;
  const uint8_t* wrec;   // candidate record of window W
  const Pend* pprev;     // P_{W-1} (also the eval part's row overrides)
  const int32_t* pprev_n;
  Pend* pnext;           // P_W
  int32_t* pnext_n;
  ksg_pod_summary* sums;
  uint64_t* stamps;      // diagnostic stamps of window W's fixup (16 slots), or null
  uint64_t* estamps;     // diagnostic stamps of window E's eval blocks (16 slots), or null
  // profiles with TaintToleration / NodeAffinity: static records of a ring of
  // stat_ring queue pods (pod q at slot (q - first) % stat_ring) and their static maxima
  const StaticRec* stat;
  uint32_t stat_ring;
  uint32_t stat_n, stat_base;  // a record row holds stat_n nodes from global node stat_base (node-sharded: every node)
  uint32_t G;                  // nodes of the whole cluster
  const int64_t* mpred;  // [2 * (q - first)]: Taint, NodeAffinity (-1: no statically feasible node)
  // sharded: replica of every node's row, indexed by global node (kept in step by
  // every rank's identical replay); null on one shard
  RowV* xrows;
  // persistent window loop (k_window_run): the eval blocks count their window's
  // finished pod records (evd) and written outputs (flushed); the replay waits for
  // flush_need of them before it patches outputs; abortw / spin bound every wait
  uint32_t* evd;
  uint32_t* flushed;
  uint32_t flush_need;
  uint32_t* abortw;
  uint32_t spin;
  uint32_t* pub;      // the replicated "windows replayed" flag (16 lines of 32 words) and the value
  uint32_t pub_val;   // replay(W) publishes once P_W is out: W + 1
  const Pend* pcur;   // eval side: P_{E-1} and its count, published when *pubw >= pub_need
  const int32_t* pcur_n;
  const uint32_t* pubw;
  uint32_t pub_need;
  uint32_t mblocks;   // persistent loop: dedicated merge blocks (one per pod) merge the tile lists
  uint32_t astride;   // arrival counter stride (u32): 1, or 32 in the persistent loop (a line per pod)
  // persistent loop: 1 = the replay evaluates its window's pods on P_{W-1} itself
  // (the merges hand over keys and rows without waiting for P_{W-1}); 0 = the
  // merges do it once P_{W-1} is published (PriorRec)
  uint32_t prior_fix;
  // persistent loop, split hand-over (KSG_WIN_SPLIT=1): a merge counts its keys and
  // shallow rows out (evk) before its prior step, so the replay stages them while the
  // prior steps run and waits for the records (evd_wait >= evd_need; null: not split)
  // only before it reads the PriorRecs
  uint32_t split;
  uint32_t* evk;
  const uint32_t* evd_wait;
  uint32_t evd_need;
  const uint32_t* nxt_evd;  // persistent loop: the next window's record counter and its target (null: last)
  uint32_t nxt_need;
};
// the static record of (queue pod q, global node g); PER (the persistent loop,
// whose records k_static_dec may still be writing beside it): an sc1 load
template <bool PER = false>
__device__ __forceinline__ StaticRec srec_at(const WinArgs& A, uint32_t q, uint32_t g) {
  const StaticRec* p = A.stat + (size_t)((q - A.first) % A.stat_ring) * A.stat_n + (g - A.stat_base);
  if constexpr (!PER) {
    return *p;
  } else {
    const uint64_t v = ld_sc1(reinterpret_cast<const uint64_t*>(p));
    return StaticRec{(uint32_t)v, (uint32_t)(v >> 32)};
  }
}
__device__ __forceinline__ int64_t sel4(const int64_t (&v)[4], int i) {
  return i == 0 ? v[0] : i == 1 ? v[1] : i == 2 ? v[2] : v[3];
}
template <class P>
__device__ __forceinline__ uint32_t fit_filter_row(const RowV& r, const P* h, uint32_t R) {
  uint32_t bits = 0;
  if (r.podcnt + 1 > r.allowed) bits |= KSG_FIT_TOO_MANY_PODS;
  if (h->flags & KPF_ZERO_REQUEST) return bits;
  int64_t q0 = h->req[0], q1 = h->req[1];
  if (q0 > 0 && q0 > r.alloc[0] - r.req[0]) bits |= 1u << 1;
  if (q1 > 0 && q1 > r.alloc[1] - r.req[1]) bits |= 1u << 2;
  if (R > 2) {
    int64_t q2 = h->req[2];
    if (q2 > 0 && q2 > r.alloc[2] - r.req[2]) bits |= 1u << 3;
    if (R > 3) {
      int64_t q3 = h->req[3];
      if (q3 > 0 && q3 > r.alloc[3] - r.req[3]) bits |= 1u << 4;
    }
  }
  return bits;
}
__device__ __forceinline__ void alloc_req_row(const RowV& r, int res, int64_t pod_req, bool use_requested, int64_t& a,
                                              int64_t& q) {
  if (res < 0 || res > 3 || (res >= KSG_RES_EPH + 1 && pod_req == 0)) { a = 0; q = 0; return; }
  a = sel4(r.alloc, res);
  if (res == KSG_RES_CPU) q = (use_requested ? r.req[0] : r.nzc) + pod_req;
  else if (res == KSG_RES_MEM) q = (use_requested ? r.req[1] : r.nzm) + pod_req;
  else q = sel4(r.req, res) + pod_req;
}
__device__ __noinline__ int64_t rtc_fn_ool(const DevProfile& F, int64_t p) { return rtc_fn(F, p); }
__device__ __forceinline__ int64_t least_req(int64_t a, int64_t q) {  // leastRequestedScore
  return q > a ? 0 : div_small((a - q) * 100, a);
}
// leastRequestedScore for the compiled default arguments: floor((a-q)*100/a)
// from one f64 reciprocal estimate (relative error ~2^-50, quotient <= 100, so
// the truncated estimate is the quotient or one below it) and one exact
// integer correction; branch-free unless (a-q)*100 >= 2^52.
__device__ __forceinline__ int64_t least_req_q(int64_t a, int64_t q) {
  if (q > a || a <= 0) return 0;
  int64_t x = (a - q) * 100;
  if (__builtin_expect(x >= ((int64_t)1 << 52), 0)) return div_i64_slow(x, a);
  int64_t d = (int64_t)((double)x * __builtin_amdgcn_rcp((double)a));
  int64_t rem = x - d * a;
  return rem >= a ? d + 1 : (rem < 0 ? d - 1 : d);
}
template <int MODE, class P>
__device__ __forceinline__ int64_t fit_score_row(const RowV& r, const DevProfile& F, const P* h) {
  if (MODE == 1) {  // LeastAllocated, cpu:1 memory:1 (the defaults): (s_cpu + s_mem) / 2
    bool ok0 = r.alloc[0] != 0, ok1 = r.alloc[1] != 0;
    int64_t s0 = ok0 ? least_req_q(r.alloc[0], r.nzc + h->fit_score_req[0]) : 0;
    int64_t s1 = ok1 ? least_req_q(r.alloc[1], r.nzm + h->fit_score_req[1]) : 0;
    int64_t ns = s0 + s1;
    return ok0 && ok1 ? ns >> 1 : ns;
  }
  int64_t ns = 0, ws = 0;
#pragma unroll 1
  for (int i = 0; i < F.fit_n; ++i) {
    int64_t a, q;
    alloc_req_row(r, F.fit_res_d[i], h->fit_score_req[i], false, a, q);
    if (a == 0) continue;
    int64_t s, w = F.fit_w_d[i];
    if (F.fit_strategy == 2) {
      s = q > a ? rtc_fn_ool(F, 100) : rtc_fn_ool(F, div_small(q * 100, a));
      if (s <= 0) continue;
    } else if (F.fit_strategy == 1) {
      s = div_small((q > a ? a : q) * 100, a);
    } else {
      s = least_req(a, q);
    }
    ns += s * w;
    ws += w;
  }
  if (ws == 0) return 0;
  if (F.fit_strategy == 2) return (int64_t)round((double)ns / (double)ws);
  return div_small(ns, ws);
}
// balancedResourceScorer: fractions in resource order; the >2-resource case
// recomputes each fraction in a second pass instead of keeping an array.
template <int MODE, class P>
__device__ __forceinline__ int64_t ba_score_row(const RowV& r, const DevProfile& F, const P* h) {
#pragma clang fp contract(off)
  double sd = 0.0;
  if (MODE == 1) {
    bool ok0 = r.alloc[0] != 0, ok1 = r.alloc[1] != 0;
    if (ok0 && ok1) {
      double f0 = (double)(r.req[0] + h->ba_req[0]) / (double)r.alloc[0];
      double f1 = (double)(r.req[1] + h->ba_req[1]) / (double)r.alloc[1];
      if (f0 > 1) f0 = 1;
      if (f1 > 1) f1 = 1;
      sd = fabs((f0 - f1) / 2);
    }
    return (int64_t)((1 - sd) * 100.0);
  }
  int m = 0;
  double total = 0, f0 = 0, f1 = 0;
#pragma unroll 1
  for (int i = 0; i < F.ba_n; ++i) {
    int64_t a, q;
    alloc_req_row(r, F.ba_res_d[i], h->ba_req[i], true, a, q);
    if (a == 0) continue;
    double f = (double)q / (double)a;
    if (f > 1) f = 1;
    total = total + f;
    if (m == 0) f0 = f;
    else if (m == 1) f1 = f;
    m++;
  }
  if (m == 2) {
    sd = fabs((f0 - f1) / 2);
  } else if (m > 2) {
    double mean = total / (double)m;
    double sum = 0;
#pragma unroll 1
    for (int i = 0; i < F.ba_n; ++i) {
      int64_t a, q;
      alloc_req_row(r, F.ba_res_d[i], h->ba_req[i], true, a, q);
      if (a == 0) continue;
      double f = (double)q / (double)a;
      if (f > 1) f = 1;
      sum = sum + (f - mean) * (f - mean);
    }
    sd = sqrt(sum / (double)m);
  }
  return (int64_t)((1 - sd) * 100.0);
}

// Evaluate one (pod, node row) for a Fit/BA profile: filter code, raw Fit and BA, total.
template <int MODE, class P>
__device__ __forceinline__ uint32_t eval_row(const RowV& r, const DevProfile& F, const P* h, uint32_t R,
                                             int32_t& fit_s, int32_t& ba_s, int64_t& total) {
  total = 0;
  fit_s = ba_s = 0;
  if (F.pos_fit >= 0) {
    uint32_t b = fit_filter_row(r, h, R);
    if (b) return ((uint32_t)F.pos_fit << 24) | b;
    fit_s = (int32_t)fit_score_row<MODE>(r, F, h);
    total += (int64_t)fit_s * F.w_fit;
  }
  if (F.pos_ba >= 0) {
    ba_s = (int32_t)ba_score_row<MODE>(r, F, h);
    total += (int64_t)ba_s * F.w_ba;
  }
  return KSG_FILTER_PASS;
}
// Fit/BA/Taint/NodeAffinity profiles: the static record of (pod, node) supplies
// the Taint/NodeAffinity filter verdicts and raw scores; the Fit filter runs in
// its profile position; NormalizeScore uses the pod's normaliser (MT, MA).
template <int MODE, class P>
__device__ __forceinline__ uint32_t eval_row_s(const RowV& r, const DevProfile& F, const P* h, uint32_t R, StaticRec s,
                                               int64_t MT, int64_t MA, int32_t& fit_s, int32_t& ba_s, int64_t& total) {
  total = 0;
  fit_s = ba_s = 0;
  const uint32_t code = s.code;
  if (code == KSG_FILTER_NOT_EVALUATED) return code;
  if (F.pos_fit >= 0 && (code == KSG_FILTER_PASS || (uint32_t)F.pos_fit < (code >> 24))) {
    uint32_t b = fit_filter_row(r, h, R);
    if (b) return ((uint32_t)F.pos_fit << 24) | b;
  }
  if (code != KSG_FILTER_PASS) return code;
  if (F.pos_fit >= 0) fit_s = (int32_t)fit_score_row<MODE>(r, F, h);
  if (F.pos_ba >= 0) ba_s = (int32_t)ba_score_row<MODE>(r, F, h);
  // DefaultNormalizeScore (reverse for Taint), weighted; the sum is order-free
  total = (int64_t)fit_s * F.w_fit + (int64_t)ba_s * F.w_ba;
  if (F.pos_taint >= 0) {
    const uint32_t t = s.raw >> 20;
    total += (int64_t)(MT <= 0 ? 100u : 100u - udiv_small(100u * t, (uint32_t)MT)) * F.w_taint;
  }
  if (F.pos_na >= 0 && !(h->flags & KPF_SKIP_NA_SCORE)) {
    const uint32_t a = s.raw & KSG_RAW_NA_MASK;
    total += (int64_t)(MA <= 0 ? a : udiv_small(100u * a, (uint32_t)MA)) * F.w_na;
  }
  return code;
}
// raw: the static record's raw Taint/NodeAffinity scores (STAT profiles)
// P: the persistent window loop's sc1 stores (no dirty line left in this XCD's L2
// that a later write of the same output from another XCD could be overtaken by)
template <bool STAT, bool P = false>
__device__ __forceinline__ void write_pair(const DevProfile& F, uint32_t* of, int32_t* os, int32_t* ot, uint32_t N,
                                           uint32_t n, uint32_t code, int32_t fit_s, int32_t ba_s, int64_t tot,
                                           uint32_t raw) {
  auto st = [](auto* p, auto v) {
    if constexpr (P) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
  };
  st(of + n, code);
  if (code == KSG_FILTER_PASS) {
    if (F.pos_fit >= 0) st(os + (size_t)F.pos_fit * N + n, fit_s);
    if (F.pos_ba >= 0) st(os + (size_t)F.pos_ba * N + n, ba_s);
    if (STAT) {
      if (F.pos_taint >= 0) st(os + (size_t)F.pos_taint * N + n, (int32_t)(raw >> 20));
      if (F.pos_na >= 0) st(os + (size_t)F.pos_na * N + n, (int32_t)(raw & KSG_RAW_NA_MASK));
    }
    st(ot + n, (int32_t)tot);
  }
}

// Lane exchange v[lane ^ J] on the VALU (no LDS crossbar round trip as with
// ds_bpermute): DPP quad_perm for 1 and 2, DPP row rotations for 4 and 8,
// gfx950's v_permlane16_swap / v_permlane32_swap for 16 and 32.
// (dpp row_ror:N — lane i of a 16-lane row reads lane (i - N) mod 16.)
template <int J>
__device__ __forceinline__ uint32_t xor_lanes32(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63;
  if (J == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  if (J == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  if (J == 4) {
    const uint32_t a = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x12C, 0xF, 0xF, false);  // row_ror:12
    return (lane & 4) ? a : b;
  }
  if (J == 8) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  if (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? r[0] : r[1];
  }
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (lane & 32) ? r[0] : r[1];
}
template <int J>
__device__ __forceinline__ uint64_t xor_lanes(uint64_t v) {
  return ((uint64_t)xor_lanes32<J>((uint32_t)(v >> 32)) << 32) | xor_lanes32<J>((uint32_t)v);
}
template <int J>
__device__ __forceinline__ uint64_t bitonic_step(uint64_t v, bool desc) {
  const uint64_t o = xor_lanes<J>(v);
  const bool low = (threadIdx.x & J) == 0;
  return (low == desc) ? (v > o ? v : o) : (v < o ? v : o);
}
template <int K>
__device__ __forceinline__ uint64_t bitonic_stage(uint64_t v) {  // merge step of block size K
  const bool desc = K == 64 || (threadIdx.x & K) == 0;
  if (K >= 64) v = bitonic_step<32>(v, desc);
  if (K >= 32) v = bitonic_step<16>(v, desc);
  if (K >= 16) v = bitonic_step<8>(v, desc);
  if (K >= 8) v = bitonic_step<4>(v, desc);
  if (K >= 4) v = bitonic_step<2>(v, desc);
  return bitonic_step<1>(v, desc);
}
__device__ __forceinline__ uint64_t wave_sort_desc(uint64_t v) {
  v = bitonic_stage<2>(v);
  v = bitonic_stage<4>(v);
  v = bitonic_stage<8>(v);
  v = bitonic_stage<16>(v);
  v = bitonic_stage<32>(v);
  return bitonic_stage<64>(v);
}
// v: descending list, o_rev: the other descending list read in reverse lane order
__device__ __forceinline__ uint64_t wave_merge_top(uint64_t v, uint64_t o_rev) {
  v = v > o_rev ? v : o_rev;  // bitonic; its top half holds the 64 largest
  return bitonic_stage<64>(v);
}
// v read in reverse lane order (lane ^ 63)
__device__ __forceinline__ uint64_t wave_reverse(uint64_t v) {
  return xor_lanes<32>(xor_lanes<16>(xor_lanes<8>(xor_lanes<4>(xor_lanes<2>(xor_lanes<1>(v))))));
}
// Self-test of the lane exchanges against ds_bpermute shuffles (diagnostic ABI).
__global__ void k_selftest_lanes(const uint64_t* in, int32_t* bad) {
  const uint64_t v = in[threadIdx.x + blockIdx.x * 64];
  int e = 0;
  e += xor_lanes<1>(v) != __shfl_xor(v, 1, 64);
  e += xor_lanes<2>(v) != __shfl_xor(v, 2, 64);
  e += xor_lanes<4>(v) != __shfl_xor(v, 4, 64);
  e += xor_lanes<8>(v) != __shfl_xor(v, 8, 64);
  e += xor_lanes<16>(v) != __shfl_xor(v, 16, 64);
  e += xor_lanes<32>(v) != __shfl_xor(v, 32, 64);
  e += wave_reverse(v) != __shfl(v, 63 - (int)(threadIdx.x & 63), 64);
  const uint64_t srt = wave_sort_desc(v);  // descending, and a permutation (sum and xor kept)
  const uint64_t nxt = __shfl_down(srt, 1, 64);
  e += (threadIdx.x & 63) < 63 && nxt > srt;
  const uint64_t m = wave_merge_top(srt, wave_reverse(wave_sort_desc(~v)));
  const uint64_t nm = __shfl_down(m, 1, 64);
  e += (threadIdx.x & 63) < 63 && nm > m;
  int c_sorted = 0, c_in = 0;  // multiset check: occurrences of v in the input and in the sorted list
  for (int j = 0; j < 64; ++j) {
    c_sorted += __shfl(srt, j, 64) == v;
    c_in += __shfl(v, j, 64) == v;
  }
  e += c_sorted != c_in;
  for (int i = 0; i < 16; ++i) {  // udiv_small on its domain (quotient <= 100)
    const uint64_t z = splitmix64(v + (uint64_t)i);
    const uint32_t d = 1u + (uint32_t)(z % (i < 8 ? 4096u : 1048576u));
    const uint32_t x = (uint32_t)((z >> 24) % (100ull * d + 1));
    e += udiv_small(x, d) != x / d;
  }
  atomicAdd(bad, e);
}

// Per-pair output rows of queue pod q: the kept window, or a scratch ring of
// two windows (window j+1 is evaluated while window j is being patched).
__device__ __forceinline__ bool kept_q(const WinArgs& A, uint32_t q) {
  return A.keep_n && q >= A.keep_first && q < A.keep_first + A.keep_n;
}
__device__ __forceinline__ void out_ptrs(const WinArgs& A, uint32_t q, uint32_t N, uint32_t*& f, int32_t*& s,
                                         int32_t*& t) {
  if (kept_q(A, q)) {
    size_t slot = q - A.keep_first;
    f = A.kfilter + slot * N;
    s = A.kscore + slot * N * KSG_MAX_PLUGINS;
    t = A.ktotal + slot * N;
  } else {
    size_t slot = (q - A.first) % (2 * KSG_BATCH);
    f = A.sfilter + slot * N;
    s = A.sscore + slot * N * KSG_MAX_PLUGINS;
    t = A.stotal + slot * N;
  }
}
__device__ __forceinline__ void load_row(const DevCluster& C, uint32_t n, uint32_t need_eph, RowV& r) {
  r.alloc[0] = C.alloc[n];
  r.alloc[1] = C.alloc[(size_t)C.N + n];
  r.req[0] = C.req[n];
  r.req[1] = C.req[(size_t)C.N + n];
  r.alloc[2] = r.req[2] = r.alloc[3] = r.req[3] = 0;
  if (need_eph) {
#pragma unroll
    for (uint32_t c = 2; c < 4; ++c)
      if (c < C.R) {
        r.alloc[c] = C.alloc[(size_t)c * C.N + n];
        r.req[c] = C.req[(size_t)c * C.N + n];
      }
  }
  r.nzc = C.nzc[n];
  r.nzm = C.nzm[n];
  r.podcnt = C.podcnt[n];
  r.allowed = C.allowed[n];
}
__device__ __forceinline__ void store_row(const DevCluster& C, uint32_t n, const RowV& r) {
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
    if (k < C.R) C.req[(size_t)k * C.N + n] = r.req[k];
  C.nzc[n] = r.nzc;
  C.nzm[n] = r.nzm;
  C.podcnt[n] = r.podcnt;
}

// Persistent window loop (k_window_run, PER = true): what one block of the launch
// hands to another — node rows, the P lists, candidate records, per-pair outputs —
// moves by agent-scope (sc1) stores and loads (MI355X_MICROARCH.md hand-off table,
// row 1): an sc1 load never returns a line another CU's L1 or another XCD's L2
// holds stale, and an sc1 store leaves no dirty line behind in the writer's L2.
template <bool P, class T>
__device__ __forceinline__ T ldv(const T* p) {
  if constexpr (P) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool P, class T>
__device__ __forceinline__ void stv(T* p, T v) {
  if constexpr (P) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <bool P, class T>
__device__ __forceinline__ T ld_obj(const T* p) {
  if constexpr (!P) {
    return *p;
  } else {
    static_assert(sizeof(T) % 8 == 0, "8-byte words");
    T v;
    uint64_t* d = reinterpret_cast<uint64_t*>(&v);
    const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
#pragma unroll
    for (size_t i = 0; i < sizeof(T) / 8; ++i) d[i] = ld_sc1(q + i);
    return v;
  }
}
template <bool P, class T>
__device__ __forceinline__ void st_obj(T* p, const T& v) {
  if constexpr (!P) {
    *p = v;
  } else {
    static_assert(sizeof(T) % 8 == 0, "8-byte words");
    const uint64_t* s = reinterpret_cast<const uint64_t*>(&v);
    uint64_t* q = reinterpret_cast<uint64_t*>(p);
#pragma unroll
    for (size_t i = 0; i < sizeof(T) / 8; ++i) st_sc1(q + i, s[i]);
  }
}
// load_row / store_row with the columns an assume changes handed over sc1
template <bool P>
__device__ __forceinline__ void load_row_p(const DevCluster& C, uint32_t n, uint32_t need_eph, RowV& r) {
  if constexpr (!P) {
    load_row(C, n, need_eph, r);
  } else {
    r.alloc[0] = C.alloc[n];
    r.alloc[1] = C.alloc[(size_t)C.N + n];
    r.req[0] = ldv<true>(C.req + n);
    r.req[1] = ldv<true>(C.req + (size_t)C.N + n);
    r.alloc[2] = r.req[2] = r.alloc[3] = r.req[3] = 0;
    if (need_eph) {
#pragma unroll
      for (uint32_t c = 2; c < 4; ++c)
        if (c < C.R) {
          r.alloc[c] = C.alloc[(size_t)c * C.N + n];
          r.req[c] = ldv<true>(C.req + (size_t)c * C.N + n);
        }
    }
    r.nzc = ldv<true>(C.nzc + n);
    r.nzm = ldv<true>(C.nzm + n);
    r.podcnt = ldv<true>(C.podcnt + n);
    r.allowed = C.allowed[n];
  }
}
template <bool P>
__device__ __forceinline__ void store_row_p(const DevCluster& C, uint32_t n, const RowV& r) {
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
    if (k < C.R) stv<P>(C.req + (size_t)k * C.N + n, r.req[k]);
  stv<P>(C.nzc + n, r.nzc);
  stv<P>(C.nzm + n, r.nzm);
  stv<P>(C.podcnt + n, r.podcnt);
}

// Record path of a what-if step (run_whatif): pass 1 in the small tiles of
// k_static (KSG_WI_PODS pods x 256 nodes per block), every score of every
// feasible pair computed once, the step's per-pod feasible count and Taint /
// NodeAffinity max/min reduced per block (one atomic per block and pod); pass 2
// streams the records.  The thread's node row and its first four taints are
// loaded once for the block's pods (RowV evaluation of the window path; the
// record path needs <= 4 resource columns); the taint list is walked once per
// pair for both TaintToleration's Filter and its Score.
template <class RT, int MODE>  // record word; MODE: eval_row specialisation
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_whatif_rec1(
    DevCluster C, DevProfile F, WiArgs A, const uint8_t* __restrict__ progs, const uint64_t* __restrict__ prog_off) {
  __shared__ int64_t red[2][4][5];
  // grid: x = pod group (fastest: the blocks of one node tile run together and
  // share its rows in L2), y = node tile
  const uint32_t n = blockIdx.y * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pt = F.pos_taint, pa = F.pos_na;
  const bool hf = F.pos_fit >= 0, hb = F.pos_ba >= 0, ht = pt >= 0, ha = pa >= 0;
  const uint32_t R = C.R < 4 ? C.R : 4;
  const bool live = n < C.N;
  constexpr RT FEAS = (RT)1 << (8 * sizeof(RT) - 1), RANGE = FEAS >> 1;
  const uint32_t sh_t = A.bw_a, sh_tot = A.bw_a + A.bw_t;
  RowV row{};
  uint32_t t0 = 0, tc = 0;
  int32_t tr[4] = {-1, -1, -1, -1};
  if (live) {
    load_row(C, n, A.need_eph, row);
    t0 = C.toff[n];
    tc = C.toff[n + 1] - t0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((uint32_t)i < tc) tr[i] = C.tid[t0 + i];
  }
#pragma unroll 1
  for (uint32_t pi = 0; pi < KSG_WI_PODS; ++pi) {
    const uint32_t j = blockIdx.x * KSG_WI_PODS + pi;
    if (j >= A.count) break;
    const ProgView V = view(progs + prog_off[A.q0 + j]);
    const ksg_prog* h = V.h;
    int cnt = 0;
    int32_t tx = INT32_MIN, tn = INT32_MAX, ax = INT32_MIN, an = INT32_MAX;  // (raw scores < 2^20: static_fits)
    if (live) {
      RT rw = 0;
      if (!(h->flags & KPF_PREFILTER_REJECT) &&
          !((h->flags & KPF_RESTRICT) && !bit(V.u32 + h->restrict_off, h->restrict_words, (int32_t)n))) {
        // (only pass / fail matters here, and integer sums commute: the profile's
        // four plugins in a fixed order, no per-pair dispatch on the profile)
        bool pass = !hf || fit_filter_row(row, h, R) == 0;
        int64_t tpref = 0;
        if (pass && ht) {
          const uint32_t* hard = V.u32 + h->taint_hard_off;
          const uint32_t* pref = V.u32 + h->taint_pref_off;
          const int tw = h->taint_words;
          // the pod's first 64 taint bits in scalar registers (one load each per pod)
          const uint64_t hw = tw > 1 ? ((uint64_t)hard[1] << 32 | hard[0]) : tw > 0 ? hard[0] : 0;
          const uint64_t pw = tw > 1 ? ((uint64_t)pref[1] << 32 | pref[0]) : tw > 0 ? pref[0] : 0;
#pragma unroll 1
          for (uint32_t i = 0; i < tc; ++i) {
            const int32_t t = i == 0 ? tr[0] : i == 1 ? tr[1] : i == 2 ? tr[2] : i == 3 ? tr[3] : C.tid[t0 + i];
            const bool lo = (uint32_t)t < 64;
            if (lo ? ((hw >> t) & 1) : bit(hard, tw, t)) { pass = false; break; }
            tpref += (lo ? ((pw >> t) & 1) : bit(pref, tw, t)) ? 1 : 0;
          }
        }
        pass = pass && (!ha || (h->flags & KPF_SKIP_NA_FILTER) || required_na(C, V, n));
        if (pass) {
          cnt = 1;
          rw = FEAS;
          int64_t tot = 0;
          if (hf) {
            const int64_t s = fit_score_row<MODE>(row, F, h);
            if (s < 0 || s > 100) rw |= RANGE;
            else tot += s * F.w_fit;
          }
          if (hb) {
            const int64_t s = ba_score_row<MODE>(row, F, h);
            if (s < 0 || s > 100) rw |= RANGE;
            else tot += s * F.w_ba;
          }
          if (ht) {  // (field widths from the cluster's taint counts / the programs' weights)
            tx = tn = (int32_t)tpref;
            rw |= (RT)tpref << sh_t;
          }
          if (ha) {
            const int64_t s = (h->flags & KPF_SKIP_NA_SCORE) ? 0 : na_score(C, V, n);
            ax = an = (int32_t)s;
            rw |= (RT)s;
          }
          if (!(rw & RANGE)) rw |= (RT)tot << sh_tot;
        }
      }
      __builtin_nontemporal_store(rw, static_cast<RT*>(A.rec) + (size_t)j * C.N + n);
    }
    int64_t* r = red[pi & 1][w];
    const int c = wave_sum(cnt);
    tx = wave_max(tx); tn = wave_min(tn); ax = wave_max(ax); an = wave_min(an);
    if (lane == 0) { r[0] = c; r[1] = tx; r[2] = tn; r[3] = ax; r[4] = an; }
    __syncthreads();  // (red double-buffered: one barrier per pod)
    if (threadIdx.x == 0) {
      int64_t v[5] = {0, INT32_MIN, INT32_MAX, INT32_MIN, INT32_MAX};
      for (int k = 0; k < 4; ++k) {
        const int64_t* x = red[pi & 1][k];
        v[0] += x[0];
        v[1] = max(v[1], x[1]); v[2] = min(v[2], x[2]); v[3] = max(v[3], x[3]); v[4] = min(v[4], x[4]);
      }
      if (v[0]) {
        ksg_pod_summary* sm = A.sums + A.q0 + j;
        atomicAdd(&sm->feasible, (int32_t)v[0]);
        if (pt >= 0) {
          atomicMax((long long*)&sm->max_score[pt], (long long)v[1]);
          atomicMin((long long*)&sm->min_score[pt], (long long)v[2]);
        }
        if (pa >= 0) {
          atomicMax((long long*)&sm->max_score[pa], (long long)v[3]);
          atomicMin((long long*)&sm->min_score[pa], (long long)v[4]);
        }
      }
    }
  }
}

// Unsigned 32-bit division by a pod-uniform divisor (Granlund-Montgomery): one
// multiply-high, a subtract, an add and two shifts per quotient, exact for every
// 32-bit dividend.
struct UDiv {
  uint32_t m, s1, s2;
};
__device__ __forceinline__ UDiv udiv_of(uint32_t d) {
  const uint32_t l = d <= 1 ? 0u : 32u - (uint32_t)__clz(d - 1);
  const uint32_t m = (uint32_t)(((((uint64_t)1 << l) - d) << 32) / d + 1);
  return UDiv{m, l < 1 ? l : 1u, l > 1 ? l - 1 : 0u};
}
__device__ __forceinline__ uint32_t udiv(uint32_t n, const UDiv& v) {
  const uint32_t t = __umulhi(v.m, n);
  return (t + ((n - t) >> v.s1)) >> v.s2;
}

// Pass 2 from the records: NormalizeScore, weights, packed key, per-pod argmax.
// Each thread keeps the next pod's records in flight while it reduces this one's;
// KSG_WI_R2NPT nodes per thread amortise the per-pod reduction and atomics.
#define KSG_WI_R2NPT 16
template <class RT>
__global__ __launch_bounds__(256) void k_whatif_rec2(DevCluster C, DevProfile F, WiArgs A,
                                                     const uint8_t* __restrict__ progs,
                                                     const uint64_t* __restrict__ prog_off) {
  const uint32_t base = blockIdx.x * (256 * KSG_WI_R2NPT) + threadIdx.x;
  const int pt = F.pos_taint, pa = F.pos_na;
  const int64_t wt = pt >= 0 ? F.weight[pt] : 0, wa = pa >= 0 ? F.weight[pa] : 0;
  const uint32_t j0 = blockIdx.y * KSG_WI_PODS, jn = min(A.count - j0, (uint32_t)KSG_WI_PODS);
  constexpr RT FEAS = (RT)1 << (8 * sizeof(RT) - 1), RANGE = FEAS >> 1;
  const uint32_t sh_t = A.bw_a, sh_tot = A.bw_a + A.bw_t;
  const RT ma_ = (RT)(((uint64_t)1 << A.bw_a) - 1), mt_ = (RT)(((uint64_t)1 << A.bw_t) - 1),
           mtot = (RT)(((uint64_t)1 << A.bw_tot) - 1);
  const RT* rec = static_cast<const RT*>(A.rec);
  RT nx[KSG_WI_R2NPT];
  auto fetch = [&](uint32_t j, RT* r) {
#pragma unroll
    for (int k = 0; k < KSG_WI_R2NPT; ++k) {
      const uint32_t n = base + k * 256;
      r[k] = n < C.N ? __builtin_nontemporal_load(rec + (size_t)j * C.N + n) : 0;
    }
  };
  // the next pod's summary fields and program flags are requested with its records
  struct PodP {
    int32_t feas, qidx;
    uint32_t flags;
    int64_t Mt, Ma;
  };
  auto params = [&](uint32_t j) {
    const ksg_prog* h = reinterpret_cast<const ksg_prog*>(progs + prog_off[A.q0 + j]);
    const ksg_pod_summary* sm = A.sums + A.q0 + j;
    return PodP{sm->feasible, h->queue_idx, h->flags, pt >= 0 ? sm->max_score[pt] : 0, pa >= 0 ? sm->max_score[pa] : 0};
  };
  fetch(j0, nx);
  PodP np = params(j0);
#pragma unroll 1
  for (uint32_t pi = 0; pi < jn; ++pi) {
    const uint32_t j = j0 + pi, q = A.q0 + j;
    RT cur[KSG_WI_R2NPT];
#pragma unroll
    for (int k = 0; k < KSG_WI_R2NPT; ++k) cur[k] = nx[k];
    const PodP P = np;
    if (pi + 1 < jn) {
      fetch(j + 1, nx);
      np = params(j + 1);
    }
    const bool kept = A.keep_n && q >= A.keep_first && q < A.keep_first + A.keep_n;
    if (kept) continue;  // k_whatif<2> (per-pair outputs)
    ksg_pod_summary* sm = A.sums + q;
    const int32_t feas_all = P.feas;
    const int64_t Mt = P.Mt, Ma = P.Ma;
    const bool skip_na = (P.flags & KPF_SKIP_NA_SCORE) != 0;
    // DefaultNormalizeScore quotients in 32 bits while 100 x max < 2^32 (the raw
    // fields are unsigned and <= their max); the seeded tie-break hash only for the
    // nodes at the wave's best total (a lower total cannot win)
    const bool n32 = Mt < 42949672 && Ma < 42949672;
    bool range_err = false;
    uint32_t fm = 0;
    uint64_t best = 0;
    if (n32 && A.small) {  // every total < 2^31: 32-bit sums, invariant-divisor quotients
      const UDiv dt = udiv_of(Mt > 0 ? (uint32_t)Mt : 1u), da = udiv_of(Ma > 0 ? (uint32_t)Ma : 1u);
      const uint32_t wt32 = (uint32_t)wt, wa32 = (uint32_t)wa;
      uint32_t tots[KSG_WI_R2NPT];
      uint32_t tmax = 0;
#pragma unroll
      for (int k = 0; k < KSG_WI_R2NPT; ++k) {
        const RT r = cur[k];
        tots[k] = 0;
        if (!(r & FEAS)) continue;
        fm |= 1u << k;
        range_err |= (r & RANGE) != 0;
        uint32_t tot = (uint32_t)((r >> sh_tot) & mtot);
        if (pt >= 0) {
          const uint32_t x = (uint32_t)((r >> sh_t) & mt_);
          const uint32_t s = Mt == 0 ? 100u : 100u - udiv(100u * x, dt);  // (reverse)
          range_err |= s > 100u;
          tot += s * wt32;
        }
        if (pa >= 0 && !skip_na) {
          const uint32_t x = (uint32_t)(r & ma_);
          const uint32_t s = Ma == 0 ? x : udiv(100u * x, da);
          range_err |= s > 100u;
          tot += s * wa32;
        }
        if (feas_all == 1) tot = 0;  // single feasible node: no scoring
        tots[k] = tot;
        tmax = tot > tmax ? tot : tmax;
      }
      const uint32_t wm = (uint32_t)wave_max((int64_t)(fm ? tmax : 0));
#pragma unroll
      for (int k = 0; k < KSG_WI_R2NPT; ++k) {
        if (((fm >> k) & 1u) && tots[k] == wm) {
          const uint64_t key = pack_key((int64_t)tots[k], F.seed, P.qidx, C.goff + base + k * 256);
          best = key > best ? key : best;
        }
      }
    } else {
      int64_t tots[KSG_WI_R2NPT];
      int64_t tmax = INT64_MIN;
#pragma unroll
      for (int k = 0; k < KSG_WI_R2NPT; ++k) {
        const RT r = cur[k];
        tots[k] = 0;
        if (!(r & FEAS)) continue;
        fm |= 1u << k;
        range_err |= (r & RANGE) != 0;
        int64_t tot = (int64_t)((r >> sh_tot) & mtot);
        if (pt >= 0) {
          const int64_t x = (int64_t)((r >> sh_t) & mt_);
          const int64_t s = Mt == 0 ? 100
                            : 100 - (n32 ? (int64_t)((uint32_t)(100 * x) / (uint32_t)Mt) : 100 * x / Mt);  // (reverse)
          range_err |= s < 0 || s > 100;
          tot += s * wt;
        }
        if (pa >= 0 && !skip_na) {
          const int64_t x = (int64_t)(r & ma_);
          const int64_t s = Ma == 0 ? x : (n32 ? (int64_t)((uint32_t)(100 * x) / (uint32_t)Ma) : 100 * x / Ma);
          range_err |= s < 0 || s > 100;
          tot += s * wa;
        }
        if (feas_all == 1) tot = 0;  // single feasible node: no scoring
        tots[k] = tot;
        tmax = tot > tmax ? tot : tmax;
      }
      const int64_t wm = wave_max(tmax);
#pragma unroll
      for (int k = 0; k < KSG_WI_R2NPT; ++k) {
        if (((fm >> k) & 1u) && tots[k] == wm) {
          const uint64_t key = pack_key(tots[k], F.seed, P.qidx, C.goff + base + k * 256);
          best = key > best ? key : best;
        }
      }
    }
    const uint64_t b = wave_max(best);
    if (lane0() && b) atomicMax((unsigned long long*)&sm->best_key, (unsigned long long)b);
    if (feas_all > 1 && __any(range_err) && lane0()) atomicOr((uint32_t*)&sm->status, 2u);
  }
}

// ---------------------------------------------------------------- what-if class path
// A what-if step of a Fit / BA (default arguments) + TaintToleration +
// NodeAffinity profile without the per-pair record round trip.  A (pod, node)
// total is fb + wt * reverse_norm(xt) + wa * norm(xa): fb is the node's Fit/BA
// weighted sum, xt the raw Taint score (node taints the pod prefers not to be
// on), xa the raw NodeAffinity score, the sum of the weights of the matched
// preferred terms.  Both normalisers are monotone and pod-wide, so for every
// class c = xt << np | (matched-term mask, np terms) the pair that wins inside
// c is the one with the largest (fb, tie-break) key — pack_key(fb, ...) — and
// the pod's winner is the best of its classes' winners once the maxima are
// known.  Pass 1 (k_whatif_cls1) keeps per block and pod the best key of each
// class in LDS (ds_max_u64) and writes one row of KSG_WC_CLS keys per (tile,
// pod); k_whatif_cls2 folds the tiles, derives the feasible count and the raw
// maxima / minima from the present classes, then normalises and picks.
// Nothing per pair reaches memory.
#define KSG_WC_CLS 128
#define KSG_WC_PODS 32
#define KSG_WC_NPT 4   // default nodes per thread (KSG_WC_NPT=1|2|4; 4 since round 6: 18.1 vs 18.5 ms/step)
#define KSG_WC_TILE 4096  // nodes per block

// A pod of the class path, decoded once per step (k_wc_decode) into a fixed
// layout that pass 1 reads with a few wide scalar loads per (pod, sub-tile):
// the program's header fields it needs as ready operands, and its node
// selector / required terms / preferred terms as ONE flat list of requirements,
// each tagged with the bit of the term it belongs to.  Pass 1 then evaluates
// every requirement on every node of the thread (no per-term loops, no ballots,
// no pointer chasing through the program) and folds the outcomes into a
// failed-term mask: bit 0 the node selector, bits 1..15 the required terms,
// bits 16..22 the preferred terms.  Host-checked per pod (prog_need bit 19):
// flattened requirements, <= 15 required terms, <= KSG_WC_MAXREQ requirements.
#define KSG_WC_MAXREQ 24
#define KSG_WC_PREF_BIT 16
struct WcReq {          // 32 B
  uint64_t col;         // the key's label column: element offset key * N into C.label
  uint64_t arg;         // value-id mask (modes 0 / 1) or the global node index (2 / 3)
  uint32_t gbit;        // the term's bit in the failed-term mask
  uint32_t mode;        // 0 value in mask, 1 not in mask (or no value), 2 name ==, 3 name !=, 4 false
  uint64_t pad;
};
struct WcPod {
  uint32_t flags;       // bit 0: no node passes; bit 1: PreFilterResult bitmap; bit 2: PreFilter rejected the
                        // pod (static records: not evaluated); bit 3: an empty required-terms list (NodeAffinity fails)
  uint32_t nreq;        // requirements in req[]
  uint32_t npf;         // scored preferred terms (the class's mask bits)
  uint32_t reqmask;     // bits of the required terms (0: no required-terms filter)
  uint64_t hw, pw;      // taint ids: untolerated NoSchedule/NoExecute, untolerated PreferNoSchedule
  uint64_t hseed;       // tie-break hash seed of the pod
  uint64_t roff;        // PreFilterResult bitmap (rwords words): byte offset into A.progs
  uint32_t rwords, pad0;
  double q0, q1;        // Fit filter requests (-inf: not requested)
  double fs0, fs1;      // Fit score requests
  double bq0, bq1;      // BalancedAllocation requests
  uint64_t pad1[3];     // (128-byte header)
  int32_t pwt[8];       // weights of the scored preferred terms (static records' raw NodeAffinity score)
  WcReq req[KSG_WC_MAXREQ];
};
static_assert(sizeof(WcReq) == 32 && sizeof(WcPod) == 160 + 32 * KSG_WC_MAXREQ, "WcPod layout");

// Is program h a class-path pod the decoder can flatten (prog_need bit 19)?
__host__ __device__ inline bool wc_decodable(const ksg_prog* h) {
  if (!(h->flags & KPF_FLAT_NA) || h->n_req_terms > 15 || h->n_pref_terms > 7) return false;
  const ksg_sel* sel = reinterpret_cast<const ksg_sel*>(reinterpret_cast<const uint8_t*>(h) + h->off_sel);
  auto cnt = [](const ksg_sel& x) { return x.kind == 0 ? 1 : x.req_cnt; };
  int n = (h->flags & KPF_HAS_NODE_SEL) ? cnt(h->node_sel) : 0;
  if (h->flags & KPF_HAS_REQ_NA)
    for (int t = 0; t < h->n_req_terms; ++t) n += cnt(sel[h->req_terms_off + t]);
  for (int t = 0; t < h->n_pref_terms; ++t) n += cnt(sel[h->pref_terms_off + t]);
  return n <= KSG_WC_MAXREQ;
}

// One thread per pod of the chunk: WcPod of pod q0 + j (run_whatif checked
// wc_decodable for every one).  The same outcome rules as freq_match / node_sel /
// required_na: a term of kind 0 matches no node, a key outside the vocabulary is
// absent from every node.
// glob: the PreFilterResult bitmap over every node (node-sharded static records)
__device__ __forceinline__ void wc_decode_one(const DevCluster& C, const DevProfile& F, const uint8_t* progs,
                                              uint64_t off, WcPod* __restrict__ outp, bool glob) {
  const ProgView V = view(progs + off);
  const ksg_prog* h = V.h;
  const uint32_t fl = h->flags;
  const bool ht = F.pos_taint >= 0, ha = F.pos_na >= 0;
  WcPod P{};
  P.flags = (fl & KPF_PREFILTER_REJECT) ? 5u : 0u;
  if (fl & KPF_RESTRICT) {
    P.flags |= 2u;
    P.roff = off + h->off_u32 + 4ull * (uint32_t)(glob ? h->restrict_g_off : h->restrict_off);
    P.rwords = (uint32_t)(glob ? h->restrict_g_words : h->restrict_words);
  }
  P.q0 = h->req[0] > 0 ? (double)h->req[0] : -INFINITY;
  P.q1 = h->req[1] > 0 ? (double)h->req[1] : -INFINITY;
  P.fs0 = (double)h->fit_score_req[0];
  P.fs1 = (double)h->fit_score_req[1];
  P.bq0 = (double)h->ba_req[0];
  P.bq1 = (double)h->ba_req[1];
  P.hseed = F.seed ^ ((uint64_t)(uint32_t)h->queue_idx * 0x9E3779B97F4A7C15ull);
  if (ht) {
    const uint32_t* hard = V.u32 + h->taint_hard_off;
    const uint32_t* pref = V.u32 + h->taint_pref_off;
    const int tw = h->taint_words;
    P.hw = tw > 1 ? ((uint64_t)hard[1] << 32 | hard[0]) : tw > 0 ? hard[0] : 0;
    P.pw = tw > 1 ? ((uint64_t)pref[1] << 32 | pref[0]) : tw > 0 ? pref[0] : 0;
  }
  uint32_t nr = 0;
  auto emit = [&](const ksg_sel& s, uint32_t gbit) {
    if (s.kind == 0) {
      P.req[nr++] = WcReq{0, 0, gbit, 4u, 0};
      return;
    }
    for (int i = 0; i < s.req_cnt; ++i) {
      const ksg_freq f = V.fq[s.req_off + i];
      WcReq r{0, f.arg, gbit, 4u, 0};
      if (f.mode == KFR_NAME_EQ || f.mode == KFR_NAME_NE) {
        r.mode = f.mode == KFR_NAME_EQ ? 2u : 3u;
      } else if (f.mode == KFR_ANY || f.mode == KFR_NONE) {
        if (f.key >= 0 && (uint32_t)f.key < C.K) {
          r.col = (uint64_t)(uint32_t)f.key * C.N;
          r.mode = f.mode == KFR_ANY ? 0u : 1u;
        } else if (f.mode == KFR_NONE) {
          continue;  // (no node has the key: the requirement holds everywhere)
        }
      }
      P.req[nr++] = r;
    }
  };
  if (ha && !(fl & KPF_SKIP_NA_FILTER)) {
    if (fl & KPF_HAS_NODE_SEL) emit(h->node_sel, 1u);
    if (fl & KPF_HAS_REQ_NA) {
      if (h->n_req_terms == 0) P.flags |= 9u;  // (no term to match: no node passes)
      for (int t = 0; t < h->n_req_terms; ++t) {
        emit(V.sel[h->req_terms_off + t], 1u << (1 + t));
        P.reqmask |= 1u << (1 + t);
      }
    }
  }
  P.npf = (ha && !(fl & KPF_SKIP_NA_SCORE)) ? (uint32_t)h->n_pref_terms : 0u;
  for (uint32_t t = 0; t < P.npf; ++t) {
    emit(V.sel[h->pref_terms_off + t], 1u << (KSG_WC_PREF_BIT + t));
    P.pwt[t] = V.i32[h->pref_w_off + t];
  }
  P.nreq = nr;
  *outp = P;
}
__global__ __launch_bounds__(64) void k_wc_decode(DevCluster C, DevProfile F, WiArgs A, WcPod* __restrict__ out) {
  const uint32_t j = blockIdx.x * 64 + threadIdx.x;
  if (j >= A.count) return;
  wc_decode_one(C, F, A.progs, A.prog_off[A.q0 + j], out + j, false);
}
// The chunk's pods of a static-record launch (k_static_dec), one thread each.
__global__ __launch_bounds__(64) void k_st_decode(DevCluster C, DevProfile F, const uint8_t* __restrict__ progs,
                                                  const uint64_t* __restrict__ prog_off, uint32_t q0, uint32_t count,
                                                  WcPod* __restrict__ out, int glob) {
  const uint32_t j = blockIdx.x * 64 + threadIdx.x;
  if (j >= count) return;
  wc_decode_one(C, F, progs, prog_off[q0 + j], out + j, glob != 0);
}

// k_static on decoded pods (the cfg5 class path's WcPod): the same records, no
// program walking per (pod, node).  A thread holds KSG_SD_NPT nodes — their
// taint ids in node order (<= 4, ids < 64: host-checked) — while the block's
// KSG_SD_PODS pods go by; each pod's flattened requirements are evaluated into a
// failed-term mask as in k_whatif_cls1.  Record: the first failing static
// filter in profile order (TaintToleration: its first untolerated taint in
// node.spec.taints order; NodeAffinity), else the raw scores; the static maxima
// over the statically feasible nodes per pod.
#define KSG_SD_PODS 8
#define KSG_SD_NPT 2
// One item of the static records: node tile bx (BT * KSG_SD_NPT nodes), pod group
// by (KSG_SD_PODS pods).  ready (non-null: the persistent window loop reads the
// records while they are computed beside it): records stored sc1, then — after
// every wave's stores and maxima have drained and a block barrier — one
// agent-scope add to the group's counter (MI355X_MICROARCH.md hand-off table,
// row 1); a group's records and maxima are complete once its counter reaches the
// number of node tiles.
template <int BT>
__device__ __forceinline__ void static_dec_item(const DevCluster& C, const DevProfile& F, const WcPod* __restrict__ pods,
                                                const uint8_t* __restrict__ progs, uint32_t count, StaticRec* out,
                                                int64_t* mpred, uint32_t* ready, uint32_t bx, uint32_t by) {
  const bool ht = F.pos_taint >= 0, ha = F.pos_na >= 0;
  const bool taint_first = ht && (!ha || F.pos_taint < F.pos_na);
  uint32_t n[KSG_SD_NPT], tcnt[KSG_SD_NPT];
  uint32_t tids[KSG_SD_NPT];  // four 8-bit ids in node order
  uint64_t ts[KSG_SD_NPT];
  bool live[KSG_SD_NPT];
#pragma unroll
  for (int k = 0; k < KSG_SD_NPT; ++k) {
    const uint32_t nn = bx * (BT * KSG_SD_NPT) + k * BT + threadIdx.x;
    live[k] = nn < C.N;
    n[k] = live[k] ? nn : 0u;
    const uint32_t t0 = C.toff[n[k]], tc = C.toff[n[k] + 1] - t0;
    uint32_t ids = 0;
    uint64_t w = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i)
      if (i < tc) {
        const uint32_t t = (uint32_t)C.tid[t0 + i] & 63u;
        ids |= t << (8 * i);
        w |= 1ull << t;
      }
    tcnt[k] = tc < 4 ? tc : 4;
    tids[k] = ids;
    ts[k] = w;
  }
#pragma unroll 1
  for (uint32_t pi = 0; pi < KSG_SD_PODS; ++pi) {
    const uint32_t j = by * KSG_SD_PODS + pi;
    if (j >= count) break;
    const WcPod& P = pods[j];
    const uint32_t fl = P.flags;
    uint32_t failm[KSG_SD_NPT];
#pragma unroll
    for (int k = 0; k < KSG_SD_NPT; ++k) failm[k] = 0;
    const uint32_t nreq = P.nreq;
#pragma unroll 1
    for (uint32_t r = 0; r < nreq; ++r) {
      const WcReq& R = P.req[r];
      const uint32_t mode = R.mode, gb = R.gbit;
      const uint64_t arg = R.arg;
      if (mode <= 1u) {
        const int32_t* col = C.label + R.col;
        int32_t v[KSG_SD_NPT];
#pragma unroll
        for (int k = 0; k < KSG_SD_NPT; ++k) v[k] = col[n[k]];
#pragma unroll
        for (int k = 0; k < KSG_SD_NPT; ++k) {
          const bool inset = v[k] >= 0 && ((arg >> ((uint32_t)v[k] & 63u)) & 1ull);
          failm[k] |= (inset != (mode == 0u)) ? gb : 0u;
        }
      } else {
#pragma unroll
        for (int k = 0; k < KSG_SD_NPT; ++k) {
          const bool eq = (uint64_t)(C.goff + n[k]) == arg;
          const bool m = mode == 4u ? false : (eq != (mode == 3u));
          failm[k] |= m ? 0u : gb;
        }
      }
    }
    const uint64_t hw = P.hw, pw = P.pw;
    const uint32_t reqm = P.reqmask, npf = P.npf;
    int64_t mt = -1, ma = -1;
#pragma unroll
    for (int k = 0; k < KSG_SD_NPT; ++k) {
      uint32_t code = KSG_FILTER_PASS, raw = 0;
      bool evaluated = !(fl & 4u);
      if (evaluated && (fl & 2u))
        evaluated = bit(reinterpret_cast<const uint32_t*>(progs + P.roff), (int)P.rwords, (int32_t)n[k]);
      if (!evaluated) {
        code = KSG_FILTER_NOT_EVALUATED;
      } else {
        // TaintToleration Filter: the node's first untolerated NoSchedule / NoExecute taint
        uint32_t tfail = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 3; i >= 0; --i) {
          const uint32_t t = (tids[k] >> (8 * i)) & 0xFFu;
          if ((uint32_t)i < tcnt[k] && ((hw >> t) & 1ull)) tfail = t;
        }
        const bool nfail = (fl & 8u) || (failm[k] & 1u) || (reqm != 0u && (~failm[k] & reqm) == 0u);
        if (taint_first) {
          if (tfail != 0xFFFFFFFFu) code = ((uint32_t)F.pos_taint << 24) | tfail;
          else if (ha && nfail) code = (uint32_t)F.pos_na << 24;
        } else {
          if (ha && nfail) code = (uint32_t)F.pos_na << 24;
          else if (ht && tfail != 0xFFFFFFFFu) code = ((uint32_t)F.pos_taint << 24) | tfail;
        }
        if (code == KSG_FILTER_PASS) {
          const int64_t t = ht ? (int64_t)__popcll(ts[k] & pw) : 0;
          int64_t a = 0;
#pragma unroll
          for (uint32_t u = 0; u < 8; ++u)
            if (u < npf && !((failm[k] >> (KSG_WC_PREF_BIT + u)) & 1u)) a += P.pwt[u];
          raw = ((uint32_t)t << 20) | ((uint32_t)a & KSG_RAW_NA_MASK);
          mt = t > mt ? t : mt;
          ma = a > ma ? a : ma;
        }
      }
      if (live[k]) {
        StaticRec* o = out + (size_t)j * C.N + n[k];
        if (ready) st_sc1(reinterpret_cast<uint64_t*>(o), (uint64_t)code | ((uint64_t)raw << 32));
        else *o = StaticRec{code, raw};
      }
    }
    const int64_t a0 = wave_max(mt), a1 = wave_max(ma);
    if (lane0()) {
      if (a0 >= 0) atomicMax((long long*)&mpred[2 * j], (long long)a0);
      if (a1 >= 0) atomicMax((long long*)&mpred[2 * j + 1], (long long)a1);
    }
  }
  if (ready) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ready + by, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__global__ __launch_bounds__(256) void k_static_dec(DevCluster C, DevProfile F, const WcPod* __restrict__ pods,
                                                    const uint8_t* __restrict__ progs, uint32_t count, StaticRec* out,
                                                    int64_t* mpred, uint32_t* ready) {
  static_dec_item<256>(C, F, pods, progs, count, out, mpred, ready, blockIdx.x, blockIdx.y);
}
// Beside the persistent window loop: a few 1,024-thread blocks (one per CU the
// loop leaves idle, launched BEFORE the loop so that the loop's blocks take the
// other CUs) walk the items group by group; when kernels run one at a time (a
// PMC profiling pass) it simply completes before the loop starts.
__global__ __launch_bounds__(1024) void k_static_dec_run(DevCluster C, DevProfile F, const WcPod* __restrict__ pods,
                                                         const uint8_t* __restrict__ progs, uint32_t count,
                                                         StaticRec* out, int64_t* mpred, uint32_t* ready, uint32_t ntx,
                                                         uint32_t items, uint32_t* arrive) {
  // (the loop's handshake goes only once every block of this grid has started: a
  // started block runs to its end, so the loop's gates on these records complete)
  if (threadIdx.x == 0) __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint32_t i = blockIdx.x; i < items; i += gridDim.x) {
    static_dec_item<1024>(C, F, pods, progs, count, out, mpred, ready, i % ntx, i / ntx);
    __syncthreads();  // (the item's registers and the next item's loads)
  }
}

// A node of the class path's pass 1, held in registers across the block's pods:
// the columns in doubles (exact: host-checked < 2^45), taints as an id set.
struct WcNode {
  double ad0, ad1;  // allocatable cpu / memory
  double ra0, ra1;  // reciprocals of ad0 / ad1, correctly rounded (1.0 / ad: one division per node)
  double fx0, fx1;  // (allocatable - NonZeroRequested) x 100, cpu / memory (Fit; exact: < 2^53)
  double rd0, rd1;  // Requested cpu / memory (BalancedAllocation)
  double fd0, fd1;  // allocatable - requested (Fit's filter)
  uint64_t ts;      // taint ids (< 64)
  uint32_t n;       // local node (0 when out of range)
  bool ok;          // in range and room for one more pod
};
// leastRequestedScore floor((a - q) * 100 / a) for integers 0 <= q <= a < 2^45
// held exactly in doubles: x = (a - q) * 100 < 2^52 is exact, the estimate from
// the reciprocal is the quotient or one off, the fma remainder is exact.
// The quotient lies in [0, 100]: the correction is done on the int32 estimate
// (one conversion instead of double selects and a 64-bit conversion).  x is
// (a - q) * 100, formed by the caller (pass 1: the node's (a - nonzero) * 100
// less the pod's request x 100, both exact integers, |x| < 2^53).
__device__ __forceinline__ int32_t least_req_d(double ad, double ra, double x) {
  const double d = trunc(x * ra);
  const double rem = __builtin_fma(-d, ad, x);
  return (int32_t)d + (rem >= ad ? 1 : 0) - (rem < 0.0 ? 1 : 0);
}

// Pass 1: grid x = group of KSG_WC_PODS pods (fastest: a tile's rows are shared
// in L2 by its pod groups), y = tile of KSG_WC_TILE nodes; each thread holds
// NPT nodes in registers while the block's pods go by, so a pod's program is
// decoded once per NPT x 64 pairs of a wave.  The filter and the scores are
// evaluated without branches per node (pass / fail selects the outcome); a pair
// whose Fit/BA sum is below its class's best so far skips the tie-break hash.
// Host-checked (run_whatif): default Fit / BA arguments, no resource column
// beyond cpu / memory requested, cpu / memory below 2^45 on the nodes and 2^44
// in the pods, <= 4 distinct taints per node with ids < 64, every pod's
// (taints + 1) << preferred terms <= KSG_WC_CLS.
template <int NPT>
__global__ __launch_bounds__(256) void k_whatif_cls1(DevCluster C, DevProfile F, WiArgs A,
                                                     const WcPod* __restrict__ pods) {
#pragma clang fp contract(off)
  __shared__ unsigned long long slot[KSG_WC_PODS][KSG_WC_CLS];
  __shared__ uint32_t wcnt[KSG_WC_PODS];
  const uint32_t tid = threadIdx.x;
  const uint32_t j0 = blockIdx.x * KSG_WC_PODS;
  const uint32_t np = min(A.count - j0, (uint32_t)KSG_WC_PODS);
  for (uint32_t i = tid; i < KSG_WC_PODS * KSG_WC_CLS; i += 256) (&slot[0][0])[i] = 0ull;
  if (tid < KSG_WC_PODS) wcnt[tid] = 0;
  __syncthreads();
  const bool hf = F.pos_fit >= 0, hb = F.pos_ba >= 0;
  const uint32_t wfit = (uint32_t)F.w_fit, wba = (uint32_t)F.w_ba;
#pragma unroll 1
  for (uint32_t sub = 0; sub < KSG_WC_TILE / (256 * NPT); ++sub) {
    const uint32_t nb = blockIdx.y * KSG_WC_TILE + sub * (256 * NPT);
    if (nb >= C.N) break;
    WcNode x[NPT];
    uint32_t n[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const uint32_t nn = nb + k * 256 + tid;
      const bool live = nn < C.N;
      n[k] = live ? nn : 0u;
      WcNode& v = x[k];
      v.n = n[k];
      const int64_t a0 = C.alloc[n[k]], a1 = C.alloc[(size_t)C.N + n[k]];
      const int64_t r0 = C.req[n[k]], r1 = C.req[(size_t)C.N + n[k]];
      v.ad0 = (double)a0;
      v.ad1 = (double)a1;
      v.ra0 = 1.0 / (v.ad0 != 0.0 ? v.ad0 : 1.0);
      v.ra1 = 1.0 / (v.ad1 != 0.0 ? v.ad1 : 1.0);
      v.rd0 = (double)r0;
      v.rd1 = (double)r1;
      v.fd0 = (double)(a0 - r0);
      v.fd1 = (double)(a1 - r1);
      v.fx0 = (v.ad0 - (double)C.nzc[n[k]]) * 100.0;
      v.fx1 = (v.ad1 - (double)C.nzm[n[k]]) * 100.0;
      v.ok = live && !(hf && C.podcnt[n[k]] + 1 > C.allowed[n[k]]);
      const uint32_t t0 = C.toff[n[k]], tc = C.toff[n[k] + 1] - t0;
      uint64_t w = 0;
#pragma unroll
      for (uint32_t i = 0; i < 4; ++i)
        if (i < tc) w |= 1ull << ((uint32_t)C.tid[t0 + i] & 63u);
      v.ts = w;
    }
#pragma unroll 1
    for (uint32_t pi = 0; pi < np; ++pi) {
      const WcPod& P = pods[j0 + pi];
      const uint32_t fl = P.flags;
      bool pass[NPT];
#pragma unroll
      for (int k = 0; k < NPT; ++k) pass[k] = x[k].ok && !(fl & 1u);
      if (fl & 2u) {
#pragma unroll
        for (int k = 0; k < NPT; ++k)
          pass[k] &= bit(reinterpret_cast<const uint32_t*>(A.progs + P.roff), (int)P.rwords, (int32_t)n[k]);
      }
      if (hf) {  // (the pod count was checked with the node; q = -inf when not requested)
        const double q0 = P.q0, q1 = P.q1;
#pragma unroll
        for (int k = 0; k < NPT; ++k) pass[k] &= !(q0 > x[k].fd0) & !(q1 > x[k].fd1);
      }
      uint32_t xt[NPT];
      {  // TaintToleration (a node's taints are distinct: the set counts them; zero sets without the plugin)
        const uint64_t hw = P.hw, pw = P.pw;
        if (((hw | pw) >> 32) == 0) {  // (the pod's sets name only ids < 32: 32-bit tests)
          const uint32_t hl = (uint32_t)hw, pl = (uint32_t)pw;
#pragma unroll
          for (int k = 0; k < NPT; ++k) {
            pass[k] &= ((uint32_t)x[k].ts & hl) == 0u;
            xt[k] = (uint32_t)__popc((uint32_t)x[k].ts & pl);
          }
        } else {
#pragma unroll
          for (int k = 0; k < NPT; ++k) {
            pass[k] &= (x[k].ts & hw) == 0;
            xt[k] = (uint32_t)__popcll(x[k].ts & pw);
          }
        }
      }
      // NodeAffinity: every flattened requirement on every node -> failed-term masks
      uint32_t failm[NPT], n4[NPT];
#pragma unroll
      for (int k = 0; k < NPT; ++k) n4[k] = n[k] * 4u;
#pragma unroll
      for (int k = 0; k < NPT; ++k) failm[k] = 0;
      const uint32_t nreq = P.nreq;
#pragma unroll 1
      for (uint32_t r = 0; r < nreq; ++r) {
        const WcReq& R = P.req[r];
        const uint32_t mode = R.mode, gb = R.gbit;
        const uint64_t arg = R.arg;
        if (mode <= 1u && !(arg >> 63)) {
          // (value id 63 not in the mask: a node without the key (-1, bit 63) tests
          // clear with no sign test; the outcome bit shifted straight into place)
          const uint8_t* col = reinterpret_cast<const uint8_t*>(C.label + R.col);
          const uint32_t sh = (uint32_t)__builtin_ctz(gb), m0 = mode == 0u ? 1u : 0u;
          uint32_t v[NPT];
#pragma unroll
          for (int k = 0; k < NPT; ++k) v[k] = *reinterpret_cast<const uint32_t*>(col + (uint64_t)n4[k]);
#pragma unroll
          for (int k = 0; k < NPT; ++k) failm[k] |= ((((uint32_t)(arg >> (v[k] & 63u))) & 1u) ^ m0) << sh;
        } else if (mode <= 1u) {
          const int32_t* col = C.label + R.col;
          int32_t v[NPT];
#pragma unroll
          for (int k = 0; k < NPT; ++k) v[k] = col[n[k]];
#pragma unroll
          for (int k = 0; k < NPT; ++k) {
            const bool inset = v[k] >= 0 && ((arg >> ((uint32_t)v[k] & 63u)) & 1ull);
            failm[k] |= (inset != (mode == 0u)) ? gb : 0u;
          }
        } else {
#pragma unroll
          for (int k = 0; k < NPT; ++k) {
            const bool eq = (uint64_t)(C.goff + n[k]) == arg;
            const bool m = mode == 4u ? false : (eq != (mode == 3u));
            failm[k] |= m ? 0u : gb;
          }
        }
      }
      const uint32_t reqm = P.reqmask;
      const int npf = (int)P.npf;
      uint32_t mask[NPT];
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        pass[k] &= !(failm[k] & 1u) & (reqm == 0u || (~failm[k] & reqm) != 0u);
        mask[k] = (~failm[k] >> KSG_WC_PREF_BIT) & ((1u << npf) - 1u);
      }
      // Fit (LeastAllocated, cpu:1 memory:1) and BalancedAllocation (cpu, memory)
      const double fs0 = P.fs0 * 100.0, fs1 = P.fs1 * 100.0;  // (exact: < 2^51)
      const double bq0 = P.bq0, bq1 = P.bq1;
      const uint64_t hseed = P.hseed;
      uint32_t nfeas = 0;  // (feasible nodes of the wave: ballots, on the scalar unit)
      bool rng = false;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const WcNode& v = x[k];
        const bool ok0 = v.ad0 != 0.0, ok1 = v.ad1 != 0.0;
        // (32-bit: the scores are in [0, 100] or flagged bad, 100 x the weights < 2^24: host-checked)
        uint32_t fb = 0;
        bool bad = false;
        if (hf) {
          // (q <= a  <=>  x = (a - q) x 100 >= 0)
          const double x0 = v.fx0 - fs0, x1 = v.fx1 - fs1;
          const int32_t s0 = (ok0 && v.ad0 > 0.0 && x0 >= 0.0) ? least_req_d(v.ad0, v.ra0, x0) : 0;
          const int32_t s1 = (ok1 && v.ad1 > 0.0 && x1 >= 0.0) ? least_req_d(v.ad1, v.ra1, x1) : 0;
          const int32_t ns = s0 + s1;
          const int32_t sc = ok0 && ok1 ? ns >> 1 : ns;
          bad |= sc < 0 || sc > 100;
          fb += (uint32_t)sc * wfit;
        }
        if (hb) {
          double sd = 0.0;
          if (ok0 && ok1) {
            // a / ad from the node's correctly rounded reciprocal y: q = a·y, then
            // one exact remainder (FMA) and q + r·y — Markstein's correction, which
            // returns the correctly rounded quotient (RN(a / ad), Go's float64
            // division) without a division per pair (3 f64 ops instead of ~11)
            const double a0 = v.rd0 + bq0, a1 = v.rd1 + bq1;
            const double e0 = a0 * v.ra0, e1 = a1 * v.ra1;
            double f0 = __builtin_fma(__builtin_fma(-v.ad0, e0, a0), v.ra0, e0);
            double f1 = __builtin_fma(__builtin_fma(-v.ad1, e1, a1), v.ra1, e1);
            f0 = __builtin_fmin(f0, 1.0);  // (never NaN: the same as f > 1 ? 1 : f)
            f1 = __builtin_fmin(f1, 1.0);
            sd = fabs((f0 - f1) / 2);
          }
          // (a value outside int32 saturates: still < 0 or > 100, i.e. bad)
          const int32_t sc = __double2int_rz((1 - sd) * 100.0);
          bad |= sc < 0 || sc > 100;
          fb += (uint32_t)sc * wba;
        }
        const uint32_t c = (xt[k] << npf) | mask[k];
        const uint64_t top = (uint64_t)(bad ? 0u : fb) << 40;
        // (a lower Fit/BA sum than the class's best so far cannot win the class)
        if (pass[k] && top >= (slot[pi][c] & ~0xFFFFFFFFFFull)) {
          const uint32_t g = C.goff + v.n;
          const uint64_t h20 = splitmix64(hseed ^ (uint64_t)g) >> 44;
          atomicMax(&slot[pi][c], (unsigned long long)(top | ((0xFFFFFull - h20) << 20) | (uint64_t)g));
        }
        nfeas += (uint32_t)__popcll(__ballot(pass[k]));
        rng |= pass[k] && bad;
      }
      const bool anyr = __ballot(rng) != 0;
      if (lane0() && (nfeas || anyr)) atomicAdd(&wcnt[pi], nfeas | (anyr ? 0x80000000u : 0u));
    }
  }
  __syncthreads();
  // this tile's row of every pod of the group
  const size_t tile = blockIdx.y, tiles = gridDim.y;
  for (uint32_t i = tid; i < np * KSG_WC_CLS; i += 256) {
    const uint32_t pi = i / KSG_WC_CLS, c = i % KSG_WC_CLS;
    A.wc_part[((size_t)(j0 + pi) * tiles + tile) * KSG_WC_CLS + c] = (&slot[0][0])[i];
  }
  if (tid < np) A.wc_cnt[(size_t)(j0 + tid) * tiles + tile] = wcnt[tid];
}

// Pass 2, one block of KSG_WC_CLS threads per pod (thread = class).  phase 0:
// fold + summary + pick (one shard); 1: fold + summary (the table kept for
// phase 2, after the shards' summaries are merged); 2: pick from the kept table.
__global__ __launch_bounds__(KSG_WC_CLS) void k_whatif_cls2(DevProfile F, WiArgs A, uint32_t tiles, int phase) {
  __shared__ int64_t red[2][6];
  __shared__ uint32_t rcnt[2];
  const uint32_t j = blockIdx.x, c = threadIdx.x, lane = c & 63, w = c >> 6;
  const uint32_t q = A.q0 + j;
  const ksg_prog* h = reinterpret_cast<const ksg_prog*>(A.progs + A.prog_off[q]);
  const ProgView V = view(A.progs + A.prog_off[q]);
  ksg_pod_summary* sm = A.sums + q;
  const int pt = F.pos_taint, pa = F.pos_na;
  const int npf = (pa >= 0 && !(h->flags & KPF_SKIP_NA_SCORE)) ? h->n_pref_terms : 0;
  uint64_t m = 0;
  uint32_t flag = 0;
  if (phase != 2) {
    const uint64_t* p = A.wc_part + (size_t)j * tiles * KSG_WC_CLS + c;
    uint64_t m0 = 0, m1 = 0;
    uint32_t t = 0;
    for (; t + 1 < tiles; t += 2) {
      const uint64_t a = p[(size_t)t * KSG_WC_CLS], b = p[(size_t)(t + 1) * KSG_WC_CLS];
      m0 = a > m0 ? a : m0;
      m1 = b > m1 ? b : m1;
    }
    if (t < tiles) m0 = p[(size_t)t * KSG_WC_CLS] > m0 ? p[(size_t)t * KSG_WC_CLS] : m0;
    m = m0 > m1 ? m0 : m1;
    // feasible count and Fit/BA range flag over the tiles
    uint32_t cs = 0, rf = 0;
    for (uint32_t u = c; u < tiles; u += KSG_WC_CLS) {
      const uint32_t x = A.wc_cnt[(size_t)j * tiles + u];
      cs += x & 0x7FFFFFFFu;
      rf |= x >> 31;
    }
    const int32_t cw = wave_sum((int32_t)cs);
    const bool rw = __ballot(rf != 0) != 0;
    if (lane == 0) rcnt[w] = (uint32_t)cw | (rw ? 0x80000000u : 0u);
  } else {
    m = A.wc_cls[(size_t)j * KSG_WC_CLS + c];
  }
  // the class's raw scores
  const bool present = m != 0;
  const int64_t xt = (int64_t)(c >> npf);
  int64_t xa = 0;
  for (int t = 0; t < npf; ++t)
    if ((c >> t) & 1u) xa += V.i32[h->pref_w_off + t];
  if (phase != 2) {
    int64_t v[4] = {present ? xt : INT64_MIN, present ? xt : INT64_MAX, present ? xa : INT64_MIN,
                    present ? xa : INT64_MAX};
    v[0] = wave_max(v[0]); v[1] = wave_min(v[1]); v[2] = wave_max(v[2]); v[3] = wave_min(v[3]);
    if (lane == 0) for (int i = 0; i < 4; ++i) red[w][i] = v[i];
    __syncthreads();
    const int32_t feas = (int32_t)((rcnt[0] & 0x7FFFFFFFu) + (rcnt[1] & 0x7FFFFFFFu));
    flag = (rcnt[0] | rcnt[1]) >> 31;
    if (c == 0) {
      sm->feasible = feas;
      if (feas) {
        if (pt >= 0) {
          sm->max_score[pt] = max(red[0][0], red[1][0]) > sm->max_score[pt] ? max(red[0][0], red[1][0]) : sm->max_score[pt];
          sm->min_score[pt] = min(red[0][1], red[1][1]) < sm->min_score[pt] ? min(red[0][1], red[1][1]) : sm->min_score[pt];
        }
        if (pa >= 0) {
          sm->max_score[pa] = max(red[0][2], red[1][2]) > sm->max_score[pa] ? max(red[0][2], red[1][2]) : sm->max_score[pa];
          sm->min_score[pa] = min(red[0][3], red[1][3]) < sm->min_score[pa] ? min(red[0][3], red[1][3]) : sm->min_score[pa];
        }
      }
    }
    if (phase == 1) {
      A.wc_cls[(size_t)j * KSG_WC_CLS + c] = m;
      if (c == 0) A.wc_flag[j] = flag;
      return;
    }
    __syncthreads();  // (the summary above is read back below)
  } else {
    flag = A.wc_flag[j];
  }
  const bool kept = A.keep_n && q >= A.keep_first && q < A.keep_first + A.keep_n;
  if (kept) return;  // k_whatif<2> (per-pair outputs)
  const int32_t feas_all = sm->feasible;
  const int64_t Mt = pt >= 0 ? sm->max_score[pt] : 0, Ma = pa >= 0 ? sm->max_score[pa] : 0;
  const int64_t wt = pt >= 0 ? F.weight[pt] : 0, wa = pa >= 0 ? F.weight[pa] : 0;
  bool range_err = false;
  uint64_t best = 0;
  if (present) {
    int64_t tot = (int64_t)(m >> 40);
    if (pt >= 0) {
      const int64_t s = Mt == 0 ? 100 : 100 - 100 * xt / Mt;  // (reverse)
      range_err |= s < 0 || s > 100;
      tot += s * wt;
    }
    if (pa >= 0 && !(h->flags & KPF_SKIP_NA_SCORE)) {
      const int64_t s = Ma == 0 ? xa : 100 * xa / Ma;
      range_err |= s < 0 || s > 100;
      tot += s * wa;
    }
    if (feas_all == 1) tot = 0;  // single feasible node: no scoring
    best = ((uint64_t)tot << 40) | (m & 0xFFFFFFFFFFull);
  }
  best = wave_max(best);
  range_err = __ballot(range_err) != 0;
  if (lane == 0) {
    red[w][4] = (int64_t)best;
    red[w][5] = range_err ? 1 : 0;
  }
  __syncthreads();
  if (c == 0) {
    const uint64_t b = (uint64_t)red[0][4] > (uint64_t)red[1][4] ? (uint64_t)red[0][4] : (uint64_t)red[1][4];
    if (b) atomicMax((unsigned long long*)&sm->best_key, (unsigned long long)b);
    if (feas_all > 1 && (flag || red[0][5] || red[1][5])) atomicOr((uint32_t*)&sm->status, 2u);
  }
}

// Index of global node gid in P_{W-1} (lane e of pn holds entry e's node), or -1.
__device__ __forceinline__ int pend_index(int32_t gid, int32_t pn, int np) {
  int hit = -1;
  for (int e = 0; e < np; ++e) hit = __builtin_amdgcn_readlane(pn, e) == gid ? e : hit;
  return hit;
}
// LDS-only barrier: __syncthreads() would also wait (vmcnt(0)) for this
// wave's per-pair output stores, which nothing after it depends on.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// per-pair outputs of one (pod, node) held back in LDS
struct PatchV {
  uint32_t code;
  int32_t fitba;  // raw Fit | raw BalancedAllocation << 16 (both in [0, 100])
  int32_t total;
  uint32_t raw;   // static record's raw Taint / NodeAffinity scores
};
// Persistent window loop: what the pod's merging eval block adds to the window's
// candidate record (in the rows area, which the replay then no longer reads): the
// pod evaluated on P_{W-1}'s nodes once the previous replay publishes them — the
// replay's "prior" step, off its critical path — and the rows of its shallow
// candidate ranks.  Deeper ranks' rows come from the node rows: a candidate that
// is no P_{W-1} node has the same row at the end of W-1 as at the end of W-2.
struct PriorRec {
  uint64_t pkey[KSG_BATCH];  // key on prior node e (0: infeasible)
  PatchV patch[KSG_BATCH];
  int32_t pdf[KSG_BATCH];    // feasible-count change vs the snapshot (byte 0); Taint / NodeAffinity profiles:
                             // the static-max achievers' changes in bytes 1 / 2 (each an int8)
  RowV row[KSG_STAGE];       // rows of candidate ranks < KSG_STAGE (window-start rows)
  uint64_t pmask, pbest;     // candidates that are prior nodes; the best prior key
  int32_t pbest_e, np;
};
__device__ __forceinline__ PriorRec* prior_rec(uint8_t* rec) { return reinterpret_cast<PriorRec*>(rec_rows(rec)); }
__device__ __forceinline__ const PriorRec* prior_rec(const uint8_t* rec) {
  return reinterpret_cast<const PriorRec*>(rec_rows(rec));
}
static_assert(KSG_BATCH * sizeof(PriorRec) <= kRecKeys * sizeof(RowV), "prior records fit the rows area");
static_assert(sizeof(PriorRec) % 8 == 0, "8-byte words");
// The merge of pod b's T tile lists into its candidate record (the pod's
// last-arriving tile block, or in the persistent loop its merge block): LDS L as
// win_eval's, h its pod record, pnl / np P_{E-2}'s nodes.
template <int MODE, bool STAT, bool PER>
__device__ __forceinline__ void win_merge(const DevCluster& C, const DevProfile& F, const WinArgs& A, uint32_t b, uint64_t* L,
                                          const PodLite* h, const int32_t* pnl, int np) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  (void)tid;
  auto pend_lds = [&](int32_t gid) {
    int hit = -1;
    for (int e = 0; e < np; ++e) hit = pnl[e] == gid ? e : hit;
    return hit;
  };
  // last tile block of pod b: merge the T tile lists (wave w takes tiles w, w+16, ...);
  // the lists and the tiles' counts are requested together.
  int32_t f[3] = {0, 0, 0};
  {
    const uint64_t* src = A.tile_top + (size_t)b * A.T * KSG_TOPK;
    uint64_t v = 0;
    if ((uint32_t)w < A.T) v = ld_agent(src + (size_t)w * KSG_TOPK + lane);
    if (w == 0)
      for (uint32_t t = lane; t < A.T; t += 64)
#pragma unroll
        for (int k = 0; k < 3; ++k)
          f[k] += __hip_atomic_load(A.tile_feas + ((size_t)b * A.T + t) * 3 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll 1
    for (uint32_t t = w + 16; t < A.T; t += 16) v = wave_merge_top(v, ld_agent(src + (size_t)t * KSG_TOPK + 63 - lane));
    L[w * 64 + lane] = v;
  }
  lds_barrier();
  int s0 = 1;  // (waves >= T hold no list: the tree starts at the level that covers T)
  while (s0 < (int)A.T && s0 < 16) s0 <<= 1;
#pragma unroll 1
  for (int s = s0 >> 1; s >= 1; s >>= 1) {
    if (w < s) L[w * 64 + lane] = wave_merge_top(L[w * 64 + lane], L[(w + s) * 64 + 63 - lane]);
    lds_barrier();
  }
  if (PER && w == 0) {  // (persistent loop: keys, counts, shallow rows, then the prior step)
    const uint64_t v = L[lane];
    const int32_t gid = (int32_t)(v & 0xFFFFFull);
    PriorRec* pr = prior_rec(A.erec) + b;
    stv<true>(rec_keys(A.erec) + (size_t)b * KSG_CAND + lane, v);
    if (lane < KSG_STAGE) {
      RowV c;
      memset(&c, 0, sizeof(c));
      if (v) {
        const int hh = pend_lds(gid);
        if (hh >= 0) c = ld_obj<true>(&A.pprev[hh].after);
        else load_row_p<true>(C, (uint32_t)gid - C.goff, A.need_eph, c);
      }
      st_obj<true>(&pr->row[lane], c);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) f[k] = wave_sum(f[k]);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) stv<true>(reinterpret_cast<int32_t*>(A.erec) + k * KSG_BATCH + b, f[k]);
      stv<true>(A.arrive + b * A.astride, 0u);
    }
    if (A.evk) {  // (split hand-over) keys, shallow rows and counts are out: the replay may stage them
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(A.evk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the prior step: pod q on P_{E-1}'s nodes (published by the replay of E-1);
    // prior_fix: the replay evaluates it itself
    int np1 = 0;
    Pend pe;
    pe.node = -1;
    if (A.pubw && !A.prior_fix) {
      uint32_t ok = 1;
      if (lane == 0) {
        ok = 0;
        for (uint32_t it = 0; it < A.spin; ++it) {
          if (ld_sc1(A.pubw) >= A.pub_need) { ok = 1; break; }
          if ((it & 63u) == 63u && ld_sc1(A.abortw) != 0u) break;
          __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) __hip_atomic_store(A.abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (__builtin_amdgcn_readfirstlane(ok)) {  // (else the run has aborted)
        // the count and every entry requested together (one round trip, not two)
        np1 = ldv<true>(A.pcur_n);
        if (lane < KSG_BATCH) pe = ld_obj<true>(A.pcur + lane);
      }
    }
    if (lane >= np1) pe.node = -1;
    uint64_t k = 0;
    if (lane < np1) {
      int32_t fs, bs;
      int64_t tot;
      const uint32_t R = C.R < 4 ? C.R : 4;
      StaticRec sr{KSG_FILTER_PASS, 0};
      uint32_t code;
      int64_t mt = 0, ma = 0;
      if (STAT) {  // (the static maxima and records were computed before the launch)
        const uint32_t q = A.e0 + b;
        mt = ldv<PER>(A.mpred + 2 * (q - A.first));
        ma = ldv<PER>(A.mpred + 2 * (q - A.first) + 1);
        sr = srec_at<PER>(A, q, (uint32_t)pe.node);
        code = eval_row_s<MODE>(pe.after, F, h, R, sr, mt, ma, fs, bs, tot);
      } else {
        code = eval_row<MODE>(pe.after, F, h, R, fs, bs, tot);
      }
      const bool snap_ok = sr.code == KSG_FILTER_PASS && (F.pos_fit < 0 || fit_filter_row(pe.base, h, R) == 0);
      PatchV pt;
      pt.code = code;
      pt.fitba = fs | (bs << 16);
      pt.total = (int32_t)tot;
      pt.raw = sr.raw;
      k = code == KSG_FILTER_PASS ? pack_key(tot, F.seed, h->queue_idx, (uint32_t)pe.node) : 0;
      stv<true>(&pr->pkey[lane], k);
      st_obj<true>(&pr->patch[lane], pt);
      const int df = (code == KSG_FILTER_PASS ? 1 : 0) - (snap_ok ? 1 : 0);
      int dT = 0, dA = 0;
      if (STAT) {
        const bool na_on = F.pos_na >= 0 && !(h->flags & KPF_SKIP_NA_SCORE);
        dT = F.pos_taint >= 0 && (int64_t)(sr.raw >> 20) == mt ? df : 0;
        dA = na_on && (int64_t)(sr.raw & KSG_RAW_NA_MASK) == ma ? df : 0;
      }
      stv<true>(&pr->pdf[lane], (int32_t)(((uint32_t)df & 0xFFu) | (((uint32_t)dT & 0xFFu) << 8) | (((uint32_t)dA & 0xFFu) << 16)));
    }
    bool isp = false;  // candidate `lane` is a P_{E-1} node
    for (int e = 0; e < np1; ++e) isp |= v != 0 && __builtin_amdgcn_readlane(pe.node, e) == gid;
    const unsigned long long pm = __ballot(isp);
    const uint64_t kb = wave_max(k);
    const unsigned long long mb = __ballot(kb != 0 && k == kb);
    if (lane == 0) {
      if (!A.prior_fix) {
        stv<true>(&pr->pmask, (uint64_t)pm);
        stv<true>(&pr->pbest, kb);
        stv<true>(&pr->pbest_e, (int32_t)(mb ? __ffsll((long long)mb) - 1 : -1));
        stv<true>(&pr->np, np1);
      }
      if (A.estamps) atomicMax((unsigned long long*)&A.estamps[10], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the pod's record is out (wave 0 stored all of it)
    if (lane == 0) __hip_atomic_fetch_add(A.evd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (w == 0) {
    uint64_t v = L[lane];
    RowV c;
    memset(&c, 0, sizeof(c));
    int32_t gid = (int32_t)(v & 0xFFFFFull);
    int hh = pend_lds(gid);
    if (v) {
      if (hh >= 0) c = ld_obj<PER>(&A.pprev[hh].after);
      else load_row_p<PER>(C, (uint32_t)gid - C.goff, A.need_eph, c);
    }
    stv<PER>(rec_keys(A.erec) + (size_t)b * KSG_CAND + lane, v);
    if (!A.xrows) st_obj<PER>(rec_rows(A.erec) + (size_t)b * KSG_CAND + lane, c);  // (sharded: rows from the replica)
#pragma unroll
    for (int k = 0; k < 3; ++k) f[k] = wave_sum(f[k]);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) stv<PER>(reinterpret_cast<int32_t*>(A.erec) + k * KSG_BATCH + b, f[k]);
      stv<PER>(A.arrive + b * A.astride, 0u);
      if (A.estamps) atomicMax((unsigned long long*)&A.estamps[10], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
    if constexpr (PER) {  // the pod's record is out (wave 0 stored all of it): the replay may stage it
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(A.evd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
// Persistent loop, dedicated merge block of pod b: waits for the pod's T tile
// lists (the arrival counter), then merges them (win_merge) while the tile blocks
// go on to the next window.
template <int MODE, bool STAT = false>
__device__ __forceinline__ bool win_merge_block(const DevCluster& C, const DevProfile& F, const WinArgs& A, uint32_t b,
                                                uint64_t* L) {
  const int tid = threadIdx.x;
  uint32_t* wcount = reinterpret_cast<uint32_t*>(L + 16 * 64);
  PodLite* h = reinterpret_cast<PodLite*>(wcount + 96);
  int32_t* pnl = reinterpret_cast<int32_t*>(wcount + 64);
  const uint32_t q = A.e0 + b;
  constexpr int kPodW = (int)(sizeof(PodLite) / 8);
  if (tid < kPodW) reinterpret_cast<uint64_t*>(h)[tid] = reinterpret_cast<const uint64_t*>(A.plite + q)[tid];
  if (tid == 0) {
    bool ok = false;
    for (uint32_t it = 0; it < A.spin; ++it) {
      if (ld_sc1(A.arrive + b * A.astride) >= A.T) { ok = true; break; }
      if ((it & 63u) == 63u && ld_sc1(A.abortw) != 0u) break;
      __builtin_amdgcn_s_sleep(4);
    }
    if (!ok) __hip_atomic_store(A.abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    wcount[17] = ok ? 1u : 0u;
  }
  __syncthreads();
  if (!wcount[17]) return false;
  // P_{E-2} only now: the tiles arrived, so their blocks saw it published (a merge
  // block may otherwise run a window ahead of the replay that writes it)
  const int np = ldv<true>(A.pprev_n);
  if (tid < np) pnl[tid] = ldv<true>(&A.pprev[tid].node);
  __syncthreads();
  win_merge<MODE, STAT, true>(C, F, A, b, L, h, pnl, np);
  return true;
}
// Blocks 1.. of k_window: one pod x KSG_TILE nodes per block.  Tile lists are
// handed to the pod's last-arriving block with sc1 stores/loads and an agent
// counter (MI355X_MICROARCH.md, hand-off table row 1).
template <int MODE, bool STAT, bool PER = false>
__device__ __forceinline__ void win_eval(const DevCluster& C, const DevProfile& F, const WinArgs& A, uint32_t blk, uint64_t* L) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t* wcount = reinterpret_cast<uint32_t*>(L + 16 * 64);
  const uint32_t b = blk / A.T, tile = blk - b * A.T, q = A.e0 + b;
  // LDS: keys [16][64] u64 | wcount u32[64] | P_{W-1} nodes i32[32] | pod record, normaliser | wave 0's outputs
  // (the pod's fields come from LDS: as vector loads behind the output stores
  // every one of them waited for all outstanding stores)
  PodLite* h = reinterpret_cast<PodLite*>(wcount + 96);
  int64_t* mlds = reinterpret_cast<int64_t*>(wcount + 96 + sizeof(PodLite) / 4);
  // the first node's row from memory, issued before the P_{W-1} list it may be
  // replaced from (one round trip less ahead of the first evaluation)
  RowV rnext;
  {
    const uint32_t nn0 = tile * A.tile_len + tid;
    if ((uint32_t)tid < A.tile_len && nn0 < C.N) load_row_p<PER>(C, nn0, A.need_eph, rnext);
  }
  {
    constexpr int kPodW = (int)(sizeof(PodLite) / 8);
    if (tid < kPodW) reinterpret_cast<uint64_t*>(h)[tid] = reinterpret_cast<const uint64_t*>(A.plite + q)[tid];
    if (STAT && tid < 2) mlds[tid] = ldv<PER>(A.mpred + 2 * (q - A.first) + tid);
  }
  const int np = ldv<PER>(A.pprev_n);
  // P_{W-1}'s nodes in LDS (a lookup through LDS: a VGPR loaded from memory and
  // read lane by lane in a loop made the compiler wait for every outstanding
  // load and store, vmcnt(0), at each lookup)
  int32_t* pnl = reinterpret_cast<int32_t*>(wcount + 64);
  if (tid < np) pnl[tid] = ldv<PER>(&A.pprev[tid].node);
  lds_barrier();
  auto pend_lds = [&](int32_t gid) {
    int hit = -1;
    for (int e = 0; e < np; ++e) hit = pnl[e] == gid ? e : hit;
    return hit;
  };
  const uint64_t t_start = A.estamps ? __builtin_amdgcn_s_memrealtime() : 0;
  if (A.estamps && tid == 0) {
    atomicMax((unsigned long long*)&A.estamps[8], ~(unsigned long long)t_start);
    atomicMax((unsigned long long*)&A.estamps[30], (unsigned long long)t_start);
  }
  // a tile is KSG_TILE * A.npt nodes: each wave keeps the top 64 of its npt x 64 keys
  uint64_t top = 0;
  uint32_t cF = 0, cT = 0, cA = 0;
  const bool est = A.estamps && tid == 960;  // wave 15: writes its outputs directly
  uint64_t t_eval = 0, t_sort = 0, t_wait = 0;
#define KSG_ETIME(v)                             \
  __builtin_amdgcn_sched_barrier(0);         \
  const uint64_t v = __builtin_amdgcn_s_memtime(); \
  __builtin_amdgcn_sched_barrier(0);
  // per-pair outputs wait in LDS and are written once the tile list is handed
  // over: wave 0's arrival waits (vmcnt) for all of its stores, and every
  // wave's next-node loads would wait behind its previous node's stores.
  // Tiles of more than KSG_STASH_NPT nodes per thread: only wave 0 stashes.
  PatchV* stash = reinterpret_cast<PatchV*>(wcount + 192);
  const bool stash_all = A.npt <= A.stash_npt;
  static_assert(96 * 4 + sizeof(PodLite) + 16 <= 192 * 4, "eval LDS layout");
  // the next node's row and static record are loaded while this one is evaluated
  auto fetch = [&](uint32_t kk, RowV& r, StaticRec& sr, bool loaded) {
    const uint32_t to = kk * KSG_TILE + tid, nn = tile * A.tile_len + to;
    if (to < A.tile_len && nn < C.N) {
      const int hit = pend_lds((int32_t)(C.goff + nn));
      if (hit >= 0) r = ld_obj<PER>(&A.pprev[hit].after);
      else if (!loaded) load_row_p<PER>(C, nn, A.need_eph, r);
      if (STAT) sr = srec_at<PER>(A, q, C.goff + nn);
    }
  };
  StaticRec snext{KSG_FILTER_PASS, 0};
  fetch(0, rnext, snext, true);
#pragma unroll 1
  for (uint32_t k = 0; k < A.npt; ++k) {
  KSG_ETIME(t0);
  if (A.estamps && w == 15) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // diagnostic: load wait
  KSG_ETIME(tl);
  t_wait += tl - t0;
  const uint32_t to = k * KSG_TILE + tid, n = tile * A.tile_len + to;
  const RowV r = rnext;
  const StaticRec sr = snext;
  if (k + 1 < A.npt) fetch(k + 1, rnext, snext, false);
  uint64_t key = 0;
  bool feasible = false, achT = false, achA = false;
  if (to < A.tile_len && n < C.N) {
    int32_t fit_s, ba_s;
    int64_t total;
    uint32_t code, raw = 0;
    if (STAT) {
      const int64_t MT = mlds[0], MA = mlds[1];
      code = eval_row_s<MODE>(r, F, h, C.R < 4 ? C.R : 4, sr, MT, MA, fit_s, ba_s, total);
      raw = sr.raw;
      achT = F.pos_taint >= 0 && (int64_t)(raw >> 20) == MT;
      achA = F.pos_na >= 0 && !(h->flags & KPF_SKIP_NA_SCORE) && (int64_t)(raw & KSG_RAW_NA_MASK) == MA;
    } else {
      code = eval_row<MODE>(r, F, h, C.R < 4 ? C.R : 4, fit_s, ba_s, total);
    }
    if (stash_all || w == 0) {
      stash[(stash_all ? k * 16 + w : k) * 64 + lane] = PatchV{code, fit_s | (ba_s << 16), (int32_t)total, raw};
    } else {
      uint32_t* of;
      int32_t *os, *ot;
      out_ptrs(A, q, C.N, of, os, ot);
      // (persistent loop: kept outputs sc1 — the replay may patch them from
      // another XCD; the scratch ring of the others is never read)
      if (PER && kept_q(A, q)) write_pair<STAT, true>(F, of, os, ot, C.N, n, code, fit_s, ba_s, total, raw);
      else write_pair<STAT, false>(F, of, os, ot, C.N, n, code, fit_s, ba_s, total, raw);
    }
    if (code == KSG_FILTER_PASS) {
      feasible = true;
      key = pack_key(total, F.seed, h->queue_idx, C.goff + n);
    }
  }
  cF += (uint32_t)__popcll(__ballot(feasible));
  if (STAT) {
    cT += (uint32_t)__popcll(__ballot(feasible && achT));
    cA += (uint32_t)__popcll(__ballot(feasible && achA));
  }
  KSG_ETIME(t1);
  key = wave_sort_desc(key);
  top = k == 0 ? key : wave_merge_top(top, wave_reverse(key));
  KSG_ETIME(t2);
  t_eval += t1 - t0;
  t_sort += t2 - t1;
  }
  KSG_ETIME(t3);
  L[w * 64 + lane] = top;
  if (lane == 0) {
    wcount[w] = cF;
    wcount[32 + w] = cT;
    wcount[48 + w] = cA;
  }
  lds_barrier();
#pragma unroll 1
  for (int s = 8; s >= 1; s >>= 1) {
    if (w < s) L[w * 64 + lane] = wave_merge_top(L[w * 64 + lane], L[(w + s) * 64 + 63 - lane]);
    lds_barrier();
  }
  if (w == 0) {
    uint64_t* dst = A.tile_top + ((size_t)b * A.T + tile) * KSG_TOPK;
    __hip_atomic_store(dst + lane, L[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane < 3) {  // feasible nodes, Taint / NodeAffinity static-max achievers among them
      const int off = lane == 0 ? 0 : 16 + 16 * lane;
      int32_t c = 0;
      for (int k = 0; k < 16; ++k) c += (int32_t)wcount[off + k];
      __hip_atomic_store(A.tile_feas + ((size_t)b * A.T + tile) * 3 + lane, c, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    if (A.defer) {
      if (lane == 0) wcount[16] = 0u;
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      uint32_t old = 0;
      if (lane == 0) old = __hip_atomic_fetch_add(A.arrive + b * A.astride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      old = __builtin_amdgcn_readfirstlane(old);
      if (lane == 0) wcount[16] = (!A.mblocks && old == A.T - 1) ? 1u : 0u;  // (slots 17..31 unused)
    }
  }
  auto flush_stash = [&]() {
    if (!stash_all && w != 0) return;
    uint32_t* of;
    int32_t *os, *ot;
    out_ptrs(A, q, C.N, of, os, ot);
#pragma unroll 1
    for (uint32_t k = 0; k < A.npt; ++k) {
      const uint32_t to = k * KSG_TILE + tid, n = tile * A.tile_len + to;
      if (to >= A.tile_len || n >= C.N) break;
      const PatchV pt = stash[(stash_all ? k * 16 + w : k) * 64 + lane];
      if (PER && kept_q(A, q)) write_pair<STAT, true>(F, of, os, ot, C.N, n, pt.code, pt.fitba & 0xFFFF, pt.fitba >> 16, pt.total, pt.raw);
      else write_pair<STAT, false>(F, of, os, ot, C.N, n, pt.code, pt.fitba & 0xFFFF, pt.fitba >> 16, pt.total, pt.raw);
    }
  };
  // (persistent loop) this block's outputs are written: the replay may patch them
  auto signal_flushed = [&]() {
    if constexpr (PER) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(A.flushed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  lds_barrier();
  KSG_ETIME(t4);
#undef KSG_ETIME
  if (est) {
    atomicAdd((unsigned long long*)&A.estamps[13], (unsigned long long)t_eval);
    atomicAdd((unsigned long long*)&A.estamps[14], (unsigned long long)t_sort);
    atomicAdd((unsigned long long*)&A.estamps[15], (unsigned long long)(t4 - t3));
    atomicAdd((unsigned long long*)&A.estamps[18], (unsigned long long)t_wait);
  }
  if (A.estamps && tid == 0) {
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_sched_barrier(0);
    atomicMax((unsigned long long*)&A.estamps[9], (unsigned long long)t);
    atomicMax((unsigned long long*)&A.estamps[28], (unsigned long long)(t - t_start));
    atomicAdd((unsigned long long*)&A.estamps[29], (unsigned long long)(t - t_start));
    atomicAdd((unsigned long long*)&A.estamps[31], 1ull);
  }
  if (!wcount[16]) {
    flush_stash();
    signal_flushed();
    return;
  }
  win_merge<MODE, STAT, PER>(C, F, A, b, L, h, pnl, np);
  flush_stash();
  signal_flushed();
}

// ---- block 0: exact replay of window W as a fixed-point (Jacobi) iteration.
//
// Pod b's outcome is a function of the picks of pods < b only: S_b =
// f_b(S_0..S_{b-1}) = the best of (its candidates no earlier pick and no
// node of P_{W-1} touched; the nodes of P_{W-1} and the earlier picks,
// re-evaluated on their current rows).  A vector S with S_b == f_b(S_<b) for
// every b IS the sequential schedule (induction on b), so all pods iterate
// S <- f(S) at once until nothing changes; if pods < p were right and the first
// change of an iteration is at d >= p, pods <= d are right after it, so the
// stable prefix grows every iteration.  The starting guess is the greedy
// "best candidate or P_{W-1} node no earlier pod took" (serial dictatorship,
// computed in parallel rounds); on cfg2 it is right in ~2/3 of the windows.
//
// Lanes: wave w owns pods w and w+16.  Evaluations of modified nodes pack both
// pods in one wave instruction stream (lanes 0..31: pod w, 32..63: pod w+16,
// lane&31 = the earlier pick a it re-evaluates); the per-pod reduction then
// covers 64 candidate lanes + 32 P_{W-1} lanes + its 32 pick lanes.
struct SumLite {
  uint64_t best_key;
  int32_t selected, feasible, status, pad;
};
struct Delta {
  int64_t req[4];
  int64_t nzc, nzm;
  int32_t pods;
};
#define KSG_HSLOTS 128  // LDS hash tables: node -> prior entry / picks (<= 32 keys each)
struct PickTab {        // nodes picked by the window's pods under one iteration's S
  int32_t node[KSG_HSLOTS];  // -1 empty
  int32_t first[KSG_HSLOTS], last[KSG_HSLOTS], cnt[KSG_HSLOTS];
};
struct WinLDS {
  uint64_t key[KSG_BATCH][KSG_CAND];    // candidate keys (sorted, 0 = none)
  RowV row[KSG_BATCH][KSG_STAGE];       // rows of candidate ranks < KSG_STAGE
  Pend prior[KSG_BATCH];                // P_{W-1}
  PodLite pod[KSG_BATCH];
  PatchV patch[KSG_BATCH][KSG_CAND];    // [pod][prior e | 32 + pick a]
  uint64_t pkey[KSG_BATCH][KSG_BATCH];  // key of pod b on prior node e as of the window start
  int8_t pdf[KSG_BATCH][KSG_BATCH];     // its feasible-count change vs the snapshot
  uint64_t pmask[KSG_BATCH];            // bit i: candidate i of pod b is a prior node
  uint32_t nxt_ok;                      // (persistent loop) the next window's records were complete at the flush
  uint64_t pbest[KSG_BATCH];
  int32_t pbest_e[KSG_BATCH];
  int32_t S[3][KSG_BATCH];              // picks (global node, -1 none), rotating buffers
  int32_t O[3][KSG_BATCH];              // pick origins: prior e (< 32) or 64 + pod*64 + rank
  int32_t feas[KSG_BATCH];              // snapshot feasible counts
  SumLite sum[KSG_BATCH];
  int32_t ptn[KSG_HSLOTS], pte[KSG_HSLOTS];  // prior node -> entry
  int32_t gtn[KSG_HSLOTS], gtf[KSG_HSLOTS];  // guess rounds: node -> smallest proposer
  PickTab pick[3];                      // per S buffer
  uint64_t kc[KSG_BATCH][KSG_CAND];     // per iteration: candidate keys, 0 where the node was touched
  uint64_t rk[KSG_BATCH][KSG_BATCH];    // per iteration: key of pod b on the node pod a < b picked
  int8_t rdf[KSG_BATCH][KSG_BATCH];     // its feasible-count change vs the snapshot
  int32_t pf[KSG_BATCH];                // per iteration: first pick of P_{W-1} node e
  // Taint / NodeAffinity profiles (STAT): NormalizeScore's max is the static max
  // (mt, ma) while a feasible node reaches it; achiever counts track that
  int32_t achT[KSG_BATCH], achA[KSG_BATCH];  // snapshot achievers
  int64_t mt[KSG_BATCH], ma[KSG_BATCH];      // static maxima (-1: no statically feasible node)
  int64_t xmt[KSG_BATCH], xma[KSG_BATCH];    // normaliser of the pod's result (exact on fallback)
  int8_t pdfT[KSG_BATCH][KSG_BATCH], pdfA[KSG_BATCH][KSG_BATCH];  // achiever changes: prior nodes
  int8_t rdfT[KSG_BATCH][KSG_BATCH], rdfA[KSG_BATCH][KSG_BATCH];  // and picks
  int32_t fbf[KSG_BATCH];                    // pod needs the exact full re-evaluation (no achiever left)
  uint64_t red[16][4];                       // block reductions of the fallback
};

static_assert(sizeof(WinLDS) <= 160 * 1024, "window LDS exceeds the CU's 160 KiB");
// eval blocks: keys [16][64] u64 + 192 u32 of counters / pod record, then the stash
static constexpr uint32_t kStashNpt =
    (uint32_t)std::min<size_t>(KSG_STASH_NPT, (sizeof(WinLDS) - (16 * 64 * 8 + 192 * 4)) / (16 * 64 * sizeof(PatchV)));
static_assert(kStashNpt >= 1, "eval blocks' output stash exceeds the window LDS");
__device__ __forceinline__ uint32_t hslot(int32_t node) { return ((uint32_t)node * 2654435761u) >> 25; }
__device__ __forceinline__ int prior_of(const WinLDS& L, int32_t x) {
  uint32_t h = hslot(x);
  for (int k = 0; k < KSG_HSLOTS; ++k) {
    int32_t v = L.ptn[h];
    if (v == x) return L.pte[h];
    if (v == -1) return -1;
    h = (h + 1) & (KSG_HSLOTS - 1);
  }
  return -1;
}
// slot of node x in an open-addressing table (inserting it when absent)
__device__ __forceinline__ uint32_t tab_claim(int32_t* nodes, int32_t x) {
  uint32_t h = hslot(x);
  for (int k = 0; k < KSG_HSLOTS; ++k) {
    int32_t old = atomicCAS(&nodes[h], -1, x);
    if (old == -1 || old == x) return h;
    h = (h + 1) & (KSG_HSLOTS - 1);
  }
  return 0;  // unreachable: <= 64 keys in 128 slots
}
__device__ __forceinline__ int tab_find(const int32_t* nodes, int32_t x) {
  uint32_t h = hslot(x);
  for (int k = 0; k < KSG_HSLOTS; ++k) {
    int32_t v = nodes[h];
    if (v == x) return (int)h;
    if (v == -1) return -1;
    h = (h + 1) & (KSG_HSLOTS - 1);
  }
  return -1;
}
__device__ __forceinline__ void pick_insert(PickTab& T, int32_t x, int b) {
  uint32_t h = tab_claim(T.node, x);
  atomicMin(&T.first[h], b);
  atomicMax(&T.last[h], b);
  atomicAdd(&T.cnt[h], 1);
}
__device__ __forceinline__ void pick_clear(PickTab& T, int i) {  // i < KSG_HSLOTS
  T.node[i] = -1;
  T.first[i] = KSG_BATCH;
  T.last[i] = -1;
  T.cnt[i] = 0;
}
// first pod picking node x under T (KSG_BATCH: none)
__device__ __forceinline__ int first_pick(const PickTab& T, int32_t x) {
  int h = x >= 0 ? tab_find(T.node, x) : -1;
  return h >= 0 ? T.first[h] : KSG_BATCH;
}

#define KSG_ORG_NODE 0x40000000  // pick origin: node (o & 0xFFFFF) read from the node rows (fallback picks)
template <bool PER = false>
__device__ __forceinline__ void origin_rows(const DevCluster& C, const WinLDS& L, const WinArgs& A, int32_t o,
                                            RowV& start, RowV& snap) {
  if (o & KSG_ORG_NODE) {
    if (A.xrows) start = A.xrows[o & 0xFFFFF];  // (node-sharded: the replica holds every node)
    else load_row(C, (uint32_t)(o & 0xFFFFF) - C.goff, A.need_eph, start);
    snap = start;
  } else if (o < KSG_BATCH) {
    start = L.prior[o].after;
    snap = L.prior[o].base;
  } else {
    int p = (o - 64) >> 6, i = (o - 64) & 63;
    if (i < KSG_STAGE) start = L.row[p][i];
    else if (A.defer || PER) load_row_p<PER>(C, (uint32_t)(L.key[p][i] & 0xFFFFFull) - C.goff, A.need_eph, start);
    else start = rec_rows(A.wrec)[p * KSG_CAND + i];
    snap = start;
  }
}
__device__ __forceinline__ void delta_of(const PodLite& p, Delta& d) {
#pragma unroll
  for (int k = 0; k < 4; ++k) d.req[k] = p.req[k];
  d.nzc = p.nz_cpu;
  d.nzm = p.nz_mem;
  d.pods = 1;
}
__device__ __forceinline__ void delta_add(Delta& d, const PodLite& p) {
#pragma unroll
  for (int k = 0; k < 4; ++k) d.req[k] += p.req[k];
  d.nzc += p.nz_cpu;
  d.nzm += p.nz_mem;
  d.pods += 1;
}
__device__ __forceinline__ void apply_delta(RowV& r, const Delta& d, uint32_t R) {
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
    if (k < R) r.req[k] += d.req[k];
  r.nzc += d.nzc;
  r.nzm += d.nzm;
  r.podcnt += d.pods;
}
// Requests of the picks of node S[a] by pods <= a, and the next pod after a picking it.
__device__ __forceinline__ void pick_chain(const WinLDS& L, const int32_t* S, int a, int32_t x, Delta& cum, int& nx) {
  cum = Delta{};
  nx = KSG_BATCH;
  for (int j = 0; j < KSG_BATCH; ++j)
    if (S[j] == x) {
      if (j <= a) delta_add(cum, L.pod[j]);
      else if (nx == KSG_BATCH) nx = j;
    }
}
__device__ __forceinline__ uint64_t max3u(uint64_t a, uint64_t b, uint64_t c) {
  uint64_t m = a > b ? a : b;
  return m > c ? m : c;
}

// Pod b's row of global node g under the picks S of the pods < b (a local node's
// row from the node rows, another shard's from the replica).
template <bool PER = false>
__device__ __forceinline__ void row_under(const DevCluster& C, const WinLDS& L, const WinArgs& A, const int32_t* S,
                                          const PickTab& T, int b, uint32_t gu, uint32_t R, RowV& r) {
  const int32_t g = (int32_t)gu;
  const int e = prior_of(L, g);
  if (e >= 0) r = L.prior[e].after;
  else if (A.xrows) r = A.xrows[g];
  else load_row_p<PER>(C, gu - C.goff, A.need_eph, r);  // (persistent loop: rows this block rewrites)
  const int hs = tab_find(T.node, g);
  if (hs >= 0 && T.first[hs] < b) {
    Delta cum{};
    for (int j = 0; j < b; ++j)
      if (S[j] == g) delta_add(cum, L.pod[j]);
    apply_delta(r, cum, R);
  }
}
// STAT profiles, no feasible node of pod b left at the static max (rare): its
// exact result under S = L.S[cur] from two block-wide passes over all nodes —
// the normaliser over the feasible nodes, then the argmax — into L.S[nxt][b].
template <int MODE, bool PER = false>
__device__ __forceinline__ void win_exact_select(const DevCluster& C, const DevProfile& F, const WinArgs& A, WinLDS& L,
                                              int b, int cur, int nxt, uint32_t R) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const PodLite* h = &L.pod[b];
  const int32_t* S = L.S[cur];
  const PickTab& T = L.pick[cur];
  // every node of the cluster: node-sharded, from the replica and the global records
  const uint32_t g0 = A.xrows ? 0u : C.goff, gn = A.xrows ? A.G : C.N;
  int32_t feas = 0;
  int64_t lt = 0, la = 0;
#pragma unroll 1
  for (uint32_t i = tid; i < gn; i += KSG_WIN_THREADS) {
    RowV r;
    row_under<PER>(C, L, A, S, T, b, g0 + i, R, r);
    const StaticRec sr = srec_at<PER>(A, A.w0 + b, g0 + i);
    int32_t fs, bs;
    int64_t tot;
    if (eval_row_s<MODE>(r, F, h, R, sr, 0, 0, fs, bs, tot) == KSG_FILTER_PASS) {
      ++feas;
      lt = max(lt, (int64_t)(sr.raw >> 20));
      la = max(la, (int64_t)(sr.raw & KSG_RAW_NA_MASK));
    }
  }
  feas = wave_sum(feas);
  lt = wave_max(lt);
  la = wave_max(la);
  if (lane == 0) {
    L.red[wave][0] = (uint64_t)feas;
    L.red[wave][1] = (uint64_t)lt;
    L.red[wave][2] = (uint64_t)la;
  }
  lds_barrier();
  int32_t fa = 0;
  int64_t mt = 0, ma = 0;
  for (int w = 0; w < KSG_WIN_THREADS / 64; ++w) {
    fa += (int32_t)L.red[w][0];
    mt = max(mt, (int64_t)L.red[w][1]);
    ma = max(ma, (int64_t)L.red[w][2]);
  }
  uint64_t best = 0;
#pragma unroll 1
  for (uint32_t i = tid; i < gn; i += KSG_WIN_THREADS) {
    RowV r;
    row_under<PER>(C, L, A, S, T, b, g0 + i, R, r);
    int32_t fs, bs;
    int64_t tot;
    if (eval_row_s<MODE>(r, F, h, R, srec_at<PER>(A, A.w0 + b, g0 + i), mt, ma, fs, bs, tot) == KSG_FILTER_PASS) {
      const uint64_t k = pack_key(tot, F.seed, h->queue_idx, g0 + i);
      best = k > best ? k : best;
    }
  }
  best = wave_max(best);
  if (lane == 0) L.red[wave][3] = best;
  lds_barrier();
  if (tid == 0) {
    uint64_t bk = 0;
    for (int w = 0; w < KSG_WIN_THREADS / 64; ++w) bk = L.red[w][3] > bk ? L.red[w][3] : bk;
    const int32_t sel = (fa > 0 && bk) ? (int32_t)(bk & 0xFFFFFull) : -1;
    int32_t org = -1;
    if (sel >= 0) {
      const int e = prior_of(L, sel);
      org = e >= 0 ? e : (KSG_ORG_NODE | sel);
      pick_insert(L.pick[nxt], sel, b);
    }
    L.S[nxt][b] = sel;
    L.O[nxt][b] = org;
    SumLite& sm = L.sum[b];
    sm.best_key = sel >= 0 ? (fa == 1 ? (bk & 0xFFFFFFFFFFull) : bk) : 0;
    sm.selected = sel;
    sm.feasible = fa;
    sm.status = sel >= 0 ? 0 : 1;
    L.xmt[b] = mt;
    L.xma[b] = (h->flags & KPF_SKIP_NA_SCORE) ? 0 : ma;
  }
}
// ... and, once S is final, every per-pair output of such a pod.
template <int MODE, bool PER = false>
__device__ __forceinline__ void win_exact_write(const DevCluster& C, const DevProfile& F, const WinArgs& A, WinLDS& L,
                                             int b, int cur, uint32_t R) {
  const PodLite* h = &L.pod[b];
  uint32_t* of;
  int32_t *os, *ot;
  out_ptrs(A, A.w0 + b, C.N, of, os, ot);
  const int64_t mt = L.xmt[b], ma = L.xma[b];
#pragma unroll 1
  for (uint32_t i = threadIdx.x; i < C.N; i += KSG_WIN_THREADS) {  // (this shard's outputs)
    RowV r;
    row_under<PER>(C, L, A, L.S[cur], L.pick[cur], b, C.goff + i, R, r);
    const StaticRec sr = srec_at<PER>(A, A.w0 + b, C.goff + i);
    int32_t fs, bs;
    int64_t tot;
    const uint32_t code = eval_row_s<MODE>(r, F, h, R, sr, mt, ma, fs, bs, tot);
    if (PER && kept_q(A, A.w0 + b)) write_pair<true, true>(F, of, os, ot, C.N, i, code, fs, bs, tot, sr.raw);
    else write_pair<true>(F, of, os, ot, C.N, i, code, fs, bs, tot, sr.raw);
  }
}

template <int MODE, bool STAT, bool PER = false>
__device__ __forceinline__ void win_fixup(const DevCluster& C, const DevProfile& F, const WinArgs& A, WinLDS& L) {
  // (the thread index through an empty asm: every window recomputes the per-lane
  // LDS / record addresses derived from it instead of the compiler hoisting them
  // out of the persistent loop, where at the 128-VGPR cap they were spilled to
  // scratch and reloaded on the replay's critical path each window)
  int tid_ = (int)threadIdx.x;
#ifndef KSG_FIXUP_HOIST
  asm volatile("" : "+v"(tid_));
#endif
  const int tid = tid_, lane = tid & 63, wave = tid >> 6;
  const int nb = (int)A.nw;
  const uint32_t R = C.R < 4 ? C.R : 4;
#define STAMP(k)                                        \
  if (A.stamps && tid == 0) {                           \
    __builtin_amdgcn_sched_barrier(0);                  \
    A.stamps[k] = __builtin_amdgcn_s_memtime();         \
    __builtin_amdgcn_sched_barrier(0);                  \
  }
  STAMP(0);
  if (A.stamps && tid == 0) A.stamps[11] = __builtin_amdgcn_s_memrealtime();
  const int np = ldv<PER>(A.pprev_n);
  // (P_{W-1}'s nodes for wave 0's index, requested with the count, not after it)
  const int32_t pn_all = wave == 0 && lane < KSG_BATCH ? ldv<PER>(&A.pprev[lane].node) : -1;
  // ---- stage.  The small inputs (P_{W-1}, pods, counts) are loaded first and
  // stored at once; the candidate keys and rows stay in flight in registers
  // across the prior-node evaluations (vmcnt is in order) and land after them.
  constexpr int kRowW = (int)(sizeof(RowV) / 8), kPendW = (int)(sizeof(Pend) / 8);
  const uint64_t* keys = rec_keys(A.wrec);
  const uint64_t* rows = reinterpret_cast<const uint64_t*>(rec_rows(A.wrec));
  const int nk = nb * KSG_CAND, nr = A.defer ? 0 : nb * KSG_STAGE * kRowW;
  uint64_t kv[2], rv[6];
  // (persistent loop) the prior step the eval blocks did: thread = (pod, prior entry)
  const int ppb = tid >> 5, ppe = tid & 31;
  const PriorRec* PR = prior_rec(A.wrec);
  uint64_t pr_k = 0, pr_p0 = 0, pr_p1 = 0, pr_m = 0;
  int32_t pr_df = 0;
  const bool prior_rec_in = PER && !A.prior_fix;  // (else the prior step is evaluated below)
  const bool pr_late = prior_rec_in && A.evd_wait != nullptr;  // (split: after the keys and rows are requested)
  auto prior_loads = [&]() {
    if (ppb < nb) {
      pr_k = ldv<true>(&PR[ppb].pkey[ppe]);
      const uint64_t* pw = reinterpret_cast<const uint64_t*>(&PR[ppb].patch[ppe]);
      pr_p0 = ldv<true>(pw);
      pr_p1 = ldv<true>(pw + 1);
      pr_df = ldv<true>(&PR[ppb].pdf[ppe]);
      if (ppe == 0) pr_m = ldv<true>(&PR[ppb].pmask);
      if (ppe == 1) pr_m = ldv<true>(&PR[ppb].pbest);
      if (ppe == 2) pr_m = (uint64_t)(uint32_t)ldv<true>(&PR[ppb].pbest_e);
    }
  };
  if (prior_rec_in && !pr_late) prior_loads();
  {
    const uint64_t pv = tid < KSG_BATCH * kPendW ? ldv<PER>(reinterpret_cast<const uint64_t*>(A.pprev) + tid) : 0;
    constexpr int kPodW = (int)(sizeof(PodLite) / 8);
    const uint64_t qv = tid < nb * kPodW ? reinterpret_cast<const uint64_t*>(A.plite + A.w0)[tid] : 0;
    const int32_t fv = tid < nb && !A.defer ? ldv<PER>(reinterpret_cast<const int32_t*>(A.wrec) + tid) : 0;
    int32_t aT = 0, aA = 0;
    int64_t m0 = -1, m1 = -1;
    if (STAT && tid < nb) {
      if (!A.defer) {
        aT = ldv<PER>(reinterpret_cast<const int32_t*>(A.wrec) + KSG_BATCH + tid);
        aA = ldv<PER>(reinterpret_cast<const int32_t*>(A.wrec) + 2 * KSG_BATCH + tid);
      }
      m0 = ldv<PER>(A.mpred + 2 * (A.w0 - A.first + tid));
      m1 = ldv<PER>(A.mpred + 2 * (A.w0 - A.first + tid) + 1);
    }
    if (A.defer) {
      // merge pod b's T tile lists (wave w: pods w and w+16) and sum its tile counts;
      // the first 8 tiles' loads are issued together
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int b = wave + 16 * k;
        uint64_t v = 0;
        int32_t c[3] = {0, 0, 0};
        if (b < nb) {
          const uint64_t* tsrc = A.wtile_top + (size_t)b * A.T * KSG_TOPK;
          uint64_t tl[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) tl[t] = (uint32_t)t < A.T ? tsrc[(size_t)t * KSG_TOPK + lane] : 0;
          for (uint32_t t = lane; t < A.T; t += 64)
#pragma unroll
            for (int j = 0; j < 3; ++j) c[j] += A.wtile_feas[((size_t)b * A.T + t) * 3 + j];
          v = tl[0];
#pragma unroll
          for (int t = 1; t < 8; ++t)
            if ((uint32_t)t < A.T) v = wave_merge_top(v, wave_reverse(tl[t]));
#pragma unroll 1
          for (uint32_t t = 8; t < A.T; ++t) v = wave_merge_top(v, wave_reverse(tsrc[(size_t)t * KSG_TOPK + lane]));
#pragma unroll
          for (int j = 0; j < 3; ++j) c[j] = wave_sum(c[j]);
        }
        kv[k] = v;
        if (b < nb && lane == 0) {
          L.feas[b] = c[0];
          if (STAT) {
            L.achT[b] = c[1];
            L.achA[b] = c[2];
          }
        }
        if (b < nb && lane < KSG_STAGE && v) {  // candidate rows of the staged ranks (window-start rows)
          RowV rr;
          load_row(C, (uint32_t)(v & 0xFFFFFull) - C.goff, A.need_eph, rr);
          L.row[b][lane] = rr;
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        int i = tid + k * KSG_WIN_THREADS;
        kv[k] = i < nk ? ldv<PER>(keys + i) : 0;
      }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      int i = tid + k * KSG_WIN_THREADS;
      int row = i / kRowW, wd = i - row * kRowW;
      int p = row / KSG_STAGE, r = row - p * KSG_STAGE;
      if constexpr (PER) rv[k] = i < nr ? ldv<true>(reinterpret_cast<const uint64_t*>(&PR[p].row[r]) + wd) : 0;
      else rv[k] = i < nr ? rows[(size_t)(p * KSG_CAND + r) * kRowW + wd] : 0;
    }
    if (pr_late) {  // the keys and rows are in flight: wait for the window's prior steps, then their records
      if (tid == 0) {
        bool ok = false;
        for (uint32_t it = 0; it < A.spin; ++it) {
          if (ld_sc1(A.evd_wait) >= A.evd_need) { ok = true; break; }
          if ((it & 63u) == 63u && ld_sc1(A.abortw) != 0u) break;
          __builtin_amdgcn_s_sleep(1);
        }
        if (!ok) __hip_atomic_store(A.abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      lds_barrier();  // (no fence: the previous window's patch stores stay in flight)
      prior_loads();
    }
    if (tid < np * kPendW) reinterpret_cast<uint64_t*>(L.prior)[tid] = pv;
    if (tid < nb * kPodW) reinterpret_cast<uint64_t*>(L.pod)[tid] = qv;
    if (tid < nb && !A.defer) L.feas[tid] = fv;
    if (STAT && tid < nb) {
      if (!A.defer) {
        L.achT[tid] = aT;
        L.achA[tid] = aA;
      }
      L.mt[tid] = m0;
      L.ma[tid] = m1;
      L.fbf[tid] = 0;
    }
    if (tid < 3 * KSG_BATCH) {
      (&L.S[0][0])[tid] = -1;
      (&L.O[0][0])[tid] = -1;
    }
    if (tid < KSG_HSLOTS) {
#pragma unroll
      for (int t = 0; t < 3; ++t) pick_clear(L.pick[t], tid);
    }
    if (wave == 0) {  // index P_{W-1} (one wave: its LDS operations stay in order)
      const int32_t pnode = lane < np ? pn_all : -1;
      L.ptn[lane] = -1;
      L.ptn[lane + 64] = -1;
      if (lane < np) L.pte[tab_claim(L.ptn, pnode)] = lane;
    }
  }
  lds_barrier();
  STAMP(1);
  if (tid < np) {  // write P_{W-1} back (the eval blocks read those rows from the list)
    const Pend& pe = L.prior[tid];
    uint32_t nl = (uint32_t)pe.node - C.goff;
    if ((uint32_t)pe.node >= C.goff && nl < C.N) store_row_p<PER>(C, nl, pe.after);
    if (A.xrows) A.xrows[pe.node] = pe.after;  // every rank's replica, every node
  }
  if (prior_rec_in) {  // the eval blocks' prior step, staged
    if (ppb < nb) {
      L.pkey[ppb][ppe] = pr_k;
      reinterpret_cast<uint64_t*>(&L.patch[ppb][ppe])[0] = pr_p0;
      reinterpret_cast<uint64_t*>(&L.patch[ppb][ppe])[1] = pr_p1;
      L.pdf[ppb][ppe] = (int8_t)(pr_df & 0xFF);
      if (STAT) {
        L.pdfT[ppb][ppe] = (int8_t)((pr_df >> 8) & 0xFF);
        L.pdfA[ppb][ppe] = (int8_t)((pr_df >> 16) & 0xFF);
      }
      if (ppe == 0) L.pmask[ppb] = pr_m;
      if (ppe == 1) L.pbest[ppb] = pr_m;
      if (ppe == 2) L.pbest_e[ppb] = (int32_t)(uint32_t)pr_m;
    }
    STAMP(16);
  } else {  // pods on the P_{W-1} nodes as of the window start (independent of the picks)
    const int pb = 2 * wave + (lane >> 5), e = lane & 31;
    uint64_t k = 0;
    if (pb < nb && e < np) {
      const Pend& pe = L.prior[e];
      const PodLite* h = &L.pod[pb];
      int32_t fs, bs;
      int64_t tot;
      StaticRec sr{KSG_FILTER_PASS, 0};
      uint32_t code;
      if (STAT) {
        sr = srec_at<PER>(A, A.w0 + pb, (uint32_t)pe.node);
        code = eval_row_s<MODE>(pe.after, F, h, R, sr, L.mt[pb], L.ma[pb], fs, bs, tot);
      } else {
        code = eval_row<MODE>(pe.after, F, h, R, fs, bs, tot);
      }
      bool snap_ok = sr.code == KSG_FILTER_PASS && (F.pos_fit < 0 || fit_filter_row(pe.base, h, R) == 0);
      PatchV pt;
      pt.code = code;
      pt.fitba = fs | (bs << 16);
      pt.total = (int32_t)tot;
      pt.raw = sr.raw;
      L.patch[pb][e] = pt;
      k = code == KSG_FILTER_PASS ? pack_key(tot, F.seed, h->queue_idx, (uint32_t)pe.node) : 0;
      L.pkey[pb][e] = k;
      const int df = (code == KSG_FILTER_PASS ? 1 : 0) - (snap_ok ? 1 : 0);
      L.pdf[pb][e] = (int8_t)df;
      if (STAT) {
        const bool na_on = F.pos_na >= 0 && !(h->flags & KPF_SKIP_NA_SCORE);
        L.pdfT[pb][e] = (int8_t)(F.pos_taint >= 0 && (int64_t)(sr.raw >> 20) == L.mt[pb] ? df : 0);
        L.pdfA[pb][e] = (int8_t)(na_on && (int64_t)(sr.raw & KSG_RAW_NA_MASK) == L.ma[pb] ? df : 0);
      }
    }
    STAMP(16);
    // best prior node per pod: reduce within each half (DPP row ops stay inside 32 lanes
    // only up to 16; finish with one cross-half step)
    uint64_t k0 = wave_max(lane < 32 ? k : (uint64_t)0), k1 = wave_max(lane >= 32 ? k : (uint64_t)0);
    unsigned long long m0 = __ballot(k0 && lane < 32 && k == k0), m1 = __ballot(k1 && lane >= 32 && k == k1);
    if (lane == 0) {
      if (2 * wave < nb) {
        L.pbest[2 * wave] = k0;
        L.pbest_e[2 * wave] = m0 ? __ffsll((long long)m0) - 1 : -1;
      }
      if (2 * wave + 1 < nb) {
        L.pbest[2 * wave + 1] = k1;
        L.pbest_e[2 * wave + 1] = m1 ? __ffsll((long long)m1) - 1 - 32 : -1;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // kv[k] = key of pod wave + 16k, rank lane
    int i = tid + k * KSG_WIN_THREADS;
    if (i < nk) (&L.key[0][0])[i] = kv[k];
    const int b = wave + 16 * k;
    if (!prior_rec_in) {  // (PriorRec: the eval blocks' pmask)
      bool m = kv[k] != 0 && np > 0 && prior_of(L, (int32_t)(kv[k] & 0xFFFFFull)) >= 0;
      unsigned long long mask = __ballot(m);
      if (lane == 0 && b < nb) L.pmask[b] = mask;
    }
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    int i = tid + k * KSG_WIN_THREADS;
    if (i < nr) reinterpret_cast<uint64_t*>(&L.row[0][0])[i] = rv[k];
  }
  lds_barrier();
  STAMP(17);
  STAMP(2);
  if (wave == 0) {  // starting guess: serial dictatorship over (candidates, P_{W-1} nodes), parallel rounds
    const int b = lane;
    const bool valid = b < nb;
    const uint64_t pm = valid ? L.pmask[b] : 0;
    const uint64_t pbk = valid ? L.pbest[b] : 0;
    int r = 0;
    bool pok = pbk != 0;
    int32_t node = -1, org = -1;
#pragma unroll 1
    for (int round = 0; round < 64; ++round) {
      uint64_t ck = 0;
      if (valid) {  // next candidate that is not a P_{W-1} node
        uint64_t free_ = ~pm & (r < 64 ? (~0ull << r) : 0ull);
        r = free_ ? __ffsll((long long)free_) - 1 : KSG_CAND;
        ck = r < KSG_CAND ? L.key[b][r] : 0;
      }
      uint64_t pk = pok ? pbk : 0;
      uint64_t best = ck > pk ? ck : pk;
      bool from_c = best != 0 && best == ck;
      node = best ? (int32_t)(best & 0xFFFFFull) : -1;
      org = !best ? -1 : from_c ? 64 + b * 64 + r : L.pbest_e[b];
      // smallest proposer per node
      L.gtn[lane] = -1;
      L.gtn[lane + 64] = -1;
      uint32_t h = 0;
      if (node >= 0) {
        h = tab_claim(L.gtn, node);
        L.gtf[h] = KSG_BATCH;
      }
      if (node >= 0) atomicMin(&L.gtf[h], b);
      bool lose = node >= 0 && L.gtf[h] < b;
      if (__ballot(lose) == 0) break;
      if (lose) {
        if (from_c) ++r;
        else pok = false;
      }
    }
    if (valid) {
      L.S[0][b] = node;
      L.O[0][b] = org;
      if (node >= 0) pick_insert(L.pick[0], node, b);
    }
  }
  lds_barrier();
  STAMP(3);
  int cur = 0, stable = 0;
  uint32_t iters = 0;
#pragma unroll 1
  for (;;) {
    const int nxt = cur == 2 ? 0 : cur + 1;
    if (tid < KSG_HSLOTS) pick_clear(L.pick[nxt == 2 ? 0 : nxt + 1], tid);
    const PickTab& T = L.pick[cur];
    // phase A.  Waves 0..7 re-evaluate, for every pod b >= stable, the nodes the
    // pods a < b picked (pairs packed triangularly, p = b(b-1)/2 + a, so only
    // the live pairs occupy lanes); waves 8..15 mask each live pod's candidates
    // that an earlier pick touched.
    if (wave < 8) {
      const int p_hi = nb * (nb - 1) / 2;
#pragma unroll 1
      for (int base = stable * (stable - 1) / 2 + wave * 64; base < p_hi; base += 8 * 64) {
        const int p = base + lane;
        if (p < p_hi) {
          int b = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)p)) * 0.5f);
          b = b * (b - 1) / 2 > p ? b - 1 : ((b + 1) * b / 2 <= p ? b + 1 : b);
          const int a = p - b * (b - 1) / 2;
          const int32_t Sv = L.S[cur][a];
          uint64_t k = 0;
          int df = 0, dT = 0, dA = 0;
          PatchV pt;
          pt.code = KSG_NOT_PATCHED;
          pt.fitba = pt.total = 0;
          pt.raw = 0;
          if (Sv >= 0) {
            int nx = KSG_BATCH;
            Delta cum;
            delta_of(L.pod[a], cum);
            if (iters == 0) STAMP(24);
            if (T.cnt[tab_find(T.node, Sv)] > 1) pick_chain(L, L.S[cur], a, Sv, cum, nx);  // picked twice (rare)
            if (iters == 0) STAMP(25);
            if (nx >= b) {  // a is the last pick of the node before b
              RowV cur_r, snap;
              origin_rows<PER>(C, L, A, L.O[cur][a], cur_r, snap);
              apply_delta(cur_r, cum, R);
              const PodLite* h = &L.pod[b];
              int32_t fs, bs;
              int64_t tot;

              StaticRec sr{KSG_FILTER_PASS, 0};
              uint32_t code;
              if (STAT) {
                sr = srec_at<PER>(A, A.w0 + b, (uint32_t)Sv);
                code = eval_row_s<MODE>(cur_r, F, h, R, sr, L.mt[b], L.ma[b], fs, bs, tot);
              } else {
                code = eval_row<MODE>(cur_r, F, h, R, fs, bs, tot);
              }

              bool snap_ok = sr.code == KSG_FILTER_PASS && (F.pos_fit < 0 || fit_filter_row(snap, h, R) == 0);
              df = (code == KSG_FILTER_PASS ? 1 : 0) - (snap_ok ? 1 : 0);
              if (STAT) {
                const bool na_on = F.pos_na >= 0 && !(h->flags & KPF_SKIP_NA_SCORE);
                dT = F.pos_taint >= 0 && (int64_t)(sr.raw >> 20) == L.mt[b] ? df : 0;
                dA = na_on && (int64_t)(sr.raw & KSG_RAW_NA_MASK) == L.ma[b] ? df : 0;
              }
              if (code == KSG_FILTER_PASS) k = pack_key(tot, F.seed, h->queue_idx, (uint32_t)Sv);
              pt.code = code;
              pt.fitba = fs | (bs << 16);
              pt.total = (int32_t)tot;
              pt.raw = sr.raw;
            }
          }
          L.rk[b][a] = k;
          L.rdf[b][a] = (int8_t)df;
          if (STAT) {
            L.rdfT[b][a] = (int8_t)dT;
            L.rdfA[b][a] = (int8_t)dA;
          }
          L.patch[b][32 + a] = pt;
        }
      }
    } else {
      if (wave == 8 && lane < np) L.pf[lane] = first_pick(T, L.prior[lane].node);
#pragma unroll 1
      for (int b = stable + (wave - 8); b < nb; b += 8) {
        const uint64_t ck = L.key[b][lane];
        const bool mod = ((L.pmask[b] >> lane) & 1) || (ck != 0 && first_pick(T, (int32_t)(ck & 0xFFFFFull)) < b);
        L.kc[b][lane] = mod ? 0 : ck;
      }
    }
    if (iters == 0) STAMP(21);
    lds_barrier();
    if (iters == 0) STAMP(22);
    // phase B: per pod, the best of (untouched candidates, P_{W-1} nodes no
    // earlier pick touched, re-evaluated picks); waves own pods 2w and 2w+1.
#pragma unroll 1
    for (int hh = 0; hh < 2; ++hh) {
      const int b = 2 * wave + hh;
      if (b >= nb) break;
      if (b < stable) {
        if (lane == 0) {
          int32_t s = L.S[cur][b];
          L.S[nxt][b] = s;
          L.O[nxt][b] = L.O[cur][b];
          if (s >= 0) pick_insert(L.pick[nxt], s, b);
        }
        continue;
      }
      const bool pact = lane < np && L.pf[lane & 31] >= b;
      const uint64_t kc = L.kc[b][lane];
      const uint64_t kp = pact ? L.pkey[b][lane & 31] : 0;
      const uint64_t kr = lane < b ? L.rk[b][lane & 31] : 0;
      const int df = (pact ? (int)L.pdf[b][lane & 31] : 0) + (lane < b ? (int)L.rdf[b][lane & 31] : 0);
      const uint64_t best = wave_max(max3u(kc, kp, kr));
      int feasible;
      bool fb = false;
      if (STAT) {  // feasible and achiever counts in one reduction (per lane each change is in [-2, 2])
        const int dT = (pact ? (int)L.pdfT[b][lane & 31] : 0) + (lane < b ? (int)L.rdfT[b][lane & 31] : 0);
        const int dA = (pact ? (int)L.pdfA[b][lane & 31] : 0) + (lane < b ? (int)L.rdfA[b][lane & 31] : 0);
        const int sum = wave_sum((df + 2) | ((dT + 2) << 10) | ((dA + 2) << 20));
        feasible = L.feas[b] + (sum & 1023) - 128;
        const int achT = L.achT[b] + ((sum >> 10) & 1023) - 128, achA = L.achA[b] + ((sum >> 20) & 1023) - 128;
        const bool na_on = F.pos_na >= 0 && !(L.pod[b].flags & KPF_SKIP_NA_SCORE);
        fb = !(L.pod[b].flags & KPF_PREFILTER_ERROR) && !na_prescore_error(L.pod[b].flags, feasible) && feasible > 0 &&
             ((F.pos_taint >= 0 && achT <= 0) || (na_on && achA <= 0));
      } else {
        feasible = L.feas[b] + wave_sum(df);
      }
      const bool perr = (L.pod[b].flags & KPF_PREFILTER_ERROR) != 0 || na_prescore_error(L.pod[b].flags, feasible);
      const int32_t sel = (feasible > 0 && best && !perr) ? (int32_t)(best & 0xFFFFFull) : -1;
      const unsigned long long mc = __ballot(best && kc == best), mp = __ballot(best && kp == best),
                               mr = __ballot(best && kr == best);
      if (STAT && lane == 0) L.fbf[b] = fb ? 1 : 0;
      if (fb) continue;  // win_exact_select below
      if (lane == 0) {
        if (STAT) {
          L.xmt[b] = L.mt[b] < 0 ? 0 : L.mt[b];
          L.xma[b] = (F.pos_na < 0 || (L.pod[b].flags & KPF_SKIP_NA_SCORE) || L.ma[b] < 0) ? 0 : L.ma[b];
        }
        int32_t org = -1;
        if (mc) org = 64 + b * 64 + (__ffsll((long long)mc) - 1);
        else if (mp) org = __ffsll((long long)mp) - 1;
        else if (mr) org = L.O[cur][__ffsll((long long)mr) - 1];
        L.S[nxt][b] = sel;
        L.O[nxt][b] = sel >= 0 ? org : -1;
        if (sel >= 0) pick_insert(L.pick[nxt], sel, b);
        SumLite& sm = L.sum[b];
        sm.best_key = sel >= 0 ? (feasible == 1 ? (best & 0xFFFFFFFFFFull) : best) : 0;
        sm.selected = sel;
        sm.feasible = feasible;
        sm.status = perr ? 2 : (sel >= 0 ? 0 : 1);
      }
    }
    if (iters == 0) STAMP(23);
    lds_barrier();
    if (STAT) {  // pods with no feasible node left at the static max: exact re-evaluation
      unsigned long long fm = __ballot(lane < nb && lane >= stable && L.fbf[lane & 31] != 0);
      if (fm) {
        while (fm) {
          const int b = __ffsll((long long)fm) - 1;
          fm &= fm - 1;
          win_exact_select<MODE, PER>(C, F, A, L, b, cur, nxt, R);
        }
        lds_barrier();
      }
    }
    if (iters < 2) STAMP(19 + iters);
    ++iters;
    {  // every wave derives the same stable prefix
      const int32_t so = L.S[cur][lane & 31], sn = L.S[nxt][lane & 31];
      unsigned long long m = __ballot(lane < nb && lane >= stable && sn != so);
      stable = m ? min(__ffsll((long long)m), nb) : nb;
    }
    cur = nxt;
    if (stable >= nb) break;
  }
  STAMP(4);
  if (A.stamps && tid == 0) A.stamps[7] = iters;
  // (persistent loop) the two counters the flush and the next window wait on,
  // requested now: their round trips overlap the flush instead of following it
  uint32_t pre_fl = 0, pre_ev = 0;
  if (PER && tid == 0) {
    pre_fl = ld_sc1(A.flushed);
    pre_ev = A.nxt_evd ? ld_sc1(A.nxt_evd) : 0u;
  }
  // ---- flush: P_W first (the persistent loop publishes it at once: the eval
  // blocks of window W+2 wait for it), then summaries and per-pair patches
  const PickTab& T = L.pick[cur];
  if (wave == 0) {  // P_W: each node picked in the window, by its last pick
    const int a = lane;
    const int32_t Sv = a < nb ? L.S[cur][a] : -1;
    int h = Sv >= 0 ? tab_find(T.node, Sv) : -1;
    const bool last = h >= 0 && T.last[h] == a;
    unsigned long long m = __ballot(last);
    if (last) {
      Delta cum;
      delta_of(L.pod[a], cum);
      int nx;
      if (T.cnt[h] > 1) pick_chain(L, L.S[cur], a, Sv, cum, nx);
      RowV st, snap;
      origin_rows<PER>(C, L, A, L.O[cur][a], st, snap);
      Pend p;
      p.node = Sv;
      p.pad = 0;
      p.base = st;
      apply_delta(st, cum, R);
      p.after = st;
      st_obj<PER>(A.pnext + __popcll(m & ((1ull << a) - 1)), p);
    }
    if (lane == 0) stv<PER>(A.pnext_n, (int32_t)__popcll(m));
  }
  STAMP(26);
  if constexpr (PER) {  // every wave's stores of rows (P_{W-1}, at the stage) and P_W performed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(27);
    __syncthreads();
    if (tid < 16) st_sc1(A.pub + tid * 32, A.pub_val);
  }
  STAMP(6);
  if (tid < nb) {
    ksg_pod_summary& d = A.sums[A.w0 + tid];
    d.best_key = L.sum[tid].best_key;
    d.selected = L.sum[tid].selected;
    d.feasible = L.sum[tid].feasible;
    d.status = L.sum[tid].status;
    if (STAT) {
      if (F.pos_taint >= 0) d.max_score[F.pos_taint] = L.xmt[tid];
      if (F.pos_na >= 0) d.max_score[F.pos_na] = L.xma[tid];
    }
  }
  if constexpr (PER) {  // the eval blocks' outputs of this window are written before the patches
    if (tid == 0) {
      L.nxt_ok = A.nxt_evd && pre_ev >= A.nxt_need ? 1u : 0u;  // (read after the block's next barrier)
      bool ok = pre_fl >= A.flush_need;
      for (uint32_t it = 0; !ok && it < A.spin; ++it) {
        if (ld_sc1(A.flushed) >= A.flush_need) { ok = true; break; }
        if ((it & 63u) == 63u && ld_sc1(A.abortw) != 0u) break;
        __builtin_amdgcn_s_sleep(2);
      }
      if (!ok) __hip_atomic_store(A.abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    lds_barrier();  // (thread 0 acquired the count; the summaries' stores need no ack here)
  }
  {
    const int32_t Sv = L.S[cur][lane & 31];
    const int32_t pn = lane < np ? L.prior[lane].node : -1;
    const int pf = lane < np ? first_pick(T, pn) : -1;
#pragma unroll 1
    for (int hh = 0; hh < 2; ++hh) {
      const int b = 2 * wave + hh;
      if (b >= nb) break;
      if (STAT && L.fbf[b]) continue;  // rewritten whole below
      const PatchV pt = L.patch[b][lane];
      const bool wr = lane < 32 ? (lane < np && pf >= b) : (lane - 32 < b && pt.code != KSG_NOT_PATCHED);
      const int32_t node = lane < 32 ? pn : Sv;
      const uint32_t nl = (uint32_t)node - C.goff;
      if (wr && node >= 0 && (uint32_t)node >= C.goff && nl < C.N) {
        uint32_t* of;
        int32_t *os, *ot;
        out_ptrs(A, A.w0 + b, C.N, of, os, ot);
        if (PER && kept_q(A, A.w0 + b))
          write_pair<STAT, true>(F, of, os, ot, C.N, nl, pt.code, pt.fitba & 0xFFFF, pt.fitba >> 16, pt.total, pt.raw);
        else
          write_pair<STAT, false>(F, of, os, ot, C.N, nl, pt.code, pt.fitba & 0xFFFF, pt.fitba >> 16, pt.total, pt.raw);
      }
    }
  }
  if (STAT) {
    unsigned long long fm = __ballot(lane < nb && L.fbf[lane & 31] != 0);
    while (fm) {
      const int b = __ffsll((long long)fm) - 1;
      fm &= fm - 1;
      win_exact_write<MODE, PER>(C, F, A, L, b, cur, R);
    }
  }
  STAMP(5);
  if (A.stamps && tid == 0) A.stamps[12] = __builtin_amdgcn_s_memrealtime();
#undef STAMP
}

template <int MODE, bool STAT>
__global__ __launch_bounds__(KSG_WIN_THREADS) void k_window(DevCluster C, DevProfile F, WinArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  uint32_t warm = 0;
  KWarm<0, (int)((sizeof(DevCluster) + sizeof(DevProfile) + sizeof(WinArgs)) / 64 * 64)>::run(
      (const void*)__builtin_amdgcn_kernarg_segment_ptr(), warm);
  warm_wait(warm);
  if (blockIdx.x == 0) {
    if (A.nw) win_fixup<MODE, STAT>(C, F, A, *reinterpret_cast<WinLDS*>(lds_raw));
    return;
  }
  win_eval<MODE, STAT>(C, F, A, blockIdx.x - 1, reinterpret_cast<uint64_t*>(lds_raw));
}

// After the last window: write its pending rows back.
__global__ void k_apply_pend(DevCluster C, const Pend* p, const int32_t* pn) {
  int e = threadIdx.x;
  if (e >= *pn) return;
  uint32_t nl = (uint32_t)p[e].node - C.goff;
  if ((uint32_t)p[e].node >= C.goff && nl < C.N) store_row(C, nl, p[e].after);
}

// Sharded windows: every rank's header and keys (feasible counts + its
// top-KSG_CAND candidates per pod, kXchgBytes) are all-gathered; one wave per
// pod merges the R sorted lists into the global top-KSG_CAND, sums the counts and
// takes each candidate's row from the replica.  Between launches the replica
// holds the rows as of the end of window E-2 (the replay of E-1 wrote P_{E-2}
// into it first thing), which is what the owner's eval blocks computed on.
// pl / pn: P_{E-2}, whose rows the replica may not hold yet (the replay of E-1,
// which writes them into it, can run concurrently on the replay stream).
__global__ __launch_bounds__(64) void k_window_gmerge(const uint8_t* recv, uint32_t ranks, const RowV* xrows,
                                                      const Pend* pl, const int32_t* pn, uint8_t* out) {
  __shared__ uint64_t keys[8 * KSG_CAND];
  const uint32_t b = blockIdx.x;
  const int lane = threadIdx.x;
  for (uint32_t r = 0; r < ranks; ++r) keys[r * KSG_CAND + lane] = rec_keys(recv + r * kXchgBytes)[(size_t)b * KSG_CAND + lane];
  __syncthreads();
  uint64_t v = keys[lane];
  for (uint32_t r = 1; r < ranks; ++r) v = wave_merge_top(v, keys[r * KSG_CAND + 63 - lane]);
  int32_t f[3] = {0, 0, 0};
  for (uint32_t r = 0; r < ranks; ++r)
    for (int k = 0; k < 3; ++k) f[k] += reinterpret_cast<const int32_t*>(recv + r * kXchgBytes)[k * KSG_BATCH + b];
  RowV c;
  memset(&c, 0, sizeof(c));
  if (v) {
    const int32_t gid = (int32_t)(v & 0xFFFFFull);
    const int np = *pn;
    int hit = -1;
    for (int e = 0; e < np; ++e) hit = pl[e].node == gid ? e : hit;
    c = hit >= 0 ? pl[hit].after : xrows[gid];
  }
  rec_keys(out)[(size_t)b * KSG_CAND + lane] = v;
  rec_rows(out)[(size_t)b * KSG_CAND + lane] = c;
  if (lane < 3) reinterpret_cast<int32_t*>(out)[lane * KSG_BATCH + b] = f[lane];
}
// Replica set-up at the start of a sharded run: local rows packed (load_row:
// what the eval blocks read), all-gathered at a stride of the largest shard,
// unpacked by global index (shard r holds nodes [G*r/ranks, G*(r+1)/ranks)).
__global__ void k_rows_pack(DevCluster C, uint32_t need_eph, RowV* out) {
  const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n < C.N) load_row(C, n, need_eph, out[n]);
}
__global__ void k_rows_unpack(const RowV* recv, uint32_t ranks, uint32_t G, uint32_t stride, RowV* xrows) {
  const uint32_t r = blockIdx.y;
  const uint32_t lo = (uint32_t)((uint64_t)G * r / ranks), hi = (uint32_t)((uint64_t)G * (r + 1) / ranks);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; lo + i < hi; i += gridDim.x * blockDim.x)
    xrows[lo + i] = recv[(size_t)r * stride + i];
}

// ----------------------------------------------------------------- host side
#include "table_chain.hip"

// ---- The persistent window loop: every window of a run in ONE launch (Fit /
// BalancedAllocation profiles, one shard).  Block 0 replays windows 0, 1, ...;
// block 1 + b*T + t evaluates tile t of pod b of windows 0, 1, ....  The launch
// boundaries of k_window become hand-offs (agent-scope counters, sc1 data):
//   eval(E)   starts once replay(E-2) is published (Z.replayed >= E-1): the rows as of
//             the end of window E-2 (P_{E-2} from its list) — as k_window's eval part;
//   replay(W) starts once every pod of window W has its candidate record (Z.evd),
//             and writes its output patches once every eval block of W wrote its
//             outputs (Z.flushed);
// and the buffers of window parity p (tile lists, records, arrivals, P lists,
// output ring) are reused two windows later, after those waits.  A launch whose
// blocks are not all resident leaves at the handshake (run_handshake) and the
// host runs the launch-per-window loop instead.
struct WinSync {
  uint32_t replayed[16][32];  // windows replayed and published (block 0), one replica per 128-B line:
                              // each eval block polls its own (blk % 16), not all one line
  uint32_t evd[2];        // per window parity: pods whose record is out (cumulative over the launch)
  uint32_t pad1[30];
  uint32_t flushed[2];    // per window parity: eval blocks whose outputs are written (cumulative)
  uint32_t pad2[30];
  uint32_t evk[2];        // per window parity: pods whose keys and shallow rows are out (split hand-over)
  uint32_t pad3[30];
};
struct WinRunArgs {
  uint32_t nwin, first, count, T;
  uint32_t tt_sz, tf_sz;   // tile-list / tile-count slot sizes (elements)
  uint64_t* tile_top;
  int32_t* tfeas;
  uint8_t* wrec;           // 2 x kRecBytes
  Pend* pend;              // [2][KSG_BATCH]
  int32_t* pend_n;         // [2]
  uint32_t* arrive;        // [2][KSG_BATCH] counters, one 128-B line each
  uint64_t* stamps;        // diagnostic: 32 slots per window, or null
  const uint32_t* sready;  // STAT beside k_static_dec: per group of KSG_SD_PODS pods, its finished node tiles (null: before)
  uint32_t sready_need;    // ... the node tiles of k_static_dec's grid
};
// The eval blocks' gate on the static records of window pods [r0, r0 + n) (run
// offsets) when k_static_dec runs beside the loop: thread 0 polls the groups'
// counters (sc1), the block waits at a barrier.  Every other reader of a window's
// records (merges, the replay) reads them after this window's evaluation.
__device__ bool win_stat_gate(const WinRunArgs& R, uint32_t r0, uint32_t n, uint32_t* abortw, uint32_t spin,
                              uint32_t* go) {
  if (threadIdx.x == 0) {
    const uint32_t g0 = r0 / KSG_SD_PODS, g1 = (r0 + n - 1) / KSG_SD_PODS;
    bool ok = false;
    for (uint32_t it = 0; it < spin; ++it) {
      bool all = true;
      for (uint32_t g = g0; g <= g1; ++g) all &= ld_sc1(R.sready + g) >= R.sready_need;
      if (all) { ok = true; break; }
      if ((it & 63u) == 63u && ld_sc1(abortw) != 0u) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) __hip_atomic_store(abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *go = ok ? 1u : 0u;
  }
  __syncthreads();
  const bool ok = *go != 0u;
  __syncthreads();
  return ok;
}
// FENCE = false (the replay): a plain LDS barrier — __syncthreads' release fence
// would first wait for every store of the block still in flight (the previous
// window's output patches), about 2.5 us per window (round 6)
template <bool FENCE = true>
__device__ bool win_wait_ge(const uint32_t* w, uint32_t want, uint32_t* abortw, uint32_t spin, uint32_t* go) {
  if (threadIdx.x == 0) {
    bool ok = false;
    for (uint32_t it = 0; it < spin; ++it) {
      if (ld_sc1(w) >= want) { ok = true; break; }
      if ((it & 63u) == 63u && ld_sc1(abortw) != 0u) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) __hip_atomic_store(abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *go = ok ? 1u : 0u;
  }
  if constexpr (FENCE) __syncthreads(); else lds_barrier();
  const bool ok = *go != 0u;
  if constexpr (FENCE) __syncthreads(); else lds_barrier();
  return ok;
}
// STAT: Taint / NodeAffinity profiles, on static records computed for the whole
// run before the launch (round 5; the launch-per-window loop rolls a ring of chunks)
template <int MODE, bool STAT = false>
__global__ __launch_bounds__(KSG_WIN_THREADS) void k_window_run(DevCluster C, DevProfile F, WinArgs A0, WinRunArgs R,
                                                                RunSync* Y, WinSync* Z, RunCtl RC) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  __shared__ uint32_t go;
  uint32_t warm = 0;
  KWarm<0, (int)((sizeof(DevCluster) + sizeof(DevProfile) + sizeof(WinArgs)) / 64 * 64)>::run(
      (const void*)__builtin_amdgcn_kernarg_segment_ptr(), warm);
  warm_wait(warm);
  if (!run_handshake(Y, RC, &go)) return;
  uint32_t* const abortw = &Y->abort[0];
  WinArgs A = A0;
  A.abortw = abortw;
  A.spin = RC.spin;
  A.defer = 0;
  if (blockIdx.x == 0) {
    WinLDS& L = *reinterpret_cast<WinLDS*>(lds_raw);
    L.nxt_ok = 0;
    __syncthreads();
    for (uint32_t W = 0; W < R.nwin; ++W) {
      const bool ready = L.nxt_ok != 0;  // (the previous replay saw this window's records complete)
      A.ne = 0;
      A.w0 = R.first + W * KSG_BATCH;
      A.nw = min((uint32_t)KSG_BATCH, R.first + R.count - A.w0);
      A.wrec = R.wrec + (size_t)(W & 1) * kRecBytes;
      A.pnext = R.pend + (size_t)(W & 1) * KSG_BATCH;
      A.pnext_n = R.pend_n + (W & 1);
      A.pprev = R.pend + (size_t)((W + 1) & 1) * KSG_BATCH;  // P_{W-1}
      A.pprev_n = R.pend_n + ((W + 1) & 1);
      A.stamps = R.stamps ? R.stamps + (size_t)W * 32 : nullptr;
      // (the counters of a window parity only grow: every earlier window of that
      // parity is whole, KSG_BATCH pods)
      A.flushed = &Z->flushed[W & 1];
      A.flush_need = ((W >> 1) * KSG_BATCH + A.nw) * R.T;
      // (split: the keys counter gates the stage, the records counter the PriorRec reads;
      // `ready` then refers to the keys counter)
      const uint32_t need = (W >> 1) * KSG_BATCH + A.nw;
      const bool split = A0.split && !A0.prior_fix;
      // (diagnostic stamps past the windows' slots: loop top, ready, after the wait)
      uint64_t* const lt = R.stamps ? R.stamps + (size_t)R.nwin * 32 + (size_t)W * 4 : nullptr;
      if (lt && threadIdx.x == 0) {
        lt[0] = __builtin_amdgcn_s_memrealtime();
        lt[1] = ready ? 1u : 0u;
      }
      if (!ready && !win_wait_ge<false>(split ? &Z->evk[W & 1] : &Z->evd[W & 1], need, abortw, RC.spin, &go)) return;
      if (lt && threadIdx.x == 0) lt[2] = __builtin_amdgcn_s_memrealtime();
      A.evd_wait = split ? &Z->evd[W & 1] : nullptr;
      A.evd_need = need;
      A.pub = &Z->replayed[0][0];
      A.pub_val = W + 1;
      if (W + 1 < R.nwin) {
        const uint32_t w1 = W + 1, nw1 = min((uint32_t)KSG_BATCH, R.first + R.count - (R.first + w1 * KSG_BATCH));
        A.nxt_evd = split ? &Z->evk[w1 & 1] : &Z->evd[w1 & 1];
        A.nxt_need = (w1 >> 1) * KSG_BATCH + nw1;
      } else {
        A.nxt_evd = nullptr;
      }
      win_fixup<MODE, STAT, true>(C, F, A, L);  // (publishes P_W before its output patches)
      lds_barrier();  // (LDS reused by the next window; no fence: the patches need no ack before it)
    }
    return;
  }
  uint64_t* const L = reinterpret_cast<uint64_t*>(lds_raw);
  if (A0.mblocks && blockIdx.x >= 1 + KSG_BATCH * R.T) {  // the merge block of pod b
    const uint32_t b = blockIdx.x - 1 - KSG_BATCH * R.T;
    for (uint32_t E = 0; E < R.nwin; ++E) {
      A.nw = 0;
      A.e0 = R.first + E * KSG_BATCH;
      A.ne = min((uint32_t)KSG_BATCH, R.first + R.count - A.e0);
      if (b >= A.ne) break;
      A.tile_top = R.tile_top + (size_t)(E & 1) * R.tt_sz;
      A.tile_feas = R.tfeas + (size_t)(E & 1) * R.tf_sz;
      A.erec = R.wrec + (size_t)(E & 1) * kRecBytes;
      A.pprev = R.pend + (size_t)(E & 1) * KSG_BATCH;  // P_{E-2}
      A.pprev_n = R.pend_n + (E & 1);
      A.arrive = R.arrive + (size_t)(E & 1) * KSG_BATCH * 32;
      A.estamps = R.stamps ? R.stamps + (size_t)E * 32 : nullptr;
      A.evd = &Z->evd[E & 1];
      A.evk = A0.split && !A0.prior_fix ? &Z->evk[E & 1] : nullptr;
      A.pcur = R.pend + (size_t)((E + 1) & 1) * KSG_BATCH;  // P_{E-1}
      A.pcur_n = R.pend_n + ((E + 1) & 1);
      A.pubw = E >= 1 ? &Z->replayed[b & 15][0] : nullptr;
      A.pub_need = E;
      if (!win_merge_block<MODE, STAT>(C, F, A, b, L)) return;
      __syncthreads();  // (LDS reused by the next window)
    }
    return;
  }
  const uint32_t blk = blockIdx.x - 1, b = blk / R.T;
  for (uint32_t E = 0; E < R.nwin; ++E) {
    A.nw = 0;
    A.e0 = R.first + E * KSG_BATCH;
    A.ne = min((uint32_t)KSG_BATCH, R.first + R.count - A.e0);
    if (b >= A.ne) break;  // (only the last window is short)
    if (E >= 2 && !win_wait_ge(&Z->replayed[blk & 15][0], E - 1, abortw, RC.spin, &go)) return;
    A.tile_top = R.tile_top + (size_t)(E & 1) * R.tt_sz;
    A.tile_feas = R.tfeas + (size_t)(E & 1) * R.tf_sz;
    A.erec = R.wrec + (size_t)(E & 1) * kRecBytes;
    A.pprev = R.pend + (size_t)(E & 1) * KSG_BATCH;  // P_{E-2}
    A.pprev_n = R.pend_n + (E & 1);
    A.arrive = R.arrive + (size_t)(E & 1) * KSG_BATCH * 32;
    A.estamps = R.stamps ? R.stamps + (size_t)E * 32 : nullptr;
    A.evd = &Z->evd[E & 1];
    A.evk = A0.split && !A0.prior_fix ? &Z->evk[E & 1] : nullptr;
    A.flushed = &Z->flushed[E & 1];
    A.pcur = R.pend + (size_t)((E + 1) & 1) * KSG_BATCH;  // P_{E-1}
    A.pcur_n = R.pend_n + ((E + 1) & 1);
    A.pubw = E >= 1 ? &Z->replayed[blk & 15][0] : nullptr;  // (E = 0: P_{-1} is empty)
    A.pub_need = E;
    if (STAT && R.sready && !win_stat_gate(R, A.e0 - R.first, A.ne, abortw, RC.spin, &go)) return;
    win_eval<MODE, STAT, true>(C, F, A, blk, L);
    __syncthreads();  // (LDS reused by the next window)
  }
}


template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  bool alloc(size_t count, std::string& err) {
    if (count <= n && p) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
    hipError_t e = hipMalloc((void**)&p, bytes);
    if (e != hipSuccess) {
      err = std::string("hipMalloc: ") + hipGetErrorString(e);
      return false;
    }
    n = std::max<size_t>(count, 1);
    return true;
  }
  // capacity >= count, keeping the first `used` elements (doubling growth)
  bool grow(size_t count, size_t used, hipStream_t s, std::string& err) {
    if (count <= n && p) return true;
    size_t cap = std::max<size_t>(std::max<size_t>(count, 2 * n), 1);
    T* q = nullptr;
    hipError_t e = hipMalloc((void**)&q, cap * sizeof(T));
    if (e != hipSuccess) {
      err = std::string("hipMalloc: ") + hipGetErrorString(e);
      return false;
    }
    if (p && used) e = hipMemcpyAsync(q, p, std::min(used, n) * sizeof(T), hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      err = hipGetErrorString(e);
      (void)hipFree(q);
      return false;
    }
    if (p) (void)hipFree(p);
    p = q;
    n = cap;
    return true;
  }
  bool upload(const std::vector<T>& v, hipStream_t s, std::string& err) {
    if (!alloc(v.size(), err)) return false;
    if (!v.empty()) {
      hipError_t e = hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
      if (e != hipSuccess) { err = hipGetErrorString(e); return false; }
    }
    return true;
  }
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
};

struct Engine::Impl {
  EngineConfig cfg;
  // node-shard exchange (sharded batch path)
  int xmode = 0;  // 0 none, 1 RCCL all-gather on the engine stream, 2 host callback
  uint32_t xrank = 0, xranks = 1;
  ncclComm_t comm = nullptr;
  Engine::ExchangeFn xfn = nullptr;
  void* xuser = nullptr;
  DBuf<uint8_t> xsend, xrecv;
  DBuf<RowV> xrows;  // sharded windows: every node's row (run_batches)
  uint32_t G = 0;    // nodes of the whole cluster
  // host exchange (mode 2): pinned staging buffers; the callback runs as a
  // stream host function, so the exchange stays asynchronous like RCCL's
  uint8_t *hps = nullptr, *hpr = nullptr;
  size_t hps_n = 0, hpr_n = 0;
  struct HostCall {
    Impl* I;
    size_t bytes;
  };
  std::deque<HostCall> hcalls;
  std::atomic<int> xfail{0};
  DevProfile F{};
  hipStream_t stream = nullptr;
  bool own_stream = false;
  uint32_t N = 0, R = 3, K = 0, goff = 0;
  // nodes
  DBuf<int64_t> alloc, req, nzc, nzm, vnum;
  DBuf<int32_t> allowed, podcnt, label, tid;
  DBuf<uint32_t> toff, kvo;
  DBuf<uint8_t> haslab, vok, nflags;
  DBuf<uint32_t> img;
  DBuf<int32_t> ports, ports0;
  DBuf<int32_t> pvcuse, pvcuse0;  // PVC use counts (VolumeRestrictions ReadWriteOncePod)
  uint32_t n_pvc = 0;
  DBuf<int32_t> vlim, vatt, vatt0, vnode, vnode0, vref, vref0;  // NodeVolumeLimits (CSI)
  uint32_t n_vatt = 0, n_vnode = 0;
  uint32_t img_words = 0, n_ports = 0;
  NodeSoA topo;  // topology tables (host copy)
  DBuf<int32_t> topo_key_d;
  DBuf<uint32_t> topo_base_d, topo_count_d;
  // pod table
  DBuf<int32_t> ptnode, ptns, ptlab, tpod, tval;
  DBuf<uint32_t> ptflags, tcounts;
  DBuf<ksg_exist_term> terms;
  DBuf<ksg_req> treq;
  uint32_t pcap = 0, pkeys = 0, tcap = 0, rcap = 0, vcap = 0;
  DBuf<uint8_t> evprog;  // cluster events applied in place: the bound pod's program
  DBuf<int32_t> evrow;   // its existing-pod table row
  uint8_t* apstage = nullptr;  // append_program: pinned staging block (apstage_ev: its last copy)
  uint8_t* vstage = nullptr;   // victim_store: pinned staging of the store (synchronous use)
  size_t vstage_cap = 0;
  size_t apstage_cap = 0;
  hipEvent_t apstage_ev = nullptr;
  DBuf<uint8_t> apdev;
  // toggle_stage / toggle_staged: the staged candidate victims (tg_addr: each
  // entry's program, a device address in tgprog, the victim store or the queue's
  // program buffer)
  DBuf<uint8_t> tgprog;
  DBuf<uint64_t> tgaddr;
  DBuf<int32_t> tgnode, tgrow;
  DBuf<uint32_t> tgidx;
  std::vector<int32_t> tg_gnode;  // host copies: grouping, CSI entries
  std::vector<char> tg_csi;
  std::vector<uint64_t> tg_addr;
  uint32_t tg_n = 0;
  DBuf<uint8_t> vstore;  // victim_store: bound pods' programs (entry b at vstore_off[b])
  std::vector<uint64_t> vstore_off;
  std::vector<char> vstore_csi;
  DBuf<ksg_pod_summary> drysum;  // DefaultPreemption dry run: the preemptor's summary, restored after each probe
  // scratch
  DBuf<int32_t> cnt, hist_f, hist_s, ipa_aff, ipa_anti, ipa_exist, pts_min, pts_dom;
  DBuf<uint8_t> present_f, reg;
  DBuf<int64_t> ipa_score;
  DBuf<uint32_t> exist_any;
  // outputs
  DBuf<uint32_t> filter;
  DBuf<int32_t> score, total;
  DBuf<ksg_pod_summary> sums;
  DBuf<int32_t> prow;     // existing-pod table row of each assumed queue pod (-1 none)
  DBuf<uint32_t> arrive1; // block arrivals of the per-pod chain's last kernel
  bool static_ok = false; // per-pod cycles of Fit/BA/Taint/NA profiles: k_static + k_fs_static
  DBuf<uint64_t> wrec_pairs;  // what-if: pass 1's per-pair records (run_whatif)
  DBuf<uint64_t> wc_pods;     // what-if class path: the chunk's decoded pods (WcPod)
  DBuf<uint64_t> sd_pods;     // static records: the chunk's decoded pods (WcPod, k_static_dec)
  int static_dec = 1;         // k_static_dec where the chunk's pods decode (KSG_STATIC_DEC=0: k_static)
  uint32_t static_run_mb = 4096;   // static records of a whole run in the persistent window loop (KSG_STATIC_RUN_MB; 0: off;
                                   // also at most half the device's free memory, else the ring of chunks)
  uint64_t static_dec_chunks = 0;  // diagnostic: static chunks computed from decoded pods
  int static_overlap = 1;          // KSG_STATIC_OVERLAP=0: a persistent run's records all before its launch
  int static_beside_test = 0;      // tests (KSG_STATIC_BESIDE_TEST): 1 = the side kernel launched after the loop,
                                   // 2 = only after the loop's verdict (never resident beside it: the fallback)
  uint64_t static_overlaps = 0;    // diagnostic: persistent runs whose records were computed beside the loop
  DBuf<uint32_t> sready;           // ... per group of KSG_SD_PODS pods, the node tiles done
  uint32_t wi_chunk = 0;      // ... pods per chunk of the last step, and whether records were used
  bool wi_rec = false;
  bool wi_cls = false;        // ... or the class path
  uint32_t max_taints = 0;  // most taints on one node (what-if record width)
  int32_t max_tid = -1;     // largest taint id on a node (what-if class path: < 64)
  bool taint_dup = false;   // some node lists a taint twice
  bool cols_small = false;  // cpu / memory columns of every node (alloc, requested, non-zero) in (-2^45, 2^45)
  int wc_npt = KSG_WC_NPT;  // what-if class path: nodes per thread (KSG_WC_NPT)
  int64_t max_na_sum = 0;   // largest preferred NodeAffinity weight sum of a program
  bool static_fits = true; // raw scores fit the record (taints per node < 4096, NodeAffinity weights < 2^20)
  DBuf<StaticRec> stat;   // static records of a chunk of pods [chunk][N]
  DBuf<int64_t> mpred;    // [chunk][2] static max of the Taint / NodeAffinity raw scores
  DBuf<int32_t> saux;     // k_fs_static counters
  // sharded per-pod chain: pairs of topology slots whose domains span nodes, slot mask of one-node domains
  DBuf<uint32_t> spair;
  uint32_t nsp = 0, uniq = 0;
  DBuf<int64_t> xregcnt;  // merged registered-domain counts per score constraint
  // class tables (ksg_types.h "class tables")
  bool tables_on = false;   // profile with PodTopologySpread / InterPodAffinity
  DBuf<int32_t> pc_cnt, pc_dom, pc_tot, tc_val, tc_tot, tc_slot_d, slot_dom_d, cval_d;
  DBuf<uint32_t> tc_off_d, nu_base_d;
  DBuf<uint8_t> pair_node_d;
  DBuf<ksg_pclass> pcls_d;
  DBuf<ksg_cterm> cterm_d;
  DBuf<ksg_req> creq_d;
  uint32_t npc = 0, ntc = 0, NU = 0, nct = 0, ncreq = 0, ncval = 0, tc_used = 0;
  std::vector<uint32_t> tc_off_h;
  // node sharding of the class tables: ranks, every node's topology values, and
  // the classes built from this rank's existing pods alone since the last
  // cross-rank sum of their pair-level entries (UINT32_MAX: none pending)
  uint32_t shards = 1;
  DBuf<int32_t> gtopo_d;
  DBuf<int32_t> glabel, gtid;  // node-sharded static records: every node's labels [K][G] and taints (CSR)
  DBuf<uint32_t> gtoff;
  bool gstat = false;
  uint32_t red_pc0 = UINT32_MAX, red_tc0 = UINT32_MAX;
  std::vector<int32_t> tc_slot_h;
  DBuf<TabSeg> segs_d;
  // table chain (k_eval / k_ptsraw / k_final / k_select)
  DBuf<uint32_t> carrive;  // table chain: block arrivals of the cycle's last kernel
  DBuf<int2> alog;        // assumes whose existing-pod table rows k_flush_appends writes
  DBuf<int32_t> cpi, cpst;
  DBuf<int64_t> cpm, cpm2;
  DBuf<EvalTotals> cetot;
  DBuf<SoloCand> ccand;   // k_eval_solo: classes per block [cnblk][kChain]
  int solo = 0;           // one-launch cycles (k_eval_solo): 0 off, 1 on (KSG_SOLO)
  int run_on = 1;         // persistent segments (k_chain_run): KSG_RUN=0 turns them off
  int run_bt = 256;       // k_chain_run threads per block (KSG_RUN_BT=256|512)
  uint32_t run_cap512 = 0;
  uint32_t run_cap = 0;   // blocks every one of which is resident at once (k_chain_run), 0: not queried yet
  uint32_t run_min = 2;   // shortest segment launched persistently (KSG_RUN_MIN)
  DBuf<RunSync> rsync;    // k_chain_run's flag / handshake (zeroed per launch) and sticky abort word
  DBuf<uint64_t> rgran;   // k_chain_run's tagged granules: partial records [2 parities], then keys [2] (zeroed per launch)
  bool run_used = false;  // a persistent segment ran since the last sync (its abort word is checked)
  uint32_t* hverdict = nullptr;  // pinned, coherent: the handshake verdict of the last segment (the host polls it)
  uint32_t run_lag = 0;          // diagnostic (KSG_RUN_LAG): committer delay per pod, s_sleep(127) rounds
  uint32_t run_need_extra = 0;   // diagnostic (KSG_RUN_NORES=1): a grid that can never be all resident
  uint32_t run_wait_us = 5000;   // handshake limit (KSG_RUN_WAIT_US)
  uint32_t run_spin = kRunSpin;  // polls before a persistent block gives up (KSG_RUN_SPIN: tests force an abort)
  uint64_t run_fallbacks = 0;    // segments that ran on the two-launch chain (not co-resident)
  bool lost = false;             // an aborted persistent launch left the device state half-updated
  std::vector<std::shared_ptr<const void>> hold;  // host sources of queued uploads (add_classes), until the next sync
  bool unwaited = false;         // a state-changing launch was queued without a wait (Reserve's k_assume):
                                 // a failing synchronisation then leaves host mirror and device apart (lost)
  DBuf<WinSync> wsync;           // k_window_run's counters (zeroed per launch)
  int final_pm = 1;              // k_final specialised for the Fit/BA/PTS/IPA plugin set (KSG_FINAL_PM=0: generic)
  int view_slots_direct = 1;     // k_view: message slots into the host block as claimed (KSG_VIEW_SLOTS_DIRECT=0: last block copies)
  int view_narrow = 1;           // k_view: PTS / IPA raw rows by the summary's range (KSG_VIEW_NARROW=0: 4 bytes)
  int place_fused = 1;           // add_classes places the cycle's program in its upload (KSG_PLACE_FUSED=0: off)
  int pc_agg = 1;                // k_pc_build counts few-domain slots per block (KSG_PC_AGG=0: per row)
  int pc_prefetch = 1;           // k_pc_build reads the requirement keys' label columns up front (KSG_PC_PREFETCH=0: off)
  int win_run_on = 1;            // persistent window loop (k_window_run): KSG_WIN_RUN=0 turns it off
  int win_mblocks = 0;           // ... with dedicated merge blocks (KSG_WIN_MB=1; the last tile block merges: measured faster)
  int view_copy = 0;             // cycle view: 1 = the per-node arrays by a copy (KSG_VIEW_COPY), 0 = written by k_view
  int view_fuse = 1;             // fused views (Engine::view_arm; KSG_VIEW_FUSE=0: k_view always)
  bool vp_armed = false, vp_fused = false, vp_last_fused = false;  // the armed view and its launch parameters
  uint64_t views_fused = 0;      // diagnostic: views k_eval wrote (ksg_debug_views_fused)
  uint32_t vp_q = 0;
  size_t vp_k = 0;
  ViewDev vp_V{};
  uint8_t* vp_hout = nullptr;
  int run_overlap = 0;           // k_chain_run: pod k+1's class-table reads during pod k's hand-offs (KSG_RUN_OVERLAP=1; measured no faster)
  int run_defer = 1;             // k_chain_run: the owner's independent node-level assume deferred (KSG_RUN_DEFER=0: off)
  int win_split = 1;             // ... split hand-over: keys staged while the prior steps run (KSG_WIN_SPLIT=0: one counter)
  int win_pfix = 0;              // ... the replay evaluates the prior step itself (KSG_WIN_PFIX=1; measured slower)
  uint64_t win_runs = 0, win_fallbacks = 0;  // diagnostic: persistent window launches / not co-resident
  uint32_t fold_blocks = 256;  // table chain: k_fold above this many blocks (KSG_FOLD_BLOCKS; tests force it)
  uint32_t occ_blocks = 0;     // table chain: occupancy twins above this many blocks (0: 2 per CU; KSG_OCC_BLOCKS)
  bool occ_force = false;
  DBuf<uint64_t> cpr, cpk;
  uint32_t cnblk = 0;
  DBuf<int32_t> knorm;    // normalized scores of one kept pod
  DBuf<uint8_t> vblk;     // device cycle view block (Engine::view)
  DBuf<uint32_t> vdone;   // k_view's finished-block count (direct views)
  bool vblk_fresh = true;
  uint32_t vgen = 0;      // view generation (slot-table entries of older views count as empty)
  size_t prog_bytes = 0;  // used bytes of the program blob
  // kept per-pair outputs
  uint32_t keep_first = 0, keep_n = 0;
  DBuf<uint32_t> kfilter;
  DBuf<int32_t> kscore, ktotal;
  // programs
  DBuf<uint8_t> progs;
  DBuf<PodLite> plite;  // Fit/BA fields of the programs (window path)
  DBuf<uint64_t> prog_off_d;
  bool any_eph_req = false;
  // speculative batch path
  bool batch_ok = false;     // profile of Fit / BA (/ Taint / NodeAffinity) plugins only
  bool batch_static = false;
  uint32_t stat_chunk_cap = 0;
  uint32_t n_cus = 256;  // compute units of the device
  hipStream_t sstream = nullptr;  // low-priority side stream (static records of the window path)
  hipStream_t rstream = nullptr, xstream = nullptr;  // sharded windows: replay / exchange streams (run_batches_split)
  hipEvent_t xg[2] = {nullptr, nullptr}, xr[2] = {nullptr, nullptr}, xe[2] = {nullptr, nullptr}, xjoin = nullptr;
  bool static_side = false;  // KSG_STATIC_SIDE=1: measured no faster (the windows slow down beside it)
  hipEvent_t sev_ready[3] = {nullptr, nullptr, nullptr}, sev_free = nullptr;  // diagnostic: cap on the static chunk (pods, multiple of KSG_BATCH)  // ... with Taint / NodeAffinity: static records per pod (k_static)
  DBuf<uint64_t> tile_top;
  DBuf<int32_t> tfeas, pend_n;
  DBuf<uint32_t> arrive;
  DBuf<uint8_t> wrec;     // candidate records of two windows (kRecBytes each)
  DBuf<Pend> pend;        // pending rows P_j of two windows
  DBuf<uint32_t> bfilter;
  DBuf<int32_t> bscore, btotal;
  std::vector<size_t> prog_off;
  std::vector<uint32_t> prog_need;  // bit0 pts, bit1 ipa
  bool has_pts = false, has_ipa = false;
  bool force_per_pod = false;
  int eval_mode = 0;  // 1: default Fit/BA arguments (compiled specialisation)
  DBuf<int32_t> fit_res_d, ba_res_d;
  DBuf<int64_t> fit_w_d;
  bool stamps_on = false;  // diagnostic: s_memtime stamps in the fixup loop
  DBuf<uint64_t> stamps;
  bool cstamps_on = false;  // diagnostic: table chain stamps
  DBuf<uint64_t> cstamps;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float last_ms = 0;
  // pristine copies for reset()
  DBuf<int64_t> req0, nzc0, nzm0;
  DBuf<int32_t> podcnt0;
  uint32_t counts0[8] = {};
  // sampled kernel timing
  uint32_t sample_every = 0;
  std::vector<hipEvent_t> sev;
  uint32_t n_samples = 0;
  std::vector<hipEvent_t> sev_st;  // ... and around the static-record launches (k_static) of the same run
  uint32_t n_st = 0;
  uint64_t stat_pods_sampled = 0;
  uint64_t path_pods[6] = {0, 0, 0, 0, 0, 0};  // diagnostic: pods run by the table chain / the scanning chain / of the first, in one launch; what-if pod chunks on the class path; table-chain pods of persistent segments (k_chain_run) / those segments
  std::vector<Engine::KernelStat> stats;

  DevCluster cluster() const {
    DevCluster C{};
    C.N = N; C.R = R; C.K = K; C.goff = goff;
    C.alloc = alloc.p; C.req = req.p; C.nzc = nzc.p; C.nzm = nzm.p;
    C.allowed = allowed.p; C.podcnt = podcnt.p; C.label = label.p; C.toff = toff.p; C.tid = tid.p;
    C.haslab = haslab.p; C.kvo = kvo.p; C.vnum = vnum.p; C.vok = vok.p;
    C.nflags = nflags.p; C.img_words = img_words; C.img = img.p; C.n_ports = n_ports; C.ports = ports.p;
    C.pvcuse = pvcuse.p;
    C.vlim = vlim.p; C.vatt = vatt.p; C.vnode = vnode.p; C.vref = vref.p;
    C.n_topo = (uint32_t)topo.topo_key.size();
    C.pairs = topo.topo_pairs;
    C.tkey = topo_key_d.p;
    C.tbase = topo_base_d.p;
    C.tcount = topo_count_d.p;
    C.pcap = pcap; C.pkeys = pkeys; C.tcap = tcap; C.rcap = rcap; C.vcap = vcap;
    C.ptnode = ptnode.p; C.ptns = ptns.p; C.ptflags = ptflags.p; C.ptlab = ptlab.p;
    C.terms = terms.p; C.tpod = tpod.p; C.treq = treq.p; C.tval = tval.p; C.tcounts = tcounts.p;
    DevTables& T = C.T;
    T.on = tables_on ? 1 : 0;
    T.npc = npc; T.ntc = ntc; T.NU = NU; T.uniq = uniq;
    T.pc_cnt = pc_cnt.p; T.pc_dom = pc_dom.p; T.pc_tot = pc_tot.p;
    T.nu_base = nu_base_d.p; T.slot_dom = slot_dom_d.p; T.pair_node = pair_node_d.p;
    T.pcls = pcls_d.p; T.cterm = cterm_d.p; T.creq = creq_d.p; T.cval = cval_d.p;
    T.tc_val = tc_val.p; T.tc_off = tc_off_d.p; T.tc_slot = tc_slot_d.p; T.tc_tot = tc_tot.p;
    T.sharded = shards > 1 ? 1 : 0;
    T.G = G;
    T.gtv = gtopo_d.p;
    for (int s = 0; s < KSG_MAX_TOPO; ++s) {
      C.tkeyv[s] = (size_t)s < topo.topo_key.size() ? topo.topo_key[s] : -1;
      C.nubv[s] = ((size_t)s < topo.nu_base.size() && topo.nu_base[s] != 0xFFFFFFFFu) ? (int32_t)topo.nu_base[s] : -1;
    }
    return C;
  }
  // k_static over every node of a node-sharded cluster (the replicated static columns)
  DevCluster cluster_static() const {
    DevCluster C = cluster();
    if (gstat) {
      C.N = G;
      C.goff = 0;
      C.label = glabel.p;
      C.toff = gtoff.p;
      C.tid = gtid.p;
    }
    return C;
  }
  DevScratch scratch() const {
    DevScratch S{};
    S.cnt = cnt.p; S.hist_f = hist_f.p; S.present_f = present_f.p; S.hist_s = hist_s.p; S.reg = reg.p;
    S.ipa_aff = ipa_aff.p; S.ipa_anti = ipa_anti.p; S.ipa_exist = ipa_exist.p; S.ipa_score = ipa_score.p;
    S.pts_min = pts_min.p; S.pts_dom = pts_dom.p; S.exist_any = exist_any.p;
    return S;
  }
};
// Every synchronisation of the engine stream: a failure after a state-changing
// launch nobody waited for (ksg_reserve) means the host mirror counts a delta the
// device may not hold, so the context is marked lost (ksg.h: errors reported late).
static bool stream_sync(Engine::Impl& I, hipStream_t s, std::string& err) {
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    err = std::string("hipStreamSynchronize: ") + hipGetErrorString(e);
    if (I.unwaited) I.lost = true;
    return false;
  }
  if (s == I.stream) {
    I.unwaited = false;
    I.hold.clear();  // (every queued copy from them has completed)
  }
  return true;
}

Engine::Engine() : p_(new Impl()) {}
Engine::~Engine() {
  if (p_->comm) (void)ncclCommDestroy(p_->comm);
  if (p_->stream) (void)hipStreamSynchronize(p_->stream);  // (queued host exchanges use the buffers below)
  if (p_->hps) (void)hipHostFree(p_->hps);
  if (p_->hpr) (void)hipHostFree(p_->hpr);
  if (p_->hverdict) (void)hipHostFree(p_->hverdict);
  if (p_->apstage) (void)hipHostFree(p_->apstage);
  if (p_->vstage) (void)hipHostFree(p_->vstage);
  if (p_->apstage_ev) (void)hipEventDestroy(p_->apstage_ev);
  if (p_->ev0) (void)hipEventDestroy(p_->ev0);
  if (p_->ev1) (void)hipEventDestroy(p_->ev1);
  for (hipEvent_t e : {p_->sev_ready[0], p_->sev_ready[1], p_->sev_ready[2], p_->sev_free})
    if (e) (void)hipEventDestroy(e);
  if (p_->sstream) (void)hipStreamDestroy(p_->sstream);
  for (hipEvent_t e : {p_->xg[0], p_->xg[1], p_->xr[0], p_->xr[1], p_->xe[0], p_->xe[1], p_->xjoin})
    if (e) (void)hipEventDestroy(e);
  if (p_->rstream) (void)hipStreamDestroy(p_->rstream);
  if (p_->xstream) (void)hipStreamDestroy(p_->xstream);
  if (p_->own_stream && p_->stream) (void)hipStreamDestroy(p_->stream);
  delete p_;
}

bool Engine::init(const EngineConfig& cfg, std::string& err) {
  Impl& I = *p_;
  I.cfg = cfg;
  if (const char* e = std::getenv("KSG_FOLD_BLOCKS")) I.fold_blocks = (uint32_t)std::strtoul(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_SOLO")) I.solo = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_RUN")) I.run_on = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_RUN_BT")) I.run_bt = std::strtol(e, nullptr, 10) == 512 ? 512 : 256;
  if (const char* e = std::getenv("KSG_RUN_MIN")) I.run_min = std::max<uint32_t>(1, (uint32_t)std::strtoul(e, nullptr, 10));
  if (const char* e = std::getenv("KSG_RUN_LAG")) I.run_lag = std::min<uint32_t>(4096, (uint32_t)std::strtoul(e, nullptr, 10));
  if (const char* e = std::getenv("KSG_RUN_NORES")) I.run_need_extra = std::strtol(e, nullptr, 10) != 0 ? 1u : 0u;
  if (const char* e = std::getenv("KSG_WIN_RUN")) I.win_run_on = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_PC_PREFETCH")) I.pc_prefetch = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_PC_AGG")) I.pc_agg = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_PLACE_FUSED")) I.place_fused = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_VIEW_NARROW")) I.view_narrow = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_FINAL_PM")) I.final_pm = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_VIEW_SLOTS_DIRECT")) I.view_slots_direct = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_WIN_MB")) I.win_mblocks = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_WIN_PFIX")) I.win_pfix = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_WIN_SPLIT")) I.win_split = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_RUN_OVERLAP")) I.run_overlap = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_RUN_DEFER")) I.run_defer = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_VIEW_COPY")) I.view_copy = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_RUN_SPIN")) I.run_spin = std::max<uint32_t>(1, (uint32_t)std::strtoul(e, nullptr, 10));
  if (const char* e = std::getenv("KSG_RUN_WAIT_US"))
    I.run_wait_us = std::max<uint32_t>(10, std::min<uint32_t>(1000000, (uint32_t)std::strtoul(e, nullptr, 10)));
  if (const char* e = std::getenv("KSG_WC_NPT")) I.wc_npt = (int)std::strtol(e, nullptr, 10);
  if (const char* e = std::getenv("KSG_OCC_BLOCKS")) {
    I.occ_blocks = (uint32_t)std::strtoul(e, nullptr, 10);
    I.occ_force = I.occ_blocks == 0;
  }
  HIPCHK(hipSetDevice(cfg.device));
  if (cfg.stream) {
    I.stream = (hipStream_t)cfg.stream;
  } else {
    HIPCHK(hipStreamCreateWithFlags(&I.stream, hipStreamNonBlocking));
    I.own_stream = true;
  }
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg.device) == hipSuccess && cus > 0)
      I.n_cus = (uint32_t)cus;
  }
  {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = 0;
    HIPCHK(hipStreamCreateWithPriority(&I.sstream, hipStreamNonBlocking, least));
    if (const char* e = std::getenv("KSG_STATIC_SIDE")) I.static_side = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("KSG_STATIC_DEC")) I.static_dec = (int)std::strtol(e, nullptr, 10);
    if (const char* e = std::getenv("KSG_STATIC_RUN_MB")) I.static_run_mb = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = std::getenv("KSG_STATIC_OVERLAP")) I.static_overlap = (int)std::strtol(e, nullptr, 10);
    if (const char* e = std::getenv("KSG_STATIC_BESIDE_TEST")) I.static_beside_test = (int)std::strtol(e, nullptr, 10);
    if (const char* e = std::getenv("KSG_VIEW_FUSE")) I.view_fuse = (int)std::strtol(e, nullptr, 10);
  }
  HIPCHK(hipEventCreate(&I.ev0));
  HIPCHK(hipEventCreate(&I.ev1));
  if (!I.arrive1.alloc(1, err)) return false;
  HIPCHK(hipMemsetAsync(I.arrive1.p, 0, sizeof(uint32_t), I.stream));
  DevProfile& F = I.F;
  F.n = cfg.n_plugins;
  F.has_ext = 0;
  for (int i = 0; i < cfg.n_plugins; ++i) {
    F.plugins[i] = cfg.plugins[i];
    F.weight[i] = cfg.weight[i];
    int p = cfg.plugins[i];
    if (p == KP_TAINT || p == KP_NA || p == KP_PTS || p == KP_IPA) F.has_ext = 1;
    if (p == KP_PTS) I.has_pts = true;
    if (p == KP_IPA) I.has_ipa = true;
  }
  I.tables_on = I.has_pts || I.has_ipa;
  F.fit_strategy = cfg.fit_strategy;
  F.fit_n = cfg.fit_n;
  F.ba_n = cfg.ba_n;
  F.rtc_n = cfg.rtc_n;
  for (int i = 0; i < KSG_MAX_SCORE_RES; ++i) {
    F.fit_res[i] = cfg.fit_res[i];
    F.fit_w[i] = cfg.fit_w[i];
    F.ba_res[i] = cfg.ba_res[i];
  }
  for (int i = 0; i < KSG_MAX_RTC; ++i) {
    F.rtc_util[i] = cfg.rtc_util[i];
    F.rtc_score[i] = cfg.rtc_score[i];
  }
  F.ipa_hard_weight = cfg.ipa_hard_weight;
  F.ipa_ignore_existing_pref = cfg.ipa_ignore_existing_pref;
  F.seed = cfg.seed;
  F.pos_fit = F.pos_ba = F.pos_taint = F.pos_na = -1;
  F.w_fit = F.w_ba = F.w_taint = F.w_na = 0;
  for (int i = 0; i < F.n; ++i) {
    if (F.plugins[i] == KP_TAINT) { F.pos_taint = i; F.w_taint = F.weight[i]; }
    if (F.plugins[i] == KP_NA) { F.pos_na = i; F.w_na = F.weight[i]; }
    if (F.plugins[i] == KP_FIT) { F.pos_fit = i; F.w_fit = F.weight[i]; }
    if (F.plugins[i] == KP_BA) { F.pos_ba = i; F.w_ba = F.weight[i]; }
  }
  if (!set_score_resources(F.fit_res, F.ba_res, err)) return false;
  I.static_ok = F.n > 0 && (F.pos_taint >= 0 || F.pos_na >= 0);
  for (int i = 0; i < F.n; ++i)
    I.static_ok &= (F.plugins[i] == KP_FIT || F.plugins[i] == KP_BA || F.plugins[i] == KP_TAINT || F.plugins[i] == KP_NA);
  if (!I.saux.alloc(4, err)) return false;
  HIPCHK(hipMemsetAsync(I.saux.p, 0, 4 * sizeof(int32_t), I.stream));
  I.batch_ok = F.n > 0;
  for (int i = 0; i < F.n; ++i)
    I.batch_ok &= (F.plugins[i] == KP_FIT || F.plugins[i] == KP_BA || F.plugins[i] == KP_TAINT || F.plugins[i] == KP_NA);
  I.batch_static = I.batch_ok && I.static_ok;
  if (const char* e = std::getenv("KSG_STATIC_CHUNK")) {  // diagnostic (tests): smaller static chunks
    long v = std::strtol(e, nullptr, 10);
    I.stat_chunk_cap = v > 0 ? (uint32_t)std::max<long>(KSG_BATCH, v / KSG_BATCH * KSG_BATCH) : 0;
  }
  return true;
}

static uint32_t eval_tiles(uint32_t N, uint32_t cus);
static uint32_t tt_ring();
bool Engine::upload(const NodeSoA& ns, const PodTableSoA& pt, uint32_t pod_cap, uint32_t term_cap, uint32_t req_cap,
                    uint32_t val_cap, std::string& err) {
  Impl& I = *p_;
  hipStream_t s = I.stream;
  if (ns.topo_key.size() > KSG_MAX_TOPO) { err = "too many topology keys"; return false; }
  if (ns.n_res > KSG_MAX_RES) { err = "too many resources"; return false; }
  I.N = ns.n;
  I.goff = ns.global_offset;
  I.G = std::max(ns.global_n, ns.global_offset + ns.n);
  I.static_fits = true;
  I.max_taints = 0;
  for (uint32_t i = 0; i < ns.n; ++i) I.max_taints = std::max(I.max_taints, ns.taint_off[i + 1] - ns.taint_off[i]);
  I.max_tid = -1;
  for (int32_t t : ns.taint_id) I.max_tid = std::max(I.max_tid, t);
  {
    const int64_t lim = (int64_t)1 << 45;
    auto in = [&](int64_t v) { return v > -lim && v < lim; };
    I.cols_small = ns.n_res >= 2;
    for (uint32_t i = 0; i < ns.n && I.cols_small; ++i)
      I.cols_small = in(ns.alloc[i]) && in(ns.alloc[(size_t)ns.n + i]) && in(ns.requested[i]) &&
                     in(ns.requested[(size_t)ns.n + i]) && in(ns.nz_cpu[i]) && in(ns.nz_mem[i]);
  }
  I.taint_dup = false;  // a node listing one taint twice (the class path counts taint sets)
  for (uint32_t i = 0; i < ns.n && !I.taint_dup && I.max_tid < 64; ++i) {
    uint64_t seen = 0;
    for (uint32_t k = ns.taint_off[i]; k < ns.taint_off[i + 1]; ++k) {
      const uint64_t b = 1ull << (ns.taint_id[k] & 63);
      I.taint_dup |= (seen & b) != 0;
      seen |= b;
    }
  }
  I.gstat = !ns.g_label_vid.empty();
  if (I.gstat) {
    if (ns.g_label_vid.size() != (size_t)ns.n_keys * I.G || ns.g_taint_off.size() != (size_t)I.G + 1) {
      err = "sharded upload: global static columns do not match the cluster";
      return false;
    }
    for (uint32_t g = 0; g < I.G; ++g) I.max_taints = std::max(I.max_taints, ns.g_taint_off[g + 1] - ns.g_taint_off[g]);
    std::vector<int32_t> gl = ns.g_label_vid, gt = ns.g_taint_id;
    gl.resize(std::max<size_t>(gl.size(), 1), -1);
    gt.resize(std::max<size_t>(gt.size(), 1), 0);
    if (!I.glabel.upload(gl, s, err) || !I.gtoff.upload(ns.g_taint_off, s, err) || !I.gtid.upload(gt, s, err)) return false;
  }
  if (I.max_taints >= 4096) I.static_fits = false;
  I.R = ns.n_res;
  I.K = ns.n_keys;
  if (!I.alloc.upload(ns.alloc, s, err) || !I.req.upload(ns.requested, s, err) || !I.nzc.upload(ns.nz_cpu, s, err) ||
      !I.nzm.upload(ns.nz_mem, s, err) || !I.allowed.upload(ns.allowed_pods, s, err) ||
      !I.podcnt.upload(ns.pod_count, s, err) || !I.label.upload(ns.label_vid, s, err) ||
      !I.toff.upload(ns.taint_off, s, err) || !I.tid.upload(ns.taint_id, s, err) ||
      !I.haslab.upload(ns.has_labels, s, err) || !I.kvo.upload(ns.key_val_off, s, err) ||
      !I.vnum.upload(ns.val_num, s, err) || !I.vok.upload(ns.val_num_ok, s, err))
    return false;
  {
    std::vector<uint8_t> nf = ns.node_flags;
    nf.resize(ns.n, 0);
    I.img_words = ns.img_words;
    I.n_ports = ns.n_ports;
    if (ns.img_bits.size() != (size_t)ns.img_words * ns.n || ns.port_count.size() != (size_t)ns.n_ports * ns.n) {
      err = "node image / host-port columns do not match the node count";
      return false;
    }
    if (!I.nflags.upload(nf, s, err) || !I.img.upload(ns.img_bits, s, err) || !I.ports.upload(ns.port_count, s, err) ||
        !I.ports0.upload(ns.port_count, s, err))
      return false;
    std::vector<int32_t> pu = ns.pvc_use;
    pu.resize(std::max<size_t>(pu.size(), 1), 0);
    I.n_pvc = (uint32_t)pu.size();
    if (!I.pvcuse.upload(pu, s, err) || !I.pvcuse0.upload(pu, s, err)) return false;
    std::vector<int32_t> vl = ns.vol_limit, va = ns.vol_attached, vn = ns.vol_node, vr = ns.vol_ref;
    vl.resize(std::max<size_t>(vl.size(), 1), -1);
    va.resize(std::max<size_t>(va.size(), 1), 0);
    vn.resize(std::max<size_t>(vn.size(), 1), -1);
    vr.resize(std::max<size_t>(vr.size(), 1), 0);
    I.n_vatt = (uint32_t)va.size();
    I.n_vnode = (uint32_t)vn.size();
    if (!I.vlim.upload(vl, s, err) || !I.vatt.upload(va, s, err) || !I.vatt0.upload(va, s, err) ||
        !I.vnode.upload(vn, s, err) || !I.vnode0.upload(vn, s, err) || !I.vref.upload(vr, s, err) ||
        !I.vref0.upload(vr, s, err))
      return false;
  }
  I.topo = NodeSoA();
  I.topo.topo_key = ns.topo_key;
  I.topo.topo_base = ns.topo_base;
  I.topo.topo_count = ns.topo_count;
  I.topo.topo_pairs = ns.topo_pairs;
  I.topo.nu_base = ns.nu_base;
  {
    std::vector<uint32_t> sp;
    I.uniq = 0;
    for (size_t t = 0; t < ns.topo_key.size(); ++t) {
      const bool u = t < ns.topo_unique.size() && ns.topo_unique[t];
      if (u) I.uniq |= 1u << t;
      else
        for (uint32_t v = 0; v < ns.topo_count[t]; ++v) sp.push_back(ns.topo_base[t] + v);
    }
    I.nsp = (uint32_t)sp.size();
    if (!I.spair.upload(sp, s, err) || !I.xregcnt.alloc(KSG_MAX_TSC, err)) return false;
  }
  if (!I.topo_key_d.upload(ns.topo_key, s, err) || !I.topo_base_d.upload(ns.topo_base, s, err) ||
      !I.topo_count_d.upload(ns.topo_count, s, err))
    return false;
  {  // class tables: the definitions come from the host registry after the upload (add_classes)
    I.npc = I.ntc = I.nct = I.ncreq = I.ncval = I.tc_used = 0;
    I.tc_off_h.clear();
    I.tc_slot_h.clear();
    I.NU = ns.nu_pairs;
    std::vector<uint32_t> nb(KSG_MAX_TOPO, 0xFFFFFFFFu);
    std::vector<int32_t> sd(KSG_MAX_TOPO, 0);
    for (size_t t = 0; t < ns.nu_base.size() && t < KSG_MAX_TOPO; ++t) nb[t] = ns.nu_base[t];
    for (size_t t = 0; t < ns.slot_dom.size() && t < KSG_MAX_TOPO; ++t) sd[t] = ns.slot_dom[t];
    std::vector<uint8_t> pn = ns.pair_node;
    pn.resize(std::max<size_t>(ns.topo_pairs, 1), 0);
    if (!I.nu_base_d.upload(nb, s, err) || !I.slot_dom_d.upload(sd, s, err) || !I.pair_node_d.upload(pn, s, err))
      return false;
    I.shards = std::max<uint32_t>(ns.shards, 1);
    I.red_pc0 = I.red_tc0 = UINT32_MAX;
    if (I.shards > 1) {
      if (ns.gtopo.size() != ns.topo_key.size() * (size_t)I.G) { err = "sharded upload without the topology table"; return false; }
      std::vector<int32_t> gt = ns.gtopo;
      gt.resize(std::max<size_t>(gt.size(), 1), -1);
      if (!I.gtopo_d.upload(gt, s, err)) return false;
    }
    I.cnblk = std::max<uint32_t>((ns.n + kChain - 1) / kChain, 1);
    if (!I.carrive.alloc(1, err) || !I.cpi.alloc((size_t)KCP_I * I.cnblk, err) ||
        !I.cpst.alloc(I.cnblk, err) ||
        !I.cpm.alloc((size_t)2 * KCP_X * I.cnblk, err) || !I.cpm2.alloc((size_t)2 * I.cnblk, err) ||
        !I.cpr.alloc((size_t)KSG_MAX_TSC * I.cnblk, err) || !I.cpk.alloc(I.cnblk, err) ||
        !I.ccand.alloc((size_t)kChain * I.cnblk, err))
      return false;
    HIPCHK(hipMemsetAsync(I.carrive.p, 0, sizeof(uint32_t), s));
  }
  // existing-pod table (capacity for device-side appends)
  I.pcap = std::max<uint32_t>(pod_cap, pt.n);
  I.pkeys = pt.n_keys;
  I.tcap = std::max<uint32_t>(term_cap, (uint32_t)pt.terms.size());
  I.rcap = std::max<uint32_t>(req_cap, (uint32_t)pt.reqs.size());
  I.vcap = std::max<uint32_t>(val_cap, (uint32_t)pt.vals.size());
  if (!I.ptnode.alloc(I.pcap, err) || !I.ptns.alloc(I.pcap, err) || !I.ptflags.alloc(I.pcap, err) ||
      !I.ptlab.alloc((size_t)I.pcap * std::max<uint32_t>(I.pkeys, 1), err) || !I.terms.alloc(I.tcap, err) ||
      !I.tpod.alloc(I.tcap, err) || !I.treq.alloc(I.rcap, err) || !I.tval.alloc(I.vcap, err) ||
      !I.tcounts.alloc(8, err))
    return false;
  if (pt.n) {
    HIPCHK(hipMemcpyAsync(I.ptnode.p, pt.node.data(), pt.n * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(I.ptns.p, pt.ns.data(), pt.n * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(I.ptflags.p, pt.flags.data(), pt.n * 4, hipMemcpyHostToDevice, s));
    for (uint32_t k = 0; k < pt.n_keys; ++k)
      HIPCHK(hipMemcpyAsync(I.ptlab.p + (size_t)k * I.pcap, pt.label_vid.data() + (size_t)k * pt.n, pt.n * 4,
                            hipMemcpyHostToDevice, s));
  }
  if (!pt.terms.empty()) {
    HIPCHK(hipMemcpyAsync(I.terms.p, pt.terms.data(), pt.terms.size() * sizeof(ksg_exist_term), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(I.tpod.p, pt.term_pod.data(), pt.term_pod.size() * 4, hipMemcpyHostToDevice, s));
  }
  if (!pt.reqs.empty())
    HIPCHK(hipMemcpyAsync(I.treq.p, pt.reqs.data(), pt.reqs.size() * sizeof(ksg_req), hipMemcpyHostToDevice, s));
  if (!pt.vals.empty())
    HIPCHK(hipMemcpyAsync(I.tval.p, pt.vals.data(), pt.vals.size() * 4, hipMemcpyHostToDevice, s));
  uint32_t counts[8] = {pt.n, (uint32_t)pt.terms.size(), (uint32_t)pt.reqs.size(), (uint32_t)pt.vals.size(), 0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(I.tcounts.p, counts, sizeof(counts), hipMemcpyHostToDevice, s));
  std::memcpy(I.counts0, counts, sizeof(counts));
  size_t RN = (size_t)I.R * std::max<uint32_t>(I.N, 1);
  if (!I.req0.alloc(RN, err) || !I.nzc0.alloc(std::max<uint32_t>(I.N, 1), err) ||
      !I.nzm0.alloc(std::max<uint32_t>(I.N, 1), err) || !I.podcnt0.alloc(std::max<uint32_t>(I.N, 1), err))
    return false;
  HIPCHK(hipMemcpyAsync(I.req0.p, I.req.p, (size_t)I.R * I.N * 8, hipMemcpyDeviceToDevice, s));
  HIPCHK(hipMemcpyAsync(I.nzc0.p, I.nzc.p, (size_t)I.N * 8, hipMemcpyDeviceToDevice, s));
  HIPCHK(hipMemcpyAsync(I.nzm0.p, I.nzm.p, (size_t)I.N * 8, hipMemcpyDeviceToDevice, s));
  HIPCHK(hipMemcpyAsync(I.podcnt0.p, I.podcnt.p, (size_t)I.N * 4, hipMemcpyDeviceToDevice, s));
  // scratch + outputs
  size_t pairs = std::max<uint32_t>(ns.topo_pairs, 1);
  if (!I.cnt.alloc((size_t)KSG_MAX_TSC * std::max<uint32_t>(I.N, 1), err) || !I.hist_f.alloc(pairs, err) ||
      !I.hist_s.alloc(pairs, err) || !I.present_f.alloc(pairs, err) || !I.reg.alloc(pairs, err) ||
      !I.ipa_aff.alloc(pairs, err) || !I.ipa_anti.alloc(pairs, err) || !I.ipa_exist.alloc(pairs, err) ||
      !I.ipa_score.alloc(pairs, err) || !I.pts_min.alloc(KSG_MAX_TOPO, err) || !I.pts_dom.alloc(KSG_MAX_TOPO, err) ||
      !I.exist_any.alloc(1, err) || !I.filter.alloc(std::max<uint32_t>(I.N, 1), err) ||
      !I.score.alloc((size_t)KSG_MAX_PLUGINS * std::max<uint32_t>(I.N, 1), err) ||
      !I.total.alloc(std::max<uint32_t>(I.N, 1), err))
    return false;
  HIPCHK(hipMemsetAsync(I.exist_any.p, 0, 4, s));
  if (I.batch_ok && I.R <= 4) {
    uint32_t T = eval_tiles(I.N, I.n_cus);
    size_t Nn = std::max<uint32_t>(I.N, 1);
    if (!I.tile_top.alloc((size_t)tt_ring() * KSG_BATCH * T * KSG_TOPK, err) || !I.tfeas.alloc((size_t)tt_ring() * KSG_BATCH * T * 3, err) ||
        !I.arrive.alloc(2 * KSG_BATCH * 32, err) || !I.pend_n.alloc(2, err) || !I.wrec.alloc(2 * kRecBytes, err) ||
        !I.pend.alloc(2 * KSG_BATCH, err) || !I.bfilter.alloc(Nn * 2 * KSG_BATCH, err) ||
        !I.bscore.alloc(Nn * 2 * KSG_BATCH * KSG_MAX_PLUGINS, err) || !I.btotal.alloc(Nn * 2 * KSG_BATCH, err))
      return false;
    HIPCHK(hipMemsetAsync(I.arrive.p, 0, 2 * KSG_BATCH * 32 * 4, s));
    HIPCHK(hipMemsetAsync(I.pend_n.p, 0, 2 * 4, s));
    HIPCHK(hipMemsetAsync(I.wrec.p, 0, 2 * kRecBytes, s));
  }
  if (!stream_sync(I, s, err)) return false;
  return true;
}

// Eval tiles per pod: the fewest nodes per thread (npt) with which a window's
// eval blocks (one per CU: 1,024 threads, the window LDS) fit the CUs beside the
// replay block in one round; at most 16 (then several rounds).  (Tiles balanced
// to fill every CU were measured slower: the replay block's memory latency
// grows with the eval blocks around it.)
// Windows' tile-list slots (KSG_TT_RING, default 2: window parity)
static uint32_t tt_ring() {
  static const uint32_t r = [] {
    const char* e = std::getenv("KSG_TT_RING");
    const uint32_t v = e ? (uint32_t)std::strtoul(e, nullptr, 10) : 2u;
    return v < 2 ? 2u : (v > 64 ? 64u : v);
  }();
  return r;
}
static uint32_t eval_npt(uint32_t N, uint32_t cus) {
  static const uint32_t forced = [] {  // KSG_WIN_NPT: nodes per thread of the window's eval tiles (A/B)
    const char* e = std::getenv("KSG_WIN_NPT");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;
  }();
  if (forced) return std::min<uint32_t>(forced, 16);
  uint32_t npt = 1;
  while (npt < 16 && (uint64_t)KSG_BATCH * ((N + KSG_TILE * npt - 1) / (KSG_TILE * npt)) + 1 > cus) ++npt;
  return npt;
}
static uint32_t eval_tiles(uint32_t N, uint32_t cus) {
  const uint32_t npt = eval_npt(N, cus);
  return std::max<uint32_t>((N + KSG_TILE * npt - 1) / (KSG_TILE * npt), 1);
}

// The handshake verdict of the persistent launch just queued (k_chain_run,
// k_window_run): the host waits for it (the work queued before runs first).
// 1 go, 2 not co-resident (its blocks left untouched), 3 an earlier launch of the
// call aborted; 0 with err set: the launch never decided (state lost).
static uint32_t wait_verdict(Engine::Impl& I, hipStream_t s, std::string& err);
// Windows of KSG_BATCH pods, one k_window launch each (see the kernel): launch
// j evaluates window j+1 and replays window j; the sharded path all-gathers
// each window's candidate records between launches.
static bool xgather(Engine::Impl& I, size_t bytes, std::string& err, const uint8_t* src = nullptr,
                    hipStream_t st = nullptr);
static bool tables_ready(Engine::Impl& I, std::string& err);
// Sharded windows, split over three streams so that the exchange leaves the
// replay's critical path.  Window j's evaluation (eval-only k_window launch,
// engine stream) needs the rows as of the end of window j-2, i.e. only the
// replay of j-2; its all-gather and merge run on the exchange stream; the
// replay of j (replay-only launch, replay stream) waits for the merge of j.
// Per window: max(eval, exchange, replay) instead of their sum.  Buffer reuse is
// ordered by those waits: window j's tile lists, send buffer, output-ring slots
// and P-list slot are those of window j-2, whose replay it waited for (and that
// replay waited for j-2's exchange).
static bool run_batches_split(Engine::Impl& I, const WinArgs& A0, uint32_t first, uint32_t count, uint32_t T,
                              std::string& err) {
  hipStream_t s = I.stream;
  DevCluster C = I.cluster();
  if (!I.rstream) {
    HIPCHK(hipStreamCreateWithFlags(&I.rstream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&I.xstream, hipStreamNonBlocking));
    for (hipEvent_t* e : {&I.xg[0], &I.xg[1], &I.xr[0], &I.xr[1], &I.xe[0], &I.xe[1], &I.xjoin})
      HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  hipStream_t sr = I.rstream, sx = I.xstream;
  if (!I.xsend.grow(2 * kRecBytes, 0, s, err)) return false;  // one send record per window parity
  HIPCHK(hipEventRecord(I.xjoin, s));  // the other streams start after the run's set-up
  HIPCHK(hipStreamWaitEvent(sr, I.xjoin, 0));
  HIPCHK(hipStreamWaitEvent(sx, I.xjoin, 0));
  const uint32_t nwin = (count + KSG_BATCH - 1) / KSG_BATCH;
  const size_t tt_sz = (size_t)KSG_BATCH * T * KSG_TOPK, tf_sz = (size_t)KSG_BATCH * T * 3;
  const dim3 blk(KSG_WIN_THREADS);
  auto launch = [&](hipStream_t st, const WinArgs& a, uint32_t blocks) {
    if (I.eval_mode == 1) hipLaunchKernelGGL((k_window<1, false>), dim3(blocks), blk, sizeof(WinLDS), st, C, I.F, a);
    else hipLaunchKernelGGL((k_window<0, false>), dim3(blocks), blk, sizeof(WinLDS), st, C, I.F, a);
  };
  for (int64_t j = 0; j <= (int64_t)nwin; ++j) {
    if (j < (int64_t)nwin) {  // evaluation of window E = j, exchange, merge (engine stream)
      const int64_t E = j, P = E - 2;
      WinArgs a = A0;
      a.nw = 0;
      a.stamps = nullptr;
      a.e0 = first + (uint32_t)E * KSG_BATCH;
      a.ne = std::min<uint32_t>(KSG_BATCH, first + count - a.e0);
      a.tile_top = I.tile_top.p + (size_t)(E % tt_ring()) * tt_sz;
      a.tile_feas = I.tfeas.p + (size_t)(E % tt_ring()) * tf_sz;
      a.erec = I.xsend.p + (size_t)(E & 1) * kRecBytes;
      a.estamps = I.stamps_on ? I.stamps.p + (size_t)E * 32 : nullptr;
      a.pprev = I.pend.p + (size_t)(P & 1) * KSG_BATCH;
      a.pprev_n = I.pend_n.p + (P & 1);
      if (E >= 2) HIPCHK(hipStreamWaitEvent(s, I.xr[E & 1], 0));  // the replay of E-2
      const bool sampled = I.sample_every && I.n_samples * 2 + 2 <= I.sev.size();
      if (sampled) HIPCHK(hipEventRecord(I.sev[I.n_samples * 2], s));
      launch(s, a, 1 + a.ne * T);
      if (sampled) {
        HIPCHK(hipEventRecord(I.sev[I.n_samples * 2 + 1], s));
        I.n_samples++;
      }
      HIPCHK(hipEventRecord(I.xe[E & 1], s));
      HIPCHK(hipStreamWaitEvent(sx, I.xe[E & 1], 0));
      if (!xgather(I, kXchgBytes, err, a.erec, sx)) return false;
      hipLaunchKernelGGL(k_window_gmerge, dim3(a.ne), dim3(64), 0, sx, I.xrecv.p, I.xranks, I.xrows.p, a.pprev,
                         a.pprev_n, I.wrec.p + (size_t)(E & 1) * kRecBytes);
      HIPCHK(hipEventRecord(I.xg[E & 1], sx));
    }
    if (j >= 1) {  // replay of window W = j - 1 (replay stream)
      const int64_t W = j - 1, P = W - 1;
      WinArgs a = A0;
      a.ne = 0;
      a.estamps = nullptr;
      a.w0 = first + (uint32_t)W * KSG_BATCH;
      a.nw = std::min<uint32_t>(KSG_BATCH, first + count - a.w0);
      a.wrec = I.wrec.p + (size_t)(W & 1) * kRecBytes;
      a.pnext = I.pend.p + (size_t)(W & 1) * KSG_BATCH;
      a.pnext_n = I.pend_n.p + (W & 1);
      a.pprev = I.pend.p + (size_t)(P & 1) * KSG_BATCH;
      a.pprev_n = I.pend_n.p + (P & 1);
      a.stamps = I.stamps_on ? I.stamps.p + (size_t)W * 32 : nullptr;
      HIPCHK(hipStreamWaitEvent(sr, I.xg[W & 1], 0));  // its merged candidates
      launch(sr, a, 1);
      HIPCHK(hipEventRecord(I.xr[W & 1], sr));
    }
  }
  if (nwin) {
    const int64_t L = nwin - 1;
    hipLaunchKernelGGL(k_apply_pend, dim3(1), dim3(KSG_BATCH), 0, sr, C, I.pend.p + (size_t)(L & 1) * KSG_BATCH,
                       I.pend_n.p + (L & 1));
  }
  HIPCHK(hipEventRecord(I.xjoin, sr));  // everything after the run waits on the engine stream
  HIPCHK(hipStreamWaitEvent(s, I.xjoin, 0));  // (the replay stream's last wait covers the exchange stream)
  HIPCHK(hipEventRecord(I.ev1, s));
  HIPCHK(hipGetLastError());
  return true;
}
static bool run_batches(Engine::Impl& I, uint32_t first, uint32_t count, std::string& err) {
  if (I.R > 4) { err = "batch path supports at most 4 resource columns"; return false; }
  hipStream_t s = I.stream;
  DevCluster C = I.cluster();
  // nodes per eval thread: enough that one window's eval blocks fit the CUs
  // beside the replay block in one round (one 1,024-thread block per CU)
  const uint32_t T = eval_tiles(I.N, I.n_cus), npt = eval_npt(I.N, I.n_cus), tile_len = npt * KSG_TILE;
  const uint32_t nwin = (count + KSG_BATCH - 1) / KSG_BATCH;
  if (I.sample_every) {
    size_t need = 2 * (nwin + 2);
    while (I.sev.size() < need) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      I.sev.push_back(e);
    }
  }
  I.n_samples = 0;
  I.n_st = 0;
  I.stat_pods_sampled = 0;
  static bool attr = false;
  if (!attr) {
    const void* fns[4] = {(const void*)k_window<0, false>, (const void*)k_window<1, false>,
                          (const void*)k_window<0, true>, (const void*)k_window<1, true>};
    for (const void* f : fns) HIPCHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(WinLDS)));
    attr = true;
  }
  HIPCHK(hipEventRecord(I.ev0, s));
  HIPCHK(hipMemsetAsync(I.pend_n.p, 0, 2 * sizeof(int32_t), s));
  WinArgs A{};
  A.plite = I.plite.p;
  A.first = first;
  A.keep_first = I.keep_first;
  A.keep_n = I.keep_n;
  A.need_eph = I.any_eph_req ? 1u : 0u;
  A.kfilter = I.kfilter.p; A.kscore = I.kscore.p; A.ktotal = I.ktotal.p;
  A.sfilter = I.bfilter.p; A.sscore = I.bscore.p; A.stotal = I.btotal.p;
  A.T = T;
  A.npt = npt;
  A.tile_len = tile_len;
  // deferred tile merge (KSG_DEFER_MERGE=1, single shard): measured slower on
  // cfg2 and cfg3 — merging 32 pods' tile lists costs the replay block ~9 us,
  // more than the evaluation's own merge costs its chain
  A.defer = 0;
  A.stash_npt = kStashNpt;
  if (const char* e = std::getenv("KSG_DEFER_MERGE")) A.defer = (std::strtol(e, nullptr, 10) != 0 && I.xranks <= 1) ? 1u : 0u;
  const size_t tt_sz = (size_t)KSG_BATCH * T * KSG_TOPK, tf_sz = (size_t)KSG_BATCH * T * 3;
  A.tile_top = I.tile_top.p;
  A.tile_feas = I.tfeas.p;
  A.arrive = I.arrive.p;
  A.astride = 1;
  A.sums = I.sums.p;
  const bool sharded = I.xranks > 1;
  A.xrows = nullptr;
  if (sharded) {  // every node's row on every rank (kXchgBytes exchanges: keys only)
    const uint32_t G = std::max<uint32_t>(I.G, 1), stride = (G + I.xranks - 1) / I.xranks;
    if (!I.xrows.alloc(G, err)) return false;
    const size_t bytes = (size_t)stride * sizeof(RowV);
    if (!I.xsend.grow(std::max(bytes, 2 * kRecBytes), 0, s, err) || !I.xrecv.grow(bytes * I.xranks, 0, s, err))
      return false;
    if (I.N) hipLaunchKernelGGL(k_rows_pack, dim3((I.N + 255) / 256), dim3(256), 0, s, C, I.any_eph_req ? 1u : 0u,
                                reinterpret_cast<RowV*>(I.xsend.p));
    if (!xgather(I, bytes, err)) return false;
    hipLaunchKernelGGL(k_rows_unpack, dim3((stride + 255) / 256, I.xranks), dim3(256), 0, s,
                       reinterpret_cast<const RowV*>(I.xrecv.p), I.xranks, G, stride, I.xrows.p);
    A.xrows = I.xrows.p;
  }
  // static records: a ring of two chunks of whole windows (window j+1's eval and
  // window j's replay may sit in consecutive chunks); chunk c computed by k_static
  // just before the launch that evaluates its first window
  //
  // Inline: chunk c is computed on the engine stream just before the launch
  // that evaluates its first window (ring of 2 chunks).  Side stream (default):
  // k_static runs on a low-priority stream two chunks ahead, on the CUs the
  // window launches leave idle; ring of 3 chunks, two events per chunk:
  // ready(c) before the launch evaluating chunk c's first window, and the slot
  // of chunk c+2 free after the launch replaying chunk c-1's last window.
  const bool stat = I.batch_static;
  const bool side = stat && I.sstream && I.static_side;
  // the persistent window loop over static records: every record of the run
  // computed before the launch (one chunk; the loop has no ring to roll), when
  // they fit KSG_STATIC_RUN_MB (default 16 GiB of the 288 GB)
  const bool persist_ok = !sharded && I.win_run_on && nwin > 0 && 1 + (uint64_t)KSG_BATCH * T <= I.n_cus;
  const uint32_t count32 = (count + KSG_BATCH - 1) / KSG_BATCH * KSG_BATCH;
  const uint64_t run_bytes = (uint64_t)count32 * std::max<uint32_t>(I.N, 1) * sizeof(StaticRec);
  bool stat_run = stat && !side && persist_ok && I.static_run_mb > 0 && !I.stat_chunk_cap &&
                  run_bytes <= ((uint64_t)I.static_run_mb << 20);
  if (stat_run && run_bytes > I.stat.n * sizeof(StaticRec)) {
    // (a run-sized buffer only while it leaves most of the device free: another
    // context or process may hold memory; otherwise the ring of chunks)
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || run_bytes > fr / 2) {
      (void)hipGetLastError();
      stat_run = false;
    }
  }
  uint32_t chunk = 0, nchunks = 0, nslots = 2;
  const bool gstat = stat && I.gstat && sharded;  // node-sharded: records over every node
  const DevCluster CS = gstat ? I.cluster_static() : C;
  const uint32_t SN = gstat ? I.G : I.N;
  A.stat_n = std::max<uint32_t>(SN, 1);
  A.stat_base = gstat ? 0 : I.goff;
  A.G = I.G;
  if (stat) {
    const size_t Nn = std::max<uint32_t>(SN, 1);
    auto size_ring = [&]() {
      nslots = stat_run ? 1 : side ? 3 : 2;
      const size_t budget = side ? ((size_t)32 << 20) : ((size_t)64 << 20);
      chunk = (uint32_t)std::max<size_t>(KSG_BATCH, (budget / (Nn * sizeof(StaticRec))) / KSG_BATCH * KSG_BATCH);
      chunk = std::min<uint32_t>(chunk, count32);
      if (I.stat_chunk_cap) chunk = std::min<uint32_t>(chunk, I.stat_chunk_cap);  // tests: force ring roll-over
      if (stat_run) chunk = count32;
      nchunks = (count + chunk - 1) / chunk;
    };
    size_ring();
    if (!I.stat.alloc((size_t)nslots * chunk * Nn, err)) {
      if (!stat_run) return false;
      (void)hipGetLastError();  // (the run-sized buffer did not fit after all: the ring)
      stat_run = false;
      size_ring();
      if (!I.stat.alloc((size_t)nslots * chunk * Nn, err)) return false;
    }
    if (!I.mpred.alloc(2 * (size_t)std::max<uint32_t>(count, 1), err)) return false;
    A.stat = I.stat.p;
    A.stat_ring = nslots * chunk;
    A.mpred = I.mpred.p;
    if (side && !I.sev_ready[0]) {
      for (auto* e : {&I.sev_ready[0], &I.sev_ready[1], &I.sev_ready[2], &I.sev_free})
        HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
  }
  // decoded pods (k_static_dec) when every pod of the chunk flattens and the
  // nodes' taints fit the id set (KSG_STATIC_DEC=0: the program-walking k_static)
  auto static_dec_ok = [&](uint32_t q0, uint32_t cn) {
    bool dec = I.static_dec && I.max_taints <= 4 && I.max_tid < 64 && !I.taint_dup;
    for (uint32_t q = q0; dec && q < q0 + cn; ++q) dec = (I.prog_need[q] & (1u << 19)) != 0;
    return dec;
  };
  // ready: k_static_dec beside the persistent loop, counting its pod groups there
  // (the maxima already reset on the engine stream)
  auto issue_static = [&](uint32_t c, hipStream_t st, uint32_t* ready = nullptr, uint32_t run_grid = 0,
                          uint32_t* arrive = nullptr) -> bool {
    const uint32_t q0 = first + c * chunk, cn = std::min(chunk, first + count - q0);
    if (!ready)
      HIPCHK(hipMemsetAsync(I.mpred.p + 2 * (size_t)(q0 - first), 0xFF, 2 * (size_t)cn * sizeof(int64_t), st));
    const dim3 sgrid(std::max<uint32_t>((SN + 256 * KSG_ST_NPT - 1) / (256 * KSG_ST_NPT), 1),
                     (cn + KSG_ST_PODS - 1) / KSG_ST_PODS);
    const bool ssamp = I.sample_every && (st == s || ready);
    if (ssamp) {
      while (I.sev_st.size() < 2 * (size_t)(I.n_st + 1)) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        I.sev_st.push_back(e);
      }
      HIPCHK(hipEventRecord(I.sev_st[2 * I.n_st], st));
    }
    StaticRec* const sout = I.stat.p + (size_t)((q0 - first) % (nslots * chunk)) * A.stat_n;
    const bool dec = static_dec_ok(q0, cn);
    if (ready && !dec) { err = "static records beside the loop: pods that do not decode"; return false; }
    if (dec) {
      if (!I.sd_pods.alloc((size_t)chunk * (sizeof(WcPod) / 8), err)) return false;
      WcPod* wp = reinterpret_cast<WcPod*>(I.sd_pods.p);
      hipLaunchKernelGGL(k_st_decode, dim3((cn + 63) / 64), dim3(64), 0, st, CS, I.F, I.progs.p, I.prog_off_d.p, q0, cn,
                         wp, gstat ? 1 : 0);
      const dim3 dgrid(std::max<uint32_t>((SN + 256 * KSG_SD_NPT - 1) / (256 * KSG_SD_NPT), 1),
                       (cn + KSG_SD_PODS - 1) / KSG_SD_PODS);
      if (run_grid) {  // (beside the persistent loop: a few 1,024-thread blocks walking the items)
        const uint32_t ntx = std::max<uint32_t>((SN + 1024 * KSG_SD_NPT - 1) / (1024 * KSG_SD_NPT), 1);
        const uint32_t items = ntx * ((cn + KSG_SD_PODS - 1) / KSG_SD_PODS);
        hipLaunchKernelGGL(k_static_dec_run, dim3(std::min(run_grid, items)), dim3(1024), 0, st, CS, I.F, wp, I.progs.p, cn,
                           sout, I.mpred.p + 2 * (size_t)(q0 - first), ready, ntx, items, arrive);
      } else {
        hipLaunchKernelGGL(k_static_dec, dgrid, dim3(256), 0, st, CS, I.F, wp, I.progs.p, cn, sout,
                           I.mpred.p + 2 * (size_t)(q0 - first), ready);
      }
      I.static_dec_chunks++;
    } else {
      hipLaunchKernelGGL(k_static, sgrid, dim3(256), 0, st, CS, I.F, I.progs.p, I.prog_off_d.p, q0, cn, sout,
                         I.mpred.p + 2 * (size_t)(q0 - first), gstat ? 1 : 0);
    }
    if (ssamp) {
      HIPCHK(hipEventRecord(I.sev_st[2 * I.n_st + 1], st));
      I.stat_pods_sampled += cn;
      I.n_st++;
    }
    if (side) HIPCHK(hipEventRecord(I.sev_ready[c % 3], st));
    return true;
  };
  if (side) {  // the side stream starts after the engine stream's work so far (uploads, previous runs)
    HIPCHK(hipEventRecord(I.sev_free, s));
    HIPCHK(hipStreamWaitEvent(I.sstream, I.sev_free, 0));
    for (uint32_t c = 0; c < std::min<uint32_t>(2, nchunks); ++c)
      if (!issue_static(c, I.sstream)) return false;
  }
  if (sharded && !stat) return run_batches_split(I, A, first, count, T, err);
  // the persistent window loop: one launch for every window (its blocks all
  // resident: one per CU); not co-resident -> the launch-per-window loop below
  if (persist_ok && (!stat || stat_run)) {
    // dedicated merge blocks (one per pod) when they fit beside the tile blocks
    const bool mb = I.win_mblocks && 1 + (uint64_t)KSG_BATCH * (T + 1) <= I.n_cus;
    const uint32_t grid = 1 + KSG_BATCH * T + (mb ? KSG_BATCH : 0);
    // the run's records: before the launch, or (KSG_STATIC_OVERLAP, default)
    // beside it — k_static_dec_run, one 1,024-thread block per CU the loop leaves
    // idle, launched on the side stream BEFORE the loop (its blocks then hold
    // those CUs and the loop's take the rest; kernels run one at a time, as under
    // a PMC pass, it simply completes first); the eval blocks wait per window for
    // their pods' groups (win_stat_gate).  The side blocks count themselves in
    // (one word after the groups' counters) and the loop's handshake goes only
    // once all of them have started: side blocks that never become resident
    // beside the loop send it to the per-window fallback before any state changes,
    // instead of a gate running out mid-run.
    const uint32_t side_grid = I.n_cus > grid ? I.n_cus - grid : 0;
    const bool overlap = stat_run && I.static_overlap && I.sstream && side_grid > 0 && static_dec_ok(first, count);
    const uint32_t sgroups = (count + KSG_SD_PODS - 1) / KSG_SD_PODS;
    uint32_t side_blocks = 0;
    auto issue_side = [&]() -> bool {
      if (!issue_static(0, I.sstream, I.sready.p, side_grid, I.sready.p + sgroups)) return false;
      HIPCHK(hipEventRecord(I.sev_ready[0], I.sstream));
      return true;
    };
    if (overlap) {
      const uint32_t ntx = std::max<uint32_t>((SN + 1024 * KSG_SD_NPT - 1) / (1024 * KSG_SD_NPT), 1);
      side_blocks = std::min<uint32_t>(side_grid, ntx * sgroups);
      if (!I.sready.alloc(sgroups + 1, err) || !I.sd_pods.alloc((size_t)chunk * (sizeof(WcPod) / 8), err)) return false;
      HIPCHK(hipMemsetAsync(I.sready.p, 0, (sgroups + 1) * sizeof(uint32_t), s));
      HIPCHK(hipMemsetAsync(I.mpred.p, 0xFF, 2 * (size_t)count * sizeof(int64_t), s));
      if (!I.sev_ready[0])
        for (auto* e : {&I.sev_ready[0], &I.sev_ready[1], &I.sev_ready[2], &I.sev_free})
          HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
      HIPCHK(hipEventRecord(I.sev_free, s));
      HIPCHK(hipStreamWaitEvent(I.sstream, I.sev_free, 0));
      if (I.static_beside_test == 0 && !issue_side()) return false;
    } else if (stat_run && !issue_static(0, s)) {  // (every record of the run)
      return false;
    }
    if (!I.wsync.alloc(1, err) || !I.rsync.alloc(1, err)) return false;
    if (!I.hverdict) {
      HIPCHK(hipHostMalloc((void**)&I.hverdict, 64, hipHostMallocCoherent | hipHostMallocMapped));
      HIPCHK(hipMemsetAsync(I.rsync.p, 0, sizeof(RunSync), s));  // (the sticky abort word starts clear)
    }
    static bool wattr = false;
    if (!wattr) {
      HIPCHK(hipFuncSetAttribute((const void*)k_window_run<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(WinLDS)));
      HIPCHK(hipFuncSetAttribute((const void*)k_window_run<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(WinLDS)));
      HIPCHK(hipFuncSetAttribute((const void*)k_window_run<0, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(WinLDS)));
      HIPCHK(hipFuncSetAttribute((const void*)k_window_run<1, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(WinLDS)));
      wattr = true;
    }
    HIPCHK(hipMemsetAsync(I.wsync.p, 0, sizeof(WinSync), s));
    HIPCHK(hipMemsetAsync(I.rsync.p, 0, kRunSyncReset, s));
    HIPCHK(hipMemsetAsync(I.arrive.p, 0, 2 * KSG_BATCH * 32 * sizeof(uint32_t), s));
    WinRunArgs R{};
    R.nwin = nwin;
    R.first = first;
    R.count = count;
    R.T = T;
    R.tt_sz = (uint32_t)tt_sz;
    R.tf_sz = (uint32_t)tf_sz;
    R.tile_top = I.tile_top.p;
    R.tfeas = I.tfeas.p;
    R.wrec = I.wrec.p;
    R.pend = I.pend.p;
    R.pend_n = I.pend_n.p;
    R.arrive = I.arrive.p;
    R.stamps = I.stamps_on ? I.stamps.p : nullptr;
    R.sready = overlap ? I.sready.p : nullptr;
    R.sready_need = std::max<uint32_t>((SN + 1024 * KSG_SD_NPT - 1) / (1024 * KSG_SD_NPT), 1);  // (k_static_dec_run's node tiles)
    WinArgs AP = A;
    AP.mblocks = mb ? 1u : 0u;
    AP.astride = 32;
    AP.prior_fix = I.win_pfix ? 1u : 0u;
    AP.split = I.win_split ? 1u : 0u;
    __atomic_store_n(I.hverdict, 0u, __ATOMIC_RELEASE);
    RunCtl RC{grid + I.run_need_extra, I.run_wait_us * 100u, 0, I.hverdict, I.run_spin};
    if (overlap) {
      RC.side_arrive = I.sready.p + sgroups;
      RC.side_need = side_blocks;
    }
    const bool sampled = I.sample_every && I.n_samples * 2 + 2 <= I.sev.size();
    if (sampled) HIPCHK(hipEventRecord(I.sev[I.n_samples * 2], s));
    if (stat_run) {
      if (I.eval_mode == 1)
        hipLaunchKernelGGL((k_window_run<1, true>), dim3(grid), dim3(KSG_WIN_THREADS), sizeof(WinLDS), s, C, I.F, AP, R, I.rsync.p, I.wsync.p, RC);
      else
        hipLaunchKernelGGL((k_window_run<0, true>), dim3(grid), dim3(KSG_WIN_THREADS), sizeof(WinLDS), s, C, I.F, AP, R, I.rsync.p, I.wsync.p, RC);
    } else if (I.eval_mode == 1) {
      hipLaunchKernelGGL(k_window_run<1>, dim3(grid), dim3(KSG_WIN_THREADS), sizeof(WinLDS), s, C, I.F, AP, R, I.rsync.p, I.wsync.p, RC);
    } else {
      hipLaunchKernelGGL(k_window_run<0>, dim3(grid), dim3(KSG_WIN_THREADS), sizeof(WinLDS), s, C, I.F, AP, R, I.rsync.p, I.wsync.p, RC);
    }
    if (sampled) {
      HIPCHK(hipEventRecord(I.sev[I.n_samples * 2 + 1], s));
      I.n_samples++;
    }
    HIPCHK(hipGetLastError());
    if (overlap && I.static_beside_test == 1 && !issue_side()) return false;  // (tests: launched after the loop)
    I.run_used = true;
    const uint32_t v = wait_verdict(I, s, err);
    if (overlap && I.static_beside_test == 2 && !issue_side()) return false;  // (tests: after the verdict)
    if (v == 0u) return false;
    if (v == 3u) {
      I.lost = true;
      err = "persistent launch: a gate never completed (blocks not co-resident?)";
      return false;
    }
    if (v == 1u) {
      I.win_runs++;
      if (overlap) {  // (the run's last kernel after the side stream's records)
        HIPCHK(hipStreamWaitEvent(s, I.sev_ready[0], 0));
        I.static_overlaps++;
      }
      const int64_t L = nwin - 1;
      hipLaunchKernelGGL(k_apply_pend, dim3(1), dim3(KSG_BATCH), 0, s, C, I.pend.p + (size_t)(L & 1) * KSG_BATCH,
                         I.pend_n.p + (L & 1));
      HIPCHK(hipEventRecord(I.ev1, s));
      HIPCHK(hipGetLastError());
      return true;
    }
    I.win_fallbacks++;  // v == 2: its blocks left untouched; the per-window launches
    if (sampled) I.n_samples--;
    // (the side kernel's records and maxima are rewritten by the per-window loop's
    // k_static: it waits for the side kernel first)
    if (overlap) HIPCHK(hipStreamWaitEvent(s, I.sev_ready[0], 0));
  }
  for (int64_t j = -1; j < (int64_t)nwin; ++j) {
    const int64_t E = j + 1, W = j;
    A.ne = 0;
    A.nw = 0;
    A.stamps = A.estamps = nullptr;
    A.tile_top = I.tile_top.p + (size_t)(E % tt_ring()) * tt_sz;
    A.tile_feas = I.tfeas.p + (size_t)(E % tt_ring()) * tf_sz;
    A.wtile_top = I.tile_top.p + (size_t)(W % tt_ring()) * tt_sz;
    A.wtile_feas = I.tfeas.p + (size_t)(W % tt_ring()) * tf_sz;
    if (E < (int64_t)nwin) {
      A.estamps = I.stamps_on ? I.stamps.p + (size_t)E * 32 : nullptr;
      A.e0 = first + (uint32_t)E * KSG_BATCH;
      A.ne = std::min<uint32_t>(KSG_BATCH, first + count - A.e0);
      A.erec = sharded ? I.xsend.p : I.wrec.p + (size_t)(E & 1) * kRecBytes;
    }
    if (W >= 0) {
      A.w0 = first + (uint32_t)W * KSG_BATCH;
      A.nw = std::min<uint32_t>(KSG_BATCH, first + count - A.w0);
      A.wrec = I.wrec.p + (size_t)(W & 1) * kRecBytes;
      A.pnext = I.pend.p + (size_t)(W & 1) * KSG_BATCH;
      A.pnext_n = I.pend_n.p + (W & 1);
      A.stamps = I.stamps_on ? I.stamps.p + (size_t)W * 32 : nullptr;
    }
    const int64_t P = W - 1;  // P_{W-1}: the list the eval part overrides rows from, too
    A.pprev = I.pend.p + (size_t)(P & 1) * KSG_BATCH;
    A.pprev_n = I.pend_n.p + (P & 1);
    const bool chunk_start = stat && A.ne && (A.e0 - first) % chunk == 0;
    const uint32_t cidx = chunk_start ? (A.e0 - first) / chunk : 0;
    if (chunk_start) {
      if (side) HIPCHK(hipStreamWaitEvent(s, I.sev_ready[cidx % 3], 0));
      else if (!issue_static(cidx, s)) return false;
    }
    bool sampled = I.sample_every && A.ne && A.nw && I.n_samples * 2 + 2 <= I.sev.size();
    if (sampled) HIPCHK(hipEventRecord(I.sev[I.n_samples * 2], s));
    dim3 grid(1 + A.ne * T);
    const dim3 blk(KSG_WIN_THREADS);
    if (stat) {
      if (I.eval_mode == 1) hipLaunchKernelGGL((k_window<1, true>), grid, blk, sizeof(WinLDS), s, C, I.F, A);
      else hipLaunchKernelGGL((k_window<0, true>), grid, blk, sizeof(WinLDS), s, C, I.F, A);
    } else {
      if (I.eval_mode == 1) hipLaunchKernelGGL((k_window<1, false>), grid, blk, sizeof(WinLDS), s, C, I.F, A);
      else hipLaunchKernelGGL((k_window<0, false>), grid, blk, sizeof(WinLDS), s, C, I.F, A);
    }
    if (sampled) {
      HIPCHK(hipEventRecord(I.sev[I.n_samples * 2 + 1], s));
      I.n_samples++;
    }
    if (side && chunk_start && cidx + 2 < nchunks) {  // chunk cidx-1 fully replayed: its slot takes chunk cidx+2
      HIPCHK(hipEventRecord(I.sev_free, s));
      HIPCHK(hipStreamWaitEvent(I.sstream, I.sev_free, 0));
      if (!issue_static(cidx + 2, I.sstream)) return false;
    }
    if (sharded && A.ne) {
      if (!xgather(I, kXchgBytes, err)) return false;
      hipLaunchKernelGGL(k_window_gmerge, dim3(A.ne), dim3(64), 0, s, I.xrecv.p, I.xranks, I.xrows.p, A.pprev,
                         A.pprev_n, I.wrec.p + (size_t)(E & 1) * kRecBytes);
    }
  }
  if (nwin) {
    const int64_t L = nwin - 1;
    hipLaunchKernelGGL(k_apply_pend, dim3(1), dim3(KSG_BATCH), 0, s, C, I.pend.p + (size_t)(L & 1) * KSG_BATCH,
                       I.pend_n.p + (L & 1));
  }
  HIPCHK(hipEventRecord(I.ev1, s));
  HIPCHK(hipGetLastError());
  return true;
}

// The static record keeps the raw NodeAffinity score in 20 bits.
static int64_t na_weight_sum(const std::vector<uint8_t>& prog) {
  const ksg_prog* h = reinterpret_cast<const ksg_prog*>(prog.data());
  const int32_t* i32 = reinterpret_cast<const int32_t*>(prog.data() + h->off_i32);
  int64_t sum = 0;
  for (int t = 0; t < h->n_pref_terms; ++t) sum += i32[h->pref_w_off + t] > 0 ? i32[h->pref_w_off + t] : 0;
  return sum;
}
static bool na_weights_fit(const std::vector<uint8_t>& prog) { return na_weight_sum(prog) <= (int64_t)KSG_RAW_NA_MASK; }

static PodLite pod_lite(const std::vector<uint8_t>& prog) {
  const ksg_prog* h = reinterpret_cast<const ksg_prog*>(prog.data());
  PodLite q;
  for (int k = 0; k < 4; ++k) q.req[k] = h->req[k];
  for (int k = 0; k < KSG_MAX_SCORE_RES; ++k) {
    q.fit_score_req[k] = h->fit_score_req[k];
    q.ba_req[k] = h->ba_req[k];
  }
  q.nz_cpu = h->nz_cpu;
  q.nz_mem = h->nz_mem;
  q.queue_idx = h->queue_idx;
  q.flags = h->flags;
  return q;
}

// run_queue's per-pod decisions: bit0 PodTopologySpread constraints, bit1
// InterPodAffinity (existing pods' terms may apply to any pod), bit2 the table
// chain, bit3 its PodTopologySpread raw-score pass.
static uint32_t prog_need_of(const ksg_prog* h) {
  uint32_t need = 2;
  if (h->n_tsc_filter + h->n_tsc_score > 0) need |= 1;
  if (h->tab & KTAB_ON) need |= 4;
  if (h->tab & KTAB_PTS_MULTI) need |= 8;
  // bit 17: nothing but the node row and the class tables changes on its assume
  // (no host ports, volume claims or CSI volumes): a persistent segment may hold it
  if (h->n_port_own == 0 && h->n_pvc == 0 && h->n_csi == 0) need |= 1u << 17;
  // bit 18: the persistent chain's small size class (kRunLK lookups, kRunTS constraints)
  if (h->n_lk <= kRunLK && h->n_tsc_filter + h->n_tsc_score <= kRunTS) need |= 1u << 18;
  // bits 8..15: preferred NodeAffinity terms of the what-if class path (0xFF: a
  // negative weight or more than 7 terms — the record path)
  const int32_t* i32 = reinterpret_cast<const int32_t*>(reinterpret_cast<const uint8_t*>(h) + h->off_i32);
  uint32_t np = h->n_pref_terms > 7 ? 0xFFu : (uint32_t)h->n_pref_terms;
  for (int t = 0; t < h->n_pref_terms && np != 0xFFu; ++t)
    if (i32[h->pref_w_off + t] < 0) np = 0xFFu;
  // bit 16: cpu / memory requests in [0, 2^44) (the class path's doubles stay exact)
  bool small = true;
  for (int c = 0; c < 2; ++c)
    for (int64_t v : {h->req[c], h->fit_score_req[c], h->ba_req[c]}) small &= v >= 0 && v < ((int64_t)1 << 44);
  // bit 19: the class path's decoder flattens its NodeAffinity (wc_decodable)
  if (wc_decodable(h)) need |= 1u << 19;
  return need | np << 8 | (small ? 1u << 16 : 0u);
}

static bool exchange(Engine::Impl& I, const void* src, size_t bytes, std::string& err);

bool Engine::run_whatif(uint32_t first, uint32_t count, std::string& err) {
  Impl& I = *p_;
  if (first + count > I.prog_off.size()) { err = "program index out of range"; return false; }
  if (I.has_pts || I.has_ipa || !I.batch_ok) {
    // Profiles with cross-node state (PodTopologySpread / InterPodAffinity domain
    // counts, or plugins k_whatif does not evaluate): every pod of the step runs
    // its cycle without assume — the table chain reads the class tables, which
    // stay frozen for the whole step — then the step's placements are bound in
    // pod order (rows, host ports, class tables, existing-pod table rows).
    if (!run_queue(first, count, false, err)) return false;
    if (count) {
      const bool tables = I.has_pts || I.has_ipa;
      hipLaunchKernelGGL(k_whatif_bind_seq, dim3(1), dim3(64), 0, I.stream, I.cluster(), I.progs.p, I.prog_off_d.p,
                         I.sums.p, first, count, tables ? 1 : 0, I.prow.p);
      HIPCHK(hipEventRecord(I.ev1, I.stream));
      HIPCHK(hipGetLastError());
    }
    return true;
  }
  hipStream_t s = I.stream;
  DevCluster C = I.cluster();
  WiArgs A{};
  A.progs = I.progs.p;
  A.prog_off = I.prog_off_d.p;
  A.q0 = first;
  A.count = count;
  A.sums = I.sums.p;
  A.keep_first = I.keep_first;
  A.keep_n = I.keep_n;
  A.kfilter = I.kfilter.p;
  A.kscore = I.kscore.p;
  A.ktotal = I.ktotal.p;
  if (I.sample_every) {
    while (I.sev.size() < 4) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      I.sev.push_back(e);
    }
  }
  I.n_samples = 0;
  HIPCHK(hipEventRecord(I.ev0, s));
  if (count) {
    // Pass 1 leaves an 8-byte record per (pod, node) — feasibility, the Fit/BA
    // weighted sum, the raw Taint / NodeAffinity scores — so that pass 2 only
    // normalises and picks (the snapshot is frozen for the step).  Pods go in
    // chunks whose records fit KSG_WHATIF_REC_MB (default 40 GiB of the 288 GB;
    // 0: pass 2 recomputes every pair).
    const uint32_t N = std::max<uint32_t>(I.N, 1);
    size_t rec_mb = 40960;
    if (const char* e = std::getenv("KSG_WHATIF_REC_MB")) rec_mb = (size_t)std::strtoull(e, nullptr, 10);
    int64_t wsum = 0;
    for (int i = 0; i < I.F.n; ++i)
      if (I.F.plugins[i] == KP_FIT || I.F.plugins[i] == KP_BA) wsum += I.F.weight[i] > 0 ? I.F.weight[i] : 0;
    A.need_eph = I.any_eph_req ? 1u : 0u;
    // the class path (k_whatif_cls1/2): nothing per pair in memory; KSG_WHATIF_CLASSES=0 off
    // (the class key holds the Fit/BA sum in 24 bits: 100 x the weights below 2^24, none negative)
    bool wts_ok = true;
    for (int i = 0; i < I.F.n; ++i)
      if (I.F.plugins[i] == KP_FIT || I.F.plugins[i] == KP_BA) wts_ok &= I.F.weight[i] >= 0;
    bool use_cls = I.eval_mode == 1 && !I.any_eph_req && I.R <= 4 && I.static_fits && I.max_taints <= 4 &&
                   I.max_tid < 64 && !I.taint_dup && I.cols_small && rec_mb > 0 && wts_ok &&
                   100 * wsum < ((int64_t)1 << 24);
    if (const char* e = std::getenv("KSG_WHATIF_CLASSES")) use_cls &= std::strtol(e, nullptr, 10) != 0;
    for (uint32_t q = first; use_cls && q < first + count; ++q) {
      const uint32_t np = (I.prog_need[q] >> 8) & 0xFFu;
      use_cls = np <= 7 && ((I.max_taints + 1) << np) <= KSG_WC_CLS && (I.prog_need[q] & (1u << 16)) &&
                (I.prog_need[q] & (1u << 19));
    }
    const bool use_rec = !use_cls && rec_mb > 0 && I.R <= 4 && I.static_fits && 100 * wsum < (int64_t)1 << 30;
    // record fields as narrow as the cluster allows: 4-byte records when the raw
    // NodeAffinity (<= the programs' largest weight sum), raw Taint (<= most taints
    // on a node) and Fit/BA sum (<= 100 x their weights) fit 30 bits
    auto bits = [](uint64_t v) { uint32_t b = 0; while (v) { ++b; v >>= 1; } return b; };
    A.bw_a = bits((uint64_t)I.max_na_sum);
    A.bw_t = bits(I.max_taints);
    A.bw_tot = bits((uint64_t)(100 * wsum));
    {
      int64_t wall = 0;
      for (int i = 0; i < I.F.n; ++i) wall += I.F.weight[i] > 0 ? I.F.weight[i] : 0;
      A.small = 100 * wall < ((int64_t)1 << 31) && !std::getenv("KSG_WHATIF_WIDE") ? 1u : 0u;  // (WIDE: 64-bit path too)
    }
    const bool narrow = A.bw_a + A.bw_t + A.bw_tot <= 30 && !std::getenv("KSG_WHATIF_WIDE");
    if (!narrow) { A.bw_a = 20; A.bw_t = 12; A.bw_tot = 30; }
    const size_t rbytes = narrow ? 4 : 8;
    uint32_t chunk = count;
    if (use_rec) {
      const size_t per_pod = (size_t)N * rbytes;
      const size_t fit = (rec_mb << 20) / per_pod / KSG_WI_PODS * KSG_WI_PODS;
      chunk = (uint32_t)std::min<size_t>(count, std::max<size_t>(fit, KSG_WI_PODS));
      std::string aerr;  // no room: smaller chunks
      while (!I.wrec_pairs.alloc(((size_t)chunk * N * rbytes + 7) / 8, aerr) && chunk > KSG_WI_PODS) {
        (void)hipGetLastError();  // (the failed hipMalloc's error is not the run's)
        chunk = std::max<uint32_t>(chunk / 2 / KSG_WI_PODS * KSG_WI_PODS, KSG_WI_PODS);
      }
      if (((size_t)chunk * N * rbytes + 7) / 8 > I.wrec_pairs.n) { err = aerr; return false; }
    }
    const uint32_t tiles = std::max<uint32_t>((I.N + KSG_WC_TILE - 1) / KSG_WC_TILE, 1);
    // class path scratch per pod: tiles x (class row + count), folded row + flag
    const size_t wc_words = (size_t)tiles * KSG_WC_CLS + ((size_t)tiles + 1) / 2 + KSG_WC_CLS + 1;
    if (use_cls) {
      const size_t fit = (rec_mb << 20) / (wc_words * 8) / KSG_WC_PODS * KSG_WC_PODS;
      chunk = (uint32_t)std::min<size_t>(count, std::max<size_t>(fit, KSG_WC_PODS));
      if (!I.wrec_pairs.alloc((size_t)chunk * wc_words, err) ||
          !I.wc_pods.alloc((size_t)chunk * (sizeof(WcPod) / 8), err))
        return false;
    }
    const dim3 pods((count + 255) / 256);
    hipLaunchKernelGGL(k_init_summaries, pods, dim3(256), 0, s, I.sums.p + first, count, I.F);
    for (uint32_t c0 = 0; c0 < count; c0 += chunk) {
      WiArgs a = A;
      a.q0 = first + c0;
      a.count = std::min(chunk, count - c0);
      a.rec = use_rec ? (void*)I.wrec_pairs.p : nullptr;
      const dim3 grid(std::max<uint32_t>((I.N + 256 * KSG_WI_NPT - 1) / (256 * KSG_WI_NPT), 1),
                      (a.count + KSG_WI_PODS - 1) / KSG_WI_PODS);
      const dim3 grid1((a.count + KSG_WI_PODS - 1) / KSG_WI_PODS, std::max<uint32_t>((I.N + 255) / 256, 1));
      const dim3 grid2(std::max<uint32_t>((I.N + 256 * KSG_WI_R2NPT - 1) / (256 * KSG_WI_R2NPT), 1),
                       (a.count + KSG_WI_PODS - 1) / KSG_WI_PODS);
      const dim3 cpods((a.count + 255) / 256);
      const size_t xb = (size_t)a.count * sizeof(ksg_pod_summary);
      if (use_cls) {
        a.wc_part = I.wrec_pairs.p;
        a.wc_cls = a.wc_part + (size_t)a.count * tiles * KSG_WC_CLS;
        a.wc_cnt = reinterpret_cast<uint32_t*>(a.wc_cls + (size_t)a.count * KSG_WC_CLS);
        a.wc_flag = a.wc_cnt + (size_t)a.count * tiles;
      }
      const dim3 gridc((a.count + KSG_WC_PODS - 1) / KSG_WC_PODS, tiles);
      for (int pass = 1; pass <= 2; ++pass) {
        const bool sampled = I.sample_every != 0 && c0 == 0;
        if (sampled) HIPCHK(hipEventRecord(I.sev[2 * (pass - 1)], s));
        const bool kept_here = I.keep_n && I.keep_first < a.q0 + a.count && I.keep_first + I.keep_n > a.q0;
        if (pass == 1 && use_cls) {
          I.path_pods[3]++;
          WcPod* wp = reinterpret_cast<WcPod*>(I.wc_pods.p);
          hipLaunchKernelGGL(k_wc_decode, dim3((a.count + 63) / 64), dim3(64), 0, s, C, I.F, a, wp);
          if (I.wc_npt == 1) hipLaunchKernelGGL(k_whatif_cls1<1>, gridc, dim3(256), 0, s, C, I.F, a, wp);
          else if (I.wc_npt == 4) hipLaunchKernelGGL(k_whatif_cls1<4>, gridc, dim3(256), 0, s, C, I.F, a, wp);
          else hipLaunchKernelGGL(k_whatif_cls1<2>, gridc, dim3(256), 0, s, C, I.F, a, wp);
          hipLaunchKernelGGL(k_whatif_cls2, dim3(a.count), dim3(KSG_WC_CLS), 0, s, I.F, a, tiles, I.xranks > 1 ? 1 : 0);
        } else if (pass == 2 && use_cls) {
          if (I.xranks > 1) hipLaunchKernelGGL(k_whatif_cls2, dim3(a.count), dim3(KSG_WC_CLS), 0, s, I.F, a, tiles, 2);
          if (kept_here) hipLaunchKernelGGL(k_whatif<2>, grid, dim3(256), 0, s, C, I.F, a, a.progs, a.prog_off);
        } else if (pass == 1 && use_rec) {
          if (I.eval_mode == 1) {
            if (narrow) hipLaunchKernelGGL((k_whatif_rec1<uint32_t, 1>), grid1, dim3(256), 0, s, C, I.F, a, a.progs, a.prog_off);
            else hipLaunchKernelGGL((k_whatif_rec1<uint64_t, 1>), grid1, dim3(256), 0, s, C, I.F, a, a.progs, a.prog_off);
          } else {
            if (narrow) hipLaunchKernelGGL((k_whatif_rec1<uint32_t, 0>), grid1, dim3(256), 0, s, C, I.F, a, a.progs, a.prog_off);
            else hipLaunchKernelGGL((k_whatif_rec1<uint64_t, 0>), grid1, dim3(256), 0, s, C, I.F, a, a.progs, a.prog_off);
          }
        }
        else if (pass == 1) hipLaunchKernelGGL(k_whatif<1>, grid, dim3(256), 0, s, C, I.F, a, a.progs, a.prog_off);
        else if (use_rec) {
          if (narrow) hipLaunchKernelGGL(k_whatif_rec2<uint32_t>, grid2, dim3(256), 0, s, C, I.F, a, a.progs, a.prog_off);
          else hipLaunchKernelGGL(k_whatif_rec2<uint64_t>, grid2, dim3(256), 0, s, C, I.F, a, a.progs, a.prog_off);
          if (kept_here) hipLaunchKernelGGL(k_whatif<2>, grid, dim3(256), 0, s, C, I.F, a, a.progs, a.prog_off);
        } else hipLaunchKernelGGL(k_whatif<2>, grid, dim3(256), 0, s, C, I.F, a, a.progs, a.prog_off);
        if (sampled) {
          HIPCHK(hipEventRecord(I.sev[2 * (pass - 1) + 1], s));
          I.n_samples++;
        }
        if (I.xranks > 1) {  // per-pod partials of every shard -> global values on every rank
          if (!exchange(I, I.sums.p + a.q0, xb, err)) return false;
          hipLaunchKernelGGL(k_whatif_merge, cpods, dim3(256), 0, s,
                             reinterpret_cast<const ksg_pod_summary*>(I.xrecv.p), I.xranks, a.count, I.sums.p + a.q0,
                             pass);
        }
      }
    }
    I.wi_chunk = chunk;
    I.wi_rec = use_rec;
    I.wi_cls = use_cls;
    hipLaunchKernelGGL(k_whatif_select, pods, dim3(256), 0, s, A);
    hipLaunchKernelGGL(k_whatif_bind, pods, dim3(256), 0, s, C, A);
  }
  HIPCHK(hipEventRecord(I.ev1, s));
  HIPCHK(hipGetLastError());
  return true;
}

void Engine::release_scratch() {
  Impl& I = *p_;
  if (!I.wrec_pairs.p) return;
  (void)hipStreamSynchronize(I.stream);
  (void)hipFree(I.wrec_pairs.p);
  I.wrec_pairs.p = nullptr;
  I.wrec_pairs.n = 0;
}

// All-gather `bytes` from every rank into I.xrecv (rank order), on the engine stream.
static bool exchange(Engine::Impl& I, const void* src, size_t bytes, std::string& err) {
  hipStream_t s = I.stream;
  if (!I.xsend.grow(bytes, 0, s, err) || !I.xrecv.grow(bytes * I.xranks, 0, s, err)) return false;
  HIPCHK(hipMemcpyAsync(I.xsend.p, src, bytes, hipMemcpyDeviceToDevice, s));
  return xgather(I, bytes, err);
}
static void host_exchange(void* p);
// All-gather `bytes` from src (default I.xsend) into I.xrecv (rank order) on stream
// st (default the engine stream).
static bool xgather(Engine::Impl& I, size_t bytes, std::string& err, const uint8_t* src, hipStream_t st) {
  hipStream_t s = st ? st : I.stream;
  if (!src) src = I.xsend.p;
  if (I.xmode == 1) {
    ncclResult_t nr = ncclAllGather(src, I.xrecv.p, bytes, ncclUint8, I.comm, s);
    if (nr != ncclSuccess) { err = std::string("ncclAllGather: ") + ncclGetErrorString(nr); return false; }
    return true;
  }
  if (I.hps_n < bytes || I.hpr_n < bytes * I.xranks) {  // (rare: wait for every queued exchange first)
    HIPCHK(hipDeviceSynchronize());
    if (I.hps) (void)hipHostFree(I.hps);
    if (I.hpr) (void)hipHostFree(I.hpr);
    I.hps = I.hpr = nullptr;
    I.hps_n = I.hpr_n = 0;
    HIPCHK(hipHostMalloc((void**)&I.hps, bytes, hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void**)&I.hpr, bytes * I.xranks, hipHostMallocDefault));
    I.hps_n = bytes;
    I.hpr_n = bytes * I.xranks;
  }
  HIPCHK(hipMemcpyAsync(I.hps, src, bytes, hipMemcpyDeviceToHost, s));
  I.hcalls.push_back({&I, bytes});
  HIPCHK(hipLaunchHostFunc(s, host_exchange, &I.hcalls.back()));
  HIPCHK(hipMemcpyAsync(I.xrecv.p, I.hpr, bytes * I.xranks, hipMemcpyHostToDevice, s));
  return true;
}
static void host_exchange(void* p) {
  auto* c = static_cast<Engine::Impl::HostCall*>(p);
  Engine::Impl& I = *c->I;
  if (I.xfail.load()) return;
  if (I.xfn(I.xuser, I.hps, I.hpr, c->bytes) != 0) I.xfail.store(1);
}

// The host-side record of a program placed at byte offset off (append_program,
// add_classes' fused placement).
static void note_program(Engine::Impl& I, const std::vector<uint8_t>& prog, size_t off) {
  I.prog_bytes = off + prog.size();
  I.prog_off.push_back(off);
  if (!na_weights_fit(prog)) I.static_fits = false;
  I.max_na_sum = std::max(I.max_na_sum, na_weight_sum(prog));
  const ksg_prog* h = reinterpret_cast<const ksg_prog*>(prog.data());
  I.prog_need.push_back(prog_need_of(h));
  for (int c = 2; c < KSG_MAX_RES; ++c) I.any_eph_req |= h->req[c] != 0;
}
bool Engine::append_program(const std::vector<uint8_t>& prog, std::string& err) {
  Impl& I = *p_;
  hipStream_t s = I.stream;
  const size_t q = I.prog_off.size();
  const size_t off = (I.prog_bytes + 255) & ~(size_t)255;
  if (!I.progs.grow(off + prog.size(), I.prog_bytes, s, err) || !I.prog_off_d.grow(q + 1, q, s, err) ||
      !I.plite.grow(q + 1, q, s, err) || !I.sums.grow(q + 1, q, s, err) || !I.prow.grow(q + 1, q, s, err))
    return false;
  const uint64_t off64 = off;
  const PodLite pl = pod_lite(prog);
  // One pinned staging block [PodLite | program] -> one copy, and one kernel that
  // places it (program, offset, PodLite, table row, fresh summary): no wait here.
  // The block is reused once its previous copy has completed (an event).
  const size_t sbytes = kPlOff + prog.size();
  {  // (round 5) zero-copy: k_place_program reads a mapped pinned block, held until the next sync
    size_t cap = 0;
    uint8_t* blk = pinned_get(sbytes, cap);
    uint8_t* dv = blk ? pinned_dev(blk) : nullptr;
    if (dv) {
      std::memcpy(blk, &pl, sizeof(pl));
      std::memcpy(blk + kPlOff, prog.data(), prog.size());
      I.hold.push_back(std::shared_ptr<const void>(blk, [cap](const void* b) {
        Engine::pinned_put(const_cast<uint8_t*>(static_cast<const uint8_t*>(b)), cap);
      }));
      I.unwaited = true;
      hipLaunchKernelGGL(k_place_program, dim3(1), dim3(256), 0, s, dv, (uint32_t)prog.size(), I.progs.p + off,
                         I.prog_off_d.p + q, off64, (void*)(I.plite.p + q), I.prow.p + q, (int32_t)-1, I.sums.p + q,
                         I.F);
      HIPCHK(hipGetLastError());
      note_program(I, prog, off);
      return true;
    }
    if (blk) pinned_put(blk, cap);
  }
  if (!I.apstage || I.apstage_cap < sbytes) {
    if (I.apstage) {
      HIPCHK(hipEventSynchronize(I.apstage_ev));
      (void)hipHostFree(I.apstage);
      I.apstage = nullptr;
    }
    I.apstage_cap = std::max<size_t>(sbytes, 64 << 10);
    if (hipHostMalloc((void**)&I.apstage, I.apstage_cap, hipHostMallocDefault) != hipSuccess) {
      I.apstage = nullptr;
      I.apstage_cap = 0;
      err = "hipHostMalloc: program staging";
      return false;
    }
    if (!I.apstage_ev) HIPCHK(hipEventCreateWithFlags(&I.apstage_ev, hipEventDisableTiming));
  } else {
    HIPCHK(hipEventSynchronize(I.apstage_ev));  // (the previous append's copy: long done)
  }
  if (!I.apdev.grow(sbytes, 0, s, err)) return false;
  std::memcpy(I.apstage, &pl, sizeof(pl));
  std::memcpy(I.apstage + kPlOff, prog.data(), prog.size());
  HIPCHK(hipMemcpyAsync(I.apdev.p, I.apstage, sbytes, hipMemcpyHostToDevice, s));
  HIPCHK(hipEventRecord(I.apstage_ev, s));
  hipLaunchKernelGGL(k_place_program, dim3(1), dim3(256), 0, s, I.apdev.p, (uint32_t)prog.size(), I.progs.p + off,
                     I.prog_off_d.p + q, off64, (void*)(I.plite.p + q), I.prow.p + q, (int32_t)-1, I.sums.p + q, I.F);
  HIPCHK(hipGetLastError());
  note_program(I, prog, off);
  return true;
}

bool Engine::assume(uint32_t q, int32_t gnode, int sign, std::string& err, bool wait) {
  Impl& I = *p_;
  if (!tables_ready(I, err)) return false;
  if (q >= I.prog_off.size()) { err = "program index out of range"; return false; }
  DevCluster C = I.cluster();
  hipLaunchKernelGGL(k_assume, dim3(1), dim3(64), 0, I.stream, C, I.progs.p + I.prog_off[q], gnode, sign,
                     (I.has_pts || I.has_ipa) ? 1 : 0, I.prow.p + q);
  HIPCHK(hipGetLastError());
  if (wait) {
    if (!stream_sync(I, I.stream, err)) return false;
  } else {
    I.unwaited = true;
  }
  return true;
}

bool Engine::bound_deltas(const std::vector<std::vector<uint8_t>>& progs, const std::vector<int32_t>& gnode,
                          const std::vector<int32_t>& sign, const std::vector<int32_t>& slot, std::vector<int32_t>& rows,
                          std::string& err) {
  Impl& I = *p_;
  if (!tables_ready(I, err)) return false;
  const size_t n = progs.size();
  if (gnode.size() != n || sign.size() != n || slot.size() != n || rows.size() != n) { err = "bound_deltas: sizes"; return false; }
  if (!n) return true;
  std::vector<size_t> off(n);
  std::vector<uint8_t> blob;
  for (size_t i = 0; i < n; ++i) {
    if (progs[i].size() < sizeof(ksg_prog) || slot[i] < 0 || (size_t)slot[i] >= n) { err = "bound_deltas: program/slot"; return false; }
    off[i] = (blob.size() + 255) & ~(size_t)255;
    blob.resize(off[i]);
    blob.insert(blob.end(), progs[i].begin(), progs[i].end());
  }
  if (!I.evprog.alloc(blob.size(), err) || !I.evrow.alloc(n, err)) return false;
  HIPCHK(hipMemcpyAsync(I.evprog.p, blob.data(), blob.size(), hipMemcpyHostToDevice, I.stream));
  HIPCHK(hipMemcpyAsync(I.evrow.p, rows.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, I.stream));
  DevCluster C = I.cluster();
  const int table = (I.has_pts || I.has_ipa) ? 1 : 0;
  for (size_t i = 0; i < n; ++i)  // stream order: a removal sees the row its same-batch addition wrote
    hipLaunchKernelGGL(k_assume, dim3(1), dim3(64), 0, I.stream, C, I.evprog.p + off[i], gnode[i], sign[i], table,
                       I.evrow.p + slot[i]);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(rows.data(), I.evrow.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

bool Engine::toggle_pods(const std::vector<const std::vector<uint8_t>*>& progs, const std::vector<int32_t>& gnode,
                         const std::vector<int32_t>& rows, int sign, std::string& err) {
  Impl& I = *p_;
  if (!tables_ready(I, err)) return false;
  const size_t n = progs.size();
  if (gnode.size() != n || rows.size() != n) { err = "toggle_pods: sizes"; return false; }
  if (!n) return true;
  std::vector<size_t> off(n);
  std::vector<uint8_t> blob;
  for (size_t i = 0; i < n; ++i) {
    if (!progs[i] || progs[i]->size() < sizeof(ksg_prog)) { err = "toggle_pods: program"; return false; }
    off[i] = (blob.size() + 255) & ~(size_t)255;
    blob.resize(off[i]);
    blob.insert(blob.end(), progs[i]->begin(), progs[i]->end());
  }
  if (!I.evprog.alloc(blob.size(), err) || !I.evrow.alloc(n, err)) return false;
  HIPCHK(hipMemcpyAsync(I.evprog.p, blob.data(), blob.size(), hipMemcpyHostToDevice, I.stream));
  HIPCHK(hipMemcpyAsync(I.evrow.p, rows.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, I.stream));
  DevCluster C = I.cluster();
  for (size_t i = 0; i < n; ++i)
    hipLaunchKernelGGL(k_assume, dim3(1), dim3(64), 0, I.stream, C, I.evprog.p + off[i], gnode[i], sign, 2,
                       I.evrow.p + i);
  HIPCHK(hipGetLastError());
  if (!stream_sync(I, I.stream, err)) return false;  // (the host buffers are reused by the next toggle)
  return true;
}

static bool stage_entries(Engine::Impl& I, const std::vector<int32_t>& gnode, const std::vector<int32_t>& rows,
                          std::string& err);
bool Engine::toggle_stage(const std::vector<const std::vector<uint8_t>*>& progs, const std::vector<int32_t>& gnode,
                          const std::vector<int32_t>& rows, std::string& err) {
  Impl& I = *p_;
  if (!tables_ready(I, err)) return false;
  const size_t n = progs.size();
  if (gnode.size() != n || rows.size() != n) { err = "toggle_stage: sizes"; return false; }
  std::vector<uint64_t> off(n);
  I.tg_csi.assign(n, 0);
  size_t bytes = 0;
  for (size_t i = 0; i < n; ++i) {
    if (!progs[i] || progs[i]->size() < sizeof(ksg_prog)) { err = "toggle_stage: program"; return false; }
    off[i] = bytes;
    bytes = (bytes + progs[i]->size() + 255) & ~(size_t)255;
    I.tg_csi[i] = reinterpret_cast<const ksg_prog*>(progs[i]->data())->n_csi > 0 ? 1 : 0;
  }
  std::vector<uint8_t> blob(std::max<size_t>(bytes, 1));
  for (size_t i = 0; i < n; ++i) std::memcpy(blob.data() + off[i], progs[i]->data(), progs[i]->size());
  if (!I.tgprog.alloc(blob.size(), err)) return false;
  I.tg_addr.resize(n);
  for (size_t i = 0; i < n; ++i) I.tg_addr[i] = reinterpret_cast<uint64_t>(I.tgprog.p) + off[i];
  HIPCHK(hipMemcpyAsync(I.tgprog.p, blob.data(), blob.size(), hipMemcpyHostToDevice, I.stream));
  return stage_entries(I, gnode, rows, err);  // (syncs: the host blob goes out of scope)
}
// the staged entries' addresses, nodes and rows (I.tg_addr / tg_csi set by the caller)
static bool stage_entries(Engine::Impl& I, const std::vector<int32_t>& gnode, const std::vector<int32_t>& rows,
                          std::string& err) {
  const size_t n = gnode.size();
  if (!I.tgaddr.alloc(n, err) || !I.tgnode.alloc(n, err) || !I.tgrow.alloc(n, err)) return false;
  hipStream_t s = I.stream;
  if (n) {
    HIPCHK(hipMemcpyAsync(I.tgaddr.p, I.tg_addr.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(I.tgnode.p, gnode.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(I.tgrow.p, rows.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, s));
  }
  if (!stream_sync(I, s, err)) return false;
  I.tg_gnode = gnode;
  I.tg_n = (uint32_t)n;
  return true;
}
bool Engine::victim_store(const std::vector<const std::vector<uint8_t>*>& progs, std::string& err) {
  Impl& I = *p_;
  if (!tables_ready(I, err)) return false;
  const size_t n = progs.size();
  I.vstore_off.assign(n, 0);
  I.vstore_csi.assign(n, 0);
  size_t bytes = 0;
  for (size_t i = 0; i < n; ++i) {
    if (!progs[i] || progs[i]->size() < sizeof(ksg_prog)) { err = "victim_store: program"; return false; }
    I.vstore_off[i] = bytes;
    bytes = (bytes + progs[i]->size() + 15) & ~(size_t)15;
    I.vstore_csi[i] = reinterpret_cast<const ksg_prog*>(progs[i]->data())->n_csi > 0 ? 1 : 0;
  }
  // one pinned staging block, kept (a pageable blob paid its page faults and a
  // staged copy: 176 ms for 250,000 programs at cfg4 scale; round 6)
  bytes = std::max<size_t>(bytes, 1);
  if (I.vstage_cap < bytes) {
    if (I.vstage) (void)hipHostFree(I.vstage);
    I.vstage = nullptr;
    I.vstage_cap = 0;
    HIPCHK(hipHostMalloc((void**)&I.vstage, bytes + bytes / 4, hipHostMallocDefault));
    I.vstage_cap = bytes + bytes / 4;
  }
  for (size_t i = 0; i < n; ++i) std::memcpy(I.vstage + I.vstore_off[i], progs[i]->data(), progs[i]->size());
  if (!I.vstore.alloc(bytes, err)) return false;
  HIPCHK(hipMemcpyAsync(I.vstore.p, I.vstage, bytes, hipMemcpyHostToDevice, I.stream));
  return stream_sync(I, I.stream, err);
}
bool Engine::toggle_stage_refs(const std::vector<int64_t>& ref, const std::vector<int32_t>& gnode,
                               const std::vector<int32_t>& rows, const std::vector<uint8_t>& queue_csi, std::string& err) {
  Impl& I = *p_;
  if (!tables_ready(I, err)) return false;
  const size_t n = ref.size();
  if (gnode.size() != n || rows.size() != n) { err = "toggle_stage_refs: sizes"; return false; }
  I.tg_addr.resize(n);
  I.tg_csi.assign(n, 0);
  for (size_t i = 0; i < n; ++i) {
    const int64_t r = ref[i];
    if (r >= 0) {
      if ((size_t)r >= I.vstore_off.size()) { err = "toggle_stage_refs: bound pod outside the victim store"; return false; }
      I.tg_addr[i] = reinterpret_cast<uint64_t>(I.vstore.p) + I.vstore_off[(size_t)r];
      I.tg_csi[i] = I.vstore_csi[(size_t)r];
    } else {
      const size_t q = (size_t)(-1 - r);
      if (q >= I.prog_off.size() || q >= queue_csi.size()) { err = "toggle_stage_refs: queue pod"; return false; }
      I.tg_addr[i] = reinterpret_cast<uint64_t>(I.progs.p) + I.prog_off[q];
      I.tg_csi[i] = queue_csi[q];
    }
  }
  return stage_entries(I, gnode, rows, err);
}
bool Engine::toggle_staged(const std::vector<uint32_t>& idx, int sign, std::string& err) {
  Impl& I = *p_;
  if (sign != 1 && sign != -1) { err = "toggle_staged: sign"; return false; }
  if (idx.empty()) return true;
  std::vector<uint32_t> sorted;  // grouped by node (stable: a node's entries keep their order)
  sorted.reserve(idx.size());
  std::vector<uint32_t> serial;  // entries with CSI volumes: one launch each
  bool in_order = true;  // (the search's lists come node by node: no sort)
  for (uint32_t e : idx) {
    if (e >= I.tg_n) { err = "toggle_staged: index"; return false; }
    if (I.tg_csi[e]) {
      serial.push_back(e);
      continue;
    }
    in_order &= sorted.empty() || I.tg_gnode[sorted.back()] <= I.tg_gnode[e];
    sorted.push_back(e);
  }
  if (!in_order)
    std::stable_sort(sorted.begin(), sorted.end(),
                     [&](uint32_t a, uint32_t b) { return I.tg_gnode[a] < I.tg_gnode[b]; });
  std::vector<uint32_t> gs;
  for (size_t j = 0; j < sorted.size(); ++j)
    if (j == 0 || I.tg_gnode[sorted[j]] != I.tg_gnode[sorted[j - 1]]) gs.push_back((uint32_t)j);
  gs.push_back((uint32_t)sorted.size());
  const uint32_t ng = (uint32_t)gs.size() - 1;
  std::vector<uint32_t> up(sorted);
  up.insert(up.end(), gs.begin(), gs.end());
  if (!I.tgidx.alloc(up.size(), err)) return false;
  hipStream_t s = I.stream;
  HIPCHK(hipMemcpyAsync(I.tgidx.p, up.data(), up.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  DevCluster C = I.cluster();
  if (ng)
    hipLaunchKernelGGL(k_toggle_groups, dim3((ng + 255) / 256), dim3(256), 0, s, C, I.tgaddr.p, I.tgnode.p, I.tgrow.p,
                       I.tgidx.p, I.tgidx.p + sorted.size(), ng, sign);
  for (uint32_t e : serial)
    hipLaunchKernelGGL(k_assume, dim3(1), dim3(64), 0, s, C, reinterpret_cast<const uint8_t*>(I.tg_addr[e]), I.tg_gnode[e],
                       sign, 2, I.tgrow.p + e);
  HIPCHK(hipGetLastError());
  if (!stream_sync(I, s, err)) return false;  // (the host index list goes out of scope)
  return true;
}

bool Engine::dry_filter(uint32_t q, int32_t gnode, std::vector<uint32_t>& codes, std::string& err) {
  Impl& I = *p_;
  if (q >= I.prog_off.size()) { err = "program index out of range"; return false; }
  if (gnode >= 0 && ((uint32_t)gnode < I.goff || (uint32_t)gnode - I.goff >= I.N)) { err = "dry_filter: node"; return false; }
  if (!I.drysum.alloc(1, err)) return false;
  HIPCHK(hipMemcpyAsync(I.drysum.p, I.sums.p + q, sizeof(ksg_pod_summary), hipMemcpyDeviceToDevice, I.stream));
  const uint32_t kf = I.keep_first, kn = I.keep_n;
  I.keep_n = 0;  // outputs to the scratch rows: kept outputs stay as they are
  const bool ok = run_queue(q, 1, false, err);
  I.keep_first = kf;
  I.keep_n = kn;
  if (!ok) return false;
  codes.resize(gnode >= 0 ? 1 : I.N);
  HIPCHK(hipMemcpyAsync(codes.data(), I.filter.p + (gnode >= 0 ? (uint32_t)gnode - I.goff : 0),
                        codes.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, I.stream));
  HIPCHK(hipMemcpyAsync(I.sums.p + q, I.drysum.p, sizeof(ksg_pod_summary), hipMemcpyDeviceToDevice, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

bool Engine::pod_row(uint32_t q, int32_t& row, std::string& err) {
  Impl& I = *p_;
  if (q >= I.prog_off.size()) { err = "program index out of range"; return false; }
  HIPCHK(hipMemcpyAsync(&row, I.prow.p + q, sizeof(int32_t), hipMemcpyDeviceToHost, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

bool Engine::node_alloc(int32_t gnode, const std::vector<int64_t>& alloc, int32_t allowed, std::string& err) {
  Impl& I = *p_;
  if (gnode < 0 || (uint32_t)gnode < I.goff || (uint32_t)gnode - I.goff >= I.N) return true;  // another shard's node
  if (alloc.size() != I.R) { err = "node_alloc: resource count"; return false; }
  const uint32_t n = (uint32_t)gnode - I.goff;
  for (uint32_t r = 0; r < I.R; ++r)
    HIPCHK(hipMemcpyAsync(I.alloc.p + (size_t)r * I.N + n, &alloc[r], sizeof(int64_t), hipMemcpyHostToDevice, I.stream));
  HIPCHK(hipMemcpyAsync(I.allowed.p + n, &allowed, sizeof(int32_t), hipMemcpyHostToDevice, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

bool Engine::node_static(const std::vector<int32_t>& gnodes, const std::vector<int32_t>& label_vid,
                         const std::vector<uint8_t>& has_labels, const std::vector<uint8_t>& flags, std::string& err) {
  Impl& I = *p_;
  const size_t m = gnodes.size();
  if (label_vid.size() != m * I.K || has_labels.size() != m || flags.size() != m) { err = "node_static: sizes"; return false; }
  for (int32_t g : gnodes)
    if (g < 0 || (uint32_t)g >= I.G) { err = "node_static: node index"; return false; }
  hipStream_t s = I.stream;
  // per node, one column entry per key: a strided copy down the [K][N] (and [K][G])
  // columns; every copy of the batch queued, one synchronisation (the host
  // vectors stay alive until it)
  for (size_t i = 0; i < m; ++i) {
    const uint32_t g = (uint32_t)gnodes[i];
    const int32_t* lv = label_vid.data() + i * I.K;
    if (I.K && I.gstat)
      HIPCHK(hipMemcpy2DAsync(I.glabel.p + g, (size_t)I.G * 4, lv, 4, 4, I.K, hipMemcpyHostToDevice, s));
    if (g >= I.goff && g - I.goff < I.N) {
      const uint32_t n = g - I.goff;
      if (I.K) HIPCHK(hipMemcpy2DAsync(I.label.p + n, (size_t)I.N * 4, lv, 4, 4, I.K, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(I.haslab.p + n, &has_labels[i], 1, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(I.nflags.p + n, &flags[i], 1, hipMemcpyHostToDevice, s));
    }
  }
  return stream_sync(I, s, err);
}

bool Engine::node_taints(const std::vector<uint32_t>& offs, const std::vector<int32_t>& ids,
                         const std::vector<uint32_t>& gofs, const std::vector<int32_t>& gids, std::string& err) {
  Impl& I = *p_;
  hipStream_t s = I.stream;
  if (offs.size() != (size_t)I.N + 1 || offs.back() != ids.size() ||
      (I.gstat && (gofs.size() != (size_t)I.G + 1 || gofs.back() != gids.size()))) {
    err = "node_taints: taint lists do not match the node count";
    return false;
  }
  if (!stream_sync(I, s, err)) return false;  // (a re-allocation frees what a queued launch may read)
  // what upload() derives from the lists: widest list, largest id, a taint listed twice
  uint32_t mt = 0;
  int32_t mx = -1;
  bool dup = false;
  for (uint32_t i = 0; i < I.N; ++i) mt = std::max(mt, offs[i + 1] - offs[i]);
  for (int32_t t : ids) mx = std::max(mx, t);
  for (uint32_t i = 0; i < I.N && !dup && mx < 64; ++i) {
    uint64_t seen = 0;
    for (uint32_t k = offs[i]; k < offs[i + 1]; ++k) {
      const uint64_t b = 1ull << (ids[k] & 63);
      dup |= (seen & b) != 0;
      seen |= b;
    }
  }
  if (I.gstat) {
    for (uint32_t g = 0; g < I.G; ++g) mt = std::max(mt, gofs[g + 1] - gofs[g]);
    std::vector<int32_t> gt = gids;
    gt.resize(std::max<size_t>(gt.size(), 1), 0);
    if (!I.gtoff.upload(gofs, s, err) || !I.gtid.upload(gt, s, err)) return false;
  }
  if (!I.toff.upload(offs, s, err) || !I.tid.upload(ids, s, err)) return false;
  I.max_taints = mt;
  I.max_tid = mx;
  I.taint_dup = dup;
  if (mt >= 4096) I.static_fits = false;  // (other causes may hold it false: never raised here)
  if (!stream_sync(I, s, err)) return false;
  return true;
}

bool Engine::grow_table(uint32_t pod_cap, uint32_t term_cap, uint32_t req_cap, uint32_t val_cap, uint32_t n_keys,
                        std::string& err) {
  Impl& I = *p_;
  hipStream_t s = I.stream;
  pod_cap = std::max(pod_cap, I.pcap);
  term_cap = std::max(term_cap, I.tcap);
  req_cap = std::max(req_cap, I.rcap);
  val_cap = std::max(val_cap, I.vcap);
  n_keys = std::max(n_keys, I.pkeys);
  if (!stream_sync(I, s, err)) return false;
  if (pod_cap != I.pcap || n_keys != I.pkeys) {
    if (!I.ptnode.grow(pod_cap, I.pcap, s, err) || !I.ptns.grow(pod_cap, I.pcap, s, err) ||
        !I.ptflags.grow(pod_cap, I.pcap, s, err))
      return false;
    // label columns [key][row]: re-laid at the new row stride; new keys' columns -1 (no label)
    DBuf<int32_t> lab;
    if (!lab.alloc((size_t)pod_cap * std::max<uint32_t>(n_keys, 1), err)) return false;
    HIPCHK(hipMemsetAsync(lab.p, 0xFF, (size_t)pod_cap * std::max<uint32_t>(n_keys, 1) * 4, s));
    for (uint32_t k = 0; k < I.pkeys; ++k)
      HIPCHK(hipMemcpyAsync(lab.p + (size_t)k * pod_cap, I.ptlab.p + (size_t)k * I.pcap, (size_t)I.pcap * 4,
                            hipMemcpyDeviceToDevice, s));
    if (!stream_sync(I, s, err)) return false;
    std::swap(lab.p, I.ptlab.p);
    std::swap(lab.n, I.ptlab.n);
  }
  if (!I.terms.grow(term_cap, I.tcap, s, err) || !I.tpod.grow(term_cap, I.tcap, s, err) ||
      !I.treq.grow(req_cap, I.rcap, s, err) || !I.tval.grow(val_cap, I.vcap, s, err))
    return false;
  I.pcap = pod_cap;
  I.tcap = term_cap;
  I.rcap = req_cap;
  I.vcap = val_cap;
  I.pkeys = n_keys;
  if (!stream_sync(I, s, err)) return false;
  return true;
}

bool Engine::table_overflow(bool& overflow, std::string& err) {
  Impl& I = *p_;
  uint32_t f = 0;
  overflow = false;
  if (!I.tcounts.p) return true;
  HIPCHK(hipMemcpyAsync(&f, I.tcounts.p + 4, sizeof(f), hipMemcpyDeviceToHost, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  overflow = f != 0;
  return true;
}

bool Engine::table_room(uint32_t used[4], uint32_t cap[4], std::string& err) {
  Impl& I = *p_;
  for (int i = 0; i < 4; ++i) used[i] = 0;
  cap[0] = I.pcap; cap[1] = I.tcap; cap[2] = I.rcap; cap[3] = I.vcap;
  if (!I.tcounts.p) return true;
  HIPCHK(hipMemcpyAsync(used, I.tcounts.p, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

uint32_t Engine::pod_classes() const { return p_->npc; }
uint32_t Engine::term_classes() const { return p_->ntc; }

// Append a device array's new elements (capacity doubling, old contents kept).
template <class T>
static bool dev_append(DBuf<T>& b, size_t used, const std::vector<T>& v, hipStream_t s, std::string& err) {
  if (v.empty()) return true;
  if (!b.grow(used + v.size(), used, s, err)) return false;
  HIPCHK(hipMemcpyAsync(b.p + used, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
  return true;
}
template <class T>
static bool dev_zero_tail(DBuf<T>& b, size_t used, size_t count, hipStream_t s, std::string& err) {
  if (!count) return true;
  if (!b.grow(used + count, used, s, err)) return false;
  HIPCHK(hipMemsetAsync(b.p + used, 0, count * sizeof(T), s));
  return true;
}

// add_classes' uploads in one launch (unsharded drop-in cycles): segment b of
// the list copies `words` 32-bit words from mapped pinned host memory (src), or
// zeroes them (src 0), into device memory; the list itself sits in the same
// pinned block.  One launch instead of a copy or fill per array.
struct UpSeg {
  uint64_t dst, src;
  uint32_t words, pad;
};
__device__ __forceinline__ void copy_seg(const UpSeg g) {
  uint32_t* d = reinterpret_cast<uint32_t*>(g.dst);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(g.src);
  uint32_t w0 = 0;
  if (((g.dst | g.src) & 15) == 0) {  // 16-byte pieces (a source in host memory: fewer link reads)
    w0 = g.words & ~3u;
    uint4* d4 = reinterpret_cast<uint4*>(d);
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    for (uint32_t i = blockIdx.y * 256 + threadIdx.x; i < w0 / 4; i += gridDim.y * 256)
      d4[i] = src ? s4[i] : make_uint4(0, 0, 0, 0);
  }
  for (uint32_t i = w0 + blockIdx.y * 256 + threadIdx.x; i < g.words; i += gridDim.y * 256) d[i] = src ? src[i] : 0u;
}
__global__ __launch_bounds__(256) void k_upload(const UpSeg* __restrict__ segs) { copy_seg(segs[blockIdx.x]); }
// Engine::reset's restores of the snapshot's node columns in one launch (the
// segments travel as kernel arguments: one block row per segment)
constexpr int kRestoreSegs = 12;
struct RestoreSegs {
  UpSeg seg[kRestoreSegs];
};
__global__ __launch_bounds__(256) void k_restore(const RestoreSegs S) { copy_seg(S.seg[blockIdx.x]); }

// Node-sharded class tables: sum the pair-level entries of the classes built
// since the last call across ranks (each rank built them from its own existing
// pods), in one all-gather on the engine stream.  Without the exchange yet it
// stays pending: runs and in-place deltas call it first (tables_ready).
static bool reduce_tables(Engine::Impl& I, std::string& err) {
  if (I.shards <= 1 || (I.red_pc0 == UINT32_MAX && I.red_tc0 == UINT32_MAX)) return true;
  if (I.xranks != I.shards) return true;
  std::vector<TabSeg> sg;
  uint32_t total = 0;
  auto seg = [&](int32_t* p, size_t len) {
    if (!len) return;
    sg.push_back(TabSeg{p, (uint32_t)len, total});
    total += (uint32_t)len;
  };
  if (I.red_pc0 < I.npc) {
    const size_t c0 = I.red_pc0, nc = I.npc - c0;
    if (I.NU) seg(I.pc_dom.p + c0 * I.NU, nc * I.NU);
    seg(I.pc_tot.p + c0 * KSG_MAX_TOPO, nc * KSG_MAX_TOPO);
  }
  if (I.red_tc0 < I.ntc) {
    seg(I.tc_tot.p + I.red_tc0, I.ntc - I.red_tc0);
    for (uint32_t u = I.red_tc0; u < I.ntc; ++u) {
      const int32_t sl = I.tc_slot_h[u];
      if (!((I.uniq >> sl) & 1u)) seg(I.tc_val.p + I.tc_off_h[u], I.topo.topo_count[sl]);
    }
  }
  I.red_pc0 = I.red_tc0 = UINT32_MAX;
  if (!total) return true;
  hipStream_t s = I.stream;
  if (!I.segs_d.upload(sg, s, err)) return false;
  const size_t bytes = (size_t)total * 4;
  if (!I.xsend.grow(bytes, 0, s, err) || !I.xrecv.grow(bytes * I.xranks, 0, s, err)) return false;
  const uint32_t nseg = (uint32_t)sg.size(), nb = std::min<uint32_t>(nseg, 1024);
  hipLaunchKernelGGL(k_seg_pack, dim3(nb), dim3(256), 0, s, I.segs_d.p, nseg, reinterpret_cast<int32_t*>(I.xsend.p));
  if (!xgather(I, bytes, err)) return false;
  hipLaunchKernelGGL(k_seg_sum, dim3(nb), dim3(256), 0, s, I.segs_d.p, nseg, reinterpret_cast<const int32_t*>(I.xrecv.p),
                     total, I.xranks);
  HIPCHK(hipGetLastError());
  if (!stream_sync(I, s, err)) return false;  // (segment list uploaded from a host vector)
  return true;
}
// Before anything reads or changes the class tables of a sharded context.
static bool tables_ready(Engine::Impl& I, std::string& err) {
  if (I.shards <= 1 || (I.red_pc0 == UINT32_MAX && I.red_tc0 == UINT32_MAX)) return true;
  if (I.xranks != I.shards) { err = "sharded context: call ksg_set_exchange before scheduling"; return false; }
  return reduce_tables(I, err);
}

bool Engine::add_classes(const ClassUpload& u, std::string& err, const std::vector<uint8_t>* prog, bool* placed) {
  Impl& I = *p_;
  if (placed) *placed = false;
  hipStream_t s = I.stream;
  const uint32_t pc0 = I.npc, tc0 = I.ntc, npc = (uint32_t)u.pc.size(), ntc = (uint32_t)u.tc_slot.size();
  if (!npc && !ntc) return true;
  const size_t Nn = std::max<uint32_t>(I.N, 1), NUn = std::max<uint32_t>(I.NU, 1);
  // (unsharded, the upload is not waited for: its host sources are held until the
  // engine stream's next sync, and a late failure marks the context lost; the
  // copies and zero tails go out as ONE k_upload from a mapped pinned block)
  std::vector<UpSeg> segs;
  std::vector<uint8_t> pay;  // payloads, 16-byte aligned (offsets into the block after the list)
  const bool fused = I.shards <= 1;
  auto up = [&](auto& buf, size_t used, const auto& v) -> bool {  // dev_append
    if (v.empty()) return true;
    if (!fused) return dev_append(buf, used, v, s, err);
    if (!buf.grow(used + v.size(), used, s, err)) return false;
    const size_t o = (pay.size() + 15) & ~(size_t)15, b = v.size() * sizeof(v[0]);
    pay.resize(o + b);
    std::memcpy(pay.data() + o, v.data(), b);
    segs.push_back(UpSeg{reinterpret_cast<uint64_t>(buf.p + used), o + 1, (uint32_t)(b / 4), 0});  // (src: offset + 1)
    return true;
  };
  auto zero = [&](auto& buf, size_t used, size_t count) -> bool {  // dev_zero_tail
    if (!count) return true;
    if (!fused) return dev_zero_tail(buf, used, count, s, err);
    if (!buf.grow(used + count, used, s, err)) return false;
    segs.push_back(UpSeg{reinterpret_cast<uint64_t>(buf.p + used), 0, (uint32_t)(count * sizeof(buf.p[0]) / 4), 0});
    return true;
  };
  auto held = [&](auto v) {
    auto p = std::make_shared<decltype(v)>(std::move(v));
    I.hold.push_back(p);
    return p;
  };
  PcStage pst{I.nct, 0, I.ncreq, 0, I.ncval, 0, 0xFFFFFFFFu, {}, 0, {}, {}};  // (k_pc_build: the new classes' pool ranges)
  if (I.pc_agg)  // slots with at most 256 domains: pc_dom counted per block
    for (uint32_t sl = 0; sl < KSG_MAX_TOPO && sl < I.topo.topo_count.size() && sl < I.topo.nu_base.size(); ++sl) {
      const uint32_t cnt = ((I.uniq >> sl) & 1u) ? I.N : I.topo.topo_count[sl];
      if (I.topo.nu_base[sl] == 0xFFFFFFFFu || cnt == 0 || cnt > 256) continue;
      pst.hbase[sl] = (uint16_t)pst.hsum;
      pst.hcnt[sl] = (uint16_t)cnt;
      pst.hsum += cnt;
    }
  if (npc) {  // definitions, rebased onto the device pools
    auto pc = held(u.pc);
    auto ct = held(u.ct);
    auto rq = held(u.creq);
    auto cv = held(u.cval);
    for (auto& x : *pc) x.term_off += (int32_t)I.nct;
    for (auto& x : *ct) {
      x.sel.req_off += (int32_t)I.ncreq;
      x.ns_off += (int32_t)I.ncval;
    }
    pst.nk = 0;  // (k_pc_build: the distinct requirement keys, read per row up front)
    for (auto& x : *rq) {
      x.val_off += (int32_t)I.ncval;
      uint32_t j = 0;
      while (j < pst.nk && j < KSG_PCB_K && pst.key[j] != x.key) ++j;
      if (j == pst.nk) {
        if (pst.nk < KSG_PCB_K) pst.key[j] = x.key;
        ++pst.nk;
      }
    }
    if (!I.pc_prefetch) pst.nk = 0xFFFFFFFFu;
    if (!up(I.pcls_d, pc0, *pc) || !up(I.cterm_d, I.nct, *ct) || !up(I.creq_d, I.ncreq, *rq) ||
        !up(I.cval_d, I.ncval, *cv) || !zero(I.pc_cnt, (size_t)pc0 * Nn, (size_t)npc * Nn) ||
        !zero(I.pc_dom, (size_t)pc0 * NUn, (size_t)npc * NUn) ||
        !zero(I.pc_tot, (size_t)pc0 * KSG_MAX_TOPO, (size_t)npc * KSG_MAX_TOPO))
      return false;
    I.nct += (uint32_t)ct->size();
    I.ncreq += (uint32_t)rq->size();
    I.ncval += (uint32_t)cv->size();
    pst.nt = (uint32_t)ct->size();
    pst.nr = (uint32_t)rq->size();
    pst.nv = (uint32_t)cv->size();
    I.npc += npc;
  }
  if (ntc) {  // per term class: one value per (key, value) pair, or per node for one-node keys
    const std::vector<uint32_t>& off = *held(u.tc_off);
    const std::vector<int32_t>& tslot = *held(u.tc_slot);
    if (off.size() != ntc) { err = "term classes without offsets"; return false; }
    uint32_t end = I.tc_used;
    for (uint32_t i = 0; i < ntc; ++i) {
      const int32_t sl = u.tc_slot[i];
      if (sl < 0 || sl >= (int32_t)I.topo.topo_count.size()) { err = "term class without a topology slot"; return false; }
      const uint32_t len = std::max<uint32_t>(((I.uniq >> sl) & 1u) ? I.N : I.topo.topo_count[sl], 1);
      if (off[i] != end) { err = "term class offsets out of sequence"; return false; }
      end = off[i] + len;
    }
    const uint32_t add = end - I.tc_used;
    if (!zero(I.tc_val, I.tc_used, add) || !up(I.tc_off_d, tc0, off) || !up(I.tc_slot_d, tc0, tslot) ||
        !zero(I.tc_tot, tc0, ntc))
      return false;
    I.tc_used += add;
    I.tc_off_h.insert(I.tc_off_h.end(), off.begin(), off.end());
    I.tc_slot_h.insert(I.tc_slot_h.end(), u.tc_slot.begin(), u.tc_slot.end());
    I.ntc += ntc;
  }
  // the cycle's program in the same upload (what k_place_program writes: program,
  // offset, PodLite, table row, fresh summary), so a pod that brings classes costs
  // one copy kernel, not two
  if (prog && placed && fused && I.place_fused && !segs.empty() && prog->size() % 4 == 0) {
    const size_t q = I.prog_off.size();
    const size_t off = (I.prog_bytes + 255) & ~(size_t)255;
    if (!I.progs.grow(off + prog->size(), I.prog_bytes, s, err) || !I.prog_off_d.grow(q + 1, q, s, err) ||
        !I.plite.grow(q + 1, q, s, err) || !I.sums.grow(q + 1, q, s, err) || !I.prow.grow(q + 1, q, s, err))
      return false;
    auto put = [&](void* dst, const void* src, size_t b) {
      const size_t o = (pay.size() + 15) & ~(size_t)15;
      pay.resize(o + b);
      std::memcpy(pay.data() + o, src, b);
      segs.push_back(UpSeg{reinterpret_cast<uint64_t>(dst), o + 1, (uint32_t)(b / 4), 0});
    };
    const PodLite pl = pod_lite(*prog);
    const uint64_t off64 = off;
    const int32_t row = -1;
    ksg_pod_summary z = {};
    z.selected = -1;
    for (int p = 0; p < KSG_MAX_PLUGINS; ++p) {
      z.max_score[p] = (p < I.F.n && I.F.plugins[p] == KP_IPA) ? INT64_MIN : 0;
      z.min_score[p] = INT64_MAX;
    }
    put(I.progs.p + off, prog->data(), prog->size());
    put(I.prog_off_d.p + q, &off64, sizeof(off64));
    put(I.plite.p + q, &pl, sizeof(pl));
    put(I.prow.p + q, &row, sizeof(row));
    put(I.sums.p + q, &z, sizeof(z));
    note_program(I, *prog, off);
    *placed = true;
  }
  if (!segs.empty()) {  // the fused upload: [list | payloads] in one mapped pinned block
    const size_t lb = (segs.size() * sizeof(UpSeg) + 15) & ~(size_t)15, total = lb + pay.size();
    size_t cap = 0;
    uint8_t* blk = pinned_get(total, cap);
    uint8_t* dv = blk ? pinned_dev(blk) : nullptr;
    if (!dv) {
      if (blk) pinned_put(blk, cap);
      err = "add_classes: no mapped pinned memory";
      return false;
    }
    uint32_t most = 0;
    for (auto& g : segs) {
      if (g.src) g.src = reinterpret_cast<uint64_t>(dv + lb + (g.src - 1));
      most = std::max(most, g.words);
    }
    std::memcpy(blk, segs.data(), segs.size() * sizeof(UpSeg));
    if (!pay.empty()) std::memcpy(blk + lb, pay.data(), pay.size());
    I.hold.push_back(std::shared_ptr<const void>(blk, [cap](const void* q) {
      Engine::pinned_put(const_cast<uint8_t*>(static_cast<const uint8_t*>(q)), cap);
    }));
    const dim3 ug((uint32_t)segs.size(), std::max<uint32_t>(std::min<uint32_t>((most + 4095) / 4096, 64), 1));
    hipLaunchKernelGGL(k_upload, ug, dim3(256), 0, s, reinterpret_cast<const UpSeg*>(dv));
  }
  DevCluster C = I.cluster();
  if (npc && I.pcap)
    hipLaunchKernelGGL(k_pc_build, dim3((I.pcap + kPcBlock - 1) / kPcBlock), dim3(kPcBlock), 0, s, C, pc0, npc, pst);
  if (ntc && I.tcap) hipLaunchKernelGGL(k_tc_build, dim3((I.tcap + kBlock - 1) / kBlock), dim3(kBlock), 0, s, C, tc0);
  HIPCHK(hipGetLastError());
  if (npc) I.red_pc0 = std::min(I.red_pc0, pc0);
  if (ntc) I.red_tc0 = std::min(I.red_tc0, tc0);
  if (!reduce_tables(I, err)) return false;
  if (I.shards > 1) return stream_sync(I, s, err);
  I.unwaited = true;
  return true;
}

bool Engine::rebuild_class_tables(std::string& err) {
  Impl& I = *p_;
  hipStream_t s = I.stream;
  if (!I.npc && !I.ntc) return true;
  const size_t Nn = std::max<uint32_t>(I.N, 1), NUn = std::max<uint32_t>(I.NU, 1);
  if (I.npc) {
    HIPCHK(hipMemsetAsync(I.pc_cnt.p, 0, (size_t)I.npc * Nn * 4, s));
    HIPCHK(hipMemsetAsync(I.pc_dom.p, 0, (size_t)I.npc * NUn * 4, s));
    HIPCHK(hipMemsetAsync(I.pc_tot.p, 0, (size_t)I.npc * KSG_MAX_TOPO * 4, s));
  }
  if (I.ntc) {
    HIPCHK(hipMemsetAsync(I.tc_val.p, 0, (size_t)I.tc_used * 4, s));
    HIPCHK(hipMemsetAsync(I.tc_tot.p, 0, (size_t)I.ntc * 4, s));
  }
  DevCluster C = I.cluster();
  if (I.npc && I.pcap)
    hipLaunchKernelGGL(k_pc_build, dim3((I.pcap + kPcBlock - 1) / kPcBlock), dim3(kPcBlock), 0, s, C, 0u, I.npc,
                       PcStage{0, 0xFFFFFFFFu, 0, 0, 0, 0, 0xFFFFFFFFu, {}, 0, {}, {}});
  if (I.ntc && I.tcap) hipLaunchKernelGGL(k_tc_build, dim3((I.tcap + kBlock - 1) / kBlock), dim3(kBlock), 0, s, C, 0u);
  HIPCHK(hipGetLastError());
  if (I.npc) I.red_pc0 = 0;
  if (I.ntc) I.red_tc0 = 0;
  return reduce_tables(I, err);
}

bool Engine::replace_program(uint32_t q, const std::vector<uint8_t>& prog, std::string& err) {
  Impl& I = *p_;
  hipStream_t s = I.stream;
  if (q >= I.prog_off.size()) { err = "program index out of range"; return false; }
  const size_t off = (I.prog_bytes + 255) & ~(size_t)255;
  if (!I.progs.grow(off + prog.size(), I.prog_bytes, s, err)) return false;
  const uint64_t off64 = off;
  HIPCHK(hipMemcpyAsync(I.progs.p + off, prog.data(), prog.size(), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(I.prog_off_d.p + q, &off64, sizeof(off64), hipMemcpyHostToDevice, s));
  if (!stream_sync(I, s, err)) return false;  // host sources
  I.prog_bytes = off + prog.size();
  I.prog_off[q] = off;
  const ksg_prog* h = reinterpret_cast<const ksg_prog*>(prog.data());
  I.prog_need[q] = prog_need_of(h);
  if (!na_weights_fit(prog)) I.static_fits = false;
  I.max_na_sum = std::max(I.max_na_sum, na_weight_sum(prog));
  for (int c = 2; c < KSG_MAX_RES; ++c) I.any_eph_req |= h->req[c] != 0;
  return true;
}

bool Engine::normalized(uint32_t j, std::vector<int32_t>& norm, std::string& err) {
  Impl& I = *p_;
  if (!(I.keep_n && j >= I.keep_first && j < I.keep_first + I.keep_n)) { err = "outputs not kept for this pod"; return false; }
  const size_t N = I.N, k = j - I.keep_first;
  if (!I.knorm.alloc(std::max<size_t>(N, 1) * KSG_MAX_PLUGINS, err)) return false;
  DevCluster C = I.cluster();
  hipLaunchKernelGGL(k_norm_out, dim3(std::max<uint32_t>((I.N + kBlock - 1) / kBlock, 1)), dim3(kBlock), 0, I.stream, C,
                     I.F, I.progs.p + I.prog_off[j], I.sums.p + j, I.kfilter.p + k * N,
                     I.kscore.p + k * N * KSG_MAX_PLUGINS, I.knorm.p);
  HIPCHK(hipGetLastError());
  norm.resize((size_t)I.F.n * N);
  if (N) HIPCHK(hipMemcpyAsync(norm.data(), I.knorm.p, norm.size() * 4, hipMemcpyDeviceToHost, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

// ---- device cycle view (ksg_cycle_view_acquire)
static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
void Engine::view_layout(ViewLayout& lay) const {
  const Impl& I = *p_;
  lay = ViewLayout{};
  lay.N = I.N;
  lay.n_raw = (uint32_t)I.F.n;
  lay.n_slots = kViewSlots;
  for (int d = 0; d < KSG_MAX_PLUGINS; ++d) {
    lay.norm_row[d] = -1;
    if (d >= I.F.n) continue;
    const int p = I.F.plugins[d];
    if (p == KP_TAINT || p == KP_NA || p == KP_PTS || p == KP_IPA) lay.norm_row[d] = (int)lay.n_norm++;
  }
  const size_t N = std::max<uint32_t>(I.N, 1);
  lay.off_sum = al256((kViewSlots + 1) * sizeof(uint64_t));
  lay.off_rows = lay.off_sum + al256(sizeof(ksg_pod_summary));
  lay.off_fail_pos = lay.off_rows + al256(sizeof(ViewRows));
  lay.off_fail_code = lay.off_fail_pos + al256(N);
  lay.off_fail_msg = lay.off_fail_code + al256(N);
  lay.off_raw = lay.off_fail_msg + al256(2 * N);
  lay.off_norm = lay.off_raw + al256(4 * N) * lay.n_raw;  // (the widest layout: every row 4 bytes)
  lay.bytes = lay.off_norm + al256(4 * N) * lay.n_norm;
}
bool Engine::view_arm(uint32_t j, const ViewCfg& cfg, const ViewLayout& lay, uint8_t* host, std::string& err) {
  return view_impl(j, cfg, lay, host, err, false, true);
}
bool Engine::view_arm_finish(std::string& err) {
  Impl& I = *p_;
  if (!I.vp_armed) return true;
  I.vp_armed = false;
  I.vp_last_fused = I.vp_fused;
  if (I.vp_fused) {  // (k_eval wrote it)
    I.views_fused++;
    return true;
  }
  const size_t N = I.N, k = I.vp_k;
  hipLaunchKernelGGL(k_view, dim3((uint32_t)((N + 255) / 256)), dim3(256), 0, I.stream, I.cluster(), I.F,
                     I.progs.p + I.prog_off[I.vp_q], I.sums.p + I.vp_q, I.kfilter.p + k * N,
                     I.kscore.p + k * N * KSG_MAX_PLUGINS, I.vp_V, I.vblk.p, I.vp_hout, I.vdone.p);
  HIPCHK(hipGetLastError());
  return true;
}
bool Engine::view_fused() const { return p_->vp_last_fused; }
uint64_t Engine::views_fused() const { return p_->views_fused; }
bool Engine::view(uint32_t j, const ViewCfg& cfg, const ViewLayout& lay, uint8_t* host, std::string& err, bool wait) {
  p_->vp_armed = false;
  p_->vp_last_fused = false;
  return view_impl(j, cfg, lay, host, err, wait, false);
}
bool Engine::view_impl(uint32_t j, const ViewCfg& cfg, const ViewLayout& lay, uint8_t* host, std::string& err, bool wait,
                       bool arm) {
  Impl& I = *p_;
  if (!(I.keep_n && j >= I.keep_first && j < I.keep_first + I.keep_n)) { err = "outputs not kept for this pod"; return false; }
  if (lay.N != I.N || lay.n_raw != (uint32_t)I.F.n) { err = "view layout of another snapshot"; return false; }
  if (lay.bytes > I.vblk.n || !I.vblk.p) I.vblk_fresh = true;
  if (!I.vblk.alloc(lay.bytes, err)) return false;
  ViewDev V{};
  for (int d = 0; d < KSG_MAX_PLUGINS; ++d) {
    V.prof_of_dev[d] = (int8_t)cfg.prof_of_dev[d];
    V.dev_vol[d] = cfg.dev_vol[d] ? 1 : 0;
    V.norm_row[d] = (int8_t)lay.norm_row[d];
  }
  for (int p = 0; p < KSG_MAX_PROFILE; ++p) V.kind[p] = (uint8_t)cfg.kind[p];
  V.n_profile = cfg.n_profile;
  if (++I.vgen == 0) ++I.vgen;  // (generation 0: never a live entry)
  V.gen = I.vgen;
  lay.gen = I.vgen;
  V.off_sum = (uint32_t)lay.off_sum;
  V.off_fail_pos = (uint32_t)lay.off_fail_pos;
  V.off_fail_code = (uint32_t)lay.off_fail_code;
  V.off_fail_msg = (uint32_t)lay.off_fail_msg;
  V.off_raw = (uint32_t)lay.off_raw;
  V.off_norm = (uint32_t)lay.off_norm;
  V.off_rows = (uint32_t)lay.off_rows;
  V.n_norm = lay.n_norm;
  V.narrow = I.view_narrow ? 1u : 0u;
  V.slots_direct = I.view_slots_direct ? 1u : 0u;
  const size_t N = I.N, k = j - I.keep_first;
  hipStream_t s = I.stream;
  if (I.vblk_fresh) {  // a new block: generation 0 everywhere
    HIPCHK(hipMemsetAsync(I.vblk.p, 0, (kViewSlots + 1) * sizeof(uint64_t), s));
    I.vblk_fresh = false;
  }
  if (!N) {
    HIPCHK(hipMemcpyAsync(I.vblk.p + lay.off_sum, I.sums.p + j, sizeof(ksg_pod_summary), hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemsetAsync(I.vblk.p + lay.off_rows, 0, sizeof(ViewRows), s));
  }
  // the per-node arrays straight into the caller's pinned block when the device
  // can address it (one kernel, then only the slot table and summary are copied)
  uint8_t* hdev = N && !I.view_copy ? pinned_dev(host) : nullptr;
  if (hdev && I.view_slots_direct)  // (k_view writes each slot as it claims it: the rest reads empty)
    std::memset(host, 0, (kViewSlots + 1) * sizeof(uint64_t));
  if (hdev && !I.vdone.p) {
    if (!I.vdone.alloc(1, err)) return false;
    HIPCHK(hipMemsetAsync(I.vdone.p, 0, sizeof(uint32_t), s));
  }
  if (arm) {  // (launched by the next run_queue's k_eval, or by view_arm_finish)
    if (!N || !hdev) { err = "view_arm: a direct view of a non-empty snapshot only"; return false; }
    I.vp_armed = true;
    I.vp_fused = false;
    I.vp_q = j;
    I.vp_k = k;
    I.vp_V = V;
    I.vp_hout = hdev;
    return true;
  }
  if (N)
    hipLaunchKernelGGL(k_view, dim3((uint32_t)((N + 255) / 256)), dim3(256), 0, s, I.cluster(), I.F, I.progs.p + I.prog_off[j],
                       I.sums.p + j, I.kfilter.p + k * N, I.kscore.p + k * N * KSG_MAX_PLUGINS, V, I.vblk.p,
                       hdev ? hdev : I.vblk.p, I.vdone.p);
  HIPCHK(hipGetLastError());
  if (!hdev) HIPCHK(hipMemcpyAsync(host, I.vblk.p, lay.bytes, hipMemcpyDeviceToHost, s));  // (direct: k_view wrote it all)
  if (!wait) return true;  // (queued behind the cycle's run: the caller's next sync completes it)
  if (!stream_sync(I, s, err)) return false;
  return true;
}
namespace {
std::mutex g_pin_mu;
std::multimap<size_t, uint8_t*> g_pin_free;  // capacity -> block
std::unordered_map<const uint8_t*, uint8_t*> g_pin_dev;  // pinned block -> its device address
}  // namespace
uint8_t* Engine::pinned_dev(const uint8_t* host) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pin_dev.find(host);
  return it == g_pin_dev.end() ? nullptr : it->second;
}
uint8_t* Engine::pinned_get(size_t bytes, size_t& cap) {
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pin_free.lower_bound(bytes);
    if (it != g_pin_free.end() && it->first <= 4 * bytes + (1u << 20)) {
      uint8_t* p = it->second;
      cap = it->first;
      g_pin_free.erase(it);
      return p;
    }
  }
  cap = std::max<size_t>(al256(bytes), 4096);
  uint8_t* p = nullptr;
  if (hipHostMalloc((void**)&p, cap, hipHostMallocDefault) != hipSuccess) {
    p = static_cast<uint8_t*>(std::malloc(cap));  // (pageable: the copy still works, slower)
    cap |= 1;  // tag: malloc'd
  } else {
    uint8_t* d = nullptr;  // (the view kernel writes the block directly when the device can address it)
    if (hipHostGetDevicePointer((void**)&d, p, 0) == hipSuccess && d) {
      std::lock_guard<std::mutex> lk(g_pin_mu);
      g_pin_dev[p] = d;
    } else {
      (void)hipGetLastError();
    }
  }
  return p;
}
void Engine::pinned_put(uint8_t* p, size_t cap) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  if (g_pin_free.size() >= 64) {  // bounded pool: free the block
    g_pin_dev.erase(p);
    if (cap & 1) std::free(p);
    else (void)hipHostFree(p);
    return;
  }
  g_pin_free.emplace(cap, p);
}

bool Engine::set_summaries(uint32_t first, uint32_t count, const ksg_pod_summary* in, std::string& err) {
  Impl& I = *p_;
  if (first + count > I.prog_off.size()) { err = "program index out of range"; return false; }
  HIPCHK(hipMemcpyAsync(I.sums.p + first, in, count * sizeof(ksg_pod_summary), hipMemcpyHostToDevice, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

bool Engine::set_programs(const std::vector<std::vector<uint8_t>>& progs, std::string& err) {
  Impl& I = *p_;
  std::vector<uint8_t> blob;
  I.prog_off.clear();
  I.prog_need.clear();
  for (auto& p : progs) {
    size_t off = (blob.size() + 255) & ~(size_t)255;  // 256-B aligned programs
    blob.resize(off);
    I.prog_off.push_back(off);
    blob.insert(blob.end(), p.begin(), p.end());
    I.prog_need.push_back(prog_need_of(reinterpret_cast<const ksg_prog*>(p.data())));
  }
  if (!I.progs.upload(blob, I.stream, err)) return false;
  I.prog_bytes = blob.size();
  {
    std::vector<PodLite> pl(progs.size());
    for (size_t i = 0; i < progs.size(); ++i) pl[i] = pod_lite(progs[i]);
    if (!I.plite.upload(pl, I.stream, err)) return false;
  }
  std::vector<uint64_t> offs(I.prog_off.begin(), I.prog_off.end());
  if (!I.prog_off_d.upload(offs, I.stream, err)) return false;
  I.any_eph_req = false;
  I.max_na_sum = 0;
  for (auto& p : progs) {
    const ksg_prog* h = reinterpret_cast<const ksg_prog*>(p.data());
    for (int c = 2; c < KSG_MAX_RES; ++c) I.any_eph_req |= h->req[c] != 0;
    if (!na_weights_fit(p)) I.static_fits = false;
    I.max_na_sum = std::max(I.max_na_sum, na_weight_sum(p));
  }
  for (int i = 0; i < I.F.fit_n; ++i) I.any_eph_req |= I.F.fit_res[i] >= 2;
  for (int i = 0; i < I.F.ba_n; ++i) I.any_eph_req |= I.F.ba_res[i] >= 2;
  if (!I.sums.alloc(std::max<size_t>(progs.size(), 1), err) || !I.prow.alloc(std::max<size_t>(progs.size(), 1), err))
    return false;
  HIPCHK(hipMemsetAsync(I.prow.p, 0xFF, I.prow.n * sizeof(int32_t), I.stream));
  uint32_t cnt = (uint32_t)progs.size();
  if (cnt) {
    hipLaunchKernelGGL(k_init_summaries, dim3((cnt + 255) / 256), dim3(256), 0, I.stream, I.sums.p, cnt, I.F);
    HIPCHK(hipGetLastError());
  }
  return true;
}

bool Engine::keep_outputs(uint32_t keep_first, uint32_t keep_n, std::string& err) {
  Impl& I = *p_;
  I.keep_first = keep_first;
  I.keep_n = keep_n;
  if (!keep_n) return true;
  size_t N = std::max<uint32_t>(I.N, 1);
  return I.kfilter.alloc(N * keep_n, err) && I.kscore.alloc(N * keep_n * KSG_MAX_PLUGINS, err) &&
         I.ktotal.alloc(N * keep_n, err);
}

static bool run_batches(Engine::Impl& I, uint32_t first, uint32_t count, std::string& err);

bool Engine::run_queue(uint32_t first, uint32_t count, bool commit, std::string& err) {
  Impl& I = *p_;
  if (first + count > I.prog_off.size()) { err = "program index out of range"; return false; }
  if (!tables_ready(I, err)) return false;
  if (commit && batch_path()) return run_batches(I, first, count, err);
  hipStream_t s = I.stream;
  DevCluster C = I.cluster();
  DevScratch S = I.scratch();
  const DevProfile& F = I.F;
  uint32_t N = I.N;
  dim3 gN((N + kBlock - 1) / kBlock), b(kBlock);
  int pts_pos = -1;
  for (int i = 0; i < F.n; ++i)
    if (F.plugins[i] == KP_PTS) pts_pos = i;
  if (I.sample_every) {
    size_t need = 2 * ((count + I.sample_every - 1) / I.sample_every + 1);
    while (I.sev.size() < need) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      I.sev.push_back(e);
    }
  }
  I.n_samples = 0;
  HIPCHK(hipEventRecord(I.ev0, s));
  const bool xchain = I.xranks > 1;  // sharded per-pod chain (exchange points X1..X4)
  if (I.static_ok && I.static_fits && !xchain) {
    const size_t Nn = std::max<uint32_t>(N, 1);
    const uint32_t chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(count, ((size_t)64 << 20) / (Nn * sizeof(StaticRec))));
    if (!I.stat.alloc((size_t)chunk * Nn, err) || !I.mpred.alloc(2 * (size_t)chunk, err)) return false;
    for (uint32_t c0 = first; c0 < first + count; c0 += chunk) {
      const uint32_t cn = std::min(chunk, first + count - c0);
      HIPCHK(hipMemsetAsync(I.mpred.p, 0xFF, 2 * (size_t)cn * sizeof(int64_t), s));  // -1: no statically feasible node
      const dim3 grid(std::max<uint32_t>((N + 256 * KSG_ST_NPT - 1) / (256 * KSG_ST_NPT), 1),
                      (cn + KSG_ST_PODS - 1) / KSG_ST_PODS);
      hipLaunchKernelGGL(k_static, grid, dim3(256), 0, s, C, F, I.progs.p, I.prog_off_d.p, c0, cn, I.stat.p, I.mpred.p, 0);
      for (uint32_t j = c0; j < c0 + cn; ++j) {
        const uint8_t* prog = I.progs.p + I.prog_off[j];
        const int mode = commit ? 1 : 0;
        DevOut O{I.filter.p, I.score.p, I.total.p, I.sums.p + j, nullptr, mode, I.prow.p + j};
        if (I.keep_n && j >= I.keep_first && j < I.keep_first + I.keep_n) {
          size_t k = j - I.keep_first;
          O.filter = I.kfilter.p + k * N;
          O.score = I.kscore.p + k * N * KSG_MAX_PLUGINS;
          O.total = I.ktotal.p + k * N;
        }
        bool sampled = I.sample_every && (j % I.sample_every) == 0 && I.n_samples * 2 + 2 <= I.sev.size();
        if (sampled) HIPCHK(hipEventRecord(I.sev[I.n_samples * 2], s));
        hipLaunchKernelGGL(k_fs_static, gN, b, 0, s, C, F, O, prog, I.stat.p + (size_t)(j - c0) * Nn,
                           I.mpred.p + 2 * (size_t)(j - c0), I.saux.p);
        if (sampled) {
          HIPCHK(hipEventRecord(I.sev[I.n_samples * 2 + 1], s));
          I.n_samples++;
        }
      }
    }
    HIPCHK(hipEventRecord(I.ev1, s));
    HIPCHK(hipGetLastError());
    return true;
  }
  const XLay XL{I.nsp, I.spair.p, I.uniq};
  // one exchange point: pack (device), all-gather, merge (device)
  auto xrun = [&](size_t len, auto pack, auto merge) -> bool {
    const size_t bytes = std::max<size_t>(len, 1) * sizeof(int64_t);
    if (!I.xsend.grow(bytes, 0, s, err) || !I.xrecv.grow(bytes * I.xranks, 0, s, err)) return false;
    pack(reinterpret_cast<int64_t*>(I.xsend.p));
    if (!xgather(I, bytes, err)) return false;
    merge(reinterpret_cast<const int64_t*>(I.xrecv.p));
    return true;
  };
  const uint32_t xr = I.xranks;
  // table chain (table_chain.hip): pod index on the device, partials per block
  ChainArgs CA{};
  CA.progs = I.progs.p;
  CA.prog_off = I.prog_off_d.p;
  CA.sums = I.sums.p;
  CA.keep_first = I.keep_first;
  CA.keep_n = I.keep_n;
  CA.kfilter = I.kfilter.p; CA.kscore = I.kscore.p; CA.ktotal = I.ktotal.p;
  CA.filter = I.filter.p; CA.score = I.score.p; CA.total = I.total.p;
  CA.nblk = I.cnblk;
  CA.pi = I.cpi.p; CA.pm = I.cpm.p; CA.pr = I.cpr.p; CA.pm2 = I.cpm2.p; CA.pk = I.cpk.p; CA.pst = I.cpst.p;
  CA.mode = commit ? (1 | ((I.has_pts || I.has_ipa) ? 2 : 0)) : 0;
  CA.prow = I.prow.p;
  CA.need_eph = I.any_eph_req ? 1u : 0u;
  if (!I.alog.alloc(std::max<uint32_t>(count, 1), err)) return false;
  CA.alog = I.alog.p;
  CA.log_base = first;
  CA.arrive = I.carrive.p;
  CA.stamps = I.cstamps_on ? I.cstamps.p : nullptr;
  CA.etot = nullptr;
  CA.xsend = nullptr;
  CA.cand = I.ccand.p;
  // one-launch cycles (k_eval_solo) for pods of normalising profiles whose outputs
  // are not kept, unsharded, committing cycles only (a dry run reads the per-node
  // filter codes, which k_eval_solo does not write); opt-in (KSG_SOLO=1): measured
  // slower than the two-launch chain on cfg4 (63.6 vs 35.2 us/pod, r03)
  const bool solo_ok = commit && !xchain && F.has_ext && I.solo == 1;
  if (I.cnblk > I.fold_blocks || xchain) {  // fold k_eval's partials once (k_fold, or the X2 merge) above this many blocks
    if (!I.cetot.alloc(1, err)) return false;
    CA.etot = I.cetot.p;
  }
  if (xchain) {  // node-sharded table chain: the X2 / X3 / X4 records
    const size_t xb = (size_t)kX2 * sizeof(int64_t);
    if (!I.xsend.grow(xb, 0, s, err) || !I.xrecv.grow(xb * I.xranks, 0, s, err)) return false;
  }
  int64_t* const xs = reinterpret_cast<int64_t*>(I.xsend.p);
  const int64_t* const xrv = reinterpret_cast<const int64_t*>(I.xrecv.p);
  const int rowm = I.R > 4 ? 0 : (I.eval_mode == 1 ? 2 : 1);
  bool pending = false;           // logged assumes whose existing-pod table rows are not written yet
  // rows of the logged pods [log_base, j); the log restarts at `next` (a pod of the
  // scanning chain is not logged: the log restarts after it)
  auto flush = [&](uint32_t j, uint32_t next) {
    if (pending) hipLaunchKernelGGL(k_flush_appends, dim3(1), b, 0, s, C, CA, j - CA.log_base);
    pending = false;
    CA.log_base = next;
  };
  uint32_t pmask = 0;  // the profile's device plugins (kernel specialisations)
  for (int i = 0; i < F.n; ++i) pmask |= 1u << F.plugins[i];
  if (__builtin_popcount(pmask) != F.n) pmask = ~0u;  // (a plugin at two positions: the generic kernels, kNPos)
  // persistent segments (k_chain_run): consecutive eligible pods in one launch
  auto kept_pod = [&](uint32_t j) { return I.keep_n && j >= I.keep_first && j < I.keep_first + I.keep_n; };
  bool run_ok = commit && !xchain && F.has_ext && rowm != 0 && I.run_on != 0;
  if (run_ok && !I.run_cap) {
    int occ1 = 0, occ2 = 0;
    int occ3 = 0, occ4 = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ1, k_chain_run<1, ~0u>, kChain, 0));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ2, k_chain_run<2, ~0u>, kChain, 0));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ3, k_chain_run<2, kPmTab>, kChain, 0));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ4, k_chain_run<2, kPmTabTN>, kChain, 0));
    int occ5 = 0, occ6 = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ5, (k_chain_run<2, kPmTab, kRunLK, kRunTS>), kChain, 0));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ6, (k_chain_run<2, kPmTab, kRunLK, kRunTS, 512>), 512, 0));
    const int occ = std::min(std::min(std::min(occ1, occ2), std::min(occ3, occ4)), occ5);
    I.run_cap512 = occ6 <= 0 ? 0u : I.n_cus * (uint32_t)(occ6 >= 2 ? occ6 - 1 : occ6);
    // (MI355X_MICROARCH.md: the hardware may admit one block per CU fewer than the query)
    I.run_cap = occ <= 0 ? 1u : I.n_cus * (uint32_t)(occ >= 2 ? occ - 1 : occ);
    if (occ <= 0) I.run_on = 0;
  }
  // 512-thread blocks (KSG_RUN_BT=512): half the blocks, for the small size class of the cfg4 plugin set
  const uint32_t nb512 = (I.N + 511) / 512;
  const bool bt512 = I.run_bt == 512 && (pmask & ~kPmTab) == 0 && rowm == 2 && nb512 + 1 <= I.run_cap512 && nb512 <= (uint32_t)kChain;
  run_ok = run_ok && I.run_on != 0 && I.cnblk + 1 <= I.run_cap && I.cnblk <= (uint32_t)kChain;  // (+1: the committer)
  auto run_elig = [&](uint32_t j) {
    const uint32_t nd = I.prog_need[j];
    return (nd & 4) && !(nd & 8) && (nd & (1u << 17)) && !kept_pod(j);
  };
  if (run_ok) {
    if (!I.rsync.alloc(1, err) || !I.rgran.alloc(4 * kRunSlot, err)) return false;
    if (!I.hverdict) {
      HIPCHK(hipHostMalloc((void**)&I.hverdict, 64, hipHostMallocCoherent | hipHostMallocMapped));
      HIPCHK(hipMemsetAsync(I.rsync.p, 0, sizeof(RunSync), s));  // (the sticky abort word starts clear)
    }
  }
  for (uint32_t j = first; j < first + count; ++j) {
    const uint8_t* prog = I.progs.p + I.prog_off[j];
    if (run_ok && run_elig(j)) {
      // a segment: consecutive eligible pods of one size class
      const uint32_t cls = I.prog_need[j] & (1u << 18);
      uint32_t j1 = j + 1;
      while (j1 < first + count && run_elig(j1) && (I.prog_need[j1] & (1u << 18)) == cls) ++j1;
      if (j1 - j >= I.run_min) {
        CA.q = j;
        CA.prog = prog;
        CA.xsend = nullptr;
        ChainArgs RA = CA;  // (stamps: k_chain_run's own slots)
        HIPCHK(hipMemsetAsync(I.rsync.p, 0, kRunSyncReset, s));
        HIPCHK(hipMemsetAsync(I.rgran.p, 0, 4 * kRunSlot * sizeof(uint64_t), s));
        const bool sampled = I.sample_every && I.n_samples * 2 + 2 <= I.sev.size();
        if (sampled) HIPCHK(hipEventRecord(I.sev[I.n_samples * 2], s));
        uint64_t* const g1 = I.rgran.p;
        uint64_t* const g2 = I.rgran.p + 2 * kRunSlot;
        const bool l512 = bt512 && cls;
        const uint32_t grid = (l512 ? nb512 : I.cnblk) + 1;  // node blocks + the committer
        uint32_t* const hv = I.hverdict;
        __atomic_store_n(hv, 0u, __ATOMIC_RELEASE);  // (the previous segment's verdict was read)
        const RunCtl RC{grid + I.run_need_extra, I.run_wait_us * 100u, I.run_lag, hv, I.run_spin, I.run_overlap ? 1u : 0u,
                        I.run_defer ? 1u : 0u};
        const dim3 gr(grid), bk(kChain);
        if (l512) {
          ChainArgs R5 = RA;
          R5.nblk = nb512;
          hipLaunchKernelGGL((k_chain_run<2, kPmTab, kRunLK, kRunTS, 512>), gr, dim3(512), 0, s, C, F, R5, j1 - j,
                             I.rsync.p, g1, g2, RC, RA.progs, RA.prog_off);
        } else if (rowm == 2 && (pmask & ~kPmTab) == 0 && cls)
          hipLaunchKernelGGL((k_chain_run<2, kPmTab, kRunLK, kRunTS>), gr, bk, 0, s, C, F, RA, j1 - j, I.rsync.p, g1, g2, RC, RA.progs, RA.prog_off);
        else if (rowm == 2 && (pmask & ~kPmTab) == 0)
          hipLaunchKernelGGL((k_chain_run<2, kPmTab>), gr, bk, 0, s, C, F, RA, j1 - j, I.rsync.p, g1, g2, RC, RA.progs, RA.prog_off);
        else if (rowm == 2 && (pmask & ~kPmTabTN) == 0)
          hipLaunchKernelGGL((k_chain_run<2, kPmTabTN>), gr, bk, 0, s, C, F, RA, j1 - j, I.rsync.p, g1, g2, RC, RA.progs, RA.prog_off);
        else if (rowm == 2) hipLaunchKernelGGL((k_chain_run<2, ~0u>), gr, bk, 0, s, C, F, RA, j1 - j, I.rsync.p, g1, g2, RC, RA.progs, RA.prog_off);
        else hipLaunchKernelGGL((k_chain_run<1, ~0u>), gr, bk, 0, s, C, F, RA, j1 - j, I.rsync.p, g1, g2, RC, RA.progs, RA.prog_off);
        if (sampled) {
          HIPCHK(hipEventRecord(I.sev[I.n_samples * 2 + 1], s));
          I.n_samples++;
        }
        HIPCHK(hipGetLastError());
        I.run_used = true;
        // The handshake: the launch's blocks decide whether all of them are
        // resident before any state changes.  The host waits for that verdict (the
        // work queued before the segment runs first), then queues the rest.
        const uint32_t v = wait_verdict(I, s, err);
        if (v == 0u) return false;
        if (v == 3u) {  // an earlier segment of this call aborted: the state is not valid
          I.lost = true;
          err = "persistent table chain: a gate never completed (blocks not co-resident?)";
          return false;
        }
        if (v == 1u) {
          I.path_pods[0] += j1 - j;
          I.path_pods[4] += j1 - j;
          I.path_pods[5]++;
          pending |= (CA.mode & 2) != 0;
          j = j1 - 1;
          continue;
        }
        // v == 2: the blocks were not all resident; they left untouched.  This and
        // the call's later segments run on the two-launch chain.
        I.run_fallbacks++;
        run_ok = false;
      }
    }
    if (I.prog_need[j] & 4) {
      I.path_pods[0]++;
      CA.q = j;
      CA.prog = prog;
      CA.xsend = xchain ? xs : nullptr;
      if (solo_ok && !(I.prog_need[j] & 8) && !(I.keep_n && j >= I.keep_first && j < I.keep_first + I.keep_n)) {
        const bool sampled = I.sample_every && (j % I.sample_every) == 0 && I.n_samples * 2 + 2 <= I.sev.size();
        if (sampled) HIPCHK(hipEventRecord(I.sev[I.n_samples * 2], s));
        if (rowm == 2) hipLaunchKernelGGL(k_eval_solo<2>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CA, prog);
        else if (rowm == 1) hipLaunchKernelGGL(k_eval_solo<1>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CA, prog);
        else hipLaunchKernelGGL(k_eval_solo<0>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CA, prog);
        if (sampled) {
          HIPCHK(hipEventRecord(I.sev[I.n_samples * 2 + 1], s));
          I.n_samples++;
        }
        I.path_pods[2]++;
        pending |= (CA.mode & 2) != 0;
        continue;
      }
      const bool sampled = I.sample_every && (j % I.sample_every) == 0 && I.n_samples * 2 + 2 <= I.sev.size();
      if (sampled) HIPCHK(hipEventRecord(I.sev[I.n_samples * 2], s));
      const bool occ = I.cnblk > (I.occ_blocks ? I.occ_blocks : 2 * I.n_cus) || I.occ_force;  // many blocks per CU
      if (occ) {
        if (rowm == 2) hipLaunchKernelGGL(k_eval_occ<2>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CA, prog);
        else if (rowm == 1) hipLaunchKernelGGL(k_eval_occ<1>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CA, prog);
        else hipLaunchKernelGGL(k_eval_occ<0>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CA, prog);
      } else {
        // (a fused view: the armed view of this pod when its cycle is this one launch)
        ChainArgs CE = CA;
        if (I.vp_armed && I.vp_q == j && !I.vp_fused && I.view_fuse && !F.has_ext && !xchain && I.vblk.p) {
          CE.vf = I.vp_V;
          CE.vf_out = I.vblk.p;
          CE.vf_hout = I.vp_hout;
          I.vp_fused = true;
        }
        if (rowm == 2) hipLaunchKernelGGL(k_eval<2>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CE, prog);
        else if (rowm == 1) hipLaunchKernelGGL(k_eval<1>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CE, prog);
        else hipLaunchKernelGGL(k_eval<0>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CE, prog);
      }
      if (sampled) {
        HIPCHK(hipEventRecord(I.sev[I.n_samples * 2 + 1], s));
        I.n_samples++;
      }
      if (F.has_ext) {  // (k_final's last block selects; without ScoreExtensions k_eval's)
        if (xchain) {  // X2: the cycle's counts and normalisers over every rank
          hipLaunchKernelGGL(k_tx2_pack, dim3(1), dim3(kChain), 0, s, C, F, CA, prog, xs);
          if (!xgather(I, (size_t)kX2 * sizeof(int64_t), err)) return false;
          hipLaunchKernelGGL(k_tx2_merge, dim3(1), dim3(64), 0, s, C, CA, prog, xrv, xr);
        } else if (CA.etot) {
          hipLaunchKernelGGL(k_fold, dim3(1), dim3(kChain), 0, s, C, F, CA, prog);
        }
        if (I.prog_need[j] & 8) {
          hipLaunchKernelGGL(k_ptsraw, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CA, prog);
          if (xchain) {  // X3
            hipLaunchKernelGGL(k_tx3_pack, dim3(1), dim3(kChain), 0, s, CA, xs);
            if (!xgather(I, 2 * sizeof(int64_t), err)) return false;
            hipLaunchKernelGGL(k_tx3_merge, dim3(1), dim3(kChain), 0, s, CA, xrv, xr);
          }
        }
        if (occ) hipLaunchKernelGGL(k_final_occ, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CA, prog);
        else if ((pmask & ~kPmTab) == 0 && I.final_pm)  // (the plugin-set specialisation: kNPos)
          hipLaunchKernelGGL(k_final<kPmTab>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CA, prog);
        else hipLaunchKernelGGL(k_final<>, dim3(I.cnblk), dim3(kChain), 0, s, C, F, CA, prog);
      }
      if (xchain) {  // X4: selectHost over the ranks, the assume split by ownership
        if (!xgather(I, 3 * sizeof(int64_t), err)) return false;
        hipLaunchKernelGGL(k_tx4_select, dim3(1), dim3(64), 0, s, C, F, CA, prog, xrv, xr);
      }
      pending |= (CA.mode & 2) != 0;
      continue;
    }
    flush(j, j + 1);  // the scanning chain reads the existing-pod table
    I.path_pods[1]++;
    const int mode = commit ? (1 | ((I.has_pts || I.has_ipa) ? 2 : 0)) : 0;
    DevOut O{I.filter.p, I.score.p, I.total.p, I.sums.p + j, xchain ? nullptr : I.arrive1.p, mode, I.prow.p + j};
    bool kept = I.keep_n && j >= I.keep_first && j < I.keep_first + I.keep_n;
    if (kept) {
      size_t k = j - I.keep_first;
      O.filter = I.kfilter.p + k * N;
      O.score = I.kscore.p + k * N * KSG_MAX_PLUGINS;
      O.total = I.ktotal.p + k * N;
    }
    bool pts = I.has_pts && (I.prog_need[j] & 1);
    bool ipa = I.has_ipa;
    if (pts || ipa) {
      uint32_t work = std::max<uint32_t>(KSG_MAX_TSC * N, I.topo.topo_pairs);
      uint32_t gb = std::min<uint32_t>((work + kBlock - 1) / kBlock, 2048);
      hipLaunchKernelGGL(k_begin, dim3(std::max<uint32_t>(gb, 1)), b, 0, s, C, S, prog);
      uint32_t pc = I.pcap;  // grid covers capacity; kernel reads the live count
      hipLaunchKernelGGL(k_scan_pods, dim3((pc + kBlock - 1) / kBlock), b, 0, s, C, F, S, O, prog);
      if (ipa)
        hipLaunchKernelGGL(k_scan_terms, dim3((I.tcap + kBlock - 1) / kBlock), b, 0, s, C, F, S, O, prog);
      const dim3 gr(std::max<uint32_t>(std::min<uint32_t>(gN.x, 256), 1));
      if (pts) {
        hipLaunchKernelGGL(k_pts_prep, gN, b, 0, s, C, S, prog);
        hipLaunchKernelGGL(k_pts_reduce, gr, b, 0, s, C, S, prog, xchain ? I.uniq : ~0u);
      }
      if (xchain) {  // X1
        const size_t len = (size_t)7 * I.nsp + 2 + 2 * KSG_MAX_TOPO;
        if (!xrun(len, [&](int64_t* o) { hipLaunchKernelGGL(k_x1_pack, dim3(1), b, 0, s, S, O, XL, o); },
                  [&](const int64_t* r) { hipLaunchKernelGGL(k_x1_merge, dim3(1), b, 0, s, S, O, XL, r, xr); }))
          return false;
        if (pts) hipLaunchKernelGGL(k_pts_reduce, gr, b, 0, s, C, S, prog, ~I.uniq);
      }
    }
    bool sampled = I.sample_every && (j % I.sample_every) == 0 && I.n_samples * 2 + 2 <= I.sev.size();
    if (sampled) HIPCHK(hipEventRecord(I.sev[I.n_samples * 2], s));
    hipLaunchKernelGGL(k_filter_score, gN, b, 0, s, C, F, S, O, prog);
    if (sampled) {
      HIPCHK(hipEventRecord(I.sev[I.n_samples * 2 + 1], s));
      I.n_samples++;
    }
    if (xchain) {  // X2
      const size_t len = 3 + 2 * KSG_MAX_PLUGINS + (size_t)I.nsp + KSG_MAX_TSC;
      if (!xrun(len, [&](int64_t* o) { hipLaunchKernelGGL(k_x2_pack, dim3(1), b, 0, s, C, S, O, prog, XL, o); },
                [&](const int64_t* r) {
                  hipLaunchKernelGGL(k_x2_merge, dim3(1), b, 0, s, S, O, XL, r, xr, I.xregcnt.p);
                }))
        return false;
    }
    if (F.has_ext) {
      if (pts_pos >= 0 && pts) {
        hipLaunchKernelGGL(k_pts_weights, dim3(1), b, 0, s, C, S, O, prog, xchain ? I.xregcnt.p : nullptr, I.uniq);
        hipLaunchKernelGGL(k_pts_score, gN, b, 0, s, C, S, O, prog, pts_pos);
        if (xchain &&  // X3
            !xrun(2 * KSG_MAX_PLUGINS, [&](int64_t* o) { hipLaunchKernelGGL(k_x3_pack, dim3(1), b, 0, s, O, o); },
                  [&](const int64_t* r) { hipLaunchKernelGGL(k_x3_merge, dim3(1), b, 0, s, O, r, xr); }))
          return false;
      }
      hipLaunchKernelGGL(k_finalize, gN, b, 0, s, C, F, S, O, prog);
    }
    if (xchain) {  // X4, then selectHost + assume on the owner of the node
      if (!xrun(2, [&](int64_t* o) { hipLaunchKernelGGL(k_x4_pack, dim3(1), b, 0, s, O, o); },
                [&](const int64_t* r) { hipLaunchKernelGGL(k_x4_merge, dim3(1), b, 0, s, O, r, xr); }))
        return false;
      hipLaunchKernelGGL(k_commit, dim3(1), dim3(64), 0, s, C, F, O, prog, mode, I.prow.p + j);
    }
    // unsharded: selectHost + assume folded into the last block of the cycle's last kernel
  }
  flush(first + count, first + count);
  HIPCHK(hipEventRecord(I.ev1, s));
  HIPCHK(hipGetLastError());
  return true;
}

static uint32_t wait_verdict(Engine::Impl& I, hipStream_t s, std::string& err) {
  uint32_t* const hv = I.hverdict;
  uint32_t v = 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t it = 0; (v = __atomic_load_n(hv, __ATOMIC_ACQUIRE)) == 0u; ++it) {
    if ((it & 1023u) == 1023u) {
      if (hipStreamQuery(s) == hipSuccess && (v = __atomic_load_n(hv, __ATOMIC_ACQUIRE)) == 0u) {
        I.lost = true;
        err = "persistent launch ended without a handshake";
        return 0;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
        I.lost = true;
        err = "persistent launch did not start within 60 s";
        return 0;
      }
      std::this_thread::yield();
    }
  }
  return v;
}

bool Engine::sync(std::string& err) {
  Impl& I = *p_;
  // (the sticky abort word read behind the run on the stream, into a spare word of
  // the pinned verdict block: no second blocking round trip after the sync)
  const bool abort_async = I.run_used && I.hverdict;
  if (abort_async) {
    __atomic_store_n(&I.hverdict[8], 0u, __ATOMIC_RELAXED);
    HIPCHK(hipMemcpyAsync(&I.hverdict[8], I.rsync.p->abort, sizeof(uint32_t), hipMemcpyDeviceToHost, I.stream));
  }
  if (!stream_sync(I, I.stream, err)) return false;
  I.hcalls.clear();  // every queued host exchange has run
  if (I.xfail.exchange(0)) { err = "exchange callback failed"; return false; }
  if (I.run_used) {  // a persistent segment whose poll ran out left the launch early
    I.run_used = false;
    uint32_t ab = 0;
    if (abort_async) ab = __atomic_load_n(&I.hverdict[8], __ATOMIC_ACQUIRE);
    else HIPCHK(hipMemcpy(&ab, I.rsync.p->abort, sizeof(ab), hipMemcpyDeviceToHost));
    if (ab) {
      // the segment (and every later one of its call, which left at the handshake)
      // left summaries unwritten and assumes half applied: the state is lost
      HIPCHK(hipMemset(I.rsync.p->abort, 0, sizeof(ab)));
      I.lost = true;
      err = "persistent table chain: a gate never completed (blocks not co-resident?)";
      return false;
    }
  }
  HIPCHK(hipEventElapsedTime(&I.last_ms, I.ev0, I.ev1));
  return true;
}

bool Engine::summaries(uint32_t first, uint32_t count, ksg_pod_summary* out, std::string& err) {
  Impl& I = *p_;
  HIPCHK(hipMemcpyAsync(out, I.sums.p + first, count * sizeof(ksg_pod_summary), hipMemcpyDeviceToHost, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

bool Engine::outputs(uint32_t j, PodOutputs& out, std::string& err) {
  Impl& I = *p_;
  if (!(I.keep_n && j >= I.keep_first && j < I.keep_first + I.keep_n)) { err = "outputs not kept for this pod"; return false; }
  size_t N = I.N, k = j - I.keep_first;
  out.filter.resize(N);
  out.score.resize(N * KSG_MAX_PLUGINS);
  out.total.resize(N);
  HIPCHK(hipMemcpyAsync(out.filter.data(), I.kfilter.p + k * N, N * 4, hipMemcpyDeviceToHost, I.stream));
  // (the profile's device positions only: rows F.n.. are never read)
  HIPCHK(hipMemcpyAsync(out.score.data(), I.kscore.p + k * N * KSG_MAX_PLUGINS, N * (size_t)I.F.n * 4,
                        hipMemcpyDeviceToHost, I.stream));
  HIPCHK(hipMemcpyAsync(out.total.data(), I.ktotal.p + k * N, N * 4, hipMemcpyDeviceToHost, I.stream));
  HIPCHK(hipMemcpyAsync(&out.summary, I.sums.p + j, sizeof(ksg_pod_summary), hipMemcpyDeviceToHost, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

bool Engine::read_requested(std::vector<int64_t>& requested, std::vector<int32_t>& pod_count, std::string& err) {
  Impl& I = *p_;
  requested.resize((size_t)I.R * I.N);
  pod_count.resize(I.N);
  HIPCHK(hipMemcpyAsync(requested.data(), I.req.p, requested.size() * 8, hipMemcpyDeviceToHost, I.stream));
  HIPCHK(hipMemcpyAsync(pod_count.data(), I.podcnt.p, pod_count.size() * 4, hipMemcpyDeviceToHost, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

bool Engine::read_nonzero(std::vector<int64_t>& nz, std::string& err) {
  Impl& I = *p_;
  nz.resize((size_t)2 * I.N);
  HIPCHK(hipMemcpyAsync(nz.data(), I.nzc.p, (size_t)I.N * 8, hipMemcpyDeviceToHost, I.stream));
  HIPCHK(hipMemcpyAsync(nz.data() + I.N, I.nzm.p, (size_t)I.N * 8, hipMemcpyDeviceToHost, I.stream));
  if (!stream_sync(I, I.stream, err)) return false;
  return true;
}

bool Engine::reset(std::string& err) {
  Impl& I = *p_;
  hipStream_t s = I.stream;
  {  // the node columns from their snapshot copies: one launch (was nine device copies)
    RestoreSegs R{};
    uint32_t n = 0, ny = 1;
    auto add = [&](const void* dst, const void* src, size_t bytes) {
      if (!bytes || !dst || !src) return;
      R.seg[n++] = UpSeg{(uint64_t)(uintptr_t)dst, (uint64_t)(uintptr_t)src, (uint32_t)(bytes / 4), 0};
      ny = std::max<uint32_t>(ny, std::min<uint32_t>(64, (uint32_t)((bytes / 4 + 4095) / 4096)));
    };
    add(I.req.p, I.req0.p, (size_t)I.R * I.N * 8);
    add(I.nzc.p, I.nzc0.p, (size_t)I.N * 8);
    add(I.nzm.p, I.nzm0.p, (size_t)I.N * 8);
    add(I.podcnt.p, I.podcnt0.p, (size_t)I.N * 4);
    if (I.n_ports) add(I.ports.p, I.ports0.p, (size_t)I.n_ports * I.N * 4);
    add(I.pvcuse.p, I.pvcuse0.p, (size_t)I.n_pvc * 4);
    add(I.vatt.p, I.vatt0.p, (size_t)I.n_vatt * 4);
    add(I.vnode.p, I.vnode0.p, (size_t)I.n_vnode * 4);
    add(I.vref.p, I.vref0.p, (size_t)I.n_vnode * 4);
    static_assert(kRestoreSegs >= 9, "restore segments");
    if (n) hipLaunchKernelGGL(k_restore, dim3(n, ny), dim3(256), 0, s, R);
  }
  HIPCHK(hipMemcpyAsync(I.tcounts.p, I.counts0, sizeof(I.counts0), hipMemcpyHostToDevice, s));
  if (!rebuild_class_tables(err)) return false;  // from the restored existing-pod table
  uint32_t cnt = (uint32_t)I.prog_off.size();
  if (cnt) hipLaunchKernelGGL(k_init_summaries, dim3((cnt + 255) / 256), dim3(256), 0, s, I.sums.p, cnt, I.F);
  HIPCHK(hipGetLastError());
  return true;
}

void Engine::sample_kernel(uint32_t every) { p_->sample_every = every; }

bool Engine::set_exchange(int mode, const void* nccl_id, uint32_t rank, uint32_t ranks, ExchangeFn fn, void* user,
                          std::string& err) {
  Impl& I = *p_;
  if (ranks < 1 || rank >= ranks || ranks > 8) { err = "exchange: 1 <= ranks <= 8, rank < ranks"; return false; }
  if (I.comm) { (void)ncclCommDestroy(I.comm); I.comm = nullptr; }
  I.xmode = mode;
  I.xrank = rank;
  I.xranks = ranks;
  I.xfn = fn;
  I.xuser = user;
  if (ranks == 1) { I.xmode = 0; return true; }
  const size_t rec = kRecBytes;
  if (!I.xsend.alloc(rec, err) || !I.xrecv.alloc(rec * ranks, err)) return false;
  HIPCHK(hipMemset(I.xsend.p, 0, rec));
  if (mode == 1) {
    ncclUniqueId id;
    std::memcpy(&id, nccl_id, sizeof(id));
    HIPCHK(hipSetDevice(I.cfg.device));
    ncclResult_t nr = ncclCommInitRank(&I.comm, (int)ranks, id, (int)rank);
    if (nr != ncclSuccess) { err = std::string("ncclCommInitRank: ") + ncclGetErrorString(nr); return false; }
  } else if (mode == 2) {
    if (!fn) { err = "exchange: host mode needs a callback"; return false; }
    I.xfail.store(0);
  } else {
    err = "exchange: unknown mode";
    return false;
  }
  return tables_ready(I, err);  // class tables built before the exchange existed
}

uint32_t Engine::exchange_ranks() const { return p_->xranks; }
void Engine::path_counts(uint64_t out[8]) const {
  for (int i = 0; i < 6; ++i) out[i] = p_->path_pods[i];
  out[6] = p_->run_fallbacks + p_->win_fallbacks;
  out[7] = p_->win_runs;
}
bool Engine::lost() const { return p_->lost; }
uint64_t Engine::static_dec_chunks() const { return p_->static_dec_chunks; }
uint64_t Engine::static_overlaps() const { return p_->static_overlaps; }
void Engine::clear_lost() {
  Impl& I = *p_;
  if (I.rsync.p && (I.lost || I.run_used)) {  // (the sticky abort word: a call that failed before its sync left it set)
    (void)hipStreamSynchronize(I.stream);
    (void)hipMemset(I.rsync.p, 0, sizeof(RunSync));
    I.run_used = false;
  }
  I.lost = false;
}

bool Engine::nccl_unique_id(void* out128, std::string& err) {
  ncclUniqueId id;
  ncclResult_t nr = ncclGetUniqueId(&id);
  if (nr != ncclSuccess) { err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(nr); return false; }
  std::memcpy(out128, &id, sizeof(id));
  return true;
}
// Diagnostic (ksg_debug_rccl_selftest): the RCCL exchange's calls on this device
// with a ONE-rank communicator — unique id, ncclCommInitRank, ncclAllGather on a
// created stream, a byte-exact check of the gathered buffer, ncclCommDestroy.  A
// one-GPU box cannot hold two RCCL ranks (RCCL refuses a duplicate device), so
// this is the only RCCL call a single-GPU run can make; the sharded paths
// themselves are tested over the host exchange.
bool rccl_selftest(int device, size_t bytes, std::string& err) {
  HIPCHK(hipSetDevice(device));
  ncclUniqueId id;
  ncclResult_t nr = ncclGetUniqueId(&id);
  if (nr != ncclSuccess) { err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(nr); return false; }
  ncclComm_t comm = nullptr;
  nr = ncclCommInitRank(&comm, 1, id, 0);
  if (nr != ncclSuccess) { err = std::string("ncclCommInitRank: ") + ncclGetErrorString(nr); return false; }
  hipStream_t s = nullptr;
  uint8_t *a = nullptr, *b = nullptr;
  std::vector<uint8_t> h(bytes), back(bytes);
  for (size_t i = 0; i < bytes; ++i) h[i] = (uint8_t)(i * 131 + 7);
  bool ok = hipStreamCreate(&s) == hipSuccess && hipMalloc(&a, bytes) == hipSuccess && hipMalloc(&b, bytes) == hipSuccess &&
            hipMemcpyAsync(a, h.data(), bytes, hipMemcpyHostToDevice, s) == hipSuccess &&
            hipMemsetAsync(b, 0, bytes, s) == hipSuccess;
  if (!ok) err = "rccl selftest: buffers";
  if (ok && (nr = ncclAllGather(a, b, bytes, ncclUint8, comm, s)) != ncclSuccess) {
    err = std::string("ncclAllGather: ") + ncclGetErrorString(nr);
    ok = false;
  }
  if (ok && (hipMemcpyAsync(back.data(), b, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
             hipStreamSynchronize(s) != hipSuccess)) {
    err = "rccl selftest: copy back";
    ok = false;
  }
  if (ok && back != h) {
    err = "rccl selftest: gathered bytes differ";
    ok = false;
  }
  if (s) (void)hipStreamSynchronize(s);
  (void)ncclCommDestroy(comm);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  if (s) (void)hipStreamDestroy(s);
  return ok;
}
void Engine::set_path(int per_pod) { p_->force_per_pod = per_pod != 0; }
// The resource columns of the Fit / BalancedAllocation scoring arguments (known
// once the snapshot's resource vocabulary is: after every vocabulary build).
bool Engine::set_score_resources(const int32_t* fit_res, const int32_t* ba_res, std::string& err) {
  Impl& I = *p_;
  DevProfile& F = I.F;
  for (int i = 0; i < KSG_MAX_SCORE_RES; ++i) {
    F.fit_res[i] = fit_res[i];
    F.ba_res[i] = ba_res[i];
  }
  std::vector<int32_t> fr(F.fit_res, F.fit_res + KSG_MAX_SCORE_RES), br(F.ba_res, F.ba_res + KSG_MAX_SCORE_RES);
  std::vector<int64_t> fw(F.fit_w, F.fit_w + KSG_MAX_SCORE_RES);
  if (!I.fit_res_d.upload(fr, I.stream, err) || !I.ba_res_d.upload(br, I.stream, err) ||
      !I.fit_w_d.upload(fw, I.stream, err))
    return false;
  F.fit_res_d = I.fit_res_d.p;
  F.fit_w_d = I.fit_w_d.p;
  F.ba_res_d = I.ba_res_d.p;
  I.eval_mode = (F.fit_strategy == 0 && F.fit_n == 2 && F.fit_res[0] == 0 && F.fit_res[1] == 1 && F.fit_w[0] == 1 &&
                 F.fit_w[1] == 1 && F.ba_n == 2 && F.ba_res[0] == 0 && F.ba_res[1] == 1)
                    ? 1
                    : 0;
  return true;
}

bool Engine::eval_stamps(bool on, std::vector<uint64_t>* out, std::string& err) {
  Impl& I = *p_;  // table chain stamps (table_chain.hip CS_*): 64 slots
  if (!out) {
    I.cstamps_on = on;
    if (on) {
      if (!I.cstamps.alloc(64, err)) return false;
      HIPCHK(hipMemset(I.cstamps.p, 0, 64 * 8));
    }
    return true;
  }
  out->assign(64, 0);
  if (!stream_sync(I, I.stream, err)) return false;
  if (I.cstamps_on) HIPCHK(hipMemcpy(out->data(), I.cstamps.p, 64 * 8, hipMemcpyDeviceToHost));
  return true;
}

bool Engine::fixup_stamps(uint32_t count, std::vector<uint64_t>* out, std::string& err) {
  Impl& I = *p_;
  if (!out) {
    I.stamps_on = count > 0;
    if (count) {
      if (!I.stamps.alloc((size_t)(count + KSG_BATCH) * 8, err)) return false;
      HIPCHK(hipMemset(I.stamps.p, 0, (size_t)(count + KSG_BATCH) * 8 * 8));
    }
    return true;
  }
  out->resize((size_t)count * 8);
  HIPCHK(hipMemcpy(out->data(), I.stamps.p, out->size() * 8, hipMemcpyDeviceToHost));
  return true;
}
bool Engine::batch_path() const {
  const Impl& I = *p_;
  if (!I.batch_ok || I.force_per_pod || I.R > 4) return false;
  // node-sharded Taint / NodeAffinity windows: every rank holds every node's static data
  return !I.batch_static || (I.static_fits && (I.xranks <= 1 || I.gstat));
}

bool Engine::kernel_time(float& avg_ms, uint32_t& samples, std::string& err) {
  Impl& I = *p_;
  double tot = 0;
  for (uint32_t i = 0; i < I.n_samples; ++i) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, I.sev[2 * i], I.sev[2 * i + 1]));
    tot += ms;
  }
  samples = I.n_samples;
  avg_ms = I.n_samples ? (float)(tot / I.n_samples) : 0.f;
  return true;
}

bool Engine::static_time(float& total_ms, uint32_t& launches, uint64_t& pods, std::string& err) {
  Impl& I = *p_;
  double tot = 0;
  for (uint32_t i = 0; i < I.n_st; ++i) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, I.sev_st[2 * i], I.sev_st[2 * i + 1]));
    tot += ms;
  }
  total_ms = (float)tot;
  launches = I.n_st;
  pods = I.stat_pods_sampled;
  return true;
}
uint32_t Engine::n_nodes() const { return p_->N; }
void* Engine::stream() const { return p_->stream; }
float Engine::last_ms() const { return p_->last_ms; }
std::vector<Engine::KernelStat> Engine::kernel_stats() const { return p_->stats; }

}  // namespace ksg

// Diagnostic: lane-exchange / sort self-test on the device (tests/test_wave_ops_gpu.py).
extern "C" int ksg_debug_lane_selftest(int32_t* bad) {
  if (!bad) return -1;
  const int nb = 64;
  std::vector<uint64_t> h((size_t)nb * 64);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < h.size(); ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h[i] = (i % 5 == 0) ? (x & 0xFF) : x;  // duplicates and small values too
  }
  uint64_t* d = nullptr;
  int32_t* db = nullptr;
  if (hipMalloc((void**)&d, h.size() * 8) != hipSuccess) return -2;
  if (hipMalloc((void**)&db, 4) != hipSuccess) { (void)hipFree(d); return -2; }
  int rc = 0;
  if (hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice) != hipSuccess || hipMemset(db, 0, 4) != hipSuccess)
    rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(ksg::k_selftest_lanes, dim3(nb), dim3(64), 0, 0, d, db);
    hipLaunchKernelGGL(ksg::k_selftest_fold, dim3(nb / 4), dim3(256), 0, 0, d, db);  // (the same words, 256 a block)
    if (hipGetLastError() != hipSuccess || hipMemcpy(bad, db, 4, hipMemcpyDeviceToHost) != hipSuccess) rc = -2;
  }
  (void)hipFree(d);
  (void)hipFree(db);
  return rc;
}
