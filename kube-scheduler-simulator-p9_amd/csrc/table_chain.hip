// The table chain: one scheduling cycle in three launches for pods whose
// PodTopologySpread / InterPodAffinity inputs are read from the class tables
// (ksg_types.h "class tables"), and for every profile without those plugins.
// Included by engine.hip (shares its device helpers).
//
//   k_eval   one thread per node: the Filter chain in profile order (first
//            failure stops), every raw Score; per block a partial record
//            (feasible / ignored counts, status bits, the normalisers' max / min,
//            PodTopologySpread's registered domains) — no global atomics
//   k_ptsraw PodTopologySpread raw scores when the pod has several score
//            constraints (one constraint: max / min follow from the counts)
//   k_final  every block folds the partials, then per node: NormalizeScore,
//            [0,100] check, weights, packed argmax key; per block the best key;
//            the last-arriving block: selectHost over the block keys, the
//            summary, and the assume delta (node row, class tables; the
//            existing-pod table row is logged and written by k_flush_appends)
//   (a profile without ScoreExtensions: k_eval's last block selects)
//
// Every node's inputs are loaded up front (the row, the topology values, the
// class-table counts the pod reads, at offsets the program carries) so their
// latencies overlap; block reductions take one barrier.
// Upstream: schedule_one.go findNodesThatPassFilters / prioritizeNodes /
// selectHost, framework.go RunFilterPlugins / RunScorePlugins, the plugins'
// Filter / Score / NormalizeScore (restated in oracle/ksg_oracle.cpp).

// Threads per block of k_eval / k_ptsraw / k_final.  256 measured faster than
// 512 on cfg4 (32.4 vs 34.6 us per pod: the 8-wave block barriers cost more
// than the halved partial folds and block arrivals save).
constexpr int kChain = 256;
// A thread's topology values in the block's LDS image [KSG_MAX_TOPO][kChain].
template <int BT>
struct ChainVidsT {
  const int32_t* base;
  __device__ __forceinline__ int32_t operator()(int s) const { return base[s * BT]; }
};
using ChainVids = ChainVidsT<kChain>;

#define KCP_X_DECL 4
// The cycle view's device description (k_view; a fused view rides in ChainArgs)
struct ViewDev {
  int8_t prof_of_dev[KSG_MAX_PLUGINS];  // device position -> profile position (a volume run: its first plugin)
  uint8_t dev_vol[KSG_MAX_PLUGINS];     // the device position is a volume run
  int8_t norm_row[KSG_MAX_PLUGINS];     // device position -> normalized row, -1: none (output == raw)
  uint8_t kind[KSG_MAX_PROFILE];        // per profile position: the framework code of its Filter failure
  int32_t n_profile;
  uint32_t gen;  // this view's generation: a slot (or the overflow word) holds gen << 32 | code
  uint32_t off_sum, off_fail_pos, off_fail_code, off_fail_msg, off_raw, off_norm;  // byte offsets in the block
  uint32_t off_rows, n_norm;  // the score-row table (Engine::ViewRows); normalized rows
  uint32_t narrow;            // PodTopologySpread / InterPodAffinity raw rows sized by the summary's range
  uint32_t slots_direct;      // direct: slots written to the host block as claimed (no last-block copy)
};
struct EvalTotals;
struct SoloCand;
struct ChainArgs {
  const uint8_t* progs;
  const uint64_t* prog_off;
  uint32_t q;              // the cycle's queue pod and its program (per launch)
  const uint8_t* prog;
  ksg_pod_summary* sums;
  uint32_t keep_first, keep_n;
  uint32_t* kfilter;
  int32_t *kscore, *ktotal;
  uint32_t* filter;        // outputs of pods not kept
  int32_t *score, *total;
  uint32_t nblk;           // blocks of k_eval / k_ptsraw / k_final
  uint32_t need_eph;       // some pod requests a resource column beyond cpu / memory
  int32_t* pi;             // [KCP_I][nblk] feasible, ignored, status bits
  int64_t* pm;             // [2 * KCP_X][nblk] normaliser max / min per normalised plugin
  uint64_t* pr;            // [KSG_MAX_TSC][nblk] registered values of small score keys (bit = value)
  int64_t* pm2;            // [2][nblk] PodTopologySpread raw max / min (k_ptsraw)
  uint64_t* pk;            // [nblk] best key of the block (k_final, or k_eval without normalised plugins)
  int32_t* pst;            // [nblk] status bits of k_final
  int mode;                // commit mode (as k_commit)
  int32_t* prow;           // existing-pod table row of each queue pod
  int2* alog;              // per pod of the run since the last flush: (queue pod, local node or -1)
  uint32_t log_base;       // the run position alog[0] belongs to
  uint32_t* arrive;        // block arrivals of the cycle's last kernel (its last block selects)
  uint64_t* stamps;        // diagnostic (Engine::eval_stamps): block 0's s_memrealtime deltas, or null
  EvalTotals* etot;        // k_eval's partials folded once by k_fold (large clusters), or null: every block folds
  int64_t* xsend;          // node-sharded: the cycle's last block leaves its local (key, feasible, status) here
                           // for the X4 exchange instead of selecting (k_tx4_select selects), or null
  SoloCand* cand;          // [nblk][kChain] classes per block (k_eval_solo)
  // fused view (round 6): a kept pod of a profile without ScoreExtensions has its
  // cycle view written by k_eval itself -- every block its nodes' rows, the last
  // block the summary -- instead of by a k_view launch after it (vf_hout null: none)
  ViewDev vf;
  uint8_t* vf_out;         // the view's device block (message-slot table)
  uint8_t* vf_hout;        // the caller's pinned block, device address
};
__device__ __forceinline__ void view_fused_tail(const DevCluster& C, const DevProfile& F, const ChainArgs& A);

// Diagnostic stamps: block 0 / thread 0 of each chain kernel adds (now - entry)
// at its points (k_eval slots 0-7, k_ptsraw 8-15, k_final 16-23, its last block's select 24-27),
// entry-to-entry gaps k_eval->k_final 40, k_final->next k_eval 42 (last
// entries kept in 48-49), pods in 63.  100 MHz counter.
#define CS_ON (A.stamps && blockIdx.x == 0 && threadIdx.x == 0)
#define CS_BEGIN const uint64_t cs_t0 = CS_ON ? __builtin_amdgcn_s_memrealtime() : 0
#define CS(k) \
  if (CS_ON) atomicAdd((unsigned long long*)&A.stamps[k], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - cs_t0))
#define CS_GAP(gap, prev, mine)                                                                  \
  if (CS_ON) {                                                                                   \
    const uint64_t pv = A.stamps[prev];                                                          \
    if (pv) atomicAdd((unsigned long long*)&A.stamps[gap], (unsigned long long)(cs_t0 - pv));    \
    A.stamps[mine] = cs_t0;                                                                      \
  }

enum { KCP_FEAS = 0, KCP_IGN = 1, KCP_STAT = 2, KCP_IPAF = 3, KCP_CAND = 4, KCP_I = 5 };

// One-launch cycle (k_eval_solo, pods of normalising profiles whose outputs are
// not kept).  The total of a node is A + Σ_x w_x · NormalizeScore_x(raw_x), where
// A sums the plugins without ScoreExtensions and x runs over TaintToleration,
// NodeAffinity, PodTopologySpread and InterPodAffinity, whose normalisation
// needs the maxima over every feasible node.  Nodes with the same raw values of
// those plugins (a class) get the same normalised part, so the argmax of a
// class is its node with the largest packed key of A alone (pack_key(A) + part
// << 40 == pack_key(A + part)).  Each block keeps, per class met among its
// nodes, that best key (an LDS table of kSoloCap classes; a block meeting more
// dumps every feasible node as a class of its own); the last-arriving block
// folds the partials into the normalisers and picks the argmax over the
// classes: selectHost without a second pass over the nodes (k_final).
constexpr int kSoloCap = 64;  // classes per block before a dump (power of two)
struct SoloCand {
  int32_t v[KCP_X_DECL];      // raw scores per normalised slot (KCX_*), PTS -1: ignored node
  uint64_t key;               // pack_key(A) of the class's best node
};

// the chain kernels' arguments (DevCluster, DevProfile, ChainArgs, program) and the program header
constexpr int kArgBytes = (int)((sizeof(DevCluster) + sizeof(DevProfile) + sizeof(ChainArgs)) / 64 * 64);
constexpr int kHdrBytes = (int)(sizeof(ksg_prog) / 64 * 64);
__device__ __forceinline__ void chain_warm(const uint8_t* prog) {
  uint32_t warm = 0;
  KWarm<0, kArgBytes>::run((const void*)__builtin_amdgcn_kernarg_segment_ptr(), warm);
  KWarm<0, kHdrBytes>::run(prog, warm);
  warm_wait(warm);
}  // KCP_IPAF: block 0 only
enum { KCX_TAINT = 0, KCX_NA = 1, KCX_PTS = 2, KCX_IPA = 3, KCP_X = 4 };
static_assert(KCP_X == KCP_X_DECL, "SoloCand slots");
__device__ __forceinline__ int chain_x(int plugin) {
  return plugin == KP_TAINT ? KCX_TAINT : plugin == KP_NA ? KCX_NA : plugin == KP_PTS ? KCX_PTS
                                                                                      : plugin == KP_IPA ? KCX_IPA : -1;
}

__device__ __forceinline__ void chain_outs(const ChainArgs& A, uint32_t q, uint32_t N, uint32_t*& f, int32_t*& sc,
                                           int32_t*& tot) {
  if (A.keep_n && q >= A.keep_first && q < A.keep_first + A.keep_n) {
    const size_t k = q - A.keep_first;
    f = A.kfilter + k * N;
    sc = A.kscore + k * N * KSG_MAX_PLUGINS;
    tot = A.ktotal + k * N;
  } else {
    f = A.filter;
    sc = A.score;
    tot = A.total;
  }
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t m) {
  return (uint64_t)__ockl_wfred_or_u32((uint32_t)m) | ((uint64_t)__ockl_wfred_or_u32((uint32_t)(m >> 32)) << 32);
}
__device__ __forceinline__ int32_t wave_or(int32_t m) { return (int32_t)__ockl_wfred_or_u32((uint32_t)m); }

// The per-block / per-pod record the chain reduces.
struct ChainRec {
  int32_t feas, ign, st, pad;
  int64_t mx[KCP_X], mn[KCP_X];
  uint64_t reg[KSG_MAX_TSC];
  uint64_t key;
};
__device__ __forceinline__ void rec_init(ChainRec& r) {
  r.feas = r.ign = r.st = r.pad = 0;
#pragma unroll
  for (int x = 0; x < KCP_X; ++x) {
    r.mx[x] = INT64_MIN;
    r.mn[x] = INT64_MAX;
  }
#pragma unroll
  for (int c = 0; c < KSG_MAX_TSC; ++c) r.reg[c] = 0;
  r.key = 0;
}
// run-time slot x of a record's normaliser arrays without dynamic indexing
// (which would place the record in scratch)
__device__ __forceinline__ void rec_minmax(ChainRec& r, int x, int64_t v) {
#pragma unroll
  for (int i = 0; i < KCP_X; ++i)
    if (i == x) {
      r.mx[i] = v > r.mx[i] ? v : r.mx[i];
      r.mn[i] = v < r.mn[i] ? v : r.mn[i];
    }
}
__device__ __forceinline__ int64_t rec_mx(const ChainRec& r, int x) {
  int64_t v = INT64_MIN;
#pragma unroll
  for (int i = 0; i < KCP_X; ++i) v = i == x ? r.mx[i] : v;
  return v;
}
__device__ __forceinline__ int64_t rec_mn(const ChainRec& r, int x) {
  int64_t v = INT64_MAX;
#pragma unroll
  for (int i = 0; i < KCP_X; ++i) v = i == x ? r.mn[i] : v;
  return v;
}
// Block reduction of the record fields `what` names (RB_*; xmask / nreg: the
// normaliser slots / registration masks in use): wave folds on the DPP, one LDS
// record per wave, one barrier; every thread returns the block's record (the
// other fields keep their values).
enum { RB_CNT = 1, RB_CNT16 = 2, RB_ST = 4, RB_KEY = 8 };  // RB_CNT16: feas, ign < 2^15 per wave (one sum)
template <int TS = KSG_MAX_TSC, int BT = kChain>  // (TS: registration words a caller can have, nreg <= TS; BT: block threads)
__device__ __forceinline__ void rec_block(ChainRec& r, ChainRec* lds, uint32_t xmask, int nreg, uint32_t what,
                                          uint64_t* dbg = nullptr) {
  // dbg (diagnostic, one thread): time to the wave folds [0], the LDS record [1],
  // past the barrier [2], the end [61] (the eval-stamp slots that are free)
  const uint64_t rb0 = dbg ? __builtin_amdgcn_s_memrealtime() : 0;
#define RBS(i) \
  if (dbg) atomicAdd((unsigned long long*)&dbg[i], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - rb0))
  if (what & RB_CNT16) {
    const int32_t p = wave_sum(r.feas | (r.ign << 16));
    r.feas = p & 0xFFFF;
    r.ign = p >> 16;
  } else if (what & RB_CNT) {
    r.feas = wave_sum(r.feas);
    r.ign = wave_sum(r.ign);
  }
  if (what & RB_ST) r.st = wave_or(r.st);
  if (xmask) {
    // normalisers whose values (raw scores) all fit 32 bits reduce in one DPP pass
    // each instead of two (the unset sentinels map to the 32-bit extremes)
    bool wide = false;
#pragma unroll
    for (int x = 0; x < KCP_X; ++x)
      if ((xmask >> x) & 1u) {
        wide |= r.mx[x] != INT64_MIN && (r.mx[x] <= INT32_MIN || r.mx[x] >= INT32_MAX);
        wide |= r.mn[x] != INT64_MAX && (r.mn[x] <= INT32_MIN || r.mn[x] >= INT32_MAX);
      }
    if (__ballot(wide) == 0ull) {
#pragma unroll
      for (int x = 0; x < KCP_X; ++x)
        if ((xmask >> x) & 1u) {
          const int32_t a = wave_max(r.mx[x] == INT64_MIN ? INT32_MIN : (int32_t)r.mx[x]);
          const int32_t b = wave_min(r.mn[x] == INT64_MAX ? INT32_MAX : (int32_t)r.mn[x]);
          r.mx[x] = a == INT32_MIN ? INT64_MIN : (int64_t)a;
          r.mn[x] = b == INT32_MAX ? INT64_MAX : (int64_t)b;
        }
    } else {
#pragma unroll
      for (int x = 0; x < KCP_X; ++x)
        if ((xmask >> x) & 1u) {
          r.mx[x] = wave_max(r.mx[x]);
          r.mn[x] = wave_min(r.mn[x]);
        }
    }
  }
#pragma unroll
  for (int c = 0; c < TS; ++c)
    if (c < nreg) r.reg[c] = wave_or64(r.reg[c]);
  if (what & RB_KEY) r.key = wave_max(r.key);
  RBS(0);
  ChainRec* w = lds + (threadIdx.x >> 6);
  if (lane0()) {
    w->feas = r.feas;
    w->ign = r.ign;
    w->st = r.st;
#pragma unroll
    for (int x = 0; x < KCP_X; ++x)
      if ((xmask >> x) & 1u) {
        w->mx[x] = r.mx[x];
        w->mn[x] = r.mn[x];
      }
#pragma unroll
    for (int c = 0; c < TS; ++c)
      if (c < nreg) w->reg[c] = r.reg[c];
    w->key = r.key;
  }
  RBS(1);
  __syncthreads();
  RBS(2);
  const bool cnt = (what & (RB_CNT | RB_CNT16)) != 0;
  if (cnt) r.feas = r.ign = 0;
  if (what & RB_ST) r.st = 0;
#pragma unroll
  for (int i = 0; i < BT / 64; ++i) {
    const ChainRec* o = lds + i;
    if (cnt) {
      r.feas += o->feas;
      r.ign += o->ign;
    }
    if (what & RB_ST) r.st |= o->st;
#pragma unroll
    for (int x = 0; x < KCP_X; ++x)
      if ((xmask >> x) & 1u) {
        r.mx[x] = o->mx[x] > r.mx[x] ? o->mx[x] : r.mx[x];
        r.mn[x] = o->mn[x] < r.mn[x] ? o->mn[x] : r.mn[x];
      }
#pragma unroll
    for (int c = 0; c < TS; ++c)
      if (c < nreg) r.reg[c] |= o->reg[c];
    if (what & RB_KEY) r.key = o->key > r.key ? o->key : r.key;
  }
  RBS(61);
#undef RBS
}

// ---- Interleaved wave folds (round 5).  rec_block folds each field with its own
// wave reduction (ockl wfred: DPP steps, each waiting for the previous one, plus
// the hazard nops), one field after the other: at one wave per SIMD the eight
// folds of a cfg4 record took ~0.8 us and reading the four wave records back
// ~0.7 us (stamps, profiles/r05_*).  fold_block runs the DPP steps of ALL fields
// together (one step's latency paid once for every field: the other fields'
// instructions fill the hazard slots), then one LDS row of words per wave, one
// barrier and one read sweep.  Fields are 32-bit words; every lane of the block
// takes part (no divergent caller).
enum { FO_ADD = 0, FO_MAXI = 1, FO_MINI = 2, FO_OR = 3, FO_MAXU = 4 };
template <int OP>
__device__ __forceinline__ uint32_t fo(uint32_t a, uint32_t b) {
  if constexpr (OP == FO_ADD) return a + b;
  else if constexpr (OP == FO_MAXI) return (uint32_t)((int32_t)a > (int32_t)b ? (int32_t)a : (int32_t)b);
  else if constexpr (OP == FO_MINI) return (uint32_t)((int32_t)a < (int32_t)b ? (int32_t)a : (int32_t)b);
  else if constexpr (OP == FO_OR) return a | b;
  else return a > b ? a : b;
}
template <int OP>
__device__ __forceinline__ constexpr uint32_t fo_id() {
  return OP == FO_MAXI ? 0x80000000u : OP == FO_MINI ? 0x7FFFFFFFu : 0u;
}
// one DPP step of a fold: lanes without a source in the pattern (bound_ctrl off, or
// rows the row mask leaves out) see the identity
template <int OP, int CTRL, int RM>
__device__ __forceinline__ uint32_t fo_step(uint32_t v) {
  return fo<OP>(v, (uint32_t)__builtin_amdgcn_update_dpp((int)fo_id<OP>(), (int)v, CTRL, RM, 0xF, false));
}
template <int... OPS>
struct WFold {
  static constexpr int K = sizeof...(OPS);
  template <int CTRL, int RM, size_t... I>
  static __device__ __forceinline__ void step_(uint32_t (&v)[K], std::index_sequence<I...>) {
    ((v[I] = fo_step<OPS, CTRL, RM>(v[I])), ...);
  }
  template <int CTRL, int RM>
  static __device__ __forceinline__ void step(uint32_t (&v)[K]) {
    step_<CTRL, RM>(v, std::make_index_sequence<K>{});
  }
  template <size_t... I>
  static __device__ __forceinline__ void cross_(uint32_t (&v)[K], const uint32_t* row, std::index_sequence<I...>) {
    ((v[I] = fo<OPS>(v[I], row[I])), ...);
  }
  // the wave's fold: row_shr 1, 2, 4, 8 (a row's total in its lane 15), then
  // row_bcast 15 / 31 (the wave's total in lane 63), read back as uniform values
  static __device__ __forceinline__ void wave(uint32_t (&v)[K]) {
    step<0x111, 0xF>(v);
    step<0x112, 0xF>(v);
    step<0x114, 0xF>(v);
    step<0x118, 0xF>(v);
    step<0x142, 0xA>(v);
    step<0x143, 0xC>(v);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = (uint32_t)__builtin_amdgcn_readlane((int)v[k], 63);
  }
  // the block's fold: wave folds, one row of K words per wave in LDS (stride 16
  // words), one barrier, every thread folds the rows.  lds: NW * 16 words.
  template <int NW>
  static __device__ __forceinline__ void block(uint32_t (&v)[K], uint32_t* lds) {
    static_assert(K <= 16, "fold row");
    wave(v);
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) lds[(threadIdx.x >> 6) * 16 + k] = v[k];
    }
    __syncthreads();
    uint32_t row[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = lds[k];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
#pragma unroll
      for (int k = 0; k < K; ++k) row[k] = lds[w * 16 + k];
      cross_(v, row, std::make_index_sequence<K>{});
    }
  }
};
// N signed minima then one OR (eval_body's pod-uniform setup)
template <int N, int... OPS>
struct MinsThenOr : MinsThenOr<N - 1, FO_MINI, OPS...> {};
template <int... OPS>
struct MinsThenOr<0, OPS...> {
  using W = WFold<OPS..., FO_OR>;
};
// int64 normaliser fields as 32-bit words (callers checked the values fit): the
// unset sentinels map to the 32-bit extremes and back
__device__ __forceinline__ uint32_t mx32(int64_t v) { return v == INT64_MIN ? 0x80000000u : (uint32_t)(int32_t)v; }
__device__ __forceinline__ uint32_t mn32(int64_t v) { return v == INT64_MAX ? 0x7FFFFFFFu : (uint32_t)(int32_t)v; }
__device__ __forceinline__ int64_t mx64(uint32_t v) { return v == 0x80000000u ? INT64_MIN : (int64_t)(int32_t)v; }
__device__ __forceinline__ int64_t mn64(uint32_t v) { return v == 0x7FFFFFFFu ? INT64_MAX : (int64_t)(int32_t)v; }
__device__ __forceinline__ bool fits32(const ChainRec& r, int x) {
  return (r.mx[x] == INT64_MIN || (r.mx[x] > INT32_MIN && r.mx[x] < INT32_MAX)) &&
         (r.mn[x] == INT64_MAX || (r.mn[x] > INT32_MIN && r.mn[x] < INT32_MAX));
}
// The persistent chain's record folds (rec_block's results, fast): a partial
// record with the counts, status, the normalisers of slots XA / XB (KCX_*) and one
// registration word — what a table-chain pod of k_chain_run's size class reduces
// (<= 1 PodTopologySpread score constraint; cfg4's PodTopologySpread +
// InterPodAffinity); the generic rec_block when a normaliser needs 64 bits.
template <int XA, int XB, int BT>
__device__ __forceinline__ void fold_partial(ChainRec& r, ChainRec* lds, uint32_t xmask, int nreg, bool cnt16) {
  bool wide = false;
  if ((xmask >> XA) & 1u) wide |= !fits32(r, XA);
  if ((xmask >> XB) & 1u) wide |= !fits32(r, XB);
  // (the choice is the block's: a barrier-OR, which also orders the rows' reuse)
  if (__syncthreads_or(wide) || nreg > 1 || (xmask & ~((1u << XA) | (1u << XB)))) {
    rec_block<KSG_MAX_TSC, BT>(r, lds, xmask, nreg, (cnt16 ? RB_CNT16 : RB_CNT) | RB_ST);
    return;
  }
  uint32_t v[9] = {(uint32_t)r.feas, (uint32_t)r.ign, (uint32_t)r.st, mx32(r.mx[XA]), mn32(r.mn[XA]), mx32(r.mx[XB]),
                   mn32(r.mn[XB]), nreg ? (uint32_t)r.reg[0] : 0u, nreg ? (uint32_t)(r.reg[0] >> 32) : 0u};
  WFold<FO_ADD, FO_ADD, FO_OR, FO_MAXI, FO_MINI, FO_MAXI, FO_MINI, FO_OR, FO_OR>::block<BT / 64>(
      v, reinterpret_cast<uint32_t*>(lds));
  r.feas = (int32_t)v[0];
  r.ign = (int32_t)v[1];
  r.st = (int32_t)v[2];
  if ((xmask >> XA) & 1u) { r.mx[XA] = mx64(v[3]); r.mn[XA] = mn64(v[4]); }
  if ((xmask >> XB) & 1u) { r.mx[XB] = mx64(v[5]); r.mn[XB] = mn64(v[6]); }
  if (nreg) r.reg[0] = (uint64_t)v[7] | ((uint64_t)v[8] << 32);
}
// The key folds: status (or) and the 64-bit best key (its high word, then the low
// word among the lanes holding the winning high word).
template <int BT>
__device__ __forceinline__ void fold_key(ChainRec& r, ChainRec* lds) {
  __syncthreads();  // (lds reused)
  uint32_t* w = reinterpret_cast<uint32_t*>(lds);
  uint32_t v[2] = {(uint32_t)r.st, (uint32_t)(r.key >> 32)};
  WFold<FO_OR, FO_MAXU>::wave(v);
  uint32_t lo[1] = {(uint32_t)(r.key >> 32) == v[1] ? (uint32_t)r.key : 0u};
  WFold<FO_MAXU>::wave(lo);
  if ((threadIdx.x & 63) == 0) {
    w[(threadIdx.x >> 6) * 16 + 0] = v[0];
    w[(threadIdx.x >> 6) * 16 + 1] = v[1];
    w[(threadIdx.x >> 6) * 16 + 2] = lo[0];
  }
  __syncthreads();
  uint32_t st = 0, hi = 0, l = 0;
#pragma unroll
  for (int i = 0; i < BT / 64; ++i) {
    const uint32_t s0 = w[i * 16], h0 = w[i * 16 + 1], l0 = w[i * 16 + 2];
    st |= s0;
    if (h0 > hi || (h0 == hi && l0 > l)) { hi = h0; l = l0; }
  }
  r.st = (int32_t)st;
  r.key = ((uint64_t)hi << 32) | l;
}

// Self-test of the interleaved folds (ksg_debug_lane_selftest): a block fold of
// every operation against LDS atomics, and the key fold against a plain scan.
__global__ __launch_bounds__(256) void k_selftest_fold(const uint64_t* in, int32_t* bad) {
  __shared__ uint32_t rows[4 * 16];
  __shared__ uint32_t ref[5];
  __shared__ ChainRec lrec[4];
  __shared__ unsigned long long kref;
  const uint64_t x = in[blockIdx.x * 256 + threadIdx.x];
  const uint32_t a = (uint32_t)x, b = (uint32_t)(x >> 32);
  if (threadIdx.x == 0) {
    ref[0] = 0; ref[1] = 0x80000000u; ref[2] = 0x7FFFFFFFu; ref[3] = 0; ref[4] = 0;
    kref = 0;
  }
  __syncthreads();
  atomicAdd(&ref[0], a & 0xFFFu);
  atomicMax((int*)&ref[1], (int)a);
  atomicMin((int*)&ref[2], (int)b);
  atomicOr(&ref[3], a & 0xF0F0u);
  atomicMax(&ref[4], b);
  atomicMax(&kref, (unsigned long long)(x & ~0xFull));
  __syncthreads();
  uint32_t v[5] = {a & 0xFFFu, a, b, a & 0xF0F0u, b};
  WFold<FO_ADD, FO_MAXI, FO_MINI, FO_OR, FO_MAXU>::block<4>(v, rows);
  int e = 0;
  for (int k = 0; k < 5; ++k) e += v[k] != ref[k];
  ChainRec r;
  rec_init(r);
  r.key = x & ~0xFull;
  r.st = (int32_t)(a & 3u);
  fold_key<256>(r, lrec);
  e += r.key != kref;
  atomicAdd(bad, e);
}

// PodTopologySpread score count of constraint c at local node n (its pair's
// TopologyPairToPodCounts, or the node's own count for the hostname key).
__device__ __forceinline__ int64_t pts_count_tab(const DevCluster& C, const ProgView& V, int c, uint32_t n, int32_t v) {
  const ksg_tsc& t = V.h->tsc[c];
  if (t.is_hostname) return t.cls < 0 ? 0 : C.T.pc_cnt[(size_t)t.cls * C.N + n];
  int64_t s = 0;
  for (int k = 0; k < t.sc_n; ++k) s += pc_count(C, V.i32[t.sc_off + k], t.nub, n, v);
  return s;
}

template <int BT>
struct EvalSharedT {
  int32_t tv[KSG_MAX_TOPO * BT];
  uint32_t setup[BT / 64 * 16];  // eval_body's setup fold (rows of its own: rec's may still be read)
  ChainRec rec[BT / 64];
};
using EvalShared = EvalSharedT<kChain>;

// The assume delta's node row as fire-and-forget atomics (no load on the
// chain's critical path).
__device__ __forceinline__ void assume_row_atomic(DevCluster& C, const ProgView& V, uint32_t n, int sign) {
  const ksg_prog* h = V.h;
  for (uint32_t r = 0; r < C.R; ++r)
    if (h->req[r]) atomicAdd((unsigned long long*)&C.req[(size_t)r * C.N + n], (unsigned long long)(sign * h->req[r]));
  atomicAdd((unsigned long long*)&C.nzc[n], (unsigned long long)(sign * h->nz_cpu));
  atomicAdd((unsigned long long*)&C.nzm[n], (unsigned long long)(sign * h->nz_mem));
  atomicAdd(&C.podcnt[n], sign);
  for (int i = 0; i < h->n_port_own; ++i) atomicAdd(&C.ports[(size_t)V.i32[h->port_own_off + i] * C.N + n], sign);
  for (int i = 0; i < h->n_pvc; ++i) atomicAdd(&C.pvcuse[V.i32[h->pvc_off + i]], sign);
  csi_assume(C, V, n, sign);
}

// selectHost's outcome (the argmax key over every feasible node, the feasible
// count, status bits) → the summary and the assume delta, by the whole block
// (the last wave writes the summary and the node row, every lane the class tables).
__device__ __forceinline__ int32_t chain_commit(DevCluster& C, const ChainArgs& A, const ProgView& V, uint64_t key,
                                                int32_t feas, int32_t st, uint64_t cs_t0) {
  const ksg_prog* h = V.h;
  const uint32_t q = A.q;
  const bool error = (st & 2) || ((st & 4) && feas > 1) || (h->flags & KPF_PREFILTER_ERROR) ||
                     na_prescore_error(h->flags, feas);
  int32_t node = -1;
  const uint32_t g = (uint32_t)(key & 0xFFFFFull);
  if (!error && feas > 0 && (A.mode & 1) && g >= C.goff && g - C.goff < C.N) node = (int32_t)(g - C.goff);
  if (threadIdx.x == blockDim.x - 64) {  // (the last wave: wave 0 takes the class tables meanwhile)
    __hip_atomic_store(A.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ksg_pod_summary* S = A.sums + q;
    S->feasible = feas;
    S->best_key = key;
    if (error) { S->status = 2; S->selected = -1; }
    else if (feas == 0) { S->status = 1; S->selected = -1; }
    else { S->status = 0; S->selected = (int32_t)g; }
    A.prow[q] = -1;
    // the existing-pod table row: written after the run (k_flush_appends)
    A.alog[q - A.log_base] = make_int2((int)q, node >= 0 && (A.mode & 2) ? node : -1);
    if (node >= 0) assume_row_atomic(C, V, (uint32_t)node, +1);
  }
  CS(26);
  if (node >= 0) tables_assume(C, V, (uint32_t)node, +1, threadIdx.x, blockDim.x);
  CS(27);
  if (CS_ON) atomicAdd((unsigned long long*)&A.stamps[63], 1ull);
  return node;
}

// selectHost + the assume, by the last-arriving block of the cycle's last
// kernel: the block keys / statuses were stored sc1 before each block arrived
// (MI355X_MICROARCH.md hand-off: agent-scope stores, counter, agent-scope loads).
__device__ __forceinline__ void chain_last_select(DevCluster& C, const DevProfile& F, const ChainArgs& A, ChainRec* lds,
                                                  const uint8_t* __restrict__ prog) {
  __shared__ uint32_t last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(A.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last) return;
  const uint64_t cs_t0 = CS_ON ? __builtin_amdgcn_s_memrealtime() : 0;
  const uint32_t q = A.q, NB = A.nblk;
  const ProgView V = view(prog);
  const ksg_prog* h = V.h;
  ChainRec r;
  rec_init(r);
  for (uint32_t b = threadIdx.x; b < NB; b += blockDim.x) {
    const uint64_t k = ld_sc1(A.pk + b);
    r.key = k > r.key ? k : r.key;
    r.feas += ld_sc1(A.pi + KCP_FEAS * NB + b);
    r.st |= ld_sc1(A.pi + KCP_STAT * NB + b) | ld_sc1(A.pst + b);
  }
  CS(24);
  rec_block(r, lds, 0u, 0, RB_CNT | RB_ST | RB_KEY);
  CS(25);
  if (A.xsend) {  // node-sharded: this rank's part of selectHost goes to the X4 exchange
    if (threadIdx.x == 0) {
      __hip_atomic_store(A.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      A.xsend[0] = (int64_t)r.key;
      A.xsend[1] = r.feas;
      A.xsend[2] = r.st;
    }
    return;
  }
  chain_commit(C, A, V, r.key, r.feas, r.st, cs_t0);
  if (A.vf_hout) {  // (a fused view: the summary is out, its copy and the row table follow)
    __syncthreads();
    view_fused_tail(C, F, A);
  }
}

// ROWM: 0 resource columns read by the plugins (more than 4 columns), 1 the
// node row loaded up front (RowV), 2 the same with the default Fit / BA
// arguments compiled in.
struct SoloShared {
  uint32_t tag[kSoloCap], ready[kSoloCap];
  int32_t v[kSoloCap][KCP_X];
  unsigned long long best[kSoloCap];
  uint32_t wcnt[kChain / 64];
  uint32_t dump, count;
};
__device__ void solo_last_select(DevCluster& C, const DevProfile& F, const ChainArgs& A, ChainRec* lds,
                                 const uint8_t* __restrict__ prog, uint32_t ipa_flags, uint64_t cs_t0);
__device__ __forceinline__ uint32_t solo_hash(int32_t a, int32_t b, int32_t c, int32_t d) {
  uint32_t h = 0x9E3779B9u;
  h = (h ^ (uint32_t)a) * 0x85EBCA6Bu;
  h = (h ^ (uint32_t)b) * 0xC2B2AE35u;
  h = (h ^ (uint32_t)c) * 0x27D4EB2Fu;
  h = (h ^ (uint32_t)d) * 0x165667B1u;
  return (h ^ (h >> 15)) | 1u;
}
// One lane of a wave: class (a, b, c, d) with best key `best` into the block's
// LDS table (claim by CAS on the tag; a wave meeting a claimed tag waits for the
// claimer's values, then compares them).  A full table sets dump.
__device__ __forceinline__ void solo_insert(SoloShared& S, int32_t a, int32_t b, int32_t c, int32_t d, uint64_t best) {
  const uint32_t t = solo_hash(a, b, c, d);
  for (int k = 0; k < kSoloCap; ++k) {
    const int i = (int)((t + (uint32_t)k) & (kSoloCap - 1));
    const uint32_t old = atomicCAS(&S.tag[i], 0u, t);
    if (old == 0u) {
      S.v[i][0] = a;
      S.v[i][1] = b;
      S.v[i][2] = c;
      S.v[i][3] = d;
      __threadfence_block();
      atomicExch(&S.ready[i], 1u);
      atomicMax(&S.best[i], (unsigned long long)best);
      return;
    }
    if (old == t) {
      while (__hip_atomic_load(&S.ready[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
      }
      __threadfence_block();
      if (S.v[i][0] == a && S.v[i][1] == b && S.v[i][2] == c && S.v[i][3] == d) {
        atomicMax(&S.best[i], (unsigned long long)best);
        return;
      }
    }
  }
  atomicOr(&S.dump, 1u);
}
__device__ __forceinline__ void st_cand(SoloCand* p, const int32_t v[KCP_X], uint64_t key) {
  uint64_t* w = reinterpret_cast<uint64_t*>(p);
  st_sc1(w, (uint64_t)(uint32_t)v[0] | ((uint64_t)(uint32_t)v[1] << 32));
  st_sc1(w + 1, (uint64_t)(uint32_t)v[2] | ((uint64_t)(uint32_t)v[3] << 32));
  st_sc1(w + 2, key);
}

// What one node's evaluation leaves for the persistent chain (MODE kRun): its raw
// scores per profile position, feasibility, and the block's reduced record.
struct EvalOut {
  bool abort;                    // a poll ran out (k_chain_run leaves)
  int32_t raw[KSG_MAX_PLUGINS];  // (as k_final reads them back from the per-pair scores)
  bool feasible;
  uint32_t ipa_flags;
  ChainRec rec;
};
enum { kEval = 0, kSolo = 1, kRun = 2 };  // eval_body modes: k_eval, k_eval_solo, k_chain_run
// k_chain_run's evaluation in two stages (eval_body STG): 1 issues every
// class-table read of the node (the lookup plan, minMatchNum candidates,
// InterPodAffinity map totals) and leaves the values in flight in an EvalPre;
// 2 finishes from it (row-only plugins on the row as of then, filters, scores,
// the block's record).  0: both at once.
struct EvalPre {
  int32_t lkv[KSG_LK_MAX], lks[KSG_LK_MAX];
  uint8_t mpn[KSG_MAX_TSC];
  int32_t mcnt[KSG_MAX_TSC];
  int32_t ubv;
  uint32_t ubbit;
};
// Class-table reads: plain loads in a launch of one cycle; in the persistent chain
// the tables change under the launch (other blocks' assumes), so every read is an
// agent-scope (sc1) load of what the assuming block wrote by atomics
// (MI355X_MICROARCH.md hand-off table, row 3).
template <int MODE>
__device__ __forceinline__ int32_t ld_tab(const int32_t* p) {
  if constexpr (MODE == kRun) return ld_sc1(p);
  else return *p;
}
// PM: the plugins the kernel is compiled for (bit KP_*; ~0u every one).  A launch
// whose profile uses a subset runs a specialisation without the other plugins'
// code: the generic evaluation is ~75-130 KB of code, beyond the 64 KB
// instruction cache two CUs share, and misses it on every cycle.
#define PMH(p) ((PM >> (p)) & 1u)
// Device positions a kernel specialised on plugin set PM can see (the host picks
// such a kernel only when the profile's positions are PM's plugins, each once):
// the per-position loops unroll that many times instead of KSG_MAX_PLUGINS.
template <uint32_t PM>
constexpr int kNPos = PM == ~0u ? KSG_MAX_PLUGINS
                                : (__builtin_popcount(PM) < KSG_MAX_PLUGINS ? __builtin_popcount(PM) : KSG_MAX_PLUGINS);
// k_chain_run: the flag this block waits for before its class-table reads (the
// previous pod's assume by the block owning its node; want 0: none)
struct RunWait;
__device__ bool run_wait_flag(const RunWait& W);
// LK / TS: the lookup-plan entries and spread constraints a pod of the launch has
// at most (k_chain_run size classes; smaller unrolled loops, less code).
// The row-only plugins of a persistent-chain pod computed ahead, during the
// previous pod's key hand-off (k_chain_run): Fit's filter bits, Fit's and
// BalancedAllocation's raw scores on the row as of then (the owner of the
// previous pod's node recomputes that node's after its assume).
struct RowPre {
  uint32_t fb;
  int64_t fs, bs;
};
template <int ROWM, uint32_t PM, class P>
__device__ __forceinline__ void row_pre(const RowV& row, const DevProfile& F, const P* h, uint32_t R, RowPre& o) {
  o.fb = 0;
  o.fs = o.bs = 0;
  if (PMH(KP_FIT)) {
    o.fb = fit_filter_row(row, h, R);
    o.fs = ROWM == 2 ? fit_score_row<1>(row, F, h) : fit_score_row<0>(row, F, h);
  }
  if (PMH(KP_BA)) o.bs = ROWM == 2 ? ba_score_row<1>(row, F, h) : ba_score_row<0>(row, F, h);
}
template <int ROWM, int MODE = kEval, uint32_t PM = ~0u, int LK = KSG_LK_MAX, int TS = KSG_MAX_TSC, int BT = kChain,
          int STG = 0>
__device__ __forceinline__ void eval_body(DevCluster& C, const DevProfile& F, const ChainArgs& A,
                                          const uint8_t* __restrict__ prog, EvalSharedT<BT>* Lrun = nullptr,
                                          RowV* rowrun = nullptr, EvalOut* eo = nullptr, const RunWait* W = nullptr,
                                          EvalPre* pre = nullptr, const RowPre* rp = nullptr) {
  constexpr bool SOLO = MODE == kSolo, RUN = MODE == kRun;
  static_assert(STG == 0 || RUN, "staged evaluation: the persistent chain only");
  static_assert(BT == kChain || RUN, "other block sizes: the persistent chain only");
  if constexpr (!RUN) chain_warm(prog);
  CS_BEGIN;
  CS_GAP(42, 49, 48);
  CS(13);
  const uint32_t q = A.q;
  const ProgView V = view(prog);
  const ksg_prog* h = V.h;
  EvalSharedT<BT>* Lp;  // (k_chain_run: the caller's)
  if constexpr (RUN) {
    Lp = Lrun;
  } else {
    __shared__ EvalSharedT<BT> Lown;
    Lp = &Lown;
  }
  EvalSharedT<BT>& L = *Lp;
  uint32_t* of;
  int32_t *os, *ot;
  chain_outs(A, q, C.N, of, os, ot);
  const uint32_t n = blockIdx.x * BT + threadIdx.x;
  const bool active = n < C.N;
  const uint32_t nn = active ? n : 0;  // loads of inactive lanes read node 0 (results unused)
  int pts_pos = -1, ipa_pos = -1;
  uint32_t xmask = 0;
  for (int p = 0; p < F.n; ++p) {
    if (PMH(KP_PTS) && F.plugins[p] == KP_PTS) pts_pos = p;
    if (PMH(KP_IPA) && F.plugins[p] == KP_IPA) ipa_pos = p;
    const int x = chain_x(F.plugins[p]);
    if (x >= 0) xmask |= 1u << x;
  }
  const int nf = h->n_tsc_filter, ns = h->n_tsc_score;
  const bool pts_f = pts_pos >= 0 && !(h->flags & KPF_SKIP_PTS_FILTER);
  const bool pts_score = pts_pos >= 0 && ns > 0 && !(h->flags & KPF_SKIP_PTS_SCORE);
  // ---- every input in flight together: the node's topology values first (the
  // class-table reads need them), its row, then the pod-uniform setup inputs
  // (minMatchNum candidates: value tid of each filter key; InterPodAffinity map
  // totals: plan entry tid).  Consumed only after the lookups are issued.
  const uint32_t ntopo = C.n_topo < KSG_MAX_TOPO ? C.n_topo : KSG_MAX_TOPO;
  int32_t vid[KSG_MAX_TOPO];
  if constexpr (!RUN) node_slot_vids(C, nn, vid);  // (k_chain_run: in L.tv for the whole run)
  RowV rowl;
  RowV& row = RUN ? *rowrun : rowl;
  if (ROWM && !RUN) load_row(C, nn, A.need_eph, row);
  // the row-only plugins (Fit filter, Fit / BalancedAllocation scores) computed
  // before the class-table reads: in k_chain_run their compute overlaps the wait
  // for the previous pod's assume (the rows of this block's nodes are final: only
  // the owner's changes, in its own registers)
  uint32_t fit_b = 0;
  int64_t fit_s = 0, ba_s = 0;
  if constexpr (RUN && ROWM != 0) {
    if (rp) {  // (computed during the previous pod's key hand-off)
      fit_b = rp->fb;
      fit_s = rp->fs;
      ba_s = rp->bs;
    } else if (STG != 1) {  // (staged: on the row as of the finish)
      if (PMH(KP_FIT)) {
        fit_b = fit_filter_row(row, h, C.R);
        fit_s = ROWM == 2 ? fit_score_row<1>(row, F, h) : fit_score_row<0>(row, F, h);
      }
      if (PMH(KP_BA)) ba_s = ROWM == 2 ? ba_score_row<1>(row, F, h) : ba_score_row<0>(row, F, h);
    }
    CS(14);
    if (STG != 2 && W && !run_wait_flag(*W)) {
      eo->abort = true;
      return;
    }
    CS(15);
  }
  uint8_t mpn[KSG_MAX_TSC];
  int32_t mcnt[KSG_MAX_TSC];
#pragma unroll
  for (int c = 0; c < TS; ++c) {
    mpn[c] = 0;
    mcnt[c] = 0;
    if constexpr (STG == 2) {
      mpn[c] = pre->mpn[c];
      mcnt[c] = pre->mcnt[c];
    } else if (pts_f && c < nf && threadIdx.x < (uint32_t)h->tsc[c].nvals) {
      const ksg_tsc& t = h->tsc[c];
      mpn[c] = C.T.pair_node[t.pair_base + threadIdx.x];
      if (t.eff_cls >= 0) mcnt[c] = ld_tab<MODE>(C.T.pc_dom + (size_t)t.eff_cls * C.T.NU + (uint32_t)t.nub + threadIdx.x);
    }
  }
  int32_t ubv = 0;
  uint32_t ubbit = 0;
  if constexpr (STG == 2) {
    ubv = pre->ubv;
    ubbit = pre->ubbit;
  } else if (ipa_pos >= 0 && h->n_ub > 0) {  // entry tid of the plan (uniform reads, then a per-lane pick)
    int32_t idx = 0, kind = 0;
#pragma unroll
    for (int i = 0; i < KSG_UB_MAX; ++i) {
      const int32_t ei = h->ub[i].idx, ek = h->ub[i].kind, eb = h->ub[i].bit;
      if (threadIdx.x == (uint32_t)i) {
        idx = ei;
        kind = ek;
        ubbit = (uint32_t)eb;
      }
    }
    if (threadIdx.x < (uint32_t)h->n_ub) ubv = ld_tab<MODE>(kind == 1 ? C.T.pc_tot + idx : C.T.tc_tot + idx);
  }
  CS(7);
  CS(11);
  CS(12);
  if constexpr (!RUN) {
#pragma unroll
    for (int s = 0; s < KSG_MAX_TOPO; ++s)
      if ((uint32_t)s < ntopo) L.tv[s * BT + threadIdx.x] = vid[s];
  }
  const ChainVidsT<BT> tv{L.tv + threadIdx.x};  // (each thread reads back only its own column)
  CS(8);
  // ---- the lookup plan (ksg_look): every class-table count of this node
  int32_t lkv[KSG_LK_MAX], lks[KSG_LK_MAX];
#pragma unroll
  for (int i = 0; i < LK; ++i) {
    lkv[i] = 0;
    lks[i] = -1;
    if constexpr (STG == 2) {
      lkv[i] = pre->lkv[i];
      lks[i] = pre->lks[i];
    } else if (i < h->n_lk) {
      const ksg_look& e = h->lk[i];
      const uint32_t sku = e.sku;
      const int32_t kind = ksg_lk_kind(sku);
      const int32_t v = tv(ksg_lk_slot(sku));
      lks[i] = v;
      if (kind != KLK_NONE) {
        const uint32_t at = (uint32_t)e.base + ((kind == KLK_PC_NODE || kind == KLK_TC_NODE) ? nn : (uint32_t)(v < 0 ? 0 : v));
        lkv[i] = ld_tab<MODE>((kind == KLK_PC_NODE ? C.T.pc_cnt : kind == KLK_PC_DOM ? C.T.pc_dom : C.T.tc_val) + at);
      }
    }
  }
  CS(9);
  if constexpr (STG == 1) {  // the reads are in flight: the caller finishes later (STG 2)
#pragma unroll
    for (int i = 0; i < LK; ++i) {
      pre->lkv[i] = lkv[i];
      pre->lks[i] = lks[i];
    }
#pragma unroll
    for (int c = 0; c < TS; ++c) {
      pre->mpn[c] = mpn[c];
      pre->mcnt[c] = mcnt[c];
    }
    pre->ubv = ubv;
    pre->ubbit = ubbit;
    return;
  }
  // ---- pod-uniform setup: minMatchNum per filter constraint, InterPodAffinity
  // bits — one interleaved block fold (one barrier; the results uniform in registers)
  uint32_t su[TS + 1];
#pragma unroll
  for (int c = 0; c < TS; ++c) {
    int32_t m = 0x7FFFFFFF;
    if (pts_f && c < nf) {
      const ksg_tsc& t = h->tsc[c];
      if (threadIdx.x < (uint32_t)t.nvals && mpn[c]) m = mcnt[c];
      for (uint32_t i = threadIdx.x + BT; i < (uint32_t)t.nvals; i += BT)  // keys beyond one value per thread
        if (C.T.pair_node[t.pair_base + i]) {
          const int32_t x = t.eff_cls < 0 ? 0 : ld_tab<MODE>(C.T.pc_dom + (size_t)t.eff_cls * C.T.NU + (uint32_t)t.nub + i);
          m = x < m ? x : m;
        }
    }
    su[c] = (uint32_t)m;
  }
  su[TS] = ipa_pos >= 0 && ubv > 0 ? ubbit : 0u;
  MinsThenOr<TS>::W::template block<BT / 64>(su, L.setup);
  CS(10);
  // ---- the counts, folded into what the filters and scores read
  int32_t ptsm[KSG_MAX_TSC];
#pragma unroll
  for (int c = 0; c < TS; ++c) ptsm[c] = 0;
  int64_t pts_cnt = 0, ipa_raw = 0;
  bool aff_miss = false, aff_zero = false, anti_hit = false, exist_hit = false;
#pragma unroll
  for (int i = 0; i < LK; ++i) {
    if (i >= h->n_lk) continue;
    const ksg_look& e = h->lk[i];
    const uint32_t sku = e.sku;
    const int32_t v = lks[i];
    const int32_t x = v < 0 ? 0 : lkv[i];
    switch (ksg_lk_use(sku)) {
      case KLU_PTSF:
#pragma unroll
        for (int c = 0; c < TS; ++c)
          if (c == ksg_lk_aux(sku)) ptsm[c] = x;
        break;
      case KLU_PTSS: pts_cnt += x; break;
      case KLU_AFF:
        aff_miss |= v < 0;
        aff_zero |= x <= 0;
        break;
      case KLU_ANTI: anti_hit |= x > 0; break;
      case KLU_RAW: ipa_raw += (int64_t)x * e.weight; break;
      case KLU_EXANTI: exist_hit |= x > 0; break;
      default: break;
    }
  }
  bool counted = pts_score;
  if (pts_score)
    for (int c = nf; c < nf + ns; ++c) counted &= tv(h->tsc[c].topo) >= 0;
  if (h->tab & KTAB_PTS_MULTI) pts_cnt = 0;  // (k_ptsraw computes the raw scores)
  const uint32_t ipa_flags = su[TS];
  uint32_t code = KSG_FILTER_NOT_EVALUATED;
  bool err = false;
  if (active && !(h->flags & KPF_PREFILTER_REJECT) &&
      !((h->flags & KPF_RESTRICT) && !bit(V.u32 + h->restrict_off, h->restrict_words, (int32_t)n))) {
    code = KSG_FILTER_PASS;
#pragma unroll 1
    for (int pos = 0; pos < F.n; ++pos) {
      uint32_t detail = 0;
      bool fail = false;
      switch (F.plugins[pos]) {  // (plugins outside PM compile to nothing)
        case KP_FIT:
          if constexpr (PMH(KP_FIT)) {
            const uint32_t b = (RUN && ROWM) ? fit_b : ROWM ? fit_filter_row(row, h, C.R) : fit_filter(C, V, n);
            if (b) { fail = true; detail = b; }
          }
          break;
        case KP_TAINT:
          if constexpr (PMH(KP_TAINT)) {
            const int32_t t = untolerated_taint(C, V, n);
            if (t >= 0) { fail = true; detail = (uint32_t)t; }
          }
          break;
        case KP_NA:
          if constexpr (PMH(KP_NA))
            if (!(h->flags & KPF_SKIP_NA_FILTER) && !required_na(C, V, n)) fail = true;
          break;
        case KP_PTS:  // filtering.go: skew = matchNum + selfMatch - minMatchNum > maxSkew
          if constexpr (PMH(KP_PTS))
            if (!(h->flags & KPF_SKIP_PTS_FILTER))
#pragma unroll
              for (int c = 0; c < TS; ++c) {
                if (c >= nf || fail || err) continue;
                const ksg_tsc& t = h->tsc[c];
                const int32_t dom = t.dom;
                if (tv(t.topo) < 0) { fail = true; detail = KSG_PTS_MISSING_LABEL; continue; }
                if (dom == 0) { err = true; continue; }  // minMatchNum: no domains -> Error
                const int64_t mn = dom < t.min_domains ? 0 : (int64_t)(int32_t)su[c];
                if ((int64_t)ptsm[c] + t.self_match - mn > t.max_skew) { fail = true; detail = KSG_PTS_SKEW; }
              }
          break;
        case KP_IPA:  // filtering.go: affinity, anti-affinity, existing pods' anti-affinity
          if constexpr (PMH(KP_IPA)) {
            if (aff_miss || (h->n_req_aff > 0 && aff_zero && !(!(ipa_flags & 1u) && h->self_matches_all))) {
              fail = true;
              detail = KSG_IPA_AFFINITY;
            } else if (anti_hit) {
              fail = true;
              detail = KSG_IPA_ANTI_AFFINITY;
            } else if ((ipa_flags & 4u) && exist_hit) {
              fail = true;
              detail = KSG_IPA_EXISTING_ANTI;
            }
          }
          break;
        case KP_UNSCHED:
          if constexpr (PMH(KP_UNSCHED)) fail = unsched_fails(C, V, n);
          break;
        case KP_NODENAME:
          if constexpr (PMH(KP_NODENAME)) fail = nodename_fails(C, V, n);
          break;
        case KP_PORTS:
          if constexpr (PMH(KP_PORTS))
            if (!(h->flags & KPF_SKIP_PORTS)) fail = ports_fail(C, V, n);
          break;
        case KP_VOLUMES:
          if constexpr (PMH(KP_VOLUMES)) {
            detail = volume_filter(C, V, pos, n);
            fail = detail != 0;
          }
          break;
        default: break;
      }
      if (fail) {
        code = ((uint32_t)pos << 24) | (detail & 0xFFFFFFu);
        break;
      }
    }
  }
  const bool feasible = active && code == KSG_FILTER_PASS;
  const bool kept_run = RUN && A.keep_n && q >= A.keep_first && q < A.keep_first + A.keep_n;
  if ((MODE == kEval || kept_run) && active) of[n] = code;
  CS(3);
  counted &= feasible;
  ChainRec rec;
  rec_init(rec);
  int64_t tot = 0;
  bool range_err = false;
  int64_t sa = 0;                           // SOLO: A, the plugins without ScoreExtensions
  int64_t cv[KCP_X] = {0, 0, 0, 0};         // SOLO: the node's class (raw scores per normalised slot)
  if constexpr (RUN) {
#pragma unroll
    for (int i = 0; i < kNPos<PM>; ++i) eo->raw[i] = 0;
  }
  if (feasible) {
#pragma unroll 1
    for (int pos = 0; pos < F.n; ++pos) {
      const int p = F.plugins[pos];
      int64_t sc = 0;
      switch (p) {
        case KP_FIT:
          if constexpr (PMH(KP_FIT))
            sc = (RUN && ROWM) ? fit_s : ROWM == 2 ? fit_score_row<1>(row, F, h) : ROWM == 1 ? fit_score_row<0>(row, F, h) : fit_score(C, F, V, n);
          break;
        case KP_BA:
          if constexpr (PMH(KP_BA))
            sc = (RUN && ROWM) ? ba_s : ROWM == 2 ? ba_score_row<1>(row, F, h) : ROWM == 1 ? ba_score_row<0>(row, F, h) : ba_score(C, F, V, n);
          break;
        case KP_TAINT:
          if constexpr (PMH(KP_TAINT)) sc = taint_score(C, V, n);
          break;
        case KP_NA:
          if constexpr (PMH(KP_NA)) sc = (h->flags & KPF_SKIP_NA_SCORE) ? 0 : na_score(C, V, n);
          break;
        case KP_IMAGE:
          if constexpr (PMH(KP_IMAGE)) sc = image_score(C, V, n);
          break;
        case KP_IPA: sc = ipa_raw; break;  // scoring.go: the topology score map at the node's pairs
        case KP_PTS:  // the count of the single score constraint (or a placeholder); -1: ignored node
          sc = !pts_score ? 0 : (!counted ? -1 : ((h->tab & KTAB_PTS_MULTI) ? 0 : pts_cnt));
          break;
        default: break;
      }
      if (MODE == kEval || kept_run) os[(size_t)pos * C.N + n] = (int32_t)sc;
      if constexpr (RUN) {
#pragma unroll
        for (int i = 0; i < kNPos<PM>; ++i)
          if (i == pos) eo->raw[i] = (int32_t)sc;
      }
      const int x = chain_x(p);
      if (x >= 0 && (p != KP_PTS || counted)) rec_minmax(rec, x, sc);
      if (SOLO) {
        if (x >= 0) {
#pragma unroll
          for (int i = 0; i < KCP_X; ++i)
            if (i == x) cv[i] = sc;
        } else {  // (no normalisation: the raw score is the score, its [0,100] check is the node's)
          if (sc < 0 || sc > 100) range_err = true;
          sa += sc * F.weight[pos];
        }
      }
      if (!F.has_ext) {
        if (sc < 0 || sc > 100) range_err = true;
        tot += sc * F.weight[pos];
      }
    }
  }
  rec.feas = feasible ? 1 : 0;
  rec.ign = feasible && pts_score && !counted ? 1 : 0;
  rec.st = (err ? 2 : 0) | (range_err ? 4 : 0);
  int nreg = 0;
  if (F.has_ext) {
    nreg = ns;
#pragma unroll
    for (int c = 0; c < TS; ++c) {  // registered values of the score constraints' small keys (initPreScoreState)
      if (c >= ns) continue;
      const ksg_tsc& t = h->tsc[nf + c];
      const int32_t v = tv(t.topo);
      if (counted && !t.is_hostname && t.first_of_key && !((C.T.uniq >> t.topo) & 1u) && v < KSG_TAB_REGV)
        rec.reg[c] = 1ull << v;
    }
  } else if (feasible) {
    ot[n] = (int32_t)tot;
    rec.key = pack_key(tot, F.seed, h->queue_idx, C.goff + n);
  }
  CS(4);
  if constexpr (RUN) {  // the block's record; the caller publishes it
    // diagnostic: each wave of block 0 adds its own arrival (absolute clock) here
    // (slots 56..59), thread 0 its entry (slot 60)
    if (A.stamps && blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (threadIdx.x >> 6) < 4) {
      atomicAdd((unsigned long long*)&A.stamps[56 + (threadIdx.x >> 6)], (unsigned long long)__builtin_amdgcn_s_memrealtime());
      if (threadIdx.x == 0) atomicAdd((unsigned long long*)&A.stamps[60], (unsigned long long)cs_t0);
    }
    fold_partial<KCX_PTS, KCX_IPA, BT>(rec, L.rec, xmask, nreg, true);
    CS(5);
    eo->feasible = feasible;
    eo->ipa_flags = ipa_flags;
    eo->rec = rec;
    return;
  }
  if (SOLO) {
    __shared__ SoloShared S;
    if (threadIdx.x < kSoloCap) {
      S.tag[threadIdx.x] = 0u;
      S.ready[threadIdx.x] = 0u;
      S.best[threadIdx.x] = 0ull;
    }
    if (threadIdx.x == 0) S.dump = 0u;
    bool fits = true;
#pragma unroll
    for (int i = 0; i < KCP_X; ++i) fits &= cv[i] >= INT32_MIN && cv[i] <= INT32_MAX;
    rec_block<TS, BT>(rec, L.rec, xmask, nreg, RB_CNT16 | RB_ST);  // (its barrier orders the table's reset)
    CS(5);
    if (feasible && !fits) atomicOr(&S.dump, 1u);
    lds_barrier();
    const uint64_t keya = feasible ? pack_key(sa, F.seed, h->queue_idx, C.goff + n) : 0ull;
    const int32_t c0 = (int32_t)cv[0], c1 = (int32_t)cv[1], c2 = (int32_t)cv[2], c3 = (int32_t)cv[3];
    const uint32_t lane = threadIdx.x & 63u;
    if (!S.dump) {  // each wave: its classes, one leader lane per class, into the block's table
      bool pend = feasible;
      for (;;) {
        const uint64_t m = __ballot(pend);
        if (!m) break;
        const int ld = __ffsll((unsigned long long)m) - 1;
        const int32_t l0 = __builtin_amdgcn_readlane(c0, ld), l1 = __builtin_amdgcn_readlane(c1, ld);
        const int32_t l2 = __builtin_amdgcn_readlane(c2, ld), l3 = __builtin_amdgcn_readlane(c3, ld);
        const bool same = pend && c0 == l0 && c1 == l1 && c2 == l2 && c3 == l3;
        const uint64_t best = wave_max_u64(same ? keya : (uint64_t)0);
        pend = pend && !same;
        if (lane == 0) solo_insert(S, l0, l1, l2, l3, best);
      }
    }
    lds_barrier();
    SoloCand* out = A.cand + (size_t)blockIdx.x * kChain;
    if (S.dump) {  // every feasible node a class of its own, in node order
      const uint64_t fb = __ballot(feasible);
      if (lane == 0) S.wcnt[threadIdx.x >> 6] = (uint32_t)__popcll(fb);
      lds_barrier();
      uint32_t at = (uint32_t)__popcll(fb & ((1ull << lane) - 1ull)), cnt = 0;
#pragma unroll
      for (int w = 0; w < kChain / 64; ++w) {
        if (w < (int)(threadIdx.x >> 6)) at += S.wcnt[w];
        cnt += S.wcnt[w];
      }
      if (feasible) {
        const int32_t cc[KCP_X] = {c0, c1, c2, c3};
        st_cand(out + at, cc, keya);
      }
      if (threadIdx.x == 0) S.count = cnt;
    } else if (threadIdx.x < 64) {  // the table's classes, compacted
      const bool has = S.tag[lane] != 0u;
      const uint64_t hb = __ballot(has);
      if (has) st_cand(out + __popcll(hb & ((1ull << lane) - 1ull)), S.v[lane], S.best[lane]);
      if (lane == 0) S.count = (uint32_t)__popcll(hb);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (threadIdx.x == 0) {
      const uint32_t b = blockIdx.x, NB = A.nblk;
      st_sc1(A.pi + KCP_FEAS * NB + b, rec.feas);
      st_sc1(A.pi + KCP_IGN * NB + b, rec.ign);
      st_sc1(A.pi + KCP_STAT * NB + b, rec.st);
      st_sc1(A.pi + KCP_CAND * NB + b, (int32_t)S.count);
#pragma unroll
      for (int x = 0; x < KCP_X; ++x) {
        st_sc1(A.pm + (2 * x) * NB + b, rec.mx[x]);
        st_sc1(A.pm + (2 * x + 1) * NB + b, rec.mn[x]);
      }
#pragma unroll
      for (int c = 0; c < TS; ++c)
        if (c < nreg) st_sc1(A.pr + (size_t)c * NB + b, rec.reg[c]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    CS(6);
    __shared__ uint32_t last;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t old = __hip_atomic_fetch_add(A.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = old == gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (last) solo_last_select(C, F, A, L.rec, prog, ipa_flags, cs_t0);
    return;
  }
  rec_block<TS, BT>(rec, L.rec, F.has_ext ? xmask : 0u, nreg, RB_CNT16 | RB_ST | (F.has_ext ? 0u : RB_KEY));
  CS(5);
  if (threadIdx.x == 0) {
    const uint32_t b = blockIdx.x, NB = A.nblk;
    A.pi[KCP_FEAS * NB + b] = rec.feas;
    A.pi[KCP_IGN * NB + b] = rec.ign;
    A.pi[KCP_STAT * NB + b] = rec.st;
    if (b == 0) A.pi[KCP_IPAF * NB] = (int32_t)ipa_flags;
    if (F.has_ext) {
#pragma unroll
      for (int x = 0; x < KCP_X; ++x) {
        A.pm[(2 * x) * NB + b] = rec.mx[x];
        A.pm[(2 * x + 1) * NB + b] = rec.mn[x];
      }
#pragma unroll
      for (int c = 0; c < TS; ++c)
        if (c < nreg) A.pr[(size_t)c * NB + b] = rec.reg[c];
    } else {  // no ScoreExtensions: this is the cycle's last kernel
      st_sc1(A.pk + b, rec.key);
      st_sc1(A.pst + b, 0);
      st_sc1(A.pi + KCP_FEAS * NB + b, rec.feas);
      st_sc1(A.pi + KCP_STAT * NB + b, rec.st);
    }
  }
  CS(6);
  if (!F.has_ext) chain_last_select(C, F, A, L.rec, prog);
}

// k_eval's partials folded (every block of k_ptsraw / k_final does it for itself)
// and topologyNormalizingWeight per score constraint.
struct EvalTotals {
  ChainRec r;
  double w[KSG_MAX_TSC];
};
// topologyNormalizingWeight per score constraint from the folded record.
__device__ __forceinline__ void eval_weights(const DevCluster& C, const ksg_prog* h, EvalTotals& E) {
  const ChainRec& r = E.r;
  const int nf = h->n_tsc_filter, ns = h->n_tsc_score;
#pragma unroll
  for (int c = 0; c < KSG_MAX_TSC; ++c) E.w[c] = 0;
#pragma unroll 1
  for (int c = 0; c < ns; ++c) {  // scoring.go initPreScoreState topoSize (one go_log in the code, not eight)
    const ksg_tsc& t = h->tsc[nf + c];
    uint64_t reg = 0;
#pragma unroll
    for (int i = 0; i < KSG_MAX_TSC; ++i) reg = i == c ? r.reg[i] : reg;
    int64_t size = 0;  // hostname: filtered - ignored nodes; else the key's registered values
    if (t.is_hostname) size = (int64_t)r.feas - r.ign;
    else if (t.first_of_key)  // a key with one node per value registers one value per counted node
      size = ((C.T.uniq >> t.topo) & 1u) ? (int64_t)r.feas - r.ign : (int64_t)__popcll(reg);
    const double w = go_log((double)(size + 2));
#pragma unroll
    for (int i = 0; i < KSG_MAX_TSC; ++i)
      if (i == c) E.w[i] = w;
  }
}
__device__ __forceinline__ void reduce_eval(const DevCluster& C, const DevProfile& F, const ChainArgs& A, const ksg_prog* h,
                                            EvalTotals& E, ChainRec* lds) {
  const uint32_t NB = A.nblk;
  uint32_t xmask = 0;
  for (int p = 0; p < F.n; ++p) {
    const int x = chain_x(F.plugins[p]);
    if (x >= 0) xmask |= 1u << x;
  }
  const int ns = h->n_tsc_score;
  ChainRec& r = E.r;
  rec_init(r);
  for (uint32_t b = threadIdx.x; b < NB; b += blockDim.x) {
    r.feas += A.pi[KCP_FEAS * NB + b];
    r.ign += A.pi[KCP_IGN * NB + b];
    r.st |= A.pi[KCP_STAT * NB + b];
#pragma unroll
    for (int x = 0; x < KCP_X; ++x) {
      if (!((xmask >> x) & 1u)) continue;
      const int64_t a = A.pm[(2 * x) * NB + b], c = A.pm[(2 * x + 1) * NB + b];
      r.mx[x] = a > r.mx[x] ? a : r.mx[x];
      r.mn[x] = c < r.mn[x] ? c : r.mn[x];
    }
#pragma unroll
    for (int c = 0; c < KSG_MAX_TSC; ++c)
      if (c < ns) r.reg[c] |= A.pr[(size_t)c * NB + b];
  }
  rec_block(r, lds, xmask, ns, RB_CNT | RB_ST);
  eval_weights(C, h, E);
}

// PodTopologySpread raw score of a counted node (scoring.go Score): the constraints'
// cnt * weight + (maxSkew - 1), in constraint order, rounded half away from zero.
__device__ __forceinline__ int64_t pts_raw(const DevCluster& C, const ProgView& V, const EvalTotals& E, uint32_t n,
                                           const ChainVids& tv) {
#pragma clang fp contract(off)
  const ksg_prog* h = V.h;
  const int nf = h->n_tsc_filter, ns = h->n_tsc_score;
  double score = 0;
#pragma unroll
  for (int c = 0; c < KSG_MAX_TSC; ++c) {
    if (c >= ns) continue;
    const ksg_tsc& t = h->tsc[nf + c];
    const int32_t v = tv(t.topo);
    if (v < 0) continue;
    const int64_t cnt = pts_count_tab(C, V, nf + c, n, v);
    score = __dadd_rn(score, __dadd_rn(__dmul_rn((double)cnt, E.w[c]), (double)(t.max_skew - 1)));
  }
  return (int64_t)round(score);
}
__device__ __forceinline__ int64_t pts_raw1(const ksg_prog* h, const EvalTotals& E, int64_t cnt) {
#pragma clang fp contract(off)
  const ksg_tsc& t = h->tsc[h->n_tsc_filter];
  return (int64_t)round(__dadd_rn(0.0, __dadd_rn(__dmul_rn((double)cnt, E.w[0]), (double)(t.max_skew - 1))));
}

// Many blocks (large clusters): k_eval's partials folded once, by one block,
// instead of by every block of k_ptsraw / k_final (O(blocks^2) partial reads).
__global__ __launch_bounds__(kChain) void k_fold(DevCluster C, DevProfile F, ChainArgs A, const uint8_t* __restrict__ prog) {
  __shared__ ChainRec lds[kChain / 64];
  EvalTotals E;
  reduce_eval(C, F, A, view(prog).h, E, lds);
  if (threadIdx.x == 0) *A.etot = E;
}
__device__ __forceinline__ void eval_totals(const DevCluster& C, const DevProfile& F, const ChainArgs& A, const ksg_prog* h,
                                            EvalTotals& E, ChainRec* lds) {
  if (A.etot) E = *A.etot;
  else reduce_eval(C, F, A, h, E, lds);
}

// ---- node-sharded table chain: every rank keeps the global
// class tables (pair-level deltas applied by all ranks), so k_eval is rank-local
// and a cycle needs two exchange points (three with several PodTopologySpread
// score constraints):
//   X2 after k_eval: feasible / ignored (SUM), status (OR), normalisers' max /
//      min (MAX / MIN), PodTopologySpread score registrations (OR) — then the
//      normalising weights, identical on every rank;
//   X3 after k_ptsraw: PodTopologySpread raw max / min;
//   X4 after NormalizeScore: argmax key (unsigned MAX), feasible (SUM), status
//      (OR) — selectHost, and the assume: the owner applies the node row and
//      node-level tables, every rank the pair-level ones.
constexpr int kX2 = 3 + 2 * KCP_X + KSG_MAX_TSC;  // int64 words
__global__ __launch_bounds__(kChain) void k_tx2_pack(DevCluster C, DevProfile F, ChainArgs A, const uint8_t* __restrict__ prog,
                                                     int64_t* out) {
  __shared__ ChainRec lds[kChain / 64];
  EvalTotals E;
  reduce_eval(C, F, A, view(prog).h, E, lds);
  if (threadIdx.x == 0) {
    out[0] = E.r.feas;
    out[1] = E.r.ign;
    out[2] = E.r.st;
#pragma unroll
    for (int x = 0; x < KCP_X; ++x) {
      out[3 + x] = E.r.mx[x];
      out[3 + KCP_X + x] = E.r.mn[x];
    }
#pragma unroll
    for (int c = 0; c < KSG_MAX_TSC; ++c) out[3 + 2 * KCP_X + c] = (int64_t)E.r.reg[c];
  }
}
__global__ void k_tx2_merge(DevCluster C, ChainArgs A, const uint8_t* __restrict__ prog, const int64_t* recv, uint32_t ranks) {
  if (threadIdx.x != 0) return;
  EvalTotals E;
  rec_init(E.r);
  for (uint32_t k = 0; k < ranks; ++k) {
    const int64_t* v = recv + (size_t)k * kX2;
    E.r.feas += (int32_t)v[0];
    E.r.ign += (int32_t)v[1];
    E.r.st |= (int32_t)v[2];
#pragma unroll
    for (int x = 0; x < KCP_X; ++x) {
      E.r.mx[x] = v[3 + x] > E.r.mx[x] ? v[3 + x] : E.r.mx[x];
      E.r.mn[x] = v[3 + KCP_X + x] < E.r.mn[x] ? v[3 + KCP_X + x] : E.r.mn[x];
    }
#pragma unroll
    for (int c = 0; c < KSG_MAX_TSC; ++c) E.r.reg[c] |= (uint64_t)v[3 + 2 * KCP_X + c];
  }
  eval_weights(C, view(prog).h, E);
  *A.etot = E;
}
__global__ __launch_bounds__(kChain) void k_tx3_pack(ChainArgs A, int64_t* out) {
  __shared__ ChainRec lds[kChain / 64];
  ChainRec r;
  rec_init(r);
  for (uint32_t b = threadIdx.x; b < A.nblk; b += blockDim.x) {
    r.mx[KCX_PTS] = A.pm2[b] > r.mx[KCX_PTS] ? A.pm2[b] : r.mx[KCX_PTS];
    r.mn[KCX_PTS] = A.pm2[A.nblk + b] < r.mn[KCX_PTS] ? A.pm2[A.nblk + b] : r.mn[KCX_PTS];
  }
  rec_block(r, lds, 1u << KCX_PTS, 0, 0u);
  if (threadIdx.x == 0) {
    out[0] = r.mx[KCX_PTS];
    out[1] = r.mn[KCX_PTS];
  }
}
// the merged PodTopologySpread raw max / min as block 0's partial (the others neutral)
__global__ void k_tx3_merge(ChainArgs A, const int64_t* recv, uint32_t ranks) {
  int64_t mx = INT64_MIN, mn = INT64_MAX;
  for (uint32_t k = 0; k < ranks; ++k) {
    mx = recv[2 * k] > mx ? recv[2 * k] : mx;
    mn = recv[2 * k + 1] < mn ? recv[2 * k + 1] : mn;
  }
  for (uint32_t b = threadIdx.x; b < A.nblk; b += blockDim.x) {
    A.pm2[b] = b == 0 ? mx : INT64_MIN;
    A.pm2[A.nblk + b] = b == 0 ? mn : INT64_MAX;
  }
}
// X4: selectHost over the ranks' (key, feasible, status), the summary, and the
// assume (chain_last_select's, split by ownership).  One wave.
__global__ __launch_bounds__(64) void k_tx4_select(DevCluster C, DevProfile F, ChainArgs A, const uint8_t* __restrict__ prog,
                                                   const int64_t* recv, uint32_t ranks) {
  const uint32_t q = A.q;
  const ProgView V = view(prog);
  const ksg_prog* h = V.h;
  uint64_t key = 0;
  int32_t feas = 0, st = 0;
  for (uint32_t k = 0; k < ranks; ++k) {
    const uint64_t x = (uint64_t)recv[3 * k];
    key = x > key ? x : key;
    feas += (int32_t)recv[3 * k + 1];
    st |= (int32_t)recv[3 * k + 2];
  }
  const bool error = (st & 2) || ((st & 4) && feas > 1) || (h->flags & KPF_PREFILTER_ERROR) || na_prescore_error(h->flags, feas);
  const uint32_t g = (uint32_t)(key & 0xFFFFFull);
  const bool place = !error && feas > 0 && (A.mode & 1);
  const bool mine = place && g >= C.goff && g - C.goff < C.N;
  if (threadIdx.x == 0) {
    ksg_pod_summary* S = A.sums + q;
    S->feasible = feas;
    S->best_key = key;
    if (error) { S->status = 2; S->selected = -1; }
    else if (feas == 0) { S->status = 1; S->selected = -1; }
    else { S->status = 0; S->selected = (int32_t)g; }
    A.prow[q] = -1;
    A.alog[q - A.log_base] = make_int2((int)q, mine && (A.mode & 2) ? (int)(g - C.goff) : -1);
    if (mine) assume_row_atomic(C, V, g - C.goff, +1);
  }
  if (mine) tables_assume(C, V, g - C.goff, +1, threadIdx.x, blockDim.x);
  else if (place) tables_assume_remote(C, V, g, +1, threadIdx.x, blockDim.x);
}

// The normalisers per profile position from the folded partials (the summary's
// max / min; PodTopologySpread's from the raw score of its single constraint).
template <uint32_t PM = ~0u>
__device__ __forceinline__ void chain_norms(const DevProfile& F, const ksg_prog* h, const EvalTotals& E,
                                            int64_t (&smx)[KSG_MAX_PLUGINS], int64_t (&smn)[KSG_MAX_PLUGINS],
                                            int64_t pmx, int64_t pmn) {
#pragma unroll
  for (int pos = 0; pos < kNPos<PM>; ++pos) {
    smx[pos] = 0;
    smn[pos] = INT64_MAX;
    if (pos >= F.n) continue;
    const int p = F.plugins[pos], x = chain_x(p);
    if (p == KP_IPA) smx[pos] = INT64_MIN;
    if (x < 0) continue;
    if (p == KP_PTS) {
      if (pmx != INT64_MIN) { smx[pos] = pmx > 0 ? pmx : 0; smn[pos] = pmn; }
    } else if (rec_mx(E.r, x) != INT64_MIN) {
      const int64_t m = rec_mx(E.r, x);
      smx[pos] = p == KP_IPA ? m : (m > 0 ? m : 0);
      smn[pos] = rec_mn(E.r, x);
    }
  }
}
__device__ __forceinline__ void chain_summary(const ChainArgs& A, const DevProfile& F, const ksg_prog* h,
                                              const EvalTotals& E, const int64_t (&smx)[KSG_MAX_PLUGINS],
                                              const int64_t (&smn)[KSG_MAX_PLUGINS], uint32_t ipa_flags) {
  ksg_pod_summary* S = A.sums + A.q;
  S->feasible = E.r.feas;
  S->ignored = E.r.ign;
  S->ipa_flags = ipa_flags;
#pragma unroll
  for (int pos = 0; pos < KSG_MAX_PLUGINS; ++pos)
    if (pos < F.n) {
      S->max_score[pos] = smx[pos];
      S->min_score[pos] = smn[pos];
    }
#pragma unroll
  for (int c = 0; c < KSG_MAX_TSC; ++c)
    if (c < h->n_tsc_score) S->pts_weight[c] = E.w[c];
}

// k_eval_solo's last-arriving block: the partials folded (normalisers, the
// PodTopologySpread weights), the summary, every block's classes normalised and
// weighted (the [0,100] check per class), the argmax, then the commit.
__device__ void solo_last_select(DevCluster& C, const DevProfile& F, const ChainArgs& A, ChainRec* lds,
                                 const uint8_t* __restrict__ prog, uint32_t ipa_flags, uint64_t cs_t0) {
  const ProgView V = view(prog);
  const ksg_prog* h = V.h;
  const uint32_t NB = A.nblk;
  uint32_t xmask = 0;
  for (int p = 0; p < F.n; ++p) {
    const int x = chain_x(F.plugins[p]);
    if (x >= 0) xmask |= 1u << x;
  }
  const int ns = h->n_tsc_score;
  EvalTotals E;
  ChainRec& r = E.r;
  rec_init(r);
  for (uint32_t b = threadIdx.x; b < NB; b += blockDim.x) {
    r.feas += ld_sc1(A.pi + KCP_FEAS * NB + b);
    r.ign += ld_sc1(A.pi + KCP_IGN * NB + b);
    r.st |= ld_sc1(A.pi + KCP_STAT * NB + b);
#pragma unroll
    for (int x = 0; x < KCP_X; ++x) {
      if (!((xmask >> x) & 1u)) continue;
      const int64_t a = ld_sc1(A.pm + (2 * x) * NB + b), c = ld_sc1(A.pm + (2 * x + 1) * NB + b);
      r.mx[x] = a > r.mx[x] ? a : r.mx[x];
      r.mn[x] = c < r.mn[x] ? c : r.mn[x];
    }
#pragma unroll
    for (int c = 0; c < KSG_MAX_TSC; ++c)
      if (c < ns) r.reg[c] |= ld_sc1(A.pr + (size_t)c * NB + b);
  }
  CS(24);
  rec_block(r, lds, xmask, ns, RB_CNT | RB_ST);
  eval_weights(C, h, E);
  int64_t pmx = INT64_MIN, pmn = INT64_MAX;
  if (E.r.mx[KCX_PTS] != INT64_MIN) {  // one score constraint: raw is monotone in the count
    pmx = pts_raw1(h, E, E.r.mx[KCX_PTS]);
    pmn = pts_raw1(h, E, E.r.mn[KCX_PTS]);
  }
  int64_t smx[KSG_MAX_PLUGINS], smn[KSG_MAX_PLUGINS];
  chain_norms(F, h, E, smx, smn, pmx, pmn);
  if (threadIdx.x == 0) chain_summary(A, F, h, E, smx, smn, ipa_flags);
  CS(25);
  // every block's classes
  const bool pts_skip = (h->flags & KPF_SKIP_PTS_SCORE) != 0;
  ChainRec k;
  rec_init(k);
  for (uint32_t b = threadIdx.x; b < NB; b += blockDim.x) {
    const uint32_t cnt = (uint32_t)ld_sc1(A.pi + KCP_CAND * NB + b);
    const uint64_t* base = reinterpret_cast<const uint64_t*>(A.cand + (size_t)b * kChain);
    for (uint32_t e = 0; e < cnt; ++e) {
      const uint64_t w0 = ld_sc1(base + 3 * e), w1 = ld_sc1(base + 3 * e + 1), key = ld_sc1(base + 3 * e + 2);
      const int32_t cvv[KCP_X] = {(int32_t)(uint32_t)w0, (int32_t)(uint32_t)(w0 >> 32), (int32_t)(uint32_t)w1,
                                  (int32_t)(uint32_t)(w1 >> 32)};
      int64_t part = 0;
      bool rerr = false;
#pragma unroll
      for (int pos = 0; pos < KSG_MAX_PLUGINS; ++pos) {
        if (pos >= F.n) continue;
        const int p = F.plugins[pos], x = chain_x(p);
        if (x < 0) continue;
        int64_t sv = 0;
#pragma unroll
        for (int i = 0; i < KCP_X; ++i)
          if (i == x) sv = cvv[i];
        bool pts_keys = false;
        if (p == KP_PTS) {
          pts_keys = sv >= 0 && ns > 0;
          if (sv < 0) sv = 0;
          else if (ns > 0 && !pts_skip) sv = pts_raw1(h, E, sv);
        }
        bool use;
        const int64_t v = normalize_pos(p, h, sv, smx[pos], smn[pos], ipa_flags, pts_keys, use);
        if (use) {
          if (v < 0 || v > 100) rerr = true;
          part += v * F.weight[pos];
        }
      }
      const uint64_t kk = E.r.feas == 1 ? (key & 0xFFFFFFFFFFull) : key + ((uint64_t)part << 40);
      k.key = kk > k.key ? kk : k.key;
      if (rerr) k.st |= 4;
    }
  }
  CS(26);
  __syncthreads();  // (lds reused)
  rec_block(k, lds, 0u, 0, RB_ST | RB_KEY);
  const int32_t st = E.r.st | (E.r.feas > 1 ? (k.st & 4) : 0);
  chain_commit(C, A, V, k.key, E.r.feas, st, cs_t0);
}

struct FinalShared {
  int32_t tv[KSG_MAX_TOPO * kChain];
  ChainRec rec[kChain / 64];
  uint32_t ipa_flags;
};

// PodTopologySpread raw scores of a pod with several score constraints.
__global__ __launch_bounds__(kChain) void k_ptsraw(DevCluster C, DevProfile F, ChainArgs A, const uint8_t* __restrict__ prog) {
  const uint32_t q = A.q;
  const ProgView V = view(prog);
  __shared__ FinalShared L;
  uint32_t* of;
  int32_t *os, *ot;
  chain_outs(A, q, C.N, of, os, ot);
  int pts_pos = -1;
  for (int p = 0; p < F.n; ++p)
    if (F.plugins[p] == KP_PTS) pts_pos = p;
  const uint32_t n = blockIdx.x * kChain + threadIdx.x;
  const bool active = n < C.N;
  {
    int32_t vid[KSG_MAX_TOPO];
    node_slot_vids(C, active ? n : 0, vid);
#pragma unroll
    for (int t = 0; t < KSG_MAX_TOPO; ++t)
      if ((uint32_t)t < C.n_topo) L.tv[t * kChain + threadIdx.x] = vid[t];
  }
  const ChainVids tv{L.tv + threadIdx.x};
  EvalTotals E;
  eval_totals(C, F, A, V.h, E, L.rec);
  ChainRec r;
  rec_init(r);
  if (active && of[n] == KSG_FILTER_PASS) {
    int32_t* slot = os + (size_t)pts_pos * C.N + n;
    if (*slot >= 0) {
      const int64_t s = pts_raw(C, V, E, n, tv);
      *slot = (int32_t)s;
      r.mx[KCX_PTS] = r.mn[KCX_PTS] = s;
    }
  }
  __syncthreads();  // L.rec reused
  rec_block(r, L.rec, 1u << KCX_PTS, 0, 0u);
  if (threadIdx.x == 0) {
    A.pm2[blockIdx.x] = r.mx[KCX_PTS];
    A.pm2[A.nblk + blockIdx.x] = r.mn[KCX_PTS];
  }
}

template <uint32_t PM = ~0u>
__device__ __forceinline__ void final_body(DevCluster& C, const DevProfile& F, const ChainArgs& A,
                                           const uint8_t* __restrict__ prog) {
  chain_warm(prog);
  CS_BEGIN;
  CS_GAP(40, 48, 49);
  const uint32_t q = A.q;
  const ProgView V = view(prog);
  const ksg_prog* h = V.h;
  __shared__ FinalShared L;
  uint32_t* of;
  int32_t *os, *ot;
  chain_outs(A, q, C.N, of, os, ot);
  const uint32_t n = blockIdx.x * kChain + threadIdx.x;
  const bool mine = n < C.N && of[n] == KSG_FILTER_PASS;
  int32_t raw[KSG_MAX_PLUGINS];  // this node's raw scores, loaded before the folds
#pragma unroll
  for (int pos = 0; pos < kNPos<PM>; ++pos) raw[pos] = (mine && pos < F.n) ? os[(size_t)pos * C.N + n] : 0;
  const uint32_t ipa_flags = (uint32_t)A.pi[KCP_IPAF * A.nblk];  // k_eval's block 0
  EvalTotals E;
  CS(16);
  eval_totals(C, F, A, h, E, L.rec);
  CS(17);
  const bool multi = (h->tab & KTAB_PTS_MULTI) != 0;
  int64_t pmx = INT64_MIN, pmn = INT64_MAX;  // PodTopologySpread raw max / min over counted nodes
  if (multi) {
    ChainRec r;
    rec_init(r);
    for (uint32_t b = threadIdx.x; b < A.nblk; b += blockDim.x) {
      r.mx[KCX_PTS] = A.pm2[b] > r.mx[KCX_PTS] ? A.pm2[b] : r.mx[KCX_PTS];
      r.mn[KCX_PTS] = A.pm2[A.nblk + b] < r.mn[KCX_PTS] ? A.pm2[A.nblk + b] : r.mn[KCX_PTS];
    }
    __syncthreads();  // L.rec reused
    rec_block(r, L.rec, 1u << KCX_PTS, 0, 0u);
    pmx = r.mx[KCX_PTS];
    pmn = r.mn[KCX_PTS];
  } else if (E.r.mx[KCX_PTS] != INT64_MIN) {  // one constraint: raw is monotone in the count
    pmx = pts_raw1(h, E, E.r.mx[KCX_PTS]);
    pmn = pts_raw1(h, E, E.r.mn[KCX_PTS]);
  }
  CS(18);
  // the summary's normalisers per position (max over feasible nodes; unset as k_init_summaries)
  int64_t smx[KSG_MAX_PLUGINS], smn[KSG_MAX_PLUGINS];
#pragma unroll
  for (int pos = 0; pos < kNPos<PM>; ++pos) {
    smx[pos] = 0;
    smn[pos] = INT64_MAX;
    if (pos >= F.n) continue;
    const int p = F.plugins[pos], x = chain_x(p);
    if (p == KP_IPA) smx[pos] = INT64_MIN;
    if (x < 0) continue;
    if (p == KP_PTS) {
      if (pmx != INT64_MIN) { smx[pos] = pmx > 0 ? pmx : 0; smn[pos] = pmn; }
    } else if (rec_mx(E.r, x) != INT64_MIN) {
      const int64_t m = rec_mx(E.r, x);
      smx[pos] = p == KP_IPA ? m : (m > 0 ? m : 0);
      smn[pos] = rec_mn(E.r, x);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ksg_pod_summary* S = A.sums + q;
    S->feasible = E.r.feas;
    S->ignored = E.r.ign;
    S->ipa_flags = ipa_flags;
#pragma unroll
    for (int pos = 0; pos < kNPos<PM>; ++pos)
      if (pos < F.n) {
        S->max_score[pos] = smx[pos];
        S->min_score[pos] = smn[pos];
      }
#pragma unroll
    for (int c = 0; c < KSG_MAX_TSC; ++c)
      if (c < h->n_tsc_score) S->pts_weight[c] = E.w[c];
  }
  ChainRec r;
  rec_init(r);
  if (mine) {
    int64_t tot = 0;
    bool pts_keys = false, range_err = false;
#pragma unroll
    for (int pos = 0; pos < kNPos<PM>; ++pos) {
      if (pos >= F.n) continue;
      const int p = F.plugins[pos];
      int64_t s = raw[pos];
      if (p == KP_PTS) {
        pts_keys = s >= 0 && h->n_tsc_score > 0;
        if (s < 0) s = 0;
        else if (!multi && h->n_tsc_score > 0 && !(h->flags & KPF_SKIP_PTS_SCORE)) s = pts_raw1(h, E, s);
        os[(size_t)pos * C.N + n] = (int32_t)s;
      }
      bool use;
      const int64_t v = normalize_pos(p, h, s, smx[pos], smn[pos], ipa_flags, pts_keys, use);
      if (use) {
        if (v < 0 || v > 100) range_err = true;
        tot += v * F.weight[pos];
      }
    }
    if (E.r.feas == 1) tot = 0;  // single feasible node: no scoring
    ot[n] = (int32_t)tot;
    r.key = pack_key(tot, F.seed, h->queue_idx, C.goff + n);
    r.st = (E.r.feas > 1 && range_err) ? 4 : 0;
  }
  CS(19);
  __syncthreads();  // L.rec reused
  rec_block(r, L.rec, 0u, 0, RB_ST | RB_KEY);
  if (threadIdx.x == 0) {
    st_sc1(A.pk + blockIdx.x, r.key);
    st_sc1(A.pst + blockIdx.x, r.st);
  }
  CS(20);
  chain_last_select(C, F, A, L.rec, prog);
}

// ---- The persistent chain (k_chain_run): a segment of consecutive table-chain
// pods in ONE launch, the pod loop on the device.  One block
// per tile of kChain nodes (at most kChain blocks), every block resident (the host
// checks the grid against the occupancy query); each block keeps its nodes'
// topology values in LDS and their rows in registers for the whole segment.  Per
// pod k, with no grid barrier:
//   eval    as k_eval (class-table counts read sc1: assumes change them under the
//           launch); the block's partial record goes out as tagged granules;
//   fold    every block polls every block's partial granules until their tags
//           read k + 1, folds them (normalisers, PodTopologySpread weights), then
//           NormalizeScore / weights / packed key of its own nodes; its best key
//           goes out as tagged granules;
//   select  every block polls every block's key granules and takes the same
//           argmax (selectHost); block 0 writes the summary; the block owning the
//           selected node applies the assume — the node row (its register copy and
//           the global row), the class-table deltas with the node's topology values
//           from its LDS — drains those atomics and raises the pod's flag;
//   the other blocks wait for that flag only before pod k + 1's class-table reads
//   (the next program header is pulled into the scalar cache meanwhile).
// Granule = one 8-byte {data, tag} written by ONE sc1 store and read by sc1
// loads (MI355X_MICROARCH.md: R2 granules need no ordering; the flag hand-off is
// table row 1).  Every poll is bounded: a block that waits ~seconds raises
// `abort`, the others leave at their next poll, the host reports the run failed.
// Eligible pods (host): table chain, at most one PodTopologySpread score
// constraint, no host ports / volume claims / CSI volumes (nothing but the rows
// and the class tables changes during the segment), outputs not kept, committing
// cycles of an unsharded context whose profile normalises.
// Launch handshake: every block adds to `arrive` on entry and waits (bounded by
// RunCtl::wait_ticks) until the whole grid has arrived; the first block to decide
// sets `verdict` by compare-and-swap (1: every block resident, go; 2: not
// co-resident; 3: an earlier segment of the call aborted) and publishes it to the
// host's pinned word; a block seeing anything but 1 leaves before touching any
// state, so the host can run the segment's pods on the two-launch chain instead.
// Granules are double-buffered by pod parity: pod k's slot is rewritten only by
// pod k + 2, whose class-table wait needs flag >= k + 1, i.e. the committer done
// with pod k (it is allowed to lag the node blocks by one pod).
struct RunSync {
  uint64_t flag[16];     // k + 1: pod k's assume is applied (written by the committer)
  uint32_t arrive[32];   // blocks that entered the launch (handshake)
  uint32_t verdict[32];  // handshake outcome (0 undecided)
  uint32_t abort[32];    // a poll ran out: every block leaves; sticky until Engine::sync reads it
};
constexpr size_t kRunSyncReset = offsetof(RunSync, abort);  // bytes zeroed per launch (the abort word is kept)
struct RunCtl {
  uint32_t need;           // blocks that must be resident (the grid; more forces the fallback: tests)
  uint32_t wait_ticks;     // handshake limit in s_memrealtime ticks (100 MHz)
  uint32_t lag;            // diagnostic: the committer's s_sleep(127) rounds before each pod's granule reads
  uint32_t* host_verdict;  // pinned host word the deciding block writes (the host polls it), or null
  uint32_t spin;           // polls before a block gives up (kRunSpin; tests force an abort with few)
  uint32_t overlap;        // issue pod k+1's class-table reads during pod k's hand-offs (KSG_RUN_OVERLAP)
  uint32_t defer;          // the owner's node-level assume after the next partial record when independent (KSG_RUN_DEFER)
  // blocks of another kernel this launch waits on (k_static_dec_run beside the window
  // loop: its blocks count themselves in here as they start); go only once side_need
  // of them have started, so every later wait on their output is on running blocks
  const uint32_t* side_arrive;
  uint32_t side_need;
};
// Pod j+1 (header n) may read the class tables before pod j's (header h) assume:
// it reads none of the pair-level nor node-level entries pod j writes (its row,
// the only other change, is read only at the finish, after the assume).
__device__ __forceinline__ bool run_indep(const ksg_prog* h, const ksg_prog* n) {
  return (h->tab_md & n->tab_rd) == 0 && (h->nd_md & n->nd_rd) == 0;
}
constexpr uint32_t kRunSpin = 1u << 22;  // polls (~1 us each with the load) before a block gives up
#ifndef KSG_RUN_SLEEP
#define KSG_RUN_SLEEP 8
#endif
constexpr int kRunSleep = KSG_RUN_SLEEP;  // s_sleep between polls (x 64 cycles): every block polls every block
constexpr int kRunG1 = 2 + 4 * KCP_X + 2 * KSG_MAX_TSC;  // partial-record granules per block (max)
constexpr int kRunG2 = 3;                                // key granules per block
constexpr int kRunGS = 64;                               // granules per block (uint64)
constexpr size_t kRunSlot = (size_t)kChain * kRunGS;     // one parity slot of one granule kind (uint64)
// Granule j of block b sits at j * kGF + b * kGB of its slot.  Field-major (the
// default, round 5): the readers' lanes are the blocks, so one poll or record load
// of a wave reads 64 consecutive granules (8 lines) instead of one line per lane
// (64); KSG_RUN_GT=0 restores the block-major layout.
#ifndef KSG_RUN_GT
#define KSG_RUN_GT 1
#endif
constexpr size_t kGB = KSG_RUN_GT ? 1 : kRunGS;
constexpr size_t kGF = KSG_RUN_GT ? kChain : 1;
__device__ __forceinline__ uint64_t gran(uint32_t tag, uint32_t v) { return ((uint64_t)tag << 32) | v; }
__device__ __forceinline__ bool run_aborted(uint32_t i, const RunSync* Y) {
  return (i & 63u) == 63u && ld_sc1(&Y->abort[0]) != 0u;
}
__device__ __forceinline__ void run_raise(RunSync* Y) {
  __hip_atomic_store(&Y->abort[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The launch handshake (every thread of the block; thread 0 decides): true = go.
__device__ bool run_handshake(RunSync* Y, const RunCtl& R, uint32_t* go) {
  if (threadIdx.x == 0) {
    uint32_t want = 1;
    if (ld_sc1(&Y->abort[0]) != 0u) {
      want = 3;
    } else {
      __hip_atomic_fetch_add(&Y->arrive[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      want = 2;
      for (;;) {
        if (ld_sc1(&Y->arrive[0]) >= R.need && (!R.side_arrive || ld_sc1(R.side_arrive) >= R.side_need)) {
          want = 1;
          break;
        }
        if (ld_sc1(&Y->verdict[0]) != 0u) break;  // decided by another block
        if (__builtin_amdgcn_s_memrealtime() - t0 > R.wait_ticks) break;
        __builtin_amdgcn_s_sleep(4);
      }
    }
    uint32_t old = 0;
    __hip_atomic_compare_exchange_strong(&Y->verdict[0], &old, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t v = old == 0 ? want : old;
    if (old == 0 && R.host_verdict) __hip_atomic_store(R.host_verdict, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    *go = v;
  }
  __syncthreads();
  const bool ok = *go == 1u;
  __syncthreads();  // (go is reused by the body)
  return ok;
}
template <int BT>
struct RunSharedT {
  EvalSharedT<BT> L;
  uint32_t go;    // LDS broadcast of a poll's outcome
  uint32_t seen;  // the highest flag value this block has read (a wait it already covers polls nothing)
};
// The flag counts the pods of the segment whose assumes are all applied: pod k's
// owner (block 0 for a pod that places nothing) raises it to k + 1 once it
// reads k (thread 0; bounded like every poll).
__device__ __forceinline__ void run_advance(RunSync* Y, uint32_t k, uint32_t spin) {
  bool ok = false;
  for (uint32_t it = 0; it < spin; ++it) {
    if (ld_sc1(&Y->flag[0]) >= k) { ok = true; break; }
    if (run_aborted(it, Y)) return;
    __builtin_amdgcn_s_sleep(2);
  }
  if (!ok) { run_raise(Y); return; }
  st_sc1(&Y->flag[0], (uint64_t)(k + 1u));
}
struct RunWait {
  RunSync* Y;
  uint32_t want;   // flag value awaited (0: none)
  uint32_t* go;    // RunShared::go
  uint32_t* seen;  // RunShared::seen
  uint64_t* rst;   // diagnostic stamps (block 0), or null
  uint32_t owned;  // this block applied the previous pod's node-level assume
  uint32_t spin;   // RunCtl::spin
};
// Every thread of the block: thread 0 polls the flag, the block joins it.  The
// owner's node-level atomics of the previous pod were issued by the item lanes of
// some waves and are read by lanes of others: every wave drains its own, and a
// barrier orders them before any wave's class-table reads.
__device__ bool run_wait_flag(const RunWait& W) {
  if (W.owned) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the owner's node-level atomics)
  // a flag value already read (during the previous pod's key poll) covers the
  // wait of a pod independent of its predecessor: no poll round trip
  if (!W.want || *W.seen >= W.want) {
    if (W.owned) __syncthreads();
    return true;
  }
  if (threadIdx.x == 0) {
    const uint64_t w0 = W.rst ? __builtin_amdgcn_s_memrealtime() : 0;
    bool ok = false;
    for (uint32_t it = 0; it < W.spin; ++it) {
      // (seen is not updated here: the other waves read it at the top of this call
      // with no barrier in between; it changes only in the key poll, between barriers)
      if (ld_sc1(&W.Y->flag[0]) >= W.want) { ok = true; break; }
      if (run_aborted(it, W.Y)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) run_raise(W.Y);
    *W.go = ok ? 1u : 0u;
    if (W.rst) atomicAdd((unsigned long long*)&W.rst[38], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - w0));
  }
  __syncthreads();
  return *W.go != 0u;
}
__device__ __forceinline__ int run_g1_count(uint32_t xmask, int ns) { return 2 + 4 * __popc(xmask) + 2 * ns; }
__device__ __forceinline__ bool gtag(uint64_t g, uint32_t tag) { return (uint32_t)(g >> 32) == tag; }
__device__ __forceinline__ int64_t g64(uint64_t lo, uint64_t hi) { return (int64_t)((uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32)); }
// thread t < NB: block t's partial record, polled until every granule carries tag
template <int TS>
__device__ __forceinline__ bool run_read_g1(const uint64_t* g, uint32_t tag, uint32_t xmask, int ns, ChainRec& r,
                                            const RunSync* Y, uint32_t spin) {
  const int last = run_g1_count(xmask, ns) - 1;
  for (uint32_t it = 0; it < spin; ++it) {
    // one granule per poll until it carries the tag (few loads in flight chip-wide),
    // then the whole record (whose tags are checked again)
    if (!gtag(ld_sc1(g + last * kGF), tag)) {
      if (run_aborted(it, Y)) return false;
      __builtin_amdgcn_s_sleep(kRunSleep);
      continue;
    }
    bool ok = true;
    const uint64_t w0 = ld_sc1(g), w1 = ld_sc1(g + kGF);
    ok &= gtag(w0, tag) && gtag(w1, tag);
    int j = 2;
#pragma unroll
    for (int x = 0; x < KCP_X; ++x)
      if ((xmask >> x) & 1u) {
        const uint64_t a = ld_sc1(g + j * kGF), b = ld_sc1(g + (j + 1) * kGF), c = ld_sc1(g + (j + 2) * kGF),
                       d = ld_sc1(g + (j + 3) * kGF);
        ok &= gtag(a, tag) && gtag(b, tag) && gtag(c, tag) && gtag(d, tag);
        r.mx[x] = g64(a, b);
        r.mn[x] = g64(c, d);
        j += 4;
      }
#pragma unroll
    for (int c = 0; c < TS; ++c)
      if (c < ns) {
        const uint64_t a = ld_sc1(g + j * kGF), b = ld_sc1(g + (j + 1) * kGF);
        ok &= gtag(a, tag) && gtag(b, tag);
        r.reg[c] = (uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)b << 32);
        j += 2;
      }
    r.feas = (int32_t)((uint32_t)w0 & 0xFFFFu);
    r.ign = (int32_t)(((uint32_t)w0 >> 16) & 0xFFFFu);
    r.st = (int32_t)(uint32_t)w1;
    if (ok) return true;
    if (run_aborted(it, Y)) return false;
    __builtin_amdgcn_s_sleep(kRunSleep);
  }
  run_raise(const_cast<RunSync*>(Y));
  return false;
}

// P / PO: the programs and their offsets as __restrict__ kernel arguments, so the
// wave-uniform header reads stay scalar loads (s_load) despite the launch's own
// stores: through ChainArgs' plain pointers they were vector loads, each waited
// for with vmcnt(0) (round 5).
template <int ROWM, uint32_t PM, int LK, int TS, int BT>
__device__ __forceinline__ void run_body(DevCluster& C, const DevProfile& F, const ChainArgs& A0, uint32_t count,
                                         RunSync* Y, uint64_t* G1s, uint64_t* G2s, const RunCtl& R,
                                         const uint8_t* __restrict__ P, const uint64_t* __restrict__ PO) {
  static_assert(ROWM != 0, "the persistent chain keeps the node row in registers");
  __shared__ RunSharedT<BT> S;
  EvalSharedT<BT>& L = S.L;
  if (!run_handshake(Y, R, &S.go)) return;
  const uint32_t NB = A0.nblk, b = blockIdx.x;
  const uint32_t n = b * BT + threadIdx.x;
  const bool active = n < C.N;
  const uint32_t nn = active ? n : 0;
  {
    int32_t vid[KSG_MAX_TOPO];
    node_slot_vids(C, nn, vid);
#pragma unroll
    for (int s = 0; s < KSG_MAX_TOPO; ++s)
      if ((uint32_t)s < C.n_topo) L.tv[s * BT + threadIdx.x] = vid[s];
  }
  RowV row;
  load_row(C, nn, A0.need_eph, row);
  if (threadIdx.x == 0) S.seen = 0;
  uint32_t xmask = 0;
  for (int p = 0; p < F.n; ++p) {
    const int x = chain_x(F.plugins[p]);
    if (x >= 0) xmask |= 1u << x;
  }
  // diagnostic stamps (Engine::eval_stamps): block 0's phase ends since the pod's
  // start, slots 30..34, 39, 47, the pod's end 50, pods 35; the owner's commit time 36, commits 37; block
  // 0's wait for the previous pod's flag 38
  uint64_t* const rst = A0.stamps;
  const bool rs_on = rst && b == 0 && threadIdx.x == 0;
  uint64_t rs_t0 = 0;
#define RS(k) \
  if (rs_on) atomicAdd((unsigned long long*)&rst[k], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - rs_t0))
  __syncthreads();
  uint32_t wait_for = 0;  // the flag value this block needs before its next class-table read (0: none)
  uint32_t owned = 0;     // this block applied a node-level assume not yet drained before a class-table read
  // The owner's node-level assume deferred past the next pod's evaluation when
  // that pod reads none of the entries it writes (node-level Bloom filters): its
  // atomics then go out after the next partial record (their acknowledgement
  // overlaps the partials' hand-off) instead of being drained at the start of
  // the next evaluation, which made the owner block the last one of the pod
  // (KSG_RUN_DEFER=0: drained as before).
  uint32_t dfr_node = 0xFFFFFFFFu;  // (per item lane: its deferred item, this node)
  int32_t dfr_cls = -1;
  ksg_exist_term dfr_term;
  dfr_term.cls = -1;
  bool dfr_is_cls = false;
  bool dfr_any = false;  // (block-uniform: some lane holds a deferred item)
  // Overlap (KSG_RUN_OVERLAP): when pod k+1 is independent of pod k (run_indep),
  // its class-table reads are issued right after pod k's partial record goes out
  // and stay in flight across pod k's fold, selection and assume; pod k+1 then
  // finishes from them (eval_body stages 1 / 2) on its row as of then.
  bool have = false;       // pre holds pod k's reads (issued during pod k-1)
  EvalPre pre;
  RowPre rpre;             // pod k's row-only plugins, computed during pod k-1's key hand-off
  bool rpre_ok = false;
  const ksg_prog* ph = nullptr;  // pod k-1's header
  for (uint32_t k = 0; k < count; ++k) {
    ChainArgs A = A0;  // (A.stamps: eval_body's own k_eval slots, block 0)
    A.q = A0.q + k;
    const uint8_t* prog = P + PO[A.q];
    const uint32_t tag = k + 1u;
    uint64_t* const G1 = G1s + (k & 1u) * kRunSlot;  // (parity slots)
    uint64_t* const G2 = G2s + (k & 1u) * kRunSlot;
    if (rs_on) rs_t0 = __builtin_amdgcn_s_memrealtime();
    const ProgView V = view(prog);
    const ksg_prog* h = V.h;
    // ---- eval: this block's nodes (waiting for the previous pod's assume before
    // the class-table reads), its partial record
    EvalOut eo;
    eo.abort = false;
    if (have) {
      eval_body<ROWM, kRun, PM, LK, TS, BT, 2>(C, F, A, prog, &L, &row, &eo, nullptr, &pre);
    } else {
      const RunWait W{Y, wait_for, &S.go, &S.seen, rs_on ? rst : nullptr, owned, R.spin};
      eval_body<ROWM, kRun, PM, LK, TS, BT>(C, F, A, prog, &L, &row, &eo, &W, nullptr, rpre_ok ? &rpre : nullptr);
      owned = 0;
    }
    if (eo.abort) return;
    wait_for = 0;
    const int ns = h->n_tsc_score;
    // the partial record's granules, stored by one lane field after field (a
    // per-lane pick of its granule was a long select chain on every lane)
    if (threadIdx.x == 0) {
      uint64_t* g = G1 + (size_t)b * kGB;
      const ChainRec& rr = eo.rec;
      st_sc1(g, gran(tag, (uint32_t)rr.feas | ((uint32_t)rr.ign << 16)));
      st_sc1(g + kGF, gran(tag, (uint32_t)rr.st));
      int j = 2;
#pragma unroll
      for (int x = 0; x < KCP_X; ++x)
        if ((xmask >> x) & 1u) {
          st_sc1(g + j * kGF, gran(tag, (uint32_t)(uint64_t)rr.mx[x]));
          st_sc1(g + (j + 1) * kGF, gran(tag, (uint32_t)((uint64_t)rr.mx[x] >> 32)));
          st_sc1(g + (j + 2) * kGF, gran(tag, (uint32_t)(uint64_t)rr.mn[x]));
          st_sc1(g + (j + 3) * kGF, gran(tag, (uint32_t)((uint64_t)rr.mn[x] >> 32)));
          j += 4;
        }
#pragma unroll
      for (int c = 0; c < TS; ++c)
        if (c < ns) {
          st_sc1(g + j * kGF, gran(tag, (uint32_t)rr.reg[c]));
          st_sc1(g + (j + 1) * kGF, gran(tag, (uint32_t)(rr.reg[c] >> 32)));
          j += 2;
        }
    }
    if (dfr_node != 0xFFFFFFFFu) {  // (the previous pod's deferred node-level items)
      int32_t v[KSG_MAX_TOPO];
      const uint32_t ln = dfr_node % BT;
#pragma unroll
      for (int s2 = 0; s2 < KSG_MAX_TOPO; ++s2) v[s2] = (uint32_t)s2 < C.n_topo ? L.tv[s2 * BT + ln] : -1;
      if (dfr_is_cls) pc_add(C, dfr_cls, dfr_node, +1, v, TP_NODE);
      else tc_add(C, dfr_term, dfr_node, +1, v, TP_NODE);
      dfr_node = 0xFFFFFFFFu;
    }
    if (dfr_any) {  // (drained before the next class-table read that may see them)
      owned = 1;
      dfr_any = false;
    }
    RS(30);
    // diagnostic: the latest block's partial store (absolute clock, per pod parity)
    if (rst && threadIdx.x == 0) atomicMax((unsigned long long*)&rst[52 + (k & 1)], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    // ---- pod k+1's class-table reads, in flight across this pod's hand-offs
    const ksg_prog* nh = k + 1 < count ? reinterpret_cast<const ksg_prog*>(P + PO[A.q + 1]) : nullptr;
    const bool tnext = R.overlap && nh && run_indep(h, nh);
    if (tnext) {
      ChainArgs A1 = A0;
      A1.q = A.q + 1;
      // the assumes before pod k (before pod k-1 when pod k+1 is independent of it too)
      const RunWait W1{Y, (ph && run_indep(ph, nh)) ? (k ? k - 1 : 0u) : k, &S.go, &S.seen, nullptr, owned, R.spin};
      EvalOut ea;
      ea.abort = false;
      eval_body<ROWM, kRun, PM, LK, TS, BT, 1>(C, F, A1, P + PO[A1.q], &L, &row, &ea, &W1, &pre);
      if (ea.abort) return;
      owned = 0;
      if (rs_on) atomicAdd((unsigned long long*)&rst[40], 1ull);  // (pods whose reads went ahead)
    }
    // ---- fold every block's partials (as reduce_eval)
    EvalTotals E;
    {
      ChainRec& r = E.r;
      rec_init(r);
      bool ok = true;
      if (threadIdx.x < NB) ok = run_read_g1<TS>(G1 + (size_t)threadIdx.x * kGB, tag, xmask, ns, r, Y, R.spin);
      if (__syncthreads_or(!ok)) return;
      RS(31);
      if (rs_on) {  // the latest block's partial vs this pod's start in block 0 (slot 51)
        const uint64_t lt = __hip_atomic_load(&rst[52 + (k & 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lt > rs_t0) atomicAdd((unsigned long long*)&rst[51], (unsigned long long)(lt - rs_t0));
        __hip_atomic_store(&rst[52 + (k & 1)], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      fold_partial<KCX_PTS, KCX_IPA, BT>(r, L.rec, xmask, ns, false);
      RS(39);
      eval_weights(C, h, E);
    }
    RS(32);
    int64_t pmx = INT64_MIN, pmn = INT64_MAX;  // single score constraint: raw is monotone in the count
    if (E.r.mx[KCX_PTS] != INT64_MIN) {
      pmx = pts_raw1(h, E, E.r.mx[KCX_PTS]);
      pmn = pts_raw1(h, E, E.r.mn[KCX_PTS]);
    }
    int64_t smx[KSG_MAX_PLUGINS], smn[KSG_MAX_PLUGINS];
    chain_norms<PM>(F, h, E, smx, smn, pmx, pmn);
    if (b == 0 && threadIdx.x == 0) chain_summary(A, F, h, E, smx, smn, eo.ipa_flags);
    // ---- NormalizeScore, weights, packed key of this block's nodes (final_body)
    ChainRec r;
    rec_init(r);
    if (eo.feasible) {
      int64_t tot = 0;
      bool range_err = false;
#pragma unroll
      for (int pos = 0; pos < kNPos<PM>; ++pos) {
        if (pos >= F.n) continue;
        const int p = F.plugins[pos];
        int64_t sv = eo.raw[pos];
        bool pts_keys = false;
        if (p == KP_PTS) {
          pts_keys = sv >= 0 && ns > 0;
          if (sv < 0) sv = 0;
          else if (ns > 0 && !(h->flags & KPF_SKIP_PTS_SCORE)) sv = pts_raw1(h, E, sv);
        }
        bool use;
        const int64_t v = normalize_pos<PM>(p, h, sv, smx[pos], smn[pos], eo.ipa_flags, pts_keys, use);
        if (use) {
          if (v < 0 || v > 100) range_err = true;
          tot += v * F.weight[pos];
        }
      }
      if (E.r.feas == 1) tot = 0;  // single feasible node: no scoring
      r.key = pack_key(tot, F.seed, h->queue_idx, C.goff + n);
      r.st = (E.r.feas > 1 && range_err) ? 4 : 0;
    }
    RS(47);
    fold_key<BT>(r, L.rec);
    if (threadIdx.x == 0) {
      uint64_t* g = G2 + (size_t)b * kGB;
      st_sc1(g, gran(tag, (uint32_t)r.key));
      st_sc1(g + kGF, gran(tag, (uint32_t)(r.key >> 32)));
      st_sc1(g + 2 * kGF, gran(tag, (uint32_t)r.st));
    }
    RS(33);
    if (rst && threadIdx.x == 0) atomicMax((unsigned long long*)&rst[54 + (k & 1)], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    if (threadIdx.x == BT - 32 && k + 1 < count) {  // the next program header into the scalar cache
      uint32_t warm = 0;
      const uint64_t a = (uint64_t)(P + PO[A.q + 1]);  // (uniform: into scalar registers)
      const uint64_t su = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32);
      KWarm<0, kHdrBytes>::run(reinterpret_cast<const void*>(su), warm);
      warm_wait(warm);  // (the loads land in one scalar register the compiler may reuse: wait here)
    }
    // the next pod's row-only plugins while the keys arrive (not when its reads go
    // ahead: the staged evaluation computes them itself)
    rpre_ok = false;
    if (nh && !tnext) {
      row_pre<ROWM, PM>(row, F, view(P + PO[A.q + 1]).h, C.R, rpre);
      rpre_ok = true;
    }
    // the assume's items (class ids, own affinity terms) into registers while the
    // keys arrive: the owner's commit then issues its atomics without a load
    const uint32_t npm = (uint32_t)h->n_pc_match, nitems = npm + (uint32_t)h->n_exist_terms;
    int32_t it_cls = -1;
    ksg_exist_term it_term;
    it_term.cls = -1;
    if (C.T.on && threadIdx.x < nitems) {
      if (threadIdx.x < npm) it_cls = V.i32[h->pc_match_off + threadIdx.x];
      else it_term = V.et[h->exist_terms_off + (threadIdx.x - npm)];
    }
    // ---- selectHost: every block takes the argmax of every block's key
    ChainRec sk;
    rec_init(sk);
    {
      bool ok = true;
      if (threadIdx.x < NB) {
        const uint64_t* g = G2 + (size_t)threadIdx.x * kGB;
        ok = false;
        // (thread 0 also reads the assume flag: the next pod's wait then needs no poll
        // when this value covers it — every assume before this pod's, normally)
        const uint64_t fseen = threadIdx.x == 0 ? ld_sc1(&Y->flag[0]) : 0;
        for (uint32_t it = 0; it < R.spin; ++it) {
          const uint64_t d = ld_sc1(g + 2 * kGF), a = ld_sc1(g), c = ld_sc1(g + kGF);  // (3 granules: all per poll)
          if (gtag(a, tag) && gtag(c, tag) && gtag(d, tag)) {
            sk.key = (uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)c << 32);
            sk.st = (int32_t)(uint32_t)d;
            ok = true;
            break;
          }
          if (run_aborted(it, Y)) break;
          __builtin_amdgcn_s_sleep(kRunSleep);
        }
        if (!ok && !ld_sc1(&Y->abort[0])) run_raise(Y);
        if (threadIdx.x == 0 && (uint32_t)fseen > S.seen) S.seen = (uint32_t)fseen;
      }
      if (__syncthreads_or(!ok)) return;
    }
    fold_key<BT>(sk, L.rec);
    RS(34);
    if (rs_on) {  // the latest block's key vs this pod's start in block 0 (slot 53)
      const uint64_t lt = __hip_atomic_load(&rst[54 + (k & 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lt > rs_t0) atomicAdd((unsigned long long*)&rst[53], (unsigned long long)(lt - rs_t0));
      __hip_atomic_store(&rst[54 + (k & 1)], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int32_t feas = E.r.feas, st = E.r.st | sk.st;
    const bool error = (st & 2) || ((st & 4) && feas > 1) || (h->flags & KPF_PREFILTER_ERROR) || na_prescore_error(h->flags, feas);
    const uint32_t g = (uint32_t)(sk.key & 0xFFFFFull);
    int32_t node = -1;
    if (!error && feas > 0 && (A.mode & 1) && g >= C.goff && g - C.goff < C.N) node = (int32_t)(g - C.goff);
    if (b == 0 && threadIdx.x == 0) {  // the summary (chain_commit's)
      ksg_pod_summary* Sm = A.sums + A.q;
      Sm->feasible = feas;
      Sm->best_key = sk.key;
      if (error) { Sm->status = 2; Sm->selected = -1; }
      else if (feas == 0) { Sm->status = 1; Sm->selected = -1; }
      else { Sm->status = 0; Sm->selected = (int32_t)g; }
      A.prow[A.q] = -1;
      A.alog[A.q - A.log_base] = make_int2((int)A.q, node >= 0 && (A.mode & 2) ? node : -1);
    }
    if (node >= 0 && (uint32_t)node / BT == b) {
      // ---- the owner: its register row and the node-level class-table entries
      // (only this block reads them; drained before its next class-table reads,
      // run_wait_flag); the committer block applies the rest
      owned = 1;
      const uint64_t c0 = rst && threadIdx.x == 0 ? __builtin_amdgcn_s_memrealtime() : 0;
      const uint32_t ln = (uint32_t)node % BT;
      if (threadIdx.x == ln) {  // (assume_row_atomic's delta)
#pragma unroll
        for (uint32_t c = 0; c < 4; ++c)
          if (c < C.R && (c < 2 || A.need_eph)) row.req[c] += h->req[c];
        row.nzc += h->nz_cpu;
        row.nzm += h->nz_mem;
        row.podcnt += 1;
        if (rpre_ok) row_pre<ROWM, PM>(row, F, view(P + PO[A.q + 1]).h, C.R, rpre);  // (its row changed)
      }
      const bool defer = R.defer && nh && !tnext && nitems <= (uint32_t)BT && (h->nd_md & nh->nd_rd) == 0;
      if (defer) {
        if (C.T.on && threadIdx.x < nitems) {
          dfr_node = (uint32_t)node;
          dfr_is_cls = threadIdx.x < npm;
          dfr_cls = it_cls;
          dfr_term = it_term;
        }
        dfr_any = C.T.on && nitems > 0;
        owned = 0;
      } else if (C.T.on && threadIdx.x < nitems) {
        int32_t v[KSG_MAX_TOPO];
#pragma unroll
        for (int s = 0; s < KSG_MAX_TOPO; ++s) v[s] = (uint32_t)s < C.n_topo ? L.tv[s * BT + ln] : -1;
        if (threadIdx.x < npm) pc_add(C, it_cls, (uint32_t)node, +1, v, TP_NODE);
        else tc_add(C, it_term, (uint32_t)node, +1, v, TP_NODE);
        if (nitems > (uint32_t)BT)  // (items beyond one per thread)
          tables_assume_items(C, V, (uint32_t)node, v, +1, threadIdx.x + BT, BT, TP_NODE);
      }
      if (rst && threadIdx.x == 0) {
        atomicAdd((unsigned long long*)&rst[36], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - c0));
        atomicAdd((unsigned long long*)&rst[37], 1ull);
      }
    }
    // the flag this block waits for before the next pod's class-table reads: every
    // assume up to this pod's if the next pod reads an entry this one writes
    // (tab_rd / tab_md), else every assume before this pod's
    have = tnext;
    if (nh && !tnext) wait_for = (node >= 0 && (h->tab_md & nh->tab_rd) != 0) ? tag : k;
    ph = h;
    RS(50);
    if (rs_on) atomicAdd((unsigned long long*)&rst[35], 1ull);
  }
#undef RS
}
// The committer (the launch's last block, no nodes): per pod it folds the
// feasible count / status from the partial granules and the argmax from the key
// granules like every block, then applies the assume's pair-level part — node
// row atomics, pod-class pc_tot / pc_dom and term-class tc_tot / shared tc_val
// at the node's topology values — drains it and advances the flag.
template <uint32_t PM, int TS, int BT>
__device__ __forceinline__ void run_commit_body(DevCluster& C, const DevProfile& F, const ChainArgs& A0, uint32_t count,
                                                RunSync* Y, const uint64_t* G1s, const uint64_t* G2s, const RunCtl& R,
                                                const uint8_t* __restrict__ P, const uint64_t* __restrict__ PO) {
  __shared__ ChainRec lrec[BT / 64];
  __shared__ uint32_t go;
  if (!run_handshake(Y, R, &go)) return;
  const uint32_t NB = A0.nblk;
  uint32_t xmask = 0;
  for (int p = 0; p < F.n; ++p) {
    const int x = chain_x(F.plugins[p]);
    if (x >= 0) xmask |= 1u << x;
  }
  for (uint32_t k = 0; k < count; ++k) {
    const uint32_t q = A0.q + k, tag = k + 1u;
    const uint64_t* const G1 = G1s + (k & 1u) * kRunSlot;  // (parity slots)
    const uint64_t* const G2 = G2s + (k & 1u) * kRunSlot;
    for (uint32_t i = 0; i < R.lag; ++i) __builtin_amdgcn_s_sleep(127);  // (diagnostic: a lagging committer)
    const uint8_t* prog = P + PO[q];
    const ProgView V = view(prog);
    const ksg_prog* h = V.h;
    const int ns = h->n_tsc_score;
    const uint32_t npm = (uint32_t)h->n_pc_match, nitems = npm + (uint32_t)h->n_exist_terms;
    int32_t it_cls = -1;
    ksg_exist_term it_term;
    it_term.cls = -1;
    if (C.T.on && threadIdx.x < nitems) {
      if (threadIdx.x < npm) it_cls = V.i32[h->pc_match_off + threadIdx.x];
      else it_term = V.et[h->exist_terms_off + (threadIdx.x - npm)];
    }
    ChainRec r;
    rec_init(r);
    bool ok = true;
    if (threadIdx.x < NB) ok = run_read_g1<TS>(G1 + (size_t)threadIdx.x * kGB, tag, xmask, ns, r, Y, R.spin);
    if (__syncthreads_or(!ok)) return;
    fold_partial<KCX_PTS, KCX_IPA, BT>(r, lrec, 0u, 0, false);
    ChainRec sk;
    rec_init(sk);
    ok = true;
    if (threadIdx.x < NB) {
      const uint64_t* g = G2 + (size_t)threadIdx.x * kGB;
      ok = false;
      for (uint32_t it = 0; it < R.spin; ++it) {
        const uint64_t d = ld_sc1(g + 2 * kGF), a = ld_sc1(g), c = ld_sc1(g + kGF);
        if (gtag(a, tag) && gtag(c, tag) && gtag(d, tag)) {
          sk.key = (uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)c << 32);
          sk.st = (int32_t)(uint32_t)d;
          ok = true;
          break;
        }
        if (run_aborted(it, Y)) break;
        __builtin_amdgcn_s_sleep(kRunSleep);
      }
      if (!ok && !ld_sc1(&Y->abort[0])) run_raise(Y);
    }
    if (__syncthreads_or(!ok)) return;
    fold_key<BT>(sk, lrec);
    const int32_t feas = r.feas, st = r.st | sk.st;
    const bool error = (st & 2) || ((st & 4) && feas > 1) || (h->flags & KPF_PREFILTER_ERROR) || na_prescore_error(h->flags, feas);
    const uint32_t g = (uint32_t)(sk.key & 0xFFFFFull);
    if (!error && feas > 0 && (A0.mode & 1) && g >= C.goff && g - C.goff < C.N) {
      const uint32_t node = g - C.goff;
      if (threadIdx.x == 0) assume_row_atomic(C, V, node, +1);
      if (C.T.on && threadIdx.x < nitems) {
        int32_t v[KSG_MAX_TOPO];
        node_slot_vids(C, node, v);
        if (threadIdx.x < npm) pc_add(C, it_cls, node, +1, v, TP_PAIR);
        else tc_add(C, it_term, node, +1, v, TP_PAIR);
        if (nitems > (uint32_t)BT) tables_assume_items(C, V, node, v, +1, threadIdx.x + BT, BT, TP_PAIR);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's atomics performed
    }
    __syncthreads();
    if (threadIdx.x == 0) run_advance(Y, k, R.spin);
  }
}

// Plugin sets with a specialisation (PM): the PodTopologySpread / InterPodAffinity
// profile of cfg4 (with or without TaintToleration / NodeAffinity), every plugin.
constexpr uint32_t kPmTab = (1u << KP_FIT) | (1u << KP_BA) | (1u << KP_PTS) | (1u << KP_IPA);
constexpr uint32_t kPmTabTN = kPmTab | (1u << KP_TAINT) | (1u << KP_NA);
// Size classes: pods with at most kRunLK lookup-plan entries and kRunTS spread
// constraints (cfg4's) run the small instantiation, the others the generic one.
constexpr int kRunLK = 8, kRunTS = 4;
template <int ROWM, uint32_t PM, int LK = KSG_LK_MAX, int TS = KSG_MAX_TSC, int BT = kChain>
__global__ __launch_bounds__(BT) void k_chain_run(DevCluster C, DevProfile F, ChainArgs A, uint32_t count, RunSync* Y,
                                                  uint64_t* G1, uint64_t* G2, RunCtl R, const uint8_t* __restrict__ P,
                                                  const uint64_t* __restrict__ PO) {
  if (blockIdx.x == A.nblk) run_commit_body<PM, TS, BT>(C, F, A, count, Y, G1, G2, R, P, PO);  // (the extra block)
  else run_body<ROWM, PM, LK, TS, BT>(C, F, A, count, Y, G1, G2, R, P, PO);
}

// Kernels.  The *_occ twins cap registers at 4 waves per SIMD (a few spills)
// for clusters of many blocks per CU; the plain ones keep every register for
// the latency of one block per CU (cfg4).
__device__ __forceinline__ void view_body(const DevCluster& C, const DevProfile& F, const uint8_t* prog,
                                          const ksg_pod_summary* sum, const uint32_t* filter, const int32_t* score,
                                          const ViewDev& V, uint8_t* out, uint8_t* hout, uint32_t* done);
template <int ROWM>
__global__ __launch_bounds__(kChain) void k_eval(DevCluster C, DevProfile F, ChainArgs A, const uint8_t* __restrict__ prog) {
  eval_body<ROWM>(C, F, A, prog);
  if (A.vf_hout) {  // fused view: this block's nodes, from the kept outputs it just wrote
    uint32_t* of;
    int32_t *os, *ot;
    chain_outs(A, A.q, C.N, of, os, ot);
    __syncthreads();
    view_body(C, F, prog, nullptr, of, os, A.vf, A.vf_out, A.vf_hout, nullptr);
  }
}
template <int ROWM>
__global__ __launch_bounds__(kChain) __attribute__((amdgpu_waves_per_eu(4))) void k_eval_occ(
    DevCluster C, DevProfile F, ChainArgs A, const uint8_t* __restrict__ prog) {
  eval_body<ROWM>(C, F, A, prog);
}
template <int ROWM>
__global__ __launch_bounds__(kChain) void k_eval_solo(DevCluster C, DevProfile F, ChainArgs A,
                                                      const uint8_t* __restrict__ prog) {
  eval_body<ROWM, kSolo>(C, F, A, prog);
}
template <uint32_t PM = ~0u>
__global__ __launch_bounds__(kChain) void k_final(DevCluster C, DevProfile F, ChainArgs A, const uint8_t* __restrict__ prog) {
  final_body<PM>(C, F, A, prog);
}
__global__ __launch_bounds__(kChain) __attribute__((amdgpu_waves_per_eu(4))) void k_final_occ(
    DevCluster C, DevProfile F, ChainArgs A, const uint8_t* __restrict__ prog) {
  final_body(C, F, A, prog);
}

// The existing-pod table rows of the run's logged assumes, in log order (one
// block): exclusive scans of their entry counts, then every row written at its
// offsets; the programs' prow entries point at them.
__global__ __launch_bounds__(kBlock) void k_flush_appends(DevCluster C, ChainArgs A, uint32_t cnt) {
  __shared__ uint32_t base[4], tot[4];
  __shared__ uint32_t scan[4][kBlock];
  __shared__ int32_t over;
  if (threadIdx.x < 4) base[threadIdx.x] = C.tcounts[threadIdx.x];
  if (threadIdx.x == 0) over = 0;
  __syncthreads();
  const uint32_t cap[4] = {C.pcap, C.tcap, C.rcap, C.vcap};
  for (uint32_t c0 = 0; c0 < cnt; c0 += blockDim.x) {
    const uint32_t i = c0 + threadIdx.x;
    uint32_t need[4] = {0, 0, 0, 0};
    int2 e = make_int2(0, 0);
    if (i < cnt) {
      e = A.alog[i];
      if (e.y >= 0) table_need(view(A.progs + A.prog_off[e.x]), need);
    }
    for (int k = 0; k < 4; ++k) scan[k][threadIdx.x] = need[k];
    __syncthreads();
    for (uint32_t d = 1; d < blockDim.x; d <<= 1) {  // inclusive scans
      uint32_t v[4];
      for (int k = 0; k < 4; ++k) v[k] = threadIdx.x >= d ? scan[k][threadIdx.x - d] : 0;
      __syncthreads();
      for (int k = 0; k < 4; ++k) scan[k][threadIdx.x] += v[k];
      __syncthreads();
    }
    if (threadIdx.x == blockDim.x - 1)
      for (int k = 0; k < 4; ++k) tot[k] = scan[k][threadIdx.x];
    if (i < cnt && e.y >= 0) {
      uint32_t off[4];
      bool fits = true;
      for (int k = 0; k < 4; ++k) {
        off[k] = base[k] + scan[k][threadIdx.x] - need[k];
        fits &= off[k] + need[k] <= cap[k];
      }
      if (fits) {
        table_write(C, view(A.progs + A.prog_off[e.x]), (uint32_t)e.y, off[0], off[1], off[2], off[3]);
        A.prow[e.x] = (int32_t)off[0];
      } else {
        over = 1;  // capacity is checked before every run: never, unless the host's count is wrong
      }
    }
    __syncthreads();
    if (threadIdx.x < 4) base[threadIdx.x] += tot[threadIdx.x];
    __syncthreads();
  }
  if (threadIdx.x < 4) C.tcounts[threadIdx.x] = base[threadIdx.x] < cap[threadIdx.x] ? base[threadIdx.x] : cap[threadIdx.x];
  if (threadIdx.x == 0 && over) C.tcounts[4] = 1;
}

// ---- class tables: build from the existing-pod table
// pod classes [c0, c0 + nc): every live existing pod matching a class adds to its tables
// One thread per existing-pod row; pc_add's counts, with pc_tot (ONE address per
// (class, slot)) counted per wave before its atomic.
// The new classes' definitions (their pool ranges, appended together by
// add_classes) are staged in LDS first when they fit: the per-row selector walk
// then reads LDS instead of a chain of dependent global loads (class -> term ->
// requirement -> values) per row.  st.nt == UINT32_MAX: read the pools in place.
#define KSG_PCB_K 4
struct PcStage {
  uint32_t t0, nt, r0, nr, v0, nv;
  // the distinct label keys the staged requirements name (host-collected; nk >
  // KSG_PCB_K: none): their label columns are read for every row up front, in
  // parallel with the row's own loads, instead of one dependent load per
  // requirement after the class walk reached it
  uint32_t nk;
  int32_t key[KSG_PCB_K];
  // the slots with few domains (hcnt > 0: a zone, not a hostname): their pc_dom
  // entries, like pc_tot, are counted per block in LDS and added once per block.
  // Every matching row of a class adds to one entry of such a slot — with 20
  // zones, 20 addresses in one cache line — so row-level atomics serialise at one
  // L2 channel (class c's entries at LDS c_local * hsum + hbase[slot] + value).
  uint32_t hsum;
  uint16_t hbase[KSG_MAX_TOPO], hcnt[KSG_MAX_TOPO];
};
#define KSG_PCB_C 16
#define KSG_PCB_T 64
#define KSG_PCB_R 128
#define KSG_PCB_V 512
#define KSG_PCB_H 4096
constexpr uint32_t kPcBlock = 1024;  // rows per block (fewer blocks: fewer per-block adds to the hot lines)
__global__ __launch_bounds__(kPcBlock) void k_pc_build(DevCluster C, uint32_t c0, uint32_t nc, PcStage st) {
  __shared__ ksg_pclass s_pc[KSG_PCB_C];
  __shared__ ksg_cterm s_ct[KSG_PCB_T];
  __shared__ ksg_req s_rq[KSG_PCB_R];
  __shared__ int32_t s_cv[KSG_PCB_V];
  __shared__ int32_t s_tot[KSG_PCB_C * KSG_MAX_TOPO];
  __shared__ int32_t s_dom[KSG_PCB_H];
  const bool staged = st.nt != 0xFFFFFFFFu && nc <= KSG_PCB_C && st.nt <= KSG_PCB_T && st.nr <= KSG_PCB_R &&
                      st.nv <= KSG_PCB_V;
  const bool agg = staged && st.hsum > 0 && nc * st.hsum <= KSG_PCB_H;
  const bool pre = staged && st.nk <= KSG_PCB_K;  // requirement keys as indices into kv below
  // the row's loads first, independent of the table use and of the class
  // definitions (rows past the use are read but never counted: p < pcap)
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t pp = p < C.pcap ? p : C.pcap - 1;
  const uint32_t fl = C.ptflags[pp];
  const int32_t node = C.ptnode[pp], ns = C.ptns[pp];
  int32_t kv[KSG_PCB_K];
#pragma unroll
  for (int j = 0; j < KSG_PCB_K; ++j) {
    const int32_t k = st.key[j];
    kv[j] = (pre && (uint32_t)j < st.nk && k >= 0 && (uint32_t)k < C.pkeys) ? C.ptlab[(size_t)k * C.pcap + pp] : -1;
  }
  const bool live = p < C.tcounts[0] && !(fl & KEF_DELETED);
  const ksg_pclass* PCs = C.T.pcls;
  const ksg_cterm* CTs = C.T.cterm;
  const ksg_req* RQs = C.T.creq;
  const int32_t* CVs = C.T.cval;
  uint32_t cbase = 0;
  if (staged) {  // (copies rebased onto the staged ranges: every offset indexes the LDS arrays from 0)
    for (uint32_t i = threadIdx.x; i < nc; i += blockDim.x) {
      ksg_pclass x = C.T.pcls[c0 + i];
      x.term_off -= (int32_t)st.t0;
      s_pc[i] = x;
    }
    for (uint32_t i = threadIdx.x; i < st.nt; i += blockDim.x) {
      ksg_cterm x = C.T.cterm[st.t0 + i];
      x.sel.req_off -= (int32_t)st.r0;
      x.ns_off -= (int32_t)st.v0;
      s_ct[i] = x;
    }
    for (uint32_t i = threadIdx.x; i < st.nr; i += blockDim.x) {
      ksg_req x = C.T.creq[st.r0 + i];
      x.val_off -= (int32_t)st.v0;
      if (pre) {  // key -> its index in st.key (-1: a key the rows never carry)
        int32_t j = -1;
        for (uint32_t t = 0; t < st.nk; ++t)
          if (st.key[t] == x.key) j = (int32_t)t;
        x.key = j;
      }
      s_rq[i] = x;
    }
    for (uint32_t i = threadIdx.x; i < st.nv; i += blockDim.x) s_cv[i] = C.T.cval[st.v0 + i];
    for (uint32_t i = threadIdx.x; i < nc * KSG_MAX_TOPO; i += blockDim.x) s_tot[i] = 0;
    if (agg)
      for (uint32_t i = threadIdx.x; i < nc * st.hsum; i += blockDim.x) s_dom[i] = 0;
    __syncthreads();
    PCs = s_pc;
    CTs = s_ct;
    RQs = s_rq;
    CVs = s_cv;
    cbase = c0;
  }
  auto vid = [&](int32_t k) -> int32_t {
    if (pre) {
      int32_t v = -1;
#pragma unroll
      for (int j = 0; j < KSG_PCB_K; ++j)
        if (k == j) v = kv[j];
      return v;
    }
    return (k >= 0 && (uint32_t)k < C.pkeys) ? C.ptlab[(size_t)k * C.pcap + pp] : -1;
  };
  int32_t nv[KSG_MAX_TOPO];
  node_slot_vids(C, live ? (uint32_t)node : 0u, nv);
  const DevTables& T = C.T;
  for (uint32_t c = c0; c < c0 + nc; ++c) {
    const ksg_pclass pc = PCs[c - cbase];
    bool ok = live && pc.n_terms > 0 && !(pc.excl_term && (fl & KEF_TERMINATING));
    for (int i = 0; i < pc.n_terms && ok; ++i) {
      const ksg_cterm& t = CTs[pc.term_off + i];
      ok = (t.ns_all || in_list(ns, CVs + t.ns_off, t.ns_cnt)) && sel_eval(t.sel, RQs, CVs, vid);
    }
    if (c >= T.npc) continue;  // (pc_add's guard)
    if (ok) atomicAdd(&T.pc_cnt[(size_t)c * C.N + (uint32_t)node], 1);
#pragma unroll
    for (int sl = 0; sl < KSG_MAX_TOPO; ++sl) {
      const bool m = ok && nv[sl] >= 0;
      const uint64_t b = __ballot(m);
      if (!b) continue;
      if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((unsigned long long)b) - 1)) {
        if (staged) atomicAdd(&s_tot[(c - c0) * KSG_MAX_TOPO + sl], (int)__popcll(b));
        else atomicAdd(&T.pc_tot[(size_t)c * KSG_MAX_TOPO + sl], (int)__popcll(b));
      }
      // (per-row domain atomics: a per-wave loop over the distinct domains measured
      // slower — 38 vs 32 µs per build, up to 170 on many-valued slots)
      if (m && C.nubv[sl] >= 0) {
        if (agg && (uint32_t)nv[sl] < st.hcnt[sl]) atomicAdd(&s_dom[(c - c0) * st.hsum + st.hbase[sl] + nv[sl]], 1);
        else atomicAdd(T.pc_dom + (size_t)c * T.NU + (uint32_t)C.nubv[sl] + nv[sl], 1);
      }
    }
  }
  if (!staged) return;
  __syncthreads();  // the block's counts, added once
  for (uint32_t i = threadIdx.x; i < nc * KSG_MAX_TOPO; i += blockDim.x) {
    const uint32_t c = c0 + i / KSG_MAX_TOPO;
    if (s_tot[i] && c < T.npc) atomicAdd(&T.pc_tot[(size_t)c * KSG_MAX_TOPO + i % KSG_MAX_TOPO], s_tot[i]);
  }
  if (agg)
    for (uint32_t i = threadIdx.x; i < nc * st.hsum; i += blockDim.x) {
      const int32_t x = s_dom[i];
      const uint32_t c = c0 + i / st.hsum, r = i % st.hsum;
      if (!x || c >= T.npc) continue;
      for (int sl = 0; sl < KSG_MAX_TOPO; ++sl)
        if (st.hcnt[sl] && r >= st.hbase[sl] && r < (uint32_t)st.hbase[sl] + st.hcnt[sl] && C.nubv[sl] >= 0)
          atomicAdd(T.pc_dom + (size_t)c * T.NU + (uint32_t)C.nubv[sl] + (r - st.hbase[sl]), x);
    }
}
// term classes [u0, ...): every live existing pod's term of such a class
__global__ void k_tc_build(DevCluster C, uint32_t u0) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= C.tcounts[1]) return;
  const int32_t p = C.tpod[t];
  if (C.ptflags[p] & KEF_DELETED) return;
  const ksg_exist_term& e = C.terms[t];
  if (e.cls < 0 || (uint32_t)e.cls < u0) return;
  tc_add(C, e, (uint32_t)C.ptnode[p], +1);
}

// ---- node-sharded class tables: the pair-level entries a rank built from its
// own existing pods are summed across ranks (segments of int32 entries packed
// in one canonical order, all-gathered, summed in place).
struct TabSeg {
  int32_t* p;
  uint32_t len, off;  // entries, offset in the packed vector
};
__global__ void k_seg_pack(const TabSeg* sg, uint32_t nseg, int32_t* out) {
  for (uint32_t k = blockIdx.x; k < nseg; k += gridDim.x) {
    const TabSeg s = sg[k];
    for (uint32_t i = threadIdx.x; i < s.len; i += blockDim.x) out[s.off + i] = s.p[i];
  }
}
__global__ void k_seg_sum(const TabSeg* sg, uint32_t nseg, const int32_t* recv, uint32_t total, uint32_t ranks) {
  for (uint32_t k = blockIdx.x; k < nseg; k += gridDim.x) {
    const TabSeg s = sg[k];
    for (uint32_t i = threadIdx.x; i < s.len; i += blockDim.x) {
      int32_t v = 0;
      for (uint32_t r = 0; r < ranks; ++r) v += recv[(size_t)r * total + s.off + i];
      s.p[i] = v;
    }
  }
}

// Normalized scores of a kept pod (finalscore-result / ksg_normalized_scores):
// NormalizeScore of every position from the pod's raw scores and summary, with
// the normalize_pos the selection used.
__global__ void k_norm_out(DevCluster C, DevProfile F, const uint8_t* prog, const ksg_pod_summary* sum,
                           const uint32_t* filter, const int32_t* score, int32_t* norm) {
  const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= C.N) return;
  const ProgView V = view(prog);
  const ksg_prog* h = V.h;
  const bool feasible = filter[n] == KSG_FILTER_PASS;
  const int nf = h->n_tsc_filter, ns = h->n_tsc_score;
  const bool pts_keys = ns > 0 && pts_has_keys(C, V, nf, nf + ns, n);
  for (int pos = 0; pos < F.n; ++pos) {
    int64_t s = 0;
    if (feasible) {
      bool use;
      s = normalize_pos(F.plugins[pos], h, score[(size_t)pos * C.N + n], sum->max_score[pos], sum->min_score[pos],
                        sum->ipa_flags, pts_keys, use);
    }
    norm[(size_t)pos * C.N + n] = (int32_t)s;
  }
}

// ---- ksg_cycle_view on the device (the drop-in path's per-node lookups).  One
// thread per node turns the kept filter code into what the framework's Filter
// call returns there: the first failing profile position, its framework code
// (Fit: UnschedulableAndUnresolvable when a failing request exceeds the node's
// allocatable, fit.go) and a message index — the slot of the code in a small
// open-addressing table of the pod's distinct failing codes (each wave inserts a
// code once), whose text the host renders per slot.  It also copies the raw
// scores and writes NormalizeScore's output for the normalising positions, so
// one device-to-host copy carries the whole view (wrappedplugin.go:523-548
// Filter, :420-445 Score, :388-415 NormalizeScore).
constexpr int kViewSlots = 256;
enum { kVkUnresolvable = 0, kVkUnsched = 1, kVkFit = 2, kVkPts = 3, kVkIpa = 4 };
// Score-row widths of a view, the same in every thread: 1 byte for the rows whose
// values are within [0, 100] by construction when the cycle has no Score error
// (Fit and BalancedAllocation raw, every normalized row); PodTopologySpread's and
// InterPodAffinity's raw rows as narrow as the summary's range over the feasible
// nodes allows (1, 2 or 4 bytes; the range widened by PodTopologySpread's -1 of
// an ignored node and 0), else 4; rows packed from off_raw, each 256-B aligned.
// (Values of nodes that failed a filter are unspecified in the view: clamped.)
// (sum null: a fused view, written before the summary exists -- no Score error
// assumed, PodTopologySpread / InterPodAffinity rows, which need ScoreExtensions
// and so never fuse, at 4 bytes; the host rebuilds the view when the summary
// reports an error)
__device__ __forceinline__ void view_rows(const DevProfile& F, const ViewDev& V, const ksg_pod_summary* sum, uint32_t N,
                                          Engine::ViewRows& R) {
  const bool err = sum != nullptr && sum->status == 2;
  uint32_t off = V.off_raw;
  auto al = [](uint32_t x) { return (x + 255u) & ~255u; };
  for (int d = 0; d < 2 * KSG_MAX_PLUGINS; ++d) {
    R.off[d] = 0;
    R.bytes[d] = 0;
  }
  for (int d = 0; d < F.n; ++d) {
    const int p = F.plugins[d];
    uint8_t w = 4;
    if (!err && (p == KP_FIT || p == KP_BA)) {
      w = 1;
    } else if (!err && V.narrow && sum != nullptr && (p == KP_PTS || p == KP_IPA)) {
      int64_t lo = sum->min_score[d], hi = sum->max_score[d];
      if (lo == INT64_MAX || hi == INT64_MIN) lo = hi = 0;  // (no feasible / counted node)
      lo = lo < -1 ? lo : -1;
      hi = hi > 0 ? hi : 0;
      w = (lo >= -128 && hi <= 127) ? 1 : (lo >= -32768 && hi <= 32767) ? 2 : 4;
    }
    R.bytes[d] = w;
    R.off[d] = off;
    off += al(N * R.bytes[d]);
  }
  for (uint32_t r = 0; r < V.n_norm; ++r) {
    R.bytes[KSG_MAX_PLUGINS + r] = err ? 4 : 1;
    R.off[KSG_MAX_PLUGINS + r] = off;
    off += al(N * R.bytes[KSG_MAX_PLUGINS + r]);
  }
}
__device__ __forceinline__ void view_put(uint8_t* base, uint32_t off, uint8_t w, uint32_t n, int64_t v) {
  if (w == 1) reinterpret_cast<int8_t*>(base + off)[n] = (int8_t)(v < -128 ? -128 : v > 127 ? 127 : v);
  else if (w == 2) reinterpret_cast<int16_t*>(base + off)[n] = (int16_t)(v < -32768 ? -32768 : v > 32767 ? 32767 : v);
  else reinterpret_cast<int32_t*>(base + off)[n] = (int32_t)v;
}
// slot of `code` in the table (entries of other generations count as empty: no
// clearing per view).  htab (or null): the host block's copy of the table, zeroed
// by the host before the launch — a claimed slot never changes within a
// generation, so the claiming lane writes it there too.
__device__ __forceinline__ uint32_t view_slot(unsigned long long* tab, uint32_t gen, uint32_t code,
                                              unsigned long long* htab) {
  const unsigned long long want = ((unsigned long long)gen << 32) | code;
  uint32_t h = (code * 2654435761u) >> 24;
  for (int k = 0; k < kViewSlots; ++k) {
    unsigned long long cur = __hip_atomic_load(&tab[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while ((uint32_t)(cur >> 32) != gen) {  // stale: claim it
      const unsigned long long old = atomicCAS(&tab[h], cur, want);
      if (old == cur) {
        if (htab) htab[h] = want;
        return h;
      }
      cur = old;
    }
    if (cur == want) return h;
    h = (h + 1) & (kViewSlots - 1);
  }
  atomicMax(&tab[kViewSlots], (unsigned long long)gen << 32);  // overflow (the host renders the view itself)
  if (htab) htab[kViewSlots] = (unsigned long long)gen << 32;
  return kViewSlots;
}
// out: the device block (slot table, summary); hout: where the per-node arrays go —
// the host's pinned block itself (written over the link by this kernel, no copy
// launch after it) or out.
// (sum null: a fused view inside k_eval -- the per-node part only; its last block
// writes the summary and the row table, view_fused_tail)
__device__ __forceinline__ void view_body(const DevCluster& C, const DevProfile& F, const uint8_t* prog,
                                          const ksg_pod_summary* sum, const uint32_t* filter, const int32_t* score,
                                          const ViewDev& V, uint8_t* out, uint8_t* hout, uint32_t* done) {
  const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = n < C.N;
  const ProgView PV = view(prog);
  const ksg_prog* h = PV.h;
  const uint32_t code = act ? filter[n] : KSG_FILTER_NOT_EVALUATED;
  int fp = -1, fc = 0;
  bool need = false;
  if (code == KSG_FILTER_PASS) {
    fp = V.n_profile;
  } else if (code != KSG_FILTER_NOT_EVALUATED) {
    const uint32_t d = code >> 24;
    const bool vol = V.dev_vol[d] != 0;
    fp = V.prof_of_dev[d] + (vol ? (int)((code >> 16) & 0xFFu) : 0);
    const uint32_t detail = vol ? code & 0xFFFFu : code & 0xFFFFFFu;
    switch (V.kind[fp]) {
      case kVkUnsched: fc = 2; break;
      case kVkFit:
        fc = 2;
        for (uint32_t r = 0; r < C.R && r < KSG_MAX_RES; ++r)
          if ((detail >> (1 + r)) & 1u)
            if (h->req[r] > C.alloc[(size_t)r * C.N + n]) fc = 3;
        break;
      case kVkPts: fc = detail == KSG_PTS_MISSING_LABEL ? 3 : 2; break;
      case kVkIpa: fc = detail == KSG_IPA_AFFINITY ? 3 : 2; break;
      default: fc = 3;
    }
    need = true;
  }
  // message slots: one insert per distinct code of the wave
  unsigned long long* tab = reinterpret_cast<unsigned long long*>(out);
  if (n == 0 && hout == out && sum) *reinterpret_cast<ksg_pod_summary*>(out + V.off_sum) = *sum;
  uint32_t msg = 0;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t m = __ballot(need); m; m = __ballot(need)) {
    const int leader = __ffsll((long long)m) - 1;
    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)code, leader);
    uint32_t s = 0;
    if ((int)lane == leader)
      s = view_slot(tab, V.gen, c0,
                    (hout != out && V.slots_direct) ? reinterpret_cast<unsigned long long*>(hout) : nullptr);
    s = (uint32_t)__builtin_amdgcn_readlane((int)s, leader);
    if (need && code == c0) {
      msg = s < kViewSlots ? s + 1 : 0;
      need = false;
    }
  }
  Engine::ViewRows RW;
  view_rows(F, V, sum, C.N, RW);
  if (n == 0 && sum) {  // (direct: straight into the host block, like the per-node arrays)
    *reinterpret_cast<Engine::ViewRows*>(hout + V.off_rows) = RW;
    *reinterpret_cast<ksg_pod_summary*>(hout + V.off_sum) = *sum;
  }
  // The block's per-node arrays are staged in LDS (one segment of 256 entries
  // per array, in the block layout's order) and written out in 16-byte pieces:
  // wide writes over the host link instead of one 1-4 byte write per lane (round 5).
  __shared__ __attribute__((aligned(16))) uint8_t vst[256 * (4 + 8 * KSG_MAX_PLUGINS)];
  const uint32_t tid = threadIdx.x;
  auto lput = [&](uint32_t loff, uint8_t w, int64_t v) {
    if (w == 1) reinterpret_cast<int8_t*>(vst + loff)[tid] = (int8_t)(v < -128 ? -128 : v > 127 ? 127 : v);
    else if (w == 2) reinterpret_cast<int16_t*>(vst + loff)[tid] = (int16_t)(v < -32768 ? -32768 : v > 32767 ? 32767 : v);
    else reinterpret_cast<int32_t*>(vst + loff)[tid] = (int32_t)v;
  };
  uint32_t lraw[KSG_MAX_PLUGINS], lnorm[KSG_MAX_PLUGINS];  // LDS segment offsets (uniform)
  uint32_t lo = 1024;
  for (int d = 0; d < KSG_MAX_PLUGINS; ++d) {
    lraw[d] = lo;
    if (d < F.n) lo += 256u * RW.bytes[d];
  }
  for (int r = 0; r < KSG_MAX_PLUGINS; ++r) {
    lnorm[r] = lo;
    if ((uint32_t)r < V.n_norm) lo += 256u * RW.bytes[KSG_MAX_PLUGINS + r];
  }
  if (act) {
    reinterpret_cast<int8_t*>(vst)[tid] = (int8_t)fp;
    reinterpret_cast<int8_t*>(vst + 256)[tid] = (int8_t)fc;
    reinterpret_cast<uint16_t*>(vst + 512)[tid] = (uint16_t)msg;
    const bool feasible = code == KSG_FILTER_PASS;
    const int nf = h->n_tsc_filter, ns = h->n_tsc_score;
    bool pts_keys = false, pk_done = false;
    for (int pos = 0; pos < F.n; ++pos) {
      const int32_t s = score[(size_t)pos * C.N + n];
      lput(lraw[pos], RW.bytes[pos], s);
      const int r = V.norm_row[pos];
      if (r < 0 || !sum) continue;
      int64_t v = 0;
      if (feasible) {
        if (F.plugins[pos] == KP_PTS && !pk_done) {
          pts_keys = ns > 0 && pts_has_keys(C, PV, nf, nf + ns, n);
          pk_done = true;
        }
        bool use;
        v = normalize_pos(F.plugins[pos], h, s, sum->max_score[pos], sum->min_score[pos], sum->ipa_flags, pts_keys, use);
      }
      lput(lnorm[r], RW.bytes[KSG_MAX_PLUGINS + r], v);
    }
  }
  __syncthreads();
  {
    const uint32_t n0 = blockIdx.x * blockDim.x, cnt = C.N - n0 < blockDim.x ? C.N - n0 : blockDim.x;
    auto flush = [&](uint32_t loff, uint32_t dst, uint32_t w) {  // entries [n0, n0 + cnt) of one array
      uint8_t* d = hout + dst + (size_t)n0 * w;
      const uint8_t* src = vst + loff;
      const uint32_t bytes = cnt * w, n16 = bytes / 16;
      for (uint32_t i = tid; i < n16; i += blockDim.x)
        reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(src)[i];
      for (uint32_t i = n16 * 16 + tid; i < bytes; i += blockDim.x) d[i] = src[i];
    };
    flush(0, V.off_fail_pos, 1);
    flush(256, V.off_fail_code, 1);
    flush(512, V.off_fail_msg, 2);
    for (int d = 0; d < F.n; ++d) flush(lraw[d], RW.off[d], RW.bytes[d]);
    for (uint32_t r = 0; r < V.n_norm; ++r) flush(lnorm[r], RW.off[KSG_MAX_PLUGINS + r], RW.bytes[KSG_MAX_PLUGINS + r]);
  }
  // direct: the last block to finish copies the message-slot table (every
  // block's inserts done) into the host block, so no copy launch follows
  if (hout != out && done && !V.slots_direct) {
    __shared__ uint32_t last;
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      last = atomicAdd(done, 1u) == gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (last) {
      __threadfence();
      unsigned long long* htab = reinterpret_cast<unsigned long long*>(hout);
      for (uint32_t i = threadIdx.x; i <= (uint32_t)kViewSlots; i += blockDim.x)
        htab[i] = __hip_atomic_load(&tab[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (threadIdx.x == 0) *done = 0;  // (the next view's count)
    }
  }
}
__global__ __launch_bounds__(256) void k_view(DevCluster C, DevProfile F, const uint8_t* prog, const ksg_pod_summary* sum,
                                              const uint32_t* filter, const int32_t* score, ViewDev V, uint8_t* out,
                                              uint8_t* hout, uint32_t* done) {
  view_body(C, F, prog, sum, filter, score, V, out, hout, done);
}
// A fused view's last part, by the cycle's last block once its summary is out:
// the summary and the row table into the caller's block (thread 0)
__device__ __forceinline__ void view_fused_tail(const DevCluster& C, const DevProfile& F, const ChainArgs& A) {
  if (threadIdx.x != 0) return;
  const ksg_pod_summary* sum = A.sums + A.q;
  Engine::ViewRows RW;
  view_rows(F, A.vf, nullptr, C.N, RW);
  *reinterpret_cast<Engine::ViewRows*>(A.vf_hout + A.vf.off_rows) = RW;
  *reinterpret_cast<ksg_pod_summary*>(A.vf_hout + A.vf.off_sum) = *sum;
}
