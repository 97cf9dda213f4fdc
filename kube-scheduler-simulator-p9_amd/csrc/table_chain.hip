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
//   k_final  every block reduces the partials it needs, then per node:
//            NormalizeScore, [0,100] check, weights, packed argmax key; per
//            block the best key
//   k_select one block: selectHost over the block keys, the summary, and the
//            assume (node row, class tables, existing-pod table)
//
// The pod index lives on the device (A.cur, advanced by k_select), so a run of
// pods is the same launches repeated (and a HIP graph can replay them).
// Upstream: schedule_one.go findNodesThatPassFilters / prioritizeNodes /
// selectHost, framework.go RunFilterPlugins / RunScorePlugins, the plugins'
// Filter / Score / NormalizeScore (restated in oracle/ksg_oracle.cpp).

struct ChainArgs {
  const uint8_t* progs;
  const uint64_t* prog_off;
  uint32_t* cur;           // pod index of the running cycle (device)
  uint32_t end;            // cycles stop at this queue index
  ksg_pod_summary* sums;
  uint32_t keep_first, keep_n;
  uint32_t* kfilter;
  int32_t *kscore, *ktotal;
  uint32_t* filter;        // outputs of pods not kept
  int32_t *score, *total;
  uint32_t nblk;           // blocks of k_eval / k_ptsraw / k_final
  int32_t* pi;             // [KCP_I][nblk] feasible, ignored, status bits
  int64_t* pm;             // [2 * KCP_X][nblk] normaliser max / min per normalised plugin
  uint64_t* pr;            // [KSG_MAX_TSC][nblk] registered values of small score keys (bit = value)
  int64_t* pm2;            // [2][nblk] PodTopologySpread raw max / min (k_ptsraw)
  uint64_t* pk;            // [nblk] best key of the block (k_final, or k_eval without normalised plugins)
  int32_t* pst;            // [nblk] status bits of k_final
  int mode;                // commit mode (as k_commit)
  int32_t* prow;           // existing-pod table row of each queue pod
};

enum { KCP_FEAS = 0, KCP_IGN = 1, KCP_STAT = 2, KCP_I = 3 };
enum { KCX_TAINT = 0, KCX_NA = 1, KCX_PTS = 2, KCX_IPA = 3, KCP_X = 4 };
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

// block reductions through LDS (one value per wave, then lane 0 of wave 0)
template <class T, class Op>
__device__ __forceinline__ T block_reduce(T v, T* red, Op op) {
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if (lane0()) red[w] = v;
  __syncthreads();
  T r = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = op(r, red[i]);
  return r;
}

// PodTopologySpread score count of constraint c at local node n (its pair's
// TopologyPairToPodCounts, or the node's own count for the hostname key).
__device__ __forceinline__ int64_t pts_count_tab(const DevCluster& C, const ProgView& V, int c, uint32_t n, int32_t v) {
  const ksg_tsc& t = V.h->tsc[c];
  if (t.is_hostname) return t.cls < 0 ? 0 : C.T.pc_cnt[(size_t)t.cls * C.N + n];
  int64_t s = 0;
  for (int k = 0; k < t.sc_n; ++k) s += pc_count(C, V.i32[t.sc_off + k], t.topo, n, v);
  return s;
}

// InterPodAffinity's map-emptiness bits from the class tables, this thread's
// share (OR over the block): bit0 affinityCounts non-empty (a pod matching every
// required term on a node with a term's key), bit2 an existing pod's required
// anti-affinity term matches the pod (existingAntiAffinityCounts), bit3 the
// topology score map is non-empty (PreScore not Skip).
__device__ uint32_t ipa_table_bits(const DevCluster& C, const DevProfile& F, const ProgView& V) {
  const ksg_prog* h = V.h;
  const ksg_aterm* aff = V.at + h->aterm_off;
  const ksg_aterm* pref = aff + h->n_req_aff + h->n_req_anti;
  const int npref = (h->flags & KPF_IPA_HAS_CONSTRAINTS) ? h->n_pref_aff + h->n_pref_anti : 0;
  const bool score_on = !(F.ipa_ignore_existing_pref && !(h->flags & KPF_IPA_HAS_CONSTRAINTS));
  const int nt = h->n_req_aff + npref + h->n_tc_match;
  uint32_t bits = 0;
  for (int i = threadIdx.x; i < nt; i += blockDim.x) {
    if (i < h->n_req_aff) {
      if (h->aff_cls >= 0 && C.T.pc_tot[(size_t)h->aff_cls * KSG_MAX_TOPO + aff[i].topo] > 0) bits |= 1u;
    } else if (i < h->n_req_aff + npref) {
      const ksg_aterm& t = pref[i - h->n_req_aff];
      if (t.cls >= 0 && C.T.pc_tot[(size_t)t.cls * KSG_MAX_TOPO + t.topo] > 0) bits |= 8u;
    } else {
      const int j = i - h->n_req_aff - npref;
      if (C.T.tc_tot[V.i32[h->tc_match_off + j]] > 0) {
        const int grp = V.i32[h->tc_match_off + h->n_tc_match + j];
        if (grp == KSG_TC_ANTI) bits |= 4u;
        else if (score_on && (grp == KSG_TC_PREF || F.ipa_hard_weight > 0)) bits |= 8u;
      }
    }
  }
  return bits;
}

// Pod-uniform inputs of k_eval, per block: minMatchNum of every filter
// constraint (the smallest count over the key's values present on nodes) and
// InterPodAffinity's map-emptiness bits.
struct EvalShared {
  int32_t tv[KSG_MAX_TOPO * kBlock];
  int32_t minm[KSG_MAX_TSC];
  uint32_t ipa_flags;
  int64_t red64[kBlock / 64];
  uint64_t redu[kBlock / 64];
  int32_t red32[kBlock / 64];
};

__device__ void eval_setup(const DevCluster& C, const DevProfile& F, const ProgView& V, EvalShared& L, bool pts_on,
                           bool ipa_on) {
  const ksg_prog* h = V.h;
  if (threadIdx.x < KSG_MAX_TSC) L.minm[threadIdx.x] = 0x7FFFFFFF;
  if (threadIdx.x == 0) L.ipa_flags = 0;
  __syncthreads();
  if (pts_on && !(h->flags & KPF_SKIP_PTS_FILTER)) {
    for (int c = 0; c < h->n_tsc_filter; ++c) {
      const ksg_tsc& t = h->tsc[c];
      const uint32_t base = C.tbase[t.topo], cnt = C.tcount[t.topo];
      int32_t m = 0x7FFFFFFF;
      for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x)
        if (C.T.pair_node[base + i]) {
          const int32_t x = t.eff_cls < 0 ? 0 : C.T.pc_dom[(size_t)t.eff_cls * C.T.NU + C.T.nu_base[t.topo] + i];
          m = x < m ? x : m;
        }
      m = wave_min(m);
      if (lane0() && m != 0x7FFFFFFF) atomicMin(&L.minm[c], m);
    }
  }
  if (ipa_on) {
    const uint32_t bits = __ockl_wfred_or_u32(ipa_table_bits(C, F, V));
    if (lane0() && bits) atomicOr(&L.ipa_flags, bits);
  }
  __syncthreads();
}

__global__ __launch_bounds__(kBlock) void k_eval(DevCluster C, DevProfile F, ChainArgs A) {
  const uint32_t q = *A.cur;
  if (q >= A.end) return;
  const ProgView V = view(A.progs + A.prog_off[q]);
  const ksg_prog* h = V.h;
  __shared__ EvalShared L;
  uint32_t* of;
  int32_t *os, *ot;
  chain_outs(A, q, C.N, of, os, ot);
  const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
  const bool active = n < C.N;
  int pts_pos = -1, ipa_pos = -1;
  for (int p = 0; p < F.n; ++p) {
    if (F.plugins[p] == KP_PTS) pts_pos = p;
    if (F.plugins[p] == KP_IPA) ipa_pos = p;
  }
  load_slot_vids(C, n, active, L.tv);
  const SlotVids tv{L.tv + threadIdx.x};
  eval_setup(C, F, V, L, pts_pos >= 0, ipa_pos >= 0);
  const uint32_t ipa_flags = L.ipa_flags;
  const ksg_aterm* aff = V.at + h->aterm_off;
  const ksg_aterm* anti = aff + h->n_req_aff;
  const ksg_aterm* pref = anti + h->n_req_anti;
  uint32_t code = KSG_FILTER_NOT_EVALUATED;
  bool err = false;
  if (active && !(h->flags & KPF_PREFILTER_REJECT) &&
      !((h->flags & KPF_RESTRICT) && !bit(V.u32 + h->restrict_off, h->restrict_words, (int32_t)n))) {
    code = KSG_FILTER_PASS;
#pragma unroll 1
    for (int pos = 0; pos < F.n; ++pos) {
      uint32_t detail = 0;
      bool fail = false;
      switch (F.plugins[pos]) {
        case KP_FIT: {
          const uint32_t b = fit_filter(C, V, n);
          if (b) { fail = true; detail = b; }
          break;
        }
        case KP_TAINT: {
          const int32_t t = untolerated_taint(C, V, n);
          if (t >= 0) { fail = true; detail = (uint32_t)t; }
          break;
        }
        case KP_NA:
          if (!(h->flags & KPF_SKIP_NA_FILTER) && !required_na(C, V, n)) fail = true;
          break;
        case KP_PTS:  // filtering.go: skew = matchNum + selfMatch - minMatchNum > maxSkew
          if (!(h->flags & KPF_SKIP_PTS_FILTER))
            for (int c = 0; c < h->n_tsc_filter; ++c) {
              const ksg_tsc& t = h->tsc[c];
              const int32_t v = tv(t.topo);
              const int32_t dom = C.T.slot_dom[t.topo];
              if (v < 0) { fail = true; detail = KSG_PTS_MISSING_LABEL; break; }
              if (dom == 0) { err = true; break; }  // minMatchNum: no domains -> Error
              const int64_t mn = dom < t.min_domains ? 0 : L.minm[c];
              if ((int64_t)pc_count(C, t.eff_cls, t.topo, n, v) + t.self_match - mn > t.max_skew) {
                fail = true;
                detail = KSG_PTS_SKEW;
                break;
              }
            }
          break;
        case KP_IPA: {  // filtering.go: affinity, anti-affinity, existing pods' anti-affinity
          bool pods_exist = true, miss = false;
          for (int i = 0; i < h->n_req_aff; ++i) {
            const int32_t v = tv(aff[i].topo);
            if (v < 0) { miss = true; break; }
            if (pc_count(C, h->aff_cls, aff[i].topo, n, v) <= 0) pods_exist = false;
          }
          if (miss || (!pods_exist && !(!(ipa_flags & 1u) && h->self_matches_all))) {
            fail = true;
            detail = KSG_IPA_AFFINITY;
            break;
          }
          for (int i = 0; i < h->n_req_anti && !fail; ++i) {
            const int32_t v = tv(anti[i].topo);
            if (v >= 0 && pc_count(C, anti[i].cls, anti[i].topo, n, v) > 0) { fail = true; detail = KSG_IPA_ANTI_AFFINITY; }
          }
          if (!fail && (ipa_flags & 4u))
            for (int i = 0; i < h->n_tc_match; ++i) {
              if (V.i32[h->tc_match_off + h->n_tc_match + i] != KSG_TC_ANTI) continue;
              const int32_t u = V.i32[h->tc_match_off + i];
              if (tc_value(C, u, n, tv(C.T.tc_slot[u])) > 0) { fail = true; detail = KSG_IPA_EXISTING_ANTI; break; }
            }
          break;
        }
        case KP_UNSCHED: fail = unsched_fails(C, V, n); break;
        case KP_NODENAME: fail = nodename_fails(C, V, n); break;
        case KP_PORTS:
          if (!(h->flags & KPF_SKIP_PORTS)) fail = ports_fail(C, V, n);
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
  if (active) of[n] = code;
  // raw scores, the normalisers' inputs, PodTopologySpread registration
  const int nf = h->n_tsc_filter, ns = h->n_tsc_score;
  const bool pts_score = pts_pos >= 0 && ns > 0 && !(h->flags & KPF_SKIP_PTS_SCORE);
  bool counted = false;
  if (feasible && pts_score) {
    counted = true;
    for (int c = nf; c < nf + ns; ++c) counted &= tv(h->tsc[c].topo) >= 0;
  }
  int64_t mx[KCP_X], mn[KCP_X];
#pragma unroll
  for (int x = 0; x < KCP_X; ++x) {
    mx[x] = INT64_MIN;
    mn[x] = INT64_MAX;
  }
  int64_t tot = 0;
  bool range_err = false;
  if (feasible) {
    const bool score_on = !(F.ipa_ignore_existing_pref && !(h->flags & KPF_IPA_HAS_CONSTRAINTS));
#pragma unroll 1
    for (int pos = 0; pos < F.n; ++pos) {
      const int p = F.plugins[pos];
      int64_t sc = 0;
      switch (p) {
        case KP_FIT: sc = fit_score(C, F, V, n); break;
        case KP_BA: sc = ba_score(C, F, V, n); break;
        case KP_TAINT: sc = taint_score(C, V, n); break;
        case KP_NA: sc = (h->flags & KPF_SKIP_NA_SCORE) ? 0 : na_score(C, V, n); break;
        case KP_IMAGE: sc = image_score(C, V, n); break;
        case KP_IPA: {  // scoring.go: the topology score map, read at the node's (key, value) pairs
          if (h->flags & KPF_IPA_HAS_CONSTRAINTS)
            for (int i = 0; i < h->n_pref_aff + h->n_pref_anti; ++i) {
              const ksg_aterm& t = pref[i];
              const int64_t k = pc_count(C, t.cls, t.topo, n, tv(t.topo));
              sc += i < h->n_pref_aff ? k * t.weight : -k * t.weight;
            }
          if (score_on)
            for (int i = 0; i < h->n_tc_match; ++i) {
              const int grp = V.i32[h->tc_match_off + h->n_tc_match + i];
              if (grp == KSG_TC_ANTI || (grp == KSG_TC_HARD && F.ipa_hard_weight <= 0)) continue;
              const int32_t u = V.i32[h->tc_match_off + i];
              const int64_t k = tc_value(C, u, n, tv(C.T.tc_slot[u]));
              sc += grp == KSG_TC_HARD ? k * F.ipa_hard_weight : k;
            }
          break;
        }
        case KP_PTS:  // the count of the single score constraint (or a placeholder); -1: ignored node
          if (!pts_score) sc = 0;
          else if (!counted) sc = -1;
          else if (h->tab & KTAB_PTS_MULTI) sc = 0;
          else sc = pts_count_tab(C, V, nf, n, tv(h->tsc[nf].topo));
          break;
        default: break;
      }
      os[(size_t)pos * C.N + n] = (int32_t)sc;
      const int x = chain_x(p);
      if (x >= 0 && (p != KP_PTS || counted)) {
        mx[x] = sc > mx[x] ? sc : mx[x];
        mn[x] = sc < mn[x] ? sc : mn[x];
      }
      if (!F.has_ext) {
        if (sc < 0 || sc > 100) range_err = true;
        tot += sc * F.weight[pos];
      }
    }
  }
  // per block partials
  const uint32_t b = blockIdx.x, NB = A.nblk;
  const int32_t feas = block_reduce<int32_t>(wave_sum(feasible ? 1 : 0), L.red32, [](int32_t x, int32_t y) { return x + y; });
  const int32_t ign = block_reduce<int32_t>(wave_sum(feasible && pts_score && !counted ? 1 : 0), L.red32,
                                            [](int32_t x, int32_t y) { return x + y; });
  const int32_t st = block_reduce<int32_t>((int32_t)__ockl_wfred_or_u32((err ? 2u : 0u) | (range_err ? 4u : 0u)), L.red32,
                                           [](int32_t x, int32_t y) { return x | y; });
  if (threadIdx.x == 0) {
    A.pi[KCP_FEAS * NB + b] = feas;
    A.pi[KCP_IGN * NB + b] = ign;
    A.pi[KCP_STAT * NB + b] = st;
  }
  if (F.has_ext) {
#pragma unroll
    for (int x = 0; x < KCP_X; ++x) {
      const int64_t a = block_reduce<int64_t>(wave_max(mx[x]), L.red64, [](int64_t u, int64_t w) { return u > w ? u : w; });
      const int64_t c = block_reduce<int64_t>(wave_min(mn[x]), L.red64, [](int64_t u, int64_t w) { return u < w ? u : w; });
      if (threadIdx.x == 0) {
        A.pm[(2 * x) * NB + b] = a;
        A.pm[(2 * x + 1) * NB + b] = c;
      }
    }
    for (int c = nf; c < nf + ns; ++c) {  // registered values of the score constraints' small keys (initPreScoreState)
        const ksg_tsc& t = h->tsc[c];
        uint64_t m = 0;
        const int32_t v = tv(t.topo);
        if (counted && !t.is_hostname && t.first_of_key && !((C.T.uniq >> t.topo) & 1u) && v < KSG_TAB_REGV)
          m = 1ull << v;
        m = (uint64_t)__ockl_wfred_or_u32((uint32_t)m) | ((uint64_t)__ockl_wfred_or_u32((uint32_t)(m >> 32)) << 32);
        const uint64_t all = block_reduce<uint64_t>(m, L.redu, [](uint64_t u, uint64_t w) { return u | w; });
        if (threadIdx.x == 0) A.pr[(size_t)(c - nf) * NB + b] = all;
      }
  } else {
    const uint64_t key = feasible ? pack_key(tot, F.seed, h->queue_idx, C.goff + n) : 0;
    if (feasible) ot[n] = (int32_t)tot;
    const uint64_t best = block_reduce<uint64_t>(wave_max(key), L.redu, [](uint64_t u, uint64_t w) { return u > w ? u : w; });
    if (threadIdx.x == 0) {
      A.pk[b] = best;
      A.pst[b] = 0;
    }
  }
}

// Reduce k_eval's partials (every block of k_ptsraw / k_final does it for itself).
struct EvalTotals {
  int32_t feasible, ignored, status;
  int64_t mx[KCP_X], mn[KCP_X];
  uint64_t reg[KSG_MAX_TSC];
  double w[KSG_MAX_TSC];
};
__device__ void reduce_eval(const ChainArgs& A, const ksg_prog* h, uint32_t C_uniq, EvalTotals& E, int64_t* red64,
                            uint64_t* redu, int32_t* red32) {
  const uint32_t NB = A.nblk;
  int32_t f = 0, ig = 0, st = 0;
  int64_t mx[KCP_X], mn[KCP_X];
  for (int x = 0; x < KCP_X; ++x) { mx[x] = INT64_MIN; mn[x] = INT64_MAX; }
  uint64_t reg[KSG_MAX_TSC] = {};
  const int ns = h->n_tsc_score;
  for (uint32_t b = threadIdx.x; b < NB; b += blockDim.x) {
    f += A.pi[KCP_FEAS * NB + b];
    ig += A.pi[KCP_IGN * NB + b];
    st |= A.pi[KCP_STAT * NB + b];
    for (int x = 0; x < KCP_X; ++x) {
      const int64_t a = A.pm[(2 * x) * NB + b], c = A.pm[(2 * x + 1) * NB + b];
      mx[x] = a > mx[x] ? a : mx[x];
      mn[x] = c < mn[x] ? c : mn[x];
    }
    for (int c = 0; c < ns; ++c) reg[c] |= A.pr[(size_t)c * NB + b];
  }
  E.feasible = block_reduce<int32_t>(wave_sum(f), red32, [](int32_t x, int32_t y) { return x + y; });
  E.ignored = block_reduce<int32_t>(wave_sum(ig), red32, [](int32_t x, int32_t y) { return x + y; });
  E.status = block_reduce<int32_t>((int32_t)__ockl_wfred_or_u32((uint32_t)st), red32, [](int32_t x, int32_t y) { return x | y; });
  for (int x = 0; x < KCP_X; ++x) {
    E.mx[x] = block_reduce<int64_t>(wave_max(mx[x]), red64, [](int64_t u, int64_t w) { return u > w ? u : w; });
    E.mn[x] = block_reduce<int64_t>(wave_min(mn[x]), red64, [](int64_t u, int64_t w) { return u < w ? u : w; });
  }
  for (int c = 0; c < ns; ++c) {
    const uint64_t m = (uint64_t)__ockl_wfred_or_u32((uint32_t)reg[c]) |
                       ((uint64_t)__ockl_wfred_or_u32((uint32_t)(reg[c] >> 32)) << 32);
    E.reg[c] = block_reduce<uint64_t>(m, redu, [](uint64_t u, uint64_t w) { return u | w; });
  }
  // topologyNormalizingWeight per score constraint (scoring.go initPreScoreState)
  const int nf = h->n_tsc_filter;
  for (int c = 0; c < ns; ++c) {
    const ksg_tsc& t = h->tsc[nf + c];
    int64_t size = 0;  // topoSize: hostname: filtered - ignored nodes; else the key's registered values
    if (t.is_hostname) size = (int64_t)E.feasible - E.ignored;
    else if (t.first_of_key)  // a key with one node per value registers one value per counted node
      size = ((C_uniq >> t.topo) & 1u) ? (int64_t)E.feasible - E.ignored : (int64_t)__popcll(E.reg[c]);
    E.w[c] = go_log((double)(size + 2));
  }
}

// PodTopologySpread raw score of a counted node (scoring.go Score): the constraints'
// cnt * weight + (maxSkew - 1), in constraint order, rounded half away from zero.
__device__ __forceinline__ int64_t pts_raw(const DevCluster& C, const ProgView& V, const EvalTotals& E, uint32_t n,
                                           const SlotVids& tv) {
#pragma clang fp contract(off)
  const ksg_prog* h = V.h;
  const int nf = h->n_tsc_filter, ns = h->n_tsc_score;
  double score = 0;
  for (int c = nf; c < nf + ns; ++c) {
    const ksg_tsc& t = h->tsc[c];
    const int32_t v = tv(t.topo);
    if (v < 0) continue;
    const int64_t cnt = pts_count_tab(C, V, c, n, v);
    score = __dadd_rn(score, __dadd_rn(__dmul_rn((double)cnt, E.w[c - nf]), (double)(t.max_skew - 1)));
  }
  return (int64_t)round(score);
}
__device__ __forceinline__ int64_t pts_raw1(const ksg_prog* h, const EvalTotals& E, int64_t cnt) {
#pragma clang fp contract(off)
  const ksg_tsc& t = h->tsc[h->n_tsc_filter];
  return (int64_t)round(__dadd_rn(0.0, __dadd_rn(__dmul_rn((double)cnt, E.w[0]), (double)(t.max_skew - 1))));
}

struct FinalShared {
  int32_t tv[KSG_MAX_TOPO * kBlock];
  EvalTotals E;
  int64_t red64[kBlock / 64];
  uint64_t redu[kBlock / 64];
  int32_t red32[kBlock / 64];
};

// PodTopologySpread raw scores of a pod with several score constraints.
__global__ __launch_bounds__(kBlock) void k_ptsraw(DevCluster C, DevProfile F, ChainArgs A) {
  const uint32_t q = *A.cur;
  if (q >= A.end) return;
  const ProgView V = view(A.progs + A.prog_off[q]);
  __shared__ FinalShared L;
  uint32_t* of;
  int32_t *os, *ot;
  chain_outs(A, q, C.N, of, os, ot);
  int pts_pos = -1;
  for (int p = 0; p < F.n; ++p)
    if (F.plugins[p] == KP_PTS) pts_pos = p;
  const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
  const bool active = n < C.N;
  load_slot_vids(C, n, active, L.tv);
  const SlotVids tv{L.tv + threadIdx.x};
  EvalTotals E;
  reduce_eval(A, V.h, C.T.uniq, E, L.red64, L.redu, L.red32);
  int64_t s = 0;
  bool counted = false;
  if (active && of[n] == KSG_FILTER_PASS) {
    int32_t* slot = os + (size_t)pts_pos * C.N + n;
    if (*slot >= 0) {
      counted = true;
      s = pts_raw(C, V, E, n, tv);
      *slot = (int32_t)s;
    }
  }
  const int64_t a = block_reduce<int64_t>(wave_max(counted ? s : INT64_MIN), L.red64,
                                          [](int64_t u, int64_t w) { return u > w ? u : w; });
  const int64_t c = block_reduce<int64_t>(wave_min(counted ? s : INT64_MAX), L.red64,
                                          [](int64_t u, int64_t w) { return u < w ? u : w; });
  if (threadIdx.x == 0) {
    A.pm2[blockIdx.x] = a;
    A.pm2[A.nblk + blockIdx.x] = c;
  }
}

__global__ __launch_bounds__(kBlock) void k_final(DevCluster C, DevProfile F, ChainArgs A) {
  const uint32_t q = *A.cur;
  if (q >= A.end) return;
  const ProgView V = view(A.progs + A.prog_off[q]);
  const ksg_prog* h = V.h;
  __shared__ FinalShared L;
  uint32_t* of;
  int32_t *os, *ot;
  chain_outs(A, q, C.N, of, os, ot);
  EvalTotals E;
  reduce_eval(A, h, C.T.uniq, E, L.red64, L.redu, L.red32);
  const bool multi = (h->tab & KTAB_PTS_MULTI) != 0;
  int64_t pmx = INT64_MIN, pmn = INT64_MAX;  // PodTopologySpread raw max / min over counted nodes
  if (multi) {
    for (uint32_t b = threadIdx.x; b < A.nblk; b += blockDim.x) {
      pmx = A.pm2[b] > pmx ? A.pm2[b] : pmx;
      pmn = A.pm2[A.nblk + b] < pmn ? A.pm2[A.nblk + b] : pmn;
    }
    pmx = block_reduce<int64_t>(wave_max(pmx), L.red64, [](int64_t u, int64_t w) { return u > w ? u : w; });
    pmn = block_reduce<int64_t>(wave_min(pmn), L.red64, [](int64_t u, int64_t w) { return u < w ? u : w; });
  } else if (E.mx[KCX_PTS] != INT64_MIN) {  // one constraint: raw is monotone in the count
    pmx = pts_raw1(h, E, E.mx[KCX_PTS]);
    pmn = pts_raw1(h, E, E.mn[KCX_PTS]);
  }
  // the summary's normalisers per position (max over feasible nodes; unset as k_init_summaries)
  int64_t smx[KSG_MAX_PLUGINS], smn[KSG_MAX_PLUGINS];
  for (int pos = 0; pos < F.n; ++pos) {
    const int p = F.plugins[pos], x = chain_x(p);
    smx[pos] = p == KP_IPA ? INT64_MIN : 0;
    smn[pos] = INT64_MAX;
    if (x < 0) continue;
    if (p == KP_PTS) {
      if (pmx != INT64_MIN) { smx[pos] = pmx > 0 ? pmx : 0; smn[pos] = pmn; }
    } else if (E.mx[x] != INT64_MIN) {
      smx[pos] = p == KP_IPA ? E.mx[x] : (E.mx[x] > 0 ? E.mx[x] : 0);
      smn[pos] = E.mn[x];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ksg_pod_summary* S = A.sums + q;
    S->feasible = E.feasible;
    S->ignored = E.ignored;
    S->ipa_flags = 0;
    for (int pos = 0; pos < F.n; ++pos) {
      S->max_score[pos] = smx[pos];
      S->min_score[pos] = smn[pos];
    }
    for (int c = 0; c < h->n_tsc_score; ++c) S->pts_weight[c] = E.w[c];
  }
  const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
  uint64_t key = 0;
  bool range_err = false;
  uint32_t ipa_flags = 0;
  {  // InterPodAffinity PreScore Skip: from the tables, as k_eval's blocks did
    __shared__ uint32_t fl;
    if (threadIdx.x == 0) fl = 0;
    __syncthreads();
    bool ipa = false;
    for (int p = 0; p < F.n; ++p) ipa |= F.plugins[p] == KP_IPA;
    if (ipa) {
      const uint32_t bits = __ockl_wfred_or_u32(ipa_table_bits(C, F, V));
      if (lane0() && bits) atomicOr(&fl, bits);
    }
    __syncthreads();
    ipa_flags = fl;
    if (blockIdx.x == 0 && threadIdx.x == 0) A.sums[q].ipa_flags = ipa_flags;
  }
  if (n < C.N && of[n] == KSG_FILTER_PASS) {
    int64_t tot = 0;
    bool pts_keys = false;
#pragma unroll 1
    for (int pos = 0; pos < F.n; ++pos) {
      const int p = F.plugins[pos];
      int64_t raw = os[(size_t)pos * C.N + n];
      if (p == KP_PTS) {
        pts_keys = raw >= 0 && h->n_tsc_score > 0;
        if (raw < 0) raw = 0;
        else if (!multi && h->n_tsc_score > 0 && !(h->flags & KPF_SKIP_PTS_SCORE)) raw = pts_raw1(h, E, raw);
        os[(size_t)pos * C.N + n] = (int32_t)raw;
      }
      bool use;
      const int64_t s = normalize_pos(p, h, raw, smx[pos], smn[pos], ipa_flags, pts_keys, use);
      if (use) {
        if (s < 0 || s > 100) range_err = true;
        tot += s * F.weight[pos];
      }
    }
    if (E.feasible == 1) tot = 0;  // single feasible node: no scoring
    ot[n] = (int32_t)tot;
    key = pack_key(tot, F.seed, h->queue_idx, C.goff + n);
  }
  const uint64_t best = block_reduce<uint64_t>(wave_max(key), L.redu, [](uint64_t u, uint64_t w) { return u > w ? u : w; });
  const int32_t st = block_reduce<int32_t>((E.feasible > 1 && range_err) ? 4 : 0, L.red32,
                                           [](int32_t x, int32_t y) { return x | y; });
  if (threadIdx.x == 0) {
    A.pk[blockIdx.x] = best;
    A.pst[blockIdx.x] = st;
  }
}

// selectHost + the assume: one block.
__global__ __launch_bounds__(kBlock) void k_select(DevCluster C, DevProfile F, ChainArgs A) {
  const uint32_t q = *A.cur;
  if (q >= A.end) return;
  const ProgView V = view(A.progs + A.prog_off[q]);
  const ksg_prog* h = V.h;
  __shared__ uint64_t redu[kBlock / 64];
  __shared__ int32_t red32[kBlock / 64];
  __shared__ int32_t s_node;
  uint64_t best = 0;
  int32_t f = 0, st = 0;
  for (uint32_t b = threadIdx.x; b < A.nblk; b += blockDim.x) {
    best = A.pk[b] > best ? A.pk[b] : best;
    f += A.pi[KCP_FEAS * A.nblk + b];
    st |= A.pi[KCP_STAT * A.nblk + b] | A.pst[b];
  }
  best = block_reduce<uint64_t>(wave_max(best), redu, [](uint64_t u, uint64_t w) { return u > w ? u : w; });
  f = block_reduce<int32_t>(wave_sum(f), red32, [](int32_t x, int32_t y) { return x + y; });
  st = block_reduce<int32_t>((int32_t)__ockl_wfred_or_u32((uint32_t)st), red32, [](int32_t x, int32_t y) { return x | y; });
  if (threadIdx.x == 0) {
    ksg_pod_summary* S = A.sums + q;
    S->feasible = f;
    S->best_key = best;
    int32_t node = -1;
    const bool error = (st & 2) || ((st & 4) && f > 1) || (h->flags & KPF_PREFILTER_ERROR);
    if (error) { S->status = 2; S->selected = -1; }
    else if (f == 0) { S->status = 1; S->selected = -1; }
    else {
      const uint32_t g = (uint32_t)(best & 0xFFFFFull);
      S->selected = (int32_t)g;
      S->status = 0;
      if ((A.mode & 1) && g >= C.goff && g - C.goff < C.N) node = (int32_t)(g - C.goff);
    }
    s_node = node;
    A.prow[q] = -1;
  }
  __syncthreads();
  const int32_t node = s_node;
  if (node >= 0) {
    if (threadIdx.x == 0) assume_pod(C, V, (uint32_t)node, +1, (A.mode & 2) != 0, A.prow + q, blockDim.x);
    tables_assume(C, V, (uint32_t)node, +1, threadIdx.x, blockDim.x);
  }
  __syncthreads();
  if (threadIdx.x == 0) *A.cur = q + 1;
}

__global__ void k_set_cur(uint32_t* cur, uint32_t q) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *cur = q;
}

// ---- class tables: build from the existing-pod table
// pod classes [c0, c0 + nc): every live existing pod matching a class adds to its tables
__global__ void k_pc_build(DevCluster C, uint32_t c0, uint32_t nc) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= C.tcounts[0]) return;
  const uint32_t fl = C.ptflags[p];
  if (fl & KEF_DELETED) return;
  const int32_t node = C.ptnode[p], ns = C.ptns[p];
  auto vid = [&](int32_t k) -> int32_t { return (k >= 0 && (uint32_t)k < C.pkeys) ? C.ptlab[(size_t)k * C.pcap + p] : -1; };
  for (uint32_t c = c0; c < c0 + nc; ++c) {
    const ksg_pclass& pc = C.T.pcls[c];
    if (pc.excl_term && (fl & KEF_TERMINATING)) continue;
    bool ok = pc.n_terms > 0;
    for (int i = 0; i < pc.n_terms && ok; ++i) {
      const ksg_cterm& t = C.T.cterm[pc.term_off + i];
      ok = (t.ns_all || in_list(ns, C.T.cval + t.ns_off, t.ns_cnt)) && sel_eval(t.sel, C.T.creq, C.T.cval, vid);
    }
    if (ok) pc_add(C, (int32_t)c, (uint32_t)node, +1);
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
  tc_add(C, e.cls, (uint32_t)C.ptnode[p], eterm_inc(e), +1);
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
