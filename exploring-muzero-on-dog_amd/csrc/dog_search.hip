// run_muzero_mcts of the DOG slice (MuZero_DOG/muzero_dog.py:101-137: mctx.gumbel_muzero_policy with
// qtransform_completed_by_mix_value(value_scale=0.5), gumbel_scale = temperature) at A = 806, as ONE persistent
// kernel per search -- k_gumbel_search's structure (csrc/search.hip) with wide nodes:
//
//  * a workgroup owns 16 games; game `row` has 32 lanes and lane `sub` holds children sub, sub + 32, ..., sub + 800
//    (26 slots, 832 per node; slots >= 806 are padding);
//  * every node's children (the root's included) live in the workspace, [n][S+1][832] per field; the root's legal
//    words sit in LDS (word j bit `sub` is child sub + 32 j, the layout of muz_dog_legal's mask);
//  * sums over a node's children run in the lane order oracle/mctx_gumbel.py lane_tree_sum restates (each lane its
//    slots in turn, then a balanced tree over the 32 lanes), maxima / minima / integer sums are exact, exp is
//    correctly rounded and nothing contracts to fma -- so with identical network outputs the tree arithmetic
//    agrees with the restatement bit for bit;
//  * expand runs DynamicsNetwork4 + PredictionNetwork4 at A = 806 on the 16-row tile (nn.hpp, dog_nets.hpp), the
//    806 prior logits going from the logits chunks straight into the new node's children.
#include "dog_nets.hpp"
#include "launch.hpp"
#include "rng.hpp"

namespace muz {

constexpr int kWJ = 26;                      // child slots per lane
constexpr int kWPad = kRowLanes * kWJ;       // 832 children per node
constexpr int kWMaxSims = 100, kWMaxNodes = kWMaxSims + 1, kWMaxDepth = 64;
constexpr int kWWords = 26;                  // legal mask words (MUZ_DOG_MASK_WORDS)
constexpr float kWFMin = -3.4028234663852886e38f;
static_assert(kRowLanes == 32, "one game per 32 lanes");
static_assert(kWPad >= kDogA && kWWords * 32 >= kDogA, "slots");
static_assert(2 * kRows * kDogA <= kArenaFloats, "the walk's per-child arrays live in the idle network arena");

struct WTree {
  int32_t* c_index;
  float* c_prior;
  float* c_value;
  int32_t* c_visits;
  float* c_reward;
  float* c_disc;
  float* emb;
  float* gum;    // [n][832] the root's Gumbel noise, drawn once per search
  int N;
  __device__ __forceinline__ size_t ca(int g, int node, int a) const { return ((size_t)g * N + node) * kWPad + a; }
  __device__ __forceinline__ AS1 float* e(int g, int node) const { return gpw(emb) + ((size_t)g * N + node) * LAT; }
  __device__ __forceinline__ AS1 int32_t* index() const { return gpw(c_index); }
  __device__ __forceinline__ AS1 float* prior() const { return gpw(c_prior); }
  __device__ __forceinline__ AS1 float* value() const { return gpw(c_value); }
  __device__ __forceinline__ AS1 int32_t* visits() const { return gpw(c_visits); }
  __device__ __forceinline__ AS1 float* reward() const { return gpw(c_reward); }
  __device__ __forceinline__ AS1 float* disc() const { return gpw(c_disc); }
};

static size_t wide_children_bytes(int64_t n, int N) { return (size_t)n * N * kWPad * 4; }

static WTree carve_wide(void* ws, int n, int N) {
  char* p = (char*)ws;
  const size_t cb = wide_children_bytes(n, N);
  WTree t;
  t.c_index = (int32_t*)p;
  p += cb;
  t.c_prior = (float*)p;
  p += cb;
  t.c_value = (float*)p;
  p += cb;
  t.c_visits = (int32_t*)p;
  p += cb;
  t.c_reward = (float*)p;
  p += cb;
  t.c_disc = (float*)p;
  p += cb;
  t.emb = (float*)p;
  p += (size_t)n * N * LAT * 4;
  t.gum = (float*)p;
  t.N = N;
  return t;
}

// exp correctly rounded (float64, rounded once): oracle/mctx_gumbel.py exp_cr, search.hip exp_cr
__device__ __forceinline__ float exp_cr_w(float x) {
#ifdef MUZ_DOG_EXPT_FASTEXP   // timing experiment only (wrong rounding)
  return __expf(x);
#else
  return (float)exp((double)x);
#endif
}

// sum of this game's 806 entries f(j) (this lane's slot j; padding slots give -0) in the lane order of
// oracle/mctx_gumbel.py lane_tree_sum: each lane its slots in turn, then a balanced tree over the 32 lanes
template <class F>
__device__ __forceinline__ float wsum(F f) {
  float s = f(0);
#pragma unroll
  for (int j = 1; j < kWJ; ++j) {
    s = s + f(j);
    if ((j & 1) == 1) __builtin_amdgcn_sched_barrier(0);   // bounded interleaving of the slots (registers)
  }
  return row_sum(s);   // xor1, xor2, half mirror, mirror, swap16: the balanced tree in lane order
}

// argmax over the row's 806 children of score f(j) (this lane's slot j), jnp.argmax tie-break (first index):
// this lane's slots in ascending order (strict >), then row_argmax's (value, index) order across the lanes.
// Streams the scores: no per-slot array is kept.
template <class F>
__device__ __forceinline__ int wargmax(F f, int sub) {
  float v = -INFINITY;
  int i = sub;
#pragma unroll
  for (int j = 0; j < kWJ; ++j) {
    const float x = f(j);
    if (x > v) {
      v = x;
      i = sub + kRowLanes * j;
    }
    if ((j & 1) == 1) __builtin_amdgcn_sched_barrier(0);   // bounded interleaving of the slots (registers)
  }
  auto pick = [](float& v, int& i, float ov, int oi) {
    if (ov > v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  };
  pick(v, i, dpp<DPP_XOR1>(v), dpp<DPP_XOR1>(i));
  pick(v, i, dpp<DPP_XOR2>(v), dpp<DPP_XOR2>(i));
  pick(v, i, dpp<DPP_HALF_MIRROR>(v), dpp<DPP_HALF_MIRROR>(i));
  pick(v, i, dpp<DPP_MIRROR>(v), dpp<DPP_MIRROR>(i));
  const LoHi<float> pv = swap16(v);
  const LoHi<int> pi = swap16(i);
  v = pv.lo;
  i = pi.lo;
  pick(v, i, pv.hi, pi.hi);
  return i;
}

__device__ __forceinline__ bool wok(int sub, int j) { return sub + kRowLanes * j < kDogA; }

// seq_halving.get_sequence_of_considered_visits(m, S)[idx] (search.hip considered_visit)
__device__ __forceinline__ int wconsidered_visit(int m, int S, int idx) {
  if (m <= 1) return idx;
  int log2max = 0;
  while ((1 << log2max) < m) ++log2max;
  int k = m, v = 0, len = 0;
  while (len < S) {
    const int extra = max(1, S / (log2max * k));
    for (int e = 0; e < extra; ++e) {
      if (idx < len + k) return v;
      len += k;
      ++v;
    }
    k = max(2, k / 2);
  }
  return v;
}

// One node's children in this lane's slots + qtransform_completed_by_mix_value (value_scale, maxvisit_init,
// rescale, mixed value, eps 1e-8): pr = prior logits, cq = the transformed completed Q (both in LDS: the tile's
// network arena is idle during the walk -- dyn16 rewrites it from registers after the walk's barrier -- and 2 x 16 x
// 806 floats fit it), vis = visit counts (registers).  With pr / cq in registers beside the networks' ~225 VGPRs
// the kernel spilled; the exponentials are recomputed where they are needed for the same reason.
struct WNode {
  float* pr;     // [806] of this row, LDS
  float* cq;     // [806] of this row, LDS
  int vis[kWJ];
  float pm;      // max prior logit
  int sv, mv;    // sum / max of the visit counts
};

__device__ __forceinline__ void wnode_load(WNode& nd, const WTree& T, int g, int node, int sub, float raw,
                                           const SearchArgs& sa) {
#pragma clang fp contract(off)
  float pm = -INFINITY;
  int sv = 0, mv = 0;
#pragma unroll
  for (int j = 0; j < kWJ; ++j) {
    // (padding slots are read too -- they exist in the node's 832 -- and their values dropped: one base address per
    // field with immediate offsets)
    const int a = sub + kRowLanes * j;
    const bool ok = wok(sub, j);
    const size_t e = T.ca(g, node, a);
    const float pr = tree_ld(T.prior() + e);
    const int vs = tree_ld(T.visits() + e);
    const float rw = tree_ld(T.reward() + e), dc = tree_ld(T.disc() + e), vl = tree_ld(T.value() + e);
    nd.vis[j] = ok ? vs : 0;
    if (ok) {
      nd.pr[a] = pr;
      nd.cq[a] = rw + dc * vl;   // q (Tree.qvalues)
      pm = fmaxf(pm, pr);
    }
    sv += nd.vis[j];
    mv = max(mv, nd.vis[j]);
    // at most four slots' loads in flight: unfenced, the scheduler hoists all 130 loads of the node (130 VGPRs)
    if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  }
  pm = row_max(pm);
  sv = row_isum(sv);
  mv = row_imax(mv);
  const float es = wsum([&](int j) { return wok(sub, j) ? exp_cr_w(nd.pr[sub + kRowLanes * j] - pm) : -0.0f; });
  // prior probabilities of the visited children, floored at tiny (only those enter the mixed value)
  auto ppv = [&](int j) -> float {
    float x = 0.f;
    if (nd.vis[j] > 0) x = fmaxf(kTinyF, exp_cr_w(nd.pr[sub + kRowLanes * j] - pm) / es);
    return x;
  };
  const float sp = wsum([&](int j) { return wok(sub, j) ? ppv(j) : -0.0f; });
  const float wq = wsum([&](int j) {
    float x = wok(sub, j) ? 0.f : -0.0f;
    if (nd.vis[j] > 0) x = ppv(j) * nd.cq[sub + kRowLanes * j] / sp;
    return x;
  });
  const float mixed = (raw + (float)sv * wq) / (float)(sv + 1);
  float lo = INFINITY, hi = -INFINITY;
#pragma unroll
  for (int j = 0; j < kWJ; ++j) {
    const int a = sub + kRowLanes * j;
    if (wok(sub, j)) {
      const float c = nd.vis[j] > 0 ? nd.cq[a] : mixed;
      nd.cq[a] = c;
      lo = fminf(lo, c);
      hi = fmaxf(hi, c);
    }
  }
  lo = row_min(lo);
  hi = row_max(hi);
  const float den = fmaxf(hi - lo, 1e-8f);
  const float scale = (sa.maxvisit_init + (float)mv) * sa.value_scale;
#pragma unroll
  for (int j = 0; j < kWJ; ++j) {
    const int a = sub + kRowLanes * j;
    if (wok(sub, j)) nd.cq[a] = scale * ((nd.cq[a] - lo) / den);
  }
  nd.pm = pm;
  nd.sv = sv;
  nd.mv = mv;
}

__global__ __launch_bounds__(kThreads, 1) void k_dog_search(muz_dog_net_w Wt, SearchArgs sa,
                                                        const float* __restrict__ root_logits,
                                                        const float* __restrict__ root_value,
                                                        const float* __restrict__ root_emb,
                                                        const uint32_t* __restrict__ legal,
                                                        const float* __restrict__ gumbel_in, int n, WTree T,
                                                        int32_t* out_action, float* out_weights, float* out_value) {
#pragma clang fp contract(off)
  (void)Wt;
  __shared__ __attribute__((aligned(16))) float smem[kArenaFloats];
  __shared__ int s_visits[kRows][kWMaxNodes];
  __shared__ float s_raw[kRows][kWMaxNodes];
  __shared__ float s_val[kRows][kWMaxNodes];
  __shared__ int p_node[kRows][kWMaxDepth];
  __shared__ int p_act[kRows][kWMaxDepth];
  __shared__ int p_cvis[kRows][kWMaxDepth];
  __shared__ float p_rew[kRows][kWMaxDepth];
  __shared__ float p_disc[kRows][kWMaxDepth];
  __shared__ uint32_t s_legal[kRows][kWWords];
  __shared__ int s_act[kRows], s_parent[kRows], s_next[kRows], s_depth[kRows];

  if ((int)blockIdx.x * kRows >= n) return;
  const Arena ar = Arena::carve(smem);
  const int row = trow(), sub = tsub();
  const int g0 = blockIdx.x * kRows;
  const int g = g0 + row;
  const bool valid = g < n;
  int gid = g, gturn = sa.turn;
  int ncons = 0;

  // ---------------- root: instantiate_tree_from_root with masked logits (policies.py _mask_invalid_actions)
  if (valid) {
    gid = sa.key_game ? sa.key_game[g] : g;
    gturn = sa.key_turn ? sa.key_turn[gid] : sa.turn;
    int cnt = 0;
    if (sub < kWWords) {
      uint32_t w = legal[(size_t)g * kWWords + sub];
      if (sub == kWWords - 1) w &= (1u << (kDogA - 32 * (kWWords - 1))) - 1u;   // bits past action 805
      s_legal[row][sub] = w;
      cnt = __popc(w);
    }
    ncons = min(sa.max_considered, row_isum(cnt));
    float lm = -INFINITY;
#pragma unroll
    for (int j = 0; j < kWJ; ++j) {
      const int a = sub + kRowLanes * j;
      if (a < kDogA) lm = fmaxf(lm, root_logits[(size_t)g * kDogA + a]);
    }
    lm = row_max(lm);
#pragma unroll
    for (int j = 0; j < kWJ; ++j) {
      const int a = sub + kRowLanes * j;
      if (a < kDogA) {
        const uint32_t w = legal[(size_t)g * kWWords + j];
        const bool inv = ((w >> sub) & 1u) == 0u;
        const size_t e = T.ca(g, 0, a);
        tree_st(T.prior() + e, inv ? kWFMin : root_logits[(size_t)g * kDogA + a] - lm);
        tree_st(T.index() + e, -1);
        tree_st(T.visits() + e, 0);
        tree_st(T.value() + e, 0.f);
        tree_st(T.reward() + e, 0.f);
        tree_st(T.disc() + e, 0.f);
        gpw(T.gum)[(size_t)g * kWPad + a] =
            gumbel_in ? gumbel_in[(size_t)g * kDogA + a] : sa.gumbel_scale * gumbel_noise(sa.seed, gid, gturn, a);
      }
    }
    AS1 float* e0 = T.e(g, 0);
    for (int c = sub; c < LAT; c += kRowLanes) e0[c] = root_emb[(size_t)g * LAT + c];
    if (sub == 0) {
      const float v = root_value[g];
      s_visits[row][0] = 1;
      s_raw[row][0] = v;
      s_val[row][0] = v;
    }
  }
  __syncthreads();

  // (drawn once above: hashing the 806 draws inside the simulation loop made the compiler hoist their per-slot
  // constants out of it, 52 VGPRs live across the networks)
  auto gumbel_of = [&](int a) -> float { return tree_ld(gpw(T.gum) + (size_t)g * kWPad + a); };
  auto legal_of = [&](int j) -> bool { return (s_legal[row][j] >> sub) & 1u; };

  Pf pf;
  pf_issue<NT256>(pf, &kernarg0<muz_dog_net_w>()->dyn.d3, LAT, LAT);
#pragma unroll 1
  for (int sim = 0; sim < sa.S; ++sim) {
    const AS4 muz_dog_net_w* wl = kernarg0<muz_dog_net_w>();
    DynIn din;
    int dact = 0;
    // ---------------- simulate: walk from the root
    if (valid) {
      int node = 0, depth = 0, act = 0, nxt = -1;
      while (true) {
        WNode nd;
        nd.pr = smem + row * kDogA;
        nd.cq = smem + (kRows + row) * kDogA;
        int bi;
#ifdef MUZ_DOG_EXPT_NOSELECT   // timing experiment only (wrong results): a fixed child, no node load
        bi = (node * 131 + sim * 7 + depth) % kDogA;
        if (false) {
#else
        wnode_load(nd, T, g, node, sub, s_raw[row][node], sa);
        if (depth == 0) {
#endif
          // gumbel_muzero_root_action_selection: score_considered + masked_argmax
          const int cv = wconsidered_visit(ncons, sa.S, nd.sv);
          bi = wargmax([&](int j) {
            const int a = sub + kRowLanes * j;
            if (!wok(sub, j) || !legal_of(j)) return -INFINITY;
            return fmaxf(-1e9f, gumbel_of(a) + (nd.pr[a] - nd.pm) + nd.cq[a]) + (nd.vis[j] == cv ? 0.f : -INFINITY);
          }, sub);
        } else {
          // gumbel_muzero_interior_action_selection: softmax(prior + cq) - N / (1 + sum N)
          float zm = -INFINITY;
#pragma unroll
          for (int j = 0; j < kWJ; ++j)
            if (wok(sub, j)) zm = fmaxf(zm, nd.pr[sub + kRowLanes * j] + nd.cq[sub + kRowLanes * j]);
          zm = row_max(zm);
          auto z = [&](int j) { return (nd.pr[sub + kRowLanes * j] + nd.cq[sub + kRowLanes * j]) - zm; };
          const float zs = wsum([&](int j) { return wok(sub, j) ? exp_cr_w(z(j)) : -0.0f; });
          const float inv_n = (float)(1 + nd.sv);
          bi = wargmax([&](int j) {
            return wok(sub, j) ? (exp_cr_w(z(j)) / zs - (float)nd.vis[j] / inv_n) : -INFINITY;
          }, sub);
        }
        const size_t eb = T.ca(g, node, bi);
        const int child = tree_ld(T.index() + eb);
        if (sub == 0) {
          p_node[row][depth] = node;
          p_act[row][depth] = bi;
          p_rew[row][depth] = tree_ld(T.reward() + eb);
          p_disc[row][depth] = tree_ld(T.disc() + eb);
          p_cvis[row][depth] = tree_ld(T.visits() + eb);
        }
        act = bi;
        nxt = child;
        ++depth;
        if (child == -1 || depth >= sa.D) break;
        node = child;
      }
      din = dyn_load(wl->dyn, kDogA, T.e(g, node), act);
      dact = act;
      if (sub == 0) {
        s_parent[row] = node;
        s_act[row] = act;
        s_next[row] = (nxt == -1) ? sim + 1 : nxt;
        s_depth[row] = depth;
      }
    } else {
      din = dyn_load(wl->dyn, kDogA, nullptr, 0);
      if (sub == 0) s_act[row] = 0;
    }
    SYNC();
    // ---------------- expand: recurrent_fn on the 16 parents; the 806 prior logits go to the new nodes' children
    const int nx = s_next[row];
    dyn16<NT256, true, false>(wl->dyn, kDogA, din, dact, ar, pf, &wl->pred.rb[0].d0, LAT, LAT, &wl->pred.ln0,
                              valid ? T.e(g, nx) : nullptr);
    pred16<NT256, true, false, false, NT256, true>(wl->pred, kDogA, ar.T, ar, pf, nullptr, 0, 0);
    // (the hand-out re-reads the new node from LDS: with `nx` itself the compiler precomputed the 806 store
    // addresses before the networks and spilled them)
    dog_logits16<NT256>(wl, ar, pf, [&](int r, int col, float v) {
      if (valid) tree_st(T.prior() + T.ca(g0 + r, s_next[r], col), v);
    }, &wl->dyn.d3, LAT, LAT);
    if (valid) {
      const int nx = s_next[row];
      const bool fresh = nx == sim + 1;
      if (fresh) {
#pragma unroll
        for (int j = 0; j < kWJ; ++j) {
          const int a = sub + kRowLanes * j;
          if (a < kDogA) {
            const size_t e = T.ca(g, nx, a);
            tree_st(T.index() + e, -1);
            tree_st(T.visits() + e, 0);
            tree_st(T.value() + e, 0.f);
            tree_st(T.reward() + e, 0.f);
            tree_st(T.disc() + e, 0.f);
          }
        }
      }
      const int par = s_parent[row], pa = s_act[row];
      const float v = ar.v0[row], rw = ar.v1[row], dc = ar.v2[row];
      if (sub == 0) {
        const size_t eb = T.ca(g, par, pa);
        tree_st(T.index() + eb, nx);
        tree_st(T.reward() + eb, rw);
        tree_st(T.disc() + eb, dc);
        s_raw[row][nx] = v;
        s_val[row][nx] = v;
        s_visits[row][nx] = fresh ? 1 : s_visits[row][nx] + 1;
      }
      // ---------------- backward along the recorded path, one level per lane (search.hip's scheme; the root's
      // edges are tree entries here)
      const int d = s_depth[row];
      float carry = v, carry_v = v;
      for (int base = ((d - 1) / kRowLanes) * kRowLanes; base >= 0; base -= kRowLanes) {
        const int l = base + sub;
        const int top = min(d, base + kRowLanes) - 1 - base;
        const bool on = sub <= top;
        int parent = 0, pact = 0, cvis = 0, cnt = 0;
        float r = 0.f, dsc = 0.f, pval = 0.f;
        if (on) {
          parent = p_node[row][l];
          pact = p_act[row][l];
          cvis = p_cvis[row][l];
          r = (l == d - 1) ? rw : p_rew[row][l];
          dsc = (l == d - 1) ? dc : p_disc[row][l];
          cnt = s_visits[row][parent];
          pval = s_val[row][parent];
        }
        const unsigned long long tb = __ballot(sub == top);
        const int k0 = max(tb & 0xFFFFFFFFull ? 31 - __builtin_clz((unsigned)tb) : -1,
                           tb >> 32 ? 31 - __builtin_clz((unsigned)(tb >> 32)) : -1);
        float leaf = 0.f;
        for (int k = k0; k >= 0; --k) {
          const float up = dpp<DPP_WAVE_SHL1>(leaf);
          if (sub == k && on) leaf = r + dsc * (sub == top ? carry : up);
        }
        const float pv = (pval * (float)cnt + leaf) / ((float)cnt + 1.0f);
        const float pv_up = dpp<DPP_WAVE_SHL1>(pv);
        const float child_v = (sub == top) ? carry_v : pv_up;
        if (on) {
          const size_t ei = T.ca(g, parent, pact);
          tree_st(T.value() + ei, child_v);
          tree_st(T.visits() + ei, cvis + 1);
          s_val[row][parent] = pv;
          s_visits[row][parent] = cnt + 1;
        }
        carry = __shfl(leaf, 0, kRowLanes);
        carry_v = __shfl(pv, 0, kRowLanes);
      }
    }
    SYNC();
  }

  // ---------------- final action + action_weights (policies.py gumbel_muzero_policy tail)
  if (valid) {
    WNode nd;
    nd.pr = smem + row * kDogA;
    nd.cq = smem + (kRows + row) * kDogA;
    wnode_load(nd, T, g, 0, sub, s_raw[row][0], sa);
    const int bi = wargmax([&](int j) {
      const int a = sub + kRowLanes * j;
      if (!wok(sub, j) || !legal_of(j)) return -INFINITY;
      return fmaxf(-1e9f, gumbel_of(a) + (nd.pr[a] - nd.pm) + nd.cq[a]) +
             (nd.vis[j] == nd.mv ? 0.f : -INFINITY);   // considered_visit = max(visit_counts)
    }, sub);
    // action_weights = softmax(_mask_invalid_actions(prior + completed_q))
    float zm = -INFINITY;
#pragma unroll
    for (int j = 0; j < kWJ; ++j)
      if (wok(sub, j)) zm = fmaxf(zm, nd.pr[sub + kRowLanes * j] + nd.cq[sub + kRowLanes * j]);
    zm = row_max(zm);
    auto zz = [&](int j) {
      return !legal_of(j) ? kWFMin : (nd.pr[sub + kRowLanes * j] + nd.cq[sub + kRowLanes * j]) - zm;
    };
    float mm = -INFINITY;
#pragma unroll
    for (int j = 0; j < kWJ; ++j)
      if (wok(sub, j)) mm = fmaxf(mm, zz(j));
    mm = row_max(mm);
    const float zs = wsum([&](int j) { return wok(sub, j) ? exp_cr_w(zz(j) - mm) : -0.0f; });
#pragma unroll
    for (int j = 0; j < kWJ; ++j)
      if (wok(sub, j)) out_weights[(size_t)g * kDogA + sub + kRowLanes * j] = exp_cr_w(zz(j) - mm) / zs;
    if (sub == 0) {
      out_action[g] = ncons > 0 ? bi : -1;   // no legal action: -1, the self-play loop's no_step
      out_value[g] = s_val[row][0];
    }
  }
}

int64_t dog_search_workspace_bytes(int n, int S) {
  const int N = S + 1;
  return (int64_t)wide_children_bytes(n, N) * 6 + (int64_t)n * N * LAT * 4 + (int64_t)n * kWPad * 4;
}

int launch_dog_search(const muz_dog_net_w& w, const SearchArgs& sa, const float* root_logits, const float* root_value,
                      const float* root_emb, const uint32_t* legal, const float* gumbel, int n, void* workspace,
                      int32_t* action, float* weights, float* value, hipStream_t s) {
  WTree T = carve_wide(workspace, n, sa.S + 1);
  k_dog_search<<<(n + kRows - 1) / kRows, kThreads, 0, s>>>(w, sa, root_logits, root_value, root_emb, legal, gumbel, n,
                                                            T, action, weights, value);
  return muz_last_launch_error();
}

int check_dog_net(const muz_dog_net_w* w);

}  // namespace muz

using namespace muz;

extern "C" {

int64_t muz_dog_search_workspace_bytes(int32_t n, const muz_search_cfg* cfg) {
  if (!cfg || n < 0) return -1;
  return dog_search_workspace_bytes(n, cfg->num_simulations);
}

int muz_dog_gumbel_search(const muz_dog_net_w* w, const muz_search_cfg* cfg, const float* root_logits,
                          const float* root_value, const float* root_embedding, const uint32_t* legal,
                          const float* gumbel, int32_t n, void* workspace, int64_t workspace_bytes, int32_t* action,
                          float* action_weights, float* root_value_out, void* stream) {
  int rc = check_dog_net(w);
  if (rc) return rc;
  if (!cfg) return MUZ_E_INVALID;
  if (cfg->num_simulations < 1 || cfg->num_simulations > kWMaxSims) return MUZ_E_UNSUPPORTED;
  if (cfg->max_depth < 1 || cfg->max_depth > kWMaxDepth) return MUZ_E_UNSUPPORTED;
  if (cfg->max_num_considered < 1) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(n >= 0 && root_logits && root_value && root_embedding && legal && workspace && action &&
                 action_weights && root_value_out);
  MUZ_HOST_CHECK(workspace_bytes >= dog_search_workspace_bytes(n, cfg->num_simulations));
  if (n == 0) return MUZ_OK;
  SearchArgs sa;
  sa.S = cfg->num_simulations;
  sa.D = cfg->max_depth;
  sa.max_considered = cfg->max_num_considered;
  sa.value_scale = cfg->value_scale;
  sa.maxvisit_init = cfg->maxvisit_init;
  sa.gumbel_scale = cfg->gumbel_scale;
  sa.seed = cfg->seed;
  sa.turn = cfg->turn;
  return launch_dog_search(*w, sa, root_logits, root_value, root_embedding, legal, gumbel, n, workspace, action,
                           action_weights, root_value_out, (hipStream_t)stream);
}

}  // extern "C"
