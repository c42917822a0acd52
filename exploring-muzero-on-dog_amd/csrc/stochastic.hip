// Stochastic MuZero for classic MADN: the networks of MuZero_Classic_MADN/muzero_classic_madn.py and
// mctx.stochastic_muzero_policy (as called by run_stochastic_muzero_mcts, 464-517) as ONE persistent
// kernel per search.
//
// The tree interleaves decision nodes (state embeddings, children = the A = 4 pins) and chance nodes
// (afterstates, children = the C = 6 die outcomes); internally a node has A' = A + C child slots, as in
// mctx.  A workgroup owns 16 games for the whole search.  Per simulation:
//   select  -- decision nodes: PUCT with qtransform_by_parent_and_siblings (+1e-7 tie-break noise, root
//              mask at depth 0); chance nodes: argmax softmax(chance_logits) / (n + 1);
//   expand  -- a decision parent runs action_dynamics (+ Pred4 on the afterstate for its value), a chance
//              parent chance_dynamics (+ Pred4 for action logits and value).  Only the network a row needs
//              is meaningful; a tile runs each network at most once (skipped when no row needs it);
//   backup  -- as in mctx search.backward.
// mctx evaluates both recurrent functions for every expansion and keeps one per lane; the other output is
// never read, so evaluating only the needed one gives identical trees.
#include "launch.hpp"
#include "rng.hpp"
#include "sdyn.hpp"

namespace muz {

constexpr int kSMaxSims = 100;
constexpr int kSMaxNodes = kSMaxSims + 1;
constexpr int kSMaxDepth = 64;
constexpr int kSA = 16;                 // child slots per node (A' = 10 used)
constexpr int kCls = 4, kChance = MUZ_CHANCE_OUTCOMES, kAp = kCls + kChance;
constexpr float kSFMin = -3.4028234663852886e38f;

#ifdef MUZ_BRANCH_STATS
__device__ unsigned long long g_branch_hist[(kRows + 1) * (kRows + 1)];
#endif

struct STree {
  int32_t* c_index;
  float* c_prior;
  float* c_value;
  int32_t* c_visits;
  float* c_reward;
  float* c_disc;
  float* emb;    // [n][N][256]  decision: state embedding, chance: afterstate
  float* info;   // [n][N][2]    chance nodes: (reward, discount) of the decision step (afterstate_with_info)
  int N;
  __device__ __forceinline__ size_t ca(int g, int node, int a) const { return ((size_t)g * N + node) * kSA + a; }
  __device__ __forceinline__ AS1 float* e(int g, int node) const { return gpw(emb) + ((size_t)g * N + node) * LAT; }
  __device__ __forceinline__ AS1 float* inf(int g, int node) const { return gpw(info) + ((size_t)g * N + node) * 2; }
  __device__ __forceinline__ AS1 int32_t* index() const { return gpw(c_index); }
  __device__ __forceinline__ AS1 float* prior() const { return gpw(c_prior); }
  __device__ __forceinline__ AS1 float* value() const { return gpw(c_value); }
  __device__ __forceinline__ AS1 int32_t* visits() const { return gpw(c_visits); }
  __device__ __forceinline__ AS1 float* reward() const { return gpw(c_reward); }
  __device__ __forceinline__ AS1 float* disc() const { return gpw(c_disc); }
};

static inline size_t stree_child_bytes(int64_t n, int N) { return (size_t)n * N * kSA * 4; }

static STree carve_stree(void* ws, int n, int N) {
  char* p = (char*)ws;
  const size_t cb = stree_child_bytes(n, N);
  STree t;
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
  t.info = (float*)p;
  t.N = N;
  return t;
}

struct SKid {
  float prior, value, reward, disc;
  int visits, index;
};

__device__ __forceinline__ void srow_argmax(float& v, int& i) {
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
  {
    const LoHi<float> pv = swap16(v);
    const LoHi<int> pi = swap16(i);
    v = pv.lo;
    i = pi.lo;
    pick(v, i, pv.hi, pi.hi);
  }
  if constexpr (kRowLanes == 64) {
    const LoHi<float> pv = swap32(v);
    const LoHi<int> pi = swap32(i);
    v = pv.lo;
    i = pi.lo;
    pick(v, i, pv.hi, pi.hi);
  }
}

// ---- FiLM tables (muz_classic_net_prepare) -------------------------------------------------------
// tab[o][0:512] = film(relu(embed(one_hot(o)))) for o < nrow, row nrow = zero one-hot.
__device__ __forceinline__ void film_row(const muz_dense& embed, const muz_dense& film, int nrow, float* tab) {
  __shared__ float e[64];
  const int o = blockIdx.x, c = threadIdx.x;
  if (c < 64) e[c] = fmaxf((o < nrow ? embed.w[o * 64 + c] : 0.f) + embed.b[c], 0.f);
  __syncthreads();
  const int w = (c >> 4) / NT512, t = (c >> 4) % NT512;
  float acc = 0.f;
  for (int k = 0; k < 64; ++k) {
    const int kb = k >> 4, lane = ((k & 15) >> 2) * 16 + (c & 15), j = k & 3;
    acc = fmaf(e[k], film.w[((((size_t)w * 4 + kb) * 64 + lane) * NT512 + t) * 4 + j], acc);
  }
  tab[o * 512 + c] = acc + film.b[c];
}
__global__ __launch_bounds__(512) void k_sfilm(muz_sdyn_w D, int A) {
  if ((int)blockIdx.x <= A) film_row(D.act_embed, D.act_film, A, D.act_film_tab);
}
__global__ __launch_bounds__(512) void k_cfilm(muz_sdyn_w D) {
  film_row(D.chance_embed, D.chance_film, kChance, D.chance_film_tab);
}

// ---- batched recurrent functions (for parity tests and external callers) --------------------------
__global__ __launch_bounds__(kThreads) void k_classic_decision(muz_classic_net_w Wt, const int32_t* __restrict__ action,
                                                          const float* __restrict__ emb, int n, float* after,
                                                          float* reward, float* discount, float* chance_logits,
                                                          float* avalue) {
  __shared__ __attribute__((aligned(16))) float smem[kArenaFloats];
  const Arena a = Arena::carve(smem);
  const AS4 muz_classic_net_w* W = kernarg0<muz_classic_net_w>();
  const int A = Wt.num_actions;
  const int row = trow(), sub = tsub();
  const int gr = blockIdx.x * kRows + row;
  const bool valid = gr < n;
  const int ar = valid ? action[gr] : 0;
  const FilmIn fin = film_load(W->sdyn.act_film_tab, A, W->sdyn.act_input_ln, valid ? gp(emb) + (size_t)gr * LAT : nullptr, ar);
  Pf pf;
  pf_issue<NT256>(pf, &W->sdyn.act_dense1, LAT, LAT);
  sdyn_action16<NT256>(W->sdyn, A, fin, ar, a, pf, &W->pred.rb[0].d0, LAT, LAT);
  if (valid) {
    for (int c = sub; c < LAT; c += kRowLanes) after[(size_t)gr * LAT + c] = a.T[row * LD + c];
    if (sub < kChance) chance_logits[(size_t)gr * kChance + sub] = a.E[row * LDE + sub];
    if (sub == 0) {
      reward[gr] = a.v1[row];
      discount[gr] = a.v2[row];
    }
  }
  // no barrier: pred16 reads a.T first and overwrites it only after its first SYNC; a.E is not touched
  pred16<1>(W->pred, A, a.T, a, pf, nullptr, 0, 0);
  if (valid && sub == 0) avalue[gr] = a.v0[row];
}

__global__ __launch_bounds__(kThreads) void k_classic_chance(muz_classic_net_w Wt, const int32_t* __restrict__ chance,
                                                        const float* __restrict__ after, int n, float* next_emb,
                                                        float* logits, float* value) {
  __shared__ __attribute__((aligned(16))) float smem[kArenaFloats];
  const Arena a = Arena::carve(smem);
  const AS4 muz_classic_net_w* W = kernarg0<muz_classic_net_w>();
  const int A = Wt.num_actions;
  const int row = trow(), sub = tsub();
  const int gr = blockIdx.x * kRows + row;
  const bool valid = gr < n;
  const int c = valid ? chance[gr] : 0;
  const FilmIn fin = film_load(W->sdyn.chance_film_tab, kChance, W->sdyn.chance_input_ln,
                               valid ? gp(after) + (size_t)gr * LAT : nullptr, c);
  Pf pf;
  pf_issue<NT256>(pf, &W->sdyn.chance_dense1, LAT, LAT);
  sdyn_chance16<NT256>(W->sdyn, fin, a, pf, &W->pred.rb[0].d0, LAT, LAT);
  if (valid)
    for (int k = sub; k < LAT; k += kRowLanes) next_emb[(size_t)gr * LAT + k] = a.T[row * LD + k];
  pred16<1>(W->pred, A, a.T, a, pf, nullptr, 0, 0);
  if (valid) {
    if (sub < A) logits[(size_t)gr * A + sub] = a.U[row * LD + sub];
    if (sub == 0) value[gr] = a.v0[row];
  }
}

// ---- the search -----------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads, 1) void k_stochastic_search(
    muz_classic_net_w Wt, SArgs sa, const float* __restrict__ root_logits, const float* __restrict__ root_value,
    const float* __restrict__ root_emb, const uint32_t* __restrict__ legal, const float* __restrict__ dirichlet_in,
    const float* __restrict__ gumbel_in, const int32_t* __restrict__ game_id, int n, const int* __restrict__ n_dev,
    STree T, int32_t* out_action, float* out_weights, float* out_value) {
  // tree arithmetic exactly as written (no fused multiply-add), like the NumPy restatement of mctx
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float smem[kArenaFloats];
  __shared__ int s_visits[kRows][kSMaxNodes];
  __shared__ float s_raw[kRows][kSMaxNodes];
  __shared__ float s_val[kRows][kSMaxNodes];
  __shared__ uint8_t s_dec[kRows][kSMaxNodes];
  __shared__ int p_node[kRows][kSMaxDepth];
  __shared__ int p_act[kRows][kSMaxDepth];
  __shared__ int p_cvis[kRows][kSMaxDepth];
  __shared__ float p_rew[kRows][kSMaxDepth];
  __shared__ float p_disc[kRows][kSMaxDepth];
  __shared__ int s_act[kRows], s_parent[kRows], s_next[kRows], s_depth[kRows], s_decp[kRows];
  __shared__ float s_newr[kRows], s_newd[kRows], s_rootv[kRows];
  __shared__ float s_cl[kRows][kChance];

  if (n_dev) n = *n_dev;
  if ((int)blockIdx.x * kRows >= n) return;
  const Arena ar = Arena::carve(smem);
  const int A = sa.A;
  const int row = trow(), a = tsub();
  const int g = blockIdx.x * kRows + row;
  const bool valid = g < n;
  const bool ok = a < kAp;                 // a real child slot
  const int ai = ok ? a : 0;
  const int lane = valid ? (game_id ? game_id[g] : g) : 0;
  const int gid = (valid && sa.key_game) ? sa.key_game[lane] : lane;
  const int gturn = (valid && sa.key_turn) ? sa.key_turn[gid] : sa.turn;

  // ---------------- root (policies.py stochastic_muzero_policy: noise, mask, pad with C chance slots)
  unsigned lb = 0;
  SKid rk;   // root children in registers (lane a holds child a)
  rk.prior = -INFINITY;
  rk.value = 0.f;
  rk.reward = 0.f;
  rk.disc = 0.f;
  rk.visits = 0;
  rk.index = -1;
  if (valid) {
    lb = legal[g];
    const bool act_lane = a < A;
    const float l = act_lane ? root_logits[(size_t)g * A + a] : -INFINITY;
    const float lm = row_max(l);
    const float el = act_lane ? expf(l - lm) : 0.f;
    const float pr = el / row_sum(el);
    float dn = 0.f;
    if (dirichlet_in) {
      dn = act_lane ? dirichlet_in[(size_t)g * A + a] : 0.f;
    } else {
      const float gm = act_lane ? gamma_sample(sa.dir_alpha, mix64(game_key(sa.seed ^ 0x5DEECE66Dull, gid, gturn) ^ (unsigned long long)(a + 1))) : 0.f;
      dn = gm / row_sum(gm);
    }
    const float noisy = (1.f - sa.dir_frac) * pr + sa.dir_frac * dn;
    float lg = act_lane ? logf(fmaxf(noisy, kTinyF)) : -INFINITY;
    lg = lg - row_max(lg);
    const bool inv = !act_lane || ((lb >> a) & 1u) == 0u;
    rk.prior = act_lane ? (inv ? kSFMin : lg) : -INFINITY;
    AS1 float* e0 = T.e(g, 0);
    for (int c = a; c < LAT; c += kRowLanes) e0[c] = root_emb[(size_t)g * LAT + c];
    if (a == 0) {
      const float v = root_value[g];
      s_visits[row][0] = 1;
      s_raw[row][0] = v;
      s_val[row][0] = v;
      s_dec[row][0] = 1;
    }
  }
  __syncthreads();

  auto load_kid = [&](int node) {
    SKid k;
    const size_t e = T.ca(g, node, ai);
    k.prior = ok ? T.prior()[e] : -INFINITY;
    k.value = T.value()[e];
    k.reward = T.reward()[e];
    k.disc = T.disc()[e];
    k.visits = ok ? T.visits()[e] : 0;
    k.index = T.index()[e];
    return k;
  };

  Pf pf;
  pf_issue<NT256>(pf, &kernarg0<muz_classic_net_w>()->sdyn.act_dense1, LAT, LAT);
#pragma unroll 1
  for (int sim = 0; sim < sa.S; ++sim) {
    const AS4 muz_classic_net_w* wl = kernarg0<muz_classic_net_w>();
    int dact = 0, decp = 1;
    float pr_r = 0.f, pr_d = 0.f;
    FilmIn fin;
    if (valid) {
      int node = 0, depth = 0, act = 0, nxt = -1;
      while (true) {
        const SKid k = depth == 0 ? rk : load_kid(node);
        const bool dec = s_dec[row][node] != 0;
        float sc;
        if (dec) {
          // muzero_action_selection with qtransform_by_parent_and_siblings
          const int N = s_visits[row][node];
          const float pb_c = sa.pb_c_init + logf(((float)N + sa.pb_c_base + 1.0f) / sa.pb_c_base);
          const float pm = row_max(ok ? k.prior : -INFINITY);
          const float e = ok ? expf(k.prior - pm) : 0.f;
          const float p = e / row_sum(e);
          const float q = k.reward + k.disc * k.value;
          const bool vis = k.visits > 0;
          const float nv = s_val[row][node];
          const float safe = vis ? q : nv;
          const float lo = fminf(nv, row_min(ok ? safe : INFINITY));
          const float hi = fmaxf(nv, row_max(ok ? safe : -INFINITY));
          const float vs = ((vis ? q : lo) - lo) / fmaxf(hi - lo, 1e-8f);
          const float ps = sqrtf((float)N) * pb_c * p / (float)(k.visits + 1);
          const float tb = tiebreak_uniform(sa.seed, gid, gturn, sim, depth, ai);
          sc = vs + ps + 1e-7f * tb;
          if (depth == 0 && (a >= A || ((lb >> a) & 1u) == 0u)) sc = -INFINITY;
          if (!ok) sc = -INFINITY;
        } else {
          // chance node: argmax softmax(chance logits) / (n + 1)
          const bool cl = ok && a >= A;
          const float cm = row_max(cl ? k.prior : -INFINITY);
          const float ce = cl ? expf(k.prior - cm) : 0.f;
          const float pc = ce / row_sum(ce);
          sc = cl ? pc / (float)(k.visits + 1) : -INFINITY;
        }
        int bi = a;
        srow_argmax(sc, bi);
        const int child = __shfl(k.index, bi, kRowLanes);
        if (a == bi) {
          p_node[row][depth] = node;
          p_act[row][depth] = bi;
          p_rew[row][depth] = k.reward;
          p_disc[row][depth] = k.disc;
          p_cvis[row][depth] = k.visits;
        }
        act = bi;
        nxt = child;
        ++depth;
        if (child == -1 || depth >= sa.D) break;
        node = child;
      }
      decp = s_dec[row][node];
      const AS1 float* pe = T.e(g, node);
      fin = film_load(wl->sdyn.act_film_tab, A, wl->sdyn.act_input_ln, pe, decp ? act : -1);
      if (!decp) {
        pr_r = T.inf(g, node)[0];
        pr_d = T.inf(g, node)[1];
      }
      dact = act;
      if (a == 0) {
        s_parent[row] = node;
        s_act[row] = act;
        s_next[row] = (nxt == -1) ? sim + 1 : nxt;
        s_depth[row] = depth;
        s_decp[row] = decp;
      }
    } else {
      fin = film_load(wl->sdyn.act_film_tab, A, wl->sdyn.act_input_ln, nullptr, -1);
      if (a == 0) {
        s_act[row] = 0;
        s_decp[row] = 2;   // no game: needs neither network
      }
    }
    ST(ST_SEL);
    SYNC();
    // which networks does this tile need? (uniform over the workgroup)
    int need_dec = 0, need_cha = 0;
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      need_dec |= s_decp[r] == 1;
      need_cha |= s_decp[r] == 0;
    }
#ifdef MUZ_BRANCH_STATS
    if (threadIdx.x == 0) {   // diagnostic: the tile's (decision-parent rows, chance-parent rows) of this expansion
      int nd = 0, nc = 0;
      for (int r = 0; r < kRows; ++r) {
        nd += s_decp[r] == 1;
        nc += s_decp[r] == 0;
      }
      atomicAdd(&g_branch_hist[nd * (kRows + 1) + nc], 1ull);
    }
#endif
    f32x4 keep[RowVec<LAT>::V];
    if (need_dec) {
      sdyn_action16<NT256>(wl->sdyn, A, fin, dact, ar, pf, need_cha ? &wl->sdyn.chance_dense1 : &wl->pred.rb[0].d0,
                           LAT, LAT);
#pragma unroll
      for (int i = 0; i < RowVec<LAT>::V; ++i) keep[i] = lds4(ar.T + row * LD + RowVec<LAT>::col(a, i));
      if (a == 0) {
        s_newr[row] = ar.v1[row];
        s_newd[row] = ar.v2[row];
      }
      if (a < kChance) s_cl[row][a] = ar.E[row * LDE + a];
      SYNC();
    } else if (need_cha) {
      pf_issue<NT256>(pf, &wl->sdyn.chance_dense1, LAT, LAT);
    }
    if (need_cha) {
      const FilmIn cin = film_load(wl->sdyn.chance_film_tab, kChance, wl->sdyn.chance_input_ln,
                                   valid ? T.e(g, s_parent[row]) : nullptr, (valid && !decp) ? dact - A : -1);
      sdyn_chance16<NT256>(wl->sdyn, cin, ar, pf, &wl->pred.rb[0].d0, LAT, LAT);
    }
    if (need_dec && decp == 1) {
#pragma unroll
      for (int i = 0; i < RowVec<LAT>::V; ++i) sts4(ar.T + row * LD + RowVec<LAT>::col(a, i), keep[i]);
    }
    SYNC();
    const int nx = s_next[row];
    if (valid) {
      AS1 float* ne = T.e(g, nx);
      for (int c = a; c < LAT; c += kRowLanes) ne[c] = ar.T[row * LD + c];
      if (decp && a == 0) {
        T.inf(g, nx)[0] = s_newr[row];
        T.inf(g, nx)[1] = s_newd[row];
      }
    }
    ST(ST_TREE);
    pred16<NT256>(wl->pred, A, ar.T, ar, pf, &wl->sdyn.act_dense1, LAT, LAT);
    if (valid) {
      const bool fresh = nx == sim + 1;
      // new node's prior: decision parent -> [-inf x A, chance logits]; chance parent -> [action logits, -inf x C]
      if (ok) {
        const float pv = decp ? (a < A ? -INFINITY : s_cl[row][a - A]) : (a < A ? ar.U[row * LD + a] : -INFINITY);
        const size_t nb = T.ca(g, nx, a);
        T.prior()[nb] = pv;
        if (fresh) {
          T.index()[nb] = -1;
          T.visits()[nb] = 0;
          T.value()[nb] = 0.f;
          T.reward()[nb] = 0.f;
          T.disc()[nb] = 0.f;
        }
      }
      const int par = s_parent[row], pa = s_act[row];
      const float er = decp ? 0.f : pr_r, ed = decp ? 1.f : pr_d;
      if (par == 0 && a == pa) {
        rk.index = nx;
        rk.reward = er;
        rk.disc = ed;
      }
      if (a == 0) {
        const float v = ar.v0[row];
        if (par != 0) {
          const size_t eb = T.ca(g, par, pa);
          T.index()[eb] = nx;
          T.reward()[eb] = er;
          T.disc()[eb] = ed;
        }
        s_raw[row][nx] = v;
        s_val[row][nx] = v;
        s_visits[row][nx] = fresh ? 1 : s_visits[row][nx] + 1;
        s_dec[row][nx] = decp ? 0 : 1;
        // backward (search.py) along the recorded path
        float leaf = v;
        int idx = nx;
        const int d = s_depth[row];
        for (int lvl = d - 1; lvl >= 0; --lvl) {
          const int parent = p_node[row][lvl];
          const int pact = p_act[row][lvl];
          const int cnt = s_visits[row][parent];
          const float r = (lvl == d - 1) ? er : p_rew[row][lvl];
          const float dsc = (lvl == d - 1) ? ed : p_disc[row][lvl];
          leaf = r + dsc * leaf;
          const float pv2 = (s_val[row][parent] * (float)cnt + leaf) / ((float)cnt + 1.0f);
          if (lvl > 0) {
            const size_t ei = T.ca(g, parent, pact);
            T.value()[ei] = s_val[row][idx];
            T.visits()[ei] = p_cvis[row][lvl] + 1;
          } else {
            s_rootv[row] = s_val[row][idx];
          }
          s_val[row][parent] = pv2;
          s_visits[row][parent] = cnt + 1;
          idx = parent;
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (a == p_act[row][0]) {
        rk.value = s_rootv[row];
        rk.visits += 1;
      }
    }
    ST(ST_TREE);
    SYNC();
  }

  // ---------------- _mask_tree(decision) + summary + _apply_temperature + categorical
  if (valid) {
    const bool act_lane = a < A;
    const int vc = act_lane ? rk.visits : 0;
    const int tot = row_isum(vc);
    const float w = tot > 0 ? (float)vc / (float)max(tot, 1) : 1.0f / (float)A;
    float lw = act_lane ? logf(w) : -INFINITY;
    lw = (lw - row_max(lw)) / fmaxf(kTinyF, sa.temperature);
    const float gmb = act_lane ? (gumbel_in ? gumbel_in[(size_t)g * A + a] : gumbel_noise(sa.seed ^ 0xC2B2AE3D27D4EB4Full, gid, gturn, a)) : 0.f;
    float sc = act_lane ? lw + gmb : -INFINITY;
    int bi = a;
    srow_argmax(sc, bi);
    if (act_lane) out_weights[(size_t)g * A + a] = w;
    if (a == 0) {
      out_action[g] = bi;
      out_value[g] = fminf(1.f, fmaxf(-1.f, s_val[row][0]));
    }
  }
}

int64_t stochastic_workspace_bytes(int n, int S) {
  const int N = S + 1;
  return (int64_t)(6 * stree_child_bytes(n, N) + (size_t)n * N * LAT * 4 + (size_t)n * N * 2 * 4);
}

SArgs make_sargs(const muz_stoch_cfg& cfg, int A) {
  SArgs sa;
  sa.S = cfg.num_simulations;
  sa.D = cfg.max_depth;
  sa.A = A;
  sa.dir_frac = cfg.dirichlet_fraction;
  sa.dir_alpha = cfg.dirichlet_alpha;
  sa.pb_c_init = cfg.pb_c_init;
  sa.pb_c_base = cfg.pb_c_base;
  sa.temperature = cfg.temperature;
  sa.seed = cfg.seed;
  sa.turn = cfg.turn;
  return sa;
}

int launch_stochastic_search(const muz_classic_net_w& w, const SArgs& sa, const float* root_logits,
                             const float* root_value, const float* root_emb, const uint32_t* legal,
                             const float* dirichlet, const float* gumbel, const int32_t* game_id, int n, const int* n_dev,
                             void* workspace, int32_t* action, float* weights, float* value, hipStream_t s) {
  const STree T = carve_stree(workspace, n, sa.S + 1);
  k_stochastic_search<<<(n + kRows - 1) / kRows, kThreads, 0, s>>>(w, sa, root_logits, root_value, root_emb, legal,
                                                                   dirichlet, gumbel, game_id, n, n_dev, T, action,
                                                                   weights, value);
  return muz_last_launch_error();
}

int check_classic_net(const muz_classic_net_w* w) {
  if (!w) return MUZ_E_INVALID;
  if (w->num_actions != kCls) return MUZ_E_UNSUPPORTED;
  if (w->obs_channels < 7 || w->obs_channels > 38) return MUZ_E_UNSUPPORTED;
  if (!w->sdyn.act_film_tab || !w->sdyn.chance_film_tab) return MUZ_E_INVALID;
  return MUZ_OK;
}

}  // namespace muz

using namespace muz;

extern "C" {

#ifdef MUZ_BRANCH_STATS
// diagnostic build: histogram [17][17] of (decision-parent rows, chance-parent rows) per tile expansion
int muz_diag_branch_hist(unsigned long long* host_out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(host_out, HIP_SYMBOL(muz::g_branch_hist), sizeof(unsigned long long) * 289);
  if (e != hipSuccess) return (int)e;
  if (reset) {
    unsigned long long z[289] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(muz::g_branch_hist), z, sizeof(z));
  }
  return (int)e;
}
#endif

int muz_classic_net_prepare(const muz_classic_net_w* w, void* stream) {
  if (!w || !w->sdyn.act_film_tab || !w->sdyn.chance_film_tab) return MUZ_E_INVALID;
  if (w->num_actions != kCls) return MUZ_E_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  k_sfilm<<<kCls + 1, 512, 0, s>>>(w->sdyn, kCls);
  int rc = muz_last_launch_error();
  if (rc) return rc;
  k_cfilm<<<kChance + 1, 512, 0, s>>>(w->sdyn);
  return muz_last_launch_error();
}

int muz_classic_nets_root(const muz_classic_net_w* w, const float* obs, int32_t n, void* scratch, int64_t scratch_bytes,
                          float* prior_logits, float* value, float* embedding, void* stream) {
  int rc = check_classic_net(w);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && obs && scratch && prior_logits && value && embedding);
  MUZ_HOST_CHECK(scratch_bytes >= muz_nets_root_scratch_bytes(n));
  if (n == 0) return MUZ_OK;
  return launch_root_inference(*w, obs, n, nullptr, (float*)scratch, prior_logits, value, embedding,
                               (hipStream_t)stream);
}

int muz_classic_nets_decision(const muz_classic_net_w* w, const int32_t* action, const float* embedding, int32_t n,
                              float* afterstate, float* reward, float* discount, float* chance_logits,
                              float* afterstate_value, void* stream) {
  int rc = check_classic_net(w);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && action && embedding && afterstate && reward && discount && chance_logits && afterstate_value);
  if (n == 0) return MUZ_OK;
  k_classic_decision<<<(n + kRows - 1) / kRows, kThreads, 0, (hipStream_t)stream>>>(
      *w, action, embedding, n, afterstate, reward, discount, chance_logits, afterstate_value);
  return muz_last_launch_error();
}

int muz_classic_nets_chance(const muz_classic_net_w* w, const int32_t* chance, const float* afterstate, int32_t n,
                            float* next_embedding, float* action_logits, float* value, void* stream) {
  int rc = check_classic_net(w);
  if (rc) return rc;
  MUZ_HOST_CHECK(n >= 0 && chance && afterstate && next_embedding && action_logits && value);
  if (n == 0) return MUZ_OK;
  k_classic_chance<<<(n + kRows - 1) / kRows, kThreads, 0, (hipStream_t)stream>>>(*w, chance, afterstate, n,
                                                                                 next_embedding, action_logits, value);
  return muz_last_launch_error();
}

int64_t muz_stochastic_workspace_bytes(int32_t n, int32_t num_simulations) {
  if (n < 0 || num_simulations < 1) return -1;
  return stochastic_workspace_bytes(n, num_simulations);
}

int muz_stochastic_search(const muz_classic_net_w* w, const muz_stoch_cfg* cfg, const float* root_logits,
                          const float* root_value, const float* root_embedding, const uint32_t* legal_bits,
                          const float* dirichlet, const float* gumbel, const int32_t* game_id, int32_t n,
                          void* workspace, int64_t workspace_bytes, int32_t* action, float* action_weights,
                          float* root_value_out, void* stream) {
  int rc = check_classic_net(w);
  if (rc) return rc;
  MUZ_HOST_CHECK(cfg && root_logits && root_value && root_embedding && legal_bits && workspace && action &&
                 action_weights && root_value_out && n >= 0);
  if (cfg->num_simulations < 1 || cfg->num_simulations > kSMaxSims) return MUZ_E_UNSUPPORTED;
  if (cfg->max_depth < 1 || cfg->max_depth > kSMaxDepth) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(workspace_bytes >= stochastic_workspace_bytes(n, cfg->num_simulations));
  if (n == 0) return MUZ_OK;
  return launch_stochastic_search(*w, make_sargs(*cfg, w->num_actions), root_logits, root_value, root_embedding,
                                  legal_bits, dirichlet, gumbel, game_id, n, nullptr, workspace, action, action_weights,
                                  root_value_out, (hipStream_t)stream);
}

}  // extern "C"
