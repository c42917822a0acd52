// Batched Gumbel MuZero search (mctx 0.0.6 gumbel_muzero_policy, as called by
// MuZero_det_MADN/muzero_deterministic_madn.py:663-704) as ONE persistent kernel per search.
//
// A workgroup owns 16 games for the whole search: for every simulation it walks the 16 trees
// (32 lanes per game, one action per lane, wavefront shuffles for every reduction), gathers the
// 16 parent embeddings into LDS, runs DynamicsNetwork4 + PredictionNetwork4 on MFMA over the
// 16-row tile, expands, and backs up.  No kernel boundary between simulations and no
// inter-workgroup traffic (games are independent).  Node scalars (visits, raw value, value) and
// the current path live in LDS; children arrays and node embeddings live in the workspace (HBM,
// L2/MALL resident), written lazily when a node is created.
#include "launch.hpp"
#include "nn.hpp"
#include "rng.hpp"

namespace muz {

// Diagnostic build only (make DIAG=1): per-phase shader-clock totals of the search kernel.
#ifdef MUZ_STAMPS
__device__ unsigned long long g_muz_stamps[8];
#define MUZ_STAMP(i)                                                          \
  do {                                                                        \
    if (threadIdx.x == 0) {                                                   \
      const unsigned long long _t = __builtin_amdgcn_s_memtime();             \
      st_acc[i] += _t - st_last;                                              \
      st_last = _t;                                                           \
    }                                                                         \
  } while (0)
#else
#define MUZ_STAMP(i) \
  do {               \
  } while (0)
#endif

// Two of the ~31 workgroup barriers per simulation are not needed for correctness (see the uses); removing
// them measured within noise on MI355X (B=4096 S=50: +-1 %), so they stay.  A static s_setprio 1 for
// waves 4-7 also measured within noise (profiles/r1e_prio_ab.log).

// Dyn4's reward / discount trunk inside Pred4's Dense_1 phase (nn.hpp pred16 LATE_HEADS)
#ifndef MUZ_LATE_HEADS
#define MUZ_LATE_HEADS 0
#endif
constexpr bool kLateHeads = MUZ_LATE_HEADS != 0;

constexpr int kMaxSims = 100;              // S <= 100 (config (e) uses 100)
constexpr int kMaxNodes = kMaxSims + 1;
constexpr int kMaxDepth = 64;
constexpr int kAPad = 32;                  // children arrays padded to 32 actions
constexpr float kFMin = -3.4028234663852886e38f;   // jnp.finfo(float32).min
// levels per backup chunk (one per lane); a smaller value only in the test build that exercises the chunked
// path of max_depth > 32 at ordinary depths (tests/test_gpu_search.py)
#ifndef MUZ_BACKUP_CHUNK
#define MUZ_BACKUP_CHUNK kRowLanes
#endif
constexpr int kBackupChunk = MUZ_BACKUP_CHUNK;
static_assert(kBackupChunk >= 1 && kBackupChunk <= kRowLanes, "backup chunk");

struct TreeWs {
  int32_t* c_index;
  float* c_prior;
  float* c_value;
  int32_t* c_visits;
  float* c_reward;
  float* c_disc;
  float* emb;
  int N;
  __device__ __forceinline__ size_t ca(int g, int node, int a) const { return ((size_t)g * N + node) * kAPad + a; }
  __device__ __forceinline__ AS1 float* e(int g, int node) const { return gpw(emb) + ((size_t)g * N + node) * LAT; }
  // global-address-space views (see common.hpp: keeps LDS waits independent of global loads)
  __device__ __forceinline__ AS1 int32_t* index() const { return gpw(c_index); }
  __device__ __forceinline__ AS1 float* prior() const { return gpw(c_prior); }
  __device__ __forceinline__ AS1 float* value() const { return gpw(c_value); }
  __device__ __forceinline__ AS1 int32_t* visits() const { return gpw(c_visits); }
  __device__ __forceinline__ AS1 float* reward() const { return gpw(c_reward); }
  __device__ __forceinline__ AS1 float* disc() const { return gpw(c_disc); }
};

static inline size_t ws_children_bytes(int64_t n, int N) { return (size_t)n * N * kAPad * 4; }

static TreeWs carve_ws(void* ws, int n, int N) {
  char* p = (char*)ws;
  const size_t cb = ws_children_bytes(n, N);
  TreeWs t;
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
  t.N = N;
  return t;
}

// ---- one game per 32 lanes (half a wave), one action per lane; jnp.argmax tie-break (first index) ----
__device__ __forceinline__ void row_argmax(float& v, int& i) {
  // (value, index) pairs under the order "larger value, then smaller index" (jnp.argmax tie-break)
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

// ---- the tree arithmetic, bit for bit like the NumPy restatement (oracle/mctx_gumbel.py) -------------------
// With identical network outputs on both sides the search's floats then agree exactly (tests/_parity.py):
//  * no fma contraction (q = r + d * v, the mixed value and the backup round twice, like numpy);
//  * a sum over the 24 actions in numpy's pairwise order for a contiguous row of 24: r_j = (a_j + a_{j+8}) +
//    a_{j+16} for j < 8, then ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
//  * exp correctly rounded: evaluated in float64 and rounded once (numpy's float32 exp and the device's expf
//    are each ~1 ulp off in different places; the oracle rounds the float64 exp the same way).
enum { DPP_ROW_ROR8 = 0x128 };
__device__ __forceinline__ float row_sum24(float v) {
  static_assert(kRowLanes == 32, "row_sum24: one game per 32 lanes");
  if (tsub() >= 24) v = -0.0f;                  // the additive identity for every x, -0 included
  v = v + dpp<DPP_ROW_ROR8>(v);                 // a_j + a_{j+8} (lanes 16..23: a_{16+j} + -0)
  const LoHi<float> p = swap16(v);
  v = p.lo + p.hi;                              // r_j = (a_j + a_{j+8}) + a_{j+16} in lanes j, j+8, j+16, j+24
  v = v + dpp<DPP_XOR1>(v);                     // r0 + r1 | r2 + r3 | ...
  v = v + dpp<DPP_XOR2>(v);                     // (r0 + r1) + (r2 + r3) | (r4 + r5) + (r6 + r7)
  return v + dpp<DPP_HALF_MIRROR>(v);           // lane i <-> 7 - i: the two halves
}
__device__ __forceinline__ float exp_cr(float x) { return (float)exp((double)x); }

// seq_halving.get_sequence_of_considered_visits(m, S)[idx] without the table.
__device__ __forceinline__ int considered_visit(int m, int S, int idx) {
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

// One child edge of the current node, held by lane `a` of the game's 32 lanes (ok = a < A).
struct Kid {
  float prior, value, reward, disc;
  int visits, index;
  bool ok;
};

// qtransform_completed_by_mix_value (value_scale, maxvisit_init, rescale, mixed value, eps 1e-8).
__device__ __forceinline__ float completed_q(const Kid& k, float raw, const SearchArgs& sa, int& sumv, float& pmax) {
#pragma clang fp contract(off)
  const float q = k.reward + k.disc * k.value;
  const float pm = row_max(k.ok ? k.prior : -INFINITY);
  const float e = k.ok ? exp_cr(k.prior - pm) : 0.f;
  const float es = row_sum24(e);
  const float pp = fmaxf(kTinyF, e / es);
  const bool vis = k.ok && k.visits > 0;
  const int sv = row_isum(k.ok ? k.visits : 0);
  const int mv = row_imax(k.ok ? k.visits : 0);
  const float sp = row_sum24(vis ? pp : 0.f);
  const float wq = row_sum24(vis ? pp * q / sp : 0.f);
  const float mixed = (raw + (float)sv * wq) / (float)(sv + 1);
  float cq = vis ? q : mixed;
  const float lo = row_min(k.ok ? cq : INFINITY);
  const float hi = row_max(k.ok ? cq : -INFINITY);
  const float den = fmaxf(hi - lo, 1e-8f);
  const float scale = (sa.maxvisit_init + (float)mv) * sa.value_scale;
  sumv = sv;
  pmax = pm;
  return scale * ((cq - lo) / den);
}

__global__ __launch_bounds__(kThreads, 1) void k_gumbel_search(
    muz_net_w Wt, SearchArgs sa, const float* __restrict__ root_logits, const float* __restrict__ root_value,
    const float* __restrict__ root_emb, const uint32_t* __restrict__ legal, const float* __restrict__ gumbel_in,
    const int32_t* __restrict__ game_id, int n, const int* __restrict__ n_dev, TreeWs T, int32_t* out_action,
    float* out_weights, float* out_value) {
  // tree arithmetic exactly as written (see row_sum24); the networks (nn.hpp) keep their own contraction
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float smem[kArenaFloats];
  __shared__ int s_visits[kRows][kMaxNodes];
  __shared__ float s_raw[kRows][kMaxNodes];
  __shared__ float s_val[kRows][kMaxNodes];
  __shared__ int p_node[kRows][kMaxDepth];
  __shared__ int p_act[kRows][kMaxDepth];
  __shared__ int p_cvis[kRows][kMaxDepth];
  __shared__ float p_rew[kRows][kMaxDepth];
  __shared__ float p_disc[kRows][kMaxDepth];
  __shared__ int s_act[kRows], s_parent[kRows], s_next[kRows], s_depth[kRows];
  __shared__ float s_rootv[kRows];

  if (n_dev) n = *n_dev;
  if ((int)blockIdx.x * kRows >= n) return;
  const Arena ar = Arena::carve(smem);
  const int A = Wt.num_actions;
  const int row = trow(), a = tsub();      // this lane holds action `a` of game `row`
  const int g = blockIdx.x * kRows + row;
  const bool valid = g < n;
  const bool ok = a < A;
  const int ai = ok ? a : 0;              // in-bounds alias for lanes a >= A
#ifdef MUZ_STAMPS
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif

  // ---------------- root: instantiate_tree_from_root with masked logits (policies.py _mask_invalid_actions)
  unsigned lb = 0;
  int ncons = 0;
  float gum = 0.f;
  // The root's children live in registers (lane a holds child a) for the whole search: the root is
  // visited by every simulation, so its edge data never goes through HBM.
  Kid rk;
  rk.ok = ok;
  rk.prior = kFMin;
  rk.value = 0.f;
  rk.reward = 0.f;
  rk.disc = 0.f;
  rk.visits = 0;
  rk.index = -1;
  if (valid) {
    lb = legal[g];
    const int lane = game_id ? game_id[g] : g;
    const int gid = sa.key_game ? sa.key_game[lane] : lane;
    const int gturn = sa.key_turn ? sa.key_turn[gid] : sa.turn;
    const float l = ok ? root_logits[(size_t)g * A + ai] : -INFINITY;
    const float lm = row_max(l);
    const bool inv = !ok || ((lb >> a) & 1u) == 0u;
    rk.prior = inv ? kFMin : l - lm;
    if (ok) gum = gumbel_in ? gumbel_in[(size_t)g * A + ai] : sa.gumbel_scale * gumbel_noise(sa.seed, gid, gturn, ai);
    AS1 float* e0 = T.e(g, 0);
    for (int c = a; c < LAT; c += kRowLanes) e0[c] = root_emb[(size_t)g * LAT + c];
    ncons = min(sa.max_considered, __popc(lb & ((1u << A) - 1u)));
    if (a == 0) {
      const float v = root_value[g];
      s_visits[row][0] = 1;
      s_raw[row][0] = v;
      s_val[row][0] = v;
    }
  }
  __syncthreads();

  // one node's children for this lane
  auto load_kid = [&](int node) {
    Kid k;
    const size_t e = T.ca(g, node, ai);
    k.ok = ok;
    k.prior = tree_ld(T.prior() + e);
    k.value = tree_ld(T.value() + e);
    k.reward = tree_ld(T.reward() + e);
    k.disc = tree_ld(T.disc() + e);
    k.visits = ok ? tree_ld(T.visits() + e) : 0;
    k.index = tree_ld(T.index() + e);
    return k;
  };

  st_begin();
  Pf pf;   // first k-blocks of the next dense layer (crosses the select / expand phases)
  pf_issue<NT256>(pf, &kernarg0<muz_net_w>()->dyn.d3, LAT, LAT);
#pragma unroll 1
  for (int sim = 0; sim < sa.S; ++sim) {
    MUZ_STAMP(0);
    st_sim(sim);
    // Weight table = kernel argument 0, read through the kernarg segment and laundered once per
    // simulation so the compiler re-derives the layer addresses inside the loop.
    const AS4 muz_net_w* wl = kernarg0<muz_net_w>();
    DynIn din;
    int dact = 0;
    // ---------------- simulate (search.py simulate): walk from the root
    if (valid) {
      int node = 0, depth = 0, act = 0, nxt = -1;
      while (true) {
        const Kid k = depth == 0 ? rk : load_kid(node);
        int sumv;
        float pmax;
        const float cq = completed_q(k, s_raw[row][node], sa, sumv, pmax);
        float sc;
        if (depth == 0) {
          // gumbel_muzero_root_action_selection: score_considered + masked_argmax
          const int cv = considered_visit(ncons, sa.S, sumv);
          const float s = fmaxf(-1e9f, gum + (k.prior - pmax) + cq) + (k.visits == cv ? 0.f : -INFINITY);
          sc = (!ok || ((lb >> a) & 1u) == 0u) ? -INFINITY : s;
        } else {
          // gumbel_muzero_interior_action_selection: softmax(prior + cq) - N / (1 + sum N)
          const float z = k.prior + cq;
          const float zm = row_max(ok ? z : -INFINITY);
          const float ez = ok ? exp_cr(z - zm) : 0.f;
          const float zs = row_sum24(ez);
          sc = ok ? (ez / zs - (float)k.visits / (float)(1 + sumv)) : -INFINITY;
        }
        int bi = a;
        row_argmax(sc, bi);
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
      // expand's inputs (parent embedding, FiLM rows of the action): issued by the game's own lanes now,
      // they land while the other games finish their walks
      din = dyn_load(wl->dyn, A, T.e(g, node), act);
      dact = act;
      if (a == 0) {
        s_parent[row] = node;
        s_act[row] = act;
        s_next[row] = (nxt == -1) ? sim + 1 : nxt;
        s_depth[row] = depth;
      }
    } else {
      din = dyn_load(wl->dyn, A, nullptr, 0);
      if (a == 0) s_act[row] = 0;
    }
    ST(ST_SEL);
    // (Dyn4's first pass -- LayerNorm_0 + FiLM of the parent latent -- only reads this row's own registers
    // and writes this row of the arena: this barrier is not needed for correctness, see above)
    SYNC();
    MUZ_STAMP(1);   // select
    // ---------------- expand (search.py expand): recurrent_fn on the 16 parents
    // the new node's embedding goes to the tree and Pred4's LayerNorm_0 into ar.X straight from Dyn4's
    // min-max pass (registers), so Pred4 starts with its first ResBlock
    const int nx = s_next[row];
    dyn16<NT256, true, kLateHeads>(wl->dyn, A, din, dact, ar, pf, &wl->pred.rb[0].d0, LAT, LAT, &wl->pred.ln0,
                                   valid ? T.e(g, nx) : nullptr);
    MUZ_STAMP(3);   // dynamics
    MUZ_STAMP(4);   // embedding write (fused)
    pred16<NT256, true, kLateHeads, kSplitkLogits>(wl->pred, A, ar.T, ar, pf, &wl->dyn.d3, LAT, LAT, &wl->dyn, dact);
    MUZ_STAMP(5);   // prediction
    if (valid) {
      const bool fresh = nx == sim + 1;
      if (ok) {
        const size_t nb = T.ca(g, nx, a);
        tree_st(T.prior() + nb, ar.U[row * LD + a]);
        if (fresh) {
          tree_st(T.index() + nb, -1);
          tree_st(T.visits() + nb, 0);
          tree_st(T.value() + nb, 0.f);
          tree_st(T.reward() + nb, 0.f);
          tree_st(T.disc() + nb, 0.f);
        }
      }
      const int par = s_parent[row], pa = s_act[row];
      if (par == 0 && a == pa) {   // a root edge: registers
        rk.index = nx;
        rk.reward = ar.v1[row];
        rk.disc = ar.v2[row];
      }
      const float v = ar.v0[row], rw = ar.v1[row], dc = ar.v2[row];
      if (a == 0) {
        if (par != 0) {
          const size_t eb = T.ca(g, par, pa);
          tree_st(T.index() + eb, nx);
          tree_st(T.reward() + eb, rw);
          tree_st(T.disc() + eb, dc);
        }
        s_raw[row][nx] = v;
        s_val[row][nx] = v;
        s_visits[row][nx] = fresh ? 1 : s_visits[row][nx] + 1;
      }
      // ---------------- backward (search.py backward) along the recorded path, one level per lane: lane a
      // holds level base + a (chunks of kRowLanes levels from the top when max_depth > kRowLanes).  Path nodes
      // are distinct, so every level's parent statistics are read at once; only the discounted leaf value is a
      // chain, evaluated level by level in the original order (leaf = r + discount * leaf, bit-identical to a
      // sequential walk) with the level above's value moved down one lane per step.
      const int d = s_depth[row];
      float carry = v;      // leaf value entering the chunk from the level above it
      float carry_v = v;    // new value of the node below the chunk's top level (its tree edge's value)
      for (int base = ((d - 1) / kBackupChunk) * kBackupChunk; base >= 0; base -= kBackupChunk) {
        const int l = base + a;
        const int top = min(d, base + kBackupChunk) - 1 - base;   // highest lane of this row's chunk
        const bool on = a <= top;
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
        // highest chunk lane over the wave's two rows (wave-uniform loop bound)
        const unsigned long long tb = __ballot(a == top);
        const int k0 = max(tb & 0xFFFFFFFFull ? 31 - __builtin_clz((unsigned)tb) : -1,
                           tb >> 32 ? 31 - __builtin_clz((unsigned)(tb >> 32)) : -1);
        float leaf = 0.f;
        for (int k = k0; k >= 0; --k) {
          const float up = dpp<DPP_WAVE_SHL1>(leaf);   // lane a + 1's value
          if (a == k && on) leaf = r + dsc * (a == top ? carry : up);
        }
        const float pv = (pval * (float)cnt + leaf) / ((float)cnt + 1.0f);
        const float pv_up = dpp<DPP_WAVE_SHL1>(pv);
        const float child_v = (a == top) ? carry_v : pv_up;
        if (on) {
          if (l > 0) {
            const size_t ei = T.ca(g, parent, pact);
            tree_st(T.value() + ei, child_v);
            tree_st(T.visits() + ei, cvis + 1);
          } else {
            s_rootv[row] = child_v;
          }
          s_val[row][parent] = pv;
          s_visits[row][parent] = cnt + 1;
        }
        carry = __shfl(leaf, 0, kRowLanes);
        carry_v = __shfl(pv, 0, kRowLanes);
      }
      // the root edge of this path (level 0): its lane takes the value lane 0 just backed up
      // (same wave: LDS operations of one wave complete in order)
      __builtin_amdgcn_wave_barrier();
      if (a == p_act[row][0]) {
        rk.value = s_rootv[row];
        rk.visits += 1;
      }
    }
    ST(ST_TREE);
    // (The next walk of row r reads only what row r's own lanes -- one wave -- wrote here: this barrier is
    // not needed for correctness either)
    SYNC();
    MUZ_STAMP(6);   // expand + backward
  }
#ifdef MUZ_STAMPS
  if (threadIdx.x == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&g_muz_stamps[i], st_acc[i]);
#endif
  st_end();

  // ---------------- final action + action_weights (policies.py gumbel_muzero_policy tail)
  if (valid) {
    const Kid& k = rk;
    int sumv;
    float pmax;
    const float cq = completed_q(k, s_raw[row][0], sa, sumv, pmax);
    const bool inv = !ok || ((lb >> a) & 1u) == 0u;
    const int cv = row_imax(k.visits);   // considered_visit = max(visit_counts)
    float sc = fmaxf(-1e9f, gum + (k.prior - pmax) + cq) + (k.visits == cv ? 0.f : -INFINITY);
    sc = inv ? -INFINITY : sc;
    int bi = a;
    row_argmax(sc, bi);
    // action_weights = softmax(_mask_invalid_actions(prior + completed_q))
    const float z = k.prior + cq;
    const float zm = row_max(ok ? z : -INFINITY);
    const float zz = inv ? kFMin : z - zm;
    const float mm = row_max(ok ? zz : -INFINITY);
    const float ez = ok ? exp_cr(zz - mm) : 0.f;
    const float zs = row_sum24(ez);
    if (ok) out_weights[(size_t)g * A + a] = ez / zs;
    if (a == 0) {
      out_action[g] = bi;
      out_value[g] = s_val[row][0];
    }
  }
}

int64_t search_workspace_bytes(int n, int S) {
  const int N = S + 1;
  return (int64_t)ws_children_bytes(n, N) * 6 + (int64_t)n * N * LAT * 4;
}

int launch_gumbel_search(const muz_net_w& w, const SearchArgs& sa, const float* root_logits, const float* root_value,
                         const float* root_emb, const uint32_t* legal, const float* gumbel, const int32_t* game_id,
                         int n, const int* n_dev, void* workspace, int32_t* action, float* weights, float* value,
                         hipStream_t s) {
  TreeWs T = carve_ws(workspace, n, sa.S + 1);
  k_gumbel_search<<<(n + kRows - 1) / kRows, kThreads, 0, s>>>(w, sa, root_logits, root_value, root_emb, legal,
                                                               gumbel, game_id, n, n_dev, T, action, weights, value);
  return muz_last_launch_error();
}

}  // namespace muz

using namespace muz;

extern "C" {

int64_t muz_search_workspace_bytes(int32_t n, const muz_search_cfg* cfg) {
  if (!cfg || n < 0) return -1;
  return search_workspace_bytes(n, cfg->num_simulations);
}

int muz_gumbel_search(const muz_net_w* w, const muz_search_cfg* cfg, const float* root_logits, const float* root_value,
                      const float* root_embedding, const uint32_t* legal_bits, const float* gumbel,
                      const int32_t* game_id, int32_t n, void* workspace, int64_t workspace_bytes, int32_t* action,
                      float* action_weights, float* root_value_out, void* stream) {
  if (!w || !cfg) return MUZ_E_INVALID;
  if (w->num_actions != MUZ_DET_ACTIONS) return MUZ_E_UNSUPPORTED;
  if (cfg->num_simulations < 1 || cfg->num_simulations > kMaxSims) return MUZ_E_UNSUPPORTED;
  if (cfg->max_depth < 1 || cfg->max_depth > kMaxDepth) return MUZ_E_UNSUPPORTED;
  if (cfg->max_num_considered < 1) return MUZ_E_UNSUPPORTED;
  MUZ_HOST_CHECK(n >= 0 && root_logits && root_value && root_embedding && legal_bits && workspace && action &&
                 action_weights && root_value_out);
  MUZ_HOST_CHECK(workspace_bytes >= search_workspace_bytes(n, cfg->num_simulations));
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
  return launch_gumbel_search(*w, sa, root_logits, root_value, root_embedding, legal_bits, gumbel, game_id, n, nullptr,
                              workspace, action, action_weights, root_value_out, (hipStream_t)stream);
}

#ifdef MUZ_STAMPS2
int muz_diag_stamps2(unsigned long long* host_out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_st2), sizeof(unsigned long long) * ST_N);
  if (e != hipSuccess) return (int)e;
  if (reset) {
    unsigned long long z[ST_N] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_st2), z, sizeof(z));
  }
  return (int)e;
}
#endif

#ifdef MUZ_TIMELINE
// out: kWaves x kTlMax records then kWaves counts (reset: zero the counts after the copy)
int muz_diag_timeline(unsigned long long* host_out, unsigned int* host_n, int reset) {
  hipError_t e = hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_tl), sizeof(unsigned long long) * kWaves * kTlMax);
  if (e == hipSuccess) e = hipMemcpyFromSymbol(host_n, HIP_SYMBOL(g_tl_n), sizeof(unsigned int) * kWaves);
  if (e == hipSuccess && reset) {
    unsigned int z[kWaves] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_tl_n), z, sizeof(z));
  }
  return (int)e;
}
#endif

#ifdef MUZ_STAMPS
int muz_diag_stamps(unsigned long long* host_out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_muz_stamps), sizeof(unsigned long long) * 8);
  if (e != hipSuccess) return (int)e;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_muz_stamps), z, sizeof(z));
  }
  return (int)e;
}
#endif

}  // extern "C"
