// mctx 0.0.6 gumbel_muzero_policy in C++ for any action count A (the det / DOG CPU restatements:
// oracle/cpu_selfplay.cpp at A = 24, oracle/cpu_dog.cpp at A = 806).  TEST INFRASTRUCTURE / CPU BASELINE ONLY.
//
// Follows oracle/mctx_gumbel.py function by function (itself a restatement of mctx's policies.py, search.py,
// action_selection.py, qtransforms.py, seq_halving.py) and rounds exactly like it: each product rounded on its own
// (rnd() keeps the compiler from fusing it into an fma), exp correctly rounded (float64, then rounded once), sums
// over the actions in numpy's pairwise order up to 128 actions (mctx_gumbel.row_sum) and in the wide device
// search's lane order beyond (mctx_gumbel.lane_tree_sum).  Given the same network outputs, both sides agree bit
// for bit (tests/test_cpu_baseline.py, tests/test_cpu_baseline_dog.py).
//
// One deliberate difference in cost, not in result: a node's prior probabilities softmax(prior) are computed once
// when the node is expanded (the NumPy search recomputes them at every visit; the values are the same).
#pragma once
#include "cpu_nets.hpp"

namespace {

inline float rnd(float x) {
  asm volatile("" : "+x"(x));
  return x;
}

// numpy's pairwise sum of a contiguous float32 row of n <= 128 (8 partial sums, then a tree, then the tail)
inline float numpy_pairwise_sum(const float* v, int n) {
  if (n < 8) {
    float s = -0.0f;
    for (int i = 0; i < n; ++i) s = rnd(s + v[i]);
    return s;
  }
  float r[8];
  for (int j = 0; j < 8; ++j) r[j] = v[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] = rnd(r[j] + v[i + j]);
  float s = rnd(rnd(rnd(r[0] + r[1]) + rnd(r[2] + r[3])) + rnd(rnd(r[4] + r[5]) + rnd(r[6] + r[7])));
  for (; i < n; ++i) s = rnd(s + v[i]);
  return s;
}

// mctx_gumbel.lane_tree_sum: lane l of 32 adds entries l, l + 32, ... in turn; the 32 lane sums then pair up in a
// balanced tree in lane order
inline float lane_tree_sum(const float* v, int n) {
  float s[32];
  for (int l = 0; l < 32; ++l) {
    float a = l < n ? v[l] : -0.0f;
    for (int k = l + 32; k < n; k += 32) a = rnd(a + v[k]);
    s[l] = a;
  }
  for (int w = 16; w >= 1; w >>= 1)
    for (int l = 0; l < w; ++l) s[l] = rnd(s[2 * l] + s[2 * l + 1]);
  return s[0];
}

template <int A>
inline float row_sum(const float* v) {
  if constexpr (A <= 128) return numpy_pairwise_sum(v, A);
  else return lane_tree_sum(v, A);
}

inline float exp_cr(float x) { return (float)std::exp((double)x); }

template <int A>
void softmax_tree(const float* x, float* out) {
  float m = -kInf, u[A];
  for (int i = 0; i < A; ++i) m = std::max(m, x[i]);
  for (int i = 0; i < A; ++i) u[i] = exp_cr(x[i] - m);
  const float s = row_sum<A>(u);
  for (int i = 0; i < A; ++i) out[i] = u[i] / s;
}

std::vector<int> considered_sequence(int m, int S) {   // seq_halving.get_sequence_of_considered_visits
  std::vector<int> seq;
  if (m <= 1) {
    for (int i = 0; i < S; ++i) seq.push_back(i);
    return seq;
  }
  const int log2max = (int)std::ceil(std::log2((double)m));
  std::vector<int> visits(m, 0);
  int k = m;
  while ((int)seq.size() < S) {
    const int extra = std::max(1, (int)(S / (log2max * k)));
    for (int e = 0; e < extra; ++e) {
      for (int i = 0; i < k; ++i) seq.push_back(visits[i]);
      for (int i = 0; i < k; ++i) visits[i] += 1;
    }
    k = std::max(2, k / 2);
  }
  seq.resize(S);
  return seq;
}

struct Search {
  int S, D;
  std::vector<std::vector<int>> table;   // [m][sim]
  void init(int s, int d) {
    S = s;
    D = d;
    table.clear();
    for (int m = 0; m <= 16; ++m) table.push_back(considered_sequence(m, S));
  }
};

// mctx Tree of one game: N = S + 1 nodes, children arrays [N][A]; pp = max(tiny, softmax(prior)) per node
template <int A>
struct Tree {
  int N = 0;
  std::vector<int> visits, parent, afp, c_index, c_visits;
  std::vector<float> raw, value, c_prior, c_pp, c_value, c_reward, c_disc, emb;
  void init(int n) {
    N = n;
    visits.assign(n, 0);
    parent.assign(n, -1);
    afp.assign(n, -1);
    raw.assign(n, 0.f);
    value.assign(n, 0.f);
    c_index.assign((size_t)n * A, -1);
    c_visits.assign((size_t)n * A, 0);
    c_prior.assign((size_t)n * A, 0.f);
    c_pp.assign((size_t)n * A, 0.f);
    c_value.assign((size_t)n * A, 0.f);
    c_reward.assign((size_t)n * A, 0.f);
    c_disc.assign((size_t)n * A, 0.f);
    emb.assign((size_t)n * kLat, 0.f);
  }
  void update(int node, const float* prior, float v, const float* e) {
    float* pr = &c_prior[(size_t)node * A];
    float* pp = &c_pp[(size_t)node * A];
    std::memcpy(pr, prior, sizeof(float) * A);
    softmax_tree<A>(pr, pp);
    for (int a = 0; a < A; ++a) pp[a] = std::max(kTiny, pp[a]);
    raw[node] = v;
    value[node] = v;
    visits[node] += 1;
    std::memcpy(&emb[(size_t)node * kLat], e, sizeof(float) * kLat);
  }
};

// qtransform_completed_by_mix_value(value_scale 0.5, maxvisit_init 50, rescale, mixed value, eps 1e-8)
template <int A>
void completed_q(const Tree<A>& t, int node, float* cq) {
  const size_t o = (size_t)node * A;
  const int* vis = &t.c_visits[o];
  const float* pp = &t.c_pp[o];
  float q[A], tmp[A];
  int sumv = 0, maxv = 0;
  for (int a = 0; a < A; ++a) {
    q[a] = rnd(t.c_reward[o + a] + rnd(t.c_disc[o + a] * t.c_value[o + a]));
    sumv += vis[a];
    maxv = std::max(maxv, vis[a]);
    tmp[a] = vis[a] > 0 ? pp[a] : 0.f;
  }
  const float sp = row_sum<A>(tmp);
  for (int a = 0; a < A; ++a) tmp[a] = vis[a] > 0 ? rnd(rnd(pp[a] * q[a]) / sp) : 0.f;
  const float wq = row_sum<A>(tmp);
  const float mixed = rnd(t.raw[node] + rnd((float)sumv * wq)) / (float)(sumv + 1);
  float lo = kInf, hi = -kInf;
  for (int a = 0; a < A; ++a) {
    cq[a] = vis[a] > 0 ? q[a] : mixed;
    lo = std::min(lo, cq[a]);
    hi = std::max(hi, cq[a]);
  }
  const float den = std::max(hi - lo, 1e-8f);
  const float scale = (50.0f + (float)maxv) * 0.5f;
  for (int a = 0; a < A; ++a) cq[a] = scale * ((cq[a] - lo) / den);
}

// score_considered + masked argmax (root) / softmax(prior + cq) - N / (1 + sum N) (interior)
template <int A>
int select_child(const Tree<A>& t, int node, int depth, const bool* invalid, const float* gumbel, const Search& sr,
                 int ncons) {
  float cq[A], sc[A];
  completed_q<A>(t, node, cq);
  const int* vis = &t.c_visits[(size_t)node * A];
  const float* prior = &t.c_prior[(size_t)node * A];
  int sumv = 0;
  for (int a = 0; a < A; ++a) sumv += vis[a];
  if (depth == 0) {
    const int cv = sr.table[ncons][std::min(sumv, sr.S - 1)];
    float pm = -kInf;
    for (int a = 0; a < A; ++a) pm = std::max(pm, prior[a]);
    for (int a = 0; a < A; ++a) {
      const float s = std::max(-1e9f, gumbel[a] + (prior[a] - pm) + cq[a]) + (vis[a] == cv ? 0.f : -kInf);
      sc[a] = invalid[a] ? -kInf : s;
    }
  } else {
    float z[A], p[A];
    for (int a = 0; a < A; ++a) z[a] = prior[a] + cq[a];
    softmax_tree<A>(z, p);
    for (int a = 0; a < A; ++a) sc[a] = p[a] - (float)vis[a] / (float)(1 + sumv);
  }
  return argmax(sc, A);
}

// One batched gumbel_muzero_policy over B games, root inference outputs given.  rec(action[B], emb[B][256], B,
// reward, discount, logits[B][A], value, next_emb) is the recurrent inference.
template <int A, class Rec>
void gumbel_search(const Search& sr, int B, const float* logits, const float* rvalue, const float* remb,
                   const bool* invalid, const float* gumbel, std::vector<Tree<A>>& trees, int* action_out,
                   float* weights_out, float* value_out, Rec&& rec) {
  const int S = sr.S;
  if ((int)trees.size() < B) trees.resize(B);
  std::vector<int> ncons(B), parent(B), act(B), nxt(B);
  std::vector<float> rew(B), disc(B), lg((size_t)B * A), val(B), ne((size_t)B * kLat), pe((size_t)B * kLat);
  for (int b = 0; b < B; ++b) {
    Tree<A>& t = trees[b];
    t.init(S + 1);
    std::vector<float> pr(A);
    float m = -kInf;
    for (int a = 0; a < A; ++a) m = std::max(m, logits[(size_t)b * A + a]);
    int nv = 0;
    for (int a = 0; a < A; ++a) {
      pr[a] = invalid[(size_t)b * A + a] ? kFMin : logits[(size_t)b * A + a] - m;
      nv += !invalid[(size_t)b * A + a];
    }
    ncons[b] = std::min(16, nv);
    t.update(0, pr.data(), rvalue[b], remb + (size_t)b * kLat);
  }
  for (int sim = 0; sim < S; ++sim) {
    for (int b = 0; b < B; ++b) {   // simulate
      const Tree<A>& t = trees[b];
      int node = 0, depth = 0, a = 0;
      while (true) {
        a = select_child<A>(t, node, depth, invalid + (size_t)b * A, gumbel + (size_t)b * A, sr, ncons[b]);
        const int child = t.c_index[(size_t)node * A + a];
        ++depth;
        if (child == -1 || depth >= sr.D) break;
        node = child;
      }
      parent[b] = node;
      act[b] = a;
      const int c = t.c_index[(size_t)node * A + a];
      nxt[b] = c == -1 ? sim + 1 : c;
      std::memcpy(&pe[(size_t)b * kLat], &t.emb[(size_t)node * kLat], sizeof(float) * kLat);
    }
    rec(act.data(), pe.data(), B, rew.data(), disc.data(), lg.data(), val.data(), ne.data());
    for (int b = 0; b < B; ++b) {   // expand + backward
      Tree<A>& t = trees[b];
      const int p = parent[b], a = act[b], nn = nxt[b];
      t.update(nn, &lg[(size_t)b * A], val[b], &ne[(size_t)b * kLat]);
      t.c_index[(size_t)p * A + a] = nn;
      t.c_reward[(size_t)p * A + a] = rew[b];
      t.c_disc[(size_t)p * A + a] = disc[b];
      t.parent[nn] = p;
      t.afp[nn] = a;
      float leaf = t.value[nn];
      int idx = nn;
      while (idx != 0) {
        const int pr = t.parent[idx], pa = t.afp[idx];
        const int cnt = t.visits[pr];
        const size_t e = (size_t)pr * A + pa;
        leaf = rnd(t.c_reward[e] + rnd(t.c_disc[e] * leaf));
        t.value[pr] = rnd(rnd(t.value[pr] * (float)cnt) + leaf) / ((float)cnt + 1.0f);
        t.visits[pr] = cnt + 1;
        t.c_value[e] = t.value[idx];
        t.c_visits[e] += 1;
        idx = pr;
      }
    }
  }
  for (int b = 0; b < B; ++b) {   // final action + action_weights (policies.py tail)
    const Tree<A>& t = trees[b];
    float cq[A], sc[A], z[A];
    completed_q<A>(t, 0, cq);
    int cv = 0;
    for (int a = 0; a < A; ++a) cv = std::max(cv, t.c_visits[a]);
    const float* prior = &t.c_prior[0];
    float pm = -kInf;
    for (int a = 0; a < A; ++a) pm = std::max(pm, prior[a]);
    const bool* inv = invalid + (size_t)b * A;
    for (int a = 0; a < A; ++a) {
      const float sv = std::max(-1e9f, gumbel[(size_t)b * A + a] + (prior[a] - pm) + cq[a]) +
                       (t.c_visits[a] == cv ? 0.f : -kInf);
      sc[a] = inv[a] ? -kInf : sv;
      z[a] = prior[a] + cq[a];
    }
    action_out[b] = argmax(sc, A);
    float zm = -kInf;
    for (int a = 0; a < A; ++a) zm = std::max(zm, z[a]);
    for (int a = 0; a < A; ++a) z[a] = inv[a] ? kFMin : z[a] - zm;
    softmax_tree<A>(z, weights_out + (size_t)b * A);
    value_out[b] = t.value[0];
  }
}

// counter-based Gumbel noise of the engine (csrc/rng.hpp, oracle/selfplay.py:gumbel_noise)
template <int A>
void gumbel_noise(uint64_t seed, int gid, int turn, float scale, float* out) {
  for (int a = 0; a < A; ++a) {
    const uint64_t h = mix64(seed ^ mix64(((uint64_t)(uint32_t)gid << 32) | (uint32_t)turn) ^
                             ((uint64_t)(a + 1) * 0xD6E8FEB86659FD93ull));
    float u = (float)(h >> 40) * (1.0f / 16777216.0f);
    u = std::max(u, kTiny);
    out[a] = scale * (-std::log(-std::log(u)));
  }
}

}  // namespace
