// Batched Gumbel MuZero search (mctx 0.0.6 gumbel_muzero_policy, as called by
// MuZero_det_MADN/muzero_deterministic_madn.py:663-704) as ONE persistent kernel per search.
//
// A workgroup owns 16 games for the whole search: for every simulation it walks the 16 trees
// (16 lanes per game, two actions per lane, wavefront shuffles for every reduction), gathers the
// 16 parent embeddings into LDS, runs DynamicsNetwork4 + PredictionNetwork4 on MFMA over the
// 16-row tile, expands, and backs up.  No kernel boundary between simulations and no
// inter-workgroup traffic (games are independent).  Node scalars (visits, raw value, value) and
// the current path live in LDS; children arrays and node embeddings live in the workspace (HBM,
// L2/MALL resident), written lazily when a node is created.
#include "launch.hpp"
#include "nn.hpp"

namespace muz {

constexpr int kMaxSims = 100;              // S <= 100 (config (e) uses 100)
constexpr int kMaxNodes = kMaxSims + 1;
constexpr int kMaxDepth = 64;
constexpr int kAPad = 32;                  // children arrays padded to 32 actions
constexpr float kFMin = -3.4028234663852886e38f;   // jnp.finfo(float32).min
constexpr float kTiny = 1.1754943508222875e-38f;   // jnp.finfo(float32).tiny

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
  __device__ __forceinline__ float* e(int g, int node) const { return emb + ((size_t)g * N + node) * LAT; }
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

// ---- 16-lane (one game) reductions with jnp.argmax tie-breaking (first index wins) -------------------
__device__ __forceinline__ void argmax16(float& v, int& i) {
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) {
    const float ov = __shfl_xor(v, m, 16);
    const int oi = __shfl_xor(i, m, 16);
    if (ov > v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  }
}
__device__ __forceinline__ int isum16(int v) {
  v += __shfl_xor(v, 8, 16);
  v += __shfl_xor(v, 4, 16);
  v += __shfl_xor(v, 2, 16);
  v += __shfl_xor(v, 1, 16);
  return v;
}
__device__ __forceinline__ int imax16(int v) {
  v = max(v, __shfl_xor(v, 8, 16));
  v = max(v, __shfl_xor(v, 4, 16));
  v = max(v, __shfl_xor(v, 2, 16));
  v = max(v, __shfl_xor(v, 1, 16));
  return v;
}

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

// qtransform_completed_by_mix_value over one node's children held as (a0 = sub, a1 = sub + 16).
struct Kids {
  float prior[2], value[2], reward[2], disc[2];
  int visits[2], index[2];
  bool ok[2];   // action < A
};

__device__ __forceinline__ void completed_q(const Kids& k, float raw, const SearchArgs& sa, float (&cq)[2],
                                            int& sumv, float& pmax) {
  float q[2];
  float pm = -INFINITY;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    q[h] = k.reward[h] + k.disc[h] * k.value[h];
    if (k.ok[h]) pm = fmaxf(pm, k.prior[h]);
  }
  pm = row_max16(pm);
  float e[2], es = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    e[h] = k.ok[h] ? expf(k.prior[h] - pm) : 0.f;
    es += e[h];
  }
  es = row_sum16(es);
  int sv = 0, mv = 0;
  float sp = 0.f;
  float pp[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    pp[h] = fmaxf(kTiny, e[h] / es);
    if (k.ok[h]) {
      sv += k.visits[h];
      mv = max(mv, k.visits[h]);
      if (k.visits[h] > 0) sp += pp[h];
    }
  }
  sv = isum16(sv);
  mv = imax16(mv);
  sp = row_sum16(sp);
  float wq = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (k.ok[h] && k.visits[h] > 0) wq += pp[h] * q[h] / sp;
  wq = row_sum16(wq);
  const float mixed = (raw + (float)sv * wq) / (float)(sv + 1);
  float lo = INFINITY, hi = -INFINITY;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    cq[h] = (k.visits[h] > 0) ? q[h] : mixed;
    if (k.ok[h]) {
      lo = fminf(lo, cq[h]);
      hi = fmaxf(hi, cq[h]);
    }
  }
  lo = row_min16(lo);
  hi = row_max16(hi);
  const float den = fmaxf(hi - lo, 1e-8f);
  const float scale = (sa.maxvisit_init + (float)mv) * sa.value_scale;
#pragma unroll
  for (int h = 0; h < 2; ++h) cq[h] = scale * ((cq[h] - lo) / den);
  sumv = sv;
  pmax = pm;
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// jax.random.gumbel semantics on our own counter RNG: -log(-log(U[tiny, 1)))
__device__ __forceinline__ float gumbel_noise(unsigned long long seed, int gid, int turn, int a) {
  const unsigned long long h =
      mix64(seed ^ mix64(((unsigned long long)(unsigned)gid << 32) | (unsigned)turn) ^ (unsigned long long)(a + 1) * 0xD6E8FEB86659FD93ull);
  float u = (float)(h >> 40) * (1.0f / 16777216.0f);
  u = fmaxf(u, kTiny);
  return -logf(-logf(u));
}

__global__ __launch_bounds__(256, 1) void k_gumbel_search(muz_net_w Wt, SearchArgs sa, const float* __restrict__ root_logits,
                                                          const float* __restrict__ root_value,
                                                          const float* __restrict__ root_emb,
                                                          const uint32_t* __restrict__ legal,
                                                          const float* __restrict__ gumbel_in,
                                                          const int32_t* __restrict__ game_id, int n,
                                                          const int* __restrict__ n_dev, TreeWs T,
                                                          int32_t* out_action, float* out_weights,
                                                          float* out_value) {
  __shared__ __attribute__((aligned(16))) float smem[kArenaFloats];
  __shared__ int s_visits[kRows][kMaxNodes];
  __shared__ float s_raw[kRows][kMaxNodes];
  __shared__ float s_val[kRows][kMaxNodes];
  __shared__ int p_node[kRows][kMaxDepth];
  __shared__ int p_act[kRows][kMaxDepth];
  __shared__ int p_cvis[kRows][kMaxDepth];
  __shared__ float p_rew[kRows][kMaxDepth];
  __shared__ float p_disc[kRows][kMaxDepth];
  __shared__ float s_gum[kRows][MUZ_DET_ACTIONS];
  __shared__ int s_act[kRows], s_parent[kRows], s_next[kRows], s_depth[kRows], s_ncons[kRows];
  __shared__ unsigned s_legal[kRows];

  if (n_dev) n = *n_dev;
  if ((int)blockIdx.x * kRows >= n) return;
  const Arena ar = Arena::carve(smem);
  const int A = Wt.num_actions;
  const int row = threadIdx.x >> 4, sub = threadIdx.x & 15;
  const int g = blockIdx.x * kRows + row;
  const bool valid = g < n;
  const int a0 = sub, a1 = sub + 16;
  const bool ok1 = a1 < A;

  // ---------------- root: instantiate_tree_from_root with masked logits (policies.py _mask_invalid_actions)
  if (valid) {
    const unsigned lb = legal[g];
    const int gid = game_id ? game_id[g] : g;
    float l0 = root_logits[(size_t)g * A + a0];
    float l1 = ok1 ? root_logits[(size_t)g * A + a1] : -INFINITY;
    const float lm = row_max16(fmaxf(l0, l1));
    const bool inv0 = ((lb >> a0) & 1u) == 0u, inv1 = !ok1 || ((lb >> a1) & 1u) == 0u;
    l0 = inv0 ? kFMin : l0 - lm;
    l1 = inv1 ? kFMin : l1 - lm;
    const size_t b0 = T.ca(g, 0, 0);
    T.c_prior[b0 + a0] = l0;
    T.c_index[b0 + a0] = -1;
    T.c_visits[b0 + a0] = 0;
    T.c_value[b0 + a0] = 0.f;
    T.c_reward[b0 + a0] = 0.f;
    T.c_disc[b0 + a0] = 0.f;
    if (ok1) {
      T.c_prior[b0 + a1] = l1;
      T.c_index[b0 + a1] = -1;
      T.c_visits[b0 + a1] = 0;
      T.c_value[b0 + a1] = 0.f;
      T.c_reward[b0 + a1] = 0.f;
      T.c_disc[b0 + a1] = 0.f;
    }
    s_gum[row][a0] = gumbel_in ? gumbel_in[(size_t)g * A + a0] : sa.gumbel_scale * gumbel_noise(sa.seed, gid, sa.turn, a0);
    if (ok1)
      s_gum[row][a1] = gumbel_in ? gumbel_in[(size_t)g * A + a1] : sa.gumbel_scale * gumbel_noise(sa.seed, gid, sa.turn, a1);
    float* e0 = T.e(g, 0);
    for (int c = sub; c < LAT; c += 16) e0[c] = root_emb[(size_t)g * LAT + c];
    if (sub == 0) {
      const float v = root_value[g];
      s_visits[row][0] = 1;
      s_raw[row][0] = v;
      s_val[row][0] = v;
      s_legal[row] = lb;
      s_ncons[row] = min(sa.max_considered, __popc(lb & ((1u << A) - 1u)));
    }
  }
  __syncthreads();

#pragma unroll 1
  for (int sim = 0; sim < sa.S; ++sim) {
    // ---------------- simulate (search.py simulate): walk from the root
    if (valid) {
      int node = 0, depth = 0, act = 0, nxt = -1;
      const unsigned lb = s_legal[row];
      while (true) {
        Kids k;
        const size_t base = T.ca(g, node, 0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int a = h ? a1 : a0;
          k.ok[h] = h ? ok1 : true;
          const int ai = k.ok[h] ? a : a0;
          k.prior[h] = T.c_prior[base + ai];
          k.value[h] = T.c_value[base + ai];
          k.reward[h] = T.c_reward[base + ai];
          k.disc[h] = T.c_disc[base + ai];
          k.visits[h] = k.ok[h] ? T.c_visits[base + ai] : 0;
          k.index[h] = T.c_index[base + ai];
        }
        float cq[2];
        int sumv;
        float pmax;
        completed_q(k, s_raw[row][node], sa, cq, sumv, pmax);
        float sc[2];
        if (depth == 0) {
          // gumbel_muzero_root_action_selection + seq_halving.score_considered + masked_argmax
          const int cv = considered_visit(s_ncons[row], sa.S, sumv);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int a = h ? a1 : a0;
            const float s = fmaxf(-1e9f, s_gum[row][k.ok[h] ? a : a0] + (k.prior[h] - pmax) + cq[h]) +
                            (k.visits[h] == cv ? 0.f : -INFINITY);
            const bool inv = !k.ok[h] || ((lb >> a) & 1u) == 0u;
            sc[h] = inv ? -INFINITY : s;
          }
        } else {
          // gumbel_muzero_interior_action_selection: softmax(prior + cq) - N / (1 + sum N)
          float z[2], zm = -INFINITY;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            z[h] = k.prior[h] + cq[h];
            if (k.ok[h]) zm = fmaxf(zm, z[h]);
          }
          zm = row_max16(zm);
          float ez[2], zs = 0.f;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            ez[h] = k.ok[h] ? expf(z[h] - zm) : 0.f;
            zs += ez[h];
          }
          zs = row_sum16(zs);
#pragma unroll
          for (int h = 0; h < 2; ++h)
            sc[h] = k.ok[h] ? (ez[h] / zs - (float)k.visits[h] / (float)(1 + sumv)) : -INFINITY;
        }
        float bv = sc[0];
        int bi = a0;
        if (ok1 && (sc[1] > bv)) {
          bv = sc[1];
          bi = a1;
        }
        argmax16(bv, bi);
        const int owner = bi & 15;
        const bool hi = bi >= 16;
        const int child = __shfl(hi ? k.index[1] : k.index[0], owner, 16);
        const float rw = __shfl(hi ? k.reward[1] : k.reward[0], owner, 16);
        const float dc = __shfl(hi ? k.disc[1] : k.disc[0], owner, 16);
        const int cvis = __shfl(hi ? k.visits[1] : k.visits[0], owner, 16);
        if (sub == 0) {
          p_node[row][depth] = node;
          p_act[row][depth] = bi;
          p_rew[row][depth] = rw;
          p_disc[row][depth] = dc;
          p_cvis[row][depth] = cvis;
        }
        act = bi;
        nxt = child;
        ++depth;
        if (child == -1 || depth >= sa.D) break;
        node = child;
      }
      if (sub == 0) {
        s_parent[row] = node;
        s_act[row] = act;
        s_next[row] = (nxt == -1) ? sim + 1 : nxt;
        s_depth[row] = depth;
      }
    } else if (sub == 0) {
      s_act[row] = 0;
    }
    __syncthreads();
    // ---------------- expand (search.py expand): parent embedding -> recurrent_fn
    {
      const float* pe = valid ? T.e(g, s_parent[row]) : nullptr;
      for (int c = sub; c < LAT; c += 16) ar.L[row * LD + c] = valid ? pe[c] : 0.f;
    }
    __syncthreads();
    // Launder the weight table once per simulation so the compiler re-derives the ~60 layer
    // addresses inside the loop instead of pinning them in registers across it.
    // (Wt is kernel argument 0, so it sits at offset 0 of the kernarg segment.)
    const muz_net_w* wl = (const muz_net_w*)(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(wl));
    dyn16(wl->dyn, A, s_act, ar);
    const int nx = s_next[row];
    if (valid) {
      float* ne = T.e(g, nx);
      for (int c = sub; c < LAT; c += 16) ne[c] = ar.T[row * LD + c];
    }
    __syncthreads();
    pred16(wl->pred, A, ar.T, ar);
    if (valid) {
      const bool fresh = nx == sim + 1;
      const size_t nb = T.ca(g, nx, 0);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int a = h ? a1 : a0;
        if (h && !ok1) break;
        T.c_prior[nb + a] = ar.U[row * LD + a];
        if (fresh) {
          T.c_index[nb + a] = -1;
          T.c_visits[nb + a] = 0;
          T.c_value[nb + a] = 0.f;
          T.c_reward[nb + a] = 0.f;
          T.c_disc[nb + a] = 0.f;
        }
      }
      if (sub == 0) {
        const int par = s_parent[row], act = s_act[row];
        const float v = ar.v0[row], rw = ar.v1[row], dc = ar.v2[row];
        const size_t eb = T.ca(g, par, act);
        T.c_index[eb] = nx;
        T.c_reward[eb] = rw;
        T.c_disc[eb] = dc;
        s_raw[row][nx] = v;
        s_val[row][nx] = v;
        s_visits[row][nx] = fresh ? 1 : s_visits[row][nx] + 1;
        // ---------------- backward (search.py backward) along the recorded path
        float leaf = v;
        int idx = nx;
        const int d = s_depth[row];
        for (int lvl = d - 1; lvl >= 0; --lvl) {
          const int parent = p_node[row][lvl];
          const int pa = p_act[row][lvl];
          const int cnt = s_visits[row][parent];
          const float r = (lvl == d - 1) ? rw : p_rew[row][lvl];
          const float dsc = (lvl == d - 1) ? dc : p_disc[row][lvl];
          leaf = r + dsc * leaf;
          const float pv = (s_val[row][parent] * (float)cnt + leaf) / ((float)cnt + 1.0f);
          const size_t ei = T.ca(g, parent, pa);
          T.c_value[ei] = s_val[row][idx];
          T.c_visits[ei] = p_cvis[row][lvl] + 1;
          s_val[row][parent] = pv;
          s_visits[row][parent] = cnt + 1;
          idx = parent;
        }
      }
    }
    __syncthreads();
  }

  // ---------------- final action (policies.py gumbel_muzero_policy tail)
  if (valid) {
    Kids k;
    const size_t base = T.ca(g, 0, 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int a = h ? a1 : a0;
      k.ok[h] = h ? ok1 : true;
      const int ai = k.ok[h] ? a : a0;
      k.prior[h] = T.c_prior[base + ai];
      k.value[h] = T.c_value[base + ai];
      k.reward[h] = T.c_reward[base + ai];
      k.disc[h] = T.c_disc[base + ai];
      k.visits[h] = k.ok[h] ? T.c_visits[base + ai] : 0;
      k.index[h] = -1;
    }
    float cq[2];
    int sumv;
    float pmax;
    completed_q(k, s_raw[row][0], sa, cq, sumv, pmax);
    const unsigned lb = s_legal[row];
    const int cv = imax16(max(k.visits[0], k.ok[1] ? k.visits[1] : 0));
    float sc[2], z[2];
    bool inv[2];
    float zm = -INFINITY;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int a = h ? a1 : a0;
      inv[h] = !k.ok[h] || ((lb >> a) & 1u) == 0u;
      const float s = fmaxf(-1e9f, s_gum[row][k.ok[h] ? a : a0] + (k.prior[h] - pmax) + cq[h]) +
                      (k.visits[h] == cv ? 0.f : -INFINITY);
      sc[h] = inv[h] ? -INFINITY : s;
      z[h] = k.prior[h] + cq[h];
      if (k.ok[h]) zm = fmaxf(zm, z[h]);
    }
    float bv = sc[0];
    int bi = a0;
    if (ok1 && sc[1] > bv) {
      bv = sc[1];
      bi = a1;
    }
    argmax16(bv, bi);
    // action_weights = softmax(_mask_invalid_actions(prior + completed_q))
    zm = row_max16(zm);
    float ez[2], zs = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float zz = inv[h] ? kFMin : z[h] - zm;
      ez[h] = k.ok[h] ? expf(zz - 0.f) : 0.f;
    }
    // softmax subtracts the max of the masked logits (<= 0 here; equals 0 unless all are invalid)
    float mm = -INFINITY;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (k.ok[h]) mm = fmaxf(mm, inv[h] ? kFMin : z[h] - zm);
    mm = row_max16(mm);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ez[h] = k.ok[h] ? expf((inv[h] ? kFMin : z[h] - zm) - mm) : 0.f;
      zs += ez[h];
    }
    zs = row_sum16(zs);
    out_weights[(size_t)g * A + a0] = ez[0] / zs;
    if (ok1) out_weights[(size_t)g * A + a1] = ez[1] / zs;
    if (sub == 0) {
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
  k_gumbel_search<<<(n + kRows - 1) / kRows, 256, 0, s>>>(w, sa, root_logits, root_value, root_emb, legal, gumbel,
                                                          game_id, n, n_dev, T, action, weights, value);
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

}  // extern "C"
