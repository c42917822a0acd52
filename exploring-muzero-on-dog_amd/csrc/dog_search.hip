// run_muzero_mcts of the DOG slice (MuZero_DOG/muzero_dog.py:101-137: mctx.gumbel_muzero_policy with
// qtransform_completed_by_mix_value(value_scale=0.5), gumbel_scale = temperature) at A = 806, as ONE persistent
// kernel per search -- k_gumbel_search's structure (csrc/search.hip) with wide nodes:
//
//  * a workgroup owns 16 games (8 -- one per wave -- up to 2048 games: SPARSE); game `row` has 32 lanes and lane
//    `sub` holds children sub, sub + 32, ..., sub + 800 (26 slots, 832 per node; slots >= 806 are padding);
//  * every node's children (the root's included) live in the workspace, [n][S+1][832] per field; the root's legal
//    words sit in LDS (word j bit `sub` is child sub + 32 j, the layout of muz_dog_legal's mask);
//  * sums over a node's children run in the lane order oracle/mctx_gumbel.py lane_tree_sum restates (each lane its
//    slots in turn, then a balanced tree over the 32 lanes), maxima / minima / integer sums are exact, exp is
//    correctly rounded and nothing contracts to fma -- so with identical network outputs the tree arithmetic
//    agrees with the restatement bit for bit;
//  * interior selections are certified from the visited children and the best unvisited prior (wselect_certified;
//    the exact 806-exponential path when no certificate), nodes walked before are loaded compactly from their
//    visited-child records and top-prior lists (wnode_compact), the root and first walks in full (wnode_full);
//  * expand runs DynamicsNetwork4 + PredictionNetwork4 at A = 806 on the 16-row tile (nn.hpp, dog_nets.hpp), the
//    806 prior logits going from the logits chunks straight into the new node's children.
#define MUZ_OPAQUE_TID 1   // (nn.hpp tid())
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
static_assert(kWMaxSims <= 255, "visit counts in 8 bits (WNode::vis4)");
static_assert(kWPad >= kDogA && kWWords * 32 >= kDogA, "slots");
static_assert(2 * kRows * kDogA <= kArenaFloats, "the walk's per-child arrays live in the idle network arena");

// A node's children: the 806 prior logits are written when the node is expanded; the statistics of a child are
// written only when it is first visited (its expansion writes index / reward / discount, the backups value / visits),
// and the node's visited mask says which children hold them -- every other child is {value 0, reward 0, discount 0,
// index -1, visits 0}, as mctx initialises them.  (Round 5 initialised all 806 children's statistics at every
// expansion: ~20 KB of HBM writes per expansion of the ~4.6 KB the search needs, and the root's full load per
// simulation read 24 B per child.)
struct WTree {
  float* c_prior;     // [n][N][832] prior logits
  f32x4* c_stat;      // [n][N][832] per visited child {value, reward, discount, index (int bits)}
  int32_t* c_visits;  // [n][N][832] per visited child
  uint32_t* c_vmask;  // [n][N][32] lane-major visited mask: word l, bit j <=> child l + 32 j visited
  float* emb;         // [n][N][256]
  float* gum;         // [n][832] the root's Gumbel noise + (prior - max prior), drawn once per search
  f32x4* vrec;        // [n][N][32][2] each node's visited children in first-visit order (s_vcnt: how many; -1
                      // overflow), one 32-byte record each: {child, visits, prior, value} {reward, discount, node, -}
  float* topp;        // [n][N][kWTop] each node's kWTop largest prior logits (value desc, index asc) ...
  int32_t* topi;      // [n][N][kWTop] ... and their children
  int N;
  __device__ __forceinline__ size_t ca(int g, int node, int a) const { return ((size_t)g * N + node) * kWPad + a; }
  __device__ __forceinline__ AS1 float* e(int g, int node) const { return gpw(emb) + ((size_t)g * N + node) * LAT; }
  __device__ __forceinline__ AS1 float* prior() const { return gpw(c_prior); }
  __device__ __forceinline__ AS1 f32x4* stat() const { return gpw(c_stat); }
  // field k (0 value, 1 reward, 2 discount, 3 index) of child entry e
  __device__ __forceinline__ AS1 float* fld(size_t e, int k) const {
    return gpw(reinterpret_cast<float*>(c_stat)) + 4 * e + k;
  }
  __device__ __forceinline__ AS1 int32_t* visits() const { return gpw(c_visits); }
  __device__ __forceinline__ AS1 uint32_t* vmask(int g, int node) const {
    return gpw(c_vmask) + ((size_t)g * N + node) * kRowLanes;
  }
  __device__ __forceinline__ AS1 f32x4* vr(int g, int node) const;
  __device__ __forceinline__ AS1 float* tp(int g, int node) const;
  __device__ __forceinline__ AS1 int32_t* ti(int g, int node) const;
};
constexpr int kWList = 32;   // visited children a node's list holds
#ifndef MUZ_DOG_WTOP
#define MUZ_DOG_WTOP 8       // (a build switch for the A/B of the top-prior list's length)
#endif
constexpr int kWTop = MUZ_DOG_WTOP;   // largest priors a node keeps
// The per-node sizes of the compact-load arrays: the accessors below, carve_wide and dog_search_workspace_bytes all
// derive their strides from these (round 4's kWTop = 4 fault: an accessor kept a literal 8 the carve did not)
constexpr int kWRecF4 = 2 * kWList;                        // f32x4 per node's visited list (two per record)
constexpr size_t kWRecBytes = sizeof(f32x4) * kWRecF4;     // = kWList 32-byte records
constexpr size_t kWTopBytes = sizeof(float) * kWTop;       // topp; topi the same in int32
static_assert(kWRecBytes == (size_t)kWList * 32, "a visited-child record is 32 bytes");
static_assert(sizeof(int32_t) == sizeof(float), "topi and topp share the stride");
static_assert(kWList <= kRowLanes && kWList < 127, "one record per lane (wrec_load), lengths in signed char");
static_assert(kWTop >= 2 && kWTop < kRowLanes, "top list: one entry per lane, a 32-bit ballot mask (wnode_compact)");
__device__ __forceinline__ AS1 f32x4* WTree::vr(int g, int node) const {
  return gpw(vrec) + ((size_t)g * N + node) * kWRecF4;
}
__device__ __forceinline__ AS1 float* WTree::tp(int g, int node) const {
  return gpw(topp) + ((size_t)g * N + node) * kWTop;
}
__device__ __forceinline__ AS1 int32_t* WTree::ti(int g, int node) const {
  return gpw(topi) + ((size_t)g * N + node) * kWTop;
}

static size_t wide_children_bytes(int64_t n, int N) { return (size_t)n * N * kWPad * 4; }

static WTree carve_wide(void* ws, int n, int N) {
  char* p = (char*)ws;
  const size_t cb = wide_children_bytes(n, N);
  WTree t;
  t.c_stat = (f32x4*)p;
  p += 4 * cb;
  t.c_prior = (float*)p;
  p += cb;
  t.c_visits = (int32_t*)p;
  p += cb;
  t.c_vmask = (uint32_t*)p;
  p += (size_t)n * N * kRowLanes * 4;
  t.emb = (float*)p;
  p += (size_t)n * N * LAT * 4;
  t.gum = (float*)p;
  p += (size_t)n * kWPad * 4;
  t.vrec = (f32x4*)p;
  p += (size_t)n * N * kWRecBytes;
  t.topp = (float*)p;
  p += (size_t)n * N * kWTopBytes;
  t.topi = (int32_t*)p;
  t.N = N;
  return t;
}

// exp correctly rounded (float64, rounded once): oracle/mctx_gumbel.py exp_cr, search.hip exp_cr
// (A/B, profiles/r4k_dog_ab.log: a float __expf in its place -- wrong rounding -- was 22-27 % faster per search)
__device__ __forceinline__ float exp_cr_w(float x) { return (float)exp((double)x); }

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
// (value, index) argmax across the row's lanes, row_argmax's order (larger value, then smaller index)
__device__ __forceinline__ void wargmax_row2(float& v, int& i) {
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
}
__device__ __forceinline__ int wargmax_row(float v, int i) {
  wargmax_row2(v, i);
  return i;
}

// argmax over the row's 806 children of score f(j) (this lane's slot j), jnp.argmax tie-break (first index):
// this lane's slots in ascending order (strict >), then wargmax_row.  Streams the scores: no per-slot array.
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
  return wargmax_row(v, i);
}

constexpr int kWHalf = kWJ / 2;   // slots per load batch

// score_considered + masked_argmax at the root: gp = the root's Gumbel noise + (prior - max prior) (T.gum), loaded in
// two batches of 13 slots (one at a time, the loads serialised on their uses: 26 L2 round trips)
template <class Vis, class Legal>
__device__ __forceinline__ int wroot_argmax(const WTree& T, int g, int sub, const float* cq, Vis vis,
                                            int cv, Legal legal_of) {
  float v = -INFINITY;
  int i = sub;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float gp[kWHalf];
#pragma unroll
    for (int k = 0; k < kWHalf; ++k) gp[k] = tree_ld(gpw(T.gum) + (size_t)g * kWPad + sub + kRowLanes * (kWHalf * h + k));
    __builtin_amdgcn_sched_barrier(0);   // the batch's loads in flight together
#pragma unroll
    for (int k = 0; k < kWHalf; ++k) {
      const int j = kWHalf * h + k, a = sub + kRowLanes * j;
      float x = -INFINITY;
      if (a < kDogA && legal_of(j)) x = fmaxf(-1e9f, gp[k] + cq[a]) + (vis(j) == cv ? 0.f : -INFINITY);
      if (x > v) {
        v = x;
        i = a;
      }
    }
  }
  return wargmax_row(v, i);
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
  float* cq;     // [806] of this row, LDS (the visited children's; wfill_unvisited writes the rest)
  uint32_t vis4[(kWJ + 3) / 4];   // visit counts, 8 bits per slot (<= S <= 100): registers the walk cannot spare
  __device__ __forceinline__ int vis(int j) const { return (int)((vis4[j >> 2] >> (8 * (j & 3))) & 255u); }
  float pm;      // max prior logit
  int sv, mv;    // sum / max of the visit counts
  float es;      // sum of exp(prior - pm) (the prior normaliser)
  float K;       // the transformed completed Q every unvisited child shares
  float u1, u2;  // the largest and second-largest prior logit among the unvisited children (u2 = u1 on a tie)
  int ui;        // the child holding u1 (the smallest such index)
  unsigned vm;   // this lane's visited slots (bit j: slot j)
};

// (value, index) top-2 across the row's lanes: the first by (larger value, smaller index), the second the largest
// of the rest (equal to the first on a tie).  Each butterfly step merges disjoint lane sets.
__device__ __forceinline__ void wtop2_row(float& v1, int& i1, float& v2) {
  auto merge = [&](float o1, int oi, float o2) {
    float lo1 = o1;
    if (o1 > v1 || (o1 == v1 && oi < i1)) {
      lo1 = v1;
      v1 = o1;
      i1 = oi;
    }
    v2 = fmaxf(fmaxf(v2, o2), lo1);
  };
  merge(dpp<DPP_XOR1>(v1), dpp<DPP_XOR1>(i1), dpp<DPP_XOR1>(v2));
  merge(dpp<DPP_XOR2>(v1), dpp<DPP_XOR2>(i1), dpp<DPP_XOR2>(v2));
  merge(dpp<DPP_HALF_MIRROR>(v1), dpp<DPP_HALF_MIRROR>(i1), dpp<DPP_HALF_MIRROR>(v2));
  merge(dpp<DPP_MIRROR>(v1), dpp<DPP_MIRROR>(i1), dpp<DPP_MIRROR>(v2));
  const LoHi<float> p1 = swap16(v1), p2 = swap16(v2);
  const LoHi<int> pi = swap16(i1);
  v1 = p1.lo;
  i1 = pi.lo;
  v2 = p2.lo;
  merge(p1.hi, pi.hi, p2.hi);
}

// Full load of one node: all 806 children (priors and q into LDS, visit counts into registers), their maximum prior,
// visit sum / maximum, the two largest unvisited priors and this lane's visited slots.  ces: this row's per-node sum
// of exp(prior - max prior) (the softmax normaliser of the node's prior probabilities), computed at the node's first
// walk and kept until the node is expanded again -- its priors do not change in between, so the 806 exponentials
// are not recomputed at every visit (< 0: not cached); with it the node's kWTop largest priors go to T.tp / T.ti for
// the compact loads.
__device__ __forceinline__ void wnode_full(WNode& nd, const WTree& T, int g, int node, int sub, float* ces) {
#pragma clang fp contract(off)
  st_count(13);   // (diagnostic builds: full node loads)
  float pm = -INFINITY, u1 = -INFINITY, u2 = -INFINITY;
  int sv = 0, mv = 0, ui = kDogA;
#pragma unroll
  for (int w = 0; w < (kWJ + 3) / 4; ++w) nd.vis4[w] = 0u;
  // this lane's visited slots (one 128-byte line per node); the 26 prior logits in two batches of 13, all of a batch
  // in flight together (left to itself the scheduler serialised them slot by slot to save registers: 26 round trips;
  // padding slots are read too -- they exist in the node's 832 -- and dropped); then the statistics of the few
  // visited children
  const unsigned vm_ld = tree_ld(T.vmask(g, node) + sub);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float pk[kWHalf];
#pragma unroll
    for (int k = 0; k < kWHalf; ++k) pk[k] = tree_ld(T.prior() + T.ca(g, node, sub + kRowLanes * (kWHalf * h + k)));
    __builtin_amdgcn_sched_barrier(0);
    ST(ST_PASS);   // (diagnostic builds: node loads)
#pragma unroll
    for (int k = 0; k < kWHalf; ++k) {
      const int j = kWHalf * h + k, a = sub + kRowLanes * j;
      if (a < kDogA) {
        const float p = pk[k];
        nd.pr[a] = p;
        pm = fmaxf(pm, p);
        if (((vm_ld >> j) & 1u) == 0u) {   // unvisited; slots in ascending order: the first of equal priors keeps u1
          if (p > u1) {
            u2 = u1;
            u1 = p;
            ui = a;
          } else {
            u2 = fmaxf(u2, p);
          }
        }
      }
    }
  }
#pragma unroll 1
  for (unsigned m = vm_ld; m; m &= m - 1u) {
    const int j = __ffs(m) - 1, a = sub + kRowLanes * j;
    const size_t e = T.ca(g, node, a);
    const f32x4 c4 = tree_ld(T.stat() + e);
    const int vj = tree_ld(T.visits() + e);
    nd.cq[a] = c4[1] + c4[2] * c4[0];   // q = reward + discount * value (Tree.qvalues)
    const uint32_t vb = (uint32_t)vj << (8 * (j & 3));
#pragma unroll
    for (int w = 0; w < (kWJ + 3) / 4; ++w) nd.vis4[w] |= (j >> 2) == w ? vb : 0u;   // (static indices: registers)
    sv += vj;
    mv = max(mv, vj);
  }
  pm = row_max(pm);
  sv = row_isum(sv);
  mv = row_imax(mv);
  wtop2_row(u1, ui, u2);
  float es = ces[node];
  ST(ST_OTHER);   // (diagnostic builds)
  if (es < 0.f) {   // (row-uniform)
    st_count(12);   // (diagnostic builds: first walks)
    es = wsum([&](int j) { return wok(sub, j) ? exp_cr_w(nd.pr[sub + kRowLanes * j] - pm) : -0.0f; });
    if (sub == 0) ces[node] = es;
    // the kWTop largest priors in (value desc, index asc) order, one row argmax after another
    float pv = INFINITY;
    int pi = -1;
#pragma unroll 1
    for (int r = 0; r < kWTop; ++r) {
      float v = -INFINITY;
      int i = kDogA;
#pragma unroll
      for (int j = 0; j < kWJ; ++j) {
        const int a = sub + kRowLanes * j;
        if (a < kDogA) {
          const float p = nd.pr[a];
          if ((p < pv || (p == pv && a > pi)) && p > v) {
            v = p;
            i = a;
          }
        }
      }
      wargmax_row2(v, i);
      if (sub == r) {
        T.tp(g, node)[r] = v;
        T.ti(g, node)[r] = i;
      }
      pv = v;
      pi = i;
    }
    ST(ST_FIRST);   // (diagnostic builds: first-walk normaliser + top-prior list)
  }
  unsigned vm = 0;
#pragma unroll
  for (int j = 0; j < kWJ; ++j) vm |= (nd.vis(j) > 0 ? 1u : 0u) << j;
  nd.pm = pm;
  nd.sv = sv;
  nd.mv = mv;
  nd.es = es;
  nd.u1 = u1;
  nd.u2 = u2;
  nd.ui = ui;
  nd.vm = vm;
}

// lane l: the node's l-th visited child (a < 0: none) -- its index, visit count, prior and transformed completed Q
struct WEntry {
  int a, n, child;   // child index, visit count, the node it leads to
  float p, c;        // prior, transformed completed Q
  float r, d;        // reward, discount
  float e;           // exp(prior - the node's max prior), cached in the record (NaN: not computed yet)
};

// record l of a node's visited list into e (a = -1 when l >= vc) and its q = reward + discount * value
__device__ __forceinline__ float wrec_load(WEntry& e, const WTree& T, int g, int node, int l, int vc) {
  e.a = -1;
  e.n = 0;
  e.child = -1;
  e.p = e.c = e.r = e.d = e.e = 0.f;
  float q = 0.f;
  if (l < vc) {
    const AS1 f32x4* rp = T.vr(g, node) + 2 * l;
    const f32x4 r0 = tree_ld(rp), r1 = tree_ld(rp + 1);
    e.a = __float_as_int(r0[0]);
    e.n = __float_as_int(r0[1]);
    e.p = r0[2];
    e.r = r1[0];
    e.d = r1[1];
    e.child = __float_as_int(r1[2]);
    e.e = r1[3];
    q = r1[0] + r1[1] * r0[3];   // q = reward + discount * value (Tree.qvalues)
  }
  return q;
}

// Compact load of a node walked before (its normaliser es and top-prior list cached, its visited list not
// overflowed): only the visited children (lane l the list's l-th, one 16-byte load + the visit count) and the
// top-prior list -- everything the certified selection reads; their priors / q go to LDS at their slots for the
// mixed value's lane-order sums.  nd.vis is not filled.  False when the list has fewer than two unvisited children
// (u2 unknown): the caller loads the node in full.
__device__ __forceinline__ bool wnode_compact(WNode& nd, const WTree& T, int g, int node, int sub, float es, int vc,
                                              WEntry& en) {
#pragma clang fp contract(off)
  float tp = -INFINITY;
  int ti = kDogA;
  if (sub < kWTop) {
    tp = tree_ld(T.tp(g, node) + sub);
    ti = tree_ld(T.ti(g, node) + sub);
  }
  const float q = wrec_load(en, T, g, node, sub, vc);
  ST(ST_PASS);   // (diagnostic builds: node loads)
  if (en.a >= 0) nd.cq[en.a] = q;
  // this lane's visited slots: the list entries whose child sits in this lane
  unsigned vm = 0;
  for (int k = 0; k < vc; ++k) {
    const int a = __shfl(en.a, k, kRowLanes);
    if ((a & (kRowLanes - 1)) == sub) vm |= 1u << (a >> 5);
  }
  // the first two unvisited children of the top-prior list
  const unsigned vmt = __shfl(vm, ti & (kRowLanes - 1), kRowLanes);
  const bool unv = sub < kWTop && ((vmt >> (ti >> 5)) & 1u) == 0u;
  const unsigned long long bal = __ballot(unv);
  const unsigned bits = (unsigned)(bal >> (threadIdx.x & 32u)) & ((1u << kWTop) - 1u);
  if (__popc(bits) < 2) return false;
  const int k1 = __ffs(bits) - 1, k2 = __ffs(bits & (bits - 1u)) - 1;
  nd.pm = __shfl(tp, 0, kRowLanes);   // the list's first prior is the node's largest
  // the visited children's exp(prior - max prior), kept in their records from the first time a walk needs them (the
  // node's priors and maximum do not change until it is expanded again, which resets the cache through a full load):
  // the Q transform's prior probabilities and the certified selection's normaliser read them instead of recomputing
  // the correctly rounded exponentials at every level of every walk.  nd.pr holds them (not the priors) for
  // wnode_tail<true>.
  if (en.a >= 0) {
    if (en.e != en.e) {
      en.e = exp_cr_w(en.p - nd.pm);
      tree_st(reinterpret_cast<AS1 float*>(T.vr(g, node) + 2 * sub + 1) + 3, en.e);
    }
    nd.pr[en.a] = en.e;
  }
  nd.u1 = __shfl(tp, k1, kRowLanes);
  nd.ui = __shfl(ti, k1, kRowLanes);
  nd.u2 = __shfl(tp, k2, kRowLanes);
  nd.sv = row_isum(en.n);
  nd.mv = row_imax(en.n);
  nd.es = es;
  nd.vm = vm;
  return true;
}

// qtransform_completed_by_mix_value (value_scale, maxvisit_init, rescale, mixed value, eps 1e-8) over a loaded node:
// the visited children's transformed completed Q into cq (LDS) and the value every unvisited child shares (nd.K).
// The mixed value needs the prior probabilities of the VISITED children only: sum_probs and weighted_q are summed
// over this lane's visited slots (a bit mask, in slot order) -- the unvisited ones add exact zeros in the
// restatement's order (lane_tree_sum), which change no partial sum -- so their exponentials are not recomputed.
// exps (the compact load): nd.pr holds the visited children's exp(prior - max prior) instead of their priors.
__device__ __forceinline__ void wnode_tail(WNode& nd, int sub, float raw, const SearchArgs& sa, bool exps) {
#pragma clang fp contract(off)
  const float pm = nd.pm, es = nd.es;
  const unsigned vm = nd.vm;
  auto ppa = [&](int a) { return fmaxf(kTinyF, (exps ? nd.pr[a] : exp_cr_w(nd.pr[a] - pm)) / es); };
  float spl = 0.f;
  for (unsigned m = vm; m; m &= m - 1u) spl = spl + ppa(sub + kRowLanes * (__ffs(m) - 1));
  const float sp = row_sum(spl);
  float wql = 0.f;
  for (unsigned m = vm; m; m &= m - 1u) {
    const int a = sub + kRowLanes * (__ffs(m) - 1);
    wql = wql + ppa(a) * nd.cq[a] / sp;
  }
  const float wq = row_sum(wql);
  const int sv = nd.sv;
  const float mixed = (raw + (float)sv * wq) / (float)(sv + 1);
  // completed Q: the visited children's q, `mixed` for the rest (there are unvisited children: S <= 100 < 806), so
  // its minimum / maximum are those of the visited q and `mixed`, and every unvisited child transforms to the same K
  float lo = mixed, hi = mixed;
  for (unsigned m = vm; m; m &= m - 1u) {
    const float c = nd.cq[sub + kRowLanes * (__ffs(m) - 1)];
    lo = fminf(lo, c);
    hi = fmaxf(hi, c);
  }
  lo = row_min(lo);
  hi = row_max(hi);
  const float den = fmaxf(hi - lo, 1e-8f);
  const float scale = (sa.maxvisit_init + (float)nd.mv) * sa.value_scale;
  for (unsigned m = vm; m; m &= m - 1u) {
    const int a = sub + kRowLanes * (__ffs(m) - 1);
    nd.cq[a] = scale * ((nd.cq[a] - lo) / den);
  }
  nd.K = scale * ((mixed - lo) / den);
  ST(ST_OTHER);   // (diagnostic builds: the completed-Q transform)
}

// the visited-list entries of a fully loaded node (priors / transformed Q from LDS); vc < 0 (overflowed list): none
__device__ __forceinline__ void wentries(const WNode& nd, const WTree& T, int g, int node, int sub, int vc,
                                         WEntry& en) {
  wrec_load(en, T, g, node, sub, vc);
  if (en.a >= 0) {
    en.p = nd.pr[en.a];
    en.c = nd.cq[en.a];
    en.e = exp_cr_w(en.p - nd.pm);
    // (the record's prior and cached exponential refreshed: the node's priors change when it is expanded again at
    // the depth limit)
    tree_st(reinterpret_cast<AS1 float*>(T.vr(g, node) + 2 * sub) + 2, en.p);
    tree_st(reinterpret_cast<AS1 float*>(T.vr(g, node) + 2 * sub + 1) + 3, en.e);
  }
}

// the unvisited children's transformed completed Q (K) into cq: the root's selection, the final weights and the
// interior selection's exact path read all 806
__device__ __forceinline__ void wfill_unvisited(const WNode& nd, int sub) {
#pragma unroll
  for (int j = 0; j < kWJ; ++j)
    if (wok(sub, j) && ((nd.vm >> j) & 1u) == 0u) nd.cq[sub + kRowLanes * j] = nd.K;
}

// gumbel_muzero_interior_action_selection's argmax without the 806 exponentials, when it can be certified:
// score(a) = exp(z_a - zm) / zs - N_a / (1 + sum N) with z = prior + completed Q.  Every unvisited child has the same
// completed Q (K) and N = 0, so its score is non-decreasing in its prior: the best unvisited child is the one with
// the largest prior (u1), and the candidates are it and the visited children.  Their exponentials are computed
// exactly as the exact path does; only zs is bounded instead of summed: the unvisited part is exp(K + pm - zm) x
// (es - the visited children's exp(prior - pm)), within a relative error bound of the restatement's float sum
// (argument roundings, exp, the lane-order sums).  The pick is returned when the best candidate's lower bound
// clears every other candidate's upper bound (and, when it is u1's child, when no other unvisited child can tie
// it: its exponential is more than a few ulps above the second prior's) -- then the exact path's argmax is the
// same index; otherwise -1 (the exact path runs).
__device__ __forceinline__ int wselect_certified(const WNode& nd, const WEntry& en, int sub) {
#pragma clang fp contract(off)
  const float K = nd.K, zU = nd.u1 + K;
  const bool has = en.a >= 0;
  const float z = has ? en.p + en.c : -INFINITY;
  const float zm = fmaxf(row_max(z), zU);   // fl(p + K) is monotone in p: zU is the unvisited maximum
  const float ez = has ? exp_cr_w(z - zm) : 0.f;
  const float sez = row_sum(ez);
  const float sep = row_sum(has ? en.e : 0.f);   // en.e = exp_cr_w(en.p - nd.pm) (wnode_compact / wentries)
  const double f = exp((double)K + (double)nd.pm - (double)zm);
  const double zsa = (double)sez + f * fmax((double)nd.es - (double)sep, 0.0);
  // per-element relative error of the argument roundings <= 2^-24 (c0 + 3 d) e^-d summed (d e^-d <= 1/e over 806
  // children), exp and the lane-order sums <= 2^-18; es's own sum error scaled by f; all doubled
  const double c0 = 4.0 * (fabs((double)zm) + fabs((double)K) + fabs((double)nd.pm) + 1.0);
  const double err = zsa * (0x1p-23 * (c0 + 900.0) + 0x1p-17) + f * (double)nd.es * 0x1p-17;
  if (!(zsa - err > 0.0) || !(err < 0.01 * zsa)) return -1;
  const float zlo = (float)(zsa - err) * (1.f - 0x1p-22f), zhi = (float)(zsa + err) * (1.f + 0x1p-22f);
  const float n = has ? (float)en.n / (float)(1 + nd.sv) : 0.f;
  const float q_hi = ez / zlo, slack = 0x1p-20f * (q_hi + n);
  // the best visited candidate of the row by lower bound
  float blo = has ? (ez / zhi - n) - slack : -INFINITY;
  int bi = has ? en.a : kDogA;
  wargmax_row2(blo, bi);
  const float ezU = exp_cr_w(zU - zm);
  const float loU = ezU / zhi - 0x1p-20f * (ezU / zlo), hiU = ezU / zlo + 0x1p-20f * (ezU / zlo);
  const bool pick_u = loU > blo || bi >= kDogA;
  if (pick_u) {
    bi = nd.ui;
    blo = loU;
    if (!(loU > 0x1p-100f)) return -1;   // (normal range: the ulp argument below holds)
    // no other unvisited child may reach u1's score: its exponential more than 4 ulps above the runner-up's
    if (nd.u2 != -INFINITY && !(ezU > exp_cr_w((nd.u2 + K) - zm) * (1.f + 0x1p-21f))) return -1;
  }
  // upper bounds of every other candidate
  const float hub = fmaxf(row_max(has && en.a != bi ? (q_hi - n) + slack : -INFINITY), pick_u ? -INFINITY : hiU);
  return blo > hub ? bi : -1;
}

// gumbel_muzero_interior_action_selection by certification (wselect_certified) over the node's visited-list entries,
// or -1: the exact path (exact_select, an overflowed list, or no certificate)
__device__ __forceinline__ int wselect_interior(const WNode& nd, WEntry& en, const WTree& T, int g, int node, int sub,
                                                int vc, bool compact, bool exact_select) {
  st_count(9);   // (diagnostic builds: interior selections)
  if (exact_select || vc < 0) return -1;
  if (compact) {
    en.c = en.a >= 0 ? nd.cq[en.a] : 0.f;
  } else {
    wentries(nd, T, g, node, sub, vc, en);
  }
  return wselect_certified(nd, en, sub);
}

// SPARSE: one game per wave (the even rows of the 16-row tile; the odd rows are padding the networks carry along), 8
// games per workgroup.  A wave's two rows walk their trees one after the other wherever their paths differ (depth,
// exact-path fallbacks), so with one game per wave the walk and the barrier waits behind it shrink; the networks cost
// the same per tile.  Chosen when the grid still fits the chip (n <= 2048: <= 256 workgroups of 8).
template <bool SPARSE>
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
  __shared__ float p_prior[kRows][kWMaxDepth];
  __shared__ uint32_t s_legal[kRows][kWWords];
  __shared__ float s_ces[kRows][kWMaxNodes];   // per-node softmax normalisers of the priors (wnode_full)
  __shared__ signed char s_vcnt[kRows][kWMaxNodes];   // per-node visited-list lengths (-1: overflowed)
  __shared__ int s_act[kRows], s_parent[kRows], s_next[kRows], s_depth[kRows];

  const int kGames = SPARSE ? sa.games_per_wg : kRows;   // games per workgroup
  if ((int)blockIdx.x * kGames >= n) return;
  auto game_of = [kGames](int r) { return (int)blockIdx.x * kGames + (SPARSE ? (r >> 1) : r); };
  const Arena ar = Arena::carve(smem);
  const int row = trow(), sub = tsub();
  const int g = game_of(row);
  const bool valid = (!SPARSE || ((row & 1) == 0 && (row >> 1) < kGames)) && g < n;
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
    float pr[kWJ], pm = -INFINITY;
#pragma unroll
    for (int j = 0; j < kWJ; ++j) {
      const int a = sub + kRowLanes * j;
      pr[j] = kWFMin;
      if (a < kDogA) {
        const bool inv = ((legal[(size_t)g * kWWords + j] >> sub) & 1u) == 0u;
        pr[j] = inv ? kWFMin : root_logits[(size_t)g * kDogA + a] - lm;
        pm = fmaxf(pm, pr[j]);
        tree_st(T.prior() + T.ca(g, 0, a), pr[j]);
      }
    }
    tree_st(T.vmask(g, 0) + sub, 0u);   // no child visited
    pm = row_max(pm);   // score_considered's logits.max over the root's (masked) priors, fixed for the search
#pragma unroll
    for (int j = 0; j < kWJ; ++j) {
      const int a = sub + kRowLanes * j;
      if (a < kDogA) {
        const float gm =
            gumbel_in ? gumbel_in[(size_t)g * kDogA + a] : sa.gumbel_scale * gumbel_noise(sa.seed, gid, gturn, a);
        gpw(T.gum)[(size_t)g * kWPad + a] = gm + (pr[j] - pm);
      }
    }
    for (int i = sub; i < kWMaxNodes; i += kRowLanes) {
      s_ces[row][i] = -1.f;
      s_vcnt[row][i] = 0;
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

  // (the noise is drawn once above: hashing the 806 draws inside the simulation loop made the compiler hoist their
  // per-slot constants out of it, 52 VGPRs live across the networks)
  auto legal_of = [&](int j) -> bool { return (s_legal[row][j] >> sub) & 1u; };

  Pf pf;
  pf_issue<NT256>(pf, &kernarg0<muz_dog_net_w>()->dyn.d3, LAT, LAT);
  st_begin();
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
        WEntry en;
        en.a = -1;
        bool cert = false;
        const int vc = s_vcnt[row][node];
        // interior nodes walked before: the compact load (the visited children and the top-prior list); the exact path
        // (no certificate) reloads the node in full on a second pass
        bool compact = depth > 0 && !sa.exact_select && vc >= 0 && s_ces[row][node] >= 0.f;
        if (compact) compact = wnode_compact(nd, T, g, node, sub, s_ces[row][node], vc, en);
        bi = -1;
#pragma unroll 1
        for (int pass = 0; pass < 2 && bi < 0; ++pass) {
          if (!compact) wnode_full(nd, T, g, node, sub, s_ces[row]);
          wnode_tail(nd, sub, s_raw[row][node], sa, compact);
          if (depth == 0) {
            // gumbel_muzero_root_action_selection: score_considered + masked_argmax
            const int cv = wconsidered_visit(ncons, sa.S, nd.sv);
            wfill_unvisited(nd, sub);
            bi = wroot_argmax(T, g, sub, nd.cq, [&](int j) { return nd.vis(j); }, cv, legal_of);
          } else if (pass == 0 && (bi = wselect_interior(nd, en, T, g, node, sub, vc, compact, sa.exact_select)) >= 0) {
            cert = true;
          } else if (compact) {
            compact = false;   // the exact path reads all 806 children
          } else {
            st_count(10);   // (diagnostic builds: exact-path fallbacks)
            // gumbel_muzero_interior_action_selection: softmax(prior + cq) - N / (1 + sum N), the exact path
            // (z = prior + cq, then its exponential, replace the priors in LDS: one exp per child)
            wfill_unvisited(nd, sub);
            float zm = -INFINITY;
#pragma unroll
            for (int j = 0; j < kWJ; ++j) {
              const int a = sub + kRowLanes * j;
              if (a < kDogA) {
                const float z = nd.pr[a] + nd.cq[a];
                nd.pr[a] = z;
                zm = fmaxf(zm, z);
              }
            }
            zm = row_max(zm);
            const float zs = wsum([&](int j) {
              const int a = sub + kRowLanes * j;
              if (a >= kDogA) return -0.0f;
              const float ez = exp_cr_w(nd.pr[a] - zm);
              nd.pr[a] = ez;
              return ez;
            });
            const float inv_n = (float)(1 + nd.sv);
            bi = wargmax([&](int j) {
              const int a = sub + kRowLanes * j;
              return a < kDogA ? (nd.pr[a] / zs - (float)nd.vis(j) / inv_n) : -INFINITY;
            }, sub);
          }
        }
        ST(ST_SEL);   // (diagnostic builds: scores + argmax)
        // the chosen child's place in the node's visited list (-1: not on it; -2: the list was not loaded)
        int lpos = -2;
        if (depth > 0 && !sa.exact_select && vc >= 0) {
          const unsigned bits = (unsigned)(__ballot(en.a == bi) >> (threadIdx.x & 32u));
          lpos = bits ? __ffs(bits) - 1 : -1;
        }
        int child, cvis;
        float crw, cdc, cpr;
        if (cert && lpos >= 0) {   // a visited child: its record (the tree holds the same values)
          child = __shfl(en.child, lpos, kRowLanes);
          cvis = __shfl(en.n, lpos, kRowLanes);
          crw = __shfl(en.r, lpos, kRowLanes);
          cdc = __shfl(en.d, lpos, kRowLanes);
          cpr = __shfl(en.p, lpos, kRowLanes);
        } else if (cert) {         // the unvisited child of the largest prior: not expanded, zero reward / discount
          child = -1;
          cvis = 0;
          crw = cdc = 0.f;
          cpr = nd.u1;
        } else {
          const size_t eb = T.ca(g, node, bi);
          cpr = tree_ld(T.prior() + eb);
          child = -1;
          cvis = 0;
          crw = cdc = 0.f;
          if ((tree_ld(T.vmask(g, node) + (bi & (kRowLanes - 1))) >> (bi >> 5)) & 1u) {   // visited: its statistics
            const f32x4 c4 = tree_ld(T.stat() + eb);
            child = __float_as_int(c4[3]);
            cvis = tree_ld(T.visits() + eb);
            crw = c4[1];
            cdc = c4[2];
          }
        }
        if (sub == 0) {
          p_node[row][depth] = node;
          p_act[row][depth] = bi;
          p_rew[row][depth] = crw;
          p_disc[row][depth] = cdc;
          p_prior[row][depth] = cpr;
          p_cvis[row][depth] = cvis | ((lpos + 2) << 16);
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
    ST(ST_SEL);
    SYNC();
    // ---------------- expand: recurrent_fn on the 16 parents; the 806 prior logits go to the new nodes' children
    const int nx = s_next[row];
    if (valid && nx == sim + 1) tree_st(T.vmask(g, nx) + sub, 0u);   // a new node: no child visited (priors below)
    ST(ST_TREE);
    dyn16<NT256, true, false>(wl->dyn, kDogA, din, dact, ar, pf, &wl->pred.rb[0].d0, LAT, LAT, &wl->pred.ln0,
                              valid ? T.e(g, nx) : nullptr);
    pred16<NT256, true, false, false, NT256, true>(wl->pred, kDogA, ar.T, ar, pf, nullptr, 0, 0);
    // (the hand-out re-reads the new node from LDS: with `nx` itself the compiler precomputed the 806 store
    // addresses before the networks and spilled them)
    dog_logits16<NT256>(wl, ar, pf, [&](int r, int col, float v) {
      if (valid) tree_st(T.prior() + T.ca(game_of(r), s_next[r], col), v);
    }, &wl->dyn.d3, LAT, LAT);
    if (valid) {
      const int nx = s_next[row];
      const bool fresh = nx == sim + 1;
      const int par = s_parent[row], pa = s_act[row];
      const float v = ar.v0[row], rw = ar.v1[row], dc = ar.v2[row];
      if (sub == 0) {
        // the edge's statistics (its value and visit count follow in the backup) and its bit in the visited mask
        const size_t eb = T.ca(g, par, pa);
        tree_st(T.fld(eb, 3), __int_as_float(nx));
        tree_st(T.fld(eb, 1), rw);
        tree_st(T.fld(eb, 2), dc);
        AS1 uint32_t* mw = T.vmask(g, par) + (pa & (kRowLanes - 1));
        tree_st(mw, tree_ld(mw) | (1u << (pa >> 5)));
        s_raw[row][nx] = v;
        s_val[row][nx] = v;
        s_ces[row][nx] = -1.f;   // new priors: the node's normaliser is recomputed at its next walk
        if (fresh) s_vcnt[row][nx] = 0;
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
        int parent = 0, pact = 0, cvis = 0, cnt = 0, lpos = -2;
        float r = 0.f, dsc = 0.f, pval = 0.f;
        if (on) {
          parent = p_node[row][l];
          pact = p_act[row][l];
          const int pc = p_cvis[row][l];
          cvis = pc & 0xFFFF;
          lpos = (pc >> 16) - 2;
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
          tree_st(T.fld(ei, 0), child_v);
          tree_st(T.visits() + ei, cvis + 1);
          s_val[row][parent] = pv;
          s_visits[row][parent] = cnt + 1;
          // the edge's record in the parent's visited list: appended at its first visit (a path holds a node once),
          // rewritten at later ones (place known from the selection)
          int k = lpos;
          if (cvis == 0) {
            k = s_vcnt[row][parent];
            if (k >= 0) s_vcnt[row][parent] = (signed char)(k < kWList ? k + 1 : -1);
          }
          if (k >= 0 && k < kWList) {
            const int cnode = (l == d - 1) ? nx : p_node[row][l + 1];
            AS1 f32x4* rp = T.vr(g, parent) + 2 * k;
            tree_st(rp, f32x4{__int_as_float(pact), __int_as_float(cvis + 1), p_prior[row][l], child_v});
            if (cvis == 0) {   // a new record: its cached exponential not computed yet
              tree_st(rp + 1, f32x4{r, dsc, __int_as_float(cnode), __builtin_nanf("")});
            } else {           // (keep the record's cached exponential)
              AS1 float* r1 = reinterpret_cast<AS1 float*>(rp + 1);
              tree_st(r1, r);
              tree_st(r1 + 1, dsc);
              tree_st(r1 + 2, __int_as_float(cnode));
            }
          }
        }
        carry = __shfl(leaf, 0, kRowLanes);
        carry_v = __shfl(pv, 0, kRowLanes);
      }
    }
    ST(ST_TREE);
    SYNC();
  }
  st_end();

  // ---------------- final action + action_weights (policies.py gumbel_muzero_policy tail)
  if (valid) {
    WNode nd;
    nd.pr = smem + row * kDogA;
    nd.cq = smem + (kRows + row) * kDogA;
    wnode_full(nd, T, g, 0, sub, s_ces[row]);
    wnode_tail(nd, sub, s_raw[row][0], sa, false);
    wfill_unvisited(nd, sub);
    const int bi = wroot_argmax(T, g, sub, nd.cq, [&](int j) { return nd.vis(j); }, nd.mv, legal_of);   // considered_visit = max(visits)
    // action_weights = softmax(_mask_invalid_actions(prior + completed_q))
    float zm = -INFINITY;
#pragma unroll
    for (int j = 0; j < kWJ; ++j)
      if (wok(sub, j)) zm = fmaxf(zm, nd.pr[sub + kRowLanes * j] + nd.cq[sub + kRowLanes * j]);
    zm = row_max(zm);
    float mm = -INFINITY;
#pragma unroll
    for (int j = 0; j < kWJ; ++j) {
      const int a = sub + kRowLanes * j;
      if (a < kDogA) {
        const float zz = !legal_of(j) ? kWFMin : (nd.pr[a] + nd.cq[a]) - zm;
        nd.pr[a] = zz;
        mm = fmaxf(mm, zz);
      }
    }
    mm = row_max(mm);
    const float zs = wsum([&](int j) {
      const int a = sub + kRowLanes * j;
      if (a >= kDogA) return -0.0f;
      const float ez = exp_cr_w(nd.pr[a] - mm);
      nd.pr[a] = ez;
      return ez;
    });
#pragma unroll
    for (int j = 0; j < kWJ; ++j) {
      const int a = sub + kRowLanes * j;
      if (a < kDogA) out_weights[(size_t)g * kDogA + a] = nd.pr[a] / zs;
    }
    if (sub == 0) {
      out_action[g] = ncons > 0 ? bi : -1;   // no legal action: -1, the self-play loop's no_step
      out_value[g] = s_val[row][0];
    }
  }
}

int64_t dog_search_workspace_bytes(int n, int S) {
  const int N = S + 1;
  return (int64_t)wide_children_bytes(n, N) * 6 + (int64_t)n * N * kRowLanes * 4 + (int64_t)n * N * LAT * 4 +
         (int64_t)n * kWPad * 4 +
         (int64_t)n * N * (int64_t)(kWRecBytes + 2 * kWTopBytes);
}

int launch_dog_search(const muz_dog_net_w& w, const SearchArgs& sa, const float* root_logits, const float* root_value,
                      const float* root_emb, const uint32_t* legal, const float* gumbel, int n, void* workspace,
                      int32_t* action, float* weights, float* value, bool sparse, hipStream_t s) {
  WTree T = carve_wide(workspace, n, sa.S + 1);
  if (sparse)
    k_dog_search<true><<<(n + sa.games_per_wg - 1) / sa.games_per_wg, kThreads, 0, s>>>(w, sa, root_logits, root_value, root_emb,
                                                                             legal, gumbel, n, T, action, weights, value);
  else
    k_dog_search<false><<<(n + kRows - 1) / kRows, kThreads, 0, s>>>(w, sa, root_logits, root_value, root_emb, legal,
                                                                     gumbel, n, T, action, weights, value);
  return muz_last_launch_error();
}

int check_dog_net(const muz_dog_net_w* w);

}  // namespace muz

using namespace muz;

// one game per wave while the grid fits the chip's 256 CUs; MUZ_DOG_TILE_ROWS=8 / 16 forces either form
static bool dog_search_sparse(int n) {
  if (const char* e = getenv("MUZ_DOG_TILE_ROWS")) return atoi(e) == 8;
  return n <= 2048;
}

// games per workgroup of the one-game-per-wave form: fewer than 8 while the grid still fits the chip's 256 CUs
// (a simulation waits for the slowest of the workgroup's walks): 6 at the reference's 1500 games, 250 workgroups
// -- 0.8 % faster than 8 (profiles/r5zb_dog_gpw_ab.log; 7: 0.2 % slower); MUZ_DOG_GPW overrides
static int dog_search_gpw(int n) {
  if (const char* e = getenv("MUZ_DOG_GPW")) return std::min(8, std::max(1, atoi(e)));
  return std::min(8, std::max(6, (n + 255) / 256));
}

extern "C" {

int64_t muz_dog_search_workspace_bytes(int32_t n, const muz_search_cfg* cfg) {
  if (!cfg || n < 0) return -1;
  return dog_search_workspace_bytes(n, cfg->num_simulations);
}

int32_t muz_dog_search_games_per_workgroup(int32_t n) {
  if (n < 0) return -1;
  return dog_search_sparse(n) ? dog_search_gpw(n) : 16;
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
  {   // MUZ_DOG_EXACT_SELECT=1: every interior selection on the exact path (tests of that path)
    const char* e = getenv("MUZ_DOG_EXACT_SELECT");
    sa.exact_select = e && e[0] == '1';
  }
  const bool sparse = dog_search_sparse(n);
  sa.games_per_wg = dog_search_gpw(n);
  return launch_dog_search(*w, sa, root_logits, root_value, root_embedding, legal, gumbel, n, workspace, action,
                           action_weights, root_value_out, sparse, (hipStream_t)stream);
}

#ifdef MUZ_STAMPS2
// the per-category cycle totals of k_dog_search's diagnostic build (this translation unit's g_st2)
int muz_diag_dog_stamps2(unsigned long long* host_out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_st2), sizeof(unsigned long long) * ST_N);
  if (e != hipSuccess) return (int)e;
  if (reset) {
    unsigned long long z[ST_N] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_st2), z, sizeof(z));
  }
  return (int)e;
}
#endif

}  // extern "C"
