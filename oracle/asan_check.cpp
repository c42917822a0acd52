// Host-side AddressSanitizer / UBSan run of the C++ code that executes on the host (VERDICT r5 "missing" 5; SURVEY
// §5 race detection / sanitizers): the CPU restatements that bench.py's cpu_baseline legs run inside the bench process
// (cpu_selfplay.cpp, cpu_classic.cpp, cpu_dog.cpp, cpu_search.hpp) and the TicTacToe engine of libmuz.so
// (csrc/tictactoe.cpp, plain host C++).  TEST INFRASTRUCTURE ONLY: built by `make -C oracle asan` into
// oracle/_asan/asan_check (-fsanitize=address,undefined, no GPU code), driven by tests/test_asan_host.py, which writes
// the networks' parameters into a file this driver reads (name, element count, floats per tensor).
//   usage: asan_check <det params> <classic params> <dog params>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/muz.h"

extern "C" {
void* muzcpu_net_create(const char** names, const float** data, const int64_t* sizes, int count, int obs_channels);
void muzcpu_net_destroy(void* n);
int muzcpu_selfplay(void* netp, int P, int rules, int n, int S, int D, int T, float temp, uint64_t seed, const void* tr);
int64_t muzcpu_env_bench(int P, int rules, int lanes, uint64_t seed, int threads, double seconds, double* elapsed_out);
void* muzcpu_classic_net_create(const char** names, const float** data, const int64_t* sizes, int count,
                                int obs_channels);
void muzcpu_classic_net_destroy(void* n);
int muzcpu_classic_selfplay(void* netp, int P, int rules, int n, int S, int D, int T, float temp, uint64_t seed,
                            float dirichlet_fraction, const void* tr);
int64_t muzcpu_dog_play(int P, int rules, int n, int turns, uint64_t seed, int32_t* actions);
int64_t muzcpu_dog_mz_play(void* netp, int rules, int n, int turns, int S, int D, float temp, uint64_t seed,
                           int32_t* actions);
}

struct Params {
  std::vector<std::string> names;
  std::vector<std::vector<float>> data;
  std::vector<const char*> cn;
  std::vector<const float*> cp;
  std::vector<int64_t> sizes;
};

static bool load(const char* path, Params& p) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  int32_t count = 0;
  if (fread(&count, 4, 1, f) != 1) return false;
  for (int i = 0; i < count; ++i) {
    int32_t len = 0;
    int64_t n = 0;
    if (fread(&len, 4, 1, f) != 1) return false;
    std::string name(len, '\0');
    if (fread(&name[0], 1, len, f) != (size_t)len || fread(&n, 8, 1, f) != 1) return false;
    std::vector<float> v(n);
    if (fread(v.data(), 4, n, f) != (size_t)n) return false;
    p.names.push_back(name);
    p.data.push_back(std::move(v));
  }
  fclose(f);
  for (size_t i = 0; i < p.names.size(); ++i) {
    p.cn.push_back(p.names[i].c_str());
    p.cp.push_back(p.data[i].data());
    p.sizes.push_back((int64_t)p.data[i].size());
  }
  return true;
}

#define CHECK(cond, what)                        \
  do {                                           \
    if (!(cond)) {                               \
      fprintf(stderr, "asan_check: %s\n", what); \
      return 1;                                  \
    }                                            \
  } while (0)

int main(int argc, char** argv) {
  CHECK(argc == 4, "usage: asan_check <det params> <classic params> <dog params>");
  Params det, cls, dog;
  CHECK(load(argv[1], det) && load(argv[2], cls) && load(argv[3], dog), "cannot read a parameter file");
  // rule bits (oracle/cpu_selfplay.py _FLAGS): teams 1, free pin 2, circular 4, start blocking 8, jump 16,
  // friendly fire 32, start on 1 64, bonus 6 128, traverse 256; classic dice rethrow 512
  const int det_rules[3] = {1 | 2 | 16, 4 | 8 | 32 | 256, 2 | 8 | 16 | 64 | 128};
  double el = 0.0;
  for (int r : det_rules) CHECK(muzcpu_env_bench(4, r, 8, 7, 2, 0.05, &el) > 0, "det env bench");
  CHECK(muzcpu_env_bench(2, det_rules[0], 8, 8, 1, 0.05, &el) > 0, "det env bench 2p");
  void* dn = muzcpu_net_create(det.cn.data(), det.cp.data(), det.sizes.data(), (int)det.names.size(), 34);
  CHECK(muzcpu_selfplay(dn, 4, det_rules[0], 4, 8, 6, 40, 1.0f, 11, nullptr) > 0, "det self-play");
  muzcpu_net_destroy(dn);
  void* cnet = muzcpu_classic_net_create(cls.cn.data(), cls.cp.data(), cls.sizes.data(), (int)cls.names.size(), 11);
  CHECK(muzcpu_classic_selfplay(cnet, 4, det_rules[0] | 64 | 128 | 512, 4, 8, 6, 60, 1.0f, 12, 0.25f, nullptr) > 0,
        "classic self-play");
  muzcpu_classic_net_destroy(cnet);
  std::vector<int32_t> acts(6 * 300);
  const int dog_rules = 1 | 4 | 8 | 32 | 256;
  CHECK(muzcpu_dog_play(4, dog_rules, 6, 300, 13, acts.data()) > 0, "DOG random play");
  void* gnet = muzcpu_net_create(dog.cn.data(), dog.cp.data(), dog.sizes.data(), (int)dog.names.size(), 34);
  std::vector<int32_t> macts(2 * 4);
  CHECK(muzcpu_dog_mz_play(gnet, dog_rules, 2, 4, 6, 4, 1.0f, 14, macts.data()) > 0, "DOG MuZero play");
  muzcpu_net_destroy(gnet);
  // TicTacToe (csrc/tictactoe.cpp): env, rollouts, a MuZero-style MCTS match
  muz_ttt_state s;
  CHECK(muz_ttt_reset(&s) == MUZ_OK, "ttt reset");
  int8_t rw = 0;
  uint8_t dn8 = 0;
  CHECK(muz_ttt_step(&s, 4, &rw, &dn8) == MUZ_OK, "ttt step");
  double v = 0.0;
  CHECK(muz_ttt_rollout(&s, 5, 0, &v) == MUZ_OK, "ttt rollout");
  muz_ttt_policy_out po;
  CHECK(muz_ttt_muzero_policy(&s, 25, 9, 1.0, 6, 1, &po) == MUZ_OK, "ttt muzero policy");
  printf("asan_check: all host paths ran clean\n");
  return 0;
}
