// Host-side self-test of the native runtime, built with sanitizers by
// tests/test_native_sanitizers.py (the reference has no race detection or
// sanitizers at all):
//   ASan + UBSan : randomized BlockManager workload (prefix sharing, cache hits,
//                  eviction, rollback, double free) against a shadow model, and
//                  compile_token_fsm against a naive per-token DFA walk;
//   TSan         : the FSM compiler run from several threads at once (the
//                  engine releases the GIL around it), BlockManager behind a mutex.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../runtime.h"

using namespace bcg;

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

static void block_manager_stress(unsigned seed) {
  std::mt19937 rng(seed);
  const int NB = 64, BS = 4;
  BlockManager bm(NB, BS);
  std::map<int, std::vector<int32_t>> content;  // block -> the tokens a committed prompt wrote there
  struct Live {
    std::vector<int> blocks;
    std::vector<int32_t> prompt;
  };
  std::vector<Live> live;
  std::vector<std::vector<int32_t>> agents(6);  // per-agent system prompts (shared prefixes)
  for (auto& a : agents) {
    a.resize(4 + rng() % 12);
    for (auto& t : a) t = static_cast<int32_t>(rng() % 50);
  }
  for (int step = 0; step < 4000; ++step) {
    if (live.empty() || rng() % 3) {
      std::vector<int32_t> p = agents[rng() % agents.size()];
      const int extra = static_cast<int>(rng() % 10);
      for (int i = 0; i < extra; ++i) p.push_back(static_cast<int32_t>(rng() % 50));
      Allocation a = bm.allocate(p, static_cast<int>(rng() % 6), true);
      if (!a.ok) {
        CHECK(a.blocks.empty());
        continue;
      }
      CHECK(a.num_cached_tokens % BS == 0 && a.num_cached_tokens < static_cast<int>(p.size()));
      for (int i = 0; i < a.num_cached_tokens / BS; ++i) {  // a hit must hold exactly this prompt block
        auto it = content.find(a.blocks[i]);
        CHECK(it != content.end());
        CHECK(std::equal(it->second.begin(), it->second.end(), p.begin() + i * BS));
      }
      bm.commit_prompt(a.blocks, p);
      for (int i = a.num_cached_tokens / BS; i < static_cast<int>(p.size()) / BS; ++i)
        content[a.blocks[i]] = std::vector<int32_t>(p.begin() + i * BS, p.begin() + (i + 1) * BS);
      for (int i = static_cast<int>(p.size()) / BS; i < static_cast<int>(a.blocks.size()); ++i)
        content.erase(a.blocks[i]);  // generated-token blocks are never cached
      live.push_back({a.blocks, p});
    } else {
      const size_t k = rng() % live.size();
      bm.free(live[k].blocks);
      live.erase(live.begin() + static_cast<long>(k));
    }
    CHECK(bm.num_free_blocks() >= 0 && bm.num_free_blocks() <= NB);
  }
  for (auto& l : live) bm.free(l.blocks);
  CHECK(bm.num_free_blocks() == NB);
  bool threw = false;
  Allocation a = bm.allocate({1, 2, 3, 4, 5}, 1, false);
  bm.free(a.blocks);
  try {
    bm.free(a.blocks);
  } catch (const std::logic_error&) {
    threw = true;
  }
  CHECK(threw);  // double free is detected, not silently corrupting the pool
  bm.reset_cache();
  CHECK(bm.num_free_blocks() == NB && bm.cached_blocks() == 0);
}

static void random_dfa(std::mt19937& rng, int S, std::vector<int32_t>& trans, std::vector<uint8_t>& accept) {
  trans.assign(static_cast<size_t>(S) * 256, -1);
  accept.assign(S, 0);
  for (int s = 0; s < S; ++s) {
    for (int c = 'a'; c <= 'h'; ++c)
      if (rng() % 3) trans[s * 256 + c] = static_cast<int32_t>(rng() % S);
    accept[s] = rng() % 4 == 0;
  }
}

static std::vector<std::string> random_tokens(std::mt19937& rng, int n) {
  std::vector<std::string> toks(n);
  for (int i = 0; i < n; ++i) {
    const int len = static_cast<int>(rng() % 5);  // includes empty (special) tokens
    for (int k = 0; k < len; ++k) toks[i].push_back(static_cast<char>('a' + rng() % 9));
  }
  return toks;
}

static void fsm_vs_naive(unsigned seed) {
  std::mt19937 rng(seed);
  for (int rep = 0; rep < 20; ++rep) {
    const int S = 2 + static_cast<int>(rng() % 30), V = 50 + static_cast<int>(rng() % 200);
    std::vector<int32_t> trans;
    std::vector<uint8_t> accept;
    random_dfa(rng, S, trans, accept);
    auto toks = random_tokens(rng, V);
    const int rows = V - static_cast<int>(rng() % 5);
    TokenFsmTables t = compile_token_fsm(trans.data(), accept.data(), S, toks, rows);
    for (int s = 0; s < S; ++s)
      for (int id = 0; id < rows; ++id) {
        int cur = toks[id].empty() ? -1 : s;
        for (char ch : toks[id]) cur = cur < 0 ? -1 : trans[cur * 256 + static_cast<uint8_t>(ch)];
        CHECK(t.next[static_cast<size_t>(s) * rows + id] == cur);
      }
    for (int s = 0; s < S; ++s) CHECK((t.dist[s] == 0) == (accept[s] != 0));
  }
}

static void concurrent(unsigned seed) {
  std::mutex mu;
  BlockManager bm(128, 8);
  std::vector<std::thread> th;
  for (int w = 0; w < 4; ++w)
    th.emplace_back([&, w] {
      std::mt19937 rng(seed + w);
      std::vector<int32_t> trans;
      std::vector<uint8_t> accept;
      random_dfa(rng, 16, trans, accept);
      auto toks = random_tokens(rng, 300);
      for (int rep = 0; rep < 3; ++rep) {
        TokenFsmTables t = compile_token_fsm(trans.data(), accept.data(), 16, toks, 300);
        CHECK(static_cast<int>(t.next.size()) == 16 * 300);
        std::vector<int32_t> p(20, w);
        std::lock_guard<std::mutex> lock(mu);  // the engine serialises BlockManager calls
        Allocation a = bm.allocate(p, 4, true);
        if (a.ok) {
          bm.commit_prompt(a.blocks, p);
          bm.free(a.blocks);
        }
      }
    });
  for (auto& t : th) t.join();
  CHECK(bm.num_free_blocks() == 128);
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "all";
  if (mode == "all" || mode == "asan") {
    for (unsigned s = 1; s <= 5; ++s) block_manager_stress(s);
    fsm_vs_naive(7);
  }
  if (mode == "all" || mode == "tsan") concurrent(11);
  std::printf("OK %s\n", mode.c_str());
  return 0;
}
