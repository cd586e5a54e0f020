// Token-level FSM compiler for guided JSON decoding.
//
// Input : a byte-level DFA (trans[S][256], accept[S]) compiled from a JSON
//         schema (engine/guided/json_schema.py) and the byte string of every
//         vocabulary token.
// Output: next[S][V] (int16, -1 = token forbidden in that state) and
//         dist[S]  (int16, min #tokens from the state to an accepting state).
//
// The table is uploaded once to HBM and read by the fused mask+sample HIP
// kernel (csrc/kernels/sample.hip): one int16 row gather per sequence per
// decode step, so heterogeneous schemas share one batch with no CPU work per
// token.  dist[] drives the budget-aware mode (never pick a token after which
// the JSON can no longer be closed within the remaining max_tokens).
//
// Walk: tokens are visited in lexicographic byte order and the DFA state
// after every prefix is kept on a stack, so each start state costs one pass
// over the (implicit) vocabulary trie instead of sum(len(token)).

#include <algorithm>
#include <cstdint>
#include <deque>
#include <numeric>
#include <string>
#include <vector>

#include "runtime.h"

namespace bcg {

TokenFsmTables compile_token_fsm(const int32_t* trans, const uint8_t* accept, int num_states,
                                 const std::vector<std::string>& tokens, int vocab_rows) {
  const int n_tok = static_cast<int>(tokens.size());
  std::vector<int> order(n_tok);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(),
            [&](int a, int b) { return tokens[a] < tokens[b]; });
  std::vector<int> lcp(n_tok, 0);
  size_t max_len = 0;
  for (int i = 0; i < n_tok; ++i) {
    const std::string& cur = tokens[order[i]];
    max_len = std::max(max_len, cur.size());
    if (i == 0) continue;
    const std::string& prev = tokens[order[i - 1]];
    size_t k = 0, m = std::min(prev.size(), cur.size());
    while (k < m && prev[k] == cur[k]) ++k;
    lcp[i] = static_cast<int>(k);
  }

  TokenFsmTables out;
  out.num_states = num_states;
  out.vocab_rows = vocab_rows;
  out.next.assign(static_cast<size_t>(num_states) * vocab_rows, int16_t(-1));
  out.dist.assign(num_states, int16_t(INT16_MAX));

  std::vector<int32_t> stack(max_len + 1);
  for (int s = 0; s < num_states; ++s) {
    int16_t* row = out.next.data() + static_cast<size_t>(s) * vocab_rows;
    stack[0] = s;
    for (int i = 0; i < n_tok; ++i) {
      const std::string& tok = tokens[order[i]];
      const int len = static_cast<int>(tok.size());
      if (len == 0) continue;  // special / unusable token
      for (int k = std::min(lcp[i], len); k < len; ++k) {
        const int32_t cur = stack[k];
        stack[k + 1] = cur < 0 ? -1 : trans[cur * 256 + static_cast<uint8_t>(tok[k])];
      }
      const int id = order[i];
      if (id < vocab_rows && stack[len] >= 0) row[id] = static_cast<int16_t>(stack[len]);
    }
  }

  // dist: BFS on the reversed, de-duplicated state graph.
  std::vector<std::vector<int>> rev(num_states);
  for (int s = 0; s < num_states; ++s) {
    std::vector<uint8_t> seen(num_states, 0);
    const int16_t* row = out.next.data() + static_cast<size_t>(s) * vocab_rows;
    for (int t = 0; t < vocab_rows; ++t) {
      const int16_t d = row[t];
      if (d >= 0 && !seen[d]) {
        seen[d] = 1;
        rev[d].push_back(s);
      }
    }
  }
  std::deque<int> q;
  for (int s = 0; s < num_states; ++s)
    if (accept[s]) {
      out.dist[s] = 0;
      q.push_back(s);
    }
  while (!q.empty()) {
    const int d = q.front();
    q.pop_front();
    for (int p : rev[d])
      if (out.dist[p] == INT16_MAX) {
        out.dist[p] = static_cast<int16_t>(out.dist[d] + 1);
        q.push_back(p);
      }
  }
  return out;
}

}  // namespace bcg
