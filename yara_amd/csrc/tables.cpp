// Flattening of libyara's compiled Aho-Corasick tables into the scan form.
//
// Input is exactly what YR_RULES exposes (rules.c:356-363): the interleaved
// transition table T (ahocorasick.h:37-50, built by ahocorasick.c:525-643),
// the match table M and the match-pool list links/backtracks.
//
// 1. Walk the trie out of T: a slot s+b+1 is a child of state s iff its low
//    9 bits equal b+1 (the owner-offset check of ahocorasick.h:43).
// 2. A state accepts iff M[state] != 0.  libyara builds every match list as
//    own matches ++ list(failure) (ahocorasick.c:254-300), so acceptance is
//    monotone along true failure links; this is verified here.  With depth
//    <= 4 (YR_MAX_ATOM_LENGTH, limits.h:68) the walk's state at position i
//    is the longest trie suffix of the last <= 4 bytes, hence
//        M[state_i] != 0  <=>  some minimal accepting string ends at i.
//    Those strings are the "keys" (1..4 bytes).  A non-empty root list
//    (M[0] != 0) makes every position a candidate.
// 3. Keys -> an LDS window filter (2^20 bits over the hashed 3-byte window;
//    shorter keys are inserted with every possible leading byte) and an exact
//    open-addressed hash table for the second stage.
#include "tables.h"

#include <string.h>

#include <unordered_map>

#include "../../include/yara_amd.h"
#include "internal.h"

namespace yamd {

namespace {

struct Node {
  uint32_t slot;
  uint32_t bytes;  // little-endian packed string
  uint32_t depth;
};

inline uint64_t node_key(uint32_t bytes, uint32_t depth) { return ((uint64_t)depth << 32) | bytes; }

void filter_set(std::vector<uint32_t>& f, uint32_t w3) {
  const FilterProbe fp = filter_probe(w3);
  f[fp.word] |= (1u << fp.b1) | (1u << fp.b2);
}

}  // namespace

int flatten_tables(const uint32_t* T, const uint32_t* M, uint32_t n_slots,
                   const uint32_t* pool_next, const uint16_t* pool_backtrack, uint32_t n_pool,
                   FlatTables& out) {
  if (T == nullptr || M == nullptr || n_slots < 1) return YR_AMD_INVALID_ARGUMENT;
  if (n_pool > 0 && (pool_next == nullptr || pool_backtrack == nullptr))
    return YR_AMD_INVALID_ARGUMENT;

  out.n_slots = n_slots;
  out.T.assign(T, T + n_slots);
  out.M.assign(M, M + n_slots);
  out.pool_next.assign(pool_next, pool_next + n_pool);
  out.pool_backtrack.assign(pool_backtrack, pool_backtrack + n_pool);

  // match-table / pool sanity: indexes in range and every list acyclic
  for (uint32_t s = 0; s < n_slots; ++s) {
    if (M[s] > n_pool) return YR_AMD_INVALID_ARGUMENT;
  }
  for (uint32_t k = 0; k < n_pool; ++k) {
    if (pool_next[k] > n_pool) return YR_AMD_INVALID_ARGUMENT;
  }
  {
    // every `next` chain must end (0 = unvisited, 1 = on the current walk, 2 = ends)
    std::vector<uint8_t> color(n_pool + 1, 0);
    for (uint32_t k0 = 1; k0 <= n_pool; ++k0) {
      uint32_t k = k0;
      while (k != 0 && color[k] == 0) {
        color[k] = 1;
        k = pool_next[k - 1];
      }
      if (k != 0 && color[k] == 1) return YR_AMD_INVALID_ARGUMENT;
      for (uint32_t j = k0; j != 0 && color[j] == 1; j = pool_next[j - 1]) color[j] = 2;
    }
  }

  // 1. trie from T (BFS, as ahocorasick.c:556-640 laid it out)
  std::vector<Node> nodes;
  std::unordered_map<uint64_t, uint32_t> index;  // (depth, bytes) -> node id
  std::vector<uint8_t> seen(n_slots, 0);
  nodes.push_back({0, 0, 0});
  index[node_key(0, 0)] = 0;
  seen[0] = 1;
  for (size_t q = 0; q < nodes.size(); ++q) {
    const Node cur = nodes[q];
    for (uint32_t b = 0; b < 256; ++b) {
      const uint64_t slot = (uint64_t)cur.slot + b + 1;
      if (slot >= n_slots) break;
      const uint32_t t = T[slot];
      if ((t & 0x1FFu) != b + 1) continue;
      const uint32_t child = t >> 9;
      if (child >= n_slots || seen[child]) return YR_AMD_INVALID_ARGUMENT;
      if (cur.depth + 1 > YR_AMD_MAX_ATOM_LENGTH) return YR_AMD_INVALID_ARGUMENT;
      seen[child] = 1;
      const Node n{child, cur.bytes | (b << (8 * cur.depth)), cur.depth + 1};
      index[node_key(n.bytes, n.depth)] = (uint32_t)nodes.size();
      nodes.push_back(n);
    }
  }
  out.n_states = (uint32_t)nodes.size();
  for (const Node& n : nodes) {
    out.by_depth[n.depth]++;
    if (n.depth > out.max_depth) out.max_depth = n.depth;
    if (M[n.slot] != 0) out.accepting++;
  }
  out.root_accepting = M[0] != 0;

  // 2. minimal accepting strings; verify monotonicity along true failure links
  for (const Node& n : nodes) {
    if (n.depth == 0) continue;
    bool fail_accepts = false;
    for (uint32_t k = 1; k <= n.depth; ++k) {  // longest proper suffix first
      const uint32_t sl = n.depth - k;
      const uint32_t suffix = sl == 0 ? 0u : (n.bytes >> (8 * k)) & (0xFFFFFFFFu >> (32 - 8 * sl));
      auto it = index.find(node_key(suffix, sl));
      if (it != index.end()) {
        fail_accepts = M[nodes[it->second].slot] != 0;
        break;
      }
    }
    const bool acc = M[n.slot] != 0;
    if (fail_accepts && !acc) return YR_AMD_INVALID_ARGUMENT;  // not libyara's construction
    if (acc && !fail_accepts) out.keys.push_back({n.bytes, n.depth});
  }
  for (const Key& k : out.keys) {
    out.keys_by_len[k.len]++;
    out.len_mask |= 1u << k.len;
  }

  // 3a. LDS window filter over the 3 bytes ending at each position
  out.filter.assign(kFilterWords, 0u);
  for (const Key& k : out.keys) {
    switch (k.len) {
      case 4: filter_set(out.filter, k.bytes >> 8); break;
      case 3: filter_set(out.filter, k.bytes); break;
      case 2:
        for (uint32_t x = 0; x < 256; ++x) filter_set(out.filter, x | (k.bytes << 8));
        break;
      case 1:
        for (uint32_t xy = 0; xy < 65536; ++xy) filter_set(out.filter, xy | (k.bytes << 16));
        break;
    }
  }
  for (uint32_t w : out.filter) out.filter_set_bits += (uint32_t)__builtin_popcount(w);

  // 3b. exact keys, load factor <= 1/4 (a miss costs ~1.2 probes)
  uint32_t slots = 64;
  while (slots < 4 * out.keys.size()) slots <<= 1;
  out.exact.assign(slots, 0ull);
  for (const Key& k : out.keys) {
    uint32_t s = exact_hash(k.bytes, k.len) & (slots - 1);
    while (out.exact[s] != 0) s = (s + 1) & (slots - 1);
    out.exact[s] = exact_entry(k.bytes, k.len);
  }
  return YR_AMD_SUCCESS;
}

}  // namespace yamd
