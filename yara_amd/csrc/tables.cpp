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

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <unordered_map>
#include <utility>

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

void filter_put(std::vector<uint32_t>& f, const FilterProbe& fp) {
  f[2 * fp.block] |= 1u << fp.b_lo;
  f[2 * fp.block + 1] |= 1u << fp.b_hi;
}
void filter_set(std::vector<uint32_t>& f, uint32_t w3) {
  filter_put(f, filter_probe_left(w3));
  filter_put(f, filter_probe_right(w3));
}

// Two-choice, 4-way bucketed cuckoo table of non-zero keys.  Load <= 1/2 to
// start; the bucket count doubles until every key is placed.
bool build_bucket_table(const std::vector<uint32_t>& keys, std::vector<uint32_t>& table,
                        uint32_t& n_buckets) {
  uint32_t nb = 4;
  while (nb * 4 < 2 * keys.size()) nb <<= 1;
  for (; nb <= (1u << 26); nb <<= 1) {
    table.assign((size_t)nb * 4, 0u);
    uint32_t rng = 0x2545F491u;
    bool ok = true;
    for (uint32_t key0 : keys) {
      uint32_t key = key0;
      bool placed = false;
      for (int kick = 0; kick < 512 && !placed; ++kick) {
        const uint32_t b[2] = {bucket_hash1(key) & (nb - 1), bucket_hash2(key) & (nb - 1)};
        for (int c = 0; c < 2 && !placed; ++c) {
          for (int s = 0; s < 4; ++s) {
            uint32_t& slot = table[(size_t)b[c] * 4 + s];
            if (slot == key) { placed = true; break; }   // duplicate
            if (slot == 0) { slot = key; placed = true; break; }
          }
        }
        if (!placed) {   // evict a random resident of one of the two buckets
          rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5;
          uint32_t& victim = table[(size_t)b[rng & 1] * 4 + ((rng >> 1) & 3)];
          const uint32_t v = victim;
          victim = key;
          key = v;
        }
      }
      if (!placed) { ok = false; break; }
    }
    if (ok) {
      n_buckets = nb;
      return true;
    }
  }
  return false;
}

// Two-choice, 2-way bucketed cuckoo table of {key, value} pairs (non-zero
// keys): 4 words per bucket, load <= 1/4 to start, doubled until it fits.
bool build_pair_table(const std::vector<uint32_t>& keys, const std::vector<uint32_t>& vals,
                      std::vector<uint32_t>& table, uint32_t& n_buckets) {
  uint32_t nb = 4;
  while (nb * 2 < 4 * keys.size()) nb <<= 1;
  for (; nb <= (1u << 26); nb <<= 1) {
    table.assign((size_t)nb * 4, 0u);
    uint32_t rng = 0x9E3779B9u;
    bool ok = true;
    for (size_t i = 0; i < keys.size() && ok; ++i) {
      uint32_t key = keys[i], val = vals[i];
      bool placed = false;
      for (int kick = 0; kick < 512 && !placed; ++kick) {
        const uint32_t b[2] = {bucket_hash1(key) & (nb - 1), bucket_hash2(key) & (nb - 1)};
        for (int c = 0; c < 2 && !placed; ++c)
          for (int e = 0; e < 2; ++e) {
            uint32_t* slot = &table[(size_t)b[c] * 4 + 2 * e];
            if (slot[0] == 0 || slot[0] == key) {
              slot[0] = key;
              slot[1] = val;
              placed = true;
              break;
            }
          }
        if (!placed) {
          rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5;
          uint32_t* victim = &table[(size_t)b[rng & 1] * 4 + 2 * ((rng >> 1) & 1)];
          std::swap(victim[0], key);
          std::swap(victim[1], val);
        }
      }
      ok = placed;
    }
    if (ok) {
      n_buckets = nb;
      return true;
    }
  }
  return false;
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
  // the walk (scanner.c:124-141, replayed by ac_step and the verify kernel)
  // reads T[state + byte + 1] and follows failure links T[state] >> 9: every
  // state's 256-slot row must lie inside T, and every failure link must lead
  // to a shallower state, so the walk stays in bounds and terminates
  {
    std::vector<int16_t> depth_of(n_slots, -1);
    for (const Node& n : nodes) depth_of[n.slot] = (int16_t)n.depth;
    for (const Node& n : nodes) {
      if ((uint64_t)n.slot + 256 >= n_slots) return YR_AMD_INVALID_ARGUMENT;
      if (n.depth == 0) continue;
      const uint32_t f = T[n.slot] >> 9;
      if (f >= n_slots || depth_of[f] < 0 || (uint32_t)depth_of[f] >= n.depth)
        return YR_AMD_INVALID_ARGUMENT;
    }
  }
  out.n_states = (uint32_t)nodes.size();
  for (const Node& n : nodes) {
    out.by_depth[n.depth]++;
    if (n.depth > out.max_depth) out.max_depth = n.depth;
    if (M[n.slot] != 0) out.accepting++;
  }
  out.root_accepting = M[0] != 0;
  out.deep_pair.assign(256 * 8, 0u);
  for (const Node& n : nodes) {
    if (n.depth < 2) continue;
    const uint32_t last = (n.bytes >> (8 * (n.depth - 1))) & 0xFFu;
    const uint32_t prev = (n.bytes >> (8 * (n.depth - 2))) & 0xFFu;
    // the depth-1 node of `last`, if any (its slot from the root's row)
    const uint32_t t1 = T[last + 1];
    const bool has1 = (t1 & 0x1FFu) == last + 1;
    if (has1 && M[n.slot] == M[t1 >> 9]) continue;   // the same calls as `last` alone
    out.deep_last[last >> 5] |= 1u << (last & 31);
    out.deep_pair[last * 8 + (prev >> 5)] |= 1u << (prev & 31);
  }

  // accepting nodes by string (pre-verification, internal.h kNode*)
  {
    out.nodes.assign(kNodeHeadWords, 0u);
    std::vector<uint32_t> k3, v3, k4, v4;
    for (const Node& n : nodes) {
      const uint32_t head = M[n.slot];
      if (n.depth == 0 || head == 0) continue;
      switch (n.depth) {
        case 1: out.nodes[kNodeL1 + n.bytes] = head; break;
        case 2: out.nodes[kNodeL2 + n.bytes] = head; break;
        case 3: k3.push_back(n.bytes | (1u << 24)); v3.push_back(head); break;
        default:
          if (n.bytes == 0) out.nodes[kNodeZero4] = head;
          else { k4.push_back(n.bytes); v4.push_back(head); }
      }
    }
    std::vector<uint32_t> t3, t4;
    uint32_t nb3 = 0, nb4 = 0;
    if (!build_pair_table(k3, v3, t3, nb3) || !build_pair_table(k4, v4, t4, nb4))
      return YR_AMD_INTERNAL_FATAL_ERROR;
    out.n3_off = (uint32_t)out.nodes.size();
    out.n3_mask = nb3 - 1;
    out.nodes.insert(out.nodes.end(), t3.begin(), t3.end());
    out.n4_off = (uint32_t)out.nodes.size();
    out.n4_mask = nb4 - 1;
    out.nodes.insert(out.nodes.end(), t4.begin(), t4.end());
  }

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

  // 3a. LDS window filter over the 3 bytes ending at each position; up to
  //     kMaxByteKeys 1-byte keys are tested by the kernel byte by byte instead
  if (out.keys_by_len[1] <= kMaxByteKeys) {
    for (const Key& k : out.keys)
      if (k.len == 1) out.byte_keys |= (k.bytes & 0xFFu) << (8 * out.n_byte_keys++);
  }
  // The pair filter: every key window in both roles, every position tested
  // (1-byte keys tested byte by byte are not in it).
  out.filter.assign(kFilterWords, 0u);
  for (const Key& k : out.keys) {
    if (k.len == 1 && out.n_byte_keys != 0) continue;
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
  // The even-position filter (internal.h kFilterEven): the left role alone,
  // tested at the even positions k only, a pass standing for k and k + 1.  So
  // every key must have a window ending at k whichever of k, k + 1 it ends at:
  // a 4-byte key its suffix (ending at k) and its prefix (ending at k + 1); a
  // 3-byte key (p,q,r) itself and (*,p,q) -- the 256 windows with any first
  // byte, one block's low word and 8 bits of its high word in the plain form;
  // a 2-byte key (p,q) (*,p,q) and (*,*,p) -- the 64 plain blocks with last
  // byte p, all bits.  Not with 1-byte keys in the filter (they would pass
  // every window).  Both block forms are built; random windows pass a filter
  // with probability sum over blocks of |lo bits| x |hi bits| / 2^24.
  // (YAMD_PAIR_FILTER: the pair filter regardless -- A/B measurements.)
  const bool byte_keys_all = out.keys_by_len[1] == out.n_byte_keys;
  // 2-byte keys ending at odd positions: a half-word test in stage 1 when few
  const bool pair_test = out.keys_by_len[2] <= kMaxPairKeys;
  if (byte_keys_all && diag_env("YAMD_PAIR_FILTER") == nullptr) {
    auto pass_sum = [](const std::vector<uint32_t>& f) {
      uint64_t sum = 0;
      for (uint32_t b = 0; b < kFilterWords / 2; ++b)
        sum += (uint64_t)__builtin_popcount(f[2 * b]) * __builtin_popcount(f[2 * b + 1]);
      return sum;
    };
    std::vector<uint32_t> f[2];
    uint64_t pass[2] = {0, 0};
    for (int h = 0; h < 2; ++h) {
      f[h].assign(kFilterWords, 0u);
      for (const Key& k : out.keys) {
        switch (k.len) {
          case 4:
            filter_put(f[h], filter_probe_even(k.bytes >> 8, h));        // suffix
            filter_put(f[h], filter_probe_even(k.bytes & 0xFFFFFFu, h));  // prefix
            break;
          case 3:
            filter_put(f[h], filter_probe_even(k.bytes, h));
            for (uint32_t x = 0; x < 256; ++x) filter_put(f[h], filter_probe_even(x | (k.bytes << 8), h));
            break;
          case 2:
            for (uint32_t x = 0; x < 256; ++x) filter_put(f[h], filter_probe_even(x | (k.bytes << 8), h));
            if (!pair_test)
              for (uint32_t xy = 0; xy < 65536; ++xy)
                filter_put(f[h], filter_probe_even(xy | (k.bytes << 16), h));
            break;
          default: break;   // 1-byte keys: tested byte by byte
        }
      }
      pass[h] = pass_sum(f[h]);
    }
    const char* e = diag_env("YAMD_EVEN_FILTER");
    int pick = -1;   // -1: pair, 0: even plain, 1: even hashed
    if (e != nullptr) {
      pick = strcmp(e, "hash") == 0 ? 1 : 0;
    } else if (out.len_mask == (1u << 4)) {
      // 4-byte keys only: always even; the hashed form unless the plain one
      // passes at most 4/3 as many windows (its test is one instruction shorter)
      pick = 4 * pass[1] < 3 * pass[0] ? 1 : 0;
    } else {
      // Other shapes: a per-tile issue model in VALU-equivalents per 1 KiB tile
      // (~7 us of a 4 GiB scan each; fitted to the kernel times of rx, short,
      // hex, fuzz1, fuzz4, bytekeys and C under both filters,
      // profiles/r03_even_shapes_ab.json): stage 1 (pair 91, even 55, hashed
      // even 63) + 12 per 1-byte key tested + the ring append in tiles with an
      // entry (12) + per entry of certain 1-byte-key hits 6 and per entry of
      // filter passes 5 (first level) or 23 (2-byte keys: every hit position
      // goes to the bucket probes), never below the kernel's floor (pair 100,
      // even 89: the input stream plus the loop).  A plain even block whose
      // last byte is a 1-byte key passes only at positions that are certain
      // candidates anyway, so its passes add no entries.
      const double K = out.n_byte_keys, d_filt = (out.len_mask & 6u) ? 23.0 : 5.0;
      auto is_byte_key = [&](uint32_t c) {
        for (uint32_t i = 0; i < out.n_byte_keys; ++i)
          if (((out.byte_keys >> (8 * i)) & 0xFFu) == c) return true;
        return false;
      };
      uint64_t pass_plain_new = 0;
      for (uint32_t b = 0; b < kFilterWords / 2; ++b)
        if (!is_byte_key((b >> 6) & 0xFFu))
          pass_plain_new += (uint64_t)__builtin_popcount(f[0][2 * b]) * __builtin_popcount(f[0][2 * b + 1]);
      auto cost = [&](double stage1, double floor, double p_window, int tests) {
        const double cert = 1.0 - std::pow(1.0 - K / 256.0, (double)kBytesPerLane);
        const double filt = 1.0 - std::pow(1.0 - p_window, tests);
        const double lane = 1.0 - (1.0 - cert) * (1.0 - filt);
        const double c = stage1 + 12.0 * K + 12.0 * (1.0 - std::pow(1.0 - lane, (double)kWave)) +
                         kWave * (6.0 * cert + d_filt * filt);
        return std::max(floor, c);
      };
      // (+12 per 2-byte key tested as half-words: 3 per dword, like a 1-byte key)
      const double s_pair = pair_test ? 12.0 * out.keys_by_len[2] : 0.0;
      const double c_pair = cost(91.0, 100.0, pass_sum(out.filter) / 16777216.0, kBytesPerLane);
      const double c_even[2] = {cost(55.0 + s_pair, 89.0, pass_plain_new / 16777216.0, kBytesPerLane / 2),
                                cost(63.0 + s_pair, 89.0, pass[1] / 16777216.0, kBytesPerLane / 2)};
      const int h = c_even[1] < c_even[0] ? 1 : 0;
      if (c_even[h] < 0.97 * c_pair) pick = h;
    }
    if (pick >= 0) {
      out.filter_mode = pick ? kFilterEvenHash : kFilterEven;
      out.filter = std::move(f[pick]);
      if (pair_test)
        for (const Key& k : out.keys)
          if (k.len == 2) {
            out.pair_keys[out.n_pair_keys / 2] |= (k.bytes & 0xFFFFu) << (16 * (out.n_pair_keys % 2));
            ++out.n_pair_keys;
          }
    }
  }
  for (uint32_t w : out.filter) out.filter_set_bits += (uint32_t)__builtin_popcount(w);

  // 3b. exact key sets: bitmaps for 1-2 byte keys, two-choice bucketed
  //     hash tables for 3-4 byte keys
  std::vector<uint32_t> k3, k4;
  out.exact.assign(kExactHeadWords, 0u);
  for (const Key& k : out.keys) {
    switch (k.len) {
      case 1: out.exact[kExactBm1 + (k.bytes >> 5)] |= 1u << (k.bytes & 31); break;
      case 2: out.exact[kExactBm2 + (k.bytes >> 5)] |= 1u << (k.bytes & 31); break;
      case 3:
        k3.push_back(k.bytes | (1u << 24));
        out.exact[kExactFl + fl_word(k.bytes << 8)] |= 1u << fl_bit3(k.bytes << 8);
        break;
      case 4:
        if (k.bytes == 0) out.exact_flags |= kExactZero4;
        else k4.push_back(k.bytes);
        out.exact[kExactFl + fl_word(k.bytes)] |= 1u << fl_bit4(k.bytes);
        break;
    }
  }
  std::vector<uint32_t> t3, t4;
  uint32_t nb3 = 0, nb4 = 0;
  if (!build_bucket_table(k3, t3, nb3) || !build_bucket_table(k4, t4, nb4))
    return YR_AMD_INTERNAL_FATAL_ERROR;
  out.t3_off = (uint32_t)out.exact.size();
  out.t3_mask = nb3 - 1;
  out.exact.insert(out.exact.end(), t3.begin(), t3.end());
  out.t4_off = (uint32_t)out.exact.size();
  out.t4_mask = nb4 - 1;
  out.exact.insert(out.exact.end(), t4.begin(), t4.end());
  return YR_AMD_SUCCESS;
}

}  // namespace yamd
