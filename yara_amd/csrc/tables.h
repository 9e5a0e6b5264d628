// Host-side flattening of libyara's compiled Aho-Corasick tables.
#pragma once

#include <stdint.h>

#include <vector>

namespace yamd {

struct Key {
  uint32_t bytes;  // little endian: first byte of the key in bits 0-7
  uint32_t len;    // 1..4
};

struct FlatTables {
  // verbatim host copies of the reference tables (used by the replay)
  uint32_t n_slots = 0;
  std::vector<uint32_t> T, M, pool_next;
  std::vector<uint16_t> pool_backtrack;

  // trie statistics
  uint32_t n_states = 0, max_depth = 0, accepting = 0;
  uint32_t by_depth[5] = {0, 0, 0, 0, 0};
  uint32_t keys_by_len[5] = {0, 0, 0, 0, 0};
  bool root_accepting = false;

  // flattened scan form
  std::vector<Key> keys;           // minimal accepting trie strings
  std::vector<uint32_t> filter;    // kFilterWords
  uint32_t filter_set_bits = 0;
  // kFilterEven: every key is 4 bytes long, and the filter holds each key's
  // 3-byte prefix and suffix in the left role only -- the scan tests the
  // windows ending at even positions, each pass standing for that position
  // and the next (internal.h; kFilterEvenHash: its block hashed); kFilterPair:
  // both roles, every position
  uint32_t filter_mode = 0;
  std::vector<uint32_t> exact;     // exact key sets (internal.h layout)
  uint32_t t3_off = 0, t3_mask = 0, t4_off = 0, t4_mask = 0, exact_flags = 0;
  uint32_t len_mask = 0;
  // 1-byte keys tested byte by byte in the scan kernel's stage 1 instead of
  // being inserted into the window filter (each would fill it with 65,536
  // windows): up to kMaxByteKeys key bytes, packed low byte first
  uint32_t byte_keys = 0, n_byte_keys = 0;
  // even-position filters: up to kMaxPairKeys 2-byte keys (p | q << 8, two per
  // word) tested in stage 1 as the aligned half-words of the lane, i.e. where
  // they end at an odd position, instead of as the filter's (*, *, p) windows
  // (which would pass every byte p)
  uint32_t pair_keys[2] = {0, 0}, n_pair_keys = 0;
  // bit b set: some trie node of depth >= 2 ends with byte b and has another
  // match list than b's own node (so at a position whose last byte is the
  // 1-byte key b the calls may differ from b's list)
  uint32_t deep_last[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // bit x of row b (8 words a row): some trie node of depth >= 2 ends with the
  // bytes x, b and its match list (M, ahocorasick.c: its own matches, then its
  // failure state's) is not b's -- such a position's calls may differ from
  // b's.  Deeper nodes whose lists ARE b's (no matches of their own along the
  // failure chain down to b) make the same calls, so they do not count.
  std::vector<uint32_t> deep_pair;   // 256 x 8

  // accepting trie nodes -> match-list head M[slot], by the node's string
  // (pre-verification: the walk's state at a candidate is its longest
  // accepting suffix, found with independent probes instead of 4 dependent
  // transitions; internal.h node_* layout)
  std::vector<uint32_t> nodes;
  uint32_t n3_off = 0, n3_mask = 0, n4_off = 0, n4_mask = 0;
};

// Returns a YR_AMD_* error code.
int flatten_tables(const uint32_t* T, const uint32_t* M, uint32_t n_slots,
                   const uint32_t* pool_next, const uint16_t* pool_backtrack, uint32_t n_pool,
                   FlatTables& out);

// One transition of the reference walk (libyara/scanner.c:124-141).
inline uint32_t ac_step(const uint32_t* T, uint32_t state, uint8_t byte) {
  const uint32_t index = (uint32_t)byte + 1;
  uint32_t t = T[state + index];
  while ((t & 0x1FFu) != index) {
    if (state != 0) {
      state = T[state] >> 9;
      t = T[state + index];
    } else {
      t = 0;
      break;
    }
  }
  return t >> 9;
}

}  // namespace yamd
