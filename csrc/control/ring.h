// Ring-neighbour selection over an ordered map.
//
// Same contract as the reference's `symmetric_ring_neighbors(map, key, k,
// predicate)` (src/utils.rs:5-21): alternate the nearest left and right
// neighbours of `key` (excluding it), k times each, wrapping around the ends
// and never returning an entry twice on small rings. Pinned by the three
// reference tests (src/utils.rs:29-92), reproduced in `dmlc-node selftest`.
#pragma once
#include <iterator>
#include <map>
#include <vector>

namespace dmlc {
namespace ctl {

template <typename K, typename V, typename Pred>
std::vector<K> symmetric_ring_neighbors(const std::map<K, V>& m, const K& key, int k, Pred pred) {
  // left candidates: entries < key from nearest to farthest, then (wrap) the
  // largest entries > key; right candidates: entries > key ascending, then
  // (wrap) the smallest entries < key. A shared "taken" window prevents
  // duplicates: left consumes [lo_l .. ) downward, right consumes upward.
  std::vector<const std::pair<const K, V>*> below, above;  // filtered, ascending
  for (auto it = m.begin(); it != m.end(); ++it) {
    if (!(it->first < key) && !(key < it->first)) continue;
    if (!pred(*it)) continue;
    (it->first < key ? below : above).push_back(&*it);
  }
  // Deque-like cursors: left iterator walks `below` from the back, then `above`
  // from the back; right walks `above` from the front, then `below` from the
  // front. Both draw from the same remaining pool in order so no entry is
  // returned twice.
  size_t bl = 0, bh = below.size();  // remaining below: [bl, bh)
  size_t al = 0, ah = above.size();  // remaining above: [al, ah)
  std::vector<K> out;
  for (int i = 0; i < k; ++i) {
    if (bh > bl) {
      out.push_back(below[--bh]->first);
    } else if (ah > al) {
      out.push_back(above[--ah]->first);
    }
    if (ah > al) {
      out.push_back(above[al++]->first);
    } else if (bh > bl) {
      out.push_back(below[bl++]->first);
    }
  }
  return out;
}

}  // namespace ctl
}  // namespace dmlc
