// Topology-aware GPU-set selection (GetPreferredAllocation, multi-GPU vGPU
// placement) — the native solver the device plugin calls over the amdsmi link
// matrix, instead of exec'ing a vendor tool.
//
// Reference analogues: the MLU plugin shells out to `cntopo find` and parses
// rings (pkg/device-plugin/mlu/cntopo/cntopo.go:54-98), then its board/spider
// allocators rank candidate sets by non-conflicting MLULink rings
// (pkg/device-plugin/mlu/allocator/board.go:35-194); the NVIDIA plugin's
// gpuallocator ranks by NVLink (rm/allocate.go:26-121).  SURVEY.md §2.4 M7/M8.
//
// Score of a candidate set (lexicographic, higher wins; identical to
// vgpu/deviceplugin/topology.py:score_set, which is the executable spec):
//   (#xGMI-connected pairs, -#hives, -#NUMA nodes, Σ already-used slots,
//    -(sorted positions))   — the last term makes ties deterministic.
// Exhaustive over combinations in itertools order, capped at `limit` sets:
// an 8-GPU node is ≤70 sets; a CPX-partitioned node (64 logical devices)
// relies on the cap, which a Python loop cannot afford at Allocate time.
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace {

constexpr int kLinkXgmi = 2;

struct Score {
  int pairs, neg_hives, neg_numas;
  long long busy;
  std::vector<int> neg_idx;
  bool operator>(const Score& o) const {
    if (pairs != o.pairs) return pairs > o.pairs;
    if (neg_hives != o.neg_hives) return neg_hives > o.neg_hives;
    if (neg_numas != o.neg_numas) return neg_numas > o.neg_numas;
    if (busy != o.busy) return busy > o.busy;
    return neg_idx > o.neg_idx;
  }
};

int distinct(const std::vector<int>& idx, const int* key) {
  std::vector<int> v;
  v.reserve(idx.size());
  for (int i : idx) v.push_back(key[i]);
  std::sort(v.begin(), v.end());
  return (int)(std::unique(v.begin(), v.end()) - v.begin());
}

Score score(const std::vector<int>& idx, int n, const int* links, const int* numa, const int* hive,
            const int* used) {
  Score s;
  s.pairs = 0;
  for (size_t a = 0; a < idx.size(); ++a)
    for (size_t b = a + 1; b < idx.size(); ++b)
      if (links[idx[a] * n + idx[b]] == kLinkXgmi) ++s.pairs;
  s.neg_hives = -distinct(idx, hive);
  s.neg_numas = -distinct(idx, numa);
  s.busy = 0;
  for (int i : idx) s.busy += used[i];
  for (int i : idx) s.neg_idx.push_back(-i);
  return s;
}

}  // namespace

extern "C" {

// Positions are indices into the node's device list (0..n-1).  Returns the
// number of positions written to `out` (sorted ascending, ≤ size), or -1.
__attribute__((visibility("default"))) int vgpu_topo_preferred(
    int n, const int* links, const int* numa, const int* hive, const int* used, const int* avail,
    int navail, const int* must_in, int nmust_in, int size, long long limit, int* out) {
  if (n < 0 || navail < 0 || nmust_in < 0 || size < 0 || !out) return -1;
  auto in_avail = [&](int x) { return std::find(avail, avail + navail, x) != avail + navail; };
  std::vector<int> must, rest;
  for (int i = 0; i < nmust_in; ++i)
    if (in_avail(must_in[i])) must.push_back(must_in[i]);
  for (int i = 0; i < navail; ++i)
    if (std::find(must.begin(), must.end(), avail[i]) == must.end()) rest.push_back(avail[i]);
  for (int x : must)
    if (x < 0 || x >= n) return -1;
  for (int x : rest)
    if (x < 0 || x >= n) return -1;
  const int need = size - (int)must.size();
  if (need <= 0) {
    const int k = std::min(size, (int)must.size());
    std::copy(must.begin(), must.begin() + k, out);
    return k;
  }
  if (need > (int)rest.size()) {
    std::copy(must.begin(), must.end(), out);
    std::copy(rest.begin(), rest.end(), out + must.size());
    return (int)(must.size() + rest.size());
  }
  std::vector<int> c(need);
  for (int i = 0; i < need; ++i) c[i] = i;  // combination of positions into `rest`
  bool have = false;
  Score best;
  std::vector<int> best_set, cand;
  const int r = (int)rest.size();
  for (long long count = 0; count < limit; ++count) {
    cand = must;
    for (int i : c) cand.push_back(rest[i]);
    std::sort(cand.begin(), cand.end());
    Score s = score(cand, n, links, numa, hive, used);
    if (!have || s > best) {
      best = s;
      best_set = cand;
      have = true;
    }
    int i = need - 1;  // next combination (itertools.combinations order)
    while (i >= 0 && c[i] == r - need + i) --i;
    if (i < 0) break;
    ++c[i];
    for (int j = i + 1; j < need; ++j) c[j] = c[j - 1] + 1;
  }
  std::copy(best_set.begin(), best_set.end(), out);
  return (int)best_set.size();
}

}  // extern "C"
