#include "alloc/topology.h"

#include <algorithm>
#include <climits>
#include <functional>
#include <map>
#include <set>

namespace adp::alloc {

using inventory::LinkClass;

int PairScore(const inventory::Snapshot& snap, int a, int b) {
  if (a == b) return 1000;
  const auto& ga = snap.gpus[a];
  const auto& gb = snap.gpus[b];
  int score = (ga.numa >= 0 && ga.numa == gb.numa) ? 20 : 10;
  switch (snap.Link(a, b)) {
    case LinkClass::kSame: return 1000;
    case LinkClass::kXgmi: {
      uint64_t hops = std::max<uint64_t>(1, snap.Hops(a, b));
      score += static_cast<int>(100 / hops);
      break;
    }
    case LinkClass::kPcieSameNuma:
    case LinkClass::kPcieCrossNuma:
    case LinkClass::kUnknown:
      break;
  }
  score -= 10 * (ga.xgmi_links_down + gb.xgmi_links_down);
  return score;
}

DeviceGraph::DeviceGraph(const inventory::Snapshot& snap, const std::vector<DeviceRef>& devices)
    : n_(static_cast<int>(devices.size())), parent_(devices.size()), score_(devices.size() * devices.size()) {
  for (int i = 0; i < n_; ++i) parent_[i] = devices[i].gpu;
  for (int i = 0; i < n_; ++i)
    for (int j = 0; j < n_; ++j)
      score_[i * n_ + j] = (i == j) ? 0 : PairScore(snap, devices[i].gpu, devices[j].gpu);
}

DeviceGraph::DeviceGraph(std::vector<int> parent, std::vector<int> scores)
    : n_(static_cast<int>(parent.size())), parent_(std::move(parent)), score_(std::move(scores)) {}

namespace {

constexpr int kExactMax = 12;  // exact search up to 12 whole GPUs (4096 DP states)

// Calls fn(sub) for every subset of `pool` with exactly `sz` bits, in
// lexicographic order of bit positions. No allocation.
template <typename Fn>
void Combinations(uint32_t pool, int sz, Fn&& fn) {
  int pos[32], n = 0;
  for (uint32_t a = pool; a; a &= a - 1) pos[n++] = __builtin_ctz(a);
  if (sz < 0 || sz > n) return;
  if (sz == 0) { fn(0u); return; }
  int idx[32];
  for (int i = 0; i < sz; ++i) idx[i] = i;
  while (true) {
    uint32_t m = 0;
    for (int i = 0; i < sz; ++i) m |= 1u << pos[idx[i]];
    fn(m);
    int i = sz - 1;
    while (i >= 0 && idx[i] == n - sz + i) --i;
    if (i < 0) return;
    ++idx[i];
    for (int j = i + 1; j < sz; ++j) idx[j] = idx[j - 1] + 1;
  }
}

// The reference objective, solved by memoized DP over subsets: f(S) = best total
// intra-group score of splitting S into groups of size k (plus one group of the
// remainder size when |S| is not a multiple of k).
struct ExactSearch {
  int m, k, r;
  int s[kExactMax][kExactMax];
  int memo[1 << kExactMax];

  int SetScore(uint32_t mask) const {
    int t = 0;
    for (uint32_t a = mask; a; a &= a - 1) {
      int i = __builtin_ctz(a);
      for (uint32_t b = a & (a - 1); b; b &= b - 1) t += s[i][__builtin_ctz(b)];
    }
    return t;
  }

  int F(uint32_t mask) {
    if (!mask) return 0;
    if (memo[mask] != INT_MIN) return memo[mask];
    int low = __builtin_ctz(mask);
    uint32_t rest = mask & ~(1u << low);
    int cnt = __builtin_popcount(mask);
    int best = INT_MIN / 2;
    auto try_size = [&](int sz) {
      Combinations(rest, sz - 1, [&](uint32_t sub) {
        uint32_t grp = sub | (1u << low);
        int v = SetScore(grp) + F(mask & ~grp);
        if (v > best) best = v;
      });
    };
    if (cnt >= k) try_size(k);
    if (r > 0 && cnt % k == r) try_size(r);
    return memo[mask] = best;
  }

  std::vector<int> Run(const DeviceGraph& g, const std::vector<int>& avail,
                       const std::vector<int>& required) {
    m = static_cast<int>(avail.size());
    r = m % k;
    for (int i = 0; i < m; ++i)
      for (int j = 0; j < m; ++j) s[i][j] = i == j ? 0 : g.Score(avail[i], avail[j]);
    std::fill(memo, memo + (1 << m), INT_MIN);
    uint32_t full = (1u << m) - 1, req = 0;
    for (int d : required)
      for (int i = 0; i < m; ++i)
        if (avail[i] == d) req |= 1u << i;
    uint32_t best_grp = 0;
    int best_total = INT_MIN, best_set = INT_MIN;
    Combinations(full & ~req, k - __builtin_popcount(req), [&](uint32_t sub) {
      uint32_t grp = sub | req;
      int sc = SetScore(grp);
      int total = sc + F(full & ~grp);
      if (total > best_total || (total == best_total && sc > best_set)) {
        best_total = total;
        best_set = sc;
        best_grp = grp;
      }
    });
    std::vector<int> out;
    for (uint32_t a = best_grp; a; a &= a - 1) out.push_back(avail[__builtin_ctz(a)]);
    return out;  // ascending, since avail is sorted
  }
};

// Flat-array form (parents are small dense indices): no maps/sets on the RPC
// path. Selection order is fixed by parent index and available-device order,
// so the result is deterministic.
std::vector<int> Hierarchical(const DeviceGraph& g, const std::vector<int>& avail,
                              const std::vector<int>& required, int size) {
  int np = 0;
  for (int d : avail) np = std::max(np, g.parent(d) + 1);
  // Unchosen available devices grouped by parent (counting sort keeps avail order).
  std::vector<int> begin(np + 1, 0), rep(np, -1);
  std::vector<char> is_req(g.size(), 0), in_set(np, 0);
  for (int d : required) is_req[d] = 1;
  for (int d : avail) {
    int p = g.parent(d);
    if (rep[p] < 0) rep[p] = d;
    if (!is_req[d]) ++begin[p + 1];
  }
  for (int p = 0; p < np; ++p) begin[p + 1] += begin[p];
  std::vector<int> devs(begin[np]), fill(begin.begin(), begin.end() - 1);
  for (int d : avail)
    if (!is_req[d]) devs[fill[g.parent(d)]++] = d;
  std::vector<int> next(begin.begin(), begin.end() - 1);  // first untaken per parent
  auto remaining = [&](int p) { return begin[p + 1] - next[p]; };

  std::vector<int> chosen(required.begin(), required.end());
  std::vector<int> parents;  // parents in the set, in insertion order
  for (int d : required) {
    int p = g.parent(d);
    if (!in_set[p]) { in_set[p] = 1; parents.push_back(p); }
  }
  int need = size - static_cast<int>(chosen.size());
  auto take = [&](int p) {
    while (need > 0 && next[p] < begin[p + 1]) {
      chosen.push_back(devs[next[p]++]);
      --need;
    }
    if (!in_set[p]) { in_set[p] = 1; parents.push_back(p); }
  };

  // 1. Finish on the GPUs the required devices already occupy (most room first,
  //    ties by parent index).
  std::vector<int> req_parents(parents);
  std::sort(req_parents.begin(), req_parents.end());
  std::stable_sort(req_parents.begin(), req_parents.end(),
                   [&](int a, int b) { return remaining(a) > remaining(b); });
  for (int p : req_parents) take(p);

  // 2. Grow: affinity to the GPUs already chosen, then best fit, then index.
  while (need > 0) {
    int best = -1;
    long best_aff = LONG_MIN;
    bool best_fits = false;
    int best_room = 0;
    for (int p = 0; p < np; ++p) {
      int room = remaining(p);
      if (room == 0 || in_set[p]) continue;
      long aff = 0;
      for (int q : parents) aff += g.Score(rep[p], rep[q]);
      bool fits = room >= need;
      bool better;
      if (best < 0) better = true;
      else if (aff != best_aff) better = aff > best_aff;
      else if (fits != best_fits) better = fits;
      else if (fits) better = room < best_room;   // best fit: tightest hole
      else better = room > best_room;             // else: biggest chunk first
      if (better) {
        best = p;
        best_aff = aff;
        best_fits = fits;
        best_room = room;
      }
    }
    if (best < 0) return {};
    take(best);
  }
  std::sort(chosen.begin(), chosen.end());
  return chosen;
}

}  // namespace

std::vector<int> BestEffortAllocate(const DeviceGraph& g, const std::vector<int>& available,
                                    const std::vector<int>& required, int size) {
  if (size <= 0) return {};
  std::vector<int> avail(available);
  std::sort(avail.begin(), avail.end());
  avail.erase(std::unique(avail.begin(), avail.end()), avail.end());
  std::vector<int> req(required);
  std::sort(req.begin(), req.end());
  req.erase(std::unique(req.begin(), req.end()), req.end());
  if (static_cast<int>(avail.size()) < size || static_cast<int>(req.size()) > size) return {};
  for (int d : req)
    if (!std::binary_search(avail.begin(), avail.end(), d)) return {};
  for (int d : avail)
    if (d < 0 || d >= g.size()) return {};

  std::vector<int> ps;
  ps.reserve(avail.size());
  for (int d : avail) ps.push_back(g.parent(d));
  std::sort(ps.begin(), ps.end());
  bool distinct = std::adjacent_find(ps.begin(), ps.end()) == ps.end();
  if (distinct && avail.size() <= static_cast<size_t>(kExactMax)) {
    // k == 1: every split scores 0, so the objective picks the required device or
    // the first available one -- skip the search.
    if (size == 1) return req.empty() ? std::vector<int>{avail.front()} : req;
    ExactSearch search;
    search.k = size;
    return search.Run(g, avail, req);
  }
  return Hierarchical(g, avail, req, size);
}

}  // namespace adp::alloc
