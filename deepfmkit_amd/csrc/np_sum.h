// np_sum.h — numpy's float64 summation order, for bit-exact means.
//
// np.sum / np.mean of a contiguous float64 vector (numpy 2.x,
// numpy/_core/src/umath/loops_utils.h.src pairwise_sum): blocks of <= 128 elements
// summed with 8 accumulators, larger ranges split at n2 = n/2 - (n/2)%8; vectors
// longer than the ufunc buffer (8192) are reduced chunk by chunk, left to right.
// Checked against np.sum for n = 1 .. 30001 (tests/test_host_numerics.py).
#pragma once
#include <algorithm>
#include <functional>
#include <vector>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define DFMI_NP_HD __host__ __device__ __forceinline__
#else
#define DFMI_NP_HD static inline
#endif

// numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src: blocks of
// <= 128 with 8 accumulators, split at n2 = n/2 - (n/2)%8). np.sum / np.mean of a
// contiguous float64 vector use exactly this tree.
DFMI_NP_HD double dfmi_np_leaf_sum(const double* a, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
  int i = 8;
  const int e = n - (n % 8);
  for (; i < e; i += 8) {
    r0 += a[i + 0];
    r1 += a[i + 1];
    r2 += a[i + 2];
    r3 += a[i + 3];
    r4 += a[i + 4];
    r5 += a[i + 5];
    r6 += a[i + 6];
    r7 += a[i + 7];
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += a[i];
  return res;
}

// Host: numpy's reduction tree over n elements as a level plan (wdfmi.hip
// block_np_sum runs it on the device):
//   plan[0] = leaves nl, plan[1] = levels H, plan[2 .. 2+nl] = leaf offsets,
//   then H+1 level starts into the node triples (dst, a, b) that follow;
//   nodes 0..nl-1 are the leaves, the root is node 2*nl-2.
inline std::vector<int> dfmi_pairwise_plan(int n) {
  struct Node {
    int off, len, a, b, h;
  };
  std::vector<Node> nodes;
  std::vector<int> leaves;
  // recursive build; leaves numbered left to right, internal nodes after them
  std::vector<int> order;  // internal node ids in post-order
  std::function<int(int, int)> build = [&](int off, int m) -> int {
    if (m <= 128) {
      leaves.push_back(off);
      nodes.push_back({off, m, -1, -1, 0});
      return (int)nodes.size() - 1;
    }
    int n2 = m / 2;
    n2 -= n2 % 8;
    const int l = build(off, n2), r = build(off + n2, m - n2);
    nodes.push_back({off, m, l, r, 1 + std::max(nodes[l].h, nodes[r].h)});
    return (int)nodes.size() - 1;
  };
  // numpy reduces a long vector in buffer-sized chunks of 8192 elements, adding the
  // chunks' pairwise sums left to right
  int root = build(0, n < 8192 ? n : 8192);
  for (int off = 8192; off < n; off += 8192) {
    const int c = build(off, std::min(8192, n - off));
    nodes.push_back({0, off + std::min(8192, n - off), root, c, 1 + std::max(nodes[root].h, nodes[c].h)});
    root = (int)nodes.size() - 1;
  }
  // renumber: leaves 0..nl-1 in order, internal nodes nl.. by height (root last)
  const int nl = (int)leaves.size();
  std::vector<int> id(nodes.size(), -1);
  int next = 0;
  for (size_t k = 0; k < nodes.size(); ++k)
    if (nodes[k].a < 0) id[k] = next++;
  int H = 0;
  for (auto& x : nodes) H = std::max(H, x.h);
  std::vector<int> plan = {nl, H};
  for (int k = 0; k < nl; ++k) plan.push_back(leaves[k]);
  plan.push_back(n);
  // internal nodes bucketed by height (build order within a height); O(nodes) for
  // long records, whose chunk chain makes H ~ n / 8192
  std::vector<std::vector<int>> byh(H + 1);
  for (size_t k = 0; k < nodes.size(); ++k)
    if (nodes[k].a >= 0) byh[nodes[k].h].push_back((int)k);
  std::vector<int> starts, tri;
  int cnt = 0;
  for (int h = 1; h <= H; ++h) {
    starts.push_back(cnt);
    for (int k : byh[h]) id[k] = next++, ++cnt;
  }
  starts.push_back(cnt);
  for (int h = 1; h <= H; ++h)
    for (int k : byh[h]) {
      tri.push_back(id[k]);
      tri.push_back(id[nodes[k].a]);
      tri.push_back(id[nodes[k].b]);
    }
  plan.insert(plan.end(), starts.begin(), starts.end());
  plan.insert(plan.end(), tri.begin(), tri.end());
  return plan;
}

// Host evaluation of the plan (tests and host code).
inline double dfmi_plan_sum_host(const double* a, int n) {
  const std::vector<int> plan = dfmi_pairwise_plan(n);
  const int nl = plan[0], H = plan[1];
  const int* off = plan.data() + 2;
  const int* lvl = off + nl + 1;
  const int* tri = lvl + H + 1;
  std::vector<double> nodes(2 * nl);
  for (int t = 0; t < nl; ++t) nodes[t] = dfmi_np_leaf_sum(a + off[t], off[t + 1] - off[t]);
  for (int h = 0; h < H; ++h)
    for (int j = lvl[h]; j < lvl[h + 1]; ++j) nodes[tri[3 * j]] = nodes[tri[3 * j + 1]] + nodes[tri[3 * j + 2]];
  return nodes[nl > 1 ? 2 * nl - 2 : 0];
}
