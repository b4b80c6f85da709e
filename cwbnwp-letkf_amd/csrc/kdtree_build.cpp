// kdtree_build.cpp — host construction of the localisation k-d trees, flattened for the GPU.
//
// Builds exactly the tree Kennel's kdtree2 builds for the reference (module_kdtree2.f90):
//   kdtree2_create           :598-680  (rearrange = .true., sort = .false.)
//   build_tree_for_range     :696-834  bucket_size 12 (:505), exact median m=(l+u)/2,
//                                      cut dimension = first max spread of the approximate box
//   select_on_coordinate     :897-929  (its exact swap sequence: the permutation decides
//                                      the order in which the search returns neighbours)
//   spread_in_coordinate     :931-979
// so that the GPU search returns the same neighbours in the same order, including when
// max_lz_pts truncates the list (Q4).  Nodes are emitted in pre-order (root = 0).
#include "cwbl_internal.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace cwbl {
namespace {

constexpr int kBucket = 12;

struct Builder {
  const float *data;   // (3,n) normalised
  int dim;
  std::vector<int> &ind;
  std::vector<TreeNode> &nodes;

  void spread(int c, int l, int u, float &lo, float &hi) const {
    float smin = data[3 * ind[l] + c], smax = smin;
    for (int i = l + 1; i <= u; ++i) {
      const float v = data[3 * ind[i] + c];
      smin = std::min(smin, v);
      smax = std::max(smax, v);
    }
    lo = smin;
    hi = smax;
  }

  void select(int c, int k, int li, int ui) {
    int l = li, u = ui;
    while (l < u) {
      const float pivot = data[3 * ind[l] + c];
      int m = l;
      for (int i = l + 1; i <= u; ++i)
        if (data[3 * ind[i] + c] < pivot) std::swap(ind[++m], ind[i]);
      std::swap(ind[l], ind[m]);
      if (m <= k) l = m + 1;
      if (m >= k) u = m - 1;
    }
  }

  int build(int l, int u, int parent) {
    if (u < l) return -1;
    const int me = static_cast<int>(nodes.size());
    nodes.push_back(TreeNode{});
    nodes[me].left = nodes[me].right = -1;
    nodes[me].l = l;
    nodes[me].u = u;
    for (int i = 0; i < 3; ++i) nodes[me].lo[i] = nodes[me].hi[i] = 0.0f;
    if (u - l <= kBucket) {
      for (int i = 0; i < dim; ++i) spread(i, l, u, nodes[me].lo[i], nodes[me].hi[i]);
      nodes[me].cut_dim = -1;
      nodes[me].cut_val = nodes[me].cut_val_left = nodes[me].cut_val_right = 0.0f;
      return me;
    }
    // approximate box: recompute only the parent's cut dimension (:761-773)
    for (int i = 0; i < dim; ++i) {
      if (parent < 0 || i == nodes[parent].cut_dim) {
        spread(i, l, u, nodes[me].lo[i], nodes[me].hi[i]);
      } else {
        nodes[me].lo[i] = nodes[parent].lo[i];
        nodes[me].hi[i] = nodes[parent].hi[i];
      }
    }
    int c = 0;
    float best = nodes[me].hi[0] - nodes[me].lo[0];
    for (int i = 1; i < dim; ++i) {
      const float s = nodes[me].hi[i] - nodes[me].lo[i];
      if (s > best) { best = s; c = i; }
    }
    const int m = (l + u) / 2;
    select(c, m, l, u);
    nodes[me].cut_dim = c;
    const int left = build(l, m, me);
    const int right = build(m + 1, u, me);
    TreeNode &res = nodes[me];
    const TreeNode &L = nodes[left], &R = nodes[right];
    res.left = left;
    res.right = right;
    res.cut_val_right = R.lo[c];
    res.cut_val_left = L.hi[c];
    res.cut_val = (res.cut_val_left + res.cut_val_right) / 2.0f;
    for (int i = 0; i < dim; ++i) {
      res.hi[i] = std::max(L.hi[i], R.hi[i]);
      res.lo[i] = std::min(L.lo[i], R.lo[i]);
    }
    return me;
  }
};

}  // namespace

void build_kdtree(const float *xyz3, int n, int dim, HostTree &out) {
  out.dim = dim;
  out.n = n;
  out.nodes.clear();
  out.ind.resize(n);
  for (int j = 0; j < n; ++j) out.ind[j] = j;
  if (n > 0) {
    out.nodes.reserve(static_cast<size_t>(2 * (n / (kBucket / 2) + 1)));
    Builder b{xyz3, dim, out.ind, out.nodes};
    b.build(0, n - 1, -1);
  }
  out.rdata.assign(static_cast<size_t>(4) * (n > 0 ? n : 1), 0.0f);
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d)
      out.rdata[4 * static_cast<size_t>(i) + d] = d < dim ? xyz3[3 * out.ind[i] + d] : 0.0f;
}

void build_bins(const HostTree &t, int dim, float r, HostBins &out, int div) {
  const int n = t.n;
  out = HostBins{};
  // bounds over the finite coordinates (a non-finite point is never within r: d2 <= r2 fails
  // for NaN or inf, so it may sit in any cell; it goes to cell 0)
  float lo[3] = {0.0f, 0.0f, 0.0f}, hi[3] = {0.0f, 0.0f, 0.0f};
  bool seen[3] = {false, false, false};
  for (int i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) {
      const float v = t.rdata[4 * (size_t)i + c];
      if (!std::isfinite(v)) continue;
      lo[c] = seen[c] ? std::min(lo[c], v) : v;
      hi[c] = seen[c] ? std::max(hi[c], v) : v;
      seen[c] = true;
    }
  if (dim < 3) lo[2] = hi[2] = 0.0f;
  float h = r / (float)std::max(div, 1);  // cell side r / div (div 2: the ball's box spans ~5 cells)
  long long nb[3];
  for (;;) {
    for (int c = 0; c < 3; ++c)
      nb[c] = 1 + (long long)std::min(std::floor(((double)hi[c] - (double)lo[c]) / h), 4194304.0);
    if (nb[0] * nb[1] * nb[2] <= (1LL << 22)) break;
    h *= 1.25f;
  }
  out.x0 = lo[0]; out.y0 = lo[1]; out.z0 = lo[2];
  out.binv = 1.0f / h;
  out.nbx = (int)nb[0]; out.nby = (int)nb[1]; out.nbz = (int)nb[2];
  // the kernel's cell arithmetic, in fp32 (monotone, so the query's conservative box
  // brackets every cell a point within r can fall in)
  auto cell = [&](int c, float v) {
    const float f = (v - (c == 0 ? out.x0 : c == 1 ? out.y0 : out.z0)) * out.binv;
    if (!std::isfinite(f)) return 0LL;
    return (long long)std::min<float>(std::max(std::floor(f), 0.0f), (float)(nb[c] - 1));
  };
  const long long ncell = nb[0] * nb[1] * nb[2];
  std::vector<long long> cid(n);
  out.start.assign(ncell + 1, 0);
  for (int i = 0; i < n; ++i) {
    const float *d = &t.rdata[4 * (size_t)i];
    const bool fin = std::isfinite(d[0]) && std::isfinite(d[1]) && (dim < 3 || std::isfinite(d[2]));
    const long long cz = dim == 3 ? cell(2, d[2]) : 0;
    cid[i] = fin ? cell(0, d[0]) + nb[0] * (cell(1, d[1]) + nb[1] * cz) : 0;
    ++out.start[cid[i] + 1];
  }
  for (long long c = 0; c < ncell; ++c) out.start[c + 1] += out.start[c];
  std::vector<int> fill(out.start.begin(), out.start.end() - 1);
  out.xyzs.assign(4 * (size_t)n, 0.0f);
  for (int i = 0; i < n; ++i) {  // slot order within a cell
    const int p = fill[cid[i]]++;
    std::memcpy(&out.xyzs[4 * (size_t)p], &t.rdata[4 * (size_t)i], 3 * sizeof(float));
    std::memcpy(&out.xyzs[4 * (size_t)p + 3], &i, sizeof(int));
  }
}

}  // namespace cwbl
