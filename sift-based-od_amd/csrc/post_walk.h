// post_walk.h -- the host side of post.hip (PostProcessing.py:4-112) as plain C++: the
// pair relation of one 64-bin word (the same code, and with -ffp-contract=off the same bits,
// on the device and the host), the reference's DFS visit order over the relation bitmasks,
// the dominant orientation and the final pose.  No HIP types: tests/sanitize/post_main.cpp
// builds it alone under ASan + UBSan.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

#ifdef __HIPCC__
#define SOD_POST_HD __host__ __device__ inline
#else
#define SOD_POST_HD inline
#endif

namespace sod_post {

constexpr double kRadToDeg = 180.0 / 3.141592653589793;   // CPython math.degrees factor

// word t = (row i, 64-column word) of the position / orientation relations over n bins'
// means m[n*6]; the same code (and, -ffp-contract=off, the same bits) on the host and the
// device
SOD_POST_HD void post_word(int n, int words, const double* m, const int32_t* img, int64_t t,
                           uint64_t* pos, uint64_t* ori) {
  const int i = (int)(t / words), wd = (int)(t % words);
  const double xi = m[6 * i], yi = m[6 * i + 1], ai = m[6 * i + 2], si = m[6 * i + 3];
  const double txi = m[6 * i + 4] * si / 4, tyi = m[6 * i + 5] * si / 4;
  uint64_t pb = 0, ob = 0;
  for (int k = 0; k < 64; ++k) {
    const int j = wd * 64 + k;
    if (j >= n) break;
    if (j == i || (img && img[j] != img[i])) continue;   // batch: one image's bins only
    const double xj = m[6 * j], yj = m[6 * j + 1], aj = m[6 * j + 2], sj = m[6 * j + 3];
    const double dx = fabs(xi - xj), dy = fabs(yi - yj);
    const bool close = dx <= txi && dy <= tyi && dx <= m[6 * j + 4] * sj / 4 &&
                       dy <= m[6 * j + 5] * sj / 4;
    if (close) pb |= 1ull << k;
    if (fabs((ai - aj) * kRadToDeg) <= 1) ob |= 1ull << k;
  }
  pos[t] = pb;
  ori[t] = ob;
}

// Components over indices 0..n-1 in the order of the reference's recursive dfs started
// from every unseen index in order; adj_next(node, from, seen) returns the node's next
// unseen neighbour >= from (neighbours ascending) or -1.
template <typename Adj>
void dfs_components(int n, Adj adj_next, std::vector<std::vector<int>>& comps) {
  std::vector<char> seen((size_t)n, 0);
  std::vector<std::pair<int, int>> stack;
  for (int i = 0; i < n; ++i) {
    if (seen[i]) continue;
    comps.emplace_back();
    auto& comp = comps.back();
    seen[i] = 1;
    comp.push_back(i);
    stack.assign(1, {i, 0});
    while (!stack.empty()) {
      auto& top = stack.back();
      const int nb = adj_next(top.first, top.second, seen);   // next unseen neighbour >= cursor
      if (nb < 0) {
        stack.pop_back();
        continue;
      }
      top.second = nb + 1;
      seen[nb] = 1;
      comp.push_back(nb);
      stack.push_back({nb, 0});
    }
  }
}

struct PostOut {
  std::vector<std::vector<int>> pos;                 // global ids, DFS preorder
  std::vector<std::vector<std::vector<int>>> ori;    // per position cluster
  std::vector<double> orient;                        // final orientation per cluster
  std::vector<double> pose;                          // 6 per cluster
};

// the host walk over the two relation bitmasks (rows of `words` words): position clusters,
// orientation clusters inside each, their dominant orientation and the final pose
inline int post_walk(int32_t n, int words, const uint64_t* pos, const uint64_t* ori,
              const double* means_host, PostOut& out) {
  // position clusters: neighbours of a node = set bits of its row, ascending
  auto pos_next = [&](int node, int from, const std::vector<char>& seen) -> int {
    const uint64_t* row = pos + (size_t)node * words;
    for (int w = from >> 6; w < words; ++w) {
      uint64_t bits = row[w];
      if (w == (from >> 6)) bits &= ~0ull << (from & 63);
      while (bits) {
        const int j = w * 64 + __builtin_ctzll(bits);
        if (!seen[j]) return j;
        bits &= bits - 1;
      }
    }
    return -1;
  };
  dfs_components(n, pos_next, out.pos);

  for (const auto& cl : out.pos) {
    // orientation clusters in the cluster's own indexing (local k -> global cl[k])
    const int nc = (int)cl.size();
    auto ori_next = [&](int k, int from, const std::vector<char>& seen) -> int {
      const uint64_t* row = ori + (size_t)cl[k] * words;
      for (int m = from; m < nc; ++m) {
        if (m == k || seen[m]) continue;
        const int g = cl[m];
        if ((row[g >> 6] >> (g & 63)) & 1) return m;
      }
      return -1;
    };
    std::vector<std::vector<int>> local;
    dfs_components(nc, ori_next, local);
    out.ori.emplace_back();
    for (auto& comp : local) {
      for (auto& k : comp) k = cl[k];
      out.ori.back().push_back(std::move(comp));
    }
    // find_max_orientation: the last largest cluster's mean angle, summed in order
    size_t max_vote = 0;
    double final_o = 0;
    for (const auto& comp : out.ori.back()) {
      if (comp.size() >= max_vote) {
        max_vote = comp.size();
        double acc = 0;
        for (int g : comp) acc += means_host[6 * g + 2];
        final_o = acc / (double)comp.size();
      }
    }
    out.orient.push_back(final_o);
    // get_final_pose
    double mx = 0, my = 0, ms = 0, min_area = INFINITY, mw = 0, mh = 0;
    for (int g : cl) {
      const double* r = means_host + 6 * g;
      mx += r[0];
      my += r[1];
      ms += r[3];
      const double area = (r[4] * r[3]) * (r[5] * r[3]);
      if (area < min_area) {
        min_area = area;
        mw = r[4];
        mh = r[5];
      }
    }
    const double len = (double)cl.size();
    const double p[6] = {mx / len, my / len, final_o, ms / len, mw, mh};
    out.pose.insert(out.pose.end(), p, p + 6);
  }
  return 0;
}

inline int write_post(const PostOut& o, int32_t* n_pos, int32_t* pos_off, int32_t* pos_members,
               int32_t* n_ori, int32_t* ori_pos_off, int32_t* ori_off, int32_t* ori_members,
               double* final_orientation, double* final_pose) {
  int32_t np_ = 0, no = 0, pm = 0, om = 0;
  if (pos_off) pos_off[0] = 0;
  if (ori_pos_off) ori_pos_off[0] = 0;
  if (ori_off) ori_off[0] = 0;
  for (size_t c = 0; c < o.pos.size(); ++c) {
    for (int g : o.pos[c])
      if (pos_members) pos_members[pm++] = g;
      else ++pm;
    ++np_;
    if (pos_off) pos_off[np_] = pm;
    for (const auto& comp : o.ori[c]) {
      for (int g : comp)
        if (ori_members) ori_members[om++] = g;
        else ++om;
      ++no;
      if (ori_off) ori_off[no] = om;
    }
    if (ori_pos_off) ori_pos_off[np_] = no;
    if (final_orientation) final_orientation[c] = o.orient[c];
    if (final_pose) std::memcpy(final_pose + 6 * c, o.pose.data() + 6 * c, 6 * sizeof(double));
  }
  if (n_pos) *n_pos = np_;
  if (n_ori) *n_ori = no;
  return 0;
}

}  // namespace sod_post
