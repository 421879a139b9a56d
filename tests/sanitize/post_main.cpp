// Host-only harness of post.hip's walk (post_walk.h) for the sanitizer build
// (tests/test_sanitize.py): reads n PoseBin means [n][6] (f64) from argv[1],
// computes both pair relations with post_word and runs post_walk / write_post exactly as
// sod_postprocess does on the host, and writes the outputs to argv[2] as a sequence of
// (int64 count, raw array) records: pos_off, pos_members, ori_pos_off, ori_off, ori_members
// (int32), final_orientation, final_pose (f64).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../sift-based-od_amd/csrc/post_walk.h"

using namespace sod_post;

template <typename T>
static void put(FILE* f, const std::vector<T>& v) {
  const int64_t n = (int64_t)v.size();
  std::fwrite(&n, 8, 1, f);
  if (n) std::fwrite(v.data(), sizeof(T), v.size(), f);
}

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  FILE* in = std::fopen(argv[1], "rb");
  if (!in) return 2;
  int64_t n = 0;
  if (std::fread(&n, 8, 1, in) != 1 || n < 0 || n > (1 << 20)) return 2;
  std::vector<double> m((size_t)n * 6);
  if (n && std::fread(m.data(), 8, m.size(), in) != m.size()) return 2;
  std::fclose(in);
  const int words = (int)((n + 63) / 64);
  std::vector<uint64_t> pos((size_t)n * words), ori((size_t)n * words);
  for (int64_t t = 0; t < n * words; ++t)
    post_word((int)n, words, m.data(), nullptr, t, pos.data(), ori.data());
  PostOut o;
  if (n) post_walk((int)n, words, pos.data(), ori.data(), m.data(), o);
  int32_t np_ = 0, no = 0;
  write_post(o, &np_, nullptr, nullptr, &no, nullptr, nullptr, nullptr, nullptr, nullptr);
  std::vector<int32_t> pos_off(np_ + 1), ori_pos_off(np_ + 1), ori_off(no + 1);
  std::vector<int32_t> pos_members(n), ori_members(n);
  std::vector<double> orient(np_), pose((size_t)np_ * 6);
  write_post(o, &np_, pos_off.data(), pos_members.data(), &no, ori_pos_off.data(),
             ori_off.data(), ori_members.data(), orient.data(), pose.data());
  FILE* out = std::fopen(argv[2], "wb");
  if (!out) return 2;
  put(out, pos_off);
  put(out, pos_members);
  put(out, ori_pos_off);
  put(out, ori_off);
  put(out, ori_members);
  put(out, orient);
  put(out, pose);
  std::fclose(out);
  return 0;
}
