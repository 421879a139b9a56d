// post.hip -- SURVEY §8(f) row 1: post-processing of the verified pose bins
// (PostProcessing.py:4-112, driven by main.py:159-168).
//
//   group_position      bins a, b are neighbours when |dx| <= w*s/4 and |dy| <= h*s/4 for
//                       the means of a AND of b (PostProcessing.py:18-28); position
//                       clusters are the components in recursive-DFS preorder from every
//                       unseen bin in list order, neighbours ascending (:4-11, :32-36)
//   group_orientation   inside each position cluster, neighbours when
//                       |degrees(theta_a - theta_b)| <= 1 (:39-62), DFS in the cluster's
//                       own (preorder) indexing
//   find_max_orientation  mean angle of the LAST largest orientation cluster (:64-81)
//   get_final_pose      mean centroid, that orientation, mean scale, img_size of the FIRST
//                       bin of minimum (w*s)*(h*s) (:85-112)
//
// The O(n^2) part -- both neighbour relations over all pairs -- is one device kernel
// writing two n x n bitmasks (bit j of row i, 64 per word); the components need the
// reference's exact visit order (it fixes every later sum and tie), so the DFS walks the
// bitmask rows on the host (set bits = ascending neighbours), O(n^2 / 64) word reads.
// Compiled with -ffp-contract=off: the comparisons are the reference's Python floats.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "sod_internal.h"
#include "post_walk.h"

namespace {

using namespace sod_post;

// one thread per (row i, 64-column word): bits of the position / orientation relations
__global__ void post_adjacency_kernel(int n, int words, const double* __restrict__ m,
                                      const int32_t* __restrict__ img,
                                      uint64_t* __restrict__ pos, uint64_t* __restrict__ ori) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n * words) return;
  post_word(n, words, m, img, t, pos, ori);
}

// up to this many bins the relations are computed on the host: n^2 / 2 pair tests take
// less than a device round trip (H2D means, launch, D2H bitmasks, wait: ~40-50 us)
constexpr int kHostPostMax = 64;


int run_post(sod_ctx* ctx, int32_t n, const double* means_host, const int32_t* img_host,
             PostOut& out) {
  if (n <= 0) return SOD_OK;
  const int words = (n + 63) / 64;
  if (n <= kHostPostMax) {   // small: the relations on the host
    std::vector<uint64_t> pos((size_t)n * words), ori((size_t)n * words);
    for (int64_t t = 0; t < (int64_t)n * words; ++t)
      post_word(n, words, means_host, img_host, t, pos.data(), ori.data());
    return post_walk(n, words, pos.data(), ori.data(), means_host, out);
  }
  DevBuf<double>& dm = ctx->post_m;
  DevBuf<uint64_t>& dpos = ctx->post_pos;
  DevBuf<uint64_t>& dori = ctx->post_ori;
  int rc = sod_reserve(ctx, dm, (size_t)n * 6);
  if (rc == SOD_OK && img_host) rc = sod_reserve(ctx, ctx->post_img, (size_t)n);
  if (rc == SOD_OK) rc = sod_reserve(ctx, dpos, (size_t)n * words);
  if (rc == SOD_OK) rc = sod_reserve(ctx, dori, (size_t)n * words);
  std::vector<uint64_t> pos((size_t)n * words), ori((size_t)n * words);
  if (rc == SOD_OK) {
    hipError_t e = hipMemcpyAsync(dm.p, means_host, (size_t)n * 6 * sizeof(double),
                                  hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess && img_host)
      e = hipMemcpyAsync(ctx->post_img.p, img_host, (size_t)n * 4, hipMemcpyHostToDevice,
                         ctx->stream);
    const int64_t threads = (int64_t)n * words;
    if (e == hipSuccess) {
      hipLaunchKernelGGL(post_adjacency_kernel, dim3((unsigned)((threads + 255) / 256)),
                         dim3(256), 0, ctx->stream, n, words, dm.p,
                         img_host ? ctx->post_img.p : nullptr, dpos.p, dori.p);
      e = hipGetLastError();
    }
    if (e == hipSuccess)
      e = hipMemcpyAsync(pos.data(), dpos.p, pos.size() * 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(ori.data(), dori.p, ori.size() * 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = sod_stream_sync(ctx->stream);
    if (e != hipSuccess) rc = sod_fail(ctx, SOD_EHIP, std::string("post-processing: ") + hipGetErrorString(e));
  }
  if (rc != SOD_OK) return rc;
  return post_walk(n, words, pos.data(), ori.data(), means_host, out);
}

// ---- results staging (sod_results_fetch) ----------------------------------------------
struct StageArgs {
  uint8_t* h;   // page-locked host buffer (device-visible)
  ResLayout L;
  const int32_t* idx1;
  const float *d1, *d2;
  const uint8_t* good;
  const uint32_t* vbin;
  const int64_t* voff;
  const int32_t* members;
  const double* means;
  const uint8_t* surv;
  const int32_t* fvotes;
  const double* params;
  const uint8_t* alive;
  const uint32_t* scal;   // [0] valid bins, [1] members
  int selected, affined, n_qimg;
  int alone;   // results_post_kernel without a pack launch before it
  int64_t nbins1;
};

template <typename T>
__device__ __forceinline__ void stage_copy(uint8_t* h, size_t off, const T* src, int64_t n,
                                           int64_t gt, int64_t gs) {
  T* dst = reinterpret_cast<T*>(h + off);
  for (int64_t i = gt; i < n; i += gs) dst[i] = src[i];
}

// every array of the last pipeline into the host buffer, at the sizes the device holds
// (thread gt of gs)
__device__ __forceinline__ void results_pack(const StageArgs& a, int64_t gt, int64_t gs) {
  const int64_t V = a.L.vcap ? min<int64_t>(a.scal[0], a.L.vcap) : 0;
  const int64_t M = a.L.vcap ? min<int64_t>(a.scal[1], a.L.mcap) : 0;
  if (gt == 0) {
    int64_t* hdr = reinterpret_cast<int64_t*>(a.h + a.L.hdr);
    hdr[0] = V;
    hdr[1] = M;
  }
  const int64_t nq = a.L.nq;
  stage_copy(a.h, a.L.idx1, a.idx1, nq, gt, gs);
  stage_copy(a.h, a.L.d1, a.d1, nq, gt, gs);
  stage_copy(a.h, a.L.d2, a.d2, nq, gt, gs);
  stage_copy(a.h, a.L.good, a.good, nq, gt, gs);
  if (a.L.valid || a.L.keys_only) stage_copy(a.h, a.L.vbin, a.vbin, V, gt, gs);
  if (a.L.valid) {
    stage_copy(a.h, a.L.voff, a.voff, V + 1, gt, gs);
    stage_copy(a.h, a.L.members, a.members, M, gt, gs);
    stage_copy(a.h, a.L.means, a.means, 6 * V, gt, gs);
  }
  if (!a.L.affine) return;
  stage_copy(a.h, a.L.surv, a.surv, V, gt, gs);
  stage_copy(a.h, a.L.fvotes, a.fvotes, V, gt, gs);
  stage_copy(a.h, a.L.params, a.params, 6 * V, gt, gs);
  stage_copy(a.h, a.L.alive, a.alive, M, gt, gs);
}

// post-processing input on the device: the survivors (affine survivors, else every valid
// bin) in list order -- their valid index and means into the host buffer, hdr[2] = their
// count -- and, for at most ncap of them, both relation bitmasks (post_adjacency_kernel's,
// rows of ceil(n/64) words); one work-group of 1024 threads
__device__ __forceinline__ void results_post(const StageArgs& a, double* __restrict__ sm,
                                             int32_t* __restrict__ simg) {
  __shared__ int wtot[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t V = min<int64_t>(a.scal[0], a.L.vcap);
  int32_t* sidx = reinterpret_cast<int32_t*>(a.h + a.L.sidx);
  double* smeans = reinterpret_cast<double*>(a.h + a.L.smeans);
  if (a.alone) {   // no pack launch: the header and the bins' keys (batch images) from here
    if (tid == 0) {
      reinterpret_cast<int64_t*>(a.h + a.L.hdr)[0] = V;
      reinterpret_cast<int64_t*>(a.h + a.L.hdr)[1] = min<int64_t>(a.scal[1], a.L.mcap);
    }
    stage_copy(a.h, a.L.vbin, a.vbin, V, tid, 1024);
  }
  int base = 0;
  for (int64_t c0 = 0; c0 < V; c0 += 1024) {
    const int64_t v = c0 + tid;
    const bool keep = v < V && (!a.affined || a.surv[v]);
    const uint64_t bal = __ballot(keep);
    const int pre = __popcll(bal & ((1ull << lane) - 1));
    if (lane == 0) wtot[wv] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wv; ++w) off += wtot[w];
    int tot = 0;
    for (int w = 0; w < 16; ++w) tot += wtot[w];
    if (keep) {
      const int k = off + pre;
      sidx[k] = (int32_t)v;
      for (int f = 0; f < 6; ++f) smeans[6 * (int64_t)k + f] = a.means[6 * v + f];
      if (k < a.L.ncap) {
        for (int f = 0; f < 6; ++f) sm[6 * k + f] = a.means[6 * v + f];
        simg[k] = a.n_qimg ? (int32_t)(a.vbin[v] / a.nbins1) : 0;
      }
    }
    base += tot;
    __syncthreads();   // wtot reused
  }
  const int n = base;
  if (tid == 0) reinterpret_cast<int64_t*>(a.h + a.L.hdr)[2] = n;
  __threadfence_block();
  __syncthreads();
  if (n > a.L.ncap) return;   // the host runs post_adjacency_kernel on them instead
  const int words = (n + 63) / 64;
  uint64_t* pos = reinterpret_cast<uint64_t*>(a.h + a.L.pos);
  uint64_t* ori = reinterpret_cast<uint64_t*>(a.h + a.L.ori);
  for (int64_t t = tid; t < (int64_t)n * words; t += 1024)
    post_word(n, words, sm, a.n_qimg ? simg : nullptr, t, pos, ori);
}

// the results staging as ONE launch: work-group 0 stages the post-processing input (when
// `post`), the others pack the arrays -- independent writes to the host buffer, so the two
// run side by side (one image: 11 -> ~6 us of the step's tail, one launch fewer)
__global__ __launch_bounds__(1024) void results_stage_kernel(StageArgs a, double* __restrict__ sm,
                                                             int32_t* __restrict__ simg, int post) {
  if (post && blockIdx.x == 0) {
    results_post(a, sm, simg);
    return;
  }
  const int64_t b = blockIdx.x - (post ? 1 : 0);
  results_pack(a, b * blockDim.x + threadIdx.x, (int64_t)(gridDim.x - (post ? 1 : 0)) * blockDim.x);
}

}  // namespace

int launch_results_stage(sod_ctx* ctx, const ResLayout& L, bool post) {
  StageArgs a;
  a.h = ctx->hres;
  a.L = L;
  a.idx1 = ctx->idx1.p;
  a.d1 = ctx->d1.p;
  a.d2 = ctx->d2.p;
  a.good = ctx->good.p;
  a.vbin = ctx->vbin.p;
  a.voff = ctx->voff.p;
  a.members = ctx->members.p;
  a.means = ctx->means.p;
  a.surv = ctx->surv.p;
  a.fvotes = ctx->fvotes.p;
  a.params = ctx->params.p;
  a.alive = ctx->alive.p;
  a.scal = ctx->scal.p;
  a.selected = ctx->selected ? 1 : 0;
  a.affined = ctx->affined ? 1 : 0;
  a.n_qimg = ctx->n_qimg;
  a.nbins1 = std::max<int64_t>(1, ctx->nbins1);
  // post-processing alone (Context.postprocess): one launch
  a.alone = post && ctx->selected && !L.nq && !L.valid && !L.affine;
  const int do_post = post && ctx->selected ? 1 : 0;
  unsigned pack_blocks = 0;
  if (!a.alone) {
    const int64_t work = std::max<int64_t>({L.nq, 6 * L.vcap, L.mcap, 1});
    pack_blocks = (unsigned)std::min<int64_t>(64, (work + 1023) / 1024);
  }
  if (do_post) {
    SOD_TRY(sod_reserve(ctx, ctx->post_m, (size_t)std::max<int64_t>(1, L.ncap) * 6));
    SOD_TRY(sod_reserve(ctx, ctx->post_img, (size_t)std::max<int64_t>(1, L.ncap)));
  }
  if (pack_blocks + do_post == 0) return SOD_OK;
  hipLaunchKernelGGL(results_stage_kernel, dim3(pack_blocks + do_post), dim3(1024), 0, ctx->stream,
                     a, ctx->post_m.p, ctx->post_img.p, do_post);
  SOD_HIP(ctx, hipGetLastError());
  return SOD_OK;
}

// the post-processing outputs from the staged survivors: the relations the device wrote
// (or, past ncap survivors or with the host-libm means, post_adjacency_kernel again)
int sod_post_staged(sod_ctx* ctx, const ResLayout& L, ResHost& r) {
  const int64_t* hdr = reinterpret_cast<const int64_t*>(ctx->hres + L.hdr);
  const int32_t n = (int32_t)hdr[2];
  const int32_t* sidx = reinterpret_cast<const int32_t*>(ctx->hres + L.sidx);
  const double* smeans = reinterpret_cast<const double*>(ctx->hres + L.smeans);
  r.n_bins = n;
  r.bin_index.assign(sidx, sidx + n);
  PostOut o;
  const bool exact_redo = ctx->post_exact && !ctx->trig_exact && n;
  if (exact_redo || n > L.ncap) {
    std::vector<double> sel(smeans, smeans + 6 * (size_t)n);
    std::vector<int32_t> img;
    if (ctx->n_qimg) {
      const uint32_t* vb = reinterpret_cast<const uint32_t*>(ctx->hres + L.vbin);
      for (int32_t k = 0; k < n; ++k) img.push_back((int32_t)(vb[sidx[k]] / ctx->nbins1));
    }
    if (exact_redo) SOD_TRY(sod_exact_xy_means(ctx, sidx, n, sel.data()));
    SOD_TRY(run_post(ctx, n, sel.data(), img.empty() ? nullptr : img.data(), o));
  } else {
    SOD_TRY(post_walk(n, (n + 63) / 64, reinterpret_cast<const uint64_t*>(ctx->hres + L.pos),
                      reinterpret_cast<const uint64_t*>(ctx->hres + L.ori), smeans, o));
  }
  const size_t n1 = (size_t)n + 1;
  r.pos_off.assign(n1, 0);
  r.pos_members.assign(std::max<size_t>(1, n), 0);
  r.ori_pos_off.assign(n1, 0);
  r.ori_off.assign(n1, 0);
  r.ori_members.assign(std::max<size_t>(1, n), 0);
  r.orient.assign(std::max<size_t>(1, n), 0.0);
  r.pose.assign(6 * std::max<size_t>(1, n), 0.0);
  return write_post(o, &r.n_pos, r.pos_off.data(), r.pos_members.data(), &r.n_ori,
                    r.ori_pos_off.data(), r.ori_off.data(), r.ori_members.data(), r.orient.data(),
                    r.pose.data());
}

extern "C" {

int sod_post_batch(sod_ctx* ctx, int32_t n, const double* means, int32_t* n_pos,
                   int32_t* pos_off, int32_t* pos_members, int32_t* n_ori,
                   int32_t* ori_pos_off, int32_t* ori_off, int32_t* ori_members,
                   double* final_orientation, double* final_pose) {
  if (!ctx) return SOD_EINVAL;
  SOD_HIP(ctx, hipSetDevice(ctx->device));
  if (n < 0 || (n > 0 && !means)) return sod_fail(ctx, SOD_EINVAL, "bad post-processing input");
  if (n > (1 << 20)) return sod_fail(ctx, SOD_EINVAL, "too many bins for post-processing");
  PostOut o;
  SOD_TRY(run_post(ctx, n, means, nullptr, o));
  return write_post(o, n_pos, pos_off, pos_members, n_ori, ori_pos_off, ori_off, ori_members,
                    final_orientation, final_pose);
}

int sod_exact_means(sod_ctx* ctx, int32_t nb, const int32_t* vbin, double* xy) {
  if (!ctx) return SOD_EINVAL;
  if (nb < 0 || (nb > 0 && (!vbin || !xy))) return sod_fail(ctx, SOD_EINVAL, "bad exact-means input");
  std::vector<double> m6((size_t)nb * 6, 0.0);
  SOD_TRY(sod_exact_xy_means(ctx, vbin, nb, m6.data()));
  for (int32_t i = 0; i < nb; ++i) {
    xy[2 * i] = m6[6 * (size_t)i];
    xy[2 * i + 1] = m6[6 * (size_t)i + 1];
  }
  return SOD_OK;
}

int sod_set_post_exact(sod_ctx* ctx, int on) {
  if (!ctx) return SOD_EINVAL;
  if (on != 0 && on != 1) return sod_fail(ctx, SOD_EINVAL, "post exact must be 0 or 1");
  ctx->post_exact = on != 0;
  return SOD_OK;
}

int sod_postprocess(sod_ctx* ctx, int32_t* n_bins, int32_t* bin_index, int32_t* n_pos,
                    int32_t* pos_off, int32_t* pos_members, int32_t* n_ori,
                    int32_t* ori_pos_off, int32_t* ori_off, int32_t* ori_members,
                    double* final_orientation, double* final_pose) {
  int64_t V, M;
  SOD_TRY(sod_valid_counts(ctx, &V, &M));   // joins the side stream (PoseBin means)
  std::vector<double> means((size_t)V * 6);
  std::vector<uint8_t> surv((size_t)V, 1);
  if (V) {
    SOD_HIP(ctx, hipMemcpyAsync(means.data(), ctx->means.p, means.size() * 8,
                                hipMemcpyDeviceToHost, ctx->stream));
    if (ctx->affined)   // main.py:155: post_process runs on the bins that survived
      SOD_HIP(ctx, hipMemcpyAsync(surv.data(), ctx->surv.p, (size_t)V, hipMemcpyDeviceToHost,
                                  ctx->stream));
    SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  }
  std::vector<uint32_t> lin;
  if (ctx->n_qimg && V) {   // batch of query images: post-process each image's bins apart
    lin.resize((size_t)V);
    SOD_HIP(ctx, hipMemcpyAsync(lin.data(), ctx->vbin.p, (size_t)V * 4, hipMemcpyDeviceToHost,
                                ctx->stream));
    SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  }
  std::vector<double> sel;
  std::vector<int32_t> idx, img;
  for (int64_t v = 0; v < V; ++v)
    if (surv[(size_t)v]) {
      idx.push_back((int32_t)v);
      sel.insert(sel.end(), means.begin() + 6 * v, means.begin() + 6 * v + 6);
      if (!lin.empty()) img.push_back((int32_t)(lin[(size_t)v] / ctx->nbins1));
    }
  const int32_t n = (int32_t)idx.size();
  if (n_bins) *n_bins = n;
  if (bin_index && n) std::memcpy(bin_index, idx.data(), (size_t)n * sizeof(int32_t));
  // the survivors' x / y means as the reference computes them (glibc cos / sin per member,
  // sod_exact_xy_means): the position relation's <= thresholds (PostProcessing.py:24-28) and
  // the final pose then see the reference's values bit for bit
  // (with the device's glibc cos / sin the device means are those values already)
  if (ctx->post_exact && !ctx->trig_exact && n)
    SOD_TRY(sod_exact_xy_means(ctx, idx.data(), n, sel.data()));
  PostOut o;
  SOD_TRY(run_post(ctx, n, sel.data(), img.empty() ? nullptr : img.data(), o));
  return write_post(o, n_pos, pos_off, pos_members, n_ori, ori_pos_off, ori_off, ori_members,
                    final_orientation, final_pose);
}

}  // extern "C"
