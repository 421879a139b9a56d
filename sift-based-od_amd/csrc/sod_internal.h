// sod_internal.h -- device state of one libsod context (one GPU) and shared helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <string>
#include <vector>

#include "../../include/sod.h"

// ---------------------------------------------------------------------------------------
// Matcher geometry (see match.hip for the rationale).
//   subtile = 16 DB rows x 128 dims, stored in MFMA-fragment order: [kstep 4][lane 64][8 bf16]
//   = 4 KiB.  The same packing is used for 16-query tiles.
constexpr int kDim = 128;
constexpr int kSubRows = 16;
constexpr int kSubBytes = kSubRows * kDim * 2;   // 4096
constexpr float kPadNorm = 1.0e30f;              // ||d||^2 of padding rows: never selected
// int8 matcher, thresholds shared by the DB chunks of a query: per query {max published t2,
// max published best of the even chunks, of the odd chunks} (match_i8.hip, SOD_I8_SLOTS)
constexpr int kThrWords = 3;

// Hough
constexpr int kSigmaLutHalf = 255;               // i_sigma LUT over k = oQ - oM in [-255,255]
constexpr int kSigmaLutSize = 2 * kSigmaLutHalf + 1;

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;      // capacity in elements
  bool own = true;   // false: a view of another context's buffer (sod_db_share)
};

struct SiftWork;   // sift.hip: SIFT detect + describe workspace

// Development / test switches of one context (sod_set_option; each also read once from the
// environment variable SOD_<NAME> at sod_create).  The defaults are the measured best; the
// tests flip them to cover both sides of a choice.
// sod_results_fetch: where each array lies in the page-locked staging buffer (byte offsets)
// and the capacities it was laid out for
struct ResLayout {
  int64_t nq = 0, vcap = 0, mcap = 0, ncap = 0;   // queries, valid bins, members, post bins
  int words = 0;                                  // 64-bit words per relation row (ncap)
  bool valid = false, affine = false;             // parts staged besides the match arrays
  bool keys_only = false;                         // the valid bins' keys alone (post only)
  size_t hdr = 0, idx1 = 0, d1 = 0, d2 = 0, good = 0, vbin = 0, voff = 0, members = 0,
         means = 0, surv = 0, fvotes = 0, params = 0, alive = 0, sidx = 0, smeans = 0,
         pos = 0, ori = 0, total = 0;
};
// the host-side outputs of sod_results_fetch (decoded keys, votes, post-processing)
struct ResHost {
  std::vector<int32_t> keys, votes, bin_index, pos_off, pos_members, ori_pos_off, ori_off,
      ori_members;
  std::vector<double> orient, pose;
  int32_t n_bins = 0, n_pos = 0, n_ori = 0;
};

struct sod_opts {
  int match_qt = 0;            // int8 ring kernel query tiles per wave: 0 by query count; 2, 4, 8
  int match_pf = 0;            // its LDS prefetch distance: 0 default (1); 1, 2
  int match_pair = 0;          // its waves per query slice: 0 by query count; 1, 2 (4+ tiles)
  int hough_fused = 1;         // 0: never the one-work-group Hough kernel (parity tests)
  int select_multi = 0;        // 1: small windows take the multi-kernel selection too
  int sift_stream_mask = -1;   // -1: only the lone image's slot CU-masked; 0 none; 2 all
  int sift_sort_max = -2;      // -2: kSortMax; lower: the rank path for shorter lists (tests)
  int sift_desc_range_max = -1;   // -1: kDescSide; lower limits the ranged enumeration (tests)
  int sift_layer_split = -1;   // -1: every big octave splits its top layers onto the side stream
  int sift_side_mask = 1;      // 0: the side stream on all CUs
  int sift_fork2 = 0;          // 1: the second fork event before the small-octave chain
  int sift_early_desc = 1;     // 0: descriptors after the sort, of the final list
  int sift_direct = 1;         // 0: a lone image's results copied after the sync
  int sift_eager_rank = 0;     // 1: the rank-path launches always enqueued with the sort
  int affine_fma = 0;          // remove_outliers' np.matmul(M, X): 1 fma(m1, x, m2 y), 2 fma(m2, y, m1 x) (the
                               // host numpy's dgemv on an FMA CPU; set by the Python layer)
  int debug_sync = 0;          // 1: stderr trace of long stream waits and stream re-creation
  int trig_exact = -1;         // -1: the probe decides (sod_host_trig_matches_device); 0: the
                               // fallback forced -- boundary guard + host exact-means redo armed
                               // as on a host whose libm differs (parity tests of that path);
                               // 1: refused unless the probe agrees
};

struct sod_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  int num_cus = 256;
  int num_xcds = 1;             // hipDeviceAttributeNumberOfXccs
  bool gfx950 = false;
  // CUs the matcher kernel may use / the other stages run on (sod_set_cu_reserve)
  int match_cus() const { return num_cus - reserved_cus; }
  int tail_cus() const { return reserved_cus ? reserved_cus : num_cus; }
  int impl = 1;                 // matcher: 1 = int8 MFMA 16x16x64 (default), 2 = int8 32x32x32 (match_i8.hip), 0 = bf16 (match.hip)
  sod_opts opt;                 // sod_set_option
  bool last_timed = false;      // the last matcher launch recorded begin / end events
  int mkernel = 0;              // impl 1's kernel shape (sod_match_set_kernel): 0 = by query count,
                                // 1 = LDS ring (match_i8.hip; the only shape since round 6)

  // ---- database (keypoints replicated, descriptors = shard) ----
  int64_t n_total = 0;          // keypoints in the whole DB
  int32_t n_images = 0;
  DevBuf<float> mx, my, mang;
  DevBuf<int32_t> moct, mimg;
  DevBuf<double> cent;          // [n_images*2]
  DevBuf<int32_t> isize;        // [n_images*2]
  int64_t n_shard = 0;          // descriptor rows held here
  int64_t row_offset = 0;       // global index of shard row 0
  int64_t nsub = 0;             // 16-row subtiles (padded)
  DevBuf<uint8_t> dbpack;       // nsub * 4096 bytes
  DevBuf<float> dn;             // nsub * 16

  // ---- query ----
  int32_t nq = 0;
  int32_t nqt = 0;              // query tiles (16 queries; 32 for impl 2)
  DevBuf<uint8_t> qpack;        // nqt * 4096
  DevBuf<float> qn;             // nqt * 16
  DevBuf<float> qx, qy, qang;
  DevBuf<int32_t> qoct;
  // batch of query images: image of each query, (h, w) per image;
  // the bin key space is n_qimg x nbins (image-major), 0 = one image
  int32_t n_qimg = 0;
  DevBuf<int32_t> qimg;         // [nq]
  DevBuf<int32_t> qshape;       // [n_qimg * 2] (h, w)
  std::vector<int32_t> qoff_h, qshape_h;
  int64_t nbins1 = 0;           // bins of one image (nbins = nbins1 * max(1, n_qimg))
  DevBuf<int32_t> hist_rng;     // per query chunk: first / last bin slab it can touch
  DevBuf<int32_t> bwh;          // per valid bin: query image (w, h) for the affine tolerance
  int32_t win0 = 0, winn = -1;  // query window of the Hough / select / affine stages
                                // (-1 = all queries): one query image of a batch
  DevBuf<uint8_t> stage_u8;     // upload staging for descriptors
  DevBuf<float> stage_f32;

  // ---- matcher outputs ----
  int split = 1;                // DB splits (chunks) of the current launch
  DevBuf<float> pd1, pd2;       // [split * nq_pad]
  DevBuf<int32_t> pidx;
  DevBuf<float> cd1, cd2;       // merged (this shard / after allgather: global)  [nq_pad]
  DevBuf<int32_t> cidx;
  DevBuf<int32_t> gthr;         // matcher: prefilter thresholds shared by the DB chunks
  int64_t gthr_n = 0;           //   words of one slot ([slot][words][nq_pad]); reset by the merge
  DevBuf<float> gd1, gd2;       // allgather landing [nranks * nq_pad]
  DevBuf<int32_t> gidx;
  DevBuf<float> d1, d2;         // sqrt distances [nq]
  DevBuf<int32_t> idx1;         // [nq]
  DevBuf<uint8_t> good;         // [nq]
  DevBuf<uint32_t> flags;       // [0]=invalid descriptor count, [1]=max dn bits, [2]=max qn bits
  bool matched = false, ratio_done = false;
  bool matches_given = false;   // the matches came from sod_matches_set (no distances)
  // sod_pipeline_enqueue: the ratio its final merge applies in the same kernel (-1 = none),
  // and the ratio that merge applied (valid only while ratio_fused_valid: the last merge
  // fused it), which sod_ratio_enqueue then skips
  double fuse_ratio = -1.0, ratio_fused = 0.0;
  bool ratio_fused_valid = false;

  // ---- hough ----
  int32_t bins[4] = {0, 0, 0, 0};
  int64_t nbins = 0;
  int32_t qh = 0, qw = 0;
  DevBuf<int32_t> sig_lut;      // [511]
  DevBuf<uint32_t> counts;      // [nbins]
  DevBuf<uint32_t> first;       // [nbins] min vote ordinal q*16+slot
  DevBuf<uint32_t> basekey;     // [nq] ix | iy<<8 | it<<16 | is<<24
  DevBuf<uint32_t> vmask;       // [nq] 16-bit vote mask (0 = no vote)
  DevBuf<double> pose;          // [nq*4]
  DevBuf<double> pose_b;        // the other step parity of pose / msize
  DevBuf<int32_t> msize_b;
  bool houghed = false;
  bool hist_dense = true;       // counts / first hold the vote histogram (not after the fused
                                // one-image path, hough_small_kernel: sod_hist_dense builds it)
  // boundary guard (hough.hip): records of the matches whose x / y bin may depend on the
  // last ulp of cos / sin [nq * 8], their count ([0] appended by pose_kernel, [1] handed over
  // by hist_kernel); resolved once per Hough launch, before any result is read
  DevBuf<double> grec;
  DevBuf<uint32_t> gstat;
  bool guard_done = true;
  int64_t guard_flagged = 0, guard_patched = 0;   // the last launch's records / changed bins
  int64_t guard_flagged_total = 0, guard_patched_total = 0;

  // ---- select / CSR / means ----
  DevBuf<uint64_t> selstat;     // look-back words of select_kernel (one per block)
  uint32_t sel_epoch = 0;       // select_kernel call count: tags the look-back words
  DevBuf<unsigned long long> selticket;   // select_kernel block tickets (never reset)
  uint64_t sel_tickets = 0;     // tickets drawn by the launches enqueued so far
  DevBuf<uint32_t> scal;        // device scalars: [0]=V, [1]=total members, [2]=B (all bins)
  DevBuf<uint32_t> vbin;        // [vmax] linear bin id, first-touch order
  DevBuf<int64_t> voff;         // [vmax+1]
  DevBuf<int32_t> members;      // [mmax] query index
  DevBuf<double> means;         // [vmax*6]
  DevBuf<uint32_t> scal_b;      // the other step parity of scal / voff / members / means
  DevBuf<int64_t> voff_b;
  DevBuf<int32_t> members_b;
  DevBuf<double> means_b;
  DevBuf<uint32_t> vidx;        // [nbins] bin -> valid index (0xFFFFFFFF otherwise)
  DevBuf<uint32_t> cursor;      // [vmax] member fill cursors
  DevBuf<int32_t> msize;        // [nq][2] model image (w, h) of a voting query's match
  DevBuf<double> rtab;          // [mmax] 1/(n+1) for the running means
  DevBuf<uint32_t> allbin;      // [bmax] all occupied bins, first-touch order
  int64_t vmax = 0, mmax = 0;
  int32_t vote_thr = 0;
  bool selected = false;
  bool gathered = false;        // amx / amy / aqx / aqy / aisig already hold the members' points
  bool means_deferred = false;  // the fused path's PoseBin means are not launched yet
  DevBuf<uint32_t> vfirst_s;    // hough_small_kernel: first voting query of valid bins past LDS

  // ---- affine ----
  DevBuf<float> amx, amy, aqx, aqy;  // per-member points [mmax]
  DevBuf<int32_t> aisig;        // per-bin i_sigma [vmax]
  DevBuf<uint8_t> surv;         // [vmax]
  DevBuf<int32_t> fvotes;       // [vmax]
  DevBuf<double> params;        // [vmax*6]
  DevBuf<uint8_t> alive;        // [mmax]
  bool affined = false;
  int32_t aff_qw = 0, aff_qh = 0, aff_thr = 0;   // the last sod_affine_enqueue's arguments
  double aff_xf = 0.0, aff_yf = 0.0;             // (a guard re-run repeats it)

  // ---- post-processing (post.hip) ----
  DevBuf<double> post_m;        // [n*6] bin means
  DevBuf<uint64_t> post_pos, post_ori;   // [n * ceil(n/64)] relation bitmasks
  DevBuf<int32_t> post_img;     // [n] query image of each bin (image batches)

  // ---- results staging (sod_results_fetch) ----
  uint8_t* hres = nullptr;      // page-locked host buffer the staging kernel writes into
  size_t hres_n = 0;
  ResHost res;                  // host-side outputs (decoded keys, votes, post-processing)
  // staged results still current: set by a staging pipeline enqueue or a fetch; every API
  // call that can change results bumps res_epoch (set_dev, the SIFT query hand-over)
  uint64_t res_epoch = 0, staged_epoch = ~0ull;
  int staged_parts = 0;
  ResLayout staged_L;

  // ---- SIFT on the device (sift.hip) ----
  SiftWork* sift = nullptr;

  // ---- comm ----
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  // blocks per collective the communicator was created with (ncclConfig_t.maxCTAs at
  // sod_comm_init under a CU split, 0 = RCCL's default): the split needs every block of a
  // collective resident on the reserved CUs at once (sod_set_cu_reserve checks it)
  int comm_max_channels = 0;

  // ---- DB sharing (sod_db_share): a source counts the contexts that alias its DB buffers
  // and refuses DB writes while any does; a sharer detaches (drops its views) before any DB
  // write of its own and when it is destroyed
  sod_ctx* db_src = nullptr;
  std::vector<sod_ctx*> db_sharers;

  // ---- side stream: PoseBin means run beside the affine verification ----
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  bool side_pending = false;    // main stream has not yet waited for the side work
  // per-step buffer sets read by the PoseBin means on the side stream (pose, msize: Hough;
  // scal, voff, members, means: select) are double-buffered, so the next step's kernels
  // overwrite the other set instead of waiting for the means; a set is reused only after
  // the means that read it (ev_hread / ev_sread of that parity) has finished
  int hpar = 0, spar = 0;
  hipEvent_t ev_hread[2] = {nullptr, nullptr}, ev_sread[2] = {nullptr, nullptr};
  // id of the means launch that last read a set (0 = none) and the newest id the main
  // stream has already waited for: one wait covers both sets of a step
  uint64_t hread_id[2] = {0, 0}, sread_id[2] = {0, 0}, means_id = 0, means_waited = 0;

  // ---- matcher stream (sod_match_set_overlap): the match kernel runs there and waits only
  // for the last input upload (ev_inputs) and for the merge that last read its partial-result
  // slot (two slots alternate: ev_merged[slot])
  // Optionally two matcher streams, one per partial-result slot (mstream: slot 0, mstream2:
  // slot 1), so launch k+1's work-groups take the CUs launch k's finished work-groups leave
  // instead of waiting for its slowest one (sod_set_matcher_streams; mtwo)
  hipStream_t mstream = nullptr, mstream2 = nullptr;
  bool mtwo = false;
  hipEvent_t ev_inputs = nullptr, ev_merged[2] = {nullptr, nullptr};
  hipEvent_t ev_matched = nullptr, ev_matched1 = nullptr;   // untimed completion, per slot
  hipEvent_t ev_matched_p = nullptr;   // the last matcher launch's completion event
  hipEvent_t ev_done[2] = {nullptr, nullptr};   // each slot's last matcher-stream completion
  hipStream_t mstream_of(int slot) const { return mtwo && slot ? mstream2 : mstream; }
  bool stage_timing = false;  // sod_set_stage_timing: events around the tail stages (off by
                              // default: each is a marker packet that delays the next kernel)
  bool post_exact = true;     // sod_set_post_exact: survivors' x / y means redone with glibc
                              // (only while !trig_exact)
  // the device's cos / sin (glibc_trig.h) equal the host's libm bit for bit (checked once per
  // process, sod_host_trig_matches_device): poses, bins and PoseBin means are the reference's
  // without the boundary guard's host redo or the exact-means redo, which stay armed otherwise
  bool trig_exact = false;
  bool trig_probe = false;    // the probe's own answer (opt.trig_exact may force the fallback)
  // sod_exact_xy_means: bin list + record offsets, the pose records, their pinned host copy
  DevBuf<int32_t> xr_idx;
  DevBuf<double> xr_rec;
  double* xr_host = nullptr;
  size_t xr_host_n = 0;
  bool overlap = false;
  bool mk_main = true;        // the last matcher launch went on the context stream (idle, no split)
  bool merge_norec[2] = {false, false};   // a slot's last merge released it without an event
  // sod_set_match_timing: begin/end events of every match_stride-th int8 matcher launch
  // (0: none); mlaunch counts the launches since the last setting
  int match_stride = 0;
  int64_t mlaunch = 0;
  // sod_set_cu_reserve: the top `reserved_cus` CU-mask bits (cu_reserve per XCD, mask bit i
  // is on XCD i % 8) run the context / side streams; the matcher stream gets the rest
  int cu_reserve = 0;
  int reserved_cus = 0;
  int64_t host_wait_ns = 0;     // host time blocked in enqueue calls on the slot wait
  int pslot = 0;                // partial-result slot of the last matcher launch
  int64_t pslot_n = 0;          // its size (elements per array)

  // ---- timing ----
  // per-stage device time of the last step (sod_last_stage_ms): begin / end events recorded
  // on the context stream around each stage's own launches, so host work and waits between
  // two calls (a host exchange, the other ranks) are not counted; segments of one stage add
  // up; a step starts at sod_match_enqueue / sod_matches_set
  static constexpr int kSegs = 24;
  hipEvent_t seg_ev[kSegs][2] = {};
  int seg_stage[kSegs] = {};
  int nseg = 0;
  bool seg_open = false;   // the last begin mark was recorded (not dropped at kSegs)
  hipEvent_t ev[8] = {};
  // begin/end events of the last kMatchRing matcher launches (sod_match_times), so the
  // kernel is timed inside a pipelined run, not only in isolated launches
  static constexpr int kMatchRing = 64;
  hipEvent_t mev[kMatchRing][2] = {};
  int64_t nmatch = 0;
  float last_ms[6] = {0, 0, 0, 0, 0, 0};
};

// Host wait for a stream: poll it for up to kSpinUs, then block.  A blocking
// hipStreamSynchronize returned ~20-30 us after the last kernel of a short step had ended
// (one query image: 0.20 ms of latency for a 0.14 ms device span, rocprofv3 HIP-API trace);
// polling returns within a query's cost of the end.  Longer waits (C3's 3.7 ms matcher)
// fall back to the blocking call after the spin.
constexpr int kSpinUs = 400;
// live contexts whose "debug_sync" option is on (diagnostics only; counted, so one context
// switching it off does not turn it off for another)
inline std::atomic<int> sod_debug_sync{0};
inline hipError_t sod_stream_sync(hipStream_t s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return hipSuccess;
    if (q != hipErrorNotReady) return q;
    (void)hipGetLastError();   // hipErrorNotReady is an answer, not an error
    if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSpinUs)) break;
  }
  if (sod_debug_sync) {   // diagnostics (sod_set_option "debug_sync"): which stream a long wait is on
    for (int k = 0; k < 50000; ++k) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) return hipSuccess;
      if (q != hipErrorNotReady) return q;
      (void)hipGetLastError();
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    std::fprintf(stderr, "sod: stream %p still busy after ~5 s of queries; blocking sync\n", (void*)s);
    const hipError_t e = hipStreamSynchronize(s);
    std::fprintf(stderr, "sod: stream %p blocking sync returned %d\n", (void*)s, (int)e);
    return e;
  }
  return hipStreamSynchronize(s);
}

// Blocking wait for a stream that is about to be destroyed (or whose buffers are about to be
// freed): hipStreamSynchronize, never the polling sod_stream_sync.  A CU-masked stream that
// sod_stream_sync had found idle (hipStreamQuery) and that was then destroyed hung in
// hipStreamDestroy (round 4, sod_set_cu_reserve(1 -> 0) after overlapped pipelines, about one
// run in three); the blocking synchronize before the destroy is what round 3 did, and never
// hung.
inline hipError_t sod_stream_drain(hipStream_t s) { return hipStreamSynchronize(s); }

// error helpers ---------------------------------------------------------------------------
int sod_fail(sod_ctx* ctx, int code, const std::string& msg);
#define SOD_HIP(ctx, call)                                                          \
  do {                                                                              \
    hipError_t e_ = (call);                                                         \
    if (e_ != hipSuccess)                                                           \
      return sod_fail((ctx), SOD_EHIP, std::string(#call) + ": " + hipGetErrorString(e_) + \
                      " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")");              \
  } while (0)
#define SOD_TRY(x)          \
  do {                      \
    int r_ = (x);           \
    if (r_ != SOD_OK) return r_; \
  } while (0)

template <typename T>
int sod_reserve(sod_ctx* ctx, DevBuf<T>& b, size_t n) {
  if (n == 0) n = 1;
  if (b.n >= n) return SOD_OK;
  if (b.p && b.own) (void)hipFree(b.p);
  b.p = nullptr;
  b.n = 0;
  b.own = true;
  hipError_t e = hipMalloc((void**)&b.p, n * sizeof(T));
  if (e != hipSuccess) {
    b.p = nullptr;
    return sod_fail(ctx, SOD_ENOMEM, "hipMalloc(" + std::to_string(n * sizeof(T)) + " B): " +
                                          hipGetErrorString(e));
  }
  b.n = n;
  return SOD_OK;
}
template <typename T>
void sod_release(DevBuf<T>& b) {
  if (b.p && b.own) (void)hipFree(b.p);
  b.p = nullptr;
  b.n = 0;
  b.own = true;
}
template <typename T>
void sod_view(DevBuf<T>& dst, const DevBuf<T>& src) {   // non-owning alias
  sod_release(dst);
  dst.p = src.p;
  dst.n = src.n;
  dst.own = false;
}

// kernel launchers implemented in the .hip files ----------------------------------------
// the query window the Hough-side stages work on (query batching)
inline int64_t sod_win_n(const sod_ctx* ctx) { return ctx->winn < 0 ? ctx->nq : ctx->winn; }
inline int64_t sod_win0(const sod_ctx* ctx) { return ctx->winn < 0 ? 0 : ctx->win0; }

// queries covered by the packed query tiles (tile height depends on the matcher)
inline int64_t sod_nq_pad(const sod_ctx* ctx) { return (int64_t)ctx->nqt * (ctx->impl == 2 ? 32 : kSubRows); }
int launch_pack_db(sod_ctx* ctx, const void* dsrc, int dtype, int64_t n);
int launch_pack_queries(sod_ctx* ctx, const void* dsrc, int dtype, int32_t nq);
// stage segments (api.hip): kStage* ids; mark(begin) ... mark(end) around a stage's launches
enum { kStageMatch = 0, kStageMerge = 1, kStageHough = 2, kStageSelect = 3, kStageAffine = 4,
       kStageAllreduce = 5, kStageAllgather = 6, kStages = 7 };
int sod_stage_mark(sod_ctx* ctx, int stage, bool end);
int launch_match(sod_ctx* ctx);
int launch_find_rows(sod_ctx* ctx, const float* flo, const float* fhi, const int32_t* excl,
                     int32_t* found);
int launch_find_rows_i8(sod_ctx* ctx, const float* flo, const float* fhi, const int32_t* excl,
                        int32_t* found);
int launch_pack_i8(sod_ctx* ctx, const void* dsrc, int dtype, int64_t n, bool db);
int launch_match_i8(sod_ctx* ctx);
// shared-threshold words per query of one partial-result slot
int64_t sod_thr_words(const sod_ctx* ctx);
// matcher-input writers call these around their writes; the match launchers around the
// kernel (see sod_ctx::mstream)
int sod_inputs_begin(sod_ctx* ctx);
int sod_inputs_end(sod_ctx* ctx);
// the next matcher launch: its stream and partial-result slot (n elements per array);
// then, after the kernel, the context stream's wait, and after the merge the slot release
// record the begin (end = 0) or end (end = 1) event of a matcher launch on stream ks
int sod_match_mark(sod_ctx* ctx, hipStream_t ks, int end);
int sod_match_stream_begin(sod_ctx* ctx, int64_t n, hipStream_t* ks, float** d1, int32_t** idx,
                           float** d2);
int sod_match_stream_end(sod_ctx* ctx, hipEvent_t done = nullptr);
int sod_match_events(sod_ctx* ctx, hipEvent_t* begin, hipEvent_t* end);
int sod_partials_merged(sod_ctx* ctx);
int launch_merge(sod_ctx* ctx, const float* d1, const int32_t* idx, const float* d2,
                 int nparts, int64_t stride, int32_t* reset = nullptr, bool final_merge = false);
int launch_ratio(sod_ctx* ctx, double ratio);
int launch_hough(sod_ctx* ctx, int64_t own_lo, int64_t own_hi);
// boundary guard: redo the listed matches' x / y bins with glibc cos / sin and, when one
// changes, the histogram and every stage after it (call before reading any Hough result)
int sod_guard_resolve(sod_ctx* ctx);
int launch_select(sod_ctx* ctx, int32_t thr, bool may_defer_means = false);
// the fused one-image Hough + select + gather (hough.hip hough_small_kernel) and the lazy
// dense histogram after it
bool sod_hough_small_ok(const sod_ctx* ctx);
int launch_hough_small(sod_ctx* ctx, int32_t thr);
int sod_hist_dense(sod_ctx* ctx);
// the fused path's PoseBin means run with its affine launch; alone when anything else comes
// first (every entry point but sod_affine_enqueue)
int sod_means_flush(sod_ctx* ctx);
int launch_means_affine(sod_ctx* ctx, int32_t qw, int32_t qh, double xf, double yf, int32_t thr);
int launch_all_bins(sod_ctx* ctx);
int launch_affine_gather(sod_ctx* ctx);
int launch_affine(sod_ctx* ctx, int64_t nbins_dev_scalar_or_host, bool count_on_device,
                  const int64_t* offsets, const float* mx, const float* my, const float* qx,
                  const float* qy, const int32_t* isig, int32_t qw, int32_t qh,
                  const int32_t* bwh /* per-bin (w, h) or nullptr */, double xf,
                  double yf, int32_t thr, int32_t max_iter, const double* params_in,
                  uint8_t* surv, int32_t* votes, double* params, uint8_t* alive,
                  const uint32_t* dev_count);
int launch_bin_index_batch(sod_ctx* ctx, int64_t n, const double* pose, int32_t* idx);
int launch_pose_batch(sod_ctx* ctx, int64_t n, const float* mx, const float* my,
                      const float* ma, const int32_t* mo, const float* qx, const float* qy,
                      const float* qa, const int32_t* qo, const double* cx, const double* cy,
                      double* pose, int32_t* idx, double* grec, uint32_t* gstat);
// host side of the boundary guard: one record's x, y (glibc cos / sin) and x / y bin index
void sod_guard_host_pose(const double rec[8], const int32_t bins[4], double* x, double* y,
                         int32_t* ix, int32_t* iy);
int sod_build_sigma_lut(sod_ctx* ctx, int32_t bins_sigma);
int sod_exact_xy_means(sod_ctx* ctx, const int32_t* vbin, int nb, double* means6);
// results staging (post.hip): the kernels that write every result into ctx->hres (layout
// L; post = the survivors' compaction and relations too), and the host post-processing
// over the staged survivors
int launch_results_stage(sod_ctx* ctx, const ResLayout& L, bool post);
int sod_post_staged(sod_ctx* ctx, const ResLayout& L, ResHost& r);
bool sod_host_trig_matches_device();
int launch_glibc_sincos(sod_ctx* ctx, int64_t n, const double* x, double* s, double* c);
void sod_sift_free(sod_ctx* ctx);
