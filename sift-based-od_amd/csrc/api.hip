// api.hip -- extern "C" entry points of libsod.so (declared in include/sod.h).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cctype>
#include <cstring>
#include <vector>

#include "sod_internal.h"

int sod_fail(sod_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

namespace {
thread_local std::string g_err;  // errors before a ctx exists

// Every entry point starts here; by default it also joins the side stream (PoseBin means),
// so whatever comes next on the main stream sees their results.
int set_dev(sod_ctx* ctx, bool join = true, bool flush = true) {
  if (!ctx) return SOD_EINVAL;
  ++ctx->res_epoch;   // any call may change results: staged ones are no longer current
  SOD_HIP(ctx, hipSetDevice(ctx->device));
  if (flush) SOD_TRY(sod_means_flush(ctx));
  if (join && ctx->side_pending) {
    SOD_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
    ctx->side_pending = false;
    ctx->means_waited = ctx->means_id;   // ev_join follows the newest means launch
  }
  return SOD_OK;
}

template <typename T>
int upload(sod_ctx* ctx, DevBuf<T>& b, const T* src, size_t n) {
  SOD_TRY(sod_reserve(ctx, b, n));
  if (n) SOD_HIP(ctx, hipMemcpyAsync(b.p, src, n * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
  return SOD_OK;
}

template <typename T>
int download(sod_ctx* ctx, T* dst, const T* src, size_t n) {
  if (n && dst) SOD_HIP(ctx, hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyDeviceToHost, ctx->stream));
  return SOD_OK;
}

int check_bins(sod_ctx* ctx, const int32_t bins[4]) {
  for (int i = 0; i < 4; ++i)
    if (bins[i] < 1 || bins[i] > 255)
      return sod_fail(ctx, SOD_EINVAL, "bins must be in [1,255] per axis");
  const int64_t nb = (int64_t)bins[0] * bins[1] * bins[2] * bins[3];
  const bool changed_sigma = bins[3] != ctx->bins[3] || !ctx->sig_lut.p;
  std::memcpy(ctx->bins, bins, sizeof(ctx->bins));
  ctx->nbins = nb;
  ctx->nbins1 = nb;
  if (changed_sigma) SOD_TRY(sod_build_sigma_lut(ctx, bins[3]));
  return SOD_OK;
}

int flags_reset(sod_ctx* ctx) {
  SOD_TRY(sod_reserve(ctx, ctx->flags, 4));
  return SOD_OK;
}
}  // namespace

// ---- matcher stream protocol (sod_match_set_overlap) -----------------------------------
// Writers of the matcher's inputs (packed DB / queries and their norm words) first wait for
// the last matcher kernel, then mark the inputs ready; the matcher kernel waits for the
// inputs and for the previous merge of its partial results, and the context stream waits
// for the kernel before merging.
// cross-stream wait, skipped when the host already sees the event complete (a satisfied
// wait still costs the matcher stream a barrier packet between two back-to-back launches)
static int wait_unless_done(sod_ctx* ctx, hipStream_t s, hipEvent_t ev) {
  const hipError_t q = hipEventQuery(ev);
  if (q == hipSuccess) return SOD_OK;
  if (q != hipErrorNotReady) return sod_fail(ctx, SOD_EHIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
  (void)hipGetLastError();   // hipErrorNotReady is an answer, not an error
  SOD_HIP(ctx, hipStreamWaitEvent(s, ev, 0));
  return SOD_OK;
}
int sod_inputs_begin(sod_ctx* ctx) {
  // every matcher launch still reading the inputs: the last one of each slot (two may be in
  // flight on the two matcher streams); context-stream launches are ordered already
  for (int x = 0; x < 2; ++x)
    if (ctx->ev_done[x]) SOD_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_done[x], 0));
  return SOD_OK;
}
int sod_inputs_end(sod_ctx* ctx) {
  SOD_HIP(ctx, hipEventRecord(ctx->ev_inputs, ctx->stream));
  return SOD_OK;
}
// the slot wait below, with the host time it blocks accumulated (sod_host_wait_ns): what part
// of an enqueue call is waiting for the device rather than host work
static int slot_wait(sod_ctx* ctx, hipEvent_t ev) {
  const hipError_t q = hipEventQuery(ev);
  if (q == hipSuccess) return SOD_OK;
  (void)hipGetLastError();
  const auto t0 = std::chrono::steady_clock::now();
  SOD_HIP(ctx, hipEventSynchronize(ev));
  ctx->host_wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(
                           std::chrono::steady_clock::now() - t0).count();
  return SOD_OK;
}
static bool stream_idle(hipStream_t s) {
  const hipError_t q = hipStreamQuery(s);
  if (q == hipSuccess) return true;
  (void)hipGetLastError();   // hipErrorNotReady (or an error the next call reports)
  return false;
}
int sod_match_stream_begin(sod_ctx* ctx, int64_t n, hipStream_t* ks, float** d1, int32_t** idx,
                           float** d2) {
  const int nslot = ctx->overlap ? 2 : 1;
  if (ctx->pd1.n < (size_t)(nslot * n)) {   // growing: no kernel or merge may still use them
    SOD_HIP(ctx, sod_stream_sync(ctx->mstream));
    SOD_HIP(ctx, sod_stream_sync(ctx->mstream2));
    SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  }
  SOD_TRY(sod_reserve(ctx, ctx->pd1, (size_t)(nslot * n)));
  SOD_TRY(sod_reserve(ctx, ctx->pd2, (size_t)(nslot * n)));
  SOD_TRY(sod_reserve(ctx, ctx->pidx, (size_t)(nslot * n)));
  const bool resized = n != ctx->pslot_n;
  ctx->pslot = ctx->overlap ? ctx->pslot ^ 1 : 0;
  ctx->pslot_n = n;
  *d1 = ctx->pd1.p + ctx->pslot * n;
  *d2 = ctx->pd2.p + ctx->pslot * n;
  *idx = ctx->pidx.p + ctx->pslot * n;
  // The matcher stream buys overlap with an earlier step's tail.  Without the CU split and with
  // both streams idle there is nothing to overlap: the kernel goes on the context stream, so
  // the merge after it needs no cross-stream wait (~10 us on the one-image path, where the
  // whole step is ~0.1 ms).  The slot protocol below is unchanged either way.
  ctx->mk_main = !ctx->overlap ||
                 (ctx->cu_reserve == 0 && stream_idle(ctx->stream) && stream_idle(ctx->mstream) &&
                  stream_idle(ctx->mstream2));
  if (ctx->mk_main) {
    *ks = ctx->stream;
    if (ctx->overlap) SOD_TRY(slot_wait(ctx, ctx->ev_merged[ctx->pslot]));
    return SOD_OK;
  }
  *ks = ctx->mstream_of(ctx->pslot);
  // merges that ran on the context stream right after a context-stream matcher released
  // their slot without an event (sod_partials_merged): mark them now
  for (int x = 0; x < 2; ++x)
    if (ctx->merge_norec[x]) {
      SOD_HIP(ctx, hipEventRecord(ctx->ev_merged[x], ctx->stream));
      ctx->merge_norec[x] = false;
    }
  SOD_TRY(wait_unless_done(ctx, *ks, ctx->ev_inputs));
  // the slot's previous merge (two launches back) must be done before the kernel rewrites
  // it: the host waits for it here rather than the matcher stream (a satisfied barrier packet
  // between two back-to-back matcher launches costs ~6 us per launch, C2 0.166 vs 0.160 ms per
  // step); it bounds a context to two matcher launches in flight, and the merge it waits for
  // ran right after the launch before the previous one, so the wait is normally over already
  SOD_TRY(slot_wait(ctx, ctx->ev_merged[ctx->pslot]));
  // a new slot size moves the slots' boundaries: the other slot's last merge must be done too
  if (resized) SOD_TRY(wait_unless_done(ctx, *ks, ctx->ev_merged[ctx->pslot ^ 1]));
  return SOD_OK;
}
int sod_match_mark(sod_ctx* ctx, hipStream_t ks, int end) {
  hipEvent_t& e = ctx->mev[ctx->nmatch % sod_ctx::kMatchRing][end];
  if (!e) SOD_HIP(ctx, hipEventCreate(&e));
  SOD_HIP(ctx, hipEventRecord(e, ks));
  if (end) {
    ++ctx->nmatch;
    ctx->last_timed = true;
  }
  return SOD_OK;
}
// begin / end events of the next matcher launch, recorded by the launch itself
// (hipExtLaunchKernelGGL: timestamps in the dispatch, no marker packets around the kernel)
int sod_match_events(sod_ctx* ctx, hipEvent_t* begin, hipEvent_t* end) {
  const bool timed = ctx->match_stride > 0 && ctx->mlaunch % ctx->match_stride == 0;
  ++ctx->mlaunch;
  ctx->last_timed = timed;
  if (!timed) {
    // untimed launch: no begin event (a dispatch that records one delays the next kernel of
    // its stream); a matcher-stream launch still records its completion, which the context
    // stream waits for -- by the dispatch itself: against a marker packet after the kernel,
    // one image 0.0694 vs 0.0722 ms per step, C2 0.1203 vs 0.1245 (three A/B rounds on one
    // box, tools/gpu_endev_ab.sh)
    *begin = nullptr;
    *end = ctx->mk_main ? nullptr : (ctx->pslot ? ctx->ev_matched1 : ctx->ev_matched);
    return SOD_OK;
  }
  hipEvent_t* e = ctx->mev[ctx->nmatch % sod_ctx::kMatchRing];
  for (int i = 0; i < 2; ++i)
    if (!e[i]) SOD_HIP(ctx, hipEventCreate(&e[i]));
  *begin = e[0];
  *end = e[1];
  ++ctx->nmatch;
  return SOD_OK;
}
int sod_match_stream_end(sod_ctx* ctx, hipEvent_t done) {
  const hipStream_t ks = ctx->mk_main ? ctx->stream : ctx->mstream_of(ctx->pslot);
  if (ctx->mk_main) ctx->ev_done[0] = ctx->ev_done[1] = nullptr;   // stream order from here on
  if (!done && ctx->mk_main) {   // stream order covers every reader: no event
    ctx->ev_matched_p = nullptr;
    return SOD_OK;
  }
  if (!done) {
    hipEvent_t ev = ctx->pslot ? ctx->ev_matched1 : ctx->ev_matched;
    SOD_HIP(ctx, hipEventRecord(ev, ks));
    done = ev;
  }
  ctx->ev_matched_p = done;
  if (!ctx->mk_main) ctx->ev_done[ctx->pslot] = done;
  if (!ctx->mk_main) SOD_HIP(ctx, hipStreamWaitEvent(ctx->stream, done, 0));
  return SOD_OK;
}

// the partial-result slot's release after its merge (recorded on the context stream by
// sod_partials_merged); after a context-stream matcher none -- an event there delays the
// stream's next kernel ~5 us -- and a later matcher-stream launch records it then
// (sod_match_stream_begin)
int sod_partials_merged(sod_ctx* ctx) {
  ctx->merge_norec[ctx->pslot] = ctx->mk_main && ctx->overlap;
  if (!ctx->mk_main) SOD_HIP(ctx, hipEventRecord(ctx->ev_merged[ctx->pslot], ctx->stream));
  return SOD_OK;
}

// One matcher stream for both partial-result slots (1, the default) or one per slot (2):
// consecutive launches then overlap at their boundary -- the next launch's work-groups start
// on the CUs the previous one's finished work-groups leave.  Measured (r04 ms1, one box): C2
// 0.1124 vs 0.1206 ms per step, C3 3.696 vs 3.745, one image 0.0749 vs 0.0678 (worse); a
// launch's begin/end events then span the overlap, so the per-launch time is not the kernel's.
int sod_set_matcher_streams(sod_ctx* ctx, int n) {
  SOD_TRY(set_dev(ctx));
  if (n != 1 && n != 2) return sod_fail(ctx, SOD_EINVAL, "matcher streams must be 1 or 2");
  SOD_HIP(ctx, sod_stream_sync(ctx->mstream));
  SOD_HIP(ctx, sod_stream_sync(ctx->mstream2));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->mtwo = n == 2;
  ctx->ev_done[0] = ctx->ev_done[1] = nullptr;
  return SOD_OK;
}

int sod_set_match_timing(sod_ctx* ctx, int on) {
  SOD_TRY(set_dev(ctx));
  if (on < 0 || on > 1 << 20) return sod_fail(ctx, SOD_EINVAL, "match timing stride must be in [0, 2^20]");
  ctx->match_stride = on;
  ctx->mlaunch = 0;
  return SOD_OK;
}

// ---- DB sharing bookkeeping (sod_db_share) ---------------------------------------------
// A sharer drops its views of the source's DB buffers (views are never freed by it) and
// leaves the source's list.  Its own streams must have drained any work reading them.
static void db_detach(sod_ctx* ctx) {
  sod_ctx* src = ctx->db_src;
  if (!src) return;
  auto& v = src->db_sharers;
  v.erase(std::remove(v.begin(), v.end(), ctx), v.end());
  ctx->db_src = nullptr;
  sod_release(ctx->mx); sod_release(ctx->my); sod_release(ctx->mang);
  sod_release(ctx->moct); sod_release(ctx->mimg); sod_release(ctx->cent);
  sod_release(ctx->isize); sod_release(ctx->dbpack); sod_release(ctx->dn);
  ctx->nsub = 0;
  ctx->n_total = 0;
  ctx->n_images = 0;
  ctx->n_shard = 0;
  ctx->matched = ctx->ratio_done = ctx->houghed = ctx->selected = ctx->affined = false;
}

static void drain_streams(sod_ctx* ctx) {
  if (ctx->side) (void)sod_stream_drain(ctx->side);
  if (ctx->mstream) (void)sod_stream_drain(ctx->mstream);
  if (ctx->mstream2) (void)sod_stream_drain(ctx->mstream2);
  if (ctx->stream) (void)sod_stream_drain(ctx->stream);
}

// Every DB writer calls this first: a source whose DB other contexts alias refuses (their
// matchers may be reading it on their own streams); a sharer detaches, so the write goes
// to buffers of its own and never into the source's.
static int db_writable(sod_ctx* ctx) {
  if (!ctx->db_sharers.empty())
    return sod_fail(ctx, SOD_ESTATE,
                    std::to_string(ctx->db_sharers.size()) +
                        " context(s) use this database through sod_db_share; destroy them "
                        "before changing it");
  if (ctx->db_src) {
    drain_streams(ctx);
    db_detach(ctx);
  }
  return SOD_OK;
}

// ---- stage segments (sod_last_stage_ms) ---------------------------------------------
int sod_stage_mark(sod_ctx* ctx, int stage, bool end) {
  if (!ctx->stage_timing) return SOD_OK;
  if (!end) {
    if (ctx->nseg >= sod_ctx::kSegs) {   // a step of more segments: the rest uncounted
      ctx->seg_open = false;             // (and its end mark must not move segment kSegs-1's end)
      return SOD_OK;
    }
    ctx->seg_open = true;
    hipEvent_t* e = ctx->seg_ev[ctx->nseg];
    for (int k = 0; k < 2; ++k)
      if (!e[k]) SOD_HIP(ctx, hipEventCreate(&e[k]));
    ctx->seg_stage[ctx->nseg] = stage;
    SOD_HIP(ctx, hipEventRecord(e[0], ctx->stream));
    ctx->nseg++;
  } else if (ctx->seg_open && ctx->nseg > 0 && ctx->seg_stage[ctx->nseg - 1] == stage) {
    SOD_HIP(ctx, hipEventRecord(ctx->seg_ev[ctx->nseg - 1][1], ctx->stream));
    ctx->seg_open = false;
  }
  return SOD_OK;
}

extern "C" {

int sod_abi_version(void) { return 1; }

int sod_device_count(int* n) {
  if (!n) return SOD_EINVAL;
  const hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    g_err = std::string("hipGetDeviceCount: ") + hipGetErrorString(e);
    *n = 0;
    return SOD_EHIP;
  }
  return SOD_OK;
}

namespace {
struct OptEntry {
  const char* name;
  int sod_opts::*field;
};
const OptEntry kOpts[] = {
    {"match_qt", &sod_opts::match_qt},
    {"match_pf", &sod_opts::match_pf},
    {"match_pair", &sod_opts::match_pair},
    {"hough_fused", &sod_opts::hough_fused},
    {"select_multi", &sod_opts::select_multi},
    {"sift_stream_mask", &sod_opts::sift_stream_mask},
    {"sift_sort_max", &sod_opts::sift_sort_max},
    {"sift_desc_range_max", &sod_opts::sift_desc_range_max},
    {"sift_layer_split", &sod_opts::sift_layer_split},
    {"sift_side_mask", &sod_opts::sift_side_mask},
    {"sift_fork2", &sod_opts::sift_fork2},
    {"sift_early_desc", &sod_opts::sift_early_desc},
    {"sift_direct", &sod_opts::sift_direct},
    {"sift_eager_rank", &sod_opts::sift_eager_rank},
    {"affine_fma", &sod_opts::affine_fma},
    {"debug_sync", &sod_opts::debug_sync},
    {"trig_exact", &sod_opts::trig_exact},
};
const OptEntry* find_opt(const char* name) {
  for (const OptEntry& o : kOpts)
    if (name && std::strcmp(o.name, name) == 0) return &o;
  return nullptr;
}
// SOD_<NAME> of the environment, read once at sod_create
void opts_from_env(sod_opts& op) {
  for (const OptEntry& o : kOpts) {
    std::string env = "SOD_";
    for (const char* c = o.name; *c; ++c) env += (char)std::toupper((unsigned char)*c);
    if (const char* e = std::getenv(env.c_str())) op.*(o.field) = std::atoi(e);
  }
  if (op.debug_sync) op.debug_sync = 1;
}
// ctx->trig_exact from the probe and the option (-1 auto, 0 forced fallback)
void apply_trig_opt(sod_ctx* ctx) { ctx->trig_exact = ctx->trig_probe && ctx->opt.trig_exact != 0; }
}  // namespace

int sod_set_option(sod_ctx* ctx, const char* name, int64_t value) {
  if (!ctx) return SOD_EINVAL;
  const OptEntry* o = find_opt(name);
  if (!o) return sod_fail(ctx, SOD_EINVAL, std::string("unknown option ") + (name ? name : "(null)"));
  if (value < INT32_MIN || value > INT32_MAX)
    return sod_fail(ctx, SOD_EINVAL, std::string("option ") + name + " out of the int range");
  if (o->field == &sod_opts::trig_exact) {
    if (value < -1 || value > 1)
      return sod_fail(ctx, SOD_EINVAL, "trig_exact must be -1 (auto), 0 (fallback) or 1");
    if (value == 1 && !ctx->trig_probe)
      return sod_fail(ctx, SOD_EINVAL,
                      "trig_exact 1 refused: this host's libm cos / sin differ from the device's");
  }
  if (o->field == &sod_opts::debug_sync) {
    const int on = value != 0;
    if (on != ctx->opt.debug_sync) sod_debug_sync += on ? 1 : -1;
    ctx->opt.debug_sync = on;
    return SOD_OK;
  }
  ctx->opt.*(o->field) = (int)value;
  if (o->field == &sod_opts::trig_exact) apply_trig_opt(ctx);
  return SOD_OK;
}

int sod_get_option(sod_ctx* ctx, const char* name, int64_t* value) {
  if (!ctx || !value) return SOD_EINVAL;
  const OptEntry* o = find_opt(name);
  if (!o) return sod_fail(ctx, SOD_EINVAL, std::string("unknown option ") + (name ? name : "(null)"));
  *value = ctx->opt.*(o->field);
  return SOD_OK;
}

int sod_create(int device, sod_ctx** out) {
  if (!out) return SOD_EINVAL;
  *out = nullptr;
  sod_ctx* ctx = new sod_ctx();
  ctx->device = device;
  opts_from_env(ctx->opt);
  if (ctx->opt.debug_sync) ++sod_debug_sync;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e == hipSuccess) {
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e == hipSuccess) {
      ctx->num_cus = prop.multiProcessorCount;
      ctx->gfx950 = std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
      ctx->trig_probe = sod_host_trig_matches_device();
      apply_trig_opt(ctx);
      int nx = 0;
      if (hipDeviceGetAttribute(&nx, hipDeviceAttributeNumberOfXccs, device) == hipSuccess && nx > 0)
        ctx->num_xcds = nx;
    }
  }
  for (int i = 0; i < 8 && e == hipSuccess; ++i) e = hipEventCreate(&ctx->ev[i]);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->mstream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->mstream2, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_inputs, hipEventDisableTiming);
  for (int i = 0; i < 2 && e == hipSuccess; ++i)
    e = hipEventCreateWithFlags(&ctx->ev_merged[i], hipEventDisableTiming);
  // (timing-capable: untimed matcher-stream launches record it as their dispatch's stop event)
  if (e == hipSuccess) e = hipEventCreate(&ctx->ev_matched);
  if (e == hipSuccess) e = hipEventCreate(&ctx->ev_matched1);
  if (e != hipSuccess) {
    g_err = std::string("sod_create: ") + hipGetErrorString(e);
    if (ctx->opt.debug_sync) --sod_debug_sync;
    delete ctx;
    return SOD_EHIP;
  }
  if (sod_reserve(ctx, ctx->flags, 4) != SOD_OK ||
      hipMemsetAsync(ctx->flags.p, 0, 16, ctx->stream) != hipSuccess) {
    g_err = ctx->err;
    sod_destroy(ctx);
    return SOD_ENOMEM;
  }
  *out = ctx;
  return SOD_OK;
}

void sod_destroy(sod_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->side) (void)sod_stream_drain(ctx->side);
  if (ctx->mstream) (void)sod_stream_drain(ctx->mstream);
  if (ctx->mstream2) (void)sod_stream_drain(ctx->mstream2);
  if (ctx->stream) (void)sod_stream_drain(ctx->stream);
  db_detach(ctx);
  // contexts still aliasing this DB: let their queued work finish, then drop their views
  // (they report "no database" afterwards instead of reading freed memory)
  const std::vector<sod_ctx*> sharers = ctx->db_sharers;
  for (sod_ctx* s : sharers) {
    drain_streams(s);
    db_detach(s);
  }
  (void)hipSetDevice(ctx->device);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  sod_sift_free(ctx);
  sod_release(ctx->mx); sod_release(ctx->my); sod_release(ctx->mang);
  sod_release(ctx->moct); sod_release(ctx->mimg); sod_release(ctx->cent); sod_release(ctx->isize);
  sod_release(ctx->dbpack); sod_release(ctx->dn); sod_release(ctx->qpack); sod_release(ctx->qn);
  sod_release(ctx->qx); sod_release(ctx->qy); sod_release(ctx->qang); sod_release(ctx->qoct);
  sod_release(ctx->stage_u8); sod_release(ctx->stage_f32);
  sod_release(ctx->pd1); sod_release(ctx->pd2); sod_release(ctx->pidx);
  sod_release(ctx->cd1); sod_release(ctx->cd2); sod_release(ctx->cidx); sod_release(ctx->gthr);
  sod_release(ctx->gd1); sod_release(ctx->gd2); sod_release(ctx->gidx);
  sod_release(ctx->d1); sod_release(ctx->d2); sod_release(ctx->idx1); sod_release(ctx->good);
  sod_release(ctx->flags); sod_release(ctx->sig_lut); sod_release(ctx->counts);
  sod_release(ctx->first); sod_release(ctx->basekey); sod_release(ctx->vmask);
  sod_release(ctx->pose); sod_release(ctx->selstat); sod_release(ctx->selticket); sod_release(ctx->scal); sod_release(ctx->vbin);
  sod_release(ctx->voff); sod_release(ctx->members); sod_release(ctx->means);
  sod_release(ctx->vidx); sod_release(ctx->cursor); sod_release(ctx->vfirst_s);
  sod_release(ctx->xr_idx); sod_release(ctx->xr_rec);
  if (ctx->xr_host) (void)hipHostFree(ctx->xr_host);
  ctx->xr_host = nullptr;
  if (ctx->hres) (void)hipHostFree(ctx->hres);
  ctx->hres = nullptr;
  sod_release(ctx->rtab); sod_release(ctx->msize);
  sod_release(ctx->pose_b); sod_release(ctx->msize_b); sod_release(ctx->scal_b);
  sod_release(ctx->voff_b); sod_release(ctx->members_b); sod_release(ctx->means_b);
  sod_release(ctx->allbin); sod_release(ctx->amx); sod_release(ctx->amy); sod_release(ctx->aqx);
  sod_release(ctx->aqy); sod_release(ctx->aisig); sod_release(ctx->surv);
  sod_release(ctx->fvotes); sod_release(ctx->params); sod_release(ctx->alive);
  sod_release(ctx->post_m); sod_release(ctx->post_pos); sod_release(ctx->post_ori);
  sod_release(ctx->post_img); sod_release(ctx->qimg); sod_release(ctx->qshape);
  sod_release(ctx->hist_rng); sod_release(ctx->bwh);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& pr : ctx->mev)
    for (auto& e : pr)
      if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->seg_ev)
    for (auto& x : e)
      if (x) (void)hipEventDestroy(x);
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
  for (int i = 0; i < 2; ++i) {
    if (ctx->ev_hread[i]) (void)hipEventDestroy(ctx->ev_hread[i]);
    if (ctx->ev_sread[i]) (void)hipEventDestroy(ctx->ev_sread[i]);
  }
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  if (ctx->ev_inputs) (void)hipEventDestroy(ctx->ev_inputs);
  for (auto& ev : ctx->ev_merged)
    if (ev) (void)hipEventDestroy(ev);
  if (ctx->ev_matched) (void)hipEventDestroy(ctx->ev_matched);
  if (ctx->ev_matched1) (void)hipEventDestroy(ctx->ev_matched1);
  if (ctx->mstream) (void)hipStreamDestroy(ctx->mstream);
  if (ctx->mstream2) (void)hipStreamDestroy(ctx->mstream2);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->opt.debug_sync) --sod_debug_sync;
  delete ctx;
}

const char* sod_last_error(const sod_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_err.c_str();
}

int sod_synchronize(sod_ctx* ctx) {
  SOD_TRY(set_dev(ctx));
  SOD_HIP(ctx, sod_stream_sync(ctx->mstream));
  SOD_HIP(ctx, sod_stream_sync(ctx->mstream2));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  return SOD_OK;
}

int sod_last_match_ms(sod_ctx* ctx, float* ms) {
  SOD_TRY(set_dev(ctx));
  if (!ms) return sod_fail(ctx, SOD_EINVAL, "null output");
  if (!ctx->matched) return sod_fail(ctx, SOD_ESTATE, "no matcher launch yet");
  if (!ctx->last_timed)
    return sod_fail(ctx, SOD_ESTATE, "the last matcher launch was not timed (sod_set_match_timing)");
  return sod_match_times(ctx, 1, ms);
}

int sod_match_times(sod_ctx* ctx, int n, float* ms) {
  SOD_TRY(set_dev(ctx));
  if (!ms || n < 1) return sod_fail(ctx, SOD_EINVAL, "need n >= 1 and an output array");
  if (n > sod_ctx::kMatchRing || n > ctx->nmatch)
    return sod_fail(ctx, SOD_EINVAL, "fewer matcher launches recorded than requested");
  for (int i = 0; i < n; ++i) {
    const int64_t k = ctx->nmatch - n + i;
    hipEvent_t* e = ctx->mev[k % sod_ctx::kMatchRing];
    SOD_HIP(ctx, hipEventSynchronize(e[1]));
    SOD_HIP(ctx, hipEventElapsedTime(&ms[i], e[0], e[1]));
  }
  return SOD_OK;
}

int sod_set_stage_timing(sod_ctx* ctx, int on) {
  SOD_TRY(set_dev(ctx));
  if (on != 0 && on != 1) return sod_fail(ctx, SOD_EINVAL, "stage timing must be 0 or 1");
  ctx->stage_timing = on != 0;
  return SOD_OK;
}

int sod_last_stage_ms(sod_ctx* ctx, float* ms_out, int n) {
  // [match kernel, merge + ratio, hough vote, select (+ members, means), affine, all-reduce
  //  (or the host exchange's upload), all-gather (or its upload)]: device time of each
  // stage's own launches in the last step
  SOD_TRY(set_dev(ctx));
  if (!ms_out || n < 0) return sod_fail(ctx, SOD_EINVAL, "null output");
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  float acc[kStages] = {};
  // the last matcher launch's own begin / end events (0 when that launch was not timed)
  if (ctx->matched && ctx->nmatch > 0 && ctx->last_timed) {
    hipEvent_t* m = ctx->mev[(ctx->nmatch - 1) % sod_ctx::kMatchRing];
    if (hipEventElapsedTime(&acc[kStageMatch], m[0], m[1]) != hipSuccess) {
      acc[kStageMatch] = 0.f;
      (void)hipGetLastError();   // not sticky: the next launch check must not see it
    }
  }
  for (int i = 0; i < ctx->nseg; ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ctx->seg_ev[i][0], ctx->seg_ev[i][1]) != hipSuccess) {
      ms = 0.f;
      (void)hipGetLastError();
    }
    acc[ctx->seg_stage[i]] += ms;
  }
  for (int i = 0; i < n; ++i) ms_out[i] = i < kStages ? acc[i] : 0.f;
  return SOD_OK;
}

// ---- database -------------------------------------------------------------------------
int sod_db_set_keypoints(sod_ctx* ctx, int64_t n_total, const float* x, const float* y,
                         const float* angle, const int32_t* octave, const int32_t* img,
                         int32_t n_images, const double* centroid, const int32_t* size) {
  SOD_TRY(set_dev(ctx));
  if (n_total < 0 || n_images < 1 || !x || !y || !angle || !octave || !img || !centroid || !size)
    return sod_fail(ctx, SOD_EINVAL, "sod_db_set_keypoints: bad arguments");
  SOD_TRY(db_writable(ctx));
  for (int64_t i = 0; i < n_total; ++i)
    if (img[i] < 0 || img[i] >= n_images)
      return sod_fail(ctx, SOD_EINVAL, "keypoint image id out of range");
  SOD_TRY(upload(ctx, ctx->mx, x, (size_t)n_total));
  SOD_TRY(upload(ctx, ctx->my, y, (size_t)n_total));
  SOD_TRY(upload(ctx, ctx->mang, angle, (size_t)n_total));
  SOD_TRY(upload(ctx, ctx->moct, octave, (size_t)n_total));
  SOD_TRY(upload(ctx, ctx->mimg, img, (size_t)n_total));
  SOD_TRY(upload(ctx, ctx->cent, centroid, (size_t)n_images * 2));
  SOD_TRY(upload(ctx, ctx->isize, size, (size_t)n_images * 2));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->n_total = n_total;
  ctx->n_images = n_images;
  return SOD_OK;
}

static int upload_descriptors(sod_ctx* ctx, const void* des, int dtype, int64_t n, bool db) {
  if (!des || n < 0 || (dtype != SOD_DTYPE_U8 && dtype != SOD_DTYPE_F32))
    return sod_fail(ctx, SOD_EINVAL, "bad descriptor arguments");
  const size_t elems = (size_t)n * kDim;
  const void* dsrc;
  if (dtype == SOD_DTYPE_U8) {
    SOD_TRY(upload(ctx, ctx->stage_u8, (const uint8_t*)des, elems));
    dsrc = ctx->stage_u8.p;
  } else {
    SOD_TRY(upload(ctx, ctx->stage_f32, (const float*)des, elems));
    dsrc = ctx->stage_f32.p;
  }
  SOD_HIP(ctx, hipMemsetAsync(ctx->flags.p, 0, 4, ctx->stream));  // invalid count
  SOD_TRY(sod_inputs_begin(ctx));
  if (ctx->impl != 0)
    SOD_TRY(launch_pack_i8(ctx, dsrc, dtype, n, db));
  else if (db)
    SOD_TRY(launch_pack_db(ctx, dsrc, dtype, n));
  else
    SOD_TRY(launch_pack_queries(ctx, dsrc, dtype, (int32_t)n));
  SOD_TRY(sod_inputs_end(ctx));
  uint32_t bad = 0;
  SOD_HIP(ctx, hipMemcpyAsync(&bad, ctx->flags.p, 4, hipMemcpyDeviceToHost, ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  // staging is only needed during the upload
  if (dtype == SOD_DTYPE_U8) sod_release(ctx->stage_u8); else sod_release(ctx->stage_f32);
  if (bad)
    return sod_fail(ctx, SOD_EINVAL, std::to_string(bad) +
                                         " descriptor chunk(s) hold values that are not integers in "
                                         "[0,255] (OpenCV SIFT descriptors are)");
  return SOD_OK;
}

int sod_db_upload_descriptors(sod_ctx* ctx, const void* des, int dtype, int64_t n,
                              int64_t row_offset) {
  SOD_TRY(set_dev(ctx));
  if (n < 1 || row_offset < 0 || row_offset + n > (int64_t)0x7fffffff)
    return sod_fail(ctx, SOD_EINVAL, "descriptor rows out of range");
  SOD_TRY(db_writable(ctx));
  SOD_HIP(ctx, hipMemsetAsync(ctx->flags.p + 1, 0, 4, ctx->stream));
  SOD_TRY(upload_descriptors(ctx, des, dtype, n, true));
  ctx->n_shard = n;
  ctx->row_offset = row_offset;
  ctx->matched = ctx->ratio_done = ctx->houghed = ctx->selected = ctx->affined = false;
  return SOD_OK;
}

// ---- DB shared between contexts (several query streams over one resident DB) ---------
int sod_db_share(sod_ctx* dst, sod_ctx* src) {
  SOD_TRY(set_dev(dst));
  if (src && src->db_src) src = src->db_src;   // share from the owner of the buffers
  if (!src || src == dst) return sod_fail(dst, SOD_EINVAL, "bad source context");
  if (src->device != dst->device) return sod_fail(dst, SOD_EINVAL, "contexts on different devices");
  if (!src->nsub || !src->n_total) return sod_fail(dst, SOD_ESTATE, "source has no database");
  SOD_TRY(db_writable(dst));   // dst's own DB is replaced: refused while others alias it
  dst->db_src = src;
  src->db_sharers.push_back(dst);
  sod_view(dst->mx, src->mx);
  sod_view(dst->my, src->my);
  sod_view(dst->mang, src->mang);
  sod_view(dst->moct, src->moct);
  sod_view(dst->mimg, src->mimg);
  sod_view(dst->cent, src->cent);
  sod_view(dst->isize, src->isize);
  sod_view(dst->dbpack, src->dbpack);
  sod_view(dst->dn, src->dn);
  dst->impl = src->impl;
  dst->n_total = src->n_total;
  dst->n_images = src->n_images;
  dst->n_shard = src->n_shard;
  dst->row_offset = src->row_offset;
  dst->nsub = src->nsub;
  dst->nqt = 0;   // queries must be re-uploaded in the (possibly new) layout
  // raw max ||d||^2 for sod_match_exact_order; the source's uploads are complete
  SOD_HIP(dst, sod_stream_sync(src->stream));
  SOD_HIP(dst, hipMemcpyAsync(dst->flags.p + 1, src->flags.p + 1, 4, hipMemcpyDeviceToDevice,
                              dst->stream));
  SOD_HIP(dst, sod_stream_sync(dst->stream));
  dst->matched = dst->ratio_done = dst->houghed = dst->selected = dst->affined = false;
  return SOD_OK;
}

// ---- packed DB image (DB on-disk format, upload = one memcpy) -----
// [header 64 B][packed descriptor fragments][norm words]; the fragment and norm layouts are
// the matcher's own (see match_i8.hip / match.hip), so an import is a plain copy.
namespace {
struct PackedHeader {
  char magic[8];        // "SODPK01\0"
  int32_t impl;         // matcher layout the image was packed for
  int32_t sub_bytes;    // bytes per subtile
  int64_t n_rows;       // real descriptor rows
  int64_t row_offset;   // global index of row 0
  int64_t nsub;         // subtiles (padded)
  int64_t norm_bytes;   // bytes of norm words
  uint32_t max_norm;    // raw max ||d||^2 (float bits) for sod_match_exact_order
  uint32_t pad[3];
};
static_assert(sizeof(PackedHeader) == 64, "header is 64 bytes");

int packed_layout(const sod_ctx* ctx, int* sub_bytes, int64_t* norm_bytes) {
  const int rows = ctx->impl == 2 ? 32 : kSubRows;
  *sub_bytes = ctx->impl == 0 ? kSubBytes : rows * kDim;   // bf16 4 KiB, int8 rows*128 B
  const int64_t npad = ctx->nsub * rows;
  // int8: c and parity words (2 x i32 per row); bf16: one f32 norm per row
  *norm_bytes = ctx->impl == 0 ? npad * 4 : npad * 8;
  return SOD_OK;
}
}  // namespace

int sod_db_packed_size(sod_ctx* ctx, int64_t* bytes) {
  SOD_TRY(set_dev(ctx));
  if (!ctx->nsub) return sod_fail(ctx, SOD_ESTATE, "no descriptors uploaded");
  int sb;
  int64_t nb;
  packed_layout(ctx, &sb, &nb);
  *bytes = (int64_t)sizeof(PackedHeader) + ctx->nsub * sb + nb;
  return SOD_OK;
}

int sod_db_export_packed(sod_ctx* ctx, void* out, int64_t bytes) {
  int64_t need;
  SOD_TRY(sod_db_packed_size(ctx, &need));
  if (!out || bytes < need) return sod_fail(ctx, SOD_EINVAL, "output buffer too small");
  int sb;
  int64_t nb;
  packed_layout(ctx, &sb, &nb);
  PackedHeader h{};
  std::memcpy(h.magic, "SODPK01", 8);
  h.impl = ctx->impl;
  h.sub_bytes = sb;
  h.n_rows = ctx->n_shard;
  h.row_offset = ctx->row_offset;
  h.nsub = ctx->nsub;
  h.norm_bytes = nb;
  uint8_t* o = static_cast<uint8_t*>(out);
  SOD_HIP(ctx, hipMemcpyAsync(&h.max_norm, ctx->flags.p + 1, 4, hipMemcpyDeviceToHost, ctx->stream));
  SOD_HIP(ctx, hipMemcpyAsync(o + sizeof(h), ctx->dbpack.p, (size_t)(ctx->nsub * sb),
                              hipMemcpyDeviceToHost, ctx->stream));
  SOD_HIP(ctx, hipMemcpyAsync(o + sizeof(h) + ctx->nsub * sb, ctx->dn.p, (size_t)nb,
                              hipMemcpyDeviceToHost, ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  std::memcpy(o, &h, sizeof(h));
  return SOD_OK;
}

int sod_db_import_packed(sod_ctx* ctx, const void* in, int64_t bytes) {
  SOD_TRY(set_dev(ctx));
  PackedHeader h;
  if (!in || bytes < (int64_t)sizeof(h)) return sod_fail(ctx, SOD_EINVAL, "not a packed DB image");
  std::memcpy(&h, in, sizeof(h));
  if (std::memcmp(h.magic, "SODPK01", 8) != 0) return sod_fail(ctx, SOD_EINVAL, "not a packed DB image");
  if (h.impl != ctx->impl)
    return sod_fail(ctx, SOD_EINVAL, "packed for matcher impl " + std::to_string(h.impl) +
                                         ", context uses " + std::to_string(ctx->impl));
  const int rows = ctx->impl == 2 ? 32 : kSubRows;
  const int want_sb = ctx->impl == 0 ? kSubBytes : rows * kDim;
  const int64_t want_nb = (ctx->impl == 0 ? 4 : 8) * h.nsub * rows;
  if (h.sub_bytes != want_sb || h.norm_bytes != want_nb || h.nsub < 1 || h.n_rows < 1 ||
      h.n_rows > h.nsub * rows || h.row_offset < 0 || h.row_offset + h.n_rows > 0x7fffffffLL ||
      bytes < (int64_t)sizeof(h) + h.nsub * h.sub_bytes + h.norm_bytes)
    return sod_fail(ctx, SOD_EINVAL, "inconsistent packed DB image");
  const uint8_t* src = static_cast<const uint8_t*>(in) + sizeof(h);
  SOD_TRY(db_writable(ctx));
  SOD_TRY(sod_inputs_begin(ctx));
  SOD_TRY(sod_reserve(ctx, ctx->dbpack, (size_t)(h.nsub * h.sub_bytes)));
  SOD_TRY(sod_reserve(ctx, ctx->dn, (size_t)(h.norm_bytes / 4)));
  SOD_HIP(ctx, hipMemcpyAsync(ctx->dbpack.p, src, (size_t)(h.nsub * h.sub_bytes),
                              hipMemcpyHostToDevice, ctx->stream));
  SOD_HIP(ctx, hipMemcpyAsync(ctx->dn.p, src + h.nsub * h.sub_bytes, (size_t)h.norm_bytes,
                              hipMemcpyHostToDevice, ctx->stream));
  SOD_HIP(ctx, hipMemcpyAsync(ctx->flags.p + 1, &h.max_norm, 4, hipMemcpyHostToDevice, ctx->stream));
  SOD_TRY(sod_inputs_end(ctx));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->nsub = h.nsub;
  ctx->n_shard = h.n_rows;
  ctx->row_offset = h.row_offset;
  ctx->matched = ctx->ratio_done = ctx->houghed = ctx->selected = ctx->affined = false;
  return SOD_OK;
}

int sod_query_upload(sod_ctx* ctx, const void* des, int dtype, int32_t nq, const float* x,
                     const float* y, const float* angle, const int32_t* octave) {
  SOD_TRY(set_dev(ctx));
  if (nq < 1 || nq > (1 << 27)) return sod_fail(ctx, SOD_EINVAL, "query count out of range");
  if (des) {
    SOD_HIP(ctx, hipMemsetAsync(ctx->flags.p + 2, 0, 4, ctx->stream));
    SOD_TRY(upload_descriptors(ctx, des, dtype, nq, false));
  } else {
    ctx->nqt = 0;  // keypoints only: hough on externally set matches
  }
  ctx->nq = nq;
  ctx->win0 = 0;
  ctx->winn = -1;
  ctx->n_qimg = 0;
  if (x && y && angle && octave) {
    SOD_TRY(upload(ctx, ctx->qx, x, (size_t)nq));
    SOD_TRY(upload(ctx, ctx->qy, y, (size_t)nq));
    SOD_TRY(upload(ctx, ctx->qang, angle, (size_t)nq));
    SOD_TRY(upload(ctx, ctx->qoct, octave, (size_t)nq));
    SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  }
  ctx->matched = ctx->ratio_done = ctx->houghed = ctx->selected = ctx->affined = false;
  return SOD_OK;
}

// ---- query window (several query images share one matcher pass) --
int sod_query_window(sod_ctx* ctx, int32_t first, int32_t count) {
  SOD_TRY(set_dev(ctx));
  if (count < 0) {
    ctx->win0 = 0;
    ctx->winn = -1;
  } else {
    if (first < 0 || count < 1 || (int64_t)first + count > ctx->nq)
      return sod_fail(ctx, SOD_EINVAL, "query window outside the uploaded queries");
    ctx->win0 = first;
    ctx->winn = count;
    ctx->n_qimg = 0;   // a window and an image batch are exclusive
  }
  ctx->houghed = ctx->selected = ctx->affined = false;
  return SOD_OK;
}

int sod_query_images(sod_ctx* ctx, int32_t n_images, const int32_t* q_offsets,
                     const int32_t* shapes) {
  SOD_TRY(set_dev(ctx));
  if (n_images <= 0) {
    ctx->n_qimg = 0;
    ctx->houghed = ctx->selected = ctx->affined = false;
    return SOD_OK;
  }
  if (!q_offsets || !shapes || q_offsets[0] != 0 || q_offsets[n_images] != ctx->nq)
    return sod_fail(ctx, SOD_EINVAL, "image offsets must cover the uploaded queries");
  for (int32_t b = 0; b < n_images; ++b)
    if (q_offsets[b + 1] < q_offsets[b] || shapes[2 * b] < 1 || shapes[2 * b + 1] < 1)
      return sod_fail(ctx, SOD_EINVAL, "bad image offsets or shapes");
  ctx->qoff_h.assign(q_offsets, q_offsets + n_images + 1);
  ctx->qshape_h.assign(shapes, shapes + 2 * n_images);
  std::vector<int32_t> img((size_t)ctx->nq);
  for (int32_t b = 0; b < n_images; ++b)
    for (int32_t q = q_offsets[b]; q < q_offsets[b + 1]; ++q) img[(size_t)q] = b;
  SOD_TRY(upload(ctx, ctx->qimg, img.data(), img.size()));
  SOD_TRY(upload(ctx, ctx->qshape, ctx->qshape_h.data(), ctx->qshape_h.size()));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->n_qimg = n_images;
  ctx->win0 = 0;
  ctx->winn = -1;
  ctx->houghed = ctx->selected = ctx->affined = false;
  return SOD_OK;
}

int sod_valid_images_get(sod_ctx* ctx, int32_t* image) {
  int64_t V, M;
  SOD_TRY(sod_valid_counts(ctx, &V, &M));
  std::vector<uint32_t> lin((size_t)V);
  SOD_TRY(download(ctx, lin.data(), ctx->vbin.p, (size_t)V));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  for (int64_t v = 0; v < V; ++v) image[v] = (int32_t)(lin[(size_t)v] / ctx->nbins1);
  return SOD_OK;
}

// ---- matcher --------------------------------------------------------------------------
int sod_match_enqueue(sod_ctx* ctx) {
  SOD_TRY(set_dev(ctx, false));   // writes no buffer a pending PoseBin means reads
  if (!ctx->nsub || !ctx->nqt) return sod_fail(ctx, SOD_ESTATE, "upload DB descriptors and queries first");
  ctx->ratio_fused_valid = false;   // set again by a final merge that applies the pipeline's ratio
  ctx->nseg = 0;                    // a new step for sod_last_stage_ms
  ctx->seg_open = false;
  SOD_TRY(ctx->impl != 0 ? launch_match_i8(ctx) : launch_match(ctx));
  ctx->matched = true;
  ctx->matches_given = false;
  ctx->ratio_done = ctx->houghed = ctx->selected = ctx->affined = false;
  return SOD_OK;
}

int sod_match_set_overlap(sod_ctx* ctx, int on) {
  SOD_TRY(set_dev(ctx));
  if (on != 0 && on != 1) return sod_fail(ctx, SOD_EINVAL, "overlap must be 0 or 1");
  // everything enqueued so far, on any stream, is ordered before the switch
  SOD_HIP(ctx, sod_stream_sync(ctx->mstream));
  SOD_HIP(ctx, sod_stream_sync(ctx->mstream2));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->ev_done[0] = ctx->ev_done[1] = nullptr;
  if (!on && ctx->cu_reserve)
    return sod_fail(ctx, SOD_ESTATE, "the CU split (sod_set_cu_reserve) needs the matcher stream");
  ctx->overlap = on != 0;
  ctx->gthr_n = 0;   // the next int8 launch re-initialises both threshold slots
  return SOD_OK;
}

// Split the chip between the matcher and everything else (SURVEY 8(e)/(f) overlap): a
// kernel enqueued while the matcher holds every CU gets its waves placed beside the
// matcher's and finishes only when the matcher does, so a step's Hough / select / affine
// stages (and, with several ranks, the RCCL exchanges) would serialise with the next
// matcher.  With per_xcd > 0 the context and side streams are re-created on `per_xcd` CUs
// of every XCD (CU-mask bits num_cus-8*per_xcd .. num_cus-1: bit i lies on XCD i % 8,
// measured with tools/cu_mask_probe.hip) and the matcher stream on the rest; the matcher
// grid is sized for the CUs it keeps.  Implies sod_match_set_overlap(ctx, 1).  0 restores
// unmasked streams.  Results are unchanged.
static hipError_t make_stream(hipStream_t* s, const std::vector<uint32_t>& mask) {
  if (mask.empty()) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  // cuMaskSize counts uint32 words (HIP copies [cuMask, cuMask + cuMaskSize))
  return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
}

// Every event of the context recorded once more, on stream s (empty markers, complete at
// once).  An event keeps a reference to the command it was last recorded with, and through it
// to that command's stream; sod_set_cu_reserve destroys the old (CU-masked) streams, and
// hipStreamDestroy of a stream whose commands are still referenced by events -- the slot
// release / completion events (ev_merged, ev_matched*, recorded by the merge's and the
// matcher's own dispatches), the fork / join and read events of the PoseBin means, the timing
// rings -- hung in round 4 about one suite run in three (r04e / r04f: after "streams idle",
// never "old streams destroyed"; sod_destroy, which destroys the events before the streams,
// never hung).  Re-recorded on the new context stream, no event references an old stream.
static hipError_t rebind_events(sod_ctx* ctx, hipStream_t s) {
  hipError_t e = hipSuccess;
  auto rec = [&](hipEvent_t ev) {
    if (ev && e == hipSuccess) e = hipEventRecord(ev, s);
  };
  for (auto& ev : ctx->ev) rec(ev);
  for (auto& pr : ctx->mev)
    for (auto& ev : pr) rec(ev);
  for (auto& pr : ctx->seg_ev)
    for (auto& ev : pr) rec(ev);
  rec(ctx->ev_fork);
  rec(ctx->ev_join);
  rec(ctx->ev_inputs);
  rec(ctx->ev_matched);
  rec(ctx->ev_matched1);
  for (int i = 0; i < 2; ++i) {
    rec(ctx->ev_merged[i]);
    rec(ctx->ev_hread[i]);
    rec(ctx->ev_sread[i]);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  ctx->nmatch = 0;    // the timing rings hold no launch now
  ctx->nseg = 0;
  ctx->seg_open = false;
  return e;
}

int sod_set_cu_reserve(sod_ctx* ctx, int per_xcd) {
  SOD_TRY(set_dev(ctx));
  const int nx = ctx->num_xcds;
  if (per_xcd < 0) return sod_fail(ctx, SOD_EINVAL, "cu reserve per XCD must be >= 0");
  if (per_xcd > 0) {
    // the mask-bit -> XCD map (bit i on XCD i % 8) was measured on a full MI355X
    // (tools/cu_mask_probe.hip); on another layout (a CPX/DPX partition, another SKU) the
    // reserved CUs would not be one per XCD and the matcher grid sizing would be wrong
    if (!ctx->gfx950 || nx != 8 || ctx->num_cus != 256)
      return sod_fail(ctx, SOD_EINVAL,
                      "CU split measured only on a whole MI355X (gfx950, 8 XCDs, 256 CUs); this "
                      "device has " + std::to_string(nx) + " XCD(s) and " +
                          std::to_string(ctx->num_cus) + " CUs");
    if (per_xcd * nx * 2 > ctx->num_cus)
      return sod_fail(ctx, SOD_EINVAL, "cu reserve per XCD must be in [0, CUs per XCD / 2]");
    // a collective whose blocks do not all fit the reserved CUs could wait on a block that
    // never gets a CU: the communicator must have been created (sod_comm_init under a split)
    // with at most that many blocks per collective
    if (ctx->comm && (ctx->comm_max_channels == 0 || ctx->comm_max_channels > per_xcd * nx))
      return sod_fail(ctx, SOD_ESTATE,
                      "the RCCL communicator was created with " +
                          (ctx->comm_max_channels ? "up to " + std::to_string(ctx->comm_max_channels)
                                                  : std::string("the default number of")) +
                          " blocks per collective (maxCTAs); the CU split runs collectives on " +
                          std::to_string(per_xcd * nx) +
                          " CUs: call sod_set_cu_reserve before sod_comm_init");
  }
  if (ctx->opt.debug_sync)
    std::fprintf(stderr, "sod: cu_reserve %d -> %d: stream %p side %p mstream %p\n", ctx->cu_reserve,
                 per_xcd, (void*)ctx->stream, (void*)ctx->side, (void*)ctx->mstream);
  SOD_HIP(ctx, sod_stream_drain(ctx->side));
  SOD_HIP(ctx, sod_stream_drain(ctx->mstream));
  SOD_HIP(ctx, sod_stream_drain(ctx->mstream2));
  SOD_HIP(ctx, sod_stream_drain(ctx->stream));
  ctx->side_pending = false;
  ctx->ev_done[0] = ctx->ev_done[1] = nullptr;
  const bool dbg = ctx->opt.debug_sync != 0;
  if (dbg) std::fprintf(stderr, "sod: cu_reserve streams idle\n");
  const int n = ctx->num_cus, words = (n + 31) / 32, r = per_xcd * nx;
  std::vector<uint32_t> tail, match;
  if (per_xcd > 0) {
    tail.assign(words, 0u);
    match.assign(words, 0u);
    for (int i = 0; i < n; ++i) (i >= n - r ? tail : match)[i / 32] |= 1u << (i % 32);
  }
  hipStream_t s = nullptr, sd = nullptr, ms = nullptr, ms2 = nullptr;
  hipError_t e = make_stream(&s, tail);
  if (e == hipSuccess) e = make_stream(&sd, tail);
  if (e == hipSuccess) e = make_stream(&ms, match);
  if (e == hipSuccess) e = make_stream(&ms2, match);
  if (e != hipSuccess) {
    if (s) (void)hipStreamDestroy(s);
    if (sd) (void)hipStreamDestroy(sd);
    if (ms) (void)hipStreamDestroy(ms);
    return sod_fail(ctx, SOD_EHIP, std::string("cu reserve: ") + hipGetErrorString(e));
  }
  if (dbg) std::fprintf(stderr, "sod: cu_reserve new streams %p %p %p\n", (void*)s, (void*)sd, (void*)ms);
  e = rebind_events(ctx, s);
  if (e != hipSuccess) {
    (void)hipStreamDestroy(s);
    (void)hipStreamDestroy(sd);
    (void)hipStreamDestroy(ms);
    (void)hipStreamDestroy(ms2);
    return sod_fail(ctx, SOD_EHIP, std::string("cu reserve: events: ") + hipGetErrorString(e));
  }
  if (dbg) std::fprintf(stderr, "sod: cu_reserve events re-recorded on the new stream\n");
  (void)hipStreamDestroy(ctx->stream);
  (void)hipStreamDestroy(ctx->side);
  (void)hipStreamDestroy(ctx->mstream);
  (void)hipStreamDestroy(ctx->mstream2);
  if (dbg) std::fprintf(stderr, "sod: cu_reserve old streams destroyed\n");
  ctx->stream = s;
  ctx->side = sd;
  ctx->mstream = ms;
  ctx->mstream2 = ms2;
  ctx->cu_reserve = per_xcd;
  ctx->reserved_cus = r;
  if (per_xcd > 0) ctx->overlap = true;
  ctx->gthr_n = 0;   // the next int8 launch re-initialises both threshold slots
  return SOD_OK;
}

int sod_match_set_impl(sod_ctx* ctx, int impl) {
  SOD_TRY(set_dev(ctx));
  if (impl < 0 || impl > 2)
    return sod_fail(ctx, SOD_EINVAL, "impl must be 0 (bf16), 1 (int8 16x16x64) or 2 (int8 32x32x32)");
  if (impl != ctx->impl) {  // packed operands differ: uploads must be repeated
    SOD_TRY(db_writable(ctx));
    ctx->impl = impl;
    ctx->nsub = 0;
    ctx->nqt = 0;
    ctx->matched = ctx->ratio_done = ctx->houghed = ctx->selected = ctx->affined = false;
  }
  return SOD_OK;
}

int sod_host_wait_ns(sod_ctx* ctx, int64_t* ns, int reset) {
  if (!ctx || !ns) return SOD_EINVAL;
  *ns = ctx->host_wait_ns;
  if (reset) ctx->host_wait_ns = 0;
  return SOD_OK;
}

int sod_trig_exact(sod_ctx* ctx) { return ctx ? (ctx->trig_exact ? 1 : 0) : SOD_EINVAL; }

int sod_glibc_sincos(sod_ctx* ctx, int64_t n, const double* x, double* s, double* c) {
  SOD_TRY(set_dev(ctx, false));
  if (n < 0 || (n > 0 && (!x || !s || !c))) return sod_fail(ctx, SOD_EINVAL, "bad arguments");
  if (n == 0) return SOD_OK;
  DevBuf<double> dx, ds, dc;
  int rc = upload(ctx, dx, x, (size_t)n);
  if (rc == SOD_OK) rc = sod_reserve(ctx, ds, (size_t)n);
  if (rc == SOD_OK) rc = sod_reserve(ctx, dc, (size_t)n);
  if (rc == SOD_OK) rc = launch_glibc_sincos(ctx, n, dx.p, ds.p, dc.p);
  if (rc == SOD_OK) rc = download(ctx, s, ds.p, (size_t)n);
  if (rc == SOD_OK) rc = download(ctx, c, dc.p, (size_t)n);
  if (rc == SOD_OK && sod_stream_sync(ctx->stream) != hipSuccess)
    rc = sod_fail(ctx, SOD_EHIP, "glibc sincos failed");
  (void)sod_stream_sync(ctx->stream);
  sod_release(dx);
  sod_release(ds);
  sod_release(dc);
  return rc;
}

int sod_match_set_kernel(sod_ctx* ctx, int kernel) {
  if (!ctx) return SOD_EINVAL;
  if (kernel == 2)
    return sod_fail(ctx, SOD_EINVAL, "the register-streamed kernel (2) was removed in round 6: "
                                     "2x slower than the LDS ring at every size");
  if (kernel < 0 || kernel > 1)
    return sod_fail(ctx, SOD_EINVAL, "kernel must be 0 (by query count) or 1 (LDS ring)");
  ctx->mkernel = kernel;
  return SOD_OK;
}

int sod_match_allgather_enqueue(sod_ctx* ctx) {
  SOD_TRY(set_dev(ctx, false));   // writes no buffer a pending PoseBin means reads
  if (!ctx->matched) return sod_fail(ctx, SOD_ESTATE, "sod_match_enqueue first");
  if (ctx->nranks <= 1 && !ctx->comm) return SOD_OK;   // a 1-rank communicator still runs
  if (!ctx->comm) return sod_fail(ctx, SOD_ECOMM, "no communicator");
  const size_t nq_pad = (size_t)sod_nq_pad(ctx);
  const size_t tot = nq_pad * ctx->nranks;
  SOD_TRY(sod_reserve(ctx, ctx->gd1, tot));
  SOD_TRY(sod_reserve(ctx, ctx->gd2, tot));
  SOD_TRY(sod_reserve(ctx, ctx->gidx, tot));
  SOD_TRY(sod_stage_mark(ctx, kStageAllgather, false));
  ncclResult_t r = ncclGroupStart();
  if (r == ncclSuccess) r = ncclAllGather(ctx->cd1.p, ctx->gd1.p, nq_pad, ncclFloat32, ctx->comm, ctx->stream);
  if (r == ncclSuccess) r = ncclAllGather(ctx->cidx.p, ctx->gidx.p, nq_pad, ncclInt32, ctx->comm, ctx->stream);
  if (r == ncclSuccess) r = ncclAllGather(ctx->cd2.p, ctx->gd2.p, nq_pad, ncclFloat32, ctx->comm, ctx->stream);
  ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess)
    return sod_fail(ctx, SOD_ECOMM, std::string("ncclAllGather: ") +
                                        ncclGetErrorString(r != ncclSuccess ? r : r2));
  SOD_TRY(sod_stage_mark(ctx, kStageAllgather, true));
  // global merge in rank order (lexicographic on (d^2, trainIdx): order-independent anyway)
  SOD_TRY(sod_stage_mark(ctx, kStageMerge, false));
  SOD_TRY(launch_merge(ctx, ctx->gd1.p, ctx->gidx.p, ctx->gd2.p, ctx->nranks, (int64_t)nq_pad,
                       nullptr, true));   // the global merge: final
  return sod_stage_mark(ctx, kStageMerge, true);
}

int sod_ratio_enqueue(sod_ctx* ctx, double ratio) {
  SOD_TRY(set_dev(ctx, false));   // writes no buffer a pending PoseBin means reads
  if (!ctx->matched) return sod_fail(ctx, SOD_ESTATE, "sod_match_enqueue first");
  if (!(ratio >= 0.0) || !std::isfinite(ratio))
    return sod_fail(ctx, SOD_EINVAL, "ratio must be a finite number >= 0");
  // skipped only when the final merge of this very launch applied this very ratio
  if (!ctx->ratio_fused_valid || ctx->ratio_fused != ratio) {
    SOD_TRY(sod_stage_mark(ctx, kStageMerge, false));
    SOD_TRY(launch_ratio(ctx, ratio));
    SOD_TRY(sod_stage_mark(ctx, kStageMerge, true));
  }
  ctx->ratio_done = true;
  return SOD_OK;
}

int sod_match_get(sod_ctx* ctx, int32_t* idx1, float* d1, float* d2, uint8_t* good) {
  SOD_TRY(set_dev(ctx));
  if (!ctx->ratio_done) return sod_fail(ctx, SOD_ESTATE, "sod_ratio_enqueue first");
  const size_t n = (size_t)ctx->nq;
  SOD_TRY(download(ctx, idx1, ctx->idx1.p, n));
  SOD_TRY(download(ctx, d1, ctx->d1.p, n));
  SOD_TRY(download(ctx, d2, ctx->d2.p, n));
  SOD_TRY(download(ctx, good, ctx->good.p, n));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  return SOD_OK;
}

// the integers n whose correctly rounded sqrtf is d (OpenCV's float distance): a short run
// around d^2 (one value below 2048, a few above); empty (lo > hi) for a d no real distance
// has -- squared distances of 0..255 descriptors are < 2^24, so d < 4096; the padding rows'
// 1e30 norm (a single-row DB's "second") is not one
static void sqrt_preimage(float d, float* lo, float* hi) {
  *lo = 1.0f;
  *hi = 0.0f;
  if (!(d >= 0.0f) || !(d < 4096.0f)) return;
  const double c = std::floor((double)d * (double)d);
  bool any = false;
  for (double n = std::max(0.0, c - 64.0); n <= c + 64.0; n += 1.0) {
    if (std::sqrt((float)n) != d) continue;   // float sqrt: correctly rounded (IEEE)
    if (!any) *lo = (float)n;
    *hi = (float)n;
    any = true;
  }
}

// knnMatch's float-order indices (see sod_match_knn_indices): f1 always, f2 when want2
static int knn_float_indices(sod_ctx* ctx, bool want2, std::vector<int32_t>& f1,
                             std::vector<int32_t>& f2) {
  if (!ctx->ratio_done) return sod_fail(ctx, SOD_ESTATE, "sod_match_enqueue + sod_ratio_enqueue first");
  if (ctx->matches_given)
    return sod_fail(ctx, SOD_ESTATE, "the matches were set by sod_matches_set (no distances): "
                                     "run sod_match_enqueue first");
  if (ctx->impl == 2)
    return sod_fail(ctx, SOD_ESTATE, "knnMatch's indices need the int8 16x16x64 or the bf16 "
                                     "matcher (sod_match_set_impl(ctx, 1 or 0) before the uploads)");
  if (ctx->nranks > 1 || ctx->comm || ctx->row_offset != 0)
    return sod_fail(ctx, SOD_ESTATE, "knnMatch's indices are single-context only");
  int exact = 0;
  SOD_TRY(sod_match_exact_order(ctx, &exact));
  const size_t n = (size_t)ctx->nq, np = (size_t)sod_nq_pad(ctx);
  std::vector<float> d1(n), d2(n), lo(np, 1.0f), hi(np, 0.0f);
  std::vector<int32_t> i1(n), ex(np, -1);
  f1.assign(np, 0);
  f2.assign(np, 0x7f7f7f7f);
  SOD_TRY(download(ctx, i1.data(), ctx->idx1.p, n));
  SOD_TRY(download(ctx, d1.data(), ctx->d1.p, n));
  SOD_TRY(download(ctx, d2.data(), ctx->d2.p, n));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  DevBuf<float> dlo, dhi;
  DevBuf<int32_t> dex, dfound;
  int rc = SOD_OK;
  auto pass = [&](const std::vector<float>& dist, std::vector<int32_t>& out) {
    for (size_t q = 0; q < n; ++q) sqrt_preimage(dist[q], &lo[q], &hi[q]);
    if (rc == SOD_OK) rc = upload(ctx, dlo, lo.data(), np);
    if (rc == SOD_OK) rc = upload(ctx, dhi, hi.data(), np);
    if (rc == SOD_OK) rc = upload(ctx, dex, ex.data(), np);
    if (rc == SOD_OK) rc = sod_reserve(ctx, dfound, np);
    if (rc == SOD_OK)
      rc = ctx->impl == 1 ? launch_find_rows_i8(ctx, dlo.p, dhi.p, dex.p, dfound.p)
                          : launch_find_rows(ctx, dlo.p, dhi.p, dex.p, dfound.p);
    if (rc == SOD_OK) rc = download(ctx, out.data(), dfound.p, np);
    if (rc == SOD_OK && sod_stream_sync(ctx->stream) != hipSuccess)
      rc = sod_fail(ctx, SOD_EHIP, "knn index pass failed");
  };
  // OpenCV orders by the float distance sqrtf(d^2), ties to the lower trainIdx.  With every
  // distance < 2048 (exact order) distinct squared distances have distinct floats and the
  // matcher's idx1 is OpenCV's; otherwise the lowest row at the float d1 is
  if (exact) {
    for (size_t q = 0; q < n; ++q) f1[q] = i1[q];
  } else {
    pass(d1, f1);
    for (size_t q = 0; q < n && rc == SOD_OK; ++q)
      if (f1[q] == 0x7f7f7f7f) f1[q] = i1[q];   // unreachable: the best row is at d1
  }
  // the second: the lowest row other than that one at the float d2
  if (rc == SOD_OK && want2) {
    for (size_t q = 0; q < n; ++q) ex[q] = f1[q];
    pass(d2, f2);
  }
  (void)sod_stream_sync(ctx->stream);
  sod_release(dlo);
  sod_release(dhi);
  sod_release(dex);
  sod_release(dfound);
  return rc;
}

int sod_match_knn_indices(sod_ctx* ctx, int32_t* idx1, int32_t* idx2) {
  SOD_TRY(set_dev(ctx));
  if (!idx1 && !idx2) return sod_fail(ctx, SOD_EINVAL, "null outputs");
  std::vector<int32_t> f1, f2;
  SOD_TRY(knn_float_indices(ctx, idx2 != nullptr, f1, f2));
  const size_t n = (size_t)ctx->nq;
  if (idx1) std::memcpy(idx1, f1.data(), n * 4);
  if (idx2)
    for (size_t q = 0; q < n; ++q) idx2[q] = f2[q] == 0x7f7f7f7f ? -1 : f2[q];   // single DB row
  return SOD_OK;
}

int sod_match_float_order(sod_ctx* ctx) {
  SOD_TRY(set_dev(ctx));
  int exact = 0;
  if (!ctx->ratio_done) return sod_fail(ctx, SOD_ESTATE, "sod_match_enqueue + sod_ratio_enqueue first");
  SOD_TRY(sod_match_exact_order(ctx, &exact));
  if (exact) return SOD_OK;   // the matcher's idx1 already is OpenCV's
  std::vector<int32_t> f1, f2;
  SOD_TRY(knn_float_indices(ctx, false, f1, f2));
  SOD_TRY(upload(ctx, ctx->idx1, f1.data(), (size_t)ctx->nq));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->houghed = ctx->selected = ctx->affined = false;
  return SOD_OK;
}

int sod_matches_set(sod_ctx* ctx, int32_t nq, const int32_t* idx1, const uint8_t* good) {
  SOD_TRY(set_dev(ctx));
  if (!idx1 || !good || nq != ctx->nq || nq < 1)
    return sod_fail(ctx, SOD_EINVAL, "sod_matches_set: nq must equal the uploaded query count");
  for (int32_t q = 0; q < nq; ++q)
    if (good[q] && (idx1[q] < 0 || idx1[q] >= ctx->n_total))
      return sod_fail(ctx, SOD_EINVAL, "sod_matches_set: trainIdx out of range");
  SOD_TRY(upload(ctx, ctx->idx1, idx1, (size_t)nq));
  SOD_TRY(upload(ctx, ctx->good, good, (size_t)nq));
  SOD_TRY(sod_reserve(ctx, ctx->d1, (size_t)nq));
  SOD_TRY(sod_reserve(ctx, ctx->d2, (size_t)nq));
  SOD_HIP(ctx, hipMemsetAsync(ctx->d1.p, 0, (size_t)nq * 4, ctx->stream));
  SOD_HIP(ctx, hipMemsetAsync(ctx->d2.p, 0, (size_t)nq * 4, ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->ratio_fused_valid = false;
  ctx->nseg = 0;
  ctx->seg_open = false;
  ctx->matched = ctx->ratio_done = true;
  ctx->matches_given = true;
  ctx->houghed = ctx->selected = ctx->affined = false;
  return SOD_OK;
}

int sod_match_exact_order(sod_ctx* ctx, int* exact) {
  SOD_TRY(set_dev(ctx));
  uint32_t f[4];
  SOD_HIP(ctx, hipMemcpyAsync(f, ctx->flags.p, 16, hipMemcpyDeviceToHost, ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  float dn, qn;
  std::memcpy(&dn, &f[1], 4);
  std::memcpy(&qn, &f[2], 4);
  // every distance <= |q| + |d| <= 2048  =>  squared distances <= 2^22, where distinct
  // integers have distinct correctly rounded float square roots
  *exact = (std::sqrt((double)dn) + std::sqrt((double)qn) <= 2048.0) ? 1 : 0;
  return SOD_OK;
}

// ---- hough ----------------------------------------------------------------------------
// the argument / state checks of a Hough launch (sod_hough_enqueue and the fused path)
static int hough_check(sod_ctx* ctx, int32_t query_h, int32_t query_w, const int32_t bins[4]) {
  if (!ctx->ratio_done) return sod_fail(ctx, SOD_ESTATE, "match + ratio first");
  if (!ctx->n_total || !ctx->qx.p) return sod_fail(ctx, SOD_ESTATE, "keypoints not uploaded");
  if (query_h < 1 || query_w < 1) return sod_fail(ctx, SOD_EINVAL, "bad query image shape");
  SOD_TRY(check_bins(ctx, bins));
  if (ctx->n_qimg) {   // one bin space per query image, image-major
    if (ctx->winn >= 0) return sod_fail(ctx, SOD_EINVAL, "query window and image batch are exclusive");
    ctx->nbins = ctx->nbins1 * ctx->n_qimg;
    if (ctx->nbins > 0x7fffffffLL) return sod_fail(ctx, SOD_EINVAL, "too many bins x images");
  }
  ctx->qh = query_h;
  ctx->qw = query_w;
  return SOD_OK;
}

int sod_hough_enqueue(sod_ctx* ctx, int32_t query_h, int32_t query_w, const int32_t bins[4],
                      int64_t own_lo, int64_t own_hi) {
  SOD_TRY(set_dev(ctx, false));   // writes no buffer a pending PoseBin means reads
  SOD_TRY(hough_check(ctx, query_h, query_w, bins));
  SOD_TRY(sod_stage_mark(ctx, kStageHough, false));
  SOD_TRY(launch_hough(ctx, own_lo, own_hi));
  SOD_TRY(sod_stage_mark(ctx, kStageHough, true));
  ctx->houghed = true;
  ctx->selected = ctx->affined = false;
  return SOD_OK;
}

int sod_hough_allreduce_enqueue(sod_ctx* ctx) {
  SOD_TRY(set_dev(ctx, false));   // writes no buffer a pending PoseBin means reads
  if (!ctx->houghed) return sod_fail(ctx, SOD_ESTATE, "sod_hough_enqueue first");
  if (ctx->nranks <= 1 && !ctx->comm) return SOD_OK;   // a 1-rank communicator still runs
  if (!ctx->comm) return sod_fail(ctx, SOD_ECOMM, "no communicator");
  SOD_TRY(sod_hist_dense(ctx));
  SOD_TRY(sod_stage_mark(ctx, kStageAllreduce, false));
  ncclResult_t r = ncclGroupStart();
  if (r == ncclSuccess)
    r = ncclAllReduce(ctx->counts.p, ctx->counts.p, ctx->nbins, ncclUint32, ncclSum, ctx->comm, ctx->stream);
  if (r == ncclSuccess)
    r = ncclAllReduce(ctx->first.p, ctx->first.p, ctx->nbins, ncclUint32, ncclMin, ctx->comm, ctx->stream);
  ncclResult_t r2 = ncclGroupEnd();
  SOD_TRY(sod_stage_mark(ctx, kStageAllreduce, true));
  if (r != ncclSuccess || r2 != ncclSuccess)
    return sod_fail(ctx, SOD_ECOMM, std::string("ncclAllReduce: ") +
                                        ncclGetErrorString(r != ncclSuccess ? r : r2));
  return SOD_OK;
}

int sod_hough_select_enqueue(sod_ctx* ctx, int32_t query_h, int32_t query_w,
                             const int32_t bins[4], int32_t vote_threshold) {
  SOD_TRY(set_dev(ctx, false));   // writes no buffer a pending PoseBin means reads
  if (sod_hough_small_ok(ctx)) {
    // one image of <= 2048 queries on one rank: vote + select + affine gather in one launch
    SOD_TRY(hough_check(ctx, query_h, query_w, bins));
    SOD_TRY(sod_stage_mark(ctx, kStageHough, false));
    SOD_TRY(launch_hough_small(ctx, vote_threshold));
    SOD_TRY(sod_stage_mark(ctx, kStageHough, true));
    ctx->houghed = ctx->selected = true;
    ctx->affined = false;
    ctx->vote_thr = vote_threshold;
    return SOD_OK;
  }
  const int64_t lo = ctx->nranks > 1 ? ctx->row_offset : 0;
  const int64_t hi = ctx->nranks > 1 ? ctx->row_offset + ctx->n_shard : ctx->n_total;
  SOD_TRY(sod_hough_enqueue(ctx, query_h, query_w, bins, lo, hi));
  SOD_TRY(sod_hough_allreduce_enqueue(ctx));
  return sod_select_enqueue(ctx, vote_threshold);
}

int sod_select_enqueue(sod_ctx* ctx, int32_t vote_threshold) {
  SOD_TRY(set_dev(ctx, false));   // writes no buffer a pending PoseBin means reads
  if (!ctx->houghed) return sod_fail(ctx, SOD_ESTATE, "sod_hough_enqueue first");
  SOD_TRY(sod_hist_dense(ctx));
  SOD_TRY(sod_stage_mark(ctx, kStageSelect, false));
  SOD_TRY(launch_select(ctx, vote_threshold, true));
  SOD_TRY(sod_stage_mark(ctx, kStageSelect, true));
  ctx->vote_thr = vote_threshold;
  ctx->selected = true;
  ctx->affined = false;
  return SOD_OK;
}

int sod_valid_counts(sod_ctx* ctx, int64_t* n_valid, int64_t* n_members) {
  SOD_TRY(set_dev(ctx));
  if (!ctx->selected) return sod_fail(ctx, SOD_ESTATE, "sod_select_enqueue first");
  SOD_TRY(sod_guard_resolve(ctx));
  uint32_t s[2];
  SOD_HIP(ctx, hipMemcpyAsync(s, ctx->scal.p, 8, hipMemcpyDeviceToHost, ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  if (n_valid) *n_valid = s[0];
  if (n_members) *n_members = s[1];
  return SOD_OK;
}

static void decode_keys(const sod_ctx* ctx, const std::vector<uint32_t>& lin, int32_t* keys) {
  const int by = ctx->bins[1], bt = ctx->bins[2], bs = ctx->bins[3];
  for (size_t i = 0; i < lin.size(); ++i) {
    const uint32_t l = (uint32_t)(lin[i] % ctx->nbins1);   // bin within its query image
    keys[4 * i + 3] = l % bs;
    keys[4 * i + 2] = (l / bs) % bt;
    keys[4 * i + 1] = (l / (bs * bt)) % by;
    keys[4 * i + 0] = l / (bs * bt * by);
  }
}

int sod_valid_get(sod_ctx* ctx, int32_t* keys, int32_t* votes, int64_t* offsets,
                  int32_t* members, double* means) {
  int64_t V, M;
  SOD_TRY(sod_valid_counts(ctx, &V, &M));
  std::vector<uint32_t> lin((size_t)V);
  SOD_TRY(download(ctx, lin.data(), ctx->vbin.p, (size_t)V));
  std::vector<int64_t> off((size_t)V + 1);
  SOD_TRY(download(ctx, off.data(), ctx->voff.p, (size_t)V + 1));
  SOD_TRY(download(ctx, members, ctx->members.p, (size_t)M));
  SOD_TRY(download(ctx, means, ctx->means.p, (size_t)V * 6));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  if (keys) decode_keys(ctx, lin, keys);
  if (votes)
    for (int64_t i = 0; i < V; ++i) votes[i] = (int32_t)(off[i + 1] - off[i]);
  if (offsets) std::memcpy(offsets, off.data(), off.size() * sizeof(int64_t));
  return SOD_OK;
}

int sod_bins_count(sod_ctx* ctx, int64_t* n_bins) {
  SOD_TRY(set_dev(ctx));
  if (!ctx->houghed) return sod_fail(ctx, SOD_ESTATE, "sod_hough_enqueue first");
  SOD_TRY(sod_guard_resolve(ctx));
  SOD_TRY(sod_hist_dense(ctx));
  SOD_TRY(launch_all_bins(ctx));
  uint32_t b = 0;
  SOD_HIP(ctx, hipMemcpyAsync(&b, ctx->scal.p + 2, 4, hipMemcpyDeviceToHost, ctx->stream));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  *n_bins = b;
  return SOD_OK;
}

int sod_bins_get(sod_ctx* ctx, int32_t* keys, int32_t* votes) {
  int64_t B;
  SOD_TRY(sod_bins_count(ctx, &B));
  std::vector<uint32_t> lin((size_t)B);
  SOD_TRY(download(ctx, lin.data(), ctx->allbin.p, (size_t)B));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  std::vector<uint32_t> cnt((size_t)ctx->nbins);
  SOD_TRY(download(ctx, cnt.data(), ctx->counts.p, (size_t)ctx->nbins));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  if (keys) decode_keys(ctx, lin, keys);
  if (votes)
    for (int64_t i = 0; i < B; ++i) votes[i] = (int32_t)cnt[lin[i]];
  return SOD_OK;
}

int sod_hough_guard_stats(sod_ctx* ctx, int64_t* flagged, int64_t* changed,
                          int64_t* flagged_total, int64_t* changed_total) {
  SOD_TRY(set_dev(ctx));
  SOD_TRY(sod_guard_resolve(ctx));
  if (flagged) *flagged = ctx->guard_flagged;
  if (changed) *changed = ctx->guard_patched;
  if (flagged_total) *flagged_total = ctx->guard_flagged_total;
  if (changed_total) *changed_total = ctx->guard_patched_total;
  return SOD_OK;
}

// ---- affine ---------------------------------------------------------------------------
int sod_affine_enqueue(sod_ctx* ctx, int32_t query_w, int32_t query_h, double x_factor,
                       double y_factor, int32_t threshold) {
  SOD_TRY(set_dev(ctx, false, false));   // runs beside the means (side stream or same launch)
  if (!ctx->selected) return sod_fail(ctx, SOD_ESTATE, "sod_select_enqueue first");
  if (!(x_factor != 0.0) || !(y_factor != 0.0)) return sod_fail(ctx, SOD_EINVAL, "zero factor");
  ctx->aff_qw = query_w;
  ctx->aff_qh = query_h;
  ctx->aff_xf = x_factor;
  ctx->aff_yf = y_factor;
  ctx->aff_thr = threshold;
  SOD_TRY(sod_stage_mark(ctx, kStageAffine, false));
  if (!ctx->gathered) SOD_TRY(launch_affine_gather(ctx));   // the fused path gathered them
  SOD_TRY(sod_reserve(ctx, ctx->surv, (size_t)ctx->vmax));
  SOD_TRY(sod_reserve(ctx, ctx->fvotes, (size_t)ctx->vmax));
  SOD_TRY(sod_reserve(ctx, ctx->params, (size_t)ctx->vmax * 6));
  SOD_TRY(sod_reserve(ctx, ctx->alive, (size_t)ctx->mmax));
  if (ctx->means_deferred) {   // the fused one-image path: means and affine in one launch
    SOD_TRY(launch_means_affine(ctx, query_w, query_h, x_factor, y_factor, threshold));
    SOD_TRY(sod_stage_mark(ctx, kStageAffine, true));
    ctx->affined = true;
    return SOD_OK;
  }
  SOD_TRY(launch_affine(ctx, 0, true, ctx->voff.p, ctx->amx.p, ctx->amy.p, ctx->aqx.p, ctx->aqy.p,
                        ctx->aisig.p, query_w, query_h, ctx->n_qimg ? ctx->bwh.p : nullptr,
                        x_factor, y_factor, threshold, 1 << 30,
                        nullptr, ctx->surv.p, ctx->fvotes.p, ctx->params.p, ctx->alive.p,
                        ctx->scal.p));
  SOD_TRY(sod_stage_mark(ctx, kStageAffine, true));
  ctx->affined = true;
  return SOD_OK;
}

int sod_affine_get(sod_ctx* ctx, uint8_t* survived, int32_t* votes, double* params,
                   uint8_t* member_alive) {
  int64_t V, M;
  SOD_TRY(sod_valid_counts(ctx, &V, &M));
  if (!ctx->affined) return sod_fail(ctx, SOD_ESTATE, "sod_affine_enqueue first");
  SOD_TRY(download(ctx, survived, ctx->surv.p, (size_t)V));
  SOD_TRY(download(ctx, votes, ctx->fvotes.p, (size_t)V));
  SOD_TRY(download(ctx, params, ctx->params.p, (size_t)V * 6));
  SOD_TRY(download(ctx, member_alive, ctx->alive.p, (size_t)M));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  return SOD_OK;
}

// ---- results staging -----------------------------------------------------------------
// lay out `parts` of the current results in the page-locked buffer and enqueue the kernels
// that write them there (state checks done by the caller, after set_dev)
static int results_stage(sod_ctx* ctx, int parts, ResLayout* out) {
  const bool do_post = (parts & SOD_RES_POST) && ctx->selected;
  const bool do_valid = (parts & SOD_RES_VALID) && ctx->selected;
  const bool do_aff = (parts & SOD_RES_AFFINE) && ctx->selected && ctx->affined;
  ResLayout L;
  L.nq = (parts & SOD_RES_MATCH) ? ctx->nq : 0;
  L.valid = do_valid;
  L.affine = do_aff;
  L.keys_only = do_post;   // (image batches: the host relations path needs each bin's image)
  L.vcap = do_valid || do_aff || do_post ? ctx->vmax : 0;
  L.mcap = do_valid || do_aff || do_post ? ctx->mmax : 0;
  L.ncap = do_post ? std::min<int64_t>(L.vcap, 1024) : 0;
  L.words = (int)((L.ncap + 63) / 64);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 15) & ~(size_t)15;
    return at;
  };
  L.hdr = take(64);
  L.idx1 = take((size_t)L.nq * 4);
  L.d1 = take((size_t)L.nq * 4);
  L.d2 = take((size_t)L.nq * 4);
  L.good = take((size_t)L.nq);
  L.vbin = take((size_t)L.vcap * 4);
  L.voff = take(((size_t)L.vcap + 1) * 8);
  L.members = take((size_t)L.mcap * 4);
  L.means = take((size_t)L.vcap * 48);
  L.surv = take((size_t)L.vcap);
  L.fvotes = take((size_t)L.vcap * 4);
  L.params = take((size_t)L.vcap * 48);
  L.alive = take((size_t)L.mcap);
  L.sidx = take(do_post ? (size_t)L.vcap * 4 : 0);
  L.smeans = take(do_post ? (size_t)L.vcap * 48 : 0);
  L.pos = take((size_t)L.ncap * L.words * 8);
  L.ori = take((size_t)L.ncap * L.words * 8);
  L.total = o;
  if (ctx->hres_n < L.total) {
    // a staging kernel of an earlier enqueue may still write into the old buffer
    SOD_HIP(ctx, sod_stream_sync(ctx->stream));
    if (ctx->hres) (void)hipHostFree(ctx->hres);
    ctx->hres = nullptr;
    ctx->hres_n = 0;
    SOD_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->hres), L.total, hipHostMallocDefault));
    ctx->hres_n = L.total;
  }
  SOD_TRY(launch_results_stage(ctx, L, do_post));
  *out = L;
  return SOD_OK;
}

int sod_results_fetch(sod_ctx* ctx, int parts, sod_results* out) {
  if (!ctx) return SOD_EINVAL;
  // staged by the pipeline enqueue (or an earlier fetch) and nothing called since
  const bool reuse = ctx->staged_epoch == ctx->res_epoch && (parts & ~ctx->staged_parts) == 0;
  SOD_TRY(set_dev(ctx));   // joins the side stream (PoseBin means)
  if (!out) return sod_fail(ctx, SOD_EINVAL, "null output");
  if (parts & ~SOD_RES_ALL) return sod_fail(ctx, SOD_EINVAL, "unknown result part");
  if ((parts & SOD_RES_MATCH) && !ctx->ratio_done)
    return sod_fail(ctx, SOD_ESTATE, "sod_ratio_enqueue first");
  if ((parts & ~SOD_RES_MATCH) && !ctx->selected)
    return sod_fail(ctx, SOD_ESTATE, "sod_select_enqueue first");
  if (ctx->selected) SOD_TRY(sod_guard_resolve(ctx));   // (patches the device results)
  const bool do_post = (parts & SOD_RES_POST) && ctx->selected;
  const bool do_valid = (parts & SOD_RES_VALID) && ctx->selected;
  const bool do_aff = (parts & SOD_RES_AFFINE) && ctx->selected && ctx->affined;
  ResLayout L;
  int staged = parts;
  if (reuse) {
    L = ctx->staged_L;
    staged = ctx->staged_parts;
  } else {
    SOD_TRY(results_stage(ctx, parts, &L));
  }
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  // the buffer holds these parts until the next call (a second fetch reads it again)
  ctx->staged_L = L;
  ctx->staged_parts = staged;
  ctx->staged_epoch = ctx->res_epoch;
  const int64_t* hdr = reinterpret_cast<const int64_t*>(ctx->hres + L.hdr);
  const int64_t V = L.vcap ? hdr[0] : 0, M = L.vcap ? hdr[1] : 0;
  ResHost& r = ctx->res;
  const uint8_t* h = ctx->hres;
  *out = sod_results{};
  out->nq = (parts & SOD_RES_MATCH) ? L.nq : 0;
  if (out->nq) {
    out->idx1 = reinterpret_cast<const int32_t*>(h + L.idx1);
    out->d1 = reinterpret_cast<const float*>(h + L.d1);
    out->d2 = reinterpret_cast<const float*>(h + L.d2);
    out->good = h + L.good;
  }
  if (do_valid) {
    const uint32_t* vb = reinterpret_cast<const uint32_t*>(h + L.vbin);
    const int64_t* off = reinterpret_cast<const int64_t*>(h + L.voff);
    r.keys.resize((size_t)std::max<int64_t>(1, V) * 4);
    decode_keys(ctx, std::vector<uint32_t>(vb, vb + V), r.keys.data());
    r.votes.resize((size_t)std::max<int64_t>(1, V));
    for (int64_t i = 0; i < V; ++i) r.votes[(size_t)i] = (int32_t)(off[i + 1] - off[i]);
    out->selected = 1;
    out->n_valid = V;
    out->n_members = M;
    out->keys = r.keys.data();
    out->votes = r.votes.data();
    out->offsets = off;
    out->members = reinterpret_cast<const int32_t*>(h + L.members);
    out->means = reinterpret_cast<const double*>(h + L.means);
  }
  if (do_aff) {
    out->n_valid = V;
    out->n_members = M;
    out->affined = 1;
    out->survived = h + L.surv;
    out->affine_votes = reinterpret_cast<const int32_t*>(h + L.fvotes);
    out->params = reinterpret_cast<const double*>(h + L.params);
    out->alive = h + L.alive;
  }
  if (do_post) {
    SOD_TRY(sod_post_staged(ctx, L, r));
    out->post = 1;
    out->n_bins = r.n_bins;
    out->bin_index = r.bin_index.data();
    out->n_pos = r.n_pos;
    out->n_ori = r.n_ori;
    out->pos_off = r.pos_off.data();
    out->pos_members = r.pos_members.data();
    out->ori_pos_off = r.ori_pos_off.data();
    out->ori_off = r.ori_off.data();
    out->ori_members = r.ori_members.data();
    out->final_orientation = r.orient.data();
    out->final_pose = r.pose.data();
  }
  return SOD_OK;
}

// ---- fused pipeline -------------------------------------------------------------------
int sod_pipeline_enqueue(sod_ctx* ctx, const sod_pipeline_args* a) {
  SOD_TRY(set_dev(ctx, false));   // writes no buffer a pending PoseBin means reads
  if (!a) return sod_fail(ctx, SOD_EINVAL, "null args");
  if (!(a->ratio >= 0.0) || !std::isfinite(a->ratio))
    return sod_fail(ctx, SOD_EINVAL, "ratio must be a finite number >= 0");
  ctx->fuse_ratio = a->ratio;   // the final merge applies it too
  int rc = sod_match_enqueue(ctx);
  if (rc == SOD_OK) rc = sod_match_allgather_enqueue(ctx);
  ctx->fuse_ratio = -1.0;
  SOD_TRY(rc);
  SOD_TRY(sod_ratio_enqueue(ctx, a->ratio));
  SOD_TRY(sod_hough_select_enqueue(ctx, a->query_h, a->query_w, a->bins, a->vote_threshold));
  if (a->run_affine)
    SOD_TRY(sod_affine_enqueue(ctx, a->query_w, a->query_h, a->x_factor, a->y_factor,
                               a->affine_threshold));
  // the results' staging kernels right behind the pipeline (sod_results_fetch then only
  // waits): not while the boundary guard is armed (its host resolve may still patch them)
  if (a->stage_parts & ~SOD_RES_ALL) return sod_fail(ctx, SOD_EINVAL, "unknown result part");
  if (a->stage_parts && ctx->trig_exact && ctx->selected) {
    SOD_TRY(set_dev(ctx));   // the deferred PoseBin means run, the side stream joins
    SOD_TRY(sod_guard_resolve(ctx));
    ResLayout L;
    SOD_TRY(results_stage(ctx, a->stage_parts, &L));
    ctx->staged_L = L;
    ctx->staged_parts = a->stage_parts;
    ctx->staged_epoch = ctx->res_epoch;
  }
  return SOD_OK;
}

// ---- stateless batch forms ------------------------------------------------------------
int sod_pose_batch(sod_ctx* ctx, int64_t n, const float* mx, const float* my, const float* mangle,
                   const int32_t* moctave, const float* qx, const float* qy, const float* qangle,
                   const int32_t* qoctave, const double* cx, const double* cy, int32_t query_h,
                   int32_t query_w, const int32_t bins[4], double* pose, int32_t* idx) {
  SOD_TRY(set_dev(ctx));
  if (n < 0 || query_h < 1 || query_w < 1) return sod_fail(ctx, SOD_EINVAL, "bad arguments");
  if (n == 0) return SOD_OK;
  SOD_TRY(check_bins(ctx, bins));
  ctx->qh = query_h;
  ctx->qw = query_w;
  DevBuf<float> f[6];
  DevBuf<int32_t> o[2];
  DevBuf<double> c[2], dp, grec;
  DevBuf<int32_t> di;
  DevBuf<uint32_t> gst;
  int rc = SOD_OK;
  const float* fs[6] = {mx, my, mangle, qx, qy, qangle};
  for (int i = 0; i < 6 && rc == SOD_OK; ++i) rc = upload(ctx, f[i], fs[i], (size_t)n);
  if (rc == SOD_OK) rc = upload(ctx, o[0], moctave, (size_t)n);
  if (rc == SOD_OK) rc = upload(ctx, o[1], qoctave, (size_t)n);
  if (rc == SOD_OK) rc = upload(ctx, c[0], cx, (size_t)n);
  if (rc == SOD_OK) rc = upload(ctx, c[1], cy, (size_t)n);
  if (rc == SOD_OK) rc = sod_reserve(ctx, dp, (size_t)n * 4);
  if (rc == SOD_OK) rc = sod_reserve(ctx, di, (size_t)n * 4);
  if (rc == SOD_OK) rc = sod_reserve(ctx, grec, (size_t)n * 8);
  if (rc == SOD_OK) rc = sod_reserve(ctx, gst, 1);
  if (rc == SOD_OK && hipMemsetAsync(gst.p, 0, 4, ctx->stream) != hipSuccess)
    rc = sod_fail(ctx, SOD_EHIP, "guard counter reset failed");
  if (rc == SOD_OK)
    rc = launch_pose_batch(ctx, n, f[0].p, f[1].p, f[2].p, o[0].p, f[3].p, f[4].p, f[5].p, o[1].p,
                           c[0].p, c[1].p, dp.p, di.p, grec.p, gst.p);
  if (rc == SOD_OK) rc = download(ctx, pose, dp.p, (size_t)n * 4);
  if (rc == SOD_OK) rc = download(ctx, idx, di.p, (size_t)n * 4);
  uint32_t ng = 0;
  if (rc == SOD_OK) rc = download(ctx, &ng, gst.p, 1);
  if (rc == SOD_OK && sod_stream_sync(ctx->stream) != hipSuccess)
    rc = sod_fail(ctx, SOD_EHIP, "pose batch failed");
  (void)sod_stream_sync(ctx->stream);
  // boundary guard (hough.hip): the listed elements' x, y and x / y bins with glibc cos / sin
  if (rc == SOD_OK && ng) {
    std::vector<double> rec((size_t)ng * 8);
    rc = download(ctx, rec.data(), grec.p, rec.size());
    if (rc == SOD_OK && sod_stream_sync(ctx->stream) != hipSuccess)
      rc = sod_fail(ctx, SOD_EHIP, "guard records download failed");
    int64_t changed = 0;
    for (uint32_t i = 0; rc == SOD_OK && i < ng; ++i) {
      const double* r = &rec[(size_t)i * 8];
      const int64_t e = (int64_t)r[0];
      const int32_t ox = idx[4 * e], oy = idx[4 * e + 1];
      sod_guard_host_pose(r, ctx->bins, &pose[4 * e], &pose[4 * e + 1], &idx[4 * e], &idx[4 * e + 1]);
      changed += (ox != idx[4 * e]) || (oy != idx[4 * e + 1]);
    }
    ctx->guard_flagged = ng;
    ctx->guard_patched = changed;
    ctx->guard_flagged_total += ng;
    ctx->guard_patched_total += changed;
  } else if (rc == SOD_OK) {
    ctx->guard_flagged = ctx->guard_patched = 0;
  }
  for (auto& b : f) sod_release(b);
  for (auto& b : o) sod_release(b);
  for (auto& b : c) sod_release(b);
  sod_release(dp);
  sod_release(di);
  sod_release(grec);
  sod_release(gst);
  return rc;
}

int sod_affine_batch(sod_ctx* ctx, int64_t n_bins, const int64_t* offsets, const float* mx,
                     const float* my, const float* qx, const float* qy, const int32_t* i_sigma,
                     int32_t query_w, int32_t query_h, double x_factor, double y_factor,
                     int32_t threshold, int32_t max_iter, const double* params_in,
                     uint8_t* survived, int32_t* votes, double* params, uint8_t* member_alive) {
  SOD_TRY(set_dev(ctx));
  if (n_bins < 0 || !offsets || max_iter < 0 || !(x_factor != 0.0) || !(y_factor != 0.0))
    return sod_fail(ctx, SOD_EINVAL, "bad arguments");
  if (params_in && max_iter != 1)
    return sod_fail(ctx, SOD_EINVAL, "params_in requires max_iter = 1");
  if (n_bins == 0) return SOD_OK;
  const int64_t M = offsets[n_bins];
  for (int64_t i = 0; i < n_bins; ++i)
    if (offsets[i + 1] < offsets[i]) return sod_fail(ctx, SOD_EINVAL, "offsets not monotone");
  DevBuf<int64_t> off;
  DevBuf<float> p[4];
  DevBuf<int32_t> is, vo;
  DevBuf<uint8_t> sv, al;
  DevBuf<double> pr, pin;
  int rc = upload(ctx, off, offsets, (size_t)n_bins + 1);
  if (rc == SOD_OK && params_in) rc = upload(ctx, pin, params_in, (size_t)n_bins * 6);
  const float* ps[4] = {mx, my, qx, qy};
  for (int i = 0; i < 4 && rc == SOD_OK; ++i) rc = upload(ctx, p[i], ps[i], (size_t)M);
  if (rc == SOD_OK) rc = upload(ctx, is, i_sigma, (size_t)n_bins);
  if (rc == SOD_OK) rc = sod_reserve(ctx, vo, (size_t)n_bins);
  if (rc == SOD_OK) rc = sod_reserve(ctx, sv, (size_t)n_bins);
  if (rc == SOD_OK) rc = sod_reserve(ctx, al, (size_t)M);
  if (rc == SOD_OK) rc = sod_reserve(ctx, pr, (size_t)n_bins * 6);
  if (rc == SOD_OK)
    rc = launch_affine(ctx, n_bins, false, off.p, p[0].p, p[1].p, p[2].p, p[3].p, is.p, query_w,
                       query_h, nullptr, x_factor, y_factor, threshold, max_iter,
                       params_in ? pin.p : nullptr, sv.p, vo.p, pr.p, al.p, nullptr);
  if (rc == SOD_OK) rc = download(ctx, survived, sv.p, (size_t)n_bins);
  if (rc == SOD_OK) rc = download(ctx, votes, vo.p, (size_t)n_bins);
  if (rc == SOD_OK) rc = download(ctx, params, pr.p, (size_t)n_bins * 6);
  if (rc == SOD_OK) rc = download(ctx, member_alive, al.p, (size_t)M);
  if (rc == SOD_OK && sod_stream_sync(ctx->stream) != hipSuccess)
    rc = sod_fail(ctx, SOD_EHIP, "affine batch failed");
  (void)sod_stream_sync(ctx->stream);
  sod_release(off);
  for (auto& b : p) sod_release(b);
  sod_release(is); sod_release(vo); sod_release(sv); sod_release(al); sod_release(pr);
  sod_release(pin);
  return rc;
}

int sod_bin_index_batch(sod_ctx* ctx, int64_t n, const double* pose, int32_t query_h,
                        int32_t query_w, const int32_t bins[4], int32_t* idx) {
  SOD_TRY(set_dev(ctx));
  if (n < 0 || query_h < 1 || query_w < 1 || (n && (!pose || !idx)))
    return sod_fail(ctx, SOD_EINVAL, "bad arguments");
  if (n == 0) return SOD_OK;
  SOD_TRY(check_bins(ctx, bins));
  ctx->qh = query_h;
  ctx->qw = query_w;
  DevBuf<double> dp;
  DevBuf<int32_t> di;
  int rc = upload(ctx, dp, pose, (size_t)n * 4);
  if (rc == SOD_OK) rc = sod_reserve(ctx, di, (size_t)n * 4);
  if (rc == SOD_OK) rc = launch_bin_index_batch(ctx, n, dp.p, di.p);
  if (rc == SOD_OK) rc = download(ctx, idx, di.p, (size_t)n * 4);
  if (rc == SOD_OK && sod_stream_sync(ctx->stream) != hipSuccess)
    rc = sod_fail(ctx, SOD_EHIP, "bin index batch failed");
  (void)sod_stream_sync(ctx->stream);
  sod_release(dp);
  sod_release(di);
  return rc;
}

// ---- host-side exchange ---------------------------------------------------------------
int sod_match_candidates_get(sod_ctx* ctx, float* d1sq, int32_t* idx, float* d2sq) {
  SOD_TRY(set_dev(ctx));
  if (!ctx->matched) return sod_fail(ctx, SOD_ESTATE, "sod_match_enqueue first");
  const size_t n = (size_t)ctx->nq;
  SOD_TRY(download(ctx, d1sq, ctx->cd1.p, n));
  SOD_TRY(download(ctx, idx, ctx->cidx.p, n));
  SOD_TRY(download(ctx, d2sq, ctx->cd2.p, n));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  return SOD_OK;
}

int sod_match_candidates_merge(sod_ctx* ctx, int32_t nparts, const float* d1sq,
                               const int32_t* idx, const float* d2sq) {
  SOD_TRY(set_dev(ctx));
  if (!ctx->matched) return sod_fail(ctx, SOD_ESTATE, "sod_match_enqueue first");
  if (nparts < 1 || !d1sq || !idx || !d2sq) return sod_fail(ctx, SOD_EINVAL, "bad arguments");
  const size_t n = (size_t)ctx->nq, tot = n * (size_t)nparts;
  SOD_TRY(sod_stage_mark(ctx, kStageAllgather, false));
  SOD_TRY(upload(ctx, ctx->gd1, d1sq, tot));
  SOD_TRY(upload(ctx, ctx->gidx, idx, tot));
  SOD_TRY(upload(ctx, ctx->gd2, d2sq, tot));
  SOD_TRY(sod_stage_mark(ctx, kStageAllgather, true));
  SOD_TRY(sod_stage_mark(ctx, kStageMerge, false));
  SOD_TRY(launch_merge(ctx, ctx->gd1.p, ctx->gidx.p, ctx->gd2.p, nparts, (int64_t)n));
  SOD_TRY(sod_stage_mark(ctx, kStageMerge, true));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->ratio_done = ctx->houghed = ctx->selected = ctx->affined = false;
  return SOD_OK;
}

int sod_hough_partial_get(sod_ctx* ctx, uint32_t* counts, uint32_t* first) {
  SOD_TRY(set_dev(ctx));
  if (!ctx->houghed) return sod_fail(ctx, SOD_ESTATE, "sod_hough_enqueue first");
  SOD_TRY(sod_hist_dense(ctx));
  SOD_TRY(download(ctx, counts, ctx->counts.p, (size_t)ctx->nbins));
  SOD_TRY(download(ctx, first, ctx->first.p, (size_t)ctx->nbins));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  return SOD_OK;
}

int sod_hough_partial_set(sod_ctx* ctx, const uint32_t* counts, const uint32_t* first) {
  SOD_TRY(set_dev(ctx));
  if (!ctx->houghed) return sod_fail(ctx, SOD_ESTATE, "sod_hough_enqueue first");
  if (!counts || !first) return sod_fail(ctx, SOD_EINVAL, "bad arguments");
  SOD_TRY(sod_reserve(ctx, ctx->counts, (size_t)ctx->nbins));
  SOD_TRY(sod_reserve(ctx, ctx->first, (size_t)ctx->nbins));
  ctx->hist_dense = true;
  SOD_TRY(sod_stage_mark(ctx, kStageAllreduce, false));
  SOD_HIP(ctx, hipMemcpyAsync(ctx->counts.p, counts, ctx->nbins * 4, hipMemcpyHostToDevice, ctx->stream));
  SOD_HIP(ctx, hipMemcpyAsync(ctx->first.p, first, ctx->nbins * 4, hipMemcpyHostToDevice, ctx->stream));
  SOD_TRY(sod_stage_mark(ctx, kStageAllreduce, true));
  SOD_HIP(ctx, sod_stream_sync(ctx->stream));
  ctx->selected = ctx->affined = false;
  return SOD_OK;
}

// ---- RCCL -----------------------------------------------------------------------------
int sod_comm_unique_id(uint8_t out[SOD_UNIQUE_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == SOD_UNIQUE_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    g_err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return SOD_ECOMM;
  }
  std::memcpy(out, &id, sizeof(id));
  return SOD_OK;
}

int sod_comm_init(sod_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t id[SOD_UNIQUE_ID_BYTES]) {
  SOD_TRY(set_dev(ctx));
  if (nranks < 1 || rank < 0 || rank >= nranks) return sod_fail(ctx, SOD_EINVAL, "bad rank");
  if (ctx->comm) {
    ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  ctx->nranks = nranks;
  ctx->rank = rank;
  // nranks == 1 also builds a communicator: the collectives then run (as copies), which is
  // how the RCCL path is exercised on a one-GPU machine.  Under a CU split the collectives
  // run on the reserved CUs only, so the communicator is created with at most that many
  // blocks per collective (ncclConfig_t.maxCTAs: a per-communicator setting, unlike the
  // NCCL_MAX_NCHANNELS environment variable, which RCCL reads once per process)
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  int cap = 0;
  if (ctx->reserved_cus > 0) {
    cap = ctx->reserved_cus;
    cfg.minCTAs = 1;
    cfg.maxCTAs = cap;
  }
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  const ncclResult_t r = ncclCommInitRankConfig(&ctx->comm, nranks, uid, rank, &cfg);
  if (r != ncclSuccess) {
    ctx->comm = nullptr;
    return sod_fail(ctx, SOD_ECOMM, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
  }
  ctx->comm_max_channels = cap;
  return SOD_OK;
}

int sod_comm_info(sod_ctx* ctx, int32_t* nranks, int32_t* rank) {
  if (!ctx || !nranks || !rank) return SOD_EINVAL;
  if (!ctx->comm) return sod_fail(ctx, SOD_ESTATE, "no RCCL communicator (sod_comm_init)");
  int n = 0, r = -1;
  ncclResult_t e = ncclCommCount(ctx->comm, &n);
  if (e == ncclSuccess) e = ncclCommUserRank(ctx->comm, &r);
  if (e != ncclSuccess)
    return sod_fail(ctx, SOD_ECOMM, std::string("ncclCommCount/UserRank: ") + ncclGetErrorString(e));
  *nranks = n;
  *rank = r;
  return SOD_OK;
}

}  // extern "C"
