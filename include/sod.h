/*
 * sod.h -- C ABI of libsod.so, the MI355X-native hot path of torn8to/sift-based-OD.
 *
 * Path (BASELINE.json north_star):
 *   brute-force SIFT matching k=2 + Lowe ratio  -> generalized-Hough pose-bin voting
 *   -> per-bin affine least-squares verification with outlier rejection.
 *
 * The reference has no FFI: its boundary is Python calls (main.py:6-11 `from X import *`)
 * plus OpenCV.  Each entry point below names the reference interface it replaces; the
 * Python package sift-based-od_amd/ binds them with ctypes.
 *
 * Conventions
 *   - Every function returns int status: SOD_OK (0) or a SOD_E* code; the message is
 *     available from sod_last_error(ctx).  Nothing aborts.
 *   - Host pointers are borrowed for the duration of the call, C-contiguous.
 *   - Device memory is owned by the ctx.  "enqueue" functions only enqueue work on the
 *     ctx's HIP stream; "get" functions synchronise the stream and copy to the host.
 *   - One ctx = one GPU = one host thread.  Multi-GPU = one process per GPU, each with
 *     its own ctx, joined by sod_comm_init (RCCL over xGMI).
 *   - Descriptors must be integer valued in [0,255] (OpenCV SIFT); float input is
 *     validated on the device and rejected otherwise (SOD_EINVAL).
 */
#ifndef SOD_H
#define SOD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SOD_OK 0
#define SOD_EINVAL 1   /* bad argument / invalid descriptor values            */
#define SOD_EHIP 2     /* HIP runtime error                                    */
#define SOD_ENOMEM 3   /* device allocation failed                             */
#define SOD_ESTATE 4   /* call out of order (e.g. hough before match)          */
#define SOD_ECOMM 5    /* RCCL error / communicator missing                    */

#define SOD_DTYPE_U8 0
#define SOD_DTYPE_F32 1

#define SOD_UNIQUE_ID_BYTES 128

typedef struct sod_ctx sod_ctx;

/* ---- lifetime --------------------------------------------------------------------- */
int sod_abi_version(void);
/* HIP devices visible to this process (a launcher maps one rank to each). */
int sod_device_count(int* n);
int sod_create(int device, sod_ctx** out);
void sod_destroy(sod_ctx* ctx);
const char* sod_last_error(const sod_ctx* ctx);
int sod_synchronize(sod_ctx* ctx);
/* Kernel timing of the last enqueued matcher launch (ms), measured with HIP events on
 * the ctx stream; SOD_ESTATE when that launch was not timed (sod_set_match_timing). */
int sod_last_match_ms(sod_ctx* ctx, float* ms);
/* Kernel times (ms) of the last n matcher launches, oldest first (n <= 64 and <= launches
 * so far), from begin/end HIP events recorded on the matcher's stream around each launch:
 * the kernel timed inside a pipelined run.  Waits for those launches. */
int sod_match_times(sod_ctx* ctx, int n, float* ms);
/* Device time (ms) of each stage of the last step (since the last sod_match_enqueue /
 * sod_matches_set), from begin / end events recorded on the stream around the stage's own
 * launches -- host work and waits between two calls (a host-staged exchange, other ranks)
 * are not counted: [0 matcher kernel, 1 merge + ratio kernels, 2 Hough pose + vote,
 * 3 select + members (+ PoseBin means fork), 4 affine, 5 all-reduce of the bin counts (or
 * the host exchange's upload), 6 all-gather of the candidates (or its upload)].  The matcher
 * entry is 0 when the step's launch was not timed (sod_set_match_timing stride > 1). */
int sod_last_stage_ms(sod_ctx* ctx, float* ms_out, int n);
/* Stage events (the bounds sod_last_stage_ms reads) on (1) or off (0, the default since
 * round 6): each is a marker packet on the tail's critical path (~5 us before the next
 * kernel; one query image's chain carried ~30 us of them).  With them off, sod_last_stage_ms
 * reports 0 for the stages after the matcher. */
int sod_set_stage_timing(sod_ctx* ctx, int on);
/* Begin / end events of every `on`-th int8 matcher launch, counted from this call (1: every
 * launch; 0: none, the default since round 6; sod_match_times and sod_last_match_ms read the
 * recorded ones): a dispatch that records an event delays its stream's next kernel by ~5 us,
 * a share of a one-image step.  An untimed matcher-stream launch is joined by a marker
 * event. */
int sod_set_match_timing(sod_ctx* ctx, int on);
/* Matcher streams with sod_match_set_overlap / sod_set_cu_reserve: 1 (default) = one stream
 * for both partial-result slots; 2 = one per slot, so consecutive launches overlap at their
 * boundary (higher throughput for mid-size query sets; a launch's events then span the
 * overlap).  Results are unchanged. */
int sod_set_matcher_streams(sod_ctx* ctx, int n);
/* Host time (ns) the enqueue calls spent BLOCKED waiting for the device since the last reset:
 * a matcher launch waits for the merge that last read its partial-result slot (two launches
 * in flight at most).  Enqueue wall time minus this is the host's own work.  reset != 0 zeroes
 * the counter after reading it.  (No reference counterpart: measurement.) */
int sod_host_wait_ns(sod_ctx* ctx, int64_t* ns, int reset);

/* ---- database (replaces main.py:36-66 flattening + GenerateDatabaseInfo.py format) --
 * Keypoints and the per-image table cover the WHOLE database (replicated on every
 * rank); descriptors may be a shard: rows [row_offset, row_offset + n) of it. */
int sod_db_set_keypoints(sod_ctx* ctx, int64_t n_total, const float* x, const float* y,
                         const float* angle, const int32_t* octave, const int32_t* img,
                         int32_t n_images, const double* centroid /* [n_images*2] */,
                         const int32_t* size /* [n_images*2] (w,h) */);
int sod_db_upload_descriptors(sod_ctx* ctx, const void* des, int dtype, int64_t n,
                              int64_t row_offset);

/* dst uses src's resident database (keypoints, image table, packed descriptors) without
 * a copy: several contexts -- each with its own stream and query state -- serve query
 * images concurrently over one DB.  src counts its sharers: while any exists, every DB
 * write on src (set_keypoints, upload_descriptors, import_packed, set_impl) fails with
 * SOD_ESTATE.  A DB write on dst first detaches it (dst then holds no DB until it uploads
 * one of its own).  Destroying src waits for its sharers' queued work and detaches them.
 * Contexts sharing a DB must not be driven concurrently from different host threads. */
int sod_db_share(sod_ctx* dst, sod_ctx* src);

/* ---- packed DB image (replaces the GenerateDatabaseInfo.py:35 pickle
 * + main.py:53-66 flattening as the descriptor store): the device's own fragment layout
 * with its norm words behind a 64-byte header, so a later upload is one copy (no
 * validation / packing pass).  The image is tied to the matcher impl it was packed for. */
int sod_db_packed_size(sod_ctx* ctx, int64_t* bytes);
int sod_db_export_packed(sod_ctx* ctx, void* out, int64_t bytes);
int sod_db_import_packed(sod_ctx* ctx, const void* in, int64_t bytes);

/* ---- query image features (replaces main.py:43 detectAndCompute output) ---------- */
int sod_query_upload(sod_ctx* ctx, const void* des, int dtype, int32_t nq,
                     const float* x, const float* y, const float* angle,
                     const int32_t* octave);   /* des may be NULL: keypoints only */

/* ---- query batching -------------------------------------------
 * Upload the keypoints/descriptors of several query images back to back, match and
 * ratio-test them in ONE pass over the DB, then run the per-image stages (Hough, select,
 * affine, post-processing) with the window set to each image's query range [first,
 * first+count); member lists then hold window-local query indices.  count < 0 restores
 * the whole query set (the default after sod_query_upload). */
int sod_query_window(sod_ctx* ctx, int32_t first, int32_t count);
/* The same batch with the per-image stages FUSED: declare the images (query offsets
 * [n+1] covering all uploaded queries, shapes [n*2] = rgb_query.shape (h, w) each); then
 * ONE sod_hough_enqueue / sod_select_enqueue / sod_affine_enqueue / sod_postprocess
 * covers every image (their query_h / query_w arguments are ignored): the bin key space is
 * image-major (image * nbins + bin), valid bins come out image by image in each image's
 * reference order, member lists hold batch-global query indices, and
 * sod_valid_images_get gives each valid bin's image.  n_images = 0 returns to one image. */
int sod_query_images(sod_ctx* ctx, int32_t n_images, const int32_t* q_offsets,
                     const int32_t* shapes);
int sod_valid_images_get(sod_ctx* ctx, int32_t* image /* [V] */);

/* ---- A1/A2: cv2.BFMatcher().knnMatch(des_query, des, k=2) + ratio test ------------
 * main.py:70-86.  enqueue: local shard top-2 (exact squared distances), merged over
 * this ctx's descriptor shard. */
int sod_match_enqueue(sod_ctx* ctx);
/* Matcher implementation: 1 = int8 MFMA 16x16x64 (default, fastest), 2 = int8 MFMA
 * 32x32x32, 0 = bf16 MFMA.  int8: values shifted by -128, exact i32 dot products, 2x the
 * bf16 MFMA rate.  All are bit-exact; call before the descriptor uploads (the packed
 * layouts differ; switching drops uploaded descriptors). */
int sod_match_set_impl(sod_ctx* ctx, int impl);
/* Kernel shape of the int8 16x16x64 matcher (impl 1): 0 = by query count (default), 1 =
 * the LDS-ring kernel (queries stationary, 2-8 tiles per wave, DB through LDS) -- the one
 * shape since round 6; 2 (the register-streamed kernel, 2x slower at every measured size,
 * EXPERIMENTS.md) is refused with SOD_EINVAL.  Replaces cv2.BFMatcher().knnMatch's loop
 * (main.py:70-71). */
int sod_match_set_kernel(sod_ctx* ctx, int kernel);
/* 1 when the device's cos / sin (a restatement of glibc 2.35's x86_64 FMA-variant sin / cos,
 * glibc_trig.h) equal this host's libm bit for bit -- the math.cos / math.sin that
 * estimate_object_pose calls (HoughTransformHelperFunctions.py:31-32): poses, bin indices and
 * PoseBin means (PoseBin.py:20-28) are then the reference's with no host redo.  0: another
 * libm; the boundary guard and the exact-means redo then re-do the affected values with it. */
int sod_trig_exact(sod_ctx* ctx);
/* the device's glibc sin / cos of n angles (host arrays; |x| < 105414350): a test hook */
int sod_glibc_sincos(sod_ctx* ctx, int64_t n, const double* x, double* s, double* c);
/* Tuning / test switches of this context, by name (integers; read at the next enqueue).
 * sod_create seeds each from the environment variable SOD_<NAME> once.  Names: match_qt,
 * match_pf, match_pair (LDS-ring matcher tiles per wave / prefetch / waves per query slice), hough_fused (0: never the
 * one-work-group Hough kernel), select_multi (1: multi-kernel selection for small windows),
 * sift_stream_mask, sift_sort_max, sift_desc_range_max, sift_layer_split, sift_side_mask,
 * sift_fork2, sift_early_desc, sift_direct, sift_eager_rank (SIFT scheduling A/B and the
 * rank / ranged-enumeration test paths), debug_sync (stderr trace of long stream waits)
 * change no result; affine_fma (1: remove_outliers' np.matmul(M, X), AffineParameters.py:145,
 * evaluated as fma(m1, x, m2 y) like the host numpy's BLAS on an FMA CPU; 0: two roundings)
 * selects the reference's own rounding, which the Python layer probes once per process.
 * SOD_EINVAL for an unknown name. */
int sod_set_option(sod_ctx* ctx, const char* name, int64_t value);
int sod_get_option(sod_ctx* ctx, const char* name, int64_t* value);
/* Matcher on a stream of its own (1) or on the context stream (0, default).  With 1 the
 * matcher kernel of the next sod_match_enqueue / sod_pipeline_enqueue only waits for the
 * previous merge of its partial results (and for the last descriptor upload), so it overlaps
 * the previous query's Hough / select / affine stages, which stay on the context stream in
 * order (RCCL collectives included).  The host thread waits inside the enqueue until
 * that merge (two launches back) is done, so at most two matcher launches per context are
 * in flight.  Results are unchanged. */
int sod_match_set_overlap(sod_ctx* ctx, int on);
/* Split the CUs: the matcher stream keeps all but `per_xcd` CUs of every XCD, the context
 * and side streams (Hough / select / affine, merges, RCCL collectives, memsets) run on those
 * reserved CUs, so one query's tail stages run beside the next query's matcher instead of
 * being starved by it.  Implies sod_match_set_overlap(ctx, 1); 0 restores unmasked streams.
 * Meant for streaming query batches through sod_pipeline_enqueue: every other entry point on
 * the context stream (SIFT, uploads) also runs on the reserved CUs while it is set.
 * Results are unchanged.  (No reference counterpart: an MI355X scheduling knob.)
 * SOD_EINVAL on a device other than a whole MI355X (gfx950, 8 XCDs, 256 CUs: the CU-mask
 * layout it relies on was measured there).  With an RCCL communicator every block of a
 * collective must fit the reserved CUs: sod_comm_init under an active split creates the
 * communicator with ncclConfig_t.maxCTAs = the reserved CU count, and this call fails with
 * SOD_ESTATE on a communicator created with more (or RCCL's default) blocks per collective. */
int sod_set_cu_reserve(sod_ctx* ctx, int per_xcd);
/* multi-GPU: RCCL all-gather of every rank's per-query (d1^2, idx1, d2^2) and the
 * global merge.  No-op on a single rank. */
int sod_match_allgather_enqueue(sod_ctx* ctx);
/* ratio test on the merged top-2: good = (double)d1 < ratio * (double)d2 (main.py:82). */
int sod_ratio_enqueue(sod_ctx* ctx, double ratio);
int sod_match_get(sod_ctx* ctx, int32_t* idx1, float* d1, float* d2, uint8_t* good);
/* Set the match state directly (Main.matching_keypoints assigned by the caller,
 * main.py:29,85): idx1[q] = trainIdx (global row), good[q] = keep.  nq must equal the
 * uploaded query count.  Hough/select/affine then run on these matches. */
int sod_matches_set(sod_ctx* ctx, int32_t nq, const int32_t* idx1, const uint8_t* good);
/* knnMatch's trainIdx pair as OpenCV returns it (main.py:71: m.trainIdx, n.trainIdx --
 * main.py reads only n.distance, but OpenCV fills both).  OpenCV orders by the float
 * distance sqrtf(d^2) with ties to the lower trainIdx: idx1 = the lowest row at the float
 * d1 (the matcher's own idx1 whenever every distance is < 2048, sod_match_exact_order),
 * idx2 = the lowest other row at the float d2 (-1 with a single DB row) -- found by MFMA
 * passes over the DB after an int8 (impl 1, default) or bf16 (impl 0) match, single
 * context.  SOD_ESTATE after sod_matches_set (no distances) or with impl 2. */
int sod_match_knn_indices(sod_ctx* ctx, int32_t* idx1, int32_t* idx2);
/* Make the device's trainIdx (what the Hough stage reads) OpenCV's: main.py:85 reads
 * m.trainIdx of knnMatch, whose order is the float distance.  A no-op when
 * sod_match_exact_order holds (always for SIFT input); otherwise idx1 is replaced by
 * sod_match_knn_indices' idx1 on the device.  Call after sod_ratio_enqueue. */
int sod_match_float_order(sod_ctx* ctx);
/* 1 if every distance is provably < 2048 (sqrtf then injective on the squared
 * distances, so squared-distance ordering == OpenCV's float ordering), else 0. */
int sod_match_exact_order(sod_ctx* ctx, int* exact);

/* ---- A5-A8: estimate_object_pose / calculate_bin_index / vote loop / PoseBin -------
 * HoughTransformHelperFunctions.py:4-72, main.py:89-119, PoseBin.py:6-51.
 * query_shape = rgb_query.shape[:2] = (H, W).  bins[4] = (x, y, theta, sigma) bins,
 * each in [1,255] (the live code passes one scalar for all four).  Votes are cast only
 * for good matches whose idx1 lies in [own_lo, own_hi) (this rank's shard). */
int sod_hough_enqueue(sod_ctx* ctx, int32_t query_h, int32_t query_w, const int32_t bins[4],
                      int64_t own_lo, int64_t own_hi);
/* multi-GPU: RCCL all-reduce (sum) of the partial bin counts and (min) of the
 * first-touch ordinals.  No-op on a single rank. */
int sod_hough_allreduce_enqueue(sod_ctx* ctx);
/* A10: bins with votes >= threshold in first-touch (dict insertion) order
 * (main.py:121-132), their member lists in match order, and the PoseBin running means
 * (centroid x,y, angle, scale, img_size w,h) in vote order. */
int sod_select_enqueue(sod_ctx* ctx, int32_t vote_threshold);
/* main.py:89-132 as one call: sod_hough_enqueue over this rank's shard (all rows on one
 * rank), the all-reduce, sod_select_enqueue.  One image of <= 1024 queries (kFusedQ) on one rank runs
 * as ONE kernel (pose, votes, valid bins, members, the affine inputs) without the dense bin
 * histogram, which readers that need it (sod_bins_*, another threshold, the host exchange)
 * build on demand; results identical either way.  sod_pipeline_enqueue uses it. */
int sod_hough_select_enqueue(sod_ctx* ctx, int32_t query_h, int32_t query_w,
                             const int32_t bins[4], int32_t vote_threshold);
int sod_valid_counts(sod_ctx* ctx, int64_t* n_valid, int64_t* n_members);
int sod_valid_get(sod_ctx* ctx, int32_t* keys /* [V*4] */, int32_t* votes /* [V] */,
                  int64_t* offsets /* [V+1] */, int32_t* members /* [M] query idx */,
                  double* means /* [V*6] */);
/* all occupied bins (counts), first-touch order: keys[B*4], votes[B] */
int sod_bins_count(sod_ctx* ctx, int64_t* n_bins);
int sod_bins_get(sod_ctx* ctx, int32_t* keys, int32_t* votes);
/* Boundary guard of HTHF:31-35,49-58 (x, y through cos / sin): the device lists every
 * match whose x or y bin could depend on the last ulp of cos / sin and the library redoes
 * it with the host's libm (the calls math.cos / math.sin make), then, if a bin changed, the
 * histogram and the stages after it -- before any Hough result is read.  Reports the last
 * Hough launch's (or sod_pose_batch's) listed matches and changed bins, and the running
 * totals of this context. */
int sod_hough_guard_stats(sod_ctx* ctx, int64_t* flagged, int64_t* changed,
                          int64_t* flagged_total, int64_t* changed_total);

/* ---- A11-A13: AffineParameters / remove_outliers / apply_affine_parameters -------
 * AffineParameters.py:89-160, main.py:139-157: per valid bin, fixed point of
 * {x = pinv(A^T A) A^T b ; drop members with |residual| > W*pose[3]/xf (x) or
 *  H*pose[3]/yf (y)} until nothing is dropped; survivors keep votes >= threshold. */
int sod_affine_enqueue(sod_ctx* ctx, int32_t query_w, int32_t query_h, double x_factor,
                       double y_factor, int32_t threshold);
int sod_affine_get(sod_ctx* ctx, uint8_t* survived /* [V] */, int32_t* votes /* [V] */,
                   double* params /* [V*6] m1,m2,m3,m4,tx,ty */,
                   uint8_t* member_alive /* [M] */);

/* ---- post-processing (PostProcessing.py:4-112, main.py:159-168) --
 * group_position -> group_orientation -> find_max_orientation -> get_final_pose over the
 * surviving bins (or the valid bins when no affine pass ran), in their list order.
 * Outputs (caller-sized by the bin count n; every array may be NULL):
 *   n_pos position clusters; pos_off[n_pos+1] / pos_members[n]: bin indices (into the
 *     post-processed list) in the reference's DFS order;
 *   n_ori orientation clusters; ori_pos_off[n_pos+1] = each position cluster's range of
 *     orientation clusters; ori_off[n_ori+1] / ori_members[n]: bin indices;
 *   final_orientation[n_pos]; final_pose[n_pos*6] = (x, y, orientation, scale, w, h) as
 *     main.py's final_pose ((x, y), orientation, scale, (w, h)). */
int sod_postprocess(sod_ctx* ctx, int32_t* n_bins, int32_t* bin_index /* [n] valid index */,
                    int32_t* n_pos, int32_t* pos_off, int32_t* pos_members, int32_t* n_ori,
                    int32_t* ori_pos_off, int32_t* ori_off, int32_t* ori_members,
                    double* final_orientation, double* final_pose);
/* sod_postprocess's input means: 1 (default) = the survivors' x / y PoseBin means redone
 * on the host with glibc cos / sin per member (the calls math.cos / math.sin make,
 * HoughTransformHelperFunctions.py:31-32), so the position relation's <= thresholds
 * (PostProcessing.py:24-28) and the final pose see the reference's values bit for bit;
 * 0 = the device means (device cos / sin: within ~1e-12, no host pass). */
int sod_set_post_exact(sod_ctx* ctx, int on);
/* The x / y PoseBin means (PoseBin.py:45-51) of valid bins vbin[0..nb) as the reference
 * computes them (glibc cos / sin per member pose, HoughTransformHelperFunctions.py:31-32),
 * into xy[2*nb]; what sod_postprocess uses when sod_set_post_exact is on. */
int sod_exact_means(sod_ctx* ctx, int32_t nb, const int32_t* vbin, double* xy);
/* the same on caller-supplied PoseBin means [n*6] = (x, y, angle, scale, w, h) */
int sod_post_batch(sod_ctx* ctx, int32_t n, const double* means, int32_t* n_pos,
                   int32_t* pos_off, int32_t* pos_members, int32_t* n_ori,
                   int32_t* ori_pos_off, int32_t* ori_off, int32_t* ori_members,
                   double* final_orientation, double* final_pose);

/* ---- whole pipeline on one stream (bench / Main fast path) ------------------------ */
typedef struct sod_pipeline_args {
  double ratio;           /* 0.75  main.py:82            */
  int32_t query_h, query_w;
  int32_t bins[4];        /* 15,15,15,15 main.py:183      */
  int32_t vote_threshold; /* 5     main.py:184            */
  int32_t affine_threshold; /* 4   main.py:185            */
  double x_factor, y_factor; /* 128 = pos_factor*4 main.py:141,150 */
  int32_t run_affine;
  /* SOD_RES_* parts to stage right behind the pipeline (0: none): the next
   * sod_results_fetch of those parts only waits, when no other call came in between */
  int32_t stage_parts;
} sod_pipeline_args;
int sod_pipeline_enqueue(sod_ctx* ctx, const sod_pipeline_args* args);

/* Results of the enqueued pipeline in ONE device -> host transfer (main.py's per-image
 * reads, main.py:182-186, without a copy and a wait per array): one kernel writes the
 * requested parts -- SOD_RES_MATCH the match arrays, SOD_RES_VALID the valid bins (keys
 * decoded on the host, votes, offsets, members, PoseBin means), SOD_RES_AFFINE the affine
 * results, SOD_RES_POST the survivors' post-processing (relations on the device) -- into
 * page-locked host memory the context owns (or finds them there, staged by the pipeline
 * enqueue: sod_pipeline_args.stage_parts); one wait; the post-processing walk
 * (sod_postprocess's outputs) then runs on the host.  Pointers stay valid until the next
 * sod_results_fetch, staging pipeline enqueue or sod_destroy.  SOD_ESTATE without sod_ratio_enqueue (MATCH) or
 * sod_select_enqueue (the other parts); AFFINE before sod_affine_enqueue and parts not
 * requested come back with count 0 / NULL.  The
 * same values as sod_match_get, sod_valid_get, sod_affine_get and sod_postprocess, bit for
 * bit. */
#define SOD_RES_MATCH 1
#define SOD_RES_VALID 2
#define SOD_RES_AFFINE 4
#define SOD_RES_POST 8
#define SOD_RES_ALL 15
typedef struct sod_results {
  int64_t nq;                       /* queries (0 without SOD_RES_MATCH) */
  const int32_t* idx1;              /* [nq] */
  const float* d1;                  /* [nq] */
  const float* d2;                  /* [nq] */
  const uint8_t* good;              /* [nq] */
  int32_t selected;                 /* 1: the valid-bin arrays below are set */
  int64_t n_valid, n_members;
  const int32_t* keys;              /* [n_valid*4] */
  const int32_t* votes;             /* [n_valid] */
  const int64_t* offsets;           /* [n_valid+1] */
  const int32_t* members;           /* [n_members] */
  const double* means;              /* [n_valid*6] */
  int32_t affined;                  /* 1: the affine arrays below are set */
  const uint8_t* survived;          /* [n_valid] */
  const int32_t* affine_votes;      /* [n_valid] */
  const double* params;             /* [n_valid*6] */
  const uint8_t* alive;             /* [n_members] */
  int32_t post;                     /* 1: the post-processing outputs below are set */
  int32_t n_bins;                   /* post-processed bins (survivors, or valid bins) */
  const int32_t* bin_index;         /* [n_bins] valid-bin index of each */
  int32_t n_pos, n_ori;
  const int32_t* pos_off;           /* [n_pos+1] */
  const int32_t* pos_members;       /* [n_bins] */
  const int32_t* ori_pos_off;       /* [n_pos+1] */
  const int32_t* ori_off;           /* [n_ori+1] */
  const int32_t* ori_members;       /* [n_bins] */
  const double* final_orientation;  /* [n_pos] */
  const double* final_pose;         /* [n_pos*6] */
} sod_results;
int sod_results_fetch(sod_ctx* ctx, int parts, sod_results* out);

/* ---- stateless batch forms of the per-item reference functions -------------------- */
/* estimate_object_pose + calculate_bin_index for n (model kp, query kp, centroid)
 * triples: pose[n*4] = (x, y, alpha, scale_factor), idx[n*4] = (ix, iy, itheta, isigma). */
int sod_pose_batch(sod_ctx* ctx, int64_t n, const float* mx, const float* my,
                   const float* mangle, const int32_t* moctave, const float* qx,
                   const float* qy, const float* qangle, const int32_t* qoctave,
                   const double* cx, const double* cy, int32_t query_h, int32_t query_w,
                   const int32_t bins[4], double* pose, int32_t* idx);
/* calculate_bin_index for n given poses (x, y, alpha, scale_factor): idx[n*4]. */
int sod_bin_index_batch(sod_ctx* ctx, int64_t n, const double* pose, int32_t query_h,
                        int32_t query_w, const int32_t bins[4], int32_t* idx);
/* AffineParameters + remove_outliers fixed point for host-provided bins (CSR):
 * model/query points per member (f32, as cv2.KeyPoint.pt), i_sigma = pose[3] per bin.
 * max_iter = 0: AffineParameters only (params, nothing removed);
 * max_iter = 1: one {AffineParameters; remove_outliers} round;
 * params_in != NULL (with max_iter = 1): remove_outliers with the given params
 * (posebin.affine_parameters) instead of solving. */
int sod_affine_batch(sod_ctx* ctx, int64_t n_bins, const int64_t* offsets,
                     const float* mx, const float* my, const float* qx, const float* qy,
                     const int32_t* i_sigma, int32_t query_w, int32_t query_h,
                     double x_factor, double y_factor, int32_t threshold, int32_t max_iter,
                     const double* params_in, uint8_t* survived, int32_t* votes,
                     double* params, uint8_t* member_alive);

/* ---- SIFT detect + describe on the device ------------------------
 * Replaces `sift = cv2.SIFT_create()` + `sift.detectAndCompute(gray, None)` (main.py:179,
 * :43; GenerateDatabaseInfo.py:16, :32).  OpenCV's algorithm (restated in
 * oracle/sift_oracle.c) with default parameters unless sod_sift_set_params is called
 * (nfeatures is applied by the Python layer).  detect runs the whole pyramid / extrema /
 * orientation / ordering / descriptor pipeline on the device and returns the keypoint
 * count; the keypoints are in OpenCV's output order (sorted by x, y, -size, angle,
 * -response, -octave, duplicates removed) with OpenCV's fields (pt in input pixels, size,
 * angle in degrees, response, packed octave) and descriptors are integer-valued floats
 * [n*128].  detect_bgr takes an interleaved 8-bit BGR image (cvtColor BGR2GRAY first). */
int sod_sift_set_params(sod_ctx* ctx, int32_t n_octave_layers, double contrast_threshold,
                        double edge_threshold, double sigma);
/* Orientation / descriptor histogram adds.  OpenCV sums each bin in sample order
 * (calcOrientationHist / calcSIFTDescriptor); the device keeps that order either with one
 * lane per sample (ordered) or with whole-wave adds whose same-bin lanes gfx950 applies in
 * lane order -- an undocumented property, so the context checks it on the device at its
 * first SIFT call (one wave, 512 order-sensitive trials) and uses the wave adds only when
 * it holds (and only on gfx950).  mode -1 = that automatic choice (default), 0 = always
 * the ordered adds.  sod_sift_lane_order reports the active path (1 = wave adds) and the
 * self-check result (1 = lane order held, 0 = not, -1 = not run). */
int sod_sift_set_lane_order(sod_ctx* ctx, int mode);
int sod_sift_lane_order(sod_ctx* ctx, int* active, int* probe_ok);
int sod_sift_detect(sod_ctx* ctx, const uint8_t* gray /* [h*w] */, int32_t width,
                    int32_t height, int32_t* n_keypoints);
int sod_sift_detect_bgr(sod_ctx* ctx, const uint8_t* bgr /* [h*w*3] */, int32_t width,
                        int32_t height, int32_t* n_keypoints);
/* several images (GenerateDatabaseInfo.py:19-37's loop, or a batch of query images):
 * images[i] is [h_i*w_i*channels_i] 8-bit (channels 1 = gray, 3 = BGR; channels may be
 * NULL = all gray); counts[i] = keypoints of image i.  Four images are in flight at once,
 * each on its own stream; the results are concatenated in image order. */
int sod_sift_detect_batch(sod_ctx* ctx, int32_t n_images, const uint8_t* const* images,
                          const int32_t* widths, const int32_t* heights, const int32_t* channels,
                          int32_t* counts);
/* copies the first min(total, cap) keypoints of the last detect / batch out (image order);
 * every pointer may be NULL */
int sod_sift_get(sod_ctx* ctx, int64_t cap, float* x, float* y, float* size, float* angle,
                 float* response, int32_t* octave, float* descriptors /* [cap*128] */);
/* the last detection becomes the query set (descriptors + keypoints, device to device):
 * main.py's get_query_features followed by run_matcher without a host round trip; a batch
 * is also declared as query images (sod_query_images) for the fused per-image stages */
int sod_sift_to_queries(sod_ctx* ctx);

/* ---- host-side exchange (multi-rank over a host communicator, e.g. gloo) ------------
 * The same two exchange steps as the RCCL path, with the data staged through the host:
 * candidates_get -> all-gather -> candidates_merge; partial_get -> all-reduce ->
 * partial_set.  Used when no RCCL communicator is available (and by the tests). */
int sod_match_candidates_get(sod_ctx* ctx, float* d1sq, int32_t* idx, float* d2sq);
int sod_match_candidates_merge(sod_ctx* ctx, int32_t nparts, const float* d1sq,
                               const int32_t* idx, const float* d2sq);
int sod_hough_partial_get(sod_ctx* ctx, uint32_t* counts, uint32_t* first);
int sod_hough_partial_set(sod_ctx* ctx, const uint32_t* counts, const uint32_t* first);

/* ---- multi-GPU (RCCL over xGMI) --------------------------------------------------- */
int sod_comm_unique_id(uint8_t out[SOD_UNIQUE_ID_BYTES]);
int sod_comm_init(sod_ctx* ctx, int32_t nranks, int32_t rank,
                  const uint8_t id[SOD_UNIQUE_ID_BYTES]);
/* The ctx's RCCL communicator as RCCL itself reports it (ncclCommCount,
 * ncclCommUserRank): a multi-GPU record can show that the collectives ran over nranks
 * ranks.  SOD_ESTATE when no communicator was created.  (No reference counterpart.) */
int sod_comm_info(sod_ctx* ctx, int32_t* nranks, int32_t* rank);

#ifdef __cplusplus
}
#endif
#endif /* SOD_H */
