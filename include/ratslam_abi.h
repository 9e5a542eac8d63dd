/*
 * ratslam_abi.h -- C ABI of libratslam_hip.so, the MI355X (gfx950) hot path of
 * pyratslam: the pose-cell network step and the view-template matcher.
 *
 * Plain C types only (pointers + sizes); every entry point returns an int
 * status (RS_OK == 0) and leaves a thread-local message in rs_last_error().
 * Host buffers are caller-owned and copied during the call; device memory is
 * owned by the handle.  A handle is not re-entrant: callers serialise calls on
 * one handle (the Python wrapper holds a per-handle lock); distinct handles may
 * be used from different threads concurrently (ros_simulate.py:103 vs :135).
 * Calls may return once their results have reached host memory, before the
 * device work they queued has retired: a fault or launch error in that work is
 * then returned (RS_ERR_HIP) by a later call on the same handle that waits for
 * its stream -- at the latest by rs_pc_destroy / rs_vt_destroy, which always
 * synchronise and report it after freeing the handle.
 *
 * What each entry point replaces in the reference (/root/reference/ratslam):
 *   rs_pc_create    PoseCellNetwork.__init__      posecell_network.py:24-48
 *                   + Convolution(...)/set_params convolution.py:11-91
 *   rs_pc_update    PoseCellNetwork.update        posecell_network.py:326-353
 *                   (conv_im x3 + host inhibition/normalisation/clamps/argmax,
 *                    convolution.py:404-511, posecell_network.py:336-351)
 *   rs_pc_update_odom / rs_pc_run_odom
 *                   update(v) / run() taking the odometry itself: path_integration's
 *                   control (posecell_network.py:252-308) computed in the library
 *   rs_pc_excite    update() steps 1-4 alone      posecell_network.py:336-345
 *   rs_pc_run       a loop of update() calls      simulate.py:31-34, ros_simulate.py:134-137
 *   rs_pc_inject    PoseCellNetwork.inject        posecell_network.py:322-324
 *   rs_pc_get_max   PoseCellNetwork.get_pc_max    posecell_network.py:317-319
 *   rs_pc_read/write  the .posecells ndarray      posecell_network.py:27, simulate.py:60,
 *                                                 ros_simulate.py:140,145
 *   rs_vt_create    ViewTemplates.__init__        view_templates.py:42-57 (device library)
 *   rs_vt_add       templates.append(...)         view_templates.py:68-70
 *   rs_vt_match     ViewTemplates.match           view_templates.py:63-75
 *                   (scores = ViewTemplate.match  view_templates.py:16-28)
 *   rs_vt_match_batch  a loop of ViewTemplates.match calls (exact sequential
 *                   semantics incl. in-batch appends), or a frozen-library scan
 *   rs_vt_match_stream  many frozen-library batches, one host synchronisation
 *   rs_vt_read      ViewTemplate.template         view_templates.py:11
 *   rs_vt_scores    ViewTemplate.match per pair   view_templates.py:16-28 (uint8, wrapping)
 *   rs_sad_scores   ViewTemplate.match per pair   view_templates.py:16-28 (float32/float64)
 *   rs_vt_set_threshold  the `min(match_val) > match_threshold` rule, view_templates.py:67
 *   rs_vt_set_subsample / rs_vt_match_frames
 *                   input[self.mask].reshape(...) view_templates.py:48-57,64 (on device)
 *   rs_comm_*, rs_vt_attach_comm  (new) RCCL sharding of the library over GPUs
 */
#ifndef RATSLAM_ABI_H
#define RATSLAM_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (the Python wrapper maps them to exceptions) */
#define RS_OK           0
#define RS_ERR_ARG      1   /* ValueError   (bad size / index / parameter)          */
#define RS_ERR_TYPE     2   /* TypeError    (shape/dtype mismatch, convolution.py:578-611) */
#define RS_ERR_LUT_KEY  3   /* KeyError     (filter LUT miss, posecell_network.py:249) */
#define RS_ERR_HIP      4   /* RuntimeError (HIP runtime failure)                    */
#define RS_ERR_RCCL     5   /* RuntimeError (RCCL failure)                           */
#define RS_ERR_STATE    6   /* RuntimeError (handle misuse)                          */
#define RS_ERR_NOMEM    7   /* MemoryError                                           */
#define RS_ERR_CTL_RANGE 8  /* (internal) odometry outside the uploaded control tables;
                               nothing ran, the caller computes the control itself     */

#define RS_PREC_F32 0
#define RS_PREC_F64 1

#define RS_FILTER_LEN 7     /* PC_E_DIM, posecell_network.py:12; convolution.py:40 */

/* library version, e.g. 100 for 0.1.0 */
int rs_version(void);
/* thread-local description of the last error on this thread ("" if none) */
const char* rs_last_error(void);
/* number of visible HIP devices (0 if none / no driver) */
int rs_device_count(void);
/* device buffers for callers that keep inputs resident in HBM without a framework
 * (e.g. camera frames for rs_vt_match_frames); rs_dev_copy copies in any direction */
int rs_dev_malloc(int device, size_t bytes, void** ptr);
int rs_dev_free(void* ptr);
int rs_dev_copy(void* dst, const void* src, size_t bytes);
/* pinned, GPU-visible host memory (hipHostMalloc, mapped + coherent): the target of
 * rs_pc_read_pinned, so the .posecells readback needs no host-side copy */
int rs_host_alloc(size_t bytes, void** ptr);
int rs_host_free(void* ptr);

/* ------------------------------------------------------------------------ */
/* Pose-cell network                                                         */
/* ------------------------------------------------------------------------ */
typedef struct rs_pc rs_pc;

typedef struct rs_pc_params {
    int precision;              /* RS_PREC_F32 (default) or RS_PREC_F64          */
    double global_inhibition;   /* PC_GLOBAL_INHIB = 0.2 (posecell_network.py:15) */
    /* 3-D excitation kernel K = (ge x ge x ge - gi x gi x gi) * k_scale, the exact
     * rank-2 form of diff_gaussian(order=3) (posecell_network.py:97-113). */
    double ge[RS_FILTER_LEN];
    double gi[RS_FILTER_LEN];
    double k_scale;             /* 1 / |sum(ge^3 - gi^3)|                         */
    /* table of 7x7 path-integration filters (posecell_network.py:47,50-59),
     * row-major [nfilters][7][7], F[x][y] with x along the first grid axis */
    int nfilters;
    const double* xy_filters;
} rs_pc_params;

/* Per-step control computed on the host from the odometry exactly as
 * path_integration does (posecell_network.py:253-308):
 *   ox, oy [TH]  integer shifts of each theta layer       (:262-265)
 *   fidx   [TH]  index into the xy filter table per layer  (:249,271)
 *   zf     [7]   1-D theta filter                           (:304-309)
 * Batched forms are laid out step-major: ox[n*TH], oy[n*TH], fidx[n*TH], zf[n*7]. */

int rs_pc_create(int X, int Y, int TH, const rs_pc_params* params, int device, rs_pc** out);
int rs_pc_destroy(rs_pc* h);
int rs_pc_shape(const rs_pc* h, int* X, int* Y, int* TH);

/* one full update(); out_xyz = argmax cell (first in C order), as max_pc */
int rs_pc_update(rs_pc* h, const int32_t* ox, const int32_t* oy, const int32_t* fidx,
                 const double* zf, int32_t out_xyz[3]);
/* n consecutive updates with one host round trip; out_xyz[n*3] (may be NULL) */
int rs_pc_run(rs_pc* h, int n, const int32_t* ox, const int32_t* oy, const int32_t* fidx,
              const double* zf, int32_t* out_xyz);
/* Odometry -> control inside the library (posecell_network.py:252-308), so update()
 * costs one FFI call and no NumPy.  The wrapper uploads, once, the tables the NumPy
 * path evaluates with NumPy's own functions -- per-layer cos/sin of the heading
 * (:257-261), the LUT key -> filter row map (:249), and the 1-D theta filters for
 * origins zorig_min .. zorig_min+nz-1 (:304-308) -- and the library then applies
 * only correctly rounded IEEE operations (division, one product, rint, trunc,
 * floor, no contraction), so the control is bit-identical to filters.step_control.
 * rs_pc_update_odom: RS_ERR_LUT_KEY after running steps 1-4 (the reference's state
 * when :249 raises); RS_ERR_CTL_RANGE, with nothing run, when the theta origin is
 * outside the uploaded filters (the caller then computes the control itself).
 * rs_pc_run_odom: odom[n*2] = (vtrans, vrot) per step; on a LUT miss at step s it
 * runs steps < s, then steps 1-4 of s, sets *first_bad = s and returns
 * RS_ERR_LUT_KEY (else *first_bad = -1).  A batch of 1,024 steps or more forms its
 * control on up to 8 host threads before its first launch (the same values; the
 * first failing step decides, as in order). */
int rs_pc_set_odometry_tables(rs_pc* h, double vtrans_scale, double vrot_scale,
                              const double* cos_a, const double* sin_a, int key_min,
                              int nkeys, const int32_t* key_rows, int zorig_min, int nz,
                              const double* zf_table);
int rs_pc_update_odom(rs_pc* h, double vtrans, double vrot, int32_t out_xyz[3]);
/* the same control on the host alone (no handle, no device): n steps of odom[n*2]
 * -> ox/oy/fidx[n*TH], zf[n*7] and a status per step (RS_OK, RS_ERR_LUT_KEY,
 * RS_ERR_CTL_RANGE; outputs of a failed step are partial) */
int rs_pc_odom_control(int TH, double vtrans_scale, double vrot_scale, const double* cos_a,
                       const double* sin_a, int key_min, int nkeys, const int32_t* key_rows,
                       int zorig_min, int nz, const double* zf_table, int n, const double* odom,
                       int32_t* ox, int32_t* oy, int32_t* fidx, double* zf, int32_t* status);
int rs_pc_run_odom(rs_pc* h, int n, const double* odom, int32_t* out_xyz, int* first_bad);
/* rs_pc_update_odom followed, on the same stream and before its one host sync, by the
 * export of the new volume into pinned memory from rs_host_alloc (as
 * rs_pc_read_pinned): update() and the .posecells read the ROS node makes after every
 * step (ros_simulate.py:134-145) as one round trip.  On an error the volume export
 * may not have run. */
int rs_pc_update_odom_read(rs_pc* h, double vtrans, double vrot, int32_t out_xyz[3], double* pinned_xyth);
/* steps 1-4 of update() alone (excitation, global inhibition, normalisation):
 * the state the reference leaves behind when path_integration raises KeyError */
int rs_pc_excite(rs_pc* h);
/* posecells[x][y][th] += energy; queued on the handle's stream (returns without a
 * host sync), ordered before the next update / read / argmax */
int rs_pc_inject(rs_pc* h, double energy, int x, int y, int th);
int rs_pc_get_max(rs_pc* h, int32_t out_xyz[3]);
/* whole volume as float64, C order (X, Y, TH) -- the reference's .posecells */
int rs_pc_read(rs_pc* h, double* host_xyth);
/* the same volume written by the GPU straight into pinned host memory from
 * rs_host_alloc (at least X*Y*TH doubles): one launch and a sync, no host copy --
 * the drop-in .posecells readback the ROS node pays every step (ros_simulate.py:140,145) */
int rs_pc_read_pinned(rs_pc* h, double* pinned_xyth);
int rs_pc_write(rs_pc* h, const double* host_xyth);
/* sum of all cells (float64 accumulation) */
int rs_pc_total(rs_pc* h, double* total);
/* device time of the last rs_pc_run/rs_pc_update, milliseconds (HIP events around
 * the step's launches; recorded only while profiling is enabled, else 0 -- the two
 * event records cost about 1.5 us of a 31 us update() call) */
int rs_pc_last_ms(rs_pc* h, double* ms);
/* profiling: enable = 1 records HIP events around the whole call (rs_pc_last_ms)
 * and around every launch (rs_pc_kernel_ms; the per-launch events add gaps between
 * the kernels); enable = 2 only around the whole call; 0 none.
 * rs_pc_kernel_ms: the event time of each kernel of the last rs_pc_run, summed over its
 * steps: ms[0] = the step kernel (excitation kernel of the two-launch forms, the one
 * kernel of the halo form), ms[1] = path-integration kernel (halo form: pc_halo_finish) */
int rs_pc_set_profiling(rs_pc* h, int enable);
int rs_pc_kernel_ms(rs_pc* h, double ms[2]);
/* step kernels in use: "rows" (row-tiled excite + path launches, Y <= 128),
 * "cols" (column tiles through all layers, large grids), "halo" (one launch per
 * step, the excitation recomputed on each tile's halo; float32, TH = 36, 18 or 10), "stream"
 * (layer streaming, large grids outside the column form's limits) or "tiles" (3-D tiles) */
const char* rs_pc_step_form(const rs_pc* h);
/* Test hooks (no reference counterpart):
 *   RS_PC_DBG_POISON       fill every buffer a step writes before it reads (the
 *                          excited volume, the normalisation partials, the argmax
 *                          slots and partials, the host result words) with all
 *                          bits set, so that a read of anything the step did not
 *                          write shows up as NaN state or a wrong peak;
 *   RS_PC_DBG_SKIP_EXPORT  the next update/run leaves the host result words
 *                          unwritten: the call must fail with RS_ERR_HIP (the
 *                          check that every step's argmax reached the host);
 *   RS_PC_DBG_HALO_SETTLE  (halo form) every later call ends with the state
 *                          normalised by the finishing pass instead of left
 *                          unnormalised for the next call (A/B of the two paths);
 *   RS_PC_DBG_HALO_AMBIG   (rs_pc_debug_value) how many calls had their last step
 *                          keyed by the finishing pass because a cell lay within a
 *                          relative 2^-20 of the peak (pc_halo_export's RES_AMBIG). */
#define RS_PC_DBG_POISON      1
#define RS_PC_DBG_SKIP_EXPORT 2
#define RS_PC_DBG_HALO_SETTLE 3
#define RS_PC_DBG_HALO_AMBIG  4
int rs_pc_debug(rs_pc* h, int op);
int rs_pc_debug_value(rs_pc* h, int op, int64_t* value);

/* ------------------------------------------------------------------------ */
/* View templates                                                            */
/* ------------------------------------------------------------------------ */
typedef struct rs_vt rs_vt;

/* H x W uint8 templates, row shift max_offset (ViewTemplate.max_offset = 8,
 * view_templates.py:14), strict threshold match_threshold (:67).
 * capacity = initial number of templates this rank can hold (grows by doubling). */
int rs_vt_create(int H, int W, int max_offset, uint64_t match_threshold, int64_t capacity,
                 int device, rs_vt** out);
int rs_vt_destroy(rs_vt* h);
/* global number of stored templates (over all ranks) */
int rs_vt_count(const rs_vt* h, int64_t* count);
/* append n templates unconditionally (indices count .. count+n-1) */
int rs_vt_add(rs_vt* h, int n, const uint8_t* templates, int64_t* first_index);
/* read back template `index` (only on its owning rank: index % nranks == rank) */
int rs_vt_read(rs_vt* h, int64_t index, uint8_t* out);

#define RS_VT_FROZEN     0   /* score against the current library only, never append   */
#define RS_VT_SEQUENTIAL 1   /* exactly nq successive ViewTemplates.match calls          */

/* Match nq queries (each H x W uint8, already subsampled).  queries == NULL
 * re-matches the batch staged on the device by the previous call (same nq):
 * the queries stay resident in HBM across calls.
 * best_score[i]: the minimum score (UINT64_MAX if the library was empty)
 * best_index[i]: the index ViewTemplates.match returns (first argmin, or the
 *                new template's index when is_new[i] = 1)
 * is_new[i]:     1 if query i was appended as a new template                 */
int rs_vt_match_batch(rs_vt* h, int nq, const uint8_t* queries, int mode,
                      uint64_t* best_score, int64_t* best_index, uint8_t* is_new);
/* nb batches of nq queries each against the frozen library (nb successive
 * rs_vt_match_batch(RS_VT_FROZEN) calls), queued back to back on the device
 * with one host synchronisation.  queries[nb*nq*H*W]: host memory, or device
 * memory (rs_dev_malloc) whose batches the query-form kernels read in place.
 * Sharded handles reduce each batch with the RCCL allreduce(min) on the same
 * stream.  best_score / best_index[nb*nq] as in rs_vt_match_batch. */
int rs_vt_match_stream(rs_vt* h, int nb, int nq, const uint8_t* queries, uint64_t* best_score,
                       int64_t* best_index);
/* single query, RS_VT_SEQUENTIAL semantics */
int rs_vt_match(rs_vt* h, const uint8_t* query, uint64_t* best_score, int64_t* best_index,
                int* is_new);
/* On-device subsampling (view_templates.py:64, input[self.mask].reshape(shape)):
 * pixels[H*W] are the byte offsets, in a frame of frame_bytes, of the pixels the
 * mask keeps, in template row-major order (view_templates.py:48-57).  Then
 * rs_vt_match_frames matches nf whole frames (frame_bytes each; host memory, or
 * device memory the GPU gathers from in place) with rs_vt_match_batch semantics. */
int rs_vt_set_subsample(rs_vt* h, int64_t frame_bytes, const int32_t* pixels);
int rs_vt_match_frames(rs_vt* h, int nf, const uint8_t* frames, int mode, uint64_t* best_score,
                       int64_t* best_index, uint8_t* is_new);
/* all pair scores of nq queries vs templates [t0, t0+nt) (owning rank's slots only;
 * nranks must be 1): scores[q*nt + t]  -- ViewTemplate.match per pair */
int rs_vt_scores(rs_vt* h, int nq, const uint8_t* queries, int64_t t0, int64_t nt,
                 uint64_t* scores);
/* The two halves of rs_vt_match_batch, for callers that combine the per-rank
 * keys themselves (any min-reduction over ranks; key = score << 32 | index,
 * UINT64_MAX = no template):
 *   rs_vt_scan_local  stages the queries and returns this rank's keys;
 *   rs_vt_resolve     takes the global (min over ranks) keys of the staged
 *                     queries and applies ViewTemplates.match semantics,
 *                     appending the new templates this rank owns.            */
int rs_vt_scan_local(rs_vt* h, int nq, const uint8_t* queries, uint64_t* local_keys);
int rs_vt_resolve(rs_vt* h, int nq, const uint64_t* global_keys, int mode, uint64_t* best_score,
                  int64_t* best_index, uint8_t* is_new);
/* device time (ms) of the scan kernel in the last match call (HIP events): for
 * rs_vt_match_stream over HBM-resident batches, its one scan of all batches;
 * -1 when that scan ran untimed or the call ran several scans */
int rs_vt_last_ms(rs_vt* h, double* ms);
/* HIP events around every scan (default off).  Off, a match call's keys are polled in
 * pinned host memory (a plane scan's last block exports them itself) instead of a
 * stream synchronisation; on, two stream markers bracket each scan and the call
 * synchronises (rs_vt_last_ms) */
int rs_vt_set_timing(rs_vt* h, int enable);
/* which scan kernel family the handle uses for its shape: "plane" (bit-plane
 * borrow count, W == 32, H in {32, 64}, max_offset 8), "carry" (byte-SWAR carry
 * count, max_offset 8, H in {32, 64}; RS_VT_SCAN=carry forces it) or "generic";
 * NULL for a null handle */
const char* rs_vt_scan_form(const rs_vt* h);

/* ViewTemplates.match's strict threshold (view_templates.py:67) as a double: a
 * score makes a new template when (double)score > threshold -- numpy's own
 * comparison of a uint64 score with a Python float (inf: never once the library
 * is non-empty; negative: always; NaN: never).  rs_vt_create's integer threshold
 * is the same rule for thresholds that are integers. */
int rs_vt_set_threshold(rs_vt* h, double threshold);

/* ViewTemplate.match on float arrays (view_templates.py:16-28 with float32 or
 * float64 data: no uint8 wrap, a true sum |T - Q| per row offset in the arrays'
 * precision, numpy's pairwise summation order, first strict minimum over the
 * 2*max_offset-1 offsets from +inf).  templates[nt*H*W], queries[nq*H*W] and
 * scores[nq*nt] (scores[q*nt + t]) are host arrays of dtype RS_DT_F32 / F64;
 * the scores are computed on `device`. */
#define RS_DT_F32 0
#define RS_DT_F64 1
int rs_sad_scores(int device, int dtype, int H, int W, int max_offset, int64_t nt,
                  const void* templates, int nq, const void* queries, void* scores);

/* Multi-GPU: one process per GPU, library sharded round-robin (template g lives
 * on rank g % nranks at slot g / nranks); per query the local first-argmin keys
 * (score << 32 | g) are combined with one RCCL allreduce(min, uint64).        */
#define RS_UNIQUE_ID_BYTES 128
int rs_comm_unique_id(uint8_t id[RS_UNIQUE_ID_BYTES]);
int rs_vt_attach_comm(rs_vt* h, int rank, int nranks, const uint8_t id[RS_UNIQUE_ID_BYTES]);
/* shard without a communicator (the caller reduces keys between scan_local and resolve) */
int rs_vt_set_shard(rs_vt* h, int rank, int nranks);
int rs_vt_rank(const rs_vt* h, int* rank, int* nranks);

#ifdef __cplusplus
}
#endif
#endif /* RATSLAM_ABI_H */
